"""Builds the native parts in-tree (they travel to the GPU box with the repo).

  jepsen_amd/libjh.so     the product: HIP kernels + C ABI (include/jh.h), gfx950
  jepsen_amd/libjhgen.so  synthetic-history generator (workload / test data)

`python -m jepsen_amd.build` or __graft_entry__.build(). hipcc cross-compiles
for gfx950 without a GPU. Objects are rebuilt only when a source or header is
newer.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
HIP_SOURCES = ["jh_lin.hip", "jh_counter.hip", "jh_set.hip", "jh_setfull.hip", "jh_queue.hip", "jh_api.hip", "jh_multi.hip", "jh_ingest.hip"]
HOST_SOURCES = ["jh_io.cpp"]
HEADERS = [os.path.join(CSRC, "jh_internal.h"), os.path.join(ROOT, "include", "jh.h")]
HOST_HEADERS = [os.path.join(ROOT, "include", "jh.h"), os.path.join(ROOT, "include", "jh_io.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
HIPFLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-but-set-variable"]
# Not used: -mllvm -structurizecfg-skip-uniform-regions=1. It made the DFS step
# 5-8% faster, but it miscompiles a divergent loop with data-dependent exits in
# the BFS (the cross-layer RET-drop loop of k_lin_bfs): some lanes' edges were
# dropped and a reachable set came out 11 configurations short (found by the
# exact-count test of a valid key; tools/dbg_bfs_only.py reproduces it).
HIPFLAGS += os.environ.get("JH_HIPFLAGS", "").split()   # e.g. -DJH_STEP_PROF (profiling builds)


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build_libjh(verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    jobs = []
    objs = []
    for s in HIP_SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJ, s.replace(".hip", ".o"))
        objs.append(obj)
        if _newer(obj, [src] + HEADERS):
            jobs.append([HIPCC] + HIPFLAGS + ["-c", src, "-o", obj])
    # host-only sources (history ingest, include/jh_io.h): g++, linked into libjh.so
    for s in HOST_SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJ, s.replace(".cpp", ".o"))
        objs.append(obj)
        if _newer(obj, [src] + HOST_HEADERS):
            jobs.append(["g++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-pthread", "-c", src, "-o", obj])
    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for out in ex.map(_run, jobs):
            if verbose and out.strip():
                print(out)
    lib = os.path.join(HERE, "libjh.so")
    if _newer(lib, objs):
        # linked aside and renamed: a snapshot of the tree (gpurun) never sees a half-written library
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-pthread", "-o", lib + ".tmp"] + objs)
        os.replace(lib + ".tmp", lib)
    return lib


def build_gen():
    src = os.path.join(CSRC, "gen.cpp")
    lib = os.path.join(HERE, "libjhgen.so")
    if _newer(lib, [src, os.path.join(ROOT, "include", "jh.h")]):
        _run(["g++", "-O2", "-g", "-fPIC", "-shared", "-std=c++17", "-Wall", "-pthread", "-o", lib + ".tmp", src])
        os.replace(lib + ".tmp", lib)
    return lib


def build_oracle():
    """Test infrastructure only (oracle/): the CPU restatement used as checker."""
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return os.path.join(ROOT, "oracle", "liboracle.so")


def build_harness():
    """tests/c/jh_harness: a plain-C program linked against libjh.so (the
    boundary as a JNA/cgo caller sees it; tests/test_c_harness.py)."""
    src = os.path.join(ROOT, "tests", "c", "jh_harness.c")
    exe = os.path.join(ROOT, "tests", "c", "jh_harness")
    lib = os.path.join(HERE, "libjh.so")
    if _newer(exe, [src, lib, os.path.join(ROOT, "include", "jh.h")]):
        _run(["gcc", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"), src, "-L" + HERE, "-ljh",
              "-Wl,-rpath,$ORIGIN/../../jepsen_amd", "-o", exe])
    return exe


def build_all(verbose=False):
    return [build_libjh(verbose), build_gen(), build_oracle(), build_harness()]


if __name__ == "__main__":
    for p in build_all(verbose="-v" in sys.argv):
        print(p)
