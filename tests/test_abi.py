"""The drop-in boundary: libjh.so loads and exports every symbol include/*.h
(jh.h, jh_io.h) declares, and the ctypes mirror has the C layout (no GPU, no
compute calls)."""
import ctypes as C
import os
import re
import subprocess

from conftest import ROOT
from jepsen_amd import _abi as A

HEADER = os.path.join(ROOT, "include", "jh.h")
HEADERS = [HEADER, os.path.join(ROOT, "include", "jh_io.h")]


def declared_symbols():
    src = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:int|void|int64_t|const int64_t)\s+\*?(jh_\w+)\s*\(", src, re.M)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ["jh_version", "jh_open", "jh_close", "jh_check_cas_independent", "jh_check_cas",
              "jh_check_cas_independent_device", "jh_check_counter", "jh_check_set"]:
        assert s in syms


def test_libjh_loads_and_exports_every_symbol(built):
    from jepsen_amd import _native
    L = C.CDLL(_native.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert L.jh_version() == A.JH_ABI_VERSION
    assert sorted(_native.EXPORTED_SYMBOLS) == declared_symbols()


def test_ctypes_layout_matches_header(tmp_path):
    prog = tmp_path / "sz.c"
    prog.write_text(f'''#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(jh_history), sizeof(jh_lin_opts),
         sizeof(jh_key_verdict), sizeof(jh_summary), sizeof(jh_set_result),
         offsetof(jh_history, on_device), offsetof(jh_set_result, n_runs));
  return 0; }}''')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-o", str(exe), str(prog)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(A.JhHistory), C.sizeof(A.JhLinOpts), C.sizeof(A.JhKeyVerdict),
            C.sizeof(A.JhSummary), C.sizeof(A.JhSetResult), A.JhHistory.on_device.offset,
            A.JhSetResult.n_runs.offset]
    assert got == want
    assert A.VERDICT_DTYPE.itemsize == C.sizeof(A.JhKeyVerdict)


def test_ctypes_layout_set_full_and_queue(tmp_path):
    prog = tmp_path / "sz2.c"
    prog.write_text(f'''#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(jh_set_full_result), offsetof(jh_set_full_result, worst_stale),
         offsetof(jh_set_full_result, device_ms), sizeof(jh_queue_result),
         offsetof(jh_queue_result, fail_entry), sizeof(jh_set_full_elem));
  return 0; }}''')
    exe = tmp_path / "sz2"
    subprocess.run(["gcc", "-o", str(exe), str(prog)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(A.JhSetFullResult), A.JhSetFullResult.worst_stale.offset,
            A.JhSetFullResult.device_ms.offset, C.sizeof(A.JhQueueResult),
            A.JhQueueResult.fail_entry.offset, C.sizeof(A.JhSetFullElem)]
    assert got == want


def test_open_without_gpu_fails_loudly(built):
    """No CPU fallback: without a device the product path raises."""
    import torch
    if torch.cuda.is_available():
        return
    from jepsen_amd import _native
    try:
        _native.Context(0)
    except _native.JhError as e:
        assert e.code in (A.JH_EDEVICE, A.JH_EINVAL)
    else:
        raise AssertionError("jh_open succeeded without a GPU")


def test_lin_flags_match_header():
    """Every JH_LIN_* flag jh.h defines has the same value in _abi (the
    round-6 scheduling and takeover flags included)."""
    src = open(os.path.join(ROOT, "include", "jh.h")).read()
    flags = dict(re.findall(r"^#define\s+JH_(LIN_\w+)\s+(\d+)", src, re.M))
    assert {"LIN_NO_SPEC", "LIN_SPEC_FIRST", "LIN_HELP_STALL", "LIN_NO_TAKEOVER", "LIN_TAKEOVER"} <= set(flags)
    for name, v in flags.items():
        assert getattr(A, name) == int(v), name
