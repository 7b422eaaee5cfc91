"""HBM a context holds after a C3 check (hipMemGetInfo through the HIP
runtime libjh.so loaded), for INTEGRATION.md section 4b.

    python tools/mem_probe.py [contexts]
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402
from jepsen_amd import _native, synth  # noqa: E402

_native.lib()
path = next((ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln), "libamdhip64.so")
hip = C.CDLL(path)


def free_total():
    fr, tot = C.c_size_t(), C.c_size_t()
    assert hip.hipMemGetInfo(C.byref(fr), C.byref(tot)) == 0
    return fr.value, tot.value


wl = WORKLOADS["c3"]
cols, _ = synth.cas_register(n_keys=wl["keys"], ops_per_key=500, seed=wl["seed"], **wl["gen"])
f0, tot = free_total()
ctxs, out = [], []
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    ctxs.append(_native.Context(0))
    ctxs[-1].check_cas_independent(cols, budget=wl["budget"], exact_count=False)
    f1, _ = free_total()
    out.append({"contexts": i + 1, "held_gb": (f0 - f1) / 2 ** 30})
print(json.dumps({"device_gb": tot / 2 ** 30, "after_each": out}), flush=True)
