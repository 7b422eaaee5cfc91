"""Host-buffer staging (jh_ingest.hip): histories of 2 M rows and more cross
PCIe in packed chunks (1 or 4 bytes per column value when a chunk's values
fit, else whole) and are widened back in HBM. Each test compares a call on
host buffers with the same call on the history already in HBM (staged by
torch, not by the library): the verdicts must be identical field by field."""
import numpy as np
import pytest

from jepsen_amd import _abi as A
from jepsen_amd import _native, synth

pytestmark = pytest.mark.gpu

def _device_verdicts(ctx, cols, **kw):
    """The same call on the columns already in HBM (hipMalloc + hipMemcpy
    through the runtime libjh.so loaded: no second HIP runtime from torch)."""
    import ctypes as C
    from hipcols import DevCols as _DevCols
    d = _DevCols(cols, 0)
    hip = d._hip
    p = C.c_void_p()
    nb = max(cols.n_keys, 1) * A.VERDICT_DTYPE.itemsize
    assert hip.hipMalloc(C.byref(p), nb) == 0
    try:
        s = ctx.check_cas_independent_device(d, p.value, **kw)
        v = np.zeros(max(cols.n_keys, 1), dtype=A.VERDICT_DTYPE)
        assert hip.hipMemcpy(v.ctypes.data, p.value, nb, 2) == 0          # hipMemcpyDeviceToHost
    finally:
        hip.hipFree(p)
    return v[:cols.n_keys], s


def _same(a, b):
    for f in A.VERDICT_DTYPE.names:
        assert np.array_equal(a[f], b[f]), f


def test_ingest_c3_equals_resident(ctx):
    cols, _ = synth.cas_register(n_keys=10000, ops_per_key=500, seed=3, process_limit=20)
    assert cols.n >= (1 << 21)
    vh, sh = ctx.check_cas_independent(cols, budget=1 << 20)
    vd, sd = _device_verdicts(ctx, cols, budget=1 << 20)
    _same(vh, vd)
    assert sh.valid == sd.valid and sh.first_fail_entry == sd.first_fail_entry


def test_ingest_wide_chunks_and_nil(ctx):
    """Chunk 1's values do not fit 32 bits (its value columns cross whole,
    the other chunks' packed); nil reads stay nil."""
    cols, _ = synth.cas_register(n_keys=3000, ops_per_key=500, seed=11)
    n = int(cols.n)
    assert n >= (1 << 21)
    c1 = slice(1 << 20, min(n, 2 << 20))
    for name in ("value", "value2"):
        col = getattr(cols, name).copy()
        seg = col[c1]
        seg[seg != A.NIL] += 1 << 35
        col[c1] = seg
        setattr(cols, name, col)
    assert (cols.value == A.NIL).any()
    vh, _ = ctx.check_cas_independent(cols, budget=1 << 20)
    vd, _ = _device_verdicts(ctx, cols, budget=1 << 20)
    _same(vh, vd)


def test_ingest_counter_equals_resident(ctx):
    from hipcols import DevCols as _DevCols
    cols = synth.counter(n_ops=1_500_000, n_procs=16, seed=5, n_bad_reads=3)
    assert cols.n >= (1 << 21)
    rh = ctx.check_counter(cols)
    d = _DevCols(cols, 0)
    rd = ctx.check_counter(d, reads_cap=int(cols.n), on_device=True)
    for k in ("valid", "cause", "n_reads", "n_errors", "first_err_entry"):
        assert rh[k] == rd[k], k
    assert np.array_equal(rh["reads"], rd["reads"])
