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


def test_stage_roundtrip_boundary_values(ctx):
    """the packed staging read back bit for bit (jh_stage_history)
    on the edges of its narrowing: INT32_MIN as a real value (must send its
    chunk's column whole), nil, 32-bit extremes, int8 -128 / 127 in type and
    :f (fit) and 128 (does not), a chunk wide only in the process column,
    another only in the key column, and n a multiple of neither 4 nor the
    1 M-row chunk."""
    from jepsen_amd.history import Columns
    rng = np.random.default_rng(7)
    n = (2 << 20) + 3 * (1 << 20) // 2 + 7           # 3.5 chunks + 7 rows
    C = 1 << 20
    cols = Columns(n=n, process=rng.integers(0, 50, n), type=rng.integers(0, 4, n), f=rng.integers(0, 3, n),
                   key=rng.integers(0, 1000, n), value=rng.integers(-5, 6, n), value2=rng.integers(-5, 6, n),
                   n_keys=1000)
    cols.value[rng.integers(0, n, 5000)] = A.NIL
    cols.value2[rng.integers(0, n, 5000)] = A.NIL
    cols.type[[1, 2]] = [-128, 127]; cols.f[[3, 4]] = [-128, 127]              # chunk 0: fit
    cols.value[[5, 6]] = [-(1 << 31) + 1, (1 << 31) - 1]                       # fit
    cols.f[C + 9] = 128                                                          # chunk 1: :f wide
    cols.value[C + 10] = -(1 << 31)                                              # INT32_MIN, not nil: wide
    cols.process[2 * C + 11] = 1 << 40                                           # chunk 2: process only
    cols.key[3 * C + 3] = 1 << 33                                                # chunk 3 (partial): key only
    cols.value2[n - 1] = 1 << 31                                                 # last row
    for name in ("process", "type", "f", "key", "value", "value2"):
        setattr(cols, name, np.ascontiguousarray(getattr(cols, name), dtype=np.int64))
    got = ctx.stage_history(cols)
    for i, name in enumerate(("process", "type", "f", "key", "value", "value2")):
        want = getattr(cols, name)
        bad = np.nonzero(got[i] != want)[0]
        assert len(bad) == 0, (name, bad[:5], got[i][bad[:5]], want[bad[:5]])
