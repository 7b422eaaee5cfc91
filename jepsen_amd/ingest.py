"""Native history ingest (include/jh_io.h, jepsen_amd/csrc/jh_io.cpp).

A stored Jepsen run -- history.edn (jepsen/src/jepsen/store.clj:346-357, one
prn-printed op map per line) or test.fressian (store.clj:359-366, the whole
test map; :history read out of it) -- straight into the columnar layout the
checkers take, in multi-threaded C++ inside libjh.so. The result is the
`history.Columns` that `edn.load_columns` (the Python reader) gives for the
same file, column for column and table for table (tests/test_ingest.py), at
native speed: the Python reader tokenises ~1 M ops/min, the native one
hundreds of M per minute on the host's cores.

    cols = ingest.load_columns("store/.../history.edn", independent=True)
    cols, time = ingest.load_columns(path, with_time=True)     # :time for set-full
"""
import ctypes as C

import numpy as np

from . import _abi as A
from . import edn
from . import history as H
from ._native import JhError, lib

FMT = {"auto": 0, "edn": 1, "fressian": 2}
TBL_KEYS, TBL_F, TBL_VALUES = 0, 1, 2
DEFAULT_MIN_CHUNK = 0        # jh_ingest_opts.min_chunk when a call gives none (0 = 1 MiB)


def _table(L, g, which):
    n = L.jh_ingest_table_size(g, which)
    out = []
    buf = C.create_string_buffer(256)
    for i in range(n):
        m = L.jh_ingest_table_entry(g, which, i, buf, len(buf))
        if m >= len(buf):
            buf = C.create_string_buffer(int(m) + 1)
            L.jh_ingest_table_entry(g, which, i, buf, len(buf))
        out.append(buf.value.decode("utf-8"))
    # each entry is the canonical EDN text of one interned object
    return [edn.read_all(t)[0] if t else None for t in out]


def _load(L, rc, g, err, with_time):
    if rc != A.JH_OK:
        raise JhError(rc, err.value.decode(errors="replace"))
    try:
        h = A.JhHistory()
        L.jh_ingest_history(g, C.byref(h))
        n = int(h.n)

        def col(p, m):
            return np.ctypeslib.as_array(p, shape=(m,)).copy() if m > 0 else np.zeros(0, np.int64)

        cols = H.Columns(
            n=n, process=col(h.process, n), type=col(h.type, n), f=col(h.f, n), key=col(h.key, n),
            value=col(h.value, n), value2=col(h.value2, n), n_keys=int(h.n_keys),
            aux=col(h.aux, int(h.n_aux)) if h.n_aux > 0 else np.zeros(1, np.int64))
        cols.keys = _table(L, g, TBL_KEYS)
        cols.f_names = _table(L, g, TBL_F)
        cols.values_interned = bool(L.jh_ingest_values_interned(g))
        cols.value_table = _table(L, g, TBL_VALUES) if cols.values_interned else []
        cols.ints_only = not cols.values_interned
        if with_time:
            return cols, col(L.jh_ingest_time(g), n)
        return cols
    finally:
        L.jh_ingest_free(g)


def _opts(threads, min_chunk, debug):
    mc = DEFAULT_MIN_CHUNK if min_chunk is None else min_chunk
    return A.JhIngestOpts(threads=int(threads), debug=int(bool(debug)), min_chunk=int(mc))


def load_columns(path, independent=False, fmt="auto", threads=0, with_time=False, min_chunk=None, debug=False):
    """history.edn / test.fressian file -> history.Columns (include/jh.h
    layout); keyed by independent tuple when independent=True. threads=0: all
    cores (EDN; fressian is one sequential pass). min_chunk / debug:
    jh_ingest_opts (smallest EDN chunk, 0 = 1 MiB; per-chunk timings)."""
    L = lib()
    g = C.c_void_p()
    err = C.create_string_buffer(512)
    o = _opts(threads, min_chunk, debug)
    rc = L.jh_ingest_file_opts(str(path).encode(), FMT[fmt], 1 if independent else 0, C.byref(o), C.byref(g),
                               err, len(err))
    return _load(L, rc, g, err, with_time)


def parse_columns(data, independent=False, fmt="auto", threads=0, with_time=False, min_chunk=None, debug=False):
    """The same over bytes (or str) in memory."""
    if isinstance(data, str):
        data = data.encode("utf-8")
    L = lib()
    g = C.c_void_p()
    err = C.create_string_buffer(512)
    o = _opts(threads, min_chunk, debug)
    rc = L.jh_ingest_buffer_opts(data, len(data), FMT[fmt], 1 if independent else 0, C.byref(o), C.byref(g),
                                 err, len(err))
    return _load(L, rc, g, err, with_time)
