"""TEST INFRASTRUCTURE ONLY: a numpy restatement of (checker/set-full),
jepsen/src/jepsen/checker.clj:236-534, for columnar histories too large for
the op-map oracle (oracle/set_full.py, which the reference's own known
answers pin; tests/test_set_full_oracle.py checks this one against it).
Only tests/ and bench tools may import it.

The reference's fold (checker.clj:476-534), per element and in row order:
the element's record is (re)created by its :invoke :add (:483-487); an
:ok :add sets :known if unset (set-full-add, :262-266); every :ok :read
sets :known if unset and the element is present, and keeps the read
invocation of greatest :index as :last-present / :last-absent
(set-full-read-present/-absent, :268-286); reads by non-integer processes
are ignored (:480). Here the per-read update is vectorised over elements.
"""
import numpy as np

NIL = -(1 << 63)
POINTS = (0, 0.5, 0.95, 0.99, 1)


def _freq(points, c):
    """frequency-distribution, checker.clj:347-358."""
    s = np.sort(np.asarray(c, np.int64))
    n = len(s)
    if n == 0:
        return None
    return {p: int(s[min(n - 1, int(np.floor(n * p)))]) for p in points}


def set_full_cols(cols, time, linearizable=False):
    """Returns (result map as oracle/set_full.set_full, per-element arrays)."""
    proc, typ, f = cols.process, cols.type, cols.f
    val, val2, aux = cols.value, cols.value2, cols.aux
    n = cols.n
    rows = np.arange(n, dtype=np.int64)
    client = proc >= 0
    inv_add = client & (f == 3) & (typ == 0)
    elem = np.unique(val[inv_add])
    M = len(elem)
    last_inv = np.full(M, -1, np.int64)
    np.maximum.at(last_inv, np.searchsorted(elem, val[inv_add]), rows[inv_add])
    ok_add = client & (f == 3) & (typ == 1)
    ids = np.searchsorted(elem, val[ok_add])
    inr = (ids < M) & (elem[np.minimum(ids, max(M - 1, 0))] == val[ok_add]) if M else np.zeros(0, bool)
    known = np.full(M, np.iinfo(np.int64).max, np.int64)
    okr = rows[ok_add][inr]
    okid = ids[inr]
    after = okr > last_inv[okid]
    np.minimum.at(known, okid[after], okr[after])
    # :ok reads and their invocations: the process' previous row (a :read :invoke)
    order = np.lexsort((rows, proc))
    prev = np.full(n, -1, np.int64)
    same = proc[order][1:] == proc[order][:-1]
    prev[order[1:][same]] = order[:-1][same]
    kread = np.full(M, np.iinfo(np.int64).max, np.int64)
    lp = np.full(M, -1, np.int64)
    la = np.full(M, -1, np.int64)
    for r in rows[client & (f == 0) & (typ == 1)]:
        q = prev[r]
        if q < 0 or f[q] != 0 or typ[q] != 0:
            raise ValueError(f"an :ok :read at row {r} without its invocation")
        c = 0 if (val2[r] == NIL or val[r] == NIL) else int(val2[r])
        vs = aux[val[r]:val[r] + c]
        pres = np.zeros(M, bool)
        if M and c:
            j = np.searchsorted(elem, vs)
            hit = (j < M) & (elem[np.minimum(j, M - 1)] == vs)
            pres[j[hit]] = True
        act = r > last_inv
        p = act & pres
        kread[p & (kread == np.iinfo(np.int64).max)] = r
        lp[p] = np.maximum(lp[p], q)
        a = act & ~pres
        la[a] = np.maximum(la[a], q)
    kn = np.minimum(known, kread)
    kn[kn == np.iinfo(np.int64).max] = -1
    stable = (lp >= 0) & (la < lp)
    lost = (kn >= 0) & (la >= 0) & (lp < la) & (kn < la)
    st = np.where(la >= 0, time[np.maximum(la, 0)] + 1, 0)
    lt = np.where(lp >= 0, time[np.maximum(lp, 0)] + 1, 0)
    kt = time[np.maximum(kn, 0)]
    slat = np.where(stable, np.maximum(st - kt, 0) // 1000000, -1)
    llat = np.where(lost, np.maximum(lt - kt, 0) // 1000000, -1)
    never = ~stable & ~lost
    stale = stable & (slat > 0)
    si = np.flatnonzero(stale)
    worst_order = si[np.lexsort((si, slat[si]))][::-1][:8]     # stable sort-by, reversed
    ns, nl = int(stable.sum()), int(lost.sum())
    if nl:
        valid = False
    elif ns == 0:
        valid = "unknown"
    elif linearizable and len(si):
        valid = False
    else:
        valid = True
    m = {"valid?": valid, "attempt-count": M, "stable-count": ns, "lost-count": nl,
         "lost": elem[lost].tolist(), "never-read-count": int(never.sum()),
         "never-read": elem[never].tolist(), "stale-count": len(si), "stale": elem[si].tolist(),
         "worst-stale": [(int(elem[i]), int(slat[i]), int(kn[i]), int(la[i])) for i in worst_order]}
    if ns:
        m["stable-latencies"] = _freq(POINTS, slat[stable])
    if nl:
        m["lost-latencies"] = _freq(POINTS, llat[lost])
    m["duplicated-count"] = 0
    m["duplicated"] = {}
    return m
