"""TEST INFRASTRUCTURE ONLY: a plain-Python restatement of (checker/set-full),
jepsen/src/jepsen/checker.clj:236-534, used as the checker of the device path
(tests/) on small histories. Only tests/ may import it.

Ops are dicts {"process", "type", "f", "value", "time", "index"} as in
jepsen_amd.history; a read's value is a collection of elements.
Pinned by the reference's own known answers (checker_test.clj:461-626,
tests/golden/set_full.json).
"""
import math


def _element_results(e):
    """set-full-element-results, checker.clj:289-345."""
    known, lp, la = e["known"], e["last-present"], e["last-absent"]
    stable = bool(lp is not None and (la["index"] if la else -1) < lp["index"])
    lost = bool(known is not None and la is not None
                and (lp["index"] if lp else -1) < la["index"]
                and known["index"] < la["index"])
    stable_lat = lost_lat = None
    if stable:
        st = la["time"] + 1 if la else 0
        stable_lat = _ms(max(st - known["time"], 0))
    if lost:
        lt = lp["time"] + 1 if lp else 0
        lost_lat = _ms(max(lt - known["time"], 0))
    outcome = "stable" if stable else ("lost" if lost else "never-read")
    return {"element": e["element"], "outcome": outcome, "stable-latency": stable_lat,
            "lost-latency": lost_lat, "known": known, "last-absent": la}


def _ms(nanos):
    """util/nanos->ms then long, for the non-negative latencies set-full takes
    it of: floor(nanos / 10^6)."""
    return nanos // 1000000


def frequency_distribution(points, c):
    """checker.clj:347-358."""
    s = sorted(c)
    if not s:
        return None
    n = len(s)
    return {p: s[min(n - 1, int(math.floor(n * p)))] for p in points}


def set_full(history, linearizable=False):
    """checker.clj:476-534 (check of (set-full {:linearizable? ...}))."""
    elements, reads = {}, {}
    for op in history:
        p = op.get("process")
        if not (isinstance(p, int) and not isinstance(p, bool)):
            continue                                    # (comp number? :process)
        f, t, v = op.get("f"), op.get("type"), op.get("value")
        if f == "add":
            if t == "invoke":
                elements[v] = {"element": v, "known": None, "last-present": None, "last-absent": None}
            elif v in elements and t == "ok":          # set-full-add: :ok records known
                e = elements[v]
                if e["known"] is None:
                    e["known"] = op
        elif f == "read":
            if t == "invoke":
                reads[p] = op
            elif t == "fail":
                reads.pop(p, None)
            elif t == "ok":
                inv = reads.get(p)
                vs = set(v or ())                      # (c/set nil) = #{}
                for el, e in elements.items():
                    if el in vs:                          # set-full-read-present
                        if e["known"] is None:
                            e["known"] = op
                        if e["last-present"] is None or e["last-present"]["index"] < inv["index"]:
                            e["last-present"] = inv
                    else:                                 # set-full-read-absent
                        if e["last-absent"] is None or e["last-absent"]["index"] < inv["index"]:
                            e["last-absent"] = inv
    rs = [_element_results(elements[k]) for k in sorted(elements)]
    stable = [r for r in rs if r["outcome"] == "stable"]
    lost = [r for r in rs if r["outcome"] == "lost"]
    never = [r for r in rs if r["outcome"] == "never-read"]
    stale = [r for r in stable if r["stable-latency"] > 0]
    worst = list(reversed(sorted(stale, key=lambda r: r["stable-latency"])))[:8]
    if lost:
        valid = False
    elif not stable:
        valid = "unknown"
    elif linearizable and stale:
        valid = False
    else:
        valid = True
    m = {"valid?": valid, "attempt-count": len(rs), "stable-count": len(stable),
         "lost-count": len(lost), "lost": sorted(r["element"] for r in lost),
         "never-read-count": len(never), "never-read": sorted(r["element"] for r in never),
         "stale-count": len(stale), "stale": sorted(r["element"] for r in stale),
         "worst-stale": worst}
    points = [0, 0.5, 0.95, 0.99, 1]
    sl = [r["stable-latency"] for r in rs if r["stable-latency"] is not None]
    ll = [r["lost-latency"] for r in rs if r["lost-latency"] is not None]
    if sl:
        m["stable-latencies"] = frequency_distribution(points, sl)
    if ll:
        m["lost-latencies"] = frequency_distribution(points, ll)
    # duplicates: (frequencies v) counts are >= 1, so `(< v 1)` never holds
    # (checker.clj:505-510) and :duplicated is always empty
    m["duplicated-count"] = 0
    m["duplicated"] = {}
    return m
