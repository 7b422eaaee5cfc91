"""linear.svg for an invalid linearizability result (checker.clj:146-153:
when the analysis is invalid, checker/linearizable renders it with
knossos.linear.report/render-analysis! into the test's store directory under
(:subdirectory opts), and a rendering error is only logged).

knossos' renderer is not vendored, so the picture is this library's own: one
lane per process over the rows the frontier touches, each operation a bar from
its invocation to its completion (green: linearized in every frontier
configuration, grey: pending in some, red: the failing :op), and below it the
:final-paths, one line per configuration (model, then the step that fails).
Host-side formatting of the result map only; nothing here is on the device
path.
"""
import logging
import os
from xml.sax.saxutils import escape

import numpy as np

from . import _abi as A

log = logging.getLogger(__name__)

LANE_H = 28
ROW_W = 18
LEFT = 90
TOP = 30


def store_path(test, subdirectory, name):
    """store/path! (store.clj): <store dir>/<subdirectory...>/<name>, where
    the store dir is the test map's "store-dir"; None when the test names none."""
    base = test.get("store-dir") if isinstance(test, dict) else None
    if not base:
        return None
    sub = subdirectory if isinstance(subdirectory, (list, tuple)) else ([subdirectory] if subdirectory else [])
    d = os.path.join(base, *[str(s) for s in sub])
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, name)


def _span(cols, row):
    """(invocation row, completion row or None) of the operation row belongs to."""
    p = cols.process[row]
    if int(cols.type[row]) == A.TYPE_INVOKE:
        later = np.nonzero(cols.process[row + 1:] == p)[0]
        return row, (row + 1 + int(later[0])) if len(later) else None
    earlier = np.nonzero(cols.process[:row] == p)[0]
    return (int(earlier[-1]) if len(earlier) else row), row


def _label(op):
    v = op.get("value")
    if hasattr(v, "key") and hasattr(v, "value"):
        v = v.value
    return f"{op.get('f')} {v}"


def render_analysis(cols, result, path):
    """Write the SVG for an invalid result carrying :op, :configs and
    :final-paths (checker.add_configs). Returns the path written."""
    op = result.get("op")
    configs = result.get("configs") or []
    lin_all = {int(c["last-op"]["index"]) for c in configs if c.get("last-op")}
    pend = set()
    for c in configs:
        pend |= {o["index"] for o in c["pending"]}
    lin_all -= pend
    rows = {}
    for r in sorted(lin_all | pend):
        rows[_span(cols, r)] = "#8c8" if r in lin_all else "#bbb"
    if op is not None:
        rows[_span(cols, int(op["index"]))] = "#e66"
    if not rows:
        raise ValueError("nothing to render: no :op and no :configs")
    lo = min(a for a, _ in rows)
    hi = max(b if b is not None else a for a, b in rows) + 1
    procs = sorted({int(cols.process[a]) for a, _ in rows})
    lane = {p: i for i, p in enumerate(procs)}
    from .history import decode_op
    width = LEFT + (hi - lo + 1) * ROW_W + 20
    paths = result.get("final-paths") or []
    height = TOP + len(procs) * LANE_H + 30 + 18 * len(paths) + 20
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{height}" font-family="monospace" font-size="11">',
           f'<text x="4" y="16">invalid: no configuration gets past row {escape(str(op and op["index"]))}</text>']
    for p, i in lane.items():
        out.append(f'<text x="4" y="{TOP + i * LANE_H + 17}">process {p}</text>')
    for (a, b), color in sorted(rows.items()):
        x0 = LEFT + (a - lo) * ROW_W
        x1 = LEFT + ((b if b is not None else hi) - lo) * ROW_W + ROW_W
        y = TOP + lane[int(cols.process[a])] * LANE_H + 4
        lab = escape(_label(decode_op(cols, a)))
        out.append(f'<rect x="{x0}" y="{y}" width="{x1 - x0}" height="{LANE_H - 8}" fill="{color}" stroke="#333"/>')
        out.append(f'<text x="{x0 + 3}" y="{y + 14}">{lab}</text>')
    y = TOP + len(procs) * LANE_H + 24
    out.append(f'<text x="4" y="{y}">final paths (one per frontier configuration)</text>')
    for pth in paths:
        y += 18
        steps = " -> ".join(escape(f"{_label(s['op']) if s.get('op') else 'start'}: {s.get('model')}") for s in pth)
        out.append(f'<text x="4" y="{y}">{steps}</text>')
    out.append("</svg>")
    with open(path, "w") as fh:
        fh.write("\n".join(out))
    return path


def maybe_render(test, opts, cols, result):
    """checker.clj:147-153: render an invalid result when the test has a store
    directory; a failure is logged, never raised."""
    if result.get("valid?") is not False:
        return None
    try:
        path = store_path(test, (opts or {}).get("subdirectory"), "linear.svg")
        if path is None:
            return None
        return render_analysis(cols, result, path)
    except Exception as e:           # the reference catches Throwable and warns
        log.warning("Error rendering linearizability analysis: %s", e)
        return None
