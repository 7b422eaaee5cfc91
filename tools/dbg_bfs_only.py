"""Debugging the BFS exact count: one saved heavy key (tools/data/<name>.npz),
BFS only (JH_BFS_ONLY=1: fail_entry = path length, cause = stored nodes)."""
import os, sys, numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
from jepsen_amd import _native
from jepsen_amd.history import Columns
name = sys.argv[1] if len(sys.argv) > 1 else "r6_key9152"
z = np.load(os.path.join(ROOT, "tools", "data", name + ".npz"))
n = len(z["process"])
one = Columns(n=n, process=z["process"], type=z["type"], f=z["f"], key=np.zeros(n, np.int64),
              value=z["value"], value2=z["value2"], n_keys=1, aux=np.zeros(1, np.int64))
ctx = _native.Context(0)
os.environ.setdefault("JH_BFS_ONLY", "1")
v, s = ctx.check_cas_independent(one)
print(name, "gpu", v[0])
