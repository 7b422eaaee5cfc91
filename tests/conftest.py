import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libjh.so kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def built():
    """Native libraries built in-tree (hipcc cross-compiles gfx950 without a GPU)."""
    from jepsen_amd import build
    build.build_all()
    return True


@pytest.fixture(scope="session")
def ctx(built):
    from jepsen_amd import _native
    return _native.default_context(0)


def load_npz_cols(name):
    import numpy as np
    from jepsen_amd.history import Columns
    z = np.load(os.path.join(GOLD, name))
    n = len(z["process"])
    key = z["key"] if "key" in z.files else np.full(n, -1, np.int64)
    cols = Columns(n=n, process=z["process"], type=z["type"], f=z["f"], key=key,
                   value=z["value"], value2=z["value2"],
                   n_keys=int(z["n_keys"]) if "n_keys" in z.files else 0,
                   aux=z["aux"] if "aux" in z.files else np.zeros(1, np.int64))
    return cols, z
