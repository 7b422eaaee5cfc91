"""jepsen_amd: an MI355X-native checker for Jepsen's verification phase.

Drop-in for (checker/linearizable {:model (model/cas-register)}),
jepsen.independent/checker, checker/counter and checker/set: the history is
encoded once into int64 columns (include/jh.h) and checked by hand-written
HIP kernels in libjh.so. See DESIGN.md.
"""
from . import checker, history, independent, model  # noqa: F401

__all__ = ["checker", "history", "independent", "model"]
