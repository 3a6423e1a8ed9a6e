"""MI355X-native EGNO / SEGNO trajectory-rollout hot path.

Drop-in for simone7monaco/NO-NODE-comparison's ``EGNO`` (EGNO/model/egno.py) and ``SEGNO``
(SEGNO/models/model.py): same constructors, forwards and state_dict keys; the compute runs in
hand-written gfx950 HIP kernels (libnonode.so, C ABI in include/nonode.h). There is no CPU path.
"""
from ._lib import NonodeError, lib  # noqa: F401
from .egno import EGNO  # noqa: F401
from .segno import SEGNO  # noqa: F401
from . import dataset, graph, harness, metrics, sim  # noqa: F401

__all__ = ["EGNO", "SEGNO", "NonodeError", "lib", "dataset", "graph", "harness", "metrics", "sim"]
