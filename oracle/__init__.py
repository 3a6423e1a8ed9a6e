"""CPU ORACLE — test infrastructure only. Never imported by the product path.

A plain-numpy restatement of the reference's EGNO / SEGNO trajectory-rollout hot path
(simone7monaco/NO-NODE-comparison @ 2025-07-04). Every function cites the reference
file:line it follows. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import it: it is the checker and the reported CPU baseline, never the thing measured
or shipped. Parity is PINNED: tests/test_oracle_golden.py checks it against fixtures that
tests/golden/make_golden.py recorded by running the reference itself in the build
container.

Arithmetic type: every function takes arrays of one floating dtype and computes in it
(float32 mirrors the reference's numerics; float64 gives the noise floor).
"""
from . import egno, segno, harness  # noqa: F401
