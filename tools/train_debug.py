"""Per-parameter gradient errors of the HIP training path vs the reference golden (debug aid)."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.conftest import load_golden, maxnorm_rel, params_of  # noqa: E402
from tests.test_gpu_parity import _dev, _egno  # noqa: E402
from tests.test_gpu_train import _train_step_grads  # noqa: E402

fx = load_golden("egno_fwd")
gd = load_golden("egno_grad")
B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
m = _egno(params_of(fx))
inp = {k: _dev(fx["in::" + k]) for k in ("x", "h", "row", "col", "edge_attr", "v", "loc_mean", "t_out")}
inp["edge_fea"] = inp.pop("edge_attr")
loss, losses, g, _ = _train_step_grads(m, inp, _dev(gd["in::loc_true"]), T, B, N)
for k, got in g.items():
    ref = gd["grad::" + k]
    bad = np.argwhere(~np.isfinite(got))
    print(f"{maxnorm_rel(got, ref):10.3e} nonfinite={len(bad)} {k} {bad[:4].tolist()}")
