"""CPU: how far the reference's own fp32 ops land from float64 on the EGNO guard-path case of
tests/test_gpu_parity.py::test_egno_guard_path_matches_oracle[1-70-10000.0] when only the ORDER of the
edge list (so of every scatter-add's summation) changes. The case's coordinates reach ~1e13, so its
message and force sums cancel heavily in fp32: the spread below is the fp32 floor of any summation order,
the HIP kernel's included.   python3 tools/guard_order_spread.py [orders] > profiles/r06/guard_order_spread.txt"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import no_node_comparison_amd as pkg  # noqa: E402
from oracle import egno as oe, torch_ref as tr  # noqa: E402
from tests.test_gpu_parity import _egno_case  # noqa: E402

B, N, scale, T = 1, 70, 1e4, 10
torch.manual_seed(B * 7 + N)   # the test's module (seed B * 7 + N) and case (seed N + 1)
m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2, num_timesteps=T,
             time_emb_dim=32)
p = {k: v.detach().numpy().astype(np.float64) for k, v in m.state_dict().items()}
case = _egno_case(B, N, T, seed=N + 1)
case["edge_fea"] = (case["edge_fea"] * scale).astype(np.float32)
with np.errstate(over="ignore"):
    xr, vr, hr = oe.egno_forward(p, **{k: (v.astype(np.float64) if k not in ("row", "col", "t_out") else v)
                                       for k, v in case.items()}, T=T)
p32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in p.items()}
t = lambda a: torch.tensor(np.ascontiguousarray(a))  # noqa: E731
rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())  # noqa: E731
E = case["row"].shape[0]
print("edge order          x        v        h   (max-norm relative to float64)")
worst = np.zeros(3)
orders = int(sys.argv[1]) if len(sys.argv) > 1 else 16
errs = []
for trial in range(orders):
    perm = np.arange(E) if trial == 0 else np.random.default_rng(trial).permutation(E)
    with torch.no_grad():
        f = tr.egno_forward(p32, t(case["x"]).float(), t(case["h"]).float(), t(case["row"][perm]).long(),
                            t(case["col"][perm]).long(), t(case["edge_fea"][perm]).float(), t(case["v"]).float(),
                            t(case["loc_mean"]).float(), t(case["t_out"]).float(), T=T)
    e = np.array([rel(f[0].numpy(), xr), rel(f[1].numpy(), vr), rel(f[2].numpy(), hr)])
    worst = np.maximum(worst, e)
    errs.append(e)
    print(f"{'dataset' if trial == 0 else f'perm {trial:2d}':12s} " + " ".join(f"{x:.2e}" for x in e))
print(f"{'max':12s} " + " ".join(f"{x:.2e}" for x in worst))
errs = np.array(errs)
for q in (50, 90, 99):
    print(f"{f'p{q}':12s} " + " ".join(f"{x:.2e}" for x in np.percentile(errs, q, axis=0)))
hip = {"x": 2.4e-5, "v": 9.44e-6}   # the HIP guard N=70 figures (round 5 GPU log)
for i, (k, val) in enumerate(hip.items()):
    print(f"HIP {k} {val:.2e}: {int((errs[:, i] >= val).sum())} of {orders} orders at or above it")
