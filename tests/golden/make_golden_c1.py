"""Generate tests/golden/nbody_c1/ (a charged N=20 split in the reference's on-disk format) and
tests/golden/egno_run_epoch.npz: what the REFERENCE's run_epoch (EGNO/main_simulation_simple_no.py:
190-307, rollout=False) reports for config C1 of BASELINE.json -- EGNO forward, charged n_balls=20,
num_timesteps=10, batch 8 -- on that split with seed-0 weights:
  - backprop=False (the validation / test pass): the epoch's average loss (res['loss'] / res['counter'],
    the last frame's MSE per batch, :283-288) and every batch's per-frame losses (:273);
  - backprop=True with Adam(lr 1e-4, wd 1e-8; model_confs.yaml:15-17) on a non-shuffled loader: the
    per-batch per-frame losses (the first batch's are the initial weights' training loss).

Test infrastructure only (build container). The trajectories come from the reference's own simulator
(synthetic_sim.py:149-296) laid out as generate_dataset.py:45-147 writes them. Data only; no
reference source is copied. Re-run:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c1.py
"""
import contextlib
import io
import os
import sys
import types
from pathlib import Path

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = Path(HERE) / "nbody_c1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

# torch_geometric / wandb are not installed: to_dense_batch of equal-size graphs is a
# reshape, wandb.log a no-op
tg = types.ModuleType("torch_geometric")
tg.utils = types.ModuleType("torch_geometric.utils")


def _to_dense_batch(x, batch):
    B = int(batch.max()) + 1
    return x.reshape(B, -1, *x.shape[1:]), None


tg.utils.to_dense_batch = _to_dense_batch
tg.data = types.ModuleType("torch_geometric.data")
tg.data.Data = dict
sys.modules.update({"torch_geometric": tg, "torch_geometric.utils": tg.utils, "torch_geometric.data": tg.data})
wandb = types.ModuleType("wandb")
wandb.log = lambda *a, **k: None
sys.modules["wandb"] = wandb
sys.path.insert(0, REF)
import utils as ref_utils  # noqa: E402  (root utils.py)
import EGNO.utils as egno_utils  # noqa: E402

egno_utils.random_ascending_tensor = ref_utils.random_ascending_tensor
from EGNO.model.egno import EGNO  # noqa: E402
import EGNO.main_simulation_simple_no as ms  # noqa: E402
sys.path.insert(0, os.path.join(REF, "EGNO", "simulation"))
import synthetic_sim  # noqa: E402
from dataset_simple import NBodyDynamicsDataset  # noqa: E402

N, S, T, B = 20, 16, 10, 8


def write_split():
    OUT.mkdir(exist_ok=True)
    np.random.seed(47)
    with contextlib.redirect_stdout(io.StringIO()):
        sim = synthetic_sim.ChargedParticlesSim(noise_var=0.0, n_balls=N, vel_norm=0.5)
    locs, vels, edges, qs = [], [], [], []
    for _ in range(S):
        loc, vel, e, q = sim.sample_trajectory(T=5000, sample_freq=100)
        locs.append(loc); vels.append(vel); edges.append(e); qs.append(q)
    sfx = f"_charged{N}_initvel1small"
    for k, v in (("loc", locs), ("vel", vels), ("edges", edges), ("charges", qs)):
        np.save(OUT / f"{k}_train{sfx}.npy", np.stack(v).astype(np.float32 if k in ("loc", "vel") else v[0].dtype))


def run():
    args = types.SimpleNamespace(device="cpu", n_balls=N, num_inputs=1, num_timesteps=T, traj_len=1)
    with contextlib.redirect_stdout(io.StringIO()):
        ds = NBodyDynamicsDataset("train", data_dir=OUT, dataset="charged", dataset_name="nbody_small", n_balls=N,
                                  num_timesteps=T, num_inputs=1, traj_len=1)
    fx = {"cfg::N": N, "cfg::T": T, "cfg::B": B, "cfg::S": S}

    def model():
        torch.manual_seed(0)
        return EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                    num_timesteps=T, time_emb_dim=32, device="cpu")

    m = model()
    for k, v in m.state_dict().items():
        fx["w::" + k] = v.numpy()
    rec = []
    mse = torch.nn.MSELoss(reduction="none")

    def crit(a, b):
        out = mse(a, b)
        rec.append(out.detach().mean((0, 1, 3)).numpy())
        return out

    loader = torch.utils.data.DataLoader(ds, batch_size=B, shuffle=False, drop_last=False)
    with contextlib.redirect_stdout(io.StringIO()), torch.no_grad():
        avg = ms.run_epoch(m, None, crit, 0, loader, args, backprop=False)
    fx["eval::avg_loss"] = float(avg)
    fx["eval::losses"] = np.stack(rec)
    rec.clear()
    m = model()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4, weight_decay=1e-8)
    with contextlib.redirect_stdout(io.StringIO()):
        avg_tr = ms.run_epoch(m, opt, crit, 0, loader, args, backprop=True)
    fx["train::avg_loss"] = float(avg_tr)
    fx["train::losses"] = np.stack(rec)
    return fx


if __name__ == "__main__":
    write_split()
    fx = run()
    np.savez_compressed(os.path.join(HERE, "egno_run_epoch.npz"), **fx)
    print("wrote nbody_c1/ and egno_run_epoch.npz:", fx["eval::avg_loss"], fx["train::avg_loss"])
