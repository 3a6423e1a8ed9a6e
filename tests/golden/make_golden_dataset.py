"""Generate tests/golden/nbody_tiny/ (.npy splits in the reference's on-disk format),
tests/golden/dataset_items.npz (what the REFERENCE loaders return for them: EGNO's
NBodyDynamicsDataset with num_inputs = 1 and 3 (equispaced and varDT inputs), SEGNO's NBodyDataset
(SEGNO/dataset_nbody.py:7-94) and the model inputs SEGNO's run_epoch builds from its batches,
train_nbody.py:76-123, with num_inputs = 1 and 3) and
tests/golden/metrics.npz (the reference's pearson_correlation_batch, utils.py:261-321, on
synthetic prediction / truth pairs).

Test infrastructure only (build container). The .npy files are written by the reference's own
simulators as generate_dataset.py lays them out (generate_dataset.py:45-147, names
loc_{split}_{charged|gravity}{N}_initvel1small.npy); the items come from the reference's
NBodyDynamicsDataset (EGNO/simulation/dataset_simple.py:122-178) with num_inputs = 1. Data only; no
reference source is copied. Re-run:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dataset.py
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
OUT = Path(HERE) / "nbody_tiny"

import numpy as np  # noqa: E402
import torch  # noqa: E402

# torch_geometric / wandb are not installed; the loader path only needs to import
tg = types.ModuleType("torch_geometric")
tg.utils = types.ModuleType("torch_geometric.utils")
tg.utils.to_dense_batch = lambda x, b: (x, None)
tg.data = types.ModuleType("torch_geometric.data")
tg.data.Data = dict
sys.modules.update({"torch_geometric": tg, "torch_geometric.utils": tg.utils, "torch_geometric.data": tg.data})
wandb = types.ModuleType("wandb")
wandb.log = lambda *a, **k: None
sys.modules["wandb"] = wandb
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(REF, "EGNO", "simulation"))
import synthetic_sim  # noqa: E402
from dataset_simple import NBodyDynamicsDataset  # noqa: E402
import utils as ref_utils  # noqa: E402  (root utils.py)


def write_splits():
    OUT.mkdir(exist_ok=True)
    np.random.seed(43)
    with contextlib.redirect_stdout(io.StringIO()):
        sim = synthetic_sim.ChargedParticlesSim(noise_var=0.0, n_balls=5, vel_norm=0.5)
    locs, vels, edges, qs = [], [], [], []
    for _ in range(6):
        loc, vel, e, q = sim.sample_trajectory(T=5000, sample_freq=100)
        locs.append(loc); vels.append(vel); edges.append(e); qs.append(q)
    sfx = "_charged5_initvel1small"
    for k, v in (("loc", locs), ("vel", vels), ("edges", edges), ("charges", qs)):
        np.save(OUT / f"{k}_train{sfx}.npy", np.stack(v))
    np.random.seed(44)
    gsim = synthetic_sim.GravitySim(noise_var=0.0, n_balls=5, vel_norm=0.5)
    pos, vel, force, mass = gsim.sample_trajectory_batch(T=3000, sample_freq=100, batch_size=4)
    sfx = "_gravity5_initvel1small"
    for k, v in (("loc", pos), ("vel", vel), ("edges", force), ("charges", mass)):
        np.save(OUT / f"{k}_train{sfx}.npy", v)


def items(dataset):
    d = {}
    with contextlib.redirect_stdout(io.StringIO()):
        ds = NBodyDynamicsDataset("train", data_dir=OUT, dataset=dataset, dataset_name="nbody_small", n_balls=5,
                                  num_timesteps=10, num_inputs=1, traj_len=1)
    d[f"{dataset}::len"] = len(ds)
    for i in range(len(ds)):
        loc, vel, ea, q, locs_out, f0, out_idx = ds[i]
        for k, v in (("loc", loc), ("vel", vel), ("edge_attr", ea), ("charges", q), ("locs_out", locs_out),
                     ("frame_0", f0), ("out_indices", out_idx)):
            d[f"{dataset}::{i}::{k}"] = v.numpy() if torch.is_tensor(v) else np.asarray(v)
    return d


def items_multi(dataset, var_dt, seed):
    """num_inputs = 3 items; varDT draws random_ascending_tensor (torch.randperm) per item."""
    d = {}
    torch.manual_seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        ds = NBodyDynamicsDataset("train", data_dir=OUT, dataset=dataset, dataset_name="nbody_small", n_balls=5,
                                  num_timesteps=10, num_inputs=3, traj_len=1, varDT=var_dt)
    tag = f"{dataset}::multi{int(var_dt)}"
    d[f"{tag}::seed"] = seed
    for i in range(len(ds)):
        loc, vel, ea, q, locs_out, f0, out_idx = ds[i]
        for k, v in (("loc", loc), ("vel", vel), ("locs_out", locs_out), ("frame_0", f0), ("out_indices", out_idx)):
            d[f"{tag}::{i}::{k}"] = v.numpy() if torch.is_tensor(v) else np.asarray(v)
    return d


def segno_items_and_inputs():
    """SEGNO NBodyDataset items, and the inputs run_epoch (train_nbody.py:57-123) feeds the model
    and the criterion for every batch of a non-shuffled DataLoader (batch_size 3, drop_last as
    train_nbody.py:23 uses; the reference cannot featurise a short last batch), recorded with a
    stub model."""
    import types as _t
    from torch.utils.data import DataLoader
    sys.path.insert(0, os.path.join(REF, "SEGNO"))
    import dataset_nbody  # noqa: E402
    import train_nbody  # noqa: E402
    d = {}
    for dataset in ("charged", "gravity"):
        ds = dataset_nbody.NBodyDataset(OUT, partition="train", dataset=dataset, dataset_size="small", n_balls=5)
        d[f"segno_{dataset}::len"] = len(ds)
        d[f"segno_{dataset}::start"] = ds.start
        for i in range(len(ds)):
            for k, v in zip(("loc", "vel", "edge_attr", "charges"), ds[i]):
                d[f"segno_{dataset}::{i}::{k}"] = v.numpy()

    class Rec(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.calls = []

        def forward(self, his, x, edges, v, edge_attr, T=10, in_steps=None):
            self.calls.append({"h": his, "x": x, "v": v, "edge_attr": edge_attr,
                               "in_steps": in_steps if in_steps is not None else torch.zeros(0)})
            return (x[:, -1] if x.dim() == 3 else x), his, v

    for dataset in ("charged", "gravity"):
        for ni, var_dt in ((1, False), (3, False), (3, True)):
            ds = dataset_nbody.NBodyDataset(OUT, partition="train", dataset=dataset, dataset_size="small", n_balls=5)
            rec, ends = Rec(), []

            def crit(a, b):
                ends.append(b)
                return ((a - b) ** 2).mean()

            args = _t.SimpleNamespace(device="cpu", varDT=var_dt, batch_size=3, num_inputs=ni, traj_len=1)
            np.random.seed(7)
            with contextlib.redirect_stdout(io.StringIO()):
                train_nbody.run_epoch(rec, None, crit, 0, DataLoader(ds, batch_size=3, shuffle=False, drop_last=True), args,
                                      backprop=False, num_timesteps=10)
            tag = f"segno_{dataset}::in{ni}_{int(var_dt)}"
            d[f"{tag}::np_seed"] = 7
            d[f"{tag}::batches"] = len(rec.calls)
            for k, c in enumerate(rec.calls):
                for name, v in c.items():
                    d[f"{tag}::{k}::{name}"] = v.detach().numpy()
                d[f"{tag}::{k}::loc_end"] = ends[k].detach().numpy()
    return d


def metrics():
    g = torch.Generator().manual_seed(5)
    T, B, N = 20, 4, 5
    y = torch.randn(T, B * N, 3, generator=g)
    # prediction drifting away from the truth at a per-sample rate: correlations cross 0.5
    rate = torch.tensor([0.05, 0.3, 1.0, 0.0]).repeat_interleave(N).view(1, B * N, 1)
    x = y + torch.arange(T).view(T, 1, 1) * rate * torch.randn(T, B * N, 3, generator=g)
    corr, avg_steps, first_fail = ref_utils.pearson_correlation_batch(x, y, N)
    return {"in::x": x.numpy(), "in::y": y.numpy(), "cfg::N": N, "out::corr": corr.numpy(),
            "out::avg_num_steps": float(avg_steps), "out::first_failure_index": int(first_fail)}


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), **metrics())
    write_splits()
    fx = {}
    fx.update(items("charged"))
    fx.update(items("gravity"))
    for ds_name in ("charged", "gravity"):
        fx.update(items_multi(ds_name, False, 11))
        fx.update(items_multi(ds_name, True, 12))
    fx.update(segno_items_and_inputs())
    np.savez_compressed(os.path.join(HERE, "dataset_items.npz"), **fx)
    print("wrote nbody_tiny/ and dataset_items.npz")
