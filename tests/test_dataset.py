"""The .npy dataset path against what the REFERENCE loader returns for the same
files (tests/golden/dataset_items.npz, recorded by make_golden_dataset.py from
EGNO/simulation/dataset_simple.py). CPU part here; the device batches are in test_gpu_dataset."""
import os

import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg  # noqa: F401
from no_node_comparison_amd.dataset import NBodyDynamicsDataset
from tests.conftest import GOLDEN, load_golden

TINY = os.path.join(GOLDEN, "nbody_tiny")


@pytest.mark.parametrize("dataset", ["charged", "gravity"])
def test_items_equal_reference_loader(dataset):
    g = load_golden("dataset_items")
    ds = NBodyDynamicsDataset("train", data_dir=TINY, dataset=dataset, dataset_name="nbody_small", n_balls=5,
                              num_timesteps=10)
    assert len(ds) == int(g[f"{dataset}::len"])
    for i in range(len(ds)):
        got = ds[i]
        for k, v in zip(("loc", "vel", "edge_attr", "charges", "locs_out", "frame_0", "out_indices"), got):
            want = g[f"{dataset}::{i}::{k}"]
            v = v.numpy() if torch.is_tensor(v) else np.asarray(v)
            assert v.shape == want.shape and np.array_equal(v, want), (dataset, i, k)


def test_max_samples_and_edges():
    ds = NBodyDynamicsDataset("train", data_dir=TINY, dataset="charged", n_balls=5, max_samples=3)
    assert len(ds) == 3 and ds.get_n_nodes() == 49
    r, c = ds.get_edges(2, 5)
    assert r.numel() == 2 * 20 and int(r[20]) == 5 and int(c[0]) == 1


@pytest.mark.parametrize("dataset", ["charged", "gravity"])
@pytest.mark.parametrize("var_dt", [False, True])
def test_multi_input_items_equal_reference_loader(dataset, var_dt):
    """num_inputs = 3 (dataset_simple.py:133-164): equispaced inputs, and varDT offsets drawn by
    random_ascending_tensor in the reference's order (torch seeded as when recorded)."""
    g = load_golden("dataset_items")
    tag = f"{dataset}::multi{int(var_dt)}"
    torch.manual_seed(int(g[f"{tag}::seed"]))
    ds = NBodyDynamicsDataset("train", data_dir=TINY, dataset=dataset, dataset_name="nbody_small", n_balls=5,
                              num_timesteps=10, num_inputs=3, varDT=var_dt)
    for i in range(len(ds)):
        loc, vel, _, _, locs_out, f0, oi = ds[i]
        for k, v in (("loc", loc), ("vel", vel), ("locs_out", locs_out), ("frame_0", f0), ("out_indices", oi)):
            want = g[f"{tag}::{i}::{k}"]
            assert v.shape == want.shape and np.array_equal(v.numpy(), want), (tag, i, k)


@pytest.mark.parametrize("dataset", ["charged", "gravity"])
def test_segno_items_equal_reference_loader(dataset):
    """SEGNO/dataset_nbody.py:7-94 items (whole trajectories, interaction-matrix edge features)."""
    from no_node_comparison_amd.dataset import NBodyDataset
    g = load_golden("dataset_items")
    ds = NBodyDataset(TINY, partition="train", dataset=dataset, dataset_size="small", n_balls=5)
    assert len(ds) == int(g[f"segno_{dataset}::len"]) and ds.start == int(g[f"segno_{dataset}::start"])
    for i in range(len(ds)):
        for k, v in zip(("loc", "vel", "edge_attr", "charges"), ds[i]):
            want = g[f"segno_{dataset}::{i}::{k}"]
            assert v.shape == want.shape and np.array_equal(v.numpy(), want), (dataset, i, k)
    r, c = ds.get_edges(3, 5)
    assert r.numel() == 60 and int(r[20]) == 5 and int(c[0]) == 1


def _c1_batches():
    """run_epoch's batches of the C1 split (non-shuffled, batch 8): the items collated."""
    fx = load_golden("egno_run_epoch")
    N, T, B = int(fx["cfg::N"]), int(fx["cfg::T"]), int(fx["cfg::B"])
    ds = NBodyDynamicsDataset("train", data_dir=os.path.join(GOLDEN, "nbody_c1"), dataset="charged",
                              dataset_name="nbody_small", n_balls=N, num_timesteps=T)
    for b0 in range(0, len(ds), B):
        items = [ds[i] for i in range(b0, min(b0 + B, len(ds)))]
        yield [torch.stack([torch.as_tensor(it[c]) for it in items]) for c in range(7)]


def test_oracle_run_epoch_c1_matches_reference():
    """Config C1 (EGNO forward, charged N=20, T=10, batch 8 via run_epoch, main_simulation_simple_no.py:
    190-307, backprop=False): the oracle in float64 gives the reference's per-batch per-frame losses
    and epoch loss (tests/golden/egno_run_epoch.npz, recorded from the reference's run_epoch)."""
    from oracle import egno as oe
    from oracle import harness as oh
    fx = load_golden("egno_run_epoch")
    N, T = int(fx["cfg::N"]), int(fx["cfg::T"])
    p = {k[3:]: v.astype(np.float64) for k, v in fx.items() if k.startswith("w::")}
    tot, cnt = 0.0, 0
    for k, (loc, vel, ea, q, loc_true, f0, oi) in enumerate(_c1_batches()):
        B = loc.shape[0]
        t_out = (oi - f0.reshape(-1, 1)).numpy()                  # out_indices -= in_indices.max()
        row, col = oh.full_edges(B, N)
        x, v, eattr, nodes, lm = oh.prepare_inputs(loc.double().numpy(), vel.double().numpy(),
                                                   ea.reshape(-1, 1).double().numpy(), row, col, N,
                                                   q.double().numpy())
        xo, _, _ = oe.egno_forward(p, x, nodes, row, col, eattr, v, lm, t_out, T=T)
        pred = xo.reshape(T, B, N, 3).transpose(1, 2, 0, 3)          # [B, N, T, 3]
        losses = ((pred - loc_true.double().numpy()) ** 2).mean((0, 1, 3))
        np.testing.assert_allclose(losses, fx["eval::losses"][k], rtol=1e-5)
        tot += float(losses[-1]) * B
        cnt += B
    assert abs(tot / cnt - float(fx["eval::avg_loss"])) <= 1e-5 * abs(float(fx["eval::avg_loss"]))
