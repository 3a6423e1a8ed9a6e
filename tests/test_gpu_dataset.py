"""Device batches (nonode_gather_batch / nonode_gather_rows) equal the reference loaders' items collated, and
segno_batch_inputs equals the model inputs the reference run_epoch builds."""
import os

import numpy as np
import pytest
import torch

from no_node_comparison_amd.dataset import DeviceLoader, NBodyDynamicsDataset
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu
TINY = os.path.join(GOLDEN, "nbody_tiny")


@pytest.mark.parametrize("dataset,bs", [("charged", 4), ("gravity", 3)])
def test_device_batches_equal_collated_items(dataset, bs):
    ds = NBodyDynamicsDataset("train", data_dir=TINY, dataset=dataset, n_balls=5, num_timesteps=10)
    dl = DeviceLoader(ds, batch_size=bs, shuffle=True, generator=torch.Generator().manual_seed(0))
    seen = []
    order = torch.randperm(len(ds), generator=torch.Generator().manual_seed(0))
    for k, batch in enumerate(dl):
        idx = order[k * bs:(k + 1) * bs].tolist()
        seen += idx
        items = [ds[i] for i in idx]
        for c, got in enumerate(batch):
            want = torch.stack([torch.as_tensor(it[c]) for it in items])
            assert got.is_cuda and tuple(got.shape) == tuple(want.shape), c
            assert torch.equal(got.cpu(), want.to(got.dtype)), c
    assert sorted(seen) == list(range(len(ds)))


def test_prepare_inputs_on_device_batch():
    """The batch feeds prepare_inputs directly (run_epoch, main_simulation_simple_no.py:200-218)."""
    import no_node_comparison_amd as pkg
    from oracle import harness as oh
    ds = NBodyDynamicsDataset("train", data_dir=TINY, dataset="charged", n_balls=5, num_timesteps=10)
    loc, vel, ea, q, lt, f0, oi = DeviceLoader(ds, batch_size=6).batch(range(6))
    edges = ds.get_edges(6, 5)
    x, v, eattr, nodes, lm = pkg.harness.prepare_inputs(loc, vel, ea.reshape(-1, 1), edges, 5, 1, q)
    row, col = oh.full_edges(6, 5)
    ref = oh.prepare_inputs(loc.cpu().numpy(), vel.cpu().numpy(), ea.reshape(-1, 1).cpu().numpy(), row, col, 5,
                            q.cpu().numpy())
    for got, want in zip((x, v, eattr, nodes, lm), ref):
        np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("dataset,var_dt", [("charged", False), ("charged", True), ("gravity", True)])
def test_multi_input_device_batches_equal_collated_items(dataset, var_dt):
    """num_inputs = 3: loc / vel [B, 3, N, 3], frame_0 [B, 3]; with varDT the loader draws each
    sample's input offsets in batch order, as the reference's __getitem__ calls do."""
    from tests.conftest import load_golden
    g = load_golden("dataset_items")
    tag = f"{dataset}::multi{int(var_dt)}"
    ds = NBodyDynamicsDataset("train", data_dir=TINY, dataset=dataset, n_balls=5, num_timesteps=10, num_inputs=3,
                              varDT=var_dt)
    torch.manual_seed(int(g[f"{tag}::seed"]))
    dl = DeviceLoader(ds, batch_size=2)
    i = 0
    for batch in dl:
        loc, vel, ea, q, lt, f0, oi = batch
        assert loc.shape == (2, 3, 5, 3) and f0.shape == (2, 3)
        for b in range(2):
            for c, k in ((loc, "loc"), (vel, "vel"), (lt, "locs_out"), (f0, "frame_0"), (oi, "out_indices")):
                want = g[f"{tag}::{i}::{k}"]
                assert np.array_equal(c[b].cpu().numpy(), want.astype(c.cpu().numpy().dtype)), (i, k)
            i += 1
    assert i == len(ds)


def test_device_loader_rejects_out_of_range_indices():
    ds = NBodyDynamicsDataset("train", data_dir=TINY, dataset="charged", n_balls=5, num_timesteps=10)
    dl = DeviceLoader(ds, batch_size=2)
    with pytest.raises(IndexError):
        dl.batch([0, len(ds)])
    with pytest.raises(IndexError):
        dl.batch([-1])


@pytest.mark.parametrize("dataset", ["charged", "gravity"])
def test_segno_device_batches_equal_collated_items(dataset):
    from no_node_comparison_amd.dataset import NBodyDataset, SegnoDeviceLoader
    ds = NBodyDataset(TINY, partition="train", dataset=dataset, dataset_size="small", n_balls=5)
    dl = SegnoDeviceLoader(ds, batch_size=3, shuffle=True, generator=torch.Generator().manual_seed(1))
    order = torch.randperm(len(ds), generator=torch.Generator().manual_seed(1))
    seen = []
    for k, batch in enumerate(dl):
        idx = order[k * 3:(k + 1) * 3].tolist()
        seen += idx
        for c, got in enumerate(batch):
            want = torch.stack([ds[i][c] for i in idx])
            assert got.is_cuda and torch.equal(got.cpu(), want), c
    assert sorted(seen) == list(range(len(ds)))
    with pytest.raises(IndexError):
        dl.batch([len(ds)])


@pytest.mark.parametrize("dataset", ["charged", "gravity"])
@pytest.mark.parametrize("ni,var_dt", [(1, False), (3, False), (3, True)])
def test_segno_batch_inputs_equal_reference_run_epoch(dataset, ni, var_dt):
    """segno_batch_inputs reproduces what the reference run_epoch feeds the model and the criterion
    (train_nbody.py:76-123, recorded by make_golden_dataset.py with a stub model; numpy seeded as
    there for the varDT gap draws)."""
    from no_node_comparison_amd.dataset import NBodyDataset, SegnoDeviceLoader, segno_batch_inputs
    from tests.conftest import load_golden
    g = load_golden("dataset_items")
    tag = f"segno_{dataset}::in{ni}_{int(var_dt)}"
    ds = NBodyDataset(TINY, partition="train", dataset=dataset, dataset_size="small", n_balls=5)
    dl = SegnoDeviceLoader(ds, batch_size=3, drop_last=True)
    rng = np.random.RandomState(int(g[f"{tag}::np_seed"]))
    n = 0
    for k, batch in enumerate(dl):
        h, loc, vel, ea, loc_end, in_steps, _ = segno_batch_inputs(batch, ds.start, 10, ni, var_dt, rng=rng)
        for got, name in ((h, "h"), (loc, "x"), (vel, "v"), (ea, "edge_attr"), (loc_end, "loc_end")):
            want = g[f"{tag}::{k}::{name}"]
            assert tuple(got.shape) == want.shape, name
            np.testing.assert_allclose(got.cpu().numpy(), want, rtol=2e-7, atol=1e-7, err_msg=name)
        if ni > 1:
            assert np.array_equal(in_steps.cpu().numpy(), g[f"{tag}::{k}::in_steps"])
        n += 1
    assert n == int(g[f"{tag}::batches"])


def _run_epoch_c1(model, loader, N, T, optimizer=None):
    """run_epoch (main_simulation_simple_no.py:190-307, rollout=False) over the device loader with the
    drop-in EGNO: the reference's call sequence, criterion and loss bookkeeping."""
    import no_node_comparison_amd as pkg
    crit = torch.nn.MSELoss(reduction="none")
    model.train() if optimizer is not None else model.eval()
    rec, tot, cnt = [], 0.0, 0
    for loc, vel, edge_attr, charges, loc_true, in_indices, out_indices in loader:
        out_indices = out_indices - in_indices.max()
        in_indices = in_indices - in_indices.max()
        B = loc.shape[0]
        edges = pkg.harness.get_edges(B, N, loc.device)
        if optimizer is not None:
            optimizer.zero_grad()
        x, v, ea, nodes, lm = pkg.harness.prepare_inputs(loc, vel, edge_attr.reshape(-1, edge_attr.shape[-1]), edges,
                                                         N, 1, charges)
        with torch.set_grad_enabled(optimizer is not None):
            xo, _, _ = model(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_in=in_indices, timesteps_out=out_indices)
            pred = xo.reshape(T, -1, 3).transpose(0, 1).reshape(B, N, T, 3)
            losses = crit(pred, loc_true[:, :, :T]).mean((0, 1, 3))
            if optimizer is not None:
                losses.mean().backward()
                optimizer.step()
        rec.append(losses.detach().cpu().numpy())
        tot += float(losses[-1]) * B
        cnt += B
    return tot / cnt, np.stack(rec)


def test_run_epoch_c1_with_drop_in_egno_matches_reference():
    """Config C1 end to end through the caller it names: the reference's run_epoch loop (eval pass and
    one Adam training epoch, lr 1e-4 / wd 1e-8) with the drop-in EGNO and the device loader gives the
    per-batch per-frame losses and the epoch loss the reference's run_epoch reported on the same split
    (tests/golden/egno_run_epoch.npz)."""
    import no_node_comparison_amd as pkg
    from tests.conftest import load_golden
    fx = load_golden("egno_run_epoch")
    N, T, B = int(fx["cfg::N"]), int(fx["cfg::T"]), int(fx["cfg::B"])
    ds = NBodyDynamicsDataset("train", data_dir=os.path.join(GOLDEN, "nbody_c1"), dataset="charged",
                              dataset_name="nbody_small", n_balls=N, num_timesteps=T)
    sd = {k[3:]: torch.tensor(v) for k, v in fx.items() if k.startswith("w::")}

    def model():
        m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2, num_timesteps=T,
                     time_emb_dim=32, device="cuda")
        m.load_state_dict(sd)
        return m

    avg, losses = _run_epoch_c1(model(), DeviceLoader(ds, batch_size=B), N, T)
    np.testing.assert_allclose(losses, fx["eval::losses"], rtol=1e-5)
    assert abs(avg - float(fx["eval::avg_loss"])) <= 1e-5 * abs(float(fx["eval::avg_loss"]))
    m = model()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4, weight_decay=1e-8)
    avg, losses = _run_epoch_c1(m, DeviceLoader(ds, batch_size=B), N, T, opt)
    np.testing.assert_allclose(losses, fx["train::losses"], rtol=1e-5)
    assert abs(avg - float(fx["train::avg_loss"])) <= 1e-5 * abs(float(fx["train::avg_loss"]))
