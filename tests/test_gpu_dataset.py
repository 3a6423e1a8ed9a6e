"""Device batches (nonode_gather_batch) equal the reference loader's items collated."""
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
