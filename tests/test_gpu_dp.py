"""Data-parallel EGNO training step on the HIP kernels (SURVEY §8 row e, C4's exchange step).

The ranks share cuda:0 (the gloo backend carries the collective, so no second GPU is needed): each
runs the HIP training forward + backward on its half of the batch with the reference's loss
(main_simulation_simple_no.py:273-280), every p.grad is a view into one FlatGrads buffer, and ONE
all-reduce of that buffer (then / world) gives the step's gradients. They must equal the
single-process whole-batch gradients of the same kernels to 1e-5 max-norm relative per tensor (the
two runs only sum the same fp32 terms in a different order).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import check_rel, maxnorm_rel
from tests.test_gpu_parity import _dev, _egno, _egno_case
from tests.test_gpu_train import _loss_like_reference

pytestmark = pytest.mark.gpu
N, T = 20, 10
DPTOL = 1e-5


def _inputs(B, lo, hi):
    c = _egno_case(B, N, T, seed=11)
    n0, n1 = lo * N, hi * N                       # node rows of samples lo .. hi-1
    e0, e1 = lo * N * (N - 1), hi * N * (N - 1)   # edge rows (reference order: sample-major)
    sub = dict(x=c["x"][n0:n1], h=c["h"][n0:n1], v=c["v"][n0:n1], loc_mean=c["loc_mean"][n0:n1],
               edge_fea=c["edge_fea"][e0:e1], t_out=c["t_out"][lo:hi],
               row=c["row"][e0:e1] - n0, col=c["col"][e0:e1] - n0)
    target = np.random.default_rng(5).standard_normal((B, N, T, 3)).astype(np.float32)[lo:hi]
    return {k: _dev(v) for k, v in sub.items()}, _dev(target)


def _step_grads(B, lo, hi, allreduce):
    """(gradients after the optional all-reduce, this rank's local gradients before it)."""
    from no_node_comparison_amd.sharding import FlatGrads
    m = _egno(T=T, seed=3).train()
    fg = FlatGrads(m.parameters())
    inp, target = _inputs(B, lo, hi)
    x, _, _ = m(inp["x"], inp["h"], [inp["row"], inp["col"]], inp["edge_fea"], v=inp["v"],
                loc_mean=inp["loc_mean"], timesteps_out=inp["t_out"])
    loss, _ = _loss_like_reference(x, target, T, hi - lo, N)
    # the reference loop's order (main_simulation_simple_no.py:224,278-280): zero_grad() sets every
    # p.grad to None (dropping the FlatGrads views); allreduce_() must gather them back
    torch.optim.Adam(m.parameters(), lr=1e-4).zero_grad()
    loss.backward()
    local = {k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()}
    if allreduce:
        fg.allreduce_()
    torch.cuda.synchronize()
    return {k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()}, local


def _worker(rank, world, port, out, B):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        per = B // world
        g, local = _step_grads(B, rank * per, (rank + 1) * per, allreduce=True)
        np.savez(f"{out}.{rank}", **{"dp::" + k: v for k, v in g.items()}, **{"local::" + k: v for k, v in local.items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,B", [(2, 8), (2, 512), (8, 4096)])
def test_dp_step_on_hip_kernels_equals_whole_batch(tmp_path, world, B):
    """B=512: two ranks of 256 against the whole C4 shard. B=4096: C4's global batch as its eight
    ranks of 512 (all on the one GPU, gloo carrying the all-reduce) against the whole-4096 step on
    one GPU (the N=1 point of the strong-scaling curve).

    Checks, per parameter tensor:
      - the exchange itself: every rank holds exactly (g_0 + g_1) / 2 of the ranks' local gradients;
      - the result against the single-process whole-batch gradients, to DPTOL scaled by the
        conditioning of the split, max(|g_r|) / max(|g_whole|): a gradient whose shard terms largely
        cancel (the TimeConv weights at B=512) carries each shard's fp32 error relative to the larger
        shard magnitude, which no summation order removes."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "dp_grads")
    mp.start_processes(_worker, args=(world, port, out, B), nprocs=world, join=True, start_method="spawn")
    rk = [np.load(out + f".{r}.npz") for r in range(world)]
    whole, _ = _step_grads(B, 0, B, allreduce=False)
    nonzero = 0
    for k, ref in whole.items():
        dp = rk[0]["dp::" + k]
        assert all(np.array_equal(dp, r["dp::" + k]) for r in rk[1:]), k
        mean = sum(r["local::" + k].astype(np.float64) for r in rk) / world
        assert np.abs(dp - mean).max() <= 1e-6 * max(np.abs(mean).max(), 1e-30), k
        if np.abs(ref).max() == 0:   # the last layer's h update does not reach the position loss
            assert np.abs(dp).max() == 0, k
            continue
        nonzero += 1
        cond = max(np.abs(r["local::" + k]).max() for r in rk) / np.abs(ref).max()
        check_rel(f"dp {world}x{B // world} grad {k} (split cond {cond:.1f})", dp, ref, DPTOL * max(1.0, cond))
    assert nonzero > 50
