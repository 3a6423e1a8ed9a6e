"""Multi-rank path on the CPU: world_size-2 gloo process groups.

The rollout shards by sample with no collective in the data path (no_node_comparison_amd/sharding.py);
these tests check the shard assignment, the bench's per-rank inputs, the timing reduction, and that
per-rank results reassembled on rank 0 equal a single-process run of the whole batch. The per-rank
compute here is the oracle (test infrastructure; the kernels themselves need the GPU and are
covered by tests/test_gpu_parity.py, including batch independence).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import load_golden, params_of, maxnorm_rel
from no_node_comparison_amd.sharding import shard_range, gather_samples, max_over_ranks, sum_over_ranks


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, fn, *args):
    port = _free_port()
    mp.start_processes(_entry, args=(world, port, fn, args), nprocs=world, join=True, start_method="spawn")


def _entry(rank, world, port, fn, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,world", [(0, 2), (1, 2), (7, 2), (512, 8), (4096, 8), (13, 5)])
def test_shard_range_partitions(total, world):
    parts = [shard_range(total, world, r) for r in range(world)]
    assert parts[0][0] == 0 and parts[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    sizes = [hi - lo for lo, hi in parts]
    assert max(sizes) - min(sizes) <= 1


def test_shard_range_rejects():
    with pytest.raises(ValueError):
        shard_range(8, 2, 2)
    with pytest.raises(ValueError):
        shard_range(8, 0, 0)


def _reductions(rank, world):
    assert max_over_ranks(1.5 + rank) == 1.5 + world - 1
    assert sum_over_ranks(rank + 1) == world * (world + 1) / 2
    lo, hi = shard_range(7, world, rank)
    local = torch.full((hi - lo, 2), float(rank))
    full = gather_samples(local, 7)
    assert full.shape == (7, 2)
    for r in range(world):
        a, b = shard_range(7, world, r)
        assert torch.all(full[a:b] == r)


def test_reductions_gloo_ws2():
    _run(2, _reductions)


def _exchange_world1(rank, world):
    # the collectives FlatGrads / the bench timing run at world size 1 (the world-1 early returns
    # bypassed), here over gloo; tests/test_gpu_rccl.py runs the same calls over RCCL on the GPU
    from no_node_comparison_amd.sharding import FlatGrads, allreduce_scalar
    p = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(7))]
    fg = FlatGrads(p)
    for q in p:
        q.grad = torch.randn_like(q)
    before = fg.gather_().clone()
    assert torch.equal(fg.exchange_(), before)
    assert all(q.grad.data_ptr() == v.data_ptr() for q, v in zip(fg.params, fg.views))
    assert allreduce_scalar(2.5, dist.ReduceOp.MAX) == 2.5
    assert allreduce_scalar(2.5, dist.ReduceOp.SUM) == 2.5


def test_exchange_runs_at_world1_gloo():
    _run(1, _exchange_world1)


def test_flatgrads_world1_contract():
    """Without a process group (or at world size 1) allreduce_() exchanges nothing and returns None,
    leaving autograd's gradient tensors in place; reading .flat still gives this step's gradients
    (gathered on demand), also after zero_grad(set_to_none=True) dropped the views."""
    from no_node_comparison_amd.sharding import FlatGrads
    p = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(7))]
    fg = FlatGrads(p)
    assert fg.numel == 22
    for q in p:
        q.grad = None                       # optimizer.zero_grad() (torch 2.x default)
    g = [torch.randn(5, 3), torch.randn(7)]
    for q, gg in zip(p, g):
        q.grad = gg.clone()
    assert fg.allreduce_() is None
    assert all(torch.equal(q.grad, gg) for q, gg in zip(p, g))
    assert torch.equal(fg.flat, torch.cat([gg.reshape(-1) for gg in g]))
    assert all(q.grad.data_ptr() == v.data_ptr() for q, v in zip(fg.params, fg.views))


def _bench_shards(rank, world, B_per, N):
    import bench
    loc, vel, q = bench.rank_batch(B_per, world, rank, N, seed=99)
    gl, gv, gq = bench.synthetic_charged(B_per * world, N, 99)
    lo, hi = shard_range(B_per * world, world, rank)
    assert loc.shape == (B_per, N, 3)
    assert torch.equal(loc, gl[lo:hi]) and torch.equal(vel, gv[lo:hi]) and torch.equal(q, gq[lo:hi])
    full = gather_samples(loc, B_per * world)
    assert torch.equal(full, gl)


def test_bench_rank_inputs_gloo_ws2():
    _run(2, _bench_shards, 3, 5)


def _egno_sharded(rank, world, total):
    """Each rank runs the EGNO forward (oracle) on its sample shard; rank-0 reassembly must equal
    the whole-batch run (the path has no cross-sample coupling, egno.py:37-111)."""
    from oracle import egno as oe
    from oracle import harness as oh
    fx = load_golden("egno_fwd")
    p = params_of(fx)
    N = 5
    rng = np.random.default_rng(7)
    loc = rng.standard_normal((total, N, 3)).astype(np.float32)
    vel = rng.standard_normal((total, N, 3)).astype(np.float32)
    q = rng.choice([-1.0, 1.0], size=(total, N, 1)).astype(np.float32)
    T = 10

    def run(lo, hi):
        B = hi - lo
        r, c = oh.full_edges(B, N)
        qq = q[lo:hi].reshape(-1, 1)
        x, v, ea, nodes, lm = oh.prepare_inputs(loc[lo:hi], vel[lo:hi], qq[r] * qq[c], r, c, N, q[lo:hi])
        t_out = np.tile(np.arange(1, T + 1, dtype=np.float32), (B, 1))
        xo, vo, ho = oe.egno_forward(p, x, nodes, r, c, ea, v, lm, t_out, T=T)
        return xo.reshape(T, B, N, 3).transpose(1, 0, 2, 3)     # [B, T, N, 3] per sample

    lo, hi = shard_range(total, world, rank)
    mine = torch.from_numpy(np.ascontiguousarray(run(lo, hi)))
    full = gather_samples(mine, total).numpy()
    if rank == 0:
        ref = run(0, total)
        assert maxnorm_rel(full, ref) < 1e-6


def test_egno_sharded_equals_whole_batch_gloo_ws2():
    fx = load_golden("egno_fwd")
    if "w::embedding.weight" not in fx:
        pytest.skip("golden weights missing")
    _run(2, _egno_sharded, 5)


def _dp_grads(rank, world, total):
    """Each rank: the oracle's gradients of the mean loss over its sample shard, written into a
    FlatGrads buffer and all-reduced; the result must equal the whole-batch gradients (SURVEY
    §8e: one all-reduce of the flat gradient buffer, then / world)."""
    from oracle import egno_grad as og
    from oracle import harness as oh
    from no_node_comparison_amd.sharding import FlatGrads
    fx = load_golden("egno_fwd")
    p = {k: v.astype(np.float64) for k, v in params_of(fx).items()}
    N, T = 5, 10
    rng = np.random.default_rng(3)
    loc = rng.standard_normal((total, N, 3))
    vel = rng.standard_normal((total, N, 3))
    q = rng.choice([-1.0, 1.0], size=(total, N, 1))
    target = rng.standard_normal((total, N, T, 3))

    def grads(lo, hi):
        B = hi - lo
        r, c = oh.full_edges(B, N)
        qq = q[lo:hi].reshape(-1, 1)
        x, v, ea, nodes, lm = oh.prepare_inputs(loc[lo:hi], vel[lo:hi], qq[r] * qq[c], r, c, N, q[lo:hi])
        t_out = np.tile(np.arange(1, T + 1), (B, 1))
        _, _, g = og.egno_loss_and_grads(p, x, nodes, r, c, ea, v, lm, t_out, target[lo:hi], T=T)
        return g

    names = sorted(p)
    params = [torch.nn.Parameter(torch.zeros(p[k].shape, dtype=torch.float32)) for k in names]
    fg = FlatGrads(params)
    lo, hi = shard_range(total, world, rank)
    g = grads(lo, hi)
    for prm, k in zip(params, names):
        prm.grad.copy_(torch.from_numpy(g[k]))
    fg.allreduce_()
    if rank == 0:
        ref = grads(0, total)
        for prm, k in zip(params, names):
            want = ref[k]
            if np.abs(want).max() > 0:
                assert maxnorm_rel(prm.grad.numpy(), want) < 1e-5, k


def test_dp_allreduce_equals_whole_batch_gradients_gloo_ws2():
    _run(2, _dp_grads, 4)


def _reference_loop_order(rank, world, total, set_to_none):
    """The reference training loop's order (main_simulation_simple_no.py:224,278-280):
    optimizer.zero_grad(); loss.backward(); [one all-reduce]; optimizer.step(). zero_grad() drops
    the FlatGrads views (set_to_none=True is torch 2.x's default); the all-reduce must still reduce
    the gradients the optimizer steps on, for several steps in a row."""
    from no_node_comparison_amd.sharding import FlatGrads
    torch.manual_seed(0)
    data = torch.randn(total, 6)
    target = torch.randn(total, 2)

    def make():
        torch.manual_seed(1)
        return torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.SiLU(), torch.nn.Linear(16, 2)).double()

    lo, hi = shard_range(total, world, rank)
    m = make()
    fg = FlatGrads(m.parameters())
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    ref = make()
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-2)
    for step in range(3):
        opt.zero_grad(set_to_none=set_to_none)
        loss = torch.nn.functional.mse_loss(m(data[lo:hi].double()), target[lo:hi].double())
        loss.backward()
        fg.allreduce_()
        ropt.zero_grad()
        torch.nn.functional.mse_loss(ref(data.double()), target.double()).backward()
        for (k, p), q in zip(m.named_parameters(), ref.parameters()):
            assert p.grad.data_ptr() == fg.views[[id(x) for x in fg.params].index(id(p))].data_ptr()
            assert maxnorm_rel(p.grad.numpy(), q.grad.numpy()) < 1e-12, (step, k)
        opt.step()
        ropt.step()
    for p, q in zip(m.parameters(), ref.parameters()):
        assert maxnorm_rel(p.detach().numpy(), q.detach().numpy()) < 1e-12


@pytest.mark.parametrize("set_to_none", [True, False])
def test_flatgrads_under_reference_zero_grad_gloo_ws2(set_to_none):
    _run(2, _reference_loop_order, 8, set_to_none)


def _prewarm_agreement(rank, world, out_dir):
    """bench._prewarm: ranks of different speed stop after the same number of calls (a training
    step holds a collective, so unequal counts would deadlock the timed loop)."""
    import time
    import types
    import bench
    calls = []

    def call():
        calls.append(1)
        time.sleep(0.002 * (rank + 1))   # rank 1 is twice as slow as rank 0

    bench._prewarm(call, types.SimpleNamespace(prewarm_ms=40.0), torch.device("cpu"))
    with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
        f.write(str(len(calls)))


def test_bench_prewarm_stops_all_ranks_together(tmp_path):
    _run(2, _prewarm_agreement, str(tmp_path))
    counts = [int(open(tmp_path / f"r{r}").read()) for r in range(2)]
    assert counts[0] == counts[1] > 1
