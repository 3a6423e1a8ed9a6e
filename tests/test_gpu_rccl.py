"""The RCCL code path of the data-parallel step, executed on the one GPU of the box (SURVEY §8 row e).

`FlatGrads.allreduce_`, `max_over_ranks` and `sum_over_ranks` skip their collective at world size 1,
and the gloo DP tests (tests/test_gpu_dp.py) carry theirs on the host, so without this test neither
`dist.init_process_group("nccl")`, the bench's `device_ids` barrier nor an RCCL all-reduce of a gfx950
tensor would ever run before the driver's multi-GPU bench. Here a world-size-1 `nccl` group on cuda:0
runs each of them directly (the reference's sync point is main_simulation_simple_no.py:278-280,
`loss.backward(); optimizer.step()`, single process):
- FlatGrads.exchange_() (the step's one all-reduce + / world) over the flat buffer of a real HIP
  EGNO backward: the buffer must come back bitwise unchanged (a sum over one rank);
- bench._barrier(dev) (RCCL barrier pinned to the rank's GPU) and the device-tensor path of the
  scalar reductions (bench timing: max over ranks);
- a 0.81 MB all-reduce timed over 50 calls (recorded, not asserted: the xGMI figure needs 8 GPUs).
The group lives in a spawned child process so the pytest process never holds an RCCL communicator.
"""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child(port, path):
    import time

    import numpy as np
    import torch.distributed as dist

    import bench
    from no_node_comparison_amd.sharding import FlatGrads, allreduce_scalar, max_over_ranks
    from tests.test_gpu_dp import N, T, _inputs
    from tests.test_gpu_parity import _egno
    from tests.test_gpu_train import _loss_like_reference

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    res = {}
    dist.init_process_group(backend="nccl")
    try:
        res["backend"] = dist.get_backend()
        res["world"] = dist.get_world_size()
        # a real HIP training step's gradients in the flat buffer
        m = _egno(T=T, seed=3).train()
        fg = FlatGrads(m.parameters())
        inp, target = _inputs(8, 0, 8)
        x, _, _ = m(inp["x"], inp["h"], [inp["row"], inp["col"]], inp["edge_fea"], v=inp["v"],
                    loc_mean=inp["loc_mean"], timesteps_out=inp["t_out"])
        loss, _ = _loss_like_reference(x, target, T, 8, N)
        torch.optim.Adam(m.parameters(), lr=1e-4).zero_grad()
        loss.backward()
        before = fg.gather_().clone()
        out = fg.exchange_()     # RCCL all-reduce (sum) of the gfx950 buffer, then / world
        torch.cuda.synchronize()
        res["flat_numel"] = int(out.numel())
        res["flat_device"] = str(out.device)
        res["flat_nonzero"] = int((before != 0).sum())
        res["flat_bitwise_unchanged"] = bool(torch.equal(before, out))
        res["grads_are_views"] = all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(fg.params, fg.views))
        # the bench's barrier and timing reduction on the device path
        bench._barrier(dev)
        bench.barrier_sync(1, dev)
        res["max_device"] = allreduce_scalar(3.25, dist.ReduceOp.MAX, dev)
        res["sum_device"] = allreduce_scalar(1.5, dist.ReduceOp.SUM, dev)
        res["max_over_ranks"] = max_over_ranks(2.0, dev)
        # all-reduce latency of the EGNO gradient buffer size (0.81 MB)
        buf = torch.arange(203_000, dtype=torch.float32, device=dev)
        ref = buf.clone()
        for _ in range(5):
            dist.all_reduce(buf)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            dist.all_reduce(buf)
        torch.cuda.synchronize()
        res["allreduce_0p81MB_us"] = (time.perf_counter() - t0) / 50 * 1e6
        res["allreduce_values_unchanged"] = bool(torch.equal(buf, ref))
        res["ok"] = True
    finally:
        dist.destroy_process_group()
    with open(path, "w") as f:
        json.dump(res, f)


def test_rccl_world1_flatgrads_barrier_and_scalar_reductions(tmp_path):
    path = str(tmp_path / "rccl.json")
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_child, args=(_free_port(), path))
    p.start()
    p.join(240)
    if p.is_alive():
        p.kill()
        pytest.fail("RCCL child did not finish in 240 s")
    assert p.exitcode == 0, f"RCCL child exit code {p.exitcode}"
    res = json.load(open(path))
    print("rccl:", res)
    assert res["ok"] and res["backend"] == "nccl" and res["world"] == 1
    assert res["flat_device"].startswith("cuda") and res["flat_nonzero"] > 0.5 * res["flat_numel"]
    assert res["flat_bitwise_unchanged"] and res["grads_are_views"]
    assert res["max_device"] == 3.25 and res["sum_device"] == 1.5 and res["max_over_ranks"] == 2.0
    assert res["allreduce_values_unchanged"]
    out = os.environ.get("NONODE_RCCL_REPORT")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
