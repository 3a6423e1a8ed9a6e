"""Benchmark of the EGNO / SEGNO trajectory-rollout hot path on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` — one process per GPU (launched
by torch.distributed.run for N > 1), W untimed steps, then exactly K timed steps bracketed by a
barrier + synchronize, max over ranks; rank 0 prints ONE JSON line.

A "step" is one pass of the hot path over one batch of synthetic input. Default workload
(BASELINE.json configs[1], "C2"): EGNO 4 layers, charged N=20, T=10, B=512 per GPU, fp32 — one
model call producing T=10 frames for all B trajectories. Ranks are independent replicas on their
own batch shard (the path shards by sample; inference has no collective), so scaling is weak.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "N-body trajectories/s (B×T, N=20 rollout) + pos-MSE vs ref, 1/2/4/8 MI355X"
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 vector = f32-input MFMA peak (spec)
FP16_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md: dense FP16/BF16 MFMA peak (spec)
# The layer kernel delivers fp32-accurate 64x64 products as fp16x3 split MFMAs (W_lo x_hi + W_hi x_lo +
# W_hi x_hi): three dense fp16 MFMAs per fp32 product, so the matrix-core ceiling
# for its algorithmic (fp32-equivalent) FLOPs is the dense fp16 peak / 3.
FP16X3_PEAK_TFLOPS = FP16_PEAK_TFLOPS / 3.0
HBM_PEAK_GBS = 8000.0

# Algorithmic work of one egnn_layer_kernel launch (SURVEY §8d decomposed count):
#   per edge: 8448 MAC (W2 64x64 + Wc1 64x64 + w_s/W_e/w_c2 vectors)
#   per node: 24640 MAC (P, Q projections 2x64x64, node_v 64x64+64, node MLP 128x64+64x64)
MAC_PER_EDGE = 8448
MAC_PER_NODE = 24640
# SEGNO_GCL (gcl.py:71-119): per edge W2 + Wc1 + vectors as EGNO; per node P, Q + node MLP (no phi_v)
MAC_PER_EDGE_SEGNO = 8448
MAC_PER_NODE_SEGNO = 20480


def synthetic_charged(B, N, seed):
    """SURVEY §8d generator: positions ~ N(0, sigma^2), sigma = (N/5)^(1/3); unit direction x 0.5
    velocities; charges +-1 with p = 1/2."""
    g = torch.Generator().manual_seed(seed)
    sigma = (N / 5.0) ** (1.0 / 3.0)
    loc = torch.randn(B, N, 3, generator=g) * sigma
    vel = torch.randn(B, N, 3, generator=g)
    vel = vel / vel.norm(dim=-1, keepdim=True) * 0.5
    q = (torch.randint(0, 2, (B, N, 1), generator=g) * 2 - 1).float()
    return loc, vel, q


def rank_batch(B_per, world, rank, N, seed):
    """This rank's shard of the global synthetic batch of B_per * world samples (weak scaling: the
    per-GPU batch is fixed). Concatenating every rank's shard gives the global batch."""
    from no_node_comparison_amd.sharding import shard_range
    loc, vel, q = synthetic_charged(B_per * world, N, seed)
    lo, hi = shard_range(B_per * world, world, rank)
    return loc[lo:hi], vel[lo:hi], q[lo:hi]


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NONODE_DIST_BACKEND=gloo rehearses the multi-rank bench on a box with fewer GPUs than ranks
    # (ranks then share GPUs round-robin); the default on a GPU node is RCCL ("nccl"), one GPU per rank
    gpu = torch.cuda.is_available()
    if gpu:
        local = local % torch.cuda.device_count()
    if world > 1:
        backend = os.environ.get("NONODE_DIST_BACKEND") or ("nccl" if gpu else "gloo")
        if gpu:
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    dev = torch.device(f"cuda:{local}" if gpu else "cpu")
    return world, rank, dev


def _barrier(dev):
    # NCCL (RCCL) barrier on this rank's own GPU, not a guessed one
    if dev.type == "cuda" and dist.get_backend() == "nccl":
        dist.barrier(device_ids=[dev.index])
    else:
        dist.barrier()


def barrier_sync(world, dev):
    if world > 1:
        _barrier(dev)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _prewarm(call, args, dev):
    """Untimed calls of the same step for at least --prewarm-ms of wall time, before the W warmup
    steps: an idle GPU ramps its clocks during them (on a fresh MI355X box the first ~10 ms of C3
    ran at half speed). Reported as "prewarm_ms" in the JSON line."""
    if args.prewarm_ms <= 0:
        return
    from no_node_comparison_amd.sharding import max_over_ranks
    t0 = time.perf_counter()
    while True:
        call()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        # every rank stops after the same call (a training step holds a collective)
        if max_over_ranks((time.perf_counter() - t0) * 1e3, dev) >= args.prewarm_ms:
            break


def build_egno_case(B, N, T, seed, dev, world=1, rank=0):
    import no_node_comparison_amd as pkg
    loc, vel, q = rank_batch(B, world, rank, N, seed)
    edges = pkg.harness.get_edges(B, N, dev)
    loc, vel, q = loc.to(dev), vel.to(dev), q.to(dev)
    qq = q.reshape(-1, 1)
    eao = qq[edges[0]] * qq[edges[1]]
    x, v, ea, nodes, lm = pkg.harness.prepare_inputs(loc, vel, eao, edges, N, 1, q)
    t_out = torch.arange(1, T + 1, device=dev).repeat(B, 1)
    return dict(x=x, h=nodes, edges=edges, edge_fea=ea, v=v, loc_mean=lm, t_out=t_out)


def cpu_baseline_egno(model, case, N, T, budget_s=12.0, max_b=64):
    """Oracle (numpy restatement, test infrastructure) on the host cores over a bounded sample of
    the same workload: the first samples of rank 0's batch."""
    from oracle import egno as oe
    from oracle import harness as oh
    try:
        import threadpoolctl
        cores = max(i.get("num_threads", 1) for i in threadpoolctl.threadpool_info()) or 1
    except Exception:
        cores = os.cpu_count() or 1
    p = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    Bc = max_b
    r, c = oh.full_edges(Bc, N)
    sl = lambda t, w: t[: Bc * w].detach().cpu().numpy()  # noqa: E731
    args = dict(x=sl(case["x"], N), h=sl(case["h"], N), row=r, col=c, edge_fea=sl(case["edge_fea"], N * (N - 1)),
                v=sl(case["v"], N), loc_mean=sl(case["loc_mean"], N), t_out=case["t_out"][:Bc].cpu().numpy())
    done, t0, out = 0, time.perf_counter(), None
    while True:
        out = oe.egno_forward(p, **args, T=T)
        done += 1
        if time.perf_counter() - t0 > budget_s or done >= 20:
            break
    el = time.perf_counter() - t0
    return {"value": Bc * done / el, "unit": "trajectories/s", "cores": int(cores), "kind": "port",
            "sample": f"oracle/egno.py (numpy fp32) EGNO forward, B={Bc} of the same synthetic batch, "
                      f"N={N}, T={T}, {done} calls in {el:.1f} s"}, out, Bc


def run_egno(args, world, rank, dev):
    import no_node_comparison_amd as pkg
    B, N, T = args.batch, 20, 10
    torch.manual_seed(0)
    model = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                     num_timesteps=T, time_emb_dim=32, device=dev).eval()
    case = build_egno_case(B, N, T, seed=1234, dev=dev, world=world, rank=rank)
    from no_node_comparison_amd import _lib
    call = lambda: model(case["x"], case["h"], case["edges"], case["edge_fea"], v=case["v"],  # noqa: E731
                         loc_mean=case["loc_mean"], timesteps_out=case["t_out"])
    with torch.no_grad():
        _prewarm(call, args, dev)
        for _ in range(args.warmup):
            out = call()
        barrier_sync(world, dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = call()
        barrier_sync(world, dev)
        el = time.perf_counter() - t0
        # kernel durations for the roofline: a separate instrumented pass over the same workload
        # (hipEvents recorded around every launch on its stream; kept out of the timed loop above)
        records = []
        if args.kernel_events:
            _lib.profile_begin(16 * args.steps + 64)
            for _ in range(args.steps):
                out = call()
            records = _lib.profile_end()
    layer_events = [ms for kind, ms in records if kind == _lib.VARIANT_EGNO]
    tconv_ms = [ms for kind, ms in records if kind in (2, 3)]
    from no_node_comparison_amd.sharding import max_over_ranks
    el = max_over_ranks(el, dev)
    ms = el / args.steps * 1e3
    value = B * world * args.steps / el
    res = {"metric": METRIC, "value": value, "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32", "data": "synthetic (SURVEY §8d charged generator, seeded)",
           "frames_per_s": value * T,
           "config": {"workload": "C2: EGNO forward (4 layers, hidden 64, 2 modes), charged N=20, T=10, "
                                  f"B={B} per GPU", "batch_per_gpu": B, "global_batch": B * world, "n_balls": N,
                      "num_timesteps": T, "parallelism": f"batch-sharded replicas x{world} (no collective)"}}
    # dominant kernel: egnn_layer_kernel, timed live with HIP events on the launch stream
    if layer_events:
        durs = layer_events
        avg_ms = float(np.mean(durs))
        E = T * B * N * (N - 1)
        n = T * B * N
        flop = 2.0 * (E * MAC_PER_EDGE + n * MAC_PER_NODE)
        achieved = flop / (avg_ms * 1e-3) / 1e12
        res["roofline"] = {"kernel": "egnn_layer_kernel<EGNO>", "bound": "mfma", "achieved": achieved,
                           "peak": FP16X3_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP16X3_PEAK_TFLOPS,
                           "peak_basis": "dense fp16 MFMA peak / 3 (fp16x3 split products)",
                           "frac_of_fp32_mfma_peak": achieved / FP32_PEAK_TFLOPS,
                           "traffic": pmc_traffic("egnn_layer_kernel<EGNO>"), "avg_launch_ms": avg_ms,
                           "algorithmic_gflop_per_launch": flop / 1e9, "launches_timed": len(durs),
                           "tconv_avg_launch_ms": float(np.mean(tconv_ms)) if tconv_ms else None}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, ref_out, Bc = cpu_baseline_egno(model, case, N, T)
        res["cpu_baseline"] = cb
        x = out[0].view(T, B, N, 3)[:, :Bc].reshape(-1, 3).double().cpu().numpy()
        xr = ref_out[0]
        res["parity"] = {"pos_mse_vs_oracle": float(np.mean((x - xr) ** 2)),
                         "pos_maxnorm_rel_vs_oracle": float(np.abs(x - xr).max() / np.abs(xr).max()),
                         "samples_checked": Bc}
    return res


def synthetic_gravity(B, N, seed):
    """SURVEY §8d gravity generator: masses 1 + 0.1 N(0,1); positions, velocities ~ N(0,1) with the
    centre-of-mass velocity removed (synthetic_sim.py:370-378)."""
    g = torch.Generator().manual_seed(seed)
    mass = 1.0 + 0.1 * torch.randn(B, N, 1, generator=g)
    loc = torch.randn(B, N, 3, generator=g)
    vel = torch.randn(B, N, 3, generator=g)
    vel = vel - (mass * vel).sum(1, keepdim=True) / mass.sum(1, keepdim=True)
    return loc, vel, mass


def c5_substeps(total=50, seed=0):
    """C5 multi-horizon substep list: draws in [5, 10) from default_rng(0) until they sum to 50
    (the last one clipped), SURVEY §8d."""
    rng = np.random.default_rng(seed)
    out = []
    while sum(out) < total:
        out.append(int(min(rng.integers(5, 10), total - sum(out))))
    return out


def run_segno(args, world, rank, dev, gravity=False):
    """C3 (SEGNO charged N=20, B=512 per GPU, one forward of 10 substeps) or C5 (SEGNO gravity
    N=100, B=256 per GPU, a 50-frame multi-horizon rollout: segments of c5_substeps() substeps)."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd.sharding import max_over_ranks
    N = 100 if gravity else 20
    B = args.batch if args.batch != 512 or not gravity else 256
    torch.manual_seed(0)
    model = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=4, recurrent=True, device=dev).eval()
    gen = synthetic_gravity if gravity else synthetic_charged
    loc, vel, q = gen(B * world, N, 4321)
    from no_node_comparison_amd.sharding import shard_range
    lo, hi = shard_range(B * world, world, rank)
    loc, vel, q = loc[lo:hi].to(dev), vel[lo:hi].to(dev), q[lo:hi].to(dev)
    edges = pkg.harness.get_edges(B, N, dev)
    x = loc.reshape(-1, 3)
    v = vel.reshape(-1, 3)
    qq = q.reshape(-1, 1)
    ea = torch.cat([qq[edges[0]] * qq[edges[1]], ((x[edges[0]] - x[edges[1]]) ** 2).sum(-1, keepdim=True)], 1)
    his = v.norm(dim=-1, keepdim=True)
    steps = c5_substeps() if gravity else [10]

    def call():
        if gravity:   # rollout_fn (train_nbody.py:200-236) as one native call: re-featurisation + energy
            return pkg.harness.segno_rollout(model, his, x, edges, v, ea, len(steps), num_steps=steps, charges=q,
                                             energy_dataset="gravity", batch_size=B)[0]
        return model(his, x, edges, v, ea, T=steps[0])[0]

    from no_node_comparison_amd import _lib
    with torch.no_grad():
        _prewarm(call, args, dev)
        for _ in range(args.warmup):
            call()
        barrier_sync(world, dev)
        if args.kernel_events:
            _lib.profile_begin(8 * args.steps * len(steps) + 64)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            call()
        barrier_sync(world, dev)
        el = time.perf_counter() - t0
        records = _lib.profile_end() if args.kernel_events else []
    el = max_over_ranks(el, dev)
    value = B * world * args.steps / el
    name = "C5: SEGNO gravity N=100, 50-frame multi-horizon rollout (nonode_segno_rollout: per-segment " \
        "re-featurisation + gravity energy on the GPU)" if gravity else \
        "C3: SEGNO charged N=20, 10 integrator substeps (one fused launch)"
    res = {"metric": METRIC, "value": value, "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic (SURVEY §8d, seeded)",
           "config": {"workload": f"{name}, B={B} per GPU", "batch_per_gpu": B, "global_batch": B * world,
                      "n_balls": N, "substeps": steps, "parallelism": f"batch-sharded replicas x{world}"}}
    layer = [ms for kind, ms in records if kind == _lib.VARIANT_SEGNO]
    if layer:
        E = B * N * (N - 1) * sum(steps) / len(steps)
        n = B * N * sum(steps) / len(steps)
        avg = float(np.mean(layer))
        flop = 2.0 * (E * MAC_PER_EDGE_SEGNO + n * MAC_PER_NODE_SEGNO)
        ach = flop / (avg * 1e-3) / 1e12
        res["roofline"] = {"kernel": "egnn_layer_kernel<SEGNO> (fused substeps)", "bound": "mfma",
                           "achieved": ach, "peak": FP16X3_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ach / FP16X3_PEAK_TFLOPS,
                           "peak_basis": "dense fp16 MFMA peak / 3 (fp16x3 split products)",
                           "frac_of_fp32_mfma_peak": ach / FP32_PEAK_TFLOPS,
                           "traffic": None, "avg_launch_ms": avg, "algorithmic_gflop_per_launch": flop / 1e9,
                           "launches_timed": len(layer)}
    return res


def run_egno_train(args, world, rank, dev):
    """C4: EGNO training step, charged N=20, T=10, B=512 per GPU (4096 over 8 GPUs): forward with
    saved state, the reference loss (main_simulation_simple_no.py:273-280), backward through the HIP
    kernels, ONE all-reduce of the flat gradient buffer (RCCL over xGMI), Adam(lr 1e-4, wd 1e-8,
    model_confs.yaml:15-17)."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd.sharding import FlatGrads, max_over_ranks
    from no_node_comparison_amd import _lib
    B, N, T = args.batch, 20, 10
    torch.manual_seed(0)
    model = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                     num_timesteps=T, time_emb_dim=32, device=dev).train()
    case = build_egno_case(B, N, T, seed=1234, dev=dev, world=world, rank=rank)
    g = torch.Generator().manual_seed(777 + rank)
    loc_true = torch.randn(B, N, T, 3, generator=g).to(dev)
    fg = FlatGrads(model.parameters())
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, weight_decay=1e-8)

    def step():
        fg.zero_()
        x, _, _ = model(case["x"], case["h"], case["edges"], case["edge_fea"], v=case["v"],
                        loc_mean=case["loc_mean"], timesteps_out=case["t_out"])
        pred = x.reshape(T, B, N, 3).permute(1, 2, 0, 3)
        loss = torch.nn.functional.mse_loss(pred, loc_true, reduction="none").mean((0, 1, 3)).mean()
        loss.backward()
        fg.allreduce_()
        opt.step()
        return loss

    _prewarm(step, args, dev)
    for _ in range(args.warmup):
        step()
    barrier_sync(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    barrier_sync(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, dev)
    value = B * world * args.steps / el
    return {"metric": METRIC, "value": value, "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic (SURVEY §8d, seeded)",
            "loss": float(loss.detach()),
            "config": {"workload": f"C4: EGNO training step (fwd + bwd + 1 all-reduce + Adam), charged N=20, T=10, "
                                   f"B={B} per GPU", "batch_per_gpu": B, "global_batch": B * world, "n_balls": N,
                       "num_timesteps": T, "grad_buffer_bytes": fg.flat.numel() * 4,
                       "parallelism": f"data-parallel x{world}, one RCCL all-reduce per step"}}


def _host_cores():
    try:
        import threadpoolctl
        return max(i.get("num_threads", 1) for i in threadpoolctl.threadpool_info()) or 1
    except Exception:
        return os.cpu_count() or 1


def run_egno_rollout(args, world, rank, dev):
    """rollout_fn (main_simulation_simple_no.py:342-384) at the C2 shape, traj_len =
    10 segments (the script's --traj_len default, :79) with per-frame charged energies, as ONE
    native call (nonode_egno_rollout: 10 forwards + on-device re-featurisation + energy). A
    trajectory is one 100-frame rollout of one sample."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd import _lib
    from no_node_comparison_amd.sharding import max_over_ranks
    B, N, T, L = args.batch, 20, 10, 10
    torch.manual_seed(0)
    model = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                     num_timesteps=T, time_emb_dim=32, device=dev).eval()
    loc, vel, q = rank_batch(B, world, rank, N, 1234)
    edges = pkg.harness.get_edges(B, N, dev)
    loc, vel, q = loc.to(dev), vel.to(dev), q.to(dev)
    qq = q.reshape(-1, 1)
    eao = qq[edges[0]] * qq[edges[1]]
    x, v, ea, nodes, lm = pkg.harness.prepare_inputs(loc, vel, eao, edges, N, 1, q)
    t_all = torch.arange(1, T * L + 1, device=dev, dtype=torch.float32).repeat(B, 1)
    call = lambda: pkg.harness.egno_rollout(model, nodes, x, edges, v, eao, ea, lm, N, L, B,  # noqa: E731
                                            charges=q.reshape(-1), num_steps=T, timesteps_out=t_all,
                                            energy_dataset="charged")
    _prewarm(call, args, dev)
    for _ in range(args.warmup):
        out = call()
    barrier_sync(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = call()
    barrier_sync(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, dev)
    records = []
    if args.kernel_events:
        _lib.profile_begin(16 * L * 2 + 64)
        out = call()
        records = _lib.profile_end()
    value = B * world * args.steps / el
    res = {"metric": METRIC, "value": value, "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic (SURVEY §8d, seeded)",
           "frames_per_s": value * T * L,
           "config": {"workload": f"f1: EGNO rollout_fn, charged N=20, T=10, traj_len={L} (100 frames + per-frame "
                                  f"energy), B={B} per GPU", "batch_per_gpu": B, "global_batch": B * world,
                      "n_balls": N, "num_timesteps": T, "traj_len": L,
                      "parallelism": f"batch-sharded replicas x{world} (no collective)"}}
    layer = [ms for kind, ms in records if kind == _lib.VARIANT_EGNO]
    if layer:
        avg = float(np.mean(layer))
        flop = 2.0 * (T * B * N * (N - 1) * MAC_PER_EDGE + T * B * N * MAC_PER_NODE)
        ach = flop / (avg * 1e-3) / 1e12
        res["roofline"] = {"kernel": "egnn_layer_kernel<EGNO>", "bound": "mfma", "achieved": ach,
                           "peak": FP16X3_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ach / FP16X3_PEAK_TFLOPS,
                           "peak_basis": "dense fp16 MFMA peak / 3 (fp16x3 split products)",
                           "frac_of_fp32_mfma_peak": ach / FP32_PEAK_TFLOPS,
                           "traffic": None, "avg_launch_ms": avg, "algorithmic_gflop_per_launch": flop / 1e9,
                           "launches_timed": len(layer),
                           "layer_kernel_share": float(np.sum(layer)) / (el / args.steps * 1e3)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import harness as oh
        p = {k: t.detach().cpu().numpy() for k, t in model.state_dict().items()}
        Bc = 8
        r, c = oh.full_edges(Bc, N)
        cut = lambda t, w: t[: Bc * w].detach().cpu().numpy()  # noqa: E731
        t_c = t_all[:Bc].cpu().numpy()
        done, t0 = 0, time.perf_counter()
        while True:
            ref, _, _ = oh.egno_rollout(p, cut(nodes, N), cut(x, N), r, c, cut(v, N), cut(eao, N * (N - 1)),
                                        cut(ea, N * (N - 1)), cut(lm, N), N, L, Bc, cut(q.reshape(-1), N), T=T,
                                        t_out=t_c)
            done += 1
            if time.perf_counter() - t0 > 10.0 or done >= 5:
                break
        cel = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": Bc * done / cel, "unit": "trajectories/s", "cores": int(_host_cores()),
                               "kind": "port", "sample": f"oracle/harness.py egno_rollout (numpy fp32 + f64 energy), "
                               f"B={Bc} of the same batch, traj_len={L}, {done} calls in {cel:.1f} s"}
        got = out[0][:T].reshape(T, B, N, 3)[:, :Bc].reshape(-1, 3).double().cpu().numpy()
        want = ref[:T]
        res["parity"] = {"first_segment_pos_maxnorm_rel_vs_oracle": float(np.abs(got - want.reshape(-1, 3)).max()
                                                                           / np.abs(want).max()),
                         "samples_checked": Bc}
    return res


# ChargedParticlesSim (synthetic_sim.py:244-260) per ordered pair and step, float64, as the kernel
# evaluates it: x_i.x_j (5), |x_i|^2 + |x_j|^2 - 2 x_i.x_j (3), s q_i q_j / (l2 sqrt(l2)) (5),
# F += fs (x_i - x_j) (9)
FLOP_PER_PAIR_CHARGED = 22
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector, AMD spec (not in the microarch guide)


def run_sim_charged(args, world, rank, dev):
    """ChargedParticlesSim.sample_trajectory (synthetic_sim.py:220-296) as
    generate_dataset.py's documented charged N=20 run (its header, :10: --length 20000,
    --sample-freq 100; 3000 training simulations): S trajectories integrated in one launch from
    initial states already in HBM. A trajectory is one 20000-step simulation (199 saved frames)."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd import _lib
    from no_node_comparison_amd.sharding import max_over_ranks, shard_range
    S = args.batch if args.batch != 512 else 3000
    N, Tn, freq = 20, 20000, 100
    sim = pkg.sim.ChargedParticlesSim(n_balls=N, vel_norm=0.5)
    np.random.seed(43 + rank)
    draws = [sim._draw(Tn // freq - 1, [0.5, 0.0, 0.5]) for _ in range(S)]
    q = torch.tensor(np.stack([d[0] for d in draws]).reshape(S, N), dtype=torch.float64, device=dev)
    l0 = torch.tensor(np.stack([d[1] for d in draws]), dtype=torch.float64, device=dev)
    v0 = torch.tensor(np.stack([d[2] for d in draws]), dtype=torch.float64, device=dev)
    call = lambda: sim.integrate(q, l0, v0, Tn, freq)  # noqa: E731
    _prewarm(call, args, dev)
    for _ in range(args.warmup):
        out = call()
    barrier_sync(world, dev)
    if args.kernel_events:
        _lib.profile_begin(args.steps + 8)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = call()
    barrier_sync(world, dev)
    el = time.perf_counter() - t0
    records = _lib.profile_end() if args.kernel_events else []
    el = max_over_ranks(el, dev)
    value = S * world * args.steps / el
    res = {"metric": "simulated N-body trajectories/s (charged, N=20, 20000 leapfrog steps)", "value": value,
           "unit": "trajectories/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f64", "data": "synthetic initial states (the reference's draws, np seed 43 + rank)",
           "config": {"workload": f"f3: ChargedParticlesSim N={N}, length {Tn}, sample_freq {freq}, S={S} per GPU",
                      "sims_per_gpu": S, "n_balls": N, "length": Tn, "sample_freq": freq,
                      "parallelism": f"independent simulations x{world}"}}
    sims = [ms for kind, ms in records if kind == _lib.PROF_SIM_CHARGED]
    if sims:
        avg = float(np.mean(sims))
        flop = float(FLOP_PER_PAIR_CHARGED) * S * N * (N - 1) * Tn
        ach = flop / (avg * 1e-3) / 1e12
        res["roofline"] = {"kernel": "sim_charged_kernel", "bound": "valu_fp64", "achieved": ach,
                           "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ach / FP64_PEAK_TFLOPS,
                           "traffic": None, "avg_launch_ms": avg, "algorithmic_gflop_per_launch": flop / 1e9,
                           "launches_timed": len(sims)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import sim as osim
        done, t0 = 0, time.perf_counter()
        while True:
            qi, li, vi = draws[done]
            L_ref, _ = osim.charged_trajectory(li, vi, qi, Tn, freq)
            done += 1
            if time.perf_counter() - t0 > 10.0 or done >= min(S, 20):
                break
        cel = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": done / cel, "unit": "trajectories/s", "cores": 1, "kind": "port",
                               "sample": f"oracle/sim.py charged_trajectory (numpy f64, per simulation like the "
                               f"reference), {done} of the same simulations in {cel:.1f} s"}
        got = out[0][done - 1].cpu().numpy()
        k = 10    # the first 10 saved frames (1000 steps): chaotic divergence grows after that
        res["parity"] = {"first_frames_maxabs_vs_oracle": float(np.abs(got[:k] - L_ref[:k]).max()),
                         "frames_checked": k}
    return res


def pmc_traffic(kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=512, help="samples per GPU")
    ap.add_argument("--workload", default="egno",
                    choices=["egno", "segno", "segno_gravity", "egno_train", "egno_rollout", "sim_charged"],
                    help="egno = C2 (the headline line); segno = C3; segno_gravity = C5; egno_train = C4; "
                         "egno_rollout = SURVEY row f1; sim_charged = row f3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--prewarm-ms", type=float, default=300.0,
                    help="untimed clock-ramp calls (wall ms) before the W warmup steps")
    ap.add_argument("--no-kernel-events", dest="kernel_events", action="store_false")
    args = ap.parse_args()
    world, rank, dev = setup_dist()
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if args.workload == "egno":
        res = run_egno(args, world, rank, dev)
    elif args.workload == "egno_train":
        res = run_egno_train(args, world, rank, dev)
    elif args.workload == "egno_rollout":
        res = run_egno_rollout(args, world, rank, dev)
    elif args.workload == "sim_charged":
        res = run_sim_charged(args, world, rank, dev)
    else:
        res = run_segno(args, world, rank, dev, gravity=args.workload == "segno_gravity")
    if rank == 0:
        res["prewarm_ms"] = args.prewarm_ms
        print(json.dumps(res))
    if world > 1:
        _barrier(dev)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
