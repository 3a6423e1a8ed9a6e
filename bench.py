"""Benchmark of the EGNO / SEGNO trajectory-rollout hot path on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` — one process per GPU, W untimed
steps, then exactly K timed steps bracketed by a barrier + synchronize, max over ranks; rank 0 prints
ONE JSON line. For N > 1 the driver starts the ranks with torch.distributed.run; started without it
(WORLD_SIZE unset), ``--gpus N`` launches torch.distributed.run itself as a child process before
anything touches the GPU, and every rank checks that the world it joined has exactly N ranks.

A "step" is one pass of the hot path over one batch of synthetic input. Default workload
(BASELINE.json configs[1], "C2"): EGNO 4 layers, charged N=20, T=10, B=512 per GPU, fp32 — one
model call producing T=10 frames for all B trajectories. Ranks are independent replicas on their
own batch shard (the path shards by sample; inference has no collective), so scaling is weak.
``--global-batch G`` fixes the total batch instead (G / N per GPU, "scaling": "strong"), e.g. the
C4 training config: ``--workload egno_train --global-batch 4096``.

The CPU baseline is oracle/torch_ref.py — the reference's own torch operators, op by op, on the
host cores — and the HIP outputs are checked against it on the same batch.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "N-body trajectories/s (B×T, N=20 rollout) + pos-MSE vs ref, 1/2/4/8 MI355X"
DTYPE = "fp32 (fp16x3 split-MFMA, fp32 accumulate, f32 guard)"
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
# Edge backward (edge_bwd_kernel pass 0 + pass 1): the reverse of the two per-edge
# 64x64 Linears W2 and Wc1 — data gradient (64x64) and weight gradient (64x64) each — plus the
# vector terms (w_c2, the scalar input columns). The forward recompute is not counted.
MAC_PER_EDGE_BWD = 4 * 4096 + 4 * 64
# Algorithmic HBM bytes of the reference formulation's edge aggregation at C2: messages
# [e, 64 + 3] read + node sums [n, 64 + 3] written, fp32, per layer
AGG_BYTES = lambda e, n: (e + n) * 67 * 4  # noqa: E731


# ---------------------------------------------------------------------------------------------------
# launch / distributed setup
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def maybe_launch(args):
    """--gpus N > 1 outside torch.distributed.run: run N ranks as a child torch.distributed.run
    (one process per GPU) and exit with its status. Called before anything initialises the GPU."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.stdout.flush()
    sys.exit(subprocess.call(cmd, env=env))


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the process group has {world} ranks")
    gpu = torch.cuda.is_available()
    # NONODE_DIST_BACKEND=gloo rehearses the multi-rank bench on a box with fewer GPUs than ranks
    # (ranks then share GPUs round-robin); the default on a GPU node is RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("NONODE_DIST_BACKEND") or ("nccl" if gpu else "gloo")
    if gpu:
        ndev = torch.cuda.device_count()
        if backend == "nccl" and world > ndev:
            raise SystemExit(f"bench: {world} RCCL ranks but only {ndev} visible GPUs")
        local = local % ndev
        torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group(backend=backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench: joined a world of {dist.get_world_size()}, expected {args.gpus}")
    dev = torch.device(f"cuda:{local}" if gpu else "cpu")
    return world, rank, dev, (backend if world > 1 else None)


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


def batch_plan(args, world, rank, per_gpu_default):
    """Weak scaling (default): B per GPU fixed (--batch, else the workload's default). Strong
    scaling (--global-batch G): G samples in total, shard_range(G, world, rank) on this rank."""
    from no_node_comparison_amd.sharding import shard_range
    if args.global_batch:
        G = args.global_batch
        lo, hi = shard_range(G, world, rank)
        return dict(B_global=G, B=hi - lo, lo=lo, hi=hi, scaling="strong")
    B = args.batch or per_gpu_default
    return dict(B_global=B * world, B=B, lo=B * rank, hi=B * (rank + 1), scaling="weak")


def check_launch(args, world, rank, dev, backend):
    """--check-launch: report every rank's (rank, local rank, device) without running a workload
    (the CPU test of the launcher)."""
    me = torch.tensor([rank, int(os.environ.get("LOCAL_RANK", "0")), dev.index if dev.index is not None else -1])
    if world > 1:
        me = me.to(dev) if backend == "nccl" else me
        parts = [torch.zeros_like(me) for _ in range(world)]
        dist.all_gather(parts, me)
        ranks = [p.cpu().tolist() for p in parts]
    else:
        ranks = [me.tolist()]
    return {"check_launch": True, "world_size": world, "backend": backend, "ranks": ranks, "n_gpus": world}


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


def device_info(dev):
    """What the run ran on: CU count (the layer kernels size their grid by it), arch, clocks and
    partition modes (rocm-smi, best effort) — to tell box-to-box variance from code changes."""
    if dev.type != "cuda":
        return None
    p = torch.cuda.get_device_properties(dev)
    info = {"name": p.name, "arch": getattr(p, "gcnArchName", None), "cus": p.multi_processor_count,
            "hbm_gib": round(p.total_memory / 2 ** 30, 1)}
    if "rocprof" in os.environ.get("LD_PRELOAD", ""):
        # under rocprofv3 every child process carries its preload (which initialises the GPU) and
        # rocm-smi is a script that re-execs its interpreter: skip it there
        info["smi"] = "skipped under rocprofv3"
        return info
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--showcomputepartition", "--showmemorypartition",
                            "--showpower", "--json"], capture_output=True, text=True, timeout=20)
        d = json.loads(r.stdout)
        card = next(iter(v for k, v in d.items() if k.startswith("card")), {})
        keep = ("sclk", "mclk", "fclk", "partition", "power")
        info["smi"] = {k: v for k, v in card.items() if any(s in k.lower() for s in keep)}
    except Exception as e:   # noqa: BLE001 - informational only
        info["smi"] = f"unavailable ({type(e).__name__})"
    return info


# ---------------------------------------------------------------------------------------------------
# synthetic inputs
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


def synthetic_gravity(B, N, seed):
    """SURVEY §8d gravity generator: masses 1 + 0.1 N(0,1); positions, velocities ~ N(0,1) with the
    centre-of-mass velocity removed (synthetic_sim.py:370-378)."""
    g = torch.Generator().manual_seed(seed)
    mass = 1.0 + 0.1 * torch.randn(B, N, 1, generator=g)
    loc = torch.randn(B, N, 3, generator=g)
    vel = torch.randn(B, N, 3, generator=g)
    vel = vel - (mass * vel).sum(1, keepdim=True) / mass.sum(1, keepdim=True)
    return loc, vel, mass


def rank_batch(B_per, world, rank, N, seed):
    """This rank's shard of the global synthetic batch of B_per * world samples (weak scaling: the
    per-GPU batch is fixed). Concatenating every rank's shard gives the global batch."""
    from no_node_comparison_amd.sharding import shard_range
    loc, vel, q = synthetic_charged(B_per * world, N, seed)
    lo, hi = shard_range(B_per * world, world, rank)
    return loc[lo:hi], vel[lo:hi], q[lo:hi]


def build_egno_case(B, N, T, seed, dev, world=1, rank=0, plan=None):
    import no_node_comparison_amd as pkg
    if plan is None:
        loc, vel, q = rank_batch(B, world, rank, N, seed)
    else:
        loc, vel, q = synthetic_charged(plan["B_global"], N, seed)
        loc, vel, q = loc[plan["lo"]:plan["hi"]], vel[plan["lo"]:plan["hi"]], q[plan["lo"]:plan["hi"]]
    edges = pkg.harness.get_edges(B, N, dev)
    loc, vel, q = loc.to(dev), vel.to(dev), q.to(dev)
    qq = q.reshape(-1, 1)
    eao = qq[edges[0]] * qq[edges[1]]
    x, v, ea, nodes, lm = pkg.harness.prepare_inputs(loc, vel, eao, edges, N, 1, q)
    t_out = torch.arange(1, T + 1, device=dev).repeat(B, 1)
    return dict(x=x, h=nodes, edges=edges, edge_fea=ea, v=v, loc_mean=lm, t_out=t_out, eao=eao, q=q)


# ---------------------------------------------------------------------------------------------------
# CPU baseline: the reference's torch operators on the host cores (oracle/torch_ref.py)
def cpu_time(fn, budget_s, min_calls=10, max_calls=20):
    """Median wall time of fn() over as many calls as fit in budget_s (at least min_calls)."""
    times, out = [], None
    t_all = time.perf_counter()
    while len(times) < max_calls:
        t0 = time.perf_counter()
        out = fn()
        times.append(time.perf_counter() - t0)
        if len(times) >= min_calls and time.perf_counter() - t_all + times[-1] > budget_s:
            break
    return float(np.median(times)), len(times), out


def cpu_baseline_time(fn, budget_s, min_calls=10, max_calls=20):
    """cpu_time of the CPU baseline on baseline_threads() torch threads. The threads actually used are
    recorded by _baseline (called inside the same context)."""
    with _BaselineThreads():
        return cpu_time(fn, budget_s, min_calls, max_calls)


def _cpu(t, rows=None):
    t = t.detach()
    return (t[:rows] if rows is not None else t).cpu()


def _cpu_params(model):
    return {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}


def _cgroup_cpus():
    """CPUs granted by the cgroup CPU quota (cgroup v2 cpu.max / v1 cfs quota), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(per)))
    except Exception:   # noqa: BLE001 - informational
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, q // per)
    except Exception:   # noqa: BLE001
        return None


def host_cores():
    """What the CPU baseline may run on: the host's physical cores (psutil), the CPUs this process may
    run on (affinity), the cgroup CPU quota and the pool's per-GPU thread share (OMP_NUM_THREADS, set
    by the GPU pool; the box runs one GPU's share of a larger host)."""
    try:
        import psutil
        phys = psutil.cpu_count(logical=False)
    except Exception:   # noqa: BLE001 - informational
        phys = None
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:   # noqa: BLE001
        affinity = None
    omp = os.environ.get("OMP_NUM_THREADS")
    share = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    return {"threads": torch.get_num_threads(), "cpus_allowed": affinity, "host_physical_cores": phys,
            "host_logical_cpus": os.cpu_count(), "cgroup_cpus": _cgroup_cpus(), "pool_thread_share": share}


def baseline_threads():
    """Threads for the CPU baseline. BASELINE.md §3 asks for every physical host core; on the GPU pool
    one box is one GPU's share of a larger host, so the count is capped by what this process is granted:
    min(physical cores, affinity, cgroup quota, the pool's OMP_NUM_THREADS share)."""
    hc = host_cores()
    caps = [c for c in (hc["host_physical_cores"], hc["cpus_allowed"], hc["cgroup_cpus"], hc["pool_thread_share"])
            if c]
    return max(1, min(caps)) if caps else torch.get_num_threads()


class _BaselineThreads:
    """torch intra-op threads = baseline_threads() for the CPU baseline leg, restored afterwards."""

    def __enter__(self):
        self.prev = torch.get_num_threads()
        torch.set_num_threads(baseline_threads())
        return self

    def __exit__(self, *exc):
        torch.set_num_threads(self.prev)


def _baseline(units, med, calls, sample, unit="trajectories/s"):
    hc = host_cores()
    hc["threads"] = baseline_threads()   # what cpu_baseline_time ran on
    return {"value": units / med, "unit": unit, "cores": hc["threads"], "kind": "torch-ref",
            "cores_note": "cores = torch intra-op threads used = min(host physical cores, affinity, cgroup quota, "
                          "the pool's per-GPU OMP_NUM_THREADS share); BASELINE.md §3 asks for every physical core, "
                          "but the GPU box is one GPU's share of a larger host (host fields below)",
            "host": hc, "median_s_per_call": med, "calls": calls,
            "sample": sample + f"; oracle/torch_ref.py (the reference's torch ops, op by op) on "
                               f"{hc['threads']} host threads, median of {calls} calls"}


def _parity(got, ref, key="pos"):
    got = got.double().numpy()
    ref = ref.double().numpy()
    return {f"{key}_mse_vs_ref": float(np.mean((got - ref) ** 2)),
            f"{key}_maxnorm_rel_vs_ref": float(np.abs(got - ref).max() / np.abs(ref).max())}


# ---------------------------------------------------------------------------------------------------
# workloads
def _result(args, world, plan, ms, value, name, extra_cfg, backend, allreduce_bytes=0, **kw):
    res = {"metric": METRIC, "value": value, "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": plan["scaling"],
           "vs_baseline": None, "dtype": DTYPE, "data": "synthetic (SURVEY §8d generators, seeded)",
           "world_size": world, "backend": backend, "allreduce_bytes_per_step": allreduce_bytes,
           "config": dict({"workload": name, "batch_per_gpu": plan["B"], "global_batch": plan["B_global"]},
                          **extra_cfg)}
    res.update(kw)
    return res


def run_egno(args, world, rank, dev, backend):
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd import _lib
    from no_node_comparison_amd.sharding import max_over_ranks
    N, T = 20, 10
    plan = batch_plan(args, world, rank, 512)
    B = plan["B"]
    torch.manual_seed(0)
    model = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                     num_timesteps=T, time_emb_dim=32, device=dev).eval()
    case = build_egno_case(B, N, T, seed=1234, dev=dev, plan=plan)
    r0, c0 = case["edges"]

    def edges():
        """--edges: fixed = one edge list for every step (validated once); get_edges = a fresh list per
        step from harness.get_edges (nonode_full_edges, valid by construction); fresh = fresh device
        tensors the boundary has never seen (copies), checked on the device every step -- the
        reference loop's fresh get_edges(...).to(device) per batch (main_simulation_simple_no.py:217-218)"""
        if args.edges == "get_edges":
            return pkg.harness.get_edges(B, N, dev)
        if args.edges == "fresh":
            return [r0.clone(), c0.clone()]
        return case["edges"]

    call = lambda: model(case["x"], case["h"], edges(), case["edge_fea"], v=case["v"],  # noqa: E731
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
        # host overhead per forward: with an idle GPU before each call, the host time
        # to enqueue one forward and its synchronous wall time, against the recorded kernel time
        enq, wall = [], []
        for _ in range(10):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            out = call()
            t1 = time.perf_counter()
            torch.cuda.synchronize(dev)
            enq.append(t1 - t0)
            wall.append(time.perf_counter() - t0)
    el = max_over_ranks(el, dev)
    value = plan["B_global"] * args.steps / el
    cus = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 0
    res = _result(args, world, plan, el / args.steps * 1e3, value,
                  f"C2: EGNO forward (4 layers, hidden 64, 2 modes), charged N={N}, T={T}, B={B} per GPU",
                  {"n_balls": N, "num_timesteps": T, "layer_workgroups": min(T * B, cus), "edges": args.edges,
                   "parallelism": f"batch-sharded replicas x{world} (no collective)"}, backend,
                  frames_per_s=value * T)
    kern_ms = float(np.sum([ms for _, ms in records])) / args.steps if records else None
    res["host_overhead"] = {
        "enqueue_ms_median": float(np.median(enq)) * 1e3, "sync_wall_ms_median": float(np.median(wall)) * 1e3,
        "recorded_kernel_ms_per_call": kern_ms,
        "note": "per forward with an idle GPU before the call: enqueue = host time until the call returns; "
                "sync_wall = until its kernels finish; recorded kernels = the layer and TimeConv launches "
                "(hipEvents, temb_kernel not recorded). ms_per_step is the pipelined rate (host enqueues "
                "ahead of the GPU)"}
    layer_events = [ms for kind, ms in records if kind == _lib.VARIANT_EGNO]
    tconv_ms = [ms for kind, ms in records if kind in (_lib.PROF_TCONV, _lib.PROF_TCONV_FIRST)]
    if layer_events:
        avg_ms = float(np.mean(layer_events))
        E, n = T * B * N * (N - 1), T * B * N
        flop = 2.0 * (E * MAC_PER_EDGE + n * MAC_PER_NODE)
        achieved = flop / (avg_ms * 1e-3) / 1e12
        agg_gbs = AGG_BYTES(E, n) / (avg_ms * 1e-3) / 1e9
        res["roofline"] = {"kernel": "egnn_layer_kernel<EGNO>", "bound": "mfma", "achieved": achieved,
                           "peak": FP16X3_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP16X3_PEAK_TFLOPS,
                           "peak_basis": "dense fp16 MFMA peak / 3 (fp16x3 split products)",
                           "frac_of_fp32_mfma_peak": achieved / FP32_PEAK_TFLOPS,
                           "traffic": pmc_traffic("C2", "egnn_layer_kernel<EGNO>"), "avg_launch_ms": avg_ms,
                           "algorithmic_gflop_per_launch": flop / 1e9, "launches_timed": len(layer_events),
                           "tconv_avg_launch_ms": float(np.mean(tconv_ms)) if tconv_ms else None,
                           "north_star_hbm": {
                               "materialised_aggregation_bytes_per_layer": AGG_BYTES(E, n),
                               "equivalent_GBs": agg_gbs, "frac_of_hbm_peak": agg_gbs / HBM_PEAK_GBS,
                               "note": "the reference's aggregation bytes (messages materialised, SURVEY §8d) "
                                       "over the fused layer's time; this build never materialises messages, "
                                       "so HBM is not its bound and the kernel is priced against the MFMA "
                                       "ceiling (DESIGN.md §3.1)"}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import torch_ref as tr
        p = _cpu_params(model)
        # a bounded sample (>= 10 timed calls in the budget): the first Bc samples of the batch
        Bc = min(B, args.cpu_samples or 128)
        r, c = tr.full_edges(Bc, N)
        rows, erows = Bc * N, Bc * N * (N - 1)
        inp = [_cpu(case["x"], rows), _cpu(case["h"], rows), r, c, _cpu(case["edge_fea"], erows),
               _cpu(case["v"], rows), _cpu(case["loc_mean"], rows)]
        t_out = _cpu(case["t_out"], Bc)
        with torch.no_grad():
            med, calls, ref = cpu_baseline_time(lambda: tr.egno_forward(p, *inp, t_out, T=T), args.cpu_budget)
        res["cpu_baseline"] = _baseline(Bc, med, calls, f"EGNO forward on the first {Bc} samples of the measured "
                                        f"batch (B={B}), N={N}, T={T}")
        got = _cpu(out[0]).reshape(T, B, N, 3)[:, :Bc].reshape(-1, 3)
        res["parity"] = dict(_parity(got, ref[0]), samples_checked=Bc,
                             bar="1e-5 max-norm relative (north_star)")
    return res


def run_segno(args, world, rank, dev, backend, gravity=False):
    """C3 (SEGNO charged N=20, B=512 per GPU, one forward of 10 substeps) or C5 (SEGNO gravity
    N=100, B=256 per GPU, a 50-frame multi-horizon rollout: segments of c5_substeps() substeps)."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd import _lib
    from no_node_comparison_amd.sharding import max_over_ranks
    N = 100 if gravity else 20
    plan = batch_plan(args, world, rank, 256 if gravity else 512)
    B = plan["B"]
    torch.manual_seed(0)
    model = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=4, recurrent=True, device=dev).eval()
    gen = synthetic_gravity if gravity else synthetic_charged
    loc, vel, q = gen(plan["B_global"], N, 4321)
    loc, vel, q = (t[plan["lo"]:plan["hi"]].to(dev) for t in (loc, vel, q))
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

    with torch.no_grad():
        _prewarm(call, args, dev)
        for _ in range(args.warmup):
            call()
        barrier_sync(world, dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = call()
        barrier_sync(world, dev)
        el = time.perf_counter() - t0
        records = []
        if args.kernel_events:
            _lib.profile_begin(8 * args.steps * len(steps) + 64)
            for _ in range(args.steps):
                out = call()
            records = _lib.profile_end()
    el = max_over_ranks(el, dev)
    value = plan["B_global"] * args.steps / el
    name = "C5: SEGNO gravity N=100, 50-frame multi-horizon rollout (nonode_segno_rollout: per-segment " \
        "re-featurisation + gravity energy on the GPU)" if gravity else \
        "C3: SEGNO charged N=20, 10 integrator substeps (one fused launch)"
    cus = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 0
    res = _result(args, world, plan, el / args.steps * 1e3, value, f"{name}, B={B} per GPU",
                  {"n_balls": N, "substeps": steps, "layer_workgroups": min(B, cus),
                   "parallelism": f"batch-sharded replicas x{world}"}, backend)
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
                           "traffic": pmc_traffic("C5" if gravity else "C3", "egnn_layer_kernel<SEGNO>"), "avg_launch_ms": avg,
                           "algorithmic_gflop_per_launch": flop / 1e9, "launches_timed": len(layer),
                           "launch_ms_min_max": [float(np.min(layer)), float(np.max(layer))]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import torch_ref as tr
        p = _cpu_params(model)
        if gravity:
            # the dense one-hot mean (gcl.py:16-23) needs 259 GB per substep here: the scatter-mean
            # variant (same values) on the first Bc samples
            Bc = min(B, args.cpu_samples or 4)
            r, c = tr.full_edges(Bc, N)
            rows, erows = Bc * N, Bc * N * (N - 1)
            args_c = (_cpu(his, rows), _cpu(x, rows), r, c, _cpu(v, rows), _cpu(ea, erows), steps,
                      _cpu(q.reshape(-1), rows))
            with torch.no_grad():
                med, calls, ref = cpu_baseline_time(lambda: tr.segno_rollout(p, *args_c, dense_mean=False), args.cpu_budget)
            res["cpu_baseline"] = _baseline(Bc, med, calls, f"SEGNO gravity rollout, first {Bc} samples of the "
                                            f"batch, substeps {steps}, scatter mean (the reference's dense mean "
                                            f"is infeasible at this size)")
            got = _cpu(out).reshape(len(steps), B, N, 3)[:, :Bc].reshape(len(steps), -1, 3)
            res["parity"] = dict(_parity(got[:1], ref[:1]), samples_checked=Bc,
                                 all_segments=_parity(got, ref), bar="1e-5 max-norm relative, first segment")
        else:
            # the first Bc samples: the reference's dense one-hot mean costs O(B^2) per substep
            # (34 s per call at B=512), so the sample's rate is an upper bound of the reference's at B
            Bc = min(B, args.cpu_samples or 64)
            r, c = tr.full_edges(Bc, N)
            rows, erows = Bc * N, Bc * N * (N - 1)
            args_c = (_cpu(his, rows), _cpu(x, rows), r, c, _cpu(v, rows), _cpu(ea, erows))
            with torch.no_grad():
                med, calls, ref = cpu_baseline_time(lambda: tr.segno_forward_step(p, *args_c, T=steps[0], dense_mean=True),
                                           args.cpu_budget)
            res["cpu_baseline"] = _baseline(Bc, med, calls, f"SEGNO embedding + forward_step on the first {Bc} samples "
                                            f"of the measured batch (B={B}), {steps[0]} substeps, the reference's dense "
                                            f"one-hot mean (O(B^2): the rate at B={B} is lower)")
            res["parity"] = dict(_parity(_cpu(out, rows), ref[0]), samples_checked=Bc,
                                 bar="1e-5 max-norm relative (north_star)")
    return res


def make_adam(args, params, **kw):
    """The reference's optimizer, torch.optim.Adam with its hyper-parameters (model_confs.yaml:15-17,
    train_nbody.py), in torch's fused implementation by default (--optimizer fused: the same update,
    one kernel over every parameter instead of the multi-tensor 'foreach' chain of eight launches;
    --optimizer foreach is torch's default form)."""
    return torch.optim.Adam(params, fused=args.optimizer == "fused", foreach=args.optimizer == "foreach", **kw)


def run_egno_train(args, world, rank, dev, backend):
    """C4: EGNO training step, charged N=20, T=10, B=512 per GPU (or --global-batch 4096 over the
    ranks): forward with saved state, the reference loss (main_simulation_simple_no.py:273-280),
    backward through the HIP kernels, ONE all-reduce of the flat gradient buffer (RCCL over xGMI),
    Adam(lr 1e-4, wd 1e-8, model_confs.yaml:15-17). The loop is the reference's order:
    optimizer.zero_grad(); loss.backward(); [all-reduce]; optimizer.step()."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd.sharding import FlatGrads, max_over_ranks
    from no_node_comparison_amd import _lib
    N, T = 20, 10
    plan = batch_plan(args, world, rank, 512)
    B = plan["B"]
    torch.manual_seed(0)
    model = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                     num_timesteps=T, time_emb_dim=32, device=dev).train()
    p0 = _cpu_params(model)
    case = build_egno_case(B, N, T, seed=1234, dev=dev, plan=plan)
    g = torch.Generator().manual_seed(777)
    loc_true = torch.randn(plan["B_global"], N, T, 3, generator=g)[plan["lo"]:plan["hi"]].to(dev)
    fg = FlatGrads(model.parameters())
    opt = make_adam(args, model.parameters(), lr=1e-4, weight_decay=1e-8)

    def loss_of(x):
        pred = x.reshape(T, B, N, 3).permute(1, 2, 0, 3)
        # per-rank mean over its shard; with unequal strong-scaling shards the all-reduce averages
        # shard means, so weight by the shard size to keep the global-mean gradient
        w = B * world / plan["B_global"]
        return torch.nn.functional.mse_loss(pred, loc_true, reduction="none").mean((0, 1, 3)).mean() * w

    def step():
        opt.zero_grad()
        x, _, _ = model(case["x"], case["h"], case["edges"], case["edge_fea"], v=case["v"],
                        loc_mean=case["loc_mean"], timesteps_out=case["t_out"])
        loss = loss_of(x)
        loss.backward()
        fg.allreduce_()
        opt.step()
        return loss

    grads0 = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # gradients of the first step at the initial weights, for the parity check below
        opt.zero_grad()
        x, _, _ = model(case["x"], case["h"], case["edges"], case["edge_fea"], v=case["v"],
                        loc_mean=case["loc_mean"], timesteps_out=case["t_out"])
        loss_of(x).backward()
        fg.gather_()
        grads0 = {k: _cpu(q.grad) for k, q in model.named_parameters()}
    _prewarm(step, args, dev)
    for _ in range(args.warmup):
        step()
    barrier_sync(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    barrier_sync(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, dev)
    records = []
    if args.kernel_events:
        _lib.profile_begin(64 * args.steps + 64)
        for _ in range(args.steps):
            step()
        records = _lib.profile_end()
    value = plan["B_global"] * args.steps / el
    res = _result(args, world, plan, el / args.steps * 1e3, value,
                  f"C4: EGNO training step (fwd + bwd{' + 1 all-reduce' if world > 1 else ''} + Adam), charged N={N}, T={T}, B={B} per GPU",
                  {"n_balls": N, "num_timesteps": T, "grad_buffer_bytes": fg.numel * 4,
                   "optimizer": f"torch.optim.Adam ({args.optimizer})",
                   "parallelism": (f"data-parallel x{world}, one {backend} all-reduce per step" if backend else
                                   "single GPU, no all-reduce")},
                  backend, allreduce_bytes=fg.numel * 4 if world > 1 else 0, loss=float(loss.detach()))
    e0 = [ms for kind, ms in records if kind == _lib.PROF_EDGE_BWD0]
    e1 = [ms for kind, ms in records if kind == _lib.PROF_EDGE_BWD1]
    wl_key = "C4" if B == 512 else f"C4@B={B}"   # PMC traffic is per measured shard size
    if e0 or e1:
        _check_pass_records(e0, e1)
        avg = float(np.mean(e0) + np.mean(e1))
        E = T * B * N * (N - 1)
        flop = 2.0 * E * MAC_PER_EDGE_BWD
        ach = flop / (avg * 1e-3) / 1e12
        layer = [ms for kind, ms in records if kind == _lib.VARIANT_EGNO]
        res["roofline"] = {"kernel": "edge_bwd_kernel (pass 0 + pass 1, one layer)", "bound": "mfma", "achieved": ach,
                           "peak": FP16X3_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ach / FP16X3_PEAK_TFLOPS,
                           "peak_basis": "dense fp16 MFMA peak / 3 (fp16x3 split products)",
                           "traffic": _sum_or_none(pmc_traffic(wl_key, "edge_bwd_kernel<pass 0>"),
                                                   pmc_traffic(wl_key, "edge_bwd_kernel<pass 1>")),
                           "traffic_basis": f"HBM bytes of pass 0 + pass 1 measured at {wl_key} (profiles/pmc_traffic.json)",
                           "avg_launch_ms": avg, "pass_ms": [float(np.mean(e0)), float(np.mean(e1))],
                           "algorithmic_gflop_per_launch": flop / 1e9,
                           "algorithmic_basis": "reverse of W2 and Wc1 per edge (data + weight gradients); "
                                                "the forward recompute is not counted",
                           "launches_timed": len(e0) + len(e1),
                           "share_of_step": float(np.sum(e0) + np.sum(e1)) / (el * 1e3),
                           "forward_layer_avg_ms": float(np.mean(layer)) if layer else None}
    if grads0 is not None:
        from oracle import torch_ref as tr

        def sample(Bc):
            r, c = tr.full_edges(Bc, N)
            rows, erows = Bc * N, Bc * N * (N - 1)
            return ([_cpu(case["x"], rows), _cpu(case["h"], rows), r, c, _cpu(case["edge_fea"], erows),
                     _cpu(case["v"], rows), _cpu(case["loc_mean"], rows)], _cpu(loc_true, Bc), _cpu(case["t_out"], Bc))

        def cpu_step(p, opt, Bc, inp, tgt, t_out):
            if opt is not None:
                opt.zero_grad()
            xx, _, _ = tr.egno_forward(p, *inp, t_out, T=T)
            pred = xx.reshape(T, Bc, N, 3).permute(1, 2, 0, 3)
            loss = torch.nn.functional.mse_loss(pred, tgt, reduction="none").mean((0, 1, 3)).mean()
            loss.backward()
            if opt is not None:
                opt.step()

        # timed: a bounded sample (>= 10 calls in the budget; 11 s per call at B=512)
        Bc = min(B, args.cpu_samples or 64)
        p = {k: v.clone().requires_grad_(True) for k, v in p0.items()}
        copt = torch.optim.Adam(list(p.values()), lr=1e-4, weight_decay=1e-8)
        s_inp, s_tgt, s_t = sample(Bc)
        med, calls, _ = cpu_baseline_time(lambda: cpu_step(p, copt, Bc, s_inp, s_tgt, s_t), args.cpu_budget)
        res["cpu_baseline"] = _baseline(Bc, med, calls, f"EGNO training step (forward, loss, autograd backward, "
                                        f"Adam) on the first {Bc} samples of the measured batch (B={B})")
        # parity (untimed): the first step's gradients at the whole batch, fp32 and float64 autograd
        if not args.no_grad_parity:
            inp, tgt, t_out = sample(B)
            pf = {k: v.clone().requires_grad_(True) for k, v in p0.items()}
            with _BaselineThreads():
                cpu_step(pf, None, B, inp, tgt, t_out)
            first = {k: t.grad for k, t in pf.items() if t.grad is not None}
            Bc = B
            # parity of the first step's gradients at the initial weights: against the fp32 CPU path
            # as it runs (its own fp32 accumulation error included) and against the same ops in f64
            p64 = {k: v.double().requires_grad_(True) for k, v in p0.items()}
            xx, _, _ = tr.egno_forward(p64, *[t.double() if t.is_floating_point() else t for t in inp], t_out, T=T)
            pred = xx.reshape(T, Bc, N, 3).permute(1, 2, 0, 3)
            torch.nn.functional.mse_loss(pred, tgt.double(), reduction="none").mean((0, 1, 3)).mean().backward()
            par = {"samples_checked": B, "tensors_checked": 0,
                   "note": "first step's gradients at the initial weights, max-norm relative per tensor. The parity "
                           "figure is grad_maxnorm_rel_vs_f64 (HIP backward vs float64 torch autograd of the op-by-op "
                           "restatement). The *_vs_ref_fp32 figures compare HIP with the same autograd run in fp32 and "
                           "are dominated by the fp32 torch path's own rounding: ref_fp32_own_error_vs_f64_max is that "
                           "path's distance from float64 on the same tensors"}
            g64 = {k: t.grad for k, t in p64.items() if t.grad is not None}

            def rel(a, ref):
                return {k: float((a[k].double() - ref[k].double()).abs().max() / ref[k].abs().max())
                        for k in ref if float(ref[k].abs().max()) > 0}

            for tag, ref in (("f64", g64), ("ref_fp32", first)):
                errs = rel(grads0, ref)
                worst = max(errs, key=errs.get)
                par[f"grad_maxnorm_rel_vs_{tag}_max"] = errs[worst]
                par[f"grad_maxnorm_rel_vs_{tag}_median"] = float(np.median(list(errs.values())))
                par[f"worst_tensor_vs_{tag}"] = worst
                par["tensors_checked"] = len(errs)
            own = rel(first, g64)
            par["ref_fp32_own_error_vs_f64_max"] = max(own.values())
            par["ref_fp32_own_error_worst_tensor"] = max(own, key=own.get)
            res["parity"] = par
    return res


def run_segno_train(args, world, rank, dev, backend):
    """Row †g: SEGNO training step at the C3 configuration (charged N=20, B=512 per GPU, 10 substeps
    of forward_step): forward with saved state, nn.MSELoss of the positions after T substeps
    (train_nbody.py:150-178), backward through the HIP integrator's reverse pass, ONE all-reduce of
    the flat gradient buffer, Adam. Synthetic target: x + 0.3 v (tests/test_gpu_train_segno.py)."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd import _lib
    from no_node_comparison_amd.sharding import FlatGrads, max_over_ranks
    N, T = 20, 10
    plan = batch_plan(args, world, rank, 512)
    B = plan["B"]
    torch.manual_seed(0)
    model = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=4, recurrent=True, device=dev).train()
    p0 = _cpu_params(model)
    loc, vel, q = synthetic_charged(plan["B_global"], N, 4321)
    loc, vel, q = (t[plan["lo"]:plan["hi"]].to(dev) for t in (loc, vel, q))
    edges = pkg.harness.get_edges(B, N, dev)
    x = loc.reshape(-1, 3)
    v = vel.reshape(-1, 3)
    qq = q.reshape(-1, 1)
    ea = torch.cat([qq[edges[0]] * qq[edges[1]], ((x[edges[0]] - x[edges[1]]) ** 2).sum(-1, keepdim=True)], 1)
    his = v.norm(dim=-1, keepdim=True)
    target = x + 0.3 * v
    fg = FlatGrads(model.parameters())
    opt = make_adam(args, model.parameters(), lr=1e-4)
    w = B * world / plan["B_global"]   # shard-size weight: the all-reduce averages shard means

    def step():
        opt.zero_grad()
        xo = model(his, x, edges, v, ea, T=T)[0]
        loss = torch.nn.functional.mse_loss(xo, target) * w
        loss.backward()
        fg.allreduce_()
        opt.step()
        return loss

    grads0 = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        opt.zero_grad()
        (torch.nn.functional.mse_loss(model(his, x, edges, v, ea, T=T)[0], target) * w).backward()
        fg.gather_()
        grads0 = {k: _cpu(t.grad) for k, t in model.named_parameters() if t.grad is not None}
    _prewarm(step, args, dev)
    for _ in range(args.warmup):
        step()
    barrier_sync(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier_sync(world, dev)
    el = max_over_ranks(time.perf_counter() - t0, dev)
    records = []
    if args.kernel_events:
        _lib.profile_begin(64 * args.steps * T + 64)
        for _ in range(args.steps):
            step()
        records = _lib.profile_end()
    value = plan["B_global"] * args.steps / el
    res = _result(args, world, plan, el / args.steps * 1e3, value,
                  f"SEGNO training step (forward_step of {T} substeps + MSE + HIP reverse pass"
                  f"{' + 1 all-reduce' if world > 1 else ''} + Adam), charged N={N}, B={B} per GPU",
                  {"n_balls": N, "substeps": T, "grad_buffer_bytes": fg.numel * 4,
                   "optimizer": f"torch.optim.Adam ({args.optimizer})",
                   "parallelism": (f"data-parallel x{world}, one {backend} all-reduce per step" if backend else
                                   "single GPU, no all-reduce")},
                  backend, allreduce_bytes=fg.numel * 4 if world > 1 else 0)
    e0 = [ms for kind, ms in records if kind == _lib.PROF_EDGE_BWD0]
    e1 = [ms for kind, ms in records if kind == _lib.PROF_EDGE_BWD1]
    if e0 or e1:
        _check_pass_records(e0, e1)
        avg = float(np.mean(e0) + np.mean(e1))
        E = B * N * (N - 1)   # edges per substep
        flop = 2.0 * E * MAC_PER_EDGE_BWD
        ach = flop / (avg * 1e-3) / 1e12
        res["roofline"] = {"kernel": "edge_bwd_kernel (pass 0 + pass 1, one substep, SEGNO per-edge clamp)",
                           "bound": "mfma", "achieved": ach, "peak": FP16X3_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": ach / FP16X3_PEAK_TFLOPS,
                           "peak_basis": "dense fp16 MFMA peak / 3 (fp16x3 split products)",
                           "traffic": _sum_or_none(pmc_traffic("segno_train", "edge_bwd_kernel<pass 0>"),
                                                   pmc_traffic("segno_train", "edge_bwd_kernel<pass 1>")),
                           "traffic_basis": "HBM bytes of pass 0 + pass 1 per substep (profiles/pmc_traffic.json)",
                           "avg_launch_ms": avg, "pass_ms": [float(np.mean(e0)), float(np.mean(e1))],
                           "algorithmic_gflop_per_launch": flop / 1e9,
                           "algorithmic_basis": "reverse of W2 and Wc1 per edge (data + weight gradients); "
                                                "the forward recompute is not counted",
                           "launches_timed": len(e0) + len(e1),
                           "share_of_step": float(np.sum(e0) + np.sum(e1)) / (el * 1e3)}
    if grads0 is not None:
        from oracle import torch_ref as tr
        def sample(Bc):
            r, c = tr.full_edges(Bc, N)
            rows, erows = Bc * N, Bc * N * (N - 1)
            return (_cpu(his, rows), _cpu(x, rows), r, c, _cpu(v, rows), _cpu(ea, erows)), _cpu(target, rows)

        Bc = min(B, args.cpu_samples or 64)   # the autograd tape of the dense one-hot mean grows with B^2
        inp, tgt = sample(Bc)
        p = {k: t.clone().requires_grad_(True) for k, t in p0.items()}
        copt = torch.optim.Adam(list(p.values()), lr=1e-4)

        def cstep():
            copt.zero_grad()
            xr, _, _ = tr.segno_forward_step(p, *inp, T=T, dense_mean=True)
            torch.nn.functional.mse_loss(xr, tgt).backward()
            copt.step()

        med, calls, _ = cpu_baseline_time(cstep, args.cpu_budget)
        res["cpu_baseline"] = _baseline(Bc, med, calls, f"SEGNO training step (forward_step {T} substeps with the "
                                        f"reference's dense one-hot mean, MSE, autograd backward, Adam) on the first "
                                        f"{Bc} samples of the batch")
        # gradient parity over the whole measured batch: float64 autograd with the scatter mean
        inp, tgt = sample(B)
        p64 = {k: t.double().requires_grad_(True) for k, t in p0.items()}
        xr, _, _ = tr.segno_forward_step(p64, *[t.double() if t.is_floating_point() else t for t in inp], T=T,
                                         dense_mean=False)
        torch.nn.functional.mse_loss(xr, tgt.double()).backward()
        errs = {k: float((grads0[k].double() - t.grad).abs().max() / t.grad.abs().max())
                for k, t in p64.items() if t.grad is not None and float(t.grad.abs().max()) > 0 and k in grads0}
        worst = max(errs, key=errs.get)
        res["parity"] = {"samples_checked": B, "tensors_checked": len(errs),
                         "grad_maxnorm_rel_vs_f64_max": errs[worst], "worst_tensor_vs_f64": worst,
                         "grad_maxnorm_rel_vs_f64_median": float(np.median(list(errs.values()))),
                         "note": "first step's gradients at the initial weights, HIP reverse pass vs float64 "
                                 "torch autograd of the op-by-op restatement; max-norm relative per tensor"}
    return res


def run_egno_rollout(args, world, rank, dev, backend):
    """rollout_fn (main_simulation_simple_no.py:342-384) at the C2 shape, traj_len =
    10 segments (the script's --traj_len default, :79) with per-frame charged energies, as ONE
    native call (nonode_egno_rollout: 10 forwards + on-device re-featurisation + energy). A
    trajectory is one 100-frame rollout of one sample."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd import _lib
    from no_node_comparison_amd.sharding import max_over_ranks
    N, T, L = 20, 10, 10
    plan = batch_plan(args, world, rank, 512)
    B = plan["B"]
    torch.manual_seed(0)
    model = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                     num_timesteps=T, time_emb_dim=32, device=dev).eval()
    case = build_egno_case(B, N, T, seed=1234, dev=dev, plan=plan)
    edges, eao, q = case["edges"], case["eao"], case["q"]
    x, v, ea, nodes, lm = case["x"], case["v"], case["edge_fea"], case["h"], case["loc_mean"]
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
    value = plan["B_global"] * args.steps / el
    res = _result(args, world, plan, el / args.steps * 1e3, value,
                  f"f1: EGNO rollout_fn, charged N={N}, T={T}, traj_len={L} (100 frames + per-frame energy), "
                  f"B={B} per GPU", {"n_balls": N, "num_timesteps": T, "traj_len": L,
                                     "parallelism": f"batch-sharded replicas x{world} (no collective)"},
                  backend, frames_per_s=value * T * L)
    layer = [ms for kind, ms in records if kind == _lib.VARIANT_EGNO]
    if layer:
        avg = float(np.mean(layer))
        flop = 2.0 * (T * B * N * (N - 1) * MAC_PER_EDGE + T * B * N * MAC_PER_NODE)
        ach = flop / (avg * 1e-3) / 1e12
        res["roofline"] = {"kernel": "egnn_layer_kernel<EGNO>", "bound": "mfma", "achieved": ach,
                           "peak": FP16X3_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ach / FP16X3_PEAK_TFLOPS,
                           "peak_basis": "dense fp16 MFMA peak / 3 (fp16x3 split products)",
                           "frac_of_fp32_mfma_peak": ach / FP32_PEAK_TFLOPS,
                           "traffic": pmc_traffic("f1", "egnn_layer_kernel<EGNO>"), "avg_launch_ms": avg,
                           "algorithmic_gflop_per_launch": flop / 1e9, "launches_timed": len(layer),
                           "layer_kernel_share": float(np.sum(layer)) / (el / args.steps * 1e3)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import torch_ref as tr
        p = _cpu_params(model)
        Bc = min(B, args.cpu_samples or 16)
        r, c = tr.full_edges(Bc, N)
        rows, erows = Bc * N, Bc * N * (N - 1)
        args_c = (_cpu(nodes, rows), _cpu(x, rows), r, c, _cpu(v, rows), _cpu(eao, erows), _cpu(ea, erows),
                  _cpu(lm, rows), N, L, Bc, _cpu(q.reshape(-1), rows))
        with torch.no_grad():
            med, calls, ref = cpu_baseline_time(lambda: tr.egno_rollout(p, *args_c, T=T, t_out=_cpu(t_all, Bc)),
                                       args.cpu_budget)
        res["cpu_baseline"] = _baseline(Bc, med, calls, f"EGNO rollout_fn positions, first {Bc} samples of the "
                                        f"batch, traj_len={L} (energies not included)")
        got = _cpu(out[0][:T]).reshape(T, B, N, 3)[:, :Bc].reshape(T, Bc * N, 3)
        res["parity"] = dict(_parity(got, ref[:T]), samples_checked=Bc,
                             bar="1e-5 max-norm relative, first segment (later segments are chaotic)")
    return res


def c5_substeps(total=50, seed=0):
    """C5 multi-horizon substep list: draws in [5, 10) from default_rng(0) until they sum to 50
    (the last one clipped), SURVEY §8d."""
    rng = np.random.default_rng(seed)
    out = []
    while sum(out) < total:
        out.append(int(min(rng.integers(5, 10), total - sum(out))))
    return out


# ChargedParticlesSim (synthetic_sim.py:244-260) per ordered pair and step, float64, as the kernel
# evaluates it: x_i.x_j (5), |x_i|^2 + |x_j|^2 - 2 x_i.x_j (3), s q_i q_j / (l2 sqrt(l2)) (5),
# F += fs (x_i - x_j) (9)
FLOP_PER_PAIR_CHARGED = 22   # f64 operations per pair as listed (the divide and the sqrt count one each)


def run_sim_charged(args, world, rank, dev, backend):
    """ChargedParticlesSim.sample_trajectory (synthetic_sim.py:220-296) as
    generate_dataset.py's documented charged N=20 run (its header, :10: --length 20000,
    --sample-freq 100; 3000 training simulations): S trajectories integrated in one launch from
    initial states already in HBM. A trajectory is one 20000-step simulation (199 saved frames)."""
    import no_node_comparison_amd as pkg
    from no_node_comparison_amd import _lib
    from no_node_comparison_amd.sharding import max_over_ranks
    plan = batch_plan(args, world, rank, 3000)
    S = plan["B"]
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
    value = plan["B_global"] * args.steps / el
    res = _result(args, world, plan, el / args.steps * 1e3, value,
                  f"f3: ChargedParticlesSim N={N}, length {Tn}, sample_freq {freq}, S={S} per GPU",
                  {"n_balls": N, "length": Tn, "sample_freq": freq, "parallelism": f"independent simulations x{world}"},
                  backend)
    res.update(metric="simulated N-body trajectories/s (charged, N=20, 20000 leapfrog steps)", dtype="f64",
               data="synthetic initial states (the reference's draws, np seed 43 + rank)")
    sims = [ms for kind, ms in records if kind == _lib.PROF_SIM_CHARGED]
    if sims:
        avg = float(np.mean(sims))
        flop = float(FLOP_PER_PAIR_CHARGED) * S * N * (N - 1) * Tn
        ach = flop / (avg * 1e-3) / 1e12
        res["roofline"] = {"kernel": "sim_charged_kernel", "bound": "valu_fp64", "achieved": ach,
                           "peak": None, "unit": "TFLOP/s", "frac": None,
                           "note": "f64 operation rate (22 per pair, divide and sqrt counted as one each); no "
                                   "FP64 peak is given in MI355X_MICROARCH.md, so the kernel is not priced",
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
                               "host": host_cores(),
                               "sample": f"oracle/sim.py charged_trajectory (numpy f64, per simulation like the "
                               f"reference), {done} of the same simulations in {cel:.1f} s"}
        got = out[0][done - 1].cpu().numpy()
        k = 10    # the first 10 saved frames (1000 steps): chaotic divergence grows after that
        res["parity"] = {"first_frames_maxabs_vs_oracle": float(np.abs(got[:k] - L_ref[:k]).max()),
                         "frames_checked": k}
    return res


def _check_pass_records(e0, e1):
    """The edge backward is two launches (pass A, pass B) per layer / substep: both must have been
    recorded the same number of times, else the roofline would price a partial edge backward."""
    if not e0 or len(e0) != len(e1):
        raise RuntimeError(f"edge backward profile records: {len(e0)} pass-A vs {len(e1)} pass-B launches "
                           f"(profile buffer too small?)")


def _sum_or_none(*xs):
    return None if any(x is None for x in xs) else float(sum(xs))


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` measured on `workload` (C2, C3, C4, C4@4096, C5, segno_train, ...)
    from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json, tools/pmc_traffic.py), or None
    when that workload's kernel was not measured (never another workload's figure)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return d.get(workload, {}).get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:   # noqa: BLE001 - absent file: no traffic figure
        return None


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="samples per GPU (weak scaling; 0 = the workload's default)")
    ap.add_argument("--global-batch", type=int, default=0, help="total samples over all GPUs (strong scaling)")
    ap.add_argument("--workload", default="egno",
                    choices=["egno", "segno", "segno_gravity", "egno_train", "segno_train", "egno_rollout", "sim_charged"],
                    help="egno = C2 (the headline line); segno = C3; segno_gravity = C5; egno_train = C4; "
                         "egno_rollout = SURVEY row f1; sim_charged = row f3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-grad-parity", action="store_true", help="skip the C4 whole-batch gradient parity check")
    ap.add_argument("--edges", choices=["fixed", "get_edges", "fresh"], default="fixed",
                    help="C2: the edge tensors each step gets (run_egno.edges)")
    ap.add_argument("--optimizer", choices=["fused", "foreach"], default="fused",
                    help="torch Adam implementation of the training workloads (same update rule)")
    ap.add_argument("--cpu-budget", type=float, default=25.0, help="seconds of CPU baseline work (median of calls)")
    ap.add_argument("--cpu-samples", type=int, default=0, help="CPU baseline sample size where it is bounded")
    ap.add_argument("--prewarm-ms", type=float, default=300.0,
                    help="untimed clock-ramp calls (wall ms) before the W warmup steps")
    ap.add_argument("--no-kernel-events", dest="kernel_events", action="store_false")
    ap.add_argument("--check-launch", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.global_batch and args.global_batch < args.gpus:
        ap.error("--global-batch must be >= --gpus")
    return args


def main():
    args = parse_args()
    maybe_launch(args)            # before anything touches the GPU
    world, rank, dev, backend = setup_dist(args)
    if args.check_launch:
        res = check_launch(args, world, rank, dev, backend)
    else:
        runners = {"egno": run_egno, "egno_train": run_egno_train, "segno_train": run_segno_train,
                   "egno_rollout": run_egno_rollout,
                   "sim_charged": run_sim_charged, "segno": run_segno,
                   "segno_gravity": lambda *a: run_segno(*a, gravity=True)}
        res = runners[args.workload](args, world, rank, dev, backend)
        if rank == 0:
            res["prewarm_ms"] = args.prewarm_ms
            res["device"] = device_info(dev)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        _barrier(dev)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
