"""Host-side cost of one drop-in EGNO forward (C2 shapes): cProfile over 300 calls, each behind a
synchronize (so the GPU queue is empty and the host path is what is timed).
Usage (GPU box): python3 tools/host_profile.py [batch] > gpurun_out/host_profile.txt"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import no_node_comparison_amd as pkg  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2, num_timesteps=10,
             time_emb_dim=32, device=dev).eval()
case = bench.build_egno_case(B, 20, 10, seed=1, dev=dev)
call = lambda: m(case["x"], case["h"], case["edges"], case["edge_fea"], v=case["v"],  # noqa: E731
                 loc_mean=case["loc_mean"], timesteps_out=case["t_out"])
with torch.no_grad():
    for _ in range(20):
        call()
    torch.cuda.synchronize()
    enq = []
    for _ in range(300):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        call()
        enq.append(time.perf_counter() - t0)
    enq.sort()
    print(f"B={B} enqueue per forward: median {enq[150] * 1e6:.1f} us, p10 {enq[30] * 1e6:.1f} us")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        torch.cuda.synchronize()
        call()
    pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
