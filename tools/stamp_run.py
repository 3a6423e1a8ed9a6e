"""Run the C2 forward with the stamp build and print per-section wave cycles (mean per launch).
Usage (GPU box): NONODE_LIB=no-node-comparison_amd/libnonode_stamp.so python3 tools/stamp_run.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import no_node_comparison_amd as pkg  # noqa: E402
from no_node_comparison_amd import _lib  # noqa: E402

NAMES = {0: "B head", 1: "B silu/split/mfma W2", 2: "B silu/split/mfma Wc1", 3: "B tail", 6: "A work",
         7: "A barrier", 8: "B segment prologue", 9: "B flush", 10: "B end (last seg)", 11: "B barrier",
         12: "C work", 13: "C barrier"}
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                 num_timesteps=10, time_emb_dim=32, device=dev).eval()
case = bench.build_egno_case(512, 20, 10, seed=1234, dev=dev)
L = _lib.lib()
buf = (ctypes.c_ulonglong * 16)()
with torch.no_grad():
    for it in range(3):
        model(case["x"], case["h"], case["edges"], case["edge_fea"], v=case["v"], loc_mean=case["loc_mean"],
              timesteps_out=case["t_out"])
        torch.cuda.synchronize()
        assert L.nonode_debug_stamps(buf) == 0
launches = 4
waves = 256 * int(os.environ.get("NONODE_WAVES", "8"))
tot = sum(buf)
for i in range(16):
    if buf[i]:
        print(f"{i:2d} {NAMES.get(i, '?'):28s} {buf[i] / launches / waves:10.0f} cyc/wave/launch  {buf[i] / tot:6.1%}")
print(f"   total {tot / launches / waves:.0f} cyc/wave/launch")
