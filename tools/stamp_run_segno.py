"""C3 (SEGNO forward_step, B=512, N=20, 10 substeps) with the stamp build: per-section wave cycles of
egnn_layer_kernel<SEGNO> (mean per wave per launch) and the phase shares.
Usage (GPU box): NONODE_LIB=no-node-comparison_amd/libnonode_stamp.so python3 tools/stamp_run_segno.py"""
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
B, N, T = 512, 20, 10
torch.manual_seed(0)
model = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=4, recurrent=True, device=dev).eval()
loc, vel, q = bench.synthetic_charged(B, N, 4321)
loc, vel, q = loc.to(dev), vel.to(dev), q.to(dev)
edges = pkg.harness.get_edges(B, N, dev)
x, v = loc.reshape(-1, 3), vel.reshape(-1, 3)
qq = q.reshape(-1, 1)
ea = torch.cat([qq[edges[0]] * qq[edges[1]], ((x[edges[0]] - x[edges[1]]) ** 2).sum(-1, keepdim=True)], 1)
his = v.norm(dim=-1, keepdim=True)
L = _lib.lib()
buf = (ctypes.c_ulonglong * 16)()
calls = 5
with torch.no_grad():
    model(his, x, edges, v, ea, T=T)
    torch.cuda.synchronize()
    assert L.nonode_debug_stamps(buf) == 0   # reset after the warm-up call
    for _ in range(calls):
        model(his, x, edges, v, ea, T=T)
    torch.cuda.synchronize()
    assert L.nonode_debug_stamps(buf) == 0
waves = min(B, torch.cuda.get_device_properties(dev).multi_processor_count) * 4   # one launch per call
tot = sum(buf)
for i in range(16):
    if buf[i]:
        print(f"{i:2d} {NAMES.get(i, '?'):28s} {buf[i] / calls / waves:10.0f} cyc/wave/launch  {buf[i] / tot:6.1%}")
print(f"   total {tot / calls / waves:.0f} cyc/wave/launch")
