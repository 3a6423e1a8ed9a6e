"""Per-section wave cycles of the EGNO edge backward (C4 shard: B=512, N=20, T=10) from the stamp
build (tools/stamp_build.sh). The training forward's stamps are read and discarded first.
Usage (GPU box): NONODE_LIB=$PWD/no-node-comparison_amd/libnonode_stamp.so python3 tools/stamp_train.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import no_node_comparison_amd as pkg  # noqa: E402
from no_node_comparison_amd import _lib  # noqa: E402

NAMES = {0: "B head (z1)", 1: "B silu + handoff loads", 5: "B dW2 wgrad", 6: "B W2^T",
         7: "B feat wgrad + GA/GB/GX", 8: "B phase A", 9: "B barrier A", 10: "B barrier B", 11: "B phase C",
         12: "B phase D", 13: "A head (z1)", 2: "A silu/W2/silu/Wc1/c", 15: "A gz3 + dWc1 wgrad", 3: "A Wc1^T",
         4: "A handoff stores", 14: "A phase A + barriers"}
PASS_B, PASS_A = (0, 1, 5, 6, 7, 8, 9, 10, 11, 12), (13, 2, 15, 3, 4, 14)
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                 num_timesteps=10, time_emb_dim=32, device=dev).train()
case = bench.build_egno_case(512, 20, 10, seed=1234, dev=dev)
L = _lib.lib()
buf = (ctypes.c_ulonglong * 16)()
acc = [0] * 16
reps = 3
for it in range(reps + 1):
    model.zero_grad(set_to_none=True)
    x, _, _ = model(case["x"], case["h"], case["edges"], case["edge_fea"], v=case["v"], loc_mean=case["loc_mean"],
                    timesteps_out=case["t_out"])
    loss = (x ** 2).mean()
    torch.cuda.synchronize()
    assert L.nonode_debug_stamps(buf) == 0       # forward stamps: discard
    loss.backward()
    torch.cuda.synchronize()
    assert L.nonode_debug_stamps(buf) == 0
    if it:
        acc = [a + b for a, b in zip(acc, buf)]
waves = 256 * 4 * 4 * reps    # blocks x waves x layers x reps
for idx, tag in ((PASS_B, "pass B (PASS 1)"), (PASS_A, "pass A (PASS 0)")):
    tot = sum(acc[i] for i in idx)
    print(f"{tag}: {tot / waves:.0f} cycles per wave per launch")
    for i in idx:
        if acc[i]:
            print(f"  {i:2d} {NAMES[i]:28s} {acc[i] / waves:10.0f}  {acc[i] / max(tot, 1):6.1%}")
