"""Aten ops issued per training step outside the HIP library (C4 / segno_train), to find the torch-side
fills, copies and small kernels around the kernels. GPU box:
    python3 tools/torch_ops_step.py [egno_train|segno_train]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "egno_train"
steps = 5
captured = {}


def fake_prewarm(step, args, dev):   # bench's _prewarm is the hook: grab the step closure
    captured["step"] = step
    raise StopIteration


bench._prewarm = fake_prewarm
args = bench.parse_args(["--workload", wl, "--no-cpu-baseline", "--steps", "1", "--warmup", "0"])
dev = torch.device("cuda:0")
fn = bench.run_egno_train if wl == "egno_train" else bench.run_segno_train
try:
    fn(args, 1, 0, dev, None)
except StopIteration:
    pass
step = captured["step"]
for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
rows = []
for ev in prof.key_averages():
    if ev.key.startswith("aten::") or "Optimizer" in ev.key or "autograd" in ev.key.lower():
        rows.append((ev.count / steps, ev.device_time_total / steps, ev.key))
rows.sort(key=lambda r: -r[1])
print(f"{wl}: aten ops per step (count, device us)")
for c, t, k in rows[:60]:
    print(f"{c:6.1f} {t:9.1f}  {k}")
