"""Diagnostic: flat-training TimeConv weight gradients per layer against float64 autograd, for a loss on
x only and for x + v + h, plus nonode_egno_tconv_bwd in isolation on random inputs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch

import no_node_comparison_amd as pkg
from oracle import torch_ref as tr
from tests.conftest import maxnorm_rel
from tests.test_gpu_parity import _egno_case

DEV = "cuda"
B, N, T = 6, 20, 10


def model():
    torch.manual_seed(B + 3 * N)
    return pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2, num_timesteps=T,
                    time_emb_dim=32, num_inputs=1, device=DEV, flat=True).train()


case = _egno_case(B, N, T, seed=N + 5)
rng = np.random.default_rng(B)
target = rng.standard_normal((B, N, T, 3)).astype(np.float32)
wv, wh = rng.standard_normal((T * B * N, 3)).astype(np.float32), rng.standard_normal((T * B * N, 64)).astype(np.float32)


def loss_of(x, v, h, dt, dev, mode):
    l = ((x.reshape(T, B, N, 3).permute(1, 2, 0, 3) - torch.tensor(target).to(dev, dt)) ** 2).mean((0, 1, 3)).mean()
    if mode in ("v", "vh"):
        l = l + 1e-3 * (v * torch.tensor(wv).to(dev, dt)).sum()
    if mode in ("h", "vh"):
        l = l + 1e-4 * (h * torch.tensor(wh).to(dev, dt)).sum()
    return l


for mode in ("x", "v", "h", "vh"):
    m = model()
    m.zero_grad(set_to_none=True)
    inp = {k: torch.tensor(v).to(DEV) for k, v in case.items()}
    x, v, h = m(inp["x"], inp["h"], [inp["row"], inp["col"]], inp["edge_fea"], v=inp["v"], loc_mean=inp["loc_mean"],
                timesteps_out=inp["t_out"])
    loss_of(x, v, h, torch.float32, DEV, mode).backward()
    torch.cuda.synchronize()
    dt = torch.float64
    t = {k: torch.tensor(val).to(dt) if val.dtype.kind == "f" else torch.tensor(val) for k, val in case.items()}
    p = {k: q.detach().cpu().to(dt).requires_grad_(True) for k, q in m.state_dict().items()}
    xr, vr, hr = tr.egno_forward(p, t["x"], t["h"], t["row"], t["col"], t["edge_fea"], t["v"], t["loc_mean"],
                                 t["t_out"], T=T, flat=True)
    loss_of(xr, vr, hr, dt, "cpu", mode).backward()
    worst = sorted(((maxnorm_rel(q.grad.detach().cpu().numpy(), p[k].grad.numpy()), k)
                    for k, q in m.named_parameters() if p[k].grad is not None), reverse=True)[:6]
    print(mode, ["%s %.2e" % (k, e) for e, k in worst], flush=True)

# nonode_egno_tconv_bwd alone, on the actual TimeConv inputs of a flat training forward
L = pkg._lib.lib()
m = model()
BN = B * N
m._train_state_sink = []
inp = {k: torch.tensor(v).to(DEV) for k, v in case.items()}
m(inp["x"], inp["h"], [inp["row"], inp["col"]], inp["edge_fea"], v=inp["v"], loc_mean=inp["loc_mean"],
  timesteps_out=inp["t_out"])
sink = m._train_state_sink
g = torch.Generator().manual_seed(0)
x = torch.randn(T * BN, 3, generator=g)
v = torch.randn(T * BN, 3, generator=g)
lm = torch.randn(BN, 3, generator=g)
gh = torch.randn(T * BN, 64, generator=g)
gx = torch.randn(T * BN, 3, generator=g)
gv = torch.randn(T * BN, 3, generator=g)
for i in range(4):
    h = sink[i][0].detach().cpu()
    blobs, tblobs = m._packed()
    tw = m.time_conv_modules[i].t_conv.weights1.detach().contiguous()
    txw = m.time_conv_x_modules[i].t_conv.weights1.detach().contiguous()
    d = lambda a: a.to(DEV).contiguous()  # noqa: E731
    hd, xd, vd, lmd, ghd, gxd, gvd = map(d, (h, x, v, lm, gh, gx, gv))
    outs = [torch.empty_like(hd), torch.empty_like(xd), torch.empty_like(vd), torch.empty_like(tw), torch.empty_like(txw)]
    wsb = L.nonode_egno_tconv_bwd_workspace_bytes(BN, T, m.num_modes)
    ws = torch.empty((wsb + 3) // 4, device=DEV)
    P = pkg._lib.ptr
    pkg._lib.check(L.nonode_egno_tconv_bwd(BN, T, m.num_modes, P(hd), P(xd), P(vd), P(lmd), P(tblobs[i]), P(tw), P(txw),
                                           P(ghd), P(gxd), P(gvd), *[P(o) for o in outs], P(ws), wsb,
                                           pkg._lib.stream_of(hd)))
    torch.cuda.synchronize()
    dt = torch.float64
    fwd = (sink[i][1] - sink[i][0]).detach().cpu().reshape(T, BN, 64)
    for label in ("f64", "fwd"):
        H = h.to(dt).requires_grad_(True)
        W = tw.cpu().to(dt).requires_grad_(True)
        h3 = H.reshape(T, BN, 64)
        y = tr._spectral(h3, W)
        mk = (y > 0) if label == "f64" else torch.where(fwd != 0, fwd > 0, y > 0)
        out = (h3 + torch.where(mk, y, 0.01 * y)).reshape(T * BN, 64)
        (out * gh.to(dt)).sum().backward()
        yd = y.detach()
        print("layer", i, label, "g_tw %.2e" % maxnorm_rel(outs[3].cpu().numpy(), W.grad.numpy()),
              "g_h %.2e" % maxnorm_rel(outs[0].cpu().numpy(), H.grad.numpy()),
              "min|y|/max %.2e" % float(yd.abs().min() / yd.abs().max()),
              "flips %d" % int((mk != (yd > 0)).sum()), flush=True)
