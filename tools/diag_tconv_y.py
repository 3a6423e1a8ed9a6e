"""Diagnostic: accuracy of TimeConv's pre-activation y (recovered as LeakyReLU^-1(h_out - h)) from
nonode_egno_tconv against float64, relative to max |y| (the scale the LeakyReLU kink test uses)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import no_node_comparison_amd as pkg  # noqa: E402
from oracle import torch_ref as tr  # noqa: E402

DEV = "cuda"
L = pkg._lib.lib()
for T, modes, BN in [(T, m, bn) for bn in (1024, 10240) for T in (8, 16) for m in (2, 3, 4, 5, 9)]:
    torch.manual_seed(0)
    m = pkg.EGNO(n_layers=1, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=modes,
                 num_timesteps=T, time_emb_dim=32, device=DEV).eval()
    _, tblobs = m._packed()
    g = torch.Generator().manual_seed(1)
    h = torch.randn(T * BN, 64, generator=g) * 2
    x = torch.randn(T * BN, 3, generator=g)
    v = torch.randn(T * BN, 3, generator=g)
    lm = torch.randn(BN, 3, generator=g)
    d = lambda a: a.to(DEV).contiguous()  # noqa: E731
    hd, xd, vd, lmd = map(d, (h, x, v, lm))
    ho, xo, vo = torch.empty_like(hd), torch.empty_like(xd), torch.empty_like(vd)
    txw = m.time_conv_x_modules[0].t_conv.weights1.detach().contiguous()
    P = pkg._lib.ptr
    pkg._lib.check(L.nonode_egno_tconv(BN, T, m.num_modes, P(hd), P(xd), P(vd), P(lmd), P(tblobs[0]), P(txw), P(ho),
                                       P(xo), P(vo), pkg._lib.stream_of(hd)))
    torch.cuda.synchronize()
    w = m.time_conv_modules[0].t_conv.weights1.detach().cpu().double()
    y = tr._spectral(h.double().reshape(T, BN, 64), w).reshape(T * BN, 64)
    dy = (ho.cpu().double() - h.double())
    yh = torch.where(dy >= 0, dy, dy / 0.01)
    err = (yh - y).abs()
    print(f"BN={BN} T={T} modes={modes}: max|y| {float(y.abs().max()):.3e}  max|y_hip - y| {float(err.max()):.3e}  "
          f"rel {float(err.max() / y.abs().max()):.3e}  (h-level rel {float((ho.cpu().double() - h.double() - torch.nn.functional.leaky_relu(y)).abs().max() / (h.double() + torch.nn.functional.leaky_relu(y)).abs().max()):.2e})", flush=True)
