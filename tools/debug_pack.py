"""Debug tool (GPU): decode a packed layer blob's fp16x3 fragments and their lo shifts, and run one
layer on the golden per-layer captures. python tools/debug_pack.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import no_node_comparison_amd as pkg  # noqa: E402
from tests.conftest import load_golden, maxnorm_rel, params_of  # noqa: E402

OFF_H16, OFF_H16N = 33856, 33856 + 8192
OFF_SCAL = OFF_H16 - 64
LOG2E, LN2 = 1.4426950408889634, 0.6931471805599453


def decode(halves, k):
    """[8192] fp16 of one matrix -> W [64][64] = hi + lo 2^-k"""
    d = np.arange(8192)
    j, lane, hl, mo, s = d & 7, (d >> 3) & 63, (d >> 9) & 1, (d >> 10) & 3, d >> 12
    row = 16 * mo + (lane & 15)
    col = 16 * (2 * s + (j >> 2)) + 4 * (lane >> 4) + (j & 3)
    W = np.zeros((64, 64))
    v = halves.astype(np.float64) * np.where(hl == 1, 2.0 ** -k, 1.0)
    np.add.at(W, (row, col), v)
    return W


def main():
    fx = load_golden("egno_fwd")
    torch.manual_seed(0)
    m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2, num_timesteps=10,
                 time_emb_dim=32, device="cuda")
    m.load_state_dict({k: torch.tensor(v) for k, v in params_of(fx).items()})
    m.eval()
    blobs, _ = m._packed()
    torch.cuda.synchronize()
    b = blobs[0].detach().cpu().numpy()
    p = params_of(fx)
    pre = "layers.0."
    W1 = p[pre + "edge_message_net.scalar_net.mlp.0.weight"]
    mats = {
        "W2": (OFF_H16, 0, p[pre + "edge_message_net.scalar_net.mlp.2.weight"]),
        "Wc1": (OFF_H16 + 4096, 1, p[pre + "coord_net.mlp.0.weight"]),
        "WA": (OFF_H16N, 2, -LOG2E * W1[:, 1:65]),
        "WB": (OFF_H16N + 4096, 3, -LOG2E * W1[:, 65:129]),
        "WV1": (OFF_H16N + 8192, 4, -LOG2E * p[pre + "node_v_net.mlp.0.weight"]),
        "WN1A": (OFF_H16N + 3 * 4096, 5, -LOG2E * p[pre + "node_net.mlp.0.weight"][:, :64]),
        "WN1B": (OFF_H16N + 4 * 4096, 6, p[pre + "node_net.mlp.0.weight"][:, 64:]),
        "WN2": (OFF_H16N + 5 * 4096, 7, -LN2 * p[pre + "node_net.mlp.2.weight"]),
    }
    print("scal slots 0..16:", b[OFF_SCAL:OFF_SCAL + 16])
    for name, (off, idx, Wt) in mats.items():
        us = b[OFF_SCAL + 8 + idx:OFF_SCAL + 9 + idx].view(np.uint32)[0]
        hs = np.array([us & 0xFFFF, us >> 16], dtype=np.uint16).view(np.float16)
        k = int(round(-np.log2(float(hs[0])))) if hs[0] > 0 else None
        halves = b[off:off + 4096].view(np.float16)
        Wr = decode(halves, k if k is not None else 0)
        err = np.abs(Wr - Wt).max() / np.abs(Wt).max()
        print(f"{name:5s} us=0x{us:08x} halves={hs} k={k} max|W|={np.abs(Wt).max():.4f} rel err {err:.3e}")


if __name__ == "__main__":
    main()
