"""CPU emulation of the layer kernel's fp16x3 arithmetic (tool, not product; imports the oracle).

Runs the EGNO forward (oracle/egno.py structure) with every 64-wide matrix product done the way
egnn_layer_kernel does it -- SiLU-domain scaling (-log2 e on SiLU inputs, -ln 2 on consumers),
fp16 hi/lo splits of weights and activations, fp32 accumulation -- so the error of a split scheme
against float64 can be studied on the CPU before a kernel change:

  python tools/fp16x3_emul.py [--B 16] [--scales 1,0.0625,4]

Modes:
  f32   plain fp32 products (the floor)
  cur   W_lo x_hi + W_hi x_lo + W_hi x_hi, W split unscaled (the round-2 kernel)
  wlo   W_lo stored x 2^k (k per matrix: max |W| 2^k in [2^EXP, 2^(EXP+1))), paired with
        x_hi'' = fp16(x_hi 2^-k): W_lo' x_hi'' + W_hi x_lo + W_hi x_hi
  full  W scaled x 2^k before the split, product x 2^-k
"""
import argparse
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import egno as oe  # noqa: E402

F32, F16 = np.float32, np.float16
NEG_LOG2E = F32(-1.4426950408889634)
NEG_LN2 = F32(-0.6931471805599453)


def split(x):
    x = x.astype(F32)
    hi = x.astype(F16)
    lo = (x - hi.astype(F32)).astype(F16)
    return hi, lo


def pow2_exp(W, target):
    m = float(np.abs(W).max())
    if m == 0.0:
        return 0
    return max(0, min(14, target - math.frexp(m)[1] + 1))


class Mat:
    """One packed 64-wide weight block W [out][in] as the kernel holds it."""

    def __init__(self, W, mode, target=3):
        self.W = W.astype(F32)
        self.mode = mode
        if mode in ("cur", "wlo", "full"):
            k = pow2_exp(self.W, target) if mode != "cur" else 0
            self.k = k
            if mode == "full":
                self.hi, self.lo = split(self.W * F32(2.0 ** k))
            else:
                self.hi, self.lo = split(self.W)
                if mode == "wlo":
                    self.lo = ((self.W - self.hi.astype(F32)) * F32(2.0 ** k)).astype(F16)

    def __call__(self, x):
        """x [rows][in] (f32) -> x W^T (f32)."""
        x = x.astype(F32)
        if self.mode == "f32":
            return (x @ self.W.T).astype(F32)
        xh, xl = split(x)
        Wh, Wl = self.hi.astype(np.float64), self.lo.astype(np.float64)
        xh64, xl64 = xh.astype(np.float64), xl.astype(np.float64)
        if self.mode == "wlo":
            xhs = (xh.astype(F32) * F32(2.0 ** -self.k)).astype(F16).astype(np.float64)
            acc = xhs @ Wl.T + xl64 @ Wh.T + xh64 @ Wh.T
        else:
            acc = xh64 @ Wl.T + xl64 @ Wh.T + xh64 @ Wh.T
        if self.mode == "full":
            acc = acc * 2.0 ** -self.k
        return acc.astype(F32)


def silu2(z):
    """the kernel's SiLU on -log2(e)-scaled inputs: z / (1 + 2^z) = -log2(e) SiLU(z / -log2 e)"""
    z = z.astype(F32)
    return (z / (F32(1) + np.exp2(z))).astype(F32)


def layer_emul(p, pre, x, h, row, col, ef, v, mode, target):
    g = lambda n: p[pre + n].astype(F32)  # noqa: E731
    W1 = g(".edge_message_net.scalar_net.mlp.0.weight")
    b1 = g(".edge_message_net.scalar_net.mlp.0.bias") * NEG_LOG2E
    WA = Mat(W1[:, 1:65] * NEG_LOG2E, mode, target)
    WB = Mat(W1[:, 65:129] * NEG_LOG2E, mode, target)
    Wf = W1[:, [0] + list(range(129, W1.shape[1]))] * NEG_LOG2E
    W2 = Mat(g(".edge_message_net.scalar_net.mlp.2.weight"), mode, target)
    b2 = g(".edge_message_net.scalar_net.mlp.2.bias") * NEG_LOG2E
    Wc1 = Mat(g(".coord_net.mlp.0.weight"), mode, target)
    bc1 = g(".coord_net.mlp.0.bias") * NEG_LOG2E
    wc2 = g(".coord_net.mlp.2.weight")[0] * NEG_LN2
    bc2 = g(".coord_net.mlp.2.bias")[0]
    Wv1 = Mat(g(".node_v_net.mlp.0.weight") * NEG_LOG2E, mode, target)
    bv1 = g(".node_v_net.mlp.0.bias") * NEG_LOG2E
    wv2 = g(".node_v_net.mlp.2.weight")[0] * NEG_LN2
    bv2 = g(".node_v_net.mlp.2.bias")[0]
    WN1 = g(".node_net.mlp.0.weight")
    WN1A = Mat(WN1[:, :64] * NEG_LOG2E, mode, target)
    WN1B = Mat(WN1[:, 64:], mode, target)
    bn1 = g(".node_net.mlp.0.bias") * NEG_LOG2E
    WN2 = Mat(g(".node_net.mlp.2.weight") * NEG_LN2, mode, target)
    bn2 = g(".node_net.mlp.2.bias")

    P = WA(h) + b1
    Q = WB(h)
    rij = (x[row] - x[col]).astype(F32)
    s = np.sum(rij * rij, axis=-1, keepdims=True).astype(F32)
    feat = np.concatenate([s, ef.astype(F32)], axis=-1)
    pre_ = (P[row] + Q[col] + (feat.astype(np.float64) @ Wf.T.astype(np.float64)).astype(F32)).astype(F32)
    a = silu2(pre_)
    m = silu2(W2(a) + b2)                                  # -log2e * m
    c = (silu2(Wc1(m) + bc1).astype(np.float64) @ wc2.astype(np.float64)).astype(F32) + bc2
    f = rij * c[:, None]
    n = x.shape[0]
    F = np.zeros((n, 3), F32)
    np.add.at(F, row, f)
    deg = np.bincount(row, minlength=n).astype(F32)
    phi = (silu2(Wv1(h) + bv1).astype(np.float64) @ wv2.astype(np.float64)).astype(F32) + bv2
    xn = (x + phi[:, None] * v + np.clip(F / deg[:, None], -100, 100)).astype(F32)
    M = np.zeros((n, 64), F32)
    np.add.at(M, row, m)
    z = WN1A(h) + WN1B(M) + bn1
    hn = WN2(silu2(z)) + bn2
    return xn, v, hn.astype(F32)


def forward_emul(p, x, h, row, col, ef, v, lm, t_out, mode, target, T=10):
    """oracle.egno.egno_forward with the layer replaced by layer_emul (TimeConv / embedding in f32)."""
    BN = h.shape[0]
    E = row.shape[0]
    temb = oe.timestep_embedding(t_out, 32, dtype=F32)
    Bt = temb.shape[0]
    temb = np.transpose(temb, (1, 0, 2))[:, None].repeat(BN // Bt, axis=1).reshape(T, BN, -1)
    hh = np.concatenate([np.broadcast_to(h[None], (T,) + h.shape), temb], axis=-1)
    hh = oe.linear(hh.reshape(T * BN, -1), p, "embedding").astype(F32)
    offs = (np.arange(T) * BN).repeat(E)
    row_t, col_t = np.tile(row, T) + offs, np.tile(col, T) + offs
    xx, vv, lmt, eft = np.tile(x, (T, 1)), np.tile(v, (T, 1)), np.tile(lm, (T, 1)), np.tile(ef, (T, 1))
    for i in range(4):
        hh = oe.time_conv(hh.reshape(T, BN, 64), p[f"time_conv_modules.{i}.t_conv.weights1"]).reshape(T * BN, 64)
        X = np.stack([xx - lmt, vv], axis=-1).reshape(T, BN, 3, 2)
        X = oe.time_conv_x(X, p[f"time_conv_x_modules.{i}.t_conv.weights1"])
        xx = (X[..., 0].reshape(T * BN, 3) + lmt).astype(F32)
        vv = X[..., 1].reshape(T * BN, 3).astype(F32)
        xx, vv, hh = layer_emul(p, f"layers.{i}", xx, hh.astype(F32), row_t, col_t, eft, vv, mode, target)
    return xx, vv, hh


def charged_inputs(B, N, seed):
    rng = np.random.default_rng(seed)
    sigma = (N / 5.0) ** (1 / 3)
    loc = rng.standard_normal((B, N, 3)) * sigma
    vel = rng.standard_normal((B, N, 3))
    vel = vel / np.linalg.norm(vel, axis=-1, keepdims=True) * 0.5
    q = rng.integers(0, 2, (B, N, 1)) * 2.0 - 1
    row = np.array([b * N + i for b in range(B) for i in range(N) for j in range(N) if j != i])
    col = np.array([b * N + j for b in range(B) for i in range(N) for j in range(N) if j != i])
    qf = q.reshape(-1)
    x = loc.reshape(-1, 3)
    ef = np.stack([qf[row] * qf[col], ((x[row] - x[col]) ** 2).sum(-1)], -1)
    v = vel.reshape(-1, 3)
    h = np.stack([np.linalg.norm(v, axis=-1), qf], -1)
    lm = np.repeat(loc.mean(1), N, axis=0)
    t_out = np.tile(np.arange(1, 11), (B, 1)).astype(np.float64)
    return [a.astype(F32) for a in (x, h)], row, col, [a.astype(F32) for a in (ef, v, lm)], t_out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--scales", default="1,0.0625,4")
    ap.add_argument("--modes", default="f32,cur,wlo,full")
    ap.add_argument("--target", type=int, default=3)
    args = ap.parse_args()
    d = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "egno_fwd.npz"))
    p0 = {k[3:]: d[k] for k in d.files if k.startswith("w::")}
    (x, h), row, col, (ef, v, lm), t_out = charged_inputs(args.B, 20, 7)
    for sc in (float(s) for s in args.scales.split(",")):
        p = {k: (w * sc if k.startswith("layers.") and w.ndim == 2 else w) for k, w in p0.items()}
        p64 = {k: w.astype(np.float64) for k, w in p.items()}
        ref = oe.egno_forward(p64, *(a.astype(np.float64) for a in (x, h)), row, col,
                              *(a.astype(np.float64) for a in (ef, v, lm)), t_out)
        line = [f"weights x{sc:g}:"]
        for mode in args.modes.split(","):
            out = forward_emul(p, x, h, row, col, ef, v, lm, t_out, mode, args.target)
            ex = np.abs(out[0] - ref[0]).max() / np.abs(ref[0]).max()
            eh = np.abs(out[2] - ref[2]).max() / np.abs(ref[2]).max()
            line.append(f"{mode} x {ex:.2e} h {eh:.2e}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
