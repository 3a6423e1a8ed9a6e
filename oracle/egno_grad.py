"""Oracle restatement of one EGNO training step's gradients. Test-only.

The reference gets these from torch autograd: run_epoch (main_simulation_simple_no.py:267-280) runs
the forward EGNO.forward (egno.py:37-111), loss = mean over t of MSELoss(...).mean((0,1,3)) and
loss.backward(). This file writes the reverse pass by hand in numpy, op by op over the forward of
oracle/egno.py:
  - EGNN_Layer (basic.py:167-186);
  - TimeConv / TimeConv_x (layer_no.py:80-178);
  - the embedding Linear (egno.py:63-76).
It is pinned against the reference's own gradients (tests/golden/egno_grad.npz) in
tests/test_oracle_golden.py.

Conventions: silu'(z) = s (1 + z (1 - s)) with s = sigmoid(z). torch.clamp passes the gradient
where lo <= x <= hi. LeakyReLU passes grad where x > 0, else slope * grad.
"""
import numpy as np

from .egno import linear, silu, timestep_embedding


def sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


def dsilu(z):
    s = sigmoid(z)
    return s * (1.0 + z * (1.0 - s))


def _mlp_fwd(x, p, name, last_act=False):
    """BaseMLP with caches: returns (out, z0 pre-activation, a0 hidden, z1 pre-act of the output)."""
    z0 = linear(x, p, name + ".mlp.0")
    a0 = silu(z0)
    z1 = linear(a0, p, name + ".mlp.2")
    return (silu(z1) if last_act else z1), z0, a0, z1


def _mlp_bwd(g_out, x, cache, p, name, grads, last_act=False):
    """Reverse of _mlp_fwd: accumulates .weight/.bias grads, returns d/dx."""
    z0, a0, z1 = cache
    g1 = g_out * dsilu(z1) if last_act else g_out
    _acc(grads, name + ".mlp.2.weight", g1.T @ a0)
    _acc(grads, name + ".mlp.2.bias", g1.sum(0))
    g0 = (g1 @ p[name + ".mlp.2.weight"]) * dsilu(z0)
    _acc(grads, name + ".mlp.0.weight", g0.T @ x)
    _acc(grads, name + ".mlp.0.bias", g0.sum(0))
    return g0 @ p[name + ".mlp.0.weight"]


def _acc(grads, k, v):
    grads[k] = grads[k] + v if k in grads else v.copy()


# ---- EGNN_Layer (basic.py:167-186) ------------------------------------------------------------
def egnn_layer_fwd(p, prefix, x, h, row, col, edge_fea, v):
    n = x.shape[0]
    rij = x[row] - x[col]
    s = np.sum(rij * rij, axis=-1, keepdims=True)
    inp = np.concatenate([s, h[row], h[col], edge_fea], axis=-1)
    m, ez0, ea0, ez1 = _mlp_fwd(inp, p, prefix + ".edge_message_net.scalar_net", last_act=True)
    c, cz0, ca0, cz1 = _mlp_fwd(m, p, prefix + ".coord_net")
    f = rij * c
    cnt = np.maximum(np.bincount(row, minlength=n), 1).astype(x.dtype)[:, None]
    F = np.zeros((n, 3), x.dtype)
    np.add.at(F, row, f)
    Fm = F / cnt
    tot_f = np.clip(Fm, -100, 100)
    phi, vz0, va0, vz1 = _mlp_fwd(h, p, prefix + ".node_v_net")
    x_new = x + phi * v + tot_f
    M = np.zeros((n, m.shape[1]), x.dtype)
    np.add.at(M, row, m)
    hm = np.concatenate([h, M], axis=-1)
    h_new, nz0, na0, nz1 = _mlp_fwd(hm, p, prefix + ".node_net")
    cache = dict(x=x, h=h, v=v, rij=rij, s=s, inp=inp, e=(ez0, ea0, ez1), m=m, c_=(cz0, ca0, cz1), c=c,
                 Fm=Fm, cnt=cnt, phi=phi, vcache=(vz0, va0, vz1), M=M, hm=hm, ncache=(nz0, na0, nz1),
                 row=row, col=col, edge_fea=edge_fea)
    return x_new, v, h_new, cache


def egnn_layer_bwd(p, prefix, cache, gx_new, gv_new, gh_new, grads):
    """Returns (gx, gh, gv) w.r.t. the layer inputs; accumulates parameter grads into `grads`.
    Also returns the intermediate per-node / per-edge gradients (for kernel-level tests)."""
    row, col = cache["row"], cache["col"]
    n = cache["x"].shape[0]
    hid = cache["h"].shape[1]
    # x_new = x + phi * v + clamp(F / cnt)
    gx = gx_new.copy()
    gphi = np.sum(gx_new * cache["v"], axis=-1, keepdims=True)
    gv = gv_new + gx_new * cache["phi"]
    mask = (cache["Fm"] >= -100) & (cache["Fm"] <= 100)
    gF = gx_new * mask / cache["cnt"]                                  # d/d(sum_j f_ij)
    gh = _mlp_bwd(gphi, cache["h"], cache["vcache"], p, prefix + ".node_v_net", grads)
    # h_new = node_net([h, M])
    ghm = _mlp_bwd(gh_new, cache["hm"], cache["ncache"], p, prefix + ".node_net", grads)
    gh = gh + ghm[:, :hid]
    gM = ghm[:, hid:]
    # edges: f = rij * c ; M = sum_j m
    gf = gF[row]
    gc = np.sum(gf * cache["rij"], axis=-1, keepdims=True)
    grij = gf * cache["c"]
    gm = _mlp_bwd(gc, cache["m"], cache["c_"], p, prefix + ".coord_net", grads)
    gm = gm + gM[row]
    ginp = _mlp_bwd(gm, cache["inp"], cache["e"], p, prefix + ".edge_message_net.scalar_net", grads,
                    last_act=True)
    gs = ginp[:, :1]
    np.add.at(gh, row, ginp[:, 1:1 + hid])
    np.add.at(gh, col, ginp[:, 1 + hid:1 + 2 * hid])
    grij = grij + 2.0 * gs * cache["rij"]
    np.add.at(gx, row, grij)
    np.add.at(gx, col, -grij)
    inter = dict(gF=gF, gM=gM, gphi=gphi)
    return gx, gh, gv, inter


# ---- TimeConv / TimeConv_x (layer_no.py:80-178) ------------------------------------------------
def _dft(T, M):
    t = np.arange(T)
    m = np.arange(M)
    th = 2.0 * np.pi * np.outer(m, t) / T                                # [M, T]
    cm = np.where((m == 0) | (2 * m == T), 1.0, 2.0)[:, None] / T
    return np.cos(th), np.sin(th), cm


def spectral_fwd(x, w):
    """y = irfft(pad(W * rfft(x)[:M]), n=T) in closed form: x [T, ..., Cin] -> y [T, ..., Cout]
    (layer_no.py:96-109). Returns (y, (Xr, Xi))."""
    T, M = x.shape[0], w.shape[2]
    cos, sin, cm = _dft(T, M)
    Xr = np.tensordot(cos, x, axes=(1, 0))                               # [M, ..., Cin]
    Xi = -np.tensordot(sin, x, axes=(1, 0))
    Wr, Wi = w[..., 0], w[..., 1]                                        # [Cin, Cout, M]
    Yr = np.einsum("m...i,iom->m...o", Xr, Wr) - np.einsum("m...i,iom->m...o", Xi, Wi)
    Yi = np.einsum("m...i,iom->m...o", Xr, Wi) + np.einsum("m...i,iom->m...o", Xi, Wr)
    y = np.tensordot((cm * cos).T, Yr, axes=(1, 0)) - np.tensordot((cm * sin).T, Yi, axes=(1, 0))
    return y.astype(x.dtype), (Xr, Xi)


def spectral_bwd(gy, x, X, w):
    """Reverse of spectral_fwd: returns (gx, gw) with gw shaped like w [Cin, Cout, M, 2]."""
    T, M = x.shape[0], w.shape[2]
    cos, sin, cm = _dft(T, M)
    Xr, Xi = X
    gYr = np.tensordot(cm * cos, gy, axes=(1, 0))                        # [M, ..., Cout]
    gYi = -np.tensordot(cm * sin, gy, axes=(1, 0))
    Wr, Wi = w[..., 0], w[..., 1]
    fl = lambda a: a.reshape(a.shape[0], -1, a.shape[-1])  # noqa: E731  [M, rows, C]
    gWr = np.einsum("mri,mro->iom", fl(Xr), fl(gYr)) + np.einsum("mri,mro->iom", fl(Xi), fl(gYi))
    gWi = -np.einsum("mri,mro->iom", fl(Xi), fl(gYr)) + np.einsum("mri,mro->iom", fl(Xr), fl(gYi))
    gXr = np.einsum("m...o,iom->m...i", gYr, Wr) + np.einsum("m...o,iom->m...i", gYi, Wi)
    gXi = -np.einsum("m...o,iom->m...i", gYr, Wi) + np.einsum("m...o,iom->m...i", gYi, Wr)
    gx = np.tensordot(cos.T, gXr, axes=(1, 0)) - np.tensordot(sin.T, gXi, axes=(1, 0))
    return gx, np.stack([gWr, gWi], axis=-1)


def time_conv_bwd(gout, h, w, slope=0.01):
    """TimeConv: out = h + LeakyReLU(spectral(h)) (layer_no.py:121-126)."""
    y, X = spectral_fwd(h, w)
    gy = gout * np.where(y > 0, 1.0, slope)
    gx, gw = spectral_bwd(gy, h, X, w)
    return gout + gx, gw


def time_conv_x_bwd(gout, X0, w):
    """TimeConv_x: out = X + spectral_x(X), no activation (layer_no.py:173-178)."""
    _, X = spectral_fwd(X0, w)
    gx, gw = spectral_bwd(gout, X0, X, w)
    return gout + gx, gw


# ---- EGNO.forward + loss + backward -------------------------------------------------------------
def egno_loss_and_grads(p, x, h, row, col, edge_fea, v, loc_mean, t_out, loc_true, n_layers=4, T=10,
                        hidden=64, time_emb_dim=32, keep=None):
    """One training step of run_epoch (main_simulation_simple_no.py:267-280) without the
    optimizer: returns (loss, losses[T], grads dict keyed like the state_dict).

    loc_true: [B, N, T, 3]; the prediction x [T*BN, 3] is compared as [B, N, T, 3]."""
    from .egno import spectral_conv, leaky_relu
    dt = x.dtype
    BN = h.shape[0]
    E = row.shape[0]
    temb = timestep_embedding(t_out, time_emb_dim, dtype=dt)
    Bt = temb.shape[0]
    temb = np.transpose(temb, (1, 0, 2))[:, None].repeat(BN // Bt, axis=1).reshape(T, BN, -1)
    emb_in = np.concatenate([np.broadcast_to(h[None], (T,) + h.shape), temb], axis=-1).reshape(T * BN, -1)
    hh = linear(emb_in, p, "embedding")
    offs_e = (np.arange(T) * BN).repeat(E)
    row_t = np.tile(row, T) + offs_e
    col_t = np.tile(col, T) + offs_e
    xx = np.tile(x, (T, 1))
    vv = np.tile(v, (T, 1))
    lm = np.tile(loc_mean, (T, 1))
    ef = np.tile(edge_fea, (T, 1))
    tape = []
    for i in range(n_layers):
        wt = p[f"time_conv_modules.{i}.t_conv.weights1"]
        wx = p[f"time_conv_x_modules.{i}.t_conv.weights1"]
        h_in = hh.reshape(T, BN, hidden)
        hh = (h_in + leaky_relu(spectral_conv(h_in, wt))).reshape(T * BN, hidden)
        X0 = np.stack([xx - lm, vv], axis=-1).reshape(T, BN, 3, 2)
        X1 = X0 + spectral_conv(X0, wx)
        xx = X1[..., 0].reshape(T * BN, 3) + lm
        vv = X1[..., 1].reshape(T * BN, 3)
        xx, vv, hh, cache = egnn_layer_fwd(p, f"layers.{i}", xx, hh, row_t, col_t, ef, vv)
        tape.append((h_in, X0, cache))
    B, N = loc_true.shape[0], loc_true.shape[1]
    pred = xx.reshape(T, B, N, 3).transpose(1, 2, 0, 3)                  # [B, N, T, 3]
    diff = pred - loc_true
    losses = np.mean(diff ** 2, axis=(0, 1, 3))
    loss = losses.mean()
    gpred = 2.0 * diff / diff.size                                         # d mean / d pred
    gx = gpred.transpose(2, 0, 1, 3).reshape(T * BN, 3)
    gv = np.zeros_like(vv)
    gh = np.zeros_like(hh)
    grads = {}
    inter = []
    for i in reversed(range(n_layers)):
        h_in, X0, cache = tape[i]
        gx, gh, gv, it = egnn_layer_bwd(p, f"layers.{i}", cache, gx, gv, gh, grads)
        inter.append(it)
        # TimeConv_x: X1 = [x - lm, v] (+ spectral); x_out = X1[...,0] + lm
        gX1 = np.stack([gx, gv], axis=-1).reshape(T, BN, 3, 2)
        gX0, gwx = time_conv_x_bwd(gX1, X0, p[f"time_conv_x_modules.{i}.t_conv.weights1"])
        _acc(grads, f"time_conv_x_modules.{i}.t_conv.weights1", gwx)
        gx = gX0[..., 0].reshape(T * BN, 3)
        gv = gX0[..., 1].reshape(T * BN, 3)
        gh3, gwt = time_conv_bwd(gh.reshape(T, BN, hidden), h_in, p[f"time_conv_modules.{i}.t_conv.weights1"])
        _acc(grads, f"time_conv_modules.{i}.t_conv.weights1", gwt)
        gh = gh3.reshape(T * BN, hidden)
    _acc(grads, "embedding.weight", gh.T @ emb_in)
    _acc(grads, "embedding.bias", gh.sum(0))
    if keep is not None:
        keep["inter"] = inter[::-1]
    return loss, losses, grads
