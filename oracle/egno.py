"""Oracle restatement of EGNO (reference EGNO/model/{egno,layer_no,basic}.py). Test-only.

Parameters are a dict keyed exactly like the reference state_dict
(e.g. ``layers.0.edge_message_net.scalar_net.mlp.0.weight``).
"""
import math

import numpy as np


def silu(x):
    """nn.SiLU: x * sigmoid(x)."""
    return x / (1.0 + np.exp(-x))


def leaky_relu(x, slope=0.01):
    """nn.LeakyReLU() default slope (layer_no.py:119)."""
    return np.where(x >= 0, x, x * slope)


def linear(x, p, name):
    """nn.Linear: x @ W^T + b."""
    return x @ p[name + ".weight"].T + p[name + ".bias"]


def base_mlp(x, p, name, last_act=False, flat=False):
    """BaseMLP (basic.py:34-58): Linear, act, Linear[, act]; flat=True (basic.py:38-40): Tanh, and the
    hidden width 4x (carried by the weights' shapes)."""
    act = np.tanh if flat else silu
    y = linear(act(linear(x, p, name + ".mlp.0")), p, name + ".mlp.2")
    return act(y) if last_act else y


def timestep_embedding(timesteps, embedding_dim=32, max_positions=10000, dtype=np.float32):
    """get_timestep_embedding (layer_no.py:8-17): [B, T] -> [B, T, dim]."""
    half = embedding_dim // 2
    scale = math.log(max_positions) / (half - 1)
    freqs = np.exp(np.arange(half, dtype=np.float32) * np.float32(-scale)).astype(dtype)
    e = timesteps.astype(dtype)[:, :, None] * freqs[None, None, :]
    out = np.concatenate([np.sin(e), np.cos(e)], axis=-1)
    if embedding_dim % 2 == 1:
        out = np.pad(out, ((0, 0), (0, 0), (0, 1)))
    return out.astype(dtype)


def spectral_conv(x, w):
    """SpectralConv1d / SpectralConv1d_x (layer_no.py:96-109, 152-162).

    x: [T, ..., Cin]; w: [Cin, Cout, M, 2] (real, imag). rfft along axis 0, keep the first
    M modes, complex channel mix (einsum 'mni,iom->mno', layer_no.py:74-77), irfft(n=T).
    """
    T = x.shape[0]
    M = w.shape[2]
    xf = np.fft.rfft(x, axis=0)[:M]                       # [M, ..., Cin]
    wc = (w[..., 0] + 1j * w[..., 1]).astype(xf.dtype)    # [Cin, Cout, M]
    yf = np.einsum("m...i,iom->m...o", xf, wc)
    return np.fft.irfft(yf, n=T, axis=0).astype(x.dtype)


def time_conv(h, w):
    """TimeConv.forward (layer_no.py:121-126): x + LeakyReLU(spectral(x))."""
    return h + leaky_relu(spectral_conv(h, w))


def time_conv_x(X, w):
    """TimeConv_x.forward (layer_no.py:173-178): x + spectral_x(x), no activation."""
    return X + spectral_conv(X, w)


def aggregate(message, row, n_node, aggr):
    """aggregate (basic.py:6-31): scatter_add_ then sum or mean (count clamped to 1)."""
    out = np.zeros((n_node, message.shape[1]), dtype=message.dtype)
    np.add.at(out, row, message)
    if aggr == "mean":
        cnt = np.bincount(row, minlength=n_node).astype(message.dtype)
        out = out / np.maximum(cnt, 1)[:, None]
    return out


def radial_normalize(s):
    """F.normalize(s, p=2, dim=-1) of the one-element Gram row (basic.py:140-141): s / max(|s|, 1e-12)."""
    return s / np.maximum(np.abs(s), np.asarray(1e-12, dtype=s.dtype))


def egnn_layer(p, prefix, x, h, row, col, edge_fea, v, norm=False, flat=False):
    """EGNN_Layer.forward (basic.py:167-186), with_v=True; norm normalises the radial input
    (basic.py:140-141); flat: every BaseMLP 4x wide with Tanh (basic.py:38-40).

    Edge-MLP input order is [|r|^2, h_i, h_j, e] (InvariantScalarNet basic.py:136-143
    + hij = cat(h[row], h[col], edge_fea) at basic.py:170).
    """
    rij = x[row] - x[col]
    s = np.sum(rij * rij, axis=-1, keepdims=True)          # Gram of one vector: [E, 1]
    if norm:
        s = radial_normalize(s)
    inp = np.concatenate([s, h[row], h[col], edge_fea], axis=-1)
    m = base_mlp(inp, p, prefix + ".edge_message_net.scalar_net", last_act=True, flat=flat)
    c = base_mlp(m, p, prefix + ".coord_net", flat=flat)
    f = rij * c
    tot_f = np.clip(aggregate(f, row, x.shape[0], "mean"), -100, 100)
    x = x + base_mlp(h, p, prefix + ".node_v_net", flat=flat) * v + tot_f
    tot_m = aggregate(m, row, x.shape[0], "sum")
    h = base_mlp(np.concatenate([h, tot_m], axis=-1), p, prefix + ".node_net", flat=flat)
    return x, v, h


def egno_forward(p, x, h, row, col, edge_fea, v, loc_mean, t_out, n_layers=4, T=10,
                 hidden=64, time_emb_dim=32, capture=None, norm=False, use_time_conv=True, flat=False):
    """EGNO.forward (egno.py:37-111) for num_inputs == 1 (use_time_conv=False skips egno.py:99-107).

    x, v, loc_mean: [BN, 3]; h: [BN, in_node]; row/col: [E]; edge_fea: [E, in_edge];
    t_out: [Bt, T]. Returns (x, v, h) with T-major rows (t*BN + node).
    """
    dt = x.dtype
    BN = h.shape[0]
    E = row.shape[0]
    temb = timestep_embedding(t_out, time_emb_dim, dtype=dt)       # [Bt, T, H_t]
    Bt = temb.shape[0]
    # egno.py:66 broadcast: [T, Bt, Ht] -> [T, 1, Bt, Ht] -> repeat N -> [T, BN, Ht]
    temb = np.transpose(temb, (1, 0, 2))[:, None].repeat(BN // Bt, axis=1).reshape(T, BN, -1)
    hh = np.concatenate([np.broadcast_to(h[None], (T,) + h.shape), temb], axis=-1)
    hh = linear(hh.reshape(T * BN, -1), p, "embedding")
    if capture is not None:
        capture["embedding"] = hh
    offs_e = (np.arange(T) * BN).repeat(E)
    row_t = np.tile(row, T) + offs_e
    col_t = np.tile(col, T) + offs_e
    xx = np.tile(x, (T, 1))
    vv = np.tile(v, (T, 1))
    lm = np.tile(loc_mean, (T, 1)) if use_time_conv else None
    ef = np.tile(edge_fea, (T, 1))
    for i in range(n_layers):
        if not use_time_conv:
            xx, vv, hh = egnn_layer(p, f"layers.{i}", xx, hh, row_t, col_t, ef, vv, norm=norm, flat=flat)
            continue
        hh = time_conv(hh.reshape(T, BN, hidden), p[f"time_conv_modules.{i}.t_conv.weights1"])
        hh = hh.reshape(T * BN, hidden)
        X = np.stack([xx - lm, vv], axis=-1).reshape(T, BN, 3, 2)
        X = time_conv_x(X, p[f"time_conv_x_modules.{i}.t_conv.weights1"])
        xx = X[..., 0].reshape(T * BN, 3) + lm
        vv = X[..., 1].reshape(T * BN, 3)
        if capture is not None:
            capture[f"tconv{i}"] = (hh, xx, vv)
        xx, vv, hh = egnn_layer(p, f"layers.{i}", xx, hh, row_t, col_t, ef, vv, norm=norm, flat=flat)
        if capture is not None:
            capture[f"layer{i}"] = (xx, vv, hh)
    return xx, vv, hh


def frame_inputs(num_inputs, T):
    """repeat_elements_to_exact_shape (EGNO/utils.py:115-131) as a frame -> input index map: each
    input repeated T // I times in order, then the last input T % I more times."""
    k = T // num_inputs
    return np.array([min(t // k, num_inputs - 1) if k > 0 else num_inputs - 1 for t in range(T)])


def egno_forward_multi(p, x, h, row, col, edge_fea, v, loc_mean, t_in, t_out, n_layers=4, T=10,
                       hidden=64, time_emb_dim=32, norm=False, use_time_conv=True, flat=False):
    """EGNO.forward (egno.py:37-111) for num_inputs = I > 1.

    x, v, loc_mean: [I, BN, 3]; h: [I, BN, in_node]; edge_fea: [I, E, in_edge]; t_in: [Bt, I];
    t_out: [Bt, T]. Frame t reads input frame_inputs(I, T)[t] (egno.py:80-96); the embedding input
    is [h, temb(t_in), temb(t_out)] (egno.py:44-49, 77-79), both embeddings broadcast as egno.py:66."""
    dt = x.dtype
    I, BN = h.shape[0], h.shape[1]
    E = row.shape[0]
    f = frame_inputs(I, T)

    def spread(temb):   # [Bt, T, Ht] -> [T, BN, Ht] with the egno.py:66 broadcast
        Bt = temb.shape[0]
        return np.transpose(temb, (1, 0, 2))[:, None].repeat(BN // Bt, axis=1).reshape(T, BN, -1)

    temb_in = spread(timestep_embedding(t_in[:, f], time_emb_dim, dtype=dt))
    temb_out = spread(timestep_embedding(t_out, time_emb_dim, dtype=dt))
    hh = np.concatenate([h[f], temb_in, temb_out], axis=-1)
    hh = linear(hh.reshape(T * BN, -1), p, "embedding")
    offs_e = (np.arange(T) * BN).repeat(E)
    row_t = np.tile(row, T) + offs_e
    col_t = np.tile(col, T) + offs_e
    xx = x[f].reshape(T * BN, 3)
    vv = v[f].reshape(T * BN, 3)
    lm = loc_mean[f].reshape(T * BN, 3) if use_time_conv else None
    ef = edge_fea[f].reshape(T * E, -1)
    for i in range(n_layers):
        if not use_time_conv:
            xx, vv, hh = egnn_layer(p, f"layers.{i}", xx, hh, row_t, col_t, ef, vv, norm=norm, flat=flat)
            continue
        hh = time_conv(hh.reshape(T, BN, hidden), p[f"time_conv_modules.{i}.t_conv.weights1"])
        hh = hh.reshape(T * BN, hidden)
        X = np.stack([xx - lm, vv], axis=-1).reshape(T, BN, 3, 2)
        X = time_conv_x(X, p[f"time_conv_x_modules.{i}.t_conv.weights1"])
        xx = X[..., 0].reshape(T * BN, 3) + lm
        vv = X[..., 1].reshape(T * BN, 3)
        xx, vv, hh = egnn_layer(p, f"layers.{i}", xx, hh, row_t, col_t, ef, vv, norm=norm, flat=flat)
    return xx, vv, hh


def num_modes_for(num_timesteps, num_modes):
    """egno.py:26."""
    return min(num_timesteps, num_modes) if num_timesteps != 5 else min(num_modes, 3)
