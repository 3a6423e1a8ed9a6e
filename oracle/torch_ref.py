"""Op-by-op PyTorch CPU restatement of the reference hot path. TEST / BASELINE INFRASTRUCTURE ONLY.

This is the "reference CPU path" of BASELINE.md §3 and SURVEY §8d: the same torch operators the
reference dispatches (index gathers, torch.cat, nn.Linear / SiLU, scatter_add_, torch.fft.rfft /
irfft, the dense one-hot segment mean of SEGNO) in the same order, run on the host cores. bench.py
times it as `cpu_baseline` (kind "torch-ref") and checks the HIP path against its outputs; tests/
pin it to the fixtures recorded from the reference (tests/test_torch_ref.py). Nothing in the product
package imports it.

Parameters are a dict keyed like the reference state_dict. Functions are autograd-compatible, so
the C4 baseline (forward + MSE + backward + Adam) runs through torch autograd like the reference.
"""
import math

import torch
import torch.nn.functional as F


def _lin(x, p, name):
    """nn.Linear (x @ W^T + b)."""
    return F.linear(x, p[name + ".weight"], p.get(name + ".bias"))


def _mlp(x, p, name, last_act=False, flat=False):
    """BaseMLP (basic.py:34-58): Linear, SiLU, Linear[, SiLU]; flat (basic.py:38-40): Tanh (the 4x
    hidden width is the weights' shape)."""
    act = torch.tanh if flat else F.silu
    y = _lin(act(_lin(x, p, name + ".mlp.0")), p, name + ".mlp.2")
    return act(y) if last_act else y


def timestep_embedding(t, dim=32, max_positions=10000):
    """get_timestep_embedding (layer_no.py:8-17): [B, T] -> [B, T, dim]."""
    half = dim // 2
    freqs = torch.exp(torch.arange(half, dtype=torch.float32) * -(math.log(max_positions) / (half - 1)))
    e = t.float()[..., None] * freqs
    out = torch.cat([torch.sin(e), torch.cos(e)], dim=-1)
    return F.pad(out, (0, 1)) if dim % 2 == 1 else out


def _spectral(x, w):
    """SpectralConv1d[_x] (layer_no.py:96-109, 152-162): rfft over dim 0, M-mode complex channel
    mix (einsum, layer_no.py:74-77 / 129-132), irfft(n=T) with the other modes zero."""
    T = x.shape[0]
    M = min(w.shape[2], T // 2 + 1)
    xf = torch.fft.rfft(x if x.dtype == torch.float64 else x.float(), dim=0)   # f64 kept for oracle use
    wc = torch.view_as_complex(w[:, :, :M].contiguous())             # [Cin, Cout, M]
    out = torch.zeros((T // 2 + 1,) + tuple(x.shape[1:-1]) + (w.shape[1],), dtype=xf.dtype)
    out = torch.cat([torch.einsum("m...i,iom->m...o", xf[:M], wc), out[M:]], dim=0)
    return torch.fft.irfft(out, n=T, dim=0)


def _scatter(msg, row, n, mean):
    """aggregate (basic.py:6-31): scatter_add_ sum, mean = sum / clamp(count, 1)."""
    out = torch.zeros(n, msg.shape[1], dtype=msg.dtype).index_add(0, row, msg)
    if mean:
        cnt = torch.zeros(n, dtype=msg.dtype).index_add(0, row, torch.ones_like(row, dtype=msg.dtype))
        out = out / cnt.clamp(min=1)[:, None]
    return out


def egnn_layer(p, pre, x, h, row, col, ef, v, norm=False, flat=False):
    """EGNN_Layer.forward (basic.py:167-186): with_v, flat=False; norm: F.normalize of the radial
    input (basic.py:140-141)."""
    rij = x[row] - x[col]
    s = (rij * rij).sum(-1, keepdim=True)                         # InvariantScalarNet Gram (basic.py:136-143)
    if norm:
        s = F.normalize(s, p=2, dim=-1)
    m = _mlp(torch.cat([s, h[row], h[col], ef], -1), p, pre + ".edge_message_net.scalar_net", last_act=True,
             flat=flat)
    f = rij * _mlp(m, p, pre + ".coord_net", flat=flat)
    x = x + _mlp(h, p, pre + ".node_v_net", flat=flat) * v + _scatter(f, row, x.shape[0], True).clamp(-100, 100)
    h = _mlp(torch.cat([h, _scatter(m, row, x.shape[0], False)], -1), p, pre + ".node_net", flat=flat)
    return x, v, h


def egno_forward(p, x, h, row, col, ef, v, loc_mean, t_out, n_layers=4, T=10, hidden=64, time_emb_dim=32,
                 norm=False, use_time_conv=True, lrelu_masks=None, lrelu_record=None, flat=False):
    """EGNO.forward (egno.py:37-111), num_inputs == 1. Returns (x, v, h), T-major rows.
    use_time_conv=False skips egno.py:99-107. lrelu_masks: per layer a [T, BN, hidden] bool tensor of
    given LeakyReLU branch decisions (y > 0) for TimeConv's activation (layer_no.py:123), in place of
    the decisions of this evaluation: a gradient at another evaluation's kinks (tests only);
    lrelu_record: a list that receives each layer's pre-activation y."""
    BN, E = h.shape[0], row.shape[0]
    temb = timestep_embedding(t_out, time_emb_dim)                     # [Bt, T, Ht]
    Bt = temb.shape[0]
    temb = temb.permute(1, 0, 2)[:, None].repeat(1, BN // Bt, 1, 1).reshape(T, BN, -1)   # egno.py:66
    hh = _lin(torch.cat([h[None].expand(T, -1, -1), temb], -1).reshape(T * BN, -1), p, "embedding")
    off = (torch.arange(T) * BN).repeat_interleave(E)                  # egno.py:89-96
    row_t, col_t = row.repeat(T) + off, col.repeat(T) + off
    xx, vv, eft = x.repeat(T, 1), v.repeat(T, 1), ef.repeat(T, 1)
    lm = loc_mean.repeat(T, 1) if use_time_conv else None
    for i in range(n_layers):
        if not use_time_conv:
            xx, vv, hh = egnn_layer(p, f"layers.{i}", xx, hh, row_t, col_t, eft, vv, norm=norm, flat=flat)
            continue
        h3 = hh.reshape(T, BN, hidden)
        y = _spectral(h3, p[f"time_conv_modules.{i}.t_conv.weights1"])
        if lrelu_record is not None:
            lrelu_record.append(y.detach())
        y = F.leaky_relu(y) if lrelu_masks is None else torch.where(lrelu_masks[i], y, 0.01 * y)
        hh = (h3 + y).reshape(T * BN, hidden)
        X = torch.stack([xx - lm, vv], -1).reshape(T, BN, 3, 2)
        X = X + _spectral(X, p[f"time_conv_x_modules.{i}.t_conv.weights1"])
        xx = X[..., 0].reshape(T * BN, 3) + lm
        vv = X[..., 1].reshape(T * BN, 3)
        xx, vv, hh = egnn_layer(p, f"layers.{i}", xx, hh, row_t, col_t, eft, vv, norm=norm, flat=flat)
    return xx, vv, hh


def segment_mean_dense(data, seg):
    """unsorted_segment_mean (gcl.py:16-23): dense one-hot [max(seg)+1, E] built on the CPU,
    L1 row-normalised, then a matmul."""
    M = torch.zeros(int(seg.max()) + 1, data.shape[0], dtype=data.dtype)
    M[seg, torch.arange(data.shape[0])] = 1
    return F.normalize(M, p=1, dim=1) @ data


def gcl(p, h, row, col, x, v, ea, n_sub, recurrent=True, coords_weight=1.0, dense_mean=True, tanh=False):
    """SEGNO_GCL.forward (gcl.py:111-119), attention off; tanh: coord_mlp ends in nn.Tanh (gcl.py:57-59)."""
    diff = x[row] - x[col]
    radial = (diff ** 2).sum(1, keepdim=True)                          # coord2radial gcl.py:104-109
    m = F.silu(_lin(F.silu(_lin(torch.cat([h[row], h[col], radial, ea], 1), p, "module.edge_mlp.0")),
                    p, "module.edge_mlp.2"))
    c = _lin(F.silu(_lin(m, p, "module.coord_mlp.0")), p, "module.coord_mlp.2")
    trans = (diff * (torch.tanh(c) if tanh else c)).clamp(-100, 100)
    agg = segment_mean_dense(trans, row) if dense_mean else _scatter(trans, row, x.shape[0], True)
    v = v + agg * coords_weight / n_sub
    x = x + v / n_sub
    out = _lin(F.silu(_lin(torch.cat([h, _scatter(m, row, x.shape[0], False)], 1), p, "module.node_mlp.0")),
               p, "module.node_mlp.2")
    return (h + out if recurrent else out), x, v


def segno_forward_step(p, his, x, row, col, v, ea, T=10, dense_mean=True, recurrent=True, tanh=False):
    """SEGNO embedding (model.py:73) + forward_step (model.py:95-102): T substeps, dt = 1/T.
    Returns (x, h, v)."""
    h = _lin(his, p, "embedding")
    for _ in range(T):
        h, x, v = gcl(p, h, row, col, x, v, ea, T, recurrent=recurrent, dense_mean=dense_mean, tanh=tanh)
    return x, h, v


def prepare_inputs(loc, vel, ea_o, row, col, N, charges):
    """prepare_inputs (main_simulation_simple_no.py:311-339), num_inputs == 1: loc, vel [B, N, 3]."""
    lm = loc.mean(1, keepdim=True).repeat(1, N, 1).reshape(-1, 3)
    loc, vel = loc.reshape(-1, 3), vel.reshape(-1, 3)
    nodes = torch.cat([vel.norm(dim=1, keepdim=True), charges.reshape(-1, 1)], 1)
    ea = torch.cat([ea_o, ((loc[row] - loc[col]) ** 2).sum(1, keepdim=True)], 1)
    return loc, vel, ea, nodes, lm


def egno_rollout(p, nodes, loc, row, col, vel, ea_o, ea, lm, N, traj_len, B, charges, T=10, t_out=None):
    """rollout_fn (main_simulation_simple_no.py:342-384) positions, num_inputs == 1: each segment
    restarts from its last frame and re-featurises (energies are host numpy in the reference and
    not part of this timing)."""
    preds = []
    for i in range(traj_len):
        lo, vo, _ = egno_forward(p, loc, nodes, row, col, ea, vel, lm, t_out[:, i * T:(i + 1) * T] - i * T, T=T)
        preds.append(lo)
        la, va = lo.reshape(T, B, N, 3)[-1], vo.reshape(T, B, N, 3)[-1]
        loc, vel, ea, nodes, lm = prepare_inputs(la, va, ea_o, row, col, N, charges)
    return torch.stack(preds).reshape(traj_len * T, -1, 3)


def segno_rollout(p, his, x, row, col, v, ea, num_steps, charges, dense_mean=False):
    """rollout_fn (train_nbody.py:200-236) positions, num_prev == 1, through forward_step: each
    segment predicts the endpoint after its substeps and re-featurises h = |v| and the loc_dist
    column of edge_attr (:228-233). Returns [len(num_steps), BN, 3]."""
    q = charges.reshape(-1, 1)
    prod = q[row] * q[col]
    preds = []
    for T in num_steps:
        x, _, v = segno_forward_step(p, his, x, row, col, v, ea, T=int(T), dense_mean=dense_mean)
        preds.append(x)
        his = v.norm(dim=1, keepdim=True)
        ea = torch.cat([prod, ((x[row] - x[col]) ** 2).sum(1, keepdim=True)], 1)
    return torch.stack(preds)


def full_edges(B, N):
    """get_edges (dataset_simple.py:101-111): row = receiver, col = sender, (b, i, j != i)."""
    i, j = torch.meshgrid(torch.arange(N), torch.arange(N), indexing="ij")
    keep = i != j
    off = (torch.arange(B) * N).repeat_interleave(int(keep.sum()))
    return i[keep].repeat(B) + off, j[keep].repeat(B) + off
