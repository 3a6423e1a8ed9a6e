"""Oracle restatement of SEGNO (reference SEGNO/models/model.py, models/gcl.py). Test-only."""
import numpy as np

from .egno import linear, silu


def segment_sum(data, seg, n):
    """unsorted_segment_sum (gcl.py:7-13)."""
    out = np.zeros((n, data.shape[1]), dtype=data.dtype)
    np.add.at(out, seg, data)
    return out


def segment_mean_dense(data, seg):
    """unsorted_segment_mean (gcl.py:16-23): dense one-hot [max(seg)+1, E], L1 row-normalised,
    then a matmul. O(n*E) memory: small cases only."""
    E = data.shape[0]
    M = np.zeros((seg.max() + 1, E), dtype=data.dtype)
    M[seg, np.arange(E)] = 1
    M = M / np.maximum(np.abs(M).sum(1, keepdims=True), 1e-12)
    return M @ data


def segment_mean(data, seg, n):
    """Same value as segment_mean_dense (sum / count) without the dense matrix."""
    cnt = np.bincount(seg, minlength=n).astype(data.dtype)
    return segment_sum(data, seg, n) / np.maximum(cnt, 1)[:, None]


def gcl_forward(p, h, row, col, x, v, edge_attr, n_layers, recurrent=True,
                coords_weight=1.0, dense_mean=False, tanh=False):
    """SEGNO_GCL.forward (gcl.py:111-119) with attention=False, node_attr=None; tanh: the
    coordinate MLP ends in nn.Tanh (gcl.py:57-59)."""
    diff = x[row] - x[col]                                   # coord2radial gcl.py:104-109
    radial = np.sum(diff ** 2, axis=1, keepdims=True)
    inp = np.concatenate([h[row], h[col], radial, edge_attr], axis=1)   # gcl.py:78
    m = silu(linear(silu(linear(inp, p, "module.edge_mlp.0")), p, "module.edge_mlp.2"))
    c = linear(silu(linear(m, p, "module.coord_mlp.0")), p, "module.coord_mlp.2")
    if tanh:
        c = np.tanh(c)
    trans = np.clip(diff * c, -100, 100)                      # gcl.py:97-102
    agg = segment_mean_dense(trans, row) if dense_mean else segment_mean(trans, row, x.shape[0])
    agg = agg * coords_weight
    v = v + agg * (1.0 / n_layers)
    x = x + v * (1.0 / n_layers)
    aggm = segment_sum(m, row, x.shape[0])                    # node_model gcl.py:85-95
    out = linear(silu(linear(np.concatenate([h, aggm], axis=1), p, "module.node_mlp.0")),
                 p, "module.node_mlp.2")
    h = h + out if recurrent else out
    return h, x, v


def forward_step(p, h, x, row, col, v, edge_attr, T=10, **kw):
    """SEGNO.forward_step (model.py:95-102): T substeps, dt = 1/T."""
    for _ in range(T):
        h, x, v = gcl_forward(p, h, row, col, x, v, edge_attr, n_layers=T, **kw)
    return x, h, v


def forward(p, his, x, row, col, v, edge_attr, T=10, bug_compat=True, **kw):
    """SEGNO.forward (model.py:53-92), single input.

    bug_compat=True reproduces the live reference: x_, h_, v_ are only reassigned when
    i < len(steps)-1, so with one input the inputs come back unchanged.
    bug_compat=False returns the integrator result (the shadowed forward at model.py:28-51).
    """
    h = linear(his, p, "embedding")
    if bug_compat:
        forward_step(p, h, x, row, col, v, edge_attr, T=T, **kw)
        return x, h, v
    return forward_step(p, h, x, row, col, v, edge_attr, T=T, **kw)


def attn_combine(p, loc_seq, vel_seq, his_seq):
    """prepare_node_inputs + InvariantTemporalAttention (model.py:104-139): softmax over the stacked
    inputs of attn_mlp([|v|, h]) = Linear(Tanh(Linear(.))), then attention-weighted sums."""
    speed = np.sqrt((vel_seq ** 2).sum(-1, keepdims=True))                      # (BN, K, 1)
    feats = np.concatenate([speed, his_seq], axis=-1)
    z = np.tanh(feats @ p["enc_attn_net.attn_mlp.0.weight"].T + p["enc_attn_net.attn_mlp.0.bias"])
    a = z @ p["enc_attn_net.attn_mlp.2.weight"].T + p["enc_attn_net.attn_mlp.2.bias"]   # (BN, K, 1)
    a = np.exp(a - a.max(axis=1, keepdims=True))
    a = a / a.sum(axis=1, keepdims=True)
    return (a * loc_seq).sum(1), (a * vel_seq).sum(1), (a * his_seq).sum(1)


def forward_multi(p, his, x, row, col, v, edge_attr, in_steps, T=10, multiple_agg="attn", bug_compat=True, **kw):
    """The live SEGNO.forward (model.py:53-92) with num_inputs > 1: his [BN, I, F], x, v [BN, I, 3],
    in_steps [I]. forward_step runs diff(in_steps) + [T] substeps in turn, folding each next input
    in ('sum' or 'attn'). The reference returns the state before the last forward_step
    (bug_compat=True); bug_compat=False returns that last step's result."""
    steps = list(np.diff(np.asarray(in_steps))) + [T]
    h = his @ p["embedding.weight"].T + p["embedding.bias"]
    h_, x_, v_ = h[:, 0], x[:, 0], v[:, 0]
    for i, step in enumerate(steps):
        xi, hi, vi = forward_step(p, h_, x_, row, col, v_, edge_attr, T=int(step), **kw)
        if i < len(steps) - 1:
            if multiple_agg == "sum":
                h_, x_, v_ = h[:, i + 1] + hi, x[:, i + 1] + xi, v[:, i + 1] + vi
            elif multiple_agg == "attn":
                x_, v_, h_ = attn_combine(p, np.stack([x[:, i + 1], xi], 1), np.stack([v[:, i + 1], vi], 1),
                                          np.stack([h[:, i + 1], hi], 1))
    return (x_, h_, v_) if bug_compat else (xi, hi, vi)
