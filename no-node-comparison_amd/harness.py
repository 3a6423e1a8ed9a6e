"""GPU counterparts of the reference's hot-path callers.

prepare_inputs / conserved_energy / egno_rollout / segno_rollout keep the reference's argument
meaning and return values (EGNO/main_simulation_simple_no.py:311-384, SEGNO/train_nbody.py:200-236,
utils.py:197-219) but run as HIP kernels (csrc/nonode_rollout.hip): the rollouts are ONE C call
each (segments, re-featurisation and per-frame energies on the device, no host round trip).
Like the models, these have no CPU path: tensors must be on the ROCm device.
"""
import ctypes

import torch

from . import _lib
from .graph import full_edges  # noqa: F401  (re-exported: get_edges counterpart)

ENERGY_KIND = {"charged": 0, "gravity": 1}


def _f32(t):
    return t.detach().to(torch.float32).contiguous() if t is not None else None


def get_edges(batch_size, n_nodes, device="cpu"):
    """NBodyDataset.get_edges (dataset_simple.py:101-111) for the fully connected graph."""
    r, c = full_edges(batch_size, n_nodes, device)
    return [r, c]


@torch.no_grad()
def prepare_inputs(loc, vel, edge_attr_o, edges, n_nodes, num_inputs=1, charges=None, t_in=None):
    """main_simulation_simple_no.py:311-339 (nonode_prepare_inputs; num_inputs > 1 per input slot).

    loc, vel: [B, N, 3] (one frame) or [F, B, N, 3] with ``t_in`` [B] choosing frame t_in-1 per
    sample (rollout_fn's loc_all[timesteps_in.T - 1]). edges must be the dataset's fully connected
    list (only its size is used: the kernel indexes pairs implicitly). Returns
    (loc [BN,3], vel [BN,3], edge_attr [E, n_eo+1], nodes [BN, 1(+1)], loc_mean [BN,3])."""
    if num_inputs > 1:
        return _prepare_inputs_multi(loc, vel, edge_attr_o, edges, n_nodes, num_inputs, charges)
    _lib.require_device(loc, vel, edge_attr_o, charges)
    if loc.dim() == 3:
        loc, vel = loc.unsqueeze(0), vel.unsqueeze(0)
    F, B, N = loc.shape[0], loc.shape[1], loc.shape[2]
    if N != n_nodes:
        raise ValueError(f"prepare_inputs: loc has {N} nodes per graph, n_nodes={n_nodes}")
    E = B * N * (N - 1)
    if edges is not None and edges[0].numel() != E:
        raise ValueError("prepare_inputs: edges must be the fully connected list of B graphs")
    eo = _f32(edge_attr_o).reshape(E, -1)
    n_eo = eo.shape[1]
    loc, vel = _f32(loc), _f32(vel)
    q = _f32(charges).reshape(-1) if charges is not None else None
    ti = t_in.reshape(-1).to(torch.int32).contiguous() if t_in is not None else None
    dev = loc.device
    BN = B * N
    x = torch.empty(BN, 3, device=dev)
    v = torch.empty(BN, 3, device=dev)
    nodes = torch.empty(BN, 2 if q is not None else 1, device=dev)
    ea = torch.empty(E, n_eo + 1, device=dev)
    lm = torch.empty(BN, 3, device=dev)
    L = _lib.lib()
    _lib.check(L.nonode_prepare_inputs(B, N, F, _lib.ptr(loc), _lib.ptr(vel), _lib.ptr(ti), _lib.ptr(q), _lib.ptr(eo),
                                       n_eo, _lib.ptr(x), _lib.ptr(v), _lib.ptr(nodes), _lib.ptr(ea), _lib.ptr(lm),
                                       _lib.stream_of(loc)))
    return x, v, ea, nodes, lm


def _prepare_inputs_multi(loc, vel, edge_attr_o, edges, n_nodes, num_inputs, charges):
    """main_simulation_simple_no.py:313-327 (num_inputs = I > 1), literally: loc, vel are transposed
    on their first two axes and reshaped to I slots of B*N rows ([B, I, N, 3] from the loader gives
    one slot per input); each slot is featurised like a single input (per-graph mean, |v| (+ q),
    [edge_attr_o, |x_i - x_j|^2]). Returns x, v, loc_mean [I, BN, 3], edge_attr [I, E, n_eo+1],
    nodes [I, BN, 1(+1)]."""
    I = num_inputs
    lt = loc.transpose(0, 1).contiguous().reshape(I, -1, n_nodes, 3)
    vt = vel.transpose(0, 1).contiguous().reshape(I, -1, n_nodes, 3)
    outs = [prepare_inputs(lt[i], vt[i], edge_attr_o, edges, n_nodes, 1, charges) for i in range(I)]
    x, v, ea, nodes, lm = (torch.stack([o[k] for o in outs]) for k in range(5))
    return x, v, ea, nodes, lm


@torch.no_grad()
def egno_rollout_multi(model, nodes, loc, edges, vel, edge_attr_o, edge_attr, loc_mean, n_nodes, traj_len,
                       batch_size, charges=None, num_steps=10, timesteps_in=None, timesteps_out=None,
                       energy_dataset=None):
    """rollout_fn (main_simulation_simple_no.py:342-384) for num_inputs > 1: per segment the HIP
    forward, then the frames timesteps_in - 1 of each sample become the next inputs and go through
    prepare_inputs exactly as the reference passes them ([I, B, N, 3], which prepare_inputs
    transposes). Returns (loc_preds [traj_len*T, BN, 3], energies, energies_allsteps) like
    egno_rollout."""
    T = model.num_timesteps
    B, N = batch_size, n_nodes
    t_in = timesteps_in if timesteps_in.dim() == 2 else timesteps_in.unsqueeze(-1)
    bidx = torch.arange(B, device=loc.device).unsqueeze(0).expand(t_in.shape[1], -1)
    preds = torch.empty(traj_len * T, B * N, 3, device=loc.device)
    en_all = []
    for i in range(traj_len):
        t_out = timesteps_out[:, i * T:(i + 1) * T] - i * T
        x, v, _ = model(loc, nodes, edges, edge_attr, v=vel, loc_mean=loc_mean, timesteps_out=t_out,
                        timesteps_in=t_in)
        preds[i * T:(i + 1) * T] = x.reshape(T, B * N, 3)
        loc_all, vel_all = x.view(T, B, N, 3), v.view(T, B, N, 3)
        sel = (t_in.T - 1).long()
        loc, vel = loc_all[sel, bidx], vel_all[sel, bidx]
        loc, vel, edge_attr, nodes, loc_mean = prepare_inputs(loc, vel, edge_attr_o, edges, N, t_in.shape[1],
                                                              charges)
        if energy_dataset is not None:
            en_all.append(conserved_energy(energy_dataset, loc_all.reshape(T, B * N, 3),
                                           vel_all.reshape(T, B * N, 3), charges, B))
    if energy_dataset is None:
        return preds, None, None
    en_all = torch.cat(en_all).unsqueeze(-1)
    return preds, en_all[T - 1::T], en_all


@torch.no_grad()
def conserved_energy(dataset, loc, vel, charges, batch_size):
    """conserved_energy_fun (utils.py:197-219) on the GPU: loc, vel [..., B*N, 3] (leading frame
    axes allowed), charges (charged) or masses (gravity) [B*N] -> energies [..., B]."""
    _lib.require_device(loc, vel, charges)
    B = batch_size
    lead = loc.shape[:-2]
    BN = loc.shape[-2] if loc.dim() >= 2 else loc.numel() // 3
    loc, vel = _f32(loc).reshape(-1, BN, 3), _f32(vel).reshape(-1, BN, 3)
    F, N = loc.shape[0], BN // B
    w = _f32(charges).reshape(-1)
    out = torch.empty(F, B, device=loc.device)
    _lib.check(_lib.lib().nonode_energy(ENERGY_KIND[dataset], F, B, N, _lib.ptr(loc), _lib.ptr(vel), _lib.ptr(w),
                                        _lib.ptr(out), _lib.stream_of(loc)))
    return out.reshape(*lead, B) if len(lead) else out.reshape(B)


@torch.no_grad()
def egno_rollout(model, nodes, loc, edges, vel, edge_attr_o, edge_attr, loc_mean, n_nodes, traj_len,
                 batch_size, charges=None, num_steps=10, timesteps_in=None, timesteps_out=None,
                 energy_dataset=None):
    """rollout_fn (main_simulation_simple_no.py:342-384), num_inputs == 1, as one native call.

    Returns (loc_preds [traj_len*T, BN, 3], energies [traj_len, B, 1] or None,
    energies_allsteps [traj_len*T, B, 1] or None). Unlike the reference, ``timesteps_out`` is not
    modified in place (the reference's ``t_out -= i*T`` writes into the caller's tensor)."""
    from .egno import EGNO
    if not isinstance(model, EGNO):
        raise TypeError("egno_rollout drives no_node_comparison_amd.EGNO (its packed weights)")
    if model.num_inputs > 1:
        return egno_rollout_multi(model, nodes, loc, edges, vel, edge_attr_o, edge_attr, loc_mean, n_nodes,
                                  traj_len, batch_size, charges, num_steps, timesteps_in, timesteps_out,
                                  energy_dataset)
    T = model.num_timesteps
    if num_steps != T:
        raise ValueError("rollout_fn reshapes each segment into num_steps == model.num_timesteps frames")
    _lib.require_device(loc, nodes, vel, edge_attr, loc_mean, model.embedding.weight)
    if model.flat:
        # nonode_egno_rollout runs the 64-wide SiLU layer kernels on standard layer blobs only: a flat
        # model (256-wide Tanh blobs, nonode_pack_layer_flat) rolls out segment by segment instead
        return _egno_rollout_segments(model, nodes, loc, edges, vel, edge_attr_o, edge_attr, loc_mean, n_nodes,
                                      traj_len, batch_size, charges, timesteps_in, timesteps_out, energy_dataset)
    B, N = batch_size, n_nodes
    BN, E = B * N, B * N * (N - 1)
    dev = loc.device
    if timesteps_out is None:
        timesteps_out = torch.arange(T * traj_len, device=dev).unsqueeze(0)
    t_all = _f32(timesteps_out)
    if t_all.shape[1] != T * traj_len:
        raise ValueError(f"timesteps_out must have {T * traj_len} columns")
    Bt = t_all.shape[0]
    ti = timesteps_in.reshape(-1).to(torch.int32).contiguous() if timesteps_in is not None else None
    eo = _f32(edge_attr_o).reshape(E, -1)
    q = _f32(charges).reshape(-1) if charges is not None else None
    x, h, v, ef = _f32(loc), _f32(nodes), _f32(vel), _f32(edge_attr)
    lm = _f32(loc_mean) if loc_mean is not None else None   # unused without time convolutions
    blobs, tblobs = model._packed()
    L = _lib.lib()
    P = ctypes.c_void_p * model.n_layers
    blob_p = P(*[blobs[i].data_ptr() for i in range(model.n_layers)])
    tcw_p, tcx_p, _keep = model.tconv_arrays(tblobs)
    ew, eb = _f32(model.embedding.weight), _f32(model.embedding.bias)
    preds = torch.empty(traj_len * T, BN, 3, device=dev)
    en_all = torch.empty(traj_len * T, B, device=dev) if energy_dataset is not None else None
    ws_bytes = L.nonode_egno_rollout_workspace_bytes(B, N, T, Bt, model.in_node_nf, model.in_edge_nf)
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=dev)
    kind = ENERGY_KIND[energy_dataset] if energy_dataset is not None else -1
    _lib.check(L.nonode_egno_rollout(
        B, N, T, model.n_layers, model.in_node_nf, model.in_edge_nf, model.time_emb_dim, model.num_modes, Bt,
        traj_len, _lib.ptr(x), _lib.ptr(h), _lib.ptr(v), _lib.ptr(lm), _lib.ptr(ef), _lib.ptr(t_all), _lib.ptr(ti),
        _lib.ptr(q), _lib.ptr(eo), eo.shape[1], kind, _lib.ptr(q), _lib.ptr(ew), _lib.ptr(eb), blob_p, tcw_p, tcx_p,
        _lib.ptr(preds), _lib.ptr(en_all), _lib.ptr(ws), ws_bytes, _lib.stream_of(x)))
    if en_all is None:
        return preds, None, None
    en_all = en_all.unsqueeze(-1)
    return preds, en_all[T - 1::T], en_all


@torch.no_grad()
def _egno_rollout_segments(model, nodes, loc, edges, vel, edge_attr_o, edge_attr, loc_mean, n_nodes, traj_len,
                           batch_size, charges, timesteps_in, timesteps_out, energy_dataset):
    """rollout_fn (main_simulation_simple_no.py:342-384), num_inputs == 1, as a loop of model(...)
    segments: per segment the model's own forward (flat=True: nonode_egno_forward_flat), the frame
    t_in - 1 of each sample re-featurised by prepare_inputs (loc_all[timesteps_in.T - 1]), and the
    per-frame energies. Same returns as egno_rollout."""
    T = model.num_timesteps
    B, N = batch_size, n_nodes
    BN = B * N
    dev = loc.device
    if timesteps_out is None:
        timesteps_out = torch.arange(T * traj_len, device=dev).unsqueeze(0)
    if timesteps_out.shape[1] != T * traj_len:
        raise ValueError(f"timesteps_out must have {T * traj_len} columns")
    ti = timesteps_in.reshape(-1) if timesteps_in is not None else None   # None: the last frame (t_in = T)
    preds = torch.empty(traj_len * T, BN, 3, device=dev)
    en_all = []
    for i in range(traj_len):
        t_out = timesteps_out[:, i * T:(i + 1) * T] - i * T
        x, v, _ = model(loc, nodes, edges, edge_attr, v=vel, loc_mean=loc_mean, timesteps_out=t_out)
        preds[i * T:(i + 1) * T] = x.reshape(T, BN, 3)
        if energy_dataset is not None:
            en_all.append(conserved_energy(energy_dataset, x.reshape(T, BN, 3), v.reshape(T, BN, 3), charges, B))
        loc, vel, edge_attr, nodes, loc_mean = prepare_inputs(x.reshape(T, B, N, 3), v.reshape(T, B, N, 3),
                                                              edge_attr_o, edges, N, 1, charges, t_in=ti)
    if energy_dataset is None:
        return preds, None, None
    en_all = torch.cat(en_all).unsqueeze(-1)
    return preds, en_all[T - 1::T], en_all


@torch.no_grad()
def segno_rollout(model, h, loc, edge_index, vel, edge_attr, traj_len, num_steps=10, charges=None,
                  energy_dataset=None, batch_size=None, in_steps=None):
    """rollout_fn (train_nbody.py:200-236): num_prev == 1 as one native call; several previous
    frames (loc, vel [BN, I, 3], in_steps) as a segment loop over SEGNO's multi-input forward.

    Returns (loc_preds [traj_len, BN, 3], energies [traj_len, B, 1] or None)."""
    from .graph import check_full_graph, finish
    from .segno import SEGNO
    if not isinstance(model, SEGNO):
        raise TypeError("segno_rollout drives no_node_comparison_amd.SEGNO (its packed weights)")
    if model.bug_compat:
        raise ValueError("segno_rollout integrates (bug_compat=True would return the inputs every segment)")
    if loc.dim() == 3:
        return _segno_rollout_multi(model, h, loc, edge_index, vel, edge_attr, traj_len, num_steps, charges,
                                    energy_dataset, in_steps)
    _lib.require_device(loc, h, vel, edge_attr, charges, model.embedding.weight)
    BN = loc.shape[0]
    B, N = check_full_graph(edge_index, BN)
    steps = list(num_steps) if isinstance(num_steps, (list, tuple)) else [int(num_steps)] * traj_len
    if len(steps) != traj_len:
        raise ValueError("num_steps should be a list of length traj_len")
    dev = loc.device
    x, v, his, ea = _f32(loc), _f32(vel), _f32(h), _f32(edge_attr)
    q = _f32(charges).reshape(-1)
    rows, cols = edge_index
    prod = (q[rows.long()] * q[cols.long()]).reshape(-1, 1).contiguous()   # prod_charges (train_nbody.py:203)
    blob = model._packed()
    L = _lib.lib()
    preds = torch.empty(traj_len, BN, 3, device=dev)
    en = torch.empty(traj_len, B, device=dev) if energy_dataset is not None else None
    ws_bytes = L.nonode_segno_rollout_workspace_bytes(B, N, model.in_node_nf, model.in_edge_nf)
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=dev)
    kind = ENERGY_KIND[energy_dataset] if energy_dataset is not None else -1
    steps_arr = (ctypes.c_int * traj_len)(*[int(s) for s in steps])
    ew, eb = _f32(model.embedding.weight), _f32(model.embedding.bias)
    _lib.check(L.nonode_segno_rollout(
        B, N, model.in_node_nf, model.in_edge_nf, traj_len, steps_arr, _lib.ptr(his), _lib.ptr(x), _lib.ptr(v),
        _lib.ptr(ea), _lib.ptr(prod), 1, kind, _lib.ptr(q), _lib.ptr(ew), _lib.ptr(eb), _lib.ptr(blob),
        float(model.coords_weight), int(bool(model.recurrent)), _lib.ptr(preds), _lib.ptr(en), _lib.ptr(ws), ws_bytes,
        _lib.stream_of(x)))
    finish((preds, en))
    return preds, (en.unsqueeze(-1) if en is not None else None)


@torch.no_grad()
def _segno_rollout_multi(model, h, loc, edge_index, vel, edge_attr, traj_len, num_steps, charges, energy_dataset,
                         in_steps):
    """train_nbody.py:200-236 with num_prev = I > 1: each segment's prediction is appended to the
    window of the last I frames (the oldest dropped), |v| and the last frame's distances are
    recomputed, and in_steps shifts by the segment's substeps (:221-233)."""
    from .graph import check_full_graph
    if in_steps is None:
        raise ValueError("a multi-input SEGNO rollout needs in_steps (train_nbody.py:114)")
    BN = loc.shape[0]
    B, N = check_full_graph(edge_index, BN)
    steps = list(num_steps) if isinstance(num_steps, (list, tuple)) else [int(num_steps)] * traj_len
    if len(steps) != traj_len:
        raise ValueError("num_steps should be a list of length traj_len")
    rows, cols = (t.long() for t in edge_index)
    q = _f32(charges).reshape(-1)
    prod = (q[rows] * q[cols]).reshape(-1, 1)
    preds = torch.empty(traj_len, BN, 3, device=loc.device)
    en = []
    loc, vel = _f32(loc), _f32(vel)
    for i, T in enumerate(steps):
        loc_p, _, vel_p = model(h, loc, edge_index, vel, edge_attr, T=T, in_steps=in_steps)
        if energy_dataset is not None:
            en.append(conserved_energy(energy_dataset, loc_p, vel_p, charges, B))
        preds[i] = loc_p
        loc = torch.cat((loc[:, 1:, :], loc_p.unsqueeze(1)), dim=1)
        vel = torch.cat((vel[:, 1:, :], vel_p.unsqueeze(1)), dim=1)
        h = torch.sqrt(torch.sum(vel ** 2, dim=-1)).unsqueeze(-1)
        loc_dist = torch.sum((loc[rows, -1, :] - loc[cols, -1, :]) ** 2, 1).unsqueeze(1)
        st = in_steps.tolist() if torch.is_tensor(in_steps) else list(in_steps)
        in_steps = torch.tensor(st[1:] + [T], device=loc.device) - T
        edge_attr = torch.cat([prod, loc_dist], 1)
    return preds, (torch.stack(en).unsqueeze(-1) if en else None)
