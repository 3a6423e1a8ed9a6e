"""Oracle restatement of the hot-path callers (featurisation, rollout, energy). Test-only."""
import numpy as np

from . import egno as _egno
from . import segno as _segno


def full_edges(B, N):
    """NBodyDataset edge list (dataset_simple.py:64-71) offset per sample (get_edges :101-111):
    row = receiver i, col = sender j, ordered (b, i, j != i)."""
    i, j = np.meshgrid(np.arange(N), np.arange(N), indexing="ij")
    keep = i != j
    r, c = i[keep], j[keep]
    offs = (np.arange(B) * N).repeat(r.size)
    return np.tile(r, B) + offs, np.tile(c, B) + offs


def prepare_inputs(loc, vel, edge_attr_o, row, col, n_nodes, charges):
    """prepare_inputs (main_simulation_simple_no.py:311-339), num_inputs == 1.

    loc, vel: [B, N, 3]; edge_attr_o: [E, 1]; charges [B, N, 1] -> (loc, vel, edge_attr,
    nodes, loc_mean) with loc/vel/loc_mean [BN, 3], nodes [BN, 2], edge_attr [E, 2].
    """
    B = loc.shape[0]
    loc_mean = np.repeat(loc.mean(axis=1, keepdims=True), n_nodes, axis=1).reshape(-1, 3)
    loc = loc.reshape(-1, 3)
    vel = vel.reshape(-1, 3)
    nodes = np.sqrt(np.sum(vel ** 2, axis=1))[:, None]
    if charges is not None:
        nodes = np.concatenate([nodes, charges.reshape(-1, 1)], axis=1)
    loc_dist = np.sum((loc[row] - loc[col]) ** 2, axis=1)[:, None]
    edge_attr = np.concatenate([edge_attr_o, loc_dist], axis=1)
    del B
    return loc, vel, edge_attr.astype(loc.dtype), nodes.astype(loc.dtype), loc_mean


def energy_charged_batch(loc, vel, edges, interaction_strength=1.0):
    """tot_energy_charged_batch (utils.py:126-144): loc, vel [B, N, 3]; edges [B, N, N]."""
    K = 0.5 * np.sum(np.sum(vel ** 2, axis=-1), axis=-1)
    d = np.linalg.norm(loc[:, :, None, :] - loc[:, None, :, :], axis=-1)
    d = np.where(d == 0, np.inf, d)
    U = 0.5 * interaction_strength * np.sum(edges / d, axis=(-1, -2))
    return K + U


def energy_gravity_batch(loc, vel, mass, G=1.0):
    """tot_energy_gravity_batch (utils.py:175-195): mass [B, N, 1]."""
    KE = np.squeeze(0.5 * np.sum(np.sum(mass * vel ** 2, axis=-1), axis=-1))
    dx = loc[:, None, :, :] - loc[:, :, None, :]
    r = np.sqrt(np.sum(dx ** 2, axis=-1))
    inv = np.zeros_like(r)
    nz = r > 0
    inv[nz] = 1.0 / r[nz]
    mm = mass * np.transpose(mass, (0, 2, 1))
    PE = G * np.sum(np.triu(-mm * inv, 1), axis=(-1, -2))
    return KE + PE


def conserved_energy(dataset, loc, vel, charges, B):
    """conserved_energy_fun (utils.py:197-219) for equal-size graphs: loc/vel [BN, 3]."""
    loc = loc.reshape(B, -1, 3)
    vel = vel.reshape(B, -1, 3)
    q = charges.reshape(B, -1, 1)
    if dataset == "gravity":
        return energy_gravity_batch(loc, vel, q)
    qq = q * np.transpose(q, (0, 2, 1))     # einsum('tij,tji->tij') of the repeated charges
    return energy_charged_batch(loc, vel, qq)


def egno_rollout(p, nodes, loc, row, col, vel, edge_attr_o, edge_attr, loc_mean, n_nodes,
                 traj_len, B, charges, T=10, t_out=None, energy=True, t_in=None, dataset="charged", **kw):
    """rollout_fn (main_simulation_simple_no.py:342-384) for num_inputs == 1.

    Each segment: model call, keep all T frames, restart from frame t_in[b] - 1 of each sample
    (loc_all[timesteps_in.T - 1, batch_indices], :365-368; python indexing, so t_in = 0 is the
    LAST frame; t_in None = last frame), re-featurise with prepare_inputs (:371).
    """
    preds, energies, energies_all = [], [], []
    for i in range(traj_len):
        t = t_out[:, i * T:(i + 1) * T] - i * T
        loc_o, vel_o, _ = _egno.egno_forward(p, loc, nodes, row, col, edge_attr, vel, loc_mean,
                                             t, T=T, **kw)
        preds.append(loc_o)
        la = loc_o.reshape(T, B, n_nodes, 3)
        va = vel_o.reshape(T, B, n_nodes, 3)
        fr = np.full(B, -1) if t_in is None else np.asarray(t_in).reshape(-1) - 1
        bi = np.arange(B)
        loc, vel, edge_attr, nodes, loc_mean = prepare_inputs(
            la[fr, bi], va[fr, bi], edge_attr_o, row, col, n_nodes, charges)
        if energy:
            for j in range(T):
                en = conserved_energy(dataset, la[j], va[j], charges, B)
                energies_all.append(en)
                if j == T - 1:
                    energies.append(en)
    out = np.stack(preds).reshape(traj_len * T, -1, 3)
    if energy:
        return out, np.stack(energies)[..., None], np.stack(energies_all)[..., None]
    return out, None, None


def segno_rollout(p, h, loc, row, col, vel, edge_attr, traj_len, num_steps, charges, B,
                  energy=True, dataset="charged", **kw):
    """rollout_fn (train_nbody.py:200-236), num_prev == 1, through forward_step.

    Each segment: predict the endpoint after T substeps, feed it back, recompute h = |v| and
    the loc_dist column of edge_attr (:228-233).
    """
    prod = charges.reshape(-1, 1)[row] * charges.reshape(-1, 1)[col]
    preds, energies = [], []
    for i in range(traj_len):
        T = num_steps[i] if isinstance(num_steps, (list, tuple, np.ndarray)) else num_steps
        hh = _egno.linear(h, p, "embedding")
        loc_p, _, vel_p = _segno.forward_step(p, hh, loc, row, col, vel, edge_attr, T=int(T), **kw)
        if energy:
            energies.append(conserved_energy(dataset, loc_p, vel_p, charges, B))
        preds.append(loc_p)
        loc, vel = loc_p, vel_p
        h = np.sqrt(np.sum(vel ** 2, axis=1))[:, None]
        loc_dist = np.sum((loc[row] - loc[col]) ** 2, axis=1)[:, None]
        edge_attr = np.concatenate([prod, loc_dist], axis=1).astype(loc.dtype)
    return np.stack(preds), (np.stack(energies)[..., None] if energy else None)
