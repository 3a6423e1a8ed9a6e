"""Device-side counterparts of the reference's hot-path callers.

prepare_inputs / rollout_fn keep the reference's argument meaning and return values
(EGNO/main_simulation_simple_no.py:311-384, SEGNO/train_nbody.py:200-236) but keep every
tensor on the GPU: no per-frame host round trip.
"""
import torch

from .graph import full_edges  # noqa: F401  (re-exported: get_edges counterpart)


def get_edges(batch_size, n_nodes, device="cpu"):
    """NBodyDataset.get_edges (dataset_simple.py:101-111) for the fully connected graph."""
    r, c = full_edges(batch_size, n_nodes, device)
    return [r, c]


def prepare_inputs(loc, vel, edge_attr_o, edges, n_nodes, num_inputs=1, charges=None):
    """main_simulation_simple_no.py:311-339 for num_inputs == 1."""
    if num_inputs != 1:
        raise NotImplementedError("prepare_inputs: num_inputs > 1")
    rows, cols = edges
    loc_mean = loc.mean(dim=1, keepdim=True).repeat(1, n_nodes, 1).view(-1, loc.size(-1))
    loc = loc.reshape(-1, loc.size(-1))
    vel = vel.reshape(-1, vel.size(-1))
    nodes = torch.sqrt(torch.sum(vel ** 2, dim=1)).unsqueeze(1)
    if charges is not None:
        nodes = torch.cat([nodes, charges.reshape(-1, 1)], dim=1)
    loc_dist = torch.sum((loc[rows] - loc[cols]) ** 2, 1).unsqueeze(1)
    edge_attr = torch.cat([edge_attr_o, loc_dist], 1)
    return loc, vel, edge_attr, nodes, loc_mean


def conserved_energy(dataset, loc, vel, charges, batch_size):
    """utils.py:197-219 (equal-size graphs) on device: returns [B] energies."""
    B = batch_size
    loc = loc.reshape(B, -1, 3)
    vel = vel.reshape(B, -1, 3)
    q = charges.reshape(B, -1, 1)
    diff = loc[:, :, None, :] - loc[:, None, :, :]
    if dataset == "gravity":
        ke = 0.5 * torch.sum(q * vel ** 2, dim=(-1, -2))
        r = diff.norm(dim=-1)
        inv = torch.where(r > 0, 1.0 / r, torch.zeros_like(r))
        pe = torch.triu(-(q * q.transpose(1, 2)) * inv, 1).sum(dim=(-1, -2))
        return ke + pe
    ke = 0.5 * torch.sum(vel ** 2, dim=(-1, -2))
    d = diff.norm(dim=-1)
    d = torch.where(d == 0, torch.full_like(d, float("inf")), d)
    pe = 0.5 * torch.sum((q * q.transpose(1, 2)) / d, dim=(-1, -2))
    return ke + pe


@torch.no_grad()
def egno_rollout(model, nodes, loc, edges, vel, edge_attr_o, edge_attr, loc_mean, n_nodes, traj_len,
                 batch_size, charges=None, num_steps=10, timesteps_in=None, timesteps_out=None,
                 energy_dataset=None):
    """rollout_fn (main_simulation_simple_no.py:342-384), num_inputs == 1, on device.

    Returns (loc_preds [traj_len*T, BN, 3], energies [traj_len, B, 1] or None,
    energies_allsteps [traj_len*T, B, 1] or None)."""
    T = model.num_timesteps
    preds, en, en_all = [], [], []
    for i in range(traj_len):
        t_out = timesteps_out[:, i * T:(i + 1) * T] - i * T
        loc_o, vel_o, _ = model(loc, nodes, edges, edge_attr, v=vel, loc_mean=loc_mean, timesteps_out=t_out,
                                timesteps_in=timesteps_in)
        preds.append(loc_o)
        la = loc_o.view(num_steps, batch_size, n_nodes, 3)
        va = vel_o.view(num_steps, batch_size, n_nodes, 3)
        loc, vel, edge_attr, nodes, loc_mean = prepare_inputs(la[-1], va[-1], edge_attr_o, edges, n_nodes, 1,
                                                              charges)
        if energy_dataset is not None:
            for j in range(num_steps):
                e = conserved_energy(energy_dataset, la[j], va[j], charges, batch_size)
                en_all.append(e)
                if j == num_steps - 1:
                    en.append(e)
    out = torch.stack(preds).reshape(traj_len * T, -1, 3)
    if energy_dataset is None:
        return out, None, None
    return out, torch.stack(en).unsqueeze(-1), torch.stack(en_all).unsqueeze(-1)


@torch.no_grad()
def segno_rollout(model, h, loc, edge_index, vel, edge_attr, traj_len, num_steps=10, charges=None,
                  energy_dataset=None, batch_size=None):
    """rollout_fn (train_nbody.py:200-236), num_prev == 1, on device."""
    rows, cols = edge_index
    prod = charges.reshape(-1, 1)[rows] * charges.reshape(-1, 1)[cols]
    preds, energies = [], []
    for i in range(traj_len):
        T = num_steps[i] if isinstance(num_steps, (list, tuple)) else num_steps
        loc_p, _, vel_p = model(h, loc, edge_index, vel, edge_attr, T=T)
        if energy_dataset is not None:
            energies.append(conserved_energy(energy_dataset, loc_p, vel_p, charges, batch_size))
        preds.append(loc_p)
        loc, vel = loc_p, vel_p
        h = torch.sqrt(torch.sum(vel ** 2, dim=1)).unsqueeze(1)
        loc_dist = torch.sum((loc[rows] - loc[cols]) ** 2, 1).unsqueeze(1)
        edge_attr = torch.cat([prod, loc_dist], 1)
    out = torch.stack(preds)
    return out, (torch.stack(energies).unsqueeze(-1) if energy_dataset is not None else None)
