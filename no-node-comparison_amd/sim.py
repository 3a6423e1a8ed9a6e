"""Synthetic N-body data on the GPU: drop-in ChargedParticlesSim / GravitySim
(synthetic_sim.py:149-296, 299-481) and generate_dataset (generate_dataset.py:62-104).

Initial conditions are drawn on the host with numpy in exactly the reference's call order
(np.random.choice / randn per simulation, then the observation-noise draws), so a given
np.random.seed reproduces the reference's datasets; the time integration runs in one kernel launch
for every trajectory of a batch (csrc/nonode_sim.hip, float64). Outputs are numpy arrays in the
reference's shapes; ``device=`` variants keep the trajectories on the GPU.
"""
import os

import numpy as np
import torch

from . import _lib


def _dev_f64(a, device):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(device)


def _default_device():
    if not torch.cuda.is_available():
        raise _lib.NonodeError("no CPU path: the simulators run on a ROCm GPU (the CPU restatement is "
                               "oracle/sim.py, test infrastructure)")
    return torch.device("cuda")


class ChargedParticlesSim:
    """synthetic_sim.py:149-296 (charged particles, leapfrog with clamped Coulomb forces)."""

    def __init__(self, n_balls=5, box_size=5., loc_std=1., vel_norm=0.5, interaction_strength=1., noise_var=0.):
        self.n_balls = n_balls
        self.box_size = box_size
        self.loc_std = loc_std * (float(n_balls) / 5.) ** (1 / 3)
        self.vel_norm = vel_norm
        self.interaction_strength = interaction_strength
        self.noise_var = noise_var
        self._charge_types = np.array([-1., 0., 1.])
        self._delta_T = 0.001
        self._max_F = 0.1 / self._delta_T
        self.dim = 3

    def _clamp(self, loc, vel):
        """Elastic walls at +-box_size (synthetic_sim.py:194-218), applied to the initial state."""
        assert np.all(loc < self.box_size * 3) and np.all(loc > -self.box_size * 3)
        over = loc > self.box_size
        loc[over] = 2 * self.box_size - loc[over]
        vel[over] = -np.abs(vel[over])
        under = loc < -self.box_size
        loc[under] = -2 * self.box_size - loc[under]
        vel[under] = np.abs(vel[under])
        return loc, vel

    def _draw(self, T_save, charge_prob):
        n = self.n_balls
        charges = np.random.choice(self._charge_types, size=(n, 1), p=charge_prob)
        loc = np.random.randn(self.dim, n) * self.loc_std
        vel = np.random.randn(self.dim, n)
        vel = vel * self.vel_norm / np.sqrt((vel ** 2).sum(axis=0)).reshape(1, -1)
        loc, vel = self._clamp(loc, vel)
        return charges, loc, vel

    def sample_trajectories(self, S, T=10000, sample_freq=10, charge_prob=(1. / 2, 0, 1. / 2), device=None,
                            as_numpy=True):
        """S consecutive sample_trajectory calls (the reference's RNG order) integrated in ONE launch.
        Returns loc, vel [S, T_save, 3, N], edges [S, N, N], charges [S, N, 1]."""
        assert T % sample_freq == 0
        n, T_save = self.n_balls, T // sample_freq - 1
        q, l0, v0, noise = [], [], [], []
        for _ in range(S):
            c, l, v = self._draw(T_save, list(charge_prob))
            q.append(c); l0.append(l); v0.append(v)
            noise.append((np.random.randn(T_save, self.dim, n), np.random.randn(T_save, self.dim, n)))
        q, l0, v0 = np.stack(q), np.stack(l0), np.stack(v0)
        dev = torch.device(device) if device is not None else _default_device()
        _lib.require_device(torch.empty(0, device=dev))
        ql, ld, vd = _dev_f64(q.reshape(S, n), dev), _dev_f64(l0, dev), _dev_f64(v0, dev)
        loc_d, vel_d = self.integrate(ql, ld, vd, T, sample_freq)
        if self.noise_var:
            loc_d += _dev_f64(np.stack([a for a, _ in noise]), dev) * self.noise_var
            vel_d += _dev_f64(np.stack([b for _, b in noise]), dev) * self.noise_var
        edges = q @ np.transpose(q, (0, 2, 1))
        if not as_numpy:
            return loc_d, vel_d, edges, q
        return loc_d.cpu().numpy(), vel_d.cpu().numpy(), edges, q

    def integrate(self, q, loc0, vel0, T, sample_freq):
        """The time integration of synthetic_sim.py:241-296 for S trajectories already on the GPU:
        q [S, N], loc0 / vel0 [S, 3, N] float64 (after _clamp) -> loc, vel [S, T_save, 3, N], one
        launch."""
        _lib.require_device(q, loc0, vel0)
        S, n = q.shape
        T_save = T // sample_freq - 1
        loc_d = torch.empty(S, T_save, 3, n, dtype=torch.float64, device=q.device)
        vel_d = torch.empty_like(loc_d)
        _lib.check(_lib.lib().nonode_sim_charged(S, n, T, sample_freq, self._delta_T, self._max_F,
                                                 float(self.interaction_strength), _lib.ptr(loc0), _lib.ptr(vel0),
                                                 _lib.ptr(q), _lib.ptr(loc_d), _lib.ptr(vel_d), _lib.stream_of(q)))
        return loc_d, vel_d

    def sample_trajectory(self, T=10000, sample_freq=10, charge_prob=(1. / 2, 0, 1. / 2)):
        """synthetic_sim.py:220-296: loc, vel [T_save, 3, N], edges [N, N], charges [N, 1]."""
        loc, vel, edges, q = self.sample_trajectories(1, T, sample_freq, charge_prob)
        return loc[0], vel[0], edges[0], q[0]


class GravitySim:
    """synthetic_sim.py:299-481 (softened gravity, kick-drift-kick)."""

    def __init__(self, n_balls=100, loc_std=1, vel_norm=0.5, interaction_strength=1, noise_var=0, dt=0.001,
                 softening=0.1):
        self.n_balls = n_balls
        self.loc_std = loc_std
        self.vel_norm = vel_norm
        self.interaction_strength = interaction_strength
        self.noise_var = noise_var
        self.dt = dt
        self.softening = softening
        self.dim = 3

    def sample_trajectory_batch(self, T=10000, sample_freq=10, batch_size=1, device=None, as_numpy=True):
        """synthetic_sim.py:407-456: pos, vel, force [B, T_save, N, 3], mass [B, N, 1]."""
        assert T % sample_freq == 0
        T_save, N = T // sample_freq, self.n_balls
        mass = np.ones((batch_size, N, 1))
        mass += np.random.randn(batch_size, N, 1) * self.loc_std * 0.1
        pos = np.random.randn(batch_size, N, self.dim)
        vel = np.random.randn(batch_size, N, self.dim)
        for b in range(batch_size):
            vel[b] -= np.mean(mass[b] * vel[b], 0) / np.mean(mass[b])
        noise = [np.random.randn(batch_size, T_save, N, self.dim) for _ in range(3)]
        dev = torch.device(device) if device is not None else _default_device()
        _lib.require_device(torch.empty(0, device=dev))
        out = [torch.empty(batch_size, T_save, N, 3, dtype=torch.float64, device=dev) for _ in range(3)]
        pd, vd, md = _dev_f64(pos, dev), _dev_f64(vel, dev), _dev_f64(mass.reshape(batch_size, N), dev)
        _lib.check(_lib.lib().nonode_sim_gravity(batch_size, N, T, sample_freq, float(self.dt),
                                                 float(self.interaction_strength), float(self.softening),
                                                 _lib.ptr(pd), _lib.ptr(vd), _lib.ptr(md), *[_lib.ptr(t) for t in out],
                                                 _lib.stream_of(pd)))
        if self.noise_var:
            for t, z in zip(out, noise):
                t += _dev_f64(z, dev) * self.noise_var
        if not as_numpy:
            return out[0], out[1], out[2], mass
        return out[0].cpu().numpy(), out[1].cpu().numpy(), out[2].cpu().numpy(), mass

    def sample_trajectory(self, T=10000, sample_freq=10):
        """synthetic_sim.py:360-404 (the single-trajectory form; its RNG draws differ from the batch
        form only in shape): pos, vel, force [T_save, N, 3], mass [N, 1]."""
        pos, vel, force, mass = self.sample_trajectory_batch(T, sample_freq, 1)
        return pos[0], vel[0], force[0], mass[0]


def generate_dataset(sim, num_sims, length, sample_freq):
    """generate_dataset.py:62-104: gravity in batches of 50 (sample_trajectory_batch), charged one
    simulation at a time in the reference; here every charged simulation of the split is one
    launch (same RNG order). Returns loc, vel, edges, charges as the reference stacks them."""
    if isinstance(sim, GravitySim):
        parts = [sim.sample_trajectory_batch(T=length, sample_freq=sample_freq, batch_size=50)
                 for _ in range(num_sims // 50 + (num_sims % 50 > 0))]
        return tuple(np.concatenate([p[k] for p in parts], axis=0) for k in range(4))
    return sim.sample_trajectories(num_sims, T=length, sample_freq=sample_freq)


def dataset_suffix(simulation, n_balls, initial_vel=1, suffix=""):
    """File-name suffix of generate_dataset.py:46-59 ('_charged20_initvel1small', ...)."""
    return f"_{simulation}{n_balls}_initvel{initial_vel}{suffix}"


def save_dataset(outdir, split, name_suffix, loc, vel, edges, charges):
    """The four .npy files per split that generate_dataset.py:130-147 writes."""
    os.makedirs(outdir, exist_ok=True)
    for key, arr in (("loc", loc), ("vel", vel), ("edges", edges), ("charges", charges)):
        np.save(os.path.join(outdir, f"{key}_{split}{name_suffix}.npy"), arr)
