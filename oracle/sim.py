"""Oracle restatement of the reference N-body simulators (synthetic_sim.py). Test infrastructure only.

Integrators only: the caller supplies the initial state (drawn as the reference draws it).
Pinned by tests/golden/sim_*.npz, recorded from the reference itself (make_golden_sim.py).
"""
import numpy as np


def charged_forces(loc, q, strength, max_F):
    """ChargedParticlesSim force step (synthetic_sim.py:244-260): loc [3, n], q [n, 1].
    Squared distances as ChargedParticlesSim._l2 (:173-184) computes them, diagonal zeroed, clamp."""
    A = loc.T
    nrm = (A ** 2).sum(axis=1)
    l2 = nrm[:, None] + nrm[None, :] - 2 * A.dot(A.T)
    with np.errstate(invalid="ignore", divide="ignore"):
        fs = strength * (q @ q.T) / np.power(l2, 1.5)
    np.fill_diagonal(fs, 0)
    diff = np.stack([np.subtract.outer(loc[d], loc[d]) for d in range(3)])
    F = (fs[None] * diff).sum(axis=-1)
    return np.clip(F, -max_F, max_F)


def charged_trajectory(loc0, vel0, q, T, freq, dt=0.001, max_F=100.0, strength=1.0):
    """synthetic_sim.py:262-296 from the (clamped) initial state: loc, vel [T/freq - 1, 3, n]."""
    loc, vel = loc0.copy(), vel0.copy()
    T_save = T // freq - 1
    L = np.zeros((T_save, 3, loc.shape[1]))
    V = np.zeros_like(L)
    vel = vel + dt * charged_forces(loc, q, strength, max_F)
    c = 0
    for i in range(1, T):
        loc = loc + dt * vel
        if i % freq == 0:
            L[c], V[c] = loc, vel
            c += 1
        vel = vel + dt * charged_forces(loc, q, strength, max_F)
    return L, V


def gravity_acc(pos, mass, G=1.0, softening=0.1):
    """compute_acceleration_batch (synthetic_sim.py:458-481): pos [B, N, 3], mass [B, N, 1]."""
    d = pos[:, None, :, :] - pos[:, :, None, :]          # d[b, i, j] = x_j - x_i
    r2 = (d ** 2).sum(-1) + softening ** 2
    inv = np.where(r2 > 0, r2 ** -1.5, 0.0)
    return G * np.einsum("bijk,bij,bjl->bik", d, inv, mass)


def gravity_trajectory(pos0, vel0, mass, T, freq, dt=0.001, G=1.0, softening=0.1):
    """sample_trajectory_batch's loop (synthetic_sim.py:435-450): pos, vel, force [B, T/freq, N, 3]."""
    pos, vel = pos0.copy(), vel0.copy()
    B, N, _ = pos.shape
    T_save = T // freq
    P, V, Fo = (np.zeros((B, T_save, N, 3)) for _ in range(3))
    acc = gravity_acc(pos, mass, G, softening)
    for i in range(T):
        if i % freq == 0:
            k = i // freq
            P[:, k], V[:, k], Fo[:, k] = pos, vel, acc * mass
        vel = vel + acc * dt / 2.0
        pos = pos + vel * dt
        acc = gravity_acc(pos, mass, G, softening)
        vel = vel + acc * dt / 2.0
    return P, V, Fo
