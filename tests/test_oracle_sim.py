"""The simulator oracle (oracle/sim.py) against the reference's own outputs (tests/golden/sim_*.npz,
recorded by make_golden_sim.py from synthetic_sim.py). CPU only."""
import numpy as np
import pytest

from oracle import sim as osim
from tests.conftest import load_golden


def charged_initial_states(seed, n, sims, T, freq, loc_std=1.0, vel_norm=0.5, box=5.0):
    """Replays the reference's RNG draws for `sims` consecutive sample_trajectory calls
    (synthetic_sim.py:224-238, generate_dataset.py:56) and returns the clamped initial states."""
    np.random.seed(seed)
    std = loc_std * (float(n) / 5.) ** (1 / 3)
    out = []
    T_save = T // freq - 1
    for _ in range(sims):
        q = np.random.choice(np.array([-1., 0., 1.]), size=(n, 1), p=[0.5, 0, 0.5])
        loc = np.random.randn(3, n) * std
        vel = np.random.randn(3, n)
        vel = vel * vel_norm / np.sqrt((vel ** 2).sum(axis=0)).reshape(1, -1)
        over = loc > box
        loc[over] = 2 * box - loc[over]
        vel[over] = -np.abs(vel[over])
        under = loc < -box
        loc[under] = -2 * box - loc[under]
        vel[under] = np.abs(vel[under])
        np.random.randn(T_save, 3, n)
        np.random.randn(T_save, 3, n)      # the (zero-variance) observation noise draws
        out.append((q, loc, vel))
    return out


def gravity_initial_state(seed, n, batch, T, freq, loc_std=1.0):
    """synthetic_sim.py:418-431."""
    np.random.seed(seed)
    mass = np.ones((batch, n, 1)) + np.random.randn(batch, n, 1) * loc_std * 0.1
    pos = np.random.randn(batch, n, 3)
    vel = np.random.randn(batch, n, 3)
    for b in range(batch):
        vel[b] -= np.mean(mass[b] * vel[b], 0) / np.mean(mass[b])
    return pos, vel, mass


@pytest.mark.parametrize("name", ["sim_charged", "sim_charged20"])
def test_charged_oracle_matches_reference(name):
    g = load_golden(name)
    n, sims, T, freq = (int(g[k]) for k in ("cfg::n_balls", "cfg::sims", "cfg::T", "cfg::freq"))
    for s, (q, loc0, vel0) in enumerate(charged_initial_states(int(g["cfg::seed"]), n, sims, T, freq)):
        assert np.array_equal(q, g["out::charges"][s]) and np.array_equal(q @ q.T, g["out::edges"][s])
        L, V = osim.charged_trajectory(loc0, vel0, q, T, freq)
        np.testing.assert_allclose(L, g["out::loc"][s], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(V, g["out::vel"][s], rtol=1e-9, atol=1e-9)


def test_gravity_oracle_matches_reference():
    g = load_golden("sim_gravity")
    n, B, T, freq = (int(g[k]) for k in ("cfg::n_balls", "cfg::batch", "cfg::T", "cfg::freq"))
    pos, vel, mass = gravity_initial_state(int(g["cfg::seed"]), n, B, T, freq)
    assert np.array_equal(mass, g["out::mass"])
    P, V, F = osim.gravity_trajectory(pos, vel, mass, T, freq)
    for got, key in ((P, "out::loc"), (V, "out::vel"), (F, "out::force")):
        np.testing.assert_allclose(got, g[key], rtol=1e-9, atol=1e-9)
