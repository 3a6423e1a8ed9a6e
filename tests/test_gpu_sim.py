"""GPU parity of the N-body simulators (csrc/nonode_sim.hip) against the
reference's own trajectories (tests/golden/sim_*.npz) and the oracle (oracle/sim.py).

Tolerance: max-norm relative 1e-7 in float64 on short horizons. Both sides integrate the same
expressions; the force sums run in a different order, and that 1e-16 roundoff grows through close
encounters (2.7e-8 absolute after 3000 charged steps at N=20). Long horizons are chaotic: there the
checks are energy conservation and agreement of the first samples."""
import numpy as np
import pytest

import no_node_comparison_amd as pkg
from oracle import harness as oh
from oracle import sim as osim
from tests.conftest import check_rel, load_golden, maxnorm_rel
from tests.test_oracle_sim import charged_initial_states, gravity_initial_state

pytestmark = pytest.mark.gpu
SIMTOL = 1e-7


@pytest.mark.parametrize("name", ["sim_charged", "sim_charged20"])
def test_charged_sim_reproduces_reference_dataset(name):
    g = load_golden(name)
    n, sims, T, freq = (int(g[k]) for k in ("cfg::n_balls", "cfg::sims", "cfg::T", "cfg::freq"))
    np.random.seed(int(g["cfg::seed"]))
    sim = pkg.sim.ChargedParticlesSim(noise_var=0.0, n_balls=n, vel_norm=0.5)
    loc, vel, edges, q = sim.sample_trajectories(sims, T=T, sample_freq=freq)
    assert np.array_equal(q, g["out::charges"]) and np.array_equal(edges, g["out::edges"])
    check_rel("loc", loc, g["out::loc"], SIMTOL)
    check_rel("vel", vel, g["out::vel"], SIMTOL)


def test_gravity_sim_reproduces_reference_dataset():
    g = load_golden("sim_gravity")
    n, B, T, freq = (int(g[k]) for k in ("cfg::n_balls", "cfg::batch", "cfg::T", "cfg::freq"))
    np.random.seed(int(g["cfg::seed"]))
    sim = pkg.sim.GravitySim(noise_var=0.0, n_balls=n, vel_norm=0.5)
    pos, vel, force, mass = sim.sample_trajectory_batch(T=T, sample_freq=freq, batch_size=B)
    assert np.array_equal(mass, g["out::mass"])
    for got, key in ((pos, "out::loc"), (vel, "out::vel"), (force, "out::force")):
        check_rel("got", got, g[key], SIMTOL)


@pytest.mark.parametrize("n,sims,T,freq", [(2, 2, 500, 50), (64, 2, 400, 100), (200, 1, 300, 100)])
def test_charged_sim_matches_oracle(n, sims, T, freq):
    np.random.seed(n)
    sim = pkg.sim.ChargedParticlesSim(noise_var=0.0, n_balls=n, vel_norm=0.5)
    loc, vel, _, _ = sim.sample_trajectories(sims, T=T, sample_freq=freq)
    for s, (q, l0, v0) in enumerate(charged_initial_states(n, n, sims, T, freq)):
        L, V = osim.charged_trajectory(l0, v0, q, T, freq)
        check_rel("loc[s]", loc[s], L, SIMTOL)
        check_rel("vel[s]", vel[s], V, SIMTOL)


@pytest.mark.parametrize("n,B,T,freq", [(1, 2, 200, 100), (100, 2, 300, 100), (257, 1, 200, 100)])
def test_gravity_sim_matches_oracle(n, B, T, freq):
    np.random.seed(1000 + n)
    sim = pkg.sim.GravitySim(noise_var=0.0, n_balls=n)
    pos, vel, force, mass = sim.sample_trajectory_batch(T=T, sample_freq=freq, batch_size=B)
    p0, v0, m = gravity_initial_state(1000 + n, n, B, T, freq)
    P, V, F = osim.gravity_trajectory(p0, v0, m, T, freq)
    for got, want in ((pos, P), (vel, V), (force, F)):
        check_rel("got", got, want, SIMTOL)


def test_gravity_long_horizon_conserves_energy():
    """5000 kick-drift-kick steps at N=100: the energy of the softened potential is conserved to
    1e-3 relative, and the first samples agree with the oracle to rounding."""
    np.random.seed(7)
    sim = pkg.sim.GravitySim(noise_var=0.0, n_balls=100)
    pos, vel, _, mass = sim.sample_trajectory_batch(T=5000, sample_freq=500, batch_size=4)
    p0, v0, m = gravity_initial_state(7, 100, 4, 5000, 500)
    P, V, _ = osim.gravity_trajectory(p0, v0, m, 1000, 500)
    np.testing.assert_allclose(pos[:, :2], P, rtol=1e-9, atol=1e-9)
    def soft_energy(x, v):   # the energy the softened force conserves
        d = x[:, None] - x[:, :, None]
        r = np.sqrt((d ** 2).sum(-1) + 0.1 ** 2)
        mm = mass * np.transpose(mass, (0, 2, 1))
        pe = -np.triu(mm / r, 1).sum((-1, -2))
        return 0.5 * (mass * v ** 2).sum((-1, -2)) + pe

    e = np.stack([soft_energy(pos[:, k], vel[:, k]) for k in range(pos.shape[1])])
    assert np.all(np.abs(e - e[0]) <= 1e-3 * np.abs(e[0]))
    assert oh.energy_gravity_batch(pos[:, 0], vel[:, 0], mass).shape == (4,)


def test_noise_and_dataset_files(tmp_path):
    """noise_var > 0 adds the reference's observation noise; save_dataset writes generate_dataset.py's
    four files per split with its names."""
    np.random.seed(3)
    sim = pkg.sim.ChargedParticlesSim(noise_var=0.01, n_balls=5)
    loc, vel, edges, q = pkg.sim.generate_dataset(sim, 3, 1000, 100)
    np.random.seed(3)
    ref = charged_initial_states(3, 5, 3, 1000, 100)   # same draws; noise draws are the 2 extra randn
    L, _ = osim.charged_trajectory(ref[0][1], ref[0][2], ref[0][0], 1000, 100)
    assert 1e-4 < np.abs(loc[0] - L).max() < 0.1
    sfx = pkg.sim.dataset_suffix("charged", 5, 1, "small")
    pkg.sim.save_dataset(tmp_path, "train", sfx, loc, vel, edges, q)
    for k in ("loc", "vel", "edges", "charges"):
        assert (tmp_path / f"{k}_train_charged5_initvel1small.npy").exists()
    assert np.load(tmp_path / "loc_train_charged5_initvel1small.npy").shape == (3, 9, 3, 5)
