"""Generate tests/golden/sim_charged.npz and sim_gravity.npz by running the REFERENCE simulators.

Test infrastructure only (build container; /root/reference never reaches the GPU box). Records
the outputs of synthetic_sim.py's ChargedParticlesSim.sample_trajectory (synthetic_sim.py:220-296)
and GravitySim.sample_trajectory_batch (synthetic_sim.py:407-481) exactly as generate_dataset.py
drives them (generate_dataset.py:45-104: np.random.seed(seed), noise_var=0, vel_norm=0.5), at
small sizes and short horizons. The fixtures are data; no reference source is copied. Re-run:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_sim.py
"""
import contextlib
import io
import os
import sys

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402

sys.path.insert(0, REF)
import synthetic_sim  # noqa: E402


def charged(seed=43, n_balls=5, sims=3, T=2000, freq=100):
    np.random.seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):   # the constructor prints loc_std
        sim = synthetic_sim.ChargedParticlesSim(noise_var=0.0, n_balls=n_balls, vel_norm=0.5)
    out = {"loc": [], "vel": [], "edges": [], "charges": []}
    for _ in range(sims):
        loc, vel, edges, q = sim.sample_trajectory(T=T, sample_freq=freq)
        for k, v in zip(("loc", "vel", "edges", "charges"), (loc, vel, edges, q)):
            out[k].append(v)
    d = {f"out::{k}": np.stack(v) for k, v in out.items()}
    d.update({"cfg::seed": seed, "cfg::n_balls": n_balls, "cfg::sims": sims, "cfg::T": T, "cfg::freq": freq})
    return d


def gravity(seed=43, n_balls=20, batch=3, T=1000, freq=100):
    np.random.seed(seed)
    sim = synthetic_sim.GravitySim(noise_var=0.0, n_balls=n_balls, vel_norm=0.5)
    pos, vel, force, mass = sim.sample_trajectory_batch(T=T, sample_freq=freq, batch_size=batch)
    return {"out::loc": pos, "out::vel": vel, "out::force": force, "out::mass": mass, "cfg::seed": seed,
            "cfg::n_balls": n_balls, "cfg::batch": batch, "cfg::T": T, "cfg::freq": freq}


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "sim_charged.npz"), **charged())
    np.savez_compressed(os.path.join(HERE, "sim_charged20.npz"), **charged(n_balls=20, sims=2, T=3000))
    np.savez_compressed(os.path.join(HERE, "sim_gravity.npz"), **gravity())
    print("wrote sim_charged.npz, sim_charged20.npz, sim_gravity.npz")
