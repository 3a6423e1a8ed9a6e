"""GPU parity of the rollout drivers: prepare_inputs, the energy kernel and the
one-call EGNO / SEGNO rollouts (csrc/nonode_rollout.hip) against the reference golden fixtures
and the oracle (oracle/harness.py).

Tolerances: featurisation 1e-6 (same fp32 ops as the reference's torch code); energies 1e-5
relative (the reference sums in float32 numpy, the kernel in float64); positions 1e-5 max-norm
relative.
"""
import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg
from oracle import harness as oh
from tests.conftest import check_rel, load_golden, maxnorm_rel, params_of
from tests.test_gpu_parity import DEV, TOL, _dev, _egno, _segno

pytestmark = pytest.mark.gpu


def test_prepare_inputs_matches_reference_golden():
    fx = load_golden("egno_fwd")
    B, N = int(fx["cfg::B"]), int(fx["cfg::N"])
    edges = pkg.harness.get_edges(B, N, DEV)
    loc, vel, ea, nodes, lm = pkg.harness.prepare_inputs(
        _dev(fx["raw::loc"]), _dev(fx["raw::vel"]), _dev(fx["raw::edge_attr_o"]), edges, N, 1, _dev(fx["raw::charges"]))
    for got, key in [(loc, "in::x"), (vel, "in::v"), (ea, "in::edge_attr"), (nodes, "in::h"),
                     (lm, "in::loc_mean")]:
        np.testing.assert_allclose(got.cpu().numpy(), fx[key], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("F,B,N", [(10, 5, 7), (4, 3, 2), (10, 2, 100)])
def test_prepare_inputs_frame_selection_matches_oracle(F, B, N):
    """rollout_fn restarts each sample from frame timesteps_in[b] - 1 (python index; 0 -> last)."""
    rng = np.random.default_rng(F * 100 + N)
    loc = rng.standard_normal((F, B, N, 3)).astype(np.float32)
    vel = rng.standard_normal((F, B, N, 3)).astype(np.float32)
    q = rng.choice([-1.0, 1.0], size=(B, N, 1)).astype(np.float32)
    row, col = oh.full_edges(B, N)
    eo = (q.reshape(-1, 1)[row] * q.reshape(-1, 1)[col]).astype(np.float32)
    t_in = rng.integers(0, F + 1, size=B)
    x, v, ea, nodes, lm = pkg.harness.prepare_inputs(_dev(loc), _dev(vel), _dev(eo), None, N, 1, _dev(q),
                                                     t_in=_dev(t_in))
    fr = t_in - 1
    ref = oh.prepare_inputs(loc[fr, np.arange(B)], vel[fr, np.arange(B)], eo, row, col, N, q)
    for got, want in zip((x, v, ea, nodes, lm), ref):
        np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-6, atol=1e-6)


def test_energy_charged_matches_oracle_and_skips_coincident_pairs():
    fx = load_golden("egno_fwd")
    ro = load_golden("egno_rollout")
    B = int(fx["cfg::B"])
    frames = ro["out::loc_preds"][:3]                       # [3, BN, 3] frames of the reference rollout
    vel = np.stack([fx["in::v"]] * 3)
    q = fx["raw::charges"]
    e = pkg.harness.conserved_energy("charged", _dev(frames), _dev(vel), _dev(q), B).cpu().numpy()
    for f in range(3):
        want = oh.conserved_energy("charged", frames[f].astype(np.float64), vel[f].astype(np.float64), q, B)
        np.testing.assert_allclose(e[f], want, rtol=1e-5)
    loc = frames[0].copy()
    loc[1] = loc[0]                                          # a coincident pair: 1/0 -> no contribution
    e1 = pkg.harness.conserved_energy("charged", _dev(loc), _dev(vel[0]), _dev(q), B).cpu().numpy()
    want = oh.conserved_energy("charged", loc.astype(np.float64), vel[0].astype(np.float64), q, B)
    assert np.all(np.isfinite(e1))
    np.testing.assert_allclose(e1, want, rtol=1e-5)


@pytest.mark.parametrize("B,N", [(3, 100), (4, 2), (1, 257)])
def test_energy_gravity_matches_oracle(B, N):
    rng = np.random.default_rng(N)
    loc = rng.standard_normal((B * N, 3)).astype(np.float32)
    vel = rng.standard_normal((B * N, 3)).astype(np.float32)
    m = (1 + 0.1 * rng.standard_normal((B, N, 1))).astype(np.float32)
    e = pkg.harness.conserved_energy("gravity", _dev(loc), _dev(vel), _dev(m), B).cpu().numpy()
    want = oh.conserved_energy("gravity", loc.astype(np.float64), vel.astype(np.float64), m.astype(np.float64), B)
    np.testing.assert_allclose(e, want, rtol=1e-5)


def test_egno_rollout_restart_frame_matches_oracle():
    """Two segments restarting from per-sample frames t_in - 1 (not only the last one)."""
    fx = load_golden("egno_fwd")
    p = params_of(fx)
    m = _egno(p)
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    edges = pkg.harness.get_edges(B, N, DEV)
    t_full = np.tile(np.arange(1, 2 * T + 1), (B, 1))
    t_in = np.array([0, 3, 10, 7])[:B]
    preds, en, en_all = pkg.harness.egno_rollout(
        m, _dev(fx["in::h"]), _dev(fx["in::x"]), edges, _dev(fx["in::v"]), _dev(fx["raw::edge_attr_o"]),
        _dev(fx["in::edge_attr"]), _dev(fx["in::loc_mean"]), N, 2, B, charges=_dev(fx["raw::charges"]), num_steps=T,
        timesteps_in=_dev(t_in), timesteps_out=_dev(t_full), energy_dataset="charged")
    row, col = oh.full_edges(B, N)
    ref, ren, ren_all = oh.egno_rollout(p, fx["in::h"], fx["in::x"], row, col, fx["in::v"], fx["raw::edge_attr_o"],
                                        fx["in::edge_attr"], fx["in::loc_mean"], N, 2, B, fx["raw::charges"], T=T,
                                        t_out=t_full, t_in=t_in)
    check_rel("preds[:T]", preds[:T].cpu(), ref[:T], TOL)
    assert maxnorm_rel(preds.cpu(), ref) < 1e-4     # segment 2 starts from a chaotic random-init state
    check_rel("en_all[:T]", en_all[:T].cpu(), ren_all[:T], 1e-5)
    check_rel("en", en.cpu(), ren, 1e-4)   # includes segment 2 (chaotic, see above); measured 1.4e-5
    assert en.shape == (2, B, 1) and en_all.shape == (2 * T, B, 1)


def test_segno_gravity_vardt_rollout_matches_oracle():
    """C5-shaped rollout (gravity, N=100, per-segment substep counts) at B=2, 3 segments."""
    fx = load_golden("segno_gravity")
    p = params_of(fx)
    m = _segno(p)
    B, N = int(fx["cfg::B"]), int(fx["cfg::N"])
    steps = [5, 7, 6]
    ei = pkg.harness.get_edges(B, N, DEV)
    mass = fx["in::mass"]
    preds, en = pkg.harness.segno_rollout(m, _dev(fx["in::his"]), _dev(fx["in::x"]), ei, _dev(fx["in::v"]),
                                          _dev(fx["in::edge_attr"]), 3, num_steps=steps, charges=_dev(mass),
                                          energy_dataset="gravity", batch_size=B)
    row, col = oh.full_edges(B, N)
    ref, ren = oh.segno_rollout(p, fx["in::his"], fx["in::x"], row, col, fx["in::v"], fx["in::edge_attr"], 3, steps,
                                mass, B, dataset="gravity")
    check_rel("preds[0]", preds[0].cpu(), ref[0], TOL)
    check_rel("preds", preds.cpu(), ref, TOL)
    check_rel("en", en.cpu(), ren, TOL)


def test_rollout_rejects_mismatched_features():
    fx = load_golden("egno_fwd")
    m = _egno(params_of(fx))
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    edges = pkg.harness.get_edges(B, N, DEV)
    with pytest.raises(pkg.NonodeError):   # nodes [|v|, q] need the charges
        pkg.harness.egno_rollout(m, _dev(fx["in::h"]), _dev(fx["in::x"]), edges, _dev(fx["in::v"]),
                                 _dev(fx["raw::edge_attr_o"]), _dev(fx["in::edge_attr"]), _dev(fx["in::loc_mean"]), N,
                                 2, B, charges=None, num_steps=T,
                                 timesteps_out=torch.arange(1, 2 * T + 1, device=DEV).repeat(B, 1))


def _c5_substeps(total=50, seed=0):
    """C5's per-segment substep counts: draws in [5, 10) from default_rng(0) until they
    sum to 50, the last one clipped (bench.py c5_substeps)."""
    rng = np.random.default_rng(seed)
    out = []
    while sum(out) < total:
        out.append(int(min(rng.integers(5, 10), total - sum(out))))
    return out


def _gravity_case(B, N, seed):
    """SURVEY §8d gravity generator (synthetic_sim.py:370-378): masses 1 + 0.1 N(0,1), positions and
    velocities N(0,1), centre-of-mass velocity removed; edge_attr [m_i m_j, |x_i - x_j|^2]."""
    g = torch.Generator().manual_seed(seed)
    mass = 1.0 + 0.1 * torch.randn(B, N, 1, generator=g)
    loc = torch.randn(B, N, 3, generator=g)
    vel = torch.randn(B, N, 3, generator=g)
    vel = vel - (mass * vel).sum(1, keepdim=True) / mass.sum(1, keepdim=True)
    return mass.to(DEV), loc.reshape(-1, 3).to(DEV), vel.reshape(-1, 3).to(DEV)


def _gravity_rollout(m, mass, x, v, B, N, steps):
    ei = pkg.harness.get_edges(B, N, DEV)
    mm = mass.reshape(-1, 1)
    ea = torch.cat([mm[ei[0]] * mm[ei[1]], ((x[ei[0]] - x[ei[1]]) ** 2).sum(1, keepdim=True)], 1)
    with torch.no_grad():
        return pkg.harness.segno_rollout(m, v.norm(dim=1, keepdim=True), x, ei, v, ea, len(steps), num_steps=steps,
                                         charges=mass, energy_dataset="gravity", batch_size=B)


def test_segno_c5_full_size_rollout():
    """C5 at its real size: SEGNO gravity, B=256, N=100, the 50-frame multi-horizon rollout (the 8-wave
    layer loop over 256 workgroups). First segment of 16 samples against the float64 torch path
    (oracle/torch_ref.py, scatter mean: the reference's dense mean needs 259 GB here); E(3)
    equivariance and batch independence on the whole batch."""
    from oracle import torch_ref as tr
    B, N = 256, 100
    steps = _c5_substeps()
    assert sum(steps) == 50
    m = _segno(seed=51)
    mass, x, v = _gravity_case(B, N, seed=52)
    preds, en = _gravity_rollout(m, mass, x, v, B, N, steps)
    assert preds.shape == (len(steps), B * N, 3) and torch.isfinite(preds).all() and torch.isfinite(en).all()
    # first segment, 16 samples, against float64
    Bc = 16
    rows = Bc * N
    p = {k: q.detach().cpu().double() for k, q in m.state_dict().items()}
    r, c = tr.full_edges(Bc, N)
    xd, vd, md = x[:rows].cpu().double(), v[:rows].cpu().double(), mass[:Bc].reshape(-1, 1).cpu().double()
    ea = torch.cat([md[r] * md[c], ((xd[r] - xd[c]) ** 2).sum(1, keepdim=True)], 1)
    with torch.no_grad():
        ref = tr.segno_rollout(p, vd.norm(dim=1, keepdim=True), xd, r, c, vd, ea, steps[:1], md, dense_mean=False)
    check_rel("C5 first segment (16 samples)", preds[0, :rows].cpu(), ref[0], TOL)
    # E(3): rotated and translated inputs give rotated and translated positions
    g = torch.Generator().manual_seed(53)
    R, _ = torch.linalg.qr(torch.randn(3, 3, generator=g, dtype=torch.float64))
    R = R.float().to(DEV)
    sh = torch.tensor([0.7, -0.4, 1.1], device=DEV)
    preds2, _ = _gravity_rollout(m, mass, x @ R.T + sh, v @ R.T, B, N, steps)
    check_rel("C5 E(3) first segment", (preds[0] @ R.T + sh).cpu(), preds2[0].cpu(), TOL)
    # later segments: chaotic growth of fp32 rounding differences over 50 substeps
    check_rel("C5 E(3) all segments", (preds @ R.T + sh).cpu(), preds2.cpu(), 1e-3)
    # batch independence: samples 100..102 alone give the same trajectories as inside the batch
    sl = slice(100 * N, 103 * N)
    preds3, _ = _gravity_rollout(m, mass[100:103], x[sl], v[sl], 3, N, steps)
    check_rel("C5 batch independence", preds3.cpu(), preds[:, sl].cpu(), 1e-6)


@pytest.mark.parametrize("B, N, T", [(512, 20, 10), (256, 100, 6), (3, 5, 4)])
def test_segno_substep_fusion_is_bitwise_unfused(monkeypatch, B, N, T):
    """Substep fusion of the SEGNO layer (one whole-graph chunk per workgroup: the node update of step
    t builds step t+1's projection tables and positions in LDS; with room, h and v stay in LDS too) is
    a change of where values live, not of arithmetic: fused + kept (C3), fused only (C5: the kept
    rows do not fit the LDS), and the unfused path (NONODE_NO_FUSE, read per launch) agree bitwise."""
    m = _segno(seed=61)
    g = torch.Generator().manual_seed(62)
    x = torch.randn(B * N, 3, generator=g).to(DEV)
    v = torch.randn(B * N, 3, generator=g).to(DEV)
    q = torch.randn(B * N, 1, generator=g).sign().to(DEV)
    ei = pkg.harness.get_edges(B, N, DEV)
    ea = torch.cat([q[ei[0]] * q[ei[1]], ((x[ei[0]] - x[ei[1]]) ** 2).sum(1, keepdim=True)], 1)
    his = v.norm(dim=1, keepdim=True)

    def run():
        with torch.no_grad():
            out = m(his, x, ei, v, ea, T=T)
        torch.cuda.synchronize()
        return [t.clone() for t in out]   # x, h and v (v leaves LDS only at the last substep in keep mode)

    ref = None
    for env in ({}, {"NONODE_NO_KEEP": "1"}, {"NONODE_NO_FUSE": "1"}):
        for k in ("NONODE_NO_KEEP", "NONODE_NO_FUSE"):
            monkeypatch.delenv(k, raising=False)
        for k, val in env.items():
            monkeypatch.setenv(k, val)
        out = run()
        assert all(torch.isfinite(t).all() for t in out)
        if ref is None:
            ref = out
        else:
            for a, b in zip(ref, out):
                assert torch.equal(a, b), env
