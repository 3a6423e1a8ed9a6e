"""GPU parity: the gfx950 kernels (through the C ABI) against the golden fixtures recorded from the
reference and against the numpy oracle, plus size-independent properties at the BASELINE sizes.

Tolerance: max-norm relative error <= 1e-5 on positions/velocities/hidden state (SURVEY.md §8d,
BASELINE.json north_star: "within 1e-5 relative fp32").
"""
import math

import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg
from oracle import egno as oe
from oracle import harness as oh
from oracle import segno as osg
from oracle import torch_ref as tr
from tests.conftest import check_rel, load_golden, maxnorm_rel, params_of

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def _dev(a):
    return torch.tensor(np.ascontiguousarray(a)).to(DEV)


def _egno(sd=None, T=10, modes=2, seed=0):
    torch.manual_seed(seed)
    m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=modes,
                 num_timesteps=T, time_emb_dim=32, device=DEV)
    if sd is not None:
        m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.eval()


def _segno(sd=None, seed=0, recurrent=True):
    torch.manual_seed(seed)
    m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=recurrent, device=DEV)
    if sd is not None:
        m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.eval()


def _sd_np(model):
    return {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items()}


# ------------------------------------------------------------------------------------------------
# golden fixtures (reference outputs)
# ------------------------------------------------------------------------------------------------
def test_egno_forward_matches_reference_golden():
    fx = load_golden("egno_fwd")
    m = _egno(params_of(fx))
    with torch.no_grad():
        x, v, h = m(_dev(fx["in::x"]), _dev(fx["in::h"]), [_dev(fx["in::row"]), _dev(fx["in::col"])],
                    _dev(fx["in::edge_attr"]), v=_dev(fx["in::v"]), loc_mean=_dev(fx["in::loc_mean"]),
                    timesteps_out=_dev(fx["in::t_out"]))
    check_rel("x", x.cpu(), fx["out::x"], TOL)
    check_rel("v", v.cpu(), fx["out::v"], TOL)
    check_rel("h", h.cpu(), fx["out::h"], TOL)


def test_egno_building_blocks_match_reference_layers():
    """nonode_egno_tconv and nonode_egnn_layer separately, fed with the reference's captured
    per-layer inputs (EGNO/model/egno.py:99-110)."""
    fx = load_golden("egno_fwd")
    m = _egno(params_of(fx))
    L = pkg.lib()
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    BN = B * N
    blobs, tblobs = m._packed()
    lm = _dev(fx["in::loc_mean"])
    ef = _dev(fx["in::edge_attr"])
    s = pkg._lib.stream_of(lm)
    P = pkg._lib.ptr
    for i in range(4):
        # time conv on the reference's layer-i inputs
        h_in = _dev(fx[f"cap::tconv{i}.in0"]).reshape(T * BN, 64)
        X = fx[f"cap::tconvx{i}.in0"]                           # [T, BN, 3, 2] = (x - lm, v)
        x_in = _dev(X[..., 0].reshape(T * BN, 3) + np.tile(fx["in::loc_mean"], (T, 1)))
        v_in = _dev(X[..., 1].reshape(T * BN, 3))
        ho, xo, vo = torch.empty_like(h_in), torch.empty_like(x_in), torch.empty_like(v_in)
        wx = m.time_conv_x_modules[i].t_conv.weights1.detach().contiguous()
        pkg._lib.check(L.nonode_egno_tconv(BN, T, 2, P(h_in), P(x_in), P(v_in), P(lm), P(tblobs[i]), P(wx), P(ho),
                                           P(xo), P(vo), s))
        Y = fx[f"cap::tconvx{i}.out"]
        check_rel("ho.reshape(T, BN, 64)", ho.cpu().reshape(T, BN, 64), fx[f"cap::tconv{i}.out"], TOL)
        check_rel("xo", xo.cpu(), Y[..., 0].reshape(T * BN, 3) + np.tile(fx["in::loc_mean"], (T, 1)), TOL)
        check_rel("vo", vo.cpu(), Y[..., 1].reshape(T * BN, 3), TOL)
        # EGNN layer on the reference's layer-i inputs
        x_l = _dev(fx[f"cap::layer{i}.in0"])
        h_l = _dev(fx[f"cap::tconv{i}.out"]).reshape(T * BN, 64)
        v_l = _dev(Y[..., 1].reshape(T * BN, 3))
        h2, x2 = torch.empty_like(h_l), torch.empty_like(x_l)
        pkg._lib.check(L.nonode_egnn_layer(0, T * B, N, 2, B, P(h_l), P(x_l), P(v_l), P(ef), P(blobs[i]), 0.0, 1.0,
                                           0, P(h2), P(x2), None, s))
        check_rel("x2", x2.cpu(), fx[f"cap::layer{i}.out0"], TOL)
        check_rel("h2", h2.cpu(), fx[f"cap::layer{i}.out2"], TOL)


def test_egno_rollout_matches_reference_golden():
    fx = load_golden("egno_fwd")
    ro = load_golden("egno_rollout")
    m = _egno(params_of(fx))
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    Lr = int(ro["cfg::traj_len"])
    edges = pkg.harness.get_edges(B, N, DEV)
    t_full = torch.arange(1, T * Lr + 1, device=DEV).repeat(B, 1)
    preds, en, en_all = pkg.harness.egno_rollout(
        m, _dev(fx["in::h"]), _dev(fx["in::x"]), edges, _dev(fx["in::v"]), _dev(fx["raw::edge_attr_o"]),
        _dev(fx["in::edge_attr"]), _dev(fx["in::loc_mean"]), N, Lr, B, charges=_dev(fx["raw::charges"]),
        num_steps=T, timesteps_out=t_full, energy_dataset="charged")
    check_rel("preds[:T]", preds[:T].cpu(), ro["out::loc_preds"][:T], TOL)
    # the second segment restarts from a chaotic random-init state
    # segment 2 starts from segment 1's last frame: chaotic growth of the fp32 differences (SURVEY
    # §4.2 item 5); measured 1.0e-5
    check_rel("both segments", preds.cpu(), ro["out::loc_preds"], 1e-4)
    check_rel("first-segment energies", en_all[:T].cpu(), ro["out::energies_allsteps"][:T], TOL)


def test_segno_gcl_step_and_forward_step_match_reference_golden():
    fx = load_golden("segno_fwd")
    m = _segno(params_of(fx))
    T = int(fx["cfg::T"])
    edges = [_dev(fx["in::row"]), _dev(fx["in::col"])]
    with torch.no_grad():
        x, h, v = m.forward_step(_dev(fx["in::h_emb"]), _dev(fx["in::x"]), edges, _dev(fx["in::v"]),
                                 _dev(fx["in::edge_attr"]), T=T)
        x1, h1, v1 = m.forward_step(_dev(fx["in::h_emb"]), _dev(fx["in::x"]), edges, _dev(fx["in::v"]),
                                    _dev(fx["in::edge_attr"]), T=1)
    check_rel("x", x.cpu(), fx["step::x"], TOL)
    check_rel("v", v.cpu(), fx["step::v"], TOL)
    check_rel("h", h.cpu(), fx["step::h"], TOL)
    # one substep with n_layers = T = 1 vs the oracle's single GCL step (gcl.py:111-119)
    p = params_of(fx)
    hr, xr, vr = osg.gcl_forward(p, fx["in::h_emb"], fx["in::row"], fx["in::col"], fx["in::x"], fx["in::v"],
                                 fx["in::edge_attr"], n_layers=1)
    assert maxnorm_rel(x1.cpu(), xr) < TOL and maxnorm_rel(h1.cpu(), hr) < TOL and maxnorm_rel(v1.cpu(), vr) < TOL


def test_segno_forward_integrator_and_bug_compat():
    fx = load_golden("segno_fwd")
    m = _segno(params_of(fx))
    T = int(fx["cfg::T"])
    args = (_dev(fx["in::his"]), _dev(fx["in::x"]), [_dev(fx["in::row"]), _dev(fx["in::col"])], _dev(fx["in::v"]),
            _dev(fx["in::edge_attr"]))
    with torch.no_grad():
        x, h, v = m(*args, T=T)
    assert maxnorm_rel(x.cpu(), fx["step::x"]) < TOL   # integrator result (forward_step semantics)
    m.bug_compat = True
    with torch.no_grad():
        x, h, v = m(*args, T=T)
    assert np.array_equal(x.cpu().numpy(), fx["fwd::x"]) and np.array_equal(v.cpu().numpy(), fx["fwd::v"])
    check_rel("h", h.cpu(), fx["fwd::h"], 1e-6)


def test_segno_rollout_matches_reference_golden():
    fx = load_golden("segno_fwd")
    ro = load_golden("segno_rollout")
    m = _segno(params_of(fx))
    B = int(fx["cfg::B"])
    ei = torch.stack([_dev(fx["in::row"]), _dev(fx["in::col"])])
    preds, en = pkg.harness.segno_rollout(m, _dev(fx["in::his"]), _dev(fx["in::x"]), ei, _dev(fx["in::v"]),
                                          _dev(fx["in::edge_attr"]), 2, num_steps=[int(s) for s in ro["cfg::num_steps"]],
                                          charges=_dev(fx["raw::charges"]), energy_dataset="charged", batch_size=B)
    check_rel("preds", preds.cpu(), ro["out::loc_preds"], TOL)
    check_rel("en", en.cpu(), ro["out::energies"], TOL)


def test_segno_gravity_n100_matches_reference_golden():
    fx = load_golden("segno_gravity")
    m = _segno(params_of(fx))
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    edges = pkg.harness.get_edges(B, N, DEV)
    with torch.no_grad():
        hh = torch.nn.functional.linear(_dev(fx["in::his"]), m.embedding.weight, m.embedding.bias)
        x, h, v = m.forward_step(hh, _dev(fx["in::x"]), edges, _dev(fx["in::v"]), _dev(fx["in::edge_attr"]), T=T)
    check_rel("x", x.cpu(), fx["step::x"], TOL)
    check_rel("v", v.cpu(), fx["step::v"], TOL)
    check_rel("h", h.cpu(), fx["step::h"], TOL)


# ------------------------------------------------------------------------------------------------
# oracle parity on other shapes (seeded synthetic inputs, SURVEY §8d generator)
# ------------------------------------------------------------------------------------------------
def synthetic_charged(B, N, seed=0):
    g = torch.Generator().manual_seed(seed)
    sigma = (N / 5.0) ** (1.0 / 3.0)
    loc = torch.randn(B, N, 3, generator=g) * sigma
    vel = torch.randn(B, N, 3, generator=g)
    vel = vel / vel.norm(dim=-1, keepdim=True) * 0.5
    q = (torch.randint(0, 2, (B, N, 1), generator=g) * 2 - 1).float()
    return loc, vel, q


def _egno_case(B, N, T=10, seed=0):
    loc, vel, q = synthetic_charged(B, N, seed)
    r, c = oh.full_edges(B, N)
    qq = q.reshape(-1, 1).numpy()
    eao = (qq[r] * qq[c]).astype(np.float32)
    x, v, ea, nodes, lm = oh.prepare_inputs(loc.numpy(), vel.numpy(), eao, r, c, N, q.numpy())
    t_out = np.tile(np.arange(1, T + 1), (B, 1))
    return dict(x=x, h=nodes, row=r, col=c, edge_fea=ea, v=v, loc_mean=lm, t_out=t_out)


@pytest.mark.parametrize("B,N,T", [(1, 2, 10), (3, 5, 10), (7, 20, 10), (2, 20, 5), (5, 13, 4), (2, 40, 10),
                                   (1, 100, 2), (3, 7, 16), (2, 9, 13), (4, 6, 11)])
def test_egno_matches_oracle_across_shapes(B, N, T):
    m = _egno(T=T, seed=B * 100 + N)
    case = _egno_case(B, N, T, seed=N)
    p = _sd_np(m)
    xr, vr, hr = oe.egno_forward(p, **{k: (v.astype(np.float64) if k not in ("row", "col", "t_out") else v)
                                       for k, v in case.items()}, T=T)
    with torch.no_grad():
        x, v, h = m(_dev(case["x"]), _dev(case["h"]), [_dev(case["row"]), _dev(case["col"])], _dev(case["edge_fea"]),
                    v=_dev(case["v"]), loc_mean=_dev(case["loc_mean"]), timesteps_out=_dev(case["t_out"]))
    check_rel("x", x.cpu(), xr, TOL)
    check_rel("v", v.cpu(), vr, TOL)
    check_rel("h", h.cpu(), hr, TOL)


@pytest.mark.gpu
@pytest.mark.parametrize("T,modes", [(16, 9), (12, 4), (10, 5), (7, 4)])
def test_egno_mode_and_frame_bounds_match_oracle(T, modes):
    """Every tconv_kernel build (mode bound 2 / 4 / 9 x frame bound 10 / 16) against the oracle."""
    B, N = 3, 6
    m = _egno(T=T, modes=modes, seed=T * 10 + modes)
    case = _egno_case(B, N, T, seed=modes)
    p = _sd_np(m)
    xr, vr, hr = oe.egno_forward(p, **{k: (v.astype(np.float64) if k not in ("row", "col", "t_out") else v)
                                       for k, v in case.items()}, T=T)
    with torch.no_grad():
        x, v, h = m(_dev(case["x"]), _dev(case["h"]), [_dev(case["row"]), _dev(case["col"])], _dev(case["edge_fea"]),
                    v=_dev(case["v"]), loc_mean=_dev(case["loc_mean"]), timesteps_out=_dev(case["t_out"]))
    check_rel("x", x.cpu(), xr, TOL)
    check_rel("v", v.cpu(), vr, TOL)
    check_rel("h", h.cpu(), hr, TOL)


@pytest.mark.parametrize("B,N,scale", [(2, 20, 3e4), (1, 70, 1e4)])
def test_egno_guard_path_matches_oracle(B, N, scale):
    """Edge features scaled so the edge-feature part of every layer's first Linear reaches ~2e5: the
    SiLU(pre) activations leave the fp16 range, so units take the column-scaled guard recompute, in
    the paired 4-wave loop (N = 20) and in the 8-wave single-unit loop (N = 70, N >= 64). Outputs
    grow to ~1e13 / ~1e17 and stay inside the f32 range."""
    T = 10
    m = _egno(T=T, seed=B * 7 + N)
    case = _egno_case(B, N, T, seed=N + 1)
    case["edge_fea"] = (case["edge_fea"] * scale).astype(np.float32)
    p = _sd_np(m)
    # the guard really triggers: a first-layer pre-activation exceeds the fp16 range
    w1 = p["layers.0.edge_message_net.scalar_net.mlp.0.weight"][:, -2:]
    assert float(np.abs(case["edge_fea"].astype(np.float64) @ w1.T).max()) > 2 * 65504.0
    xr, vr, hr = oe.egno_forward(p, **{k: (v.astype(np.float64) if k not in ("row", "col", "t_out") else v)
                                       for k, v in case.items()}, T=T)
    assert np.isfinite(xr).all() and np.isfinite(hr).all()
    # inputs this large are ill-conditioned in fp32 itself: the reference's own ops in fp32
    # (oracle/torch_ref.py) are up to ~1.4e-5 from float64 at N = 70; the bar is 1e-5 or twice that
    # fp32 floor, whichever is larger
    p32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in p.items()}
    t = lambda a: torch.tensor(np.ascontiguousarray(a))  # noqa: E731
    with torch.no_grad():
        f32 = tr.egno_forward(p32, t(case["x"]).float(), t(case["h"]).float(), t(case["row"]).long(),
                              t(case["col"]).long(), t(case["edge_fea"]).float(), t(case["v"]).float(),
                              t(case["loc_mean"]).float(), t(case["t_out"]).float(), T=T)
        x, v, h = m(_dev(case["x"]), _dev(case["h"]), [_dev(case["row"]), _dev(case["col"])], _dev(case["edge_fea"]),
                    v=_dev(case["v"]), loc_mean=_dev(case["loc_mean"]), timesteps_out=_dev(case["t_out"]))
    for name, out, f, ref in (("x", x, f32[0], xr), ("v", v, f32[1], vr), ("h", h, f32[2], hr)):
        check_rel(f"guard N={N} {name}", out.cpu(), ref, max(TOL, 2 * maxnorm_rel(f.numpy(), ref)))


@pytest.mark.parametrize("B,N,scale", [(3, 20, 300.0), (1, 64, 60.0), (1, 70, 60.0)])
def test_segno_guard_path_matches_oracle(B, N, scale):
    """SEGNO with scaled positions (|r|^2 also enters as an edge feature): guard recompute in both
    loops against the oracle."""
    T = 4
    m = _segno(seed=N + 3)
    loc, vel, q = synthetic_charged(B, N, seed=N)
    r, c = oh.full_edges(B, N)
    x = loc.reshape(-1, 3).numpy().astype(np.float64) * scale
    v = vel.reshape(-1, 3).numpy().astype(np.float64)
    qq = q.reshape(-1, 1).numpy()
    ea = np.concatenate([qq[r] * qq[c], ((x[r] - x[c]) ** 2).sum(1, keepdims=True)], 1)
    assert float(ea[:, 1].max()) > 65504.0
    his = np.sqrt((v ** 2).sum(1, keepdims=True))
    p = _sd_np(m)
    xr, hr, vr = osg.forward(p, his, x, r, c, v, ea, T=T, bug_compat=False)
    assert np.isfinite(xr).all() and np.isfinite(hr).all()
    p32 = {k: torch.tensor(w, dtype=torch.float32) for k, w in p.items()}
    f = lambda a: torch.tensor(np.ascontiguousarray(a)).float()  # noqa: E731
    with torch.no_grad():
        f32 = tr.segno_forward_step(p32, f(his), f(x), torch.tensor(r).long(), torch.tensor(c).long(), f(v), f(ea), T=T)
        xo, ho, vo = m(_dev(his.astype(np.float32)), _dev(x.astype(np.float32)), [_dev(r), _dev(c)],
                       _dev(v.astype(np.float32)), _dev(ea.astype(np.float32)), T=T)
    # bar: 1e-5 or twice the reference ops' own fp32 error on these inputs, whichever is larger
    for name, out, g, ref in (("xo", xo, f32[0], xr), ("vo", vo, f32[2], vr), ("ho", ho, f32[1], hr)):
        check_rel(f"segno guard N={N} {name}", out.cpu(), ref, max(TOL, 2 * maxnorm_rel(g.numpy(), ref)))


@pytest.mark.parametrize("B,N,T", [(1, 2, 3), (4, 5, 10), (9, 20, 10), (2, 60, 7), (1, 150, 2)])
def test_segno_matches_oracle_across_shapes(B, N, T):
    m = _segno(seed=N + B)
    loc, vel, q = synthetic_charged(B, N, seed=B)
    r, c = oh.full_edges(B, N)
    x = loc.reshape(-1, 3).numpy().astype(np.float64)
    v = vel.reshape(-1, 3).numpy().astype(np.float64)
    qq = q.reshape(-1, 1).numpy()
    ea = np.concatenate([qq[r] * qq[c], ((x[r] - x[c]) ** 2).sum(1, keepdims=True)], 1)
    his = np.sqrt((v ** 2).sum(1, keepdims=True))
    p = _sd_np(m)
    xr, hr, vr = osg.forward(p, his, x, r, c, v, ea, T=T, bug_compat=False)
    with torch.no_grad():
        xo, ho, vo = m(_dev(his.astype(np.float32)), _dev(x.astype(np.float32)), [_dev(r), _dev(c)],
                       _dev(v.astype(np.float32)), _dev(ea.astype(np.float32)), T=T)
    check_rel("xo", xo.cpu(), xr, TOL)
    check_rel("vo", vo.cpu(), vr, TOL)
    check_rel("ho", ho.cpu(), hr, TOL)


# ------------------------------------------------------------------------------------------------
# size-independent properties at the BASELINE sizes
# ------------------------------------------------------------------------------------------------
def _rotation(seed):
    g = torch.Generator().manual_seed(seed)
    q, _ = torch.linalg.qr(torch.randn(3, 3, generator=g, dtype=torch.float64))
    return q.float()


def _egno_full(B, N=20, T=10, seed=0):
    loc, vel, q = synthetic_charged(B, N, seed)
    loc, vel, q = loc.to(DEV), vel.to(DEV), q.to(DEV)
    edges = pkg.harness.get_edges(B, N, DEV)
    qq = q.reshape(-1, 1)
    eao = qq[edges[0]] * qq[edges[1]]
    x, v, ea, nodes, lm = pkg.harness.prepare_inputs(loc, vel, eao, edges, N, 1, q)
    t = torch.arange(1, T + 1, device=DEV).repeat(B, 1)
    return x, nodes, edges, ea, v, lm, t, (loc, vel, q, eao)


def test_egno_c2_e3_equivariance_and_batch_independence():
    """C2 size (B=512, N=20, T=10): rotating/translating the inputs rotates/translates x and v and
    leaves h unchanged; each sample's output is independent of the rest of the batch."""
    B, N, T = 512, 20, 10
    m = _egno(T=T, seed=3)
    x, nodes, edges, ea, v, lm, t, raw = _egno_full(B, N, T, seed=5)
    with torch.no_grad():
        xo, vo, ho = m(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_out=t)
        R = _rotation(1).to(DEV)
        sh = torch.tensor([0.3, -1.2, 2.0], device=DEV)
        xo2, vo2, ho2 = m(x @ R.T + sh, nodes, edges, ea, v=v @ R.T, loc_mean=lm @ R.T + sh, timesteps_out=t)
    assert torch.isfinite(xo).all() and torch.isfinite(ho).all()
    check_rel("(xo @ R.T + sh)", (xo @ R.T + sh).cpu(), xo2.cpu(), TOL)
    check_rel("(vo @ R.T)", (vo @ R.T).cpu(), vo2.cpu(), TOL)
    check_rel("ho", ho.cpu(), ho2.cpu(), TOL)
    # batch independence: samples 17..19 run alone
    loc, vel, q, eao = raw
    sl = slice(17, 20)
    e3 = pkg.harness.get_edges(3, N, DEV)
    qq = q[sl].reshape(-1, 1)
    x3, v3, ea3, n3, lm3 = pkg.harness.prepare_inputs(loc[sl], vel[sl], qq[e3[0]] * qq[e3[1]], e3, N, 1, q[sl])
    with torch.no_grad():
        xs, vs, hs = m(x3, n3, e3, ea3, v=v3, loc_mean=lm3, timesteps_out=t[:3])
    big = xo.view(T, B, N, 3)[:, sl].reshape(-1, 3)
    check_rel("xs", xs.cpu(), big.cpu(), 1e-5)


def test_egno_c2_whole_batch_matches_f64_reference():
    """The whole C2 batch (B=512, N=20, T=10) against oracle/torch_ref.py — the reference's torch
    operators, op by op — in float64 (pinned to the reference's fixtures by tests/test_torch_ref.py)."""
    from oracle import torch_ref as tr
    B, N, T = 512, 20, 10
    m = _egno(T=T, seed=11)
    x, nodes, edges, ea, v, lm, t, raw = _egno_full(B, N, T, seed=6)
    with torch.no_grad():
        xo, vo, ho = m(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_out=t)
    p = {k: v_.detach().cpu().double() for k, v_ in m.state_dict().items()}
    r, c = tr.full_edges(B, N)
    d = lambda a: a.detach().cpu().double()  # noqa: E731
    with torch.no_grad():
        xr, vr, hr = tr.egno_forward(p, d(x), d(nodes), r, c, d(ea), d(v), d(lm), t.cpu(), T=T)
    check_rel("C2 x (512 samples)", xo, xr, TOL)
    check_rel("C2 v (512 samples)", vo, vr, TOL)
    check_rel("C2 h (512 samples)", ho, hr, TOL)


def test_segno_c3_whole_batch_matches_f64_reference():
    """The whole C3 batch (B=512, N=20, 10 substeps) against the f64 torch restatement (scatter mean:
    the same values as gcl.py:16-23's dense mean, tests/test_torch_ref.py)."""
    from oracle import torch_ref as tr
    B, N, T = 512, 20, 10
    m = _segno(seed=7)
    loc, vel, q = synthetic_charged(B, N, seed=12)
    x = loc.reshape(-1, 3).to(DEV)
    v = vel.reshape(-1, 3).to(DEV)
    edges = pkg.harness.get_edges(B, N, DEV)
    qq = q.reshape(-1, 1).to(DEV)
    ea = torch.cat([qq[edges[0]] * qq[edges[1]], ((x[edges[0]] - x[edges[1]]) ** 2).sum(1, keepdim=True)], 1)
    his = v.norm(dim=1, keepdim=True)
    with torch.no_grad():
        xo, ho, vo = m(his, x, edges, v, ea, T=T)
    p = {k: v_.detach().cpu().double() for k, v_ in m.state_dict().items()}
    r, c = tr.full_edges(B, N)
    d = lambda a: a.detach().cpu().double()  # noqa: E731
    with torch.no_grad():
        xr, hr, vr = tr.segno_forward_step(p, d(his), d(x), r, c, d(v), d(ea), T=T, dense_mean=False)
    check_rel("C3 x (512 samples)", xo, xr, TOL)
    check_rel("C3 v (512 samples)", vo, vr, TOL)
    check_rel("C3 h (512 samples)", ho, hr, TOL)


def test_segno_c3_equivariance_and_permutation():
    B, N, T = 512, 20, 10
    m = _segno(seed=2)
    loc, vel, q = synthetic_charged(B, N, seed=9)
    x = loc.reshape(-1, 3).to(DEV)
    v = vel.reshape(-1, 3).to(DEV)
    edges = pkg.harness.get_edges(B, N, DEV)
    qq = q.reshape(-1, 1).to(DEV)
    ea = torch.cat([qq[edges[0]] * qq[edges[1]], ((x[edges[0]] - x[edges[1]]) ** 2).sum(1, keepdim=True)], 1)
    his = v.norm(dim=1, keepdim=True)
    with torch.no_grad():
        xo, ho, vo = m(his, x, edges, v, ea, T=T)
        R = _rotation(4).to(DEV)
        xo2, ho2, vo2 = m(his, x @ R.T + 1.5, edges, v @ R.T, ea, T=T)
    assert torch.isfinite(xo).all()
    check_rel("(xo @ R.T + 1.5)", (xo @ R.T + 1.5).cpu(), xo2.cpu(), TOL)
    check_rel("(vo @ R.T)", (vo @ R.T).cpu(), vo2.cpu(), TOL)
    check_rel("ho", ho.cpu(), ho2.cpu(), TOL)


def test_rejects_bad_inputs_loudly():
    fx = load_golden("egno_fwd")
    m = _egno(params_of(fx))
    args = [_dev(fx["in::x"]), _dev(fx["in::h"]), [_dev(fx["in::col"]), _dev(fx["in::row"])],
            _dev(fx["in::edge_attr"])]
    # swapped receiver / sender lists: checked on the device without blocking (graph.py); the call's
    # outputs are NaN and the error is raised by the next boundary call or sync_checks()
    with torch.no_grad():
        out = m(*args, v=_dev(fx["in::v"]), loc_mean=_dev(fx["in::loc_mean"]), timesteps_out=_dev(fx["in::t_out"]))
    assert all(torch.isnan(t).all() for t in out)
    with pytest.raises(ValueError, match="fully connected"):
        pkg.graph.sync_checks()
    with pytest.raises(ValueError):
        with torch.no_grad():
            m(*args[:2], [_dev(fx["in::row"]), _dev(fx["in::col"])], args[3], v=None,
              loc_mean=_dev(fx["in::loc_mean"]), timesteps_out=_dev(fx["in::t_out"]))


def test_native_library_is_what_ran():
    """The forward above went through libnonode.so (no fallback exists to take instead)."""
    import os
    maps = open(f"/proc/{os.getpid()}/maps").read()
    assert "libnonode.so" in maps
    assert math.isfinite(1.0)


def test_egno_five_modes_matches_reference_golden():
    """num_modes=5, num_timesteps=8 (five spectral modes with the Nyquist bin: the MM=9 TimeConv
    instantiation) against the reference's own forward; seed-0 weights as the reference's."""
    fx = load_golden("egno_m5")
    T, modes = int(fx["cfg::T"]), int(fx["cfg::modes"])
    m = _egno(T=T, modes=modes, seed=0)
    edges = [_dev(fx["in::row"]), _dev(fx["in::col"])]
    with torch.no_grad():
        x, v, h = m(_dev(fx["in::x"]), _dev(fx["in::h"]), edges, _dev(fx["in::edge_attr"]), v=_dev(fx["in::v"]),
                    loc_mean=_dev(fx["in::loc_mean"]), timesteps_out=_dev(fx["in::t_out"]))
    check_rel("x", x.cpu(), fx["out::x"], TOL)
    check_rel("v", v.cpu(), fx["out::v"], TOL)
    check_rel("h", h.cpu(), fx["out::h"], TOL)


def test_egno_multi_input_matches_reference_golden():
    """num_inputs=3 (nonode_egno_forward_frames: per-frame inputs, input-time embedding) against the
    reference's own forward; seed-0 weights as the reference's."""
    fx = load_golden("egno_multi")
    T, I = int(fx["cfg::T"]), int(fx["cfg::I"])
    torch.manual_seed(0)
    m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                 num_timesteps=T, time_emb_dim=32, num_inputs=I, device=DEV).eval()
    edges = [_dev(fx["in::row"]), _dev(fx["in::col"])]
    with torch.no_grad():
        x, v, h = m(_dev(fx["in::x"]), _dev(fx["in::h"]), edges, _dev(fx["in::edge_attr"]), v=_dev(fx["in::v"]),
                    loc_mean=_dev(fx["in::loc_mean"]), timesteps_in=_dev(fx["in::t_in"]),
                    timesteps_out=_dev(fx["in::t_out"]))
    check_rel("x", x.cpu(), fx["out::x"], TOL)
    check_rel("v", v.cpu(), fx["out::v"], TOL)
    check_rel("h", h.cpu(), fx["out::h"], TOL)


def test_segno_multi_input_attn_matches_reference_golden():
    """SEGNO num_inputs=3, multiple_agg='attn': the HIP integrator per segment with the attention
    fold between, against the reference (bug_compat) and its discarded last forward_step."""
    fx = load_golden("segno_multi")
    T = int(fx["cfg::T"])
    edges = [_dev(fx["in::row"]), _dev(fx["in::col"])]
    for bug, pre in ((True, "fwd"), (False, "last")):
        torch.manual_seed(0)
        m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True, multiple_agg="attn",
                      bug_compat=bug, device=DEV).eval()
        m.load_state_dict({k: torch.tensor(v) for k, v in params_of(fx).items()})
        with torch.no_grad():
            x, h, v = m(_dev(fx["in::his"]), _dev(fx["in::x"]), edges, _dev(fx["in::v"]), _dev(fx["in::edge_attr"]),
                        T=T, in_steps=_dev(fx["in::in_steps"]))
        check_rel("x", x.cpu(), fx[pre + "::x"], TOL)
        check_rel("h", h.cpu(), fx[pre + "::h"], TOL)
        check_rel("v", v.cpu(), fx[pre + "::v"], TOL)


def test_egno_multi_input_rollout_matches_reference_golden():
    """rollout_fn with num_inputs=3 (harness.egno_rollout -> egno_rollout_multi): each segment's last
    frames become the next inputs through the multi-input prepare_inputs, as the reference does."""
    fx = load_golden("egno_multi")
    ro = load_golden("egno_multi_rollout")
    B, N, T, I = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"]), int(fx["cfg::I"])
    Lr = int(ro["cfg::traj_len"])
    torch.manual_seed(0)
    m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                 num_timesteps=T, time_emb_dim=32, num_inputs=I, device=DEV).eval()
    edges = pkg.harness.get_edges(B, N, DEV)
    preds, en, en_all = pkg.harness.egno_rollout(
        m, _dev(fx["in::h"]), _dev(fx["in::x"]), edges, _dev(fx["in::v"]), _dev(ro["raw::edge_attr_o"]),
        _dev(fx["in::edge_attr"]), _dev(fx["in::loc_mean"]), N, Lr, B, charges=_dev(ro["raw::charges"]),
        num_steps=T, timesteps_in=_dev(fx["in::t_in"]), timesteps_out=_dev(ro["in::t_out"]), energy_dataset="charged")
    check_rel("preds[:T]", preds[:T].cpu(), ro["out::loc_preds"][:T], TOL)
    check_rel("preds", preds.cpu(), ro["out::loc_preds"], TOL)
    check_rel("en_all", en_all.cpu(), ro["out::energies_all"], TOL)
    check_rel("en", en.cpu(), ro["out::energies"], TOL)


def test_segno_multi_input_rollout_matches_reference_golden():
    """rollout_fn with num_prev=3 (train_nbody.py:200-236) through the integrator, 2 segments of
    10 and 5 substeps, with energies."""
    fx = load_golden("segno_multi")
    ro = load_golden("segno_multi_rollout")
    T = int(fx["cfg::T"])
    m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True, multiple_agg="attn",
                  device=DEV).eval()
    m.load_state_dict({k: torch.tensor(v) for k, v in params_of(fx).items()})
    edges = [_dev(fx["in::row"]), _dev(fx["in::col"])]
    preds, en = pkg.harness.segno_rollout(m, _dev(fx["in::his"]), _dev(fx["in::x"]), edges, _dev(fx["in::v"]),
                                          _dev(fx["in::edge_attr"]), 2, num_steps=[T, T // 2],
                                          charges=_dev(ro["raw::charges"]), energy_dataset="charged",
                                          in_steps=_dev(fx["in::in_steps"]))
    check_rel("preds[0]", preds[0].cpu(), ro["out::loc_preds"][0], TOL)
    check_rel("preds", preds.cpu(), ro["out::loc_preds"], TOL)
    check_rel("en", en.cpu(), ro["out::energies"], TOL)


@pytest.mark.parametrize("B", [64, 128, 256])
def test_egno_small_batch_chunking_matches_f64_and_fill_rule(monkeypatch, B):
    """The strong-scaling shards of C2 (B = 512 / 8, 4, 2 per GPU): inference forwards with few graphs
    per CU take the critical-path chunk size (csrc/nonode.hip launch_layer; B = 64: 3-graph chunks on
    214 workgroups instead of 2-graph chunks in two rounds). Same arithmetic per receiver, other sum
    order: against the f64 torch path and the fill rule's result (NONODE_FILL_CG=1)."""
    from oracle import torch_ref as tr
    N, T = 20, 10
    m = _egno(T=T, seed=B + 1)
    x, nodes, edges, ea, v, lm, t, _ = _egno_full(B, N, T, seed=B + 2)
    with torch.no_grad():
        out = [o.clone() for o in m(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_out=t)]
        monkeypatch.setenv("NONODE_FILL_CG", "1")
        fill = m(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_out=t)
    for name, a, b in zip("xvh", out, fill):
        check_rel(f"B={B} {name} critical-path vs fill chunks", a, b, 1e-6)
    if B == 64:
        p = {k: v_.detach().cpu().double() for k, v_ in m.state_dict().items()}
        r, c = tr.full_edges(B, N)
        d = lambda a: a.detach().cpu().double()  # noqa: E731
        with torch.no_grad():
            ref = tr.egno_forward(p, d(x), d(nodes), r, c, d(ea), d(v), d(lm), t.cpu(), T=T)
        for name, a, b in zip("xvh", out, ref):
            check_rel(f"B=64 {name} vs f64", a, b, TOL)
