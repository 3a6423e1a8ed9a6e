"""Pin the numpy oracle to fixtures recorded from the reference itself (CPU only)."""
import numpy as np
import pytest

from oracle import egno as oe
from oracle import harness as oh
from oracle import segno as osg
from tests.conftest import load_golden, maxnorm_rel, params_of

TOL32 = 1e-5   # SURVEY §8d parity bound (max-norm relative, fp32)


@pytest.fixture(scope="module")
def egno_fx():
    return load_golden("egno_fwd")


@pytest.fixture(scope="module")
def segno_fx():
    return load_golden("segno_fwd")


def _egno_inputs(fx, dtype=np.float32):
    c = lambda k: fx[k].astype(dtype)  # noqa: E731
    return dict(x=c("in::x"), h=c("in::h"), row=fx["in::row"], col=fx["in::col"],
                edge_fea=c("in::edge_attr"), v=c("in::v"), loc_mean=c("in::loc_mean"),
                t_out=fx["in::t_out"])


def test_timestep_embedding(egno_fx):
    got = oe.timestep_embedding(egno_fx["in::t_out"], 32)
    assert maxnorm_rel(got, egno_fx["out::temb"]) < 1e-6


def test_prepare_inputs(egno_fx):
    fx = egno_fx
    B, N = int(fx["cfg::B"]), int(fx["cfg::N"])
    row, col = oh.full_edges(B, N)
    assert np.array_equal(row, fx["in::row"]) and np.array_equal(col, fx["in::col"])
    loc, vel, ea, nodes, lm = oh.prepare_inputs(fx["raw::loc"], fx["raw::vel"], fx["raw::edge_attr_o"],
                                                row, col, N, fx["raw::charges"])
    for got, key in [(loc, "in::x"), (vel, "in::v"), (ea, "in::edge_attr"), (nodes, "in::h"),
                     (lm, "in::loc_mean")]:
        assert maxnorm_rel(got, fx[key]) < 1e-6, key


def test_spectral_layers_match(egno_fx):
    fx = egno_fx
    p = params_of(fx)
    for i in range(4):
        h_in = fx[f"cap::tconv{i}.in0"]
        got = oe.time_conv(h_in, p[f"time_conv_modules.{i}.t_conv.weights1"])
        assert maxnorm_rel(got, fx[f"cap::tconv{i}.out"]) < 1e-6
        X = fx[f"cap::tconvx{i}.in0"]
        got = oe.time_conv_x(X, p[f"time_conv_x_modules.{i}.t_conv.weights1"])
        assert maxnorm_rel(got, fx[f"cap::tconvx{i}.out"]) < 1e-6


@pytest.mark.parametrize("dtype,tol", [(np.float32, TOL32), (np.float64, TOL32)])
def test_egno_forward(egno_fx, dtype, tol):
    fx = egno_fx
    p = {k: v.astype(dtype) for k, v in params_of(fx).items()}
    cap = {}
    x, v, h = oe.egno_forward(p, **_egno_inputs(fx, dtype), capture=cap)
    assert maxnorm_rel(x, fx["out::x"]) < tol
    assert maxnorm_rel(v, fx["out::v"]) < tol
    assert maxnorm_rel(h, fx["out::h"]) < tol
    for i in range(4):
        for k, got in enumerate(cap[f"layer{i}"]):
            assert maxnorm_rel(got, fx[f"cap::layer{i}.out{k}"]) < tol


def test_egno_rollout_two_segments(egno_fx):
    fx = egno_fx
    ro = load_golden("egno_rollout")
    p = params_of(fx)
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    L = int(ro["cfg::traj_len"])
    t_full = np.tile(np.arange(1, T * L + 1), (B, 1))
    preds, en, en_all = oh.egno_rollout(
        p, fx["in::h"], fx["in::x"], fx["in::row"], fx["in::col"], fx["in::v"],
        fx["raw::edge_attr_o"], fx["in::edge_attr"], fx["in::loc_mean"], N, L, B,
        fx["raw::charges"], T=T, t_out=t_full)
    # segment 0 is a plain forward; segment 1 starts from a chaotic state
    assert maxnorm_rel(preds[:T], ro["out::loc_preds"][:T]) < TOL32
    assert maxnorm_rel(preds, ro["out::loc_preds"]) < 1e-4
    assert maxnorm_rel(en_all[:T], ro["out::energies_allsteps"][:T]) < 1e-4


def test_egno_loss_matches(egno_fx):
    fx = egno_fx
    g = load_golden("egno_grad")
    p = params_of(fx)
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    x, _, _ = oe.egno_forward(p, **_egno_inputs(fx))
    pred = x.reshape(T, B * N, 3).transpose(1, 0, 2).reshape(B, N, T, 3)
    losses = ((pred - g["in::loc_true"]) ** 2).mean(axis=(0, 1, 3))
    assert maxnorm_rel(losses, g["out::losses"]) < TOL32
    assert abs(losses.mean() - float(g["out::loss"])) / float(g["out::loss"]) < TOL32


def test_segno_gcl_and_forward_step(segno_fx):
    fx = segno_fx
    p = params_of(fx)
    T = int(fx["cfg::T"])
    row, col = fx["in::row"], fx["in::col"]
    h, x, v = osg.gcl_forward(p, fx["in::h_emb"], row, col, fx["in::x"], fx["in::v"],
                              fx["in::edge_attr"], n_layers=T, dense_mean=True)
    assert maxnorm_rel(h, fx["gcl::h"]) < TOL32
    assert maxnorm_rel(x, fx["gcl::x"]) < TOL32
    assert maxnorm_rel(v, fx["gcl::v"]) < TOL32
    for dense in (True, False):
        x, h, v = osg.forward_step(p, fx["in::h_emb"], fx["in::x"], row, col, fx["in::v"],
                                   fx["in::edge_attr"], T=T, dense_mean=dense)
        assert maxnorm_rel(x, fx["step::x"]) < TOL32
        assert maxnorm_rel(v, fx["step::v"]) < TOL32
        assert maxnorm_rel(h, fx["step::h"]) < TOL32


def test_segno_forward_bug_compat(segno_fx):
    fx = segno_fx
    p = params_of(fx)
    x, h, v = osg.forward(p, fx["in::his"], fx["in::x"], fx["in::row"], fx["in::col"], fx["in::v"],
                          fx["in::edge_attr"], T=int(fx["cfg::T"]), bug_compat=True)
    assert np.array_equal(x, fx["fwd::x"]) and np.array_equal(v, fx["fwd::v"])
    assert maxnorm_rel(h, fx["fwd::h"]) < 1e-6


def test_segno_rollout(segno_fx):
    fx = segno_fx
    ro = load_golden("segno_rollout")
    p = params_of(fx)
    B = int(fx["cfg::B"])
    preds, en = oh.segno_rollout(p, fx["in::his"], fx["in::x"], fx["in::row"], fx["in::col"],
                                 fx["in::v"], fx["in::edge_attr"], 2, list(ro["cfg::num_steps"]),
                                 fx["raw::charges"], B)
    assert maxnorm_rel(preds, ro["out::loc_preds"]) < TOL32
    assert maxnorm_rel(en, ro["out::energies"]) < 1e-4


def test_segno_gravity_n100():
    fx = load_golden("segno_gravity")
    p = params_of(fx)
    B, N = int(fx["cfg::B"]), int(fx["cfg::N"])
    row, col = oh.full_edges(B, N)
    hh = oe.linear(fx["in::his"], p, "embedding")
    x, h, v = osg.forward_step(p, hh, fx["in::x"], row, col, fx["in::v"], fx["in::edge_attr"],
                               T=int(fx["cfg::T"]))
    assert maxnorm_rel(x, fx["step::x"]) < TOL32
    assert maxnorm_rel(v, fx["step::v"]) < TOL32
    assert maxnorm_rel(h, fx["step::h"]) < TOL32


def test_oracle_gradients_match_reference_golden():
    """oracle/egno_grad.py (hand-written reverse pass) vs the reference's autograd gradients of one
    training step (main_simulation_simple_no.py:267-280), recorded in egno_grad.npz."""
    from oracle import egno_grad as og
    fx = load_golden("egno_fwd")
    gd = load_golden("egno_grad")
    p = {k: v.astype(np.float64) for k, v in params_of(fx).items()}
    i = lambda k: fx["in::" + k].astype(np.float64)  # noqa: E731
    loss, losses, g = og.egno_loss_and_grads(p, i("x"), i("h"), fx["in::row"], fx["in::col"], i("edge_attr"),
                                             i("v"), i("loc_mean"), fx["in::t_out"],
                                             gd["in::loc_true"].astype(np.float64), T=int(fx["cfg::T"]))
    assert abs(loss - float(gd["out::loss"])) <= 1e-5 * abs(float(gd["out::loss"]))
    np.testing.assert_allclose(losses, gd["out::losses"], rtol=1e-5)
    assert set(g) == set(p)
    for k in p:
        ref = gd["grad::" + k]
        if np.abs(ref).max() == 0:          # parameters that do not reach the loss (nograd list)
            assert np.abs(g[k]).max() == 0, k
        else:
            assert maxnorm_rel(g[k], ref) < 2e-6, k


def test_egno_five_modes_matches_reference():
    """num_modes=5 at num_timesteps=8 (5 spectral modes including the Nyquist bin): the drop-in's
    seed-0 initialisation reproduces the reference's weights (per-tensor sums) and the oracle
    reproduces the reference's forward."""
    import torch
    import no_node_comparison_amd as pkg
    fx = load_golden("egno_m5")
    T, modes = int(fx["cfg::T"]), int(fx["cfg::modes"])
    torch.manual_seed(0)
    m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=modes,
                 num_timesteps=T, time_emb_dim=32)
    sd = {k: v.detach().numpy() for k, v in m.state_dict().items()}
    for k, v in sd.items():
        assert abs(float(v.astype(np.float64).sum()) - float(fx["wsum::" + k])) <= 1e-6 * max(1.0, abs(float(fx["wsum::" + k]))), k
    x, v, h = oe.egno_forward({k: a.astype(np.float64) for k, a in sd.items()},
                              **_egno_inputs(fx, np.float64), T=T)
    assert maxnorm_rel(x, fx["out::x"]) < TOL32
    assert maxnorm_rel(v, fx["out::v"]) < TOL32
    assert maxnorm_rel(h, fx["out::h"]) < TOL32


def test_oracle_gradients_five_modes_match_reference_golden():
    """The reverse pass at num_modes=5, num_timesteps=8 (model_confs.yaml:12's alternative: 5 spectral
    modes incl. the Nyquist bin) against the reference's autograd gradients in egno_m5.npz."""
    import torch
    import no_node_comparison_amd as pkg
    from oracle import egno_grad as og
    fx = load_golden("egno_m5")
    T, modes = int(fx["cfg::T"]), int(fx["cfg::modes"])
    torch.manual_seed(0)
    m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=modes,
                 num_timesteps=T, time_emb_dim=32)
    p = {k: v.detach().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    i = lambda k: fx["in::" + k].astype(np.float64)  # noqa: E731
    loss, _, g = og.egno_loss_and_grads(p, i("x"), i("h"), fx["in::row"], fx["in::col"], i("edge_attr"), i("v"),
                                        i("loc_mean"), fx["in::t_out"], i("loc_true"), T=T)
    assert abs(loss - float(fx["out::loss"])) <= 1e-5 * abs(float(fx["out::loss"]))
    for k in p:
        ref = fx["grad::" + k]
        if np.abs(ref).max() == 0:
            assert np.abs(g[k]).max() == 0, k
        else:
            assert maxnorm_rel(g[k], ref) < 2e-6, k


def test_egno_multi_input_matches_reference():
    """num_inputs=3 (egno.py:44-96 multi-input branch): seed-0 initialisation of the drop-in equals
    the reference's (per-tensor sums), and the oracle's multi-input forward reproduces the
    reference's output."""
    import torch
    import no_node_comparison_amd as pkg
    fx = load_golden("egno_multi")
    T, I = int(fx["cfg::T"]), int(fx["cfg::I"])
    torch.manual_seed(0)
    m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                 num_timesteps=T, time_emb_dim=32, num_inputs=I)
    sd = {k: v.detach().numpy() for k, v in m.state_dict().items()}
    for k, v in sd.items():
        want = float(fx["wsum::" + k])
        assert abs(float(v.astype(np.float64).sum()) - want) <= 1e-6 * max(1.0, abs(want)), k
    d = lambda k: fx[k].astype(np.float64)  # noqa: E731
    x, v, h = oe.egno_forward_multi({k: a.astype(np.float64) for k, a in sd.items()}, d("in::x"), d("in::h"),
                                    fx["in::row"], fx["in::col"], d("in::edge_attr"), d("in::v"),
                                    d("in::loc_mean"), fx["in::t_in"], fx["in::t_out"], T=T)
    assert maxnorm_rel(x, fx["out::x"]) < TOL32
    assert maxnorm_rel(v, fx["out::v"]) < TOL32
    assert maxnorm_rel(h, fx["out::h"]) < TOL32


def test_segno_multi_input_attn_matches_reference():
    """SEGNO live forward with num_inputs=3, multiple_agg='attn' (model.py:53-92, 104-139): the oracle
    reproduces the reference's output (bug_compat: the state before the last forward_step) and the
    last forward_step the reference discards."""
    fx = load_golden("segno_multi")
    p = {k: v.astype(np.float64) for k, v in params_of(fx).items()}
    T = int(fx["cfg::T"])
    d = lambda k: fx[k].astype(np.float64)  # noqa: E731
    args = (p, d("in::his"), d("in::x"), fx["in::row"], fx["in::col"], d("in::v"), d("in::edge_attr"),
            fx["in::in_steps"])
    for bug, pre in ((True, "fwd"), (False, "last")):
        x, h, v = osg.forward_multi(*args, T=T, multiple_agg="attn", bug_compat=bug, dense_mean=True)
        assert maxnorm_rel(x, fx[pre + "::x"]) < TOL32
        assert maxnorm_rel(h, fx[pre + "::h"]) < TOL32
        assert maxnorm_rel(v, fx[pre + "::v"]) < TOL32
