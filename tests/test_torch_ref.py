"""Pin oracle/torch_ref.py (the op-by-op torch CPU path bench.py times as `cpu_baseline`) to the
fixtures recorded from the reference itself (CPU only)."""
import numpy as np
import torch

from oracle import torch_ref as tr
from tests.conftest import load_golden, maxnorm_rel, params_of

TOL = 1e-6     # fp32 restatement of the same ops: within the fp32 noise floor


def _p(fx, grad=False):
    return {k: torch.tensor(v, requires_grad=grad) for k, v in params_of(fx).items()}


def _t(fx, k):
    return torch.tensor(fx[k])


def test_edges_match_dataset_order():
    fx = load_golden("egno_fwd")
    r, c = tr.full_edges(int(fx["cfg::B"]), int(fx["cfg::N"]))
    assert np.array_equal(r.numpy(), fx["in::row"]) and np.array_equal(c.numpy(), fx["in::col"])


def test_prepare_inputs_matches_reference():
    fx = load_golden("egno_fwd")
    N = int(fx["cfg::N"])
    out = tr.prepare_inputs(_t(fx, "raw::loc"), _t(fx, "raw::vel"), _t(fx, "raw::edge_attr_o"),
                            _t(fx, "in::row"), _t(fx, "in::col"), N, _t(fx, "raw::charges"))
    for got, k in zip(out, ["in::x", "in::v", "in::edge_attr", "in::h", "in::loc_mean"]):
        assert maxnorm_rel(got.numpy(), fx[k]) < TOL, k


def test_egno_forward_matches_reference():
    fx = load_golden("egno_fwd")
    with torch.no_grad():
        x, v, h = tr.egno_forward(_p(fx), _t(fx, "in::x"), _t(fx, "in::h"), _t(fx, "in::row"), _t(fx, "in::col"),
                                  _t(fx, "in::edge_attr"), _t(fx, "in::v"), _t(fx, "in::loc_mean"),
                                  _t(fx, "in::t_out"), T=int(fx["cfg::T"]))
    for got, k in ((x, "out::x"), (v, "out::v"), (h, "out::h")):
        assert maxnorm_rel(got.numpy(), fx[k]) < TOL, k


def test_egno_autograd_gradients_match_reference():
    """One training step's loss and gradients (main_simulation_simple_no.py:267-280) through torch
    autograd of the restatement, against the reference's own autograd (egno_grad.npz)."""
    fx = load_golden("egno_fwd")
    gd = load_golden("egno_grad")
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    p = _p(fx, grad=True)
    x, _, _ = tr.egno_forward(p, _t(fx, "in::x"), _t(fx, "in::h"), _t(fx, "in::row"), _t(fx, "in::col"),
                              _t(fx, "in::edge_attr"), _t(fx, "in::v"), _t(fx, "in::loc_mean"),
                              _t(fx, "in::t_out"), T=T)
    pred = x.reshape(T, B, N, 3).permute(1, 2, 0, 3)
    loss = ((pred - _t(gd, "in::loc_true")) ** 2).mean((0, 1, 3)).mean()
    loss.backward()
    assert abs(float(loss.detach()) - float(gd["out::loss"])) <= 1e-6 * abs(float(gd["out::loss"]))
    for k, t in p.items():
        ref = gd["grad::" + k]
        if np.abs(ref).max() == 0:
            assert t.grad is None or float(t.grad.abs().max()) == 0, k
        else:
            assert maxnorm_rel(t.grad.numpy(), ref) < 1e-5, k


def test_segno_autograd_gradients_match_reference():
    """One SEGNO training step (train_nbody.py:150-178 through forward_step, nn.MSELoss): loss and
    every parameter gradient of torch autograd through the restatement, in float32 against the
    reference's own autograd (segno_grad.npz) and in float64 (the bar the GPU test uses)."""
    gd = load_golden("segno_grad")
    T = int(gd["cfg::T"])
    for dt, tol in ((torch.float32, 1e-5), (torch.float64, 1e-5)):
        p = {k: torch.tensor(v, dtype=dt, requires_grad=True) for k, v in params_of(gd).items()}
        t = lambda k: torch.tensor(gd[k]).to(dt) if gd[k].dtype.kind == "f" else torch.tensor(gd[k])  # noqa: E731
        x, _, _ = tr.segno_forward_step(p, t("in::his"), t("in::x"), t("in::row"), t("in::col"), t("in::v"),
                                        t("in::edge_attr"), T=T, dense_mean=False)
        loss = torch.nn.functional.mse_loss(x, t("in::loc_end"))
        loss.backward()
        assert abs(float(loss.detach()) - float(gd["out::loss"])) <= 1e-6 * abs(float(gd["out::loss"]))
        n = 0
        for k, q in p.items():
            if "grad::" + k not in gd:
                assert q.grad is None or float(q.grad.abs().max()) == 0, k   # coord_mlp_vel
                continue
            n += 1
            assert maxnorm_rel(q.grad.double().numpy(), gd["grad::" + k]) < tol, (dt, k)
        assert n == 14


def test_segno_forward_step_dense_and_scatter():
    fx = load_golden("segno_fwd")
    p = _p(fx)
    for dense in (True, False):
        with torch.no_grad():
            x, h, v = tr.segno_forward_step(p, _t(fx, "in::his"), _t(fx, "in::x"), _t(fx, "in::row"),
                                            _t(fx, "in::col"), _t(fx, "in::v"), _t(fx, "in::edge_attr"),
                                            T=int(fx["cfg::T"]), dense_mean=dense)
        for got, k in ((x, "step::x"), (h, "step::h"), (v, "step::v")):
            assert maxnorm_rel(got.numpy(), fx[k]) < TOL, (dense, k)


def test_segno_gravity_n100():
    fx = load_golden("segno_gravity")
    B, N = int(fx["cfg::B"]), int(fx["cfg::N"])
    r, c = tr.full_edges(B, N)
    with torch.no_grad():
        x, h, v = tr.segno_forward_step(_p(fx), _t(fx, "in::his"), _t(fx, "in::x"), r, c, _t(fx, "in::v"),
                                        _t(fx, "in::edge_attr"), T=int(fx["cfg::T"]), dense_mean=False)
    for got, k in ((x, "step::x"), (h, "step::h"), (v, "step::v")):
        assert maxnorm_rel(got.numpy(), fx[k]) < 1e-5, k


def test_egno_rollout_first_segment_matches_reference():
    fx = load_golden("egno_fwd")
    ro = load_golden("egno_rollout")
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    L = int(ro["cfg::traj_len"])
    t_full = torch.arange(1, T * L + 1).repeat(B, 1)
    with torch.no_grad():
        preds = tr.egno_rollout(_p(fx), _t(fx, "in::h"), _t(fx, "in::x"), _t(fx, "in::row"), _t(fx, "in::col"),
                                _t(fx, "in::v"), _t(fx, "raw::edge_attr_o"), _t(fx, "in::edge_attr"),
                                _t(fx, "in::loc_mean"), N, L, B, _t(fx, "raw::charges"), T=T, t_out=t_full)
    assert maxnorm_rel(preds[:T].numpy(), ro["out::loc_preds"][:T]) < TOL
    assert maxnorm_rel(preds.numpy(), ro["out::loc_preds"]) < 1e-4     # chaotic second segment


def test_segno_rollout_matches_reference():
    fx = load_golden("segno_fwd")
    ro = load_golden("segno_rollout")
    with torch.no_grad():
        preds = tr.segno_rollout(_p(fx), _t(fx, "in::his"), _t(fx, "in::x"), _t(fx, "in::row"), _t(fx, "in::col"),
                                 _t(fx, "in::v"), _t(fx, "in::edge_attr"), list(ro["cfg::num_steps"]),
                                 _t(fx, "raw::charges"), dense_mean=True)
    assert maxnorm_rel(preds.numpy(), ro["out::loc_preds"]) < 1e-5
