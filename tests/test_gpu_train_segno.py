"""GPU parity of SEGNO training (train_nbody.py:150-178 through forward_step, model.py:95-102): the
gradients of one step of nn.MSELoss(x after T substeps, loc_end) through the HIP integrator's
reverse pass (nonode_segno_forward_train / nonode_segno_backward, autograd.SEGNOStepTrain).

Bars (max-norm relative per parameter tensor):
  - vs the reference's own autograd gradients (tests/golden/segno_grad.npz): 1e-5;
  - vs torch autograd of the op-by-op restatement (oracle/torch_ref.py) in float64 on other shapes,
    up to the C3 size (B=512): 1e-5.
"""
import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg
from oracle import torch_ref as tr
from tests.conftest import check_rel, load_golden, params_of
from tests.test_gpu_parity import DEV, _dev

pytestmark = pytest.mark.gpu
GTOL = 1e-5


def _segno(sd=None, seed=0, recurrent=True, cw=1.0):
    torch.manual_seed(seed)
    m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=recurrent, coords_weight=cw,
                  device=DEV)
    if sd is not None:
        m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.train()


def _case(B, N, seed):
    """Charged inputs featurised as train_nbody.py:84-123 (h = |v|, edge_attr = [q_i q_j, |x_i - x_j|^2])."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B * N, 3, generator=g) * (N / 5) ** (1 / 3)
    v = torch.randn(B * N, 3, generator=g) * 0.5
    q = torch.randint(0, 2, (B * N, 1), generator=g).float() * 2 - 1
    r, c = tr.full_edges(B, N)
    ea = torch.cat([q[r] * q[c], ((x[r] - x[c]) ** 2).sum(1, keepdim=True)], 1)
    his = v.norm(dim=1, keepdim=True)
    target = x + v * 0.3 + 0.05 * torch.randn(B * N, 3, generator=g)
    return his, x, v, r, c, ea, target


def _hip_step(m, his, x, v, r, c, ea, target, T):
    m.zero_grad(set_to_none=True)
    edges = [_dev(r), _dev(c)]
    xo, ho, vo = m(_dev(his), _dev(x), edges, _dev(v), _dev(ea), T=T)
    loss = torch.nn.functional.mse_loss(xo, _dev(target))
    loss.backward()
    torch.cuda.synchronize()
    return loss, xo


def _ref_step(m, his, x, v, r, c, ea, target, T, recurrent=True, cw=1.0, dt=torch.float64):
    p = {k: q.detach().cpu().to(dt).requires_grad_(True) for k, q in m.state_dict().items()}
    xr, _, _ = tr.segno_forward_step(p, his.to(dt), x.to(dt), r, c, v.to(dt), ea.to(dt), T=T, dense_mean=False,
                                     recurrent=recurrent) if cw == 1.0 else _ref_cw(p, his, x, r, c, v, ea, T,
                                                                                       recurrent, cw, dt)
    loss = torch.nn.functional.mse_loss(xr, target.to(dt))
    loss.backward()
    return loss, p


def _ref_cw(p, his, x, r, c, v, ea, T, recurrent, cw, dt):
    h = tr._lin(his.to(dt), p, "embedding")
    x, v = x.to(dt), v.to(dt)
    for _ in range(T):
        h, x, v = tr.gcl(p, h, r, c, x, v, ea.to(dt), T, recurrent=recurrent, coords_weight=cw, dense_mean=False)
    return x, h, v


def _check_grads(m, p, bar, tag):
    n = 0
    for k, q in m.named_parameters():
        ref = p[k].grad
        if ref is None or float(ref.abs().max()) == 0:
            assert q.grad is None or float(q.grad.abs().max()) == 0, k
            continue
        if float(ref.abs().max()) < 1e-12:
            # zero in exact arithmetic (the attention output bias: softmax ignores a constant shift);
            # float64 leaves ~1e-17, float32 ~1e-9: both are rounding residue
            assert float(q.grad.abs().max()) < 1e-7, k
            continue
        n += 1
        check_rel(f"{tag} grad {k}", q.grad, ref, bar)
    return n


def test_segno_gradients_match_reference_golden():
    gd = load_golden("segno_grad")
    B, N, T = int(gd["cfg::B"]), int(gd["cfg::N"]), int(gd["cfg::T"])
    m = _segno(params_of(gd))
    edges = [_dev(gd["in::row"]), _dev(gd["in::col"])]
    xo, _, _ = m(_dev(gd["in::his"]), _dev(gd["in::x"]), edges, _dev(gd["in::v"]), _dev(gd["in::edge_attr"]), T=T)
    loss = torch.nn.MSELoss()(xo, _dev(gd["in::loc_end"]))
    loss.backward()
    torch.cuda.synchronize()
    check_rel("x", xo, gd["out::x"], 1e-5)
    assert abs(float(loss.detach()) - float(gd["out::loss"])) <= 1e-5 * abs(float(gd["out::loss"]))
    n = 0
    for k, q in m.named_parameters():
        if "grad::" + k not in gd:
            assert q.grad is None or float(q.grad.abs().max()) == 0, k   # coord_mlp_vel: not on the path
            continue
        n += 1
        check_rel(f"grad {k}", q.grad, gd["grad::" + k], GTOL)
    assert n == 14


@pytest.mark.parametrize("B,N,T,recurrent,cw", [(3, 7, 4, True, 1.0), (2, 20, 10, True, 1.0), (4, 5, 10, False, 1.0),
                                                (2, 20, 3, True, 0.5), (5, 2, 6, True, 1.0), (1, 31, 3, True, 1.0),
                                                (1, 64, 3, True, 1.0), (1, 100, 2, True, 1.0)])
def test_segno_gradients_match_f64_reference(B, N, T, recurrent, cw):
    m = _segno(seed=B * 10 + N, recurrent=recurrent, cw=cw)
    case = _case(B, N, seed=N + T)
    loss, xo = _hip_step(m, *case, T)
    lr, p = _ref_step(m, *case, T, recurrent=recurrent, cw=cw)
    assert abs(float(loss.detach()) - float(lr.detach())) <= 1e-5 * abs(float(lr.detach()))
    assert _check_grads(m, p, GTOL, f"B={B} N={N} T={T}") == 14


def test_segno_c3_shard_gradients_match_f64_reference():
    """C3 size (B=512, N=20, 10 substeps): every parameter gradient against float64 autograd."""
    B, N, T = 512, 20, 10
    m = _segno(seed=7)
    case = _case(B, N, seed=8)
    loss, _ = _hip_step(m, *case, T)
    lr, p = _ref_step(m, *case, T)
    assert abs(float(loss.detach()) - float(lr.detach())) <= 1e-6 * abs(float(lr.detach()))
    assert _check_grads(m, p, GTOL, "C3") == 14


def test_segno_train_forward_equals_inference_forward():
    """The training forward_step (one launch per substep, saved state) gives bitwise the fused
    inference launch's outputs from the same embedded h. (The training embedding is torch's Linear,
    the inference one a HIP kernel: those may differ in the last bit, so both start from one h.)"""
    B, N, T = 8, 20, 10
    m = _segno(seed=3)
    his, x, v, r, c, ea, _ = _case(B, N, seed=4)
    h = torch.randn(B * N, 64, generator=torch.Generator().manual_seed(5))
    args = (_dev(h), _dev(x), [_dev(r), _dev(c)], _dev(v), _dev(ea))
    xa, ha, va = m.forward_step(*args, T=T)
    assert xa.requires_grad
    with torch.no_grad():
        xb, hb, vb = m.forward_step(*args, T=T)
    for a, b in ((xa, xb), (ha, hb), (va, vb)):
        assert torch.equal(a.detach(), b)


def test_segno_train_model_forward_equals_inference_forward():
    """SEGNO.forward in training (autograd.SEGNOTrain: nonode_embedding_forward, then the training
    launch of the T substeps) gives bitwise the inference forward's outputs (the same embedding
    kernel and layer arithmetic)."""
    B, N, T = 8, 20, 10
    m = _segno(seed=3)
    his, x, v, r, c, ea, _ = _case(B, N, seed=4)
    args = (_dev(his), _dev(x), [_dev(r), _dev(c)], _dev(v), _dev(ea))
    xa, ha, va = m(*args, T=T)
    assert xa.requires_grad
    with torch.no_grad():
        xb, hb, vb = m(*args, T=T)
    for a, b in ((xa, xb), (ha, hb), (va, vb)):
        assert torch.equal(a.detach(), b)


@pytest.mark.parametrize("fused", [False, True])
def test_segno_adam_step_runs_and_repacks(fused):
    """An optimizer step changes the GCL weights in place; the next forward must use the re-packed
    forward and backward blobs (fused=True: no version bump, only the optimizer step hook drops them)."""
    B, N, T = 2, 6, 5
    m = _segno(seed=5)
    case = _case(B, N, seed=6)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, fused=fused)
    _hip_step(m, *case, T)
    opt.step()
    loss, _ = _hip_step(m, *case, T)
    lr, p = _ref_step(m, *case, T)
    assert abs(float(loss.detach()) - float(lr.detach())) <= 1e-5 * abs(float(lr.detach()))
    _check_grads(m, p, GTOL, "after step")


def test_segno_multi_input_attn_gradients_match_f64_reference():
    """num_inputs = 3, multiple_agg='attn' (model.py:53-92, 104-139): gradients through the three
    integrator segments and the attention folds (the attention MLP is a torch op on the tape)."""
    B, N, T, I = 2, 6, 10, 3
    torch.manual_seed(9)
    m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True, multiple_agg="attn",
                  device=DEV).train()
    g = torch.Generator().manual_seed(10)
    x = torch.randn(B * N, I, 3, generator=g)
    v = torch.randn(B * N, I, 3, generator=g) * 0.5
    his = v.norm(dim=-1, keepdim=True)
    r, c = tr.full_edges(B, N)
    ea = torch.cat([torch.randn(B * N * (N - 1), 1, generator=g).sign(),
                    ((x[r, -1] - x[c, -1]) ** 2).sum(1, keepdim=True)], 1)
    in_steps = torch.tensor([0, 2, 5])
    target = torch.randn(B * N, 3, generator=g)
    m.zero_grad(set_to_none=True)
    xo, _, _ = m(_dev(his), _dev(x), [_dev(r), _dev(c)], _dev(v), _dev(ea), T=T, in_steps=in_steps)
    loss = torch.nn.functional.mse_loss(xo, _dev(target))
    loss.backward()
    torch.cuda.synchronize()
    # float64 reference: the same segment loop on the restatement
    dt = torch.float64
    p = {k: q.detach().cpu().to(dt).requires_grad_(True) for k, q in m.state_dict().items()}
    h = tr._lin(his.to(dt), p, "embedding")
    xs, vs = x.to(dt), v.to(dt)
    steps = [2, 3, T]

    def attn(ls, vls, hs):
        speed = vls.norm(dim=-1, keepdim=True)
        z = torch.tanh(tr._lin(torch.cat([speed, hs], -1), p, "enc_attn_net.attn_mlp.0"))
        a = tr._lin(z, p, "enc_attn_net.attn_mlp.2").softmax(dim=1)
        return (a * ls).sum(1), (a * vls).sum(1), (a * hs).sum(1)

    h_, x_, v_ = h[:, 0], xs[:, 0], vs[:, 0]
    for i, st in enumerate(steps):
        hi = h_
        xi, vi = x_, v_
        for _ in range(st):
            hi, xi, vi = tr.gcl(p, hi, r, c, xi, vi, ea.to(dt), st, dense_mean=False)
        if i < len(steps) - 1:
            x_, v_, h_ = attn(torch.stack([xs[:, i + 1], xi], 1), torch.stack([vs[:, i + 1], vi], 1),
                              torch.stack([h[:, i + 1], hi], 1))
    lr = torch.nn.functional.mse_loss(xi, target.to(dt))
    lr.backward()
    assert abs(float(loss.detach()) - float(lr.detach())) <= 1e-5 * abs(float(lr.detach()))
    assert _check_grads(m, p, GTOL, "attn") == 17


def test_segno_his_gradient_and_saved_input_version():
    """SEGNO.forward in training (autograd.SEGNOTrain) with an input `his` that requires grad: dL/dhis
    through the embedding Linear (model.py:73) against float64 autograd; and `his` is saved through
    save_for_backward, so editing it in place after the forward raises instead of silently changing
    the embedding weight gradient."""
    B, N, T = 3, 7, 4
    m = _segno(seed=11)
    his, x, v, r, c, ea, target = _case(B, N, seed=12)
    hd = _dev(his).requires_grad_(True)
    m.zero_grad(set_to_none=True)
    xo, _, _ = m(hd, _dev(x), [_dev(r), _dev(c)], _dev(v), _dev(ea), T=T)
    torch.nn.functional.mse_loss(xo, _dev(target)).backward()
    torch.cuda.synchronize()
    dt = torch.float64
    p = {k: q.detach().cpu().to(dt).requires_grad_(True) for k, q in m.state_dict().items()}
    hr = his.to(dt).requires_grad_(True)
    xr, _, _ = tr.segno_forward_step(p, hr, x.to(dt), r, c, v.to(dt), ea.to(dt), T=T, dense_mean=False)
    torch.nn.functional.mse_loss(xr, target.to(dt)).backward()
    check_rel("dL/dhis", hd.grad, hr.grad, GTOL)
    assert _check_grads(m, p, GTOL, "his") == 14
    h2 = _dev(his)
    xo, _, _ = m(h2, _dev(x), [_dev(r), _dev(c)], _dev(v), _dev(ea), T=T)
    h2.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        torch.nn.functional.mse_loss(xo, _dev(target)).backward()
