"""GPU parity of the reference constructor options (tests/test_options.py pins the oracle side):
EGNO norm=True (radial input normalised, basic.py:140-141), EGNO use_time_conv=False
(egno.py:27-33, 99-107 skipped), SEGNO tanh=True (coord_mlp ends in nn.Tanh, gcl.py:57-59) --
forward and training gradients through the HIP kernels; EGNO flat=True (basic.py:38-40, 256-wide
Tanh MLPs, csrc/nonode_flat.hip) -- forward and training (autograd.FlatLayerTrain).

Bars (max-norm relative): 1e-5 against the reference's own outputs / autograd gradients
(egno_norm / egno_notc / segno_tanh fixtures) and against float64 references on other shapes.
"""
import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg
from oracle import egno as oe
from oracle import harness as oh
from oracle import torch_ref as tr
from tests.conftest import check_rel, load_golden, params_of
from tests.test_gpu_parity import DEV, _dev, _egno_case
from tests.test_gpu_train import _hip_lrelu_masks

pytestmark = pytest.mark.gpu
TOL = 1e-5
OPTS = {"egno_norm": dict(norm=True), "egno_notc": dict(use_time_conv=False)}


def _egno(opts, sd=None, seed=0, T=10, num_inputs=1):
    torch.manual_seed(seed)
    m = pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2, num_timesteps=T,
                 time_emb_dim=32, num_inputs=num_inputs, device=DEV, **opts)
    if sd is not None:
        m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m


def _run(m, inp):
    return m(inp["x"], inp["h"], [inp["row"], inp["col"]], inp["edge_fea"], v=inp["v"], loc_mean=inp["loc_mean"],
             timesteps_out=inp["t_out"])


def _golden_inputs(fx):
    inp = {k: _dev(fx["in::" + k]) for k in ("x", "h", "row", "col", "edge_attr", "v", "loc_mean", "t_out")}
    inp["edge_fea"] = inp.pop("edge_attr")
    return inp


@pytest.mark.parametrize("name", sorted(OPTS))
def test_egno_option_forward_and_gradients_match_reference_golden(name):
    fx = load_golden(name)
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    m = _egno(OPTS[name], params_of(fx)).eval()
    inp = _golden_inputs(fx)
    with torch.no_grad():
        x, v, h = _run(m, inp)
    check_rel(f"{name} x", x.cpu(), fx["out::x"], TOL)
    check_rel(f"{name} v", v.cpu(), fx["out::v"], TOL)
    check_rel(f"{name} h", h.cpu(), fx["out::h"], TOL)
    m.train()
    m.zero_grad(set_to_none=True)
    x, _, _ = _run(m, inp)
    pred = x.reshape(T, B, N, 3).permute(1, 2, 0, 3)
    loss = ((pred - _dev(fx["in::loc_true"])) ** 2).mean((0, 1, 3)).mean()
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss.detach()) - float(fx["out::loss"])) <= 1e-5 * abs(float(fx["out::loss"]))
    for k, p in m.named_parameters():
        ref = fx["grad::" + k]
        if np.abs(ref).max() == 0:
            assert p.grad is None or float(p.grad.abs().max()) <= 1e-6, k
        else:
            check_rel(f"{name} grad {k}", p.grad, ref, TOL)


@pytest.mark.parametrize("name", sorted(OPTS))
@pytest.mark.parametrize("B,N", [(64, 20), (3, 7)])
def test_egno_option_forward_matches_f64_oracle(name, B, N):
    T = 10
    m = _egno(OPTS[name], seed=B + N).eval()
    case = _egno_case(B, N, T, seed=N + 1)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    f64 = {k: (v.astype(np.float64) if k not in ("row", "col", "t_out") else v) for k, v in case.items()}
    xr, vr, hr = oe.egno_forward(p, **f64, T=T, **OPTS[name])
    with torch.no_grad():
        x, v, h = _run(m, {k: _dev(val) for k, val in case.items()})
    check_rel("x", x.cpu(), xr, TOL)
    check_rel("v", v.cpu(), vr, TOL)
    check_rel("h", h.cpu(), hr, TOL)


@pytest.mark.parametrize("name", sorted(OPTS))
def test_egno_option_gradients_match_f64_autograd(name):
    B, N, T = 6, 20, 10
    m = _egno(OPTS[name], seed=7).train()
    case = _egno_case(B, N, T, seed=9)
    target = np.random.default_rng(3).standard_normal((B, N, T, 3)).astype(np.float32)
    m.zero_grad(set_to_none=True)
    x, _, _ = _run(m, {k: _dev(v) for k, v in case.items()})
    loss = ((x.reshape(T, B, N, 3).permute(1, 2, 0, 3) - _dev(target)) ** 2).mean((0, 1, 3)).mean()
    loss.backward()
    torch.cuda.synchronize()
    dt = torch.float64
    p = {k: v.detach().cpu().to(dt).requires_grad_(True) for k, v in m.state_dict().items()}
    t = {k: torch.tensor(v).to(dt) if v.dtype.kind == "f" else torch.tensor(v) for k, v in case.items()}
    xr, _, _ = tr.egno_forward(p, t["x"], t["h"], t["row"], t["col"], t["edge_fea"], t["v"], t["loc_mean"],
                               t["t_out"], T=T, **OPTS[name])
    lr = ((xr.reshape(T, B, N, 3).permute(1, 2, 0, 3) - torch.tensor(target).to(dt)) ** 2).mean((0, 1, 3)).mean()
    lr.backward()
    assert abs(float(loss.detach()) - float(lr.detach())) <= 1e-5 * abs(float(lr.detach()))
    for k, q in m.named_parameters():
        ref = p[k].grad
        if ref is None or float(ref.abs().max()) == 0:
            assert q.grad is None or float(q.grad.abs().max()) <= 1e-6, k
            continue
        check_rel(f"{name} grad {k}", q.grad, ref, TOL)


def test_egno_no_time_conv_multi_input_matches_oracle():
    """use_time_conv=False with num_inputs = 3 (egno.py:44-96 without the TimeConvs)."""
    B, N, T, I = 2, 6, 10, 3
    m = _egno(OPTS["egno_notc"], seed=21, num_inputs=I).eval()
    rng = np.random.default_rng(4)
    x = rng.standard_normal((I, B * N, 3)).astype(np.float32)
    v = rng.standard_normal((I, B * N, 3)).astype(np.float32) * 0.5
    h = np.concatenate([np.linalg.norm(v, axis=-1, keepdims=True), np.ones((I, B * N, 1), np.float32)], -1)
    row, col = tr.full_edges(B, N)
    ea = rng.standard_normal((I, B * N * (N - 1), 2)).astype(np.float32)
    t_in = np.tile(np.array([-2.0, -1.0, 0.0], np.float32), (B, 1))
    t_out = np.tile(np.arange(1, T + 1, dtype=np.float32), (B, 1))
    p = {k: q.detach().cpu().numpy().astype(np.float64) for k, q in m.state_dict().items()}
    xr, vr, hr = oe.egno_forward_multi(p, x.astype(np.float64), h.astype(np.float64), row.numpy(), col.numpy(),
                                       ea.astype(np.float64), v.astype(np.float64), None, t_in, t_out, T=T,
                                       use_time_conv=False)
    with torch.no_grad():
        xo, vo, ho = m(_dev(x), _dev(h), [_dev(row), _dev(col)], _dev(ea), v=_dev(v), loc_mean=None,
                       timesteps_in=_dev(t_in), timesteps_out=_dev(t_out))
    check_rel("x", xo.cpu(), xr, TOL)
    check_rel("v", vo.cpu(), vr, TOL)
    check_rel("h", ho.cpu(), hr, TOL)


FLAT = {"flat": dict(flat=True), "flat_norm": dict(flat=True, norm=True),
        "flat_notc": dict(flat=True, use_time_conv=False)}


def test_egno_flat_forward_and_gradients_match_reference_golden():
    """flat=True against the reference's own outputs, loss and autograd gradients (egno_flat fixture):
    one training step of main_simulation_simple_no.py:267-280 with --flat."""
    fx = load_golden("egno_flat")
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    m = _egno(FLAT["flat"], params_of(fx)).eval()
    inp = _golden_inputs(fx)
    with torch.no_grad():
        x, v, h = _run(m, inp)
    check_rel("flat x", x.cpu(), fx["out::x"], TOL)
    check_rel("flat v", v.cpu(), fx["out::v"], TOL)
    check_rel("flat h", h.cpu(), fx["out::h"], TOL)
    m.train()
    m.zero_grad(set_to_none=True)
    xt, vt, ht = _run(m, inp)
    check_rel("flat train x", xt.detach().cpu(), fx["out::x"], TOL)
    check_rel("flat train h", ht.detach().cpu(), fx["out::h"], TOL)
    pred = xt.reshape(T, B, N, 3).permute(1, 2, 0, 3)
    loss = ((pred - _dev(fx["in::loc_true"])) ** 2).mean((0, 1, 3)).mean()
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss.detach()) - float(fx["out::loss"])) <= 1e-5 * abs(float(fx["out::loss"]))
    n = 0
    for k, p in m.named_parameters():
        ref = fx["grad::" + k]
        if np.abs(ref).max() == 0:
            assert p.grad is None or float(p.grad.abs().max()) <= 1e-6, k
            continue
        n += 1
        check_rel(f"flat grad {k}", p.grad, ref, TOL)
    assert n >= 16 * 4 - 4 + 2 + 8


@pytest.mark.parametrize("name", sorted(FLAT))
@pytest.mark.parametrize("B,N", [(6, 20), (3, 7)])
def test_egno_flat_gradients_match_f64_autograd(name, B, N):
    """flat=True training against float64 torch autograd of the restatement, every option pairing and
    ragged receiver tiles; the loss also reads v and h so every output's reverse is exercised. As in
    test_gpu_train's B=512 case, TimeConv's LeakyReLU kink: the float64 reference is evaluated at the
    HIP reverse's own branch decisions (the head of nonode_egno_tconv_bwd's workspace, the layout of
    the training state's), and every element whose decision differs from float64's lies at the kink
    (|y| tiny against the layer's scale: layer 1 of the (6, 20) case holds one at |y| = 2.5e-8 max)."""
    T = 10
    m = _egno(FLAT[name], seed=B + 3 * N).train()
    case = _egno_case(B, N, T, seed=N + 5)
    rng = np.random.default_rng(B)
    target = rng.standard_normal((B, N, T, 3)).astype(np.float32)
    wv, wh = rng.standard_normal((T * B * N, 3)).astype(np.float32), rng.standard_normal((T * B * N, 64)).astype(np.float32)
    m.zero_grad(set_to_none=True)
    m._train_bwd_sink = []
    x, v, h = _run(m, {k: _dev(val) for k, val in case.items()})
    loss = ((x.reshape(T, B, N, 3).permute(1, 2, 0, 3) - _dev(target)) ** 2).mean((0, 1, 3)).mean() + \
        1e-3 * (v * _dev(wv)).sum() + 1e-4 * (h * _dev(wh)).sum()
    loss.backward()
    torch.cuda.synchronize()
    sink = dict(m._train_bwd_sink)
    del m._train_bwd_sink
    dt = torch.float64
    t = {k: torch.tensor(val).to(dt) if val.dtype.kind == "f" else torch.tensor(val) for k, val in case.items()}
    tw, tv = torch.tensor(wv).to(dt), torch.tensor(wh).to(dt)

    def f64(**kw):
        p = {k: q.detach().cpu().to(dt).requires_grad_(True) for k, q in m.state_dict().items()}
        xr, vr, hr = tr.egno_forward(p, t["x"], t["h"], t["row"], t["col"], t["edge_fea"], t["v"], t["loc_mean"],
                                     t["t_out"], T=T, **FLAT[name], **kw)
        lr = ((xr.reshape(T, B, N, 3).permute(1, 2, 0, 3) - torch.tensor(target).to(dt)) ** 2).mean((0, 1, 3)).mean() + \
            1e-3 * (vr * tw).sum() + 1e-4 * (hr * tv).sum()
        lr.backward()
        return lr, p

    ys = []
    lr, p = f64(lrelu_record=ys)
    assert abs(float(loss.detach()) - float(lr.detach())) <= 1e-5 * abs(float(lr.detach()))
    if FLAT[name].get("use_time_conv", True):
        assert sorted(sink) == list(range(m.n_layers))
        masks = [_hip_lrelu_masks(sink[i], 1, T, B * N)[0] for i in range(m.n_layers)]
        for i, (mk, y) in enumerate(zip(masks, ys)):
            flip = mk != (y > 0)
            assert int(flip.sum()) <= 16, (i, int(flip.sum()))
            if flip.any():
                assert float(y[flip].abs().max()) <= 1e-5 * float(y.abs().max()), i   # at the kink
        _, p = f64(lrelu_masks=masks)
    for k, q in m.named_parameters():
        ref = p[k].grad
        if ref is None or float(ref.abs().max()) == 0:
            assert q.grad is None or float(q.grad.abs().max()) <= 1e-6, k
            continue
        check_rel(f"{name} grad {k}", q.grad, ref, TOL)


def test_egno_flat_training_step_updates_and_repacks():
    """Three optimizer steps (the reference loop's Adam) on a flat model: each forward sees the updated
    weights (re-packed blobs, forward and reverse), and the training forward (torch embedding, one
    autograd node per layer) equals the one-call eval forward."""
    B, N, T = 4, 20, 10
    m = _egno(FLAT["flat"], seed=51).train()
    inp = {k: _dev(v) for k, v in _egno_case(B, N, T, seed=52).items()}
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(3):
        opt.zero_grad()
        x, _, _ = _run(m, inp)
        loss = ((x - inp["x"].repeat(T, 1)) ** 2).mean()
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert all(np.isfinite(losses)) and losses[2] != losses[0]
    with torch.no_grad():
        xe, ve, he = _run(m.eval(), inp)
    xt, vt, ht = _run(m.train(), inp)
    for name, a, b in (("x", xt, xe), ("v", vt, ve), ("h", ht, he)):
        check_rel(f"train vs eval {name}", a.detach(), b.cpu().numpy(), 1e-6)


@pytest.mark.parametrize("name", sorted(FLAT))
@pytest.mark.parametrize("B,N", [(3, 7), (16, 20), (1, 37)])
def test_egno_flat_forward_matches_f64_oracle(name, B, N):
    """Ragged receiver tiles (B N T not a multiple of 16), N above one tile, every option pairing."""
    T = 10
    m = _egno(FLAT[name], seed=B + 2 * N).eval()
    case = _egno_case(B, N, T, seed=N + 3)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    f64 = {k: (v.astype(np.float64) if k not in ("row", "col", "t_out") else v) for k, v in case.items()}
    xr, vr, hr = oe.egno_forward(p, **f64, T=T, **FLAT[name])
    with torch.no_grad():
        x, v, h = _run(m, {k: _dev(val) for k, val in case.items()})
    check_rel("x", x.cpu(), xr, TOL)
    check_rel("v", v.cpu(), vr, TOL)
    check_rel("h", h.cpu(), hr, TOL)


def test_egno_flat_multi_input_matches_oracle():
    B, N, T, I = 2, 6, 10, 3
    m = _egno(FLAT["flat"], seed=23, num_inputs=I).eval()
    rng = np.random.default_rng(5)
    x = rng.standard_normal((I, B * N, 3)).astype(np.float32)
    v = rng.standard_normal((I, B * N, 3)).astype(np.float32) * 0.5
    lm = x.mean(1, keepdims=True).repeat(B * N, 1)
    h = np.concatenate([np.linalg.norm(v, axis=-1, keepdims=True), np.ones((I, B * N, 1), np.float32)], -1)
    row, col = tr.full_edges(B, N)
    ea = rng.standard_normal((I, B * N * (N - 1), 2)).astype(np.float32)
    t_in = np.tile(np.array([-2.0, -1.0, 0.0], np.float32), (B, 1))
    t_out = np.tile(np.arange(1, T + 1, dtype=np.float32), (B, 1))
    p = {k: q.detach().cpu().numpy().astype(np.float64) for k, q in m.state_dict().items()}
    d = lambda a: a.astype(np.float64)  # noqa: E731
    xr, vr, hr = oe.egno_forward_multi(p, d(x), d(h), row.numpy(), col.numpy(), d(ea), d(v), d(lm), t_in, t_out, T=T,
                                       flat=True)
    with torch.no_grad():
        xo, vo, ho = m(_dev(x), _dev(h), [_dev(row), _dev(col)], _dev(ea), v=_dev(v), loc_mean=_dev(lm),
                       timesteps_in=_dev(t_in), timesteps_out=_dev(t_out))
    check_rel("x", xo.cpu(), xr, TOL)
    check_rel("v", vo.cpu(), vr, TOL)
    check_rel("h", ho.cpu(), hr, TOL)


def test_egno_no_time_conv_rollout_first_segment_is_the_forward():
    """rollout_fn (main_simulation_simple_no.py:342-384) through the native driver with
    use_time_conv=False: segment 0 is exactly the model's forward."""
    B, N, T = 4, 20, 10
    m = _egno(OPTS["egno_notc"], seed=5).eval()
    case = _egno_case(B, N, T, seed=6)
    inp = {k: _dev(v) for k, v in case.items()}
    loc_p = inp["x"]
    with torch.no_grad():
        x, _, _ = _run(m, inp)
        t_full = _dev(np.tile(np.arange(1, 2 * T + 1), (B, 1)))
        preds, _, _ = pkg.harness.egno_rollout(m, inp["h"], loc_p, [inp["row"], inp["col"]], inp["v"],
                                               inp["edge_fea"][:, :1].contiguous(), inp["edge_fea"], None, N, 2, B,
                                               charges=inp["h"][:, 1:2].contiguous(), num_steps=T,
                                               timesteps_out=t_full)
    torch.cuda.synchronize()
    assert torch.equal(preds[:T].reshape(-1, 3), x)
    assert bool(torch.isfinite(preds).all())


def _rollout_case(B, N, T, seed):
    case = _egno_case(B, N, T, seed=seed)
    f64 = {k: (v.astype(np.float64) if v.dtype.kind == "f" else v) for k, v in case.items()}
    eo = case["edge_fea"][:, :1].copy()          # edge_attr_o = q_i q_j (prepare_inputs appends |x_i - x_j|^2)
    q = case["h"][:, 1:2].copy()                 # nodes = [|v|, q]
    return case, f64, eo, q


@pytest.mark.parametrize("name", ["flat", "flat_notc"])
def test_egno_flat_rollout_matches_oracle(name):
    """rollout_fn (main_simulation_simple_no.py:342-384, reachable with --flat through :231) on a
    flat=True model. The one-call native rollout runs the 64-wide SiLU layer kernels only, so a flat
    model rolls out segment by segment through its own forward (harness._egno_rollout_segments):
    segment 0 is bitwise the flat forward, both segments (restarting from per-sample frames t_in - 1)
    against the float64 oracle's rollout."""
    B, N, T = 4, 20, 10
    m = _egno(FLAT[name], seed=31).eval()
    case, f64, eo, q = _rollout_case(B, N, T, seed=32)
    inp = {k: _dev(v) for k, v in case.items()}
    t_full = np.tile(np.arange(1, 2 * T + 1), (B, 1))
    t_in = np.array([0, 3, 10, 7])
    with torch.no_grad():
        x, _, _ = _run(m, inp)
        preds, en, en_all = pkg.harness.egno_rollout(
            m, inp["h"], inp["x"], [inp["row"], inp["col"]], inp["v"], _dev(eo), inp["edge_fea"], inp["loc_mean"], N, 2,
            B, charges=_dev(q), num_steps=T, timesteps_in=_dev(t_in), timesteps_out=_dev(t_full),
            energy_dataset="charged")
    torch.cuda.synchronize()
    assert torch.equal(preds[:T].reshape(-1, 3), x)
    assert en.shape == (2, B, 1) and en_all.shape == (2 * T, B, 1)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    ref, ren, ren_all = oh.egno_rollout(p, f64["h"], f64["x"], case["row"], case["col"], f64["v"], eo.astype(np.float64),
                                        f64["edge_fea"], f64["loc_mean"], N, 2, B, q.astype(np.float64), T=T,
                                        t_out=t_full, t_in=t_in, **FLAT[name])
    check_rel("flat preds[:T]", preds[:T].cpu(), ref[:T], TOL)
    check_rel("flat preds", preds.cpu(), ref, 1e-4)     # segment 2 restarts from a random-init model's output
    check_rel("flat en_all[:T]", en_all[:T].cpu(), ren_all[:T], 1e-5)


def test_egno_segment_rollout_equals_native_rollout():
    """The segment-loop rollout (the flat models' path) and the one-call native rollout compute the same
    trajectories and energies on a standard model: same forward kernels, same featurisation kernel."""
    B, N, T = 5, 20, 10
    m = _egno({}, seed=33).eval()
    case, _, eo, q = _rollout_case(B, N, T, seed=34)
    inp = {k: _dev(v) for k, v in case.items()}
    args = (m, inp["h"], inp["x"], [inp["row"], inp["col"]], inp["v"], _dev(eo), inp["edge_fea"], inp["loc_mean"], N,
            3, B)
    t_full = _dev(np.tile(np.arange(1, 3 * T + 1), (B, 1)))
    t_in = _dev(np.array([0, 3, 10, 7, 1]))
    with torch.no_grad():
        a = pkg.harness.egno_rollout(*args, charges=_dev(q), num_steps=T, timesteps_in=t_in, timesteps_out=t_full,
                                     energy_dataset="charged")
        b = pkg.harness._egno_rollout_segments(*args, _dev(q), t_in, t_full, "charged")
    torch.cuda.synchronize()
    for name, u, w in zip(("preds", "energies", "energies_allsteps"), a, b):
        assert u.shape == w.shape, name
        check_rel(f"segments vs native {name}", w.cpu(), u.cpu().numpy(), 1e-6)


@pytest.mark.parametrize("B,N,T", [(2, 5, 10), (16, 20, 10)])
def test_segno_tanh_matches_golden_and_f64(B, N, T):
    fx = load_golden("segno_tanh")
    torch.manual_seed(4)
    m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True, tanh=True, norm_diff=True,
                  device=DEV)
    if (B, N) == (int(fx["cfg::B"]), int(fx["cfg::N"])):
        m.load_state_dict({k: torch.tensor(v) for k, v in params_of(fx).items()})
        his, x, v, ea = (torch.tensor(fx[k]) for k in ("in::his", "in::x", "in::v", "in::edge_attr"))
        r, c = torch.tensor(fx["in::row"]), torch.tensor(fx["in::col"])
        target = torch.tensor(fx["in::loc_end"])
    else:
        g = torch.Generator().manual_seed(B)
        x = torch.randn(B * N, 3, generator=g) * 1.5
        v = torch.randn(B * N, 3, generator=g) * 0.5
        q = torch.randint(0, 2, (B * N, 1), generator=g).float() * 2 - 1
        r, c = tr.full_edges(B, N)
        ea = torch.cat([q[r] * q[c], ((x[r] - x[c]) ** 2).sum(1, keepdim=True)], 1)
        his = v.norm(dim=1, keepdim=True)
        target = x + 0.3 * v
    m.train()
    m.zero_grad(set_to_none=True)
    xo, ho, vo = m(_dev(his), _dev(x), [_dev(r), _dev(c)], _dev(v), _dev(ea), T=T)
    loss = torch.nn.functional.mse_loss(xo, _dev(target))
    loss.backward()
    torch.cuda.synchronize()
    dt = torch.float64
    p = {k: q.detach().cpu().to(dt).requires_grad_(True) for k, q in m.state_dict().items()}
    xr, hr, vr = tr.segno_forward_step(p, his.to(dt), x.to(dt), r, c, v.to(dt), ea.to(dt), T=T, dense_mean=False,
                                       tanh=True)
    lr = torch.nn.functional.mse_loss(xr, target.to(dt))
    lr.backward()
    check_rel("x", xo, xr.detach(), TOL)
    check_rel("h", ho, hr.detach(), TOL)
    check_rel("v", vo, vr.detach(), TOL)
    if (B, N) == (int(fx["cfg::B"]), int(fx["cfg::N"])):
        check_rel("x vs reference", xo, fx["out::x"], TOL)
        assert abs(float(loss.detach()) - float(fx["out::loss"])) <= 1e-5 * abs(float(fx["out::loss"]))
    n = 0
    for k, q in m.named_parameters():
        ref = p[k].grad
        if ref is None or float(ref.abs().max()) == 0:
            assert q.grad is None or float(q.grad.abs().max()) == 0, k
            continue
        n += 1
        check_rel(f"tanh grad {k}", q.grad, ref, TOL)
        if (B, N) == (int(fx["cfg::B"]), int(fx["cfg::N"])):
            check_rel(f"tanh grad {k} vs reference", q.grad, fx["grad::" + k], TOL)
    assert n == 14
