"""Reference constructor options beyond the BASELINE configs (CPU only): EGNO norm=True
(basic.py:140-141), EGNO use_time_conv=False (egno.py:27-33, 99-107), EGNO with_v=False
(basic.py:156-160, 180-183), SEGNO tanh=True / norm_diff=True (gcl.py:32-63).

Pins the seeded constructors, the numpy oracle and the torch restatement to fixtures recorded from
the reference itself (tests/golden/make_golden.py options -> egno_norm / egno_notc / segno_tanh).
The GPU side is tests/test_gpu_options.py."""
import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg
from oracle import egno as oe
from oracle import segno as osg
from oracle import torch_ref as tr
from tests.conftest import load_golden, maxnorm_rel, params_of

EGNO_CASES = [("egno_norm", 2, dict(norm=True)), ("egno_notc", 3, dict(use_time_conv=False)),
              ("egno_flat", 5, dict(flat=True))]


def _egno(seed, **opts):
    torch.manual_seed(seed)
    return pkg.EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                    num_timesteps=10, time_emb_dim=32, **opts)


def _same_state(m, fx):
    sd = m.state_dict()
    ref = params_of(fx)
    assert list(sd.keys()) == list(ref.keys())   # registration order
    for k in ref:
        assert np.array_equal(sd[k].numpy(), ref[k]), k   # RNG consumption order


@pytest.mark.parametrize("name,seed,opts", EGNO_CASES)
def test_egno_option_seeded_init_matches_reference(name, seed, opts):
    _same_state(_egno(seed, **opts), load_golden(name))


def test_segno_tanh_seeded_init_matches_reference():
    torch.manual_seed(4)
    m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True, norm_diff=True, tanh=True)
    _same_state(m, load_golden("segno_tanh"))
    assert isinstance(m.module.coord_mlp[-1], torch.nn.Tanh)


def test_egno_norm_fixture_hits_the_eps_branch():
    """The fixture has two coincident nodes: their radial input is 0 < 1e-12, so F.normalize leaves
    0 there (1 elsewhere) -- both branches of s / max(s, eps) are exercised."""
    fx = load_golden("egno_norm")
    x = fx["in::x"]
    assert np.array_equal(x[0], x[1]) and np.array_equal(fx["in::v"][0], fx["in::v"][1])
    s = np.array([[0.0], [1e-13], [0.5], [3e20]], np.float32)
    assert np.array_equal(oe.radial_normalize(s)[:, 0], np.array([0.0, 0.1, 1.0, 1.0], np.float32))


@pytest.mark.parametrize("name,seed,opts", EGNO_CASES)
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_egno_option_oracle_forward_matches_reference(name, seed, opts, dtype):
    fx = load_golden(name)
    p = {k: v.astype(dtype) for k, v in params_of(fx).items()}
    c = lambda k: fx[k].astype(dtype)  # noqa: E731
    x, v, h = oe.egno_forward(p, c("in::x"), c("in::h"), fx["in::row"], fx["in::col"], c("in::edge_attr"),
                              c("in::v"), c("in::loc_mean"), fx["in::t_out"], T=int(fx["cfg::T"]), **opts)
    for got, k in ((x, "out::x"), (v, "out::v"), (h, "out::h")):
        assert maxnorm_rel(got, fx[k]) < 1e-5, k


@pytest.mark.parametrize("name,seed,opts", EGNO_CASES)
@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_egno_option_autograd_gradients_match_reference(name, seed, opts, dt):
    """One training step (main_simulation_simple_no.py:267-280) through torch autograd of the
    restatement, against the reference's own gradients."""
    fx = load_golden(name)
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    p = {k: torch.tensor(v, dtype=dt, requires_grad=True) for k, v in params_of(fx).items()}
    t = lambda k: torch.tensor(fx[k]).to(dt) if fx[k].dtype.kind == "f" else torch.tensor(fx[k])  # noqa: E731
    x, _, _ = tr.egno_forward(p, t("in::x"), t("in::h"), t("in::row"), t("in::col"), t("in::edge_attr"), t("in::v"),
                              t("in::loc_mean"), t("in::t_out"), T=T, **opts)
    loss = ((x.reshape(T, B, N, 3).permute(1, 2, 0, 3) - t("in::loc_true")) ** 2).mean((0, 1, 3)).mean()
    loss.backward()
    assert abs(float(loss.detach()) - float(fx["out::loss"])) <= 1e-6 * abs(float(fx["out::loss"]))
    n = 0
    for k, q in p.items():
        ref = fx["grad::" + k]
        if np.abs(ref).max() == 0:
            assert q.grad is None or float(q.grad.abs().max()) == 0, k
            continue
        n += 1
        assert maxnorm_rel(q.grad.double().numpy(), ref) < 1e-5, (k, dt)
    assert n >= 16 * 4 - 4 + 2   # every layer parameter (the last node_net has no path to x) + embedding


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_segno_tanh_forward_and_gradients_match_reference(dt):
    fx = load_golden("segno_tanh")
    T = int(fx["cfg::T"])
    c = lambda k: fx[k].astype(np.float64)  # noqa: E731
    p64 = {k: v.astype(np.float64) for k, v in params_of(fx).items()}
    h = c("in::his") @ p64["embedding.weight"].T + p64["embedding.bias"]
    xo, ho, vo = osg.forward_step(p64, h, c("in::x"), fx["in::row"], fx["in::col"], c("in::v"), c("in::edge_attr"),
                                  T=T, tanh=True)
    for got, k in ((xo, "out::x"), (ho, "out::h"), (vo, "out::v")):
        assert maxnorm_rel(got, fx[k]) < 1e-5, k
    p = {k: torch.tensor(v, dtype=dt, requires_grad=True) for k, v in params_of(fx).items()}
    t = lambda k: torch.tensor(fx[k]).to(dt) if fx[k].dtype.kind == "f" else torch.tensor(fx[k])  # noqa: E731
    x, _, _ = tr.segno_forward_step(p, t("in::his"), t("in::x"), t("in::row"), t("in::col"), t("in::v"),
                                    t("in::edge_attr"), T=T, dense_mean=False, tanh=True)
    loss = torch.nn.functional.mse_loss(x, t("in::loc_end"))
    loss.backward()
    assert abs(float(loss.detach()) - float(fx["out::loss"])) <= 1e-6 * abs(float(fx["out::loss"]))
    n = 0
    for k, q in p.items():
        if "grad::" + k not in fx:
            assert q.grad is None or float(q.grad.abs().max()) == 0, k
            continue
        n += 1
        assert maxnorm_rel(q.grad.double().numpy(), fx["grad::" + k]) < 1e-5, (k, dt)
    assert n == 14


def test_egno_with_v_false_builds_reference_tree_and_cannot_run():
    """with_v=False: no node_v_net in the state_dict (basic.py:156-160) and, as in the reference
    (v.repeat at egno.py:95 / node_v_net(h) at basic.py:180-181), no usable forward."""
    torch.manual_seed(0)
    m = pkg.EGNO(n_layers=2, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=False, num_timesteps=10)
    assert not any("node_v_net" in k for k in m.state_dict())
    z = torch.zeros(10, 3)
    with pytest.raises(TypeError, match="with_v=False"):
        m(z, torch.zeros(10, 2), pkg.graph.full_edges(2, 5), torch.zeros(40, 2), v=z, loc_mean=z)


def test_egno_flat_training_is_device_only_and_packs_egno_layers_only():
    """flat=True (basic.py:38-40: every BaseMLP 4x wide with Tanh) builds the reference tree; its forward
    and training run on their own kernels (tests/test_gpu_options.py). On the CPU both stop at the device
    check; multi-input flat training is refused before any device work; the flat packers refuse SEGNO
    layers, unknown option bits and null pointers without touching the device."""
    m = _egno(0, flat=True)
    e = m.layers[0].edge_message_net.scalar_net.mlp
    assert e[0].weight.shape == (256, 2 * 64 + 1 + 2) and isinstance(e[1], torch.nn.Tanh)
    z = torch.zeros(10, 3)
    with pytest.raises(pkg._lib.NonodeError, match="no CPU path"):
        m.train()(z, torch.zeros(10, 2), pkg.graph.full_edges(2, 5), torch.zeros(40, 2), v=z, loc_mean=z)
    torch.manual_seed(0)
    mi = pkg.EGNO(n_layers=2, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_timesteps=10,
                  num_inputs=2, flat=True)
    with pytest.raises(NotImplementedError, match="num_inputs=1"):
        mi.train()(z[None].repeat(2, 1, 1), torch.zeros(2, 10, 2), pkg.graph.full_edges(2, 5),
                   torch.zeros(2, 40, 2), v=z[None].repeat(2, 1, 1), loc_mean=z[None].repeat(2, 1, 1))
    L = pkg._lib.lib()
    w = pkg._lib.LayerWeights(*([16] * 16))   # never dereferenced: the variant check fails first
    for variant in (pkg._lib.VARIANT_SEGNO, pkg._lib.VARIANT_EGNO | pkg._lib.LAYER_TANH_COORD):
        assert L.nonode_pack_layer_flat(w, variant, 64, 2, 16, None) == 1
    assert L.nonode_pack_layer_flat_bwd(w, 2, None, None) == 1
    assert L.nonode_flat_blob_floats() > L.nonode_layer_blob_floats()
    assert L.nonode_egnn_layer_flat_bwd(0, 5, 2, 1, *([None] * 14)) != 0


def test_pack_rejects_option_bits_of_the_other_variant():
    """NORM_RADIAL is an EGNO option and TANH_COORD a SEGNO one; unknown bits are refused (checked
    before any device work, so this runs without a GPU)."""
    L = pkg._lib.lib()
    w = pkg._lib.LayerWeights(*([16] * 16))   # never dereferenced: the option check fails first
    for pack in (L.nonode_pack_layer, L.nonode_pack_layer_bwd):
        for variant in (pkg._lib.VARIANT_SEGNO | pkg._lib.LAYER_NORM_RADIAL,
                        pkg._lib.VARIANT_EGNO | pkg._lib.LAYER_TANH_COORD, pkg._lib.VARIANT_EGNO | 0x400):
            assert pack(w, variant, 64, 2, 16, None) == 1
        assert b"option" in L.nonode_last_error()
