"""GPU parity of the layer-granular reverse entry points (SURVEY §8(b) egno_layer_bwd /
spectral_tconv_bwd), called through the C ABI: nonode_egnn_layer_bwd for one EGNN_Layer
(basic.py:167-186) and nonode_egno_tconv_bwd for one TimeConv + TimeConv_x (layer_no.py:80-178,
egno.py:99-108), against the reference's own autograd of those blocks in the training step of
tests/golden/egno_grad.npz (tests/golden/egno_layer_grads.npz, recorded by wrapping the reference
modules' forwards). Bar: 1e-5 max-norm relative per tensor (as the whole-model gradients).
"""
import ctypes

import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg
from no_node_comparison_amd import _lib
from oracle import egno_grad as og
from tests.conftest import check_rel, load_golden, params_of
from tests.test_gpu_parity import DEV, _dev, _egno, _egno_case, _sd_np

pytestmark = pytest.mark.gpu
GTOL = 1e-5


def _model():
    return _egno(params_of(load_golden("egno_fwd")))


@pytest.mark.parametrize("i", [1, 3])
def test_egnn_layer_bwd_matches_reference_layer_autograd(i):
    lg = load_golden("egno_layer_grads")
    m = _model()
    L = pkg.lib()
    B, N, T = int(lg["cfg::B"]), int(lg["cfg::N"]), int(lg["cfg::T"])
    n_graphs = T * B
    x, h, ef, v = (_dev(lg[f"lay{i}::in{j}"]) for j in range(4))
    gxo, gvo, gho = (_dev(lg[f"lay{i}::gout{j}"]) for j in range(3))
    blobs, _ = m._packed()
    bblobs = m._packed_bwd()
    names = m.layer_param_names(i)
    grads = {nm: torch.empty_like(dict(m.named_parameters())[nm]) for nm in names}
    lgs = _lib.LayerGrads(*[grads[nm].data_ptr() for nm in names])
    ghi, gxi, gvi = torch.empty_like(h), torch.empty_like(x), torch.empty_like(v)
    ws_bytes = L.nonode_egnn_layer_bwd_workspace_bytes(n_graphs, N)
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=DEV)
    P = _lib.ptr
    _lib.check(L.nonode_egnn_layer_bwd(_lib.VARIANT_EGNO, n_graphs, N, 2, n_graphs, P(h), P(x), P(v), P(ef),
                                       P(blobs[i]), P(bblobs[i]), P(gxo), P(gvo), P(gho), ctypes.byref(lgs), P(ghi),
                                       P(gxi), P(gvi), P(ws), ws_bytes, _lib.stream_of(x)))
    torch.cuda.synchronize()
    for nm in names:
        ref = lg["grad::" + nm]
        if np.abs(ref).max() == 0:
            assert float(grads[nm].abs().max()) == 0, nm
            continue
        check_rel(f"layer {i} grad {nm}", grads[nm], ref, GTOL)
    check_rel(f"layer {i} dL/dx_in", gxi, lg[f"lay{i}::gin0"], GTOL)
    check_rel(f"layer {i} dL/dh_in", ghi, lg[f"lay{i}::gin1"], GTOL)
    check_rel(f"layer {i} dL/dv_in", gvi, lg[f"lay{i}::gin3"], GTOL)


@pytest.mark.parametrize("i", [1, 3])
def test_egno_tconv_bwd_matches_reference_block_autograd(i):
    lg = load_golden("egno_layer_grads")
    fx = load_golden("egno_fwd")
    m = _model()
    L = pkg.lib()
    T = int(lg["cfg::T"])
    h = lg[f"tc{i}::in0"]                       # [T, BN, 64]
    X = lg[f"tcx{i}::in0"]                      # [T, BN, 3, 2] = (x - loc_mean, v)
    BN = h.shape[1]
    lm = fx["in::loc_mean"]                     # [BN, 3]
    x = X[..., 0] + lm[None]
    gX = lg[f"tcx{i}::gout0"]
    _, tblobs = m._packed()
    tw = m.time_conv_modules[i].t_conv.weights1.detach().contiguous()
    txw = m.time_conv_x_modules[i].t_conv.weights1.detach().contiguous()
    dh, dx, dv = (_dev(a) for a in (h.reshape(T * BN, 64), x.reshape(T * BN, 3), X[..., 1].reshape(T * BN, 3)))
    dgh = _dev(lg[f"tc{i}::gout0"].reshape(T * BN, 64))
    dgx, dgv = _dev(gX[..., 0].reshape(T * BN, 3)), _dev(gX[..., 1].reshape(T * BN, 3))
    ghi, gxi, gvi = torch.empty_like(dh), torch.empty_like(dx), torch.empty_like(dv)
    gtw, gtxw = torch.empty_like(tw), torch.empty_like(txw)
    dlm = _dev(lm)
    ws_bytes = L.nonode_egno_tconv_bwd_workspace_bytes(BN, T, m.num_modes)
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=DEV)
    P = _lib.ptr
    _lib.check(L.nonode_egno_tconv_bwd(BN, T, m.num_modes, P(dh), P(dx), P(dv), P(dlm), P(tblobs[i]), P(tw),
                                       P(txw), P(dgh), P(dgx), P(dgv), P(ghi), P(gxi), P(gvi), P(gtw), P(gtxw), P(ws),
                                       ws_bytes, _lib.stream_of(dh)))
    torch.cuda.synchronize()
    check_rel(f"tconv {i} grad weights1", gtw, lg[f"grad::time_conv_modules.{i}.t_conv.weights1"], GTOL)
    check_rel(f"tconv_x {i} grad weights1", gtxw, lg[f"grad::time_conv_x_modules.{i}.t_conv.weights1"], GTOL)
    check_rel(f"tconv {i} dL/dh_in", ghi, lg[f"tc{i}::gin0"].reshape(T * BN, 64), GTOL)
    gXi = lg[f"tcx{i}::gin0"]
    check_rel(f"tconv_x {i} dL/dx_in", gxi, gXi[..., 0].reshape(T * BN, 3), GTOL)
    check_rel(f"tconv_x {i} dL/dv_in", gvi, gXi[..., 1].reshape(T * BN, 3), GTOL)


def _layer_bwd(m, i, n_graphs, N, h, x, v, ef, gxo, gvo, gho):
    L = pkg.lib()
    blobs, _ = m._packed()
    bblobs = m._packed_bwd()
    names = m.layer_param_names(i)
    grads = {nm: torch.empty_like(dict(m.named_parameters())[nm]) for nm in names}
    lgs = _lib.LayerGrads(*[grads[nm].data_ptr() for nm in names])
    ghi, gxi, gvi = torch.empty_like(h), torch.empty_like(x), torch.empty_like(v)
    ws_bytes = L.nonode_egnn_layer_bwd_workspace_bytes(n_graphs, N)
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=DEV)
    P = _lib.ptr
    _lib.check(L.nonode_egnn_layer_bwd(_lib.VARIANT_EGNO, n_graphs, N, 2, n_graphs, P(h), P(x), P(v), P(ef),
                                       P(blobs[i]), P(bblobs[i]), P(gxo), P(gvo), P(gho), ctypes.byref(lgs), P(ghi),
                                       P(gxi), P(gvi), P(ws), ws_bytes, _lib.stream_of(x)))
    torch.cuda.synchronize()
    return grads, ghi, gxi, gvi


@pytest.mark.parametrize("N", [26, 31, 64, 100, 115])
def test_egnn_layer_bwd_large_n_matches_float64_oracle(N):
    """The layer entry point up to the top of the training range (N <= 115, set by pass A's LDS tables;
    N > 31 takes pass B's large-N form), against the float64 reverse pass of oracle/egno_grad.py
    (basic.py:167-186)."""
    B, i = 3, 2
    c = _egno_case(B, N, 10, seed=N)
    m = _egno(T=10, seed=N)
    rng = np.random.default_rng(N)
    h = rng.standard_normal((B * N, 64)) * 0.7
    gxo, gvo, gho = (rng.standard_normal(s) * 1e-3 for s in ((B * N, 3), (B * N, 3), (B * N, 64)))
    grads, ghi, gxi, gvi = _layer_bwd(m, i, B, N, _dev(h.astype(np.float32)), _dev(c["x"]), _dev(c["v"]),
                                      _dev(c["edge_fea"]), *(_dev(a.astype(np.float32)) for a in (gxo, gvo, gho)))
    p = _sd_np(m)
    f64 = lambda a: np.asarray(a, np.float64)  # noqa: E731
    h32 = f64(h.astype(np.float32))
    _, _, _, cache = og.egnn_layer_fwd(p, f"layers.{i}", f64(c["x"]), h32, c["row"], c["col"], f64(c["edge_fea"]),
                                       f64(c["v"]))
    rg = {}
    gx, gh, gv, _ = og.egnn_layer_bwd(p, f"layers.{i}", cache, *(f64(a.astype(np.float32)) for a in (gxo, gvo, gho)),
                                      rg)
    for nm in m.layer_param_names(i):
        check_rel(f"N={N} grad {nm}", grads[nm], rg[nm], GTOL)
    check_rel(f"N={N} dL/dx_in", gxi, gx, GTOL)
    check_rel(f"N={N} dL/dh_in", ghi, gh, GTOL)
    check_rel(f"N={N} dL/dv_in", gvi, gv, GTOL)


def test_layer_bwd_rejects_n_beyond_the_tables_before_any_launch():
    L = pkg.lib()
    lg = _lib.LayerGrads()
    t = torch.zeros(16, device=DEV)
    P = _lib.ptr
    N = 116
    ws = L.nonode_egnn_layer_bwd_workspace_bytes(2, N)
    rc = L.nonode_egnn_layer_bwd(_lib.VARIANT_EGNO, 2, N, 2, 2, *([P(t)] * 9), ctypes.byref(lg), P(t), P(t), P(t),
                                 P(t), ws, _lib.stream_of(t))
    assert rc != 0 and b"egnn_layer_bwd: N=116 too large" in L.nonode_last_error()


def test_layer_bwd_rejects_segno_and_small_workspace():
    L = pkg.lib()
    lg = _lib.LayerGrads()
    z = ctypes.c_void_p(0)
    rc = L.nonode_egnn_layer_bwd(_lib.VARIANT_SEGNO, 2, 5, 2, 2, *([z] * 9), ctypes.byref(lg), z, z, z, z, 0, z)
    assert rc != 0 and b"EGNO" in L.nonode_last_error()
    t = torch.zeros(16, device=DEV)
    P = _lib.ptr
    rc = L.nonode_egnn_layer_bwd(_lib.VARIANT_EGNO, 2, 5, 2, 2, *([P(t)] * 9), ctypes.byref(lg), P(t), P(t), P(t), P(t),
                                 64, _lib.stream_of(t))
    assert rc != 0 and b"workspace" in L.nonode_last_error()
