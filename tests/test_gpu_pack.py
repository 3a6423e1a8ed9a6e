"""The batched pack entry points (nonode_pack_layers / nonode_pack_layers_bwd / nonode_pack_tconvs, one
launch for every layer) give the per-layer entry points' blobs bitwise (include/nonode.h)."""
import ctypes

import pytest
import torch

import no_node_comparison_amd as pkg
from no_node_comparison_amd import _lib
from tests.test_gpu_parity import _egno

pytestmark = pytest.mark.gpu


def test_batched_packs_equal_per_layer_packs():
    m = _egno(T=10, modes=2, seed=7)
    L = _lib.lib()
    dev = m.embedding.weight.device
    nl = m.n_layers
    ws = [layer.weight_struct() for layer in m.layers]
    WP = ctypes.POINTER(_lib.LayerWeights)
    P = ctypes.c_void_p * nl
    for batched, single, floats in ((L.nonode_pack_layers, L.nonode_pack_layer, L.nonode_layer_blob_floats()),
                                    (L.nonode_pack_layers_bwd, L.nonode_pack_layer_bwd, L.nonode_bwd_blob_floats())):
        a = torch.full((nl, floats), float("nan"), device=dev)
        b = torch.full((nl, floats), float("nan"), device=dev)
        _lib.check(batched((WP * nl)(*[ctypes.pointer(w) for w in ws]), nl, m._pack_variant(), m.hidden_nf,
                           m.in_edge_nf, P(*[a[i].data_ptr() for i in range(nl)]), _lib.stream_of(a)))
        for i, w in enumerate(ws):
            _lib.check(single(ctypes.byref(w), m._pack_variant(), m.hidden_nf, m.in_edge_nf, _lib.ptr(b[i]), _lib.stream_of(a)))
        torch.cuda.synchronize()
        assert torch.equal(a.isnan(), b.isnan()) and torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))
    n = L.nonode_tconv_blob_floats(m.num_modes)
    tws = [mod.t_conv.weights1.detach().float().contiguous() for mod in m.time_conv_modules]
    a = torch.zeros(nl, n, device=dev)
    b = torch.zeros(nl, n, device=dev)
    _lib.check(L.nonode_pack_tconvs(P(*[t.data_ptr() for t in tws]), nl, m.num_modes, m.num_timesteps,
                                    P(*[a[i].data_ptr() for i in range(nl)]), _lib.stream_of(a)))
    for i, t in enumerate(tws):
        _lib.check(L.nonode_pack_tconv(_lib.ptr(t), m.num_modes, m.num_timesteps, _lib.ptr(b[i]), _lib.stream_of(a)))
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    # the batched entry validates every layer: a null weight pointer in layer 2 fails the call
    ws[2].edge_w1 = None
    for entry in (L.nonode_pack_layers, L.nonode_pack_layers_bwd):
        with pytest.raises(_lib.NonodeError, match="missing weight pointer"):
            _lib.check(entry((WP * nl)(*[ctypes.pointer(w) for w in ws]), nl, m._pack_variant(),
                             m.hidden_nf, m.in_edge_nf, P(*[a[i].data_ptr() for i in range(nl)]), _lib.stream_of(a)))
