"""CPU tests: the C-ABI library loads and exports include/nonode.h; host-side logic of the drop-in
modules (state_dict keys, RNG-order init parity, graph validation, no CPU fallback)."""
import os
import re
import subprocess

import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg
from no_node_comparison_amd import _lib
from oracle import harness as oh
from tests.conftest import ROOT, load_golden


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "nonode.h")).read()
    return sorted(set(re.findall(r"^(?:const char\*|size_t|int)\s+(nonode_[a-z0-9_]+)\(", src, re.M)))


def test_library_exports_every_header_symbol():
    L = pkg.lib()
    declared = _header_symbols()
    assert declared == sorted(_lib.SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (nonode_[a-z0-9_]+)", out))
    assert set(declared) <= exported
    for s in declared:
        assert hasattr(L, s)
    assert b"gfx950" in L.nonode_version()


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob       # the embedded offload bundle targets gfx950
    assert b"egnn_layer_kernel" in blob


def test_size_queries_need_no_gpu():
    L = pkg.lib()
    assert L.nonode_layer_blob_floats() == 33856 + 8192 + 6 * 4096
    B, N, T = 512, 20, 10
    ws = L.nonode_egno_workspace_bytes(B, N, T, B)
    assert ws == (B * N * T * 67 + B * T * 64 + 64) * 4
    assert L.nonode_segno_workspace_bytes(B, N) == (3 * B * N * 64 + 12 * B * N + 64) * 4


def test_status_codes_and_last_error():
    L = pkg.lib()
    # invalid shapes are rejected before any HIP call
    rc = L.nonode_egnn_layer(0, 0, 20, 2, 1, None, None, None, None, None, 0.0, 1.0, 0, None, None, None, None)
    assert rc == 3
    assert b"n_graphs=0" in L.nonode_last_error()
    rc = L.nonode_egno_tconv(10, 40, 2, *([None] * 10))
    assert rc == 3
    with pytest.raises(pkg.NonodeError):
        _lib.check(rc)


@pytest.mark.parametrize("entry", ["nonode_pack_layers", "nonode_pack_layers_bwd"])
def test_batched_pack_validates_every_layer_before_any_launch(entry):
    """A null weight pointer in layer 9 (the second PACK_MAX chunk) fails the batched call before any
    kernel launch: here, with no GPU, an earlier launch of layers 0-7 would fail as a launch error
    instead (the pointers are fake and never dereferenced on the host)."""
    import ctypes
    L = pkg.lib()
    nl = 10

    def fake(i):
        w = _lib.LayerWeights()
        for name, _ in _lib.LayerWeights._fields_:
            setattr(w, name, 0x1000 + 64 * i)
        return w

    ws = [fake(i) for i in range(nl)]
    WP = ctypes.POINTER(_lib.LayerWeights)
    blobs = (ctypes.c_void_p * nl)(*[0x100000 + 4096 * i for i in range(nl)])
    fn = getattr(L, entry)
    for field in ("edge_w1", "coord_b2", "node_w2"):
        bad = fake(9)
        setattr(bad, field, None)
        arr = (WP * nl)(*[ctypes.pointer(w) for w in ws[:9]], ctypes.pointer(bad))
        rc = fn(arr, nl, 0, 64, 2, blobs, None)
        assert rc != 0
        assert b"missing weight pointer" in L.nonode_last_error()


def _egno_ctor(**kw):
    args = dict(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                num_timesteps=10, time_emb_dim=32)
    args.update(kw)
    return pkg.EGNO(**args)


def test_egno_state_dict_and_seeded_init_match_reference():
    ref = load_golden("init_seed0")
    torch.manual_seed(0)
    m = _egno_ctor()
    sd = m.state_dict()
    keys = [k[len("egno::"):] for k in ref if k.startswith("egno::")]
    assert list(sd.keys()) == keys               # same keys, same registration order
    for k in keys:
        assert np.array_equal(sd[k].numpy(), ref["egno::" + k]), k   # same RNG consumption order


def test_segno_state_dict_and_seeded_init_match_reference():
    ref = load_golden("init_seed0")
    torch.manual_seed(0)
    m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True, norm_diff=False,
                  tanh=False)
    sd = m.state_dict()
    keys = [k[len("segno::"):] for k in ref if k.startswith("segno::")]
    assert list(sd.keys()) == keys
    for k in keys:
        assert np.array_equal(sd[k].numpy(), ref["segno::" + k]), k


def test_reference_checkpoint_loads():
    fx = load_golden("egno_fwd")
    m = _egno_ctor()
    m.load_state_dict({k[3:]: torch.tensor(v) for k, v in fx.items() if k.startswith("w::")})
    s = load_golden("segno_fwd")
    m2 = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True)
    m2.load_state_dict({k[3:]: torch.tensor(v) for k, v in s.items() if k.startswith("w::")})


def test_unsupported_configs_raise():
    with pytest.raises(NotImplementedError):
        _egno_ctor(num_inputs=0)
    with pytest.raises(NotImplementedError):
        _egno_ctor(hidden_nf=32)
    # num_inputs > 1 is supported (inference): the embedding takes both time embeddings (egno.py:12-16)
    assert _egno_ctor(num_inputs=3).embedding.weight.shape == (64, 2 + 2 * 32)
    _egno_ctor(flat=True)   # flat=True: forward and single-input training (tests/test_options.py)
    with pytest.raises(NotImplementedError):
        pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=32)
    with pytest.raises(ValueError):
        pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, multiple_agg="max")


def test_segno_train_mode_has_no_cpu_path():
    """Training goes through the HIP reverse pass (autograd.SEGNOStepTrain); on CPU tensors both
    the training and the inference path stop at the device check (no silent CPU fallback)."""
    m = pkg.SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True).train()
    z = torch.zeros(20, 3)
    with pytest.raises(pkg.NonodeError, match="no CPU path"):
        m(torch.zeros(20, 1), z, pkg.graph.full_edges(1, 20), z, torch.zeros(380, 2), T=10)
    with pytest.raises(pkg.NonodeError, match="no CPU path"):
        with torch.no_grad():
            m(torch.zeros(20, 1), z, pkg.graph.full_edges(1, 20), z, torch.zeros(380, 2), T=10)
    assert [n for n in m.gcl_param_names() if n] == [k for k, _ in m.module.named_parameters(prefix="module")
                                                      if "coord_mlp_vel" not in k and "node_mlp" not in k] + \
        [k for k, _ in m.module.named_parameters(prefix="module") if "node_mlp" in k]


def test_no_cpu_fallback():
    fx = load_golden("egno_fwd")
    m = _egno_ctor()
    g = lambda k: torch.tensor(fx[k])  # noqa: E731
    with pytest.raises(pkg.NonodeError, match="no CPU path"):
        with torch.no_grad():
            m(g("in::x"), g("in::h"), [g("in::row"), g("in::col")], g("in::edge_attr"), v=g("in::v"),
              loc_mean=g("in::loc_mean"), timesteps_out=g("in::t_out"))


@pytest.mark.parametrize("B,N", [(1, 2), (3, 5), (4, 20), (2, 100)])
def test_full_edges_match_dataset_order(B, N):
    r, c = pkg.graph.full_edges(B, N)
    ro, co = oh.full_edges(B, N)
    assert np.array_equal(r.numpy(), ro) and np.array_equal(c.numpy(), co)
    assert pkg.graph.check_full_graph([r, c], B * N) == (B, N)
    assert pkg.graph.check_full_graph(torch.stack([r, c]), B * N) == (B, N)


def test_check_full_graph_rejects_other_topologies():
    r, c = pkg.graph.full_edges(2, 5)
    with pytest.raises(ValueError):
        pkg.graph.check_full_graph([c, r], 10)          # swapped receiver/sender
    with pytest.raises(ValueError):
        pkg.graph.check_full_graph([r[:-1], c[:-1]], 10)  # ragged
    rr = r.clone()
    rr[7] = 0                                        # edge (1, 3) rewired to receiver 0
    with pytest.raises(ValueError):
        pkg.graph.check_full_graph([rr, c], 10)


def test_harness_has_no_cpu_path():
    """The rollout callers run as HIP kernels only: CPU tensors raise."""
    fx = load_golden("egno_fwd")
    B, N = int(fx["cfg::B"]), int(fx["cfg::N"])
    edges = pkg.harness.get_edges(B, N)
    with pytest.raises(pkg.NonodeError):
        pkg.harness.prepare_inputs(torch.tensor(fx["raw::loc"]), torch.tensor(fx["raw::vel"]),
                                   torch.tensor(fx["raw::edge_attr_o"]), edges, N, 1, torch.tensor(fx["raw::charges"]))
    with pytest.raises(pkg.NonodeError):
        pkg.harness.conserved_energy("charged", torch.zeros(B * N, 3), torch.zeros(B * N, 3), torch.ones(B * N), B)


def test_edge_check_cache_is_not_fooled_by_reused_memory():
    """A validated edge list is cached; a different list later allocated at the same address must
    still be checked (the cache keeps its tensors alive, so addresses cannot be recycled)."""
    from no_node_comparison_amd.graph import check_full_graph, full_edges
    for _ in range(20):
        r, c = full_edges(3, 5)
        assert check_full_graph([r.clone(), c.clone()], 15) == (3, 5)
        with pytest.raises(ValueError):
            check_full_graph([c.clone(), r.clone()], 15)
