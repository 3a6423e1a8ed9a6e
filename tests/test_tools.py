"""Profiling helpers: rocprofv3 kernel names map to the right per-kernel traffic keys."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pmc_traffic_kernel_keys():
    k = _load("pmc_traffic").kernel_key
    assert k("void (anonymous namespace)::tconv_kernel<true, 2, 10>((anonymous namespace)::TconvArgs)") \
        == "tconv_kernel<first>"
    assert k("void (anonymous namespace)::tconv_kernel<false, 2, 10>((anonymous namespace)::TconvArgs)") \
        == "tconv_kernel"
    assert k("_ZN12_GLOBAL__N_112tconv_kernelILb1ELi2ELi10EEEvNS_9TconvArgsE") == "tconv_kernel<first>"
    assert k("void (anonymous namespace)::egnn_layer_kernel<0, 1, 4, true>(LayerArgs)") == "egnn_layer_kernel<EGNO>"
    assert k("void (anonymous namespace)::egnn_layer_kernel<1, 1, 4, true>(LayerArgs)") == "egnn_layer_kernel<SEGNO>"
    assert k("(anonymous namespace)::temb_kernel(int, int, int, int, float const*)") == "temb_kernel"
    assert k("__amd_rocclr_copyBuffer") is None
    assert k("(anonymous namespace)::node_wgrad_kernel(nonode_tu::NodeWgradArgs)") == "node_wgrad_kernel"
    assert k("void (anonymous namespace)::tconv_bwd_kernel<2>(nonode_tu::TconvBwdArgs)") == "tconv_bwd_kernel"
    assert k("void (anonymous namespace)::edge_bwd_kernel<2, 1>((anonymous namespace)::EdgeBwdArgs)") \
        == "edge_bwd_kernel<pass 1>"


def test_build_units_cover_every_source():
    """Every csrc/*.hip is one of build()'s translation units or is included by one (a source file that
    neither is would silently drop its kernels from libnonode.so)."""
    import re
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    csrc = os.path.join(ROOT, "no-node-comparison_amd", "csrc")
    units = [u[0] for u in g.UNITS]
    assert all(os.path.exists(os.path.join(csrc, u)) for u in units)
    included = set()
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h")):
            included |= set(re.findall(r'#include "([^"]+\.(?:hip|h))"', open(os.path.join(csrc, f)).read()))
    for f in os.listdir(csrc):
        if f.endswith(".hip"):
            assert f in units or f in included, f"{f} is neither a build unit nor included by one"
    # the shared headers exist and units differ in scheduler where DESIGN.md says so
    assert dict((u, s) for u, s, _ in g.UNITS)["nonode.hip"] == "iterative-ilp"
    assert dict((u, s) for u, s, _ in g.UNITS)["nonode_node.hip"] == ""


def test_inline_asm_mfma_blocks_are_padded():
    """Every inline-asm MFMA block of the built library's edge backward (pass A) keeps its wait-state
    pads (tools/isa_pads.py): round 4's first version, whose compiler-inserted v_accvgpr_mov copies
    read MFMA results too early and gave 0.2-1.0 relative gradient errors on the GPU only, fails here."""
    import pytest
    t = _load("isa_pads")
    lib = os.path.join(ROOT, "no-node-comparison_amd", "libnonode.so")
    if not os.path.exists(lib):
        pytest.skip("libnonode.so not built")
    res = t.check_library(lib)
    assert len(res) == 5   # edge_bwd_kernel<NE, 0>, NE = 0..4
    for name, (n, bad) in res.items():
        assert n >= 48, name   # at least the pair loop's four amfma32_block statements
        assert not bad, (name, bad[:3])


def test_isa_pad_checker_catches_the_round4_failure():
    t = _load("isa_pads")
    blk = [("s_nop", ["1"])] + [("v_mfma_f32_16x16x32_f16", [f"a[{4 * k}:{4 * k + 3}]", "v[0:3]", "v[4:7]",
                                                               f"a[{4 * k}:{4 * k + 3}]"]) for k in range(4)]
    good = blk + [("s_nop", ["11"]), ("v_accvgpr_mov_b32", ["a20", "a1"])]
    assert t.check_function(good) == (4, [])
    # one statement per MFMA, no trailing pad: the compiler's copy reads a result 3 states later
    n, bad = t.check_function(blk + [("v_accvgpr_mov_b32", ["a20", "a1"])])
    assert n == 4 and bad and "v_accvgpr_mov_b32" in bad[0]
    # a fresh VALU write of an MFMA operand right before the block, without the leading pad
    n, bad = t.check_function([("v_cvt_f16_f32", ["v5", "v9"])] + blk[1:] + [("s_nop", ["11"])])
    assert bad and "wrote 0 wait states before" in bad[0]
