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
