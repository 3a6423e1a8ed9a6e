"""ctypes binding of the C ABI in include/nonode.h (libnonode.so, built for gfx950).

This is the reference-side binding a Python caller needs. The product path has
no CPU fallback: if the library is missing or the tensors are not on a ROCm device, calls raise.
"""
import ctypes
import os
import weakref

import torch  # load torch's HIP runtime first so libnonode.so binds to the same libamdhip64

_HERE = os.path.dirname(os.path.abspath(__file__))
# NONODE_LIB selects an in-tree diagnostic build of the same sources (tools/stamp_build.sh)
LIB_PATH = os.environ.get("NONODE_LIB") or os.path.join(_HERE, "libnonode.so")

# every symbol include/nonode.h declares (tests check the .so exports exactly these)
SYMBOLS = (
    "nonode_version", "nonode_last_error", "nonode_layer_blob_floats", "nonode_pack_layer",
    "nonode_egno_workspace_bytes", "nonode_egno_forward", "nonode_egno_forward_frames", "nonode_segno_workspace_bytes",
    "nonode_flat_blob_floats", "nonode_pack_layer_flat", "nonode_egno_flat_workspace_bytes", "nonode_egno_forward_flat",
    "nonode_segno_forward_step", "nonode_egno_tconv", "nonode_egnn_layer", "nonode_profile_begin",
    "nonode_profile_end", "nonode_tconv_blob_floats", "nonode_pack_tconv",
    "nonode_bwd_blob_floats", "nonode_pack_layer_bwd", "nonode_egno_train_state_bytes",
    "nonode_egno_forward_train", "nonode_egno_backward_workspace_bytes", "nonode_egno_backward",
    "nonode_segno_train_state_bytes", "nonode_segno_forward_train", "nonode_segno_backward_workspace_bytes",
    "nonode_segno_backward", "nonode_gather_rows",
    "nonode_egno_forward_train_frames", "nonode_egno_backward_frames",
    "nonode_prepare_inputs", "nonode_energy", "nonode_egno_rollout_workspace_bytes", "nonode_egno_rollout",
    "nonode_segno_rollout_workspace_bytes", "nonode_segno_rollout", "nonode_sim_charged", "nonode_sim_gravity",
    "nonode_gather_batch", "nonode_rollout_metrics",
    "nonode_egnn_layer_bwd_workspace_bytes", "nonode_egnn_layer_bwd",
    "nonode_egno_tconv_bwd_workspace_bytes", "nonode_egno_tconv_bwd",
    "nonode_pack_layers", "nonode_pack_layers_bwd", "nonode_pack_tconvs",
    "nonode_embedding_forward", "nonode_embedding_backward_workspace_bytes", "nonode_embedding_backward",
    "nonode_full_edges", "nonode_check_full_edges", "nonode_poison_if_flagged",
    "nonode_egnn_layer_flat_state_floats", "nonode_egnn_layer_flat", "nonode_flat_bwd_blob_floats",
    "nonode_pack_layer_flat_bwd", "nonode_egnn_layer_flat_bwd_node_floats", "nonode_egnn_layer_flat_bwd_edge_floats",
    "nonode_egnn_layer_flat_bwd",
)

VARIANT_EGNO = 0
VARIANT_SEGNO = 1
# option bits OR-ed into the pack variant (nonode.h NONODE_LAYER_*)
LAYER_NORM_RADIAL = 0x100   # EGNO(norm=True), basic.py:140-141
LAYER_TANH_COORD = 0x200    # SEGNO(tanh=True), gcl.py:57-59
# profile_end() record kinds beyond the two layer variants (csrc/nonode.hip ProfScope)
PROF_TCONV, PROF_TCONV_FIRST, PROF_SIM_CHARGED, PROF_SIM_GRAVITY, PROF_EDGE_BWD0, PROF_EDGE_BWD1 = 2, 3, 4, 5, 6, 7

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t


class NonodeError(RuntimeError):
    """A nonzero nonode_status, or the HIP extension is unavailable."""


class LayerWeights(ctypes.Structure):
    """nonode_layer_weights."""
    _fields_ = [(n, _vp) for n in (
        "edge_w1", "edge_b1", "edge_w2", "edge_b2", "coord_w1", "coord_b1", "coord_w2", "coord_b2",
        "vel_w1", "vel_b1", "vel_w2", "vel_b2", "node_w1", "node_b1", "node_w2", "node_b2")]


class LayerGrads(ctypes.Structure):
    """nonode_layer_grads (same fields as LayerWeights, written by nonode_egno_backward)."""
    _fields_ = LayerWeights._fields_


_lib = None
_packed_modules = weakref.WeakSet()
_step_hook = None
_param_gen = 0   # bumped whenever any module registers a parameter or a submodule (param_list)


def _bump_param_gen(*args):
    global _param_gen
    _param_gen += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_param_gen)
torch.nn.modules.module.register_module_module_registration_hook(_bump_param_gen)


def param_list(module, key, build):
    """The list build() returns (a module-tree traversal such as [p for l in layers for p in
    l.parameters()]), cached per module and key. The traversal was ~70% of the host time of a forward
    (tools/host_profile.py); the cache is rebuilt after any parameter or submodule registration anywhere
    (torch's global registration hooks), so a Parameter assigned to a module attribute is never missed."""
    cache = module.__dict__.setdefault("_nonode_plists", {})
    hit = cache.get(key)
    if hit is not None and hit[0] == _param_gen:
        return hit[1]
    lst = build()
    cache[key] = (_param_gen, lst)
    return lst


def track_packs(module):
    """Register a module whose packed weight blobs are cached under its parameters' tensor versions
    (EGNO._packed, SEGNO._packed, ...). torch's fused optimizers (Adam(fused=True) and the like)
    update parameters in place WITHOUT bumping those versions, so the key alone would keep stale
    blobs after such a step: a global optimizer step post-hook drops the packs of every tracked
    module that shares a parameter with the optimizer that stepped. module._drop_packs() does it."""
    global _step_hook
    _packed_modules.add(module)
    if _step_hook is None:
        import torch.optim.optimizer as topt
        _step_hook = topt.register_optimizer_step_post_hook(_after_optimizer_step)


def _after_optimizer_step(optimizer, args, kwargs):
    ids = {id(p) for g in optimizer.param_groups for p in g["params"]}
    for m in list(_packed_modules):
        if any(id(p) in ids for p in m.parameters()):
            m._drop_packs()


def lib():
    """Load libnonode.so once (raises NonodeError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NonodeError(f"HIP extension not built: {LIB_PATH} is missing "
                          "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    L = ctypes.CDLL(LIB_PATH)
    L.nonode_version.restype = ctypes.c_char_p
    L.nonode_last_error.restype = ctypes.c_char_p
    L.nonode_layer_blob_floats.restype = _sz
    L.nonode_pack_layer.argtypes = [ctypes.POINTER(LayerWeights), _i, _i, _i, _vp, _vp]
    L.nonode_pack_layers.argtypes = [ctypes.POINTER(ctypes.POINTER(LayerWeights)), _i, _i, _i, _i,
                                     ctypes.POINTER(_vp), _vp]
    L.nonode_pack_layers_bwd.argtypes = L.nonode_pack_layers.argtypes
    L.nonode_pack_tconvs.argtypes = [ctypes.POINTER(_vp), _i, _i, _i, ctypes.POINTER(_vp), _vp]
    L.nonode_egno_workspace_bytes.argtypes = [_i, _i, _i, _i]
    L.nonode_egno_workspace_bytes.restype = _sz
    L.nonode_egno_forward.argtypes = ([_i] * 9 + [_vp] * 8 + [ctypes.POINTER(_vp)] * 3 + [_vp] * 4
                                      + [_sz, _vp])
    L.nonode_egno_forward_frames.argtypes = ([_i] * 9 + [_vp] * 9 + [ctypes.POINTER(_vp)] * 3 + [_vp] * 4
                                             + [_sz, _vp])
    L.nonode_flat_blob_floats.restype = _sz
    L.nonode_pack_layer_flat.argtypes = [ctypes.POINTER(LayerWeights), _i, _i, _i, _vp, _vp]
    L.nonode_egno_flat_workspace_bytes.argtypes = [_i, _i, _i, _i]
    L.nonode_egno_flat_workspace_bytes.restype = _sz
    L.nonode_egno_forward_flat.argtypes = L.nonode_egno_forward_frames.argtypes
    L.nonode_segno_workspace_bytes.argtypes = [_i, _i]
    L.nonode_segno_workspace_bytes.restype = _sz
    L.nonode_segno_forward_step.argtypes = ([_i] * 5 + [_vp] * 8 + [_f, _i] + [_vp] * 4 + [_sz, _vp])
    L.nonode_egno_tconv.argtypes = [_i, _i, _i] + [_vp] * 10
    L.nonode_egnn_layer.argtypes = [_i] * 5 + [_vp] * 5 + [_f, _f, _i] + [_vp] * 4
    L.nonode_tconv_blob_floats.argtypes = [_i]
    L.nonode_tconv_blob_floats.restype = _sz
    L.nonode_pack_tconv.argtypes = [_vp, _i, _i, _vp, _vp]
    L.nonode_bwd_blob_floats.restype = _sz
    L.nonode_pack_layer_bwd.argtypes = [ctypes.POINTER(LayerWeights), _i, _i, _i, _vp, _vp]
    L.nonode_egno_train_state_bytes.argtypes = [_i] * 6
    L.nonode_egno_train_state_bytes.restype = _sz
    L.nonode_egno_forward_train.argtypes = ([_i] * 9 + [_vp] * 8 + [ctypes.POINTER(_vp)] * 3 + [_vp] * 4
                                            + [_sz, _vp, _sz, _vp])
    L.nonode_egno_forward_train_frames.argtypes = ([_i] * 9 + [_vp] * 9 + [ctypes.POINTER(_vp)] * 3 + [_vp] * 4
                                                   + [_sz, _vp, _sz, _vp])
    L.nonode_egno_backward_frames.argtypes = ([_i] * 10 + [_vp] * 2 + [ctypes.POINTER(_vp)] * 3 + [_vp] * 4
                                              + [ctypes.POINTER(LayerGrads), ctypes.POINTER(_vp),
                                                 ctypes.POINTER(_vp)] + [_vp] * 3 + [_sz, _vp])
    L.nonode_egno_backward_workspace_bytes.argtypes = [_i] * 4
    L.nonode_egno_backward_workspace_bytes.restype = _sz
    L.nonode_egno_backward.argtypes = ([_i] * 9 + [_vp] * 2 + [ctypes.POINTER(_vp)] * 3 + [_vp] * 4
                                       + [ctypes.POINTER(LayerGrads), ctypes.POINTER(_vp), ctypes.POINTER(_vp)]
                                       + [_vp] * 3 + [_sz, _vp])
    L.nonode_segno_train_state_bytes.argtypes = [_i] * 3
    L.nonode_segno_train_state_bytes.restype = _sz
    L.nonode_segno_forward_train.argtypes = [_i] * 4 + [_vp] * 5 + [_f, _i] + [_vp] * 4 + [_sz, _vp]
    L.nonode_segno_backward_workspace_bytes.argtypes = [_i] * 2
    L.nonode_segno_backward_workspace_bytes.restype = _sz
    L.nonode_segno_backward.argtypes = ([_i] * 4 + [_f, _i] + [_vp] * 6 + [ctypes.POINTER(LayerGrads)]
                                        + [_vp] * 4 + [_sz, _vp])
    L.nonode_embedding_forward.argtypes = [_i, _i] + [_vp] * 5
    L.nonode_embedding_backward_workspace_bytes.argtypes = [_i, _i]
    L.nonode_embedding_backward_workspace_bytes.restype = _sz
    L.nonode_embedding_backward.argtypes = [_i, _i] + [_vp] * 5 + [_sz, _vp]
    L.nonode_egnn_layer_bwd_workspace_bytes.argtypes = [_i, _i]
    L.nonode_egnn_layer_bwd_workspace_bytes.restype = _sz
    L.nonode_egnn_layer_bwd.argtypes = ([_i] * 5 + [_vp] * 9 + [ctypes.POINTER(LayerGrads)] + [_vp] * 4
                                        + [_sz, _vp])
    L.nonode_egno_tconv_bwd_workspace_bytes.argtypes = [_i] * 3
    L.nonode_egno_tconv_bwd_workspace_bytes.restype = _sz
    L.nonode_egno_tconv_bwd.argtypes = [_i] * 3 + [_vp] * 16 + [_sz, _vp]
    L.nonode_prepare_inputs.argtypes = [_i, _i, _i] + [_vp] * 5 + [_i] + [_vp] * 6
    L.nonode_energy.argtypes = [_i] * 4 + [_vp] * 5
    L.nonode_egno_rollout_workspace_bytes.argtypes = [_i] * 6
    L.nonode_egno_rollout_workspace_bytes.restype = _sz
    L.nonode_egno_rollout.argtypes = ([_i] * 10 + [_vp] * 9 + [_i, _i] + [_vp] * 3 + [ctypes.POINTER(_vp)] * 3
                                      + [_vp] * 3 + [_sz, _vp])
    L.nonode_segno_rollout_workspace_bytes.argtypes = [_i] * 4
    L.nonode_segno_rollout_workspace_bytes.restype = _sz
    L.nonode_segno_rollout.argtypes = ([_i] * 5 + [_vp] * 6 + [_i, _i] + [_vp] * 4 + [_f, _i] + [_vp] * 3
                                       + [_sz, _vp])
    _d = ctypes.c_double
    L.nonode_sim_charged.argtypes = [_i] * 4 + [_d] * 3 + [_vp] * 6
    L.nonode_sim_gravity.argtypes = [_i] * 4 + [_d] * 3 + [_vp] * 7
    L.nonode_gather_batch.argtypes = [_i] * 6 + [_vp] * 13
    L.nonode_gather_rows.argtypes = [_i, ctypes.c_longlong, _i, _vp, _vp, _vp, _vp]
    L.nonode_rollout_metrics.argtypes = [_i] * 3 + [_vp] * 5
    _ll = ctypes.c_longlong
    L.nonode_full_edges.argtypes = [_i, _i, _vp, _vp, _vp]
    L.nonode_check_full_edges.argtypes = [_vp, _vp, _i, _ll, _i, _i, _vp, _vp]
    L.nonode_poison_if_flagged.argtypes = [_vp, _i, ctypes.POINTER(_vp), ctypes.POINTER(_ll), _vp]
    L.nonode_egnn_layer_flat_state_floats.argtypes = [_i, _i]
    L.nonode_egnn_layer_flat_state_floats.restype = _sz
    L.nonode_egnn_layer_flat.argtypes = [_i] * 4 + [_vp] * 9
    L.nonode_flat_bwd_blob_floats.restype = _sz
    L.nonode_pack_layer_flat_bwd.argtypes = [ctypes.POINTER(LayerWeights), _i, _vp, _vp]
    L.nonode_egnn_layer_flat_bwd_node_floats.argtypes = [_i, _i]
    L.nonode_egnn_layer_flat_bwd_node_floats.restype = _sz
    L.nonode_egnn_layer_flat_bwd_edge_floats.argtypes = [_i, _i]
    L.nonode_egnn_layer_flat_bwd_edge_floats.restype = _sz
    L.nonode_egnn_layer_flat_bwd.argtypes = [_i] * 4 + [_vp] * 14
    L.nonode_profile_begin.argtypes = [_i]
    L.nonode_profile_end.argtypes = [ctypes.POINTER(_f), ctypes.POINTER(_i), _i]
    for s in SYMBOLS:
        if not hasattr(L, s):
            raise NonodeError(f"{LIB_PATH} does not export {s}")
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise NonodeError(f"nonode status {rc}: {lib().nonode_last_error().decode()}")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(*tensors):
    for t in tensors:
        if t is not None and (not t.is_cuda):
            raise NonodeError("no CPU path: the EGNO/SEGNO hot path runs only on a ROCm GPU "
                              "(move the model and inputs to 'cuda'); the CPU restatement lives "
                              "in oracle/ and is test infrastructure")


def profile_begin(max_records):
    check(lib().nonode_profile_begin(int(max_records)))


def profile_end(max_records=1 << 16):
    """Return [(kind, ms)] for the launches recorded since profile_begin (synchronises)."""
    ms = (_f * max_records)()
    kd = (_i * max_records)()
    n = lib().nonode_profile_end(ms, kd, max_records)
    if n < 0:
        check(-n)
    return [(kd[i], ms[i]) for i in range(n)]
