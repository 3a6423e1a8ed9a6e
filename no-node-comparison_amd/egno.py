"""Drop-in EGNO (EGNO/model/egno.py:8-111) whose forward runs the gfx950 kernels in libnonode.so.

Same constructor signature, same forward signature and return order (x, v, h), same state_dict
keys and shapes, and the same RNG consumption order in __init__ (so ``torch.manual_seed(s)``
yields the reference's initial weights). The module tree mirrors the reference names only
because the state_dict keys are part of the boundary (checkpoints written by
EGNO/utils.py:271-277 must load); none of the reference classes is reused.
"""
import ctypes

import torch
from torch import nn

from . import _lib
from .graph import check_full_graph, finish


class _MLP(nn.Module):
    """Two Linear layers with SiLU between (and after, if last_act) — BaseMLP's parameters
    (basic.py:34-58) under the attribute name ``mlp``. flat (basic.py:38-40): Tanh and a 4x wider
    hidden layer."""

    def __init__(self, din, dhid, dout, last_act=False, flat=False):
        super().__init__()
        act = nn.Tanh if flat else nn.SiLU
        dhid = 4 * dhid if flat else dhid
        layers = [nn.Linear(din, dhid), act(), nn.Linear(dhid, dout)]
        if last_act:
            layers.append(act())
        self.mlp = nn.Sequential(*layers)


class _InvariantEdgeNet(nn.Module):
    """Holds the edge-message MLP under ``scalar_net`` (InvariantScalarNet, basic.py:107-123)."""

    def __init__(self, din, hidden, flat=False):
        super().__init__()
        self.scalar_net = _MLP(din, hidden, hidden, last_act=True, flat=flat)


class EGNNLayerParams(nn.Module):
    """Parameters of one EGNN_Layer (basic.py:147-165); compute lives in the fused HIP kernel (flat:
    the 256-wide layer kernels). with_v=False has no node_v_net (basic.py:156-160)."""

    def __init__(self, in_edge_nf, hidden_nf, with_v=True, flat=False):
        super().__init__()
        self.edge_message_net = _InvariantEdgeNet(1 + 2 * hidden_nf + in_edge_nf, hidden_nf, flat)
        self.coord_net = _MLP(hidden_nf, hidden_nf, 1, flat=flat)
        self.node_v_net = _MLP(hidden_nf, hidden_nf, 1, flat=flat) if with_v else None
        self.node_net = _MLP(2 * hidden_nf, hidden_nf, hidden_nf, flat=flat)

    def weight_struct(self):
        e, c, v, n = (self.edge_message_net.scalar_net.mlp, self.coord_net.mlp,
                      self.node_v_net.mlp, self.node_net.mlp)
        return _lib.LayerWeights(*[t.data_ptr() for t in (
            e[0].weight, e[0].bias, e[2].weight, e[2].bias, c[0].weight, c[0].bias, c[2].weight,
            c[2].bias, v[0].weight, v[0].bias, v[2].weight, v[2].bias, n[0].weight, n[0].bias,
            n[2].weight, n[2].bias)])


class _SpectralWeights(nn.Module):
    """SpectralConv1d / SpectralConv1d_x parameter (layer_no.py:191-205 / 246-261)."""

    def __init__(self, cin, cout, modes, scale):
        super().__init__()
        self.weights1 = nn.Parameter(scale * torch.rand(cin, cout, modes, 2, dtype=torch.float))


class _TimeConvParams(nn.Module):
    def __init__(self, cin, cout, modes, scale):
        super().__init__()
        self.t_conv = _SpectralWeights(cin, cout, modes, scale)


def num_modes_for(num_timesteps, num_modes):
    """egno.py:26."""
    return min(num_timesteps, num_modes) if num_timesteps != 5 else min(num_modes, 3)


class EGNO(nn.Module):
    """EGNO neural operator (egno.py:8-111) — drop-in, MI355X kernels underneath.

    Supported: hidden_nf=64, SiLU activation, any num_inputs, norm (the radial input normalised,
    basic.py:140-141), use_time_conv (False: no TimeConv modules, egno.py:27-33, 99-107 skipped).
    with_v=False builds the reference's module tree (no node_v_net) but, as in the reference, cannot
    run forward (egno.py:95 / basic.py:180-181 need v and node_v_net). flat=True (every BaseMLP 4x
    wide with Tanh, basic.py:38-40; main_simulation_simple_no.py --flat) runs forward on its own layer
    kernels (csrc/nonode_flat.hip); its training (num_inputs=1) runs one autograd node per layer
    (autograd.FlatLayerTrain: HIP reverse kernels write the operands, weight gradients are GEMMs).
    """

    def __init__(self, n_layers, in_node_nf, in_edge_nf, hidden_nf, activation=nn.SiLU(), device='cpu',
                 with_v=False, flat=False, norm=False, use_time_conv=True, num_modes=2, num_timesteps=8,
                 time_emb_dim=32, num_inputs=1, varDT=False, fix_out_size=False):
        super().__init__()
        unsupported = []
        if num_inputs < 1:
            unsupported.append(f"num_inputs={num_inputs}")
        if hidden_nf != 64:
            unsupported.append(f"hidden_nf={hidden_nf}")
        if not isinstance(activation, nn.SiLU):
            unsupported.append(f"activation={activation}")
        if in_edge_nf > 4 or in_node_nf > 8:
            unsupported.append(f"in_edge_nf={in_edge_nf}, in_node_nf={in_node_nf}")
        if unsupported:
            raise NotImplementedError("EGNO (MI355X kernels) does not implement " + ", ".join(unsupported))
        self.time_emb_dim = time_emb_dim
        self.num_inputs = num_inputs
        self.varDT = varDT
        self.n_layers = n_layers
        self.with_v = with_v
        self.norm = norm
        self.hidden_nf = hidden_nf
        self.in_node_nf = in_node_nf
        self.in_edge_nf = in_edge_nf
        self.use_time_conv = use_time_conv
        self.flat = flat
        self.num_timesteps = num_timesteps if not fix_out_size else 10
        self.device = device
        modes = num_modes_for(num_timesteps, num_modes)
        self.num_modes = modes
        # registration + RNG order of EGNN.__init__ (basic.py:193-205): layers list, embedding
        # Linear, then each layer; then the per-layer time convs (egno.py:28-33)
        self.layers = nn.ModuleList()
        # egno.py:12-16: the multi-input model also embeds each frame's input time
        self.embedding = nn.Linear(in_node_nf + (2 if num_inputs > 1 else 1) * time_emb_dim, hidden_nf)
        for _ in range(n_layers):
            self.layers.append(EGNNLayerParams(in_edge_nf, hidden_nf, with_v, flat))
        if use_time_conv:
            self.time_conv_modules = nn.ModuleList()
            self.time_conv_x_modules = nn.ModuleList()
            for _ in range(n_layers):
                self.time_conv_modules.append(_TimeConvParams(hidden_nf, hidden_nf, modes,
                                                              1.0 / (hidden_nf * hidden_nf)))
                self.time_conv_x_modules.append(_TimeConvParams(2, 2, modes, 0.1))
        self._blobs = None
        self._blob_key = None
        self._bblobs = None
        self._bblob_key = None
        _lib.track_packs(self)   # packs dropped after any optimizer step over these parameters
        self.to(device)

    # ---- packed weights (re-packed whenever a parameter changed in place) ----
    def _drop_packs(self):
        """Forget the packed blobs (the next forward / backward re-packs): _lib.track_packs."""
        self._blob_key = None
        self._bblob_key = None

    def _pack_variant(self):
        return _lib.VARIANT_EGNO | (_lib.LAYER_NORM_RADIAL if self.norm else 0)

    def _packed(self):
        """Packed kernel weights (layer blobs, TimeConv blobs or None without time convolutions),
        rebuilt whenever a parameter changed in place (optimizer step) or moved (flat: the flat
        layer blobs of nonode_pack_layer_flat)."""
        params = _lib.param_list(self, "pack", lambda: [p for l in self.layers for p in l.parameters()] + (
            [m.t_conv.weights1 for m in self.time_conv_modules] if self.use_time_conv else []))
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._blobs is not None and key == self._blob_key:
            return self._blobs
        L = _lib.lib()
        n = L.nonode_flat_blob_floats() if self.flat else L.nonode_layer_blob_floats()
        dev = self.embedding.weight.device
        blobs = torch.empty(self.n_layers, n, dtype=torch.float32, device=dev)
        tblobs = torch.empty(self.n_layers, L.nonode_tconv_blob_floats(self.num_modes), dtype=torch.float32,
                             device=dev) if self.use_time_conv else None
        stream = _lib.stream_of(blobs)
        # every layer in one launch per blob kind (nonode_pack_layers / nonode_pack_tconvs)
        ws = [layer.weight_struct() for layer in self.layers]
        WP = ctypes.POINTER(_lib.LayerWeights)
        P = ctypes.c_void_p * self.n_layers
        if self.flat:
            for i, w in enumerate(ws):
                _lib.check(L.nonode_pack_layer_flat(ctypes.byref(w), self._pack_variant(), self.hidden_nf,
                                                    self.in_edge_nf, blobs[i].data_ptr(), stream))
        else:
            _lib.check(L.nonode_pack_layers((WP * self.n_layers)(*[ctypes.pointer(w) for w in ws]), self.n_layers,
                                            self._pack_variant(), self.hidden_nf, self.in_edge_nf,
                                            P(*[blobs[i].data_ptr() for i in range(self.n_layers)]), stream))
        if self.use_time_conv:
            tws = [m.t_conv.weights1.detach().float().contiguous() for m in self.time_conv_modules]
            _lib.check(L.nonode_pack_tconvs(P(*[t.data_ptr() for t in tws]), self.n_layers, self.num_modes,
                                            self.num_timesteps, P(*[tblobs[i].data_ptr() for i in range(self.n_layers)]),
                                            stream))
        self._blobs, self._blob_key = (blobs, tblobs), key
        return self._blobs

    def tconv_arrays(self, tblobs):
        """(tconv_blobs, tconvx_w) host pointer arrays for the C ABI plus the tensors they point
        into (keep them alive for the call); (None, None, []) without time convolutions."""
        if not self.use_time_conv:
            return None, None, []
        P = ctypes.c_void_p * self.n_layers
        tcx = [m.t_conv.weights1.detach().to(torch.float32).contiguous() for m in self.time_conv_x_modules]
        return (P(*[tblobs[i].data_ptr() for i in range(self.n_layers)]), P(*[t.data_ptr() for t in tcx]), tcx)

    def _launch_arrays(self, blobs, tblobs):
        """(layer blob pointers, tconv_arrays(...)) of a forward launch, cached while the packed blobs and
        the TimeConv_x parameters' storage stay the same (the kernels read those parameters live, so an
        in-place optimizer step needs no rebuild); rebuilt per call if a TimeConv_x weight is not fp32
        contiguous (tconv_arrays then points at a converted copy)."""
        tcx = _lib.param_list(self, "tcx", lambda: [m.t_conv.weights1 for m in self.time_conv_x_modules]
                              if self.use_time_conv else [])
        if not all(t.dtype == torch.float32 and t.is_contiguous() for t in tcx):
            P = ctypes.c_void_p * self.n_layers
            return P(*[blobs[i].data_ptr() for i in range(self.n_layers)]), self.tconv_arrays(tblobs)
        key = (blobs.data_ptr(), tblobs.data_ptr() if tblobs is not None else 0, tuple(t.data_ptr() for t in tcx))
        c = getattr(self, "_larrays", None)
        if c is not None and c[0] == key and c[1] is blobs:
            return c[2]
        P = ctypes.c_void_p * self.n_layers
        arrays = (P(*[blobs[i].data_ptr() for i in range(self.n_layers)]), self.tconv_arrays(tblobs))
        self._larrays = (key, blobs, arrays)
        return arrays

    def layer_param_names(self, i):
        """Parameter names of layer i in nonode_layer_weights / nonode_layer_grads field order."""
        pre = f"layers.{i}."
        e, c, v, n = ("edge_message_net.scalar_net.mlp", "coord_net.mlp", "node_v_net.mlp", "node_net.mlp")
        return [pre + f"{mlp}.{k}.{wb}" for mlp in (e, c, v, n) for k in (0, 2) for wb in ("weight", "bias")]

    def _packed_bwd(self):
        """Backward fragments (unscaled forward + transposed) per layer, rebuilt like _packed()."""
        params = _lib.param_list(self, "pack_bwd", lambda: [p for l in self.layers for p in l.parameters()])
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._bblobs is not None and key == self._bblob_key:
            return self._bblobs
        L = _lib.lib()
        dev = self.embedding.weight.device
        bb = torch.empty(self.n_layers, L.nonode_bwd_blob_floats(), dtype=torch.float32, device=dev)
        stream = _lib.stream_of(bb)
        ws = [layer.weight_struct() for layer in self.layers]   # one launch for every layer
        WP = ctypes.POINTER(_lib.LayerWeights)
        P = ctypes.c_void_p * self.n_layers
        _lib.check(L.nonode_pack_layers_bwd((WP * self.n_layers)(*[ctypes.pointer(w) for w in ws]), self.n_layers,
                                            self._pack_variant(), self.hidden_nf, self.in_edge_nf,
                                            P(*[bb[i].data_ptr() for i in range(self.n_layers)]), stream))
        self._bblobs, self._bblob_key = bb, key
        return bb

    def _packed_flat_bwd(self):
        """Transposed 256-wide fragments per flat layer (nonode_pack_layer_flat_bwd), rebuilt like _packed()."""
        params = _lib.param_list(self, "pack_bwd", lambda: [p for l in self.layers for p in l.parameters()])
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._bblobs is not None and key == self._bblob_key:
            return self._bblobs
        L = _lib.lib()
        bb = torch.empty(self.n_layers, L.nonode_flat_bwd_blob_floats(), dtype=torch.float32,
                         device=self.embedding.weight.device)
        stream = _lib.stream_of(bb)
        for i, layer in enumerate(self.layers):
            w = layer.weight_struct()
            _lib.check(L.nonode_pack_layer_flat_bwd(ctypes.byref(w), self.in_edge_nf, bb[i].data_ptr(), stream))
        self._bblobs, self._bblob_key = bb, key
        return bb

    def forward(self, x, h, edge_index, edge_fea, v=None, loc_mean=None, timesteps_in=None, timesteps_out=None):
        """egno.py:37-111. x, v, loc_mean: [BN, 3]; h: [BN, in_node_nf]; edge_index: 2 x [E]
        (fully connected, the dataset's edge order); edge_fea: [E, in_edge_nf];
        timesteps_out: [B, T]. Returns (x, v, h) of shapes [T*BN, 3], [T*BN, 3], [T*BN, 64]."""
        if not self.with_v:
            raise TypeError("EGNO(with_v=False) has no node_v_net: the reference forward fails on it too "
                            "(v.repeat at egno.py:95 for v=None, node_v_net(h) at basic.py:180-181 otherwise)")
        if v is None or (loc_mean is None and self.use_time_conv):
            raise ValueError("EGNO.forward needs v and loc_mean (the time convolution stacks "
                             "x - loc_mean with v, egno.py:103-105)")
        if self.flat and self._trains() and self.num_inputs > 1:
            raise NotImplementedError("EGNO(flat=True) training runs the single-input model (num_inputs=1)")
        if self.num_inputs > 1:
            return self._forward_multi(x, h, edge_index, edge_fea, v, loc_mean, timesteps_in, timesteps_out)
        _lib.require_device(x, h, v, loc_mean, edge_fea, self.embedding.weight)
        T = self.num_timesteps
        BN = h.shape[0]
        if timesteps_out is None:
            timesteps_out = torch.arange(T, device=x.device).unsqueeze(0)
        if timesteps_out.dim() != 2 or timesteps_out.shape[1] != T:
            raise ValueError(f"timesteps_out must be [B, {T}], got {tuple(timesteps_out.shape)}")
        Bt = timesteps_out.shape[0]
        if BN % Bt:
            raise ValueError("number of nodes must be a multiple of timesteps_out.shape[0] (egno.py:66)")
        B, N = check_full_graph(edge_index, BN)
        if edge_fea.shape != (B * N * (N - 1), self.in_edge_nf):
            raise ValueError(f"edge_fea must be [{B * N * (N - 1)}, {self.in_edge_nf}], got {tuple(edge_fea.shape)}")
        if self._trains():
            if self.flat:
                from .autograd import egno_flat_train
                return finish(egno_flat_train(self, x, h, edge_fea, v, loc_mean, timesteps_out, B, N))
            from .autograd import egno_forward_train
            return finish(egno_forward_train(self, x, h, edge_fea, v, loc_mean, timesteps_out, B, N))
        return finish(self._forward_kernels(x, h, edge_fea, v, loc_mean, timesteps_out, B, N))

    def _trains(self):
        """Training forward: train mode, gradients enabled and a parameter that requires grad."""
        return self.training and torch.is_grad_enabled() and any(
            p.requires_grad for p in _lib.param_list(self, "all", lambda: list(self.parameters())))

    def frame_inputs(self, T):
        """Input index of each of the T frames: repeat_elements_to_exact_shape (EGNO/utils.py:115-131)
        repeats each of the I inputs T // I times in order, then the last input T % I more times."""
        I = self.num_inputs
        k = T // I
        return [min(t // k, I - 1) if k > 0 else I - 1 for t in range(T)]

    def _forward_multi(self, x, h, edge_index, edge_fea, v, loc_mean, timesteps_in, timesteps_out):
        """egno.py:37-111 with num_inputs = I > 1: x, v, loc_mean [I, BN, 3], h [I, BN, in_node_nf],
        edge_fea [I, E, in_edge_nf] (prepare_inputs, main_simulation_simple_no.py:313-327),
        timesteps_in [B, I], timesteps_out [B, T]. Frame t uses input frame_inputs(T)[t]
        (egno.py:44-49, 80-96); its embedding adds the input time's embedding (egno.py:77-79)."""
        I, T = self.num_inputs, self.num_timesteps
        if x.dim() != 3 or x.shape[0] != I or h.dim() != 3 or h.shape[0] != I:
            raise ValueError(f"num_inputs={I}: x, v, loc_mean must be [{I}, BN, 3] and h [{I}, BN, F]")
        if timesteps_in is None or timesteps_in.dim() != 2 or timesteps_in.shape[1] != I:
            raise ValueError(f"num_inputs={I}: timesteps_in must be [B, {I}]")
        _lib.require_device(x, h, v, loc_mean, edge_fea, timesteps_in, self.embedding.weight)
        BN = h.shape[1]
        if timesteps_out is None or timesteps_out.dim() != 2 or timesteps_out.shape[1] != T:
            raise ValueError(f"timesteps_out must be [B, {T}]")
        Bt = timesteps_out.shape[0]
        if BN % Bt or timesteps_in.shape[0] != Bt:
            raise ValueError("timesteps_in / timesteps_out rows must divide the node count (egno.py:66)")
        B, N = check_full_graph(edge_index, BN)
        E = B * N * (N - 1)
        if edge_fea.dim() != 3 or edge_fea.shape != (I, E, self.in_edge_nf):
            raise ValueError(f"edge_fea must be [{I}, {E}, {self.in_edge_nf}], got {tuple(edge_fea.shape)}")
        fidx = torch.tensor(self.frame_inputs(T), device=x.device)
        f32 = lambda t: t.detach().to(torch.float32)  # noqa: E731
        per_frame = lambda t: None if t is None else f32(t)[fidx].reshape(T * t.shape[1], t.shape[2]).contiguous()  # noqa: E731,E501
        with torch.no_grad():
            xf, hf, vf, lmf, eff = (per_frame(t) for t in (x, h, v, loc_mean, edge_fea))
            t_in = f32(timesteps_in)[:, fidx].contiguous()
            t_out = f32(timesteps_out).contiguous()
        if self._trains():
            from .autograd import egno_forward_train
            return finish(egno_forward_train(self, xf, hf, eff, vf, lmf, t_out, B, N, t_in=t_in))
        L = _lib.lib()
        with torch.no_grad():
            return finish(self._launch_forward(L.nonode_egno_forward_flat if self.flat else L.nonode_egno_forward_frames,
                                               B, N, xf, hf, vf, lmf, eff, t_out, t_in=t_in))

    def _t_out_f32(self, t_out):
        """timesteps_out as f32 (cached per tensor/version: callers pass the same int64 tensor)."""
        if t_out.dtype == torch.float32 and t_out.is_contiguous():
            return t_out
        key = (t_out.data_ptr(), t_out._version, tuple(t_out.shape), t_out.stride(), t_out.dtype, t_out.device)
        c = getattr(self, "_tcache", None)
        if c is not None and c[0] == key:
            return c[1]
        tt = t_out.detach().to(torch.float32).contiguous()
        self._tcache = (key, tt, t_out)      # keep t_out alive so its pointer cannot be reused
        return tt

    @torch.no_grad()
    def _forward_kernels(self, x, h, edge_fea, v, loc_mean, t_out, B, N):
        f32 = lambda t: None if t is None else t.detach().to(torch.float32).contiguous()  # noqa: E731
        x, h, v, lm, ef = f32(x), f32(h), f32(v), f32(loc_mean), f32(edge_fea)
        if self.flat:   # nonode_egno_forward_flat: t_in NULL = the single-input embedding
            return self._launch_forward(_lib.lib().nonode_egno_forward_flat, B, N, x, h, v, lm, ef,
                                        self._t_out_f32(t_out), t_in=False)
        return self._launch_forward(_lib.lib().nonode_egno_forward, B, N, x, h, v, lm, ef, self._t_out_f32(t_out))

    def _launch_forward(self, entry, B, N, x, h, v, lm, ef, tt, t_in=None):
        """nonode_egno_forward (single input) or nonode_egno_forward_frames (t_in given)."""
        T = self.num_timesteps
        blobs, tblobs = self._packed()
        dev = x.device
        n = T * B * N
        x_out = torch.empty(n, 3, device=dev)
        v_out = torch.empty(n, 3, device=dev)
        h_out = torch.empty(n, self.hidden_nf, device=dev)
        L = _lib.lib()
        ws_bytes = (L.nonode_egno_flat_workspace_bytes if self.flat else L.nonode_egno_workspace_bytes)(
            B, N, T, tt.shape[0])
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=dev)
        blob_p, (tcw_p, tcx_p, _keep) = self._launch_arrays(blobs, tblobs)
        f32 = lambda t: t if t.dtype == torch.float32 and t.is_contiguous() else t.detach().to(torch.float32).contiguous()  # noqa: E731,E501
        ew, eb = f32(self.embedding.weight), f32(self.embedding.bias)
        tail = (_lib.ptr(ew), _lib.ptr(eb), blob_p, tcw_p, tcx_p, _lib.ptr(x_out), _lib.ptr(v_out),
                _lib.ptr(h_out), _lib.ptr(ws), ws_bytes, _lib.stream_of(x))
        head = (B, N, T, self.n_layers, self.in_node_nf, self.in_edge_nf, self.time_emb_dim, self.num_modes,
                tt.shape[0], _lib.ptr(x), _lib.ptr(h), _lib.ptr(v), _lib.ptr(lm), _lib.ptr(ef))
        if t_in is None:
            _lib.check(entry(*head, _lib.ptr(tt), *tail))
        else:   # (t_in=False: the flat entry's NULL input-time embedding)
            _lib.check(entry(*head, _lib.ptr(t_in) if t_in is not False else None, _lib.ptr(tt), *tail))
        return x_out, v_out, h_out
