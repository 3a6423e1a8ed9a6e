"""Drop-in SEGNO (SEGNO/models/model.py:6-102) on the gfx950 kernels in libnonode.so.

Same constructor and forward signatures, return order (x, h, v), state_dict keys, and RNG
consumption order in __init__ (model.py:10-25, gcl.py:27-69).

Semantics note: the reference's live ``forward`` (model.py:53-92)
discards the integrator result for a single input and returns its inputs. This class returns
the integrator result (what the shadowed forward at model.py:28-51 and ``forward_step`` compute);
``bug_compat=True`` reproduces the reference's identity behaviour exactly.

Training (train_nbody.py:168-179): in train mode with gradients enabled, forward goes through
autograd.SEGNOTrain: the embedding Linear (nonode_embedding_forward / _backward) and the HIP
integrator forward with saved substeps and its hand-written reverse pass, so loss.backward() reaches
every parameter. forward_step (an already-embedded h) and several inputs go through
autograd.SEGNOStepTrain with the embedding as torch ops on the tape.
"""
import ctypes

import torch
from torch import nn

from . import _lib
from .graph import check_full_graph, finish


class GCLParams(nn.Module):
    """Parameters of SEGNO_GCL (gcl.py:26-69) in its registration and RNG order."""

    def __init__(self, input_nf, output_nf, hidden_nf, edges_in_d=0, act_fn=nn.SiLU(), tanh=False):
        super().__init__()
        self.edge_mlp = nn.Sequential(nn.Linear(2 * input_nf + 1 + edges_in_d, hidden_nf), act_fn,
                                      nn.Linear(hidden_nf, hidden_nf), act_fn)
        self.node_mlp = nn.Sequential(nn.Linear(hidden_nf + input_nf, hidden_nf), act_fn,
                                      nn.Linear(hidden_nf, output_nf))
        layer = nn.Linear(hidden_nf, 1, bias=True)
        torch.nn.init.xavier_uniform_(layer.weight, gain=0.001)
        # tanh=True appends nn.Tanh (gcl.py:57-59): no parameters, same state_dict keys; the
        # reference's coords_range (a plain tensor, never used in forward) is kept for fidelity
        self.coord_mlp = nn.Sequential(nn.Linear(hidden_nf, hidden_nf), act_fn, layer, *([nn.Tanh()] if tanh else []))
        if tanh:
            self.coords_range = torch.ones(1) * 3
        # coord_mlp_vel exists in the reference state_dict but is never used in forward
        self.coord_mlp_vel = nn.Sequential(nn.Linear(input_nf, hidden_nf), act_fn, nn.Linear(hidden_nf, 1))

    def weight_struct(self):
        e, c, n = self.edge_mlp, self.coord_mlp, self.node_mlp
        ptrs = [e[0].weight, e[0].bias, e[2].weight, e[2].bias, c[0].weight, c[0].bias, c[2].weight,
                c[2].bias, None, None, None, None, n[0].weight, n[0].bias, n[2].weight, n[2].bias]
        return _lib.LayerWeights(*[t.data_ptr() if t is not None else None for t in ptrs])


class SEGNO(nn.Module):
    """SEGNO neural ODE (model.py:6-102) — drop-in, MI355X kernels underneath.

    Supported: SiLU, hidden_nf=64, in_edge_nf <= 4, tanh (coordinate MLP output through tanh,
    gcl.py:57-59), norm_diff (stored, unused in the reference's forward, gcl.py:32,63); single
    input (x [BN, 3]) or several (x [BN, I, 3] with in_steps, multiple_agg 'sum' / 'attn').
    """

    def __init__(self, in_node_nf, in_edge_nf, hidden_nf, device='cpu', act_fn=nn.SiLU(), n_layers=4,
                 coords_weight=1.0, recurrent=False, norm_diff=False, tanh=False, invariant=True,
                 norm_vel=True, varDT=False, multiple_agg=None, bug_compat=False):
        super().__init__()
        unsupported = []
        if hidden_nf != 64:
            unsupported.append(f"hidden_nf={hidden_nf}")
        if not isinstance(act_fn, nn.SiLU):
            unsupported.append(f"act_fn={act_fn}")
        if in_edge_nf > 4 or in_node_nf > 8:
            unsupported.append(f"in_edge_nf={in_edge_nf}, in_node_nf={in_node_nf}")
        if multiple_agg not in (None, "attn", "sum"):
            raise ValueError("Invalid multiple aggregation method specified.")
        if unsupported:
            raise NotImplementedError("SEGNO (MI355X kernels) does not implement " + ", ".join(unsupported))
        self.hidden_nf = hidden_nf
        self.varDT = varDT
        self.multiple_agg = multiple_agg
        if multiple_agg == "attn":
            # InvariantTemporalAttention parameters (model.py:126-139), created first as in the
            # reference so the RNG stream matches
            self.enc_attn_net = nn.Module()
            self.enc_attn_net.attn_mlp = nn.Sequential(nn.Linear(hidden_nf + 1, hidden_nf), nn.Tanh(),
                                                       nn.Linear(hidden_nf, 1))
        self.device = device
        self.n_layers = n_layers
        self.embedding = nn.Linear(in_node_nf, hidden_nf)
        self.invariant = invariant
        self.norm_vel = norm_vel
        self.sigmoid = nn.Sigmoid()
        self.module = GCLParams(hidden_nf, hidden_nf, hidden_nf, edges_in_d=in_edge_nf, act_fn=act_fn, tanh=tanh)
        self.tanh = tanh
        self.norm_diff = norm_diff
        self.coords_weight = coords_weight
        self.recurrent = recurrent
        self.in_node_nf = in_node_nf
        self.in_edge_nf = in_edge_nf
        self.bug_compat = bug_compat
        self._blob = None
        self._blob_key = None
        self._bblob = None
        self._bblob_key = None
        _lib.track_packs(self)   # packs dropped after any optimizer step over these parameters
        self.to(device)

    def _drop_packs(self):
        """Forget the packed blobs (the next forward / backward re-packs): _lib.track_packs."""
        self._blob_key = None
        self._bblob_key = None

    def gcl_param_names(self):
        """Parameter names in nonode_layer_grads field order (vel_* = None: coord_mlp_vel is not on
        the forward path, gcl.py:111-119)."""
        pre = "module."
        e, c, n = "edge_mlp", "coord_mlp", "node_mlp"
        names = [pre + f"{mlp}.{k}.{wb}" for mlp in (e, c) for k in (0, 2) for wb in ("weight", "bias")]
        return names + [None] * 4 + [pre + f"{n}.{k}.{wb}" for k in (0, 2) for wb in ("weight", "bias")]

    def _packed_bwd(self):
        """Backward fragments of the GCL (unscaled forward + transposed), rebuilt like _packed()."""
        params = _lib.param_list(self, "gcl", lambda: list(self.module.parameters()))
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._bblob is not None and key == self._bblob_key:
            return self._bblob
        L = _lib.lib()
        bb = torch.empty(L.nonode_bwd_blob_floats(), dtype=torch.float32, device=self.embedding.weight.device)
        w = self.module.weight_struct()
        _lib.check(L.nonode_pack_layer_bwd(ctypes.byref(w), self._pack_variant(), self.hidden_nf, self.in_edge_nf,
                                           _lib.ptr(bb), _lib.stream_of(bb)))
        self._bblob, self._bblob_key = bb, key
        return bb

    def _pack_variant(self):
        return _lib.VARIANT_SEGNO | (_lib.LAYER_TANH_COORD if self.tanh else 0)

    def _training(self):
        return self.training and torch.is_grad_enabled() and any(
            p.requires_grad for p in _lib.param_list(self, "all", lambda: list(self.parameters())))

    def _packed(self):
        params = _lib.param_list(self, "gcl", lambda: list(self.module.parameters()))
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._blob is not None and key == self._blob_key:
            return self._blob
        L = _lib.lib()
        blob = torch.empty(L.nonode_layer_blob_floats(), dtype=torch.float32, device=self.embedding.weight.device)
        w = self.module.weight_struct()
        _lib.check(L.nonode_pack_layer(ctypes.byref(w), self._pack_variant(), self.hidden_nf, self.in_edge_nf,
                                       _lib.ptr(blob), _lib.stream_of(blob)))
        self._blob, self._blob_key = blob, key
        return blob

    def forward(self, his, x, edges, v, edge_attr, T=10, in_steps=None):
        """model.py:53-92 (single input). his [BN, in_node_nf], x, v [BN, 3], edges 2 x [E],
        edge_attr [E, in_edge_nf]. Returns (x, h, v) after T substeps of dt = 1/T.

        In train mode with gradients enabled (nn.Module's default state) this records the autograd
        tape: the embedding and one training-forward launch of the T substeps that saves every
        substep's state for the reverse pass (autograd.SEGNOTrain), heavier in memory than the
        inference launch.
        Inference should run under model.eval() or torch.no_grad(), as the reference's test loops do."""
        if x.dim() == 3:
            return self._forward_multi(his, x, edges, v, edge_attr, int(T), in_steps)
        if self.bug_compat:
            # the live reference forward returns its inputs (and the embedded h)
            return x, self._embed(his), v
        if self._training():
            if his.shape[-1] > 40:   # (nonode_embedding_* take up to 40 input features)
                return self._step(self._embed(his), x, edges, v, edge_attr, int(T))
            # the embedding and the T substeps as one autograd node (autograd.SEGNOTrain)
            B, N = self._check_inputs(x, edges, v, edge_attr)
            _lib.require_device(his, self.embedding.weight)
            from .autograd import segno_train
            return finish(segno_train(self, his, x, v, edge_attr, int(T), B, N))
        return self._run(his, None, x, edges, v, edge_attr, int(T))

    def _forward_multi(self, his, x, edges, v, edge_attr, T, in_steps):
        """model.py:53-92 with num_inputs = I > 1: his [BN, I, F], x, v [BN, I, 3], in_steps [I]
        (input frame offsets, train_nbody.py:114). forward_step (the HIP integrator) runs
        diff(in_steps) + [T] substeps in turn; after each but the last, the next input is folded in
        by multiple_agg ('sum': added; 'attn': InvariantTemporalAttention weights over the pair,
        model.py:104-139, a small torch MLP on the device). Returns the last forward_step's result;
        bug_compat=True returns the state before it, as the reference does."""
        if in_steps is None:
            raise ValueError("SEGNO with several inputs needs in_steps (train_nbody.py:114)")
        if his.dim() != 3 or v.dim() != 3 or his.shape[1] != x.shape[1] or v.shape[1] != x.shape[1]:
            raise ValueError("his, x, v must be [BN, I, .] with the same I")
        _lib.require_device(his, x, v, edge_attr, self.embedding.weight)
        st = in_steps.tolist() if torch.is_tensor(in_steps) else list(in_steps)
        steps = [int(b) - int(a) for a, b in zip(st[:-1], st[1:])] + [int(T)]
        with torch.set_grad_enabled(self._training()):
            h = self._embed(his.to(torch.float32))
            h_, x_, v_ = h[:, 0].contiguous(), x[:, 0].contiguous(), v[:, 0].contiguous()
            for i, step in enumerate(steps):
                xi, hi, vi = self._step(h_, x_, edges, v_, edge_attr, step)
                if i < len(steps) - 1:
                    if self.multiple_agg == "sum":
                        h_, x_, v_ = h[:, i + 1] + hi, x[:, i + 1] + xi, v[:, i + 1] + vi
                    elif self.multiple_agg == "attn":
                        x_, v_, h_ = self._attn_combine(torch.stack([x[:, i + 1], xi], 1),
                                                        torch.stack([v[:, i + 1], vi], 1),
                                                        torch.stack([h[:, i + 1], hi], 1))
            return (x_, h_, v_) if self.bug_compat else (xi, hi, vi)

    def _attn_combine(self, loc_seq, vel_seq, his_seq):
        """prepare_node_inputs (model.py:104-121) with InvariantTemporalAttention (model.py:126-139)."""
        speed = vel_seq.float().norm(dim=-1, keepdim=True)
        a = self.enc_attn_net.attn_mlp(torch.cat([speed, his_seq.float()], dim=-1)).softmax(dim=1)
        return (a * loc_seq).sum(1), (a * vel_seq).sum(1), (a * his_seq).sum(1)

    def forward_step(self, h, x, edges, v, edge_attr, T=10):
        """model.py:95-102: T substeps of the shared layer from an already-embedded h."""
        self.module.n_layers = T
        self.n_layers = T
        return self._step(h, x, edges, v, edge_attr, int(T))

    def _step(self, h, x, edges, v, edge_attr, T):
        """forward_step from an embedded h: on the autograd tape in training, else the fused
        inference launch."""
        if not self._training():
            return self._run(None, h, x, edges, v, edge_attr, T)
        _lib.require_device(h)
        B, N = self._check_inputs(x, edges, v, edge_attr)
        from .autograd import segno_step_train
        return finish(segno_step_train(self, h, x, v, edge_attr, T, B, N))

    def _check_inputs(self, x, edges, v, edge_attr):
        """(B, N) of a training call's fully connected graph, after the device and shape checks."""
        _lib.require_device(x, v, edge_attr, self.embedding.weight)
        B, N = check_full_graph(edges, x.shape[0])
        if edge_attr.shape != (B * N * (N - 1), self.in_edge_nf):
            raise ValueError(f"edge_attr must be [{B * N * (N - 1)}, {self.in_edge_nf}]")
        return B, N

    def _embed(self, his):
        """SEGNO.embedding (model.py:73): a torch op on the device, so it is on the autograd tape
        in training."""
        _lib.require_device(his, self.embedding.weight)
        x, w = his.to(torch.float32), self.embedding.weight
        if x.shape[-1] > 8:
            return torch.nn.functional.linear(x, w, self.embedding.bias)
        # K = in_node_nf <= 8: broadcast multiply-adds (elementwise kernels, and reductions in the
        # backward) instead of a K-deep GEMM, for which the BLAS picks a slow tile (83 us at the C3
        # size for K = 1, the largest torch op of the training step)
        out = self.embedding.bias + x[..., :1] * w[:, 0]
        for k in range(1, x.shape[-1]):
            out = out + x[..., k:k + 1] * w[:, k]
        return out

    @torch.no_grad()
    def _run(self, his, h_in, x, edges, v, edge_attr, T):
        _lib.require_device(x, v, edge_attr, self.embedding.weight)
        BN = x.shape[0]
        B, N = check_full_graph(edges, BN)
        if edge_attr.shape != (B * N * (N - 1), self.in_edge_nf):
            raise ValueError(f"edge_attr must be [{B * N * (N - 1)}, {self.in_edge_nf}]")
        f32 = lambda t: t.detach().to(torch.float32).contiguous() if t is not None else None  # noqa: E731
        x, v, ea = f32(x), f32(v), f32(edge_attr)
        his, h_in = f32(his), f32(h_in)
        dev = x.device
        blob = self._packed()
        x_out = torch.empty(BN, 3, device=dev)
        v_out = torch.empty(BN, 3, device=dev)
        h_out = torch.empty(BN, self.hidden_nf, device=dev)
        L = _lib.lib()
        ws_bytes = L.nonode_segno_workspace_bytes(B, N)
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=dev)
        ew, eb = f32(self.embedding.weight), f32(self.embedding.bias)
        _lib.check(L.nonode_segno_forward_step(
            B, N, T, self.in_node_nf, self.in_edge_nf, _lib.ptr(his), _lib.ptr(h_in), _lib.ptr(x), _lib.ptr(v),
            _lib.ptr(ea), _lib.ptr(ew), _lib.ptr(eb), _lib.ptr(blob), float(self.coords_weight),
            int(bool(self.recurrent)), _lib.ptr(x_out), _lib.ptr(v_out), _lib.ptr(h_out), _lib.ptr(ws),
            ws_bytes, _lib.stream_of(x)))
        return finish((x_out, h_out, v_out))
