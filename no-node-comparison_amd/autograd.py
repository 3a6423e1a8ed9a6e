"""Training entry for EGNO: loss.backward() of run_epoch (main_simulation_simple_no.py:267-280).

EGNOTrain is a torch.autograd.Function around the C ABI: its forward runs
nonode_egno_forward_train (same kernels and outputs as the inference forward, plus the saved
state), its backward runs nonode_egno_backward and returns the gradient of every parameter. The
reference's training loop (criterion, loss.backward(), optimizer.step()) runs unchanged on top.
"""
import ctypes

import torch

from . import _lib


def _f32(t):
    return t.detach().to(torch.float32).contiguous()


class EGNOTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, x, h, edge_fea, v, loc_mean, t_out, t_in, B, N, *params):
        # t_in is None for a single input; else the inputs are per frame (num_inputs > 1) and t_in
        # [Bt, T] is each frame's input time (nonode_egno_forward_train_frames)
        L = _lib.lib()
        T = model.num_timesteps
        dev = x.device
        x, h, v, ef = _f32(x), _f32(h), _f32(v), _f32(edge_fea)
        tt = model._t_out_f32(t_out)   # cached per tensor / version: no int64 -> f32 copy per step
        lm = _f32(loc_mean) if loc_mean is not None else None   # unused without time convolutions
        emb_cols = model.time_emb_dim * (1 if t_in is None else 2)
        Bt = tt.shape[0]
        blobs, tblobs = model._packed()
        n = T * B * N
        x_out = torch.empty(n, 3, device=dev)
        v_out = torch.empty(n, 3, device=dev)
        h_out = torch.empty(n, model.hidden_nf, device=dev)
        ws_bytes = L.nonode_egno_workspace_bytes(B, N, T, Bt)
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=dev)
        st_bytes = L.nonode_egno_train_state_bytes(B, N, T, model.n_layers, model.in_node_nf, emb_cols)
        state = torch.empty((st_bytes + 3) // 4, dtype=torch.float32, device=dev)
        P = ctypes.c_void_p * model.n_layers
        tcw_p, tcx_p, _keep = model.tconv_arrays(tblobs)
        ew, eb = _f32(model.embedding.weight), _f32(model.embedding.bias)
        head = (B, N, T, model.n_layers, model.in_node_nf, model.in_edge_nf, model.time_emb_dim, model.num_modes, Bt,
                _lib.ptr(x), _lib.ptr(h), _lib.ptr(v), _lib.ptr(lm), _lib.ptr(ef))
        tail = (_lib.ptr(ew), _lib.ptr(eb), P(*[blobs[i].data_ptr() for i in range(model.n_layers)]), tcw_p, tcx_p,
                _lib.ptr(x_out), _lib.ptr(v_out), _lib.ptr(h_out), _lib.ptr(state), st_bytes, _lib.ptr(ws), ws_bytes,
                _lib.stream_of(x))
        if t_in is None:
            _lib.check(L.nonode_egno_forward_train(*head, _lib.ptr(tt), *tail))
        else:
            ti = _f32(t_in)
            _lib.check(L.nonode_egno_forward_train_frames(*head, _lib.ptr(ti), _lib.ptr(tt), *tail))
        ctx.frames = t_in is not None
        # outputs the loss does not use (v, h for the reference's loss on x) arrive as None rather
        # than as zero-filled tensors: the library zeroes its own output-gradient buffers for them
        ctx.set_materialize_grads(False)
        ctx.model, ctx.B, ctx.N, ctx.Bt = model, B, N, Bt
        ctx.state, ctx.lm, ctx.ef = state, lm, ef
        ctx.n_params = len(params)
        sink = getattr(model, "_train_state_sink", None)
        if sink is not None:   # tests: the saved state (its head holds TimeConv's LeakyReLU decisions)
            sink.append(state)
        # the backward repacks the parameters' current values: saving them lets autograd's version
        # check raise if any was modified in place between forward and backward (e.g. an optimizer
        # step before a second backward), instead of returning gradients for the wrong weights
        ctx.save_for_backward(*params)
        return x_out, v_out, h_out

    @staticmethod
    def backward(ctx, gx, gv, gh):
        model, B, N, Bt = ctx.model, ctx.B, ctx.N, ctx.Bt
        _ = ctx.saved_tensors   # raises if a parameter changed in place since the forward
        L = _lib.lib()
        T = model.num_timesteps
        dev = ctx.state.device
        nl = model.n_layers
        bblobs = model._packed_bwd()
        grads = {name: torch.empty_like(p) for name, p in model.named_parameters()}
        lg = (_lib.LayerGrads * nl)()
        for i in range(nl):
            names = model.layer_param_names(i)
            lg[i] = _lib.LayerGrads(*[grads[nm].data_ptr() for nm in names])
        P = ctypes.c_void_p * nl
        tw_p = txw_p = g_tc = g_tcx = None   # use_time_conv=False: no TimeConv arrays
        if model.use_time_conv:
            tw = [_f32(m.t_conv.weights1) for m in model.time_conv_modules]
            txw = [_f32(m.t_conv.weights1) for m in model.time_conv_x_modules]
            tw_p, txw_p = P(*[t.data_ptr() for t in tw]), P(*[t.data_ptr() for t in txw])
            g_tc = P(*[grads[f"time_conv_modules.{i}.t_conv.weights1"].data_ptr() for i in range(nl)])
            g_tcx = P(*[grads[f"time_conv_x_modules.{i}.t_conv.weights1"].data_ptr() for i in range(nl)])
        ws_bytes = L.nonode_egno_backward_workspace_bytes(B, N, T, model.num_modes)
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=dev)
        gx = _f32(gx) if gx is not None else torch.zeros(T * B * N, 3, device=dev)
        gv = _f32(gv) if gv is not None else None
        gh = _f32(gh) if gh is not None else None
        head = (B, N, T, nl, model.in_node_nf, model.in_edge_nf, model.time_emb_dim)
        tail = (model.num_modes, Bt,
                _lib.ptr(ctx.lm), _lib.ptr(ctx.ef), P(*[bblobs[i].data_ptr() for i in range(nl)]),
                tw_p, txw_p, _lib.ptr(ctx.state),
                _lib.ptr(gx), _lib.ptr(gv), _lib.ptr(gh), lg, g_tc, g_tcx,
                _lib.ptr(grads["embedding.weight"]), _lib.ptr(grads["embedding.bias"]), _lib.ptr(ws), ws_bytes,
                _lib.stream_of(gx))
        if ctx.frames:
            _lib.check(L.nonode_egno_backward_frames(*head, 1, *tail))
        else:
            _lib.check(L.nonode_egno_backward(*head, *tail))
        ctx.state = None
        out = [grads[name] for name, _ in model.named_parameters()]
        return (None,) * 10 + tuple(out)


def egno_forward_train(model, x, h, edge_fea, v, loc_mean, t_out, B, N, t_in=None):
    """EGNO forward that records the kernels' backward on the autograd tape (t_in: per-frame
    multi-input form, see EGNO._forward_multi)."""
    params = [p for _, p in model.named_parameters()]
    return EGNOTrain.apply(model, x, h, edge_fea, v, loc_mean, t_out, t_in, B, N, *params)


def _segno_forward(ctx, model, h, x, v, edge_attr, T, B, N):
    """nonode_segno_forward_train from an embedded h (f32, contiguous): (x, h, v) after T substeps;
    ctx keeps the saved state for _segno_backward."""
    L = _lib.lib()
    dev = x.device
    x, v, ea = _f32(x), _f32(v), _f32(edge_attr)
    blob = model._packed()
    n = B * N
    x_out = torch.empty(n, 3, device=dev)
    v_out = torch.empty(n, 3, device=dev)
    h_out = torch.empty(n, model.hidden_nf, device=dev)
    st_bytes = L.nonode_segno_train_state_bytes(B, N, T)
    state = torch.empty((st_bytes + 3) // 4, dtype=torch.float32, device=dev)
    _lib.check(L.nonode_segno_forward_train(B, N, T, model.in_edge_nf, _lib.ptr(h), _lib.ptr(x), _lib.ptr(v),
                                            _lib.ptr(ea), _lib.ptr(blob), float(model.coords_weight),
                                            int(bool(model.recurrent)), _lib.ptr(x_out), _lib.ptr(v_out),
                                            _lib.ptr(h_out), _lib.ptr(state), st_bytes, _lib.stream_of(x)))
    ctx.model, ctx.T, ctx.B, ctx.N = model, T, B, N
    ctx.state, ctx.ea = state, ea
    ctx.set_materialize_grads(False)   # unused outputs: None, zeroed by the library (see EGNOTrain)
    return x_out, h_out, v_out


def _segno_backward(ctx, gx, gh, gv, want_h, want_x, want_v):
    """nonode_segno_backward: ({GCL parameter name: gradient}, g_h, g_x, g_v) with each input gradient
    None unless wanted (the library writes only the requested ones)."""
    model, T, B, N = ctx.model, ctx.T, ctx.B, ctx.N
    L = _lib.lib()
    dev = ctx.state.device
    n = B * N
    bblob = model._packed_bwd()
    names = model.gcl_param_names()
    named = dict(model.named_parameters())
    grads = {nm: torch.empty_like(named[nm]) for nm in names if nm is not None}
    lg = _lib.LayerGrads(*[grads[nm].data_ptr() if nm is not None else None for nm in names])
    ws_bytes = L.nonode_segno_backward_workspace_bytes(B, N)
    ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=dev)
    gx = _f32(gx) if gx is not None else None
    gv = _f32(gv) if gv is not None else None
    gh = _f32(gh) if gh is not None else None
    g_h = torch.empty(n, model.hidden_nf, device=dev) if want_h else None
    g_x = torch.empty(n, 3, device=dev) if want_x else None
    g_v = torch.empty(n, 3, device=dev) if want_v else None
    _lib.check(L.nonode_segno_backward(B, N, T, model.in_edge_nf, float(model.coords_weight),
                                       int(bool(model.recurrent)), _lib.ptr(ctx.ea), _lib.ptr(bblob),
                                       _lib.ptr(ctx.state), _lib.ptr(gx), _lib.ptr(gv), _lib.ptr(gh),
                                       ctypes.byref(lg), _lib.ptr(g_h), _lib.ptr(g_x), _lib.ptr(g_v),
                                       _lib.ptr(ws), ws_bytes, _lib.stream_of(ws)))
    ctx.state = None
    return grads, g_h, g_x, g_v


class SEGNOStepTrain(torch.autograd.Function):
    """SEGNO.forward_step (SEGNO/models/model.py:95-102) on the autograd tape: T substeps of
    SEGNO_GCL (gcl.py:111-119) from an embedded h. Forward: nonode_segno_forward_train (one launch
    for the T substeps, saving each substep's state); backward: nonode_segno_backward (gradients of
    the shared GCL weights and of h, x, v)."""

    @staticmethod
    def forward(ctx, model, h, x, v, edge_attr, T, B, N, *params):
        ctx.save_for_backward(*params)   # version check of the parameters (see EGNOTrain.forward)
        return _segno_forward(ctx, model, _f32(h), x, v, edge_attr, T, B, N)

    @staticmethod
    def backward(ctx, gx, gh, gv):
        model = ctx.model
        _ = ctx.saved_tensors   # raises if a parameter changed in place since the forward
        grads, g_h, g_x, g_v = _segno_backward(ctx, gx, gh, gv, *ctx.needs_input_grad[1:4])
        out = [grads.get(nm) for nm, _ in model.module.named_parameters(prefix="module")]
        return (None, g_h, g_x, g_v, None, None, None, None) + tuple(out)


def segno_step_train(model, h, x, v, edge_attr, T, B, N):
    """forward_step that records the kernels' backward on the autograd tape."""
    params = [p for _, p in model.module.named_parameters()]
    return SEGNOStepTrain.apply(model, h, x, v, edge_attr, T, B, N, *params)


class SEGNOTrain(torch.autograd.Function):
    """SEGNO.forward in training with one input (SEGNO/models/model.py:53-102, train_nbody.py:168): the
    embedding Linear (model.py:73) and forward_step's T substeps as ONE node of the tape. The
    embedding runs as nonode_embedding_forward and its weight gradient as nonode_embedding_backward
    from the g_h the reverse pass returns, instead of broadcast torch ops and their autograd reverse."""

    @staticmethod
    def forward(ctx, model, his, x, v, edge_attr, T, B, N, *params):
        L = _lib.lib()
        ctx.his_dtype = his.dtype
        his = _f32(his)
        h = torch.empty(B * N, model.hidden_nf, device=x.device)
        ew, eb = _f32(model.embedding.weight), _f32(model.embedding.bias)
        _lib.check(L.nonode_embedding_forward(B * N, his.shape[1], _lib.ptr(his), _lib.ptr(ew), _lib.ptr(eb),
                                              _lib.ptr(h), _lib.stream_of(his)))
        # his through save_for_backward: autograd checks its version (an in-place edit after the
        # forward raises instead of silently changing the embedding gradient)
        ctx.save_for_backward(his, *params)
        return _segno_forward(ctx, model, h, x, v, edge_attr, T, B, N)

    @staticmethod
    def backward(ctx, gx, gh, gv):
        model = ctx.model
        his = ctx.saved_tensors[0]
        grads, g_h, g_x, g_v = _segno_backward(ctx, gx, gh, gv, True, *ctx.needs_input_grad[2:4])
        L = _lib.lib()
        n, din = his.shape
        gw = torch.empty_like(model.embedding.weight)
        gb = torch.empty_like(model.embedding.bias)
        ws_bytes = L.nonode_embedding_backward_workspace_bytes(n, din)
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=g_h.device)
        _lib.check(L.nonode_embedding_backward(n, din, _lib.ptr(his), _lib.ptr(g_h), _lib.ptr(gw), _lib.ptr(gb),
                                               _lib.ptr(ws), ws_bytes, _lib.stream_of(g_h)))
        # dL/dhis of the embedding Linear (model.py:73), only when the caller's his requires grad
        g_his = (g_h @ _f32(model.embedding.weight)).to(ctx.his_dtype) if ctx.needs_input_grad[1] else None
        out = [grads.get(nm) for nm, _ in model.module.named_parameters(prefix="module")]
        return (None, g_his, g_x, g_v, None, None, None, None, gw, gb) + tuple(out)


def segno_train(model, his, x, v, edge_attr, T, B, N):
    """SEGNO.forward (one input, training): embedding + T substeps on the autograd tape."""
    params = [model.embedding.weight, model.embedding.bias] + [p for _, p in model.module.named_parameters()]
    return SEGNOTrain.apply(model, his, x, v, edge_attr, T, B, N, *params)


# ---- EGNO(flat=True) training (main_simulation_simple_no.py --flat; basic.py:38-40) ------------------
# One autograd node per layer: TimeConv + TimeConv_x (nonode_egno_tconv / nonode_egno_tconv_bwd) and the
# flat EGNN layer (nonode_egnn_layer_flat / nonode_egnn_layer_flat_bwd: the per-node and per-edge reverse
# of the 256-wide Tanh MLPs as HIP kernels). The weight gradients are sums over nodes or edges of the
# operand rows the reverse kernels write, i.e. plain GEMMs (torch.mm on the device: hipBLASLt / rocBLAS).
# The embedding Linear and the T-fold replication (egno.py:63-96) stay torch ops on the tape.
_FN = dict(GHP=0, GM=64, GF=128, GX=132, GA=136, GB=392, T=648, GT=904, U=1160, GU=1416, GPHI=1672, STRIDE=1676)
_FE = dict(A=0, M=256, C1=320, GZ3=576, GZ2=832, GPRE=896, GC=1152, S=1153, FE=1154, STRIDE=1160)


def _flat_layer_params(model, i):
    lay = model.layers[i]
    e, c, v, n = (lay.edge_message_net.scalar_net.mlp, lay.coord_net.mlp, lay.node_v_net.mlp, lay.node_net.mlp)
    return [e[0].weight, e[0].bias, e[2].weight, e[2].bias, c[0].weight, c[0].bias, c[2].weight, c[2].bias,
            v[0].weight, v[0].bias, v[2].weight, v[2].bias, n[0].weight, n[0].bias, n[2].weight, n[2].bias]


class FlatLayerTrain(torch.autograd.Function):
    """TimeConv (+ TimeConv_x) of layer i, then its flat EGNN layer (egno.py:99-111 with flat=True)."""

    @staticmethod
    def forward(ctx, model, i, B, N, h, x, v, loc_mean, ef, *params):
        L = _lib.lib()
        T = model.num_timesteps
        dev = h.device
        BN, n = B * N, T * B * N
        h, x, v, ef = _f32(h), _f32(x), _f32(v), _f32(ef)
        blobs, tblobs = model._packed()
        s = _lib.stream_of(h)
        if model.use_time_conv:
            lm = _f32(loc_mean)
            tcx = _f32(model.time_conv_x_modules[i].t_conv.weights1)
            ht, xt, vt = torch.empty(n, 64, device=dev), torch.empty(n, 3, device=dev), torch.empty(n, 3, device=dev)
            _lib.check(L.nonode_egno_tconv(BN, T, model.num_modes, _lib.ptr(h), _lib.ptr(x), _lib.ptr(v), _lib.ptr(lm),
                                           _lib.ptr(tblobs[i]), _lib.ptr(tcx), _lib.ptr(ht), _lib.ptr(xt), _lib.ptr(vt),
                                           s))
        else:
            lm, ht, xt, vt = None, h, x, v
        state = torch.empty(L.nonode_egnn_layer_flat_state_floats(T * B, N), device=dev)
        h_out, x_out = torch.empty(n, 64, device=dev), torch.empty(n, 3, device=dev)
        _lib.check(L.nonode_egnn_layer_flat(T * B, N, model.in_edge_nf, B, _lib.ptr(ht), _lib.ptr(xt), _lib.ptr(vt),
                                            _lib.ptr(ef), _lib.ptr(blobs[i]), _lib.ptr(h_out), _lib.ptr(x_out),
                                            _lib.ptr(state), s))
        ctx.set_materialize_grads(False)
        ctx.model, ctx.i, ctx.B, ctx.N = model, i, B, N
        ctx.keep = (h, x, v, lm, ef, ht, xt, vt, state)
        ctx.save_for_backward(*params)
        return h_out, x_out, vt.clone() if vt is v else vt

    @staticmethod
    def backward(ctx, gh, gx, gv):
        model, i, B, N = ctx.model, ctx.i, ctx.B, ctx.N
        params = ctx.saved_tensors
        h, x, v, lm, ef, ht, xt, vt, state = ctx.keep
        ctx.keep = None
        L = _lib.lib()
        T = model.num_timesteps
        dev = h.device
        n, E = T * B * N, T * B * N * (N - 1)
        z = lambda k: torch.zeros(n, k, device=dev)  # noqa: E731
        gh = _f32(gh) if gh is not None else z(64)
        gx = _f32(gx) if gx is not None else z(3)
        gv = _f32(gv) if gv is not None else z(3)
        blobs, _ = model._packed()
        bb = model._packed_flat_bwd()
        nops = torch.empty(n, _FN["STRIDE"], device=dev)
        eops = torch.empty(E, _FE["STRIDE"], device=dev)
        gvt = torch.empty(n, 3, device=dev)
        s = _lib.stream_of(gh)
        _lib.check(L.nonode_egnn_layer_flat_bwd(T * B, N, model.in_edge_nf, B, _lib.ptr(ht), _lib.ptr(xt), _lib.ptr(vt),
                                                _lib.ptr(ef), _lib.ptr(blobs[i]), _lib.ptr(bb[i]), _lib.ptr(state),
                                                _lib.ptr(gx), _lib.ptr(gv), _lib.ptr(gh), _lib.ptr(nops), _lib.ptr(eops),
                                                _lib.ptr(gvt), s))
        cols = lambda a, k, w: a[:, k:k + w]  # noqa: E731
        F_, E_ = _FN, _FE
        GA, GB = cols(nops, F_["GA"], 256), cols(nops, F_["GB"], 256)
        gpre, a_, m_ = cols(eops, E_["GPRE"], 256), cols(eops, E_["A"], 256), cols(eops, E_["M"], 64)
        gz3, gz2, c1 = cols(eops, E_["GZ3"], 256), cols(eops, E_["GZ2"], 64), cols(eops, E_["C1"], 256)
        gc, sr = eops[:, E_["GC"]], eops[:, E_["S"]]
        gt, t_ = cols(nops, F_["GT"], 256), cols(nops, F_["T"], 256)
        gu, u_ = cols(nops, F_["GU"], 256), cols(nops, F_["U"], 256)
        gphi = nops[:, F_["GPHI"]]
        M = state[n * 512:n * 576].view(n, 64)
        w1 = params[0]
        ne = model.in_edge_nf
        # the first Linear's columns [s, h_i, h_j, e] (EGNO order): GA / GB carry its h_i / h_j parts
        dw1 = torch.cat([(gpre.t() @ sr)[:, None], GA.t() @ ht, GB.t() @ ht] +
                        ([gpre.t() @ eops[:, E_["FE"]:E_["FE"] + ne]] if ne else []), 1)
        grads = [dw1, GA.sum(0), gz2.t() @ a_, gz2.sum(0),              # edge MLP
                 gz3.t() @ m_, gz3.sum(0), (gc @ c1)[None], gc.sum()[None],   # coord MLP
                 gt.t() @ ht, gt.sum(0), (gphi @ t_)[None], gphi.sum()[None],  # node_v MLP
                 gu.t() @ torch.cat([ht, M], 1), gu.sum(0), gh.t() @ u_, gh.sum(0)]   # node MLP
        ght = cols(nops, F_["GHP"], 64) + GA @ w1[:, 1:65] + GB @ w1[:, 65:129]
        gxt = cols(nops, F_["GX"], 3).contiguous()
        ght = ght.contiguous()
        grads = [g.reshape(p.shape).to(p.dtype) for g, p in zip(grads, params[:16])]
        if not model.use_time_conv:
            return (None,) * 4 + (ght, gxt, gvt, None, None) + tuple(grads)
        g_h, g_x, g_v = torch.empty_like(h), torch.empty_like(x), torch.empty_like(v)
        tw, txw = _f32(params[16]), _f32(params[17])      # kept alive over the call
        g_tw, g_txw = torch.empty_like(tw), torch.empty_like(txw)
        ws_bytes = L.nonode_egno_tconv_bwd_workspace_bytes(B * N, T, model.num_modes)
        ws = torch.empty((ws_bytes + 3) // 4, device=dev)
        _, tblobs = model._packed()
        _lib.check(L.nonode_egno_tconv_bwd(B * N, T, model.num_modes, _lib.ptr(h), _lib.ptr(x), _lib.ptr(v), _lib.ptr(lm),
                                           _lib.ptr(tblobs[i]), _lib.ptr(tw), _lib.ptr(txw), _lib.ptr(ght),
                                           _lib.ptr(gxt), _lib.ptr(gvt), _lib.ptr(g_h), _lib.ptr(g_x), _lib.ptr(g_v),
                                           _lib.ptr(g_tw), _lib.ptr(g_txw), _lib.ptr(ws), ws_bytes, s))
        sink = getattr(model, "_train_bwd_sink", None)
        if sink is not None:   # tests: the workspace head holds the LeakyReLU decisions the reverse used
            sink.append((i, ws))
        return (None,) * 4 + (g_h, g_x, g_v, None, None) + tuple(grads) + (g_tw.to(params[16].dtype),
                                                                             g_txw.to(params[17].dtype))


def egno_flat_train(model, x, h, edge_fea, v, loc_mean, t_out, B, N):
    """EGNO(flat=True).forward in training (egno.py:37-111, num_inputs == 1): the time embedding and the
    embedding Linear as torch ops, then one FlatLayerTrain node per layer."""
    import math
    T = model.num_timesteps
    BN = B * N
    dim, half = model.time_emb_dim, model.time_emb_dim // 2
    # get_timestep_embedding (layer_no.py:8-17)
    freqs = torch.exp(torch.arange(half, dtype=torch.float32, device=x.device) * -(math.log(10000) / (half - 1)))
    ang = t_out.float()[..., None] * freqs
    temb = torch.cat([torch.sin(ang), torch.cos(ang)], dim=-1)
    if dim % 2 == 1:
        temb = torch.nn.functional.pad(temb, (0, 1))
    Bt = temb.shape[0]
    temb = temb.permute(1, 0, 2)[:, None].repeat(1, BN // Bt, 1, 1).reshape(T, BN, -1)   # egno.py:66
    hh = model.embedding(torch.cat([h.float()[None].expand(T, -1, -1), temb], -1).reshape(T * BN, -1))
    xx, vv = x.float().repeat(T, 1), v.float().repeat(T, 1)                             # egno.py:89-96
    lm = loc_mean.float() if model.use_time_conv else None
    for i in range(model.n_layers):
        params = _flat_layer_params(model, i)
        if model.use_time_conv:
            params += [model.time_conv_modules[i].t_conv.weights1, model.time_conv_x_modules[i].t_conv.weights1]
        hh, xx, vv = FlatLayerTrain.apply(model, i, B, N, hh, xx, vv, lm, edge_fea, *params)
    return xx, vv, hh
