"""Generate tests/golden/egno_layer_grads.npz: the REFERENCE's autograd at the granularity of one
EGNN_Layer (EGNO/model/basic.py:167-186) and one TimeConv / TimeConv_x (layer_no.py:80-178), in the
training step of tests/golden/egno_grad.npz (egno_fwd.npz's weights and inputs, its loc_true, the
loss of main_simulation_simple_no.py:267-280).

For every layer i the reference's own modules run unchanged; their forwards are wrapped so that each
block's inputs and outputs are separate autograd nodes (x.clone() is the identity for values and
gradients) and keep their .grad. Recorded per block: the inputs, the gradients of the outputs and of
the inputs; and every parameter's gradient. These pin the layer-granular C entry points
(nonode_egnn_layer_bwd, nonode_egno_tconv_bwd) to the reference's per-block reverse.

Test infrastructure only (build container). Data only; no reference source is copied. Re-run:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_layer_grads.py
"""
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.set_num_threads(8)
tg = types.ModuleType("torch_geometric")
tg.utils = types.ModuleType("torch_geometric.utils")
tg.utils.to_dense_batch = lambda x, b: (x.reshape(int(b.max()) + 1, -1, *x.shape[1:]), None)
tg.data = types.ModuleType("torch_geometric.data")
tg.data.Data = dict
sys.modules.update({"torch_geometric": tg, "torch_geometric.utils": tg.utils, "torch_geometric.data": tg.data})
sys.path.insert(0, REF)
from EGNO.model.egno import EGNO  # noqa: E402


def _np(t):
    return t.detach().cpu().numpy().copy() if t is not None else None


def main():
    fx = dict(np.load(os.path.join(HERE, "egno_fwd.npz")))
    gd = dict(np.load(os.path.join(HERE, "egno_grad.npz")))
    B, N, T = int(fx["cfg::B"]), int(fx["cfg::N"]), int(fx["cfg::T"])
    model = EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, device="cpu", with_v=True, num_modes=2,
                 num_timesteps=T, time_emb_dim=32)
    model.load_state_dict({k[3:]: torch.tensor(v) for k, v in fx.items() if k.startswith("w::")})
    model.train()
    cap = {}

    def wrap(name, module, layer):
        orig = module.forward

        def fwd(*args, **kw):
            args = [a.clone() if torch.is_tensor(a) and a.is_floating_point() else a for a in args]
            kw = {k: (v.clone() if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in kw.items()}
            ins = [a for a in args if torch.is_tensor(a) and a.is_floating_point()] + [v for v in kw.values()
                                                                                      if torch.is_tensor(v)]
            for a in ins:
                a.retain_grad()
            out = orig(*args, **kw)
            outs = [o.clone() for o in out] if isinstance(out, tuple) else [out.clone()]
            for o in outs:
                o.retain_grad()
            cap[name] = (ins, outs)
            return tuple(outs) if isinstance(out, tuple) else outs[0]
        module.forward = fwd

    for i in range(4):
        wrap(f"lay{i}", model.layers[i], True)
        wrap(f"tc{i}", model.time_conv_modules[i], False)
        wrap(f"tcx{i}", model.time_conv_x_modules[i], False)
    # every float input requires grad so that each block input carries a .grad (the parameter
    # gradients do not change)
    g = lambda k: torch.tensor(fx["in::" + k]).requires_grad_(fx["in::" + k].dtype.kind == "f")  # noqa: E731
    model.zero_grad()
    x, v, h = model(g("x"), g("h"), [g("row"), g("col")], g("edge_attr"), v=g("v"), loc_mean=g("loc_mean"),
                    timesteps_out=g("t_out"))
    loc_pred = x.reshape(T, -1, 3).transpose(0, 1).reshape(B, N, T, 3)
    losses = torch.nn.MSELoss(reduction="none")(loc_pred, torch.tensor(gd["in::loc_true"])).mean((0, 1, 3))
    loss = losses.mean()
    loss.backward()
    assert abs(float(loss) - float(gd["out::loss"])) <= 1e-6 * abs(float(gd["out::loss"]))
    # kept: layers 1 (every output gradient nonzero) and 3 (the last: its h output does not reach the
    # loss, so dL/dh_out = 0), to keep the fixture small
    keep = (1, 3)
    out = {"cfg::B": B, "cfg::N": N, "cfg::T": T, "cfg::layers": np.array(keep), "out::loss": _np(loss)}
    for name, (ins, outs) in cap.items():
        if int(name[-1]) not in keep:
            continue
        for j, a in enumerate(ins):
            out[f"{name}::in{j}"] = _np(a)
            out[f"{name}::gin{j}"] = _np(a.grad) if a.grad is not None else np.zeros(tuple(a.shape), np.float32)
        for j, o in enumerate(outs):
            out[f"{name}::gout{j}"] = _np(o.grad) if o.grad is not None else np.zeros(tuple(o.shape), np.float32)
    for k, p in model.named_parameters():
        if any(k.startswith(f"{pre}.{i}.") for pre in ("layers", "time_conv_modules", "time_conv_x_modules")
               for i in keep):
            out["grad::" + k] = _np(p.grad) if p.grad is not None else np.zeros(tuple(p.shape), np.float32)
    np.savez_compressed(os.path.join(HERE, "egno_layer_grads.npz"), **out)
    print("wrote egno_layer_grads.npz", sorted(k for k in out if k.startswith("lay1")))


if __name__ == "__main__":
    main()
