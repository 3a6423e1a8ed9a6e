"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Test infrastructure only. This script imports simone7monaco/NO-NODE-comparison from
/root/reference (available in the build container, never on the GPU box) and records
inputs, weights and outputs as small .npz files. The fixtures are data; no reference
source is copied. Re-run with:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What each fixture pins (reference file:line):
  egno_fwd.npz        EGNO.forward (EGNO/model/egno.py:37-111) at B=4,N=20,T=10, plus the
                      per-layer states after TimeConv / TimeConv_x / EGNN_Layer
                      (layer_no.py:112-178, basic.py:167-186) and the timestep embedding
                      (layer_no.py:8-17). Inputs come from the reference ChargedParticlesSim
                      (synthetic_sim.py:220-296, np seed 43) through prepare_inputs
                      (main_simulation_simple_no.py:311-339).
  egno_rollout.npz    rollout_fn (main_simulation_simple_no.py:342-384), 2 segments, with the
                      per-frame conserved energy (utils.py:126-144,197-219).
  egno_grad.npz       one training step's loss + parameter gradients
                      (main_simulation_simple_no.py:267-280).
  segno_fwd.npz       SEGNO_GCL.forward (gcl.py:111-119), SEGNO.forward_step T=10
                      (model.py:95-102) and the live SEGNO.forward (model.py:53-92).
  segno_rollout.npz   train_nbody.rollout_fn (train_nbody.py:200-236), 2 segments, driven
                      through forward_step (the integrator the shadowed forward intends).
  segno_gravity.npz   forward_step at N=100, B=2, T=5 on GravitySim-style inputs
                      (synthetic_sim.py:360-404).
  egno_m5.npz         EGNO.forward with num_modes=5, num_timesteps=8, and one training step's loss and
                      gradients there (5 spectral modes incl. the
                      Nyquist bin; model_confs.yaml:12's alternative), seed-0 weights.
  egno_multi.npz      EGNO.forward with num_inputs=3 (multi-input branch, egno.py:44-96), seed-0 weights,
                      and one training step's parameter gradients; egno_multi_rollout.npz: its
                      2-segment rollout_fn with energies.
  segno_multi.npz     SEGNO live forward with num_inputs=3, multiple_agg='attn' (model.py:53-92,
                      104-139) and the discarded last forward_step; segno_multi_rollout.npz: the
                      2-segment num_prev = 3 rollout_fn through the integrator.
  segno_grad.npz      one SEGNO training step of run_epoch (train_nbody.py:150-178, num_inputs=1)
                      routed through forward_step (model.py:95-102, the integrator): criterion =
                      nn.MSELoss (train_nbody.py:31), loss and every parameter gradient, T=10.
  egno_norm.npz       EGNO(norm=True) (InvariantScalarNet's F.normalize of the radial input,
                      basic.py:140-141) at B=2,N=5,T=10, one pair of coincident nodes (radial
                      below the 1e-12 eps), seed-2 weights: forward + one training step's gradients.
  egno_notc.npz       EGNO(use_time_conv=False) (no TimeConv modules, egno.py:27-33, 99-107 skipped),
                      seed-3 weights recorded right after construction: forward + gradients.
  segno_tanh.npz      SEGNO(tanh=True, norm_diff=True) (coord_mlp ends in nn.Tanh, gcl.py:57-59;
                      norm_diff is stored and unused), seed-4 weights: forward_step T=10 + one
                      training step's gradients through it.
  init_seed0.npz      state_dicts produced by EGNO(...)/SEGNO(...) right after
                      torch.manual_seed(0) (RNG-consumption order of the constructors).
"""
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

import numpy as np
import torch

torch.set_num_threads(8)


# ---------------------------------------------------------------------------------
# Stubs for the reference's non-arithmetic dependencies that are not installed here.
# torch_geometric is used only for equal-size to_dense_batch reshapes and the Data
# container; wandb only for logging.
# ---------------------------------------------------------------------------------
def _to_dense_batch(x, batch):
    B = int(batch.max().item()) + 1
    n = x.shape[0] // B
    out = x.reshape(B, n, *x.shape[1:])
    return out, torch.ones(B, n, dtype=torch.bool)


tg = types.ModuleType("torch_geometric")
tg_utils = types.ModuleType("torch_geometric.utils")
tg_utils.to_dense_batch = _to_dense_batch
tg_data = types.ModuleType("torch_geometric.data")
tg_data.Data = dict
tg.utils, tg.data = tg_utils, tg_data
sys.modules.update({"torch_geometric": tg, "torch_geometric.utils": tg_utils,
                    "torch_geometric.data": tg_data})
wb = types.ModuleType("wandb")
wb.log = lambda *a, **k: None
sys.modules["wandb"] = wb

sys.path.insert(0, REF)
import utils as ref_utils  # noqa: E402  (root utils.py)
import EGNO.utils as egno_utils  # noqa: E402

egno_utils.random_ascending_tensor = ref_utils.random_ascending_tensor
from EGNO.model.egno import EGNO  # noqa: E402
from EGNO.model.layer_no import get_timestep_embedding  # noqa: E402
import EGNO.main_simulation_simple_no as egno_main  # noqa: E402
from synthetic_sim import ChargedParticlesSim  # noqa: E402

sys.path.insert(0, os.path.join(REF, "SEGNO"))
from models.model import SEGNO  # noqa: E402
import train_nbody as segno_train  # noqa: E402  (SEGNO/train_nbody.py)


def _np(t):
    return t.detach().cpu().numpy().copy()


def _sd(model, prefix="w::"):
    return {prefix + k: _np(v) for k, v in model.state_dict().items()}


def full_edges(B, N):
    """Same edge list as dataset_simple.py:64-71 + get_edges 101-111."""
    rows, cols = [], []
    for i in range(N):
        for j in range(N):
            if i != j:
                rows.append(i)
                cols.append(j)
    r = torch.tensor(rows)
    c = torch.tensor(cols)
    return [torch.cat([r + N * b for b in range(B)]), torch.cat([c + N * b for b in range(B)])]


def charged_trajectories(S, N, T=6000, freq=100, seed=43):
    np.random.seed(seed)
    sim = ChargedParticlesSim(n_balls=N, box_size=5.0, noise_var=0.0, vel_norm=0.5)
    locs, vels, charges = [], [], []
    for _ in range(S):
        loc, vel, edges, q = sim.sample_trajectory(T=T, sample_freq=freq)
        locs.append(loc)
        vels.append(vel)
        charges.append(q)
    # on-disk layout [S, frames, 3, N] -> loader transposes to [S, frames, N, 3]
    loc = np.ascontiguousarray(np.transpose(np.stack(locs), (0, 1, 3, 2)).astype(np.float32))
    vel = np.ascontiguousarray(np.transpose(np.stack(vels), (0, 1, 3, 2)).astype(np.float32))
    q = np.stack(charges).astype(np.float32)  # [S, N, 1]
    return loc, vel, q


def edge_attr_o(q):
    """q_i q_j per edge in (i, j != i) order, as dataset_simple.py:46-48,64-72."""
    S, N, _ = q.shape
    out = []
    for s in range(S):
        qq = q[s, :, 0]
        out.append([qq[i] * qq[j] for i in range(N) for j in range(N) if i != j])
    return torch.tensor(np.array(out, dtype=np.float32)).unsqueeze(-1)  # [S, N(N-1), 1]


def make_egno(B=4, N=20, T=10, traj_len=2):
    loc_all, vel_all, q = charged_trajectories(B, N)
    start = 30
    loc = torch.tensor(np.ascontiguousarray(loc_all[:, start]))
    vel = torch.tensor(np.ascontiguousarray(vel_all[:, start]))
    charges = torch.tensor(q)
    eao = edge_attr_o(q).reshape(-1, 1)
    edges = full_edges(B, N)
    loc_p, vel_p, edge_attr, nodes, loc_mean = egno_main.prepare_inputs(
        loc, vel, eao, edges, N, 1, charges)
    t_out = torch.arange(1, T + 1).repeat(B, 1)  # out_indices - in_indices.max()
    t_in = torch.zeros(B, dtype=torch.long)

    torch.manual_seed(0)
    model = EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True,
                 num_modes=2, num_timesteps=T, time_emb_dim=32)
    model.eval()

    # per-layer capture via forward hooks (EGNO/model/egno.py:99-110)
    cap = {}

    def hook(name):
        def f(mod, inp, out):
            if isinstance(out, tuple):
                for k, o in enumerate(out):
                    cap[f"{name}.out{k}"] = _np(o)
            else:
                cap[f"{name}.out"] = _np(out)
            cap[f"{name}.in0"] = _np(inp[0])
        return f

    for i in range(4):
        model.time_conv_modules[i].register_forward_hook(hook(f"tconv{i}"))
        model.time_conv_x_modules[i].register_forward_hook(hook(f"tconvx{i}"))
        model.layers[i].register_forward_hook(hook(f"layer{i}"))
    model.embedding.register_forward_hook(hook("embedding"))

    with torch.no_grad():
        x_out, v_out, h_out = model(loc_p, nodes, edges, edge_attr, v=vel_p, loc_mean=loc_mean,
                                    timesteps_in=t_in, timesteps_out=t_out)
    temb = get_timestep_embedding(t_out, embedding_dim=32, max_positions=10000)

    fx = dict(_sd(model))
    fx.update({f"cap::{k}": v for k, v in cap.items()})
    fx.update({
        "cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T),
        "raw::loc": loc_all[:, start], "raw::vel": vel_all[:, start], "raw::charges": q,
        "raw::edge_attr_o": _np(eao),
        "in::x": _np(loc_p), "in::h": _np(nodes), "in::v": _np(vel_p),
        "in::loc_mean": _np(loc_mean), "in::edge_attr": _np(edge_attr),
        "in::row": _np(edges[0]), "in::col": _np(edges[1]),
        "in::t_out": _np(t_out), "in::t_in": _np(t_in),
        "out::x": _np(x_out), "out::v": _np(v_out), "out::h": _np(h_out),
        "out::temb": _np(temb),
        "truth::locs_out": loc_all[:, start + 1:start + 1 + T * traj_len],  # [B, T*traj, N, 3]
        "truth::vels_out": vel_all[:, start + 1:start + 1 + T * traj_len],
    })
    np.savez_compressed(os.path.join(HERE, "egno_fwd.npz"), **fx)

    # ---- rollout (main_simulation_simple_no.py:342-384) with conserved energy ----
    class _DS:  # energy_fun as dataset_simple.py:33-34
        dataset = "charged"

        def energy_fun(self, loc, vel, edges, batch=None):
            return ref_utils.conserved_energy_fun("charged", loc, vel, edges, batch=batch)

    t_out_full = torch.arange(1, T * traj_len + 1).repeat(B, 1)
    with torch.no_grad():
        preds, energies, energies_all = egno_main.rollout_fn(
            model, nodes, loc_p, edges, vel_p, eao, edge_attr, loc_mean, N, traj_len, B,
            charges=charges, num_steps=T, timesteps_in=t_in.clone(),
            timesteps_out=t_out_full.clone(), energy_fun=_DS().energy_fun)
    np.savez_compressed(os.path.join(HERE, "egno_rollout.npz"), **{
        "cfg::traj_len": np.array(traj_len),
        "out::loc_preds": _np(preds), "out::energies": _np(energies),
        "out::energies_allsteps": _np(energies_all),
    })

    # ---- one training step gradient (main_simulation_simple_no.py:267-280) ----
    model.train()
    model.zero_grad()
    loc_true = torch.tensor(loc_all[:, start + 1:start + 1 + T]).transpose(1, 2)  # [B,N,T,3]
    crit = torch.nn.MSELoss(reduction="none")
    loc_pred, _, _ = model(loc_p, nodes, edges, edge_attr, v=vel_p, loc_mean=loc_mean,
                           timesteps_in=t_in, timesteps_out=t_out)
    loc_pred = loc_pred.reshape(T, -1, 3).transpose(0, 1)
    loc_pred = _to_dense_batch(loc_pred, torch.arange(B).repeat_interleave(N))[0]
    losses = crit(loc_pred, loc_true[:, :, :loc_pred.size(2)]).mean((0, 1, 3))
    loss = losses.mean()
    loss.backward()
    # parameters that do not reach the loss (layers.3.node_net: the last h is unused) get
    # grad None in torch; they are recorded as zeros.
    g = {"grad::" + k: (_np(p.grad) if p.grad is not None else np.zeros(tuple(p.shape), np.float32))
         for k, p in model.named_parameters()}
    g["nograd"] = np.array([k for k, p in model.named_parameters() if p.grad is None])
    g["out::loss"] = _np(loss)
    g["out::losses"] = _np(losses)
    g["in::loc_true"] = _np(loc_true)
    np.savez_compressed(os.path.join(HERE, "egno_grad.npz"), **g)
    return model


def make_segno(B=4, N=20, T=10):
    loc_all, vel_all, q = charged_trajectories(B, N, seed=44)
    start = 30
    edges = full_edges(B, N)
    rows, cols = edges
    loc = torch.tensor(np.ascontiguousarray(loc_all[:, start])).reshape(-1, 3)
    vel = torch.tensor(np.ascontiguousarray(vel_all[:, start])).reshape(-1, 3)
    charges = torch.tensor(q).reshape(-1, 1)
    prod = charges[rows] * charges[cols]
    h = torch.sqrt(torch.sum(vel ** 2, dim=1)).unsqueeze(-1)  # train_nbody.py:121
    loc_dist = torch.sum((loc[rows] - loc[cols]) ** 2, 1).unsqueeze(1)
    edge_attr = torch.cat([prod, loc_dist], 1)  # train_nbody.py:123

    torch.manual_seed(0)
    model = SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True,
                  norm_diff=False, tanh=False, device="cpu", varDT=False, multiple_agg=None)
    model.eval()
    edge_index = torch.stack(edges)
    with torch.no_grad():
        h_emb = model.embedding(h)
        model.module.n_layers = T
        gcl_h, gcl_x, gcl_v, _ = model.module(h_emb, edge_index, loc, vel, vel, edge_attr=edge_attr)
        fs_x, fs_h, fs_v = model.forward_step(h_emb, loc, edge_index, vel, edge_attr, T=T)
        fw_x, fw_h, fw_v = model(h, loc, edges, vel, edge_attr, T=T)
    fx = dict(_sd(model))
    fx.update({
        "cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T),
        "raw::charges": q,
        "in::x": _np(loc), "in::v": _np(vel), "in::his": _np(h), "in::edge_attr": _np(edge_attr),
        "in::row": _np(rows), "in::col": _np(cols), "in::h_emb": _np(h_emb),
        "gcl::h": _np(gcl_h), "gcl::x": _np(gcl_x), "gcl::v": _np(gcl_v),
        "step::x": _np(fs_x), "step::h": _np(fs_h), "step::v": _np(fs_v),
        "fwd::x": _np(fw_x), "fwd::h": _np(fw_h), "fwd::v": _np(fw_v),
    })
    np.savez_compressed(os.path.join(HERE, "segno_fwd.npz"), **fx)

    # ---- rollout through the integrator (train_nbody.py:200-236) ----
    class _Integrator(torch.nn.Module):
        """Routes the reference rollout_fn through SEGNO.forward_step (model.py:95-102)."""

        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, his, x, edges, v, edge_attr, T=10, in_steps=None):
            hh = self.m.embedding(his)
            xo, ho, vo = self.m.forward_step(hh, x, edges, v, edge_attr, T=T)
            return xo, ho, vo

    batch = torch.arange(B).repeat_interleave(N)
    with torch.no_grad():
        preds, energies = segno_train.rollout_fn(
            _Integrator(model), h, loc, edge_index, vel, edge_attr, batch, 2,
            num_steps=[T, T // 2], num_prev=1, charges=charges,
            energy_fun=lambda l, v, e, batch=None: ref_utils.conserved_energy_fun(
                "charged", l, v, e, batch=batch))
    np.savez_compressed(os.path.join(HERE, "segno_rollout.npz"), **{
        "cfg::num_steps": np.array([T, T // 2]),
        "out::loc_preds": _np(preds), "out::energies": _np(energies)})


def make_segno_grad(B=4, N=20, T=10):
    """One training step (train_nbody.py:150-178) through forward_step. The live forward returns
    its inputs, so loss.backward() on it fails in the reference; the
    gradients recorded here are those of the integrator the shadowed forward intends."""
    loc_all, vel_all, q = charged_trajectories(B, N, seed=45)
    start = 20
    edges = full_edges(B, N)
    rows, cols = edges
    loc = torch.tensor(np.ascontiguousarray(loc_all[:, start])).reshape(-1, 3)
    vel = torch.tensor(np.ascontiguousarray(vel_all[:, start])).reshape(-1, 3)
    loc_end = torch.tensor(np.ascontiguousarray(loc_all[:, start + T])).reshape(-1, 3)
    charges = torch.tensor(q).reshape(-1, 1)
    prod = charges[rows] * charges[cols]
    h = torch.sqrt(torch.sum(vel ** 2, dim=1)).unsqueeze(-1)                     # train_nbody.py:121
    loc_dist = torch.sum((loc[rows] - loc[cols]) ** 2, 1).unsqueeze(1)
    edge_attr = torch.cat([prod, loc_dist], 1)                                     # train_nbody.py:123
    torch.manual_seed(1)
    model = SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True,
                  norm_diff=False, tanh=False, device="cpu", varDT=False, multiple_agg=None)
    model.train()
    model.zero_grad()
    edge_index = torch.stack(edges)
    hh = model.embedding(h)
    x_pred, h_pred, v_pred = model.forward_step(hh, loc.detach(), edge_index, vel.detach(), edge_attr, T=T)
    loss = torch.nn.MSELoss()(x_pred, loc_end)
    loss.backward()
    fx = dict(_sd(model))
    fx.update({
        "cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T),
        "in::x": _np(loc), "in::v": _np(vel), "in::his": _np(h), "in::edge_attr": _np(edge_attr),
        "in::row": _np(rows), "in::col": _np(cols), "in::loc_end": _np(loc_end),
        "out::x": _np(x_pred.detach()), "out::loss": np.array(float(loss.detach())),
    })
    for k, p in model.named_parameters():
        if p.grad is not None:
            fx["grad::" + k] = _np(p.grad)
    np.savez_compressed(os.path.join(HERE, "segno_grad.npz"), **fx)


def make_segno_gravity(B=2, N=100, T=5):
    rng = np.random.RandomState(7)
    # GravitySim init (synthetic_sim.py:370-378): masses, positions, velocities, COM removed
    mass = (1.0 + 0.1 * rng.randn(B, N, 1)).astype(np.float32)
    pos = rng.randn(B, N, 3).astype(np.float32)
    vel = rng.randn(B, N, 3).astype(np.float32)
    vel -= (mass * vel).sum(1, keepdims=True) / mass.sum(1, keepdims=True)
    edges = full_edges(B, N)
    rows, cols = edges
    loc = torch.tensor(pos).reshape(-1, 3)
    v = torch.tensor(vel).reshape(-1, 3)
    m = torch.tensor(mass).reshape(-1, 1)
    prod = m[rows] * m[cols]
    h = torch.sqrt(torch.sum(v ** 2, dim=1)).unsqueeze(-1)
    loc_dist = torch.sum((loc[rows] - loc[cols]) ** 2, 1).unsqueeze(1)
    edge_attr = torch.cat([prod, loc_dist], 1)
    torch.manual_seed(1)
    model = SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True,
                  norm_diff=False, tanh=False, device="cpu")
    with torch.no_grad():
        hh = model.embedding(h)
        xo, ho, vo = model.forward_step(hh, loc, torch.stack(edges), v, edge_attr, T=T)
    fx = dict(_sd(model))
    fx.update({"cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T),
               "in::x": _np(loc), "in::v": _np(v), "in::his": _np(h),
               "in::edge_attr": _np(edge_attr), "in::mass": mass,
               "step::x": _np(xo), "step::h": _np(ho), "step::v": _np(vo)})
    np.savez_compressed(os.path.join(HERE, "segno_gravity.npz"), **fx)


def make_init():
    torch.manual_seed(0)
    e = EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
             num_timesteps=10, time_emb_dim=32)
    torch.manual_seed(0)
    s = SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True,
              norm_diff=False, tanh=False)
    fx = _sd(e, "egno::")
    fx.update(_sd(s, "segno::"))
    np.savez_compressed(os.path.join(HERE, "init_seed0.npz"), **fx)


def make_egno_modes(B=2, N=5, T=8, modes=5):
    """EGNO.forward with num_modes=5 at num_timesteps=8 (model_confs.yaml:12's alternative value):
    M = min(T, modes) = 5 = T/2 + 1 spectral modes, so the Nyquist bin is mixed. Weights are the
    seed-0 initialisation (the drop-in reproduces the constructor's RNG order); only inputs,
    outputs and per-tensor weight sums (to confirm that initialisation) are stored."""
    loc_all, vel_all, q = charged_trajectories(B, N)
    start = 20
    loc = torch.tensor(np.ascontiguousarray(loc_all[:, start]))
    vel = torch.tensor(np.ascontiguousarray(vel_all[:, start]))
    eao = edge_attr_o(q).reshape(-1, 1)
    edges = full_edges(B, N)
    loc_p, vel_p, edge_attr, nodes, loc_mean = egno_main.prepare_inputs(
        loc, vel, eao, edges, N, 1, torch.tensor(q))
    t_out = torch.arange(1, T + 1).repeat(B, 1)
    torch.manual_seed(0)
    model = EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True,
                 num_modes=modes, num_timesteps=T, time_emb_dim=32)
    model.eval()
    with torch.no_grad():
        x_out, v_out, h_out = model(loc_p, nodes, edges, edge_attr, v=vel_p, loc_mean=loc_mean,
                                    timesteps_out=t_out)
    fx = {f"wsum::{k}": np.array(float(v.double().sum())) for k, v in model.state_dict().items()}
    fx.update({
        "cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T), "cfg::modes": np.array(modes),
        "in::x": _np(loc_p), "in::h": _np(nodes), "in::v": _np(vel_p),
        "in::loc_mean": _np(loc_mean), "in::edge_attr": _np(edge_attr),
        "in::row": _np(edges[0]), "in::col": _np(edges[1]), "in::t_out": _np(t_out),
        "out::x": _np(x_out), "out::v": _np(v_out), "out::h": _np(h_out),
    })
    # one training step's gradients at this configuration (main_simulation_simple_no.py:267-280, as
    # make_egno): the reverse of TimeConv / TimeConv_x at 5 modes
    model.train()
    model.zero_grad()
    loc_true = torch.tensor(loc_all[:, start + 1:start + 1 + T]).transpose(1, 2)  # [B,N,T,3]
    crit = torch.nn.MSELoss(reduction="none")
    loc_pred, _, _ = model(loc_p, nodes, edges, edge_attr, v=vel_p, loc_mean=loc_mean, timesteps_out=t_out)
    loc_pred = loc_pred.reshape(T, -1, 3).transpose(0, 1)
    loc_pred = _to_dense_batch(loc_pred, torch.arange(B).repeat_interleave(N))[0]
    losses = crit(loc_pred, loc_true[:, :, :loc_pred.size(2)]).mean((0, 1, 3))
    loss = losses.mean()
    loss.backward()
    fx.update({"grad::" + k: (_np(p.grad) if p.grad is not None else np.zeros(tuple(p.shape), np.float32))
               for k, p in model.named_parameters()})
    fx["out::loss"] = _np(loss)
    fx["in::loc_true"] = _np(loc_true)
    np.savez_compressed(os.path.join(HERE, "egno_m5.npz"), **fx)


def make_egno_multi(B=2, N=5, T=10, I=3):
    """EGNO.forward with num_inputs=3 (main.py --num_inputs; _schedule.yaml:58 sweeps 2 and 3):
    inputs are frames start-2 .. start of a reference trajectory through prepare_inputs'
    multi-input branch (main_simulation_simple_no.py:313-327); timesteps_in / _out as run_epoch
    adjusts them (in - max(in), out - max(in)). Seed-0 weights; inputs, outputs, weight sums."""
    loc_all, vel_all, q = charged_trajectories(B, N)
    start = 20
    loc = torch.tensor(np.ascontiguousarray(loc_all[:, start - I + 1:start + 1]))   # [B, I, N, 3]
    vel = torch.tensor(np.ascontiguousarray(vel_all[:, start - I + 1:start + 1]))
    eao = edge_attr_o(q).reshape(-1, 1)
    edges = full_edges(B, N)
    loc_p, vel_p, edge_attr, nodes, loc_mean = egno_main.prepare_inputs(
        loc, vel, eao, edges, N, I, torch.tensor(q))
    t_in = torch.arange(-I + 1, 1).repeat(B, 1)                  # [B, I]
    t_out = torch.arange(1, T + 1).repeat(B, 1)                  # [B, T]
    torch.manual_seed(0)
    model = EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True,
                 num_modes=2, num_timesteps=T, time_emb_dim=32, num_inputs=I)
    model.eval()
    with torch.no_grad():
        x_out, v_out, h_out = model(loc_p, nodes, edges, edge_attr, v=vel_p, loc_mean=loc_mean,
                                    timesteps_in=t_in, timesteps_out=t_out)
    fx = {f"wsum::{k}": np.array(float(v.double().sum())) for k, v in model.state_dict().items()}
    fx.update({
        "cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T), "cfg::I": np.array(I),
        "in::x": _np(loc_p), "in::h": _np(nodes), "in::v": _np(vel_p),
        "in::loc_mean": _np(loc_mean), "in::edge_attr": _np(edge_attr),
        "in::row": _np(edges[0]), "in::col": _np(edges[1]),
        "in::t_in": _np(t_in), "in::t_out": _np(t_out),
        "out::x": _np(x_out), "out::v": _np(v_out), "out::h": _np(h_out),
    })
    # one training step's gradients through the multi-input model (main_simulation_simple_no.py:267-280)
    model.train()
    model.zero_grad()
    loc_true = torch.tensor(loc_all[:, start + 1:start + 1 + T]).transpose(1, 2)  # [B, N, T, 3]
    loc_pred, _, _ = model(loc_p, nodes, edges, edge_attr, v=vel_p, loc_mean=loc_mean,
                           timesteps_in=t_in, timesteps_out=t_out)
    loc_pred = loc_pred.reshape(T, -1, 3).transpose(0, 1)
    loc_pred = _to_dense_batch(loc_pred, torch.arange(B).repeat_interleave(N))[0]
    loss = torch.nn.MSELoss(reduction="none")(loc_pred, loc_true).mean((0, 1, 3)).mean()
    loss.backward()
    fx.update({"grad::" + k: (_np(p.grad) if p.grad is not None else np.zeros(tuple(p.shape), np.float32))
               for k, p in model.named_parameters()})
    fx["out::loss"] = _np(loss)
    fx["in::loc_true"] = _np(loc_true)
    np.savez_compressed(os.path.join(HERE, "egno_multi.npz"), **fx)

    # ---- multi-input rollout_fn (main_simulation_simple_no.py:342-384), 2 segments, energies ----
    class _DS:
        def energy_fun(self, loc, vel, edges, batch=None):
            return ref_utils.conserved_energy_fun("charged", loc, vel, edges, batch=batch)

    model.eval()
    traj_len = 2
    t_out_full = torch.arange(1, T * traj_len + 1).repeat(B, 1)
    with torch.no_grad():
        preds, energies, energies_all = egno_main.rollout_fn(
            model, nodes, loc_p, edges, vel_p, eao, edge_attr, loc_mean, N, traj_len, B,
            charges=torch.tensor(q), num_steps=T, timesteps_in=t_in.clone(), timesteps_out=t_out_full.clone(),
            energy_fun=_DS().energy_fun)
    np.savez_compressed(os.path.join(HERE, "egno_multi_rollout.npz"), **{
        "cfg::traj_len": np.array(traj_len), "raw::edge_attr_o": _np(eao), "raw::charges": q,
        "in::t_out": _np(t_out_full), "out::loc_preds": _np(preds), "out::energies": _np(energies),
        "out::energies_all": _np(energies_all)})


def make_segno_multi(B=2, N=5, T=10, I=3):
    """SEGNO with num_inputs=3, multiple_agg='attn' (main.py:111): the live forward (model.py:53-92)
    on inputs taken as train_nbody.py:97-123 takes them (frames start-6, start-3, start; in_steps
    = indices - start; edge_attr from the last frame). Stores the reference forward's output
    (which stops before the last forward_step) and that last forward_step's
    result from the returned state."""
    loc_all, vel_all, q = charged_trajectories(B, N, seed=45)
    start = 30
    steps = [T // I] * (I - 1)
    indices = np.flip(start - np.cumsum([0] + steps)).copy()
    edges = full_edges(B, N)
    rows, cols = edges
    loc = torch.tensor(np.ascontiguousarray(loc_all[:, indices])).permute(0, 2, 1, 3).reshape(B * N, I, 3)
    vel = torch.tensor(np.ascontiguousarray(vel_all[:, indices])).permute(0, 2, 1, 3).reshape(B * N, I, 3)
    charges = torch.tensor(q).reshape(-1, 1)
    prod = charges[rows] * charges[cols]
    in_steps = torch.tensor(indices - start).int()
    h = torch.sqrt(torch.sum(vel ** 2, dim=-1)).unsqueeze(-1)                       # (BN, I, 1)
    loc_dist = torch.sum((loc[rows, -1, :] - loc[cols, -1, :]) ** 2, 1).unsqueeze(1)
    edge_attr = torch.cat([prod, loc_dist], 1)
    torch.manual_seed(0)
    model = SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True,
                  norm_diff=False, tanh=False, device="cpu", varDT=False, multiple_agg="attn")
    model.eval()
    with torch.no_grad():
        fx_, fh_, fv_ = model(h, loc, edges, vel, edge_attr, T=T, in_steps=in_steps)
        lx, lh, lv = model.forward_step(fh_, fx_, edges, fv_, edge_attr, T=T)
    fx = dict(_sd(model))
    fx.update({
        "cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T), "cfg::I": np.array(I),
        "in::x": _np(loc), "in::v": _np(vel), "in::his": _np(h), "in::edge_attr": _np(edge_attr),
        "in::row": _np(rows), "in::col": _np(cols), "in::in_steps": _np(in_steps),
        "fwd::x": _np(fx_), "fwd::h": _np(fh_), "fwd::v": _np(fv_),
        "last::x": _np(lx), "last::h": _np(lh), "last::v": _np(lv),
    })
    np.savez_compressed(os.path.join(HERE, "segno_multi.npz"), **fx)

    # ---- multi-input rollout_fn (train_nbody.py:200-236, num_prev = 3), through a wrapper whose
    # call runs the live forward and then the forward_step it discards (the integrator result) ----
    class _Integrated(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, his, x, edges, v, edge_attr, T=10, in_steps=None):
            xo, ho, vo = self.m(his, x, edges, v, edge_attr, T=T, in_steps=in_steps)
            return self.m.forward_step(ho, xo, edges, vo, edge_attr, T=T)

    batch = torch.arange(B).repeat_interleave(N)
    with torch.no_grad():
        preds, energies = segno_train.rollout_fn(
            _Integrated(model), h, loc, edges, vel, edge_attr, batch, 2, num_steps=[T, T // 2], num_prev=I,
            charges=charges, energy_fun=lambda l, v, e, batch=None: ref_utils.conserved_energy_fun(
                "charged", l, v, e, batch=batch), in_steps=in_steps.clone())
    np.savez_compressed(os.path.join(HERE, "segno_multi_rollout.npz"), **{
        "out::loc_preds": _np(preds), "out::energies": _np(energies), "raw::charges": _np(charges)})


def _egno_opt_case(B, N, seed):
    """prepare_inputs (main_simulation_simple_no.py:311-339) on reference ChargedParticlesSim frames."""
    loc_all, vel_all, q = charged_trajectories(B, N, seed=seed)
    start = 30
    loc = torch.tensor(np.ascontiguousarray(loc_all[:, start]))
    vel = torch.tensor(np.ascontiguousarray(vel_all[:, start]))
    eao = edge_attr_o(q).reshape(-1, 1)
    edges = full_edges(B, N)
    loc_p, vel_p, edge_attr, nodes, loc_mean = egno_main.prepare_inputs(loc, vel, eao, edges, N, 1, torch.tensor(q))
    return loc_all, start, edges, loc_p, vel_p, edge_attr, nodes, loc_mean


def _egno_opt(name, seed, B=2, N=5, T=10, coincide=False, **opts):
    loc_all, start, edges, x, v, ea, nodes, lm = _egno_opt_case(B, N, 46 + seed)
    if coincide:   # node 1 of graph 0 on top of node 0 with its velocity: radial 0 < eps on edges
        x, v = x.clone(), v.clone()   # (0, 1), (1, 0) through the TimeConvs into layer 0
        x[1] = x[0]
        v[1] = v[0]
        nodes = nodes.clone()
        nodes[1, 0] = nodes[0, 0]
        r, c = edges
        ea = ea.clone()
        ea[:, 1] = ((x[r] - x[c]) ** 2).sum(1)
    t_out = torch.arange(1, T + 1).repeat(B, 1)
    t_in = torch.zeros(B, dtype=torch.long)
    torch.manual_seed(seed)
    model = EGNO(n_layers=4, in_node_nf=2, in_edge_nf=2, hidden_nf=64, with_v=True, num_modes=2,
                 num_timesteps=T, time_emb_dim=32, **opts)
    fx = dict(_sd(model))
    model.eval()
    with torch.no_grad():
        xo, vo, ho = model(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_in=t_in, timesteps_out=t_out)
    model.train()
    model.zero_grad()
    loc_true = torch.tensor(loc_all[:, start + 1:start + 1 + T]).transpose(1, 2)   # [B, N, T, 3]
    xp, _, _ = model(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_in=t_in, timesteps_out=t_out)
    xp = _to_dense_batch(xp.reshape(T, -1, 3).transpose(0, 1), torch.arange(B).repeat_interleave(N))[0]
    loss = torch.nn.MSELoss(reduction="none")(xp, loc_true).mean((0, 1, 3)).mean()   # :267-277
    loss.backward()
    fx.update({"cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T),
               "in::x": _np(x), "in::h": _np(nodes), "in::v": _np(v), "in::loc_mean": _np(lm),
               "in::edge_attr": _np(ea), "in::row": _np(edges[0]), "in::col": _np(edges[1]),
               "in::t_out": _np(t_out), "in::loc_true": _np(loc_true),
               "out::x": _np(xo), "out::v": _np(vo), "out::h": _np(ho), "out::loss": np.array(float(loss))})
    for k, p in model.named_parameters():
        fx["grad::" + k] = _np(p.grad) if p.grad is not None else np.zeros(tuple(p.shape), np.float32)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **fx)


def make_segno_tanh(B=2, N=5, T=10, seed=4):
    loc_all, vel_all, q = charged_trajectories(B, N, seed=50)
    start = 20
    edges = full_edges(B, N)
    rows, cols = edges
    loc = torch.tensor(np.ascontiguousarray(loc_all[:, start])).reshape(-1, 3)
    vel = torch.tensor(np.ascontiguousarray(vel_all[:, start])).reshape(-1, 3)
    loc_end = torch.tensor(np.ascontiguousarray(loc_all[:, start + T])).reshape(-1, 3)
    charges = torch.tensor(q).reshape(-1, 1)
    h = torch.sqrt(torch.sum(vel ** 2, dim=1)).unsqueeze(-1)                     # train_nbody.py:121
    edge_attr = torch.cat([charges[rows] * charges[cols],
                           torch.sum((loc[rows] - loc[cols]) ** 2, 1).unsqueeze(1)], 1)   # :123
    torch.manual_seed(seed)
    model = SEGNO(in_node_nf=1, in_edge_nf=2, hidden_nf=64, n_layers=8, recurrent=True,
                  norm_diff=True, tanh=True, device="cpu", varDT=False, multiple_agg=None)
    fx = dict(_sd(model))
    edge_index = torch.stack(edges)
    model.train()
    model.zero_grad()
    hh = model.embedding(h)
    x_pred, h_pred, v_pred = model.forward_step(hh, loc, edge_index, vel, edge_attr, T=T)
    loss = torch.nn.MSELoss()(x_pred, loc_end)
    loss.backward()
    fx.update({"cfg::B": np.array(B), "cfg::N": np.array(N), "cfg::T": np.array(T),
               "in::x": _np(loc), "in::v": _np(vel), "in::his": _np(h), "in::edge_attr": _np(edge_attr),
               "in::row": _np(rows), "in::col": _np(cols), "in::loc_end": _np(loc_end),
               "out::x": _np(x_pred), "out::h": _np(h_pred), "out::v": _np(v_pred),
               "out::loss": np.array(float(loss))})
    for k, p in model.named_parameters():
        if p.grad is not None:
            fx["grad::" + k] = _np(p.grad)
    np.savez_compressed(os.path.join(HERE, "segno_tanh.npz"), **fx)


def make_flat():
    """EGNO(flat=True) (main_simulation_simple_no.py --flat: every BaseMLP 4x wide with Tanh,
    basic.py:38-40), seed-5 weights."""
    _egno_opt("egno_flat", 5, flat=True)


def make_options():
    _egno_opt("egno_norm", 2, coincide=True, norm=True)
    _egno_opt("egno_notc", 3, use_time_conv=False)
    make_segno_tanh()


if __name__ == "__main__":
    if sys.argv[1:] == ["options"]:
        make_options()
        sys.exit(0)
    if sys.argv[1:] == ["flat"]:
        make_flat()
        sys.exit(0)
    if sys.argv[1:] == ["segno_multi"]:
        make_segno_multi()
        sys.exit(0)
    if sys.argv[1:] == ["egno_m5"]:
        make_egno_modes()
        sys.exit(0)
    if sys.argv[1:] == ["segno_grad"]:
        make_segno_grad()
        sys.exit(0)
    if sys.argv[1:] == ["egno_multi"]:
        make_egno_multi()
        sys.exit(0)
    make_egno()
    make_segno()
    make_segno_gravity()
    make_init()
    with open(os.path.join(HERE, "PROVENANCE.txt"), "w") as f:
        f.write(f"generated by tests/golden/make_golden.py\n"
                f"reference snapshot: /root/reference (simone7monaco/NO-NODE-comparison 2025-07-04)\n"
                f"torch {torch.__version__}, numpy {np.__version__}, CPU fp32, 8 threads\n")
    print("golden fixtures written to", HERE)
