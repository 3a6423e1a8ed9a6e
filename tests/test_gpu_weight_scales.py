"""GPU parity beyond init-scale weights: the fp16x3 split products must keep the
fp32 bar for the weight magnitudes of a trained model and for weights much smaller or larger than
the init scale, where an unshifted fp16 residual W_lo would fall into the fp16 subnormal range.

Cases, C2 (EGNO forward, N=20, T=10) and C3 (SEGNO forward_step, N=20, 10 substeps):
  - trained: 200 Adam steps at lr 1e-3 through the HIP training path on charged trajectories from
    the HIP simulator (sim.ChargedParticlesSim, synthetic_sim.py:149-296), then the forward at
    B=512 against float64;
  - rescaled: every weight matrix (and the TimeConv weights) x1/16 and x4, at B=128 against float64.
Bar: 1e-5 max-norm relative (north_star), or twice the error of the reference's own ops in fp32
(oracle/torch_ref.py) on the same inputs where that is larger (x4 weights: the inputs of the later
layers are ill-conditioned in fp32 itself)."""
import numpy as np
import pytest
import torch

import no_node_comparison_amd as pkg
from oracle import torch_ref as tr
from tests.conftest import check_rel, maxnorm_rel
from tests.test_gpu_parity import DEV, _egno, _egno_full, _segno, synthetic_charged

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _sim_batch(S, N=20, frames=11, seed=0):
    """S charged trajectories (HIP simulator, reference RNG order): loc, vel [S, frames, N, 3], q [S, N, 1]."""
    np.random.seed(seed)
    sim = pkg.sim.ChargedParticlesSim(n_balls=N)
    loc, vel, _, q = sim.sample_trajectories(S, T=(frames + 1) * 100, sample_freq=100, device=DEV, as_numpy=False)
    loc = loc.permute(0, 1, 3, 2).float().contiguous()
    vel = vel.permute(0, 1, 3, 2).float().contiguous()
    return loc, vel, torch.tensor(q, dtype=torch.float32, device=DEV)


def _egno_inputs(loc0, vel0, q, T):
    B, N = loc0.shape[0], loc0.shape[1]
    edges = pkg.harness.get_edges(B, N, DEV)
    qq = q.reshape(-1, 1)
    eao = qq[edges[0]] * qq[edges[1]]
    x, v, ea, nodes, lm = pkg.harness.prepare_inputs(loc0, vel0, eao, edges, N, 1, q)
    t = torch.arange(1, T + 1, device=DEV).repeat(B, 1)
    return x, nodes, edges, ea, v, lm, t


def _train_egno(m, steps=200, B=64, T=10, lr=1e-3):
    loc, vel, q = _sim_batch(4 * B, frames=T + 1, seed=5)
    opt = torch.optim.Adam(m.parameters(), lr=lr)
    m.train()
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        idx = torch.randperm(loc.shape[0], generator=g)[:B].to(DEV)
        x, nodes, edges, ea, v, lm, t = _egno_inputs(loc[idx, 0], vel[idx, 0], q[idx], T)
        opt.zero_grad(set_to_none=True)
        xo, _, _ = m(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_out=t)
        pred = xo.reshape(T, B, -1, 3).permute(1, 2, 0, 3)
        loss = torch.nn.functional.mse_loss(pred, loc[idx, 1:T + 1].permute(0, 2, 1, 3))
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    return m.eval()


def _scale_weights(m, s):
    with torch.no_grad():
        for k, p in m.named_parameters():
            if k.endswith("weight") or k.endswith("weights1"):
                p.mul_(s)
    return m


def _check_egno(m, B, seed, tag):
    T, N = 10, 20
    x, nodes, edges, ea, v, lm, t, _ = _egno_full(B, N, T, seed=seed)
    with torch.no_grad():
        xo, vo, ho = m(x, nodes, edges, ea, v=v, loc_mean=lm, timesteps_out=t)
    r, c = tr.full_edges(B, N)
    outs = []
    for dt in (torch.float64, torch.float32):
        p = {k: q.detach().cpu().to(dt) for k, q in m.state_dict().items()}
        d = lambda a: a.detach().cpu().to(dt)  # noqa: E731
        with torch.no_grad():
            outs.append(tr.egno_forward(p, d(x), d(nodes), r, c, d(ea), d(v), d(lm), t.cpu(), T=T))
    ref, f32 = outs
    for name, got, rr, ff in (("x", xo, ref[0], f32[0]), ("v", vo, ref[1], f32[1]), ("h", ho, ref[2], f32[2])):
        bar = max(TOL, 2 * maxnorm_rel(ff.numpy(), rr.numpy()))
        check_rel(f"{tag} {name}", got, rr, bar)


def test_egno_c2_trained_weights_match_f64_reference():
    m = _egno(T=10, seed=31)
    w0 = {k: p.detach().clone() for k, p in m.named_parameters()}
    _train_egno(m)
    # the weights moved well away from their init values (|W| <= 1/sqrt(64) = 0.125 at init)
    assert max(float((p - w0[k]).abs().max()) for k, p in m.named_parameters()) > 0.05
    _check_egno(m, 512, seed=32, tag="C2 trained")


@pytest.mark.parametrize("s", [1 / 16, 4.0])
def test_egno_c2_rescaled_weights_match_f64_reference(s):
    _check_egno(_scale_weights(_egno(T=10, seed=33), s), 128, seed=34, tag=f"C2 weights x{s:g}")


def _segno_case(B, N, seed):
    loc, vel, q = synthetic_charged(B, N, seed=seed)
    x = loc.reshape(-1, 3).to(DEV)
    v = vel.reshape(-1, 3).to(DEV)
    edges = pkg.harness.get_edges(B, N, DEV)
    qq = q.reshape(-1, 1).to(DEV)
    ea = torch.cat([qq[edges[0]] * qq[edges[1]], ((x[edges[0]] - x[edges[1]]) ** 2).sum(1, keepdim=True)], 1)
    return v.norm(dim=1, keepdim=True), x, edges, v, ea


def _train_segno(m, steps=200, B=64, T=10, lr=1e-3):
    loc, vel, q = _sim_batch(4 * B, frames=T + 1, seed=6)
    opt = torch.optim.Adam(m.parameters(), lr=lr)
    m.train()
    g = torch.Generator().manual_seed(2)
    N = loc.shape[2]
    edges = pkg.harness.get_edges(B, N, DEV)
    for _ in range(steps):
        idx = torch.randperm(loc.shape[0], generator=g)[:B].to(DEV)
        x = loc[idx, 0].reshape(-1, 3)
        v = vel[idx, 0].reshape(-1, 3)
        qq = q[idx].reshape(-1, 1)
        ea = torch.cat([qq[edges[0]] * qq[edges[1]], ((x[edges[0]] - x[edges[1]]) ** 2).sum(1, keepdim=True)], 1)
        opt.zero_grad(set_to_none=True)
        xo, _, _ = m(v.norm(dim=1, keepdim=True), x, edges, v, ea, T=T)
        loss = torch.nn.functional.mse_loss(xo, loc[idx, T].reshape(-1, 3))
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    return m.eval()


def _check_segno(m, B, seed, tag, T=10):
    N = 20
    his, x, edges, v, ea = _segno_case(B, N, seed)
    with torch.no_grad():
        xo, ho, vo = m(his, x, edges, v, ea, T=T)
    r, c = tr.full_edges(B, N)
    outs = []
    for dt in (torch.float64, torch.float32):
        p = {k: q.detach().cpu().to(dt) for k, q in m.state_dict().items()}
        d = lambda a: a.detach().cpu().to(dt)  # noqa: E731
        with torch.no_grad():
            outs.append(tr.segno_forward_step(p, d(his), d(x), r, c, d(v), d(ea), T=T, dense_mean=False))
    ref, f32 = outs
    for name, got, rr, ff in (("x", xo, ref[0], f32[0]), ("h", ho, ref[1], f32[1]), ("v", vo, ref[2], f32[2])):
        bar = max(TOL, 2 * maxnorm_rel(ff.numpy(), rr.numpy()))
        check_rel(f"{tag} {name}", got, rr, bar)


def test_segno_c3_trained_weights_match_f64_reference():
    m = _segno(seed=41)
    w0 = {k: p.detach().clone() for k, p in m.named_parameters()}
    _train_segno(m)
    assert max(float((p - w0[k]).abs().max()) for k, p in m.named_parameters()) > 0.05
    _check_segno(m, 512, seed=42, tag="C3 trained")


@pytest.mark.parametrize("s", [1 / 16, 4.0])
def test_segno_c3_rescaled_weights_match_f64_reference(s):
    _check_segno(_scale_weights(_segno(seed=43), s), 128, seed=44, tag=f"C3 weights x{s:g}")
