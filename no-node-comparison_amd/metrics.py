"""Rollout metrics on the GPU: the reference's evaluation numbers for predicted
trajectories (utils.py:221-321, main_simulation_simple_no.py:237-273), reduced by one HIP kernel
(nonode_rollout_metrics) per call."""
import torch

from . import _lib


def _f32(t):
    return t.detach().to(torch.float32).contiguous()


def _run(pred, truth, N, want_corr=True, want_sqerr=True):
    _lib.require_device(pred, truth)
    T, BN = pred.shape[0], pred.shape[1]
    B = BN // N
    p, y = _f32(pred), _f32(truth)
    corr = torch.empty(B, T, device=p.device) if want_corr else None
    sq = torch.empty(T, B, device=p.device) if want_sqerr else None
    _lib.check(_lib.lib().nonode_rollout_metrics(T, B, N, _lib.ptr(p), _lib.ptr(y), _lib.ptr(corr), _lib.ptr(sq),
                                                 _lib.stream_of(p)))
    return corr, sq


def pearson_correlation_batch(x, y, N):
    """utils.py:261-321: x, y [T, B*N, 3] -> (correlation [B, cut] with cut = int(0.4 T), mean over
    samples of the number of steps before the correlation first drops below 0.5, first step at
    which ANY sample is below 0.5 (T-cut columns if none))."""
    T = x.shape[0]
    cut = int(0.4 * T)
    corr, _ = _run(x[:cut], y[:cut], N, want_sqerr=False)
    below = corr < 0.5
    steps = torch.where(below.any(1), below.int().argmax(1), torch.full_like(below[:, 0], cut, dtype=torch.long))
    mask = torch.all(~below, dim=0)
    first = corr.size(1) if bool(mask.all()) else int(torch.argmax((~mask).int()).item())
    return corr, float(steps.float().mean().item()), first


def horizon_mse(pred, truth, N):
    """Per-horizon loss criterion(loc_pred, loc_true).mean((0, 1, 3)) (main_simulation_simple_no.py:273)
    for pred, truth [T, B*N, 3] -> [T]."""
    _, sq = _run(pred, truth, N, want_corr=False)
    return sq.sum(1) / (pred.shape[1] * 3)


def energy_drift(energies, eps=1e-10):
    """compute_energy_drift (utils.py:221-243) from per-frame energies [T, B(, 1)]:
    |(E_t - E_0) / (E_0 + eps)|."""
    return torch.abs((energies - energies[:1]) / (energies[:1] + eps))
