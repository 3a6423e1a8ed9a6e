"""The drop-in boundary without host synchronisation (graph.py): the reference's loop hands every batch
fresh edge tensors (main_simulation_simple_no.py:217-218 `loader.dataset.get_edges(...)` then `.to(device)`),
so the edge-list check is on the step's path. On the device it is a kernel that sets a flag; a failed
check NaN-fills that forward's outputs and raises ValueError at a later boundary call.
"""
import time

import pytest
import torch

import no_node_comparison_amd as pkg
from tests.test_gpu_parity import DEV, _dev, _egno, _egno_case, _segno

pytestmark = pytest.mark.gpu


def _inputs(B, N, T, seed):
    case = _egno_case(B, N, T, seed=seed)
    return {k: _dev(v) for k, v in case.items()}


def _fwd(m, inp, rows, cols):
    with torch.no_grad():
        return m(inp["x"], inp["h"], [rows, cols], inp["edge_fea"], v=inp["v"], loc_mean=inp["loc_mean"],
                 timesteps_out=inp["t_out"])


def _sleep_calibrated(seconds):
    """A spin kernel on the current stream that runs for about `seconds` (torch.cuda._sleep cycles,
    calibrated on this device)."""
    cycles = 1 << 24
    for _ in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda._sleep(cycles)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dt >= 0.05:
            break
        cycles *= 4
    return int(cycles * seconds / dt)


def test_reference_loop_fresh_edges_never_block_the_host():
    """Three batches of the reference-order loop, each with fresh device edge tensors that the
    boundary has never seen (device copies of get_edges, so the device-side check runs on every one),
    queued behind a ~0.6 s spin kernel: the three forwards return to the host long before the spin
    ends (no synchronising call inside), and their outputs equal the forward on validated edges."""
    B, N, T = 64, 20, 10
    m = _egno(seed=41)
    inp = _inputs(B, N, T, seed=42)
    r0, c0 = pkg.harness.get_edges(B, N, DEV)
    ref = [t.clone() for t in _fwd(m, inp, r0, c0)]
    _fwd(m, inp, r0.clone(), c0.clone())          # warm every lazy init (pinned flag, events)
    pkg.graph.sync_checks()
    cycles = _sleep_calibrated(0.6)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(cycles)
    outs = []
    for _ in range(3):
        rows, cols = r0.clone(), c0.clone()        # fresh tensors: a cache miss, checked on the device
        outs.append(_fwd(m, inp, rows, cols))
    host_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    total_s = time.perf_counter() - t0
    assert host_s < 0.25 * total_s, (host_s, total_s)
    pkg.graph.sync_checks()                         # all three checks passed
    for out in outs:
        for a, b in zip(out, ref):
            assert torch.equal(a, b)


@pytest.mark.parametrize("idx_dtype", [torch.int64, torch.int32])
def test_wrong_device_edges_poison_outputs_and_raise_later(idx_dtype):
    """A device edge list that is not the fully connected one (receiver and sender swapped, or one
    edge rewired): the forward returns without blocking, its outputs are NaN, and the error is raised
    at the next boundary call (or by sync_checks); the edges are then re-checked on any later use, and a
    correct list works again."""
    B, N, T = 4, 20, 10
    m = _egno(seed=43)
    inp = _inputs(B, N, T, seed=44)
    r, c = pkg.harness.get_edges(B, N, DEV)
    good = [t.clone() for t in _fwd(m, inp, r, c)]
    bad_r = c.to(idx_dtype)
    bad_c = r.to(idx_dtype)
    x, v, h = _fwd(m, inp, bad_r, bad_c)
    torch.cuda.synchronize()
    assert torch.isnan(x).all() and torch.isnan(v).all() and torch.isnan(h).all()
    with pytest.raises(ValueError, match="fully connected"):
        _fwd(m, inp, r, c)
    out = _fwd(m, inp, r, c)                        # the flag was cleared: valid edges work again
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(out, good))
    rr = r.clone()
    rr[30] = 0                                      # edge (1, 12) rewired to receiver 0
    _fwd(m, inp, rr, c)
    with pytest.raises(ValueError, match="fully connected"):
        pkg.graph.sync_checks()
    _fwd(m, inp, rr, c)                             # still not trusted: checked (and rejected) again
    with pytest.raises(ValueError, match="fully connected"):
        pkg.graph.sync_checks()


def test_segno_fresh_device_edges_checked_on_device():
    """SEGNO's forward through the same boundary: fresh edge tensors pass the device-side check and
    give the same outputs; swapped ones give NaN outputs and a ValueError."""
    B, N, T = 8, 20, 10
    m = _segno(seed=45)
    g = torch.Generator().manual_seed(46)
    x = torch.randn(B * N, 3, generator=g).to(DEV)
    v = torch.randn(B * N, 3, generator=g).to(DEV)
    q = torch.randn(B * N, 1, generator=g).sign().to(DEV)
    r, c = pkg.harness.get_edges(B, N, DEV)
    ea = torch.cat([q[r] * q[c], ((x[r] - x[c]) ** 2).sum(1, keepdim=True)], 1)
    his = v.norm(dim=1, keepdim=True)
    with torch.no_grad():
        ref = [t.clone() for t in m(his, x, [r, c], v, ea, T=T)]
        out = m(his, x, [r.clone(), c.clone()], v, ea, T=T)
        pkg.graph.sync_checks()
        assert all(torch.equal(a, b) for a, b in zip(out, ref))
        out = m(his, x, [c.clone(), r.clone()], v, ea, T=T)
        torch.cuda.synchronize()
        assert all(torch.isnan(t).all() for t in out)
        with pytest.raises(ValueError, match="fully connected"):
            pkg.graph.sync_checks()


def test_device_full_edges_match_host_order():
    """nonode_full_edges (get_edges on the device) is the reference order, bitwise."""
    for B, N in ((1, 2), (3, 5), (512, 20), (2, 100)):
        r, c = pkg.graph.full_edges(B, N, DEV)
        rh, ch = pkg.graph.full_edges(B, N)
        assert torch.equal(r.cpu(), rh) and torch.equal(c.cpu(), ch)
