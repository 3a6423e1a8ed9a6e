"""Batch sharding across ranks (one process per GPU).

The rollout path partitions by trajectory sample: every sample's graph, edge features and
trajectory are independent of every other sample (EGNO/model/egno.py:37-111 and
SEGNO/models/model.py:95-102 never mix rows of different samples). A job over B_global samples
on W ranks therefore gives rank r the contiguous sample range shard_range(B_global, W, r), runs
the kernels on it with no collective in the data path, and only the timing (max over ranks) and
optional result collection touch the process group.

The reference runs single-process (main.py:27-31 picks one device); this module is the
MI355X-side replacement for "one big batch on one device".
"""
import torch
import torch.distributed as dist


def shard_range(total, world, rank):
    """Contiguous, balanced [lo, hi) slice of `total` samples for `rank` of `world`
    (sizes differ by at most one; the union over ranks is exactly range(total))."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    if total < 0:
        raise ValueError(f"bad total {total}")
    return (total * rank) // world, (total * (rank + 1)) // world


def _initialized():
    return dist.is_available() and dist.is_initialized()


def _reduce_device(dev):
    # RCCL reduces device tensors; gloo reduces host tensors
    return dev if dist.get_backend() == "nccl" else torch.device("cpu")


def allreduce_scalar(value, op, dev=torch.device("cpu")):
    """One scalar all-reduce of a host number over the process group (a device tensor under RCCL,
    a host tensor under gloo). Runs the collective at any world size, 1 included."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=_reduce_device(dev))
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(value, dev=torch.device("cpu")):
    """Max of a host float over all ranks (the bench's step time): one scalar all-reduce."""
    if not _initialized() or dist.get_world_size() == 1:
        return float(value)
    return allreduce_scalar(value, dist.ReduceOp.MAX, dev)


def sum_over_ranks(value, dev=torch.device("cpu")):
    """Sum of a host number over all ranks (e.g. samples processed)."""
    if not _initialized() or dist.get_world_size() == 1:
        return float(value)
    return allreduce_scalar(value, dist.ReduceOp.SUM, dev)


def gather_samples(local, total):
    """Concatenate every rank's per-sample rows (dim 0 = local samples of shard_range order) into
    the full [total, ...] tensor on every rank. Result collection only — outside timed regions."""
    if not _initialized() or dist.get_world_size() == 1:
        return local
    world = dist.get_world_size()
    dev = _reduce_device(local.device)
    sizes = [shard_range(total, world, r) for r in range(world)]
    pad = max(hi - lo for lo, hi in sizes)
    buf = torch.zeros((pad,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    buf[: local.shape[0]] = local.to(dev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return torch.cat([p[: hi - lo] for p, (lo, hi) in zip(parts, sizes)]).to(local.device)


class FlatGrads:
    """Data-parallel gradient exchange with ONE collective per step.

    Every parameter's .grad is a view into one contiguous buffer (fp32 for the models), so autograd accumulates
    straight into it and the step needs a single all-reduce (sum) of the flat buffer (0.81 MB
    for EGNO) followed by a division by the world size: with equal shards this is the gradient of
    the global mean loss.

    Return contract of allreduce_(): the reduced flat buffer at world size > 1; None at world size 1
    (or without a process group), where there is nothing to exchange and the parameters keep
    autograd's gradient tensors as they are (no copy into the buffer on the step's path). Reading
    ``flat`` at any world size gathers first, so it always holds the gradients the optimizer will
    step on (tests/test_sharding.py pins both)."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev, dt = self.params[0].device, self.params[0].dtype
        if any(p.dtype != dt or p.device != dev for p in self.params):
            raise ValueError("FlatGrads needs every parameter on one device with one dtype")
        self.numel = n
        self._buf = torch.zeros(n, dtype=dt, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            self.views.append(self._buf[off:off + p.numel()].view_as(p))
            off += p.numel()
        self._bind()

    @property
    def flat(self):
        """The flat gradient buffer, gathered from the parameters' current .grad first."""
        return self.gather_()

    def _bind(self):
        for p, v in zip(self.params, self.views):
            p.grad = v

    def zero_(self):
        self._buf.zero_()
        self._bind()

    def gather_(self):
        """Bring every p.grad back into the flat buffer. The reference loop calls
        optimizer.zero_grad() each step (main_simulation_simple_no.py:224), which in torch 2.x sets
        p.grad = None, so the next backward allocates fresh local tensors instead of accumulating
        into the views. Those (or a None, i.e. zero) are copied into the buffer and the views are
        re-bound, so the all-reduce always reduces the gradients the optimizer will step on."""
        stale = [i for i, (p, v) in enumerate(zip(self.params, self.views))
                 if p.grad is None or p.grad.data_ptr() != v.data_ptr()]
        if not stale:
            return self._buf
        if len(stale) == len(self.params):
            # the usual case after zero_grad(): one concatenation into the buffer
            parts = [(p.grad if p.grad is not None else torch.zeros_like(v)).reshape(-1)
                     for p, v in zip(self.params, self.views)]
            torch.cat(parts, out=self._buf)
        else:
            for i in stale:
                p, v = self.params[i], self.views[i]
                if p.grad is None:
                    v.zero_()
                else:
                    v.copy_(p.grad)
        self._bind()
        return self._buf

    def exchange_(self):
        """The step's one collective: sum of the flat buffer over the ranks, then / world size
        (runs at any world size; allreduce_ skips it when there is nothing to exchange)."""
        dist.all_reduce(self._buf, op=dist.ReduceOp.SUM)
        self._buf.div_(dist.get_world_size())
        return self._buf

    def allreduce_(self):
        """The step's exchange: the reduced flat buffer, or None at world size 1 (class docstring)."""
        if not _initialized() or dist.get_world_size() == 1:
            return None
        self.gather_()
        return self.exchange_()
