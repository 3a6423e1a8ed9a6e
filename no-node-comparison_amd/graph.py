"""Fully connected, equal-size graph batches — the only topology the reference builds.

The reference materialises int64 edge lists per batch (EGNO/simulation/dataset_simple.py:64-71,
101-111; SEGNO/dataset_nbody.py:84-94): receiver row i, sender col j, ordered (b, i, j != i).
The kernels index that pattern implicitly, so the boundary checks that the caller's edge_index is
exactly it.

- Host (CPU) edge tensors are checked on the spot: ValueError otherwise.
- Device edge tensors are checked on the device without blocking the host (the reference's loop
  builds fresh edge tensors every batch, main_simulation_simple_no.py:217-218, so a check per new
  tensor is on the step's path): ``nonode_check_full_edges`` sets a device flag on any mismatch; the
  forward that used the edges ends with ``finish()``, which NaN-fills its outputs if the flag is set
  (``nonode_poison_if_flagged``) and copies the flag to pinned host memory behind an event. The next
  boundary call on that device that finds the event complete and the flag set raises ValueError
  (``sync_checks()`` waits for it). So a wrong edge list never yields silently wrong numbers: its
  forward's outputs are NaN, and the error is raised one call later at most.
- Edge lists made by ``full_edges`` on the device (the ``get_edges`` counterpart, one kernel) are valid
  by construction and enter the cache without a check.
"""
from collections import OrderedDict

import torch

# validated edge tensors, keyed by address / version / shape. Each entry holds a reference to its
# tensors, so their memory cannot be freed and reused by a different edge list while the entry
# exists (a key built from addresses alone would then match a tensor it never checked).
_checked = OrderedDict()
_CACHE = 8
_states = {}


def _key(rows, cols, E, n_nodes):
    return (rows.data_ptr(), cols.data_ptr(), rows._version, cols._version, E, n_nodes, str(rows.device),
            rows.dtype, cols.dtype)


def _remember(key, B, N, rows, cols):
    _checked[key] = (B, N, rows, cols)
    _checked.move_to_end(key)
    while len(_checked) > _CACHE:
        _checked.popitem(last=False)


def _full_edges_host(B, N, device):
    """Pure elementwise index arithmetic (no boolean mask: nothing synchronises on a device)."""
    e = torch.arange(B * N * (N - 1), device=device)
    per = N * (N - 1)
    b, rem = e // per, e % per
    i, k = rem // (N - 1), rem % (N - 1)
    return b * N + i, b * N + k + (k >= i).to(torch.int64)


def full_edges(B, N, device="cpu"):
    """Edge list of B fully connected N-node graphs in the reference order (row, col), int64.
    On a ROCm device: one nonode_full_edges launch, and the pair is known valid (no check later)."""
    device = torch.device(device)
    if device.type != "cuda":
        return _full_edges_host(B, N, device)
    from . import _lib
    E = B * N * (N - 1)
    rows = torch.empty(E, dtype=torch.int64, device=device)
    cols = torch.empty(E, dtype=torch.int64, device=device)
    _lib.check(_lib.lib().nonode_full_edges(B, N, _lib.ptr(rows), _lib.ptr(cols), _lib.stream_of(rows)))
    _remember(_key(rows, cols, E, B * N), B, N, rows, cols)
    return rows, cols


def _split(edge_index):
    if isinstance(edge_index, (list, tuple)):
        if len(edge_index) != 2:
            raise ValueError("edge_index must be [rows, cols]")
        return edge_index[0], edge_index[1]
    if torch.is_tensor(edge_index) and edge_index.dim() == 2 and edge_index.shape[0] == 2:
        return edge_index[0], edge_index[1]
    raise ValueError("edge_index must be a pair of index tensors or a [2, E] tensor")


_NOT_FULL = ("edge_index is not the dataset's fully connected edge list (receiver i, sender j != i, ordered "
             "by sample, i, j); the MI355X kernels index that pattern implicitly")


class _DeviceChecks:
    """Pending device-side edge checks of one device (see the module docstring)."""

    def __init__(self, device):
        self.flag = torch.zeros(1, dtype=torch.int32, device=device)
        self.host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.event = None      # recorded after the flag's copy to self.host
        self.in_flight = []    # cache keys whose checks that copy covers
        self.unconfirmed = []  # cache keys checked after it (not covered by a copy yet)

    def pending(self):
        return bool(self.in_flight or self.unconfirmed)

    def poll(self, block=False):
        """Read the flag copy if it has landed; raise ValueError if a check failed."""
        if self.event is None:
            return
        if block:
            self.event.synchronize()
        elif not self.event.query():
            return
        bad = int(self.host[0]) != 0
        self.event = None
        if not bad:
            self.in_flight = []
            return
        # which of the checked lists failed is not known: forget every unconfirmed one (a later use
        # re-checks it), clear the flag behind the checks already launched, report
        for k in self.in_flight + self.unconfirmed:
            _checked.pop(k, None)
        self.in_flight, self.unconfirmed = [], []
        self.flag.zero_()
        self.host.zero_()
        raise ValueError(_NOT_FULL + " (found by the device-side check of an earlier call, whose outputs "
                         "were filled with NaN)")

    def launch(self, rows, cols, E, B, N):
        from . import _lib
        if rows.dtype != cols.dtype or rows.dtype not in (torch.int32, torch.int64):
            rows, cols = rows.to(torch.int64), cols.to(torch.int64)
        rows, cols = rows.contiguous(), cols.contiguous()
        _lib.check(_lib.lib().nonode_check_full_edges(_lib.ptr(rows), _lib.ptr(cols), rows.element_size(), E, B, N,
                                                      _lib.ptr(self.flag), _lib.stream_of(rows)))

    def finish(self, outs):
        """After a forward on edges with pending checks: NaN-fill its fp32 outputs if the flag is
        set, and copy the flag to the host behind an event (one copy in flight at a time)."""
        import ctypes
        from . import _lib
        bufs = [t for t in outs if torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float32
                and t.is_contiguous()][:4]
        if bufs:
            P = ctypes.c_void_p * len(bufs)
            C = ctypes.c_longlong * len(bufs)
            _lib.check(_lib.lib().nonode_poison_if_flagged(_lib.ptr(self.flag), len(bufs),
                                                           P(*[t.data_ptr() for t in bufs]),
                                                           C(*[t.numel() for t in bufs]), _lib.stream_of(bufs[0])))
        if self.event is None and self.unconfirmed:
            self.host.copy_(self.flag, non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record()
            self.in_flight, self.unconfirmed = self.unconfirmed, []


def _state(device):
    st = _states.get(device)
    if st is None:
        st = _states[device] = _DeviceChecks(device)
    return st


def check_full_graph(edge_index, n_nodes):
    """Return (B, N) for an edge list of B fully connected N-node graphs covering n_nodes nodes.
    Host tensors: ValueError at once if edge_index is anything else. Device tensors: checked on the
    device (module docstring); a failed check raises ValueError at a later call."""
    rows, cols = _split(edge_index)
    E = rows.numel()
    if cols.numel() != E or n_nodes <= 0 or E % n_nodes:
        raise ValueError(f"edge_index with {E} edges is not a fully connected batch over {n_nodes} nodes")
    N = E // n_nodes + 1
    if n_nodes % N or N < 2:
        raise ValueError(f"edge_index with {E} edges is not a fully connected batch over {n_nodes} nodes")
    B = n_nodes // N
    if rows.device != cols.device:
        raise ValueError("edge_index rows and cols must be on one device")
    on_device = rows.is_cuda
    if on_device:
        _state(rows.device).poll()
    key = _key(rows, cols, E, n_nodes)
    hit = _checked.get(key)
    if hit is not None:
        _checked.move_to_end(key)
        return hit[0], hit[1]
    if on_device:
        st = _state(rows.device)
        st.launch(rows, cols, E, B, N)
        st.unconfirmed.append(key)
    else:
        r, c = _full_edges_host(B, N, rows.device)
        if not (torch.equal(rows.to(torch.int64), r) and torch.equal(cols.to(torch.int64), c)):
            raise ValueError(_NOT_FULL)
    _remember(key, B, N, rows, cols)
    return B, N


def finish(outs):
    """Pass a forward's outputs (a tuple of tensors) through the pending edge checks of their device
    (NaN-filled if one failed; see the module docstring). Returns outs."""
    dev = next((t.device for t in outs if torch.is_tensor(t) and t.is_cuda), None)
    if dev is not None:
        st = _states.get(dev)
        if st is not None and st.pending():
            st.finish(outs)
    return outs


def sync_checks(device=None):
    """Wait for the device-side edge checks issued so far and raise ValueError if one failed."""
    for dev, st in list(_states.items()):
        if device is not None and dev != torch.device(device):
            continue
        st.poll(block=True)
        if st.unconfirmed:        # checks launched after the last copy: copy the flag once more
            st.finish(())
            st.poll(block=True)
