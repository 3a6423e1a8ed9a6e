"""N-body datasets: the reference's .npy splits, loaded once, batched on the GPU.

EGNO: ``NBodyDynamicsDataset`` keeps the reference's constructor, file names, layout rules and
``__getitem__`` (EGNO/simulation/dataset_simple.py:6-178), including several inputs per sample
(num_inputs > 1, equispaced or varDT random offsets), vectorised (no per-edge Python loop).
``DeviceLoader`` replaces ``torch.utils.data.DataLoader`` for it: the whole split sits in HBM and
every batch is ONE gather launch (nonode_gather_batch) over the implicit fully connected edge list
(no int64 edge arrays), returning the 7-tuple run_epoch unpacks (main_simulation_simple_no.py:
200-201) already on the device.

SEGNO: ``NBodyDataset`` mirrors SEGNO/dataset_nbody.py:7-94 (whole trajectories per item);
``SegnoDeviceLoader`` yields its collated batches from a device-resident split (nonode_gather_rows);
``segno_batch_inputs`` is the featurisation run_epoch does on every batch (SEGNO/train_nbody.py:
76-123: |v| node features, [q_i q_j, |x_i - x_j|^2] edge features, the input frames and loc_end),
with the edge features from the featurize kernel.
"""
from pathlib import Path

import numpy as np
import torch

from . import _lib
from .graph import full_edges

_FRAME0 = {"nbody": 6, "nbody_small": 30, "nbody_small_out_dist": 20}   # dataset_simple.py:126,145


def random_ascending_tensor(length, min_value=0, max_value=9):
    """Root utils.py:15-31 (the one dataset_simple.py:3 imports): `length` distinct values of
    [min_value, max_value] in ascending order, drawn with torch.randperm on the global RNG."""
    return (torch.randperm(max_value - min_value + 1)[:length] + min_value).sort().values


def _check_idx(idx, S):
    if idx.numel() == 0:
        raise ValueError("empty batch")
    lo, hi = int(idx.min()), int(idx.max())
    if lo < 0 or hi >= S:
        raise IndexError(f"sample index out of range [0, {S}): {lo if lo < 0 else hi}")


class NBodyDynamicsDataset:
    """dataset_simple.py:122-178 (and NBodyDataset :6-111)."""

    def __init__(self, partition='train', data_dir='.', max_samples=1e8, dataset="charged", dataset_name="nbody_small",
                 n_balls=5, num_timesteps=10, num_inputs=1, traj_len=1, dT=1, varDT=False):
        self.partition = partition
        self.data_dir = Path(data_dir)
        self.suffix = "valid" if partition == "val" else partition
        if dataset_name == "nbody":
            self.suffix += f"_{dataset}{n_balls}_initvel1"
        elif dataset_name in ("nbody_small", "nbody_small_out_dist"):
            self.suffix += f"_{dataset}{n_balls}_initvel1small"
        else:
            raise Exception("Wrong dataset name %s" % dataset_name)
        self.dataset_name = dataset_name
        self.dataset = dataset
        self.n_balls = n_balls
        self.max_samples = int(max_samples)
        self.num_timesteps = num_timesteps
        self.traj_len = traj_len
        self.num_inputs = num_inputs
        self.var_dt = varDT
        self.dT = dT
        self.start = _FRAME0.get(dataset_name) if dataset == "charged" else 0
        self.data, self.edges = self.load()

    def load(self):
        """dataset_simple.py:36-50: loc / vel [S, frames, N, 3] (transposed from [S, frames, 3, N]
        when stored that way), charges [S, N, 1], edge attributes q_i q_j."""
        loc = np.load(self.data_dir / f"loc_{self.suffix}.npy")
        vel = np.load(self.data_dir / f"vel_{self.suffix}.npy")
        if loc.shape[-2:] != (self.n_balls, 3):
            loc = np.transpose(loc, (0, 1, 3, 2))
            vel = np.transpose(vel, (0, 1, 3, 2))
            assert loc.shape[-2:] == (self.n_balls, 3) and vel.shape[-2:] == (self.n_balls, 3), "Shape mismatch!"
        charges = np.load(self.data_dir / f"charges_{self.suffix}.npy")
        loc = torch.tensor(loc).float()[:self.max_samples]
        vel = torch.tensor(vel).float()[:self.max_samples]
        charges = charges[:self.max_samples]
        N = loc.size(2)
        i, j = np.nonzero(~np.eye(N, dtype=bool))            # (i, j != i), row-major (:64-71)
        q = charges[:, :, 0]
        edge_attr = torch.tensor((q[:, i] * q[:, j]).astype(np.float64)).float().unsqueeze(2)
        return (loc, vel, edge_attr, torch.tensor(charges).float()), [i.tolist(), j.tolist()]

    def set_max_samples(self, max_samples):
        self.max_samples = int(max_samples)
        self.data, self.edges = self.load()

    def get_n_nodes(self):
        return self.data[0].size(1)

    def __len__(self):
        return len(self.data[0])

    def frames(self):
        """(frame_0, out_indices) of one item (dataset_simple.py:130-164). frame_0 is an int for a
        single input, else the num_inputs input frames, all at or before the start frame; with
        varDT their offsets come from random_ascending_tensor, one torch.randperm draw per call,
        as every reference __getitem__ makes."""
        assert self.num_inputs <= self.num_timesteps
        frame_0 = self.start
        frame_T = frame_0 + self.num_timesteps * self.traj_len * self.dT
        if self.num_inputs > 1:
            if self.var_dt:
                ts = random_ascending_tensor(length=self.num_inputs - 1, max_value=self.num_timesteps - 1, min_value=1)
                ts = torch.cat((torch.tensor([0]), ts), dim=0)
            else:
                ts = (torch.arange(self.num_timesteps) * self.dT)[:self.num_inputs]
            ts = -torch.flip(ts, dims=(0,))
            frame_0 = frame_0 + ts * self.dT
            if (frame_0 < 0).any():
                frame_T += -frame_0.min()
                frame_0 += -frame_0.min()
            out = torch.arange(frame_0[-1] + 1, frame_T + 1, self.dT)
        else:
            out = torch.arange(frame_0 + 1, frame_T + 1, self.dT)
        if out.max() >= self.data[0].size(1):
            out = out[out < self.data[0].size(1)]
        return frame_0, out

    def __getitem__(self, i):
        loc, vel, edge_attr, charges = (d[i] for d in self.data)
        frame_0, out_indices = self.frames()
        return loc[frame_0], vel[frame_0], edge_attr, charges, loc[out_indices].transpose(1, 0), frame_0, out_indices

    def get_edges(self, batch_size, n_nodes):
        """dataset_simple.py:101-111 (vectorised)."""
        r, c = full_edges(batch_size, n_nodes)
        return [r, c]

    def energy_fun(self, loc, vel, edges, batch=None):
        """conserved_energy_fun (utils.py:197-219) on the GPU; returns numpy like the reference."""
        from .harness import conserved_energy
        B = int(batch.max().item()) + 1 if batch is not None else 1
        return conserved_energy(self.dataset, loc, vel, edges, B).cpu().numpy()


class DeviceLoader:
    """DataLoader over NBodyDynamicsDataset with the split resident in HBM.

    Yields (loc, vel, edge_attr [B,N(N-1),1], charges [B,N,1], loc_true [B,N,To,3], frame_0,
    out_indices [B,To] int64), all on ``device``, as run_epoch's ``[d.to(device) for d in data]``
    would hold them: loc / vel [B,N,3] and frame_0 [B] for a single input, [B,I,N,3] and [B,I] for
    num_inputs = I > 1. The split is copied to the device once. With varDT the input frames are
    drawn per sample in batch order (the reference's __getitem__ draws); ``shuffle`` draws
    torch.randperm from ``generator`` each epoch (DataLoader's RandomSampler draws its own
    permutation from a derived seed, so the sample order differs from the reference's for the same
    seed)."""

    def __init__(self, dataset, batch_size=1, shuffle=False, drop_last=False, device="cuda", generator=None):
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.generator = generator
        dev = torch.device(device)
        loc, vel, edge_attr, charges = dataset.data
        _lib.require_device(torch.empty(0, device=dev))
        self.ea = edge_attr.reshape(len(dataset), -1).contiguous().to(dev)
        self.loc = loc.contiguous().to(dev)
        self.vel = vel.contiguous().to(dev)
        self.q = charges.reshape(len(dataset), -1).contiguous().to(dev)
        self._fixed = None
        if not (dataset.num_inputs > 1 and dataset.var_dt):
            self._fixed = dataset.frames()     # the same frames for every sample

    def __len__(self):
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def batch(self, idx):
        """Gather the samples idx (sequence or tensor) as one batch."""
        dev = self.loc.device
        idx = torch.as_tensor(idx, dtype=torch.int64).reshape(-1)
        S, Tf, N, _ = self.loc.shape
        _check_idx(idx, S)
        B = idx.numel()
        I = self.dataset.num_inputs
        draws = [self._fixed] * B if self._fixed is not None else [self.dataset.frames() for _ in range(B)]
        To = draws[0][1].numel()
        if any(d[1].numel() != To for d in draws):
            raise RuntimeError("DeviceLoader: samples of one batch have different numbers of target frames")
        f0 = torch.tensor([list(np.atleast_1d(np.asarray(d[0]))) for d in draws], dtype=torch.int32)
        oi = torch.stack([d[1] for d in draws]).to(torch.int32)
        # frame indices past the stored trajectory: the reference's loc[frame_0] raises IndexError
        # (dataset_simple.py:128-163); the gather kernel would read past the sample instead
        for name, fr in (("frame_0", f0), ("target frame", oi)):
            if fr.numel() and (int(fr.min()) < 0 or int(fr.max()) >= Tf):
                raise IndexError(f"DeviceLoader: {name} index out of range [0, {Tf}) "
                                 f"(got {int(fr.min())}..{int(fr.max())})")
        f0_dev, oi_dev, idx_dev = f0.to(dev), oi.to(dev), idx.to(torch.int32).to(dev)
        loc0 = torch.empty(B, I, N, 3, device=dev)
        vel0 = torch.empty(B, I, N, 3, device=dev)
        q = torch.empty(B, N, 1, device=dev)
        ea = torch.empty(B, N * (N - 1), 1, device=dev)
        lt = torch.empty(B, N, To, 3, device=dev)
        _lib.check(_lib.lib().nonode_gather_batch(S, Tf, N, B, I, To, _lib.ptr(self.loc), _lib.ptr(self.vel),
                                                  _lib.ptr(self.q), _lib.ptr(self.ea), _lib.ptr(idx_dev),
                                                  _lib.ptr(f0_dev), _lib.ptr(oi_dev),
                                                  _lib.ptr(loc0), _lib.ptr(vel0), _lib.ptr(q), _lib.ptr(ea),
                                                  _lib.ptr(lt), _lib.stream_of(self.loc)))
        if I == 1:
            return (loc0[:, 0], vel0[:, 0], ea, q, lt, f0_dev[:, 0].long(), oi_dev.long())
        return (loc0, vel0, ea, q, lt, f0_dev.long(), oi_dev.long())

    def __iter__(self):
        n = len(self.dataset)
        order = torch.randperm(n, generator=self.generator) if self.shuffle else torch.arange(n)
        for k in range(len(self)):
            yield self.batch(order[k * self.batch_size:(k + 1) * self.batch_size])


class NBodyDataset:
    """SEGNO/dataset_nbody.py:7-94: whole trajectories per item. Files
    ``{loc,vel,edges,charges}_{split}_{dataset}{n_balls}_initvel1{dataset_size}.npy`` (:17-20, 30-33);
    loc / vel [S, frames, N, 3] (transposed from [S, frames, 3, N]); edge_attr [S, N(N-1), 1] from the
    simulator's interaction matrix edges[:, i, j] in (i, j != i) order (:50-61); start frame 30 for
    charged, 0 for gravity (:22)."""

    def __init__(self, root, partition='train', max_samples=1e8, dataset="charged", dataset_size="small", n_balls=5):
        self.root = Path(root)
        self.partition = partition
        self.suffix = 'valid' if partition == 'val' else partition
        self.dataset = dataset
        self.n_balls = n_balls
        self.suffix += f"_{dataset}{n_balls}_initvel1{dataset_size}"
        self.start = 30 if dataset == "charged" else 0
        self.max_samples = int(max_samples)
        self.data, self.edges = self.load()

    def energy_fun(self, loc, vel, edges, batch=None):
        """conserved_energy_fun (utils.py:197-219) on the GPU; returns numpy like the reference."""
        from .harness import conserved_energy
        B = int(batch.max().item()) + 1 if batch is not None else 1
        return conserved_energy(self.dataset, loc, vel, edges, B).cpu().numpy()

    def load(self):
        loc = np.load(self.root / f'loc_{self.suffix}.npy')
        vel = np.load(self.root / f'vel_{self.suffix}.npy')
        edges = np.load(self.root / f'edges_{self.suffix}.npy')
        charges = np.load(self.root / f'charges_{self.suffix}.npy')
        if self.dataset == "gravity":
            assert (charges > 0).all(), "Charges (i.e. masses) in gravity dataset should be positive"
        if loc.shape[2:] == (3, self.n_balls):
            loc, vel = torch.Tensor(loc).transpose(2, 3), torch.Tensor(vel).transpose(2, 3)
        else:
            loc, vel = torch.Tensor(loc).float(), torch.Tensor(vel).float()
        assert loc.shape[2:] == (self.n_balls, 3), "Location tensor shape mismatch"
        loc, vel = loc[:self.max_samples], vel[:self.max_samples]
        charges = torch.Tensor(charges[:self.max_samples])
        N = loc.size(2)
        i, j = np.nonzero(~np.eye(N, dtype=bool))
        edge_attr = torch.Tensor(np.ascontiguousarray(edges[:, i, j])).unsqueeze(2)
        return (loc, vel, edge_attr, charges), [i.tolist(), j.tolist()]

    def set_max_samples(self, max_samples):
        self.max_samples = int(max_samples)
        self.data, self.edges = self.load()

    def get_n_nodes(self):
        return self.data[0].size(1)

    def __getitem__(self, i):
        loc, vel, edge_attr, charges = self.data
        return loc[i], vel[i], edge_attr[i], charges[i]

    def __len__(self):
        return len(self.data[0])

    def get_edges(self, batch_size, n_nodes):
        """dataset_nbody.py:84-94 (vectorised)."""
        r, c = full_edges(batch_size, n_nodes)
        return [r, c]


class SegnoDeviceLoader:
    """DataLoader over the SEGNO NBodyDataset with the split resident in HBM: yields the collated
    (loc [B,frames,N,3], vel [B,frames,N,3], edge_attr [B,N(N-1),1], charges [B,N,1]) on ``device``
    that run_epoch receives (train_nbody.py:82-83), one nonode_gather_rows launch per array.
    ``shuffle`` / ``generator`` as DeviceLoader."""

    def __init__(self, dataset, batch_size=1, shuffle=False, drop_last=False, device="cuda", generator=None):
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.generator = generator
        dev = torch.device(device)
        _lib.require_device(torch.empty(0, device=dev))
        self.arrays = [d.float().contiguous().to(dev) for d in dataset.data]

    def __len__(self):
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def batch(self, idx):
        idx = torch.as_tensor(idx, dtype=torch.int64).reshape(-1)
        S = self.arrays[0].shape[0]
        _check_idx(idx, S)
        dev = self.arrays[0].device
        idx_dev = idx.to(torch.int32).to(dev)
        out = []
        for a in self.arrays:
            o = torch.empty((idx.numel(),) + tuple(a.shape[1:]), device=dev)
            _lib.check(_lib.lib().nonode_gather_rows(S, a[0].numel(), idx.numel(), _lib.ptr(a), _lib.ptr(idx_dev),
                                                     _lib.ptr(o), _lib.stream_of(a)))
            out.append(o)
        return tuple(out)

    def __iter__(self):
        n = len(self.dataset)
        order = torch.randperm(n, generator=self.generator) if self.shuffle else torch.arange(n)
        for k in range(len(self)):
            yield self.batch(order[k * self.batch_size:(k + 1) * self.batch_size])


def segno_batch_inputs(batch, start, num_timesteps=10, num_inputs=1, var_dt=False, rng=np.random):
    """What run_epoch builds from one SEGNO batch (train_nbody.py:76-123), on the device:
    (h, loc, vel, edge_attr, loc_end, in_steps, edge_index). ``batch`` is a collated
    (loc, vel, edge_attr, charges) as SegnoDeviceLoader yields it; ``start`` the dataset's start
    frame. Single input: h [BN,1] = |v|, loc / vel [BN,3] at frame `start`, in_steps None. With
    num_inputs = I > 1: the I input frames end at `start`, num_timesteps // I apart (or with gaps
    drawn by rng.randint(1, num_timesteps // I, size=I - 1) when var_dt, the reference's
    np.random.randint draw), shifted to start at frame 0 if the first would be negative; loc / vel
    [BN,I,3], h [BN,I,1], in_steps [I] relative to the last input. edge_attr [E,2] = [q_i q_j,
    |x_i - x_j|^2 of the last input] (featurize kernel); loc_end = loc at the last input + T."""
    locs, vels, _, charges = batch
    B, Tf, N = locs.shape[0], locs.shape[1], locs.shape[2]
    dev = locs.device
    _lib.require_device(locs)
    BN = B * N
    # run_epoch's transform (train_nbody.py:84-90): [B, F, N, 3] -> [F, B*N, 3]
    locs = locs.transpose(0, 1).reshape(Tf, BN, 3).contiguous()
    vels = vels.transpose(0, 1).reshape(Tf, BN, 3).contiguous()
    q = charges.reshape(BN, 1)
    rows, cols = full_edges(B, N, dev)
    prod = (q[rows] * q[cols]).contiguous()
    T = num_timesteps
    if num_inputs > 1:
        if var_dt:
            steps = rng.randint(1, T // num_inputs, size=num_inputs - 1).tolist()
        else:
            steps = [T // num_inputs for _ in range(num_inputs - 1)]
        indices = np.flip(start - np.cumsum([0] + steps))
        if (indices < 0).any():
            indices = indices + -indices.min()
            start = indices.min()
        indices = indices.copy()
        frame = int(indices[-1])
        end = frame + T
        in_steps = torch.tensor(indices - start).int().to(dev)
    else:
        frame, end, in_steps = start, start + T, None
    x = torch.empty(BN, 3, device=dev)
    v = torch.empty(BN, 3, device=dev)
    nodes = torch.empty(BN, 1, device=dev)
    ea = torch.empty(rows.numel(), 2, device=dev)
    t_in = torch.full((B,), frame + 1, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().nonode_prepare_inputs(B, N, Tf, _lib.ptr(locs), _lib.ptr(vels), _lib.ptr(t_in), None,
                                                _lib.ptr(prod), 1, _lib.ptr(x), _lib.ptr(v), _lib.ptr(nodes),
                                                _lib.ptr(ea), None, _lib.stream_of(locs)))
    loc_end = locs[end]
    if num_inputs > 1:
        idx = torch.as_tensor(indices, device=dev)
        loc, vel = locs[idx].transpose(0, 1).contiguous(), vels[idx].transpose(0, 1).contiguous()
        h = torch.sqrt(torch.sum(vel ** 2, dim=-1)).unsqueeze(-1)
        return h, loc, vel, ea, loc_end, in_steps, torch.stack([rows, cols])
    return nodes, x, v, ea, loc_end, None, torch.stack([rows, cols])
