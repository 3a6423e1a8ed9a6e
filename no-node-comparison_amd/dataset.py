"""N-body datasets: the reference's .npy splits, loaded once, batched on the GPU.

``NBodyDynamicsDataset`` keeps the reference's constructor, file names, layout rules and
``__getitem__`` (EGNO/simulation/dataset_simple.py:6-178, num_inputs == 1), vectorised (no
per-edge Python loop). ``DeviceLoader`` replaces ``torch.utils.data.DataLoader`` for it: the whole
split sits in HBM and every batch is ONE gather launch (nonode_gather_batch) over the implicit
fully connected edge list (no int64 edge arrays), returning the 7-tuple run_epoch unpacks
(main_simulation_simple_no.py:200-201) already on the device.
"""
from pathlib import Path

import numpy as np
import torch

from . import _lib
from .graph import full_edges

_FRAME0 = {"nbody": 6, "nbody_small": 30, "nbody_small_out_dist": 20}   # dataset_simple.py:126,145


class NBodyDynamicsDataset:
    """dataset_simple.py:122-178 (and NBodyDataset :6-111) for num_inputs == 1."""

    def __init__(self, partition='train', data_dir='.', max_samples=1e8, dataset="charged", dataset_name="nbody_small",
                 n_balls=5, num_timesteps=10, num_inputs=1, traj_len=1, dT=1, varDT=False):
        if num_inputs != 1:
            raise NotImplementedError("NBodyDynamicsDataset: num_inputs > 1")
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
        """(frame_0, out_indices) of every sample (num_inputs == 1, dataset_simple.py:150-176)."""
        frame_0 = self.start
        frame_T = frame_0 + self.num_timesteps * self.traj_len * self.dT
        out = torch.arange(frame_0 + 1, frame_T + 1, self.dT)
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

    Yields (loc [B,N,3], vel [B,N,3], edge_attr [B,N(N-1),1], charges [B,N,1], loc_true [B,N,To,3],
    frame_0 [B] int64, out_indices [B,To] int64), all on ``device``, as run_epoch's
    ``[d.to(device) for d in data]`` would hold them (the split, including the loader's per-sample
    edge features, is copied to the device once). ``shuffle`` draws torch.randperm from
    ``generator`` each epoch (DataLoader's RandomSampler draws its own permutation from a derived
    seed, so the sample order differs from the reference's for the same seed)."""

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
        f0, out = dataset.frames()
        self.frame_0 = int(f0)
        self.out_indices = out
        self._out_dev = out.to(torch.int32).to(dev)

    def __len__(self):
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def batch(self, idx):
        """Gather the samples idx (sequence or tensor) as one batch."""
        dev = self.loc.device
        idx = torch.as_tensor(idx, dtype=torch.int32).to(dev)
        B, (S, Tf, N, _), To = idx.numel(), self.loc.shape, self.out_indices.numel()
        f0 = torch.full((B,), self.frame_0, dtype=torch.int32, device=dev)
        oi = self._out_dev.unsqueeze(0).expand(B, To).contiguous()
        loc0 = torch.empty(B, N, 3, device=dev)
        vel0 = torch.empty(B, N, 3, device=dev)
        q = torch.empty(B, N, 1, device=dev)
        ea = torch.empty(B, N * (N - 1), 1, device=dev)
        lt = torch.empty(B, N, To, 3, device=dev)
        _lib.check(_lib.lib().nonode_gather_batch(S, Tf, N, B, To, _lib.ptr(self.loc), _lib.ptr(self.vel),
                                                  _lib.ptr(self.q), _lib.ptr(self.ea), _lib.ptr(idx), _lib.ptr(f0),
                                                  _lib.ptr(oi),
                                                  _lib.ptr(loc0), _lib.ptr(vel0), _lib.ptr(q), _lib.ptr(ea),
                                                  _lib.ptr(lt), _lib.stream_of(self.loc)))
        return (loc0, vel0, ea, q, lt, f0.long(), oi.long())

    def __iter__(self):
        n = len(self.dataset)
        order = torch.randperm(n, generator=self.generator) if self.shuffle else torch.arange(n)
        for k in range(len(self)):
            yield self.batch(order[k * self.batch_size:(k + 1) * self.batch_size])
