"""Fully connected, equal-size graph batches — the only topology the reference builds.

The reference materialises int64 edge lists per batch (EGNO/simulation/dataset_simple.py:64-71,
101-111; SEGNO/dataset_nbody.py:84-94): receiver row i, sender col j, ordered (b, i, j != i).
The kernels index that pattern implicitly, so the boundary checks once per edge tensor that the
caller's edge_index is exactly it, and raises ValueError otherwise.
"""
from collections import OrderedDict

import torch

# validated edge tensors, keyed by address / version / shape. Each entry holds a reference to its
# tensors, so their memory cannot be freed and reused by a different edge list while the entry
# exists (a key built from addresses alone would then match a tensor it never checked).
_checked = OrderedDict()
_CACHE = 8


def full_edges(B, N, device="cpu"):
    """Edge list of B fully connected N-node graphs in the reference order (row, col)."""
    i = torch.arange(N, device=device).repeat_interleave(N)
    j = torch.arange(N, device=device).repeat(N)
    keep = i != j
    i, j = i[keep], j[keep]
    off = (torch.arange(B, device=device) * N).repeat_interleave(i.numel())
    return i.repeat(B) + off, j.repeat(B) + off


def _split(edge_index):
    if isinstance(edge_index, (list, tuple)):
        if len(edge_index) != 2:
            raise ValueError("edge_index must be [rows, cols]")
        return edge_index[0], edge_index[1]
    if torch.is_tensor(edge_index) and edge_index.dim() == 2 and edge_index.shape[0] == 2:
        return edge_index[0], edge_index[1]
    raise ValueError("edge_index must be a pair of index tensors or a [2, E] tensor")


def check_full_graph(edge_index, n_nodes):
    """Return (B, N) for an edge list of B fully connected N-node graphs covering n_nodes nodes;
    raise ValueError if edge_index is anything else."""
    rows, cols = _split(edge_index)
    E = rows.numel()
    if cols.numel() != E or n_nodes <= 0 or E % n_nodes:
        raise ValueError(f"edge_index with {E} edges is not a fully connected batch over {n_nodes} nodes")
    N = E // n_nodes + 1
    if n_nodes % N or N < 2:
        raise ValueError(f"edge_index with {E} edges is not a fully connected batch over {n_nodes} nodes")
    B = n_nodes // N
    key = (rows.data_ptr(), cols.data_ptr(), rows._version, cols._version, E, n_nodes, str(rows.device))
    hit = _checked.get(key)
    if hit is not None:
        _checked.move_to_end(key)
        return hit[0], hit[1]
    r, c = full_edges(B, N, rows.device)
    if not (torch.equal(rows.to(torch.int64), r) and torch.equal(cols.to(torch.int64), c)):
        raise ValueError("edge_index is not the dataset's fully connected edge list "
                         "(receiver i, sender j != i, ordered by sample, i, j); the MI355X kernels "
                         "index that pattern implicitly")
    _checked[key] = (B, N, rows, cols)
    while len(_checked) > _CACHE:
        _checked.popitem(last=False)
    return B, N
