"""Full-graph preprocessing on the device, mirroring the
steps of ``get_data`` (vq_gnn_v2/utils/misc.py:178-224) with the arithmetic in
HIP (include/vqgnn.h §10):

* ``to_symmetric(adj_t)``  — ``data.adj_t.to_symmetric()`` (misc.py:190, :211)
* ``metis(adj_t, num_parts)`` — misc.py:93-111.  METIS (torch_sparse.partition)
  is absent; the substitute orders nodes by connected component, then BFS
  level from the component's smallest node, then id, and cuts that order into
  equal contiguous bands.  Same contract: ``(perm, ptr)`` with
  ``cluster_indices = arange(N).split(ptr diffs)`` after ``permute``.
* ``permute(data, perm)`` — misc.py:113-130 (node tensors ``[perm]``, the
  adjacency ``SparseTensor.permute``).
* ``norm_adj(data, conv_type)`` — misc.py:14-34, exact.

Graphs are ``DeviceGraph`` objects (loader.py): they expose ``.csr()`` and
``sparse_sizes()`` like the torch_sparse ``adj_t`` the reference holds.
"""
from __future__ import annotations

import copy
import time

import torch

from . import kernels
from .loader import DeviceGraph


def _graph(adj_t, device="cuda") -> DeviceGraph:
    if isinstance(adj_t, DeviceGraph):
        return adj_t
    n = adj_t.sparse_sizes()[0] if hasattr(adj_t, "sparse_sizes") else None
    return DeviceGraph.from_adj(adj_t, n, device)


def _values(g: DeviceGraph):
    return g.value if g.has_value else None


def to_symmetric(adj_t, device="cuda") -> DeviceGraph:
    """A + A^T pattern (duplicates summed when the graph has values)."""
    g = _graph(adj_t, device)
    rp, cl, vl = kernels.to_symmetric(g.rowptr, g.col, _values(g), g.N)
    out = DeviceGraph(rp, cl, vl, g.N, g.device)
    out.has_value = g.has_value
    return out


def norm_adj_graph(adj_t, conv_type, device="cuda") -> DeviceGraph:
    g = _graph(adj_t, device)
    rp, cl, vl = kernels.norm_adj(g.rowptr, g.col, _values(g), g.N, conv_type)
    return DeviceGraph(rp, cl, vl, g.N, g.device)


def norm_adj(data, conv_type, device="cuda"):
    """misc.py:14-34: data.adj_t <- the normalised adjacency (a DeviceGraph)."""
    data.adj_t = norm_adj_graph(data.adj_t, conv_type, device)
    return data


def metis(adj_t, num_parts: int, recursive: bool = False, log: bool = True, device="cuda"):
    """misc.py:93-111 contract: (perm, ptr) of a contiguous clustering."""
    t = time.perf_counter()
    if log:
        print(f'Computing METIS partitioning with {num_parts} parts...', end=' ', flush=True)
    g = _graph(adj_t, device)
    if num_parts <= 1:
        perm = torch.arange(g.N, device=g.device)
        ptr = torch.tensor([0, g.N], device=g.device)
    else:
        perm, ptr, _ = kernels.partition(g.rowptr, g.col, g.N, num_parts)
    if log:
        print(f'Done! [{time.perf_counter() - t:.2f}s]')
    return perm, ptr


def permute_graph(adj_t, perm, device="cuda") -> DeviceGraph:
    g = _graph(adj_t, device)
    rp, cl, vl = kernels.csr_permute(g.rowptr, g.col, _values(g), g.N, perm)
    out = DeviceGraph(rp, cl, vl, g.N, g.device)
    out.has_value = g.has_value
    return out


def permute(data, perm, log: bool = True, device="cuda"):
    """misc.py:113-130: node-sized tensors indexed by perm, the adjacency
    permuted; edge-sized tensors raise NotImplementedError as there."""
    t = time.perf_counter()
    if log:
        print('Permuting data...', end=' ', flush=True)
    data = copy.copy(data)
    n = int(data.num_nodes)
    for key, value in list(vars(data).items()):
        if key == "adj_t":
            data.adj_t = permute_graph(value, perm, device)
        elif isinstance(value, torch.Tensor) and value.dim() > 0 and value.size(0) == n:
            setattr(data, key, value[perm.to(value.device)])
        elif isinstance(value, torch.Tensor) and value.dim() > 0 and \
                value.size(0) == getattr(data, "num_edges", -1):
            raise NotImplementedError
    if log:
        print(f'Done! [{time.perf_counter() - t:.2f}s]')
    return data


__all__ = ["to_symmetric", "norm_adj", "norm_adj_graph", "metis", "permute", "permute_graph"]
