"""CPU restatement of the reference's mini-batch construction (TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the product).

  k_hop_subgraph      vq_gnn_v2/dataloader.py:98-148 (OurDataLoader._k_hop_subgraph)
  sparse_tensor_csr   vq_gnn_v2/utils/misc.py:73 (SparseTensor(row=, col=, value=):
                      entries sorted by (row, col), stable)

torch CPU ops in the reference's sequence: node mask -> index_select of the
row mask -> neighbour columns per hop (:113-117), unique with inverse
(:119; CPU torch.unique returns ascending values whatever ``sorted`` says —
checked on torch 2.10), batch nodes moved to the front (:122-126), the
edge mask (:130-138), relabelling (:142-145).  The reference module is not
importable here (torch_geometric / ogb absent), so this restatement is pinned
by the hand-computed known answers in tests/test_host_logic.py.
"""
from __future__ import annotations

import torch


def _coo_rows(rowptr: torch.Tensor) -> torch.Tensor:
    counts = rowptr[1:] - rowptr[:-1]
    return torch.repeat_interleave(torch.arange(counts.numel(), dtype=torch.int64), counts)


def k_hop_subgraph(rowptr, col, val, N, node_idx, num_hops=1, train_flag=True):
    """-> (subset int64 [n], edge_index int64 [2, E], edge_w fp32 [E])."""
    rowptr = torch.as_tensor(rowptr, dtype=torch.int64)
    col = torch.as_tensor(col, dtype=torch.int64)
    val = torch.as_tensor(val, dtype=torch.float32)
    node_idx = torch.as_tensor(node_idx, dtype=torch.int64).flatten()
    row = _coo_rows(rowptr)

    reached = [node_idx]
    mask = torch.zeros(N, dtype=torch.bool)
    for _ in range(num_hops):
        mask.zero_()
        mask[reached[-1]] = True
        reached.append(col[mask.index_select(0, row)])

    uniq, inverse = torch.unique(torch.cat(reached), sorted=True, return_inverse=True)
    inverse = inverse[: node_idx.numel()]
    rest = torch.ones(uniq.numel(), dtype=torch.bool)
    rest[inverse] = False
    subset = torch.cat([uniq[inverse], uniq[rest]])
    assert torch.equal(node_idx, subset[: node_idx.numel()])

    mask.zero_()
    if train_flag:
        mask[subset] = True
        keep = mask[row] & mask[col]
    else:
        mask[node_idx] = True
        keep = mask[row]
    local = torch.full((N,), -1, dtype=torch.int64)
    local[subset] = torch.arange(subset.numel(), dtype=torch.int64)
    edge_index = local[torch.stack([row[keep], col[keep]])]
    return subset, edge_index, val[keep]


def sparse_tensor_csr(row, col, value, n_rows, n_cols):
    """-> (rowptr int64 [n_rows+1], col int64, value fp32) sorted by (row, col)."""
    row = torch.as_tensor(row, dtype=torch.int64)
    col = torch.as_tensor(col, dtype=torch.int64)
    value = torch.as_tensor(value, dtype=torch.float32) if value is not None else \
        torch.ones(row.numel(), dtype=torch.float32)
    order = torch.argsort(row * max(int(n_cols), 1) + col, stable=True)
    row, col, value = row[order], col[order], value[order]
    rowptr = torch.zeros(int(n_rows) + 1, dtype=torch.int64)
    rowptr[1:] = torch.cumsum(torch.bincount(row, minlength=int(n_rows)), 0)
    return rowptr, col, value


# ---------------------------------------------------------------------------
# Random walks of the 'edge' / 'rw' / 'cont' samplers (dataloader.py:70-90):
# SparseTensor.random_walk -> torch_cluster random_walk (p = q = 1).
# torch_cluster is a dependency the reference does not vendor; its uniform
# step (rw_cpu.cpp) draws rand = torch.rand([n, walk_length]) and moves from
# v to col[rowptr[v] + (int64)(rand * deg(v))], staying on v when deg(v) = 0.
# The step uniforms here are the HIP kernel's counter-based stream
# (include/vqgnn.h §9b), restated so the GPU walk is checked bit for bit;
# the structure is pinned by known answers (tests/test_subgraph_oracle.py),
# torch's RNG stream is not reproduced ("parity unpinned" for the draws).
# ---------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def walk_mix(z: int) -> int:
    """splitmix64 finaliser (include/vqgnn.h §9b)."""
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def walk_uniforms(seed: int, n: int, walk_length: int):
    """u[i][l] in [0, 1) as float32: (mix(mix(seed ^ mix(i)) + l) >> 40) * 2^-24."""
    import numpy as np
    u = np.empty((n, walk_length), dtype=np.float32)
    for i in range(n):
        base = walk_mix((seed & _M64) ^ walk_mix(i))
        for l in range(walk_length):
            u[i, l] = np.float32((walk_mix((base + l) & _M64) >> 40) * 2.0 ** -24)
    return u


def random_walk(rowptr, col, start, walk_length, u):
    """torch_cluster's uniform random walk given the step uniforms u [n, L]:
    [n, L + 1] int64, out[:, 0] = start."""
    import numpy as np
    rowptr = np.asarray(rowptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    start = np.asarray(start, dtype=np.int64)
    out = np.empty((start.shape[0], walk_length + 1), dtype=np.int64)
    for i, v in enumerate(start):
        out[i, 0] = v
        for l in range(walk_length):
            rs, re = rowptr[v], rowptr[v + 1]
            if re > rs:
                e = rs + int(np.float32(u[i, l]) * np.float32(re - rs))
                v = col[min(e, re - 1)]
            out[i, l + 1] = v
    return out
