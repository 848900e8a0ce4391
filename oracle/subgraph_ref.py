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
