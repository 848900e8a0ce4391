"""CPU restatement of VQ-GNN v1's ``mapper`` (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` and ``__graft_entry__.smoke()`` may import this module; the
product path is ``vqgnn_mapper`` in libvqgnn.so (include/vqgnn.h §11).

Reference: ``vq_gnn_v1/utils/dataloader.py:144-192`` (``mapper``): the
compressed (B+M) x (B+M) adjacency of one branch, in which every out-of-batch
neighbour is replaced by its codeword node ``B + c[j]``:

  rows/cols/values, concatenated in this order (``:148-170``):
    P0 A_BN:                (r, B + c[j], v)
    P1 A_NB (if A_NB_v):    (B + c[j], r, v_nb)
    P2 A_BB (if A_BB):      (r, s, v)                       (exact in-batch edges)
    P3 A_BB (if A_BB):      (r, B + c[batch_idx[s]], -v)    (their codeword copy removed)
    P4 (if A_BB and A_NB):  (B + c[batch_idx[r]], s, -v)
  ``coalesce(idx, val, m=dim, n=dim)`` (``:175``; torch_sparse: stable sort by
  row * dim + col, then segment_csr sum = sequential fp32 sum in that order),
  keep value > 0 (``:177-180``: sign cancellation drops the codeword copies of
  in-batch neighbours), then for gnn_type != 'SAGE' append self loops
  (i, i, deg_inv[i]) for i < B (``:182-185``), ``SparseTensor(row, col,
  value)`` (``:187``; a stable sort by (row, col), duplicates kept), and for
  'GCN' ``to_symmetric()`` (``:189-190``: A and A^T concatenated, stably
  sorted, repeated (row, col) summed sequentially).

Third-party semantics restated: torch_sparse ``coalesce`` / ``SparseStorage``
(sort + ``segment_csr``), ``SparseTensor.to_symmetric(reduce='sum')``.  The
sorts are taken as stable.  CPU ``torch.argsort`` (stable=False, what
torch_sparse calls) is not stable at every size on torch 2.10 (checked: it
differs from the stable order at 1,000 keys, matches at 10 and 10^5), so for a
(row, col) repeated three or more times the reference's own summation order
is unspecified; the stable order is the deterministic choice.  The reference
ships no fixtures for this function: parity is pinned by the hand-computed
known answers in ``tests/test_mapper_oracle.py``.
"""
from __future__ import annotations

import numpy as np


def _seq_coalesce(key: np.ndarray, val: np.ndarray):
    """Stable sort by key, repeated keys summed sequentially in fp32."""
    order = np.argsort(key, kind="stable")
    key = key[order]
    val = np.asarray(val, np.float32)[order]
    if key.size == 0:
        return key, val
    head = np.ones(key.size, bool)
    head[1:] = key[1:] != key[:-1]
    starts = np.nonzero(head)[0]
    ends = np.append(starts[1:], key.size)
    sums = np.empty(starts.size, np.float32)
    for i, (a, b) in enumerate(zip(starts, ends)):
        s = np.float32(0.0)
        for t in range(a, b):
            s = np.float32(s + val[t])
        sums[i] = s
    return key[starts], sums


def mapper(bn_row, bn_col, bn_val, c, num_B, num_M, gnn_type="GCN", nb_val=None,
           bb=None, batch_idx=None, deg_inv=None):
    """Returns (rowptr int64 [dim+1], col int64, val float32) of adj_input.

    bn_*: A_BN COO (local batch row, global column, value); c: codeword per
    global node; bb: (r, s, v) A_BB COO in local ids or None; nb_val: A_NB_v
    or None; deg_inv: [B] (needed unless gnn_type == 'SAGE')."""
    B, M = int(num_B), int(num_M)
    dim = B + M
    c = np.asarray(c, np.int64)
    r0 = np.asarray(bn_row, np.int64)
    j0 = np.asarray(bn_col, np.int64)
    v0 = np.asarray(bn_val, np.float32)
    cm = c[j0] + B
    rows, cols, vals = [r0], [cm], [v0]
    if nb_val is not None:
        rows.append(cm)
        cols.append(r0)
        vals.append(np.asarray(nb_val, np.float32))
    if bb is not None:
        br, bs, bv = (np.asarray(bb[0], np.int64), np.asarray(bb[1], np.int64),
                      np.asarray(bb[2], np.float32))
        bi = np.asarray(batch_idx, np.int64)
        rows.append(br)
        cols.append(bs)
        vals.append(bv)
        neg = (np.float32(-1.0) * bv).astype(np.float32)
        rows.append(br)
        cols.append(c[bi[bs]] + B)
        vals.append(neg)
        if nb_val is not None:
            rows.append(c[bi[br]] + B)
            cols.append(bs)
            vals.append(neg)
    row = np.concatenate(rows)
    col = np.concatenate(cols)
    val = np.concatenate(vals).astype(np.float32)
    key, s = _seq_coalesce(row * dim + col, val)
    keep = s > 0
    key, s = key[keep], s[keep]
    if gnn_type != "SAGE":
        loops = np.arange(B, dtype=np.int64)
        key = np.concatenate([key, loops * dim + loops])
        s = np.concatenate([s, np.asarray(deg_inv, np.float32)])
    order = np.argsort(key, kind="stable")   # SparseTensor(row=, col=, value=)
    key, s = key[order], s[order]
    if gnn_type == "GCN":                    # to_symmetric(): A and A^T, summed
        r, cc = key // dim, key % dim
        key, s = _seq_coalesce(np.concatenate([r * dim + cc, cc * dim + r]),
                               np.concatenate([s, s]))
    r, cc = key // dim, key % dim
    rowptr = np.zeros(dim + 1, np.int64)
    np.add.at(rowptr, r + 1, 1)
    return np.cumsum(rowptr), cc, s.astype(np.float32)


def mapper_torch(bn_row, bn_col, bn_val, c, num_B, num_M, gnn_type="GCN", nb_val=None, bb=None,
                 batch_idx=None, deg_inv=None):
    """The same op sequence in CPU torch tensors (the CPU baseline of
    scripts/bench_mapper.py): torch.cat, a stable sort by row * dim + col,
    index_add_ over the unique keys (sequential per key on the CPU), the
    value > 0 mask, the self loops, a stable sort, and to_symmetric."""
    import torch
    B, M = int(num_B), int(num_M)
    dim = B + M
    cm = c[bn_col].long() + B
    rows, cols, vals = [bn_row.long()], [cm], [bn_val]
    if nb_val is not None:
        rows.append(cm)
        cols.append(bn_row.long())
        vals.append(nb_val)
    if bb is not None:
        br, bs, bv = bb[0].long(), bb[1].long(), bb[2]
        rows += [br, br]
        cols += [bs, c[batch_idx[bs]].long() + B]
        vals += [bv, -1.0 * bv]
        if nb_val is not None:
            rows.append(c[batch_idx[br]].long() + B)
            cols.append(bs)
            vals.append(-1.0 * bv)
    key = torch.cat(rows) * dim + torch.cat(cols)
    val = torch.cat(vals)

    def coalesce(key, val):
        key, perm = torch.sort(key, stable=True)
        uk, inv = torch.unique_consecutive(key, return_inverse=True)
        s = torch.zeros(uk.numel(), dtype=val.dtype).index_add_(0, inv, val[perm])
        return uk, s

    key, s = coalesce(key, val)
    keep = s > 0
    key, s = key[keep], s[keep]
    if gnn_type != "SAGE":
        loops = torch.arange(B, dtype=torch.int64)
        key = torch.cat([key, loops * dim + loops])
        s = torch.cat([s, deg_inv])
    key, perm = torch.sort(key, stable=True)
    s = s[perm]
    if gnn_type == "GCN":
        r, cc = key // dim, key % dim
        key, s = coalesce(torch.cat([key, cc * dim + r]), torch.cat([s, s]))
    return key, s
