"""CPU restatement of the reference's full-graph preprocessing (TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the product).

  norm_adj       vq_gnn_v2/utils/misc.py:14-34 (torch_sparse set_diag, sum(dim=1),
                 pow, row / column scaling)
  to_symmetric   SparseTensor.to_symmetric() used at misc.py:190, :211
  permute        SparseTensor.permute(perm) used at misc.py:113-130

Arithmetic notes (checked on torch 2.10, CPU capability AVX512):
* ``deg.pow(-1/2)`` runs ATen's CPU rsqrt, which is not the correctly
  rounded 1/sqrt: it is up to 2 ulp away (91 of the integers 1..19999 differ
  from fl(1/fl(sqrt(x)))), and which bits come out depends on the CPU build.
  ``norm_adj(..., rsqrt='ieee')`` restates the device's fl(1/fl(sqrt)) (bit
  for bit); ``rsqrt='torch'`` uses torch.pow as the reference does.
* ``deg.pow(-1)`` is fl(1/x) exactly (all floats checked).
* ``adj_t.sum(dim=1)`` is a sequential fp32 sum per row (torch_scatter's CPU
  segment_csr), restated with a float32 cumulative sum.
"""
from __future__ import annotations

import numpy as np
import torch


def _rows(rowptr):
    rowptr = np.asarray(rowptr, dtype=np.int64)
    return np.repeat(np.arange(rowptr.shape[0] - 1), np.diff(rowptr))


def _csr_from_sorted(r, c, v, N):
    rowptr = np.zeros(N + 1, dtype=np.int64)
    rowptr[1:] = np.cumsum(np.bincount(r, minlength=N))
    return rowptr, c.astype(np.int64), v.astype(np.float32)


def set_diag(rowptr, col, val, N):
    """torch_sparse set_diag(values=None): existing diagonal removed, a
    diagonal of ones inserted; entries stay sorted by (row, col)."""
    r = _rows(rowptr)
    c = np.asarray(col, dtype=np.int64)
    v = np.ones(c.shape[0], np.float32) if val is None else np.asarray(val, np.float32)
    off = r != c
    r = np.concatenate([r[off], np.arange(N)])
    c = np.concatenate([c[off], np.arange(N)])
    v = np.concatenate([v[off], np.ones(N, np.float32)])
    order = np.lexsort((c, r))
    return _csr_from_sorted(r[order], c[order], v[order], N)


def row_sums_sequential(rowptr, val):
    """adj_t.sum(dim=1) in CSR order, one fp32 rounding per add."""
    out = np.zeros(len(rowptr) - 1, np.float32)
    for i in range(len(rowptr) - 1):
        a, b = rowptr[i], rowptr[i + 1]
        if b > a:
            out[i] = np.cumsum(val[a:b], dtype=np.float32)[-1]
    return out


def norm_adj(rowptr, col, val, N, conv_type, rsqrt="ieee"):
    """-> (rowptr int64, col int64, val fp32) of the normalised adjacency."""
    if conv_type in ("GCN", "GAT"):
        rowptr, col, val = set_diag(rowptr, col, val, N)
    else:
        rowptr = np.asarray(rowptr, np.int64)
        col = np.asarray(col, np.int64)
        val = np.ones(col.shape[0], np.float32) if val is None else np.asarray(val, np.float32)
    deg = row_sums_sequential(rowptr, val)
    r = _rows(rowptr)
    if conv_type == "GCN":
        if rsqrt == "ieee":
            with np.errstate(divide="ignore"):
                dis = np.float32(1) / np.sqrt(deg)
        else:
            dis = torch.from_numpy(deg).pow(-1 / 2).numpy()
        dis[np.isinf(dis)] = 0
        v = (dis[r] * val) * dis[col]
    elif conv_type in ("SAGE", "GAT"):
        with np.errstate(divide="ignore"):
            di = torch.from_numpy(deg).pow(-1).numpy()
        di[np.isinf(di)] = 0
        v = di[r] * val
    else:
        raise ValueError('GNN conv type not supported')
    return rowptr, col, v.astype(np.float32)


def to_symmetric(rowptr, col, val, N):
    """A and A^T concatenated, coalesced: repeats summed (val None: pattern)."""
    r = _rows(rowptr)
    c = np.asarray(col, np.int64)
    v = np.ones(c.shape[0], np.float32) if val is None else np.asarray(val, np.float32)
    rr = np.concatenate([r, c])
    cc = np.concatenate([c, r])
    vv = np.concatenate([v, v])
    key = rr * N + cc
    order = np.argsort(key, kind="stable")
    key, vv = key[order], vv[order]
    uniq, start = np.unique(key, return_index=True)
    sums = np.add.reduceat(vv, start) if key.size else vv
    if val is None:
        sums = np.ones(uniq.shape[0], np.float32)
    return _csr_from_sorted(uniq // N, uniq % N, sums, N)


def permute(rowptr, col, val, N, perm):
    """SparseTensor.permute(perm): node i of the result = node perm[i]."""
    perm = np.asarray(perm, np.int64)
    inv = np.empty(N, np.int64)
    inv[perm] = np.arange(N)
    r = inv[_rows(rowptr)]
    c = inv[np.asarray(col, np.int64)]
    v = np.ones(c.shape[0], np.float32) if val is None else np.asarray(val, np.float32)
    order = np.lexsort((c, r))
    return _csr_from_sorted(r[order], c[order], v[order], N)
