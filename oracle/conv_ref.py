"""Oracle for the aggregation half (reference: vq_gnn_v2/convs.py,
models.py:157-189).  TEST INFRASTRUCTURE ONLY.

spmm_seq restates torch_sparse's CPU spmm_sum (csrc/cpu/spmm_cpu.cpp): per
row, ``out = 0; for e in row (CSR order): out = out + val[e] * x[col[e]]`` in
fp32 with a separate multiply and add — vectorised here over the k-th edge of
every row so it stays numpy-fast.  spmm_fp64 is an independent fp64
index_add formulation for cross-checking.
"""
from __future__ import annotations

import numpy as np
import torch


def spmm_seq(rowptr, col, val, x):
    """out[i] = sum_{e in row i} val[e] * x[col[e]] (fp32, CSR order, mul+add)."""
    rowptr = np.asarray(rowptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    val = np.asarray(val, dtype=np.float32)
    x = np.asarray(x, dtype=np.float32)
    n = rowptr.shape[0] - 1
    out = np.zeros((n, x.shape[1]), dtype=np.float32)
    deg = np.diff(rowptr)
    if n == 0 or deg.max(initial=0) == 0:
        return out
    for k in range(int(deg.max())):
        rows = np.nonzero(deg > k)[0]
        e = rowptr[rows] + k
        prod = (val[e][:, None] * x[col[e]]).astype(np.float32)
        out[rows] = (out[rows] + prod).astype(np.float32)
    return out


def spmm_fp64(rowptr, col, val, x):
    rowptr = torch.as_tensor(np.asarray(rowptr), dtype=torch.int64)
    n = rowptr.shape[0] - 1
    row = torch.repeat_interleave(torch.arange(n), rowptr[1:] - rowptr[:-1])
    xd = torch.as_tensor(np.asarray(x)).double()
    v = torch.as_tensor(np.asarray(val)).double()
    c = torch.as_tensor(np.asarray(col), dtype=torch.int64)
    out = torch.zeros(n, xd.shape[1], dtype=torch.float64)
    out.index_add_(0, row, xd[c] * v[:, None])
    return out.numpy()


def gather_input(x, subset, B, codes, emb_out, D):
    """models.py:157-174: x_input = cat([x, cat_b emb_out[b][c_b[subset[B:]], :D]]).
    codes: [N, nb] int16 (column b = branch b's c_indices); emb_out [nb, M, 2D]."""
    x = torch.as_tensor(x)
    first = torch.as_tensor(np.asarray(subset[B:]), dtype=torch.int64)
    codes = torch.as_tensor(codes)
    nb = codes.shape[1]
    parts = []
    for b in range(nb):
        c = codes[first, b].to(torch.long)                 # :168
        cb = torch.as_tensor(emb_out[b])[c]                # :169
        parts.append(cb[:, :D])                            # :170
    return torch.cat([x, torch.cat(parts, dim=1)]) if nb else x   # :173-174


def grad_first_order(subset, B, codes, emb_out, D):
    first = torch.as_tensor(np.asarray(subset[B:]), dtype=torch.int64)
    codes = torch.as_tensor(codes)
    parts = [torch.as_tensor(emb_out[b])[codes[first, b].long()][:, D:] for b in range(codes.shape[1])]
    return torch.cat(parts, dim=1)                          # :171-173
