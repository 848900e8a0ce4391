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


# ---------------------------------------------------------------------------
# GAT (convs.py:165-266, utils/vq_softmax.py:33-57, models.py:178-179/:187-189)
# ---------------------------------------------------------------------------
def gat_forward(x_in, att_l, att_r, rowptr, col, val, B=None, normalize=False, slope=0.2):
    """The reference GAT aggregation in fp32 torch CPU ops, op for op:

    alpha_l = (x * att_l).sum(-1)                                 convs.py:189
    scale   = sqrt(max(alpha_l)**2 + 1) * sqrt(max(alpha_r)**2 + 1)   :209-210
    alpha_l /= scale; alpha_r /= scale                            :211-212
    a       = alpha_l[j] + alpha_r[i]   (j = col = source, i = row)   :254
    coef    = exp(leaky_relu(a, 0.2)) * w    (vq_softmax = exp)   :255-264
    out[i]  = sum_{e in row i} x_j * coef   (segment_csr, CSR order)  :266
    normalize: out[:B, :-1] /= out[:B, -1:] + 1e-16; drop the last column
                                                            models.py:187-189
    x_in [n, C] includes the ones column when the layer appends it."""
    x = torch.as_tensor(np.asarray(x_in, dtype=np.float32))
    attl = torch.as_tensor(np.asarray(att_l, dtype=np.float32)).view(-1)
    attr = torch.as_tensor(np.asarray(att_r, dtype=np.float32)).view(-1)
    al = (x * attl).sum(-1)
    ar = (x * attr).sum(-1)
    scale = torch.sqrt(torch.max(al) ** 2 + 1) * torch.sqrt(torch.max(ar) ** 2 + 1)
    al = al / scale
    ar = ar / scale
    rowptr = np.asarray(rowptr, dtype=np.int64)
    row = torch.as_tensor(np.repeat(np.arange(rowptr.shape[0] - 1), np.diff(rowptr)))
    j = torch.as_tensor(np.asarray(col, dtype=np.int64))
    a = al[j] + ar[row]
    a = torch.nn.functional.leaky_relu(a, slope)
    coef = a.exp() * torch.as_tensor(np.asarray(val, dtype=np.float32))
    out = torch.as_tensor(spmm_seq(rowptr, col, coef.numpy(), x.numpy()))
    if normalize:
        out[:B, :-1] /= out[:B, -1:] + 1e-16
        out = out[:, :-1]
    return out, coef


def gat_forward_fp64(x, x_first, att_l, att_r, rowptr, col, val, B, slope=0.2):
    """Differentiable fp64 restatement of the layer's GAT path (ones column
    appended, rows < B normalised) for gradient checks: inputs are torch
    tensors (x requires grad; att_l / att_r [C] require grad)."""
    n = B + x_first.shape[0]
    xin = torch.cat([torch.cat([x.double(), x_first.double()], 0),
                     torch.ones(n, 1, dtype=torch.float64)], 1)
    al = (xin * att_l.double()).sum(-1)
    ar = (xin * att_r.double()).sum(-1)
    scale = torch.sqrt(torch.max(al) ** 2 + 1) * torch.sqrt(torch.max(ar) ** 2 + 1)
    al, ar = al / scale, ar / scale
    rowptr = np.asarray(rowptr, dtype=np.int64)
    row = torch.as_tensor(np.repeat(np.arange(n), np.diff(rowptr)))
    j = torch.as_tensor(np.asarray(col, dtype=np.int64))
    coef = torch.nn.functional.leaky_relu(al[j] + ar[row], slope).exp() * \
        torch.as_tensor(np.asarray(val, dtype=np.float64))
    out = torch.zeros(n, xin.shape[1], dtype=torch.float64).index_add(
        0, row, xin[j] * coef[:, None])
    head = out[:B, :-1] / (out[:B, -1:] + 1e-16)
    return torch.cat([head, out[B:, :-1]], 0)
