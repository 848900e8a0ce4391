"""Drop-in message-passing convolutions (reference: vq_gnn_v2/convs.py).

``OurGCNConv`` (convs.py:26-101) — used for both GCN and SAGE layers
(models.py:93-94) — is ``out = A @ x`` over the batch adjacency
(PyG GCNConv.message_and_aggregate -> torch_sparse.matmul(adj_t, x,
reduce='add')); no weight, bias or normalisation inside (convs.py:69-99 are
commented out).  Here the product is the HIP edge-balanced SpMM, and the
layer's input ``x_input = [x ; x_first_order]`` (models.py:168-174) may be
passed as a ``GatheredInput`` pair so the concatenation is never copied: the
kernel reads rows < B from x and rows >= B from x_first_order -- or as a
``CodebookInput``, where x_first_order is never formed and the kernel reads
each out-of-batch row's codewords from an LDS image of the codebook.
"""
from __future__ import annotations

import math
import os
from typing import NamedTuple

import torch
from torch import nn

from . import kernels
from .sparse import CSR, as_csr


class GatheredInput(NamedTuple):
    """x_input = cat([x, x_first_order]) (models.py:174) without the cat.

    x: [B, F] batch rows (requires grad); x_first: [n - B, F] codeword rows of
    the out-of-batch nodes (a buffer: no gradient, models.py:169-173)."""
    x: torch.Tensor
    x_first: torch.Tensor

    @property
    def shape(self):
        return (self.x.shape[0] + self.x_first.shape[0], self.x.shape[1])

    def materialize(self):
        return torch.cat([self.x, self.x_first])


class CodebookInput(NamedTuple):
    """x_input = cat([x, x_first_order]) with x_first_order never formed:
    row j >= B is the codeword feature halves of node subset[j]'s codes
    (models.py:168-173), read by the SpMM from an LDS image of emb_out
    (kernels.spmm_codebook, include/vqgnn.h §6b)."""
    x: torch.Tensor
    subset: torch.Tensor
    codes: torch.Tensor
    emb_out: torch.Tensor
    D: int

    def supported(self, n_rows=None):
        """Whether the codebook-source kernel serves this input (its own
        shape limits, include/vqgnn.h §6b); else ``gathered()`` is used."""
        F = self.x.shape[1]
        return (hasattr(kernels.lib(), "vqgnn_spmm_task_cb") and
                kernels.codebook_source_ok(self.x, F, self.emb_out.shape[1], self.D,
                                           codes=self.codes,
                                           n_rows=n_rows if n_rows is not None
                                           else self.subset.numel(),
                                           n_branches=self.emb_out.shape[0],
                                           emb_out=self.emb_out))

    def gathered(self):
        """The GatheredInput form (x_first_order materialised by the gather)."""
        xf, _ = kernels.gather_codewords(self.subset, self.x.shape[0], self.codes,
                                         self.emb_out, self.D, nb=self.x.shape[1] // self.D)
        return GatheredInput(self.x, xf)


class _VQHook:
    """Backward-time VQ update (the LowRankGNNBlock.hook of models.py:39-56),
    applied to all branches of a layer in one batched call."""

    def __init__(self, layer, x_detached, batch_idx):
        self.layer, self.x, self.batch_idx = layer, x_detached, batch_idx

    def __call__(self, grad_out_B):
        self.layer._backward_vq_update(self.x, grad_out_B, self.batch_idx)

    def start(self, grad_out_B):
        """Run the update; with VQGNN_HOOK_OVERLAP=1 (single process) on a side
        stream beside the caller's A^T product (the two are independent:
        the update reads X and dOut[:B], writes codes and codebook; the
        product reads dOut and the transposed adjacency).  Returns the side
        stream to join after the product, or None."""
        if os.environ.get("VQGNN_HOOK_OVERLAP", "0") != "1" or \
                getattr(self.layer._bank, "comm", None) is not None:
            self(grad_out_B)
            return None
        main = torch.cuda.current_stream()
        side = _side_stream(grad_out_B.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self(grad_out_B)
        grad_out_B.record_stream(side)
        return side


_SIDE = {}


def _side_stream(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


def _join(side):
    if side is not None:
        torch.cuda.current_stream().wait_stream(side)


class GatherSpMMFunction(torch.autograd.Function):
    """out = A @ [x ; x_first]; d/dx = (A^T @ dout)[:B] (x_first_order is a
    buffer, models.py:169-174, so it receives no gradient)."""

    @staticmethod
    def forward(ctx, x, adj, x_first, hook, anchor):
        B, F = x.shape
        n = adj.size(0)
        xc = x if (x.stride(1) == 1 and x.stride(0) % 4 == 0 and
                   x.data_ptr() % 16 == 0) else x.contiguous()
        out = kernels.spmm(adj.rowptr, adj.col, adj.value, n, adj.nnz(), xc, F, X2=x_first, B=B,
                           plan=adj.plan(F, B=B))
        ctx.adj, ctx.B, ctx.hook = adj, B, hook
        return out

    @staticmethod
    def backward(ctx, dout):
        B = ctx.B
        dout = dout.contiguous()
        side = ctx.hook.start(dout[:B]) if ctx.hook is not None else None
        dx = None
        if ctx.needs_input_grad[0]:
            at = ctx.adj.transposed()
            F = dout.shape[1]
            # rows [0, B) of A^T = columns [0, B) of A; the merge kernel bounds
            # the walk with the full nnz, so no host read of t_rowptr[B] is needed
            dx = kernels.spmm(at.rowptr, at.col, at.value, B, at.nnz(), dout, F,
                              plan=at.plan(F, n_rows=B))
        _join(side)
        return dx, None, None, None, None


class CodebookSpMMFunction(GatherSpMMFunction):
    """GatherSpMMFunction with the out-of-batch rows read from the codebook
    (kernels.spmm_codebook); same backward (A^T dout)[:B]."""

    @staticmethod
    def forward(ctx, x, adj, src, hook, anchor):
        B, F = x.shape
        n = adj.size(0)
        xc = x if (x.stride(1) == 1 and x.stride(0) % 4 == 0 and
                   x.data_ptr() % 16 == 0) else x.contiguous()
        plan = adj.plan_codebook(B, src.subset, src.codes.shape[0])
        out = kernels.spmm_codebook(adj.rowptr, n, adj.nnz(), xc, F, B, src.codes, src.emb_out,
                                    src.D, plan)
        ctx.adj, ctx.B, ctx.hook = adj, B, hook
        return out


class SpMMFunction(torch.autograd.Function):
    """out = A @ x for a dense x (the plain OurGCNConv call)."""

    @staticmethod
    def forward(ctx, x, adj):
        n_cols, F = x.shape
        pad = (-F) % 4
        xc = x.contiguous()
        if pad:
            xc = torch.nn.functional.pad(xc, (0, pad))
        out = kernels.spmm(adj.rowptr, adj.col, adj.value, adj.size(0), adj.nnz(), xc, F + pad,
                           plan=adj.plan(F + pad))
        ctx.adj, ctx.pad, ctx.F = adj, pad, F
        return out[:, :F] if pad else out

    @staticmethod
    def backward(ctx, dout):
        at = ctx.adj.transposed()
        d = dout.contiguous()
        if ctx.pad:
            d = torch.nn.functional.pad(d, (0, ctx.pad))
        dx = kernels.spmm(at.rowptr, at.col, at.value, at.size(0), at.nnz(), d, ctx.F + ctx.pad,
                          plan=at.plan(ctx.F + ctx.pad))
        return (dx[:, :ctx.F] if ctx.pad else dx), None


def _glorot_(t):
    stdv = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-stdv, stdv)


class OurGCNConv(nn.Module):
    """Reference: convs.py:26-101 (subclass of PyG GCNConv with forward =
    propagate only).  Keeps GCNConv's parameters (``weight`` [in, out] glorot,
    ``bias`` zeros) so the parameter set and the RNG stream at construction
    match the reference; both are unused in forward, as in the reference."""

    def __init__(self, in_channels, out_channels, improved=False, cached=False,
                 add_self_loops=True, normalize=True, bias=True, **kwargs):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.improved, self.cached = improved, cached
        self.add_self_loops, self.normalize = add_self_loops, normalize
        self.weight = nn.Parameter(torch.empty(in_channels, out_channels))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        _glorot_(self.weight)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x, edge_index, edge_weight=None, _hook=None):
        adj = as_csr(edge_index)
        if isinstance(x, CodebookInput):
            # narrower tiles than the full-width walk lose to the gather
            # (kernels.codebook_source_preferred)
            if x.supported(adj.size(0)) and kernels.codebook_source_preferred(x.emb_out.shape[1]):
                anchor = None
                if _hook is not None and not x.x.requires_grad:
                    anchor = torch.zeros((), device=x.x.device, requires_grad=True)
                return CodebookSpMMFunction.apply(x.x, adj, x, _hook, anchor)
            x = x.gathered()
        if isinstance(x, GatheredInput):
            anchor = None
            if _hook is not None and not x.x.requires_grad:
                # the v1 hook must run even for a first layer whose input needs
                # no grad (models.py:184 requires_grad_() on the output slice)
                anchor = torch.zeros((), device=x.x.device, requires_grad=True)
            return GatherSpMMFunction.apply(x.x, adj, x.x_first, _hook, anchor)
        return SpMMFunction.apply(x, adj)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"


__all__ = ["OurGCNConv", "GatheredInput", "CodebookInput", "CSR"]
