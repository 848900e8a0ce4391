"""Drop-in GAT convolution (reference: vq_gnn_v2/convs.py:124-266,
utils/vq_softmax.py:33-57, and the ones-column normalisation in
models.py:178-179 / :187-189).

OurGATConv keeps PyG GATConv's parameters (``lin_l`` = ``lin_r`` Linear with
no bias, ``att_l`` / ``att_r`` [1, heads, C], optional ``bias``) and their
initialisation order, so the RNG stream at construction matches the reference.
The arithmetic runs in HIP (include/vqgnn.h §8):

  alpha_l/r = x_in . att_l/r (+ global max -> scale s,    vqgnn_gat_alpha
              alpha / s once per node, convs.py:209-211)
  coef_e    = exp(leaky(alpha_l[j]/s + alpha_r[i]/s)) * w  } vqgnn_gat_spmm_task (one
  out       = sum_e coef_e * x_in[j]                       } fused kernel; the
  rows < B  : out /= sum_e coef_e + 1e-16                  } coefficients stay in
                                                              registers)

The backward (dX for the batch rows, d att_l, d att_r) differentiates the same
chain: the transposed-coefficient SpMM, vqgnn_gat_edge_grad for the
coefficient chain (exp, leaky_relu, the 1/s scaling), the global-max
gradient, and the x_in^T d alpha reductions.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import kernels
from .convs import _join
from .sparse import as_csr


def _glorot_(t):
    stdv = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-stdv, stdv)


class GATFunction(torch.autograd.Function):
    """z = GAT aggregation of x_in = [x ; x_first ; 1 (if ones)] over adj.

    normalize=True: rows < B divided by their ones-column sum (the layer's
    GAT path).  x_first (may be None) receives no gradient (models.py: a
    buffer of codewords)."""

    @staticmethod
    def forward(ctx, x, x_first, att_l, att_r, adj, B, ones, normalize, slope, hook, anchor):
        n, nnz = adj.size(0), adj.nnz()
        F = x.shape[1]
        xc = x.contiguous()
        al, ar, params, als, ars = kernels.gat_alpha(xc, att_l, att_r, F, X2=x_first, B=B,
                                                     ones=ones)
        # the fused attention path runs on the task plan (coefficients computed
        # per edge record), also for dense-block adjacencies
        plan = adj.plan(F, kind="task")
        # fused: coefficients, ones-column sums and the normalisation in the
        # aggregation kernel; coef / den kept only when a backward follows
        # (grad mode is off inside forward: ask the context what the backward
        # will need)
        grad = any(ctx.needs_input_grad[:4])
        out, den, coef = kernels.gat_spmm(
            adj.rowptr, adj.col, adj.value, n, nnz, xc, F, als, ars, plan, adj.rows(),
            X2=x_first, B=B if x_first is not None else None,
            norm_B=B if normalize else 0, negative_slope=slope, want_den=grad,
            want_coef=grad)
        ctx.save_for_backward(xc, x_first if x_first is not None else xc, att_l, att_r, al, ar,
                              als, ars, params, coef, den, out)
        ctx.has_first = x_first is not None
        ctx.adj, ctx.B, ctx.ones, ctx.normalize, ctx.slope, ctx.hook = \
            adj, B, ones, normalize, slope, hook
        return out

    @staticmethod
    def backward(ctx, dz):
        xc, x_first, att_l, att_r, al, ar, als, ars, params, coef, den, z = ctx.saved_tensors
        if not ctx.has_first:
            x_first = None
        adj, B, F = ctx.adj, ctx.B, xc.shape[1]
        nnz = adj.nnz()
        dz = dz.contiguous()
        eps = 1e-16
        dden = None
        if ctx.normalize:
            # z = y / (den + eps) for rows < B  ->  dy = dz / (den + eps),
            # d den = -sum_c dz * z / (den + eps)
            q = den[:B] + eps
            dy = dz.clone()
            dy[:B] = dz[:B] / q[:, None]
            dden = torch.zeros_like(den)
            dden[:B] = -(dz[:B] * z[:B]).sum(1) / q
        else:
            dy = dz
        side = ctx.hook.start(dy[:B]) if ctx.hook is not None else None
        # coefficient chain -> d alpha_l, d alpha_r, d s
        dal, dar, dsr = kernels.gat_edge_grad(adj.rows(), adj.col, coef, nnz, xc, F, dy, dden,
                                              als, ars, params, X2=x_first, B=B,
                                              negative_slope=ctx.slope)
        ds = dsr.sum()
        # s = sqrt(max_l^2+1) sqrt(max_r^2+1); torch.max spreads its gradient
        # evenly over tied maxima
        ml, mr = params[0], params[1]
        tl = (al == ml).to(al.dtype)
        tr = (ar == mr).to(ar.dtype)
        dal = dal + tl * (ds * params[3] / tl.sum())
        dar = dar + tr * (ds * params[4] / tr.sum())
        # alpha = x_in . att
        C = att_l.numel()

        def datt(da):
            g = torch.zeros(C, dtype=torch.float32, device=da.device)
            g[:F] = xc.t().mv(da[:B])
            if x_first is not None and x_first.shape[0]:
                g[:F] += x_first.t().mv(da[B:])
            if ctx.ones:
                g[F] = da.sum()
            return g

        if (ctx.needs_input_grad[2] or ctx.needs_input_grad[3]) and F % 4 == 0:
            gl, gr = kernels.gat_att_grad(xc, F, dal, dar, X2=x_first, B=B, ones=ctx.ones)
            d_att_l = gl.view_as(att_l) if ctx.needs_input_grad[2] else None
            d_att_r = gr.view_as(att_r) if ctx.needs_input_grad[3] else None
        else:
            d_att_l = datt(dal).view_as(att_l) if ctx.needs_input_grad[2] else None
            d_att_r = datt(dar).view_as(att_r) if ctx.needs_input_grad[3] else None
        dx = None
        if ctx.needs_input_grad[0]:
            t = adj.transposed()
            tcoef = coef[adj.t_perm.long()]
            # rows [0, B) of A_coef^T dy: the transpose's task plan with the
            # coefficients as record weights (no new plan, no host read)
            cplan = t.plan(F, kind="task").with_values(t.col, tcoef)
            dx = kernels.spmm(t.rowptr, t.col, tcoef, B, nnz, dy, F, plan=cplan)
            dx += dal[:B, None] * att_l.view(-1)[:F] + dar[:B, None] * att_r.view(-1)[:F]
        _join(side)
        return dx, None, d_att_l, d_att_r, None, None, None, None, None, None, None


class OurGATConv(nn.Module):
    """Reference: convs.py:124-266 (PyG GATConv subclass).  Only heads = 1 is
    used by VQ-GNN (models.py:97: OurGATConv(C, C, bias=False,
    add_self_loops=False), C = in_channels + 1)."""

    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2,
                 dropout=0.0, add_self_loops=True, bias=True, **kwargs):
        super().__init__()
        if heads != 1:
            raise NotImplementedError("OurGATConv: heads > 1 is not used by VQ-GNN")
        if not isinstance(in_channels, int):
            raise NotImplementedError("OurGATConv: bipartite (x_l, x_r) inputs")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.heads, self.concat = heads, concat
        self.negative_slope, self.dropout = float(negative_slope), float(dropout)
        self.add_self_loops = add_self_loops
        self.lin_l = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.lin_r = self.lin_l
        self.att_l = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_r = nn.Parameter(torch.empty(1, heads, out_channels))
        if bias and concat:
            self.bias = nn.Parameter(torch.empty(heads * out_channels))
        elif bias and not concat:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self._alpha = None
        self.reset_parameters()

    def reset_parameters(self):   # PyG GATConv.reset_parameters order
        _glorot_(self.lin_l.weight)
        _glorot_(self.lin_r.weight)
        _glorot_(self.att_l)
        _glorot_(self.att_r)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def _check(self):
        if self.dropout > 0 and self.training:
            raise NotImplementedError("OurGATConv: attention dropout > 0 (VQ-GNN uses 0)")

    def forward(self, x, edge_index, size=None, return_attention_weights=None):
        """Reference forward on a dense x [n, C] (convs.py:165-245): no
        normalisation, no ones column added here; returns [n, C] (+ bias)."""
        self._check()
        if return_attention_weights:
            raise NotImplementedError("return_attention_weights")
        if self.add_self_loops:
            raise NotImplementedError("add_self_loops=True (VQ-GNN constructs with False)")
        adj = as_csr(edge_index)
        n, C = x.shape
        pad = (-C) % 4
        xp = torch.nn.functional.pad(x, (0, pad)) if pad else x
        al = torch.nn.functional.pad(self.att_l.view(-1), (0, pad)) if pad else self.att_l.view(-1)
        ar = torch.nn.functional.pad(self.att_r.view(-1), (0, pad)) if pad else self.att_r.view(-1)
        out = GATFunction.apply(xp, None, al, ar, adj, n, False, False, self.negative_slope,
                                None, None)
        out = out[:, :C] if pad else out
        if self.bias is not None:
            out = out + self.bias
        return out

    def fused_forward(self, x, adj, x_first, B, hook=None):
        """The layer's GAT path (models.py:174-189) without materialising x_in:
        x [B, F] (with grad), x_first [n-B, F] (buffer), implicit ones column;
        returns out [n, F] with rows < B normalised by their ones-column sum."""
        self._check()
        adj = as_csr(adj)
        F = x.shape[1]
        if self.att_l.numel() != F + 1:
            raise ValueError(f"att has {self.att_l.numel()} channels, expected {F + 1}")
        if self.bias is not None:
            # the reference adds the bias before the ones-column division; the
            # layer constructs the conv with bias=False (models.py:97)
            raise NotImplementedError("fused GAT path with bias")
        anchor = None
        if hook is not None and not x.requires_grad:
            # the v1 hook must run even when the layer input needs no grad
            anchor = torch.zeros((), device=x.device, requires_grad=True)
        return GATFunction.apply(x, x_first, self.att_l.view(-1), self.att_r.view(-1), adj, B,
                                 True, True, self.negative_slope, hook, anchor)

    def __repr__(self):
        return (f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, "
                f"heads={self.heads})")


__all__ = ["OurGATConv", "GATFunction"]
