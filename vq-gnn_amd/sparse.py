"""CSR container for the mini-batch adjacency.

The reference passes a torch_sparse ``SparseTensor`` built in
``prepare_batch_input`` (vq_gnn_v2/utils/misc.py:73): rows sorted by
(row, col), n x n, with the normalised edge weights as values.  torch_sparse is
not a dependency here; ``CSR`` keeps the surface the hot path uses
(``csr()``, ``coo()``, ``sparse_sizes()``, ``nnz()``, ``to()``) and the
device-side int32 index arrays the HIP kernels read.  ``as_csr`` also accepts a
torch_sparse-like object (anything with ``.csr()`` / ``sparse_sizes()``) or a
``torch.sparse_csr`` tensor, so a caller holding the reference's adjacency can
pass it unchanged.
"""
from __future__ import annotations

import torch


class CSR:
    __slots__ = ("rowptr", "col", "value", "_sizes", "_t", "_host_nnz", "_rows", "t_perm",
                 "_plans")

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, value: torch.Tensor | None,
                 sparse_sizes):
        self.rowptr = rowptr.to(torch.int32).contiguous()
        self.col = col.to(torch.int32).contiguous()
        if value is None:
            value = torch.ones(self.col.shape[0], dtype=torch.float32, device=self.col.device)
        self.value = value.to(torch.float32).contiguous()
        self._sizes = (int(sparse_sizes[0]), int(sparse_sizes[1]))
        self._t = None
        self._rows = None
        self.t_perm = None
        self._plans = {}
        self._host_nnz = int(self.col.shape[0])
        if self.rowptr.shape[0] != self._sizes[0] + 1:
            raise ValueError("rowptr must have n_rows + 1 entries")

    # ---- construction (same ordering rule as SparseTensor(row=, col=, ...)) ----
    @classmethod
    def from_coo(cls, row, col, value, sparse_sizes, is_sorted=False):
        n_rows, n_cols = int(sparse_sizes[0]), int(sparse_sizes[1])
        row = row.to(torch.int64)
        col = col.to(torch.int64)
        if not is_sorted and row.numel() > 0:
            key = row * max(n_cols, 1) + col
            perm = torch.argsort(key, stable=True)
            row, col = row[perm], col[perm]
            if value is not None:
                value = value[perm]
        counts = torch.bincount(row, minlength=n_rows) if row.numel() else \
            torch.zeros(n_rows, dtype=torch.int64, device=row.device)
        rowptr = torch.zeros(n_rows + 1, dtype=torch.int64, device=row.device)
        rowptr[1:] = torch.cumsum(counts, 0)
        return cls(rowptr, col, value, (n_rows, n_cols))

    # ---- torch_sparse-compatible surface ----
    def sparse_sizes(self):
        return self._sizes

    def sizes(self):
        return list(self._sizes)

    def size(self, dim):
        return self._sizes[dim]

    def nnz(self) -> int:
        return self._host_nnz

    def csr(self):
        return self.rowptr.to(torch.int64), self.col.to(torch.int64), self.value

    def coo(self):
        counts = self.rowptr[1:] - self.rowptr[:-1]
        row = torch.repeat_interleave(
            torch.arange(self._sizes[0], device=self.rowptr.device), counts.to(torch.int64))
        return row, self.col.to(torch.int64), self.value

    def has_value(self):
        return True

    @property
    def device(self):
        return self.col.device

    def to(self, device, non_blocking=False):
        out = CSR.__new__(CSR)
        out.rowptr = self.rowptr.to(device, non_blocking=non_blocking)
        out.col = self.col.to(device, non_blocking=non_blocking)
        out.value = self.value.to(device, non_blocking=non_blocking)
        out._sizes = self._sizes
        out._t = None
        out._rows = None
        out.t_perm = None
        out._plans = {}
        out._host_nnz = self._host_nnz
        return out

    def cuda(self, device=None):
        return self.to(device if device is not None else "cuda")

    def transposed(self):
        """A^T as CSR, built on the device by vqgnn_csr_transpose; cached, with
        the permutation ``t_perm`` (transposed entry -> input entry)."""
        if self._t is None:
            from . import kernels
            tr, tc, tv, tp = kernels.csr_transpose(self.rowptr, self.col, self.value,
                                                   self._sizes[0], self._sizes[1],
                                                   self._host_nnz, want_perm=True)
            t = CSR.__new__(CSR)
            t.rowptr, t.col, t.value = tr, tc, tv
            t._sizes = (self._sizes[1], self._sizes[0])
            t._t = self
            t._host_nnz = self._host_nnz
            t._rows = None
            t.t_perm = None
            t._plans = {}
            self.t_perm = tp
            self._t = t
        return self._t

    def plan(self, F=None, B=None, n_rows=None, kind=None):
        """SpMM plan, cached like torch_sparse's storage caches: the task plan
        (include/vqgnn.h §6) -- per-edge records of this CSR's values, task
        starts and fix-up jobs, valid for any F and any leading row count
        (products with other values on the same structure, e.g. GAT's
        coefficients: ``plan().with_values(col, values)``).  F, B, n_rows and
        kind are accepted for call-site symmetry and do not change the plan
        (kind must be None or "task"; the dense-block and hot-column tile
        plans were measured slower and removed)."""
        from . import kernels
        if kind not in (None, "task"):
            raise ValueError(f"CSR.plan: unknown kind {kind!r} (only the task plan remains, "
                             "DESIGN.md §4.2b, §4.2c)")
        p = self._plans.get("task")
        if p is None:
            p = kernels.spmm_task_plan(self.rowptr, self.col, self.value, self._sizes[0],
                                       self._host_nnz, n_cols=self._sizes[1])
            self._plans["task"] = p
        return p

    def plan_codebook(self, B, subset, n_nodes):
        """The codebook-source plan of kernels.spmm_codebook (columns >= B
        name the node subset[j]), cached per (B, subset) like plan()."""
        # the entry keeps the subset tensor: a cached plan is reused only for
        # that same tensor, unmodified (its version counter), never for new
        # node ids that happen to sit at the same address
        key = ("cb", int(B), int(n_nodes))
        ent = self._plans.get(key)
        if ent is not None and ent[0] is subset and ent[1] == subset._version:
            return ent[2]
        p = self.plan().with_codebook_source(B, subset, n_nodes)
        self._plans[key] = (subset, subset._version, p)
        return p

    def rows(self):
        """COO row index of every entry (int32, on the device); cached."""
        if self._rows is None:
            from . import kernels
            self._rows = kernels.csr_expand_rows(self.rowptr, self._sizes[0], self._host_nnz)
        return self._rows

    def __repr__(self):
        return f"CSR(sizes={self._sizes}, nnz={self._host_nnz}, device={self.device})"


def as_csr(adj) -> CSR:
    """Accept our CSR, a torch_sparse-like SparseTensor, or torch.sparse_csr."""
    if isinstance(adj, CSR):
        return adj
    if isinstance(adj, torch.Tensor) and adj.layout == torch.sparse_csr:
        return CSR(adj.crow_indices(), adj.col_indices(), adj.values(), adj.shape)
    if hasattr(adj, "csr") and hasattr(adj, "sparse_sizes"):
        cached = getattr(adj, "_vqgnn_csr", None)
        if cached is not None:
            return cached
        rowptr, col, value = adj.csr()
        out = CSR(rowptr, col, value, adj.sparse_sizes())
        try:
            adj._vqgnn_csr = out
        except AttributeError:
            pass
        return out
    raise TypeError(f"unsupported adjacency type {type(adj)}")
