"""Thin torch-tensor wrappers over the C-ABI (include/vqgnn.h).

Each function validates shapes on the host, allocates outputs / workspace from
the PyTorch caching allocator and queues exactly the HIP kernels the C-ABI
entry point launches, on the current stream.  No function here computes
anything on the CPU or through ATen math: the arithmetic is in
csrc/*.hip.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import check, lib, ptr, require_gpu, stream_ptr, workspace

# bn_finalize modes (include/vqgnn.h §2)
BN_EVAL, BN_TRAIN, BN_TRAIN_INIT, BN_EVAL_INIT = 0, 1, 2, 3
# BatchNorm arithmetic of an input (include/vqgnn.h §2, oracle/bn_ref.py)
BN_FP64, BN_STRIDED, BN_CONTIG = 0, 1, 2


def _ld(t: torch.Tensor) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"expected a row-major 2-D view, got shape {tuple(t.shape)} "
                         f"strides {t.stride()}")
    return t.stride(0)


def bn_arith_of(t: torch.Tensor, D: int) -> int:
    """The ATen BatchNorm path the reference takes for each D-column branch
    slice of ``t`` [B, nb*D]: contiguous iff the slice is (row stride D, or
    one row), else strided (models.py:162-165 slices x[:, D*i:D*(i+1)])."""
    return BN_CONTIG if (_ld(t) == D or t.shape[0] <= 1) else BN_STRIDED


def bn_stats(X: torch.Tensor, G: torch.Tensor | None, F: int,
             with_count: bool = False) -> torch.Tensor:
    """fp64 column sums [4, F]: sum x, sum x^2, sum g, sum g^2 (vq.py:162/223).
    with_count: a flat [4F + 2] buffer: element 4F is the row count B (summed
    with the statistics by the multi-GPU all-reduce; bn_finalize with count=0
    reads it on the device), element 4F + 1 the over-capacity flag
    (CodebookSync.allreduce_stats_), 0 here."""
    require_gpu(X, "bn_stats")
    B = X.shape[0]
    L = lib()
    ws = workspace(L.vqgnn_bn_stats_workspace(B, F), X.device)
    flat = torch.empty(4 * F + 2 * int(with_count), dtype=torch.float64, device=X.device)
    sums = flat[:4 * F].view(4, F)
    # the kernels write every element (zeros for the g half without G; with
    # the count: flat[4F] = B, flat[4F + 1] = 0)
    fn = L.vqgnn_bn_stats_count if with_count else L.vqgnn_bn_stats
    check(fn(ptr(X), _ld(X), ptr(G), _ld(G) if G is not None else 0, B, F,
             int(G is not None), ptr(flat), ptr(ws), stream_ptr()), "bn_stats")
    return flat if with_count else sums


def _coef(F, with_grad, dev):
    coef = torch.empty(6, F, dtype=torch.float32, device=dev)
    if not with_grad:
        coef[2:4].zero_()
        coef[5].zero_()
    return coef


def bn_finalize(sums, count, F, with_grad, mode, mom_f, eps_f, mom_g, eps_g, eps_std,
                rm_f, rv_f, rm_g=None, rv_g=None, want_batch=False, nbt_f=None, nbt_g=None,
                D=0, arith_x=BN_FP64, arith_g=BN_FP64):
    """-> (coef [6, F], batch_out [4, F] or None); updates running stats in place
    and, when given, num_batches_tracked (nbt_f / nbt_g [F // D] int64) += 1.
    Batch statistics come from the fp64 sums (FP64 arithmetic); arith_x /
    arith_g choose the form of the eval coefficients."""
    dev = rm_f.device
    coef = _coef(F, with_grad, dev)
    batch = torch.empty(4, F, dtype=torch.float32, device=dev) if want_batch else None
    check(lib().vqgnn_bn_finalize(ptr(sums), int(count), F, int(with_grad), int(mode),
                                  int(arith_x), int(arith_g),
                                  float(mom_f), float(eps_f), float(mom_g), float(eps_g),
                                  float(eps_std), ptr(rm_f), ptr(rv_f), ptr(rm_g), ptr(rv_g),
                                  ptr(coef), ptr(batch), ptr(nbt_f), ptr(nbt_g), int(D),
                                  stream_ptr()), "bn_finalize")
    return coef, batch


def bn_stats_finalize(X, G, F, mode, mom_f, eps_f, mom_g, eps_g, eps_std, rm_f, rv_f,
                      rm_g=None, rv_g=None, want_batch=False, nbt_f=None, nbt_g=None, D=0,
                      want_sums=False, arith_x=BN_FP64, arith_g=BN_FP64, ref_threads=1):
    """Batch statistics + finalize for a single process (count = B) in the
    given arithmetic (BN_FP64 / BN_STRIDED / BN_CONTIG per half).
    -> (coef [6, F], batch_out or None, sums or None); sums only for FP64."""
    require_gpu(X, "bn_stats_finalize")
    B = X.shape[0]
    dev = X.device
    with_grad = G is not None
    L = lib()
    ws = workspace(L.vqgnn_bn_stats_workspace(B, F), dev)
    coef = _coef(F, with_grad, dev)
    batch = torch.empty(4, F, dtype=torch.float32, device=dev) if want_batch else None
    sums = torch.zeros(4, F, dtype=torch.float64, device=dev) if want_sums else None
    check(L.vqgnn_bn_stats_finalize(ptr(X), _ld(X), ptr(G), _ld(G) if with_grad else 0, B, F,
                                    int(with_grad), ptr(sums), int(mode), int(arith_x),
                                    int(arith_g), int(ref_threads), float(mom_f),
                                    float(eps_f), float(mom_g), float(eps_g), float(eps_std),
                                    ptr(rm_f), ptr(rv_f), ptr(rm_g), ptr(rv_g), ptr(coef),
                                    ptr(batch), ptr(nbt_f), ptr(nbt_g), int(D), ptr(ws),
                                    stream_ptr()), "bn_stats_finalize")
    return coef, batch, sums


class BnFold:
    """BatchNorm statistics whose finalize runs in the prologue of the next
    vq_assign (include/vqgnn.h §5b): the cascade partials are on the device,
    coef / batch are filled (and the running statistics, num_batches_tracked
    updated) by the assign's launch, in stream order.  Pass it as vq_assign's
    ``coef``; it serves one assign call over the same X / G."""
    __slots__ = ("ws", "X", "G", "F", "mode", "arith_x", "arith_g", "moms", "rm_f", "rv_f",
                 "rm_g", "rv_g", "coef", "batch", "nbt_f", "nbt_g", "D", "used")


def bn_fold_supported(B, nb, D, M, W) -> bool:
    """Whether vq_assign can fold the BatchNorm finalize for this shape."""
    return bool(lib().vqgnn_vq_assign_bn_supported(int(B), int(nb), int(D), int(M), int(W)))


def bn_stats_partial(X, G, F, mode, mom_f, eps_f, mom_g, eps_g, eps_std, rm_f, rv_f,
                     rm_g=None, rv_g=None, want_batch=False, nbt_f=None, nbt_g=None, D=0,
                     arith_x=BN_STRIDED, arith_g=BN_STRIDED) -> BnFold:
    """bn_stats_finalize's statistics pass alone (FP64 / STRIDED arithmetic);
    its finalize is folded into the vq_assign that receives the returned
    BnFold.  Same arguments and results as bn_stats_finalize."""
    require_gpu(X, "bn_stats_partial")
    if BN_CONTIG in (arith_x, arith_g if G is not None else arith_x):
        raise ValueError("bn_stats_partial: the CONTIG arithmetic has no folded finalize")
    B = X.shape[0]
    dev = X.device
    with_grad = G is not None
    L = lib()
    f = BnFold()
    f.ws = workspace(L.vqgnn_bn_stats_workspace(B, F), dev)
    check(L.vqgnn_bn_stats_partial(ptr(X), _ld(X), ptr(G), _ld(G) if with_grad else 0, B, F,
                                   int(with_grad), ptr(f.ws), stream_ptr()), "bn_stats_partial")
    f.X, f.G, f.F, f.mode, f.D = X, G, F, int(mode), int(D)
    f.arith_x, f.arith_g = int(arith_x), int(arith_g)
    f.moms = (float(mom_f), float(eps_f), float(mom_g), float(eps_g), float(eps_std))
    f.rm_f, f.rv_f, f.rm_g, f.rv_g = rm_f, rv_f, rm_g, rv_g
    f.nbt_f, f.nbt_g = nbt_f, nbt_g
    f.coef = _coef(F, with_grad, dev)
    f.batch = torch.empty(4, F, dtype=torch.float32, device=dev) if want_batch else None
    f.used = False
    return f


def stat_shifts(stat_count: int, grad_scale: float) -> tuple[int, int]:
    """Fixed-point scale of the EMA statistic slabs (include/vqgnn.h §3)."""
    import ctypes
    sf, sg = ctypes.c_int32(), ctypes.c_int32()
    lib().vqgnn_vq_stat_shifts(int(stat_count), float(grad_scale), ctypes.byref(sf),
                               ctypes.byref(sg))
    return sf.value, sg.value


def decode_stats(stats: torch.Tensor, D: int, stat_count: int, grad_scale: float) -> torch.Tensor:
    """int64 slab(s) [..., M, W+1] -> float64 (count, sum of normalised x)."""
    sf, sg = stat_shifts(stat_count, grad_scale)
    W = stats.shape[-1] - 1
    scale = torch.tensor([1.0] + [2.0 ** -sf] * D + [2.0 ** -sg] * (W - D), dtype=torch.float64,
                         device=stats.device)
    return stats.to(torch.float64) * scale


def vq_assign(X, G, coef, grad_scale, emb, D, W, idx_out=None, codes=None, batch_idx=None,
              want_stats=False, stat_count=None, stats_out=None):
    """Nearest codeword for every (row, branch); optional EMA statistics.

    emb: [nb, M, ldw] view (row-major per branch, arbitrary branch stride).
    Returns the EMA partial slabs [P, nb, M, W+1] (int64 fixed point, see
    decode_stats) if want_stats, else None; their sum over P is the statistic
    (vq_ema_reduce).  stat_count: rows behind the BN statistics (default B).
    stats_out: a caller-owned slab [P, nb, M, W+1] int64 that is already ZERO
    (e.g. left so by vq_ema_finalize(zero_after=True)); it is filled and
    returned, and the call skips zeroing it."""
    require_gpu(X, "vq_assign")
    B = X.shape[0]
    nb, M, ldw = emb.shape
    if emb.stride(2) != 1 or emb.stride(1) != ldw:
        raise ValueError("codebook must be row-major per branch")
    L = lib()
    parts = None
    ws = None
    # scratch: EMA row ids (non-fused path)
    ws = workspace(L.vqgnn_vq_assign_workspace(B, nb, M, W), X.device)
    if want_stats:
        P = L.vqgnn_vq_ema_parts(B, nb, M, W)
    ldc = 0
    if codes is not None:
        if codes.dtype != torch.int16 or codes.stride(1) != 1:
            raise ValueError("codes must be an int16 [N, ldc] row-major view")
        ldc = codes.stride(0)
    zeroed = 0
    if want_stats:
        if stats_out is not None:
            if (stats_out.dtype != torch.int64 or tuple(stats_out.shape) != (P, nb, M, W + 1)
                    or not stats_out.is_contiguous()):
                raise ValueError(f"stats_out must be a contiguous int64 [{P}, {nb}, {M}, {W + 1}]")
            parts, zeroed = stats_out, 1
        else:
            parts = torch.empty(P, nb, M, W + 1, dtype=torch.int64, device=X.device)
    count = int(stat_count if stat_count is not None else B)
    if isinstance(coef, BnFold):
        f = coef
        if f.used or f.X is not X or f.G is not G or f.F != nb * D:
            raise ValueError("vq_assign: a BnFold serves one assign over the X / G of its "
                             "bn_stats_partial")
        f.used = True
        mf, ef, mg, eg, es = f.moms
        check(L.vqgnn_vq_assign_bn(ptr(X), _ld(X), ptr(G), _ld(G) if G is not None else 0, B,
                                   nb, D, M, W, float(grad_scale), ptr(emb), ldw, emb.stride(0),
                                   ptr(idx_out), ptr(codes), ldc, ptr(batch_idx), ptr(parts),
                                   zeroed, count, ptr(ws), ptr(f.ws), f.mode, f.arith_x,
                                   f.arith_g, mf, ef, mg, eg, es, ptr(f.rm_f), ptr(f.rv_f),
                                   ptr(f.rm_g), ptr(f.rv_g), ptr(f.coef), ptr(f.batch),
                                   ptr(f.nbt_f), ptr(f.nbt_g), f.D, stream_ptr()), "vq_assign_bn")
        return parts
    check(L.vqgnn_vq_assign(ptr(X), _ld(X), ptr(G), _ld(G) if G is not None else 0, B, nb, D,
                            M, W, ptr(coef), float(grad_scale), ptr(emb), ldw, emb.stride(0),
                            ptr(idx_out), ptr(codes), ldc, ptr(batch_idx), ptr(parts), zeroed,
                            count, ptr(ws), stream_ptr()), "vq_assign")
    return parts


def vq_ema_reduce(parts):
    """[P, nb, M, W+1] -> [1, nb, M, W+1] (exact integer sum)."""
    P = parts.shape[0]
    if P == 1:
        return parts
    out = torch.empty((1,) + tuple(parts.shape[1:]), dtype=torch.int64, device=parts.device)
    check(lib().vqgnn_vq_ema_reduce(ptr(parts), P, parts[0].numel(), ptr(out), stream_ptr()),
          "vq_ema_reduce")
    return out


def vq_ema_finalize(parts, D, W, decay, laplace, grad_scale, epsilon, cs, ema_w, emb, emb_out,
                    rm_f, rv_f, rm_g, rv_g, bad_flag, stat_count, zero_after=False):
    P, nb, M, _ = parts.shape
    ldw = emb.shape[2]
    if not (ema_w.stride() == emb.stride() == emb_out.stride()):
        raise ValueError("ema_w / embedding / output must share one layout")
    if parts.dtype != torch.int64:
        raise ValueError("EMA statistic slabs are int64 fixed point")
    check(lib().vqgnn_vq_ema_finalize(ptr(parts), P, int(bool(zero_after)), int(stat_count), nb,
                                      M, D, W, ldw,
                                      float(decay),
                                      int(laplace), float(grad_scale), float(epsilon), ptr(cs),
                                      cs.stride(0), ptr(ema_w), ptr(emb), ptr(emb_out),
                                      emb.stride(0), ptr(rm_f), ptr(rv_f), ptr(rm_g), ptr(rv_g),
                                      ptr(bad_flag), stream_ptr()), "vq_ema_finalize")


def ema_finalize_args(parts, D, W, decay, laplace, grad_scale, epsilon, cs, ema_w, emb, emb_out,
                      rm_f, rv_f, rm_g, rv_g, bad_flag, stat_count, zero_after=False):
    """vq_ema_finalize's operands as include/vqgnn.h §4b's record, for
    spmm_codebook(finalize=...): the same checks; the tensors must outlive
    the call that consumes the record."""
    P, nb, M, _ = parts.shape
    if not (ema_w.stride() == emb.stride() == emb_out.stride()):
        raise ValueError("ema_w / embedding / output must share one layout")
    if parts.dtype != torch.int64:
        raise ValueError("EMA statistic slabs are int64 fixed point")
    from ._lib import EmaFinalizeArgs
    return EmaFinalizeArgs(
        ema_parts=parts.data_ptr(), nparts=P, zero_after=int(bool(zero_after)),
        stat_count=int(stat_count), nb=nb, M=M, D=D, W=W, ldw=emb.shape[2],
        decay=float(decay), laplace=int(laplace), grad_scale=float(grad_scale),
        epsilon=float(epsilon), cluster_size=cs.data_ptr(), cs_bstride=cs.stride(0),
        ema_w=ema_w.data_ptr(), embedding=emb.data_ptr(), embedding_output=emb_out.data_ptr(),
        emb_bstride=emb.stride(0), rm_f=rm_f.data_ptr(), rv_f=rv_f.data_ptr(),
        rm_g=rm_g.data_ptr() if rm_g is not None else None,
        rv_g=rv_g.data_ptr() if rv_g is not None else None, bad_init=bad_flag.data_ptr())


def gather_codewords(subset, B, codes, emb_out, D, col_offset=0, want_x=True,
                     want_codes=False, nb=None):
    """models.py:168-173 for all branches: returns (xt [n-B, nb*D] or None,
    lcodes [n-B, nb] int16 or None).  col_offset 0 = feature halves
    (x_first_order), D = grad halves (grad_first_order).  nb = the codebook's
    branch count (emb_out.shape[0]); codes may hold more columns (a strided
    c_indices view), never fewer."""
    n = subset.shape[0]
    if subset.dtype != torch.int64 or subset.dim() != 1 or subset.stride(0) != 1:
        raise ValueError("gather_codewords: subset must be a contiguous int64 [n] tensor")
    if codes.dtype != torch.int16 or codes.dim() != 2 or codes.stride(1) != 1:
        raise ValueError("gather_codewords: codes must be an int16 [N, ldc] row-major view")
    if nb is None:
        if emb_out is None:
            raise ValueError("gather_codewords: nb is needed when emb_out is None")
        nb = emb_out.shape[0]
    nb = int(nb)
    if codes.shape[1] < nb:
        raise ValueError(f"gather_codewords: codes has {codes.shape[1]} columns < {nb} branches")
    if emb_out is not None and emb_out.shape[0] < nb:
        raise ValueError(f"gather_codewords: emb_out has {emb_out.shape[0]} branches < nb={nb}")
    dev = codes.device
    xt = torch.empty(n - B, nb * D, dtype=torch.float32, device=dev) if want_x else None
    lc = torch.empty(n - B, nb, dtype=torch.int16, device=dev) if want_codes else None
    if emb_out is not None:
        n_br, M, ldw = (int(v) for v in emb_out.shape)
        if emb_out.stride(2) != 1 or emb_out.stride(1) != ldw:
            raise ValueError("gather_codewords: emb_out must be row-major per branch")
        bstride = emb_out.stride(0)
    else:
        n_br, M, ldw, bstride = nb, 1, 0, 0
    check(lib().vqgnn_gather_codewords(ptr(subset), B, n, ptr(codes), codes.stride(0),
                                       codes.shape[0], nb, D, ptr(emb_out), n_br, M, ldw,
                                       bstride, int(col_offset), ptr(xt), nb * D, ptr(lc),
                                       stream_ptr()), "gather_codewords")
    return xt, lc


def codes_wire_record(nb: int, M: int) -> int:
    """Bytes per record of the multi-GPU code exchange (include/vqgnn.h §5b)."""
    return int(lib().vqgnn_codes_wire_record(int(nb), int(M)))


def pack_codes(batch_idx, local, M, max_B, send, codes=None):
    """Records of (batch_idx, local codes) + padding into ``send`` (uint8);
    with ``codes`` the rows are also scattered into this rank's c_indices."""
    B, nb = local.shape
    check(lib().vqgnn_pack_codes(ptr(batch_idx), B, ptr(local), nb, int(M), int(max_B), ptr(send),
                                 ptr(codes), codes.stride(0) if codes is not None else 0,
                                 stream_ptr()), "pack_codes")


def scatter_wire(recv, n_records, nb, M, winner, codes, epoch):
    """All ranks' records into ``codes``; the last record of a node wins.
    winner: int64 [N] stamp table, zero-initialised once; epoch: 1, 2, ... per
    call on the same table (include/vqgnn.h §5b)."""
    if winner.dtype != torch.int64 or winner.numel() < codes.shape[0]:
        raise ValueError("scatter_wire: winner must be an int64 [N] stamp table")
    check(lib().vqgnn_scatter_wire(ptr(recv), int(n_records), int(nb), int(M), ptr(winner),
                                   int(epoch), codes.shape[0], ptr(codes), codes.stride(0),
                                   stream_ptr()), "scatter_wire")


def scatter_codes(batch_idx: torch.Tensor, local: torch.Tensor, codes: torch.Tensor) -> None:
    """codes[batch_idx[i]] = local[i] (batch_idx < 0 entries are padding)."""
    B, nb = local.shape
    check(lib().vqgnn_scatter_codes(ptr(batch_idx), B, ptr(local), nb, ptr(codes),
                                    codes.stride(0), stream_ptr()), "scatter_codes")


class TaskPlan:
    """Task plan of a CSR for vqgnn_spmm_task (include/vqgnn.h §6): per-edge
    records (column, row-end flag, weight), the tasks' first edges and rows,
    and the fix-up jobs (cut rows, empty rows); built once per batch
    adjacency, valid for any F and any leading row count.  Building it reads
    the two job counts back to the host (one sync per plan)."""

    def __init__(self, plan, records, K, nnz, n_rows, val, n_jobs, n_empty, rowptr=None,
                 n_cols=None):
        self.plan, self.records, self.K = plan, records, K
        self.nnz, self.n_rows = nnz, n_rows
        self.n_cols = n_cols          # columns of the planned CSR (None: not recorded)
        self.val_ptr = val.data_ptr() if val is not None else 0
        self.n_jobs, self.n_empty = n_jobs, n_empty
        self.rowptr = rowptr

    def with_values(self, col, val, records=None):
        """The same plan over other edge values on the same structure (GAT's
        coefficients): new records only (vqgnn_spmm_task_records, no host
        read); ``records`` may be a reused int64 [nnz] buffer."""
        if records is None:
            records = torch.empty(max(self.nnz, 1), dtype=torch.int64, device=val.device)
        check(lib().vqgnn_spmm_task_records(ptr(self.rowptr), ptr(col), ptr(val), self.n_rows,
                                            self.nnz, ptr(records), stream_ptr()),
              "spmm_task_records")
        return TaskPlan(self.plan, records, self.K, self.nnz, self.n_rows, val, self.n_jobs,
                        self.n_empty, self.rowptr, self.n_cols)

    def with_codebook_source(self, B, subset, n_nodes):
        """The plan of spmm_codebook (include/vqgnn.h §6b): a copy of the
        records whose columns j >= B name the node subset[j] (B + node id),
        so the kernel reads that node's codes instead of an x_first row."""
        if subset.dtype != torch.int64 or subset.dim() != 1 or subset.stride(0) != 1:
            raise ValueError("with_codebook_source: subset must be a contiguous int64 [n] "
                             "tensor (the kernel reads it as int64 by record column)")
        if self.n_cols is not None and subset.numel() != self.n_cols:
            raise ValueError(f"with_codebook_source: subset has {subset.numel()} nodes, the "
                             f"adjacency {self.n_cols} columns")
        if not 0 <= int(B) <= subset.numel():
            raise ValueError(f"with_codebook_source: B={B} outside [0, {subset.numel()}]")
        records = self.records.clone()
        check(lib().vqgnn_spmm_task_records_cb(ptr(records), self.nnz, int(B), ptr(subset),
                                               int(subset.numel()), int(n_nodes), stream_ptr()),
              "spmm_task_records_cb")
        p = TaskPlan(self.plan, records, self.K, self.nnz, self.n_rows, None, self.n_jobs,
                     self.n_empty, self.rowptr, self.n_cols)
        p.val_ptr = self.val_ptr
        p.cb_B = int(B)
        return p


TASK_K = 64


def spmm_task_plan(rowptr, col, val, n_rows, nnz, K=None, n_cols=None):
    L = lib()
    K = int(K or TASK_K)
    dev = rowptr.device
    m = L.vqgnn_spmm_task_size(int(nnz), K, int(n_rows))
    plan = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
    records = torch.empty(max(int(nnz), 1), dtype=torch.int64, device=dev)
    counts = torch.empty(2, dtype=torch.int32, device=dev)
    check(L.vqgnn_spmm_task_plan(ptr(rowptr), ptr(col), ptr(val), int(n_rows), int(nnz), K,
                                 ptr(plan), ptr(records), ptr(counts), stream_ptr()),
          "spmm_task_plan")
    n_jobs, n_empty = (int(v) for v in counts.tolist())
    return TaskPlan(plan, records, K, int(nnz), int(n_rows), val, n_jobs, n_empty, rowptr,
                    None if n_cols is None else int(n_cols))


def spmm(rowptr, col, val, n_rows, nnz, X, F, X2=None, B=None, out=None, plan=None):
    """out[i] = sum_e val[e] * xin[col[e]]; xin = X rows (< B), X2 rows (>= B).
    Every column index must be < the rows of xin (X rows, or B + X2 rows)."""
    require_gpu(X, "spmm")
    if rowptr.dtype != torch.int32 or (col is not None and col.dtype != torch.int32):
        raise TypeError("spmm: rowptr / col must be int32 device arrays (CSR.rowptr / CSR.col; "
                        "CSR.csr() returns int64 copies)")
    dev = X.device
    if out is None:
        out = torch.empty(n_rows, F, dtype=torch.float32, device=dev)
    L = lib()
    Bv = int(B) if X2 is not None else 0
    n_cols = Bv + X2.shape[0] if X2 is not None else X.shape[0]
    if X2 is not None and X.shape[0] < Bv:
        raise ValueError(f"spmm: X has {X.shape[0]} rows < B={Bv}")
    if plan is None:            # a one-off product: plan it here (one host read)
        plan = spmm_task_plan(rowptr, col, val, rowptr.numel() - 1, nnz)
    if isinstance(plan, TaskPlan):
        if (val.data_ptr() if val is not None else 0) != plan.val_ptr:
            raise ValueError("spmm: the task plan's records hold other values than val")
        if plan.nnz != int(nnz) or int(n_rows) > plan.n_rows:
            raise ValueError(f"spmm: task plan for nnz={plan.nnz}, rows={plan.n_rows}; called "
                             f"with nnz={nnz}, n_rows={n_rows}")
        ws = workspace(L.vqgnn_spmm_task_workspace(int(nnz), plan.K, F), dev)
        check(L.vqgnn_spmm_task(ptr(rowptr), int(n_rows), int(n_cols), int(nnz), Bv, ptr(X),
                                _ld(X), ptr(X2), _ld(X2) if X2 is not None else 0, F, ptr(out),
                                _ld(out), ptr(plan.plan), ptr(plan.records), plan.K,
                                plan.n_jobs, plan.n_empty, ptr(ws), stream_ptr()), "spmm_task")
        return out
    raise TypeError(f"spmm: plan must be a TaskPlan (CSR.plan), got {type(plan)}")


def codebook_source_ok(X, F, M, D, out=None, codes=None, n_rows=None, n_branches=None,
                       emb_out=None):
    """Whether spmm_codebook serves this layer shape (include/vqgnn.h §6b):
    the kernel's own checks (vqgnn_spmm_task_cb_supported) plus the host-side
    alignment of X, out and the codeword rows of emb_out (the entry's own
    layout check: ldw >= D, ldw and the branch stride multiples of 4, 16-byte
    aligned base).  codes / n_rows / n_branches default to shapes that pass
    their checks; out defaults to a dense [n_rows, F]."""
    if not (X.dim() == 2 and X.stride(1) == 1 and X.stride(0) % 4 == 0 and
            X.data_ptr() % 16 == 0):
        return False
    if emb_out is not None:
        if not (emb_out.dim() == 3 and emb_out.stride(2) == 1 and emb_out.stride(1) >= D and
                emb_out.stride(1) % 4 == 0 and emb_out.stride(0) % 4 == 0 and
                emb_out.data_ptr() % 16 == 0):
            return False
    if out is not None and not (out.stride(1) == 1 and out.stride(0) % 4 == 0 and
                                out.data_ptr() % 16 == 0):
        return False
    B = X.shape[0]
    nr = int(n_rows) if n_rows is not None else B
    ldo = out.stride(0) if out is not None else F
    nn, ldc = (codes.shape[0], codes.stride(0)) if codes is not None else (0, F // max(D, 1))
    nbr = int(n_branches) if n_branches is not None else F // max(D, 1)
    return bool(lib().vqgnn_spmm_task_cb_supported(int(nr), int(B), int(X.stride(0)), int(F),
                                                   int(ldo), int(nn), int(ldc), nbr, int(M),
                                                   int(D)))


def codebook_source_preferred(M):
    """Whether the codebook source is the faster aggregation for a codebook of
    M codewords: only where its LDS image fits the full-width walk (32 lanes
    per task, 128-column tiles: M <= 319, the image's zero row beside it).  At M = 1,024 the 32-column tiles
    walk every edge four times: 129 us against 103 us for gather + two-source
    SpMM on the arxiv GAT batch (profiles/r05_cb_m1024_probe.txt)."""
    return int(lib().vqgnn_spmm_task_cb_lds(int(M))) == (int(M) + 1) * 16 * 32


def _cb_prepare(rowptr, n_rows, nnz, X, F, B, codes, emb_out, D, plan_cb, out, what):
    """Checks and the argument tuple shared by the codebook-source entries."""
    require_gpu(X, what)
    if getattr(plan_cb, "cb_B", None) != int(B):
        raise ValueError(f"{what}: plan_cb must come from TaskPlan.with_codebook_source "
                         f"for B={B}")
    if plan_cb.nnz != int(nnz) or int(n_rows) > plan_cb.n_rows:
        raise ValueError(f"{what}: task plan for nnz={plan_cb.nnz}, rows={plan_cb.n_rows}; "
                         f"called with nnz={nnz}, n_rows={n_rows}")
    if codes.dtype != torch.int16 or emb_out.dtype != torch.float32:
        raise TypeError(f"{what}: codes must be int16 and emb_out float32")
    if codes.dim() != 2 or codes.stride(1) != 1:
        raise ValueError(f"{what}: codes must be an int16 [N, ldc] row-major view")
    n_br, M, ldw = (int(v) for v in emb_out.shape)
    if emb_out.stride(2) != 1 or emb_out.stride(1) != ldw:
        raise ValueError(f"{what}: emb_out must be row-major per branch")
    dev = X.device
    if out is None:
        out = torch.empty(n_rows, F, dtype=torch.float32, device=dev)
    ws = workspace(lib().vqgnn_spmm_task_workspace(int(nnz), plan_cb.K, F), dev)
    args = (ptr(rowptr), int(n_rows), int(nnz), int(B), ptr(X), _ld(X), F,
            ptr(codes), codes.stride(0), codes.shape[0], ptr(emb_out),
            emb_out.stride(1), emb_out.stride(0), n_br, M, int(D), ptr(out),
            _ld(out), ptr(plan_cb.plan), ptr(plan_cb.records), plan_cb.K,
            plan_cb.n_jobs, plan_cb.n_empty, ptr(ws))
    return out, ws, args


def _finalize_record(finalize):
    fin_args, fin_kw = getattr(finalize, "operands", finalize)
    return ema_finalize_args(*fin_args, **fin_kw)


def spmm_codebook(rowptr, n_rows, nnz, X, F, B, codes, emb_out, D, plan_cb, out=None,
                  finalize=None):
    """out = A @ [X[:B] ; x_first_order] with x_first_order's rows (the
    codeword feature halves of each out-of-batch node's codes, models.py:
    168-173) read from an LDS image of emb_out (vqgnn_spmm_task_cb); plan_cb
    from TaskPlan.with_codebook_source.  Equals spmm(..., X2=gather_codewords
    (subset, B, codes, emb_out, D)[0], B=B).

    finalize: a pending EMA finalize (VQBank.take_fused_finalize's handle, or
    vq_ema_finalize's (args, kw)) run inside the SpMM's fix-up launch
    (vqgnn_spmm_task_cb_fin): the same results as this call followed by
    vq_ema_finalize, one launch fewer.  A handle is retired (done()) only
    once the launch is queued: if this call raises, the bank keeps the
    finalize pending for finish_update()."""
    out, ws, args = _cb_prepare(rowptr, n_rows, nnz, X, F, B, codes, emb_out, D, plan_cb, out,
                                "spmm_codebook")
    L = lib()
    if finalize is None:
        check(L.vqgnn_spmm_task_cb(*args, stream_ptr()), "spmm_task_cb")
    else:
        rec = _finalize_record(finalize)
        check(L.vqgnn_spmm_task_cb_fin(*args, ctypes.byref(rec), stream_ptr()),
              "spmm_task_cb_fin")
        if hasattr(finalize, "done"):
            finalize.done()
    return out


class CodebookWalk:
    """A codebook-source aggregation whose walk is queued (or ready to be) and
    whose fix-up is not (spmm_codebook_walk -> spmm_codebook_fixup)."""

    def __init__(self, out, ws, args, stream, fork):
        self.out, self.ws, self.args, self.stream, self.fork = out, ws, args, stream, fork
        self.launched = self.fixed = False

    def launch(self):
        """Queue the walk on its stream, after the caller's stream as it was
        when the walk was created (the fork event): work queued on the
        caller's stream since then runs beside it."""
        if self.launched:
            return
        if self.fork is not None:
            self.stream.wait_event(self.fork)
        with torch.cuda.stream(self.stream):
            check(lib().vqgnn_spmm_task_cb_walk(*self.args, stream_ptr()), "spmm_task_cb_walk")
        self.launched = True


def spmm_codebook_walk(rowptr, n_rows, nnz, X, F, B, codes, emb_out, D, plan_cb, out=None,
                       stream=None, deferred=False):
    """spmm_codebook's walk alone (vqgnn_spmm_task_cb_walk, include/vqgnn.h
    §6b) -> CodebookWalk; spmm_codebook_fixup finishes it.  stream: a second
    stream to walk on, beside what the caller queues next on its own stream --
    the VQ update of the same batch (its assign writes only the batch nodes'
    codes; the walk reads X, the out-of-batch nodes' codes and emb_out).  The
    walk runs after the caller's stream as it is now (an event); out and the
    workspace are allocated on the caller's stream before that event, which
    joins the walk (fix-up) before it can free them.  deferred: create the
    walk now, queue it later with .launch() (e.g. VQBank.update's
    before_assign, so the update's BatchNorm pass is queued first and runs
    while the walk's launch crosses streams).  The rows that span tasks and
    the empty rows of out are written only by the fix-up."""
    out, ws, args = _cb_prepare(rowptr, n_rows, nnz, X, F, B, codes, emb_out, D, plan_cb, out,
                                "spmm_codebook_walk")
    cur = torch.cuda.current_stream()
    s = cur if stream is None else stream
    fork = None
    if s != cur:
        fork = torch.cuda.Event()
        fork.record(cur)
    walk = CodebookWalk(out, ws, args, s, fork)
    if not deferred:
        walk.launch()
    return walk


def spmm_codebook_fixup(walk, finalize=None):
    """The fix-up of a CodebookWalk on the current stream, after the walk (the
    current stream waits for the walk's), with the pending EMA finalize
    inside it as in spmm_codebook -> out, equal bit for bit to
    spmm_codebook's."""
    if walk.fixed:
        raise RuntimeError("spmm_codebook_fixup: this walk was fixed up already")
    walk.launch()                           # (a deferred walk nobody launched)
    cur = torch.cuda.current_stream()
    if walk.stream != cur:
        cur.wait_stream(walk.stream)
    L = lib()
    rec = None if finalize is None else _finalize_record(finalize)
    check(L.vqgnn_spmm_task_cb_fixup(*walk.args, ctypes.byref(rec) if rec is not None else None,
                                     stream_ptr()), "spmm_task_cb_fixup")
    walk.fixed = True
    if finalize is not None and hasattr(finalize, "done"):
        finalize.done()
    return walk.out


def csr_transpose(rowptr, col, val, n_rows, n_cols, nnz, want_perm=False):
    """-> (t_rowptr, t_col, t_val[, t_perm]); t_perm[k] = input edge of entry k."""
    dev = rowptr.device
    t_rowptr = torch.empty(n_cols + 1, dtype=torch.int32, device=dev)
    t_col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    t_val = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    t_perm = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev) if want_perm else None
    L = lib()
    ws = workspace(L.vqgnn_csr_transpose_workspace(n_rows, n_cols, nnz), dev)
    check(L.vqgnn_csr_transpose(ptr(rowptr), ptr(col), ptr(val), n_rows, n_cols, nnz,
                                ptr(t_rowptr), ptr(t_col), ptr(t_val), ptr(t_perm), ptr(ws),
                                stream_ptr()), "csr_transpose")
    if want_perm:
        return t_rowptr, t_col[:nnz], t_val[:nnz], t_perm[:nnz]
    return t_rowptr, t_col[:nnz], t_val[:nnz]


def csr_expand_rows(rowptr, n_rows, nnz):
    """COO row index of every CSR entry (int32 [nnz])."""
    rows = torch.empty(max(nnz, 1), dtype=torch.int32, device=rowptr.device)
    check(lib().vqgnn_csr_expand_rows(ptr(rowptr), int(n_rows), int(nnz), ptr(rows),
                                      stream_ptr()), "csr_expand_rows")
    return rows[:nnz]


# ---- GAT (include/vqgnn.h §8) ----

def gat_alpha(X, att_l, att_r, F, X2=None, B=None, ones=True):
    """-> (alpha_l, alpha_r [n], params [5] = (max_l, max_r, s, ds/dmax_l,
    ds/dmax_r), alpha_l / s, alpha_r / s [n]).  The scaled scalars are what
    every per-edge consumer reads (convs.py:209-211 divides once per node)."""
    require_gpu(X, "gat_alpha")
    dev = X.device
    Bv = int(B) if X2 is not None else X.shape[0]
    n = Bv + (X2.shape[0] if X2 is not None else 0)
    al = torch.empty(n, dtype=torch.float32, device=dev)
    ar = torch.empty(n, dtype=torch.float32, device=dev)
    als = torch.empty(n, dtype=torch.float32, device=dev)
    ars = torch.empty(n, dtype=torch.float32, device=dev)
    params = torch.empty(5, dtype=torch.float32, device=dev)
    L = lib()
    ws = workspace(L.vqgnn_gat_alpha_workspace(n), dev)
    check(L.vqgnn_gat_alpha(ptr(X), _ld(X), ptr(X2), _ld(X2) if X2 is not None else 0, Bv, n,
                            int(F), int(bool(ones)), ptr(att_l), ptr(att_r), ptr(al), ptr(ar),
                            ptr(als), ptr(ars), ptr(params), ptr(ws), stream_ptr()), "gat_alpha")
    return al, ar, params, als, ars


def gat_coef(rowptr, col, val, n_rows, nnz, als, ars, negative_slope=0.2):
    """als, ars: alpha / s per node (gat_alpha) -> (coef [nnz], den [n_rows])."""
    dev = als.device
    coef = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    den = torch.empty(n_rows, dtype=torch.float32, device=dev)
    check(lib().vqgnn_gat_coef(ptr(rowptr), ptr(col), ptr(val), int(n_rows), int(nnz), ptr(als),
                               ptr(ars), float(negative_slope), ptr(coef), ptr(den),
                               stream_ptr()), "gat_coef")
    return coef[:nnz], den


def gat_spmm(rowptr, col, val, n_rows, nnz, X, F, als, ars, plan, erow, X2=None,
             B=None, norm_B=0, negative_slope=0.2, want_den=False, want_coef=False, out=None):
    """Fused GAT aggregation (include/vqgnn.h §8b) on a task plan built from
    this CSR's values (als, ars: alpha / s per node from gat_alpha):
    coefficients in the kernel, the ones column as the
    per-row sum, rows < norm_B normalised.  -> (out [n_rows, F], den or None,
    coef [nnz] (CSR order) or None)."""
    require_gpu(X, "gat_spmm")
    if not isinstance(plan, TaskPlan):
        raise ValueError("gat_spmm: needs the CSR's task plan")
    if (val.data_ptr() if val is not None else 0) != plan.val_ptr:
        raise ValueError("gat_spmm: the task plan's records hold other values than val")
    dev = X.device
    L = lib()
    if out is None:
        out = torch.empty(n_rows, F, dtype=torch.float32, device=dev)
    Bv = int(B) if X2 is not None else 0
    n_cols = Bv + X2.shape[0] if X2 is not None else X.shape[0]
    den = torch.empty(max(int(n_rows), 1), dtype=torch.float32, device=dev) if want_den else None
    coef = torch.empty(max(int(nnz), 1), dtype=torch.float32, device=dev) if want_coef else None
    ws = workspace(L.vqgnn_spmm_task_workspace(int(nnz), plan.K, F), dev)
    check(L.vqgnn_gat_spmm_task(ptr(rowptr), int(n_rows), int(n_cols), int(nnz), Bv, ptr(X),
                                _ld(X), ptr(X2), _ld(X2) if X2 is not None else 0, F, ptr(out),
                                _ld(out), ptr(plan.plan), ptr(plan.records), plan.K,
                                plan.n_jobs, plan.n_empty, ptr(erow), ptr(als), ptr(ars),
                                float(negative_slope), int(norm_B), ptr(den),
                                ptr(coef), ptr(ws), stream_ptr()), "gat_spmm")
    return out, (den[:n_rows] if den is not None else None), \
        (coef[:nnz] if coef is not None else None)


def gat_normalize(out, B, F, den, eps=1e-16):
    check(lib().vqgnn_gat_normalize(ptr(out), _ld(out), int(B), int(F), ptr(den), float(eps),
                                    stream_ptr()), "gat_normalize")


def gat_edge_grad(rows, col, coef, nnz, X, F, dy, dden, als, ars, params, X2=None, B=None,
                  negative_slope=0.2):
    """-> (dalpha_l [n], dalpha_r [n], ds_row [n]) for the coefficient chain
    (als, ars: alpha / s per node; params[2] = s)."""
    dev = X.device
    n = als.shape[0]
    dal = torch.zeros(n, dtype=torch.float32, device=dev)
    dar = torch.zeros(n, dtype=torch.float32, device=dev)
    dsr = torch.zeros(n, dtype=torch.float32, device=dev)
    Bv = int(B) if X2 is not None else X.shape[0]
    check(lib().vqgnn_gat_edge_grad(ptr(rows), ptr(col), ptr(coef), int(nnz), ptr(X), _ld(X),
                                    ptr(X2), _ld(X2) if X2 is not None else 0, Bv, int(F),
                                    ptr(dy), _ld(dy), ptr(dden), ptr(als), ptr(ars), ptr(params),
                                    float(negative_slope), ptr(dal), ptr(dar), ptr(dsr),
                                    stream_ptr()), "gat_edge_grad")
    return dal, dar, dsr


def gat_att_grad(X, F, dal, dar, X2=None, B=None, ones=True):
    """(x_in^T dal, x_in^T dar) [F + ones] with x_in = [X ; X2 ; 1] (§8b)."""
    dev = X.device
    n = dal.shape[0]
    C = F + int(bool(ones))
    Bv = int(B) if X2 is not None else X.shape[0]
    gl = torch.empty(C, dtype=torch.float32, device=dev)
    gr = torch.empty(C, dtype=torch.float32, device=dev)
    L = lib()
    ws = workspace(L.vqgnn_gat_att_grad_workspace(n, int(F), int(bool(ones))), dev)
    check(L.vqgnn_gat_att_grad(ptr(X), _ld(X), ptr(X2), _ld(X2) if X2 is not None else 0, Bv, n,
                               int(F), int(bool(ones)), ptr(dal), ptr(dar), ptr(gl), ptr(gr),
                               ptr(ws), stream_ptr()), "gat_att_grad")
    return gl, gr


# ---- mini-batch construction (include/vqgnn.h §9) ----

KHOP_ORDER_CSR, KHOP_ORDER_REF = 0, 1
KHOP_OUT_OF_RANGE = 2


def _khop_status(status: int) -> None:
    if status & KHOP_OUT_OF_RANGE:
        # node_mask[subsets[-1]] = True (dataloader.py:115) raises IndexError
        raise IndexError("k_hop_subgraph: node index out of range")


def random_walk(rowptr, col, N, start, walk_length, seed):
    """torch_cluster random_walk (p = q = 1) of every start node on the
    device graph (rowptr int64 [N+1], col int32): [n_start, walk_length + 1]
    int64 (include/vqgnn.h §9b; the step uniforms come from ``seed``)."""
    require_gpu(rowptr, "random_walk")
    dev = rowptr.device
    start = start.to(device=dev, dtype=torch.int64).contiguous()
    n = int(start.numel())
    out = torch.empty(n, int(walk_length) + 1, dtype=torch.int64, device=dev)
    status = torch.empty(1, dtype=torch.int64, device=dev)
    check(lib().vqgnn_random_walk(ptr(rowptr), ptr(col), int(N), ptr(start), n, int(walk_length),
                                  int(seed) & ((1 << 64) - 1), ptr(out), ptr(status),
                                  stream_ptr()), "random_walk")
    if int(status.item()) != 0:
        raise IndexError("random_walk: start node outside [0, N)")
    return out


def khop_subgraph(rowptr, col, val, N, node_idx, num_hops=1, train_flag=True,
                  order=KHOP_ORDER_CSR):
    """_k_hop_subgraph (dataloader.py:98-148) of node_idx on the full graph
    (rowptr int64 [N+1], col int32, val fp32, all on the device).

    Returns dict(subset int64 [n], node_map int32 [N], rowptr int32 [rows+1],
    col int32 [nnz], val fp32 [nnz], row int32 [nnz] (ORDER_REF only), n, nnz,
    rows).  One device->host read of the sizes (the outputs are data-sized)."""
    require_gpu(rowptr, "khop_subgraph")
    dev = rowptr.device
    node_idx = node_idx.to(device=dev, dtype=torch.int64).contiguous()
    B = int(node_idx.numel())
    N = int(N)
    L = lib()
    node_map = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
    subset = torch.empty(max(N, 1), dtype=torch.int64, device=dev)
    rows = torch.empty(max(N, 1), dtype=torch.int64, device=dev) if order == KHOP_ORDER_REF \
        else None
    out_rowptr = torch.empty(N + 1, dtype=torch.int32, device=dev)
    sizes = torch.zeros(4, dtype=torch.int64, device=dev)
    ws = workspace(L.vqgnn_khop_workspace(N), dev)
    check(L.vqgnn_khop_subset(ptr(rowptr), ptr(col), N, ptr(node_idx), B, int(num_hops),
                              int(bool(train_flag)), int(order), ptr(node_map), ptr(subset),
                              ptr(rows), ptr(out_rowptr), ptr(sizes), ptr(ws), stream_ptr()),
          "khop_subset")
    n, nnz, nrows, status = (int(v) for v in sizes.cpu())
    _khop_status(status)
    out_col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    out_val = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    out_row = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev) \
        if order == KHOP_ORDER_REF else None
    emit = rows if order == KHOP_ORDER_REF else subset
    ws2 = workspace(L.vqgnn_khop_edges_workspace(nrows, nnz), dev)
    check(L.vqgnn_khop_edges(ptr(rowptr), ptr(col), ptr(val), N, ptr(node_map), ptr(emit), nrows,
                             n, B, int(bool(train_flag)), int(order), ptr(out_rowptr), nnz,
                             ptr(out_col), ptr(out_val), ptr(out_row), ptr(ws2), stream_ptr()),
          "khop_edges")
    return dict(subset=subset[:n], node_map=node_map[:N], rowptr=out_rowptr[:nrows + 1],
                col=out_col[:nnz], val=out_val[:nnz],
                row=out_row[:nnz] if out_row is not None else None,
                rows=rows[:nrows] if rows is not None else None, n=n, nnz=nnz)


def coo_to_csr(row, col, val, n_rows, n_cols):
    """SparseTensor(row=, col=, value=, sparse_sizes=(n_rows, n_cols)) ->
    (rowptr int32, col int32, val fp32) sorted by (row, col), stable."""
    require_gpu(row, "coo_to_csr")
    dev = row.device
    row = row.to(torch.int64).contiguous()
    col = col.to(device=dev, dtype=torch.int64).contiguous()
    nnz = int(row.numel())
    if val is None:
        val = torch.ones(nnz, dtype=torch.float32, device=dev)
    val = val.to(device=dev, dtype=torch.float32).contiguous()
    L = lib()
    out_rowptr = torch.empty(int(n_rows) + 1, dtype=torch.int32, device=dev)
    out_col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    out_val = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = workspace(L.vqgnn_coo_to_csr_workspace(nnz, int(n_rows), int(n_cols)), dev)
    check(L.vqgnn_coo_to_csr(ptr(row), ptr(col), ptr(val), nnz, int(n_rows), int(n_cols),
                             ptr(out_rowptr), ptr(out_col), ptr(out_val), ptr(status), ptr(ws),
                             stream_ptr()), "coo_to_csr")
    if int(status.item()) & KHOP_OUT_OF_RANGE:
        raise IndexError("coo_to_csr: index out of range")
    return out_rowptr, out_col[:nnz], out_val[:nnz]


# ---- full-graph preprocessing (include/vqgnn.h §10) ----

CONV_TYPES = {"GCN": 0, "SAGE": 1, "GAT": 2}


def norm_adj(rowptr, col, val, N, conv_type):
    """-> (rowptr int64 [N+1], col int32, val fp32) of the normalised graph."""
    require_gpu(rowptr, "norm_adj")
    if conv_type not in CONV_TYPES:
        raise ValueError('GNN conv type not supported')           # misc.py:34
    dev = rowptr.device
    nnz = int(col.numel())
    cap = nnz + (N if conv_type != "SAGE" else 0)
    out_rowptr = torch.empty(N + 1, dtype=torch.int64, device=dev)
    out_col = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    out_val = torch.empty(max(cap, 1), dtype=torch.float32, device=dev)
    L = lib()
    ws = workspace(L.vqgnn_norm_adj_workspace(N), dev)
    check(L.vqgnn_norm_adj(ptr(rowptr), ptr(col), ptr(val), int(N), CONV_TYPES[conv_type],
                           ptr(out_rowptr), ptr(out_col), ptr(out_val), ptr(ws), stream_ptr()),
          "norm_adj")
    n = int(out_rowptr[N].item()) if N else 0
    return out_rowptr, out_col[:n], out_val[:n]


def to_symmetric(rowptr, col, val, N):
    """SparseTensor.to_symmetric(): A and A^T merged, repeats summed (val None:
    pattern with unit values).  -> (rowptr int64, col int32, val fp32)."""
    require_gpu(rowptr, "to_symmetric")
    dev = rowptr.device
    nnz = int(col.numel())
    out_rowptr = torch.empty(N + 1, dtype=torch.int64, device=dev)
    out_col = torch.empty(max(2 * nnz, 1), dtype=torch.int32, device=dev)
    out_val = torch.empty(max(2 * nnz, 1), dtype=torch.float32, device=dev)
    out_nnz = torch.zeros(1, dtype=torch.int64, device=dev)
    L = lib()
    ws = workspace(L.vqgnn_to_symmetric_workspace(N, nnz), dev)
    check(L.vqgnn_to_symmetric(ptr(rowptr), ptr(col), ptr(val), int(N), nnz, ptr(out_rowptr),
                               ptr(out_col), ptr(out_val), ptr(out_nnz), ptr(ws), stream_ptr()),
          "to_symmetric")
    n = int(out_nnz.item())
    return out_rowptr, out_col[:n], out_val[:n]


def csr_permute(rowptr, col, val, N, perm):
    """SparseTensor.permute(perm): node i of the result = node perm[i]."""
    require_gpu(rowptr, "csr_permute")
    dev = rowptr.device
    nnz = int(col.numel())
    perm = perm.to(device=dev, dtype=torch.int64).contiguous()
    if perm.numel() != N:
        raise ValueError("perm must have N entries")
    out_rowptr = torch.empty(N + 1, dtype=torch.int64, device=dev)
    out_col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    out_val = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int64, device=dev)
    L = lib()
    ws = workspace(L.vqgnn_csr_permute_workspace(N, nnz), dev)
    check(L.vqgnn_csr_permute(ptr(rowptr), ptr(col), ptr(val), int(N), nnz, ptr(perm),
                              ptr(out_rowptr), ptr(out_col), ptr(out_val), ptr(status), ptr(ws),
                              stream_ptr()), "csr_permute")
    if int(status.item()):
        raise IndexError("permute: index out of range")
    return out_rowptr, out_col[:nnz], out_val[:nnz]


def partition(rowptr, col, N, num_parts):
    """METIS substitute: -> (perm int64 [N], ptr int64 [num_parts+1], steps)."""
    require_gpu(rowptr, "partition")
    import ctypes
    dev = rowptr.device
    perm = torch.empty(max(N, 1), dtype=torch.int64, device=dev)
    ptr_ = torch.empty(num_parts + 1, dtype=torch.int64, device=dev)
    steps = ctypes.c_int32(0)
    L = lib()
    ws = workspace(L.vqgnn_partition_workspace(N), dev)
    check(L.vqgnn_partition(ptr(rowptr), ptr(col), int(N), int(num_parts), ptr(perm), ptr(ptr_),
                            ctypes.addressof(steps), ptr(ws), stream_ptr()), "partition")
    return perm[:N], ptr_, int(steps.value)


_CONV = {"GCN": 0, "SAGE": 1, "GAT": 2}


def mapper(bn, c, num_B, num_M, gnn_type="GCN", nb_val=None, bb=None, batch_idx=None,
           deg_inv=None):
    """vqgnn_mapper (include/vqgnn.h §11): the v1 compressed (B+M)^2 adjacency
    as (rowptr int64 [B+M+1], col int32, val fp32) device tensors.
    bn = (row, col, val) of A_BN; c = int16 codes of one branch ([N], any
    stride); bb = (row, col, val) of A_BB in local ids or None."""
    require_gpu(bn[2], "mapper")
    dev = bn[2].device
    L = lib()
    i32 = lambda t: t.to(device=dev, dtype=torch.int32).contiguous()
    f32 = lambda t: t.to(device=dev, dtype=torch.float32).contiguous()
    r, j, v = i32(bn[0]), i32(bn[1]), f32(bn[2])
    E = int(v.numel())
    nbv = f32(nb_val) if nb_val is not None else None
    if bb is not None:
        br, bs, bv = i32(bb[0]), i32(bb[1]), f32(bb[2])
        E2 = int(bv.numel())
        bi = batch_idx.to(device=dev, dtype=torch.int64).contiguous()
    else:
        br = bs = bv = bi = None
        E2 = 0
    if c.dtype != torch.int16:
        raise ValueError("mapper: codes must be int16 (c_indices)")
    ldc = c.stride(0) if c.dim() == 1 else c.stride(0)
    conv = _CONV[gnn_type] if gnn_type in _CONV else _CONV["GAT"]
    di = f32(deg_inv) if deg_inv is not None else None
    B, M = int(num_B), int(num_M)
    cap = L.vqgnn_mapper_capacity(E, E2, B, int(nbv is not None), int(bb is not None), conv)
    rowptr = torch.empty(B + M + 1, dtype=torch.int64, device=dev)
    col = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    val = torch.empty(max(cap, 1), dtype=torch.float32, device=dev)
    nnz = torch.zeros(1, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = workspace(L.vqgnn_mapper_workspace(E, E2, B, int(nbv is not None), int(bb is not None)),
                   dev)
    check(L.vqgnn_mapper(ptr(r), ptr(j), ptr(v), E, ptr(nbv), ptr(br), ptr(bs), ptr(bv), E2,
                         ptr(bi), B, ptr(c), ldc, M, ptr(di), conv, ptr(rowptr), ptr(col),
                         ptr(val), ptr(nnz), ptr(status), ptr(ws), stream_ptr()), "mapper")
    n = int(nnz.item())
    if int(status.item()) != 0:
        raise ValueError("mapper: a codeword index is outside [0, num_M)")
    return rowptr, col[:n], val[:n]
