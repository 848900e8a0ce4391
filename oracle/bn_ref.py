"""Oracle: ATen's CPU BatchNorm1d arithmetic (train and eval), restated in
numpy.  TEST INFRASTRUCTURE ONLY — imported by tests/ and smoke(), never by
the product path.

The reference normalises every VQ input with ``nn.BatchNorm1d(D,
affine=False)`` (vq_gnn_v2/vq.py:162, :223) and initialises the running
stats with ``torch.mean`` / ``torch.var`` (vq.py:216-221).  ATen (torch
2.10, aten/src/ATen/native/Normalization.cpp ``batch_norm_cpu`` /
``batch_norm_cpu_update_stats_template``, native/cpu/batch_norm_kernel.cpp,
native/cpu/SumKernel.cpp) takes one of two arithmetic paths, chosen by the
layout of the [B, D] input:

* **strided** (the input is not contiguous — what the reference's layers
  pass: ``x[:, D*i:D*(i+1)]`` of a [B, F] activation, models.py:162-165):
  mean = ``at::mean`` = float cascade sum / B (``cascade_sum``); variance
  sum = serial double sum of (x - mean)^2; output ((x - mean) * invstd);
  running stats in double.  Independent of the thread count.
* **contiguous** (a standalone [B, D] tensor, e.g. the golden fixtures):
  the channels-last collect-stats kernel: per-thread fp32 row chunks
  (``at::parallel_for`` over B rows, grain 1, T threads), folded in double;
  variance chunks are fp32 fma chains; output fma(x, invstd, -mean*invstd);
  running stats in float.  Depends on T = torch.get_num_threads().

Every function was checked bit for bit against ATen in the build container
(tests/test_bn_oracle.py re-checks it on every CPU test run).
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
f64 = np.float64


def _ceil_log2(x: int) -> int:
    return (int(x) - 1).bit_length() if x > 1 else 0


def cascade_level_power(size: int) -> int:
    """SumKernel.cpp multi_row_sum: level_power = max(4, CeilLog2(size) / 4)."""
    return max(4, _ceil_log2(size) // 4)


def _seq_sum32(a: np.ndarray, axis=0) -> np.ndarray:
    """Sequential fp32 sum from 0 along ``axis`` (np.add.accumulate is
    sequential; np.sum would be pairwise)."""
    a = np.asarray(a, dtype=f32)
    if a.shape[axis] == 0:
        return np.zeros(np.delete(a.shape, axis), f32)
    return np.add.accumulate(a, axis=axis, dtype=f32).take(-1, axis=axis)


def cascade_sum(X: np.ndarray) -> np.ndarray:
    """ATen's float cascade sum over rows of X [B, C] (SumKernel.cpp
    ``multi_row_sum`` with num_levels = 4), per column.

    acc[0] sums ``step`` rows; after each block acc[1] += acc[0]; every
    ``step`` blocks acc[2] += acc[1]; every ``step**2`` blocks acc[3] +=
    acc[2].  The tail rows go to acc[0], then acc[0] += acc[1], acc[2],
    acc[3] in that order."""
    X = np.asarray(X, dtype=f32)
    B, C = X.shape
    lp = cascade_level_power(B)
    step = 1 << lp
    nblk = B // step
    main = X[: nblk * step].reshape(nblk, step, C)
    blk = _seq_sum32(main, axis=1) if nblk else np.zeros((0, C), f32)   # level 0
    nsb = nblk // step
    sb = _seq_sum32(blk[: nsb * step].reshape(nsb, step, C), axis=1) if nsb else \
        np.zeros((0, C), f32)                                           # level 1
    ngr = nsb // step
    gr = _seq_sum32(sb[: ngr * step].reshape(ngr, step, C), axis=1) if ngr else \
        np.zeros((0, C), f32)                                           # level 2
    acc3 = _seq_sum32(gr, axis=0) if ngr else np.zeros(C, f32)
    acc2 = _seq_sum32(sb[ngr * step:], axis=0)
    acc1 = _seq_sum32(blk[nsb * step:], axis=0)
    tail = _seq_sum32(X[nblk * step:], axis=0)
    return ((tail + acc1).astype(f32) + acc2).astype(f32) + acc3


def torch_mean(X: np.ndarray) -> np.ndarray:
    """torch.mean(X, dim=0) for float X [B, C]: cascade sum / B in float."""
    return (cascade_sum(X) / f32(X.shape[0])).astype(f32)


def torch_var(X: np.ndarray) -> np.ndarray:
    """torch.var(X, dim=0) (unbiased): Welford in double, rounded to float;
    restated as the two-pass double variance (equal after the rounding)."""
    Xd = np.asarray(X, dtype=f64)
    m = Xd.mean(axis=0)
    return (((Xd - m) ** 2).sum(axis=0) / (X.shape[0] - 1)).astype(f32)


def _chunks(B: int, T: int):
    """at::parallel_for(0, B, 1, f) with T OpenMP threads: thread t gets
    [t*c, min(B, (t+1)*c)), c = ceil(B / min(T, B))."""
    nt = min(T, B)
    c = -(-B // nt)
    return [(t * c, min(B, (t + 1) * c)) for t in range(nt) if t * c < B]


def _fma32(a, b, c):
    return (np.asarray(a, f64) * np.asarray(b, f64) + np.asarray(c, f64)).astype(f32)


def train_stats_contig(X: np.ndarray, T: int):
    """batch_norm_cpu_collect_stats_channels_last_impl: -> (mean f32,
    var_sum f32).  Per-thread fp32 buffers (vec::map2 adds, vec::map3
    y + (x-mean)^2 compiled to an fma), folded over threads in double."""
    X = np.asarray(X, dtype=f32)
    B, C = X.shape
    ch = _chunks(B, T)
    s = np.zeros(C, f64)
    for a, b in ch:
        s += _seq_sum32(X[a:b], axis=0)
    mean = (s / B).astype(f32)
    v = np.zeros(C, f64)
    for a, b in ch:
        acc = np.zeros(C, f32)
        for i in range(a, b):
            d = (X[i] - mean).astype(f32)
            acc = _fma32(d, d, acc)
        v += acc
    return mean, v.astype(f32)


def bn_train(X: np.ndarray, rm: np.ndarray, rv: np.ndarray, momentum: float, eps: float,
             contiguous: bool, threads: int = 1):
    """BatchNorm1d(affine=False) train-mode forward -> (out, rm', rv',
    mean, invstd, shift, alpha, beta) with out = fma(x - shift, alpha, beta)."""
    X = np.asarray(X, dtype=f32)
    B = X.shape[0]
    rm = np.asarray(rm, f32)
    rv = np.asarray(rv, f32)
    if contiguous:
        mean, vs = train_stats_contig(X, threads)
        invstd = (1.0 / np.sqrt((vs / f32(B)).astype(f32).astype(f64) + eps)).astype(f32)
        momf = f32(momentum)
        rm2 = (momf * mean + (f32(1) - momf) * rm).astype(f32)
        vu = (vs / f32(B - 1)).astype(f32).astype(f64)
        rv2 = (f64(momf) * vu + ((f32(1) - momf) * rv).astype(f32).astype(f64)).astype(f32)
        shift = np.zeros_like(mean)
        alpha = invstd
        beta = (-(mean * invstd)).astype(f32)
        out = _fma32(X, alpha, beta)
    else:
        mean = torch_mean(X)
        md = mean.astype(f64)
        vs = ((X.astype(f64) - md) ** 2).sum(axis=0)
        invstd = (1.0 / np.sqrt(vs / B + eps)).astype(f32)
        rm2 = (momentum * md + (1 - momentum) * rm.astype(f64)).astype(f32)
        rv2 = (momentum * (vs / (B - 1)) + (1 - momentum) * rv.astype(f64)).astype(f32)
        shift, alpha, beta = mean, invstd, np.zeros_like(mean)
        out = ((X - mean).astype(f32) * invstd).astype(f32)
    return out, rm2, rv2, mean, invstd, shift, alpha, beta


def bn_eval(X: np.ndarray, rm: np.ndarray, rv: np.ndarray, eps: float, contiguous: bool):
    """BatchNorm1d eval-mode forward -> (out, shift, alpha, beta)."""
    X = np.asarray(X, dtype=f32)
    rm = np.asarray(rm, f32)
    rv = np.asarray(rv, f32)
    invstd = (f32(1) / np.sqrt((rv + f32(eps)).astype(f32))).astype(f32)
    if contiguous:
        beta = (-(rm * invstd)).astype(f32)
        return _fma32(X, invstd, beta), np.zeros_like(rm), invstd, beta
    return ((X - rm).astype(f32) * invstd).astype(f32), rm, invstd, np.zeros_like(rm)
