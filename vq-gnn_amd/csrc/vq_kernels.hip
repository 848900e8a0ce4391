// Product-quantised VQ kernels for gfx950 (MI355X): BatchNorm statistics,
// nearest-codeword assignment on f32 MFMA, EMA sufficient statistics and the
// EMA codebook finalize.  Reference: vq_gnn_v2/vq.py (VectorQuantizerEMA).
//
// Numerics (checked against ATen CPU in this container):
//  * BatchNorm1d(train) output = fma(x, invstd, -(mean*invstd))     (ATen
//    batch_norm_cpu_collect_linear_and_constant_terms + Vectorized fmadd)
//  * torch.sum(x**2, dim=1) over W <= 8 columns = sequential left-to-right add
//  * MKL sgemm with K = W <= 8 = sequential fma chain over k — exactly the
//    k-ordered fma chain of v_mfma_f32_16x16x4_f32 (cdna_hip_programming §3)
//  * d = (|x|^2 + |e|^2) - 2 x.e  ==  fma(-2, x.e, |x|^2 + |e|^2)
// so for identical normalisation coefficients the codeword index is bit-exact.
// The library is compiled with -ffp-contract=off; every fma is explicit.

#include "common.h"
#include "ema_finalize.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <vector>
#include <atomic>

#include <cfloat>
#include <cstdlib>
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>

namespace vqgnn {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// 1. BatchNorm column statistics (fp64 sums)          vq.py:162, vq.py:223
//    Work item = (row, float4 column chunk); X chunks then G chunks.  Each
//    thread accumulates 8 doubles (sum, sum of squares of 4 columns) over its
//    rows; the row phases of a workgroup are folded in LDS (fixed order), then
//    a second kernel folds the chunk partials (fixed order): deterministic.
// ---------------------------------------------------------------------------
constexpr int kStatsThreads = 256;
constexpr int kStatsMaxChunks = 512;

static int stats_chunks(int B, int C4) {
  const int rows_per_iter = C4 >= kStatsThreads ? 1 : kStatsThreads / C4;
  int c = (B + rows_per_iter * 8 - 1) / (rows_per_iter * 8);
  return c < 1 ? 1 : (c > kStatsMaxChunks ? kStatsMaxChunks : c);
}

__global__ void __launch_bounds__(kStatsThreads)
bn_stats_partial_kernel(const float* __restrict__ X, int64_t ldx,
                        const float* __restrict__ G, int64_t ldg,
                        int B, int F4, int C4, int rows_per_chunk,
                        double* __restrict__ part) {
  __shared__ double red[kStatsThreads][9];  // 8 sums (+1 pad vs bank conflicts)
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(B, r0 + rows_per_chunk);
  const int C = C4 * 4;
  double* out = part + (int64_t)blockIdx.x * 2 * C;
  const float4* X4 = reinterpret_cast<const float4*>(X);
  const float4* G4 = reinterpret_cast<const float4*>(G);
  const int64_t ldx4 = ldx / 4, ldg4 = ldg / 4;
  const int phases = C4 >= kStatsThreads ? 1 : kStatsThreads / C4;
  for (int cbase = 0; cbase < C4; cbase += kStatsThreads) {
    const int c4 = cbase + (C4 >= kStatsThreads ? t : t % C4);
    const int ph = C4 >= kStatsThreads ? 0 : t / C4;
    double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
    if (ph < phases && c4 < C4) {
      const float4* base = c4 < F4 ? X4 + c4 : G4 + (c4 - F4);
      const int64_t ld = c4 < F4 ? ldx4 : ldg4;
      int r = r0 + ph;
      for (; r + phases < r1; r += 2 * phases) {
        const float4 a = base[(int64_t)r * ld];
        const float4 b = base[(int64_t)(r + phases) * ld];
        const double av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s[k] += av[k];
          q[k] = fma(av[k], av[k], q[k]);
          s[k] += bv[k];
          q[k] = fma(bv[k], bv[k], q[k]);
        }
      }
      if (r < r1) {
        const float4 a = base[(int64_t)r * ld];
        const double av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s[k] += av[k];
          q[k] = fma(av[k], av[k], q[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[t][k] = s[k];
      red[t][4 + k] = q[k];
    }
    __syncthreads();
    if (ph == 0 && c4 < C4) {
      double a[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] = red[t][k];
      for (int p = 1; p < phases; ++p) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += red[p * C4 + t][k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        out[c4 * 4 + k] = a[k];
        out[C + c4 * 4 + k] = a[4 + k];
      }
    }
    __syncthreads();
  }
}

// Scalar variant for column sets that are not float4-aligned (e.g. D = 2 on
// one branch): thread t -> column t % C, row phase t / C.
__global__ void __launch_bounds__(kStatsThreads)
bn_stats_partial_scalar_kernel(const float* __restrict__ X, int64_t ldx,
                               const float* __restrict__ G, int64_t ldg, int B, int F, int C,
                               int rows_per_chunk, double* __restrict__ part) {
  __shared__ double red[2][kStatsThreads];
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(B, r0 + rows_per_chunk);
  double* out = part + (int64_t)blockIdx.x * 2 * C;
  for (int cbase = 0; cbase < C; cbase += kStatsThreads) {
    const int cols = min(C - cbase, kStatsThreads);
    const int phases = kStatsThreads / cols;
    const int c = cbase + t % cols, ph = t / cols;
    double sm = 0.0, sq = 0.0;
    if (ph < phases) {
      const float* base = (c < F) ? (X + c) : (G + (c - F));
      const int64_t ld = (c < F) ? ldx : ldg;
      for (int r = r0 + ph; r < r1; r += phases) {
        const double v = (double)base[(int64_t)r * ld];
        sm += v;
        sq = fma(v, v, sq);
      }
    }
    red[0][t] = sm;
    red[1][t] = sq;
    __syncthreads();
    if (t < cols) {
      double a = 0.0, b = 0.0;
      for (int p = 0; p < phases; ++p) {
        a += red[0][p * cols + t];
        b += red[1][p * cols + t];
      }
      out[cbase + t] = a;
      out[C + cbase + t] = b;
    }
    __syncthreads();
  }
}

// Fold chunk partials -> sums[4][F]: one wave per value column (sum or sum
// of squares of one data column); lanes stride the chunks, then a fixed
// butterfly across the wave (deterministic).
constexpr int kReduceWaves = 4;
// Without gradients (C == F) the g half of sums is written as zeros; tail
// (optional): tail[0] = count, tail[1] = 0 (the multi-GPU row count and
// over-capacity flag that travel with the sums, vqgnn_bn_stats_count).
__global__ void __launch_bounds__(kReduceWaves * 64)
bn_stats_reduce_kernel(const double* __restrict__ part, int chunks, int F, int C,
                       double* __restrict__ sums, double* __restrict__ tail, double count) {
  const int lane = threadIdx.x & 63;
  const int v = blockIdx.x * kReduceWaves + (threadIdx.x >> 6);   // value column in [0, 2C)
  if (C == F && blockIdx.x == 0) {
    for (int i = threadIdx.x; i < 2 * F; i += blockDim.x) sums[2 * F + i] = 0.0;
  }
  if (tail && blockIdx.x == 0 && threadIdx.x < 2) tail[threadIdx.x] = threadIdx.x == 0 ? count : 0.0;
  if (v >= 2 * C) return;
  double a = 0.0;
  for (int p = lane; p < chunks; p += 64) a += part[(int64_t)p * 2 * C + v];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
  if (lane == 0) {
    const bool sq = v >= C;
    const int c = sq ? v - C : v;
    if (c < F) sums[(sq ? F : 0) + c] = a;
    else sums[(sq ? 3 * F : 2 * F) + (c - F)] = a;
  }
}

// ---------------------------------------------------------------------------
// 2. BatchNorm finalize
//
// Coefficients: coef[6][F] = alpha_f, beta_f, alpha_g, beta_g, shift_f,
// shift_g; every consumer normalises as fma(x - shift, alpha, beta)
// (bn_apply), which is each ATen path's exact expression:
//   strided input (the reference layers' x[:, D*i:D*(i+1)] slices):
//       ((x - mean) * invstd) * 1 + 0          -> shift = mean, beta = 0
//   contiguous input / fp64 sums:
//       fma(x, invstd, -(mean * invstd))       -> shift = 0
// Arithmetic per column (include/vqgnn.h VQGNN_BN_*; oracle/bn_ref.py):
//   FP64     mean and variance from fp64 sums (deterministic and independent
//            of the number of ranks: the multi-GPU path all-reduces them)
//   STRIDED  batch_norm_cpu_update_stats_template, non-contiguous branch:
//            mean = float cascade sum / B (at::mean), var_sum = sum (x-mean)^2
//            in double, invstd = 1/sqrt(var_sum/B + eps) in double, running
//            stats in double
//   CONTIG   batch_norm_cpu_collect_stats_channels_last_impl: fp32 per-thread
//            row chunks folded in double, var_sum stored as float, running
//            stats in float (momentum_ is float)
// Eval (every arithmetic): invstd = 1/sqrtf(rv + (float)eps) in float.
// Init (update()'s first call, vq.py:216-221): rm = torch.mean (cascade sum
// / B), rv = torch.var (unbiased, double then float).
// ---------------------------------------------------------------------------
enum : int { kBnFp64 = 0, kBnStrided = 1, kBnContig = 2 };

struct BnCol {            // batch statistics of one column
  float mean;             // the arithmetic's batch mean
  double var_sum;         // sum (x - mean)^2 (FP64 / STRIDED: double; CONTIG: float value)
  float tmean;            // torch.mean (init, logging)
  double var_u;           // unbiased variance about the exact mean (torch.var)
};

__device__ __forceinline__ void bn_column(const BnCol& st, bool have, int64_t n, int mode,
                                          int arith, double mom, double eps, double eps_std,
                                          float* rm, float* rv, float* alpha, float* beta,
                                          float* shift, float* mean_out, float* std_out) {
  const bool train = (mode == 1 || mode == 2);
  const bool init = mode >= 2;
  const double nd = (double)n;
  if (have) {
    if (mean_out) *mean_out = st.tmean;
    if (std_out) *std_out = sqrtf(__fadd_rn((float)st.var_u, (float)eps_std));
  }
  if (init) {  // vq.py:216-221: running stats <- torch.mean / torch.var(unbiased)
    *rm = st.tmean;
    *rv = (float)st.var_u;
  }
  if (!train) {  // BatchNorm1d eval: float invstd from the running stats
    const float invstd = 1.0f / sqrtf(__fadd_rn(*rv, (float)eps));
    *alpha = invstd;
    if (arith == kBnStrided) {
      *shift = *rm;
      *beta = 0.f;
    } else {
      *shift = 0.f;
      *beta = -__fmul_rn(*rm, invstd);
    }
    return;
  }
  if (arith == kBnContig) {
    const float momf = (float)mom, vs = (float)st.var_sum;
    const float one_m = __fsub_rn(1.0f, momf);
    *rm = __fadd_rn(__fmul_rn(momf, st.mean), __fmul_rn(one_m, *rm));
    const float vu = __fdiv_rn(vs, (float)(n - 1));
    *rv = (float)((double)momf * (double)vu + (double)__fmul_rn(one_m, *rv));
    const float invstd = (float)(1.0 / sqrt((double)__fdiv_rn(vs, (float)n) + eps));
    *alpha = invstd;
    *beta = -__fmul_rn(st.mean, invstd);
    *shift = 0.f;
    return;
  }
  const double md = (double)st.mean;
  *rm = (float)(mom * md + (1.0 - mom) * (double)(*rm));
  const double vu = n > 1 ? st.var_sum / (nd - 1.0) : NAN;
  *rv = (float)(mom * vu + (1.0 - mom) * (double)(*rv));
  const float invstd = (float)(1.0 / sqrt(st.var_sum / nd + eps));
  *alpha = invstd;
  if (arith == kBnStrided) {
    *shift = st.mean;
    *beta = 0.f;
  } else {
    *shift = 0.f;
    *beta = -__fmul_rn(st.mean, invstd);
  }
}

// FP64 statistics from the sums: mean = s / n, var_sum = s2 - s*mean.
__device__ __forceinline__ BnCol bn_from_sums(double s, double s2, int64_t n) {
  BnCol st;
  const double nd = (double)n;
  const double mean = s / nd;
  double m2 = s2 - s * mean;
  if (m2 < 0.0) m2 = 0.0;
  st.mean = (float)mean;
  st.tmean = (float)mean;
  st.var_sum = m2;
  st.var_u = n > 1 ? m2 / (nd - 1.0) : NAN;
  return st;
}

struct BnArgs {           // per-call BatchNorm parameters (feature / gradient half)
  int mode, arith_x, arith_g;
  double mom_f, eps_f, mom_g, eps_g, eps_std;
  float *rm_f, *rv_f, *rm_g, *rv_g;
  float* coef;            // [6][F]
  float* batch_out;       // [4][F] or null
  long long *nbt_f, *nbt_g;
  int D;
};

// column k of half g (0: features, 1: gradients) of F columns
__device__ __forceinline__ void bn_emit(const BnArgs& a, int F, int g, int k, const BnCol& st,
                                        bool have, int64_t n) {
  if (a.D > 0 && k % a.D == 0 && (a.mode == 1 || a.mode == 2)) {
    long long* nbt = g ? a.nbt_g : a.nbt_f;   // BatchNorm1d.num_batches_tracked += 1
    if (nbt) nbt[k / a.D] += 1;
  }
  const int o = g ? 2 * F : 0;
  bn_column(st, have, n, a.mode, g ? a.arith_g : a.arith_x, g ? a.mom_g : a.mom_f,
            g ? a.eps_g : a.eps_f, a.eps_std, (g ? a.rm_g : a.rm_f) + k,
            (g ? a.rv_g : a.rv_f) + k, a.coef + o + k, a.coef + o + F + k,
            a.coef + (g ? 5 * F : 4 * F) + k,
            a.batch_out ? a.batch_out + o + k : nullptr,
            a.batch_out ? a.batch_out + o + F + k : nullptr);
}

__global__ void bn_finalize_kernel(const double* __restrict__ sums, int64_t n, int F,
                                   int with_grad, BnArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= F) return;
  const bool have = sums != nullptr;
  // n <= 0: the row count travels in sums[4F] (multi-GPU: summed by the same
  // all-reduce as the statistics, so no host round trip)
  if (have && n <= 0) n = (int64_t)sums[4 * F];
  bn_emit(a, F, 0, c, have ? bn_from_sums(sums[c], sums[F + c], n) : BnCol{}, have, n);
  if (with_grad)
    bn_emit(a, F, 1, c, have ? bn_from_sums(sums[2 * F + c], sums[3 * F + c], n) : BnCol{},
            have, n);
}

// Single-process fusion of bn_stats_reduce + bn_finalize (FP64 arithmetic).
// Block = 32 data columns; lane l of every wave reads value column (l / 32 ?
// sum of squares : sum) of data column 32*block + l % 32, so a half-wave
// reads 256 contiguous bytes of a chunk row; wave w sums its slice of the
// chunks in order, the 16 slices are folded in order in LDS (deterministic),
// then one thread per data column runs its BatchNorm update.  No all-reduce
// can sit between the two here, so multi-GPU callers keep vqgnn_bn_stats +
// vqgnn_bn_finalize.
constexpr int kRfThreads = 1024;
constexpr int kRfWaves = kRfThreads / 64;
__global__ void __launch_bounds__(kRfThreads)
bn_reduce_finalize_kernel(const double* __restrict__ part, int chunks, int F, int C,
                          double* __restrict__ sums, int64_t n, BnArgs a) {
  __shared__ double red[kRfWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 32 + (lane & 31);            // data column
  const int h = lane >> 5;                                // 0: sum, 1: sum of squares
  const int per = (chunks + kRfWaves - 1) / kRfWaves;
  const int p0 = wave * per, p1 = min(chunks, p0 + per);
  double acc = 0.0;
  if (c < C) {
    // all of a slice's loads in flight before the in-order adds (the
    // partials come from every XCD: each round trip is an L2 miss)
    const double* col = part + (int64_t)h * C + c;
    for (int p = p0; p < p1; p += 32) {
      double t[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) t[u] = p + u < p1 ? col[(int64_t)(p + u) * 2 * C] : 0.0;
#pragma unroll
      for (int u = 0; u < 32; ++u)
        if (p + u < p1) acc += t[u];
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (threadIdx.x >= 32) return;
  const int t = threadIdx.x;
  if (c >= C) return;
  double sm = red[0][t], sq = red[0][32 + t];
#pragma unroll
  for (int w = 1; w < kRfWaves; ++w) {
    sm += red[w][t];
    sq += red[w][32 + t];
  }
  const bool g = c >= F;
  const int k = g ? c - F : c;
  if (sums) {
    sums[(g ? 2 * F : 0) + k] = sm;
    sums[(g ? 3 * F : F) + k] = sq;
  }
  bn_emit(a, F, g, k, bn_from_sums(sm, sq, n), true, n);
}

// ---------------------------------------------------------------------------
// 2b. ATen-arithmetic statistics (STRIDED / CONTIG columns)
//
// at::mean's float cascade sum (SumKernel.cpp multi_row_sum, 4 levels):
// level 0 sums blocks of step = 2^lp rows sequentially, level 1 sums `step`
// blocks (a superblock), level 2 `step` superblocks (a group), level 3 the
// groups; the tail rows and the unfinished levels are added last as
// ((tail + acc1) + acc2) + acc3.  lp = max(4, ceil_log2(B) / 4).
// bn_cascade_partial_kernel: four waves per (superblock, 64-column tile) — the
// lanes of column c sum its superblock's blocks in the reference's order and
// also accumulates P = sum (x - x0), Q = sum (x - x0)^2 in double about the
// column's first value x0 (the variance terms, cancellation-free).
// bn_contig_chunk_kernel: the channels-last per-thread row chunks (CONTIG
// columns only; a serial fp32 chain per chunk, as the CPU thread runs it).
// bn_aten_finalize_kernel: one wave per column folds the partials and runs
// the BatchNorm update of its arithmetic.
// ---------------------------------------------------------------------------
constexpr int kCasWaves = 4;       // waves per (superblock, 64-column tile)
constexpr int kCasMaxStep = 64;    // block sums a workgroup holds (lp <= 6)

__device__ __forceinline__ const float* bn_col_base(const float* X, int64_t ldx, const float* G,
                                                    int64_t ldg, int F, int c, int64_t* ld) {
  *ld = c < F ? ldx : ldg;
  return c < F ? X + c : G + (c - F);
}

// One workgroup per (superblock, tile): wave w sums blocks w, w + 4, ... of
// the superblock (16 rows in flight per lane) into an LDS table, then wave 0
// adds the block sums in block order -- the reference's level-1 chain, bit
// for bit -- and the waves' fp64 (P, Q) in wave order.  Superblocks of more
// than kCasMaxStep blocks (B > 2^27 rows) are summed by wave 0 alone.
__global__ void __launch_bounds__(kCasWaves * 64)
bn_cascade_partial_kernel(const float* __restrict__ X, int64_t ldx,
                          const float* __restrict__ G, int64_t ldg, int B, int F, int C,
                          int lp, int nsb, int ntiles, float* __restrict__ sb_sum,
                          double* __restrict__ sb_p, double* __restrict__ sb_q,
                          float* __restrict__ tail) {
  __shared__ float s_bs[kCasMaxStep][64];
  __shared__ double s_pq[2][kCasWaves][64];
  const int sb = blockIdx.x / ntiles, tile = blockIdx.x % ntiles;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = tile * 64 + lane;
  const bool live = c < C;
  int64_t ld;
  const float* base = bn_col_base(X, ldx, G, ldg, F, live ? c : 0, &ld);
  const double x0 = (double)base[0];
  const int step = 1 << lp;
  const int nblk_all = B >> lp;
  const int nblk = min(step, nblk_all - (sb << lp));     // complete blocks in this superblock
  const int64_t r0 = (int64_t)sb << (2 * lp);
  const bool split = step <= kCasMaxStep;
  const int kstride = split ? kCasWaves : 1;
  double p = 0.0, q = 0.0;
  float acc1 = 0.f;
  if (live && (split || wave == 0)) {
    for (int k = split ? wave : 0; k < nblk; k += kstride) {
      const float* rp = base + (r0 + ((int64_t)k << lp)) * ld;
      float bs = 0.f;
      for (int i0 = 0; i0 < step; i0 += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = rp[(int64_t)(i0 + u) * ld];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          bs = __fadd_rn(bs, v[u]);
          const double d = (double)v[u] - x0;
          p += d;
          q = fma(d, d, q);
        }
      }
      if (split) s_bs[k][lane] = bs;
      else acc1 = __fadd_rn(acc1, bs);
    }
  }
  s_pq[0][wave][lane] = p;
  s_pq[1][wave][lane] = q;
  __syncthreads();
  if (wave != 0 || !live) return;
  if (split) {
    for (int k = 0; k < nblk; ++k) acc1 = __fadd_rn(acc1, s_bs[k][lane]);
    p = s_pq[0][0][lane];
    q = s_pq[1][0][lane];
#pragma unroll
    for (int w = 1; w < kCasWaves; ++w) {
      p += s_pq[0][w][lane];
      q += s_pq[1][w][lane];
    }
  }
  if (sb == nsb - 1) {        // the tail rows (B mod step) follow the last complete block
    float ts = 0.f;
    for (int64_t r = (int64_t)nblk_all << lp; r < B; ++r) {
      const float v = base[r * ld];
      ts = __fadd_rn(ts, v);
      const double d = (double)v - x0;
      p += d;
      q = fma(d, d, q);
    }
    tail[c] = ts;
  }
  const int64_t o = (int64_t)c * nsb + sb;
  sb_sum[o] = acc1;
  sb_p[o] = p;
  sb_q[o] = q;
}

// pass 0: buf[t][c] = fp32 sum of chunk t; pass 1: fp32 fma chain of
// (x - mean)^2 with mean = (float)(sum_t buf0[t][c] / B)  (CONTIG columns)
__global__ void __launch_bounds__(256)
bn_contig_chunk_kernel(const float* __restrict__ X, int64_t ldx, const float* __restrict__ G,
                       int64_t ldg, int B, int F, int C, int arith_x, int arith_g, int T,
                       int chunk, int pass, const float* __restrict__ buf0,
                       float* __restrict__ buf) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int t = blockIdx.y;
  if (c >= C || (c < F ? arith_x : arith_g) != kBnContig) return;
  int64_t ld;
  const float* base = bn_col_base(X, ldx, G, ldg, F, c, &ld);
  const int64_t r0 = (int64_t)t * chunk, r1 = min((int64_t)B, r0 + chunk);
  float s = 0.f;
  if (pass == 0) {
    for (int64_t r = r0; r < r1; ++r) s = __fadd_rn(s, base[r * ld]);
  } else {
    double m = 0.0;
    for (int u = 0; u < T; ++u) m += (double)buf0[(int64_t)u * C + c];
    const float mean = (float)(m / (double)B);
    for (int64_t r = r0; r < r1; ++r) {
      const float d = __fsub_rn(base[r * ld], mean);
      s = fmaf(d, d, s);
    }
  }
  buf[(int64_t)t * C + c] = s;
}

// The finalize's fold of one column c, in three phases separated by the
// caller's barriers (bn_aten_finalize_kernel: a one-wave block; the fused
// assign prologue of vq_filter_kernel: one wave per k slot).  sbs is the
// column's LDS scratch: [nsb] superblock sums, then [nsb >> lp] group sums.
// Phase 1 (every lane): the superblock sums into sbs, the fp64 (P, Q) summed
// over the lanes by a fixed butterfly (every lane ends with the totals).
__device__ __forceinline__ void bn_fold_load(int c, int nsb, const float* __restrict__ sb_sum,
                                             const double* __restrict__ sb_p,
                                             const double* __restrict__ sb_q, float* sbs,
                                             int lane, double* pp, double* qq) {
  const int64_t o = (int64_t)c * nsb;
  double p = 0.0, q = 0.0;
  // eight rounds of loads in flight before the in-order adds (one memory
  // round trip up to nsb = 512 instead of one per 64 superblocks)
  constexpr int U = 8;
  for (int i0 = lane; i0 < nsb; i0 += 64 * U) {
    float sv[U];
    double pv[U], qv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 64 * u;
      sv[u] = i < nsb ? sb_sum[o + i] : 0.f;
      pv[u] = i < nsb ? sb_p[o + i] : 0.0;
      qv[u] = i < nsb ? sb_q[o + i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 64 * u;
      if (i < nsb) {
        sbs[i] = sv[u];
        p += pv[u];
        q += qv[u];
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {   // fixed butterfly: deterministic
    p += __shfl_xor(p, off);
    q += __shfl_xor(q, off);
  }
  *pp = p;
  *qq = q;
}

// Phase 2 (every lane): the level-2 group sums, one lane per group
__device__ __forceinline__ void bn_fold_groups(int B, int lp, int nsb, float* sbs, int lane) {
  const int step = 1 << lp;
  const int nblk = B >> lp, nsb_full = nblk >> lp, ngr = nsb_full >> lp;
  float* grp = sbs + nsb;
  for (int gi = lane; gi < ngr; gi += 64) {
    float acc2 = 0.f;
    for (int k0 = 0; k0 < step; k0 += 16) {     // step = 2^lp, lp >= 4: whole runs of 16
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = sbs[gi * step + k0 + u];
#pragma unroll
      for (int u = 0; u < 16; ++u) acc2 = __fadd_rn(acc2, v[u]);
    }
    grp[gi] = acc2;
  }
}

// Phase 3 (one lane): the cascade total ((tail + acc1) + acc2) + acc3 and the
// column's statistics in its arithmetic
__device__ __forceinline__ BnCol bn_fold_stats(const float* X, int64_t ldx, const float* G,
                                               int64_t ldg, int B, int F, int C, int lp, int nsb,
                                               const float* sbs, const float* __restrict__ tail,
                                               int T, const float* __restrict__ cbuf0,
                                               const float* __restrict__ cbuf1, int c, int arith,
                                               double p, double q) {
  const int step = 1 << lp;
  const int nblk = B >> lp, nsb_full = nblk >> lp, ngr = nsb_full >> lp;
  const float* grp = sbs + nsb;
  // the two global loads first: their round trip overlaps the LDS chains
  int64_t ld;
  const float x0f = bn_col_base(X, ldx, G, ldg, F, c, &ld)[0];
  const float tc = tail[c];
  float acc3 = 0.f;
  for (int g0 = 0; g0 < ngr; g0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = g0 + u < ngr ? grp[g0 + u] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (g0 + u < ngr) acc3 = __fadd_rn(acc3, v[u]);
  }
  float acc2 = 0.f;
  for (int k = ngr * step; k < nsb_full; ++k) acc2 = __fadd_rn(acc2, sbs[k]);
  const float acc1 = nsb_full < nsb ? sbs[nsb_full] : 0.f;
  const float total = __fadd_rn(__fadd_rn(__fadd_rn(tc, acc1), acc2), acc3);
  const double x0 = (double)x0f;
  const double nd = (double)B;
  BnCol st;
  st.tmean = __fdiv_rn(total, (float)B);
  double vs_exact = q - p * (p / nd);       // sum (x - exact mean)^2
  if (vs_exact < 0.0) vs_exact = 0.0;
  st.var_u = B > 1 ? vs_exact / (nd - 1.0) : NAN;
  if (arith == kBnContig) {
    double s = 0.0, v = 0.0;
    for (int u = 0; u < T; ++u) {
      s += (double)cbuf0[(int64_t)u * C + c];
      v += (double)cbuf1[(int64_t)u * C + c];
    }
    st.mean = (float)(s / nd);
    st.var_sum = (double)(float)v;
  } else if (arith == kBnStrided) {
    st.mean = st.tmean;
    const double dm = (double)st.mean - x0;
    double vs = q - dm * (2.0 * p - nd * dm);  // sum (x - mean)^2 about the float mean
    st.var_sum = vs < 0.0 ? 0.0 : vs;
  } else {
    const double md = x0 + p / nd;
    st.mean = (float)md;
    st.var_sum = vs_exact;
  }
  return st;
}

__global__ void __launch_bounds__(64)
bn_aten_finalize_kernel(const float* __restrict__ X, int64_t ldx, const float* __restrict__ G,
                        int64_t ldg, int B, int F, int C, int lp, int nsb,
                        const float* __restrict__ sb_sum, const double* __restrict__ sb_p,
                        const double* __restrict__ sb_q, const float* __restrict__ tail,
                        int T, const float* __restrict__ cbuf0, const float* __restrict__ cbuf1,
                        BnArgs a) {
  extern __shared__ float sbs[];
  const int c = blockIdx.x, lane = threadIdx.x;
  double p, q;
  bn_fold_load(c, nsb, sb_sum, sb_p, sb_q, sbs, lane, &p, &q);
  __syncthreads();
  bn_fold_groups(B, lp, nsb, sbs, lane);
  __syncthreads();
  if (lane != 0) return;
  const bool g = c >= F;
  const int k = g ? c - F : c;
  const int arith = g ? a.arith_g : a.arith_x;
  const BnCol st = bn_fold_stats(X, ldx, G, ldg, B, F, C, lp, nsb, sbs, tail, T, cbuf0, cbuf1, c,
                                 arith, p, q);
  bn_emit(a, F, g, k, st, true, (int64_t)B);
}

// The finalize folded into vq_filter_kernel's prologue (single-process
// BatchNorm of the cascade arithmetic): the partials of
// bn_cascade_partial_kernel and the finalize's parameters.  Every workgroup
// of branch b folds b's k-slot columns itself; part 0's workgroups are the
// owners that update the running statistics, num_batches_tracked, the
// coefficient table and the batch stash, exactly as bn_aten_finalize_kernel.
struct BnFold {
  const float* sb_sum;
  const double* sb_p;
  const double* sb_q;
  const float* tail;
  int lp, nsb, C;
  BnArgs a;
};

// LDS scratch of the fold: W columns of nsb + ngr floats (+1 for alignment)
static inline size_t bn_fold_scratch(int nsb, int lp, int W) {
  return (size_t)W * (size_t)(nsb + (nsb >> lp) + 1) * sizeof(float);
}

// ---------------------------------------------------------------------------
// 3. PQ assignment on MFMA f32 (v_mfma_f32_16x16x4_f32)
//
// Workgroup = (branch b, row part); 16 waves.  The branch's codebook is staged
// in LDS once and reused for every row of the part; each wave owns 64 rows
// per iteration (4 groups of 16) and prefetches the next iteration's raw rows
// into registers while the MFMA sweep runs.  MFMA tile: A = 16 codewords x 4 k
// (LDS), B = 4 k x 16 rows (registers), D[16 codewords][16 rows]:
//   lane l: q = l>>4, j = l&15; A operand E[m0+j][kc*4+q], B operand
//   Xn[row j][kc*4+q]; D reg r = codeword m0 + 4q + r for row j.
// Per lane a running (best, index) over its codewords in increasing order with
// strict '<' keeps the first index; the 4 q-lanes of a row merge with
// (d, index) lexicographic order -> torch.argmin semantics (first index).
//
// LDS: codebook as [q][m][KC] floats (q stride padded so the 16-lane halves of
// a ds_read hit disjoint banks), |e|^2 per codeword, and (fused EMA) the
// per-codeword count + sum of normalised x accumulated with ds_add_f32; the
// accumulators leave as one partial slab per (part, branch) — a handful of
// parts, summed in order by the finalize kernel (deterministic).
// ---------------------------------------------------------------------------
constexpr int kAssignThreads = 1024;       // non-fused EMA kernel block
constexpr size_t kLdsBudget = 160 * 1024;
// codewords of LDS slack after each staged chunk: the sweep prefetches one
// tile pair ahead without a bound check (staged as e = 0, |e|^2 = +inf)
constexpr int kSweepSlack = 32;

struct AssignGeom {
  int parts;          // row parts per branch (= EMA partial slabs)
  int rows_per_part;
  int iters;          // 1024-row iterations per part
  int mpad;           // M rounded up to 16
  int chunk;          // codewords per LDS chunk (multiple of 16)
  int kc;             // k-chunks of 4 (W padded to 4*kc)
  bool fused;         // EMA statistics accumulated in the assign kernel
  int wv;             // waves per workgroup (8 or 16)
  bool filter;        // vq_filter_kernel (W <= 8) instead of vq_assign_kernel
  size_t lds;         // dynamic LDS of the filter kernel's launch
  int elds;           // filter: f32 codebook copy in LDS for the resolve
  bool co;            // filter, several chunks: chunk-outer passes (each chunk staged
                      // once per workgroup; per-row state between passes in the workspace)
};

template <int KC>
__host__ __device__ constexpr int q_pad_bytes() {
  // >= kSweepSlack codewords of each plane; mod 256 B (one pass over the 64
  // banks) the planes keep the bank offsets 16 (KC=1) / 32 (KC=2) / 0 (KC=4)
  return KC == 1 ? 320 : (KC == 2 ? 384 : 512);
}

template <int KC>
__host__ __device__ inline int q_stride_floats(int chunk) {
  return chunk * KC + q_pad_bytes<KC>() / 4;
}

// codebook planes + |e|^2, each with kSweepSlack codewords of slack
static size_t cb_lds_bytes(int kc, int chunk) {
  const int pad = kc == 1 ? q_pad_bytes<1>() : (kc == 2 ? q_pad_bytes<2>() : q_pad_bytes<4>());
  return (size_t)4 * (chunk * kc * 4 + pad) + (size_t)(chunk + kSweepSlack) * 4;
}

// EMA sufficient statistics are int64 fixed point.  Every normalised value
// is rounded once to an int32 multiple of 2^-shift and the products of the
// one-hot reduction are integer sums: associative, so the statistic is
// bit-identical whatever the thread order, the part split or the rank count
// (an int64 all-reduce is exact).  The shifts follow from the train-mode
// BatchNorm bound |z| <= sqrt(count - 1) (EMA updates only run in training,
// vq.py:176/241, with batch statistics): count * 2^shift * bound < 2^62.
// The count column is in units of 1.
// (timing probe, experiments builds: the fused assigns without their
// final slab fold; results invalid)
#ifndef VQGNN_ASG_NO_FLUSH
#define VQGNN_ASG_NO_FLUSH 0
#endif

struct StatShift {
  int f, g;
};
static StatShift stat_shift(int64_t count, float grad_scale) {
  const double bound = std::sqrt((double)(count > 1 ? count : 1));
  auto shift_for = [](double vmax) {
    if (!(vmax > 0.0)) return 30;
    int e = 0;
    std::frexp(vmax, &e);          // vmax < 2^e
    const int s = 30 - e;          // |v| * 2^s < 2^30 (< int32, ties to even)
    return s < -100 ? -100 : (s > 100 ? 100 : s);
  };
  return {shift_for(bound), shift_for(bound * std::fabs((double)grad_scale))};
}

__device__ __forceinline__ unsigned long long to_fixed(float v, int shift) {
  // v_ldexp + v_rndne + v_cvt_i32 (saturating); sign-extended to 64 bits
  const int t = (int)rintf(ldexpf(v, shift));
  return (unsigned long long)(long long)t;
}

// Waves per workgroup: 8, or 16 where the LDS footprint (a large codebook,
// or the fused EMA slab of M = 1024) leaves one workgroup per CU — the
// choice with more resident waves per CU (assign_geom).
constexpr int kAsgGroups = 2;   // 16-row groups per wave and iteration

template <int KC, bool FUSED, int WM, int WV>
__global__ void __launch_bounds__(WV * 64)
vq_assign_kernel(const float* __restrict__ X, int64_t ldx,
                 const float* __restrict__ Gr, int64_t ldg,
                 int B, int nb, int D, int M, int W,
                 const float* __restrict__ coef, float grad_scale,
                 const float* __restrict__ emb, int ldw, int64_t emb_bstride,
                 int64_t* __restrict__ idx_out, int16_t* __restrict__ codes, int64_t ldc,
                 const int64_t* __restrict__ batch_idx,
                 int* __restrict__ idx32, unsigned long long* __restrict__ partial,
                 int rows_per_part, int chunk, int shift_f, int shift_g, int m_sweep);

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
constexpr int kFltSlack = 32;          // one tile pair of prefetch past a chunk
constexpr int kFltBytesPerCode = 52;   // 3 f16 planes of 16 B + |e|^2 (f32)

static size_t flt_lds_bytes(int chunk) {
  return (size_t)kFltBytesPerCode * (chunk + kFltSlack);
}

// Per-wave fragment buffer of vq_filter_kernel (after the codebook planes
// and the fused slab): [16 rows][12 dwords], one row group at a time

// filtered assignment for W <= 8 (section 3b)
template <bool FUSED, int WM, int WV, bool CO>
__global__ void __launch_bounds__(WV * 64)
vq_filter_kernel(const float* __restrict__ X, int64_t ldx, const float* __restrict__ Gr,
                 int64_t ldg, int B, int nb, int D, int M, int W,
                 const float* __restrict__ coef, float grad_scale,
                 const float* __restrict__ emb, int ldw, int64_t emb_bstride,
                 int64_t* __restrict__ idx_out, int16_t* __restrict__ codes, int64_t ldc,
                 const int64_t* __restrict__ batch_idx, int* __restrict__ idx32,
                 unsigned long long* __restrict__ partial, int* __restrict__ flags,
                 int rows_per_part, int chunk, int shift_f, int shift_g, int m_sweep, int elds,
                 BnFold fold, unsigned long long* __restrict__ co_state, int co_pass);

// the filter's row-load mode: 2 -> W = 8 = 2D, D = 4; 1 -> W = D = 4 (float4
// rows, aligned); 0 -> general
static int flt_mode(int W, int D, int64_t ldx, int64_t ldg, const void* X, const void* G) {
  const bool ax = (ldx & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  const bool ag = G && (ldg & 3) == 0 && (reinterpret_cast<uintptr_t>(G) & 15) == 0;
  if (D == 4 && W == 8 && ax && ag) return 2;
  if (D == 4 && W == 4 && ax) return 1;
  return 0;
}

template <int WV>
static const void* flt_fn_wv(bool fused, int wm, bool co) {
  if (fused) return wm == 1 ? (const void*)vq_filter_kernel<true, 1, WV, false>
                  : wm == 2 ? (const void*)vq_filter_kernel<true, 2, WV, false>
                            : (const void*)vq_filter_kernel<true, 0, WV, false>;
  if (co) return wm == 1 ? (const void*)vq_filter_kernel<false, 1, WV, true>
                 : wm == 2 ? (const void*)vq_filter_kernel<false, 2, WV, true>
                           : (const void*)vq_filter_kernel<false, 0, WV, true>;
  return wm == 1 ? (const void*)vq_filter_kernel<false, 1, WV, false>
       : wm == 2 ? (const void*)vq_filter_kernel<false, 2, WV, false>
                 : (const void*)vq_filter_kernel<false, 0, WV, false>;
}
static const void* flt_fn(bool fused, int wm, int wv, bool co) {
  return wv == 16 ? flt_fn_wv<16>(fused, wm, co) : flt_fn_wv<8>(fused, wm, co);
}

// the filtered path serves W <= 8 (VQGNN_ASSIGN_EXACT=1: the exact f32 sweep
// for every W, a measurement and cross-check knob)
static bool use_filter(int W) {
  static const int exact_env = path_env("VQGNN_ASSIGN_EXACT", 0);
  return W <= 8 && !exact_env;
}

// k-slot layout: 0 general (W < 4*KC, padded), 1 W == 4*KC == D (features),
// 2 W == 4*KC == 2*D (features then grads)
static int slot_mode(int kc, int W, int D) {
  if (W != 4 * kc) return 0;
  return W == D ? 1 : 2;
}

template <int KC, int WV>
static const void* assign_fn_wv(bool fused, int wm) {
  if (fused) return wm == 1 ? (const void*)vq_assign_kernel<KC, true, 1, WV>
                  : wm == 2 ? (const void*)vq_assign_kernel<KC, true, 2, WV>
                            : (const void*)vq_assign_kernel<KC, true, 0, WV>;
  return wm == 1 ? (const void*)vq_assign_kernel<KC, false, 1, WV>
       : wm == 2 ? (const void*)vq_assign_kernel<KC, false, 2, WV>
                 : (const void*)vq_assign_kernel<KC, false, 0, WV>;
}
template <int KC>
static const void* assign_fn(bool fused, int wm, int wv) {
  return wv == 16 ? assign_fn_wv<KC, 16>(fused, wm) : assign_fn_wv<KC, 8>(fused, wm);
}

// Workgroups of the assign kernel the current device holds at once (register
// and LDS limited), cached per configuration.  Without a device (host-only
// queries) a static estimate is returned; the value only sizes the grid.
static int assign_capacity(int kc, bool fused, int wm, size_t lds, int wv, bool flt,
                           bool co = false) {
  const int fallback = 512 * 8 / wv;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return fallback;
  }
  static std::mutex mu;
  static std::map<std::tuple<int, int, bool, size_t>, int> cache;
  const auto key = std::make_tuple(dev, (((co ? 16 : 0) + (flt ? 8 : 0) + kc) * 128 + wm * 32 + wv),
                                   fused, lds);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const void* fn = flt ? flt_fn(fused, wm, wv, co)
                 : kc == 1 ? assign_fn<1>(fused, wm, wv)
                 : kc == 2 ? assign_fn<2>(fused, wm, wv) : assign_fn<4>(fused, wm, wv);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int cap = fallback;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, wv * 64, lds) == hipSuccess &&
      per_cu > 0 && cus > 0)
    cap = per_cu * cus;
  (void)hipGetLastError();
  cache[key] = cap;
  return cap;
}

static AssignGeom assign_geom(int B, int nb, int M, int W) {
  AssignGeom g;
  g.kc = W <= 4 ? 1 : (W <= 8 ? 2 : 4);
  g.filter = use_filter(W);
  g.mpad = (M + 15) / 16 * 16;
  const size_t acc = (size_t)M * (W + 1) * sizeof(unsigned long long);
  if (g.filter) {
    // staged in tile pairs: chunks of 32 codewords
    g.mpad = (M + 31) / 32 * 32;
    g.fused = flt_lds_bytes(g.mpad) + acc <= kLdsBudget;
    int c = g.mpad;
    if (!g.fused)
      while (c > 32 && flt_lds_bytes(c) > kLdsBudget) c = (c / 2 + 31) / 32 * 32;
    // measurement knob: a smaller staged chunk of the filter (multiple of 32)
    const int fenv = VQGNN_KNOB("VQGNN_FLT_CHUNK", 0);
    if (!g.fused && fenv >= 32 && fenv < c) c = fenv / 32 * 32;
    g.chunk = c;
  } else if (cb_lds_bytes(g.kc, g.mpad) + acc <= kLdsBudget) {
    // fused EMA when codebook + accumulators share the LDS
    g.fused = true;
    g.chunk = g.mpad;
  } else {
    g.fused = false;
    int c = g.mpad;
    while (c > 16 && cb_lds_bytes(g.kc, c) > kLdsBudget) c = (c / 2 + 15) / 16 * 16;
    // measurement knob: a smaller staged chunk (more resident workgroups,
    // the codebook restaged once per chunk and row block)
    const int cenv = VQGNN_KNOB("VQGNN_ASG_CHUNK", 0);
    if (cenv >= 32 && cenv < c) c = cenv / 32 * 32;
    g.chunk = c;
  }
  size_t lds = g.filter ? flt_lds_bytes(g.chunk) : cb_lds_bytes(g.kc, g.chunk);
  if (g.fused) lds += acc;
  const size_t scr8 = 0;   // (the filter hands fragments over by permlane swaps: no scratch)
  const int wm = g.filter ? (W == 8 ? 2 : (W == 4 ? 1 : 0)) : (W == 4 * g.kc ? 2 : 0);
  // several chunks: chunk-outer passes, one launch per chunk, unless
  // VQGNN_ASG_CO=0 (chunk-inner: every chunk restaged for every 1,024-row
  // iteration).  A fused launch holds its whole codebook in one chunk.
  g.co = g.filter && !g.fused && g.chunk < M && VQGNN_KNOB("VQGNN_ASG_CO", 1) != 0;
  // waves per workgroup: the choice with more resident waves per CU (ties: 8).
  // (10-wave filter workgroups -- 20 resident waves at 5 per SIMD instead of
  // 16 -- measured 1.9x slower at arxiv update, 188 vs 98 us, and 1.4x at
  // feature_update: profiles/r04d_assign_waves_ab.txt)
  const int cap8 = assign_capacity(g.kc, g.fused, wm, lds + scr8, 8, g.filter, g.co);
  const int cap16 = assign_capacity(g.kc, g.fused, wm, lds + 2 * scr8, 16, g.filter, g.co);
  const int wenv = VQGNN_KNOB("VQGNN_ASG_WAVES", 0);
  g.wv = cap16 * 16 > cap8 * 8 ? 16 : 8;
  if (wenv == 8 || wenv == 16) g.wv = wenv;
  g.lds = lds + (g.wv == 16 ? 2 * scr8 : scr8);
  // the filter's f32 codebook copy, when it fits without costing resident
  // workgroups and the sweep leaves the LDS room: at chunks above 512
  // codewords the sweep's fragment reads dominate the LDS and the resolve
  // reads its candidates faster through L1 (arxiv_gat M = 1024: 274 us with
  // the copy, 253 us without; arxiv M = 256: 98 us with, 121 without).
  // VQGNN_FLT_ELDS=0/1 forces it off/on where it fits.
  g.elds = 0;
  if (g.filter) {
    const size_t ef = (size_t)(g.chunk + kFltSlack) * 32;
    const int wmv = wm;
    const int cap = g.wv == 16 ? cap16 : cap8;
    const int env = VQGNN_KNOB("VQGNN_FLT_ELDS", -1);
    if (g.lds + ef <= kLdsBudget && env != 0 &&
        (env == 1 || (g.chunk <= 512 &&
                      assign_capacity(g.kc, g.fused, wmv, g.lds + ef, g.wv, true, g.co) >= cap))) {
      g.elds = 1;
      g.lds += ef;
    }
  }
  // rows per workgroup iteration: the filter's lanes own one row each
  const int rows_per_iter = g.filter ? g.wv * 64 : g.wv * 16 * kAsgGroups;
  const int row_blocks = (B + rows_per_iter - 1) / rows_per_iter;
  // one full round of resident workgroups: parts x nb <= what the device
  // holds at once (every part has the same row count, so no tail round)
  const int target = VQGNN_KNOB("VQGNN_ASG_TARGET", g.wv == 16 ? cap16 : cap8);
  int parts = target / nb;
  if (parts < 1) parts = 1;
  if (parts > row_blocks) parts = row_blocks;
  g.parts = parts;
  g.rows_per_part = (B + parts - 1) / parts;
  g.iters = (g.rows_per_part + rows_per_iter - 1) / rows_per_iter;
  return g;
}

template <int KC>
struct Frag {
  float v[KC];
};

template <int KC>
__device__ __forceinline__ Frag<KC> lds_frag(const float* p) {
  Frag<KC> f;
  if constexpr (KC == 1) {
    f.v[0] = p[0];
  } else if constexpr (KC == 2) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    f.v[0] = t.x;
    f.v[1] = t.y;
  } else {
    const float4 t = *reinterpret_cast<const float4*>(p);
    f.v[0] = t.x;
    f.v[1] = t.y;
    f.v[2] = t.z;
    f.v[3] = t.w;
  }
  return f;
}

// plain v_min_f32 (no canonicalising v_max around it); inputs are finite or
// +inf here
__device__ __forceinline__ float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ float vmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

template <int NG>
__device__ __forceinline__ int pickn(const int (&a)[NG], int i) {
  int v = a[0];
#pragma unroll
  for (int g = 1; g < NG; ++g) v = (i == g) ? a[g] : v;
  return v;
}

// stage codebook rows [mc0, mc0+chunk) of E into LDS (cb [4][qs], se [chunk]),
// and the slack after them as empty codewords (e = 0, |e|^2 = +inf)
template <int KC, int NT>
__device__ __forceinline__ void stage_chunk(const float* __restrict__ E, int ldw, int W,
                                            int mc0, int mcount, int chunk, int qs,
                                            float* cb, float* se, int tid) {
  for (int m = tid; m < chunk + kSweepSlack; m += NT) {
    float e[4 * KC];
    const bool mv = m < mcount;
#pragma unroll
    for (int k = 0; k < 4 * KC; ++k) e[k] = (mv && k < W) ? E[(int64_t)(mc0 + m) * ldw + k] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4 * KC; ++k)
      if (k < W) s = (k == 0) ? __fmul_rn(e[k], e[k]) : __fadd_rn(s, __fmul_rn(e[k], e[k]));
    se[m] = mv ? s : INFINITY;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      if constexpr (KC == 1) {
        cb[qq * qs + m] = e[qq];
      } else if constexpr (KC == 2) {
        *reinterpret_cast<float2*>(cb + qq * qs + m * 2) = make_float2(e[qq], e[4 + qq]);
      } else {
        *reinterpret_cast<float4*>(cb + qq * qs + m * 4) =
            make_float4(e[qq], e[4 + qq], e[8 + qq], e[12 + qq]);
      }
    }
  }
}

template <int KC, bool FUSED, int WM, int WV>
__global__ void __launch_bounds__(WV * 64)
vq_assign_kernel(const float* __restrict__ X, int64_t ldx,
                 const float* __restrict__ Gr, int64_t ldg,
                 int B, int nb, int D, int M, int W,
                 const float* __restrict__ coef, float grad_scale,
                 const float* __restrict__ emb, int ldw, int64_t emb_bstride,
                 int64_t* __restrict__ idx_out, int16_t* __restrict__ codes, int64_t ldc,
                 const int64_t* __restrict__ batch_idx,
                 int* __restrict__ idx32, unsigned long long* __restrict__ partial,
                 int rows_per_part, int chunk, int shift_f, int shift_g, int m_sweep) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NG = kAsgGroups, NT = WV * 64, K4 = 4 * KC;
  const int F = nb * D;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wg % nb;
  const int part = wg / nb;
  const int qs = q_stride_floats<KC>(chunk);
  float* cb = smem;                       // [4][qs]
  float* se = smem + 4 * qs;              // [chunk]
  // [M][W+1] int64 fixed-point accumulators (FUSED), 8-byte aligned
  unsigned long long* acc =
      reinterpret_cast<unsigned long long*>(se + chunk + kSweepSlack);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, j = lane & 15;
  const float* E = emb + (int64_t)b * emb_bstride;
  const int nchunks = (M + chunk - 1) / chunk;
  // whole codeword rows as float4 in the resolve step
  const bool vec_rows = WM != 0 && (ldw & 3) == 0 && (emb_bstride & 3) == 0 &&
                        (reinterpret_cast<uintptr_t>(emb) & 15) == 0;

  const int b_rows = B, rpp = rows_per_part;

  if constexpr (FUSED) {
    for (int i = tid; i < M * (W + 1); i += NT) acc[i] = 0ull;
  }
  if (nchunks == 1) stage_chunk<KC, NT>(E, ldw, W, 0, M, chunk, qs, cb, se, tid);

  // k-slot k = kc*4 + q of this lane: column, normalisation coefficients
  float al[KC], be[KC], sh[KC];
  bool isg[KC], kval[KC];
  int colx[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    const int k = kc * 4 + q;
    kval[kc] = WM != 0 || k < W;
    if constexpr (WM == 1) isg[kc] = false;
    else if constexpr (WM == 2) isg[kc] = KC == 1 ? (q >= 2) : (kc >= KC / 2);
    else isg[kc] = k >= D;
    const int kk = isg[kc] ? k - D : k;
    const int c = b * D + kk;
    colx[kc] = c;
    al[kc] = kval[kc] ? coef[(isg[kc] ? 2 * F : 0) + c] : 0.f;
    be[kc] = kval[kc] ? coef[(isg[kc] ? 3 * F : F) + c] : 0.f;
    sh[kc] = kval[kc] ? coef[(isg[kc] ? 5 * F : 4 * F) + c] : 0.f;
  }

  const int part_begin = part * rpp;
  const int part_end = min(b_rows, part_begin + rpp);
  const int n_iters = part_end > part_begin ? (part_end - part_begin + NG * 16 * WV - 1) /
                                                  (NG * 16 * WV)
                                            : 0;

  // lane (q, j) of row group g holds row row0 + 16g + j, k-slots kc*4 + q.
  // Rows past the part are clamped to its last row: MFMA columns are
  // independent and those lanes write nothing.
  constexpr int RPW = 16 * NG;                 // rows per wave per iteration
  constexpr int RPI = WV * RPW;                // rows per workgroup iteration
  // X / G as buffer resources: 32-bit row offsets (the host checks that
  // B*ld*4 < 2^32), no 64-bit address arithmetic per load
  constexpr bool kBuf = WM != 0 && KC >= 2;   // k-slot -> X or G is compile-time
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, 0, (int)(uint32_t)min((int64_t)B * ldx * 4, (int64_t)0xFFFFFFFF), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Gr ? Gr : X), 0,
      (int)(uint32_t)min((int64_t)B * (Gr ? ldg : ldx) * 4, (int64_t)0xFFFFFFFF), 0x00020000);
  auto load_rows = [&](int it, float (&raw)[NG][KC]) {
    const int row0 = part_begin + it * RPI + wave * RPW;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int rowi = min(row0 + g * 16 + j, part_end - 1);
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        float v = 0.f;
        if constexpr (kBuf) {
          const bool gk = isg[kc];
          const uint32_t off = ((uint32_t)rowi * (uint32_t)(gk ? ldg : ldx) + (uint32_t)colx[kc]) * 4u;
          v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gk ? rsg : rsx, off, 0, 0));
        } else {
          const int64_t row = rowi;
          if (kval[kc]) v = isg[kc] ? Gr[row * ldg + colx[kc]] : X[row * ldx + colx[kc]];
        }
        raw[g][kc] = v;
      }
    }
  };

  float nxt[NG][KC];
  int64_t nbi = -1;                       // batch_idx of this lane's output row
  auto load_bidx = [&](int it) {
    const int row = part_begin + it * RPI + wave * RPW + q * 16 + j;
    return (codes && q < NG && row < part_end) ? batch_idx[row] : (int64_t)-1;
  };
  if (n_iters > 0) {
    load_rows(0, nxt);
    nbi = load_bidx(0);
  }
  if (nchunks == 1) __syncthreads();

  for (int it = 0; it < n_iters; ++it) {
    const int row0 = part_begin + it * RPI + wave * RPW;
    float xk[NG][KC];
    float sx[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        float v = fmaf(__fsub_rn(nxt[g][kc], sh[kc]), al[kc], be[kc]);   // BatchNorm1d (bn_apply)
        if (isg[kc]) v = __fmul_rn(v, grad_scale);        // vq.py:224
        xk[g][kc] = kval[kc] ? v : 0.f;                   // padded k-slots are 0
      }
    }
    const int64_t cur_bi = nbi;
    if (it + 1 < n_iters) {                                // prefetch under the MFMA sweep
      load_rows(it + 1, nxt);
      nbi = load_bidx(it + 1);
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      // |x|^2 summed sequentially over k = 0..W-1 (torch.sum(x**2, dim=1))
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < K4; ++k) {
        const float v = __shfl(xk[g][k >> 2], j + 16 * (k & 3));
        if (WM != 0 || k < W) s = (k == 0) ? __fmul_rn(v, v) : __fadd_rn(s, __fmul_rn(v, v));
      }
      sx[g] = s;
    }

    float best[NG];
    int bidx[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      best[g] = INFINITY;
      bidx[g] = 0;
    }

    for (int ch = 0; ch < nchunks; ++ch) {
      const int mc0 = ch * chunk;
      const int mcount = min(chunk, M - mc0);
      if (nchunks > 1) {
        __syncthreads();
        stage_chunk<KC, NT>(E, ldw, W, mc0, mcount, chunk, qs, cb, se, tid);
        __syncthreads();
      }
      // Sweep: per lane and row group only the running minimum distance and
      // the tile that first reached it (strict <: earliest tile wins ties).
      // Which codeword of the tile it was is resolved after the sweep by an
      // exact recompute (the f32 MFMA is bit-for-bit a k-ordered fma chain),
      // which keeps v_cmp/v_cndmask (4-cycle issue) out of the per-element
      // path: 3 v_min + 1 v_cmp + 1 v_min + 1 v_cndmask per 4 distances.
      float cbest[NG];
      // the tile that first reached cbest, recorded as the LDS offset register
      // the sweep read it through (no v_mov of a tile index): the codebook-
      // plane offset for the even tile of a pair, the |e|^2 offset for the
      // odd one; the two ranges are disjoint, decoded after the sweep
      const uint32_t a0 = (uint32_t)(q * qs + j * KC) * 4u;      // plane q, codeword j
      const uint32_t s0 = (uint32_t)(4 * qs + 4 * q) * 4u;       // |e|^2 of codewords 4q..4q+3
      uint32_t cmark[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        cbest[g] = INFINITY;
        cmark[g] = a0;                                            // tile 0
      }
      const char* lds = reinterpret_cast<const char*>(smem);
      auto tile = [&](const Frag<KC>& a, const float4& s4, uint32_t mark) {
        floatx4 d[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          d[g] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kc = 0; kc < KC; ++kc)
            d[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[kc], xk[g][kc], d[g], 0, 0, 0);
        }
        const float sev[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          float dist[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) dist[r] = fmaf(-2.f, d[g][r], __fadd_rn(sx[g], sev[r]));
          // n = min(cbest, tile min); n < cbest <=> the tile min < cbest
          // (strict: the earliest tile wins ties)
          const float n = vmin3(cbest[g], vmin3(dist[0], dist[1], dist[2]), dist[3]);
          cmark[g] = (n < cbest[g]) ? mark : cmark[g];
          cbest[g] = n;
        }
      };
      // Sweep over tile pairs: per lane and row group only the running minimum
      // and the tile that first reached it.  Which codeword of the tile it was
      // is resolved after the sweep by an exact recompute (the f32 MFMA is
      // bit-for-bit a k-ordered fma chain), which keeps v_cmp/v_cndmask
      // (4-cycle issue) out of the per-element path.  Operands of the next
      // pair are read while this pair computes (past the last tile: slack).
      uint32_t ao = a0, so = s0;
      Frag<KC> a_n0 = lds_frag<KC>(reinterpret_cast<const float*>(lds + ao));
      Frag<KC> a_n1 = lds_frag<KC>(reinterpret_cast<const float*>(lds + ao + 16 * KC * 4));
      float4 s_n0 = *reinterpret_cast<const float4*>(lds + so);
      float4 s_n1 = *reinterpret_cast<const float4*>(lds + so + 64);
      const int mlim = min(mcount, m_sweep);
      for (int m0 = 0; m0 < mlim; m0 += 32) {
        const Frag<KC> a_0 = a_n0, a_1 = a_n1;
        const float4 s_0 = s_n0, s_1 = s_n1;
        a_n0 = lds_frag<KC>(reinterpret_cast<const float*>(lds + ao + 32 * KC * 4));
        a_n1 = lds_frag<KC>(reinterpret_cast<const float*>(lds + ao + 48 * KC * 4));
        s_n0 = *reinterpret_cast<const float4*>(lds + so + 128);
        s_n1 = *reinterpret_cast<const float4*>(lds + so + 192);
        tile(a_0, s_0, ao);
        tile(a_1, s_1, so);          // past mcount: empty codewords, never < cbest
        ao += 32 * KC * 4;
        so += 128;
      }
      int ctile[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g)
        ctile[g] = cmark[g] >= (uint32_t)(4 * qs * 4) ? (int)((cmark[g] - s0) >> 2) + 16
                                                      : (int)((cmark[g] - a0) / (KC * 4));
      // Resolve, spread over the 4 q-lanes of a row: the row minimum, the
      // first (tile, q-lane) that reached it (index order = (tile, q, r)),
      // then lane q recomputes candidate r = q of that lane's codewords with
      // the operations and order of staging + MFMA + epilogue (bit-exact);
      // the smallest matching r wins.  All 4 lanes of a row end up holding
      // the same (best, idx).  Codewords come from global memory (L1): the
      // LDS planes bank-conflict for lane-divergent rows.
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        float rmin = cbest[g];
        rmin = vmin(rmin, __shfl_xor(rmin, 16));
        rmin = vmin(rmin, __shfl_xor(rmin, 32));
        int key = (cbest[g] == rmin) ? ctile[g] + 4 * q : 0x7fffffff;
        key = min(key, __shfl_xor(key, 16));
        key = min(key, __shfl_xor(key, 32));
        float xr[K4];
#pragma unroll
        for (int k = 0; k < K4; ++k) xr[k] = __shfl(xk[g][k >> 2], j + 16 * (k & 3));
        const int c = mc0 + key + q;                 // this lane's candidate codeword
        const bool cv = c < M;
        const float* er = E + (int64_t)(cv ? c : M - 1) * ldw;
        float e[K4];
        if (vec_rows) {
#pragma unroll
          for (int v = 0; v < KC; ++v) {
            const float4 t = *reinterpret_cast<const float4*>(er + 4 * v);
            e[4 * v] = t.x;
            e[4 * v + 1] = t.y;
            e[4 * v + 2] = t.z;
            e[4 * v + 3] = t.w;
          }
        } else {
#pragma unroll
          for (int k = 0; k < K4; ++k) e[k] = (WM != 0 || k < W) ? er[k] : 0.f;
        }
        float dot = 0.f;
#pragma unroll
        for (int k = 0; k < K4; ++k) {
          if (WM != 0 || k < W) dot = (k == 0) ? __fmul_rn(e[k], xr[k]) : fmaf(e[k], xr[k], dot);
        }
        // |e|^2 as staged (same operations; +inf past the codebook end)
        const float se_c = se[min(key + q, chunk - 1)];
        const float dist = fmaf(-2.f, dot, __fadd_rn(sx[g], cv ? se_c : INFINITY));
        int r = (dist == rmin) ? q : 4;
        r = min(r, __shfl_xor(r, 16));
        r = min(r, __shfl_xor(r, 32));
        if (rmin < best[g]) {                        // earlier chunk wins ties
          best[g] = rmin;
          bidx[g] = mc0 + key + (r & 3);
        }
      }
    }

    // ---- outputs: lane (q, j) writes group q's row j ----
    if (q < NG) {
      const int lrow = row0 + q * 16 + j;
      if (lrow < part_end) {
        const int row = lrow;
        const int m = pickn<NG>(bidx, q);
        if (idx_out) idx_out[(int64_t)b * B + row] = (int64_t)m;
        if (idx32) idx32[(int64_t)b * B + row] = m;
        if (codes) codes[cur_bi * ldc + b] = (int16_t)m;
      }
    }

    if constexpr (FUSED) {   // ds_add_u64: ~13x the rate of ds_add_f32 on gfx950
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if (row0 + g * 16 + j < part_end) {
          unsigned long long* a = acc + bidx[g] * (W + 1);
          if (q == 0) atomicAdd(a, 1ull);
#pragma unroll
          for (int kc = 0; kc < KC; ++kc)
            if (kval[kc]) atomicAdd(a + 1 + kc * 4 + q, to_fixed(xk[g][kc], isg[kc] ? shift_g : shift_f));
        }
      }
    }
  }

  if constexpr (FUSED) {   // fold into the single zeroed slab: integer, exact, order-free
    __syncthreads();
    unsigned long long* out = partial + (int64_t)b * M * (W + 1);
    // (VQGNN_ASG_NO_FLUSH: a timing probe without this fold, results invalid)
    if constexpr (VQGNN_ASG_NO_FLUSH == 0)
      for (int i = tid; i < M * (W + 1); i += NT)
        if (acc[i]) atomicAdd(out + i, acc[i]);
  }
}

// ---------------------------------------------------------------------------
// 3b. Filtered assignment, W <= 8 (the default path)
//
// The sweep scores every codeword on v_mfma_f32_16x16x32_f16 (16 cycles per
// 16x16 tile against 2 x 32 for the exact f32 MFMA at W = 8) from an f16
// split of both operands, and only the codewords that can win are computed
// in the reference's f32 arithmetic.  K slots of one MFMA (quad q of the A/B
// fragments holds k = 8q .. 8q+7):
//   quad 0: (-2 e_hi) . x_hi      quad 1: (-2 e_lo) . x_hi
//   quad 2: (-2 e_hi) . x_lo      quad 3: (|e|^2 split in three f16) . 1
//                                         + 1 . (|x|^2 + 1 split in three f16)
// with v_hi = f16(v), v_lo = f16(v - v_hi), so each score is
//   s = |x|^2 + 1 + |e|^2 - 2 x.e  (+ the split and accumulation error),
// the reference distance plus 1: positive, so scores compare as unsigned
// integers (v_min3_u32 / v_med3_u32, no float canonicalisation).
// Per lane and row group the sweep keeps the minimum over tile pairs (32
// codewords: 8 scores per lane), the pair that first reached it and the
// second-smallest pair minimum.  The resolve recomputes the winner lane's 8
// codewords of the winning pair with vq.py's operations and order (bit-exact,
// first index on ties); when any other codeword's score lies within the
// error bound Delta of the minimum (a near-tie), the row is appended to the
// workgroup's list and swept exactly after the row loop.  Delta
// (DESIGN.md §4.1): per codeword |score - (ref. distance + 1)| <=
// 2^-24 (89.5 |x|^2 + 88.5 |e|^2 + 36) for W <= 8, |e|^2 of any codeword within
// 1 of the minimum <= 4.01 |x|^2 + 2 |t| + 2.1 (t = minimum - |x|^2 - 1),
// twice that with a 10 % margin: Delta = 2^-24 (978 |x|^2 + 390 |t| + 489).
// The accumulation term assumes every internal add of the MFMA rounds to
// f32 or better (32 u of the summed magnitudes; scripts/probes/
// f16_mfma_accum.hip measured at most 5.1 u) and f16 subnormal operands
// kept (measured).  Rows with |x|^2 >= 2^16 go to the exact path.  Codewords
// with |e|^2 >= 2^15 (dead codewords of a trained codebook reach 10^10) are
// scored +inf; a row is decided by the filter only if the smallest such
// |e|^2, E0, keeps all of them out: (sqrt(E0) - |x|)^2 > score + Delta.
// ---------------------------------------------------------------------------

// (a & m) | o in one VOP3 (the compiler splits it when m and o are both
// wave-uniform: one scalar operand per VOP3 on gfx950); o goes through a VGPR
__device__ __forceinline__ uint32_t and_or_u32(uint32_t a, uint32_t m, uint32_t o) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(m), "v"(o));
  return r;
}

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;   // operands are VALU results (never raw MFMA results: no hazard)
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Position of codeword m in the resolve's f32 planes (ef k-planes, |e|^2):
// the two 16-codeword halves of a tile pair swap places when bit 1 of the
// pair index is set.  A resolve read (one k-plane, one half t, a run of 4
// codewords of the winning quad) then falls on bank slot 8 (pair & 1) +
// 4 (t ^ (pair >> 1 & 1)) + quad: 16 slots over the 32 (pair, quad) sets of
// a 256-codeword chunk instead of 8, fewer lanes of a 16-lane group on one
// bank.  Runs of 4 stay contiguous; chunks are multiples of 32 codewords.
// Wave priorities (s_setprio) of the filter's phases in the single-pass
// instances: the sweep's fold at 2, the row phase (row loads, BatchNorm
// apply, f16 split, B fragments) at 1, the resolve not raised -- arxiv
// assign 87.0-88.0 against 89.9-91.4 us, arxiv_gat 216.0-219.3 against
// 220.0-225.0 us (profiles/r06y2_assign_phase_prio_ab.txt).  The chunk-outer
// (CO) instances keep the fold at 1 and the row phase at 0: ppi's assign
// was 1 % slower with the raised row phase.  Compile-time; experiments
// builds set them (VQGNN_ASG_FOLD_PRIO / _ROW_PRIO / _RES_PRIO).
#ifndef VQGNN_ASG_FOLD_PRIO
#define VQGNN_ASG_FOLD_PRIO 2
#endif
#ifndef VQGNN_ASG_ROW_PRIO
#define VQGNN_ASG_ROW_PRIO 1
#endif
#ifndef VQGNN_ASG_CO_PRIO
#define VQGNN_ASG_CO_PRIO 0
#endif
#ifndef VQGNN_ASG_RES_PRIO
#define VQGNN_ASG_RES_PRIO 0
#endif
#ifndef VQGNN_ASG_OUT_PRIO
#define VQGNN_ASG_OUT_PRIO 0
#endif
#ifndef VQGNN_ASG_DEFER_STORES
#define VQGNN_ASG_DEFER_STORES 0
#endif
// dead waves leave the filter's row loop: arxiv assign 83.6-85.1 against
// 85.9-88.0 us, arxiv_gat 205-210 against 214-220, ppi 498-502 against
// 531-536 (profiles/r06y6_assign_tail_exit_ab.txt)
#ifndef VQGNN_ASG_TAIL_EXIT
#define VQGNN_ASG_TAIL_EXIT 1
#endif

__device__ __forceinline__ int flt_pos(int m) { return m ^ (((m >> 6) & 1) << 4); }

// stage codebook rows [mc0, mc0 + chunk + slack) of E: planes -2 e_hi,
// -2 e_lo, (|e|^2 split, 1, 1, 1, 0, 0) and |e|^2 in f32 (vq.py's order);
// past mcount: zero planes, |e|^2 = +inf.  Codewords with |e|^2 >= 2^15 (or
// NaN) are staged like empty ones and their smallest |e|^2 (0 for NaN) is
// folded into *bigmin (f32 bits; positive floats order as integers).
template <int NT>
__device__ __forceinline__ void stage_filter(const float* __restrict__ E, int ldw, int W, int mc0,
                                             int mcount, int chunk, char* smem, int tid,
                                             unsigned int* bigmin, float* ef = nullptr) {
  const int cs = chunk + kFltSlack;
  half8* p0 = reinterpret_cast<half8*>(smem);
  half8* p1 = p0 + cs;
  half8* p2 = p1 + cs;
  float* sef = reinterpret_cast<float*>(p2 + cs);
  for (int m = tid; m < cs; m += NT) {
    float e[8];
    const bool mv = m < mcount;
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = (mv && k < W) ? E[(int64_t)(mc0 + m) * ldw + k] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < W) s = (k == 0) ? __fmul_rn(e[k], e[k]) : __fadd_rn(s, __fmul_rn(e[k], e[k]));
    const bool big = mv && !(s < 32768.f);
    if (big) atomicMin(bigmin, s == s ? __float_as_uint(s) : 0u);
    half8 hi, lo, sp;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float ek = big ? 0.f : e[k];
      const _Float16 h = (_Float16)ek;
      const float hf = (float)h;
      const _Float16 l = (_Float16)__fsub_rn(ek, hf);
      hi[k] = (_Float16)(-2.f * hf);                 // exact: a doubled f16
      lo[k] = (_Float16)(-2.f * (float)l);
    }
    if (mv && !big) {
      const _Float16 s0 = (_Float16)s;
      const float r1 = __fsub_rn(s, (float)s0);      // exact
      const _Float16 s1 = (_Float16)r1;
      const _Float16 s2 = (_Float16)__fsub_rn(r1, (float)s1);
      sp = half8{s0, s1, s2, (_Float16)1.f, (_Float16)1.f, (_Float16)1.f, (_Float16)0.f,
                 (_Float16)0.f};
    } else {
      sp = half8{(_Float16)INFINITY, (_Float16)0.f, (_Float16)0.f, (_Float16)1.f, (_Float16)1.f,
                 (_Float16)1.f, (_Float16)0.f, (_Float16)0.f};
    }
    p0[m] = hi;
    p1[m] = lo;
    p2[m] = sp;
    sef[flt_pos(m)] = mv ? s : INFINITY;
    if (ef) {                     // k-planes [8][cs]: a run of 4 codewords is one float4
#pragma unroll
      for (int k = 0; k < 8; ++k) ef[k * cs + flt_pos(m)] = e[k];
    }
  }
}


// 4 x 4 transpose over (quad, group) of per-lane values r[g]: afterwards
// lane (q = g, j) holds r[t] = the value of quad t, group g, column j (two
// permlane32 and two permlane16 swaps, VALU; scripts/probes/permlane_swap.hip)
__device__ __forceinline__ void transpose_quads(uint32_t (&r)[4]) {
  const auto s02 = __builtin_amdgcn_permlane32_swap(r[0], r[2], false, false);
  r[0] = s02[0];
  r[2] = s02[1];
  const auto s13 = __builtin_amdgcn_permlane32_swap(r[1], r[3], false, false);
  r[1] = s13[0];
  r[3] = s13[1];
  const auto s01 = __builtin_amdgcn_permlane16_swap(r[0], r[1], false, false);
  r[0] = s01[0];
  r[1] = s01[1];
  const auto s23 = __builtin_amdgcn_permlane16_swap(r[2], r[3], false, false);
  r[2] = s23[0];
  r[3] = s23[1];
}

// WM: 2 -> W = 8 = 2D with D = 4 (features then gradients); 1 -> W = D = 4;
//     0 -> any W <= 8
//
// Work layout: a wave takes 64 rows per iteration, lane l owning row row0 + l
// (group g = l >> 4, the B columns of the g-th MFMA); the owner lane loads
// and normalises its whole row, builds its f16 split and, after the sweep,
// resolves it alone.  The sweep itself runs in the MFMA layout: lane (q, j)
// keeps, for each group g, the running minimum over its quad's codewords
// 4q .. 4q+3 of every tile; a 4 x 4 transpose over the quads (permlane
// swaps, VALU) hands the owner lane the four quads' minima of its row.
template <bool FUSED, int WM, int WV, bool CO>
__global__ void __launch_bounds__(WV * 64)
vq_filter_kernel(const float* __restrict__ X, int64_t ldx, const float* __restrict__ Gr,
                 int64_t ldg, int B, int nb, int D_, int M, int W_,
                 const float* __restrict__ coef, float grad_scale,
                 const float* __restrict__ emb, int ldw, int64_t emb_bstride,
                 int64_t* __restrict__ idx_out, int16_t* __restrict__ codes, int64_t ldc,
                 const int64_t* __restrict__ batch_idx, int* __restrict__ idx32,
                 unsigned long long* __restrict__ partial, int* __restrict__ flags,
                 int rows_per_part, int chunk, int shift_f, int shift_g, int m_sweep, int elds,
                 BnFold fold, unsigned long long* __restrict__ co_state, int co_pass) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NT = WV * 64;
  constexpr bool kCoPrio = CO && VQGNN_ASG_CO_PRIO == 0;     // chunk-outer: fold 1, row 0
  constexpr int kFoldPrio = kCoPrio ? 1 : VQGNN_ASG_FOLD_PRIO;   // wave priorities (above)
  constexpr int kRowPrio = kCoPrio ? 0 : VQGNN_ASG_ROW_PRIO;
  const int W = WM == 2 ? 8 : (WM == 1 ? 4 : W_);          // compile-time in the row modes
  const int D = WM != 0 ? 4 : D_;
  const int F = nb * D;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wg % nb;
  const int part = wg / nb;
  const int cs = chunk + kFltSlack;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, j = lane & 15;
  char* lds = reinterpret_cast<char*>(smem);
  const float* sef = reinterpret_cast<const float*>(lds + (size_t)48 * cs);
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(lds + (size_t)52 * cs);
  // the chunk's codewords in f32 [cs][8] for the resolve's exact candidates
  // (elds: when the LDS has room; else they are read from global memory)
  float* ef = elds ? reinterpret_cast<float*>(lds + (size_t)52 * cs +
                                              (FUSED ? (size_t)M * (W + 1) * 8 : 0))
                   : nullptr;
  const float* E = emb + (int64_t)b * emb_bstride;
  // a fused launch holds its whole codebook in one chunk (assign_geom): a
  // static single pass drops the restaging loop's code and 21 of its 40 SGPR
  // spills (arxiv update assign 92.5-93.0 against 94.1-96.3 us,
  // profiles/r06f_assign_single_chunk_ab.txt)
  const int nchunks = FUSED ? 1 : (M + chunk - 1) / chunk;
  const bool vec_rows = (ldw & 3) == 0 && (emb_bstride & 3) == 0 &&
                        (reinterpret_cast<uintptr_t>(emb) & 15) == 0;
  __shared__ int s_nflag;
  __shared__ unsigned int s_bigmin;
  // k-slot table: alpha, beta, shift, grad scale per k (field-major, so the
  // packed-f32 normalisation reads k-pairs as register pairs); grad scale is
  // 1 for features (v * 1 is exact)
  __shared__ __attribute__((aligned(16))) float s_kt[4][8];
  if (tid == 0) {
    s_nflag = 0;
    s_bigmin = 0x7f800000u;                           // +inf: no out-of-range codeword
  }
  if (fold.sb_sum) {
    // the BatchNorm finalize of this branch's W columns, one wave per k slot
    // (the finalize kernel's phases, bit for bit), in the planes' LDS before
    // they are staged; part 0's workgroup is the owner of the state updates
    const int percol = fold.nsb + (fold.nsb >> fold.lp) + 1;
    const bool fw = wave < W;
    const int k = fw ? wave : 0;
    const bool gk = W != D && k >= D;
    const int col = b * D + (gk ? k - D : k);
    const int c = gk ? F + col : col;
    float* sbs = reinterpret_cast<float*>(lds) + (size_t)k * percol;
    double p = 0.0, qq = 0.0;
    if (fw) bn_fold_load(c, fold.nsb, fold.sb_sum, fold.sb_p, fold.sb_q, sbs, lane, &p, &qq);
    __syncthreads();
    if (fw) bn_fold_groups(B, fold.lp, fold.nsb, sbs, lane);
    __syncthreads();
    if (fw && lane == 0) {
      const BnArgs& ba = fold.a;
      const int arith = gk ? ba.arith_g : ba.arith_x;
      const BnCol st = bn_fold_stats(X, ldx, Gr, ldg, B, F, fold.C, fold.lp, fold.nsb, sbs,
                                     fold.tail, 1, nullptr, nullptr, c, arith, p, qq);
      float al, be, sh;
      if (part == 0) {
        bn_emit(ba, F, gk ? 1 : 0, col, st, true, (int64_t)B);
        const int o = gk ? 2 * F : 0;            // this thread's own stores, read back
        al = ba.coef[o + col];
        be = ba.coef[o + F + col];
        sh = ba.coef[(gk ? 5 * F : 4 * F) + col];
      } else {
        // the same column arithmetic into registers; the running statistics
        // are read only by the eval form (mode 0), which nothing writes
        float rm = 0.f, rv = 0.f;
        if (ba.mode == 0) {
          rm = (gk ? ba.rm_g : ba.rm_f)[col];
          rv = (gk ? ba.rv_g : ba.rv_f)[col];
        }
        bn_column(st, true, (int64_t)B, ba.mode, arith, gk ? ba.mom_g : ba.mom_f,
                  gk ? ba.eps_g : ba.eps_f, ba.eps_std, &rm, &rv, &al, &be, &sh, nullptr,
                  nullptr);
      }
      s_kt[0][k] = al;
      s_kt[1][k] = be;
      s_kt[2][k] = sh;
    }
    if (tid < 8) {
      if (tid >= W) s_kt[0][tid] = s_kt[1][tid] = s_kt[2][tid] = 0.f;
      s_kt[3][tid] = (W != D && tid >= D) ? grad_scale : 1.f;
    }
  } else if (tid < 8) {
    const int k = tid;
    const bool kvv = k < W;
    const bool gk = W != D && k >= D;
    const int c = b * D + (gk ? k - D : k);
    s_kt[0][k] = kvv ? coef[(gk ? 2 * F : 0) + c] : 0.f;
    s_kt[1][k] = kvv ? coef[(gk ? 3 * F : F) + c] : 0.f;
    s_kt[2][k] = kvv ? coef[(gk ? 5 * F : 4 * F) + c] : 0.f;
    s_kt[3][k] = gk ? grad_scale : 1.f;
  }
  if constexpr (FUSED) {
    for (int i = tid; i < M * (W + 1); i += NT) acc[i] = 0ull;
  }
  int* const flist = flags + (int64_t)wg * rows_per_part;
  __syncthreads();
  if (CO)                     // chunk-outer launch: this pass's chunk, once
    stage_filter<NT>(E, ldw, W, co_pass * chunk, min(chunk, M - co_pass * chunk), chunk, lds,
                     tid, &s_bigmin, ef);
  else if (nchunks == 1)
    stage_filter<NT>(E, ldw, W, 0, M, chunk, lds, tid, &s_bigmin, ef);

  const int part_begin = part * rows_per_part;
  const int part_end = min(B, part_begin + rows_per_part);
  constexpr int RPI = WV * 64;
  const int n_iters = part_end > part_begin ? (part_end - part_begin + RPI - 1) / RPI : 0;
  // A-fragment byte offset of this lane: plane (q: 0 -> hi, 1 -> lo, 2 -> hi,
  // 3 -> |e|^2 parts), codeword j of tile 0
  const uint32_t a_lane = (uint32_t)(((q == 1) ? 1 : (q == 3 ? 2 : 0)) * cs + j) * 16u;
  if (CO || nchunks == 1) __syncthreads();

  // the owner lane's raw row (k-slot order: features, then gradients)
  auto load_raw = [&](int rowi, float (&raw)[8]) {
    if constexpr (WM != 0) {
      const float4 a = *reinterpret_cast<const float4*>(X + (int64_t)rowi * ldx + b * 4);
      raw[0] = a.x; raw[1] = a.y; raw[2] = a.z; raw[3] = a.w;
      if constexpr (WM == 2) {
        const float4 c = *reinterpret_cast<const float4*>(Gr + (int64_t)rowi * ldg + b * 4);
        raw[4] = c.x; raw[5] = c.y; raw[6] = c.z; raw[7] = c.w;
      } else {
        raw[4] = raw[5] = raw[6] = raw[7] = 0.f;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool gk = W != D && k >= D;
        const int c = b * D + (gk ? k - D : k);
        raw[k] = k < W ? (gk ? Gr[(int64_t)rowi * ldg + c] : X[(int64_t)rowi * ldx + c]) : 0.f;
      }
    }
  };
  // the k-slot coefficients, wave-uniform: read once into scalar registers in
  // the row modes (an LDS table re-read per iteration costs 8 LDS reads)
  float kt[4][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
      kt[f][k] = WM != 0 ? __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s_kt[f][k]))) : 0.f;
  }
  auto kc = [&](int f, int k) {
    if constexpr (WM != 0) return kt[f][k];
    else return s_kt[f][k];
  };
  // normalised as vq.py's bn_apply (+ vq.py:224's grad scale); returns |x|^2
  // summed in k order
  auto row_vals = [&](const float (&raw)[8], float (&xv)[8]) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = 0.f;
      if (k < W) {
        v = fmaf(__fsub_rn(raw[k], kc(2, k)), kc(0, k), kc(1, k));
        // grad scale on the gradient slots only (v * 1 is v: features skip it)
        if (WM == 0 || (WM == 2 && k >= 4)) v = __fmul_rn(v, kc(3, k));
        s = (k == 0) ? __fmul_rn(v, v) : __fadd_rn(s, __fmul_rn(v, v));
      }
      xv[k] = v;
    }
    return s;
  };

  float raw[8];                                       // the next row, loaded ahead
  // its node id for the code scatter too (a dependent load right before the
  // store would stall the wave on a memory round trip every iteration)
  int64_t nid = 0;
  // chunk-outer (CO: one launch per chunk, pass co_pass): the launch stages
  // its chunk once and runs every row against it, carrying each row's best
  // exact distance, index and near-tie flag to the next launch in co_state;
  // only the last pass writes the outputs.  Chunk-inner (nchunks > 1, not
  // CO): every row iteration walks all chunks, restaging each.  Same
  // comparisons in the same chunk order: the same indices.  (One launch per
  // pass, not a pass loop: the loop kept 20 more VGPRs live across the row
  // loop -- 139 instead of 119 at 8 waves, spills at 16.)
  const bool co = CO && co_state != nullptr;
  if (n_iters > 0) {
    const int r0 = min(part_begin + wave * 64 + lane, part_end - 1);
    load_raw(r0, raw);
    if (codes) nid = batch_idx[r0];
  }
  // (VQGNN_ASG_DEFER_STORES) a row's index / code stores are issued in the
  // next iteration, after its row loads were waited for: gfx950 counts
  // stores and loads in one in-order counter, so stores issued right before
  // the loop's back edge made the wait for the prefetched row a wait for
  // their write acknowledgements as well
  bool st_do = false;
  int st_idx = 0, st_row = 0;
  int64_t st_node = 0;
  auto flush_stores = [&]() {
    if (st_do) {
      if (idx_out) idx_out[(int64_t)b * B + st_row] = (int64_t)st_idx;
      if (idx32) idx32[(int64_t)b * B + st_row] = st_idx;
      if (codes) codes[st_node * ldc + b] = (int16_t)st_idx;
    }
  };
  for (int it = 0; it < n_iters; ++it) {
    const int row0 = part_begin + it * RPI + wave * 64;
    // (VQGNN_ASG_TAIL_EXIT) a wave whose rows all lie past its part leaves
    // the row loop: the part's last iteration is partial (arxiv: 172 of 512
    // rows), and its dead waves would sweep clamped rows beside the live ones.
    // Not where the chunk-inner loop restages behind workgroup barriers.
    if constexpr (VQGNN_ASG_TAIL_EXIT != 0)
      if ((CO || nchunks == 1) && row0 >= part_end) break;
    const bool live = row0 + lane < part_end;
    float sx;
    half8 bop[4];
    float xr[8];                                      // the row: scores, resolve, EMA
    const int64_t node = nid;
    if constexpr (kRowPrio != 0) __builtin_amdgcn_s_setprio(kRowPrio);
    {
      float (&xv)[8] = xr;
      sx = row_vals(raw, xv);
      if (it + 1 < n_iters) {                         // in flight under the sweep
        const int rn = min(row0 + RPI + lane, part_end - 1);
        load_raw(rn, raw);
        if (codes) nid = batch_idx[rn];
      }
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const half2_t h = half2_t{(_Float16)xv[2 * i], (_Float16)xv[2 * i + 1]};
        const half2_t l = half2_t{(_Float16)__fsub_rn(xv[2 * i], (float)h[0]),
                                  (_Float16)__fsub_rn(xv[2 * i + 1], (float)h[1])};
        hw[i] = __builtin_bit_cast(uint32_t, h);
        lw[i] = __builtin_bit_cast(uint32_t, l);
      }
      // quad 3: (1, 1, 1, |x|^2 + 1 split in three f16, 0, 0)
      const float c1 = __fadd_rn(sx, 1.f);
      const _Float16 c0 = (_Float16)c1;
      const float r1 = __fsub_rn(c1, (float)c0);
      const _Float16 cl = (_Float16)r1;
      const _Float16 cll = (_Float16)__fsub_rn(r1, (float)cl);
      const uint4 f3 = {0x3c003c00u, __builtin_bit_cast(uint32_t, half2_t{(_Float16)1.f, c0}),
                        __builtin_bit_cast(uint32_t, half2_t{cl, cll}), 0u};
      // lane (q, j)'s B fragment for group g is part q of row (g, j) (x_hi for
      // quads 0 and 1, x_lo for 2, the quad-3 parts for 3): per dword, a
      // 4 x 4 transpose over (quad, group) of (x_hi, x_hi, x_lo, quad 3) --
      // permlane swaps, no LDS round trip
      const uint32_t f3w[4] = {f3.x, f3.y, f3.z, f3.w};
      uint32_t bw[4][4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t r[4] = {hw[d], hw[d], lw[d], f3w[d]};
        transpose_quads(r);
#pragma unroll
        for (int g = 0; g < 4; ++g) bw[g][d] = r[g];
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
        bop[g] = __builtin_bit_cast(half8, uint4{bw[g][0], bw[g][1], bw[g][2], bw[g][3]});
    }
    if constexpr (kRowPrio != 0) __builtin_amdgcn_s_setprio(0);
    if constexpr (VQGNN_ASG_DEFER_STORES != 0) {    // the previous iteration's outputs
      flush_stores();
      st_do = false;
    }
    float best = INFINITY;
    int bidx = 0;
    bool ntie = !(sx < 65536.f);
    if (co && co_pass > 0 && live) {                  // the earlier chunks' result
      const unsigned long long st = co_state[(int64_t)b * B + row0 + lane];
      best = __uint_as_float((uint32_t)(st >> 32));
      bidx = (int)((uint32_t)st & 0x7fffffffu);
      ntie = ((uint32_t)st >> 31) != 0;
    }

    for (int ch = CO ? co_pass : 0; ch < (CO ? co_pass + 1 : nchunks); ++ch) {
      const int mc0 = ch * chunk;
      const int mcount = min(chunk, M - mc0);
      if (nchunks > 1 && !CO) {
        __syncthreads();
        stage_filter<NT>(E, ldw, W, mc0, mcount, chunk, lds, tid, &s_bigmin, ef);
        __syncthreads();
      }
      uint32_t cb[4], s2[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        cb[g] = 0xffffffffu;
        s2[g] = 0xffffffffu;
      }
      const char* ap = lds + a_lane;
      const int mlim = min(mcount, m_sweep);
      // the pair index rides in the low bits of each pair minimum (the score's
      // last pb bits are replaced: |change| < 2^pb ulp, paid for in the
      // acceptance margin below), so min() keeps the earliest pair of equal
      // minima without a compare-and-select per pair
      const int npair = (mlim + 31) >> 5;
      const uint32_t pmask = npair > 1 ? (2u << (31 - __builtin_clz((uint32_t)npair - 1))) - 1 : 0u;
      const floatx4 zero = {0.f, 0.f, 0.f, 0.f};
      auto ld_a = [&](int off) { return *reinterpret_cast<const half8*>(ap + off); };
      auto sweep_pair = [&](const half8 a0, const half8 a1, int p) {
        if constexpr (WM != 0) {
          // both tiles' eight MFMAs issue back to back into their own
          // accumulators, then the VALU folds them (sched_group_barrier:
          // without it the compiler reads each MFMA's result right after it,
          // in two accumulator sets, and waits out every MFMA's latency in
          // s_nop).  arxiv assign -2.5 %, arxiv_gat -1..3 %, ppi -3 %
          // (profiles/r04s_sweep_schedule_ab.txt); 121 VGPRs at 8 waves, 128
          // at 16.
          floatx4 d0[4], d1[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) d0[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bop[g], zero, 0, 0, 0);
#pragma unroll
          for (int g = 0; g < 4; ++g) d1[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bop[g], zero, 0, 0, 0);
          // the fold at raised wave priority: a wave whose MFMA results are
          // in gets its VALU issued first and returns to the matrix pipe
          // sooner (arxiv_gat assign 220-224 against 234-236 us, ppi 540-542
          // against 562-566, arxiv 86-88 against 89.5-90;
          // profiles/r06t_setprio_ab.txt; raised while issuing the MFMAs
          // instead: no gain, r06s_assign_setprio_ab.txt)
          __builtin_amdgcn_s_setprio(kFoldPrio);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            // by value: clang's __builtin_bit_cast of a vector-element
            // subscript reads element 0 (ROCm 7.2's clang)
            uint32_t mm = min(min(__float_as_uint(d0[g][0]), __float_as_uint(d0[g][1])),
                              min(__float_as_uint(d0[g][2]), __float_as_uint(d0[g][3])));
            mm = min(min(mm, __float_as_uint(d1[g][0])), __float_as_uint(d1[g][1]));
            mm = min(min(mm, __float_as_uint(d1[g][2])), __float_as_uint(d1[g][3]));
            const uint32_t mt = and_or_u32(mm, ~pmask, (uint32_t)p);
            s2[g] = umed3(mt, cb[g], s2[g]);            // min(s2, max(mt, cb)): cb <= s2
            cb[g] = min(mt, cb[g]);                     // equal scores: the earliest pair
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);    // the 8 MFMAs first
          __builtin_amdgcn_sched_group_barrier(0x002, 40, 0);   // then the VALU
          __builtin_amdgcn_s_setprio(0);
        } else {   // WM 0 (any W): one tile's accumulators at a time (> 128 VGPRs otherwise)
          uint32_t m4[4];
          {
            floatx4 d[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) d[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bop[g], zero, 0, 0, 0);
#pragma unroll
            for (int g = 0; g < 4; ++g)
              m4[g] = min(min(__float_as_uint(d[g][0]), __float_as_uint(d[g][1])),
                          min(__float_as_uint(d[g][2]), __float_as_uint(d[g][3])));
          }
          __builtin_amdgcn_sched_barrier(0);
          {
            floatx4 d[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) d[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bop[g], zero, 0, 0, 0);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              // a chain, not a tree: two v_min3_u32
              uint32_t mm = min(min(m4[g], __float_as_uint(d[g][0])), __float_as_uint(d[g][1]));
              mm = min(min(mm, __float_as_uint(d[g][2])), __float_as_uint(d[g][3]));
              const uint32_t mt = and_or_u32(mm, ~pmask, (uint32_t)p);
              s2[g] = umed3(mt, cb[g], s2[g]);
              cb[g] = min(mt, cb[g]);
            }
          }
        }
      };
      // each wave loads the next pair's A fragments under this pair's MFMAs,
      // two register sets in turn (the kFltSlack codewords past the chunk
      // absorb the read one pair past the last).  It fits 4 waves per SIMD
      // (<= 128 VGPRs), which is what both workgroup shapes reach anyway (2
      // 8-wave or 1 16-wave workgroups per CU); WM 0 instances would not fit.
      constexpr bool kPrefetchA = WM != 0;
      if constexpr (kPrefetchA) {
        half8 x0 = ld_a(0), x1 = ld_a(256);
        for (int p = 0; mlim > 0; p += 2, ap += 1024) {
          const half8 y0 = ld_a(512), y1 = ld_a(768);
          sweep_pair(x0, x1, p);
          if ((p + 1) * 32 >= mlim) break;
          x0 = ld_a(1024);
          x1 = ld_a(1280);
          sweep_pair(y0, y1, p + 1);
          if ((p + 2) * 32 >= mlim) break;
        }
      } else {
        for (int p = 0; p * 32 < mlim; ++p, ap += 512) sweep_pair(ld_a(0), ld_a(256), p);
      }
      // ---- hand the owner lane the four quads' statistics of its row: a
      // 4 x 4 transpose over (quad, group); keys carry their quad (index order
      // = pair, then quad)
      if constexpr (VQGNN_ASG_RES_PRIO != 0) __builtin_amdgcn_s_setprio(VQGNN_ASG_RES_PRIO);
      uint32_t kk[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) kk[g] = ((cb[g] & pmask) << 2) | (uint32_t)q;
      transpose_quads(cb);
      transpose_quads(s2);
      transpose_quads(kk);
      // ---- resolve (owner lane)
      const uint32_t rmin = min(min(cb[0], cb[1]), min(cb[2], cb[3]));
      uint32_t key = 0xffffffffu;
#pragma unroll
      for (int t = 0; t < 4; ++t) key = min(key, cb[t] == rmin ? kk[t] : 0xffffffffu);
      uint32_t sec = 0xffffffffu;                     // smallest score outside the 8 candidates
#pragma unroll
      for (int t = 0; t < 4; ++t) sec = min(sec, kk[t] == key ? s2[t] : cb[t]);
      const float fmin = __uint_as_float(rmin);
      const float fsec = __uint_as_float(sec);
      const float tmin = fmin - (sx + 1.f);
      // + the pair-index bits: each of fmin, fsec is within pmask ulp
      // (<= pmask * 2^-23 * value) of its score, so 2 (pmask + 1) 2^-23 fsec
      // covers both
      const float delta = (978.f * sx + 390.f * fabsf(tmin) + 489.f) * 5.9604645e-8f +
                          (float)(pmask + 1) * 2.3841858e-7f * fsec;
      bool exact_ok = (fsec - fmin > delta) && (delta < 0.25f);
      const unsigned int bigm = s_bigmin;
      if (bigm != 0x7f800000u) {                      // out-of-range codewords staged
        // v_sqrt_f32 (1 ulp): the 1e-4 margin below covers it
        const float r = __builtin_amdgcn_sqrtf(__uint_as_float(bigm)) - __builtin_amdgcn_sqrtf(sx);
        exact_ok = exact_ok && r > 0.f && r * r * 0.9999f > fmin + delta;
      }
      // the 8 candidates (winning pair pw, quad qw: codewords pw*32 + 16t +
      // 4qw + r) in the reference arithmetic, in index order: strict < keeps
      // the first index of a tie
      const int pw = (int)(key >> 2), qw = (int)(key & 3);
      float dm = INFINITY;
      int im = 0;
      if (ef) {
        // staged f32 k-planes: each run of 4 candidates is one float4 per
        // plane, the four dot chains advance together (k order per chain)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int m0 = pw * 32 + t * 16 + 4 * qw;
          const int p0 = flt_pos(m0);
          float d4[4];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if (k < W) {
              const float4 ek = *reinterpret_cast<const float4*>(ef + k * cs + p0);
              const float ev[4] = {ek.x, ek.y, ek.z, ek.w};
#pragma unroll
              for (int c = 0; c < 4; ++c)
                d4[c] = (k == 0) ? __fmul_rn(ev[c], xr[k]) : fmaf(ev[c], xr[k], d4[c]);
            }
          }
          const float4 s4 = *reinterpret_cast<const float4*>(sef + p0);
          const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
          float dq[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) dq[c] = fmaf(-2.f, d4[c], __fadd_rn(sx, sv[c]));
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int ci = m0 + c;
            const float dd = ci < mcount ? dq[c] : INFINITY;
            if (dd < dm) {
              dm = dd;
              im = ci;
            }
          }
        }
      } else {
#pragma unroll 2
      for (int c = 0; c < 8; ++c) {
        const int ci = pw * 32 + (c >> 2) * 16 + 4 * qw + (c & 3);
        const bool cv = ci < mcount;
        const float* er = E + (int64_t)(mc0 + (cv ? ci : 0)) * ldw;
        float e[8];
        if (vec_rows && W > 4) {
          const float4 t0 = *reinterpret_cast<const float4*>(er);
          const float4 t1 = *reinterpret_cast<const float4*>(er + 4);
          e[0] = t0.x; e[1] = t0.y; e[2] = t0.z; e[3] = t0.w;
          e[4] = t1.x; e[5] = t1.y; e[6] = t1.z; e[7] = t1.w;
        } else if (vec_rows && W == 4) {
          const float4 t0 = *reinterpret_cast<const float4*>(er);
          e[0] = t0.x; e[1] = t0.y; e[2] = t0.z; e[3] = t0.w;
          e[4] = e[5] = e[6] = e[7] = 0.f;
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) e[k] = k < W ? er[k] : 0.f;
        }
        float dot = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (k < W) dot = (k == 0) ? __fmul_rn(e[k], xr[k]) : fmaf(e[k], xr[k], dot);
        const float se_c = sef[cv ? flt_pos(ci) : 0];
        const float dd = cv ? fmaf(-2.f, dot, __fadd_rn(sx, se_c)) : INFINITY;
        if (dd < dm) {
          dm = dd;
          im = ci;
        }
      }
      }
      if constexpr (VQGNN_ASG_RES_PRIO != 0) __builtin_amdgcn_s_setprio(0);
      if (dm < best) {                                // earlier chunk wins ties
        best = dm;
        bidx = mc0 + im;
      }
      ntie = ntie || (!exact_ok && m_sweep >= mcount);
    }
    if (co && co_pass + 1 < nchunks) {                // not the last chunk: carry the state
      if (live)
        co_state[(int64_t)b * B + row0 + lane] =
            ((unsigned long long)__float_as_uint(best) << 32) | ((uint32_t)ntie << 31) |
            (uint32_t)bidx;
      continue;
    }

    // ---- outputs (owner lane); a near-tie row is appended to the
    // workgroup's list instead (resolved after the row loop)
    const bool near_tie = live && ntie;
    if constexpr (VQGNN_ASG_OUT_PRIO != 0) __builtin_amdgcn_s_setprio(VQGNN_ASG_OUT_PRIO);
    if constexpr (VQGNN_ASG_DEFER_STORES != 0) {
      st_do = live && !ntie;
      st_idx = bidx;
      st_row = row0 + lane;
      st_node = node;
    } else if (live && !ntie) {
      if (idx_out) idx_out[(int64_t)b * B + row0 + lane] = (int64_t)bidx;
      if (idx32) idx32[(int64_t)b * B + row0 + lane] = bidx;
      if (codes) codes[node * ldc + b] = (int16_t)bidx;
    }
    const uint64_t am = __ballot(near_tie);
    if (am) {                                         // wave-uniform
      int base = 0;
      if (lane == 0) base = atomicAdd(&s_nflag, __popcll(am));
      base = __shfl(base, 0);
      if (near_tie) flist[base + __popcll(am & ((1ull << lane) - 1))] = row0 + lane;
    }
    if constexpr (FUSED) {
      if (live && !ntie) {
        unsigned long long* a = acc + bidx * (W + 1);
        atomicAdd(a, 1ull);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (k < W) atomicAdd(a + 1 + k, to_fixed(xr[k], (W != D && k >= D) ? shift_g : shift_f));
      }
    }
    if constexpr (VQGNN_ASG_OUT_PRIO != 0) __builtin_amdgcn_s_setprio(0);
  }

  if constexpr (VQGNN_ASG_DEFER_STORES != 0) flush_stores();   // the last iteration's outputs

  // ---- near-tie rows of this workgroup: one wave per row sweeps every
  // codeword in vq.py's arithmetic (BatchNorm apply, |x|^2 and |e|^2 summed
  // in k order, the k-ordered dot, fma(-2, dot, |x|^2 + |e|^2)) and takes the
  // lexicographic (distance, index) minimum -- torch.argmin's first index
  __syncthreads();
  const int n_near = s_nflag;
  for (int i = wave; i < n_near; i += WV) {
    const int row = flist[i];
    float xv[8];
    float sxr = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = 0.f;
      if (k < W) {
        const bool gk = W != D && k >= D;
        const int c = b * D + (gk ? k - D : k);
        const float raw = gk ? Gr[(int64_t)row * ldg + c] : X[(int64_t)row * ldx + c];
        // the k-slot table (with the BatchNorm fold, coef is written by part
        // 0's workgroups of this same launch: only s_kt is this one's)
        v = __fmul_rn(fmaf(__fsub_rn(raw, s_kt[2][k]), s_kt[0][k], s_kt[1][k]), s_kt[3][k]);
        sxr = (k == 0) ? __fmul_rn(v, v) : __fadd_rn(sxr, __fmul_rn(v, v));
      }
      xv[k] = v;
    }
    float bd = INFINITY;
    int bm = 0x7fffffff;
    for (int m = lane; m < M; m += 64) {
      const float* er = E + (int64_t)m * ldw;
      float dot = 0.f, se_m = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (k < W) {
          const float ek = er[k];
          dot = (k == 0) ? __fmul_rn(ek, xv[k]) : fmaf(ek, xv[k], dot);
          se_m = (k == 0) ? __fmul_rn(ek, ek) : __fadd_rn(se_m, __fmul_rn(ek, ek));
        }
      }
      const float dd = fmaf(-2.f, dot, __fadd_rn(sxr, se_m));
      if (dd < bd) {                                  // increasing m: the first index stays
        bd = dd;
        bm = m;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {               // lexicographic (d, m) minimum
      const float od = __shfl_xor(bd, o);
      const int om = __shfl_xor(bm, o);
      if (od < bd || (od == bd && om < bm)) {
        bd = od;
        bm = om;
      }
    }
    if (lane == 0) {
      if (idx_out) idx_out[(int64_t)b * B + row] = (int64_t)bm;
      if (idx32) idx32[(int64_t)b * B + row] = bm;
      if (codes) codes[batch_idx[row] * ldc + b] = (int16_t)bm;
    }
    if constexpr (FUSED) {
      unsigned long long* a = acc + bm * (W + 1);
      if (lane == 0) atomicAdd(a, 1ull);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < W && lane == k)
          atomicAdd(a + 1 + k, to_fixed(xv[k], (W != D && k >= D) ? shift_g : shift_f));
    }
  }

  if constexpr (FUSED) {   // fold into the single zeroed slab: integer, exact, order-free
    __syncthreads();
    unsigned long long* out = partial + (int64_t)b * M * (W + 1);
    // (VQGNN_ASG_NO_FLUSH: a timing probe without this fold, results invalid)
    if constexpr (VQGNN_ASG_NO_FLUSH == 0)
      for (int i = tid; i < M * (W + 1); i += NT)
        if (acc[i]) atomicAdd(out + i, acc[i]);
  }
}

// Separate EMA statistics (codebook too large to share the LDS with the
// accumulators): int64 fixed-point LDS accumulators for the whole codebook of
// one branch; rows re-read and re-normalised.  use_lds == 0: global int64
// atomics into partial (caller zeroes it; single slab).
__global__ void __launch_bounds__(kAssignThreads)
vq_ema_partial_kernel(const float* __restrict__ X, int64_t ldx,
                      const float* __restrict__ Gr, int64_t ldg,
                      int B, int nb, int D, int M, int W,
                      const float* __restrict__ coef, float grad_scale,
                      const int* __restrict__ idx32, unsigned long long* __restrict__ partial,
                      int rows_per_part, int use_lds, int shift_f, int shift_g) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long smem64[];
  const int F = nb * D;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wg % nb;
  const int part = wg / nb;
  const int tid = threadIdx.x;
  unsigned long long* acc = use_lds ? smem64 : (partial + (int64_t)b * M * (W + 1));
  if (use_lds) {
    for (int i = tid; i < M * (W + 1); i += kAssignThreads) acc[i] = 0ull;
    __syncthreads();
  }
  const int row_begin = part * rows_per_part;
  const int row_end = min(B, row_begin + rows_per_part);
  const int slots = W + 1;
  const int rows_per_pass = kAssignThreads / slots;
  const int rph = tid / slots, k1 = tid % slots;
  if (rph < rows_per_pass) {
    for (int r = row_begin + rph; r < row_end; r += rows_per_pass) {
      const int m = idx32[(int64_t)b * B + r];
      unsigned long long* a = acc + m * (W + 1);
      if (k1 == 0) {
        atomicAdd(a, 1ull);
      } else {
        const int k = k1 - 1;
        const bool g = k >= D;
        const int c = g ? b * D + (k - D) : b * D + k;
        const float raw = g ? Gr[(int64_t)r * ldg + c] : X[(int64_t)r * ldx + c];
        float v = fmaf(__fsub_rn(raw, coef[(g ? 5 * F : 4 * F) + c]), coef[(g ? 2 * F : 0) + c],
                       coef[(g ? 3 * F : F) + c]);
        if (g) v = __fmul_rn(v, grad_scale);
        atomicAdd(a + k1, to_fixed(v, g ? shift_g : shift_f));
      }
    }
  }
  if (use_lds) {
    __syncthreads();
    unsigned long long* out = partial + (int64_t)b * M * (W + 1);
    for (int i = tid; i < M * (W + 1); i += kAssignThreads)
      if (acc[i]) atomicAdd(out + i, acc[i]);
  }
}

// Split EMA statistics for a slab larger than the LDS (ppi: M = 4096, W = 8:
// 295 KB per branch).  Workgroup = (branch, codeword range h of M / H, row
// part): the range's slab sits in LDS; a thread takes one row per pass,
// reads its index and, when it falls in the range, the row's W values, then
// adds the count and the fixed-point values with ds_add_u64.  Indices are read
// by every range (B ints per branch per range), row values once overall.  The
// LDS slab is folded into the global one with int64 atomics: integer, exact,
// order-free, so the result equals vq_ema_partial_kernel's.
constexpr int kSplitThreads = 1024;
constexpr size_t kSplitSlab = 80 * 1024;      // two workgroups per CU

__global__ void __launch_bounds__(kSplitThreads)
vq_ema_split_kernel(const float* __restrict__ X, int64_t ldx,
                    const float* __restrict__ Gr, int64_t ldg,
                    int B, int nb, int D, int M, int W,
                    const float* __restrict__ coef, float grad_scale,
                    const int* __restrict__ idx32, unsigned long long* __restrict__ partial,
                    int H, int mrange, int rows_per_part, int shift_f, int shift_g) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long smem64[];
  const int F = nb * D;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wg % nb;
  const int h = (wg / nb) % H;
  const int part = wg / (nb * H);
  const int tid = threadIdx.x;
  const int slots = W + 1;
  const int m0 = h * mrange, m1 = min(M, m0 + mrange);
  for (int i = tid; i < (m1 - m0) * slots; i += kSplitThreads) smem64[i] = 0ull;
  __syncthreads();
  const int row_begin = part * rows_per_part;
  const int row_end = min(B, row_begin + rows_per_part);
  const int* idx = idx32 + (int64_t)b * B;
  const bool vec4 = D == 4 && (W == 4 || W == 8) && (ldx & 3) == 0 &&
                    ((uintptr_t)X & 15) == 0 &&
                    (W == 4 || ((ldg & 3) == 0 && ((uintptr_t)Gr & 15) == 0));
  int r = row_begin + tid;
  int m = r < row_end ? idx[r] : -1;
  for (; r < row_end; r += kSplitThreads) {
    const int rn = r + kSplitThreads;
    const int mn = rn < row_end ? idx[rn] : -1;       // next pass's index, in flight
    if (m >= m0 && m < m1) {
      unsigned long long* a = smem64 + (m - m0) * slots;
      atomicAdd(a, 1ull);
      if (vec4) {                          // D = 4: both halves as one float4 load each
        float v[8];
        const float4 xv = *reinterpret_cast<const float4*>(X + (int64_t)r * ldx + b * 4);
        v[0] = xv.x; v[1] = xv.y; v[2] = xv.z; v[3] = xv.w;
        if (W == 8) {
          const float4 gv = *reinterpret_cast<const float4*>(Gr + (int64_t)r * ldg + b * 4);
          v[4] = gv.x; v[5] = gv.y; v[6] = gv.z; v[7] = gv.w;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k >= W) break;
          const bool g = k >= 4;
          const int c = b * 4 + (k & 3);
          float t = fmaf(__fsub_rn(v[k], coef[(g ? 5 * F : 4 * F) + c]), coef[(g ? 2 * F : 0) + c],
                         coef[(g ? 3 * F : F) + c]);
          if (g) t = __fmul_rn(t, grad_scale);
          atomicAdd(a + 1 + k, to_fixed(t, g ? shift_g : shift_f));
        }
        m = mn;
        continue;
      }
      for (int k = 0; k < W; ++k) {
        const bool g = k >= D;
        const int c = g ? b * D + (k - D) : b * D + k;
        const float raw = g ? Gr[(int64_t)r * ldg + c] : X[(int64_t)r * ldx + c];
        float v = fmaf(__fsub_rn(raw, coef[(g ? 5 * F : 4 * F) + c]), coef[(g ? 2 * F : 0) + c],
                       coef[(g ? 3 * F : F) + c]);
        if (g) v = __fmul_rn(v, grad_scale);
        atomicAdd(a + 1 + k, to_fixed(v, g ? shift_g : shift_f));
      }
    }
    m = mn;
  }
  __syncthreads();
  unsigned long long* out = partial + ((int64_t)b * M + m0) * slots;
  for (int i = tid; i < (m1 - m0) * slots; i += kSplitThreads)
    if (smem64[i]) atomicAdd(out + i, smem64[i]);
}

// out[i] = sum over parts of parts[p][i] (integer: exact, order-free)
__global__ void vq_ema_reduce_kernel(const long long* __restrict__ parts, int nparts,
                                     int64_t per_part, long long* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per_part) return;
  long long s = parts[i];
  for (int p = 1; p < nparts; ++p) s += parts[(int64_t)p * per_part + i];
  out[i] = s;
}

// ---------------------------------------------------------------------------
// 4. EMA finalize: one workgroup per branch.        vq.py:177-200, :242-277
// ---------------------------------------------------------------------------
// (kFinThreads, EmaFin and the body: ema_finalize.h, shared with the
// aggregation's fix-up launch, vqgnn_spmm_task_cb_fin)
__global__ void __launch_bounds__(kFinThreads)
vq_ema_finalize_kernel(EmaFin f) {
  extern __shared__ float cs_s[];            // [M]
  ema_finalize_branch(f, blockIdx.x, threadIdx.x, cs_s);
}

// Large codebooks (M >= 1024): the per-codeword half of the finalize spread
// over (branch, 256-codeword slice) workgroups once vq_ema_finalize_kernel
// (split = 1) has written the branch's cluster sizes.  A branch with an
// empty cluster is skipped (the finalize flagged it and cleared its slab).
// Same operations per element as the single-kernel form.
constexpr int kApplyThreads = 256;
constexpr int kApplySlice = 256;

__global__ void __launch_bounds__(kApplyThreads)
vq_ema_apply_kernel(long long* __restrict__ stats, int nparts, int64_t part_stride,
                    int zero_after, int shift_f, int shift_g, int M, int D, int W, int ldw,
                    float decay, float grad_scale, float epsilon,
                    const float* __restrict__ cluster_size, int64_t cs_bstride,
                    float* __restrict__ ema_w, float* __restrict__ emb,
                    float* __restrict__ emb_out, int64_t emb_bstride,
                    const float* __restrict__ rm_f, const float* __restrict__ rv_f,
                    const float* __restrict__ rm_g, const float* __restrict__ rv_g) {
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const float* cs = cluster_size + (int64_t)b * cs_bstride;
  int zero = 0;
  for (int m = tid; m < M; m += kApplyThreads) zero |= cs[m] == 0.f;
  if (__syncthreads_or(zero)) return;
  long long* st = stats + (int64_t)b * M * (W + 1);
  auto stat = [&](int64_t i, int shift) {
    long long v = st[i];
    if (zero_after) st[i] = 0;
    for (int p = 1; p < nparts; ++p) {
      v += st[(int64_t)p * part_stride + i];
      if (zero_after) st[(int64_t)p * part_stride + i] = 0;
    }
    return (float)ldexp((double)v, -shift);
  };
  float* ew = ema_w + (int64_t)b * emb_bstride;
  float* e = emb + (int64_t)b * emb_bstride;
  float* eo = emb_out + (int64_t)b * emb_bstride;
  const float one_m_decay = (float)(1.0 - (double)decay);
  const int m0 = blockIdx.x * kApplySlice, m1 = min(M, m0 + kApplySlice);
  for (int i = m0 * W + tid; i < m1 * W; i += kApplyThreads) {
    const int m = i / W, k = i % W;
    const int64_t o = (int64_t)m * ldw + k;
    const float dw = stat((int64_t)m * (W + 1) + 1 + k, k < D ? shift_f : shift_g);
    const float w = __fadd_rn(__fmul_rn(ew[o], decay), __fmul_rn(one_m_decay, dw));
    ew[o] = w;
    const float ev = __fdiv_rn(w, cs[m]);
    e[o] = ev;
    float out;
    if (k < D) {
      const float sd = sqrtf(__fadd_rn(rv_f[b * D + k], 1e-5f));
      out = __fadd_rn(__fmul_rn(ev, sd), rm_f[b * D + k]);
    } else {
      const int kg = k - D;
      const float div = (float)((double)grad_scale + (double)epsilon);
      const float sd = sqrtf(__fadd_rn(rv_g[b * D + kg], epsilon));
      out = __fadd_rn(__fmul_rn(__fdiv_rn(ev, div), sd), rm_g[b * D + kg]);
      if (grad_scale == 0.f) out = __fmul_rn(out, 0.f);
    }
    eo[o] = out;
  }
}

}  // namespace vqgnn

// ===========================================================================
// C-ABI
// ===========================================================================
using namespace vqgnn;

// ATen-arithmetic workspace layout (after the FP64 partials): superblock
// sums [C][nsb] f32, P and Q [C][nsb] f64, tail [C] f32, CONTIG chunk
// buffers 2 x [T][C] f32.
constexpr int kMaxRefThreads = 1024;

struct CascadeGeom {
  int lp, nsb;
};

static CascadeGeom cascade_geom(int B) {
  int cl = 0;
  while ((int64_t(1) << cl) < (int64_t)B) ++cl;     // CeilLog2
  CascadeGeom g;
  g.lp = std::max(4, cl / 4);
  const int64_t sbrows = int64_t(1) << (2 * g.lp);
  g.nsb = (int)(((int64_t)B + sbrows - 1) / sbrows);
  if (g.nsb < 1) g.nsb = 1;
  return g;
}

static size_t fp64_ws_bytes(int B, int F) {
  const int C4 = (2 * F + 3) / 4;  // worst case with grads
  return align_up((size_t)stats_chunks(B, C4) * 2 * C4 * 4 * sizeof(double), 256);
}

static size_t aten_ws_bytes(int B, int F) {
  const int C = 2 * F;
  const CascadeGeom g = cascade_geom(B);
  size_t s = align_up((size_t)C * g.nsb * sizeof(float), 256);
  s += 2 * align_up((size_t)C * g.nsb * sizeof(double), 256);
  s += align_up((size_t)C * sizeof(float), 256);
  s += 2 * align_up((size_t)kMaxRefThreads * C * sizeof(float), 256);
  return s;
}

// the cascade arithmetic's workspace: superblock sums, fp64 (P, Q), tails,
// the CONTIG chunk buffers
struct CascadeWs {
  float* sb_sum;
  double* sb_p;
  double* sb_q;
  float* tail;
  float* cb0;
  float* cb1;
};

static CascadeWs cascade_ws(void* workspace, int C, const CascadeGeom& g) {
  CascadeWs ws;
  char* w = reinterpret_cast<char*>(workspace);
  ws.sb_sum = reinterpret_cast<float*>(w);
  w += align_up((size_t)C * g.nsb * sizeof(float), 256);
  ws.sb_p = reinterpret_cast<double*>(w);
  w += align_up((size_t)C * g.nsb * sizeof(double), 256);
  ws.sb_q = reinterpret_cast<double*>(w);
  w += align_up((size_t)C * g.nsb * sizeof(double), 256);
  ws.tail = reinterpret_cast<float*>(w);
  w += align_up((size_t)C * sizeof(float), 256);
  ws.cb0 = reinterpret_cast<float*>(w);
  w += align_up((size_t)kMaxRefThreads * C * sizeof(float), 256);
  ws.cb1 = reinterpret_cast<float*>(w);
  return ws;
}

static void launch_cascade_partial(const float* X, int64_t ldx, const float* G, int64_t ldg,
                                   int B, int F, int C, const CascadeGeom& g, const CascadeWs& ws,
                                   hipStream_t s) {
  const int ntiles = (C + 63) / 64;
  hipLaunchKernelGGL(bn_cascade_partial_kernel, dim3(g.nsb * ntiles), dim3(kCasWaves * 64), 0, s,
                     X, ldx, G, ldg, B, F, C, g.lp, g.nsb, ntiles, ws.sb_sum, ws.sb_p, ws.sb_q,
                     ws.tail);
}

extern "C" size_t vqgnn_bn_stats_workspace(int32_t B, int32_t F) {
  return std::max(fp64_ws_bytes(B, F), aten_ws_bytes(B, F));
}

static int bn_stats_launch(const float* X, int64_t ldx, const float* G, int64_t ldg, int32_t B,
                           int32_t F, int32_t with_grad, double* sums, double* tail,
                           void* workspace, vqgnn_stream_t stream) {
  VQGNN_REQUIRE(X && sums && workspace, "bn_stats: null pointer");
  VQGNN_REQUIRE(B > 0 && F > 0 && ldx >= F, "bn_stats: bad shape B=%d F=%d ldx=%lld", B, F,
                (long long)ldx);
  VQGNN_REQUIRE(!with_grad || (G && ldg >= F), "bn_stats: grads required");
  const bool vec = F % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X & 15) == 0 &&
                   (!with_grad || (ldg % 4 == 0 && ((uintptr_t)G & 15) == 0));
  const int C = with_grad ? 2 * F : F;
  const int C4 = (C + 3) / 4;
  const int chunks = stats_chunks(B, C4);
  const int rpc = (B + chunks - 1) / chunks;
  double* part = reinterpret_cast<double*>(workspace);
  hipStream_t s = as_stream(stream);
  if (vec) {
    hipLaunchKernelGGL(bn_stats_partial_kernel, dim3(chunks), dim3(kStatsThreads), 0, s, X, ldx,
                       G, ldg, B, F / 4, C4, rpc, part);
  } else {
    hipLaunchKernelGGL(bn_stats_partial_scalar_kernel, dim3(chunks), dim3(kStatsThreads), 0, s,
                       X, ldx, G, ldg, B, F, C, rpc, part);
  }
  hipLaunchKernelGGL(bn_stats_reduce_kernel, dim3((2 * C + kReduceWaves - 1) / kReduceWaves),
                     dim3(kReduceWaves * 64), 0, s, part,
                     chunks, F, C, sums, tail, (double)B);
  return check_launch("bn_stats");
}

extern "C" int vqgnn_bn_stats(const float* X, int64_t ldx, const float* G, int64_t ldg,
                              int32_t B, int32_t F, int32_t with_grad, double* sums,
                              void* workspace, vqgnn_stream_t stream) {
  clear_error();
  return bn_stats_launch(X, ldx, G, ldg, B, F, with_grad, sums, nullptr, workspace, stream);
}

extern "C" int vqgnn_bn_stats_count(const float* X, int64_t ldx, const float* G, int64_t ldg,
                                    int32_t B, int32_t F, int32_t with_grad, double* sums,
                                    void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(sums, "bn_stats_count: null pointer");
  return bn_stats_launch(X, ldx, G, ldg, B, F, with_grad, sums, sums + 4 * (int64_t)F,
                         workspace, stream);
}

static BnArgs bn_args(int mode, int arith_x, int arith_g, double mom_f, double eps_f,
                      double mom_g, double eps_g, double eps_std, float* rm_f, float* rv_f,
                      float* rm_g, float* rv_g, float* coef, float* batch_out, int64_t* nbt_f,
                      int64_t* nbt_g, int nbt_d) {
  BnArgs a;
  a.mode = mode;
  a.arith_x = arith_x;
  a.arith_g = arith_g;
  a.mom_f = mom_f;
  a.eps_f = eps_f;
  a.mom_g = mom_g;
  a.eps_g = eps_g;
  a.eps_std = eps_std;
  a.rm_f = rm_f;
  a.rv_f = rv_f;
  a.rm_g = rm_g;
  a.rv_g = rv_g;
  a.coef = coef;
  a.batch_out = batch_out;
  a.nbt_f = reinterpret_cast<long long*>(nbt_f);
  a.nbt_g = reinterpret_cast<long long*>(nbt_g);
  a.D = nbt_d;
  return a;
}

static bool arith_ok(int a) { return a == kBnFp64 || a == kBnStrided || a == kBnContig; }

extern "C" int vqgnn_bn_finalize(const double* sums, int64_t count, int32_t F, int32_t with_grad,
                                 int32_t mode, int32_t arith_x, int32_t arith_g,
                                 double momentum_f, double eps_f, double momentum_g,
                                 double eps_g, double eps_std, float* rm_f, float* rv_f,
                                 float* rm_g, float* rv_g, float* coef, float* batch_out,
                                 int64_t* nbt_f, int64_t* nbt_g, int32_t nbt_d,
                                 vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(F > 0 && coef && rm_f && rv_f, "bn_finalize: bad arguments");
  VQGNN_REQUIRE(mode >= 0 && mode <= 3, "bn_finalize: mode must be 0..3");
  VQGNN_REQUIRE(arith_ok(arith_x) && arith_ok(arith_g), "bn_finalize: bad arithmetic code");
  VQGNN_REQUIRE(mode == 0 || sums, "bn_finalize: sums required");
  VQGNN_REQUIRE(!with_grad || (rm_g && rv_g), "bn_finalize: grad running stats required");
  // batch statistics from fp64 sums follow the FP64 arithmetic; the eval
  // coefficients take the form of the requested path
  const bool batch = mode != 0;
  const BnArgs a = bn_args(mode, batch ? kBnFp64 : arith_x, batch ? kBnFp64 : arith_g,
                           momentum_f, eps_f, momentum_g, eps_g, eps_std, rm_f, rv_f, rm_g,
                           rv_g, coef, batch_out, nbt_f, nbt_g, nbt_d);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((F + 255) / 256), dim3(256), 0, as_stream(stream),
                     sums, count, F, with_grad, a);
  return check_launch("bn_finalize");
}

extern "C" int vqgnn_bn_stats_finalize(const float* X, int64_t ldx, const float* G, int64_t ldg,
                                       int32_t B, int32_t F, int32_t with_grad, double* sums,
                                       int32_t mode, int32_t arith_x, int32_t arith_g,
                                       int32_t ref_threads, double momentum_f, double eps_f,
                                       double momentum_g, double eps_g, double eps_std,
                                       float* rm_f, float* rv_f, float* rm_g, float* rv_g,
                                       float* coef, float* batch_out, int64_t* nbt_f,
                                       int64_t* nbt_g, int32_t nbt_d, void* workspace,
                                       vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(X && coef && rm_f && rv_f && workspace, "bn_stats_finalize: null pointer");
  VQGNN_REQUIRE(B > 0 && F > 0 && ldx >= F, "bn_stats_finalize: bad shape B=%d F=%d", B, F);
  VQGNN_REQUIRE(B <= (1 << 23), "bn_stats_finalize: B=%d rows exceed 2^23", B);
  VQGNN_REQUIRE(mode >= 0 && mode <= 3, "bn_stats_finalize: mode must be 0..3");
  VQGNN_REQUIRE(!with_grad || (G && ldg >= F && rm_g && rv_g), "bn_stats_finalize: grads required");
  VQGNN_REQUIRE(arith_ok(arith_x) && arith_ok(arith_g), "bn_stats_finalize: bad arithmetic code");
  const bool contig = arith_x == kBnContig || (with_grad && arith_g == kBnContig);
  VQGNN_REQUIRE(!contig || (ref_threads >= 1 && ref_threads <= kMaxRefThreads),
                "bn_stats_finalize: ref_threads=%d outside 1..%d", ref_threads, kMaxRefThreads);
  const int C = with_grad ? 2 * F : F;
  const BnArgs a = bn_args(mode, arith_x, with_grad ? arith_g : kBnFp64, momentum_f, eps_f,
                           momentum_g, eps_g, eps_std, rm_f, rv_f, rm_g, rv_g, coef, batch_out,
                           nbt_f, nbt_g, nbt_d);
  hipStream_t s = as_stream(stream);
  if (arith_x == kBnFp64 && (!with_grad || arith_g == kBnFp64)) {
    const bool vec = F % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X & 15) == 0 &&
                     (!with_grad || (ldg % 4 == 0 && ((uintptr_t)G & 15) == 0));
    const int C4 = (C + 3) / 4;
    const int chunks = stats_chunks(B, C4);
    const int rpc = (B + chunks - 1) / chunks;
    double* part = reinterpret_cast<double*>(workspace);
    if (vec) {
      hipLaunchKernelGGL(bn_stats_partial_kernel, dim3(chunks), dim3(kStatsThreads), 0, s, X,
                         ldx, G, ldg, B, F / 4, C4, rpc, part);
    } else {
      hipLaunchKernelGGL(bn_stats_partial_scalar_kernel, dim3(chunks), dim3(kStatsThreads), 0,
                         s, X, ldx, G, ldg, B, F, C, rpc, part);
    }
    hipLaunchKernelGGL(bn_reduce_finalize_kernel, dim3((C + 31) / 32), dim3(kRfThreads), 0, s,
                       part, chunks, F, C, sums, (int64_t)B, a);
    return check_launch("bn_stats_finalize");
  }
  VQGNN_REQUIRE(sums == nullptr, "bn_stats_finalize: fp64 sums exist only for the FP64 arithmetic");
  const CascadeGeom g = cascade_geom(B);
  const CascadeWs ws = cascade_ws(workspace, C, g);
  float* sb_sum = ws.sb_sum;
  double* sb_p = ws.sb_p;
  double* sb_q = ws.sb_q;
  float* tail = ws.tail;
  float* cb0 = ws.cb0;
  float* cb1 = ws.cb1;
  launch_cascade_partial(X, ldx, G, ldg, B, F, C, g, ws, s);
  int T = 1;
  if (contig) {
    // at::parallel_for(0, B, 1): min(T, B) threads of ceil(B / threads) rows
    T = std::min(ref_threads, B);
    const int chunk = (B + T - 1) / T;
    const dim3 grid((C + 255) / 256, T);
    hipLaunchKernelGGL(bn_contig_chunk_kernel, grid, dim3(256), 0, s, X, ldx, G, ldg, B, F, C,
                       arith_x, with_grad ? arith_g : kBnFp64, T, chunk, 0, nullptr, cb0);
    hipLaunchKernelGGL(bn_contig_chunk_kernel, grid, dim3(256), 0, s, X, ldx, G, ldg, B, F, C,
                       arith_x, with_grad ? arith_g : kBnFp64, T, chunk, 1, cb0, cb1);
  }
  const size_t fin_lds = (size_t)(g.nsb + (g.nsb >> g.lp) + 1) * sizeof(float);
  hipLaunchKernelGGL(bn_aten_finalize_kernel, dim3(C), dim3(64), fin_lds, s, X,
                     ldx, G, ldg, B, F, C, g.lp, g.nsb, sb_sum, sb_p, sb_q, tail, T, cb0, cb1, a);
  return check_launch("bn_stats_finalize");
}

extern "C" int32_t vqgnn_vq_ema_parts(int32_t B, int32_t nb, int32_t M, int32_t W) {
  // the workgroups fold their partial statistics into one slab (int64
  // atomics: exact); kept as a query so callers need not assume it
  return (B <= 0 || nb <= 0 || M <= 0 || W <= 0) ? 0 : 1;
}

// Workspace of vq_assign: [the non-fused EMA path's row indices][the
// filtered path's per-workgroup near-tie row lists: rows_per_part ints per
// workgroup]
static size_t idx32_bytes(const AssignGeom& g, int B, int nb) {
  return g.fused ? 256 : align_up((size_t)nb * B * sizeof(int), 256);
}
static size_t flag_bytes(const AssignGeom& g, int nb) {
  if (!g.filter) return 0;
  return align_up((size_t)g.parts * nb * g.rows_per_part * sizeof(int), 256);
}

// chunk-outer passes: one packed state word per (branch, row) -- the best
// exact distance so far (high 32 bits), the near-tie flag (bit 31), its index
static size_t co_bytes(const AssignGeom& g, int B, int nb) {
  return g.co ? align_up((size_t)nb * B * sizeof(unsigned long long), 256) : 0;
}

extern "C" size_t vqgnn_vq_assign_workspace(int32_t B, int32_t nb, int32_t M, int32_t W) {
  if (B <= 0 || nb <= 0 || M <= 0 || W <= 0) return 0;
  const AssignGeom g = assign_geom(B, nb, M, W);
  return idx32_bytes(g, B, nb) + flag_bytes(g, nb) + co_bytes(g, B, nb);
}

// Measurement facility for bench.py: while enabled, every vq_assign_kernel
// launch is issued with hipExtLaunchKernelGGL and a start/stop event pair, so
// its duration is the kernel's own (no gap before the launch, unlike events
// recorded around it on the stream).  Library-owned events, one mutex.
// The events skip the system-scope fence (hipEventDisableSystemFence): they
// only time, and are read after the caller's full synchronisation; a fenced
// event pair costs each step a cache write-back and invalidate before the
// assign and again before the next kernel (≈ 11 µs of idle GPU per arxiv
// step, profiles/r05r_event_fence_ab.txt).
static std::mutex g_timing_mu;
static bool g_timing_on = false;
static std::vector<std::pair<hipEvent_t, hipEvent_t>> g_timing_ev;

static void timing_events(hipEvent_t* a, hipEvent_t* b) {
  *a = *b = nullptr;
  std::lock_guard<std::mutex> lk(g_timing_mu);
  if (!g_timing_on) return;
  if (hipEventCreateWithFlags(a, hipEventDisableSystemFence) != hipSuccess ||
      hipEventCreateWithFlags(b, hipEventDisableSystemFence) != hipSuccess) {
    (void)hipGetLastError();
    *a = *b = nullptr;
    return;
  }
  g_timing_ev.emplace_back(*a, *b);
}

static int launch_ema_tail(const float* X, int64_t ldx, const float* G, int64_t ldg, int B,
                           int nb, int D, int M, int W, const float* coef, float grad_scale,
                           const int* idx32, unsigned long long* parts, const AssignGeom& g,
                           const StatShift& sh, hipStream_t s);

template <int KC>
static int launch_assign(const float* X, int64_t ldx, const float* G, int64_t ldg, int B,
                         int nb, int D, int M, int W, const float* coef, float grad_scale,
                         const float* emb, int ldw, int64_t emb_bstride, int64_t* idx_out,
                         int16_t* codes, int64_t ldc, const int64_t* batch_idx,
                         unsigned long long* parts, int ema_zeroed, int64_t stat_count,
                         void* workspace, hipStream_t s) {
  const AssignGeom g = assign_geom(B, nb, M, W);
  const StatShift sh = stat_shift(stat_count, grad_scale);
  const bool want_ema = parts != nullptr;
  const bool fused = want_ema && g.fused;
  int* idx32 = (want_ema && !g.fused) ? reinterpret_cast<int*>(workspace) : nullptr;
  size_t lds = cb_lds_bytes(KC, g.chunk);
  if (fused) lds += (size_t)M * (W + 1) * sizeof(unsigned long long);
  if (lds > kLdsBudget) {
    set_error("vq_assign: LDS %zu B exceeds 160 KiB (M=%d W=%d)", lds, M, W);
    return VQGNN_ERR_UNSUPPORTED;
  }
  const int wgs = g.parts * nb;
  const int wm = slot_mode(KC, W, D);
  if (want_ema && !ema_zeroed)
    (void)hipMemsetAsync(parts, 0, (size_t)nb * M * (W + 1) * sizeof(unsigned long long), s);
#define VQ_LAUNCH(FU, WMV, WVV)                                                               \
  do {                                                                                        \
    const void* fn = (const void*)vq_assign_kernel<KC, FU, WMV, WVV>;                         \
    if (lds > 64 * 1024)                                                                      \
      (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);    \
    hipEvent_t ev0 = nullptr, ev1 = nullptr;                                                  \
    timing_events(&ev0, &ev1);                                                                \
    hipExtLaunchKernelGGL((vq_assign_kernel<KC, FU, WMV, WVV>), dim3(wgs), dim3(WVV * 64),      \
                          (uint32_t)lds, s, ev0, ev1, 0, X, ldx, G, ldg, B, nb, D, M, W, coef, \
                          grad_scale, emb, ldw, emb_bstride, idx_out, codes, ldc, batch_idx,   \
                          idx32, parts, g.rows_per_part, g.chunk, sh.f, sh.g, m_sweep);       \
  } while (0)
#define VQ_LAUNCH_WV(FU, WMV)                                                                 \
  do {                                                                                        \
    if (g.wv == 16) VQ_LAUNCH(FU, WMV, 16);                                                   \
    else VQ_LAUNCH(FU, WMV, 8);                                                               \
  } while (0)
#define VQ_LAUNCH_WM(FU)                                                                      \
  do {                                                                                        \
    if (wm == 1) VQ_LAUNCH_WV(FU, 1);                                                         \
    else if (wm == 2) VQ_LAUNCH_WV(FU, 2);                                                    \
    else VQ_LAUNCH_WV(FU, 0);                                                                 \
  } while (0)
  // codewords swept per chunk: all (VQGNN_ASSIGN_MSWEEP, experiments builds
  // only: a profiling knob that shortens the sweep and breaks the results)
  static const int msw_env = VQGNN_KNOB("VQGNN_ASSIGN_MSWEEP", -1);
  const int m_sweep = msw_env >= 0 ? msw_env : (1 << 30);
  if (fused) VQ_LAUNCH_WM(true); else VQ_LAUNCH_WM(false);
#undef VQ_LAUNCH_WM
#undef VQ_LAUNCH_WV
#undef VQ_LAUNCH
  int rc = check_launch("vq_assign");
  if (rc || !want_ema || fused) return rc;
  return launch_ema_tail(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, idx32, parts, g, sh, s);
}

// EMA statistics after an assign that could not fuse them (row indices in
// idx32): one workgroup per (branch, part) with an LDS slab, or the split
// kernel when the slab exceeds the LDS
static int launch_ema_tail(const float* X, int64_t ldx, const float* G, int64_t ldg, int B,
                           int nb, int D, int M, int W, const float* coef, float grad_scale,
                           const int* idx32, unsigned long long* parts, const AssignGeom& g,
                           const StatShift& sh, hipStream_t s) {
  const int wgs = g.parts * nb;
  const size_t acc_bytes = (size_t)M * (W + 1) * sizeof(unsigned long long);
  if (acc_bytes <= kLdsBudget) {
    if (acc_bytes > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)vq_ema_partial_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)acc_bytes);
    hipLaunchKernelGGL(vq_ema_partial_kernel, dim3(wgs), dim3(kAssignThreads), acc_bytes, s, X,
                       ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, idx32, parts,
                       g.rows_per_part, 1, sh.f, sh.g);
  } else if (!path_env("VQGNN_EMA_GLOBAL", 0)) {
    // codeword ranges whose slab fits kSplitSlab; enough row parts for
    // about two workgroups per CU
    const size_t slot_bytes = (size_t)(W + 1) * sizeof(unsigned long long);
    const int mrange = (int)std::max<size_t>(1, kSplitSlab / slot_bytes);
    const int H = (M + mrange - 1) / mrange;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int want = 2 * ncu;
    int rparts = std::max(1, (want + nb * H - 1) / (nb * H));
    rparts = std::min(rparts, std::max(1, B / kSplitThreads));
    const int rpp = (B + rparts - 1) / rparts;
    const size_t slab = (size_t)mrange * slot_bytes;
    if (slab > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)vq_ema_split_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)slab);
    hipLaunchKernelGGL(vq_ema_split_kernel, dim3(nb * H * rparts), dim3(kSplitThreads), slab, s,
                       X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, idx32, parts, H, mrange,
                       rpp, sh.f, sh.g);
  } else {  // global atomics (measurement reference: VQGNN_EMA_GLOBAL=1)
    hipLaunchKernelGGL(vq_ema_partial_kernel, dim3(wgs), dim3(kAssignThreads), 0, s, X, ldx, G,
                       ldg, B, nb, D, M, W, coef, grad_scale, idx32, parts, g.rows_per_part, 0,
                       sh.f, sh.g);
  }
  return check_launch("vq_ema_partial");
}


// Filtered path (W <= 8): vq_filter_kernel (near-tie rows included).
static int launch_filter(const float* X, int64_t ldx, const float* G, int64_t ldg, int B, int nb,
                         int D, int M, int W, const float* coef, float grad_scale,
                         const float* emb, int ldw, int64_t emb_bstride, int64_t* idx_out,
                         int16_t* codes, int64_t ldc, const int64_t* batch_idx,
                         unsigned long long* parts, int ema_zeroed, int64_t stat_count,
                         void* workspace, hipStream_t s, const BnFold* bn_fold = nullptr) {
  const AssignGeom g = assign_geom(B, nb, M, W);
  const StatShift sh = stat_shift(stat_count, grad_scale);
  const bool want_ema = parts != nullptr;
  const bool fused = want_ema && g.fused;
  const BnFold fold = bn_fold ? *bn_fold : BnFold{};
  int* idx32 = (want_ema && !g.fused) ? reinterpret_cast<int*>(workspace) : nullptr;
  int* flags = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) + idx32_bytes(g, B, nb));
  unsigned long long* co_state =
      g.co ? reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(workspace) +
                                                   idx32_bytes(g, B, nb) + flag_bytes(g, nb))
           : nullptr;
  // the geometry sized the slab in when the EMA statistics fuse; without
  // them the kernel does not touch it (the same LDS is reserved)
  size_t lds = g.lds;
  if (g.fused && !fused) lds -= (size_t)M * (W + 1) * sizeof(unsigned long long);
  if (lds > kLdsBudget) {
    set_error("vq_assign: LDS %zu B exceeds 160 KiB (M=%d W=%d)", lds, M, W);
    return VQGNN_ERR_UNSUPPORTED;
  }
  const int wgs = g.parts * nb;
  const int wm = flt_mode(W, D, ldx, ldg, X, G);
  if (want_ema && !ema_zeroed)
    (void)hipMemsetAsync(parts, 0, (size_t)nb * M * (W + 1) * sizeof(unsigned long long), s);
  static const int msw_env = VQGNN_KNOB("VQGNN_ASSIGN_MSWEEP", -1);
  const int m_sweep = msw_env >= 0 ? msw_env : (1 << 30);
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  timing_events(&ev0, &ev1);
  // chunk-outer: one launch per chunk (pass), the assign's timing events on
  // the first and the last; the BatchNorm fold only in the first (it
  // updates the running statistics and writes coef, which the later passes
  // read like an unfolded launch)
  const int npass = g.co ? (M + g.chunk - 1) / g.chunk : 1;
#define FLT_LAUNCH_CO(FU, WMV, WVV, COV)                                                      \
  do {                                                                                        \
    const void* fn = (const void*)vq_filter_kernel<FU, WMV, WVV, COV>;                        \
    if (lds > 64 * 1024)                                                                      \
      (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);    \
    for (int pass = 0; pass < npass; ++pass)                                                  \
      hipExtLaunchKernelGGL((vq_filter_kernel<FU, WMV, WVV, COV>), dim3(wgs), dim3(WVV * 64),   \
                            (uint32_t)lds, s, pass == 0 ? ev0 : nullptr,                      \
                            pass + 1 == npass ? ev1 : nullptr, 0, X, ldx, G, ldg, B, nb, D,   \
                            M, W, coef, grad_scale, emb, ldw, emb_bstride, idx_out, codes,    \
                            ldc, batch_idx, idx32, parts, flags, g.rows_per_part, g.chunk,    \
                            sh.f, sh.g, m_sweep, g.elds, pass == 0 ? fold : BnFold{},         \
                            co_state, pass);                                                  \
  } while (0)
#define FLT_LAUNCH(FU, WMV, WVV)                                                              \
  do {                                                                                        \
    if (!FU && g.co) FLT_LAUNCH_CO(false, WMV, WVV, true);                                    \
    else FLT_LAUNCH_CO(FU, WMV, WVV, false);                                                  \
  } while (0)
#define FLT_LAUNCH_WV(FU, WMV)                                                                \
  do {                                                                                        \
    if (g.wv == 16) FLT_LAUNCH(FU, WMV, 16);                                                  \
    else FLT_LAUNCH(FU, WMV, 8);                                                              \
  } while (0)
#define FLT_LAUNCH_WM(FU)                                                                     \
  do {                                                                                        \
    if (wm == 1) FLT_LAUNCH_WV(FU, 1);                                                        \
    else if (wm == 2) FLT_LAUNCH_WV(FU, 2);                                                   \
    else FLT_LAUNCH_WV(FU, 0);                                                                \
  } while (0)
  if (fused) FLT_LAUNCH_WM(true); else FLT_LAUNCH_WM(false);
#undef FLT_LAUNCH_WM
#undef FLT_LAUNCH_WV
#undef FLT_LAUNCH
#undef FLT_LAUNCH_CO
  const int rc = check_launch("vq_filter");
  if (rc || !want_ema || fused) return rc;
  return launch_ema_tail(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, idx32, parts, g, sh, s);
}

static int assign_check(const float* X, int64_t ldx, const float* G, int64_t ldg, int32_t B,
                        int32_t nb, int32_t D, int32_t M, int32_t W, const float* embedding,
                        int32_t ldw, int64_t emb_bstride, int16_t* codes, int64_t ldc,
                        const int64_t* batch_idx, int64_t* ema_parts, int64_t stat_count,
                        void* workspace);

extern "C" int vqgnn_vq_assign(const float* X, int64_t ldx, const float* G, int64_t ldg,
                               int32_t B, int32_t nb, int32_t D, int32_t M, int32_t W,
                               const float* coef, float grad_scale, const float* embedding,
                               int32_t ldw, int64_t emb_bstride, int64_t* idx_out,
                               int16_t* codes, int64_t ldc, const int64_t* batch_idx,
                               int64_t* ema_parts, int32_t ema_zeroed, int64_t stat_count,
                               void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(coef, "vq_assign: null pointer");
  const int rc = assign_check(X, ldx, G, ldg, B, nb, D, M, W, embedding, ldw, emb_bstride, codes,
                              ldc, batch_idx, ema_parts, stat_count, workspace);
  if (rc != VQGNN_OK) return rc;
  hipStream_t s = as_stream(stream);
  unsigned long long* parts = reinterpret_cast<unsigned long long*>(ema_parts);
  if (use_filter(W))
    return launch_filter(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, embedding, ldw,
                         emb_bstride, idx_out, codes, ldc, batch_idx, parts, ema_zeroed,
                         stat_count, workspace, s);
  const int kc = W <= 4 ? 1 : (W <= 8 ? 2 : 4);
  if (kc == 1)
    return launch_assign<1>(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, embedding, ldw,
                            emb_bstride, idx_out, codes, ldc, batch_idx, parts, ema_zeroed, stat_count,
                            workspace, s);
  if (kc == 2)
    return launch_assign<2>(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, embedding, ldw,
                            emb_bstride, idx_out, codes, ldc, batch_idx, parts, ema_zeroed, stat_count,
                            workspace, s);
  return launch_assign<4>(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, embedding, ldw,
                          emb_bstride, idx_out, codes, ldc, batch_idx, parts, ema_zeroed, stat_count,
                          workspace, s);
}

extern "C" int32_t vqgnn_vq_assign_bn_supported(int32_t B, int32_t nb, int32_t D, int32_t M,
                                                int32_t W) {
  if (B <= 1 || B > (1 << 23) || nb <= 0 || D <= 0 || M <= 0 || !(W == D || W == 2 * D) ||
      !use_filter(W))
    return 0;
  const AssignGeom g = assign_geom(B, nb, M, W);
  // a chunked codebook (chunk-outer passes, one launch each) is not folded:
  // its later passes would read the coef the first pass wrote, a combination
  // no parity test pins; the separate finalize serves it
  if (g.co) return 0;
  const CascadeGeom cg = cascade_geom(B);
  // the fold's scratch lives in the codebook planes' LDS before they are staged
  return bn_fold_scratch(cg.nsb, cg.lp, W) <= (size_t)kFltBytesPerCode * (g.chunk + kFltSlack)
             ? 1 : 0;
}

extern "C" int vqgnn_bn_stats_partial(const float* X, int64_t ldx, const float* G, int64_t ldg,
                                      int32_t B, int32_t F, int32_t with_grad, void* workspace,
                                      vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(X && workspace, "bn_stats_partial: null pointer");
  VQGNN_REQUIRE(B > 0 && F > 0 && ldx >= F, "bn_stats_partial: bad shape B=%d F=%d", B, F);
  VQGNN_REQUIRE(B <= (1 << 23), "bn_stats_partial: B=%d rows exceed 2^23", B);
  VQGNN_REQUIRE(!with_grad || (G && ldg >= F), "bn_stats_partial: grads required");
  const int C = with_grad ? 2 * F : F;
  const CascadeGeom g = cascade_geom(B);
  launch_cascade_partial(X, ldx, G, ldg, B, F, C, g, cascade_ws(workspace, C, g),
                         as_stream(stream));
  return check_launch("bn_stats_partial");
}

extern "C" int vqgnn_vq_assign_bn(const float* X, int64_t ldx, const float* G, int64_t ldg,
                                  int32_t B, int32_t nb, int32_t D, int32_t M, int32_t W,
                                  float grad_scale, const float* embedding, int32_t ldw,
                                  int64_t emb_bstride, int64_t* idx_out, int16_t* codes,
                                  int64_t ldc, const int64_t* batch_idx, int64_t* ema_parts,
                                  int32_t ema_zeroed, int64_t stat_count, void* workspace,
                                  const void* bn_workspace, int32_t mode, int32_t arith_x,
                                  int32_t arith_g, double momentum_f, double eps_f,
                                  double momentum_g, double eps_g, double eps_std, float* rm_f,
                                  float* rv_f, float* rm_g, float* rv_g, float* coef,
                                  float* batch_out, int64_t* nbt_f, int64_t* nbt_g,
                                  int32_t nbt_d, vqgnn_stream_t stream) {
  clear_error();
  const int rc = assign_check(X, ldx, G, ldg, B, nb, D, M, W, embedding, ldw, emb_bstride, codes,
                              ldc, batch_idx, ema_parts, stat_count, workspace);
  if (rc != VQGNN_OK) return rc;
  const bool with_grad = W == 2 * D;
  VQGNN_REQUIRE(vqgnn_vq_assign_bn_supported(B, nb, D, M, W),
                "vq_assign_bn: no fused BatchNorm fold for B=%d nb=%d M=%d W=%d "
                "(vqgnn_vq_assign_bn_supported)", B, nb, M, W);
  VQGNN_REQUIRE(bn_workspace && coef && rm_f && rv_f && (!with_grad || (rm_g && rv_g)),
                "vq_assign_bn: null pointer");
  VQGNN_REQUIRE(mode >= 0 && mode <= 3, "vq_assign_bn: mode must be 0..3");
  VQGNN_REQUIRE(arith_ok(arith_x) && arith_x != kBnContig &&
                    (!with_grad || (arith_ok(arith_g) && arith_g != kBnContig)),
                "vq_assign_bn: the cascade arithmetic (FP64 / STRIDED) only");
  // all-FP64 single-process statistics take vqgnn_bn_stats_finalize's fp64
  // sums, not the cascade: no fold of them here (same bits as that call only)
  VQGNN_REQUIRE(!(arith_x == kBnFp64 && (!with_grad || arith_g == kBnFp64)),
                "vq_assign_bn: all-FP64 statistics use vqgnn_bn_stats_finalize");
  const int F = nb * D;
  const int C = with_grad ? 2 * F : F;
  const CascadeGeom cg = cascade_geom(B);
  const CascadeWs ws = cascade_ws(const_cast<void*>(bn_workspace), C, cg);
  BnFold fold;
  fold.sb_sum = ws.sb_sum;
  fold.sb_p = ws.sb_p;
  fold.sb_q = ws.sb_q;
  fold.tail = ws.tail;
  fold.lp = cg.lp;
  fold.nsb = cg.nsb;
  fold.C = C;
  fold.a = bn_args(mode, arith_x, with_grad ? arith_g : kBnFp64, momentum_f, eps_f, momentum_g,
                   eps_g, eps_std, rm_f, rv_f, rm_g, rv_g, coef, batch_out, nbt_f, nbt_g, nbt_d);
  return launch_filter(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, embedding, ldw,
                       emb_bstride, idx_out, codes, ldc, batch_idx,
                       reinterpret_cast<unsigned long long*>(ema_parts), ema_zeroed, stat_count,
                       workspace, as_stream(stream), &fold);
}

static int assign_check(const float* X, int64_t ldx, const float* G, int64_t ldg, int32_t B,
                        int32_t nb, int32_t D, int32_t M, int32_t W, const float* embedding,
                        int32_t ldw, int64_t emb_bstride, int16_t* codes, int64_t ldc,
                        const int64_t* batch_idx, int64_t* ema_parts, int64_t stat_count,
                        void* workspace) {
  VQGNN_REQUIRE(X && embedding, "vq_assign: null pointer");
  VQGNN_REQUIRE(B > 0 && nb > 0 && D > 0 && M > 0, "vq_assign: bad shape");
  VQGNN_REQUIRE(W == D || W == 2 * D, "vq_assign: W must be D or 2D (W=%d D=%d)", W, D);
  VQGNN_REQUIRE(W <= 16, "vq_assign: W=%d > 16 not implemented", W);
  VQGNN_REQUIRE(ldx >= (int64_t)nb * D, "vq_assign: ldx too small");
  VQGNN_REQUIRE(W == D || (G && ldg >= (int64_t)nb * D), "vq_assign: grads required for W=2D");
  VQGNN_REQUIRE(ldw >= W && emb_bstride >= (int64_t)M * ldw, "vq_assign: bad codebook layout");
  VQGNN_REQUIRE(!codes || (batch_idx && ldc >= nb), "vq_assign: codes needs batch_idx, ldc>=nb");
  VQGNN_REQUIRE(workspace || (!ema_parts && !use_filter(W)),
                "vq_assign: workspace required (vqgnn_vq_assign_workspace)");
  VQGNN_REQUIRE(M <= 32767 || !codes, "vq_assign: int16 codes need M <= 32767");
  VQGNN_REQUIRE(!ema_parts || stat_count >= B, "vq_assign: stat_count < B");
  VQGNN_REQUIRE((int64_t)B * ldx * 4 < ((int64_t)1 << 32) &&
                    (!G || (int64_t)B * ldg * 4 < ((int64_t)1 << 32)),
                "vq_assign: B*ldx (and B*ldg) must span < 4 GiB");
  return VQGNN_OK;
}

extern "C" void vqgnn_vq_stat_shifts(int64_t stat_count, float grad_scale, int32_t* shift_f,
                                     int32_t* shift_g) {
  const StatShift sh = stat_shift(stat_count, grad_scale);
  if (shift_f) *shift_f = sh.f;
  if (shift_g) *shift_g = sh.g;
}

extern "C" int vqgnn_vq_ema_reduce(const int64_t* parts, int32_t nparts, int64_t part_elems,
                                   int64_t* out, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(parts && out && nparts > 0 && part_elems > 0, "ema_reduce: bad arguments");
  hipLaunchKernelGGL(vq_ema_reduce_kernel, dim3((part_elems + 255) / 256), dim3(256), 0,
                     as_stream(stream), reinterpret_cast<const long long*>(parts), nparts,
                     part_elems, reinterpret_cast<long long*>(out));
  return check_launch("ema_reduce");
}

namespace vqgnn {

int ema_fin_prepare(const vqgnn_ema_finalize_args* a, EmaFin* f) {
  VQGNN_REQUIRE(a, "ema_finalize: null arguments");
  VQGNN_REQUIRE(a->ema_parts && a->cluster_size && a->ema_w && a->embedding &&
                    a->embedding_output && a->bad_init,
                "ema_finalize: null pointer");
  VQGNN_REQUIRE(a->rm_f && a->rv_f, "ema_finalize: feature running stats required");
  VQGNN_REQUIRE(a->W == a->D || (a->W == 2 * a->D && a->rm_g && a->rv_g),
                "ema_finalize: W must be D or 2D");
  VQGNN_REQUIRE(a->nb > 0 && a->M > 0 && a->ldw >= a->W && a->nparts > 0,
                "ema_finalize: bad shape");
  VQGNN_REQUIRE(a->stat_count > 0, "ema_finalize: stat_count must be > 0");
  VQGNN_REQUIRE((size_t)a->M * 4 <= 136 * 1024, "ema_finalize: M=%d too large for the LDS", a->M);
  const StatShift sh = stat_shift(a->stat_count, a->grad_scale);
  EmaFin& e = *f;
  e.stats = reinterpret_cast<long long*>(a->ema_parts);
  e.nparts = a->nparts;
  e.part_stride = (int64_t)a->nb * a->M * (a->W + 1);
  e.zero_after = a->zero_after;
  e.shift_f = sh.f;
  e.shift_g = sh.g;
  e.M = a->M;
  e.D = a->D;
  e.W = a->W;
  e.ldw = a->ldw;
  e.decay = a->decay;
  e.laplace = a->laplace;
  e.grad_scale = a->grad_scale;
  e.epsilon = a->epsilon;
  e.cluster_size = a->cluster_size;
  e.cs_bstride = a->cs_bstride;
  e.ema_w = a->ema_w;
  e.emb = a->embedding;
  e.emb_out = a->embedding_output;
  e.emb_bstride = a->emb_bstride;
  e.rm_f = a->rm_f;
  e.rv_f = a->rv_f;
  e.rm_g = a->rm_g;
  e.rv_g = a->rv_g;
  e.bad_init = a->bad_init;
  // M >= 1024: the per-codeword half runs in a second, wider launch
  e.split = a->M >= 1024 && !VQGNN_KNOB("VQGNN_EMA_FIN_ONE", 0);
  return VQGNN_OK;
}

void ema_fin_lds_attr(const void* kernel) {
  (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 136 * 1024);
}

// the finalize's own launches (and the apply half when split)
static int ema_fin_launch(const EmaFin& f, int nb, hipStream_t s) {
  const size_t lds = (size_t)f.M * sizeof(float);
  if (lds > 48 * 1024) {
    static std::once_flag once;
    std::call_once(once, [] { ema_fin_lds_attr((const void*)vq_ema_finalize_kernel); });
  }
  hipLaunchKernelGGL(vq_ema_finalize_kernel, dim3(nb), dim3(kFinThreads), lds, s, f);
  if (f.split)
    hipLaunchKernelGGL(vq_ema_apply_kernel, dim3((f.M + kApplySlice - 1) / kApplySlice, nb),
                       dim3(kApplyThreads), 0, s, f.stats, f.nparts, f.part_stride,
                       f.zero_after, f.shift_f, f.shift_g, f.M, f.D, f.W, f.ldw, f.decay,
                       f.grad_scale, f.epsilon, f.cluster_size, f.cs_bstride, f.ema_w, f.emb,
                       f.emb_out, f.emb_bstride, f.rm_f, f.rv_f, f.rm_g, f.rv_g);
  return check_launch("ema_finalize");
}

int ema_fin_run(const EmaFin& f, int nb, hipStream_t s) { return ema_fin_launch(f, nb, s); }

}  // namespace vqgnn

extern "C" int vqgnn_vq_ema_finalize(int64_t* ema_parts, int32_t nparts, int32_t zero_after,
                                     int64_t stat_count, int32_t nb,
                                     int32_t M, int32_t D, int32_t W, int32_t ldw, float decay,
                                     int32_t laplace, float grad_scale, float epsilon,
                                     float* cluster_size, int64_t cs_bstride, float* ema_w,
                                     float* embedding, float* embedding_output,
                                     int64_t emb_bstride, const float* rm_f, const float* rv_f,
                                     const float* rm_g, const float* rv_g, int32_t* bad_init,
                                     vqgnn_stream_t stream) {
  clear_error();
  vqgnn_ema_finalize_args a{};
  a.ema_parts = ema_parts;
  a.nparts = nparts;
  a.zero_after = zero_after;
  a.stat_count = stat_count;
  a.nb = nb;
  a.M = M;
  a.D = D;
  a.W = W;
  a.ldw = ldw;
  a.decay = decay;
  a.laplace = laplace;
  a.grad_scale = grad_scale;
  a.epsilon = epsilon;
  a.cluster_size = cluster_size;
  a.cs_bstride = cs_bstride;
  a.ema_w = ema_w;
  a.embedding = embedding;
  a.embedding_output = embedding_output;
  a.emb_bstride = emb_bstride;
  a.rm_f = rm_f;
  a.rv_f = rv_f;
  a.rm_g = rm_g;
  a.rv_g = rv_g;
  a.bad_init = bad_init;
  EmaFin f{};
  const int rc = ema_fin_prepare(&a, &f);
  if (rc != VQGNN_OK) return rc;
  return ema_fin_run(f, nb, as_stream(stream));
}

extern "C" int vqgnn_assign_timing(int32_t enable) {
  std::lock_guard<std::mutex> lk(g_timing_mu);
  for (auto& e : g_timing_ev) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  g_timing_ev.clear();
  g_timing_on = enable != 0;
  return VQGNN_OK;
}

extern "C" int32_t vqgnn_assign_timing_read(float* ms, int32_t cap) {
  std::lock_guard<std::mutex> lk(g_timing_mu);
  int32_t n = 0;
  for (auto& e : g_timing_ev) {
    if (n >= cap) break;
    float t = 0.f;
    if (hipEventSynchronize(e.second) != hipSuccess ||
        hipEventElapsedTime(&t, e.first, e.second) != hipSuccess) {
      (void)hipGetLastError();
      t = -1.f;
    }
    ms[n++] = t;
  }
  return n;
}
