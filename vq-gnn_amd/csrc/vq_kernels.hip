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

#include <cfloat>
#include <cmath>

namespace vqgnn {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// 1. BatchNorm column statistics (fp64 sums)          vq.py:162, vq.py:223
// ---------------------------------------------------------------------------
constexpr int kStatsThreads = 256;
constexpr int kStatsMaxChunks = 1024;

static int stats_chunks(int B) {
  int c = (B + 255) / 256;
  return c < 1 ? 1 : (c > kStatsMaxChunks ? kStatsMaxChunks : c);
}

// Grid: chunks of rows.  Thread t handles column (t % C) for rows of phase t / C
// (C <= 256) or columns t, t+256, ... (C > 256).  Partials [chunk][2][C].
__global__ void __launch_bounds__(kStatsThreads)
bn_stats_partial_kernel(const float* __restrict__ X, int64_t ldx,
                        const float* __restrict__ G, int64_t ldg,
                        int B, int F, int C, int rows_per_chunk,
                        double* __restrict__ part) {
  __shared__ double red[2][kStatsThreads];
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(B, r0 + rows_per_chunk);
  double* out = part + (int64_t)blockIdx.x * 2 * C;
  if (C <= kStatsThreads) {
    const int phases = kStatsThreads / C;
    const int c = t % C, ph = t / C;
    double s = 0.0, s2 = 0.0;
    if (ph < phases) {
      const float* base = (c < F) ? (X + c) : (G + (c - F));
      const int64_t ld = (c < F) ? ldx : ldg;
      for (int r = r0 + ph; r < r1; r += phases) {
        const double v = (double)base[(int64_t)r * ld];
        s += v;
        s2 = fma(v, v, s2);
      }
    }
    red[0][t] = s;
    red[1][t] = s2;
    __syncthreads();
    if (t < C) {
      double a = 0.0, b = 0.0;
      for (int p = 0; p < phases; ++p) {
        a += red[0][p * C + t];
        b += red[1][p * C + t];
      }
      out[t] = a;
      out[C + t] = b;
    }
  } else {
    for (int c = t; c < C; c += kStatsThreads) {
      const float* base = (c < F) ? (X + c) : (G + (c - F));
      const int64_t ld = (c < F) ? ldx : ldg;
      double s = 0.0, s2 = 0.0;
      for (int r = r0; r < r1; ++r) {
        const double v = (double)base[(int64_t)r * ld];
        s += v;
        s2 = fma(v, v, s2);
      }
      out[c] = s;
      out[C + c] = s2;
    }
  }
}

// Sum partials in chunk order (deterministic) -> sums[4][F] (sx, sxx, sg, sgg).
__global__ void bn_stats_reduce_kernel(const double* __restrict__ part, int chunks,
                                       int F, int C, double* __restrict__ sums) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, b = 0.0;
  for (int p = 0; p < chunks; ++p) {
    a += part[(int64_t)p * 2 * C + c];
    b += part[(int64_t)p * 2 * C + C + c];
  }
  if (c < F) {
    sums[c] = a;
    sums[F + c] = b;
  } else {
    sums[2 * F + (c - F)] = a;
    sums[3 * F + (c - F)] = b;
  }
}

// ---------------------------------------------------------------------------
// 2. BatchNorm finalize (one thread per column)
//    ATen batch_norm_cpu_update_stats_template: mean/var in double
//    (acc_type<float, CPU> = double), invstd = 1/sqrt(var_biased + eps),
//    running = momentum*batch + (1-momentum)*running  (double, stored float),
//    running_var uses the unbiased variance.  Eval: invstd = 1/sqrtf(rv+eps)
//    in float (opmath).  beta = -(mean*alpha) in float.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void bn_column(double s, double s2, int64_t n, int mode,
                                          float momentum, float eps, float eps_std,
                                          float* rm, float* rv, float* alpha, float* beta,
                                          float* mean_out, float* std_out) {
  const bool train = (mode == 1 || mode == 2);
  const bool init = mode >= 2;
  const double nd = (double)n;
  double mean = 0.0, var_b = 0.0, var_u = 0.0;
  if (train || init) {
    mean = s / nd;
    double m2 = s2 - s * mean;            // sum (x - mean)^2
    if (m2 < 0.0) m2 = 0.0;
    var_b = m2 / nd;
    var_u = (n > 1) ? m2 / (nd - 1.0) : NAN;
    if (mean_out) *mean_out = (float)mean;
    if (std_out) *std_out = sqrtf(__fadd_rn((float)var_u, eps_std));
  }
  if (init) {  // vq.py:216-221: running stats <- torch.mean / torch.var(unbiased)
    *rm = (float)mean;
    *rv = (float)var_u;
  }
  if (!train) {  // BatchNorm1d eval: float invstd from the running stats
    const float invstd = 1.0f / sqrtf(__fadd_rn(*rv, eps));
    *alpha = invstd;
    *beta = -__fmul_rn(*rm, invstd);
    return;
  }
  const double mom = (double)momentum;
  *rm = (float)(mom * mean + (1.0 - mom) * (double)(*rm));
  *rv = (float)(mom * var_u + (1.0 - mom) * (double)(*rv));
  const float invstd = (float)(1.0 / sqrt(var_b + (double)eps));
  const float mean32 = (float)mean;
  *alpha = invstd;
  *beta = -__fmul_rn(mean32, invstd);
}

__global__ void bn_finalize_kernel(const double* __restrict__ sums, int64_t n, int F, int with_grad,
                                   int mode, float mom_f, float eps_f, float mom_g, float eps_g,
                                   float eps_std, float* rm_f, float* rv_f, float* rm_g,
                                   float* rv_g, float* __restrict__ coef,
                                   float* __restrict__ batch_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= F) return;
  bn_column(sums[c], sums[F + c], n, mode, mom_f, eps_f, eps_std, rm_f + c, rv_f + c,
            coef + c, coef + F + c, batch_out ? batch_out + c : nullptr,
            batch_out ? batch_out + F + c : nullptr);
  if (with_grad) {
    bn_column(sums[2 * F + c], sums[3 * F + c], n, mode, mom_g, eps_g, eps_std, rm_g + c,
              rv_g + c, coef + 2 * F + c, coef + 3 * F + c,
              batch_out ? batch_out + 2 * F + c : nullptr,
              batch_out ? batch_out + 3 * F + c : nullptr);
  }
}

// ---------------------------------------------------------------------------
// 3. PQ assignment on MFMA f32 (v_mfma_f32_16x16x4_f32)
//
// Workgroup = (branch b, row range); 4 waves, each wave owns 64 rows per
// iteration as 4 groups of 16.  MFMA tile: A = 16 codewords x 4 k (from LDS),
// B = 4 k x 16 rows (registers), D[16 codewords][16 rows]:
//   lane l: q = l>>4, j = l&15; A operand E[m0+j][kc*4+q], B operand
//   Xn[row j][kc*4+q]; D reg r = codeword m0 + 4q + r for row j.
// Per lane a running (best, index) over its codewords in increasing order with
// strict '<' keeps the first index; the 4 q-lanes of a row merge with
// (d, index) lexicographic order -> torch.argmin semantics (first index).
//
// LDS: codebook chunk as [q][m][KC] floats (q stride padded so the 16-lane
// halves of a ds_read hit disjoint banks), |e|^2 per codeword, and (fused EMA)
// the per-codeword count + sum of normalised x accumulated with ds_add.
// ---------------------------------------------------------------------------
constexpr int kAssignThreads = 256;
constexpr int kRowsPerIter = 256;      // 4 waves x 64 rows
constexpr int kTargetWgs = 2048;       // ~8 per CU
constexpr int kMaxChunk = 1024;        // codewords per LDS chunk
constexpr int kFuseEmaMaxM = 1024;     // fused EMA accumulators when M <= this

struct AssignGeom {
  int iters_per_wg;   // row iterations (256 rows each) per workgroup
  int ranges;         // row ranges per branch (= partial slabs)
  int wgs;            // total workgroups = ranges * nb
  int mpad;           // M rounded up to 16
  int chunk;          // codewords per LDS chunk (multiple of 16)
  int kc;             // k-chunks of 4 (W padded to 4*kc)
  bool fused;         // EMA statistics accumulated in the assign kernel
};

static AssignGeom assign_geom(int B, int nb, int M, int W) {
  AssignGeom g;
  const int row_blocks = (B + kRowsPerIter - 1) / kRowsPerIter;
  int target_ranges = (kTargetWgs + nb - 1) / nb;
  if (target_ranges < 1) target_ranges = 1;
  if (target_ranges > row_blocks) target_ranges = row_blocks;
  g.iters_per_wg = (row_blocks + target_ranges - 1) / target_ranges;
  g.ranges = (row_blocks + g.iters_per_wg - 1) / g.iters_per_wg;
  if (g.ranges < 1) g.ranges = 1;
  g.wgs = g.ranges * nb;
  g.mpad = (M + 15) / 16 * 16;
  g.chunk = g.mpad < kMaxChunk ? g.mpad : kMaxChunk;
  g.kc = W <= 4 ? 1 : (W <= 8 ? 2 : 4);
  g.fused = M <= kFuseEmaMaxM;
  return g;
}

template <int KC>
__host__ __device__ constexpr int q_pad_bytes() {
  return KC == 1 ? 64 : (KC == 2 ? 128 : 0);
}

template <int KC>
__host__ __device__ inline int q_stride_floats(int chunk) {
  return chunk * KC + q_pad_bytes<KC>() / 4;
}

template <int KC>
static size_t assign_lds_bytes(const AssignGeom& g, int M, int W) {
  size_t b = (size_t)4 * q_stride_floats<KC>(g.chunk) * 4;  // codebook chunk
  b += (size_t)g.chunk * 4;                                   // |e|^2
  if (g.fused) b += (size_t)M * (W + 1) * 4;                  // EMA accumulators
  return b;
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

__device__ __forceinline__ float pick4(const float (&a)[4], int i) {
  return i == 0 ? a[0] : (i == 1 ? a[1] : (i == 2 ? a[2] : a[3]));
}
__device__ __forceinline__ int pick4(const int (&a)[4], int i) {
  return i == 0 ? a[0] : (i == 1 ? a[1] : (i == 2 ? a[2] : a[3]));
}

template <int KC, bool FUSED>
__global__ void __launch_bounds__(kAssignThreads)
vq_assign_kernel(const float* __restrict__ X, int64_t ldx,
                 const float* __restrict__ Gr, int64_t ldg,
                 int B, int nb, int D, int M, int W,
                 const float* __restrict__ coef, float grad_scale,
                 const float* __restrict__ emb, int ldw, int64_t emb_bstride,
                 int64_t* __restrict__ idx_out, int16_t* __restrict__ codes, int64_t ldc,
                 const int64_t* __restrict__ batch_idx,
                 int* __restrict__ idx32, float* __restrict__ partial,
                 int iters_per_wg, int ranges, int chunk) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int F = nb * D;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wg % nb;
  const int range = wg / nb;
  const int qs = q_stride_floats<KC>(chunk);
  float* cb = smem;                       // [4][qs]
  float* se = smem + 4 * qs;              // [chunk]
  float* acc = se + chunk;                // [M][W+1] (FUSED)
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, j = lane & 15;
  const float* E = emb + (int64_t)b * emb_bstride;

  if constexpr (FUSED) {
    for (int i = tid; i < M * (W + 1); i += kAssignThreads) acc[i] = 0.f;
  }

  // per-column normalisation coefficients for this lane's k values
  float al[KC], be[KC];
  bool isg[KC], kval[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    const int k = kc * 4 + q;
    kval[kc] = k < W;
    isg[kc] = k >= D;
    const int c = isg[kc] ? (b * D + (k - D)) : (b * D + k);
    al[kc] = kval[kc] ? coef[(isg[kc] ? 2 * F : 0) + c] : 0.f;
    be[kc] = kval[kc] ? coef[(isg[kc] ? 3 * F : F) + c] : 0.f;
  }

  const int nchunks = (M + chunk - 1) / chunk;
  const int row_begin = range * iters_per_wg * kRowsPerIter;

  for (int it = 0; it < iters_per_wg; ++it) {
    const int row0 = row_begin + it * kRowsPerIter + wave * 64;
    // ---- load + normalise this wave's 64 rows (4 groups of 16) ----
    float xk[4][KC];
    float sx[4];
    bool rv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = row0 + g * 16 + j;
      rv[g] = row < B;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        float v = 0.f;
        if (rv[g] && kval[kc]) {
          const int k = kc * 4 + q;
          const float raw = isg[kc] ? Gr[(int64_t)row * ldg + b * D + (k - D)]
                                    : X[(int64_t)row * ldx + b * D + k];
          v = fmaf(raw, al[kc], be[kc]);        // BatchNorm1d (ATen: x*alpha+beta fused)
          if (isg[kc]) v = __fmul_rn(v, grad_scale);  // vq.py:224
        }
        xk[g][kc] = v;
      }
      // |x|^2 summed sequentially over k = 0..W-1 (torch.sum(x**2, dim=1))
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 4 * KC; ++k) {
        const float v = __shfl(xk[g][k >> 2], j + 16 * (k & 3));
        if (k < W) s = (k == 0) ? __fmul_rn(v, v) : __fadd_rn(s, __fmul_rn(v, v));
      }
      sx[g] = s;
    }

    float best[4];
    int bidx[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      best[g] = INFINITY;
      bidx[g] = 0;
    }

    for (int ch = 0; ch < nchunks; ++ch) {
      const int mc0 = ch * chunk;
      const int mcount = min(chunk, M - mc0);
      __syncthreads();
      // stage chunk: cb[q][m][kc] = E[mc0+m][kc*4+q] (0 beyond W / M), se[m]
      for (int m = tid; m < chunk; m += kAssignThreads) {
        float e[4 * KC];
        float s = 0.f;
        const bool mv = m < mcount;
#pragma unroll
        for (int k = 0; k < 4 * KC; ++k) {
          e[k] = (mv && k < W) ? E[(int64_t)(mc0 + m) * ldw + k] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 4 * KC; ++k)
          if (k < W) s = (k == 0) ? __fmul_rn(e[k], e[k]) : __fadd_rn(s, __fmul_rn(e[k], e[k]));
        se[m] = mv ? s : INFINITY;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
#pragma unroll
          for (int kc = 0; kc < KC; ++kc) cb[qq * qs + m * KC + kc] = e[kc * 4 + qq];
        }
      }
      __syncthreads();

      const float* cbq = cb + q * qs;
      for (int m0 = 0; m0 < mcount; m0 += 16) {
        const Frag<KC> a = lds_frag<KC>(cbq + (m0 + j) * KC);
        const float4 s4 = *reinterpret_cast<const float4*>(se + m0 + 4 * q);
        floatx4 d[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          d[g] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kc = 0; kc < KC; ++kc)
            d[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[kc], xk[g][kc], d[g], 0, 0, 0);
        }
        const int mb = mc0 + m0 + 4 * q;
        const float sev[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dist = fmaf(-2.f, d[g][r], __fadd_rn(sx[g], sev[r]));
            const bool take = dist < best[g];
            best[g] = take ? dist : best[g];
            bidx[g] = take ? (mb + r) : bidx[g];
          }
        }
      }
    }

    // ---- merge the 4 q-lanes of each row: (d, idx) lexicographic ----
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {
        const float od = __shfl_xor(best[g], off);
        const int oi = __shfl_xor(bidx[g], off);
        const bool take = (od < best[g]) || (od == best[g] && oi < bidx[g]);
        best[g] = take ? od : best[g];
        bidx[g] = take ? oi : bidx[g];
      }
    }

    // ---- outputs: lane (q, j) writes group q's row j ----
    {
      const int row = row0 + q * 16 + j;
      if (row < B) {
        const int m = pick4(bidx, q);
        if (idx_out) idx_out[(int64_t)b * B + row] = (int64_t)m;
        if (idx32) idx32[(int64_t)b * B + row] = m;
        if (codes) codes[batch_idx[row] * ldc + b] = (int16_t)m;
      }
    }

    if constexpr (FUSED) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (rv[g]) {
          float* a = acc + bidx[g] * (W + 1);
          if (q == 0) atomicAdd(a, 1.0f);
#pragma unroll
          for (int kc = 0; kc < KC; ++kc)
            if (kval[kc]) atomicAdd(a + 1 + kc * 4 + q, xk[g][kc]);
        }
      }
    }
  }

  if constexpr (FUSED) {
    __syncthreads();
    float* out = partial + ((int64_t)range * nb + b) * M * (W + 1);
    for (int i = tid; i < M * (W + 1); i += kAssignThreads) out[i] = acc[i];
  }
}

// Separate EMA statistics (M above the fused limit): LDS accumulators for the
// whole codebook of one branch; rows re-read and re-normalised.
template <int KC>
__global__ void __launch_bounds__(kAssignThreads)
vq_ema_partial_kernel(const float* __restrict__ X, int64_t ldx,
                      const float* __restrict__ Gr, int64_t ldg,
                      int B, int nb, int D, int M, int W,
                      const float* __restrict__ coef, float grad_scale,
                      const int* __restrict__ idx32, float* __restrict__ partial,
                      int iters_per_wg, int use_lds) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int F = nb * D;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wg % nb;
  const int range = wg / nb;
  const int tid = threadIdx.x;
  float* acc = use_lds ? smem : (partial + (int64_t)b * M * (W + 1));
  if (use_lds) {
    for (int i = tid; i < M * (W + 1); i += kAssignThreads) acc[i] = 0.f;
    __syncthreads();
  }
  const int row_begin = range * iters_per_wg * kRowsPerIter;
  const int row_end = min(B, row_begin + iters_per_wg * kRowsPerIter);
  // thread -> (row phase, k); W + 1 work slots per row (count + W values)
  for (int r = row_begin + tid / (W + 1); r < row_end; r += kAssignThreads / (W + 1)) {
    if (tid / (W + 1) >= kAssignThreads / (W + 1)) break;
    const int k1 = tid % (W + 1);
    const int m = idx32[(int64_t)b * B + r];
    float* a = acc + m * (W + 1);
    if (k1 == 0) {
      atomicAdd(a, 1.0f);
    } else {
      const int k = k1 - 1;
      const bool g = k >= D;
      const int c = g ? b * D + (k - D) : b * D + k;
      const float raw = g ? Gr[(int64_t)r * ldg + c] : X[(int64_t)r * ldx + c];
      float v = fmaf(raw, coef[(g ? 2 * F : 0) + c], coef[(g ? 3 * F : F) + c]);
      if (g) v = __fmul_rn(v, grad_scale);
      atomicAdd(a + k1, v);
    }
  }
  if (use_lds) {
    __syncthreads();
    float* out = partial + ((int64_t)range * nb + b) * M * (W + 1);
    for (int i = tid; i < M * (W + 1); i += kAssignThreads) out[i] = acc[i];
  }
}

// stats[b][m][c] = sum over ranges (in order) of partial[range][b][m][c]
__global__ void vq_ema_reduce_kernel(const float* __restrict__ partial, int ranges,
                                     int64_t per_range, float* __restrict__ stats) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per_range) return;
  float s = 0.f;
  for (int p = 0; p < ranges; ++p) s = __fadd_rn(s, partial[(int64_t)p * per_range + i]);
  stats[i] = s;
}

// ---------------------------------------------------------------------------
// 4. EMA finalize: one workgroup per branch.        vq.py:177-200, :242-277
// ---------------------------------------------------------------------------
constexpr int kFinThreads = 256;

__global__ void __launch_bounds__(kFinThreads)
vq_ema_finalize_kernel(const float* __restrict__ stats, int M, int D, int W, int ldw,
                       float decay, int laplace, float grad_scale, float epsilon,
                       float* __restrict__ cluster_size, int64_t cs_bstride,
                       float* __restrict__ ema_w, float* __restrict__ emb,
                       float* __restrict__ emb_out, int64_t emb_bstride,
                       const float* __restrict__ rm_f, const float* __restrict__ rv_f,
                       const float* __restrict__ rm_g, const float* __restrict__ rv_g,
                       int* __restrict__ bad_init) {
  __shared__ float red[kFinThreads];
  __shared__ int bad;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* st = stats + (int64_t)b * M * (W + 1);
  float* cs = cluster_size + (int64_t)b * cs_bstride;
  float* ew = ema_w + (int64_t)b * emb_bstride;
  float* e = emb + (int64_t)b * emb_bstride;
  float* eo = emb_out + (int64_t)b * emb_bstride;
  const float one_m_decay = (float)(1.0 - (double)decay);  // python (1 - decay) -> float scalar
  if (tid == 0) bad = 0;

  // cs = cs*decay + (1-decay)*counts  (vq.py:177-178; fp32 tensor ops)
  for (int m = tid; m < M; m += kFinThreads)
    cs[m] = __fadd_rn(__fmul_rn(cs[m], decay), __fmul_rn(one_m_decay, st[(int64_t)m * (W + 1)]));
  __syncthreads();

  if (laplace) {  // vq.py:182-186
    // n = torch.sum(cs): per-thread sequential partials over a strided slice,
    // then a fixed tree — deterministic (ATen's CPU cascade order differs by ulps)
    float s = 0.f;
    for (int m = tid; m < M; m += kFinThreads) s = __fadd_rn(s, cs[m]);
    red[tid] = s;
    __syncthreads();
    for (int w = kFinThreads / 2; w > 0; w >>= 1) {
      if (tid < w) red[tid] = __fadd_rn(red[tid], red[tid + w]);
      __syncthreads();
    }
    const float n = red[0];
    const float den = __fadd_rn(n, (float)((double)M * 1e-5));  // n + M*1e-5 (python float -> f32)
    for (int m = tid; m < M; m += kFinThreads)
      cs[m] = __fmul_rn(__fdiv_rn(__fadd_rn(cs[m], 1e-5f), den), n);
    __syncthreads();
  }

  for (int m = tid; m < M; m += kFinThreads)
    if (cs[m] == 0.f) bad = 1;  // vq.py:188 count_nonzero(cs) != M
  __syncthreads();
  if (bad) {  // reference raises before touching ema_w / embedding
    if (tid == 0) atomicOr(bad_init, 1);
    return;
  }

  // ema_w = ema_w*decay + (1-decay)*dw ; embedding = ema_w / cs ; output
  const int nw = M * W;
  for (int i = tid; i < nw; i += kFinThreads) {
    const int m = i / W, k = i % W;
    const int64_t o = (int64_t)m * ldw + k;
    const float dw = st[(int64_t)m * (W + 1) + 1 + k];
    const float w = __fadd_rn(__fmul_rn(ew[o], decay), __fmul_rn(one_m_decay, dw));
    ew[o] = w;
    const float ev = __fdiv_rn(w, cs[m]);
    e[o] = ev;
    float out;
    if (k < D) {  // vq.py:198-200 / :267-272 feature half: emb*sqrt(rv+1e-5)+rm
      const float sd = sqrtf(__fadd_rn(rv_f[b * D + k], 1e-5f));
      out = __fadd_rn(__fmul_rn(ev, sd), rm_f[b * D + k]);
    } else {      // vq.py:263 /= (scale + eps); :267 sqrt(rv_g + eps)
      const int kg = k - D;
      const float div = (float)((double)grad_scale + (double)epsilon);
      const float sd = sqrtf(__fadd_rn(rv_g[b * D + kg], epsilon));
      out = __fadd_rn(__fmul_rn(__fdiv_rn(ev, div), sd), rm_g[b * D + kg]);
      if (grad_scale == 0.f) out = __fmul_rn(out, 0.f);  // vq.py:274-275
    }
    eo[o] = out;
  }
}

}  // namespace vqgnn

// ===========================================================================
// C-ABI
// ===========================================================================
using namespace vqgnn;

extern "C" size_t vqgnn_bn_stats_workspace(int32_t B, int32_t F) {
  const int C = 2 * F;  // worst case with grads
  return align_up((size_t)stats_chunks(B) * 2 * C * sizeof(double), 256);
}

extern "C" int vqgnn_bn_stats(const float* X, int64_t ldx, const float* G, int64_t ldg,
                              int32_t B, int32_t F, int32_t with_grad, double* sums,
                              void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(X && sums && workspace, "bn_stats: null pointer");
  VQGNN_REQUIRE(B > 0 && F > 0 && ldx >= F, "bn_stats: bad shape B=%d F=%d ldx=%lld", B, F,
                (long long)ldx);
  VQGNN_REQUIRE(!with_grad || (G && ldg >= F), "bn_stats: grads required");
  const int C = with_grad ? 2 * F : F;
  const int chunks = stats_chunks(B);
  const int rpc = (B + chunks - 1) / chunks;
  double* part = reinterpret_cast<double*>(workspace);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(bn_stats_partial_kernel, dim3(chunks), dim3(kStatsThreads), 0, s, X, ldx,
                     G, ldg, B, F, C, rpc, part);
  hipLaunchKernelGGL(bn_stats_reduce_kernel, dim3((C + 255) / 256), dim3(256), 0, s, part,
                     chunks, F, C, sums);
  return check_launch("bn_stats");
}

extern "C" int vqgnn_bn_finalize(const double* sums, int64_t count, int32_t F, int32_t with_grad,
                                 int32_t mode, float momentum_f, float eps_f, float momentum_g,
                                 float eps_g, float eps_std, float* rm_f, float* rv_f,
                                 float* rm_g, float* rv_g, float* coef, float* batch_out,
                                 vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(F > 0 && coef && rm_f && rv_f, "bn_finalize: bad arguments");
  VQGNN_REQUIRE(mode >= 0 && mode <= 3, "bn_finalize: mode must be 0..3");
  VQGNN_REQUIRE(mode == 0 || (sums && count > 0), "bn_finalize: sums/count required");
  VQGNN_REQUIRE(!with_grad || (rm_g && rv_g), "bn_finalize: grad running stats required");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((F + 255) / 256), dim3(256), 0, as_stream(stream),
                     sums, count, F, with_grad, mode, momentum_f, eps_f, momentum_g, eps_g,
                     eps_std, rm_f, rv_f, rm_g, rv_g, coef, batch_out);
  return check_launch("bn_finalize");
}

extern "C" size_t vqgnn_vq_assign_workspace(int32_t B, int32_t nb, int32_t M, int32_t W) {
  if (B <= 0 || nb <= 0 || M <= 0 || W <= 0) return 0;
  const AssignGeom g = assign_geom(B, nb, M, W);
  size_t bytes = align_up((size_t)g.ranges * nb * M * (W + 1) * sizeof(float), 256);
  if (!g.fused) bytes += align_up((size_t)nb * B * sizeof(int), 256);
  return bytes;
}

template <int KC>
static int launch_assign(const float* X, int64_t ldx, const float* G, int64_t ldg, int B,
                         int nb, int D, int M, int W, const float* coef, float grad_scale,
                         const float* emb, int ldw, int64_t emb_bstride, int64_t* idx_out,
                         int16_t* codes, int64_t ldc, const int64_t* batch_idx, float* stats,
                         void* workspace, hipStream_t s) {
  const AssignGeom g = assign_geom(B, nb, M, W);
  const bool want_ema = stats != nullptr;
  float* partial = reinterpret_cast<float*>(workspace);
  int* idx32 = nullptr;
  if (want_ema && !g.fused) {
    idx32 = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) +
                                   align_up((size_t)g.ranges * nb * M * (W + 1) * sizeof(float), 256));
  }
  const bool fused = want_ema && g.fused;
  AssignGeom lg = g;
  lg.fused = fused;
  const size_t lds = assign_lds_bytes<KC>(lg, M, W);
  if (lds > 160 * 1024) {
    set_error("vq_assign: LDS %zu B exceeds 160 KiB (M=%d W=%d)", lds, M, W);
    return VQGNN_ERR_UNSUPPORTED;
  }
  if (lds > 64 * 1024) {
    (void)hipFuncSetAttribute(fused ? (const void*)vq_assign_kernel<KC, true>
                                    : (const void*)vq_assign_kernel<KC, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  }
  if (fused) {
    hipLaunchKernelGGL((vq_assign_kernel<KC, true>), dim3(g.wgs), dim3(kAssignThreads), lds, s,
                       X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, emb, ldw, emb_bstride,
                       idx_out, codes, ldc, batch_idx, idx32, partial, g.iters_per_wg, g.ranges,
                       g.chunk);
  } else {
    hipLaunchKernelGGL((vq_assign_kernel<KC, false>), dim3(g.wgs), dim3(kAssignThreads), lds, s,
                       X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, emb, ldw, emb_bstride,
                       idx_out, codes, ldc, batch_idx, idx32, partial, g.iters_per_wg, g.ranges,
                       g.chunk);
  }
  int rc = check_launch("vq_assign");
  if (rc || !want_ema) return rc;
  const int64_t per_range = (int64_t)nb * M * (W + 1);
  if (!fused) {
    const size_t acc_bytes = (size_t)M * (W + 1) * sizeof(float);
    const int use_lds = acc_bytes <= 160 * 1024;
    if (use_lds) {
      if (acc_bytes > 64 * 1024)
        (void)hipFuncSetAttribute((const void*)vq_ema_partial_kernel<KC>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)acc_bytes);
      hipLaunchKernelGGL((vq_ema_partial_kernel<KC>), dim3(g.wgs), dim3(kAssignThreads),
                         acc_bytes, s, X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, idx32,
                         partial, g.iters_per_wg, 1);
    } else {
      // global-atomic fallback straight into the stats buffer
      (void)hipMemsetAsync(stats, 0, per_range * sizeof(float), s);
      hipLaunchKernelGGL((vq_ema_partial_kernel<KC>), dim3(g.wgs), dim3(kAssignThreads), 0, s,
                         X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, idx32, stats,
                         g.iters_per_wg, 0);
      return check_launch("vq_ema_partial(global)");
    }
    rc = check_launch("vq_ema_partial");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(vq_ema_reduce_kernel, dim3((per_range + 255) / 256), dim3(256), 0, s,
                     partial, g.ranges, per_range, stats);
  return check_launch("vq_ema_reduce");
}

extern "C" int vqgnn_vq_assign(const float* X, int64_t ldx, const float* G, int64_t ldg,
                               int32_t B, int32_t nb, int32_t D, int32_t M, int32_t W,
                               const float* coef, float grad_scale, const float* embedding,
                               int32_t ldw, int64_t emb_bstride, int64_t* idx_out,
                               int16_t* codes, int64_t ldc, const int64_t* batch_idx,
                               float* ema_stats, void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(X && coef && embedding, "vq_assign: null pointer");
  VQGNN_REQUIRE(B > 0 && nb > 0 && D > 0 && M > 0, "vq_assign: bad shape");
  VQGNN_REQUIRE(W == D || W == 2 * D, "vq_assign: W must be D or 2D (W=%d D=%d)", W, D);
  VQGNN_REQUIRE(W <= 16, "vq_assign: W=%d > 16 not implemented", W);
  VQGNN_REQUIRE(ldx >= (int64_t)nb * D, "vq_assign: ldx too small");
  VQGNN_REQUIRE(W == D || (G && ldg >= (int64_t)nb * D), "vq_assign: grads required for W=2D");
  VQGNN_REQUIRE(ldw >= W && emb_bstride >= (int64_t)M * ldw, "vq_assign: bad codebook layout");
  VQGNN_REQUIRE(!codes || (batch_idx && ldc >= nb), "vq_assign: codes needs batch_idx, ldc>=nb");
  VQGNN_REQUIRE(!ema_stats || workspace, "vq_assign: workspace required for EMA statistics");
  VQGNN_REQUIRE(M <= 32767 || !codes, "vq_assign: int16 codes need M <= 32767");
  hipStream_t s = as_stream(stream);
  const int kc = W <= 4 ? 1 : (W <= 8 ? 2 : 4);
  if (kc == 1)
    return launch_assign<1>(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, embedding, ldw,
                            emb_bstride, idx_out, codes, ldc, batch_idx, ema_stats, workspace, s);
  if (kc == 2)
    return launch_assign<2>(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, embedding, ldw,
                            emb_bstride, idx_out, codes, ldc, batch_idx, ema_stats, workspace, s);
  return launch_assign<4>(X, ldx, G, ldg, B, nb, D, M, W, coef, grad_scale, embedding, ldw,
                          emb_bstride, idx_out, codes, ldc, batch_idx, ema_stats, workspace, s);
}

extern "C" int vqgnn_vq_ema_finalize(const float* ema_stats, int32_t nb, int32_t M, int32_t D,
                                     int32_t W, int32_t ldw, float decay, int32_t laplace,
                                     float grad_scale, float epsilon, float* cluster_size,
                                     int64_t cs_bstride, float* ema_w, float* embedding,
                                     float* embedding_output, int64_t emb_bstride,
                                     const float* rm_f, const float* rv_f, const float* rm_g,
                                     const float* rv_g, int32_t* bad_init,
                                     vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(ema_stats && cluster_size && ema_w && embedding && embedding_output && bad_init,
                "ema_finalize: null pointer");
  VQGNN_REQUIRE(rm_f && rv_f, "ema_finalize: feature running stats required");
  VQGNN_REQUIRE(W == D || (W == 2 * D && rm_g && rv_g), "ema_finalize: W must be D or 2D");
  VQGNN_REQUIRE(nb > 0 && M > 0 && ldw >= W, "ema_finalize: bad shape");
  hipLaunchKernelGGL(vq_ema_finalize_kernel, dim3(nb), dim3(kFinThreads), 0, as_stream(stream),
                     ema_stats, M, D, W, ldw, decay, laplace, grad_scale, epsilon, cluster_size,
                     cs_bstride, ema_w, embedding, embedding_output, emb_bstride, rm_f, rv_f,
                     rm_g, rv_g, bad_init);
  return check_launch("ema_finalize");
}
