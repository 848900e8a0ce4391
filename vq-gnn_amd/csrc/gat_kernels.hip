// GAT attention aggregation for gfx950 (MI355X).
//
// Reference: OurGATConv.forward / message (vq_gnn_v2/convs.py:165-266) with
// vq_softmax (utils/vq_softmax.py:33-57) and the normalisation in
// LowRankGNNLayer.forward (models.py:178-179, :187-189):
//   x_in      = [x ; x_first_order ; 1]            (n rows, C = F + 1 columns)
//   alpha_l   = x_in . att_l,  alpha_r = x_in . att_r              (:189-190)
//   s         = sqrt(max(alpha_l)^2 + 1) * sqrt(max(alpha_r)^2 + 1) (:209-211)
//   coef_e    = exp(leaky_relu(alpha_l[j]/s + alpha_r[i]/s, 0.2)) * w_e
//               (j = col = source, i = row = target; exp without max-shift,
//                no softmax normalisation: vq_softmax returns src.exp())
//   out[i]    = sum_e coef_e * x_in[j]     (segment_csr sum, CSR order)
//   rows < B: out[i][:F] /= out[i][F] + 1e-16   (the ones column = sum coef)
//
// The aggregation itself is the SpMM (spmm_kernels.hip) with coef as the
// edge values; this file adds the attention scalars, the coefficients with the
// per-row ones-column sum, the row normalisation, and the backward of the
// coefficient chain.

#include "common.h"

#include <cmath>

namespace vqgnn {

constexpr int kGatThreads = 256;
constexpr int kGatRowsPerWave = 4;

// alpha_l / alpha_r of n rows (one wave per kGatRowsPerWave rows, lanes over
// columns, fixed butterfly) and one (max_l, max_r) pair per block.
// Vector form (F % 4 == 0, 16-byte rows): half a wave per row, float4
// pieces, every row of the wave loaded before any sum (4 rows per wave);
// a 5-step butterfly inside each half.  Same per-block maxima.
__global__ void __launch_bounds__(kGatThreads)
gat_alpha4_kernel(const float* __restrict__ X, int64_t ldx, const float* __restrict__ X2,
                  int64_t ldx2, int B, int n, int F, int ones, const float* __restrict__ att_l,
                  const float* __restrict__ att_r, float* __restrict__ al, float* __restrict__ ar,
                  float* __restrict__ block_max) {
  __shared__ float red[2][kGatThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int F4 = F >> 2;
  const int base = (blockIdx.x * (kGatThreads / 64) + wave) * kGatRowsPerWave;
  float ml = -INFINITY, mr = -INFINITY;
  float sl[kGatRowsPerWave / 2], sr[kGatRowsPerWave / 2];
#pragma unroll
  for (int k = 0; k < kGatRowsPerWave / 2; ++k) {
    sl[k] = 0.f;
    sr[k] = 0.f;
  }
  for (int c4 = l32; c4 < F4; c4 += 32) {
    const float4 wl = reinterpret_cast<const float4*>(att_l)[c4];
    const float4 wr = reinterpret_cast<const float4*>(att_r)[c4];
    float4 v[kGatRowsPerWave / 2];
#pragma unroll
    for (int k = 0; k < kGatRowsPerWave / 2; ++k) {
      const int i = base + 2 * k + half;
      v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < n) {
        const float* row = i < B ? X + (int64_t)i * ldx : X2 + (int64_t)(i - B) * ldx2;
        v[k] = reinterpret_cast<const float4*>(row)[c4];
      }
    }
#pragma unroll
    for (int k = 0; k < kGatRowsPerWave / 2; ++k) {
      sl[k] = fmaf(v[k].w, wl.w, fmaf(v[k].z, wl.z, fmaf(v[k].y, wl.y, fmaf(v[k].x, wl.x, sl[k]))));
      sr[k] = fmaf(v[k].w, wr.w, fmaf(v[k].z, wr.z, fmaf(v[k].y, wr.y, fmaf(v[k].x, wr.x, sr[k]))));
    }
  }
#pragma unroll
  for (int k = 0; k < kGatRowsPerWave / 2; ++k) {
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) {
      sl[k] = __fadd_rn(sl[k], __shfl_xor(sl[k], off));
      sr[k] = __fadd_rn(sr[k], __shfl_xor(sr[k], off));
    }
    const int i = base + 2 * k + half;
    if (i < n) {
      if (ones) {  // the appended ones column is the last term of the sum
        sl[k] = __fadd_rn(sl[k], att_l[F]);
        sr[k] = __fadd_rn(sr[k], att_r[F]);
      }
      if (l32 == 0) {
        al[i] = sl[k];
        ar[i] = sr[k];
      }
      ml = fmaxf(ml, sl[k]);
      mr = fmaxf(mr, sr[k]);
    }
  }
  ml = fmaxf(ml, __shfl_xor(ml, 32));
  mr = fmaxf(mr, __shfl_xor(mr, 32));
  if (lane == 0) {
    red[0][wave] = ml;
    red[1][wave] = mr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = red[0][0], b = red[1][0];
    for (int w = 1; w < kGatThreads / 64; ++w) {
      a = fmaxf(a, red[0][w]);
      b = fmaxf(b, red[1][w]);
    }
    block_max[2 * blockIdx.x] = a;
    block_max[2 * blockIdx.x + 1] = b;
  }
}

__global__ void __launch_bounds__(kGatThreads)
gat_alpha_kernel(const float* __restrict__ X, int64_t ldx, const float* __restrict__ X2,
                 int64_t ldx2, int B, int n, int F, int ones, const float* __restrict__ att_l,
                 const float* __restrict__ att_r, float* __restrict__ al, float* __restrict__ ar,
                 float* __restrict__ block_max) {
  __shared__ float red[2][kGatThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ml = -INFINITY, mr = -INFINITY;
  for (int k = 0; k < kGatRowsPerWave; ++k) {
    const int i = (blockIdx.x * (kGatThreads / 64) + wave) * kGatRowsPerWave + k;
    if (i >= n) break;
    const float* row = i < B ? X + (int64_t)i * ldx : X2 + (int64_t)(i - B) * ldx2;
    float sl = 0.f, sr = 0.f;
    for (int c = lane; c < F; c += 64) {
      const float v = row[c];
      sl = __fadd_rn(sl, __fmul_rn(v, att_l[c]));
      sr = __fadd_rn(sr, __fmul_rn(v, att_r[c]));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      sl = __fadd_rn(sl, __shfl_xor(sl, off));
      sr = __fadd_rn(sr, __shfl_xor(sr, off));
    }
    if (ones) {  // the appended ones column is the last term of the sum
      sl = __fadd_rn(sl, att_l[F]);
      sr = __fadd_rn(sr, att_r[F]);
    }
    if (lane == 0) {
      al[i] = sl;
      ar[i] = sr;
    }
    ml = fmaxf(ml, sl);
    mr = fmaxf(mr, sr);
  }
  if (lane == 0) {
    red[0][wave] = ml;
    red[1][wave] = mr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = red[0][0], b = red[1][0];
    for (int w = 1; w < kGatThreads / 64; ++w) {
      a = fmaxf(a, red[0][w]);
      b = fmaxf(b, red[1][w]);
    }
    block_max[2 * blockIdx.x] = a;
    block_max[2 * blockIdx.x + 1] = b;
  }
}

// params[0..4] = max_l, max_r, s, ds/dmax_l, ds/dmax_r  (torch: scale =
// sqrt(max_l**2 + 1) * sqrt(max_r**2 + 1), fp32 tensor ops)
__global__ void __launch_bounds__(1024)
gat_scale_kernel(const float* __restrict__ block_max, int nblocks, float* __restrict__ params) {
  __shared__ float red[2][1024];
  float a = -INFINITY, b = -INFINITY;
  for (int k = threadIdx.x; k < nblocks; k += 1024) {
    a = fmaxf(a, block_max[2 * k]);
    b = fmaxf(b, block_max[2 * k + 1]);
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] = fmaxf(red[0][threadIdx.x], red[0][threadIdx.x + w]);
      red[1][threadIdx.x] = fmaxf(red[1][threadIdx.x], red[1][threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float ml = red[0][0], mr = red[1][0];
    const float ql = sqrtf(__fadd_rn(__fmul_rn(ml, ml), 1.f));
    const float qr = sqrtf(__fadd_rn(__fmul_rn(mr, mr), 1.f));
    params[0] = ml;
    params[1] = mr;
    params[2] = __fmul_rn(ql, qr);
    params[3] = __fmul_rn(__fdiv_rn(ml, ql), qr);   // ds/dmax_l
    params[4] = __fmul_rn(ql, __fdiv_rn(mr, qr));   // ds/dmax_r
  }
}

// als[i] = alpha_l[i] / s, ars[i] = alpha_r[i] / s once per node: the
// reference scales the attention scalars per node (convs.py:209-211, alpha_l =
// alpha_l / scale) and only adds them per edge (:256), so every per-edge
// consumer reads these instead of dividing twice per edge (bit-identical).
__global__ void gat_div_kernel(const float* __restrict__ al, const float* __restrict__ ar, int n,
                               const float* __restrict__ params, float* __restrict__ als,
                               float* __restrict__ ars) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = params[2];
  als[i] = __fdiv_rn(al[i], s);
  ars[i] = __fdiv_rn(ar[i], s);
}

// coef[e] = exp(leaky(als[j] + ars[i])) * w[e] (als, ars: alpha / s per node);
// den[i] = sum_e coef[e] in CSR order (the ones column of the aggregation).
// One wave per row.
__global__ void __launch_bounds__(kGatThreads)
gat_coef_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                const float* __restrict__ val, int n_rows, const float* __restrict__ als,
                const float* __restrict__ ars, float slope, float* __restrict__ coef,
                float* __restrict__ den) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * (kGatThreads / 64) + (threadIdx.x >> 6);
  if (i >= n_rows) return;
  const float ari = ars[i];
  const int rb = rowptr[i], re = rowptr[i + 1];
  float d = 0.f;
  for (int base = rb; base < re; base += 64) {
    const int e = base + lane;
    float c = 0.f;
    if (e < re) {
      float a = __fadd_rn(als[col[e]], ari);
      a = a > 0.f ? a : __fmul_rn(a, slope);
      c = __fmul_rn(expf(a), val[e]);
      coef[e] = c;
    }
    const int cnt = min(64, re - base);
    for (int k = 0; k < cnt; ++k)
      d = __fadd_rn(d, __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                     __builtin_bit_cast(int, c), k)));
  }
  if (lane == 0) den[i] = d;
}

// rows < B: out[i][:F] /= den[i] + eps  (models.py:188)
__global__ void gat_normalize_kernel(float* __restrict__ out, int64_t ldo, int B, int F,
                                     const float* __restrict__ den, float eps) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * F) return;
  const int64_t i = t / F;
  const int c = (int)(t % F);
  float* p = out + i * ldo + c;
  *p = __fdiv_rn(*p, __fadd_rn(den[i], eps));
}

// Backward of the coefficient chain, one thread per edge e (row i, col j):
//   dcoef = dy[i] . x_in[j][:F] + dden[i]      (dden = grad of the ones column)
//   da    = dcoef * coef * (a > 0 ? 1 : slope),  a = als[j] + ars[i]
//   (als, ars = alpha / s per node, vqgnn_gat_alpha)
//   dal[j] += da / s;  dar[i] += da / s;  dsrow[i] += -da * a / s
__global__ void __launch_bounds__(kGatThreads)
gat_edge_grad_kernel(const int32_t* __restrict__ rows, const int32_t* __restrict__ col,
                     const float* __restrict__ coef, int nnz, const float* __restrict__ X,
                     int64_t ldx, const float* __restrict__ X2, int64_t ldx2, int B, int F,
                     const float* __restrict__ dy, int64_t lddy, const float* __restrict__ dden,
                     const float* __restrict__ als, const float* __restrict__ ars,
                     const float* __restrict__ params, float slope, float* __restrict__ dal,
                     float* __restrict__ dar, float* __restrict__ dsrow) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const int i = rows[e], j = col[e];
  const float* xr = j < B ? X + (int64_t)j * ldx : X2 + (int64_t)(j - B) * ldx2;
  const float* g = dy + (int64_t)i * lddy;
  float dot = 0.f;
  if ((F & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(xr);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int c = 0; c < F / 4; ++c) {
      const float4 a = x4[c], b = g4[c];
      dot = fmaf(a.x, b.x, dot);
      dot = fmaf(a.y, b.y, dot);
      dot = fmaf(a.z, b.z, dot);
      dot = fmaf(a.w, b.w, dot);
    }
  } else {
    for (int c = 0; c < F; ++c) dot = fmaf(xr[c], g[c], dot);
  }
  const float dcoef = dot + (dden ? dden[i] : 0.f);
  const float s = params[2];
  const float a = __fadd_rn(als[j], ars[i]);
  const float da = dcoef * coef[e] * (a > 0.f ? 1.f : slope);
  const float q = da / s;
  atomicAdd(dal + j, q);
  atomicAdd(dar + i, q);
  atomicAdd(dsrow + i, -q * a);
}

// Group form of the coefficient-chain backward (F % 4 == 0, rows 16-byte
// aligned): a wave takes 16 consecutive edges, a group of 16 lanes 4 of them,
// each lane float4 pieces of x_in[j] . dy[i] (coalesced 256-byte row reads;
// the 4 edges' loads in flight together), reduced across the 16 lanes; lane 0
// of the group applies the chain and the atomics as the per-edge kernel does.
template <int P>   // float4 pieces per lane: P * 16 * 4 >= F
__global__ void __launch_bounds__(kGatThreads)
gat_edge_grad_grp_kernel(const int32_t* __restrict__ rows, const int32_t* __restrict__ col,
                         const float* __restrict__ coef, int nnz, const float* __restrict__ X,
                         int64_t ldx, const float* __restrict__ X2, int64_t ldx2, int B, int F,
                         const float* __restrict__ dy, int64_t lddy,
                         const float* __restrict__ dden, const float* __restrict__ als,
                         const float* __restrict__ ars, const float* __restrict__ params,
                         float slope, float* __restrict__ dal, float* __restrict__ dar,
                         float* __restrict__ dsrow) {
  constexpr int U = 4;
  const int64_t wave = (blockIdx.x * (int64_t)kGatThreads + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  const int64_t e0 = wave * 16 + g * U;
  if (wave * 16 >= nnz) return;
  const int F4 = F >> 2;
  int ii[U], jj[U];
  bool ok[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t e = e0 + u;
    ok[u] = e < nnz;
    ii[u] = ok[u] ? rows[e] : 0;
    jj[u] = ok[u] ? col[e] : 0;
  }
  float dot[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float4* x4 = reinterpret_cast<const float4*>(
        jj[u] < B ? X + (int64_t)jj[u] * ldx : X2 + (int64_t)(jj[u] - B) * ldx2);
    const float4* g4 = reinterpret_cast<const float4*>(dy + (int64_t)ii[u] * lddy);
    float d = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int c = l16 + 16 * p;
      if (ok[u] && c < F4) {
        const float4 a = x4[c], b = g4[c];
        d = fmaf(a.x, b.x, d);
        d = fmaf(a.y, b.y, d);
        d = fmaf(a.z, b.z, d);
        d = fmaf(a.w, b.w, d);
      }
    }
    dot[u] = d;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) dot[u] += __shfl_xor(dot[u], o);
  }
  if (l16 != 0) return;
  const float s = params[2];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!ok[u]) continue;
    const int i = ii[u], j = jj[u];
    const float dcoef = dot[u] + (dden ? dden[i] : 0.f);
    const float a = __fadd_rn(als[j], ars[i]);
    const float da = dcoef * coef[e0 + u] * (a > 0.f ? 1.f : slope);
    const float q = da / s;
    atomicAdd(dal + j, q);
    atomicAdd(dar + i, q);
    atomicAdd(dsrow + i, -q * a);
  }
}

// d att = x_in^T d alpha for both attention vectors at once (x_in = [X ; X2 ;
// ones]): block b sums rows [b*kAttRows, ...) — thread = (row phase, float4
// column) — into partial[b][2][C] (fixed order), then gat_att_reduce_kernel
// folds the partials in block order (deterministic).  C = F + ones.
constexpr int kAttRows = 1024;
__global__ void __launch_bounds__(kGatThreads)
gat_att_partial_kernel(const float* __restrict__ X, int64_t ldx, const float* __restrict__ X2,
                       int64_t ldx2, int B, int n, int F, int ones,
                       const float* __restrict__ dal, const float* __restrict__ dar,
                       float* __restrict__ partial) {
  __shared__ float4 red_l[kGatThreads], red_r[kGatThreads];
  __shared__ float red_s[2][kGatThreads];
  const int F4 = F >> 2;
  const int C = F + ones;
  const int cols = F4 < kGatThreads ? F4 : kGatThreads;
  const int phases = kGatThreads / cols;
  const int tid = threadIdx.x;
  const int ph = tid / cols, c4 = tid % cols;
  const int r0 = blockIdx.x * kAttRows, r1 = min(n, r0 + kAttRows);
  float* out = partial + (int64_t)blockIdx.x * 2 * C;
  for (int cb = 0; cb < F4; cb += cols) {           // column blocks of `cols` float4
    const int c = cb + c4;
    float4 gl = make_float4(0.f, 0.f, 0.f, 0.f), gr = gl;
    float sl = 0.f, sr = 0.f;
    if (ph < phases && c < F4) {
      for (int r = r0 + ph; r < r1; r += phases) {
        const float4 x = reinterpret_cast<const float4*>(
            r < B ? X + (int64_t)r * ldx : X2 + (int64_t)(r - B) * ldx2)[c];
        const float a = dal[r], b = dar[r];
        gl.x = fmaf(a, x.x, gl.x); gl.y = fmaf(a, x.y, gl.y);
        gl.z = fmaf(a, x.z, gl.z); gl.w = fmaf(a, x.w, gl.w);
        gr.x = fmaf(b, x.x, gr.x); gr.y = fmaf(b, x.y, gr.y);
        gr.z = fmaf(b, x.z, gr.z); gr.w = fmaf(b, x.w, gr.w);
        if (cb == 0 && c4 == 0) {
          sl += a;
          sr += b;
        }
      }
    }
    red_l[tid] = gl;
    red_r[tid] = gr;
    red_s[0][tid] = sl;
    red_s[1][tid] = sr;
    __syncthreads();
    if (ph == 0 && c < F4) {
      for (int p = 1; p < phases; ++p) {
        const float4 u = red_l[p * cols + c4], v = red_r[p * cols + c4];
        gl.x += u.x; gl.y += u.y; gl.z += u.z; gl.w += u.w;
        gr.x += v.x; gr.y += v.y; gr.z += v.z; gr.w += v.w;
      }
      reinterpret_cast<float4*>(out)[c] = gl;
      reinterpret_cast<float4*>(out + C)[c] = gr;
    }
    if (cb == 0 && tid == 0 && ones) {
      float tl = 0.f, tr = 0.f;
      for (int p = 0; p < phases; ++p) {
        tl += red_s[0][p * cols];
        tr += red_s[1][p * cols];
      }
      out[F] = tl;
      out[C + F] = tr;
    }
    __syncthreads();
  }
}

__global__ void gat_att_reduce_kernel(const float* __restrict__ partial, int nblocks, int C,
                                      float* __restrict__ att_l, float* __restrict__ att_r) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * C) return;
  float acc = 0.f;
  for (int b = 0; b < nblocks; ++b) acc += partial[(int64_t)b * 2 * C + c];
  if (c < C) att_l[c] = acc; else att_r[c - C] = acc;
}

}  // namespace vqgnn

using namespace vqgnn;

extern "C" size_t vqgnn_gat_att_grad_workspace(int32_t n, int32_t F, int32_t ones) {
  const int nb = (n + kAttRows - 1) / kAttRows;
  return align_up((size_t)(nb > 0 ? nb : 1) * 2 * (F + (ones ? 1 : 0)) * sizeof(float), 256);
}

extern "C" int vqgnn_gat_att_grad(const float* X, int64_t ldx, const float* X2, int64_t ldx2,
                                  int32_t B, int32_t n, int32_t F, int32_t ones,
                                  const float* dalpha_l, const float* dalpha_r, float* datt_l,
                                  float* datt_r, void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(n > 0 && F > 0 && F % 4 == 0 && B >= 0 && B <= n,
                "gat_att_grad: bad shape (n=%d B=%d F=%d)", n, B, F);
  VQGNN_REQUIRE(X && dalpha_l && dalpha_r && datt_l && datt_r && workspace && (B == n || X2),
                "gat_att_grad: null pointer");
  VQGNN_REQUIRE(((((uintptr_t)X | (uintptr_t)X2) & 15) == 0 && ldx % 4 == 0 &&
                 (!X2 || ldx2 % 4 == 0)),
                "gat_att_grad: rows must be 16-byte aligned");
  const int C = F + (ones ? 1 : 0);
  const int nb = (n + kAttRows - 1) / kAttRows;
  float* part = reinterpret_cast<float*>(workspace);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(gat_att_partial_kernel, dim3(nb), dim3(kGatThreads), 0, s, X, ldx, X2, ldx2, B,
                     n, F, ones ? 1 : 0, dalpha_l, dalpha_r, part);
  hipLaunchKernelGGL(gat_att_reduce_kernel, dim3((2 * C + 255) / 256), dim3(256), 0, s, part, nb,
                     C, datt_l, datt_r);
  return check_launch("gat_att_grad");
}

extern "C" size_t vqgnn_gat_alpha_workspace(int32_t n) {
  const int rows_per_block = (kGatThreads / 64) * kGatRowsPerWave;
  const int64_t nblocks = (n + rows_per_block - 1) / rows_per_block;
  return align_up((size_t)(nblocks > 0 ? nblocks : 1) * 2 * sizeof(float), 256);
}

extern "C" int vqgnn_gat_alpha(const float* X, int64_t ldx, const float* X2, int64_t ldx2,
                               int32_t B, int32_t n, int32_t F, int32_t ones,
                               const float* att_l, const float* att_r, float* alpha_l,
                               float* alpha_r, float* alpha_l_s, float* alpha_r_s, float* params,
                               void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(n > 0 && F > 0 && B >= 0 && B <= n, "gat_alpha: bad shape (n=%d B=%d F=%d)",
                n, B, F);
  VQGNN_REQUIRE(X && att_l && att_r && alpha_l && alpha_r && params && workspace,
                "gat_alpha: null pointer");
  VQGNN_REQUIRE(B == n || X2, "gat_alpha: X2 required for rows >= B");
  VQGNN_REQUIRE(ldx >= F && (!X2 || ldx2 >= F), "gat_alpha: ld < F");
  hipStream_t s = as_stream(stream);
  const int rows_per_block = (kGatThreads / 64) * kGatRowsPerWave;
  const int nblocks = (n + rows_per_block - 1) / rows_per_block;
  float* bm = reinterpret_cast<float*>(workspace);
  const bool vec = F % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X & 15) == 0 &&
                   (!X2 || (ldx2 % 4 == 0 && ((uintptr_t)X2 & 15) == 0)) &&
                   ((uintptr_t)att_l & 15) == 0 && ((uintptr_t)att_r & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(gat_alpha4_kernel, dim3(nblocks), dim3(kGatThreads), 0, s, X, ldx, X2,
                       ldx2, B, n, F, ones, att_l, att_r, alpha_l, alpha_r, bm);
  else
    hipLaunchKernelGGL(gat_alpha_kernel, dim3(nblocks), dim3(kGatThreads), 0, s, X, ldx, X2,
                       ldx2, B, n, F, ones, att_l, att_r, alpha_l, alpha_r, bm);
  hipLaunchKernelGGL(gat_scale_kernel, dim3(1), dim3(1024), 0, s, bm, nblocks, params);
  VQGNN_REQUIRE((alpha_l_s == nullptr) == (alpha_r_s == nullptr),
                "gat_alpha: alpha_l_s and alpha_r_s go together");
  if (alpha_l_s)
    hipLaunchKernelGGL(gat_div_kernel, dim3((n + 255) / 256), dim3(256), 0, s, alpha_l, alpha_r, n,
                       params, alpha_l_s, alpha_r_s);
  return check_launch("gat_alpha");
}

extern "C" int vqgnn_gat_coef(const int32_t* rowptr, const int32_t* col, const float* val,
                              int32_t n_rows, int64_t nnz, const float* alpha_l_s,
                              const float* alpha_r_s, float negative_slope, float* coef,
                              float* den, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(n_rows >= 0 && nnz >= 0 && nnz < (int64_t)INT32_MAX, "gat_coef: bad shape");
  if (n_rows == 0) return VQGNN_OK;
  VQGNN_REQUIRE(rowptr && alpha_l_s && alpha_r_s && den && (nnz == 0 || (col && val && coef)),
                "gat_coef: null pointer");
  const int wpb = kGatThreads / 64;
  hipLaunchKernelGGL(gat_coef_kernel, dim3((n_rows + wpb - 1) / wpb), dim3(kGatThreads), 0,
                     as_stream(stream), rowptr, col, val, n_rows, alpha_l_s, alpha_r_s,
                     negative_slope, coef, den);
  return check_launch("gat_coef");
}

extern "C" int vqgnn_gat_normalize(float* out, int64_t ldo, int32_t B, int32_t F,
                                   const float* den, float eps, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(B >= 0 && F > 0 && ldo >= F, "gat_normalize: bad shape");
  if (B == 0) return VQGNN_OK;
  VQGNN_REQUIRE(out && den, "gat_normalize: null pointer");
  const int64_t tot = (int64_t)B * F;
  hipLaunchKernelGGL(gat_normalize_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     as_stream(stream), out, ldo, B, F, den, eps);
  return check_launch("gat_normalize");
}

extern "C" int vqgnn_gat_edge_grad(const int32_t* rows, const int32_t* col, const float* coef,
                                   int64_t nnz, const float* X, int64_t ldx, const float* X2,
                                   int64_t ldx2, int32_t B, int32_t F, const float* dy,
                                   int64_t lddy, const float* dden, const float* alpha_l_s,
                                   const float* alpha_r_s, const float* params,
                                   float negative_slope, float* dalpha_l, float* dalpha_r,
                                   float* ds_row, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(nnz >= 0 && nnz < (int64_t)INT32_MAX && F > 0, "gat_edge_grad: bad shape");
  if (nnz == 0) return VQGNN_OK;
  VQGNN_REQUIRE(rows && col && coef && X && dy && alpha_l_s && alpha_r_s && params && dalpha_l &&
                    dalpha_r && ds_row,
                "gat_edge_grad: null pointer");
  VQGNN_REQUIRE((F & 3) != 0 || ((((uintptr_t)X | (uintptr_t)dy | (uintptr_t)X2) & 15) == 0 &&
                                 ldx % 4 == 0 && lddy % 4 == 0 && (!X2 || ldx2 % 4 == 0)),
                "gat_edge_grad: F%%4==0 needs 16-byte aligned rows");
  const int n = (int)nnz;
  const bool grp = (F & 3) == 0 && F <= 512 &&
                   ((((uintptr_t)X | (uintptr_t)dy | (uintptr_t)X2) & 15) == 0 && ldx % 4 == 0 &&
                    lddy % 4 == 0 && (!X2 || ldx2 % 4 == 0));
  if (grp) {   // 16 lanes per edge, coalesced row reads
    const int64_t threads = ((int64_t)n + 15) / 16 * 64;
    const dim3 grid((unsigned)((threads + kGatThreads - 1) / kGatThreads));
    const int P = (F / 4 + 15) / 16;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, dim3(kGatThreads), 0, as_stream(stream), rows, col, coef, n,
                         X, ldx, X2, ldx2, B, F, dy, lddy, dden, alpha_l_s, alpha_r_s, params,
                         negative_slope, dalpha_l, dalpha_r, ds_row);
    };
    if (P <= 1) go(gat_edge_grad_grp_kernel<1>);
    else if (P <= 2) go(gat_edge_grad_grp_kernel<2>);
    else if (P <= 4) go(gat_edge_grad_grp_kernel<4>);
    else go(gat_edge_grad_grp_kernel<8>);
  } else {
    hipLaunchKernelGGL(gat_edge_grad_kernel, dim3((n + kGatThreads - 1) / kGatThreads),
                       dim3(kGatThreads), 0, as_stream(stream), rows, col, coef, n, X, ldx, X2,
                       ldx2, B, F, dy, lddy, dden, alpha_l_s, alpha_r_s, params, negative_slope,
                       dalpha_l, dalpha_r, ds_row);
  }
  return check_launch("gat_edge_grad");
}
