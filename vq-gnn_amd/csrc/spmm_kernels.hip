// Fused codebook-gather + CSR SpMM for gfx950 (MI355X), the out-of-batch code
// gather, and the CSR transpose for the backward product.
//
// Reference path: LowRankGNNLayer.forward (vq_gnn_v2/models.py:157-179) builds
// x_input = [x ; concat_b codebook_b[c_b[subset[B:]], :D]] and calls
// OurGCNConv.forward (convs.py:65-101) -> PyG GCNConv.message_and_aggregate ->
// torch_sparse.matmul(adj_t, x_input, reduce='add') (spmm_sum).  Here the
// [B', F] codeword rows are never materialised: an edge to j >= B reads the
// node's int16 code per branch and the codeword's feature half straight from
// the (L2-resident) _embedding_output.
//
// Work decomposition: merge-based / edge-balanced.  The nnz range is cut into
// chunks of S edges; one lane group (G lanes, each owning float4 column
// chunks) walks one chunk, summing each row's edges in CSR order with
// separate mul and add (spmm_sum's `out = out + val * x`, init 0) and storing
// rows that end inside the chunk.  A row that crosses a chunk boundary leaves
// one partial per chunk ("carry"); a fix-up kernel adds them in chunk order.
// Zipf hub rows therefore spread over many groups instead of serialising one.

#include "common.h"

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

namespace vqgnn {

constexpr int kSpmmThreads = 256;

__device__ __forceinline__ int lower_bound_i32(const int32_t* __restrict__ a, int n, int key) {
  // first i in [0, n] with a[i] >= key  (a has n+1 entries, non-decreasing)
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

struct SpmmArgs {
  const int32_t* rowptr;
  const int32_t* col;
  const float* val;
  int n_rows;
  int nnz;
  int S;          // edges per chunk
  int nchunks;
  int B;          // columns < B read X; >= B read the codebook (GATHER)
  const float* X;
  int64_t ldx4;   // in float4
  int F4;         // F / 4
  int D;
  const int16_t* lcodes;
  int nb;
  const float* emb;
  int64_t ldw;
  int64_t emb_bstride;
  float* out;
  int64_t ldo4;
  float* carry;   // [nchunks][2][F]
  int* carry_row; // [nchunks]
};

// Accumulate edges [eb, ee) into acc (float4 x NCH), in order.
template <int G, int NCH, bool GATHER>
__device__ __forceinline__ void spmm_segment(const SpmmArgs& a, int eb, int ee, int lg,
                                             float4 (&acc)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* X4 = reinterpret_cast<const float4*>(a.X);
  constexpr int U = 4;
  for (int e = eb; e < ee; e += U) {
    int jj[U];
    float ww[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = e + u < ee;
      jj[u] = ok ? a.col[e + u] : -1;
      ww[u] = ok ? a.val[e + u] : 0.f;
    }
    float4 v[U][NCH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jj[u];
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int cc = lg + c * G;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j >= 0 && cc < a.F4) {
          if (!GATHER || j < a.B) {
            x = X4[(int64_t)j * a.ldx4 + cc];
          } else {
            const int col0 = cc * 4;
            const int br = col0 / a.D, off = col0 - br * a.D;
            const int code = a.lcodes[(int64_t)(j - a.B) * a.nb + br];
            x = *reinterpret_cast<const float4*>(a.emb + br * a.emb_bstride +
                                                 (int64_t)code * a.ldw + off);
          }
        }
        v[u][c] = x;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (jj[u] >= 0) {
        const float w = ww[u];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          acc[c].x = __fadd_rn(acc[c].x, __fmul_rn(w, v[u][c].x));
          acc[c].y = __fadd_rn(acc[c].y, __fmul_rn(w, v[u][c].y));
          acc[c].z = __fadd_rn(acc[c].z, __fmul_rn(w, v[u][c].z));
          acc[c].w = __fadd_rn(acc[c].w, __fmul_rn(w, v[u][c].w));
        }
      }
    }
  }
}

template <int G, int NCH>
__device__ __forceinline__ void store_row(float4* dst, int lg, int F4, const float4 (&acc)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int cc = lg + c * G;
    if (cc < F4) dst[cc] = acc[c];
  }
}

template <int G, int NCH, bool GATHER>
__global__ void __launch_bounds__(kSpmmThreads)
spmm_merge_kernel(SpmmArgs a) {
  constexpr int GPW = kSpmmThreads / G;  // groups per workgroup
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = wg * GPW + threadIdx.x / G;
  const int lg = threadIdx.x % G;
  if (chunk >= a.nchunks) return;
  const int e0 = chunk * a.S;
  const int e1 = min(e0 + a.S, a.nnz);
  const bool last = e1 == a.nnz;
  float4* out4 = reinterpret_cast<float4*>(a.out);
  float4* carry4 = reinterpret_cast<float4*>(a.carry);
  const int F4 = a.F4;

  int i = lower_bound_i32(a.rowptr, a.n_rows, e0);
  int crow = -1;
  float4 acc[NCH];
  if (i > 0 && a.rowptr[i] > e0) {  // row i-1 started before this chunk
    const int re = min(a.rowptr[i], e1);
    spmm_segment<G, NCH, GATHER>(a, e0, re, lg, acc);
    store_row<G, NCH>(carry4 + (int64_t)chunk * 2 * F4, lg, F4, acc);
    crow = i - 1;
  }
  for (; i < a.n_rows; ++i) {
    const int rb = a.rowptr[i];
    if (!(rb < e1 || last)) break;
    const int re_full = a.rowptr[i + 1];
    const int re = min(re_full, e1);
    spmm_segment<G, NCH, GATHER>(a, rb, re, lg, acc);
    if (re_full <= e1) {
      store_row<G, NCH>(out4 + (int64_t)i * a.ldo4, lg, F4, acc);
    } else {
      store_row<G, NCH>(carry4 + ((int64_t)chunk * 2 + 1) * F4, lg, F4, acc);
      break;
    }
  }
  if (lg == 0) a.carry_row[chunk] = crow;
}

// For every row that spans chunks, the chunk where it ends adds the partials:
// carry_last[start chunk] + carry_first[start+1 .. end] (chunk order).
template <int G, int NCH>
__global__ void __launch_bounds__(kSpmmThreads)
spmm_fixup_kernel(SpmmArgs a) {
  constexpr int GPW = kSpmmThreads / G;
  const int chunk = blockIdx.x * GPW + threadIdx.x / G;
  const int lg = threadIdx.x % G;
  if (chunk >= a.nchunks) return;
  const int r = a.carry_row[chunk];
  if (r < 0) return;
  const int e1 = min(chunk * a.S + a.S, a.nnz);
  if (a.rowptr[r + 1] > e1) return;  // not the end chunk of row r
  const int gs = a.rowptr[r] / a.S;
  const int F4 = a.F4;
  const float4* carry4 = reinterpret_cast<const float4*>(a.carry);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int cc = lg + c * G;
    if (cc >= F4) continue;
    float4 s = carry4[((int64_t)gs * 2 + 1) * F4 + cc];
    for (int g = gs + 1; g <= chunk; ++g) {
      const float4 t = carry4[(int64_t)g * 2 * F4 + cc];
      s.x = __fadd_rn(s.x, t.x);
      s.y = __fadd_rn(s.y, t.y);
      s.z = __fadd_rn(s.z, t.z);
      s.w = __fadd_rn(s.w, t.w);
    }
    reinterpret_cast<float4*>(a.out)[(int64_t)r * a.ldo4 + cc] = s;
  }
}

__global__ void zero_rows_kernel(float* out, int64_t ldo, int n_rows, int F) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n_rows * F) return;
  out[(i / F) * ldo + (i % F)] = 0.f;
}

// lcodes[j][b] = codes[subset[B + j]][b]                         models.py:168
__global__ void gather_codes_kernel(const int64_t* __restrict__ subset, int B, int nprime,
                                    const int16_t* __restrict__ codes, int64_t ldc, int nb,
                                    int16_t* __restrict__ lcodes) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nprime * nb) return;
  const int64_t j = t / nb;
  const int b = (int)(t % nb);
  lcodes[t] = codes[subset[B + j] * ldc + b];
}

// codes[batch_idx[i]][b] = local[i][b]
__global__ void scatter_codes_kernel(const int64_t* __restrict__ batch_idx, int B,
                                     const int16_t* __restrict__ local, int nb,
                                     int16_t* __restrict__ codes, int64_t ldc) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * nb) return;
  const int64_t i = t / nb;
  const int b = (int)(t % nb);
  const int64_t node = batch_idx[i];
  if (node >= 0) codes[node * ldc + b] = local[t];
}

// ---- CSR transpose helpers ----
__global__ void expand_rows_kernel(const int32_t* __restrict__ rowptr, int n_rows,
                                   int32_t* __restrict__ rows, int32_t* __restrict__ iota,
                                   int nnz) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  // binary search the row containing e
  int lo = 0, hi = n_rows - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rowptr[mid] <= e) lo = mid; else hi = mid - 1;
  }
  rows[e] = lo;
  iota[e] = e;
}

__global__ void transpose_finish_kernel(const int32_t* __restrict__ sorted_cols,
                                        const int32_t* __restrict__ perm,
                                        const int32_t* __restrict__ rows,
                                        const float* __restrict__ val, int nnz, int n_cols,
                                        int32_t* __restrict__ t_rowptr,
                                        int32_t* __restrict__ t_col, float* __restrict__ t_val) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nnz) {
    const int e = perm[t];
    t_col[t] = rows[e];
    if (t_val) t_val[t] = val[e];
  }
  if (t <= n_cols) {  // t_rowptr[c] = first position with sorted_col >= c
    int lo = 0, hi = nnz;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sorted_cols[mid] < t) lo = mid + 1; else hi = mid;
    }
    t_rowptr[t] = lo;
  }
}

static int spmm_chunk_edges(int F4) { return F4 > 32 ? 64 : 128; }

}  // namespace vqgnn

using namespace vqgnn;

extern "C" size_t vqgnn_spmm_workspace(int32_t n_rows, int64_t nnz, int32_t F) {
  (void)n_rows;
  if (nnz <= 0 || F <= 0) return 256;
  const int S = spmm_chunk_edges((F + 3) / 4);
  const int64_t nchunks = (nnz + S - 1) / S;
  return align_up((size_t)nchunks * 2 * F * sizeof(float), 256) +
         align_up((size_t)nchunks * sizeof(int), 256);
}

template <int G, int NCH, bool GATHER>
static void launch_spmm(const SpmmArgs& a, hipStream_t s) {
  constexpr int GPW = kSpmmThreads / G;
  const int grid = (a.nchunks + GPW - 1) / GPW;
  hipLaunchKernelGGL((spmm_merge_kernel<G, NCH, GATHER>), dim3(grid), dim3(kSpmmThreads), 0, s, a);
  hipLaunchKernelGGL((spmm_fixup_kernel<G, NCH>), dim3(grid), dim3(kSpmmThreads), 0, s, a);
}

template <bool GATHER>
static int dispatch_spmm(const SpmmArgs& a, hipStream_t s) {
  const int F4 = a.F4;
  if (F4 <= 16) launch_spmm<16, 1, GATHER>(a, s);
  else if (F4 <= 32) launch_spmm<32, 1, GATHER>(a, s);
  else if (F4 <= 64) launch_spmm<64, 1, GATHER>(a, s);
  else if (F4 <= 128) launch_spmm<64, 2, GATHER>(a, s);
  else if (F4 <= 192) launch_spmm<64, 3, GATHER>(a, s);
  else if (F4 <= 256) launch_spmm<64, 4, GATHER>(a, s);
  else if (F4 <= 512) launch_spmm<64, 8, GATHER>(a, s);
  else {
    set_error("spmm: F=%d > 2048 not implemented", F4 * 4);
    return VQGNN_ERR_UNSUPPORTED;
  }
  return check_launch("spmm");
}

extern "C" int vqgnn_spmm(const int32_t* rowptr, const int32_t* col, const float* val,
                          int32_t n_rows, int64_t nnz, int32_t B, const float* X, int64_t ldx,
                          int32_t F, int32_t D, const int16_t* lcodes, int32_t nb,
                          const float* emb_out, int32_t ldw, int64_t emb_bstride, float* out,
                          int64_t ldo, void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(rowptr && out && n_rows >= 0, "spmm: null pointer");
  VQGNN_REQUIRE(F > 0 && F % 4 == 0, "spmm: F=%d must be a positive multiple of 4", F);
  VQGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= F && ldo >= F,
                "spmm: ldx/ldo must be multiples of 4 and >= F");
  VQGNN_REQUIRE(((uintptr_t)X & 15) == 0 && ((uintptr_t)out & 15) == 0,
                "spmm: X/out must be 16-byte aligned");
  VQGNN_REQUIRE(nnz < (int64_t)INT32_MAX, "spmm: nnz >= 2^31");
  hipStream_t s = as_stream(stream);
  if (n_rows == 0) return VQGNN_OK;
  if (nnz == 0) {
    const int64_t tot = (int64_t)n_rows * F;
    hipLaunchKernelGGL(zero_rows_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, out, ldo,
                       n_rows, F);
    return check_launch("spmm(zero)");
  }
  VQGNN_REQUIRE(col && val && X && workspace, "spmm: null pointer");
  const bool gather = lcodes != nullptr;
  if (gather) {
    VQGNN_REQUIRE(D > 0 && D % 4 == 0 && F % D == 0 && nb == F / D,
                  "spmm: codebook gather needs D %% 4 == 0 and nb == F/D (D=%d F=%d nb=%d)", D, F,
                  nb);
    VQGNN_REQUIRE(emb_out && ldw % 4 == 0 && emb_bstride % 4 == 0 &&
                      ((uintptr_t)emb_out & 15) == 0,
                  "spmm: codebook must be 16-byte aligned with ldw, stride multiples of 4");
  }
  SpmmArgs a;
  a.rowptr = rowptr;
  a.col = col;
  a.val = val;
  a.n_rows = n_rows;
  a.nnz = (int)nnz;
  a.F4 = F / 4;
  a.S = spmm_chunk_edges(a.F4);
  a.nchunks = (int)((nnz + a.S - 1) / a.S);
  a.B = B;
  a.X = X;
  a.ldx4 = ldx / 4;
  a.D = D;
  a.lcodes = lcodes;
  a.nb = nb;
  a.emb = emb_out;
  a.ldw = ldw;
  a.emb_bstride = emb_bstride;
  a.out = out;
  a.ldo4 = ldo / 4;
  a.carry = reinterpret_cast<float*>(workspace);
  a.carry_row = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) +
                                       align_up((size_t)a.nchunks * 2 * F * sizeof(float), 256));
  return gather ? dispatch_spmm<true>(a, s) : dispatch_spmm<false>(a, s);
}

extern "C" int vqgnn_gather_codes(const int64_t* subset, int32_t B, int32_t n,
                                  const int16_t* codes, int64_t ldc, int32_t nb,
                                  int16_t* lcodes, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(n >= B && B >= 0 && nb > 0 && ldc >= nb, "gather_codes: bad shape");
  const int64_t tot = (int64_t)(n - B) * nb;
  if (tot == 0) return VQGNN_OK;
  VQGNN_REQUIRE(subset && codes && lcodes, "gather_codes: null pointer");
  hipLaunchKernelGGL(gather_codes_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     as_stream(stream), subset, B, n - B, codes, ldc, nb, lcodes);
  return check_launch("gather_codes");
}

extern "C" int vqgnn_scatter_codes(const int64_t* batch_idx, int32_t B, const int16_t* local,
                                   int32_t nb, int16_t* codes, int64_t ldc,
                                   vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(B >= 0 && nb > 0 && ldc >= nb, "scatter_codes: bad shape");
  const int64_t tot = (int64_t)B * nb;
  if (tot == 0) return VQGNN_OK;
  VQGNN_REQUIRE(batch_idx && local && codes, "scatter_codes: null pointer");
  hipLaunchKernelGGL(scatter_codes_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     as_stream(stream), batch_idx, B, local, nb, codes, ldc);
  return check_launch("scatter_codes");
}

// ---- CSR transpose: stable radix sort of edge ids by column (rocPRIM) ----
static size_t sort_temp_bytes(int64_t nnz, int n_cols) {
  size_t bytes = 0;
  const int bits = 32 - __builtin_clz((unsigned)(n_cols > 1 ? n_cols - 1 : 1));
  (void)rocprim::radix_sort_pairs((void*)nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                            (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)nnz, 0, bits);
  return bytes;
}

extern "C" size_t vqgnn_csr_transpose_workspace(int32_t n_rows, int32_t n_cols, int64_t nnz) {
  (void)n_rows;
  if (nnz <= 0) return 256;
  const size_t a = align_up((size_t)nnz * 4, 256);
  return 4 * a + align_up(sort_temp_bytes(nnz, n_cols), 256);
}

extern "C" int vqgnn_csr_transpose(const int32_t* rowptr, const int32_t* col, const float* val,
                                   int32_t n_rows, int32_t n_cols, int64_t nnz,
                                   int32_t* t_rowptr, int32_t* t_col, float* t_val,
                                   void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(rowptr && t_rowptr && n_rows >= 0 && n_cols >= 0, "csr_transpose: bad args");
  VQGNN_REQUIRE(nnz < (int64_t)INT32_MAX, "csr_transpose: nnz >= 2^31");
  hipStream_t s = as_stream(stream);
  if (nnz == 0) {
    (void)hipMemsetAsync(t_rowptr, 0, (size_t)(n_cols + 1) * sizeof(int32_t), s);
    return check_launch("csr_transpose(empty)");
  }
  VQGNN_REQUIRE(col && t_col && workspace, "csr_transpose: null pointer");
  const size_t a = align_up((size_t)nnz * 4, 256);
  char* ws = reinterpret_cast<char*>(workspace);
  int32_t* rows = reinterpret_cast<int32_t*>(ws);
  int32_t* iota = reinterpret_cast<int32_t*>(ws + a);
  int32_t* keys_out = reinterpret_cast<int32_t*>(ws + 2 * a);
  int32_t* perm = reinterpret_cast<int32_t*>(ws + 3 * a);
  void* temp = ws + 4 * a;
  size_t temp_bytes = align_up(sort_temp_bytes(nnz, n_cols), 256);
  const int n = (int)nnz;
  hipLaunchKernelGGL(expand_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rowptr, n_rows,
                     rows, iota, n);
  int rc = check_launch("csr_transpose(expand)");
  if (rc) return rc;
  const int bits = 32 - __builtin_clz((unsigned)(n_cols > 1 ? n_cols - 1 : 1));
  hipError_t e = rocprim::radix_sort_pairs(
      temp, temp_bytes, reinterpret_cast<const uint32_t*>(col),
      reinterpret_cast<uint32_t*>(keys_out), iota, perm, (size_t)nnz, 0, bits, s);
  if (e != hipSuccess) {
    set_error("csr_transpose: radix sort failed: %s", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  const int tot = n > n_cols + 1 ? n : n_cols + 1;
  hipLaunchKernelGGL(transpose_finish_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, keys_out,
                     perm, rows, val, n, n_cols, t_rowptr, t_col, t_val);
  return check_launch("csr_transpose");
}
