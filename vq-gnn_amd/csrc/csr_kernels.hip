// Codeword gather, code scatter and the CSR transpose for gfx950 (MI355X).
//
// Reference path: LowRankGNNLayer.forward (vq_gnn_v2/models.py:157-179) builds
// x_input = [x ; concat_b codebook_b[c_b[subset[B:]], :D]]; the aggregation
// (convs.py:95, torch_sparse.matmul) is spmm_tasks.hip.
//
// gather_codewords writes x_first_order [B', F] once per out-of-batch node
// (one coalesced 4*F-byte row per node; the codebooks are L2-resident) --
// measured 2.3x faster than gathering codewords per edge, where each edge
// touches nb different codebook lines.  The task SpMM then reads rows j < B
// from x and rows j >= B from x_first_order (no torch.cat copy).
//
// The transpose (torch_sparse's csr2csc for the backward A^T * dOut) is a
// stable rocPRIM radix sort of edge ids by column: within a column the
// entries keep their row order.

#include "common.h"

#include <rocprim/device/device_radix_sort.hpp>

namespace vqgnn {

// x_first_order[j][b*D + k] = emb_out[b][codes[subset[B + j]][b]][off + k]
// (models.py:168-173; off = 0 feature half, off = D grad half), and optionally
// lcodes[j][b] = the code.  Thread per (node, branch); D == 4 stores float4.
// Bounds: a node outside [0, n_nodes) or a code outside [0, M) reads nothing
// (its D values are written as zeros; lcodes gets -1 for a bad node, the code
// as read for a bad code).  The host checks nb <= the codebook's branches.
__global__ void gather_codewords_kernel(const int64_t* __restrict__ subset, int B, int nprime,
                                        const int16_t* __restrict__ codes, int64_t ldc,
                                        int64_t n_nodes, int nb, int D,
                                        const float* __restrict__ emb, int M, int ldw,
                                        int64_t bstride, int off, float* __restrict__ xt,
                                        int64_t ldt, int16_t* __restrict__ lcodes) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nprime * nb) return;
  const int64_t j = t / nb;
  const int b = (int)(t % nb);
  const int64_t node = subset[B + j];
  const bool nok = node >= 0 && node < n_nodes;
  const int code = nok ? (int)codes[node * ldc + b] : -1;
  if (lcodes) lcodes[t] = (int16_t)code;
  if (!xt) return;
  float* dst = xt + j * ldt + (int64_t)b * D;
  if (code < 0 || code >= M) {
    for (int k = 0; k < D; ++k) dst[k] = 0.f;
    return;
  }
  const float* src = emb + b * bstride + (int64_t)code * ldw + off;
  if (D == 4 && ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0) {
    *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
  } else {
    for (int k = 0; k < D; ++k) dst[k] = src[k];
  }
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
  if (iota) iota[e] = e;
}

__global__ void transpose_finish_kernel(const int32_t* __restrict__ sorted_cols,
                                        const int32_t* __restrict__ perm,
                                        const int32_t* __restrict__ rows,
                                        const float* __restrict__ val, int nnz, int n_cols,
                                        int32_t* __restrict__ t_rowptr,
                                        int32_t* __restrict__ t_col, float* __restrict__ t_val,
                                        int32_t* __restrict__ t_perm) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nnz) {
    const int e = perm[t];
    t_col[t] = rows[e];
    if (t_val) t_val[t] = val[e];
    if (t_perm) t_perm[t] = e;
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

}  // namespace vqgnn

using namespace vqgnn;

extern "C" int vqgnn_gather_codewords(const int64_t* subset, int32_t B, int32_t n,
                                      const int16_t* codes, int64_t ldc, int64_t n_nodes,
                                      int32_t nb, int32_t D, const float* emb_out,
                                      int32_t n_branches, int32_t M, int32_t ldw,
                                      int64_t emb_bstride, int32_t col_offset, float* xt,
                                      int64_t ldt, int16_t* lcodes, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(n >= B && B >= 0 && nb > 0 && ldc >= nb && D > 0 && n_nodes >= 0,
                "gather_codewords: bad shape");
  const int64_t tot = (int64_t)(n - B) * nb;
  if (tot == 0) return VQGNN_OK;
  VQGNN_REQUIRE(subset && codes && (xt || lcodes), "gather_codewords: null pointer");
  // every branch read must exist in the codebook (emb_out [n_branches][M][ldw])
  VQGNN_REQUIRE(!xt || (emb_out && nb <= n_branches && M > 0),
                "gather_codewords: %d code columns read past the codebook's %d branches "
                "(M=%d)", nb, n_branches, M);
  VQGNN_REQUIRE(!xt || (ldt >= (int64_t)nb * D && col_offset >= 0 && col_offset + D <= ldw &&
                        (n_branches == 1 || emb_bstride >= (int64_t)M * ldw)),
                "gather_codewords: bad codebook / output layout");
  hipLaunchKernelGGL(gather_codewords_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     as_stream(stream), subset, B, n - B, codes, ldc, n_nodes, nb, D, emb_out, M,
                     ldw, emb_bstride, col_offset, xt, ldt, lcodes);
  return check_launch("gather_codewords");
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
                                   int32_t* t_perm, void* workspace, vqgnn_stream_t stream) {
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
                     perm, rows, val, n, n_cols, t_rowptr, t_col, t_val, t_perm);
  return check_launch("csr_transpose");
}

extern "C" int vqgnn_csr_expand_rows(const int32_t* rowptr, int32_t n_rows, int64_t nnz,
                                     int32_t* rows, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(nnz < (int64_t)INT32_MAX && n_rows >= 0, "csr_expand_rows: bad shape");
  if (nnz == 0) return VQGNN_OK;
  VQGNN_REQUIRE(rowptr && rows && n_rows > 0, "csr_expand_rows: null pointer");
  const int n = (int)nnz;
  hipLaunchKernelGGL(expand_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     rowptr, n_rows, rows, (int32_t*)nullptr, n);
  return check_launch("csr_expand_rows");
}
