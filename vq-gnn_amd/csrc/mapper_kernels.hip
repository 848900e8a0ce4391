// VQ-GNN v1 compressed adjacency for gfx950 (MI355X).
//
// Reference: vq_gnn_v1/utils/dataloader.py:144-192 (`mapper`), called per
// branch from vq_gnn_v1/models.py:170.  One branch's (B+M) x (B+M) adjacency
// in which every out-of-batch neighbour j is replaced by its codeword node
// B + c[j]: five COO parts concatenated, coalesced (torch_sparse: stable sort
// by row*dim + col, segment_csr sum), entries with a sum <= 0 dropped (the
// sign cancellation of the in-batch neighbours' codeword copies), self loops
// appended (non-SAGE), sorted (SparseTensor ctor) and, for GCN, symmetrised
// (to_symmetric: A and A^T concatenated, sorted, repeats summed).
//
// Integer/byte work plus one fp32 segmented sum: no GEMM shape.  Every stage
// is a streaming pass (coalesced), a rocPRIM radix sort (LSD: stable, so the
// repeated keys keep their concatenation order) or a scan; the sums run one
// thread per unique key, sequentially in sorted order — bit-identical to
// segment_csr's CPU loop.

#include "common.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

namespace vqgnn {

struct MapperIn {
  const int32_t *bn_row, *bn_col;
  const float *bn_val, *nb_val;
  int64_t E;
  const int32_t *bb_row, *bb_col;
  const float* bb_val;
  int64_t E2;
  const int64_t* batch_idx;
  int B, M;
  const int16_t* codes;
  int64_t ldc;
  int64_t* status;
};

__device__ __forceinline__ int64_t map_code(const MapperIn& a, int64_t node) {
  const int code = a.codes[node * a.ldc];
  if (code < 0 || code >= a.M) {
    atomicOr(reinterpret_cast<unsigned long long*>(a.status), 1ull);
    return a.B;
  }
  return (int64_t)a.B + code;
}

// entry i of the concatenation [P0 | P1 | P2 | P3 | P4] -> (key, value)
__global__ void mapper_build_kernel(MapperIn a, int64_t n, unsigned long long* __restrict__ keys,
                                    float* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t dim = (int64_t)a.B + a.M;
  const bool nb = a.nb_val != nullptr;
  int64_t r, c;
  float v;
  int64_t k = i;
  if (k < a.E) {                                  // P0 A_BN: (r, B + c[j], v)
    r = a.bn_row[k];
    c = map_code(a, a.bn_col[k]);
    v = a.bn_val[k];
  } else if (k -= a.E, nb && k < a.E) {          // P1 A_NB: (B + c[j], r, v_nb)
    r = map_code(a, a.bn_col[k]);
    c = a.bn_row[k];
    v = a.nb_val[k];
  } else {
    if (nb) k -= a.E;
    if (k < a.E2) {                               // P2 A_BB: (r, s, v)
      r = a.bb_row[k];
      c = a.bb_col[k];
      v = a.bb_val[k];
    } else if (k -= a.E2, k < a.E2) {             // P3: (r, B + c[batch_idx[s]], -v)
      r = a.bb_row[k];
      c = map_code(a, a.batch_idx[a.bb_col[k]]);
      v = -1.0f * a.bb_val[k];
    } else {                                      // P4: (B + c[batch_idx[r]], s, -v)
      k -= a.E2;
      r = map_code(a, a.batch_idx[a.bb_row[k]]);
      c = a.bb_col[k];
      v = -1.0f * a.bb_val[k];
    }
  }
  keys[i] = (unsigned long long)(r * dim + c);
  vals[i] = v;
}

// head[i] = 1 where a new key starts (sorted keys)
__global__ void mapper_heads_kernel(const unsigned long long* __restrict__ k, int64_t n,
                                    int32_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) head[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

// start of every run of equal keys: starts[pos[i] - 1] = i at each head;
// starts[nu] = n closes the last run
__global__ void mapper_starts_kernel(const int32_t* __restrict__ head,
                                     const int32_t* __restrict__ pos, int64_t n,
                                     int32_t* __restrict__ starts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && head[i]) starts[pos[i] - 1] = (int32_t)i;
  if (i == n - 1) starts[pos[i]] = (int32_t)n;
}

// one thread per unique key: sequential fp32 sum from 0 over its run (the
// segment_csr loop), values fetched 8 at a time ahead of the in-order adds.
// positive_only: keep flag = sum > 0 (the value_input > 0 slice).  The
// padding key (dim*dim, above every entry, sorted last) is never summed.
__global__ void mapper_segsum_kernel(const unsigned long long* __restrict__ k,
                                     const float* __restrict__ v,
                                     const int32_t* __restrict__ starts,
                                     const int32_t* __restrict__ nu_dev,
                                     unsigned long long* __restrict__ uk, float* __restrict__ us,
                                     int32_t* __restrict__ keep, int positive_only,
                                     unsigned long long pad) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= *nu_dev) return;
  const int64_t a = starts[u], b = starts[u + 1];
  const unsigned long long key = k[a];
  float s = 0.f;
  if (key != pad) {
    for (int64_t j = a; j < b; j += 8) {
      float t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) t[q] = j + q < b ? v[j + q] : 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (j + q < b) s = __fadd_rn(s, t[q]);
    }
  }
  uk[u] = key;
  us[u] = s;
  if (keep) keep[u] = positive_only ? (s > 0.f ? 1 : 0) : 1;
}

// compaction of (uk, us) by keep (kpos = inclusive scan), then the B self
// loops (i, i, deg_inv[i]) appended behind the survivors
__global__ void mapper_compact_kernel(const unsigned long long* __restrict__ uk,
                                      const float* __restrict__ us,
                                      const int32_t* __restrict__ keep,
                                      const int32_t* __restrict__ kpos, int64_t nu,
                                      const int32_t* __restrict__ nu_dev, int B, int64_t dim,
                                      const float* __restrict__ deg_inv,
                                      unsigned long long* __restrict__ ok, float* __restrict__ ov,
                                      int64_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = *nu_dev;   // unique keys (device)
  const int64_t kept = m > 0 ? kpos[m - 1] : 0;
  if (i < m && keep[i]) {
    ok[kpos[i] - 1] = uk[i];
    ov[kpos[i] - 1] = us[i];
  }
  if (deg_inv && i < B) {
    ok[kept + i] = (unsigned long long)(i * dim + i);
    ov[kept + i] = deg_inv[i];
  }
  if (i == 0) *count = kept + (deg_inv ? B : 0);
  (void)nu;
}

// to_symmetric input: entry i < n -> (r, c), i >= n -> (c, r)
__global__ void mapper_sym_kernel(const unsigned long long* __restrict__ k,
                                  const float* __restrict__ v, const int64_t* __restrict__ count,
                                  int64_t dim, unsigned long long* __restrict__ k2,
                                  float* __restrict__ v2, int64_t cap, unsigned long long pad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = *count;
  if (i >= cap) return;
  if (i < n) {
    k2[i] = k[i];
    v2[i] = v[i];
    const uint64_t r = k[i] / dim, c = k[i] % dim;
    k2[n + i] = c * dim + r;
    v2[n + i] = v[i];
  } else if (i >= 2 * n && i < cap) {
    k2[i] = pad;   // padding sorts last
    v2[i] = 0.f;
  }
}

__global__ void mapper_pad_kernel(unsigned long long* __restrict__ k, float* __restrict__ v,
                                  const int64_t* __restrict__ count, int64_t cap,
                                  unsigned long long pad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap && i >= *count) {
    k[i] = pad;
    v[i] = 0.f;
  }
}

__global__ void mapper_count_kernel(const int32_t* __restrict__ nu,
                                    const unsigned long long* __restrict__ k,
                                    int64_t* __restrict__ count, unsigned long long pad) {
  const int64_t m = *nu;
  *count = (m > 0 && k[m - 1] == pad) ? m - 1 : m;
}

// CSR from sorted keys: rowptr[r] = first entry with row >= r; col, val
__global__ void mapper_csr_kernel(const unsigned long long* __restrict__ k,
                                  const float* __restrict__ v, const int64_t* __restrict__ count,
                                  int64_t dim, int64_t* __restrict__ rowptr,
                                  int32_t* __restrict__ col, float* __restrict__ val) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = *count;
  if (i < n) {
    col[i] = (int32_t)(k[i] % dim);
    val[i] = v[i];
  }
  if (i <= dim) {
    const unsigned long long key = (unsigned long long)i * dim;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (k[mid] < key) lo = mid + 1; else hi = mid;
    }
    rowptr[i] = lo;
  }
}

static int key_bits(int64_t dim) {
  const unsigned long long mx = (unsigned long long)dim * (unsigned long long)dim;
  int b = 1;
  while (b < 64 && (1ull << b) < mx) ++b;
  return b;
}

struct MapperWs {
  unsigned long long *k0, *k1, *k2;
  float *v0, *v1, *v2;
  int32_t *head, *pos, *keep, *kpos, *nu, *starts;
  int64_t* count;
  void* temp;
  size_t temp_bytes;
};

static int64_t mapper_inputs(int64_t E, int64_t E2, int nb, int bb) {
  return E + (nb ? E : 0) + (bb ? (nb ? 3 : 2) * E2 : 0);
}

static MapperWs mapper_ws(void* ws, int64_t cap, size_t* total) {
  MapperWs w{};
  char* p = reinterpret_cast<char*>(ws);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = p ? p + off : nullptr;
    off += align_up(bytes > 0 ? bytes : 1, 256);
    return q;
  };
  const size_t c = (size_t)(cap > 0 ? cap : 1);
  w.k0 = (unsigned long long*)take(c * 8);
  w.k1 = (unsigned long long*)take(c * 8);
  w.k2 = (unsigned long long*)take(c * 8);
  w.v0 = (float*)take(c * 4);
  w.v1 = (float*)take(c * 4);
  w.v2 = (float*)take(c * 4);
  w.head = (int32_t*)take(c * 4);
  w.pos = (int32_t*)take(c * 4);
  w.keep = (int32_t*)take(c * 4);
  w.kpos = (int32_t*)take(c * 4);
  w.starts = (int32_t*)take(c * 4 + 4);
  w.nu = (int32_t*)take(256);
  w.count = (int64_t*)take(256);
  size_t a = 0, b = 0;
  (void)rocprim::radix_sort_pairs(nullptr, a, (const unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (const float*)nullptr,
                                  (float*)nullptr, c, 0, 64, (hipStream_t)0);
  (void)rocprim::inclusive_scan(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr, c,
                                rocprim::plus<int32_t>(), (hipStream_t)0);
  w.temp_bytes = a > b ? a : b;
  w.temp = take(w.temp_bytes);
  if (total) *total = off;
  return w;
}

// sort (k_in, v_in)[0, n) -> (k_out, v_out); coalesce with sequential sums ->
// (uk, us) + keep flags; the unique count lands in *nu (device)
static hipError_t sort_coalesce(MapperWs& w, unsigned long long* k_in, float* v_in, int64_t n,
                                int bits, unsigned long long* k_out, float* v_out,
                                unsigned long long* uk, float* us, int positive_only,
                                unsigned long long pad, hipStream_t s) {
  size_t tb = w.temp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(w.temp, tb, k_in, k_out, v_in, v_out, (size_t)n, 0,
                                           bits, s);
  if (e != hipSuccess) return e;
  const int nbk = (int)((n + 255) / 256);
  hipLaunchKernelGGL(mapper_heads_kernel, dim3(nbk), dim3(256), 0, s, k_out, n, w.head);
  tb = w.temp_bytes;
  e = rocprim::inclusive_scan(w.temp, tb, w.head, w.pos, (size_t)n, rocprim::plus<int32_t>(), s);
  if (e != hipSuccess) return e;
  // unique count = pos[n-1]
  (void)hipMemcpyAsync(w.nu, w.pos + (n - 1), sizeof(int32_t), hipMemcpyDeviceToDevice, s);
  hipLaunchKernelGGL(mapper_starts_kernel, dim3(nbk), dim3(256), 0, s, w.head, w.pos, n,
                     w.starts);
  hipLaunchKernelGGL(mapper_segsum_kernel, dim3(nbk), dim3(256), 0, s, k_out, v_out, w.starts,
                     w.nu, uk, us, w.keep, positive_only, pad);
  return hipSuccess;
}

}  // namespace vqgnn

using namespace vqgnn;

extern "C" int64_t vqgnn_mapper_capacity(int64_t E, int64_t E2, int32_t B, int32_t has_nb,
                                         int32_t has_bb, int32_t conv_type) {
  const int64_t n = mapper_inputs(E, E2, has_nb, has_bb) + (conv_type != VQGNN_CONV_SAGE ? B : 0);
  return conv_type == VQGNN_CONV_GCN ? 2 * n : n;
}

extern "C" size_t vqgnn_mapper_workspace(int64_t E, int64_t E2, int32_t B, int32_t has_nb,
                                         int32_t has_bb) {
  const int64_t cap = 2 * (mapper_inputs(E, E2, has_nb, has_bb) + B) + 1;
  size_t total = 0;
  (void)mapper_ws(nullptr, cap, &total);
  return total;
}

extern "C" int vqgnn_mapper(const int32_t* bn_row, const int32_t* bn_col, const float* bn_val,
                            int64_t E, const float* nb_val, const int32_t* bb_row,
                            const int32_t* bb_col, const float* bb_val, int64_t E2,
                            const int64_t* batch_idx, int32_t B, const int16_t* codes,
                            int64_t ldc, int32_t M, const float* deg_inv, int32_t conv_type,
                            int64_t* out_rowptr, int32_t* out_col, float* out_val,
                            int64_t* out_nnz, int64_t* status, void* workspace,
                            vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(B >= 0 && M > 0 && E >= 0 && E2 >= 0 && ldc >= 1, "mapper: bad shape");
  VQGNN_REQUIRE(conv_type == VQGNN_CONV_GCN || conv_type == VQGNN_CONV_SAGE ||
                    conv_type == VQGNN_CONV_GAT,
                "mapper: bad conv_type %d", conv_type);
  VQGNN_REQUIRE(out_rowptr && out_nnz && status && workspace && codes, "mapper: null pointer");
  VQGNN_REQUIRE(E == 0 || (bn_row && bn_col && bn_val), "mapper: A_BN pointers");
  const bool bb = bb_row != nullptr;
  VQGNN_REQUIRE(!bb || (bb_col && bb_val && batch_idx), "mapper: A_BB pointers");
  VQGNN_REQUIRE(conv_type == VQGNN_CONV_SAGE || B == 0 || deg_inv,
                "mapper: deg_inv needed for self loops");
  const int64_t dim = (int64_t)B + M;
  VQGNN_REQUIRE(dim < (int64_t)INT32_MAX, "mapper: B + M too large");
  hipStream_t s = as_stream(stream);
  const int64_t n_in = mapper_inputs(E, bb ? E2 : 0, nb_val != nullptr, bb);
  const int64_t cap = 2 * (n_in + B) + 1;
  MapperWs w = mapper_ws(workspace, cap, nullptr);
  (void)hipMemsetAsync(status, 0, sizeof(int64_t), s);
  (void)hipMemsetAsync(w.count, 0, sizeof(int64_t), s);
  (void)hipMemsetAsync(w.nu, 0, sizeof(int32_t), s);
  // keys are row * dim + col < dim^2; dim^2 pads the fixed-capacity sorts
  const unsigned long long pad = (unsigned long long)dim * (unsigned long long)dim;
  const int bits = key_bits(dim) + 1;
  MapperIn a{bn_row, bn_col, bn_val, nb_val, E, bb_row, bb_col, bb_val, bb ? E2 : 0,
             batch_idx, B, M, codes, ldc, status};
  hipError_t e = hipSuccess;
  if (n_in > 0) {
    hipLaunchKernelGGL(mapper_build_kernel, dim3((n_in + 255) / 256), dim3(256), 0, s, a, n_in,
                       w.k0, w.v0);
    // coalesce(): stable sort + sequential sums, then value > 0
    e = sort_coalesce(w, w.k0, w.v0, n_in, bits, w.k1, w.v1, w.k2, w.v2, 1, pad, s);
    if (e == hipSuccess) {
      size_t tb = w.temp_bytes;
      e = rocprim::inclusive_scan(w.temp, tb, w.keep, w.kpos, (size_t)n_in,
                                  rocprim::plus<int32_t>(), s);
    }
  }
  if (e != hipSuccess) {
    set_error("mapper: rocPRIM failed: %s", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  const float* loops = conv_type != VQGNN_CONV_SAGE ? deg_inv : nullptr;
  {
    const int64_t m = n_in > B ? n_in : B;
    hipLaunchKernelGGL(mapper_compact_kernel, dim3((m + 255) / 256 + 1), dim3(256), 0, s, w.k2,
                       w.v2, w.keep, w.kpos, n_in, w.nu, B, dim, loops, w.k0, w.v0, w.count);
  }
  const int64_t n1 = n_in + (loops ? B : 0);   // capacity of the list
  // SparseTensor(row=, col=, value=): stable sort (self loops behind equal keys)
  hipLaunchKernelGGL(mapper_pad_kernel, dim3((n1 + 255) / 256 + 1), dim3(256), 0, s, w.k0, w.v0,
                     w.count, n1, pad);
  size_t tb = w.temp_bytes;
  if (n1 > 0)
    e = rocprim::radix_sort_pairs(w.temp, tb, w.k0, w.k1, w.v0, w.v1, (size_t)n1, 0, bits, s);
  if (e != hipSuccess) {
    set_error("mapper: sort failed: %s", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  unsigned long long* fk = w.k1;
  float* fv = w.v1;
  if (conv_type == VQGNN_CONV_GCN && n1 > 0) {
    // to_symmetric(): [A ; A^T] sorted, repeats summed sequentially
    const int64_t n2 = 2 * n1;
    hipLaunchKernelGGL(mapper_sym_kernel, dim3((n2 + 255) / 256), dim3(256), 0, s, w.k1, w.v1,
                       w.count, dim, w.k0, w.v0, n2, pad);
    e = sort_coalesce(w, w.k0, w.v0, n2, bits, w.k1, w.v1, w.k2, w.v2, 0, pad, s);
    if (e != hipSuccess) {
      set_error("mapper: symmetric coalesce failed: %s", hipGetErrorString(e));
      return VQGNN_ERR_LAUNCH;
    }
    // the padding keys form one trailing unique key: not an entry
    hipLaunchKernelGGL(mapper_count_kernel, dim3(1), dim3(1), 0, s, w.nu, w.k2, w.count, pad);
    fk = w.k2;
    fv = w.v2;
  }
  hipLaunchKernelGGL(mapper_csr_kernel, dim3((cap + dim + 255) / 256 + 1), dim3(256), 0, s, fk, fv,
                     w.count, dim, out_rowptr, out_col, out_val);
  (void)hipMemcpyAsync(out_nnz, w.count, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
  return check_launch("mapper");
}
