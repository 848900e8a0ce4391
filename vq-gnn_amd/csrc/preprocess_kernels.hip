// Full-graph preprocessing on the device:
//   norm_adj              vq_gnn_v2/utils/misc.py:14-34
//   SparseTensor.to_symmetric (get_data, misc.py:190/211; torch_sparse, reduce='sum')
//   SparseTensor.permute  (permute, misc.py:113-130)
//   metis substitute      (metis, misc.py:93-111: METIS itself is the
//                          third-party library torch_sparse.partition wraps;
//                          absent here — this orders nodes by a BFS from each
//                          connected component's smallest node and cuts the
//                          order into equal bands)
// Integer / index work plus per-row fp32 sums and one multiply chain per
// entry; no reshaping into GEMMs.
#include "common.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

namespace vqgnn {

namespace {

constexpr int kPpThreads = 256;
constexpr int kPpWaves = kPpThreads / 64;

template <typename T>
T* carve(char*& p, size_t count) {
  T* r = reinterpret_cast<T*>(p);
  p += align_up(count * sizeof(T), 256);
  return r;
}

__device__ __forceinline__ unsigned long long below_mask(int lane) {
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// ---- norm_adj -------------------------------------------------------------

// 1 if row i holds its diagonal entry (columns sorted)
__device__ __forceinline__ bool row_has_diag(const int64_t* rowptr, const int32_t* col, int64_t i) {
  int64_t lo = rowptr[i], hi = rowptr[i + 1];
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (col[mid] < i) lo = mid + 1;
    else hi = mid;
  }
  return lo < rowptr[i + 1] && col[lo] == i;
}

__global__ void __launch_bounds__(kPpThreads)
na_count_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col, int64_t N,
                int self_loops, int64_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (i >= N) return;
  int64_t c = rowptr[i + 1] - rowptr[i];
  if (self_loops) c += row_has_diag(rowptr, col, i) ? 0 : 1;   // set_diag: replace or insert
  count[i] = c;
}

// one wave per row: the row's entries (set_diag: the old diagonal dropped,
// a diagonal of value 1 inserted in column order)
__global__ void __launch_bounds__(kPpThreads)
na_fill_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
               const float* __restrict__ val, int64_t N, int self_loops,
               const int64_t* __restrict__ optr, int32_t* __restrict__ ocol,
               float* __restrict__ oval) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kPpWaves + (threadIdx.x >> 6);
  if (i >= N) return;
  const int64_t e0 = rowptr[i], e1 = rowptr[i + 1];
  int64_t base = optr[i];
  const unsigned long long below = below_mask(lane);
  bool inserted = !self_loops;
  for (int64_t eb = e0; eb < e1; eb += 64) {
    const int64_t e = eb + lane;
    int c = -1;
    bool keep = false;
    if (e < e1) {
      c = col[e];
      keep = !(self_loops && c == i);
    }
    // the diagonal goes before the first kept column > i
    const unsigned long long after = __ballot(keep && c > i);
    if (!inserted && after) {
      const int first = __ffsll((long long)after) - 1;
      const unsigned long long m = __ballot(keep);
      const int pos = __popcll(m & below_mask(first));
      if (lane == 0) {
        ocol[base + pos] = (int32_t)i;
        oval[base + pos] = 1.0f;
      }
      if (keep) {
        const int p = __popcll(m & below) + (c > i ? 1 : 0);
        ocol[base + p] = c;
        oval[base + p] = val ? val[e] : 1.0f;
      }
      base += __popcll(m) + 1;
      inserted = true;
      continue;
    }
    const unsigned long long m = __ballot(keep);
    if (keep) {
      const int p = __popcll(m & below);
      ocol[base + p] = c;
      oval[base + p] = val ? val[e] : 1.0f;
    }
    base += __popcll(m);
  }
  if (!inserted && lane == 0) {
    ocol[base] = (int32_t)i;
    oval[base] = 1.0f;
  }
}

// deg = adj_t.sum(dim=1): a sequential fp32 sum per row (torch_scatter's CPU
// segment_csr); then deg.pow(-1/2) (ATen: 1 / sqrt) or deg.pow(-1) (1 / x),
// inf -> 0
__global__ void __launch_bounds__(kPpThreads)
na_deg_kernel(const int64_t* __restrict__ optr, const float* __restrict__ oval, int64_t N,
              int gcn, float* __restrict__ scale) {
  const int64_t i = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (i >= N) return;
  float d = 0.f;
  for (int64_t e = optr[i]; e < optr[i + 1]; ++e) d = __fadd_rn(d, oval[e]);
  float s = gcn ? __fdiv_rn(1.0f, __fsqrt_rn(d)) : __fdiv_rn(1.0f, d);
  if (isinf(s)) s = 0.f;
  scale[i] = s;
}

// GCN: v = (dis[row] * v) * dis[col]; SAGE / GAT: v = di[row] * v
__global__ void __launch_bounds__(kPpThreads)
na_scale_kernel(const int64_t* __restrict__ optr, const int32_t* __restrict__ ocol, int64_t N,
                int gcn, const float* __restrict__ scale, float* __restrict__ oval) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kPpWaves + (threadIdx.x >> 6);
  if (i >= N) return;
  const float si = scale[i];
  for (int64_t e = optr[i] + lane; e < optr[i + 1]; e += 64) {
    float v = __fmul_rn(si, oval[e]);
    if (gcn) v = __fmul_rn(v, scale[ocol[e]]);
    oval[e] = v;
  }
}

// ---- COO -> sorted keys ------------------------------------------------------

// keys of A (and, sym, of A^T): (row, col) -> row * N + col
__global__ void __launch_bounds__(kPpThreads)
sym_keys_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                const float* __restrict__ val, int64_t N, int64_t nnz,
                unsigned long long* __restrict__ keys, float* __restrict__ vals) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kPpWaves + (threadIdx.x >> 6);
  if (r >= N) return;
  for (int64_t e = rowptr[r] + lane; e < rowptr[r + 1]; e += 64) {
    const int64_t c = col[e];
    const float v = val ? val[e] : 1.0f;
    keys[e] = (unsigned long long)r * (unsigned long long)N + (unsigned long long)c;
    vals[e] = v;
    keys[nnz + e] = (unsigned long long)c * (unsigned long long)N + (unsigned long long)r;
    vals[nnz + e] = v;
  }
}

// unique sorted keys -> col, rowptr; values: summed duplicates or 1 (pattern)
__global__ void __launch_bounds__(kPpThreads)
keys_to_csr_kernel(const unsigned long long* __restrict__ keys, const float* __restrict__ sums,
                   const long long* __restrict__ count, int64_t N, int pattern,
                   int64_t* __restrict__ optr, int32_t* __restrict__ ocol,
                   float* __restrict__ oval) {
  const int64_t i = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  const int64_t n = *count;
  if (i >= n) {
    if (n == 0 && i <= N) optr[i] = 0;
    return;
  }
  const unsigned long long k = keys[i];
  const int64_t r = (int64_t)(k / (unsigned long long)N);
  ocol[i] = (int32_t)(k % (unsigned long long)N);
  oval[i] = pattern ? 1.0f : sums[i];
  const int64_t rp = i > 0 ? (int64_t)(keys[i - 1] / (unsigned long long)N) : -1;
  for (int64_t q = rp + 1; q <= r; ++q) optr[q] = i;
  if (i == n - 1)
    for (int64_t q = r + 1; q <= N; ++q) optr[q] = n;
}

// ---- permute ---------------------------------------------------------------

__global__ void __launch_bounds__(kPpThreads)
perm_inverse_kernel(const int64_t* __restrict__ perm, int64_t N, int32_t* __restrict__ inv,
                    unsigned long long* __restrict__ status) {
  const int64_t i = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (i >= N) return;
  const int64_t p = perm[i];
  if (p < 0 || p >= N) {
    atomicOr(status, 1ull);
    return;
  }
  inv[p] = (int32_t)i;
}

__global__ void __launch_bounds__(kPpThreads)
perm_count_kernel(const int64_t* __restrict__ rowptr, const int64_t* __restrict__ perm,
                  int64_t N, int64_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (i >= N) return;
  const int64_t p = perm[i];
  count[i] = (p >= 0 && p < N) ? rowptr[p + 1] - rowptr[p] : 0;
}

// new row i = old row perm[i], columns relabelled through inv (unsorted)
__global__ void __launch_bounds__(kPpThreads)
perm_fill_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                 const float* __restrict__ val, const int64_t* __restrict__ perm, int64_t N,
                 const int32_t* __restrict__ inv, const int64_t* __restrict__ optr,
                 int32_t* __restrict__ tcol, float* __restrict__ tval) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kPpWaves + (threadIdx.x >> 6);
  if (i >= N) return;
  const int64_t p = perm[i];
  if (p < 0 || p >= N) return;
  const int64_t e0 = rowptr[p], o = optr[i] - e0;
  for (int64_t e = e0 + lane; e < rowptr[p + 1]; e += 64) {
    tcol[o + e] = inv[col[e]];
    tval[o + e] = val ? val[e] : 1.0f;
  }
}

// ---- METIS substitute: components, BFS levels, ordering ----------------------

__global__ void __launch_bounds__(kPpThreads)
cc_init_kernel(int64_t N, int32_t* __restrict__ label, int32_t* __restrict__ level) {
  const int64_t i = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (i >= N) return;
  label[i] = (int32_t)i;
  level[i] = -1;
}

// label[v] = min over v's neighbours' labels (and its own); changed -> flag
__global__ void __launch_bounds__(kPpThreads)
cc_step_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col, int64_t N,
               int32_t* __restrict__ label, int* __restrict__ changed) {
  const int lane = threadIdx.x & 63;
  const int64_t v = (int64_t)blockIdx.x * kPpWaves + (threadIdx.x >> 6);
  if (v >= N) return;
  int m = label[v];
  for (int64_t e = rowptr[v] + lane; e < rowptr[v + 1]; e += 64) m = min(m, label[col[e]]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
  if (lane == 0 && m < label[v]) {
    atomicMin(label + v, m);
    *changed = 1;
  }
}

// pointer jumping: label[v] = label[label[v]]
__global__ void __launch_bounds__(kPpThreads)
cc_jump_kernel(int64_t N, int32_t* __restrict__ label) {
  const int64_t v = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (v >= N) return;
  const int l = label[v];
  const int ll = label[l];
  if (ll < l) label[v] = ll;
}

// level 0 = each component's smallest node
__global__ void __launch_bounds__(kPpThreads)
bfs_seed_kernel(int64_t N, const int32_t* __restrict__ label, int32_t* __restrict__ level) {
  const int64_t v = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (v >= N) return;
  if (label[v] == v) level[v] = 0;
}

// one wave per node at level d: unvisited neighbours -> d + 1
__global__ void __launch_bounds__(kPpThreads)
bfs_step_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col, int64_t N,
                int d, int32_t* __restrict__ level, int* __restrict__ grew) {
  const int lane = threadIdx.x & 63;
  const int64_t v = (int64_t)blockIdx.x * kPpWaves + (threadIdx.x >> 6);
  if (v >= N || level[v] != d) return;
  bool any = false;
  for (int64_t e = rowptr[v] + lane; e < rowptr[v + 1]; e += 64) {
    const int u = col[e];
    if (level[u] < 0) {
      level[u] = d + 1;
      any = true;
    }
  }
  if (__ballot(any) && lane == 0) *grew = 1;
}

// key = (component label, BFS level); values = node ids (ascending: a stable
// sort keeps id order within a level)
__global__ void __launch_bounds__(kPpThreads)
order_keys_kernel(int64_t N, const int32_t* __restrict__ label, const int32_t* __restrict__ level,
                  unsigned long long* __restrict__ keys, int64_t* __restrict__ ids) {
  const int64_t v = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (v >= N) return;
  keys[v] = ((unsigned long long)(uint32_t)label[v] << 32) | (uint32_t)level[v];
  ids[v] = v;
}

// initial bands: the node at position i of the BFS order -> part i*k/N
__global__ void __launch_bounds__(kPpThreads)
band_init_kernel(const int64_t* __restrict__ order, int64_t N, int parts,
                 int32_t* __restrict__ part, int32_t* __restrict__ size) {
  const int64_t i = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (i >= N) return;
  const int q = (int)(i * parts / N);
  part[order[i]] = q;
  atomicAdd(size + q, 1);
}

// Label propagation step, wave per node: the most frequent partition among the
// neighbours (ties: the smallest id), wanted if strictly more frequent than
// the node's own.  LDS histogram of `parts` bins per wave.
constexpr int kMaxParts = 1024;
__global__ void __launch_bounds__(kPpThreads)
lpa_want_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col, int64_t N,
                int parts, const int32_t* __restrict__ part, unsigned long long* __restrict__ key,
                int64_t* __restrict__ ids) {
  __shared__ int hist[kPpWaves][kMaxParts];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t v = (int64_t)blockIdx.x * kPpWaves + w;
  int* h = hist[w];
  for (int q = lane; q < parts; q += 64) h[q] = 0;
  __syncthreads();
  if (v < N)
    for (int64_t e = rowptr[v] + lane; e < rowptr[v + 1]; e += 64) atomicAdd(h + part[col[e]], 1);
  __syncthreads();
  if (v >= N) return;
  int bc = -1, bq = 0;
  for (int q = lane; q < parts; q += 64)
    if (h[q] > bc) { bc = h[q]; bq = q; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int oc = __shfl_xor(bc, o), oq = __shfl_xor(bq, o);
    if (oc > bc || (oc == bc && oq < bq)) { bc = oc; bq = oq; }
  }
  if (lane == 0) {
    const int p = part[v], cur = h[p];
    const bool want = bq != p && bc > cur;
    // moves grouped by target, best gain first; node ids stay ascending
    key[v] = want ? ((unsigned long long)bq << 32) | (0xFFFFFFFFull - (unsigned)(bc - cur))
                  : ~0ull;
    ids[v] = v;
  }
}

// the moves into a target are taken in (gain, id) order while it has room
// (capacity against the sizes at the start of the step)
__global__ void __launch_bounds__(kPpThreads)
lpa_move_kernel(const unsigned long long* __restrict__ skey, const int64_t* __restrict__ sids,
                int64_t N, int cap, const int32_t* __restrict__ size,
                int32_t* __restrict__ part, int32_t* __restrict__ new_size) {
  const int64_t i = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (i >= N) return;
  const unsigned long long k = skey[i];
  if (k == ~0ull) return;
  const unsigned q = (unsigned)(k >> 32);
  int64_t lo = 0, hi = i;                       // first index of target q
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((unsigned)(skey[mid] >> 32) < q) lo = mid + 1;
    else hi = mid;
  }
  if (i - lo >= (int64_t)cap - size[q]) return;
  const int64_t v = sids[i];
  const int p = part[v];
  part[v] = (int32_t)q;
  atomicAdd(new_size + q, 1);
  atomicSub(new_size + p, 1);
}

// final order key: (partition, BFS level), node ids ascending
__global__ void __launch_bounds__(kPpThreads)
part_keys_kernel(int64_t N, const int32_t* __restrict__ part, const int32_t* __restrict__ level,
                 unsigned long long* __restrict__ keys, int64_t* __restrict__ ids) {
  const int64_t v = (int64_t)blockIdx.x * kPpThreads + threadIdx.x;
  if (v >= N) return;
  keys[v] = ((unsigned long long)(uint32_t)part[v] << 32) | (uint32_t)level[v];
  ids[v] = v;
}

__global__ void parts_ptr_kernel(const int32_t* __restrict__ size, int parts,
                                 int64_t* __restrict__ ptr) {
  int64_t a = 0;
  ptr[0] = 0;
  for (int k = 0; k < parts; ++k) {
    a += size[k];
    ptr[k + 1] = a;
  }
}

constexpr int kLpaSteps = 12;

int bits64(unsigned long long x) {
  int b = 1;
  while (b < 64 && (x >> b)) ++b;
  return b;
}

size_t scan64_temp(int64_t n) {
  size_t bytes = 0;
  (void)rocprim::inclusive_scan(nullptr, bytes, (const int64_t*)nullptr, (int64_t*)nullptr,
                                (size_t)(n > 0 ? n : 1), rocprim::plus<int64_t>(), (hipStream_t)0);
  return bytes;
}

int scan_rowptr(void* temp, size_t bytes, const int64_t* count, int64_t* optr, int64_t N,
                hipStream_t s, const char* what) {
  (void)hipMemsetAsync(optr, 0, sizeof(int64_t), s);
  if (N == 0) return check_launch(what);
  const hipError_t e = rocprim::inclusive_scan(temp, bytes, count, optr + 1, (size_t)N,
                                               rocprim::plus<int64_t>(), s);
  if (e != hipSuccess) {
    set_error("%s: scan failed: %s", what, hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  return check_launch(what);
}

dim3 grid_rows(int64_t N) { return dim3((unsigned)((N + kPpThreads - 1) / kPpThreads)); }
dim3 grid_waves(int64_t N) { return dim3((unsigned)((N + kPpWaves - 1) / kPpWaves)); }

}  // namespace

}  // namespace vqgnn

using namespace vqgnn;

extern "C" size_t vqgnn_norm_adj_workspace(int64_t N) {
  return align_up((size_t)(N > 0 ? N : 1) * 8, 256) + align_up((size_t)(N > 0 ? N : 1) * 4, 256) +
         align_up(scan64_temp(N), 256) + 256;
}

extern "C" int vqgnn_norm_adj(const int64_t* rowptr, const int32_t* col, const float* val,
                              int64_t N, int32_t conv_type, int64_t* out_rowptr,
                              int32_t* out_col, float* out_val, void* workspace,
                              vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(N >= 0 && N < (int64_t)INT32_MAX, "norm_adj: bad N");
  VQGNN_REQUIRE(conv_type >= VQGNN_CONV_GCN && conv_type <= VQGNN_CONV_GAT,
                "norm_adj: GNN conv type not supported");
  VQGNN_REQUIRE(out_rowptr && workspace && (N == 0 || (rowptr && col && out_col && out_val)),
                "norm_adj: null pointer");
  hipStream_t s = as_stream(stream);
  char* p = reinterpret_cast<char*>(workspace);
  int64_t* count = carve<int64_t>(p, N > 0 ? N : 1);
  float* scale = carve<float>(p, N > 0 ? N : 1);
  const size_t tb = align_up(scan64_temp(N), 256);
  void* temp = p;
  const int loops = conv_type != VQGNN_CONV_SAGE;    // GCN, GAT: set_diag()
  const int gcn = conv_type == VQGNN_CONV_GCN;
  if (N == 0) return scan_rowptr(temp, tb, count, out_rowptr, 0, s, "norm_adj");
  hipLaunchKernelGGL(na_count_kernel, grid_rows(N), dim3(kPpThreads), 0, s, rowptr, col, N, loops,
                     count);
  int rc = scan_rowptr(temp, tb, count, out_rowptr, N, s, "norm_adj(rowptr)");
  if (rc) return rc;
  hipLaunchKernelGGL(na_fill_kernel, grid_waves(N), dim3(kPpThreads), 0, s, rowptr, col, val, N,
                     loops, out_rowptr, out_col, out_val);
  hipLaunchKernelGGL(na_deg_kernel, grid_rows(N), dim3(kPpThreads), 0, s, out_rowptr, out_val, N,
                     gcn, scale);
  hipLaunchKernelGGL(na_scale_kernel, grid_waves(N), dim3(kPpThreads), 0, s, out_rowptr, out_col,
                     N, gcn, scale, out_val);
  return check_launch("norm_adj");
}

extern "C" size_t vqgnn_to_symmetric_workspace(int64_t N, int64_t nnz) {
  const size_t n2 = (size_t)(nnz > 0 ? 2 * nnz : 1);
  size_t sort_bytes = 0, rbk_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_bytes, (const unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (const float*)nullptr,
                                  (float*)nullptr, n2, 0, 64, (hipStream_t)0);
  (void)rocprim::reduce_by_key(nullptr, rbk_bytes, (const unsigned long long*)nullptr,
                               (const float*)nullptr, n2, (unsigned long long*)nullptr,
                               (float*)nullptr, (long long*)nullptr, rocprim::plus<float>(),
                               rocprim::equal_to<unsigned long long>(), (hipStream_t)0);
  (void)N;
  return 3 * align_up(n2 * 8, 256) + 3 * align_up(n2 * 4, 256) +
         align_up(sort_bytes > rbk_bytes ? sort_bytes : rbk_bytes, 256) + 512;
}

extern "C" int vqgnn_to_symmetric(const int64_t* rowptr, const int32_t* col, const float* val,
                                  int64_t N, int64_t nnz, int64_t* out_rowptr, int32_t* out_col,
                                  float* out_val, int64_t* out_nnz, void* workspace,
                                  vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(N >= 0 && N < (int64_t)INT32_MAX && nnz >= 0 && 2 * nnz < ((int64_t)1 << 40),
                "to_symmetric: bad shape");
  VQGNN_REQUIRE(out_rowptr && out_nnz && workspace, "to_symmetric: null pointer");
  hipStream_t s = as_stream(stream);
  (void)hipMemsetAsync(out_nnz, 0, sizeof(int64_t), s);
  if (nnz == 0 || N == 0) {
    (void)hipMemsetAsync(out_rowptr, 0, (size_t)(N + 1) * 8, s);
    return check_launch("to_symmetric(empty)");
  }
  VQGNN_REQUIRE(rowptr && col && out_col && out_val, "to_symmetric: null pointer");
  const size_t n2 = (size_t)(2 * nnz);
  char* p = reinterpret_cast<char*>(workspace);
  auto* keys = carve<unsigned long long>(p, n2);
  auto* skeys = carve<unsigned long long>(p, n2);
  auto* ukeys = carve<unsigned long long>(p, n2);
  float* vals = carve<float>(p, n2);
  float* svals = carve<float>(p, n2);
  float* sums = carve<float>(p, n2);
  size_t sort_bytes = 0, rbk_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_bytes, (const unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (const float*)nullptr,
                                  (float*)nullptr, n2, 0, 64, s);
  (void)rocprim::reduce_by_key(nullptr, rbk_bytes, (const unsigned long long*)nullptr,
                               (const float*)nullptr, n2, (unsigned long long*)nullptr,
                               (float*)nullptr, (long long*)nullptr, rocprim::plus<float>(),
                               rocprim::equal_to<unsigned long long>(), s);
  void* temp = p;
  hipLaunchKernelGGL(sym_keys_kernel, grid_waves(N), dim3(kPpThreads), 0, s, rowptr, col, val, N,
                     nnz, keys, vals);
  int rc = check_launch("to_symmetric(keys)");
  if (rc) return rc;
  const int bits = bits64((unsigned long long)N * (unsigned long long)N);
  hipError_t e = rocprim::radix_sort_pairs(temp, sort_bytes, keys, skeys, vals, svals, n2, 0, bits, s);
  if (e == hipSuccess)
    e = rocprim::reduce_by_key(temp, rbk_bytes, skeys, svals, n2, ukeys, sums,
                               reinterpret_cast<long long*>(out_nnz), rocprim::plus<float>(),
                               rocprim::equal_to<unsigned long long>(), s);
  if (e != hipSuccess) {
    set_error("to_symmetric: rocPRIM failed: %s", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  const int64_t tot = (int64_t)n2 > N + 1 ? (int64_t)n2 : N + 1;
  hipLaunchKernelGGL(keys_to_csr_kernel, grid_rows(tot), dim3(kPpThreads), 0, s, ukeys, sums,
                     reinterpret_cast<const long long*>(out_nnz), N, val ? 0 : 1, out_rowptr,
                     out_col, out_val);
  return check_launch("to_symmetric");
}

extern "C" size_t vqgnn_csr_permute_workspace(int64_t N, int64_t nnz) {
  size_t bytes = 0;
  (void)rocprim::segmented_radix_sort_pairs(
      nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const float*)nullptr,
      (float*)nullptr, (size_t)(nnz > 0 ? nnz : 1), (unsigned)(N > 0 ? N : 1),
      (const int64_t*)nullptr, (const int64_t*)nullptr, 0, 32, (hipStream_t)0);
  const size_t n1 = (size_t)(N > 0 ? N : 1), e1 = (size_t)(nnz > 0 ? nnz : 1);
  return align_up(n1 * 4, 256) + align_up(n1 * 8, 256) + 2 * align_up(e1 * 4, 256) +
         align_up(bytes > scan64_temp(N) ? bytes : scan64_temp(N), 256) + 512;
}

extern "C" int vqgnn_csr_permute(const int64_t* rowptr, const int32_t* col, const float* val,
                                 int64_t N, int64_t nnz, const int64_t* perm, int64_t* out_rowptr,
                                 int32_t* out_col, float* out_val, int64_t* status,
                                 void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(N >= 0 && N < (int64_t)INT32_MAX && nnz >= 0 && nnz < (int64_t)INT32_MAX,
                "csr_permute: bad shape");
  VQGNN_REQUIRE(out_rowptr && status && workspace, "csr_permute: null pointer");
  hipStream_t s = as_stream(stream);
  (void)hipMemsetAsync(status, 0, sizeof(int64_t), s);
  char* p = reinterpret_cast<char*>(workspace);
  int32_t* inv = carve<int32_t>(p, N > 0 ? N : 1);
  int64_t* count = carve<int64_t>(p, N > 0 ? N : 1);
  int32_t* tcol = carve<int32_t>(p, nnz > 0 ? nnz : 1);
  float* tval = carve<float>(p, nnz > 0 ? nnz : 1);
  void* temp = p;
  size_t sort_bytes = 0;
  (void)rocprim::segmented_radix_sort_pairs(
      nullptr, sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const float*)nullptr,
      (float*)nullptr, (size_t)(nnz > 0 ? nnz : 1), (unsigned)(N > 0 ? N : 1),
      (const int64_t*)nullptr, (const int64_t*)nullptr, 0, 32, s);
  const size_t tb = align_up(sort_bytes > scan64_temp(N) ? sort_bytes : scan64_temp(N), 256);
  if (N == 0) return scan_rowptr(temp, tb, count, out_rowptr, 0, s, "csr_permute");
  VQGNN_REQUIRE(rowptr && perm && (nnz == 0 || (col && out_col && out_val)),
                "csr_permute: null pointer");
  hipLaunchKernelGGL(perm_inverse_kernel, grid_rows(N), dim3(kPpThreads), 0, s, perm, N, inv,
                     reinterpret_cast<unsigned long long*>(status));
  hipLaunchKernelGGL(perm_count_kernel, grid_rows(N), dim3(kPpThreads), 0, s, rowptr, perm, N,
                     count);
  int rc = scan_rowptr(temp, tb, count, out_rowptr, N, s, "csr_permute(rowptr)");
  if (rc || nnz == 0) return rc;
  hipLaunchKernelGGL(perm_fill_kernel, grid_waves(N), dim3(kPpThreads), 0, s, rowptr, col, val,
                     perm, N, inv, out_rowptr, tcol, tval);
  rc = check_launch("csr_permute(fill)");
  if (rc) return rc;
  // index_select(0, perm).index_select(1, perm): every row sorted by its new columns
  const hipError_t e = rocprim::segmented_radix_sort_pairs(
      temp, sort_bytes, reinterpret_cast<const uint32_t*>(tcol),
      reinterpret_cast<uint32_t*>(out_col), tval, out_val, (size_t)nnz, (unsigned)N, out_rowptr,
      out_rowptr + 1, 0, bits64((unsigned long long)(N > 1 ? N - 1 : 1)), s);
  if (e != hipSuccess) {
    set_error("csr_permute: segmented sort failed: %s", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  return check_launch("csr_permute");
}

extern "C" size_t vqgnn_partition_workspace(int64_t N) {
  const size_t n1 = (size_t)(N > 0 ? N : 1);
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (const int64_t*)nullptr,
                                  (int64_t*)nullptr, n1, 0, 64, (hipStream_t)0);
  return 3 * align_up(n1 * 4, 256) + 2 * align_up(n1 * 8, 256) + 2 * align_up(n1 * 8, 256) +
         2 * align_up((size_t)kMaxParts * 4, 256) + align_up(bytes, 256) + 1024;
}

extern "C" int vqgnn_partition(const int64_t* rowptr, const int32_t* col, int64_t N,
                               int32_t num_parts, int64_t* perm, int64_t* ptr,
                               int32_t* iterations, void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(N >= 0 && N < (int64_t)INT32_MAX && num_parts >= 1 && num_parts <= kMaxParts,
                "partition: bad shape (N=%lld, parts=%d <= %d)", (long long)N, num_parts,
                kMaxParts);
  VQGNN_REQUIRE(perm && ptr && workspace && (N == 0 || (rowptr && col)), "partition: null pointer");
  hipStream_t s = as_stream(stream);
  char* p = reinterpret_cast<char*>(workspace);
  int32_t* label = carve<int32_t>(p, N > 0 ? N : 1);
  int32_t* level = carve<int32_t>(p, N > 0 ? N : 1);
  int32_t* part = carve<int32_t>(p, N > 0 ? N : 1);
  auto* keys = carve<unsigned long long>(p, N > 0 ? N : 1);
  auto* skeys = carve<unsigned long long>(p, N > 0 ? N : 1);
  int64_t* ids = carve<int64_t>(p, N > 0 ? N : 1);
  int64_t* sids = carve<int64_t>(p, N > 0 ? N : 1);
  int32_t* size = carve<int32_t>(p, kMaxParts);
  int32_t* size2 = carve<int32_t>(p, kMaxParts);
  int* flag = carve<int>(p, 2);
  void* temp = p;
  (void)hipMemsetAsync(size, 0, (size_t)num_parts * 4, s);
  if (N == 0) {
    hipLaunchKernelGGL(parts_ptr_kernel, dim3(1), dim3(1), 0, s, size, num_parts, ptr);
    return check_launch("partition(empty)");
  }
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (const int64_t*)nullptr,
                                  (int64_t*)nullptr, (size_t)N, 0, 64, s);
  auto sort = [&](const char* what) {
    const hipError_t e = rocprim::radix_sort_pairs(temp, bytes, keys, skeys, ids, sids, (size_t)N,
                                                   0, 64, s);
    if (e != hipSuccess) set_error("partition: %s sort failed: %s", what, hipGetErrorString(e));
    return e == hipSuccess ? VQGNN_OK : VQGNN_ERR_LAUNCH;
  };
  int flag_h = 0;
  int iters = 0;
  hipLaunchKernelGGL(cc_init_kernel, grid_rows(N), dim3(kPpThreads), 0, s, N, label, level);
  // connected components: min-label propagation + pointer jumping, until stable
  do {
    (void)hipMemsetAsync(flag, 0, sizeof(int), s);
    hipLaunchKernelGGL(cc_step_kernel, grid_waves(N), dim3(kPpThreads), 0, s, rowptr, col, N,
                       label, flag);
    hipLaunchKernelGGL(cc_jump_kernel, grid_rows(N), dim3(kPpThreads), 0, s, N, label);
    if (hipMemcpyAsync(&flag_h, flag, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return check_launch("partition(components)");
    ++iters;
  } while (flag_h && iters < 1 << 20);
  // multi-source BFS from every component's smallest node
  hipLaunchKernelGGL(bfs_seed_kernel, grid_rows(N), dim3(kPpThreads), 0, s, N, label, level);
  for (int d = 0;; ++d) {
    (void)hipMemsetAsync(flag, 0, sizeof(int), s);
    hipLaunchKernelGGL(bfs_step_kernel, grid_waves(N), dim3(kPpThreads), 0, s, rowptr, col, N, d,
                       level, flag);
    if (hipMemcpyAsync(&flag_h, flag, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return check_launch("partition(bfs)");
    ++iters;
    if (!flag_h) break;
  }
  // initial bands of the (component, level, id) order
  hipLaunchKernelGGL(order_keys_kernel, grid_rows(N), dim3(kPpThreads), 0, s, N, label, level,
                     keys, ids);
  int rc = sort("order");
  if (rc) return rc;
  hipLaunchKernelGGL(band_init_kernel, grid_rows(N), dim3(kPpThreads), 0, s, sids, N, num_parts,
                     part, size);
  // balanced label propagation: capacity 1.05 N / k
  const int cap = (int)((N * 105 + 100LL * num_parts - 1) / (100LL * num_parts));
  for (int t = 0; t < kLpaSteps && num_parts > 1; ++t) {
    (void)hipMemcpyAsync(size2, size, (size_t)num_parts * 4, hipMemcpyDeviceToDevice, s);
    hipLaunchKernelGGL(lpa_want_kernel, grid_waves(N), dim3(kPpThreads), 0, s, rowptr, col, N,
                       num_parts, part, keys, ids);
    if ((rc = sort("moves"))) return rc;
    hipLaunchKernelGGL(lpa_move_kernel, grid_rows(N), dim3(kPpThreads), 0, s, skeys, sids, N, cap,
                       size, part, size2);
    (void)hipMemcpyAsync(size, size2, (size_t)num_parts * 4, hipMemcpyDeviceToDevice, s);
  }
  // order: partition, BFS level, node id
  hipLaunchKernelGGL(part_keys_kernel, grid_rows(N), dim3(kPpThreads), 0, s, N, part, level, keys,
                     ids);
  if ((rc = sort("final"))) return rc;
  (void)hipMemcpyAsync(perm, sids, (size_t)N * 8, hipMemcpyDeviceToDevice, s);
  hipLaunchKernelGGL(parts_ptr_kernel, dim3(1), dim3(1), 0, s, size, num_parts, ptr);
  if (iterations) *iterations = iters;
  return check_launch("partition");
}
