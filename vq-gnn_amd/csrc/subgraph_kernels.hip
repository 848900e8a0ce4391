// Mini-batch construction on the device:
//   OurDataLoader._k_hop_subgraph  (vq_gnn_v2/dataloader.py:98-148)
//   SparseTensor(row=, col=, value=) of prepare_batch_input (vq_gnn_v2/utils/misc.py:73)
//
// _k_hop_subgraph, restated as mask / scan / compaction work (integer, HBM-
// and latency-bound; no arithmetic on the values):
//   1. seed: node_map[node_idx[i]] = i, mark = 1.  A node repeated in
//      node_idx keeps every copy in subset[:B] (the assert at :128 holds) and
//      the relabelling node_idx[subset] = arange (:144) lets the last copy
//      win: atomicMax; rows of the earlier copies stay empty.
//   2. hop h: every neighbour of a node marked h that is unmarked gets h+1
//      (the union over hops equals unique(cat(subsets)), :113-119)
//   3. B' = marked, non-batch nodes in ascending global id (CPU torch.unique
//      sorts; :121-126), node_map = B + rank, subset = [node_idx ; B']
//   4. kept entries: train -> both ends in subset (:132-133); eval -> the row
//      is a batch node (:136-138); relabelled through node_map (:142-145)
// Emission order: ORDER_CSR = rows in subset order, entries sorted by local
// column (what SparseTensor builds, misc.py:73); ORDER_REF = the reference's
// edge_index order (global row, then global column: edge_index[:, edge_mask]).
#include "common.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

namespace vqgnn {

namespace {

constexpr int kSgThreads = 256;
constexpr int kSgWaves = kSgThreads / 64;

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) {
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

__global__ void __launch_bounds__(kSgThreads)
khop_seed_kernel(const int64_t* __restrict__ node_idx, int B, int64_t N, int* __restrict__ node_map,
                 uint8_t* __restrict__ mark, int64_t* __restrict__ subset,
                 unsigned long long* __restrict__ status) {
  const int i = blockIdx.x * kSgThreads + threadIdx.x;
  if (i >= B) return;
  const int64_t v = node_idx[i];
  if (v < 0 || v >= N) {
    atomicOr(status, (unsigned long long)VQGNN_KHOP_OUT_OF_RANGE);
    return;
  }
  atomicMax(node_map + v, i);            // node_map starts at -1
  mark[v] = 1;
  subset[i] = v;
}

// one wave per frontier node: nodes of the list (hop 1) or nodes with
// mark == level (later hops); unmarked neighbours get level + 1
__global__ void __launch_bounds__(kSgThreads)
khop_expand_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                   const int64_t* __restrict__ list, int64_t count, int64_t nnodes,
                   uint8_t* __restrict__ mark, int level) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * kSgWaves + (threadIdx.x >> 6);
  if (w >= count) return;
  int64_t v;
  if (list) {
    v = list[w];
    if (v < 0 || v >= nnodes) return;     // flagged by the seed kernel
  } else {
    v = w;
    if (mark[v] != level) return;
  }
  const int64_t e0 = rowptr[v], e1 = rowptr[v + 1];
  for (int64_t e = e0 + lane; e < e1; e += 64) {
    const int u = col[e];
    if (mark[u] == 0) mark[u] = (uint8_t)(level + 1);
  }
}

// flag[v] = 1 for the nodes a compaction keeps (in ascending v)
//   what == 0: B' nodes (marked, not a batch node)
//   what == 1: every node of subset (reference row order, train)
//   what == 2: batch nodes only (reference row order, eval)
__global__ void __launch_bounds__(kSgThreads)
khop_flag_kernel(const uint8_t* __restrict__ mark, const int* __restrict__ node_map, int64_t N,
                 int B, int what, int* __restrict__ flag) {
  const int64_t v = (int64_t)blockIdx.x * kSgThreads + threadIdx.x;
  if (v >= N) return;
  const int m = node_map[v];
  int f;
  if (what == 0) f = mark[v] != 0 && m < 0;
  else if (what == 1) f = mark[v] != 0;
  else f = m >= 0 && m < B;
  flag[v] = f;
}

// pos = inclusive scan of flag (pos[v] = kept nodes <= v)
__global__ void __launch_bounds__(kSgThreads)
khop_compact_kernel(const int* __restrict__ flag, const int* __restrict__ pos, int64_t N, int base,
                    int* __restrict__ node_map, int64_t* __restrict__ out) {
  const int64_t v = (int64_t)blockIdx.x * kSgThreads + threadIdx.x;
  if (v >= N || !flag[v]) return;
  const int p = base + pos[v] - 1;
  if (node_map) node_map[v] = p;
  out[p] = v;
}

__global__ void khop_sizes_kernel(const int* __restrict__ pos, int64_t N, int B, int what,
                                  long long* __restrict__ sizes) {
  const long long tot = N > 0 ? pos[N - 1] : 0;
  if (what == 0) sizes[0] = B + tot;      // n
  else sizes[2] = tot;                    // rows emitted (reference order)
}

// keep rule of entry (row g, neighbour u): train -> u in subset; eval -> the
// row is a batch node (then every neighbour is in subset: 1 <= num_hops)
__device__ __forceinline__ bool khop_keep(int train, int lr, int B, int mu) {
  return train ? mu >= 0 : (lr >= 0 && lr < B);
}

// count[r] = kept entries of emitted row r (one wave per row; rows past the
// device row count write 0, so the scan may run over the capacity)
__global__ void __launch_bounds__(kSgThreads)
khop_count_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                  const int64_t* __restrict__ rows, const long long* __restrict__ sizes,
                  int nrows_slot, int64_t cap, int64_t nnodes, const int* __restrict__ node_map,
                  int train, int B, int csr, int* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kSgWaves + (threadIdx.x >> 6);
  if (r >= cap) return;
  int c = 0;
  const int64_t g = r < sizes[nrows_slot] ? rows[r] : -1;
  // invalid ids are flagged by the seed kernel; in CSR order a row emits only
  // as its node's local id (earlier copies of a repeated batch node: empty)
  const int lr = (g >= 0 && g < nnodes) ? node_map[g] : -1;
  if (lr >= 0 && (!csr || lr == r)) {
    const int64_t e0 = rowptr[g], e1 = rowptr[g + 1];
    for (int64_t e = e0 + lane; e < e1; e += 64)
      c += khop_keep(train, lr, B, node_map[col[e]]) ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  }
  if (lane == 0) count[r] = c;
}

// out_ptr[0] = 0; out_ptr[r + 1] = inclusive scan; sizes[1] = nnz
__global__ void khop_nnz_kernel(int* __restrict__ out_ptr, const long long* __restrict__ sizes,
                                int nrows_slot, long long* __restrict__ sizes_out) {
  out_ptr[0] = 0;
  sizes_out[1] = out_ptr[sizes[nrows_slot]];
}

// one wave per emitted row: kept entries in neighbour order, relabelled
__global__ void __launch_bounds__(kSgThreads)
khop_fill_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                 const float* __restrict__ val, const int64_t* __restrict__ rows, int64_t nrows,
                 int64_t nnodes, const int* __restrict__ node_map, int train, int B, int csr,
                 const int* __restrict__ lptr,
                 int* __restrict__ out_col, float* __restrict__ out_val, int* __restrict__ out_row) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kSgWaves + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const int64_t g = rows[r];
  if (g < 0 || g >= nnodes) return;
  const int lr = node_map[g];
  if (csr && lr != r) return;
  const int64_t e0 = rowptr[g], e1 = rowptr[g + 1];
  int base = lptr[r];
  const unsigned long long below = lanemask_lt(lane);
  for (int64_t eb = e0; eb < e1; eb += 64) {
    const int64_t e = eb + lane;
    int mu = -1;
    bool k = false;
    if (e < e1) {
      mu = node_map[col[e]];
      k = khop_keep(train, lr, B, mu);
    }
    const unsigned long long m = __ballot(k);
    if (k) {
      const int p = base + __popcll(m & below);
      out_col[p] = mu;
      out_val[p] = val[e];
      if (out_row) out_row[p] = lr;
    }
    base += __popcll(m);
  }
}

__global__ void __launch_bounds__(kSgThreads)
coo_keys_kernel(const int64_t* __restrict__ row, const int64_t* __restrict__ col, int64_t nnz,
                int64_t n_rows, int64_t n_cols, unsigned long long* __restrict__ keys,
                int* __restrict__ iota, unsigned long long* __restrict__ status) {
  const int64_t i = (int64_t)blockIdx.x * kSgThreads + threadIdx.x;
  if (i >= nnz) return;
  const int64_t r = row[i], c = col[i];
  if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) {
    atomicOr(status, (unsigned long long)VQGNN_KHOP_OUT_OF_RANGE);
    keys[i] = 0;
  } else {
    keys[i] = (unsigned long long)r * (unsigned long long)n_cols + (unsigned long long)c;
  }
  iota[i] = (int)i;
}

// sorted keys -> col, permuted values, rowptr (rowptr[r] = first entry of a
// row >= r: every entry marks the boundaries between its row and the next)
__global__ void __launch_bounds__(kSgThreads)
coo_finish_kernel(const unsigned long long* __restrict__ keys, const int* __restrict__ perm,
                  const float* __restrict__ val, int64_t nnz, int64_t n_rows, int64_t n_cols,
                  int* __restrict__ out_ptr, int* __restrict__ out_col, float* __restrict__ out_val) {
  const int64_t i = (int64_t)blockIdx.x * kSgThreads + threadIdx.x;
  if (i < nnz) {
    const unsigned long long k = keys[i];
    const int64_t r = (int64_t)(k / (unsigned long long)n_cols);
    out_col[i] = (int)(k % (unsigned long long)n_cols);
    out_val[i] = val ? val[perm[i]] : 1.0f;
    const int64_t rp = i > 0 ? (int64_t)(keys[i - 1] / (unsigned long long)n_cols) : -1;
    for (int64_t q = rp + 1; q <= r; ++q) out_ptr[q] = (int)i;
    if (i == nnz - 1)
      for (int64_t q = r + 1; q <= n_rows; ++q) out_ptr[q] = (int)nnz;
  }
}

template <typename T>
T* carve(char*& p, size_t count) {
  T* r = reinterpret_cast<T*>(p);
  p += align_up(count * sizeof(T), 256);
  return r;
}

size_t scan_temp_bytes(int64_t n) {
  size_t bytes = 0;
  (void)rocprim::inclusive_scan(nullptr, bytes, (const int*)nullptr, (int*)nullptr, (size_t)n,
                                rocprim::plus<int>(), (hipStream_t)0);
  return bytes;
}

int inclusive_scan(void* temp, size_t temp_bytes, const int* in, int* out, int64_t n,
                   hipStream_t s, const char* what) {
  if (n <= 0) return VQGNN_OK;
  const hipError_t e =
      rocprim::inclusive_scan(temp, temp_bytes, in, out, (size_t)n, rocprim::plus<int>(), s);
  if (e != hipSuccess) {
    set_error("%s: scan failed: %s", what, hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  return check_launch(what);
}

int bits_for(int64_t n) {
  int b = 1;
  while (b < 63 && ((int64_t)1 << b) < n) ++b;
  return b;
}

// Uniform random walks (torch_cluster random_walk with p = q = 1, which
// SparseTensor.random_walk calls for the 'edge' / 'rw' / 'cont' samplers,
// dataloader.py:70-90): one thread per walk; step l draws u in [0, 1) and
// moves to col[rowptr[v] + (int64)(u * (float)deg)], or stays on v when it
// has no neighbour.  u is the top 24 bits of splitmix64(seed, walk, step)
// scaled by 2^-24 (a float in [0, 1), like torch.rand).
__device__ __forceinline__ unsigned long long walk_mix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(kSgThreads)
random_walk_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col, int64_t N,
                   const int64_t* __restrict__ start, int64_t n_start, int walk_length,
                   unsigned long long seed, long long* __restrict__ out,
                   long long* __restrict__ status) {
  const int64_t i = blockIdx.x * (int64_t)kSgThreads + threadIdx.x;
  if (i >= n_start) return;
  int64_t v = start[i];
  long long* o = out + i * (walk_length + 1);
  o[0] = v;
  if (v < 0 || v >= N) {
    *status = VQGNN_KHOP_OUT_OF_RANGE;
    for (int l = 1; l <= walk_length; ++l) o[l] = v;
    return;
  }
  const unsigned long long base = walk_mix(seed ^ walk_mix((unsigned long long)i));
  for (int l = 0; l < walk_length; ++l) {
    const int64_t rs = rowptr[v], re = rowptr[v + 1];
    if (re > rs) {
      const unsigned long long h = walk_mix(base + (unsigned long long)l);
      const float u = (float)(h >> 40) * 5.9604644775390625e-08f;   // 2^-24
      const int64_t e = rs + (int64_t)(u * (float)(re - rs));
      v = col[e < re ? e : re - 1];
    }
    o[l + 1] = v;
  }
}

}  // namespace

}  // namespace vqgnn

using namespace vqgnn;

extern "C" size_t vqgnn_khop_workspace(int64_t N) {
  if (N <= 0) return 256;
  return align_up((size_t)N, 256) + 2 * align_up((size_t)N * 4, 256) +
         align_up((size_t)N * 4, 256) + align_up(scan_temp_bytes(N), 256) + 256;
}

extern "C" int vqgnn_khop_subset(const int64_t* rowptr, const int32_t* col, int64_t N,
                                 const int64_t* node_idx, int32_t B, int32_t num_hops,
                                 int32_t train_flag, int32_t order, int32_t* node_map,
                                 int64_t* subset, int64_t* rows, int32_t* out_rowptr,
                                 int64_t* sizes, void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(N >= 0 && N < (int64_t)INT32_MAX && B >= 0 && B <= N && num_hops >= 1 &&
                    num_hops < 250,
                "khop_subset: bad shape (N=%lld B=%d hops=%d)", (long long)N, B, num_hops);
  VQGNN_REQUIRE(order == VQGNN_KHOP_ORDER_CSR || order == VQGNN_KHOP_ORDER_REF,
                "khop_subset: bad order %d", order);
  VQGNN_REQUIRE(sizes && workspace && (N == 0 || (rowptr && node_map && subset && out_rowptr)),
                "khop_subset: null pointer");
  VQGNN_REQUIRE(order == VQGNN_KHOP_ORDER_CSR || rows, "khop_subset: rows needed for ORDER_REF");
  VQGNN_REQUIRE(B == 0 || node_idx, "khop_subset: null node_idx");
  hipStream_t s = as_stream(stream);
  (void)hipMemsetAsync(sizes, 0, 4 * sizeof(int64_t), s);
  if (N == 0) return check_launch("khop_subset(empty)");
  char* p = reinterpret_cast<char*>(workspace);
  uint8_t* mark = carve<uint8_t>(p, N);
  int* flag = carve<int>(p, N);
  int* pos = carve<int>(p, N);
  int* count = carve<int>(p, N);
  const size_t tb = align_up(scan_temp_bytes(N), 256);
  void* temp = carve<char>(p, tb);
  unsigned long long* status = reinterpret_cast<unsigned long long*>(sizes + 3);
  long long* sz = reinterpret_cast<long long*>(sizes);

  (void)hipMemsetAsync(node_map, 0xFF, (size_t)N * sizeof(int32_t), s);
  (void)hipMemsetAsync(mark, 0, (size_t)N, s);
  const dim3 gN((unsigned)((N + kSgThreads - 1) / kSgThreads));
  if (B > 0) {
    const dim3 gB((B + kSgThreads - 1) / kSgThreads);
    hipLaunchKernelGGL(khop_seed_kernel, gB, dim3(kSgThreads), 0, s, node_idx, B, N, node_map,
                       mark, subset, status);
    // hop 1 from the seed list; later hops from mark == level
    hipLaunchKernelGGL(khop_expand_kernel, dim3((B + kSgWaves - 1) / kSgWaves), dim3(kSgThreads),
                       0, s, rowptr, col, node_idx, (int64_t)B, N, mark, 1);
    for (int h = 2; h <= num_hops; ++h)
      hipLaunchKernelGGL(khop_expand_kernel, dim3((unsigned)((N + kSgWaves - 1) / kSgWaves)),
                         dim3(kSgThreads), 0, s, rowptr, col, (const int64_t*)nullptr, N, N, mark, h);
  }
  int rc = check_launch("khop_subset(expand)");
  if (rc) return rc;
  // B' in ascending global id
  hipLaunchKernelGGL(khop_flag_kernel, gN, dim3(kSgThreads), 0, s, mark, node_map, N, B, 0, flag);
  if ((rc = inclusive_scan(temp, tb, flag, pos, N, s, "khop_subset(scan B')"))) return rc;
  hipLaunchKernelGGL(khop_compact_kernel, gN, dim3(kSgThreads), 0, s, flag, pos, N, B, node_map,
                     subset);
  hipLaunchKernelGGL(khop_sizes_kernel, dim3(1), dim3(1), 0, s, pos, N, B, 0, sz);
  const int64_t* emit = subset;
  int slot = 0;
  if (order == VQGNN_KHOP_ORDER_REF) {
    hipLaunchKernelGGL(khop_flag_kernel, gN, dim3(kSgThreads), 0, s, mark, node_map, N, B,
                       train_flag ? 1 : 2, flag);
    if ((rc = inclusive_scan(temp, tb, flag, pos, N, s, "khop_subset(scan rows)"))) return rc;
    hipLaunchKernelGGL(khop_compact_kernel, gN, dim3(kSgThreads), 0, s, flag, pos, N, 0,
                       (int*)nullptr, rows);
    hipLaunchKernelGGL(khop_sizes_kernel, dim3(1), dim3(1), 0, s, pos, N, B, 1, sz);
    emit = rows;
    slot = 2;
  }
  // per-row counts over the capacity N, then the row pointers
  hipLaunchKernelGGL(khop_count_kernel, dim3((unsigned)((N + kSgWaves - 1) / kSgWaves)),
                     dim3(kSgThreads), 0, s, rowptr, col, emit, sz, slot, N, N, node_map,
                     train_flag ? 1 : 0, B, order == VQGNN_KHOP_ORDER_CSR ? 1 : 0, count);
  if ((rc = inclusive_scan(temp, tb, count, out_rowptr + 1, N, s, "khop_subset(scan rowptr)")))
    return rc;
  hipLaunchKernelGGL(khop_nnz_kernel, dim3(1), dim3(1), 0, s, out_rowptr, sz, slot, sz);
  if (order == VQGNN_KHOP_ORDER_CSR)   // rows emitted = n (all of subset)
    (void)hipMemcpyAsync(sizes + 2, sizes, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
  return check_launch("khop_subset");
}

extern "C" size_t vqgnn_khop_edges_workspace(int64_t nrows, int64_t nnz) {
  if (nnz <= 0) return 256;
  size_t bytes = 0;
  (void)rocprim::segmented_radix_sort_pairs(
      nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const float*)nullptr,
      (float*)nullptr, (size_t)nnz, (unsigned)(nrows > 0 ? nrows : 1), (const int*)nullptr,
      (const int*)nullptr, 0, 32, (hipStream_t)0);
  return 2 * align_up((size_t)nnz * 4, 256) + align_up(bytes, 256) + 256;
}

extern "C" int vqgnn_khop_edges(const int64_t* rowptr, const int32_t* col, const float* val,
                                int64_t N, const int32_t* node_map, const int64_t* rows,
                                int64_t nrows, int64_t n, int32_t B, int32_t train_flag,
                                int32_t order, const int32_t* out_rowptr, int64_t nnz,
                                int32_t* out_col, float* out_val, int32_t* out_row,
                                void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(N >= 0 && nrows >= 0 && nrows <= N && n >= 0 && n <= N && nnz >= 0 &&
                    nnz < (int64_t)INT32_MAX && B >= 0,
                "khop_edges: bad shape");
  VQGNN_REQUIRE(order == VQGNN_KHOP_ORDER_CSR || order == VQGNN_KHOP_ORDER_REF,
                "khop_edges: bad order %d", order);
  if (nrows == 0 || nnz == 0) return VQGNN_OK;
  VQGNN_REQUIRE(rowptr && col && val && node_map && rows && out_rowptr && out_col && out_val &&
                    workspace,
                "khop_edges: null pointer");
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)((nrows + kSgWaves - 1) / kSgWaves));
  if (order == VQGNN_KHOP_ORDER_REF) {
    hipLaunchKernelGGL(khop_fill_kernel, grid, dim3(kSgThreads), 0, s, rowptr, col, val, rows,
                       nrows, N, node_map, train_flag ? 1 : 0, B, 0, out_rowptr, out_col, out_val,
                       out_row);
    return check_launch("khop_edges(ref)");
  }
  // CSR: fill in neighbour order, then sort every row by local column
  // (columns of a row are distinct; stable anyway)
  char* p = reinterpret_cast<char*>(workspace);
  int* tcol = carve<int>(p, nnz);
  float* tval = carve<float>(p, nnz);
  size_t bytes = 0;
  (void)rocprim::segmented_radix_sort_pairs(
      nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const float*)nullptr,
      (float*)nullptr, (size_t)nnz, (unsigned)nrows, (const int*)nullptr, (const int*)nullptr, 0,
      32, s);
  void* temp = p;
  hipLaunchKernelGGL(khop_fill_kernel, grid, dim3(kSgThreads), 0, s, rowptr, col, val, rows,
                     nrows, N, node_map, train_flag ? 1 : 0, B, 1, out_rowptr, tcol, tval, out_row);
  int rc = check_launch("khop_edges(fill)");
  if (rc) return rc;
  const hipError_t e = rocprim::segmented_radix_sort_pairs(
      temp, bytes, reinterpret_cast<const uint32_t*>(tcol), reinterpret_cast<uint32_t*>(out_col),
      tval, out_val, (size_t)nnz, (unsigned)nrows, out_rowptr, out_rowptr + 1, 0,
      bits_for(n > 1 ? n : 2), s);
  if (e != hipSuccess) {
    set_error("khop_edges: segmented sort failed: %s", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  return check_launch("khop_edges(sort)");
}

extern "C" size_t vqgnn_coo_to_csr_workspace(int64_t nnz, int64_t n_rows, int64_t n_cols) {
  if (nnz <= 0) return 256;
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (const int*)nullptr, (int*)nullptr,
                                  (size_t)nnz, 0, 64, (hipStream_t)0);
  (void)n_rows;
  (void)n_cols;
  return 2 * align_up((size_t)nnz * 8, 256) + 2 * align_up((size_t)nnz * 4, 256) +
         align_up(bytes, 256) + 256;
}

extern "C" int vqgnn_coo_to_csr(const int64_t* row, const int64_t* col, const float* val,
                                int64_t nnz, int64_t n_rows, int64_t n_cols, int32_t* out_rowptr,
                                int32_t* out_col, float* out_val, int64_t* status,
                                void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(nnz >= 0 && nnz < (int64_t)INT32_MAX && n_rows >= 0 && n_cols >= 0 &&
                    n_rows < (int64_t)INT32_MAX && n_cols < (int64_t)INT32_MAX,
                "coo_to_csr: bad shape");
  VQGNN_REQUIRE(out_rowptr && status, "coo_to_csr: null pointer");
  hipStream_t s = as_stream(stream);
  (void)hipMemsetAsync(status, 0, sizeof(int64_t), s);
  if (nnz == 0) {
    (void)hipMemsetAsync(out_rowptr, 0, (size_t)(n_rows + 1) * 4, s);
    return check_launch("coo_to_csr(empty)");
  }
  VQGNN_REQUIRE(row && col && out_col && out_val && workspace, "coo_to_csr: null pointer");
  VQGNN_REQUIRE(n_rows > 0 && n_cols > 0, "coo_to_csr: entries in an empty matrix");
  char* p = reinterpret_cast<char*>(workspace);
  auto* keys = carve<unsigned long long>(p, nnz);
  auto* keys_out = carve<unsigned long long>(p, nnz);
  int* iota = carve<int>(p, nnz);
  int* perm = carve<int>(p, nnz);
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (const int*)nullptr, (int*)nullptr,
                                  (size_t)nnz, 0, 64, s);
  void* temp = p;
  const dim3 grid((unsigned)((nnz + kSgThreads - 1) / kSgThreads));
  hipLaunchKernelGGL(coo_keys_kernel, grid, dim3(kSgThreads), 0, s, row, col, nnz, n_rows, n_cols,
                     keys, iota, reinterpret_cast<unsigned long long*>(status));
  int rc = check_launch("coo_to_csr(keys)");
  if (rc) return rc;
  // stable: entries with equal (row, col) keep their input order
  const int bits = bits_for(n_rows * n_cols);
  const hipError_t e =
      rocprim::radix_sort_pairs(temp, bytes, keys, keys_out, iota, perm, (size_t)nnz, 0, bits, s);
  if (e != hipSuccess) {
    set_error("coo_to_csr: radix sort failed: %s", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  hipLaunchKernelGGL(coo_finish_kernel, grid, dim3(kSgThreads), 0, s, keys_out, perm, val, nnz,
                     n_rows, n_cols, out_rowptr, out_col, out_val);
  return check_launch("coo_to_csr");
}

extern "C" int vqgnn_random_walk(const int64_t* rowptr, const int32_t* col, int64_t N,
                                 const int64_t* start, int64_t n_start, int32_t walk_length,
                                 uint64_t seed, int64_t* out, int64_t* status,
                                 vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(rowptr && status && N >= 0 && n_start >= 0 && walk_length >= 0,
                "random_walk: bad arguments");
  VQGNN_REQUIRE(n_start == 0 || (start && out && col), "random_walk: null pointer");
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(status, 0, sizeof(int64_t), s) != hipSuccess)
    return check_launch("random_walk memset");
  if (n_start > 0)
    hipLaunchKernelGGL(random_walk_kernel, dim3((unsigned)((n_start + kSgThreads - 1) / kSgThreads)),
                       dim3(kSgThreads), 0, s, rowptr, col, N, start, n_start, walk_length,
                       (unsigned long long)seed, reinterpret_cast<long long*>(out),
                       reinterpret_cast<long long*>(status));
  return check_launch("random_walk");
}
