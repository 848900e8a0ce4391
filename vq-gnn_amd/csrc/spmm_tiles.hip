// Tiled CSR SpMM for gfx950 (MI355X) on batches whose adjacency has dense
// (row window x column tile) blocks — the reddit-shaped batches, where ~80 %
// of a row's ~490 edges fall inside its own METIS-like cluster, i.e. inside a
// few thousand consecutive columns next to the row.  Same product as
// spmm_tasks.hip (out = A * [X ; X2], LowRankGNNLayer's aggregation,
// vq_gnn_v2/models.py:174 + convs.py:95), split in two:
//
//  * dense part: blocks of kTR rows x kTC columns holding >= min_edges edges.
//    A workgroup owns one row window and one 64-float column slice; for each
//    dense block of its window it stages the block's kTC source rows (slice
//    only, 32 KB), its row pointers and records in LDS once (the next block's
//    are loaded into registers under this block's work), and reads every
//    edge's source row from LDS (each staged row is reused ~20x on reddit),
//    accumulating its 256 rows in registers (16 lanes x float4 per row).
//    Records are padded per (row, block) to 4 edges: a group reads 4 records
//    with two 16-byte LDS broadcasts; records past the 5,120 an LDS buffer
//    holds are read from global memory.
//  * sparse remainder (edges of the other blocks): its own CSR, aggregated by
//    the task kernel in accumulate mode (vqgnn_spmm_task_acc) after the tile
//    kernel has written every row.
//
// Per row the sum is: dense blocks in column-tile order (each a sequential fma
// chain in column order), then the sparse edges' chain added once.
// Deterministic and independent of the launch geometry; within 1e-5 relative
// of the fp64 sum (north_star tolerance), like the task kernel.
//
// Plan (once per batch adjacency, any F; include/vqgnn.h §6f): phase A counts
// the edges of every block and numbers the dense ones; the caller reads the
// counts back and sizes phase B's arrays (block list and window starts,
// per-block row pointers, padded dense records, the sparse CSR).

#include "common.h"

#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <mutex>

namespace vqgnn {

constexpr int kTR = 256;        // rows per window
constexpr int kTC = 128;        // columns per tile
constexpr int kTL = 16;         // lanes per row: 16 x float4 = a 64-float slice
constexpr int kTThreads = 256;  // 16 rows in flight per workgroup
constexpr int kTPad = 4;        // records per (row, block) padded to a multiple of 4

__device__ __forceinline__ int lower_bound_col(const int32_t* __restrict__ col, int lo, int hi,
                                               int key) {
  // first e in [lo, hi) with col[e] >= key (col sorted within a row)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (col[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// ---- plan, phase A ---------------------------------------------------------
// One wave per row: every (row, tile) segment adds its length to its block.
__global__ void __launch_bounds__(256)
tile_count_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                  int n_rows, int T, int32_t* __restrict__ cnt) {
  const int r = (int)((blockIdx.x * 256u + threadIdx.x) >> 6), lane = threadIdx.x & 63;
  if (r >= n_rows) return;
  const int rs = rowptr[r], re = rowptr[r + 1];
  const int64_t wrow = (int64_t)(r / kTR) * T;
  for (int e = rs + lane; e < re; e += 64) {
    const int t = col[e] / kTC;
    if (e == rs || col[e - 1] / kTC != t) {
      const int end = lower_bound_col(col, e, re, (t + 1) * kTC);
      atomicAdd(cnt + wrow + t, end - e);
    }
  }
}

__global__ void tile_flags_kernel(const int32_t* __restrict__ cnt, int64_t nblk, int min_edges,
                                  int32_t* __restrict__ flag, int32_t* __restrict__ dense_edges) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i > nblk) return;
  const bool d = i < nblk && cnt[i] >= min_edges;
  flag[i] = d ? 1 : 0;
  if (d) atomicAdd(dense_edges, cnt[i]);
}

// phase B recovers the dense flags from the block ids: dense iff bid[i+1] > bid[i]
__global__ void tile_flags_from_bid_kernel(const int32_t* __restrict__ bid, int64_t nblk,
                                           int32_t* __restrict__ flag) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < nblk) flag[i] = bid[i + 1] > bid[i] ? 1 : 0;
}

// ---- plan, phase B ---------------------------------------------------------
// Dense block keys (w * T + t) in id order, and each window's first block id.
__global__ void tile_blocks_kernel(const int32_t* __restrict__ flag, const int32_t* __restrict__ bid,
                                   int64_t nblk, int W, int T, int n_dense,
                                   int32_t* __restrict__ blocks) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i < nblk && flag[i]) blocks[bid[i]] = (int32_t)i;
  if (i <= W) blocks[n_dense + i] = bid[i * (int64_t)T];
}

// One wave per row: the padded length of every dense (row, block) segment and
// the row's count of sparse edges.
__global__ void __launch_bounds__(256)
tile_segments_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                     int n_rows, int T, const int32_t* __restrict__ flag,
                     const int32_t* __restrict__ bid, int32_t* __restrict__ segcnt,
                     int32_t* __restrict__ scnt) {
  const int r = (int)((blockIdx.x * 256u + threadIdx.x) >> 6), lane = threadIdx.x & 63;
  if (r >= n_rows) return;
  const int rs = rowptr[r], re = rowptr[r + 1];
  const int64_t wrow = (int64_t)(r / kTR) * T;
  int sparse = 0;
  for (int e = rs + lane; e < re; e += 64) {
    const int t = col[e] / kTC;
    if (!flag[wrow + t]) {
      ++sparse;
    } else if (e == rs || col[e - 1] / kTC != t) {
      const int len = lower_bound_col(col, e, re, (t + 1) * kTC) - e;
      segcnt[(int64_t)bid[wrow + t] * kTR + (r % kTR)] = (len + kTPad - 1) / kTPad * kTPad;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sparse += __shfl_xor(sparse, o);
  if (lane == 0) scnt[r] = sparse;
}

// One workgroup per dense block: exclusive scan of its kTR padded segment
// lengths -> rowptr_b[id][0..kTR], and the block's total in btot[id].
__global__ void __launch_bounds__(kTR)
tile_rowptr_kernel(const int32_t* __restrict__ segcnt, int32_t* __restrict__ rowptr_b,
                   int32_t* __restrict__ btot) {
  __shared__ int32_t s[kTR];
  const int id = blockIdx.x, i = threadIdx.x;
  const int v = segcnt[(int64_t)id * kTR + i];
  s[i] = v;
  __syncthreads();
  for (int o = 1; o < kTR; o <<= 1) {       // Hillis-Steele inclusive scan
    const int x = i >= o ? s[i - o] : 0;
    __syncthreads();
    s[i] += x;
    __syncthreads();
  }
  int32_t* rp = rowptr_b + (int64_t)id * (kTR + 1);
  rp[i] = s[i] - v;
  if (i == kTR - 1) {
    rp[kTR] = s[i];
    btot[id] = s[i];
  }
}

// One wave per row: dense edges to their padded slots in the block records
// (local column, weight; padding = the zero row kTC with weight 0), sparse
// edges to the remainder CSR in row order.
__global__ void __launch_bounds__(256)
tile_scatter_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                    const float* __restrict__ val, int n_rows, int T,
                    const int32_t* __restrict__ flag, const int32_t* __restrict__ bid,
                    const int32_t* __restrict__ rowptr_b, const int32_t* __restrict__ boff,
                    int2* __restrict__ drec, const int32_t* __restrict__ s_rowptr,
                    int32_t* __restrict__ s_col, float* __restrict__ s_val) {
  const int r = (int)((blockIdx.x * 256u + threadIdx.x) >> 6), lane = threadIdx.x & 63;
  if (r >= n_rows) return;
  const int rs = rowptr[r], re = rowptr[r + 1];
  const int64_t wrow = (int64_t)(r / kTR) * T;
  const int ri = r % kTR;
  int sp = s_rowptr[r];
  for (int eb = rs; eb < re; eb += 64) {
    const int e = eb + lane;
    const bool in = e < re;
    const int c = in ? col[e] : 0;
    const int t = c / kTC;
    const bool dense = in && flag[wrow + t];
    if (dense) {
      const int id = bid[wrow + t];
      const int s0 = lower_bound_col(col, rs, re, t * kTC);
      const int base = boff[id] + rowptr_b[(int64_t)id * (kTR + 1) + ri];
      const float w = val ? val[e] : 1.f;
      drec[base + (e - s0)] = make_int2(c - t * kTC, __float_as_int(w));
      // the segment's last edge pads its slots up to the multiple of kTPad
      if (e + 1 == re || col[e + 1] / kTC != t) {
        const int len = e + 1 - s0;
        const int padded = (len + kTPad - 1) / kTPad * kTPad;
        for (int k = len; k < padded; ++k) drec[base + k] = make_int2(kTC, 0);
      }
    }
    const uint64_t m = __ballot(in && !dense);
    if (in && !dense) {
      const int pos = sp + __popcll(m & ((1ull << lane) - 1));
      s_col[pos] = c;
      s_val[pos] = val ? val[e] : 1.f;
    }
    sp += __popcll(m);
  }
}

// ---- the tile kernel -------------------------------------------------------
struct TileArgs {
  const int32_t* blocks;     // [n_dense] keys, then [W + 1] window starts
  const int32_t* rowptr_b;   // [n_dense][kTR + 1]
  const int32_t* boff;       // [n_dense + 1] first record of each block
  const int4* drec;          // padded records, 2 per int4
  int n_dense, W, T;
  int n_rows, n_cols, B;
  const float* X;
  int64_t ldx;
  const float* X2;
  int64_t ldx2;
  int F;
  float* out;
  int64_t ldo;
  int dbg;                   // experiments (results invalid): 1 = no row work, 2 = no staging
};

// LDS of one workgroup: the block's kTC staged source rows + one zero row
// (the padding records' column), its records (the first kTRecCap of them) and
// its row pointers.  The next block's source rows, records and row pointers
// are loaded into registers while the current block computes (one global
// round trip per block, hidden behind the previous block's work).
constexpr int kTRecCap = 5120;                    // records of a block held in LDS
constexpr int kTRecRegs = kTRecCap / 2 / kTThreads;   // int4 (2 records) per thread: 8
constexpr int kTXRegs = kTC / (kTThreads / kTL);      // float4 of the tile per thread: 8
constexpr size_t kTileXs = (size_t)(kTC + 1) * kTL * sizeof(float4);
constexpr size_t kTileLds = kTileXs + (size_t)kTRecCap * 8 + (size_t)(kTR + 4) * 4;

// One group (16 lanes = one row's 64-float slice) accumulates one row's
// records [p, p + len) (len a multiple of 4) into A: per step two 16-byte
// record reads (the same address for the 16 lanes: a broadcast), four
// 16-byte source-row reads from the staged tile, 16 fma.
__device__ __forceinline__ void tile_fma(float4& A, const int4& c0r, const int4& c1r,
                                         const float4& v0, const float4& v1, const float4& v2,
                                         const float4& v3) {
  const float w0 = __int_as_float(c0r.y), w1 = __int_as_float(c0r.w);
  const float w2 = __int_as_float(c1r.y), w3 = __int_as_float(c1r.w);
  A.x = fmaf(w0, v0.x, A.x); A.y = fmaf(w0, v0.y, A.y);
  A.z = fmaf(w0, v0.z, A.z); A.w = fmaf(w0, v0.w, A.w);
  A.x = fmaf(w1, v1.x, A.x); A.y = fmaf(w1, v1.y, A.y);
  A.z = fmaf(w1, v1.z, A.z); A.w = fmaf(w1, v1.w, A.w);
  A.x = fmaf(w2, v2.x, A.x); A.y = fmaf(w2, v2.y, A.y);
  A.z = fmaf(w2, v2.z, A.z); A.w = fmaf(w2, v2.w, A.w);
  A.x = fmaf(w3, v3.x, A.x); A.y = fmaf(w3, v3.y, A.y);
  A.z = fmaf(w3, v3.z, A.z); A.w = fmaf(w3, v3.w, A.w);
}

// One group (16 lanes = one row's 64-float slice) accumulates one row's
// records [p, p + len) (len a multiple of 4) into A.  Per 4-record step: two
// 16-byte record reads (the same address for the 16 lanes: a broadcast),
// four 16-byte source-row reads from the staged tile, 16 fma; software-
// pipelined so the next step's record and source-row reads are in flight
// under this step's fma (one LDS round trip per step is exposed, not two).
__device__ __forceinline__ void tile_row(float4& A, const int4* __restrict__ rq, int len,
                                         const float4* __restrict__ xs, int l16) {
  if (len <= 0) return;
  int4 c0r = rq[0], c1r = rq[1];
  float4 v0 = xs[c0r.x * kTL + l16], v1 = xs[c0r.z * kTL + l16];
  float4 v2 = xs[c1r.x * kTL + l16], v3 = xs[c1r.z * kTL + l16];
  for (int k = 4; k < len; k += 4) {
    const int4 n0 = rq[k >> 1], n1 = rq[(k >> 1) + 1];
    const float4 u0 = xs[n0.x * kTL + l16], u1 = xs[n0.z * kTL + l16];
    const float4 u2 = xs[n1.x * kTL + l16], u3 = xs[n1.z * kTL + l16];
    tile_fma(A, c0r, c1r, v0, v1, v2, v3);
    c0r = n0;
    c1r = n1;
    v0 = u0;
    v1 = u1;
    v2 = u2;
    v3 = u3;
  }
  tile_fma(A, c0r, c1r, v0, v1, v2, v3);
}

__global__ void __launch_bounds__(kTThreads, 2)
spmm_tile_kernel(TileArgs a) {
  extern __shared__ float4 xs[];
  int4* recs = reinterpret_cast<int4*>(reinterpret_cast<char*>(xs) + kTileXs);
  int32_t* rps = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(xs) + kTileXs +
                                            (size_t)kTRecCap * 8);
  const int w = blockIdx.x, s = blockIdx.y;
  const int tid = threadIdx.x, grp = tid >> 4, l16 = tid & 15;
  const int F4 = a.F >> 2;
  const int piece = s * kTL + l16;
  const bool pv = piece < F4;
  constexpr int kGroups = kTThreads / kTL;        // 16 rows in flight
  constexpr int kRows = kTR / kGroups;            // rows per group: 16
  float4 acc[kRows];
#pragma unroll
  for (int i = 0; i < kRows; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (tid < kTL) xs[kTC * kTL + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int b0 = ((const __attribute__((address_space(4))) int32_t*)a.blocks)[a.n_dense + w];
  const int b1 = ((const __attribute__((address_space(4))) int32_t*)a.blocks)[a.n_dense + w + 1];
  // kernel arguments as values (a lambda capturing the struct by reference
  // would read them through memory, serialising every staged load)
  const float* __restrict__ X = a.X;
  const float* __restrict__ X2 = a.X2;
  const int64_t ldx = a.ldx, ldx2 = a.ldx2;
  const int nB = a.B, n_cols = a.n_cols, T = a.T;
  // block metadata through the constant address space: uniform indices ->
  // scalar loads (s_load), which the vector-load counter never waits on
  using cint = const __attribute__((address_space(4))) int32_t;
  cint* blocks = (cint*)a.blocks;
  cint* boff = (cint*)a.boff;
  const int32_t* __restrict__ rowptr_b = a.rowptr_b;
  const int4* __restrict__ drec = a.drec;

  // next block, in registers
  float4 xr[kTXRegs];
  int4 rr[kTRecRegs];
  int rp0 = 0, rp1 = 0;                  // rowptr_b[tid], rowptr_b[256] (thread 0)
  auto load_block = [&](int blk) {
    const int key = blocks[blk];
    const int c0 = (key % T) * kTC;
#pragma unroll
    for (int k = 0; k < kTXRegs; ++k) {
      const int c = c0 + grp + kGroups * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pv && c < n_cols) {
        const float* row = c < nB ? X + (int64_t)c * ldx : X2 + (int64_t)(c - nB) * ldx2;
        v = *reinterpret_cast<const float4*>(row + 4 * piece);
      }
      xr[k] = v;
    }
    const int32_t* rpb = rowptr_b + (int64_t)blk * (kTR + 1);
    rp0 = rpb[tid];
    rp1 = tid == 0 ? rpb[kTR] : 0;
    const int base = boff[blk];
    const int nrec = min(boff[blk + 1] - base, kTRecCap);
    const int4* src = drec + (base >> 1);
#pragma unroll
    for (int k = 0; k < kTRecRegs; ++k) {
      const int q = tid + kTThreads * k;
      rr[k] = 2 * q < nrec ? src[q] : make_int4(kTC, 0, kTC, 0);
    }
  };
  if (b0 < b1) load_block(b0);
  for (int blk = b0; blk < b1; ++blk) {
    __syncthreads();                       // the previous block's reads are done
#pragma unroll
    for (int k = 0; k < kTXRegs; ++k) xs[(grp + kGroups * k) * kTL + l16] = xr[k];
#pragma unroll
    for (int k = 0; k < kTRecRegs; ++k) recs[tid + kTThreads * k] = rr[k];
    rps[tid] = rp0;
    if (tid == 0) rps[kTR] = rp1;
    __syncthreads();
    const int base = boff[blk];
    if (blk + 1 < b1 && !(a.dbg & 2)) load_block(blk + 1);   // in flight under this block's work
    if (a.dbg & 1) continue;
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int ri = grp + kGroups * i;
      const int p = rps[ri], len = rps[ri + 1] - p;
      // records past the LDS copy (blocks of > kTRecCap records) from global
      if (p + len <= kTRecCap) tile_row(acc[i], recs + (p >> 1), len, xs, l16);
      else tile_row(acc[i], drec + ((base + p) >> 1), len, xs, l16);
    }
  }
  if (!pv) return;
#pragma unroll
  for (int i = 0; i < kRows; ++i) {
    const int row = w * kTR + grp + kGroups * i;
    if (row < a.n_rows) *reinterpret_cast<float4*>(a.out + (int64_t)row * a.ldo + 4 * piece) = acc[i];
  }
}

static int64_t tile_blocks(int32_t n_rows, int32_t n_cols, int* W, int* T) {
  *W = (n_rows + kTR - 1) / kTR;
  *T = (n_cols + kTC - 1) / kTC;
  return (int64_t)*W * *T;
}

static size_t scan_temp_bytes(int64_t len) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr, 0,
                                (size_t)(len > 0 ? len : 1), rocprim::plus<int32_t>(),
                                (hipStream_t)0);
  return align_up(bytes, 256);
}

}  // namespace vqgnn

using namespace vqgnn;

extern "C" int vqgnn_spmm_tile_dims(int32_t n_rows, int32_t n_cols, int32_t* windows,
                                    int32_t* tiles, int32_t* rows_per_window,
                                    int32_t* cols_per_tile) {
  int W = 0, T = 0;
  tile_blocks(n_rows, n_cols, &W, &T);
  if (windows) *windows = W;
  if (tiles) *tiles = T;
  if (rows_per_window) *rows_per_window = kTR;
  if (cols_per_tile) *cols_per_tile = kTC;
  return VQGNN_OK;
}

extern "C" size_t vqgnn_spmm_tile_plan_workspace(int32_t n_rows, int32_t n_cols, int64_t nnz) {
  (void)nnz;
  int W = 0, T = 0;
  const int64_t nblk = tile_blocks(n_rows, n_cols, &W, &T);
  // flags [nblk + 1], sparse counts per row [n_rows + 1], block totals
  // [nblk + 1], the scan temp of the longest scan
  const int64_t lmax = std::max<int64_t>(nblk + 1, (int64_t)n_rows + 1);
  return align_up((size_t)(nblk + 1) * 4, 256) + align_up((size_t)(n_rows + 1) * 4, 256) +
         align_up((size_t)(nblk + 1) * 4, 256) + scan_temp_bytes(lmax);
}

static int tile_check(const int32_t* rowptr, const int32_t* col, int32_t n_rows, int32_t n_cols,
                      int64_t nnz) {
  VQGNN_REQUIRE(rowptr && n_rows >= 0 && n_cols >= 0 && nnz >= 0 && nnz < ((int64_t)1 << 31),
                "spmm_tile_plan: bad arguments");
  VQGNN_REQUIRE(nnz == 0 || col, "spmm_tile_plan: null col");
  int W = 0, T = 0;
  VQGNN_REQUIRE(tile_blocks(n_rows, n_cols, &W, &T) < ((int64_t)1 << 28),
                "spmm_tile_plan: %d x %d blocks is too many", W, T);
  return VQGNN_OK;
}

// Phase A: grid[0][nblk] = edges per block, grid[1][nblk + 1] = exclusive
// scan of the dense flags (block ids); counts[0] = dense blocks, counts[1] =
// edges in dense blocks.
extern "C" int vqgnn_spmm_tile_plan_count(const int32_t* rowptr, const int32_t* col,
                                          int32_t n_rows, int32_t n_cols, int64_t nnz,
                                          int32_t min_edges, int32_t* grid, int32_t* counts,
                                          void* workspace, vqgnn_stream_t stream) {
  clear_error();
  const int rc = tile_check(rowptr, col, n_rows, n_cols, nnz);
  if (rc != VQGNN_OK) return rc;
  VQGNN_REQUIRE(grid && counts && workspace && min_edges >= 1, "spmm_tile_plan_count: bad arguments");
  hipStream_t s = as_stream(stream);
  int W = 0, T = 0;
  const int64_t nblk = tile_blocks(n_rows, n_cols, &W, &T);
  int32_t* cnt = grid;
  int32_t* bid = grid + nblk;
  char* ws = reinterpret_cast<char*>(workspace);
  int32_t* flag = reinterpret_cast<int32_t*>(ws);
  ws += align_up((size_t)(nblk + 1) * 4, 256) + align_up((size_t)(n_rows + 1) * 4, 256) +
        align_up((size_t)(nblk + 1) * 4, 256);
  const int64_t lmax = std::max<int64_t>(nblk + 1, (int64_t)n_rows + 1);
  size_t tb = scan_temp_bytes(lmax);
  if (hipMemsetAsync(cnt, 0, (size_t)nblk * 4, s) != hipSuccess ||
      hipMemsetAsync(counts, 0, 2 * 4, s) != hipSuccess)
    return check_launch("tile memset");
  if (n_rows > 0)
    hipLaunchKernelGGL(tile_count_kernel, dim3((unsigned)(((int64_t)n_rows * 64 + 255) / 256)),
                       dim3(256), 0, s, rowptr, col, n_rows, T, cnt);
  hipLaunchKernelGGL(tile_flags_kernel, dim3((unsigned)((nblk + 256) / 256)), dim3(256), 0, s, cnt,
                     nblk, min_edges, flag, counts + 1);
  if (rocprim::exclusive_scan(ws, tb, flag, bid, 0, (size_t)(nblk + 1), rocprim::plus<int32_t>(),
                              s) != hipSuccess)
    return check_launch("tile scan");
  // counts[0] = bid[nblk] (dense blocks); counts[1] = their edges (atomics above)
  if (hipMemcpyAsync(counts, bid + nblk, 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return check_launch("tile counts");
  return check_launch("spmm_tile_plan_count");
}

// Phase B: blocks [n_dense + W + 1] (dense block keys w*T+t in id order, then
// each window's first id), rowptr_b [n_dense][kTR + 1] (padded, per block),
// boff [n_dense + 1] (first record of each block; boff[n_dense] = records),
// drec [rec_cap] int64 records, the sparse CSR s_rowptr [n_rows + 1], s_col,
// s_val [nnz].  segcnt: caller scratch [n_dense][kTR] int32.
extern "C" int vqgnn_spmm_tile_plan_fill(const int32_t* rowptr, const int32_t* col,
                                         const float* val, int32_t n_rows, int32_t n_cols,
                                         int64_t nnz, const int32_t* grid, int32_t n_dense,
                                         int32_t* blocks, int32_t* rowptr_b, int32_t* boff,
                                         int32_t* segcnt, int64_t* drec, int64_t rec_cap,
                                         int32_t* s_rowptr, int32_t* s_col, float* s_val,
                                         void* workspace, vqgnn_stream_t stream) {
  clear_error();
  const int rc = tile_check(rowptr, col, n_rows, n_cols, nnz);
  if (rc != VQGNN_OK) return rc;
  VQGNN_REQUIRE(grid && blocks && boff && s_rowptr && workspace && n_dense >= 0,
                "spmm_tile_plan_fill: bad arguments");
  VQGNN_REQUIRE(n_dense == 0 || (rowptr_b && segcnt && drec), "spmm_tile_plan_fill: null arrays");
  VQGNN_REQUIRE(rec_cap >= 0 && rec_cap < ((int64_t)1 << 31), "spmm_tile_plan_fill: rec_cap");
  hipStream_t s = as_stream(stream);
  int W = 0, T = 0;
  const int64_t nblk = tile_blocks(n_rows, n_cols, &W, &T);
  const int32_t* cnt = grid;
  const int32_t* bid = grid + nblk;
  char* ws = reinterpret_cast<char*>(workspace);
  int32_t* flag = reinterpret_cast<int32_t*>(ws);
  ws += align_up((size_t)(nblk + 1) * 4, 256);
  int32_t* scnt = reinterpret_cast<int32_t*>(ws);
  ws += align_up((size_t)(n_rows + 1) * 4, 256);
  int32_t* btot = reinterpret_cast<int32_t*>(ws);
  ws += align_up((size_t)(nblk + 1) * 4, 256);
  const int64_t lmax = std::max<int64_t>(nblk + 1, (int64_t)n_rows + 1);
  size_t tb = scan_temp_bytes(lmax);
  (void)cnt;
  if (nblk > 0)
    hipLaunchKernelGGL(tile_flags_from_bid_kernel, dim3((unsigned)((nblk + 255) / 256)), dim3(256),
                       0, s, bid, nblk, flag);
  hipLaunchKernelGGL(tile_blocks_kernel, dim3((unsigned)((std::max<int64_t>(nblk, W + 1) + 255) / 256)),
                     dim3(256), 0, s, flag, bid, nblk, W, T, n_dense, blocks);
  if (n_dense > 0 &&
      hipMemsetAsync(segcnt, 0, (size_t)n_dense * kTR * 4, s) != hipSuccess)
    return check_launch("tile memset");
  if (n_rows > 0)
    hipLaunchKernelGGL(tile_segments_kernel, dim3((unsigned)(((int64_t)n_rows * 64 + 255) / 256)),
                       dim3(256), 0, s, rowptr, col, n_rows, T, flag, bid, segcnt, scnt);
  if (n_dense > 0)
    hipLaunchKernelGGL(tile_rowptr_kernel, dim3(n_dense), dim3(kTR), 0, s, segcnt, rowptr_b, btot);
  if (hipMemsetAsync(btot + n_dense, 0, 4, s) != hipSuccess ||
      hipMemsetAsync(scnt + n_rows, 0, 4, s) != hipSuccess)
    return check_launch("tile memset");
  if (rocprim::exclusive_scan(ws, tb, btot, boff, 0, (size_t)n_dense + 1, rocprim::plus<int32_t>(),
                              s) != hipSuccess ||
      rocprim::exclusive_scan(ws, tb, scnt, s_rowptr, 0, (size_t)n_rows + 1,
                              rocprim::plus<int32_t>(), s) != hipSuccess)
    return check_launch("tile scan");
  if (n_rows > 0)
    hipLaunchKernelGGL(tile_scatter_kernel, dim3((unsigned)(((int64_t)n_rows * 64 + 255) / 256)),
                       dim3(256), 0, s, rowptr, col, val, n_rows, T, flag, bid, rowptr_b, boff,
                       reinterpret_cast<int2*>(drec), s_rowptr, s_col, s_val);
  return check_launch("spmm_tile_plan_fill");
}

extern "C" int vqgnn_spmm_tile(int32_t n_rows, int32_t n_cols, int32_t B, const float* X,
                               int64_t ldx, const float* X2, int64_t ldx2, int32_t F, float* out,
                               int64_t ldo, const int32_t* blocks, int32_t n_dense,
                               const int32_t* rowptr_b, const int32_t* boff, const int64_t* drec,
                               vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(out && blocks && boff && n_rows >= 0 && n_cols >= 0 && n_dense >= 0,
                "spmm_tile: bad arguments");
  VQGNN_REQUIRE(n_dense == 0 || (X && rowptr_b && drec), "spmm_tile: null pointer");
  VQGNN_REQUIRE(F > 0 && F % 4 == 0, "spmm_tile: F=%d must be a positive multiple of 4", F);
  VQGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && (!X2 || ldx2 % 4 == 0) &&
                    ((uintptr_t)X & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                    ((uintptr_t)X2 & 15) == 0 && ((uintptr_t)drec & 15) == 0,
                "spmm_tile: rows and records must be 16-byte aligned");
  VQGNN_REQUIRE(B >= 0 && (X2 || B == 0), "spmm_tile: B=%d without X2", B);
  TileArgs a{};
  int W = 0, T = 0;
  tile_blocks(n_rows, n_cols, &W, &T);
  a.blocks = blocks;
  a.rowptr_b = rowptr_b;
  a.boff = boff;
  a.drec = reinterpret_cast<const int4*>(drec);
  a.n_dense = n_dense;
  a.W = W;
  a.T = T;
  a.n_rows = n_rows;
  a.n_cols = n_cols;
  a.B = X2 ? B : n_cols;
  a.X = X;
  a.ldx = ldx;
  a.X2 = X2 ? X2 : X;
  a.ldx2 = X2 ? ldx2 : ldx;
  a.F = F;
  a.out = out;
  a.ldo = ldo;
  if (const char* d = getenv("VQGNN_TILE_DBG")) a.dbg = atoi(d);
  if (W > 0) {
    static std::once_flag once;
    std::call_once(once, [] {
      (void)hipFuncSetAttribute((const void*)spmm_tile_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTileLds);
    });
    const int slices = (F / 4 + kTL - 1) / kTL;
    hipLaunchKernelGGL(spmm_tile_kernel, dim3(W, slices), dim3(kTThreads), kTileLds,
                       as_stream(stream), a);
  }
  return check_launch("spmm_tile");
}
