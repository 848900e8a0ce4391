// Codeword gather, two-source CSR SpMM, code scatter and CSR transpose for
// gfx950 (MI355X).
//
// Reference path: LowRankGNNLayer.forward (vq_gnn_v2/models.py:157-179) builds
// x_input = [x ; concat_b codebook_b[c_b[subset[B:]], :D]] and calls
// OurGCNConv.forward (convs.py:65-101) -> PyG GCNConv.message_and_aggregate ->
// torch_sparse.matmul(adj_t, x_input, reduce='add') (spmm_sum).
//
// Here: (1) gather_codewords writes x_first_order [B', F] once per
// out-of-batch node (one coalesced 4*F-byte row per node; the codebooks are
// L2-resident) — measured 2.3x faster than gathering codewords per edge,
// where each edge touches nb different codebook lines; (2) the SpMM reads
// rows j < B from x and rows j >= B from x_first_order (no torch.cat copy).
//
// SpMM work decomposition: edge-balanced.  The nnz range is cut into chunks
// of S edges; a lane group (G lanes, float4 column chunks each) owns the rows
// that START in its chunk and sums each of them in CSR order with separate
// mul and add (spmm_sum's `out = out + val * x`, init 0) — bit-identical to
// the reference loop.  Rows longer than L edges are cut at chunk boundaries
// instead; their per-chunk partials ("carries") are added in chunk order by
// a fix-up kernel, so Zipf hub rows spread over many groups.

#include "common.h"

#include <cstdlib>
#include <utility>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

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
  int L;          // rows longer than L edges are split at chunk boundaries
  int nchunks;
  int B;          // columns < B read X; >= B read X2 (row j - B)
  const float* X;
  int64_t ldx4;   // in float4
  const float* X2;
  int64_t ldx24;
  int F4;         // F / 4
  float* out;
  int64_t ldo4;
  float* carry;   // [nchunks][2][F]
  int* carry_row; // [nchunks]
  // wave kernel: X and X2 addressed as one 32-bit byte range from ubase
  const char* ubase;
  uint32_t span;  // bytes (buffer range; loads outside it return 0)
  uint32_t offx, ldxb;    // X row j at offx + j*ldxb
  uint32_t offx2, ldx2b;  // X2 row j-B at offx2 + (j-B)*ldx2b
  int kpw;                // wave kernel: consecutive chunks per wave
  const int* chunk_row;   // [nchunks] first row starting at or after chunk*S (or null)
  int dbg;                // experiments: 1 = no gathers, 2 = no output stores, 4 = stamps
  unsigned long long* stamps;  // dbg & 4: [waves][8] s_memtime stamps
};

template <int NCH>
__host__ __device__ constexpr int spmm_unroll() {
  return NCH <= 2 ? 8 : (NCH <= 4 ? 4 : 2);
}

// Accumulate edges [eb, ee) into acc (float4 x NCH), in CSR order.  The
// group's lanes first load up to G consecutive (col, val) pairs with one
// coalesced access each, then walk them U at a time: every lane fetches U
// independent float4 rows (X for j < B; for j >= B the int16 code first,
// then the codeword's feature half) before adding them in order.
template <int G, int NCH, bool TWO>
__device__ __forceinline__ void spmm_segment(const SpmmArgs& a, int eb, int ee, int lg,
                                             float4 (&acc)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* X4 = reinterpret_cast<const float4*>(a.X);
  const float4* Y4 = reinterpret_cast<const float4*>(a.X2);
  constexpr int U = spmm_unroll<NCH>();
  for (int base = eb; base < ee; base += G) {
    const int e = base + lg;
    const bool ok = e < ee;
    const int myj = ok ? a.col[e] : -1;
    const float myw = ok ? a.val[e] : 0.f;
    const int cnt = min(G, ee - base);
    for (int k = 0; k < cnt; k += U) {
      int jj[U];
      float ww[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int src = min(k + u, G - 1);
        const int j = __shfl(myj, src, G);
        const float w = __shfl(myw, src, G);
        const bool v = k + u < cnt;
        jj[u] = v ? j : -1;
        ww[u] = v ? w : 0.f;
      }
      float4 v[U][NCH];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = jj[u];
        const float4* row = (!TWO || j < a.B) ? X4 + (int64_t)j * a.ldx4
                                              : Y4 + (int64_t)(j - a.B) * a.ldx24;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int cc = lg + c * G;
          v[u][c] = (j >= 0 && cc < a.F4) ? row[cc] : make_float4(0.f, 0.f, 0.f, 0.f);
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
}

template <int G, int NCH>
__device__ __forceinline__ void store_row(float4* dst, int lg, int F4, const float4 (&acc)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int cc = lg + c * G;
    if (cc < F4) dst[cc] = acc[c];
  }
}

// Row ownership: chunk g owns every row whose first edge lies in
// [g*S, (g+1)*S) (plus, for the last chunk, trailing empty rows).  A row of at
// most L edges is summed entirely by its owner, even past the chunk end, so
// it is bit-identical to spmm_sum's sequential loop; only rows longer than L
// are cut at chunk boundaries and leave per-chunk partials ("carries").
// Chunk -> XCD placement (speed only): each XCD receives a contiguous 1/8 of
// the chunks before the split edge (rows < B: batch rows, whose neighbours are
// mostly intra-cluster and therefore L2-local) and a contiguous 1/8 of the
// chunks after it (the out-of-batch rows, whose gathers are mostly random), so
// neither the L2 locality nor the XCD balance is lost.  Blocks b and b+8
// share an XCD under the observed round-robin dispatch.
__device__ __forceinline__ int spmm_chunk_of(int blk, int group, int gpw, int nchunks,
                                             int split) {
  const int xcd = blk % kNumXcd, local = blk / kNumXcd;
  const int c1 = split, c2 = nchunks - split;
  const int a1 = xcd * c1 / kNumXcd, n1 = (xcd + 1) * c1 / kNumXcd - a1;
  const int a2 = split + xcd * c2 / kNumXcd, n2 = split + (xcd + 1) * c2 / kNumXcd - a2;
  const int lc = local * gpw + group;
  if (lc < n1) return a1 + lc;
  if (lc < n1 + n2) return a2 + (lc - n1);
  return -1;
}

template <int G, int NCH, bool TWO>
__global__ void __launch_bounds__(kSpmmThreads)
spmm_merge_kernel(SpmmArgs a) {
  constexpr int GPW = kSpmmThreads / G;  // groups per workgroup
  const int lg = threadIdx.x % G;
  int split = a.nchunks;
  if (TWO && a.B < a.n_rows) split = min(a.nchunks, a.rowptr[a.B] / a.S);
  const int chunk = spmm_chunk_of(blockIdx.x, threadIdx.x / G, GPW, a.nchunks, split);
  if (chunk < 0) return;
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
    const int rs = a.rowptr[i - 1];
    if (a.rowptr[i] - rs > a.L) {     // long row: this chunk's piece is a carry
      const int re = min(a.rowptr[i], e1);
      spmm_segment<G, NCH, TWO>(a, e0, re, lg, acc);
      store_row<G, NCH>(carry4 + (int64_t)chunk * 2 * F4, lg, F4, acc);
      crow = i - 1;
    }
  }
  int rb = (i < a.n_rows) ? a.rowptr[i] : 0;
  for (; i < a.n_rows; ++i) {
    if (!(rb < e1 || last)) break;
    const int re_full = a.rowptr[i + 1];
    if (re_full - rb <= a.L) {
      spmm_segment<G, NCH, TWO>(a, rb, re_full, lg, acc);
      store_row<G, NCH>(out4 + (int64_t)i * a.ldo4, lg, F4, acc);
    } else {
      const int re = min(re_full, e1);
      spmm_segment<G, NCH, TWO>(a, rb, re, lg, acc);
      if (re_full <= e1) {
        store_row<G, NCH>(out4 + (int64_t)i * a.ldo4, lg, F4, acc);
      } else {
        store_row<G, NCH>(carry4 + ((int64_t)chunk * 2 + 1) * F4, lg, F4, acc);
        break;
      }
    }
    rb = re_full;
  }
  if (lg == 0) a.carry_row[chunk] = crow;
}

// ---------------------------------------------------------------------------
// Wave kernel for F = 64*V (V = 1, 2, 4): one wave owns a chunk (same row
// ownership and carries as the merge kernel) and each lane owns V consecutive
// columns of every row.  The edge stream is wave-uniform and costs no per-lane
// address arithmetic: a 64-edge window of (input-row byte offset, weight) is
// staged with one coalesced load per 64 edges (lane l holds edge wb + l), and
// edge k is read back with v_readlane into SGPRs, which feed the buffer
// load's scalar offset and the multiply directly.  X and X2 (the two input
// sources) are one 32-bit byte range from ubase, so there is no per-edge
// source select.  Per edge and wave: 2 v_readlane, 1 buffer load of 4*F
// bytes, V v_mul + V v_add (spmm_sum order) — against ~30 VALU per edge for
// the lane-group kernel, which is VALU-bound on address math and shuffles.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}


template <int V>
__device__ __forceinline__ void buf_load(__amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t so,
                                         float (&v)[V]) {
  // bit_cast the builtin's result straight to float2/float4: extracting the
  // elements of its integer-vector type miscompiles here (ROCm 7.2 clang
  // loads only the first dword)
  if constexpr (V == 1) {
    v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0));
  } else if constexpr (V == 2) {
    const float2 t = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0));
    v[0] = t.x;
    v[1] = t.y;
  } else {
    const float4 t =
        __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0));
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  }
}

template <int V>
__device__ __forceinline__ void vstore(float* p, const float (&v)[V]) {
  if constexpr (V == 1) {
    *p = v[0];
  } else if constexpr (V == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// lane l of the window holds edge wb + l: where its input row is (a 32-bit
// offset into the buffer range, or — FAR — the row's 64-bit address when X
// and X2 are more than 4 GiB apart) and its weight
template <bool FAR>
struct EdgeWindow {
  int wb;
  uint32_t off;   // FAR: low half of the address
  uint32_t hi;    // FAR: high half
  float w;
};

template <bool FAR>
__device__ __forceinline__ void window_stage(const SpmmArgs& a, EdgeWindow<FAR>& win, int wb,
                                             int lane) {
  win.wb = wb;
  const int e = wb + lane;
  const bool ok = e < a.nnz;
  const int j = ok ? a.col[e] : 0;
  win.w = ok ? a.val[e] : 0.f;
  if constexpr (FAR) {
    const float* row = j < a.B ? a.X + (int64_t)j * a.ldx4 * 4
                               : a.X2 + (int64_t)(j - a.B) * a.ldx24 * 4;
    const uint64_t p = (uint64_t)(uintptr_t)row;
    win.off = (uint32_t)p;
    win.hi = (uint32_t)(p >> 32);
  } else {
    win.off = j < a.B ? a.offx + (uint32_t)j * a.ldxb : a.offx2 + (uint32_t)(j - a.B) * a.ldx2b;
    win.hi = 0;
  }
}

// lane l holds rowptr[base + l]: row bounds by v_readlane, no scalar-load
// round trip at every row boundary (rows average ~16 edges)
struct RowWindow {
  int base;
  int rp;
};

__device__ __forceinline__ int row_at(const SpmmArgs& a, RowWindow& rw, int idx, int lane) {
  if (idx < rw.base || idx >= rw.base + 64) {
    rw.base = idx;
    rw.rp = a.rowptr[min(idx + lane, a.n_rows)];
  }
  return __builtin_amdgcn_readlane(rw.rp, uni(idx - rw.base));
}

// row k of the window, this lane's V columns
template <int V, bool FAR>
__device__ __forceinline__ void window_load(__amdgpu_buffer_rsrc_t rs, const EdgeWindow<FAR>& win,
                                            int k, uint32_t lo, int lane, float (&v)[V]) {
  if constexpr (FAR) {
    const uint32_t plo = __builtin_amdgcn_readlane(win.off, k);
    const uint32_t phi = __builtin_amdgcn_readlane(win.hi, k);
    // a buffer descriptor over this one row (built in SGPRs from the
    // read-back address): the same scalar-base load as the near path
    const uint64_t p = ((uint64_t)phi << 32) | plo;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>((uintptr_t)p), 0, 64 * V * 4, 0x00020000);
    buf_load<V>(rr, lo, 0, v);
  } else {
    buf_load<V>(rs, lo, __builtin_amdgcn_readlane(win.off, k), v);
  }
}

template <int V, int U, bool FAR>
__device__ __forceinline__ void wave_segment(const SpmmArgs& a, __amdgpu_buffer_rsrc_t rs,
                                             EdgeWindow<FAR>& win, int eb, int ee, int lane,
                                             float (&acc)[V]) {
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = 0.f;
  const uint32_t lo = (uint32_t)lane * V * 4;
  int e = eb;
  while (e < ee) {
    if (e < win.wb || e >= win.wb + 64) window_stage(a, win, e, lane);
    const int lim = min(ee, win.wb + 64);
    for (; e + U <= lim; e += U) {
      const int k0 = e - win.wb;
      float v[U][V];
      float ww[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ww[u] = __builtin_bit_cast(float,
                                   __builtin_amdgcn_readlane(__builtin_bit_cast(int, win.w), k0 + u));
        window_load<V, FAR>(rs, win, k0 + u, lo, lane, v[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] = __fadd_rn(acc[k], __fmul_rn(ww[u], v[u][k]));
      }
    }
    for (; e < lim; ++e) {
      const int k0 = e - win.wb;
      const float w =
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, win.w), k0));
      float v[V];
      window_load<V, FAR>(rs, win, k0, lo, lane, v);
#pragma unroll
      for (int k = 0; k < V; ++k) acc[k] = __fadd_rn(acc[k], __fmul_rn(w, v[k]));
    }
  }
}

// ---------------------------------------------------------------------------
// Paired variant for F = 128: the row's edges are taken two at a time, one
// dwordx4 wave-instruction loading edge e into lanes 0-31 and edge e+1 into
// lanes 32-63 (the texture addresser costs the same per wave-instruction, so
// this halves its work per edge: probe scripts/probes/gather_shape.hip, 1.75x
// the rows/s of one 512-B row per instruction).  Each half multiplies by its
// own weight; v_permlane32_swap moves the upper half's product to lanes 0-31,
// which add p_e then p_e+1 — the sequential CSR order of spmm_sum, bit-exact.
// acc (4 floats) is meaningful in lanes 0-31 only.
// ---------------------------------------------------------------------------
struct U32x2 {
  unsigned a, b;
};

__device__ __forceinline__ float upper_to_lower(float p) {
  // lanes 0-31 <- lanes 32-63 of p (second result of the swap; element
  // access by struct bit_cast: vector subscripts miscompile here)
  const U32x2 r = __builtin_bit_cast(
      U32x2, __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, p),
                                              __builtin_bit_cast(unsigned, p), false, false));
  return __builtin_bit_cast(float, r.b);
}

template <bool FAR>
__device__ __forceinline__ void pair_load(__amdgpu_buffer_rsrc_t rs, const EdgeWindow<FAR>& win,
                                          int ka, int kb, bool upper, uint32_t lo16,
                                          float (&v)[4]) {
  if constexpr (FAR) {
    const uint32_t la = __builtin_amdgcn_readlane(win.off, ka);
    const uint32_t ha = __builtin_amdgcn_readlane(win.hi, ka);
    const uint32_t lb = __builtin_amdgcn_readlane(win.off, kb);
    const uint32_t hb = __builtin_amdgcn_readlane(win.hi, kb);
    const uint64_t p = upper ? (((uint64_t)hb << 32) | lb) : (((uint64_t)ha << 32) | la);
    const float4 t = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(p) + lo16);
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  } else {
    const uint32_t sa = __builtin_amdgcn_readlane(win.off, ka);
    const uint32_t sb = __builtin_amdgcn_readlane(win.off, kb);
    const float4 t = __builtin_bit_cast(
        float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (upper ? sb : sa) + lo16, 0, 0));
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  }
}

template <bool FAR>
__device__ __forceinline__ void single_load(__amdgpu_buffer_rsrc_t rs, const EdgeWindow<FAR>& win,
                                            int k, uint32_t lo16, float (&v)[4]) {
  if constexpr (FAR) {
    const uint32_t l = __builtin_amdgcn_readlane(win.off, k);
    const uint32_t h = __builtin_amdgcn_readlane(win.hi, k);
    const float4 t = *reinterpret_cast<const float4*>(
        reinterpret_cast<const char*>((((uint64_t)h << 32) | l)) + lo16);
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  } else {
    const float4 t = __builtin_bit_cast(
        float4, __builtin_amdgcn_raw_buffer_load_b128(rs, lo16, __builtin_amdgcn_readlane(win.off, k),
                                                      0));
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  }
}

template <int UP, bool FAR>
__device__ __forceinline__ void wave_segment_pair(const SpmmArgs& a, __amdgpu_buffer_rsrc_t rs,
                                                  EdgeWindow<FAR>& win, int eb, int ee, int lane,
                                                  float (&acc)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = 0.f;
  const bool upper = lane >= 32;
  const uint32_t lo16 = (uint32_t)(lane & 31) * 16;
  const int up4 = upper ? 4 : 0;
  int e = eb;
  while (e < ee) {
    if (e < win.wb || e >= win.wb + 64) window_stage(a, win, e, lane);
    const int lim = min(ee, win.wb + 64);
    for (; e + 2 * UP <= lim; e += 2 * UP) {
      const int k0 = uni(e - win.wb);
      // lane reads window lane k0 + 2u + upper: one address per group, the
      // pair index in ds_bpermute's immediate offset
      const int addr = k0 * 4 + up4;
      float v[UP][4];
      float ww[UP];
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        int off, wbits;
        if constexpr (FAR) {
          const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(addr + 8 * u, (int)win.off);
          const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(addr + 8 * u, (int)win.hi);
          const float4 t = *reinterpret_cast<const float4*>(
              reinterpret_cast<const char*>((((uint64_t)hi << 32) | lo)) + lo16);
          v[u][0] = t.x;
          v[u][1] = t.y;
          v[u][2] = t.z;
          v[u][3] = t.w;
          off = 0;
        } else {
          off = __builtin_amdgcn_ds_bpermute(addr + 8 * u, (int)win.off);
          const float4 t = (a.dbg & 1) ? make_float4(1.f, 1.f, 1.f, (float)off) : __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)off + lo16, 0, 0));
          v[u][0] = t.x;
          v[u][1] = t.y;
          v[u][2] = t.z;
          v[u][3] = t.w;
        }
        wbits = __builtin_amdgcn_ds_bpermute(addr + 8 * u, __builtin_bit_cast(int, win.w));
        ww[u] = __builtin_bit_cast(float, wbits);
      }
#pragma unroll
      for (int u = 0; u < UP; ++u) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float p = __fmul_rn(ww[u], v[u][k]);
          acc[k] = __fadd_rn(__fadd_rn(acc[k], p), upper_to_lower(p));
        }
      }
    }
    for (; e + 2 <= lim; e += 2) {
      const int ka = uni(e - win.wb), kb = ka + 1;
      const float wa = __builtin_bit_cast(
          float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, win.w), ka));
      const float wb = __builtin_bit_cast(
          float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, win.w), kb));
      float v[4];
      pair_load<FAR>(rs, win, ka, kb, upper, lo16, v);
      const float w = upper ? wb : wa;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float p = __fmul_rn(w, v[k]);
        acc[k] = __fadd_rn(__fadd_rn(acc[k], p), upper_to_lower(p));
      }
    }
    if (e < lim) {   // odd last edge of the row (or window): lanes 0-31 only
      const int k = uni(e - win.wb);
      const float w = __builtin_bit_cast(
          float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, win.w), k));
      if (!upper) {
        float v[4];
        single_load<FAR>(rs, win, k, lo16, v);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __fadd_rn(acc[c], __fmul_rn(w, v[c]));
      }
      ++e;
    }
  }
}

// chunk_row[c] = first row whose start is >= c*S: one thread per chunk, the
// searches in parallel instead of as a dependent chain at every wave's head
__global__ void spmm_chunk_rows_kernel(const int32_t* __restrict__ rowptr, int n_rows, int S,
                                       int nchunks, int* __restrict__ chunk_row) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nchunks) chunk_row[c] = lower_bound_i32(rowptr, n_rows, c * S);
}

// One chunk (rows owned by chunk, carries) starting at row i; returns the
// first row of the next chunk.  PAIR: F = 128 in the paired form (acc = 4
// floats in lanes 0-31; V must be 4).
template <int V, int U, bool FAR, bool PAIR>
__device__ __forceinline__ void segment(const SpmmArgs& a, __amdgpu_buffer_rsrc_t rs,
                                        EdgeWindow<FAR>& win, int eb, int ee, int lane,
                                        float (&acc)[V]) {
  if constexpr (PAIR) wave_segment_pair<U / 2, FAR>(a, rs, win, eb, ee, lane, acc);
  else wave_segment<V, U, FAR>(a, rs, win, eb, ee, lane, acc);
}

// Seg: seg(eb, ee, acc) sums edges [eb, ee) of the CSR into acc in CSR order
// (the wave's edge window and sources live in the functor).  st: this lane
// stores output columns.
template <int V, class Seg>
__device__ __forceinline__ int wave_chunk_rows(const SpmmArgs& a, Seg& seg, RowWindow& rw,
                                               int chunk, int i, int lane, bool st) {
  const int e0 = chunk * a.S;
  const int e1 = min(e0 + a.S, a.nnz);
  const bool last = e1 == a.nnz;
  const int F = a.F4 * 4;
  const int ldo = (int)(a.ldo4 * 4);
  int crow = -1;
  float acc[V];
  if (i > 0) {
    const int ri = row_at(a, rw, i, lane);
    if (ri > e0) {  // row i-1 started before this chunk
      const int rs0 = row_at(a, rw, i - 1, lane);
      if (ri - rs0 > a.L) {
        const int re = min(ri, e1);
        seg(e0, re, acc);
        if (st) vstore<V>(a.carry + (int64_t)chunk * 2 * F + lane * V, acc);
        crow = i - 1;
      }
    }
  }
  int next = -1;
  int rb = (i < a.n_rows) ? row_at(a, rw, i, lane) : 0;
  for (; i < a.n_rows; ++i) {
    if (!(rb < e1 || last)) break;
    const int re_full = row_at(a, rw, i + 1, lane);
    if (re_full - rb <= a.L) {
      seg(rb, re_full, acc);
      if (st) vstore<V>(a.out + (int64_t)i * ldo + lane * V, acc);
    } else {
      const int re = min(re_full, e1);
      seg(rb, re, acc);
      if (re_full <= e1) {
        if (st) vstore<V>(a.out + (int64_t)i * ldo + lane * V, acc);
      } else {
        if (st) vstore<V>(a.carry + ((int64_t)chunk * 2 + 1) * F + lane * V, acc);
        next = i + 1;   // the row continues into the next chunk
        break;
      }
    }
    rb = re_full;
  }
  if (lane == 0) a.carry_row[chunk] = crow;
  return next >= 0 ? next : i;
}

template <int V, int U, bool FAR, bool PAIR>
struct WaveSeg {
  const SpmmArgs& a;
  __amdgpu_buffer_rsrc_t rs;
  EdgeWindow<FAR>& win;
  int lane;
  __device__ __forceinline__ void operator()(int eb, int ee, float (&acc)[V]) {
    segment<V, U, FAR, PAIR>(a, rs, win, eb, ee, lane, acc);
  }
};

template <int V, int U, bool FAR, bool PAIR>
__device__ __forceinline__ int wave_chunk(const SpmmArgs& a, __amdgpu_buffer_rsrc_t rs,
                                          EdgeWindow<FAR>& win, RowWindow& rw, int chunk, int i,
                                          int lane) {
  WaveSeg<V, U, FAR, PAIR> seg{a, rs, win, lane};
  const bool st = (!PAIR || lane < 32) && !(a.dbg & 2);    // lanes that own output columns
  return wave_chunk_rows<V>(a, seg, rw, chunk, i, lane, st);
}

// ---------------------------------------------------------------------------
// Code-source SpMM: x_first_order is never materialised.  Rows j >= B of
// x_input are concat_b codebook_b[code(j, b)][:D] (models.py:168-174), so the
// codebooks' feature halves (nb*M*D floats, at most kCodesLdsFloats) are
// staged once per workgroup into LDS, and an edge from an out-of-batch source
// reads its 2*nb-byte code record (lcodes [B', nb], L2-resident) plus, per
// lane, V columns from LDS — instead of a 4*F-byte row from x_first_order.
// Rows, carries, CSR order and the separate mul/add are those of
// spmm_wave_kernel (bit-identical output).  The edge window marks which of
// its 64 edges come from codes (a ballot); a row is walked as runs of one
// source type, each run U-unrolled like wave_segment.
// Persistent: the LDS image allows one 16-wave workgroup per CU; the waves of
// an XCD stride over that XCD's chunks, so at any time they work on
// neighbouring chunks (the L2 locality of the dispatch-ordered kernel).
// ---------------------------------------------------------------------------
constexpr int kCodesThreads = 1024;
constexpr int kCodesLdsFloats = 32768;   // 128 KiB of the CU's 160 KiB

struct CodesSrc {
  const int16_t* lcodes;   // [n_cols - B][ldlc]
  uint32_t ldlcb;          // bytes per lcodes row
  uint32_t lcspan;         // bytes of lcodes
  const float* emb;        // feature half of codeword (b, m): emb + b*bstride + m*ldw + off
  int64_t bstride;
  int ldw, off, M, D, nb;
};

struct CodeWindow {
  int wb;
  uint32_t off;            // X row byte offset (j < B) or code-record byte offset (j >= B)
  float w;
  uint64_t cmask;          // bit l: edge wb + l reads codes
};

__device__ __forceinline__ void code_window_stage(const SpmmArgs& a, const CodesSrc& c,
                                                  CodeWindow& win, int wb, int lane) {
  win.wb = wb;
  const int e = wb + lane;
  const bool ok = e < a.nnz;
  const int j = ok ? a.col[e] : 0;
  win.w = ok ? a.val[e] : 0.f;
  const bool code = ok && j >= a.B;
  win.off = code ? (uint32_t)(j - a.B) * c.ldlcb : (uint32_t)j * a.ldxb;
  const uint64_t bm = __ballot(code);
  win.cmask = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(bm >> 32)) << 32) |
              (uint32_t)__builtin_amdgcn_readfirstlane((int)bm);
}

template <int V, int U>
struct CodeSeg {
  const SpmmArgs& a;
  const CodesSrc& c;
  __amdgpu_buffer_rsrc_t rsx;   // X
  __amdgpu_buffer_rsrc_t rsc;   // lcodes
  CodeWindow& win;
  int lane;
  uint32_t lo;                  // this lane's byte offset in an X row
  uint32_t coff;                // this lane's byte offset in a code record
  const float* cb;              // this lane's LDS codebook base (branch, first column)

  __device__ __forceinline__ float wt(int k) const {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, win.w), k));
  }
  __device__ __forceinline__ void cw(unsigned code, float (&v)[V]) const {
    const float* p = cb + code * (unsigned)c.D;
    if constexpr (V == 1) {
      v[0] = p[0];
    } else if constexpr (V == 2) {
      const float2 t = *reinterpret_cast<const float2*>(p);
      v[0] = t.x;
      v[1] = t.y;
    } else {
      const float4 t = *reinterpret_cast<const float4*>(p);
      v[0] = t.x;
      v[1] = t.y;
      v[2] = t.z;
      v[3] = t.w;
    }
  }
  __device__ __forceinline__ unsigned code_at(int k) const {
    return __builtin_amdgcn_raw_buffer_load_b16(rsc, coff, __builtin_amdgcn_readlane(win.off, k), 0);
  }
  // Runs are walked U edges at a time.  The short last group re-loads its
  // last valid edge into the unused slots (no branches around the loads, so
  // all U are in flight before the first add) and leaves its add chain early
  // with a wave-uniform branch: a run's tail costs one memory latency, not one
  // per edge.  (The empty asm keeps the compiler from turning the early exits
  // into per-column selects.)
  template <class Load>
  __device__ __forceinline__ void run(int e, int lim, float (&acc)[V], Load&& load) {
    for (; e + U <= lim; e += U) {
      const int k0 = uni(e - win.wb);
      float v[U][V];
      float ww[U];
      load(k0, U - 1, v, ww);
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] = __fadd_rn(acc[k], __fmul_rn(ww[u], v[u][k]));
      }
    }
    if (e < lim) {
      const int k0 = uni(e - win.wb);
      const int cnt = uni(lim - e);
      float v[U][V];
      float ww[U];
      load(k0, cnt - 1, v, ww);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u >= cnt) break;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] = __fadd_rn(acc[k], __fmul_rn(ww[u], v[u][k]));
      }
    }
  }
  __device__ __forceinline__ void x_run(int e, int lim, float (&acc)[V]) {
    run(e, lim, acc, [&](int k0, int last, float (&v)[U][V], float (&ww)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = k0 + min(u, last);
        ww[u] = wt(kk);
        buf_load<V>(rsx, lo, __builtin_amdgcn_readlane(win.off, kk), v[u]);
      }
    });
  }
  __device__ __forceinline__ void code_run(int e, int lim, float (&acc)[V]) {
    run(e, lim, acc, [&](int k0, int last, float (&v)[U][V], float (&ww)[U]) {
      unsigned cd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = k0 + min(u, last);
        ww[u] = wt(kk);
        cd[u] = code_at(kk);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) cw(cd[u], v[u]);
    });
  }
  __device__ __forceinline__ void operator()(int eb, int ee, float (&acc)[V]) {
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    int e = eb;
    while (e < ee) {
      if (e < win.wb || e >= win.wb + 64) code_window_stage(a, c, win, e, lane);
      const int lim = uni(min(ee, win.wb + 64));
      while (e < lim) {
        // the run of edges with this edge's source type (CSR sorts a row's
        // columns, so a row is one X run then one code run; any order works)
        const int k = uni(e - win.wb);
        const uint64_t m = win.cmask >> k;
        const bool code = (m & 1ull) != 0;
        const uint64_t t = code ? ~m : m;
        const int r = uni(min(lim, e + (t ? (int)__builtin_ctzll(t) : 64)));
        if (code) code_run(e, r, acc);
        else x_run(e, r, acc);
        e = r;
      }
    }
  }
};

// ---------------------------------------------------------------------------
// Flat chunk walk: the wave issues the loads of G consecutive edges at once,
// across row boundaries, and then adds them in CSR order, closing a row (store
// + reset) when the add reaches its end.  Rows are still summed sequentially
// from zero in CSR order with separate mul and add (bit-identical), but up to
// G rows are in flight per wave instead of at most U of one row, and a row's
// tail costs no extra memory latency.  Segments (what the adds close) follow
// wave_chunk_rows' ownership: the head piece of a long row that began in an
// earlier chunk (carry slot 0), then the rows that start in the chunk (a row
// longer than L cut at the chunk end: carry slot 1).
// CODES: an edge whose source is >= B reads its code record and then its V
// columns of the codeword from the LDS codebook (cb = this lane's base).
// ---------------------------------------------------------------------------
struct FlatSrc {
  __amdgpu_buffer_rsrc_t rsx;   // X (CODES) or the X/X2 range
  __amdgpu_buffer_rsrc_t rsc;   // lcodes (CODES)
  uint32_t lo;                  // this lane's byte offset in an input row
  uint32_t coff;                // this lane's byte offset in a code record
  const float* cb;              // this lane's LDS codebook base (CODES)
  uint32_t D;
  uint32_t ldlcb;               // bytes per code record
};

template <bool CODES>
__device__ __forceinline__ void flat_stage(const SpmmArgs& a, const FlatSrc& f, CodeWindow& win,
                                           int wb, int lane) {
  win.wb = wb;
  const int e = wb + lane;
  const bool ok = e < a.nnz;
  const int j = ok ? a.col[e] : 0;
  win.w = ok ? a.val[e] : 0.f;
  if constexpr (CODES) {
    const bool code = ok && j >= a.B;
    win.off = code ? (uint32_t)(j - a.B) * f.ldlcb : (uint32_t)j * a.ldxb;
    const uint64_t bm = __ballot(code);
    win.cmask = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(bm >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((int)bm);
  } else {
    win.off = j < a.B ? a.offx + (uint32_t)j * a.ldxb : a.offx2 + (uint32_t)(j - a.B) * a.ldx2b;
    win.cmask = 0;
  }
}

template <int V, int G, bool CODES>
__device__ __forceinline__ void flat_chunk(const SpmmArgs& a, const FlatSrc& f, CodeWindow& win,
                                           RowWindow& rw, int chunk, int i0, int lane) {
  const int e0 = chunk * a.S;
  const int e1 = min(e0 + a.S, a.nnz);
  const int F = a.F4 * 4;
  const int64_t ldo = a.ldo4 * 4;
  const bool st = !(a.dbg & 2);
  // rows starting in [e0, e1): [i0, ir); the last chunk also owns trailing empty rows
  const int ir = chunk + 1 < a.nchunks
                     ? uni(a.chunk_row ? min(a.chunk_row[chunk + 1], a.n_rows)
                                       : lower_bound_i32(a.rowptr, a.n_rows, e1))
                     : a.n_rows;
  // one row window over [i0 - 1, i0 + 63): the closes below re-stage it only
  // for chunks owning more than 62 rows (a dependent load there drains the
  // group's loads)
  {
    const int lo = i0 > 0 ? i0 - 1 : 0;
    const int hi = min(ir, lo + 63);
    if (lo < rw.base || hi >= rw.base + 64) {
      rw.base = lo;
      rw.rp = a.rowptr[min(lo + lane, a.n_rows)];
    }
  }
  // empty owned rows are zeroed up front, so that the add phase below closes
  // at most one row per edge (one conditional store: the waitcnt pass keeps
  // its per-load counts instead of draining at every edge)
  for (int r = i0; r < ir; ++r) {
    if (row_at(a, rw, r, lane) == row_at(a, rw, r + 1, lane) && st) {
      float z[V];
#pragma unroll
      for (int k = 0; k < V; ++k) z[k] = 0.f;
      vstore<V>(a.out + (int64_t)r * ldo + lane * V, z);
    }
  }
  int crow = -1;
  int i = i0;
  int s_end = 0;
  float* dptr = nullptr;   // wave-uniform destination row of the open segment
  bool more = true;
  bool head = false;
  if (i0 > 0) {
    const int ri = row_at(a, rw, i0, lane);
    if (ri > e0) {
      const int rs0 = row_at(a, rw, i0 - 1, lane);
      if (ri - rs0 > a.L) {   // the piece of a long row that started before e0
        head = true;
        crow = i0 - 1;
        s_end = min(ri, e1);
        dptr = a.carry + (int64_t)chunk * 2 * F;
      }
    }
  }
  // next non-empty owned row: [start, s_end) -> dptr
  auto next_row = [&]() -> bool {
    while (more && i < ir) {
      const int rb = row_at(a, rw, i, lane);
      const int re_full = row_at(a, rw, i + 1, lane);
      const int r = i++;
      if (re_full == rb) continue;
      if (re_full - rb <= a.L) {
        s_end = re_full;
        dptr = a.out + (int64_t)r * ldo;
      } else {
        s_end = min(re_full, e1);
        if (re_full <= e1) {
          dptr = a.out + (int64_t)r * ldo;
        } else {
          dptr = a.carry + ((int64_t)chunk * 2 + 1) * F;
          more = false;
        }
      }
      return true;
    }
    return false;
  };
  int E0, E;
  if (head) {
    E0 = e0;
    E = s_end;
  } else {
    E0 = i0 < ir ? row_at(a, rw, i0, lane) : e0;
    E = E0;
  }
  if (ir > i0) {
    const int r = ir - 1;
    const int rs = row_at(a, rw, r, lane), re = row_at(a, rw, r + 1, lane);
    E = re - rs > a.L ? min(re, e1) : re;
  }
  bool live = head || next_row();
  float acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = 0.f;
  for (int e = E0; e < E; e += G) {
    const int cnt = uni(min(G, E - e));
    if (e < win.wb || e + cnt > win.wb + 64) flat_stage<CODES>(a, f, win, e, lane);
    const int k0 = uni(e - win.wb);
    float v[G][V];
    float ww[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int k = k0 + min(u, cnt - 1);   // unused slots re-read the last edge (no add)
      ww[u] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, win.w), k));
      const uint32_t so = __builtin_amdgcn_readlane(win.off, k);
      if constexpr (CODES) {
        if ((win.cmask >> k) & 1ull) {   // the code, in v[u][0]'s register
          v[u][0] = __builtin_bit_cast(
              float, (unsigned)__builtin_amdgcn_raw_buffer_load_b16(f.rsc, f.coff, so, 0));
        } else {
          buf_load<V>(f.rsx, f.lo, so, v[u]);
        }
      } else {
        buf_load<V>(f.rsx, f.lo, so, v[u]);
      }
    }
    if constexpr (CODES) {
#pragma unroll
      for (int u = 0; u < G; ++u) {
        if ((win.cmask >> (k0 + min(u, cnt - 1))) & 1ull) {
          const float* p = f.cb + __builtin_bit_cast(unsigned, v[u][0]) * f.D;
          if constexpr (V == 1) {
            v[u][0] = p[0];
          } else if constexpr (V == 2) {
            const float2 t = *reinterpret_cast<const float2*>(p);
            v[u][0] = t.x;
            v[u][1] = t.y;
          } else {
            const float4 t = *reinterpret_cast<const float4*>(p);
            v[u][0] = t.x;
            v[u][1] = t.y;
            v[u][2] = t.z;
            v[u][3] = t.w;
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (u < cnt) {
        if (e + u == s_end) {   // the open row ends before this edge: close it
          if (st) vstore<V>(dptr + lane * V, acc);
#pragma unroll
          for (int k = 0; k < V; ++k) acc[k] = 0.f;
          live = next_row();
        }
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] = __fadd_rn(acc[k], __fmul_rn(ww[u], v[u][k]));
      }
    }
  }
  if (live && st) vstore<V>(dptr + lane * V, acc);
  if (lane == 0) a.carry_row[chunk] = crow;
}

// Non-persistent flat kernel (one wave per chunk, as spmm_wave_kernel): X and
// X2 as one 32-bit buffer range.
template <int V, int G>
__global__ void __launch_bounds__(kSpmmThreads)
spmm_flat_kernel(SpmmArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  int split = a.nchunks;
  if (a.B < a.n_rows) split = min(a.nchunks, uni(a.rowptr[a.B]) / a.S);
  const int ch = spmm_chunk_of(blockIdx.x, wave, kSpmmThreads / 64, a.nchunks, split);
  if (ch < 0) return;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ubase, 0, a.span, 0x00020000);
  const FlatSrc f{rs, rs, (uint32_t)lane * V * 4, 0, nullptr, 0, 0};
  CodeWindow win;
  win.wb = INT32_MIN / 2;
  win.cmask = 0;
  RowWindow rw;
  rw.base = INT32_MIN / 2;
  const int i = uni(a.chunk_row ? min(a.chunk_row[ch], a.n_rows)
                                : lower_bound_i32(a.rowptr, a.n_rows, ch * a.S));
  flat_chunk<V, G, false>(a, f, win, rw, ch, i, lane);
}

template <int V, int U>
__global__ void __launch_bounds__(kCodesThreads)
spmm_codes_kernel(SpmmArgs a, CodesSrc c) {
  __shared__ float cbs[kCodesLdsFloats];
  // stage the feature halves of every branch's codebook: cbs[(b*M + m)*D + k]
  const int nbm = c.nb * c.M;
  for (int t = threadIdx.x; t < nbm; t += kCodesThreads) {
    const int b = t / c.M, m = t - b * c.M;
    const float* src = c.emb + b * c.bstride + (int64_t)m * c.ldw + c.off;
    if (c.D == 4 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
      *reinterpret_cast<float4*>(cbs + 4 * t) = *reinterpret_cast<const float4*>(src);
    } else {
      for (int k = 0; k < c.D; ++k) cbs[t * c.D + k] = src[k];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  constexpr int WPB = kCodesThreads / 64;
  // this XCD's chunks: a contiguous 1/8 before the row-B split and a
  // contiguous 1/8 after it (as spmm_chunk_of), strided over its waves
  int split = a.nchunks;
  if (a.B < a.n_rows) split = min(a.nchunks, uni(a.rowptr[a.B]) / a.S);
  const int xcd = blockIdx.x % kNumXcd;
  const int lw = (blockIdx.x / kNumXcd) * WPB + wave;
  const int nwx = (gridDim.x / kNumXcd) * WPB;
  const int c2 = a.nchunks - split;
  const int a1 = xcd * split / kNumXcd, n1 = (xcd + 1) * split / kNumXcd - a1;
  const int a2 = split + xcd * c2 / kNumXcd, n2 = split + (xcd + 1) * c2 / kNumXcd - a2;
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.X, 0, a.span, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc =
      __builtin_amdgcn_make_buffer_rsrc((void*)c.lcodes, 0, c.lcspan, 0x00020000);
  const int col0 = lane * V;                 // first column of this lane
  const int br = col0 / c.D;                 // its branch (V divides D)
  CodeWindow win;
  win.wb = INT32_MIN / 2;
  win.cmask = 0;
  RowWindow rw;
  rw.base = INT32_MIN / 2;
  const FlatSrc f{rsx, rsc, (uint32_t)lane * V * 4, (uint32_t)br * 2,
                  cbs + (int64_t)br * c.M * c.D + (col0 - br * c.D), (uint32_t)c.D, c.ldlcb};
  for (int t = lw; t < n1 + n2; t += nwx) {
    const int ch = t < n1 ? a1 + t : a2 + (t - n1);
    const int i = uni(a.chunk_row ? min(a.chunk_row[ch], a.n_rows)
                                  : lower_bound_i32(a.rowptr, a.n_rows, ch * a.S));
    flat_chunk<V, U, true>(a, f, win, rw, ch, i, lane);
  }
}

// Each wave walks K consecutive chunks (its edge window and row cursor carry
// over; only the first chunk needs the row search).
template <int V, int U, bool FAR, bool PAIR>
__global__ void __launch_bounds__(kSpmmThreads)
spmm_wave_kernel(SpmmArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const bool stp = (a.dbg & 4) != 0;
  unsigned long long t0 = stp ? stamp() : 0ull;
  const int K = a.kpw;
  const int nsuper = (a.nchunks + K - 1) / K;
  int split = nsuper;
  if (a.B < a.n_rows) split = min(nsuper, uni(a.rowptr[a.B]) / (a.S * K));
  const int sc = spmm_chunk_of(blockIdx.x, wave, kSpmmThreads / 64, nsuper, split);
  if (sc < 0) return;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ubase, 0, a.span, 0x00020000);
  EdgeWindow<FAR> win;
  win.wb = INT32_MIN / 2;
  RowWindow rw;
  rw.base = INT32_MIN / 2;
  const int c0 = sc * K, c1 = min(a.nchunks, c0 + K);
  // a plan built over more rows than n_rows (the backward's row-restricted
  // transpose) clamps to the restricted search's answer (rowptr is monotone)
  int i = uni(a.chunk_row ? min(a.chunk_row[c0], a.n_rows)
                          : lower_bound_i32(a.rowptr, a.n_rows, c0 * a.S));
  unsigned long long t1 = stp ? stamp() : 0ull;
  for (int c = c0; c < c1; ++c)
    i = uni(wave_chunk<V, U, FAR, PAIR>(a, rs, win, rw, c, i, lane));
  if (stp) {
    const unsigned long long t2 = stamp();
    if (lane == 0) {
      unsigned long long* o = a.stamps + (int64_t)sc * 4;
      o[0] = t0;
      o[1] = t1;
      o[2] = t2;
      o[3] = (unsigned long long)(c1 - c0);
    }
  }
}

// For every row that spans chunks, the chunk where it ends adds the partials:
// carry_last[start chunk] + carry_first[start+1 .. end] (chunk order).
// One wave scans 64 chunks and serves the few that end a spanning row.
__global__ void __launch_bounds__(256)
spmm_fixup_kernel(SpmmArgs a) {
  // rows longer than L: out[row] = carry1[gs] + carry0[gs+1] + ... + carry0[ch]
  // (chunk order).  A wave finds the rows that end in its 64 chunks, then
  // sums R of them at once (R = 64 / the column group, 2 at F = 128), with the
  // carry loads of up to 8 chunks in flight ahead of the in-order adds.
  const int lane = threadIdx.x & 63;
  const int chunk = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 + lane;
  bool need = false;
  int r = -1;
  if (chunk < a.nchunks) {
    r = a.carry_row[chunk];
    if (r >= 0) {
      const int e1 = min(chunk * a.S + a.S, a.nnz);
      need = a.rowptr[r + 1] <= e1;
    }
  }
  unsigned long long mask = __ballot(need);
  const int F4 = a.F4;
  int cw = 1;                                  // lanes per row: pow2 >= F4, <= 64
  while (cw < F4 && cw < 64) cw <<= 1;
  const int R = 64 / cw;
  const int h = lane / cw, c0 = lane % cw;
  const float4* carry4 = reinterpret_cast<const float4*>(a.carry);
  float4* out4 = reinterpret_cast<float4*>(a.out);
  auto add4 = [](float4 s, float4 t) {
    s.x = __fadd_rn(s.x, t.x);
    s.y = __fadd_rn(s.y, t.y);
    s.z = __fadd_rn(s.z, t.z);
    s.w = __fadd_rn(s.w, t.w);
    return s;
  };
  while (mask) {
    // the h-th of the next R set bits
    unsigned long long m = mask;
    int src = -1;
    for (int i = 0; i < R && m; ++i) {
      const int b = __ffsll((long long)m) - 1;
      m &= m - 1;
      if (i == h) src = b;
    }
    mask = m;
    const int ch = __shfl(chunk, src < 0 ? 0 : src);
    const int row = __shfl(r, src < 0 ? 0 : src);
    if (src < 0) continue;
    const int gs = a.rowptr[row] / a.S;
    for (int cc = c0; cc < F4; cc += cw) {
      float4 s = carry4[((int64_t)gs * 2 + 1) * F4 + cc];
      int g = gs + 1;
      for (; g + 8 <= ch + 1; g += 8) {
        float4 t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = carry4[(int64_t)(g + u) * 2 * F4 + cc];
#pragma unroll
        for (int u = 0; u < 8; ++u) s = add4(s, t[u]);
      }
      for (; g <= ch; ++g) s = add4(s, carry4[(int64_t)g * 2 * F4 + cc]);
      out4[(int64_t)row * a.ldo4 + cc] = s;
    }
  }
}

__global__ void zero_rows_kernel(float* out, int64_t ldo, int n_rows, int F) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n_rows * F) return;
  out[(i / F) * ldo + (i % F)] = 0.f;
}

// x_first_order[j][b*D + k] = emb_out[b][codes[subset[B + j]][b]][off + k]
// (models.py:168-173; off = 0 feature half, off = D grad half), and optionally
// lcodes[j][b] = the code.  Thread per (node, branch); D == 4 stores float4.
__global__ void gather_codewords_kernel(const int64_t* __restrict__ subset, int B, int nprime,
                                        const int16_t* __restrict__ codes, int64_t ldc, int nb,
                                        int D, const float* __restrict__ emb, int ldw,
                                        int64_t bstride, int off, float* __restrict__ xt,
                                        int64_t ldt, int16_t* __restrict__ lcodes) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nprime * nb) return;
  const int64_t j = t / nb;
  const int b = (int)(t % nb);
  const int code = codes[subset[B + j] * ldc + b];
  if (lcodes) lcodes[t] = (int16_t)code;
  if (!xt) return;
  const float* src = emb + b * bstride + (int64_t)code * ldw + off;
  float* dst = xt + j * ldt + (int64_t)b * D;
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

static unsigned long long* g_stamps = nullptr;   // debug only (VQGNN_SPMM_DEBUG & 4)
static size_t g_stamp_cap = 0;
static int64_t g_stamp_n = 0;

static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
static int spmm_chunk_edges(int F4) {
  static const int s_env = env_int("VQGNN_SPMM_S", 0);
  if (s_env > 0) return s_env;
  return F4 > 32 ? 32 : 64;
}
static int spmm_long_row(int S) {
  static const int l_env = env_int("VQGNN_SPMM_L", 0);
  return l_env > 0 ? l_env : 4 * S;
}

}  // namespace vqgnn

using namespace vqgnn;

extern "C" size_t vqgnn_spmm_workspace(int32_t n_rows, int64_t nnz, int32_t F) {
  (void)n_rows;
  if (nnz <= 0 || F <= 0) return 256;
  const int S = spmm_chunk_edges((F + 3) / 4);
  const int64_t nchunks = (nnz + S - 1) / S;
  return align_up((size_t)nchunks * 2 * F * sizeof(float), 256) +
         2 * align_up((size_t)nchunks * sizeof(int), 256);
}

template <int G, int NCH, bool TWO>
static void launch_spmm(const SpmmArgs& a, hipStream_t s) {
  constexpr int GPW = kSpmmThreads / G;
  // per XCD at most ceil(c1/8) + ceil(c2/8) <= ceil(nchunks/8) + 1 chunks
  const int per_xcd = (a.nchunks + kNumXcd - 1) / kNumXcd + 1;
  const int grid = kNumXcd * ((per_xcd + GPW - 1) / GPW);
  hipLaunchKernelGGL((spmm_merge_kernel<G, NCH, TWO>), dim3(grid), dim3(kSpmmThreads), 0, s, a);
  hipLaunchKernelGGL(spmm_fixup_kernel, dim3((a.nchunks + 255) / 256), dim3(256), 0, s, a);
}

template <int V, int U, bool FAR, bool PAIR = false>
static void launch_spmm_wave(SpmmArgs& a, hipStream_t s) {
  constexpr int WPB = kSpmmThreads / 64;
  static const int kpw = env_int("VQGNN_SPMM_K", 1);
  a.kpw = kpw < 1 ? 1 : kpw;
  const int nsuper = (a.nchunks + a.kpw - 1) / a.kpw;
  static const int plan = env_int("VQGNN_SPMM_PLAN", 1);
  if (!a.chunk_row && plan) {
    int* cr = a.carry_row + align_up((size_t)a.nchunks * sizeof(int), 256) / sizeof(int);
    hipLaunchKernelGGL(spmm_chunk_rows_kernel, dim3((a.nchunks + 255) / 256), dim3(256), 0, s,
                       a.rowptr, a.n_rows, a.S, a.nchunks, cr);
    a.chunk_row = cr;
  }
  const int per_xcd = (nsuper + kNumXcd - 1) / kNumXcd + 1;
  const int grid = kNumXcd * ((per_xcd + WPB - 1) / WPB);
  hipLaunchKernelGGL((spmm_wave_kernel<V, U, FAR, PAIR>), dim3(grid), dim3(kSpmmThreads), 0, s, a);
  hipLaunchKernelGGL(spmm_fixup_kernel, dim3((a.nchunks + 255) / 256), dim3(256), 0, s, a);
}

// flat kernel group size (0 = off)
static int spmm_flat() {
  static const int g = env_int("VQGNN_SPMM_FLAT", 0);
  return g;
}

template <int V>
static void launch_spmm_flat(SpmmArgs& a, hipStream_t s) {
  constexpr int WPB = kSpmmThreads / 64;
  if (!a.chunk_row) {
    int* cr = a.carry_row + align_up((size_t)a.nchunks * sizeof(int), 256) / sizeof(int);
    hipLaunchKernelGGL(spmm_chunk_rows_kernel, dim3((a.nchunks + 255) / 256), dim3(256), 0, s,
                       a.rowptr, a.n_rows, a.S, a.nchunks, cr);
    a.chunk_row = cr;
  }
  const int per_xcd = (a.nchunks + kNumXcd - 1) / kNumXcd + 1;
  const int grid = kNumXcd * ((per_xcd + WPB - 1) / WPB);
  if (spmm_flat() == 8)
    hipLaunchKernelGGL((spmm_flat_kernel<V, 8>), dim3(grid), dim3(kSpmmThreads), 0, s, a);
  else if (spmm_flat() == 32)
    hipLaunchKernelGGL((spmm_flat_kernel<V, 32>), dim3(grid), dim3(kSpmmThreads), 0, s, a);
  else
    hipLaunchKernelGGL((spmm_flat_kernel<V, 16>), dim3(grid), dim3(kSpmmThreads), 0, s, a);
  hipLaunchKernelGGL(spmm_fixup_kernel, dim3((a.nchunks + 255) / 256), dim3(256), 0, s, a);
}

// 0 = automatic (wave kernel where it applies), 1 = lane-group kernel only,
// 2 = wave kernel with 64-bit row addresses (FAR) even when the range fits
static int spmm_mode() {
  static const int m = env_int("VQGNN_SPMM_MODE", 0);
  return m;
}

// X rows [0, rows_x) and X2 rows [0, rows_x2) as one byte range of < 4 GiB
static bool wave_layout(SpmmArgs& a, int64_t rows_x, int64_t rows_x2) {
  const uint64_t x0 = (uint64_t)(uintptr_t)a.X;
  const uint64_t x1 = x0 + (uint64_t)rows_x * (uint64_t)a.ldx4 * 16;
  uint64_t lo = x0, hi = x1, y0 = x0;
  if (a.X2 && rows_x2 > 0) {
    y0 = (uint64_t)(uintptr_t)a.X2;
    const uint64_t y1 = y0 + (uint64_t)rows_x2 * (uint64_t)a.ldx24 * 16;
    lo = y0 < lo ? y0 : lo;
    hi = y1 > hi ? y1 : hi;
  }
  if (hi - lo >= 0xFFFFFFFFull || (uint64_t)a.ldx4 * 16 > 0xFFFFFFFFull ||
      (uint64_t)a.ldx24 * 16 > 0xFFFFFFFFull)
    return false;
  a.ubase = reinterpret_cast<const char*>((uintptr_t)lo);
  a.span = (uint32_t)(hi - lo);
  a.offx = (uint32_t)(x0 - lo);
  a.ldxb = (uint32_t)(a.ldx4 * 16);
  a.offx2 = (uint32_t)(y0 - lo);
  a.ldx2b = (uint32_t)(a.ldx24 * 16);
  return true;
}

template <bool TWO>
static int dispatch_spmm(SpmmArgs& a, int64_t rows_x, int64_t rows_x2, hipStream_t s) {
  const int F = a.F4 * 4;
  const bool al = (((uintptr_t)a.out | (uintptr_t)a.carry | (uintptr_t)(a.ldo4 * 16)) & 15) == 0;
  if (spmm_mode() != 1 && al && (F == 64 || F == 128 || F == 256)) {
    // one 32-bit buffer range over X and X2 when they are within 4 GiB of
    // each other (the usual case); else 64-bit row addresses (FAR)
    const bool near = spmm_mode() != 2 && wave_layout(a, rows_x, rows_x2);
    if (!near) {
      a.ubase = nullptr;
      a.span = 0;
    }
    static const int pair = env_int("VQGNN_SPMM_PAIR", 0);
    static const int pu = env_int("VQGNN_SPMM_U", 8);
    if (F == 128 && pair && pu == 16) {
      if (near) launch_spmm_wave<4, 16, false, true>(a, s);
      else launch_spmm_wave<4, 16, true, true>(a, s);
    } else if (F == 128 && pair) {
      if (near) launch_spmm_wave<4, 8, false, true>(a, s);
      else launch_spmm_wave<4, 8, true, true>(a, s);
    } else if (F == 128 && near && spmm_flat() > 0) {
      launch_spmm_flat<2>(a, s);
    } else if (F == 128) {
      if (near) launch_spmm_wave<2, 8, false>(a, s); else launch_spmm_wave<2, 8, true>(a, s);
    } else if (F == 256) {
      if (near) launch_spmm_wave<4, 4, false>(a, s); else launch_spmm_wave<4, 4, true>(a, s);
    } else {
      if (near) launch_spmm_wave<1, 8, false>(a, s); else launch_spmm_wave<1, 8, true>(a, s);
    }
    return check_launch("spmm");
  }
  const int F4 = a.F4;
  if (F4 <= 16) launch_spmm<16, 1, TWO>(a, s);
  else if (F4 <= 32) launch_spmm<32, 1, TWO>(a, s);
  else if (F4 <= 64) launch_spmm<64, 1, TWO>(a, s);
  else if (F4 <= 128) launch_spmm<64, 2, TWO>(a, s);
  else if (F4 <= 192) launch_spmm<64, 3, TWO>(a, s);
  else if (F4 <= 256) launch_spmm<64, 4, TWO>(a, s);
  else if (F4 <= 512) launch_spmm<64, 8, TWO>(a, s);
  else {
    set_error("spmm: F=%d > 2048 not implemented", F4 * 4);
    return VQGNN_ERR_UNSUPPORTED;
  }
  return check_launch("spmm");
}

extern "C" int64_t vqgnn_spmm_plan_size(int64_t nnz, int32_t F) {
  if (nnz <= 0 || F <= 0) return 0;
  const int S = spmm_chunk_edges((F + 3) / 4);
  return (nnz + S - 1) / S;
}

extern "C" int vqgnn_spmm_plan(const int32_t* rowptr, int32_t n_rows, int64_t nnz, int32_t F,
                               int32_t* plan, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(n_rows >= 0 && nnz >= 0 && nnz < (int64_t)INT32_MAX && F > 0,
                "spmm_plan: bad shape");
  const int64_t nchunks = vqgnn_spmm_plan_size(nnz, F);
  if (nchunks == 0) return VQGNN_OK;
  VQGNN_REQUIRE(rowptr && plan, "spmm_plan: null pointer");
  const int S = spmm_chunk_edges((F + 3) / 4);
  hipLaunchKernelGGL(spmm_chunk_rows_kernel, dim3((nchunks + 255) / 256), dim3(256), 0,
                     as_stream(stream), rowptr, n_rows, S, (int)nchunks, plan);
  return check_launch("spmm_plan");
}

extern "C" int vqgnn_spmm(const int32_t* rowptr, const int32_t* col, const float* val,
                          int32_t n_rows, int32_t n_cols, int64_t nnz, int32_t B,
                          const float* X, int64_t ldx,
                          const float* X2, int64_t ldx2, int32_t F, float* out, int64_t ldo,
                          const int32_t* plan, void* workspace, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(rowptr && out && n_rows >= 0, "spmm: null pointer");
  VQGNN_REQUIRE(F > 0 && F % 4 == 0, "spmm: F=%d must be a positive multiple of 4", F);
  VQGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= F && ldo >= F,
                "spmm: ldx/ldo must be multiples of 4 and >= F");
  VQGNN_REQUIRE(!X2 || (ldx2 % 4 == 0 && ldx2 >= F && ((uintptr_t)X2 & 15) == 0),
                "spmm: X2 must be 16-byte aligned with ldx2 a multiple of 4, >= F");
  VQGNN_REQUIRE(((uintptr_t)X & 15) == 0 && ((uintptr_t)out & 15) == 0,
                "spmm: X/out must be 16-byte aligned");
  VQGNN_REQUIRE(nnz < (int64_t)INT32_MAX, "spmm: nnz >= 2^31");
  VQGNN_REQUIRE(n_cols >= 0 && (!X2 || (B >= 0 && B <= n_cols)),
                "spmm: need 0 <= B <= n_cols with X2 (n_cols=%d B=%d)", n_cols, B);
  hipStream_t s = as_stream(stream);
  if (n_rows == 0) return VQGNN_OK;
  if (nnz == 0) {
    const int64_t tot = (int64_t)n_rows * F;
    hipLaunchKernelGGL(zero_rows_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, out, ldo,
                       n_rows, F);
    return check_launch("spmm(zero)");
  }
  VQGNN_REQUIRE(col && val && X && workspace, "spmm: null pointer");
  SpmmArgs a;
  a.rowptr = rowptr;
  a.col = col;
  a.val = val;
  a.n_rows = n_rows;
  a.nnz = (int)nnz;
  a.F4 = F / 4;
  a.S = spmm_chunk_edges(a.F4);
  a.L = spmm_long_row(a.S);
  a.nchunks = (int)((nnz + a.S - 1) / a.S);
  a.B = X2 ? B : INT32_MAX;
  a.X = X;
  a.ldx4 = ldx / 4;
  a.X2 = X2;
  a.ldx24 = X2 ? ldx2 / 4 : 0;
  a.out = out;
  a.ldo4 = ldo / 4;
  a.carry = reinterpret_cast<float*>(workspace);
  a.carry_row = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) +
                                       align_up((size_t)a.nchunks * 2 * F * sizeof(float), 256));
  a.kpw = 1;
  a.chunk_row = plan;
  a.dbg = env_int("VQGNN_SPMM_DEBUG", 0);
  a.stamps = nullptr;
  if (a.dbg & 4) {
    const size_t need = (size_t)a.nchunks * 4 * sizeof(unsigned long long);
    if (need > g_stamp_cap) {
      if (g_stamps) (void)hipFree(g_stamps);
      (void)hipMalloc(&g_stamps, need);
      g_stamp_cap = need;
    }
    g_stamp_n = (int64_t)a.nchunks * 4;
    a.stamps = g_stamps;
  }
  a.ubase = nullptr;
  a.span = a.offx = a.ldxb = a.offx2 = a.ldx2b = 0;
  return X2 ? dispatch_spmm<true>(a, B, (int64_t)n_cols - B, s)
            : dispatch_spmm<false>(a, n_cols, 0, s);
}

extern "C" int vqgnn_spmm_codes_supported(int32_t F, int32_t nb, int32_t M, int32_t D) {
  if (F != 64 && F != 128 && F != 256) return 0;
  const int V = F / 64;
  if (D <= 0 || nb <= 0 || M <= 0 || nb * D != F || D % V != 0) return 0;
  return (int64_t)nb * M * D <= kCodesLdsFloats ? 1 : 0;
}

extern "C" int vqgnn_spmm_codes(const int32_t* rowptr, const int32_t* col, const float* val,
                                int32_t n_rows, int32_t n_cols, int64_t nnz, int32_t B,
                                const float* X, int64_t ldx, const int16_t* lcodes,
                                int64_t ldlc, int32_t nb, const float* emb, int32_t M, int32_t D,
                                int32_t ldw, int64_t emb_bstride, int32_t col_offset, int32_t F,
                                float* out, int64_t ldo, const int32_t* plan, void* workspace,
                                vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(rowptr && out && n_rows >= 0, "spmm_codes: null pointer");
  if (!vqgnn_spmm_codes_supported(F, nb, M, D)) {
    set_error("spmm_codes: F=%d nb=%d M=%d D=%d outside the LDS codebook path", F, nb, M, D);
    return VQGNN_ERR_UNSUPPORTED;
  }
  VQGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= F && ldo >= F,
                "spmm_codes: ldx/ldo must be multiples of 4 and >= F");
  VQGNN_REQUIRE(((uintptr_t)X & 15) == 0 && ((uintptr_t)out & 15) == 0,
                "spmm_codes: X/out must be 16-byte aligned");
  VQGNN_REQUIRE(nnz < (int64_t)INT32_MAX, "spmm_codes: nnz >= 2^31");
  VQGNN_REQUIRE(B >= 0 && B <= n_cols && ldlc >= nb, "spmm_codes: need 0 <= B <= n_cols, ldlc >= nb");
  VQGNN_REQUIRE(col_offset >= 0 && col_offset + D <= ldw, "spmm_codes: bad codebook layout");
  VQGNN_REQUIRE((uint64_t)B * (uint64_t)ldx * 4 < 0xFFFFFFFFull &&
                (uint64_t)(n_cols - B) * (uint64_t)ldlc * 2 < 0xFFFFFFFFull,
                "spmm_codes: X or lcodes spans 4 GiB");
  hipStream_t s = as_stream(stream);
  if (n_rows == 0) return VQGNN_OK;
  if (nnz == 0) {
    const int64_t tot = (int64_t)n_rows * F;
    hipLaunchKernelGGL(zero_rows_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, out, ldo,
                       n_rows, F);
    return check_launch("spmm_codes(zero)");
  }
  VQGNN_REQUIRE(col && val && (X || B == 0) && emb && workspace && (lcodes || B == n_cols),
                "spmm_codes: null pointer");
  SpmmArgs a;
  memset(&a, 0, sizeof(a));
  a.rowptr = rowptr;
  a.col = col;
  a.val = val;
  a.n_rows = n_rows;
  a.nnz = (int)nnz;
  a.F4 = F / 4;
  a.S = spmm_chunk_edges(a.F4);
  a.L = spmm_long_row(a.S);
  a.nchunks = (int)((nnz + a.S - 1) / a.S);
  a.B = B;
  a.X = X;
  a.ldx4 = ldx / 4;
  a.out = out;
  a.ldo4 = ldo / 4;
  a.carry = reinterpret_cast<float*>(workspace);
  a.carry_row = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) +
                                       align_up((size_t)a.nchunks * 2 * F * sizeof(float), 256));
  a.kpw = 1;
  a.chunk_row = plan;
  a.dbg = env_int("VQGNN_SPMM_DEBUG", 0) & 2;
  a.span = (uint32_t)((uint64_t)B * ldx * 4);
  a.ldxb = (uint32_t)(ldx * 4);
  CodesSrc c;
  c.lcodes = lcodes;
  c.ldlcb = (uint32_t)(ldlc * 2);
  c.lcspan = (uint32_t)((uint64_t)(n_cols - B) * ldlc * 2);
  c.emb = emb;
  c.bstride = emb_bstride;
  c.ldw = ldw;
  c.off = col_offset;
  c.M = M;
  c.D = D;
  c.nb = nb;
  if (!plan) {
    int* cr = a.carry_row + align_up((size_t)a.nchunks * sizeof(int), 256) / sizeof(int);
    hipLaunchKernelGGL(spmm_chunk_rows_kernel, dim3((a.nchunks + 255) / 256), dim3(256), 0, s,
                       a.rowptr, a.n_rows, a.S, a.nchunks, cr);
    a.chunk_row = cr;
  }
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  static const int per_cu = env_int("VQGNN_SPMM_CODES_WG", 1);
  const int grid = kNumXcd * ((ncu * (per_cu < 1 ? 1 : per_cu) + kNumXcd - 1) / kNumXcd);
  static const int uc = env_int("VQGNN_SPMM_CODES_G", 16);
  if (F == 128) {
    if (uc == 8) hipLaunchKernelGGL((spmm_codes_kernel<2, 8>), dim3(grid), dim3(kCodesThreads), 0, s, a, c);
    else hipLaunchKernelGGL((spmm_codes_kernel<2, 16>), dim3(grid), dim3(kCodesThreads), 0, s, a, c);
  } else if (F == 256) {
    hipLaunchKernelGGL((spmm_codes_kernel<4, 8>), dim3(grid), dim3(kCodesThreads), 0, s, a, c);
  } else {
    hipLaunchKernelGGL((spmm_codes_kernel<1, 32>), dim3(grid), dim3(kCodesThreads), 0, s, a, c);
  }
  int rc = check_launch("spmm_codes");
  if (rc) return rc;
  hipLaunchKernelGGL(spmm_fixup_kernel, dim3((a.nchunks + 255) / 256), dim3(256), 0, s, a);
  return check_launch("spmm_codes(fixup)");
}

extern "C" int vqgnn_gather_codewords(const int64_t* subset, int32_t B, int32_t n,
                                      const int16_t* codes, int64_t ldc, int32_t nb, int32_t D,
                                      const float* emb_out, int32_t ldw, int64_t emb_bstride,
                                      int32_t col_offset, float* xt, int64_t ldt,
                                      int16_t* lcodes, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(n >= B && B >= 0 && nb > 0 && ldc >= nb && D > 0, "gather_codewords: bad shape");
  const int64_t tot = (int64_t)(n - B) * nb;
  if (tot == 0) return VQGNN_OK;
  VQGNN_REQUIRE(subset && codes && (xt || lcodes), "gather_codewords: null pointer");
  VQGNN_REQUIRE(!xt || (emb_out && ldt >= (int64_t)nb * D && col_offset >= 0 &&
                        col_offset + D <= ldw),
                "gather_codewords: bad codebook / output layout");
  hipLaunchKernelGGL(gather_codewords_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     as_stream(stream), subset, B, n - B, codes, ldc, nb, D, emb_out, ldw,
                     emb_bstride, col_offset, xt, ldt, lcodes);
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

// debug: copy the stamp buffer of the last spmm launch (dbg & 4) to host;
// returns the number of entries ([chunk-groups][t0, t1, t2, nchunks])
extern "C" int64_t vqgnn_debug_spmm_stamps(unsigned long long* host, int64_t n) {
  if (!g_stamps || n <= 0) return g_stamp_n;
  const int64_t m = n < g_stamp_n ? n : g_stamp_n;
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(host, g_stamps, (size_t)m * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  return m;
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

// ===========================================================================
// Segment-pair SpMM (F = 128).  Same row semantics and bits as vqgnn_spmm:
// a row of at most L edges is summed whole from 0 in CSR order with separate
// mul and add; a longer row is cut at the global S-aligned chunk boundaries
// (the pieces spmm_wave_kernel leaves as carries) and its pieces are added in
// order by spmm_pair_fixup_kernel (first piece as the initial value, as
// spmm_fixup_kernel does) — so the output is bit-identical to vqgnn_spmm.
//
// Why: the gather of a 512-B row per wave-instruction (dwordx2 per lane) runs
// at ~35 G rows/s from L2, dwordx4 with two rows per instruction at ~62 G
// rows/s (scripts/probes/gather_shape.hip on MI355X); the per-instruction cost
// dominates.  Here each half-wave owns one segment (a row, or a piece of a
// long row): one buffer_load_dwordx4 fetches edge k of both halves' segments.
// The two segments of a pair have (nearly) equal lengths because the plan
// sorts segments by length inside row windows, so the halves rarely idle.
// Per half-wave step: the edge's input-row offset and weight come from a
// staged 32-edge window by ds_bpermute (LDS crossbar, no VALU), one v_add for
// the lane's column offset, then 2 v_pk_mul + 2 v_pk_add.
//
// Plan (built once per batch and F, on the device, vqgnn_spmm_pair_plan):
//   hdr[16]      : [0] segments, [1] long rows, [2..10] xcd_begin[0..8]
//   segs[cap]    : int4 {first edge, length, dst, 0}; dst >= 0: output row;
//                  dst <= -2: carry slot -dst-2 (a piece of a long row)
//   longrows[lc] : int4 {row, first slot, pieces, 0}
// Segment order: key = (xcd, row window of 2048 rows, -length).  XCD x gets an
// edge-balanced contiguous range of the batch rows (< B) and one of the
// out-of-batch rows, as spmm_wave_kernel's chunk placement does, so the
// gathers of an XCD stay cluster-local in its L2; length-sorting only inside
// 2048-row windows keeps that locality (LRU simulation of the arxiv batch:
// 64.9% L2 hits against 64.5% in CSR order, 56% for a global length sort).
// ===========================================================================

namespace vqgnn {

constexpr int kPairHdr = 16;
constexpr int kPairWinShift = 11;   // row windows of 2048 rows

static inline int64_t pair_seg_cap(int32_t n_rows, int64_t nnz, int S, int L) {
  return (int64_t)n_rows + nnz / S + nnz / (L > 0 ? L : 1) + 16;
}
static inline int64_t pair_long_cap(int64_t nnz, int L) { return nnz / (L > 0 ? L : 1) + 1; }

// per row: segments and carry slots it needs
__global__ void pair_count_kernel(const int32_t* __restrict__ rowptr, int n_rows, int S, int L,
                                  int32_t* __restrict__ nseg, int32_t* __restrict__ nslot) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int rs = rowptr[r], re = rowptr[r + 1];
  const int len = re - rs;
  if (len <= L) {
    nseg[r] = 1;
    nslot[r] = 0;
  } else {
    const int np = (re - 1) / S - rs / S + 1;
    nseg[r] = np;
    nslot[r] = np;
  }
}

__device__ __forceinline__ uint32_t pair_key(int xcd, int r, int len) {
  const uint32_t win = min((uint32_t)r >> kPairWinShift, (1u << 19) - 1);
  return ((uint32_t)xcd << 28) | (win << 9) | (uint32_t)(511 - min(len, 511));
}

// per row: its segment records (unsorted), sort keys, long-row entries
__global__ void pair_fill_kernel(const int32_t* __restrict__ rowptr, int n_rows, int B, int S,
                                 int L, const int32_t* __restrict__ seg_off,
                                 const int32_t* __restrict__ slot_off, int4* __restrict__ useg,
                                 uint32_t* __restrict__ keys, int4* __restrict__ longrows,
                                 int32_t* __restrict__ nlong) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int rs = rowptr[r], re = rowptr[r + 1];
  const int len = re - rs;
  // edge-balanced XCD ranges: batch rows and out-of-batch rows separately
  const int64_t eb = rowptr[B], en = rowptr[n_rows];
  int xcd;
  if (r < B) xcd = eb > 0 ? (int)((int64_t)rs * kNumXcd / eb) : 0;
  else xcd = en > eb ? (int)((int64_t)(rs - eb) * kNumXcd / (en - eb)) : 0;
  xcd = min(max(xcd, 0), kNumXcd - 1);
  const int p0 = seg_off[r];
  if (len <= L) {
    useg[p0] = make_int4(rs, len, r, 0);
    keys[p0] = pair_key(xcd, r, len);
    return;
  }
  const int np = (re - 1) / S - rs / S + 1;
  const int sb = slot_off[r];
  const int li = atomicAdd(nlong, 1);
  longrows[li] = make_int4(r, sb, np, 0);
  for (int i = 0; i < np; ++i) {
    const int a = i == 0 ? rs : (rs / S + i) * S;
    const int b = min(re, (rs / S + i + 1) * S);
    useg[p0 + i] = make_int4(a, b - a, -(sb + i) - 2, 0);
    keys[p0 + i] = pair_key(xcd, r, b - a);
  }
}

__global__ void pair_pad_kernel(uint32_t* __restrict__ keys, uint32_t* __restrict__ iota,
                                const int32_t* __restrict__ seg_off,
                                const int32_t* __restrict__ nseg, int n_rows, int64_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const int64_t total = n_rows > 0 ? (int64_t)seg_off[n_rows - 1] + nseg[n_rows - 1] : 0;
  if (i >= total) keys[i] = 0xFFFFFFFFu;
  iota[i] = (uint32_t)i;
}

__global__ void pair_gather_kernel(const int4* __restrict__ useg, const uint32_t* __restrict__ idx,
                                   const uint32_t* __restrict__ skeys, int4* __restrict__ segs,
                                   int64_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  segs[i] = skeys[i] == 0xFFFFFFFFu ? make_int4(0, 0, -1, 0) : useg[idx[i]];
}

// hdr: segment count, long-row count, xcd_begin[0..8] (binary search on the
// sorted keys)
__global__ void pair_hdr_kernel(const uint32_t* __restrict__ skeys, int64_t cap,
                                const int32_t* __restrict__ nlong, int32_t* __restrict__ hdr) {
  const int t = threadIdx.x;
  if (t <= kNumXcd) {
    int64_t lo = 0, hi = cap;
    const uint32_t k = (uint32_t)t << 28;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (skeys[mid] < k) lo = mid + 1; else hi = mid;
    }
    hdr[2 + t] = (int32_t)lo;
    if (t == kNumXcd) hdr[0] = (int32_t)lo;
  }
  if (t == 0) hdr[1] = *nlong;
}

struct PairArgs {
  const int32_t* col;
  const float* val;
  const int4* segs;
  const int32_t* hdr;
  const int4* longrows;
  const char* ubase;
  uint32_t span, offx, ldxb, offx2, ldx2b;
  int B;
  float* out;
  int64_t ldo;   // floats
  float* carry;  // [slots][128]
  int dbg;       // experiments: 1 = no gathers, 2 = no stores, 8 = no adds
};

constexpr int kPairG = 8;   // steps (edges per half) whose loads are in flight together

// Window of a half's next 32 edges: lane c of the half holds edge k0 + c as
// (input-row byte offset, weight).  Edges past the segment get the offset
// `span` (outside the buffer range: the load returns 0) and weight 0, so a
// masked step adds +0 — a no-op on the accumulator, which is never -0 (it
// starts at +0 and round-to-nearest sums give -0 only from two -0s) — and
// no step needs a guard.
struct PairWin {
  uint32_t o;
  float w;
};

__device__ __forceinline__ PairWin pair_window(const PairArgs& a, int start, int len, int k0,
                                               int c) {
  const int kk = k0 + c;
  PairWin r{a.span, 0.f};
  if (kk < len) {
    const int j = a.col[start + kk];
    r.w = a.val[start + kk];
    r.o = j < a.B ? a.offx + (uint32_t)j * a.ldxb : a.offx2 + (uint32_t)(j - a.B) * a.ldx2b;
  }
  return r;
}

// issue the gathers of steps kw .. kw+G-1 of the window (kw = 0 or 16): the
// row offset by ds_bpermute from the half's window lane (immediate offset),
// one v_add for this lane's column bytes, one dwordx4 load for both halves
// Broadcast lane K of each 32-lane half to the whole half: ds_swizzle in
// bitmask mode (and 0, or K): no address operand, unlike ds_bpermute
template <int K>
__device__ __forceinline__ int half_bcast(int v) {
  return __builtin_amdgcn_ds_swizzle(v, K << 5);
}

template <int DBG, int KW>
__device__ __forceinline__ void pair_issue_k(const __amdgpu_buffer_rsrc_t& rs, const PairWin& win,
                                             uint32_t lo, float4* x, float* w) {
  auto step = [&](auto uc) {
    constexpr int u = decltype(uc)::value;
    const uint32_t o = (uint32_t)half_bcast<KW + u>((int)win.o);
    w[u] = __builtin_bit_cast(float, half_bcast<KW + u>(__builtin_bit_cast(int, win.w)));
    if constexpr (DBG & 1) {
      x[u] = make_float4(__builtin_bit_cast(float, o), 0.f, 0.f, 0.f);
    } else {
      x[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + lo, 0, 0));
    }
  };
  [&]<int... U>(std::integer_sequence<int, U...>) {
    (step(std::integral_constant<int, U>{}), ...);
  }(std::make_integer_sequence<int, kPairG>{});
}

// issue the gathers of steps k0 .. k0+G-1 (window slot (k0 & 31) / G)
template <int DBG = 0>
__device__ __forceinline__ void pair_issue(const __amdgpu_buffer_rsrc_t& rs, const PairWin& win,
                                           int k0, uint32_t lo, float4* x, float* w) {
  static_assert(kPairG == 8, "window slots assume 8-step groups");
  switch ((k0 >> 3) & 3) {
    case 0: pair_issue_k<DBG, 0>(rs, win, lo, x, w); break;
    case 1: pair_issue_k<DBG, 8>(rs, win, lo, x, w); break;
    case 2: pair_issue_k<DBG, 16>(rs, win, lo, x, w); break;
    default: pair_issue_k<DBG, 24>(rs, win, lo, x, w); break;
  }
}

// acc += w * x per column with separate IEEE mul and add (-ffp-contract=off),
// written as explicit 2-wide vectors: one v_pk_mul_f32 + one v_pk_add_f32 per
// column pair (left to the SLP vectoriser, the scalar form was re-paired
// across edges with v_mov shuffles)
typedef float pair_f2 __attribute__((ext_vector_type(2)));

template <int DBG = 0>
__device__ __forceinline__ void pair_add(const float4* x, const float* w, pair_f2& lo,
                                         pair_f2& hi) {
#pragma unroll
  for (int u = 0; u < kPairG; ++u) {
    if constexpr (DBG & 8) {
      asm volatile("" ::"v"(x[u].x), "v"(x[u].y), "v"(x[u].z), "v"(x[u].w), "v"(w[u]));
      continue;
    }
    const pair_f2 ww = {w[u], w[u]};
    const pair_f2 a = {x[u].x, x[u].y};
    const pair_f2 b = {x[u].z, x[u].w};
    lo = lo + ww * a;
    hi = hi + ww * b;
  }
}

__device__ __forceinline__ void pair_segs(const PairArgs& a, int sb, int se, int q, int4& s0,
                                          int4& s1) {
  const int i0 = sb + 2 * q;
  const int4 t0 = a.segs[i0];
  const int4 t1 = i0 + 1 < se ? a.segs[i0 + 1] : make_int4(0, 0, -1, 0);
  // wave-uniform records: keep them in SGPRs
  s0 = make_int4(__builtin_amdgcn_readfirstlane(t0.x), __builtin_amdgcn_readfirstlane(t0.y),
                 __builtin_amdgcn_readfirstlane(t0.z), 0);
  s1 = make_int4(__builtin_amdgcn_readfirstlane(t1.x), __builtin_amdgcn_readfirstlane(t1.y),
                 __builtin_amdgcn_readfirstlane(t1.z), 0);
}

// Waves of XCD x walk that XCD's pairs with a stride.  The next pair's
// window loads are issued behind the current pair's first gathers, and the
// segment records of the pair after that one pair earlier still (scalar
// loads).  (A software pipeline over 8-step groups — the next group's gathers
// issued before the current group's adds — measured 20% slower: 102 VGPRs,
// 4 waves/SIMD, against 64 VGPRs and 8 waves/SIMD here.)
template <int DBG>
__global__ void __launch_bounds__(kSpmmThreads)
spmm_pair_kernel(PairArgs a) {
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5;
  const int c = lane & 31;
  const int xcd = blockIdx.x % kNumXcd;
  const int wx = __builtin_amdgcn_readfirstlane((blockIdx.x / kNumXcd) * (kSpmmThreads / 64) +
                                                (threadIdx.x >> 6));
  const int nwx = (gridDim.x / kNumXcd) * (kSpmmThreads / 64);
  const int sb = __builtin_amdgcn_readfirstlane(a.hdr[2 + xcd]);
  const int se = __builtin_amdgcn_readfirstlane(a.hdr[3 + xcd]);
  const int npairs = (se - sb + 1) >> 1;
  if (wx >= npairs) return;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ubase, 0, a.span, 0x00020000);
  const uint32_t lo = (uint32_t)c * 16;
  int q = wx;
  int4 s0, s1, n0, n1;
  pair_segs(a, sb, se, q, s0, s1);
  PairWin win = pair_window(a, half ? s1.x : s0.x, half ? s1.y : s0.y, 0, c);
  if (q + nwx < npairs) pair_segs(a, sb, se, q + nwx, n0, n1);
  while (true) {
    const int qn = q + nwx;
    const int my_start = half ? s1.x : s0.x;
    const int my_len = half ? s1.y : s0.y;
    const int emax = max(s0.y, s1.y);
    pair_f2 alo = {0.f, 0.f}, ahi = {0.f, 0.f};
    float4 x[kPairG];
    float w[kPairG];
    if (emax > 0) pair_issue<DBG>(rs, win, 0, lo, x, w);
    // next pair: its window now, the one after's segment records
    PairWin nwin{a.span, 0.f};
    int4 m0 = make_int4(0, 0, -1, 0), m1 = m0;
    if (qn < npairs) {
      nwin = pair_window(a, half ? n1.x : n0.x, half ? n1.y : n0.y, 0, c);
      if (qn + nwx < npairs) pair_segs(a, sb, se, qn + nwx, m0, m1);
    }
    if (emax > 0) pair_add<DBG>(x, w, alo, ahi);
#pragma unroll 1
    for (int k0 = kPairG; k0 < emax; k0 += kPairG) {   // segments longer than kPairG
      if ((k0 & 31) == 0) win = pair_window(a, my_start, my_len, k0, c);
      pair_issue<DBG>(rs, win, k0, lo, x, w);
      pair_add<DBG>(x, w, alo, ahi);
    }
    const float4 acc = make_float4(alo.x, alo.y, ahi.x, ahi.y);
    const int d = half ? s1.z : s0.z;
    if (DBG & 2) {
      if (acc.x == 1234.5f) a.out[0] = acc.y;   // keep the sums alive
    } else if (d >= 0) {
      *reinterpret_cast<float4*>(a.out + (int64_t)d * a.ldo + c * 4) = acc;
    } else if (d <= -2) {
      *reinterpret_cast<float4*>(a.carry + (int64_t)(-d - 2) * 128 + c * 4) = acc;
    }
    if (qn >= npairs) break;
    q = qn;
    s0 = n0;
    s1 = n1;
    n0 = m0;
    n1 = m1;
    win = nwin;
  }
}

// long rows: out[row] = piece0 + piece1 + ... in order; one half-wave per row,
// up to 8 piece loads in flight ahead of the in-order adds
__global__ void __launch_bounds__(kSpmmThreads)
spmm_pair_fixup_kernel(PairArgs a) {
  const int lane = threadIdx.x & 63;
  const int c = lane & 31;
  const int nlong = a.hdr[1];
  const int nh = gridDim.x * (kSpmmThreads / 32);
  for (int h = blockIdx.x * (kSpmmThreads / 32) + (threadIdx.x >> 5); h < nlong; h += nh) {
    const int4 lr = a.longrows[h];
    const float4* p = reinterpret_cast<const float4*>(a.carry + (int64_t)lr.y * 128) + c;
    float4 acc = p[0];
    for (int i = 1; i < lr.z; i += 8) {
      float4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = i + u < lr.z ? p[(int64_t)(i + u) * 32] : acc;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (i + u < lr.z) {
          acc.x = __fadd_rn(acc.x, t[u].x);
          acc.y = __fadd_rn(acc.y, t[u].y);
          acc.z = __fadd_rn(acc.z, t[u].z);
          acc.w = __fadd_rn(acc.w, t[u].w);
        }
      }
    }
    *reinterpret_cast<float4*>(a.out + (int64_t)lr.x * a.ldo + c * 4) = acc;
  }
}

struct PairPlanWs {
  int32_t *nseg, *nslot, *seg_off, *slot_off, *counter;
  uint32_t *keys, *skeys, *iota, *sidx;
  int4* useg;
  void* temp;
  size_t temp_bytes;
};

static size_t pair_temp_bytes(int64_t n_rows, int64_t cap) {
  size_t a = 0, b = 0;
  (void)rocprim::exclusive_scan(nullptr, a, (const int32_t*)nullptr, (int32_t*)nullptr, 0,
                                (size_t)(n_rows > 0 ? n_rows : 1), rocprim::plus<int32_t>(),
                                (hipStream_t)0);
  (void)rocprim::radix_sort_pairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (size_t)(cap > 0 ? cap : 1), 0, 32, (hipStream_t)0);
  return a > b ? a : b;
}

static PairPlanWs pair_ws_layout(void* ws, int32_t n_rows, int64_t cap, size_t* total) {
  PairPlanWs w{};
  char* p = reinterpret_cast<char*>(ws);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = p ? p + off : nullptr;
    off += align_up(bytes > 0 ? bytes : 1, 256);
    return q;
  };
  const size_t nr = (size_t)(n_rows > 0 ? n_rows : 1);
  w.nseg = (int32_t*)take(nr * 4);
  w.nslot = (int32_t*)take(nr * 4);
  w.seg_off = (int32_t*)take(nr * 4);
  w.slot_off = (int32_t*)take(nr * 4);
  w.counter = (int32_t*)take(256);
  w.keys = (uint32_t*)take((size_t)cap * 4);
  w.skeys = (uint32_t*)take((size_t)cap * 4);
  w.iota = (uint32_t*)take((size_t)cap * 4);
  w.sidx = (uint32_t*)take((size_t)cap * 4);
  w.useg = (int4*)take((size_t)cap * 16);
  w.temp_bytes = pair_temp_bytes(n_rows, cap);
  w.temp = take(w.temp_bytes);
  if (total) *total = off;
  return w;
}

}  // namespace vqgnn

using namespace vqgnn;

extern "C" int vqgnn_spmm_pair_supported(int32_t F) { return F == 128 ? 1 : 0; }

extern "C" int64_t vqgnn_spmm_pair_plan_size(int32_t n_rows, int64_t nnz, int32_t F) {
  if (n_rows < 0 || nnz < 0 || F <= 0) return 0;
  const int S = spmm_chunk_edges((F + 3) / 4), L = spmm_long_row(S);
  return kPairHdr + 4 * pair_seg_cap(n_rows, nnz, S, L) + 4 * pair_long_cap(nnz, L);
}

extern "C" size_t vqgnn_spmm_pair_plan_workspace(int32_t n_rows, int64_t nnz, int32_t F) {
  if (n_rows < 0 || nnz < 0 || F <= 0) return 256;
  const int S = spmm_chunk_edges((F + 3) / 4), L = spmm_long_row(S);
  size_t total = 0;
  (void)pair_ws_layout(nullptr, n_rows, pair_seg_cap(n_rows, nnz, S, L), &total);
  return total;
}

extern "C" int vqgnn_spmm_pair_plan(const int32_t* rowptr, int32_t n_rows, int64_t nnz,
                                    int32_t F, int32_t B, int32_t* plan, void* workspace,
                                    vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(vqgnn_spmm_pair_supported(F), "spmm_pair_plan: F=%d unsupported", F);
  VQGNN_REQUIRE(rowptr && plan && workspace && n_rows >= 0 && nnz >= 0 &&
                    nnz < (int64_t)INT32_MAX,
                "spmm_pair_plan: bad arguments");
  VQGNN_REQUIRE(B >= 0 && B <= n_rows, "spmm_pair_plan: need 0 <= B <= n_rows (B=%d)", B);
  VQGNN_REQUIRE((n_rows >> kPairWinShift) < (1 << 19), "spmm_pair_plan: too many rows");
  hipStream_t s = as_stream(stream);
  const int S = spmm_chunk_edges((F + 3) / 4), L = spmm_long_row(S);
  const int64_t cap = pair_seg_cap(n_rows, nnz, S, L);
  PairPlanWs w = pair_ws_layout(workspace, n_rows, cap, nullptr);
  int32_t* hdr = plan;
  int4* segs = reinterpret_cast<int4*>(plan + kPairHdr);
  int4* longrows = segs + cap;
  (void)hipMemsetAsync(w.counter, 0, 256, s);
  if (n_rows == 0) {
    (void)hipMemsetAsync(hdr, 0, kPairHdr * 4, s);
    return check_launch("spmm_pair_plan(empty)");
  }
  const int nbk = (n_rows + 255) / 256;
  hipLaunchKernelGGL(pair_count_kernel, dim3(nbk), dim3(256), 0, s, rowptr, n_rows, S, L, w.nseg,
                     w.nslot);
  size_t tb = w.temp_bytes;
  hipError_t e = rocprim::exclusive_scan(w.temp, tb, w.nseg, w.seg_off, 0, (size_t)n_rows,
                                         rocprim::plus<int32_t>(), s);
  tb = w.temp_bytes;
  if (e == hipSuccess)
    e = rocprim::exclusive_scan(w.temp, tb, w.nslot, w.slot_off, 0, (size_t)n_rows,
                                rocprim::plus<int32_t>(), s);
  if (e != hipSuccess) {
    set_error("spmm_pair_plan: scan failed (%s)", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  const int cbk = (int)((cap + 255) / 256);
  hipLaunchKernelGGL(pair_pad_kernel, dim3(cbk), dim3(256), 0, s, w.keys, w.iota, w.seg_off,
                     w.nseg, n_rows, cap);
  hipLaunchKernelGGL(pair_fill_kernel, dim3(nbk), dim3(256), 0, s, rowptr, n_rows, B, S, L,
                     w.seg_off, w.slot_off, w.useg, w.keys, longrows, w.counter);
  tb = w.temp_bytes;
  e = rocprim::radix_sort_pairs(w.temp, tb, w.keys, w.skeys, w.iota, w.sidx, (size_t)cap, 0, 32,
                                s);
  if (e != hipSuccess) {
    set_error("spmm_pair_plan: sort failed (%s)", hipGetErrorString(e));
    return VQGNN_ERR_LAUNCH;
  }
  hipLaunchKernelGGL(pair_gather_kernel, dim3(cbk), dim3(256), 0, s, w.useg, w.sidx, w.skeys,
                     segs, cap);
  hipLaunchKernelGGL(pair_hdr_kernel, dim3(1), dim3(64), 0, s, w.skeys, cap, w.counter, hdr);
  return check_launch("spmm_pair_plan");
}

extern "C" int vqgnn_spmm_pair(const int32_t* rowptr, const int32_t* col, const float* val,
                               int32_t n_rows, int32_t n_cols, int64_t nnz, int32_t B,
                               const float* X, int64_t ldx, const float* X2, int64_t ldx2,
                               int32_t F, float* out, int64_t ldo, const int32_t* plan,
                               const int32_t* chunk_plan, void* workspace,
                               vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(vqgnn_spmm_pair_supported(F), "spmm_pair: F=%d unsupported", F);
  VQGNN_REQUIRE(rowptr && out && plan && n_rows >= 0, "spmm_pair: null pointer");
  VQGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= F && ldo >= F,
                "spmm_pair: ldx/ldo must be multiples of 4 and >= F");
  VQGNN_REQUIRE(!X2 || (ldx2 % 4 == 0 && ldx2 >= F && ((uintptr_t)X2 & 15) == 0),
                "spmm_pair: X2 must be 16-byte aligned with ldx2 a multiple of 4, >= F");
  VQGNN_REQUIRE(((uintptr_t)X & 15) == 0 && ((uintptr_t)out & 15) == 0,
                "spmm_pair: X/out must be 16-byte aligned");
  VQGNN_REQUIRE(nnz < (int64_t)INT32_MAX, "spmm_pair: nnz >= 2^31");
  VQGNN_REQUIRE(n_cols >= 0 && (!X2 || (B >= 0 && B <= n_cols)),
                "spmm_pair: need 0 <= B <= n_cols with X2 (n_cols=%d B=%d)", n_cols, B);
  if (n_rows == 0 || nnz == 0)
    return vqgnn_spmm(rowptr, col, val, n_rows, n_cols, nnz, B, X, ldx, X2, ldx2, F, out, ldo,
                      chunk_plan, workspace, stream);
  VQGNN_REQUIRE(col && val && X && workspace, "spmm_pair: null pointer");
  SpmmArgs t{};
  t.X = X;
  t.ldx4 = ldx / 4;
  t.X2 = X2;
  t.ldx24 = X2 ? ldx2 / 4 : 0;
  const int64_t rows_x = X2 ? B : n_cols, rows_x2 = X2 ? (int64_t)n_cols - B : 0;
  // X and X2 more than 4 GiB apart: the chunk kernels (64-bit row addresses)
  if (!wave_layout(t, rows_x, rows_x2) || t.span > 0xFFFFF000u)
    return vqgnn_spmm(rowptr, col, val, n_rows, n_cols, nnz, B, X, ldx, X2, ldx2, F, out, ldo,
                      chunk_plan, workspace, stream);
  PairArgs a;
  a.col = col;
  a.val = val;
  a.hdr = plan;
  a.segs = reinterpret_cast<const int4*>(plan + kPairHdr);
  const int S = spmm_chunk_edges(F / 4), L = spmm_long_row(S);
  a.longrows = a.segs + pair_seg_cap(n_rows, nnz, S, L);
  a.ubase = t.ubase;
  a.span = t.span;
  a.offx = t.offx;
  a.ldxb = t.ldxb;
  a.offx2 = t.offx2;
  a.ldx2b = t.ldx2b;
  a.B = X2 ? B : INT32_MAX;
  a.out = out;
  a.ldo = ldo;
  a.carry = reinterpret_cast<float*>(workspace);
  hipStream_t s = as_stream(stream);
  static const int bpc = env_int("VQGNN_PAIR_BPC", 8);   // workgroups per CU
  const int grid = 256 * (bpc > 0 ? bpc : 8);
  static const int dbg = env_int("VQGNN_SPMM_DEBUG", 0);
  a.dbg = dbg;
  switch (a.dbg & 11) {
    case 0: hipLaunchKernelGGL(spmm_pair_kernel<0>, dim3(grid), dim3(kSpmmThreads), 0, s, a); break;
    case 1: hipLaunchKernelGGL(spmm_pair_kernel<1>, dim3(grid), dim3(kSpmmThreads), 0, s, a); break;
    case 2: hipLaunchKernelGGL(spmm_pair_kernel<2>, dim3(grid), dim3(kSpmmThreads), 0, s, a); break;
    case 8: hipLaunchKernelGGL(spmm_pair_kernel<8>, dim3(grid), dim3(kSpmmThreads), 0, s, a); break;
    case 10: hipLaunchKernelGGL(spmm_pair_kernel<10>, dim3(grid), dim3(kSpmmThreads), 0, s, a); break;
    default: hipLaunchKernelGGL(spmm_pair_kernel<3>, dim3(grid), dim3(kSpmmThreads), 0, s, a); break;
  }
  hipLaunchKernelGGL(spmm_pair_fixup_kernel, dim3(256), dim3(kSpmmThreads), 0, s, a);
  return check_launch("spmm_pair");
}
