// Task-split CSR SpMM for gfx950 (MI355X): out = A * xin with
// xin = [X (rows < B) ; X2 (rows >= B)] — LowRankGNNLayer's aggregation
// (vq_gnn_v2/models.py:174 + convs.py:95: torch_sparse.matmul(adj, x_input,
// reduce='add')) without materialising the torch.cat.
//
// Work split (merge-based SpMM).  The nnz range is cut into tasks of K
// consecutive edges.  A group of 8 lanes walks one task edge by edge; a wave
// holds 8 groups, i.e. 8 tasks in lock-step — every group runs exactly K
// steps, so the wave is balanced whatever the row lengths (arxiv: median 7,
// max 1,460 edges).  Per step a lane gathers NC float4 pieces of the edge's
// source row (piece i of lane k is float4 column 8i + k: each gather
// wave-instruction reads one contiguous 128-byte line per group, 1 KiB per
// instruction), multiplies by the weight and accumulates with fma.  When the
// edge ends its row the group stores the row (or, for a row that began in an
// earlier task, its head partial) and resets; a row still open at the task's
// end leaves a tail partial.  spmm_task_fixup_kernel adds, for every row
// that spans tasks, tail[first task] + ... + tail[last-1] + head[last] in
// task order, and writes zeros to empty rows.
//
// Per-batch plan (vqgnn_spmm_task_plan): one 8-byte record per edge — source
// column (bits 0-25), "row ends here" (bit 31) and the number of empty rows
// that follow (bits 26-30, 31 = look it up), and the weight — plus the row
// containing each task's first edge.  The kernel reads no rowptr / col / val.
//
// Numerics: each row is a sequential fma chain over its edges in CSR order
// (rows split across tasks: the task partials added in task order).
// Deterministic and independent of the launch geometry; within 1e-5 relative
// of the fp64 sum (north_star tolerance), not the bit pattern of spmm_sum's
// separate multiply and add.

#include "common.h"

#include <type_traits>
#include <utility>

namespace vqgnn {

constexpr int kTaskThreads = 256;             // 4 waves
constexpr uint32_t kColMask = (1u << 26) - 1;
constexpr uint32_t kEndBit = 1u << 31;
constexpr int kSkipShift = 26;
constexpr uint32_t kSkipEsc = 31;

struct TaskArgs {
  const int2* rec;          // [nnz] (col | skip << 26 | end << 31, weight bits)
  const int32_t* task_start;  // [ntasks + 1] first edge of each task (row-aligned unless split)
  const int32_t* task_row;    // [ntasks] row containing the task's first edge
  const int32_t* jobs;        // fixup: [ntasks][3] slots, n_jobs used (row, first task,
                              // last task), then [n_rows] slots, n_empty used (empty rows)
  int n_jobs, n_empty;
  const int32_t* rowptr;    // [n_rows + 1] (fixup, skip escapes)
  int n_rows, nnz, K, ntasks;
  int B;                    // columns < B read X, >= B read X2 (row j - B)
  const float* X;
  int64_t ldx;              // floats
  const float* X2;
  int64_t ldx2;
  int F;                    // columns (multiple of 4)
  float* out;
  int64_t ldo;
  float* carry;             // [ntasks][2][cf]: head partial, tail partial (cf = F + 4:
                            // GAT keeps the row's coefficient sum in slot F)
  int cf;
  // near path: X and X2 as one 32-bit buffer range from ubase
  const char* ubase;
  uint32_t span, offx, ldxb, offx2, ldx2b;
  uint32_t ldob;            // near path: ldo in bytes (rows addressed with a 24-bit multiply)
  int dbg;                  // experiments: 1 = no row stores (results invalid)
  // GAT mode (OurGATConv + the layer's ones-column normalisation): edge
  // weight = exp(leaky(al[j] + ar[i])) * w with al, ar = alpha / s per node,
  // rows < norm_B divided by their coefficient sum + 1e-16
  const int32_t* erow;      // [nnz] COO row of every edge
  const float* al;          // [n] alpha_l / s, alpha_r / s of x_in rows
  const float* ar;
  float slope;
  int norm_B;
  float* den;               // [n_rows] optional: coefficient sums
  float* coef;              // [nnz] optional: the coefficients (for the backward)
};

__device__ __forceinline__ int upper_bound_i32(const int32_t* __restrict__ a, int n, int key) {
  // first i in [0, n] with a[i] > key  (a non-decreasing, n + 1 entries read)
  int lo = 0, hi = n + 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// ---- plan ----------------------------------------------------------------
__global__ void task_records_kernel(const int32_t* __restrict__ col, const float* __restrict__ val,
                                    int nnz, int2* __restrict__ rec) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  rec[e] = make_int2(col[e] & (int)kColMask, val ? __float_as_int(val[e]) : __float_as_int(1.f));
}

__global__ void task_row_ends_kernel(const int32_t* __restrict__ rowptr, int n_rows,
                                     int2* __restrict__ rec) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int e1 = rowptr[r + 1];
  if (e1 == rowptr[r]) return;             // empty row: no edge to mark
  uint32_t skip = 0;
  for (int k = r + 1; k < n_rows && skip < kSkipEsc && rowptr[k + 1] == rowptr[k]; ++k) ++skip;
  int2 v = rec[e1 - 1];
  v.x = (int)(((uint32_t)v.x & kColMask) | (skip << kSkipShift) | kEndBit);
  rec[e1 - 1] = v;
}

// Task t nominally starts at edge t*K.  A row of at most K/2 edges that holds
// the nominal start is not split: the task starts at the next row instead
// (the previous task takes the whole row), so tasks hold K/2..3K/2 edges and
// only rows longer than K/2 are cut (their partials summed by the fixup).
__global__ void task_first_row_kernel(const int32_t* __restrict__ rowptr, int n_rows, int nnz,
                                      int K, int snap, int ntasks, int32_t* __restrict__ task_start,
                                      int32_t* __restrict__ task_row) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntasks) return;
  int st = t == ntasks ? nnz : t * K;
  if (t > 0 && t < ntasks) {
    const int r = upper_bound_i32(rowptr, n_rows, st) - 1;   // row containing edge st
    const int rs = rowptr[r], re = rowptr[r + 1];
    if (rs < st && re - rs <= snap) st = re;
  }
  task_start[t] = st;
  if (t < ntasks) task_row[t] = st < nnz ? upper_bound_i32(rowptr, n_rows, st) - 1 : n_rows - 1;
}

// Fix-up jobs: a row cut by task boundaries (its first edge in task ts, its
// last in task t > ts) -> (row, ts, t); an empty row -> its index.  Appended
// with atomics (the order does not matter: every job writes its own row).
__global__ void task_jobs_kernel(const int32_t* __restrict__ rowptr, int n_rows, int ntasks,
                                 const int32_t* __restrict__ task_start,
                                 const int32_t* __restrict__ task_row, int32_t* __restrict__ jobs,
                                 int32_t* __restrict__ empties, int32_t* __restrict__ counts) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int nnz = task_start[ntasks];
  if (x < ntasks && task_start[x] < nnz) {
    const int e0 = task_start[x];
    const int r = task_row[x];
    const int rs = rowptr[r], re = rowptr[r + 1];
    if (rs < e0 && re <= task_start[x + 1]) {
      const int ts = upper_bound_i32(task_start, ntasks, rs) - 1;
      const int j = atomicAdd(counts, 1);
      jobs[3 * j] = r;
      jobs[3 * j + 1] = ts;
      jobs[3 * j + 2] = x;
    }
  }
  if (x < n_rows && rowptr[x + 1] == rowptr[x]) empties[atomicAdd(counts + 1, 1)] = x;
}

// ---- main kernel ---------------------------------------------------------
// Source of record word x (column j = x & kColMask).  Near path: one 24-bit
// multiply-add, j * ld + base, with (ld, base) = (ldxb, offx + lane_off) or
// (ldx2b, offx2 - B * ldx2b + lane_off) (mod 2^32; task_setup guarantees
// columns, strides and the range below 2^24 / 2^31).  v_mad_u32_u24 reads
// only bits 0-23 of x, so the flag bits need no mask.
template <bool FAR>
__device__ __forceinline__ void row_src(const TaskArgs& a, uint32_t x, uint32_t b1, uint32_t b2,
                                        uint32_t lane_off, uint32_t* off, const char** p) {
  const uint32_t j = x & kColMask;
  if constexpr (FAR) {
    const float* row = (int)j < a.B ? a.X + (int64_t)j * a.ldx : a.X2 + (int64_t)((int)j - a.B) * a.ldx2;
    *p = reinterpret_cast<const char*>(row) + lane_off;
  } else {
    const bool s1 = (int)j < a.B;
    *off = __umul24(x, s1 ? a.ldxb : a.ldx2b) + (s1 ? b1 : b2);
  }
}

// out[u] = x of lane u of this lane's group (ds_swizzle bit mode inside each
// 32-lane half: lane id -> (id & AND) | u); the pattern must be an immediate
template <int AND, int... Us>
__device__ __forceinline__ void group_bcast(int x, int (&out)[sizeof...(Us)],
                                            std::integer_sequence<int, Us...>) {
  ((out[Us] = __builtin_amdgcn_ds_swizzle(x, AND | (Us << 5))), ...);
}

// G lanes per task (64 / G tasks per wave), NC float4 pieces per lane (piece
// i of lane k is float4 column G*i + k: a column tile of 4*G*NC floats), U
// edges per block
// GAT coefficient of one edge (convs.py:209-264, vq_softmax.py:33-57, the
// op order of gat_coef_kernel): exp(leaky(al[j] + ar[i])) * w, al / ar
// already divided by s per node as the reference does (convs.py:209-211)
__device__ __forceinline__ float gat_edge_coef(const TaskArgs& a, int e, uint32_t j, float w) {
  float x = __fadd_rn(a.al[j], a.ar[a.erow[e]]);
  x = x > 0.f ? x : __fmul_rn(x, a.slope);
  return __fmul_rn(expf(x), w);
}

// PART (near path): the last column tile is partial (F/4 not a multiple of
// G*NC): its lanes past F load nothing (an offset past the buffer range
// returns 0 without a memory access) instead of reading the next row
template <int G, int NC, int U, bool FAR, bool GAT, bool PART>
__device__ __forceinline__ void task_walk(const TaskArgs& a, int wv, int nwaves) {
  constexpr int TPW = 64 / G;
  const int lane = threadIdx.x & 63;
  const int g = lane / G, k = lane % G;
  const int t = wv * TPW + g;
  // a call over the first n_rows rows of a larger CSR (the backward's
  // transpose restricted to batch rows) covers edges [0, rowptr[n_rows])
  const int nnz = min(a.nnz, a.rowptr[a.n_rows]);
  if (wv >= nwaves || wv * TPW >= a.ntasks) return;
  // the wave's records are addressed from its first task's first edge: 32-bit
  // buffer offsets cover any nnz < 2^31 (a wave spans at most 64 tasks)
  const int wbase = a.task_start[wv * TPW];
  if (wbase >= nnz) return;
  const bool tv = t < a.ntasks;
  const int e0 = tv ? min(a.task_start[t], nnz) : nnz;
  const bool valid = e0 < nnz;
  const int e1 = valid ? min(nnz, a.task_start[t + 1]) : e0;

  const int F4 = a.F >> 2;
  const int c4base = (int)blockIdx.y * NC * G + k;   // this lane's first float4 column
  bool pv[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) pv[i] = c4base + G * i < F4;
  const uint32_t lane_off = (uint32_t)c4base * 16u;
  uint32_t kill[NC];                        // PART: 2^31 (> the range) for pieces past F
#pragma unroll
  for (int i = 0; i < NC; ++i) kill[i] = PART && !pv[i] ? 0x80000000u : 0u;
  const uint32_t b1 = a.offx + lane_off;
  const uint32_t b2 = a.offx2 - (uint32_t)a.B * a.ldx2b + lane_off;

  int r = valid ? a.task_row[t] : 0;
  bool head = valid && a.rowptr[r] < e0;    // first row began in an earlier task

  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ubase, 0, FAR ? 0 : (int)a.span, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.rec + wbase), 0,
      (int)(uint32_t)min((int64_t)(a.nnz - wbase) * 8, (int64_t)0x7FFFFFFF), 0x00020000);

  float4 acc[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);

  // Records: lane k < U of a group holds the record of edge e + k of the
  // current block (one coalesced 8-byte load per lane); step u reads edge
  // e + u's record from lane u of its group by a ds_swizzle broadcast.
  // Records outside [e0, e1) read as weight 0 without a row end.
  static_assert(U <= G, "records of a block live in the group's first U lanes");
  constexpr int kAnd = 0x1F & ~(G - 1);               // keep the group bits (32-lane swizzle)
  // GAT: the record lane computes its edge's coefficient and broadcasts it as
  // the weight (and, on column tile 0, stores it for the backward)
  // The load is issued a block ahead and masked only when its block starts,
  // so no wait for it sits between a block's gathers and the next block's.
  auto load_rec = [&](int e) -> int2 {
    return __builtin_bit_cast(
        int2, __builtin_amdgcn_raw_buffer_load_b64(rsr, (uint32_t)(e - wbase + k) * 8u, 0, 0));
  };
  auto mask_rec = [&](int2 q, int e) -> int2 {
    const int eu = e + k;
    const bool in = k < U && eu >= e0 && eu < e1;
    if constexpr (GAT) {
      if (!in) return make_int2(0, 0);
      const float c = gat_edge_coef(a, eu, (uint32_t)q.x & kColMask, __int_as_float(q.y));
      if (a.coef && blockIdx.y == 0) a.coef[eu] = c;
      return make_int2(q.x, __float_as_int(c));
    } else {
      return in ? q : make_int2(0, 0);
    }
  };
  float den = 0.f;     // GAT: the row's coefficient sum (the ones column), edge order

  // the wave runs as many U-edge blocks as its longest task needs
  int len = e1 - e0;
#pragma unroll
  for (int o = G; o < 64; o <<= 1) len = max(len, __shfl_xor(len, o));

  // one block: broadcast its records to the group and issue its gathers (v);
  // consume: the fma chain and the row ends, in edge order.
  // Near path: the record lane computes its edge's source-row byte offset
  // (column -> X or X2 row, one 24-bit multiply-add) once for the block and
  // the group receives offsets (co) beside the record words (cx: row ends,
  // skip counts) and weights (cw).  Far path: 64-bit addresses per step.
  struct Blk {
    int cx[U];      // record words: column, skip count, row end
    int cw[U];      // weights (GAT: coefficients)
    int co[U];      // near: source-row byte offsets
  };
  auto issue = [&](int2 rcur, int e, Blk& bk, float4 (&v)[U][NC]) {
    group_bcast<kAnd>(rcur.x, bk.cx, std::make_integer_sequence<int, U>{});
    if constexpr (!FAR) {
      const uint32_t x = (uint32_t)rcur.x;
      const bool s1 = (int)(x & kColMask) < a.B;
      const uint32_t roff = __umul24(x, s1 ? a.ldxb : a.ldx2b) +
                            (s1 ? a.offx : a.offx2 - (uint32_t)a.B * a.ldx2b);
      group_bcast<kAnd>((int)roff, bk.co, std::make_integer_sequence<int, U>{});
    }
    group_bcast<kAnd>(rcur.y, bk.cw, std::make_integer_sequence<int, U>{});
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        if constexpr (FAR) {
          const char* p = nullptr;
          uint32_t off = 0;
          row_src<FAR>(a, (uint32_t)bk.cx[u], b1, b2, lane_off, &off, &p);
          v[u][i] = pv[i] ? *reinterpret_cast<const float4*>(p + 16 * G * i)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {   // pieces past F read the next row (or 0 past the range): never stored
          const uint32_t off = (uint32_t)bk.co[u] + lane_off + 16u * G * i;
          const uint32_t o = PART ? (off | kill[i]) : off;
          v[u][i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsx, o, 0, 0));
        }
      }
    }
  };
  auto consume = [&](int e, const Blk& bk, const float4 (&v)[U][NC]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float w = __int_as_float(bk.cw[u]);
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        acc[i].x = fmaf(w, v[u][i].x, acc[i].x);
        acc[i].y = fmaf(w, v[u][i].y, acc[i].y);
        acc[i].z = fmaf(w, v[u][i].z, acc[i].z);
        acc[i].w = fmaf(w, v[u][i].w, acc[i].w);
      }
      if constexpr (GAT) den = __fadd_rn(den, w);
      const uint32_t x = (uint32_t)bk.cx[u];
      if (x & kEndBit) {                   // the row ends at this edge
        float* dst = head ? a.carry + (int64_t)t * 2 * a.cf
                   : FAR  ? a.out + (int64_t)r * a.ldo
                          : reinterpret_cast<float*>(reinterpret_cast<char*>(a.out) +
                                                     (uint64_t)(uint32_t)__umul24((uint32_t)r, a.ldob));
        if constexpr (GAT) {
          if (head) {                      // partial: the fixup sums and normalises
            if (k == 0 && blockIdx.y == 0) dst[a.F] = den;
          } else {
            if (a.den && k == 0 && blockIdx.y == 0) a.den[r] = den;
            if (r < a.norm_B) {            // models.py:188: out[:, :F] /= out[:, F] + 1e-16
              // one v_rcp_f32 (1 ulp) and four multiplies instead of four IEEE
              // divisions (≈ 2 ulp, inside the 1e-5 bound; the walker is
              // VALU-bound and this path runs at every row end)
              const float rq = __builtin_amdgcn_rcpf(__fadd_rn(den, 1e-16f));
#pragma unroll
              for (int i = 0; i < NC; ++i) {
                acc[i].x = __fmul_rn(acc[i].x, rq);
                acc[i].y = __fmul_rn(acc[i].y, rq);
                acc[i].z = __fmul_rn(acc[i].z, rq);
                acc[i].w = __fmul_rn(acc[i].w, rq);
              }
            }
          }
          den = 0.f;
        }
#pragma unroll
        for (int i = 0; i < NC; ++i) {
          if (pv[i] && !(a.dbg & 1))
            *reinterpret_cast<float4*>(dst + 4 * (c4base + G * i)) = acc[i];
          acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const uint32_t skip = (x >> kSkipShift) & kSkipEsc;
        r = skip == kSkipEsc ? upper_bound_i32(a.rowptr, a.n_rows, e + u + 1) - 1
                             : r + 1 + (int)skip;
        head = false;
      }
    }
  };

  // wave-uniform (every lane holds the max): an SGPR loop, not an exec-masked one
  const int nblk = __builtin_amdgcn_readfirstlane((len + U - 1) / U);
  if constexpr (GAT && G >= 16) {
    // GAT, pipelined: records are loaded two blocks ahead and the coefficient
    // inputs al[j], ar[i] one block ahead, both issued before the current
    // block's gathers, so the gathers' wait covers them and no dependent load
    // sits at a block start.  The row i of each edge comes from the group's
    // row at the block start plus a prefix sum of the row-end increments
    // (1 + empty rows skipped) of the earlier edges (DPP within the 16-lane
    // record row), not from an erow load; a block holding a skip escape (31
    // or more empty rows in a row) reads erow for it and for the next block.
    int rb = r;            // group's row at the next prepared block's first edge
    bool known = true;     // rb is exact
    auto prep = [&](int2 q, int eb, float& alv, float& arv) {
      const int eu = eb + k;
      const bool in = k < U && eu >= e0 && eu < e1;
      const uint32_t x = in ? (uint32_t)q.x : 0u;
      const uint32_t skip = (x >> kSkipShift) & kSkipEsc;
      const int inc = (x & kEndBit) ? 1 + (int)skip : 0;
      int incl = inc;
      incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xF, 0xF, true);   // row_shr:1
      incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xF, 0xF, true);   // row_shr:2
      incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xF, 0xF, true);   // row_shr:4
      incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xF, 0xF, true);   // row_shr:8
      const int total = __builtin_amdgcn_ds_swizzle(incl, kAnd | (15 << 5));
      const uint64_t em = __ballot((x & kEndBit) && skip == kSkipEsc);
      const bool gesc = ((em >> (lane & ~(G - 1))) & (G == 64 ? ~0ull : ((1ull << G) - 1))) != 0;
      int row;
      if (known && !gesc) {
        row = rb + incl - inc;
      } else {               // exact rows from erow (rare)
        row = in ? a.erow[eu] : 0;
        rb = __builtin_amdgcn_ds_swizzle(row, kAnd);    // the group's first edge
        row = in ? row : 0;
      }
      known = !gesc;
      rb += total;
      alv = in ? a.al[x & kColMask] : 0.f;
      arv = in ? a.ar[row] : 0.f;
    };
    auto coef = [&](int2 q, int eb, float alv, float arv) -> int2 {
      const int eu = eb + k;
      if (!(k < U && eu >= e0 && eu < e1)) return make_int2(0, 0);
      float z = __fadd_rn(alv, arv);        // alpha / s per node (convs.py:209-211, :256)
      z = z > 0.f ? z : __fmul_rn(z, a.slope);
      const float c = __fmul_rn(expf(z), __int_as_float(q.y));
      if (a.coef && blockIdx.y == 0) a.coef[eu] = c;
      return make_int2(q.x, __float_as_int(c));
    };
    int2 r0 = load_rec(e0), r1 = load_rec(e0 + U);
    float al0, ar0;
    prep(r0, e0, al0, ar0);
    for (int bi = 0; bi < nblk; ++bi) {
      const int e = e0 + bi * U;
      const int2 r2 = load_rec(e + 2 * U);
      float al1, ar1;
      prep(r1, e + U, al1, ar1);
      Blk bk;
      float4 v[U][NC];
      issue(coef(r0, e, al0, ar0), e, bk, v);
      consume(e, bk, v);
      r0 = r1;
      r1 = r2;
      al0 = al1;
      ar0 = ar1;
    }
  } else {
    int2 rraw = load_rec(e0);
    for (int bi = 0; bi < nblk; ++bi) {
      const int e = e0 + bi * U;
      // next block's records (past the buffer: zeros; outside the task: masked)
      const int2 rnxt = load_rec(e + U);
      Blk bk;
      float4 v[U][NC];
      issue(mask_rec(rraw, e), e, bk, v);
      consume(e, bk, v);
      rraw = rnxt;
    }
  }
  // the task's last row continues in the next task unless its last edge ends
  // a row (records outside the task carry no row end)
  const bool open = valid && !(__builtin_amdgcn_raw_buffer_load_b32(rsr, (uint32_t)(e1 - 1 - wbase) * 8u,
                                                                    0, 0) & (int)kEndBit);
  if (open) {
    float* dst = a.carry + ((int64_t)t * 2 + 1) * a.cf;
#pragma unroll
    for (int i = 0; i < NC; ++i)
      if (pv[i]) *reinterpret_cast<float4*>(dst + 4 * (c4base + G * i)) = acc[i];
    if constexpr (GAT) {
      if (k == 0 && blockIdx.y == 0) dst[a.F] = den;
    }
  }
}

// the default shape (G = 32, NC = 1) at most 128 VGPRs: 4 waves per SIMD (64
// gathers in flight per SIMD at U = 16); the wider experiment shapes unbounded
template <int G, int NC, int U, bool FAR, bool GAT = false, bool PART = false>
__global__ void __launch_bounds__(kTaskThreads)
__attribute__((amdgpu_waves_per_eu((G == 32 && NC == 1) ? 4 : 1)))
spmm_task_kernel(TaskArgs a) {
  const int nwaves = (int)gridDim.x * (kTaskThreads / 64);
  // wave-uniform in an SGPR: the record buffer resource built from it is then
  // scalar (a VGPR-derived resource costs a readfirstlane loop per block)
  const int wv = __builtin_amdgcn_readfirstlane(
      xcd_remap(blockIdx.x, gridDim.x) * (kTaskThreads / 64) + (threadIdx.x >> 6));
  task_walk<G, NC, U, FAR, GAT, PART>(a, wv, nwaves);
}

// One wave per fix-up job.  A cut row: out[row] = tail[ts] + ... + tail[t-1]
// + head[t], in task order (loads 8 tasks ahead of the in-order adds); GAT
// sums the coefficient slot the same way, then normalises rows < norm_B.
// An empty row: zeros.  Rows at or past n_rows (a call over leading rows)
// are skipped.
template <bool GAT>
__global__ void __launch_bounds__(256)
spmm_task_fixup_kernel(TaskArgs a) {
  // L lanes per job: 32 when a row (plus the GAT slot) fits 32 float4 pieces,
  // so a wave finishes two rows
  const int F4 = a.F >> 2;
  const int L = F4 <= 32 ? 32 : 64;          // (GAT's slot column F4 is skipped below)
  const int lane = threadIdx.x & (L - 1);
  const int w = (blockIdx.x * 256 + threadIdx.x) / L;
  const int C4 = a.cf >> 2;                 // carry row stride in float4
  if (w < a.n_jobs) {
    const int r = a.jobs[3 * w], ts = a.jobs[3 * w + 1], t = a.jobs[3 * w + 2];
    if (r < 0 || r >= a.n_rows) return;
    const float4* c4 = reinterpret_cast<const float4*>(a.carry);
    auto add4 = [](float4 x, float4 y) {
      return make_float4(__fadd_rn(x.x, y.x), __fadd_rn(x.y, y.y), __fadd_rn(x.z, y.z),
                         __fadd_rn(x.w, y.w));
    };
    // column F4 (GAT) is the coefficient-sum slot
    const int ncol = GAT ? F4 + 1 : F4;
    float q = 1.f;
    bool norm = false;
    if constexpr (GAT) {                   // every lane needs the row's coefficient sum
      float d = a.carry[((int64_t)ts * 2 + 1) * a.cf + a.F];
      int u = ts + 1;
      for (; u + 8 <= t; u += 8) {         // loads 8 tasks ahead of the in-order adds
        float dv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) dv[i] = a.carry[((int64_t)(u + i) * 2 + 1) * a.cf + a.F];
#pragma unroll
        for (int i = 0; i < 8; ++i) d = __fadd_rn(d, dv[i]);
      }
      for (; u < t; ++u) d = __fadd_rn(d, a.carry[((int64_t)u * 2 + 1) * a.cf + a.F]);
      d = __fadd_rn(d, a.carry[(int64_t)t * 2 * a.cf + a.F]);
      if (a.den && lane == 0) a.den[r] = d;
      norm = r < a.norm_B;
      // the walker's normalisation (one v_rcp_f32, then multiplies), so a row
      // gets the same bits whether or not the plan cuts it across tasks
      q = __builtin_amdgcn_rcpf(__fadd_rn(d, 1e-16f));
    }
    for (int c = lane; c < ncol; c += L) {
      if (GAT && c == F4) continue;
      float4 sum = c4[((int64_t)ts * 2 + 1) * C4 + c];
      int u = ts + 1;
      for (; u + 8 <= t; u += 8) {
        float4 qq[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) qq[i] = c4[((int64_t)(u + i) * 2 + 1) * C4 + c];
#pragma unroll
        for (int i = 0; i < 8; ++i) sum = add4(sum, qq[i]);
      }
      for (; u < t; ++u) sum = add4(sum, c4[((int64_t)u * 2 + 1) * C4 + c]);
      sum = add4(sum, c4[(int64_t)t * 2 * C4 + c]);
      if (norm) {
        sum.x = __fmul_rn(sum.x, q);
        sum.y = __fmul_rn(sum.y, q);
        sum.z = __fmul_rn(sum.z, q);
        sum.w = __fmul_rn(sum.w, q);
      }
      reinterpret_cast<float4*>(a.out + (int64_t)r * a.ldo)[c] = sum;
    }
  } else if (w < a.n_jobs + a.n_empty) {
    if constexpr (GAT) {
      const int r0 = a.jobs[3 * a.ntasks + (w - a.n_jobs)];
      if (a.den && lane == 0 && r0 >= 0 && r0 < a.n_rows) a.den[r0] = 0.f;
    }
    const int r = a.jobs[3 * a.ntasks + (w - a.n_jobs)];    // the empty-row list
    if (r < 0 || r >= a.n_rows) return;
    float4* o = reinterpret_cast<float4*>(a.out + (int64_t)r * a.ldo);
    for (int c = lane; c < F4; c += L) o[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

static int task_env(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

template <int G, int NC, int U, bool FAR, bool GAT, bool PART = false>
static void launch_task(const TaskArgs& a, int tiles, hipStream_t s) {
  const int waves = (a.ntasks + 64 / G - 1) / (64 / G);
  const int blocks = (waves + 3) / 4;
  hipLaunchKernelGGL((spmm_task_kernel<G, NC, U, FAR, GAT, PART>), dim3(blocks, tiles),
                     dim3(kTaskThreads), 0, s, a);
}

// U edges per block, at most G (a block's records live in the group's lanes)
template <int G, int NC, bool GAT>
static void launch_task_u(const TaskArgs& a, int tiles, int U, bool near, hipStream_t s) {
  if (U > G) U = G;
  if (near) {
    if constexpr (G >= 16) {
      if (U == 16) {
        if constexpr (!GAT && NC == 1) {   // the default shape: a partial last tile
          if ((a.F >> 2) % (G * NC) != 0) return launch_task<G, NC, 16, false, GAT, true>(a, tiles, s);
        }
        return launch_task<G, NC, 16, false, GAT>(a, tiles, s);
      }
    }
    if (U == 8) return launch_task<G, NC, 8, false, GAT>(a, tiles, s);
    if (U == 4) return launch_task<G, NC, 4, false, GAT>(a, tiles, s);
    return launch_task<G, NC, 2, false, GAT>(a, tiles, s);
  }
  if constexpr (G >= 16) {
    if (U == 16) return launch_task<G, NC, 16, true, GAT>(a, tiles, s);
  }
  if (U == 8) return launch_task<G, NC, 8, true, GAT>(a, tiles, s);
  if (U == 4) return launch_task<G, NC, 4, true, GAT>(a, tiles, s);
  return launch_task<G, NC, 2, true, GAT>(a, tiles, s);
}


// ---- hot-column tiles: the default GCN/SAGE aggregation --------------------
//
// The task kernel above gathers every edge's 512-byte source row from the L2
// (1.06 GB per arxiv launch) and sits on the per-CU gather rate (DESIGN.md
// §4.2).  The batch comes from a cluster sampler (dataloader.py:28-38) over a
// graph with Zipf-weighted hubs, so the rows of a contiguous row tile reuse
// a small set of source rows many times (arxiv: the 1,024 most referenced
// source rows of a 16 k-edge tile carry 64 % of its edges, ~10 uses each).
// The hot plan cuts the rows into row-aligned tiles of about Et edges and
// picks, per tile, its (at most C) most referenced source rows used at least
// twice.  A workgroup = (tile, 32-float column slice): it stages those rows'
// slices in LDS (C x 128 B), walks the tile's tasks (K edges each, 8 lanes per
// task, one float4 per lane) reading hot rows from LDS and the others from
// global memory, then sums the tile's cut rows itself (rows never span
// tiles: no fix-up kernel).  Per-row arithmetic is the task kernel's: a
// sequential fma chain in CSR order, cut rows' partials added in task order;
// which rows are hot changes where a value is read from, never its bits.
//
// Hot records: the task records with bits 0-24 = source column, or (bit 25
// set) the row's LDS slot; bits 26-31 as above (skip count, row end).

constexpr int kHotLdsBytes = 128 * 1024;      // staged hot slices per workgroup (at most)
constexpr int kHotMaxC = 1024;                // hot rows per tile (128-byte slices)
constexpr uint32_t kLocalBit = 1u << 25;
constexpr uint32_t kHotColMask = (1u << 25) - 1;
constexpr int kHotTab = 24576;                // plan hash table (keys 96 KiB + u16 counts 48 KiB)
constexpr int kHotProbe = 64;
constexpr int kHotHeader = 8;                 // plan ints: T, C, Et, ntasks, K, 0, 0, 0

struct HotView {
  int32_t* head;
  int32_t* tile_row;    // [T + 1] first row of each tile (row-aligned)
  int32_t* tile_task;   // [T + 1] first task of each tile
  int32_t* hot_n;       // [T] hot rows per tile
  int32_t* task_start;  // [NT + 1]
  int32_t* task_row;    // [NT]
  int32_t* hot;         // [T][C] source column of each LDS slot
};

inline int hot_tiles(int64_t nnz, int Et) { return nnz > 0 ? (int)((nnz + Et - 1) / Et) : 1; }
inline int hot_ntasks_max(int64_t nnz, int K, int T) { return (int)(nnz / K) + T + 1; }

inline HotView hot_view(int32_t* base, int T, int NT, int C) {
  HotView v;
  v.head = base;
  v.tile_row = base + kHotHeader;
  v.tile_task = v.tile_row + T + 1;
  v.hot_n = v.tile_task + T + 1;
  v.task_start = v.hot_n + T;
  v.task_row = v.task_start + NT + 1;
  v.hot = v.task_row + NT;
  return v;
}

__device__ __forceinline__ int lower_bound_i32(const int32_t* __restrict__ a, int n, int key) {
  // first i in [0, n) with a[i] >= key (n if none)
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// tile t starts at the first row whose first edge is at or past t * Et
__global__ void hot_tiles_kernel(const int32_t* __restrict__ rowptr, int n_rows, int nnz, int Et,
                                 int T, int32_t* __restrict__ tile_row) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > T) return;
  tile_row[t] = t == 0 ? 0 : t == T ? n_rows
                      : lower_bound_i32(rowptr, n_rows + 1, (int)min((int64_t)t * Et, (int64_t)nnz));
}

// tile_task = exclusive scan of ceil(edges / K) over the tiles (one block)
__global__ void __launch_bounds__(1024)
hot_scan_kernel(const int32_t* __restrict__ rowptr, int T, int K, int C, int Et,
                const int32_t* __restrict__ tile_row, int32_t* __restrict__ tile_task,
                int32_t* __restrict__ head) {
  __shared__ int part[1024];
  const int per = (T + 1023) / 1024;
  const int t0 = threadIdx.x * per, t1 = min(T, t0 + per);
  auto ntask = [&](int t) {
    const int E = rowptr[tile_row[t + 1]] - rowptr[tile_row[t]];
    return (E + K - 1) / K;
  };
  int sum = 0;
  for (int t = t0; t < t1; ++t) sum += ntask(t);
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = (int)threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int t = t0; t < t1; ++t) {
    tile_task[t] = run;
    run += ntask(t);
  }
  if (threadIdx.x == 1023) {
    tile_task[T] = part[1023];
    head[0] = T;
    head[1] = C;
    head[2] = Et;
    head[3] = part[1023];        // tasks in all tiles
    head[4] = K;
  }
}

// start of task kk (of ntask) of a tile [te0, te1): nominal starts every K
// edges from the tile's first edge, snapped past rows of at most K/2 edges
// (as task_first_row_kernel); kk == ntask: the tile's end
__device__ __forceinline__ int hot_task_start(const int32_t* __restrict__ rowptr, int n_rows,
                                              int K, int te0, int te1, int kk, int ntask) {
  if (kk >= ntask) return te1;
  int st = te0 + kk * K;
  if (kk > 0) {
    const int r = upper_bound_i32(rowptr, n_rows, st) - 1;
    const int rs = rowptr[r], re = rowptr[r + 1];
    if (rs < st && re - rs <= K / 2) st = re;
  }
  return st;
}

// task x: its first edge, and its first row with two flags: bit 31 "head"
// (the row began in an earlier task), bit 30 "open" (the task's last row
// continues in the next task) -- so the SpMM reads no rowptr per task
constexpr uint32_t kHeadBit = 1u << 31, kOpenBit = 1u << 30, kRowMask = (1u << 30) - 1;
__global__ void hot_tasks_kernel(const int32_t* __restrict__ rowptr, int n_rows, int nnz, int K,
                                 int T, const int32_t* __restrict__ tile_row,
                                 const int32_t* __restrict__ tile_task,
                                 const int32_t* __restrict__ head, int32_t* __restrict__ task_start,
                                 int32_t* __restrict__ task_row) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = head[3];
  if (x > total) return;
  if (x == total) {
    task_start[x] = nnz;
    return;
  }
  const int t = upper_bound_i32(tile_task, T, x) - 1;
  const int kk = x - tile_task[t];
  const int ntask = tile_task[t + 1] - tile_task[t];
  const int te0 = rowptr[tile_row[t]], te1 = rowptr[tile_row[t + 1]];
  const int st = hot_task_start(rowptr, n_rows, K, te0, te1, kk, ntask);
  const int en = hot_task_start(rowptr, n_rows, K, te0, te1, kk + 1, ntask);
  task_start[x] = st;
  uint32_t row = (uint32_t)(tile_row[t + 1] - 1), flags = 0;
  if (st < en) {
    row = (uint32_t)(upper_bound_i32(rowptr, n_rows, st) - 1);
    if (rowptr[row] < st) flags |= kHeadBit;
    const int rl = upper_bound_i32(rowptr, n_rows, en - 1) - 1;   // the row of the last edge
    if (rowptr[rl + 1] > en) flags |= kOpenBit;
  }
  task_row[x] = (int)(row | flags);
}

__device__ __forceinline__ int hot_hash(int c) {
  return (int)(((uint64_t)((uint32_t)c * 2654435761u) * kHotTab) >> 32);
}

// One workgroup per tile: count the tile's source columns in an LDS hash
// table, keep the (at most C) most referenced ones used at least twice (a
// count threshold from a histogram; ties at the threshold in table order),
// number them in table order, and rewrite the tile's records (bit 25 + slot
// for a hot column).  Columns the table cannot place within kHotProbe probes
// stay global (speed only).
__global__ void __launch_bounds__(1024)
hot_select_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, int C,
                  const int32_t* __restrict__ tile_row, int32_t* __restrict__ hot_n,
                  int32_t* __restrict__ hot, int2* __restrict__ rec) {
  __shared__ int32_t keys[kHotTab];
  __shared__ uint32_t cnt[kHotTab / 2];        // u16 counts, then u16 slots (0xFFFF: none)
  __shared__ int32_t sc[1024];
  __shared__ int32_t hist[1024];
  __shared__ int32_t vstar_s;
  const int tid = threadIdx.x;
  const int t = blockIdx.x;
  const int e0 = rowptr[tile_row[t]], e1 = rowptr[tile_row[t + 1]];
  for (int i = tid; i < kHotTab; i += 1024) keys[i] = -1;
  for (int i = tid; i < kHotTab / 2; i += 1024) cnt[i] = 0;
  hist[tid] = 0;
  if (tid == 0) vstar_s = 1024;
  __syncthreads();
  for (int e = e0 + tid; e < e1; e += 1024) {
    const int c = col[e];
    int i = hot_hash(c);
    for (int p = 0; p < kHotProbe; ++p) {
      int k = keys[i];
      if (k == -1) {
        k = atomicCAS(&keys[i], -1, c);
        if (k == -1) k = c;
      }
      if (k == c) {
        atomicAdd(&cnt[i >> 1], 1u << (16 * (i & 1)));
        break;
      }
      i = i + 1 == kHotTab ? 0 : i + 1;
    }
  }
  __syncthreads();
  auto count_of = [&](int i) { return (int)((cnt[i >> 1] >> (16 * (i & 1))) & 0xFFFFu); };
  for (int i = tid; i < kHotTab; i += 1024) {
    const int n = count_of(i);
    if (n >= 2) atomicAdd(&hist[min(n, 1023)], 1);
  }
  __syncthreads();
  // ge(v) = entries with capped count >= v: a suffix scan of the histogram
  sc[tid] = hist[1023 - tid];
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = tid >= o ? sc[tid - o] : 0;
    __syncthreads();
    sc[tid] += v;
    __syncthreads();
  }
  auto ge = [&](int v) { return v >= 1024 ? 0 : sc[1023 - v]; };
  // v*: the smallest count >= 2 whose class and above fit in C
  if (tid >= 2 && ge(tid) <= C && (tid == 2 || ge(tid - 1) > C)) vstar_s = tid;
  __syncthreads();
  const int vstar = vstar_s;
  const int tie = vstar - 1;                     // the partly taken class (if >= 2)
  const int quota = tie >= 2 ? C - ge(vstar) : 0;
  constexpr int kPer = kHotTab / 1024;           // 24 entries per thread, in table order
  const int i0 = tid * kPer;
  int nties = 0;
  for (int i = i0; i < i0 + kPer; ++i) nties += min(count_of(i), 1023) == tie;
  __syncthreads();
  sc[tid] = nties;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = tid >= o ? sc[tid - o] : 0;
    __syncthreads();
    sc[tid] += v;
    __syncthreads();
  }
  int tie_rank = sc[tid] - nties;
  bool sel[kPer];
  int nsel = 0;
  for (int j = 0; j < kPer; ++j) {
    const int n = min(count_of(i0 + j), 1023);
    bool s = n >= 2 && n >= vstar;
    if (n == tie && tie >= 2) {
      s = tie_rank < quota;
      ++tie_rank;
    }
    sel[j] = s;
    nsel += s;
  }
  __syncthreads();
  sc[tid] = nsel;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = tid >= o ? sc[tid - o] : 0;
    __syncthreads();
    sc[tid] += v;
    __syncthreads();
  }
  int slot = sc[tid] - nsel;
  const int total = sc[1023];
  __syncthreads();
  for (int j = 0; j < kPer; j += 2) {            // this thread's u16 pairs (i0 even)
    uint32_t w = 0;
    for (int h = 0; h < 2; ++h) {
      uint32_t v = 0xFFFFu;
      if (sel[j + h]) {
        hot[(int64_t)t * C + slot] = keys[i0 + j + h];
        v = (uint32_t)slot++;
      }
      w |= v << (16 * h);
    }
    cnt[(i0 + j) >> 1] = w;
  }
  if (tid == 0) hot_n[t] = min(total, C);
  __syncthreads();
  for (int e = e0 + tid; e < e1; e += 1024) {
    const int c = col[e];
    int i = hot_hash(c);
    uint32_t low = (uint32_t)c & kHotColMask;
    for (int p = 0; p < kHotProbe; ++p) {
      const int k = keys[i];
      if (k == c) {
        const uint32_t sl = (cnt[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
        if (sl != 0xFFFFu) low = kLocalBit | sl;
        break;
      }
      if (k == -1) break;
      i = i + 1 == kHotTab ? 0 : i + 1;
    }
    int2 v = rec[e];
    v.x = (int)(((uint32_t)v.x & ~kColMask) | low);
    rec[e] = v;
  }
}

struct HotArgs {
  const int2* rec;
  const int32_t* tile_row;
  const int32_t* tile_task;
  const int32_t* hot_n;
  const int32_t* task_start;
  const int32_t* task_row;
  const int32_t* hot;
  const int32_t* rowptr;
  int n_rows, nnz, K, T, C, S;
  int B;
  const float* X;
  int64_t ldx;
  const float* X2;
  int64_t ldx2;
  int F;
  float* out;
  int64_t ldo;
  float* carry;
  int cf;
  const char* ubase;
  uint32_t span, offx, ldxb, offx2, ldx2b, ldob;
  int dbg;    // experiments (VQGNN_HOT_DBG): 1 no fix-up kernel, 2 no stores, 4 all edges global
};

// Byte offset (near) / address (far) of source row j's slice piece.
template <bool FAR>
__device__ __forceinline__ const char* hot_far_row(const HotArgs& a, int j) {
  const float* row = j < a.B ? a.X + (int64_t)j * a.ldx : a.X2 + (int64_t)(j - a.B) * a.ldx2;
  return reinterpret_cast<const char*>(row);
}

// G lanes per task, one float4 each: a column slice of 4G floats (G = 32:
// 512-byte slices, two tasks per wave as the task kernel walks them; G = 8:
// 128-byte slices, eight tasks per wave).  NW waves per workgroup: 16 (one
// workgroup per CU) or 8 (two per CU: one's staging overlaps the other's walk).
template <int G, bool FAR, bool PART, int NW>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(4)))
spmm_hot_kernel(HotArgs a) {
  extern __shared__ float4 lds[];                    // [C][G] float4
  constexpr int U = 16, NT = NW * 64;
  constexpr int TPW = 64 / G;                        // tasks per wave and round
  const int L = xcd_remap(blockIdx.x, gridDim.x);   // a tile's slices: one XCD, consecutive
  const int t = L / a.S, sl = L - t * a.S;
  const int r0 = a.tile_row[t];
  const int r1 = min(a.tile_row[t + 1], a.n_rows);
  if (r0 >= r1) return;                              // workgroup-uniform
  const int nlim = a.rowptr[r1];                     // edges of the rows computed here
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane / G, k = lane % G;
  const int F4 = a.F >> 2;
  const int c4 = sl * G + k;                         // this lane's float4 column
  const bool pv = c4 < F4;
  const uint32_t lane_off = (uint32_t)c4 * 16u;
  const uint32_t kill = PART && !pv ? 0x80000000u : 0u;
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ubase, 0, FAR ? 0 : (int)a.span, 0x00020000);

  // this wave's first round of tasks: its metadata is issued before the
  // staging, so the two latencies overlap; every later round's metadata is
  // issued one round ahead
  const int x0 = a.tile_task[t], x1 = a.tile_task[t + 1];
  struct Meta { int ws, s0, s1, tr; };
  auto meta = [&](int xbb) {
    Meta m{0, 0, 0, 0};
    const int x = xbb + g;
    if (xbb < x1) m.ws = a.task_start[xbb];
    if (x < x1) {
      m.s0 = a.task_start[x];
      m.s1 = a.task_start[x + 1];
      m.tr = a.task_row[x];
    }
    return m;
  };
  int xb = x0 + wv * TPW;
  Meta cur = meta(xb);

  // 1. stage the tile's hot rows (this slice) in LDS: G lanes per row
  const int nh = min(a.hot_n[t], a.C);
  const int32_t* hot = a.hot + (int64_t)t * a.C;
  for (int s0 = tid / G; s0 < nh; s0 += 8 * (NT / G)) {
    float4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int s = s0 + i * (NT / G);
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s < nh && pv) {
        const int j = hot[s];
        if constexpr (FAR) {
          v[i] = *reinterpret_cast<const float4*>(hot_far_row<FAR>(a, j) + lane_off);
        } else {
          const bool s1 = j < a.B;
          const uint32_t off = __umul24((uint32_t)j, s1 ? a.ldxb : a.ldx2b) +
                               (s1 ? a.offx : a.offx2 - (uint32_t)a.B * a.ldx2b) + lane_off;
          v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int s = s0 + i * (NT / G);
      if (s < nh) lds[s * G + k] = v[i];
    }
  }
  __syncthreads();

  // 2. the tile's tasks: a wave takes TPW consecutive tasks per round; the
  //    rows cut across tasks are summed by spmm_hot_fixup_kernel
  constexpr int kAnd = 0x1F & ~(G - 1);
  const char* ldsb = reinterpret_cast<const char*>(lds);
  int2 pq0 = make_int2(0, 0), pq1 = make_int2(0, 0);   // next round's first records, loaded
  bool pre = false;                                    // during this round's last block
  for (; xb < x1; xb += NW * TPW) {
    const Meta nxt = meta(xb + NW * TPW);            // next round's metadata in flight
    const int x = xb + g;
    const bool tv = x < x1;
    const int wbase = __builtin_amdgcn_readfirstlane(min(cur.ws, nlim));
    const int e0 = tv ? min(cur.s0, nlim) : nlim;
    const int e1 = tv ? min(cur.s1, nlim) : e0;
    const bool valid = e0 < e1;
    const uint32_t trw = (uint32_t)cur.tr;
    int r = (int)(trw & kRowMask);
    bool head = valid && (trw & kHeadBit);
    // a task clipped at the caller's last row ends at a row end
    const bool open = valid && (trw & kOpenBit) && cur.s1 <= nlim;
    cur = nxt;
    const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.rec + wbase), 0,
        (int)(uint32_t)min((int64_t)(a.nnz - wbase) * 8, (int64_t)0x7FFFFFFF), 0x00020000);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int len = e1 - e0;
#pragma unroll
    for (int o = G; o < 64; o <<= 1) len = max(len, __shfl_xor(len, o));
    const int nblk = __builtin_amdgcn_readfirstlane((len + U - 1) / U);
    // lane k of a group holds the record of edge e + k (and, when a block
    // holds more edges than the group has lanes, of edge e + G + k)
    auto load_rec = [&](int e, int2& q0, int2& q1) {
      q0 = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(
                                        rsr, (uint32_t)(e - wbase + k) * 8u, 0, 0));
      if constexpr (G < U)
        q1 = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(
                                          rsr, (uint32_t)(e - wbase + G + k) * 8u, 0, 0));
      else
        q1 = make_int2(0, 0);
    };
    int2 q0, q1;
    if (pre) {
      q0 = pq0;
      q1 = pq1;
    } else {
      load_rec(e0, q0, q1);
    }
    pre = false;
    const int xn = xb + NW * TPW;                      // the next round (cur: its metadata)
    for (int bi = 0; bi < nblk; ++bi) {
      const int e = e0 + bi * U;
      int2 n0, n1;
      if (bi + 1 < nblk) {
        load_rec(e + U, n0, n1);
      } else if (xn < x1) {
        // the next round's first block, issued under this block's gathers
        const int nwb = __builtin_amdgcn_readfirstlane(min(cur.ws, nlim));
        const int ne0 = xn + g < x1 ? min(cur.s0, nlim) : nlim;
        const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.rec + nwb), 0,
            (int)(uint32_t)min((int64_t)(a.nnz - nwb) * 8, (int64_t)0x7FFFFFFF), 0x00020000);
        pq0 = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(
                                           rn, (uint32_t)(ne0 - nwb + k) * 8u, 0, 0));
        if constexpr (G < U)
          pq1 = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(
                                             rn, (uint32_t)(ne0 - nwb + G + k) * 8u, 0, 0));
        pre = true;
      }
      const bool in0 = k < U && e + k >= e0 && e + k < e1;
      const bool in1 = e + G + k >= e0 && e + G + k < e1;
      int2 m0 = in0 ? q0 : make_int2(0, 0), m1 = in1 ? q1 : make_int2(0, 0);
      if (a.dbg & 4) {               // experiment: every edge from memory
        m0.x &= ~(int)kLocalBit;
        m1.x &= ~(int)kLocalBit;
      }
      int cx[U], cw[U];
      constexpr int UB = G < U ? G : U;              // edges broadcast per record register
      group_bcast<kAnd>(m0.x, *reinterpret_cast<int(*)[UB]>(cx), std::make_integer_sequence<int, UB>{});
      group_bcast<kAnd>(m0.y, *reinterpret_cast<int(*)[UB]>(cw), std::make_integer_sequence<int, UB>{});
      if constexpr (G < U) {
        group_bcast<kAnd>(m1.x, *reinterpret_cast<int(*)[UB]>(cx + G), std::make_integer_sequence<int, UB>{});
        group_bcast<kAnd>(m1.y, *reinterpret_cast<int(*)[UB]>(cw + G), std::make_integer_sequence<int, UB>{});
      }
      // every lane reads LDS first (a global edge reads slot 0, overwritten
      // below), then the global edges load under their exec mask: a global
      // load waits only for the LDS reads ahead of it, not a full LDS drain
      // per divergent edge (the register WAW between the two paths).  Each
      // lane derives the source offset from the broadcast record word (LDS
      // slot, or a 24-bit multiply-add for the global row).
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t xw = (uint32_t)cx[u];
        const uint32_t lo = xw & kLocalBit ? (xw & 0xFFFFu) * (uint32_t)(G * 16) : 0u;
        v[u] = *reinterpret_cast<const float4*>(ldsb + lo + k * 16);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t xw = (uint32_t)cx[u];
        if (!(xw & kLocalBit)) {
          if constexpr (FAR) {
            v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (pv) v[u] = *reinterpret_cast<const float4*>(
                        hot_far_row<FAR>(a, (int)(xw & kHotColMask)) + lane_off);
          } else {
            const uint32_t j = xw & kHotColMask;
            const bool s1 = (int)j < a.B;
            const uint32_t o = (__umul24(j, s1 ? a.ldxb : a.ldx2b) +
                                (s1 ? a.offx : a.offx2 - (uint32_t)a.B * a.ldx2b) + lane_off) | kill;
            v[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsx, o, 0, 0));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float w = __int_as_float(cw[u]);
        acc.x = fmaf(w, v[u].x, acc.x);
        acc.y = fmaf(w, v[u].y, acc.y);
        acc.z = fmaf(w, v[u].z, acc.z);
        acc.w = fmaf(w, v[u].w, acc.w);
        const uint32_t xw = (uint32_t)cx[u];
        if (xw & kEndBit) {
          float* dst = head ? a.carry + (int64_t)x * 2 * a.cf
                     : FAR  ? a.out + (int64_t)r * a.ldo
                            : reinterpret_cast<float*>(reinterpret_cast<char*>(a.out) +
                                                       (uint64_t)(uint32_t)__umul24((uint32_t)r, a.ldob));
          if (pv && !(a.dbg & 2)) *reinterpret_cast<float4*>(dst + 4 * c4) = acc;
          acc = make_float4(0.f, 0.f, 0.f, 0.f);
          const uint32_t skip = (xw >> kSkipShift) & kSkipEsc;
          r = skip == kSkipEsc ? upper_bound_i32(a.rowptr, a.n_rows, e + u + 1) - 1
                               : r + 1 + (int)skip;
          head = false;
        }
      }
      if (bi + 1 < nblk) {
        q0 = n0;
        q1 = n1;
      }
    }
    if (open && pv) *reinterpret_cast<float4*>(a.carry + ((int64_t)x * 2 + 1) * a.cf + 4 * c4) = acc;
  }
}

// Rows cut across tasks: 8 lanes per task whose first row began in an
// earlier task and ends in it -> tail[ts] + ... + tail[x-1] + head[x], in
// task order, all columns (the tasks inside a row longer than K/2 start every
// K edges, so ts = x - ceil((e0 - row start) / K)).  Then one thread per row:
// empty rows get zeros.
__global__ void __launch_bounds__(256)
spmm_hot_fixup_kernel(HotArgs a, int task_blocks) {
  const int F4 = a.F >> 2, C4 = a.cf >> 2;
  const int nlim = a.rowptr[a.n_rows];
  if ((int)blockIdx.x < task_blocks) {
    const int x = (blockIdx.x * 256 + threadIdx.x) >> 3, k = threadIdx.x & 7;
    if (x >= a.tile_task[a.T]) return;
    const int e0 = min(a.task_start[x], nlim), e1 = min(a.task_start[x + 1], nlim);
    const uint32_t trw = (uint32_t)a.task_row[x];
    if (e0 >= e1 || !(trw & kHeadBit)) return;
    const int r = (int)(trw & kRowMask);
    const int rs = a.rowptr[r], re = a.rowptr[r + 1];
    if (re > e1) return;                             // the row continues: a later task sums it
    const int ts = x - (e0 - rs + a.K - 1) / a.K;
    const float4* c4p = reinterpret_cast<const float4*>(a.carry);
    auto add4 = [](float4 p, float4 q) {
      return make_float4(__fadd_rn(p.x, q.x), __fadd_rn(p.y, q.y), __fadd_rn(p.z, q.z),
                         __fadd_rn(p.w, q.w));
    };
    for (int c = k; c < F4; c += 8) {
      float4 sum = c4p[((int64_t)ts * 2 + 1) * C4 + c];
      int u = ts + 1;
      for (; u + 8 <= x; u += 8) {                   // loads 8 tasks ahead of the in-order adds
        float4 qq[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) qq[i] = c4p[((int64_t)(u + i) * 2 + 1) * C4 + c];
#pragma unroll
        for (int i = 0; i < 8; ++i) sum = add4(sum, qq[i]);
      }
      for (; u < x; ++u) sum = add4(sum, c4p[((int64_t)u * 2 + 1) * C4 + c]);
      sum = add4(sum, c4p[(int64_t)x * 2 * C4 + c]);
      reinterpret_cast<float4*>(a.out + (int64_t)r * a.ldo)[c] = sum;
    }
  } else {
    const int r = (blockIdx.x - task_blocks) * 256 + threadIdx.x;
    if (r >= a.n_rows || a.rowptr[r] != a.rowptr[r + 1]) return;
    float4* o = reinterpret_cast<float4*>(a.out + (int64_t)r * a.ldo);
    for (int c = 0; c < F4; ++c) o[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// the records' weights replaced (same structure and hot slots: the GAT
// backward's coefficient records on the transpose's hot plan)
__global__ void records_set_values_kernel(const int2* __restrict__ src, const float* __restrict__ val,
                                          int nnz, int2* __restrict__ dst) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  dst[e] = make_int2(src[e].x, val ? __float_as_int(val[e]) : __float_as_int(1.f));
}


}  // namespace vqgnn

using namespace vqgnn;

static int task_count(int64_t nnz, int K) { return (int)((nnz + K - 1) / K); }

extern "C" int64_t vqgnn_spmm_task_size(int64_t nnz, int32_t K, int32_t n_rows) {
  if (K <= 0) K = 64;
  // starts [ntasks + 1], first rows [ntasks], jobs [ntasks][3], empty rows [n_rows]
  return 5 * (int64_t)task_count(nnz, K) + 1 + (n_rows > 0 ? n_rows : 0);
}

static void task_records(const int32_t* rowptr, const int32_t* col, const float* val,
                         int32_t n_rows, int64_t nnz, int2* rec, hipStream_t s) {
  if (nnz <= 0) return;
  hipLaunchKernelGGL(task_records_kernel, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s,
                     col, val, (int)nnz, rec);
  if (n_rows > 0)
    hipLaunchKernelGGL(task_row_ends_kernel, dim3((n_rows + 255) / 256), dim3(256), 0, s, rowptr,
                       n_rows, rec);
}

extern "C" int vqgnn_spmm_task_records(const int32_t* rowptr, const int32_t* col, const float* val,
                                       int32_t n_rows, int64_t nnz, int64_t* records,
                                       vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(rowptr && n_rows >= 0 && nnz >= 0 && nnz < (int64_t)1 << 31,
                "spmm_task_records: bad arguments");
  VQGNN_REQUIRE(nnz == 0 || (col && records), "spmm_task_records: null pointer");
  task_records(rowptr, col, val, n_rows, nnz, reinterpret_cast<int2*>(records), as_stream(stream));
  return check_launch("spmm_task_records");
}

extern "C" int vqgnn_spmm_task_plan(const int32_t* rowptr, const int32_t* col, const float* val,
                                    int32_t n_rows, int64_t nnz, int32_t K, int32_t* plan,
                                    int64_t* records, int32_t* counts, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(rowptr && plan && counts && n_rows >= 0 && nnz >= 0 && nnz < (int64_t)1 << 31,
                "spmm_task_plan: bad arguments");
  VQGNN_REQUIRE(K >= 8 && K % 4 == 0 && K <= 4096,
                "spmm_task_plan: K=%d must be a multiple of 4 in [8, 4096]", K);
  VQGNN_REQUIRE(nnz == 0 || (col && records), "spmm_task_plan: null pointer");
  hipStream_t s = as_stream(stream);
  const int ntasks = task_count(nnz, K);
  int32_t* task_start = plan;
  int32_t* task_row = plan + ntasks + 1;
  int32_t* jobs = task_row + ntasks;
  int32_t* empties = jobs + 3 * ntasks;
  if (hipMemsetAsync(counts, 0, 2 * sizeof(int32_t), s) != hipSuccess)
    return check_launch("spmm_task_plan memset");
  task_records(rowptr, col, val, n_rows, nnz, reinterpret_cast<int2*>(records), s);
  hipLaunchKernelGGL(task_first_row_kernel, dim3((ntasks + 256) / 256), dim3(256), 0, s, rowptr,
                     n_rows, (int)nnz, K, task_env("VQGNN_TASK_SNAP", 1) ? K / 2 : 0, ntasks,
                     task_start, task_row);
  const int nx = ntasks > n_rows ? ntasks : n_rows;
  if (nx > 0)
    hipLaunchKernelGGL(task_jobs_kernel, dim3((nx + 255) / 256), dim3(256), 0, s, rowptr, n_rows,
                       ntasks, task_start, task_row, jobs, empties, counts);
  return check_launch("spmm_task_plan");
}

extern "C" size_t vqgnn_spmm_task_workspace(int64_t nnz, int32_t K, int32_t F) {
  // carries: [ntasks][2][F + 4] (slot F: the GAT coefficient sum)
  return align_up((size_t)task_count(nnz, K > 0 ? K : 64) * 2 * (F + 4) * sizeof(float), 256) +
         256;
}

// Shared setup of vqgnn_spmm_task / vqgnn_gat_spmm_task: validation, the
// task geometry and the near (one 32-bit buffer range) or far source path.
static int task_setup(TaskArgs& a, const int32_t* rowptr, int32_t n_rows, int32_t n_cols,
                      int64_t nnz, int32_t B, const float* X, int64_t ldx, const float* X2,
                      int64_t ldx2, int32_t F, float* out, int64_t ldo, const int32_t* plan,
                      const int64_t* records, int32_t K, int32_t n_jobs, int32_t n_empty,
                      void* workspace, bool* near) {
  VQGNN_REQUIRE(rowptr && out && plan && (nnz == 0 || (X && records && workspace)),
                "spmm_task: null pointer");
  VQGNN_REQUIRE(n_jobs >= 0 && n_empty >= 0, "spmm_task: bad job counts");
  VQGNN_REQUIRE(F > 0 && F % 4 == 0, "spmm_task: F=%d must be a positive multiple of 4", F);
  VQGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && (!X2 || ldx2 % 4 == 0) &&
                    ((uintptr_t)X & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                    ((uintptr_t)X2 & 15) == 0,
                "spmm_task: rows must be 16-byte aligned");
  VQGNN_REQUIRE(ldx >= F && ldo >= F && (!X2 || ldx2 >= F), "spmm_task: leading dimension < F");
  VQGNN_REQUIRE(n_cols <= (int32_t)kColMask, "spmm_task: %d columns exceed 2^26", n_cols);
  VQGNN_REQUIRE(B >= 0 && (X2 || B == 0), "spmm_task: B=%d without X2", B);
  VQGNN_REQUIRE(K >= 8 && K % 4 == 0, "spmm_task: K=%d", K);
  a.rec = reinterpret_cast<const int2*>(records);
  a.ntasks = task_count(nnz, K);
  a.task_start = plan;
  a.task_row = plan + a.ntasks + 1;
  a.jobs = a.task_row + a.ntasks;
  a.n_jobs = n_jobs;
  a.n_empty = n_empty;
  a.rowptr = rowptr;
  a.n_rows = n_rows;
  a.nnz = (int)nnz;
  a.K = K;
  a.B = X2 ? B : n_cols;
  a.X = X;
  a.ldx = ldx;
  a.X2 = X2 ? X2 : X;
  a.ldx2 = X2 ? ldx2 : ldx;
  a.F = F;
  a.cf = F + 4;
  a.out = out;
  a.ldo = ldo;
  a.carry = reinterpret_cast<float*>(workspace);
  const int nx = a.B, nx2 = X2 ? n_cols - B : 0;
  const uintptr_t x0 = (uintptr_t)X;
  const uintptr_t x1 = x0 + (uintptr_t)((int64_t)(nx > 0 ? nx - 1 : 0) * ldx + F) * 4;
  uintptr_t lo = x0, hi = x1;
  uintptr_t y0 = 0, y1 = 0;
  if (nx2 > 0) {
    y0 = (uintptr_t)X2;
    y1 = y0 + (uintptr_t)((int64_t)(nx2 - 1) * ldx2 + F) * 4;
    lo = lo < y0 ? lo : y0;
    hi = hi > y1 ? hi : y1;
  }
  // near: 32-bit buffer offsets from one base, and 24-bit row multiplies
  // (columns, rows and strides below 2^24, the output below 4 GiB)
  *near = hi - lo < 0x7FFFFFF0ull && (int64_t)ldx * 4 < (1 << 24) &&
          (int64_t)a.ldx2 * 4 < (1 << 24) && (int64_t)ldo * 4 < (1 << 24) &&
          n_cols < (1 << 24) && n_rows < (1 << 24) &&
          (int64_t)n_rows * ldo * 4 < ((int64_t)1 << 32) && !task_env("VQGNN_SPMM_FAR", 0);
  if (*near) {
    a.ubase = reinterpret_cast<const char*>(lo);
    a.span = (uint32_t)(hi - lo);
    a.offx = (uint32_t)(x0 - lo);
    a.ldxb = (uint32_t)(ldx * 4);
    a.offx2 = nx2 > 0 ? (uint32_t)(y0 - lo) : 0;
    a.ldx2b = (uint32_t)(a.ldx2 * 4);
    a.ldob = (uint32_t)(ldo * 4);
  }
  a.dbg = task_env("VQGNN_TASK_DBG", 0);
  return VQGNN_OK;
}

template <bool GAT>
static void task_fixup(const TaskArgs& a, hipStream_t s) {
  const int nfix = a.n_jobs + a.n_empty;
  if (nfix > 0) {
    const int jobs_per_block = a.F / 4 <= 32 ? 8 : 4;
    hipLaunchKernelGGL(spmm_task_fixup_kernel<GAT>, dim3((nfix + jobs_per_block - 1) / jobs_per_block),
                       dim3(256), 0, s, a);
  }
}

template <bool GAT>
static void task_launch(const TaskArgs& a, bool near, hipStream_t s) {
  if (a.nnz > 0) {
    const int F4 = a.F / 4;
    // lanes per task: VQGNN_TASK_G (8, 16 or 32; default 32); pieces per lane
    // so that one column tile covers min(F, 128) floats
    int G = task_env("VQGNN_TASK_G", 32);
    G = G >= 32 ? 32 : (G >= 16 ? 16 : 8);
    int nc = 1;
    while (nc * G < F4 && nc * G * 4 < 128) nc *= 2;      // 4*G*nc floats <= 128
    const int tiles = (F4 + nc * G - 1) / (nc * G);
    const int Ue = task_env("VQGNN_TASK_U", 16);
    const int U = Ue >= 16 ? 16 : (Ue >= 8 ? 8 : (Ue >= 4 ? 4 : 2));
    if (G == 8) {
      if (nc == 1) launch_task_u<8, 1, GAT>(a, tiles, U, near, s);
      else if (nc == 2) launch_task_u<8, 2, GAT>(a, tiles, U, near, s);
      else launch_task_u<8, 4, GAT>(a, tiles, U, near, s);
    } else if (G == 16) {
      if (nc == 1) launch_task_u<16, 1, GAT>(a, tiles, U, near, s);
      else launch_task_u<16, 2, GAT>(a, tiles, U, near, s);
    } else {
      launch_task_u<32, 1, GAT>(a, tiles, U, near, s);
    }
  }
  task_fixup<GAT>(a, s);
}

extern "C" int vqgnn_spmm_task(const int32_t* rowptr, int32_t n_rows, int32_t n_cols, int64_t nnz,
                               int32_t B, const float* X, int64_t ldx, const float* X2,
                               int64_t ldx2, int32_t F, float* out, int64_t ldo,
                               const int32_t* plan, const int64_t* records, int32_t K,
                               int32_t n_jobs, int32_t n_empty, void* workspace,
                               vqgnn_stream_t stream) {
  clear_error();
  TaskArgs a{};
  bool near = false;
  const int rc = task_setup(a, rowptr, n_rows, n_cols, nnz, B, X, ldx, X2, ldx2, F, out, ldo,
                            plan, records, K, n_jobs, n_empty, workspace, &near);
  if (rc != VQGNN_OK) return rc;
  task_launch<false>(a, near, as_stream(stream));
  return check_launch("spmm_task");
}

extern "C" int vqgnn_gat_spmm_task(const int32_t* rowptr, int32_t n_rows, int32_t n_cols,
                                   int64_t nnz, int32_t B, const float* X, int64_t ldx,
                                   const float* X2, int64_t ldx2, int32_t F, float* out,
                                   int64_t ldo, const int32_t* plan, const int64_t* records,
                                   int32_t K, int32_t n_jobs, int32_t n_empty,
                                   const int32_t* erow, const float* alpha_l_s,
                                   const float* alpha_r_s, float negative_slope, int32_t norm_B, float* den, float* coef,
                                   void* workspace, vqgnn_stream_t stream) {
  clear_error();
  TaskArgs a{};
  bool near = false;
  const int rc = task_setup(a, rowptr, n_rows, n_cols, nnz, B, X, ldx, X2, ldx2, F, out, ldo,
                            plan, records, K, n_jobs, n_empty, workspace, &near);
  if (rc != VQGNN_OK) return rc;
  VQGNN_REQUIRE(nnz == 0 || (erow && alpha_l_s && alpha_r_s), "gat_spmm_task: null pointer");
  VQGNN_REQUIRE(norm_B >= 0, "gat_spmm_task: norm_B=%d", norm_B);
  a.erow = erow;
  a.al = alpha_l_s;
  a.ar = alpha_r_s;
  a.slope = negative_slope;
  a.norm_B = norm_B;
  a.den = den;
  a.coef = coef;
  task_launch<true>(a, near, as_stream(stream));
  return check_launch("gat_spmm_task");
}

// ---- hot-column tile plan / SpMM (include/vqgnn.h §6h) ----
extern "C" int64_t vqgnn_spmm_hot_size(int64_t nnz, int32_t K, int32_t Et, int32_t C) {
  if (K <= 0) K = 64;
  if (Et <= 0) Et = 16384;
  if (C <= 0) C = kHotMaxC;
  const int T = hot_tiles(nnz, Et);
  const int NT = hot_ntasks_max(nnz, K, T);
  return kHotHeader + 3 * (int64_t)(T + 1) + (int64_t)NT + 1 + NT + (int64_t)T * C;
}

extern "C" size_t vqgnn_spmm_hot_workspace(int64_t nnz, int32_t K, int32_t Et, int32_t F) {
  if (K <= 0) K = 64;
  if (Et <= 0) Et = 16384;
  const int T = hot_tiles(nnz, Et);
  return align_up((size_t)hot_ntasks_max(nnz, K, T) * 2 * (F + 4) * sizeof(float), 256) + 256;
}

extern "C" int vqgnn_spmm_hot_plan(const int32_t* rowptr, const int32_t* col, const float* val,
                                   int32_t n_rows, int32_t n_cols, int64_t nnz, int32_t K,
                                   int32_t Et, int32_t C, int32_t* plan, int64_t* records,
                                   vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(rowptr && plan && n_rows > 0 && nnz >= 0 && nnz < (int64_t)1 << 31,
                "spmm_hot_plan: bad arguments");
  VQGNN_REQUIRE(K >= 8 && K % 4 == 0 && K <= 4096,
                "spmm_hot_plan: K=%d must be a multiple of 4 in [8, 4096]", K);
  VQGNN_REQUIRE(Et >= K && Et <= kHotTab * 2 / 3,
                "spmm_hot_plan: Et=%d must be in [K, %d]", Et, kHotTab * 2 / 3);
  VQGNN_REQUIRE(C >= 0 && C <= kHotMaxC, "spmm_hot_plan: C=%d must be in [0, %d]", C, kHotMaxC);
  VQGNN_REQUIRE(n_cols >= 0 && n_cols <= (int32_t)kHotColMask,
                "spmm_hot_plan: %d columns exceed 2^25", n_cols);
  VQGNN_REQUIRE(nnz == 0 || (col && records), "spmm_hot_plan: null pointer");
  hipStream_t s = as_stream(stream);
  const int T = hot_tiles(nnz, Et);
  const int NT = hot_ntasks_max(nnz, K, T);
  HotView v = hot_view(plan, T, NT, C);
  task_records(rowptr, col, val, n_rows, nnz, reinterpret_cast<int2*>(records), s);
  hipLaunchKernelGGL(hot_tiles_kernel, dim3((T + 256) / 256), dim3(256), 0, s, rowptr, n_rows,
                     (int)nnz, Et, T, v.tile_row);
  hipLaunchKernelGGL(hot_scan_kernel, dim3(1), dim3(1024), 0, s, rowptr, T, K, C, Et,
                     v.tile_row, v.tile_task, v.head);
  hipLaunchKernelGGL(hot_tasks_kernel, dim3((NT + 256) / 256), dim3(256), 0, s, rowptr, n_rows,
                     (int)nnz, K, T, v.tile_row, v.tile_task, v.head, v.task_start, v.task_row);
  // (also for nnz == 0: every tile's hot_n is written)
  hipLaunchKernelGGL(hot_select_kernel, dim3(T), dim3(1024), 0, s, rowptr, col, C, v.tile_row,
                     v.hot_n, v.hot, reinterpret_cast<int2*>(records));
  return check_launch("spmm_hot_plan");
}

extern "C" int vqgnn_spmm_records_set_values(const int64_t* records, const float* val, int64_t nnz,
                                             int64_t* out, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(nnz >= 0 && nnz < (int64_t)1 << 31, "spmm_records_set_values: bad nnz");
  if (nnz == 0) return VQGNN_OK;
  VQGNN_REQUIRE(records && out, "spmm_records_set_values: null pointer");
  hipLaunchKernelGGL(records_set_values_kernel, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0,
                     as_stream(stream), reinterpret_cast<const int2*>(records), val, (int)nnz,
                     reinterpret_cast<int2*>(out));
  return check_launch("spmm_records_set_values");
}

extern "C" int vqgnn_spmm_hot(const int32_t* rowptr, int32_t n_rows, int32_t n_cols, int64_t nnz,
                              int32_t B, const float* X, int64_t ldx, const float* X2,
                              int64_t ldx2, int32_t F, float* out, int64_t ldo,
                              const int32_t* plan, const int64_t* records, int32_t K, int32_t Et,
                              int32_t C, void* workspace, vqgnn_stream_t stream) {
  clear_error();
  TaskArgs ta{};
  bool near = false;
  // validation and the near / far source path shared with the task kernel
  // (its task geometry fields are unused here)
  int rc = task_setup(ta, rowptr, n_rows, n_cols, nnz, B, X, ldx, X2, ldx2, F, out, ldo, plan,
                      records, K, 0, 0, workspace, &near);
  if (rc != VQGNN_OK) return rc;
  VQGNN_REQUIRE(C >= 0 && C <= kHotMaxC && Et >= K, "spmm_hot: bad plan geometry");
  VQGNN_REQUIRE(n_cols <= (int32_t)kHotColMask, "spmm_hot: %d columns exceed 2^25", n_cols);
  if (n_rows == 0) return VQGNN_OK;
  VQGNN_REQUIRE(n_rows < (1 << 30), "spmm_hot: %d rows exceed 2^30", n_rows);
  const int T = hot_tiles(nnz, Et);
  const int NT = hot_ntasks_max(nnz, K, T);
  HotView v = hot_view(const_cast<int32_t*>(plan), T, NT, C);
  HotArgs a{};
  a.rec = reinterpret_cast<const int2*>(records);
  a.tile_row = v.tile_row;
  a.tile_task = v.tile_task;
  a.hot_n = v.hot_n;
  a.task_start = v.task_start;
  a.task_row = v.task_row;
  a.hot = v.hot;
  a.rowptr = rowptr;
  a.n_rows = n_rows;
  a.nnz = (int)nnz;
  a.K = K;
  a.T = T;
  a.C = C;
  // slices of 4G floats: G = 32 (512-byte rows, at most 256 hot rows) when
  // the plan's hot rows fit, else G = 8 (128-byte slices, up to 1,024)
  const int G = task_env("VQGNN_HOT_G", C <= kHotLdsBytes / 512 ? 32 : 8) >= 32 ? 32 : 8;
  VQGNN_REQUIRE((size_t)C * G * 16 <= (size_t)kHotLdsBytes,
                "spmm_hot: %d hot rows of %d bytes exceed the LDS", C, G * 16);
  a.S = (F / 4 + G - 1) / G;
  a.B = ta.B;
  a.X = ta.X;
  a.ldx = ta.ldx;
  a.X2 = ta.X2;
  a.ldx2 = ta.ldx2;
  a.F = F;
  a.out = out;
  a.ldo = ldo;
  a.carry = reinterpret_cast<float*>(workspace);
  a.cf = F + 4;
  a.ubase = ta.ubase;
  a.span = ta.span;
  a.offx = ta.offx;
  a.ldxb = ta.ldxb;
  a.offx2 = ta.offx2;
  a.ldx2b = ta.ldx2b;
  a.ldob = ta.ldob;
  a.dbg = task_env("VQGNN_HOT_DBG", 0);
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)((int64_t)T * a.S));
  const bool part = (F / 4) % G != 0;
  const size_t lds = (size_t)(C > 0 ? C : 1) * G * 16;
  // 16-wave workgroups (one per CU) when the slices take more than half the
  // LDS, else 8-wave workgroups two per CU; VQGNN_HOT_WAVES forces 8 or 16
  const int nw_env = task_env("VQGNN_HOT_WAVES", 0);
  const bool wide = nw_env ? nw_env >= 16 : lds > (size_t)kHotLdsBytes / 2;
  // dynamic LDS above 64 KiB: allowed once per kernel instance
  static const bool attrs = [] {
    void (*ks[])(HotArgs) = {
        spmm_hot_kernel<8, true, false, 16>,  spmm_hot_kernel<8, false, true, 16>,
        spmm_hot_kernel<8, false, false, 16>, spmm_hot_kernel<8, true, false, 8>,
        spmm_hot_kernel<8, false, true, 8>,   spmm_hot_kernel<8, false, false, 8>,
        spmm_hot_kernel<32, true, false, 16>,  spmm_hot_kernel<32, false, true, 16>,
        spmm_hot_kernel<32, false, false, 16>, spmm_hot_kernel<32, true, false, 8>,
        spmm_hot_kernel<32, false, true, 8>,   spmm_hot_kernel<32, false, false, 8>};
    for (auto k : ks)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kHotLdsBytes);
    return true;
  }();
  (void)attrs;
  auto go = [&](void (*kern)(HotArgs), int threads) {
    hipLaunchKernelGGL(kern, grid, dim3(threads), lds, s, a);
  };
  auto pick = [&](auto gtag) {
    constexpr int GG = decltype(gtag)::value;
    if (wide) {
      if (!near) go(spmm_hot_kernel<GG, true, false, 16>, 1024);
      else if (part) go(spmm_hot_kernel<GG, false, true, 16>, 1024);
      else go(spmm_hot_kernel<GG, false, false, 16>, 1024);
    } else {
      if (!near) go(spmm_hot_kernel<GG, true, false, 8>, 512);
      else if (part) go(spmm_hot_kernel<GG, false, true, 8>, 512);
      else go(spmm_hot_kernel<GG, false, false, 8>, 512);
    }
  };
  if (G == 32) pick(std::integral_constant<int, 32>{});
  else pick(std::integral_constant<int, 8>{});
  // rows cut across tasks and empty rows (unless VQGNN_HOT_DBG bit 0)
  if (!(a.dbg & 1)) {
    const int task_blocks = (NT * 8 + 255) / 256;
    const int row_blocks = (n_rows + 255) / 256;
    hipLaunchKernelGGL(spmm_hot_fixup_kernel, dim3(task_blocks + row_blocks), dim3(256), 0, s, a,
                       task_blocks);
  }
  return check_launch("spmm_hot");
}
