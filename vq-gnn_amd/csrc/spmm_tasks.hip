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
#include "ema_finalize.h"

#include <mutex>
#include <utility>

namespace vqgnn {

constexpr int kTaskThreads = 256;             // 4 waves
constexpr unsigned kRoundRobinGrid = 1u << 16; // task-kernel grids this large skip xcd_remap
constexpr uint32_t kColMask = (1u << 26) - 1;
constexpr uint32_t kEndBit = 1u << 31;
constexpr int kSkipShift = 26;
constexpr uint32_t kSkipEsc = 31;
constexpr uint32_t kHeadBit = 1u << 31;   // task_row: the first row began in an earlier task
constexpr int kRowMask = 0x7fffffff;

struct TaskArgs {
  const int2* rec;          // [nnz] (col | skip << 26 | end << 31, weight bits)
  const int32_t* task_start;  // [ntasks + 1] first edge of each task (row-aligned unless split)
  const int32_t* task_row;    // [ntasks] row containing the task's first edge (| kHeadBit:
                              // that row began in an earlier task)
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
  int xcd;                  // 1: XCD-contiguous task ranges (VQGNN_TASK_XCD=0, experiments
                            // builds only: the dispatcher's round-robin order)
  int dbg;                  // VQGNN_TASK_DBG (experiments builds only): 1 = no row
                            // stores, results invalid; 0 in the default library
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
  // codebook source (CB): the records of columns >= B hold B + the node id,
  // whose source row is its codewords -- column c of the row is feature
  // c % D of codeword codes[node][c / D] of branch c / D -- read from an LDS
  // image of the codebook's feature halves instead of a gathered row
  const int16_t* codes;     // [nodes][ldc]
  uint32_t codes_bytes;     // buffer range of codes (< 2^31)
  uint32_t ldcb;            // ldc in bytes
  const float* cbe;         // codewords: branch b, codeword m, feature d at
  int64_t cb_ldw, cb_bstride;   //   cbe[b * cb_bstride + m * cb_ldw + d]
  int cb_M, cb_D;
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

// codebook-source records: a column j >= B becomes B + nodes[j] (the node
// whose codes give the row); flags and weight kept.  A column past the subset
// or a node outside [0, n_nodes) becomes B + n_nodes, past the codes' buffer
// range (its code reads as 0 with no memory access), with weight 0: it adds
// 0 x codeword 0, the zero row gather_codewords writes for it (invalid input)
__global__ void task_remap_cb_kernel(int2* __restrict__ rec, int nnz, int B, int n_cols,
                                     const int64_t* __restrict__ nodes, int64_t n_nodes) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const uint32_t x = (uint32_t)rec[e].x;
  const uint32_t j = x & kColMask;
  if ((int)j >= B) {
    int64_t node = (int)j < n_cols ? nodes[j] : n_nodes;
    if (node < 0 || node >= n_nodes) {      // invalid: no contribution (gather_codewords' zero row)
      node = n_nodes;
      rec[e].y = 0;
    }
    rec[e].x = (int)((x & ~kColMask) | ((uint32_t)B + (uint32_t)node));
  }
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
  if (t < ntasks) {
    // bit 31: the task's first row began in an earlier task (its partial is a
    // head for the fix-up), decided here so the walk needs no rowptr read
    int r = n_rows - 1;
    uint32_t head = 0;
    if (st < nnz) {
      r = upper_bound_i32(rowptr, n_rows, st) - 1;
      head = rowptr[r] < st ? kHeadBit : 0u;
    }
    task_row[t] = (int32_t)((uint32_t)r | head);
  }
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
    const int r = task_row[x] & kRowMask;
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
// Cache-policy bits (buffer instruction aux: 1 sc0, 2 nt, 16 sc1) of the
// record loads and the output-row stores; 0 = the default policy
#ifndef VQGNN_REC_AUX
#define VQGNN_REC_AUX 0
#endif
#ifndef VQGNN_OUT_AUX
#define VQGNN_OUT_AUX 0
#endif
// 1: the two-source walk issues a block's gathers at raised wave priority
// (as the codebook walk does); experiments builds only
#ifndef VQGNN_TASK_PRIO
#define VQGNN_TASK_PRIO 0
#endif
// the codebook walk's consume (fma chain, row stores) at this wave priority
// (0: not raised; experiments builds)
#ifndef VQGNN_CB_CONS_PRIO
#define VQGNN_CB_CONS_PRIO 0
#endif
typedef int v4i __attribute__((ext_vector_type(4)));

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

// GAT coefficient of one edge (convs.py:209-264, vq_softmax.py:33-57, the
// op order of gat_coef_kernel): exp(leaky(al[j] + ar[i])) * w, al / ar
// already divided by s per node as the reference does (convs.py:209-211)
__device__ __forceinline__ float gat_edge_coef(const TaskArgs& a, int e, uint32_t j, float w) {
  float x = __fadd_rn(a.al[j], a.ar[a.erow[e]]);
  x = x > 0.f ? x : __fmul_rn(x, a.slope);
  return __fmul_rn(expf(x), w);
}

// The four plan words a wave's walk starts from (its first task's first edge,
// and this lane's task's first / end edge and first row), read together --
// independent loads, one memory round trip -- and, by the persistent kernel,
// one unit ahead of the walk that uses them
struct UnitInfo {
  int wbase, e0, e1, row;
};

template <int G>
__device__ __forceinline__ UnitInfo unit_info(const TaskArgs& a, int wv, int nnz) {
  constexpr int TPW = 64 / G;
  const int t = wv * TPW + (int)((threadIdx.x & 63) / G);
  const int tw = min(wv * TPW, a.ntasks);           // task_start has ntasks + 1 entries
  const int tc = min(t, a.ntasks - 1);
  UnitInfo u;
  u.wbase = a.task_start[tw];
  const int s0 = a.task_start[max(tc, 0)], s1 = a.task_start[max(tc, 0) + 1];
  const int rw = a.task_row[max(tc, 0)];
  const bool tv = t < a.ntasks;
  u.e0 = tv ? s0 : nnz;
  u.e1 = tv ? s1 : nnz;
  u.row = tv ? rw : 0;
  return u;
}

// the edges a call covers: a call over the first n_rows rows of a larger CSR
// (the backward's transpose restricted to batch rows) covers [0, rowptr[n_rows])
__device__ __forceinline__ int call_nnz(const TaskArgs& a) { return min(a.nnz, a.rowptr[a.n_rows]); }

// G lanes per task (64 / G tasks per wave), NC float4 pieces per lane (piece
// i of lane k is float4 column G*i + k: a column tile of 4*G*NC floats), U
// edges per block.  PART (near path): the last column tile is partial (F/4
// not a multiple of G*NC): its lanes past F load nothing (an offset past the
// buffer range returns 0 without a memory access) instead of reading the
// next row
template <int G, int NC, int U, bool FAR, bool GAT, bool PART, bool CB = false>
__device__ __forceinline__ void task_walk(const TaskArgs& a, int wv, int nwaves, const UnitInfo& ui,
                                          int nnz) {
  static_assert(!CB || (NC == 1 && !FAR && !GAT && !PART), "CB: the near shape, one piece per lane");
  constexpr int TPW = 64 / G;
  const int lane = threadIdx.x & 63;
  const int g = lane / G, k = lane % G;
  const int t = wv * TPW + g;
  if (wv >= nwaves || wv * TPW >= a.ntasks) return;
  // the wave's records are addressed from its first task's first edge: 32-bit
  // buffer offsets cover any nnz < 2^31 (a wave spans at most 64 tasks)
  const int wbase = __builtin_amdgcn_readfirstlane(ui.wbase);
  if (wbase >= nnz) return;
  const bool tv = t < a.ntasks;
  const int e0 = tv ? min(ui.e0, nnz) : nnz;
  const bool valid = e0 < nnz;
  const int e1 = valid ? min(nnz, ui.e1) : e0;

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

  int r = valid ? (ui.row & kRowMask) : 0;
  bool head = valid && ((uint32_t)ui.row & kHeadBit);   // first row began in an earlier task

  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ubase, 0, FAR ? 0 : (int)a.span, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.rec + wbase), 0,
      (int)(uint32_t)min((int64_t)(a.nnz - wbase) * 8, (int64_t)0x7FFFFFFF), 0x00020000);
  // CB: the codes' buffer, this lane's branch code offset, its LDS column
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(
      CB ? (void*)a.codes : (void*)a.rec, 0, CB ? (int)a.codes_bytes : 0, 0x00020000);
  uint32_t lane_boff = 0, lane16 = 0, cb_m = 0;
  const char* cb_img = nullptr;
  if constexpr (CB) {
    cb_m = (uint32_t)a.cb_M;              // a code >= M reads the image's zero row M
    extern __shared__ __attribute__((aligned(16))) char cb_smem[];
    lane_boff = (uint32_t)((4 * c4base) / a.cb_D) * 2u;
    lane16 = (uint32_t)k * 16u;
    cb_img = cb_smem;
  }

  float4 acc[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  // output rows through a buffer resource when a store cache policy is set
  // (near path: row offsets below 4 GiB)
  const __amdgpu_buffer_rsrc_t rso =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.out, 0, (int)0xFFFFFFFFu, 0x00020000);

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
        int2, __builtin_amdgcn_raw_buffer_load_b64(rsr, (uint32_t)(e - wbase + k) * 8u, 0, VQGNN_REC_AUX));
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
    if constexpr (CB) {
      // X rows: the row's byte offset; codebook rows: 2^31 | the node's code
      // row offset (bit 31 pushes either offset out of the other's range)
      const uint32_t x = (uint32_t)rcur.x;
      const uint32_t j = x & kColMask;
      const bool s1 = (int)j < a.B;
      const uint32_t roff = s1 ? __umul24(x, a.ldxb) + a.offx
                               : 0x80000000u | __umul24(j - (uint32_t)a.B, a.ldcb);
      group_bcast<kAnd>((int)roff, bk.co, std::make_integer_sequence<int, U>{});
    } else if constexpr (!FAR) {
      const uint32_t x = (uint32_t)rcur.x;
      const bool s1 = (int)(x & kColMask) < a.B;
      const uint32_t roff = __umul24(x, s1 ? a.ldxb : a.ldx2b) +
                            (s1 ? a.offx : a.offx2 - (uint32_t)a.B * a.ldx2b);
      group_bcast<kAnd>((int)roff, bk.co, std::make_integer_sequence<int, U>{});
    }
    group_bcast<kAnd>(rcur.y, bk.cw, std::make_integer_sequence<int, U>{});
    if constexpr (CB) {
      // codes first (an X edge's offset is out of range: no access), then
      // the X rows, then -- once the codes are in -- the codewords from LDS;
      // lane k's float4 is column 4 (32 tile + k): branch (4 (32 tile + k)) / D
      // the block's loads at raised wave priority, so they are in flight
      // before other waves' fma chains take the issue port (codebook SpMM
      // 79.8-80.9 against 81.1-82.8 us, profiles/r06t_setprio_ab.txt)
      uint32_t cd[U];
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int u = 0; u < U; ++u)
        cd[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(
            rsc, ((uint32_t)bk.co[u] ^ 0x80000000u) + lane_boff, 0, 0);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (bk.co[u] >= 0)
          v[u][0] = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(rsx, (uint32_t)bk.co[u] + lane_off, 0, 0));
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (bk.co[u] < 0)
          v[u][0] = *reinterpret_cast<const float4*>(cb_img + min(cd[u] & 0xffffu, cb_m) * (16u * G) +
                                                     lane16);
      __builtin_amdgcn_s_setprio(0);
      return;
    }
    if constexpr (VQGNN_TASK_PRIO != 0) __builtin_amdgcn_s_setprio(1);
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
    if constexpr (VQGNN_TASK_PRIO != 0) __builtin_amdgcn_s_setprio(0);
  };
  auto consume = [&](int e, const Blk& bk, const float4 (&v)[U][NC]) {
    if constexpr (CB && VQGNN_CB_CONS_PRIO != 0) __builtin_amdgcn_s_setprio(VQGNN_CB_CONS_PRIO);
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
          if (pv[i] && !(a.dbg & 1)) {
            if constexpr (VQGNN_OUT_AUX != 0 && !FAR) {
              if (!head) {
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(v4i, acc[i]), rso,
                    (uint32_t)__umul24((uint32_t)r, a.ldob) + 16u * (uint32_t)(c4base + G * i), 0,
                    VQGNN_OUT_AUX);
              } else {
                *reinterpret_cast<float4*>(dst + 4 * (c4base + G * i)) = acc[i];
              }
            } else {
              *reinterpret_cast<float4*>(dst + 4 * (c4base + G * i)) = acc[i];
            }
          }
          acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const uint32_t skip = (x >> kSkipShift) & kSkipEsc;
        r = skip == kSkipEsc ? upper_bound_i32(a.rowptr, a.n_rows, e + u + 1) - 1
                             : r + 1 + (int)skip;
        head = false;
      }
    }
    if constexpr (CB && VQGNN_CB_CONS_PRIO != 0) __builtin_amdgcn_s_setprio(0);
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
#ifdef VQGNN_EXPERIMENTS
  // VQGNN_TASK_XCD: 1 contiguous eighths, 0 round-robin, C > 1 chunks of C
  // workgroups dealt to the XCDs in turn (XCD x: chunks x, x + 8, ...)
  int blk;
  if (a.xcd == 1) {
    blk = xcd_remap(blockIdx.x, gridDim.x);
  } else if (a.xcd > 1) {
    const int p = blockIdx.x, C = a.xcd, full = (int)gridDim.x / (8 * C) * (8 * C);
    const int local = p / 8;
    blk = p < full ? ((local / C) * 8 + p % 8) * C + local % C : p;
  } else {
    blk = (int)blockIdx.x;
  }
#else
  // XCD-contiguous eighths of the tasks (each XCD's L2 keeps its rows'
  // cluster), except for grids of 2^16 workgroups and more (> 33 M edges),
  // where the dispatcher's round-robin order balances the XCDs' mix of rows
  // (reddit layer 2: 4,072-4,093 against 4,348-4,374 us; arxiv, contiguous:
  // 74 against 106 us round-robin; profiles/r06n_task_xcd_chunks.txt)
  const int blk = gridDim.x >= kRoundRobinGrid ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
#endif
  const int wv = __builtin_amdgcn_readfirstlane(blk * (kTaskThreads / 64) + (threadIdx.x >> 6));
  const int nnz = call_nnz(a);
  task_walk<G, NC, U, FAR, GAT, PART>(a, wv, nwaves, unit_info<G>(a, wv, nnz), nnz);
}

// Codebook-source task kernel: persistent 16-wave workgroups (the LDS
// image leaves one per CU), one per CU and column tile; the workgroup stages
// its tile's codeword features -- image row m = the 4G columns of codeword
// m's branches (G float4 pieces: 512 B at G = 32), so lane k always reads
// banks 4k..4k+3 of its row: conflict-free within a task whatever the codes
// -- and its waves walk task groups round-robin.  Row M of the image is
// zeros (a code >= M reads it).  G = 32 (128-column tiles) serves M <= 319;
// G = 16 (64 columns) M <= 639, G = 8 (32 columns) M <= 1,279: narrower
// tiles fit larger codebooks, each tile walking every edge.
constexpr int kCbThreads = 1024;
constexpr size_t kCbLdsMax = 160 * 1024;
constexpr int kCbStage = (int)(kCbLdsMax / 16 / kCbThreads);   // image pieces per thread (10)

template <int G, int U, int NT = kCbThreads>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4)))
spmm_task_cb_kernel(TaskArgs a, int nunits) {
  extern __shared__ __attribute__((aligned(16))) char cb_smem[];
  const int tile = blockIdx.y;
  // every piece of this thread's share of the image in flight at once (at
  // most kCbStage float4 per thread: M x G <= 10,240), then the LDS writes:
  // a load-then-write loop waited one memory round trip per piece, eight of
  // them at M = 256 before any wave could walk.  Loads past the image repeat
  // its last piece.
  // (the tile's columns lie inside F: cb_lanes needs F % 4G == 0).  Image
  // row M is zeros: the walk reads a code >= M (invalid input) there.
  // (NT < kCbThreads, an experiments-build workgroup shape: several rounds)
  const int npc = (a.cb_M + 1) * G;
  // the first unit's plan words are requested before the image: their round
  // trip overlaps the staging loads' instead of following the barrier
  const int wave = threadIdx.x >> 6;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int stride = (int)gridDim.x * (NT / 64);
  const int nnz = call_nnz(a);
  int u0 = g * (NT / 64);
  UnitInfo cur = unit_info<G>(a, __builtin_amdgcn_readfirstlane(u0 + wave), nnz);
#pragma unroll
  for (int base = 0; base < kCbThreads * kCbStage; base += NT * kCbStage) {
    float4 v[kCbStage];
#pragma unroll
    for (int r = 0; r < kCbStage; ++r) {
      const int i = min(base + (int)threadIdx.x + r * NT, npc - 1);
      const int m = i / G, col = 4 * (tile * G + (i % G));
      const int b = col / a.cb_D, d = col % a.cb_D;
      v[r] = m < a.cb_M ? *reinterpret_cast<const float4*>(a.cbe + b * a.cb_bstride +
                                                            (int64_t)min(m, a.cb_M - 1) * a.cb_ldw + d)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // (unconditional writes: a piece past the image rewrites the last one with
    // its own value -- a branch here would let the compiler sink each load
    // into it, one wait per piece again)
#pragma unroll
    for (int r = 0; r < kCbStage; ++r) {
      const int i = min(base + (int)threadIdx.x + r * NT, npc - 1);
      *reinterpret_cast<float4*>(cb_smem + (size_t)i * 16) = v[r];
    }
  }
  __syncthreads();
  // the next unit's plan words are read while this unit is walked
  for (; u0 < nunits; u0 += stride) {
    const int wv = __builtin_amdgcn_readfirstlane(u0 + wave);
    const UnitInfo nxt = unit_info<G>(a, wv + stride, nnz);
    task_walk<G, 1, U, false, false, false, true>(a, wv, nunits, cur, nnz);
    cur = nxt;
  }
}

// lanes per task of the codebook-source walk for a codebook of M codewords
// over F columns: the widest tile whose LDS image fits (0: none)
static int cb_lanes(int F, int M) {
  for (int G = 32; G >= 8; G >>= 1)
    if (F % (4 * G) == 0 && (size_t)(M + 1) * G * 16 <= kCbLdsMax) return G;
  return 0;
}

// One wave per fix-up job.  A cut row: out[row] = tail[ts] + ... + tail[t-1]
// + head[t], in task order (loads 8 tasks ahead of the in-order adds); GAT
// sums the coefficient slot the same way, then normalises rows < norm_B.
// An empty row: zeros.  Rows at or past n_rows (a call over leading rows)
// are skipped.
template <bool GAT>
__device__ __forceinline__ void task_fixup_thread(const TaskArgs& a, int gtid) {
  // L lanes per job: 32 when a row (plus the GAT slot) fits 32 float4 pieces,
  // so a wave finishes two rows
  const int F4 = a.F >> 2;
  const int L = F4 <= 32 ? 32 : 64;          // (GAT's slot column F4 is skipped below)
  const int lane = gtid & (L - 1);
  const int w = gtid / L;
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

template <bool GAT>
__global__ void __launch_bounds__(256)
spmm_task_fixup_kernel(TaskArgs a) {
  task_fixup_thread<GAT>(a, blockIdx.x * 256 + threadIdx.x);
}

// The fix-up launch with the EMA finalize beside it (vqgnn_spmm_task_cb_fin):
// workgroups [0, nb) finalize branch blockIdx.x (ema_finalize.h, the body of
// vq_ema_finalize_kernel), the rest take the fix-up jobs.  Disjoint data: the
// finalize touches the slabs and the codebook state, the fix-up the carries
// and the output rows; the walk that read the codebook has finished.
__global__ void __launch_bounds__(kFinThreads)
spmm_fixup_fin_kernel(TaskArgs a, EmaFin f, int nb) {
  extern __shared__ float fin_cs[];          // [M]
  if ((int)blockIdx.x < nb) {
    ema_finalize_branch(f, blockIdx.x, threadIdx.x, fin_cs);
    return;
  }
  task_fixup_thread<false>(a, ((int)blockIdx.x - nb) * kFinThreads + threadIdx.x);
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
                     n_rows, (int)nnz, K, VQGNN_KNOB("VQGNN_TASK_SNAP", 1) ? K / 2 : 0, ntasks,
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
          (int64_t)n_rows * ldo * 4 < ((int64_t)1 << 32) && !path_env("VQGNN_SPMM_FAR", 0);
  if (*near) {
    a.ubase = reinterpret_cast<const char*>(lo);
    a.span = (uint32_t)(hi - lo);
    a.offx = (uint32_t)(x0 - lo);
    a.ldxb = (uint32_t)(ldx * 4);
    a.offx2 = nx2 > 0 ? (uint32_t)(y0 - lo) : 0;
    a.ldx2b = (uint32_t)(a.ldx2 * 4);
    a.ldob = (uint32_t)(ldo * 4);
  }
  a.dbg = VQGNN_KNOB("VQGNN_TASK_DBG", 0);
  a.xcd = VQGNN_KNOB("VQGNN_TASK_XCD", 1);
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

static void task_fixup_fin(const TaskArgs& a, const EmaFin& f, int nb, hipStream_t s) {
  const int nfix = a.n_jobs + a.n_empty;
  const int L = a.F / 4 <= 32 ? 32 : 64;     // lanes per fix-up job (task_fixup_thread)
  const int per = kFinThreads / L;
  const size_t lds = (size_t)f.M * sizeof(float);
  if (lds > 48 * 1024) {
    static std::once_flag once;
    std::call_once(once, [] { ema_fin_lds_attr((const void*)spmm_fixup_fin_kernel); });
  }
  hipLaunchKernelGGL(spmm_fixup_fin_kernel, dim3(nb + (nfix + per - 1) / per), dim3(kFinThreads),
                     lds, s, a, f, nb);
}

template <bool GAT>
static void task_launch(const TaskArgs& a, bool near, hipStream_t s) {
  if (a.nnz > 0) {
    const int F4 = a.F / 4;
    // lanes per task: VQGNN_TASK_G (8, 16 or 32; default 32); pieces per lane
    // so that one column tile covers min(F, 128) floats
    int G = VQGNN_KNOB("VQGNN_TASK_G", 32);
    G = G >= 32 ? 32 : (G >= 16 ? 16 : 8);
    int nc = 1;
    while (nc * G < F4 && nc * G * 4 < 128) nc *= 2;      // 4*G*nc floats <= 128
    const int tiles = (F4 + nc * G - 1) / (nc * G);
    const int Ue = VQGNN_KNOB("VQGNN_TASK_U", 16);
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

extern "C" int vqgnn_spmm_task_records_cb(int64_t* records, int64_t nnz, int32_t B,
                                          const int64_t* nodes, int32_t n_cols, int64_t n_nodes,
                                          vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(nnz >= 0 && nnz < (int64_t)1 << 31 && B >= 0 && n_cols >= B && n_nodes >= 0,
                "spmm_task_records_cb: bad arguments");
  VQGNN_REQUIRE(nnz == 0 || (records && (n_cols == B || nodes)),
                "spmm_task_records_cb: null pointer");
  VQGNN_REQUIRE((int64_t)B + n_nodes <= (int64_t)kColMask,
                "spmm_task_records_cb: B + %lld nodes exceed 2^26", (long long)n_nodes);
  if (nnz > 0 && n_cols > B)
    hipLaunchKernelGGL(task_remap_cb_kernel, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<int2*>(records), (int)nnz, B, n_cols, nodes,
                       n_nodes);
  return check_launch("spmm_task_records_cb");
}

extern "C" size_t vqgnn_spmm_task_cb_lds(int32_t M) {
  // bytes of the LDS image per column tile at the tile width M allows (any F
  // the width divides); 0 when no tile fits
  if (M <= 0) return 0;
  for (int G = 32; G >= 8; G >>= 1)       // M codeword rows + the zero row
    if ((size_t)(M + 1) * G * 16 <= kCbLdsMax) return (size_t)(M + 1) * G * 16;
  return 0;
}

// The shapes vqgnn_spmm_task_cb serves (its own checks below plus the near
// path of task_setup for X [B][ldx] and out [n_rows][ldo]); 0 -> use
// gather_codewords + vqgnn_spmm_task, which has a 64-bit far path.
static const char* cb_unsupported(int32_t n_rows, int32_t B, int64_t ldx, int32_t F, int64_t ldo,
                                  int64_t n_nodes, int64_t ldc, int32_t n_branches, int32_t M,
                                  int32_t D) {
  if (F <= 0 || F % 32 != 0) return "F must be a multiple of 32";
  if (D <= 0 || D % 4 != 0 || F % D != 0) return "D must be a multiple of 4 dividing F";
  if (F / D > n_branches) return "F / D code columns exceed the codebook's branches";
  if (M <= 0 || cb_lanes(F, M) == 0)
    return "M above the LDS image ((M + 1) x 16G bytes <= 160 KiB with 4G | F: M <= 319 at F % "
           "128 == 0, 639 at F % 64 == 0, 1279)";
  if (ldc < F / D || n_nodes < 0 || n_nodes >= (1 << 24) ||
      n_nodes * ldc * 2 >= ((int64_t)1 << 31) || ldc * 2 >= (1 << 24) ||
      (int64_t)B + n_nodes > (int64_t)kColMask)
    return "codes out of range";
  if (n_rows < 0 || n_rows >= (1 << 24) || B < 0 || B >= (1 << 24)) return "rows above 2^24";
  if (ldx < F || ldo < F || ldx * 4 >= (1 << 24) || ldo * 4 >= (1 << 24))
    return "leading dimension off the near path";
  if ((int64_t)(B > 0 ? B - 1 : 0) * ldx * 4 + (int64_t)F * 4 >= 0x7FFFFFF0ll)
    return "X above the 2 GiB near range";
  if ((int64_t)n_rows * ldo * 4 >= ((int64_t)1 << 32)) return "out above 4 GiB";
  if (path_env("VQGNN_SPMM_FAR", 0)) return "VQGNN_SPMM_FAR forces the 64-bit far path";
  return nullptr;
}

extern "C" int32_t vqgnn_spmm_task_cb_supported(int32_t n_rows, int32_t B, int64_t ldx, int32_t F,
                                                int64_t ldo, int64_t n_nodes, int64_t ldc,
                                                int32_t n_branches, int32_t M, int32_t D) {
  return cb_unsupported(n_rows, B, ldx, F, ldo, n_nodes, ldc, n_branches, M, D) ? 0 : 1;
}

static int spmm_task_cb_impl(const int32_t* rowptr, int32_t n_rows, int64_t nnz, int32_t B,
                             const float* X, int64_t ldx, int32_t F, const int16_t* codes,
                             int64_t ldc, int64_t n_nodes, const float* codewords, int64_t ldw,
                             int64_t bstride, int32_t n_branches, int32_t M, int32_t D, float* out,
                             int64_t ldo, const int32_t* plan, const int64_t* records_cb,
                             int32_t K, int32_t n_jobs, int32_t n_empty, void* workspace,
                             const vqgnn_ema_finalize_args* fin, vqgnn_stream_t stream,
                             int phases = 3) {
  // phases: 1 the walk, 2 the fix-up (+ finalize), 3 both (same checks either way)
  clear_error();
  EmaFin ef{};
  if (fin) {                                // checked before anything is launched
    const int frc = ema_fin_prepare(fin, &ef);
    if (frc != VQGNN_OK) return frc;
  }
  const char* why = cb_unsupported(n_rows, B, ldx, F, ldo, n_nodes, ldc, n_branches, M, D);
  VQGNN_REQUIRE(!why, "spmm_task_cb: %s (n_rows=%d B=%d F=%d D=%d M=%d branches=%d codes "
                "[%lld x %lld])", why ? why : "", n_rows, B, F, D, M, n_branches,
                (long long)n_nodes, (long long)ldc);
  TaskArgs a{};
  bool near = false;
  const int rc = task_setup(a, rowptr, n_rows, B, nnz, B, X, ldx, X, ldx, F, out, ldo, plan,
                            records_cb, K, n_jobs, n_empty, workspace, &near);
  if (rc != VQGNN_OK) return rc;
  VQGNN_REQUIRE(near, "spmm_task_cb: X and out must fit the 32-bit near path");
  VQGNN_REQUIRE(nnz == 0 || (codes && codewords), "spmm_task_cb: null pointer");
  VQGNN_REQUIRE(ldw >= D && ldw % 4 == 0 && bstride % 4 == 0 && ((uintptr_t)codewords & 15) == 0,
                "spmm_task_cb: codeword rows must be 16-byte aligned");
  a.codes = codes;
  a.codes_bytes = (uint32_t)(n_nodes * ldc * 2);
  a.ldcb = (uint32_t)(ldc * 2);
  a.cbe = codewords;
  a.cb_ldw = ldw;
  a.cb_bstride = bstride;
  a.cb_M = M;
  a.cb_D = D;
  hipStream_t s = as_stream(stream);
  if (nnz > 0 && (phases & 1)) {
    int G = cb_lanes(F, M);
    const size_t lds = (size_t)(M + 1) * G * 16;
    // U = 8 edges per block (96 VGPRs at G = 32); U = 12 measured the same
    // (77.6 against 77.7 us on the arxiv batch), U = 16 spills
    static const bool attr_set = [] {
      for (const void* f : {(const void*)spmm_task_cb_kernel<32, 8>,
                            (const void*)spmm_task_cb_kernel<16, 8>,
                            (const void*)spmm_task_cb_kernel<8, 8>})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCbLdsMax);
#ifdef VQGNN_EXPERIMENTS
      for (const void* f : {(const void*)spmm_task_cb_kernel<32, 8, 512>,
                            (const void*)spmm_task_cb_kernel<16, 8, 512>,
                            (const void*)spmm_task_cb_kernel<8, 8, 512>})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCbLdsMax);
#endif
      return true;
    }();
    (void)attr_set;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    const int tpw = 64 / G;                                  // tasks per wave
    const int nunits = (a.ntasks + tpw - 1) / tpw;
    int wgs = (nunits + kCbThreads / 64 - 1) / (kCbThreads / 64);
    wgs = wgs < cus ? wgs : cus;
#ifdef VQGNN_EXPERIMENTS
    // measurement knobs (overlap study): a narrower tile, 8-wave workgroups,
    // fewer workgroups per column tile
    const int g_env = path_env("VQGNN_CB_G", 0), nt_env = path_env("VQGNN_CB_NT", 0),
              wg_env = path_env("VQGNN_CB_WGS", 0);
    if (g_env && g_env < G && (g_env == 16 || g_env == 8)) G = g_env;
    if (nt_env == 512 || wg_env > 0) {
      const int nt = nt_env == 512 ? 512 : kCbThreads;
      const int tpw2 = 64 / G;
      const int nu = (a.ntasks + tpw2 - 1) / tpw2;
      int w2 = (nu + nt / 64 - 1) / (nt / 64);
      const int cap = wg_env > 0 ? wg_env : cus;
      w2 = w2 < cap ? w2 : cap;
      const size_t lds2 = (size_t)(M + 1) * G * 16;
      const dim3 grid2(w2, F / (4 * G));
#define CB_LAUNCH(GG, NN) \
      hipLaunchKernelGGL((spmm_task_cb_kernel<GG, 8, NN>), grid2, dim3(NN), lds2, s, a, nu)
      if (nt == 512) {
        if (G == 32) CB_LAUNCH(32, 512); else if (G == 16) CB_LAUNCH(16, 512); else CB_LAUNCH(8, 512);
      } else {
        if (G == 32) CB_LAUNCH(32, 1024); else if (G == 16) CB_LAUNCH(16, 1024); else CB_LAUNCH(8, 1024);
      }
#undef CB_LAUNCH
      goto walked;
    }
    {
      const int tpw2 = 64 / G;
      const int nu = (a.ntasks + tpw2 - 1) / tpw2;
      wgs = (nu + kCbThreads / 64 - 1) / (kCbThreads / 64);
      wgs = wgs < cus ? wgs : cus;
      const size_t lds2 = (size_t)(M + 1) * G * 16;
      const dim3 grid2(wgs, F / (4 * G));
      if (G == 32)
        hipLaunchKernelGGL((spmm_task_cb_kernel<32, 8>), grid2, dim3(kCbThreads), lds2, s, a, nu);
      else if (G == 16)
        hipLaunchKernelGGL((spmm_task_cb_kernel<16, 8>), grid2, dim3(kCbThreads), lds2, s, a, nu);
      else
        hipLaunchKernelGGL((spmm_task_cb_kernel<8, 8>), grid2, dim3(kCbThreads), lds2, s, a, nu);
      goto walked;
    }
#endif
    {
      const dim3 grid(wgs, F / (4 * G));
      if (G == 32)
        hipLaunchKernelGGL((spmm_task_cb_kernel<32, 8>), grid, dim3(kCbThreads), lds, s, a, nunits);
      else if (G == 16)
        hipLaunchKernelGGL((spmm_task_cb_kernel<16, 8>), grid, dim3(kCbThreads), lds, s, a, nunits);
      else
        hipLaunchKernelGGL((spmm_task_cb_kernel<8, 8>), grid, dim3(kCbThreads), lds, s, a, nunits);
    }
  }
#ifdef VQGNN_EXPERIMENTS
walked:
#endif
  if (!(phases & 2)) {
    // the walk alone: its fix-up comes later (vqgnn_spmm_task_cb_fixup)
  } else if (!fin) {
    task_fixup<false>(a, s);
  } else if (!ef.split) {
    task_fixup_fin(a, ef, fin->nb, s);      // one launch: fix-up + finalize
  } else {                                  // the finalize's two-kernel form
    task_fixup<false>(a, s);
    const int frc = ema_fin_run(ef, fin->nb, s);
    if (frc != VQGNN_OK) return frc;
  }
  return check_launch("spmm_task_cb");
}

extern "C" int vqgnn_spmm_task_cb(const int32_t* rowptr, int32_t n_rows, int64_t nnz, int32_t B,
                                  const float* X, int64_t ldx, int32_t F, const int16_t* codes,
                                  int64_t ldc, int64_t n_nodes, const float* codewords,
                                  int64_t ldw, int64_t bstride, int32_t n_branches, int32_t M,
                                  int32_t D, float* out, int64_t ldo, const int32_t* plan,
                                  const int64_t* records_cb, int32_t K, int32_t n_jobs,
                                  int32_t n_empty, void* workspace, vqgnn_stream_t stream) {
  return spmm_task_cb_impl(rowptr, n_rows, nnz, B, X, ldx, F, codes, ldc, n_nodes, codewords, ldw,
                           bstride, n_branches, M, D, out, ldo, plan, records_cb, K, n_jobs,
                           n_empty, workspace, nullptr, stream);
}

extern "C" int vqgnn_spmm_task_cb_fin(const int32_t* rowptr, int32_t n_rows, int64_t nnz,
                                      int32_t B, const float* X, int64_t ldx, int32_t F,
                                      const int16_t* codes, int64_t ldc, int64_t n_nodes,
                                      const float* codewords, int64_t ldw, int64_t bstride,
                                      int32_t n_branches, int32_t M, int32_t D, float* out,
                                      int64_t ldo, const int32_t* plan, const int64_t* records_cb,
                                      int32_t K, int32_t n_jobs, int32_t n_empty,
                                      void* workspace, const vqgnn_ema_finalize_args* fin,
                                      vqgnn_stream_t stream) {
  return spmm_task_cb_impl(rowptr, n_rows, nnz, B, X, ldx, F, codes, ldc, n_nodes, codewords, ldw,
                           bstride, n_branches, M, D, out, ldo, plan, records_cb, K, n_jobs,
                           n_empty, workspace, fin, stream);
}

// The walk and the fix-up as two calls (include/vqgnn.h §6b): the walk can
// run on a second stream beside the VQ update, the fix-up -- with the
// update's EMA finalize -- after both.  The same arguments to both calls.
extern "C" int vqgnn_spmm_task_cb_walk(const int32_t* rowptr, int32_t n_rows, int64_t nnz,
                                       int32_t B, const float* X, int64_t ldx, int32_t F,
                                       const int16_t* codes, int64_t ldc, int64_t n_nodes,
                                       const float* codewords, int64_t ldw, int64_t bstride,
                                       int32_t n_branches, int32_t M, int32_t D, float* out,
                                       int64_t ldo, const int32_t* plan, const int64_t* records_cb,
                                       int32_t K, int32_t n_jobs, int32_t n_empty,
                                       void* workspace, vqgnn_stream_t stream) {
  return spmm_task_cb_impl(rowptr, n_rows, nnz, B, X, ldx, F, codes, ldc, n_nodes, codewords, ldw,
                           bstride, n_branches, M, D, out, ldo, plan, records_cb, K, n_jobs,
                           n_empty, workspace, nullptr, stream, 1);
}

extern "C" int vqgnn_spmm_task_cb_fixup(const int32_t* rowptr, int32_t n_rows, int64_t nnz,
                                        int32_t B, const float* X, int64_t ldx, int32_t F,
                                        const int16_t* codes, int64_t ldc, int64_t n_nodes,
                                        const float* codewords, int64_t ldw, int64_t bstride,
                                        int32_t n_branches, int32_t M, int32_t D, float* out,
                                        int64_t ldo, const int32_t* plan,
                                        const int64_t* records_cb, int32_t K, int32_t n_jobs,
                                        int32_t n_empty, void* workspace,
                                        const vqgnn_ema_finalize_args* fin,
                                        vqgnn_stream_t stream) {
  return spmm_task_cb_impl(rowptr, n_rows, nnz, B, X, ldx, F, codes, ldc, n_nodes, codewords, ldw,
                           bstride, n_branches, M, D, out, ldo, plan, records_cb, K, n_jobs,
                           n_empty, workspace, fin, stream, 2);
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

