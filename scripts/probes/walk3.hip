// Probe (round 6): "split-pass" codebook-source SpMM walk.
//
// One wave per task, every edge wave-uniform: 64 lanes x float2 cover a
// 128-column tile.  A task holds at most R rows; its edges are split into an
// X stream (columns < B, gathered rows) and a codebook stream (columns >= B,
// codeword rows from an LDS image), each in row order.  Pass 1 walks the X
// stream and parks each row's partial in a register slot (dynamic index),
// pass 2 walks the codebook stream into a second set of slots, then each row
// is stored as X partial + codebook partial.  Records (byte offset of the source row / code row,
// weight) are read by scalar loads and used as soffset / SGPR operands: no
// per-edge broadcast, no per-edge X / codebook branch.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

namespace w3 {

struct Args {
  const char* xbase;
  uint32_t xbytes;
  const char* cbase;
  uint32_t cbytes;
  const float* cbe;
  long long cb_ldw, cb_bstride;
  int M, D;
  float* out;
  uint32_t ldob;
  float* carry;
  int cf;
  int ntasks;
  uint32_t xpad, cpad;   // first pad record of each stream (valid offsets, never summed)
};

constexpr int kThreads = 1024;
constexpr int kStage = 10;

__device__ __forceinline__ int xcd_remap(int orig, int n) {
  const int q = n / 8, r = n % 8;
  const int xcd = orig % 8, local = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

template <int U>
struct alignas(64) Blk {
  int2 r[U];
};

template <int R>
struct Slots {
  typedef float V __attribute__((ext_vector_type(2 * R)));
  V v;
};

template <int U, int R, bool PF = false>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
walk3_kernel(const uint32_t* __restrict__ meta, const int2* __restrict__ xrec,
             const int2* __restrict__ crec, Args a) {
  extern __shared__ __attribute__((aligned(16))) char img[];
  const int tile = blockIdx.y;
  {
    const int npc = a.M * 32;
    float4 v[kStage];
#pragma unroll
    for (int r = 0; r < kStage; ++r) {
      const int i = min((int)threadIdx.x + r * kThreads, npc - 1);
      const int m = i / 32, col = 4 * (tile * 32 + (i % 32));
      const int b = col / a.D, d = col % a.D;
      v[r] = *reinterpret_cast<const float4*>(a.cbe + b * a.cb_bstride + (long long)m * a.cb_ldw + d);
    }
#pragma unroll
    for (int r = 0; r < kStage; ++r) {
      const int i = min((int)threadIdx.x + r * kThreads, npc - 1);
      *reinterpret_cast<float4*>(img + (size_t)i * 16) = v[r];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t vx = (uint32_t)tile * 512u + (uint32_t)lane * 8u;
  const uint32_t vc = ((uint32_t)tile * 32u + ((uint32_t)lane >> 1)) * 2u;
  const uint32_t vl = (uint32_t)lane * 8u;
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xbase, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.cbase, 0, (int)a.cbytes, 0x00020000);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int stride = (int)gridDim.x * (kThreads / 64);
  for (int t0 = g * (kThreads / 64) + wave; t0 < a.ntasks; t0 += stride) {
    const int t = __builtin_amdgcn_readfirstlane(t0);
    const uint32_t* m = meta + (size_t)t * 16;
    const uint32_t xs = m[0], nx = m[1], cs = m[2], nc = m[3];
    const uint64_t xm = (uint64_t)m[4] | ((uint64_t)m[5] << 32);
    const uint64_t cm = (uint64_t)m[6] | ((uint64_t)m[7] << 32);
    const uint32_t xsl = m[8], csl = m[9], r0 = m[10], nrows = m[11], fl = m[12];
    Slots<R> sl, sc;     // X partials, codebook partials (rows without edges of a kind: 0)
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) {
      sl.v[i] = 0.f;
      sc.v[i] = 0.f;
    }
    // ---- pass 1: X stream (full blocks, then the tail) ----
    {
      float ax = 0.f, ay = 0.f;
      uint32_t k = 0;
      auto xblock = [&](uint32_t b0, uint32_t rem, auto tail, const Blk<U>& rb) {
        constexpr bool TAIL = decltype(tail)::value;
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (!TAIL || (uint32_t)u < rem)
            v[u] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsx, vx, rb.r[u].x, 0));
        const uint32_t bm = (uint32_t)(xm >> b0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (!TAIL || (uint32_t)u < rem) {
            const float w = __int_as_float(rb.r[u].y);
            ax = fmaf(w, v[u].x, ax);
            ay = fmaf(w, v[u].y, ay);
            if ((bm >> u) & 1u) {
              const uint32_t s = (xsl >> (4 * k)) & 15u;
              sl.v[2 * s] = ax;
              sl.v[2 * s + 1] = ay;
              ax = 0.f;
              ay = 0.f;
              ++k;
            }
          }
        }
      };
      uint32_t b0 = 0;
      // PF: the next block's records are read while this block's rows are
      // gathered (an explicit lgkmcnt(0) first: scalar loads return out of
      // order, so the wait for this block's records must not cover them)
      Blk<U> rcur = *reinterpret_cast<const Blk<U>*>(xrec + xs);
      for (; b0 + U <= nx; b0 += U) {
        if constexpr (PF) {
          __builtin_amdgcn_s_waitcnt(0xc07f);
          const Blk<U> rn = *reinterpret_cast<const Blk<U>*>(xrec + xs + b0 + U);
          xblock(b0, U, std::false_type{}, rcur);
          rcur = rn;
        } else {
          xblock(b0, U, std::false_type{}, *reinterpret_cast<const Blk<U>*>(xrec + xs + b0));
        }
      }
      if (b0 < nx) {
        if constexpr (PF) xblock(b0, nx - b0, std::true_type{}, rcur);
        else xblock(b0, nx - b0, std::true_type{}, *reinterpret_cast<const Blk<U>*>(xrec + xs + b0));
      }
    }
    // ---- pass 2: codebook stream, into its own slots ----
    {
      float ax = 0.f, ay = 0.f;
      uint32_t k = 0;
      auto cblock = [&](uint32_t b0, uint32_t rem, auto tail, const Blk<U>& rb) {
        constexpr bool TAIL = decltype(tail)::value;
        uint32_t cd[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (!TAIL || (uint32_t)u < rem)
            cd[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rsc, vc, rb.r[u].x, 0);
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (!TAIL || (uint32_t)u < rem)
            v[u] = *reinterpret_cast<const float2*>(img + ((cd[u] & 0xffffu) << 9) + vl);
        const uint32_t bm = (uint32_t)(cm >> b0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (!TAIL || (uint32_t)u < rem) {
            const float w = __int_as_float(rb.r[u].y);
            ax = fmaf(w, v[u].x, ax);
            ay = fmaf(w, v[u].y, ay);
            if ((bm >> u) & 1u) {
              const uint32_t s = (csl >> (4 * k)) & 15u;
              sc.v[2 * s] = ax;
              sc.v[2 * s + 1] = ay;
              ax = 0.f;
              ay = 0.f;
              ++k;
            }
          }
        }
      };
      uint32_t b0 = 0;
      Blk<U> rcur = *reinterpret_cast<const Blk<U>*>(crec + cs);
      for (; b0 + U <= nc; b0 += U) {
        if constexpr (PF) {
          __builtin_amdgcn_s_waitcnt(0xc07f);
          const Blk<U> rn = *reinterpret_cast<const Blk<U>*>(crec + cs + b0 + U);
          cblock(b0, U, std::false_type{}, rcur);
          rcur = rn;
        } else {
          cblock(b0, U, std::false_type{}, *reinterpret_cast<const Blk<U>*>(crec + cs + b0));
        }
      }
      if (b0 < nc) {
        if constexpr (PF) cblock(b0, nc - b0, std::true_type{}, rcur);
        else cblock(b0, nc - b0, std::true_type{}, *reinterpret_cast<const Blk<U>*>(crec + cs + b0));
      }
    }
    // ---- rows out ----
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if ((uint32_t)s < nrows) {
        char* dst;
        if ((uint32_t)s == nrows - 1 && (fl & 2u))
          dst = reinterpret_cast<char*>(a.carry + ((size_t)t * 2 + 1) * a.cf);
        else if (s == 0 && (fl & 1u))
          dst = reinterpret_cast<char*>(a.carry + (size_t)t * 2 * a.cf);
        else
          dst = reinterpret_cast<char*>(a.out) + (size_t)(r0 + s) * a.ldob;
        *reinterpret_cast<float2*>(dst + vx) =
            make_float2(__fadd_rn(sl.v[2 * s], sc.v[2 * s]), __fadd_rn(sl.v[2 * s + 1], sc.v[2 * s + 1]));
      }
    }
  }
}


// ---- walk4: the same split streams, software-pipelined ----------------------
// A task's X and codebook streams advance together in steps of U edges each
// (an X block and a codebook block per step).  While step s is consumed
// (codeword reads from LDS, fma chains, row ends into the slots) the loads of
// the next step -- of this task or of the wave's next task -- are already in
// flight, and a task's rows are stored only after the next task's first loads
// were issued (stores count in vmcnt too).  Records of the next step are read
// by scalar loads one step ahead.
struct Meta {
  uint32_t xs, nx, cs, nc, xm0, xm1, cm0, cm1, xsl, csl, r0, nrows, fl;
};

__device__ __forceinline__ Meta load_meta(const uint32_t* __restrict__ meta, int t) {
  const uint32_t* m = meta + (size_t)t * 16;
  Meta r;
  r.xs = m[0]; r.nx = m[1]; r.cs = m[2]; r.nc = m[3];
  r.xm0 = m[4]; r.xm1 = m[5]; r.cm0 = m[6]; r.cm1 = m[7];
  r.xsl = m[8]; r.csl = m[9]; r.r0 = m[10]; r.nrows = m[11]; r.fl = m[12];
  return r;
}

template <int U>
struct Stage {
  float2 vx[U];
  uint32_t cd[U];
};

template <int U>
struct Recs {
  Blk<U> x, c;
};

template <int U, int R, int NT>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT / 256)))
walk4_kernel(const uint32_t* __restrict__ meta, const int2* __restrict__ xrec,
             const int2* __restrict__ crec, Args a) {
  extern __shared__ __attribute__((aligned(16))) char img[];
  const int tile = blockIdx.y;
  {
    const int npc = a.M * 32;
    constexpr int kSt = kStage * kThreads / NT;
    float4 v[kSt];
#pragma unroll
    for (int r = 0; r < kSt; ++r) {
      const int i = min((int)threadIdx.x + r * NT, npc - 1);
      const int m = i / 32, col = 4 * (tile * 32 + (i % 32));
      const int b = col / a.D, d = col % a.D;
      v[r] = *reinterpret_cast<const float4*>(a.cbe + b * a.cb_bstride + (long long)m * a.cb_ldw + d);
    }
#pragma unroll
    for (int r = 0; r < kSt; ++r) {
      const int i = min((int)threadIdx.x + r * NT, npc - 1);
      *reinterpret_cast<float4*>(img + (size_t)i * 16) = v[r];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t vx = (uint32_t)tile * 512u + (uint32_t)lane * 8u;
  const uint32_t vc = ((uint32_t)tile * 32u + ((uint32_t)lane >> 1)) * 2u;
  const uint32_t vl = (uint32_t)lane * 8u;
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xbase, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.cbase, 0, (int)a.cbytes, 0x00020000);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int stride = (int)gridDim.x * (NT / 64);
  int t = g * (NT / 64) + wave;
  if (t >= a.ntasks) return;
  t = __builtin_amdgcn_readfirstlane(t);

  auto nsteps_of = [&](const Meta& m) {
    const uint32_t a1 = (m.nx + U - 1) / U, a2 = (m.nc + U - 1) / U;
    return a1 > a2 ? a1 : a2;
  };
  auto load_recs = [&](const Meta& m, uint32_t st) {
    Recs<U> r;
    r.x = *reinterpret_cast<const Blk<U>*>(xrec + m.xs + st * U);
    r.c = *reinterpret_cast<const Blk<U>*>(crec + m.cs + st * U);
    return r;
  };
  // every step issues exactly U code loads and U row loads (records past a
  // task's stream are other tasks' or pad records: valid offsets whose data
  // is never summed), so the wait counts are static
  auto issue = [&](const Recs<U>& r, Stage<U>& sg) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      sg.cd[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rsc, vc, r.c.r[u].x, 0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      sg.vx[u] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsx, vx, r.x.r[u].x, 0));
  };
  auto load_recs_at = [&](uint32_t xo, uint32_t co) {
    Recs<U> r;
    r.x = *reinterpret_cast<const Blk<U>*>(xrec + xo);
    r.c = *reinterpret_cast<const Blk<U>*>(crec + co);
    return r;
  };

  Slots<R> sl, sc;
#pragma unroll
  for (int i = 0; i < 2 * R; ++i) {
    sl.v[i] = 0.f;
    sc.v[i] = 0.f;
  }
  float axx = 0.f, axy = 0.f, acx = 0.f, acy = 0.f;
  uint32_t kx = 0, kc = 0;

  auto consume = [&](const Meta& m, uint32_t st, const Recs<U>& r, const Stage<U>& sg) {
    const uint32_t e0 = st * U;
    const uint32_t remc = m.nc > e0 ? m.nc - e0 : 0u;
    const uint32_t remx = m.nx > e0 ? m.nx - e0 : 0u;
    float2 vcw[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      vcw[u] = *reinterpret_cast<const float2*>(img + ((sg.cd[u] & 0xffffu) << 9) + vl);
    const uint64_t xm = (uint64_t)m.xm0 | ((uint64_t)m.xm1 << 32);
    const uint64_t cm = (uint64_t)m.cm0 | ((uint64_t)m.cm1 << 32);
    const uint32_t bx = (uint32_t)(xm >> e0), bc = (uint32_t)(cm >> e0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if ((uint32_t)u < remx) {
        const float w = __int_as_float(r.x.r[u].y);
        axx = fmaf(w, sg.vx[u].x, axx);
        axy = fmaf(w, sg.vx[u].y, axy);
        if ((bx >> u) & 1u) {
          const uint32_t s = (m.xsl >> (4 * kx)) & 15u;
          sl.v[2 * s] = axx;
          sl.v[2 * s + 1] = axy;
          axx = 0.f;
          axy = 0.f;
          ++kx;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if ((uint32_t)u < remc) {
        const float w = __int_as_float(r.c.r[u].y);
        acx = fmaf(w, vcw[u].x, acx);
        acy = fmaf(w, vcw[u].y, acy);
        if ((bc >> u) & 1u) {
          const uint32_t s = (m.csl >> (4 * kc)) & 15u;
          sc.v[2 * s] = acx;
          sc.v[2 * s + 1] = acy;
          acx = 0.f;
          acy = 0.f;
          ++kc;
        }
      }
    }
  };
  auto store_rows = [&](const Meta& m, int tt) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if ((uint32_t)s < m.nrows) {
        char* dst;
        if ((uint32_t)s == m.nrows - 1 && (m.fl & 2u))
          dst = reinterpret_cast<char*>(a.carry + ((size_t)tt * 2 + 1) * a.cf);
        else if (s == 0 && (m.fl & 1u))
          dst = reinterpret_cast<char*>(a.carry + (size_t)tt * 2 * a.cf);
        else
          dst = reinterpret_cast<char*>(a.out) + (size_t)(m.r0 + s) * a.ldob;
        *reinterpret_cast<float2*>(dst + vx) =
            make_float2(__fadd_rn(sl.v[2 * s], sc.v[2 * s]), __fadd_rn(sl.v[2 * s + 1], sc.v[2 * s + 1]));
      }
    }
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) {
      sl.v[i] = 0.f;
      sc.v[i] = 0.f;
    }
    kx = 0;
    kc = 0;
  };

  Meta mc = load_meta(meta, t);
  int tn = t + stride;
  // past the wave's last task: an empty task reading pad records
  auto meta_or_pad = [&](int tt) {
    Meta m;
    if (tt < a.ntasks) {
      m = load_meta(meta, tt);
    } else {
      m = Meta{};
      m.xs = a.xpad;
      m.cs = a.cpad;
    }
    return m;
  };
  Meta mn = meta_or_pad(tn);
  uint32_t s = 0, ns = nsteps_of(mc);
  Recs<U> rc = load_recs_at(mc.xs, mc.cs);
  Stage<U> A, B;
  issue(rc, A);
  // one step: issue the next step's loads into nxt (the next task's first
  // step after a task's last: scalar selects, no branch), consume cur, and
  // after a task's last step store its rows; false: the wave is done
  auto step = [&](Stage<U>& cur, Stage<U>& nxt) -> bool {
    const bool last = s + 1 >= ns;
    const uint32_t xo = last ? mn.xs : mc.xs + (s + 1) * U;
    const uint32_t co = last ? mn.cs : mc.cs + (s + 1) * U;
    const Recs<U> rn = load_recs_at(xo, co);
    issue(rn, nxt);
    consume(mc, s, rc, cur);
    rc = rn;
    if (last) {
      store_rows(mc, t);
      if (tn >= a.ntasks) return false;
      t = tn;
      mc = mn;
      tn += stride;
      mn = meta_or_pad(tn);
      s = 0;
      ns = nsteps_of(mc);
    } else {
      ++s;
    }
    return true;
  };
  while (step(A, B) && step(B, A)) {
  }
}


// ---- walk5: the split streams, two edges per gather instruction ------------
// One task per wave; a step takes records 2j (lanes 0-31) and 2j+1 (lanes
// 32-63) of a stream, each half a float4 per lane (128 columns), so one
// buffer_load_dwordx4 gathers two rows.  Lane l of the task's record vector
// holds record 2l (l < 32) or 2(l-32)+1 (l >= 32): a ds_swizzle broadcast
// within each 32-lane half hands step j's records to its half.  Each half
// keeps its own partial (even / odd records); at a row end the halves are
// added through one v_permlane32_swap (both halves get the same sum) and the
// row is parked in a slot as a float2 per lane (lane (h, k): columns
// 4k + 2h, 4k + 2h + 1).
template <int U, int R>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
walk5_kernel(const uint32_t* __restrict__ meta, const int2* __restrict__ xrec,
             const int2* __restrict__ crec, Args a) {
  extern __shared__ __attribute__((aligned(16))) char img[];
  const int tile = blockIdx.y;
  {
    const int npc = a.M * 32;
    float4 v[kStage];
#pragma unroll
    for (int r = 0; r < kStage; ++r) {
      const int i = min((int)threadIdx.x + r * kThreads, npc - 1);
      const int m = i / 32, col = 4 * (tile * 32 + (i % 32));
      const int b = col / a.D, d = col % a.D;
      v[r] = *reinterpret_cast<const float4*>(a.cbe + b * a.cb_bstride + (long long)m * a.cb_ldw + d);
    }
#pragma unroll
    for (int r = 0; r < kStage; ++r) {
      const int i = min((int)threadIdx.x + r * kThreads, npc - 1);
      *reinterpret_cast<float4*>(img + (size_t)i * 16) = v[r];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, k = lane & 31;
  const uint32_t vxb = (uint32_t)tile * 512u + (uint32_t)k * 16u;        // X row byte offset
  const uint32_t vcb = ((uint32_t)tile * 32u + (uint32_t)k) * 2u;         // code byte offset
  const uint32_t vlb = (uint32_t)k * 16u;                                  // image row byte offset
  const uint32_t vob = (uint32_t)tile * 512u + (uint32_t)(k * 16 + h * 8); // output float2
  const uint32_t gl = lane < 32 ? 2u * lane : 2u * (lane - 32) + 1u;       // record of this lane
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xbase, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.cbase, 0, (int)a.cbytes, 0x00020000);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int stride = (int)gridDim.x * (kThreads / 64);
  typedef float V2 __attribute__((ext_vector_type(2 * R)));
  for (int t0 = g * (kThreads / 64) + wave; t0 < a.ntasks; t0 += stride) {
    const int t = __builtin_amdgcn_readfirstlane(t0);
    const uint32_t* m = meta + (size_t)t * 16;
    const uint32_t xs = m[0], nx = m[1], cs = m[2], nc = m[3];
    const uint64_t xm = (uint64_t)m[4] | ((uint64_t)m[5] << 32);
    const uint64_t cm = (uint64_t)m[6] | ((uint64_t)m[7] << 32);
    const uint32_t xsl = m[8], csl = m[9], r0 = m[10], nrows = m[11], fl = m[12];
    const int2 rx = xrec[xs + gl];
    const int2 rcb = crec[cs + gl];
    V2 sx, sc;
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) {
      sx[i] = 0.f;
      sc[i] = 0.f;
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t kk = 0;
    // a row end: halves summed (v_permlane32_swap), parked in slot nib(kk)
    auto row_end = [&](V2& sl, uint32_t nibs) {
      const auto px = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc.x), __float_as_uint(acc.x), false, false);
      const auto py = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc.y), __float_as_uint(acc.y), false, false);
      const auto pz = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc.z), __float_as_uint(acc.z), false, false);
      const auto pw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc.w), __float_as_uint(acc.w), false, false);
      const float sxv = __fadd_rn(__uint_as_float(px[0]), __uint_as_float(px[1]));
      const float syv = __fadd_rn(__uint_as_float(py[0]), __uint_as_float(py[1]));
      const float szv = __fadd_rn(__uint_as_float(pz[0]), __uint_as_float(pz[1]));
      const float swv = __fadd_rn(__uint_as_float(pw[0]), __uint_as_float(pw[1]));
      const uint32_t s = (nibs >> (4 * kk)) & 15u;
      sl[2 * s] = h ? szv : sxv;
      sl[2 * s + 1] = h ? swv : syv;
      acc = make_float4(0.f, 0.f, 0.f, 0.f);
      ++kk;
    };
    auto fma4 = [&](const float4& v, float w) {
      acc.x = fmaf(w, v.x, acc.x);
      acc.y = fmaf(w, v.y, acc.y);
      acc.z = fmaf(w, v.z, acc.z);
      acc.w = fmaf(w, v.w, acc.w);
    };
    // one stream: nsteps = ceil(n / 2) steps in groups of U, fully unrolled
    // over the 32 steps a 64-record stream can hold
    auto walk = [&](const int2 rr, uint32_t n, uint64_t em, uint32_t nibs, V2& sl, auto cb) {
      constexpr bool CB = decltype(cb)::value;
      const uint32_t nst = (n + 1) >> 1;
      kk = 0;
      acc = make_float4(0.f, 0.f, 0.f, 0.f);
      // one group of U steps, step indices compile-time (swizzle immediates)
      auto group = [&]<int G, int... Us>(std::integer_sequence<int, Us...>) {
        float4 v[U];
        float wv[U];
        uint32_t so[U];
        ((so[Us] = (uint32_t)__builtin_amdgcn_ds_swizzle(rr.x, (G * U + Us) << 5)), ...);
        ((wv[Us] = __int_as_float(__builtin_amdgcn_ds_swizzle(rr.y, (G * U + Us) << 5))), ...);
        // every step of the group loads (no branch around a load: the wait
        // counts stay static); steps past the stream re-read step G*U's row
        // (an L1 hit) and are never summed
#pragma unroll
        for (int u = 1; u < U; ++u)
          if ((uint32_t)(G * U + u) >= nst) so[u] = so[0];
        if constexpr (CB) {
          uint32_t cd[U];
#pragma unroll
          for (int u = 0; u < U; ++u)
            cd[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rsc, so[u] + vcb, 0, 0);
#pragma unroll
          for (int u = 0; u < U; ++u)
            v[u] = *reinterpret_cast<const float4*>(img + ((cd[u] & 0xffffu) << 9) + vlb);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u)
            v[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsx, so[u] + vxb, 0, 0));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = G * U + u;
          if ((uint32_t)j < nst) {
            const bool ev = (em >> (2 * j)) & 1u;           // record 2j ends its row
            const bool od = (em >> (2 * j + 1)) & 1u;       // record 2j + 1 ends its row
            const bool one = (uint32_t)(2 * j + 1) >= n;    // no record 2j + 1
            if (!ev && !one) {
              fma4(v[u], wv[u]);
              if (od) row_end(sl, nibs);
            } else {
              if (h == 0) fma4(v[u], wv[u]);
              if (ev) row_end(sl, nibs);
              if (!one) {
                if (h == 1) fma4(v[u], wv[u]);
                if (od) row_end(sl, nibs);
              }
            }
          }
        }
      };
      auto groups = [&]<int... Gs>(std::integer_sequence<int, Gs...>) {
        // stop after the group holding the last step
        (void)((((uint32_t)(Gs * U) < nst) ? (group.template operator()<Gs>(std::make_integer_sequence<int, U>{}), true)
                                           : false) && ...);
      };
      groups(std::make_integer_sequence<int, 32 / U>{});
    };
    walk(rx, nx, xm, xsl, sx, std::false_type{});
    walk(rcb, nc, cm, csl, sc, std::true_type{});
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if ((uint32_t)s < nrows) {
        char* dst;
        if ((uint32_t)s == nrows - 1 && (fl & 2u))
          dst = reinterpret_cast<char*>(a.carry + ((size_t)t * 2 + 1) * a.cf);
        else if (s == 0 && (fl & 1u))
          dst = reinterpret_cast<char*>(a.carry + (size_t)t * 2 * a.cf);
        else
          dst = reinterpret_cast<char*>(a.out) + (size_t)(r0 + s) * a.ldob;
        *reinterpret_cast<float2*>(dst + vob) =
            make_float2(__fadd_rn(sx[2 * s], sc[2 * s]), __fadd_rn(sx[2 * s + 1], sc[2 * s + 1]));
      }
    }
  }
}


// ---- walk6: walk3 with its records in VGPRs --------------------------------
// A task's meta (16 dwords) and its two record streams (<= 64 records each)
// are vector loads, lane i holding dword / record i, issued one task ahead
// (the meta two tasks ahead: the records' addresses come from it), so no
// scalar-memory round trip sits in a task; a block's offsets and weights are
// read into SGPRs by v_readlane.  PIPE: a block's loads are issued before the
// previous block of the same stream is consumed.
template <int U, int R, bool PIPE, bool ALWAYS = false>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
walk6_kernel(const uint32_t* __restrict__ meta, const int2* __restrict__ xrec,
             const int2* __restrict__ crec, Args a) {
  extern __shared__ __attribute__((aligned(16))) char img[];
  const int tile = blockIdx.y;
  {
    const int npc = a.M * 32;
    float4 v[kStage];
#pragma unroll
    for (int r = 0; r < kStage; ++r) {
      const int i = min((int)threadIdx.x + r * kThreads, npc - 1);
      const int m = i / 32, col = 4 * (tile * 32 + (i % 32));
      const int b = col / a.D, d = col % a.D;
      v[r] = *reinterpret_cast<const float4*>(a.cbe + b * a.cb_bstride + (long long)m * a.cb_ldw + d);
    }
#pragma unroll
    for (int r = 0; r < kStage; ++r) {
      const int i = min((int)threadIdx.x + r * kThreads, npc - 1);
      *reinterpret_cast<float4*>(img + (size_t)i * 16) = v[r];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t vx = (uint32_t)tile * 512u + (uint32_t)lane * 8u;
  const uint32_t vc = ((uint32_t)tile * 32u + ((uint32_t)lane >> 1)) * 2u;
  const uint32_t vl = (uint32_t)lane * 8u;
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xbase, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.cbase, 0, (int)a.cbytes, 0x00020000);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int stride = (int)gridDim.x * (kThreads / 64);
  int t = g * (kThreads / 64) + wave;
  if (t >= a.ntasks) return;
  t = __builtin_amdgcn_readfirstlane(t);
  // lane i < 16: dword i of a task's meta (a task past the end: 0s)
  auto load_meta_v = [&](int tt) -> uint32_t {
    return tt < a.ntasks && lane < 16 ? meta[(size_t)tt * 16 + lane] : 0u;
  };
  auto rl = [&](uint32_t v, int i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, i); };
  // records of a task (lane l: record l of each stream); past the end: pad
  auto load_recs_v = [&](uint32_t mv, int2& rxv, int2& rcv) {
    const uint32_t xs = rl(mv, 0), cs = rl(mv, 2);
    rxv = xrec[xs + lane];
    rcv = crec[cs + lane];
  };
  uint32_t m0 = load_meta_v(t);
  uint32_t m1 = load_meta_v(t + stride);
  int2 rx0, rc0;
  load_recs_v(m0, rx0, rc0);
  typedef float V2 __attribute__((ext_vector_type(2 * R)));
  while (true) {
    // this task: m0, rx0, rc0; next: m1 (records loaded below), then the meta after
    int2 rx1, rc1;
    load_recs_v(m1, rx1, rc1);
    const uint32_t m2 = load_meta_v(t + 2 * stride);
    const uint32_t nx = rl(m0, 1), nc = rl(m0, 3);
    const uint64_t xm = (uint64_t)rl(m0, 4) | ((uint64_t)rl(m0, 5) << 32);
    const uint64_t cm = (uint64_t)rl(m0, 6) | ((uint64_t)rl(m0, 7) << 32);
    const uint32_t xsl = rl(m0, 8), csl = rl(m0, 9), r0 = rl(m0, 10), nrows = rl(m0, 11),
                   fl = rl(m0, 12);
    V2 sl, sc;
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) {
      sl[i] = 0.f;
      sc[i] = 0.f;
    }
    // ---- X stream ----
    {
      float ax = 0.f, ay = 0.f;
      uint32_t k = 0;
      auto issue = [&](uint32_t b0, float2 (&v)[U]) {
        uint32_t so[U];
#pragma unroll
        for (int u = 0; u < U; ++u) so[u] = rl((uint32_t)rx0.x, (int)(b0 + u) & 63);
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsx, vx, so[u], 0));
      };
      auto consume = [&](uint32_t b0, const float2 (&v)[U]) {
        const uint32_t rem = nx - b0;
        const uint32_t bm = (uint32_t)(xm >> b0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if ((uint32_t)u < rem) {
            const float w = __uint_as_float(rl((uint32_t)rx0.y, (int)(b0 + u) & 63));
            ax = fmaf(w, v[u].x, ax);
            ay = fmaf(w, v[u].y, ay);
            if ((bm >> u) & 1u) {
              const uint32_t s = (xsl >> (4 * k)) & 15u;
              sl[2 * s] = ax;
              sl[2 * s + 1] = ay;
              ax = 0.f;
              ay = 0.f;
              ++k;
            }
          }
        }
      };
      if constexpr (PIPE) {
        float2 va[U], vb[U];
        uint32_t b0 = 0;
        // ALWAYS: the next block is issued even past the stream (records
        // there are other tasks' or pad: valid offsets, never summed), so
        // every wait count is static
        if (ALWAYS || nx > 0) issue(0, va);
        while (b0 < nx) {
          if (ALWAYS || b0 + U < nx) issue(b0 + U, vb);
          consume(b0, va);
          b0 += U;
          if (b0 >= nx) break;
          if (ALWAYS || b0 + U < nx) issue(b0 + U, va);
          consume(b0, vb);
          b0 += U;
        }
      } else {
        for (uint32_t b0 = 0; b0 < nx; b0 += U) {
          float2 v[U];
          issue(b0, v);
          consume(b0, v);
        }
      }
    }
    // ---- codebook stream ----
    {
      float ax = 0.f, ay = 0.f;
      uint32_t k = 0;
      auto issue = [&](uint32_t b0, uint32_t (&cd)[U]) {
        uint32_t so[U];
#pragma unroll
        for (int u = 0; u < U; ++u) so[u] = rl((uint32_t)rc0.x, (int)(b0 + u) & 63);
#pragma unroll
        for (int u = 0; u < U; ++u)
          cd[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rsc, vc, so[u], 0);
      };
      auto consume = [&](uint32_t b0, const uint32_t (&cd)[U]) {
        const uint32_t rem = nc - b0;
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] = *reinterpret_cast<const float2*>(img + ((cd[u] & 0xffffu) << 9) + vl);
        const uint32_t bm = (uint32_t)(cm >> b0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if ((uint32_t)u < rem) {
            const float w = __uint_as_float(rl((uint32_t)rc0.y, (int)(b0 + u) & 63));
            ax = fmaf(w, v[u].x, ax);
            ay = fmaf(w, v[u].y, ay);
            if ((bm >> u) & 1u) {
              const uint32_t s = (csl >> (4 * k)) & 15u;
              sc[2 * s] = ax;
              sc[2 * s + 1] = ay;
              ax = 0.f;
              ay = 0.f;
              ++k;
            }
          }
        }
      };
      if constexpr (PIPE) {
        uint32_t ca[U], cb2[U];
        uint32_t b0 = 0;
        if (ALWAYS || nc > 0) issue(0, ca);
        while (b0 < nc) {
          if (ALWAYS || b0 + U < nc) issue(b0 + U, cb2);
          consume(b0, ca);
          b0 += U;
          if (b0 >= nc) break;
          if (ALWAYS || b0 + U < nc) issue(b0 + U, ca);
          consume(b0, cb2);
          b0 += U;
        }
      } else {
        for (uint32_t b0 = 0; b0 < nc; b0 += U) {
          uint32_t cd[U];
          issue(b0, cd);
          consume(b0, cd);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if ((uint32_t)s < nrows) {
        char* dst;
        if ((uint32_t)s == nrows - 1 && (fl & 2u))
          dst = reinterpret_cast<char*>(a.carry + ((size_t)t * 2 + 1) * a.cf);
        else if (s == 0 && (fl & 1u))
          dst = reinterpret_cast<char*>(a.carry + (size_t)t * 2 * a.cf);
        else
          dst = reinterpret_cast<char*>(a.out) + (size_t)(r0 + s) * a.ldob;
        *reinterpret_cast<float2*>(dst + vx) =
            make_float2(__fadd_rn(sl[2 * s], sc[2 * s]), __fadd_rn(sl[2 * s + 1], sc[2 * s + 1]));
      }
    }
    t += stride;
    if (t >= a.ntasks) break;
    m0 = m1;
    m1 = m2;
    rx0 = rx1;
    rc0 = rc1;
  }
}

// cut rows: out[row] = tail[ts] + ... + tail[te-1] + head[te] (task order)
__global__ void walk3_fixup(const int32_t* __restrict__ jobs, int n_jobs, const float* __restrict__ carry,
                            int cf, int F, float* __restrict__ out, long long ldo) {
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 5;
  const int lane = threadIdx.x & 31;
  if (w >= n_jobs) return;
  const int r = jobs[3 * w], ts = jobs[3 * w + 1], te = jobs[3 * w + 2];
  const int C4 = cf >> 2;
  const float4* c4 = reinterpret_cast<const float4*>(carry);
  for (int c = lane; c < F / 4; c += 32) {
    float4 s = c4[((size_t)ts * 2 + 1) * C4 + c];
    for (int u = ts + 1; u < te; ++u) {
      const float4 q = c4[((size_t)u * 2 + 1) * C4 + c];
      s.x = __fadd_rn(s.x, q.x); s.y = __fadd_rn(s.y, q.y);
      s.z = __fadd_rn(s.z, q.z); s.w = __fadd_rn(s.w, q.w);
    }
    const float4 q = c4[(size_t)te * 2 * C4 + c];
    s.x = __fadd_rn(s.x, q.x); s.y = __fadd_rn(s.y, q.y);
    s.z = __fadd_rn(s.z, q.z); s.w = __fadd_rn(s.w, q.w);
    reinterpret_cast<float4*>(out + (size_t)r * ldo)[c] = s;
  }
}

}  // namespace w3

using namespace w3;

template <int U, int R, int V, int NT = kThreads>
static int launch(const uint32_t* meta, const int2* xrec, const int2* crec, const Args& a, int F,
                  const int32_t* jobs, int n_jobs, hipStream_t s) {
  const void* fn = V == 4   ? (const void*)walk4_kernel<U, R, NT>
                   : V == 5 ? (const void*)walk3_kernel<U, R, true>
                   : V == 6 ? (const void*)walk5_kernel<U, R>
                   : V == 7 ? (const void*)walk6_kernel<U, R, false>
                   : V == 8 ? (const void*)walk6_kernel<U, R, true>
                   : V == 9 ? (const void*)walk6_kernel<U, R, true, true>
                            : (const void*)walk3_kernel<U, R>;
  static bool once = [fn] {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)once;
  const size_t lds = (size_t)a.M * 512;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  int wgs = (a.ntasks + NT / 64 - 1) / (NT / 64);
  wgs = wgs < cus ? wgs : cus;
  if (V == 4)
    hipLaunchKernelGGL((walk4_kernel<U, R, NT>), dim3(wgs, F / 128), dim3(NT), lds, s, meta, xrec,
                       crec, a);
  else if (V == 7)
    hipLaunchKernelGGL((walk6_kernel<U, R, false>), dim3(wgs, F / 128), dim3(kThreads), lds, s, meta,
                       xrec, crec, a);
  else if (V == 8)
    hipLaunchKernelGGL((walk6_kernel<U, R, true>), dim3(wgs, F / 128), dim3(kThreads), lds, s, meta,
                       xrec, crec, a);
  else if (V == 9)
    hipLaunchKernelGGL((walk6_kernel<U, R, true, true>), dim3(wgs, F / 128), dim3(kThreads), lds, s,
                       meta, xrec, crec, a);
  else if (V == 6)
    hipLaunchKernelGGL((walk5_kernel<U, R>), dim3(wgs, F / 128), dim3(kThreads), lds, s, meta, xrec,
                       crec, a);
  else if (V == 5)
    hipLaunchKernelGGL((walk3_kernel<U, R, true>), dim3(wgs, F / 128), dim3(kThreads), lds, s, meta,
                       xrec, crec, a);
  else
    hipLaunchKernelGGL((walk3_kernel<U, R>), dim3(wgs, F / 128), dim3(kThreads), lds, s, meta, xrec,
                       crec, a);
  if (n_jobs > 0)
    hipLaunchKernelGGL(walk3_fixup, dim3((n_jobs * 32 + 255) / 256), dim3(256), 0, s, jobs, n_jobs,
                       a.carry, a.cf, F, a.out, (long long)(a.ldob / 4));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int walk3_run(int U, int R, const uint32_t* meta, const int2* xrec, const int2* crec,
                         int ntasks, uint32_t xpad, uint32_t cpad, const char* xbase, uint32_t xbytes, const char* cbase,
                         uint32_t cbytes, const float* cbe, long long ldw, long long bstride, int M,
                         int D, float* out, uint32_t ldob, float* carry, int cf, int F,
                         const int32_t* jobs, int n_jobs, void* stream) {
  Args a{};
  a.xbase = xbase;
  a.xbytes = xbytes;
  a.cbase = cbase;
  a.cbytes = cbytes;
  a.cbe = cbe;
  a.cb_ldw = ldw;
  a.cb_bstride = bstride;
  a.M = M;
  a.D = D;
  a.out = out;
  a.ldob = ldob;
  a.carry = carry;
  a.cf = cf;
  a.ntasks = ntasks;
  a.xpad = xpad;
  a.cpad = cpad;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (U == 16 && R == 8) return launch<16, 8, 3>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 8 && R == 8) return launch<8, 8, 3>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 704) return launch<4, 8, 9>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 708) return launch<8, 8, 9>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 508) return launch<8, 8, 7>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 516) return launch<16, 8, 7>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 608) return launch<8, 8, 8>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 604) return launch<4, 8, 8>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 408) return launch<8, 8, 6>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 404) return launch<4, 8, 6>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 416) return launch<16, 8, 6>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 308) return launch<8, 8, 5>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 316) return launch<16, 8, 5>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 108) return launch<8, 8, 4>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 208) return launch<8, 8, 4, 512>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 212) return launch<12, 8, 4, 512>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 216) return launch<16, 8, 4, 512>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  return 2;
}
