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

template <int U, int R>
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
      auto xblock = [&](uint32_t b0, uint32_t rem, auto tail) {
        constexpr bool TAIL = decltype(tail)::value;
        const Blk<U> rb = *reinterpret_cast<const Blk<U>*>(xrec + xs + b0);
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
      for (; b0 + U <= nx; b0 += U) xblock(b0, U, std::false_type{});
      if (b0 < nx) xblock(b0, nx - b0, std::true_type{});
    }
    // ---- pass 2: codebook stream, into its own slots ----
    {
      float ax = 0.f, ay = 0.f;
      uint32_t k = 0;
      auto cblock = [&](uint32_t b0, uint32_t rem, auto tail) {
        constexpr bool TAIL = decltype(tail)::value;
        const Blk<U> rb = *reinterpret_cast<const Blk<U>*>(crec + cs + b0);
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
      for (; b0 + U <= nc; b0 += U) cblock(b0, U, std::false_type{});
      if (b0 < nc) cblock(b0, nc - b0, std::true_type{});
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
  const void* fn = V == 4 ? (const void*)walk4_kernel<U, R, NT> : (const void*)walk3_kernel<U, R>;
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
  if (U == 108) return launch<8, 8, 4>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 208) return launch<8, 8, 4, 512>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 212) return launch<12, 8, 4, 512>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  if (U == 216) return launch<16, 8, 4, 512>(meta, xrec, crec, a, F, jobs, n_jobs, s);
  return 2;
}
