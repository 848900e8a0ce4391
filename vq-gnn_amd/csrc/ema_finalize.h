// The EMA finalize of one branch, vq.py:177-200 and :242-277, as a device
// function of one 1,024-thread workgroup.  Two launches run it:
// vq_ema_finalize_kernel (vq_kernels.hip, one workgroup per branch) and the
// SpMM fix-up launch of vqgnn_spmm_task_cb_fin (spmm_tasks.hip), whose first
// nb workgroups finalize the branches beside the cut-row sums.  One body, so
// both give the same bits.
#pragma once

#include "common.h"

namespace vqgnn {

constexpr int kFinThreads = 1024;
constexpr int kFinWaves = kFinThreads / 64;

// the finalize's operands (vqgnn_vq_ema_finalize's, after the host checks;
// shift_f / shift_g from stat_shift(stat_count, grad_scale))
struct EmaFin {
  long long* stats;          // [nparts][nb][M][W + 1] fixed-point slabs
  int nparts;
  int64_t part_stride;
  int zero_after, shift_f, shift_g, M, D, W, ldw;
  float decay;
  int laplace;
  float grad_scale, epsilon;
  float* cluster_size;
  int64_t cs_bstride;
  float* ema_w;
  float* emb;
  float* emb_out;
  int64_t emb_bstride;
  const float* rm_f;
  const float* rv_f;
  const float* rm_g;
  const float* rv_g;
  int* bad_init;
  int split;                 // M >= 1,024: stop after the cluster sizes (vq_ema_apply_kernel)
};

// Branch b by the calling workgroup (kFinThreads threads, tid = its thread);
// cs_s: M floats of LDS.  cs lives there between the phases, so the only
// global traffic is the slab, the state and the outputs.
__device__ __forceinline__ void ema_finalize_branch(const EmaFin& f, int b, int tid,
                                                    float* cs_s) {
  __shared__ float wred[kFinWaves];
  __shared__ int bad;
  const int lane = tid & 63, wave = tid >> 6;
  const int M = f.M, W = f.W, D = f.D;
  long long* st = f.stats + (int64_t)b * M * (W + 1);
  // statistic = integer sum of the per-part fixed-point slabs, decoded once:
  // round(exact sum * 2^-shift) to fp32 (count column: shift 0).  Every entry
  // is read by exactly one thread; zero_after clears it behind the read so
  // the slab is zero for the next vqgnn_vq_assign (ema_zeroed = 1).
  auto stat = [&](int64_t i, int shift) {
    long long v = st[i];
    if (f.zero_after) st[i] = 0;
    for (int p = 1; p < f.nparts; ++p) {
      v += st[(int64_t)p * f.part_stride + i];
      if (f.zero_after) st[(int64_t)p * f.part_stride + i] = 0;
    }
    return (float)ldexp((double)v, -shift);
  };
  float* cs = f.cluster_size + (int64_t)b * f.cs_bstride;
  float* ew = f.ema_w + (int64_t)b * f.emb_bstride;
  float* e = f.emb + (int64_t)b * f.emb_bstride;
  float* eo = f.emb_out + (int64_t)b * f.emb_bstride;
  const float decay = f.decay;
  const float one_m_decay = (float)(1.0 - (double)decay);  // python (1 - decay) -> float scalar
  if (tid == 0) bad = 0;

  // cs = cs*decay + (1-decay)*counts  (vq.py:177-178; fp32 tensor ops)
#pragma unroll 4
  for (int m = tid; m < M; m += kFinThreads)
    cs_s[m] = __fadd_rn(__fmul_rn(cs[m], decay), __fmul_rn(one_m_decay, stat((int64_t)m * (W + 1), 0)));
  __syncthreads();

  if (f.laplace) {  // vq.py:182-186
    // n = torch.sum(cs): per-thread sequential partials over a strided slice,
    // a fixed butterfly per wave, then the waves in order — deterministic
    // (ATen's CPU cascade order differs by ulps)
    float sum = 0.f;
    for (int m = tid; m < M; m += kFinThreads) sum = __fadd_rn(sum, cs_s[m]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum = __fadd_rn(sum, __shfl_xor(sum, off));
    if (lane == 0) wred[wave] = sum;
    __syncthreads();
    float n = wred[0];
#pragma unroll
    for (int w = 1; w < kFinWaves; ++w) n = __fadd_rn(n, wred[w]);
    const float den = __fadd_rn(n, (float)((double)M * 1e-5));  // n + M*1e-5 (python float -> f32)
    for (int m = tid; m < M; m += kFinThreads)
      cs_s[m] = __fmul_rn(__fdiv_rn(__fadd_rn(cs_s[m], 1e-5f), den), n);
    __syncthreads();
  }

  for (int m = tid; m < M; m += kFinThreads) {
    const float c = cs_s[m];
    cs[m] = c;
    if (c == 0.f) bad = 1;  // vq.py:188 count_nonzero(cs) != M
  }
  __syncthreads();
  if (bad) {  // reference raises before touching ema_w / embedding
    if (tid == 0) atomicOr(f.bad_init, 1);
    if (f.zero_after)
      for (int i = tid; i < M * W; i += kFinThreads)
        for (int p = 0; p < f.nparts; ++p)
          st[(int64_t)p * f.part_stride + (int64_t)(i / W) * (W + 1) + 1 + i % W] = 0;
    return;
  }
  if (f.split) return;                       // vq_ema_apply_kernel takes the rest

  // ema_w = ema_w*decay + (1-decay)*dw ; embedding = ema_w / cs ; output
  // (unrolled: the loads of four elements per thread in flight together)
  const int nw = M * W;
  const int ldw = f.ldw;
#pragma unroll 4
  for (int i = tid; i < nw; i += kFinThreads) {
    const int m = i / W, k = i % W;
    const int64_t o = (int64_t)m * ldw + k;
    const float dw = stat((int64_t)m * (W + 1) + 1 + k, k < D ? f.shift_f : f.shift_g);
    const float w = __fadd_rn(__fmul_rn(ew[o], decay), __fmul_rn(one_m_decay, dw));
    ew[o] = w;
    const float ev = __fdiv_rn(w, cs_s[m]);
    e[o] = ev;
    float out;
    if (k < D) {  // vq.py:198-200 / :267-272 feature half: emb*sqrt(rv+1e-5)+rm
      const float sd = sqrtf(__fadd_rn(f.rv_f[b * D + k], 1e-5f));
      out = __fadd_rn(__fmul_rn(ev, sd), f.rm_f[b * D + k]);
    } else {      // vq.py:263 /= (scale + eps); :267 sqrt(rv_g + eps)
      const int kg = k - D;
      const float div = (float)((double)f.grad_scale + (double)f.epsilon);
      const float sd = sqrtf(__fadd_rn(f.rv_g[b * D + kg], f.epsilon));
      out = __fadd_rn(__fmul_rn(__fdiv_rn(ev, div), sd), f.rm_g[b * D + kg]);
      if (f.grad_scale == 0.f) out = __fmul_rn(out, 0.f);  // vq.py:274-275
    }
    eo[o] = out;
  }
}

// Host: the checked operands of a finalize (vq_kernels.hip; the error text
// is set on failure).  Shared by vqgnn_vq_ema_finalize and
// vqgnn_spmm_task_cb_fin.
int ema_fin_prepare(const vqgnn_ema_finalize_args* a, EmaFin* f);
// Host: set a finalize kernel's LDS limit (M up to 34,816 floats)
void ema_fin_lds_attr(const void* kernel);
// Host: the finalize as its own launches (vq_ema_finalize_kernel, and
// vq_ema_apply_kernel when f.split) on stream s
int ema_fin_run(const EmaFin& f, int nb, hipStream_t s);

}  // namespace vqgnn
