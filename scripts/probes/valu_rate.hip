// VALU issue-rate probe: independent chains of v_add_f32 / v_pk_add_f32 /
// v_cndmask / mfma_f32_16x16x4 mixes at several waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void probe(float* out, int iters, float s) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
  f2 p[4];
  for (int i = 0; i < 4; ++i) p[i] = f2{a[2 * i], a[2 * i + 1]};
  f4 acc[2] = {f4{0, 0, 0, 0}, f4{0, 0, 0, 0}};
  int idx[8] = {0};
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {  // 8 independent v_add_f32
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = a[i] + s;
    } else if constexpr (MODE == 1) {  // 4 v_pk_add_f32 (8 adds)
#pragma unroll
      for (int i = 0; i < 4; ++i) p[i] = p[i] + f2{s, s};
    } else if constexpr (MODE == 2) {  // 8 x (cmp + 2 cndmask) independent
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = s * (float)(i + 1);
        const bool t = d < a[i];
        a[i] = t ? d : a[i];
        idx[i] = t ? it : idx[i];
      }
    } else if constexpr (MODE == 3) {  // 4 mfma f32 16x16x4 (2 chains)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], a[i + 2], acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 4], a[i + 6], acc[i], 0, 0, 0);
      }
    } else if constexpr (MODE == 4) {  // 4 mfma + 8 add (mixed)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], a[i + 2], acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 4], a[i + 6], acc[i], 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = a[i] + s;
    }
  }
  float r = 0;
  for (int i = 0; i < 8; ++i) r += a[i] + (float)idx[i];
  for (int i = 0; i < 4; ++i) r += p[i].x + p[i].y;
  r += acc[0][0] + acc[1][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  float* out;
  hipMalloc(&out, 1 << 26);
  const char* names[] = {"8x v_add_f32", "4x v_pk_add_f32", "8x(cmp+2cnd)", "4x mfma16x16x4f32",
                         "4 mfma + 8 add"};
  const int instrs[] = {8, 4, 24, 4, 12};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096;
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = 256, threads = 256 * wps / 1;  // waves per SIMD = wps (1 block/CU)
    for (int mode = 0; mode < 5; ++mode) {
      auto launch = [&]() {
        switch (mode) {
          case 0: hipLaunchKernelGGL(probe<0>, blocks, threads, 0, 0, out, iters, 1e-7f); break;
          case 1: hipLaunchKernelGGL(probe<1>, blocks, threads, 0, 0, out, iters, 1e-7f); break;
          case 2: hipLaunchKernelGGL(probe<2>, blocks, threads, 0, 0, out, iters, 1e-7f); break;
          case 3: hipLaunchKernelGGL(probe<3>, blocks, threads, 0, 0, out, iters, 1e-7f); break;
          case 4: hipLaunchKernelGGL(probe<4>, blocks, threads, 0, 0, out, iters, 1e-7f); break;
        }
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
      // cycles per instruction per SIMD at 2.4 GHz (wave instrs per SIMD = wps*iters*n)
      const double per_simd = (double)wps * iters * instrs[mode];
      printf("waves/SIMD=%d %-20s %8.3f ms  %.2f ns/instr/SIMD (%.2f cyc @2.4GHz)\n", wps,
             names[mode], ms, ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
    }
  }
  return 0;
}
