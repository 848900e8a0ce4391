// Row-gather throughput by load shape, 512-B rows from an L2-resident table.
// MODE 0: dwordx2, one row per wave-instruction (64 lanes x 8 B)
// MODE 1: dwordx4, two rows per wave-instruction (lanes 0-31 row a, 32-63 row b)
// MODE 2: dwordx4, one row per wave-instruction, lanes 32-63 idle
// MODE 3: dwordx2 with per-lane (VGPR) row offsets instead of a scalar offset
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ void __launch_bounds__(256) gather(const float* __restrict__ tab, int nrows_tab,
                                              int steps, float* out) {
  const int lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)tab, 0, nrows_tab * 512, 0x00020000);
  uint32_t h = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2654435761u;
  float acc[4] = {0, 0, 0, 0};
  for (int s = 0; s < steps; s += 8) {
    float v[8][4];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      h = h * 1664525u + 1013904223u;
      const uint32_t ra = __builtin_amdgcn_readfirstlane((h >> 8) % nrows_tab);
      const uint32_t rb = __builtin_amdgcn_readfirstlane((h >> 16) % nrows_tab);
      if constexpr (MODE == 0) {
        const float2 t = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, lane * 8, ra * 512, 0));
        v[u][0] = t.x; v[u][1] = t.y; v[u][2] = 0; v[u][3] = 0;
      } else if constexpr (MODE == 1) {
        const uint32_t off = (lane < 32 ? ra : rb) * 512 + (lane & 31) * 16;
        const float4 t = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = t.w;
      } else if constexpr (MODE == 2) {
        if (lane < 32) {
          const float4 t = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, ra * 512, 0));
          v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = t.w;
        } else {
          v[u][0] = v[u][1] = v[u][2] = v[u][3] = 0;
        }
      } else {
        const uint32_t off = ra * 512 + lane * 8;
        const float2 t = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
        v[u][0] = t.x; v[u][1] = t.y; v[u][2] = 0; v[u][3] = 0;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += v[u][k];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main() {
  const int nrows = 1024;
  float *tab, *out;
  (void)hipMalloc(&tab, nrows * 512);
  (void)hipMemset(tab, 0, nrows * 512);
  (void)hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int steps = 512;
  for (int blocks : {2048, 8192}) {
    for (int mode = 0; mode < 4; ++mode) {
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(gather<0>, blocks, 256, 0, 0, tab, nrows, steps, out);
        if (mode == 1) hipLaunchKernelGGL(gather<1>, blocks, 256, 0, 0, tab, nrows, steps, out);
        if (mode == 2) hipLaunchKernelGGL(gather<2>, blocks, 256, 0, 0, tab, nrows, steps, out);
        if (mode == 3) hipLaunchKernelGGL(gather<3>, blocks, 256, 0, 0, tab, nrows, steps, out);
      };
      launch();
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 3; ++r) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 3;
      const double rows = (double)blocks * 4 * steps * (mode == 1 ? 2 : 1);
      printf("blocks=%5d mode=%d  %8.3f ms  %6.2f TB/s  %.2f Grows/s\n", blocks, mode, ms,
             rows * 512 / ms / 1e9, rows / ms / 1e6);
    }
  }
  return 0;
}
