// LDS atomic cost probe: no-return ds_add_{f32,u32,u64} and ds_add_rtn_f32,
// 8 waves per workgroup, addresses: random within an M*(W+1) slab, or
// consecutive per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE, bool RANDOM>
__global__ void __launch_bounds__(512) probe(float* out, int iters, int slots) {
  __shared__ uint64_t acc64[2304];
  float* accf = reinterpret_cast<float*>(acc64);
  uint32_t* accu = reinterpret_cast<uint32_t*>(acc64);
  for (int i = threadIdx.x; i < 2304; i += 512) acc64[i] = 0;
  __syncthreads();
  uint32_t h = threadIdx.x * 2654435761u + blockIdx.x * 40503u;
  for (int it = 0; it < iters; ++it) {
    h = h * 1664525u + 1013904223u;
    const int lane = threadIdx.x & 63;
    const int row = (h >> 8) % 256;
    const int a = RANDOM ? row * 9 + 1 + (lane >> 4) : ((threadIdx.x + it * 64) % slots);
    if constexpr (MODE == 0) atomicAdd(accf + a, 1.0f);
    else if constexpr (MODE == 1) atomicAdd(accu + a, 3u);
    else if constexpr (MODE == 2) atomicAdd((unsigned long long*)(acc64 + a), 3ull);
  }
  __syncthreads();
  float s = 0;
  for (int i = threadIdx.x; i < 2304; i += 512) s += accf[i] + (float)accu[i] + (float)acc64[i];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 24);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 2048, blocks = 512;
  const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_add_u64"};
  for (int rnd = 0; rnd < 2; ++rnd)
    for (int mode = 0; mode < 3; ++mode) {
      auto launch = [&]() {
        if (rnd) {
          if (mode == 0) hipLaunchKernelGGL((probe<0, true>), blocks, 512, 0, 0, out, iters, 2304);
          if (mode == 1) hipLaunchKernelGGL((probe<1, true>), blocks, 512, 0, 0, out, iters, 2304);
          if (mode == 2) hipLaunchKernelGGL((probe<2, true>), blocks, 512, 0, 0, out, iters, 2304);
        } else {
          if (mode == 0) hipLaunchKernelGGL((probe<0, false>), blocks, 512, 0, 0, out, iters, 2304);
          if (mode == 1) hipLaunchKernelGGL((probe<1, false>), blocks, 512, 0, 0, out, iters, 2304);
          if (mode == 2) hipLaunchKernelGGL((probe<2, false>), blocks, 512, 0, 0, out, iters, 2304);
        }
      };
      launch();
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
      // wave-instructions per CU: blocks/256 * 8 waves * iters
      const double per_cu = (double)blocks / 256 * 8 * iters;
      printf("%-8s %-11s %8.3f ms  %.1f cycles/wave-instr/CU @2.4GHz\n",
             rnd ? "random" : "consec", names[mode], ms, ms * 1e-3 * 2.4e9 / per_cu);
    }
  return 0;
}
