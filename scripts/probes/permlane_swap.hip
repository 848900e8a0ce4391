// Probe: lane mapping of v_permlane32_swap / v_permlane16_swap (gfx950) and
// the 4 x 4 quad transpose vq_filter_kernel builds from them.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(unsigned* out) {
  const unsigned l = threadIdx.x;
  unsigned v = l;
  auto a = __builtin_amdgcn_permlane32_swap(v, v + 100, false, false);
  auto c = __builtin_amdgcn_permlane16_swap(v, v + 100, false, false);
  out[l * 4 + 0] = a[0];
  out[l * 4 + 1] = a[1];
  out[l * 4 + 2] = c[0];
  out[l * 4 + 3] = c[1];
  // transpose: r[g] = 16 * (quad q) + g encodes (source quad, index g)
  const unsigned q = l >> 4;
  unsigned r0 = q * 16 + 0, r1 = q * 16 + 1, r2 = q * 16 + 2, r3 = q * 16 + 3;
  auto s02 = __builtin_amdgcn_permlane32_swap(r0, r2, false, false);
  r0 = s02[0]; r2 = s02[1];
  auto s13 = __builtin_amdgcn_permlane32_swap(r1, r3, false, false);
  r1 = s13[0]; r3 = s13[1];
  auto s01 = __builtin_amdgcn_permlane16_swap(r0, r1, false, false);
  r0 = s01[0]; r1 = s01[1];
  auto s23 = __builtin_amdgcn_permlane16_swap(r2, r3, false, false);
  r2 = s23[0]; r3 = s23[1];
  out[256 + l * 4 + 0] = r0;
  out[256 + l * 4 + 1] = r1;
  out[256 + l * 4 + 2] = r2;
  out[256 + l * 4 + 3] = r3;
}
int main() {
  unsigned* d;
  unsigned h[512];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 1, 15, 16, 17, 31, 32, 33, 47, 48, 63})
    printf("lane %2d: swap32 (v, v+100) -> %3u %3u | swap16 -> %3u %3u\n", l, h[l * 4], h[l * 4 + 1],
           h[l * 4 + 2], h[l * 4 + 3]);
  for (int l : {0, 16, 32, 48, 5, 21, 37, 53})
    printf("lane %2d (q=%d): transposed r0..r3 = (q%u,g%u) (q%u,g%u) (q%u,g%u) (q%u,g%u)\n", l, l >> 4,
           h[256 + l * 4] / 16, h[256 + l * 4] % 16, h[256 + l * 4 + 1] / 16, h[256 + l * 4 + 1] % 16,
           h[256 + l * 4 + 2] / 16, h[256 + l * 4 + 2] % 16, h[256 + l * 4 + 3] / 16, h[256 + l * 4 + 3] % 16);
  return 0;
}
