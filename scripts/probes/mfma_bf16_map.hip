// Probe: v_mfma_f32_16x16x32_bf16 operand maps with exact small-integer data.
// A[i][k] (16x32), B[k][j] (32x16); lane l: A[l&15][8(l>>4)+e], B[8(l>>4)+e][l&15];
// D reg r of lane l = D[4(l>>4)+r][l&15].  Prints the max |D - ref|.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__device__ unsigned short bf(float v) { return (unsigned short)(__float_as_uint(v) >> 16); }
__global__ void k(const float* A, const float* Bm, float* D) {
  const int l = threadIdx.x, q = l >> 4, j = l & 15;
  s8 a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = (short)bf(A[j * 32 + 8 * q + e]);
    b[e] = (short)bf(Bm[(8 * q + e) * 16 + j]);
  }
  f4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, f4{0, 0, 0, 0}, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * q + r) * 16 + j] = d[r];
}
int main() {
  float hA[16 * 32], hB[32 * 16], ref[256], out[256];
  for (int i = 0; i < 16 * 32; ++i) hA[i] = (float)((i * 7 + 3) % 11 - 5);
  for (int i = 0; i < 32 * 16; ++i) hB[i] = (float)((i * 5 + 1) % 13 - 6);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      float s = 0;
      for (int kk = 0; kk < 32; ++kk) s += hA[i * 32 + kk] * hB[kk * 16 + j];
      ref[i * 16 + j] = s;
    }
  float *dA, *dB, *dD;
  (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB); (void)hipMalloc(&dD, 1024);
  (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, dA, dB, dD);
  (void)hipMemcpy(out, dD, 1024, hipMemcpyDeviceToHost);
  float mx = 0;
  for (int i = 0; i < 256; ++i) mx = fmaxf(mx, fabsf(out[i] - ref[i]));
  printf("max |D - ref| = %g  (D[0]=%g ref=%g, D[17]=%g ref=%g)\n", mx, out[0], ref[0], out[17], ref[17]);
  return 0;
}
