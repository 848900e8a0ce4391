// Probe: accumulation error and subnormal handling of v_mfma_f32_16x16x32_f16
// (the filter sweep of vq_assign_kernel relies on a bound for both).
// Random trials of D = C + A*B (16x16x32, f16 in, f32 acc) against an exact
// (long double) sum; reports max |err| / (2^-24 (|C| + sum |a b|)) and whether
// f16 subnormal operands are flushed.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void mfma_probe(const _Float16* A, const _Float16* B, const float* C, float* D, int n) {
  const int t = blockIdx.x;          // trial
  if (t >= n) return;
  const int l = threadIdx.x, i = l & 15, q = l >> 4;
  half8 a, b;
  for (int jj = 0; jj < 8; ++jj) {
    a[jj] = A[(size_t)t * 512 + i * 32 + 8 * q + jj];      // A[i][k]
    b[jj] = B[(size_t)t * 512 + (8 * q + jj) * 16 + i];    // B[k][j=i]
  }
  floatx4 c;
  for (int r = 0; r < 4; ++r) c[r] = C[(size_t)t * 256 + (4 * q + r) * 16 + i];
  floatx4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(size_t)t * 256 + (4 * q + r) * 16 + i] = d[r];
}

int main() {
  const int n = 4096;
  std::vector<_Float16> A(n * 512), B(n * 512);
  std::vector<float> C(n * 256), D(n * 256);
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  std::uniform_real_distribution<double> ud(-20, 10);
  for (int t = 0; t < n; ++t) {
    const int kind = t % 4;
    for (int e = 0; e < 512; ++e) {
      double va = nd(rng), vb = nd(rng);
      if (kind == 1) { va *= std::exp2(ud(rng) * 0.5); vb *= std::exp2(ud(rng) * 0.5); }
      if (kind == 3 && (e % 3 == 0)) { va = std::exp2(-20 + (e % 5)); }   // f16 subnormals
      A[t * 512 + e] = (_Float16)va;
      B[t * 512 + e] = (_Float16)vb;
    }
    for (int e = 0; e < 256; ++e) {
      double vc = nd(rng) * (kind == 2 ? 1e3 : 4.0);
      C[t * 256 + e] = (float)vc;
    }
  }
  _Float16 *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma_probe, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD, n);
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  double worst[4] = {0, 0, 0, 0};
  long flushed = 0, sub_terms = 0;
  for (int t = 0; t < n; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        long double s = C[t * 256 + i * 16 + j], mag = std::fabs((double)C[t * 256 + i * 16 + j]);
        long double sub = 0;
        for (int k = 0; k < 32; ++k) {
          const long double p = (long double)(float)A[t * 512 + i * 32 + k] * (float)B[t * 512 + k * 16 + j];
          s += p;
          mag += std::fabs((double)p);
          if (std::fabs((float)A[t * 512 + i * 32 + k]) < 6.1035e-5f && A[t * 512 + i * 32 + k] != 0) sub += p;
        }
        const double err = std::fabs((double)(D[t * 256 + i * 16 + j] - s));
        const double r = err / (std::ldexp((double)mag, -24));
        if (r > worst[t % 4]) worst[t % 4] = r;
        if ((t % 4) == 3 && sub != 0) {
          ++sub_terms;
          if (std::fabs((double)(D[t * 256 + i * 16 + j] - (s - sub))) < 0.25 * std::fabs((double)sub)) ++flushed;
        }
      }
  printf("max err / (2^-24 (|C|+sum|ab|)): normal %.3f  wide-range %.3f  large-C %.3f  subnormal %.3f\n",
         worst[0], worst[1], worst[2], worst[3]);
  printf("subnormal outputs that look flushed: %ld of %ld\n", flushed, sub_terms);
  return 0;
}
