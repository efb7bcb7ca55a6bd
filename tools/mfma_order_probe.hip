// Are v_mfma_f32_16x16x16_f16 and v_mfma_f32_32x32x16_f16 bit-identical per output element (same 16 products
// of a K-block added to the same accumulator)? If so, a node-GEMM tiling on 16x16x16 keeps k_node_gemm's
// results bit for bit. One wave per test; inputs with wide exponent spread so that summation order shows.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// C[32][32] = A[32][16] B[16][32]^T... computed as C[m][n] = acc0 + sum_k A[m][k] * B[n][k]
__global__ void k32(const _Float16* A, const _Float16* B, const float* C0, float* C) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f16x8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = A[r * 16 + 8 * h + e]; b[e] = B[r * 16 + 8 * h + e]; }
  f32x16 acc;
  // C^T layout as k_node_gemm: acc = mfma(W frag, A frag): output row = A row (lane r32), columns of W
  for (int i = 0; i < 16; ++i) {
    const int n = (i / 4) * 8 + 4 * h + (i % 4);  // 32x32 accumulator layout: col group
    acc[i] = C0[r * 32 + n];
  }
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc, 0, 0, 0);
  for (int i = 0; i < 16; ++i) {
    const int n = (i / 4) * 8 + 4 * h + (i % 4);
    C[r * 32 + n] = acc[i];
  }
}
__global__ void k16(const _Float16* A, const _Float16* B, const float* C0, float* C) {
  // four 16x16 blocks of the same 32x32 output, each v_mfma_f32_16x16x16_f16 (K = 16: lane l holds row l & 15,
  // k chunk (l >> 4) * 4 .. +3)
  const int l = threadIdx.x, r = l & 15, q = l >> 4;
  for (int bm = 0; bm < 2; ++bm)
    for (int bn = 0; bn < 2; ++bn) {
      f16x4 a, b;
      for (int e = 0; e < 4; ++e) { a[e] = A[(16 * bm + r) * 16 + 4 * q + e]; b[e] = B[(16 * bn + r) * 16 + 4 * q + e]; }
      f32x4 acc;
      // C^T: acc = mfma(b, a): lane holds row 16 bm + r... output element (row = A row, col = B row):
      // for mfma(srcA = b, srcB = a) the result is [b rows][a rows]^T... we store transposed consistently below
      for (int i = 0; i < 4; ++i) acc[i] = C0[(16 * bm + r) * 32 + 16 * bn + 4 * q + i];
      acc = __builtin_amdgcn_mfma_f32_16x16x16f16(b, a, acc, 0, 0, 0);
      for (int i = 0; i < 4; ++i) C[(16 * bm + r) * 32 + 16 * bn + 4 * q + i] = acc[i];
    }
}
int main() {
  std::vector<_Float16> A(32 * 16), B(32 * 16);
  std::vector<float> C0(32 * 32), c1(32 * 32), c2(32 * 32), ref(32 * 32);
  srand(7);
  auto rnd = [] { return (rand() / (float)RAND_MAX - 0.5f); };
  _Float16 *dA, *dB; float *dC0, *dC1, *dC2;
  hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2); hipMalloc(&dC0, 4096); hipMalloc(&dC1, 4096); hipMalloc(&dC2, 4096);
  int diff = 0, cells = 0, reforder = 0;
  for (int trial = 0; trial < 200; ++trial) {
    for (int i = 0; i < 32 * 16; ++i) {
      A[i] = (_Float16)(rnd() * ldexpf(1.0f, rand() % 12 - 6));
      B[i] = (_Float16)(rnd() * ldexpf(1.0f, rand() % 12 - 6));
    }
    for (int i = 0; i < 1024; ++i) C0[i] = rnd() * ldexpf(1.0f, rand() % 16 - 8);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dC0, C0.data(), 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dC0, dC1);
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC0, dC2);
    hipMemcpy(c1.data(), dC1, 4096, hipMemcpyDeviceToHost);
    hipMemcpy(c2.data(), dC2, 4096, hipMemcpyDeviceToHost);
    for (int m = 0; m < 32; ++m)
      for (int n = 0; n < 32; ++n) {
        float s = C0[m * 32 + n];  // sequential fp32 order, for reference only
        for (int k = 0; k < 16; ++k) s = s + (float)A[m * 16 + k] * (float)B[n * 16 + k];
        ++cells;
        if (c1[m * 32 + n] != c2[m * 32 + n]) ++diff;
        if (c1[m * 32 + n] != s) ++reforder;
      }
  }
  printf("cells %d: 32x32x16 vs 16x16x16 differ in %d; 32x32x16 vs sequential fp32 differ in %d\n", cells, diff, reforder);
  return 0;
}
