// MFMA-rate probe: v_mfma_f32_32x32x16_f16 back to back, 8 waves per CU (2 per SIMD),
// 8 independent accumulators per wave (the edge GEMM's shape), no memory traffic.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(512, 1) void k(float* out, int iters) {
  f16x8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = (_Float16)(0.001f * (threadIdx.x + e)); b[e] = (_Float16)(0.002f * e); }
  f32x16 acc[8];
  for (int j = 0; j < 8; ++j)
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int rep = 0; rep < 3; ++rep)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[j], 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < 8; ++j)
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  if (s == 12345.f) out[threadIdx.x] = s;
}
int main() {
  float* d; (void)hipMalloc(&d, 4096);
  const int blocks = 256 * 25, iters = 48 * 8;
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, d, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, d, iters);
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 5;
  const double flops = (double)blocks * 8 * iters * 24 * 32 * 32 * 16 * 2;
  printf("mfma f16 32x32x16: %.3f ms, %.1f TF (f16), blocks %d\n", ms, flops / ms / 1e9, blocks);
  return 0;
}
