// MFMA shape probe on random fp16 operands: v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16 at the
// same output tile per wave (128 accumulator registers), one or two waves per SIMD, operands in
// registers (no memory traffic in the loop). Reports TF/s and the in-kernel shader clock
// (s_memtime / s_memrealtime) per variant; variants are interleaved over rounds in one process.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_shape_probe.hip -o tools/mfma_shape_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ inline unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }
__device__ inline unsigned long long ct() { return __builtin_amdgcn_s_memtime(); }

template <int SHAPE, int WPS>  // SHAPE 32: 32x32x16 (8 acc), 16: 16x16x32 (32 acc); WPS waves per SIMD
__global__ __launch_bounds__(256 * WPS, 1) void k(const _Float16* src, float* out, unsigned long long* clk, int iters) {
  const int tid = threadIdx.x;
  f16x8 a[3], b[3];
  for (int p = 0; p < 3; ++p)
    for (int e = 0; e < 8; ++e) {
      a[p][e] = src[(tid * 48 + p * 8 + e) & 65535];
      b[p][e] = src[(tid * 48 + 24 + p * 8 + e) & 65535];
    }
  const unsigned long long r0 = rt(), c0 = ct();
  float s = 0.f;
  if constexpr (SHAPE == 32) {
    f32x16 acc[8];
    for (int j = 0; j < 8; ++j)
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[p], b[(p + j) % 3], acc[j], 0, 0, 0);
    }
    for (int j = 0; j < 8; ++j)
      for (int r = 0; r < 16; ++r) s += acc[j][r];
  } else {
    f32x4 acc[32];
    for (int j = 0; j < 32; ++j)
      for (int r = 0; r < 4; ++r) acc[j][r] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 32; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[p], b[(p + j) % 3], acc[j], 0, 0, 0);
    }
    for (int j = 0; j < 32; ++j)
      for (int r = 0; r < 4; ++r) s += acc[j][r];
  }
  const unsigned long long r1 = rt(), c1 = ct();
  if (tid == 0) {
    clk[2 * blockIdx.x] = c1 - c0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  if (s == 1234.5f) out[tid] = s;
}

__global__ void fill(_Float16* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    unsigned x = i * 2654435761u + 12345u;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (_Float16)(((x & 0xffff) / 65536.0f) * 2.0f - 1.0f);
  }
}

template <int SHAPE, int WPS>
void run(const _Float16* src, float* out, unsigned long long* clk, int blocks, int iters, const char* name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // 96 KB of dynamic LDS per block: one block per CU, so WPS really is the waves per SIMD
  (void)hipFuncSetAttribute((const void*)k<SHAPE, WPS>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  for (int rep = 0; rep < 4; ++rep)  // back-to-back launches (the clock settles under load); the last is timed
    hipLaunchKernelGGL((k<SHAPE, WPS>), dim3(blocks), dim3(256 * WPS), 96 * 1024, 0, src, out, clk, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k<SHAPE, WPS>), dim3(blocks), dim3(256 * WPS), 96 * 1024, 0, src, out, clk, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(2 * blocks);
  (void)hipMemcpy(h.data(), clk, 16 * blocks, hipMemcpyDeviceToHost);
  double cs = 0, rs = 0;
  for (int b = 0; b < blocks; ++b) { cs += h[2 * b]; rs += h[2 * b + 1]; }
  const double ghz = cs / rs * 0.1;  // s_memrealtime ticks at 100 MHz
  // per iteration: 3 x 8 MFMAs of 32x32x16 or 3 x 32 MFMAs of 16x16x32 (twice the flops of the former)
  const double flops = (double)blocks * 4 * WPS * iters * 3.0 * (SHAPE == 32 ? 8 * 32768.0 : 32 * 16384.0);
  printf("%-28s %8.3f ms %7.1f TF  clock %.2f GHz\n", name, ms, flops / ms / 1e9, ghz);
}

int main() {
  _Float16* src;
  float* out;
  unsigned long long* clk;
  (void)hipMalloc(&src, 65536 * 2);
  (void)hipMalloc(&out, 4096 * 4);
  (void)hipMalloc(&clk, 16 * 4096);
  hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, src, 65536);
  const int iters = 12000;
  for (int round = 0; round < 3; ++round) {
    run<32, 1>(src, out, clk, 256 * 4, iters, "32x32x16 f16, 1 wave/SIMD");
    run<16, 1>(src, out, clk, 256 * 4, iters, "16x16x32 f16, 1 wave/SIMD");
    run<32, 2>(src, out, clk, 256 * 4, iters / 2, "32x32x16 f16, 2 waves/SIMD");
    run<16, 2>(src, out, clk, 256 * 4, iters / 2, "16x16x32 f16, 2 waves/SIMD");
  }
  return 0;
}
