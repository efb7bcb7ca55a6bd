// Main-loop probe of a fused edge-MLP kernel (DESIGN.md "Fused edge MLP"): S would stay in registers as
// the second GEMM's operand, which pins 16 edges x all 512 output columns to one wave (one wave per
// SIMD, 4 waves per CU). This probe runs only the first GEMM's K loop of that design (D.f, K = 768,
// split16: three v_mfma_f32_16x16x32_f16 products per 16x16 block) on random operands:
//   * each wave owns 16 edges; its F fragments (hi / lo) come straight from global memory;
//   * the CU's four waves share one W (D) K-tile of 512 columns x 32 k (hi / lo fp16, 64 KB) staged by
//     global_load_lds into a 2-deep LDS ring (XOR-swizzled like k_edge16), and every wave reads all of
//     it: 64 ds_read_b128 per lane per K-tile (W fragment reuse 1);
//   * 96 MFMAs per wave per K-tile, 128 accumulator registers.
// Reported: TF/s of fp16 MFMA work (3 products counted), to compare with the current two kernels'
// main loops (edge layer 1: 644 GFLOP fp32-equivalent x 3 products in ~1.30 ms = ~1.49 PF fp16).
//   hipcc --offload-arch=gfx950 -O3 tools/fused_probe.hip -o tools/fused_probe && tools/fused_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e_ = (x);                                        \
    if (e_ != hipSuccess) {                                     \
      printf("%s: %s\n", #x, hipGetErrorString(e_));            \
      return 1;                                                 \
    }                                                           \
  } while (0)

constexpr int NCOL = 512, KT = 32, ROWB = KT * 2 * 2;  // one K-tile row = 128 B (hi 32 | lo 32)
constexpr int WTILE = NCOL * ROWB;                      // 64 KB per W K-tile

// W: [NCOL][nk][64 halfs] split rows; F: [E][nk][64 halfs]; out: one float per wave (keeps the work)
__global__ __launch_bounds__(256, 1) void k_probe(const _Float16* __restrict__ W, const _Float16* __restrict__ F,
                                                  float* __restrict__ out, int nk, int reps) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g4 = lane >> 4;
  const long e0 = ((long)blockIdx.x * 4 + wave) * 16;
  const long rowB = (long)nk * ROWB;
  const char* Wb = reinterpret_cast<const char*>(W);
  const char* Fb = reinterpret_cast<const char*>(F) + (e0 + l16) * rowB;
  // staging: 64 KB per K-tile = 64 wave-instructions of 1 KB (8 rows of 128 B); wave w issues 16
  auto stage = [&](int t, int slot) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = (wave * 16 + q) * 8 + (lane >> 3);  // W row (output column)
      const int pc = lane & 7, lc = pc ^ ((r >> 1) & 7);
      __builtin_amdgcn_global_load_lds((gbl_void*)(Wb + (long)r * rowB + (long)t * ROWB + 16 * lc),
                                       (lds_void*)(lds + slot * WTILE + (wave * 16 + q) * 1024), 16, 0, 0);
    }
  };
  f32x4 acc[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int swz = (l16 >> 1) & 7;
  const int ch0 = 16 * (g4 ^ swz), ch1 = 16 * ((4 + g4) ^ swz);
  for (int rep = 0; rep < reps; ++rep) {
    stage(0, 0);
    for (int t = 0; t < nk; ++t) {
      // this edge's F fragments (hi: chunk g4, lo: chunk 4 + g4 of the row's K-tile line)
      const f16x8 ah = *reinterpret_cast<const f16x8*>(Fb + (long)t * ROWB + 16 * g4);
      const f16x8 al = *reinterpret_cast<const f16x8*>(Fb + (long)t * ROWB + 64 + 16 * g4);
      if (t + 1 < nk) {
        stage(t + 1, (t + 1) & 1);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // K-tile t's stage (and the F loads) landed
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const char* S = lds + (t & 1) * WTILE + l16 * ROWB;
#pragma unroll
      for (int c = 0; c < 32; ++c) {  // 16-column groups: fragment of rows 16c + l16
        const f16x8 wh = *reinterpret_cast<const f16x8*>(S + c * 16 * ROWB + ch0);
        const f16x8 wl = *reinterpret_cast<const f16x8*>(S + c * 16 * ROWB + ch1);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, ah, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, al, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ah, acc[c], 0, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();  // everyone is done with this stage before it is refilled
      asm volatile("" ::: "memory");
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 32; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[(long)blockIdx.x * 256 + tid] = s;
}

int main() {
  const int nk = 768 / KT;            // edge layer 1's K
  const int blocks = 256 * 25;        // 25 rounds of one block per CU (6400 x 64 edges = 409600 edges)
  const long E = (long)blocks * 64;
  const int reps = 1;
  std::vector<_Float16> hw((size_t)NCOL * nk * 64), hf((size_t)E * nk * 64);
  unsigned s = 1;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 9) & 0xffff) / 65536.f - 0.5f; };
  for (auto& v : hw) v = (_Float16)rnd();
  for (size_t i = 0; i < hf.size(); i += 4096) hf[i] = (_Float16)rnd();  // (sparse init: random enough, fast)
  _Float16 *dw, *df;
  float* dout;
  CK(hipMalloc(&dw, hw.size() * 2));
  CK(hipMalloc(&df, hf.size() * 2));
  CK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
  CK(hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(df, hf.data(), hf.size() * 2, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)k_probe, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * WTILE));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(256), 2 * WTILE, 0, dw, df, dout, nk, reps);
  CK(hipDeviceSynchronize());
  const int runs = 10;
  CK(hipEventRecord(a));
  for (int it = 0; it < runs; ++it)
    hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(256), 2 * WTILE, 0, dw, df, dout, nk, reps);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= runs;
  const double flops = 2.0 * E * NCOL * 768 * 3 * reps;  // fp16 MFMA work, 3 products
  printf("fused-MLP first-GEMM probe: %ld edges, K = 768, 512 columns: %.3f ms, %.0f TF/s fp16 MFMA "
         "(= %.0f TF/s fp32-equivalent)\n", E, ms, flops / (ms * 1e-3) / 1e12, flops / 3 / (ms * 1e-3) / 1e12);
  return 0;
}
