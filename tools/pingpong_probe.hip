// Ping-pong probe: can one wave group's GEMM main loop run beside the other group's epilogue on the
// same SIMDs? (the edge-kernel epilogue overlap)
// One 512-thread workgroup per CU: group 0 = waves 0-3 (one per SIMD), group 1 = waves 4-7. Every
// "step" ends in one s_barrier shared by both groups (the coupled-barrier ping-pong form). A main-loop
// step of a wave: 8 global_load_lds issues (16 B per lane, a stage of operands), 16 ds_read_b128
// fragment reads and 48 v_mfma_f32_16x16x32_f16 (a 64x64 wave tile, 3 split products, K = 32). An
// epilogue step of a wave: E elements per lane of the edge layer-1 epilogue's arithmetic (two LDS
// operand adds, SiLU = exp + rcp, running max, scale, fp16 hi / lo split) and their 16-B stores.
// Modes: 0 both groups main loop (two waves per SIMD, the current kernels), 1 group 0 main loop +
// group 1 epilogue (ping-pong), 2 group 0 main loop alone, 3 group 1 epilogue alone.
//   hipcc --offload-arch=gfx950 -O3 tools/pingpong_probe.hip -o tools/pingpong_probe && ./tools/pingpong_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

constexpr int LDS_BYTES = 128 * 1024;

__device__ __forceinline__ void main_step(const char* lds, const char* gsrc, int lane, int wave, int step,
                                          f32x4 (&acc)[4][4]) {
  // stage: 8 x 1 KB per wave into this group's half of the LDS, ring of 2 (no reader of it: traffic only)
  char* ring = (char*)lds + (wave >> 2) * (64 * 1024) + (step & 1) * 32 * 1024 + (wave & 3) * 8 * 1024;
  // (an L2-resident source: 1 MB per XCD, as the edge kernels' W stream and re-read A rows)
  const char* src = gsrc + ((long)((blockIdx.x & 15) * 8 + wave) * 8 + (step & 7)) * 8192 + lane * 16;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    __builtin_amdgcn_global_load_lds((gbl_void*)(src + q * 1024), (lds_void*)(ring + q * 1024), 16, 0, 0);
  const char* fr = lds + (wave >> 2) * (64 * 1024) + ((step + 1) & 1) * 32 * 1024 + lane * 16;
  f16x8 fa[4][2], fw[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      fa[i][p] = *reinterpret_cast<const f16x8*>(fr + (i * 2 + p) * 1024);
      fw[i][p] = *reinterpret_cast<const f16x8*>(fr + 8192 + (i * 2 + p) * 1024);
    }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][1], fa[i][0], acc[i][j], 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][1], acc[i][j], 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][0], acc[i][j], 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}

// Software-pipelined form (as the edge kernels): the fragments of step s were read during step s-1;
// half of the MFMAs, the step's barrier (supplied by the caller between the halves: `mid`), then the
// other half with the next step's 16 fragment reads spread between them (one read per MFMA pair
// slot, sched_group_barrier).
template <class Mid>
__device__ __forceinline__ void main_step_pipe(const char* lds, const char* gsrc, int lane, int wave, int step,
                                               f32x4 (&acc)[4][4], f16x8 (&fa)[2][4][2], f16x8 (&fw)[2][4][2],
                                               int cur, Mid&& mid) {
  char* ring = (char*)lds + (wave >> 2) * (64 * 1024) + (step & 1) * 32 * 1024 + (wave & 3) * 8 * 1024;
  const char* src = gsrc + ((long)((blockIdx.x & 15) * 8 + wave) * 8 + (step & 7)) * 8192 + lane * 16;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    __builtin_amdgcn_global_load_lds((gbl_void*)(src + q * 1024), (lds_void*)(ring + q * 1024), 16, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[cur][j][1], fa[cur][i][0], acc[i][j], 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[cur][j][0], fa[cur][i][1], acc[i][j], 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  mid();
  const char* fr = lds + (wave >> 2) * (64 * 1024) + ((step + 1) & 1) * 32 * 1024 + lane * 16;
  const int nx = cur ^ 1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      fa[nx][i][p] = *reinterpret_cast<const f16x8*>(fr + (i * 2 + p) * 1024);
      fw[nx][i][p] = *reinterpret_cast<const f16x8*>(fr + 8192 + (i * 2 + p) * 1024);
    }
#pragma unroll
  for (int j = 2; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[cur][j][0], fa[cur][i][1], acc[i][j], 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[cur][j][0], fa[cur][i][0], acc[i][j], 0, 0, 0);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
  }
  __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): next step's fragments are in
}

template <int E>
__device__ __forceinline__ void epi_step(const char* lds, _Float16* gdst, int lane, int wave, int step, float& mx,
                                         f32x4 (&v)[4][4]) {
  const float* pq = reinterpret_cast<const float*>(lds + (wave >> 2) * (64 * 1024) + lane * 16);
  _Float16* out = gdst + ((long)(blockIdx.x * 8 + wave) * 64 + (step & 63)) * 1024 + lane * 8;
#pragma unroll
  for (int e4 = 0; e4 < E; e4 += 4) {
    const f32x4 p = *reinterpret_cast<const f32x4*>(pq + (e4 & 15) * 64);
    const f32x4 q = *reinterpret_cast<const f32x4*>(pq + 4096 + (e4 & 15) * 64);
    f16x8 hl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = v[(e4 >> 2) & 3][(e4 >> 4) & 3][r] + p[r] + q[r];
      x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      mx = fmaxf(mx, fabsf(x));
      const float xs = x * 0.5f;
      const _Float16 h = (_Float16)xs;
      hl[2 * r] = h;
      hl[2 * r + 1] = (_Float16)(xs - (float)h);
      v[(e4 >> 2) & 3][(e4 >> 4) & 3][r] = x;
    }
    *reinterpret_cast<f16x8*>(out + (e4 >> 2) * 512) = hl;
  }
}

template <int MODE, int E>
__global__ __launch_bounds__(512, 1) void k_probe(const char* gsrc, _Float16* gdst, float* sink, int steps,
                                                  unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  for (int k = tid; k < LDS_BYTES / 4; k += 512) reinterpret_cast<float*>(lds)[k] = 0.001f * (k & 255);
  __syncthreads();
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.01f * i, 0.02f * j, 0.f, 1.f};
  float mx = 0.f;
  const int mode = MODE & 3;
  const bool do_main = mode == 0 || (grp == 0 && mode != 3);
  const bool do_epi = grp == 1 && (mode == 1 || mode == 3);
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  if constexpr ((MODE & 4) == 0) {
    for (int s = 0; s < steps; ++s) {
      if (do_main) main_step(lds, gsrc, lane, wave, s, acc);
      if (do_epi) epi_step<E>(lds, gdst, lane, wave, s, mx, acc);
      __builtin_amdgcn_s_barrier();
    }
  } else {  // pipelined main loop; the epilogue group does its step before the shared barrier
    f16x8 fa[2][4][2], fw[2][4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        fa[0][i][p] = *reinterpret_cast<const f16x8*>(lds + lane * 16 + (i * 2 + p) * 1024);
        fw[0][i][p] = *reinterpret_cast<const f16x8*>(lds + lane * 16 + 8192 + (i * 2 + p) * 1024);
        fa[1][i][p] = fa[0][i][p];
        fw[1][i][p] = fw[0][i][p];
      }
    auto bar = [] { __builtin_amdgcn_s_barrier(); };
    for (int s = 0; s < steps; s += 2) {
      if (do_main) {
        main_step_pipe(lds, gsrc, lane, wave, s, acc, fa, fw, 0, bar);
        main_step_pipe(lds, gsrc, lane, wave, s + 1, acc, fa, fw, 1, bar);
      } else {
        if (do_epi) epi_step<E>(lds, gdst, lane, wave, s, mx, acc);
        __builtin_amdgcn_s_barrier();
        if (do_epi) epi_step<E>(lds, gdst, lane, wave, s + 1, mx, acc);
        __builtin_amdgcn_s_barrier();
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  float t = mx;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][3];
  if (t == 1234.5f) sink[tid] = t;
  if (tid == 0) clk[blockIdx.x] = c1 - c0;
}

template <int MODE, int E>
double run(const char* gsrc, _Float16* gdst, float* sink, unsigned long long* clk, int blocks, int steps, double* cyc) {
  (void)hipFuncSetAttribute((const void*)k_probe<MODE, E>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL((k_probe<MODE, E>), dim3(blocks), dim3(512), LDS_BYTES, 0, gsrc, gdst, sink, steps, clk);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k_probe<MODE, E>), dim3(blocks), dim3(512), LDS_BYTES, 0, gsrc, gdst, sink, steps, clk);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(blocks);
  (void)hipMemcpy(h.data(), clk, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double s = 0;
  for (auto v : h) s += (double)v;
  *cyc = s / blocks / steps;  // s_memtime ticks (100 MHz constant clock on gfx9: x the shader clock ratio)
  return ms * 1e3 / steps;    // us per step
}

int main(int argc, char** argv) {
  int dev = 0, ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = ncu, steps = argc > 1 ? atoi(argv[1]) : 4800;
  char* gsrc;
  _Float16* gdst;
  float* sink;
  unsigned long long* clk;
  const size_t srcb = (size_t)blocks * 8 * 64 * 8192;
  (void)hipMalloc(&gsrc, srcb);
  (void)hipMemset(gsrc, 0x11, srcb);
  (void)hipMalloc(&gdst, (size_t)blocks * 8 * 64 * 1024 * 2 * 2);
  (void)hipMalloc(&sink, 4096);
  (void)hipMalloc(&clk, blocks * sizeof(unsigned long long));
  const double flops_main = 48.0 * 16 * 16 * 32 * 2;  // per wave per step
  printf("CUs %d, steps %d; per step per wave: 48 x 16x16x32 f16 MFMA (%.0f flop), 8 glds, 16 ds_read_b128\n", ncu,
         steps, flops_main);
  for (int rep = 0; rep < 2; ++rep) {
    double c;
    double t0 = run<4, 8>(gsrc, gdst, sink, clk, blocks, steps, &c);
    printf("PIPELINED mode 0 both groups main loop : %7.3f us/step  %6.0f TF/s (2 waves/SIMD)\n", t0,
           flops_main * 8 * blocks / (t0 * 1e-6) / 1e12);
    double t2 = run<6, 8>(gsrc, gdst, sink, clk, blocks, steps, &c);
    printf("PIPELINED mode 2 main loop alone       : %7.3f us/step  %6.0f TF/s (1 wave/SIMD)\n", t2,
           flops_main * 4 * blocks / (t2 * 1e-6) / 1e12);
#define EPIP(E)                                                                                                    \
  {                                                                                                                \
    double t1 = run<5, E>(gsrc, gdst, sink, clk, blocks, steps, &c);                                              \
    printf("PIPELINED E=%2d ping-pong %7.3f us/step = %.2f x main alone, %6.0f TF/s\n", E, t1, t1 / t2,            \
           flops_main * 4 * blocks / (t1 * 1e-6) / 1e12);                                                         \
  }
    EPIP(4) EPIP(8) EPIP(12)
  }
  for (int rep = 0; rep < 1; ++rep) {
    double c;
    double t0 = run<0, 8>(gsrc, gdst, sink, clk, blocks, steps, &c);
    printf("mode 0 both groups main loop : %7.3f us/step  %6.0f TF/s (2 waves/SIMD)\n", t0,
           flops_main * 8 * blocks / (t0 * 1e-6) / 1e12);
    double t2 = run<2, 8>(gsrc, gdst, sink, clk, blocks, steps, &c);
    printf("mode 2 main loop alone       : %7.3f us/step  %6.0f TF/s (1 wave/SIMD)\n", t2,
           flops_main * 4 * blocks / (t2 * 1e-6) / 1e12);
    const double tm = t2;
#define EPI(E)                                                                                                     \
  {                                                                                                                \
    double t3 = run<3, E>(gsrc, gdst, sink, clk, blocks, steps, &c);                                              \
    double t1 = run<1, E>(gsrc, gdst, sink, clk, blocks, steps, &c);                                              \
    printf("E=%2d epilogue alone %7.3f us/step | ping-pong %7.3f us/step = %.2f x main alone, %6.0f TF/s\n", E, t3, \
           t1, t1 / tm, flops_main * 4 * blocks / (t1 * 1e-6) / 1e12);                                           \
  }
    EPI(4) EPI(8) EPI(12) EPI(16)
  }
  return 0;
}
