// Per-CU store rate against the number of CUs storing at once: `nb` blocks (one per CU: 160 KB of
// LDS each), every block writes `reps` x 256 KB with edge layer 1's S pattern ("rows": 32 B of a
// 128-B line per lane pair) or whole lines, into its own region of a 3.36 GB buffer.
// Round 5 adds the pair epilogue's pattern ("dpp": each instruction writes 8 rows' whole 128-B lines, a line's
// 8 lanes being l16 in {2m, 2m+1} x g4 = 0..3, so every quarter-wave of 16 lanes holds 32 B of 8 lines) and
// "quad" (8 rows' whole lines again, a line's 8 lanes consecutive: a quarter-wave holds 2 whole lines).
//   hipcc --offload-arch=gfx950 -O3 tools/store_cu_bench.hip -o tools/store_cu_bench && tools/store_cu_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                  \
  do {                                                         \
    hipError_t e_ = (x);                                       \
    if (e_ != hipSuccess) {                                    \
      printf("%s: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                \
    }                                                          \
  } while (0)

template <int PAT>  // 1 rows, 0 lines, 2 dpp, 3 quad
__global__ __launch_bounds__(512) void k_store(char* __restrict__ out, long tiles_per_block, int reps) {
  extern __shared__ char lds[];  // (only to hold one block per CU)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const f32x4 v = {1.f, 2.f, 3.f, (float)tid};
  if (reps < 0) lds[tid] = 0;
  for (int r = 0; r < reps; ++r) {
    char* base = out + ((long)blockIdx.x * tiles_per_block + r % tiles_per_block) * 256L * 1024;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      long off;
      if (PAT == 2) {  // k: 16 row groups of 8 rows x 2 (the st_e / st_o stores), 4 chunks cycled
        const int l16 = lane & 15, g4 = lane >> 4, odd = l16 & 1;
        const int row = wave * 32 + (k >> 2) % 4 * 8 + (l16 >> 1), cc = k & 3;
        off = (long)row * 2048 + cc * 128 + g4 * 16 + odd * 64;
      } else if (PAT == 3) {
        const int row = wave * 32 + (k >> 2) % 4 * 8 + (lane >> 3), cc = k & 3;
        off = (long)row * 2048 + cc * 128 + (lane & 7) * 16;
      } else if (PAT == 1) {
        const int i = k >> 4, j = (k >> 2) & 3, sidx = k & 3;
        const int row = (wave & 3) * 64 + i * 32 + r32;
        const int inl = (sidx & 1) * 16 + (sidx >> 1) * 64 + h * 32;
        off = (long)row * 1024 + ((wave >> 2) * 4 + j) * 128 + inl;
      } else {
        const int row = wave * 32 + k;
        off = (long)row * 1024 + lane * 16;
      }
      *reinterpret_cast<f32x4*>(base + off) = v;
    }
  }
}

int main() {
  const long big = 3360L << 20;
  char* buf;
  CK(hipMalloc(&buf, big));
  for (const void* k : {(const void*)k_store<0>, (const void*)k_store<1>, (const void*)k_store<2>, (const void*)k_store<3>})
    CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 48;  // 12 MB per block
  for (int pass = 0; pass < 2; ++pass)
    for (int rows : {1, 0, 2, 3})
      for (int nb : {8, 32, 64, 128, 192, 256}) {
        const long tpb = big / (256L * 1024) / 256;  // each block's region: 51 tiles of 256 KB
        auto launch = [&] {
          if (rows == 1)
            hipLaunchKernelGGL(k_store<1>, dim3(nb), dim3(512), 160 * 1024, 0, buf, tpb, reps);
          else if (rows == 0)
            hipLaunchKernelGGL(k_store<0>, dim3(nb), dim3(512), 160 * 1024, 0, buf, tpb, reps);
          else if (rows == 2)
            hipLaunchKernelGGL(k_store<2>, dim3(nb), dim3(512), 160 * 1024, 0, buf, tpb, reps);
          else
            hipLaunchKernelGGL(k_store<3>, dim3(nb), dim3(512), 160 * 1024, 0, buf, tpb, reps);
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 3;
        const double bytes = (double)nb * reps * 256 * 1024;
        if (pass == 1)
          printf("%-5s pattern, %3d CUs storing: %.3f ms, %.2f TB/s total, %.1f GB/s per CU\n", rows == 1 ? "rows" : rows == 0 ? "lines" : rows == 2 ? "dpp" : "quad", nb,
                 ms, bytes / (ms * 1e-3) / 1e12, bytes / nb / (ms * 1e-3) / 1e9);
      }
  return 0;
}
