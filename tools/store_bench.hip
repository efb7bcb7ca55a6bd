// Store-path microbenchmark: the rate at which all CUs can write S-like data.
//   hipcc --offload-arch=gfx950 -O3 tools/store_bench.hip -o tools/store_bench && tools/store_bench
// Pattern "rows": each store instruction writes 16 B per lane into 32 rows of 2 KB (two lanes per
// row, 32 B per 128-B line), as edge layer 1's epilogue does. Pattern "lines": each instruction
// writes 1 KB contiguous (8 whole lines). Targets: a 3.36 GB buffer (HBM) and a 16 MB buffer that
// every block rewrites (L2-resident), and (`tools/store_bench sweep`) targets of 32-512 MB that the
// same 3.36 GB of stores cycle through (Infinity-Cache-sized). One 512-thread block per CU, 256 KB
// per block per pass.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <initializer_list>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                                        \
      return 1;                                                                             \
    }                                                                                       \
  } while (0)

// block b writes column half (b & 1) of row tile (b >> 1) % ntiles: 256 rows x 1 KB (256 KB)
template <bool ROWS>
__global__ __launch_bounds__(512) void k_store(char* __restrict__ out, long ntiles, int reps) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const long tile = (blockIdx.x >> 1) % ntiles;
  char* base = out + tile * 256L * 2048 + (blockIdx.x & 1) * 1024;  // rows of 2 KB, this block's half
  const f32x4 v = {1.f, 2.f, 3.f, (float)tid};
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {  // 32 instructions x 1 KB per wave = 32 KB per wave, 256 KB per block
      long off;
      if (ROWS) {  // edge layer 1's S stores: k = (i, j, s); lanes h = 0, 1 of a row 32 B apart
        const int i = k >> 4, j = (k >> 2) & 3, sidx = k & 3;
        const int row = (wave & 3) * 64 + i * 32 + r32;
        const int inl = (sidx & 1) * 16 + (sidx >> 1) * 64 + h * 32;
        off = (long)row * 2048 + ((wave >> 2) * 4 + j) * 128 + inl;
      } else {  // the same 256 KB, 1 KB contiguous per instruction (whole lines)
        const int row = wave * 32 + k;
        off = (long)row * 2048 + lane * 16;
      }
      *reinterpret_cast<f32x4*>(base + off) = v;
    }
  }
}

int main(int argc, char** argv) {
  const bool sweep = argc > 1;
  const long big = 3360L << 20, small = 16L << 20;
  char* buf;
  CK(hipMalloc(&buf, big));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int pass = 0; pass < 2; ++pass)
    for (int rows = 1; rows >= 0; --rows)
      for (long sz : sweep ? std::initializer_list<long>{big, 512L << 20, 256L << 20, 192L << 20, 128L << 20, 64L << 20, 32L << 20, small}
                           : std::initializer_list<long>{big, small}) {
        const long ntiles = sz / (256L * 2048);
        const long blocks = 2 * (big / (256L * 2048));  // same bytes written in every case
        auto launch = [&] {
          if (rows)
            hipLaunchKernelGGL(k_store<true>, dim3((unsigned)blocks), dim3(512), 0, 0, buf, ntiles, 1);
          else
            hipLaunchKernelGGL(k_store<false>, dim3((unsigned)blocks), dim3(512), 0, 0, buf, ntiles, 1);
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 5; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        if (pass == 1)
          printf("%-5s pattern, %5ld MB target: %.3f ms for %.2f GB = %.2f TB/s\n", rows ? "rows" : "lines",
                 sz >> 20, ms, big / 1e9, big / (ms * 1e-3) / 1e12);
      }
  return 0;
}
