// Standalone microbenchmark of the decoder GEMM kernels (edge shapes at 512x40).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCHM_MICROBENCH tools/gemm_bench.cpp chemeleon_amd/csrc/kernels.hip \
//         chemeleon_amd/csrc/gemm_bf16x3.hip chemeleon_amd/csrc/split16.hip chemeleon_amd/csrc/edge16.hip \
//         chemeleon_amd/csrc/node_gemm.hip -o tools/gemm_bench && tools/gemm_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <functional>
#include <cmath>
#include <string>

#include "../chemeleon_amd/csrc/chm_internal.h"

using namespace chm;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void split_h(const float* x, long n, _Float16* out) {  // split rows [..][K/32][2][32]
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const _Float16 h = (_Float16)x[i];
  const long o = (i / 32) * 64 + i % 32;
  out[o] = h;
  out[o + 32] = (_Float16)(x[i] - (float)h);
}

__global__ void k_empty() {}

__global__ void fill(float* p, long n, unsigned seed, float scale) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)(i * 2654435761u) ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  p[i] = ((x & 0xFFFFFF) / 16777216.0f - 0.5f) * scale;
}

static float time_it(int reps, hipStream_t s, const std::function<void()>& f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const long M = argc > 1 ? atol(argv[1]) : 2L * 819200;  // rows (2E for the message GEMM)
  const int N = argc > 4 ? atoi(argv[4]) : 512;
  const int K = argc > 2 ? atoi(argv[2]) : 512;
  hipStream_t s; CK(hipStreamCreate(&s));
  float *A, *W, *C, *bias;
  void* W3;
  CK(hipMalloc(&A, M * K * 4)); CK(hipMalloc(&W, (long)N * K * 4)); CK(hipMalloc(&C, M * N * 4));
  CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&W3, 3L * N * K * 2));
  fill<<<(M * K + 255) / 256, 256, 0, s>>>(A, M * K, 1, 2.0f);
  fill<<<(N * K + 255) / 256, 256, 0, s>>>(W, (long)N * K, 2, 0.1f);
  fill<<<(N + 255) / 256, 256, 0, s>>>(bias, N, 3, 0.1f);
  CK(split_planes(W, (long)N * K, W3, s));
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = K; g.A2 = A; g.lda2 = K; g.ksplit = K;
  g.W = W; g.ldw = K; g.C = C; g.ldc = N; g.bias = bias; g.act = 1; g.gb_rowmod = 1; g.Wp3 = W3;
  const double flops = 2.0 * M * N * K;
  if (argc > 3 && std::string(argv[3]) == "edge") {  // glds edge GEMM only (PMC runs); "edge0" = no C stores
    void* W2h; float* wsc; _Float16* Ah;
    CK(hipMalloc(&W2h, 2L * N * K * 2)); CK(hipMalloc(&wsc, N * 4)); CK(hipMalloc(&Ah, 2L * M * K * 2));
    CK(split_rows_h(W, N, K, W2h, wsc, 0, s));
    split_h<<<(M * K + 255) / 256, 256, 0, s>>>(A, M * K, Ah);
    EdgeArgs ea{};
    ea.M = M; ea.N = N; ea.K = K; ea.A = Ah; ea.W = W2h; ea.wscale = wsc; ea.C = C; ea.ldc = N;
    float te = time_it(5, s, [&] { CK(edge_gemm16(ea, EPI_STD, s)); });
    ea.C = nullptr;
    float t0 = time_it(5, s, [&] { CK(edge_gemm16(ea, EPI_STD, s)); });
    printf("M=%ld K=%d glds edge GEMM: %.3f ms %.1f TF fp32-eq; without C stores %.3f ms %.1f TF\n", M, K, te,
           flops / te / 1e9, t0, flops / t0 / 1e9);
    for (int dbg = 1; dbg < 4; ++dbg) {
      ea.dbg = dbg;
      float td = time_it(5, s, [&] { CK(edge_gemm16(ea, EPI_STD, s)); });
      printf("  ablation %d (%s%s): %.3f ms %.1f TF\n", dbg, dbg & 1 ? "no loop loads " : "", dbg & 2 ? "no barriers" : "",
             td, flops / td / 1e9);
    }
    ea.dbg = 0;
    return 0;
  }
  if (argc > 3 && std::string(argv[3]) == "f16") {  // fp16x2 big only (PMC runs)
    float* wsc;
    CK(hipMalloc(&wsc, N * 4));
    printf("M=%ld N=%d K=%d\n", M, N, K);
    // glds edge GEMM on pre-split rows
    _Float16* Ah; int* aexp; void* W2r;
    CK(hipMalloc(&Ah, 2L * M * K * 2)); CK(hipMalloc(&aexp, M * 4)); CK(hipMemset(aexp, 0, M * 4));
    CK(hipMalloc(&W2r, 2L * N * K * 2));
    CK(split_rows_h(W, N, K, W2r, wsc, 0, s));
    split_h<<<(M * K + 255) / 256, 256, 0, s>>>(A, M * K, Ah);
    EdgeArgs ea{};
    ea.M = M; ea.N = N; ea.K = K; ea.A = Ah; ea.W = W2r; ea.wscale = wsc; ea.C = C; ea.ldc = N;
    float te = time_it(5, s, [&] { CK(edge_gemm16(ea, EPI_STD, s)); });
    printf("  glds edge GEMM: %.3f ms %.1f TF fp32-equivalent\n", te, flops / te / 1e9);
    std::vector<float> c1(65536 * 4), c2(65536 * 4);
    GemmArgs gp = g; gp.bias = nullptr; gp.act = 0;
    CK(gemm(gp, EPI_STD, s)); CK(hipStreamSynchronize(s));
    CK(hipMemcpy(c1.data(), C, c1.size() * 4, hipMemcpyDeviceToHost));
    CK(edge_gemm16(ea, EPI_STD, s)); CK(hipStreamSynchronize(s));
    CK(hipMemcpy(c2.data(), C, c2.size() * 4, hipMemcpyDeviceToHost));
    double mx = 0, ref = 0;
    for (size_t i = 0; i < c1.size(); ++i) { mx = fmax(mx, fabs((double)c1[i] - c2[i])); ref = fmax(ref, fabs((double)c1[i])); }
    printf("  max |edge - f32mfma| = %.3e (max |C| %.3e)\n", mx, ref);
    if (K % 128 == 0 && K <= 512) {
      ea.aexp = aexp;
      float ta = time_it(5, s, [&] { CK(edge_gemm16(ea, EPI_STD, s)); });
      CK(hipMemcpy(c2.data(), C, c2.size() * 4, hipMemcpyDeviceToHost));
      mx = 0;
      for (size_t i = 0; i < c1.size(); ++i) mx = fmax(mx, fabs((double)c1[i] - c2[i]));
      printf("  glds edge GEMM, chunk-scaled A: %.3f ms %.1f TF, max err %.3e\n", ta, flops / ta / 1e9, mx);
    }
    return 0;
  }
  if (argc > 3 && std::string(argv[3]) == "nodefix") {  // split16 node GEMM time vs K (fixed cost = intercept)
    CK(node_gemm_init());
    void* W16; float* wsc16; float* amax;
    CK(hipMalloc(&W16, 2L * N * K * 2)); CK(hipMalloc(&wsc16, N * 4)); CK(hipMalloc(&amax, M * 4));
    CK(split_rows_h(W, N, K, W16, wsc16, 0, s, 16));
    std::vector<float> one(M, 1.0f);
    CK(hipMemcpy(amax, one.data(), M * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep)
      for (int k = 64; k <= K; k *= 2) {
        GemmArgs g16 = g; g16.Wp3 = W16; g16.wscale = wsc16; g16.amax = amax; g16.K = k; g16.ksplit = k;
        g16.lda = K; g16.lda2 = K;
        float t = time_it(50, s, [&] { CK(node_gemm(g16, s)); });
        GemmArgs g0 = g16; g0.bias = nullptr; g0.act = 0;
        float t0 = time_it(50, s, [&] { CK(node_gemm(g0, s)); });
        float tr[2][3];  // [64 / 128 rows][2, 3, 4 blocks per CU]
        for (int r = 0; r < 2; ++r)
          for (int nb = 2; nb <= 4; ++nb) {
            tr[r][nb - 2] = 0.f;
            if ((r == 0 && nb == 2) || (r == 1 && nb == 4)) continue;
            g_node_rows = r ? 128 : 64;
            g_node_blocks = nb;
            tr[r][nb - 2] = time_it(50, s, [&] { CK(node_gemm(g16, s)); });
          }
        // bit-identity of the 64-row tiling against the 128-row one
        const size_t nc = (size_t)M * N;
        std::vector<float> c64(nc), c128(nc);
        g_node_rows = 64; g_node_blocks = 3;
        CK(node_gemm(g16, s)); CK(hipStreamSynchronize(s));
        CK(hipMemcpy(c64.data(), C, nc * 4, hipMemcpyDeviceToHost));
        g_node_rows = 128; g_node_blocks = 2;
        CK(node_gemm(g16, s)); CK(hipStreamSynchronize(s));
        CK(hipMemcpy(c128.data(), C, nc * 4, hipMemcpyDeviceToHost));
        g_node_rows = 0; g_node_blocks = 0;
        printf("M=%ld N=%d K=%d: default %.2f us (no bias/act %.2f us) | 128 rows: 2 blocks/CU %.2f, 3 %.2f | "
               "64 rows: 3 blocks/CU %.2f, 4 %.2f us | 64-row bit-identical: %s\n", M, N, k, t * 1e3, t0 * 1e3,
               tr[1][0] * 1e3, tr[1][1] * 1e3, tr[0][1] * 1e3, tr[0][2] * 1e3, c64 == c128 ? "yes" : "NO");
      }
    float te = time_it(50, s, [&] { hipLaunchKernelGGL(k_empty, dim3(160), dim3(256), 0, s); });
    printf("empty kernel, 160 blocks: %.2f us per launch\n", te * 1e3);
    return 0;
  }
  if (argc > 3 && std::string(argv[3]) == "node64") {  // short grids: 64x128 vs 64x64 split16 node tiles
    CK(node_gemm_init());
    void* W16; float* wsc16; float* amax;
    CK(hipMalloc(&W16, 2L * N * K * 2)); CK(hipMalloc(&wsc16, N * 4)); CK(hipMalloc(&amax, M * 4));
    CK(split_rows_h(W, N, K, W16, wsc16, 0, s, 16));
    std::vector<float> one(M, 1.0f);
    CK(hipMemcpy(amax, one.data(), M * 4, hipMemcpyHostToDevice));
    GemmArgs g16 = g; g16.Wp3 = W16; g16.wscale = wsc16; g16.amax = amax;
    const size_t nc = (size_t)M * N;
    std::vector<float> c0(nc), c1(nc);
    for (int rep = 0; rep < 2; ++rep) {
      float t[3];
      const int cols[3] = {128, 64, 128};
      for (int v = 0; v < 3; ++v) {
        g_node_rows = 64; g_node_blocks = 3; g_node_cols = cols[v];
        t[v] = time_it(50, s, [&] { CK(node_gemm(g16, s)); });
      }
      g_node_rows = 64; g_node_blocks = 3; g_node_cols = 128;
      CK(node_gemm(g16, s)); CK(hipStreamSynchronize(s));
      CK(hipMemcpy(c0.data(), C, nc * 4, hipMemcpyDeviceToHost));
      CK(hipMemset(C, 0, nc * 4));
      g_node_cols = 64;
      CK(node_gemm(g16, s)); CK(hipStreamSynchronize(s));
      CK(hipMemcpy(c1.data(), C, nc * 4, hipMemcpyDeviceToHost));
      g_node_rows = 0; g_node_blocks = 0; g_node_cols = 0;
      printf("M=%ld N=%d K=%d: 64x128 tiles %.2f us | 64x64 tiles %.2f us | 64x128 again %.2f us | bit-identical: %s\n",
             M, N, K, t[0] * 1e3, t[1] * 1e3, t[2] * 1e3, c0 == c1 ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::string(argv[3]) == "s16order") {  // split16 default vs explicit 128-row / 3-block launch, interleaved
    CK(node_gemm_init());
    void* W16; float* wsc16; float* amax;
    CK(hipMalloc(&W16, 2L * N * K * 2)); CK(hipMalloc(&wsc16, N * 4)); CK(hipMalloc(&amax, M * 4));
    CK(split_rows_h(W, N, K, W16, wsc16, 0, s, 16));
    std::vector<float> one(M, 1.0f);
    CK(hipMemcpy(amax, one.data(), M * 4, hipMemcpyHostToDevice));
    GemmArgs g16 = g; g16.Wp3 = W16; g16.wscale = wsc16; g16.amax = amax;
    for (int rep = 0; rep < 4; ++rep) {
      g_node_rows = 0; g_node_blocks = 0;
      float td = time_it(50, s, [&] { CK(node_gemm(g16, s)); });
      g_node_rows = 128; g_node_blocks = 3;
      float te = time_it(50, s, [&] { CK(node_gemm(g16, s)); });
      g_node_rows = 0; g_node_blocks = 0;
      printf("split16 M=%ld N=%d K=%d: default %.2f us | explicit 128 rows x 3 blocks %.2f us\n", M, N, K, td * 1e3, te * 1e3);
    }
    return 0;
  }
  if (argc > 3 && std::string(argv[3]) == "b3rows") {  // bf16x3 node GEMM: 128- vs 64-row tiles (short grids)
    CK(node_gemm_init());
    const size_t nc = (size_t)M * N;
    std::vector<float> c128(nc), c64(nc);
    for (int rep = 0; rep < 2; ++rep) {
      g_node_rows = 128;
      float t128 = time_it(50, s, [&] { CK(node_gemm(g, s)); });
      CK(node_gemm(g, s)); CK(hipStreamSynchronize(s));
      CK(hipMemcpy(c128.data(), C, nc * 4, hipMemcpyDeviceToHost));
      CK(hipMemset(C, 0, nc * 4));
      g_node_rows = 64;
      float t64 = time_it(50, s, [&] { CK(node_gemm(g, s)); });
      CK(node_gemm(g, s)); CK(hipStreamSynchronize(s));
      CK(hipMemcpy(c64.data(), C, nc * 4, hipMemcpyDeviceToHost));
      g_node_rows = 0;
      printf("bf16x3 M=%ld N=%d K=%d: 128-row tiles %.2f us | 64-row tiles %.2f us | bit-identical: %s\n", M, N, K,
             t128 * 1e3, t64 * 1e3, c128 == c64 ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::string(argv[3]) == "node") {  // node GEMM shapes: glds kernel vs register-staged
    CK(node_gemm_init());
    for (int rep = 0; rep < 2; ++rep) {
      g_gemm3_variant = 0;
      float tr = time_it(10, s, [&] { CK(gemm_bf16x3(g, EPI_STD, s)); });
      float tn = time_it(10, s, [&] { CK(node_gemm(g, s)); });
      GemmArgs g0 = g; g0.bias = nullptr; g0.act = 0;
      float tn0 = time_it(10, s, [&] { CK(node_gemm(g0, s)); });
      g_node_variant = 1;
      float tv = time_it(10, s, [&] { CK(node_gemm(g0, s)); });
      g_node_variant = 0;
      printf("M=%ld N=%d K=%d  k_gemm3 %.1f us %.1f TF | k_node_gemm %.1f us %.1f TF (no bias/act %.1f us, no split %.1f us)\n",
             M, N, K, tr * 1e3, flops / tr / 1e9, tn * 1e3, flops / tn / 1e9, tn0 * 1e3, tv * 1e3);
    }
    // split16 variant: W as 16-column fp16 hi/lo rows with row scales
    void* W16; float* wsc16;
    CK(hipMalloc(&W16, 2L * N * K * 2)); CK(hipMalloc(&wsc16, N * 4));
    CK(split_rows_h(W, N, K, W16, wsc16, 0, s, 16));
    GemmArgs g16 = g; g16.Wp3 = W16; g16.wscale = wsc16;
    for (int rep = 0; rep < 2; ++rep) {
      float t16 = time_it(10, s, [&] { CK(node_gemm(g16, s)); });
      GemmArgs g160 = g16; g160.bias = nullptr; g160.act = 0;
      float t160 = time_it(10, s, [&] { CK(node_gemm(g160, s)); });
      g_node_variant = 1;
      float t16v = time_it(10, s, [&] { CK(node_gemm(g160, s)); });
      g_node_variant = 0;
      printf("  split16 k_node_gemm %.1f us %.1f TF (no bias/act %.1f us, no split %.1f us)\n", t16 * 1e3,
             flops / t16 / 1e9, t160 * 1e3, t16v * 1e3);
    }
    for (int nb : {2, 3}) {
      g_node_blocks = nb;
      float tb = time_it(10, s, [&] { CK(node_gemm(g16, s)); });
      printf("  split16 %d blocks/CU: %.1f us %.1f TF\n", nb, tb * 1e3, flops / tb / 1e9);
    }
    g_node_blocks = 3;
    CK(node_gemm(g16, s)); CK(hipStreamSynchronize(s));
    g_node_blocks = 0;
    {
      std::vector<float> r3((size_t)std::min<long>(M, 4096) * N), r2(r3.size());
      CK(hipMemcpy(r3.data(), C, r3.size() * 4, hipMemcpyDeviceToHost));
      CK(node_gemm(g16, s)); CK(hipStreamSynchronize(s));
      CK(hipMemcpy(r2.data(), C, r2.size() * 4, hipMemcpyDeviceToHost));
      printf("  3 blocks/CU bit-identical to 2: %s\n", r2 == r3 ? "yes" : "NO");
    }
    const size_t nc = (size_t)std::min<long>(M, 4096) * N;
    std::vector<float> c1(nc), c2(nc), c3(nc);
    CK(gemm(g, EPI_STD, s)); CK(hipStreamSynchronize(s));  // fp32 MFMA reference
    CK(hipMemcpy(c3.data(), C, nc * 4, hipMemcpyDeviceToHost));
    CK(gemm_bf16x3(g, EPI_STD, s)); CK(hipStreamSynchronize(s));
    CK(hipMemcpy(c1.data(), C, nc * 4, hipMemcpyDeviceToHost));
    CK(node_gemm(g, s)); CK(hipStreamSynchronize(s));
    CK(hipMemcpy(c2.data(), C, nc * 4, hipMemcpyDeviceToHost));
    double mx = 0, e3 = 0, e16 = 0, ref = 0;
    for (size_t i = 0; i < nc; ++i) {
      mx = fmax(mx, fabs((double)c1[i] - c2[i]));
      e3 = fmax(e3, fabs((double)c1[i] - c3[i]));
      ref = fmax(ref, fabs((double)c3[i]));
    }
    CK(node_gemm(g16, s)); CK(hipStreamSynchronize(s));
    CK(hipMemcpy(c2.data(), C, nc * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nc; ++i) e16 = fmax(e16, fabs((double)c2[i] - c3[i]));
    printf("  max |node - gemm3| = %.3e; vs f32 MFMA: bf16x3 %.3e, split16 %.3e (max |C| %.3e)\n", mx, e3, e16, ref);
    return 0;
  }
  float t32 = time_it(5, s, [&] { CK(gemm(g, EPI_STD, s)); });
  printf("M=%ld N=%d K=%d  f32-mfma: %.3f ms %.1f TF\n", M, N, K, t32, flops / t32 / 1e9);
  for (int v = 0; v < 4; ++v) {
    g_gemm3_variant = v;
    float t3 = time_it(5, s, [&] { CK(gemm_bf16x3(g, EPI_STD, s)); });
    printf("  bf16x3 variant %d (prefetch %d, xcd remap %d): %.3f ms %.1f TF fp32-equivalent\n", v, (v & 1) + 1,
           (v >> 1) & 1, t3, flops / t3 / 1e9);
  }
  g_gemm3_variant = 3;
  {
    float tb = time_it(5, s, [&] { CK(gemm_bf16x3_big(g, EPI_STD, s)); });
    printf("  bf16x3 big (256x256, 8 waves): %.3f ms %.1f TF fp32-equivalent\n", tb, flops / tb / 1e9);
    std::vector<float> c1(65536 * 4), c2(65536 * 4);
    CK(gemm_bf16x3(g, EPI_STD, s)); CK(hipStreamSynchronize(s));
    CK(hipMemcpy(c1.data(), C, c1.size() * 4, hipMemcpyDeviceToHost));
    CK(gemm_bf16x3_big(g, EPI_STD, s)); CK(hipStreamSynchronize(s));
    CK(hipMemcpy(c2.data(), C, c2.size() * 4, hipMemcpyDeviceToHost));
    double mx = 0;
    for (size_t i = 0; i < c1.size(); ++i) mx = fmax(mx, fabs((double)c1[i] - c2[i]));
    printf("  max |big - small| = %.3e\n", mx);
  }
  // accuracy of bf16x3 against the f32-MFMA result
  std::vector<float> c32(M > 65536 ? 65536 * N : M * N), c3(c32.size());
  CK(gemm(g, EPI_STD, s)); CK(hipStreamSynchronize(s));
  CK(hipMemcpy(c32.data(), C, c32.size() * 4, hipMemcpyDeviceToHost));
  CK(gemm_bf16x3(g, EPI_STD, s)); CK(hipStreamSynchronize(s));
  CK(hipMemcpy(c3.data(), C, c3.size() * 4, hipMemcpyDeviceToHost));
  double mx = 0, ms = 0;
  for (size_t i = 0; i < c32.size(); ++i) {
    double d = fabs((double)c3[i] - c32[i]);
    mx = d > mx ? d : mx; ms += (double)c32[i] * c32[i];
  }
  printf("max |bf16x3 - f32| = %.3e (rms value %.3e)\n", mx, sqrt(ms / c32.size()));
  return 0;
}
