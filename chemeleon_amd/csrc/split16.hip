// Operand preparation of the split16 GEMMs (edge16.hip, node_gemm.hip): weights split once into
// row-scaled fp16 hi/lo split rows, and the Fourier edge features (cspnet.py:38-52) computed straight
// into that form. Split row = [K/cw][hi cw | lo cw] fp16, x = hi + lo, every scaled entry <= 1.
#include "chm_internal.h"

namespace chm {

#include "edge_common.h"

// W [N][K] -> split rows [N][K/cw][hi cw | lo cw] of W * 2^-e_n, e_n the exponent of
// max_k |W[n][k]| (every scaled entry <= 1), and wscale[n] = 2^e_n. One block per row. cw = 32
// for the edge GEMMs, 16 for the split16 node GEMMs.
// perm 2 (cw = 32): the column permutation within each 32-chunk that edge layer 1's epilogue writes S
// in (k_edge16's C^T fragments: 16a + 4g + r -> 8g + 4a + r), applied to W2's K index.
__global__ __launch_bounds__(256) void k_split_rows_h(const float* __restrict__ W, int K, _Float16* __restrict__ out,
                                                      float* __restrict__ wscale, int perm, int cw) {
  __shared__ float red[4];
  const int n = blockIdx.x;
  const float* row = W + (long)n * K;
  float m = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) m = fmaxf(m, fabsf(row[k]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int e = exp_of(m);
  const float sc = ldexpf(1.0f, -e);
  _Float16* o = out + (long)n * 2 * K;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float x = row[k] * sc;
    const _Float16 hi = (_Float16)x;
    const int c = k % cw;
    const int pc = perm == 2 ? 8 * ((c >> 2) & 3) + 4 * (c >> 4) + (c & 3) : c;  // 16a + 4g + r -> 8g + 4a + r
    o[(k / cw) * 2 * cw + pc] = hi;
    o[(k / cw) * 2 * cw + cw + pc] = (_Float16)(x - (float)hi);
  }
  if (threadIdx.x == 0) wscale[n] = ldexpf(1.0f, e);
}

hipError_t split_rows_h(const float* W, int N, int K, void* out, float* wscale, int perm, hipStream_t s, int chunk) {
  if ((chunk != 32 && chunk != 16) || K % chunk || (perm != 0 && perm != 2) || (perm && chunk != 32))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_split_rows_h, dim3(N), dim3(256), 0, s, W, K, reinterpret_cast<_Float16*>(out), wscale, perm,
                     chunk);
  return hipGetLastError();
}

// Fourier features (cspnet.py:38-52 as k_fourier) written split, rows [768/32][hi 32 | lo 32].
// One thread per (edge, axis, 8 consecutive frequencies): 8 sincosf, four 16-B stores.
// fd != null (knn edges): the edge's displacement is given (cspnet.py:342-343, no % 1.0)
__global__ __launch_bounds__(256) void k_fourier_h(const float* __restrict__ x, const int* __restrict__ ei,
                                                   const int* __restrict__ ej, const float* __restrict__ fd, long E,
                                                   _Float16* __restrict__ F) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int G = NF / 8;  // groups of 8 frequencies per axis
  if (idx >= E * 3 * G) return;
  const long e = idx / (3 * G);
  const int r = (int)(idx - e * 3 * G);
  const int a = r / G, k0 = (r - a * G) * 8;
  float d;
  if (fd) {
    d = fd[e * 3 + a];
  } else {  // torch.remainder(d, 1.0): fmod, negatives shifted by +1 (k_fourier's rem1)
    d = fmodf(__fsub_rn(x[(long)ej[e] * 3 + a], x[(long)ei[e] * 3 + a]), 1.0f);
    if (d < 0.0f) d = __fadd_rn(d, 1.0f);
  }
  f16x8 sh, sl, ch, cl;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float arg = __fmul_rn(d, __fmul_rn(6.28318548202514648f, (float)(k0 + u)));
    float sv, cv;
    sincosf(arg, &sv, &cv);
    sh[u] = (_Float16)sv;
    sl[u] = (_Float16)(sv - (float)sh[u]);
    ch[u] = (_Float16)cv;
    cl[u] = (_Float16)(cv - (float)ch[u]);
  }
  _Float16* f = F + e * (2 * FD);
  const int cs = a * NF + k0, cc = 3 * NF + a * NF + k0;  // feature columns (8-aligned, inside one 32-chunk)
  *reinterpret_cast<f16x8*>(f + (cs / 32) * 64 + cs % 32) = sh;
  *reinterpret_cast<f16x8*>(f + (cs / 32) * 64 + 32 + cs % 32) = sl;
  *reinterpret_cast<f16x8*>(f + (cc / 32) * 64 + cc % 32) = ch;
  *reinterpret_cast<f16x8*>(f + (cc / 32) * 64 + 32 + cc % 32) = cl;
}

hipError_t fourier_h(const float* x, const int* ei, const int* ej, long E, void* F, hipStream_t s, const float* fd) {
  const long n = E * 3 * (NF / 8);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fourier_h, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ei, ej, fd, E,
                     reinterpret_cast<_Float16*>(F));
  return hipGetLastError();
}

}  // namespace chm
