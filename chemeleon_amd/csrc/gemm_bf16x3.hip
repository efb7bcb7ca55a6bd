// fp32-accurate GEMM on gfx950 bf16 matrix cores ("bf16x3").
//
// Each fp32 operand x is split exactly into x = x0 + x1 + x2 + r with
// x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1), |r| <= 2^-24 |x|.
// A product is rebuilt from the six bf16 products whose weight is >= 2^-16:
//   a.w ~ a0w0 + a0w1 + a1w0 + a0w2 + a1w1 + a2w0
// (dropped terms <= ~3 * 2^-24 relative), each exact in fp32 and accumulated
// in fp32 by v_mfma_f32_32x32x16_bf16. Six bf16 MFMAs cost 6/16 of one
// fp32 MFMA for the same product count: 2.67x the fp32-MFMA peak at fp32
// accuracy (MI355X_MICROARCH.md: bf16 MFMA = 16x the f32 MFMA rate).
//
// Tiles: 128x128 output per 256-thread block (4 waves, 2x2, 64x64 each =
// 2x2 accumulators of 32x32), K chunks of 16 (one bf16 k-step); A is read
// as fp32 from global memory, split in registers and staged as three bf16
// planes in LDS; W planes are pre-split [3][N][K]. LDS rows are 24 bf16
// (48 B): conflict-free ds_read_b128 for the MFMA fragments. Two LDS stages,
// register prefetch of the next chunk.
#include "chm_internal.h"

namespace chm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float silu3(float x) { return x / (1.0f + expf(-x)); }

constexpr int XBM = 128, XBN = 128, XBK = 16, XLP = 24;  // LDS row pitch, bf16 elements
constexpr int PLANE = 128 * XLP;                         // bf16 elements per plane per stage

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  const float r2 = r1 - (float)m;
  l = (__bf16)r2;
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm3(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2][6 * PLANE];  // [stage][A0 A1 A2 W0 W1 W2]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = g.N / XBN;
  const int bn = blockIdx.x % ntn;
  const int n0 = bn * XBN;
  long row0, nrows;
  int seg_c = 0;
  int2 seg = {0, 0};
  if (EPI == EPI_SEGMEAN) {
    const long rest = blockIdx.x / ntn;
    seg_c = (int)(rest % g.npairs);
    seg = g.tiles[rest / g.npairs];
    const long es0 = g.node_estart[seg.x];
    const long es1 = (seg.y < g.nnodes) ? g.node_estart[seg.y] : g.E;
    row0 = (long)seg_c * g.E + es0;
    nrows = es1 - es0;
  } else {
    row0 = (long)(blockIdx.x / ntn) * XBM;
    nrows = g.M - row0 < XBM ? g.M - row0 : XBM;
  }
  const __bf16* Wpl = reinterpret_cast<const __bf16*>(g.Wp3);
  const long wplane = (long)g.N * g.K;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  f32x4 ra[2];
  u32x4 rw[3];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx >> 2, c4 = idx & 3;
      const int k = k0 + 4 * c4;
      if (row < nrows) {
        const long m = row0 + row;
        const float* src = (k < g.ksplit) ? g.A + m * g.lda + k : g.A2 + m * g.lda2 + (k - g.ksplit);
        ra[q] = *reinterpret_cast<const f32x4*>(src);
      } else {
        ra[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    const int wr = tid >> 1, wh = tid & 1;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      rw[p] = *reinterpret_cast<const u32x4*>(Wpl + p * wplane + (long)(n0 + wr) * g.K + k0 + 8 * wh);
  };
  auto lstore = [&](int st) {
    __bf16* S = smem[st];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx >> 2, c4 = idx & 3;
      bf16x4 h, m, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 a, b, c;
        split3(ra[q][e], a, b, c);
        h[e] = a; m[e] = b; l[e] = c;
      }
      const int off = row * XLP + 4 * c4;
      *reinterpret_cast<bf16x4*>(S + 0 * PLANE + off) = h;
      *reinterpret_cast<bf16x4*>(S + 1 * PLANE + off) = m;
      *reinterpret_cast<bf16x4*>(S + 2 * PLANE + off) = l;
    }
    const int wr = tid >> 1, wh = tid & 1;
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x4*>(S + (3 + p) * PLANE + wr * XLP + 8 * wh) = rw[p];
  };

  const int h = lane >> 5, r32 = lane & 31;
  const int nk = g.K / XBK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * XBK);
    const __bf16* S = smem[st];
    bf16x8 a[3][2], w[3][2];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[p][i] = *reinterpret_cast<const bf16x8*>(S + p * PLANE + (wm * 64 + i * 32 + r32) * XLP + 8 * h);
        w[p][i] = *reinterpret_cast<const bf16x8*>(S + (3 + p) * PLANE + (wn * 64 + i * 32 + r32) * XLP + 8 * h);
      }
    // small terms first, the leading product last
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], w[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], w[1][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], w[2][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], w[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], w[1][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], w[0][j], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) lstore(st ^ 1);
    __syncthreads();
  }

  if (EPI == EPI_SEGMEAN) {
    // messages m = SiLU(acc + b2) -> LDS tile [128][129] fp32 -> per-node column sums in
    // edge order j = 0..n-1 (the reference's scatter_add_ order) -> mean -> agg
    float* T = reinterpret_cast<float*>(&smem[0][0]);
    constexpr int TP = XBN + 1;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int col = wn * 64 + j * 32 + r32;
          T[row * TP + col] = silu3(acc[i][j][r] + g.bias[n0 + col]);
        }
    __syncthreads();
    const int col = tid & (XBN - 1);
    const long es0 = g.node_estart[seg.x];
    for (int nd = seg.x + (tid >> 7); nd < seg.y; nd += 2) {
      const int n = g.natoms[g.n2g[nd]];
      const int r0 = (int)(g.node_estart[nd] - es0);
      float s = 0.f;
      for (int j = 0; j < n; ++j) s += T[(r0 + j) * TP + col];
      g.agg[((long)seg_c * g.nnodes + nd) * g.ldc + n0 + col] = s / (float)(n < 1 ? 1 : n);
    }
    return;
  }

#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long lrow = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (lrow >= nrows) continue;
      const long row = row0 + lrow;
      if (EPI == EPI_EDGE) {
        const long ii = g.ei[row], jj = g.ej[row];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wn * 64 + j * 32 + r32;
          const float v = acc[i][j][r];
          for (int c = 0; c < g.npairs; ++c) {
            const float p = g.PQ[(c * g.nnodes + ii) * (2 * H) + col];
            const float q = g.PQ[(c * g.nnodes + jj) * (2 * H) + H + col];
            g.C[((long)c * g.E + row) * g.ldc + col] = silu3((v + p) + q);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wn * 64 + j * 32 + r32;
          float v = acc[i][j][r];
          if (g.bias) v += g.bias[col];
          if (g.gb && col < g.gb_cols) v += g.gb[(long)g.row2g[row % g.gb_rowmod] * g.ldgb + col];
          if (g.act == 1) v = silu3(v);
          if (g.R) v += g.R[row * g.ldr + col];
          g.C[row * g.ldc + col] = v;
        }
      }
    }
  }
}

hipError_t gemm_bf16x3(const GemmArgs& g, int epi, hipStream_t s) {
  if (g.N % XBN || g.K % XBK || !g.Wp3) return hipErrorInvalidValue;
  if (g.ksplit % XBK) return hipErrorInvalidValue;
  long blocks;
  if (epi == EPI_SEGMEAN) {
    if (g.N != H || !g.tiles || !g.agg) return hipErrorInvalidValue;
    blocks = (long)g.ntiles * g.npairs * (g.N / XBN);
  } else {
    if (g.M <= 0) return hipErrorInvalidValue;
    blocks = ((g.M + XBM - 1) / XBM) * (g.N / XBN);
  }
  if (epi == EPI_EDGE)
    hipLaunchKernelGGL(k_gemm3<EPI_EDGE>, dim3((unsigned)blocks), dim3(256), 0, s, g);
  else if (epi == EPI_SEGMEAN)
    hipLaunchKernelGGL(k_gemm3<EPI_SEGMEAN>, dim3((unsigned)blocks), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(k_gemm3<EPI_STD>, dim3((unsigned)blocks), dim3(256), 0, s, g);
  return hipGetLastError();
}

__global__ void k_split_planes(const float* __restrict__ src, long n, __bf16* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  __bf16 a, b, c;
  split3(src[i], a, b, c);
  dst[i] = a;
  dst[n + i] = b;
  dst[2 * n + i] = c;
}

hipError_t split_planes(const float* src, long n, void* dst, hipStream_t s) {
  hipLaunchKernelGGL(k_split_planes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, n,
                     reinterpret_cast<__bf16*>(dst));
  return hipGetLastError();
}

}  // namespace chm
