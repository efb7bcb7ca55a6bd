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
// epilogue SiLU: hardware exp2 + reciprocal (~2 ulp; the reference's own
// x / (1 + exp(-x)) is matched to ~1e-7 relative)
__device__ __forceinline__ float silu_fast(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}

constexpr int XBM = 128, XBN = 128, XBK = 16, XLP = 24;  // LDS row pitch, bf16 elements
constexpr int PLANE = 128 * XLP;                         // bf16 elements per plane per stage

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  const float r2 = r1 - (float)m;
  l = (__bf16)r2;
}

// blocks that share A rows (same row tile, different column tiles) are placed on
// one XCD (blocks b, b+8, ... share an XCD): bijective remap of the linear id
__device__ __forceinline__ long xcd_remap(long b, long nb) {
  const long q = nb / 8, r = nb % 8, xcd = b % 8, idx = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}


template <int EPI, int PF, int REMAP>
__global__ __launch_bounds__(256, 2) void k_gemm3(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2][6 * PLANE];  // [stage][A0 A1 A2 W0 W1 W2]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = g.N / XBN;
  const long bid = REMAP ? xcd_remap(blockIdx.x, gridDim.x) : (long)blockIdx.x;
  const int bn = (int)(bid % ntn);
  const int n0 = bn * XBN;
  long row0, nrows;
  int seg_c = 0;
  int2 seg = {0, 0};
  if (EPI == EPI_SEGMEAN) {
    const long rest = bid / ntn;
    seg_c = (int)(rest % g.npairs);
    seg = g.tiles[rest / g.npairs];
    const long es0 = g.node_estart[seg.x];
    const long es1 = (seg.y < g.nnodes) ? g.node_estart[seg.y] : g.E;
    row0 = (long)seg_c * g.E + es0;
    nrows = es1 - es0;
  } else {
    row0 = (bid / ntn) * XBM;
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

  // per-thread global sources, computed once: A rows are clamped to a valid
  // row (padding rows compute garbage that is never stored or aggregated),
  // so the loads carry no branch and no 64-bit address arithmetic per chunk
  const int arow0 = tid >> 2, c4 = tid & 3;
  const long ar0 = row0 + (arow0 < nrows ? arow0 : nrows - 1);
  const long ar1 = row0 + (arow0 + 64 < nrows ? arow0 + 64 : nrows - 1);
  const float* pa0 = g.A + ar0 * g.lda + 4 * c4;
  const float* pa1 = g.A + ar1 * g.lda + 4 * c4;
  const float* pb0 = g.A2 + ar0 * g.lda2 + 4 * c4 - g.ksplit;
  const float* pb1 = g.A2 + ar1 * g.lda2 + 4 * c4 - g.ksplit;
  const int wr = tid >> 1, wh = tid & 1;
  const __bf16* pw = Wpl + (long)(n0 + wr) * g.K + 8 * wh;

  f32x4 ra[PF][2];
  u32x4 rw[PF][3];
  auto gload = [&](int set, int k0) {
    if (k0 < g.ksplit) {
      ra[set][0] = *reinterpret_cast<const f32x4*>(pa0 + k0);
      ra[set][1] = *reinterpret_cast<const f32x4*>(pa1 + k0);
    } else {
      ra[set][0] = *reinterpret_cast<const f32x4*>(pb0 + k0);
      ra[set][1] = *reinterpret_cast<const f32x4*>(pb1 + k0);
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) rw[set][p] = *reinterpret_cast<const u32x4*>(pw + p * wplane + k0);
  };
  auto lstore = [&](int set, int st) {
    __bf16* S = smem[st];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      bf16x4 h, m, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 a, b, c;
        split3(ra[set][q][e], a, b, c);
        h[e] = a; m[e] = b; l[e] = c;
      }
      const int off = (arow0 + 64 * q) * XLP + 4 * c4;
      *reinterpret_cast<bf16x4*>(S + 0 * PLANE + off) = h;
      *reinterpret_cast<bf16x4*>(S + 1 * PLANE + off) = m;
      *reinterpret_cast<bf16x4*>(S + 2 * PLANE + off) = l;
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x4*>(S + (3 + p) * PLANE + wr * XLP + 8 * wh) = rw[set][p];
  };

  const int h = lane >> 5, r32 = lane & 31;
  auto compute = [&](int st) {
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
    constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
    constexpr int PW[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[PW[t]][j], a[PA[t]][i], acc[i][j], 0, 0, 0);
  };

  const int nk = g.K / XBK;
  if (PF == 1) {
    gload(0, 0);
    lstore(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int st = kt & 1;
      if (kt + 1 < nk) gload(0, (kt + 1) * XBK);
      compute(st);
      if (kt + 1 < nk) lstore(0, st ^ 1);
      __syncthreads();
    }
  } else {
    // two chunks in flight: set 0 holds even chunks, set 1 odd chunks (nk is even)
    gload(0, 0);
    if (nk > 1) gload(1 % PF, XBK);
    lstore(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      if (kt + 2 < nk) gload(0, (kt + 2) * XBK);
      compute(0);
      if (kt + 1 < nk) lstore(1 % PF, 1);
      __syncthreads();
      if (kt + 1 < nk) {
        if (kt + 3 < nk) gload(1 % PF, (kt + 3) * XBK);
        compute(1);
        if (kt + 2 < nk) lstore(0, 0);
        __syncthreads();
      }
    }
  }

  // accumulators hold C^T tiles (W fragments are the MFMA A operand): lane l owns
  // output row wm*64 + i*32 + (l & 31) and, per 4-register group q, the four
  // consecutive columns wn*64 + j*32 + 8q + 4h .. +3
  if (EPI == EPI_SEGMEAN) {
    float* T = reinterpret_cast<float*>(&smem[0][0]);
    constexpr int TP = XBN + 4;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = wn * 64 + j * 32 + 8 * q + 4 * h;
        const f32x4 b = *reinterpret_cast<const f32x4*>(g.bias + n0 + col);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = silu_fast(acc[i][j][4 * q + e] + b[e]);
          *reinterpret_cast<f32x4*>(T + (wm * 64 + i * 32 + r32) * TP + col) = v;
        }
      }
    __syncthreads();
    const int col = tid & (XBN - 1);
    const long es0 = g.node_estart[seg.x];
    for (int nd = seg.x + (tid >> 7); nd < seg.y; nd += 2) {
      const int n = g.natoms[g.n2g[nd]];
      const int r0 = (int)(g.node_estart[nd] - es0);
      float sacc = 0.f;
      for (int j = 0; j < n; ++j) sacc += T[(r0 + j) * TP + col];
      g.agg[((long)seg_c * g.nnodes + nd) * g.ldc + n0 + col] = sacc / (float)(n < 1 ? 1 : n);
    }
    return;
  }

#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long lr = wm * 64 + i * 32 + r32;
    if (lr >= nrows) continue;
    const long row = row0 + lr;
    if (EPI == EPI_EDGE) {
      const long ii = g.ei[row], jj = g.ej[row];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = n0 + wn * 64 + j * 32 + 8 * q + 4 * h;
          for (int c = 0; c < g.npairs; ++c) {
            const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
            const f32x4 p = *reinterpret_cast<const f32x4*>(Pc + ii * (2 * H) + col);
            const f32x4 qv = *reinterpret_cast<const f32x4*>(Pc + jj * (2 * H) + H + col);
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = silu_fast((acc[i][j][4 * q + e] + p[e]) + qv[e]);
            *reinterpret_cast<f32x4*>(g.C + ((long)c * g.E + row) * g.ldc + col) = v;
          }
        }
    } else {
      const float* gbrow = g.gb ? g.gb + (long)g.row2g[row % g.gb_rowmod] * g.ldgb : nullptr;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = n0 + wn * 64 + j * 32 + 8 * q + 4 * h;
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
          if (g.bias) v += *reinterpret_cast<const f32x4*>(g.bias + col);
          if (gbrow && col < g.gb_cols) v += *reinterpret_cast<const f32x4*>(gbrow + col);
          if (g.act == 1)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = silu_fast(v[e]);
          if (g.R) v += *reinterpret_cast<const f32x4*>(g.R + row * g.ldr + col);
          *reinterpret_cast<f32x4*>(g.C + row * g.ldc + col) = v;
        }
    }
  }
}

// ---------------------------------------------------------------------------
// Large-tile variant for the edge GEMMs (M = E or 2E rows, N = 512):
// 256x256 output per 512-thread block, 8 waves as 4 (M) x 2 (N), each wave
// 64x128 = 2x4 accumulators of 32x32 (128 registers). Per 16-deep K chunk a
// wave issues 48 bf16 MFMAs against 18 fragment reads, twice the work per
// barrier of the 128x128 kernel. LDS: two stages of 3 A planes + 3 W planes,
// 256 rows x 24 bf16 each = 144 KB (one block per CU, two waves per SIMD).
// ---------------------------------------------------------------------------
constexpr int LBM = 256, LBN = 256;
constexpr int LPLANE = 256 * XLP;

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm3_big(GemmArgs g) {
  constexpr int NP = 3;  // planes per operand
  extern __shared__ __attribute__((aligned(16))) __bf16 lsm[];  // [2][2*NP][LPLANE]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = g.N / LBN;
  const long bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bn = (int)(bid % ntn);
  const int n0 = bn * LBN;
  long row0, nrows;
  int seg_c = 0;
  int2 seg = {0, 0};
  if (EPI == EPI_SEGMEAN) {
    const long rest = bid / ntn;
    seg_c = (int)(rest % g.npairs);
    seg = g.tiles[rest / g.npairs];
    const long es0 = g.node_estart[seg.x];
    const long es1 = (seg.y < g.nnodes) ? g.node_estart[seg.y] : g.E;
    row0 = (long)seg_c * g.E + es0;
    nrows = es1 - es0;
  } else {
    row0 = (bid / ntn) * LBM;
    nrows = g.M - row0 < LBM ? g.M - row0 : LBM;
  }
  const __bf16* Wpl = reinterpret_cast<const __bf16*>(g.Wp3);
  const long wplane = (long)g.N * g.K;

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // staging: thread -> (row = tid >> 1, k half = tid & 1): 8 fp32 of A, 8 bf16 of each W plane
  const int srow = tid >> 1, shalf = tid & 1;
  const long ar = row0 + (srow < nrows ? srow : nrows - 1);
  const float* pa = g.A + ar * g.lda + 8 * shalf;
  const float* pb = g.A2 + ar * g.lda2 + 8 * shalf - g.ksplit;
  const __bf16* pw = Wpl + (long)(n0 + srow) * g.K + 8 * shalf;
  // two register sets: the global loads of K-tile t+2 are issued while tile t is
  // computed and tile t+1 is converted into LDS (two tiles of latency cover)
  f32x4 ra0[2], ra1[2];
  u32x4 rw[2][NP];
  auto gload = [&](int set, int k0) {
    const float* src = k0 < g.ksplit ? pa + k0 : pb + k0;
    ra0[set] = *reinterpret_cast<const f32x4*>(src);
    ra1[set] = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
    for (int p = 0; p < NP; ++p) rw[set][p] = *reinterpret_cast<const u32x4*>(pw + p * wplane + k0);
  };
  auto lstore = [&](int set, int st) {
    __bf16* S = lsm + st * 2 * NP * LPLANE;
    const int off = srow * XLP + 8 * shalf;
    bf16x8 hh, mm, ll;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      __bf16 a, b, c;
      split3(ra0[set][e], a, b, c);
      hh[e] = a; mm[e] = b; ll[e] = c;
      split3(ra1[set][e], a, b, c);
      hh[4 + e] = a; mm[4 + e] = b; ll[4 + e] = c;
    }
    *reinterpret_cast<bf16x8*>(S + 0 * LPLANE + off) = hh;
    *reinterpret_cast<bf16x8*>(S + 1 * LPLANE + off) = mm;
    *reinterpret_cast<bf16x8*>(S + 2 * LPLANE + off) = ll;
#pragma unroll
    for (int p = 0; p < NP; ++p) *reinterpret_cast<u32x4*>(S + (NP + p) * LPLANE + off) = rw[set][p];
  };

  const int h = lane >> 5, r32 = lane & 31;
  // W fragments are the MFMA A operand, activations the B operand: the
  // accumulators hold C^T tiles (lane = output row, registers = columns)
  auto compute = [&](int st) {
    const __bf16* S = lsm + st * 2 * NP * LPLANE;
    bf16x8 a[3][2];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[p][i] = *reinterpret_cast<const bf16x8*>(S + p * LPLANE + (wm * 64 + i * 32 + r32) * XLP + 8 * h);
    // W plane 2 pairs with A0; W plane 1 with A1, A0; W plane 0 with A2, A1, A0 (small terms first)
#pragma unroll
    for (int p = 2; p >= 0; --p) {
      bf16x8 w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[j] = *reinterpret_cast<const bf16x8*>(S + (3 + p) * LPLANE + (wn * 128 + j * 32 + r32) * XLP + 8 * h);
#pragma unroll
      for (int q = 2 - p; q >= 0; --q)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[j], a[q][i], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = g.K / XBK;
  // loads and stores are unconditional (past the end they re-read the last K-tile and
  // fill the idle stage) so the compiler can keep counted vmcnt waits across the loop
  const int klast = (nk - 1) * XBK;
  gload(0, 0);
  gload(1, XBK < klast ? XBK : klast);
  lstore(0, 0);
  __syncthreads();
  // tile t lives in register set t & 1 and LDS stage t & 1 (the set index must be a
  // compile-time constant, hence the two-step body)
  auto step = [&](int kt, int par) {
    const int kn = (kt + 2) * XBK;
    gload(par, kn < klast ? kn : klast);
    compute(par);
    lstore(par ^ 1, par ^ 1);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, 0);
    if (kt + 1 < nk) step(kt + 1, 1);
  }

  // lane l owns output row wm*64 + i*32 + (l & 31) and, per 4-register group q,
  // the four consecutive columns wn*128 + j*32 + 8q + 4h .. +3
  if (EPI == EPI_SEGMEAN) {
    // two passes of 128 columns: the wn-th half of the waves writes SiLU(acc + b2) to an
    // LDS tile [256][132], then every thread sums node segments of one column in edge order
    float* T = reinterpret_cast<float*>(lsm);
    constexpr int TP = 132;
    const long es0 = g.node_estart[seg.x];
    for (int half = 0; half < 2; ++half) {
      if (wn == half) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int col = j * 32 + 8 * q + 4 * h;
            const f32x4 b = *reinterpret_cast<const f32x4*>(g.bias + n0 + half * 128 + col);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              const int row = wm * 64 + i * 32 + r32;
              f32x4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = silu_fast(acc[i][j][4 * q + e] + b[e]);
              *reinterpret_cast<f32x4*>(T + row * TP + col) = v;
            }
          }
      }
      __syncthreads();
      const int col = tid & 127;
      for (int nd = seg.x + (tid >> 7); nd < seg.y; nd += 4) {
        const int n = g.natoms[g.n2g[nd]];
        const int r0 = (int)(g.node_estart[nd] - es0);
        float sacc = 0.f;
        for (int j = 0; j < n; ++j) sacc += T[(r0 + j) * TP + col];
        g.agg[((long)seg_c * g.nnodes + nd) * g.ldc + n0 + half * 128 + col] = sacc / (float)(n < 1 ? 1 : n);
      }
      __syncthreads();
    }
    return;
  }

#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long lr = wm * 64 + i * 32 + r32;
    if (lr >= nrows) continue;
    const long row = row0 + lr;
    if (EPI == EPI_EDGE) {
      const long ii = g.ei[row], jj = g.ej[row];
      for (int c = 0; c < g.npairs; ++c) {
        const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int col = n0 + wn * 128 + j * 32 + 8 * q + 4 * h;
            const f32x4 p = *reinterpret_cast<const f32x4*>(Pc + ii * (2 * H) + col);
            const f32x4 qv = *reinterpret_cast<const f32x4*>(Pc + jj * (2 * H) + H + col);
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = silu_fast((acc[i][j][4 * q + e] + p[e]) + qv[e]);
            *reinterpret_cast<f32x4*>(g.C + ((long)c * g.E + row) * g.ldc + col) = v;
          }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = n0 + wn * 128 + j * 32 + 8 * q + 4 * h;
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
          if (g.bias) v += *reinterpret_cast<const f32x4*>(g.bias + col);
          if (g.act == 1)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = silu_fast(v[e]);
          if (g.R) v += *reinterpret_cast<const f32x4*>(g.R + row * g.ldr + col);
          *reinterpret_cast<f32x4*>(g.C + row * g.ldc + col) = v;
        }
    }
  }
}

constexpr size_t kBigLds = 2 * 6 * LPLANE * sizeof(__bf16);  // 147456 B (also holds EPI_SEGMEAN's [256][132] tile)
static_assert((size_t)LBM * 132 * sizeof(float) <= kBigLds, "segment tile fits the staging area");

// opt the large dynamic-LDS kernels in; called at model creation, outside any
// stream capture (a function attribute call is not a stream operation)
static hipError_t gemm_init_once() {
  const void* ks[] = {(const void*)k_gemm3_big<EPI_STD>, (const void*)k_gemm3_big<EPI_EDGE>,
                      (const void*)k_gemm3_big<EPI_SEGMEAN>};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kBigLds);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// (set once per process; a function-local static initialiser is thread-safe)
hipError_t gemm_init() {
  static const hipError_t e = gemm_init_once();
  return e;
}

hipError_t gemm_bf16x3_big(const GemmArgs& g, int epi, hipStream_t s) {
  if (g.N % LBN || g.K % XBK || !g.Wp3 || g.ksplit % XBK || g.gb) return hipErrorInvalidValue;
  long blocks;
  if (epi == EPI_SEGMEAN) {
    if (g.N != H || !g.tiles || !g.agg) return hipErrorInvalidValue;
    blocks = (long)g.ntiles * g.npairs * (g.N / LBN);
  } else {
    if (g.M <= 0) return hipErrorInvalidValue;
    blocks = ((g.M + LBM - 1) / LBM) * (g.N / LBN);
  }
  if (hipError_t e = gemm_init(); e != hipSuccess) return e;
  if (epi == EPI_EDGE)
    hipLaunchKernelGGL((k_gemm3_big<EPI_EDGE>), dim3((unsigned)blocks), dim3(512), kBigLds, s, g);
  else if (epi == EPI_SEGMEAN)
    hipLaunchKernelGGL((k_gemm3_big<EPI_SEGMEAN>), dim3((unsigned)blocks), dim3(512), kBigLds, s, g);
  else
    hipLaunchKernelGGL((k_gemm3_big<EPI_STD>), dim3((unsigned)blocks), dim3(512), kBigLds, s, g);
  return hipGetLastError();
}


template <int PF, int REMAP>
static void launch3(const GemmArgs& g, int epi, long blocks, hipStream_t s) {
  if (epi == EPI_EDGE)
    hipLaunchKernelGGL((k_gemm3<EPI_EDGE, PF, REMAP>), dim3((unsigned)blocks), dim3(256), 0, s, g);
  else if (epi == EPI_SEGMEAN)
    hipLaunchKernelGGL((k_gemm3<EPI_SEGMEAN, PF, REMAP>), dim3((unsigned)blocks), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((k_gemm3<EPI_STD, PF, REMAP>), dim3((unsigned)blocks), dim3(256), 0, s, g);
}

int g_gemm3_variant = 0;  // bit 0: two chunks in flight, bit 1: XCD remap (0 measured fastest for node GEMMs)

hipError_t gemm_bf16x3(const GemmArgs& g, int epi, hipStream_t s) {
  if (g.N % XBN || g.K % (2 * XBK) || !g.Wp3) return hipErrorInvalidValue;
  if (g.ksplit % XBK) return hipErrorInvalidValue;
  long blocks;
  if (epi == EPI_SEGMEAN) {
    if (g.N != H || !g.tiles || !g.agg) return hipErrorInvalidValue;
    blocks = (long)g.ntiles * g.npairs * (g.N / XBN);
  } else {
    if (g.M <= 0) return hipErrorInvalidValue;
    blocks = ((g.M + XBM - 1) / XBM) * (g.N / XBN);
  }
  switch (g_gemm3_variant & 3) {
    case 0: launch3<1, 0>(g, epi, blocks, s); break;
    case 1: launch3<2, 0>(g, epi, blocks, s); break;
    case 2: launch3<1, 1>(g, epi, blocks, s); break;
    default: launch3<2, 1>(g, epi, blocks, s); break;
  }
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
