// Node GEMMs of the decoder (FiLM projection, per-node halves of edge layer 1, node MLP, heads,
// conditioning; cspnet.py:78-97, 150-181, 396-403) in fp32-accurate "bf16x3" arithmetic:
// C[M,N] = epi(A[M,K] . W[N,K]^T), A fp32, W pre-split into three bf16 planes [3][N][K].
//
// Both operands are staged global -> LDS with global_load_lds (no VGPR round trip, no LDS stores
// from registers): A as raw fp32, W as its three planes. Each wave splits its own A fragments
// (8 fp32 per lane and k-step) into three bf16 parts in registers for the six MFMA products
// (a2w0 + a1w1 + a0w2 + a1w0 + a0w1 + a0w0, small terms first); the loop is software-pipelined
// so the next K-tile's fragment reads and split run between the current tile's MFMAs.
// Bit-identical to k_gemm3 (same products, same order); 5-10% faster in isolation.
//
// S16 (split16 mode): W pre-split into fp16 hi/lo rows [N][K/16][hi 16 | lo 16] of W * 2^-e_n
// (split_rows_h, per-row power-of-two scale wscale[n] = 2^e_n, undone in the epilogue), A split by
// each wave into fp16 hi/lo (round to nearest), three fp16 MFMA products (a_lo w_hi + a_hi w_lo +
// a_hi w_hi): half the MFMAs of bf16x3, ~3.5 VALU per A element. A row r is scaled by 2^-e_r
// before its split, e_r the exponent of max |A[r, :]| (g.amax / g.amax2, written by the kernel
// that produced A: embed, film_ln, the segment-mean epilogue, or this kernel's own epilogue via
// g.cmax), so every scaled entry is below 1 whatever the activations' range (the lattice terms
// grow ~10^4x over a 1000-step trajectory); 2^e_r is applied again in the epilogue.
//
// 128x128 tiles, 256 threads (4 waves of 64x64, C^T accumulators as in gemm_bf16x3.hip),
// K-tiles of 16, a 4-deep ring of 20 KB stages (4 K-tiles in flight), two blocks per CU; S16 uses
// 16 KB stages, 5 deep with two blocks per CU or 3 deep with three (large grids). Small grids
// (S16, NMT = 64): 64x128 tiles (4 waves of 32x64), 12 KB stages, 4 deep with three blocks per CU
// or 3 deep with four: twice the blocks of the 128-row tiling, so the per-GPU shard's node GEMMs
// (M = 5120: 160 blocks of 128 rows on 256 CUs, one wave per SIMD) fill the chip.
// LDS image per stage: A [128 rows][4 pieces of 4 fp32], piece p of row r at p ^ ((r >> 2) & 3);
// W plane q [128 rows][2 pieces of 8 bf16], piece p of row r at p ^ ((r >> 3) & 1): the
// fragment reads of every 16-lane group then cover all 64 banks.
#include "chm_internal.h"

#include <type_traits>

namespace chm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

namespace {

constexpr int NN = 128, NK = 16;
constexpr int A_ROWB = NK * 4, W_ROWB = NK * 2;  // 64 B, 32 B
constexpr int W_PLB = NN * W_ROWB;               // 4 KB per plane
template <int NMT> constexpr int A_STB = NMT * A_ROWB;  // 8 KB (128 rows), 4 KB (64 rows)
// bf16x3: A + three W planes (20 KB) x 4 stages; S16: A + W hi/lo rows (8 + 8 KB) x 5 stages
template <bool S16, int NMT = 128> constexpr int STB = S16 ? A_STB<NMT> + 2 * W_PLB : A_STB<NMT> + 3 * W_PLB;
// NB = blocks per CU. 128-row tiles: 2 (bf16x3: 4 stages; S16: 5) or, S16 only, 3 (3 stages of
// 16 KB); 64-row tiles (S16): 3 (4 stages of 12 KB) or 4 (3 stages)
template <bool S16, int NB, int NMT = 128>
constexpr int NST = NMT == 64 ? (!S16 ? 5 : NB == 3 ? 4 : 3) : NB == 3 ? 3 : (S16 ? 5 : 4);
constexpr int NODE_LDS = 80 * 1024;  // two blocks per CU
static_assert(STB<true> * NST<true, 2> <= NODE_LDS && STB<false> * NST<false, 2> <= NODE_LDS, "LDS");
static_assert(3 * STB<true> * NST<true, 3> <= 160 * 1024, "LDS");
static_assert(3 * STB<true, 64> * NST<true, 3, 64> <= 160 * 1024 && 4 * STB<true, 64> * NST<true, 4, 64> <= 160 * 1024, "LDS");
static_assert(STB<false, 64> * NST<false, 2, 64> <= NODE_LDS, "LDS");  // bf16x3 64-row tiles, two blocks per CU
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// K-loop ablations of A/B builds only (-DCHM_NODE_ABL=n; wrong results, read in cycles): bit 0 = no per-K-step barrier,
// 1 = no operand loads in the loop, 2 = no A split (one conversion instead: the VAR 1 probe in every kernel)
#ifndef CHM_NODE_ABL
#define CHM_NODE_ABL 0
#endif
constexpr bool kNAblBar = CHM_NODE_ABL & 1, kNAblLd = CHM_NODE_ABL & 2, kNAblSplit = CHM_NODE_ABL & 4;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ long xcd_remap(long b, long nb) {
  const long q = nb / 8, r = nb % 8, xcd = b % 8, idx = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ float silu_n(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}

__device__ __forceinline__ void split3n(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

}  // namespace

// exponent e with m = f 2^e, f in [0.5, 1) (0 for m == 0): the split scale 2^-e keeps |x 2^-e| < 1
__device__ __forceinline__ int exp_of_n(float m) {
  int e = 0;
  if (m > 0.f) frexpf(m, &e);
  return e;
}

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// The epilogue of a pre-split GEMM whose output feeds another one (GemmArgs::Cs): C (fp32, optional) and C
// as split rows [rows][N/16][hi 16 | lo 16] scaled by 2^-e per (row, this block's 128 columns), e from the
// row's max over the block's columns (the two column halves of a row sit in waves wn = 0 / 1: one LDS
// exchange), with the packed exponent byte cex[row] byte n0 / 128.
template <int NI, int NM>
__device__ __forceinline__ void node_epilogue_split(const GemmArgs& g, f32x16 (&acc)[NI][2], const float (&aun)[NI],
                                                    long row0, long nrows, int n0, int wm, int wn, int r32, int h) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* xm = reinterpret_cast<float*>(lds);  // [2 wm][2 wn][NM / 2 rows]
  float cm[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const long lr = wm * (NM / 2) + i * 32 + r32;
    const long row = row0 + (lr < nrows ? lr : nrows - 1);
    const float* gbrow = g.gb ? g.gb + (long)g.row2g[row % g.gb_rowmod] * g.ldgb : nullptr;
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = n0 + wn * 64 + j * 32 + 8 * q + 4 * h;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
        v *= *reinterpret_cast<const f32x4*>(g.wscale + col) * aun[i];
        if (g.bias) v += *reinterpret_cast<const f32x4*>(g.bias + col);
        if (gbrow && col < g.gb_cols) v += *reinterpret_cast<const f32x4*>(gbrow + col);
        if (g.act == 1)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = silu_n(v[e]);
        if (g.R) v += *reinterpret_cast<const f32x4*>(g.R + row * g.ldr + col);
        if (g.C && lr < nrows) *reinterpret_cast<f32x4*>(g.C + row * g.ldc + col) = v;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] = v[e];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      }
    cm[i] = fmaxf(m, __shfl_xor(m, 32, 64));  // lanes r32 and r32 + 32 hold the same row
  }
  __syncthreads();  // every wave is past its K loop: the stages are free
  if (h == 0)
#pragma unroll
    for (int i = 0; i < NI; ++i) xm[(wm * 2 + wn) * (NM / 2) + 32 * i + r32] = cm[i];
  __syncthreads();
  _Float16* Cs = reinterpret_cast<_Float16*>(g.Cs);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const long lr = wm * (NM / 2) + i * 32 + r32;
    if (lr >= nrows) continue;
    const long row = row0 + lr;
    const int ex = exp_of_n(fmaxf(cm[i], xm[(wm * 2 + (wn ^ 1)) * (NM / 2) + 32 * i + r32]));
    const float sc = ldexpf(1.0f, -ex);
    _Float16* out = Cs + row * (2L * g.N);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gc = n0 + wn * 64 + j * 32 + 8 * q + 4 * h;  // 16-column K-tile gc >> 4, offset gc & 15
        f16x4 hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = acc[i][j][4 * q + e] * sc;
          hi[e] = (_Float16)x;
          lo[e] = (_Float16)(x - (float)hi[e]);
        }
        *reinterpret_cast<f16x4*>(out + (gc >> 4) * 32 + (gc & 15)) = hi;
        *reinterpret_cast<f16x4*>(out + (gc >> 4) * 32 + 16 + (gc & 15)) = lo;
      }
    if (wn == 0 && h == 0) reinterpret_cast<signed char*>(g.cex)[row * 4 + n0 / 128] = (signed char)ex;
  }
}

// VAR (microbenchmark only): 1 = A split replaced by one conversion (wrong results; VALU probe)
// PS (S16 only): A arrives pre-split (GemmArgs::aex): its fragments are read from LDS as they are, the
// accumulators are rescaled by 2^(e_prev - e_next) where a 128-column chunk of K ends (exact), and the
// epilogue can write C split the same way (GemmArgs::Cs).
// NNT (split16, 64-row tiles only): tile columns, 128 or 64 (4 waves of 32x32: twice the blocks again, for
// grids still short of the CUs). Every output element's K sum runs in the same order whatever the tile
// shape, so all tilings are bit-identical.
template <int VAR, bool S16, int NB, int NMT = 128, bool PS = false, int NNT = 128>
__global__ __launch_bounds__(256, NB) void k_node_gemm(GemmArgs g) {
  static_assert(NMT == 128 ? NB == 2 || (S16 && NB == 3) : NMT == 64 && (S16 ? NB == 3 || NB == 4 : NB == 2),
                "tiling");
  static_assert(!PS || S16, "pre-split A is a split16 form");
  static_assert(NNT == 128 || (NNT == 64 && S16 && !PS && NMT == 64), "64-column tiles: split16, 64 rows");
  constexpr int NM = NMT, NI = NMT / 64;  // tile rows; 32-row fragment groups per wave
  constexpr int NJ = NNT / 64;            // 32-column fragment groups per wave
  constexpr int A_STB_ = A_STB<NMT>;
  // K-tiles in flight: all NST stages. Tile t's stage is read in step t-1 (read_raw(t)), so after
  // step t's barrier it takes tile t + NST while tiles t+1 .. t+NST-1 are in flight or landed.
  constexpr int STB_ = NNT == 128 ? STB<S16, NMT> : A_STB_ + NNT * 64;
  constexpr int NST_ = NNT == 128 ? NST<S16, NB, NMT> : 4, AHEAD = NST_;
  constexpr int NWI = S16 ? NNT / 64 : 3;                                // W glds per thread and K-tile
  constexpr int GL = S16 ? NWI + NI : 3 + NI;                            // glds per thread and K-tile
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, r32 = lane & 31;
  const int ntn = g.N / NNT;
  // XCD-aware order (workgroups go round-robin to the 8 XCDs): each XCD takes a contiguous range of
  // tiles, so the column tiles of a row tile run on one XCD and read their A rows once from HBM
  // (without it every column tile fetched A again into another XCD's L2: 538 MB per launch vs 84-168)
  const long bid = g.linear_order ? (long)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int n0 = (int)(bid % ntn) * NNT;
  const long row0 = (bid / ntn) * NM;
  const long nrows = g.M - row0 < NM ? g.M - row0 : NM;
  const int nk = g.K / NK;

  // ---- glds sources. A: instruction q (of 8, or 4 for 64 rows) covers rows 16q + (L >> 2), LDS
  // piece L & 3 holding logical piece (L & 3) ^ ((L >> 4) & 3); wave w issues q = NI w .. NI w + NI-1.
  // W: instruction q (of 12) is plane q >> 2, rows 32 (q & 3) + (L >> 1), LDS piece L & 1 holding
  // logical piece (L & 1) ^ ((L >> 4) & 1); wave w issues q = 3w .. 3w + 2.
  const int alp = (lane & 3) ^ ((lane >> 4) & 3);
  const float* asrc[NI];
  const float* asrc2[NI];
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int r = 16 * (NI * wave + u) + (lane >> 2);
    const long ar = row0 + (r < nrows ? r : nrows - 1);
    asrc[u] = g.A + ar * g.lda + 4 * alp;
    asrc2[u] = g.A2 + ar * g.lda2 + 4 * alp - g.ksplit;
  }
  // W (bf16x3): instruction q (of 12) is plane q >> 2, rows 32 (q & 3) + (L >> 1), LDS piece L & 1
  // holding logical piece (L & 1) ^ ((L >> 4) & 1); wave w issues q = 3w .. 3w + 2.
  // W (S16): rows of 64 B [hi 16 | lo 16] per K-tile, swizzled like A; instruction q (of 8) covers
  // rows 16q + (L >> 2), LDS piece L & 3 holding logical piece alp; wave w issues q = NWI w .. NWI w + NWI-1.
  const int wlp = (lane & 1) ^ ((lane >> 4) & 1);
  const __bf16* Wpl = reinterpret_cast<const __bf16*>(g.Wp3);
  const long wplane = (long)g.N * g.K;
  const __bf16* wsrc[NWI];
  int wdst[NWI];
#pragma unroll
  for (int u = 0; u < NWI; ++u) {
    if constexpr (S16) {
      const int q = NWI * wave + u;
      wsrc[u] = Wpl + (long)(n0 + 16 * q + (lane >> 2)) * 2 * g.K + 8 * alp;
      wdst[u] = A_STB_ + q * 1024;
    } else {
      const int q = 3 * wave + u, p = q >> 2, rq = q & 3;
      wsrc[u] = Wpl + p * wplane + (long)(n0 + 32 * rq + (lane >> 1)) * g.K + 8 * wlp;
      wdst[u] = A_STB_ + p * W_PLB + 32 * rq * W_ROWB;
    }
  }
  auto issue = [&](int t) {
    const int k0 = (t < nk ? t : nk - 1) * NK;  // past the end: re-read the last tile into an idle stage
    char* st = lds + (t % NST_) * STB_;
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const float* src = k0 < g.ksplit ? asrc[u] + k0 : asrc2[u] + k0;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(st + 16 * (NI * wave + u) * A_ROWB), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < NWI; ++u)
      __builtin_amdgcn_global_load_lds((gbl_void*)(wsrc[u] + (S16 ? 2 * k0 : k0)), (lds_void*)(st + wdst[u]), 16, 0, 0);
  };

  // Short grids (64-row split16 tiles, one to two blocks per CU and nothing else to run): the epilogue's per-column
  // vectors (W scales, bias or the per-graph row terms, and on 64 x 64 tiles the residual rows) are loaded here,
  // ahead of the operand stream, so their latency runs under the K loop instead of opening the epilogue (the same
  // values in the same expressions: bit-identical)
  constexpr bool PRE = S16 && !PS && NMT == 64 && (NNT == 64 || NB == 3), PRE_R = PRE && NNT == 64;
  f32x4 pws[PRE ? NJ : 1][4], pv2[PRE ? NJ : 1][4], prr[PRE_R ? NJ : 1][4];
  bool pre_gb = false;
  if constexpr (PRE) {
    static_assert(NI == 1, "one row per lane");
    const long lr = wm * (NM / 2) + r32;
    const long prow_ = row0 + (lr < nrows ? lr : nrows - 1);
    pre_gb = !g.bias && g.gb;
    const float* gbrow = pre_gb ? g.gb + (long)g.row2g[prow_ % g.gb_rowmod] * g.ldgb : nullptr;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = n0 + wn * (NNT / 2) + j * 32 + 8 * q + 4 * h;
        pws[j][q] = *reinterpret_cast<const f32x4*>(g.wscale + col);
        if (g.bias)
          pv2[j][q] = *reinterpret_cast<const f32x4*>(g.bias + col);
        else if (gbrow && col < g.gb_cols)
          pv2[j][q] = *reinterpret_cast<const f32x4*>(gbrow + col);
        if constexpr (PRE_R)
          if (g.R) prr[j][q] = *reinterpret_cast<const f32x4*>(g.R + prow_ * g.ldr + col);
      }
  }

  f32x16 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // fragment offsets: A row wm*NM/2 + 32i + r32 pieces 2h, 2h+1; W row wn*64 + 32j + r32 piece h
  const int asw = (r32 >> 2) & 3, wsw = (r32 >> 3) & 1;
  // S16: this lane's A rows (wm*NM/2 + 32i + r32) and their power-of-two scales
  float asc[NI], aun[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) asc[i] = aun[i] = 1.0f;
  // PS: this lane's rows' chunk exponents (chunks [0, nc1) from aex, the rest from aex2)
  int pex[NI], pex2[NI];
  const int nc1 = g.ksplit / 128;
  auto chunk_e = [&](int i, int c) __attribute__((always_inline)) {
    return c < nc1 ? (int)(signed char)(pex[i] >> (8 * c)) : (int)(signed char)(pex2[i] >> (8 * (c - nc1)));
  };
  if constexpr (PS) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int lr = wm * (NM / 2) + 32 * i + r32;
      const long ar = row0 + (lr < nrows ? lr : nrows - 1);
      pex[i] = g.aex[ar];
      pex2[i] = g.aex2 ? g.aex2[ar] : 0;
      aun[i] = ldexpf(1.0f, chunk_e(i, g.K / 128 - 1));  // (the last chunk's scale, undone in the epilogue)
    }
  } else if constexpr (S16) {
    if (g.amax) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int lr = wm * (NM / 2) + 32 * i + r32;
        const long ar = row0 + (lr < nrows ? lr : nrows - 1);
        float m = g.amax[ar];
        if (g.amax2) m = fmaxf(m, g.amax2[ar]);
        int e = 0;
        if (m > 0.f) frexpf(m, &e);
        asc[i] = ldexpf(1.0f, -e);
        aun[i] = ldexpf(1.0f, e);
      }
    }
  }
  const int fa0 = (wm * (NM / 2) + r32) * A_ROWB + 16 * ((2 * h) ^ asw);
  const int fa1 = (wm * (NM / 2) + r32) * A_ROWB + 16 * ((2 * h + 1) ^ asw);
  const int fw = A_STB_ + (wn * 64 + r32) * W_ROWB + 16 * (h ^ wsw);
  const int fw16[2] = {A_STB_ + (wn * (NNT / 2) + r32) * 64 + 16 * (h ^ asw),         // hi piece h
                       A_STB_ + (wn * (NNT / 2) + r32) * 64 + 16 * ((2 + h) ^ asw)};  // lo piece 2 + h

  // Software pipeline (VAR 0): while the 24 MFMAs of K-tile t run, the fragments of tile t+1 are
  // read from LDS and its A part is split, both interleaved between the MFMAs (the split's VALU
  // issues in the MFMAs' shadow). Fragment sets alternate, so the loop is unrolled by two.
  constexpr int NP = S16 ? 2 : 3;  // operand parts
  typedef std::conditional_t<S16, f16x8, bf16x8> frag;
  f32x4 ra0[NI], ra1[NI];
  frag fa[2][NP][NI], fwt[2][NP][NJ];  // [set][part][i / j]
  // PS: the A fragments as they are (hi piece h, lo piece 2 + h of the row's 64-B K-tile, swizzled like W16)
  const int fa16[2] = {(wm * (NM / 2) + r32) * A_ROWB + 16 * (h ^ asw), (wm * (NM / 2) + r32) * A_ROWB + 16 * ((2 + h) ^ asw)};
  auto read_raw = [&](int t, int set) {
    const char* st = lds + (t % NST_) * STB_;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if constexpr (PS) {
        fa[set][0][i] = *reinterpret_cast<const frag*>(st + fa16[0] + i * 32 * A_ROWB);
        fa[set][1][i] = *reinterpret_cast<const frag*>(st + fa16[1] + i * 32 * A_ROWB);
      } else {
        ra0[i] = *reinterpret_cast<const f32x4*>(st + fa0 + i * 32 * A_ROWB);
        ra1[i] = *reinterpret_cast<const f32x4*>(st + fa1 + i * 32 * A_ROWB);
      }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        fwt[set][p][j] = S16 ? *reinterpret_cast<const frag*>(st + fw16[p] + j * 32 * 64)
                             : *reinterpret_cast<const frag*>(st + fw + p * W_PLB + j * 32 * W_ROWB);
  };
  auto split = [&](int set) {
    if constexpr (PS) return;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if constexpr (S16) {
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 x = (e < 4 ? f32x2{ra0[i][e], ra0[i][e + 1]} : f32x2{ra1[i][e - 4], ra1[i][e - 3]}) * asc[i];
          const f16x2 hi = __builtin_convertvector(x, f16x2);
          const f16x2 lo = (VAR == 1 || kNAblSplit) ? hi : __builtin_convertvector(x - __builtin_convertvector(hi, f32x2), f16x2);
          fa[set][0][i][e] = hi[0]; fa[set][0][i][e + 1] = hi[1];
          fa[set][1][i][e] = lo[0]; fa[set][1][i][e + 1] = lo[1];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          __bf16 x0, x1, x2;
          if (VAR == 1) {
            x0 = x1 = x2 = (__bf16)(e < 4 ? ra0[i][e] : ra1[i][e - 4]);
          } else {
            split3n(e < 4 ? ra0[i][e] : ra1[i][e - 4], x0, x1, x2);
          }
          fa[set][0][i][e] = x0;
          fa[set][1][i][e] = x1;
          fa[set][2][i][e] = x2;
        }
      }
    }
  };
  // small terms first, the leading product last (as gemm_bf16x3.hip)
  constexpr int PA[6] = {S16 ? 1 : 2, S16 ? 0 : 1, 0, 1, 0, 0};
  constexpr int PW[6] = {0, 1, S16 ? 0 : 2, 0, 1, 0};
  auto mfmas = [&](int set, int k0, int k1) {
#pragma unroll
    for (int k = k0; k < k1; ++k)
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if constexpr (S16)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fwt[set][PW[k]][j], fa[set][PA[k]][i], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fwt[set][PW[k]][j], fa[set][PA[k]][i], acc[i][j], 0, 0,
                                                                 0);
        }
  };
#pragma unroll
  for (int t = 0; t < AHEAD; ++t) issue(t);
  vm_wait<(AHEAD - 1) * GL>();  // tile 0 has landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_raw(0, 0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  split(0);
  auto step = [&](int t, auto CUR) {
    constexpr int cur = decltype(CUR)::value;
    if constexpr (PS) {  // tile t opens a new 128-column chunk of A: move the accumulators to its scale
      if (t > 0 && (t & 7) == 0) {
        const int c = t >> 3;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const float f = ldexpf(1.0f, chunk_e(i, c - 1) - chunk_e(i, c));
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] *= f;
        }
      }
    }
    // this thread's part of tile t+1 has landed (AHEAD - 2 tiles may stay in flight)
    vm_wait<(AHEAD - 2) * GL>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (!kNAblBar) __builtin_amdgcn_s_barrier();      // everyone's; tile t's stage has been read
    asm volatile("" ::: "memory");
    if (!kNAblLd) issue(t + AHEAD);                   // into tile t's stage; past the end: re-reads
    __builtin_amdgcn_s_setprio(1);
    read_raw(t + 1, cur ^ 1);                         // past the end: reads a re-read tile
    if constexpr (S16) {
      mfmas(cur, 0, 1);                               // NI NJ MFMAs beside the 2 NI + 2 NJ fragment reads
      constexpr int MF1 = NI * NJ, RD1 = (2 * NI + 2 * NJ + MF1 - 1) / MF1;
#pragma unroll
      for (int k = 0; k < MF1; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, RD1, 0);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      split(cur ^ 1);
      mfmas(cur, 1, 3);                               // 2 NI NJ MFMAs, the split's VALU between them
#pragma unroll
      for (int k = 0; k < 2 * NI * NJ; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 1);
      }
    } else {
      mfmas(cur, 0, 2);                               // 8 MFMAs beside the 10 fragment reads
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      split(cur ^ 1);
      mfmas(cur, 2, 6);                               // 16 MFMAs, the split's VALU between them
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 1);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  for (int t = 0; t < nk; t += 2) {  // nk = K / 16 is even for every node GEMM (K = 512, 640, 1024)
    step(t, std::integral_constant<int, 0>{});
    step(t + 1, std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail re-reads land before the block exits

  // lane l owns output row wm*NM/2 + 32i + (l & 31) and, per 4-register group q, the four
  // consecutive columns wn*64 + 32j + 8q + 4h .. +3
  if constexpr (PS) {
    if (g.Cs) {  // the output as split rows too: this block's 128 columns are one chunk of the next GEMM's A
      node_epilogue_split<NI, NM>(g, acc, aun, row0, nrows, n0, wm, wn, r32, h);
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const long lr = wm * (NM / 2) + i * 32 + r32;
    float cm = 0.f;  // max |C| over this lane's columns of the row
    if (lr < nrows) {
      const long row = row0 + lr;
      const float* gbrow = g.gb && !pre_gb ? g.gb + (long)g.row2g[row % g.gb_rowmod] * g.ldgb : nullptr;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = n0 + wn * (NNT / 2) + j * 32 + 8 * q + 4 * h;
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
          if constexpr (PRE) {
            v *= pws[j][q] * aun[i];  // undo the scales
            if (g.bias) v += pv2[j][q];
            if (pre_gb && col < g.gb_cols) v += pv2[j][q];
            if (!pre_gb && gbrow && col < g.gb_cols) v += *reinterpret_cast<const f32x4*>(gbrow + col);  // (bias and gb)
          } else {
            if constexpr (S16) v *= *reinterpret_cast<const f32x4*>(g.wscale + col) * aun[i];  // undo the scales
            if (g.bias) v += *reinterpret_cast<const f32x4*>(g.bias + col);
            if (gbrow && col < g.gb_cols) v += *reinterpret_cast<const f32x4*>(gbrow + col);
          }
          if (g.act == 1)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = silu_n(v[e]);
          if constexpr (PRE_R) {
            if (g.R) v += prr[j][q];
          } else {
            if (g.R) v += *reinterpret_cast<const f32x4*>(g.R + row * g.ldr + col);
          }
          *reinterpret_cast<f32x4*>(g.C + row * g.ldc + col) = v;
          if constexpr (S16) cm = fmaxf(cm, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        }
    }
    if constexpr (S16) {
      if (g.cmax) {  // lanes r32 and r32 + 32 hold the same row
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
        if (h == 0 && lr < nrows) atomicMax(g.cmax + row0 + lr, __float_as_uint(cm));
      }
    }
  }
}

int g_node_variant = 0;

constexpr int LDS3 = STB<true> * NST<true, 3>;
constexpr int LDS64_3 = STB<true, 64> * NST<true, 3, 64>, LDS64_4 = STB<true, 64> * NST<true, 4, 64>;
constexpr int LDS64_B3 = STB<false, 64> * NST<false, 2, 64>;  // bf16x3 64-row tiles (5 stages of 16 KB)

static hipError_t node_gemm_init_once() {
  const void* ks[15] = {(const void*)k_node_gemm<0, false, 2, 64>,(const void*)k_node_gemm<0, false, 2>,    (const void*)k_node_gemm<1, false, 2>,
                        (const void*)k_node_gemm<0, true, 2>,     (const void*)k_node_gemm<1, true, 2>,
                        (const void*)k_node_gemm<0, true, 3>,     (const void*)k_node_gemm<1, true, 3>,
                        (const void*)k_node_gemm<0, true, 3, 64>, (const void*)k_node_gemm<1, true, 3, 64>,
                        (const void*)k_node_gemm<0, true, 4, 64>, (const void*)k_node_gemm<1, true, 4, 64>,
                        (const void*)k_node_gemm<0, true, 2, 128, true>, (const void*)k_node_gemm<0, true, 3, 128, true>,
                        (const void*)k_node_gemm<0, true, 3, 64, true>, (const void*)k_node_gemm<0, true, 4, 64, true>};
  const int bytes[15] = {LDS64_B3, NODE_LDS, NODE_LDS, NODE_LDS, NODE_LDS, LDS3, LDS3, LDS64_3, LDS64_3, LDS64_4, LDS64_4,
                         NODE_LDS, LDS3, LDS64_3, LDS64_4};
  hipError_t e = hipSuccess;
  for (int i = 0; i < 15 && e == hipSuccess; ++i) e = hipFuncSetAttribute(ks[i], hipFuncAttributeMaxDynamicSharedMemorySize, bytes[i]);
  return e;
}

// (set once per process; a function-local static initialiser is thread-safe)
hipError_t node_gemm_init() {
  static const hipError_t e = node_gemm_init_once();
  return e;
}

int g_node_blocks = 0;  // S16 blocks per CU override (microbenchmarks): 0 = default
int g_node_rows = 0;    // tile rows override (microbenchmarks): 0 = default, 64, 128
int g_node_cols = 0;    // S16 64-row tile columns override (microbenchmarks): 0 = default, 64, 128

// bf16x3 when g.wscale is null (g.Wp3 = three bf16 planes), S16 otherwise (g.Wp3 = split_rows_h
// rows of 16-column chunks, g.wscale = their row scales)
hipError_t node_gemm(const GemmArgs& g_in, hipStream_t s) {
  static const int linear = getenv("CHM_NODE_LINEAR") ? atoi(getenv("CHM_NODE_LINEAR")) : 0;  // (A/B only)
  GemmArgs g = g_in;
  g.linear_order = linear;
  if (g.M <= 0 || g.N % NN || g.K % (2 * NK) || g.ksplit % NK || !g.Wp3 || !g.A || (!g.C && !g.Cs))
    return hipErrorInvalidValue;
  if ((g.lda | g.lda2 | g.ldc) % 4) return hipErrorInvalidValue;  // 16-B aligned rows
  if (hipError_t e = node_gemm_init(); e != hipSuccess) return e;
  const long blocks = ((g.M + 127) / 128) * (g.N / NN);
  const dim3 grid((unsigned)blocks), block(256);
  const bool v1 = g_node_variant == 1;
  // S16, grids short of one 128-row block per CU: 64-row tiles (twice the blocks; M = 5120: 23 vs
  // 26 us at K = 512); above that 128-row tiles at three blocks per CU (M = 20480: 54 vs 65 us with
  // two), profiles/r2/node/node64_micro.log
  const int rows = g_node_rows ? g_node_rows : (blocks < 256 ? 64 : 128);
  if (g.aex) {  // pre-split A (split16 only)
    if (!g.wscale || g.K % 128 || g.ksplit % 128 || (g.Cs && (g.N % 128 || !g.cex))) return hipErrorInvalidValue;
    const int nb = g_node_blocks ? g_node_blocks : 3;
    if (rows == 64) {
      const dim3 grid64((unsigned)(((g.M + 63) / 64) * (g.N / NN)));
      if (nb == 4)
        hipLaunchKernelGGL((k_node_gemm<0, true, 4, 64, true>), grid64, block, LDS64_4, s, g);
      else
        hipLaunchKernelGGL((k_node_gemm<0, true, 3, 64, true>), grid64, block, LDS64_3, s, g);
    } else if (nb == 3) {
      hipLaunchKernelGGL((k_node_gemm<0, true, 3, 128, true>), grid, block, LDS3, s, g);
    } else {
      hipLaunchKernelGGL((k_node_gemm<0, true, 2, 128, true>), grid, block, NODE_LDS, s, g);
    }
    return hipGetLastError();
  }
  // 64x64 tiles where even the 64x128 grid is short of one block per CU (M = 2560, N = 512: 17.3 -> 15.3 us
  // at K = 512, 28.3 -> 25.7 at K = 1024; from 256 blocks on they lose: profiles/r5/node/node64.txt)
  const bool cols64 = g_node_cols ? g_node_cols == 64 : ((g.M + 63) / 64) * (g.N / NN) < 256;
  if (g.wscale && rows == 64 && cols64 && !g.aex) {
    const dim3 grid6464((unsigned)(((g.M + 63) / 64) * (g.N / 64)));
    hipLaunchKernelGGL((k_node_gemm<0, true, 4, 64, false, 64>), grid6464, block, 4 * (A_STB<64> + 64 * 64), s, g);
    return hipGetLastError();
  }
  if (g.wscale && rows == 64) {
    const dim3 grid64((unsigned)(((g.M + 63) / 64) * (g.N / NN)));
    if (g_node_blocks == 4)
      hipLaunchKernelGGL((v1 ? k_node_gemm<1, true, 4, 64> : k_node_gemm<0, true, 4, 64>), grid64, block, LDS64_4, s, g);
    else
      hipLaunchKernelGGL((v1 ? k_node_gemm<1, true, 3, 64> : k_node_gemm<0, true, 3, 64>), grid64, block, LDS64_3, s, g);
    return hipGetLastError();
  }
  // S16: three blocks per CU (3 stages each): more waves to hide the K-loop latency (-7% at
  // M = 40960, -17% at M = 20480 against two blocks with 5 stages)
  const int nb = g_node_blocks ? g_node_blocks : 3;
  if (!g.wscale && !v1 && (g_node_rows ? g_node_rows == 64 : 2 * blocks <= 256)) {
    // bf16x3 where even the 64-row grid fits the CUs in one round (the heads and conditioning GEMMs at the small
    // shapes): 64-row tiles, half of each wave's MFMAs per K-step on the K loop's dependent chain; bit-identical.
    // (heads, K = 512: M = 10240 31.3 -> 22.2 us, but M = 20480 34.8 -> 38.9: profiles/r5/node_b3rows/)
    const dim3 grid64((unsigned)(((g.M + 63) / 64) * (g.N / NN)));
    hipLaunchKernelGGL((k_node_gemm<0, false, 2, 64>), grid64, block, LDS64_B3, s, g);
    return hipGetLastError();
  }
  if (g.wscale && nb == 3)
    hipLaunchKernelGGL((v1 ? k_node_gemm<1, true, 3> : k_node_gemm<0, true, 3>), grid, block, LDS3, s, g);
  else if (g.wscale)
    hipLaunchKernelGGL((v1 ? k_node_gemm<1, true, 2> : k_node_gemm<0, true, 2>), grid, block, NODE_LDS, s, g);
  else
    hipLaunchKernelGGL((v1 ? k_node_gemm<1, false, 2> : k_node_gemm<0, false, 2>), grid, block, NODE_LDS, s, g);
  return hipGetLastError();
}

}  // namespace chm
