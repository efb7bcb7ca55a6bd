// The two edge GEMMs of a CSP layer in "split16" arithmetic (cspnet.py:134-150:
// edge_mlp = Linear(1801, H) . SiLU . Linear(H, H) . SiLU over all n^2 edges).
//
// Both operands arrive pre-split into fp16 hi/lo planes, x = hi + lo, and a
// product is rebuilt from three fp16 MFMA products (a_hi w_lo + a_lo w_hi +
// a_hi w_hi, fp32 accumulation on v_mfma_f32_32x32x16_f16). Power-of-two
// scales keep every split operand <= 1 in magnitude, so the dropped a_lo w_lo
// term and the fp16 subnormal floor stay at fp32-rounding level:
//   * W rows: wscale[n] (split_planes_h), undone in the epilogue;
//   * edge layer 1's A = the Fourier features, |f| <= 1, unscaled;
//   * edge layer 2's A = S, scaled per (row, 128-column chunk) by 2^-e with e
//     from the chunk's max |S|. Edge layer 1's epilogue computes e and writes
//     S directly as scaled hi/lo planes; edge layer 2 rescales its fp32
//     accumulators by 2^(e_prev - e_next) at each chunk boundary (exact).
//
// Because no operand needs converting on the way in, all four planes are staged
// global -> LDS with global_load_lds (no VGPR round trip): a 4-deep LDS ring of
// K-tiles of 16 (32 KB each), counted vmcnt waits and one raw barrier per tile
// (cdna_hip_programming.md §5 'Pipelining across barriers'). 256x256 output
// tiles, 8 waves of 64x128; accumulators are C^T fragments (the W fragment is
// the MFMA A operand), so a lane owns an output row and float4 column groups.
//
// LDS image per plane and stage: [256 rows][16 fp16] = 32 B rows, the two 16-B
// k-halves of row r stored swapped when (r >> 3) & 1 (the glds source address is
// permuted, the LDS destination stays lane-linear), which makes the fragment
// reads (lanes 0-15 = rows 0-15, one k-half) cover all 64 banks.
#include "chm_internal.h"

#include <type_traits>

namespace chm {

#include "edge_common.h"

// Edge layer 1 epilogue, shared by both edge-GEMM kernels: acc holds D f for rows
// row0 + wm*64 + i*32 + r32 (i = 0, 1), columns n0 + wn*128 + j*32 + 8q + 4h + e, already
// multiplied by wscale. NW waves, ldsb bytes of free LDS.
template <int NW>
__device__ __forceinline__ void edge_epilogue(const EdgeArgs& g, f32x16 (&acc)[2][4], char* lds, int ldsb, int wave,
                                              int lane, long row0, long nrows, int n0, bool pre = false) {
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, r32 = lane & 31;
  const int PQ_ROWS = ldsb / (PQ_PITCH * 4);
    // S[c][e] = SiLU(acc + P_c[i] + Q_c[j]) written as hi/lo fp16 planes scaled by 2^-e per
    // 128-column chunk (this wave's columns), e from the chunk's max |S|. The tile's rows are
    // consecutive edges, so they touch few distinct nodes: the P rows of sources [ilo, ihi] and
    // the Q rows of the targets [jlo, jhi] (whole crystals) are staged into the free ring LDS
    // (this block's 256 columns, pitch 260 floats: the Q reads of 16 consecutive edges cover all
    // banks, the P reads broadcast) and read from there; tiles spanning too many nodes (crystals
    // of <= 3 atoms, crystal-boundary tiles at n > 75) gather from global memory instead.
    const long rl = row0 + nrows - 1;
    const int ilo = g.ei[row0], ihi = g.ei[rl];
    const int glo = g.n2g[ilo], ghi = g.n2g[ihi];
    const int jlo = g.node_off[glo], jhi = g.node_off[ghi] + g.natoms[ghi] - 1;
    const int nP = ihi - ilo + 1, nQ = jhi - jlo + 1;
    // pre: the main loop already staged both conditionings (rows [0, nR) and [PRE_ROW1, ...))
    const bool staged = pre || nP + nQ <= PQ_ROWS;
    const float* T = reinterpret_cast<const float*>(lds + PQ_OFF);
    long rowv[2];
    int pr[2], qr[2];  // staged: LDS rows; gathered: node indices
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long lr = wm * 64 + i * 32 + r32;
      rowv[i] = row0 + (lr < nrows ? lr : nrows - 1);
      pr[i] = g.ei[rowv[i]];
      qr[i] = g.ej[rowv[i]];
      if (staged) {
        pr[i] -= ilo;
        qr[i] = nP + qr[i] - jlo;
      }
    }
    _Float16* S0 = reinterpret_cast<_Float16*>(g.S);
    // Stores count in vmcnt (gfx9), so a load issued after conditioning 0's S stores and then
    // waited on would wait for those stores to drain: when both conditionings' rows fit, they are
    // staged together before any store (rows [c * nR, (c + 1) * nR)).
    const int nR = nP + nQ;
    const bool both = pre || (staged && g.npairs * nR <= PQ_ROWS);
    auto stage = [&](int c0, int c1) {  // conditionings [c0, c1)
      if (!staged || pre) return;
      if (c0 > 0) __syncthreads();  // everyone is done reading the previous conditioning
      for (int c = c0; c < c1; ++c) {
        const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
        const int rb = both ? c * nR : 0;
        for (int r = wave; r < nR; r += NW) {
          const float* src = Pc + (r < nP ? (long)(ilo + r) * (2 * H) : (long)(jlo + r - nP) * (2 * H) + H) + n0 + 4 * lane;
          __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds + PQ_OFF + (rb + r) * PQ_PITCH * 4), 16, 0,
                                           0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    };
    // conditioning c; LAST: the final one, whose SiLU values may overwrite acc; STG: P / Q rows
    // from the staged LDS image (else gathered from global memory). Both flags are compile-time
    // so each path is straight-line code.
    const bool nostore = g.dbg & 4;  // (profiling)
    auto run = [&](int c, auto LAST, auto STG) {
      constexpr bool last = decltype(LAST)::value, stg = decltype(STG)::value;
      const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
      const int rb = pre ? c * PRE_ROW1 : (both ? c * nR : 0);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const long lr = wm * 64 + i * 32 + r32;  // rows past nrows compute clamped copies, never stored
        const long row = rowv[i];
        const float* prow;
        const float* qrow;
        if constexpr (stg) {
          prow = T + (rb + pr[i]) * PQ_PITCH + wn * 128 + 4 * h;
          qrow = T + (rb + qr[i]) * PQ_PITCH + wn * 128 + 4 * h;
        } else {
          prow = Pc + (long)pr[i] * (2 * H) + n0 + wn * 128 + 4 * h;
          qrow = Pc + (long)qr[i] * (2 * H) + H + n0 + wn * 128 + 4 * h;
        }
        // SiLU values: conditioning 0 in v (acc is needed again), the last one in place
        f32x4 v[4][4];
        float mx = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 p = *reinterpret_cast<const f32x4*>(prow + j * 32 + 8 * q);
            const f32x4 qv = *reinterpret_cast<const f32x4*>(qrow + j * 32 + 8 * q);
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              const f32x2e a2 = {acc[i][j][4 * q + e], acc[i][j][4 * q + e + 1]};
              const f32x2e x = silu_e2((a2 + f32x2e{p[e], p[e + 1]}) + f32x2e{qv[e], qv[e + 1]});
              mx = fmaxf(mx, fmaxf(fabsf(x.x), fabsf(x.y)));
              if constexpr (last) {
                acc[i][j][4 * q + e] = x.x;
                acc[i][j][4 * q + e + 1] = x.y;
              } else {
                v[j][q][e] = x.x;
                v[j][q][e + 1] = x.y;
              }
            }
          }
        auto val = [&](int j, int q, int e) {
          if constexpr (last) return acc[i][j][4 * q + e];
          else return v[j][q][e];
        };
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));  // lanes h = 0, 1 share the row
        const int ex2 = exp_of(mx);
        const float sc = ldexpf(1.0f, -ex2);
        const long orow = (long)c * g.E + row;
        _Float16* srow = S0 + orow * (2 * H) + ((n0 + wn * 128) / 32) * 64 + 16 * h;  // [H/32][hi 32 | lo 32]
        // S is stored with the columns of each 32-chunk permuted, 8q + 4h + e -> 16h + 4q + e
        // (W2's K index carries the same permutation, split_rows_h(perm)), so a lane's 16 values
        // of a chunk are contiguous: two 16-B stores per plane. (Routing the lines through LDS so
        // that each instruction writes 8 whole lines measured no faster.)
        if (lr < nrows && !nostore) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f16x8 hv[2], lv[2];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float x = val(j, q, e) * sc;
                const _Float16 hx = (_Float16)x;
                hv[q >> 1][4 * (q & 1) + e] = hx;
                lv[q >> 1][4 * (q & 1) + e] = (_Float16)(x - (float)hx);
              }
            _Float16* d = srow + j * 64;
            *reinterpret_cast<f16x8*>(d) = hv[0];
            *reinterpret_cast<f16x8*>(d + 8) = hv[1];
            *reinterpret_cast<f16x8*>(d + 32) = lv[0];
            *reinterpret_cast<f16x8*>(d + 40) = lv[1];
          }
          if (h == 0) reinterpret_cast<signed char*>(g.sexp)[orow * 4 + (n0 + wn * 128) / CHUNK] = (signed char)ex2;
        }
      }
    };
    using F = std::integral_constant<bool, false>;
    using Tr = std::integral_constant<bool, true>;
    auto all = [&](auto STG) {
      if (g.npairs > 1) {
        if (both) {
          stage(0, 2);
          if (g.trace && !(g.dbg & 4096) && threadIdx.x == 0) g.trace[6 * blockIdx.x + 4] = rtime();
          run(0, F{}, STG);
          if (g.trace && !(g.dbg & 4096) && threadIdx.x == 0) g.trace[6 * blockIdx.x + 5] = rtime();
        } else {
          stage(0, 1);
          run(0, F{}, STG);
          stage(1, 2);
        }
        run(1, Tr{}, STG);
      } else {
        stage(0, 1);
        run(0, Tr{}, STG);
      }
    };
    if (staged)
      all(Tr{});
    else
      all(F{});
}

// VAR (microbenchmark variants of the main-loop schedule; the product uses 0 = 3, the explicit
// MFMA / memory-op interleave): 1 = compiler schedule without s_setprio around the MFMA groups,
// 2 = compiler schedule with the A loads between the MFMA groups, 4 = compiler schedule
template <int EPI, bool ASC, int VAR = 0>
__global__ __launch_bounds__(512, 1) void k_edge_gemm(EdgeArgs g) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, r32 = lane & 31;
  const int ntn = g.N / BN;
  const long bid = remap(blockIdx.x, gridDim.x);
  const int n0 = (int)(bid % ntn) * BN;
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
    row0 = (bid / ntn) * BM;
    nrows = g.M - row0 < BM ? g.M - row0 : BM;
  }
  const int K = g.K, nk = K / BK;
  const unsigned long long t0 = g.trace ? rtime() : 0;
  const unsigned long long c0 = (g.trace && (g.dbg & 4096)) ? ctime() : 0;  // (clock probe)
  // Every block of a launch does the same work, so CUs that start together stay in lockstep and
  // their epilogues (S / agg stores, VALU-only) coincide: the store bursts then saturate HBM while
  // no CU computes. Holding back every other CU of the first round by about half a tile
  // (blocks 0-255 take one CU each; XCD = block % 8) keeps half the chip in its main loop
  // whenever the other half is in its epilogue, for the rest of the launch.
  if (g.stagger > 0 && blockIdx.x < 256 && ((blockIdx.x >> 3) & 1))
    for (int k = 0; k < g.stagger; ++k) __builtin_amdgcn_s_sleep(127);

  // ---- glds sources. Operand rows are stored [K/32][hi 32 | lo 32] (fp16): the K-tile of a row
  // is one 128-B line. Wave w stages rows 32w..32w+31 of both operands, 8 rows per instruction;
  // lane -> (row 32w + 8q + (lane >> 3), LDS chunk lane & 7) holding line chunk
  // (lane & 7) ^ swz(row), swz(row) = (row >> 1) & 7.
  const char* Ab = reinterpret_cast<const char*>(g.A);
  const char* Wb = reinterpret_cast<const char*>(g.W);
  const long rowB = (long)K * 4;  // bytes per operand row
  // uniform block bases + 32-bit per-lane offsets (keeps the address VGPRs few)
  const char* Ablk = Ab + row0 * rowB;
  const char* Wblk = Wb + (long)n0 * rowB;
  const int lr0 = wave * 32 + (lane >> 3);
  // swz(r + 8q) = ((r >> 1) + 4q) & 7 = swz(r) ^ 4 (q & 1): the chunk offset alternates with q
  const unsigned lc16 = 16u * (unsigned)((lane & 7) ^ ((lr0 >> 1) & 7));
  const unsigned lc16x = lc16 ^ 64u;
  // A rows past the tile's nrows are read unclamped: the A buffers (F, S) carry 256 rows of
  // padding, and those rows' accumulators are never stored. A and W then share one set of
  // per-lane offsets (no per-issue clamp arithmetic in the loop).
  const unsigned woff = (unsigned)(lr0 * rowB) + lc16;
  const unsigned wq = (unsigned)(8 * rowB);
  char* dst = lds + wave * 32 * ROW_B;
  // past the end of K the loads re-read the last tile into an idle stage
  auto issueA = [&](int t) {
    const char* src = Ablk + (long)(t < nk ? t : nk - 1) * ROW_B;
    char* d = dst + (t % NSA) * OPND_B;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (woff + q * wq + ((q & 1) ? (lc16x - lc16) : 0u))),
                                       (lds_void*)(d + q * 8 * ROW_B), 16, 0, 0);
  };
  auto issueW = [&](int t) {
    const char* src = Wblk + (long)(t < nk ? t : nk - 1) * ROW_B;
    char* d = dst + W_RING + (t % NSW) * OPND_B;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (woff + q * wq + ((q & 1) ? (lc16x - lc16) : 0u))),
                                       (lds_void*)(d + q * 8 * ROW_B), 16, 0, 0);
  };

  // ---- row exponents of the A chunks (edge layer 2)
  int ex[2] = {0, 0};
  if (ASC) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long lr = wm * 64 + i * 32 + r32;
      ex[i] = g.aexp[row0 + (lr < nrows ? lr : nrows - 1)];
    }
  }

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // fragment (plane p, k-step ks, k-half h) of row r: logical chunk c = 4p + 2ks + h at
  // physical chunk c ^ swz(r); swz depends on r32 only (tile rows are multiples of 16 apart)
  const int swz = (r32 >> 1) & 7;
  const int fa = (wm * 64 + r32) * ROW_B;
  const int fw = (wn * 128 + r32) * ROW_B;
  f16x8 fa_[2][2][2], fw_[2][2][4];  // [set][plane][i / j]
  auto read_frags = [&](int set, int t, int ks) {
    const char* SA = lds + (t % NSA) * OPND_B;
    const char* SW = lds + W_RING + (t % NSW) * OPND_B;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ch = 16 * ((4 * p + 2 * ks + h) ^ swz);
#pragma unroll
      for (int i = 0; i < 2; ++i) fa_[set][p][i] = *reinterpret_cast<const f16x8*>(SA + fa + i * 32 * ROW_B + ch);
#pragma unroll
      for (int j = 0; j < 4; ++j) fw_[set][p][j] = *reinterpret_cast<const f16x8*>(SW + fw + j * 32 * ROW_B + ch);
    }
  };
  auto mfma_group = [&](int set, int pw, int pa) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fw_[set][pw][j], fa_[set][pa][i], acc[i][j], 0, 0, 0);
  };
  auto mfmas = [&](int set) {
    if (VAR != 1) __builtin_amdgcn_s_setprio(1);
    // small terms first: w_lo a_hi, w_hi a_lo, then w_hi a_hi
    mfma_group(set, 1, 0);
    mfma_group(set, 0, 1);
    mfma_group(set, 0, 0);
    if (VAR != 1) __builtin_amdgcn_s_setprio(0);
  };
  auto rescale = [&](int t) {
    if (ASC && t > 0 && (t * BK) % CHUNK == 0) {
      const int c = (t * BK) / CHUNK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ep = (int)(signed char)(ex[i] >> (8 * (c - 1)));
        const int en = (int)(signed char)(ex[i] >> (8 * c));
        const float f = ldexpf(1.0f, ep - en);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] *= f;
      }
    }
  };

  // rings: A tile t in A stage t % 3 (two tiles of HBM latency cover), W tile t in W stage t % 2.
  // Fragments are double-buffered per 16-deep k-step: the barrier that publishes tile t+1 (and
  // frees tile t's stages) sits between tile t's two MFMA groups, so LDS reads run under MFMAs.
  // Issue order W0 A0 A1 W1 A2 | W2 A3 | W3 A4 ...: when tile t+1 is needed only A(t+2) may be
  // outstanding, vmcnt(4).
  issueW(0);
  issueA(0);
  issueA(1);
  issueW(1);
  issueA(2);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_frags(0, 0, 0);
  // EPI_EDGE: stage the epilogue's P / Q rows during the last two K-tiles (their latency then hides
  // under those MFMAs) when the ring layout allows (nk % 6 == 0) and the rows fit (nR <= PRE_MAX)
  bool pre = false;
  int p_ilo = 0, p_jlo = 0, p_nP = 0, p_nR = 0;
  if constexpr (EPI == EPI_EDGE) {
    if (nk % 6 == 0 && !(g.dbg & 2048)) {
      const long rl = row0 + nrows - 1;
      p_ilo = g.ei[row0];
      const int ihi = g.ei[rl], ghi = g.n2g[ihi];
      p_jlo = g.node_off[g.n2g[p_ilo]];
      p_nP = ihi - p_ilo + 1;
      p_nR = p_nP + g.node_off[ghi] + g.natoms[ghi] - p_jlo;
      pre = p_nR <= PRE_MAX;
    }
  }
  auto stage_rows = [&](int c, int rbase) {
    const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
    for (int r = wave; r < p_nR; r += 8) {
      const float* src = Pc + (r < p_nP ? (long)(p_ilo + r) * (2 * H) : (long)(p_jlo + r - p_nP) * (2 * H) + H) + n0 +
                         4 * lane;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds + (rbase + r) * PQ_PITCH * 4), 16, 0, 0);
    }
  };
  const int nmain = pre ? nk - 3 : nk;
  for (int t = 0; t < nmain; ++t) {
    __builtin_amdgcn_s_waitcnt(0xC07F);                // lgkmcnt(0): set 0 (read under the last MFMAs) is in
    if (VAR == 0 || VAR == 3 || VAR >= 5) {
      // explicit interleave: each fragment read / load issue sits between two MFMAs (+7.5% over
      // the compiler's schedule, which clusters the 8 load issues and 12 reads ahead of the MFMAs;
      // VAR 4 keeps that schedule for comparison)
      rescale(t);
      if (VAR != 7) __builtin_amdgcn_s_setprio(1);
      read_frags(1, t, 1);
      mfma_group(0, 1, 0);
      mfma_group(0, 0, 1);
      mfma_group(0, 0, 0);
      if (VAR != 3) {  // reads spread one per two MFMAs (VAR 3: the first twelve MFMAs)
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
      }
      if (VAR != 7) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (VAR != 7) __builtin_amdgcn_s_setprio(1);
      issueW(t + 2);
      issueA(t + 3);
      read_frags(0, t + 1, 0);
      mfma_group(1, 1, 0);
      mfma_group(1, 0, 1);
      mfma_group(1, 0, 0);
      if (VAR == 6) {  // (microbenchmark) load issues first, then reads between MFMAs
        __builtin_amdgcn_sched_group_barrier(0x010, 8, 1);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 12, 1);
      } else if (VAR == 5) {  // (microbenchmark) load issues and reads mixed 2 : 3 between MFMAs
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 1);
      } else if (VAR == 8) {  // (microbenchmark) reads first (they feed the next tile), loads later
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 1);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
        }
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 1);
      }
      if (VAR != 7) __builtin_amdgcn_s_setprio(0);
      continue;
    }
    read_frags(1, t, 1);
    rescale(t);
    mfmas(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);                // this wave is done reading tile t
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // this thread's part of tile t+1 has landed
    if (!(g.dbg & 2)) __builtin_amdgcn_s_barrier();   // everyone's has; tile t's stages are free
    asm volatile("" ::: "memory");
    if (VAR == 2) {
      if (!(g.dbg & 1)) issueW(t + 2);
      read_frags(0, t + 1, 0);
      __builtin_amdgcn_s_setprio(1);
      mfma_group(1, 1, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (!(g.dbg & 1)) issueA(t + 3);
      __builtin_amdgcn_sched_barrier(0);
      mfma_group(1, 0, 1);
      mfma_group(1, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      continue;
    }
    if (!(g.dbg & 1)) {
      issueW(t + 2);
      issueA(t + 3);
    }
    read_frags(0, t + 1, 0);                           // past the end: reads a re-read tile
    mfmas(1);
  }
  // pre-staging: the last three K-tiles, without the tail re-reads (their stages receive the
  // epilogue's data instead)
  for (int t = nk - 3; pre && t < nk; ++t) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    read_frags(1, t, 1);
    rescale(t);
    mfmas(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);                 // this wave is done reading tile t
    if (t == nk - 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile nk-2 (A nk-1 in flight)
    if (t == nk - 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile nk-1
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t == nk - 3) issueW(t + 2);
    if constexpr (EPI == EPI_EDGE) {
      if (t == nk - 2) stage_rows(0, 0);
      if (t == nk - 1 && g.npairs > 1) stage_rows(1, PRE_ROW1);
    }

    if (t < nk - 1) read_frags(0, t + 1, 0);
    mfmas(1);
  }
  // EPI_SEGMEAN: the epilogue's per-column W scale and bias, one column group ahead (double-buffered
  // in act() below); the first group is issued here, behind the ring's last loads
  f32x4 sc[2][4], bb[2][4];
  auto ld_sb = [&](auto jc) {
    constexpr int j = decltype(jc)::value;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = n0 + wn * 128 + j * 32 + 8 * q + 4 * h;
      sc[j & 1][q] = *reinterpret_cast<const f32x4*>(g.wscale + c);
      bb[j & 1][q] = *reinterpret_cast<const f32x4*>(g.bias + c);
    }
  };
  // drain the ring (the tail re-reads still land in LDS) before the epilogue reuses it
  if constexpr (EPI == EPI_SEGMEAN) {
    if (!(g.dbg & 128)) {
      ld_sb(std::integral_constant<int, 0>{});
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // everything but those 8 loads
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  // EPI_SEGMEAN: the tile's node list {atom count, first row in the tile} for thread tid < nodes,
  // loaded first so its two dependent loads overlap the scale loads and the SiLU below
  int2 my = {0, 0};
  if (EPI == EPI_SEGMEAN && !(g.dbg & 128)) {
    const long es0 = g.node_estart[seg.x];
    if (tid < seg.y - seg.x) {
      const int nd = seg.x + tid;
      my.x = g.node_n[nd];  // independent loads (no n2g -> natoms chain)
      my.y = (int)(g.node_estart[nd] - es0);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep them issued here, ahead of the scale undo and SiLU
  }

  // ---- undo the scales: W rows (columns of the output) and the last A chunk
  float rs[2] = {1.0f, 1.0f};
  if (ASC) {
#pragma unroll
    for (int i = 0; i < 2; ++i) rs[i] = ldexpf(1.0f, (int)(signed char)(ex[i] >> (8 * (K / CHUNK - 1))));
  }
  if constexpr (EPI != EPI_SEGMEAN) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 sc = *reinterpret_cast<const f32x4*>(g.wscale + n0 + wn * 128 + j * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] *= sc[e] * rs[i];
      }
  }

  // lane l owns output row wm*64 + i*32 + (l & 31) and, per 4-register group q,
  // the four consecutive columns wn*128 + j*32 + 8q + 4h .. +3
  if (EPI == EPI_SEGMEAN) {
    // two passes of 128 columns: the wn-th half of the waves writes SiLU(acc + b2) to an
    // LDS tile [256][132], then every thread sums node segments of one column in edge order.
    // The tile's node list (atom count, first row; loaded before the scale undo) is kept in LDS
    // after the tile (int2 [<= 256]).
    if (g.dbg & 128) return;  // (profiling: main loop only)
    const unsigned long long tm = g.trace ? rtime() : 0;
    float* T = reinterpret_cast<float*>(lds);
    int2* info = reinterpret_cast<int2*>(lds + SEG_B);
    const int nn = seg.y - seg.x;
    // every wave undoes the scales and applies bias + SiLU to its accumulators first (all eight
    // waves at once), then the owners of each 128-column half write it to the tile. The scale and
    // bias vectors are loaded one column group ahead (double-buffered) rather than all up front,
    // which would spill.
    auto act = [&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (j < 3) ld_sb(std::integral_constant<int, j + 1>{});
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2e a2 = {acc[i][j][4 * q + e], acc[i][j][4 * q + e + 1]};
            const f32x2e s2 = f32x2e{sc[j & 1][q][e], sc[j & 1][q][e + 1]} * rs[i];
            const f32x2e x = silu_e2(a2 * s2 + f32x2e{bb[j & 1][q][e], bb[j & 1][q][e + 1]});
            acc[i][j][4 * q + e] = x.x;
            acc[i][j][4 * q + e + 1] = x.y;
          }
      // pin this group's math ahead of the next group's loads (which stay behind the clobber)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          asm volatile("" : "+v"(acc[i][j][4 * q]), "+v"(acc[i][j][4 * q + 1]), "+v"(acc[i][j][4 * q + 2]),
                       "+v"(acc[i][j][4 * q + 3])::"memory");
    };
    act(std::integral_constant<int, 0>{});
    act(std::integral_constant<int, 1>{});
    act(std::integral_constant<int, 2>{});
    act(std::integral_constant<int, 3>{});
    if (g.trace && !(g.dbg & 4096) && tid == 0) g.trace[6 * blockIdx.x + 4] = rtime();  // (profiling) SiLU done
    for (int half = 0; half < 2; ++half) {
      if (half == 1 && g.trace && !(g.dbg & 4096) && tid == 0) g.trace[6 * blockIdx.x + 5] = rtime();  // first half summed
      if (wn == half) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int col = j * 32 + 8 * q + 4 * h;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              const int row = wm * 64 + i * 32 + r32;
              f32x4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
              *reinterpret_cast<f32x4*>(T + row * SEG_TP + col) = v;
            }
          }
      }
      if (half == 0 && tid < nn) info[tid] = my;
      __syncthreads();
      const int col = tid & 127;
      for (int k = tid >> 7; k < nn && !(g.dbg & 256); k += 4) {
        const int2 ni = info[k];
        const float* src = T + ni.y * SEG_TP + col;
        // sequential sum in edge order (scatter_add's order); loads issued eight at a time
        float sacc = 0.f;
        int j = 0;
        for (; j + 8 <= ni.x; j += 8) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = src[(j + u) * SEG_TP];
#pragma unroll
          for (int u = 0; u < 8; ++u) sacc += v[u];
        }
        for (; j < ni.x; ++j) sacc += src[j * SEG_TP];
        const float mean = sacc / (float)(ni.x < 1 ? 1 : ni.x);
        if (!(g.dbg & 4)) g.agg[((long)seg_c * g.nnodes + seg.x + k) * H + n0 + half * 128 + col] = mean;
        if (g.agg_max) {  // the node row's max |agg| for the split16 node GEMM reading it (a wave = one node)
          float m = fabsf(mean);
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
          if (lane == 0) atomicMax(g.agg_max + (long)seg_c * g.nnodes + seg.x + k, __float_as_uint(m));
        }
      }
      __syncthreads();
    }
    if (g.trace && tid == 0) {
      unsigned long long* o = g.trace + 6 * blockIdx.x;
      o[0] = hwid(); o[1] = t0; o[2] = tm; o[3] = rtime();
      if (g.dbg & 4096) { o[4] = c0; o[5] = ctime(); }
    }
    return;
  }

  if (EPI == EPI_EDGE) {
    const unsigned long long tm = g.trace ? rtime() : 0;
    edge_epilogue<8>(g, acc, lds, LDS_B, wave, lane, row0, nrows, n0, pre);
    if (g.trace) {
      __syncthreads();
      if (tid == 0) {
        unsigned long long* o = g.trace + 6 * blockIdx.x;
        o[0] = hwid(); o[1] = t0; o[2] = tm; o[3] = rtime();
        if (g.dbg & 4096) { o[4] = c0; o[5] = ctime(); }
      }
    }
    return;
  }

  if (EPI == EPI_STD && !g.C) return;  // (microbenchmark: main loop only)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long lr = wm * 64 + i * 32 + r32;
    if (lr >= nrows) continue;
    const long row = row0 + lr;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = n0 + wn * 128 + j * 32 + 8 * q + 4 * h;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
        *reinterpret_cast<f32x4*>(g.C + row * g.ldc + col) = v;
      }
  }
}

hipError_t edge_gemm_init() {
  const void* ks[] = {(const void*)k_edge_gemm<EPI_STD, false>, (const void*)k_edge_gemm<EPI_EDGE, false>,
                      (const void*)k_edge_gemm<EPI_SEGMEAN, true>, (const void*)k_edge_gemm<EPI_STD, true>};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_B);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

#ifdef CHM_MICROBENCH  // (tools/gemm_bench.cpp: main-loop schedule variants)
hipError_t edge_gemm_variant(const EdgeArgs& g, int var, hipStream_t s) {
  const void* ks[] = {(const void*)k_edge_gemm<EPI_STD, false, 0>, (const void*)k_edge_gemm<EPI_STD, false, 1>,
                      (const void*)k_edge_gemm<EPI_STD, false, 2>, (const void*)k_edge_gemm<EPI_STD, false, 3>,
                      (const void*)k_edge_gemm<EPI_STD, false, 4>, (const void*)k_edge_gemm<EPI_STD, false, 5>,
                      (const void*)k_edge_gemm<EPI_STD, false, 6>, (const void*)k_edge_gemm<EPI_STD, false, 7>,
                      (const void*)k_edge_gemm<EPI_STD, false, 8>};
  if (var < 0 || var > 8) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    for (const void* k : ks) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_B);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  const long blocks = ((g.M + BM - 1) / BM) * (g.N / BN);
  EdgeArgs ga = g;
  void* args[] = {&ga};
  return hipLaunchKernel(ks[var], dim3((unsigned)blocks), dim3(512), args, LDS_B, s);
}

#endif

hipError_t edge_gemm(const EdgeArgs& g, int epi, hipStream_t s) {
  if (g.N % BN || g.K % BK || !g.A || !g.W || !g.wscale) return hipErrorInvalidValue;
  const bool asc = g.aexp != nullptr;
  if (asc && (g.K % CHUNK || g.K / CHUNK > 4)) return hipErrorInvalidValue;
  long blocks;
  if (epi == EPI_SEGMEAN) {
    if (g.N != H || !g.tiles || !g.agg || !g.bias || !asc || !g.node_n) return hipErrorInvalidValue;
    blocks = (long)g.ntiles * g.npairs * (g.N / BN);
  } else {
    if (g.M <= 0 || g.row_base) return hipErrorInvalidValue;  // (row ranges: k_edge16 only)
    if (epi == EPI_EDGE && (g.N != H || !g.S || !g.sexp || !g.PQ || !g.node_off || !g.natoms || !g.n2g || asc)) return hipErrorInvalidValue;
    blocks = ((g.M + BM - 1) / BM) * (g.N / BN);
  }
  static bool attr = false;
  if (!attr) {
    hipError_t e = edge_gemm_init();
    if (e != hipSuccess) return e;
    attr = true;
  }
  const dim3 grid((unsigned)blocks), block(512);
  if (epi == EPI_EDGE)
    hipLaunchKernelGGL((k_edge_gemm<EPI_EDGE, false>), grid, block, LDS_B, s, g);
  else if (epi == EPI_SEGMEAN)
    hipLaunchKernelGGL((k_edge_gemm<EPI_SEGMEAN, true>), grid, block, LDS_B, s, g);
  else if (asc)
    hipLaunchKernelGGL((k_edge_gemm<EPI_STD, true>), grid, block, LDS_B, s, g);
  else
    hipLaunchKernelGGL((k_edge_gemm<EPI_STD, false>), grid, block, LDS_B, s, g);
  return hipGetLastError();
}

// W [N][K] -> split rows [N][K/cw][hi cw | lo cw] of W * 2^-e_n, e_n the exponent of
// max_k |W[n][k]| (every scaled entry <= 1), and wscale[n] = 2^e_n. One block per row. cw = 32
// for the edge GEMMs, 16 for the split16 node GEMMs.
// perm (cw = 32): the column permutation within each 32-chunk that edge layer 1's epilogue writes S
// in, applied to W2's K index: 1 = k_edge_gemm (8q + 4h + e -> 16h + 4q + e), 2 = k_edge16
// (16a + 4g + r -> 8g + 4a + r).
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
    const int pc = perm == 1 ? 16 * ((c >> 2) & 1) + 4 * (c >> 3) + (c & 3)     // 8q + 4h + e -> 16h + 4q + e
                 : perm == 2 ? 8 * ((c >> 2) & 3) + 4 * (c >> 4) + (c & 3)      // 16a + 4g + r -> 8g + 4a + r
                 : c;
    o[(k / cw) * 2 * cw + pc] = hi;
    o[(k / cw) * 2 * cw + cw + pc] = (_Float16)(x - (float)hi);
  }
  if (threadIdx.x == 0) wscale[n] = ldexpf(1.0f, e);
}

hipError_t split_rows_h(const float* W, int N, int K, void* out, float* wscale, int perm, hipStream_t s, int chunk) {
  if ((chunk != 32 && chunk != 16) || K % chunk || (perm && chunk != 32)) return hipErrorInvalidValue;
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
