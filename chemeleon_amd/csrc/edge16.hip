// The two split16 edge GEMMs of a CSP layer (cspnet.py:134-160: edge_mlp over all n^2 edges, then
// scatter_mean) on v_mfma_f32_16x16x32_f16.
//
// Split rows [K/32][hi 32 | lo 32] fp16 (split16.hip) staged by global_load_lds into a 3-deep A ring
// and a 2-deep W ring, 256x256 output tiles, 8 waves of 64 rows x 128 columns, one block per CU,
// three fp16 MFMA products per fp32 product. The MFMA shape: both 16x16x32 and 32x32x16 run the matrix
// pipe at the same FLOP per cycle, but under load the chip holds a higher clock on 16x16x32: back-to-
// back on random operands at two waves per SIMD, 1.91 GHz against 1.67 GHz for 32x32x16 (+14% FLOP/s,
// tools/mfma_shape_probe.hip, profiles/r2/mfma_shape_probe.log; the round-1 32x32x16 kernels were
// removed in round 3).
//
// Per K-tile of 32 a wave reads its four 16-row A fragments and, in four quarters of 32 columns,
// its W fragments (lane l: row l & 15, k-chunk l >> 4 of the 128-B line, XOR-swizzled so every
// 16-lane group of a ds_read_b128 covers all 64 banks); the 96 MFMAs of the tile run as four
// quarters of 24 with the next quarter's fragment reads between them, the tile's barrier before
// the last quarter, and the next tile's A fragments read under that quarter.
//
// Accumulators are C^T fragments: lane l holds edge row (l & 15) of each 16-row group and output
// columns 16j + 4(l >> 4) .. +3 of each 16-column group j. Edge layer 1 stores S with the columns
// of each 32-chunk permuted, 16a + 4g + r -> 8g + 4a + r (one 16-B store per plane), and W2's K
// index is split with the same permutation (split_rows_h perm 2).
#include "chm_internal.h"

#include <algorithm>
#include <type_traits>

namespace chm {

#include "edge_common.h"

// the segment-mean epilogue reads its row tile's node list from the host-built table (EdgeArgs::rinfo)
// instead of deriving it through dependent loads (A/B builds: -DCHM_SEG_TABLE=0)
#ifndef CHM_SEG_TABLE
#define CHM_SEG_TABLE 1
#endif
constexpr bool kSegTable = CHM_SEG_TABLE;
// block timelines of the pair grid (CHM_EDGE_TRACE_LAYER=4) are compiled in only by A/B builds
// (CHM_BUILD_DEFS=-DCHM_GRID_TRACE=1): the product kernel's registers stay as they are
#ifndef CHM_GRID_TRACE
#define CHM_GRID_TRACE 0
#endif
constexpr bool kGridTrace = CHM_GRID_TRACE;
// K-loop ablations of A/B builds only (CHM_BUILD_DEFS=-DCHM_LOOP_ABL=n; wrong results, read in cycles): bit 0 = no
// per-K-tile s_barrier, 1 = no vmcnt waits, 2 = no operand loads in the loop, 3 = no lgkmcnt waits before the quarters
#ifndef CHM_LOOP_ABL
#define CHM_LOOP_ABL 0
#endif
constexpr bool kAblBar = CHM_LOOP_ABL & 1, kAblVm = CHM_LOOP_ABL & 2, kAblLd = CHM_LOOP_ABL & 4, kAblLgkm = CHM_LOOP_ABL & 8;
// Branch-free K loops (r6): every K-tile issues its operand loads (past the end of K they re-read the last tile into the
// stage just freed) and waits with one vmcnt, so the tile body is one basic block and its sched_group_barrier
// interleaving of loads and MFMAs takes effect (conditional loads were a block of their own, issued as a burst).
// Not for the directed layer-1 tiles (EPI_EDGE), whose last K-tiles stage P / Q rows into the A ring.
// (A/B builds: -DCHM_LOOP_UNI=0 restores the conditional form)
#ifndef CHM_LOOP_UNI
#define CHM_LOOP_UNI 1
#endif
constexpr bool kLoopUni = CHM_LOOP_UNI;
// The epilogues' profiling ablations (CHM_EDGE_DBG 4 no stores, 131072 / 262144 reverse-direction store variants,
// 524288 P / Q rows not loaded, 2097152 no exponent bytes; edge layer 2: 4 no agg stores, 32 no segment sums) in A/B
// builds only (-DCHM_PAIR_ABL=1): as runtime tests in the product they cost the pair epilogue a zero-fill and a
// branch around every P / Q read (r6)
#ifndef CHM_PAIR_ABL
#define CHM_PAIR_ABL 0
#endif
constexpr bool kPairAbl = CHM_PAIR_ABL;
// (edge layer 2's SiLU ablation select, dbg 8: compiled in only by A/B builds -DCHM_L2_SEL=1; r6 same-box A/B without it
// 512x40 50.87 -> 50.71 ms per step, 64x40 7.37 -> 7.31, 64x20 2.647 -> 2.625, bit-identical: profiles/r6/l2_sel/)
#ifndef CHM_L2_SEL
#define CHM_L2_SEL 0
#endif
constexpr bool kL2Sel = CHM_L2_SEL;

namespace {

__device__ __forceinline__ f32x4 mfma16(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// f(integral_constant<int, k>) for k = 0 .. N-1: compile-time register indices in epilogue loops
// whose bodies are too large for the unroller (a runtime index would put acc in scratch)
template <int K, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    static_for<K + 1, N>(f);
  }
}

// Cross-tile exchange of the row-tile segment sums (tiles of one grid on different XCDs): the
// partial sums and continued rows are stored and loaded as agent-scope atomics (sc1: written through
// to memory, read past the XCD's L2), ordered by s_waitcnt around the counter. No agent-scope fences:
// those write back / invalidate the whole L2 of the XCD (measured: edge layer 2 +20%).
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// edge_events_* (chm_internal.h): wait timeouts and repairs, counted on the device
__device__ unsigned long long g_edge_events[EV_COUNT];
__device__ __forceinline__ void count_event(int k) {
  __hip_atomic_fetch_add(&g_edge_events[k], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the XCD (XCC) this wave runs on
__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}

}  // namespace

// k_edge16_layer's block -> job map (host and device: chm_debug_layer_jobs tests it). XCD x = b % 8
// walks row tiles [R x / 8, R (x + 1) / 8) as groups i = 0 .. n + d - 1: layer-1 tiles (i, 0), (i, 1)
// while i < n, then the layer-2 tiles of row tile i - d (P conditionings x 2 column tiles) from i = d.
// kind 0 = no job (padding), 1 = layer 1 with tile index bid = row tile * 2 + column tile, 2 = layer 2
// with bid = (row tile * P + conditioning) * 2 + column tile.
struct LayerJob { int kind; long bid; };
__host__ __device__ inline LayerJob layer_job(long b, long R, int P, int D) {
  const long x = b & 7, k = b >> 3;
  const long lo = R * x / 8, hi = R * (x + 1) / 8, n = hi - lo;
  const long G = 2 + 2L * P, d = D < n ? D : n;
  long i, s;
  if (k < 2 * d) {
    i = k / 2;
    s = k % 2;
  } else if (k - 2 * d < (n - d) * G) {
    i = d + (k - 2 * d) / G;
    s = (k - 2 * d) % G;
  } else {
    const long k2 = k - 2 * d - (n - d) * G;
    if (k2 >= d * 2 * P) return LayerJob{0, 0};
    i = n + k2 / (2 * P);
    s = 2 + k2 % (2 * P);
  }
  if (s < 2) return LayerJob{1, (lo + i) * 2 + s};
  return LayerJob{2, ((lo + i - d) * P + (s - 2) / 2) * 2 + (s - 2) % 2};
}

// one output tile: virtual block vb of nvb (the XCD-aware remap turns it into a tile index), or the
// tile index itself (bid_in >= 0). ONE (k_edge16_layer, both edge layers in one grid): layer-2 tiles
// wait for the layer-1 tiles of their rows (EdgeArgs::lflags) and read S through the XCD's L2, which
// is coherent only if those layer-1 tiles ran on the same XCD: the layer-1 tiles record their XCD in
// the flag word and a layer-2 tile that finds another one raises *xbad (the runtime's repair launches
// then recompute the layer).
// RG: 16-row groups per wave (4: 256-row tiles; 3: edge layer 2's 192-row tiles, k_edge16_short). The operand
// staging loads 256 A rows either way (the rows past a short tile are read, never used).
template <int EPI, bool ASC, bool ONE = false, int RG = 4>
__device__ __forceinline__ void edge16_tile(const EdgeArgs& g, long vb, long nvb, long bid_in = -1, int tid_in = -1) {
  static_assert(RG == 4 || (RG == 3 && EPI == EPI_SEGMEAN && !ONE), "short row tiles: edge layer 2's own launch");
  constexpr int RW = 16 * RG;  // rows per wave row (wm)
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // (tid_in >= 0: the persistent kernel's opaque copy of threadIdx.x, so its loop does not hoist the
  // tile's index math out of the loop and keep it in registers)
  const int tid = tid_in >= 0 ? tid_in : (int)threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int ntn = g.N / BN;
  const long bid = bid_in >= 0 ? bid_in : remap(vb, nvb);
  const int n0 = (int)(bid % ntn) * BN;
  long row0, nrows;
  int seg_c = 0;
  int2 seg = {0, 0};
  long rtile = 0;  // row-tile mode: the tile index
  if (EPI == EPI_SEGMEAN) {
    const long rest = bid / ntn;
    seg_c = (int)(rest % g.npairs);
    if (g.rtiles) {  // edge rows [256 t, 256 t + 256) of conditioning seg_c, nodes cut at the tile ends
      // (a mixed tiling's launch: its tiles from rt_first on, rt_h rows each from row rt_e0)
      const long tl = rest / g.npairs;
      const long th = g.rt_h ? g.rt_h : BM;
      rtile = g.rt_first + tl;
      const long e0 = g.rt_e0 + tl * th;
      row0 = (long)seg_c * g.E + e0;
      nrows = g.E - e0 < th ? g.E - e0 : th;
    } else {
      seg = g.tiles[rest / g.npairs];
      const long es0 = g.node_estart[seg.x];
      const long es1 = (seg.y < g.nnodes) ? g.node_estart[seg.y] : g.E;
      row0 = (long)seg_c * g.E + es0;
      nrows = es1 - es0;
    }
  } else {
    row0 = g.row_base + (bid / ntn) * BM;
    nrows = g.M - row0 < BM ? g.M - row0 : BM;
  }
  const int K = g.K, nk = K / BK;
  const unsigned long long t0 = g.trace ? rtime() : 0;  // (profiling: CHM_EDGE_TRACE block timelines)
  // (dbg 4096 with a trace: slots 4 / 5 = the shader clock counter at the block's start / end instead of the epilogue
  // markers, for the block's mean clock: tools/trace_summary.py --clock)
  const unsigned long long c0 = g.trace && (g.dbg & 4096) ? ctime() : 0;
  unsigned long long tmain = 0;
  auto stamp = [&](int slot) __attribute__((always_inline)) {
    if (g.trace && tid == 0 && !(g.dbg & 4096)) g.trace[6 * vb + slot] = rtime();
  };
  auto stamp_end = [&]() __attribute__((always_inline)) {
    if (g.trace && tid == 0) {
      unsigned long long* o = g.trace + 6 * vb;
      o[0] = hwid(); o[1] = t0; o[2] = tmain; o[3] = rtime();
      if (g.dbg & 4096) { o[4] = c0; o[5] = ctime(); }
    }
  };

  // ---- glds sources: wave w stages rows 32w..32w+31 of both operands, 8 rows per
  // instruction; lane -> row 32w + 8q + (lane >> 3), LDS chunk lane & 7 holding line chunk
  // (lane & 7) ^ swz(row), swz(row) = (row >> 1) & 7. A rows past nrows are read unclamped (F and S
  // carry 256 rows of padding; those rows' results are never stored).
  const char* Ab = reinterpret_cast<const char*>(g.A);
  const char* Wb = reinterpret_cast<const char*>(g.W);
  const long rowB = (long)K * 4;
  // (dbg 32768 / 65536, profiling: layer-1 / layer-2 tiles read their A rows from the first 16 row tiles,
  // which stay L2-resident: the launch time without the A operand's HBM misses)
  const bool a_l2 = (EPI == EPI_EDGE && (g.dbg & 32768)) || (EPI == EPI_SEGMEAN && (g.dbg & 65536));
  const char* Ablk = Ab + (a_l2 ? row0 % (16 * BM) : row0) * rowB;
  const char* Wblk = Wb + (long)n0 * rowB;
  const int lr0 = wave * 32 + (lane >> 3);
  const unsigned lc16 = 16u * (unsigned)((lane & 7) ^ ((lr0 >> 1) & 7));
  const unsigned lc16x = lc16 ^ 64u;
  const unsigned woff = (unsigned)(lr0 * rowB) + lc16;
  const unsigned wq = (unsigned)(8 * rowB);
  char* dst = lds + wave * 32 * ROW_B;
  auto issueA = [&](int t) __attribute__((always_inline)) {
    const char* src = Ablk + (long)(t < nk ? t : nk - 1) * ROW_B;
    char* d = dst + (t % NSA) * OPND_B;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (woff + q * wq + ((q & 1) ? (lc16x - lc16) : 0u))),
                                       (lds_void*)(d + q * 8 * ROW_B), 16, 0, 0);
  };
  auto issueW = [&](int t) __attribute__((always_inline)) {
    const char* src = Wblk + (long)(t < nk ? t : nk - 1) * ROW_B;
    char* d = dst + W_RING + (t % NSW) * OPND_B;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (woff + q * wq + ((q & 1) ? (lc16x - lc16) : 0u))),
                                       (lds_void*)(d + q * 8 * ROW_B), 16, 0, 0);
  };

  if (EPI == EPI_EDGE && g.zero_flags && vb == 0 && tid < g.nzero) g.zero_flags[tid] = 0u;  // (for the next grid)
  if (EPI == EPI_EDGE && g.flags && (g.dbg & 8192))  // (tests: the segment tiles' waits time out)
    for (int k = 0; k < 2500; ++k) __builtin_amdgcn_s_sleep(127);
  if (EPI == EPI_SEGMEAN && g.flags) {
    // k_edge16_tail: a segment tile whose edge rows reach into [flag_row0, E) waits until the layer-1
    // tiles of this grid that write those rows (dispatched first, never waiting themselves) have
    // published them, then acquires at agent scope before any load of S or its exponents. The spin
    // is bounded (~0.3 s), so a broken invariant can never hang the device.
    // A wait that times out raises *g.xbad (and counts EV_TAIL_TIMEOUT): this tile then goes on with S
    // that may not be written, and the repair launches behind the grid recompute edge layer 2.
    const long e0 = row0 - (long)seg_c * g.E, e1 = e0 + nrows;
    if (e1 > g.flag_row0) {
      if (tid == 0) {
        const long lo = (e0 > g.flag_row0 ? e0 : g.flag_row0) - g.flag_row0, hi = e1 - 1 - g.flag_row0;
        const unsigned need = (unsigned)(g.N / BN);
        const unsigned limit = (g.dbg & 8192) ? (1u << 10) : (1u << 21);
        bool late = false;
        for (long r = lo / BM; r <= hi / BM; ++r) {
          unsigned spins = 0;
          while (__hip_atomic_load(g.flags + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need && spins < limit) {
            ++spins;
            __builtin_amdgcn_s_sleep(4);
          }
          late |= spins >= limit;
        }
        if (late && g.xbad) {
          __hip_atomic_store(g.xbad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          count_event(EV_TAIL_TIMEOUT);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      __syncthreads();
    }
  }

  if constexpr (ONE && EPI == EPI_SEGMEAN) {
    // k_edge16_layer: wait (bounded) until both layer-1 column tiles of these rows have stored S and
    // its exponents (flag word: count in bits 0-7, each layer-1 tile's XCD + 1 in bits 8 + 4 n0), check
    // that they ran on this XCD, then count this tile as a consumer (the last of the 2 P resets it)
    if (tid == 0) {
      unsigned* f = g.lflags + rtile;
      const unsigned need = (unsigned)(g.N / BN);
      unsigned spins = 0, v;
      while (((v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & 0xffu) < need &&
             ++spins < (1u << 21))
        __builtin_amdgcn_s_sleep(4);
      const unsigned me = xcc_id() + 1u;
      const bool timeout = (v & 0xffu) < need, other = ((v >> 8) & 15u) != me || ((v >> 12) & 15u) != me;
      if (timeout || other || (g.dbg & 512))
        __hip_atomic_store(g.xbad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (timeout) count_event(EV_LAYER_TIMEOUT);
      else if (other) count_event(EV_LAYER_XCD);
      const unsigned last = need + 2u * (unsigned)g.npairs - 1u;
      if ((__hip_atomic_fetch_add(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffu) == last)
        __hip_atomic_store(f, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    stamp(4);  // (traces of this grid: slot 4 = the wait for the layer-1 tiles is over)
  }

  // ---- row exponents of the A chunks (edge layer 2): the lane's RG rows
  int ex[RG];
#pragma unroll
  for (int i = 0; i < RG; ++i) ex[i] = 0;
  if (ASC) {
#pragma unroll
    for (int i = 0; i < RG; ++i) {
      const long lr = wm * RW + 16 * i + l16;
      const int* pe = g.aexp + row0 + (lr < nrows ? lr : nrows - 1);
      ex[i] = *pe;
    }
  }

  f32x4 acc[RG][8];
#pragma unroll
  for (int i = 0; i < RG; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment of row r (16-row group base + l16), k-chunk g4 of plane p: logical chunk 4p + g4 at
  // physical chunk (4p + g4) ^ swz(r); swz depends on l16 only (group bases are multiples of 16)
  const int swz = (l16 >> 1) & 7;
  const int ch0 = 16 * (g4 ^ swz), ch1 = 16 * ((4 + g4) ^ swz);
  const int fa = (wm * RW + l16) * ROW_B, fw = (wn * 128 + l16) * ROW_B;
  f16x8 fA[2][2][RG];  // [set][plane][row group]
  f16x8 fW[2][2][2];  // [set][plane][column group of the quarter]
  auto read_A = [&](int set, int t) __attribute__((always_inline)) {
    const char* SA = lds + (t % NSA) * OPND_B + fa;
#pragma unroll
    for (int i = 0; i < RG; ++i) {
      fA[set][0][i] = *reinterpret_cast<const f16x8*>(SA + i * 16 * ROW_B + ch0);
      fA[set][1][i] = *reinterpret_cast<const f16x8*>(SA + i * 16 * ROW_B + ch1);
    }
  };
  auto read_W = [&](int set, int t, int qq) __attribute__((always_inline)) {
    const char* SW = lds + W_RING + (t % NSW) * OPND_B + fw + qq * 32 * ROW_B;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      fW[set][0][jj] = *reinterpret_cast<const f16x8*>(SW + jj * 16 * ROW_B + ch0);
      fW[set][1][jj] = *reinterpret_cast<const f16x8*>(SW + jj * 16 * ROW_B + ch1);
    }
  };
  // one quarter: columns 32qq .. 32qq+31 of the wave, all RG row groups, three products
  // (small terms first: w_lo a_hi, w_hi a_lo, then w_hi a_hi)
  auto mfq = [&](int aset, int wset, int qq) __attribute__((always_inline)) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int i = 0; i < RG; ++i) acc[i][2 * qq + jj] = mfma16(fW[wset][1][jj], fA[aset][0][i], acc[i][2 * qq + jj]);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int i = 0; i < RG; ++i) acc[i][2 * qq + jj] = mfma16(fW[wset][0][jj], fA[aset][1][i], acc[i][2 * qq + jj]);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int i = 0; i < RG; ++i) acc[i][2 * qq + jj] = mfma16(fW[wset][0][jj], fA[aset][0][i], acc[i][2 * qq + jj]);
  };
  auto rescale = [&](int t) __attribute__((always_inline)) {
    if (ASC && t > 0 && (t * BK) % CHUNK == 0) {
      const int c = (t * BK) / CHUNK;
#pragma unroll
      for (int i = 0; i < RG; ++i) {
        const int ep = (int)(signed char)(ex[i] >> (8 * (c - 1)));
        const int en = (int)(signed char)(ex[i] >> (8 * c));
        const float f = ldexpf(1.0f, ep - en);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] *= f;
      }
    }
  };
  // quarter with n fragment reads spread between its 6 RG MFMAs (one per two MFMAs)
  auto sched_reads = [&](auto NR) __attribute__((always_inline)) {
    constexpr int nr = decltype(NR)::value;
#pragma unroll
    for (int k = 0; k < nr; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 6 * RG - 2 * nr, 0);
  };

  // prologue (issue order W0 A0 A1 W1 A2): tile 0 landed when 12 glds remain
  issueW(0);
  issueA(0);
  issueA(1);
  issueW(1);
  issueA(2);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_A(0, 0);
  read_W(0, 0, 0);

  // EPI_EDGE: the epilogue's P / Q rows are staged during the last K-tiles (their latency then hides
  // under those MFMAs) when the ring layout allows it (nk % 6 == 0: tiles nk-3, nk-2 sit in A stages
  // 0, 1 and tile nk-1 in A stage 2 / W stage 1) and the rows fit (nR <= PRE_MAX): conditioning 0 at
  // row 0 (A stages 0-1, free after the barrier of tile nk-2), conditioning 1 at row PRE_ROW1 (free
  // after the barrier of tile nk-1).
  bool pre = false;
  int p_ilo = 0, p_jlo = 0, p_nP = 0, p_nR = 0;
  if constexpr (EPI == EPI_EDGE) {
    if (nk % 6 == 0 && !(g.dbg & 2048)) {
      const long rl = row0 + nrows - 1;
      // (block-uniform: kept in SGPRs, they stay live across the main loop)
      p_ilo = __builtin_amdgcn_readfirstlane(g.ei[row0]);
      const int ihi = __builtin_amdgcn_readfirstlane(g.ei[rl]);
      const int ghi = __builtin_amdgcn_readfirstlane(g.n2g[ihi]);
      p_jlo = __builtin_amdgcn_readfirstlane(g.node_off[__builtin_amdgcn_readfirstlane(g.n2g[p_ilo])]);
      p_nP = ihi - p_ilo + 1;
      p_nR = p_nP + __builtin_amdgcn_readfirstlane(g.node_off[ghi] + g.natoms[ghi]) - p_jlo;
      pre = p_nR <= PRE_MAX;
    }
  }
  auto stage_rows = [&](int c, int rbase) __attribute__((always_inline)) {
    const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
    for (int r = wave; r < p_nR; r += 8) {
      const float* src = Pc + (r < p_nP ? (long)(p_ilo + r) * (2 * H) : (long)(p_jlo + r - p_nP) * (2 * H) + H) + n0 +
                         4 * lane;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds + (rbase + r) * PQ_PITCH * 4), 16, 0, 0);
    }
  };

  // tile t: A fragments in set a = t & 1, W quarter fragments alternating sets 0, 1, 0, 1.
  // Pre-staging blocks (EPI_EDGE) skip the loads past the end of K and stage conditioning 0's P / Q
  // rows after the barrier of tile nk-2, conditioning 1's after that of nk-1 (block-uniform
  // branches; the loop keeps its shape, which keeps the register allocation spill-free).
  auto tile = [&](int t, auto CUR) __attribute__((always_inline)) {
    constexpr int a = decltype(CUR)::value;
    rescale(t);
    if (!kAblLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): A_t and W_t quarter 0 are in
    __builtin_amdgcn_s_setprio(1);
    read_W(1, t, 1);
    mfq(a, 0, 0);
    sched_reads(std::integral_constant<int, 4>{});
    __builtin_amdgcn_s_setprio(0);
    if (!kAblLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_setprio(1);
    read_W(0, t, 2);
    mfq(a, 1, 1);
    sched_reads(std::integral_constant<int, 4>{});
    __builtin_amdgcn_s_setprio(0);
    if (!kAblLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_setprio(1);
    read_W(1, t, 3);
    mfq(a, 0, 2);
    sched_reads(std::integral_constant<int, 4>{});
    __builtin_amdgcn_s_setprio(0);
    // this wave is done reading tile t; this thread's part of tile t+1 has landed (only A(t+2) may
    // still be in flight; near the end everything is waited for); after the barrier everyone's
    // has, and tile t's stages are free
    if (!kAblLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);
    constexpr bool uni = kLoopUni && EPI != EPI_EDGE;
    if (!kAblVm) {
      if (uni || t < nk - 2)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (!kAblBar) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    if ((uni || t + 2 < nk) && !kAblLd) issueW(t + 2);  // (uni: past the end of K, a re-read of the last tile)
    if ((uni || t + 3 < nk) && !kAblLd) issueA(t + 3);
    if (EPI == EPI_EDGE && pre) {
      if (t == nk - 2) stage_rows(0, 0);
      if (t == nk - 1 && g.npairs > 1) stage_rows(1, PRE_ROW1);
    }
    read_A(a ^ 1, t + 1);  // past the end: reads stale stages (never used)
    read_W(0, t + 1, 0);
    mfq(a, 1, 3);
    // 6 RG MFMAs: 8 beside the operand loads, 2 RG + 4 beside the fragment reads, the rest (RG = 4: 4) alone
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
    }
#pragma unroll
    for (int k = 0; k < 2 * RG + 4; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
    }
    if constexpr (4 * RG > 12) __builtin_amdgcn_sched_group_barrier(0x008, 4 * RG - 12, 1);
    __builtin_amdgcn_s_setprio(0);
  };
  for (int t = 0; t < nk; t += 2) {  // nk = K / 32 is even (K = 512, 768)
    tile(t, std::integral_constant<int, 0>{});
    tile(t + 1, std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (staged P / Q rows) land before the LDS is reused
  __syncthreads();
  if (g.trace) tmain = rtime();

  // row scale of the last A chunk (edge layer 2)
  float rs[RG];
#pragma unroll
  for (int i = 0; i < RG; ++i) rs[i] = 1.0f;
  if (ASC) {
#pragma unroll
    for (int i = 0; i < RG; ++i) rs[i] = ldexpf(1.0f, (int)(signed char)(ex[i] >> (8 * (K / CHUNK - 1))));
  }
  const int cw = n0 + wn * 128 + 4 * g4;  // this lane's first output column (+ 16 j)

  if constexpr (EPI == EPI_STD) {
    if (!g.C) return;  // (microbenchmark: main loop only)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 sc = *reinterpret_cast<const f32x4*>(g.wscale + cw + 16 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long lr = wm * 64 + 16 * i + l16;
        if (lr < nrows) *reinterpret_cast<f32x4*>(g.C + (row0 + lr) * g.ldc + cw + 16 * j) = acc[i][j] * sc * rs[i];
      }
    }
    return;
  }

  if ((EPI == EPI_EDGE || EPI == EPI_SEGMEAN) && (g.dbg & 16)) {  // (profiling: main loop only)
#pragma unroll
    for (int i = 0; i < RG; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }

  if constexpr (EPI == EPI_EDGE) {
    // S[c][e] = SiLU(D f + P_c[i] + Q_c[j]) as scaled hi/lo fp16 split rows (the P / Q rows of the
    // tile's <= 8 source atoms and 1-2 crystals staged in LDS).
    const int PQ_ROWS = LDS_B / (PQ_PITCH * 4);
    // the tile's source-node range [ilo, ilo + nP) and target rows [jlo, jlo + nR - nP): pre-staging
    // blocks took them before the main loop (SGPRs); the others load them here (a chain of four
    // dependent loads, ~1 us each under load, that would otherwise open every pre-staged epilogue)
    int ilo, jlo, nP, nR;
    if (pre) {
      ilo = p_ilo;
      jlo = p_jlo;
      nP = p_nP;
      nR = p_nR;
    } else {
      const long rl = row0 + nrows - 1;
      ilo = g.ei[row0];
      const int ihi = g.ei[rl];
      const int glo = g.n2g[ilo], ghi = g.n2g[ihi];
      jlo = g.node_off[glo];
      nP = ihi - ilo + 1;
      nR = nP + g.node_off[ghi] + g.natoms[ghi] - jlo;
    }
    const bool staged = pre || nR <= PQ_ROWS;
    const bool both = pre || (staged && g.npairs * nR <= PQ_ROWS);
    const float* T = reinterpret_cast<const float*>(lds + PQ_OFF);
    long rowv[4];
    int pr[4], qr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long lr = wm * 64 + 16 * i + l16;
      rowv[i] = row0 + (lr < nrows ? lr : nrows - 1);
      pr[i] = g.ei[rowv[i]];
      qr[i] = g.ej[rowv[i]];
      if (staged) {
        pr[i] -= ilo;
        qr[i] = nP + qr[i] - jlo;
      }
    }
    // undo the W row scales (after the row-index loads above are issued: their latency runs under these)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 sc = *reinterpret_cast<const f32x4*>(g.wscale + cw + 16 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] *= sc;
    }
    auto stage = [&](int c0, int c1) __attribute__((always_inline)) {  // conditionings [c0, c1), each at rows [rb, rb + nR)
      if (pre) return;                 // (staged by the main loop's last tiles)
      if (c0 > 0) __syncthreads();     // everyone is done reading the previous conditioning
      for (int c = c0; c < c1; ++c) {
        const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
        const int rb = both ? c * nR : 0;
        for (int r = wave; r < nR; r += 8) {
          const float* src = Pc + (r < nP ? (long)(ilo + r) * (2 * H) : (long)(jlo + r - nP) * (2 * H) + H) + n0 + 4 * lane;
          __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds + PQ_OFF + (rb + r) * PQ_PITCH * 4), 16, 0,
                                           0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    };
    _Float16* S0 = reinterpret_cast<_Float16*>(g.S);
    const bool nostore = g.dbg & 4;  // (profiling)
    auto run = [&](int c, auto LAST, auto STG) __attribute__((always_inline)) {
      constexpr bool last = decltype(LAST)::value, stg = decltype(STG)::value;
      const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
      const int rb = pre ? c * PRE_ROW1 : (both ? c * nR : 0);
      static_for<0, 4>([&](auto IC) __attribute__((always_inline)) {
        constexpr int i = decltype(IC)::value;
        const long lr = wm * 64 + 16 * i + l16;  // rows past nrows compute clamped copies, never stored
        const float* prow;
        const float* qrow;
        if constexpr (stg) {
          prow = T + (rb + pr[i]) * PQ_PITCH + wn * 128 + 4 * g4;
          qrow = T + (rb + qr[i]) * PQ_PITCH + wn * 128 + 4 * g4;
        } else {
          prow = Pc + (long)pr[i] * (2 * H) + cw;
          qrow = Pc + (long)qr[i] * (2 * H) + H + cw;
        }
        f32x4 v[8];  // SiLU values (the last conditioning's overwrite acc, which is no longer needed)
        float mx = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const f32x4 p = *reinterpret_cast<const f32x4*>(prow + 16 * j);
          const f32x4 q = *reinterpret_cast<const f32x4*>(qrow + 16 * j);
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2e a2 = {acc[i][j][e], acc[i][j][e + 1]};
            const f32x2e x = silu_e2((a2 + f32x2e{p[e], p[e + 1]}) + f32x2e{q[e], q[e + 1]});
            mx = fmaxf(mx, fmaxf(fabsf(x.x), fabsf(x.y)));
            v[j][e] = x.x;
            v[j][e + 1] = x.y;
          }
        }
        // the row's 128 columns of this wave sit in the 4 lanes l16 + 16 g
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const int ex2 = exp_of(mx);
        const float sc = ldexpf(1.0f, -ex2);
        const long orow = (long)c * g.E + rowv[i];
        // Whole-line stores: a row's 32-column chunk is one 128-B line [hi 32 | lo 32], held by the
        // row's four lanes (16 B of hi and 16 B of lo each). Lanes l16 and l16 ^ 1 (rows 2p, 2p+1)
        // swap a piece (DPP), so that one store writes row 2p's whole line (even lanes its hi half,
        // odd lanes its lo half) and the next row 2p+1's: 8 full lines per instruction instead of
        // 16 half lines (the per-CU store path, not HBM, bounds this epilogue).
        const bool odd = l16 & 1;
        const long lre = lr & ~1L, lro = lr | 1L;  // the pair's rows (tile-relative)
        const long orow_e = (long)c * g.E + row0 + lre, orow_o = orow_e + 1;
        const int off = ((n0 + wn * 128) / 32) * 64 + 8 * g4 + (odd ? 32 : 0);
        _Float16* se = S0 + orow_e * (2 * H) + off;
        _Float16* so = S0 + orow_o * (2 * H) + off;
        const bool st_e = lre < nrows && !nostore, st_o = lro < nrows && !nostore;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {  // 32-column chunks: column groups 2cc, 2cc + 1
          f16x8 hv, lv;
#pragma unroll
          for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float x = v[2 * cc + a2][r] * sc;
              const _Float16 hx = (_Float16)x;
              hv[4 * a2 + r] = hx;
              lv[4 * a2 + r] = (_Float16)(x - (float)hx);
            }
          // even lanes pass their lo piece to the odd partner, odd lanes their hi piece to the even
          typedef int i32x4 __attribute__((ext_vector_type(4)));
          const i32x4 snd = __builtin_bit_cast(i32x4, odd ? hv : lv);
          i32x4 rcv;
#pragma unroll
          for (int w = 0; w < 4; ++w) rcv[w] = __builtin_amdgcn_mov_dpp(snd[w], 0xB1, 0xF, 0xF, false);  // lane ^ 1
          const f16x8 r8 = __builtin_bit_cast(f16x8, rcv);
          if (st_e) *reinterpret_cast<f16x8*>(se + cc * 64) = odd ? r8 : hv;  // row 2p: hi (even), lo (odd)
          if (st_o) *reinterpret_cast<f16x8*>(so + cc * 64) = odd ? lv : r8;  // row 2p+1
        }
        if (lr < nrows && !nostore && g4 == 0) {
          signed char* pe = reinterpret_cast<signed char*>(g.sexp) + orow * 4 + (n0 + wn * 128) / CHUNK;
          *pe = (signed char)ex2;
        }
      });
    };
    using F = std::integral_constant<bool, false>;
    using Tr = std::integral_constant<bool, true>;
    auto all = [&](auto STG) __attribute__((always_inline)) {
      constexpr bool stg = decltype(STG)::value;
      if (g.npairs > 1) {
        if (stg) stage(0, both ? 2 : 1);
        run(0, F{}, STG);
        stamp(4);
        if (stg && !both) stage(1, 2);
        run(1, Tr{}, STG);
      } else {
        if (stg) stage(0, 1);
        run(0, Tr{}, STG);
      }
    };
    if (staged)
      all(Tr{});
    else
      all(F{});
    if constexpr (ONE) {
      // k_edge16_layer: every store of this tile has reached the XCD's L2; count the column tile and
      // record this XCD for the layer-2 tiles' check
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_fetch_add(g.lflags + (row0 / BM), 1u + ((xcc_id() + 1u) << (8 + 4 * (n0 / BN))), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (g.flags) {
      // k_edge16_tail: publish this tile (S rows + exponents) to the segment tiles of the same grid
      // that read it: every wave's stores have reached L2, one agent-scope release writes the XCD's
      // L2 back, then the tile's counter is bumped (one per column tile)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(g.flags + (row0 - g.flag_row0) / BM, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    stamp_end();
    return;
  }

  if constexpr (EPI == EPI_SEGMEAN) {
    // agg[c][node] = mean over the node's edges of SiLU(acc * wscale * rowscale + b2): the wn-th half
    // of the waves writes its 128 columns to an LDS tile [256][132], then every thread sums node
    // segments of one column in edge order (scatter_add's order).
    float* T = reinterpret_cast<float*>(lds);
    // node list: {node, rows in this tile | first row in the tile << 10 | kind << 20}; kind 0 = a whole
    // node, 1 = the head part of a node cut at the tile end (row tiles: listed first), 2 = the rest of a
    // node begun in the previous tile (listed last)
    int2* info = reinterpret_cast<int2*>(lds + SEG_B);
    int nn;
    int2 my = {0, 0};
    if (kSegTable && g.rinfo) {
      // the host-built list: two independent loads, consumed only after the bias + SiLU pass below
      nn = g.rinfo_n[rtile];
      if (tid < kRowInfo) my = g.rinfo[rtile * kRowInfo + tid];
    } else if (g.rtiles) {
      const int4 rt = g.rtiles[rtile];
      const long e0 = rtile * BM, e1 = e0 + nrows;
      const int nreg = rt.y - rt.x;
      const bool head = nreg > 0 && g.node_estart[rt.y - 1] + g.node_n[rt.y - 1] > e1;
      const bool cont = rt.z >= 0;
      nn = nreg + (cont ? 1 : 0);
      if (tid < nn) {
        if (cont && tid == nn - 1) {
          my.x = rt.z;
          my.y = (int)(g.node_estart[rt.z] + g.node_n[rt.z] - e0) | (2 << 20);
        } else {
          my.x = rt.x + (head ? (tid == 0 ? nreg - 1 : tid - 1) : tid);
          const long es = g.node_estart[my.x], end = es + g.node_n[my.x];
          my.y = (int)((end > e1 ? e1 : end) - es) | ((int)(es - e0) << 10) | ((head && tid == 0) ? 1 << 20 : 0);
        }
      }
    } else {
      nn = seg.y - seg.x;
      const long es0 = g.node_estart[seg.x];
      if (tid < nn) {
        my.x = seg.x + tid;
        my.y = g.node_n[my.x] | ((int)(g.node_estart[my.x] - es0) << 10);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // scale undo + bias + SiLU per column group; the next group's scale / bias loads are issued
    // ahead of the current group's math (pinned there, else all 16 loads are hoisted and spill)
    f32x4 scv[2], bbv[2];
    scv[0] = *reinterpret_cast<const f32x4*>(g.wscale + cw);
    bbv[0] = *reinterpret_cast<const f32x4*>(g.bias + cw);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < 7) {
        scv[(j + 1) & 1] = *reinterpret_cast<const f32x4*>(g.wscale + cw + 16 * (j + 1));
        bbv[(j + 1) & 1] = *reinterpret_cast<const f32x4*>(g.bias + cw + 16 * (j + 1));
      }
#pragma unroll
      for (int i = 0; i < RG; ++i)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f32x2e a2 = {acc[i][j][e], acc[i][j][e + 1]};
          const f32x2e s2 = f32x2e{scv[j & 1][e], scv[j & 1][e + 1]} * rs[i];
          const f32x2e y = a2 * s2 + f32x2e{bbv[j & 1][e], bbv[j & 1][e + 1]};
          // (dbg 8, profiling, A/B builds only: in r2 removing this uniform select made edge layer 2 ~3% slower
          // under the compiler's schedule, profiles/r2/layer/epilogue_select_ab.txt; in r6 its removal gains)
          const f32x2e x = (kL2Sel && (g.dbg & 8)) ? y : silu_e2(y);
          acc[i][j][e] = x.x;
          acc[i][j][e + 1] = x.y;
        }
#pragma unroll
      for (int i = 0; i < RG; ++i) asm volatile("" : "+v"(acc[i][j])::"memory");
    }
    if (!ONE) stamp(4);
    for (int half = 0; half < 2; ++half) {
      if (half == 1 && !ONE) stamp(5);
      if (wn == half) {
#pragma unroll
        for (int i = 0; i < RG; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            *reinterpret_cast<f32x4*>(T + (wm * RW + 16 * i + l16) * SEG_TP + 16 * j + 4 * g4) = acc[i][j];
      }
      if (half == 0 && tid < nn) info[tid] = my;
      // LDS-only barriers in this loop: a __syncthreads() fence would also wait for the agg stores and
      // the agg_max atomics still in flight (~3000 cycles each under load, twice per tile)
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the tile rows and the node list are in LDS
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // one wave per node, two adjacent columns per lane (8 node slots: a tile's ~6 nodes of 40 edges run
      // side by side instead of two per slot); each column is still one sequential sum over its rows
      const int col = 2 * (tid & 63);
      const int gcol = n0 + half * 128 + col;
      auto finish = [&](int node, f32x2e sacc, int cnt) __attribute__((always_inline)) {
        const float dv = (float)(cnt < 1 ? 1 : cnt);
        f32x2e mean;
        mean.x = sacc.x / dv;
        mean.y = sacc.y / dv;
        if (g.aggs) {
          // pre-split node GEMMs: this wave's 128 columns are one chunk of the node MLP's A operand, written
          // as a split row scaled by 2^-e (e from the chunk's max |agg|) with the chunk's exponent byte
          float m = fmaxf(fabsf(mean.x), fabsf(mean.y));
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
          const int ex = exp_of(m);
          const float sc = ldexpf(1.0f, -ex);
          const float x0 = mean.x * sc, x1 = mean.y * sc;
          typedef _Float16 f16x2s __attribute__((ext_vector_type(2)));
          f16x2s hi, lo;
          hi[0] = (_Float16)x0;
          hi[1] = (_Float16)x1;
          lo[0] = (_Float16)(x0 - (float)hi[0]);
          lo[1] = (_Float16)(x1 - (float)hi[1]);
          const long row = (long)seg_c * g.nnodes + node;
          _Float16* o16 = reinterpret_cast<_Float16*>(g.aggs) + row * (2 * H) + (gcol >> 4) * 32 + (gcol & 15);
          if (!(kPairAbl && (g.dbg & 4))) {
            *reinterpret_cast<f16x2s*>(o16) = hi;
            *reinterpret_cast<f16x2s*>(o16 + 16) = lo;
            if (lane == 0) reinterpret_cast<signed char*>(g.agge)[row * 4 + (gcol >> 7)] = (signed char)ex;
          }
          return;
        }
        if (!(kPairAbl && (g.dbg & 4))) *reinterpret_cast<f32x2e*>(g.agg + ((long)seg_c * g.nnodes + node) * H + gcol) = mean;
        if (g.agg_max) {  // the node row's max |agg| for the split16 node GEMM reading it
          float m = fmaxf(fabsf(mean.x), fabsf(mean.y));
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
          if (lane == 0) atomicMax(g.agg_max + (long)seg_c * g.nnodes + node, __float_as_uint(m));
        }
      };
      // row tiles: one counter per (conditioning, boundary tile, column half)
      const int cidx = (n0 / BN) * 4 + half * 2;
      for (int k = tid >> 6; k < nn && !(kPairAbl && (g.dbg & 32)); k += 8) {  // (dbg 32: profiling, no sums)
        const int2 nk = info[k];
        const int4 ni = {nk.y & 1023, (nk.y >> 10) & 1023, nk.x, nk.y >> 20};  // {rows, first row, node, kind}
        const float* src = T + ni.y * SEG_TP + col;
        f32x2e sacc = {0.f, 0.f};
        bool own = true;  // this wave finishes the node
        if (ni.w == 2) {
          // The rest of a node begun in tile t-1, whose head wave publishes the partial sum of its rows
          // (sbuf) and bumps the counter. Normally that has happened (tile t-1 was dispatched first and
          // handles its head node first): continue the sum from it. Otherwise (bounded wait; tile t-1 may
          // still be queued, e.g. on the previous XCD's share of the grid) leave these rows in msgbuf and
          // bump the counter: whichever of the two arrives second finishes the node.
          unsigned* cnt = g.rcnt + ((long)seg_c * g.ntiles + rtile) * 8 + cidx;
          unsigned v = 0;
          if (!(g.dbg & 64) && lane == 0) {
            unsigned spins = 0;
            while ((v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u && ++spins < 256u)
              __builtin_amdgcn_s_sleep(2);
          }
          if (__builtin_amdgcn_readfirstlane(v) == 0u) {
            float* mb = g.msgbuf + ((long)seg_c * g.r2tot + g.rtiles[rtile].w) * H + gcol;
            for (int r = 0; r < ni.x; ++r) {
              st_agent(mb + (long)r * H, src[r * SEG_TP]);
              st_agent(mb + (long)r * H + 1, src[r * SEG_TP + 1]);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (written through before the count)
            unsigned old = 0;
            if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            own = __builtin_amdgcn_readfirstlane(old) != 0u;
          }
          if (own) {
            asm volatile("" ::: "memory");
            const float* sb = g.sbuf + ((long)seg_c * g.ntiles + rtile) * H + gcol;
            sacc.x = ld_agent(sb);
            sacc.y = ld_agent(sb + 1);
            if (lane == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (next launch)
          }
        }
        if (own) {
          int jj = 0;
          for (; jj + 8 <= ni.x; jj += 8) {
            f32x2e v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x2e*>(src + (jj + u) * SEG_TP);
#pragma unroll
            for (int u = 0; u < 8; ++u) sacc += v[u];
          }
          for (; jj < ni.x; ++jj) sacc += *reinterpret_cast<const f32x2e*>(src + jj * SEG_TP);
        }
        if (ni.w == 0) {
          finish(ni.z, sacc, ni.x);
        } else if (ni.w == 2) {
          if (own) finish(ni.z, sacc, g.node_n[ni.z]);
        } else {
          // head part of a node cut at the tile end: publish the partial sum for tile t+1; if tile t+1
          // has already left its rows in msgbuf, finish the node here
          const long tb = rtile + 1;
          unsigned* cnt = g.rcnt + ((long)seg_c * g.ntiles + tb) * 8 + cidx;
          float* sb = g.sbuf + ((long)seg_c * g.ntiles + tb) * H + gcol;
          st_agent(sb, sacc.x);
          st_agent(sb + 1, sacc.y);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (written through before the count)
          unsigned old = 0;
          if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__builtin_amdgcn_readfirstlane(old) != 0u) {
            asm volatile("" ::: "memory");
            if (lane == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int deg = g.node_n[ni.z];
            const int r2 = deg - ni.x;  // the node's rows in tile t+1
            const float* mb = g.msgbuf + ((long)seg_c * g.r2tot + g.rtiles[tb].w) * H + gcol;
            for (int r = 0; r < r2; ++r) {
              sacc.x += ld_agent(mb + (long)r * H);
              sacc.y += ld_agent(mb + (long)r * H + 1);
            }
            finish(ni.z, sacc, deg);
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // everyone's tile reads are done before the next half is written
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    stamp_end();
  }
}

template <int EPI, bool ASC>
__global__ __launch_bounds__(512, 1) void k_edge16(EdgeArgs g) {
  edge16_tile<EPI, ASC>(g, blockIdx.x, gridDim.x);
}

// Edge layer 2 on 192-row tiles (3 row groups per wave: three quarters of a 256-row tile's MFMAs and epilogue):
// the second launch of a mixed row tiling, whose 256-row tiles fill whole rounds of the CUs and whose short tiles
// take the partial last round (runtime.hip short_row_tiles)
__global__ __launch_bounds__(512, 1) void k_edge16_short(EdgeArgs g) {
  edge16_tile<EPI_SEGMEAN, true, false, 3>(g, blockIdx.x, gridDim.x);
}

// Edge layer 1's partial last round and edge layer 2 in one grid: blocks [0, nb1) are layer-1 tiles
// (g1, rows [g1.row_base, g1.M)), the rest are all of edge layer 2's segment tiles (g2). Workgroups
// are dispatched in index order on every XCD, so the layer-1 tiles start first and the layer-2 tiles
// fill the CUs they leave idle; the few segment tiles that read layer-1 rows of this grid (the last
// ones of the tile order) wait for them through g1.flags / g2.flags (edge16_tile). nb1 is a multiple
// of 8 (blocks past the layer-1 tiles return at once), so the layer-2 part keeps its XCD-aware order.
__global__ __launch_bounds__(512, 1) void k_edge16_tail(EdgeArgs g1, EdgeArgs g2, int nb1, int nt1) {
  if ((int)blockIdx.x < nb1) {
    if ((int)blockIdx.x < nt1) edge16_tile<EPI_EDGE, false>(g1, blockIdx.x, nt1);
  } else {
    edge16_tile<EPI_SEGMEAN, true>(g2, blockIdx.x - nb1, gridDim.x - nb1);
  }
}

// Both edge layers of a CSP layer in one grid (fc batches on row tiles): every XCD (blockIdx % 8) walks
// its own contiguous range of row tiles, layer-1 tiles (2 column tiles) of row tile i interleaved with
// the layer-2 tiles (P conditionings x 2 column tiles) of row tile i - D, so a layer-2 tile normally
// starts after the layer-1 tiles it reads have finished, and the two layers' phases (layer 1's
// epilogue store bursts, layer 2's MFMA-bound main loop) overlap across the CUs instead of every CU
// storing at once. Dependencies only point to earlier blocks of the same XCD's sequence (dispatched
// in index order), and the waits are bounded.
__global__ __launch_bounds__(512, 1) void k_edge16_layer(EdgeArgs g1, EdgeArgs g2, int R, int D) {
  const LayerJob j = layer_job(blockIdx.x, R, g2.npairs, D);
  if (j.kind == 1)
    edge16_tile<EPI_EDGE, false, true>(g1, blockIdx.x, gridDim.x, j.bid);
  else if (j.kind == 2)
    edge16_tile<EPI_SEGMEAN, true, true>(g2, blockIdx.x, gridDim.x, j.bid);
}

// The persistent form of k_edge16_layer (option edge_layer_dyn; the default from kDynMinTiles row tiles
// on): one block per CU, each looping over jobs of its XCD's sequence (an atomic per job on the XCD's
// counter). The sequence has the static map's group structure (layer-1 tiles of local row i interleaved
// with the layer-2 tiles of local row i - D; seq_job). XCD x's first ns local rows are its static rows
// x ns .. (x + 1) ns - 1; the rest of the grid's row tiles, [8 ns, R) (edge_pool percent), form a pool
// its later local rows claim from at run time through one counter shared by all XCDs, so an XCD that
// runs faster claims more of them (with the static map every XCD gets R / 8 rows and the slowest one
// sets the launch time: the XCDs' last blocks ended 240 us apart in a 4.8 ms launch at 512x40,
// profiles/r3/traces). Per layer and launch (zeroed per decoder call): sched[x] the jobs taken on XCD x,
// sched[8] the pool rows claimed, and the slots sched[16 + x * cap + i] of XCD x's pool rows (0 = not
// yet resolved, row + 1, or ~0u = no row). Claims go in local-row order (the claim of row i waits for
// row i-1's), so each XCD's valid rows are a prefix: a block that takes a layer-2 job of an invalid row
// knows every later job of its XCD is invalid and exits; a layer-1 job of an invalid row is skipped.
// Every wait is for a job taken earlier by a running block (deadlock-free whatever the residency), and
// bounded: a timed-out wait raises the layer's repair request.
struct SeqJob { int kind; long row; int sub; };  // kind 1: layer 1 (sub = column tile), 2: layer 2 (sub = cond * 2 + col)
// Job k of an XCD's sequence: the first 2D jobs are the layer-1 tiles of local rows 0 .. D-1, then groups
// i = D, D+1, ... of [layer 1 of row i (2 jobs), layer 2 of row i - D (2P)] (the static map's pattern,
// unbounded). Measured and not kept: the pool rows' layer-1 tiles running ahead twice as fast (so
// that a backlog of layer-2 tiles covers the last row's layer-1 + layer-2 chain at the end): 512x40
// 59.2 -> 60.6 ms per step (profiles/r3/ab/ab_ra64/, ab_ra512/).
__host__ __device__ inline SeqJob seq_job(long k, int P, int D) {
  const long G = 2 + 2L * P;
  if (k < 2L * D) return SeqJob{1, k / 2, (int)(k % 2)};
  const long q = k - 2L * D, i = D + q / G;
  const int sub = (int)(q % G);
  if (sub < 2) return SeqJob{1, i, sub};
  return SeqJob{2, i - D, sub - 2};
}

namespace {
__device__ __forceinline__ unsigned wait_slot(const unsigned* p, bool& late) {
  unsigned v, spins = 0;
  while ((v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u && spins < (1u << 20)) {
    ++spins;
    __builtin_amdgcn_s_sleep(2);
  }
  if (v == 0u) late = true;
  return v;
}
}  // namespace

// (A static row's job costs only the XCD counter's atomic, about what the hardware dispatch of a block
// of the static map costs; claiming every row from the pool measured slower: 512x40 58.15 vs 57.9 ms
// per step at edge_pool 30 vs 15.)
// skip_x >= 0 (tests only, option edge_dyn_skip_xcd): the blocks on XCD skip_x exit at once, as if that
// XCD did not exist, so the self-check below must catch it.
__global__ __launch_bounds__(512, 1) void k_edge16_layer_dyn(EdgeArgs g1, EdgeArgs g2, int R, int D, unsigned* sched,
                                                             int cap, int ns, int skip_x) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const unsigned x = xcc_id();
  const int P = g2.npairs;
  unsigned* slots = sched + 16 + (long)x * cap;  // local row ns + i -> slots[i]
  unsigned long long* done = reinterpret_cast<unsigned long long*>(sched + 10);  // finished layer-2 tiles | exits << 32
  int* bc = reinterpret_cast<int*>(lds);
  for (;;) {
    if (threadIdx.x == 0) {
      const long k = (long)__hip_atomic_fetch_add(sched + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const SeqJob j = seq_job(k, P, D);
      int code = 0;  // 0 = exit, 1 = layer 1, 2 = layer 2, 3 = skip
      unsigned v = 0;  // the row + 1, ~0u = none
      bool late = false;
      const long jd = j.row - ns;  // pool slot of a local row past the static ones
      if ((int)x == skip_x) {
        code = 0;
      } else if (jd >= cap) {
        v = ~0u;  // (beyond every possible row: its layer-2 row is invalid too)
      } else if (jd < 0) {
        v = (unsigned)(x * ns + j.row) + 1u;
      } else if (j.kind == 1 && j.sub == 0) {  // claim, after the previous local row's claim (valid rows: a prefix)
        const unsigned prev = jd > 0 ? wait_slot(slots + jd - 1, late) : 1u;
        v = ~0u;
        if (prev != ~0u && prev != 0u) {
          const unsigned r = (unsigned)(8 * ns) + __hip_atomic_fetch_add(sched + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (r < (unsigned)R) v = r + 1u;
        }
        __hip_atomic_store(slots + jd, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        v = wait_slot(slots + jd, late);
        if (v == 0u) v = ~0u;
      }
      long bid = 0;
      if ((int)x == skip_x) {
      } else if (j.kind == 1) {
        code = v == ~0u ? 3 : 1;
        bid = (long)(v - 1u) * 2 + j.sub;
      } else {
        code = v == ~0u ? 0 : 2;
        bid = ((long)(v - 1u) * P + j.sub / 2) * 2 + (j.sub & 1);
      }
      if (code == 0) {
        // Exit. Self-check: the static rows of an XCD that does not exist (a device or
        // partition mode with fewer than 8 XCDs) would never be computed. Layer-2 tiles add 1 to
        // done[0] as they finish and exiting blocks add 2^32; the last block out sees every finished
        // tile in the same word (one location: its coherence order holds every block's finish before
        // its exit) and raises the repair request if any layer-2 tile is missing.
        const unsigned long long old = __hip_atomic_fetch_add(done, 1ull << 32, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT);
        if ((old >> 32) + 1ull == (unsigned long long)gridDim.x &&
            (old & 0xffffffffull) != (unsigned long long)R * P * 2) {
          __hip_atomic_store(g2.xbad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          count_event(EV_LAYER_INCOMPLETE);
        }
      }
      if (late) {  // (never in a healthy run: the layer is recomputed by the repair launches)
        __hip_atomic_store(g2.xbad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        count_event(EV_LAYER_TIMEOUT);
      }
      bc[0] = code;
      bc[1] = (int)bid;
      bc[2] = (int)(8 * k + x);
    }
    __syncthreads();
    const int code = bc[0], bid = bc[1], vb = bc[2];
    __syncthreads();
    if (code == 0) break;
    if (code == 3) continue;  // (a layer-1 job of a row past the end: no tile)
    // (the tiles read their arguments through laundered kernarg pointers: otherwise the compiler keeps
    // both argument blocks in SGPRs across the loop and spills them)
    typedef const __attribute__((address_space(4))) char* kptr;
    kptr kp = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    constexpr long off2 = (sizeof(EdgeArgs) + alignof(EdgeArgs) - 1) / alignof(EdgeArgs) * alignof(EdgeArgs);
    const EdgeArgs* a1 = (const EdgeArgs*)(const __attribute__((address_space(4))) EdgeArgs*)kp;
    const EdgeArgs* a2 = (const EdgeArgs*)(const __attribute__((address_space(4))) EdgeArgs*)(kp + off2);
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    if (code == 1)
      edge16_tile<EPI_EDGE, false, true>(*a1, vb, 0, bid, tid);
    else
      edge16_tile<EPI_SEGMEAN, true, true>(*a2, vb, 0, bid, tid);
    __syncthreads();
    if (code == 2 && threadIdx.x == 0) __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The XCDs a grid's blocks run on (bit x = XCC_ID x), for the persistent kernel's 8-XCD assumption.
__global__ void k_xcd_probe(unsigned* mask) {
  if (threadIdx.x == 0) atomicOr(mask, 1u << xcc_id());
}

hipError_t xcd_mask(int blocks, unsigned* out) {
  unsigned* d = nullptr;
  hipError_t e = hipMalloc(&d, sizeof(unsigned));
  if (e != hipSuccess) return e;
  e = hipMemset(d, 0, sizeof(unsigned));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_xcd_probe, dim3((unsigned)blocks), dim3(64), 0, 0, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, d, sizeof(unsigned), hipMemcpyDeviceToHost);
  const hipError_t ef = hipFree(d);
  return e != hipSuccess ? e : ef;
}

// Repair of a k_edge16_layer launch whose check failed (*g.xbad != 0: some layer-2 tile read S written
// on another XCD, so its L2 view may have been stale): one layer on the two-launch schedule, grid-
// stride over the tiles so that the normal case (nothing to repair) costs one small grid that exits.
// The layer-1 pass also clears the layer's agg row maxima (the failed launch may have max-ed garbage).
// ev >= 0: count the repair (block 0) as that event.
// (The layer-1 pass also clears the row-tile partial-sum counters rcnt: when a launch ended with tiles
// that never ran, k_edge16_layer_dyn with an XCD missing, a head tile's count has no partner left.)
template <int EPI, bool ASC>
__global__ __launch_bounds__(512, 1) void k_edge16_repair(EdgeArgs g, long nvb, unsigned* agg_max, long nmax,
                                                          unsigned* lflags, long nrt, int ev, unsigned* rcnt = nullptr,
                                                          long nrcnt = 0) {
  if (__hip_atomic_load(g.xbad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  if (ev >= 0 && blockIdx.x == 0 && threadIdx.x == 0) count_event(ev);
  if (EPI == EPI_EDGE) {  // (and the row-tile flags, in case a wait timed out; null pointers come with 0 counts)
    for (long k = (long)blockIdx.x * 512 + threadIdx.x; agg_max && k < nmax; k += (long)gridDim.x * 512) agg_max[k] = 0u;
    for (long k = (long)blockIdx.x * 512 + threadIdx.x; lflags && k < nrt; k += (long)gridDim.x * 512) lflags[k] = 0u;
    for (long k = (long)blockIdx.x * 512 + threadIdx.x; rcnt && k < nrcnt; k += (long)gridDim.x * 512) rcnt[k] = 0u;
  }
  for (long vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
    edge16_tile<EPI, ASC>(g, vb, nvb);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// Edge layer 1 on unordered pairs (option edge_pairs; fc batches). The reference's Fourier features of
// edge (j, i) are those of edge (i, j) with the sine half negated: frac_diff_ji = (x_i - x_j) % 1 is
// 1 - frac_diff_ij (or 0 with it), sin(2 pi k (1 - d)) = -sin(2 pi k d), cos(2 pi k (1 - d)) = cos(2 pi k d)
// (cspnet.py:38-52, 324; exact in real arithmetic; in fp32 the reference's two argument roundings differ
// by up to 8e-5 on the k = 127 features, which moves the decoder outputs by ~2e-6 of their scale). With
// V = D_sin f_sin and U = D_cos f_cos over the pair's features, D f_ij = U + V and D f_ji = U - V: one GEMM
// row of K = 768 per pair (i <= j) instead of two directed rows, half of edge layer 1's matrix work. The K
// loop runs the 12 sine K-tiles into V, then the 12 cosine K-tiles into U; the epilogue writes both
// directions' S rows (S_ij = SiLU(U + V + P_i + Q_j), S_ji = SiLU(U - V + P_j + Q_i)) into the directed
// row layout edge layer 2 reads, exactly as edge16_tile's EPI_EDGE epilogue writes them.
// Tile: 128 pairs x 256 columns, 8 waves of 32 pairs x 128 columns (two accumulator sets of 64 registers:
// the budget of edge16_tile's one set of 128); split rows, swizzle, MFMA and C^T layout as edge16_tile.
namespace {
constexpr int PBM = 128;                 // pairs per tile
constexpr int P_NSA = 3, P_NSW = 2;      // ring depths: A (streamed), W (L2-resident)
constexpr int P_OPA = PBM * ROW_B;       // 16 KB per A stage
constexpr int P_WRING = P_NSA * P_OPA;   // W stages follow the A stages (32 KB each)
static_assert(P_WRING + P_NSW * OPND_B <= LDS_B, "LDS");
static_assert(PBM == kPairRows, "pair tile rows (host tables)");
// the epilogue's staged P / Q rows: per node [P 256 | Q 256 | 8 pad] floats of this column tile (a pitch of 8
// dwords mod 64 banks: the 16 lanes of a ds_read_b128 group, rows of consecutive nodes, hit distinct banks)
constexpr int P_QP = 520;
constexpr int P_QROWS = LDS_B / (P_QP * 4);  // 78 node rows
}  // namespace

// one pair tile: bid = pair tile * 2 + column tile (tid_in: the persistent kernel's opaque copy of threadIdx.x)
__device__ __forceinline__ void pair_tile(const EdgeArgs& g, long bid, int tid_in) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = tid_in, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // rows 32 wm, columns 128 wn of the tile
  const int l16 = lane & 15, g4 = lane >> 4;
  const int n0 = (int)(bid & 1) * BN;
  const long row0 = (bid >> 1) * PBM;
  const long nrows = g.Mp - row0 < PBM ? g.Mp - row0 : PBM;
  constexpr int nk = FD / BK;        // 24: K-tiles [0, 12) sine features, [12, 24) cosine
  constexpr int rowB = FD * 4;       // one split row of K = 768
  // glds: wave w stages A rows 16 w .. 16 w + 15 (2 instructions) and W rows 32 w .. 32 w + 31 (4); lane ->
  // row base + 8 q + (lane >> 3), LDS chunk lane & 7 holding line chunk (lane & 7) ^ ((row >> 1) & 7)
  // (traced A/B builds only, dbg 32768: the pair tiles read their F rows from the first 16 pair tiles, which stay
  // L2-resident: the tile time without F's HBM reads; wrong results)
  const long arow0 = (kGridTrace && (g.dbg & 32768)) ? row0 % (16 * PBM) : row0;
  const char* Ablk = reinterpret_cast<const char*>(g.A) + arow0 * rowB;
  const char* Wblk = reinterpret_cast<const char*>(g.W) + (long)n0 * rowB;
  const int ra0 = wave * 16 + (lane >> 3), rw0 = wave * 32 + (lane >> 3);
  const unsigned aoff = (unsigned)(ra0 * rowB) + 16u * (unsigned)((lane & 7) ^ ((ra0 >> 1) & 7));
  const unsigned woff = (unsigned)(rw0 * rowB) + 16u * (unsigned)((lane & 7) ^ ((rw0 >> 1) & 7));
  const unsigned q8 = (unsigned)(8 * rowB);
  // (row + 8: its swizzle differs in bit 2, i.e. the source chunk moves by 64 bytes; the move is a 32-bit
  // unsigned difference, so it is added to the offset BEFORE the pointer: offset + move never wraps)
  const unsigned aodd = (((unsigned)(lane & 7) ^ (unsigned)((ra0 >> 1) & 7)) ^ 4u) * 16u - 16u * (unsigned)((lane & 7) ^ ((ra0 >> 1) & 7));
  const unsigned wodd = (((unsigned)(lane & 7) ^ (unsigned)((rw0 >> 1) & 7)) ^ 4u) * 16u - 16u * (unsigned)((lane & 7) ^ ((rw0 >> 1) & 7));
  char* dstA = lds + wave * 16 * ROW_B;
  char* dstW = lds + P_WRING + wave * 32 * ROW_B;
  auto issueA = [&](int t) __attribute__((always_inline)) {
    const char* src = Ablk + (long)(t < nk ? t : nk - 1) * ROW_B;
    char* d = dstA + (t % P_NSA) * P_OPA;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (aoff + q * q8 + (q & 1 ? aodd : 0u))), (lds_void*)(d + q * 8 * ROW_B),
                                       16, 0, 0);
  };
  auto issueW = [&](int t) __attribute__((always_inline)) {
    const char* src = Wblk + (long)(t < nk ? t : nk - 1) * ROW_B;
    char* d = dstW + (t % P_NSW) * OPND_B;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (woff + q * q8 + (q & 1 ? wodd : 0u))), (lds_void*)(d + q * 8 * ROW_B),
                                       16, 0, 0);
  };

  f32x4 accV[2][8], accU[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) accV[i][j] = accU[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int swz = (l16 >> 1) & 7;
  const int ch0 = 16 * (g4 ^ swz), ch1 = 16 * ((4 + g4) ^ swz);
  const int fa = (wm * 32 + l16) * ROW_B, fw = (wn * 128 + l16) * ROW_B;
  f16x8 fA[2][2][2];  // [set][plane][row group]
  f16x8 fW[2][2][2];  // [set][plane][column group of the quarter]
  auto read_A = [&](int set, int t) __attribute__((always_inline)) {
    const char* SA = lds + (t % P_NSA) * P_OPA + fa;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      fA[set][0][i] = *reinterpret_cast<const f16x8*>(SA + i * 16 * ROW_B + ch0);
      fA[set][1][i] = *reinterpret_cast<const f16x8*>(SA + i * 16 * ROW_B + ch1);
    }
  };
  auto read_W = [&](int set, int t, int qq) __attribute__((always_inline)) {
    const char* SW = lds + P_WRING + (t % P_NSW) * OPND_B + fw + qq * 32 * ROW_B;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      fW[set][0][jj] = *reinterpret_cast<const f16x8*>(SW + jj * 16 * ROW_B + ch0);
      fW[set][1][jj] = *reinterpret_cast<const f16x8*>(SW + jj * 16 * ROW_B + ch1);
    }
  };
  // one quarter (32 columns of the wave, both row groups, three products: small terms first)
  auto mfq = [&](f32x4 (&acc)[2][8], int aset, int wset, int qq) __attribute__((always_inline)) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i][2 * qq + jj] = mfma16(fW[wset][1][jj], fA[aset][0][i], acc[i][2 * qq + jj]);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i][2 * qq + jj] = mfma16(fW[wset][0][jj], fA[aset][1][i], acc[i][2 * qq + jj]);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i][2 * qq + jj] = mfma16(fW[wset][0][jj], fA[aset][0][i], acc[i][2 * qq + jj]);
  };
  auto sched_reads = [&](auto NR) __attribute__((always_inline)) {  // NR fragment reads among 12 MFMAs
    constexpr int nr = decltype(NR)::value;
#pragma unroll
    for (int k = 0; k < nr; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 12 - 2 * nr, 0);
  };

  // the node range of the epilogue's P / Q rows (one load, issued ahead of the operand stream: in by tile 0)
  int2 pqn = {0, 0};
  if (g.pnode) pqn = g.pnode[row0 / PBM];
  // prologue (issue order W0 A0 A1 W1 A2): tile 0 has landed when 8 glds remain (A1 2, W1 4, A2 2)
  issueW(0);
  issueA(0);
  issueA(1);
  issueW(1);
  issueA(2);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // (block-uniform: SGPRs across the main loop)
  const int q_lo = __builtin_amdgcn_readfirstlane(pqn.x), q_n = __builtin_amdgcn_readfirstlane(pqn.y);
  read_A(0, 0);
  read_W(0, 0, 0);

  auto tile = [&](f32x4 (&acc)[2][8], int t, auto CUR) __attribute__((always_inline)) {
    constexpr int a = decltype(CUR)::value;
    if (!kAblLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): A_t and W_t quarter 0 are in
    __builtin_amdgcn_s_setprio(1);
    read_W(1, t, 1);
    mfq(acc, a, 0, 0);
    sched_reads(std::integral_constant<int, 4>{});
    __builtin_amdgcn_s_setprio(0);
    if (!kAblLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_setprio(1);
    read_W(0, t, 2);
    mfq(acc, a, 1, 1);
    sched_reads(std::integral_constant<int, 4>{});
    __builtin_amdgcn_s_setprio(0);
    if (!kAblLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_setprio(1);
    read_W(1, t, 3);
    mfq(acc, a, 0, 2);
    sched_reads(std::integral_constant<int, 4>{});
    __builtin_amdgcn_s_setprio(0);
    // this wave is done reading tile t; this thread's part of tile t+1 has landed (only A(t+2) may still
    // be in flight: 2 glds; near the end everything is waited for); after the barrier everyone's has
    if (!kAblLgkm) __builtin_amdgcn_s_waitcnt(0xC07F);
    if (!kAblVm) {
      if (kLoopUni || t < nk - 2)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (!kAblBar) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    if ((kLoopUni || t + 2 < nk) && !kAblLd) issueW(t + 2);
    if ((kLoopUni || t + 3 < nk) && !kAblLd) issueA(t + 3);
    read_A(a ^ 1, t + 1);  // past the end: reads stale stages (never used)
    read_W(0, t + 1, 0);
    mfq(acc, a, 1, 3);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
    __builtin_amdgcn_s_setprio(0);
  };
  for (int t = 0; t < nk / 2; t += 2) {  // the sine half of K into V
    tile(accV, t, std::integral_constant<int, 0>{});
    tile(accV, t + 1, std::integral_constant<int, 1>{});
  }
  for (int t = nk / 2; t < nk; t += 2) {  // the cosine half into U
    tile(accU, t, std::integral_constant<int, 0>{});
    tile(accU, t + 1, std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (g.dbg & 16) {  // (profiling: main loop only)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(accU[i][j]), "v"(accV[i][j]));
    return;
  }

  // ---- epilogue: undo the W row scales, then per conditioning and direction S = SiLU(U +- V + P + Q)
  // The P / Q rows of the tile's nodes [q_lo, q_lo + q_n) are staged in LDS (global_load_lds, one latency for all
  // of them instead of one per conditioning, direction and row group): both conditionings when they fit, else
  // conditioning 0's; more nodes than P_QROWS (crystals of 78+ atoms): all read from global memory.
  const bool stg = g.pnode && q_n <= P_QROWS && !(g.dbg & 1048576);  // (dbg 1048576: profiling, never staged)
  const bool both = stg && g.npairs * q_n <= P_QROWS;
  auto stage_pq = [&](int c0, int c1) __attribute__((always_inline)) {
    for (int c = c0; c < c1; ++c) {
      const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H) + n0 + 4 * lane;
      const int rb = both ? c * q_n : 0;
      for (int r = wave; r < q_n; r += 8) {
        const float* src = Pc + (long)(q_lo + r) * (2 * H);
        char* dst = lds + (rb + r) * (P_QP * 4);
        __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gbl_void*)(src + H), (lds_void*)(dst + BN * 4), 16, 0, 0);
      }
    }
  };
  if (stg) stage_pq(0, both ? g.npairs : 1);  // (lands while the scales and the pair tables load)
  const int cw = n0 + wn * 128 + 4 * g4;  // this lane's first output column (+ 16 j)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f32x4 sc = *reinterpret_cast<const f32x4*>(g.wscale + cw + 16 * j);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      accU[i][j] *= sc;
      accV[i][j] *= sc;
    }
  }
  int ni[2], nj[2];
  int2 pe[2];
  bool ok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long lr = wm * 32 + 16 * i + l16;
    const long p = row0 + (lr < nrows ? lr : nrows - 1);
    ni[i] = g.pi[p];
    nj[i] = g.pj[p];
    pe[i] = g.pe[p];
    ok[i] = lr < nrows;
  }
  if (stg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  _Float16* S0 = reinterpret_cast<_Float16*>(g.S);
  const bool odd = l16 & 1;
  const bool nostore = kPairAbl && (g.dbg & 4);  // (profiling)
  const float* T = reinterpret_cast<const float*>(lds);
  auto conditioning = [&](int c, auto STG) __attribute__((always_inline)) {
    constexpr bool staged = decltype(STG)::value;
    const float* Pc = g.PQ + (long)c * g.nnodes * (2 * H);
    const int rb = both ? c * q_n : 0;
    static_for<0, 2>([&](auto DIR) __attribute__((always_inline)) {
      constexpr int dir = decltype(DIR)::value;
      static_for<0, 2>([&](auto IC) __attribute__((always_inline)) {
        constexpr int i = decltype(IC)::value;
        // forward (i, j): P_i + Q_j, row pe.x; reverse (j, i): P_j + Q_i, row pe.y (none for a self pair)
        const int rp = dir ? nj[i] : ni[i], rq = dir ? ni[i] : nj[i];
        const float* prow;
        const float* qrow;
        if constexpr (staged) {
          prow = T + (rb + rp - q_lo) * P_QP + wn * 128 + 4 * g4;
          qrow = T + (rb + rq - q_lo) * P_QP + BN + wn * 128 + 4 * g4;
        } else {
          prow = Pc + (long)rp * (2 * H) + cw;
          qrow = Pc + (long)rq * (2 * H) + H + cw;
        }
        // (dbg 131072 / 262144, profiling: no reverse-direction stores / the reverse rows stored at the forward
        // rows' places: what the scattered reverse rows cost; wrong results)
        const long orow = (long)c * g.E + (dir && !(kPairAbl && (g.dbg & 262144)) ? pe[i].y : pe[i].x);
        const bool st = ok[i] && !nostore && (dir == 0 || (ni[i] != nj[i] && !(kPairAbl && (g.dbg & 131072))));
        f32x4 v[8];
        float mx = 0.f;
        const bool nopq = kPairAbl && (g.dbg & 524288);  // (profiling: P / Q rows not loaded; wrong results)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const f32x4 pv = nopq ? f32x4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(prow + 16 * j);
          const f32x4 qv = nopq ? f32x4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(qrow + 16 * j);
          const f32x4 x = dir ? accU[i][j] - accV[i][j] : accU[i][j] + accV[i][j];
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2e y = silu_e2((f32x2e{x[e], x[e + 1]} + f32x2e{pv[e], pv[e + 1]}) + f32x2e{qv[e], qv[e + 1]});
            mx = fmaxf(mx, fmaxf(fabsf(y.x), fabsf(y.y)));
            v[j][e] = y.x;
            v[j][e + 1] = y.y;
          }
        }
        // the row's 128 columns of this wave sit in the 4 lanes l16 + 16 g
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const int ex2 = exp_of(mx);
        const float sc = ldexpf(1.0f, -ex2);
        // whole-line stores as edge16_tile's: lanes l16, l16 ^ 1 swap a piece (DPP) so that one store writes
        // the even lane's row's whole 128-B line and the next the odd lane's (rows anywhere in S)
        const long orow_p = ((long)__shfl_xor((int)(orow >> 32), 1, 64) << 32) | (unsigned)__shfl_xor((int)orow, 1, 64);
        const int st_p = __shfl_xor(st ? 1 : 0, 1, 64);
        const long orow_e = odd ? orow_p : orow, orow_o = odd ? orow : orow_p;
        const bool st_e = odd ? st_p != 0 : st, st_o = odd ? st : st_p != 0;
        const int off = ((n0 + wn * 128) / 32) * 64 + 8 * g4 + (odd ? 32 : 0);
        _Float16* se = S0 + orow_e * (2 * H) + off;
        _Float16* so = S0 + orow_o * (2 * H) + off;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {  // 32-column chunks: column groups 2cc, 2cc + 1
          f16x8 hv, lv;
#pragma unroll
          for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float xx = v[2 * cc + a2][r] * sc;
              const _Float16 hx = (_Float16)xx;
              hv[4 * a2 + r] = hx;
              lv[4 * a2 + r] = (_Float16)(xx - (float)hx);
            }
          typedef int i32x4 __attribute__((ext_vector_type(4)));
          const i32x4 snd = __builtin_bit_cast(i32x4, odd ? hv : lv);
          i32x4 rcv;
#pragma unroll
          for (int w = 0; w < 4; ++w) rcv[w] = __builtin_amdgcn_mov_dpp(snd[w], 0xB1, 0xF, 0xF, false);  // lane ^ 1
          const f16x8 r8 = __builtin_bit_cast(f16x8, rcv);
          if (st_e) *reinterpret_cast<f16x8*>(se + cc * 64) = odd ? r8 : hv;  // even lane's row: hi (even), lo (odd)
          if (st_o) *reinterpret_cast<f16x8*>(so + cc * 64) = odd ? lv : r8;  // odd lane's row
        }
        if (st && g4 == 0 && !(kPairAbl && (g.dbg & 2097152))) {  // (dbg 2097152, profiling: no exponent bytes; wrong results)
          signed char* px = reinterpret_cast<signed char*>(g.sexp) + orow * 4 + (n0 + wn * 128) / CHUNK;
          *px = (signed char)ex2;
        }
      });
    });
  };
  // (only conditioning 0's rows staged: conditioning 1 reads its rows from global memory, since staging them
  // now would have to wait for conditioning 0's S stores too: vmcnt counts loads and stores in one counter)
  for (int c = 0; c < g.npairs; ++c) {
    if (stg && (c == 0 || both))
      conditioning(c, std::integral_constant<bool, true>{});
    else
      conditioning(c, std::integral_constant<bool, false>{});
  }
}

// the pair grid's first repair launch (exits at once unless the grid raised its repair request): clear layer
// 2's agg row maxima and row-tile counters, then recompute every pair tile (grid-stride); the layer-2 repair
// launch behind it recomputes edge layer 2
__global__ __launch_bounds__(512, 1) void k_edge16_pairs_repair(EdgeArgs g, long ntiles, unsigned* agg_max, long nmax,
                                                                unsigned* rcnt, long nrcnt) {
  if (__hip_atomic_load(g.xbad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  for (long k = (long)blockIdx.x * 512 + threadIdx.x; k < nmax; k += (long)gridDim.x * 512) agg_max[k] = 0u;
  for (long k = (long)blockIdx.x * 512 + threadIdx.x; k < nrcnt; k += (long)gridDim.x * 512) rcnt[k] = 0u;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    pair_tile(g, t, threadIdx.x);
    __syncthreads();
  }
}

// edge layer 1 on pairs as a launch of its own (the two-launch schedule; the pair grid's repairs use
// k_edge16_pairs_repair)
__global__ __launch_bounds__(512, 1) void k_edge16_pairs(EdgeArgs g) {
  pair_tile(g, remap(blockIdx.x, gridDim.x), threadIdx.x);
}

hipError_t edge_gemm16_pairs(const EdgeArgs& g, hipStream_t s) {
  if (g.N != H || g.K != FD || !g.A || !g.W || !g.wscale || !g.S || !g.sexp || !g.PQ || !g.pi || !g.pj || !g.pe ||
      g.Mp < 1 || g.npairs < 1 || g.npairs > 2 || g.nnodes < 1 || g.E < g.Mp)
    return hipErrorInvalidValue;
  if (hipError_t e = edge16_init(); e != hipSuccess) return e;
  const long blocks = (g.Mp + PBM - 1) / PBM * (H / BN);
  hipLaunchKernelGGL(k_edge16_pairs, dim3((unsigned)blocks), dim3(512), LDS_B, s, g);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Both edge layers of a CSP layer in one grid, edge layer 1 on pairs (chm_internal.h PairSched).
// The directed one-grid kernels (k_edge16_layer*) pair layer-1 row tile t with layer-2 row tile t; on pairs,
// layer-2 row tile t reads the S rows of every pair tile of its crystals up to its last node's pair row, a
// contiguous range [lo(t), hi(t)] (pair_plan). Each XCD runs a contiguous range of row tiles and all the pair
// tiles they read, so every S row a layer-2 tile reads was written through the same XCD's L2 (list x = the
// jobs of one XCD). Ranges of neighbouring lists may share a pair tile: both compute it and write identical bytes.
void pair_plan(const std::vector<int>& nat, long E, long Ep, long R, int P, int lag, PairPlan& out) {
  const int B = (int)nat.size();
  std::vector<long> eoff(B + 1, 0), poff(B + 1, 0);
  for (int g = 0; g < B; ++g) {
    eoff[g + 1] = eoff[g] + (long)nat[g] * nat[g];
    poff[g + 1] = poff[g] + (long)nat[g] * (nat[g] + 1) / 2;
  }
  auto crystal_of = [&](long row) {  // the crystal holding directed edge row `row`
    return (int)(std::upper_bound(eoff.begin(), eoff.end(), row) - eoff.begin()) - 1;
  };
  out.rng.assign(R, make_int2(0, 0));
  for (long t = 0; t < R; ++t) {
    const long r0 = t * BM, r1 = (t * BM + BM < E ? t * BM + BM : E) - 1;
    const int g0 = crystal_of(r0), g1 = crystal_of(r1);
    const long n1 = nat[g1], i1 = (r1 - eoff[g1]) / n1;
    // first pair of the first crystal (the first node's reverse rows read pairs from its crystal's start);
    // last pair of the last node's pair row (its forward rows)
    const long lo = poff[g0], hi = poff[g1] + i1 * n1 - i1 * (i1 - 1) / 2 + (n1 - 1 - i1);
    out.rng[t] = make_int2((int)(lo / PBM), (int)(hi / PBM));
  }
  const long NP = (Ep + PBM - 1) / PBM;
  out.pa.assign(8, 0);
  out.pb.assign(8, 0);
  out.njobs.assign(8, 0);
  std::vector<std::vector<int2>> jl(8);
  for (int x = 0; x < 8; ++x) {
    const long ra = R * x / 8, rb = R * (x + 1) / 8;
    if (ra >= rb) continue;
    const int pa = out.rng[ra].x, pb = out.rng[rb - 1].y + 1;
    out.pa[x] = pa;
    out.pb[x] = pb < NP ? pb : (int)NP;
    long t = ra;
    auto emit_row = [&](long tt) {
      for (int c = 0; c < P; ++c)
        for (int col = 0; col < 2; ++col) jl[x].push_back(make_int2(2, (int)((tt * P + c) * 2 + col)));
    };
    for (int p = pa; p < out.pb[x]; ++p) {
      jl[x].push_back(make_int2(1, p * 2));
      jl[x].push_back(make_int2(1, p * 2 + 1));
      for (; t < rb && out.rng[t].y + lag <= p; ++t) emit_row(t);
    }
    for (; t < rb; ++t) emit_row(t);
    out.njobs[x] = (int)jl[x].size();
  }
  out.jstride = 0;
  out.npx = 1;
  for (int x = 0; x < 8; ++x) {
    out.jstride = std::max(out.jstride, out.njobs[x]);
    out.npx = std::max(out.npx, out.pb[x] - out.pa[x]);
  }
  out.jobs.assign((size_t)8 * out.jstride, make_int2(0, 0));
  for (int x = 0; x < 8; ++x) std::copy(jl[x].begin(), jl[x].end(), out.jobs.begin() + (size_t)x * out.jstride);
  // the device records: flag indices relative to the list's first pair tile, so a block loads nothing else
  out.djobs.assign(out.jobs.size(), make_int4(0, 0, 0, 0));
  for (int x = 0; x < 8; ++x)
    for (int k = 0; k < out.njobs[x]; ++k) {
      const int2 j = out.jobs[(size_t)x * out.jstride + k];
      int4& d = out.djobs[(size_t)x * out.jstride + k];
      if (j.x == 1) {
        d = make_int4(1, j.y, j.y / 2 - out.pa[x], 0);
      } else {
        const int2 r = out.rng[j.y / (2 * P)];
        d = make_int4(2, j.y, r.x - out.pa[x], r.y - out.pa[x]);
      }
    }
}

// every device record's flag indices inside its list's flag words (checked on the host before any upload)
bool pair_plan_ok(const PairPlan& pl) {
  if (pl.djobs.size() != (size_t)8 * pl.jstride || pl.npx < 1) return false;
  for (const int4& d : pl.djobs) {
    if (d.x == 1 && (d.z < 0 || d.z >= pl.npx)) return false;
    if (d.x == 2 && (d.z < 0 || d.z > d.w || d.w >= pl.npx)) return false;
    if (d.x < 0 || d.x > 2) return false;
  }
  return true;
}

// The static-grid form (option edge_pairs_layer = 1): block 8 k + x runs job k of list x (pair_plan), one
// tile per block, no job loop. Workgroups are dispatched in index order and round-robin over the XCDs, so
// the blocks of list x share one XCD (which one depends on where the dispatcher's rotation stands: measured
// under graph replay, it is not always x) and every pair tile a layer-2 job waits for belongs to an earlier
// block of the same list: dispatched before it, never waiting itself. Each column tile of a pair tile adds
// 1 + (its XCD + 1) << (8 + 4 col) to its flag; a layer-2 job that finds another XCD there (S written through
// another L2) or times out raises the layer's repair request (the repair launches recompute the layer).
__global__ __launch_bounds__(512, 1) void k_edge16_pairs_grid(EdgeArgs g1, EdgeArgs g2, PairSched ps) {
  const int xs = (int)(blockIdx.x & 7u), k = (int)(blockIdx.x >> 3);
  const int4 j = ps.jobs[(long)xs * ps.jstride + k];  // (past the end of list xs: kind 0)
  const unsigned me = xcc_id();
  unsigned* pf = ps.pflag + (long)xs * ps.npx;
  const unsigned long long t0 = kGridTrace && ps.trace ? rtime() : 0;  // (profiling: block timelines)
  unsigned long long tw = t0;
  auto trace_end = [&]() __attribute__((always_inline)) {
    if (kGridTrace && ps.trace && threadIdx.x == 0) {
      unsigned long long* o = ps.trace + 6 * (long)blockIdx.x;
      o[0] = hwid(); o[1] = t0; o[2] = tw; o[3] = rtime(); o[4] = (unsigned)j.x; o[5] = (unsigned)j.y;
    }
  };
  if (j.x == 1) {
    pair_tile(g1, j.y, threadIdx.x);
    // every store of this tile has reached the XCD's L2; count the column tile (and a misplaced block)
    // (dbg 4194304, profiling: published without waiting for the stores, the drain's cost; wrong results)
    if (!(g1.dbg & 4194304)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    } else {
      __builtin_amdgcn_s_barrier();  // (an LDS-only barrier: __syncthreads() would wait for the stores)
    }
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(pf + j.z, 1u + ((me + 1u) << (8 + 4 * (j.y & 1))), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    trace_end();
    return;
  }
  if (j.x != 2) return;
  if (threadIdx.x < 64) {
    // wait (bounded) until both column tiles of every pair tile read are in: lane l polls flag j.z + l (64 at a
    // time), so the pair tiles' flags cost one load latency together instead of one each
    const int lane = (int)threadIdx.x;
    bool late = false, other = false;
    for (int p0 = j.z; p0 <= j.w && !late; p0 += 64) {
      const int p = p0 + lane;
      const bool mine = p <= j.w;
      unsigned v = mine ? __hip_atomic_load(pf + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 2u;
      unsigned spins = 0;
      while (__any((v & 0xffu) < 2u) && ++spins < (1u << 21)) {
        __builtin_amdgcn_s_sleep(4);
        if ((v & 0xffu) < 2u) v = __hip_atomic_load(pf + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      late = __any((v & 0xffu) < 2u);
      other |= __any(mine && (((v >> 8) & 15u) != me + 1u || ((v >> 12) & 15u) != me + 1u));
    }
    if (lane == 0) {
      if (late || other || (g2.dbg & 512))  // (dbg 512, tests: option edge_layer_repair)
        __hip_atomic_store(g2.xbad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (late) count_event(EV_LAYER_TIMEOUT);
      else if (other) count_event(EV_LAYER_XCD);
      if (kGridTrace && ps.trace) tw = rtime();
    }
  }
  __syncthreads();
  edge16_tile<EPI_SEGMEAN, true>(g2, 0, 0, j.y);
  if (kGridTrace && ps.trace) {
    __syncthreads();
    trace_end();
  }
}

hipError_t edge_gemm16_pairs_layer(const EdgeArgs& g1, const EdgeArgs& g2, const PairSched& ps, int repair_grid,
                                   hipStream_t s) {
  if (g1.N != H || g1.K != FD || !g1.A || !g1.W || !g1.wscale || !g1.S || !g1.sexp || !g1.PQ || !g1.pi || !g1.pj ||
      !g1.pe || g1.Mp < 1 || g1.npairs != g2.npairs || g1.E < g1.Mp || !g1.xbad || g1.xbad != g2.xbad)
    return hipErrorInvalidValue;
  if (g2.N != H || g2.K % CHUNK || g2.K / CHUNK > 4 || !g2.rtiles || !g2.sbuf || !g2.msgbuf || !g2.rcnt || !g2.agg ||
      !g2.bias || !g2.aexp || !g2.node_n || !g2.A || !g2.W || !g2.wscale || g2.flags || g2.lflags ||
      (long)g2.ntiles != ps.R || (long)g2.ntiles * BM < g2.E || g2.rt_first || g2.rt_count || g2.rt_h || g2.rt_e0)
    return hipErrorInvalidValue;  // (uniform 256-row tiles only)
  if (!ps.jobs || !ps.pflag || ps.jstride < 1 || ps.npx < 1) return hipErrorInvalidValue;
  if (hipError_t e = edge16_init(); e != hipSuccess) return e;
  hipLaunchKernelGGL(k_edge16_pairs_grid, dim3((unsigned)(8 * ps.jstride)), dim3(512), LDS_B, s, g1, g2, ps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || (g1.dbg & 16384)) return e;  // (dbg 16384: profiling / tests, no repair launches)
  // the repair launches (exit at once unless a wait timed out or saw another XCD): clear layer 2's agg row
  // maxima and row-tile counters and recompute every pair tile, then every layer-2 tile (two launches; r5: the
  // clearing and the pair tiles were two launches, 4.5 us more per layer when nothing is repaired)
  const unsigned rg = (unsigned)(repair_grid > 0 ? repair_grid : 256);
  EdgeArgs r1 = g1, r2 = g2;
  const long nb1 = (g1.Mp + PBM - 1) / PBM * (H / BN);
  hipLaunchKernelGGL(k_edge16_pairs_repair, dim3(rg), dim3(512), LDS_B, s, r1, nb1, g2.agg_max,
                     g2.agg_max ? (long)g2.npairs * g2.nnodes : 0L, g2.rcnt, g2.rcnt ? (long)g2.npairs * g2.ntiles * 8 : 0L);
  const long nb2 = (long)g2.ntiles * g2.npairs * (g2.N / BN);
  hipLaunchKernelGGL((k_edge16_repair<EPI_SEGMEAN, true>), dim3(rg), dim3(512), LDS_B, s, r2, nb2, (unsigned*)nullptr,
                     0L, (unsigned*)nullptr, 0L, (int)EV_LAYER_REPAIR);
  return hipGetLastError();
}

static hipError_t edge16_init_once() {
  const void* ks[] = {(const void*)k_edge16<EPI_STD, false>, (const void*)k_edge16<EPI_EDGE, false>,
                      (const void*)k_edge16<EPI_SEGMEAN, true>, (const void*)k_edge16<EPI_STD, true>,
                      (const void*)k_edge16_tail, (const void*)k_edge16_layer, (const void*)k_edge16_layer_dyn,
                      (const void*)k_edge16_repair<EPI_EDGE, false>, (const void*)k_edge16_repair<EPI_SEGMEAN, true>,
                      (const void*)k_edge16_pairs, (const void*)k_edge16_pairs_grid, (const void*)k_edge16_pairs_repair,
                      (const void*)k_edge16_short};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_B);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// the kernels' LDS attribute, set once per process (thread-safe: a function-local static initialiser)
hipError_t edge16_init() {
  static const hipError_t e = edge16_init_once();
  return e;
}

hipError_t edge_events_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_edge_events), sizeof(unsigned long long) * EV_COUNT, 0,
                             hipMemcpyDeviceToHost);
}

hipError_t edge_events_reset() {
  static const unsigned long long zero[EV_COUNT] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_edge_events), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}

hipError_t edge_gemm16_tail(const EdgeArgs& g1, const EdgeArgs& g2, int repair_grid, hipStream_t s) {
  if (g1.N != H || g1.K % (2 * BK) || g1.aexp || !g1.S || !g1.sexp || !g1.PQ || !g1.node_off || !g1.natoms ||
      !g1.n2g || !g1.A || !g1.W || !g1.wscale || g1.npairs > 2 || g1.M <= g1.row_base || g1.row_base < 0 ||
      !g1.flags || g1.flags != g2.flags || g1.flag_row0 != g1.row_base || g2.flag_row0 != g1.row_base ||
      !g2.xbad)
    return hipErrorInvalidValue;
  if (g2.N != H || g2.K % CHUNK || g2.K / CHUNK > 4 || !g2.tiles || g2.ntiles < 1 || !g2.agg || !g2.bias ||
      !g2.aexp || !g2.node_n || !g2.A || !g2.W || !g2.wscale || g2.rt_first || g2.rt_count || g2.rt_h || g2.rt_e0 ||
      (g2.rtiles && (!g2.sbuf || !g2.msgbuf || !g2.rcnt || (long)g2.ntiles * BM < g2.E)))
    return hipErrorInvalidValue;  // (uniform tiles only)
  if (hipError_t e = edge16_init(); e != hipSuccess) return e;
  const long nt1 = ((g1.M - g1.row_base + BM - 1) / BM) * (g1.N / BN);
  const long nb1 = (nt1 + 7) / 8 * 8;
  const long nt2 = (long)g2.ntiles * g2.npairs * (g2.N / BN);
  hipLaunchKernelGGL(k_edge16_tail, dim3((unsigned)(nb1 + nt2)), dim3(512), LDS_B, s, g1, g2, (int)nb1, (int)nt1);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || (g2.dbg & 16384)) return e;
  // the repair pair (exits at once unless a segment tile's wait timed out): the first clears layer 2's
  // agg row maxima (the failed tiles may have max-ed garbage; S itself was complete when the grid
  // ended), the second recomputes every segment tile of edge layer 2 without intra-grid waits
  EdgeArgs r1 = g1, r2 = g2;
  r1.flags = r2.flags = nullptr;
  r1.xbad = g2.xbad;
  const unsigned rg = (unsigned)(repair_grid > 0 ? repair_grid : 256);
  hipLaunchKernelGGL((k_edge16_repair<EPI_EDGE, false>), dim3(rg), dim3(512), LDS_B, s, r1, 0L, g2.agg_max,
                     g2.agg_max ? (long)g2.npairs * g2.nnodes : 0L, (unsigned*)nullptr, 0L, -1);
  hipLaunchKernelGGL((k_edge16_repair<EPI_SEGMEAN, true>), dim3(rg), dim3(512), LDS_B, s, r2, nt2, (unsigned*)nullptr,
                     0L, (unsigned*)nullptr, 0L, (int)EV_TAIL_REPAIR);
  return hipGetLastError();
}

long edge16_layer_blocks(long R, int P) { return 8 * ((R + 7) / 8) * (2 + 2L * P); }

// (host) the job of every block of a k_edge16_layer grid: out[2 b] = kind, out[2 b + 1] = tile index
void edge16_layer_jobs(long R, int P, int D, long* out) {
  const long nb = edge16_layer_blocks(R, P);
  for (long b = 0; b < nb; ++b) {
    const LayerJob j = layer_job(b, R, P, D);
    out[2 * b] = j.kind;
    out[2 * b + 1] = j.bid;
  }
}

void edge16_seq_jobs(long n, int P, int D, long* out) {
  for (long k = 0; k < n; ++k) {
    const SeqJob j = seq_job(k, P, D);
    out[3 * k] = j.kind;
    out[3 * k + 1] = j.row;
    out[3 * k + 2] = j.sub;
  }
}

hipError_t edge_gemm16_layer(const EdgeArgs& g1, const EdgeArgs& g2, int lag, int repair_grid, hipStream_t s,
                             unsigned* sched, int cap, int grid, int pool, int skip_xcd) {
  if (g1.N != H || g1.K % (2 * BK) || g1.aexp || !g1.S || !g1.sexp || !g1.PQ || !g1.node_off || !g1.natoms ||
      !g1.n2g || !g1.A || !g1.W || !g1.wscale || g1.npairs > 2 || g1.row_base != 0 || g1.flags || !g1.lflags ||
      !g1.xbad || g1.xbad != g2.xbad)
    return hipErrorInvalidValue;
  if (g2.N != H || g2.K % CHUNK || g2.K / CHUNK > 4 || !g2.rtiles || !g2.sbuf || !g2.msgbuf || !g2.rcnt || !g2.agg ||
      !g2.bias || !g2.aexp || !g2.node_n || !g2.A || !g2.W || !g2.wscale || g2.flags || g2.lflags != g1.lflags ||
      g2.npairs != g1.npairs || (long)g2.ntiles * BM < g2.E || (long)g2.ntiles * BM - g2.E >= BM || g1.M != g1.E ||
      lag < 1 || g2.rt_first || g2.rt_count || g2.rt_h || g2.rt_e0)
    return hipErrorInvalidValue;  // (uniform 256-row tiles only)
  if (hipError_t e = edge16_init(); e != hipSuccess) return e;
  const long R = g2.ntiles;
  if (sched) {  // persistent, the last rows claimed at run time (k_edge16_layer_dyn)
    if (grid < 1 || cap < R + lag + 64 || pool < 0 || pool > 100) return hipErrorInvalidValue;
    const int ns = (int)((R - (R * pool + 99) / 100) / 8);  // static rows per XCD
    hipLaunchKernelGGL(k_edge16_layer_dyn, dim3((unsigned)grid), dim3(512), LDS_B, s, g1, g2, (int)R, lag, sched, cap,
                       ns, skip_xcd);
  } else {
    const long blocks = edge16_layer_blocks(R, g2.npairs);
    hipLaunchKernelGGL(k_edge16_layer, dim3((unsigned)blocks), dim3(512), LDS_B, s, g1, g2, (int)R, lag);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || (g1.dbg & 16384)) return e;  // (dbg 16384: profiling / tests, no repair launches)
  // the repair pair (exits at once unless a layer-2 tile flagged another XCD's layer-1 tile)
  EdgeArgs r1 = g1, r2 = g2;
  r1.lflags = r2.lflags = nullptr;
  const long nb1 = ((g1.M + BM - 1) / BM) * (g1.N / BN), nb2 = (long)g2.ntiles * g2.npairs * (g2.N / BN);
  const unsigned rg = (unsigned)(repair_grid > 0 ? repair_grid : 256);
  hipLaunchKernelGGL((k_edge16_repair<EPI_EDGE, false>), dim3(rg), dim3(512), LDS_B, s, r1, nb1, g2.agg_max,
                     (long)g2.npairs * g2.nnodes, g1.lflags, R, -1, g2.rcnt, (long)g2.npairs * R * 8);
  hipLaunchKernelGGL((k_edge16_repair<EPI_SEGMEAN, true>), dim3(rg), dim3(512), LDS_B, s, r2, nb2, (unsigned*)nullptr, 0L,
                     (unsigned*)nullptr, 0L, (int)EV_LAYER_REPAIR);
  return hipGetLastError();
}

hipError_t edge_gemm16(const EdgeArgs& g, int epi, hipStream_t s) {
  if (g.N % BN || g.K % (2 * BK) || !g.A || !g.W || !g.wscale) return hipErrorInvalidValue;
  const bool asc = g.aexp != nullptr;
  if (asc && (g.K % CHUNK || g.K / CHUNK > 4)) return hipErrorInvalidValue;
  long blocks;
  bool short_tiles = false;
  if (epi == EPI_SEGMEAN) {
    if (g.N != H || !g.tiles || !g.agg || !g.bias || !asc || !g.node_n) return hipErrorInvalidValue;
    long nt = g.ntiles;
    if (g.rtiles) {
      if (!g.sbuf || !g.msgbuf || !g.rcnt) return hipErrorInvalidValue;
      if (g.rt_first || g.rt_count || g.rt_h || g.rt_e0) {
        // one launch of a mixed tiling: tiles [rt_first, rt_first + rt_count) of ntiles, each with at least one row
        nt = g.rt_count;
        if ((g.rt_h != 0 && g.rt_h != BM && g.rt_h != kShortRows) || g.rt_first < 0 || nt < 1 ||
            g.rt_first + nt > g.ntiles || g.rt_e0 < 0 || g.rt_e0 + (nt - 1) * (g.rt_h ? g.rt_h : BM) >= g.E)
          return hipErrorInvalidValue;
        short_tiles = g.rt_h == kShortRows;
      } else if ((long)g.ntiles * BM < g.E) {
        return hipErrorInvalidValue;
      }
    } else if (g.rt_first || g.rt_count || g.rt_h || g.rt_e0) {
      return hipErrorInvalidValue;
    }
    blocks = nt * g.npairs * (g.N / BN);
  } else {
    if (g.M <= g.row_base || g.row_base < 0) return hipErrorInvalidValue;
    if (epi == EPI_EDGE &&
        (g.N != H || !g.S || !g.sexp || !g.PQ || !g.node_off || !g.natoms || !g.n2g || asc || g.npairs > 2))
      return hipErrorInvalidValue;
    blocks = ((g.M - g.row_base + BM - 1) / BM) * (g.N / BN);
  }
  if (hipError_t e = edge16_init(); e != hipSuccess) return e;
  const EdgeArgs& ga = g;
  const dim3 grid((unsigned)blocks), block(512);
  if (epi == EPI_EDGE)
    hipLaunchKernelGGL((k_edge16<EPI_EDGE, false>), grid, block, LDS_B, s, ga);
  else if (epi == EPI_SEGMEAN && short_tiles)
    hipLaunchKernelGGL(k_edge16_short, grid, block, LDS_B, s, ga);
  else if (epi == EPI_SEGMEAN)
    hipLaunchKernelGGL((k_edge16<EPI_SEGMEAN, true>), grid, block, LDS_B, s, ga);
  else if (asc)
    hipLaunchKernelGGL((k_edge16<EPI_STD, true>), grid, block, LDS_B, s, ga);
  else
    hipLaunchKernelGGL((k_edge16<EPI_STD, false>), grid, block, LDS_B, s, ga);
  return hipGetLastError();
}

}  // namespace chm
