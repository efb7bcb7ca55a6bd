// Internal declarations shared by kernels.hip and runtime.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace chm {

constexpr int H = 512;       // hidden_dim (the build implements the shipped config)
constexpr int NF = 128;      // num_freqs
constexpr int FD = 6 * NF;   // Fourier feature width, 768
constexpr int TD = 128;      // time_dim
constexpr int HEADS_N = 128; // type_out (A <= 125) + coord_out (3) packed, padded
constexpr int kMaxLayers = 64;  // num_layers accepted by chm_model_create

// C[M,N] = epi(A[M,K] . W[N,K]^T), fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32.
struct GemmArgs {
  long M;
  int N, K;
  const float* A; long lda;
  const float* A2; long lda2; int ksplit;  // columns k >= ksplit come from A2[:, k - ksplit]
  const float* W; long ldw;                // [N][K] row-major (nn.Linear layout)
  float* C; long ldc;
  const float* bias;                       // [N] or null
  const float* R; long ldr;                // residual added after the activation, or null
  const int* row2g; long gb_rowmod; const float* gb; long ldgb; int gb_cols;  // per-graph row bias
  int act;                                 // 0 = identity, 1 = SiLU
  // EPI_EDGE: S[c][e][n] = silu(acc + PQ[c*N + ei[e]][n] + PQ[c*N + ej[e]][H + n])
  const int* ei; const int* ej; const float* PQ; long nnodes; int npairs; long E;
  // bf16x3 path: W split into three bf16 planes [3][N][K] (hi, mid, lo)
  const void* Wp3;
  // split16 node GEMMs (node_gemm.hip): Wp3 = fp16 hi/lo rows [N][K/16][hi 16 | lo 16] of W scaled
  // by wscale[n]^-1 (split_rows_h with 16-column chunks); null wscale = bf16x3 planes
  const float* wscale;
  // split16 node GEMMs: per A row, max |A[row, :]| (amax, and amax2 for the A2 columns; float
  // values, >= 0) sets the row's power-of-two scale; null = unscaled. cmax != null: max |C[row, :]|
  // of the output (after bias / activation / residual) is atomically max-ed into cmax[row] (float
  // bits as unsigned), for the next GEMM that reads C.
  const float* amax; const float* amax2; unsigned* cmax;
  // split16 node GEMMs with PRE-SPLIT A (model option node_ps): A / A2 are then split rows [rows][K/16][hi 16 |
  // lo 16] fp16 of A scaled per (row, 128-column chunk) by 2^-e, written by the kernel that produced A (no split
  // inside the K loop: the register split was two thirds of the loop's VALU, PMC r4); aex / aex2 hold per row
  // the 4 packed int8 exponents e of its 128-column chunks (A2's for the columns k >= ksplit); lda / lda2 in
  // 4-byte units as for fp32 rows (one split row of K columns is K * 4 bytes). Cs / cex: the output C
  // written the same way (the block's 128 columns are one chunk), besides or instead of the fp32 C.
  const int* aex; const int* aex2; void* Cs; int* cex;
  // EPI_SEGMEAN (message GEMM + scatter_mean): row tiles cover whole nodes
  const int2* tiles; int ntiles;          // node ranges [x, y) of one conditioning
  const long* node_estart;                // first edge row of each node
  const int* natoms; const int* n2g;
  float* agg;                             // [P][N][H]
  int linear_order;                       // node_gemm: 1 = tiles in launch order (A/B only), 0 = XCD-aware
};

enum { EPI_STD = 0, EPI_EDGE = 1, EPI_SEGMEAN = 2 };

// split16 edge GEMMs (edge16.hip): both operands split into fp16 hi/lo, stored per row as
// [K/32][hi 32 | lo 32] (a 32-deep K-tile of a row = one 128-B line), three fp16 MFMA products,
// staged by global_load_lds.
constexpr int kPairRows = 128;  // pairs per tile of edge layer 1 on pairs (k_edge16_pairs / the pair grid)
constexpr int kRowInfo = 260;  // EdgeArgs::rinfo entries per row tile (a tile holds at most 257 nodes)
constexpr int kShortRows = 192;  // edge layer 2's short row tiles (a mixed tiling's last round)
struct EdgeArgs {
  long M;                        // EPI_STD / EPI_EDGE: rows [row_base, M)
  long row_base;
  int N, K;
  const void* A;                  // split rows [rows][K/32][2][32] fp16, readable 256 rows past the last
  const int* aexp;               // per A row: 4 packed int8 exponents of its 128-column chunks, or null
  const void* W;                 // split rows [N][K/32][2][32], rows scaled by 1 / wscale
  const float* wscale;
  float* C; long ldc;            // EPI_STD output
  // EPI_EDGE: S[c][e] = SiLU(acc + PQ[c][ei[e]][:H] + PQ[c][ej[e]][H:]) written as scaled fp16 planes
  const int* ei; const int* ej; const float* PQ; long nnodes; int npairs; long E;
  const int* node_off;           // EPI_EDGE: first node of each graph (with natoms, n2g)
  void* S; int* sexp;            // S as split rows [P*E][H/32][2][32] (columns permuted within each
                                 // 32-chunk, see edge16.hip) + packed chunk exponents
  // EPI_SEGMEAN: agg[c][node] = mean over the node's edges of SiLU(acc + bias)
  const float* bias;
  const int2* tiles; int ntiles;
  const long* node_estart;
  const int* natoms; const int* n2g;
  const int* node_n;             // EPI_SEGMEAN: atom count of each node's crystal
  float* agg;
  unsigned* agg_max;             // EPI_SEGMEAN: max |agg[c][node][:]| atomically max-ed per row, or null
  void* aggs; int* agge;         // EPI_SEGMEAN, pre-split node GEMMs: agg written as split rows [P*N][H/16][hi 16 |
                                 // lo 16] scaled per 128-column chunk + the packed chunk exponents (agg then
                                 // stays unwritten); null = fp32 agg
  // EPI_SEGMEAN on row tiles (k_edge16, fc batches): tile t = edge rows [256 t, 256 t + 256) of each
  // conditioning, nodes cut at tile ends (ntiles = row tiles). rtiles[t] = {first node starting in
  // the tile, first node starting after it, the node continued from tile t-1 or -1, its rows' offset
  // in msgbuf}. A cut node's sum stays one sequential sum over its edges: tile t-1 publishes the
  // partial sum of its head part (sbuf [P][ntiles][H]), tile t continues it (rcnt [P][ntiles][8]:
  // one counter per column group of 64; msgbuf [P][r2tot][H]: the continued rows, written only when
  // tile t-1 has not published in time). null rtiles = node tiles (tiles / ntiles).
  const int4* rtiles; float* sbuf; float* msgbuf; unsigned* rcnt; long r2tot;
  // a mixed row tiling (r6, short last round): this launch runs rt_count row tiles from rt_first on (0 = all
  // ntiles), tile rt_first + k = rows [rt_e0 + k rt_h, + rt_h) (rt_h 0 = 256); 192-row tiles run in k_edge16_short
  // (3 row groups per wave). Tile indices stay global (rtiles, rinfo, sbuf and rcnt are indexed by them).
  int rt_first, rt_count, rt_h; long rt_e0;
  // fc row tiles: each tile's node list as the segment-mean epilogue uses it, built on the host with the
  // batch (rinfo [ntiles][kRowInfo] {node, rows | first row << 10 | kind << 20}, rinfo_n [ntiles] entries),
  // so the epilogue loads it in one round trip instead of deriving it through dependent loads; or null
  const int2* rinfo; const int* rinfo_n;
  // k_edge16_layer (both edge layers in one grid): per row tile, the count of layer-1 column tiles that
  // have written S through, then of the layer-2 tiles that have read it (the last one resets it to 0)
  unsigned* lflags;
  unsigned* xbad;  // k_edge16_layer: raised by a layer-2 tile that read S of another XCD or whose wait timed
                   // out; k_edge16_tail: raised by a segment tile whose wait for this grid's layer-1 tiles
                   // timed out. Either way the repair launches behind the grid recompute the layer.
  // k_edge16_tail: per layer-1 row tile from flag_row0 on, the count of its finished column tiles
  // (EPI_EDGE bumps, EPI_SEGMEAN tiles reading rows >= flag_row0 wait); null = no intra-grid waits.
  // zero_flags / nzero: an EPI_EDGE launch's block 0 clears them for the next grid.
  unsigned* flags; long flag_row0;
  unsigned* zero_flags; int nzero;
  // edge layer 1 on unordered pairs (k_edge16_pairs, fc batches, option edge_pairs): A = the pairs' Fourier
  // features (Mp rows: per crystal the pairs i <= j, row-major), pi / pj = the pair's nodes, pe = its edge
  // rows {(i, j), (j, i)} (equal for i == j)
  const int* pi; const int* pj; const int2* pe; long Mp;
  // per pair tile (kPairRows pairs): {first node, node count} of the P / Q rows its epilogue reads (the tile's
  // first pair's i up to the end of the crystal of its last pair), staged in LDS when they fit
  const int2* pnode;
  unsigned long long* trace;  // profiling: per block {hw id, t0, t_mainloop, t_end} (s_memrealtime) or null
  int stagger;  // first-round start delay (units of s_sleep 127) of every other CU, 0 = none
  int dbg;  // profiling ablations (0 in the product; wrong results): bit 0 = no K-loop loads, bit 1 = no
            // barriers, bit 2 = no epilogue stores (EDGE / SEGMEAN); k_edge16 also: bit 3 = no SiLU (SEGMEAN),
            // bit 4 = main loop only (no epilogue), bit 5 = no segment sums (SEGMEAN); bit 6 (tests, exact
            // results) = row tiles never wait for the previous tile's partial sums (msgbuf path); bit 9
            // (tests, exact results) = k_edge16_layer's layer-2 tiles always request the repair launches;
            // bit 13 (tests, exact results) = k_edge16_tail's layer-1 tiles start ~10 ms late and its
            // segment tiles wait ~2^10 spins only (a real timeout: they read S before it is written);
            // bit 14 (profiling / tests, WRONG results after a failed check) = no repair launches behind
            // k_edge16_tail or k_edge16_layer; bits 15 / 16 (profiling) = layer-1 / layer-2 tiles read their A
            // rows from the first 16 row tiles (L2-resident)
};
// Device event counters of the edge kernels (edge16.hip), cumulative over launches and graph replays
// until chm_prof_events_reset: wait timeouts and repair launches that ran (each must read 0 in a
// healthy run; a repair doubles the cost of its layer).
enum { EV_LAYER_TIMEOUT = 0, EV_LAYER_XCD = 1, EV_LAYER_REPAIR = 2, EV_TAIL_TIMEOUT = 3, EV_TAIL_REPAIR = 4,
       EV_LAYER_INCOMPLETE = 5, EV_COUNT = 8 };
// the XCD ids (bit x = XCC_ID x) the blocks of a `blocks`-block grid ran on (synchronous; model creation)
hipError_t xcd_mask(int blocks, unsigned* out);
hipError_t edge_events_read(unsigned long long* out);  // EV_COUNT values
hipError_t edge_events_reset();
// knn (radius-graph) edges, knn.hip: per-crystal scratch at cand_off[b] (n^2 * 27 entries; the final
// list at 2 * cand_off[b]), outputs sorted by source node into ei / ej / fd at node_estart
struct KnnArgs {
  const float* x; const float* lat; const int* natoms; const int* node_off;
  const long* cand_off; unsigned* cand_key; float* cand_d2; unsigned* cand2; int* atom_cnt; int max_nb;
  unsigned* fin_key; float* fin_fd; int* deg; int* cryst_fin;
  const long* node_estart; int* ei; int* ej; float* fd;
};
hipError_t knn_candidates(const KnnArgs& g, int B, hipStream_t s);  // pairs, cap, symmetric list, degrees
hipError_t knn_place(const KnnArgs& g, int B, hipStream_t s);       // grouped by source (node_estart set)
// training forward / validation loss (kernels.hip; chemeleon.py:137-244)
struct TrainArgs {
  long N; int B, A, T;
  const int64_t* t;        // [B] timestep per graph
  const int64_t* a0; const float* x0; const float* l0;
  const float* rand_a; const float* noise_l; const float* noise_x;  // [N,A], [B,3,3] (masked), [N,3]
  const float* coef;       // [T+1][4]: sqrt(abar), sqrt(1 - abar), sigma_x, sigma_norm
  const float* q_one_step; const float* q_mats;
  const int* n2g;
  int64_t* a_t; float* x_t; float* l_t; float* target_x;  // noised state, score target
  const float* HO; const float* LAT;                  // decoder heads on the noised state
  float* part;             // [N][2] per-node KL, CE
  float hybrid, cost_a, cost_l, cost_x;
  float* out;              // [6]: loss, vb, ce, loss_atom_types, loss_lattice, loss_coords
};
hipError_t train_noise(const TrainArgs& g, hipStream_t s);
hipError_t train_loss(const TrainArgs& g, hipStream_t s);
// the split16 edge GEMMs on v_mfma_f32_16x16x32_f16 (edge16.hip; S / W2 column permutation 2)
hipError_t edge_gemm16(const EdgeArgs& g, int epi, hipStream_t s);
// one grid: edge layer 1 (EPI_EDGE, g1: a row range) first, then edge layer 2 (EPI_SEGMEAN, g2: segment
// tiles that read none of g1's rows)
// g2.xbad: raised on a timed-out wait; the repair launches behind the grid then recompute layer 2
hipError_t edge_gemm16_tail(const EdgeArgs& g1, const EdgeArgs& g2, int repair_grid, hipStream_t s);
// both edge layers in one grid (row tiles; layer-2 tiles of row tile i - lag behind layer 1's row tile i)
// sched != null: the persistent form (grid blocks; the last pool% of the row tiles claimed at run time;
// sched = the layer's zeroed scheduling words, 16 + 8 * cap, cap >= R + lag + 64)
hipError_t edge_gemm16_layer(const EdgeArgs& g1, const EdgeArgs& g2, int lag, int repair_grid, hipStream_t s,
                             unsigned* sched = nullptr, int cap = 0, int grid = 0, int pool = 15, int skip_xcd = -1);
void edge16_seq_jobs(long n, int P, int D, long* out);  // (host) the persistent form's per-XCD job sequence
long edge16_layer_blocks(long R, int P);                        // its grid size
void edge16_layer_jobs(long R, int P, int D, long* out);         // (host) its block -> job map
hipError_t edge16_init();
// edge layer 1 on unordered pairs: S rows of both directions of every pair from one GEMM row (edge16.hip)
hipError_t edge_gemm16_pairs(const EdgeArgs& g, hipStream_t s);
// Both edge layers of a CSP layer in one static grid with edge layer 1 on pairs (k_edge16_pairs_grid): list x
// holds the row tiles [R x / 8, R (x + 1) / 8) of edge layer 2 and every pair tile they read (the tiles of two
// neighbouring lists' ranges may overlap: both compute them, identically), in the order of a host-built job list
// (pair tiles in order, a row tile's 2 P layer-2 jobs placed `lag` pair tiles behind the last pair tile it reads);
// its blocks share one XCD. A layer-2 job waits (bounded) until its list has finished every pair tile of its
// range, so S goes through that XCD's L2. Per batch and layer: pflag [8][npx], zeroed per decoder call.
struct PairSched {
  // [8][jstride] one record per block, all it needs in one load (padding: kind 0): {kind, tile, a, b}. kind 1 = pair
  // (tile = pair tile * 2 + column tile, a = its flag index in the list), 2 = layer 2 (tile = (row tile * P +
  // conditioning) * 2 + column tile, [a, b] = the flag indices of the pair tiles it reads)
  const int4* jobs;
  int jstride;
  int npx;             // pflag entries per list
  unsigned* pflag;     // [8][npx]: finished column tiles | their XCD + 1 << (8 + 4 col)
  long R;
  unsigned long long* trace = nullptr;  // (profiling, CHM_EDGE_TRACE_LAYER=4: per block {hw id, t0, t_wait, t_end, kind, tile})
};
// k_edge16_pairs_grid: static grid of 8 x jstride blocks, block 8 k + x = job k of list x, then the repair launches
hipError_t edge_gemm16_pairs_layer(const EdgeArgs& g1, const EdgeArgs& g2, const PairSched& ps, int repair_grid,
                                   hipStream_t s);
// (host) the job lists of k_edge16_pairs_grid for an fc batch: row tiles' pair-tile ranges, per list its first
// pair tile and job list (lag in pair tiles)
struct PairPlan {
  std::vector<int2> rng;
  std::vector<int> pa, pb, njobs;
  std::vector<int2> jobs;   // [8][jstride] {kind, tile}
  std::vector<int4> djobs;  // [8][jstride] the device records (PairSched::jobs)
  int jstride = 0, npx = 0;
};
void pair_plan(const std::vector<int>& nat, long E, long Ep, long R, int P, int lag, PairPlan& out);
bool pair_plan_ok(const PairPlan& pl);  // the device records' flag indices within [0, npx)
// (split16.hip) W -> row-scaled split rows (perm 0, or 2 = k_edge16's S column order for W2)
hipError_t split_rows_h(const float* W, int N, int K, void* out, float* wscale, int perm, hipStream_t s,
                        int chunk = 32);
hipError_t fourier_h(const float* x, const int* ei, const int* ej, long E, void* F, hipStream_t s,
                     const float* fd = nullptr);

hipError_t gemm(const GemmArgs& g, int epi, hipStream_t s);
// fp32-accurate GEMM on bf16 MFMA: A split on the fly into hi/mid/lo bf16,
// W pre-split; six products per fp32 product, fp32 accumulation.
hipError_t gemm_bf16x3(const GemmArgs& g, int epi, hipStream_t s);
// 256x256-tile variant (edge GEMMs); EPI_SEGMEAN tiles must then hold <= 256 rows
hipError_t gemm_bf16x3_big(const GemmArgs& g, int epi, hipStream_t s);
hipError_t gemm_init();  // one-time kernel attributes (call outside stream capture)
// node GEMMs, bf16x3 with global_load_lds staging (node_gemm.hip); EPI_STD semantics of gemm_bf16x3
hipError_t node_gemm(const GemmArgs& g, hipStream_t s);
hipError_t node_gemm_init();
extern int g_node_variant;  // microbenchmark probes of node_gemm (0 in the product)
extern int g_node_blocks;   // S16 node GEMM blocks per CU override (microbenchmarks; 0 = default)
extern int g_node_rows;     // node GEMM tile rows override (microbenchmarks; 0 = default, 64, 128)
extern int g_node_cols;     // S16 64-row node GEMM tile columns override (microbenchmarks; 0 = default, 64, 128)
// 256x256 tile, fp16 hi/lo split (three products) for operands with |A| <= 1 (Fourier features)
hipError_t split_planes(const float* src, long n, void* dst, hipStream_t s);
extern int g_gemm3_variant;  // tuning switch of gemm_bf16x3 (bench only)

hipError_t fourier(const float* x, const int* ei, const int* ej, long E, float* F, hipStream_t s);
hipError_t segment_mean(const float* msg, float* agg, const int* n2g, const int* node_off, const long* edge_off,
                        const int* natoms, long N, long E, int P, hipStream_t s);
// d_t != null: the time-embedding row is temb + (*d_t) * TD, shared by all graphs
hipError_t build_cond_in(const float* temb, int tstride, const int* d_t, const float* text0, const float* text1,
                         int text_dim, float* cin, int B, int P, hipStream_t s);
hipError_t decrement(int* d_t, hipStream_t s);
constexpr int kGBLayers = 16;
struct GraphBiasArgs { const float* Wc[kGBLayers]; const float* b1[kGBLayers]; };
// out[l] (l < nl, [B][H] each, consecutive) = the per-graph term of edge layer 1 of layer l
hipError_t graph_bias(const float* lat, const GraphBiasArgs& a, int nl, long ldwc, float* out, int B, hipStream_t s);
// rmax != null: rmax[row] = max |Hout[row, :]|
// (Hs / He: also the rows split for the pre-split node GEMMs, GemmArgs::aex; film_ln's Hls / Hle likewise)
// ga != null: the same launch also writes graph_bias(lat, *ga, nl, ldwc, gout, B)'s per-graph terms, and zeroes
// z0[0, n0) and z1[0, n1) (the words a decoder call starts from clear)
hipError_t embed(const int64_t* a, const float* emb, float* Hout, long N, int P, hipStream_t s, float* rmax = nullptr,
                 void* Hs = nullptr, int* He = nullptr, const float* lat = nullptr, const GraphBiasArgs* ga = nullptr,
                 int nl = 0, long ldwc = 0, float* gout = nullptr, int B = 0, unsigned* z0 = nullptr, long n0 = 0,
                 unsigned* z1 = nullptr, long n1 = 0);
// rmx != null (split16 node GEMMs): rows of the four row-max arrays [4][rstride] (RMX_*): writes
// max |Hl[row, :]| to RMX_HL and zeroes RMX_H, RMX_AGG, RMX_U for this layer's atomic maxima
enum { RMX_H = 0, RMX_HL = 1, RMX_AGG = 2, RMX_U = 3 };
hipError_t film_ln(const float* Y, float* Hres, float* Hl, const float* cond_emb, const int* n2g, long N, int B, int P,
                   const float* fw, const float* fb, const float* lw, const float* lb, hipStream_t s,
                   float* rmx = nullptr, long rstride = 0, void* Hls = nullptr, int* Hle = nullptr);
hipError_t layer_norm(const float* X, float* Y, long rows, const float* w, const float* b, hipStream_t s);
hipError_t graph_heads(const float* Hf, const float* Wlat, const float* lat, const int* node_off, const int* natoms,
                       long N, int B, int P, float* lat_out, hipStream_t s);
hipError_t split_heads(const float* HO, long rows, int A, float* types, float* coords, hipStream_t s);
hipError_t copy_rows(const float* src, long ld_src, float* dst, long ld_dst, long rows, int cols, hipStream_t s);

struct StepArgs {
  int t, T, A;
  const int* d_t;                  // if set, t is read from device memory (graph replay)
  long N; int B;
  float cs_null, cs_cond;          // (1 - s), s
  const float* coef;               // [T+1][8]
  const float* q_one_step;         // [T+1][A][A]
  const float* q_mats;             // [T+1][A][A]
  const float* HO;                 // [2][N][HEADS_N] cond then null
  const float* LAT;                // [2][B][9]
  int64_t* a; float* x; float* l;
  const int* n2g;
  const float *ra, *rl, *rx1, *rx2;  // host noise or null
  uint64_t seed; int64_t node_base, graph_base;
};
hipError_t step_predictor(const StepArgs& a, hipStream_t s);
// out[i] = Philox uniform (normal = 0) or normal (normal = 1) of (seed, t, kind, base + i)
hipError_t philox_fill(uint64_t seed, int t, int kind, int64_t base, long n, int normal, float* out, hipStream_t s);
hipError_t step_corrector(const StepArgs& a, hipStream_t s);
hipError_t d3pm_sample(int N, int A, int T, const float* logits, long ld_logits, const float* logits2,
                       float w1, float w2, const int64_t* xt, const int64_t* tnode, int t_const, const int* d_t,
                       const float* noise,
                       const float* q1, const float* qm, int64_t* out, uint64_t seed, int64_t node_base,
                       hipStream_t s, int* bad = nullptr);  // bad: see k_d3pm (caller indices checked)

}  // namespace chm

