// Host runtime + C ABI (include/chemeleon_hip.h) of the Chemeleon sampling path.
//
// chm_model  : packed device copy of the CSPNet decoder weights.
// chm_batch  : one (ragged) batch of crystals: index tables of the implicit
//              fully connected edge layout + the decoder workspace, all
//              allocated once at creation. Decoder calls and sampler steps
//              allocate nothing, synchronise nothing and are capturable.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/chemeleon_hip.h"
#include "chm_internal.h"

using namespace chm;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
// (for the host-only entry points of other translation units, host_noise.cpp)
int chm_fail_host(int code, const char* msg) { return fail(code, msg); }

#define HIPCHK(expr)                                                                         \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      return fail(CHM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));             \
  } while (0)

struct LayerW {
  const float *WAB, *Wcl, *b1, *D, *W2, *b2, *W3, *b3, *W4, *b4, *lw, *lb;
  const void *WAB3, *D3, *W23, *W33, *W43;  // bf16 hi/mid/lo planes of the GEMM weights
  void* D2h;                                 // fp16 hi/lo split rows of the edge-GEMM weights (row-scaled)
  void* W22h16;                              // W2's split rows with k_edge16's K permutation (perm 2)
  float *Dsc, *W2sc;                         // their per-row power-of-two scales
  void *WAB16, *W316, *W416;                 // split16 node GEMMs: fp16 hi/lo rows, 16-column chunks
  float *WABsc, *W3sc, *W4sc;                // (row-scaled like D2h)
};

enum MathMode { MATH_BF16X3 = 0, MATH_F32 = 1, MATH_SPLIT16 = 2 };
constexpr long kTileRows = 256;  // rows of the edge-GEMM tiles (gemm_bf16x3_big)
constexpr int kMaxTailTiles = 512;  // layer-1 row tiles of a partial round (< CUs / 2)
// k_edge16_layer only from 256 row tiles (32 per XCD) on: 64x20 (100 row tiles, 12-13 per XCD, mostly
// inside the layer-2 lag) measured 0.186 vs 0.176 ms for the two launches; 64x40 (400) gains 5%
constexpr long kLayerMinTiles = 256;
constexpr int kMaxLag = 1000;
// the persistent one-grid kernel from this many row tiles on (same-box A/B, profiles/r3/ab_*: 512x40 (3200)
// 60.2 -> 59.2 ms per step; 64x40 (400) 8.34 -> 8.44: the per-job atomic costs more than the XCD
// balancing gains in a short grid)
constexpr long kDynMinTiles = 1024;  // edge_lag's upper bound (sizes the persistent one-grid kernel's row slots)

struct chm_model {
  chm_dims d;
  float* mem = nullptr;
  size_t mem_floats = 0;
  const float *emb, *Wc, *bc, *Wp, *bp, *fw, *fb, *Whead, *bhead, *Wlat, *flw, *flb;
  const void *Wc3, *Wp3, *Whead3;
  void* mem3 = nullptr;  // bf16 planes arena
  void* mem2 = nullptr;  // fp16 planes + scales arena
  void* mem16 = nullptr; // split16 node-GEMM weights arena
  const void* Wp16 = nullptr;
  float* Wpsc = nullptr;
  int math = MATH_SPLIT16;
  int edge_dbg = 0;      // CHM_EDGE_DBG: edge-GEMM ablations for profiling only (wrong results)
  int node_glds = 1;     // CHM_NODE_GLDS=0: node GEMMs on the register-staged k_gemm3 (bit-identical, 2-3% slower)
  int node16 = 1;        // CHM_NODE16=0: split16 mode keeps its node GEMMs on bf16x3
  int node_ps = 0;       // CHM_NODE_PS=1: split16 node GEMMs read their A operands pre-split by the producing
                         // kernels instead of splitting them in the K loop (r4; measured 0.5% slower per step,
                         // DESIGN.md §4 "Node GEMMs")
  int edge_stagger = 0;  // CHM_EDGE_STAGGER: first-round start delay of every other CU (edge16.hip)
  int edge_split = 1;    // CHM_EDGE_SPLIT=0: no partial-round tail split of edge layer 1 (see run_decoder)
  int edge_rows = 1;     // CHM_EDGE_ROWS=0: edge layer 2 on node-aligned segment tiles instead of row tiles
  int edge_layer = 1;    // CHM_EDGE_LAYER=0: edge layers 1 and 2 as two launches (else one grid, k_edge16_layer)
  int edge_lag = 8;      // CHM_EDGE_LAG: its layer-2 lag behind layer 1, in row tiles per XCD (pair grid: pair tiles; r6: 8)
  long edge_layer_min = kLayerMinTiles;  // CHM_EDGE_LAYER_MIN: row tiles from which the one-grid kernel runs
  int edge_dyn = 1;      // CHM_EDGE_DYN: one-grid kernel form, 0 static block -> job map (k_edge16_layer), 1 the
                         // persistent form (k_edge16_layer_dyn) from kDynMinTiles row tiles on, 2 always persistent
  int edge_pool = 15;    // CHM_EDGE_POOL: the persistent form's run-time-claimed share of the row tiles (%)
  int edge_pairs = 1;    // CHM_EDGE_PAIRS / option edge_pairs: fc edge layer 1 on unordered pairs (k_edge16_pairs:
                         // half its matrix work; both directions' S from one GEMM row), then edge layer 2
  int edge_pairs_layer = 1;  // CHM_EDGE_PAIRS_LAYER / option edge_pairs_layer: both edge layers on pairs in one
                             // static grid (k_edge16_pairs_grid) from edge_layer_min row tiles on; 0 = two launches
  int edge_rows_short = 1;   // CHM_EDGE_ROWS_SHORT / option edge_rows_short: batches below edge_layer_min row tiles whose
                             // last round of 256-row tiles is at most 3/4 full take that round as 192-row tiles
                             // (short_row_tiles, set at batch creation; bit-identical)
  int ncu = 0;          // compute units of the device the model lives on
  int device = 0;        // its HIP device ordinal (the current device at chm_model_create)
  unsigned xcd_mask = 0; // XCC ids a grid's blocks ran on at model creation (the persistent edge kernel needs 0xff)
  int edge_skip_xcd = -1;  // (tests) option edge_dyn_skip_xcd: the persistent kernel's blocks on that XCD exit
  int repair_grid = 0;   // CHM_REPAIR_GRID: blocks of the edge kernels' repair launches (default: ncu)
  int film = 1;          // 0: time_dim = text_dim = 0 (no FilmLayer: the CrystalClip graph encoder)
  const char* edge_trace = nullptr;  // CHM_EDGE_TRACE=file: one edge-GEMM launch's block timeline
  int edge_trace_layer = 1;          // CHM_EDGE_TRACE_LAYER: 1 or 2 (two-launch schedule), 3 (k_edge16_layer), 4 (pair grid)
  std::vector<LayerW> layers;
};

struct chm_batch {
  const chm_model* m;
  int B, P;
  long N, E;
  std::vector<int> h_natoms;
  // index tables
  int *natoms, *node_off, *n2g, *ei, *ej;
  long *edge_off, *node_estart;
  int* node_n;  // atom count of each node's crystal
  // fc: the unordered pairs (i <= j) of every crystal for edge layer 1 on pairs (BatchTables::pi / pj / pe)
  int *pi = nullptr, *pj = nullptr;
  int2* pe = nullptr;
  int2* pnode = nullptr;  // per pair tile: the node range of its P / Q rows (EdgeArgs::pnode)
  long Ep = 0;
  // fc, split16: the job lists of both edge layers in one static grid on pairs (k_edge16_pairs_grid), built for
  // P = max_pairs and the model's edge_lag at creation; per layer 8 npx pair-tile flags (psched)
  PairPlan pplan;
  int4* pjobs = nullptr;  // the pair grid's block records (PairSched::jobs)
  unsigned* psched = nullptr;
  int2* tiles;  // node ranges [x, y) whose edge rows fit one 256-row GEMM tile
  int ntiles;
  // fc batches: edge layer 2 (k_edge16) on row tiles of exactly 256 edge rows, nodes cut at the tile
  // ends (EdgeArgs::rtiles); null for knn batches
  int4* rtiles = nullptr;
  int2* rinfo = nullptr;    // per row tile: its node list (EdgeArgs::rinfo), and its length
  int* rinfo_n = nullptr;
  long nrt = 0, r2tot = 0;  // row tiles; rows of the nodes continued from a previous tile
  // a mixed row tiling (short_row_tiles): tiles [0, rt_nbig) have 256 rows, the rest kShortRows; -1 = all 256
  long rt_nbig = -1;
  float *sbuf = nullptr, *msgbuf = nullptr;
  unsigned* rcnt = nullptr;
  unsigned* lflags = nullptr;  // k_edge16_layer: per row tile (returns to 0 at the end of every launch)
  unsigned* xbad = nullptr;    // k_edge16_layer: per layer, raised when its repair launches must run
  unsigned* sched = nullptr;   // k_edge16_layer_dyn: per layer 16 + 8 * sched_cap words, zeroed per decoder call
  long sched_cap = 0;
  int math;     // arithmetic mode fixed at creation (copied from the model)
  // workspace
  float *cin, *cemb, *Hres, *Hl, *Y, *agg, *PQ, *gbias, *F, *S, *M, *Hf, *HO, *LAT;
  float* rmx;        // split16 node GEMMs: the four row-max arrays [4][P*N] (RMX_*)
  // split16 pre-split node GEMMs (node_ps): the node GEMMs' A operands as split rows [P*N][H/16][hi 16 | lo 16]
  // fp16 + per row the packed int8 exponents of its four 128-column chunks: the residual stream (FiLM
  // projection), the layer-normed rows (P / Q halves, node MLP 1), agg (node MLP 1), U (node MLP 2)
  void *Hs, *Hls, *aggs, *Us;
  int *He, *Hle, *agge, *Ue;
  unsigned* rowmax;  // split16: per S row, the packed int8 exponents of its four 128-column chunks, [P][E]
  void* owned = nullptr;  // the library's own allocation (chm_batch_create); null for caller workspaces
  size_t bytes = 0;
  // edge layer 1's partial last round (split16 / k_edge16, see run_decoder): rows [0, l1_rows_a) fill
  // whole rounds of the grid; the rest runs in one grid with edge layer 2, whose segment tiles from
  // l2_tile_a on read those rows. 0 = no split.
  long l1_rows_a = 0;
  int l2_tile_a = 0;
  unsigned* tail_flags = nullptr;  // [kMaxTailTiles] per layer-1 row tile of the partial round
  // knn (radius-graph) batches: edges rebuilt every decoder call (knn.hip); E is then the current
  // graph's edge count and E_cap the capacity the edge buffers are sized for
  int knn = 0, knn_max_nb = 20;
  long E_cap = 0, C_cap = 0;
  long* cand_off = nullptr;
  unsigned *cand_key = nullptr, *cand2 = nullptr, *fin_key = nullptr;
  float *cand_d2 = nullptr, *fin_fd = nullptr, *fd = nullptr;
  int *atom_cnt = nullptr, *deg = nullptr, *cryst_fin = nullptr;
  std::vector<int> h_deg, h_fin;
  std::vector<long> h_estart;
  std::vector<int2> h_tiles;
};

extern "C" const char* chm_last_error(void) { return g_err.c_str(); }
extern "C" const char* chm_version(void) { return "chemeleon-mi355x 0.3 (gfx950; split16 / bf16x3 / f32 MFMA)"; }

// (time_dim = text_dim = 0: a CSPNet without FilmLayer, cspnet.py:210-211, e.g. CrystalClip's graph encoder)
static bool film_less(const chm_dims* d) { return d->time_dim == 0 && d->text_dim == 0; }
extern "C" int chm_num_params(const chm_dims* d) { return d ? (film_less(d) ? 1 : 7) + 10 * d->num_layers + 6 : 0; }

static int check_dims(const chm_dims* d) {
  if (!d) return fail(CHM_E_ARG, "dims is NULL");
  if (d->hidden_dim != H) return fail(CHM_E_UNSUPPORTED, "hidden_dim must be 512 in this build");
  if (d->num_freqs != NF) return fail(CHM_E_UNSUPPORTED, "num_freqs must be 128 in this build");
  if (d->time_dim != TD && !film_less(d))
    return fail(CHM_E_UNSUPPORTED, "time_dim must be 128 in this build (or time_dim = text_dim = 0)");
  if (d->text_dim < 0 || (TD + d->text_dim) % 16) return fail(CHM_E_UNSUPPORTED, "time_dim + text_dim must be a multiple of 16");
  if (d->max_atoms < 1 || d->max_atoms + 3 > HEADS_N) return fail(CHM_E_UNSUPPORTED, "max_atoms must be in [1, 125]");
  if (d->num_layers < 1 || d->num_layers > kMaxLayers) return fail(CHM_E_ARG, "num_layers out of range");
  return CHM_OK;
}

extern "C" int chm_model_create(const chm_dims* dims, const float* const* p, int n_params, void* stream,
                                chm_model** out) {
  if (!out) return fail(CHM_E_ARG, "out is NULL");
  *out = nullptr;
  int rc = check_dims(dims);
  if (rc) return rc;
  if (n_params != chm_num_params(dims)) return fail(CHM_E_ARG, "wrong number of parameter tensors");
  for (int i = 0; i < n_params; ++i)
    if (!p[i]) return fail(CHM_E_ARG, "parameter pointer " + std::to_string(i) + " is NULL");
  hipStream_t s = (hipStream_t)stream;
  const int A = dims->max_atoms, L = dims->num_layers, X = dims->text_dim;
  const bool film = !film_less(dims);
  const int CIN = film ? TD + X : 0, W1K = 2 * H + 9 + FD;
  const int PL = film ? 7 : 1;  // first layer parameter
  {
    hipError_t e0 = gemm_init();
    if (e0 == hipSuccess) e0 = edge16_init();
    if (e0 == hipSuccess) e0 = node_gemm_init();
    if (e0 != hipSuccess) return fail(CHM_E_HIP, std::string("gemm_init: ") + hipGetErrorString(e0));
  }

  // layout of the packed arena (each piece 256-byte aligned)
  size_t off = 0;
  auto take = [&](size_t n) { size_t o = off; off += (n + 63) / 64 * 64; return o; };
  const size_t o_emb = take((size_t)A * H), o_Wc = take((size_t)2 * H * CIN), o_bc = take(2 * H), o_Wp = take(H * H),
               o_bp = take(H), o_fw = take(H), o_fb = take(H);
  std::vector<size_t> lo(L * 12);
  for (int l = 0; l < L; ++l) {
    lo[l * 12 + 0] = take((size_t)2 * H * H);  // WAB
    lo[l * 12 + 1] = take((size_t)H * 9);      // Wcl
    lo[l * 12 + 2] = take(H);                  // b1
    lo[l * 12 + 3] = take((size_t)H * FD);     // D
    lo[l * 12 + 4] = take((size_t)H * H);      // W2
    lo[l * 12 + 5] = take(H);                  // b2
    lo[l * 12 + 6] = take((size_t)H * 2 * H);  // W3
    lo[l * 12 + 7] = take(H);                  // b3
    lo[l * 12 + 8] = take((size_t)H * H);      // W4
    lo[l * 12 + 9] = take(H);                  // b4
    lo[l * 12 + 10] = take(H);                 // lw
    lo[l * 12 + 11] = take(H);                 // lb
  }
  const size_t o_Wh = take((size_t)HEADS_N * H), o_bh = take(HEADS_N), o_Wl = take(9 * H), o_flw = take(H),
               o_flb = take(H);

  chm_model* m = new chm_model();
  m->d = *dims;
  m->film = film;
  m->mem_floats = off;
  hipError_t e = hipMalloc(&m->mem, off * sizeof(float));
  if (e != hipSuccess) {
    delete m;
    return fail(CHM_E_HIP, std::string("hipMalloc(model): ") + hipGetErrorString(e));
  }
  float* base = m->mem;
  auto cp = [&](size_t o, const float* src, size_t n) {
    return hipMemcpyAsync(base + o, src, n * sizeof(float), hipMemcpyDeviceToDevice, s);
  };
  // 2-D copy of a column block of a row-major [rows][src_ld] matrix
  auto cp2 = [&](size_t o, size_t dst_ld, const float* src, size_t src_ld, size_t col0, size_t cols, size_t rows) {
    return hipMemcpy2DAsync(base + o, dst_ld * sizeof(float), src + col0, src_ld * sizeof(float), cols * sizeof(float),
                            rows, hipMemcpyDeviceToDevice, s);
  };
#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t _e = (x);                                                                       \
    if (_e != hipSuccess) {                                                                    \
      (void)hipFree(m->mem);                                                                   \
      delete m;                                                                                \
      return fail(CHM_E_HIP, std::string("weight packing: ") + hipGetErrorString(_e));         \
    }                                                                                          \
  } while (0)
  CK(hipMemsetAsync(base, 0, off * sizeof(float), s));
  CK(cp(o_emb, p[0], (size_t)A * H));
  if (film) {  // (film-less: the FiLM arena stays zero and is never read)
    CK(cp(o_Wc, p[1], (size_t)2 * H * CIN));
    CK(cp(o_bc, p[2], 2 * H));
    CK(cp(o_Wp, p[3], H * H));
    CK(cp(o_bp, p[4], H));
    CK(cp(o_fw, p[5], H));
    CK(cp(o_fb, p[6], H));
  }
  for (int l = 0; l < L; ++l) {
    const float* const* q = p + PL + 10 * l;
    // edge_mlp.0.weight [H][2H+9+FD] -> WAB = [W1[:, 0:H] ; W1[:, H:2H]], Wcl = W1[:, 2H:2H+9], D = W1[:, 2H+9:]
    CK(cp2(lo[l * 12 + 0], H, q[0], W1K, 0, H, H));
    CK(cp2(lo[l * 12 + 0] + (size_t)H * H, H, q[0], W1K, H, H, H));
    CK(cp2(lo[l * 12 + 1], 9, q[0], W1K, 2 * H, 9, H));
    CK(cp2(lo[l * 12 + 3], FD, q[0], W1K, 2 * H + 9, FD, H));
    CK(cp(lo[l * 12 + 2], q[1], H));
    CK(cp(lo[l * 12 + 4], q[2], (size_t)H * H));
    CK(cp(lo[l * 12 + 5], q[3], H));
    CK(cp(lo[l * 12 + 6], q[4], (size_t)H * 2 * H));
    CK(cp(lo[l * 12 + 7], q[5], H));
    CK(cp(lo[l * 12 + 8], q[6], (size_t)H * H));
    CK(cp(lo[l * 12 + 9], q[7], H));
    CK(cp(lo[l * 12 + 10], q[8], H));
    CK(cp(lo[l * 12 + 11], q[9], H));
  }
  const float* const* hq = p + PL + 10 * L;  // coord_out.w, lattice_out.w, type_out.w, type_out.b, final_ln.w, final_ln.b
  CK(cp(o_Wh, hq[2], (size_t)A * H));                 // rows 0..A-1: type_out
  CK(cp(o_Wh + (size_t)A * H, hq[0], (size_t)3 * H)); // rows A..A+2: coord_out
  CK(cp(o_bh, hq[3], A));
  CK(cp(o_Wl, hq[1], 9 * H));
  CK(cp(o_flw, hq[4], H));
  CK(cp(o_flb, hq[5], H));
  CK(hipStreamSynchronize(s));
#undef CK
  m->emb = base + o_emb; m->Wc = base + o_Wc; m->bc = base + o_bc; m->Wp = base + o_Wp; m->bp = base + o_bp;
  m->fw = base + o_fw; m->fb = base + o_fb; m->Whead = base + o_Wh; m->bhead = base + o_bh; m->Wlat = base + o_Wl;
  m->flw = base + o_flw; m->flb = base + o_flb;
  m->layers.resize(L);
  for (int l = 0; l < L; ++l) {
    LayerW& w = m->layers[l];
    const size_t* o = &lo[l * 12];
    w.WAB = base + o[0]; w.Wcl = base + o[1]; w.b1 = base + o[2]; w.D = base + o[3]; w.W2 = base + o[4];
    w.b2 = base + o[5]; w.W3 = base + o[6]; w.b3 = base + o[7]; w.W4 = base + o[8]; w.b4 = base + o[9];
    w.lw = base + o[10]; w.lb = base + o[11];
  }
  // bf16x3 planes of every GEMM weight (fp32-accurate bf16 MFMA path)
  {
    const char* env = getenv("CHM_MATH");
    const std::string mode = env ? env : "";
    m->math = mode == "f32" ? MATH_F32 : mode == "bf16x3" ? MATH_BF16X3 : MATH_SPLIT16;
    const char* dbg = getenv("CHM_EDGE_DBG");
    m->edge_dbg = dbg ? atoi(dbg) : 0;
    const char* ng = getenv("CHM_NODE_GLDS");
    if (ng) m->node_glds = atoi(ng);
    const char* n16 = getenv("CHM_NODE16");
    if (n16) m->node16 = atoi(n16);
    const char* nps = getenv("CHM_NODE_PS");
    if (nps) m->node_ps = atoi(nps);
    m->edge_trace = getenv("CHM_EDGE_TRACE");
    const char* tl = getenv("CHM_EDGE_TRACE_LAYER");
    if (tl) m->edge_trace_layer = atoi(tl);
    const char* stg = getenv("CHM_EDGE_STAGGER");
    if (stg) m->edge_stagger = atoi(stg);
    const char* spl = getenv("CHM_EDGE_SPLIT");
    if (spl) m->edge_split = atoi(spl);
    const char* rows = getenv("CHM_EDGE_ROWS");
    if (rows) m->edge_rows = atoi(rows);
    const char* lay = getenv("CHM_EDGE_LAYER");
    if (lay) m->edge_layer = atoi(lay);
    const char* lag = getenv("CHM_EDGE_LAG");
    if (lag) m->edge_lag = atoi(lag) > 0 ? atoi(lag) : 1;
    const char* lmin = getenv("CHM_EDGE_LAYER_MIN");
    if (lmin) m->edge_layer_min = atol(lmin);
    const char* rg = getenv("CHM_REPAIR_GRID");
    if (rg) m->repair_grid = atoi(rg);
    const char* dyn = getenv("CHM_EDGE_DYN");
    if (dyn) m->edge_dyn = atoi(dyn);
    const char* pool = getenv("CHM_EDGE_POOL");
    if (pool) m->edge_pool = atoi(pool);
    const char* pairs = getenv("CHM_EDGE_PAIRS");
    if (pairs) m->edge_pairs = atoi(pairs);
    const char* player = getenv("CHM_EDGE_PAIRS_LAYER");
    if (player) m->edge_pairs_layer = atoi(player);
    const char* rshort = getenv("CHM_EDGE_ROWS_SHORT");
    if (rshort) m->edge_rows_short = atoi(rshort);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&m->ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      m->ncu = 0;
    m->device = dev;
    // k_edge16_layer_dyn gives each of 8 XCDs static rows: on a device or partition mode with fewer XCDs
    // it would leave rows to its self-check and repair launches, so it runs only where 8 were seen
    if (m->ncu > 0 && xcd_mask(8 * m->ncu, &m->xcd_mask) != hipSuccess) m->xcd_mask = 0;
    struct Job { const float* src; size_t n; const void** dst; };
    std::vector<Job> jobs;
    jobs.push_back({m->Wc, (size_t)2 * H * CIN, &m->Wc3});
    jobs.push_back({m->Wp, (size_t)H * H, &m->Wp3});
    jobs.push_back({m->Whead, (size_t)HEADS_N * H, &m->Whead3});
    for (auto& w : m->layers) {
      jobs.push_back({w.WAB, (size_t)2 * H * H, &w.WAB3});
      jobs.push_back({w.D, (size_t)H * FD, &w.D3});
      jobs.push_back({w.W2, (size_t)H * H, &w.W23});
      jobs.push_back({w.W3, (size_t)H * 2 * H, &w.W33});
      jobs.push_back({w.W4, (size_t)H * H, &w.W43});
    }
    size_t total = 0;
    for (auto& j : jobs) total += (3 * j.n * 2 + 255) / 256 * 256;
    hipError_t e2 = hipMalloc(&m->mem3, total);
    if (e2 != hipSuccess) {
      (void)hipFree(m->mem);
      delete m;
      return fail(CHM_E_HIP, std::string("hipMalloc(planes): ") + hipGetErrorString(e2));
    }
    char* p3 = (char*)m->mem3;
    for (auto& j : jobs) {
      *j.dst = p3;
      hipError_t e3 = j.n ? split_planes(j.src, (long)j.n, p3, s) : hipSuccess;  // (film-less: no Wc)
      if (e3 != hipSuccess) {
        (void)hipFree(m->mem); (void)hipFree(m->mem3);
        delete m;
        return fail(CHM_E_HIP, std::string("split_planes: ") + hipGetErrorString(e3));
      }
      p3 += (3 * j.n * 2 + 255) / 256 * 256;
    }
    // fp16 hi/lo planes (+ row scales) of the two edge-GEMM weights of every layer
    const size_t per_layer = (2 * (size_t)H * FD * 2 + 2 * (size_t)H * H * 2 + 2 * H * 4 + 1023) / 1024 * 1024;
    e2 = hipMalloc(&m->mem2, per_layer * L);
    for (int l = 0; l < L && e2 == hipSuccess; ++l) {
      char* q = (char*)m->mem2 + per_layer * l;
      LayerW& w = m->layers[l];
      w.D2h = q;
      w.W22h16 = q + 2 * (size_t)H * FD * 2;
      w.Dsc = (float*)(q + 2 * (size_t)H * FD * 2 + 2 * (size_t)H * H * 2);
      w.W2sc = w.Dsc + H;
      e2 = split_rows_h(w.D, H, FD, w.D2h, w.Dsc, 0, s);
      if (e2 == hipSuccess) e2 = split_rows_h(w.W2, H, H, w.W22h16, w.W2sc, 2, s);  // (k_edge16's S layout)
    }
    // fp16 hi/lo rows (16-column chunks, + row scales) of the node-GEMM weights (split16 node GEMMs)
    if (e2 == hipSuccess) {
      struct J16 { const float* src; int n, k; void** dst; float** sc; };
      std::vector<J16> j16;
      void* wp16 = nullptr;
      j16.push_back({m->Wp, H, H, &wp16, &m->Wpsc});
      for (auto& w : m->layers) {
        j16.push_back({w.WAB, 2 * H, H, &w.WAB16, &w.WABsc});
        j16.push_back({w.W3, H, 2 * H, &w.W316, &w.W3sc});
        j16.push_back({w.W4, H, H, &w.W416, &w.W4sc});
      }
      auto sz = [](const J16& j) { return ((size_t)j.n * j.k * 4 + 255) / 256 * 256 + ((size_t)j.n * 4 + 255) / 256 * 256; };
      size_t tot = 0;
      for (auto& j : j16) tot += sz(j);
      e2 = hipMalloc(&m->mem16, tot);
      char* q = (char*)m->mem16;
      for (auto& j : j16) {
        if (e2 != hipSuccess) break;
        *j.dst = q;
        *j.sc = (float*)(q + ((size_t)j.n * j.k * 4 + 255) / 256 * 256);
        e2 = split_rows_h(j.src, j.n, j.k, *j.dst, *j.sc, 0, s, 16);
        q += sz(j);
      }
      m->Wp16 = wp16;
    }
    if (e2 == hipSuccess) e2 = hipStreamSynchronize(s);
    if (e2 != hipSuccess) {
      (void)hipFree(m->mem); (void)hipFree(m->mem3); (void)hipFree(m->mem2); (void)hipFree(m->mem16);
      delete m;
      return fail(CHM_E_HIP, std::string("plane split: ") + hipGetErrorString(e2));
    }
  }
  *out = m;
  return CHM_OK;
}

extern "C" int chm_model_set_math(chm_model* m, int mode) {
  if (!m) return fail(CHM_E_ARG, "model is NULL");
  if (mode != CHM_MATH_BF16X3 && mode != CHM_MATH_F32 && mode != CHM_MATH_SPLIT16)
    return fail(CHM_E_ARG, "unknown math mode");
  m->math = mode;
  return CHM_OK;
}

extern "C" int chm_model_get_math(const chm_model* m) { return m ? m->math : -1; }

extern "C" int chm_model_set_option(chm_model* m, const char* key, int64_t value) {
  if (!m || !key) return fail(CHM_E_ARG, "NULL argument");
  const std::string k = key;
  if (k == "node_ps") {  // split16 node GEMMs read pre-split A operands (1) or split them in the K loop (0)
    m->node_ps = value != 0;
    return CHM_OK;
  }
  if (k == "edge_split") {
    m->edge_split = value != 0;
    return CHM_OK;
  }
  if (k == "edge16") {  // (the round-1 32x32x16 edge kernels were removed in round 3)
    if (value == 0) return fail(CHM_E_UNSUPPORTED, "edge16 = 0: the 32x32x16 edge kernels were removed");
    return CHM_OK;
  }
  if (k == "edge_rows") {  // edge layer 2 on 256-row tiles (fc batches) or node-aligned tiles; bit-identical
    m->edge_rows = value != 0;
    return CHM_OK;
  }
  if (k == "edge_layer") {  // both edge layers in one grid (fc batches, row tiles); bit-identical
    m->edge_layer = value != 0;
    return CHM_OK;
  }
  if (k == "edge_layer_dyn") {  // persistent one-grid kernel: 0 never, 1 from kDynMinTiles row tiles on, 2 always
    if (value < 0 || value > 2) return fail(CHM_E_ARG, "edge_layer_dyn must be 0, 1 or 2");
    m->edge_dyn = (int)value;
    return CHM_OK;
  }
  if (k == "edge_dyn_skip_xcd") {  // (tests) the persistent kernel's blocks on XCD `value` exit at once (-1: none)
    if (value < -1 || value > 7) return fail(CHM_E_ARG, "edge_dyn_skip_xcd must be in [-1, 7]");
    m->edge_skip_xcd = (int)value;
    return CHM_OK;
  }
  if (k == "xcd_mask") {  // (tests) override the XCD mask probed at creation
    m->xcd_mask = (unsigned)value;
    return CHM_OK;
  }
  if (k == "edge_layer_min") {  // row tiles from which both edge layers run in one grid (default 256)
    if (value < 1) return fail(CHM_E_ARG, "edge_layer_min must be >= 1");
    m->edge_layer_min = (long)value;
    return CHM_OK;
  }
  if (k == "edge_pool") {  // its run-time-claimed share of the row tiles, percent (0: static rows only)
    if (value < 0 || value > 100) return fail(CHM_E_ARG, "edge_pool must be in [0, 100]");
    m->edge_pool = (int)value;
    return CHM_OK;
  }
  if (k == "edge_pairs") {  // fc edge layer 1 on unordered pairs (k_edge16_pairs), then edge layer 2 (within fp32
                            // rounding of the directed edges: DESIGN.md §4 "Edge layer 1 on pairs")
    m->edge_pairs = value != 0;
    return CHM_OK;
  }
  if (k == "edge_pairs_layer") {  // both edge layers on pairs in one static grid (k_edge16_pairs_grid): 1 on, 0 off
    m->edge_pairs_layer = value != 0;
    return CHM_OK;
  }
  if (k == "edge_rows_short") {  // short last-round row tiles for the batches created from now on (bit-identical)
    m->edge_rows_short = value != 0;
    return CHM_OK;
  }
  if (k == "edge_lag") {
    if (value < 1 || value > kMaxLag) return fail(CHM_E_ARG, "edge_lag must be in [1, 1000]");
    m->edge_lag = (int)value;
    return CHM_OK;
  }
  if (k == "edge_layer_repair") {  // (tests) k_edge16_layer always runs its repair launches
    m->edge_dbg = value ? (m->edge_dbg | 512) : (m->edge_dbg & ~512);
    return CHM_OK;
  }
  if (k == "edge_tail_timeout") {  // (tests) k_edge16_tail's waits time out (producers delayed), repaired
    m->edge_dbg = value ? (m->edge_dbg | 8192) : (m->edge_dbg & ~8192);
    return CHM_OK;
  }
  if (k == "edge_tail_norepair") {  // (tests; WRONG results after a timeout) no repair launches behind the tail
    m->edge_dbg = value ? (m->edge_dbg | 16384) : (m->edge_dbg & ~16384);
    return CHM_OK;
  }
  if (k == "edge_pairs_pq_global") {  // (tests) the pair epilogue reads its P / Q rows from global memory (no LDS staging)
    m->edge_dbg = value ? (m->edge_dbg | 1048576) : (m->edge_dbg & ~1048576);
    return CHM_OK;
  }
  if (k == "edge_rows_nowait") {  // (tests) row tiles never wait for the previous tile: the msgbuf path
    m->edge_dbg = value ? (m->edge_dbg | 64) : (m->edge_dbg & ~64);
    return CHM_OK;
  }
  return fail(CHM_E_ARG, "unknown option: " + k);
}

extern "C" void chm_model_destroy(chm_model* m) {
  if (!m) return;
  (void)hipFree(m->mem);
  (void)hipFree(m->mem3);
  (void)hipFree(m->mem2);
  (void)hipFree(m->mem16);
  delete m;
}

// Host-side index tables of a batch (the implicit fc edge layout) and the byte layout of its
// device memory: index tables first, then the decoder workspace, each piece 256-byte aligned.
// The same carve() sequence sizes the block (base == null) and binds a batch to it.
struct BatchOpts {
  int knn = 0, max_nb = 20, per_atom = 128;
};

static int batch_opts(const chm_batch_options* o, BatchOpts& bo) {
  if (!o) return CHM_OK;
  if (o->edge_style != CHM_EDGES_FC && o->edge_style != CHM_EDGES_KNN) return fail(CHM_E_ARG, "unknown edge_style");
  bo.knn = o->edge_style == CHM_EDGES_KNN;
  bo.max_nb = o->max_neighbors;  // <= 0: no neighbour cap (get_max_neighbors_mask, data_utils.py:341-348)
  if (o->knn_edges_per_atom) bo.per_atom = o->knn_edges_per_atom;
  if (bo.per_atom < 1 || bo.per_atom > 4096) return fail(CHM_E_ARG, "knn_edges_per_atom out of range");
  return CHM_OK;
}

struct BatchTables {
  std::vector<int> nat, noff, n2g, ei, ej, nn;
  std::vector<long> eoff, estart, coff;
  std::vector<int2> tiles;
  std::vector<int4> rtiles;  // fc: row tiles of edge layer 2 (EdgeArgs::rtiles)
  std::vector<int2> rinfo;   // fc: the row tiles' node lists (EdgeArgs::rinfo, kRowInfo per tile)
  std::vector<int> rinfo_n;
  long nrt = 0, r2tot = 0;
  long rt_nbig = -1;  // fc: 256-row tiles before the kShortRows ones (-1: all 256 rows; set before batch_fill)
  long N = 0, E = 0;  // knn: E = the edge capacity
  // fc: the unordered pairs i <= j of every crystal, row-major (edge layer 1 on pairs, k_edge16_pairs)
  std::vector<int> pi, pj;
  std::vector<int2> pe, pnode;
  long Ep = 0;
  long C = 0;         // knn: candidate scratch entries (sum of n^2 * 27)
  bool knn = false;
};

static int batch_tables(const int32_t* h_natoms, int B, BatchTables& t, const BatchOpts& bo = BatchOpts()) {
  t.nat.assign(h_natoms, h_natoms + B);
  t.noff.assign(B + 1, 0);
  t.eoff.assign(B + 1, 0);
  long N = 0, E = 0;
  for (int g = 0; g < B; ++g) {
    if (t.nat[g] < 1) return fail(CHM_E_ARG, "every crystal needs at least one atom");
    if (t.nat[g] > kTileRows) return fail(CHM_E_UNSUPPORTED, "crystals above 256 atoms are not supported");
    t.noff[g] = (int)N;
    t.eoff[g] = E;
    N += t.nat[g];
    E += (long)t.nat[g] * t.nat[g];
    t.Ep += (long)t.nat[g] * (t.nat[g] + 1) / 2;
    if (N > (1L << 30) || E > (1L << 31) - 1) return fail(CHM_E_ARG, "batch too large");
  }
  t.noff[B] = (int)N;
  t.eoff[B] = E;
  t.N = N;
  t.E = E;
  t.knn = bo.knn;
  if (bo.knn) {  // radius graph: candidates n^2 * 27 per crystal, edges up to per_atom per atom
    t.coff.assign(B + 1, 0);
    for (int g = 0; g < B; ++g) t.coff[g + 1] = t.coff[g] + (long)t.nat[g] * t.nat[g] * 27;
    t.C = t.coff[B];
    t.E = N * (long)bo.per_atom;
    if (t.E > (1L << 31) - 1) return fail(CHM_E_ARG, "batch too large");
  }
  return CHM_OK;
}

// Row-tile geometry: tiles [0, nbig) of 256 rows, then tiles of kShortRows (nbig < 0: all 256 rows)
static long rt_count(long E, long nbig) {
  return nbig < 0 ? (E + kTileRows - 1) / kTileRows : nbig + (E - nbig * kTileRows + kShortRows - 1) / kShortRows;
}
static long rt_start(long k, long nbig) {
  return nbig < 0 || k <= nbig ? k * kTileRows : nbig * kTileRows + (k - nbig) * kShortRows;
}

// Row tiles of an fc batch (edge rows grouped by source node; node v's rows [estart, estart + n)):
// tile t = rows [256 t, 256 t + 256) (a mixed tiling: rt_start), {first node starting in it, first node starting
// after it, the node that began in tile t-1 and continues here (-1: none), the offset of those continued rows in
// msgbuf}. Returns the continued rows' total (msgbuf rows per conditioning); out null: sizing only.
static long row_tiles(const BatchTables& t, std::vector<int4>* out) {
  const long E = t.E, nrt = rt_count(E, t.rt_nbig), nb = t.rt_nbig;
  if (out) out->assign(nrt, make_int4((int)t.N, (int)t.N, -1, 0));
  long r2tot = 0, tc = 0, node = 0;
  long prev_end = 0;  // end row of the previous node
  for (size_t g = 0; g < t.nat.size(); ++g)
    for (int i = 0; i < t.nat[g]; ++i, ++node) {
      const long es = t.eoff[g] + (long)i * t.nat[g];
      for (; tc < nrt && rt_start(tc, nb) <= es; ++tc) {  // tiles starting in (previous start, es]
        const long s0 = rt_start(tc, nb);
        int4 r = make_int4((int)node, (int)t.N, -1, 0);
        if (node > 0 && prev_end > s0 && s0 < es) {  // node-1 began before the tile and reaches into it
          r.z = (int)(node - 1);
          r.w = (int)r2tot;
          r2tot += prev_end - s0;
        }
        if (out) (*out)[tc] = r;
      }
      prev_end = es + t.nat[g];
    }
  for (; tc < nrt; ++tc) {  // tiles after the last node start (the last node's rest)
    const long s0 = rt_start(tc, nb);
    int4 r = make_int4((int)t.N, (int)t.N, -1, 0);
    if (prev_end > s0) {
      r.z = (int)(t.N - 1);
      r.w = (int)r2tot;
      r2tot += prev_end - s0;
    }
    if (out) (*out)[tc] = r;
  }
  if (out)
    for (long k = 0; k < nrt; ++k) (*out)[k].y = k + 1 < nrt ? (*out)[k + 1].x : (int)t.N;
  return r2tot;
}

// The node list of every row tile, exactly as edge16.hip's segment-mean epilogue would derive it from
// rtiles / node_estart / node_n: {node, rows in the tile | first row in the tile << 10 | kind << 20},
// kind 0 = a whole node, 1 = the head part of a node cut at the tile end (listed first), 2 = the rest of
// a node begun in the previous tile (listed last). Unused entries are zero.
static void row_tile_nodes(BatchTables& t) {
  const long nrt = (long)t.rtiles.size(), E = t.E;
  t.rinfo.assign((size_t)nrt * kRowInfo, make_int2(0, 0));
  t.rinfo_n.assign(nrt, 0);
  for (long k = 0; k < nrt; ++k) {
    const int4 rt = t.rtiles[k];
    const long e0 = rt_start(k, t.rt_nbig), e1 = std::min<long>(E, rt_start(k + 1, t.rt_nbig));
    const int nreg = rt.y - rt.x;
    const bool head = nreg > 0 && t.estart[rt.y - 1] + t.nn[rt.y - 1] > e1;
    const bool cont = rt.z >= 0;
    const int nn = nreg + (cont ? 1 : 0);
    int2* o = t.rinfo.data() + (size_t)k * kRowInfo;
    for (int i = 0; i < nn; ++i) {
      if (cont && i == nn - 1) {
        o[i] = make_int2(rt.z, (int)(t.estart[rt.z] + t.nn[rt.z] - e0) | (2 << 20));
      } else {
        const int v = rt.x + (head ? (i == 0 ? nreg - 1 : i - 1) : i);
        const long es = t.estart[v], end = es + t.nn[v];
        o[i] = make_int2(v, (int)((end > e1 ? e1 : end) - es) | ((int)(es - e0) << 10) | ((head && i == 0) ? 1 << 20 : 0));
      }
    }
    t.rinfo_n[k] = nn;
  }
}

// fills the per-node / per-edge tables (only when the batch is really built)
static void batch_fill(BatchTables& t) {
  const int B = (int)t.nat.size();
  const long N = t.N, E = t.E;
  t.n2g.resize(N);
  t.nn.resize(N);
  for (int g = 0; g < B; ++g)
    for (int i = 0; i < t.nat[g]; ++i) {
      t.n2g[t.noff[g] + i] = g;
      t.nn[t.noff[g] + i] = t.nat[g];
    }
  if (t.knn) return;  // (edge tables are built per decoder call)
  t.pi.resize(t.Ep);
  t.pj.resize(t.Ep);
  t.pe.resize(t.Ep);
  for (int g = 0, p = 0; g < B; ++g) {
    const int n = t.nat[g], o = t.noff[g];
    for (int i = 0; i < n; ++i)
      for (int j = i; j < n; ++j, ++p) {
        t.pi[p] = o + i;
        t.pj[p] = o + j;
        t.pe[p] = make_int2((int)(t.eoff[g] + (long)i * n + j), (int)(t.eoff[g] + (long)j * n + i));
      }
  }
  // the pair tiles' P / Q node ranges: from the first pair's i (pairs are ordered by crystal, then i <= j, so every
  // node of the tile is >= it) to the end of the crystal of the last pair (every j of the tile is below it)
  t.pnode.resize((t.Ep + kPairRows - 1) / kPairRows);
  for (size_t k = 0; k < t.pnode.size(); ++k) {
    const long p0 = (long)k * kPairRows, p1 = std::min<long>(p0 + kPairRows, t.Ep) - 1;
    const int gl = t.n2g[t.pi[p1]];
    t.pnode[k] = make_int2(t.pi[p0], t.noff[gl] + t.nat[gl] - t.pi[p0]);
  }
  t.ei.resize(E);
  t.ej.resize(E);
  t.estart.resize(N);
  for (int g = 0; g < B; ++g) {
    long e = t.eoff[g];
    for (int i = 0; i < t.nat[g]; ++i)
      for (int j = 0; j < t.nat[g]; ++j, ++e) {
        t.ei[e] = t.noff[g] + i;
        t.ej[e] = t.noff[g] + j;
      }
  }
  // segment tiles: runs of whole nodes whose edge rows fit one 256-row GEMM tile
  int cur0 = 0;
  long rows = 0;
  t.tiles.clear();
  for (int g = 0; g < B; ++g)
    for (int i = 0; i < t.nat[g]; ++i) {
      const int node = t.noff[g] + i;
      t.estart[node] = t.eoff[g] + (long)i * t.nat[g];
      if (rows + t.nat[g] > kTileRows) {
        t.tiles.push_back(make_int2(cur0, node));
        cur0 = node;
        rows = 0;
      }
      rows += t.nat[g];
    }
  t.tiles.push_back(make_int2(cur0, (int)N));
  t.r2tot = row_tiles(t, &t.rtiles);
  t.nrt = (long)t.rtiles.size();
  row_tile_nodes(t);
}

// number of segment tiles without building the tables (sizing only)
static long count_tiles(const BatchTables& t) {
  if (t.knn) return t.N + 1;
  long n = 1, rows = 0;
  for (size_t g = 0; g < t.nat.size(); ++g)
    for (int i = 0; i < t.nat[g]; ++i) {
      if (rows + t.nat[g] > kTileRows) {
        ++n;
        rows = 0;
      }
      rows += t.nat[g];
    }
  return n;
}

// A mixed row tiling for edge layer 2 (r6). Below edge_layer_min row tiles edge layer 2 runs on the
// two-launch schedule, where a last round of 256-row tiles may leave CUs idle (64x20: 400 tiles on 256 CUs, the second
// round 56% full). When that round is at most 3/4 full, its rows fit one round of 192-row tiles, which cost ~3/4 of a
// 256-row tile: tiles [0, nbig) fill whole rounds with 256 rows (one launch), the rest run on kShortRows rows
// (k_edge16_short, a second launch). Returns nbig, or -1 for the uniform tiling. A cut node's sum stays one sequential
// sum over its edges across tile ends, so every output is bit-identical to the uniform tiling's.
static long short_row_tiles(const BatchTables& t, int P, long ncu, long layer_min) {
  if (t.knn || t.E <= 0 || ncu <= 0 || P < 1) return -1;
  const long R = (t.E + kTileRows - 1) / kTileRows;
  if (R >= layer_min) return -1;  // (the one-grid schedules take uniform tiles)
  for (int n : t.nat)
    if (n > kShortRows) return -1;  // (a node then spans at most two tiles)
  const long J = 2L * P, per = ncu / J;  // jobs per row tile (conditionings x column tiles); row tiles per round
  if (per < 1) return -1;
  const long rounds = (R * J + ncu - 1) / ncu;
  const long nbig = (rounds - 1) * per;
  if (rt_count(t.E, nbig) - nbig > per) return -1;  // more than one round of short tiles
  return nbig;
}
static long short_row_tiles(const BatchTables& t, const chm_model* m, int P) {
  if (m->math != MATH_SPLIT16 || !m->edge_rows_short || !m->edge_rows) return -1;
  return short_row_tiles(t, P, m->ncu, m->edge_layer_min);
}

// carves every device buffer of `b` from `base` (null: sizing pass); returns the bytes used
static size_t batch_layout(chm_batch* b, const chm_model* m, char* base, long ntiles) {
  const int P = b->P, L = m->d.num_layers, X = m->d.text_dim, B = b->B;
  const long N = b->N, E = b->E;
  size_t off = 0;
  auto carve = [&](size_t bytes) -> void* {
    const size_t o = off;
    off += (bytes + 255) / 256 * 256;
    return base ? base + o : nullptr;
  };
  auto fl = [&](size_t n) { return (float*)carve(n * sizeof(float)); };
  b->natoms = (int*)carve(B * sizeof(int));
  b->node_off = (int*)carve((B + 1) * sizeof(int));
  b->edge_off = (long*)carve((B + 1) * sizeof(long));
  b->n2g = (int*)carve(N * sizeof(int));
  b->ei = (int*)carve(E * sizeof(int));
  b->ej = (int*)carve(E * sizeof(int));
  b->node_estart = (long*)carve(N * sizeof(long));
  b->node_n = (int*)carve(N * sizeof(int));
  b->tiles = (int2*)carve(ntiles * sizeof(int2));
  if (!b->knn && b->Ep > 0) {  // fc: the pair tables of edge layer 1 on pairs
    b->pi = (int*)carve(b->Ep * sizeof(int));
    b->pj = (int*)carve(b->Ep * sizeof(int));
    b->pe = (int2*)carve(b->Ep * sizeof(int2));
    b->pnode = (int2*)carve((b->Ep + kPairRows - 1) / kPairRows * sizeof(int2));
  }
  if (!b->pplan.jobs.empty()) {  // (and the one-grid pair schedule: job lists, ranges, per-layer words)
    b->pjobs = (int4*)carve(b->pplan.djobs.size() * sizeof(int4));
    b->psched = (unsigned*)carve((size_t)L * 8 * b->pplan.npx * sizeof(unsigned));
  }
  if (b->nrt > 0) {  // fc: row tiles of edge layer 2, the partial sums of cut nodes, the fallback rows
    b->rtiles = (int4*)carve(b->nrt * sizeof(int4));
    b->rinfo = (int2*)carve((size_t)b->nrt * kRowInfo * sizeof(int2));
    b->rinfo_n = (int*)carve(b->nrt * sizeof(int));
    b->sbuf = fl((size_t)P * b->nrt * H);
    b->msgbuf = fl((size_t)P * (b->r2tot + 1) * H);
    b->rcnt = (unsigned*)carve((size_t)P * b->nrt * 8 * sizeof(unsigned));
    b->lflags = (unsigned*)carve(b->nrt * sizeof(unsigned));
    b->xbad = (unsigned*)carve(2 * kMaxLayers * sizeof(unsigned));  // layer l: [l]; tail of layer l: [kMaxLayers + l]
    b->sched_cap = b->nrt + kMaxLag + 64;
    b->sched = (unsigned*)carve((size_t)L * (16 + 8 * b->sched_cap) * sizeof(unsigned));
  }
  if (b->knn) {  // (E = the edge capacity E_cap)
    b->cand_off = (long*)carve((B + 1) * sizeof(long));
    b->cand_key = (unsigned*)carve(b->C_cap * sizeof(unsigned));
    b->cand2 = (unsigned*)carve(b->C_cap * sizeof(unsigned));
    b->cand_d2 = (float*)carve(b->C_cap * sizeof(float));
    b->fin_key = (unsigned*)carve(2 * b->C_cap * sizeof(unsigned));
    b->fin_fd = (float*)carve(6 * b->C_cap * sizeof(float));
    b->fd = (float*)carve(3 * E * sizeof(float));
    b->atom_cnt = (int*)carve(N * sizeof(int));
    b->deg = (int*)carve(N * sizeof(int));
    b->cryst_fin = (int*)carve(B * sizeof(int));
  }
  b->cin = fl((size_t)P * B * (TD + X));
  b->cemb = fl((size_t)P * B * 2 * H);
  b->Hres = fl((size_t)P * N * H);
  b->Hl = fl((size_t)P * N * H);
  b->Y = fl((size_t)P * N * H);
  b->agg = fl((size_t)P * N * H);
  b->PQ = fl((size_t)P * N * 2 * H);
  b->gbias = fl((size_t)L * B * H);
  // (F and S carry kTileRows rows of padding: the split16 edge GEMMs read whole 256-row tiles)
  b->F = fl((size_t)(E + kTileRows) * FD);
  b->S = fl(((size_t)P * E + kTileRows) * H);
  b->M = b->math == MATH_F32 ? fl((size_t)P * E * H) : nullptr;
  b->rowmax = b->math == MATH_SPLIT16 ? (unsigned*)fl((size_t)P * E) : nullptr;
  b->rmx = fl((size_t)4 * P * N);
  if (b->math == MATH_SPLIT16 && m->node_ps) {  // (option node_ps at batch creation: ~335 MB at 512x40, P = 2)
    void** sp[4] = {&b->Hs, &b->Hls, &b->aggs, &b->Us};
    int** se[4] = {&b->He, &b->Hle, &b->agge, &b->Ue};
    for (int k = 0; k < 4; ++k) {
      *sp[k] = carve((size_t)P * N * H * 4);
      *se[k] = (int*)carve((size_t)P * N * sizeof(int));
    }
  } else {
    b->Hs = b->Hls = b->aggs = b->Us = nullptr;
    b->He = b->Hle = b->agge = b->Ue = nullptr;
  }
  b->tail_flags = (unsigned*)carve(kMaxTailTiles * sizeof(unsigned));
  b->Hf = fl((size_t)P * N * H);
  b->HO = fl((size_t)P * N * HEADS_N);
  b->LAT = fl((size_t)P * B * 9);
  return off;
}

static int batch_build(const chm_model* m, const int32_t* h_natoms, int B, int max_pairs, void* d_ws,
                       size_t ws_bytes, hipStream_t s, chm_batch** out, const BatchOpts& bo = BatchOpts()) {
  if (!out) return fail(CHM_E_ARG, "out is NULL");
  *out = nullptr;
  if (!m || !h_natoms || B < 1) return fail(CHM_E_ARG, "bad batch arguments");
  if (max_pairs < 1 || max_pairs > 2) return fail(CHM_E_ARG, "max_pairs must be 1 or 2");
  if (bo.knn && m->math != MATH_SPLIT16)
    return fail(CHM_E_UNSUPPORTED, "knn edges need the split16 arithmetic (the k_edge16 kernels)");
  BatchTables t;
  int rc = batch_tables(h_natoms, B, t, bo);
  if (rc) return rc;
  t.rt_nbig = short_row_tiles(t, m, max_pairs);
  batch_fill(t);
  chm_batch* b = new chm_batch();
  b->m = m;
  b->math = m->math;
  b->B = B;
  b->P = max_pairs;
  b->N = t.N;
  b->E = t.E;
  b->h_natoms = t.nat;
  b->knn = bo.knn;
  b->knn_max_nb = bo.max_nb;
  b->E_cap = t.E;
  b->C_cap = t.C;
  b->ntiles = t.knn ? (int)(t.N + 1) : (int)t.tiles.size();
  b->nrt = t.knn ? 0 : t.nrt;
  b->r2tot = t.knn ? 0 : t.r2tot;
  b->rt_nbig = t.knn ? -1 : t.rt_nbig;
  b->Ep = t.knn ? 0 : t.Ep;
  if (!t.knn && b->math == MATH_SPLIT16 && t.E > 0 && t.rt_nbig < 0) {  // (the pair grid: uniform row tiles)
    pair_plan(t.nat, t.E, t.Ep, t.nrt, b->P, m->edge_lag, b->pplan);
    if (!pair_plan_ok(b->pplan)) {
      delete b;
      return fail(CHM_E_UNSUPPORTED, "pair grid plan: a flag index outside its list");
    }
  }
  const size_t need = batch_layout(b, m, nullptr, b->ntiles);
  char* base = (char*)d_ws;
  if (!base) {
    if (hipMalloc(&b->owned, need) != hipSuccess) {
      delete b;
      return fail(CHM_E_HIP, "hipMalloc failed for the batch workspace (" + std::to_string(need) + " bytes)");
    }
    base = (char*)b->owned;
  } else if (ws_bytes < need || ((uintptr_t)base & 255)) {
    delete b;
    return fail(CHM_E_ARG, "workspace too small or not 256-byte aligned (need " + std::to_string(need) + " bytes)");
  }
  b->bytes = batch_layout(b, m, base, b->ntiles);
  {  // edge layer 1 tail split: whole rounds of 256x256 tiles first (needs ncu, an even count of tiles).
     // Only for a short partial round (<= 1/4 of the CUs): 64x40 (32 of 256 tiles) gains 6% per step;
     // at 256x40 (128 of 256) the split grid lost 0.8% (profiles/r2/split_*)
    const long tiles1 = (t.E + kTileRows - 1) / kTileRows * (H / 256);
    if (!t.knn && t.rt_nbig < 0 && m->ncu > 0 && tiles1 > m->ncu && tiles1 % m->ncu && (tiles1 % m->ncu) * 4 <= m->ncu) {
      long full = tiles1 / m->ncu * m->ncu;
      full -= full % (H / 256);
      const long rows_a = full / (H / 256) * kTileRows;
      int ta = 0;
      while (ta < (int)t.tiles.size() && (t.tiles[ta].y < t.N ? t.estart[t.tiles[ta].y] : t.E) <= rows_a) ++ta;
      if (rows_a < t.E && ta > 0 && ta < (int)t.tiles.size() && (t.E - rows_a + kTileRows - 1) / kTileRows <= kMaxTailTiles) {
        b->l1_rows_a = rows_a;
        b->l2_tile_a = ta;
      }
    }
  }
  // index tables (setup only: the host vectors must outlive the copies, so the stream is drained)
  hipError_t e = hipSuccess;
  auto up = [&](void* dst, const void* src, size_t bytes) {
    if (e == hipSuccess && bytes) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
  };
  up(b->natoms, t.nat.data(), B * sizeof(int));
  up(b->node_off, t.noff.data(), (B + 1) * sizeof(int));
  up(b->edge_off, t.eoff.data(), (B + 1) * sizeof(long));
  up(b->n2g, t.n2g.data(), t.N * sizeof(int));
  if (t.knn) {
    up(b->cand_off, t.coff.data(), (B + 1) * sizeof(long));
    b->E = 0;  // no graph yet
    b->ntiles = 0;
  } else {
    up(b->ei, t.ei.data(), t.E * sizeof(int));
    up(b->ej, t.ej.data(), t.E * sizeof(int));
    up(b->node_estart, t.estart.data(), t.N * sizeof(long));
    up(b->node_n, t.nn.data(), t.N * sizeof(int));
    up(b->tiles, t.tiles.data(), t.tiles.size() * sizeof(int2));
    up(b->rtiles, t.rtiles.data(), t.rtiles.size() * sizeof(int4));
    up(b->rinfo, t.rinfo.data(), t.rinfo.size() * sizeof(int2));
    up(b->rinfo_n, t.rinfo_n.data(), t.rinfo_n.size() * sizeof(int));
    up(b->pi, t.pi.data(), t.pi.size() * sizeof(int));
    up(b->pj, t.pj.data(), t.pj.size() * sizeof(int));
    up(b->pe, t.pe.data(), t.pe.size() * sizeof(int2));
    up(b->pnode, t.pnode.data(), t.pnode.size() * sizeof(int2));
    if (b->pjobs) {
      up(b->pjobs, b->pplan.djobs.data(), b->pplan.djobs.size() * sizeof(int4));
    }
    if (e == hipSuccess && b->rcnt)  // (the counters return to 0 at the end of every launch)
      e = hipMemsetAsync(b->rcnt, 0, (size_t)b->P * b->nrt * 8 * sizeof(unsigned), s);
    if (e == hipSuccess && b->lflags) e = hipMemsetAsync(b->lflags, 0, b->nrt * sizeof(unsigned), s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    chm_batch_destroy(b);
    return fail(CHM_E_HIP, std::string("index upload: ") + hipGetErrorString(e));
  }
  *out = b;
  return CHM_OK;
}

extern "C" int64_t chm_debug_layer_jobs(int64_t R, int P, int lag, int64_t* out, int64_t cap) {
  if (R < 1 || P < 1 || P > 2 || lag < 1) return fail(CHM_E_ARG, "bad arguments");
  const long nb = edge16_layer_blocks(R, P);
  if (out && cap >= 2 * nb) edge16_layer_jobs(R, P, lag, reinterpret_cast<long*>(out));
  return nb;
}

extern "C" int chm_debug_layer_seq(int64_t n, int P, int lag, int64_t* out) {
  if (n < 0 || P < 1 || P > 2 || lag < 1 || !out) return fail(CHM_E_ARG, "bad arguments");
  edge16_seq_jobs(n, P, lag, reinterpret_cast<long*>(out));
  return CHM_OK;
}

extern "C" int chm_debug_row_nodes_ex(const int32_t* h_natoms, int B, int64_t nbig, int32_t* out2, int64_t cap2,
                                      int32_t* counts, int64_t cap) {
  if (!h_natoms || B < 1) return fail(CHM_E_ARG, "bad batch arguments");
  BatchTables t;
  int rc = batch_tables(h_natoms, B, t);
  if (rc) return rc;
  if (nbig >= 0 && nbig * kTileRows >= t.E) return fail(CHM_E_ARG, "nbig: no short tile left");
  t.rt_nbig = nbig < 0 ? -1 : nbig;
  batch_fill(t);
  const long R = (long)t.rtiles.size();
  if (out2 && cap2 >= 2 * (int64_t)t.rinfo.size())
    for (size_t k = 0; k < t.rinfo.size(); ++k) {
      out2[2 * k] = t.rinfo[k].x;
      out2[2 * k + 1] = t.rinfo[k].y;
    }
  if (counts && cap >= R)
    for (long k = 0; k < R; ++k) counts[k] = t.rinfo_n[k];
  return (int)R;
}

extern "C" int chm_debug_row_nodes(const int32_t* h_natoms, int B, int32_t* out2, int64_t cap2, int32_t* counts,
                                   int64_t cap) {
  return chm_debug_row_nodes_ex(h_natoms, B, -1, out2, cap2, counts, cap);
}

extern "C" int chm_debug_row_tiles_ex(const int32_t* h_natoms, int B, int64_t nbig, int32_t* out4, int64_t cap4,
                                      int64_t* r2tot) {
  if (!h_natoms || B < 1) return fail(CHM_E_ARG, "bad batch arguments");
  BatchTables t;
  int rc = batch_tables(h_natoms, B, t);
  if (rc) return rc;
  if (nbig >= 0 && nbig * kTileRows >= t.E) return fail(CHM_E_ARG, "nbig: no short tile left");
  t.rt_nbig = nbig < 0 ? -1 : nbig;
  std::vector<int4> rt;
  const long r2 = row_tiles(t, &rt);
  if (r2tot) *r2tot = r2;
  if (out4 && cap4 >= 4 * (int64_t)rt.size())
    for (size_t k = 0; k < rt.size(); ++k) {
      out4[4 * k] = rt[k].x; out4[4 * k + 1] = rt[k].y; out4[4 * k + 2] = rt[k].z; out4[4 * k + 3] = rt[k].w;
    }
  return (int)rt.size();
}

extern "C" int chm_debug_row_tiles(const int32_t* h_natoms, int B, int32_t* out4, int64_t cap4, int64_t* r2tot) {
  return chm_debug_row_tiles_ex(h_natoms, B, -1, out4, cap4, r2tot);
}

// the mixed row tiling short_row_tiles chooses for a batch (256-row tiles before the short ones, -1: uniform)
extern "C" int64_t chm_debug_short_row_tiles(const int32_t* h_natoms, int B, int P, int ncu, int64_t layer_min) {
  if (!h_natoms || B < 1 || P < 1 || P > 2) return fail(CHM_E_ARG, "bad batch arguments");
  BatchTables t;
  int rc = batch_tables(h_natoms, B, t);
  if (rc) return rc;
  return short_row_tiles(t, P, ncu, layer_min);
}

// the row tiling of a batch as it was created (256-row tiles before the short ones, -1: uniform)
extern "C" int64_t chm_batch_short_row_tiles(const chm_batch* b) {
  if (!b) return fail(CHM_E_ARG, "batch is NULL");
  return b->rt_nbig;
}

extern "C" int chm_batch_create(const chm_model* m, const int32_t* h_natoms, int B, int max_pairs, chm_batch** out) {
  return batch_build(m, h_natoms, B, max_pairs, nullptr, 0, nullptr, out);
}

extern "C" size_t chm_batch_workspace_bytes_ex(const chm_model* m, const int32_t* h_natoms, int B, int max_pairs,
                                               const chm_batch_options* opts) {
  if (!m || !h_natoms || B < 1 || max_pairs < 1 || max_pairs > 2) {
    fail(CHM_E_ARG, "bad batch arguments");
    return 0;
  }
  BatchOpts bo;
  if (batch_opts(opts, bo)) return 0;
  BatchTables t;
  if (batch_tables(h_natoms, B, t, bo)) return 0;
  chm_batch b;
  b.m = m;
  b.math = m->math;
  b.B = B;
  b.P = max_pairs;
  b.N = t.N;
  b.E = t.E;
  b.knn = bo.knn;
  b.C_cap = t.C;
  if (!t.knn) {
    t.rt_nbig = short_row_tiles(t, m, max_pairs);
    b.nrt = rt_count(t.E, t.rt_nbig);
    b.r2tot = row_tiles(t, nullptr);
    b.Ep = t.Ep;
    if (b.math == MATH_SPLIT16 && t.E > 0 && t.rt_nbig < 0) pair_plan(t.nat, t.E, t.Ep, b.nrt, b.P, m->edge_lag, b.pplan);
  }
  return batch_layout(&b, m, nullptr, count_tiles(t));
}

extern "C" size_t chm_batch_workspace_bytes(const chm_model* m, const int32_t* h_natoms, int B, int max_pairs) {
  return chm_batch_workspace_bytes_ex(m, h_natoms, B, max_pairs, nullptr);
}

extern "C" int chm_batch_create_ex(const chm_model* m, const int32_t* h_natoms, int B, int max_pairs,
                                   const chm_batch_options* opts, void* d_workspace, size_t workspace_bytes,
                                   void* stream, chm_batch** out) {
  BatchOpts bo;
  const int rc = batch_opts(opts, bo);
  if (rc) return rc;
  return batch_build(m, h_natoms, B, max_pairs, d_workspace, workspace_bytes, (hipStream_t)stream, out, bo);
}

extern "C" int chm_batch_create_with_workspace(const chm_model* m, const int32_t* h_natoms, int B, int max_pairs,
                                               void* d_workspace, size_t workspace_bytes, void* stream,
                                               chm_batch** out) {
  if (!d_workspace) return fail(CHM_E_ARG, "workspace is NULL");
  return batch_build(m, h_natoms, B, max_pairs, d_workspace, workspace_bytes, (hipStream_t)stream, out);
}

extern "C" void chm_batch_destroy(chm_batch* b) {
  if (!b) return;
  if (b->owned) (void)hipFree(b->owned);
  delete b;
}

extern "C" size_t chm_batch_device_bytes(const chm_batch* b) { return b ? b->bytes : 0; }
extern "C" int64_t chm_batch_num_nodes(const chm_batch* b) { return b ? b->N : -1; }
extern "C" int64_t chm_batch_num_edges(const chm_batch* b) { return b ? b->E : -1; }
// (host only, tests) the one-grid pair schedule of an fc batch: see include/chemeleon_hip.h
extern "C" int64_t chm_debug_pair_plan(const int32_t* h_natoms, int B, int P, int lag, int32_t* rng, int64_t cap_rng,
                                       int32_t* pa, int32_t* pb, int32_t* njobs, int32_t* jobs, int64_t cap_jobs) {
  if (!h_natoms || B < 1 || P < 1 || P > 2 || lag < 1) return fail(CHM_E_ARG, "bad arguments");
  BatchTables t;
  if (int rc = batch_tables(h_natoms, B, t)) return rc;
  const long R = (t.E + kTileRows - 1) / kTileRows;
  PairPlan pl;
  pair_plan(t.nat, t.E, t.Ep, R, P, lag, pl);
  if (!pair_plan_ok(pl)) return fail(CHM_E_UNSUPPORTED, "pair grid plan: a flag index outside its list");
  if (rng && cap_rng >= 2 * R)
    for (long k = 0; k < R; ++k) { rng[2 * k] = pl.rng[k].x; rng[2 * k + 1] = pl.rng[k].y; }
  for (int x = 0; x < 8; ++x) {
    if (pa) pa[x] = pl.pa[x];
    if (pb) pb[x] = pl.pb[x];
    if (njobs) njobs[x] = pl.njobs[x];
  }
  if (jobs && cap_jobs >= 2L * 8 * pl.jstride)
    for (size_t k = 0; k < pl.jobs.size(); ++k) { jobs[2 * k] = pl.jobs[k].x; jobs[2 * k + 1] = pl.jobs[k].y; }
  return pl.jstride;
}

// (host only, tests) the pair tiles' P / Q node ranges of an fc batch: see include/chemeleon_hip.h
extern "C" int64_t chm_debug_pair_nodes(const int32_t* h_natoms, int B, int32_t* out, int64_t cap) {
  if (!h_natoms || B < 1) return fail(CHM_E_ARG, "bad arguments");
  BatchTables t;
  if (int rc = batch_tables(h_natoms, B, t)) return rc;
  batch_fill(t);
  const int64_t NP = (int64_t)t.pnode.size();
  if (out && cap >= 2 * NP)
    for (int64_t k = 0; k < NP; ++k) { out[2 * k] = t.pnode[k].x; out[2 * k + 1] = t.pnode[k].y; }
  return NP;
}

extern "C" int chm_batch_device(const chm_batch* b) { return b ? b->m->device : fail(CHM_E_ARG, "batch is NULL"); }
extern "C" int chm_batch_info(const chm_batch* b, chm_dims* dims, int64_t* num_graphs, int* max_pairs, int* knn) {
  if (!b) return fail(CHM_E_ARG, "batch is NULL");
  if (dims) *dims = b->m->d;
  if (num_graphs) *num_graphs = b->B;
  if (max_pairs) *max_pairs = b->P;
  if (knn) *knn = b->knn;
  return CHM_OK;
}

// ---------------------------------------------------------------- instrumentation
namespace {
struct ProfRec { int id; hipEvent_t a, b; };
bool g_prof_on = false;
std::mutex g_prof_mu;
std::vector<hipEvent_t> g_pool;
std::vector<ProfRec> g_recs;
size_t g_pool_next = 0;
constexpr size_t kPoolPairs = 8192;

struct ProfScope {
  int id; hipStream_t s; hipEvent_t b = nullptr;
  ProfScope(int id_, hipStream_t s_) : id(id_), s(s_) {
    if (!g_prof_on) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (g_pool_next + 2 > g_pool.size()) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;  // not in graphs
    hipEvent_t a = g_pool[g_pool_next++];
    b = g_pool[g_pool_next++];
    if (hipEventRecord(a, s) != hipSuccess) { b = nullptr; return; }
    g_recs.push_back({id, a, b});
  }
  ~ProfScope() { if (b) (void)hipEventRecord(b, s); }
};
}  // namespace

extern "C" int chm_prof_enable(int on) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (on && g_pool.empty()) {
    g_pool.resize(2 * kPoolPairs);
    for (auto& e : g_pool)
      if (hipEventCreate(&e) != hipSuccess) return fail(CHM_E_HIP, "hipEventCreate failed");
  }
  g_prof_on = on != 0;
  return CHM_OK;
}

extern "C" int chm_prof_reset(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_recs.clear();
  g_pool_next = 0;
  return CHM_OK;
}

extern "C" int chm_prof_read(int kernel, int64_t* launches, double* total_ms) {
  if (!launches || !total_ms) return fail(CHM_E_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(g_prof_mu);
  int64_t n = 0;
  double tot = 0;
  for (const auto& r : g_recs) {
    if (r.id != kernel) continue;
    float ms = 0;
    hipError_t e = hipEventElapsedTime(&ms, r.a, r.b);
    if (e != hipSuccess) return fail(CHM_E_HIP, std::string("hipEventElapsedTime: ") + hipGetErrorString(e));
    ++n;
    tot += ms;
  }
  *launches = n;
  *total_ms = tot;
  return CHM_OK;
}

extern "C" int chm_prof_events(int64_t* out, int n) {
  if (!out || n < 1) return fail(CHM_E_ARG, "NULL argument");
  unsigned long long v[EV_COUNT];
  hipError_t e = edge_events_read(v);
  if (e != hipSuccess) return fail(CHM_E_HIP, std::string("edge_events_read: ") + hipGetErrorString(e));
  for (int k = 0; k < n; ++k) out[k] = k < EV_COUNT ? (int64_t)v[k] : 0;
  return CHM_OK;
}

extern "C" int chm_prof_events_reset(void) {
  hipError_t e = edge_events_reset();
  if (e != hipSuccess) return fail(CHM_E_HIP, std::string("edge_events_reset: ") + hipGetErrorString(e));
  return CHM_OK;
}

static GemmArgs gargs(long M, int N, int K, const float* A, long lda, const float* W, float* C, long ldc) {
  GemmArgs g;
  std::memset(&g, 0, sizeof(g));
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.A2 = A; g.lda2 = lda; g.ksplit = K;
  g.W = W; g.ldw = K; g.C = C; g.ldc = ldc; g.gb_rowmod = 1;
  return g;
}

// W16 / wsc: the split16 node-GEMM rows of the same weight (null: bf16x3 in every mode)
static hipError_t run_gemm(const chm_batch* b, GemmArgs g, int epi, const void* W3, hipStream_t s,
                           const void* W16 = nullptr, const float* wsc = nullptr) {
  if (b->math == MATH_F32) return gemm(g, epi, s);
  if (b->math == MATH_SPLIT16 && W16 && (g.amax || g.aex) && b->m->node16 && b->m->node_glds && epi == EPI_STD) {
    g.Wp3 = W16; g.wscale = wsc;
    return node_gemm(g, s);
  }
  g.Wp3 = W3;
  if (epi == EPI_STD && b->m->node_glds) return node_gemm(g, s);
  return gemm_bf16x3(g, epi, s);
}

// the two edge GEMMs (M = E or P*E rows) in f32 / bf16x3 mode: 256x256 bf16x3 tiles
static hipError_t run_edge_gemm(const chm_batch* b, GemmArgs g, int epi, const void* W3, hipStream_t s) {
  if (b->math == MATH_F32) return gemm(g, epi, s);
  g.Wp3 = W3;
  return gemm_bf16x3_big(g, epi, s);
}

// profiling (CHM_EDGE_TRACE=file, CHM_EDGE_TRACE_LAYER=1-4): the 4th eager launch of edge layer
// 1 or 2 records {hw id, t0, t_mainloop, t_end, ...} per block (s_memrealtime), dumped to the file
template <class F>
static hipError_t traced_edge_launch(const chm_model* m, EdgeArgs& ea, int which, long E, hipStream_t s, F&& launch) {
  static std::atomic<int> traced{0};
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  const bool tr = m->edge_trace && m->edge_trace_layer == which && traced < 4 &&
                  hipStreamIsCapturing(s, &cst) == hipSuccess && cst == hipStreamCaptureStatusNone && ++traced == 4;
  if (!tr) return launch();
  unsigned long long* tbuf = nullptr;
  // (3: slot 8 k + XCD; 4, the pair grid: 8 x its longest job list, at most E / 32 jobs)
  const long tblocks = (which == 4 ? E / 4 : which == 3 ? 48 * (E / 256 + 1) : 4 * (E / 128 + 1)) + 4096;
  hipError_t e = hipMalloc(&tbuf, tblocks * 48);
  if (e == hipSuccess) e = hipMemsetAsync(tbuf, 0, tblocks * 48, s);
  if (e != hipSuccess) return e;
  ea.trace = tbuf;
  e = launch();
  ea.trace = nullptr;
  std::vector<unsigned long long> h(tblocks * 6);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipMemcpy(h.data(), tbuf, tblocks * 48, hipMemcpyDeviceToHost);
  if (e == hipSuccess) {
    FILE* f = fopen(m->edge_trace, "wb");
    if (f) {
      fwrite(h.data(), 8, h.size(), f);
      fclose(f);
    }
  }
  (void)hipFree(tbuf);
  return e;
}

// heads: bit 0 = node heads (types + coords), bit 1 = lattice head
// knn batches: the radius graph of these coordinates (knn.hip), edges grouped by source node. One
// stream sync reads the out-degrees back to size the launches and build the segment tiles.
static int knn_build(chm_batch* b, const float* x, const float* lat, hipStream_t s) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
    return fail(CHM_E_UNSUPPORTED, "knn batches rebuild their edges on the host's schedule: no graph capture");
  const int B = b->B;
  const long N = b->N;
  KnnArgs k;
  std::memset(&k, 0, sizeof(k));
  k.x = x; k.lat = lat; k.natoms = b->natoms; k.node_off = b->node_off; k.cand_off = b->cand_off;
  k.cand_key = b->cand_key; k.cand_d2 = b->cand_d2; k.cand2 = b->cand2; k.atom_cnt = b->atom_cnt;
  k.max_nb = b->knn_max_nb; k.fin_key = b->fin_key; k.fin_fd = b->fin_fd; k.deg = b->deg; k.cryst_fin = b->cryst_fin;
  k.node_estart = b->node_estart; k.ei = b->ei; k.ej = b->ej; k.fd = b->fd;
  HIPCHK(knn_candidates(k, B, s));
  b->h_deg.resize(N);
  HIPCHK(hipMemcpyAsync(b->h_deg.data(), b->deg, N * sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  b->h_estart.resize(N);
  b->h_tiles.clear();
  long E = 0, rows = 0;
  int cur0 = 0;
  for (long v = 0; v < N; ++v) {  // segment tiles: runs of whole nodes of <= 256 edge rows (as batch_fill)
    const int d = b->h_deg[v];
    if (d > kTileRows) return fail(CHM_E_UNSUPPORTED, "knn: a node with more than 256 edges");
    b->h_estart[v] = E;
    E += d;
    if (rows + d > kTileRows || v - cur0 >= kTileRows) {  // (<= 256 nodes: isolated atoms add no rows)
      b->h_tiles.push_back(make_int2(cur0, (int)v));
      cur0 = (int)v;
      rows = 0;
    }
    rows += d;
  }
  b->h_tiles.push_back(make_int2(cur0, (int)N));
  if (E > b->E_cap)
    return fail(CHM_E_UNSUPPORTED, "knn: the graph has " + std::to_string(E) + " edges, above the batch capacity " +
                                       std::to_string(b->E_cap) + " (chm_batch_options.knn_edges_per_atom)");
  HIPCHK(hipMemcpyAsync(b->node_estart, b->h_estart.data(), N * sizeof(long), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(b->node_n, b->h_deg.data(), N * sizeof(int), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(b->tiles, b->h_tiles.data(), b->h_tiles.size() * sizeof(int2), hipMemcpyHostToDevice, s));
  HIPCHK(knn_place(k, B, s));
  b->E = E;
  b->ntiles = (int)b->h_tiles.size();
  return CHM_OK;
}

// reuse_cond: the FiLM conditioning (cond_in + the conditioning MLP) of the previous call on this batch
// is still valid (same t and text: the corrector call of a reverse step, chemeleon.py:438-448)
static int run_decoder(chm_batch* b, int P, const int64_t* a, const float* x, const float* lat, const float* temb,
                       int tstride, const int* d_t, const float* text0, const float* text1, int heads,
                       hipStream_t s, bool reuse_cond = false) {
  const chm_model* m = b->m;
  if (b->knn) {
    const int rc = knn_build(b, x, lat, s);
    if (rc) return rc;
  }
  const int L = m->d.num_layers, X = m->d.text_dim, B = b->B;
  const long N = b->N, E = b->E, R = (long)P * N;
  const int CIN = TD + X;
  ProfScope whole(CHM_K_DECODER, s);
  // split16 node GEMMs: row maxima of their A operands, written by the producing kernels
  const bool n16 = b->math == MATH_SPLIT16 && m->node16 && m->node_glds;
  // pre-split node GEMMs: the producers write the A operands split (no row-max atomics then)
  const bool ps = n16 && m->node_ps && b->Hs;
  const long RS = (long)b->P * N;
  auto rmx = [&](int k) { return n16 && !ps ? b->rmx + k * RS : nullptr; };
  if (m->film && !reuse_cond) {
    HIPCHK(build_cond_in(temb, tstride, d_t, text0, text1, X, b->cin, B, P, s));
    GemmArgs g = gargs((long)P * B, 2 * H, CIN, b->cin, CIN, m->Wc, b->cemb, 2 * H);
    g.bias = m->bc; g.act = 1;
    HIPCHK(run_gemm(b, g, EPI_STD, m->Wc3, s));
  }
  // fc edge layer 1 on unordered pairs (option edge_pairs): F holds the pairs' features only
  const bool pairs = b->math == MATH_SPLIT16 && m->edge_pairs && b->pe && !b->knn && E > 0;
  // (edge layer 1 on pairs as two launches, the default below 256 row tiles: no intra-grid waits, nothing to clear;
  // the memsets cost 4.8 us each per call, 0.9% of a 64x20 step)
  // both edge layers on pairs in one grid (k_edge16_pairs_grid) for this call
  const bool pair_grid = pairs && m->edge_pairs_layer && m->edge_rows && b->rtiles && m->edge_layer && b->psched &&
                         P == b->P && b->nrt >= m->edge_layer_min && m->ncu > 0 && m->xcd_mask == 0xffu &&
                         b->rt_nbig < 0;
  const bool waits = !pairs || pair_grid;
  // the pair grid's repair requests and per-layer flags start clear in every call: zeroed by the embedding launch
  // below (two memset nodes less per call)
  const bool zero_grid = b->xbad && b->math == MATH_SPLIT16 && pair_grid;
  // the embedding rows and the first kGBLayers layers' per-graph terms of edge layer 1 in one launch
  GraphBiasArgs ga0;
  const int nl0 = L < kGBLayers ? L : kGBLayers;
  for (int l = 0; l < nl0; ++l) {
    ga0.Wc[l] = m->layers[l].Wcl;
    ga0.b1[l] = m->layers[l].b1;
  }
  HIPCHK(embed(a, m->emb, b->Hres, N, P, s, rmx(RMX_H), ps ? b->Hs : nullptr, ps ? b->He : nullptr, lat,
               nl0 > 0 ? &ga0 : nullptr, nl0, 9, b->gbias, B, zero_grid ? b->xbad : nullptr,
               zero_grid ? 2L * kMaxLayers : 0L, zero_grid ? b->psched : nullptr,
               zero_grid ? (long)L * 8 * b->pplan.npx : 0L));
  if (pairs)
    HIPCHK(fourier_h(x, b->pi, b->pj, b->Ep, b->F, s, nullptr));  // (the (i, j) edges' features, i <= j)
  else if (b->math == MATH_SPLIT16)
    HIPCHK(fourier_h(x, b->ei, b->ej, E, b->F, s, b->knn ? b->fd : nullptr));  // fp16 hi/lo split rows
  else
    HIPCHK(fourier(x, b->ei, b->ej, E, b->F, s));
  for (int l0 = kGBLayers; l0 < L; l0 += kGBLayers) {  // the per-graph terms of layers past the first 16
    GraphBiasArgs ga;
    const int nl = L - l0 < kGBLayers ? L - l0 : kGBLayers;
    for (int l = 0; l < nl; ++l) {
      ga.Wc[l] = m->layers[l0 + l].Wcl;
      ga.b1[l] = m->layers[l0 + l].b1;
    }
    HIPCHK(graph_bias(lat, ga, nl, 9, b->gbias + (size_t)l0 * B * H, B, s));
  }
  if (b->xbad && b->math == MATH_SPLIT16 && waits && !pair_grid) {
    // k_edge16_layer / k_edge16_tail: repair requests (layer l: xbad[l], tail of layer l: xbad[kMaxLayers + l])
    // and row-tile flags start clear in every call (the flags also return to 0 at the end of every
    // launch; this keeps a timed-out wait from leaking into later calls)
    HIPCHK(hipMemsetAsync(b->xbad, 0, 2 * kMaxLayers * sizeof(unsigned), s));
    if (!pairs && m->edge_rows && m->edge_layer && m->edge_dyn && b->sched)
      HIPCHK(hipMemsetAsync(b->sched, 0, (size_t)L * (16 + 8 * b->sched_cap) * sizeof(unsigned), s));
    if (!pairs && m->edge_rows && m->edge_layer) HIPCHK(hipMemsetAsync(b->lflags, 0, b->nrt * sizeof(unsigned), s));
  }
  for (int l = 0; l < L; ++l) {
    const LayerW& w = m->layers[l];
    if (m->film) {  // FiLM projection (cspnet.py:92)
      GemmArgs g = gargs(R, H, H, ps ? (const float*)b->Hs : b->Hres, H, m->Wp, b->Y, H);
      g.bias = m->bp; g.amax = rmx(RMX_H);
      if (ps) g.aex = b->He;
      HIPCHK(run_gemm(b, g, EPI_STD, m->Wp3, s, m->Wp16, m->Wpsc));
    }
    // FiLM + residual + the layer's LayerNorm (film-less: the LayerNorm only)
    HIPCHK(film_ln(m->film ? b->Y : nullptr, b->Hres, b->Hl, b->cemb, b->n2g, N, B, P, m->fw, m->fb, w.lw, w.lb, s,
                   rmx(0), RS, ps ? b->Hls : nullptr, ps ? b->Hle : nullptr));
    {  // per-node halves of the first edge layer: [P | Q] = Hl [A ; Bm]^T, P += b1 + C vec(LL^T)
      GemmArgs g = gargs(R, 2 * H, H, ps ? (const float*)b->Hls : b->Hl, H, w.WAB, b->PQ, 2 * H);
      g.gb = b->gbias + (size_t)l * B * H; g.ldgb = H; g.gb_cols = H; g.row2g = b->n2g; g.gb_rowmod = N;
      g.amax = rmx(RMX_HL);
      if (ps) g.aex = b->Hle;
      HIPCHK(run_gemm(b, g, EPI_STD, w.WAB3, s, w.WAB16, w.WABsc));
    }
    if (b->math == MATH_SPLIT16 && E == 0) {  // (knn: no atom within any other's radius: every mean is 0)
      HIPCHK(hipMemsetAsync(b->agg, 0, (size_t)P * N * H * sizeof(float), s));
      if (ps) {
        HIPCHK(hipMemsetAsync(b->aggs, 0, (size_t)P * N * H * 4, s));
        HIPCHK(hipMemsetAsync(b->agge, 0, (size_t)P * N * sizeof(int), s));
      }
    } else if (b->math == MATH_SPLIT16) {
      // split16: fp16 hi/lo split rows throughout (edge16.hip). S lives in S's bytes as
      // split rows [P*E][H/32][2][32] plus one packed exponent word per row (rowmax buffer).
      int* sexp = reinterpret_cast<int*>(b->rowmax);
      // edge layer 1: S_c = SiLU(D f_ij + P_c[i] + Q_c[j]), D f shared by the pair
      EdgeArgs e1;
      std::memset(&e1, 0, sizeof(e1));
      e1.M = E; e1.N = H; e1.K = FD; e1.A = b->F; e1.W = w.D2h; e1.wscale = w.Dsc;
      e1.ei = b->ei; e1.ej = b->ej; e1.PQ = b->PQ; e1.nnodes = N; e1.npairs = P; e1.E = E;
      e1.node_off = b->node_off; e1.natoms = b->natoms; e1.n2g = b->n2g;
      e1.S = b->S; e1.sexp = sexp; e1.dbg = m->edge_dbg; e1.stagger = m->edge_stagger;
      // edge layer 2 fused with the aggregation: agg = mean_j SiLU(S W2^T + b2)
      EdgeArgs e2;
      std::memset(&e2, 0, sizeof(e2));
      e2.M = (long)P * E; e2.N = H; e2.K = H; e2.A = b->S; e2.aexp = sexp;
      e2.W = w.W22h16; e2.wscale = w.W2sc; e2.bias = w.b2; e2.tiles = b->tiles;
      e2.ntiles = b->ntiles;
      e2.node_estart = b->node_estart; e2.natoms = b->natoms; e2.n2g = b->n2g; e2.agg = b->agg;
      e2.node_n = b->node_n; e2.agg_max = reinterpret_cast<unsigned*>(rmx(RMX_AGG));
      if (ps) { e2.aggs = b->aggs; e2.agge = b->agge; }
      e2.nnodes = N; e2.npairs = P; e2.E = E; e2.dbg = m->edge_dbg; e2.stagger = m->edge_stagger;
      if (m->edge_rows && b->rtiles) {  // 256-row tiles, cut nodes continued across tiles
        e2.rtiles = b->rtiles; e2.ntiles = (int)b->nrt; e2.sbuf = b->sbuf; e2.msgbuf = b->msgbuf;
        e2.rinfo = b->rinfo; e2.rinfo_n = b->rinfo_n;
        e2.rcnt = b->rcnt; e2.r2tot = b->r2tot;
      }
      // edge layer 2 on the two-launch schedule: one launch, or on a mixed row tiling (short_row_tiles) its 256-row
      // tiles, then its 192-row tiles (k_edge16_short)
      auto layer2 = [&](const EdgeArgs& ga) -> hipError_t {
        if (!ga.rtiles || b->rt_nbig < 0) return edge_gemm16(ga, EPI_SEGMEAN, s);
        if (b->rt_nbig > 0) {
          EdgeArgs gb = ga;
          gb.rt_count = (int)b->rt_nbig;
          if (hipError_t r = edge_gemm16(gb, EPI_SEGMEAN, s); r != hipSuccess) return r;
        }
        EdgeArgs gs = ga;
        gs.rt_first = (int)b->rt_nbig;
        gs.rt_count = (int)(b->nrt - b->rt_nbig);
        gs.rt_h = kShortRows;
        gs.rt_e0 = b->rt_nbig * kTileRows;
        return edge_gemm16(gs, EPI_SEGMEAN, s);
      };
      // (instrumented eager launches keep one launch per layer, so the per-kernel timings stay whole;
      // captured launches are never instrumented)
      hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
      const bool instrumented = g_prof_on && hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone;
      // (same-box A/B, static grid against two launches: 64x40 8.47 -> 7.77 ms per step, 512x40 54.9 -> 54.8,
      // 64x20 2.95 -> 3.10: 100 row tiles leave each XCD's job list too short to pack; profiles/r5/grid/)
      if (pair_grid) {
        // both edge layers in one grid, layer 1 on pairs (k_edge16_pairs_grid)
        EdgeArgs e1p = e1;
        e1p.M = b->Ep; e1p.Mp = b->Ep; e1p.pi = b->pi; e1p.pj = b->pj; e1p.pe = b->pe; e1p.pnode = b->pnode;
        e1p.xbad = e2.xbad = b->xbad + l;
        PairSched ps;
        ps.jobs = b->pjobs; ps.jstride = b->pplan.jstride;
        ps.npx = b->pplan.npx; ps.pflag = b->psched + (size_t)l * 8 * b->pplan.npx; ps.R = b->nrt;
        ProfScope ps_(CHM_K_EDGE_LAYER, s);
        // (CHM_EDGE_TRACE_LAYER=4: block timelines of this grid, slot = blockIdx)
        HIPCHK(traced_edge_launch(m, e2, 4, E, s, [&] {
          ps.trace = e2.trace;
          e2.trace = nullptr;
          const hipError_t r = edge_gemm16_pairs_layer(e1p, e2, ps, m->repair_grid, s);
          ps.trace = nullptr;
          return r;
        }));
      } else if (pairs) {
        // edge layer 1 on pairs (both directions' S rows per pair), then edge layer 2 on its row tiles
        EdgeArgs e1p = e1;
        e1p.M = b->Ep; e1p.Mp = b->Ep; e1p.pi = b->pi; e1p.pj = b->pj; e1p.pe = b->pe; e1p.pnode = b->pnode;
        {
          ProfScope ps(CHM_K_EDGE_FOURIER, s);
          HIPCHK(edge_gemm16_pairs(e1p, s));
        }
        ProfScope ps(CHM_K_EDGE_MESSAGE, s);
        HIPCHK(layer2(e2));
      } else if (e2.rtiles && m->edge_layer && b->nrt >= m->edge_layer_min && b->rt_nbig < 0 &&
                 (!m->edge_trace || m->edge_trace_layer == 3)) {
        // both layers in one grid: layer 2's row tiles behind layer 1's (k_edge16_layer)
        e1.lflags = e2.lflags = b->lflags;
        e1.xbad = e2.xbad = b->xbad + l;
        ProfScope ps(CHM_K_EDGE_LAYER, s);
        // (CHM_EDGE_TRACE_LAYER=3: block timelines of this grid, slot = blockIdx)
        HIPCHK(traced_edge_launch(m, e1, 3, E, s, [&] {
          e2.trace = e1.trace;
          const hipError_t r =
              m->ncu > 0 && m->xcd_mask == 0xffu &&
                      (m->edge_dyn == 2 || (m->edge_dyn == 1 && b->nrt >= kDynMinTiles))
                  ? edge_gemm16_layer(e1, e2, m->edge_lag, m->repair_grid, s,
                                      b->sched + (size_t)l * (16 + 8 * b->sched_cap), (int)b->sched_cap, m->ncu,
                                      m->edge_pool, m->edge_skip_xcd)
                  : edge_gemm16_layer(e1, e2, m->edge_lag, m->repair_grid, s);
          e2.trace = nullptr;
          return r;
        }));
      } else if (b->l1_rows_a > 0 && b->xbad && m->edge_split && !instrumented && !m->edge_trace) {
        // Edge layer 1 in whole rounds of the grid (rows [0, l1_rows_a)), then one grid with its
        // partial last round first and all of edge layer 2's segment tiles behind it (the few that
        // read those rows wait for them inside the grid). Same tiles, same arithmetic: bit-identical
        // to one launch per layer.
        EdgeArgs e1b = e1;
        e1.M = b->l1_rows_a;
        e1.zero_flags = b->tail_flags;
        e1.nzero = (int)((E - b->l1_rows_a + kTileRows - 1) / kTileRows);
        e1b.row_base = b->l1_rows_a;
        e1b.flags = e2.flags = b->tail_flags;
        e1b.flag_row0 = e2.flag_row0 = b->l1_rows_a;
        e2.xbad = b->xbad + kMaxLayers + l;  // (a timed-out wait: the repair launches recompute edge layer 2)
        HIPCHK(edge_gemm16(e1, EPI_EDGE, s));
        HIPCHK(edge_gemm16_tail(e1b, e2, m->repair_grid, s));
      } else {
        {
          ProfScope ps(CHM_K_EDGE_FOURIER, s);
          HIPCHK(traced_edge_launch(m, e1, 1, E, s, [&] {
            return edge_gemm16(e1, EPI_EDGE, s);
          }));
        }
        ProfScope ps(CHM_K_EDGE_MESSAGE, s);
        HIPCHK(traced_edge_launch(m, e2, 2, E, s, [&] {
          return layer2(e2);
        }));
      }
    } else {
      {  // edge layer 1: S_c = SiLU(D f_ij + P_c[i] + Q_c[j]), D f shared by the pair
        GemmArgs g = gargs(E, H, FD, b->F, FD, w.D, b->S, H);
        g.ei = b->ei; g.ej = b->ej; g.PQ = b->PQ; g.nnodes = N; g.npairs = P; g.E = E;
        ProfScope ps(CHM_K_EDGE_FOURIER, s);
        HIPCHK(run_edge_gemm(b, g, EPI_EDGE, w.D3, s));
      }
      if (b->math == MATH_F32) {
        {  // edge layer 2: M = SiLU(S W2^T + b2)
          GemmArgs g = gargs((long)P * E, H, H, b->S, H, w.W2, b->M, H);
          g.bias = w.b2; g.act = 1;
          ProfScope ps(CHM_K_EDGE_MESSAGE, s);
          HIPCHK(gemm(g, EPI_STD, s));
        }
        ProfScope ps(CHM_K_SEGMENT_MEAN, s);
        HIPCHK(segment_mean(b->M, b->agg, b->n2g, b->node_off, b->edge_off, b->natoms, N, E, P, s));
      } else {  // edge layer 2 fused with the aggregation: agg = mean_j SiLU(S W2^T + b2), M never stored
        GemmArgs g = gargs((long)P * E, H, H, b->S, H, w.W2, nullptr, H);
        g.bias = w.b2; g.act = 1; g.tiles = b->tiles; g.ntiles = b->ntiles; g.node_estart = b->node_estart;
        g.natoms = b->natoms; g.n2g = b->n2g; g.agg = b->agg; g.nnodes = N; g.npairs = P; g.E = E;
        ProfScope ps(CHM_K_EDGE_MESSAGE, s);
        HIPCHK(run_edge_gemm(b, g, EPI_SEGMEAN, w.W23, s));
      }
    }
    {  // node MLP 1: U = SiLU([Hl | agg] W3^T + b3)
      GemmArgs g = gargs(R, H, 2 * H, b->Hl, H, w.W3, b->Y, H);
      g.A2 = b->agg; g.lda2 = H; g.ksplit = H; g.bias = w.b3; g.act = 1;
      g.amax = rmx(RMX_HL); g.amax2 = rmx(RMX_AGG); g.cmax = reinterpret_cast<unsigned*>(rmx(RMX_U));
      if (ps) {  // U exists only as the next GEMM's split operand
        g.A = (const float*)b->Hls; g.A2 = (const float*)b->aggs; g.aex = b->Hle; g.aex2 = b->agge;
        g.C = nullptr; g.Cs = b->Us; g.cex = b->Ue;
      }
      HIPCHK(run_gemm(b, g, EPI_STD, w.W33, s, w.W316, w.W3sc));
    }
    {  // node MLP 2 + residual: Hres += SiLU(U W4^T + b4)
      GemmArgs g = gargs(R, H, H, b->Y, H, w.W4, b->Hres, H);
      g.bias = w.b4; g.act = 1; g.R = b->Hres; g.ldr = H;
      g.amax = rmx(RMX_U); g.cmax = reinterpret_cast<unsigned*>(rmx(RMX_H));
      if (ps) {  // (and the residual stream split for the next layer's FiLM projection)
        g.A = (const float*)b->Us; g.aex = b->Ue;
        if (l + 1 < L && m->film) { g.Cs = b->Hs; g.cex = b->He; }
      }
      HIPCHK(run_gemm(b, g, EPI_STD, w.W43, s, w.W416, w.W4sc));
    }
  }
  HIPCHK(layer_norm(b->Hres, b->Hf, R, m->flw, m->flb, s));
  if (heads & 1) {
    GemmArgs g = gargs(R, HEADS_N, H, b->Hf, H, m->Whead, b->HO, HEADS_N);
    g.bias = m->bhead;
    HIPCHK(run_gemm(b, g, EPI_STD, m->Whead3, s));  // (bf16x3: A is LayerNorm output, M small)
  }
  if (heads & 2) HIPCHK(graph_heads(b->Hf, m->Wlat, lat, b->node_off, b->natoms, N, B, P, b->LAT, s));
  return CHM_OK;
}

extern "C" int chm_decoder_forward(chm_batch* b, int pairs, const int64_t* a, const float* x, const float* lat,
                                   const float* temb, int time_stride, const float* text, float* types_out,
                                   float* lattice_out, float* coords_out, float* node_out, void* stream) {
  if (!b) return fail(CHM_E_ARG, "batch is NULL");
  if (pairs < 1 || pairs > b->P) return fail(CHM_E_ARG, "pairs must be in [1, max_pairs]");
  if (!a || !x || !lat || (b->m->film && !temb)) return fail(CHM_E_ARG, "inputs must not be NULL");
  const int X = b->m->d.text_dim;
  if (X > 0 && !text) return fail(CHM_E_ARG, "text embeddings required (text_dim > 0)");
  hipStream_t s = (hipStream_t)stream;
  const float* t0 = text;
  const float* t1 = text ? text + (size_t)b->B * X : nullptr;
  const int heads = ((types_out || coords_out) ? 1 : 0) | (lattice_out ? 2 : 0);
  int rc = run_decoder(b, pairs, a, x, lat, temb, time_stride, nullptr, t0, t1, heads, s);
  if (rc) return rc;
  const long R = (long)pairs * b->N;
  if (heads & 1) HIPCHK(split_heads(b->HO, R, b->m->d.max_atoms, types_out, coords_out, s));
  if (lattice_out)
    HIPCHK(hipMemcpyAsync(lattice_out, b->LAT, (size_t)pairs * b->B * 9 * sizeof(float), hipMemcpyDeviceToDevice, s));
  if (node_out) HIPCHK(hipMemcpyAsync(node_out, b->Hf, (size_t)R * H * sizeof(float), hipMemcpyDeviceToDevice, s));
  return CHM_OK;
}

// the element counts of a step's buffers against the batch (N nodes, B crystals) and its model
static int check_step_io(const chm_batch* b, const chm_step_io* io, bool noise_required, bool noise_allowed) {
  if (!io) return fail(CHM_E_ARG, "io is NULL");
  const long N = b->N, B = b->B, A = b->m->d.max_atoms, X = b->m->d.text_dim;
  auto want = [&](const void* p, int64_t n, long expect, const char* name) -> int {
    if (!p) return fail(CHM_E_ARG, std::string(name) + " is NULL");
    if (n != expect)
      return fail(CHM_E_ARG, std::string(name) + ": " + std::to_string(n) + " elements, the batch needs " +
                                 std::to_string(expect));
    return CHM_OK;
  };
  int rc;
  if ((rc = want(io->d_atom_types, io->n_atom_types, N, "atom_types [N]"))) return rc;
  if ((rc = want(io->d_frac, io->n_frac, 3 * N, "frac [N,3]"))) return rc;
  if ((rc = want(io->d_lattices, io->n_lattices, 9 * B, "lattices [B,3,3]"))) return rc;
  if (X > 0) {
    if ((rc = want(io->d_cond, io->n_cond, B * X, "cond [B,text_dim]"))) return rc;
    if ((rc = want(io->d_null, io->n_null, B * X, "null [B,text_dim]"))) return rc;
  }
  const int given = (io->d_rand_a != nullptr) + (io->d_rand_l != nullptr) + (io->d_rand_x1 != nullptr) +
                    (io->d_rand_x2 != nullptr);
  if (given != 0 && given != 4) return fail(CHM_E_ARG, "noise: all four buffers or none");
  if (given && !noise_allowed) return fail(CHM_E_ARG, "this entry point draws device noise: the noise buffers must be NULL");
  if (!given && noise_required) return fail(CHM_E_ARG, "all four noise buffers are required");
  if (given) {
    if ((rc = want(io->d_rand_a, io->n_rand_a, N * A, "rand_a [N,A]"))) return rc;
    if ((rc = want(io->d_rand_l, io->n_rand_l, 9 * B, "rand_l [B,3,3]"))) return rc;
    if ((rc = want(io->d_rand_x1, io->n_rand_x1, 3 * N, "rand_x1 [N,3]"))) return rc;
    if ((rc = want(io->d_rand_x2, io->n_rand_x2, 3 * N, "rand_x2 [N,3]"))) return rc;
  }
  return CHM_OK;
}

static int sample_step(chm_batch* b, const chm_schedule* sc, int t, int* d_t, float cond_scale, const chm_step_io* io,
                       bool noise_required, bool noise_allowed, uint64_t seed, int64_t node_base, int64_t graph_base,
                       hipStream_t s) {
  if (!b || !sc) return fail(CHM_E_ARG, "batch / schedule is NULL");
  if (b->P < 2) return fail(CHM_E_ARG, "sampling needs a batch created with max_pairs = 2");
  if (!b->m->film) return fail(CHM_E_ARG, "sampling needs a time-conditioned decoder (time_dim > 0)");
  if (sc->T < 1) return fail(CHM_E_ARG, "schedule: T must be >= 1");
  if (!d_t && (t < 1 || t > sc->T)) return fail(CHM_E_ARG, "t out of range");
  if (!sc->d_coef || !sc->d_time_emb || !sc->d_q_one_step || !sc->d_q_mats)
    return fail(CHM_E_ARG, "NULL schedule table");
  if (sc->num_classes != b->m->d.max_atoms || sc->time_dim != b->m->d.time_dim)
    return fail(CHM_E_ARG, "schedule: num_classes " + std::to_string(sc->num_classes) + " / time_dim " +
                               std::to_string(sc->time_dim) + " do not match the model's " +
                               std::to_string(b->m->d.max_atoms) + " / " + std::to_string(b->m->d.time_dim));
  int rc = check_step_io(b, io, noise_required, noise_allowed);
  if (rc) return rc;
  const bool host_noise = io->d_rand_a != nullptr;
  int64_t* d_a = io->d_atom_types;
  float *d_x = io->d_frac, *d_l = io->d_lattices;
  const float *d_cond = b->m->d.text_dim > 0 ? io->d_cond : nullptr, *d_null = b->m->d.text_dim > 0 ? io->d_null : nullptr;
  // time-embedding row: host t -> pointer offset; device t -> offset inside the kernel
  const float* temb = d_t ? sc->d_time_emb : sc->d_time_emb + (size_t)t * TD;
  rc = run_decoder(b, 2, d_a, d_x, d_l, temb, 0, d_t, d_cond, d_null, 3, s);
  if (rc) return rc;
  StepArgs sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.t = t; sa.d_t = d_t; sa.T = sc->T; sa.A = b->m->d.max_atoms; sa.N = b->N; sa.B = b->B;
  sa.cs_null = (float)(1.0 - (double)cond_scale); sa.cs_cond = cond_scale;
  sa.coef = sc->d_coef; sa.q_one_step = sc->d_q_one_step; sa.q_mats = sc->d_q_mats;
  sa.HO = b->HO; sa.LAT = b->LAT; sa.a = d_a; sa.x = d_x; sa.l = d_l; sa.n2g = b->n2g;
  if (host_noise) { sa.ra = io->d_rand_a; sa.rl = io->d_rand_l; sa.rx1 = io->d_rand_x1; sa.rx2 = io->d_rand_x2; }
  sa.seed = seed; sa.node_base = node_base; sa.graph_base = graph_base;
  HIPCHK(step_predictor(sa, s));
  // corrector: same t and text as the predictor, so its FiLM conditioning is reused
  rc = run_decoder(b, 2, d_a, d_x, d_l, temb, 0, d_t, d_cond, d_null, 1, s, true);
  if (rc) return rc;
  HIPCHK(step_corrector(sa, s));
  if (d_t) HIPCHK(decrement(d_t, s));
  return CHM_OK;
}

extern "C" int chm_sample_step(chm_batch* b, const chm_schedule* sc, int t, float cond_scale, const chm_step_io* io,
                               uint64_t seed, int64_t node_base, int64_t graph_base, void* stream) {
  return sample_step(b, sc, t, nullptr, cond_scale, io, false, true, seed, node_base, graph_base, (hipStream_t)stream);
}

extern "C" int chm_sample_step_dt(chm_batch* b, const chm_schedule* sc, int32_t* d_t, float cond_scale,
                                  const chm_step_io* io, uint64_t seed, int64_t node_base, int64_t graph_base,
                                  void* stream) {
  if (!d_t) return fail(CHM_E_ARG, "d_t is NULL");
  return sample_step(b, sc, 0, d_t, cond_scale, io, false, false, seed, node_base, graph_base, (hipStream_t)stream);
}

extern "C" int chm_sample_step_dt_noise(chm_batch* b, const chm_schedule* sc, int32_t* d_t, float cond_scale,
                                        const chm_step_io* io, void* stream) {
  if (!d_t) return fail(CHM_E_ARG, "d_t is NULL");
  return sample_step(b, sc, 0, d_t, cond_scale, io, true, true, 0, 0, 0, (hipStream_t)stream);
}

extern "C" int chm_segment_mean(chm_batch* b, int pairs, const float* msg, int64_t msg_count, float* agg,
                                int64_t agg_count, void* stream) {
  if (!b || !msg || !agg) return fail(CHM_E_ARG, "NULL argument");
  if (pairs < 1) return fail(CHM_E_ARG, "pairs must be >= 1");
  if (b->knn) return fail(CHM_E_UNSUPPORTED, "segment_mean: the fc edge layout only (knn edges change per call)");
  const long H_ = b->m->d.hidden_dim;
  if (msg_count != (int64_t)pairs * b->E * H_)
    return fail(CHM_E_ARG, "msg: " + std::to_string(msg_count) + " elements, pairs x E x hidden_dim = " +
                               std::to_string((int64_t)pairs * b->E * H_));
  if (agg_count != (int64_t)pairs * b->N * H_)
    return fail(CHM_E_ARG, "agg: " + std::to_string(agg_count) + " elements, pairs x N x hidden_dim = " +
                               std::to_string((int64_t)pairs * b->N * H_));
  HIPCHK(segment_mean(msg, agg, b->n2g, b->node_off, b->edge_off, b->natoms, b->N, b->E, pairs, (hipStream_t)stream));
  return CHM_OK;
}

extern "C" int chm_d3pm_sample(int N, int A, int T, const float* logits, const int64_t* xt, const int64_t* tn,
                               const float* noise, const float* q1, const float* qm, int64_t* out, void* stream) {
  if (N < 0 || A < 1 || A > 128 || T < 1) return fail(CHM_E_ARG, "bad sizes");
  if (N == 0) return CHM_OK;
  if (!logits || !xt || !tn || !noise || !q1 || !qm || !out) return fail(CHM_E_ARG, "NULL argument");
  hipStream_t s = (hipStream_t)stream;
  // the device range check: the first node with t outside [1, T] or x_t outside [0, A) (N = none), recorded in
  // one flag word per (host thread, device), allocated on first use; the kernel writes -1 for such a node
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  thread_local std::vector<int*> flag_words;
  if ((int)flag_words.size() <= dev) flag_words.resize(dev + 1, nullptr);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIPCHK(hipStreamIsCapturing(s, &cap));
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (!flag_words[dev]) {
    if (capturing) return fail(CHM_E_UNSUPPORTED, "chm_d3pm_sample: call it once outside capture on this thread first");
    HIPCHK(hipMalloc((void**)&flag_words[dev], sizeof(int)));
  }
  int* d_bad = flag_words[dev];
  int h_bad = N;
  hipError_t e = hipMemsetAsync(d_bad, 0x7f, sizeof(int), s);  // (0x7f7f7f7f: above any node index)
  if (e == hipSuccess)
    e = d3pm_sample(N, A, T, logits, A, nullptr, 1.f, 0.f, xt, tn, 0, nullptr, noise, q1, qm, out, 0, 0, s, d_bad);
  // under stream capture (a graph): no host readback; out-of-range nodes are the ones with out = -1
  if (capturing) {
    if (e != hipSuccess) return fail(CHM_E_HIP, std::string("chm_d3pm_sample: ") + hipGetErrorString(e));
    return CHM_OK;
  }
  if (e == hipSuccess) e = hipMemcpyAsync(&h_bad, d_bad, sizeof(int), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return fail(CHM_E_HIP, std::string("chm_d3pm_sample: ") + hipGetErrorString(e));
  if (h_bad < N)
    return fail(CHM_E_ARG, "d3pm_sample: node " + std::to_string(h_bad) + " has t outside [1, " + std::to_string(T) +
                               "] or x_t outside [0, " + std::to_string(A) + ")");
  return CHM_OK;
}

extern "C" int chm_debug_philox(uint64_t seed, int t, int kind, int64_t base, int64_t n, int normal, float* out,
                                void* stream) {
  if (n < 0 || !out || kind < 0 || kind > 3) return fail(CHM_E_ARG, "bad arguments");
  HIPCHK(philox_fill(seed, t, kind, base, n, normal, out, (hipStream_t)stream));
  return CHM_OK;
}

extern "C" int chm_debug_d3pm_philox(int N, int A, int T, const float* logits, const int64_t* xt, const int64_t* tn,
                                     const float* q1, const float* qm, uint64_t seed, int64_t node_base, int64_t* out,
                                     void* stream) {
  if (N < 0 || A < 1 || A > 128 || T < 1) return fail(CHM_E_ARG, "bad sizes");
  if (N == 0) return CHM_OK;
  if (!logits || !xt || !tn || !q1 || !qm || !out) return fail(CHM_E_ARG, "NULL argument");
  HIPCHK(d3pm_sample(N, A, T, logits, A, nullptr, 1.f, 0.f, xt, tn, 0, nullptr, nullptr, q1, qm, out, seed, node_base,
                     (hipStream_t)stream));
  return CHM_OK;
}

extern "C" int chm_edge_features(chm_batch* b, const float* x, float* feat, void* stream) {
  if (!b || !x || !feat) return fail(CHM_E_ARG, "NULL argument");
  HIPCHK(fourier(x, b->ei, b->ej, b->E, feat, (hipStream_t)stream));
  return CHM_OK;
}

extern "C" int chm_training_loss(chm_batch* b, const chm_train_tables* tt, const int64_t* d_t, const int64_t* a0,
                                 const float* x0, const float* l0, const float* temb, const float* text,
                                 const float* rand_a, const float* noise_l, const float* noise_x, float* out,
                                 int64_t* a_t, float* x_t, float* l_t, float* target_x, float* pred_lattice,
                                 float* pred_coords, void* stream) {
  if (!b || !tt || !d_t || !a0 || !x0 || !l0 || !rand_a || !noise_l || !noise_x || !out)
    return fail(CHM_E_ARG, "NULL argument");
  if (!a_t || !x_t || !l_t || !target_x) return fail(CHM_E_ARG, "the noised-state outputs are required");
  if (!tt->d_coef4 || !tt->d_q_one_step || !tt->d_q_mats || tt->T < 1) return fail(CHM_E_ARG, "bad tables");
  const chm_model* m = b->m;
  if (!m->film || !temb) return fail(CHM_E_ARG, "the training forward needs a time-conditioned decoder");
  if (m->d.text_dim > 0 && !text) return fail(CHM_E_ARG, "text embeddings required (text_dim > 0)");
  hipStream_t s = (hipStream_t)stream;
  const long N = b->N;
  const int B = b->B;
  TrainArgs g;
  std::memset(&g, 0, sizeof(g));
  g.N = N; g.B = B; g.A = m->d.max_atoms; g.T = tt->T; g.t = d_t; g.a0 = a0; g.x0 = x0; g.l0 = l0;
  g.rand_a = rand_a; g.noise_l = noise_l; g.noise_x = noise_x; g.coef = tt->d_coef4;
  g.q_one_step = tt->d_q_one_step; g.q_mats = tt->d_q_mats; g.n2g = b->n2g;
  g.a_t = a_t; g.x_t = x_t; g.l_t = l_t; g.target_x = target_x;
  g.hybrid = tt->hybrid_coeff; g.cost_a = tt->cost_atom_types; g.cost_l = tt->cost_lattice; g.cost_x = tt->cost_coords;
  g.HO = b->HO; g.LAT = b->LAT; g.part = b->Y;  // (Y: decoder scratch, free after the call)
  g.out = out;
  HIPCHK(train_noise(g, s));
  int rc = run_decoder(b, 1, a_t, x_t, l_t, temb, m->d.time_dim, nullptr, text, nullptr, 3, s);
  if (rc) return rc;
  HIPCHK(train_loss(g, s));
  if (pred_lattice) HIPCHK(hipMemcpyAsync(pred_lattice, b->LAT, (size_t)B * 9 * sizeof(float), hipMemcpyDeviceToDevice, s));
  if (pred_coords)
    HIPCHK(hipMemcpy2DAsync(pred_coords, 3 * sizeof(float), b->HO + m->d.max_atoms, HEADS_N * sizeof(float),
                            3 * sizeof(float), N, hipMemcpyDeviceToDevice, s));
  return CHM_OK;
}

extern "C" int chm_knn_edges(chm_batch* b, const float* x, const float* lat, int32_t* src, int32_t* dst, float* fd,
                             int64_t capacity, int64_t* n_edges, void* stream) {
  if (!b || !x || !lat || !n_edges) return fail(CHM_E_ARG, "NULL argument");
  if (!b->knn) return fail(CHM_E_ARG, "not a knn batch");
  hipStream_t s = (hipStream_t)stream;
  int rc = knn_build(b, x, lat, s);
  if (rc) return rc;
  *n_edges = b->E;
  if (b->E > capacity) return CHM_OK;
  if (src) HIPCHK(hipMemcpyAsync(src, b->ei, b->E * sizeof(int), hipMemcpyDeviceToDevice, s));
  if (dst) HIPCHK(hipMemcpyAsync(dst, b->ej, b->E * sizeof(int), hipMemcpyDeviceToDevice, s));
  if (fd) HIPCHK(hipMemcpyAsync(fd, b->fd, b->E * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
  return CHM_OK;
}

extern "C" int chm_edge_features_split(chm_batch* b, const float* x, void* split, void* stream) {
  if (!b || !x || !split) return fail(CHM_E_ARG, "NULL argument");
  // (knn batches: the features of the graph built by the last decoder call / chm_knn_edges)
  HIPCHK(fourier_h(x, b->ei, b->ej, b->E, split, (hipStream_t)stream, b->knn ? b->fd : nullptr));
  return CHM_OK;
}
