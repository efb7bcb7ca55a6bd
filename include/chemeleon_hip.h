/* chemeleon_hip.h — C ABI of the MI355X (gfx950) sampling path of Chemeleon.
 *
 * The hot path of ryannduma/chemeleon is the reverse-diffusion loop
 * `Chemeleon.sample()` -> `_sample_generator()` -> `model_predictions()` ->
 * `CSPNet.forward()` plus the D3PM / DDPM / VE predictor-corrector updates
 * (chemeleon/modules/chemeleon.py:246-490, chemeleon/modules/cspnet.py:184-405,
 * chemeleon/utils/diff_utils.py:152-329). The reference is pure Python over
 * ATen, so there is no reference C interface to replace; each entry point
 * below names the Python interface whose behaviour it takes over.
 *
 * Conventions
 *  - Every pointer argument named d_* is a DEVICE pointer, caller-owned,
 *    fp32 unless stated; int64 where the reference uses torch.long.
 *  - All work is enqueued on the caller's HIP stream `stream`
 *    (a hipStream_t passed as void*); nothing synchronises the host except
 *    chm_model_create / chm_batch_create (setup).
 *  - No allocation inside chm_decoder_forward / chm_sample_step: the batch
 *    object owns a workspace sized at creation. Calls are graph-capturable.
 *  - Every function returns 0 on success or a negative CHM_E_* code;
 *    chm_last_error() returns a thread-local message for the last failure.
 *  - Conditioning index c: 0 = text ("cond"), 1 = null text ("null").
 */
#ifndef CHEMELEON_HIP_H
#define CHEMELEON_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CHM_OK 0
#define CHM_E_ARG (-1)      /* bad argument / shape */
#define CHM_E_HIP (-2)      /* HIP runtime error */
#define CHM_E_UNSUPPORTED (-3)

/* Hyper-parameters of the score network; mirrors the CSPNet constructor
 * (chemeleon/modules/cspnet.py:185-202). This build implements
 * hidden_dim = 512, num_freqs = 128, time_dim = 128 (or time_dim = text_dim = 0:
 * no FilmLayer), ln = ip = 1, smooth = 0, act "silu", dis_emb "sin"; other values
 * return CHM_E_UNSUPPORTED from chm_model_create. The edge style ("fc" or
 * "knn") is a property of the batch (chm_batch_options). */
typedef struct {
  int hidden_dim;  /* 512 */
  int time_dim;    /* 128 */
  int text_dim;    /* 512 */
  int num_layers;  /* 6 */
  int max_atoms;   /* 104 classes (103 elements + dummy) */
  int num_freqs;   /* 128 */
} chm_dims;

typedef struct chm_model chm_model;
typedef struct chm_batch chm_batch;

/* Last error message of the calling thread ("" if none). */
const char* chm_last_error(void);

/* Version string of the library build. */
const char* chm_version(void);

/* Number of decoder parameter tensors chm_model_create expects for `dims`
 * (= len(CSPNet.state_dict()) for ln=True, smooth=False). */
int chm_num_params(const chm_dims* dims);

/* Builds the packed device copy of the decoder weights.
 * Replaces: CSPNet.__init__ + load_state_dict (cspnet.py:185-234).
 * d_params[i] points to the i-th state_dict tensor in this order (row-major,
 * contiguous, fp32, nn.Linear layout [out][in]):
 *   node_embedding.weight, film_layer.mlp_cond.0.{weight,bias},
 *   film_layer.proj.{weight,bias}, film_layer.norm.{weight,bias} (not when
 *   time_dim = text_dim = 0),
 *   for l in 0..L-1: csp_layer_l.{edge_mlp.0.weight, edge_mlp.0.bias,
 *     edge_mlp.2.weight, edge_mlp.2.bias, node_mlp.0.weight, node_mlp.0.bias,
 *     node_mlp.2.weight, node_mlp.2.bias, layer_norm.weight, layer_norm.bias},
 *   coord_out.weight, lattice_out.weight, type_out.{weight,bias},
 *   final_layer_norm.{weight,bias}.
 * Synchronises `stream` before returning. */
int chm_model_create(const chm_dims* dims, const float* const* d_params, int n_params, void* stream,
                     chm_model** out);
void chm_model_destroy(chm_model* m);

/* Launch-schedule options (not thread-safe against concurrent steps of the same model):
 *   "edge_split" (0 / 1): when edge layer 1's 256x256 tiles leave a partial last round of the
 *     grid, run that round in one grid with the edge-layer-2 tiles that do not read its rows.
 *   "edge16" (1): accepted for compatibility (the round-1 32x32x16 kernels were removed; 0 fails).
 *   "edge_rows", "edge_layer", "edge_layer_dyn", "edge_pool", "edge_lag", "edge_layer_min": edge-layer
 *     schedules (bit-identical). A batch plans its pair-grid job lists (and sizes their
 *     buffers) with the edge_lag of its creation: a later change reaches batches created after it only.
 *   "node_ps" (0 / 1): split16 node GEMMs read their A operands pre-split by the producing kernels (not
 *     bit-identical to 0: within fp32 rounding; DESIGN.md §4 "Node GEMMs"); a batch carves their buffers only
 *     when created while the option is set (batches created without it keep the in-loop split).
 *   "edge_pairs" (0 / 1, default 1): fc edge layer 1 computed once per unordered pair of atoms (the reverse
 *     edge's Fourier features are the forward ones with the sine half negated), both directions' messages
 *     from one GEMM row; within fp32 rounding of the directed form (DESIGN.md §4 "Edge layer 1 on pairs").
 *   "edge_pairs_layer" (0 / 1, default 1): with edge_pairs, both edge layers in one static grid from
 *     "edge_layer_min" row tiles on (k_edge16_pairs_grid; bit-identical to two launches).
 *   The persistent one-grid kernel (edge_layer_dyn) runs only where model creation saw 8 XCDs ("xcd_mask" =
 *     0xff); tests: "edge_dyn_skip_xcd" (its blocks on one XCD exit, the launch's self-check must raise the
 *     repair), "edge_layer_repair", "edge_tail_timeout", "edge_tail_norepair" (WRONG results after a
 *     timeout), "edge_rows_nowait", "edge_pairs_pq_global" (the pair epilogue's P / Q rows from global memory
 *     instead of LDS).
 * Returns CHM_E_ARG for an unknown key. */
int chm_model_set_option(chm_model* m, const char* key, int64_t value);

/* Arithmetic of the decoder GEMMs (all fp32-accurate, fp32 accumulation):
 *   CHM_MATH_SPLIT16 (default): the two edge GEMMs split each operand into an
 *     fp16 hi/lo pair (three fp16 MFMA products per fp32 product); W rows and
 *     activation rows carry power-of-two scales so every split operand is
 *     <= 1 in magnitude (the Fourier features already are; edge layer 1
 *     records max|S| per row for edge layer 2). Node GEMMs use bf16x3.
 *   CHM_MATH_BF16X3: every GEMM splits each operand into three bf16 parts,
 *     six bf16 MFMA products per fp32 product.
 *   CHM_MATH_F32: v_mfma_f32_32x32x2_f32 (exact fp32 fma chains); standalone
 *     aggregation kernel.
 * In the two split modes the edge message GEMM is fused with scatter_mean.
 * CHM_MATH=f32 / bf16x3 / split16 in the environment selects the mode at
 * creation. A batch keeps the mode its model had when the batch was created. */
#define CHM_MATH_BF16X3 0
#define CHM_MATH_F32 1
#define CHM_MATH_SPLIT16 2
int chm_model_set_math(chm_model* m, int mode);
int chm_model_get_math(const chm_model* m);

/* Describes a (possibly ragged) batch of crystals and owns the workspace of
 * its decoder calls. Replaces: Batch.from_data_list + the fc edge builder
 * (chemeleon.py:335-343, cspnet.py:319-324): node i of crystal g is global
 * node node_off[g] + i; the fully connected edges of crystal g are visited in
 * the reference's row-major (i, j) order, self loops included, but never
 * materialised as a dense N x N matrix. `max_pairs` is 1 (plain decoder
 * calls) or 2 (cond + null classifier-free-guidance pairs). */
int chm_batch_create(const chm_model* m, const int32_t* h_natoms, int num_graphs, int max_pairs, chm_batch** out);
void chm_batch_destroy(chm_batch* b);
/* Device bytes the batch uses (workspace + index tables). */
size_t chm_batch_device_bytes(const chm_batch* b);

/* Caller-owned workspace (SURVEY 8(b) Ownership): chm_batch_workspace_bytes returns the
 * device bytes a batch of these crystals needs with the model's current arithmetic (0 on bad
 * arguments), and chm_batch_create_with_workspace builds the batch inside the caller's
 * allocation d_workspace (>= that many bytes, 256-byte aligned; e.g. a block from the PyTorch
 * caching allocator). The index tables are uploaded on `stream`, which is synchronised before
 * return; the workspace must outlive the batch, and chm_batch_destroy never frees it. A batch
 * is scratch for one stream at a time: samplers that run concurrently on different streams use
 * different batches. */
size_t chm_batch_workspace_bytes(const chm_model* m, const int32_t* h_natoms, int num_graphs, int max_pairs);
int chm_batch_create_with_workspace(const chm_model* m, const int32_t* h_natoms, int num_graphs, int max_pairs,
                                    void* d_workspace, size_t workspace_bytes, void* stream, chm_batch** out);

/* Edge styles (CSPNet(edge_style=...), cspnet.py:319-343). CHM_EDGES_KNN is the reference's radius
 * graph (radius_graph_pbc + neighbour cap + symmetric reorder, data_utils.py:151-398,
 * cspnet.py:236-343; the reference needs torch_scatter's segment ops for it). Its edges depend on the
 * coordinates, so every decoder call of a knn batch rebuilds them on the device and synchronises
 * `stream` once to size the launches: knn batches cannot be captured into a graph. split16
 * arithmetic only. */
#define CHM_EDGES_FC 0
#define CHM_EDGES_KNN 1
typedef struct chm_batch_options {
  int32_t edge_style;          /* CHM_EDGES_FC (default) or CHM_EDGES_KNN */
  int32_t max_neighbors;       /* knn: max_num_neighbors_threshold (CSPNet max_neighbors, 20 in the shipped
                                  config); <= 0 keeps every pair within the radius, as the reference's
                                  get_max_neighbors_mask (data_utils.py:341-348) */
  int32_t knn_edges_per_atom;  /* knn: edge capacity per atom after symmetrisation (default 128); a
                                  decoder call whose graph has more edges fails with CHM_E_UNSUPPORTED */
  int32_t reserved;
} chm_batch_options;
/* chm_batch_workspace_bytes / chm_batch_create_with_workspace with options (NULL = fc defaults);
 * d_workspace NULL: the library allocates (as chm_batch_create). */
size_t chm_batch_workspace_bytes_ex(const chm_model* m, const int32_t* h_natoms, int num_graphs, int max_pairs,
                                    const chm_batch_options* opts);
int chm_batch_create_ex(const chm_model* m, const int32_t* h_natoms, int num_graphs, int max_pairs,
                        const chm_batch_options* opts, void* d_workspace, size_t workspace_bytes, void* stream,
                        chm_batch** out);
/* knn batches: build the edge list of these coordinates now (as a decoder call does) and copy it out,
 * grouped by source node in the reference's order within each node: d_src / d_dst [capacity] int32
 * global node indices, d_frac_diff [capacity, 3]; *n_edges = the edge count (nothing is copied when it
 * exceeds capacity). Any of the output pointers may be NULL. */
int chm_knn_edges(chm_batch* b, const float* d_frac, const float* d_lattices, int32_t* d_src, int32_t* d_dst,
                  float* d_frac_diff, int64_t capacity, int64_t* n_edges, void* stream);

/* One decoder call for `pairs` conditionings that share atom types,
 * coordinates and lattices (pairs = 1: CSPNet.forward, cspnet.py:345-405;
 * pairs = 2: the two calls of Chemeleon.model_predictions, chemeleon.py:258-285).
 *   d_atom_types [N] int64, d_frac [N,3], d_lattices [B,3,3]
 *   d_time_emb   [B,128] rows, row stride time_stride floats (0 = one row for all graphs)
 *   d_text       [pairs,B,text_dim] (row stride text_dim) or NULL if text_dim == 0
 * Outputs (any may be NULL to skip it):
 *   d_types_out [pairs,N,A], d_lattice_out [pairs,B,3,3], d_coords_out [pairs,N,3],
 *   d_node_out  [pairs,N,H] (final-LayerNorm node features). */
/* (A model created with time_dim = text_dim = 0 has no FilmLayer, cspnet.py:210-211: the reference's
 * CrystalClip graph encoder. Its parameter list omits the six film_layer.* tensors, d_time_emb may be
 * NULL, and it cannot sample.) */
int chm_decoder_forward(chm_batch* b, int pairs, const int64_t* d_atom_types, const float* d_frac,
                        const float* d_lattices, const float* d_time_emb, int time_stride, const float* d_text,
                        float* d_types_out, float* d_lattice_out, float* d_coords_out, float* d_node_out,
                        void* stream);

/* Training forward / validation loss (Chemeleon.forward, chemeleon.py:137-244) for a batch created
 * with max_pairs >= 1: q_sample of (d_a0, d_x0, d_l0) at the per-graph timesteps d_t [B] (int64,
 * 1..T) with the caller's noise (d_rand_a [N,A] uniforms, d_noise_l [B,3,3] normals already masked by
 * [[1,0,1],[1,1,1],[0,0,1]], d_noise_x [N,3] normals), one decoder call on the noised state with
 * d_time_emb [B,time_dim] and d_text [B,text_dim] (or NULL), then the D3PM hybrid loss, lattice and
 * coordinate MSEs. Tables (device fp32): d_coef4 [T+1][4] = {sqrt(abar_t), sqrt(1 - abar_t),
 * sigma_t, sigmas_norm_t}, d_q_one_step / d_q_mats [T+1][A][A] as in chm_schedule.
 * Outputs: d_out[6] = {loss, vb_loss, ce_loss, loss_atom_types, loss_lattice, loss_coords};
 * optional (NULL to skip) d_a_t [N] int64, d_x_t [N,3], d_l_t [B,3,3], d_target_x [N,3] (the score
 * target), d_pred_lattice [B,3,3], d_pred_coords [N,3]. */
typedef struct chm_train_tables {
  int T;
  const float* d_coef4;
  const float* d_q_one_step;
  const float* d_q_mats;
  float hybrid_coeff, cost_atom_types, cost_lattice, cost_coords;
} chm_train_tables;
int chm_training_loss(chm_batch* b, const chm_train_tables* tt, const int64_t* d_t, const int64_t* d_a0,
                      const float* d_x0, const float* d_l0, const float* d_time_emb, const float* d_text,
                      const float* d_rand_a, const float* d_noise_l, const float* d_noise_x, float* d_out,
                      int64_t* d_a_t, float* d_x_t, float* d_l_t, float* d_target_x, float* d_pred_lattice,
                      float* d_pred_coords, void* stream);

/* Per-timestep schedule tables (device, fp32), computed once by the host from
 * the reference schedules (diff_utils.py:57-131, chemeleon.py:413-457):
 *   d_coef [T+1][8]: {c0, c1, sigma_l, step_x, std_x, sqrt(sigma_norm),
 *                     step_lr*(sigma_t/sigma_begin)^2, sqrt(2*that)}
 *   d_time_emb [T+1][time_dim]: SinusoidalTimeEmbeddings(t) (cspnet.py:21-35)
 *   d_q_one_step, d_q_mats [T+1][A][A]: D3PM buffers (diff_utils.py:168-185)
 * num_classes (= A) and time_dim describe the tables; a step refuses a schedule
 * whose num_classes / time_dim differ from its batch's model (CHM_E_ARG). */
typedef struct {
  int T;
  int num_classes;
  int time_dim;
  int reserved;
  const float* d_coef;
  const float* d_time_emb;
  const float* d_q_one_step;
  const float* d_q_mats;
} chm_schedule;

/* The device buffers of one reverse step, each with its ELEMENT count. Every count is
 * checked against the batch (N nodes, B crystals) and its model (A = max_atoms classes,
 * text_dim) before anything is enqueued: a mis-sized buffer returns CHM_E_ARG with
 * chm_last_error() naming it, never an out-of-bounds access on the device.
 *   d_atom_types [N] int64, d_frac [N,3], d_lattices [B,3,3]: the state, updated in place;
 *   d_cond, d_null [B,text_dim]: conditioning vectors (NULL / 0 when text_dim = 0);
 *   parity-mode noise, all four or none (NULL: device Philox noise):
 *   d_rand_a [N,A] uniforms, d_rand_l [B,3,3], d_rand_x1 [N,3], d_rand_x2 [N,3] normals. */
typedef struct chm_step_io {
  int64_t* d_atom_types;
  int64_t n_atom_types;
  float* d_frac;
  int64_t n_frac;
  float* d_lattices;
  int64_t n_lattices;
  const float* d_cond;
  int64_t n_cond;
  const float* d_null;
  int64_t n_null;
  const float* d_rand_a;
  int64_t n_rand_a;
  const float* d_rand_l;
  int64_t n_rand_l;
  const float* d_rand_x1;
  int64_t n_rand_x1;
  const float* d_rand_x2;
  int64_t n_rand_x2;
} chm_step_io;

/* One reverse-diffusion step t -> t-1 of Chemeleon._sample_generator
 * (chemeleon.py:379-466): predictor CFG pair, D3PM atom-type sampling
 * (diff_utils.py:307-329), DDPM lattice update (clip at t == T), VE
 * predictor half step, corrector CFG pair, Langevin corrector, wrap to [0,1).
 * Buffers: `io` (state updated in place). With the four noise buffers the
 * host-drawn tensors of the reference's RNG stream are used (parity mode;
 * ignored at t == 1 as in the reference); without them noise comes from a
 * counter-based Philox generator keyed by (seed, t, global node / graph
 * index), so results do not depend on how samples are sharded across GPUs.
 * `node_base`/`graph_base` are the global indices of this batch's first
 * node / graph for that key. */
int chm_sample_step(chm_batch* b, const chm_schedule* sched, int t, float cond_scale, const chm_step_io* io,
                    uint64_t seed, int64_t node_base, int64_t graph_base, void* stream);

/* Graph-capturable form of chm_sample_step: t is read from device memory
 * (*d_t, int32) and decremented by the step's last kernel, so one captured
 * step (hipStreamBeginCapture ... hipGraphLaunch) replayed T times walks
 * t = T .. 1. Noise comes from the counter-based Philox generator only (the
 * noise buffers of `io` must be NULL). */
int chm_sample_step_dt(chm_batch* b, const chm_schedule* sched, int32_t* d_t, float cond_scale, const chm_step_io* io,
                       uint64_t seed, int64_t node_base, int64_t graph_base, void* stream);

/* The same with the noise read from the four fixed device buffers of `io` (required): the
 * caller refills them before every replay (the reference's CPU RNG stream drawn on the host and
 * copied in stream order), so parity-mode sampling also runs as one captured step. At t == 1 the
 * buffers are not read (their stale contents are finite uniforms / normals). */
int chm_sample_step_dt_noise(chm_batch* b, const chm_schedule* sched, int32_t* d_t, float cond_scale,
                             const chm_step_io* io, void* stream);

/* Standalone message-passing aggregation (scatter_mean of edge messages onto
 * their source node; chemeleon/utils/scatter.py:88-112 as called from
 * cspnet.py:155-160) over this batch's fc edge layout:
 *   d_msg [pairs,E,H] (msg_count elements) -> d_agg [pairs,N,H] (agg_count elements),
 *   agg[i] = sum_j msg[(i,j)] / max(n_g,1), H = hidden_dim (512); the counts must be
 * exactly pairs*E*H and pairs*N*H (CHM_E_ARG otherwise); fc batches only
 * (CHM_E_UNSUPPORTED for knn). */
int chm_segment_mean(chm_batch* b, int pairs, const float* d_msg, int64_t msg_count, float* d_agg, int64_t agg_count,
                     void* stream);

/* D3PM reverse sampling for explicit inputs (diff_utils.py:307-329):
 * d_logits [N,A], d_xt [N] int64, d_t [N] int64 per-node timestep,
 * d_noise [N,A] uniform -> d_out [N] int64. Tables as in chm_schedule.
 * Every t must lie in [1, T] and every x_t in [0, A) (the reference indexes its
 * tables with them and raises otherwise): the kernel checks them on the device,
 * and an out-of-range index makes the call return CHM_E_ARG with chm_last_error()
 * naming the first offending node (its d_out entry is -1). The check needs the
 * result, so this entry point synchronises `stream` before returning, except while
 * `stream` is capturing a graph: then nothing is read back and the call returns at
 * once; out-of-range nodes are the d_out entries of -1 (the flag word the check uses
 * is allocated per host thread and device by the first, uncaptured call:
 * CHM_E_UNSUPPORTED if the first call on a thread is captured). */
int chm_d3pm_sample(int N, int A, int T, const float* d_logits, const int64_t* d_xt, const int64_t* d_t,
                    const float* d_noise, const float* d_q_one_step, const float* d_q_mats, int64_t* d_out,
                    void* stream);

/* Test hooks for the perf-mode noise (the device Philox4x32-10 streams the step kernels draw
 * from; the reference draws torch.rand / torch.randn on its CPU generator instead,
 * chemeleon.py:400-404,418,435,455):
 *   chm_debug_philox: d_out[i] = uniform in [0,1) (normal = 0) or standard normal (normal = 1)
 *     of key (seed, t, kind, base + i); kind 0 atom-type uniforms, 1 lattice, 2 / 3 coordinates.
 *   chm_debug_d3pm_philox: chm_d3pm_sample with the Gumbel noise drawn from that stream (kind 0,
 *     index (node_base + node) * 128 + class), as the sampler does in perf mode. */
int chm_debug_philox(uint64_t seed, int t, int kind, int64_t base, int64_t n, int normal, float* d_out, void* stream);
int chm_debug_d3pm_philox(int N, int A, int T, const float* d_logits, const int64_t* d_xt, const int64_t* d_t,
                          const float* d_q_one_step, const float* d_q_mats, uint64_t seed, int64_t node_base,
                          int64_t* d_out, void* stream);

/* Host-only test hook (no device): the row tiles edge layer 2 runs on for an fc batch of these
 * crystals (EdgeArgs::rtiles; DESIGN.md "Edge layer 2 on row tiles"). Returns the tile count R (or a
 * negative CHM_E_*); if out4 holds >= 4 R int32 it receives per tile {first node starting in the tile,
 * first node starting after it, the node continued from the previous tile or -1, that node's row
 * offset in the continued-rows buffer}, and *r2tot the buffer's rows. */
int chm_debug_row_tiles(const int32_t* h_natoms, int B, int32_t* out4, int64_t cap4, int64_t* r2tot);
/* (host only) the row tiles' node lists (EdgeArgs::rinfo: kRowInfo = 260 {node, packed} pairs per tile) and
 * their lengths, as edge layer 2's segment-mean epilogue reads them; returns the number of row tiles */
int chm_debug_row_nodes(const int32_t* h_natoms, int B, int32_t* out2, int64_t cap2, int32_t* counts, int64_t cap);
/* The same two on a mixed row tiling (r6): tiles [0, nbig) of 256 edge rows, then tiles of 192 rows (nbig < 0: the
 * uniform tiling; CHM_E_ARG when the 256-row tiles leave no row). A batch takes such a tiling at creation when edge
 * layer 2 runs on the two-launch schedule (fewer than the option edge_layer_min row tiles, crystals of at most 192
 * atoms, split16, option edge_rows_short on) and its last round of 256-row tiles would be at most 3/4 full: that
 * round's rows then run as one round of 192-row tiles (k_edge16_short, a launch of their own). Bit-identical.
 * chm_debug_short_row_tiles: the nbig a batch of these crystals takes for P conditionings on a device of ncu CUs with
 * edge_layer_min = layer_min (-1: uniform); chm_batch_short_row_tiles: the one a created batch took. */
int chm_debug_row_tiles_ex(const int32_t* h_natoms, int B, int64_t nbig, int32_t* out4, int64_t cap4, int64_t* r2tot);
int chm_debug_row_nodes_ex(const int32_t* h_natoms, int B, int64_t nbig, int32_t* out2, int64_t cap2, int32_t* counts,
                           int64_t cap);
int64_t chm_debug_short_row_tiles(const int32_t* h_natoms, int B, int P, int ncu, int64_t layer_min);
int64_t chm_batch_short_row_tiles(const chm_batch* b);
/* Host-only test hook: the block -> job map of the one-grid edge-layer kernel (k_edge16_layer) for R
 * row tiles, P conditionings and layer-2 lag `lag`. Returns the grid size nb (or a negative CHM_E_*);
 * if out holds >= 2 nb int64 it receives per block {kind (0 none, 1 edge layer 1, 2 edge layer 2),
 * tile index (layer 1: row tile * 2 + column tile; layer 2: (row tile * P + conditioning) * 2 +
 * column tile)}. */
int64_t chm_debug_layer_jobs(int64_t R, int P, int lag, int64_t* out, int64_t cap);
/* The persistent form of that kernel (option edge_layer_dyn, the default from 1024 row tiles on): job k
 * of an XCD's sequence as out[3k] = kind (1 = layer 1, 2 = layer 2), out[3k+1] = the XCD's local row
 * (the first ones its static rows, the rest claimed from the shared pool at run time), out[3k+2] =
 * column tile (layer 1) or conditioning * 2 + column tile (layer 2), for k < n. */
int chm_debug_layer_seq(int64_t n, int P, int lag, int64_t* out);

/* Host-only test hook: the schedule of both edge layers in one static grid on pairs (k_edge16_pairs_grid; block
 * 8 k + x runs job k of list x) for an fc batch of these crystals, P conditionings and lag `lag` (pair tiles).
 * Returns the job-list stride J (or a negative CHM_E_*); when the buffers are large enough: rng [2 R] = per
 * layer-2 row tile the pair tiles [lo, hi] it reads, pa / pb [8] = list x's pair tiles [pa, pb), njobs [8],
 * jobs [8][J][2] = {kind
 * (1 pair, 2 layer 2), tile index (pair tile * 2 + column tile; (row tile * P + conditioning) * 2 + column
 * tile)}. */
int64_t chm_debug_pair_plan(const int32_t* h_natoms, int B, int P, int lag, int32_t* rng, int64_t cap_rng, int32_t* pa,
                            int32_t* pb, int32_t* njobs, int32_t* jobs, int64_t cap_jobs);
/* Host-only test hook: per pair tile (128 unordered pairs i <= j of an fc batch, crystal-major) the node range
 * [out[2k], out[2k] + out[2k+1]) whose P / Q rows its epilogue stages in LDS (edge layer 1 on pairs). Returns the
 * number of pair tiles (or a negative CHM_E_*); out is filled when cap >= 2 x that number. */
int64_t chm_debug_pair_nodes(const int32_t* h_natoms, int B, int32_t* out, int64_t cap);
/* Fourier edge features of this batch's fc edges (cspnet.py:38-52,324):
 * d_frac [N,3] -> d_feat [E, 6*num_freqs]. */
int chm_edge_features(chm_batch* b, const float* d_frac, float* d_feat, void* stream);
/* The same features in the form the split16 edge GEMM consumes (the sampler's k_fourier_h):
 * d_split [E, 6*num_freqs/32, 2, 32] fp16, per 32-column chunk the hi parts then the lo parts
 * (feature = hi + lo, |lo| <= 2^-11 |hi|); E * 6*num_freqs * 4 bytes. */
int chm_edge_features_split(chm_batch* b, const float* d_frac, void* d_split, void* stream);

/* Bench instrumentation: while enabled, the runtime brackets every launch of
 * the kernels below with HIP events on the launch stream (a pool of 8192
 * pairs; recording stops when it is exhausted). After synchronising the
 * device, chm_prof_read returns the launch count and summed duration.
 * Launches made while the stream is being captured into a graph are not
 * instrumented (time a graph by replaying it; time kernels eagerly).
 *   CHM_K_EDGE_FOURIER  edge layer 1 (Fourier projection + node terms + SiLU)
 *   CHM_K_EDGE_MESSAGE  edge layer 2 (message GEMM + SiLU)
 *   CHM_K_SEGMENT_MEAN  message-passing aggregation (scatter_mean)
 *   CHM_K_DECODER       one whole decoder call (all its kernels)
 *   CHM_K_EDGE_LAYER    both edge layers of a CSP layer in one grid (k_edge16_layer + its repair pair) */
#define CHM_K_EDGE_FOURIER 0
#define CHM_K_EDGE_MESSAGE 1
#define CHM_K_SEGMENT_MEAN 2
#define CHM_K_DECODER 3
#define CHM_K_EDGE_LAYER 4
int chm_prof_enable(int on);
int chm_prof_reset(void);
int chm_prof_read(int kernel, int64_t* launches, double* total_ms);
/* Health counters of the edge kernels, counted on the device over every launch and graph replay
 * since the last chm_prof_events_reset (synchronous device reads; not while capturing):
 *   out[CHM_EV_LAYER_TIMEOUT]  k_edge16_layer: layer-2 tiles whose wait for their layer-1 tiles timed out
 *   out[CHM_EV_LAYER_XCD]      k_edge16_layer: layer-2 tiles whose layer-1 tiles ran on another XCD
 *   out[CHM_EV_LAYER_REPAIR]   k_edge16_layer launches recomputed by their repair pair
 *   out[CHM_EV_TAIL_TIMEOUT]   k_edge16_tail: segment tiles whose wait for this grid's layer-1 tiles timed out
 *   out[CHM_EV_TAIL_REPAIR]    k_edge16_tail launches whose edge layer 2 was recomputed
 *   out[CHM_EV_LAYER_INCOMPLETE] k_edge16_layer_dyn launches that ended with layer-2 tiles not computed (an
 *                              XCD missing: the persistent kernel's static rows assume 8 XCDs; repaired)
 * Results never depend on these (a raised check is repaired before the layer's output is used); a
 * non-zero count means the run paid for the repairs. n <= 8 values are written. */
#define CHM_EV_LAYER_TIMEOUT 0
#define CHM_EV_LAYER_XCD 1
#define CHM_EV_LAYER_REPAIR 2
#define CHM_EV_TAIL_TIMEOUT 3
#define CHM_EV_TAIL_REPAIR 4
#define CHM_EV_LAYER_INCOMPLETE 5
int chm_prof_events(int64_t* out, int n);
int chm_prof_events_reset(void);

/* Host-only (no device): parity-mode atom-type noise for a shard of a sample-parallel run. Continues
 * the MT19937 stream of the CPU torch generator (state[624], left, next as in ATen's
 * mt19937_engine, i.e. the words of torch.Generator.get_state()) over `count` float uniforms, the
 * stream torch.rand(count) draws (chemeleon.py:400-404: one 32-bit output y per element,
 * (y & (2^24 - 1)) * 2^-24), and writes only elements [lo, hi) to out[hi - lo]. state / left / next
 * are advanced in place. Replaces, per rank: torch.rand(N, A)[rows of this shard]. */
int chm_mt19937_uniform(uint32_t* state, int32_t* left, int32_t* next, int64_t count, int64_t lo, int64_t hi,
                        float* out);

/* Sizes of the batch (for callers that allocate outputs). */
int64_t chm_batch_num_nodes(const chm_batch* b);
int64_t chm_batch_num_edges(const chm_batch* b);

/* The model dimensions behind a batch and its sizes (any pointer may be NULL): *dims = the
 * model's chm_dims, *num_graphs = B, *max_pairs = the pairs it was created for, *knn = 1 for a
 * knn-edge batch. Callers that allocate outputs or validate shapes use it (the torch-op layer,
 * chemeleon_amd/csrc/torch_ops.cpp, checks every tensor against it before a launch). */
int chm_batch_info(const chm_batch* b, chm_dims* dims, int64_t* num_graphs, int* max_pairs, int* knn);
/* The HIP device ordinal the batch (and its model) lives on: every buffer passed with the batch
 * must be memory of that device (the torch-op layer checks each tensor's device against it and
 * launches under a device guard for it). Negative CHM_E_ARG for a NULL batch. */
int chm_batch_device(const chm_batch* b);

#ifdef __cplusplus
}
#endif
#endif /* CHEMELEON_HIP_H */
