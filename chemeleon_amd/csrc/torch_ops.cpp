// The torch-op layer over the C ABI (SURVEY.md §8(b) "torch op wrapper"): the sampling path's objects and
// entry points registered with the dispatcher (TORCH_LIBRARY), so torch-native callers (TorchScript, C++
// frontends, torch.compile graphs) build and drive the sampler without the Python ctypes binding:
//   * torch.classes.chemeleon.Model / Batch / Schedule (torch::CustomClassHolder, reference-counted): the
//     packed decoder weights (chm_model), a crystal batch with its workspace (chm_batch; it holds its Model),
//     and the per-timestep tables (chm_schedule; it holds its tensors). An op takes these objects, never a raw
//     address, so nothing it reads can be freed under it;
//   * every launch goes on the current HIP stream of the batch's device, under a device guard for that
//     device; every tensor must live on that device (checked on the host before any launch);
//   * a Batch is scratch for one stream at a time: an op on another stream than the batch's last one first
//     makes its stream wait for the last one's work (an event) and records the workspace as used on it
//     (record_stream), so uses on several streams are ordered and the caching allocator reuses the
//     workspace only after every stream that used it is done;
//   * outputs and workspaces come from the PyTorch caching allocator (at::empty);
//   * shapes, dtypes and devices are checked on the host, the C ABI checks element counts again, and a
//     failing call raises through TORCH_CHECK with chm_last_error() (RuntimeError in Python).
// The reference interfaces these replace: CSPNet.__init__ / load_state_dict and CSPNet.forward
// (chemeleon/modules/cspnet.py:185-234, 345-405), one reverse step of Chemeleon._sample_generator
// (chemeleon/modules/chemeleon.py:379-466) with its schedule buffers (chemeleon/utils/diff_utils.py:57-185),
// scatter_mean (chemeleon/utils/scatter.py:88-112) and D3PM.p_logits (chemeleon/utils/diff_utils.py:307-329).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <hip/hip_runtime_api.h>

#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/chemeleon_hip.h"

namespace {

using c10::hip::HIPGuardMasqueradingAsCUDA;

void* stream() { return (void*)c10::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed (code ", rc, "): ", chm_last_error()); }

void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, ": chemeleon ops run on a HIP device only (no CPU fallback)");
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected ", dt, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": expected a contiguous tensor");
}

void need_on(const at::Tensor& t, const c10::Device& dev, at::ScalarType dt, const char* name) {
  need(t, dt, name);
  TORCH_CHECK(t.device() == dev, name, " is on ", t.device(), ", the batch on ", dev);
}

void need_shape(const at::Tensor& t, at::IntArrayRef shape, const char* name) {
  TORCH_CHECK(t.sizes() == shape, name, ": expected shape ", shape, ", got ", t.sizes());
}

// ---------------------------------------------------------------- objects
struct Model : torch::CustomClassHolder {
  chm_model* m = nullptr;
  chm_dims d{};
  c10::Device device{c10::kCUDA, 0};

  // params: the decoder's state_dict tensors in order (chm_model_create), fp32 contiguous on one HIP device
  Model(std::vector<at::Tensor> params, int64_t hidden_dim, int64_t time_dim, int64_t text_dim, int64_t num_layers,
        int64_t max_atoms, int64_t num_freqs) {
    TORCH_CHECK(!params.empty(), "Model: no parameter tensors");
    device = params[0].device();
    for (size_t i = 0; i < params.size(); ++i) need_on(params[i], device, at::kFloat, "Model parameter");
    d = chm_dims{(int)hidden_dim, (int)time_dim, (int)text_dim, (int)num_layers, (int)max_atoms, (int)num_freqs};
    HIPGuardMasqueradingAsCUDA guard(device);
    std::vector<const float*> ptrs;
    for (auto& p : params) ptrs.push_back(p.data_ptr<float>());
    check(chm_model_create(&d, ptrs.data(), (int)ptrs.size(), stream(), &m), "chm_model_create");
  }
  ~Model() override {
    if (m) chm_model_destroy(m);
  }
  void set_math(const std::string& mode) {
    const int code = mode == "split16" ? CHM_MATH_SPLIT16 : mode == "bf16x3" ? CHM_MATH_BF16X3 : mode == "f32" ? CHM_MATH_F32 : -1;
    TORCH_CHECK(code >= 0, "set_math: 'split16', 'bf16x3' or 'f32', got '", mode, "'");
    check(chm_model_set_math(m, code), "chm_model_set_math");
  }
  std::string get_math() const {
    const int c = chm_model_get_math(m);
    return c == CHM_MATH_SPLIT16 ? "split16" : c == CHM_MATH_BF16X3 ? "bf16x3" : "f32";
  }
  void set_option(const std::string& key, int64_t value) { check(chm_model_set_option(m, key.c_str(), value), "chm_model_set_option"); }
};

struct Batch : torch::CustomClassHolder {
  c10::intrusive_ptr<Model> model;  // the weights outlive every batch built on them
  at::Tensor workspace;             // caller-owned workspace (caching allocator), freed after the batch
  chm_batch* b = nullptr;
  int64_t N = 0, E = 0, B = 0;
  int P = 0, knn = 0;
  std::mutex mu;                    // guards last / ev (ops from several host threads)
  hipStream_t last = nullptr;       // the stream of the last op on this batch (creation: its stream)
  hipEvent_t ev = nullptr;

  // natoms: atoms per crystal; max_pairs 1 (plain decoder calls) or 2 (CFG pairs, sampling); knn: the
  // reference's radius graph instead of fc edges (max_neighbors as CSPNet's)
  Batch(c10::intrusive_ptr<Model> model_, std::vector<int64_t> natoms, int64_t max_pairs, bool knn_edges,
        int64_t max_neighbors)
      : model(std::move(model_)) {
    TORCH_CHECK(!natoms.empty(), "Batch: natoms is empty");
    std::vector<int32_t> nat;
    for (int64_t n : natoms) {
      TORCH_CHECK(n >= 1 && n <= (1 << 20), "Batch: atoms per crystal must be in [1, 2^20], got ", n);
      nat.push_back((int32_t)n);
    }
    chm_batch_options opts{knn_edges ? CHM_EDGES_KNN : CHM_EDGES_FC, (int32_t)max_neighbors, 0, 0};
    const size_t need_b = chm_batch_workspace_bytes_ex(model->m, nat.data(), (int)nat.size(), (int)max_pairs, &opts);
    TORCH_CHECK(need_b > 0, "chm_batch_workspace_bytes_ex failed: ", chm_last_error());
    HIPGuardMasqueradingAsCUDA guard(model->device);
    workspace = at::empty({(int64_t)need_b}, at::TensorOptions().dtype(at::kByte).device(model->device));
    check(chm_batch_create_ex(model->m, nat.data(), (int)nat.size(), (int)max_pairs, &opts, workspace.data_ptr(), need_b,
                              stream(), &b),
          "chm_batch_create_ex");
    chm_dims d;
    check(chm_batch_info(b, &d, &B, &P, &knn), "chm_batch_info");
    TORCH_CHECK(chm_batch_device(b) == model->device.index(), "Batch: the library placed the batch on device ",
                chm_batch_device(b), ", the model is on ", model->device);
    N = chm_batch_num_nodes(b);
    E = chm_batch_num_edges(b);
    last = (hipStream_t)stream();
    TORCH_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess, "Batch: hipEventCreate failed");
  }
  ~Batch() override {
    if (b) chm_batch_destroy(b);
    if (ev) (void)hipEventDestroy(ev);
  }
  // called under the device guard, before an op launches on the current stream: order it behind the work of the
  // batch's last stream and keep the workspace alive for this stream (caching allocator)
  void use_current_stream() {
    // (the CUDA-typed view of the HIP stream: PyTorch-ROCm's caching allocator keys streams as CUDA)
    const c10::hip::HIPStreamMasqueradingAsCUDA cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA();
    std::lock_guard<std::mutex> lk(mu);
    if (cur.stream() == last) return;
    TORCH_CHECK(hipEventRecord(ev, last) == hipSuccess && hipStreamWaitEvent(cur.stream(), ev, 0) == hipSuccess,
                "Batch: ordering the batch's previous stream before this one failed");
    workspace.record_stream(cur.unwrap());
    last = cur.stream();
  }
  const chm_dims& dims() const { return model->d; }
  const c10::Device& device() const { return model->device; }
  int64_t num_nodes() const { return N; }
  int64_t num_edges() const { return E; }
  int64_t num_graphs() const { return B; }
};

struct Schedule : torch::CustomClassHolder {
  at::Tensor coef, time_emb, q_one_step, q_mats;  // held: chm_schedule points into them
  chm_schedule s{};

  // coef [T+1, 8], time_emb [T+1, time_dim], q_one_step / q_mats [T+1, A, A] (Chemeleon.schedule_tables)
  Schedule(at::Tensor coef_, at::Tensor time_emb_, at::Tensor q_one_step_, at::Tensor q_mats_)
      : coef(std::move(coef_)), time_emb(std::move(time_emb_)), q_one_step(std::move(q_one_step_)),
        q_mats(std::move(q_mats_)) {
    const c10::Device dev = coef.device();
    need_on(coef, dev, at::kFloat, "coef");
    need_on(time_emb, dev, at::kFloat, "time_emb");
    need_on(q_one_step, dev, at::kFloat, "q_one_step");
    need_on(q_mats, dev, at::kFloat, "q_mats");
    TORCH_CHECK(coef.dim() == 2 && coef.size(1) == 8 && coef.size(0) >= 2, "coef must be [T+1, 8]");
    const int64_t T1 = coef.size(0);
    TORCH_CHECK(time_emb.dim() == 2 && time_emb.size(0) == T1, "time_emb must be [T+1, time_dim]");
    TORCH_CHECK(q_mats.dim() == 3 && q_mats.size(0) == T1 && q_mats.size(1) == q_mats.size(2) &&
                    q_one_step.sizes() == q_mats.sizes(),
                "q_one_step / q_mats must be [T+1, A, A]");
    s.T = (int)(T1 - 1);
    s.num_classes = (int)q_mats.size(1);
    s.time_dim = (int)time_emb.size(1);
    s.d_coef = coef.data_ptr<float>();
    s.d_time_emb = time_emb.data_ptr<float>();
    s.d_q_one_step = q_one_step.data_ptr<float>();
    s.d_q_mats = q_mats.data_ptr<float>();
  }
  int64_t num_timesteps() const { return s.T; }
};

// ---------------------------------------------------------------- ops
void need_state(const Batch& b, const at::Tensor& a, const at::Tensor& x, const at::Tensor& l) {
  need_on(a, b.device(), at::kLong, "atom_types");
  need_on(x, b.device(), at::kFloat, "frac");
  need_on(l, b.device(), at::kFloat, "lattices");
  need_shape(a, {b.N}, "atom_types");
  need_shape(x, {b.N, 3}, "frac");
  need_shape(l, {b.B, 3, 3}, "lattices");
}

const float* fptr_on(const c10::optional<at::Tensor>& t, const Batch& b, const char* name) {
  if (!t.has_value()) return nullptr;
  need_on(*t, b.device(), at::kFloat, name);
  return t->data_ptr<float>();
}

// CSPNet.forward for `pairs` conditionings sharing atoms / coordinates / lattices (pairs = 2: the CFG pair
// of Chemeleon.model_predictions): time_emb [B, >= time_dim] (row stride = its last size), text
// [pairs, B, text_dim] -> (types [pairs,N,max_atoms], lattice [pairs,B,3,3], coords [pairs,N,3],
// node features [pairs,N,hidden_dim])
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> decoder_forward(const c10::intrusive_ptr<Batch>& bp,
                                                                           int64_t pairs, const at::Tensor& atom_types,
                                                                           const at::Tensor& frac,
                                                                           const at::Tensor& lattices,
                                                                           const c10::optional<at::Tensor>& time_emb,
                                                                           const c10::optional<at::Tensor>& text) {
  const Batch& b = *bp;
  const chm_dims& d = b.dims();
  TORCH_CHECK(pairs >= 1 && pairs <= b.P, "pairs must be in [1, ", b.P, "] for this batch");
  need_state(b, atom_types, frac, lattices);
  const bool film = d.time_dim > 0 || d.text_dim > 0;
  int64_t tstride = 0;
  if (film) {
    TORCH_CHECK(time_emb.has_value(), "time_emb is required (the model has a FiLM layer)");
    TORCH_CHECK(time_emb->dim() == 2 && time_emb->size(0) == b.B && time_emb->size(1) >= d.time_dim,
                "time_emb must be [B, >= time_dim]");
    tstride = time_emb->size(1);
  }
  if (d.text_dim > 0) {
    TORCH_CHECK(text.has_value(), "text embeddings are required (text_dim > 0)");
    need_shape(*text, {pairs, b.B, d.text_dim}, "text");
  }
  const float* te = film ? fptr_on(time_emb, b, "time_emb") : nullptr;
  const float* tx = d.text_dim > 0 ? fptr_on(text, b, "text") : nullptr;
  HIPGuardMasqueradingAsCUDA guard(b.device());
  bp->use_current_stream();
  auto o = frac.options();
  at::Tensor types = at::empty({pairs, b.N, d.max_atoms}, o), latt = at::empty({pairs, b.B, 3, 3}, o),
             coords = at::empty({pairs, b.N, 3}, o), nodes = at::empty({pairs, b.N, d.hidden_dim}, o);
  check(chm_decoder_forward(b.b, (int)pairs, atom_types.data_ptr<int64_t>(), frac.data_ptr<float>(),
                            lattices.data_ptr<float>(), te, (int)tstride, tx, types.data_ptr<float>(),
                            latt.data_ptr<float>(), coords.data_ptr<float>(), nodes.data_ptr<float>(), stream()),
        "chm_decoder_forward");
  return {types, latt, coords, nodes};
}

// One reverse step t -> t-1, state updated in place. Noise tensors given: the reference's CPU stream
// (parity mode); absent: device Philox noise keyed by (seed, t, global index).
void sample_step(const c10::intrusive_ptr<Batch>& bp, const c10::intrusive_ptr<Schedule>& sp, int64_t t,
                 double cond_scale, at::Tensor atom_types, at::Tensor frac, at::Tensor lattices,
                 const c10::optional<at::Tensor>& cond, const c10::optional<at::Tensor>& null,
                 const c10::optional<at::Tensor>& rand_a, const c10::optional<at::Tensor>& rand_l,
                 const c10::optional<at::Tensor>& rand_x1, const c10::optional<at::Tensor>& rand_x2, int64_t seed,
                 int64_t node_base, int64_t graph_base) {
  const Batch& b = *bp;
  const Schedule& sc = *sp;
  const chm_dims& d = b.dims();
  TORCH_CHECK(b.P >= 2, "sample_step needs a batch created for 2 pairs (the CFG pair)");
  TORCH_CHECK(sc.coef.device() == b.device(), "schedule is on ", sc.coef.device(), ", the batch on ", b.device());
  TORCH_CHECK(sc.s.num_classes == d.max_atoms && sc.s.time_dim == d.time_dim, "schedule tables (A = ", sc.s.num_classes,
              ", time_dim = ", sc.s.time_dim, ") do not match the model (", d.max_atoms, ", ", d.time_dim, ")");
  TORCH_CHECK(t >= 1 && t <= sc.s.T, "t must be in [1, ", sc.s.T, "]");
  need_state(b, atom_types, frac, lattices);
  const bool guide = d.text_dim > 0;
  TORCH_CHECK(cond.has_value() == guide && null.has_value() == guide,
              guide ? "cond and null text embeddings are required" : "this model takes no text embeddings");
  if (guide) {
    need_shape(*cond, {b.B, d.text_dim}, "cond");
    need_shape(*null, {b.B, d.text_dim}, "null");
  }
  const bool noise = rand_a.has_value();
  TORCH_CHECK(noise == rand_l.has_value() && noise == rand_x1.has_value() && noise == rand_x2.has_value(),
              "pass all four noise tensors (parity mode) or none (device noise)");
  if (noise) {
    need_shape(*rand_a, {b.N, d.max_atoms}, "rand_a");
    need_shape(*rand_l, {b.B, 3, 3}, "rand_l");
    need_shape(*rand_x1, {b.N, 3}, "rand_x1");
    need_shape(*rand_x2, {b.N, 3}, "rand_x2");
  }
  chm_step_io io{};
  io.d_atom_types = atom_types.data_ptr<int64_t>(); io.n_atom_types = atom_types.numel();
  io.d_frac = frac.data_ptr<float>(); io.n_frac = frac.numel();
  io.d_lattices = lattices.data_ptr<float>(); io.n_lattices = lattices.numel();
  io.d_cond = fptr_on(cond, b, "cond"); io.n_cond = guide ? cond->numel() : 0;
  io.d_null = fptr_on(null, b, "null"); io.n_null = guide ? null->numel() : 0;
  io.d_rand_a = fptr_on(rand_a, b, "rand_a"); io.n_rand_a = noise ? rand_a->numel() : 0;
  io.d_rand_l = fptr_on(rand_l, b, "rand_l"); io.n_rand_l = noise ? rand_l->numel() : 0;
  io.d_rand_x1 = fptr_on(rand_x1, b, "rand_x1"); io.n_rand_x1 = noise ? rand_x1->numel() : 0;
  io.d_rand_x2 = fptr_on(rand_x2, b, "rand_x2"); io.n_rand_x2 = noise ? rand_x2->numel() : 0;
  HIPGuardMasqueradingAsCUDA guard(b.device());
  bp->use_current_stream();
  check(chm_sample_step(b.b, &sc.s, (int)t, (float)cond_scale, &io, (uint64_t)seed, node_base, graph_base, stream()),
        "chm_sample_step");
}

// scatter_mean of per-edge messages [pairs,E,hidden_dim] onto their source nodes -> [pairs,N,hidden_dim]
at::Tensor segment_mean(const c10::intrusive_ptr<Batch>& bp, int64_t pairs, const at::Tensor& msg) {
  const Batch& b = *bp;
  TORCH_CHECK(!b.knn, "segment_mean: fc batches only");
  TORCH_CHECK(pairs >= 1, "pairs must be >= 1");
  need_on(msg, b.device(), at::kFloat, "msg");
  need_shape(msg, {pairs, b.E, b.dims().hidden_dim}, "msg");
  HIPGuardMasqueradingAsCUDA guard(b.device());
  bp->use_current_stream();
  at::Tensor agg = at::empty({pairs, b.N, b.dims().hidden_dim}, msg.options());
  check(chm_segment_mean(b.b, (int)pairs, msg.data_ptr<float>(), msg.numel(), agg.data_ptr<float>(), agg.numel(),
                         stream()),
        "chm_segment_mean");
  return agg;
}

// D3PM reverse sampling (Gumbel argmax of the posterior logits) for explicit inputs -> [N] int64. t and x_t are
// range-checked on the device (the call synchronises the stream); an out-of-range index raises.
at::Tensor d3pm_sample(const at::Tensor& logits, const at::Tensor& xt, const at::Tensor& t, const at::Tensor& noise,
                       const at::Tensor& q_one_step, const at::Tensor& q_mats) {
  const c10::Device dev = logits.device();
  need_on(logits, dev, at::kFloat, "logits");
  need_on(xt, dev, at::kLong, "x_t");
  need_on(t, dev, at::kLong, "t");
  need_on(noise, dev, at::kFloat, "noise");
  need_on(q_one_step, dev, at::kFloat, "q_one_step");
  need_on(q_mats, dev, at::kFloat, "q_mats");
  TORCH_CHECK(logits.dim() == 2 && noise.sizes() == logits.sizes(), "logits / noise must be [N, A]");
  const int64_t N = logits.size(0), A = logits.size(1);
  TORCH_CHECK(A >= 1 && A <= 128, "at most 128 classes");
  TORCH_CHECK(xt.numel() == N && t.numel() == N, "x_t / t must have N entries");
  TORCH_CHECK(q_mats.dim() == 3 && q_mats.size(1) == A && q_mats.size(2) == A && q_one_step.sizes() == q_mats.sizes(),
              "q tables must be [T+1, A, A]");
  HIPGuardMasqueradingAsCUDA guard(dev);
  at::Tensor out = at::empty({N}, xt.options());
  check(chm_d3pm_sample((int)N, (int)A, (int)q_mats.size(0) - 1, logits.data_ptr<float>(), xt.data_ptr<int64_t>(),
                        t.data_ptr<int64_t>(), noise.data_ptr<float>(), q_one_step.data_ptr<float>(),
                        q_mats.data_ptr<float>(), out.data_ptr<int64_t>(), stream()),
        "chm_d3pm_sample");
  return out;
}

}  // namespace

TORCH_LIBRARY(chemeleon, m) {
  m.class_<Model>("Model")
      .def(torch::init<std::vector<at::Tensor>, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>())
      .def("set_math", &Model::set_math)
      .def("get_math", &Model::get_math)
      .def("set_option", &Model::set_option);
  m.class_<Batch>("Batch")
      .def(torch::init<c10::intrusive_ptr<Model>, std::vector<int64_t>, int64_t, bool, int64_t>())
      .def("num_nodes", &Batch::num_nodes)
      .def("num_edges", &Batch::num_edges)
      .def("num_graphs", &Batch::num_graphs);
  m.class_<Schedule>("Schedule")
      .def(torch::init<at::Tensor, at::Tensor, at::Tensor, at::Tensor>())
      .def("num_timesteps", &Schedule::num_timesteps);
  m.def("decoder_forward(__torch__.torch.classes.chemeleon.Batch batch, int pairs, Tensor atom_types, Tensor frac, "
        "Tensor lattices, Tensor? time_emb, Tensor? text) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("sample_step(__torch__.torch.classes.chemeleon.Batch batch, __torch__.torch.classes.chemeleon.Schedule "
        "schedule, int t, float cond_scale, Tensor(a!) atom_types, Tensor(b!) frac, Tensor(c!) lattices, Tensor? cond, "
        "Tensor? null, Tensor? rand_a, Tensor? rand_l, Tensor? rand_x1, Tensor? rand_x2, int seed, int node_base, "
        "int graph_base) -> ()");
  m.def("segment_mean(__torch__.torch.classes.chemeleon.Batch batch, int pairs, Tensor msg) -> Tensor");
  m.def("d3pm_sample(Tensor logits, Tensor x_t, Tensor t, Tensor noise, Tensor q_one_step, Tensor q_mats) -> Tensor");
}

TORCH_LIBRARY_IMPL(chemeleon, CUDA, m) {
  m.impl("decoder_forward", decoder_forward);
  m.impl("sample_step", sample_step);
  m.impl("segment_mean", segment_mean);
  m.impl("d3pm_sample", d3pm_sample);
}
