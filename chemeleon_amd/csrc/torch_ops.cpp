// The torch-op layer over the C ABI (SURVEY.md §8(b) "torch op wrapper"): the sampling path's entry
// points registered as `torch.ops.chemeleon.*` (TORCH_LIBRARY), so torch-native callers (TorchScript,
// torch.compile graphs, C++ frontends) reach the same kernels as the ctypes binding:
//   * every launch goes on the caller's current HIP stream (c10::hip::getCurrentHIPStream());
//   * outputs are allocated through the PyTorch caching allocator (at::empty on the inputs' device);
//   * shapes, devices and dtypes are checked on the host before any launch, and a failing C-ABI call
//     raises through TORCH_CHECK with chm_last_error() (RuntimeError in Python).
// Model and batch objects stay the library's (int64 handles from chm_model_create / chm_batch_create,
// which chemeleon_amd.modules.cspnet.HipModel / HipBatch own); the reference's interfaces these replace:
// CSPNet.forward (chemeleon/modules/cspnet.py:345-405), one reverse step of Chemeleon._sample_generator
// (chemeleon/modules/chemeleon.py:379-466), scatter_mean (chemeleon/utils/scatter.py:88-112) and
// D3PM.p_logits (chemeleon/utils/diff_utils.py:307-329).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <tuple>

#include "../../include/chemeleon_hip.h"

namespace {

void* stream() { return (void*)c10::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed (code ", rc, "): ", chm_last_error()); }

void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, ": chemeleon ops run on a HIP device only (no CPU fallback)");
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected ", dt, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": expected a contiguous tensor");
}

const float* fptr(const c10::optional<at::Tensor>& t, const char* name) {
  if (!t.has_value()) return nullptr;
  need(*t, at::kFloat, name);
  return t->data_ptr<float>();
}

// A batch handle with its model's dimensions: every tensor is checked against these on the host before a
// launch (the kernels trust their sizes: a mis-sized tensor would be an out-of-bounds access on the device)
struct Batch {
  chm_batch* b;
  chm_dims d;
  int64_t N, E, B;
  int P, knn;
};

Batch batch_of(int64_t handle) {
  TORCH_CHECK(handle != 0, "batch handle is 0");
  Batch r{};
  r.b = reinterpret_cast<chm_batch*>(handle);
  check(chm_batch_info(r.b, &r.d, &r.B, &r.P, &r.knn), "chm_batch_info");
  r.N = chm_batch_num_nodes(r.b);
  r.E = chm_batch_num_edges(r.b);
  return r;
}

void need_shape(const at::Tensor& t, at::IntArrayRef shape, const char* name) {
  TORCH_CHECK(t.sizes() == shape, name, ": expected shape ", shape, ", got ", t.sizes());
}

void need_state(const Batch& b, const at::Tensor& a, const at::Tensor& x, const at::Tensor& l) {
  need(a, at::kLong, "atom_types");
  need(x, at::kFloat, "frac");
  need(l, at::kFloat, "lattices");
  need_shape(a, {b.N}, "atom_types");
  need_shape(x, {b.N, 3}, "frac");
  need_shape(l, {b.B, 3, 3}, "lattices");
  TORCH_CHECK(a.device() == x.device() && a.device() == l.device(), "state tensors on different devices");
}

// CSPNet.forward for `pairs` conditionings sharing atoms / coordinates / lattices (pairs = 2: the CFG pair
// of Chemeleon.model_predictions): time_emb [B, >= time_dim] (row stride = its last size), text
// [pairs, B, text_dim] -> (types [pairs,N,max_atoms], lattice [pairs,B,3,3], coords [pairs,N,3],
// node features [pairs,N,hidden_dim])
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> decoder_forward(int64_t batch, int64_t pairs,
                                                                           const at::Tensor& atom_types,
                                                                           const at::Tensor& frac,
                                                                           const at::Tensor& lattices,
                                                                           const c10::optional<at::Tensor>& time_emb,
                                                                           const c10::optional<at::Tensor>& text) {
  const Batch b = batch_of(batch);
  TORCH_CHECK(pairs >= 1 && pairs <= b.P, "pairs must be in [1, ", b.P, "] for this batch");
  need_state(b, atom_types, frac, lattices);
  const bool film = b.d.time_dim > 0 || b.d.text_dim > 0;
  int64_t tstride = 0;
  if (film) {
    TORCH_CHECK(time_emb.has_value(), "time_emb is required (the model has a FiLM layer)");
    TORCH_CHECK(time_emb->dim() == 2 && time_emb->size(0) == b.B && time_emb->size(1) >= b.d.time_dim,
                "time_emb must be [B, >= time_dim]");
    tstride = time_emb->size(1);
  }
  if (b.d.text_dim > 0) {
    TORCH_CHECK(text.has_value(), "text embeddings are required (text_dim > 0)");
    need_shape(*text, {pairs, b.B, b.d.text_dim}, "text");
  }
  auto o = frac.options();
  at::Tensor types = at::empty({pairs, b.N, b.d.max_atoms}, o), latt = at::empty({pairs, b.B, 3, 3}, o),
             coords = at::empty({pairs, b.N, 3}, o), nodes = at::empty({pairs, b.N, b.d.hidden_dim}, o);
  check(chm_decoder_forward(b.b, (int)pairs, atom_types.data_ptr<int64_t>(), frac.data_ptr<float>(),
                            lattices.data_ptr<float>(), film ? fptr(time_emb, "time_emb") : nullptr, (int)tstride,
                            b.d.text_dim > 0 ? fptr(text, "text") : nullptr, types.data_ptr<float>(),
                            latt.data_ptr<float>(), coords.data_ptr<float>(), nodes.data_ptr<float>(), stream()),
        "chm_decoder_forward");
  return {types, latt, coords, nodes};
}

// One reverse step t -> t-1, state updated in place. `schedule` is the address of a chm_schedule (the
// device tables of Chemeleon.schedule_tables); noise tensors given: the reference's CPU stream (parity
// mode), absent: device Philox noise keyed by (seed, t, global index).
void sample_step(int64_t batch, int64_t schedule, int64_t t, double cond_scale, at::Tensor atom_types,
                 at::Tensor frac, at::Tensor lattices, const c10::optional<at::Tensor>& cond,
                 const c10::optional<at::Tensor>& null, const c10::optional<at::Tensor>& rand_a,
                 const c10::optional<at::Tensor>& rand_l, const c10::optional<at::Tensor>& rand_x1,
                 const c10::optional<at::Tensor>& rand_x2, int64_t seed, int64_t node_base, int64_t graph_base) {
  const Batch b = batch_of(batch);
  TORCH_CHECK(b.P >= 2, "sample_step needs a batch created for 2 pairs (the CFG pair)");
  TORCH_CHECK(schedule != 0, "schedule is 0");
  need_state(b, atom_types, frac, lattices);
  const bool guide = b.d.text_dim > 0;
  TORCH_CHECK(cond.has_value() == guide && null.has_value() == guide,
              guide ? "cond and null text embeddings are required" : "this model takes no text embeddings");
  if (guide) {
    need_shape(*cond, {b.B, b.d.text_dim}, "cond");
    need_shape(*null, {b.B, b.d.text_dim}, "null");
  }
  const bool noise = rand_a.has_value();
  TORCH_CHECK(noise == rand_l.has_value() && noise == rand_x1.has_value() && noise == rand_x2.has_value(),
              "pass all four noise tensors (parity mode) or none (device noise)");
  if (noise) {
    need_shape(*rand_a, {b.N, b.d.max_atoms}, "rand_a");
    need_shape(*rand_l, {b.B, 3, 3}, "rand_l");
    need_shape(*rand_x1, {b.N, 3}, "rand_x1");
    need_shape(*rand_x2, {b.N, 3}, "rand_x2");
  }
  check(chm_sample_step(b.b, reinterpret_cast<const chm_schedule*>(schedule), (int)t, (float)cond_scale,
                        atom_types.data_ptr<int64_t>(), frac.data_ptr<float>(), lattices.data_ptr<float>(),
                        fptr(cond, "cond"), fptr(null, "null"), fptr(rand_a, "rand_a"), fptr(rand_l, "rand_l"),
                        fptr(rand_x1, "rand_x1"), fptr(rand_x2, "rand_x2"), (uint64_t)seed, node_base, graph_base,
                        stream()),
        "chm_sample_step");
}

// scatter_mean of per-edge messages [pairs,E,hidden_dim] onto their source nodes -> [pairs,N,hidden_dim]
at::Tensor segment_mean(int64_t batch, int64_t pairs, const at::Tensor& msg) {
  const Batch b = batch_of(batch);
  TORCH_CHECK(!b.knn, "segment_mean: fc batches only");
  TORCH_CHECK(pairs >= 1, "pairs must be >= 1");
  need(msg, at::kFloat, "msg");
  need_shape(msg, {pairs, b.E, b.d.hidden_dim}, "msg");
  at::Tensor agg = at::empty({pairs, b.N, b.d.hidden_dim}, msg.options());
  check(chm_segment_mean(b.b, (int)pairs, msg.data_ptr<float>(), agg.data_ptr<float>(), stream()), "chm_segment_mean");
  return agg;
}

// D3PM reverse sampling (Gumbel argmax of the posterior logits) for explicit inputs -> [N] int64
at::Tensor d3pm_sample(const at::Tensor& logits, const at::Tensor& xt, const at::Tensor& t, const at::Tensor& noise,
                       const at::Tensor& q_one_step, const at::Tensor& q_mats) {
  need(logits, at::kFloat, "logits");
  need(xt, at::kLong, "x_t");
  need(t, at::kLong, "t");
  need(noise, at::kFloat, "noise");
  need(q_one_step, at::kFloat, "q_one_step");
  need(q_mats, at::kFloat, "q_mats");
  TORCH_CHECK(logits.dim() == 2 && noise.sizes() == logits.sizes(), "logits / noise must be [N, A]");
  const int64_t N = logits.size(0), A = logits.size(1);
  TORCH_CHECK(A >= 1 && A <= 128, "at most 128 classes");
  TORCH_CHECK(xt.numel() == N && t.numel() == N, "x_t / t must have N entries");
  TORCH_CHECK(q_mats.dim() == 3 && q_mats.size(1) == A && q_mats.size(2) == A && q_one_step.sizes() == q_mats.sizes(),
              "q tables must be [T+1, A, A]");
  at::Tensor out = at::empty({N}, xt.options());
  check(chm_d3pm_sample((int)N, (int)A, (int)q_mats.size(0) - 1, logits.data_ptr<float>(), xt.data_ptr<int64_t>(),
                        t.data_ptr<int64_t>(), noise.data_ptr<float>(), q_one_step.data_ptr<float>(),
                        q_mats.data_ptr<float>(), out.data_ptr<int64_t>(), stream()),
        "chm_d3pm_sample");
  return out;
}

}  // namespace

TORCH_LIBRARY(chemeleon, m) {
  m.def("decoder_forward(int batch, int pairs, Tensor atom_types, Tensor frac, Tensor lattices, Tensor? time_emb, "
        "Tensor? text) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("sample_step(int batch, int schedule, int t, float cond_scale, Tensor(a!) atom_types, Tensor(b!) frac, "
        "Tensor(c!) lattices, Tensor? cond, Tensor? null, Tensor? rand_a, Tensor? rand_l, Tensor? rand_x1, "
        "Tensor? rand_x2, int seed, int node_base, int graph_base) -> ()");
  m.def("segment_mean(int batch, int pairs, Tensor msg) -> Tensor");
  m.def("d3pm_sample(Tensor logits, Tensor x_t, Tensor t, Tensor noise, Tensor q_one_step, Tensor q_mats) -> Tensor");
}

TORCH_LIBRARY_IMPL(chemeleon, CUDA, m) {
  m.impl("decoder_forward", decoder_forward);
  m.impl("sample_step", sample_step);
  m.impl("segment_mean", segment_mean);
  m.impl("d3pm_sample", d3pm_sample);
}
