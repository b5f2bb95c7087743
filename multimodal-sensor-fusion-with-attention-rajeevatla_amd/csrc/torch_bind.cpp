// mmf_torch: the eager module path's autograd nodes in C++ (libtorch), over libmmfusion.so's C-ABI.
//
// HybridFusion.forward in eager mode (src/fusion.py:344-427, called from src/train.py's step) and
// the criterion nn.CrossEntropyLoss(label_smoothing) (src/train.py:185-186) are, at the reference's
// 2-D inputs, a handful of short HIP launches each: the step is bound by the host work around them.
// This module is that host work without Python: HybridFusion's forward records one C++ autograd
// node whose backward writes every parameter gradient straight into the module's flat gradient
// buffer (the grad sink: parameters outside the autograd graph, their .grad the buffer's views),
// and the cross-entropy forward records one node holding the kernel's d loss / d logits.  Same
// semantics as mmf_ops.HybridSink / CrossEntropyEager (the Python twins, used when this module is
// not built): same entry points, same buffers, same gradient modes.
//
// The library's entry points come in by address from the Python loader (mmf_native.lib(): the
// library the rest of the package calls, MMF_LIB_PATH overrides included) -- this module links
// libtorch only.  No compute here: every kernel is libmmfusion.so's.

#include <torch/extension.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/functions/utils.h>
#include <torch/csrc/autograd/graph_task.h>
#include <torch/csrc/autograd/saved_variable.h>
#include <torch/csrc/autograd/variable.h>
#include <c10/hip/HIPStream.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mmfusion.h"

namespace {

using torch::autograd::Node;
using torch::autograd::SavedVariable;
using torch::autograd::variable_list;

// ---------------------------------------------------------------------------------- entry points
struct Api {
  size_t (*saved_bytes)(const mmf_hybrid_desc*) = nullptr;
  size_t (*ws_bytes)(const mmf_hybrid_desc*) = nullptr;
  int (*fwd)(const mmf_hybrid_desc*, const mmf_hybrid_params*, const float* const*, const float*,
             const uint64_t*, void*, float*, float*, float* const*, void*) = nullptr;
  int (*bwd)(const mmf_hybrid_desc*, const mmf_hybrid_params*, const float* const*, const float*, const void*,
             const float*, void*, const mmf_hybrid_grads*, float* const*, void*) = nullptr;
  int (*ce)(int32_t, int32_t, const float*, const int64_t*, float, float, float*, float*, void*) = nullptr;
  const char* (*last_error)() = nullptr;
};
Api g_api;

template <typename F>
void bind_one(F& f, const py::dict& a, const char* name) {
  if (!a.contains(name)) throw std::runtime_error(std::string("mmf_torch.bind: missing ") + name);
  f = reinterpret_cast<F>(a[name].cast<uintptr_t>());
}

void bind(const py::dict& a) {
  bind_one(g_api.saved_bytes, a, "mmf_hybrid_saved_bytes");
  bind_one(g_api.ws_bytes, a, "mmf_hybrid_workspace_bytes");
  bind_one(g_api.fwd, a, "mmf_hybrid_forward");
  bind_one(g_api.bwd, a, "mmf_hybrid_backward");
  bind_one(g_api.ce, a, "mmf_cross_entropy_ls");
  bind_one(g_api.last_error, a, "mmf_last_error");
}

void need_api() {
  if (!g_api.fwd) throw std::runtime_error("mmf_torch: library entry points not bound (mmf_ops.torch_ext())");
}

void check(int rc, const char* what) {
  if (rc != 0) {
    const char* msg = g_api.last_error ? g_api.last_error() : "";
    throw std::runtime_error(std::string("mmfusion ") + what + " failed (code " + std::to_string(rc) +
                             "): " + (msg ? msg : ""));
  }
}

void* stream_of(const at::Tensor& t) {
  // (a host tensor -- the CPU unit tests bind stub entry points -- has no stream)
  if (!t.is_cuda()) return nullptr;
  return static_cast<void*>(c10::hip::getCurrentHIPStream(t.device().index()).stream());
}

// ------------------------------------------------------------------------------------ grad sink
// The flat gradient buffer of one HybridFusion module (mmf_ops.GradSink's layout: the operator's
// parameter order, 256-byte-aligned offsets given by the caller) and the parameters' pointer table.
struct Sink {
  std::vector<at::Tensor> params;
  std::vector<int64_t> offsets;
  int64_t nelem = 0;
  int M = 0, P = 0;
  at::Tensor flat;
  std::vector<at::Tensor> views;
  bool fresh = true;
  mmf_hybrid_params pstruct{};
  std::vector<const void*> pptrs;

  Sink(std::vector<at::Tensor> ps, std::vector<int64_t> offs, int64_t n, int m, int p)
      : params(std::move(ps)), offsets(std::move(offs)), nelem(n), M(m), P(p) {
    if (params.empty() || params.size() != offsets.size() || (int64_t)params.size() != 2 * (M + 4 * P + M + 2))
      throw std::runtime_error("mmf_torch.Sink: parameter list does not match (M, P)");
    for (size_t i = 0; i < params.size(); ++i)
      if (offsets[i] + params[i].numel() > nelem) throw std::runtime_error("mmf_torch.Sink: offsets overflow");
    flat = at::zeros({nelem}, params[0].options().dtype(at::kFloat));
    views.reserve(params.size());
    for (size_t i = 0; i < params.size(); ++i)
      views.push_back(flat.as_strided(params[i].sizes(), params[i].strides(), offsets[i]));
    pptrs.assign(params.size(), nullptr);
  }

  // the C-ABI parameter table, rebuilt when an address moved (p.data = ..., a reallocation)
  const mmf_hybrid_params* table() {
    bool same = true;
    for (size_t i = 0; i < params.size(); ++i)
      if (params[i].data_ptr() != pptrs[i]) { same = false; break; }
    if (!same) {
      for (size_t i = 0; i < params.size(); ++i) pptrs[i] = params[i].data_ptr();
      size_t k = 0;
      auto lin = [&](mmf_linear& l) {
        l.w = static_cast<const float*>(pptrs[k++]);
        l.b = static_cast<const float*>(pptrs[k++]);
      };
      for (int m = 0; m < M; ++m) lin(pstruct.proj[m]);
      for (int g = 0; g < P; ++g) { lin(pstruct.q[g]); lin(pstruct.k[g]); lin(pstruct.v[g]); lin(pstruct.o[g]); }
      for (int m = 0; m < M; ++m) lin(pstruct.gate[m]);
      lin(pstruct.cls1);
      lin(pstruct.cls2);
    }
    return &pstruct;
  }

  // the gradient table of a flat buffer in this layout
  mmf_hybrid_grads grads_in(const at::Tensor& buf) const {
    mmf_hybrid_grads g{};
    float* base = buf.data_ptr<float>();
    size_t k = 0;
    auto lin = [&](mmf_linear_grad& l) {
      l.w = base + offsets[k++];
      l.b = base + offsets[k++];
    };
    for (int m = 0; m < M; ++m) lin(g.proj[m]);
    for (int q = 0; q < P; ++q) { lin(g.q[q]); lin(g.k[q]); lin(g.v[q]); lin(g.o[q]); }
    for (int m = 0; m < M; ++m) lin(g.gate[m]);
    lin(g.cls1);
    lin(g.cls2);
    return g;
  }

  // the node keeps autograd's semantics for these parameters: every one trainable and none with a
  // tensor hook (register_hook can rewrite a gradient before accumulation: those modules go through
  // the per-parameter path, mmf_ops.HybridEager); post-accumulate hooks the node calls itself.
  // Nor may anything observe the parameters' AccumulateGrad nodes: hooks on an existing grad
  // accumulator (DistributedDataParallel's reducer registers its all-reduce there; those never run
  // when the node writes the gradients itself) send the module to the per-parameter path as well.
  // Conservative: a parameter whose hooks were all removed keeps an empty hook wrapper here, so
  // false sends the caller to the exact Python check (mmf_ops._sink_ok)
  bool ok() const {
    for (const auto& p : params)
      if (!p.requires_grad() || !torch::autograd::impl::hooks(p).empty()) return false;
    return !accumulator_hooked();
  }
  // a hook on some parameter's AccumulateGrad node (the exact Python check cannot see these)
  bool accumulator_hooked() const {
    for (const auto& p : params) {
      const auto acc = torch::autograd::impl::try_get_grad_accumulator(p);
      if (acc && (!acc->post_hooks().empty() || !acc->pre_hooks().empty() || !acc->tensor_pre_hooks().empty()))
        return true;
    }
    return false;
  }

  bool matches(const std::vector<at::Tensor>& ps) const {
    return ps.size() == params.size() && ps[0].device() == flat.device();
  }

  // a trainer applied the gradients: true iff every .grad is this buffer's view (then the next
  // backward writes afresh, the attributes stay); harness.DPTrainer resets them otherwise
  bool consumed() {
    for (size_t i = 0; i < params.size(); ++i)
      if (!params[i].grad().is_same(views[i])) return false;
    fresh = true;
    return true;
  }
};

// ------------------------------------------------------------------------------ HybridFusion node
struct HybridSinkBackward : public Node {
  std::shared_ptr<Sink> sink;
  mmf_hybrid_desc desc{};
  SavedVariable mask_;
  std::vector<SavedVariable> xs_;
  at::Tensor saved_;   // the forward's saved bytes (never an output: no reference cycle)
  std::vector<uint32_t> versions_;   // the parameters' version counters at the forward

  std::string name() const override { return "HybridSinkBackward"; }

  void release_variables() override {
    mask_.reset_data();
    for (auto& x : xs_) x.reset_data();
    saved_.reset();
  }

  variable_list apply(variable_list&& grads) override {
    const size_t nx = xs_.size();
    variable_list out(nx);
    if (grads.empty() || !grads[0].defined()) return out;
    if (!saved_.defined())
      throw std::runtime_error(
          "Trying to backward through the graph a second time (or directly access saved tensors after they "
          "have already been freed). Specify retain_graph=True if you need to backward a second time.");
    const at::Tensor dl = grads[0].contiguous();
    const at::Tensor mask = mask_.unpack();
    std::vector<at::Tensor> xs;
    xs.reserve(nx);
    for (auto& x : xs_) xs.push_back(x.unpack());
    Sink& s = *sink;
    const auto& params = s.params;
    const size_t np = params.size();
    // what autograd checks for a saved tensor: a weight modified in place between the forward and
    // this backward would otherwise be read silently
    for (size_t i = 0; i < np; ++i)
      if (params[i]._version() != versions_[i])
        throw std::runtime_error(
            "one of the variables needed for gradient computation has been modified by an inplace operation: "
            "HybridFusion parameter " + std::to_string(i) + " (shape " + c10::str(params[i].sizes()) + ") is at version " +
            std::to_string(params[i]._version()) + "; expected version " + std::to_string(versions_[i]) +
            " instead.");
    // a graph task that asks for some inputs only (torch.autograd.grad(out, inputs), backward(inputs=...))
    // must leave every parameter's .grad alone: the parameter gradients go to a scratch buffer
    const auto* exec_info = torch::autograd::get_current_graph_task_exec_info();
    const bool partial = exec_info && !exec_info->empty();
    // gradient mode (mmf_ops.HybridSink.backward): 0 write into the sink (every .grad None, or the
    // sink's views after a trainer consumed them); 1 add into the sink (its views hold gradients
    // still to be applied); 2 someone else's .grad tensors: add into them; 3 discard (partial task)
    bool all_none = true, all_view_or_none = true, all_view = true;
    for (size_t i = 0; i < np; ++i) {
      const at::Tensor& g = params[i].grad();
      if (g.defined()) all_none = false;
      const bool v = g.defined() && g.is_same(s.views[i]);
      if (!v) all_view = false;
      if (g.defined() && !v) all_view_or_none = false;
    }
    const int mode = partial ? 3 : (all_none || (s.fresh && all_view_or_none)) ? 0 : all_view ? 1 : 2;
    at::Tensor dst = mode == 0 ? s.flat : at::zeros({s.nelem}, s.flat.options());
    at::Tensor ws = at::empty({(int64_t)g_api.ws_bytes(&desc)}, mask.options().dtype(at::kByte));
    desc.workspace_capacity = (uint64_t)ws.numel();   // (saved_capacity and plan_flags: the forward's)
    const float* xp[MMF_MAX_MODALITIES] = {};
    float* dxp[MMF_MAX_MODALITIES] = {};
    for (size_t m = 0; m < nx; ++m) {
      xp[m] = xs[m].data_ptr<float>();
      if (should_compute_output(m)) {
        out[m] = at::empty_like(xs[m]);
        dxp[m] = out[m].data_ptr<float>();
      }
    }
    const mmf_hybrid_grads gt = s.grads_in(dst);
    check(g_api.bwd(&desc, s.table(), xp, mask.data_ptr<float>(), saved_.data_ptr(), dl.data_ptr<float>(),
                    ws.data_ptr(), &gt, dxp, stream_of(dl)),
          "HybridFusion backward");
    if (mode == 3) return out;   // (no parameter gradient, no post-accumulate hook: not accumulated)
    if (mode == 0) {
      for (size_t i = 0; i < np; ++i) {
        at::Tensor p = params[i];
        if (!p.grad().defined()) p.mutable_grad() = s.views[i];
      }
      s.fresh = false;
    } else if (mode == 1) {
      s.flat.add_(dst);
    } else {
      std::vector<at::Tensor> have, add;
      for (size_t i = 0; i < np; ++i) {
        at::Tensor p = params[i];
        at::Tensor v = dst.as_strided(p.sizes(), p.strides(), s.offsets[i]);
        if (p.grad().defined()) {
          have.push_back(p.grad());
          add.push_back(v);
        } else {
          p.mutable_grad() = v;
        }
      }
      if (!have.empty()) at::_foreach_add_(have, add);
    }
    // what AccumulateGrad does after accumulating
    for (size_t i = 0; i < np; ++i) {
      auto& hook = torch::autograd::impl::post_acc_grad_hooks(params[i]);
      if (hook) (*hook)(params[i]);
    }
    return out;
  }
};

// forward: -> [logits, fusion_weights, attention maps...].  desc_addr: a mmf_hybrid_desc the caller
// keeps (copied here); rng_state advanced in place by the library; mask (B, M) and xs fp32
// contiguous on the parameters' device (HybridFusion._forward checked them).
std::vector<at::Tensor> hybrid_sink_forward(const std::shared_ptr<Sink>& sink, uintptr_t desc_addr,
                                            const at::Tensor& rng_state, const at::Tensor& mask,
                                            const std::vector<at::Tensor>& xs) {
  need_api();
  mmf_hybrid_desc d = *reinterpret_cast<const mmf_hybrid_desc*>(desc_addr);   // (a copy: capacities set here)
  Sink& s = *sink;
  const int M = d.num_modalities, P = d.num_pairs;
  if ((int)xs.size() != M || M != s.M || P != s.P || M > MMF_MAX_MODALITIES)
    throw std::runtime_error("mmf_torch.hybrid_sink_forward: inputs do not match the descriptor");
  c10::DeviceGuard guard(mask.device());
  const auto f32 = mask.options().dtype(at::kFloat);
  at::Tensor saved = at::empty({(int64_t)g_api.saved_bytes(&d)}, mask.options().dtype(at::kByte));
  d.saved_capacity = (uint64_t)saved.numel();
  std::vector<at::Tensor> outs;
  outs.reserve(2 + (d.return_attention ? P : 0));
  outs.push_back(at::empty({d.batch, d.num_classes}, f32));
  outs.push_back(at::empty({d.batch, M}, f32));
  float* mp[MMF_MAX_PAIRS] = {};
  if (d.return_attention) {
    for (int g = 0; g < P; ++g) {
      const int64_t lq = std::max(d.seq_len[d.pair_q[g]], 1), lk = std::max(d.seq_len[d.pair_k[g]], 1);
      outs.push_back(at::empty({d.batch, d.num_heads, lq, lk}, f32));
      mp[g] = outs.back().data_ptr<float>();
    }
  }
  const float* xp[MMF_MAX_MODALITIES] = {};
  for (int m = 0; m < M; ++m) xp[m] = xs[m].data_ptr<float>();
  check(g_api.fwd(&d, s.table(), xp, mask.data_ptr<float>(),
                  rng_state.defined() ? static_cast<const uint64_t*>(rng_state.data_ptr()) : nullptr,
                  saved.data_ptr(), outs[0].data_ptr<float>(), outs[1].data_ptr<float>(),
                  d.return_attention ? mp : nullptr, stream_of(mask)),
        "HybridFusion forward");
  if (at::GradMode::is_enabled()) {
    // edges to the modality inputs only: the parameters are outside the graph (the node writes
    // their gradients itself), and logits has this node as grad_fn even when no input requires grad
    auto node = std::shared_ptr<HybridSinkBackward>(new HybridSinkBackward(), torch::autograd::deleteNode);
    node->set_next_edges(torch::autograd::collect_next_edges(xs));
    node->sink = sink;
    node->desc = d;
    node->mask_ = SavedVariable(mask, false);
    node->xs_.reserve(M);
    for (int m = 0; m < M; ++m) node->xs_.emplace_back(xs[m], false);
    node->saved_ = saved;
    node->versions_.reserve(s.params.size());
    for (const auto& p : s.params) node->versions_.push_back(p._version());
    torch::autograd::set_history(outs[0], node);
  }
  return outs;
}

// ------------------------------------------------------------------------------ cross-entropy node
struct CrossEntropyBackward : public Node {
  at::Tensor dlogits;
  std::string name() const override { return "CrossEntropyBackward"; }
  void release_variables() override { dlogits.reset(); }
  variable_list apply(variable_list&& grads) override {
    variable_list out(1);
    if (grads.empty() || !grads[0].defined()) return out;
    if (!dlogits.defined()) throw std::runtime_error("Trying to backward through the graph a second time");
    if (should_compute_output(0)) out[0] = dlogits * grads[0];
    return out;
  }
};

// nn.CrossEntropyLoss(label_smoothing=eps), reduction "mean", ignore_index -100 (mmf_ops.cross_entropy)
at::Tensor cross_entropy(const at::Tensor& logits, const at::Tensor& labels, double eps) {
  need_api();
  c10::DeviceGuard guard(logits.device());
  const int64_t B = logits.size(0), C = logits.size(1);
  at::Tensor loss = at::empty({}, logits.options());
  at::Tensor dlogits = at::empty({B, C}, logits.options());
  check(g_api.ce((int32_t)B, (int32_t)C, logits.data_ptr<float>(), labels.data_ptr<int64_t>(), (float)eps, 1.f,
                 loss.data_ptr<float>(), dlogits.data_ptr<float>(), stream_of(logits)),
        "CrossEntropyLoss(label_smoothing)");
  if (at::GradMode::is_enabled() && logits.requires_grad()) {
    auto node = std::shared_ptr<CrossEntropyBackward>(new CrossEntropyBackward(), torch::autograd::deleteNode);
    node->set_next_edges(torch::autograd::collect_next_edges(logits));
    node->dlogits = dlogits;
    torch::autograd::set_history(loss, node);
  }
  return loss;
}

}  // namespace

PYBIND11_MODULE(mmf_torch, m) {
  m.doc() = "HybridFusion / cross-entropy autograd nodes in C++ over libmmfusion.so (eager module path)";
  m.def("bind", &bind, "hand over the library's entry points: {name: address}");
  py::class_<Sink, std::shared_ptr<Sink>>(m, "Sink")
      .def(py::init<std::vector<at::Tensor>, std::vector<int64_t>, int64_t, int, int>())
      .def_readonly("flat", &Sink::flat)
      .def_readonly("views", &Sink::views)
      .def_readonly("offsets", &Sink::offsets)
      .def_readonly("nelem", &Sink::nelem)
      .def_readwrite("fresh", &Sink::fresh)
      .def("matches", &Sink::matches)
      .def("ok", &Sink::ok)
      .def("accumulator_hooked", &Sink::accumulator_hooked)
      .def("consumed", &Sink::consumed);
  m.def("hybrid_sink_forward", &hybrid_sink_forward);
  m.def("cross_entropy", &cross_entropy);
}
