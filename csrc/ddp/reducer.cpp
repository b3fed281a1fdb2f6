#include "reducer.h"

#include "../comm/stream_sync.h"

#include <c10/hip/HIPGuard.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>

#include <c10/hip/HIPStream.h>

#include <cstdlib>
#include <stdexcept>

#include "../kernels/kernels.h"

namespace py = pybind11;

namespace pdt {

struct ReducerState {
  std::vector<at::Tensor> params;
  std::vector<at::Tensor> views;
  std::vector<int64_t> bucket_of;
  std::vector<at::Tensor> flats;
  std::vector<std::vector<int64_t>> members;  // params per bucket
  std::shared_ptr<RcclComm> comm;
  std::shared_ptr<XgmiComm> xgmi;  // direct xGMI reduce-scatter/all-gather backend (instead of comm)
  std::vector<int64_t> flat_off;   // per bucket: element offset in the xGMI gradient buffer
  py::object py_launch, py_finalize;
  bool average = true;
  bool wire_bf16 = false;
  std::vector<at::Tensor> wire;  // bf16 staging per bucket (lazy)

  std::vector<std::shared_ptr<torch::autograd::Node>> accumulators;

  // comm timing (RCCL and xGMI paths): first bucket start / last bucket end on the comm stream, and
  // the end of backward compute on the caller's stream -> all-reduce time and its exposed tail
  bool timing = false;
  bool timed = false;  // events of the last finished iteration are valid
  hipEvent_t ev_start = nullptr, ev_end = nullptr, ev_bwd = nullptr;
  // debug: a gradient marked ready again after its bucket's all-reduce was issued means a kernel
  // wrote into memory an in-flight collective reads -> error instead of a silent race
  bool strict = false;
  int64_t duplicate_marks = 0;
  // diagnostics only (PDT_REDUCER_SKIP_COLL=1): keep every stream wait/event of the RCCL path
  // but issue no collective -- separates RCCL's own cost from the ordering's cost
  bool skip_collectives = false;
  // side stream that produces some gradients (weight-gradient GEMMs run there, concurrent with
  // the input-gradient chain): every bucket all-reduce also waits for it
  hipStream_t aux = nullptr;
  hipEvent_t ev_aux = nullptr;

  // LOCAL mode: one process, no communicator -- the optimizer-overlap stream only
  bool local = false;
  bool tail_on_cur = false;  // this iteration's last bucket was updated on the caller's stream
  bool tail_local = false;   // A/B: keep the last bucket on the overlap stream (PDT_TAIL_LOCAL=1)
  hipStream_t local_stream = nullptr;
  hipEvent_t ev_local = nullptr, ev_join = nullptr;
  // per-bucket fused SGD (optimizer in backward)
  float* sgd_p = nullptr;
  const float* grad_base = nullptr;
  at::Tensor grad_flat;          // for its version counter
  std::vector<int64_t> goff;     // element offset of each bucket in the flat buffers
  bool sgd_armed = false;
  float sgd_lr = 0.f, sgd_mom = 0.f, sgd_damp = 0.f, sgd_wd = 0.f;
  bool sgd_nest = false, sgd_first = false;
  float* sgd_buf = nullptr;
  uint16_t* sgd_pb = nullptr;
  int64_t sgd_applied = 0;
  std::pair<int64_t, int64_t> sgd_last{-1, -1};

  std::mutex mu;
  bool enabled = true;
  bool expecting = false;
  bool callback_queued = false;
  std::vector<int64_t> pending;
  std::vector<char> param_ready;
  std::vector<char> bucket_ready;
  int64_t next_launch = 0;
  std::vector<int64_t> launch_order, last_order;
  int64_t iters = 0;

  void reset_counters() {
    pending.assign(flats.size(), 0);
    for (size_t b = 0; b < flats.size(); ++b) pending[b] = (int64_t)members[b].size();
    param_ready.assign(params.size(), 0);
    bucket_ready.assign(flats.size(), 0);
    next_launch = 0;
    launch_order.clear();
  }

  // the fused SGD over bucket b's flat range, on stream s behind its reduction
  void apply_sgd(int64_t b, hipStream_t s) {
    if (!sgd_armed) return;
    const int64_t off = goff[b];
    launch_sgd(sgd_p + off, grad_base + off, sgd_buf ? sgd_buf + off : nullptr, flats[b].numel(), sgd_lr,
               sgd_mom, sgd_damp, sgd_wd, sgd_nest, sgd_first, 1.f, s, sgd_pb ? sgd_pb + off : nullptr);
    ++sgd_applied;
  }

  void launch_bucket(int64_t b) {
    const bool first = launch_order.empty();
    launch_order.push_back(b);
    if (local) {
      if (!sgd_armed) return;  // nothing to reduce in one process: only the update runs here
      const int dev = params[0].get_device();
      c10::hip::HIPGuard guard((c10::DeviceIndex)dev);
      hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
      if (b + 1 == (int64_t)flats.size() && !tail_local) {
        // the last bucket (stem / layer-1 gradients, final at the very end of backward): its update
        // runs on the caller's stream behind one wait for the side stream.  On the overlap stream it
        // cost two unsatisfied cross-queue waits on the step's critical tail (overlap stream waits
        // for the side stream, then the caller's stream for the overlap stream: ~50 us each, r9a)
        if (aux) stream_handoff(aux, cur, ev_aux);
        if (timing) {
          hipEventRecord(ev_bwd, cur);
          if (first) hipEventRecord(ev_start, cur);
        }
        apply_sgd(b, cur);
        tail_on_cur = true;
        return;
      }
      stream_handoff(cur, local_stream, ev_local);
      if (aux) stream_handoff(aux, local_stream, ev_aux);
      if (timing && first) hipEventRecord(ev_start, local_stream);
      apply_sgd(b, local_stream);
      return;
    }
    if (xgmi) {
      xgmi->check();  // a peer timed out earlier: raise here, out of backward()
      c10::hip::HIPGuard guard((c10::DeviceIndex)xgmi->device());
      xgmi->comm_wait_current();
      if (aux) {
        stream_handoff(aux, xgmi->stream(), ev_aux);
      }
      if (timing && first) hipEventRecord(ev_start, xgmi->stream());
      xgmi->reduce_bucket((int)b, flat_off[b], flats[b].numel(), average);
      apply_sgd(b, xgmi->stream());
      return;
    }
    if (comm) {
      comm->check();  // a timed-out / failed communicator: raise here, out of backward()
      const at::Tensor& f = flats[b];
      c10::hip::HIPGuard guard((c10::DeviceIndex)comm->device());
      comm->comm_wait_current();
      hipStream_t cs = comm->stream();
      if (aux) {
        stream_handoff(aux, cs, ev_aux);
      }
      if (timing && first) hipEventRecord(ev_start, cs);
      if (wire_bf16) {
        if (!wire[b].defined())
          wire[b] = at::empty({f.numel()}, f.options().dtype(at::kBFloat16));
        launch_cast_f32_bf16(f.data_ptr<float>(), reinterpret_cast<uint16_t*>(wire[b].data_ptr()),
                             f.numel(), cs);
        comm->all_reduce_raw(wire[b].data_ptr(), (size_t)f.numel(), ncclBfloat16, ncclSum);
        float scale = average ? 1.f / (float)comm->world() : 1.f;
        launch_cast_bf16_f32(reinterpret_cast<const uint16_t*>(wire[b].data_ptr()),
                             f.data_ptr<float>(), f.numel(), scale, cs);
      } else if (!skip_collectives) {
        comm->all_reduce_raw(f.data_ptr(), (size_t)f.numel(), RcclComm::dtype_of(f),
                             average ? ncclAvg : ncclSum);
      }
      apply_sgd(b, cs);
    } else {
      if (aux) {
        // device gradients through a non-RCCL group (gloo on GPU tensors): the collective runs
        // behind the caller's stream, so that stream joins the side stream first
        const int dev = params[0].get_device();
        c10::hip::HIPGuard guard((c10::DeviceIndex)dev);
        hipEventRecord(ev_aux, aux);
        hipStreamWaitEvent(c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream(), ev_aux, 0);
      }
      py::gil_scoped_acquire gil;
      py_launch(b);
    }
  }

  void launch_ready_in_order() {
    while (next_launch < (int64_t)flats.size() && bucket_ready[next_launch]) {
      launch_bucket(next_launch);
      ++next_launch;
    }
  }

  void mark_param(int64_t idx, bool zero_if_missing) {
    if (param_ready[idx]) {
      ++duplicate_marks;
      if (strict && bucket_of[idx] < next_launch)
        throw std::runtime_error("Reducer: gradient of parameter " + std::to_string(idx) +
                                 " marked ready again after its bucket's all-reduce was issued "
                                 "(write/collective race)");
      return;
    }
    param_ready[idx] = 1;
    at::Tensor& p = params[idx];
    const at::Tensor& v = views[idx];
    at::Tensor& g = p.mutable_grad();
    if (g.defined()) {
      if (g.data_ptr() != v.data_ptr() || g.strides() != v.strides()) {
        v.copy_(g);
        g = v;
      }
    } else if (zero_if_missing) {
      v.zero_();
      g = v;
    }
    int64_t b = bucket_of[idx];
    if (--pending[b] == 0) {
      bucket_ready[b] = 1;
      launch_ready_in_order();
    }
  }

  // a parameter's gradient is final in its flat view (from its AccumulateGrad hook, or written
  // in place by a fused native backward that then calls mark_ready_external)
  void on_ready(int64_t idx) {
    std::lock_guard<std::mutex> lk(mu);
    if (!enabled || !expecting) return;
    if (!callback_queued) {
      callback_queued = true;
      std::weak_ptr<ReducerState> w2 = self;
      torch::autograd::Engine::get_default_engine().queue_callback([w2]() {
        if (auto s2 = w2.lock()) s2->finalize();
      });
    }
    mark_param(idx, /*zero_if_missing=*/false);
  }

  std::weak_ptr<ReducerState> self;

  void finalize() {
    std::lock_guard<std::mutex> lk(mu);
    // parameters that received no gradient this iteration (unused in forward): zero views
    for (size_t i = 0; i < params.size(); ++i)
      if (!param_ready[i]) mark_param((int64_t)i, /*zero_if_missing=*/true);
    if (local) {
      if (!(sgd_armed && sgd_applied > 0)) {
        timed = false;
      } else {
      const int dev = params[0].get_device();
      c10::hip::HIPGuard guard((c10::DeviceIndex)dev);
      hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
      if (timing && !tail_on_cur) hipEventRecord(ev_bwd, cur);
      stream_handoff(local_stream, cur, ev_join);
      if (timing) {  // every bucket's update done (the caller's stream joined the overlap stream)
        hipEventRecord(ev_end, cur);
        timed = !launch_order.empty();
      }
      }
      tail_on_cur = false;
    } else if (xgmi) {
      if (timing) {
        c10::hip::HIPGuard guard((c10::DeviceIndex)xgmi->device());
        hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)xgmi->device()).stream();
        hipEventRecord(ev_bwd, cur);
        hipEventRecord(ev_end, xgmi->stream());
        timed = !launch_order.empty();
      }
      xgmi->current_wait_comm();
    } else if (comm) {
      if (timing) {
        c10::hip::HIPGuard guard((c10::DeviceIndex)comm->device());
        hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)comm->device()).stream();
        hipEventRecord(ev_bwd, cur);
        hipEventRecord(ev_end, comm->stream());
        timed = !launch_order.empty();
      }
      comm->current_wait_comm();
    } else {
      py::gil_scoped_acquire gil;
      py_finalize();
    }
    last_order = launch_order;
    if (sgd_armed) {
      sgd_last = {sgd_applied, grad_flat.defined() ? (int64_t)grad_flat._version() : -1};
      sgd_armed = false;
    }
    expecting = false;
    callback_queued = false;
    ++iters;
  }
};

Reducer::Reducer(std::vector<at::Tensor> params, std::vector<at::Tensor> grad_views,
                 std::vector<int64_t> bucket_of_param, std::vector<at::Tensor> bucket_flats,
                 std::shared_ptr<RcclComm> comm, py::object py_launch, py::object py_finalize,
                 bool average, std::string wire_dtype, std::shared_ptr<XgmiComm> xgmi)
    : st_(std::make_shared<ReducerState>()) {
  if (params.size() != grad_views.size() || params.size() != bucket_of_param.size())
    throw std::runtime_error("Reducer: params/views/bucket_of size mismatch");
  st_->params = std::move(params);
  st_->views = std::move(grad_views);
  st_->bucket_of = std::move(bucket_of_param);
  st_->flats = std::move(bucket_flats);
  st_->comm = std::move(comm);
  st_->xgmi = std::move(xgmi);
  if (st_->xgmi) {
    if (st_->comm) throw std::runtime_error("Reducer: give either the RCCL or the xGMI communicator");
    if (wire_dtype != "fp32") throw std::runtime_error("Reducer: the xGMI backend reduces fp32 gradients");
    // every bucket must be a slice of the communicator's shared gradient buffer
    const float* base = st_->xgmi->grad_buffer().data_ptr<float>();
    for (const auto& f : st_->flats) {
      const int64_t off = f.data_ptr<float>() - base;
      if (!f.is_contiguous() || off < 0 || off + f.numel() > st_->xgmi->numel())
        throw std::runtime_error("Reducer: bucket is not a slice of the xGMI gradient buffer");
      st_->flat_off.push_back(off);
    }
  }
  st_->local = !st_->comm && !st_->xgmi && py_launch.is_none();
  if (st_->local) {
    if (st_->params.empty() || !st_->params[0].is_cuda())
      throw std::runtime_error("Reducer: local mode (no communicator, no Python launch) needs device parameters");
    c10::hip::HIPGuard guard((c10::DeviceIndex)st_->params[0].get_device());
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (hipStreamCreateWithPriority(&st_->local_stream, hipStreamNonBlocking, lo) != hipSuccess ||
        hipEventCreateWithFlags(&st_->ev_local, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&st_->ev_join, hipEventDisableTiming) != hipSuccess)
      throw std::runtime_error("Reducer: local stream / events");
  }
  st_->py_launch = std::move(py_launch);
  st_->py_finalize = std::move(py_finalize);
  st_->average = average;
  st_->wire_bf16 = (wire_dtype == "bf16");
  if (st_->wire_bf16 && !st_->comm) throw std::runtime_error("bf16 wire format needs the RCCL comm");
  st_->wire.resize(st_->flats.size());
  st_->members.resize(st_->flats.size());
  for (size_t i = 0; i < st_->params.size(); ++i) {
    int64_t b = st_->bucket_of[i];
    if (b < 0 || b >= (int64_t)st_->flats.size()) throw std::runtime_error("Reducer: bad bucket id");
    st_->members[b].push_back((int64_t)i);
  }
  st_->reset_counters();
  if (const char* e = std::getenv("PDT_DEBUG_REDUCER")) st_->strict = e[0] == '1';
  if (const char* e = std::getenv("PDT_REDUCER_SKIP_COLL")) st_->skip_collectives = e[0] == '1';
  // A/B (PDT_TAIL_LOCAL=1): the last bucket's update on the overlap stream like every other bucket
  if (const char* e = std::getenv("PDT_TAIL_LOCAL")) st_->tail_local = e[0] == '1';

  std::weak_ptr<ReducerState> weak = st_;
  st_->self = weak;
  for (size_t i = 0; i < st_->params.size(); ++i) {
    auto acc = torch::autograd::impl::grad_accumulator(st_->params[i]);
    if (!acc) throw std::runtime_error("Reducer: parameter has no grad accumulator (requires_grad?)");
    int64_t idx = (int64_t)i;
    acc->add_post_hook(std::make_unique<torch::autograd::utils::LambdaPostHook>(
        [weak, idx](const torch::autograd::variable_list& outputs,
                    const torch::autograd::variable_list& inputs) {
          // The engine runs AccumulateGrad -- and its post hooks -- even when the gradient that
          // reaches it is undefined.  That is the case for every parameter a fused native
          // backward accumulated in place into its flat view (it returns None to autograd and
          // calls mark_ready_external itself, BEFORE this node runs) and for parameters unused
          // this iteration (finalize handles them).  Neither is a readiness event.
          if (!inputs.empty() && !inputs[0].defined()) return outputs;
          if (auto s = weak.lock()) s->on_ready(idx);
          return outputs;
        }));
    st_->accumulators.push_back(std::move(acc));
  }
}

Reducer::~Reducer() {
  for (hipEvent_t e : {st_->ev_start, st_->ev_end, st_->ev_bwd, st_->ev_aux, st_->ev_local, st_->ev_join})
    if (e) hipEventDestroy(e);
  if (st_->local_stream) {
    hipStreamSynchronize(st_->local_stream);
    hipStreamDestroy(st_->local_stream);
  }
}

void Reducer::set_timing(bool on) {
  std::lock_guard<std::mutex> lk(st_->mu);
  if (on && !st_->comm && !st_->xgmi && !st_->local)
    throw std::runtime_error("Reducer timing needs a native communicator (or local mode)");
  if (on && !st_->ev_start) {
    c10::hip::HIPGuard guard((c10::DeviceIndex)(st_->comm ? st_->comm->device()
                                                : st_->xgmi ? st_->xgmi->device() : st_->params[0].get_device()));
    for (hipEvent_t* e : {&st_->ev_start, &st_->ev_end, &st_->ev_bwd})
      if (hipEventCreate(e) != hipSuccess) throw std::runtime_error("hipEventCreate failed");
  }
  st_->timing = on;
  st_->timed = false;
}

std::pair<double, double> Reducer::comm_timing() {
  std::lock_guard<std::mutex> lk(st_->mu);
  if (!st_->timing || !st_->timed) return {-1.0, -1.0};
  hipEventSynchronize(st_->ev_end);
  hipEventSynchronize(st_->ev_bwd);
  float total = 0.f, tail = 0.f;
  hipEventElapsedTime(&total, st_->ev_start, st_->ev_end);
  hipEventElapsedTime(&tail, st_->ev_bwd, st_->ev_end);
  return {(double)total, tail > 0.f ? (double)tail : 0.0};
}

void Reducer::set_strict(bool on) { st_->strict = on; }

void Reducer::set_aux_stream(uintptr_t stream) {
  std::lock_guard<std::mutex> lk(st_->mu);
  if (st_->params.empty() || !st_->params[0].is_cuda())
    throw std::runtime_error("Reducer aux stream needs device parameters");
  if (!st_->ev_aux) {
    c10::hip::HIPGuard guard((c10::DeviceIndex)st_->params[0].get_device());
    if (hipEventCreateWithFlags(&st_->ev_aux, hipEventDisableTiming) != hipSuccess)
      throw std::runtime_error("hipEventCreate failed");
  }
  st_->aux = reinterpret_cast<hipStream_t>(stream);
}
int64_t Reducer::duplicate_marks() const { return st_->duplicate_marks; }

void Reducer::set_optimizer(const at::Tensor& param_flat, const at::Tensor& grad_flat) {
  std::lock_guard<std::mutex> lk(st_->mu);
  if (!st_->comm && !st_->xgmi && !st_->local)
    throw std::runtime_error("Reducer: the optimizer overlap needs a native communicator or local mode");
  if (!param_flat.is_cuda() || param_flat.scalar_type() != at::kFloat || !param_flat.is_contiguous() ||
      !grad_flat.is_cuda() || grad_flat.scalar_type() != at::kFloat || !grad_flat.is_contiguous() ||
      param_flat.numel() != grad_flat.numel())
    throw std::runtime_error("Reducer::set_optimizer: contiguous fp32 device flat buffers of one size");
  const float* base = grad_flat.data_ptr<float>();
  std::vector<int64_t> off;
  for (const auto& f : st_->flats) {
    const int64_t o = f.data_ptr<float>() - base;
    if (o < 0 || o + f.numel() > grad_flat.numel())
      throw std::runtime_error("Reducer::set_optimizer: a bucket is not a slice of grad_flat");
    off.push_back(o);
  }
  st_->goff = std::move(off);
  st_->grad_base = base;
  st_->grad_flat = grad_flat;
  st_->sgd_p = param_flat.data_ptr<float>();
}

void Reducer::arm_optimizer(double lr, double momentum, double dampening, double weight_decay, bool nesterov,
                            bool first, const at::Tensor& momentum_buf, const at::Tensor& mirror_bf16) {
  std::lock_guard<std::mutex> lk(st_->mu);
  if (!st_->sgd_p) throw std::runtime_error("Reducer::arm_optimizer before set_optimizer");
  const int64_t n = st_->grad_flat.numel();
  if (momentum != 0.0 && !(momentum_buf.defined() && momentum_buf.numel() == n &&
                           momentum_buf.scalar_type() == at::kFloat && momentum_buf.is_contiguous()))
    throw std::runtime_error("Reducer::arm_optimizer: momentum needs a contiguous fp32 flat buffer");
  if (mirror_bf16.defined() && (mirror_bf16.numel() != n || mirror_bf16.scalar_type() != at::kBFloat16 ||
                                !mirror_bf16.is_contiguous()))
    throw std::runtime_error("Reducer::arm_optimizer: the weight mirror must be a contiguous bf16 flat buffer");
  st_->sgd_lr = (float)lr;
  st_->sgd_mom = (float)momentum;
  st_->sgd_damp = (float)dampening;
  st_->sgd_wd = (float)weight_decay;
  st_->sgd_nest = nesterov;
  st_->sgd_first = first;
  st_->sgd_buf = momentum != 0.0 ? momentum_buf.data_ptr<float>() : nullptr;
  st_->sgd_pb = mirror_bf16.defined() ? reinterpret_cast<uint16_t*>(mirror_bf16.data_ptr()) : nullptr;
  st_->sgd_applied = 0;
  st_->sgd_armed = true;
  st_->sgd_last = {-1, -1};
}

std::pair<int64_t, int64_t> Reducer::optimizer_applied() const { return st_->sgd_last; }
void Reducer::consume_optimizer() { st_->sgd_last = {-1, -1}; }
bool Reducer::local() const { return st_->local; }

void Reducer::prepare_for_backward() {
  std::lock_guard<std::mutex> lk(st_->mu);
  st_->reset_counters();
  st_->expecting = st_->enabled;
  st_->callback_queued = false;
}

void Reducer::mark_ready_external(const std::vector<int64_t>& idx) {
  for (int64_t i : idx) {
    if (i < 0 || i >= (int64_t)st_->params.size()) throw std::runtime_error("mark_ready_external: bad index");
    st_->on_ready(i);
  }
}

void Reducer::set_enabled(bool enabled) {
  std::lock_guard<std::mutex> lk(st_->mu);
  st_->enabled = enabled;
}

bool Reducer::enabled() const { return st_->enabled; }
int64_t Reducer::num_buckets() const { return (int64_t)st_->flats.size(); }
std::vector<int64_t> Reducer::last_launch_order() const { return st_->last_order; }
int64_t Reducer::iterations() const { return st_->iters; }

}  // namespace pdt
