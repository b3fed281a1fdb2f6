// Native gradient reducer for data-parallel training.
//
// Plays the role of c10d's C++ Reducer that DistributedDataParallel creates at
// torch/nn/parallel/distributed.py:1227 (reference resnet/main.py:80), designed
// for the MI355X path:
//   * every parameter's .grad is a view into ONE flat fp32 gradient buffer,
//     partitioned into buckets in reverse-definition (= grad-ready) order, so a
//     bucket all-reduce is a single contiguous RCCL call and the optimizer can
//     run one fused kernel over the whole flat buffer;
//   * an autograd post-hook on each parameter's AccumulateGrad node marks it
//     ready (copying the grad into its view only when autograd did not already
//     accumulate in place); a full bucket is launched immediately -- in bucket
//     order, as collectives must be issued identically on every rank -- on the
//     RCCL comm stream behind an event, so the all-reduce overlaps the rest of
//     backward;
//   * averaging is folded into the collective (ncclAvg), optionally with bf16
//     wire format (halves xGMI bytes) cast back into the fp32 buffer;
//   * a final autograd callback makes the caller's stream wait for the comm
//     stream, zero-fills buckets of parameters that got no gradient, and resets.
// Non-RCCL process groups (gloo on CPU, used by the tests) plug in via Python
// launch/finalize callbacks while keeping all the bookkeeping here.
//
// Optimizer in backward: with set_optimizer + arm_optimizer, the fused SGD
// runs over each bucket's flat range right behind that bucket's all-reduce, on the same stream, so
// only the last bucket's update is left after backward (torch.optim.SGD math, sgd.hip).  In a
// single process without a communicator the reducer runs in LOCAL mode (py_launch = None): no
// collective, a private low-priority stream that waits for the compute and weight-gradient streams
// and runs each bucket's update as soon as its gradients are final.
#pragma once
#include <ATen/ATen.h>
#include <pybind11/pybind11.h>

#include <memory>
#include <mutex>
#include <string>
#include <cstdint>
#include <utility>
#include <vector>

#include "../comm/rccl_comm.h"
#include "../comm/xgmi_comm.h"

namespace pdt {

struct ReducerState;

class Reducer {
 public:
  Reducer(std::vector<at::Tensor> params, std::vector<at::Tensor> grad_views,
          std::vector<int64_t> bucket_of_param, std::vector<at::Tensor> bucket_flats,
          std::shared_ptr<RcclComm> comm, pybind11::object py_launch,
          pybind11::object py_finalize, bool average, std::string wire_dtype,
          std::shared_ptr<XgmiComm> xgmi = nullptr);
  ~Reducer();

  void prepare_for_backward();
  // gradients already accumulated into their flat views by a fused native backward
  void mark_ready_external(const std::vector<int64_t>& idx);
  void set_enabled(bool enabled);
  bool enabled() const;
  int64_t num_buckets() const;
  std::vector<int64_t> last_launch_order() const;
  int64_t iterations() const;
  // RCCL path: record events around each iteration's all-reduces; comm_timing() returns
  // (ms from first bucket start to last bucket end, ms the all-reduce tail outlasted backward)
  // of the last finished iteration, or (-1, -1).
  void set_timing(bool on);
  std::pair<double, double> comm_timing();
  // error (instead of ignoring) when a gradient is marked ready after its bucket was launched
  void set_strict(bool on);
  // bucket all-reduces additionally wait for this stream (gradients produced on a side stream)
  void set_aux_stream(uintptr_t stream);
  int64_t duplicate_marks() const;
  // per-bucket fused SGD: param_flat / grad_flat are the flat buffers the buckets are slices of
  void set_optimizer(const at::Tensor& param_flat, const at::Tensor& grad_flat);
  // arm the update for the next backward (hyperparameters of torch.optim.SGD; momentum_buf and
  // mirror_bf16 -- the flat bf16 weight mirror the SGD kernel also writes -- may be undefined)
  void arm_optimizer(double lr, double momentum, double dampening, double weight_decay, bool nesterov,
                     bool first, const at::Tensor& momentum_buf, const at::Tensor& mirror_bf16);
  // (buckets updated by the last finished backward, grad_flat's version counter at its end);
  // (-1, -1) when it applied none or the result was consumed
  std::pair<int64_t, int64_t> optimizer_applied() const;
  void consume_optimizer();
  bool local() const;

 private:
  std::shared_ptr<ReducerState> st_;
};

}  // namespace pdt
