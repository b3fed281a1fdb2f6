// Native RCCL communicator (one per process / GPU) used by the gradient reducer.
//
// The reference gets its collectives from c10d's ProcessGroupNCCL
// (init_process_group("nccl"), resnet/main.py:74).  Here the data-parallel hot
// path talks to RCCL directly: the unique id is exchanged once through the
// rendezvous store, every collective runs on a dedicated (normal-priority) HIP
// stream, and compute<->comm ordering is expressed with HIP events so gradient
// all-reduces overlap the remaining backward kernels.  On an 8x MI355X node the
// transport is xGMI (7 point-to-point links per GPU); RCCL picks rings/trees
// over those links, our job is to hand it few, large, well-timed buckets.
#pragma once
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>

namespace pdt {

class RcclComm {
 public:
  static std::string unique_id();  // 128 raw bytes (NCCL_UNIQUE_ID_BYTES)
  RcclComm(const std::string& uid, int rank, int world, int device);
  ~RcclComm();

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  hipStream_t stream() const { return stream_.stream(); }
  c10::hip::HIPStream hip_stream() const { return stream_; }

  // Collectives enqueue on the comm stream after it waits for the caller's current stream
  // (when `wait_current` is set).  Tensors must be contiguous device tensors.
  void all_reduce(const at::Tensor& t, const std::string& op, bool wait_current = true);
  void broadcast(const at::Tensor& t, int root, bool wait_current = true);
  void reduce_scatter(const at::Tensor& in, const at::Tensor& out, const std::string& op,
                      bool wait_current = true);
  void all_gather(const at::Tensor& in, const at::Tensor& out, bool wait_current = true);
  // raw-pointer form used by the reducer (already ordered by the caller)
  void all_reduce_raw(void* ptr, size_t count, ncclDataType_t dt, ncclRedOp_t op);

  // ordering helpers
  void comm_wait_current();  // comm stream waits for the current compute stream
  void current_wait_comm();  // current compute stream waits for the comm stream
  void synchronize();        // host waits for the comm stream
  void barrier();
  void abort();

  static ncclDataType_t dtype_of(const at::Tensor& t);
  static ncclRedOp_t op_of(const std::string& op);

 private:
  ncclComm_t comm_ = nullptr;
  int rank_, world_, device_;
  c10::hip::HIPStream stream_;
  hipEvent_t ev_a_ = nullptr, ev_b_ = nullptr;
  at::Tensor barrier_buf_;
};

void rccl_check(ncclResult_t r, const char* what);

}  // namespace pdt
