// Native RCCL communicator (one per process / GPU) used by the gradient reducer.
//
// The reference gets its collectives from c10d's ProcessGroupNCCL
// (init_process_group("nccl"), resnet/main.py:74), and with it ProcessGroupNCCL's failure
// handling: a watchdog thread, async-error checks and a 10-minute collective timeout.  Here the
// data-parallel hot path talks to RCCL directly, so this class carries that failure handling too:
//
//  * init is bounded by a deadline: ncclCommInitRankConfig runs on a helper thread the
//    constructor waits for, so a peer that never joins makes init throw a clear error after
//    `init_timeout_s` instead of blocking forever.  The communicator itself is BLOCKING:
//    a non-blocking one (PDT_RCCL_NONBLOCKING=1, blocking = 0) makes every collective's issuing
//    thread poll for the async enqueue;
//  * a monitor thread polls ncclCommGetAsyncError and the completion event of every enqueued
//    collective; an async error or a collective older than `op_timeout_s` aborts the
//    communicator (ncclCommAbort unblocks kernels waiting on a dead peer), records the error --
//    every later call on this communicator (and the reducer's next bucket launch) throws it --
//    and, with `exit_on_error`, ends the process so the launcher's fail-fast tears the job down
//    (ProcessGroupNCCL's async error handling);
//  * every use of the communicator goes through an AbortGate (comm/abort_gate.h): an abort from
//    the monitor or the user never frees it while another thread is inside an RCCL call on it --
//    it runs as soon as that call returns -- and a call after the abort is refused with the
//    recorded error instead of reaching the freed communicator;
//  * per-communicator channel bounds (config.minCTAs / maxCTAs) are the RCCL knob for how many
//    rings/channels a collective spreads over the 7 point-to-point xGMI links of a GPU.
//
// The unique id is exchanged once through the rendezvous store, every collective runs on a
// dedicated (normal-priority) HIP stream, and compute<->comm ordering is expressed with HIP
// events so gradient all-reduces overlap the remaining backward kernels.
#pragma once
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "comm/abort_gate.h"

#include <atomic>
#include <chrono>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace pdt {

struct RcclOptions {
  double init_timeout_s = 600.0;  // non-blocking init deadline
  double op_timeout_s = 600.0;    // a collective not complete after this long -> abort (0 = off)
  bool exit_on_error = false;     // monitor ends the process after an abort (launcher fail-fast)
  int min_channels = 0;           // ncclConfig_t minCTAs / maxCTAs (0 = RCCL's choice)
  int max_channels = 0;
  double poll_s = 0.05;           // monitor period
};

class RcclComm {
 public:
  static std::string unique_id();  // 128 raw bytes (NCCL_UNIQUE_ID_BYTES)
  RcclComm(const std::string& uid, int rank, int world, int device, const RcclOptions& opt = {});
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

  // failure state: check() throws the recorded error (async RCCL error, collective timeout or
  // abort); healthy() / error() inspect it without throwing
  void check() const;
  bool healthy() const { return !failed_.load(); }
  std::string error() const;
  // test hook: make the next collective's completion wait `seconds` on a host callback
  // (a stalled peer without hanging the GPU)
  void inject_delay(double seconds);
  double init_seconds() const { return init_s_; }
  // diagnostics: the rank count RCCL itself reports (ncclCommCount; -1 when aborted) and the
  // RCCL library version (ncclGetVersion, e.g. 22606)
  int comm_count();
  static int version();
  const RcclOptions& options() const { return opt_; }

  static ncclDataType_t dtype_of(const at::Tensor& t);
  static ncclRedOp_t op_of(const std::string& op);

 private:
  // one gated RCCL call: `enqueue` runs under the abort gate (and, on a non-blocking
  // communicator, the poll for its async enqueue); an error fails the communicator and throws
  template <class F>
  void issue(const char* what, F&& enqueue);
  ncclResult_t wait_async(const char* what);      // ncclInProgress -> poll until done
  void track(const char* what);                   // completion event for the monitor
  void fail(const std::string& msg);
  void monitor_loop();

  ncclComm_t comm_ = nullptr;
  int rank_, world_, device_;
  RcclOptions opt_;
  c10::hip::HIPStream stream_;
  hipEvent_t ev_a_ = nullptr, ev_b_ = nullptr;
  at::Tensor barrier_buf_;
  double init_s_ = 0.0;
  bool nonblocking_ = false;  // PDT_RCCL_NONBLOCKING=1: ncclConfig_t.blocking = 0

  struct Pending {
    hipEvent_t ev;
    std::chrono::steady_clock::time_point t;
    const char* what;
  };
  mutable std::mutex mu_;
  std::deque<Pending> pending_;
  std::vector<hipEvent_t> free_events_;
  std::string error_;
  std::atomic<bool> failed_{false};
  std::unique_ptr<AbortGate> gate_;  // created once the communicator exists
  std::atomic<bool> stop_{false};
  std::thread monitor_;
  double delay_s_ = 0.0;
};

void rccl_check(ncclResult_t r, const char* what);

}  // namespace pdt
