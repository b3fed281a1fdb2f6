#include "rccl_comm.h"

#include "stream_sync.h"

#include <c10/hip/HIPGuard.h>

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>

namespace pdt {

// Exit status of a process ended by the communicator monitor: the watchdog's (utils/watchdog.py
// EXIT_CODE), so the launcher reports both the same way.
constexpr int kCommExitCode = 124;

void rccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(r));
  }
}

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static double since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

// The comm stream is an ordinary-priority stream.  A high-priority stream was measured to cost
// +16.5 ms per ResNet-50 step on MI355X (21.6 -> 38.1 ms, world-1 forced reducer) even with the
// collectives skipped (PDT_REDUCER_SKIP_COLL=1: 38.0 ms): its event waits, not RCCL, stall the
// compute queues.  Measured: profiles/r2_comm_stream_priority_ab.md.
static bool comm_high_priority() { return false; }

// Communicator mode.  Default: a BLOCKING communicator whose init runs on a helper thread that
// the constructor waits for with a deadline.  A non-blocking communicator (PDT_RCCL_NONBLOCKING=1)
// makes every collective return ncclInProgress and the issuing thread -- the autograd thread, which
// also issues the rest of the backward -- poll ncclCommGetAsyncError until RCCL's async enqueue
// finishes.  A/B on MI355X with the world-1 forced reducer showed no step-time difference
// (r3w: 28.47 vs 28.52 ms, both then dominated by the stream-priority effect described in
// ops/streams.py), so the default is the one whose collectives need no host polling.
static bool rccl_nonblocking() {
  const char* e = std::getenv("PDT_RCCL_NONBLOCKING");
  return e && e[0] == '1';
}

namespace {
// Shared between the constructor and the init thread: the thread outlives a timed-out constructor
// (it stays blocked inside ncclCommInitRankConfig until its peers arrive or the process exits).
struct InitJob {
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  ncclResult_t r = ncclInProgress;
  ncclComm_t comm = nullptr;
};
}  // namespace

RcclComm::RcclComm(const std::string& uid, int rank, int world, int device, const RcclOptions& opt)
    : rank_(rank), world_(world), device_(device), opt_(opt),
      stream_(c10::hip::getStreamFromPool(comm_high_priority(), (c10::DeviceIndex)device)) {
  if (uid.size() != sizeof(ncclUniqueId::internal)) throw std::runtime_error("bad RCCL unique id size");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  ncclUniqueId id;
  memcpy(id.internal, uid.data(), sizeof(id.internal));
  // Init is bounded by a deadline (ProcessGroupNCCL's init timeout): an unbounded
  // ncclCommInitRank whose peer never arrives would hang this rank forever.
  nonblocking_ = rccl_nonblocking();
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = nonblocking_ ? 0 : 1;
  if (opt_.min_channels > 0) cfg.minCTAs = opt_.min_channels;
  if (opt_.max_channels > 0) cfg.maxCTAs = opt_.max_channels;
  const auto t0 = std::chrono::steady_clock::now();
  ncclResult_t st = ncclInProgress;
  if (nonblocking_) {
    ncclResult_t r = ncclCommInitRankConfig(&comm_, world, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (comm_) ncclCommAbort(comm_);
      comm_ = nullptr;
      rccl_check(r, "ncclCommInitRankConfig");
    }
    while (true) {
      if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) st = ncclInternalError;
      if (st != ncclInProgress) break;
      if (since(t0) > opt_.init_timeout_s) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  } else {
    auto job = std::make_shared<InitJob>();
    std::thread([job, id, world, rank, device, cfg]() mutable {
      ncclComm_t c = nullptr;
      ncclResult_t r = ncclInvalidUsage;
      if (hipSetDevice(device) == hipSuccess) r = ncclCommInitRankConfig(&c, world, id, rank, &cfg);
      std::lock_guard<std::mutex> lk(job->m);
      job->comm = c;
      job->r = r;
      job->done = true;
      job->cv.notify_all();
    }).detach();
    std::unique_lock<std::mutex> lk(job->m);
    const auto limit = std::chrono::duration<double>(opt_.init_timeout_s);
    if (job->cv.wait_for(lk, limit, [&] { return job->done; })) {
      st = job->r;
      comm_ = job->comm;
    }  // else: still in progress; the detached thread keeps the half-built communicator
  }
  init_s_ = since(t0);
  if (st != ncclSuccess) {
    if (comm_) ncclCommAbort(comm_);
    comm_ = nullptr;
    char buf[512];
    if (st == ncclInProgress)
      snprintf(buf, sizeof(buf),
               "RCCL communicator init timed out after %.1f s on rank %d of %d (device %d): a peer "
               "rank never joined (crashed, hung, or took another code path before its init)",
               init_s_, rank, world, device);
    else
      snprintf(buf, sizeof(buf), "RCCL communicator init failed on rank %d of %d (device %d): %s",
               rank, world, device, ncclGetErrorString(st));
    throw std::runtime_error(buf);
  }
  gate_ = std::make_unique<AbortGate>([this]() { ncclCommAbort(comm_); });
  hip_check(hipEventCreateWithFlags(&ev_a_, hipEventDisableTiming), "hipEventCreate");
  hip_check(hipEventCreateWithFlags(&ev_b_, hipEventDisableTiming), "hipEventCreate");
  barrier_buf_ = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device));
  monitor_ = std::thread([this]() { monitor_loop(); });
}

RcclComm::~RcclComm() {
  stop_.store(true);
  if (monitor_.joinable()) monitor_.join();
  // teardown through the gate: waits for a call still inside the communicator, and does nothing
  // if an abort already released it
  if (gate_) {
    gate_->finalize([&]() {
      if (!nonblocking_) {
        // blocking communicator: destroy only once the comm stream has drained (bounded wait); a
        // collective stuck on a dead peer is aborted instead of blocking our exit
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t q;
        while ((q = hipStreamQuery(stream())) == hipErrorNotReady && since(t0) < 10.0)
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
        if (q == hipSuccess) ncclCommDestroy(comm_);
        else ncclCommAbort(comm_);
      } else {
        // non-blocking communicator: finalize (flushes outstanding work) must complete before
        // destroy; a peer that died mid-teardown must not hang our exit, so the wait is bounded
        ncclResult_t r = ncclCommFinalize(comm_);
        ncclResult_t st = r;
        const auto t0 = std::chrono::steady_clock::now();
        while (r == ncclSuccess || r == ncclInProgress) {
          if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess || st != ncclInProgress) break;
          if (since(t0) > 10.0) break;
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        if (st == ncclSuccess) ncclCommDestroy(comm_);
        else ncclCommAbort(comm_);
      }
    });
  }
  comm_ = nullptr;
  if (ev_a_) hipEventDestroy(ev_a_);
  if (ev_b_) hipEventDestroy(ev_b_);
  for (auto& p : pending_) hipEventDestroy(p.ev);
  for (hipEvent_t e : free_events_) hipEventDestroy(e);
}

// Both failure paths only REQUEST the abort: the gate runs ncclCommAbort at once when no thread
// is inside an RCCL call on this communicator, else right after that call returns (the issuing
// thread runs it on its way out; the monitor retries every poll).  failed_ is set first, so a
// caller that has not yet entered the gate is refused by check() with the recorded error.
void RcclComm::abort() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (error_.empty()) error_ = "RCCL communicator was aborted";
    failed_.store(true);
  }
  if (gate_) gate_->request_abort();
}

void RcclComm::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (failed_.load()) return;
    error_ = msg;
    failed_.store(true);
  }
  fprintf(stderr, "[rccl] rank %d: %s; aborting the communicator%s\n", rank_, msg.c_str(),
          opt_.exit_on_error ? " and exiting" : "");
  fflush(stderr);
  if (gate_) gate_->request_abort();
  if (opt_.exit_on_error) std::_Exit(kCommExitCode);
}

void RcclComm::check() const {
  if (failed_.load()) {
    std::lock_guard<std::mutex> lk(mu_);
    throw std::runtime_error("RCCL communicator (rank " + std::to_string(rank_) + ") is unusable: " + error_);
  }
}

std::string RcclComm::error() const {
  std::lock_guard<std::mutex> lk(mu_);
  return error_;
}

void RcclComm::monitor_loop() {
  const auto period = std::chrono::microseconds((int64_t)(opt_.poll_s * 1e6));
  while (!stop_.load()) {
    std::this_thread::sleep_for(period);
    if (failed_.load()) {
      gate_->drain();  // an abort still pending behind a call that was in flight
      continue;
    }
    // skipped while another thread is inside an RCCL call (never blocks behind a slow enqueue)
    ncclResult_t st = ncclSuccess, qr = ncclInternalError;
    gate_->try_call([&]() { qr = ncclCommGetAsyncError(comm_, &st); });
    if (qr == ncclSuccess && st != ncclSuccess && st != ncclInProgress) {
      fail(std::string("asynchronous RCCL error: ") + ncclGetErrorString(st));
      continue;
    }
    std::string timeout_msg;
    {
      std::lock_guard<std::mutex> lk(mu_);
      while (!pending_.empty()) {
        Pending& p = pending_.front();
        const hipError_t q = hipEventQuery(p.ev);
        if (q == hipSuccess) {
          free_events_.push_back(p.ev);
          pending_.pop_front();
          continue;
        }
        if (q != hipErrorNotReady) {
          timeout_msg = std::string("completion query of '") + p.what + "' failed: " + hipGetErrorString(q);
        } else if (opt_.op_timeout_s > 0 && since(p.t) > opt_.op_timeout_s) {
          char buf[256];
          snprintf(buf, sizeof(buf), "collective '%s' did not complete within %.1f s (timeout %.1f s): a "
                   "peer rank is hung, dead or issued a different collective", p.what, since(p.t),
                   opt_.op_timeout_s);
          timeout_msg = buf;
        }
        break;
      }
    }
    if (!timeout_msg.empty()) fail(timeout_msg);
  }
}

// A/B knob (PDT_RCCL_TRACK=0): no per-collective completion event, so the monitor sees only
// asynchronous RCCL errors (no collective timeout)
static bool rccl_track() {
  static const bool on = [] {
    const char* e = std::getenv("PDT_RCCL_TRACK");
    return !(e && e[0] == '0');
  }();
  return on;
}

void RcclComm::track(const char* what) {
  if (!rccl_track()) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream(), &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
    return;  // captured collectives run at replay; the process watchdog covers graph mode
  std::lock_guard<std::mutex> lk(mu_);
  hipEvent_t ev;
  if (!free_events_.empty()) {
    ev = free_events_.back();
    free_events_.pop_back();
  } else {
    hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  }
  hip_check(hipEventRecord(ev, stream()), "hipEventRecord");
  pending_.push_back({ev, std::chrono::steady_clock::now(), what});
}

// Non-blocking communicator: the enqueue returned ncclInProgress.  Poll its completion with ONE
// ncclCommGetAsyncError per gate call, so the gate is free between polls: an abort requested by
// the monitor, the watchdog or the user runs between two polls (RCCL allows ncclCommAbort to
// cancel an in-progress non-blocking operation) instead of waiting out the whole poll.
// Returns ncclInProgress on timeout and ncclInvalidUsage when the communicator was aborted.
ncclResult_t RcclComm::wait_async(const char* what) {
  (void)what;
  const auto t0 = std::chrono::steady_clock::now();
  ncclResult_t st = ncclInProgress;
  while (st == ncclInProgress) {
    const bool ran = gate_->call([&]() {
      if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) st = ncclInternalError;
    });
    if (!ran) return ncclInvalidUsage;  // aborted between polls
    if (st == ncclInProgress && since(t0) > opt_.init_timeout_s) break;
    if (st == ncclInProgress) std::this_thread::yield();
  }
  return st;
}

template <class F>
void RcclComm::issue(const char* what, F&& enqueue) {
  check();
  ncclResult_t r = ncclSuccess;
  const bool ran = gate_->call([&]() { r = enqueue(); });
  const bool aborted_in_poll = ran && r == ncclInProgress && (r = wait_async(what)) == ncclInvalidUsage &&
                               !gate_->usable();
  if (!ran || aborted_in_poll) {  // aborted before or while the call completed: the recorded error
    check();
    throw std::runtime_error(std::string("RCCL communicator (rank ") + std::to_string(rank_) +
                             ") was aborted " + (ran ? "while completing " : "before ") + what);
  }
  if (r == ncclInProgress) {
    fail(std::string(what) + " still in progress after the init timeout");
    check();
  }
  if (r != ncclSuccess) {
    fail(std::string(what) + " failed: " + ncclGetErrorString(r));
    check();
  }
  track(what);
}

int RcclComm::comm_count() {
  int n = -1;
  if (!gate_->call([&]() { rccl_check(ncclCommCount(comm_, &n), "ncclCommCount"); })) return -1;
  return n;
}

int RcclComm::version() {
  int v = 0;
  rccl_check(ncclGetVersion(&v), "ncclGetVersion");
  return v;
}

void RcclComm::inject_delay(double seconds) {
  check();
  // host callback on the comm stream that sleeps: the stream (and anything tracked behind it)
  // stalls for `seconds` exactly like a collective waiting on a slow peer, with no GPU kernel
  // spinning and no RCCL kernel queued behind it
  auto* secs = new double(seconds);
  hip_check(hipLaunchHostFunc(
                stream(),
                [](void* p) {
                  double* s = static_cast<double*>(p);
                  std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(*s * 1e6)));
                  delete s;
                },
                secs),
            "hipLaunchHostFunc");
  track("inject_delay");
}

ncclDataType_t RcclComm::dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: throw std::runtime_error("RcclComm: unsupported dtype");
  }
}

ncclRedOp_t RcclComm::op_of(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  throw std::runtime_error("RcclComm: unknown reduce op " + op);
}

void RcclComm::comm_wait_current() {
  hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream();
  stream_handoff(cur, stream(), ev_a_);
}

void RcclComm::current_wait_comm() {
  hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream();
  stream_handoff(stream(), cur, ev_b_);
}

void RcclComm::synchronize() {
  check();
  hip_check(hipStreamSynchronize(stream()), "hipStreamSynchronize");
  check();  // an abort while we waited: the stream drained because the collectives were killed
}

static void check_dev(const at::Tensor& t, int device) {
  if (!t.is_cuda() || t.get_device() != device || !t.is_contiguous())
    throw std::runtime_error("RcclComm: tensor must be a contiguous tensor on the comm device");
}

void RcclComm::all_reduce_raw(void* ptr, size_t count, ncclDataType_t dt, ncclRedOp_t op) {
  issue("ncclAllReduce", [&]() { return ncclAllReduce(ptr, ptr, count, dt, op, comm_, stream()); });
}

void RcclComm::all_reduce(const at::Tensor& t, const std::string& op, bool wait_current) {
  check_dev(t, device_);
  if (wait_current) comm_wait_current();
  all_reduce_raw(t.data_ptr(), (size_t)t.numel(), dtype_of(t), op_of(op));
}

void RcclComm::broadcast(const at::Tensor& t, int root, bool wait_current) {
  check_dev(t, device_);
  check();
  if (wait_current) comm_wait_current();
  issue("ncclBroadcast", [&]() {
    return ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), root, comm_, stream());
  });
}

void RcclComm::reduce_scatter(const at::Tensor& in, const at::Tensor& out, const std::string& op,
                              bool wait_current) {
  check_dev(in, device_);
  check_dev(out, device_);
  check();
  if (in.numel() != out.numel() * world_) throw std::runtime_error("reduce_scatter: size mismatch");
  if (wait_current) comm_wait_current();
  const ncclRedOp_t rop = op_of(op);
  issue("ncclReduceScatter", [&]() {
    return ncclReduceScatter(in.data_ptr(), out.data_ptr(), (size_t)out.numel(), dtype_of(in), rop, comm_, stream());
  });
}

void RcclComm::all_gather(const at::Tensor& in, const at::Tensor& out, bool wait_current) {
  check_dev(in, device_);
  check_dev(out, device_);
  check();
  if (out.numel() != in.numel() * world_) throw std::runtime_error("all_gather: size mismatch");
  if (wait_current) comm_wait_current();
  issue("ncclAllGather", [&]() {
    return ncclAllGather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), dtype_of(in), comm_, stream());
  });
}

void RcclComm::barrier() {
  all_reduce(barrier_buf_, "sum", true);
  synchronize();
}

}  // namespace pdt
