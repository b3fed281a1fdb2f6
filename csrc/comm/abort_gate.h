// Abort-safe access to a communicator that one thread may abort while others use it.
//
// ncclCommAbort frees the communicator.  The RCCL wrapper has three kinds of callers: the
// thread that issues collectives (the autograd thread), the monitor thread that polls
// ncclCommGetAsyncError and aborts on an error or a collective timeout, and the user (abort()).
// Without a gate an abort could land between a caller's "is it still usable?" check and its
// RCCL call -- a use-after-free on the freed communicator.  The gate serialises them:
//
//   * call(f): f (one RCCL call) runs under the gate's lock unless the communicator is already
//     aborted, in which case f is skipped and call() returns false;
//   * try_call(f): the same, but skipped when another thread is inside a call (the monitor's
//     poll never blocks behind a collective that is slow to enqueue);
//   * request_abort(): the abort runs NOW if no other thread is inside a call, else as soon as
//     that call returns (the caller leaving call() runs it) -- never while another thread is
//     inside the communicator.  drain() retries a pending abort (the monitor calls it every poll).
//
// The lock is recursive so an abort requested from inside f (a failed collective's own error
// path) runs at once: that thread's RCCL call has already returned.  Host-only, no HIP/RCCL
// dependency: tests/test_comm_gate_cpu.py stress-tests it under AddressSanitizer.
#pragma once
#include <atomic>
#include <functional>
#include <mutex>
#include <utility>

namespace pdt {

class AbortGate {
 public:
  explicit AbortGate(std::function<void()> abort_fn) : abort_fn_(std::move(abort_fn)) {}
  AbortGate(const AbortGate&) = delete;
  AbortGate& operator=(const AbortGate&) = delete;

  template <class F>
  bool call(F&& f) {
    {
      std::lock_guard<std::recursive_mutex> lk(mu_);
      if (aborted_.load()) return false;
      f();
    }
    drain();
    return true;
  }

  template <class F>
  bool try_call(F&& f) {
    std::unique_lock<std::recursive_mutex> lk(mu_, std::try_to_lock);
    if (!lk.owns_lock() || aborted_.load()) return false;
    f();
    return true;
  }

  void request_abort() {
    pending_.store(true);
    drain();
  }

  // Runs a pending abort if no other thread is inside a call.  A thread holding the lock when
  // request_abort() ran reads `pending_` after it unlocks (call() -> drain()), so a requested
  // abort is never lost; a spurious try_lock failure is retried by the next drain().
  void drain() {
    if (!pending_.load() || aborted_.load()) return;
    std::unique_lock<std::recursive_mutex> lk(mu_, std::try_to_lock);
    if (!lk.owns_lock()) return;
    if (!aborted_.load()) {
      aborted_.store(true);
      abort_fn_();
    }
  }

  // false once the communicator has been aborted (or finalized)
  bool usable() const { return !aborted_.load(); }

  // Blocking form for teardown: waits for an in-flight call, then runs f (destroy/abort) once
  // unless the communicator was already aborted.
  template <class F>
  bool finalize(F&& f) {
    std::lock_guard<std::recursive_mutex> lk(mu_);
    if (aborted_.exchange(true)) return false;
    f();
    return true;
  }

  bool aborted() const { return aborted_.load(); }
  bool abort_pending() const { return pending_.load() && !aborted_.load(); }

 private:
  std::function<void()> abort_fn_;
  std::recursive_mutex mu_;
  std::atomic<bool> pending_{false};
  std::atomic<bool> aborted_{false};
};

}  // namespace pdt
