#include "stream_sync.h"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>

namespace pdt {

static void sync_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("stream_handoff: ") + what + ": " + hipGetErrorString(e));
}

bool stream_sync_value() {
  static const bool v = [] {
    const char* e = std::getenv("PDT_STREAM_SYNC");
    return e && std::strcmp(e, "value") == 0;
  }();
  return v;
}

namespace {
// one 64-bit signal slot per producer stream, in signal memory of the producer's device
struct Slots {
  std::mutex mu;
  // producer stream -> its 8-byte signal word (hipMallocSignalMemory allocates one word at a
  // time), allocated on the device current at its first hand-off
  std::unordered_map<hipStream_t, uint64_t*> slot_of;
  std::unordered_map<hipStream_t, uint64_t> ticket;    // last ticket written by that producer
};
Slots& slots() {
  static Slots s;
  return s;
}
}  // namespace

static bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

void stream_handoff(hipStream_t producer, hipStream_t consumer, hipEvent_t ev) {
  if (!stream_sync_value() || capturing(producer) || capturing(consumer)) {
    sync_check(hipEventRecord(ev, producer), "hipEventRecord");
    sync_check(hipStreamWaitEvent(consumer, ev, 0), "hipStreamWaitEvent");
    return;
  }
  Slots& S = slots();
  // the lock spans the two enqueues: tickets of one producer reach its stream in order
  std::lock_guard<std::mutex> lk(S.mu);
  uint64_t* ptr;
  uint64_t t;
  {
    auto it = S.slot_of.find(producer);
    if (it == S.slot_of.end()) {
      uint64_t* p = nullptr;
      sync_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&p), sizeof(uint64_t), hipMallocSignalMemory),
                 "hipExtMallocWithFlags(signal)");
      sync_check(hipMemset(p, 0, sizeof(uint64_t)), "hipMemset");
      sync_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      it = S.slot_of.emplace(producer, p).first;
    }
    ptr = it->second;
    t = ++S.ticket[producer];
  }
  sync_check(hipStreamWriteValue64(producer, ptr, t, 0), "hipStreamWriteValue64");
  sync_check(hipStreamWaitValue64(consumer, ptr, t, hipStreamWaitValueGte, ~0ull), "hipStreamWaitValue64");
}

}  // namespace pdt
