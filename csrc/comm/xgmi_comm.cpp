#include "xgmi_comm.h"

#include "stream_sync.h"

#include <c10/hip/HIPGuard.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "../kernels/kernels.h"

namespace pdt {

static void hipc(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("xgmi: ") + what + ": " + hipGetErrorString(e));
}

XgmiComm::XgmiComm(int rank, int world, int device, int64_t numel, int nbuckets, double timeout_s,
                   const std::string& wire, int max_blocks, bool exit_on_error)
    : rank_(rank), world_(world), device_(device), numel_(numel), nbuckets_(nbuckets),
      timeout_s_(timeout_s), max_blocks_(max_blocks), exit_on_error_(exit_on_error),
      stream_(c10::hip::getStreamFromPool(false, (c10::DeviceIndex)device)) {
  if (wire != "fp32" && wire != "bf16") throw std::runtime_error("xgmi: wire must be 'fp32' or 'bf16'");
  if (max_blocks < 1) throw std::runtime_error("xgmi: max_blocks must be >= 1");
  if (world < 1 || world > xgmi_max_ranks()) throw std::runtime_error("xgmi: world size must be 1..8");
  if (rank < 0 || rank >= world) throw std::runtime_error("xgmi: bad rank");
  if (numel <= 0 || nbuckets <= 0) throw std::runtime_error("xgmi: empty gradient space");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  hipc(hipMalloc(&g_, numel * sizeof(float)), "hipMalloc(grad)");
  hipc(hipMalloc(&red_, numel * sizeof(float)), "hipMalloc(reduced)");
  const size_t fbytes = (size_t)nbuckets * xgmi_slots_per_bucket() * 8 * sizeof(unsigned);
  // The per-bucket epoch flags are stored into by PEER GPUs and spin-polled here: keep them in
  // uncached (fine-grained) device memory, as RCCL does for its cross-GPU flags and FIFOs, so a
  // poll never hits a stale line of the local L2 whatever the coherence of peer stores through
  // xGMI.  Fall back to plain memory only if the runtime cannot export the allocation.
  flags_uncached_ = false;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), fbytes, hipDeviceMallocUncached) == hipSuccess) {
    hipIpcMemHandle_t probe;
    if (hipIpcGetMemHandle(&probe, flags_) == hipSuccess) {
      flags_uncached_ = true;
    } else {
      (void)hipGetLastError();
      hipFree(flags_);
      flags_ = nullptr;
    }
  } else {
    (void)hipGetLastError();
    flags_ = nullptr;
  }
  if (!flags_uncached_) {
    fprintf(stderr, "[xgmi] uncached flag memory not exportable here; using plain device memory\n");
    hipc(hipMalloc(&flags_, fbytes), "hipMalloc(flags)");
  }
  hipc(hipMemset(g_, 0, numel * sizeof(float)), "hipMemset");
  if (wire == "bf16") {
    hipc(hipMalloc(&g16_, numel * sizeof(uint16_t)), "hipMalloc(grad bf16)");
    hipc(hipMalloc(&red16_, numel * sizeof(uint16_t)), "hipMalloc(reduced bf16)");
  }
  hipc(hipMemset(flags_, 0, fbytes), "hipMemset");
  hipc(hipHostMalloc(&err_host_, sizeof(unsigned), hipHostMallocMapped), "hipHostMalloc");
  *err_host_ = 0u;
  hipc(hipHostGetDevicePointer((void**)&err_dev_, err_host_, 0), "hipHostGetDevicePointer");
  int khz = 0;
  hipc(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device), "wall clock rate");
  timeout_ticks_ = (uint64_t)(timeout_s * 1000.0 * (double)(khz > 0 ? khz : 100000));
  epoch_.assign(nbuckets, 0u);
  gp_[rank] = g_;
  rp_[rank] = red_;
  fp_[rank] = flags_;
  g16p_[rank] = g16_;
  r16p_[rank] = red16_;
  hipc(hipEventCreateWithFlags(&ev_a_, hipEventDisableTiming), "hipEventCreate");
  hipc(hipEventCreateWithFlags(&ev_b_, hipEventDisableTiming), "hipEventCreate");
  hipc(hipDeviceSynchronize(), "hipDeviceSynchronize");  // zeroed flags visible before any peer signals
  monitor_ = std::thread([this]() { monitor_loop(); });
}

// Host monitor (the xGMI analogue of the RCCL communicator's): the device error word is set by a
// bounded wait that timed out or saw a peer's POISON.  The failing rank's gradients are NaN-poisoned
// on the device (xgmi.hip), and with exit_on_error (default for world > 1) the process ends here
// with the watchdog's exit code, so the launcher's fail-fast tears the job down before an eval or
// checkpoint can run on this rank.
void XgmiComm::monitor_loop() {
  while (!stop_.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    if (error_code() == 0) continue;
    fprintf(stderr, "[xgmi] %s%s\n", error_message().c_str(), exit_on_error_ ? "; exiting" : "");
    fflush(stderr);
    if (exit_on_error_) std::_Exit(124);
    return;  // reported once; every later reduce_bucket / synchronize raises it
  }
}

XgmiComm::~XgmiComm() {
  stop_.store(true);
  if (monitor_.joinable()) monitor_.join();
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  hipStreamSynchronize(stream());
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  if (g_) hipFree(g_);
  if (red_) hipFree(red_);
  if (flags_) hipFree(flags_);
  if (g16_) hipFree(g16_);
  if (red16_) hipFree(red16_);
  if (err_host_) hipHostFree(err_host_);
  if (ev_a_) hipEventDestroy(ev_a_);
  if (ev_b_) hipEventDestroy(ev_b_);
}

std::string XgmiComm::ipc_handles() const {
  hipIpcMemHandle_t h[5];
  hipc(hipIpcGetMemHandle(&h[0], g_), "hipIpcGetMemHandle(grad)");
  hipc(hipIpcGetMemHandle(&h[1], red_), "hipIpcGetMemHandle(reduced)");
  hipc(hipIpcGetMemHandle(&h[2], flags_), "hipIpcGetMemHandle(flags)");
  const int n = g16_ ? 5 : 3;
  if (g16_) {
    hipc(hipIpcGetMemHandle(&h[3], g16_), "hipIpcGetMemHandle(grad bf16)");
    hipc(hipIpcGetMemHandle(&h[4], red16_), "hipIpcGetMemHandle(reduced bf16)");
  }
  return std::string(reinterpret_cast<const char*>(h), n * sizeof(hipIpcMemHandle_t));
}

void XgmiComm::open_peers(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::runtime_error("xgmi: need one handle set per rank");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  for (int q = 0; q < world_; ++q) {
    if (q == rank_) continue;
    const int n = g16_ ? 5 : 3;
    if (handles[q].size() != n * sizeof(hipIpcMemHandle_t))
      throw std::runtime_error("xgmi: bad handle size (peers must agree on the wire format)");
    hipIpcMemHandle_t h[5];
    memcpy(h, handles[q].data(), n * sizeof(hipIpcMemHandle_t));
    void* p[5];
    for (int i = 0; i < n; ++i) {
      hipc(hipIpcOpenMemHandle(&p[i], h[i], hipIpcMemLazyEnablePeerAccess),
           ("hipIpcOpenMemHandle(rank " + std::to_string(q) + ")").c_str());
      opened_.push_back(p[i]);
    }
    // plain (cached) flag memory is only safe while every peer shares this GPU's L2: across
    // devices a poll could spin on a stale line, so the fallback is refused there
    if (!flags_uncached_) {
      hipPointerAttribute_t attr{};
      const bool known = hipPointerGetAttributes(&attr, p[2]) == hipSuccess;
      (void)hipGetLastError();
      if (!known || attr.device != device_)
        throw std::runtime_error("xgmi: peer rank " + std::to_string(q) + " is on another device, but uncached "
                                 "flag memory could not be exported here; use comm='rccl'");
    }
    gp_[q] = static_cast<const float*>(p[0]);
    rp_[q] = static_cast<const float*>(p[1]);
    fp_[q] = static_cast<unsigned*>(p[2]);
    if (g16_) {
      g16p_[q] = static_cast<const uint16_t*>(p[3]);
      r16p_[q] = static_cast<const uint16_t*>(p[4]);
    }
  }
  linked_ = true;
}

void XgmiComm::link_local(const std::vector<std::shared_ptr<XgmiComm>>& all) {
  if ((int)all.size() != world_) throw std::runtime_error("xgmi: need one communicator per rank");
  for (int q = 0; q < world_; ++q) {
    if (all[q]->rank_ != q || all[q]->world_ != world_ || all[q]->numel_ != numel_ ||
        all[q]->wire_bf16() != wire_bf16())
      throw std::runtime_error("xgmi: link_local expects ranks 0..world-1 of one gradient space");
    gp_[q] = all[q]->g_;
    rp_[q] = all[q]->red_;
    fp_[q] = all[q]->flags_;
    g16p_[q] = all[q]->g16_;
    r16p_[q] = all[q]->red16_;
  }
  linked_ = true;
}

at::Tensor XgmiComm::grad_buffer() {
  auto self = shared_from_this();
  return at::from_blob(g_, {numel_}, [self](void*) {},
                       at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
}

void XgmiComm::reduce_bucket(int bucket, int64_t offset, int64_t count, bool average) {
  reduce_bucket_phases(bucket, offset, count, average, 0, 5);
}

void XgmiComm::reduce_bucket_phases(int bucket, int64_t offset, int64_t count, bool average, int lo, int hi) {
  check();
  if (!linked_ && world_ > 1) throw std::runtime_error("xgmi: peers not mapped (open_peers / link_local)");
  if (bucket < 0 || bucket >= nbuckets_) throw std::runtime_error("xgmi: bad bucket index");
  if (offset < 0 || count < 0 || offset + count > numel_) throw std::runtime_error("xgmi: bucket out of range");
  if (count == 0) return;
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  if (lo == 0) ++epoch_[bucket];
  XgmiBuffers B{};
  for (int q = 0; q < world_; ++q) {
    B.g[q] = gp_[q];
    B.red[q] = rp_[q];
    B.flags[q] = fp_[q];
    B.g16[q] = g16p_[q];
    B.red16[q] = r16p_[q];
  }
  launch_xgmi_bucket(B, world_, rank_, bucket, offset, count, epoch_[bucket], average, timeout_ticks_, err_dev_,
                     stream(), lo, hi, max_blocks_);
}

void XgmiComm::comm_wait_current() {
  hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream();
  stream_handoff(cur, stream(), ev_a_);
}

void XgmiComm::current_wait_comm() {
  hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream();
  stream_handoff(stream(), cur, ev_b_);
}

void XgmiComm::synchronize() {
  hipc(hipStreamSynchronize(stream()), "hipStreamSynchronize");
  check();
}

int XgmiComm::error_code() const {
  return (int)__atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
}

std::string XgmiComm::error_message() const {
  const unsigned e = (unsigned)error_code();
  if (e == 0) return "";
  const unsigned code = e & 0xffffu;
  const int b = (int)(code - 1) / 2;
  std::string m = "xgmi all-reduce (rank " + std::to_string(rank_) + "): bucket " + std::to_string(b);
  if (e & kXgmiPeerFailed) {
    m += " -- peer rank " + std::to_string((e >> 16) & 0x7fffu) + " failed first (it signalled POISON" +
         std::string(code % 2 ? " instead of its gradients" : " instead of its reduced shard") + ")";
  } else {
    m += std::string(code % 2 ? " -- peers never marked their gradients ready" :
                                " -- peers never published their reduced shards") +
         " within " + std::to_string(timeout_s_) +
         " s (a peer rank died, hung or issued a different bucket sequence)";
  }
  return m + "; this rank's bucket gradients were poisoned with NaN";
}

void XgmiComm::check() const {
  if (error_code() != 0) throw std::runtime_error(error_message());
}

}  // namespace pdt
