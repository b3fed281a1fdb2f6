#include "xgmi_comm.h"

#include <c10/hip/HIPGuard.h>

#include <cstring>
#include <stdexcept>

#include "../kernels/kernels.h"

namespace pdt {

static void hipc(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("xgmi: ") + what + ": " + hipGetErrorString(e));
}

XgmiComm::XgmiComm(int rank, int world, int device, int64_t numel, int nbuckets, double timeout_s)
    : rank_(rank), world_(world), device_(device), numel_(numel), nbuckets_(nbuckets),
      timeout_s_(timeout_s), stream_(c10::hip::getStreamFromPool(false, (c10::DeviceIndex)device)) {
  if (world < 1 || world > xgmi_max_ranks()) throw std::runtime_error("xgmi: world size must be 1..8");
  if (rank < 0 || rank >= world) throw std::runtime_error("xgmi: bad rank");
  if (numel <= 0 || nbuckets <= 0) throw std::runtime_error("xgmi: empty gradient space");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  hipc(hipMalloc(&g_, numel * sizeof(float)), "hipMalloc(grad)");
  hipc(hipMalloc(&red_, numel * sizeof(float)), "hipMalloc(reduced)");
  const size_t fbytes = (size_t)nbuckets * 2 * 8 * sizeof(unsigned);
  hipc(hipMalloc(&flags_, fbytes), "hipMalloc(flags)");
  hipc(hipMemset(g_, 0, numel * sizeof(float)), "hipMemset");
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
  hipc(hipEventCreateWithFlags(&ev_a_, hipEventDisableTiming), "hipEventCreate");
  hipc(hipEventCreateWithFlags(&ev_b_, hipEventDisableTiming), "hipEventCreate");
  hipc(hipDeviceSynchronize(), "hipDeviceSynchronize");  // zeroed flags visible before any peer signals
}

XgmiComm::~XgmiComm() {
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  hipStreamSynchronize(stream());
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  if (g_) hipFree(g_);
  if (red_) hipFree(red_);
  if (flags_) hipFree(flags_);
  if (err_host_) hipHostFree(err_host_);
  if (ev_a_) hipEventDestroy(ev_a_);
  if (ev_b_) hipEventDestroy(ev_b_);
}

std::string XgmiComm::ipc_handles() const {
  hipIpcMemHandle_t h[3];
  hipc(hipIpcGetMemHandle(&h[0], g_), "hipIpcGetMemHandle(grad)");
  hipc(hipIpcGetMemHandle(&h[1], red_), "hipIpcGetMemHandle(reduced)");
  hipc(hipIpcGetMemHandle(&h[2], flags_), "hipIpcGetMemHandle(flags)");
  return std::string(reinterpret_cast<const char*>(h), sizeof(h));
}

void XgmiComm::open_peers(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::runtime_error("xgmi: need one handle set per rank");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  for (int q = 0; q < world_; ++q) {
    if (q == rank_) continue;
    if (handles[q].size() != 3 * sizeof(hipIpcMemHandle_t)) throw std::runtime_error("xgmi: bad handle size");
    hipIpcMemHandle_t h[3];
    memcpy(h, handles[q].data(), sizeof(h));
    void* p[3];
    for (int i = 0; i < 3; ++i) {
      hipc(hipIpcOpenMemHandle(&p[i], h[i], hipIpcMemLazyEnablePeerAccess),
           ("hipIpcOpenMemHandle(rank " + std::to_string(q) + ")").c_str());
      opened_.push_back(p[i]);
    }
    gp_[q] = static_cast<const float*>(p[0]);
    rp_[q] = static_cast<const float*>(p[1]);
    fp_[q] = static_cast<unsigned*>(p[2]);
  }
  linked_ = true;
}

void XgmiComm::link_local(const std::vector<std::shared_ptr<XgmiComm>>& all) {
  if ((int)all.size() != world_) throw std::runtime_error("xgmi: need one communicator per rank");
  for (int q = 0; q < world_; ++q) {
    if (all[q]->rank_ != q || all[q]->world_ != world_ || all[q]->numel_ != numel_)
      throw std::runtime_error("xgmi: link_local expects ranks 0..world-1 of one gradient space");
    gp_[q] = all[q]->g_;
    rp_[q] = all[q]->red_;
    fp_[q] = all[q]->flags_;
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
  launch_xgmi_bucket(gp_, rp_, fp_, world_, rank_, bucket, offset, count, epoch_[bucket], average, timeout_ticks_,
                     err_dev_, stream(), lo, hi);
}

void XgmiComm::comm_wait_current() {
  hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream();
  hipc(hipEventRecord(ev_a_, cur), "hipEventRecord");
  hipc(hipStreamWaitEvent(stream(), ev_a_, 0), "hipStreamWaitEvent");
}

void XgmiComm::current_wait_comm() {
  hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream();
  hipc(hipEventRecord(ev_b_, stream()), "hipEventRecord");
  hipc(hipStreamWaitEvent(cur, ev_b_, 0), "hipStreamWaitEvent");
}

void XgmiComm::synchronize() {
  hipc(hipStreamSynchronize(stream()), "hipStreamSynchronize");
  check();
}

int XgmiComm::error_code() const {
  return (int)__atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
}

void XgmiComm::check() const {
  const int e = error_code();
  if (e != 0) {
    const int b = (e - 1) / 2;
    throw std::runtime_error("xgmi all-reduce (rank " + std::to_string(rank_) + "): bucket " + std::to_string(b) +
                             (e % 2 ? " -- peers never marked their gradients ready" :
                                      " -- peers never published their reduced shards") +
                             " within " + std::to_string(timeout_s_) +
                             " s (a peer rank died, hung or issued a different bucket sequence)");
  }
}

}  // namespace pdt
