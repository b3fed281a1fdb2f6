#include "rccl_comm.h"

#include <c10/hip/HIPGuard.h>

#include <cstdlib>
#include <stdexcept>

namespace pdt {

void rccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(r));
  }
}

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

// The comm stream is an ordinary-priority stream.  A high-priority stream was measured to cost
// +16.5 ms per ResNet-50 step on MI355X (21.6 -> 38.1 ms, world-1 forced reducer) even with the
// collectives skipped (PDT_REDUCER_SKIP_COLL=1: 38.0 ms): its event waits, not RCCL, stall the
// compute queues.  PDT_COMM_HIGH_PRIORITY=1 restores it for A/B runs
// (profiles/r2_comm_stream_priority_ab.md).
static bool comm_high_priority() {
  const char* e = std::getenv("PDT_COMM_HIGH_PRIORITY");
  return e && e[0] == '1';
}

RcclComm::RcclComm(const std::string& uid, int rank, int world, int device)
    : rank_(rank), world_(world), device_(device),
      stream_(c10::hip::getStreamFromPool(comm_high_priority(), (c10::DeviceIndex)device)) {
  if (uid.size() != sizeof(ncclUniqueId::internal)) throw std::runtime_error("bad RCCL unique id size");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  ncclUniqueId id;
  memcpy(id.internal, uid.data(), sizeof(id.internal));
  rccl_check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
  hip_check(hipEventCreateWithFlags(&ev_a_, hipEventDisableTiming), "hipEventCreate");
  hip_check(hipEventCreateWithFlags(&ev_b_, hipEventDisableTiming), "hipEventCreate");
  barrier_buf_ = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device));
}

RcclComm::~RcclComm() {
  if (comm_) {
    ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
  if (ev_a_) hipEventDestroy(ev_a_);
  if (ev_b_) hipEventDestroy(ev_b_);
}

void RcclComm::abort() {
  if (comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
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
  hip_check(hipEventRecord(ev_a_, cur), "hipEventRecord");
  hip_check(hipStreamWaitEvent(stream(), ev_a_, 0), "hipStreamWaitEvent");
}

void RcclComm::current_wait_comm() {
  hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream();
  hip_check(hipEventRecord(ev_b_, stream()), "hipEventRecord");
  hip_check(hipStreamWaitEvent(cur, ev_b_, 0), "hipStreamWaitEvent");
}

void RcclComm::synchronize() { hip_check(hipStreamSynchronize(stream()), "hipStreamSynchronize"); }

static void check_dev(const at::Tensor& t, int device) {
  if (!t.is_cuda() || t.get_device() != device || !t.is_contiguous())
    throw std::runtime_error("RcclComm: tensor must be a contiguous tensor on the comm device");
}

void RcclComm::all_reduce_raw(void* ptr, size_t count, ncclDataType_t dt, ncclRedOp_t op) {
  rccl_check(ncclAllReduce(ptr, ptr, count, dt, op, comm_, stream()), "ncclAllReduce");
}

void RcclComm::all_reduce(const at::Tensor& t, const std::string& op, bool wait_current) {
  check_dev(t, device_);
  if (wait_current) comm_wait_current();
  all_reduce_raw(t.data_ptr(), (size_t)t.numel(), dtype_of(t), op_of(op));
}

void RcclComm::broadcast(const at::Tensor& t, int root, bool wait_current) {
  check_dev(t, device_);
  if (wait_current) comm_wait_current();
  rccl_check(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), root, comm_,
                           stream()),
             "ncclBroadcast");
}

void RcclComm::reduce_scatter(const at::Tensor& in, const at::Tensor& out, const std::string& op,
                              bool wait_current) {
  check_dev(in, device_);
  check_dev(out, device_);
  if (in.numel() != out.numel() * world_) throw std::runtime_error("reduce_scatter: size mismatch");
  if (wait_current) comm_wait_current();
  rccl_check(ncclReduceScatter(in.data_ptr(), out.data_ptr(), (size_t)out.numel(), dtype_of(in),
                               op_of(op), comm_, stream()),
             "ncclReduceScatter");
}

void RcclComm::all_gather(const at::Tensor& in, const at::Tensor& out, bool wait_current) {
  check_dev(in, device_);
  check_dev(out, device_);
  if (out.numel() != in.numel() * world_) throw std::runtime_error("all_gather: size mismatch");
  if (wait_current) comm_wait_current();
  rccl_check(ncclAllGather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), dtype_of(in), comm_,
                           stream()),
             "ncclAllGather");
}

void RcclComm::barrier() {
  all_reduce(barrier_buf_, "sum", true);
  synchronize();
}

}  // namespace pdt
