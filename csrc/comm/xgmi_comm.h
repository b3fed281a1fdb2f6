// Direct xGMI gradient all-reduce: per-rank buffers shared through IPC handles, one-hop
// reduce-scatter + all-gather over every peer link at once (kernels: csrc/kernels/xgmi.hip).
//
// The rank's flat fp32 gradient buffer IS one of the shared buffers (hipMalloc'd here and handed
// to the DDP flat parameter space through grad_buffer()), so a bucket needs no copy in or out:
// peers read the shards they own straight from it and the reduced shards land back in it.
#pragma once
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace pdt {

class XgmiComm : public std::enable_shared_from_this<XgmiComm> {
 public:
  // wire: "fp32" or "bf16" (packed copies on the wire, fp32 sums); max_blocks: CU budget of the
  // data kernels; exit_on_error: a host monitor thread ends the process (exit code 124, the
  // watchdog's) as soon as the device error word is set -- a wait timed out or a peer failed
  XgmiComm(int rank, int world, int device, int64_t numel, int nbuckets, double timeout_s,
           const std::string& wire = "fp32", int max_blocks = 16, bool exit_on_error = false);
  ~XgmiComm();

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  int64_t numel() const { return numel_; }
  hipStream_t stream() const { return stream_.stream(); }

  bool wire_bf16() const { return g16_ != nullptr; }
  bool flags_uncached() const { return flags_uncached_; }
  int max_blocks() const { return max_blocks_; }
  // IPC handles of (gradient buffer, reduced-shard buffer, flag array[, bf16 gradient copy,
  // bf16 reduced shards]), concatenated
  std::string ipc_handles() const;
  // map every peer's buffers from their handles (index = rank; the own entry is ignored)
  void open_peers(const std::vector<std::string>& handles);
  // in-process ranks (tests): use the other objects' device pointers directly, no IPC
  void link_local(const std::vector<std::shared_ptr<XgmiComm>>& all);
  // fp32 [numel] tensor over the shared gradient buffer (keeps this object alive)
  at::Tensor grad_buffer();

  // all-reduce elements [offset, offset + count) of the gradient buffer as bucket `bucket`
  // (average: divide by world), enqueued on the comm stream; the caller orders it after the
  // gradients' producers (comm_wait_current / events)
  void reduce_bucket(int bucket, int64_t offset, int64_t count, bool average);
  // phases [lo, hi] of the bucket protocol only (0 signal ready, 1 wait, 2 reduce-scatter,
  // 3 signal reduced, 4 wait, 5 all-gather); phase 0 starts a new epoch.  In-process rank groups
  // (tests) enqueue every rank's phase p before any rank's phase p+1.
  void reduce_bucket_phases(int bucket, int64_t offset, int64_t count, bool average, int lo, int hi);

  void comm_wait_current();
  void current_wait_comm();
  void synchronize();
  // 0 = healthy; otherwise 1 + 2*bucket (ready wait timed out) or 2 + 2*bucket (reduced wait),
  // with kXgmiPeerFailed | (peer << 16) set when the wait saw that peer's POISON signal
  int error_code() const;
  std::string error_message() const;  // "" when healthy
  void check() const;

 private:
  int rank_, world_, device_;
  int64_t numel_;
  int nbuckets_;
  double timeout_s_;
  uint64_t timeout_ticks_ = 0;
  float* g_ = nullptr;
  float* red_ = nullptr;
  unsigned* flags_ = nullptr;
  bool flags_uncached_ = false;  // flags in hipDeviceMallocUncached memory (fine-grained)
  uint16_t* g16_ = nullptr;   // bf16 wire only
  uint16_t* red16_ = nullptr;
  int max_blocks_ = 16;
  bool exit_on_error_ = false;
  std::atomic<bool> stop_{false};
  std::thread monitor_;
  void monitor_loop();
  unsigned* err_host_ = nullptr;  // pinned, device-visible error word
  unsigned* err_dev_ = nullptr;
  const float* gp_[8] = {};
  const float* rp_[8] = {};
  unsigned* fp_[8] = {};
  const uint16_t* g16p_[8] = {};
  const uint16_t* r16p_[8] = {};
  std::vector<void*> opened_;
  std::vector<unsigned> epoch_;
  bool linked_ = false;
  c10::hip::HIPStream stream_;
  hipEvent_t ev_a_ = nullptr, ev_b_ = nullptr;
};

}  // namespace pdt
