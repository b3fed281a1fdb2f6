// Direct one-hop gradient all-reduce over xGMI peer memory (reduce-scatter + all-gather).
//
// An 8x MI355X node is fully connected: every GPU has 7 point-to-point xGMI links.  A ring
// all-reduce pushes each byte through ONE link per step, so it runs at one link's rate; here
// every rank reads its 1/W shard of a bucket from ALL peers at once (W-1 links in parallel),
// sums it in fp32, and then every rank copies the W-1 reduced shards it does not own back
// from their owners (again all links at once) -- 2*(W-1)/W of the bucket per rank, spread
// over W-1 links instead of one (option 2).
//
// Peer buffers are hipMalloc'd by each rank (csrc/comm/xgmi_comm.cpp) and mapped into the others
// with IPC handles exchanged through the rendezvous store.  Cross-process ordering uses epoch
// flags in each rank's own flag array, written by peers:
//   ready[b][q]   = e  : rank q's gradients of bucket b, epoch e, are final (kernel boundary
//                        on q's stream = its writes are visible device-wide; the flag store is a
//                        system-scope release)
//   reduced[b][q] = e  : rank q's reduced shard of bucket b is final
// A waiting kernel is ONE wave that polls its own flags (system-scope acquire loads, s_sleep
// between polls) with a bounded spin: past the deadline it records an error code in a
// host-visible word and returns -- it never hangs the GPU; the data kernels that follow check
// that word and skip their work.  The data kernels run after the wait kernel on the same stream
// and open with a system-scope acquire fence in every workgroup (each XCD's L2 drops stale
// copies of peer lines before reading them).
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace pdt {

constexpr int kXgmiMaxRanks = 8;

struct XgmiPtrs {
  const float* g[kXgmiMaxRanks];    // every rank's gradient buffer (own included)
  const float* red[kXgmiMaxRanks];  // every rank's reduced-shard buffer
  unsigned* flags[kXgmiMaxRanks];   // every rank's flag array
};

__device__ __forceinline__ unsigned ld_acquire_sys(const unsigned* p) {
  return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// thread q < world stores `epoch` into rank q's flags[slot*8 + rank]
__global__ void xgmi_signal_kernel(XgmiPtrs P, int world, int rank, int slot, unsigned epoch) {
  const int q = threadIdx.x;
  if (q < world) {
    __hip_atomic_store(P.flags[q] + slot * kXgmiMaxRanks + rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// one wave: wait until own flags[slot*8 + q] >= epoch for every q < world (wrap-safe compare),
// or record `code` in *err once the deadline (wall-clock ticks, 100 MHz) has passed
__global__ void xgmi_wait_kernel(const unsigned* flags, int world, int slot, unsigned epoch,
                                 unsigned long long timeout_ticks, unsigned* err, unsigned code) {
  const int q = threadIdx.x;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;  // already failed
  const unsigned long long t0 = wall_clock64();
  bool done = q >= world;
  while (true) {
    if (!done) done = (int)(ld_acquire_sys(flags + slot * kXgmiMaxRanks + q) - epoch) >= 0;
    if (__all(done)) break;
    if (wall_clock64() - t0 > timeout_ticks) {
      if (q == 0) {  // keep the FIRST failure's code
        unsigned expected = 0u;
        __hip_atomic_compare_exchange_strong(err, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

__device__ __forceinline__ bool xgmi_failed(const unsigned* err) {
  return __hip_atomic_load(const_cast<unsigned*>(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}

// red_own[i] = sum_{q=0..W-1} g_q[i] (rank order, fp32) for i in [lo, hi)
template <bool VEC>
__global__ void __launch_bounds__(256) xgmi_reduce_scatter_kernel(XgmiPtrs P, int world, int rank,
                                                                  int64_t lo, int64_t hi,
                                                                  const unsigned* err) {
  if (xgmi_failed(err)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: drop stale peer lines
  float* out = const_cast<float*>(P.red[rank]);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (VEC) {
    for (int64_t i = lo / 4 + t; i < hi / 4; i += stride) {
      float4 s = reinterpret_cast<const float4*>(P.g[0])[i];
      for (int q = 1; q < world; ++q) {
        const float4 v = reinterpret_cast<const float4*>(P.g[q])[i];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      reinterpret_cast<float4*>(out)[i] = s;
    }
  } else {
    for (int64_t i = lo + t; i < hi; i += stride) {
      float s = P.g[0][i];
      for (int q = 1; q < world; ++q) s += P.g[q][i];
      out[i] = s;
    }
  }
}

// g_own[i] = red_{owner(i)}[i] / world (average) or red_{owner(i)}[i] (sum), over the bucket
// [lo, hi) whose shard q is [lo + q*shard, lo + (q+1)*shard)
template <bool VEC>
__global__ void __launch_bounds__(256) xgmi_all_gather_kernel(XgmiPtrs P, int world, int rank,
                                                              int64_t lo, int64_t hi, int64_t shard,
                                                              int average, const unsigned* err) {
  if (xgmi_failed(err)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  float* g = const_cast<float*>(P.g[rank]);
  const float w = (float)world;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (VEC) {
    for (int64_t i = lo / 4 + t; i < hi / 4; i += stride) {
      const int q = (int)((i * 4 - lo) / shard);
      float4 v = reinterpret_cast<const float4*>(P.red[q])[i];
      if (average) { v.x /= w; v.y /= w; v.z /= w; v.w /= w; }
      reinterpret_cast<float4*>(g)[i] = v;
    }
  } else {
    for (int64_t i = lo + t; i < hi; i += stride) {
      const int q = (int)((i - lo) / shard);
      const float v = P.red[q][i];
      g[i] = average ? v / w : v;
    }
  }
}

static XgmiPtrs make_ptrs(const float* const* g, const float* const* red, unsigned* const* flags, int world) {
  if (world < 1 || world > kXgmiMaxRanks) throw std::runtime_error("xgmi: world must be 1..8");
  XgmiPtrs P{};
  for (int q = 0; q < world; ++q) {
    P.g[q] = g[q];
    P.red[q] = red[q];
    P.flags[q] = flags[q];
  }
  return P;
}

static void check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

int xgmi_max_ranks() { return kXgmiMaxRanks; }

void launch_xgmi_bucket(const float* const* g, const float* const* red, unsigned* const* flags, int world,
                        int rank, int bucket, int64_t lo, int64_t count, unsigned epoch, bool average,
                        uint64_t timeout_ticks, unsigned* err, hipStream_t st, int phase_lo, int phase_hi) {
  const XgmiPtrs P = make_ptrs(g, red, flags, world);
  const int64_t hi = lo + count;
  // shard size: a multiple of 4 elements so shard boundaries keep float4 alignment when the bucket
  // does; the last shard may be shorter (or empty)
  const int64_t shard = ((count + world - 1) / world + 3) / 4 * 4;
  const bool vec = (lo % 4) == 0 && (count % 4) == 0;
  const int64_t own_lo = std::min(hi, lo + rank * shard), own_hi = std::min(hi, own_lo + shard);
  const int slot_ready = bucket * 2, slot_red = bucket * 2 + 1;
  auto blocks = [](int64_t n) {
    int64_t b = (n + 1023) / 1024;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, 1024));
  };
  auto on = [&](int ph) { return ph >= phase_lo && ph <= phase_hi; };
  // phase 0: signal ready, 1: wait ready, 2: reduce-scatter, 3: signal reduced, 4: wait reduced,
  // 5: all-gather (in-process rank groups enqueue phase-major so that no rank's wait can sit in a
  // hardware queue ahead of another rank's signal)
  if (on(0)) hipLaunchKernelGGL(xgmi_signal_kernel, dim3(1), dim3(64), 0, st, P, world, rank, slot_ready, epoch);
  if (on(1)) hipLaunchKernelGGL(xgmi_wait_kernel, dim3(1), dim3(64), 0, st, P.flags[rank], world, slot_ready, epoch,
                                (unsigned long long)timeout_ticks, err, 1u + 2u * (unsigned)bucket);
  if (on(2) && own_hi > own_lo) {
    if (vec) hipLaunchKernelGGL(xgmi_reduce_scatter_kernel<true>, dim3(blocks(own_hi - own_lo)), dim3(256), 0, st,
                                P, world, rank, own_lo, own_hi, err);
    else hipLaunchKernelGGL(xgmi_reduce_scatter_kernel<false>, dim3(blocks(own_hi - own_lo)), dim3(256), 0, st,
                            P, world, rank, own_lo, own_hi, err);
  }
  if (on(3)) hipLaunchKernelGGL(xgmi_signal_kernel, dim3(1), dim3(64), 0, st, P, world, rank, slot_red, epoch);
  if (on(4)) hipLaunchKernelGGL(xgmi_wait_kernel, dim3(1), dim3(64), 0, st, P.flags[rank], world, slot_red, epoch,
                                (unsigned long long)timeout_ticks, err, 2u + 2u * (unsigned)bucket);
  if (!on(5)) {
    check("xgmi bucket");
    return;
  }
  if (vec) hipLaunchKernelGGL(xgmi_all_gather_kernel<true>, dim3(blocks(count)), dim3(256), 0, st, P, world, rank,
                              lo, hi, shard, average ? 1 : 0, err);
  else hipLaunchKernelGGL(xgmi_all_gather_kernel<false>, dim3(blocks(count)), dim3(256), 0, st, P, world, rank,
                          lo, hi, shard, average ? 1 : 0, err);
  check("xgmi bucket");
}

}  // namespace pdt
