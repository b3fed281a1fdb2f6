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
// host-visible word and returns -- it never hangs the GPU.  Failure is never silent:
//   * a rank whose error word is set signals POISON instead of its epoch, so a peer waiting on
//     it fails too (its own error word records "peer q failed") instead of reading a shard that
//     was never reduced (a late peer would otherwise see a current epoch and gather stale data);
//   * the reduce-scatter of a failed rank is skipped and its all-gather writes NaN over the
//     bucket, so an optimizer step that still runs on this rank cannot use local, unreduced
//     gradients (the communicator's host monitor ends the process meanwhile, xgmi_comm.cpp).
// The data kernels run after the wait kernel on the same stream and open with a system-scope
// acquire fence in every workgroup (each XCD's L2 drops stale copies of peer lines).
//
// CU budget: the data kernels run at most `max_blocks` workgroups (RCCL-channel-like, default
// 16): they stream over xGMI beside the backward pass, and a full-chip grid would take the CUs
// the remaining backward kernels need.  Each thread keeps UNROLL 16-byte loads per peer in
// flight (remote latency is microseconds), loads are nontemporal (read once), and the shard
// owner of an all-gather element comes from the loop structure, not a division.
//
// Wire formats: fp32 (the shared gradient buffer itself) or bf16 (half the xGMI bytes): each
// rank first packs its bucket into a shared bf16 copy, shards are summed in fp32 from the bf16
// inputs and published as bf16, and the all-gather widens back into the fp32 buffer -- two
// roundings per element (input, reduced sum), the bound tests/test_wire_cpu.py pins for 8 ranks.
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace pdt {

constexpr int kXgmiMaxRanks = 8;
constexpr unsigned kXgmiPoison = 0xffffffffu;  // flag value: the signalling rank has failed
// RS -> AG pipelining: a bucket's shards are reduced, published and gathered in up to
// kXgmiMaxChunks chunks, so the all-gather of chunk c starts while peers still reduce chunk c+1
// (one reduced-flag slot per chunk; the ready slot is shared)
constexpr int kXgmiMaxChunks = 4;
constexpr int kXgmiSlotsPerBucket = 1 + kXgmiMaxChunks;
constexpr int64_t kXgmiMinChunk = 1 << 18;  // elements of one rank's shard per chunk (1 MB fp32)

struct XgmiPtrs {
  const float* g[kXgmiMaxRanks];    // every rank's gradient buffer (own included)
  const float* red[kXgmiMaxRanks];  // every rank's reduced-shard buffer (fp32 wire)
  unsigned* flags[kXgmiMaxRanks];   // every rank's flag array
  const uint16_t* g16[kXgmiMaxRanks];    // bf16 wire: packed gradient copies
  const uint16_t* red16[kXgmiMaxRanks];  // bf16 wire: reduced shards
};

__device__ __forceinline__ unsigned ld_acquire_sys(const unsigned* p) {
  return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ bool xgmi_failed(const unsigned* err) {
  return __hip_atomic_load(const_cast<unsigned*>(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}

// thread q < world stores `epoch` (or POISON once this rank has failed) into rank q's
// flags[slot*8 + rank]
__global__ void xgmi_signal_kernel(XgmiPtrs P, int world, int rank, int slot, unsigned epoch, const unsigned* err) {
  const int q = threadIdx.x;
  if (q < world) {
    const unsigned v = xgmi_failed(err) ? kXgmiPoison : epoch;
    __hip_atomic_store(P.flags[q] + slot * kXgmiMaxRanks + rank, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// one wave: wait until own flags[slot*8 + q] >= epoch for every q < world (wrap-safe compare).
// Past the deadline (wall-clock ticks, 100 MHz) record `code`; a POISON flag records
// kXgmiPeerFailed | (q << 16) | code at once.
__global__ void xgmi_wait_kernel(const unsigned* flags, int world, int slot, unsigned epoch,
                                 unsigned long long timeout_ticks, unsigned* err, unsigned code) {
  const int q = threadIdx.x;
  if (xgmi_failed(err)) return;  // already failed: the next signal poisons the peers
  const unsigned long long t0 = wall_clock64();
  bool done = q >= world;
  while (true) {
    bool poison = false;
    if (!done) {
      const unsigned v = ld_acquire_sys(flags + slot * kXgmiMaxRanks + q);
      poison = v == kXgmiPoison;
      done = !poison && (int)(v - epoch) >= 0;
    }
    const unsigned long long pm = __ballot(poison);
    if (pm != 0ull) {
      if (q == 0) {  // keep the FIRST failure's code
        const unsigned who = (unsigned)__builtin_ctzll(pm);
        unsigned expected = 0u;
        __hip_atomic_compare_exchange_strong(err, &expected, kXgmiPeerFailed | (who << 16) | code, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      break;
    }
    if (__all(done)) break;
    if (wall_clock64() - t0 > timeout_ticks) {
      if (q == 0) {
        unsigned expected = 0u;
        __hip_atomic_compare_exchange_strong(err, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

constexpr int kXgmiUnroll = 4;  // 16-byte loads per peer in flight per thread

typedef float xv4f __attribute__((ext_vector_type(4)));
typedef unsigned xv4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldnt4(const float* p, int64_t i) {
  const xv4f v = __builtin_nontemporal_load(reinterpret_cast<const xv4f*>(p) + i);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stnt4(float* p, int64_t i, float4 v) {
  __builtin_nontemporal_store(xv4f{v.x, v.y, v.z, v.w}, reinterpret_cast<xv4f*>(p) + i);
}
__device__ __forceinline__ uint4 ldnt_u4(const void* p, int64_t i) {
  const xv4u v = __builtin_nontemporal_load(reinterpret_cast<const xv4u*>(p) + i);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stnt_u4(void* p, int64_t i, uint4 v) {
  __builtin_nontemporal_store(xv4u{v.x, v.y, v.z, v.w}, reinterpret_cast<xv4u*>(p) + i);
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// bf16 <-> fp32 for 8 packed values (round to nearest even; NaN stays NaN via the conversion
// instruction: MI355X_MICROARCH correctness table)
__device__ __forceinline__ uint4 pack8_bf16(float4 a, float4 b) {
  auto cv = [](float lo, float hi) {
    const __bf16 l = (__bf16)lo, h = (__bf16)hi;
    return (unsigned)__builtin_bit_cast(uint16_t, l) | ((unsigned)__builtin_bit_cast(uint16_t, h) << 16);
  };
  return make_uint4(cv(a.x, a.y), cv(a.z, a.w), cv(b.x, b.y), cv(b.z, b.w));
}
__device__ __forceinline__ void unpack8_bf16(uint4 u, float4& a, float4& b) {
  auto lo = [](unsigned w) { return __uint_as_float(w << 16); };
  auto hi = [](unsigned w) { return __uint_as_float(w & 0xffff0000u); };
  a = make_float4(lo(u.x), hi(u.x), lo(u.y), hi(u.y));
  b = make_float4(lo(u.z), hi(u.z), lo(u.w), hi(u.w));
}

// red_own[i] = sum_{q=0..W-1} g_q[i] (rank order, fp32) for i in [lo, hi), float4 units.
// WORLD > 0: compile-time rank count (loads of every peer issued before the adds); 0: runtime.
// Element range [a, b) of a kernel: the body runs in U-element vector units over
// [ceil_U(a), floor_U(b)); the at most 2(U-1) edge elements go to threads 0..U-1 of block 0.
struct XRange {
  int64_t va, vb;  // vector body in units
};
// Body units [ceil(a/U), floor(b/U)), empty when [a, b) holds no whole unit (then vb = va).  The
// edges are [a, min(b, va*U)) and [max(vb*U, min(b, va*U)), b): disjoint, inside [a, b), and
// together with the body exactly [a, b) -- also when the range sits inside one unit at an
// unaligned offset (a = 5, b = 7 with U = 4: left edge 5, 6; no body; no right edge).
template <int U>
__device__ __forceinline__ XRange xrange(int64_t a, int64_t b) {
  const int64_t va = (a + U - 1) / U;
  const int64_t vb = b / U > va ? b / U : va;
  return {va, vb};
}
template <int U, class F>
__device__ __forceinline__ void xedges(int64_t a, int64_t b, F&& f) {
  const XRange r = xrange<U>(a, b);
  const int t = threadIdx.x;
  if (blockIdx.x == 0 && t < U) {
    const int64_t lend = b < r.va * U ? b : r.va * U;
    const int64_t rbeg = r.vb * U > lend ? r.vb * U : lend;
    if (a + t < lend) f(a + t);
    if (rbeg + t < b) f(rbeg + t);
  }
}

template <int WORLD>
__global__ void __launch_bounds__(256) xgmi_reduce_scatter_kernel(XgmiPtrs P, int world, int rank, int64_t a,
                                                                  int64_t b, const unsigned* err) {
  if (xgmi_failed(err)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: drop stale peer lines
  constexpr int W = WORLD > 0 ? WORLD : kXgmiMaxRanks;
  const int nw = WORLD > 0 ? WORLD : world;
  float* out = const_cast<float*>(P.red[rank]);
  xedges<4>(a, b, [&](int64_t e) {
    float s = P.g[0][e];
    for (int q = 1; q < nw; ++q) s += P.g[q][e];
    out[e] = s;
  });
  const XRange r = xrange<4>(a, b);
  const int64_t lo4 = r.va, hi4 = r.vb;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = lo4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (kXgmiUnroll - 1) * stride < hi4; i += kXgmiUnroll * stride) {
    float4 v[kXgmiUnroll][W];
#pragma unroll
    for (int q = 0; q < W; ++q)
      if (q < nw)
#pragma unroll
        for (int u = 0; u < kXgmiUnroll; ++u) v[u][q] = ldnt4(P.g[q], i + u * stride);
#pragma unroll
    for (int u = 0; u < kXgmiUnroll; ++u) {
      float4 s = v[u][0];
#pragma unroll
      for (int q = 1; q < W; ++q)
        if (q < nw) s = add4(s, v[u][q]);
      stnt4(out, i + u * stride, s);
    }
  }
  for (; i < hi4; i += stride) {
    float4 s = ldnt4(P.g[0], i);
    for (int q = 1; q < nw; ++q) s = add4(s, ldnt4(P.g[q], i));
    stnt4(out, i, s);
  }
}

// bf16 wire: red16_own[8i..8i+7] = bf16(sum_q float(g16_q[...])) for 8-element units [lo8, hi8)
__device__ __forceinline__ float bf16f(uint16_t v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ uint16_t f2bf16(float v) { return __builtin_bit_cast(uint16_t, (__bf16)v); }

template <int WORLD>
__global__ void __launch_bounds__(256) xgmi_reduce_scatter_bf16_kernel(XgmiPtrs P, int world, int rank,
                                                                       int64_t a, int64_t b, const unsigned* err) {
  if (xgmi_failed(err)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  constexpr int W = WORLD > 0 ? WORLD : kXgmiMaxRanks;
  const int nw = WORLD > 0 ? WORLD : world;
  uint16_t* out16 = const_cast<uint16_t*>(P.red16[rank]);
  xedges<8>(a, b, [&](int64_t e) {
    float s = bf16f(P.g16[0][e]);
    for (int q = 1; q < nw; ++q) s += bf16f(P.g16[q][e]);
    out16[e] = f2bf16(s);
  });
  const XRange r = xrange<8>(a, b);
  uint4* out = reinterpret_cast<uint4*>(out16);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = r.va + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.vb; i += stride) {
    uint4 v[W];
#pragma unroll
    for (int q = 0; q < W; ++q)
      if (q < nw) v[q] = ldnt_u4(P.g16[q], i);
    float4 a, b;
    unpack8_bf16(v[0], a, b);
#pragma unroll
    for (int q = 1; q < W; ++q)
      if (q < nw) {
        float4 c, d;
        unpack8_bf16(v[q], c, d);
        a = add4(a, c);
        b = add4(b, d);
      }
    stnt_u4(out, i, pack8_bf16(a, b));
  }
}

// bf16 wire, before signalling ready: g16_own[lo8..hi8) = bf16(g_own)
__global__ void __launch_bounds__(256) xgmi_pack_bf16_kernel(XgmiPtrs P, int rank, int64_t a, int64_t b) {
  uint16_t* o16 = const_cast<uint16_t*>(P.g16[rank]);
  xedges<8>(a, b, [&](int64_t e) { o16[e] = f2bf16(P.g[rank][e]); });
  const XRange r = xrange<8>(a, b);
  const float4* g = reinterpret_cast<const float4*>(P.g[rank]);
  uint4* o = reinterpret_cast<uint4*>(o16);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = r.va + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.vb; i += stride)
    o[i] = pack8_bf16(g[2 * i], g[2 * i + 1]);
}

// g_own[i] = red_{q}[i] / world (average) or red_q[i] (sum) for i in shard q of the bucket
// [lo, hi): shard q = [max(lo, base + q*shard), min(hi, base + (q+1)*shard)), base = lo rounded
// down to 8.  A failed rank writes NaN over the bucket instead (poison; see the header).
// Chunk [sub_off, sub_off + sub_len) of every shard (the whole shard: 0, shard).
template <bool BF16>
__global__ void __launch_bounds__(256) xgmi_all_gather_kernel(XgmiPtrs P, int world, int rank, int64_t lo,
                                                              int64_t hi, int64_t shard, int64_t sub_off,
                                                              int64_t sub_len, int average, const unsigned* err) {
  float* g = const_cast<float*>(P.g[rank]);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (xgmi_failed(err)) {
    const float nan = __builtin_nanf("");
    for (int64_t i = lo + t0; i < hi; i += stride) g[i] = nan;
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  // divide (not multiply by 1/world): bitwise the torch DDP / gloo average, sum / world
  const float w = average ? (float)world : 1.0f;
  const int64_t base = lo / 8 * 8;
  for (int q = 0; q < world; ++q) {
    const int64_t s0 = base + q * shard;
    const int64_t a = std::max(lo, std::min(hi, s0 + sub_off));
    const int64_t b = std::min(hi, std::min(s0 + shard, s0 + sub_off + sub_len));
    if (a >= b) continue;
    if constexpr (BF16) {
      const uint16_t* r16 = P.red16[q];
      xedges<8>(a, b, [&](int64_t e) { g[e] = bf16f(r16[e]) / w; });
      const XRange r = xrange<8>(a, b);
      const uint4* src = reinterpret_cast<const uint4*>(r16);
      float4* dst = reinterpret_cast<float4*>(g);
      for (int64_t i = r.va + t0; i < r.vb; i += stride) {
        float4 x, y;
        unpack8_bf16(ldnt_u4(src, i), x, y);
        dst[2 * i] = make_float4(x.x / w, x.y / w, x.z / w, x.w / w);
        dst[2 * i + 1] = make_float4(y.x / w, y.y / w, y.z / w, y.w / w);
      }
    } else {
      const float* rq = P.red[q];
      xedges<4>(a, b, [&](int64_t e) { g[e] = rq[e] / w; });
      const XRange r = xrange<4>(a, b);
      int64_t i = r.va + t0;
      for (; i + (kXgmiUnroll - 1) * stride < r.vb; i += kXgmiUnroll * stride) {
        float4 v[kXgmiUnroll];
#pragma unroll
        for (int u = 0; u < kXgmiUnroll; ++u) v[u] = ldnt4(rq, i + u * stride);
#pragma unroll
        for (int u = 0; u < kXgmiUnroll; ++u)
          reinterpret_cast<float4*>(g)[i + u * stride] = make_float4(v[u].x / w, v[u].y / w, v[u].z / w, v[u].w / w);
      }
      for (; i < r.vb; i += stride) {
        const float4 v = ldnt4(rq, i);
        reinterpret_cast<float4*>(g)[i] = make_float4(v.x / w, v.y / w, v.z / w, v.w / w);
      }
    }
  }
}

static XgmiPtrs make_ptrs(const XgmiBuffers& B, int world) {
  if (world < 1 || world > kXgmiMaxRanks) throw std::runtime_error("xgmi: world must be 1..8");
  XgmiPtrs P{};
  for (int q = 0; q < world; ++q) {
    P.g[q] = B.g[q];
    P.red[q] = B.red[q];
    P.flags[q] = B.flags[q];
    P.g16[q] = B.g16[q];
    P.red16[q] = B.red16[q];
  }
  return P;
}

static void check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

int xgmi_max_ranks() { return kXgmiMaxRanks; }
int xgmi_slots_per_bucket() { return kXgmiSlotsPerBucket; }

// Test hook: pin the chunk count of every bucket (1..kXgmiMaxChunks), or -1 for the size policy.
static int g_xgmi_chunks = -1;
void xgmi_force_chunks(int n) { g_xgmi_chunks = n; }

// chunks per bucket: one per kXgmiMinChunk elements of a shard, at most kXgmiMaxChunks; world 1
// has no peers to overlap with
static int xgmi_chunks(int64_t shard, int world) {
  if (g_xgmi_chunks > 0) return std::min(kXgmiMaxChunks, g_xgmi_chunks);
  if (world <= 1) return 1;
  return (int)std::max<int64_t>(1, std::min<int64_t>(kXgmiMaxChunks, shard / kXgmiMinChunk));
}

// shard of the bucket [lo, lo + count): a multiple of 8 elements counted from lo rounded down to
// 8, so every interior shard boundary is 32-B aligned (float4 / 8 x bf16 units stay whole); the
// last shard may be shorter or empty
int64_t xgmi_shard(int64_t lo, int64_t count, int world) {
  const int64_t span = lo + count - lo / 8 * 8;
  return ((span + world - 1) / world + 7) / 8 * 8;
}

template <int W>
static void launch_rs(const XgmiPtrs& P, bool bf16, int world, int rank, int64_t a, int64_t b, unsigned grid,
                      const unsigned* err, hipStream_t st) {
  if (bf16)
    hipLaunchKernelGGL(xgmi_reduce_scatter_bf16_kernel<W>, dim3(grid), dim3(256), 0, st, P, world, rank, a, b, err);
  else
    hipLaunchKernelGGL(xgmi_reduce_scatter_kernel<W>, dim3(grid), dim3(256), 0, st, P, world, rank, a, b, err);
}

void launch_xgmi_bucket(const XgmiBuffers& B, int world, int rank, int bucket, int64_t lo, int64_t count,
                        unsigned epoch, bool average, uint64_t timeout_ticks, unsigned* err, hipStream_t st,
                        int phase_lo, int phase_hi, int max_blocks) {
  const XgmiPtrs P = make_ptrs(B, world);
  const bool bf16 = B.g16[0] != nullptr;
  const int64_t hi = lo + count;
  const int64_t shard = xgmi_shard(lo, count, world);
  const int64_t base = lo / 8 * 8;
  const int64_t own_lo = std::max(lo, std::min(hi, base + rank * shard));
  const int64_t own_hi = std::min(hi, base + (rank + 1) * shard);
  const int slot_ready = bucket * kXgmiSlotsPerBucket;
  const int nch = xgmi_chunks(shard, world);
  const int64_t cs = ((shard + nch - 1) / nch + 7) / 8 * 8;  // chunk of a shard, 32-B aligned
  auto slot_red = [&](int c) { return slot_ready + 1 + c; };
  const int cap = std::max(1, max_blocks);
  auto blocks = [&](int64_t units) {
    const int64_t b = (units + 255) / 256;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, cap));
  };
  auto on = [&](int ph) { return ph >= phase_lo && ph <= phase_hi; };
  // phase 0: (bf16 wire: pack) + signal ready, 1: wait ready, 2: reduce-scatter, 3: signal
  // reduced, 4: wait reduced, 5: all-gather.  Chunked buckets run phase 2 as (reduce-scatter,
  // signal) per chunk and phase 4 as (wait, all-gather) per chunk; phases 3 and 5 are then empty.
  // In-process rank groups enqueue phase-major so that no rank's wait can sit in a hardware queue
  // ahead of another rank's signal.
  if (on(0)) {
    if (bf16)
      hipLaunchKernelGGL(xgmi_pack_bf16_kernel, dim3(blocks(count / 8 + 1)), dim3(256), 0, st, P, rank, lo, hi);
    hipLaunchKernelGGL(xgmi_signal_kernel, dim3(1), dim3(64), 0, st, P, world, rank, slot_ready, epoch, err);
  }
  if (on(1))
    hipLaunchKernelGGL(xgmi_wait_kernel, dim3(1), dim3(64), 0, st, P.flags[rank], world, slot_ready, epoch,
                       (unsigned long long)timeout_ticks, err, 1u + 2u * (unsigned)bucket);
  // world 1, fp32 wire: the reduced bucket IS the gradient (sum of one rank, divided by 1) --
  // only the flag protocol runs (RCCL's world-1 all-reduce is likewise no data movement)
  const bool data = world > 1 || bf16;
  const int64_t s_own = base + rank * shard;
  auto rs = [&](int64_t a, int64_t b) {
    if (!data || b <= a) return;
    const unsigned grid = blocks((b - a) / (bf16 ? 8 : 4 * kXgmiUnroll) + 1);
    switch (world) {
      case 1: launch_rs<1>(P, bf16, world, rank, a, b, grid, err, st); break;
      case 2: launch_rs<2>(P, bf16, world, rank, a, b, grid, err, st); break;
      case 4: launch_rs<4>(P, bf16, world, rank, a, b, grid, err, st); break;
      case 8: launch_rs<8>(P, bf16, world, rank, a, b, grid, err, st); break;
      default: launch_rs<0>(P, bf16, world, rank, a, b, grid, err, st); break;
    }
  };
  auto ag = [&](int64_t sub_off, int64_t sub_len) {
    if (!data) return;
    const unsigned grid = blocks(sub_len / (bf16 ? 8 : 4 * kXgmiUnroll) + 1);
    if (bf16)
      hipLaunchKernelGGL(xgmi_all_gather_kernel<true>, dim3(grid), dim3(256), 0, st, P, world, rank, lo, hi, shard,
                         sub_off, sub_len, average ? 1 : 0, err);
    else
      hipLaunchKernelGGL(xgmi_all_gather_kernel<false>, dim3(grid), dim3(256), 0, st, P, world, rank, lo, hi, shard,
                         sub_off, sub_len, average ? 1 : 0, err);
  };
  auto wait_red = [&](int c) {
    hipLaunchKernelGGL(xgmi_wait_kernel, dim3(1), dim3(64), 0, st, P.flags[rank], world, slot_red(c), epoch,
                       (unsigned long long)timeout_ticks, err, 2u + 2u * (unsigned)bucket);
  };
  auto signal_red = [&](int c) {
    hipLaunchKernelGGL(xgmi_signal_kernel, dim3(1), dim3(64), 0, st, P, world, rank, slot_red(c), epoch, err);
  };
  if (nch == 1) {
    if (on(2)) rs(own_lo, own_hi);
    if (on(3)) signal_red(0);
    if (on(4)) wait_red(0);
    if (on(5)) ag(0, shard);
  } else {
    if (on(2))
      for (int c = 0; c < nch; ++c) {
        rs(std::max(lo, std::min(hi, s_own + c * cs)), std::min(hi, std::min(s_own + shard, s_own + (c + 1) * cs)));
        signal_red(c);
      }
    if (on(4))
      for (int c = 0; c < nch; ++c) {
        wait_red(c);
        ag(c * cs, cs);
      }
  }
  check("xgmi bucket");
}

}  // namespace pdt
