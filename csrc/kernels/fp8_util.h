// Device helpers shared by the fp8 kernels (fp8.hip) and the fp8-emitting BatchNorm passes
// (bn_act.hip): saturating OCP e4m3 / e5m2 conversion and the delayed-scaling protocol.
#pragma once
#include "common.h"

namespace pdt {

// ------------------------------------------------------------------ conversion
constexpr float E4M3_MAX = 448.f;
constexpr float E5M2_MAX = 57344.f;

// two floats -> two e4m3 bytes (low 16 bits), saturating (the hardware convert does not clamp)
__device__ __forceinline__ uint32_t cvt2_e4m3(float a, float b) {
  a = fminf(fmaxf(a, -E4M3_MAX), E4M3_MAX);
  b = fminf(fmaxf(b, -E4M3_MAX), E4M3_MAX);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false) & 0xffffu;
}
__device__ __forceinline__ uint32_t cvt4_e4m3(float a, float b, float c, float d) {
  return cvt2_e4m3(a, b) | (cvt2_e4m3(c, d) << 16);
}

// Delayed per-tensor scaling.  State (fp8_state_floats() floats): for each of the last three calls
// an amax sharded over AMAX_SHARDS 128-byte lines, then the three calls' dequantization factors.
// Call t quantizes with s_t = 2^floor(log2(E4M3_HEADROOM / amax_{t-1})) (1 before any history),
// publishes deq[t%3] = 1/s_t for its consumers, accumulates amax_t into slot t%3 and clears slot
// (t+1)%3 for the next call -- no host sync, no extra launch.  The shards keep the per-block
// atomics off a single address (one device-scope atomic per ~12 ns on a shared word:
// MI355X_MICROARCH.md fan-in row).
constexpr float E4M3_HEADROOM = 224.f;    // one binade of margin below 448 for growth between steps
constexpr float E5M2_HEADROOM = 28672.f;  // the same for e5m2 (gradients)
constexpr int AMAX_SHARDS = 64;
constexpr int SHARD_STRIDE = 32;        // floats: one 128-B line per shard
constexpr int SLOT_FLOATS = AMAX_SHARDS * SHARD_STRIDE;
constexpr int DEQ_OFFSET = 3 * SLOT_FLOATS;

// every thread of the block gets s_t (wave 0 reduces the previous call's shards)
template <bool E5M2 = false>
__device__ __forceinline__ float delayed_scale(const float* state, int slot) {
  __shared__ float s_prev;
  if (threadIdx.x < 64) {
    float v = state[((slot + 2) % 3) * SLOT_FLOATS + threadIdx.x * SHARD_STRIDE];
    v = wave_max(v);
    if (threadIdx.x == 0) s_prev = v;
  }
  __syncthreads();
  const float prev = s_prev;
  if (!(prev > 0.f)) return 1.f;
  const float s = exp2f(floorf(log2f((E5M2 ? E5M2_HEADROOM : E4M3_HEADROOM) / prev)));
  return fminf(fmaxf(s, 0x1p-32f), 0x1p32f);  // wide: gradients can be tiny
}

__device__ __forceinline__ void publish_scale(float* state, int slot, float s) {
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    if (threadIdx.x == 0) state[DEQ_OFFSET + slot] = 1.f / s;
    state[((slot + 1) % 3) * SLOT_FLOATS + threadIdx.x * SHARD_STRIDE] = 0.f;
  }
}

// block max of a non-negative value, one atomic per block into its shard (float bits order as
// uint for x >= 0)
__device__ __forceinline__ void block_amax(float v, float* slot_base) {
  __shared__ float sm[16];
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sm[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = sm[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, sm[i]);
    atomicMax(reinterpret_cast<unsigned int*>(slot_base + (blockIdx.x % AMAX_SHARDS) * SHARD_STRIDE),
              __float_as_uint(m));
  }
}

// two floats -> two e5m2 bytes (low 16 bits), saturating
__device__ __forceinline__ uint32_t cvt2_e5m2(float a, float b) {
  a = fminf(fmaxf(a, -E5M2_MAX), E5M2_MAX);
  b = fminf(fmaxf(b, -E5M2_MAX), E5M2_MAX);
  return (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false) & 0xffffu;
}
__device__ __forceinline__ uint32_t cvt4_e5m2(float a, float b, float c, float d) {
  return cvt2_e5m2(a, b) | (cvt2_e5m2(c, d) << 16);
}

}  // namespace pdt

