// Shared device helpers of the implicit-GEMM kernels (conv_igemm.hip: forward / input gradient,
// wgrad.hip: weight gradient): fast division, XCD-aware block remap, LDS-DMA staging and counted
// waits, the MFMA wrapper and the transposing-read LDS images.
#pragma once
#include "common.h"

namespace pdt {

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- utilities
struct FastDiv {  // n / d for 0 <= n < 2^31 via mul-hi
  uint32_t mul, shr;
};
static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.shr = l;
  f.mul = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t hi = __umulhi(n, f.mul);
  return (hi + n) >> f.shr;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: blocks b, b+8, b+16, ... (one XCD under round-robin dispatch) get consecutive ids
  int q = nwg / 8, r = nwg % 8;
  int xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

__device__ __forceinline__ v4i buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ v4f mfma16(const v4i& a, const v4i& b, const v4f& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a),
                                                __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}

constexpr uint32_t OOB = 0x80000000u;  // any offset >= num_records reads 0

// 16-byte LDS-DMA: every lane fetches 16 B at its own buffer offset (out-of-range -> 0) and the
// wave's 64 results land contiguously at `lds` (wave-uniform base, lane-linear image).
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)(reinterpret_cast<uintptr_t>(lds)), 16, voff, 0, 0, 0);
}

// The LDS-DMA as inline asm, for kernels that read their tiles with ds_read_b64_tr_b16: hipcc
// puts an `s_waitcnt vmcnt(0)` in front of every LDS read it cannot prove disjoint from a pending
// LDS-DMA it knows about, which drains a multi-stage ring at every fragment read.  Issued through
// asm, the DMA is invisible to that analysis; the kernel orders it with its own counted vmcnt +
// barrier (a compiler-placed vmcnt for its own loads only ever waits for more, never less).  `r`
// is the buffer descriptor (rsrc_words), `lds` the wave-uniform LDS byte address of the 1-KiB
// destination.
__device__ __forceinline__ v4i rsrc_words(const void* p, uint32_t num_bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  return v4i{(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xffffu), (int)num_bytes, 0x00020000};
}
__device__ __forceinline__ void glds16_asm(const v4i& r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %1\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
               :: "v"(voff), "s"(__builtin_amdgcn_readfirstlane(lds)), "s"(r) : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>(p);
}

// Wait until at most N of this wave's vector-memory ops (LDS-DMA included) are outstanding.
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Workgroup barrier WITHOUT the memory-model fence of __syncthreads(): that fence makes the compiler
// emit s_waitcnt vmcnt(0) before s_barrier, draining every in-flight LDS-DMA and defeating a
// multi-stage pipeline.  Callers order memory themselves: their own counted vmcnt wait covers the
// DMA into the buffer about to be read, and every ds_read of the buffer about to be refilled has
// been consumed (lgkmcnt 0) by the MFMAs before the barrier.  The "memory" clobber keeps the
// compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_barrier" ::: "memory"); }

// Multi-stage pipelines: every K-step issues LPS DMA ops per wave; wait until the oldest pending
// step has landed while `younger` later steps (wave-uniform, < 5) may stay in flight.
template <int LPS>
__device__ __forceinline__ void wait_steps(int younger) {
  if (younger >= 4) wait_vm<4 * LPS>();
  else if (younger == 3) wait_vm<3 * LPS>();
  else if (younger == 2) wait_vm<2 * LPS>();
  else if (younger == 1) wait_vm<LPS>();
  else wait_vm<0>();
}

// TM 8, TN 4).  C64 (per-tap 64-channel K-steps) loader only.
// barrier that also retires this wave's own LDS reads first: the quarter refilled right after it
// must not have a fragment read of any wave still in flight (the MFMAs that consume the reads
// are not memory operations, so the compiler may place them -- and their lgkmcnt wait -- after
// an asm barrier)
__device__ __forceinline__ void lds_barrier_rd() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS image of a [64 m][128 col] bf16 tile: 256-B rows, 16-B chunks XOR-swizzled by
// swz(m)<<1 with swz(m) = (m&3) | ((m>>3)&1)<<2.  The transposing fragment read
// (ds_read_b64_tr_b16: per 32-lane half, rows {m..m+3, m+8..m+11} x 32 B) then hits
// 8 distinct 32-B bank windows: conflict-free; ds_write_b128 groups stay in one half-row.
__device__ __forceinline__ int swz256(int row, int chunk) {
  int sw = (row & 3) | (((row >> 3) & 1) << 2);
  return row * 256 + ((chunk ^ (sw << 1)) << 4);
}

typedef short v4s_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4s_t ds_read_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s_t*)(reinterpret_cast<uintptr_t>(p)));
}

// The same read as inline asm.  hipcc places an `s_waitcnt vmcnt(0)` in front of every
// ds_read_tr builtin that follows an LDS-DMA (it cannot tell the DMA's destination from the
// read's source), which drains every prefetched K-step at each fragment read and turns a
// multi-stage LDS-DMA ring into a synchronous load.  The asm form is invisible to that pass:
// the caller orders it against the DMA with its own counted vmcnt + barrier, and against its
// consumers with lds_wait_frags() (the compiler does not know the result is asynchronous).
template <int OFF = 0>
__device__ __forceinline__ v4s_t ds_read_tr_asm(const char* p) {
  v4s_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"((uint32_t)reinterpret_cast<uintptr_t>(p)), "n"(OFF));
  return r;
}

__device__ __forceinline__ v4i cat_frag(v4s_t lo, v4s_t hi) {
  return __builtin_bit_cast(v4i, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// 128-B-row variant for the [64 m][64 kout] A tile of a BMG = 64 wgrad: swizzle
// sw(m) = ((m>>1)&1) | ((m>>3)&1)<<1 applied as chunk ^ (sw<<1) keeps each tr-read chunk pair
// together; a half-wave's rows {m..m+3, m+8..m+11} land in 8 distinct 32-B bank windows
// ((m&1)*4 + (pair ^ sw)), so the 128-B image is conflict-free too and the tile DMA moves only
// the bytes the MFMAs consume (the 256-B image fetched a never-read upper half).
__device__ __forceinline__ int swz128_tr(int row, int chunk) {
  int sw = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return row * 128 + ((chunk ^ (sw << 1)) << 4);
}

// 512-B rows (the [64 m][256 kout] dy tile of a BMG = 256 wgrad): the swz256 XOR on chunk bits
// 1..3 -- LDS banks repeat every 256 B, so a half-wave's rows {m..m+3, m+8..m+11} still land in 8
// distinct 32-B bank windows.
__device__ __forceinline__ int swz512(int row, int chunk) {
  int sw = (row & 3) | (((row >> 3) & 1) << 2);
  return row * 512 + ((chunk ^ (sw << 1)) << 4);
}

template <int ROWB>
__device__ __forceinline__ int swz_img(int row, int chunk) {
  if constexpr (ROWB == 512) return swz512(row, chunk);
  else if constexpr (ROWB == 256) return swz256(row, chunk);
  else return swz128_tr(row, chunk);
}

}  // namespace pdt
