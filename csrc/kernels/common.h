// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC bf16 (stored as raw uint16 bits), channel count a
//     multiple of 8 so one 16-byte vector = 8 channels;
//   * wave = 64 lanes (never 32); block sizes are multiples of 64;
//   * memory-bound kernels move 16 B per lane per access (Guideline 13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

typedef uint16_t bf16;
typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

// Hardware round-to-nearest-even conversion (v_cvt_pk_bf16_f32 at -O3; NaN stays NaN).
__device__ __forceinline__ bf16 f2bf(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

// Two floats -> two RNE bf16 in one dword: ONE v_cvt_pk_bf16_f32 (the scalar-conversion form
// above, or-ed together, compiles to two conversions + shift + or where the pair is not
// recognised -- 4 VALU per pair in the conv epilogues).
typedef float pdt_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 pdt_bf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(pdt_f2{lo, hi}, pdt_bf2));
}

// 16-byte vector of 8 bf16 <-> 8 floats
struct f8 { float v[8]; };

__device__ __forceinline__ f8 unpack8(const uint4 u) {
  f8 r;
  r.v[0] = __uint_as_float(u.x << 16); r.v[1] = __uint_as_float(u.x & 0xffff0000u);
  r.v[2] = __uint_as_float(u.y << 16); r.v[3] = __uint_as_float(u.y & 0xffff0000u);
  r.v[4] = __uint_as_float(u.z << 16); r.v[5] = __uint_as_float(u.z & 0xffff0000u);
  r.v[6] = __uint_as_float(u.w << 16); r.v[7] = __uint_as_float(u.w & 0xffff0000u);
  return r;
}

__device__ __forceinline__ uint4 pack8(const f8& a) {
  uint4 u;
  u.x = pack2bf(a.v[0], a.v[1]); u.y = pack2bf(a.v[2], a.v[3]);
  u.z = pack2bf(a.v[4], a.v[5]); u.w = pack2bf(a.v[6], a.v[7]);
  return u;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over the 16 lanes of a DPP row (lanes 16r..16r+15), result in every lane of the row.
// Four v_add_f32 with DPP modifiers (quad_perm xor1, xor2, row_ror 4, row_ror 8): no LDS traffic,
// unlike __shfl_xor which lowers to ds_swizzle / ds_bpermute.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x128>(v);  // row_ror:8
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Chan et al. parallel variance merge of (count, mean, M2) triples.
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2,
                                           float nb, float meanb, float m2b) {
  if (nb <= 0.f) return;
  float nn = n + nb;
  float d = meanb - mean;
  float f = nb / nn;
  mean += d * f;
  m2 += m2b + d * d * n * f;
  n = nn;
}

// Buffer resource for bounds-checked loads: offsets >= num_bytes read 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t num_bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)num_bytes, 0x00020000);
}

__host__ __device__ __forceinline__ int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace pdt
