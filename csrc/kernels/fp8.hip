// FP8 (OCP e4m3 / e5m2) support for the MX-rate MFMA path on gfx950.
//
// v_mfma_scale_f32_16x16x128_f8f6f4 is the only fp8 MFMA at twice the bf16 rate (the unscaled
// 16x16x32 fp8 form runs at the bf16 rate, MI355X_MICROARCH.md "Matrix cores").  Its operands are
// 32 fp8 values per lane; scales are E8M0 (power-of-two, bias 127) per 32-k block.  The conv
// kernels use unit block scales and carry the real per-tensor / per-channel scales in fp32
// (folded into the epilogue), so the only thing the hardware block scale must be is 1.0.
//
// This file: a register-level probe of that MFMA (operand lane map and scale semantics are
// verified by tests/test_fp8_gpu.py against exact integer data), fp8 weight packing with
// per-output-channel scales, and delayed-scaling activation quantization.
#include "common.h"
#include "fp8_util.h"
#include "kernels.h"

#include <stdexcept>

namespace pdt {

int fp8_state_floats() { return DEQ_OFFSET + 4; }
int fp8_deq_offset() { return DEQ_OFFSET; }

typedef int v8i_t __attribute__((ext_vector_type(8)));

template <int FA, int FB>
__global__ void mfma_f8_probe_kernel(const v8i_t* __restrict__ a, const v8i_t* __restrict__ b,
                                     float4* __restrict__ d, int scale_a, int scale_b, int use_scale) {
  const int l = threadIdx.x;
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  if (use_scale)
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, FA, FB, 0, scale_a, 0, scale_b);
  else
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, FA, FB, 0, 0, 0, 0);
  d[l] = make_float4(acc[0], acc[1], acc[2], acc[3]);
}

void launch_mfma_f8_probe(const void* a_regs, const void* b_regs, float* d, int fmt_a, int fmt_b,
                          int scale_a, int scale_b, int use_scale, hipStream_t st) {
  auto A = reinterpret_cast<const v8i_t*>(a_regs);
  auto B = reinterpret_cast<const v8i_t*>(b_regs);
  auto D = reinterpret_cast<float4*>(d);
  if (fmt_a == 0 && fmt_b == 0)
    hipLaunchKernelGGL((mfma_f8_probe_kernel<0, 0>), dim3(1), dim3(64), 0, st, A, B, D, scale_a, scale_b, use_scale);
  else if (fmt_a == 1 && fmt_b == 0)
    hipLaunchKernelGGL((mfma_f8_probe_kernel<1, 0>), dim3(1), dim3(64), 0, st, A, B, D, scale_a, scale_b, use_scale);
  else if (fmt_a == 0 && fmt_b == 1)
    hipLaunchKernelGGL((mfma_f8_probe_kernel<0, 1>), dim3(1), dim3(64), 0, st, A, B, D, scale_a, scale_b, use_scale);
  else
    hipLaunchKernelGGL((mfma_f8_probe_kernel<1, 1>), dim3(1), dim3(64), 0, st, A, B, D, scale_a, scale_b, use_scale);
}

// ------------------------------------------------------------------ weights
// One block per output channel k: amax over its R*S*C weights, wq[k][r][s][c] = e4m3(w / ws_k)
// (zero for c >= C), oscale[k] = ws_k * act_deq with ws_k = amax_k / 448.
__global__ void __launch_bounds__(256) pack_weight_fp8_kernel(const float* __restrict__ w, WStridesF8 st,
                                                              uint8_t* __restrict__ wq,
                                                              float* __restrict__ oscale,
                                                              const float* __restrict__ act_deq,
                                                              int C, int R, int S, int Cp) {
  const int k = blockIdx.x;
  const int n = R * S * Cp;
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int c = i % Cp, rs = i / Cp;
    const int r = rs / S, s_ = rs - r * S;
    if (c < C) m = fmaxf(m, fabsf(w[k * st.k + c * st.c + r * st.r + s_ * st.s]));
  }
  __shared__ float sm[4];
  __shared__ float s_scale;
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float amax = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    const float ws = amax > 0.f ? amax / E4M3_MAX : 1.f;
    s_scale = ws;
    oscale[k] = ws * (act_deq != nullptr ? act_deq[0] : 1.f);
  }
  __syncthreads();
  const float inv = 1.f / s_scale;
  // 4 consecutive elements per thread -> one 32-bit store
  for (int i = threadIdx.x * 4; i < n; i += blockDim.x * 4) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ii = i + e;
      const int c = ii % Cp, rs = ii / Cp;
      const int r = rs / S, s_ = rs - r * S;
      v[e] = (ii < n && c < C) ? w[k * st.k + c * st.c + r * st.r + s_ * st.s] * inv : 0.f;
    }
    *reinterpret_cast<uint32_t*>(wq + (int64_t)k * n + i) = cvt4_e4m3(v[0], v[1], v[2], v[3]);
  }
}

void launch_pack_weight_fp8(const float* w, const int64_t* strides, uint8_t* wq, float* oscale,
                            const float* act_deq, int K, int C, int R, int S, int Cp, hipStream_t st) {
  if ((R * S * Cp) % 4 != 0) throw std::runtime_error("pack_weight_fp8: R*S*Cp must be a multiple of 4");
  WStridesF8 ws{strides[0], strides[1], strides[2], strides[3]};
  hipLaunchKernelGGL(pack_weight_fp8_kernel, dim3(K), dim3(256), 0, st, w, ws, wq, oscale, act_deq, C, R,
                     S, Cp);
}

// Row-wise e4m3 quantization of bf16 weight images living in one flat mirror (KRSC rows = one
// output channel each for the forward, CRSK rows = one input channel for dgrad): one wave per
// row, scale[row] = amax(row)/448, q = e4m3(w / scale).  One launch for every conv of the model.
struct QRowEntry { int64_t off, soff; int rows, rowlen; };

__global__ void __launch_bounds__(256) quant_rows_e4m3_kernel(const uint16_t* __restrict__ src,
                                                              uint8_t* __restrict__ dst,
                                                              float* __restrict__ scale,
                                                              const QRowEntry* __restrict__ tab) {
  const QRowEntry e = tab[blockIdx.y];
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= e.rows) return;
  const int lane = threadIdx.x & 63;
  const uint4* r = reinterpret_cast<const uint4*>(src + e.off + (int64_t)row * e.rowlen);
  const int nv = e.rowlen / 8;
  float m = 0.f;
  for (int v = lane; v < nv; v += 64) {
    const f8 a = unpack8(r[v]);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(a.v[j]));
  }
  m = wave_max(m);
  const float sc = m > 0.f ? m / E4M3_MAX : 1.f;
  if (lane == 0) scale[e.soff + row] = sc;
  const float inv = 1.f / sc;
  uint2* o = reinterpret_cast<uint2*>(dst + e.off + (int64_t)row * e.rowlen);
  for (int v = lane; v < nv; v += 64) {
    const f8 a = unpack8(r[v]);
    o[v] = make_uint2(cvt4_e4m3(a.v[0] * inv, a.v[1] * inv, a.v[2] * inv, a.v[3] * inv),
                      cvt4_e4m3(a.v[4] * inv, a.v[5] * inv, a.v[6] * inv, a.v[7] * inv));
  }
}

void launch_quant_rows_e4m3(const uint16_t* src, uint8_t* dst, float* scale, const void* table,
                            int ntensors, int max_rows, hipStream_t st) {
  if (ntensors <= 0) return;
  hipLaunchKernelGGL(quant_rows_e4m3_kernel, dim3((max_rows + 3) / 4, ntensors), dim3(256), 0, st, src, dst,
                     scale, reinterpret_cast<const QRowEntry*>(table));
}

size_t quant_rows_entry_bytes() { return sizeof(QRowEntry); }

// ------------------------------------------------------------------ activations
// bf16 -> e4m3 with delayed scaling (8 elements = one 16-B load, one 8-B store per thread-step)
__global__ void __launch_bounds__(256) quant_e4m3_kernel(const uint4* __restrict__ x, uint2* __restrict__ q,
                                                         int64_t nvec, float* __restrict__ state, int slot) {
  const float s = delayed_scale(state, slot);
  publish_scale(state, slot, s);
  float m = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const f8 a = unpack8(x[v]);
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m = fmaxf(m, fabsf(a.v[j]));
      t[j] = a.v[j] * s;
    }
    q[v] = make_uint2(cvt4_e4m3(t[0], t[1], t[2], t[3]), cvt4_e4m3(t[4], t[5], t[6], t[7]));
  }
  block_amax(m, state + slot * SLOT_FLOATS);
}

static int q_blocks(int64_t nvec) {
  const int64_t b = (nvec + 255) / 256;
  return (int)(b < 4096 ? b : 4096);
}

void launch_quant_e4m3(const uint16_t* x, uint8_t* q, int64_t n, float* state, int slot, hipStream_t st) {
  if (n % 8 != 0) throw std::runtime_error("quant_e4m3: size must be a multiple of 8");
  const int64_t nvec = n / 8;
  hipLaunchKernelGGL(quant_e4m3_kernel, dim3(q_blocks(nvec)), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(x), reinterpret_cast<uint2*>(q), nvec, state, slot);
}

// BatchNorm apply (+residual)(+ReLU) that also emits the e4m3 copy the next conv reads:
// z = act(y*scale + shift (+res)) in bf16 (kept for the weight gradient, the residual path and
// backward masks) and q = e4m3(bf16(z) * s_t)
template <bool RES, bool RELU>
__global__ void __launch_bounds__(256) bn_act_fwd_q8_kernel(const uint4* __restrict__ y,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const uint4* __restrict__ res,
                                                            uint4* __restrict__ z, uint2* __restrict__ q,
                                                            int64_t nvec, int K8, float* __restrict__ state,
                                                            int slot, uint8_t* __restrict__ zmask) {
  const float s = delayed_scale(state, slot);
  publish_scale(state, slot, s);
  float m = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int c0 = (int)(v % K8) * 8;
    f8 a = unpack8(y[v]);
    const float4 s0 = *reinterpret_cast<const float4*>(scale + c0);
    const float4 s1 = *reinterpret_cast<const float4*>(scale + c0 + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(shift + c0);
    const float4 h1 = *reinterpret_cast<const float4*>(shift + c0 + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    f8 r;
    if (RES) r = unpack8(res[v]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = fmaf(a.v[j], sc[j], sh[j]);
      if (RES) t += r.v[j];
      if (RELU) t = fmaxf(t, 0.f);
      a.v[j] = t;
    }
    const uint4 zb = pack8(a);
    if (z != nullptr) z[v] = zb;  // fp8-only storage: no bf16 consumer (uniform branch)
    const f8 zr = unpack8(zb);  // quantize exactly the bf16 value the bf16 consumers see
    float t[8];
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m = fmaxf(m, fabsf(zr.v[j]));
      t[j] = zr.v[j] * s;
      bits |= (zr.v[j] > 0.f ? 1u : 0u) << j;
    }
    if (zmask != nullptr) zmask[v] = (uint8_t)bits;
    q[v] = make_uint2(cvt4_e4m3(t[0], t[1], t[2], t[3]), cvt4_e4m3(t[4], t[5], t[6], t[7]));
  }
  block_amax(m, state + slot * SLOT_FLOATS);
}

void launch_bn_act_fwd_q8(const uint16_t* y, const float* scale, const float* shift, const uint16_t* res,
                          bool relu, uint16_t* z, uint8_t* q, int64_t M, int K, float* state, int slot,
                          hipStream_t st, uint8_t* zmask) {
  const int64_t nvec = M * K / 8;
  const int K8 = K / 8;
  dim3 g(q_blocks(nvec)), b(256);
  auto Y = reinterpret_cast<const uint4*>(y);
  auto R = reinterpret_cast<const uint4*>(res);
  auto Z = reinterpret_cast<uint4*>(z);
  auto Q = reinterpret_cast<uint2*>(q);
  if (res) {
    if (relu) hipLaunchKernelGGL((bn_act_fwd_q8_kernel<true, true>), g, b, 0, st, Y, scale, shift, R, Z, Q, nvec, K8, state, slot, zmask);
    else hipLaunchKernelGGL((bn_act_fwd_q8_kernel<true, false>), g, b, 0, st, Y, scale, shift, R, Z, Q, nvec, K8, state, slot, zmask);
  } else {
    if (relu) hipLaunchKernelGGL((bn_act_fwd_q8_kernel<false, true>), g, b, 0, st, Y, scale, shift, R, Z, Q, nvec, K8, state, slot, zmask);
    else hipLaunchKernelGGL((bn_act_fwd_q8_kernel<false, false>), g, b, 0, st, Y, scale, shift, R, Z, Q, nvec, K8, state, slot, zmask);
  }
}

}  // namespace pdt
