// Fused SGD + momentum + weight decay over ONE flat fp32 parameter buffer.
//
// torch.optim.SGD (foreach) issues ~4 multi-tensor kernels per step over 161
// (ResNet-50) tensors (torch/optim/sgd.py:425-470); here the DDP wrapper homes
// every parameter, gradient and momentum buffer in flat storage with identical
// ordering, so the whole update is a single streaming pass: 3 reads + 2 writes
// per element, 16 B per lane.  Semantics (torch/optim/sgd.py:343-380):
//   d = g*scale + wd*p ; buf = first ? d : m*buf + (1-damp)*d ;
//   d = nesterov ? d + m*buf : buf ; p -= lr*d
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <stdexcept>

namespace pdt {

// MIRROR: also write bf16(p') to pb -- the KRSC bf16 weights the next forward's convs consume
// (conv weights are channels_last, so the flat fp32 order already is KRSC), saving a pack pass.
// `lead` elements before the first 16-B-aligned one (a bucket slice of the flat buffers can start
// anywhere) and the tail are updated one at a time; the body in float4.  p, g, buf and pb share one
// element offset from 16-B-aligned bases, so one lead aligns all four.
template <bool MOM, bool NEST, bool MIRROR>
__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ buf, int64_t n, float lr,
                                                  float mom, float damp1, float wd, bool first,
                                                  float scale, uint16_t* __restrict__ pb, int lead) {
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  auto step = [&](float& pp, float gg, float& bb) {
    float d = fmaf(wd, pp, gg * scale);
    if (MOM) {
      bb = first ? d : fmaf(mom, bb, damp1 * d);
      d = NEST ? fmaf(mom, bb, d) : bb;
    }
    pp = fmaf(-lr, d, pp);
  };
  auto one = [&](int64_t i) {
    float pv = p[i], bv = MOM ? buf[i] : 0.f;
    step(pv, g[i], bv);
    p[i] = pv;
    if (MOM) buf[i] = bv;
    if (MIRROR) pb[i] = f2bf(pv);
  };
  if (tid < lead) one(tid);
  const int64_t n4 = (n - lead) / 4;
  float4* p4 = reinterpret_cast<float4*>(p + lead);
  const float4* g4 = reinterpret_cast<const float4*>(g + lead);
  float4* b4 = reinterpret_cast<float4*>(buf + lead);
  uint2* pb4 = reinterpret_cast<uint2*>(pb + lead);
  for (int64_t i = tid; i < n4; i += stride) {
    float4 pv = p4[i];
    float4 gv = g4[i];
    float4 bv = MOM ? b4[i] : make_float4(0, 0, 0, 0);
    step(pv.x, gv.x, bv.x); step(pv.y, gv.y, bv.y); step(pv.z, gv.z, bv.z); step(pv.w, gv.w, bv.w);
    p4[i] = pv;
    if (MOM) b4[i] = bv;
    if (MIRROR) pb4[i] = make_uint2(pack2bf(pv.x, pv.y), pack2bf(pv.z, pv.w));
  }
  for (int64_t i = lead + n4 * 4 + tid; i < n; i += stride) one(i);
}

template <bool MIRROR>
static void launch_sgd_t(float* p, const float* g, float* buf, int64_t n, float lr, float momentum,
                         float dampening, float wd, bool nesterov, bool first, float grad_scale,
                         hipStream_t st, uint16_t* pb) {
  if (n <= 0) return;
  const int lead = (int)std::min<int64_t>(n, (int64_t)(((16 - ((uintptr_t)p & 15)) & 15) >> 2));
  if (((uintptr_t)g & 15) != ((uintptr_t)p & 15) || (buf && ((uintptr_t)buf & 15) != ((uintptr_t)p & 15)) ||
      (pb && ((uintptr_t)(pb + lead) & 7) != 0) || ((uintptr_t)p & 3))
    throw std::runtime_error("sgd: flat buffers must share their 16-byte alignment");
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  dim3 gr((unsigned)blocks), bl(256);
  float damp1 = 1.f - dampening;
  if (momentum == 0.f)
    hipLaunchKernelGGL((sgd_kernel<false, false, MIRROR>), gr, bl, 0, st, p, g, buf, n, lr, momentum, damp1, wd, first, grad_scale, pb, lead);
  else if (nesterov)
    hipLaunchKernelGGL((sgd_kernel<true, true, MIRROR>), gr, bl, 0, st, p, g, buf, n, lr, momentum, damp1, wd, first, grad_scale, pb, lead);
  else
    hipLaunchKernelGGL((sgd_kernel<true, false, MIRROR>), gr, bl, 0, st, p, g, buf, n, lr, momentum, damp1, wd, first, grad_scale, pb, lead);
}

void launch_sgd(float* p, const float* g, float* buf, int64_t n, float lr, float momentum,
                float dampening, float wd, bool nesterov, bool first, float grad_scale,
                hipStream_t st, uint16_t* p_bf16) {
  if (p_bf16) launch_sgd_t<true>(p, g, buf, n, lr, momentum, dampening, wd, nesterov, first, grad_scale, st, p_bf16);
  else launch_sgd_t<false>(p, g, buf, n, lr, momentum, dampening, wd, nesterov, first, grad_scale, st, nullptr);
}

__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(const float* __restrict__ x,
                                                            uint16_t* __restrict__ y, int64_t n) {
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = f2bf(x[i]);
}

__global__ void __launch_bounds__(256) cast_bf16_f32_kernel(const uint16_t* __restrict__ x,
                                                            float* __restrict__ y, int64_t n,
                                                            float scale) {
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = bf2f(x[i]) * scale;
}

void launch_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st) {
  int64_t b = (n + 255) / 256;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3((unsigned)(b < 4096 ? (b ? b : 1) : 4096)), dim3(256), 0, st, x, y, n);
}

void launch_cast_bf16_f32(const uint16_t* x, float* y, int64_t n, float scale, hipStream_t st) {
  int64_t b = (n + 255) / 256;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3((unsigned)(b < 4096 ? (b ? b : 1) : 4096)), dim3(256), 0, st, x, y, n, scale);
}

}  // namespace pdt
