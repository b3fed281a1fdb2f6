// Layout kernels: image NCHW fp32 -> NHWC bf16, and conv-weight packing into the
// implicit-GEMM B layouts (KRSC for fwd, CRSK for dgrad).  All tiny next to the
// convolutions; written for coalesced 16-byte stores.
#include "common.h"
#include "kernels.h"

namespace pdt {

// one thread per output pixel: reads C strided fp32 (coalesced across w), writes Cp bf16
__global__ void __launch_bounds__(256) image_to_nhwc_kernel(const float* __restrict__ x,
                                                            uint16_t* __restrict__ y, int N,
                                                            int C, int HW, int Cp) {
  int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)N * HW;
  if (pix >= total) return;
  int n = (int)(pix / HW);
  int hw = (int)(pix - (int64_t)n * HW);
  const float* src = x + (int64_t)n * C * HW + hw;
  uint4* dst = reinterpret_cast<uint4*>(y + pix * Cp);
  for (int c0 = 0; c0 < Cp; c0 += 8) {
    f8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int c = c0 + j;
      v.v[j] = c < C ? src[(int64_t)c * HW] : 0.f;
    }
    dst[c0 / 8] = pack8(v);
  }
}

void launch_image_to_nhwc(const float* x, uint16_t* y, int N, int C, int H, int W, int Cp,
                          hipStream_t st) {
  int64_t total = (int64_t)N * H * W;
  int blocks = (int)((total + 255) / 256);
  hipLaunchKernelGGL(image_to_nhwc_kernel, dim3(blocks), dim3(256), 0, st, x, y, N, C, H * W, Cp);
}

struct WStrides { int64_t k, c, r, s; };

// out[k][r][s][c] (c < Cp)
__global__ void __launch_bounds__(256) pack_weight_kernel(const float* __restrict__ w, WStrides ws,
                                                          uint16_t* __restrict__ out, int K, int C,
                                                          int R, int S, int Cp) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)K * R * S * Cp;
  if (i >= total) return;
  int c = (int)(i % Cp);
  int64_t t = i / Cp;
  int s = (int)(t % S); t /= S;
  int r = (int)(t % R);
  int k = (int)(t / R);
  float v = c < C ? w[k * ws.k + c * ws.c + r * ws.r + s * ws.s] : 0.f;
  out[i] = f2bf(v);
}

// out[c][r][s][k]
__global__ void __launch_bounds__(256) pack_weight_t_kernel(const float* __restrict__ w, WStrides ws,
                                                            uint16_t* __restrict__ out, int K,
                                                            int C, int R, int S) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)K * R * S * C;
  if (i >= total) return;
  int k = (int)(i % K);
  int64_t t = i / K;
  int s = (int)(t % S); t /= S;
  int r = (int)(t % R);
  int c = (int)(t / R);
  out[i] = f2bf(w[k * ws.k + c * ws.c + r * ws.r + s * ws.s]);
}

void launch_pack_weight(const float* w, const int64_t* strides, uint16_t* out, int K, int C, int R,
                        int S, int Cp, hipStream_t st) {
  WStrides ws{strides[0], strides[1], strides[2], strides[3]};
  int64_t total = (int64_t)K * R * S * Cp;
  hipLaunchKernelGGL(pack_weight_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     w, ws, out, K, C, R, S, Cp);
}

void launch_pack_weight_t(const float* w, const int64_t* strides, uint16_t* out, int K, int C,
                          int R, int S, hipStream_t st) {
  WStrides ws{strides[0], strides[1], strides[2], strides[3]};
  int64_t total = (int64_t)K * R * S * C;
  hipLaunchKernelGGL(pack_weight_t_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     w, ws, out, K, C, R, S);
}

}  // namespace pdt
