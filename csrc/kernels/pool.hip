// Pooling kernels, NHWC bf16.
//   max pool 3x3 / stride 2 / pad 1 (ResNet stem): forward stores the argmax
//   position (0..8) in one byte per output element; backward is a gather over
//   the <= 4 windows that contain each input pixel, so it is deterministic and
//   needs no atomics.  Tie-break = first maximum in row-major window order,
//   the same rule as ATen's max_pool2d_with_indices.
//   global average pool (head): [N,H,W,C] -> fp32 [N,C] and its backward.
#include "common.h"
#include "kernels.h"

namespace pdt {

__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const uint4* __restrict__ x,
                                                          uint4* __restrict__ y,
                                                          uint2* __restrict__ idx, int N, int H,
                                                          int W, int C8, int Ho, int Wo) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)N * Ho * Wo * C8;
  if (t >= total) return;
  int c8 = (int)(t % C8);
  int64_t p = t / C8;
  int wo = (int)(p % Wo);
  int64_t q = p / Wo;
  int ho = (int)(q % Ho);
  int n = (int)(q / Ho);
  float best[8];
  uint8_t bi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
  for (int kh = 0; kh < 3; ++kh) {
    int h = ho * 2 - 1 + kh;
    if (h < 0 || h >= H) continue;
    for (int kw = 0; kw < 3; ++kw) {
      int w = wo * 2 - 1 + kw;
      if (w < 0 || w >= W) continue;
      f8 v = unpack8(x[(((int64_t)n * H + h) * W + w) * C8 + c8]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (v.v[j] > best[j] || __builtin_isnan(v.v[j])) { best[j] = v.v[j]; bi[j] = (uint8_t)(kh * 3 + kw); }
      }
    }
  }
  f8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.v[j] = best[j];
  y[t] = pack8(o);
  uint2 id;
  id.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
  id.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
  idx[t] = id;
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const uint4* __restrict__ dy,
                                                          const uint2* __restrict__ idx,
                                                          uint4* __restrict__ dx, int N, int H,
                                                          int W, int C8, int Ho, int Wo) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)N * H * W * C8;
  if (t >= total) return;
  int c8 = (int)(t % C8);
  int64_t p = t / C8;
  int w = (int)(p % W);
  int64_t q = p / W;
  int h = (int)(q % H);
  int n = (int)(q / H);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int ho0 = (h + 1) / 2 - ((h + 1) % 2 == 0 ? 1 : 0);  // = ceil((h-1)/2) for h >= 0
  ho0 = max(ho0, 0);
  int ho1 = min((h + 1) / 2, Ho - 1);
  int wo0 = max((w + 1) / 2 - ((w + 1) % 2 == 0 ? 1 : 0), 0);
  int wo1 = min((w + 1) / 2, Wo - 1);
  for (int ho = ho0; ho <= ho1; ++ho) {
    int kh = h - (ho * 2 - 1);
    if (kh < 0 || kh > 2) continue;
    for (int wo = wo0; wo <= wo1; ++wo) {
      int kw = w - (wo * 2 - 1);
      if (kw < 0 || kw > 2) continue;
      uint32_t pos = (uint32_t)(kh * 3 + kw);
      int64_t o = (((int64_t)n * Ho + ho) * Wo + wo) * C8 + c8;
      uint2 id = idx[o];
      f8 g = unpack8(dy[o]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint32_t word = j < 4 ? id.x : id.y;
        uint32_t b = (word >> (8 * (j & 3))) & 0xffu;
        if (b == pos) acc[j] += g.v[j];
      }
    }
  }
  f8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.v[j] = acc[j];
  dx[t] = pack8(o);
}

void launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C,
                        int Ho, int Wo, hipStream_t st) {
  int C8 = C / 8;
  int64_t total = (int64_t)N * Ho * Wo * C8;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(x), reinterpret_cast<uint4*>(y),
                     reinterpret_cast<uint2*>(idx), N, H, W, C8, Ho, Wo);
}

void launch_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W,
                        int C, int Ho, int Wo, hipStream_t st) {
  int C8 = C / 8;
  int64_t total = (int64_t)N * H * W * C8;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(dy), reinterpret_cast<const uint2*>(idx),
                     reinterpret_cast<uint4*>(dx), N, H, W, C8, Ho, Wo);
}

// ------------------------------------------------------------- global avgpool
// block = (n, 256 channels); 16-byte loads would need 8 channels per thread, but
// C >= 512 here and HW = 49 (224 px) so one channel per thread keeps 256 lanes busy.
__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const uint16_t* __restrict__ x,
                                                          float* __restrict__ y, int HW, int C) {
  int n = blockIdx.y;
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const uint16_t* p = x + (int64_t)n * HW * C + c;
  float s = 0.f;
  for (int i = 0; i < HW; ++i) s += bf2f(p[(int64_t)i * C]);
  y[(int64_t)n * C + c] = s / (float)HW;
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const float* __restrict__ dy,
                                                          uint4* __restrict__ dx, int HW, int C8,
                                                          int64_t nvec, float inv, int splits,
                                                          int64_t split_stride) {
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    int c8 = (int)(v % C8);
    int64_t n = v / ((int64_t)C8 * HW);
    const float* g = dy + n * C8 * 8 + c8 * 8;
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = g[j];
    for (int z = 1; z < splits; ++z)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += g[z * split_stride + j];
    f8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o.v[j] = s[j] * inv;
    dx[v] = pack8(o);
  }
}

// 8 channels per thread (16-byte loads; the scalar form's 2-byte loads ran the ResNet-50 head,
// 256 x 7 x 7 x 2048, at ~1.4 TB/s: 18.5 us in-step).  Same fixed summation order per channel.
__global__ void __launch_bounds__(256) avgpool_fwd8_kernel(const uint4* __restrict__ x, float4* __restrict__ y,
                                                           int HW, int C8, int64_t total) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int64_t n = t / C8, c8 = t - n * C8;
  const uint4* p = x + n * HW * C8 + c8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 7
  for (int i = 0; i < HW; ++i) {
    const f8 v = unpack8(p[(int64_t)i * C8]);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += v.v[j];
  }
  const float inv = (float)HW;
  y[2 * t] = make_float4(s[0] / inv, s[1] / inv, s[2] / inv, s[3] / inv);
  y[2 * t + 1] = make_float4(s[4] / inv, s[5] / inv, s[6] / inv, s[7] / inv);
}

void launch_avgpool_fwd(const uint16_t* x, float* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
    const int64_t total = (int64_t)N * (C / 8);
    hipLaunchKernelGGL(avgpool_fwd8_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(x), reinterpret_cast<float4*>(y), HW, C / 8, total);
    return;
  }
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(ceil_div(C, 256), N), dim3(256), 0, st, x, y, HW, C);
}

void launch_avgpool_bwd(const float* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st, int splits) {
  int64_t nvec = (int64_t)N * HW * C / 8;
  int64_t b = (nvec + 255) / 256;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3((unsigned)(b < 8192 ? b : 8192)), dim3(256), 0, st,
                     dy, reinterpret_cast<uint4*>(dx), HW, C / 8, nvec, 1.f / (float)HW, splits,
                     (int64_t)N * C);
}

}  // namespace pdt
