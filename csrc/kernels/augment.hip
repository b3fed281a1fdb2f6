// Batched training-data augmentation on the device: the reference's per-sample PIL chain
// RandomCrop(H, padding) -> RandomHorizontalFlip -> ToTensor -> Normalize (resnet/main.py:87-92,
// run on 8 CPU worker processes there) as ONE gather kernel over a device-resident dataset.
//
// out[b][c][y][x] = norm(src[idx[b]][c][y + oy[b] - pad][flip ? W-1-x+ox[b]-pad : x+ox[b]-pad])
// with zero padding applied BEFORE normalization (torchvision pads the [0,1] tensor with 0, so a
// pad pixel becomes -mean/std), ToTensor's /255 for uint8 sources, and the same fp32 operation
// order as the batched torch path in data/loader.py (x * (1/255) -- ATen divides by a scalar
// through its reciprocal -- then (x - mean)/std), so both paths
// agree bit for bit.  One thread per output pixel-row segment of 4 pixels (16-B stores).
#include "common.h"
#include "kernels.h"

#include <stdexcept>

namespace pdt {

template <bool U8, bool NORM>
__global__ void __launch_bounds__(256) augment_kernel(const void* __restrict__ src_, const int64_t* __restrict__ idx,
                                                      const int64_t* __restrict__ oy, const int64_t* __restrict__ ox,
                                                      const bool* __restrict__ flip, float* __restrict__ out,
                                                      int B, int C, int H, int W, int pad, float m0, float m1,
                                                      float m2, float s0, float s1, float s2) {
  const int W4 = W / 4;
  const int64_t total = (int64_t)B * C * H * W4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int x4 = (int)(t % W4);
  int64_t r = t / W4;
  const int y = (int)(r % H);
  r /= H;
  const int c = (int)(r % C);
  const int b = (int)(r / C);
  const int64_t n = idx[b];
  const int sy = y + (int)oy[b] - pad;
  const bool fl = flip != nullptr && flip[b];
  const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
  const float stdv = c == 0 ? s0 : (c == 1 ? s1 : s2);
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int x = x4 * 4 + q;
    const int sx = (fl ? (W - 1 - x) : x) + (int)ox[b] - pad;
    float p = 0.f;
    if ((unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W) {
      const int64_t o = ((n * C + c) * H + sy) * W + sx;
      if constexpr (U8) p = (float)reinterpret_cast<const uint8_t*>(src_)[o] * (1.0f / 255.0f);
      else p = reinterpret_cast<const float*>(src_)[o];
    }
    if constexpr (NORM) p = (p - mean) / stdv;
    v[q] = p;
  }
  *reinterpret_cast<float4*>(out + t * 4) = make_float4(v[0], v[1], v[2], v[3]);
}

void launch_augment(const void* src, bool src_u8, const int64_t* idx, const int64_t* oy, const int64_t* ox,
                    const bool* flip, float* out, int B, int C, int H, int W, int pad, bool normalize,
                    const float* mean, const float* stdv, hipStream_t st) {
  if (W % 4 != 0) throw std::runtime_error("augment: width must be a multiple of 4");
  if (C > 3) throw std::runtime_error("augment: at most 3 channels");
  const int64_t total = (int64_t)B * C * H * (W / 4);
  const unsigned blocks = (unsigned)((total + 255) / 256);
#define PDT_AUG(U8, NRM)                                                                          \
  hipLaunchKernelGGL((augment_kernel<U8, NRM>), dim3(blocks), dim3(256), 0, st, src, idx, oy, ox, flip, \
                     out, B, C, H, W, pad, mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2])
  if (src_u8) { if (normalize) PDT_AUG(true, true); else PDT_AUG(true, false); }
  else { if (normalize) PDT_AUG(false, true); else PDT_AUG(false, false); }
#undef PDT_AUG
}

}  // namespace pdt
