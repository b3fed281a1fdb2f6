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

// ---------------------------------------------------------------------------------------------
// Batched dgrad-layout pack: for every conv weight of a flat parameter space, the bf16 KRSC mirror
// slice src[off .. off + K*RS*C) (written by the fused SGD step) is transposed to CRSK at
// dst[off ..].  One launch for all layers: blockIdx.y = tensor, blockIdx.x walks that tensor's
// (tap, 64-k, 64-c) tiles; a 64x64 tile goes through LDS so reads (c-contiguous) and writes
// (k-contiguous) are both 16-B vectors.  Row pitch 66 halves (33 dwords): the transposed gather
// (lane (k-chunk m, c row r) reads tile[8m + q][r]) lands on banks 8m + r/2 + 33q -- distinct
// for the 8 k-chunks (the 72-half pitch put chunks m and m+2 on one bank: 4-way conflicts).
struct PackTEntry { int64_t off; int K, C, RS, tiles_k, tiles_c; };

__global__ void __launch_bounds__(256) pack_t_batched_kernel(const uint16_t* __restrict__ src,
                                                             uint16_t* __restrict__ dst,
                                                             const PackTEntry* __restrict__ tab) {
  __shared__ uint16_t tile[64][66];
  const PackTEntry e = tab[blockIdx.y];
  const int per_tap = e.tiles_k * e.tiles_c;
  const int ntiles = e.RS * per_tap;
  const int t = threadIdx.x;
  for (int tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
    const int tap = tile_id / per_tap;
    const int rem = tile_id - tap * per_tap;
    const int tk = rem / e.tiles_c, tc = rem - (rem / e.tiles_c) * e.tiles_c;
    const int k0 = tk * 64, c0 = tc * 64;
    // read 64 k-rows x 64 c (8 lanes per row, 8 bf16 each)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int row = it * 32 + (t >> 3), cc = (t & 7) * 8;
      const int k = k0 + row, c = c0 + cc;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (k < e.K && c < e.C)
        v = *reinterpret_cast<const uint4*>(src + e.off + ((int64_t)k * e.RS + tap) * e.C + c);
      const uint16_t* pv = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int q = 0; q < 8; ++q) tile[row][cc + q] = pv[q];
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int row = it * 32 + (t >> 3), kk = (t & 7) * 8;  // row = c within tile
      const int c = c0 + row, k = k0 + kk;
      if (c < e.C && k < e.K) {
        uint16_t o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = tile[kk + q][row];
        *reinterpret_cast<uint4*>(dst + e.off + ((int64_t)c * e.RS + tap) * e.K + k) =
            *reinterpret_cast<const uint4*>(o);
      }
    }
    __syncthreads();
  }
}

void launch_pack_t_batched(const uint16_t* src, uint16_t* dst, const void* table, int ntensors,
                           int max_tiles, hipStream_t st) {
  if (ntensors <= 0) return;
  const int bx = max_tiles < 512 ? max_tiles : 512;
  hipLaunchKernelGGL(pack_t_batched_kernel, dim3(bx > 0 ? bx : 1, ntensors), dim3(256), 0, st, src,
                     dst, reinterpret_cast<const PackTEntry*>(table));
}

size_t pack_t_entry_bytes() { return sizeof(PackTEntry); }

// ------------------------------------------------------------------------------------ stem
// one thread per output super-pixel (8 bf16 = 16 B store); reads the <= 8 source floats
__global__ void __launch_bounds__(256) stem_image_kernel(const float* __restrict__ x,
                                                         uint16_t* __restrict__ xsp, int N, int C,
                                                         int H, int W, int pad, int Hp, int Wsp) {
  const int64_t total = (int64_t)N * Hp * Wsp;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int ws = (int)(i % Wsp);
  const int64_t t = i / Wsp;
  const int hp = (int)(t % Hp);
  const int n = (int)(t / Hp);
  const int h = hp - pad;
  float v[8];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int w = 2 * ws + q - pad - 1;
    const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      v[q * 4 + c] = (in && c < C) ? x[(((int64_t)n * C + c) * H + h) * W + w] : 0.f;
  }
  uint4 o;
  o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
  o.z = pack2bf(v[4], v[5]); o.w = pack2bf(v[6], v[7]);
  reinterpret_cast<uint4*>(xsp)[i] = o;
}

void launch_stem_image(const float* x, uint16_t* xsp, int N, int C, int H, int W, int pad, int Hp,
                       int Wsp, hipStream_t st) {
  const int64_t total = (int64_t)N * Hp * Wsp;
  hipLaunchKernelGGL(stem_image_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, xsp,
                     N, C, H, W, pad, Hp, Wsp);
}

__global__ void stem_pack_weight_kernel(const float* __restrict__ w, WStrides ws,
                                        uint16_t* __restrict__ out, int K, int C, int R, int S,
                                        int Sp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = K * R * Sp * 8;
  if (i >= total) return;
  const int cq = i % 8, q = cq / 4, c = cq % 4;
  int t = i / 8;
  const int p = t % Sp; t /= Sp;
  const int r = t % R;
  const int k = t / R;
  const int s = 2 * p + q - 1;
  const float v = (c < C && s >= 0 && s < S) ? w[k * ws.k + c * ws.c + r * ws.r + s * ws.s] : 0.f;
  out[i] = f2bf(v);
}

void launch_stem_pack_weight(const float* w, const int64_t* strides, uint16_t* wsp, int K, int C,
                             int R, int S, int Sp, hipStream_t st) {
  WStrides ws{strides[0], strides[1], strides[2], strides[3]};
  const int total = K * R * Sp * 8;
  hipLaunchKernelGGL(stem_pack_weight_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w, ws, wsp,
                     K, C, R, S, Sp);
}

__global__ void stem_wgrad_unpack_kernel(const float* __restrict__ dwsp, float* __restrict__ out,
                                         WStrides os, int K, int C, int R, int S, int Sp,
                                         int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = K * C * R * S;
  if (i >= total) return;
  const int s = i % S;
  int t = i / S;
  const int r = t % R; t /= R;
  const int c = t % C;
  const int k = t / C;
  const int p = (s + 1) >> 1, q = (s + 1) & 1;
  const float v = dwsp[((k * R + r) * Sp + p) * 8 + q * 4 + c];
  float* o = out + k * os.k + c * os.c + r * os.r + s * os.s;
  *o = accumulate ? *o + v : v;
}

void launch_stem_wgrad_unpack(const float* dwsp, float* out, const int64_t* strides, int K, int C,
                              int R, int S, int Sp, bool accumulate, hipStream_t st) {
  WStrides os{strides[0], strides[1], strides[2], strides[3]};
  const int total = K * C * R * S;
  hipLaunchKernelGGL(stem_wgrad_unpack_kernel, dim3((total + 255) / 256), dim3(256), 0, st, dwsp, out,
                     os, K, C, R, S, Sp, accumulate ? 1 : 0);
}

}  // namespace pdt
