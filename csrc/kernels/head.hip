// Classifier head kernels: fused softmax cross-entropy (forward loss AND the
// logits gradient in one pass over the logits) and the top-1 correct counter
// used by evaluation (replaces max + eq + sum + .item() of resnet/main.py:32-34).
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace pdt {

// one 256-thread block per row
__global__ void __launch_bounds__(256) softmax_xent_kernel(const float* __restrict__ logits,
                                                           const int64_t* __restrict__ labels,
                                                           float* __restrict__ dlogits,
                                                           float* __restrict__ row_loss, int V,
                                                           float invN) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const float* x = logits + (int64_t)row * V;
  float* g = dlogits + (int64_t)row * V;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  float m = -INFINITY;
  for (int i = t; i < V; i += 256) m = fmaxf(m, x[i]);
  m = wave_max(m);
  if (lane == 0) red[wid] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int i = t; i < V; i += 256) s += __expf(x[i] - m);
  s = wave_sum(s);
  if (lane == 0) red[wid] = s;
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  const float inv_s = 1.f / s;
  const int64_t lab = labels[row];
  for (int i = t; i < V; i += 256) {
    float p = __expf(x[i] - m) * inv_s;
    g[i] = (p - (i == lab ? 1.f : 0.f)) * invN;
  }
  if (t == 0) row_loss[row] = (logf(s) + m - x[lab]);
}

// deterministic mean of the per-row losses (single block)
__global__ void __launch_bounds__(256) mean_kernel(const float* __restrict__ v, int n,
                                                   float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1] + red[2] + red[3]) / (float)n;
}

void launch_softmax_xent(const float* logits, const int64_t* labels, float* loss, float* dlogits,
                         float* ws, int N, int V, hipStream_t st) {
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(N), dim3(256), 0, st, logits, labels, dlogits, ws, V,
                     1.f / (float)N);
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, st, ws, N, loss);
}

// y = x * alpha[0] (alpha on the device: no host sync for the loss gradient)
__global__ void __launch_bounds__(256) scale_kernel(const float4* __restrict__ x, const float* __restrict__ alpha,
                                                    float4* __restrict__ y, int64_t n4) {
  const float a = alpha[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = x[i];
    v.x *= a; v.y *= a; v.z *= a; v.w *= a;
    y[i] = v;
  }
}

__global__ void scale_tail_kernel(const float* __restrict__ x, const float* __restrict__ alpha,
                                  float* __restrict__ y, int64_t start, int64_t n) {
  const int64_t i = start + threadIdx.x;
  if (i < n) y[i] = x[i] * alpha[0];
}

void launch_scale(const float* x, const float* alpha, float* y, int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4;
  if (n4 > 0) {
    const int64_t b = std::min<int64_t>((n4 + 255) / 256, 4096);
    hipLaunchKernelGGL(scale_kernel, dim3((unsigned)b), dim3(256), 0, st, reinterpret_cast<const float4*>(x),
                       alpha, reinterpret_cast<float4*>(y), n4);
  }
  if (n4 * 4 < n)
    hipLaunchKernelGGL(scale_tail_kernel, dim3(1), dim3(64), 0, st, x, alpha, y, n4 * 4, n);
}

__global__ void __launch_bounds__(256) add_one_i64_kernel(int64_t* __restrict__ x, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += 1;
}

void launch_add_one_i64(int64_t* x, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(add_one_i64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n);
}

__global__ void __launch_bounds__(256) top1_kernel(const float* __restrict__ logits,
                                                   const int64_t* __restrict__ labels,
                                                   unsigned long long* __restrict__ count, int V) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x;
  const float* x = logits + (int64_t)row * V;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = t; i < V; i += 256) {
    float v = x[i];
    if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(bv, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  if (lane == 0) { sv[wid] = bv; si[wid] = bi; }
  __syncthreads();
  if (t == 0) {
    for (int w = 1; w < 4; ++w)
      if (sv[w] > bv || (sv[w] == bv && si[w] < bi)) { bv = sv[w]; bi = si[w]; }
    if ((int64_t)bi == labels[row]) atomicAdd(count, 1ull);
  }
}

void launch_top1(const float* logits, const int64_t* labels, int64_t* count, int N, int V,
                 hipStream_t st) {
  hipMemsetAsync(count, 0, sizeof(int64_t), st);
  hipLaunchKernelGGL(top1_kernel, dim3(N), dim3(256), 0, st, logits, labels,
                     reinterpret_cast<unsigned long long*>(count), V);
}

}  // namespace pdt
