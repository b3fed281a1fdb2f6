// Fused BatchNorm (+residual add) (+ReLU): statistics finalize, forward apply,
// backward reduction and backward apply.  NHWC bf16 activations, fp32 math.
//
// Training-mode BN needs a grid-wide per-channel reduction before the
// normalize; the conv epilogue already produced per-64-row partials
// (sum, M2) in registers, so forward BN is: finalize (tiny, two-level Chan
// merge) + ONE read-y/write-z pass.  Backward is one reduction pass over
// (dz, z, y) and one elementwise pass producing dy and the residual gradient.
#include "common.h"
#include "kernels.h"

namespace pdt {

// ------------------------------------------------------------------ finalize
// Stage 1: block (cx, p) merges groups [p*GPB, (p+1)*GPB) for 32 channels.
constexpr int FIN_CH = 32;
constexpr int FIN_ROWS = 8;                 // threads per channel in a block
constexpr int FIN_GPB = FIN_ROWS * 32;      // groups per block

__global__ void __launch_bounds__(256) bn_finalize_stage1(const float* __restrict__ part, int ngroups,
                                                          int grows, int M, int K,
                                                          float* __restrict__ ws) {
  __shared__ float sn[FIN_ROWS][FIN_CH], smu[FIN_ROWS][FIN_CH], sm2[FIN_ROWS][FIN_CH];
  int tx = threadIdx.x & (FIN_CH - 1), ty = threadIdx.x / FIN_CH;
  int k = blockIdx.x * FIN_CH + tx;
  int g0 = blockIdx.y * FIN_GPB;
  int g1 = min(ngroups, g0 + FIN_GPB);
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (k < K) {
    for (int g = g0 + ty; g < g1; g += FIN_ROWS) {
      float cnt = (float)min(grows, M - g * grows);
      float s = part[((int64_t)g * 2 + 0) * K + k];
      float q = part[((int64_t)g * 2 + 1) * K + k];
      chan_merge(n, mu, m2, cnt, s / cnt, q);
    }
  }
  sn[ty][tx] = n; smu[ty][tx] = mu; sm2[ty][tx] = m2;
  __syncthreads();
  if (ty == 0 && k < K) {
    for (int r = 1; r < FIN_ROWS; ++r) chan_merge(n, mu, m2, sn[r][tx], smu[r][tx], sm2[r][tx]);
    float* o = ws + ((int64_t)blockIdx.y * 3) * K;
    o[k] = n; o[K + k] = mu; o[2 * K + k] = m2;
  }
}

__global__ void __launch_bounds__(256) bn_finalize_stage2(const float* __restrict__ ws, int P, int M,
                                                          int K, float* __restrict__ rm,
                                                          float* __restrict__ rv,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          float momentum, float eps,
                                                          float* __restrict__ out) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int p = 0; p < P; ++p) {
    const float* o = ws + ((int64_t)p * 3) * K;
    chan_merge(n, mu, m2, o[k], o[K + k], o[2 * K + k]);
  }
  float var = m2 / (float)M;
  float invstd = rsqrtf(var + eps);
  if (rm != nullptr) {
    float unb = M > 1 ? m2 / (float)(M - 1) : var;
    rm[k] = (1.f - momentum) * rm[k] + momentum * mu;
    rv[k] = (1.f - momentum) * rv[k] + momentum * unb;
  }
  float sc = gamma[k] * invstd;
  out[k] = mu;
  out[K + k] = invstd;
  out[2 * K + k] = sc;
  out[3 * K + k] = beta[k] - mu * sc;
}

int bn_finalize_partitions(int ngroups) { return ceil_div(ngroups, FIN_GPB); }

void launch_bn_finalize(const float* part, int ngroups, int grows, int M, int K, float* rm, float* rv,
                        const float* gamma, const float* beta, float momentum, float eps,
                        float* out, hipStream_t st) {
  // workspace for stage-1 partials lives after out[4][K] (caller allocates 4K + 3K*P floats)
  int P = ceil_div(ngroups, FIN_GPB);
  float* ws = out + 4 * (int64_t)K;
  hipLaunchKernelGGL(bn_finalize_stage1, dim3(ceil_div(K, FIN_CH), P), dim3(256), 0, st, part,
                     ngroups, grows, M, K, ws);
  hipLaunchKernelGGL(bn_finalize_stage2, dim3(ceil_div(K, 256)), dim3(256), 0, st, ws, P, M, K, rm,
                     rv, gamma, beta, momentum, eps, out);
}

__global__ void bn_eval_params_kernel(const float* rm, const float* rv, const float* gamma,
                                      const float* beta, float eps, int K, float* out) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float invstd = rsqrtf(rv[k] + eps);
  float sc = gamma[k] * invstd;
  out[k] = rm[k];
  out[K + k] = invstd;
  out[2 * K + k] = sc;
  out[3 * K + k] = beta[k] - rm[k] * sc;
}

void launch_bn_eval_params(const float* rm, const float* rv, const float* gamma, const float* beta,
                           float eps, int K, float* out, hipStream_t st) {
  hipLaunchKernelGGL(bn_eval_params_kernel, dim3(ceil_div(K, 256)), dim3(256), 0, st, rm, rv, gamma,
                     beta, eps, K, out);
}

// ------------------------------------------------------------------- forward
template <bool RES, bool RELU>
__global__ void __launch_bounds__(256) bn_act_fwd_kernel(const uint4* __restrict__ y,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         const uint4* __restrict__ res,
                                                         uint4* __restrict__ z, int64_t nvec,
                                                         int K8) {
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    int c0 = (int)(v % K8) * 8;
    f8 a = unpack8(y[v]);
    float4 s0 = *reinterpret_cast<const float4*>(scale + c0);
    float4 s1 = *reinterpret_cast<const float4*>(scale + c0 + 4);
    float4 h0 = *reinterpret_cast<const float4*>(shift + c0);
    float4 h1 = *reinterpret_cast<const float4*>(shift + c0 + 4);
    float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    f8 r;
    if (RES) r = unpack8(res[v]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = fmaf(a.v[j], sc[j], sh[j]);
      if (RES) t += r.v[j];
      if (RELU) t = fmaxf(t, 0.f);
      a.v[j] = t;
    }
    z[v] = pack8(a);
  }
}

static int ew_blocks(int64_t nvec) {
  int64_t b = (nvec + 255) / 256;
  return (int)(b < 8192 ? b : 8192);
}

void launch_bn_act_fwd(const uint16_t* y, const float* scale, const float* shift,
                       const uint16_t* res, bool relu, uint16_t* z, int64_t M, int K,
                       hipStream_t st) {
  int64_t nvec = M * K / 8;
  int K8 = K / 8;
  dim3 g(ew_blocks(nvec)), b(256);
  auto Y = reinterpret_cast<const uint4*>(y);
  auto R = reinterpret_cast<const uint4*>(res);
  auto Z = reinterpret_cast<uint4*>(z);
  if (res) {
    if (relu) hipLaunchKernelGGL((bn_act_fwd_kernel<true, true>), g, b, 0, st, Y, scale, shift, R, Z, nvec, K8);
    else hipLaunchKernelGGL((bn_act_fwd_kernel<true, false>), g, b, 0, st, Y, scale, shift, R, Z, nvec, K8);
  } else {
    if (relu) hipLaunchKernelGGL((bn_act_fwd_kernel<false, true>), g, b, 0, st, Y, scale, shift, R, Z, nvec, K8);
    else hipLaunchKernelGGL((bn_act_fwd_kernel<false, false>), g, b, 0, st, Y, scale, shift, R, Z, nvec, K8);
  }
}

// ------------------------------------------------------------ backward reduce
// Block b reduces rows [b*RPB, (b+1)*RPB) for all channels; requires 256 % K8 == 0.
constexpr int RED_BLOCKS_MAX = 1024;

static int red_blocks(int64_t M) {
  int64_t b = (M + 255) / 256;  // >= 256 rows per block
  return (int)(b < RED_BLOCKS_MAX ? b : RED_BLOCKS_MAX);
}

size_t bn_bwd_ws_floats(int64_t M, int K) { return (size_t)red_blocks(M) * 2 * K; }

template <bool RELU>
__global__ void __launch_bounds__(256) bn_bwd_reduce_stage1(const uint4* __restrict__ dz,
                                                            const uint4* __restrict__ z,
                                                            const uint4* __restrict__ y,
                                                            const float* __restrict__ mean,
                                                            int64_t M, int K8,
                                                            float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int t = threadIdx.x;
  const int c8 = t % K8;
  const int rpi = 256 / K8;  // rows per iteration
  const int roff = t / K8;
  int64_t rows_per_block = (M + gridDim.x - 1) / gridDim.x;
  int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t r1 = min(M, r0 + rows_per_block);
  float mu[8];
  {
    float4 m0 = *reinterpret_cast<const float4*>(mean + c8 * 8);
    float4 m1 = *reinterpret_cast<const float4*>(mean + c8 * 8 + 4);
    mu[0] = m0.x; mu[1] = m0.y; mu[2] = m0.z; mu[3] = m0.w;
    mu[4] = m1.x; mu[5] = m1.y; mu[6] = m1.z; mu[7] = m1.w;
  }
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = r0 + roff; r < r1; r += rpi) {
    int64_t v = r * K8 + c8;
    f8 d = unpack8(dz[v]);
    f8 yy = unpack8(y[v]);
    f8 zz;
    if (RELU) zz = unpack8(z[v]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = d.v[j];
      if (RELU) g = zz.v[j] > 0.f ? g : 0.f;
      sg[j] += g;
      sgx[j] = fmaf(g, yy.v[j] - mu[j], sgx[j]);
    }
  }
  // block reduction over threads with equal c8: sh[roff][c8*16 + j]
  float* my = sh + (size_t)t * 16;
#pragma unroll
  for (int j = 0; j < 8; ++j) { my[j] = sg[j]; my[8 + j] = sgx[j]; }
  __syncthreads();
  for (int s = rpi / 2; s > 0; s >>= 1) {
    if (roff < s) {
      float* o = sh + (size_t)(t + s * K8) * 16;
#pragma unroll
      for (int j = 0; j < 16; ++j) my[j] += o[j];
    }
    __syncthreads();
  }
  if (roff == 0) {
    int K = K8 * 8;
    float* o = ws + (int64_t)blockIdx.x * 2 * K;
#pragma unroll
    for (int j = 0; j < 8; ++j) { o[c8 * 8 + j] = my[j]; o[K + c8 * 8 + j] = my[8 + j]; }
  }
}

// block = 32 channels x 8 partial-lanes; each lane sums nb/8 stage-1 partials (independent
// loads, pipelined), then an LDS combine.  Deterministic (fixed order).
__global__ void __launch_bounds__(256) bn_bwd_reduce_stage2(const float* __restrict__ ws, int nb,
                                                            int K, float* __restrict__ sums) {
  __shared__ float sa[8][33], sb[8][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int k = blockIdx.x * 32 + tx;
  float a = 0.f, b = 0.f;
  if (k < K) {
#pragma unroll 4
    for (int i = ty; i < nb; i += 8) {
      a += ws[(int64_t)i * 2 * K + k];
      b += ws[(int64_t)i * 2 * K + K + k];
    }
  }
  sa[ty][tx] = a;
  sb[ty][tx] = b;
  __syncthreads();
  if (ty == 0 && k < K) {
    for (int r = 1; r < 8; ++r) { a += sa[r][tx]; b += sb[r][tx]; }
    sums[k] = a;       // sum g          (= dbeta)
    sums[K + k] = b;   // sum g*(y-mean) (dgamma = b*invstd)
  }
}

void launch_bn_act_bwd_reduce(const uint16_t* dz, const uint16_t* z, const uint16_t* y,
                              const float* mean, bool relu, int64_t M, int K, float* ws,
                              float* sums, hipStream_t st) {
  int K8 = K / 8;
  int nb = red_blocks(M);
  size_t shmem = 256 * 16 * sizeof(float);
  auto DZ = reinterpret_cast<const uint4*>(dz);
  auto Z = reinterpret_cast<const uint4*>(z);
  auto Y = reinterpret_cast<const uint4*>(y);
  if (relu)
    hipLaunchKernelGGL(bn_bwd_reduce_stage1<true>, dim3(nb), dim3(256), shmem, st, DZ, Z, Y, mean, M, K8, ws);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_stage1<false>, dim3(nb), dim3(256), shmem, st, DZ, Z, Y, mean, M, K8, ws);
  hipLaunchKernelGGL(bn_bwd_reduce_stage2, dim3(ceil_div(K, 32)), dim3(256), 0, st, ws, nb, K, sums);
}

// ------------------------------------------------------------- backward apply
template <bool RELU, bool TRAIN, bool DRES>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const uint4* __restrict__ dz, const uint4* __restrict__ z, const uint4* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ sums, int64_t nvec, int K8,
    float invM, uint4* __restrict__ dy, uint4* __restrict__ dres) {
  const int K = K8 * 8;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    int c0 = (int)(v % K8) * 8;
    f8 d = unpack8(dz[v]);
    f8 zz, yy;
    if (RELU) zz = unpack8(z[v]);
    if (TRAIN) yy = unpack8(y[v]);
    f8 o, gr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int c = c0 + j;
      float g = d.v[j];
      if (RELU) g = zz.v[j] > 0.f ? g : 0.f;
      gr.v[j] = g;
      float is = invstd[c];
      float k1 = gamma[c] * is;
      if (TRAIN) {
        float sg = sums[c] * invM;                 // mean of g
        float k2 = sums[K + c] * is * is * invM;   // mean of g*xhat, divided by std
        o.v[j] = k1 * (g - sg - (yy.v[j] - mean[c]) * k2);
      } else {
        o.v[j] = k1 * g;
      }
    }
    dy[v] = pack8(o);
    if (DRES) dres[v] = pack8(gr);
  }
}

void launch_bn_act_bwd_apply(const uint16_t* dz, const uint16_t* z, const uint16_t* y,
                             const float* mean, const float* invstd, const float* gamma,
                             const float* sums, bool relu, bool training, int64_t M, int K,
                             uint16_t* dy, uint16_t* dres, hipStream_t st) {
  int64_t nvec = M * K / 8;
  int K8 = K / 8;
  dim3 g(ew_blocks(nvec)), b(256);
  auto DZ = reinterpret_cast<const uint4*>(dz);
  auto Z = reinterpret_cast<const uint4*>(z);
  auto Y = reinterpret_cast<const uint4*>(y);
  auto DY = reinterpret_cast<uint4*>(dy);
  auto DR = reinterpret_cast<uint4*>(dres);
  float invM = 1.f / (float)M;
#define PDT_BWD(RL, TR, DRS)                                                                     \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<RL, TR, DRS>), g, b, 0, st, DZ, Z, Y, mean, invstd, \
                     gamma, sums, nvec, K8, invM, DY, DR)
  bool dr = dres != nullptr;
  if (relu) {
    if (training) { if (dr) PDT_BWD(true, true, true); else PDT_BWD(true, true, false); }
    else { if (dr) PDT_BWD(true, false, true); else PDT_BWD(true, false, false); }
  } else {
    if (training) { if (dr) PDT_BWD(false, true, true); else PDT_BWD(false, true, false); }
    else { if (dr) PDT_BWD(false, false, true); else PDT_BWD(false, false, false); }
  }
#undef PDT_BWD
}

}  // namespace pdt
