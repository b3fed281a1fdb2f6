// Fused BatchNorm (+residual add) (+ReLU): statistics finalize, forward apply,
// backward reduction and backward apply.  NHWC bf16 activations, fp32 math.
//
// Training-mode BN needs a grid-wide per-channel reduction before the
// normalize; the conv epilogue already produced per-64-row partials
// (sum, M2) in registers, so forward BN is: finalize (tiny, two-level Chan
// merge) + ONE read-y/write-z pass.  Backward is one reduction pass over
// (dz, z, y) and one elementwise pass producing dy and the residual gradient.
#include "common.h"
#include "fp8_util.h"
#include "igemm_common.h"
#include "kernels.h"
#include "pool_quad.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <unordered_map>

namespace pdt {

__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// ------------------------------------------------------------------ finalize
// Group g (grows rows, the last one possibly fewer) carries (s_g, q_g) = (sum, M2 about its mean).
// With S = sum s_g, A = sum q_g, B = sum s_g^2/n_g:  mean = S/M,  M2 = A + B - S^2/M
// (exact decomposition of the total sum of squares; only plain sums -> fully parallel, no
// serial divide chain).  Stage 1: block (32 channels, partition p of FIN_GPB groups);
// stage 2: per channel sum over partitions, fixed order (deterministic).
// Block shape (PDT_FIN_CH channels x 256/PDT_FIN_CH group rows): a tall block gives each thread
// fewer dependent partial loads (the reduction is latency-bound: ~100 of these tiny launches sit
// on the critical path of a ResNet-50 step).
#ifndef PDT_FIN_CH
#define PDT_FIN_CH 32
#endif
constexpr int FIN_CH = PDT_FIN_CH;
constexpr int FIN_ROWS = 256 / FIN_CH;      // threads per channel in a block
constexpr int FIN_GPB = FIN_ROWS * 16;      // groups per block (16 independent loads per thread)
// Up to FIN_SINGLE groups, ONE block per 32-channel tile reads them all and finishes in place:
// no partial round trip and no last-block handshake (a dependent sc1 store / atomic / sc1 load
// chain worth ~2-3 us of a ~6 us launch; every ResNet-50 layer2-4 BN qualifies).
constexpr int FIN_SINGLE = 512;
static int fin_single() {  // PDT_FIN_SINGLE=0: always two-level (A/B knob)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PDT_FIN_SINGLE");
    v = e ? std::max(0, atoi(e)) : FIN_SINGLE;
  }
  return v;
}
static int fin_gpb(int G) { return G <= fin_single() ? std::max(G, 1) : FIN_GPB; }

// Per-channel-tile completion counters for the single-launch two-level reductions below
// (zero-initialised once; the last block of a tile resets its counter, so launches on one stream
// can reuse them back to back).  One bank of kTileCounters per stream (counter_bank(): the first
// kCounterBanks distinct streams -- compute, capture, side, warm-up -- get a bank each), so
// reductions on different streams, e.g. a graph replay beside eager work, never share a counter.
// A stream seen after the banks are used up gets NO bank (-1): its reductions take the two-launch
// path (partials, then finalize), which needs no counter at all.  Sharing a bank between two
// streams would let concurrent launches count each other's blocks (early or never-completing
// handshake).  Within a bank, forward finalize uses [0, 2048) and backward reduce [2048, 4096).
constexpr int kTileCounters = 4096;
constexpr int kCounterBanks = 8;
__device__ unsigned int g_tile_counters[kCounterBanks * kTileCounters];

static int counter_bank(hipStream_t st) {
  static std::mutex mu;
  static std::unordered_map<hipStream_t, int> banks;
  std::lock_guard<std::mutex> lock(mu);
  auto it = banks.find(st);
  if (it != banks.end()) return it->second < 0 ? -1 : it->second * kTileCounters;
  const int b = banks.size() < (size_t)kCounterBanks ? (int)banks.size() : -1;
  banks.emplace(st, b);
  return b < 0 ? -1 : b * kTileCounters;
}

// Test introspection: the bank (0..kCounterBanks-1) a stream's single-launch reductions use, or -1
// when it got none and runs the two-launch path.  Registers the stream like a launch would.
int bn_counter_bank(hipStream_t st) {
  const int off = counter_bank(st);
  return off < 0 ? -1 : off / kTileCounters;
}

// PDT_BN_LASTBLOCK=0: two launches (partials, then finalize) instead of the last-block handshake
static bool bn_lastblock() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PDT_BN_LASTBLOCK");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// Last-arriver handshake without fences (MI355X_MICROARCH "Hand-offs measured with sc1 loads",
// first row): every block publishes its stage-1 partial with write-through stores (st_wt: agent-
// scope relaxed = global_store sc1), every storing wave drains them (vmcnt 0), a barrier, then ONE
// lane adds to the tile's unsharded counter; the block whose add returns nblocks-1 is the last one
// and reads the partials with L1-bypassing loads (ld_wt: global_load sc1).  No agent release
// (buffer_wbl2, >= 1.7 us) in every block and no acquire (buffer_inv, ~1.7 us) in the last one:
// both sat on the critical path of ~100 tiny reductions per ResNet-50 step.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool last_block_of_tile(int tile, unsigned int nblocks) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its st_wt stores landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int prev = __hip_atomic_fetch_add(&g_tile_counters[tile], 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
    const bool last = prev == nblocks - 1;
    if (last) __hip_atomic_store(&g_tile_counters[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last ? 1 : 0;
  }
  __syncthreads();
  return s_last != 0;
}

// Stage 1 per block (32 channels x FIN_GPB groups) -> ws[p][3][K]; the last partition block of a
// channel tile then sums the P partials in fixed order (deterministic) and writes mean, invstd,
// scale, shift and the running-stat update: one launch per BatchNorm.
__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ part, int ngroups,
                                                          int grows, int M, int K,
                                                          float* __restrict__ ws,
                                                          float* __restrict__ rm,
                                                          float* __restrict__ rv,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          float momentum, float eps,
                                                          float* __restrict__ out, int mode,
                                                          int nparts, int cbase, int gpb) {
  // mode 0: partials + last-block finalize (one launch); 1: partials only; 2: finalize only
  __shared__ float sS[FIN_ROWS][FIN_CH + 1], sA[FIN_ROWS][FIN_CH + 1], sB[FIN_ROWS][FIN_CH + 1];
  const int tx = threadIdx.x & (FIN_CH - 1), ty = threadIdx.x / FIN_CH;
  const int k = blockIdx.x * FIN_CH + tx;
  const int g0 = blockIdx.y * gpb;
  const int g1 = min(ngroups, g0 + gpb);
  float S = 0.f, A = 0.f, B = 0.f;
  if (mode != 2) {
  if (k < K) {
#pragma unroll 8
    for (int g = g0 + ty; g < g1; g += FIN_ROWS) {
      const float cnt = (float)min(grows, M - g * grows);
      const float sg = part[((int64_t)g * 2 + 0) * K + k];
      const float qg = part[((int64_t)g * 2 + 1) * K + k];
      S += sg;
      A += qg;
      B = fmaf(sg, sg / cnt, B);
    }
  }
  sS[ty][tx] = S; sA[ty][tx] = A; sB[ty][tx] = B;
  __syncthreads();
  const bool direct = mode == 0 && gridDim.y == 1;  // one partition: finish in place
  if (ty == 0 && k < K) {
    for (int r = 1; r < FIN_ROWS; ++r) { S += sS[r][tx]; A += sA[r][tx]; B += sB[r][tx]; }
    if (!direct) {
      float* o = ws + ((int64_t)blockIdx.y * 3) * K;
      st_wt(o + k, S); st_wt(o + K + k, A); st_wt(o + 2 * K + k, B);
    }
  }
  if (mode == 1) return;
  if (direct) {
    if (ty != 0 || k >= K) return;
  } else if (!last_block_of_tile(cbase + blockIdx.x, gridDim.y)) {
    return;
  }
  }
  const bool direct = mode == 0 && gridDim.y == 1;
  const int P = mode == 2 ? nparts : gridDim.y;
  if (!direct) {
  S = 0.f; A = 0.f; B = 0.f;
  if (k < K) {
#pragma unroll 8
    for (int p = ty; p < P; p += FIN_ROWS) {
      const float* o = ws + ((int64_t)p * 3) * K;
      S += ld_wt(o + k); A += ld_wt(o + K + k); B += ld_wt(o + 2 * K + k);
    }
  }
  sS[ty][tx] = S; sA[ty][tx] = A; sB[ty][tx] = B;
  __syncthreads();
  if (ty != 0 || k >= K) return;
  for (int r = 1; r < FIN_ROWS; ++r) { S += sS[r][tx]; A += sA[r][tx]; B += sB[r][tx]; }
  }
  const float mu = S / (float)M;
  const float m2 = fmaxf(A + B - S * mu, 0.f);
  const float var = m2 / (float)M;
  const float invstd = rsqrtf(var + eps);
  if (rm != nullptr) {
    const float unb = M > 1 ? m2 / (float)(M - 1) : var;
    rm[k] = (1.f - momentum) * rm[k] + momentum * mu;
    rv[k] = (1.f - momentum) * rv[k] + momentum * unb;
  }
  const float sc = gamma[k] * invstd;
  out[k] = mu;
  out[K + k] = invstd;
  out[2 * K + k] = sc;
  out[3 * K + k] = beta[k] - mu * sc;
}

int bn_finalize_partitions(int ngroups) { return ceil_div(ngroups, fin_gpb(ngroups)); }

void launch_bn_finalize(const float* part, int ngroups, int grows, int M, int K, float* rm, float* rv,
                        const float* gamma, const float* beta, float momentum, float eps,
                        float* out, hipStream_t st) {
  // workspace for stage-1 partials lives after out[4][K] (caller allocates 4K + 3K*P floats)
  const int gpb = fin_gpb(ngroups);
  int P = ceil_div(ngroups, gpb);
  float* ws = out + 4 * (int64_t)K;
  if (ceil_div(K, FIN_CH) > kTileCounters / 2) throw std::runtime_error("bn_finalize: too many channels");
  const int bank = (bn_lastblock() && P > 1) ? counter_bank(st) : 0;
  if (bn_lastblock() && bank >= 0) {
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(K, FIN_CH), P), dim3(256), 0, st, part,
                       ngroups, grows, M, K, ws, rm, rv, gamma, beta, momentum, eps, out, 0, P,
                       bank, gpb);
  } else {
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(K, FIN_CH), P), dim3(256), 0, st, part,
                       ngroups, grows, M, K, ws, rm, rv, gamma, beta, momentum, eps, out, 1, P, 0, gpb);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(K, FIN_CH), 1), dim3(256), 0, st, part,
                       ngroups, grows, M, K, ws, rm, rv, gamma, beta, momentum, eps, out, 2, P, 0, gpb);
  }
}

// Finalize from fp64 totals (kernels.h BnFwdFuse): one thread per channel; the sums are read once
// and re-zeroed for the next conv that accumulates into them.
__global__ void __launch_bounds__(256) bn_finalize_sums_kernel(double* __restrict__ acc, int M, int K,
                                                               float* __restrict__ rm, float* __restrict__ rv,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float momentum,
                                                               float eps, float* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  // every load issued up front: one memory round trip on the critical stream, not two
  double s[kStatSlots], q[kStatSlots];
#pragma unroll
  for (int x = 0; x < kStatSlots; ++x) {  // the conv's per-XCD slots
    s[x] = acc[(size_t)x * 2 * K + k];
    q[x] = acc[(size_t)x * 2 * K + K + k];
  }
  const float g = gamma[k], bt = beta[k];
  const float rm0 = rm != nullptr ? rm[k] : 0.f, rv0 = rm != nullptr ? rv[k] : 0.f;
  double S = 0.0, Q = 0.0;
#pragma unroll
  for (int x = 0; x < kStatSlots; ++x) {  // fixed order
    S += s[x];
    Q += q[x];
    acc[(size_t)x * 2 * K + k] = 0.0;
    acc[(size_t)x * 2 * K + K + k] = 0.0;
  }
  const double Md = (double)M;
  const double mu = S / Md;
  const double var = fmax(Q / Md - mu * mu, 0.0);
  const float invstd = rsqrtf((float)var + eps);
  if (rm != nullptr) {
    const float unb = M > 1 ? (float)(var * Md / (Md - 1.0)) : (float)var;
    rm[k] = (1.f - momentum) * rm0 + momentum * (float)mu;
    rv[k] = (1.f - momentum) * rv0 + momentum * unb;
  }
  const float sc = g * invstd;
  out[k] = (float)mu;
  out[K + k] = invstd;
  out[2 * K + k] = sc;
  out[3 * K + k] = bt - (float)mu * sc;
}

void launch_bn_finalize_sums(const BnFwdFuse& bn, int M, int K, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_sums_kernel, dim3(ceil_div(K, 256)), dim3(256), 0, st, bn.acc, M, K, bn.rm,
                     bn.rv, bn.gamma, bn.beta, bn.momentum, bn.eps, bn.out);
}

// ------------------------------------------------------------ folded BN backward
// DgradFold weights (kernels.h).  Per output channel k of the 1x1 conv (K of them), from its BN
// statistics and backward sums over M rows:
//   k1 = gamma * invstd,  k2 = s1 * invstd^2 / M,  a = -k1 * k2,  b = -k1 * (s0 / M - mean * k2)
// so that the BN-backward apply is dy = k1*g + a*y + b.  With wt[C][K] the transposed weights:
//   wfold[c][0:K]   = bf16(wt[c][k] * k1[k])
//   wfold[c][K + c'] = bf16(G[c][c']),  G = sum_k wt[c][k] * a[k] * wt[c'][k]   (fp32 sums)
//   bias[c]        = sum_k wt[c][k] * b[k]
// One launch: blocks [0, nG) compute 32x32 tiles of G (the tj == 0 column of tiles also the bias of
// their 32 rows), the other nS blocks scale wt.  a[] and b[] are built once per block in LDS; the
// K loop prefetches the next 64-wide chunk into registers while the current one is multiplied.
struct FoldCoef {
  const float* stats;
  const float* gamma;
  const float* sums;
  int K;
  float invM;
  __device__ __forceinline__ void ab(int k, float& a, float& b) const {
    const float is = stats[K + k], mu = stats[k];
    const float k1 = gamma[k] * is;
    const float k2 = sums[K + k] * is * is * invM;
    a = -k1 * k2;
    b = -k1 * (sums[k] * invM - mu * k2);
  }
};

constexpr int kFoldMaxK = 2048;
// bn_act_fwd's column-sum accumulator (CSUM, below): slots and grid cap
constexpr int kCsumSlots = 128, kCsumBlocks = 4096;
typedef __bf16 fold_v8bf __attribute__((ext_vector_type(8)));

// Per-channel coefficients (a, b) of the fold into coef[2][K]: its own tiny launch so that the
// GEMM below needs no LDS -- both then fit on CUs whose LDS the weight-gradient blocks of the side
// stream hold (a kernel that needs LDS waits for one of those long-lived blocks to retire: the
// 16-KB-LDS version of this kernel measured 38 us per call in-step against ~5 us of work).
__global__ void __launch_bounds__(256) bn_fold_coef_kernel(FoldCoef cf, float* __restrict__ coef) {
  __builtin_amdgcn_s_setprio(3);
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k < cf.K) cf.ab(k, coef[k], coef[cf.K + k]);
}

// G tiles on the matrix cores: a 4-wave workgroup per 32 x 32 tile, wave w taking the K quarter w
// (4 waves per CU hide the fragment-load latency the one-wave form was bound by: 38 us at C = 512),
// partial tiles summed through 12 KB of LDS.  Each wave runs K/64 v_mfma_f32_32x32x16_bf16 with
// A = (wt rows c) * a and B = wt rows c', fragments straight from global memory one 64-k batch
// ahead.  Lane l: fragment row l & 31, k = 8 * (l >> 5) .. +7 of each 16-k step; accumulator
// element e: column l & 31, row 8 * (e >> 2) + 4 * (l >> 5) + (e & 3) (G is symmetric, so a
// transposed tile would read the same).  Waves of the first column of tiles also form the bias.
__global__ void __launch_bounds__(256) bn_fold_weights_kernel(const uint16_t* __restrict__ wt, FoldCoef cf,
                                                              const float* __restrict__ coef, int C, int nG,
                                                              uint16_t* __restrict__ wfold,
                                                              float* __restrict__ bias,
                                                              float* __restrict__ part) {
  // on the critical stream, sharing SIMDs with the side stream's weight-gradient waves: ask for
  // issue priority over them
  __builtin_amdgcn_s_setprio(3);
  const int K = cf.K, t = threadIdx.x;
  const int KC = K + C;
  const int bid = blockIdx.x;
  if (bid >= nG) {  // scaled weights: 8 consecutive k of one row per thread
    const int64_t e = ((int64_t)(bid - nG) * 256 + t) * 8;
    if (e >= (int64_t)C * K) return;
    const int c = (int)(e / K), k = (int)(e - (int64_t)c * K);
    f8 v = unpack8(*reinterpret_cast<const uint4*>(wt + e));
    float g8[8], i8[8];
    load8(cf.gamma + k, g8);
    load8(cf.stats + K + k, i8);
#pragma unroll
    for (int q = 0; q < 8; ++q) v.v[q] *= g8[q] * i8[q];
    *reinterpret_cast<uint4*>(wfold + (size_t)c * KC + k) = pack8(v);
    return;
  }
  const int nt = C / 32;
  const int ti = bid / nt, tj = bid - ti * nt;
  const int c0 = ti * 32, d0 = tj * 32;
  const int wv = t >> 6, lane = t & 63;
  const int r = lane & 31, kh = (lane >> 5) * 8;
  const bool with_bias = d0 == 0;
  const int kq = K / 4, kbeg = wv * kq;  // this wave's K quarter (K % 256 == 0)
  const uint16_t* pa = wt + (size_t)(c0 + r) * K + kbeg + kh;
  const uint16_t* pb = wt + (size_t)(d0 + r) * K + kbeg + kh;
  const float* ca_ = coef + kbeg + kh;
  const float* cb_ = coef + K + kbeg + kh;
  v16f acc = {};
  float bacc = 0.f;
  constexpr int B4 = 4;  // 16-k steps per batch
  uint4 xa[B4], xb[B4], ya[B4], yb[B4];
#pragma unroll
  for (int q = 0; q < B4; ++q) {
    xa[q] = *reinterpret_cast<const uint4*>(pa + q * 16);
    xb[q] = *reinterpret_cast<const uint4*>(pb + q * 16);
  }
  for (int k0 = 0; k0 < kq; k0 += 16 * B4) {
    const bool more = k0 + 16 * B4 < kq;
    if (more) {
#pragma unroll
      for (int q = 0; q < B4; ++q) {
        ya[q] = *reinterpret_cast<const uint4*>(pa + k0 + 16 * B4 + q * 16);
        yb[q] = *reinterpret_cast<const uint4*>(pb + k0 + 16 * B4 + q * 16);
      }
    }
#pragma unroll
    for (int q = 0; q < B4; ++q) {
      const int kb = k0 + q * 16;
      float a8[8];
      load8(ca_ + kb, a8);
      f8 fa = unpack8(xa[q]);
      if (with_bias) {
        float b8[8];
        load8(cb_ + kb, b8);
#pragma unroll
        for (int e = 0; e < 8; ++e) bacc = fmaf(fa.v[e], b8[e], bacc);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) fa.v[e] *= a8[e];
      const uint4 qa = pack8(fa);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(fold_v8bf, qa),
                                                    __builtin_bit_cast(fold_v8bf, xb[q]), acc, 0, 0, 0);
    }
    if (more) {
#pragma unroll
      for (int q = 0; q < B4; ++q) { xa[q] = ya[q]; xb[q] = yb[q]; }
    }
  }
  // the K-quarter partials meet in this block's slice of the global scratch `part`, not in LDS: a
  // kernel that declares LDS waits for a CU with that much LDS free, and the side stream's
  // weight-gradient blocks hold 128-160 KB of a CU's 160 KB for their whole K range (the 13-KB-LDS
  // version ran 74-83 us per call in layer 1 against ~10 us of work, r9e).  __syncthreads orders
  // the global stores and loads at workgroup scope.
  float* pw = part + (size_t)bid * (3 * 17 * 64);
  if (wv > 0) {
    float* q = pw + (wv - 1) * (17 * 64);
#pragma unroll
    for (int e = 0; e < 16; ++e) q[e * 64 + lane] = acc[e];
    q[16 * 64 + lane] = bacc;
  }
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float v = acc[e] + pw[e * 64 + lane] + pw[17 * 64 + e * 64 + lane] + pw[34 * 64 + e * 64 + lane];
    const int row = 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
    wfold[(size_t)(c0 + row) * KC + K + d0 + (lane & 31)] = f2bf(v);
  }
  if (with_bias) {
    bacc += pw[16 * 64 + lane] + pw[33 * 64 + lane] + pw[50 * 64 + lane];
    bacc += __shfl_xor(bacc, 32, 64);  // the two k halves of row r
    if (lane < 32) bias[c0 + r] = bacc;
  }
}

// Weight gradient of the folded unit (ops/fused.py DgradFold path): with dy = k1*g + a*y + b and
// y = W x, dW = sum_m dy^T x = diag(k1) T1 + diag(a) W Gram + b (x) colsum, where T1 = g^T x (the
// ordinary weight gradient of g), Gram = x^T x and colsum = sum_m x.  out[k][c] (the flat gradient
// buffer) += that; block 0 also adds dgamma += s1 * invstd, dbeta += s0 (the apply's job before).
// W is the bf16 mirror the forward used (wt[C][K], the transposed copy bn_fold_weights reads), so
// the fold's dW matches apply-then-wgrad exactly up to summation order.
// Blocks: 64x64 tiles of out over (k, c), 4x4 outputs per thread; the K x C x C product W Gram runs
// through LDS in 32-deep q chunks, two ds_read_b128 per 16 FMAs (the 32x32 / 2x2 version was
// LDS-issue bound: ~41 us per call in-step, on the weight-gradient stream that ends the step).
// `done` non-null (consume mode): T1, Gram and the BN-sum accumulator `sums` are persistent
// workspaces the caller never re-zeroes -- every T1 element is cleared by the thread that reads it;
// the last block of each 64-column group (counter done[tc]) clears that group's Gram columns; the
// last group to finish (counter done[nc]) clears sums if `zero_sums` and resets the counters.  No
// memset or fill launch on the weight-gradient stream.
constexpr int kFoldTile = 64;
__global__ void __launch_bounds__(256) bn_fold_wgrad_kernel(float* __restrict__ t1,
                                                            float* __restrict__ gram,
                                                            const float* __restrict__ colsum,
                                                            const uint16_t* __restrict__ wt, FoldCoef cf, int C,
                                                            float* __restrict__ out, float* __restrict__ dgamma,
                                                            float* __restrict__ dbeta, int* __restrict__ done,
                                                            int zero_sums, int csum_slots) {
  const int K = cf.K, t = threadIdx.x;
  const int nc = C / kFoldTile;
  const int tk = blockIdx.x / nc, tc = blockIdx.x - tk * nc;
  const int k0 = tk * kFoldTile, c0 = tc * kFoldTile;
  if (blockIdx.x == 0 && dgamma != nullptr) {
    for (int k = t; k < K; k += 256) {
      const float is = cf.stats[K + k];
      dgamma[k] += cf.sums[K + k] * is;
      dbeta[k] += cf.sums[k];
    }
  }
  __shared__ __attribute__((aligned(16))) float sW[32][kFoldTile];  // W^T chunk: [q][k]
  __shared__ __attribute__((aligned(16))) float sG[32][kFoldTile];  // Gram chunk: [q][c]
  __shared__ float sCs[4][kFoldTile];  // column sums of this block's 64 columns (row 0 after the reduce)
  __shared__ int last;
  {
    const int j = t & (kFoldTile - 1), ph = t >> 6;  // column, slot phase (4 phases)
    float a = 0.f;
    if (csum_slots == 1) {
      if (ph == 0) a = colsum[c0 + j];
    } else {
#pragma unroll 8
      for (int sl = ph; sl < kCsumSlots; sl += 4) a += colsum[(size_t)sl * C + c0 + j];
    }
    sCs[ph][j] = a;
    __syncthreads();
    if (t < kFoldTile) sCs[0][t] = sCs[0][t] + sCs[1][t] + sCs[2][t] + sCs[3][t];
    // (visible to every thread after the first barrier of the K loop below)
  }
  const int ty = t >> 4, tx = t & 15;  // outputs (k0 + 4ty + i, c0 + 4tx + j)
  float acc[4][4] = {};
  for (int q0 = 0; q0 < C; q0 += 32) {
    {  // W: 32 rows q of 64 consecutive k (128 B of bf16): one 16-B load per thread
      const int q = t >> 3, kk = (t & 7) * 8;
      f8 v = unpack8(*reinterpret_cast<const uint4*>(wt + (size_t)(q0 + q) * K + k0 + kk));
      *reinterpret_cast<float4*>(&sW[q][kk]) = make_float4(v.v[0], v.v[1], v.v[2], v.v[3]);
      *reinterpret_cast<float4*>(&sW[q][kk + 4]) = make_float4(v.v[4], v.v[5], v.v[6], v.v[7]);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // Gram: 32 rows q of 64 columns: two float4 per thread
      const int e = t + h * 256, q = e >> 4, cc = (e & 15) * 4;
      *reinterpret_cast<float4*>(&sG[q][cc]) = *reinterpret_cast<const float4*>(gram + (size_t)(q0 + q) * C + c0 + cc);
    }
    __syncthreads();
#pragma unroll 8
    for (int q = 0; q < 32; ++q) {
      const float4 w = *reinterpret_cast<const float4*>(&sW[q][ty * 4]);
      const float4 g = *reinterpret_cast<const float4*>(&sG[q][tx * 4]);
      const float wv[4] = {w.x, w.y, w.z, w.w}, gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(wv[i], gv[j], acc[i][j]);
    }
    __syncthreads();
  }
  // colsum: one [C] vector (a reduction pass), or the forward apply's slots [kCsumSlots][C], summed
  // into sCs by the whole block up front (4 threads per column, unrolled: a per-thread loop over
  // 128 slots ran as 128 dependent L2 round trips, ~90 us per call)
  const float csv[4] = {sCs[0][tx * 4], sCs[0][tx * 4 + 1], sCs[0][tx * 4 + 2], sCs[0][tx * 4 + 3]};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + ty * 4 + i;
    const float is = cf.stats[K + k], mu = cf.stats[k];
    const float k1 = cf.gamma[k] * is;
    const float k2 = cf.sums[K + k] * is * is * cf.invM;
    const float a = -k1 * k2, b = -k1 * (cf.sums[k] * cf.invM - mu * k2);
    const size_t o = (size_t)k * C + c0 + tx * 4;
    float4 tv = *reinterpret_cast<const float4*>(t1 + o);
    float4 ov = *reinterpret_cast<const float4*>(out + o);
    ov.x += k1 * tv.x + a * acc[i][0] + b * csv[0];
    ov.y += k1 * tv.y + a * acc[i][1] + b * csv[1];
    ov.z += k1 * tv.z + a * acc[i][2] + b * csv[2];
    ov.w += k1 * tv.w + a * acc[i][3] + b * csv[3];
    *reinterpret_cast<float4*>(out + o) = ov;
    if (done != nullptr) *reinterpret_cast<float4*>(t1 + o) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (done == nullptr) return;
  // every read of gram / sums by this block has returned (their values are consumed above)
  __syncthreads();
  if (t == 0) {
    __threadfence();
    const int nk = K / kFoldTile;
    int v = atomicAdd(done + tc, 1) == nk - 1 ? 1 : 0;  // last block of column group tc
    if (v) {
      done[tc] = 0;
      __threadfence();
      v = atomicAdd(done + nc, 1) == nc - 1 ? 2 : 1;    // ... and the last group overall
      if (v == 2) done[nc] = 0;
    }
    last = v;
  }
  __syncthreads();
  if (last == 0) return;
  __threadfence();
  for (int e = t; e < C * (kFoldTile / 4); e += 256) {  // this group's Gram columns c0 .. c0+63
    const int q = e >> 4, cc = (e & 15) * 4;
    *reinterpret_cast<float4*>(gram + (size_t)q * C + c0 + cc) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (csum_slots > 1)  // forward-accumulated column sums: this group's columns of every slot
    for (int e = t; e < csum_slots * kFoldTile; e += 256)
      const_cast<float*>(colsum)[(size_t)(e / kFoldTile) * C + c0 + (e % kFoldTile)] = 0.f;
  if (last == 2 && zero_sums) {
    float* sm = const_cast<float*>(cf.sums);
    for (int e = t; e < 2 * K; e += 256) sm[e] = 0.f;
  }
}

void launch_bn_fold_wgrad(float* t1, float* gram, const float* colsum, const uint16_t* wt,
                          const float* stats, const float* gamma, const float* sums, int M, int C, int K,
                          float* out, float* dgamma, float* dbeta, int* done, bool zero_sums, hipStream_t st,
                          int csum_slots) {
  if (C % kFoldTile != 0 || K % kFoldTile != 0)
    throw std::runtime_error("bn_fold_wgrad: needs C % 64 == 0, K % 64 == 0");
  if (csum_slots != 1 && (csum_slots != kCsumSlots || done == nullptr))
    throw std::runtime_error("bn_fold_wgrad: column sums come as 1 vector, or bn_act_fwd's slots in consume mode");
  FoldCoef cf{stats, gamma, sums, K, 1.f / (float)M};
  hipLaunchKernelGGL(bn_fold_wgrad_kernel, dim3((K / kFoldTile) * (C / kFoldTile)), dim3(256), 0, st, t1, gram,
                     colsum, wt, cf, C, out, dgamma, dbeta, done, zero_sums ? 1 : 0, csum_slots);
}

int64_t bn_fold_weights_ws_floats(int C, int K) { return C + 2 * (int64_t)K + (int64_t)(C / 32) * (C / 32) * 3 * 17 * 64; }

void launch_bn_fold_weights(const uint16_t* wt, const float* stats, const float* gamma, const float* sums,
                            int M, int C, int K, uint16_t* wfold, float* bias, hipStream_t st) {
  if (C % 32 != 0 || K % 256 != 0 || K > kFoldMaxK)
    throw std::runtime_error("bn_fold_weights: needs C % 32 == 0, K % 256 == 0, K <= 2048");
  const int nG = (C / 32) * (C / 32);
  const int nS = (int)(((int64_t)C * K / 8 + 255) / 256);
  FoldCoef cf{stats, gamma, sums, K, 1.f / (float)M};
  // scratch after the bias (the caller allocates bn_fold_weights_ws_floats(C, K)): coef [2][K],
  // then the G tiles' cross-wave partials [nG][3][17][64]
  float* coef = bias + C;
  float* part = coef + 2 * K;
  hipLaunchKernelGGL(bn_fold_coef_kernel, dim3(ceil_div(K, 256)), dim3(256), 0, st, cf, coef);
  hipLaunchKernelGGL(bn_fold_weights_kernel, dim3(nG + nS), dim3(256), 0, st, wt, cf, coef, C, nG, wfold, bias,
                     part);
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

// RESBN: the residual is a raw (pre-BN) conv output with its own BatchNorm -- the projection
// shortcut of a downsampling block.  It is normalised here and rounded to bf16 exactly as a
// separate apply pass would have stored it, so the block output is bit-identical to the unfused
// path while the normalised shortcut is never written or read back (2 x |shortcut| of HBM).
// CSUM: also the per-channel column sums of the stored bf16 z, fp32-atomically added into one of
// kCsumSlots slots of csum[kCsumSlots][K] (the folded weight gradient's sum_m x, ops/fused.py
// DgradFold: the unit's output is the next 1x1 conv's input, so its reduction pass on the
// weight-gradient stream -- one 233 us launch at the end of layer 1 -- is gone).  Needs 256 % K8
// == 0.  Same-address fp32 atomics serialise at the memory side (~0.15 us each): with 8 slots and
// 8192 blocks the pass ran 155-204 us instead of 9-33 (r9s), so the grid is capped at
// kCsumBlocks and the blocks spread over kCsumSlots slots (<= 32 atomics per address).
template <bool RES, bool RELU, bool MASK = false, bool RESBN = false, int U = 1, bool CSUM = false>
__global__ void __launch_bounds__(256) bn_act_fwd_kernel(const uint4* __restrict__ y,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         const uint4* __restrict__ res,
                                                         uint4* __restrict__ z, int64_t nvec,
                                                         int K8, uint8_t* __restrict__ zmask = nullptr,
                                                         const float* __restrict__ rscale = nullptr,
                                                         const float* __restrict__ rshift = nullptr,
                                                         float* __restrict__ csum = nullptr) {
  // the grid stride is a multiple of K8 (ew_blocks), so a thread's 8-channel group and its
  // scale/shift are fixed over the loop (no 64-bit modulo and 4 coefficient loads per vector)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(v0 % K8) * 8;
  float sc[8], sh[8], rsc[8], rsh[8], cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = 0.f;
  load8(scale + c0, sc);
  load8(shift + c0, sh);
  if constexpr (RESBN) {
    load8(rscale + c0, rsc);
    load8(rshift + c0, rsh);
  }
  auto body = [&](int64_t v, const uint4 yv, const uint4 rv) {
    f8 a = unpack8(yv);
    f8 r;
    if (RES) r = unpack8(rv);
    if constexpr (RESBN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r.v[j] = bf2f(f2bf(fmaf(r.v[j], rsc[j], rsh[j])));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = fmaf(a.v[j], sc[j], sh[j]);
      if (RES) t += r.v[j];
      if (RELU) t = fmaxf(t, 0.f);
      a.v[j] = t;
    }
    const uint4 zb = pack8(a);
    z[v] = zb;
    if constexpr (CSUM) {
      const f8 zr = unpack8(zb);
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[j] += zr.v[j];
    }
    if constexpr (MASK) {  // bit j = stored bf16 z > 0 (exactly what a z read would test)
      const f8 zr = unpack8(zb);
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) bits |= (zr.v[j] > 0.f ? 1u : 0u) << j;
      zmask[v] = (uint8_t)bits;
    }
  };
  int64_t v = v0;
  if constexpr (U > 1) {
    // U vectors per thread per iteration: every load of the batch is issued before the first
    // store (the compiler cannot hoist a load above a store that may alias it)
    for (; v + (U - 1) * stride < nvec; v += U * stride) {
      uint4 yv[U], rv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        yv[u] = y[v + u * stride];
        if (RES) rv[u] = res[v + u * stride];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) body(v + u * stride, yv[u], RES ? rv[u] : yv[u]);
    }
  }
  for (; v < nvec; v += stride) body(v, y[v], RES ? res[v] : uint4{});
  if constexpr (CSUM) {
    // threads t, t + K8, ... hold the same 8 channels (256 % K8 == 0): sum them in LDS, then one
    // atomic per channel and block into this XCD's slot
    __shared__ float red[256][9];
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = cs[j];
    __syncthreads();
    if ((int)threadIdx.x < K8) {
      float t8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t8[j] = 0.f;
      for (int u = threadIdx.x; u < 256; u += K8)
#pragma unroll
        for (int j = 0; j < 8; ++j) t8[j] += red[u][j];
      float* slot = csum + (size_t)(blockIdx.x % kCsumSlots) * (K8 * 8) + threadIdx.x * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) unsafeAtomicAdd(slot + j, t8[j]);
    }
  }
}

// grid of an 8-channel-vector elementwise pass: at most kEwCap (kEwCapResidual for the residual
// apply) blocks of 256, rounded so that the grid stride (blocks * 256) is a multiple of K8 --
// every thread then keeps one channel group
static int ew_block_cap_env() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PDT_EW_BLOCKS");  // A/B knob: grid cap of every streaming BN pass
    v = e ? std::max(256, atoi(e)) : 0;
  }
  return v;
}

// Grid caps measured per pass on MI355X (round-1 sweep of 4096..32768 blocks): the residual-add
// forward apply (2 reads + 1 write + mask per vector) is fastest with one vector per thread
// (cap 32768: 102 -> 96.5 us per layer2 call), the other passes with 8192.  Capped multi-iteration
// grids are checked against the default in tests/test_tiles_gpu.py (PDT_EW_BLOCKS=256).
constexpr int kEwCap = 8192;
constexpr int kEwCapResidual = 32768;

static int ew_blocks(int64_t nvec, int K8, int cap_default = kEwCap) {
  int64_t b = (nvec + 255) / 256;
  const int64_t cap = ew_block_cap_env() > 0 ? ew_block_cap_env() : cap_default;
  b = b < cap ? b : cap;
  const int64_t q = K8 / std::gcd(K8, 256);
  return (int)(((b + q - 1) / q) * q);
}

template <bool RES, bool RELU, bool MASK, bool RESBN>
static void fwd_launch(dim3 g, dim3 b, hipStream_t st, const uint4* Y, const float* scale, const float* shift,
                       const uint4* R, uint4* Z, int64_t nvec, int K8, uint8_t* zmask = nullptr,
                       const float* rscale = nullptr, const float* rshift = nullptr) {
  hipLaunchKernelGGL((bn_act_fwd_kernel<RES, RELU, MASK, RESBN, 1>), g, b, 0, st, Y, scale, shift, R, Z, nvec, K8,
                     zmask, rscale, rshift);
}

int bn_csum_slots() { return kCsumSlots; }

void launch_bn_act_fwd(const uint16_t* y, const float* scale, const float* shift,
                       const uint16_t* res, bool relu, uint16_t* z, int64_t M, int K,
                       hipStream_t st, uint8_t* zmask, const float* rscale, const float* rshift,
                       float* csum) {
  int64_t nvec = M * K / 8;
  int K8 = K / 8;
  dim3 g(ew_blocks(nvec, K8, res ? kEwCapResidual : kEwCap)), b(256);
  auto Y = reinterpret_cast<const uint4*>(y);
  auto R = reinterpret_cast<const uint4*>(res);
  auto Z = reinterpret_cast<uint4*>(z);
  if (csum != nullptr) {
    if (res || zmask || rscale || !relu || K8 > 256 || 256 % K8 != 0)
      throw std::runtime_error("bn_act_fwd: column sums only on the plain BN+ReLU pass, 256 % (K/8) == 0");
    // >= 8 vectors per thread: the atomics per block are fixed (K per block), so small tensors
    // (layer 4: one vector per thread at the default grid) would be atomic-bound
    const int64_t want = std::max<int64_t>(1, nvec / (256 * 8));
    const dim3 gc(ew_blocks(std::min<int64_t>(nvec, want * 256), K8, kCsumBlocks));
    hipLaunchKernelGGL((bn_act_fwd_kernel<false, true, false, false, 1, true>), gc, b, 0, st, Y, scale, shift,
                       R, Z, nvec, K8, nullptr, nullptr, nullptr, csum);
    return;
  }
  if (rscale != nullptr) {  // residual = BN(raw shortcut conv output), normalised on the fly
    if (!res || !rshift) throw std::runtime_error("bn_act_fwd: residual BN needs the residual and its shift");
    if (zmask) {
      if (!relu) throw std::runtime_error("bn_act_fwd: a ReLU mask needs relu");
      fwd_launch<true, true, true, true>(g, b, st, Y, scale, shift, R, Z, nvec, K8,
                         zmask, rscale, rshift);
    } else if (relu) {
      fwd_launch<true, true, false, true>(g, b, st, Y, scale, shift, R, Z, nvec,
                         K8, nullptr, rscale, rshift);
    } else {
      fwd_launch<true, false, false, true>(g, b, st, Y, scale, shift, R, Z, nvec,
                         K8, nullptr, rscale, rshift);
    }
    return;
  }
  if (zmask) {
    if (!relu) throw std::runtime_error("bn_act_fwd: a ReLU mask needs relu");
    if (res) fwd_launch<true, true, true, false>(g, b, st, Y, scale, shift, R, Z, nvec, K8, zmask);
    else fwd_launch<false, true, true, false>(g, b, st, Y, scale, shift, R, Z, nvec, K8, zmask);
  } else if (res) {
    if (relu) fwd_launch<true, true, false, false>(g, b, st, Y, scale, shift, R, Z, nvec, K8);
    else fwd_launch<true, false, false, false>(g, b, st, Y, scale, shift, R, Z, nvec, K8);
  } else {
    if (relu) fwd_launch<false, true, false, false>(g, b, st, Y, scale, shift, R, Z, nvec, K8);
    else fwd_launch<false, false, false, false>(g, b, st, Y, scale, shift, R, Z, nvec, K8);
  }
}

// ------------------------------------------------------------ backward reduce
// Block (bx, by) reduces rows [bx*RPB, (bx+1)*RPB) of channel chunk by (<= RED_CH8 8-channel
// groups = 256 channels).  Chunking the channels keeps >= 8 rows in flight per iteration and
// gives wide layers (K = 1024/2048 at M = 50176/12544) a grid that fills the chip: with all K
// channels in one block a 2048-channel reduction ran on 49 blocks at ~0.5 TB/s.
constexpr int RED_BLOCKS_MAX = 1024;
constexpr int RED_CH8 = 32;
constexpr int RED_TARGET = 2048;  // blocks per launch (8 per CU)

static int red_chunks(int K) {
  const int K8 = K / 8;
  return K8 > RED_CH8 ? K8 / RED_CH8 : 1;
}

static int red_blocks(int64_t M, int K) {
  const int64_t by_rows = (M + 31) / 32;  // >= 32 rows per block
  int64_t b = (RED_TARGET + red_chunks(K) - 1) / red_chunks(K);
  b = std::max<int64_t>(b, (M + 1023) / 1024);  // <= 1024 rows per block
  b = std::min<int64_t>(std::min<int64_t>(b, by_rows), RED_BLOCKS_MAX);
  return (int)std::max<int64_t>(b, 1);
}

size_t bn_bwd_ws_floats(int64_t M, int K) { return (size_t)red_blocks(M, K) * 2 * K; }

// Relu-mask modes of the backward kernels: 0 = no ReLU, 1 = mask from the saved output z (z > 0),
// 2 = mask recomputed from y (y*scale + shift > 0, bit-identical to the forward's fp32 math) --
// used for units without a residual input so backward never reads z (saves 2 B/element/pass).
template <int MASK>
__device__ __forceinline__ float relu_grad(float g, float zv, float yv, float sc, float sh) {
  if (MASK == 1) return zv > 0.f ? g : 0.f;
  if (MASK == 2) return fmaf(yv, sc, sh) > 0.f ? g : 0.f;
  return g;
}

// Tree sum over the `rpi` threads that share a channel group (thread t = roff * step + c): 16
// values per thread in a value-major LDS image sh[j * 256 + t]; the totals end in the roff == 0
// threads' slots.  256 threads per block.
__device__ __forceinline__ void block_tree_sum16(float* sh, int t, int rpi, int step, const float (&a)[8],
                                                 const float (&b)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[j * 256 + t] = a[j];
    sh[(8 + j) * 256 + t] = b[j];
  }
  __syncthreads();
  const int roff = t / step;
  for (int s = rpi / 2; s > 0; s >>= 1) {
    if (roff < s) {
#pragma unroll
      for (int j = 0; j < 16; ++j) sh[j * 256 + t] += sh[j * 256 + t + s * step];
    }
    __syncthreads();
  }
}

// stats = [4][K]: mean, invstd, scale, shift (bn_finalize output)
template <int MASK>
__global__ void __launch_bounds__(256) bn_bwd_reduce_stage1(const uint4* __restrict__ dz,
                                                            const uint4* __restrict__ z,
                                                            const uint4* __restrict__ y,
                                                            const float* __restrict__ stats,
                                                            int64_t M, int K8,
                                                            float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int K = K8 * 8;
  const int CH8 = K8 < RED_CH8 ? K8 : RED_CH8;  // 8-channel groups of this block's chunk
  const int t = threadIdx.x;
  const int c8 = blockIdx.y * CH8 + t % CH8;
  const int rpi = 256 / CH8;  // rows per iteration
  const int roff = t / CH8;
  int64_t rows_per_block = (M + gridDim.x - 1) / gridDim.x;
  int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t r1 = min(M, r0 + rows_per_block);
  float mu[8], sc[8], shf[8];
  load8(stats + c8 * 8, mu);
  if (MASK == 2) { load8(stats + 2 * K + c8 * 8, sc); load8(stats + 3 * K + c8 * 8, shf); }
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 4
  for (int64_t r = r0 + roff; r < r1; r += rpi) {
    int64_t v = r * K8 + c8;
    f8 d = unpack8(dz[v]);
    f8 yy = unpack8(y[v]);
    f8 zz;
    if (MASK == 1) zz = unpack8(z[v]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = relu_grad<MASK>(d.v[j], MASK == 1 ? zz.v[j] : 0.f, yy.v[j],
                                MASK == 2 ? sc[j] : 0.f, MASK == 2 ? shf[j] : 0.f);
      sg[j] += g;
      sgx[j] = fmaf(g, yy.v[j] - mu[j], sgx[j]);
    }
  }
  // block reduction over threads with equal c8, in a value-major LDS image sh[j][thread]:
  // consecutive lanes hit consecutive banks (the thread-major [thread][16] image cost ~16
  // conflict cycles per LDS instruction, profiles/r2s2_sq_mfma_busy_per_kernel.txt)
  block_tree_sum16(sh, t, rpi, CH8, sg, sgx);
  if (roff == 0) {
    float* o = ws + (int64_t)blockIdx.x * 2 * K;
#pragma unroll
    for (int j = 0; j < 8; ++j) { o[c8 * 8 + j] = sh[j * 256 + t]; o[K + c8 * 8 + j] = sh[(8 + j) * 256 + t]; }
  }
}

// block = CH channels x (256/CH) partial-lanes; each lane sums its share of the nb stage-1
// partials (independent loads, pipelined), then an LDS combine.  Deterministic (fixed order).
// CH = 32 for wide layers; CH = 8 when K/32 blocks would leave most of the chip idle.
template <int CH>
__global__ void __launch_bounds__(256) bn_bwd_reduce_stage2(const float* __restrict__ ws, int nb,
                                                            int K, float* __restrict__ sums,
                                                            const float* __restrict__ invstd,
                                                            float* __restrict__ dgamma,
                                                            float* __restrict__ dbeta) {
  constexpr int L = 256 / CH;
  __shared__ float sa[L][CH + 1], sb[L][CH + 1];
  const int tx = threadIdx.x % CH, ty = threadIdx.x / CH;
  const int k = blockIdx.x * CH + tx;
  float a = 0.f, b = 0.f;
  if (k < K) {
#pragma unroll 4
    for (int i = ty; i < nb; i += L) {
      a += ws[(int64_t)i * 2 * K + k];
      b += ws[(int64_t)i * 2 * K + K + k];
    }
  }
  sa[ty][tx] = a;
  sb[ty][tx] = b;
  __syncthreads();
  if (ty == 0 && k < K) {
    for (int r = 1; r < L; ++r) { a += sa[r][tx]; b += sb[r][tx]; }
    sums[k] = a;       // sum g          (= dbeta)
    sums[K + k] = b;   // sum g*(y-mean) (dgamma = b*invstd)
    if (dgamma != nullptr) {
      dgamma[k] += b * invstd[k];
      dbeta[k] += a;
    }
  }
}

// Partials produced by a BN-fused dgrad: block (32 channels, FIN_GPB groups) sums its groups
// into ws[p][2][K]; the last partition block of a channel tile sums the P partials (fixed order)
// into sums[2][K] and optionally dgamma += b*invstd, dbeta += a.  One launch.
__global__ void __launch_bounds__(256) bn_bwd_part_kernel(const float* __restrict__ part, int G, int K,
                                                          float* __restrict__ ws,
                                                          float* __restrict__ sums,
                                                          const float* __restrict__ invstd,
                                                          float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta, int mode,
                                                          int nparts, int cbase, int gpb) {
  __shared__ float sa[FIN_ROWS][FIN_CH + 1], sb[FIN_ROWS][FIN_CH + 1];
  const int tx = threadIdx.x & (FIN_CH - 1), ty = threadIdx.x / FIN_CH;
  const int k = blockIdx.x * FIN_CH + tx;
  const int g0 = blockIdx.y * gpb;
  const int g1 = min(G, g0 + gpb);
  float a = 0.f, b = 0.f;
  if (mode != 2) {
  if (k < K) {
#pragma unroll 8
    for (int g = g0 + ty; g < g1; g += FIN_ROWS) {
      a += part[((int64_t)g * 2 + 0) * K + k];
      b += part[((int64_t)g * 2 + 1) * K + k];
    }
  }
  sa[ty][tx] = a;
  sb[ty][tx] = b;
  __syncthreads();
  const bool direct = mode == 0 && gridDim.y == 1;  // one partition: finish in place
  if (ty == 0 && k < K) {
    for (int r = 1; r < FIN_ROWS; ++r) { a += sa[r][tx]; b += sb[r][tx]; }
    if (!direct) {
      float* o = ws + (int64_t)blockIdx.y * 2 * K;
      st_wt(o + k, a);
      st_wt(o + K + k, b);
    }
  }
  if (mode == 1) return;
  if (direct) {
    if (ty != 0 || k >= K) return;
  } else if (!last_block_of_tile(cbase + kTileCounters / 2 + blockIdx.x, gridDim.y)) {
    return;
  }
  }
  const bool direct = mode == 0 && gridDim.y == 1;
  const int P = mode == 2 ? nparts : gridDim.y;
  if (!direct) {
  a = 0.f; b = 0.f;
  if (k < K) {
#pragma unroll 8
    for (int p = ty; p < P; p += FIN_ROWS) {
      a += ld_wt(ws + (int64_t)p * 2 * K + k);
      b += ld_wt(ws + (int64_t)p * 2 * K + K + k);
    }
  }
  sa[ty][tx] = a;
  sb[ty][tx] = b;
  __syncthreads();
  if (ty != 0 || k >= K) return;
  for (int r = 1; r < FIN_ROWS; ++r) { a += sa[r][tx]; b += sb[r][tx]; }
  }
  sums[k] = a;
  sums[K + k] = b;
  if (dgamma != nullptr) {
    dgamma[k] += b * invstd[k];
    dbeta[k] += a;
  }
}

size_t bn_bwd_part_ws_floats(int G, int K) { return (size_t)ceil_div(G, fin_gpb(G)) * 2 * K; }

void launch_bn_act_bwd_reduce(const uint16_t* dz, const uint16_t* z, const uint16_t* y,
                              const float* stats, int mask, int64_t M, int K, float* ws,
                              float* sums, float* dgamma, float* dbeta, hipStream_t st) {
  int K8 = K / 8;
  if (K8 > RED_CH8 ? (K8 % RED_CH8 != 0) : (256 % K8 != 0))
    throw std::runtime_error("bn_act_bwd_reduce: channel count not supported");
  int nb = red_blocks(M, K);
  dim3 grid(nb, red_chunks(K));
  size_t shmem = 256 * 16 * sizeof(float);
  auto DZ = reinterpret_cast<const uint4*>(dz);
  auto Z = reinterpret_cast<const uint4*>(z);
  auto Y = reinterpret_cast<const uint4*>(y);
  if (mask == 1)
    hipLaunchKernelGGL(bn_bwd_reduce_stage1<1>, grid, dim3(256), shmem, st, DZ, Z, Y, stats, M, K8, ws);
  else if (mask == 2)
    hipLaunchKernelGGL(bn_bwd_reduce_stage1<2>, grid, dim3(256), shmem, st, DZ, Z, Y, stats, M, K8, ws);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_stage1<0>, grid, dim3(256), shmem, st, DZ, Z, Y, stats, M, K8, ws);
  if (K >= 1024)
    hipLaunchKernelGGL(bn_bwd_reduce_stage2<32>, dim3(ceil_div(K, 32)), dim3(256), 0, st, ws, nb, K,
                       sums, stats + K, dgamma, dbeta);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_stage2<8>, dim3(ceil_div(K, 8)), dim3(256), 0, st, ws, nb, K,
                       sums, stats + K, dgamma, dbeta);
}

// ------------------------------------------------------------- backward apply
// Grid-stride with gridDim*256 a multiple of K/8, so every thread keeps one fixed 8-channel
// group: the per-channel coefficients are computed once per thread, not per element.
// Q8: also dy8 = e5m2(bf16(dy) * s_t) with delayed scaling (fp8_util.h) for an fp8 dgrad
template <int MASK, bool TRAIN, bool DRES, bool Q8 = false, int U = 1>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const uint4* __restrict__ dz, const uint4* __restrict__ z, const uint4* __restrict__ y,
    const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ sums, int64_t nvec, int K8, float invM, uint4* __restrict__ dy,
    uint4* __restrict__ dres, uint2* __restrict__ dy8 = nullptr, float* __restrict__ state = nullptr,
    int slot = 0, float* __restrict__ dgamma = nullptr, float* __restrict__ dbeta = nullptr) {
  const int K = K8 * 8;
  float qs = 1.f, qm = 0.f;
  if constexpr (Q8) {
    qs = delayed_scale<true>(state, slot);
    publish_scale(state, slot, qs);
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(tid % K8) * 8;
  float k1[8], sgm[8], k2[8], mu[8], sc[8], shf[8];
  {
    float is[8], gm[8], s0[8], s1[8];
    load8(stats + K + c0, is);
    load8(gamma + c0, gm);
    load8(stats + c0, mu);
    load8(sums + c0, s0);
    load8(sums + K + c0, s1);
    if (MASK == 2) { load8(stats + 2 * K + c0, sc); load8(stats + 3 * K + c0, shf); }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k1[j] = gm[j] * is[j];
      sgm[j] = s0[j] * invM;                 // mean of g
      k2[j] = s1[j] * is[j] * is[j] * invM;  // mean of g*xhat, divided by std
    }
    // BN parameter gradients from the finished sums (sums accumulated by the producing dgrad's
    // epilogue atomics: no separate reduce launch): one thread per 8-channel group
    if (dgamma != nullptr && tid < K8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        dgamma[c0 + j] += s1[j] * is[j];
        dbeta[c0 + j] += s0[j];
      }
    }
  }
  auto body = [&](int64_t v, const uint4 dv, const uint4 zv, const uint4 yv) {
    f8 d = unpack8(dv);
    f8 zz, yy;
    if (MASK == 1) zz = unpack8(zv);
    if (TRAIN || MASK == 2) yy = unpack8(yv);
    f8 o, gr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = relu_grad<MASK>(d.v[j], MASK == 1 ? zz.v[j] : 0.f, (TRAIN || MASK == 2) ? yy.v[j] : 0.f,
                                MASK == 2 ? sc[j] : 0.f, MASK == 2 ? shf[j] : 0.f);
      gr.v[j] = g;
      o.v[j] = TRAIN ? k1[j] * (g - sgm[j] - (yy.v[j] - mu[j]) * k2[j]) : k1[j] * g;
    }
    const uint4 ob = pack8(o);
    if (!Q8 || dy != nullptr) dy[v] = ob;  // Q8 with dy null: fp8-only dy (every consumer reads dy8)
    if (DRES) dres[v] = pack8(gr);
    if constexpr (Q8) {
      const f8 r = unpack8(ob);  // quantize exactly the bf16 dy the weight gradient reads
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        qm = fmaxf(qm, fabsf(r.v[j]));
        t[j] = r.v[j] * qs;
      }
      dy8[v] = make_uint2(cvt4_e5m2(t[0], t[1], t[2], t[3]), cvt4_e5m2(t[4], t[5], t[6], t[7]));
    }
  };
  constexpr bool RZ = MASK == 1, RY = TRAIN || MASK == 2;
  int64_t v = tid;
  if constexpr (U > 1) {  // U vectors of every operand in flight before the first store
    for (; v + (U - 1) * stride < nvec; v += U * stride) {
      uint4 dv[U], zv[U], yv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        dv[u] = dz[v + u * stride];
        if (RZ) zv[u] = z[v + u * stride];
        if (RY) yv[u] = y[v + u * stride];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) body(v + u * stride, dv[u], RZ ? zv[u] : dv[u], RY ? yv[u] : dv[u]);
    }
  }
  for (; v < nvec; v += stride) body(v, dz[v], RZ ? z[v] : uint4{}, RY ? y[v] : uint4{});
  if constexpr (Q8) block_amax(qm, state + slot * SLOT_FLOATS);
}

void launch_bn_act_bwd_apply(const uint16_t* dz, const uint16_t* z, const uint16_t* y,
                             const float* stats, const float* gamma, const float* sums, int mask,
                             bool training, int64_t M, int K, uint16_t* dy, uint16_t* dres,
                             hipStream_t st, float* dgamma, float* dbeta) {
  int64_t nvec = M * K / 8;
  int K8 = K / 8;
  dim3 g(ew_blocks(nvec, K8)), b(256);
  auto DZ = reinterpret_cast<const uint4*>(dz);
  auto Z = reinterpret_cast<const uint4*>(z);
  auto Y = reinterpret_cast<const uint4*>(y);
  auto DY = reinterpret_cast<uint4*>(dy);
  auto DR = reinterpret_cast<uint4*>(dres);
  float invM = 1.f / (float)M;
#define PDT_BWD_U(MK, TR, DRS, UU)                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<MK, TR, DRS, false, UU>), g, b, 0, st, DZ, Z, Y, stats, gamma, \
                     sums, nvec, K8, invM, DY, DR, nullptr, nullptr, 0, dgamma, dbeta)
#define PDT_BWD(MK, TR, DRS) PDT_BWD_U(MK, TR, DRS, 1)
#define PDT_BWD_T(MK)                                                             \
  if (training) { if (dres) PDT_BWD(MK, true, true); else PDT_BWD(MK, true, false); } \
  else { if (dres) PDT_BWD(MK, false, true); else PDT_BWD(MK, false, false); }
  if (mask == 1) { PDT_BWD_T(1) }
  else if (mask == 2) { PDT_BWD_T(2) }
  else { PDT_BWD_T(0) }
#undef PDT_BWD_T
#undef PDT_BWD
#undef PDT_BWD_U
}

void launch_bn_act_bwd_apply_q8(const uint16_t* dz, const uint16_t* z, const uint16_t* y,
                                const float* stats, const float* gamma, const float* sums, int mask,
                                bool training, int64_t M, int K, uint16_t* dy, uint16_t* dres,
                                uint8_t* dy8, float* state, int slot, hipStream_t st, float* dgamma,
                                float* dbeta) {
  if (!training) throw std::runtime_error("bn_act_bwd_apply_q8: training mode only");
  int64_t nvec = M * K / 8;
  int K8 = K / 8;
  int64_t b = (nvec + 255) / 256;
  dim3 g((unsigned)(b < 4096 ? b : 4096)), blk(256);  // multiple of K8: 256 % K8 == 0 (checked by binding)
  auto DZ = reinterpret_cast<const uint4*>(dz);
  auto Z = reinterpret_cast<const uint4*>(z);
  auto Y = reinterpret_cast<const uint4*>(y);
  auto DY = reinterpret_cast<uint4*>(dy);
  auto DR = reinterpret_cast<uint4*>(dres);
  auto D8 = reinterpret_cast<uint2*>(dy8);
  float invM = 1.f / (float)M;
#define PDT_BWDQ(MK, DRS)                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<MK, true, DRS, true>), g, blk, 0, st, DZ, Z, Y, stats, \
                     gamma, sums, nvec, K8, invM, DY, DR, D8, state, slot, dgamma, dbeta)
  if (mask == 1) { if (dres) PDT_BWDQ(1, true); else PDT_BWDQ(1, false); }
  else if (mask == 2) { if (dres) PDT_BWDQ(2, true); else PDT_BWDQ(2, false); }
  else { if (dres) PDT_BWDQ(0, true); else PDT_BWDQ(0, false); }
#undef PDT_BWDQ
}

void launch_bn_bwd_part_reduce(const float* part, int G, int K, float* ws, float* sums,
                               const float* invstd, float* dgamma, float* dbeta, hipStream_t st) {
  const int gpb = fin_gpb(G);
  const int P = ceil_div(G, gpb);
  if (ceil_div(K, FIN_CH) > kTileCounters / 2) throw std::runtime_error("bn reduce: too many channels");
  const int bank = (bn_lastblock() && P > 1) ? counter_bank(st) : 0;
  if (bn_lastblock() && bank >= 0) {
    hipLaunchKernelGGL(bn_bwd_part_kernel, dim3(ceil_div(K, FIN_CH), P), dim3(256), 0, st, part, G, K, ws,
                       sums, invstd, dgamma, dbeta, 0, P, bank, gpb);
  } else {
    hipLaunchKernelGGL(bn_bwd_part_kernel, dim3(ceil_div(K, FIN_CH), P), dim3(256), 0, st, part, G, K, ws,
                       sums, invstd, dgamma, dbeta, 1, P, 0, gpb);
    hipLaunchKernelGGL(bn_bwd_part_kernel, dim3(ceil_div(K, FIN_CH), 1), dim3(256), 0, st, part, G, K, ws,
                       sums, invstd, dgamma, dbeta, 2, P, 0, gpb);
  }
}


// ---------------------------------------------- stem: BN + ReLU + 3x3/s2/p1 max pool, fused
// Forward: every window element is normalised, ReLU'd and rounded to bf16 exactly as bn_act_fwd
// would store it, then max-pooled in registers (same first-maximum tie rule as maxpool_fwd):
// the full-resolution z (411 MB at batch 256) is never written nor read back.  Backward: the
// pooled gradient is gathered back to the full-resolution position inside the BN reduction and
// apply passes (pool_grad8, the maxpool_bwd gather), so dz is never materialised either.
// The ReLU mask is recomputed from y (mode 2).  Requires K8 <= 32 and 256 % K8 == 0.
__device__ __forceinline__ float bf16_round(float x) { return bf2f(f2bf(x)); }

// pool_grad_quad / quad_coords: pool_quad.h (shared with the fused stem weight gradient)

__global__ void __launch_bounds__(256) bn_relu_maxpool_kernel(const uint4* __restrict__ y,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              uint4* __restrict__ out,
                                                              uint2* __restrict__ idx,
                                                              uint4* __restrict__ uarg, uint32_t total,
                                                              int H, int W, int lc8, int Ho, int Wo) {
  // XCD-contiguous block order: the output rows one XCD pools in turn share their input rows
  // (stride 2, window 3) in that XCD's L2, instead of every row pair straddling two XCDs
  const uint32_t t = (uint32_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int C8 = 1 << lc8;
  const int c8 = (int)(t & (uint32_t)(C8 - 1));
  int n, ho, wo;
  quad_coords(t >> lc8, Ho, Wo, n, ho, wo);
  float sc[8], sh[8];
  load8(scale + c8 * 8, sc);
  load8(shift + c8 * 8, sh);
  float best[8], ub[8];
  uint32_t bi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; ub[j] = 0.f; }
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int h = ho * 2 - 1 + kh;
    if (h < 0 || h >= H) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int w = wo * 2 - 1 + kw;
      if (w < 0 || w >= W) continue;
      const f8 v = unpack8(y[(((int64_t)n * H + h) * W + w) * C8 + c8]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float z = bf16_round(fmaxf(fmaf(v.v[j], sc[j], sh[j]), 0.f));
        if (z > best[j] || __builtin_isnan(z)) { best[j] = z; bi[j] = (uint32_t)(kh * 3 + kw); ub[j] = v.v[j]; }
      }
    }
  }
  f8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.v[j] = best[j];
  out[t] = pack8(o);
  idx[t] = make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                      bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
  if (uarg != nullptr) {  // the pre-BN value at the argmax (bf16-exact: a copy of y's element)
    f8 u;
#pragma unroll
    for (int j = 0; j < 8; ++j) u.v[j] = ub[j];
    uarg[t] = pack8(u);
  }
}

// stage 1 of the stem BN backward reduction, dz gathered per quad from the pooled gradient
__global__ void __launch_bounds__(256) pool_bn_bwd_reduce_kernel(const uint4* __restrict__ dp,
                                                                 const uint2* __restrict__ idx,
                                                                 const uint4* __restrict__ y,
                                                                 const float* __restrict__ stats,
                                                                 int NQ, int K8, int H, int W,
                                                                 int Ho, int Wo, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int K = K8 * 8;
  const int t = threadIdx.x;
  const int c8 = t % K8;
  const int rpi = 256 / K8;
  const int roff = t / K8;
  const int per_block = (NQ + (int)gridDim.x - 1) / (int)gridDim.x;
  const int q0 = (int)blockIdx.x * per_block;
  const int q1 = min(NQ, q0 + per_block);
  float mu[8], sc[8], shf[8];
  load8(stats + c8 * 8, mu);
  load8(stats + 2 * K + c8 * 8, sc);
  load8(stats + 3 * K + c8 * 8, shf);
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int qd = q0 + roff; qd < q1; qd += rpi) {
    int n, a, b;
    quad_coords((uint32_t)qd, Ho, Wo, n, a, b);
    // the quad's 4 y vectors are issued first: they do not depend on the argmax gather below (an
    // odd-edge pixel reads its clamped neighbour and is skipped)
    uint4 yv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int h = min(2 * a + (e >> 1), H - 1), w = min(2 * b + (e & 1), W - 1);
      yv[e] = y[(((int64_t)n * H + h) * W + w) * K8 + c8];
    }
    const PoolQuad pq = pool_grad_quad(dp, idx, n, a, b, c8, K8, Ho, Wo);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int h = 2 * a + (e >> 1), w = 2 * b + (e & 1);
      if (h >= H || w >= W) continue;
      const f8 yy = unpack8(yv[e]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = relu_grad<2>(pq.g[e].v[j], 0.f, yy.v[j], sc[j], shf[j]);
        sg[j] += g;
        sgx[j] = fmaf(g, yy.v[j] - mu[j], sgx[j]);
      }
    }
  }
  block_tree_sum16(sh, t, rpi, K8, sg, sgx);  // value-major LDS image: conflict-free
  if (roff == 0) {
    float* o = ws + (int64_t)blockIdx.x * 2 * K;
#pragma unroll
    for (int j = 0; j < 8; ++j) { o[c8 * 8 + j] = sh[j * 256 + t]; o[K + c8 * 8 + j] = sh[(8 + j) * 256 + t]; }
  }
}

template <bool TRAIN>
__global__ void __launch_bounds__(256) pool_bn_bwd_apply_kernel(
    const uint4* __restrict__ dp, const uint2* __restrict__ idx, const uint4* __restrict__ y,
    const float* __restrict__ stats, const float* __restrict__ gamma, const float* __restrict__ sums,
    int nvq, int K8, int H, int W, int Ho, int Wo, float invM, uint4* __restrict__ dy) {
  const int K = K8 * 8;
  const int stride = (int)(gridDim.x * blockDim.x);
  const int tid = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int c8 = tid % K8;
  const int c0 = c8 * 8;
  float k1[8], sgm[8], k2[8], mu[8], sc[8], shf[8];
  {
    float is[8], gm[8], s0[8], s1[8];
    load8(stats + K + c0, is);
    load8(gamma + c0, gm);
    load8(stats + c0, mu);
    load8(sums + c0, s0);
    load8(sums + K + c0, s1);
    load8(stats + 2 * K + c0, sc);
    load8(stats + 3 * K + c0, shf);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k1[j] = gm[j] * is[j];
      sgm[j] = s0[j] * invM;
      k2[j] = s1[j] * is[j] * is[j] * invM;
    }
  }
  for (int v = tid; v < nvq; v += stride) {
    int n, a, b;
    quad_coords((uint32_t)(v / K8), Ho, Wo, n, a, b);
    const PoolQuad pq = pool_grad_quad(dp, idx, n, a, b, c8, K8, Ho, Wo);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int h = 2 * a + (e >> 1), w = 2 * b + (e & 1);
      if (h >= H || w >= W) continue;
      const int64_t off = (((int64_t)n * H + h) * W + w) * K8 + c8;
      const f8 yy = unpack8(y[off]);
      f8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = relu_grad<2>(pq.g[e].v[j], 0.f, yy.v[j], sc[j], shf[j]);
        o.v[j] = TRAIN ? k1[j] * (g - sgm[j] - (yy.v[j] - mu[j]) * k2[j]) : k1[j] * g;
      }
      dy[off] = pack8(o);
    }
  }
}

static void check_pool_bn_channels(int K) {
  const int K8 = K / 8;
  if (K % 8 != 0 || K8 > 32 || 256 % K8 != 0)
    throw std::runtime_error("fused BN + max pool: channels must be 8..256 and divide 2048");
}

static int log2_exact(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

void launch_bn_relu_maxpool(const uint16_t* y, const float* scale, const float* shift, uint16_t* out,
                            uint8_t* idx, uint16_t* uarg, int N, int H, int W, int C, int Ho, int Wo,
                            hipStream_t st) {
  check_pool_bn_channels(C);
  const int C8 = C / 8;
  const int64_t total = (int64_t)N * Ho * Wo * C8;
  if ((int64_t)N * H * W * C8 >= (int64_t)1 << 31) throw std::runtime_error("bn_relu_maxpool: tensor too large");
  hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(y), scale, shift, reinterpret_cast<uint4*>(out),
                     reinterpret_cast<uint2*>(idx), reinterpret_cast<uint4*>(uarg), (uint32_t)total, H, W,
                     log2_exact(C8), Ho, Wo);
}

// The stem's fused pool/BN reduction gathers each 2x2 quad's pooled gradient (dependent loads)
// before its y loads, so it needs more blocks in flight than the plain reduction to reach HBM
// rate: up to 4096 (16 per CU requested; ~2.1 TB/s with the plain reduction's 1024).
constexpr int POOL_RED_BLOCKS = 4096;
static int pool_red_blocks(int NQ) { return std::max(1, std::min(POOL_RED_BLOCKS, NQ / 8)); }
size_t pool_bn_bwd_ws_floats(int64_t M, int K) {
  return std::max(bn_bwd_ws_floats(M, K), (size_t)POOL_RED_BLOCKS * 2 * K);
}

void launch_pool_bn_bwd_reduce(const uint16_t* dpool, const uint8_t* idx, const uint16_t* y,
                               const float* stats, int N, int H, int W, int K, int Ho, int Wo,
                               float* ws, float* sums, float* dgamma, float* dbeta, hipStream_t st) {
  check_pool_bn_channels(K);
  const int K8 = K / 8;
  const int64_t M = (int64_t)N * H * W;
  if (M * K8 >= (int64_t)1 << 31) throw std::runtime_error("pool_bn_bwd_reduce: tensor too large");
  const int NQ = N * Ho * Wo;
  const int nb = pool_red_blocks(NQ);  // <= pool_bn_bwd_ws_floats(M, K) rows
  hipLaunchKernelGGL(pool_bn_bwd_reduce_kernel, dim3(nb), dim3(256), 256 * 16 * sizeof(float), st,
                     reinterpret_cast<const uint4*>(dpool), reinterpret_cast<const uint2*>(idx),
                     reinterpret_cast<const uint4*>(y), stats, NQ, K8, H, W, Ho, Wo, ws);
  hipLaunchKernelGGL(bn_bwd_reduce_stage2<8>, dim3(ceil_div(K, 8)), dim3(256), 0, st, ws, nb, K, sums,
                     stats + K, dgamma, dbeta);
}

void launch_pool_bn_bwd_apply(const uint16_t* dpool, const uint8_t* idx, const uint16_t* y,
                              const float* stats, const float* gamma, const float* sums, bool training,
                              int N, int H, int W, int K, int Ho, int Wo, uint16_t* dy, hipStream_t st) {
  check_pool_bn_channels(K);
  const int K8 = K / 8;
  const int64_t M = (int64_t)N * H * W;
  if (M * K8 >= (int64_t)1 << 31) throw std::runtime_error("pool_bn_bwd_apply: tensor too large");
  const int nvq = N * Ho * Wo * K8;
  dim3 g(ew_blocks(nvq, K8)), b(256);  // ew_blocks * 256 is a multiple of K8
  const float invM = 1.f / (float)M;
  auto DP = reinterpret_cast<const uint4*>(dpool);
  auto ID = reinterpret_cast<const uint2*>(idx);
  auto Y = reinterpret_cast<const uint4*>(y);
  auto DY = reinterpret_cast<uint4*>(dy);
  if (training)
    hipLaunchKernelGGL(pool_bn_bwd_apply_kernel<true>, g, b, 0, st, DP, ID, Y, stats, gamma, sums, nvq,
                       K8, H, W, Ho, Wo, invM, DY);
  else
    hipLaunchKernelGGL(pool_bn_bwd_apply_kernel<false>, g, b, 0, st, DP, ID, Y, stats, gamma, sums, nvq,
                       K8, H, W, Ho, Wo, invM, DY);
}

}  // namespace pdt
