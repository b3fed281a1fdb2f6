// Classifier GEMMs of the ResNet head (torchvision fc: Linear(2048 -> 1000), resnet/main.py:76),
// forward and both backward products, on the bf16 MFMA with fp32 accumulation.
//
//   forward   logits[N][V]  = pooled[N][C] . W[V][C]^T + b          (A, B both k-contiguous)
//   dgrad     dpooled[N][C] = dlogits[N][V] . W[V][C]               (B k-strided)
//   wgrad     dW[V][C]     += dlogits[N][V]^T . pooled[N][C]        (A and B k-strided)
//   bias      db[V]        += sum_n dlogits[n][v]
//
// One kernel for all three: C(m, n) = alpha * sum_k A(m, k) B(k, n) with element strides for
// every operand axis, so no transpose is ever materialised.  The shapes are small (~1 GFLOP
// each at batch 256): a 64x64 workgroup tile of four 32x32 wave tiles, fragments loaded straight
// from global memory (L2-resident operands; no LDS round trip, no barriers), fp32 -> bf16 on the
// load, and split-K over blockIdx.z so every product launches ~256 workgroups.  Split partials go
// to a workspace and are summed in a fixed order by the consumer (deterministic): the forward
// reduce also adds the bias, the avg-pool backward sums the dgrad partials itself.  `alpha` is a
// device scalar (the upstream loss gradient), so no elementwise rescale kernel runs either.
#include "common.h"
#include "kernels.h"

#include <stdexcept>

namespace pdt {

typedef __bf16 fc_v8bf __attribute__((ext_vector_type(8)));

// LDS image of one operand tile: [64 rows][32 k] bf16, 80-byte row pitch (64 B + 16 B pad: the
// 16 lanes of a fragment read hit 16 different 16-byte bank slots), and the 16-B k-chunk of row r
// stored at chunk ^ ((r >> 4) & 3): constant over a fragment's 16 rows (reads unchanged), but the
// transposing store of a k-strided operand -- 8 row groups x 4 dwords per wave instruction, whose
// unswizzled rows 8 apart all fell on 2 bank offsets (4-way conflicts, 10-12 conflict cycles per
// LDS instruction measured, profiles/r2s2_sq_mfma_busy_per_kernel.txt) -- now hits 32 distinct banks
constexpr int FC_PITCH = 80;
constexpr int FC_TILE_BYTES = 64 * FC_PITCH;
__device__ __forceinline__ int fc_off(int row, int chunk) { return row * FC_PITCH + ((chunk ^ ((row >> 4) & 3)) << 4); }

// Global -> register stage of one operand tile (64 rows x 32 k, fp32): 8 values per thread.
// KC (k-contiguous): thread t holds row t/4, k 8*(t%4)..+7 (two 16-byte loads);
// otherwise (row-contiguous): k = t/8, rows 8*(t%8)..+7 (two 16-byte loads along the rows).
template <bool KC>
struct FcStage {
  float v[8];
  __device__ __forceinline__ void load(const float* __restrict__ base, int64_t s_row, int64_t s_k, int row0,
                                       int rows, int k0, int kend, bool vec) {
    const int t = threadIdx.x;
    if (KC) {
      const int r = row0 + t / 4, k = k0 + (t % 4) * 8;
      const float* p = base + (int64_t)r * s_row + k;
      if (vec && r < rows && k + 8 <= kend) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (r < rows && k + j < kend) ? p[j] : 0.f;
      }
    } else {
      const int k = k0 + t / 8, r = row0 + (t % 8) * 8;
      const float* p = base + (int64_t)k * s_k + r;
      if (vec && k < kend && r + 8 <= rows) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (k < kend && r + j < rows) ? p[j] : 0.f;
      }
    }
  }
  __device__ __forceinline__ void store(char* lds) const {
    const int t = threadIdx.x;
    if (KC) {
      fc_v8bf f;
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = (__bf16)v[j];
      *reinterpret_cast<fc_v8bf*>(lds + fc_off(t / 4, t % 4)) = f;
    } else {
      const int k = t / 8, r = (t % 8) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<__bf16*>(lds + fc_off(r + j, k >> 3) + (k & 7) * 2) = (__bf16)v[j];
    }
  }
  __device__ __forceinline__ void add_rows(float (&rs)[8]) const {  // row-contiguous stage only
#pragma unroll
    for (int j = 0; j < 8; ++j) rs[j] += v[j];
  }
};

// AK / BK: A / B is k-contiguous.  Both operands are staged through LDS as [row][k] bf16 (the
// k-strided one transposed on the way in), the next K-step's global loads are issued before the
// current step's MFMAs.  ROWSUM (dW launch): the workgroups of the first column tile also sum
// A's rows in fp32 -- the bias gradient db[v] = sum_n dlogits[n][v] comes out of the same pass.
template <bool AK, bool BK, bool ROWSUM>
__global__ void __launch_bounds__(256) fc_gemm_kernel(const FcArgs p) {
  static_assert(!(ROWSUM && AK), "row sums are taken from the row-contiguous A stage");
  __shared__ __attribute__((aligned(16))) char lds[2 * FC_TILE_BYTES];
  char* As = lds;
  char* Bs = lds + FC_TILE_BYTES;
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int wm = wid & 1, wn = wid >> 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int kbeg = blockIdx.z * p.kper;
  const int kend = min(p.K, kbeg + p.kper);
  // 16-byte loads need every loaded run 16-byte aligned: rows (KC) or k-rows (row-contiguous)
  const bool aligned_a = (reinterpret_cast<uintptr_t>(p.a) & 15) == 0;
  const bool aligned_b = (reinterpret_cast<uintptr_t>(p.b) & 15) == 0;
  const bool avec = aligned_a && (AK ? (p.sam % 4 == 0) : (p.sak % 4 == 0));
  const bool bvec = aligned_b && (BK ? (p.sbn % 4 == 0) : (p.sbk % 4 == 0));
  const bool rows_sum = ROWSUM && blockIdx.x == 0;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // fp32 partial row sums of A (ROWSUM)
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  FcStage<AK> sa;
  FcStage<BK> sb;
  sa.load(p.a, p.sam, p.sak, m0, p.M, kbeg, kend, avec);
  sb.load(p.b, p.sbn, p.sbk, n0, p.N, kbeg, kend, bvec);
  for (int k0 = kbeg; k0 < kend; k0 += 32) {
    __syncthreads();  // previous step's fragment reads done
    sa.store(As);
    sb.store(Bs);
    if constexpr (ROWSUM && !AK) {
      if (rows_sum) sa.add_rows(rs);
    }
    __syncthreads();
    if (k0 + 32 < kend) {  // next step's global loads overlap this step's MFMAs
      sa.load(p.a, p.sam, p.sak, m0, p.M, k0 + 32, kend, avec);
      sb.load(p.b, p.sbn, p.sbk, n0, p.N, k0 + 32, kend, bvec);
    }
    v4i af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      af[i] = *reinterpret_cast<const v4i*>(As + fc_off(wm * 32 + i * 16 + fr, fq));
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bfr[j] = *reinterpret_cast<const v4i*>(Bs + fc_off(wn * 32 + j * 16 + fr, fq));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(fc_v8bf, af[i]),
                                                           __builtin_bit_cast(fc_v8bf, bfr[j]), acc[i][j], 0, 0, 0);
  }
  const float alpha = p.alpha ? p.alpha[0] : 1.f;
  if constexpr (ROWSUM && !AK) {
    if (rows_sum) {  // workgroup-uniform: every thread reaches both barriers
      // thread (k-row t/8, rows 8*(t%8)..+7) holds partial sums over its k's: [32][64] in LDS,
      // then row r = column r summed over the 32 k-rows in fixed order
      __syncthreads();
      float* part = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int j = 0; j < 8; ++j) part[(t / 8) * 64 + (t % 8) * 8 + j] = rs[j];
      __syncthreads();
      if (t < 64 && m0 + t < p.M) {
        float v = 0.f;
        for (int k = 0; k < 32; ++k) v += part[k * 64 + t];
        v *= alpha;
        p.db[m0 + t] = p.accumulate ? p.db[m0 + t] + v : v;
      }
    }
  }
  // lane (fq, fr), register e of acc[i][j]: C[m0 + wm*32 + i*16 + fq*4 + e][n0 + wn*32 + j*16 + fr]
  float* out = p.splits > 1 ? p.ws + (int64_t)blockIdx.z * p.M * p.N : p.c;
  const int64_t ld = p.splits > 1 ? p.N : p.ldc;
  const bool acc_out = p.splits == 1 && p.accumulate;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + fr;
      if (n >= p.N) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 32 + i * 16 + fq * 4 + e;
        if (m >= p.M) continue;
        float v = acc[i][j][e] * alpha;
        if (p.splits == 1 && p.bias) v += p.bias[n];
        float* dst = out + (int64_t)m * ld + n;
        *dst = acc_out ? *dst + v : v;
      }
    }
}

// c[m][n] = sum_s ws[s][m][n] (+ bias[n]), fixed order
__global__ void __launch_bounds__(256) fc_splitk_reduce_kernel(const float* __restrict__ ws, int splits,
                                                               int M, int N, const float* __restrict__ bias,
                                                               float* __restrict__ c, int ldc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
  float v = bias ? bias[n] : 0.f;
  for (int s = 0; s < splits; ++s) v += ws[(int64_t)s * M * N + i];
  c[(int64_t)m * ldc + n] = v;
}

// db[v] (+)= alpha * sum_n g[n][v]: one thread per column, rows summed in order (deterministic)
__global__ void __launch_bounds__(256) fc_colsum_kernel(const float* __restrict__ g, int rows, int cols,
                                                        const float* __restrict__ alpha, float* __restrict__ db,
                                                        int accumulate) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= cols) return;
  float s = 0.f;
  for (int n = 0; n < rows; ++n) s += g[(int64_t)n * cols + v];
  s *= alpha ? alpha[0] : 1.f;
  db[v] = accumulate ? db[v] + s : s;
}

int fc_splits(int M, int N, int K) {
  const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
  int s = 1;
  while (tiles * s < 256 && K / (s * 2) >= 256) s *= 2;  // >= 256 k per slice
  return s;
}

void launch_fc_gemm(const FcArgs& a, hipStream_t st) {
  if (a.splits > 1 && a.ws == nullptr) throw std::runtime_error("fc_gemm: split-K needs a workspace");
  if (a.db && (a.splits != 1 || a.sak == 1)) throw std::runtime_error("fc_gemm: db needs splits 1 and a row-contiguous A");
  if ((a.sak != 1 && a.sam != 1) || (a.sbk != 1 && a.sbn != 1))
    throw std::runtime_error("fc_gemm: every operand must be contiguous along k or along its rows");
  // (misaligned operands -- e.g. a flat-buffer view at an odd offset -- take the scalar loads)
  dim3 g((a.N + 63) / 64, (a.M + 63) / 64, a.splits);
  const bool ak = a.sak == 1, bk = a.sbk == 1;
  if (a.db) hipLaunchKernelGGL((fc_gemm_kernel<false, false, true>), g, dim3(256), 0, st, a);
  else if (ak && bk) hipLaunchKernelGGL((fc_gemm_kernel<true, true, false>), g, dim3(256), 0, st, a);
  else if (ak) hipLaunchKernelGGL((fc_gemm_kernel<true, false, false>), g, dim3(256), 0, st, a);
  else if (bk) hipLaunchKernelGGL((fc_gemm_kernel<false, true, false>), g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((fc_gemm_kernel<false, false, false>), g, dim3(256), 0, st, a);
}

void launch_fc_splitk_reduce(const float* ws, int splits, int M, int N, const float* bias, float* c,
                             int ldc, hipStream_t st) {
  const int64_t n = (int64_t)M * N;
  hipLaunchKernelGGL(fc_splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ws, splits,
                     M, N, bias, c, ldc);
}

void launch_fc_colsum(const float* g, int rows, int cols, const float* alpha, float* db, bool accumulate,
                      hipStream_t st) {
  hipLaunchKernelGGL(fc_colsum_kernel, dim3((cols + 255) / 256), dim3(256), 0, st, g, rows, cols, alpha, db,
                     accumulate ? 1 : 0);
}

}  // namespace pdt
