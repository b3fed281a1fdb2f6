// ResNet stem forward (7x7 / stride 2 / pad 3, 3 input channels -> 64) as a halo-staged implicit
// GEMM on the bf16 MFMA.
//
// The image is first re-laid out as "super-pixels" (layout.hip, launch_stem_image): pairs of
// horizontally adjacent pixels form one 8-channel pixel, so the 7x7/s2 filter becomes 7 rows x 4
// super-pixel taps of 8 channels, stride (2, 1): K_gemm = 7*4*8 = 224.  The generic NT kernel
// gathers that im2col matrix through LDS-DMA one 16-byte tap at a time: every input super-pixel is
// fetched ~14 times (7 rows x 4 taps / stride 2), about 2 GB of L2->LDS traffic per step at batch
// 256, and the stem ran at 267 us against a ~95 us HBM floor (profiles/r3a_step_calls.txt).
//
// Here a workgroup of ROWS waves owns ROWS consecutive output rows of one image (wave w = row
// ho0 + w, all Wo pixels, all 64 channels).  It stages ONCE the 2*ROWS+5 input super-pixel rows
// those outputs read -- one contiguous span of the image, copied by LDS-DMA -- plus the packed
// weights, and every tap's MFMA operand is a shifted ds_read_b128 view of the staged rows:
//   B operand (pixels): lane (pixel fr, k-group fq) of tap row r reads super-pixel (2w + r, wo + fq)
//   A operand (weights): lane (channel fr, k-group fq) reads wsp[ch][r][fq][0..7]
// so K-step r (32 of K) is one filter row, k-group fq one super-pixel tap.  Consecutive pixels of
// a fragment read consecutive 16-byte LDS slots (conflict-free); the weight image is padded to a
// 464-byte row pitch, which spreads its 16 fragment rows over 16 distinct slots.
//
// Epilogue: BN statistics per output row (sum and M2 about the row mean, two passes over the
// fp32 accumulators -- no cancellation), one partial group per (image, output row), and the bf16
// output written as 8-byte channel quads.
#include "common.h"
#include "kernels.h"
#include "pool_quad.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace pdt {

namespace {

constexpr int STEM_K = 64;          // output channels
constexpr int STEM_R = 7;           // filter rows
constexpr int STEM_SP = 4;          // super-pixel taps per row
constexpr int STEM_ROWS = 4;        // output rows (= waves) per workgroup
constexpr int W_PITCH = 464;        // bytes per packed weight row in LDS (448 + 16 pad)
constexpr int W_BYTES = STEM_K * W_PITCH;
constexpr uint32_t OOB = 0x80000000u;

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)(reinterpret_cast<uintptr_t>(lds)), 16, voff, 0, 0, 0);
}

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

__device__ __forceinline__ v4f mfma16(const v4i& a, const v4i& b, const v4f& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c,
                                                0, 0, 0);
}

struct StemArgs {
  const uint16_t* xsp;   // [N][Hp][Wsp][8]
  const uint16_t* wsp;   // [64][7][4][8]
  uint16_t* y;           // [N][Ho][Wo][64]
  float* part;           // [N*Ho][2][64] or null
  uint32_t xsp_bytes;
  int Hp, Wsp, Ho, Wo;
  int nimg;              // images
  int rblocks;           // row groups per image = ceil(Ho / ROWS)
  int halo_rows;         // 2*ROWS + R - 2
  int halo_alloc;        // bytes reserved for the halo (whole KiB)
};

}  // namespace

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS barrier without the compiler's memory-model drain: ds traffic is waited for, VMEM (the
// previous group's output stores, the next halo's DMA) stays in flight
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void buf_store16(const uint4& v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, r, (int)off, 0, 0);
}

// Persistent: the grid is sized to the resident capacity (2 workgroups per CU) and each workgroup
// walks row groups g = blockIdx.x, +gridDim.x, ...; the packed weights are staged once, and the
// halo of the NEXT row group is fetched by LDS-DMA into the second halo buffer while this one
// computes.  Per group every wave issues exactly N_AFTER vector-memory ops after that DMA (its BN
// partial and output stores: buffer stores whose masked lanes get an out-of-range offset, so the
// instruction count never depends on the data or the shape), so the halo wait one group later is
// vmcnt(N_AFTER) -- the output stores keep draining underneath the next group's MFMA.
//
// Output: after the MFMA loop (and a barrier) the finished halo buffer is reused as a per-wave
// [16 px][128 B] staging tile (16-byte chunks XOR-swizzled by pixel), so every output store
// instruction writes 1 KB of contiguous y (8 whole pixels).  Stored straight from the MFMA layout
// the same bytes leave as 16 x 32-byte fragments per instruction and run at ~40% of the rate
// (scripts/bench_stem.py: 2.4 vs 5.9 TB/s for the output alone).
template <int TM, bool STATS>
__global__ void __launch_bounds__(STEM_ROWS * 64, 2) stem_conv_kernel(const StemArgs P) {
  constexpr int N_AFTER = 2 * TM + (STATS ? 8 : 0);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ws = smem;
  const int t = threadIdx.x;
  const int lane = t & 63, wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(P.xsp, P.xsp_bytes);
  const int ngroups = P.nimg * P.rblocks;

  // input rows 2*ho0 .. 2*ho0 + halo_rows - 1 of the group's image: one contiguous span
  auto issue_halo = [&](int grp, char* dst) {
    const int n = grp / P.rblocks;
    const int ho0 = (grp - n * P.rblocks) * STEM_ROWS;
    const int rows = min(P.halo_rows, P.Hp - 2 * ho0);
    const uint32_t span = (uint32_t)rows * P.Wsp * 16;
    const uint32_t src0 = ((uint32_t)(n * P.Hp + 2 * ho0) * P.Wsp) * 16;
    for (int q = wid; q * 1024 < P.halo_alloc; q += STEM_ROWS) {
      const uint32_t o = (uint32_t)q * 1024 + lane * 16;
      glds16(rx, dst + q * 1024, o < span ? src0 + o : OOB);
    }
  };

  int grp = blockIdx.x;
  if (grp < ngroups) issue_halo(grp, smem + W_BYTES);
  {  // packed weights, once per workgroup
    const uint4* wg = reinterpret_cast<const uint4*>(P.wsp);
    for (int i = t; i < STEM_K * 28; i += STEM_ROWS * 64) {
      const int row = i / 28, c16 = i - row * 28;
      *reinterpret_cast<uint4*>(Ws + row * W_PITCH + c16 * 16) = wg[i];
    }
  }
  const int fr = lane & 15, fq = lane >> 4;
  const char* wrow = Ws + fr * W_PITCH + fq * 16;
  const bool lastok = (TM - 1) * 16 + fr < P.Wo;  // the last pixel fragment may be partial
  for (int it = 0; grp < ngroups; grp += gridDim.x, ++it) {
    char* Hs = smem + W_BYTES + (it & 1) * P.halo_alloc;
    if (it == 0) wait_vm<0>();
    else wait_vm<N_AFTER>();  // this group's halo landed (the last group's stores may not have)
    lds_barrier();            // ... for every wave; and every wave is done with the other buffer
    const int nxt = grp + gridDim.x;
    if (nxt < ngroups) issue_halo(nxt, smem + W_BYTES + ((it + 1) & 1) * P.halo_alloc);

    const int n = grp / P.rblocks;
    const int ho = (grp - n * P.rblocks) * STEM_ROWS + wid;
    const bool valid = ho < P.Ho;  // a wave past the image's last row stores nothing (all offsets OOB)
    const int g = n * P.Ho + min(ho, P.Ho - 1);  // BN partial group = this output row

    v4f acc[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    const char* hrow = Hs + (2 * wid) * P.Wsp * 16 + (fr + fq) * 16;
#pragma unroll
    for (int r = 0; r < STEM_R; ++r) {
      v4i a[4], b[TM];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = *reinterpret_cast<const v4i*>(wrow + j * 16 * W_PITCH + r * STEM_SP * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i) b[i] = *reinterpret_cast<const v4i*>(hrow + (r * P.Wsp + i * 16) * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[j], b[i], acc[i][j]);
    }

    // ---- BN partials: lane (fr, fq), register e of acc[i][j] = pixel i*16 + fr, channel
    // j*16 + fq*4 + e; per channel the row's sum and M2 about the row mean (two passes)
    if constexpr (STATS) {
      const __amdgpu_buffer_rsrc_t rp = make_rsrc(P.part + (int64_t)g * 2 * STEM_K, valid ? 2 * STEM_K * 4 : 0);
      const float inv = 1.f / (float)P.Wo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float sm[4], q[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i) v += (i < TM - 1 || lastok) ? acc[i][j][e] : 0.f;
          v = row_sum16(v);
          const float mean = v * inv;
          float m2 = 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const float d = acc[i][j][e] - mean;
            m2 = (i < TM - 1 || lastok) ? fmaf(d, d, m2) : m2;
          }
          sm[e] = v;
          q[e] = row_sum16(m2);
        }
        const uint32_t off = (uint32_t)(j * 16 + fq * 4) * 4;
        buf_store16(make_uint4(__float_as_uint(sm[0]), __float_as_uint(sm[1]), __float_as_uint(sm[2]),
                               __float_as_uint(sm[3])), rp, fr == 0 ? off : OOB);
        buf_store16(make_uint4(__float_as_uint(q[0]), __float_as_uint(q[1]), __float_as_uint(q[2]),
                               __float_as_uint(q[3])), rp, fr == 0 ? off + STEM_K * 4 : OOB);
      }
    }

    // ---- output through the staging tile
    lds_barrier();  // every wave is done reading this halo buffer
    char* stg = Hs + wid * 2048;
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(P.y + (int64_t)g * P.Wo * STEM_K, valid ? P.Wo * STEM_K * 2 : 0);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint2 v;
        v.x = pack2bf(acc[i][j][0], acc[i][j][1]);
        v.y = pack2bf(acc[i][j][2], acc[i][j][3]);
        const int c = 2 * j + (fq >> 1);
        *reinterpret_cast<uint2*>(stg + fr * 128 + ((c ^ (fr & 7)) * 16) + (fq & 1) * 8) = v;
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int pp = k * 8 + (lane >> 3), c = lane & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(stg + pp * 128 + ((c ^ (pp & 7)) * 16));
        const int px = i * 16 + pp;
        buf_store16(v, ry, px < P.Wo ? (uint32_t)(px * STEM_K + c * 8) * 2 : OOB);
      }
    }
  }
  wait_vm<0>();
}

bool stem_halo_supported(int K, int R, int Sp, int Wo) {
  return K == STEM_K && R == STEM_R && Sp == STEM_SP && Wo >= 1 && Wo <= 128;
}

void launch_stem_conv_fwd(const uint16_t* xsp, const uint16_t* wsp, uint16_t* y, float* part, int N, int Hp,
                          int Wsp, int Ho, int Wo, hipStream_t st) {
  if (Wo < 1 || Wo > 128 || Wsp != Wo + STEM_SP - 1 || 2 * (Ho - 1) + STEM_R > Hp)
    throw std::runtime_error("stem_conv_fwd: unsupported geometry");
  StemArgs a{};
  a.xsp = xsp; a.wsp = wsp; a.y = y; a.part = part;
  a.xsp_bytes = (uint32_t)((int64_t)N * Hp * Wsp * 16);
  a.Hp = Hp; a.Wsp = Wsp; a.Ho = Ho; a.Wo = Wo;
  a.nimg = N;
  a.rblocks = ceil_div(Ho, STEM_ROWS);
  a.halo_rows = 2 * STEM_ROWS + STEM_R - 2;
  const int tm = ceil_div(Wo, 16);
  // every fragment read stays inside the allocation: last row + the widest tap past Wo
  const int need = std::max(a.halo_rows * Wsp, (a.halo_rows - 1) * Wsp + tm * 16 + STEM_SP) * 16;
  // (at least the ROWS x 2 KB output staging tiles that reuse a finished halo buffer)
  a.halo_alloc = std::max(ceil_div(need, 1024) * 1024, STEM_ROWS * 2048);
  const int smem = W_BYTES + 2 * a.halo_alloc;  // weights + double-buffered halo
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int resident = 2 * std::max(cus, 1);  // 2 workgroups per CU (LDS: 2 x 78 KB at 224 px)
  dim3 grid(std::max(1, std::min(N * a.rblocks, resident))), blk(STEM_ROWS * 64);
#define PDT_STEM_S(T, S)                                                                          \
  {                                                                                               \
    static bool attr = false;                                                                     \
    if (!attr) {                                                                                  \
      hipFuncSetAttribute((const void*)stem_conv_kernel<T, S>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                          160 * 1024);                                                            \
      attr = true;                                                                                \
    }                                                                                             \
    hipLaunchKernelGGL((stem_conv_kernel<T, S>), grid, blk, smem, st, a);                         \
  }
#define PDT_STEM(T)                                                                               \
  case T:                                                                                         \
    if (part != nullptr) PDT_STEM_S(T, true) else PDT_STEM_S(T, false)                            \
    break;
  switch (tm) {
    PDT_STEM(1) PDT_STEM(2) PDT_STEM(3) PDT_STEM(4) PDT_STEM(5) PDT_STEM(6) PDT_STEM(7) PDT_STEM(8)
    default: throw std::runtime_error("stem_conv_fwd: Wo > 128");
  }
#undef PDT_STEM
#undef PDT_STEM_S
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("stem_conv_fwd: ") + hipGetErrorString(e));
}

// ============================================================================
//     Stem backward: BN-backward apply (through the max-pool gradient gather) fused into the
//                    weight gradient -- the full-resolution stem gradient is never stored
// ============================================================================
// The stem's input gradient is not needed (the image takes no gradient), so dy = BN_bwd(maxpool_bwd
// (dpool)) has exactly one consumer: the weight gradient.  Each workgroup loops over (image, output
// row pair) items; per item it
//   1. stages the 9 input super-pixel rows the pair reads (LDS-DMA, one contiguous span), and
//   2. computes dy of the pair's 2*Wo pixels x 64 channels in registers -- pool quad gather
//      (pool_quad.h), ReLU mask recomputed from y, BN-backward apply with the finished sums --
//      straight into an LDS tile [pixel][channel] (128-B rows, swz128_tr layout),
//   3. accumulates dW[64][224] += dy^T x im2col over the 2*Wo pixels on the MFMA: both operands
//      have the pixel (reduction) index as their strided dimension, so fragments come from the
//      CDNA4 transposing read ds_read_b64_tr_b16 -- on the halo the 32 (tap, channel) columns of
//      a filter row are contiguous bytes starting at the pixel's super-pixel, rows overlapping.
// Wave w owns dW column fragments {w, w+4, w+8, w+12} (< 14) for all four 16-row output-channel
// fragments; the block's partial dW leaves once, at the end (fp32 atomics, or a private slab
// reduced in fixed order for deterministic runs).  Replaces pool_bn_bwd_apply (writes dy, 411 MB
// at batch 256) + the generic TN weight gradient (reads it back).
// Pipelining: the next item's raw loads (y, argmax, pooled gradient: registers) and its halo
// (asm LDS-DMA into the other of two halo buffers) are issued before this item's MFMAs, and the
// BN coefficients live in LDS to leave registers for that prefetch, and dy = k1 g + (A y + B) is
// two FMAs per element: 320 -> 279 us at batch 256
// (scripts/bench_stem_bwd.py); the rest is mostly the dy phase VALU work (pool gather selects).
namespace {

constexpr int SB_THREADS = 256;
constexpr int SB_COLS = STEM_R * STEM_SP * 8;  // 224 dW columns = (r, s, c)
constexpr int SB_NJ = SB_COLS / 16;            // 14 column fragments

struct StemBwdArgs {
  const uint4* dp;       // pooled gradient [N][Hq][Wq][8] (8-channel vectors)
  const uint2* idx;      // argmax bytes, same indexing
  const uint4* y;        // stem conv output [N][Ho][Wo][8]
  const float* stats;    // [4][64] mean, invstd, scale, shift
  const float* gamma;    // [64]
  const float* sums;     // [2][64] sum g, sum g*(y - mean)
  float invM;
  int train;
  const uint16_t* xsp;
  uint32_t xsp_bytes;
  float* out;            // atomic: [64][224] (zeroed); slab: [gridDim.x][64*224]
  int slab;
  int Ho, Wo, Hq, Wq, Hp, Wsp;
  int items;             // N * Ho / 2
  int halo_alloc;
};

__device__ __forceinline__ int swz_tr128(int row, int chunk) {  // = conv_igemm.hip swz128_tr
  const int sw = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return row * 128 + ((chunk ^ (sw << 1)) << 4);
}

typedef short v4s_tr __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4s_tr tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s_tr*)(reinterpret_cast<uintptr_t>(p)));
}

__device__ __forceinline__ v4i tr_frag(const char* lo, const char* hi) {
  return __builtin_bit_cast(v4i, __builtin_shufflevector(tr_read(lo), tr_read(hi), 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}


// Raw loads of one dy unit (quad b of the item's row pair x channel group c8): the 4 y vectors and
// the 4 covering pooled windows' (argmax, gradient).  Issued one item ahead (into registers) so
// their latency hides behind the previous item's MFMAs; windows past the pooled edge load the
// quad's own window (a valid address) and are masked at use.
struct SbRaw {
  uint4 y[4];
  uint2 id[4];
  uint4 g[4];
};

__device__ __forceinline__ void sb_load(const StemBwdArgs& P, int n, int a, int b, int c8, SbRaw& r) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
    r.y[e] = P.y[((int64_t)(n * P.Ho + 2 * a + (e >> 1)) * P.Wo + 2 * b + (e & 1)) * 8 + c8];
#pragma unroll
  for (int wi = 0; wi < 4; ++wi) {
    const int ho = a + (wi >> 1), wo = b + (wi & 1);
    const bool ok = ho < P.Hq && wo < P.Wq;
    const int64_t o = (((int64_t)n * P.Hq + (ok ? ho : a)) * P.Wq + (ok ? wo : b)) * 8 + c8;
    r.id[wi] = P.idx[o];
    r.g[wi] = P.dp[o];
  }
}

// Opaque use of the prefetched registers at the start of the dy phase: everything computed from
// them depends on these asm outputs, so the compiler cannot hoist that work (and its vmcnt wait)
// above the item's barrier into the MFMA loop, where it would stall on the prefetch.
__device__ __forceinline__ void sb_pin(SbRaw& r) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    asm volatile("" : "+v"(r.y[e].x), "+v"(r.y[e].y), "+v"(r.y[e].z), "+v"(r.y[e].w));
    asm volatile("" : "+v"(r.g[e].x), "+v"(r.g[e].y), "+v"(r.g[e].z), "+v"(r.g[e].w));
    asm volatile("" : "+v"(r.id[e].x), "+v"(r.id[e].y));
  }
}

// asm LDS-DMA (16 B per lane): invisible to the compiler's waitcnt pass, which would otherwise put a
// vmcnt(0) -- draining the register prefetch -- in front of every LDS read after it; ordered by the
// kernel's own vmcnt(0) + barrier
__device__ __forceinline__ void sb_glds16(const v4i& r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %1\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
               :: "v"(voff), "s"(__builtin_amdgcn_readfirstlane(lds)), "s"(r) : "memory", "m0");
}

}  // namespace

__global__ void __launch_bounds__(SB_THREADS, 2) stem_bwd_fused_kernel(const StemBwdArgs P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x;
  const int lane = t & 63, wid = __builtin_amdgcn_readfirstlane(t >> 6);
  char* Ds = smem;                       // dy tile [2*Wo][64] bf16
  char* Hs0 = smem + 2 * P.Wo * 128;     // 9 input rows, double-buffered (item parity)
  const uint64_t xa = reinterpret_cast<uint64_t>(P.xsp);
  const v4i rx = v4i{(int)(uint32_t)xa, (int)((uint32_t)(xa >> 32) & 0xffffu), (int)P.xsp_bytes, 0x00020000};

  // BN-backward coefficients per channel in LDS (cf[64][8]: k1, A, B, scale, shift), read per
  // channel inside the dy loop (registers go to the one-item-ahead prefetch instead).  Training:
  // dy = k1 * (g - s0/M - (y - mean) * k2) = k1 * g + (A * y + B), A = -k1 k2, B = k1 (mean k2 - s0/M);
  // eval: dy = k1 * g (A = B = 0).
  float* cf = reinterpret_cast<float*>(Hs0 + 2 * P.halo_alloc);
  if (t < 64) {
    const float is = P.stats[64 + t], k1 = P.gamma[t] * is;
    const float k2 = P.train ? P.sums[64 + t] * is * is * P.invM : 0.f;
    const float sg = P.train ? P.sums[t] * P.invM : 0.f;
    float4* o = reinterpret_cast<float4*>(cf + t * 8);
    o[0] = make_float4(k1, -k1 * k2, k1 * (P.stats[t] * k2 - sg), P.stats[128 + t]);
    o[1] = make_float4(P.stats[192 + t], 0.f, 0.f, 0.f);
  }
  const int c8 = t & 7;  // this thread's fixed 8-channel group (256 % 8 == 0)

  const int li = lane & 15, g = lane >> 4;
  const int tq = li >> 2, tp = li & 3;
  const bool j3 = wid + 12 < SB_NJ;  // waves 0, 1 own a fourth column fragment
  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int hq2 = P.Ho >> 1;
  const int npx = 2 * P.Wo;
  const int nu = P.Wq * 8;  // dy units of an item (<= 512: at most two per thread)
  const bool v0 = t < nu, v1 = t + SB_THREADS < nu;
  const int b0 = v0 ? t >> 3 : 0, b1 = v1 ? (t + SB_THREADS) >> 3 : 0;

  // halo of item `it` (input rows 4a .. 4a + 8 of image n) into buffer `buf`
  auto halo = [&](int it, int buf) {
    const int n = it / hq2, a = it - n * hq2;
    const int rows = min(9, P.Hp - 4 * a);
    const uint32_t span = (uint32_t)rows * P.Wsp * 16;
    const uint32_t src0 = ((uint32_t)(n * P.Hp + 4 * a) * P.Wsp) * 16;
    const uint32_t dst = (uint32_t)reinterpret_cast<uintptr_t>(Hs0 + buf * P.halo_alloc);
    for (int q = wid; q * 1024 < P.halo_alloc; q += SB_THREADS / 64) {
      const uint32_t o = (uint32_t)q * 1024 + lane * 16;
      sb_glds16(rx, dst + q * 1024, o < span ? src0 + o : OOB);
    }
  };
  SbRaw r0, r1;  // raw loads of the item after the current one (two dy units per thread)
  auto prefetch = [&](int it) {
    const int n = it / hq2, a = it - n * hq2;
    sb_load(P, n, a, b0, c8, r0);  // both units unconditionally (b1 clamped): every prefetched
    sb_load(P, n, a, b1, c8, r1);  // register is consumed each item, so no stale-load wait
  };
  // dy of unit (a, b) from its raw loads -> LDS.  The pool gather is pool_grad_quad_regs evaluated
  // per channel (same sums, same order) so no unpacked quad is held: channel j of the four pixels
  // is built, BN-applied and packed before channel j + 1.
  auto dy_unit = [&](const SbRaw& r, int a, int b, bool store) {
    uint32_t sel[4][2];  // argmax byte words of the four windows; 0xff.. = past the pooled edge
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) {
      const bool ok = a + (wi >> 1) < P.Hq && b + (wi & 1) < P.Wq;
      sel[wi][0] = ok ? r.id[wi].x : 0xffffffffu;
      sel[wi][1] = ok ? r.id[wi].y : 0xffffffffu;
    }
    uint32_t ow[4][4];  // packed bf16 output words: pixel e, channel pair
    float lo[4];        // pixel e's even channel, waiting for its pair
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 ca = *reinterpret_cast<const float4*>(cf + (c8 * 8 + j) * 8);  // k1, A, B, scale
      const float sft = cf[(c8 * 8 + j) * 8 + 4];
      auto gv = [&](const uint4& v) {
        const uint32_t w = (&v.x)[j >> 1];
        return __uint_as_float((j & 1) ? (w & 0xffff0000u) : (w << 16));
      };
      uint32_t sb[4];
#pragma unroll
      for (int wi = 0; wi < 4; ++wi) sb[wi] = (sel[wi][j >> 2] >> (8 * (j & 3))) & 0xffu;
      const float g00 = gv(r.g[0]), g01 = gv(r.g[1]), g10 = gv(r.g[2]), g11 = gv(r.g[3]);
      float pg[4];
      pg[0] = sb[0] == 4u ? g00 : 0.f;
      pg[1] = (sb[0] == 5u ? g00 : 0.f) + (sb[1] == 3u ? g01 : 0.f);
      pg[2] = (sb[0] == 7u ? g00 : 0.f) + (sb[2] == 1u ? g10 : 0.f);
      pg[3] = ((sb[0] == 8u ? g00 : 0.f) + (sb[1] == 6u ? g01 : 0.f)) +
              ((sb[2] == 2u ? g10 : 0.f) + (sb[3] == 0u ? g11 : 0.f));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float yy = gv(r.y[e]);
        const float gr = fmaf(yy, ca.w, sft) > 0.f ? pg[e] : 0.f;
        const float o = fmaf(ca.x, gr, fmaf(ca.y, yy, ca.z));
        if (j & 1) ow[e][j >> 1] = pack2bf(lo[e], o);
        else lo[e] = o;
      }
    }
    if (store) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int hh = e >> 1, w = 2 * b + (e & 1);
        *reinterpret_cast<uint4*>(Ds + swz_tr128(hh * P.Wo + w, c8)) = make_uint4(ow[e][0], ow[e][1], ow[e][2], ow[e][3]);
      }
    }
  };

  __syncthreads();  // cf written
  // The pass with cur < 0 only issues the block's first item: every prefetch has ONE load site, so
  // the loop-carried registers need no copies (a copy would wait on the loads it copies).
  int par = 1;
  for (int cur = (int)blockIdx.x - (int)gridDim.x; cur < P.items; cur += gridDim.x, par ^= 1) {
    const bool live = cur >= 0;
    if (live) {
      const int a = cur - (cur / hq2) * hq2;
      // 1. dy of the row pair (2a, 2a + 1) from the prefetched loads
      sb_pin(r0);
      dy_unit(r0, a, b0, v0);
      sb_pin(r1);
      dy_unit(r1, a, b1, v1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this item's halo (asm DMA) landed
      __syncthreads();
    }
    // 2. next item's raw loads and halo in flight under this item's MFMAs
    // (the loads unconditionally -- clamped to the last item when there is no next one -- so the
    // loop-carried registers have no "kept old value" path, whose copies would wait on them)
    const int nxt = cur + gridDim.x;
    prefetch(min(nxt, P.items - 1));
    if (nxt < P.items) halo(nxt, par ^ 1);
    if (!live) continue;
    // 3. dW += dy^T x im2col over the pair's pixels, 32 per K-step
    const char* Hs = Hs0 + par * P.halo_alloc;
    for (int s = 0; s < npx / 32; ++s) {
      const int p0 = s * 32 + 8 * g;           // this lane group's 8 pixels (one row: Wo % 16 == 0)
      const int hh = p0 >= P.Wo ? 1 : 0;
      const int wo0 = p0 - hh * P.Wo;
      v4i af[4], bf[4];
#pragma unroll
      for (int im = 0; im < 4; ++im) {
        const int ch = im * 2 + (tp >> 1), sub = (tp & 1) * 8;
        af[im] = tr_frag(Ds + swz_tr128(p0 + tq, ch) + sub, Ds + swz_tr128(p0 + 4 + tq, ch) + sub);
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int jn = jj < 3 || j3 ? wid + 4 * jj : wid;  // a 4th fragment only on waves 0, 1
        const int r = jn >> 1, col0 = (jn & 1) * 16;
        const char* base = Hs + ((2 * hh + r) * P.Wsp + wo0 + tq) * 16 + (col0 + 4 * tp) * 2;
        bf[jj] = tr_frag(base, base + 4 * 16);
      }
#pragma unroll
      for (int im = 0; im < 4; ++im)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[im][jj] = mfma16(af[im], bf[jj], acc[im][jj]);
    }
    // every wave's LDS reads retired before the next item overwrites Ds / this halo buffer; no
    // vmcnt here (the prefetch stays in flight)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // partial dW out: lane (fr = li, fq = g) of acc[im][jj] = row im*16 + g*4 + e, column jn*16 + li
  float* o = P.slab ? P.out + (int64_t)blockIdx.x * 64 * SB_COLS : P.out;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    if (jj == 3 && !j3) break;
    const int col = (wid + 4 * jj) * 16 + li;
#pragma unroll
    for (int im = 0; im < 4; ++im)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float* dst = o + (im * 16 + g * 4 + e) * SB_COLS + col;
        if (P.slab) *dst = acc[im][jj][e];
        else unsafeAtomicAdd(dst, acc[im][jj][e]);
      }
  }
}

// Deterministic slab sum: 16 outputs per block, 16 phases per output (phase p adds slabs p, p+16, ...
// in order), then the 16 phase sums in order -- fixed order, and 32 loads in flight per thread
// instead of one thread walking all 512 slabs (186 us on the step's tail, r9a)
__global__ void __launch_bounds__(256) stem_slab_reduce_kernel(const float* __restrict__ ws, int nslab,
                                                               float* __restrict__ out) {
  __shared__ float part[16][17];
  const int o = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + o;
  float s = 0.f;
  if (i < 64 * SB_COLS) {
#pragma unroll 8
    for (int b = ph; b < nslab; b += 16) s += ws[(int64_t)b * 64 * SB_COLS + i];
  }
  part[ph][o] = s;
  __syncthreads();
  if (threadIdx.x < 16 && i < 64 * SB_COLS) {
    float t = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) t += part[p][threadIdx.x];
    out[i] = t;
  }
}

bool stem_bwd_fused_supported(int K, int R, int Sp, int Ho, int Wo) {
  return K == STEM_K && R == STEM_R && Sp == STEM_SP && Ho % 2 == 0 && Wo % 16 == 0 && Wo >= 16 && Wo <= 128;
}

int stem_bwd_fused_blocks(int N, int Ho) {  // 2 resident blocks per CU (62 KB LDS each at 224 px)
  return std::max(1, std::min(N * Ho / 2, 512));
}

void launch_stem_bwd_fused(const uint16_t* dpool, const uint8_t* idx, const uint16_t* y, const float* stats,
                           const float* gamma, const float* sums, bool training, const uint16_t* xsp, int N,
                           int Ho, int Wo, int Hp, int Wsp, float* dwsp, float* ws, hipStream_t st) {
  if (!stem_bwd_fused_supported(STEM_K, STEM_R, STEM_SP, Ho, Wo) || Wsp != Wo + STEM_SP - 1 ||
      2 * (Ho - 1) + STEM_R > Hp)
    throw std::runtime_error("stem_bwd_fused: unsupported geometry");
  StemBwdArgs a{};
  a.dp = reinterpret_cast<const uint4*>(dpool);
  a.idx = reinterpret_cast<const uint2*>(idx);
  a.y = reinterpret_cast<const uint4*>(y);
  a.stats = stats; a.gamma = gamma; a.sums = sums;
  a.invM = 1.f / (float)((int64_t)N * Ho * Wo);
  a.train = training ? 1 : 0;
  a.xsp = xsp;
  a.xsp_bytes = (uint32_t)((int64_t)N * Hp * Wsp * 16);
  a.Ho = Ho; a.Wo = Wo; a.Hq = Ho / 2; a.Wq = Wo / 2; a.Hp = Hp; a.Wsp = Wsp;
  a.items = N * Ho / 2;
  a.halo_alloc = ceil_div(9 * Wsp * 16, 1024) * 1024;
  const int grid = stem_bwd_fused_blocks(N, Ho);
  a.slab = ws != nullptr ? 1 : 0;
  a.out = ws != nullptr ? ws : dwsp;
  if (!a.slab) hipMemsetAsync(dwsp, 0, 64 * SB_COLS * sizeof(float), st);
  const int smem = 2 * Wo * 128 + 2 * a.halo_alloc + 64 * 8 * 4;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)stem_bwd_fused_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(stem_bwd_fused_kernel, dim3(grid), dim3(SB_THREADS), smem, st, a);
  if (a.slab)
    hipLaunchKernelGGL(stem_slab_reduce_kernel, dim3(ceil_div(64 * SB_COLS, 16)), dim3(256), 0, st, ws, grid,
                       dwsp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("stem_bwd_fused: ") + hipGetErrorString(e));
}

}  // namespace pdt
