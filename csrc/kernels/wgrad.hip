// Weight gradient of the implicit-GEMM convolution (round 5 rebuild), gfx950 / MI355X.
//
//   dW[Kout][R*S*C] = sum over pixels m of dy[m][Kout]^T * im2col(x)[m][(tap, c)]
//
// Both operands have the reduction index (pixels) as the strided dimension: 64-pixel K-steps
// are staged in LDS row-major by pixel ([64 m][BM kout] and [64 m][BN cols], 16-B chunks XOR-
// swizzled) and every MFMA fragment is two ds_read_b64_tr_b16 (the read transposes), as in the
// round-1..4 TN kernel.  What changed, and why (profiles/r4f_pmc_tn_ntq.txt):
//
//   * the old kernel ran 4-wave 128x128 blocks, two per CU, on a two-stage pipeline whose every
//     K-step waited for the loads issued at the top of that same step (one 512-cycle compute
//     step of lead against a 1-2.5 us loaded L2/HBM latency: 17.5 % MFMA busy per wave).  It
//     needed ~4 blocks per CU of split-K parallelism to hide that, and split-K is paid in fp32
//     atomics: every wgrad flushed ~32 MB of them, ~25 us of the memory-side atomic rate
//     (MI355X_MICROARCH "Global float atomics": ~1.3 TB/s chip-wide) at the end of a 60-140 us
//     kernel, with every block reaching its flush at the same time.
//   * hipcc put an `s_waitcnt vmcnt(0)` in front of every ds_read_tr builtin that follows an
//     LDS-DMA builtin (it cannot tell the DMA's destination from the read's source), so the old
//     kernel's "two-stage pipeline" drained every prefetch at every fragment read.  Here the DMA
//     is inline asm (igemm_common.h glds16_asm), invisible to that analysis; the kernel orders it
//     with its own counted vmcnt + barrier, and the reads stay builtins whose lgkmcnt waits the
//     compiler places exactly;
//   * ONE 8-wave block per CU streams its share of the reduction through a 4-slot LDS ring
//     (32-40 KB per K64 slot), and reads every step's fragments one step ahead: the LDS reads of
//     step j+1 are in flight while the MFMAs of step j run.  The two waves of a SIMD (w and w+4)
//     own the same 64x64 accumulator tile and split every K64 step into its two k32 halves, so
//     the SIMD's matrix pipe gets 32 MFMAs per barrier from two independent instruction streams
//     while each wave holds 64 accumulators.  The pair's partial tiles are summed through LDS at
//     the end (a + b == b + a: the result does not depend on which wave adds), so a block flushes
//     ONE accumulator set: 256 blocks x 64 KB = 16 MB of atomics instead of ~32;
//   * split-K is planned for ~one block per CU, not for ~4.
// Measured (r5e/r5i, one MI355X): all ResNet-50 wgrads isolated 4.93 -> 4.63 ms (layer-3/4 1x1:
// -15 %); ResNet-50 step 18.70 -> 18.45 ms in the same call.  What still bounds the main loop
// (PMC, r5h: 24 % MFMA busy on the layer-3 1x1, 31 % of wave time at waits, TD stalled on the TC):
// the L2 -> LDS rate of 64x64 wave tiles -- a 64 KB-per-step 256x256 tile would halve the bytes
// per FLOP but flush 4x the split-K partials.
// Tile shapes (4 accumulator tiles of 64x64 per block): 128x128 (2x2), 64x256 (1x4: Kout = 64)
// and 256x64 (4x1: the layer-1 64-channel inputs with 256 output channels).  Loaders: pointwise
// (1x1/s1: reduction row = pixel) and general (any R, S, stride, padding: each B row decomposed
// once and advanced with carries).  Deterministic mode writes per-split fp32 slabs with plain
// stores and sums them in fixed order (wg_splitk_reduce_kernel), bitwise run-to-run.
#include "common.h"
#include "igemm_common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace pdt {

struct WgArgs {
  const uint16_t* dy;  // [Mred][Kout]
  const uint16_t* x;   // [N][H][W][C]
  float* out;          // dw [Kout][Ncols], or the slab base [splits][Kout][Ncols]
  uint32_t dy_bytes, x_bytes;
  int Mred, Kout, Ncols;
  int H, W, C, S, stride, pad, stride_w;
  FastDiv div_hw, div_w;  // reduction row m -> n = m / (Ho*Wo), ho = rem / Wo
  int HoWo, Wo, Ho;
  int steps_per_split, nsteps;
  int adv_r, adv_qh, adv_qn;  // 64 rows = (adv_qn images, adv_qh output rows, adv_r columns)
  int mode;                   // WG_ATOMIC, WG_STORE (slab or single split), WG_ACCUM (+= single split)
  int64_t slab_stride;        // floats between the slabs of consecutive splits (0: no slabs)
  float* zero;                // optional: zero_n floats workgroup 0 clears (a consumed BN-sum
  int zero_n;                 //   accumulator, re-zeroed without a memset launch)
};

constexpr int WG_ATOMIC = 0, WG_STORE = 1, WG_ACCUM = 2;

template <int WM, int WN>
struct WgCfg {
  static_assert(WM * WN == 4, "four 64x64 accumulator tiles per block");
  static constexpr int NT = 512;
  static constexpr int BM = WM * 64, BN = WN * 64;
  static constexpr int A_ROWB = BM * 2, B_ROWB = BN * 2;   // bytes per pixel row of each image
  static constexpr int A_BYTES = 64 * A_ROWB, B_BYTES = 64 * B_ROWB;
  static constexpr int STAGE = A_BYTES + B_BYTES;          // 32 KB (2x2) or 40 KB (1x4, 4x1)
#ifndef PDT_WG_STAGES
#define PDT_WG_STAGES 4
#endif
  static constexpr int STAGES = PDT_WG_STAGES;             // (>= 3: fragments are read one step ahead)
  static constexpr int SMEM = STAGES * STAGE;              // 128 or 160 KB: one block per CU
  static_assert(SMEM <= 163840, "LDS");
  static constexpr int A_LPR = A_ROWB / 16, A_RPI = 64 / A_LPR;  // lanes per row / rows per piece
  static constexpr int B_LPR = B_ROWB / 16, B_RPI = 64 / B_LPR;
  static constexpr int A_PW = A_BYTES / 1024 / 8;          // 1-KB DMA pieces per wave per K-step
  static constexpr int B_PW = B_BYTES / 1024 / 8;
  static_assert(A_PW * 8192 == A_BYTES && B_PW * 8192 == B_BYTES, "tile DMA split");
};

template <int WM, int WN, bool PW>
__global__ void __launch_bounds__(512, 2) wgrad_kernel(const WgArgs P) {
  using CFG = WgCfg<WM, WN>;
  constexpr int A_PW = CFG::A_PW, B_PW = CFG::B_PW, ST = CFG::STAGES;
  constexpr int LPS = A_PW + B_PW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (P.zero != nullptr && blockIdx.x == 0)  // ordered after the accumulator's consumer by the caller
    for (int i = threadIdx.x; i < P.zero_n; i += blockDim.x) P.zero[i] = 0.f;

  const int ntn = (P.Ncols + CFG::BN - 1) / CFG::BN;
  const int ntm = (P.Kout + CFG::BM - 1) / CFG::BM;
  const int tiles = ntm * ntn;
  // split-major logical ids after the XCD remap: the tiles of one split read the same dy rows and
  // overlapping x rows, and run on one XCD (its L2)
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / tiles;
  const int bid = lid - split * tiles;
  const int tmi = bid / ntn, tni = bid - tmi * ntn;
  const int k0 = tmi * CFG::BM, c0 = tni * CFG::BN;
  const int s_begin = split * P.steps_per_split;
  const int s_end = min(P.nsteps, s_begin + P.steps_per_split);

  const int t = threadIdx.x;
  const int lane = t & 63, wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const v4i rdy = rsrc_words(P.dy, P.dy_bytes);
  const v4i rx = rsrc_words(P.x, P.x_bytes);
  const uint32_t sbase = lds_addr(smem);

  // A (dy): piece p of wave w covers rows (w*A_PW + p)*A_RPI + lane/A_LPR; LDS slot lane%A_LPR of a
  // row holds source chunk swz(slot) (the XOR is an involution), so the lane-linear DMA image IS
  // the swizzled image the fragment reads expect.  Out-of-range columns carry the OOB poison;
  // rows past Mred lie past the end of the buffer: both read 0.
  int a_lane[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int arow = (wid * A_PW + i) * CFG::A_RPI + lane / CFG::A_LPR;
    const int slot = lane % CFG::A_LPR;
    const int chk = (swz_img<CFG::A_ROWB>(arow, slot) - arow * CFG::A_ROWB) >> 4;
    const int acol = k0 + chk * 8;
    a_lane[i] = acol < P.Kout ? (arow * P.Kout + acol) * 2 : (int)OOB;
  }
  // B (x): column chunk -> (tap, channel) per lane, fixed for the whole loop
  int brow[B_PW], b_dh[B_PW], b_dw[B_PW], b_chb[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    brow[i] = (wid * B_PW + i) * CFG::B_RPI + lane / CFG::B_LPR;
    const int slot = lane % CFG::B_LPR;
    const int chk = (swz_img<CFG::B_ROWB>(brow[i], slot) - brow[i] * CFG::B_ROWB) >> 4;
    const int col = c0 + chk * 8;
    const int tap = col / P.C;
    b_chb[i] = col < P.Ncols ? (col - tap * P.C) * 2 : (int)OOB;
    const int r = tap / P.S;
    b_dh[i] = r - P.pad;
    b_dw[i] = (tap - r * P.S) - P.pad;
  }
  const int WC2 = P.W * P.C * 2, HWC2 = P.H * WC2, C2 = P.C * 2;
  // general loader: (n, ho, wo) of each B row decomposed once, then advanced by 64 rows per
  // issued K-step (issue() runs for consecutive steps) with two conditional carries
  uint32_t b_n[B_PW], b_ho[B_PW], b_wo[B_PW];
  if constexpr (!PW) {
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const uint32_t m = (uint32_t)(s_begin * 64 + brow[i]);
      b_n[i] = fdiv(m, P.div_hw);
      const uint32_t rem = m - b_n[i] * (uint32_t)P.HoWo;
      b_ho[i] = fdiv(rem, P.div_w);
      b_wo[i] = rem - b_ho[i] * (uint32_t)P.Wo;
    }
  }

  auto issue = [&](int step, int buf) {
    const uint32_t As = sbase + buf * CFG::STAGE;
    const uint32_t Bs = As + CFG::A_BYTES;
    const int mb = step * 64;
    const int abase = mb * P.Kout * 2;
#pragma unroll
    for (int i = 0; i < A_PW; ++i)
      glds16_asm(rdy, As + (wid * A_PW + i) * 1024, (uint32_t)(abase + a_lane[i]));
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      uint32_t off;
      if constexpr (PW) {
        off = (uint32_t)((mb + brow[i]) * C2 + b_chb[i]);
      } else {
        // 24-bit multiplies (every factor < 2^24, products < 2^32), computed unconditionally
        const uint32_t h = __umul24(b_ho[i], (uint32_t)P.stride) + (uint32_t)b_dh[i];
        const uint32_t w = __umul24(b_wo[i], (uint32_t)P.stride_w) + (uint32_t)b_dw[i];
        const bool ok = h < (uint32_t)P.H && w < (uint32_t)P.W;
        const uint32_t o = __umul24(b_n[i], (uint32_t)HWC2) + __umul24(h, (uint32_t)WC2) +
                           __umul24(w, (uint32_t)C2) + (uint32_t)b_chb[i];
        off = ok ? o : OOB;
        uint32_t wo = b_wo[i] + (uint32_t)P.adv_r;
        const uint32_t c1 = wo >= (uint32_t)P.Wo ? 1u : 0u;
        b_wo[i] = c1 ? wo - (uint32_t)P.Wo : wo;
        uint32_t ho = b_ho[i] + (uint32_t)P.adv_qh + c1;
        const uint32_t c2 = ho >= (uint32_t)P.Ho ? 1u : 0u;
        b_ho[i] = c2 ? ho - (uint32_t)P.Ho : ho;
        b_n[i] += (uint32_t)P.adv_qn + c2;
      }
      glds16_asm(rx, Bs + (wid * B_PW + i) * 1024, off);
    }
  };

  const int half = wid >> 2, q = wid & 3;        // waves w, w+4: same SIMD, same tile, k32 halves
  const int wm = q % WM, wn = q / WM;
  const int li = lane & 15, g = lane >> 4;        // group g covers k rows 8g..8g+7 of a k32 half
  const int tq = li >> 2, tp = li & 3;            // tr-read: lane 4q+p -> row q, columns 4p..4p+3

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  auto frag_a = [&](const char* base, int row, int col) -> const char* {
    return base + swz_img<CFG::A_ROWB>(row, col >> 3) + ((col & 7) << 1);
  };
  auto frag_b = [&](const char* base, int row, int col) -> const char* {
    return base + swz_img<CFG::B_ROWB>(row, col >> 3) + ((col & 7) << 1);
  };

  // Ring of ST K64 slots, slot j in buffer j % ST, fragments read ONE step ahead: iteration j waits
  // until step j+1 landed, passes the barrier (RAW for slot j+1; WAR for buffer (j+ST-1) % ST =
  // (j-1) % ST, whose fragments were read in iteration j-2 and consumed by the MFMAs of iteration
  // j-1), refills that buffer with step j+ST-1, issues the reads of slot j+1 and runs the MFMAs of
  // step j on the fragments read one iteration earlier -- the LDS reads of the next step overlap
  // the MFMAs of this one (the compiler places the lgkmcnt waits: the reads are builtins, only the
  // DMA is asm).  Two fragment sets, the loop unrolled by two, so no register copies.
  const int nst = s_end - s_begin;
#pragma unroll
  for (int p = 0; p < ST - 1; ++p)
    if (p < nst) issue(s_begin + p, p);
  const int rowA = half * 32 + 8 * g + tq;  // m row of this wave's first tr block
  auto read = [&](int j, v4i (&af)[4], v4i (&bfr)[4]) {
    const char* As = smem + (j % ST) * CFG::STAGE;
    const char* Bs = As + CFG::A_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = wm * 64 + i * 16 + 4 * tp;
      const char* pa = frag_a(As, rowA, col);  // row + 4: same swizzle class, +4 rows of bytes
      af[i] = cat_frag(ds_read_tr(pa), ds_read_tr(pa + 4 * CFG::A_ROWB));
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int col = wn * 64 + jj * 16 + 4 * tp;
      const char* pb = frag_b(Bs, rowA, col);
      bfr[jj] = cat_frag(ds_read_tr(pb), ds_read_tr(pb + 4 * CFG::B_ROWB));
    }
  };
  auto body = [&](int j, v4i (&af)[4], v4i (&bfr)[4], v4i (&an)[4], v4i (&bn)[4]) {
    // this body's fragments (read by the previous body) have landed: a compiler-visible
    // lgkmcnt(0), so the waitcnt pass knows it and places no wait on the newer reads in front of
    // the MFMAs below (it cannot count 32 reads in flight -- lgkmcnt holds 15 -- and would stall
    // them behind the next step's reads)
    __builtin_amdgcn_s_waitcnt(0xc07f);
    if (j + 1 < nst) {
      wait_steps<LPS>(min(nst - 1, j + ST - 2) - (j + 1));
      lds_barrier_rd();
      if (j + ST - 1 < nst) issue(s_begin + j + ST - 1, (j + ST - 1) % ST);
      read(j + 1, an, bn);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = mfma16(af[i], bfr[jj], acc[i][jj]);
  };
  v4i fa0[4], fb0[4], fa1[4], fb1[4];
  if (nst > 0) {
    wait_steps<LPS>(min(nst - 1, ST - 2));
    lds_barrier_rd();
    read(0, fa0, fb0);
  }
  for (int j = 0; j < nst; j += 2) {
    body(j, fa0, fb0, fa1, fb1);
    if (j + 1 < nst) body(j + 1, fa1, fb1, fa0, fb0);
  }
  __syncthreads();  // every DMA landed (last wait was vmcnt(0)) and every fragment read retired

  // pair reduction: wave half 0 keeps accumulator rows i = 0, 1 (tile rows 0..31), half 1 keeps
  // i = 2, 3; each sends the other half of its tile through a lane-linear LDS image (conflict-free)
  float* xch = reinterpret_cast<float*>(smem);
  const int keep = half ? 2 : 0, send = half ? 0 : 2;
  {
    float* mine = xch + wid * 2048;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) mine[((ii * 4 + jj) * 4 + e) * 64 + lane] = acc[send + ii][jj][e];
  }
  __syncthreads();
  {
    const float* part = xch + (wid ^ 4) * 2048;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[keep + ii][jj][e] += part[((ii * 4 + jj) * 4 + e) * 64 + lane];
  }
  __syncthreads();

  // staged flush: the 16x16 accumulator layout gives a store / atomic wave-instruction four 64-B
  // row pieces; through a wave-private row-major image every instruction covers one 256-B segment
  // of a dW row (the full-rate atomic shape).  Column XOR 16 on rows 4..7 mod 8 keeps the
  // fragment writes (lanes fq = 0/1 are 4 rows apart) and the row reads conflict-free.
  const int fq = lane >> 4, fr = lane & 15;
  float* stg = xch + wid * 2048;  // 32 rows x 64 fp32
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = ii * 16 + fq * 4 + e;
        stg[r * 64 + ((jj * 16 + fr) ^ (((r >> 2) & 1) << 4))] = acc[keep + ii][jj][e];
      }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the region is wave-private
  __builtin_amdgcn_wave_barrier();
  float* o = P.out + split * P.slab_stride;
  const int col = c0 + wn * 64 + lane;
  const int row0 = k0 + wm * 64 + keep * 16;
  if (col < P.Ncols) {
#pragma unroll 8
    for (int r = 0; r < 32; ++r) {
      const float v = stg[r * 64 + (lane ^ (((r >> 2) & 1) << 4))];
      if (row0 + r < P.Kout) {
        float* dst = o + (int64_t)(row0 + r) * P.Ncols + col;
        if (P.mode == WG_ATOMIC) unsafeAtomicAdd(dst, v);
        else if (P.mode == WG_ACCUM) *dst += v;
        else *dst = v;
      }
    }
  }
}


// ============================================================================================
//     3x3 / stride 1 / pad 1: halo-staged activations, one filter tap row per block
// ============================================================================================
// The im2col B row of tap (r, s) and output pixel (n, h, w) is x(n, h + r - 1, w + s - 1).  In
// "padded coordinates" -- images stacked with ONE zero row between neighbours and one zero
// column on each side, a padded row being W + 2 pixels -- output pixel q = (n*(H+1) + h)*(W+2) + w
// reads x_pad[q + r*(W+2) + s]: every tap is a constant shift of ONE staged x image.  A block
// owns the three taps of one filter row r for a BC-channel block: per K-step it stages 62 dy rows
// (q0 .. q0+61; the two padded output columns and the separator row carry dy = 0) and the 64 x_pad
// rows q0 + r*(W+2) .. +63 ONCE, contiguous pixel runs instead of per-tap gathers, and the three
// taps read them shifted by s = 0, 1, 2 rows.  The 64-row MFMA step covers 62 q-rows: A rows 62,
// 63 are zero (OOB loads) and two zero rows after every B slot absorb the reads t + s >= 64.
// Against the general loader per 128x(3x64) tile: the x traffic into LDS drops 3x (one image for
// three taps) and every byte of it is a streaming read; ~3-25 % of the MFMA work is spent on the
// padding (q-space / output space = (H+1)(W+2) / (HW) * 64/62).
struct WhArgs {
  const uint16_t* dy;  // [N][H][W][K]
  const uint16_t* x;   // [N][H][W][C]
  float* out;          // dw [K][3][3][C] (or slabs)
  uint32_t dy_bytes, x_bytes;
  int K, C, H, W;
  int Wp, Hp;          // W + 2, H + 1
  FastDiv div_wp, div_hp;
  int aw, ag, an;      // 62 q-rows = (an images, ag padded rows, aw padded columns)
  int steps_per_split, nsteps;
  int mode;
  int64_t slab_stride;
  float* zero;
  int zero_n;
};

constexpr int WH_STEP = 62;

template <int WM, int WC, int TC>
struct WhCfg {
  static_assert(WM * WC == 4, "four wave pairs");
  static constexpr int BM = WM * 64, BC = WC * TC * 16;
  static constexpr int A_ROWB = BM * 2, B_ROWB = BC * 2;
  static constexpr int A_BYTES = 64 * A_ROWB;
  static constexpr int B_BYTES = 66 * B_ROWB;  // 64 staged rows + 2 zero rows
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int STAGES = 163840 / STAGE > 8 ? 8 : 163840 / STAGE;
  static constexpr int SMEM = STAGES * STAGE;
  static constexpr int A_LPR = A_ROWB / 16, A_RPI = 64 / A_LPR;
  static constexpr int B_LPR = B_ROWB / 16, B_RPI = 64 / B_LPR;
  static constexpr int A_PW = A_BYTES / 8192;
  static constexpr int B_PW = 64 * B_ROWB / 8192;
  static_assert(A_PW * 8192 == A_BYTES && B_PW * 8192 == 64 * B_ROWB, "tile DMA split");
  static constexpr int NB = 3 * TC;                  // B fragments per wave: 3 taps x TC blocks of 16 ch
  static constexpr int PITCH = TC == 1 ? 84 : 104;   // flush image row pitch (floats, conflict-free)
  static_assert(8 * 2 * NB * 4 * 64 * 4 <= SMEM && 8 * 32 * PITCH * 4 <= SMEM, "epilogue LDS");
};

// s_waitcnt vmcnt(y * LPS) for a wave-uniform y <= Y
template <int LPS, int Y>
__device__ __forceinline__ void wait_younger(int y) {
  if constexpr (Y <= 0) {
    wait_vm<0>();
  } else {
    if (y >= Y) wait_vm<Y * LPS>();
    else wait_younger<LPS, Y - 1>(y);
  }
}

template <int WM, int WC, int TC>
__global__ void __launch_bounds__(512, 2) wgrad_halo3_kernel(const WhArgs P) {
  using CFG = WhCfg<WM, WC, TC>;
  constexpr int A_PW = CFG::A_PW, B_PW = CFG::B_PW, ST = CFG::STAGES, NB = CFG::NB;
  constexpr int LPS = A_PW + B_PW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (P.zero != nullptr && blockIdx.x == 0)
    for (int i = threadIdx.x; i < P.zero_n; i += blockDim.x) P.zero[i] = 0.f;

  const int ntc = P.C / CFG::BC;
  const int ntm = (P.K + CFG::BM - 1) / CFG::BM;
  const int tiles = ntm * ntc * 3;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / tiles;
  const int bid = lid - split * tiles;
  const int tr = bid / (ntm * ntc);
  const int rem = bid - tr * (ntm * ntc);
  const int tmi = rem / ntc, tci = rem - (rem / ntc) * ntc;
  const int k0 = tmi * CFG::BM, cb0 = tci * CFG::BC;
  const int s_begin = split * P.steps_per_split;
  const int s_end = min(P.nsteps, s_begin + P.steps_per_split);

  const int t = threadIdx.x;
  const int lane = t & 63, wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const v4i rdy = rsrc_words(P.dy, P.dy_bytes);
  const v4i rx = rsrc_words(P.x, P.x_bytes);
  const uint32_t sbase = lds_addr(smem);

  // the two zero rows after every B slot (never DMA targets); the first loop barrier publishes them
  for (int i = t; i < ST * (2 * CFG::B_ROWB / 16); i += 512) {
    const int sl = i / (2 * CFG::B_ROWB / 16), o16 = i - sl * (2 * CFG::B_ROWB / 16);
    *reinterpret_cast<v4i*>(smem + sl * CFG::STAGE + CFG::A_BYTES + 64 * CFG::B_ROWB + o16 * 16) = v4i{0, 0, 0, 0};
  }

  const int HW = P.H * P.W, K2 = P.K * 2, C2 = P.C * 2;
  // A rows (dy, q-space) and B rows (x_pad) of this lane, each as (n, padded row, padded column),
  // decomposed once and advanced by 62 q-rows per issued K-step with two conditional carries
  int a_kb[A_PW];
  uint32_t a_n[A_PW], a_h[A_PW], a_w[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int arow = (wid * A_PW + i) * CFG::A_RPI + lane / CFG::A_LPR;
    const int slot = lane % CFG::A_LPR;
    const int chk = (swz_img<CFG::A_ROWB>(arow, slot) - arow * CFG::A_ROWB) >> 4;
    const int kcol = k0 + chk * 8;
    a_kb[i] = (kcol < P.K && arow < WH_STEP) ? kcol * 2 : (int)OOB;
    const uint32_t q = (uint32_t)(s_begin * WH_STEP + arow);
    const uint32_t G = fdiv(q, P.div_wp);
    a_w[i] = q - G * (uint32_t)P.Wp;
    a_n[i] = fdiv(G, P.div_hp);
    a_h[i] = G - a_n[i] * (uint32_t)P.Hp;
  }
  int b_cb[B_PW];
  uint32_t b_n[B_PW], b_g[B_PW], b_w[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int brow = (wid * B_PW + i) * CFG::B_RPI + lane / CFG::B_LPR;
    const int slot = lane % CFG::B_LPR;
    const int chk = (swz_img<CFG::B_ROWB>(brow, slot) - brow * CFG::B_ROWB) >> 4;
    b_cb[i] = (cb0 + chk * 8) * 2;
    const uint32_t pq = (uint32_t)(s_begin * WH_STEP + tr * P.Wp + brow);
    const uint32_t G = fdiv(pq, P.div_wp);
    b_w[i] = pq - G * (uint32_t)P.Wp;
    b_n[i] = fdiv(G, P.div_hp);
    b_g[i] = G - b_n[i] * (uint32_t)P.Hp;
  }
  auto advance = [&](uint32_t& n, uint32_t& g, uint32_t& w) {
    uint32_t w2 = w + (uint32_t)P.aw;
    const uint32_t c1 = w2 >= (uint32_t)P.Wp ? 1u : 0u;
    w = c1 ? w2 - (uint32_t)P.Wp : w2;
    uint32_t g2 = g + (uint32_t)P.ag + c1;
    const uint32_t c2 = g2 >= (uint32_t)P.Hp ? 1u : 0u;
    g = c2 ? g2 - (uint32_t)P.Hp : g2;
    n += (uint32_t)P.an + c2;
  };

  auto issue = [&](int buf) {
    const uint32_t As = sbase + buf * CFG::STAGE;
    const uint32_t Bs = As + CFG::A_BYTES;
#pragma unroll
    for (int i = 0; i < A_PW; ++i) {
      // output pixel (n, h, w) exists for h < H, w < W; the padded ones carry dy = 0
      const bool ok = a_h[i] < (uint32_t)P.H && a_w[i] < (uint32_t)P.W;
      const uint32_t pix = __umul24(a_n[i], (uint32_t)HW) + __umul24(a_h[i], (uint32_t)P.W) + a_w[i];
      const uint32_t off = ok ? __umul24(pix, (uint32_t)K2) + (uint32_t)a_kb[i] : OOB;
      glds16_asm(rdy, As + (wid * A_PW + i) * 1024, off);
      advance(a_n[i], a_h[i], a_w[i]);
    }
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      // padded row g, column w -> image row g - 1, column w - 1 (row 0 / columns 0, W+1: zero)
      const bool ok = b_g[i] >= 1u && b_w[i] >= 1u && b_w[i] <= (uint32_t)P.W;
      const uint32_t pix = __umul24(b_n[i], (uint32_t)HW) + __umul24(b_g[i] - 1u, (uint32_t)P.W) + (b_w[i] - 1u);
      const uint32_t off = ok ? __umul24(pix, (uint32_t)C2) + (uint32_t)b_cb[i] : OOB;
      glds16_asm(rx, Bs + (wid * B_PW + i) * 1024, off);
      advance(b_n[i], b_g[i], b_w[i]);
    }
  };

  const int half = wid >> 2, q = wid & 3;
  const int wm = q % WM, wc = q / WM;
  const int li = lane & 15, g = lane >> 4;
  const int tq = li >> 2, tp = li & 3;

  v4f acc[4][NB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // the ring as in wgrad_kernel: fragments read one step ahead, two fragment sets, unrolled by two
  const int nst = s_end - s_begin;
#pragma unroll
  for (int p = 0; p < ST - 1; ++p)
    if (p < nst) issue(p);
  const int rowA = half * 32 + 8 * g + tq;
  auto read = [&](int j, v4i (&af)[4], v4i (&bfr)[NB]) {
    const char* As = smem + (j % ST) * CFG::STAGE;
    const char* Bs = As + CFG::A_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = wm * 64 + i * 16 + 4 * tp;
      const char* pa = As + swz_img<CFG::A_ROWB>(rowA, col >> 3) + ((col & 7) << 1);
      af[i] = cat_frag(ds_read_tr(pa), ds_read_tr(pa + 4 * CFG::A_ROWB));
    }
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int c = 0; c < TC; ++c) {
        const int col = wc * 16 * TC + c * 16 + 4 * tp;
        const int rb = rowA + s;  // tap s: the image shifted by s rows (swizzle differs at rb + 4)
        bfr[s * TC + c] = cat_frag(ds_read_tr(Bs + swz_img<CFG::B_ROWB>(rb, col >> 3) + ((col & 7) << 1)),
                                   ds_read_tr(Bs + swz_img<CFG::B_ROWB>(rb + 4, col >> 3) + ((col & 7) << 1)));
      }
  };
  auto body = [&](int j, v4i (&af)[4], v4i (&bfr)[NB], v4i (&an)[4], v4i (&bn)[NB]) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // this body's fragments landed (see wgrad_kernel)
    if (j + 1 < nst) {
      wait_younger<LPS, ST - 2>(min(nst - 1, j + ST - 2) - (j + 1));
      lds_barrier_rd();
      if (j + ST - 1 < nst) issue((j + ST - 1) % ST);
      read(j + 1, an, bn);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[i][n] = mfma16(af[i], bfr[n], acc[i][n]);
  };
  v4i fa0[4], fb0[NB], fa1[4], fb1[NB];
  if (nst > 0) {
    wait_younger<LPS, ST - 2>(min(nst - 1, ST - 2));
    lds_barrier_rd();
    read(0, fa0, fb0);
  }
  for (int j = 0; j < nst; j += 2) {
    body(j, fa0, fb0, fa1, fb1);
    if (j + 1 < nst) body(j + 1, fa1, fb1, fa0, fb0);
  }
  __syncthreads();

  // pair reduction (as wgrad_kernel), then a staged flush of 32 rows x (3 taps x 16*TC channels)
  float* xch = reinterpret_cast<float*>(smem);
  const int keep = half ? 2 : 0, send = half ? 0 : 2;
  constexpr int XW = 2 * NB * 4 * 64;  // floats per wave of the exchange image
  {
    float* mine = xch + wid * XW;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e) mine[((ii * NB + n) * 4 + e) * 64 + lane] = acc[send + ii][n][e];
  }
  __syncthreads();
  {
    const float* part = xch + (wid ^ 4) * XW;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[keep + ii][n][e] += part[((ii * NB + n) * 4 + e) * 64 + lane];
  }
  __syncthreads();
  const int fq = lane >> 4, fr = lane & 15;
  float* stg = xch + wid * (32 * CFG::PITCH);
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int e = 0; e < 4; ++e) stg[(ii * 16 + fq * 4 + e) * CFG::PITCH + n * 16 + fr] = acc[keep + ii][n][e];
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the region is wave-private
  __builtin_amdgcn_wave_barrier();
  constexpr int LPR = 16 * TC, RPI = 64 / LPR;  // lanes per dW row segment, rows per instruction
  const int cc = lane % LPR, rr = lane / LPR;
  const int ncols = 9 * P.C;
  float* o = P.out + split * P.slab_stride;
  const int row0 = k0 + wm * 64 + keep * 16;
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int colg = (tr * 3 + s) * P.C + cb0 + wc * 16 * TC + cc;
#pragma unroll 4
    for (int it = 0; it < 32 / RPI; ++it) {
      const int r = it * RPI + rr;
      const float v = stg[r * CFG::PITCH + s * 16 * TC + cc];
      if (row0 + r < P.K) {
        float* dst = o + (int64_t)(row0 + r) * ncols + colg;
        if (P.mode == WG_ATOMIC) unsafeAtomicAdd(dst, v);
        else if (P.mode == WG_ACCUM) *dst += v;
        else *dst = v;
      }
    }
  }
}

// Fixed-order sum of the split-K slabs: ws[splits][n4] float4 -> out[n4].  A 256-thread block
// owns 16 float4 columns; thread (column c, lane k) sums slabs k, k+16, k+32, ... in order, and the
// 16 partials of a column are added in k order through LDS -- the same summation tree on every
// run (bitwise deterministic), with 16x more loads in flight than one thread per column (the
// layer-1 weight gradients have ~256 slabs of only 16K floats).
__global__ void __launch_bounds__(256) wg_splitk_reduce_kernel(const float4* __restrict__ ws, int splits,
                                                               int64_t n4, float4* __restrict__ out,
                                                               int accumulate) {
  __shared__ float4 part[16][17];
  const int c = threadIdx.x & 15, k = threadIdx.x >> 4;
  const int64_t col = (int64_t)blockIdx.x * 16 + c;
  float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < n4) {
    int i = k;
#pragma unroll 1
    for (; i + 48 < splits; i += 64) {  // four slabs in flight per thread, added in slab order
      const float4 v0 = ws[(int64_t)i * n4 + col], v1 = ws[(int64_t)(i + 16) * n4 + col];
      const float4 v2 = ws[(int64_t)(i + 32) * n4 + col], v3 = ws[(int64_t)(i + 48) * n4 + col];
      sm.x += v0.x; sm.y += v0.y; sm.z += v0.z; sm.w += v0.w;
      sm.x += v1.x; sm.y += v1.y; sm.z += v1.z; sm.w += v1.w;
      sm.x += v2.x; sm.y += v2.y; sm.z += v2.z; sm.w += v2.w;
      sm.x += v3.x; sm.y += v3.y; sm.z += v3.z; sm.w += v3.w;
    }
    for (; i < splits; i += 16) {
      const float4 v = ws[(int64_t)i * n4 + col];
      sm.x += v.x; sm.y += v.y; sm.z += v.z; sm.w += v.w;
    }
  }
  part[k][c] = sm;
  __syncthreads();
  if (k == 0 && col < n4) {
    float4 t = part[0][c];
#pragma unroll
    for (int q = 1; q < 16; ++q) {
      const float4 v = part[q][c];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    if (accumulate) {
      const float4 o = out[col];
      t.x += o.x; t.y += o.y; t.z += o.z; t.w += o.w;
    }
    out[col] = t;
  }
}

// ------------------------------------------------------------------------------------- host
static void wg_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Kernel family of a weight gradient: KIND_GEN (wgrad_kernel, any conv) or KIND_HALO3 (3x3/s1/p1).
constexpr int KIND_GEN = 0, KIND_HALO3 = 1;

struct WgPlan {
  int kind, wm, wn, tc;         // tile layout: 4 wave pairs as wm x wn (x tc channel blocks: HALO3)
  int bm, bn;                   // tile rows (output channels) x columns (dW columns)
  int tiles, splits, steps_per_split, nsteps;
  bool slab;                    // split-K partials in private slabs + fixed-order reduce (else atomics)
};

// CUs the split-K plan fills: the device's, minus a reserve for the gradient-collective kernels
// when the step all-reduces (measured in-step at world 1, one MI355X, atomic split-K: planning
// for 128 or 256 CUs gave the same step, 96 was 1.2 % slower, r5: 224 vs 256 +0.2 %).  A weight-
// gradient block holds its CU's LDS and registers for the whole of its K range (one 512-thread
// block per CU), so with a grid of >= CUs blocks an RCCL channel block or an xGMI data kernel
// launched beside it waits for a whole wgrad kernel -- and every peer rank's channel spins
// meanwhile.  A plan of at most (CUs - reserve) blocks per round keeps the reserve free for them
// (a soft reservation: the hardware dispatcher places blocks anywhere; grids above the plan's
// budget still fill the chip).  Set by the DDP wrapper (conv_wgrad_set_cu_reserve).
static int g_wg_reserve = 0;
void conv_wgrad_set_cu_reserve(int n) { g_wg_reserve = n < 0 ? 0 : n; }
int conv_wgrad_cu_reserve() { return g_wg_reserve; }

static int wg_cus() {
  static int v = -1;
  if (v < 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      v = n;
    else
      v = 256;
  }
  return std::max(v / 2, v - g_wg_reserve);
}

// Split-K factor: one 512-thread block per CU at a time, so a plan of tiles * splits blocks runs
// in ceil(tiles * splits / CUs) rounds of ceil(nsteps / splits) K-steps, and every block flushes
// its fp32 tile (atomics at ~1.3 TB/s chip-wide, MI355X_MICROARCH; slabs at the store rate).
// Minimise rounds * steps * t_step + flush + a per-round ramp.
static int choose_splits(int tiles, int nsteps, double t_step_us, double tile_bytes, bool slab, double* est_us) {
  const int cus = wg_cus();
  const double flush_bw = slab ? 5.0e6 : 1.3e6;  // bytes per us
  int best = 1;
  double best_t = 1e30;
  const int smax = std::max(1, std::min(1024, nsteps / 4));
  for (int sp = 1; sp <= smax; ++sp) {
    const int sps = (nsteps + sp - 1) / sp;
    const int eff = (nsteps + sps - 1) / sps;  // splits actually launched
    if (eff != sp) continue;
    const int rounds = (tiles * sp + cus - 1) / cus;
    double t = rounds * (sps * t_step_us + 2.0) + tiles * (double)sp * tile_bytes / flush_bw;
    // slabs: the fixed-order reduce pass reads every slab and read-modify-writes dW (+ a launch)
    if (slab && sp > 1) t += (sp + 2) * (tiles * tile_bytes) / 5.0e6 + 3.0;
    if (t < best_t - 1e-9) { best_t = t; best = sp; }
  }
  *est_us = best_t;
  return best;
}

// The halo kernel runs the Kout = 64 3x3 convs (ResNet layer 1: 0.112 vs 0.139 ms isolated).  With
// Kout >= 128 its 128 x (3 x 64) tile lost to the general loader (layer 2-4: 0.109-0.152 vs
// 0.089-0.109 ms isolated, and 0.3 % on the step, r5c / r5g): both main loops are bound by the
// L2 -> LDS rate, and the 48-column taps cost the wider tile its fragment reuse.
static bool halo3_shape(const ConvShape& s) {
  return s.K <= 64 && s.R == 3 && s.S == 3 && s.stride == 1 && s.sw() == 1 && s.pad == 1 &&
         s.Ho == s.H && s.Wo == s.W && s.C % 64 == 0 && s.K % 64 == 0;
}

static WgPlan plan_wg(const ConvShape& s, bool deterministic) {
  WgPlan p{};
  const int ncols = s.R * s.S * s.C;
  double mfma_cyc, stage_bytes;
  if (halo3_shape(s)) {
    p.kind = KIND_HALO3;
    p.wm = 1; p.wn = 4; p.tc = 1;  // 64 x (3 taps x 64 channels)
    p.bm = p.wm * 64;
    const int bc = p.wn * p.tc * 16;
    p.bn = 3 * bc;
    p.tiles = ((s.K + p.bm - 1) / p.bm) * (s.C / bc) * 3;
    const int64_t q = (int64_t)s.N * (s.H + 1) * (s.W + 2);
    p.nsteps = (int)((q + WH_STEP - 1) / WH_STEP);
    stage_bytes = 64.0 * p.bm * 2 + 64.0 * bc * 2;
  } else {
    p.kind = KIND_GEN;
    p.tc = 0;
    if (s.K <= 64) { p.wm = 1; p.wn = 4; }                          // 64 x 256
    else if (ncols <= 64 && s.K % 256 == 0) { p.wm = 4; p.wn = 1; }  // 256 x 64
    else { p.wm = 2; p.wn = 2; }                                    // 128 x 128
    p.bm = p.wm * 64; p.bn = p.wn * 64;
    p.tiles = ((s.K + p.bm - 1) / p.bm) * ((ncols + p.bn - 1) / p.bn);
    const int64_t mred = (int64_t)s.N * s.Ho * s.Wo;
    p.nsteps = (int)((mred + 63) / 64);
    stage_bytes = 64.0 * (p.bm + p.bn) * 2;
  }
  mfma_cyc = (double)p.bm * p.bn * 64 * 2 / 4096.0;  // per K-step per CU at the MFMA peak
  // a K-step's cost: its MFMAs at ~50 % of peak, or its LDS-DMA bytes at ~50 GB/s per CU
  const double t_step = std::max(mfma_cyc * 2.0 / 2400.0, stage_bytes / 50.0e3);
  // split-K reduction: fp32 atomics (~1.3 TB/s, memory side), or -- deterministic runs -- private
  // slabs written at the store rate plus one fixed-order reduce launch.  Slabs also won the cost
  // model for many non-deterministic shapes but lost in the step (18.40 vs 18.26 ms, r5i): the
  // reduce launches queue on the weight-gradient stream.
  double est_us = 0.0;
  p.slab = deterministic;
  int splits = choose_splits(p.tiles, p.nsteps, t_step, (double)p.bm * p.bn * 4, p.slab, &est_us);
  if (p.slab) {  // slab workspace: splits * |dW| * 4 bytes, capped at 64 MB
    const int64_t dw_bytes = (int64_t)s.K * ncols * 4;
    splits = (int)std::min<int64_t>(splits, std::max<int64_t>(1, ((int64_t)64 << 20) / dw_bytes));
  }
  p.steps_per_split = (p.nsteps + splits - 1) / splits;
  p.splits = (p.nsteps + p.steps_per_split - 1) / p.steps_per_split;
  if (p.splits <= 1) p.slab = false;
  return p;
}

void conv_wgrad_plan(const ConvShape& s, bool deterministic, int out[4]) {
  const WgPlan p = plan_wg(s, deterministic);
  out[0] = p.bm; out[1] = p.bn; out[2] = p.tiles; out[3] = p.splits;
}

size_t conv_wgrad_ws_floats(const ConvShape& s, bool deterministic) {
  const WgPlan p = plan_wg(s, deterministic);
  if (!p.slab) return 0;
  return (size_t)p.splits * s.K * s.R * s.S * s.C;
}

template <int WM, int WN, bool PW>
static void run_wg(const WgArgs& a, int nb, hipStream_t st) {
  using CFG = WgCfg<WM, WN>;
  auto kfn = wgrad_kernel<WM, WN, PW>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, CFG::SMEM);
    attr_set = true;
  }
  hipLaunchKernelGGL(kfn, dim3(nb), dim3(CFG::NT), CFG::SMEM, st, a);
  wg_check("wgrad_kernel");
}

template <int WM, int WC, int TC>
static void run_wh(const WhArgs& a, int nb, hipStream_t st) {
  using CFG = WhCfg<WM, WC, TC>;
  auto kfn = wgrad_halo3_kernel<WM, WC, TC>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, CFG::SMEM);
    attr_set = true;
  }
  hipLaunchKernelGGL(kfn, dim3(nb), dim3(512), CFG::SMEM, st, a);
  wg_check("wgrad_halo3_kernel");
}

void launch_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* dw, float* ws,
                          const ConvShape& s, bool deterministic, bool accumulate, hipStream_t st,
                          float* zero, int zero_n) {
  if (s.C % 8 != 0 || s.K % 8 != 0) throw std::runtime_error("conv_wgrad: channels must be multiples of 8");
  const WgPlan p = plan_wg(s, deterministic);
  const bool slab = p.slab;
  const bool atomic = !p.slab && p.splits > 1;
  if (slab && ws == nullptr) throw std::runtime_error("conv_wgrad: the slab plan needs its workspace");
  const int mode = atomic ? WG_ATOMIC : (slab ? WG_STORE : (accumulate ? WG_ACCUM : WG_STORE));
  const int64_t n = (int64_t)s.K * s.R * s.S * s.C;
  if (atomic && !accumulate) hipMemsetAsync(dw, 0, n * sizeof(float), st);
  const int nb = p.tiles * p.splits;
  const uint32_t dy_bytes = (uint32_t)((int64_t)s.N * s.Ho * s.Wo * s.K * 2);
  const uint32_t x_bytes = (uint32_t)((int64_t)s.N * s.H * s.W * s.C * 2);
  if (p.kind == KIND_HALO3) {
    WhArgs a{};
    a.dy = dy; a.x = x; a.out = slab ? ws : dw;
    a.dy_bytes = dy_bytes; a.x_bytes = x_bytes;
    a.K = s.K; a.C = s.C; a.H = s.H; a.W = s.W;
    a.Wp = s.W + 2; a.Hp = s.H + 1;
    a.div_wp = make_fastdiv((uint32_t)a.Wp);
    a.div_hp = make_fastdiv((uint32_t)a.Hp);
    a.aw = WH_STEP % a.Wp;
    a.ag = (WH_STEP / a.Wp) % a.Hp;
    a.an = (WH_STEP / a.Wp) / a.Hp;
    a.steps_per_split = p.steps_per_split;
    a.nsteps = p.nsteps;
    a.mode = mode;
    a.slab_stride = slab ? n : 0;
    a.zero = zero_n > 0 ? zero : nullptr;
    a.zero_n = zero_n;
    run_wh<1, 4, 1>(a, nb, st);
  } else {
    WgArgs a{};
    a.dy = dy; a.x = x;
    a.out = slab ? ws : dw;
    a.dy_bytes = dy_bytes; a.x_bytes = x_bytes;
    a.Mred = s.N * s.Ho * s.Wo; a.Kout = s.K; a.Ncols = s.R * s.S * s.C;
    a.H = s.H; a.W = s.W; a.C = s.C; a.S = s.S; a.stride = s.stride; a.pad = s.pad; a.stride_w = s.sw();
    a.HoWo = s.Ho * s.Wo; a.Wo = s.Wo; a.Ho = s.Ho;
    a.div_hw = make_fastdiv((uint32_t)a.HoWo);
    a.div_w = make_fastdiv((uint32_t)s.Wo);
    a.steps_per_split = p.steps_per_split;
    a.nsteps = p.nsteps;
    a.adv_r = 64 % s.Wo;
    a.adv_qh = (64 / s.Wo) % s.Ho;
    a.adv_qn = (64 / s.Wo) / s.Ho;
    a.mode = mode;
    a.slab_stride = slab ? n : 0;
    a.zero = zero_n > 0 ? zero : nullptr;
    a.zero_n = zero_n;
    const bool pw = s.R == 1 && s.S == 1 && s.stride == 1 && s.sw() == 1 && s.pad == 0 &&
                    s.H == s.Ho && s.W == s.Wo;
    if (p.wm == 2) { if (pw) run_wg<2, 2, true>(a, nb, st); else run_wg<2, 2, false>(a, nb, st); }
    else if (p.wm == 1) { if (pw) run_wg<1, 4, true>(a, nb, st); else run_wg<1, 4, false>(a, nb, st); }
    else { if (pw) run_wg<4, 1, true>(a, nb, st); else run_wg<4, 1, false>(a, nb, st); }
  }
  if (slab) {
    if (n % 4 != 0) throw std::runtime_error("conv_wgrad: dW size must be a multiple of 4 floats");
    const int64_t n4 = n / 4;
    hipLaunchKernelGGL(wg_splitk_reduce_kernel, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(ws), p.splits, n4, reinterpret_cast<float4*>(dw),
                       accumulate ? 1 : 0);
    wg_check("splitk_reduce");
  }
}

}  // namespace pdt
