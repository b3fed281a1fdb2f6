// Host-side launchers of the gfx950 kernels.  Plain C++ signatures (raw device
// pointers + hipStream_t) so the .hip translation units compile without any
// PyTorch headers; csrc/bindings.cpp adapts them to torch tensors.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

// ---------------------------------------------------------------- layout.hip
// NCHW fp32 image -> NHWC bf16 padded to Cp channels (Cp % 8 == 0).
void launch_image_to_nhwc(const float* x, uint16_t* y, int N, int C, int H, int W, int Cp,
                          hipStream_t st);
// fp32 weight [K][C][R][S] with arbitrary strides -> bf16 [K][R][S][Cp] (zero pad c >= C)
void launch_pack_weight(const float* w, const int64_t* strides, uint16_t* out, int K, int C,
                        int R, int S, int Cp, hipStream_t st);
// fp32 weight [K][C][R][S] -> bf16 [C][R][S][K] (dgrad B operand; no flip, taps indexed explicitly)
// batched CRSK pack of many KRSC bf16 weights living in one flat mirror (same offsets in dst);
// table = device array of ntensors entries of pack_t_entry_bytes() bytes:
// {int64 off; int K, C, RS, tiles_k = ceil(K/64), tiles_c = ceil(C/64)}; K, C multiples of 8
void launch_pack_t_batched(const uint16_t* src, uint16_t* dst, const void* table, int ntensors,
                           int max_tiles, hipStream_t st);
size_t pack_t_entry_bytes();
// Stem (7x7/s2, C <= 4) as a "super-pixel" conv: pairs of horizontally adjacent input pixels
// become one 8-channel pixel (4 channels each), the 7 horizontal taps fold into 4 tap pairs, and
// the image is pre-padded, so the conv is R x 4 taps, stride (2, 1), pad 0, C = 8:
// K_gemm = 7*4*8 = 224 instead of 7*7*8 = 392, and no bounds checks in the A loads.
// xsp[N][H+2pad][Wsp][q*4+c] = x[n][c][hp-pad][2*ws+q-pad-1] (0 outside / c >= C)
void launch_stem_image(const float* x, uint16_t* xsp, int N, int C, int H, int W, int pad, int Hp,
                       int Wsp, hipStream_t st);
// wsp[k][r][p][q*4+c] = w[k][c][r][2p+q-1] (0 outside), w fp32 with strides
// Halo-staged stem forward (stem.hip): y[N][Ho][Wo][64] = conv(xsp, wsp) with K = 64, R = 7,
// Sp = 4 super-pixel taps, stride (2, 1); part (optional) = BN partials [N*Ho][2][64], one group
// per output row (Wo rows each).  Supported when stem_halo_supported(K, R, Sp, Wo).
bool stem_halo_supported(int K, int R, int Sp, int Wo);
void launch_stem_conv_fwd(const uint16_t* xsp, const uint16_t* wsp, uint16_t* y, float* part, int N, int Hp,
                          int Wsp, int Ho, int Wo, hipStream_t st);
// Fused stem backward (stem.hip): dwsp[64][7][4][8] (fp32) = weight gradient of the super-pixel
// stem conv for dy = BN-backward-apply(maxpool_bwd(dpool, idx)) computed on the fly (ReLU mask from
// y, training-mode or eval apply with stats [4][64], gamma, sums [2][64]).  ws: null (fp32 atomics)
// or stem_bwd_fused_blocks(N, Ho) * 64 * 224 floats (deterministic slabs).
bool stem_bwd_fused_supported(int K, int R, int Sp, int Ho, int Wo);
int stem_bwd_fused_blocks(int N, int Ho);
void launch_stem_bwd_fused(const uint16_t* dpool, const uint8_t* idx, const uint16_t* y, const float* stats,
                           const float* gamma, const float* sums, bool training, const uint16_t* xsp, int N,
                           int Ho, int Wo, int Hp, int Wsp, float* dwsp, float* ws, hipStream_t st);
void launch_stem_pack_weight(const float* w, const int64_t* strides, uint16_t* wsp, int K, int C,
                             int R, int S, int Sp, hipStream_t st);
// out[k][c][r][s] (+)= dwsp[k][r][(s+1)/2][((s+1)%2)*4+c], out channels_last (strides k:CRS... given)
void launch_stem_wgrad_unpack(const float* dwsp, float* out, const int64_t* strides, int K, int C,
                              int R, int S, int Sp, bool accumulate, hipStream_t st);
void launch_pack_weight_t(const float* w, const int64_t* strides, uint16_t* out, int K, int C,
                          int R, int S, hipStream_t st);

// ---------------------------------------------------------- conv_igemm.hip
struct ConvShape {
  int N, H, W, C;      // input activation (C = channel stride, multiple of 8)
  int K, R, S;         // filter: K outputs, RxS taps
  int Ho, Wo;          // output spatial
  int stride, pad;
  int stride_w = 0;    // horizontal stride when different from `stride` (fwd and wgrad only)
  int sw() const { return stride_w > 0 ? stride_w : stride; }
};
// y[N,Ho,Wo,K] = conv(x, w[K][R][S][C]); if part != nullptr also writes per-group
// BN partials part[ceil(M/G)][2][K] = (sum, M2 about the group mean), G = conv_nt_group_rows(M, K,
// R*S*C*elem_bytes) = the BM of the workgroup tile the launch uses (one group per row tile).
int conv_nt_group_rows(int M, int Nout, int kg_bytes);
// (BM, BN) of the NT workgroup tile the fwd / dgrad launch of such a GEMM runs (test introspection)
void conv_nt_tile(int M, int Nout, int kg_bytes, int* bm, int* bn);
// tests: force the NT main loop (k32 1 / 0) and disable the 128x256 tile (mid 0); -1 = policy
void conv_nt_force(int k32, int mid, int wide = -1);
// number of stream-K NT launches so far in this process (tests: which path ran)
// PDT_NT_TIMING builds (scripts/build_variant.sh): per-workgroup phase timestamps of NT launches
// (s_memtime at start / first operands in LDS / main loop done / epilogue stats done / end, plus
// s_memrealtime and the CU id), 8 values per block id, copied into `host`; other builds return 0.
int nt_timing_fetch(unsigned long long* host, int n);
// BatchNorm statistics as fp64 totals (non-deterministic training runs): every workgroup of the
// forward conv adds its per-channel sum and sum of squares of the bf16 output to acc[2][K] (agent-
// scope atomics, no partials buffer); then launch_bn_finalize_sums (one thread per channel) turns
// them into out[4][K] (mean, invstd, scale, shift), updates the running statistics and re-zeroes acc.
constexpr int kStatSlots = 8;  // acc slots: one per XCD
struct BnFwdFuse {
  double* acc;           // [kStatSlots][2][K], zero on entry, zero again on exit
  const float* gamma;
  const float* beta;
  float* rm;             // running mean / var, or null
  float* rv;
  float* out;            // [4][K]
  float momentum, eps;
};
void launch_bn_finalize_sums(const BnFwdFuse& bn, int M, int K, hipStream_t st);
void launch_conv_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part,
                     const ConvShape& s, hipStream_t st, const BnFwdFuse* bn = nullptr);
// dx[N,H,W,C] = dgrad(dy[N,Ho,Wo,K], wt[C][R][S][K]) (+ addend[N,H,W,C] if non-null);
// all stride/pad combos (stride > 1 as stride^2 parity classes)
// Optional fused BatchNorm backward of the unit whose output x was (dx = dL/dx of that unit's
// activation): the kernel stores g = dx * relu'(.) instead of dx (mask 0: none, 1: z > 0,
// 2: y*scale + shift > 0) and writes per-row-group partials part[G][2][C] of
// (sum g, sum g*(y - mean)), G = conv_dgrad_bn_groups(s, bytes per dy element); reduce them with
// launch_bn_bwd_part_reduce.
struct BnBwdFuse {
  const uint16_t* y;     // [N,H,W,C] pre-BN output of that unit
  const uint16_t* z;     // [N,H,W,C] its activation output (mask 1), its ReLU bitmask (mask 3:
                         // uint8 [N*H*W*C/8], bit q of byte i = z[8i + q] > 0), or null
  const float* stats;    // [4][C] mean, invstd, scale, shift
  float* part;           // [G][2][C]
  int mask;
  float* acc = nullptr;  // non-null: partials fp32-atomically summed into [2][C] (part unused)
  // optional second BN fed by the same g (a downsampling block's projection-shortcut BN): its y,
  // statistics and [2][C] accumulator of (sum g, sum g*(y2 - mean2)); acc mode, mask 3, addend only
  const uint16_t* y2 = nullptr;
  const float* stats2 = nullptr;
  float* acc2 = nullptr;
};
int conv_dgrad_bn_groups(const ConvShape& s, int elem_bytes = 2);
// addend_sub = 2: addend is a compact [N, ceil(H/2), ceil(W/2), C] map added at even (h, w) only
// (the input gradient of a 1x1/s2 projection shortcut, computed as a dense 1x1 dgrad)
// BN backward folded into a 1x1 / stride-1 input gradient (ops/fused.py, last unit of a
// bottleneck): with dy = k1*g + a*y + b per output channel k (the BN-backward apply written out) and
// y = W z (the conv's own output), dx = W^T diag(k1) g + (W^T diag(a) W) z + W^T b -- one GEMM over
// the K-concatenation [g | z] with B rows [wt*k1 | G] (bn_fold_weights) plus a per-channel bias, so
// the apply that materialises dy leaves the critical path (it still feeds the weight gradient).
struct DgradFold {
  const uint16_t* a2;  // z: [M][CA2] bf16, the conv input (CA2 = its channels = the dgrad's Nout)
  int CA2;
  const float* bias;   // [Nout] fp32
};
// wfold[C][K + C] bf16 and bias[C] fp32 (followed by 2K floats of scratch) of a DgradFold for the
// 1x1 conv with transposed bf16
// weights wt[C][K], BN statistics stats[4][K] (mean, invstd, ...), gamma[K] and backward sums
// sums[2][K] (sum g, sum g*(y - mean)) over M rows
int64_t bn_fold_weights_ws_floats(int C, int K);  // bias + coefficient / partials scratch
void launch_bn_fold_weights(const uint16_t* wt, const float* stats, const float* gamma, const float* sums,
                            int M, int C, int K, uint16_t* wfold, float* bias, hipStream_t st);
// its weight gradient: out[K][C] += diag(k1) t1 + diag(a) W gram + b colsum^T (t1 = g^T x [K][C],
// gram = x^T x [C][C], colsum = sum of x [C], W from the bf16 mirror wt[C][K]); dgamma/dbeta (optional)
// += s1 * invstd, s0.  done != null: consume mode -- t1, gram (and sums if zero_sums) are cleared for
// their next use (done: an int completion counter, 0 between launches)
void launch_bn_fold_wgrad(float* t1, float* gram, const float* colsum, const uint16_t* wt,
                          const float* stats, const float* gamma, const float* sums, int M, int C, int K,
                          float* out, float* dgamma, float* dbeta, int* done, bool zero_sums, hipStream_t st,
                          int csum_slots = 1);  // bn_csum_slots(): bn_act_fwd's [slots][C], re-zeroed here
void launch_conv_dgrad(const uint16_t* dy, const uint16_t* wt, uint16_t* dx, const uint16_t* addend,
                       const ConvShape& s, hipStream_t st, const BnBwdFuse* bn = nullptr,
                       int addend_sub = 0, const DgradFold* fold = nullptr);
// dw[K][R][S][C] (fp32) = wgrad(dy, x).  Split-K partials are combined with fp32 atomics, or
// (deterministic) in private slabs ws[conv_wgrad_ws_floats()] reduced in fixed order.
size_t conv_wgrad_ws_floats(const ConvShape& s, bool deterministic);
// the weight-gradient launch plan: {tile rows (output channels), tile cols, tiles, split-K factor}
void conv_wgrad_plan(const ConvShape& s, bool deterministic, int out[4]);
// CUs the weight-gradient split-K plan leaves free for collective kernels (0: plan the whole chip)
void conv_wgrad_set_cu_reserve(int n);
int conv_wgrad_cu_reserve();
// accumulate: dw += wgrad (autograd accumulation semantics; lets the block write straight into
// the flat gradient buffer), else dw = wgrad.
// fp8 weight gradient: dw[K][R][S][C] (+)= wgrad(dy8 e5m2 [N,Ho,Wo,K] * dy_deq, x8 e4m3 [N,H,W,C] * x_deq),
// fp32 atomics (non-deterministic order); C % 16 == 0, K % 64 == 0.  plan: (bmg, tiles, splits, steps/split)
void conv_wgrad_fp8_plan(const ConvShape& s, int out[4]);
void launch_conv_wgrad_fp8(const uint8_t* dy8, const uint8_t* x8, const float* dy_deq, const float* x_deq,
                           float* dw, const ConvShape& s, bool accumulate, hipStream_t st);
// zero / zero_n: optional fp32 buffer the weight-gradient kernel clears (workgroup 0) -- the BN-sum
// accumulator whose consumer is ordered before this launch (ops/fused.py _BN_ACC)
void launch_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* dw, float* ws,
                       const ConvShape& s, bool deterministic, bool accumulate, hipStream_t st,
                       float* zero = nullptr, int zero_n = 0);

// -------------------------------------------------------------- bn_act.hip
// part[ngroups][2][K] (group g has min(grows, M-grows*g) rows) -> out[4][K] = mean, invstd,
// scale, shift; updates running stats in place (unbiased var) when rm/rv non-null.
// `out` must have room for 4*K + 3*K*bn_finalize_partitions(ngroups) floats (stage-1 scratch).
int bn_finalize_partitions(int ngroups);
// completion-counter bank of a stream's single-launch BN reductions, -1 = two-launch path
int bn_counter_bank(hipStream_t st);
void launch_bn_finalize(const float* part, int ngroups, int grows, int M, int K, float* rm, float* rv,
                        const float* gamma, const float* beta, float momentum, float eps,
                        float* out, hipStream_t st);
void launch_bn_eval_params(const float* rm, const float* rv, const float* gamma, const float* beta,
                           float eps, int K, float* out, hipStream_t st);
// z = act(y*scale + shift (+res)); zmask (optional, with relu): one byte per 8 channels, bit q =
// z[8i + q] > 0 -- the ReLU mask a later backward reads instead of z (1/16 of the bytes)
// rscale/rshift (optional): the residual is a raw conv output to normalise as bf16(res*rscale +
// rshift) first -- a downsampling block's projection shortcut, whose BN apply is fused here
void launch_bn_act_fwd(const uint16_t* y, const float* scale, const float* shift,
                       const uint16_t* res, bool relu, uint16_t* z, int64_t M, int K,
                       hipStream_t st, uint8_t* zmask = nullptr, const float* rscale = nullptr,
                       const float* rshift = nullptr, float* csum = nullptr);  // csum: [bn_csum_slots()][K]
int bn_csum_slots();
// Backward BN.  stats = bn_finalize output [4][K] (mean, invstd, scale, shift).  mask: 0 = no
// ReLU, 1 = ReLU mask from z (> 0), 2 = ReLU mask recomputed from y (y*scale + shift > 0).
// sums[2][K] = (sum g, sum g*(y-mean)) with g = dz * mask; ws >= bn_bwd_ws_floats(M, K)
size_t bn_bwd_ws_floats(int64_t M, int K);
// If dgamma/dbeta are non-null the final stage also accumulates dgamma += sum_gx*invstd and
// dbeta += sum_g into them (parameter gradients written in place).
// Reduce row-group partials part[G][2][K] (from a BN-fused dgrad) to sums[2][K]; ws holds
// bn_bwd_part_ws_floats(G, K) floats.  Optional dgamma += sum_b*invstd, dbeta += sum_a.
size_t bn_bwd_part_ws_floats(int G, int K);
void launch_bn_bwd_part_reduce(const float* part, int G, int K, float* ws, float* sums,
                               const float* invstd, float* dgamma, float* dbeta, hipStream_t st);
void launch_bn_act_bwd_reduce(const uint16_t* dz, const uint16_t* z, const uint16_t* y,
                              const float* stats, int mask, int64_t M, int K, float* ws,
                              float* sums, float* dgamma, float* dbeta, hipStream_t st);
// dy = gamma*invstd*(g - sum_g/M - (y-mean)*sum_gx*invstd^2/M) (training) or gamma*invstd*g;
// dres = g (if non-null)
void launch_bn_act_bwd_apply(const uint16_t* dz, const uint16_t* z, const uint16_t* y,
                             const float* stats, const float* gamma, const float* sums, int mask,
                             bool training, int64_t M, int K, uint16_t* dy, uint16_t* dres,
                             hipStream_t st, float* dgamma = nullptr, float* dbeta = nullptr);
// dgamma/dbeta (optional): += sums[1]*invstd, += sums[0] (the BN parameter gradients, for sums
// accumulated by the producing dgrad's epilogue atomics -- BnBwdFuse::acc)

// Stem BN + ReLU + 3x3/s2/p1 max pool fused (bn_act.hip): out/idx as maxpool_fwd of the ReLU'd
// bf16 z, which is never written.  Backward: the BN reduction / apply with dz gathered from the
// pooled gradient (mask mode 2); ws >= pool_bn_bwd_ws_floats(N*H*W, K).  K <= 256.
void launch_bn_relu_maxpool(const uint16_t* y, const float* scale, const float* shift, uint16_t* out,
                            uint8_t* idx, uint16_t* uarg, int N, int H, int W, int C, int Ho, int Wo,
                            hipStream_t st);
size_t pool_bn_bwd_ws_floats(int64_t M, int K);
void launch_pool_bn_bwd_reduce(const uint16_t* dpool, const uint8_t* idx, const uint16_t* y,
                               const float* stats, int N, int H, int W, int K, int Ho, int Wo,
                               float* ws, float* sums, float* dgamma, float* dbeta, hipStream_t st);
void launch_pool_bn_bwd_apply(const uint16_t* dpool, const uint8_t* idx, const uint16_t* y,
                              const float* stats, const float* gamma, const float* sums, bool training,
                              int N, int H, int W, int K, int Ho, int Wo, uint16_t* dy, hipStream_t st);

// ---------------------------------------------------------------- pool.hip
void launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C,
                        int Ho, int Wo, hipStream_t st);
void launch_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W,
                        int C, int Ho, int Wo, hipStream_t st);
void launch_avgpool_fwd(const uint16_t* x, float* y, int N, int HW, int C, hipStream_t st);
// dy = sum of `splits` consecutive [N][C] partials (a split-K fc dgrad), summed in order
void launch_avgpool_bwd(const float* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st, int splits = 1);

// ------------------------------------------------------------------ fc.hip
// C(m, n) = alpha * sum_k A(m, k) B(k, n) (+ bias[n]) on the bf16 MFMA (fp32 accumulate), with
// A(m, k) = a[m*sam + k*sak], B(k, n) = b[n*sbn + k*sbk]; alpha: device scalar or null (1).
// splits > 1: slice z of K (kper each) writes ws[z][M][N], summed by fc_splitk_reduce (+ bias) or
// by the consumer; splits == 1 writes c (row stride ldc), accumulating when `accumulate`.
// db (optional, row-contiguous A and splits == 1 only): db[m] (+)= alpha * sum_k A(m, k), taken in
// fp32 from the same A loads (the fc bias gradient rides on the dW product).
struct FcArgs {
  const float* a; const float* b; float* c; float* ws; const float* bias; const float* alpha; float* db;
  int M, N, K;
  int64_t sam, sak, sbn, sbk;
  int ldc, splits, kper, accumulate;
};
int fc_splits(int M, int N, int K);
void launch_fc_gemm(const FcArgs& a, hipStream_t st);
void launch_fc_splitk_reduce(const float* ws, int splits, int M, int N, const float* bias, float* c,
                             int ldc, hipStream_t st);
void launch_fc_colsum(const float* g, int rows, int cols, const float* alpha, float* db, bool accumulate,
                      hipStream_t st);

// ---------------------------------------------------------------- head.hip
// loss[0] = mean CE, dlogits = (softmax - onehot)/N ; ws >= N floats
void launch_softmax_xent(const float* logits, const int64_t* labels, float* loss, float* dlogits,
                         float* ws, int N, int V, hipStream_t st);
void launch_top1(const float* logits, const int64_t* labels, int64_t* count, int N, int V,
                 hipStream_t st);
// x[i] += 1 (the BatchNorm num_batches_tracked counters, one flat int64 buffer)
void launch_add_one_i64(int64_t* x, int64_t n, hipStream_t st);
// y = x * alpha[0], alpha a device scalar (x, y 16-byte aligned fp32)
void launch_scale(const float* x, const float* alpha, float* y, int64_t n, hipStream_t st);

// ----------------------------------------------------------------- sgd.hip
// torch.optim.SGD on flat fp32 buffers; grad is scaled by grad_scale first.
void launch_sgd(float* p, const float* g, float* buf, int64_t n, float lr, float momentum,
                float dampening, float wd, bool nesterov, bool first, float grad_scale,
                hipStream_t st, uint16_t* p_bf16 = nullptr);
// fp32 -> bf16 cast (used for bf16 gradient buckets) and back
void launch_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st);
void launch_cast_bf16_f32(const uint16_t* x, float* y, int64_t n, float scale, hipStream_t st);

// ------------------------------------------------------------- augment.hip
// Fused gather + RandomCrop(pad) + RandomHorizontalFlip + (/255) + Normalize of a device-resident
// NCHW dataset (uint8 or fp32) into fp32 NCHW out[B][C][H][W]; per-sample crop offsets oy/ox in
// [0, 2*pad] and flip flags (may be null) are drawn by the caller.  mean/std: host arrays of 3.
void launch_augment(const void* src, bool src_u8, const int64_t* idx, const int64_t* oy, const int64_t* ox,
                    const bool* flip, float* out, int B, int C, int H, int W, int pad, bool normalize,
                    const float* mean, const float* stdv, hipStream_t st);

// ----------------------------------------------------------------- fp8.hip
// One v_mfma_scale_f32_16x16x128_f8f6f4 on raw per-lane operand registers (64 lanes x 32 bytes
// each for A and B), D = 64 lanes x 4 fp32.  fmt 0 = e4m3, 1 = e5m2; scales are E8M0 bytes
// (use_scale = 0 passes the literal 0 the way composable_kernel does).
void launch_mfma_f8_probe(const void* a_regs, const void* b_regs, float* d, int fmt_a, int fmt_b,
                          int scale_a, int scale_b, int use_scale, hipStream_t st);
struct WStridesF8 { int64_t k, c, r, s; };
// fp32 weight [K][C][R][S] (strides) -> e4m3 [K][R][S][Cp] with per-output-channel scale
// ws_k = amax_k/448; oscale[k] = ws_k * act_deq[0] (act_deq may be null: 1) is the conv
// epilogue's dequantization factor for column k.
void launch_pack_weight_fp8(const float* w, const int64_t* strides, uint8_t* wq, float* oscale,
                            const float* act_deq, int K, int C, int R, int S, int Cp, hipStream_t st);
// Delayed-scaling state: float[fp8_state_floats()] = sharded amax of the last 3 calls, then their
// dequant factors; `slot` = call index % 3 (kept by the caller).  The dequant factor of this call
// lands in state[fp8_deq_offset() + slot].
int fp8_state_floats();
int fp8_deq_offset();
void launch_quant_e4m3(const uint16_t* x, uint8_t* q, int64_t n, float* state, int slot, hipStream_t st);
// bn_act_fwd that also writes the e4m3 copy q of z (same delayed-scaling contract)
void launch_bn_act_fwd_q8(const uint16_t* y, const float* scale, const float* shift, const uint16_t* res,
                          bool relu, uint16_t* z, uint8_t* q, int64_t M, int K, float* state, int slot,
                          hipStream_t st, uint8_t* zmask = nullptr);
// Batched row-wise e4m3 quantization of bf16 weight images in a flat mirror: table = device
// array of ntensors {int64 off (elements, same in src and dst), int64 soff (first scale index),
// int rows, int rowlen (multiple of 8)}; scale[soff + row] = amax(row) / 448.
void launch_quant_rows_e4m3(const uint16_t* src, uint8_t* dst, float* scale, const void* table,
                            int ntensors, int max_rows, hipStream_t st);
size_t quant_rows_entry_bytes();
// fp8 forward conv: x e4m3 NHWC (C % 16 == 0), w e4m3 [K][R][S][C],
// y bf16 = (x*w) * oscale[k] * (ascale ? ascale[0] : 1)
void launch_conv_fwd_fp8(const uint8_t* x, const uint8_t* w, const float* oscale, const float* ascale,
                         uint16_t* y, float* part, const ConvShape& s, hipStream_t st,
                         const BnFwdFuse* bn = nullptr);
// fp8 dgrad: dy e5m2 NHWC (K % 128 == 0), wt e4m3 [C][R][S][K] with per-C scale oscale[c],
// activation (dy) dequant factor ascale[0]; otherwise as launch_conv_dgrad
void launch_conv_dgrad_fp8(const uint8_t* dy, const uint8_t* wt, const float* oscale, const float* ascale,
                           uint16_t* dx, const uint16_t* addend, const ConvShape& s, hipStream_t st,
                           const BnBwdFuse* bn = nullptr, int addend_sub = 0);
// bn_act_bwd_apply that also writes dy8 = e5m2(bf16(dy) * s_t) (delayed scaling, fp8 state contract)
void launch_bn_act_bwd_apply_q8(const uint16_t* dz, const uint16_t* z, const uint16_t* y,
                                const float* stats, const float* gamma, const float* sums, int mask,
                                bool training, int64_t M, int K, uint16_t* dy, uint16_t* dres,
                                uint8_t* dy8, float* state, int slot, hipStream_t st,
                                float* dgamma = nullptr, float* dbeta = nullptr);

// ---------------------------------------------------------------- xgmi.hip
// Direct one-hop all-reduce of elements [lo, lo + count) of every rank's fp32 gradient buffer
// (bucket `bucket`, epoch `epoch`): (bf16 wire: pack) signal ready -> wait (bounded) -> reduce own
// shard from all peers -> signal reduced -> wait -> gather every shard back (divided by world when
// `average`).  Buffers: device pointers of every rank's buffers as mapped in this process (g16 /
// red16 null: fp32 wire); err: device view of a host word set to a nonzero code when a wait passes
// timeout_ticks (wall clock) or a peer signalled POISON (failed).  The data kernels use at most
// `max_blocks` workgroups (the CU budget beside the backward pass).
constexpr unsigned kXgmiPeerFailed = 0x80000000u;  // err | (peer << 16) | code: a peer failed first
struct XgmiBuffers {
  const float* g[8];
  const float* red[8];
  unsigned* flags[8];
  const uint16_t* g16[8];
  const uint16_t* red16[8];
};
int xgmi_max_ranks();
int xgmi_slots_per_bucket();   // flag slots per bucket: ready + one reduced slot per chunk
void xgmi_force_chunks(int n);  // test hook: chunks per bucket (1..4), -1 = size policy
int64_t xgmi_shard(int64_t lo, int64_t count, int world);
void launch_xgmi_bucket(const XgmiBuffers& bufs, int world, int rank, int bucket, int64_t lo, int64_t count,
                        unsigned epoch, bool average, uint64_t timeout_ticks, unsigned* err, hipStream_t st,
                        int phase_lo = 0, int phase_hi = 5, int max_blocks = 16);

}  // namespace pdt
