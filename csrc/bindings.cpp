// Python bindings of the native extension `pytorch_distributed_tutorials_amd._C`.
//
// Adapts torch tensors to the raw-pointer launchers of csrc/kernels (which are
// compiled without any PyTorch headers), allocates outputs/workspaces through
// the PyTorch caching allocator and launches on the current HIP stream, so the
// ops compose with autograd, streams and graph capture.  Also exposes the RCCL
// communicator and the gradient reducer.
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdlib>
#include <optional>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <unordered_map>

#include "comm/rccl_comm.h"
#include "comm/xgmi_comm.h"
#include "ddp/reducer.h"
#include "kernels/kernels.h"

namespace py = pybind11;
using at::Tensor;

namespace {

// ---------------------------------------------------------------- debug mode
// PDT_SYNC_CHECK=1 (or _C.set_sync_check(True)): every op synchronizes the device after its
// launches and turns an asynchronous kernel fault into an exception naming the op that caused
// it (the role CUDA_LAUNCH_BLOCKING / AMD_SERIALIZE_KERNEL play, scoped to this extension).
bool g_sync_check = [] {
  const char* e = std::getenv("PDT_SYNC_CHECK");
  return e && e[0] == '1';
}();

void sync_check(const char* op) {
  if (!g_sync_check) return;
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess)
    throw std::runtime_error(std::string("PDT_SYNC_CHECK: ") + op + ": " + hipGetErrorString(e));
}

template <typename R, typename... A>
auto checked(const char* op, R (*f)(A...)) {
  return [op, f](A... a) -> R {
    if constexpr (std::is_void_v<R>) {
      f(std::forward<A>(a)...);
      sync_check(op);
    } else {
      R r = f(std::forward<A>(a)...);
      sync_check(op);
      return r;
    }
  };
}

hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.get_device()).stream();
}

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_bf16_nhwc(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.dim() == 4, name, " must be 4-D NHWC");
  TORCH_CHECK(t.size(3) % 8 == 0, name, " channels must be a multiple of 8");
  TORCH_CHECK(t.numel() < (int64_t(1) << 30), name, " too large for 32-bit buffer addressing");
}

void check_state(const Tensor& st, int64_t slot) {
  check_cuda(st, "fp8 state");
  TORCH_CHECK(st.scalar_type() == at::kFloat && st.numel() == pdt::fp8_state_floats(),
              "fp8 state must be fp32 [fp8_state_floats()]");
  TORCH_CHECK(slot >= 0 && slot < 3, "fp8 slot must be 0..2");
}

void check_u8_nhwc(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kByte && t.dim() == 4, name, " must be uint8 (fp8 bits) NHWC");
  TORCH_CHECK(t.size(3) % 16 == 0, name, " channels must be a multiple of 16");
  TORCH_CHECK(t.numel() < (int64_t(1) << 31), name, " too large for 32-bit buffer addressing");
}

uint16_t* bf(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
const uint16_t* cbf(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }

// ------------------------------------------------------------------ layout
Tensor image_to_nhwc(const Tensor& x) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 4, "image must be fp32 NCHW");
  c10::hip::HIPGuard g(x.get_device());
  int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  int Cp = ((C + 7) / 8) * 8;
  auto y = at::empty({N, H, W, Cp}, x.options().dtype(at::kBFloat16));
  pdt::launch_image_to_nhwc(x.data_ptr<float>(), bf(y), N, C, H, W, Cp, cur_stream(x));
  return y;
}

Tensor pack_weight(const Tensor& w, int64_t cpad) {
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kFloat, "weight must be fp32 4-D");
  c10::hip::HIPGuard g(w.get_device());
  int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  int Cp = std::max<int>((int)cpad, C);
  auto out = at::empty({K, R, S, Cp}, w.options().dtype(at::kBFloat16));
  int64_t st[4] = {w.stride(0), w.stride(1), w.stride(2), w.stride(3)};
  pdt::launch_pack_weight(w.data_ptr<float>(), st, bf(out), K, C, R, S, Cp, cur_stream(w));
  return out;
}

Tensor pack_weight_t(const Tensor& w) {
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kFloat, "weight must be fp32 4-D");
  c10::hip::HIPGuard g(w.get_device());
  int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  auto out = at::empty({C, R, S, K}, w.options().dtype(at::kBFloat16));
  int64_t st[4] = {w.stride(0), w.stride(1), w.stride(2), w.stride(3)};
  pdt::launch_pack_weight_t(w.data_ptr<float>(), st, bf(out), K, C, R, S, cur_stream(w));
  return out;
}

// -------------------------------------------------------------------- conv
pdt::ConvShape shape_of(int N, int H, int W, int C, int K, int R, int S, int stride, int pad) {
  pdt::ConvShape s;
  s.N = N; s.H = H; s.W = W; s.C = C; s.K = K; s.R = R; s.S = S;
  s.stride = stride; s.pad = pad;
  s.Ho = (H + 2 * pad - R) / stride + 1;
  s.Wo = (W + 2 * pad - S) / stride + 1;
  return s;
}

// returns (y, part); part is empty when stats == false
std::tuple<Tensor, Tensor> conv_fwd(const Tensor& x, const Tensor& wk, int64_t stride, int64_t pad,
                                    bool stats) {
  check_bf16_nhwc(x, "x");
  check_cuda(wk, "wk");
  TORCH_CHECK(wk.dim() == 4 && wk.size(3) == x.size(3), "packed weight must be [K,R,S,Cx]");
  c10::hip::HIPGuard g(x.get_device());
  auto s = shape_of(x.size(0), x.size(1), x.size(2), x.size(3), wk.size(0), wk.size(1), wk.size(2),
                    stride, pad);
  TORCH_CHECK(s.K % 8 == 0, "output channels must be a multiple of 8");
  auto y = at::empty({s.N, s.Ho, s.Wo, s.K}, x.options());
  Tensor part;
  float* pp = nullptr;
  int M = s.N * s.Ho * s.Wo;
  if (stats) {
    int grows = pdt::conv_nt_group_rows(M, s.K, s.R * s.S * s.C * 2);
    int ng = (M + grows - 1) / grows;
    part = at::empty({ng, 2, s.K}, x.options().dtype(at::kFloat));
    pp = part.data_ptr<float>();
  }
  pdt::launch_conv_fwd(cbf(x), cbf(wk), bf(y), pp, s, cur_stream(x));
  return {y, part};
}

// Addend of a dgrad: the full [N,H,W,C] layout of dx (0), or a compact stride-2 map
// [N, ceil(H/2), ceil(W/2), C] that contributes at even (h, w) only (2).
static int addend_layout(const Tensor& addend, const Tensor& dx) {
  check_bf16_nhwc(addend, "addend");
  if (addend.sizes() == dx.sizes()) return 0;
  TORCH_CHECK(addend.size(0) == dx.size(0) && addend.size(1) == (dx.size(1) + 1) / 2 &&
              addend.size(2) == (dx.size(2) + 1) / 2 && addend.size(3) == dx.size(3),
              "dgrad addend must have the shape of dx or be its stride-2 compact map");
  return 2;
}

// wt: optional pre-packed bf16 [C][R][S][K] weights (flat-space dgrad mirror)
Tensor packed_t_or_pack(const Tensor& w, const std::optional<Tensor>& wt) {
  if (wt.has_value() && wt->defined()) {
    TORCH_CHECK(wt->scalar_type() == at::kBFloat16 && wt->is_contiguous() && wt->dim() == 4 &&
                wt->size(0) == w.size(1) && wt->size(1) == w.size(2) && wt->size(2) == w.size(3) &&
                wt->size(3) == w.size(0), "wt must be bf16 [C,R,S,K] contiguous");
    return *wt;
  }
  return pack_weight_t(w);
}

Tensor conv_dgrad(const Tensor& dy, const Tensor& w, std::vector<int64_t> xs, int64_t stride,
                  int64_t pad, const std::optional<Tensor>& addend, const std::optional<Tensor>& wt_in) {
  check_bf16_nhwc(dy, "dy");
  TORCH_CHECK(xs.size() == 4, "x shape must be NHWC");
  TORCH_CHECK(xs[3] == w.size(1), "dgrad: x channels must equal weight in-channels");
  c10::hip::HIPGuard g(dy.get_device());
  auto s = shape_of(xs[0], xs[1], xs[2], xs[3], w.size(0), w.size(2), w.size(3), stride, pad);
  TORCH_CHECK(s.Ho == dy.size(1) && s.Wo == dy.size(2) && s.K == dy.size(3), "dgrad: dy shape mismatch");
  Tensor wt = packed_t_or_pack(w, wt_in);
  auto dx = at::empty({s.N, s.H, s.W, s.C}, dy.options());
  const uint16_t* ap = nullptr;
  int asub = 0;
  if (addend.has_value() && addend->defined()) {
    asub = addend_layout(*addend, dx);
    ap = cbf(*addend);
  }
  pdt::launch_conv_dgrad(cbf(dy), cbf(wt), bf(dx), ap, s, cur_stream(dy), nullptr, asub);
  return dx;
}

// dgrad with the BatchNorm backward of the unit that produced x fused into the epilogue:
// returns (g, sums) with g = dx * relu'(unit) (mask 0/1/2 as bn_act_bwd_reduce) and
// sums[2][C] = (sum g, sum g*(y - mean)); optional dgamma/dbeta accumulate like
// bn_act_bwd_reduce.  bn_act_bwd_apply(g, ..., mask=0) then yields that unit's dy.
// shared body of conv_dgrad_bn / conv_dgrad_bn_fp8: `launch(s, dx, addend, bn, stream)` runs the
// BN-fused dgrad
// optional second BN on the same gradient (kernels.h BnBwdFuse::y2): a downsampling block's
// projection-shortcut BN, reduced by the same epilogue into its own [2][C] accumulator
struct SecondBn {
  std::optional<Tensor> y, stats, acc;
};

template <typename Launch>
std::tuple<Tensor, Tensor> dgrad_bn_core(const Tensor& dy_like, const pdt::ConvShape& s,
                                         const std::optional<Tensor>& addend, const Tensor& y,
                                         const std::optional<Tensor>& z, const Tensor& stats, int64_t mask,
                                         const std::optional<Tensor>& dgamma,
                                         const std::optional<Tensor>& dbeta, const std::optional<Tensor>& acc,
                                         const SecondBn& bn2, Launch&& launch) {
  check_bf16_nhwc(y, "y");
  TORCH_CHECK(y.size(0) == s.N && y.size(1) == s.H && y.size(2) == s.W && y.size(3) == s.C,
              "dgrad_bn: y must have the shape of x");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.numel() == 4 * s.C && stats.is_contiguous(),
              "stats must be fp32 [4, C]");
  TORCH_CHECK(mask >= 0 && mask <= 3, "mask must be 0, 1, 2 or 3");
  const uint16_t* zp = nullptr;
  if (mask == 1) {
    TORCH_CHECK(z.has_value() && z->defined(), "mask 1 needs z");
    check_bf16_nhwc(*z, "z");
    TORCH_CHECK(z->sizes() == y.sizes(), "z shape mismatch");
    zp = cbf(*z);
  } else if (mask == 3) {  // ReLU bitmask from bn_act_fwd_mask: one byte per 8 channels
    TORCH_CHECK(z.has_value() && z->defined(), "mask 3 needs the ReLU bitmask");
    check_cuda(*z, "zmask");
    TORCH_CHECK(z->scalar_type() == at::kByte && z->numel() * 8 == y.numel(), "zmask must be uint8 [numel/8]");
    zp = reinterpret_cast<const uint16_t*>(z->data_ptr());
  }
  auto dx = at::empty({s.N, s.H, s.W, s.C}, y.options());
  const uint16_t* ap = nullptr;
  int asub = 0;
  if (addend.has_value() && addend->defined()) {
    asub = addend_layout(*addend, dx);
    ap = cbf(*addend);
  }
  hipStream_t st = cur_stream(dy_like);
  if (acc.has_value() && acc->defined()) {
    // partials fp32-atomically summed by the epilogue into the caller's zeroed [2][C] accumulator:
    // no partial buffer, no reduce launch; the BN parameter gradients are added by the consuming
    // bn_act_bwd_apply(dgamma=, dbeta=), which runs after the sums are complete
    TORCH_CHECK(acc->is_cuda() && acc->scalar_type() == at::kFloat && acc->is_contiguous() &&
                acc->numel() == 2 * s.C, "acc must be a contiguous fp32 [2, C] device tensor");
    TORCH_CHECK(!(dgamma.has_value() && dgamma->defined()), "acc mode: pass dgamma/dbeta to the apply");
    pdt::BnBwdFuse bn{cbf(y), zp, stats.data_ptr<float>(), nullptr, (int)mask, acc->data_ptr<float>()};
    if (bn2.y.has_value() && bn2.y->defined()) {
      check_bf16_nhwc(*bn2.y, "y2");
      TORCH_CHECK(bn2.y->sizes() == y.sizes(), "y2 must have the shape of y");
      TORCH_CHECK(bn2.stats.has_value() && bn2.stats->defined() && bn2.stats->numel() == 4 * s.C &&
                  bn2.stats->scalar_type() == at::kFloat && bn2.stats->is_contiguous(), "stats2 must be fp32 [4, C]");
      TORCH_CHECK(bn2.acc.has_value() && bn2.acc->defined() && bn2.acc->numel() == 2 * s.C &&
                  bn2.acc->scalar_type() == at::kFloat && bn2.acc->is_contiguous() && bn2.acc->is_cuda(),
                  "acc2 must be a contiguous fp32 [2, C] device tensor");
      TORCH_CHECK(mask == 3 && ap != nullptr, "the second BN needs mask 3 and the residual addend");
      bn.y2 = cbf(*bn2.y);
      bn.stats2 = bn2.stats->data_ptr<float>();
      bn.acc2 = bn2.acc->data_ptr<float>();
    }
    launch(s, bf(dx), ap, &bn, st, asub);
    return {dx, acc->view({2, s.C})};
  }
  const int G = pdt::conv_dgrad_bn_groups(s, (int)dy_like.element_size());
  auto fopt = y.options().dtype(at::kFloat);
  // sums, partials and the reduction workspace as slices of ONE allocation (host issue: each
  // caching-allocator call is ~1-2 us, and this binding runs once per BatchNorm per step)
  const int64_t n_sums = 2 * (int64_t)s.C, n_part = (int64_t)G * 2 * s.C;
  const int64_t n_ws = (int64_t)pdt::bn_bwd_part_ws_floats(G, s.C);
  auto fbuf = at::empty({n_sums + n_part + n_ws}, fopt);
  auto sums = fbuf.narrow(0, 0, n_sums).view({2, s.C});
  auto part = fbuf.narrow(0, n_sums, n_part);
  auto ws = fbuf.narrow(0, n_sums + n_part, n_ws);
  TORCH_CHECK(!(bn2.y.has_value() && bn2.y->defined()), "the second BN needs acc mode");
  pdt::BnBwdFuse bn{cbf(y), zp, stats.data_ptr<float>(), part.data_ptr<float>(), (int)mask};
  launch(s, bf(dx), ap, &bn, st, asub);
  float* dg = nullptr;
  float* db = nullptr;
  if (dgamma.has_value() && dgamma->defined()) {
    TORCH_CHECK(dbeta.has_value() && dbeta->defined(), "dgamma and dbeta go together");
    TORCH_CHECK(dgamma->is_contiguous() && dbeta->is_contiguous() && dgamma->numel() == s.C &&
                dbeta->numel() == s.C && dgamma->scalar_type() == at::kFloat, "dgamma/dbeta: fp32 [C]");
    dg = dgamma->data_ptr<float>();
    db = dbeta->data_ptr<float>();
  }
  pdt::launch_bn_bwd_part_reduce(part.data_ptr<float>(), G, s.C, ws.data_ptr<float>(),
                                 sums.data_ptr<float>(), stats.data_ptr<float>() + s.C, dg, db, st);
  return {dx, sums};
}

std::tuple<Tensor, Tensor> conv_dgrad_bn(const Tensor& dy, const Tensor& w, std::vector<int64_t> xs,
                                         int64_t stride, int64_t pad,
                                         const std::optional<Tensor>& addend, const Tensor& y,
                                         const std::optional<Tensor>& z, const Tensor& stats,
                                         int64_t mask, const std::optional<Tensor>& dgamma,
                                         const std::optional<Tensor>& dbeta,
                                         const std::optional<Tensor>& wt_in, const std::optional<Tensor>& acc,
                                         const std::optional<Tensor>& y2, const std::optional<Tensor>& stats2,
                                         const std::optional<Tensor>& acc2) {
  check_bf16_nhwc(dy, "dy");
  TORCH_CHECK(xs.size() == 4, "x shape must be NHWC");
  TORCH_CHECK(xs[3] == w.size(1), "dgrad: x channels must equal weight in-channels");
  c10::hip::HIPGuard g(dy.get_device());
  auto s = shape_of(xs[0], xs[1], xs[2], xs[3], w.size(0), w.size(2), w.size(3), stride, pad);
  TORCH_CHECK(s.Ho == dy.size(1) && s.Wo == dy.size(2) && s.K == dy.size(3), "dgrad: dy shape mismatch");
  Tensor wt = packed_t_or_pack(w, wt_in);
  return dgrad_bn_core(dy, s, addend, y, z, stats, mask, dgamma, dbeta, acc, SecondBn{y2, stats2, acc2},
                       [&](const pdt::ConvShape& sh, uint16_t* dx, const uint16_t* ap, const pdt::BnBwdFuse* bn,
                           hipStream_t st, int asub) {
                         pdt::launch_conv_dgrad(cbf(dy), cbf(wt), dx, ap, sh, st, bn, asub);
                       });
}

// Folded BN backward (kernels.h DgradFold): (wfold [C][K + C] bf16, bias [C] fp32) for the 1x1 conv
// whose transposed bf16 weights are wt [C][K] (or [C][1][1][K]), from its output BN's statistics,
// gamma and backward sums over `count` rows.
std::tuple<Tensor, Tensor> bn_fold_weights(const Tensor& wt, const Tensor& stats, const Tensor& gamma,
                                           const Tensor& sums, int64_t count) {
  check_cuda(wt, "wt");
  TORCH_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() && wt.numel() == wt.size(0) * wt.size(-1),
              "wt must be contiguous bf16 [C][K]");
  const int C = wt.size(0), K = wt.size(-1);
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.is_contiguous() && stats.numel() == 4 * K, "stats: fp32 [4, K]");
  TORCH_CHECK(gamma.scalar_type() == at::kFloat && gamma.numel() == K, "gamma: fp32 [K]");
  TORCH_CHECK(sums.scalar_type() == at::kFloat && sums.is_contiguous() && sums.numel() == 2 * K, "sums: fp32 [2, K]");
  c10::hip::HIPGuard g(wt.get_device());
  auto wfold = at::empty({C, K + C}, wt.options());
  auto bias_ws = at::empty({pdt::bn_fold_weights_ws_floats(C, K)}, stats.options());  // bias, then the kernel's scratch
  auto bias = bias_ws.narrow(0, 0, C);
  pdt::launch_bn_fold_weights(reinterpret_cast<const uint16_t*>(wt.data_ptr()), stats.data_ptr<float>(),
                              gamma.data_ptr<float>(), sums.data_ptr<float>(), (int)count, C, K,
                              reinterpret_cast<uint16_t*>(wfold.data_ptr()), bias.data_ptr<float>(), cur_stream(wt));
  return {wfold, bias};
}

static std::pair<float*, float*> bn_param_sinks(const std::optional<Tensor>& dgamma,
                                                const std::optional<Tensor>& dbeta, int64_t K);

// Weight gradient of a folded unit (kernels.h launch_bn_fold_wgrad): out [K,C,1,1] fp32 (a KRSC-dense
// view, e.g. the flat gradient buffer) += diag(k1) t1 + diag(a) W gram + b colsum^T with W the bf16
// mirror wt [C][K] (the operand bn_fold_weights read); dgamma/dbeta (optional) take the BN parameter
// gradients.  done (an int32 [1] counter, 0 between calls): consume mode -- t1 and gram are persistent
// workspaces the kernel clears after reading, and `sums` too when zero_sums.
void bn_fold_wgrad(Tensor t1, Tensor gram, const Tensor& colsum, const Tensor& wt,
                   const Tensor& stats, const Tensor& gamma, const Tensor& sums, int64_t count, Tensor out,
                   const std::optional<Tensor>& dgamma, const std::optional<Tensor>& dbeta,
                   const std::optional<Tensor>& done, bool zero_sums) {
  check_cuda(wt, "wt");
  check_cuda(colsum, "colsum");
  TORCH_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() && wt.numel() == wt.size(0) * wt.size(-1),
              "wt must be contiguous bf16 [C][K]");
  const int C = wt.size(0), K = wt.size(-1);
  TORCH_CHECK(t1.scalar_type() == at::kFloat && t1.numel() == (int64_t)K * C, "t1: fp32 [K, C]");
  TORCH_CHECK(gram.scalar_type() == at::kFloat && gram.numel() == (int64_t)C * C, "gram: fp32 [C, C]");
  // colsum: fp32 [C] (a reduction pass) or [S, C] (bn_act_fwd's S = bn_csum_slots() slots, consume
  // mode: re-zeroed)
  const int S = pdt::bn_csum_slots();
  TORCH_CHECK(colsum.scalar_type() == at::kFloat && colsum.is_contiguous() &&
              (colsum.numel() == C || (colsum.dim() == 2 && colsum.size(0) == S && colsum.size(1) == C)),
              "colsum: fp32 [C] or [bn_csum_slots(), C]");
  const int csum_slots = colsum.dim() == 2 ? S : 1;
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() == (int64_t)K * C, "out: fp32 [K, C, 1, 1]");
  for (const Tensor* x : {(const Tensor*)&t1, (const Tensor*)&gram, (const Tensor*)&out}) {
    // 1x1: [K,C,1,1] in either memory format is [K][C] memory when its two big strides are (C, 1)
    TORCH_CHECK(x->stride(0) == x->size(1) && x->stride(1) == 1, "fold wgrad: [K][C]-dense operands");
  }
  TORCH_CHECK(stats.numel() == 4 * K && gamma.numel() == K && sums.numel() == 2 * K && sums.is_contiguous(),
              "BN operands: [4,K], [K], [2,K]");
  int* dp = nullptr;
  if (done.has_value() && done->defined()) {
    TORCH_CHECK(done->is_cuda() && done->scalar_type() == at::kInt && done->numel() >= C / 64 + 1,
                "done: int32 device counters [C / 64 + 1]");
    dp = done->data_ptr<int>();
  }
  TORCH_CHECK(!zero_sums || dp != nullptr, "zero_sums needs the completion counter");
  c10::hip::HIPGuard g(wt.get_device());
  auto pg = bn_param_sinks(dgamma, dbeta, K);
  pdt::launch_bn_fold_wgrad(t1.data_ptr<float>(), gram.data_ptr<float>(), colsum.data_ptr<float>(),
                            reinterpret_cast<const uint16_t*>(wt.data_ptr()), stats.data_ptr<float>(),
                            gamma.data_ptr<float>(), sums.data_ptr<float>(), (int)count, C, K, out.data_ptr<float>(),
                            pg.first, pg.second, dp, zero_sums, cur_stream(wt), csum_slots);
}

// BN-fused dgrad of a 1x1 / stride-1 conv with the NEXT unit's BN backward folded in (kernels.h
// DgradFold): dx = [g | z] x wfold^T + bias, then the usual BN-fused epilogue (mask, sums into acc).
// g [N,H,W,K] is that BN's masked gradient, z [N,H,W,C] the conv's input; acc mode only.
std::tuple<Tensor, Tensor> conv_dgrad_bn_fold(const Tensor& g, const Tensor& z_in, const Tensor& wfold,
                                              const Tensor& bias, const Tensor& y, const std::optional<Tensor>& z,
                                              const Tensor& stats, int64_t mask, const std::optional<Tensor>& acc,
                                              const std::optional<Tensor>& dgamma,
                                              const std::optional<Tensor>& dbeta) {
  check_bf16_nhwc(g, "g");
  check_bf16_nhwc(z_in, "z_in");
  const int K = g.size(3), C = z_in.size(3);
  TORCH_CHECK(z_in.size(0) == g.size(0) && z_in.size(1) == g.size(1) && z_in.size(2) == g.size(2),
              "fold: g and z must share N, H, W");
  TORCH_CHECK(wfold.scalar_type() == at::kBFloat16 && wfold.is_contiguous() && wfold.size(0) == C &&
              wfold.size(1) == K + C, "wfold must be bf16 [C][K + C]");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() == C, "bias: fp32 [C]");
  c10::hip::HIPGuard gd(g.get_device());
  auto s = shape_of(g.size(0), g.size(1), g.size(2), C, K, 1, 1, 1, 0);
  pdt::DgradFold fold{cbf(z_in), C, bias.data_ptr<float>()};
  // acc: fp32-atomic BN sums of the unit before (default runs); without it (deterministic runs) the
  // fixed-order partials + reduce path, with that unit's dgamma / dbeta sinks
  return dgrad_bn_core(g, s, std::nullopt, y, z, stats, mask, dgamma, dbeta, acc, SecondBn{},
                       [&](const pdt::ConvShape& sh, uint16_t* dx, const uint16_t* ap, const pdt::BnBwdFuse* bn,
                           hipStream_t st, int asub) {
                         pdt::launch_conv_dgrad(cbf(g), reinterpret_cast<const uint16_t*>(wfold.data_ptr()), dx,
                                                ap, sh, st, bn, asub, &fold);
                       });
}

// fp8 dgrad operands: dy8 e5m2 NHWC [N,Ho,Wo,K], wt8 e4m3 [C,R,S,K] with per-C scale wscale,
// dy dequant factor ascale (device scalar)
pdt::ConvShape fp8_dgrad_shape(const Tensor& dy8, const Tensor& wt8, const Tensor& wscale, const Tensor& ascale,
                               const std::vector<int64_t>& xs, int64_t stride, int64_t pad) {
  check_u8_nhwc(dy8, "dy8");
  check_cuda(wt8, "wt8");
  TORCH_CHECK(wt8.scalar_type() == at::kByte && wt8.dim() == 4, "wt8 must be uint8 [C,R,S,K]");
  TORCH_CHECK(xs.size() == 4 && xs[3] == wt8.size(0), "dgrad: x channels must equal weight in-channels");
  TORCH_CHECK(wscale.is_cuda() && wscale.scalar_type() == at::kFloat && wscale.numel() == wt8.size(0),
              "wscale must be fp32 [C]");
  TORCH_CHECK(ascale.is_cuda() && ascale.scalar_type() == at::kFloat && ascale.numel() >= 1,
              "ascale must be a device fp32 scalar");
  auto s = shape_of(xs[0], xs[1], xs[2], xs[3], wt8.size(3), wt8.size(1), wt8.size(2), stride, pad);
  TORCH_CHECK(s.Ho == dy8.size(1) && s.Wo == dy8.size(2) && s.K == dy8.size(3), "dgrad: dy shape mismatch");
  TORCH_CHECK(s.K % 128 == 0 || (s.K % 16 == 0 && s.stride == 1),
              "fp8 dgrad: output channels must be a multiple of 128 (or of 16 at stride 1)");
  return s;
}

Tensor conv_dgrad_fp8(const Tensor& dy8, const Tensor& wt8, const Tensor& wscale, const Tensor& ascale,
                      std::vector<int64_t> xs, int64_t stride, int64_t pad,
                      const std::optional<Tensor>& addend) {
  c10::hip::HIPGuard g(dy8.get_device());
  auto s = fp8_dgrad_shape(dy8, wt8, wscale, ascale, xs, stride, pad);
  auto dx = at::empty({s.N, s.H, s.W, s.C}, dy8.options().dtype(at::kBFloat16));
  const uint16_t* ap = nullptr;
  int asub = 0;
  if (addend.has_value() && addend->defined()) {
    asub = addend_layout(*addend, dx);
    ap = cbf(*addend);
  }
  pdt::launch_conv_dgrad_fp8(dy8.data_ptr<uint8_t>(), wt8.data_ptr<uint8_t>(), wscale.data_ptr<float>(),
                             ascale.data_ptr<float>(), bf(dx), ap, s, cur_stream(dy8), nullptr, asub);
  return dx;
}

std::tuple<Tensor, Tensor> conv_dgrad_bn_fp8(const Tensor& dy8, const Tensor& wt8, const Tensor& wscale,
                                             const Tensor& ascale, std::vector<int64_t> xs, int64_t stride,
                                             int64_t pad, const std::optional<Tensor>& addend,
                                             const Tensor& y, const std::optional<Tensor>& z,
                                             const Tensor& stats, int64_t mask,
                                             const std::optional<Tensor>& dgamma,
                                             const std::optional<Tensor>& dbeta,
                                             const std::optional<Tensor>& acc) {
  c10::hip::HIPGuard g(dy8.get_device());
  auto s = fp8_dgrad_shape(dy8, wt8, wscale, ascale, xs, stride, pad);
  return dgrad_bn_core(dy8, s, addend, y, z, stats, mask, dgamma, dbeta, acc, SecondBn{},
                       [&](const pdt::ConvShape& sh, uint16_t* dx, const uint16_t* ap, const pdt::BnBwdFuse* bn,
                           hipStream_t st, int asub) {
                         pdt::launch_conv_dgrad_fp8(dy8.data_ptr<uint8_t>(), wt8.data_ptr<uint8_t>(),
                                                    wscale.data_ptr<float>(), ascale.data_ptr<float>(), dx,
                                                    ap, sh, st, bn, asub);
                       });
}

// dw as an fp32 channels_last tensor of logical shape [K, C, R, S]
static Tensor conv_wgrad_impl(const Tensor& dy, const Tensor& x, std::vector<int64_t> ws, int64_t stride,
                              int64_t pad, bool deterministic, const std::optional<Tensor>& out,
                              float* zero, int zero_n);

Tensor conv_wgrad(const Tensor& dy, const Tensor& x, std::vector<int64_t> ws, int64_t stride,
                  int64_t pad, bool deterministic, const std::optional<Tensor>& out) {
  return conv_wgrad_impl(dy, x, ws, stride, pad, deterministic, out, nullptr, 0);
}

// zero / zero_n: a buffer the weight-gradient kernel clears (see launch_conv_wgrad)
static Tensor conv_wgrad_impl(const Tensor& dy, const Tensor& x, std::vector<int64_t> ws, int64_t stride,
                              int64_t pad, bool deterministic, const std::optional<Tensor>& out,
                              float* zero, int zero_n) {
  check_bf16_nhwc(dy, "dy");
  check_bf16_nhwc(x, "x");
  TORCH_CHECK(ws.size() == 4, "weight shape must be [K,C,R,S]");
  c10::hip::HIPGuard g(x.get_device());
  int K = ws[0], C = ws[1], R = ws[2], S = ws[3];
  int Cx = x.size(3);
  auto s = shape_of(x.size(0), x.size(1), x.size(2), Cx, K, R, S, stride, pad);
  TORCH_CHECK(s.Ho == dy.size(1) && s.Wo == dy.size(2) && K == dy.size(3), "wgrad: dy shape mismatch");
  auto fopt = x.options().dtype(at::kFloat);
  size_t wsn = pdt::conv_wgrad_ws_floats(s, deterministic);
  Tensor wsb = wsn ? at::empty({(int64_t)wsn}, fopt) : Tensor();
  if (out.has_value() && out->defined()) {
    // accumulate into a caller-owned [K,C,R,S] fp32 tensor whose memory is KRSC-contiguous
    // (a channels_last view of the flat gradient buffer)
    const Tensor& o = *out;
    TORCH_CHECK(Cx == C, "in-place wgrad needs unpadded input channels");
    TORCH_CHECK(o.scalar_type() == at::kFloat && o.dim() == 4 && o.size(0) == K && o.size(1) == C &&
                o.size(2) == R && o.size(3) == S, "wgrad out: bad shape/dtype");
    // KRSC-dense: strides (RSC, 1, SC, C); a size-1 dim may carry any stride
    const int64_t want[4] = {(int64_t)R * S * C, 1, (int64_t)S * C, (int64_t)C};
    for (int d = 0; d < 4; ++d)
      TORCH_CHECK(o.size(d) == 1 || o.stride(d) == want[d], "wgrad out must be channels_last (KRSC) dense");
    pdt::launch_conv_wgrad(cbf(dy), cbf(x), o.data_ptr<float>(), wsn ? wsb.data_ptr<float>() : nullptr,
                           s, deterministic, true, cur_stream(x), zero, zero_n);
    return o;
  }
  auto dwp = at::empty({K, R, S, Cx}, fopt);
  pdt::launch_conv_wgrad(cbf(dy), cbf(x), dwp.data_ptr<float>(), wsn ? wsb.data_ptr<float>() : nullptr,
                         s, deterministic, false, cur_stream(x), zero, zero_n);
  Tensor krsc = Cx == C ? dwp : dwp.narrow(3, 0, C).contiguous();
  return krsc.permute({0, 3, 1, 2});  // [K,C,R,S] view with channels_last strides
}

// conv_wgrad issued on the weight-gradient side stream (ops/fused.py, ops/streams.py) in one call:
// the side stream waits for the work queued so far on the current stream (one reusable event per
// device: a wait binds to the record made just before it), the wgrad runs with the side stream as
// the current stream (its workspace is allocated for that stream), and dy / x are recorded for the
// side stream so the caching allocator keeps their memory until it is done.  Replaces torch's
// wait_stream + stream context + two record_stream calls: ~25 us of host issue per weight
// gradient (scripts/host_profile.py), 20-53 of them per step.
Tensor conv_wgrad_side(int64_t side, const Tensor& dy, const Tensor& x, std::vector<int64_t> ws,
                       int64_t stride, int64_t pad, bool deterministic, const std::optional<Tensor>& out,
                       const std::optional<Tensor>& zero) {
  TORCH_CHECK(side != 0, "conv_wgrad_side: null side stream");
  c10::hip::HIPGuard g(x.get_device());
  const auto dev = (c10::DeviceIndex)x.get_device();
  // per calling thread (autograd runs a device's backward on one long-lived engine thread) and
  // device; kept for the process lifetime like torch's own stream pool
  static thread_local std::unordered_map<int, hipEvent_t> evs;
  hipEvent_t& ev = evs[(int)dev];
  if (ev == nullptr)
    TORCH_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
  auto sst = c10::hip::getStreamFromExternal(reinterpret_cast<hipStream_t>(side), dev);
  TORCH_CHECK(hipEventRecord(ev, c10::hip::getCurrentHIPStream(dev).stream()) == hipSuccess, "hipEventRecord failed");
  TORCH_CHECK(hipStreamWaitEvent(sst.stream(), ev, 0) == hipSuccess, "hipStreamWaitEvent failed");
  Tensor r;
  {
    c10::hip::HIPStreamGuard sg(sst);
    // `zero`: a BN-sum accumulator whose consumer (the apply just queued on the current stream) is
    // done at this point of the side stream: the weight-gradient kernel itself re-zeroes it for its
    // next use (workgroup 0), off the critical path and without a memset launch
    float* zp = nullptr;
    int zn = 0;
    if (zero.has_value() && zero->defined()) {
      TORCH_CHECK(zero->scalar_type() == at::kFloat && zero->is_contiguous(), "zero: contiguous fp32");
      zp = zero->data_ptr<float>();
      zn = (int)zero->numel();
    }
    r = conv_wgrad_impl(dy, x, ws, stride, pad, deterministic, out, zp, zn);
  }
  c10::hip::HIPCachingAllocator::recordStream(dy.storage().data_ptr(), sst);
  c10::hip::HIPCachingAllocator::recordStream(x.storage().data_ptr(), sst);
  return r;
}

// fp8 weight gradient (conv_igemm.hip igemm_tn_f8_kernel): dy8 e5m2 [N,Ho,Wo,K] and x8 e4m3 [N,H,W,C]
// with their dequantization factors (device fp32 scalars).  Accumulates into `out` (a KRSC-dense fp32
// view, e.g. the flat gradient buffer) or returns a fresh [K,C,R,S] channels_last tensor.  side != 0:
// issued on that stream after the current stream's queued work, like conv_wgrad_side.
Tensor conv_wgrad_fp8(int64_t side, const Tensor& dy8, const Tensor& x8, const Tensor& dy_deq, const Tensor& x_deq,
                      std::vector<int64_t> ws, int64_t stride, int64_t pad, const std::optional<Tensor>& out,
                      const std::optional<Tensor>& zero) {
  TORCH_CHECK(dy8.is_cuda() && x8.is_cuda() && dy8.scalar_type() == at::kByte && x8.scalar_type() == at::kByte &&
              dy8.dim() == 4 && x8.dim() == 4 && dy8.is_contiguous() && x8.is_contiguous(),
              "conv_wgrad_fp8: dy8 / x8 must be contiguous uint8 NHWC device tensors");
  TORCH_CHECK(dy_deq.is_cuda() && x_deq.is_cuda() && dy_deq.scalar_type() == at::kFloat &&
              x_deq.scalar_type() == at::kFloat && dy_deq.numel() >= 1 && x_deq.numel() >= 1,
              "conv_wgrad_fp8: dequantization factors must be device fp32 scalars");
  TORCH_CHECK(ws.size() == 4, "weight shape must be [K,C,R,S]");
  c10::hip::HIPGuard g(x8.get_device());
  const int K = ws[0], C = ws[1], R = ws[2], S = ws[3];
  TORCH_CHECK(x8.size(3) == C && C % 16 == 0 && K % 64 == 0, "conv_wgrad_fp8: needs C % 16 == 0, K % 64 == 0");
  auto s = shape_of(x8.size(0), x8.size(1), x8.size(2), C, K, R, S, stride, pad);
  TORCH_CHECK(s.Ho == dy8.size(1) && s.Wo == dy8.size(2) && K == dy8.size(3) && s.N == dy8.size(0),
              "conv_wgrad_fp8: dy shape mismatch");
  const auto dev = (c10::DeviceIndex)x8.get_device();
  hipStream_t st = cur_stream(x8);
  std::optional<c10::hip::HIPStreamGuard> sg;
  if (side != 0) {
    static thread_local std::unordered_map<int, hipEvent_t> evs;
    hipEvent_t& ev = evs[(int)dev];
    if (ev == nullptr)
      TORCH_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
    auto sst = c10::hip::getStreamFromExternal(reinterpret_cast<hipStream_t>(side), dev);
    TORCH_CHECK(hipEventRecord(ev, st) == hipSuccess, "hipEventRecord failed");
    TORCH_CHECK(hipStreamWaitEvent(sst.stream(), ev, 0) == hipSuccess, "hipStreamWaitEvent failed");
    sg.emplace(sst);
    st = sst.stream();
  }
  Tensor r;
  if (out.has_value() && out->defined()) {
    const Tensor& o = *out;
    TORCH_CHECK(o.scalar_type() == at::kFloat && o.dim() == 4 && o.size(0) == K && o.size(1) == C &&
                o.size(2) == R && o.size(3) == S, "wgrad out: bad shape/dtype");
    const int64_t want[4] = {(int64_t)R * S * C, 1, (int64_t)S * C, (int64_t)C};
    for (int d = 0; d < 4; ++d)
      TORCH_CHECK(o.size(d) == 1 || o.stride(d) == want[d], "wgrad out must be channels_last (KRSC) dense");
    pdt::launch_conv_wgrad_fp8(dy8.data_ptr<uint8_t>(), x8.data_ptr<uint8_t>(), dy_deq.data_ptr<float>(),
                               x_deq.data_ptr<float>(), o.data_ptr<float>(), s, true, st);
    r = o;
  } else {
    auto dwp = at::empty({K, R, S, C}, x8.options().dtype(at::kFloat));
    pdt::launch_conv_wgrad_fp8(dy8.data_ptr<uint8_t>(), x8.data_ptr<uint8_t>(), dy_deq.data_ptr<float>(),
                               x_deq.data_ptr<float>(), dwp.data_ptr<float>(), s, false, st);
    r = dwp.permute({0, 3, 1, 2});
  }
  // a consumed BN-sum accumulator: cleared by a memset AFTER the kernel (the bf16 weight gradient
  // clears it in its workgroup 0 instead; done that way here, the fp8 ResNet-50 parity runs fell
  // behind in 4 of 7 runs against 0 of 7 with the memset -- profiles/r6_fp8_parity.txt)
  if (zero.has_value() && zero->defined())
    TORCH_CHECK(hipMemsetAsync(zero->data_ptr(), 0, zero->nbytes(), st) == hipSuccess, "memset");
  if (side != 0) {
    auto sst = c10::hip::getStreamFromExternal(reinterpret_cast<hipStream_t>(side), dev);
    for (const Tensor* t : {&dy8, &x8, &dy_deq, &x_deq})
      c10::hip::HIPCachingAllocator::recordStream(t->storage().data_ptr(), sst);
  }
  return r;
}

// -------------------------------------------------------------------- stem
// 7x7/s2 stem with C <= 4 input channels as a super-pixel conv (kernels.h): returns
// (xsp, y, part) -- xsp is the bf16 super-pixel image (kept for the weight gradient)
std::tuple<Tensor, Tensor, Tensor, int64_t> stem_conv_fwd(const Tensor& x, const Tensor& w, int64_t stride,
                                                          int64_t pad, bool stats) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 4, "stem: image must be fp32 NCHW");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4, "stem: weight must be fp32 4-D");
  TORCH_CHECK(stride == 2 && x.size(1) <= 4 && w.size(1) == x.size(1), "stem: stride 2, <= 4 channels");
  c10::hip::HIPGuard g(x.get_device());
  Tensor xc = x.contiguous();
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int K = w.size(0), R = w.size(2), S = w.size(3);
  const int Ho = (H + 2 * pad - R) / 2 + 1, Wo = (W + 2 * pad - S) / 2 + 1;
  const int Sp = (S + 2) / 2, Hp = H + 2 * pad, Wsp = Wo + Sp - 1;
  TORCH_CHECK(2 * (Ho - 1) + R <= Hp, "stem: padded height too small");
  auto xsp = at::empty({N, Hp, Wsp, 8}, x.options().dtype(at::kBFloat16));
  hipStream_t st = cur_stream(x);
  pdt::launch_stem_image(xc.data_ptr<float>(), bf(xsp), N, C, H, W, (int)pad, Hp, Wsp, st);
  auto wsp = at::empty({K, R, Sp, 8}, w.options().dtype(at::kBFloat16));
  int64_t ws[4] = {w.stride(0), w.stride(1), w.stride(2), w.stride(3)};
  pdt::launch_stem_pack_weight(w.data_ptr<float>(), ws, bf(wsp), K, C, R, S, Sp, st);
  pdt::ConvShape s;
  s.N = N; s.H = Hp; s.W = Wsp; s.C = 8; s.K = K; s.R = R; s.S = Sp;
  s.Ho = Ho; s.Wo = Wo; s.stride = 2; s.stride_w = 1; s.pad = 0;
  TORCH_CHECK(xsp.numel() < (int64_t(1) << 30), "stem: image too large for 32-bit addressing");
  auto y = at::empty({N, Ho, Wo, K}, xsp.options());
  Tensor part;
  float* pp = nullptr;
  const int M = N * Ho * Wo;
  const bool halo = pdt::stem_halo_supported(K, R, Sp, Wo);
  // BN partial groups: one per output row on the halo kernel, one per NT row tile otherwise
  const int grows = halo ? Wo : pdt::conv_nt_group_rows(M, K, R * Sp * 8 * 2);
  if (stats) {
    part = at::empty({(M + grows - 1) / grows, 2, K}, x.options());
    pp = part.data_ptr<float>();
  }
  if (halo) pdt::launch_stem_conv_fwd(cbf(xsp), cbf(wsp), bf(y), pp, N, Hp, Wsp, Ho, Wo, st);
  else pdt::launch_conv_fwd(cbf(xsp), cbf(wsp), bf(y), pp, s, st);
  return {xsp, y, part, (int64_t)grows};
}

// weight gradient of the stem from the super-pixel image; accumulates into `out` (fp32 [K,C,R,S],
// any strides) when given, else returns a fresh channels_last tensor
Tensor stem_wgrad(const Tensor& dy, const Tensor& xsp, std::vector<int64_t> wsz, bool deterministic,
                  const std::optional<Tensor>& out) {
  check_bf16_nhwc(dy, "dy");
  check_bf16_nhwc(xsp, "xsp");
  TORCH_CHECK(wsz.size() == 4, "weight shape must be [K,C,R,S]");
  c10::hip::HIPGuard g(dy.get_device());
  const int K = wsz[0], C = wsz[1], R = wsz[2], S = wsz[3];
  const int Sp = (S + 2) / 2;
  pdt::ConvShape s;
  s.N = xsp.size(0); s.H = xsp.size(1); s.W = xsp.size(2); s.C = 8; s.K = K; s.R = R; s.S = Sp;
  s.Ho = dy.size(1); s.Wo = dy.size(2); s.stride = 2; s.stride_w = 1; s.pad = 0;
  TORCH_CHECK(dy.size(3) == K && s.Wo + Sp - 1 == s.W, "stem_wgrad: shape mismatch");
  auto fopt = dy.options().dtype(at::kFloat);
  size_t wsn = pdt::conv_wgrad_ws_floats(s, deterministic);
  Tensor wsb = wsn ? at::empty({(int64_t)wsn}, fopt) : Tensor();
  auto dwsp = at::empty({K, R, Sp, 8}, fopt);
  hipStream_t st = cur_stream(dy);
  pdt::launch_conv_wgrad(cbf(dy), cbf(xsp), dwsp.data_ptr<float>(), wsn ? wsb.data_ptr<float>() : nullptr,
                         s, deterministic, false, st);
  Tensor o;
  bool acc = false;
  if (out.has_value() && out->defined()) {
    o = *out;
    TORCH_CHECK(o.scalar_type() == at::kFloat && o.dim() == 4 && o.size(0) == K && o.size(1) == C &&
                o.size(2) == R && o.size(3) == S, "stem_wgrad out: bad shape/dtype");
    acc = true;
  } else {
    o = at::empty({K, C, R, S}, fopt.memory_format(at::MemoryFormat::ChannelsLast));
  }
  int64_t os[4] = {o.stride(0), o.stride(1), o.stride(2), o.stride(3)};
  pdt::launch_stem_wgrad_unpack(dwsp.data_ptr<float>(), o.data_ptr<float>(), os, K, C, R, S, Sp, acc, st);
  return o;
}

// stem backward with the BN/pool apply fused into the weight gradient: accumulates dW into `out`
// (fp32 [K,C,R,S], any strides) when given, else returns a fresh channels_last tensor
Tensor stem_bwd_fused(const Tensor& dpool, const Tensor& idx, const Tensor& y, const Tensor& stats,
                      const Tensor& gamma, const Tensor& sums, bool training, const Tensor& xsp,
                      std::vector<int64_t> wsz, bool deterministic, const std::optional<Tensor>& out) {
  check_bf16_nhwc(dpool, "dpool");
  check_bf16_nhwc(y, "y");
  check_bf16_nhwc(xsp, "xsp");
  TORCH_CHECK(wsz.size() == 4, "weight shape must be [K,C,R,S]");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.is_contiguous() &&
              idx.numel() == dpool.numel(), "idx: uint8 argmax map like dpool");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.numel() == 4 * y.size(3) &&
              sums.scalar_type() == at::kFloat && sums.numel() == 2 * y.size(3), "stats [4][K], sums [2][K]");
  c10::hip::HIPGuard g(y.get_device());
  const int K = wsz[0], C = wsz[1], R = wsz[2], S = wsz[3];
  const int Sp = (S + 2) / 2;
  const int N = y.size(0), Ho = y.size(1), Wo = y.size(2);
  TORCH_CHECK(y.size(3) == K && pdt::stem_bwd_fused_supported(K, R, Sp, Ho, Wo), "stem_bwd_fused: unsupported shape");
  TORCH_CHECK(dpool.size(0) == N && dpool.size(1) == Ho / 2 && dpool.size(2) == Wo / 2 && dpool.size(3) == K,
              "stem_bwd_fused: dpool must be the 3x3/s2/p1 max pool of y");
  TORCH_CHECK(xsp.size(0) == N && xsp.size(2) == Wo + Sp - 1 && xsp.size(3) == 8, "stem_bwd_fused: xsp shape");
  auto fopt = y.options().dtype(at::kFloat);
  auto dwsp = at::empty({K, R, Sp, 8}, fopt);
  Tensor wsb;
  if (deterministic) wsb = at::empty({(int64_t)pdt::stem_bwd_fused_blocks(N, Ho) * K * R * Sp * 8}, fopt);
  hipStream_t st = cur_stream(y);
  pdt::launch_stem_bwd_fused(cbf(dpool), idx.data_ptr<uint8_t>(), cbf(y), stats.data_ptr<float>(),
                             gamma.data_ptr<float>(), sums.data_ptr<float>(), training, cbf(xsp), N, Ho, Wo,
                             xsp.size(1), xsp.size(2), dwsp.data_ptr<float>(),
                             deterministic ? wsb.data_ptr<float>() : nullptr, st);
  Tensor o;
  bool acc = false;
  if (out.has_value() && out->defined()) {
    o = *out;
    TORCH_CHECK(o.scalar_type() == at::kFloat && o.dim() == 4 && o.size(0) == K && o.size(1) == C &&
                o.size(2) == R && o.size(3) == S, "stem_bwd_fused out: bad shape/dtype");
    acc = true;
  } else {
    o = at::empty({K, C, R, S}, fopt.memory_format(at::MemoryFormat::ChannelsLast));
  }
  int64_t os[4] = {o.stride(0), o.stride(1), o.stride(2), o.stride(3)};
  pdt::launch_stem_wgrad_unpack(dwsp.data_ptr<float>(), o.data_ptr<float>(), os, K, C, R, S, Sp, acc, st);
  return o;
}

// ---------------------------------------------------------------------- BN
Tensor bn_finalize(const Tensor& part, int64_t count, const Tensor& rm, const Tensor& rv,
                   const Tensor& gamma, const Tensor& beta, double momentum, double eps, int64_t grows_in) {
  check_cuda(part, "part");
  c10::hip::HIPGuard g(part.get_device());
  int ng = part.size(0), K = part.size(2);
  // the producing conv's row group is its NT tile's BM (64, 128 or 256; conv_nt_group_rows): the
  // only one of those giving ng groups over `count` rows; a single group covers every row.  A
  // producer with another grouping (the halo stem: one group per output row) passes grows_in.
  int grows = 0;
  if (grows_in > 0) {
    TORCH_CHECK((count + grows_in - 1) / grows_in == ng, "bn_finalize: grows does not match the partials");
    grows = (int)grows_in;
  } else if (ng == 1) {
    grows = (int)count;
  } else {
    for (int g : {64, 128, 256})
      if ((count + g - 1) / g == ng) { grows = g; break; }
  }
  TORCH_CHECK(grows > 0, "bn_finalize: partial layout mismatch");
  int P = pdt::bn_finalize_partitions(ng);
  auto out = at::empty({4 * K + 3 * K * P}, part.options());
  TORCH_CHECK(gamma.scalar_type() == at::kFloat && rm.scalar_type() == at::kFloat, "BN params must be fp32");
  pdt::launch_bn_finalize(part.data_ptr<float>(), ng, grows, (int)count, K,
                          rm.defined() ? rm.data_ptr<float>() : nullptr,
                          rv.defined() ? rv.data_ptr<float>() : nullptr, gamma.data_ptr<float>(),
                          beta.data_ptr<float>(), (float)momentum, (float)eps,
                          out.data_ptr<float>(), cur_stream(part));
  return out.narrow(0, 0, 4 * K).view({4, K});
}

// Training-mode conv unit forward in ONE host call: conv with BN partial statistics, then the BN
// finalize (batch mean / invstd / scale / shift, running-stat update).  Saves a Python -> C++
// round trip per conv unit (155 per ResNet-152 step) over conv_fwd + bn_finalize.
static pdt::BnFwdFuse bn_fwd_fuse(const Tensor& x, int K, int64_t count, int64_t M, const Tensor& acc,
                                   const Tensor& rm, const Tensor& rv, const Tensor& gamma,
                                   const Tensor& beta, double momentum, double eps, Tensor& stats) {
  TORCH_CHECK(M == count, "conv_fwd_bn: count mismatch");
  TORCH_CHECK(acc.scalar_type() == at::kDouble && acc.is_contiguous() && acc.numel() >= pdt::kStatSlots * 2 * K &&
              acc.device() == x.device(), "conv_fwd_bn: acc must be a contiguous fp64 [8][2][K] device tensor");
  TORCH_CHECK(gamma.scalar_type() == at::kFloat && beta.scalar_type() == at::kFloat && gamma.numel() == K,
              "BN params must be fp32 [K]");
  TORCH_CHECK(!rm.defined() || (rm.scalar_type() == at::kFloat && rv.defined() && rm.numel() == K),
              "running stats must be fp32 [K]");
  stats = at::empty({4, K}, x.options().dtype(at::kFloat));
  return pdt::BnFwdFuse{acc.data_ptr<double>(), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                        rm.defined() ? rm.data_ptr<float>() : nullptr, rv.defined() ? rv.data_ptr<float>() : nullptr,
                        stats.data_ptr<float>(), (float)momentum, (float)eps};
}

// acc (fp64 [>= 2K], zero, re-zeroed by the finalize): the conv sums the statistics into it and a
// one-thread-per-channel finalize reads them (kernels.h BnFwdFuse; fp64 atomics, so not bitwise
// run-to-run: callers pass it only outside deterministic mode), else the partials + bn_finalize.
std::tuple<Tensor, Tensor> conv_fwd_bn(const Tensor& x, const Tensor& wk, int64_t stride, int64_t pad,
                                       int64_t count, const Tensor& rm, const Tensor& rv, const Tensor& gamma,
                                       const Tensor& beta, double momentum, double eps,
                                       const std::optional<Tensor>& acc) {
  if (acc.has_value() && acc->defined()) {
    check_bf16_nhwc(x, "x");
    check_cuda(wk, "wk");
    TORCH_CHECK(wk.dim() == 4 && wk.size(3) == x.size(3), "packed weight must be [K,R,S,Cx]");
    c10::hip::HIPGuard g(x.get_device());
    auto s = shape_of(x.size(0), x.size(1), x.size(2), x.size(3), wk.size(0), wk.size(1), wk.size(2),
                      stride, pad);
    TORCH_CHECK(s.K % 8 == 0, "output channels must be a multiple of 8");
    auto y = at::empty({s.N, s.Ho, s.Wo, s.K}, x.options());
    Tensor stats;
    auto f = bn_fwd_fuse(x, s.K, count, (int64_t)s.N * s.Ho * s.Wo, *acc, rm, rv, gamma, beta, momentum, eps,
                         stats);
    pdt::launch_conv_fwd(cbf(x), cbf(wk), bf(y), nullptr, s, cur_stream(x), &f);
    return {y, stats};
  }
  auto yp = conv_fwd(x, wk, stride, pad, true);
  Tensor stats = bn_finalize(std::get<1>(yp), count, rm, rv, gamma, beta, momentum, eps, 0);
  return {std::get<0>(yp), stats};
}

Tensor bn_eval_params(const Tensor& rm, const Tensor& rv, const Tensor& gamma, const Tensor& beta,
                      double eps) {
  check_cuda(rm, "running_mean");
  c10::hip::HIPGuard g(rm.get_device());
  int K = rm.numel();
  auto out = at::empty({4, K}, rm.options().dtype(at::kFloat));
  pdt::launch_bn_eval_params(rm.data_ptr<float>(), rv.data_ptr<float>(), gamma.data_ptr<float>(),
                             beta.data_ptr<float>(), (float)eps, K, out.data_ptr<float>(),
                             cur_stream(rm));
  return out;
}

// optional BatchNorm of the residual (res_scale / res_shift: fp32 [K]); returns their pointers
static std::pair<const float*, const float*> res_bn_args(const std::optional<Tensor>& res,
                                                         const std::optional<Tensor>& rsc,
                                                         const std::optional<Tensor>& rsh, int64_t K) {
  const bool has = rsc.has_value() && rsc->defined();
  TORCH_CHECK(has == (rsh.has_value() && rsh->defined()), "res_scale and res_shift go together");
  if (!has) return {nullptr, nullptr};
  TORCH_CHECK(res.has_value() && res->defined(), "a residual BatchNorm needs the residual");
  for (const Tensor* t : {&*rsc, &*rsh})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == K,
                "res_scale / res_shift must be contiguous fp32 [K] device tensors");
  return {rsc->data_ptr<float>(), rsh->data_ptr<float>()};
}

Tensor bn_act_fwd(const Tensor& y, const Tensor& scale, const Tensor& shift,
                  const std::optional<Tensor>& res, bool relu, const std::optional<Tensor>& rsc,
                  const std::optional<Tensor>& rsh, const std::optional<Tensor>& csum) {
  check_bf16_nhwc(y, "y");
  c10::hip::HIPGuard g(y.get_device());
  int K = y.size(3);
  int64_t M = y.numel() / K;
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_bf16_nhwc(*res, "residual");
    TORCH_CHECK(res->sizes() == y.sizes(), "residual shape mismatch");
    rp = cbf(*res);
  }
  auto rbn = res_bn_args(res, rsc, rsh, K);
  float* cs = nullptr;
  if (csum.has_value() && csum->defined()) {  // per-channel sums of z into fp32 [S, K] slots (atomic)
    check_cuda(*csum, "csum");
    TORCH_CHECK(csum->scalar_type() == at::kFloat && csum->is_contiguous() &&
                csum->numel() == (int64_t)pdt::bn_csum_slots() * K,
                "csum must be a contiguous fp32 [bn_csum_slots(), K] device tensor");
    cs = csum->data_ptr<float>();
  }
  auto z = at::empty_like(y);
  pdt::launch_bn_act_fwd(cbf(y), scale.data_ptr<float>(), shift.data_ptr<float>(), rp, relu, bf(z), M,
                         K, cur_stream(y), nullptr, rbn.first, rbn.second, cs);
  return z;
}

// (z, zmask): bn_act_fwd with ReLU that also writes the 1-bit-per-element ReLU mask (uint8, one
// byte per 8 channels) for a later BN-fused dgrad (mask mode 3)
std::tuple<Tensor, Tensor> bn_act_fwd_mask(const Tensor& y, const Tensor& scale, const Tensor& shift,
                                           const std::optional<Tensor>& res,
                                           const std::optional<Tensor>& rsc,
                                           const std::optional<Tensor>& rsh) {
  check_bf16_nhwc(y, "y");
  c10::hip::HIPGuard g(y.get_device());
  int K = y.size(3);
  int64_t M = y.numel() / K;
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_bf16_nhwc(*res, "residual");
    TORCH_CHECK(res->sizes() == y.sizes(), "residual shape mismatch");
    rp = cbf(*res);
  }
  auto rbn = res_bn_args(res, rsc, rsh, K);
  auto z = at::empty_like(y);
  auto zm = at::empty({y.numel() / 8}, y.options().dtype(at::kByte));
  pdt::launch_bn_act_fwd(cbf(y), scale.data_ptr<float>(), shift.data_ptr<float>(), rp, true, bf(z), M, K,
                         cur_stream(y), zm.data_ptr<uint8_t>(), rbn.first, rbn.second);
  return {z, zm};
}

Tensor bn_act_bwd_reduce(const Tensor& dz, const Tensor& z, const Tensor& y, const Tensor& stats,
                         int64_t mask, const std::optional<Tensor>& dgamma,
                         const std::optional<Tensor>& dbeta) {
  check_bf16_nhwc(dz, "dz");
  check_bf16_nhwc(y, "y");
  c10::hip::HIPGuard g(dz.get_device());
  int K = y.size(3);
  TORCH_CHECK(256 % (K / 8) == 0, "bn backward: channels must divide 2048 and be a power of two");
  TORCH_CHECK(stats.numel() == 4 * K && stats.is_contiguous(), "stats must be [4, K]");
  if (mask == 1) check_bf16_nhwc(z, "z");
  int64_t M = y.numel() / K;
  auto fopt = y.options().dtype(at::kFloat);
  auto ws = at::empty({(int64_t)pdt::bn_bwd_ws_floats(M, K)}, fopt);
  auto sums = at::empty({2, K}, fopt);
  float* dg = nullptr;
  float* db = nullptr;
  if (dgamma.has_value() && dgamma->defined()) {
    TORCH_CHECK(dbeta.has_value() && dbeta->defined(), "dgamma and dbeta go together");
    TORCH_CHECK(dgamma->numel() == K && dbeta->numel() == K && dgamma->is_contiguous() &&
                dbeta->is_contiguous() && dgamma->scalar_type() == at::kFloat, "bad dgamma/dbeta");
    dg = dgamma->data_ptr<float>();
    db = dbeta->data_ptr<float>();
  }
  pdt::launch_bn_act_bwd_reduce(cbf(dz), mask == 1 ? cbf(z) : nullptr, cbf(y), stats.data_ptr<float>(),
                                (int)mask, M, K, ws.data_ptr<float>(), sums.data_ptr<float>(), dg, db,
                                cur_stream(y));
  return sums;
}

// optional BN parameter-gradient sinks (fp32 [K], both or neither)
static std::pair<float*, float*> bn_param_sinks(const std::optional<Tensor>& dgamma,
                                                const std::optional<Tensor>& dbeta, int64_t K) {
  if (!(dgamma.has_value() && dgamma->defined())) {
    TORCH_CHECK(!(dbeta.has_value() && dbeta->defined()), "dgamma and dbeta go together");
    return {nullptr, nullptr};
  }
  TORCH_CHECK(dbeta.has_value() && dbeta->defined(), "dgamma and dbeta go together");
  TORCH_CHECK(dgamma->is_contiguous() && dbeta->is_contiguous() && dgamma->numel() == K &&
              dbeta->numel() == K && dgamma->scalar_type() == at::kFloat && dbeta->scalar_type() == at::kFloat,
              "dgamma/dbeta: fp32 [C]");
  return {dgamma->data_ptr<float>(), dbeta->data_ptr<float>()};
}

std::tuple<Tensor, Tensor> bn_act_bwd_apply(const Tensor& dz, const Tensor& z, const Tensor& y,
                                            const Tensor& stats, const Tensor& gamma,
                                            const Tensor& sums, int64_t mask, bool training,
                                            bool want_dres, const std::optional<Tensor>& dgamma,
                                            const std::optional<Tensor>& dbeta) {
  check_bf16_nhwc(dz, "dz");
  check_bf16_nhwc(y, "y");
  c10::hip::HIPGuard g(dz.get_device());
  int K = y.size(3);
  TORCH_CHECK(256 % (K / 8) == 0, "bn backward: channels must divide 2048 and be a power of two");
  TORCH_CHECK(stats.numel() == 4 * K && stats.is_contiguous(), "stats must be [4, K]");
  if (mask == 1) check_bf16_nhwc(z, "z");
  int64_t M = y.numel() / K;
  auto dy = at::empty_like(dz);
  Tensor dres;
  if (want_dres) dres = at::empty_like(dz);
  auto pg = bn_param_sinks(dgamma, dbeta, K);
  pdt::launch_bn_act_bwd_apply(cbf(dz), mask == 1 ? cbf(z) : nullptr, cbf(y), stats.data_ptr<float>(),
                               gamma.data_ptr<float>(), sums.data_ptr<float>(), (int)mask, training,
                               M, K, bf(dy), want_dres ? bf(dres) : nullptr, cur_stream(dz), pg.first,
                               pg.second);
  return {dy, dres};
}

// (dy, dres, dy8): bn_act_bwd_apply (training) that also emits dy8 = e5m2(dy * s_t)
std::tuple<Tensor, Tensor, Tensor> bn_act_bwd_apply_q8(const Tensor& dz, const Tensor& z, const Tensor& y,
                                                       const Tensor& stats, const Tensor& gamma,
                                                       const Tensor& sums, int64_t mask, bool want_dres,
                                                       Tensor state, int64_t slot, bool want_dy,
                                                       const std::optional<Tensor>& dgamma,
                                                       const std::optional<Tensor>& dbeta) {
  check_bf16_nhwc(dz, "dz");
  check_bf16_nhwc(y, "y");
  check_state(state, slot);
  c10::hip::HIPGuard g(dz.get_device());
  int K = y.size(3);
  TORCH_CHECK(256 % (K / 8) == 0, "bn backward: channels must divide 2048 and be a power of two");
  TORCH_CHECK(stats.numel() == 4 * K && stats.is_contiguous(), "stats must be [4, K]");
  if (mask == 1) check_bf16_nhwc(z, "z");
  int64_t M = y.numel() / K;
  auto pg = bn_param_sinks(dgamma, dbeta, K);
  Tensor dy, dres;
  if (want_dy) dy = at::empty_like(dz);  // else: fp8-only dy, every consumer reads dy8
  if (want_dres) dres = at::empty_like(dz);
  auto dy8 = at::empty(dz.sizes(), dz.options().dtype(at::kByte));
  pdt::launch_bn_act_bwd_apply_q8(cbf(dz), mask == 1 ? cbf(z) : nullptr, cbf(y), stats.data_ptr<float>(),
                                  gamma.data_ptr<float>(), sums.data_ptr<float>(), (int)mask, true, M, K,
                                  want_dy ? bf(dy) : nullptr, want_dres ? bf(dres) : nullptr, dy8.data_ptr<uint8_t>(),
                                  state.data_ptr<float>(), (int)slot, cur_stream(dz), pg.first, pg.second);
  return {dy, dres, dy8};
}

// batched row-wise e4m3 quantization of a flat bf16 weight mirror (table: QRowEntry bytes)
void quant_rows_e4m3(const Tensor& src, Tensor dst, Tensor scale, const Tensor& table, int64_t max_rows) {
  check_cuda(src, "src");
  check_cuda(dst, "dst");
  check_cuda(scale, "scale");
  TORCH_CHECK(src.scalar_type() == at::kBFloat16 && dst.scalar_type() == at::kByte &&
              scale.scalar_type() == at::kFloat && src.numel() == dst.numel(), "quant_rows: bf16 -> uint8");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kByte && table.is_contiguous(),
              "quant_rows: table must be a device byte tensor");
  const int64_t eb = (int64_t)pdt::quant_rows_entry_bytes();
  TORCH_CHECK(table.numel() % eb == 0, "quant_rows: table size");
  c10::hip::HIPGuard gd(src.get_device());
  pdt::launch_quant_rows_e4m3(cbf(src), dst.data_ptr<uint8_t>(), scale.data_ptr<float>(), table.data_ptr(),
                              (int)(table.numel() / eb), (int)max_rows, cur_stream(src));
}

// ---------------------------------------------------------------- augment
// images: uint8 or fp32 [N,C,H,W] (device); idx/oy/ox int64 [B]; flip bool [B] or None
Tensor augment(const Tensor& images, const Tensor& idx, const Tensor& oy, const Tensor& ox,
               const std::optional<Tensor>& flip, int64_t pad, bool normalize, std::vector<double> mean,
               std::vector<double> stdv) {
  check_cuda(images, "images");
  TORCH_CHECK(images.dim() == 4 && (images.scalar_type() == at::kByte || images.scalar_type() == at::kFloat),
              "images must be uint8 or fp32 NCHW");
  for (const Tensor* t : {&idx, &oy, &ox})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->is_contiguous() && t->numel() == idx.numel(),
                "idx/oy/ox must be device int64 [B]");
  const bool* fp = nullptr;
  if (flip.has_value() && flip->defined()) {
    TORCH_CHECK(flip->is_cuda() && flip->scalar_type() == at::kBool && flip->numel() == idx.numel(),
                "flip must be device bool [B]");
    fp = flip->data_ptr<bool>();
  }
  TORCH_CHECK(mean.size() >= (size_t)images.size(1) && stdv.size() >= (size_t)images.size(1), "mean/std per channel");
  c10::hip::HIPGuard g(images.get_device());
  const int B = idx.numel(), C = images.size(1), H = images.size(2), W = images.size(3);
  float m[3] = {0.f, 0.f, 0.f}, sd[3] = {1.f, 1.f, 1.f};
  for (int c = 0; c < C; ++c) { m[c] = (float)mean[c]; sd[c] = (float)stdv[c]; }
  auto out = at::empty({B, C, H, W}, images.options().dtype(at::kFloat));
  pdt::launch_augment(images.data_ptr(), images.scalar_type() == at::kByte, idx.data_ptr<int64_t>(),
                      oy.data_ptr<int64_t>(), ox.data_ptr<int64_t>(), fp, out.data_ptr<float>(), B, C, H, W,
                      (int)pad, normalize, m, sd, cur_stream(images));
  return out;
}

// -------------------------------------------------------------------- pool
std::tuple<Tensor, Tensor> maxpool_fwd(const Tensor& x) {
  check_bf16_nhwc(x, "x");
  c10::hip::HIPGuard g(x.get_device());
  int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  auto idx = at::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  pdt::launch_maxpool_fwd(cbf(x), bf(y), idx.data_ptr<uint8_t>(), N, H, W, C, Ho, Wo, cur_stream(x));
  return {y, idx};
}

Tensor maxpool_bwd(const Tensor& dy, const Tensor& idx, int64_t H, int64_t W) {
  check_bf16_nhwc(dy, "dy");
  c10::hip::HIPGuard g(dy.get_device());
  int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), C = dy.size(3);
  auto dx = at::empty({N, H, W, C}, dy.options());
  pdt::launch_maxpool_bwd(cbf(dy), idx.data_ptr<uint8_t>(), bf(dx), N, H, W, C, Ho, Wo, cur_stream(dy));
  return dx;
}

// stem: (pooled, idx) = maxpool3x3s2(relu(y*scale + shift)) without writing the ReLU output;
// with argmax_y also u = y at each window's argmax (what the BN backward reduction needs from y:
// it then streams the pooled tensors instead of gathering over the full-resolution y)
py::tuple bn_relu_maxpool(const Tensor& y, const Tensor& scale, const Tensor& shift, bool argmax_y) {
  check_bf16_nhwc(y, "y");
  check_cuda(scale, "scale");
  check_cuda(shift, "shift");
  c10::hip::HIPGuard g(y.get_device());
  int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  TORCH_CHECK(scale.numel() == C && shift.numel() == C && scale.scalar_type() == at::kFloat &&
              shift.scalar_type() == at::kFloat, "scale/shift must be fp32 [C]");
  int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  auto out = at::empty({N, Ho, Wo, C}, y.options());
  auto idx = at::empty({N, Ho, Wo, C}, y.options().dtype(at::kByte));
  Tensor u;
  if (argmax_y) u = at::empty({N, Ho, Wo, C}, y.options());
  pdt::launch_bn_relu_maxpool(cbf(y), scale.data_ptr<float>(), shift.data_ptr<float>(), bf(out),
                              idx.data_ptr<uint8_t>(), argmax_y ? bf(u) : nullptr, N, H, W, C, Ho, Wo,
                              cur_stream(y));
  if (argmax_y) return py::make_tuple(out, idx, u);
  return py::make_tuple(out, idx);
}

static void check_pool_grad(const Tensor& dpool, const Tensor& idx, const Tensor& y) {
  check_bf16_nhwc(dpool, "dpool");
  check_bf16_nhwc(y, "y");
  check_cuda(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.sizes() == dpool.sizes(), "idx must be uint8 like dpool");
  TORCH_CHECK(dpool.size(0) == y.size(0) && dpool.size(3) == y.size(3) &&
              dpool.size(1) == (y.size(1) - 1) / 2 + 1 && dpool.size(2) == (y.size(2) - 1) / 2 + 1,
              "dpool must be the 3x3/s2/p1 max pool of y");
}

// sums[2][K] of the stem BN backward with dz = maxpool_bwd(dpool, idx) gathered on the fly
Tensor pool_bn_bwd_reduce(const Tensor& dpool, const Tensor& idx, const Tensor& y, const Tensor& stats,
                          const std::optional<Tensor>& dgamma, const std::optional<Tensor>& dbeta) {
  check_pool_grad(dpool, idx, y);
  c10::hip::HIPGuard g(y.get_device());
  int N = y.size(0), H = y.size(1), W = y.size(2), K = y.size(3);
  TORCH_CHECK(stats.numel() == 4 * K && stats.is_contiguous(), "stats must be [4, K]");
  auto fopt = y.options().dtype(at::kFloat);
  auto ws = at::empty({(int64_t)pdt::pool_bn_bwd_ws_floats((int64_t)N * H * W, K)}, fopt);
  auto sums = at::empty({2, K}, fopt);
  float* dg = nullptr;
  float* db = nullptr;
  if (dgamma.has_value() && dgamma->defined()) {
    TORCH_CHECK(dbeta.has_value() && dbeta->defined(), "dgamma and dbeta go together");
    TORCH_CHECK(dgamma->numel() == K && dbeta->numel() == K && dgamma->is_contiguous() &&
                dbeta->is_contiguous() && dgamma->scalar_type() == at::kFloat, "bad dgamma/dbeta");
    dg = dgamma->data_ptr<float>();
    db = dbeta->data_ptr<float>();
  }
  pdt::launch_pool_bn_bwd_reduce(cbf(dpool), idx.data_ptr<uint8_t>(), cbf(y), stats.data_ptr<float>(), N, H,
                                 W, K, dpool.size(1), dpool.size(2), ws.data_ptr<float>(),
                                 sums.data_ptr<float>(), dg, db, cur_stream(y));
  return sums;
}

Tensor pool_bn_bwd_apply(const Tensor& dpool, const Tensor& idx, const Tensor& y, const Tensor& stats,
                         const Tensor& gamma, const Tensor& sums, bool training) {
  check_pool_grad(dpool, idx, y);
  c10::hip::HIPGuard g(y.get_device());
  int N = y.size(0), H = y.size(1), W = y.size(2), K = y.size(3);
  TORCH_CHECK(stats.numel() == 4 * K && stats.is_contiguous(), "stats must be [4, K]");
  TORCH_CHECK(sums.numel() == 2 * K && gamma.numel() == K, "sums [2, K] / gamma [K]");
  auto dy = at::empty_like(y);
  pdt::launch_pool_bn_bwd_apply(cbf(dpool), idx.data_ptr<uint8_t>(), cbf(y), stats.data_ptr<float>(),
                                gamma.data_ptr<float>(), sums.data_ptr<float>(), training, N, H, W, K,
                                dpool.size(1), dpool.size(2), bf(dy), cur_stream(y));
  return dy;
}

Tensor avgpool_fwd(const Tensor& x) {
  check_bf16_nhwc(x, "x");
  c10::hip::HIPGuard g(x.get_device());
  int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  auto y = at::empty({N, C}, x.options().dtype(at::kFloat));
  pdt::launch_avgpool_fwd(cbf(x), y.data_ptr<float>(), N, HW, C, cur_stream(x));
  return y;
}

// dy: fp32 [N, C], or [splits, N, C] split-K partials of the fc dgrad (summed here, in order)
Tensor avgpool_bwd(const Tensor& dy, int64_t H, int64_t W) {
  check_cuda(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == at::kFloat && dy.is_contiguous() && (dy.dim() == 2 || dy.dim() == 3),
              "avgpool_bwd: dy must be contiguous fp32 [N, C] or [splits, N, C]");
  c10::hip::HIPGuard g(dy.get_device());
  const int splits = dy.dim() == 3 ? (int)dy.size(0) : 1;
  int N = dy.size(dy.dim() - 2), C = dy.size(dy.dim() - 1);
  auto dx = at::empty({N, H, W, C}, dy.options().dtype(at::kBFloat16));
  pdt::launch_avgpool_bwd(dy.data_ptr<float>(), bf(dx), N, (int)(H * W), C, cur_stream(dy), splits);
  return dx;
}

// ---------------------------------------------------------------------- fc
static void check_f32(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous(), name, " must be contiguous fp32");
}

// logits[N][V] = pooled[N][C] . W[V][C]^T + b
Tensor fc_forward(const Tensor& pooled, const Tensor& w, const Tensor& b) {
  check_f32(pooled, "pooled"); check_f32(w, "weight"); check_f32(b, "bias");
  TORCH_CHECK(pooled.dim() == 2 && w.dim() == 2 && w.size(1) == pooled.size(1) && b.numel() == w.size(0),
              "fc_forward: pooled [N, C], weight [V, C], bias [V]");
  c10::hip::HIPGuard g(pooled.get_device());
  const int N = pooled.size(0), C = pooled.size(1), V = w.size(0);
  auto out = at::empty({N, V}, pooled.options());
  pdt::FcArgs a{};
  a.a = pooled.data_ptr<float>(); a.b = w.data_ptr<float>(); a.c = out.data_ptr<float>();
  a.bias = b.data_ptr<float>();
  a.M = N; a.N = V; a.K = C; a.sam = C; a.sak = 1; a.sbn = C; a.sbk = 1; a.ldc = V;
  a.splits = pdt::fc_splits(N, V, C);
  a.kper = (C + a.splits - 1) / a.splits;
  a.kper = (a.kper + 31) / 32 * 32;
  a.splits = (C + a.kper - 1) / a.kper;
  Tensor ws;
  if (a.splits > 1) {
    ws = at::empty({a.splits, N, V}, pooled.options());
    a.ws = ws.data_ptr<float>();
  }
  hipStream_t st = cur_stream(pooled);
  pdt::launch_fc_gemm(a, st);
  if (a.splits > 1) pdt::launch_fc_splitk_reduce(a.ws, a.splits, N, V, a.bias, a.c, V, st);
  return out;
}

// Backward of the fc: returns (dpooled partials [splits, N, C] for avgpool_bwd, dW, db).  dW / db
// accumulate into `dw_out` / `db_out` when given (flat gradient views), else come back fresh.
std::tuple<Tensor, Tensor, Tensor> fc_backward(const Tensor& dlogits, const Tensor& pooled, const Tensor& w,
                                               const std::optional<Tensor>& dw_out,
                                               const std::optional<Tensor>& db_out) {
  check_f32(dlogits, "dlogits"); check_f32(pooled, "pooled"); check_f32(w, "weight");
  const int N = dlogits.size(0), V = dlogits.size(1), C = pooled.size(1);
  TORCH_CHECK(pooled.size(0) == N && w.size(0) == V && w.size(1) == C, "fc_backward: shape mismatch");
  c10::hip::HIPGuard g(dlogits.get_device());
  hipStream_t st = cur_stream(dlogits);
  Tensor dw, db;
  const bool acc_w = dw_out.has_value() && dw_out->defined();
  const bool acc_b = db_out.has_value() && db_out->defined();
  if (acc_w) {
    TORCH_CHECK(dw_out->scalar_type() == at::kFloat && dw_out->numel() == (int64_t)V * C &&
                dw_out->stride(0) == C && dw_out->stride(1) == 1, "dw_out must be fp32 [V, C] row-major");
    dw = *dw_out;
  } else {
    dw = at::empty({V, C}, w.options());
  }
  if (acc_b) {
    TORCH_CHECK(db_out->scalar_type() == at::kFloat && db_out->numel() == V && db_out->is_contiguous(),
                "db_out must be contiguous fp32 [V]");
    db = *db_out;
  } else {
    db = at::empty({V}, w.options());
  }
  // dW[V][C] (+)= dlogits^T . pooled: A(m = v, k = n) = dlogits[n][v], B(k = n, n = c) = pooled[n][c]
  pdt::FcArgs a{};
  a.a = dlogits.data_ptr<float>(); a.b = pooled.data_ptr<float>(); a.c = dw.data_ptr<float>();
  a.M = V; a.N = C; a.K = N; a.sam = 1; a.sak = V; a.sbn = 1; a.sbk = C; a.ldc = C;
  a.splits = 1; a.kper = N; a.accumulate = acc_w ? 1 : 0;
  if (acc_w == acc_b) {  // db from the same pass (shares the accumulate flag)
    a.db = db.data_ptr<float>();
    pdt::launch_fc_gemm(a, st);
  } else {
    pdt::launch_fc_gemm(a, st);
    pdt::launch_fc_colsum(dlogits.data_ptr<float>(), N, V, nullptr, db.data_ptr<float>(), acc_b, st);
  }
  // dpooled[N][C] = dlogits . W: A(m = n, k = v) = dlogits[n][v], B(k = v, n = c) = W[v][c]
  pdt::FcArgs d{};
  d.a = dlogits.data_ptr<float>(); d.b = w.data_ptr<float>();
  d.M = N; d.N = C; d.K = V; d.sam = V; d.sak = 1; d.sbn = 1; d.sbk = C; d.ldc = C;
  d.splits = pdt::fc_splits(N, C, V);
  d.kper = ((V + d.splits - 1) / d.splits + 31) / 32 * 32;
  d.splits = (V + d.kper - 1) / d.kper;
  auto dp = at::empty({d.splits, N, C}, dlogits.options());
  if (d.splits > 1) d.ws = dp.data_ptr<float>();
  else d.c = dp.data_ptr<float>();
  pdt::launch_fc_gemm(d, st);
  return {dp, dw, db};
}

// -------------------------------------------------------------------- head
std::tuple<Tensor, Tensor> softmax_xent(const Tensor& logits_in, const Tensor& labels) {
  check_cuda(logits_in, "logits");
  c10::hip::HIPGuard g(logits_in.get_device());
  Tensor logits = logits_in.scalar_type() == at::kFloat ? logits_in : logits_in.to(at::kFloat);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  int N = logits.size(0), V = logits.size(1);
  auto loss = at::empty({}, logits.options());
  auto dl = at::empty_like(logits);
  auto ws = at::empty({N}, logits.options());
  pdt::launch_softmax_xent(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), loss.data_ptr<float>(),
                           dl.data_ptr<float>(), ws.data_ptr<float>(), N, V, cur_stream(logits));
  return {loss, dl};
}

// x * alpha for a device scalar alpha (the upstream gradient of the loss), fp32
Tensor scale_by(const Tensor& x, const Tensor& alpha) {
  check_f32(x, "x");
  check_cuda(alpha, "alpha");
  TORCH_CHECK(alpha.scalar_type() == at::kFloat && alpha.numel() == 1, "alpha must be a device fp32 scalar");
  c10::hip::HIPGuard g(x.get_device());
  auto y = at::empty_like(x);
  pdt::launch_scale(x.data_ptr<float>(), alpha.data_ptr<float>(), y.data_ptr<float>(), x.numel(), cur_stream(x));
  return y;
}

void add_one_i64(Tensor x) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kLong && x.is_contiguous(), "add_one_i64: contiguous int64");
  c10::hip::HIPGuard g(x.get_device());
  pdt::launch_add_one_i64(x.data_ptr<int64_t>(), x.numel(), cur_stream(x));
}

Tensor top1_correct(const Tensor& logits_in, const Tensor& labels) {
  check_cuda(logits_in, "logits");
  c10::hip::HIPGuard g(logits_in.get_device());
  Tensor logits = logits_in.scalar_type() == at::kFloat ? logits_in : logits_in.to(at::kFloat);
  int N = logits.size(0), V = logits.size(1);
  auto cnt = at::empty({}, labels.options().dtype(at::kLong));
  pdt::launch_top1(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), cnt.data_ptr<int64_t>(), N, V,
                   cur_stream(logits));
  return cnt;
}

// --------------------------------------------------------------------- sgd
void sgd_step(Tensor p, const Tensor& g, const std::optional<Tensor>& buf_opt, double lr, double momentum,
              double dampening, double wd, bool nesterov, bool first, double grad_scale,
              const std::optional<Tensor>& p_bf16) {
  check_cuda(p, "param");
  check_cuda(g, "grad");
  TORCH_CHECK(p.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat, "fp32 flat buffers only");
  TORCH_CHECK(p.numel() == g.numel(), "param/grad size mismatch");
  bool mom = momentum != 0.0;
  Tensor buf = buf_opt.has_value() ? *buf_opt : Tensor();  // momentum 0: no buffer (None)
  if (mom) {
    TORCH_CHECK(buf.defined(), "sgd_step: momentum != 0 needs a momentum buffer");
    check_cuda(buf, "momentum_buffer");
    TORCH_CHECK(buf.numel() == p.numel(), "momentum buffer size mismatch");
  }
  auto aligned = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  TORCH_CHECK(aligned(p.data_ptr()) && aligned(g.data_ptr()) && (!mom || aligned(buf.data_ptr())),
              "sgd_step: flat buffers must be 16-byte aligned");
  uint16_t* pb = nullptr;
  if (p_bf16.has_value() && p_bf16->defined()) {
    check_cuda(*p_bf16, "p_bf16");
    TORCH_CHECK(p_bf16->scalar_type() == at::kBFloat16 && p_bf16->numel() == p.numel(),
                "sgd_step: bf16 mirror must match the parameter buffer");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(p_bf16->data_ptr()) & 15) == 0, "mirror must be 16-B aligned");
    pb = bf(*p_bf16);
  }
  c10::hip::HIPGuard gd(p.get_device());
  pdt::launch_sgd(p.data_ptr<float>(), g.data_ptr<float>(), mom ? buf.data_ptr<float>() : nullptr,
                  p.numel(), (float)lr, (float)momentum, (float)dampening, (float)wd, nesterov, first,
                  (float)grad_scale, cur_stream(p), pb);
}

// flat fp32 -> bf16 mirror (refresh when parameters changed outside the fused SGD step)
void cast_to_bf16(const Tensor& x, Tensor y) {
  check_cuda(x, "x");
  check_cuda(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kFloat && y.scalar_type() == at::kBFloat16 && x.numel() == y.numel(),
              "cast_to_bf16: fp32 -> bf16 of equal size");
  c10::hip::HIPGuard gd(x.get_device());
  pdt::launch_cast_f32_bf16(x.data_ptr<float>(), bf(y), x.numel(), cur_stream(x));
}

// table: int64 [n][4] = (offset, K, C, RS) on the device; src/dst: flat bf16 mirrors
void pack_t_batched(const Tensor& src, Tensor dst, const Tensor& table, int64_t max_tiles) {
  check_cuda(src, "src");
  check_cuda(dst, "dst");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kByte && table.is_contiguous(),
              "pack_t_batched: table must be a device byte tensor");
  const int64_t eb = (int64_t)pdt::pack_t_entry_bytes();
  TORCH_CHECK(table.numel() % eb == 0, "pack_t_batched: table size");
  c10::hip::HIPGuard gd(src.get_device());
  pdt::launch_pack_t_batched(cbf(src), bf(dst), table.data_ptr(), (int)(table.numel() / eb),
                             (int)max_tiles, cur_stream(src));
}

int64_t pack_t_entry_bytes() { return (int64_t)pdt::pack_t_entry_bytes(); }

// ------------------------------------------------------------------- fp8
// (wq uint8 e4m3 [K,R,S,Cp], oscale fp32 [K]); act_deq: optional 1-element dequant factor of the
// activation operand, folded into oscale
std::tuple<Tensor, Tensor> pack_weight_fp8(const Tensor& w, int64_t cpad, const std::optional<Tensor>& act_deq) {
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kFloat, "weight must be fp32 4-D");
  c10::hip::HIPGuard g(w.get_device());
  int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  int Cp = std::max<int>((int)cpad, C);
  auto wq = at::empty({K, R, S, Cp}, w.options().dtype(at::kByte));
  auto osc = at::empty({K}, w.options());
  const float* ad = nullptr;
  if (act_deq.has_value() && act_deq->defined()) {
    TORCH_CHECK(act_deq->is_cuda() && act_deq->scalar_type() == at::kFloat && act_deq->numel() >= 1,
                "act_deq must be a device fp32 scalar");
    ad = act_deq->data_ptr<float>();
  }
  int64_t st[4] = {w.stride(0), w.stride(1), w.stride(2), w.stride(3)};
  pdt::launch_pack_weight_fp8(w.data_ptr<float>(), st, wq.data_ptr<uint8_t>(), osc.data_ptr<float>(), ad, K,
                              C, R, S, Cp, cur_stream(w));
  return {wq, osc};
}

Tensor quant_e4m3(const Tensor& x, Tensor state, int64_t slot) {
  check_bf16_nhwc(x, "x");
  check_state(state, slot);
  c10::hip::HIPGuard g(x.get_device());
  auto q = at::empty(x.sizes(), x.options().dtype(at::kByte));
  pdt::launch_quant_e4m3(cbf(x), q.data_ptr<uint8_t>(), x.numel(), state.data_ptr<float>(), (int)slot,
                         cur_stream(x));
  return q;
}

// (z, q, zmask); zmask is undefined unless want_mask (needs relu)
std::tuple<Tensor, Tensor, Tensor> bn_act_fwd_q8(const Tensor& y, const Tensor& scale, const Tensor& shift,
                                                 const std::optional<Tensor>& res, bool relu, Tensor state,
                                                 int64_t slot, bool want_mask, bool want_z) {
  check_bf16_nhwc(y, "y");
  check_state(state, slot);
  c10::hip::HIPGuard g(y.get_device());
  int K = y.size(3);
  int64_t M = y.numel() / K;
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_bf16_nhwc(*res, "residual");
    TORCH_CHECK(res->sizes() == y.sizes(), "residual shape mismatch");
    rp = cbf(*res);
  }
  TORCH_CHECK(!want_mask || relu, "a ReLU mask needs relu");
  Tensor z;
  if (want_z) z = at::empty_like(y);  // else: fp8-only activation, every consumer reads q
  auto q = at::empty(y.sizes(), y.options().dtype(at::kByte));
  Tensor zm;
  if (want_mask) zm = at::empty({y.numel() / 8}, y.options().dtype(at::kByte));
  pdt::launch_bn_act_fwd_q8(cbf(y), scale.data_ptr<float>(), shift.data_ptr<float>(), rp, relu,
                            want_z ? bf(z) : nullptr,
                            q.data_ptr<uint8_t>(), M, K, state.data_ptr<float>(), (int)slot, cur_stream(y),
                            want_mask ? zm.data_ptr<uint8_t>() : nullptr);
  return {z, q, zm};
}

// fp8 forward conv; with `bn` = (count, rm, rv, gamma, beta, momentum, eps, acc) the BN finalize runs
// inside the conv as in conv_fwd_bn, and the second result is the [4][K] statistics, not partials
std::tuple<Tensor, Tensor> conv_fwd_fp8(const Tensor& x, const Tensor& wq, const Tensor& oscale,
                                        int64_t stride, int64_t pad, bool stats,
                                        const std::optional<Tensor>& ascale, const std::optional<py::tuple>& bn) {
  check_u8_nhwc(x, "x");
  check_cuda(wq, "wq");
  TORCH_CHECK(wq.scalar_type() == at::kByte && wq.dim() == 4 && wq.size(3) == x.size(3),
              "packed fp8 weight must be uint8 [K,R,S,Cx]");
  TORCH_CHECK(oscale.is_cuda() && oscale.scalar_type() == at::kFloat && oscale.numel() == wq.size(0),
              "oscale must be fp32 [K]");
  c10::hip::HIPGuard g(x.get_device());
  auto s = shape_of(x.size(0), x.size(1), x.size(2), x.size(3), wq.size(0), wq.size(1), wq.size(2),
                    stride, pad);
  TORCH_CHECK(s.K % 8 == 0, "output channels must be a multiple of 8");
  auto y = at::empty({s.N, s.Ho, s.Wo, s.K}, x.options().dtype(at::kBFloat16));
  Tensor part;
  float* pp = nullptr;
  int M = s.N * s.Ho * s.Wo;
  std::optional<pdt::BnFwdFuse> fuse;
  if (bn.has_value()) {
    const py::tuple& b = *bn;
    TORCH_CHECK(b.size() == 8, "bn = (count, rm, rv, gamma, beta, momentum, eps, acc)");
    auto opt = [](const py::handle& h) { return h.is_none() ? Tensor() : h.cast<Tensor>(); };
    fuse = bn_fwd_fuse(x, s.K, b[0].cast<int64_t>(), M, b[7].cast<Tensor>(), opt(b[1]), opt(b[2]),
                       b[3].cast<Tensor>(), b[4].cast<Tensor>(), b[5].cast<double>(), b[6].cast<double>(), part);
  } else if (stats) {
    int grows = pdt::conv_nt_group_rows(M, s.K, s.R * s.S * s.C);
    part = at::empty({(M + grows - 1) / grows, 2, s.K}, x.options().dtype(at::kFloat));
    pp = part.data_ptr<float>();
  }
  const float* asp = nullptr;
  if (ascale.has_value() && ascale->defined()) {
    TORCH_CHECK(ascale->is_cuda() && ascale->scalar_type() == at::kFloat && ascale->numel() >= 1,
                "ascale must be a device fp32 scalar");
    asp = ascale->data_ptr<float>();
  }
  pdt::launch_conv_fwd_fp8(x.data_ptr<uint8_t>(), wq.data_ptr<uint8_t>(), oscale.data_ptr<float>(), asp,
                           bf(y), pp, s, cur_stream(x), fuse ? &*fuse : nullptr);
  return {y, part};
}

// a, b: uint8 [64, 32] per-lane operand registers; returns fp32 [64, 4] accumulators
Tensor mfma_f8_probe(const Tensor& a, const Tensor& b, int64_t fmt_a, int64_t fmt_b, int64_t scale_a,
                     int64_t scale_b, bool use_scale) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  TORCH_CHECK(a.scalar_type() == at::kByte && b.scalar_type() == at::kByte && a.numel() == 64 * 32 &&
              b.numel() == 64 * 32, "probe operands: uint8 [64, 32]");
  TORCH_CHECK((fmt_a == 0 || fmt_a == 1) && (fmt_b == 0 || fmt_b == 1), "fmt: 0 = e4m3, 1 = e5m2");
  c10::hip::HIPGuard g(a.get_device());
  auto d = at::empty({64, 4}, a.options().dtype(at::kFloat));
  pdt::launch_mfma_f8_probe(a.data_ptr(), b.data_ptr(), d.data_ptr<float>(), (int)fmt_a, (int)fmt_b,
                            (int)scale_a, (int)scale_b, use_scale ? 1 : 0, cur_stream(a));
  return d;
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X (gfx950) native kernels, RCCL communicator and DDP reducer";
  m.def("image_to_nhwc", checked("image_to_nhwc", &image_to_nhwc));
  m.def("pack_weight", checked("pack_weight", &pack_weight), py::arg("w"), py::arg("cpad") = 0);
  m.def("pack_weight_t", checked("pack_weight_t", &pack_weight_t));
  m.def("conv_fwd", checked("conv_fwd", &conv_fwd), py::arg("x"), py::arg("wk"), py::arg("stride"), py::arg("pad"),
        py::arg("stats"));
  m.def("conv_dgrad", checked("conv_dgrad", &conv_dgrad), py::arg("dy"), py::arg("w"), py::arg("x_shape"), py::arg("stride"),
        py::arg("pad"), py::arg("addend") = py::none(), py::arg("wt") = py::none());
  m.def("conv_dgrad_bn", checked("conv_dgrad_bn", &conv_dgrad_bn), py::arg("dy"), py::arg("w"),
        py::arg("x_shape"), py::arg("stride"), py::arg("pad"), py::arg("addend"), py::arg("y"),
        py::arg("z"), py::arg("stats"), py::arg("mask"), py::arg("dgamma") = py::none(),
        py::arg("dbeta") = py::none(), py::arg("wt") = py::none(), py::arg("acc") = py::none(),
        py::arg("y2") = py::none(), py::arg("stats2") = py::none(), py::arg("acc2") = py::none());
  m.def("conv_wgrad", checked("conv_wgrad", &conv_wgrad), py::arg("dy"), py::arg("x"), py::arg("w_shape"), py::arg("stride"),
        py::arg("pad"), py::arg("deterministic") = false, py::arg("out") = py::none());
  m.def("conv_wgrad_side", checked("conv_wgrad_side", &conv_wgrad_side), py::arg("side"), py::arg("dy"),
        py::arg("x"), py::arg("w_shape"), py::arg("stride"), py::arg("pad"), py::arg("deterministic") = false,
        py::arg("out") = py::none(), py::arg("zero") = py::none());
  m.def("conv_wgrad_fp8", checked("conv_wgrad_fp8", &conv_wgrad_fp8), py::arg("side"), py::arg("dy8"),
        py::arg("x8"), py::arg("dy_deq"), py::arg("x_deq"), py::arg("w_shape"), py::arg("stride"), py::arg("pad"),
        py::arg("out") = py::none(), py::arg("zero") = py::none());
  m.def("conv_wgrad_fp8_plan", [](std::vector<int64_t> x_shape, std::vector<int64_t> w_shape, int stride, int pad) {
    pdt::ConvShape s = shape_of((int)x_shape[0], (int)x_shape[1], (int)x_shape[2], (int)x_shape[3], (int)w_shape[0],
                                (int)w_shape[2], (int)w_shape[3], stride, pad);
    int o[4];
    pdt::conv_wgrad_fp8_plan(s, o);
    py::dict d;
    d["bm"] = o[0]; d["tiles"] = o[1]; d["splits"] = o[2]; d["steps_per_split"] = o[3];
    return d;
  }, py::arg("x_shape"), py::arg("w_shape"), py::arg("stride"), py::arg("pad"));
  m.def("stem_conv_fwd", checked("stem_conv_fwd", &stem_conv_fwd), py::arg("x"), py::arg("w"),
        py::arg("stride"), py::arg("pad"), py::arg("stats"));
  m.def("stem_wgrad", checked("stem_wgrad", &stem_wgrad), py::arg("dy"), py::arg("xsp"),
        py::arg("w_shape"), py::arg("deterministic") = false, py::arg("out") = py::none());
  m.def("stem_bwd_fused", checked("stem_bwd_fused", &stem_bwd_fused), py::arg("dpool"), py::arg("idx"),
        py::arg("y"), py::arg("stats"), py::arg("gamma"), py::arg("sums"), py::arg("training"), py::arg("xsp"),
        py::arg("w_shape"), py::arg("deterministic") = false, py::arg("out") = py::none());
  m.def("stem_bwd_fused_supported", &pdt::stem_bwd_fused_supported, py::arg("K"), py::arg("R"), py::arg("Sp"),
        py::arg("Ho"), py::arg("Wo"));
  m.def("bn_finalize", checked("bn_finalize", &bn_finalize), py::arg("part"), py::arg("count"), py::arg("rm"),
        py::arg("rv"), py::arg("gamma"), py::arg("beta"), py::arg("momentum"), py::arg("eps"),
        py::arg("grows") = 0);
  m.def("bn_eval_params", checked("bn_eval_params", &bn_eval_params));
  m.def("bn_fold_weights", checked("bn_fold_weights", &bn_fold_weights), py::arg("wt"), py::arg("stats"),
        py::arg("gamma"), py::arg("sums"), py::arg("count"));
  m.def("bn_fold_wgrad", checked("bn_fold_wgrad", &bn_fold_wgrad), py::arg("t1"), py::arg("gram"),
        py::arg("colsum"), py::arg("wt"), py::arg("stats"), py::arg("gamma"), py::arg("sums"), py::arg("count"),
        py::arg("out"), py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none(),
        py::arg("done") = py::none(), py::arg("zero_sums") = false);
  m.def("conv_dgrad_bn_fold", checked("conv_dgrad_bn_fold", &conv_dgrad_bn_fold), py::arg("g"), py::arg("z_in"),
        py::arg("wfold"), py::arg("bias"), py::arg("y"), py::arg("z"), py::arg("stats"), py::arg("mask"),
        py::arg("acc") = py::none(), py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none());
  m.def("conv_fwd_bn", checked("conv_fwd_bn", &conv_fwd_bn), py::arg("x"), py::arg("wk"), py::arg("stride"),
        py::arg("pad"), py::arg("count"), py::arg("rm"), py::arg("rv"), py::arg("gamma"), py::arg("beta"),
        py::arg("momentum"), py::arg("eps"), py::arg("acc") = py::none());
  m.def("bn_act_fwd", checked("bn_act_fwd", &bn_act_fwd), py::arg("y"), py::arg("scale"), py::arg("shift"),
        py::arg("residual"), py::arg("relu"), py::arg("res_scale") = py::none(),
        py::arg("res_shift") = py::none(), py::arg("csum") = py::none());
  m.def("bn_act_fwd_mask", checked("bn_act_fwd_mask", &bn_act_fwd_mask), py::arg("y"), py::arg("scale"),
        py::arg("shift"), py::arg("residual"), py::arg("res_scale") = py::none(),
        py::arg("res_shift") = py::none());
  m.def("bn_act_bwd_reduce", checked("bn_act_bwd_reduce", &bn_act_bwd_reduce), py::arg("dz"), py::arg("z"), py::arg("y"),
        py::arg("stats"), py::arg("mask"), py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none());
  m.def("bn_act_bwd_apply", checked("bn_act_bwd_apply", &bn_act_bwd_apply), py::arg("dz"), py::arg("z"),
        py::arg("y"), py::arg("stats"), py::arg("gamma"), py::arg("sums"), py::arg("mask"), py::arg("training"),
        py::arg("want_dres"), py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none());
  m.def("augment", checked("augment", &augment), py::arg("images"), py::arg("idx"), py::arg("oy"), py::arg("ox"),
        py::arg("flip"), py::arg("pad"), py::arg("normalize"), py::arg("mean"), py::arg("std"));
  m.def("maxpool_fwd", checked("maxpool_fwd", &maxpool_fwd));
  m.def("maxpool_bwd", checked("maxpool_bwd", &maxpool_bwd));
  m.def("bn_relu_maxpool", checked("bn_relu_maxpool", &bn_relu_maxpool), py::arg("y"), py::arg("scale"),
        py::arg("shift"), py::arg("argmax_y") = false);
  m.def("pool_bn_bwd_reduce", checked("pool_bn_bwd_reduce", &pool_bn_bwd_reduce), py::arg("dpool"),
        py::arg("idx"), py::arg("y"), py::arg("stats"), py::arg("dgamma") = py::none(),
        py::arg("dbeta") = py::none());
  m.def("pool_bn_bwd_apply", checked("pool_bn_bwd_apply", &pool_bn_bwd_apply));
  m.def("avgpool_fwd", checked("avgpool_fwd", &avgpool_fwd));
  m.def("avgpool_bwd", checked("avgpool_bwd", &avgpool_bwd));
  m.def("fc_forward", checked("fc_forward", &fc_forward), py::arg("pooled"), py::arg("weight"), py::arg("bias"));
  m.def("fc_backward", checked("fc_backward", &fc_backward), py::arg("dlogits"), py::arg("pooled"),
        py::arg("weight"), py::arg("dw_out") = py::none(), py::arg("db_out") = py::none());
  m.def("scale_by", checked("scale_by", &scale_by), py::arg("x"), py::arg("alpha"));
  m.def("add_one_i64", checked("add_one_i64", &add_one_i64), py::arg("x"));
  m.def("softmax_xent", checked("softmax_xent", &softmax_xent));
  m.def("top1_correct", checked("top1_correct", &top1_correct));
  m.def("sgd_step", checked("sgd_step", &sgd_step), py::arg("p"), py::arg("g"), py::arg("buf"),
        py::arg("lr"), py::arg("momentum"), py::arg("dampening"), py::arg("wd"), py::arg("nesterov"),
        py::arg("first"), py::arg("grad_scale"), py::arg("p_bf16") = py::none());
  m.def("cast_to_bf16", checked("cast_to_bf16", &cast_to_bf16));
  m.def("pack_t_batched", checked("pack_t_batched", &pack_t_batched));
  m.def("pack_t_entry_bytes", &pack_t_entry_bytes);
  m.def("pack_weight_fp8", checked("pack_weight_fp8", &pack_weight_fp8), py::arg("w"), py::arg("cpad") = 0,
        py::arg("act_deq") = py::none());
  m.def("quant_e4m3", checked("quant_e4m3", &quant_e4m3));
  m.def("fp8_state_floats", &pdt::fp8_state_floats);
  m.def("fp8_deq_offset", &pdt::fp8_deq_offset);
  m.def("bn_act_fwd_q8", checked("bn_act_fwd_q8", &bn_act_fwd_q8), py::arg("y"), py::arg("scale"),
        py::arg("shift"), py::arg("residual"), py::arg("relu"), py::arg("state"), py::arg("slot"),
        py::arg("want_mask") = false, py::arg("want_z") = true);
  m.def("conv_fwd_fp8", checked("conv_fwd_fp8", &conv_fwd_fp8), py::arg("x"), py::arg("wq"), py::arg("oscale"),
        py::arg("stride"), py::arg("pad"), py::arg("stats"), py::arg("ascale") = py::none(),
        py::arg("bn") = py::none());
  m.def("conv_dgrad_fp8", checked("conv_dgrad_fp8", &conv_dgrad_fp8), py::arg("dy8"), py::arg("wt8"),
        py::arg("wscale"), py::arg("ascale"), py::arg("x_shape"), py::arg("stride"), py::arg("pad"),
        py::arg("addend") = py::none());
  m.def("conv_dgrad_bn_fp8", checked("conv_dgrad_bn_fp8", &conv_dgrad_bn_fp8), py::arg("dy8"), py::arg("wt8"),
        py::arg("wscale"), py::arg("ascale"), py::arg("x_shape"), py::arg("stride"), py::arg("pad"),
        py::arg("addend"), py::arg("y"), py::arg("z"), py::arg("stats"), py::arg("mask"),
        py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none(), py::arg("acc") = py::none());
  m.def("bn_act_bwd_apply_q8", checked("bn_act_bwd_apply_q8", &bn_act_bwd_apply_q8), py::arg("dz"), py::arg("z"),
        py::arg("y"), py::arg("stats"), py::arg("gamma"), py::arg("sums"), py::arg("mask"), py::arg("want_dres"),
        py::arg("state"), py::arg("slot"), py::arg("want_dy") = true, py::arg("dgamma") = py::none(),
        py::arg("dbeta") = py::none());
  m.def("quant_rows_e4m3", checked("quant_rows_e4m3", &quant_rows_e4m3));
  m.def("quant_rows_entry_bytes", []() { return (int64_t)pdt::quant_rows_entry_bytes(); });
  m.def("mfma_f8_probe", checked("mfma_f8_probe", &mfma_f8_probe), py::arg("a"), py::arg("b"),
        py::arg("fmt_a") = 0, py::arg("fmt_b") = 0, py::arg("scale_a") = 127, py::arg("scale_b") = 127,
        py::arg("use_scale") = true);
  m.def("conv_nt_group_rows", &pdt::conv_nt_group_rows, py::arg("M"), py::arg("Nout"), py::arg("kg_bytes"));
  m.def("nt_timing_fetch", [](int n) {
    // PDT_NT_TIMING variant builds: [n] per-block phase timestamps of NT launches (else empty)
    auto out = torch::zeros({n}, torch::dtype(torch::kInt64));
    const int got = pdt::nt_timing_fetch(reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), n);
    return out.narrow(0, 0, got);
  }, py::arg("n"));
  m.def("xgmi_force_chunks", &pdt::xgmi_force_chunks, py::arg("n") = -1,
        "test hook: RS -> AG chunks per xGMI bucket (1..4), -1 = the size policy");
  m.def("conv_nt_force", &pdt::conv_nt_force, py::arg("k32") = -1, py::arg("mid") = -1, py::arg("wide") = -1);
  m.def("conv_nt_tile", [](int M, int Nout, int kg_bytes) {
    int bm = 0, bn = 0;
    pdt::conv_nt_tile(M, Nout, kg_bytes, &bm, &bn);
    return py::make_tuple(bm, bn);
  }, py::arg("M"), py::arg("Nout"), py::arg("kg_bytes"));
  m.def("bn_csum_slots", &pdt::bn_csum_slots, "slots of bn_act_fwd's column-sum accumulator");
  m.def("conv_wgrad_set_cu_reserve", &pdt::conv_wgrad_set_cu_reserve, py::arg("n"),
        "CUs the weight-gradient split-K plan leaves to the gradient-collective kernels");
  m.def("conv_wgrad_cu_reserve", &pdt::conv_wgrad_cu_reserve);
  m.def("conv_wgrad_plan", [](std::vector<int64_t> x_shape, std::vector<int64_t> w_shape, int stride, int pad,
                              bool deterministic) {
    TORCH_CHECK(x_shape.size() == 4 && w_shape.size() == 4, "x_shape [N,H,W,C], w_shape [K,C,R,S]");
    pdt::ConvShape s{};
    s.N = (int)x_shape[0]; s.H = (int)x_shape[1]; s.W = (int)x_shape[2]; s.C = (int)x_shape[3];
    s.K = (int)w_shape[0]; s.R = (int)w_shape[2]; s.S = (int)w_shape[3];
    s.stride = stride; s.pad = pad;
    s.Ho = (s.H + 2 * pad - s.R) / stride + 1; s.Wo = (s.W + 2 * pad - s.S) / stride + 1;
    int out[4];
    pdt::conv_wgrad_plan(s, deterministic, out);
    py::dict d;
    d["bm"] = out[0]; d["bn"] = out[1]; d["tiles"] = out[2]; d["splits"] = out[3];
    return d;
  }, py::arg("x_shape"), py::arg("w_shape"), py::arg("stride"), py::arg("pad"), py::arg("deterministic") = false);
  m.def("bn_counter_bank", [](uintptr_t stream) {
    return pdt::bn_counter_bank(reinterpret_cast<hipStream_t>(stream));
  }, py::arg("stream"));
  // Stream restricted to `ncu` of the device's CUs, evenly spaced over the CU index space (side
  // streams that should leave the rest of the chip to the critical path).  Returns the raw
  // hipStream_t (wrap with torch.cuda.ExternalStream); it lives until the process exits.
  m.def("cu_masked_stream", [](int device, int ncu) {
    c10::hip::HIPGuard guard((c10::DeviceIndex)device);
    int total = 0;
    if (hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || total <= 0)
      throw std::runtime_error("cu_masked_stream: cannot query the CU count");
    ncu = std::max(1, std::min(ncu, total));
    std::vector<uint32_t> mask((total + 31) / 32, 0u);
    for (int i = 0; i < ncu; ++i) {
      const int cu = (int)((int64_t)i * total / ncu);
      mask[cu / 32] |= 1u << (cu % 32);
    }
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
    if (e != hipSuccess) throw std::runtime_error(std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
    return reinterpret_cast<uintptr_t>(s);
  }, py::arg("device"), py::arg("ncu"));
  m.def("set_sync_check", [](bool on) { g_sync_check = on; });
  m.def("sync_check_enabled", []() { return g_sync_check; });

  py::class_<pdt::RcclComm, std::shared_ptr<pdt::RcclComm>>(m, "RcclComm")
      .def_static("unique_id", []() { return py::bytes(pdt::RcclComm::unique_id()); })
      .def(py::init([](const std::string& uid, int rank, int world, int device, double init_timeout,
                       double op_timeout, bool exit_on_error, int min_channels, int max_channels) {
             py::gil_scoped_release nogil;  // init polls until every rank joined (or the deadline)
             pdt::RcclOptions o;
             o.init_timeout_s = init_timeout;
             o.op_timeout_s = op_timeout;
             o.exit_on_error = exit_on_error;
             o.min_channels = min_channels;
             o.max_channels = max_channels;
             return std::make_shared<pdt::RcclComm>(uid, rank, world, device, o);
           }),
           py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("init_timeout") = 600.0, py::arg("op_timeout") = 600.0,
           py::arg("exit_on_error") = false, py::arg("min_channels") = 0, py::arg("max_channels") = 0)
      .def_property_readonly("rank", &pdt::RcclComm::rank)
      .def_property_readonly("world", &pdt::RcclComm::world)
      .def_property_readonly("device", &pdt::RcclComm::device)
      .def_property_readonly("stream_ptr",
                             [](const pdt::RcclComm& c) { return reinterpret_cast<uintptr_t>(c.stream()); })
      .def("all_reduce", &pdt::RcclComm::all_reduce, py::arg("t"), py::arg("op") = "sum",
           py::arg("wait_current") = true, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &pdt::RcclComm::broadcast, py::arg("t"), py::arg("root") = 0,
           py::arg("wait_current") = true)
      .def("reduce_scatter", &pdt::RcclComm::reduce_scatter, py::arg("inp"), py::arg("out"),
           py::arg("op") = "sum", py::arg("wait_current") = true)
      .def("all_gather", &pdt::RcclComm::all_gather, py::arg("inp"), py::arg("out"),
           py::arg("wait_current") = true)
      .def("comm_wait_current", &pdt::RcclComm::comm_wait_current)
      .def("current_wait_comm", &pdt::RcclComm::current_wait_comm)
      .def("synchronize", &pdt::RcclComm::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &pdt::RcclComm::barrier, py::call_guard<py::gil_scoped_release>())
      .def("abort", &pdt::RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def("comm_count", &pdt::RcclComm::comm_count)
      .def_static("version", &pdt::RcclComm::version)
      .def_property_readonly("min_channels", [](const pdt::RcclComm& c) { return c.options().min_channels; })
      .def_property_readonly("max_channels", [](const pdt::RcclComm& c) { return c.options().max_channels; })
      .def("check", &pdt::RcclComm::check)
      .def_property_readonly("healthy", &pdt::RcclComm::healthy)
      .def_property_readonly("error", &pdt::RcclComm::error)
      .def_property_readonly("init_seconds", &pdt::RcclComm::init_seconds)
      .def("inject_delay", &pdt::RcclComm::inject_delay, py::arg("seconds"));

  py::class_<pdt::XgmiComm, std::shared_ptr<pdt::XgmiComm>>(m, "XgmiComm")
      .def(py::init<int, int, int, int64_t, int, double, std::string, int, bool>(), py::arg("rank"),
           py::arg("world"), py::arg("device"), py::arg("numel"), py::arg("nbuckets"), py::arg("timeout") = 600.0,
           py::arg("wire") = "fp32", py::arg("max_blocks") = 16, py::arg("exit_on_error") = false)
      .def_property_readonly("wire", [](const pdt::XgmiComm& c) { return c.wire_bf16() ? "bf16" : "fp32"; })
      .def_property_readonly("max_blocks", &pdt::XgmiComm::max_blocks)
      .def_property_readonly("error_message", &pdt::XgmiComm::error_message)
      .def_property_readonly("rank", &pdt::XgmiComm::rank)
      .def_property_readonly("world", &pdt::XgmiComm::world)
      .def_property_readonly("device", &pdt::XgmiComm::device)
      .def_property_readonly("numel", &pdt::XgmiComm::numel)
      .def_property_readonly("stream_ptr",
                             [](const pdt::XgmiComm& c) { return reinterpret_cast<uintptr_t>(c.stream()); })
      .def("ipc_handles", [](const pdt::XgmiComm& c) { return py::bytes(c.ipc_handles()); })
      .def("open_peers", &pdt::XgmiComm::open_peers, py::arg("handles"))
      .def("link_local", &pdt::XgmiComm::link_local, py::arg("comms"))
      .def("grad_buffer", &pdt::XgmiComm::grad_buffer)
      .def_property_readonly("flags_uncached", &pdt::XgmiComm::flags_uncached)
      .def("reduce_bucket", &pdt::XgmiComm::reduce_bucket, py::arg("bucket"), py::arg("offset"),
           py::arg("count"), py::arg("average") = true)
      .def("reduce_bucket_phases", &pdt::XgmiComm::reduce_bucket_phases, py::arg("bucket"), py::arg("offset"),
           py::arg("count"), py::arg("average"), py::arg("lo"), py::arg("hi"))
      .def("comm_wait_current", &pdt::XgmiComm::comm_wait_current)
      .def("current_wait_comm", &pdt::XgmiComm::current_wait_comm)
      .def("synchronize", &pdt::XgmiComm::synchronize, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("error_code", &pdt::XgmiComm::error_code)
      .def("check", &pdt::XgmiComm::check);

  py::class_<pdt::Reducer>(m, "Reducer")
      .def(py::init<std::vector<Tensor>, std::vector<Tensor>, std::vector<int64_t>, std::vector<Tensor>,
                    std::shared_ptr<pdt::RcclComm>, py::object, py::object, bool, std::string,
                    std::shared_ptr<pdt::XgmiComm>>(),
           py::arg("params"), py::arg("grad_views"), py::arg("bucket_of_param"),
           py::arg("bucket_flats"), py::arg("comm"), py::arg("py_launch"), py::arg("py_finalize"),
           py::arg("average") = true, py::arg("wire_dtype") = "fp32", py::arg("xgmi") = nullptr)
      .def("prepare_for_backward", &pdt::Reducer::prepare_for_backward,
           py::call_guard<py::gil_scoped_release>())
      .def("mark_ready_external", &pdt::Reducer::mark_ready_external)
      .def("set_enabled", &pdt::Reducer::set_enabled)
      .def_property_readonly("enabled", &pdt::Reducer::enabled)
      .def_property_readonly("num_buckets", &pdt::Reducer::num_buckets)
      .def_property_readonly("iterations", &pdt::Reducer::iterations)
      .def("last_launch_order", &pdt::Reducer::last_launch_order)
      .def("set_timing", &pdt::Reducer::set_timing)
      .def("comm_timing", &pdt::Reducer::comm_timing, py::call_guard<py::gil_scoped_release>())
      .def("set_strict", &pdt::Reducer::set_strict)
      .def("set_aux_stream", &pdt::Reducer::set_aux_stream)
      .def_property_readonly("duplicate_marks", &pdt::Reducer::duplicate_marks)
      .def("set_optimizer", &pdt::Reducer::set_optimizer, py::arg("param_flat"), py::arg("grad_flat"))
      .def("arm_optimizer", [](pdt::Reducer& r, double lr, double mom, double damp, double wd, bool nest, bool first,
                               const std::optional<Tensor>& buf, const std::optional<Tensor>& mirror) {
             r.arm_optimizer(lr, mom, damp, wd, nest, first, buf.has_value() ? *buf : Tensor(),
                             mirror.has_value() ? *mirror : Tensor());
           }, py::arg("lr"), py::arg("momentum"), py::arg("dampening"), py::arg("weight_decay"),
           py::arg("nesterov"), py::arg("first"), py::arg("momentum_buf") = py::none(),
           py::arg("mirror") = py::none())
      .def("optimizer_applied", &pdt::Reducer::optimizer_applied)
      .def("consume_optimizer", &pdt::Reducer::consume_optimizer)
      .def_property_readonly("local", &pdt::Reducer::local);
}
