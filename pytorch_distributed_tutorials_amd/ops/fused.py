"""Fused ResNet building blocks as autograd Functions.

Each function dispatches on the device of its input:
  * device tensor -> the HIP kernels of the native extension (``_C``); a missing
    extension raises (``_ext.native()``), never silently falls back;
  * CPU tensor    -> ``ops.reference`` (PyTorch), which defines the semantics.

The unit of fusion is ``conv -> BatchNorm(batch stats) -> (+residual) -> ReLU``
(SURVEY.md §3.5 fusion points).  Forward launches: weight pack, implicit-GEMM
conv with per-tile BN partial statistics in its epilogue, a tiny stats
finalize (which also updates the running buffers), one fused
normalize/add/ReLU pass.  Backward: one reduction pass (dgamma, dbeta), one
elementwise pass producing dy (and the residual-branch gradient), then the
dgrad and wgrad implicit GEMMs.
"""
from __future__ import annotations

import os
import weakref
from typing import Optional

import torch
import torch.nn as nn

from . import reference as ref
from . import streams
from ..utils.seed import deterministic
from ._ext import native

_CPU_DTYPE = torch.float32  # activation dtype of the CPU reference path
# fused-backward switches (module constants; the unfused paths stay for the CPU reference and
# the fallbacks): BN backward inside the dgrad epilogue, and its cross-block handoff
_FUSE_DGRAD_BN = True
_BN_HANDOFF = True
_ZMASK = True  # 1-bit ReLU masks for the handoff (else read z)
_NAN_TRACE = os.environ.get("PDT_NAN_TRACE", "0") == "1"  # debug: report NaN in saved tensors
_FP8 = False  # forward convolutions on the MX-rate fp8 MFMA (set_fp8)
_FP8_BWD = True  # with fp8: also the input-gradient GEMMs
# with fp8 backward: weight gradients on the MX-rate MFMA from the e5m2 dy and the e4m3 conv input
# the forward already produced (igemm_tn_f8_kernel); deterministic runs keep the bf16 slab path
_FP8_WGRAD = True
# fp8-only storage: activations / input gradients whose every consumer reads the fp8 copy are not
# written in bf16 at all (interior bottleneck outputs, and dy of convs with fp8 dgrad + fp8 wgrad)
_FP8_ONLY = True
# _BN_ACC (non-deterministic runs only; deterministic runs always take the partial buffers):
# BN-backward sums of a BN-fused dgrad accumulated by its epilogue's fp32 atomics into a per-BN
# [2, C] buffer -- no partial buffer and no reduce launch on the main stream; the consuming apply
# adds the BN parameter gradients, and the buffer is re-zeroed on the weight-gradient side stream
# once the apply is done.  Round 3 measured it neutral (r3t); with round 4's kernels it pays
# (r4ab, interleaved: 18.78 / 18.72 ms on vs 18.86 / 18.85 off), so on.
_BN_ACC = True


def _bacc(p, c):
    """The zeroed [2, C] fp32 BN-backward sum accumulator of BatchNorm weight ``p``."""
    a = getattr(p, "_pdt_bacc", None)
    if a is None or a.numel() != 2 * c or a.device != p.device:
        a = torch.zeros(2, c, dtype=torch.float32, device=p.device)
        p._pdt_bacc = a
    return a


def _facc(p, c):
    """The zeroed fp64 [8, 2, C] forward BN-sum accumulator of BatchNorm weight ``p``: the conv
    producing the BN input adds its per-channel sums into it (one slot per XCD) and the finalize
    that reads them re-zeroes it (kernels.h BnFwdFuse)."""
    a = getattr(p, "_pdt_facc", None)
    if a is None or a.numel() != 16 * c or a.device != p.device:
        a = torch.zeros(8, 2, c, dtype=torch.float64, device=p.device)  # one slot per XCD
        p._pdt_facc = a
    return a


_FUSE_RES_BN = True  # shortcut BN applied in the block tail
# test hook (tests/test_blocks_gpu.py, mask-matched reference): when a list, every fused block
# forward appends its units' stored post-activation outputs (z, NHWC bf16), so an fp32 reference
# can take the native path's ReLU decisions and compare gradients without ReLU-flip noise
_CAPTURE = None
# diagnostic hook (bench.py PDT_DIAG_LEAD=1): when a list, every block forward / backward appends
# (tag, host perf_counter, timing event recorded on the current stream at its entry), so the host's
# lead over the device can be read per block after the run
_LEAD = None


def _lead_mark(tag: str) -> None:
    import time
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    _LEAD.append((tag, time.perf_counter(), ev))


_COMPACT_ADDEND = True  # stride-2 shortcut dgrad compact
# the projection-shortcut BN's backward sums taken in the next block's hand-off dgrad epilogue (the
# same output gradient g feeds both BNs of a downsampling block): no reduction pass over g and y_ds
_DUAL_BN = os.environ.get("PDT_DUAL_BN", "1") == "1"  # (A/B knob)
DUAL_CALLS = 0  # shortcut BNs whose backward sums came from the hand-off epilogue (tests)


def set_fp8(on: bool) -> None:
    """fp8 forward convolutions: activations e4m3 with delayed per-tensor scaling (emitted by the
    producing BatchNorm apply), weights e4m3 with per-output-channel scales, fp32 accumulation on
    v_mfma_f32_16x16x128_f8f6f4, bf16 output; backward GEMMs stay bf16 on the saved bf16 tensors."""
    global _FP8
    _FP8 = bool(on)


def fp8_enabled() -> bool:
    return _FP8


_Q8_STATES: list = []  # weak references to every _Q8State, creation order (fp8_phase_signature)


class _Q8State:
    """Delayed-scaling state of one fp8 activation producer (csrc/kernels/fp8.hip contract)."""

    __slots__ = ("buf", "t", "off", "__weakref__")

    def __init__(self, device):
        C = native()
        self.buf = torch.zeros(C.fp8_state_floats(), dtype=torch.float32, device=device)
        self.off = C.fp8_deq_offset()
        self.t = 0
        _Q8_STATES.append(weakref.ref(self))

    def next_slot(self) -> int:
        slot = self.t % 3
        self.t += 1
        return slot

    def deq(self, slot: int) -> torch.Tensor:
        return self.buf.narrow(0, self.off + slot, 1)


def fp8_ring_state() -> tuple:
    """Step counter of every live delayed-scaling slot ring (creation order): the host state a
    captured fp8 step bakes in (utils.graph.CapturedStep ``ring``)."""
    _Q8_STATES[:] = [r for r in _Q8_STATES if r() is not None]
    return tuple(r().t for r in _Q8_STATES)


def fp8_set_ring_state(ts: tuple) -> None:
    """Set the step counters read by fp8_ring_state (same order)."""
    live = [r() for r in _Q8_STATES if r() is not None]
    for st, t in zip(live, ts):
        st.t = t


FP8_RING = (fp8_ring_state, fp8_set_ring_state)


def _q8_state(owner, device, attr: str = "_pdt_q8") -> _Q8State:
    """Delayed-scaling state kept on ``owner`` (a module for forward activations, the BN gamma
    Parameter for backward gradients)."""
    st = getattr(owner, attr, None)
    if st is None or st.buf.device != device:
        st = _Q8State(device)
        setattr(owner, attr, st)
    return st


def _rows_e4m3(C, src2d: torch.Tensor):
    """Row-wise e4m3 quantization of one bf16 [rows, n] image (fallback when no flat mirror)."""
    import numpy as np
    rows, n = src2d.shape
    dt = np.dtype([("off", "<i8"), ("soff", "<i8"), ("rows", "<i4"), ("rowlen", "<i4")])
    tab = torch.from_numpy(np.array([(0, 0, rows, n)], dtype=dt).view(np.uint8).copy()).to(src2d.device)
    q = torch.empty(src2d.numel(), dtype=torch.uint8, device=src2d.device)
    sc = torch.empty(rows, dtype=torch.float32, device=src2d.device)
    C.quant_rows_e4m3(src2d.reshape(-1), q, sc, tab, rows)
    return q, sc


def _packed_krsc8(C, w, cx):
    """(e4m3 [K,R,S,Cx], per-K scale) forward weights: flat-mirror view or a fresh pack."""
    m = _mirror_of(w)
    v = m.krsc8_view(w) if m is not None and w.shape[1] == cx else None
    if v is not None:
        return v
    return C.pack_weight_fp8(w, cx)


def _packed_crsk8(C, w):
    """(e4m3 [C,R,S,K], per-C scale) dgrad weights: flat-mirror view or a fresh pack."""
    m = _mirror_of(w)
    v = m.crsk8_view(w) if m is not None else None
    if v is not None:
        return v
    k, c, r, s = w.shape
    q, sc = _rows_e4m3(C, C.pack_weight_t(w).view(c, r * s * k))
    return q.view(c, r, s, k), sc


def fp8_attach(x: torch.Tensor, owner: nn.Module) -> torch.Tensor:
    """Attach an e4m3 copy of the NHWC activation ``x`` (for the fp8 convs that consume it)."""
    if _FP8 and x.is_cuda and x.dim() == 4 and x.shape[3] % 16 == 0:
        st = _q8_state(owner, x.device)
        slot = st.next_slot()
        x._pdt_fp8 = (native().quant_e4m3(x, st.buf, slot), st.deq(slot))
    return x


def _nan_trace(tag, **tensors):
    if not _NAN_TRACE:
        return
    torch.cuda.synchronize()
    bad = [k for k, t in tensors.items() if t is not None and t.is_floating_point() and bool(torch.isnan(t).any())]
    if bad:
        print(f"[nan-trace] {tag}: NaN in {bad}", flush=True)


def set_cpu_activation_dtype(dtype: torch.dtype) -> None:
    global _CPU_DTYPE
    _CPU_DTYPE = dtype


def act_dtype(device: torch.device) -> torch.dtype:
    return torch.bfloat16 if device.type == "cuda" else _CPU_DTYPE


# ----------------------------------------------------------------------------
# image -> NHWC
# ----------------------------------------------------------------------------
def image_to_nhwc(x: torch.Tensor) -> torch.Tensor:
    """NCHW float image -> NHWC activation with C padded to 8 (no grad needed)."""
    if x.is_cuda:
        return native().image_to_nhwc(x.contiguous())
    return ref.image_to_nhwc(x, _CPU_DTYPE)


# ----------------------------------------------------------------------------
# conv + BN + (residual) + ReLU
# ----------------------------------------------------------------------------
class _ConvBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, residual, running_mean, running_var,
                stride, pad, relu, training, momentum, eps):
        k, c, r, s = weight.shape
        n, h, w, cx = x.shape
        count = n * ((h + 2 * pad - r) // stride + 1) * ((w + 2 * pad - s) // stride + 1)
        if x.is_cuda:
            C = native()
            wk = C.pack_weight(weight, cx)                       # bf16 [K,R,S,Cx]
            if training:
                buffers_ready()
                if running_mean is None:  # track_running_stats=False: updates go to scratch
                    running_mean = torch.zeros(k, device=x.device)
                    running_var = torch.ones(k, device=x.device)
                # the fused block's conv + statistics call (same kernels, same rounding)
                y, stats = C.conv_fwd_bn(x, wk, stride, pad, count, running_mean, running_var, gamma, beta,
                                         float(momentum), float(eps),
                                         None if deterministic() else _facc(gamma, k))
            else:
                y, _ = C.conv_fwd(x, wk, stride, pad, False)
                buffers_ready()
                stats = C.bn_eval_params(running_mean, running_var, gamma, beta, float(eps))
            mean, invstd, scale, shift = stats.unbind(0)
            z = C.bn_act_fwd(y, scale, shift, residual, relu)
        else:
            wk = None
            y = ref.conv2d_nhwc(x, weight, stride, pad).to(x.dtype)
            if training:
                mean, var = ref.bn_batch_stats(y)
                with torch.no_grad():
                    unbiased = var * count / max(count - 1, 1)
                    running_mean.mul_(1 - momentum).add_(mean, alpha=momentum)
                    running_var.mul_(1 - momentum).add_(unbiased, alpha=momentum)
            else:
                mean, var = running_mean.float(), running_var.float()
            invstd = torch.rsqrt(var + eps)
            z = ref.bn_act_fwd(y, mean, invstd, gamma, beta, residual, relu, x.dtype)
            sc = gamma.float() * invstd
            stats = torch.stack([mean, invstd, sc, beta.float() - mean * sc])
        ctx.save_for_backward(x, weight, y, z, stats, gamma)
        ctx.cfg = (stride, pad, relu, training, residual is not None)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, weight, y, z, stats, gamma = ctx.saved_tensors
        mean, invstd = stats[0], stats[1]
        stride, pad, relu, training, has_res = ctx.cfg
        dz = dz.contiguous()
        need_x = ctx.needs_input_grad[0]
        need_w = ctx.needs_input_grad[1]
        if dz.is_cuda:
            C = native()
            # ReLU mask: from z when a residual was added, else recomputed from y (no z read)
            mask = (1 if has_res else 2) if relu else 0
            sums = C.bn_act_bwd_reduce(dz, z, y, stats, mask)    # [sum g, sum g*(y-mean)]
            dbeta, dgamma = sums[0], sums[1] * invstd
            dy, dres = C.bn_act_bwd_apply(dz, z, y, stats, gamma, sums, mask, training, has_res)
            dx = C.conv_dgrad(dy, weight, list(x.shape), stride, pad) if need_x else None
            dw = C.conv_wgrad(dy, x, list(weight.shape), stride, pad, deterministic()) \
                if need_w else None
        else:
            dy, dgamma, dbeta, dres = ref.bn_act_bwd(dz, z, y, mean, invstd, gamma, relu,
                                                     training, has_res, x.dtype)
            dx = ref.conv2d_nhwc_dgrad(dy, weight, x.shape, stride, pad).to(x.dtype) if need_x else None
            dw = ref.conv2d_nhwc_wgrad(dy, x, weight.shape, stride, pad) if need_w else None
            if dw is not None:
                dw = dw.contiguous(memory_format=torch.channels_last) \
                    if weight.is_contiguous(memory_format=torch.channels_last) else dw
        if dw is not None:
            dw = dw.to(weight.dtype)
        return (dx, dw, dgamma.to(gamma.dtype), dbeta.to(gamma.dtype), dres,
                None, None, None, None, None, None, None, None)


class _StemConvBN(torch.autograd.Function):
    """Device stem: NCHW fp32 image -> conv 7x7/s2 -> BN -> ReLU as a super-pixel conv.

    The image is re-laid out so pairs of horizontally adjacent pixels form one 8-channel
    "super-pixel" (3 channels + pad each), the seven horizontal taps fold into four tap pairs,
    and the image is pre-padded: the implicit GEMM has K = 7*4*8 = 224 (vs 7*7*8 = 392 with
    channel padding alone) and no bounds checks.  The image itself needs no gradient.
    """

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, stride, pad, training,
                momentum, eps):
        C = native()
        xsp, y, part, grows = C.stem_conv_fwd(x, weight, stride, pad, training)
        k = weight.shape[0]
        count = y.shape[0] * y.shape[1] * y.shape[2]
        buffers_ready()
        if training:
            if running_mean is None:
                running_mean = torch.zeros(k, device=x.device)
                running_var = torch.ones(k, device=x.device)
            stats = C.bn_finalize(part, count, running_mean, running_var, gamma, beta,
                                  float(momentum), float(eps), grows)
        else:
            stats = C.bn_eval_params(running_mean, running_var, gamma, beta, float(eps))
        z = C.bn_act_fwd(y, stats[2], stats[3], None, True)
        _nan_trace("stem", x=x, xsp=xsp, y=y, part=part, stats=stats, z=z)
        ctx.save_for_backward(xsp, y, stats, gamma)
        ctx.weight = weight
        ctx.training = training
        return z

    @staticmethod
    def backward(ctx, dz):
        C = native()
        xsp, y, stats, gamma = ctx.saved_tensors
        weight = ctx.weight
        dz = dz.contiguous()
        sums = C.bn_act_bwd_reduce(dz, dz, y, stats, 2)
        dgamma, dbeta = sums[1] * stats[1], sums[0]
        dy, _ = C.bn_act_bwd_apply(dz, dz, y, stats, gamma, sums, 2, ctx.training, False)
        dw = None
        if ctx.needs_input_grad[1]:
            sink = _grad_sink(weight)
            if sink is not None:
                C.stem_wgrad(dy, xsp, list(weight.shape), deterministic(), sink)
                weight._pdt_flat.mark_ready([weight])
            else:
                dw = C.stem_wgrad(dy, xsp, list(weight.shape), deterministic()).to(weight.dtype)
        ctx.weight = None
        return (None, dw, dgamma.to(gamma.dtype), dbeta.to(gamma.dtype), None, None, None, None,
                None, None, None)


def _end_mirror_trust(weight) -> None:
    """The stem's backward is the native model's last backward node: end the bf16 weight mirror's
    per-step trust (parallel/flat.py WeightMirror.end_trust)."""
    sp = getattr(weight, "_pdt_flat", None)
    m = getattr(sp, "_mirror", None) if sp is not None else None
    if m is not None:
        m.end_trust()


class _StemConvBNPool(torch.autograd.Function):
    """_StemConvBN followed by the 3x3/s2/p1 max pool in ONE fused BN-apply/ReLU/pool pass.

    The full-resolution ReLU output (112x112x64 per image) is never written: forward normalises,
    rectifies and pools each window in registers (``bn_relu_maxpool``), backward gathers the
    pooled gradient back through the argmax inside the BN reduction and apply passes
    (``pool_bn_bwd_reduce`` / ``pool_bn_bwd_apply``).  Saves writing z and dz and reading each
    of them back (~1.6 GB of HBM traffic per step at batch 256).
    """

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, stride, pad, training,
                momentum, eps):
        C = native()
        xsp, y, part, grows = C.stem_conv_fwd(x, weight, stride, pad, training)
        k = weight.shape[0]
        count = y.shape[0] * y.shape[1] * y.shape[2]
        buffers_ready()
        if training:
            if running_mean is None:
                running_mean = torch.zeros(k, device=x.device)
                running_var = torch.ones(k, device=x.device)
            stats = C.bn_finalize(part, count, running_mean, running_var, gamma, beta,
                                  float(momentum), float(eps), grows)
        else:
            stats = C.bn_eval_params(running_mean, running_var, gamma, beta, float(eps))
        if training and _STEM_ARGMAX_Y:
            out, idx, u = C.bn_relu_maxpool(y, stats[2], stats[3], True)
        else:
            (out, idx), u = C.bn_relu_maxpool(y, stats[2], stats[3]), None
        _nan_trace("stem+pool", x=x, xsp=xsp, y=y, part=part, stats=stats, out=out)
        ctx.save_for_backward(xsp, y, stats, gamma, idx, u)
        ctx.weight = weight
        ctx.bn_params = (gamma, beta)
        ctx.training = training
        return out

    @staticmethod
    def backward(ctx, dout):
        C = native()
        xsp, y, stats, gamma, idx, u = ctx.saved_tensors
        weight = ctx.weight
        gp, bp = ctx.bn_params
        ctx.bn_params = None
        dout = dout.contiguous()
        sg, sb = _grad_sink(gp), _grad_sink(bp)
        sunk = []
        # BN reduction sum g, sum g*(y - mean): g is nonzero only at window argmaxes, so with u = y at
        # each argmax (saved by the forward pool) it is a plain streaming reduction over the pooled
        # tensors (2 x 103 MB at batch 256) instead of a gather over y (411 MB)
        if u is not None:
            red = lambda *o: C.bn_act_bwd_reduce(dout, u, u, stats, 2, *o)  # noqa: E731
        else:
            red = lambda *o: C.pool_bn_bwd_reduce(dout, idx, y, stats, *o)  # noqa: E731
        if sg is not None and sb is not None:  # BN parameter gradients straight into the flat buffer
            sums = red(sg, sb)
            dgamma = dbeta = None
            sunk += [gp, bp]
        else:
            sums = red()
            dgamma, dbeta = (sums[1] * stats[1]).to(gamma.dtype), sums[0].to(gamma.dtype)
        dw = None
        if ctx.needs_input_grad[1] and _STEM_BWD_FUSED and C.stem_bwd_fused_supported(
                weight.shape[0], weight.shape[2], (weight.shape[3] + 2) // 2, y.shape[1], y.shape[2]):
            # the image takes no gradient, so dy's only consumer is the weight gradient: the BN/pool
            # backward apply runs inside it and the full-resolution dy is never stored
            sink = _grad_sink(weight)
            if sink is not None:
                C.stem_bwd_fused(dout, idx, y, stats, gamma, sums, ctx.training, xsp, list(weight.shape),
                                 deterministic(), sink)
                sunk.append(weight)
            else:
                dw = C.stem_bwd_fused(dout, idx, y, stats, gamma, sums, ctx.training, xsp, list(weight.shape),
                                      deterministic()).to(weight.dtype)
            if sunk:
                sunk[0]._pdt_flat.mark_ready(sunk)
            _end_mirror_trust(weight)
            ctx.weight = None
            return (None, dw, dgamma, dbeta, None, None, None, None, None, None, None)
        dy = C.pool_bn_bwd_apply(dout, idx, y, stats, gamma, sums, ctx.training)
        if ctx.needs_input_grad[1]:
            sink = _grad_sink(weight)
            if sink is not None:
                C.stem_wgrad(dy, xsp, list(weight.shape), deterministic(), sink)
                sunk.append(weight)
            else:
                dw = C.stem_wgrad(dy, xsp, list(weight.shape), deterministic()).to(weight.dtype)
        if sunk:
            sunk[0]._pdt_flat.mark_ready(sunk)
        _end_mirror_trust(weight)
        ctx.weight = None
        return (None, dw, dgamma, dbeta, None, None, None, None, None, None, None)


_STEM_POOL = True  # debugging switch (default on)
_STEM_BWD_FUSED = True  # A/B switch (default on)
_STEM_ARGMAX_Y = True  # A/B switch (default on)


def _stem_fast(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and not x.requires_grad and x.dim() == 4 and x.shape[1] <= 4
            and conv.stride == (2, 2) and conv.kernel_size[0] == conv.kernel_size[1]
            and conv.bias is None)


def stem_conv_bn_pool(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d,
                      pool: nn.Module) -> torch.Tensor:
    """maxpool3x3s2(relu(BN(conv7x7/s2(image)))) -> NHWC bf16.  One fused BN/ReLU/pool pass on the
    device fast path; otherwise the unfused stem followed by the max pool."""
    std_pool = (isinstance(pool, nn.MaxPool2d) and pool.kernel_size in (3, (3, 3))
                and pool.stride in (2, (2, 2)) and pool.padding in (1, (1, 1))
                and pool.dilation in (1, (1, 1)) and not pool.ceil_mode)
    if _STEM_POOL and std_pool and _stem_fast(x, conv) and conv.out_channels <= 256:
        training, momentum, eps = _bn_prepare(bn)
        return _StemConvBNPool.apply(x.float(), conv.weight, bn.weight, bn.bias, bn.running_mean,
                                     bn.running_var, 2, conv.padding[0], training, momentum, eps)
    return maxpool3x3s2(stem_conv_bn(x, conv, bn))


def stem_conv_bn(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d) -> torch.Tensor:
    """z = relu(BN(conv7x7/s2(image))) -> NHWC bf16, device path for <= 4-channel fp32 images.
    Falls back to image_to_nhwc + conv_bn when the image itself needs a gradient."""
    if not _stem_fast(x, conv):
        return conv_bn(image_to_nhwc(x), conv, bn, relu=True)
    training, momentum, eps = _bn_prepare(bn)
    return _StemConvBN.apply(x.float(), conv.weight, bn.weight, bn.bias, bn.running_mean,
                             bn.running_var, 2, conv.padding[0], training, momentum, eps)


def conv_bn(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d, relu: bool,
            residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """z = act(BN(conv(x)) [+ residual]) on NHWC activations."""
    stride = conv.stride[0]
    pad = conv.padding[0]
    training, momentum, eps = _bn_prepare(bn)
    return _ConvBN.apply(x, conv.weight, bn.weight, bn.bias, residual,
                         bn.running_mean, bn.running_var, stride, pad, relu,
                         training, momentum, eps)


# ----------------------------------------------------------------------------
# max pool 3x3/s2/p1
# ----------------------------------------------------------------------------
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        if x.is_cuda:
            y, idx = native().maxpool_fwd(x)       # idx: argmax position 0..8 per output (uint8)
            _nan_trace("maxpool", x=x, y=y)
            ctx.save_for_backward(idx)
        else:
            y = ref.maxpool3x3s2_fwd(x)
            ctx.save_for_backward(x)
        ctx.hw = (x.shape[1], x.shape[2])
        return y

    @staticmethod
    def backward(ctx, dy):
        (saved,) = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.is_cuda:
            return native().maxpool_bwd(dy, saved, ctx.hw[0], ctx.hw[1])
        return ref.maxpool3x3s2_bwd(dy, saved)


def maxpool3x3s2(x: torch.Tensor) -> torch.Tensor:
    return _MaxPool.apply(x)


# ----------------------------------------------------------------------------
# global avg pool + fc
# ----------------------------------------------------------------------------
class _AvgPoolLinear(torch.autograd.Function):
    """Global average pool + the classifier Linear (torchvision fc, resnet/main.py:76).

    Device path: avg-pool kernel, then the hand-written fc GEMMs of ``csrc/kernels/fc.hip`` (bf16
    MFMA, fp32 accumulation) -- forward with the bias folded into its split-K reduction; backward
    dW (accumulated straight into the flat gradient buffer under DDP), db, and the input gradient,
    whose split-K partials the avg-pool backward sums while broadcasting over H x W.  No library
    GEMM and no ATen kernel runs for the head."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        if x.is_cuda:
            C = native()
            pooled = C.avgpool_fwd(x)           # fp32 [N, C]
            logits = C.fc_forward(pooled, weight.float().contiguous(), bias.float().contiguous())
        else:
            pooled = ref.global_avgpool(x)
            logits = torch.addmm(bias.float(), pooled, weight.float().t())
        ctx.save_for_backward(pooled, weight)
        ctx.params = (weight, bias)
        ctx.hw = (x.shape[1], x.shape[2], x.dtype)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        pooled, weight = ctx.saved_tensors
        wp, bp = ctx.params
        ctx.params = None
        h, w, dt = ctx.hw
        dlogits = dlogits.float().contiguous()
        if dlogits.is_cuda:
            C = native()
            sw, sb = _grad_sink(wp), _grad_sink(bp)
            if sw is not None and sb is not None and sw.is_contiguous():
                dp, _, _ = C.fc_backward(dlogits, pooled, weight.float().contiguous(), sw, sb)
                wp._pdt_flat.mark_ready([wp, bp])
                dw = db = None
            else:
                dp, dw, db = C.fc_backward(dlogits, pooled, weight.float().contiguous())
                dw, db = dw.to(weight.dtype), db.to(weight.dtype)
            dx = C.avgpool_bwd(dp, h, w)
            return dx, dw, db
        dw = dlogits.t().mm(pooled)
        db = dlogits.sum(0)
        dpooled = dlogits.mm(weight.float())
        dx = (dpooled / (h * w))[:, None, None, :].expand(-1, h, w, -1).to(dt).contiguous()
        return dx, dw.to(weight.dtype), db.to(weight.dtype)


def avgpool_linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    return _AvgPoolLinear.apply(x, weight, bias)


# ----------------------------------------------------------------------------
# softmax cross entropy (mean) -- fused fwd+bwd
# ----------------------------------------------------------------------------
class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        if logits.is_cuda:
            loss, dlogits = native().softmax_xent(logits.contiguous(), labels.contiguous())
        else:
            loss, dlogits = ref.softmax_xent(logits, labels)
        ctx.save_for_backward(dlogits)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (dlogits,) = ctx.saved_tensors
        if dlogits.is_cuda:  # scaled on the device by the (device) loss gradient: no host sync
            return native().scale_by(dlogits, dloss.float().reshape(1)), None
        return dlogits * dloss, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    return _SoftmaxXent.apply(logits, labels)


class CrossEntropyLoss(nn.Module):
    """Drop-in for ``nn.CrossEntropyLoss()`` (mean reduction, ``resnet/main.py:102``)."""

    def forward(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        return cross_entropy(logits, labels)


def top1_correct(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Number of rows whose argmax equals the label (``resnet/main.py:32-34``)."""
    if logits.is_cuda:
        return native().top1_correct(logits.contiguous(), labels.contiguous())
    return ref.top1_correct(logits, labels)


# ----------------------------------------------------------------------------
# whole residual block (device path): one autograd node per Bottleneck/BasicBlock
# ----------------------------------------------------------------------------
_NBT_BATCHED = 0  # > 0 inside bump_bn_counters(): the counters were already bumped in one launch

# BN buffers arriving from the DDP per-forward broadcast (torch DDP's _sync_buffers,
# torch/nn/parallel/distributed.py:1557): the broadcast runs on the comm stream and only the
# BatchNorm statistics kernels read/write those buffers, so the compute stream waits for it
# at the FIRST BN of the forward (after the stem convolution has been issued), not before the
# forward starts.  The counter bump writes the same (int64) flat buffer, so it is deferred too.
_BUFFER_WAIT = None   # callable: current stream waits for the buffer broadcast
_PENDING_BUMP = None  # num_batches_tracked tensors to bump once the buffers are ours


def defer_buffer_wait(fn) -> None:
    """Register the stream wait for an in-flight buffer broadcast (called by DDP)."""
    global _BUFFER_WAIT
    _BUFFER_WAIT = fn


def buffers_ready() -> None:
    """Make BN buffers safe to use on the current stream: run the deferred broadcast wait and
    the deferred counter bump (no-ops when nothing is pending)."""
    global _BUFFER_WAIT, _PENDING_BUMP
    if _BUFFER_WAIT is not None:
        fn, _BUFFER_WAIT = _BUFFER_WAIT, None
        fn()
    if _PENDING_BUMP is not None:
        counters, _PENDING_BUMP = _PENDING_BUMP, None
        with torch.no_grad():
            flat = _counter_flat(counters)
            if flat is not None:   # every counter is a view of one int64 buffer (DDP): one launch
                native().add_one_i64(flat)
            else:
                torch._foreach_add_(counters, 1)


def _counter_flat(counters):
    """The int64 buffer that exactly holds ``counters`` as consecutive one-element views (what
    ``parallel.flat.flatten_buffers`` builds when every int64 buffer is a BN counter), else None."""
    if not counters or not counters[0].is_cuda:
        return None
    base = counters[0]._base
    if base is None or base.dtype != torch.int64 or base.numel() != len(counters):
        return None
    p0 = base.data_ptr()
    for i, c in enumerate(counters):
        if c._base is not base or c.data_ptr() != p0 + 8 * i:
            return None
    return base


def forget_bn_modules(module: nn.Module) -> None:
    """Drop the BatchNorm list ``bump_bn_counters`` caches on ``module`` (collected at its first
    device forward).  Call after replacing or adding BatchNorm submodules; ``set_impl`` does."""
    module.__dict__.pop("_pdt_bn_list", None)
    module.__dict__.pop("_pdt_bn_counters", None)


class bump_bn_counters:
    """Context for one device forward of a whole model: bumps every training BatchNorm's
    ``num_batches_tracked`` (torch BN semantics) with ONE multi-tensor launch
    instead of one ``add_`` kernel per BN (53 launches per ResNet-50 step); the per-BN
    ``_bn_prepare`` calls inside the context then skip their own bump.  The launch itself is
    issued by the first BN of the forward (``buffers_ready``), behind any buffer broadcast."""

    def __init__(self, module: nn.Module):
        # the counter list is cached on the module: walking every submodule each forward cost
        # ~80 us of host issue per ResNet-18 step (scripts/host_profile.py).  Keyed by what
        # selects the counters (each BN's mode and buffer), so train()/eval() or a replaced
        # buffer rebuilds it.
        bns = getattr(module, "_pdt_bn_list", None)
        if bns is None:
            bns = [m for m in module.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
            module._pdt_bn_list = bns
        key = tuple((m.training, m.track_running_stats, id(m.num_batches_tracked)) for m in bns)
        cached = getattr(module, "_pdt_bn_counters", None)
        if cached is None or cached[0] != key:
            cached = (key, [m.num_batches_tracked for m in bns if m.training and m.track_running_stats
                            and m.num_batches_tracked is not None])
            module._pdt_bn_counters = cached
        self.counters = cached[1]

    def __enter__(self):
        global _NBT_BATCHED, _PENDING_BUMP
        if self.counters:
            _PENDING_BUMP = self.counters
        _NBT_BATCHED += 1
        return self

    def __exit__(self, *exc):
        global _NBT_BATCHED
        _NBT_BATCHED -= 1
        buffers_ready()  # a forward without BatchNorm still owes the wait and the bump
        return False


def _bn_prepare(bn: nn.BatchNorm2d):
    """(training, momentum, eps) for one BN call; bumps num_batches_tracked like torch."""
    training = bn.training or not bn.track_running_stats
    momentum = bn.momentum
    if training and bn.track_running_stats and not _NBT_BATCHED:
        with torch.no_grad():
            bn.num_batches_tracked.add_(1)
        if momentum is None:
            momentum = 1.0 / float(bn.num_batches_tracked.item())
    return training, (momentum if momentum is not None else 0.0), bn.eps


def _mirror_of(w):
    sp = getattr(w, "_pdt_flat", None)
    return sp._mirror if sp is not None else None


def _packed_krsc(C, w, cx):
    """bf16 [K,R,S,Cx] forward weights: a view of the flat-space mirror when current, else a pack."""
    m = _mirror_of(w)
    v = m.krsc_view(w) if m is not None else None
    if v is not None and v.shape[3] == cx:
        return v
    return C.pack_weight(w, cx)


def _packed_crsk(w):
    """bf16 [C,R,S,K] dgrad weights from the mirror, or None (the binding packs)."""
    m = _mirror_of(w)
    return m.crsk_view(w) if m is not None else None


def _unit_fwd(C, x, w, gamma, beta, rm, rv, stride, pad, relu, training, momentum, eps, residual,
              x8=None, q8=None, want_mask=False, want_z=True, csum=None):
    """conv -> BN -> (+residual) -> (ReLU) -> (z, y, stats, z8, zmask).  x8 = (e4m3 copy of x, its
    dequant factor): fp8 conv; q8 = _Q8State: also emit the e4m3 copy z8 of the output;
    want_mask (with relu): also the 1-bit ReLU mask zmask a later BN-fused dgrad reads instead of z.
    ``residual`` is an activation, or ``(y_short, stats_short)``: a projection shortcut's raw conv
    output and its BN statistics, normalised inside this unit's apply pass (never materialised).
    csum: fp32 [8, k] slots the apply adds the output's per-channel sums into (DgradFold colsum)."""
    y, stats = _unit_conv_stats(C, x, w, gamma, beta, rm, rv, stride, pad, training, momentum, eps, x8)
    k = w.shape[0]
    rsc = rsh = None
    if isinstance(residual, tuple):
        residual, rst = residual
        rsc, rsh = rst[2], rst[3]
    want_mask = want_mask and relu
    if q8 is not None and k % 16 == 0:
        assert rsc is None, "fp8 apply takes a materialised residual"
        slot = q8.next_slot()
        z, zq, zm = C.bn_act_fwd_q8(y, stats[2], stats[3], residual, relu, q8.buf, slot, want_mask, want_z)
        return z, y, stats, (zq, q8.deq(slot)), (zm if want_mask else None)
    if want_mask:
        z, zm = C.bn_act_fwd_mask(y, stats[2], stats[3], residual, rsc, rsh)
        return z, y, stats, None, zm
    z = C.bn_act_fwd(y, stats[2], stats[3], residual, relu, rsc, rsh, csum)
    return z, y, stats, None, None


_FP8_KMIN = 128


def _fp8_conv_ok(r, s, cx):
    """fp8 forward conv for a GEMM K of r*s*cx >= _FP8_KMIN (K = 64 half-fills the 128-wide fp8
    K-step).  128 (layer2's 1x1 over 128 channels on fp8, so its input needs no bf16 copy) vs 256:
    fp8 b512 31.23 vs 31.39 ms, b256 17.04 vs 17.01 ms (r3p, one box).  64 (every layer-1 1x1 on
    fp8 too, after the narrow fp8 dgrad) vs 128: b256 16.88 vs 16.77 ms, b512 31.09 vs 30.83 ms
    (r3ap, one box)."""
    return r * s * cx >= _FP8_KMIN


_FP8_DGRAD_NARROW = True


def _fp8_dgrad_ok(k, stride):
    """fp8 input gradient for a dy of k channels: whole 128-byte K-steps per tap (k % 128), or
    (_FP8_DGRAD_NARROW) any k % 16 at stride 1 -- the 64-channel layer-1 convs, whose
    dy then needs no bf16 copy at all when the weight gradient is fp8 too."""
    return k % 128 == 0 or (_FP8_DGRAD_NARROW and stride == 1 and k % 16 == 0)


def _fp8_only_ok(w_next, k, tr):
    """May unit output z (k channels, training) skip its bf16 copy?  Only when every reader takes the
    e4m3 copy: the next conv's forward GEMM and its fp8 weight gradient (backward masks of interior
    units are recomputed from y, so z itself is never read there)."""
    if not (tr and _FP8_BWD and _FP8_WGRAD and _FP8_ONLY) or deterministic():
        return False
    kn, cn, rn, sn = w_next.shape
    return cn == k and k % 16 == 0 and kn % 64 == 0 and _fp8_conv_ok(rn, sn, k)


def _unit_conv_stats(C, x, w, gamma, beta, rm, rv, stride, pad, training, momentum, eps, x8=None):
    """conv -> BN statistics (finalize, running-stat update): (y, stats[4, K])."""
    k, _, r, s = w.shape
    n, h, wd, cx = (x if x is not None else x8[0]).shape  # x None: an fp8-only activation
    count = n * ((h + 2 * pad - r) // stride + 1) * ((wd + 2 * pad - s) // stride + 1)
    if x8 is not None and not _fp8_conv_ok(r, s, cx) and x is not None:
        x8 = None  # a GEMM K of 64 (1x1 over 64 channels) half-fills the 128-wide fp8 K-step: bf16 is faster
    if x8 is None and training and not _NAN_TRACE:
        # conv + BN finalize in one host call (the running-stat update waits for the buffers first)
        buffers_ready()
        return C.conv_fwd_bn(x, _packed_krsc(C, w, cx), stride, pad, count, rm, rv, gamma, beta,
                             float(momentum), float(eps), None if deterministic() else _facc(gamma, w.shape[0]))
    if x8 is not None:
        wq, wsc = _packed_krsc8(C, w, cx)
        if training and not _NAN_TRACE and not deterministic():
            # BN finalize inside the conv (conv_fwd_bn's fused path)
            buffers_ready()
            return C.conv_fwd_fp8(x8[0], wq, wsc, stride, pad, True, x8[1],
                                  (count, rm, rv, gamma, beta, float(momentum), float(eps), _facc(gamma, k)))
        y, part = C.conv_fwd_fp8(x8[0], wq, wsc, stride, pad, training, x8[1])
    else:
        wk = _packed_krsc(C, w, cx)
        y, part = C.conv_fwd(x, wk, stride, pad, training)
    if _NAN_TRACE:
        m = _mirror_of(w)
        _nan_trace(f"unit_fwd {tuple(x.shape)}->{tuple(y.shape)} mirror={m is not None and m.krsc_view(w) is wk}",
                   x=x, wk=wk, y=y, part=part)
    buffers_ready()
    if training:
        stats = C.bn_finalize(part, count, rm, rv, gamma, beta, float(momentum), float(eps))
    else:
        stats = C.bn_eval_params(rm, rv, gamma, beta, float(eps))
    return y, stats


class _BnHandoff:
    """What a block leaves on its output tensor so the NEXT block's backward can run this
    block's last BatchNorm backward (relu mask + reduction) inside its own input-gradient
    dgrad epilogue.  The consumer deposits (g, sums); the producer uses them only if the
    gradient it receives IS that g (same storage: no other consumer added to it)."""

    __slots__ = ("y", "stats", "gamma", "beta", "zmask", "deposit", "ds")

    def __init__(self, y, stats, gamma, beta, zmask=None, ds=None):
        self.y, self.stats, self.gamma, self.beta, self.zmask = y, stats, gamma, beta, zmask
        # ds: (y, stats, gamma) of the block's projection-shortcut BN -- fed by the same output
        # gradient g, so the consumer's epilogue reduces it too (kernels.h BnBwdFuse::y2)
        self.ds = ds
        self.deposit = None


class _ResidualBlock(torch.autograd.Function):
    """z = relu(unit_n(...unit_1(x)) + shortcut(x)) with unit = conv -> BN -> (ReLU).

    One autograd node per block lets backward fuse across units: the shortcut
    gradient is summed into the block-input gradient inside the first conv's
    dgrad epilogue (no separate add kernel); each unit's BatchNorm backward
    (ReLU mask and the per-channel reduction) runs inside the epilogue of the dgrad
    that produces its input gradient (``conv_dgrad_bn``), including -- through a
    ``_BnHandoff`` -- the previous block's last unit; the remaining per-unit pass is
    one elementwise apply.
    tensors = per unit (w, gamma, beta, running_mean, running_var), chain units
    first, then the downsample unit if present.
    """

    @staticmethod
    def forward(ctx, x, spec, handoff, fp8io, *tensors):
        C = native()
        _nan_trace(f"block-in {tuple(x.shape)}", x=x)
        if _LEAD is not None:
            _lead_mark(f"fwd {tuple(x.shape)}")
        chain, ds_cfg, spec_tail = spec
        nch = len(chain)
        saved = [x]
        # fp8io = (x8, per-chain-unit _Q8State list, holder for the output's e4m3 copy) or None
        x8, q8s, holder = fp8io if fp8io is not None else (None, None, None)
        # shortcut first (it only needs x) so its output can be freed into the tail's add
        ds_join = None
        if ds_cfg is not None:
            w, g, b, rm, rv = tensors[5 * nch:5 * nch + 5]
            st, pd, tr, mo, ep = ds_cfg
            br = streams.branch_stream(x.device) if x.is_cuda and nch > 1 else None
            if q8s is None and _FUSE_RES_BN and br is not None:
                # projection shortcut on the branch stream, concurrent with the chain's first
                # units; the tail unit (which applies its BN inside the residual add) waits
                buffers_ready()  # a deferred BN-buffer wait lands on this stream, before the fork
                main = streams.fork(br, x)
                with torch.cuda.stream(br):
                    y_ds, st_ds = _unit_conv_stats(C, x, w, g, b, rm, rv, st, pd, tr, mo, ep, x8)
                ds_join = (main, streams.join(br, main, y_ds, st_ds))
                res = (y_ds, st_ds)
            elif q8s is None and _FUSE_RES_BN:
                # projection shortcut: conv + statistics only; its BN apply runs inside the block
                # tail's apply pass (bn_act_fwd RESBN), so the normalised shortcut is never stored
                y_ds, st_ds = _unit_conv_stats(C, x, w, g, b, rm, rv, st, pd, tr, mo, ep, x8)
                res = (y_ds, st_ds)
            else:
                res, y_ds, st_ds, _, _ = _unit_fwd(C, x, w, g, b, rm, rv, st, pd, False, tr, mo, ep, None, x8)
        else:
            res = x
        h, h8 = x, x8
        outs = []
        ins8 = [x8]  # e4m3 copy (q, dequant factor) of each chain unit's conv input, or None
        zmask = None
        # the last unit's folded weight gradient needs sum_m of its conv input: summed by the apply
        # that writes that input (no reduction pass in backward)
        fold_fwd = not spec_tail and fp8io is None and _fold_colsum_ok(chain, tensors, x)
        det_fwd = deterministic()
        csum = _csum_slots(tensors[5 * (nch - 1)], x.device) if fold_fwd and not det_fwd else None
        ctx.colsum = csum
        for i, (st, pd, tr, mo, ep) in enumerate(chain):
            w, g, b, rm, rv = tensors[5 * i:5 * i + 5]
            last = i == nch - 1
            if last and ds_join is not None:
                ds_join[0].wait_event(ds_join[1])
            # the block output's ReLU mask as bits: the next block's BN-fused dgrad reads it
            # instead of z (1/16 of the bytes)
            want_z = last or q8s is None or not _fp8_only_ok(tensors[5 * (i + 1)], w.shape[0], tr)
            z, y, stt, h8, zm = _unit_fwd(C, h, w, g, b, rm, rv, st, pd, True, tr, mo, ep,
                                          res if last else None, h8, q8s[i] if q8s else None,
                                          want_mask=last and tr and _ZMASK and _BN_HANDOFF and _FUSE_DGRAD_BN,
                                          want_z=want_z, csum=csum if i == nch - 2 else None)
            if z is None and h8 is None:
                raise RuntimeError("fp8-only activation without its e4m3 copy")
            if fold_fwd and det_fwd and i == nch - 2:
                # deterministic runs (no atomics): the fixed-order column-sum reduction of the last
                # unit's conv input runs here, on the weight-gradient stream -- idle during the
                # forward -- instead of at the end of backward, where that stream is the tail
                side = streams.wgrad_stream(z.device)
                streams.fork(side, z)
                with torch.cuda.stream(side):
                    ctx.colsum = C.bn_act_bwd_reduce(z, z, z, _zero_stats(z.shape[3], z.device), 0)[0]
            if last:
                zmask = zm
            else:
                ins8.append(h8)
            outs.append((z, y, stt))
            h = z
        if holder is not None and h8 is not None:
            holder.append(h8)
        if _CAPTURE is not None:
            _CAPTURE.append([z for z, _, _ in outs])
        for ui, (z, y, stt) in enumerate(outs):
            saved += [z, y, stt]
            _nan_trace(f"fwd block{id(ctx) % 10007} unit{ui} {tuple(y.shape)}", z=z, y=y, stats=stt)
        if ds_cfg is not None:
            saved += [y_ds, st_ds]
        ctx.save_for_backward(*saved, *tensors)
        ctx.params = tensors  # the Parameter objects: gradients may be written into flat views
        ctx.spec = spec
        ctx.ntensors = len(tensors)
        ctx.handoff_in = handoff  # the producer of x (previous block), or None
        ctx.fp8b = fp8io is not None and _FP8_BWD  # fp8 dgrads in backward (dy in e5m2)
        ctx.in8 = ins8 if ctx.fp8b and _FP8_WGRAD else None  # fp8 weight-gradient operands
        _, y_last, st_last = outs[-1]
        ctx.handoff_out = _BnHandoff(y_last, st_last, tensors[5 * (nch - 1) + 1],
                                     tensors[5 * (nch - 1) + 2], zmask,
                                     (y_ds, st_ds, tensors[5 * nch + 1]) if ds_cfg is not None and _DUAL_BN else None)
        return h

    @staticmethod
    def backward(ctx, dz):
        C = native()
        if _LEAD is not None:
            _lead_mark(f"bwd {tuple(dz.shape)}")
        chain, ds_cfg, _ = ctx.spec
        nch = len(chain)
        sv = ctx.saved_tensors
        x = sv[0]
        units = [sv[1 + 3 * i:4 + 3 * i] for i in range(nch)]
        pos = 1 + 3 * nch
        if ds_cfg is not None:
            y_ds, st_ds = sv[pos:pos + 2]
            pos += 2
        tensors = sv[pos:]
        if _NAN_TRACE:
            for ui, (z_, y_, s_) in enumerate(units):
                _nan_trace(f"bwd-entry block{id(ctx) % 10007} unit{ui} {tuple(y_.shape)}", z=z_, y=y_, stats=s_)
            _nan_trace(f"bwd-entry block{id(ctx) % 10007} dz", dz=dz)
        grads = [None] * ctx.ntensors
        dz = dz.contiguous()
        det = deterministic()
        g_short = None
        params = ctx.params
        sunk = []  # parameters whose gradient was accumulated in place into the flat buffer

        side = streams.begin(x.device)

        in8 = ctx.in8
        ctx.in8 = None

        deferred = {}  # unit j -> (accumulator, dgamma sink, dbeta sink): BN sums from epilogue atomics

        def wgrad(j, dy_, xin_, st_, pd_, d8_=None, x8_=None):
            w_ = tensors[j]
            sink = _grad_sink(params[j])
            dfr = deferred.pop(j, None)
            zero = dfr[0] if dfr is not None else None  # its apply is queued: re-zero on the side stream
            k_, c_ = w_.shape[0], w_.shape[1]
            if (d8_ is not None and x8_ is not None and not det and c_ % 16 == 0 and k_ % 64 == 0
                    and x8_[0].shape[3] == c_):
                # e5m2 dy x e4m3 x on the MX-rate MFMA, both already produced for the fp8 GEMMs
                if sink is not None:
                    C.conv_wgrad_fp8(side.cuda_stream if side is not None else 0, d8_[0], x8_[0], d8_[1],
                                     x8_[1], list(w_.shape), st_, pd_, sink, zero)
                    sunk.append(params[j])
                else:
                    grads[j] = C.conv_wgrad_fp8(0, d8_[0], x8_[0], d8_[1], x8_[1], list(w_.shape), st_,
                                                pd_, None, zero).to(w_.dtype)
                return
            if dy_ is None or xin_ is None:
                raise RuntimeError("fp8-only operands reached the bf16 weight gradient")
            if sink is not None:
                # weight gradient into the flat buffer on the side stream, concurrent with the
                # dgrad chain; all-reduce and optimizer wait for that stream (streams.py)
                if side is not None:  # one native call: stream hand-off, launch, record_stream
                    C.conv_wgrad_side(side.cuda_stream, dy_, xin_, list(w_.shape), st_, pd_, det, sink, zero)
                    zero = None
                else:
                    C.conv_wgrad(dy_, xin_, list(w_.shape), st_, pd_, det, sink)
                sunk.append(params[j])
            else:
                grads[j] = C.conv_wgrad(dy_, xin_, list(w_.shape), st_, pd_, det).to(w_.dtype)
            if zero is not None:
                zero.zero_()

        def bnreduce(j, dz_, z_, y_, stt_, mask_):
            if z_ is None:  # fp8-only z: interior units recompute the ReLU mask from y (mask 2)
                assert mask_ != 1
                z_ = y_
            sg, sb = _grad_sink(params[j + 1]), _grad_sink(params[j + 2])
            if sg is not None and sb is not None:
                sums_ = C.bn_act_bwd_reduce(dz_, z_, y_, stt_, mask_, sg, sb)
                sunk.extend([params[j + 1], params[j + 2]])
            else:
                sums_ = C.bn_act_bwd_reduce(dz_, z_, y_, stt_, mask_)
                grads[j + 1] = sums_[1] * stt_[1]
                grads[j + 2] = sums_[0]
            return sums_

        def apply(j, dz_, z_, y_, stt_, sums_, mask_, tr_, want_dres, need_dgrad, x8_=None, stride_=0):
            """BN backward apply of unit j -> (dy, dres, d8); d8 = (e5m2 dy, its dequant factor)
            when the dgrad consuming dy runs on fp8 (_fp8_dgrad_ok for the conv's stride), or the
            weight gradient does (K % 64 == 0 and the conv input's e4m3 copy x8_ exists)"""
            gamma_ = tensors[j + 1]
            k_ = dz_.shape[3]
            dfr = deferred.get(j)
            pg = (dfr[1], dfr[2]) if dfr is not None else (None, None)
            wgrad8 = (x8_ is not None and not det and k_ % 64 == 0 and tensors[j].shape[1] % 16 == 0
                      and x8_[0].shape[3] == tensors[j].shape[1])
            dgrad8 = _fp8_dgrad_ok(k_, stride_)
            if ctx.fp8b and tr_ and ((need_dgrad and dgrad8) or wgrad8):
                stq = _q8_state(params[j + 1], dz_.device, "_pdt_q8b")
                slot = stq.next_slot()
                # fp8-only dy: the dgrad (if any) and the weight gradient both read the e5m2 copy
                want_dy = not (_FP8_ONLY and wgrad8 and (not need_dgrad or dgrad8))
                dy_, dres_, q_ = C.bn_act_bwd_apply_q8(dz_, z_ if z_ is not None else y_, y_, stt_, gamma_,
                                                       sums_, mask_, want_dres, stq.buf, slot, want_dy, *pg)
                return dy_, dres_, (q_, stq.deq(slot))
            dy_, dres_ = C.bn_act_bwd_apply(dz_, z_ if z_ is not None else y_, y_, stt_, gamma_, sums_, mask_,
                                            tr_, want_dres, *pg)
            return dy_, dres_, None

        def dgrad(dy_, d8_, w_, xshape, st_, pd_, addend_):
            if d8_ is not None and _fp8_dgrad_ok(d8_[0].shape[3], st_):
                wt8, wsc = _packed_crsk8(C, w_)
                return C.conv_dgrad_fp8(d8_[0], wt8, wsc, d8_[1], xshape, st_, pd_, addend_)
            return C.conv_dgrad(dy_, w_, xshape, st_, pd_, addend_, _packed_crsk(w_))

        def dgrad_bn_any(dy_, d8_, w_, xshape, st_, pd_, addend_, y_, z_, stt_, mask_, sg=None, sb=None, acc=None,
                         bn2=None):
            if d8_ is not None and _fp8_dgrad_ok(d8_[0].shape[3], st_):
                assert bn2 is None
                wt8, wsc = _packed_crsk8(C, w_)
                return C.conv_dgrad_bn_fp8(d8_[0], wt8, wsc, d8_[1], xshape, st_, pd_, addend_, y_, z_,
                                           stt_, mask_, sg, sb, acc)
            if bn2 is not None:
                return C.conv_dgrad_bn(dy_, w_, xshape, st_, pd_, addend_, y_, z_, stt_, mask_, sg, sb,
                                       _packed_crsk(w_), acc, bn2[0], bn2[1], bn2[2])
            return C.conv_dgrad_bn(dy_, w_, xshape, st_, pd_, addend_, y_, z_, stt_, mask_, sg, sb,
                                   _packed_crsk(w_), acc)

        def dgrad_bn(j, dy_, d8_, w_, xshape, st_, pd_, addend_, y_, z_, stt_, mask_):
            """input gradient of a conv + BN backward reduction of unit j (its producer)"""
            sg, sb = _grad_sink(params[j + 1]), _grad_sink(params[j + 2])
            if sg is not None and sb is not None and _BN_ACC and not det:
                acc = _bacc(params[j + 1], stt_.shape[1])
                g_, sums_ = dgrad_bn_any(dy_, d8_, w_, xshape, st_, pd_, addend_, y_, z_, stt_, mask_, acc=acc)
                deferred[j] = (acc, sg, sb)  # the apply of unit j adds dgamma / dbeta
                sunk.extend([params[j + 1], params[j + 2]])
            elif sg is not None and sb is not None:
                g_, sums_ = dgrad_bn_any(dy_, d8_, w_, xshape, st_, pd_, addend_, y_, z_, stt_, mask_, sg, sb)
                sunk.extend([params[j + 1], params[j + 2]])
            else:
                g_, sums_ = dgrad_bn_any(dy_, d8_, w_, xshape, st_, pd_, addend_, y_, z_, stt_, mask_)
                grads[j + 1] = sums_[1] * stt_[1]
                grads[j + 2] = sums_[0]
            return g_, sums_

        def shortcut_backward(g_short_):
            """projection shortcut: BN backward (reduce + apply), weight gradient, and the input
            gradient that the first conv's dgrad epilogue adds (None when x needs none)"""
            st2, pd2, tr2, _, _ = ds_cfg
            wds = tensors[5 * nch]
            if sums_ds_dep is not None:
                # reduced by the next block's hand-off epilogue: the apply adds dgamma / dbeta and the
                # weight gradient re-zeroes the accumulator (as for every acc-mode BN)
                global DUAL_CALLS
                DUAL_CALLS += 1
                sums_ds = sums_ds_dep
                deferred[5 * nch] = (sums_ds, _grad_sink(params[5 * nch + 1]), _grad_sink(params[5 * nch + 2]))
                sunk.extend([params[5 * nch + 1], params[5 * nch + 2]])
            else:
                sums_ds = bnreduce(5 * nch, g_short_, g_short_, y_ds, st_ds, 0)
            dy_ds, _, d8_ds = apply(5 * nch, g_short_, g_short_, y_ds, st_ds, sums_ds, 0, tr2, False,
                                    ctx.needs_input_grad[0], in8[0] if in8 else None, st2)
            wgrad(5 * nch, dy_ds, x, st2, pd2, d8_ds, in8[0] if in8 else None)
            if not ctx.needs_input_grad[0]:
                return None
            if st2 == 2 and pd2 == 0 and wds.shape[2] == 1 and wds.shape[3] == 1 and _COMPACT_ADDEND:
                # 1x1/s2 shortcut: its input gradient is zero at every odd (h, w), so it is
                # computed as a dense 1x1 dgrad on the stride-2 grid and the first conv's
                # dgrad epilogue adds it at even positions only (no full-resolution tensor,
                # no all-zero parity-class launches)
                n_, h_, w_, c_ = x.shape
                return dgrad(dy_ds, d8_ds, wds, [n_, (h_ + 1) // 2, (w_ + 1) // 2, c_], 1, 0, None)
            return dgrad(dy_ds, d8_ds, wds, list(x.shape), st2, pd2, None)

        ds_br = streams.branch_stream(x.device) if ds_cfg is not None and x.is_cuda else None
        ds_join = None

        # gradient arriving pre-masked and pre-reduced from the next block's dgrad epilogue?
        pre = None
        ho = ctx.handoff_out
        sums_ds_dep = None  # the shortcut BN's (sum g, sum g*(y_ds - mean)) from the same epilogue
        if ho.deposit is not None:
            g_dep, sums_dep, acc_dep, acc2_dep = ho.deposit
            ho.deposit = None
            if acc2_dep is not None:
                if g_dep.data_ptr() == dz.data_ptr() and g_dep.shape == dz.shape:
                    sums_ds_dep = acc2_dep
                else:
                    acc2_dep.zero_()
            jl = 5 * (nch - 1)
            if g_dep.data_ptr() == dz.data_ptr() and g_dep.shape == dz.shape:
                pre = (dz, sums_dep)
                sunk.extend([params[jl + 1], params[jl + 2]])
                if acc_dep is not None:  # atomic sums: this block's apply adds dgamma / dbeta
                    deferred[jl] = (acc_dep, _grad_sink(params[jl + 1]), _grad_sink(params[jl + 2]))
            elif acc_dep is not None:  # another consumer contributed: discard the unused sums
                acc_dep.zero_()
            else:  # another consumer contributed: undo the deposited BN-parameter gradients
                inv = units[nch - 1][2][1]
                with torch.no_grad():
                    _grad_sink(params[jl + 1]).sub_(sums_dep[1] * inv)
                    _grad_sink(params[jl + 2]).sub_(sums_dep[0])
        ctx.handoff_out = None

        for i in reversed(range(nch)):
            st, pd, tr, mo, ep = chain[i]
            z, y, stt = units[i]
            w, gamma = tensors[5 * i], tensors[5 * i + 1]
            xin = x if i == 0 else units[i - 1][0]  # None: fp8-only (its e4m3 copy is in8[i])
            xin_shape = list((xin if xin is not None else units[i - 1][1]).shape)
            last = i == nch - 1
            need_dx = i > 0 or ctx.needs_input_grad[0]
            if pre is None:
                mask = 1 if last else 2  # inner units: ReLU mask recomputed from y, z never read
                sums = bnreduce(5 * i, dz, z, y, stt, mask)
                dy, dres, d8 = apply(5 * i, dz, z, y, stt, sums, mask, tr, last, need_dx, in8[i] if in8 else None,
                                     st)
            else:
                g, sums = pre  # g = dz * relu'(unit i), reduced in the producing epilogue
                dres = g
            fold = None
            if pre is not None and _fold_ok(i, last, w, xin, st, pd, tr, det, side, ctx.fp8b, params):
                # BN backward folded into the input gradient (kernels.h DgradFold): the dgrad below
                # reads [g | x] against [w*k1 | W^T diag(a) W] + bias instead of the applied dy, so the
                # apply -- now feeding only the weight gradient -- runs on the side stream with it
                wt = _packed_crsk(w)
                if wt is None:
                    wt = C.pack_weight_t(w)
                global FOLD_CALLS
                FOLD_CALLS += 1
                k_, c_ = w.shape[0], w.shape[1]
                count = y.numel() // k_
                fold = C.bn_fold_weights(wt.view(c_, k_), stt, gamma, sums, count)
                # the weight gradient without dy either: dW = diag(k1) g^T x + diag(a) W x^T x + b sum(x),
                # on the side stream (also the BN parameter gradients and the accumulator re-zero)
                streams.fork(side, g, stt, sums, wt, xin)
                with torch.cuda.stream(side):
                    # T1 and Gram accumulate into persistent zeroed workspaces that bn_fold_wgrad
                    # clears after reading (with the consumed BN-sum accumulator): no memset / fill
                    t1, gram, done = _fold_ws(k_, c_, xin.device)
                    C.conv_wgrad(g, xin, [k_, c_, 1, 1], 1, 0, det, t1)
                    C.conv_wgrad(xin, xin, [c_, c_, 1, 1], 1, 0, det, gram)
                    colsum = ctx.colsum  # forward: [S, C] atomic slots, or (deterministic) [C] sums
                    if colsum is None:
                        colsum = C.bn_act_bwd_reduce(xin, xin, xin, _zero_stats(c_, xin.device), 0)[0]
                    ctx.colsum = None  # consumed: bn_fold_wgrad re-zeroes the [S, C] slots
                    dfr = deferred.pop(5 * i, None)
                    C.bn_fold_wgrad(t1, gram, colsum, wt.view(c_, k_), stt, gamma, sums, count,
                                    _grad_sink(params[5 * i]), dfr[1] if dfr is not None else None,
                                    dfr[2] if dfr is not None else None, done, dfr is not None)
                sunk.append(params[5 * i])
            elif pre is not None:
                dy, _, d8 = apply(5 * i, g, g, y, stt, sums, 0, tr, False, need_dx, in8[i] if in8 else None, st)
            pre = None
            if fold is None:
                wgrad(5 * i, dy, xin, st, pd, d8, in8[i] if in8 else None)
            if last:
                g_short = dres
                if ds_cfg is not None and nch > 1 and ds_br is not None:
                    # projection-shortcut backward on the branch stream, concurrent with the
                    # chain's remaining units; the first conv's dgrad waits for its addend
                    main = streams.fork(ds_br, g_short, y_ds, st_ds, x)
                    with torch.cuda.stream(ds_br):
                        addend_br = shortcut_backward(g_short)
                    ds_join = (main, streams.join(ds_br, main, addend_br), addend_br)
            if i > 0:
                yp, sttp = units[i - 1][1], units[i - 1][2]
                if fold is not None:
                    j = 5 * (i - 1)
                    if det:  # fixed-order partials + reduce; dgamma / dbeta straight into the sinks
                        pre = C.conv_dgrad_bn_fold(g, xin, fold[0], fold[1], yp, None, sttp, 2, None,
                                                   _grad_sink(params[j + 1]), _grad_sink(params[j + 2]))
                    else:
                        acc = _bacc(params[j + 1], sttp.shape[1])
                        pre = C.conv_dgrad_bn_fold(g, xin, fold[0], fold[1], yp, None, sttp, 2, acc)
                        deferred[j] = (acc, _grad_sink(params[j + 1]), _grad_sink(params[j + 2]))
                    sunk.extend([params[j + 1], params[j + 2]])
                elif _FUSE_DGRAD_BN:
                    pre = dgrad_bn(5 * (i - 1), dy, d8, w, xin_shape, st, pd, None, yp, None, sttp, 2)
                else:
                    dz = dgrad(dy, d8, w, xin_shape, st, pd, None)
            else:
                # shortcut gradient: identity -> g_short itself; projection -> its dgrad
                if ds_join is not None:
                    ds_join[0].wait_event(ds_join[1])
                    addend = ds_join[2]
                elif ds_cfg is not None:
                    addend = shortcut_backward(g_short)
                else:
                    addend = g_short
                if not ctx.needs_input_grad[0]:
                    dz = None
                else:
                    hi = ctx.handoff_in
                    sg = _grad_sink(hi.gamma) if hi is not None else None
                    sb = _grad_sink(hi.beta) if hi is not None else None
                    if sg is not None and sb is not None and _BN_HANDOFF and _FUSE_DGRAD_BN:
                        # previous block's last unit: relu mask from its output z = x
                        zsrc, zmode = (hi.zmask, 3) if hi.zmask is not None else (x, 1)
                        if _BN_ACC and not det:
                            acc = _bacc(hi.gamma, hi.stats.shape[1])
                            # the previous block's projection-shortcut BN reduced in the same epilogue
                            ds2 = hi.ds if (hi.ds is not None and zmode == 3 and addend is not None
                                            and (d8 is None or not _fp8_dgrad_ok(d8[0].shape[3], st))
                                            and _grad_sink(hi.ds[2]) is not None) else None
                            acc2 = _bacc(hi.ds[2], hi.stats.shape[1]) if ds2 is not None else None
                            dz, sums_in = dgrad_bn_any(dy, d8, w, list(x.shape), st, pd, addend, hi.y, zsrc,
                                                       hi.stats, zmode, acc=acc,
                                                       bn2=(ds2[0], ds2[1], acc2) if ds2 is not None else None)
                            hi.deposit = (dz, sums_in, acc, acc2)
                        else:
                            dz, sums_in = dgrad_bn_any(dy, d8, w, list(x.shape), st, pd, addend, hi.y, zsrc,
                                                       hi.stats, zmode, sg, sb)
                            hi.deposit = (dz, sums_in, None, None)
                    else:
                        dz = dgrad(dy, d8, w, list(x.shape), st, pd, addend)
        ctx.handoff_in = None
        for acc_, _, _ in deferred.values():  # (every unit's weight gradient re-zeroes its own)
            acc_.zero_()
        if ctx.colsum is not None:  # summed in forward but not folded (no hand-off into this block)
            if ctx.colsum.dim() == 2:  # the atomic slots must be left zeroed
                ctx.colsum.zero_()
            ctx.colsum = None
        if sunk:
            sunk[0]._pdt_flat.mark_ready(sunk)
        return (dz, None, None, None, *grads)


# Fold the last unit's BN backward into its 1x1 input gradient (DgradFold) -- ResNet-50 b256 in the
# same calls: 18.15 vs 18.29 and 18.27 vs 18.54 ms/step (r6r / r6s); removing that apply altogether
# bounds the gain at 1.47 ms (r6f), the rest is spent in the fold-weight kernels on the critical
# stream (~20 us per block in-step) and the larger dgrad K.
_FOLD_BN = True
FOLD_CALLS = 0  # folded units so far (tests check that the path engaged)


def _fold_ok(i, last, w, xin, st, pd, tr, det, side, fp8b, params) -> bool:
    """May the last unit of a bottleneck fold its BN backward into its 1x1 input gradient
    (kernels.h DgradFold)?  bf16, training, a weight-gradient side stream, a 1x1 / stride-1 conv over
    a materialised input, and gradient sinks for the BN of the unit before (its sums go to an atomic
    accumulator, or in deterministic runs to fixed-order partials with dgamma / dbeta written by the
    reduce; the fold's weight-gradient GEMMs then take the slab split-K)."""
    if not (_FOLD_BN and last and i > 0 and tr and side is not None and not fp8b and _BN_ACC
            and _FUSE_DGRAD_BN and xin is not None):
        return False
    k, c, r, s_ = w.shape
    if r != 1 or s_ != 1 or st != 1 or pd != 0 or k % 256 or k > 2048 or c % 64 or xin.shape[3] != c:
        return False
    j = 5 * (i - 1)
    return (_grad_sink(params[j + 1]) is not None and _grad_sink(params[j + 2]) is not None
            and _grad_sink(params[5 * i]) is not None)


def _fold_colsum_ok(chain, tensors, x) -> bool:
    """Will the last unit's folded weight gradient (DgradFold) want sum_m of its conv input?  The
    static half of _fold_ok: a training bottleneck whose last conv is a foldable 1x1, bf16, with a
    weight-gradient side stream and a flat-space gradient sink."""
    nch = len(chain)
    if nch < 2 or not x.is_cuda or _FP8 or not (_FOLD_BN and _BN_ACC and _FUSE_DGRAD_BN):
        return False
    st, pd, tr, _, _ = chain[-1]
    w = tensors[5 * (nch - 1)]
    k, c, r, s_ = w.shape
    if not tr or r != 1 or s_ != 1 or st != 1 or pd != 0 or k % 256 or k > 2048 or c % 64 or 256 % (c // 8):
        return False
    return streams.wgrad_stream(x.device) is not None and _grad_sink(w) is not None


def _csum_slots(w, dev):
    """The zeroed [S, C] fp32 column-sum slots (S = C.bn_csum_slots()) the apply of the unit before
    the last atomically fills (bn_fold_wgrad re-zeroes them after use), one set per folded conv."""
    c = w.shape[1]
    cs = getattr(w, "_pdt_csum", None)
    if cs is None or cs.shape[1] != c or cs.device != dev:
        cs = torch.zeros(native().bn_csum_slots(), c, dtype=torch.float32, device=dev)
        w._pdt_csum = cs
    return cs


_ZSTATS = {}
_FOLD_WS = {}


def _fold_ws(k, c, dev):
    """Persistent (T1 [k, c, 1, 1], Gram [c, c, 1, 1], completion counter) fp32 workspaces of the
    folded weight gradient, zeroed once; every consumer (bn_fold_wgrad in consume mode) leaves them
    zeroed again.  Units of one shape reuse them in order on the weight-gradient stream."""
    ws = _FOLD_WS.get((k, c, dev))
    if ws is None:
        ws = _FOLD_WS[(k, c, dev)] = (torch.zeros(k, c, 1, 1, device=dev), torch.zeros(c, c, 1, 1, device=dev),
                                      torch.zeros(c // 64 + 1, dtype=torch.int32, device=dev))
    return ws


def _zero_stats(c, dev):
    """Zero [4, c] BN statistics (a column sum through bn_act_bwd_reduce), cached per device."""
    z = _ZSTATS.get((c, dev))
    if z is None:
        z = _ZSTATS[(c, dev)] = torch.zeros(4, c, device=dev)
    return z


def _grad_sink(p):
    """Flat-buffer gradient view to accumulate into, if the parameter lives in a FlatParamSpace."""
    sp = getattr(p, "_pdt_flat", None)
    if sp is None or not p.requires_grad or not p.is_cuda:
        return None
    return sp.grad_sink(p)


def _unit_tensors(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> list:
    """(weight, gamma, beta, running_mean, running_var) of one conv+BN unit, read from the module
    dicts directly: nn.Module.__getattr__'s fallback path for parameters and buffers was ~40 us of
    host issue per ResNet-18 step (scripts/host_profile.py)."""
    bp, bb = bn._parameters, bn._buffers
    return [conv._parameters["weight"], bp["weight"], bp["bias"], bb["running_mean"], bb["running_var"]]


def residual_block(x: torch.Tensor, chain, downsample=None, tail: bool = False) -> torch.Tensor:
    """Device path of a ResNet block: ``chain`` = [(conv, bn), ...] (ReLU after each BN, the
    shortcut added before the last ReLU), ``downsample`` = (conv, bn) or None.  ``tail``: the
    network's last block (no next block hands its last BN backward into this one, so its
    folded weight gradient cannot run and the forward takes no column sums for it)."""
    spec_chain, tensors = [], []
    for conv, bn in chain:
        tr, mo, ep = _bn_prepare(bn)
        spec_chain.append((conv.stride[0], conv.padding[0], tr, mo, ep))
        tensors += _unit_tensors(conv, bn)
    ds_spec = None
    if downsample is not None:
        conv, bn = downsample
        tr, mo, ep = _bn_prepare(bn)
        ds_spec = (conv.stride[0], conv.padding[0], tr, mo, ep)
        tensors += _unit_tensors(conv, bn)
    fp8io = None
    if _FP8:
        q8s = [_q8_state(bn, x.device) for _, bn in chain]
        fp8io = (getattr(x, "_pdt_fp8", None), q8s, [])
    out = _ResidualBlock.apply(x, (tuple(spec_chain), ds_spec, tail), getattr(x, "_pdt_handoff", None),
                               fp8io, *tensors)
    node = out.grad_fn  # the ctx of this block's node (None without autograd)
    if node is not None and getattr(node, "handoff_out", None) is not None:
        out._pdt_handoff = node.handoff_out
    if fp8io is not None and fp8io[2]:
        out._pdt_fp8 = fp8io[2][0]
    return out
