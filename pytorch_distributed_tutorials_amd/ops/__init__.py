"""Ops layer: fused ResNet ops backed by hand-written HIP kernels.

See ``fused.py`` for the autograd units and ``reference.py`` for the PyTorch
semantics they implement.  ``native_available()`` reports whether the gfx950
extension loaded.
"""
from ._ext import native, native_available  # noqa: F401
from .fused import (  # noqa: F401
    CrossEntropyLoss,
    act_dtype,
    avgpool_linear,
    buffers_ready,
    bump_bn_counters,
    forget_bn_modules,
    defer_buffer_wait,
    conv_bn,
    cross_entropy,
    fp8_attach,
    fp8_enabled,
    image_to_nhwc,
    maxpool3x3s2,
    residual_block,
    set_fp8,
    set_cpu_activation_dtype,
    stem_conv_bn,
    stem_conv_bn_pool,
    top1_correct,
)
