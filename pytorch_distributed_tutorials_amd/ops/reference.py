"""PyTorch reference implementations of every native op (NHWC layout).

Used (a) as the CPU execution path, so the whole framework -- models, DDP,
trainer -- runs and is tested on CPU/gloo without a GPU, and (b) as the fp32
numerics oracle the HIP kernels are checked against in ``tests/test_kernels_gpu.py``.

Layout conventions shared with the kernels (``csrc/kernels/*.hip``):
  activations  [N, H, W, C]  contiguous (NHWC), stem input padded to C=8
  conv weight  [K, C, R, S]  logical OIHW, channels_last memory (= KRSC)
  BN stats     per-channel fp32
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

STEM_CPAD = 8  # channel granule of the kernels' 16-byte loads (8 x bf16)


def image_to_nhwc(x: torch.Tensor, dtype: torch.dtype, cpad: int = STEM_CPAD) -> torch.Tensor:
    n, c, h, w = x.shape
    out = torch.zeros((n, h, w, cpad), dtype=dtype, device=x.device)
    out[..., :c] = x.permute(0, 2, 3, 1).to(dtype)
    return out


def conv2d_nhwc(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> torch.Tensor:
    """x [N,H,W,Cx] (Cx >= w.C; extra channels are zero padding), w [K,C,R,S]."""
    c = w.shape[1]
    xin = x[..., :c].permute(0, 3, 1, 2).float()
    y = F.conv2d(xin, w.float(), stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1)


def conv2d_nhwc_dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape, stride: int, pad: int) -> torch.Tensor:
    n, h, wd, cx = x_shape
    c = w.shape[1]
    g = torch.nn.grad.conv2d_input((n, c, h, wd), w.float(), dy.permute(0, 3, 1, 2).float(),
                                   stride=stride, padding=pad)
    g = g.permute(0, 2, 3, 1)
    if cx != c:
        g = F.pad(g, (0, cx - c))
    return g


def conv2d_nhwc_wgrad(dy: torch.Tensor, x: torch.Tensor, w_shape, stride: int, pad: int) -> torch.Tensor:
    k, c, r, s = w_shape
    xin = x[..., :c].permute(0, 3, 1, 2).float()
    return torch.nn.grad.conv2d_weight(xin, (k, c, r, s), dy.permute(0, 3, 1, 2).float(),
                                       stride=stride, padding=pad)


def bn_batch_stats(y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-channel mean and biased variance over N,H,W (fp32)."""
    yf = y.float().reshape(-1, y.shape[-1])
    mean = yf.mean(0)
    var = yf.var(0, unbiased=False)
    return mean, var


def bn_act_fwd(y: torch.Tensor, mean: torch.Tensor, invstd: torch.Tensor, gamma: torch.Tensor,
               beta: torch.Tensor, residual: Optional[torch.Tensor], relu: bool,
               out_dtype: torch.dtype) -> torch.Tensor:
    z = (y.float() - mean) * (invstd * gamma.float()) + beta.float()
    if residual is not None:
        z = z + residual.float()
    if relu:
        z = torch.relu(z)
    return z.to(out_dtype)


def bn_act_bwd(dz: torch.Tensor, z: torch.Tensor, y: torch.Tensor, mean: torch.Tensor,
               invstd: torch.Tensor, gamma: torch.Tensor, relu: bool, training: bool,
               want_dres: bool, out_dtype: torch.dtype):
    """Returns dy, dgamma, dbeta, dres (dres = dz*mask, the residual-branch grad)."""
    g = dz.float()
    if relu:
        g = g * (z.float() > 0)
    c = g.shape[-1]
    g2 = g.reshape(-1, c)
    xhat = ((y.float() - mean) * invstd).reshape(-1, c)
    dbeta = g2.sum(0)
    dgamma = (g2 * xhat).sum(0)
    m = g2.shape[0]
    scale = gamma.float() * invstd
    if training:
        dy = scale * (g2 - dbeta / m - xhat * (dgamma / m))
    else:
        dy = scale * g2
    dy = dy.reshape(g.shape).to(out_dtype)
    dres = g.to(out_dtype) if want_dres else None
    return dy, dgamma, dbeta, dres


def maxpool3x3s2_fwd(x: torch.Tensor) -> torch.Tensor:
    y = F.max_pool2d(x.permute(0, 3, 1, 2).float(), 3, 2, 1)
    return y.permute(0, 2, 3, 1).to(x.dtype).contiguous()


def maxpool3x3s2_bwd(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    xn = x.permute(0, 3, 1, 2).float().detach().requires_grad_(True)
    with torch.enable_grad():
        y = F.max_pool2d(xn, 3, 2, 1)
        (g,) = torch.autograd.grad(y, xn, dy.permute(0, 3, 1, 2).float())
    return g.permute(0, 2, 3, 1).to(x.dtype).contiguous()


def global_avgpool(x: torch.Tensor) -> torch.Tensor:
    return x.float().mean(dim=(1, 2))


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Mean-reduced cross entropy and its gradient w.r.t. logits."""
    lf = logits.float()
    loss = F.cross_entropy(lf, labels)
    p = torch.softmax(lf, dim=1)
    p[torch.arange(lf.shape[0]), labels] -= 1.0
    return loss, p / lf.shape[0]


def top1_correct(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    return (logits.argmax(1) == labels).sum()


def sgd_momentum_(params, grads, bufs, lr: float, momentum: float, dampening: float,
                  weight_decay: float, nesterov: bool, first_step: bool, grad_scale: float = 1.0):
    """torch.optim.SGD semantics (torch/optim/sgd.py:343-380) on lists of tensors."""
    for p, g, b in zip(params, grads, bufs):
        d = g if grad_scale == 1.0 else g * grad_scale
        if weight_decay != 0:
            d = d.add(p, alpha=weight_decay)
        if momentum != 0:
            if first_step:
                b.copy_(d)
            else:
                b.mul_(momentum).add_(d, alpha=1 - dampening)
            d = d.add(b, alpha=momentum) if nesterov else b
        p.add_(d, alpha=-lr)
