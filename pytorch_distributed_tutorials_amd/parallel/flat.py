"""Flat parameter / gradient storage.

All trainable parameters are re-homed into ONE contiguous fp32 buffer (and
their ``.grad`` into one contiguous gradient buffer with the same layout) in
bucket order.  Consequences:
  * a gradient bucket is a contiguous slice -> one RCCL call, no packing copies;
  * the optimizer update is a single fused kernel over the whole buffer
    (``optim.SGD`` detects the flat space), instead of ~4 multi-tensor kernels
    over 161 tensors;
  * parameters keep their identity, shape and strides (channels_last conv
    weights stay channels_last), so ``state_dict`` and user code are unchanged.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch


def _is_dense(t: torch.Tensor) -> bool:
    if t.numel() == 0:
        return True
    span = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride()))
    return span == t.numel() and t.storage_offset() >= 0


class FlatParamSpace:
    def __init__(self, params: Sequence[torch.nn.Parameter]):
        if not params:
            raise ValueError("FlatParamSpace needs at least one parameter")
        dev, dt = params[0].device, params[0].dtype
        for p in params:
            if p.device != dev or p.dtype != dt:
                raise ValueError("all parameters of a flat space must share device and dtype")
            if not _is_dense(p.data):
                raise ValueError("parameters must be dense (contiguous in some dim order)")
        self.params: List[torch.nn.Parameter] = list(params)
        self.offsets: List[int] = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += p.numel()
        self.numel = off
        self.device, self.dtype = dev, dt
        self.param_flat = torch.empty(off, device=dev, dtype=dt)
        self.grad_flat = torch.zeros(off, device=dev, dtype=dt)
        self.grad_views: List[torch.Tensor] = []
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.reducer = None  # set by DistributedDataParallel when gradients are all-reduced
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                view = torch.as_strided(self.param_flat, p.shape, p.stride(), o)
                view.copy_(p.data)
                p.data = view
                self.grad_views.append(torch.as_strided(self.grad_flat, p.shape, p.stride(), o))
                p._pdt_flat = self  # noqa: SLF001  (marker read by optim.SGD)
        self.attach_grads()

    def attach_grads(self) -> None:
        """(Re)point every ``p.grad`` at its view of the flat gradient buffer."""
        for p, g in zip(self.params, self.grad_views):
            p.grad = g

    def grads_attached(self) -> bool:
        return all(p.grad is g for p, g in zip(self.params, self.grad_views))

    def gather_grads(self) -> None:
        """Copy any gradient that autograd stored outside the flat buffer into it."""
        with torch.no_grad():
            for p, g in zip(self.params, self.grad_views):
                if p.grad is None:
                    g.zero_()
                elif p.grad is not g:
                    if p.grad.data_ptr() != g.data_ptr():
                        g.copy_(p.grad)
                p.grad = g

    def grad_sink(self, p: torch.nn.Parameter) -> torch.Tensor:
        """The flat view ``p.grad`` must live in, ready for a kernel to ACCUMULATE into
        (autograd semantics).  Used by fused native backward passes that write parameter
        gradients in place instead of returning them to autograd."""
        g = self.grad_views[self.index[id(p)]]
        if p.grad is not g:
            with torch.no_grad():
                if p.grad is None:
                    g.zero_()
                elif p.grad.data_ptr() != g.data_ptr():
                    g.copy_(p.grad)
            p.grad = g
        return g

    def mark_ready(self, params) -> None:
        """Tell the reducer that these parameters' gradients are final in their views."""
        if self.reducer is not None:
            self.reducer.mark_ready_external([self.index[id(p)] for p in params])

    def zero_grad(self) -> None:
        self.grad_flat.zero_()
        self.attach_grads()

    def slice(self, start: int, end: int, which: str = "grad") -> torch.Tensor:
        buf = self.grad_flat if which == "grad" else self.param_flat
        return buf.narrow(0, start, end - start)


def flatten_buffers(module: torch.nn.Module) -> Dict[torch.dtype, torch.Tensor]:
    """Re-home module buffers into one flat tensor per dtype (for one-call broadcasts)."""
    by_dtype: Dict[torch.dtype, List] = {}
    for mod in module.modules():
        for name, b in mod.named_buffers(recurse=False):
            if b is None:
                continue
            by_dtype.setdefault(b.dtype, []).append((mod, name, b))
    flats: Dict[torch.dtype, torch.Tensor] = {}
    for dt, items in by_dtype.items():
        total = sum(b.numel() for _, _, b in items)
        flat = torch.empty(total, dtype=dt, device=items[0][2].device)
        off = 0
        with torch.no_grad():
            for mod, name, b in items:
                view = flat.narrow(0, off, b.numel()).view(b.shape)
                view.copy_(b)
                mod._buffers[name] = view
                off += b.numel()
        flats[dt] = flat
    return flats
