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

import operator
import os
import weakref
from typing import Dict, List, Optional, Sequence

import torch


def _is_dense(t: torch.Tensor) -> bool:
    if t.numel() == 0:
        return True
    span = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride()))
    return span == t.numel() and t.storage_offset() >= 0


_VERSION = operator.attrgetter("_version")
# the dgrad-layout pack after each optimizer step: on the caller's stream right behind the update
# (default), or on the weight-gradient stream beside the next forward (PDT_PACK_SIDE=1).  Same call,
# ResNet-50 b256, four runs each: 17.88 ms vs 17.91 (s25) -- the side-stream fork's marker and
# cross-queue waits at the step boundary cost more than the 25 us pack.
_PACK_SIDE = os.environ.get("PDT_PACK_SIDE", "0") == "1"
# mirrors with a side-stream pack whose event no stream has waited on yet
_PENDING_PACKS: "weakref.WeakSet" = weakref.WeakSet()


def forget_completed_side_packs() -> None:
    """Drop the pending side-stream pack events of every mirror.  Only valid right after a device
    synchronize (the packs are done): a graph capture calls it before it starts, because waiting on
    an event recorded by eager work from inside a capture is a HIP error
    (hipErrorStreamCaptureIsolation)."""
    for m in list(_PENDING_PACKS):
        m._crsk_event = None
    _PENDING_PACKS.clear()


class FlatParamSpace:
    def __init__(self, params: Sequence[torch.nn.Parameter], grad_flat: Optional[torch.Tensor] = None):
        """``grad_flat``: caller-provided storage for the flat gradient buffer (e.g. the IPC-shared
        buffer of the xGMI all-reduce backend); zeroed here."""
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
        if grad_flat is None:
            self.grad_flat = torch.zeros(off, device=dev, dtype=dt)
        else:
            if grad_flat.numel() != off or grad_flat.dtype != dt or grad_flat.device != dev \
                    or not grad_flat.is_contiguous():
                raise ValueError("grad_flat must be a contiguous tensor of the space's size, dtype and device")
            self.grad_flat = grad_flat
            with torch.no_grad():
                self.grad_flat.zero_()
        self.grad_views: List[torch.Tensor] = []
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.reducer = None  # set by DistributedDataParallel when gradients are all-reduced
        self.version = 0     # bumped by the fused optimizer step (raw writes bump no torch counter)
        self._mirror = None
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

    def mirror(self) -> "Optional[WeightMirror]":
        """bf16 conv-weight mirror (GPU spaces only), created on first use."""
        if self._mirror is None and self.param_flat.is_cuda:
            self._mirror = WeightMirror(self)
        return self._mirror

    def zero_grad(self) -> None:
        self.grad_flat.zero_()
        self.attach_grads()

    def slice(self, start: int, end: int, which: str = "grad") -> torch.Tensor:
        buf = self.grad_flat if which == "grad" else self.param_flat
        return buf.narrow(0, start, end - start)


class WeightMirror:
    """bf16 copies of a flat space's conv weights in the two layouts the conv kernels read.

    * ``krsc``: same offsets as the fp32 flat buffer; conv weights are channels_last, so the
      flat fp32 order already IS [K][R][S][C] and the fused SGD step writes this mirror as a
      side output (``sgd_step(..., p_bf16=)``): the forward convs need no pack launches;
    * ``crsk``: the dgrad layout [C][R][S][K], produced for ALL layers by ONE batched transpose
      launch after each optimizer step (instead of one pack kernel per layer per backward).
    Validity key = (space.version, param_flat._version, sum of the conv weights' versions): our
    optimizer bumps the first; a torch in-place write to a parameter (load_state_dict, user code)
    bumps that parameter's own counter.
    """

    def __init__(self, space: "FlatParamSpace"):
        import numpy as np
        from ..ops._ext import native
        self.space = space
        C = native()
        dev = space.param_flat.device
        self.krsc = torch.empty(space.numel, dtype=torch.bfloat16, device=dev)
        self.crsk = torch.empty(space.numel, dtype=torch.bfloat16, device=dev)
        self._krsc_views: Dict[int, torch.Tensor] = {}
        self._crsk_views: Dict[int, torch.Tensor] = {}
        self._tracked: List[torch.nn.Parameter] = []
        self._trusted = None  # the key ensure() last validated (see ensure)
        ent = []
        for p, o in zip(space.params, space.offsets):
            if p.dim() != 4:
                continue
            k, c, r, s_ = p.shape
            want = (r * s_ * c, 1, s_ * c, c)  # KRSC-dense; a size-1 dim may carry any stride
            krsc = all(n == 1 or st == wst for n, st, wst in zip(p.shape, p.stride(), want))
            if k % 8 or c % 8 or not krsc:
                continue  # e.g. the C=3 stem: packed per call with channel padding
            self._tracked.append(p)
            self._krsc_views[id(p)] = self.krsc.narrow(0, o, p.numel()).view(k, r, s_, c)
            self._crsk_views[id(p)] = self.crsk.narrow(0, o, p.numel()).view(c, r, s_, k)
            ent.append((o, k, c, r * s_, (k + 63) // 64, (c + 63) // 64, 0))
        dt = np.dtype([("off", "<i8"), ("K", "<i4"), ("C", "<i4"), ("RS", "<i4"), ("tk", "<i4"),
                       ("tc", "<i4"), ("pad", "<i4")])
        assert dt.itemsize == C.pack_t_entry_bytes(), "PackTEntry layout mismatch"
        arr = np.array(ent, dtype=dt)
        self.table = torch.from_numpy(arr.view(np.uint8).copy()).to(dev)
        self.ntensors = len(ent)
        self.max_tiles = max((e[3] * e[4] * e[5] for e in ent), default=0)
        self.key = None
        self._ent = ent
        self._fp8 = None  # e4m3 images of both layouts with per-row scales, built on first use
        self.key8 = None

    # ---------------------------------------------------------------- fp8 (e4m3) images
    def _build_fp8(self) -> None:
        import numpy as np
        from ..ops._ext import native
        C = native()
        dev = self.krsc.device
        dt = np.dtype([("off", "<i8"), ("soff", "<i8"), ("rows", "<i4"), ("rowlen", "<i4")])
        assert dt.itemsize == C.quant_rows_entry_bytes(), "QRowEntry layout mismatch"
        tk, tc = [], []
        ks = cs = 0
        self._kscale_at, self._cscale_at = {}, {}
        for p, (o, k, c, rs, _, _, _) in zip(self._tracked, self._ent):
            tk.append((o, ks, k, rs * c))
            tc.append((o, cs, c, rs * k))
            self._kscale_at[id(p)] = (ks, k)
            self._cscale_at[id(p)] = (cs, c)
            ks += k
            cs += c
        mk = lambda t: torch.from_numpy(np.array(t, dtype=dt).view(np.uint8).copy()).to(dev)  # noqa: E731
        self._fp8 = {
            "krsc8": torch.empty(self.space.numel, dtype=torch.uint8, device=dev),
            "crsk8": torch.empty(self.space.numel, dtype=torch.uint8, device=dev),
            "kscale": torch.empty(max(ks, 1), dtype=torch.float32, device=dev),
            "cscale": torch.empty(max(cs, 1), dtype=torch.float32, device=dev),
            "tk": mk(tk), "tc": mk(tc),
            "mk": max((e[2] for e in tk), default=0), "mc": max((e[2] for e in tc), default=0),
        }

    def ensure_fp8(self) -> bool:
        """Quantize both bf16 images to e4m3 (one launch each) if they changed since last time.
        Under graph capture the launches are always recorded: a replayed step cannot consult the
        host key, and the weights it sees were changed by the previous replay's optimizer step
        (an eager forward just before capture -- an evaluation -- would otherwise leave the
        first captured step without its quantization)."""
        if not self.valid() or not self._tracked:
            return False
        if self._fp8 is None:
            self._build_fp8()
        if self.key8 != self.key or torch.cuda.is_current_stream_capturing():
            from ..ops._ext import native
            C, f = native(), self._fp8
            self._join_pack()  # reads crsk
            C.quant_rows_e4m3(self.krsc, f["krsc8"], f["kscale"], f["tk"], f["mk"])
            C.quant_rows_e4m3(self.crsk, f["crsk8"], f["cscale"], f["tc"], f["mc"])
            self.key8 = self.key
        return True

    def krsc8_view(self, p):
        """(e4m3 [K,R,S,C], per-K scale [K]) of a tracked conv weight, or None."""
        if id(p) not in self._krsc_views or not self.ensure_fp8():
            return None
        k, c, r, s_ = p.shape
        o = self._krsc_views[id(p)].storage_offset() - self.krsc.storage_offset()
        a, n = self._kscale_at[id(p)]
        return (self._fp8["krsc8"].narrow(0, o, p.numel()).view(k, r, s_, c),
                self._fp8["kscale"].narrow(0, a, n))

    def crsk8_view(self, p):
        """(e4m3 [C,R,S,K], per-C scale [C]) of a tracked conv weight, or None."""
        if id(p) not in self._crsk_views or not self.ensure_fp8():
            return None
        k, c, r, s_ = p.shape
        o = self._crsk_views[id(p)].storage_offset() - self.crsk.storage_offset()
        a, n = self._cscale_at[id(p)]
        return (self._fp8["crsk8"].narrow(0, o, p.numel()).view(c, r, s_, k),
                self._fp8["cscale"].narrow(0, a, n))

    def current_key(self):
        # a Parameter re-homed with ``p.data = view`` keeps its own version counter (checked on
        # every conv's weight view: map/attrgetter keeps the per-call cost at ~1/2 of a generator)
        return (self.space.version, self.space.param_flat._version,
                sum(map(_VERSION, self._tracked)))

    def _pack_t(self, side: bool = False) -> None:
        from ..ops._ext import native
        if not self.ntensors:
            return
        self._join_pack()  # a previous side-stream pack must be done before krsc changes again
        s = None
        # (not under graph capture: the fork would stay unjoined at the end of the captured step)
        if side and self.krsc.is_cuda and not torch.cuda.is_current_stream_capturing():
            from ..ops import streams
            s = streams.wgrad_stream(self.krsc.device)
        if s is None:
            native().pack_t_batched(self.krsc, self.crsk, self.table, self.max_tiles)
            return
        # the dgrad layout is first read in backward: build it beside the forward (side stream),
        # and make the first consumer's stream wait for it (crsk_view)
        s.wait_stream(torch.cuda.current_stream(self.krsc.device))
        with torch.cuda.stream(s):
            native().pack_t_batched(self.krsc, self.crsk, self.table, self.max_tiles)
            ev = torch.cuda.Event()
            ev.record(s)
        self._crsk_event = ev
        _PENDING_PACKS.add(self)

    def _join_pack(self) -> None:
        ev = getattr(self, "_crsk_event", None)
        if ev is not None:
            torch.cuda.current_stream(self.krsc.device).wait_event(ev)
            self._crsk_event = None
            _PENDING_PACKS.discard(self)

    def refresh(self) -> None:
        from ..ops._ext import native
        native().cast_to_bf16(self.space.param_flat, self.krsc)
        self._pack_t()
        self.key = self.current_key()
        self._trusted = None

    def ensure(self) -> None:
        """Called once at the start of every native model forward: re-pack if stale, then trust the
        views for this step.  The full check sums the version counters of every tracked weight
        (~5 us with ResNet-152's 155 convs); doing it per conv view cost 1.7 ms of host issue per
        ResNet-152 step (r4q).  The trust ends with the optimizer step / the next refresh, so a
        write between steps is still caught; a write between a forward and its backward is not
        (autograd rejects that for saved tensors anyway)."""
        if self.key != self.current_key():
            self.refresh()
        self._trusted = self.key

    def end_trust(self) -> None:
        """The native backward's last node (the stem) ran: the trust ensure() granted ends here, so
        it lasts exactly one forward/backward.  An optimizer other than the fused SGD, or an
        in-place weight edit (load_state_dict, clipping) before the next forward, is then caught
        by the version-counter check of the next view taken outside the model's forward."""
        self._trusted = None

    def after_optimizer_step(self) -> None:
        """The fused SGD step just wrote ``krsc``; rebuild ``crsk`` and mark both current."""
        self.space.version += 1
        self._pack_t(side=_PACK_SIDE)
        self.key = self.current_key()
        self._trusted = None

    def valid(self) -> bool:
        if self.key is None:
            return False
        if self._trusted is self.key:
            return True
        return self.key == self.current_key()

    def krsc_view(self, p) -> Optional[torch.Tensor]:
        return self._krsc_views.get(id(p)) if self.valid() else None

    def crsk_view(self, p) -> Optional[torch.Tensor]:
        if not self.valid():
            return None
        self._join_pack()
        return self._crsk_views.get(id(p))


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
