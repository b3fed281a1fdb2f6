"""SGD with momentum and weight decay -- ``torch.optim.SGD`` semantics, fused.

Reference: ``optim.SGD(ddp_model.parameters(), lr, momentum=0.9,
weight_decay=1e-5)`` (``resnet/main.py:103``); per-step math of
torch/optim/sgd.py:343-380 (first step initialises the momentum buffer with the
gradient, then ``buf = m*buf + (1-dampening)*g``).

When a param group is exactly the set of parameters of a ``FlatParamSpace``
(what our DDP wrapper creates) and lives on the GPU, the whole update is ONE
HIP kernel over the flat param/grad/momentum buffers (``csrc/kernels/sgd.hip``).
The per-parameter ``state[p]['momentum_buffer']`` entries are views into the
flat momentum buffer, so ``state_dict()`` / ``load_state_dict()`` keep torch's
format.  Anything else falls back to a per-tensor reference implementation.
"""
from __future__ import annotations

import torch

from ..ops import reference as ref
from ..ops._ext import native


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening,
                        weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, defaults)
        self._flat_bufs = {}

    def _flat_space_of(self, group):
        ps = group["params"]
        if not ps:
            return None
        sp = getattr(ps[0], "_pdt_flat", None)
        if sp is None or len(ps) != len(sp.params):
            return None
        # the group covers exactly the space's parameters; the answer is cached per group for
        # this exact parameter list (two id sets per call cost ~25 us of host issue each time
        # zero_grad / step ran).  Kept off the group dict so state_dict() stays torch's.
        ids = [id(p) for p in ps]
        cache = self.__dict__.setdefault("_flat_hits", {})
        hit = cache.get(id(group))
        if hit is not None and hit[0] is sp and hit[1] == ids:
            return sp
        if set(ids) != {id(p) for p in sp.params}:
            return None
        cache[id(group)] = (sp, ids)
        return sp

    @torch.no_grad()
    def zero_grad(self, set_to_none: bool = True):
        for group in self.param_groups:
            sp = self._flat_space_of(group)
            if sp is not None:
                sp.zero_grad()   # one memset; .grad stay views of the flat buffer
            else:
                for p in group["params"]:
                    if p.grad is None:
                        continue
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, mom, damp = group["lr"], group["momentum"], group["dampening"]
            wd, nest = group["weight_decay"], group["nesterov"]
            sp = self._flat_space_of(group)
            if sp is not None and sp.param_flat.is_cuda:
                if not sp.grads_attached():
                    sp.gather_grads()
                key = id(sp)
                first = False
                if mom != 0 and key not in self._flat_bufs:
                    buf = torch.empty_like(sp.param_flat)
                    self._flat_bufs[key] = buf
                    for p, o in zip(sp.params, sp.offsets):
                        self.state[p]["momentum_buffer"] = torch.as_strided(buf, p.shape, p.stride(), o)
                    first = not self._restored_momentum(sp)
                buf = self._flat_bufs.get(key)
                mirror = sp.mirror()
                native().sgd_step(sp.param_flat, sp.grad_flat, buf, lr, mom, damp, wd, nest,
                                  first, 1.0, mirror.krsc if mirror is not None else None)
                if mirror is not None:
                    mirror.after_optimizer_step()  # bf16 conv weights for the next forward
                continue
            params, grads, bufs, firsts = [], [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                first = "momentum_buffer" not in st or st["momentum_buffer"] is None
                if first and mom != 0:
                    st["momentum_buffer"] = torch.empty_like(p, memory_format=torch.preserve_format)
                params.append(p)
                grads.append(p.grad)
                bufs.append(st.get("momentum_buffer"))
                firsts.append(first)
            for p, g, b, f in zip(params, grads, bufs, firsts):
                ref.sgd_momentum_(
                    [p], [g], [b], lr, mom, damp, wd, nest, f)
        return loss

    def _restored_momentum(self, sp) -> bool:
        """True if load_state_dict() populated momentum buffers before the first step."""
        pending = getattr(self, "_pending_momentum", None)
        if not pending:
            return False
        for p in sp.params:
            t = pending.get(id(p))
            if t is not None:
                self.state[p]["momentum_buffer"].copy_(t)
        self._pending_momentum = None
        return True

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        # momentum buffers loaded as standalone tensors: remember them so the flat
        # buffer is initialised from them instead of from the first gradient
        self._pending_momentum = {}
        for group in self.param_groups:
            for p in group["params"]:
                b = self.state.get(p, {}).get("momentum_buffer")
                if b is not None:
                    self._pending_momentum[id(p)] = b.detach().clone()
        for key, buf in list(self._flat_bufs.items()):
            # flat buffer already exists: copy loaded values into its views
            for group in self.param_groups:
                sp = self._flat_space_of(group)
                if sp is not None and id(sp) == key:
                    for p, o in zip(sp.params, sp.offsets):
                        v = torch.as_strided(buf, p.shape, p.stride(), o)
                        t = self._pending_momentum.get(id(p))
                        if t is not None:
                            v.copy_(t)
                        self.state[p]["momentum_buffer"] = v
            self._pending_momentum = None
