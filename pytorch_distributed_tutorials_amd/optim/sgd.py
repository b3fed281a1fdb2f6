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

Optimizer in backward (``overlap``, default: wherever it applies).  When the flat space belongs to
our ``DistributedDataParallel`` on a GPU, the update is launched per gradient bucket INSIDE
backward, right behind that bucket's all-reduce (or, in one process, as soon as the bucket's
gradients are final), so only the last bucket's update follows backward; ``step()`` then only
joins.  The math is the same kernel over the same elements, so parameters are bitwise equal to the
post-backward step (``tests/test_opt_overlap_gpu.py``).  Contract, checked loudly: every synced
backward is followed by ``step()`` before the next forward, and neither the gradients nor the
hyperparameters change in between (gradient clipping, an LR change between backward and step):
``SGD(..., overlap=False)`` keeps the classic post-backward step for such loops.  ``no_sync()``
backwards are not updated (their gradients accumulate as usual).
"""
from __future__ import annotations

import os

import torch

from ..ops import reference as ref
from ..ops._ext import native


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, overlap=None):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening,
                        weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, defaults)
        self._flat_bufs = {}
        self._flat_first = {}   # flat space id -> the next update initialises the momentum buffer
        self._armed = None      # hyperparameters the reducer's per-bucket update was armed with
        self._overlap_owner = None
        if overlap is None and os.environ.get("PDT_OPT_OVERLAP", "1") == "0":
            overlap = False
        if overlap is not False:
            self._attach_overlap()

    # ------------------------------------------------------------ optimizer in backward
    def _attach_overlap(self) -> None:
        if len(self.param_groups) != 1:
            return
        sp = self._flat_space_of(self.param_groups[0])
        owner = getattr(sp, "owner", None) if sp is not None else None
        ddp = owner() if owner is not None else None
        if ddp is not None and sp.param_flat.is_cuda and ddp.attach_optimizer(self):
            self._overlap_owner = owner

    def _flat_momentum(self, sp, mom):
        """(flat momentum buffer or None, is this the buffer's first update?)"""
        key = id(sp)
        if mom != 0 and key not in self._flat_bufs:
            buf = torch.empty_like(sp.param_flat)
            self._flat_bufs[key] = buf
            for p, o in zip(sp.params, sp.offsets):
                self.state[p]["momentum_buffer"] = torch.as_strided(buf, p.shape, p.stride(), o)
            self._flat_first[key] = not self._restored_momentum(sp)
        return self._flat_bufs.get(key), self._flat_first.get(key, False)

    def _hyper(self, group):
        return (group["lr"], group["momentum"], group["dampening"], group["weight_decay"], group["nesterov"])

    def _arm_overlap(self, reducer) -> None:
        """Called by the DDP wrapper's forward before a synced backward: arm the per-bucket update."""
        if self._armed is not None and reducer.optimizer_applied()[0] >= 0:
            raise RuntimeError(
                "optimizer overlap: a backward already applied this optimizer's update per bucket, but "
                "step() was not called before the next forward.  Call optimizer.step() after every "
                "synced backward, or construct the optimizer with overlap=False")
        self._armed = None
        if torch.cuda.is_current_stream_capturing():
            return  # a captured step keeps the post-backward update (utils/graph.py)
        group = self.param_groups[0]
        sp = self._flat_space_of(group)
        if sp is None:
            return
        hp = self._hyper(group)
        lr, mom, damp, wd, nest = hp
        buf, first = self._flat_momentum(sp, mom)
        mirror = sp.mirror()
        reducer.arm_optimizer(lr, mom, damp, wd, nest, first, buf, mirror.krsc if mirror is not None else None)
        self._armed = hp

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
                mirror = sp.mirror()
                if self._armed is not None and self._overlap_step(sp, group):
                    # every bucket was updated inside backward (and the caller's stream joined it)
                    self._flat_first[id(sp)] = False
                    if mirror is not None:
                        mirror.after_optimizer_step()
                    continue
                if not sp.grads_attached():
                    sp.gather_grads()
                buf, first = self._flat_momentum(sp, mom)
                native().sgd_step(sp.param_flat, sp.grad_flat, buf, lr, mom, damp, wd, nest,
                                  first, 1.0, mirror.krsc if mirror is not None else None)
                self._flat_first[id(sp)] = False
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

    def _overlap_step(self, sp, group) -> bool:
        """True if the last backward applied this step per bucket; validates the contract."""
        owner = self._overlap_owner() if self._overlap_owner is not None else None
        armed, self._armed = self._armed, None
        if owner is None or owner.reducer is None:
            return False
        applied, gver = owner.reducer.optimizer_applied()
        if applied < 0:
            return False  # armed, but no synced backward ran (e.g. a forward without backward)
        owner.reducer.consume_optimizer()
        if applied != owner.reducer.num_buckets:
            raise RuntimeError(f"optimizer overlap: {applied} of {owner.reducer.num_buckets} buckets updated")
        if self._hyper(group) != armed:
            raise RuntimeError("optimizer overlap: hyperparameters changed between backward and step() "
                               "(the update already ran in backward); use SGD(..., overlap=False)")
        if sp.grad_flat._version != gver or not sp.grads_attached():
            raise RuntimeError("optimizer overlap: gradients were modified between backward and step() "
                               "(the update already ran in backward); use SGD(..., overlap=False)")
        return True

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
