"""Checkpoint save / resume.

Reference (``resnet/main.py:83-85,109-112``): rank 0 ``torch.save(ddp_model.state_dict(),
model_dir/model_filename)``; resume with ``torch.load(path, map_location={"cuda:0":
"cuda:r"})`` + strict ``ddp_model.load_state_dict``.  The file written here is
byte-compatible in schema: zip pickle, ``module.``-prefixed
torchvision keys, OIHW contiguous fp32 conv weights (our channels_last / flat
storage is converted on the way out), int64 ``num_batches_tracked``.

Reference defect D10 (resume restores weights only) is fixed without touching
that schema: optimizer state and the next epoch go to a SEPARATE sidecar file
``<checkpoint>.train_state.pt``.
"""
from __future__ import annotations

import os
from typing import Optional

import torch


def portable_state_dict(module: torch.nn.Module) -> dict:
    """state_dict with every tensor detached, contiguous (OIHW) and on the CPU."""
    out = {}
    for k, v in module.state_dict().items():
        out[k] = v.detach().contiguous().cpu() if isinstance(v, torch.Tensor) else v
    return out


def sidecar_path(path: str) -> str:
    return path + ".train_state.pt"


def save_checkpoint(module: torch.nn.Module, path: str, optimizer: Optional[torch.optim.Optimizer] = None,
                    epoch: Optional[int] = None) -> None:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(portable_state_dict(module), tmp)
    os.replace(tmp, path)
    if optimizer is not None or epoch is not None:
        side = {"epoch": epoch}
        if optimizer is not None:
            side["optimizer"] = optimizer.state_dict()
        torch.save(side, sidecar_path(path) + ".tmp")
        os.replace(sidecar_path(path) + ".tmp", sidecar_path(path))


def load_checkpoint(module: torch.nn.Module, path: str, device: torch.device,
                    optimizer: Optional[torch.optim.Optimizer] = None, strict: bool = True) -> Optional[int]:
    """Load weights (strict); returns the epoch to resume from if the sidecar exists."""
    sd = torch.load(path, map_location=device, weights_only=True)
    module.load_state_dict(sd, strict=strict)
    side = sidecar_path(path)
    if os.path.exists(side):
        st = torch.load(side, map_location=device, weights_only=True)
        if optimizer is not None and st.get("optimizer") is not None:
            optimizer.load_state_dict(st["optimizer"])
        return st.get("epoch")
    return None
