"""Device-side batch loader with the reference's CIFAR augmentation.

Replaces ``DataLoader(dataset, batch_size, sampler, num_workers=8)``
(``resnet/main.py:98,100``) + the PIL transform chain
``RandomCrop(32, padding=4) -> RandomHorizontalFlip -> ToTensor -> Normalize``
(``resnet/main.py:87-92``) with batched GPU ops on a device-resident dataset:
gather the sampler's indices, zero-pad by 4, random-crop via two ``gather``s,
random flip, normalize.  Padding happens before normalization exactly like
torchvision (pad pixels are black, i.e. ``-mean/std`` after normalization).
Evaluation uses no augmentation (reference defect D7 fixed).

On the GPU the whole chain (gather by index, /255, pad+crop, flip, normalize) is ONE fused HIP
kernel (``csrc/kernels/augment.hip``) fed with crop offsets and flips drawn exactly as the torch
path draws them, so both paths produce identical batches (tests/test_kernels_gpu.py).
"""
from __future__ import annotations

import math
from typing import Iterator, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .datasets import TensorImageDataset


def _normalize(x: torch.Tensor, mean, std) -> torch.Tensor:
    m = torch.tensor(mean, device=x.device, dtype=x.dtype).view(1, -1, 1, 1)
    s = torch.tensor(std, device=x.device, dtype=x.dtype).view(1, -1, 1, 1)
    return (x - m) / s


def draw_crop_flip(b: int, pad: int, device, gen: Optional[torch.Generator]):
    """Per-sample RandomCrop offsets (0..2*pad) and RandomHorizontalFlip(p=0.5) decisions."""
    oy = torch.randint(0, 2 * pad + 1, (b,), device=device, generator=gen)
    ox = torch.randint(0, 2 * pad + 1, (b,), device=device, generator=gen)
    flip = torch.rand((b,), device=device, generator=gen) < 0.5
    return oy, ox, flip


def random_crop_flip(x: torch.Tensor, pad: int, gen: Optional[torch.Generator]) -> torch.Tensor:
    """Batched RandomCrop(size=H, padding=pad) + RandomHorizontalFlip(p=0.5)."""
    b, c, h, w = x.shape
    xp = F.pad(x, (pad, pad, pad, pad))
    oy, ox, flip = draw_crop_flip(b, pad, x.device, gen)
    ar_h = torch.arange(h, device=x.device)
    ar_w = torch.arange(w, device=x.device)
    iy = (oy[:, None] + ar_h)[:, None, :, None].expand(b, c, h, w + 2 * pad)
    xr = xp.gather(2, iy)
    cols = torch.where(flip[:, None], ox[:, None] + (w - 1 - ar_w), ox[:, None] + ar_w)
    return xr.gather(3, cols[:, None, None, :].expand(b, c, h, w))


class DeviceLoader:
    """Iterates ``(images[B,3,H,W] float32, labels[B] int64)`` batches on ``device``."""

    def __init__(self, dataset: TensorImageDataset, batch_size: int, sampler=None,
                 shuffle: bool = False, augment: bool = False, device="cpu",
                 drop_last: bool = False, seed: int = 0, fused: Optional[bool] = None):
        self.ds = dataset.to(device)
        self.batch_size = batch_size
        self.sampler = sampler
        self.shuffle = shuffle
        self.augment = augment
        self.device = torch.device(device)
        self.drop_last = drop_last
        self.seed = seed
        self.epoch = 0
        # fused HIP augmentation on GPU datasets (None = when the native extension is available)
        if fused is None:
            from ..ops._ext import native_available
            fused = self.device.type == "cuda" and native_available()
        self.fused = bool(fused) and self.device.type == "cuda" and self.ds.images.shape[3] % 4 == 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def _indices(self) -> Sequence[int]:
        if self.sampler is not None:
            return list(iter(self.sampler))
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            return torch.randperm(len(self.ds), generator=g).tolist()
        return list(range(len(self.ds)))

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else len(self.ds)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        idx = torch.tensor(self._indices(), dtype=torch.long)
        gen = None
        if self.augment:
            gen = torch.Generator(device=self.device)
            gen.manual_seed(self.seed * 1000003 + self.epoch)
        idx = idx.to(self.device)
        n = idx.numel()
        stop = (n // self.batch_size) * self.batch_size if self.drop_last else n
        for s in range(0, stop, self.batch_size):
            bi = idx[s:s + self.batch_size]
            y = self.ds.labels.index_select(0, bi)
            if self.fused:
                yield self._fused_batch(bi, gen), y
                continue
            x = self.ds.images.index_select(0, bi)
            if not self.ds.normalized:
                x = x.float().div_(255.0)
                if self.augment:
                    x = random_crop_flip(x, 4, gen)
                x = _normalize(x, self.ds.mean, self.ds.std)
            elif self.augment:
                x = random_crop_flip(x, 4, gen)
            yield x.float().contiguous(), y

    def _fused_batch(self, bi: torch.Tensor, gen) -> torch.Tensor:
        from ..ops._ext import native
        b = bi.numel()
        if self.augment:
            oy, ox, flip = draw_crop_flip(b, 4, self.device, gen)
            pad = 4
        else:
            oy = ox = torch.zeros(b, dtype=torch.long, device=self.device)
            flip, pad = None, 0
        imgs = self.ds.images
        if imgs.dtype not in (torch.uint8, torch.float32):
            imgs = imgs.float()
        return native().augment(imgs.contiguous(), bi.contiguous(), oy, ox, flip, pad,
                                not self.ds.normalized, list(self.ds.mean), list(self.ds.std))
