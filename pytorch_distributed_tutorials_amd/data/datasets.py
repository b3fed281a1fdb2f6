"""Datasets: synthetic (ImageNet / CIFAR shaped) and CIFAR-10 from disk.

The reference reads CIFAR-10 through torchvision with ``download=False``
(``resnet/main.py:94-95``) and augments on 8 CPU worker processes with PIL
(``resnet/main.py:87-92``).  Here a dataset is a pair of tensors
(uint8/float images, int64 labels) that can live on the GPU; augmentation runs
batched on the device (``loader.py``), which removes the CPU worker bottleneck
(SURVEY.md §3.2 hot spots).  Benchmarks use synthetic data of the same shape
(BASELINE.json configs) because there is no network to fetch datasets.
"""
from __future__ import annotations

import os
import pickle
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)   # resnet/main.py:91
CIFAR_STD = (0.2023, 0.1994, 0.2010)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


@dataclass
class TensorImageDataset:
    """Images [N, 3, H, W] (uint8 0..255 or float, already normalized) + labels [N]."""
    images: torch.Tensor
    labels: torch.Tensor
    mean: Tuple[float, float, float] = CIFAR_MEAN
    std: Tuple[float, float, float] = CIFAR_STD
    normalized: bool = False

    def __len__(self) -> int:
        return int(self.labels.shape[0])

    def to(self, device) -> "TensorImageDataset":
        return TensorImageDataset(self.images.to(device), self.labels.to(device),
                                  self.mean, self.std, self.normalized)


def synthetic_dataset(num_samples: int, image_size: int, num_classes: int,
                      device="cpu", seed: int = 0) -> TensorImageDataset:
    """Random normalized float images (``data: synthetic``) of the given shape."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    imgs = torch.randn((num_samples, 3, image_size, image_size), generator=g)
    labels = torch.randint(0, num_classes, (num_samples,), generator=g)
    return TensorImageDataset(imgs.to(device), labels.to(device), normalized=True)


def learnable_dataset(num_samples: int, image_size: int, num_classes: int, device="cpu", seed: int = 0,
                      noise: float = 1.0, template_seed: int = 12345) -> TensorImageDataset:
    """A synthetic set a network can actually learn (convergence checks without CIFAR on disk):
    class c's images are a fixed random template t_c (shared by train and test splits through
    ``template_seed``) plus i.i.d. Gaussian noise of std ``noise``; normalized float images."""
    gt = torch.Generator(device="cpu")
    gt.manual_seed(template_seed)
    templates = torch.randn((num_classes, 3, image_size, image_size), generator=gt)
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    labels = torch.randint(0, num_classes, (num_samples,), generator=g)
    imgs = templates[labels] + noise * torch.randn((num_samples, 3, image_size, image_size), generator=g)
    return TensorImageDataset(imgs.to(device), labels.to(device), normalized=True)


class _NumpyOnlyUnpickler(pickle.Unpickler):
    """CIFAR-10 python batches are pickled dicts of numpy arrays; refuse anything else."""
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"),
        ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
        ("_codecs", "encode"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a CIFAR batch")


def _read_cifar_py(path: str):
    with open(path, "rb") as f:
        d = _NumpyOnlyUnpickler(f, encoding="latin1").load()
    data = np.asarray(d["data"], dtype=np.uint8).reshape(-1, 3, 32, 32)
    labels = np.asarray(d.get("labels", d.get("fine_labels")), dtype=np.int64)
    return data, labels


def _read_cifar_bin(path: str):
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 1 + 3 * 32 * 32)
    return raw[:, 1:].reshape(-1, 3, 32, 32), raw[:, 0].astype(np.int64)


def cifar10(root: str = "data", train: bool = True) -> TensorImageDataset:
    """Load CIFAR-10 from ``root`` (python or binary distribution; no download)."""
    py_dir = os.path.join(root, "cifar-10-batches-py")
    bin_dir = os.path.join(root, "cifar-10-batches-bin")
    if os.path.isdir(py_dir):
        files = [f"data_batch_{i}" for i in range(1, 6)] if train else ["test_batch"]
        parts = [_read_cifar_py(os.path.join(py_dir, f)) for f in files]
    elif os.path.isdir(bin_dir):
        files = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
        parts = [_read_cifar_bin(os.path.join(bin_dir, f)) for f in files]
    else:
        raise FileNotFoundError(
            f"CIFAR-10 not found under {root!r} (expected cifar-10-batches-py or "
            "cifar-10-batches-bin; download=False like resnet/main.py:94). "
            "Use --data synthetic for a synthetic dataset of the same shape.")
    data = np.concatenate([p[0] for p in parts])
    labels = np.concatenate([p[1] for p in parts])
    return TensorImageDataset(torch.from_numpy(data), torch.from_numpy(labels))


def build_dataset(kind: str, train: bool, root: str = "data", num_samples: Optional[int] = None,
                  image_size: Optional[int] = None, num_classes: int = 10,
                  seed: int = 0) -> TensorImageDataset:
    """kind: 'cifar10' (disk), 'synthetic-cifar' (32px), 'synthetic-imagenet' (224px), or
    'learnable-cifar' (32px class templates + noise: a set the model can fit)."""
    if kind == "cifar10":
        return cifar10(root, train)
    if kind == "synthetic-cifar":
        n = num_samples or (50000 if train else 10000)
        return synthetic_dataset(n, image_size or 32, num_classes, seed=seed + (0 if train else 1))
    if kind == "synthetic-imagenet":
        n = num_samples or (2048 if train else 512)
        return synthetic_dataset(n, image_size or 224, num_classes, seed=seed + (0 if train else 1))
    if kind == "learnable-cifar":
        n = num_samples or (10000 if train else 2000)
        return learnable_dataset(n, image_size or 32, num_classes, seed=seed + (0 if train else 1))
    raise ValueError(f"unknown dataset kind {kind!r}")
