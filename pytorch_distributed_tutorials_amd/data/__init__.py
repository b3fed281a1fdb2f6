from .datasets import (  # noqa: F401
    CIFAR_MEAN,
    CIFAR_STD,
    TensorImageDataset,
    build_dataset,
    cifar10,
    learnable_dataset,
    synthetic_dataset,
)
from .loader import DeviceLoader, draw_crop_flip, random_crop_flip  # noqa: F401
from .sampler import DistributedSampler  # noqa: F401
