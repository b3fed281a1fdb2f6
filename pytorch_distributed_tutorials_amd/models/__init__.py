from .resnet import (  # noqa: F401
    MODEL_SPECS,
    BasicBlock,
    Bottleneck,
    ResNet,
    build_model,
    resnet18,
    resnet34,
    resnet50,
    resnet101,
    resnet152,
)
