"""roadrestore -- MI355X (gfx950) native hot path of the road-sign
restoration-then-recognition pipeline.

Drop-in for the reference's networks (SimpleUNet, ResidualBlock, ResUNet,
VGGPerceptualLoss, VGG16 judge), their training step and batched inference.
Compute runs in hand-written HIP kernels behind a C ABI (include/roadrestore.h,
libroadrestore.so in this directory); PyTorch supplies device memory, streams
and torch.distributed (RCCL) only.
"""
from . import imgproc, ops  # noqa: F401
from ._lib import EXPORTED, LIB_PATH, lib  # noqa: F401
from .nn import (AdaptiveAvgPool2d, BatchNorm2d, Conv2d, ConvTranspose2d, Dropout,  # noqa: F401
                 L1Loss, Linear, MaxPool2d, MSELoss, PReLU, ReLU, ResidualBlock, ResUNet,
                 SimpleUNet, VGG, VGGPerceptualLoss, default_compute_dtype, unified_loss, vgg16)
from .optim import Adam, AdamW, CosineAnnealingLR, RunningLoss  # noqa: F401

__version__ = "0.1.0"
