"""CPU restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` may import it, and only as the
checker / the timed CPU baseline.  The product (``roadrestore``) never imports
it and never falls back to it.

It restates, in plain functional PyTorch-CPU fp32 over a ``state_dict``, the
networks and losses of the reference scripts (paths relative to the reference
repo):

* ``SimpleUNet``            07_train_restoration.py:75-120
* ``ResidualBlock``         14_train_unified_advanced.py:96-115
* ``ResUNet``               14_train_unified_advanced.py:117-186
* ``VGGPerceptualLoss``     14_train_unified_advanced.py:189-196 (07adv:95-112)
* VGG16 classifier          torchvision ``vgg16`` cfg "D" with the 43-class head
                            swap of 05_train_baseline.py:53-54 / 18:58-61
* train-step losses         14:238-242 (L1 + 0.1*perc), 07:142 (MSE)
* AdamW / Adam              14:222 (lr 2e-4, wd 1e-4), 07:143 (lr 1e-3)
* post-processing + PSNR    17:84-99 / 08:96-125 (clamp, x255, uint8 truncation,
                            skimage ``peak_signal_noise_ratio`` formula)
* Top-1                     18:43-49 (``torch.max(outputs, 1)``)

It dispatches the same ATen CPU kernels the reference does, so on CPU it is
bit-identical to the reference classes (checked by ``oracle/gen_golden.py``
against the imported reference and pinned by ``tests/golden``).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as tnn
import torch.nn.functional as F

BN_EPS = 1e-5        # nn.BatchNorm2d default (14:103, 14:106, 14:112)
BN_MOMENTUM = 0.1    # nn.BatchNorm2d default

# --------------------------------------------------------------------------
# primitive helpers
# --------------------------------------------------------------------------


def _conv(p, name, x, padding):
    return F.conv2d(x, p[name + ".weight"], p[name + ".bias"], padding=padding)


def _bn(p, name, x, training):
    """nn.BatchNorm2d semantics: batch stats (biased var) in train mode, running
    stats updated in place with the unbiased var, momentum 0.1, eps 1e-5."""
    rm, rv = p[name + ".running_mean"], p[name + ".running_var"]
    y = F.batch_norm(x, rm, rv, p[name + ".weight"], p[name + ".bias"],
                     training, BN_MOMENTUM, BN_EPS)
    if training and (name + ".num_batches_tracked") in p:
        p[name + ".num_batches_tracked"].add_(1)
    return y


def _prelu(p, name, x):
    return F.prelu(x, p[name + ".weight"])


def _maxpool(x):
    return F.max_pool2d(x, 2, 2)   # nn.MaxPool2d(2, 2), floor mode


def _convT(p, name, x):
    return F.conv_transpose2d(x, p[name + ".weight"], p[name + ".bias"], stride=2)


# --------------------------------------------------------------------------
# SimpleUNet  (07_train_restoration.py:75-120)
# --------------------------------------------------------------------------

def _double_conv_relu(p, prefix, x):
    # nn.Sequential(Conv3x3 p1, ReLU, Conv3x3 p1, ReLU): indices 0 and 2 carry params
    x = F.relu(_conv(p, prefix + ".0", x, 1))
    return F.relu(_conv(p, prefix + ".2", x, 1))


def simple_unet_forward(p, x):
    e1 = _double_conv_relu(p, "enc1", x)                  # 07:101
    e2 = _double_conv_relu(p, "enc2", _maxpool(e1))       # 07:102-105
    b = _double_conv_relu(p, "bottleneck", _maxpool(e2))  # 07:108
    d2 = torch.cat((_convT(p, "up2", b), e2), dim=1)      # 07:111-112 (up first, skip second)
    d2 = _double_conv_relu(p, "dec2", d2)                 # 07:113
    d1 = torch.cat((_convT(p, "up1", d2), e1), dim=1)     # 07:115-116
    d1 = _double_conv_relu(p, "dec1", d1)                 # 07:117
    return _conv(p, "final", d1, 0)                       # 07:119 (1x1, no activation)


# --------------------------------------------------------------------------
# ResUNet  (14_train_unified_advanced.py:96-186)
# --------------------------------------------------------------------------

def residual_block_forward(p, prefix, x, training, has_shortcut):
    """relu(BN(conv(PReLU(BN(conv(x))))) + shortcut(x))  -- 14:99-115."""
    cb = prefix + ".conv_block"
    h = _conv(p, cb + ".0", x, 1)
    h = _bn(p, cb + ".1", h, training)
    h = _prelu(p, cb + ".2", h)
    h = _conv(p, cb + ".3", h, 1)
    h = _bn(p, cb + ".4", h, training)
    if has_shortcut:                                     # 14:109-113 (in_c != out_c)
        s = _conv(p, prefix + ".shortcut.0", x, 0)
        s = _bn(p, prefix + ".shortcut.1", s, training)
    else:
        s = x
    return F.relu(h + s)                                 # 14:115


# (name, in_c, out_c) of every ResidualBlock, in forward order (14:125-145)
RESUNET_BLOCKS = [
    ("res1", 64, 64), ("res2", 64, 128), ("res3", 128, 256),
    ("bottleneck.0", 256, 512), ("bottleneck.1", 512, 512), ("bottleneck.2", 512, 256),
    ("dec3", 384, 128), ("dec2", 192, 64), ("dec1", 128, 64),
]
_RB = {n: (ci != co) for n, ci, co in RESUNET_BLOCKS}


def _align(d, r):
    # 14:169-182: nearest interpolate only when the sizes differ (never at 64/224)
    if d.size() != r.size():
        d = F.interpolate(d, size=r.shape[2:])
    return d


def resunet_forward(p, x, training):
    e1 = _prelu(p, "enc1.1", _conv(p, "enc1.0", x, 1))           # 14:122, 14:153
    r1 = residual_block_forward(p, "res1", e1, training, _RB["res1"])
    r2 = residual_block_forward(p, "res2", _maxpool(r1), training, _RB["res2"])
    r3 = residual_block_forward(p, "res3", _maxpool(r2), training, _RB["res3"])
    b = _maxpool(r3)
    for i in range(3):                                            # 14:137-141
        n = f"bottleneck.{i}"
        b = residual_block_forward(p, n, b, training, _RB[n])
    d3 = torch.cat((_align(_convT(p, "up3", b), r3), r3), dim=1)  # 14:167-174
    d3 = residual_block_forward(p, "dec3", d3, training, _RB["dec3"])
    d2 = torch.cat((_align(_convT(p, "up2", d3), r2), r2), dim=1)  # 14:176-180
    d2 = residual_block_forward(p, "dec2", d2, training, _RB["dec2"])
    d1 = torch.cat((_align(_convT(p, "up1", d2), r1), r1), dim=1)  # 14:182-186
    d1 = residual_block_forward(p, "dec1", d1, training, _RB["dec1"])
    return _conv(p, "final", d1, 0)


# --------------------------------------------------------------------------
# VGG16 (torchvision cfg "D") -- restated because torchvision is absent.
# --------------------------------------------------------------------------

VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M",
             512, 512, 512, "M", 512, 512, 512, "M"]


def vgg16_feature_layers():
    """[(index, kind, cin, cout)] of ``vgg16().features`` -- kind in conv/relu/pool."""
    layers, idx, cin = [], 0, 3
    for v in VGG16_CFG:
        if v == "M":
            layers.append((idx, "pool", None, None)); idx += 1
        else:
            layers.append((idx, "conv", cin, v)); idx += 1
            layers.append((idx, "relu", None, None)); idx += 1
            cin = v
    return layers


def vgg16_features_forward(p, x, upto=None, prefix="features"):
    """Run ``features[:upto]`` (upto=16 is the perceptual slice 14:192)."""
    for idx, kind, _, _ in vgg16_feature_layers():
        if upto is not None and idx >= upto:
            break
        if kind == "conv":
            x = _conv(p, f"{prefix}.{idx}", x, 1)
        elif kind == "relu":
            x = F.relu(x)
        else:
            x = _maxpool(x)
    return x


def vgg16_forward(p, x):
    """Eval-mode classifier (Dropout is identity): 18:46."""
    f = vgg16_features_forward(p, x)
    f = F.adaptive_avg_pool2d(f, (7, 7))
    f = torch.flatten(f, 1)
    f = F.relu(F.linear(f, p["classifier.0.weight"], p["classifier.0.bias"]))
    f = F.relu(F.linear(f, p["classifier.3.weight"], p["classifier.3.bias"]))
    return F.linear(f, p["classifier.6.weight"], p["classifier.6.bias"])


def perceptual_loss(p_slice, x, y):
    """mean((F(x) - F(y))^2), F = vgg16.features[:16], no input normalisation (14:195-196)."""
    fx = vgg16_features_forward(p_slice, x, upto=16, prefix="slice")
    fy = vgg16_features_forward(p_slice, y, upto=16, prefix="slice")
    return torch.mean((fx - fy) ** 2)


class TorchvisionVGG16(tnn.Module):
    """nn.Module form of torchvision's vgg16 (cfg D) with the 43-class head.

    Used (a) as the ``torchvision.models.vgg16`` stand-in when the reference
    scripts are imported in this container to generate fixtures and (b) as the
    key/shape manifest for ``features.*`` / ``classifier.*``.
    """

    def __init__(self, num_classes=43):
        super().__init__()
        mods = []
        for _, kind, cin, cout in vgg16_feature_layers():
            if kind == "conv":
                mods.append(tnn.Conv2d(cin, cout, 3, padding=1))
            elif kind == "relu":
                mods.append(tnn.ReLU(inplace=True))
            else:
                mods.append(tnn.MaxPool2d(2, 2))
        self.features = tnn.Sequential(*mods)
        self.avgpool = tnn.AdaptiveAvgPool2d((7, 7))
        self.classifier = tnn.Sequential(
            tnn.Linear(512 * 7 * 7, 4096), tnn.ReLU(True), tnn.Dropout(),
            tnn.Linear(4096, 4096), tnn.ReLU(True), tnn.Dropout(),
            tnn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))


# --------------------------------------------------------------------------
# losses / optimiser / post-processing
# --------------------------------------------------------------------------

def l1_loss(a, b):
    return torch.mean(torch.abs(a - b))       # nn.L1Loss (14:219)


def mse_loss(a, b):
    return torch.mean((a - b) ** 2)           # nn.MSELoss (07:142)


def unified_loss(out, clean, perc_params):
    """14:238-242: L1 + 0.1 * perceptual."""
    return l1_loss(out, clean) + 0.1 * perceptual_loss(perc_params, out, clean)


def adamw_step(params, grads, state, lr, betas=(0.9, 0.999), eps=1e-8,
               weight_decay=1e-2, decoupled=True):
    """One torch.optim.AdamW (decoupled=True, 14:222) / Adam (decoupled=False,
    wd 0, 07:143) step, restated with torch.optim's update order."""
    b1, b2 = betas
    state["step"] = state.get("step", 0) + 1
    t = state["step"]
    bc1 = 1 - b1 ** t
    bc2 = 1 - b2 ** t
    for k, prm in params.items():
        g = grads[k]
        if decoupled:
            prm.mul_(1 - lr * weight_decay)
        elif weight_decay:
            g = g.add(prm, alpha=weight_decay)
        m = state.setdefault(("m", k), torch.zeros_like(prm))
        v = state.setdefault(("v", k), torch.zeros_like(prm))
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        prm.addcdiv_(m, denom, value=-(lr / bc1))


def cosine_lr(base_lr, epoch, t_max, eta_min=0.0):
    """CosineAnnealingLR closed form (14:223, stepped per epoch 14:248)."""
    return eta_min + (base_lr - eta_min) * (1 + math.cos(math.pi * epoch / t_max)) / 2


def to_uint8_image(out):
    """17:84-92 / 08:96-98: clamp(0,1) -> HWC -> x255 -> astype(uint8) (truncation)."""
    o = torch.clamp(out, 0, 1).permute(0, 2, 3, 1).contiguous().numpy()
    return (o * 255).astype(np.uint8)


def psnr_u8(a, b, data_range=255.0):
    """skimage.metrics.peak_signal_noise_ratio on uint8 arrays (08:123)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    mse = np.mean((a - b) ** 2)
    if mse == 0:
        return float("inf")
    return float(10 * np.log10((data_range ** 2) / mse))


def top1(logits):
    """18:47: torch.max(outputs, 1) -> first index of the max."""
    return torch.max(logits, 1)[1]
