"""bf16-storage emulation of the ResUNet unified step -- TEST INFRASTRUCTURE ONLY.

The restatement of oracle/reference_cpu.py (14_train_unified_advanced.py:
96-196) evaluated in fp64, with every tensor the bf16 HIP path STORES rounded
to bf16 at the same point -- in the forward (activations, packed weights, the
first conv's image operand) and in the backward (the gradient of every stored
activation).  Arithmetic between storage points stays exact-ish (fp64); the
HIP path accumulates in fp32.  So this is the "ideal bf16 implementation" of
the reference step: the distance between it and the fp64 oracle is the error
that bf16 storage alone causes, and it bounds what the HIP bf16 path may be
held to (tests/test_bf16_model_gpu.py).

Rounding points (roadrestore/engine.py resunet_forward / resblock_forward /
vgg_features_forward and their backward schedules):
  * conv / convT inputs and weights (and the first conv's bias, folded into
    the bf16 K = 32 GEMM as a ones column);
  * conv outputs t1, t2, s (pre-BN), e1 pre-activation, convT outputs;
  * BN1 + PReLU output a1, residual block output, encoder max-pool outputs;
  * VGG16[:16] conv + ReLU outputs;
  * the gradient flowing into each of those tensors.
Only ``tests/`` may import this module.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import reference_cpu as R


def _rb(x):
    return x.to(torch.bfloat16).to(x.dtype)


class _Q(torch.autograd.Function):
    """bf16 storage: round the value forward and the gradient backward."""

    @staticmethod
    def forward(ctx, x):
        return _rb(x)

    @staticmethod
    def backward(ctx, g):
        return _rb(g)


def q(x):
    return _Q.apply(x)


class _QW(torch.autograd.Function):
    """packed weights: bf16 values forward, the fp32 master's gradient exact."""

    @staticmethod
    def forward(ctx, w):
        return _rb(w)

    @staticmethod
    def backward(ctx, g):
        return g


def qw(w):
    return _QW.apply(w)


def _conv(p, name, x, padding):
    return F.conv2d(x, qw(p[name + ".weight"]), p[name + ".bias"], padding=padding)


def _bn(p, name, x, training):
    return R._bn(p, name, x, training)


def residual_block_forward(p, prefix, x, training, has_shortcut):
    cb = prefix + ".conv_block"
    t1 = q(_conv(p, cb + ".0", x, 1))
    a1 = q(F.prelu(_bn(p, cb + ".1", t1, training), p[cb + ".2.weight"]))
    t2 = q(_conv(p, cb + ".3", a1, 1))
    h = _bn(p, cb + ".4", t2, training)
    if has_shortcut:
        s = q(_conv(p, prefix + ".shortcut.0", x, 0))
        s = _bn(p, prefix + ".shortcut.1", s, training)
    else:
        s = x
    return q(F.relu(h + s))


def _first_conv(p, name, x):
    # bf16 K = 32 GEMM: image, weights and bias (ones column) all bf16
    return F.conv2d(_rb_image(x), qw(p[name + ".weight"]), qw(p[name + ".bias"]), padding=1)


class _QImg(torch.autograd.Function):
    """the first conv reads the fp32 image into bf16 fragments; its image
    gradient (VGG dgrad into the restored output) is written in fp32"""

    @staticmethod
    def forward(ctx, x):
        return _rb(x)

    @staticmethod
    def backward(ctx, g):
        return g


def _rb_image(x):
    return _QImg.apply(x)


def _convT(p, name, x):
    return q(F.conv_transpose2d(x, qw(p[name + ".weight"]), p[name + ".bias"], stride=2))


def resunet_forward(p, x, training):
    # conv + PReLU fused: the activation from the fp32 accumulator, stored bf16
    e1 = q(F.prelu(_first_conv(p, "enc1.0", x), p["enc1.1.weight"]))
    r1 = residual_block_forward(p, "res1", e1, training, R._RB["res1"])
    r2 = residual_block_forward(p, "res2", R._maxpool(r1), training, R._RB["res2"])
    r3 = residual_block_forward(p, "res3", R._maxpool(r2), training, R._RB["res3"])
    b = R._maxpool(r3)
    for i in range(3):
        n = f"bottleneck.{i}"
        b = residual_block_forward(p, n, b, training, R._RB[n])
    d3 = torch.cat((R._align(_convT(p, "up3", b), r3), r3), dim=1)
    d3 = residual_block_forward(p, "dec3", d3, training, R._RB["dec3"])
    d2 = torch.cat((R._align(_convT(p, "up2", d3), r2), r2), dim=1)
    d2 = residual_block_forward(p, "dec2", d2, training, R._RB["dec2"])
    d1 = torch.cat((R._align(_convT(p, "up1", d2), r1), r1), dim=1)
    d1 = residual_block_forward(p, "dec1", d1, training, R._RB["dec1"])
    return _conv(p, "final", d1, 0)            # NCHW fp32 out of the GEMM epilogue


def vgg16_features_forward(p, x, upto=16, prefix="slice"):
    first = True
    for idx, kind, _, _ in R.vgg16_feature_layers():
        if upto is not None and idx >= upto:
            break
        if kind == "conv":
            name = f"{prefix}.{idx}"
            if first:
                x = F.conv2d(_rb_image(x), qw(p[name + ".weight"]), qw(p[name + ".bias"]), padding=1)
                first = False
            else:
                x = F.conv2d(x, qw(p[name + ".weight"]), p[name + ".bias"], padding=1)
        elif kind == "relu":
            x = q(F.relu(x))
        else:
            x = R._maxpool(x)
    return x


def unified_loss(out, clean, perc_params):
    fx = vgg16_features_forward(perc_params, out)
    fy = vgg16_features_forward(perc_params, clean)
    return R.l1_loss(out, clean) + 0.1 * torch.mean((fx - fy) ** 2)


# ---------------------------------------------------------------------------
# inference (cfg5, 17:84-86 and 18:46-47): eval-mode BN folded into the conv
# before it, as roadrestore.engine.resblock_forward_eval_folded runs it

def _fold(p, conv, bn):
    """W' = s.W, b' = s.b + t with s = gamma / sqrt(var + eps), t = beta - mean.s
    (rr_fold_conv_bn); the packed W' is stored bf16, b' stays fp32."""
    s = p[bn + ".weight"] / torch.sqrt(p[bn + ".running_var"] + R.BN_EPS)
    t = p[bn + ".bias"] - p[bn + ".running_mean"] * s
    return qw(p[conv + ".weight"] * s.view(-1, 1, 1, 1)), p[conv + ".bias"] * s + t


def residual_block_forward_folded(p, prefix, x, has_shortcut, pooled_after=False):
    cb = prefix + ".conv_block"
    w1, b1 = _fold(p, cb + ".0", cb + ".1")
    a1 = q(F.prelu(F.conv2d(x, w1, b1, padding=1), p[cb + ".2.weight"]))
    w2, b2 = _fold(p, cb + ".3", cb + ".4")
    c2 = F.conv2d(a1, w2, b2, padding=1)
    if not has_shortcut:
        return q(F.relu(c2 + x))                      # identity: one epilogue
    ws, bs = _fold(p, prefix + ".shortcut.0", prefix + ".shortcut.1")
    s = q(F.conv2d(x, ws, bs))                        # the 1x1 output, stored
    if pooled_after:
        return q(F.relu(c2 + s))                      # conv2 accumulates onto it
    return q(F.relu(q(c2) + F.conv2d(x, ws, bs)))     # the 1x1 accumulates onto t2


def resunet_forward_eval_folded(p, x):
    e1 = q(F.prelu(_first_conv(p, "enc1.0", x), p["enc1.1.weight"]))
    r1 = residual_block_forward_folded(p, "res1", e1, R._RB["res1"], True)
    r2 = residual_block_forward_folded(p, "res2", R._maxpool(r1), R._RB["res2"], True)
    r3 = residual_block_forward_folded(p, "res3", R._maxpool(r2), R._RB["res3"], True)
    b = R._maxpool(r3)
    for i in range(3):
        n = f"bottleneck.{i}"
        b = residual_block_forward_folded(p, n, b, R._RB[n])
    d3 = torch.cat((R._align(_convT(p, "up3", b), r3), r3), dim=1)
    d3 = residual_block_forward_folded(p, "dec3", d3, R._RB["dec3"])
    d2 = torch.cat((R._align(_convT(p, "up2", d3), r2), r2), dim=1)
    d2 = residual_block_forward_folded(p, "dec2", d2, R._RB["dec2"])
    d1 = torch.cat((R._align(_convT(p, "up1", d2), r1), r1), dim=1)
    d1 = residual_block_forward_folded(p, "dec1", d1, R._RB["dec1"])
    return _conv(p, "final", d1, 0)


def vgg16_forward(p, x):
    """The bf16 judge (engine.vgg_classifier_forward): conv + ReLU outputs,
    the 7x7 average pool and each Linear output stored bf16 (the logits too),
    bf16 weights, fp32 biases."""
    f = vgg16_features_forward(p, x, upto=None, prefix="features")
    f = q(torch.flatten(F.adaptive_avg_pool2d(f, (7, 7)), 1))
    f = q(F.relu(F.linear(f, qw(p["classifier.0.weight"]), p["classifier.0.bias"])))
    f = q(F.relu(F.linear(f, qw(p["classifier.3.weight"]), p["classifier.3.bias"])))
    return q(F.linear(f, qw(p["classifier.6.weight"]), p["classifier.6.bias"]))
