"""Reference-compatible modules backed by the gfx950 HIP kernels.

Same class names, constructor signatures, ``forward`` signatures and
``state_dict`` key trees as the reference (so its ``.pth`` files load
unchanged):

  SimpleUNet()              07_train_restoration.py:75-120 (26 keys)
  ResidualBlock(in_c, out_c) 14_train_unified_advanced.py:96-115
  ResUNet()                 14_train_unified_advanced.py:117-186 (195 keys)
  VGGPerceptualLoss()       14_train_unified_advanced.py:189-196
  vgg16(num_classes=43)     torchvision cfg "D" + 05:53-54 head swap
  L1Loss / MSELoss          14:219 / 07:142

Leaf modules (Conv2d, BatchNorm2d, PReLU, ...) carry the torch.nn default
initialisation and, called on their own, run one HIP op each
(roadrestore.layers); the parent networks run their whole
forward as one fused HIP schedule and their backward as one hand-written
reverse schedule (roadrestore.engine), each reached through a registered
PyTorch custom op (``torch.ops.rr.*``, roadrestore.torch_ops) with its
autograd formula.  Nothing here falls back to ATen compute: without the HIP
library or a device every forward raises.

The compute dtype (fp32 default: the parity path; bf16 for throughput) is a
per-model attribute, ``model.compute_dtype``, or ``RR_COMPUTE_DTYPE``.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as tnn

from . import engine, ops
from . import layers as _layers
from . import torch_ops as _tops

__all__ = ["Conv2d", "ConvTranspose2d", "BatchNorm2d", "PReLU", "ReLU", "MaxPool2d", "Linear",
           "Dropout", "AdaptiveAvgPool2d", "SimpleUNet", "ResidualBlock", "ResUNet",
           "VGG", "vgg16", "VGGPerceptualLoss", "L1Loss", "MSELoss", "unified_loss",
           "default_compute_dtype"]


def default_compute_dtype():
    v = os.environ.get("RR_COMPUTE_DTYPE", "float32").lower()
    return torch.bfloat16 if v in ("bf16", "bfloat16") else torch.float32


# ---------------------------------------------------------------------------
# leaf parameter containers (torch.nn default initialisation)

def _as_nchw(x):
    """an elementwise layer's [N, F] input (the VGG16 head) as [N, F, 1, 1]"""
    return x.reshape(x.shape[0], x.shape[1], 1, 1) if x.dim() == 2 else x


class _Leaf(tnn.Module):
    """A leaf layer.  Inside its parent network it is a parameter container
    (the parent runs one fused schedule and never calls it, so hooks on it do
    not fire there); called on its own -- ``model.enc1(x)``,
    ``vgg.features[:k](x)`` -- it runs its own HIP op (roadrestore.layers,
    ``torch.ops.rr.<layer>``) on NCHW fp32 tensors, with autograd."""

    def __init__(self):
        super().__init__()
        self.compute_dtype = default_compute_dtype()

    def _dt(self):
        return _layers.dtype_code(self.compute_dtype)

    @staticmethod
    def _x(x):
        if not x.is_cuda:
            raise RuntimeError("roadrestore layers run on the GPU only (no CPU fallback)")
        if x.dim() != 4:
            raise ValueError(f"expected an [N, C, H, W] input, got {tuple(x.shape)}")
        return x if x.dtype == torch.float32 else x.float()


class Conv2d(_Leaf):
    def __init__(self, in_channels, out_channels, kernel_size, padding=0, bias=True):
        super().__init__()
        k = kernel_size
        self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, (k, k)
        self.padding = (padding, padding)
        self.weight = tnn.Parameter(torch.empty(out_channels, in_channels, k, k))
        self.bias = tnn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        tnn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.weight.shape[1] * self.weight.shape[2] * self.weight.shape[3]
            b = 1 / math.sqrt(fan_in)
            tnn.init.uniform_(self.bias, -b, b)

    def forward(self, x):
        return torch.ops.rr.conv2d(self._x(x), self.weight, self.bias, self.padding[0], self._dt())


class ConvTranspose2d(_Leaf):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1):
        super().__init__()
        if kernel_size != 2 or stride != 2:
            raise NotImplementedError("only ConvTranspose2d(k=2, s=2) (07:88, 14:143)")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = tnn.Parameter(torch.empty(in_channels, out_channels, 2, 2))
        self.bias = tnn.Parameter(torch.empty(out_channels))
        tnn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        fan_in = out_channels * 4   # torch computes fan_in from weight.size(1) * k * k
        b = 1 / math.sqrt(fan_in)
        tnn.init.uniform_(self.bias, -b, b)

    def forward(self, x):
        return torch.ops.rr.conv_transpose2d(self._x(x), self.weight, self.bias, self._dt())


class BatchNorm2d(_Leaf):
    def __init__(self, num_features, eps=1e-5, momentum=0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = tnn.Parameter(torch.ones(num_features))
        self.bias = tnn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        self._op_key = _tops.register_module(self)

    def forward(self, x):
        """nn.BatchNorm2d: batch statistics in train mode (running statistics
        updated in place), running statistics in eval mode"""
        return torch.ops.rr.batch_norm(self._x(x), self.weight, self.bias, self._op_key,
                                       self.training, self._dt())[0]


class PReLU(_Leaf):
    def __init__(self, num_parameters=1, init=0.25):
        super().__init__()
        if num_parameters != 1:
            raise NotImplementedError("PReLU with one shared alpha (14:103)")
        self.weight = tnn.Parameter(torch.full((1,), float(init)))

    def forward(self, x):
        x4 = self._x(_as_nchw(x))
        return torch.ops.rr.prelu(x4, self.weight, self._dt()).view(x.shape)


class ReLU(_Leaf):
    def __init__(self, inplace=False):
        super().__init__()
        self.inplace = inplace

    def forward(self, x):
        """a new tensor also for inplace=True (the value torch returns)"""
        x4 = self._x(_as_nchw(x))
        return torch.ops.rr.relu(x4, self._dt()).view(x.shape)


class MaxPool2d(_Leaf):
    def __init__(self, kernel_size, stride=None):
        super().__init__()
        if kernel_size != 2 or (stride or 2) != 2:
            raise NotImplementedError("only MaxPool2d(2, 2)")
        self.kernel_size, self.stride = 2, 2

    def forward(self, x):
        return torch.ops.rr.max_pool2d(self._x(x), self._dt())[0]


class Linear(_Leaf):
    def __init__(self, in_features, out_features):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = tnn.Parameter(torch.empty(out_features, in_features))
        self.bias = tnn.Parameter(torch.empty(out_features))
        tnn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        b = 1 / math.sqrt(in_features)
        tnn.init.uniform_(self.bias, -b, b)

    def forward(self, x):
        """forward only (the VGG16 head is the frozen judge, 18:46)"""
        if not x.is_cuda:
            raise RuntimeError("roadrestore layers run on the GPU only (no CPU fallback)")
        if torch.is_grad_enabled() and (x.requires_grad or self.weight.requires_grad
                                        or self.bias.requires_grad):
            raise NotImplementedError("Linear runs forward-only (frozen VGG16 judge): use "
                                      "torch.no_grad() or freeze its parameters")
        lead = x.shape[:-1]
        y = torch.ops.rr.linear(x.float().reshape(-1, x.shape[-1]), self.weight, self.bias,
                                self._dt())
        return y.view(*lead, -1)


class Dropout(_Leaf):
    def __init__(self, p=0.5):
        super().__init__()
        self.p = p

    def forward(self, x):
        """eval (the judge, 18:46): the identity.  Training-mode dropout
        (VGG16 training, 05) is out of scope."""
        if self.training and self.p > 0:
            raise NotImplementedError("training-mode Dropout is out of scope (eval: identity)")
        return x


class AdaptiveAvgPool2d(_Leaf):
    def __init__(self, output_size):
        super().__init__()
        self.output_size = output_size

    def forward(self, x):
        """forward only (the frozen judge's head)"""
        x = self._x(x)
        if torch.is_grad_enabled() and x.requires_grad:
            raise NotImplementedError("AdaptiveAvgPool2d runs forward-only (frozen VGG16 judge)")
        o = self.output_size
        oh, ow = (o, o) if isinstance(o, int) else o
        return torch.ops.rr.adaptive_avg_pool2d(x, oh, ow, self._dt())


# ---------------------------------------------------------------------------
# networks: one custom op (torch.ops.rr.<name>_forward) per call, its
# registered autograd formula calls rr::<name>_backward (torch_ops.py)

class _RRNet(tnn.Module):
    """Shared plumbing of the restorers."""

    _has_bn = True
    _op = None        # torch.ops.rr.<_op>_forward runs this network

    def __init__(self):
        super().__init__()
        self.compute_dtype = default_compute_dtype()
        self._wc = engine.WeightCache()
        self._grad_hook = None
        self._op_key = _tops.register_module(self)

    def train(self, mode=True):
        super().train(mode)
        if not mode:
            self._wc.drop_folds()      # running statistics may have moved (graph replays too)
        return self

    def prefetch_weights(self):
        """Start re-packing the weights for the next forward on a side stream
        now (call at the start of a training step, after the previous
        optimizer step and before the batch's input pipeline): the next
        forward joins it instead of packing in front of its first conv.  A
        no-op before the first forward.  Returns whether a pack was forked."""
        return self._wc.prefetch()

    # data-parallel wrappers install a hook called as grad groups become final
    def set_grad_ready_hook(self, hook):
        self._grad_hook = hook

    def _check_input(self, x):
        if not x.is_cuda:
            raise RuntimeError("roadrestore networks run on the GPU only (no CPU fallback)")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected [N, 3, H, W], got {tuple(x.shape)}")
        if x.dtype != torch.float32:
            x = x.float()
        return x.contiguous()

    def _empty_forward(self, x, need):
        """An empty batch, as torch runs the reference modules on one: an empty
        output; train-mode BNs count the batch (nn.BatchNorm2d increments
        num_batches_tracked before F.batch_norm) and keep their running stats
        (ATen returns early on empty input); every parameter gets a zero grad."""
        if self.training:
            for m in self.modules():
                if isinstance(m, BatchNorm2d):
                    m.num_batches_tracked.add_(1)
        cout = self.conv_block[0].out_channels if isinstance(self, ResidualBlock) else 3
        out = x.new_zeros((0, cout) + tuple(x.shape[2:]))
        if need:
            out = out + sum(p.sum() * 0 for p in self.parameters() if p.requires_grad)
        return out

    def forward(self, x):
        x = self._check_input(x)
        params = [p for p in self.parameters()]
        need = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        if x.shape[0] == 0:
            return self._empty_forward(x, need)
        fwd = getattr(torch.ops.rr, f"{self._op}_forward")
        out, _ = fwd(x, params, self._op_key, need)
        return out

    def _make_sink(self, order, zero_params, device):
        return engine.GradSink(order, device, zero_params=zero_params, hook=self._grad_hook)

    def grad_layout(self):
        """Parameters in flat-gradient order (zero-gradient ones first)."""
        order, zero = self._grad_order()
        zs = {id(z) for z in zero}
        return [p for p in order if id(p) in zs] + [p for p in order if id(p) not in zs]


class SimpleUNet(_RRNet):
    """07_train_restoration.py:75-120 (verbatim copies at 07adv:65-92, 08:19-46, 13:59-85)."""

    _has_bn = False
    _op = "simple_unet"

    def __init__(self):
        super().__init__()
        self.enc1 = tnn.Sequential(Conv2d(3, 64, 3, padding=1), ReLU(), Conv2d(64, 64, 3, padding=1), ReLU())
        self.pool1 = MaxPool2d(2, 2)
        self.enc2 = tnn.Sequential(Conv2d(64, 128, 3, padding=1), ReLU(), Conv2d(128, 128, 3, padding=1), ReLU())
        self.pool2 = MaxPool2d(2, 2)
        self.bottleneck = tnn.Sequential(Conv2d(128, 256, 3, padding=1), ReLU(),
                                         Conv2d(256, 256, 3, padding=1), ReLU())
        self.up2 = ConvTranspose2d(256, 128, 2, stride=2)
        self.dec2 = tnn.Sequential(Conv2d(256, 128, 3, padding=1), ReLU(), Conv2d(128, 128, 3, padding=1), ReLU())
        self.up1 = ConvTranspose2d(128, 64, 2, stride=2)
        self.dec1 = tnn.Sequential(Conv2d(128, 64, 3, padding=1), ReLU(), Conv2d(64, 64, 3, padding=1), ReLU())
        self.final = Conv2d(64, 3, 1)

    def _grad_order(self):
        return engine.simple_unet_grad_order(self), []

    def _rr_forward(self, x, need_bwd):
        if x.shape[2] % 4 or x.shape[3] % 4:
            raise NotImplementedError("SimpleUNet input sizes must be multiples of 4")
        return engine.simple_unet_forward(self, x, self._wc, self.compute_dtype, need_bwd)

    def _rr_backward(self, S, g):
        order, zero = self._grad_order()
        sink = self._make_sink(order, zero, g.device)
        engine.simple_unet_backward(self, S, g, sink)
        return sink.flat


class ResidualBlock(_RRNet):
    """14_train_unified_advanced.py:96-115 (copies 15:24-41, 17:21-27).

    As a standalone module its forward takes / returns NCHW fp32 tensors; the
    ResUNet runs its blocks on NHWC activations inside one schedule."""

    _op = "resblock"

    def __init__(self, in_c, out_c):
        super().__init__()
        self.conv_block = tnn.Sequential(
            Conv2d(in_c, out_c, 3, padding=1), BatchNorm2d(out_c), PReLU(),
            Conv2d(out_c, out_c, 3, padding=1), BatchNorm2d(out_c))
        self.shortcut = tnn.Sequential()
        if in_c != out_c:
            self.shortcut = tnn.Sequential(Conv2d(in_c, out_c, 1), BatchNorm2d(out_c))

    def _check_input(self, x):
        if not x.is_cuda:
            raise RuntimeError("roadrestore networks run on the GPU only (no CPU fallback)")
        return x.float().contiguous()

    def _grad_order(self):
        return list(self.parameters()), engine.resblock_zero_grad_params(self)

    def _rr_forward(self, x, need_bwd):
        n, c, h, w = x.shape
        xn = ops.nchw_to_nhwc(x, self.compute_dtype)
        y, S = engine.resblock_forward(self, xn, None, n, h, w, self._wc, self.compute_dtype,
                                       self.training, need_bwd)
        return ops.nhwc_to_nchw(y), S

    def _rr_backward(self, S, g):
        order, zero = self._grad_order()
        sink = self._make_sink(order, zero, g.device)
        gn = ops.nchw_to_nhwc(g, self.compute_dtype)
        engine.resblock_backward(self, S, gn, sink)
        return sink.flat


class ResUNet(_RRNet):
    """14_train_unified_advanced.py:117-186 (copies 15:43-90, 17:29-55)."""

    _op = "resunet"

    def __init__(self):
        super().__init__()
        self.enc1 = tnn.Sequential(Conv2d(3, 64, 3, padding=1), PReLU())
        self.res1 = ResidualBlock(64, 64)
        self.pool1 = MaxPool2d(2, 2)
        self.res2 = ResidualBlock(64, 128)
        self.pool2 = MaxPool2d(2, 2)
        self.res3 = ResidualBlock(128, 256)
        self.pool3 = MaxPool2d(2, 2)
        self.bottleneck = tnn.Sequential(ResidualBlock(256, 512), ResidualBlock(512, 512),
                                         ResidualBlock(512, 256))
        self.up3 = ConvTranspose2d(256, 128, 2, stride=2)
        self.dec3 = ResidualBlock(256 + 128, 128)
        self.up2 = ConvTranspose2d(128, 64, 2, stride=2)
        self.dec2 = ResidualBlock(128 + 64, 64)
        self.up1 = ConvTranspose2d(64, 64, 2, stride=2)
        self.dec1 = ResidualBlock(64 + 64, 64)
        self.final = Conv2d(64, 3, 1)

    def _blocks(self):
        return [self.get_submodule(n) for n in engine.resunet_block_names()]

    def _grad_order(self):
        return engine.resunet_grad_order(self), engine.resunet_zero_grad_params(self)

    def _rr_forward(self, x, need_bwd):
        return engine.resunet_forward(self, x, self._wc, self.compute_dtype, self.training,
                                      need_bwd)

    def _rr_backward(self, S, g):
        order, zero = self._grad_order()
        sink = self._make_sink(order, zero, g.device)
        engine.resunet_backward(self, S, g, sink)
        return sink.flat


# ---------------------------------------------------------------------------
# VGG16 (torchvision cfg "D") and the perceptual loss

_CFG_D = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


def _vgg_features(upto=None):
    layers, cin = [], 3
    for v in _CFG_D:
        if v == "M":
            layers.append(MaxPool2d(2, 2))
        else:
            layers += [Conv2d(cin, v, 3, padding=1), ReLU(inplace=True)]
            cin = v
        if upto is not None and len(layers) >= upto:
            break
    layers = layers[:upto] if upto is not None else layers
    for m in layers:                 # torchvision's VGG conv init
        if isinstance(m, Conv2d):
            tnn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            tnn.init.constant_(m.bias, 0)
    return layers


class VGG(tnn.Module):
    """torchvision ``VGG`` (features / avgpool / classifier key tree)."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = tnn.Sequential(*_vgg_features())
        self.avgpool = AdaptiveAvgPool2d((7, 7))
        self.classifier = tnn.Sequential(
            Linear(512 * 7 * 7, 4096), ReLU(True), Dropout(),
            Linear(4096, 4096), ReLU(True), Dropout(),
            Linear(4096, num_classes))
        for m in self.classifier:    # torchvision's VGG linear init
            if isinstance(m, Linear):
                tnn.init.normal_(m.weight, 0, 0.01)
                tnn.init.constant_(m.bias, 0)
        self.compute_dtype = default_compute_dtype()
        self._wc = engine.WeightCache()
        self._op_key = _tops.register_module(self)

    def forward(self, x):
        """Eval-mode logits (18:46): the classifier is the fixed judge."""
        if not x.is_cuda:
            raise RuntimeError("roadrestore networks run on the GPU only (no CPU fallback)")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError("VGG16 runs as the frozen judge: use torch.no_grad()")
        return torch.ops.rr.vgg16_logits(x.float().contiguous(), list(self.parameters()),
                                         self._op_key)


def vgg16(weights=None, num_classes=43, **kw):
    """``torchvision.models.vgg16`` with the 43-class head of 05:53-54 / 18:59.

    ``weights`` must be None (no network access); load a state_dict instead."""
    if weights is not None:
        raise RuntimeError("pretrained weights need a network download; load a state_dict")
    return VGG(num_classes=num_classes)


class VGGPerceptualLoss(tnn.Module):
    """14:189-196 (07adv:95-112): mean((F(x) - F(y))^2), F = vgg16.features[:16]
    (conv1_1 .. relu3_3), frozen, inputs not ImageNet-normalised."""

    def __init__(self, vgg=None):
        super().__init__()
        feats = list(vgg.features)[:16] if vgg is not None else _vgg_features(16)
        self.slice = tnn.Sequential(*feats)
        self.slice.eval()
        for p in self.slice.parameters():
            p.requires_grad = False
        self.compute_dtype = default_compute_dtype()
        self._wc = engine.WeightCache(static=True)     # frozen: packed once, also for HIP graphs
        self._op_key = _tops.register_module(self)
        self._side = None
        self._pending = None

    def prefetch_target(self, y):
        """Start F(y), the target's features (no gradient flows into y), on a
        side stream, so it runs concurrently with what the caller launches
        next -- the distortion and the restorer's forward, which F(y) does not
        depend on.  The next perceptual / unified loss on this same ``y`` joins
        it (stream-ordered, also inside a HIP-graph capture).  Returns the
        tensor to pass to the loss.  (Forking later, at a block of the
        restorer's forward, measured within 0.4 % of forking here,
        profiles/r5x_abstep_perc_prefetch_at.txt.)"""
        y = y.float().contiguous()
        self._join()
        if self._side is None or self._side.device != y.device:
            self._side = torch.cuda.Stream(device=y.device)
        box = {}
        self._side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self._side):
            box["fy"], _ = engine.vgg_features_forward(self.slice, y, self._wc, self.compute_dtype)
            box["ev"] = torch.cuda.Event()
            box["ev"].record(self._side)
        self._pending = (y, box)
        return y

    def _join(self):
        p, self._pending = self._pending, None
        if p is not None:
            torch.cuda.current_stream().wait_event(p[1]["ev"])
        return p

    def _target_features(self, y):
        """F(y): the prefetched features when ``y`` is the prefetched tensor
        (same storage, shape and version), else computed here."""
        p = self._join()
        if p is not None and p[0].data_ptr() == y.data_ptr() and p[0].shape == y.shape and \
                p[0]._version == y._version:
            return p[1]["fy"]
        fy, _ = engine.vgg_features_forward(self.slice, y, self._wc, self.compute_dtype)
        return fy

    def _rr_forward(self, x, y, scale, need_bwd):
        fy = self._target_features(y)
        fx, S = engine.vgg_features_forward(self.slice, x, self._wc, self.compute_dtype,
                                            need_bwd=need_bwd)
        if S.layers[-1][0] != "conv_relu":
            raise RuntimeError("perceptual slice must end in a conv+ReLU (relu3_3)")
        loss = ops.loss_fwd(ops.MSE, fx, fy, scale=scale)
        return loss, S, fx, fy

    def forward(self, x, y):
        x = x.float().contiguous()
        y = y.float().contiguous()
        need = torch.is_grad_enabled() and x.requires_grad
        return torch.ops.rr.perceptual_loss(x, y, self._op_key, need)[0]


class L1Loss(tnn.Module):
    """nn.L1Loss (mean) on device tensors (14:219)."""

    def forward(self, a, b):
        return torch.ops.rr.pixel_loss(a.float().contiguous(), b.float().contiguous(), ops.L1)


class MSELoss(tnn.Module):
    """nn.MSELoss (mean) on device tensors (07:142)."""

    def forward(self, a, b):
        return torch.ops.rr.pixel_loss(a.float().contiguous(), b.float().contiguous(), ops.MSE)


def unified_loss(out, clean, perc, w=0.1, grad_scale=1.0):
    """L1(out, clean) + w * perceptual(out, clean) as ONE autograd node
    (14:238-242) with a single fused gradient; ``grad_scale`` pre-scales the
    backward (1/world_size under data parallelism).  Under ``torch.no_grad()``
    (the validation loss, 14:253-263) no backward state is kept."""
    need = torch.is_grad_enabled() and out.requires_grad
    return torch.ops.rr.unified_loss(out.contiguous(), clean.float().contiguous(), perc._op_key,
                                     float(w), float(grad_scale), need)[0]
