"""The hot path registered as PyTorch custom ops (namespace ``rr``).

Every network call of the reference's training / inference loops reaches the
HIP schedule through one of these ops, so ``torch.profiler`` attributes the
time to ``rr::resunet_forward`` etc., ``torch.library.opcheck`` can check the
schemas, and fake (meta) kernels give shapes without a device:

  rr::resunet_forward / rr::resunet_backward          14:117-186 (ResUNet)
  rr::simple_unet_forward / rr::simple_unet_backward  07:75-120 (SimpleUNet)
  rr::resblock_forward / rr::resblock_backward        14:96-115 (ResidualBlock)
  rr::unified_loss / rr::unified_loss_backward        14:238-242 (L1 + w perceptual)
  rr::perceptual_loss / rr::perceptual_loss_backward  14:189-196 (VGGPerceptualLoss)
  rr::pixel_loss / rr::pixel_loss_backward            14:219 L1Loss, 07:142 MSELoss
  rr::vgg16_logits                                    18:46 (frozen VGG16 judge)
  rr::nearest_resize                                  14:169-182 (F.interpolate)
  rr::to_uint8_hwc, rr::psnr_u8, rr::argmax_rows      17:84-92, 08:123, 18:47

Autograd is registered on the forward ops (``torch.library.register_autograd``):
the backward op is our own reverse schedule, never ATen's.  A module-level op
takes the module's parameters as a tensor list (the autograd edges) plus an
integer key naming the module object whose schedule (weight cache, compute
dtype, gradient sink) it runs; in train mode it updates that module's
BatchNorm running statistics in place, as nn.BatchNorm2d does (module state,
not an op argument: an op with mutated arguments cannot carry an autograd
formula).
The forward's saved state (activations, packed weights) lives in a per-process
table under an int64 handle tensor that the backward op consumes.  The entry
lives exactly as long as that handle: the autograd node keeps the handle, so a
graph dropped without a backward (an exception, an eval pass with grads on)
frees the state with the graph (``weakref.finalize`` on the handle), and a
forward run where no backward can follow stores nothing.  The backward pops
the entry (saved state is freed by the backward, as autograd frees saved
tensors; a second backward through a ``retain_graph`` graph raises).  A status
from the C ABI becomes a RuntimeError (``_lib.check``), as ATen's shape errors
do.  There is no CPU or ATen fallback: the real kernels need a HIP device.
"""
from __future__ import annotations

import itertools
import weakref
from typing import List, Tuple

import torch
from torch import Tensor

from . import engine, ops

__all__ = ["register_module", "OPS"]

_MODULES: dict = {}          # key -> weakref of the module whose schedule an op runs
_SAVED: dict = {}            # handle -> forward state consumed by the backward op
_HANDLES = itertools.count(1)


def register_module(mod) -> int:
    k = id(mod)
    _MODULES[k] = weakref.ref(mod)
    return k


def _module(key: int):
    r = _MODULES.get(key)
    mod = r() if r is not None else None
    if mod is None:
        raise RuntimeError(f"rr op: no live module registered under key {key}")
    return mod


def _stash(state) -> Tensor:
    """a handle tensor owning ``state``: the table entry goes with the handle"""
    h = next(_HANDLES)
    _SAVED[h] = state
    t = torch.tensor(h, dtype=torch.int64)
    weakref.finalize(t, _SAVED.pop, h, None)
    return t


def _no_state() -> Tensor:
    return torch.tensor(0, dtype=torch.int64)


def saved_state_count() -> int:
    """live forward states (diagnostics / tests)"""
    return len(_SAVED)


def _unstash(handle: Tensor):
    h = int(handle.item())
    try:
        return _SAVED.pop(h)
    except KeyError:
        raise RuntimeError("rr op: the forward state of this backward was already consumed "
                           "(backward called twice?)") from None


def _flat_views(layout, flat):
    """id(param) -> its gradient view in the flat buffer (layout order)"""
    out, off = {}, 0
    for p in layout:
        out[id(p)] = flat[off:off + p.numel()].view(p.shape)
        off += p.numel()
    return out


# ---------------------------------------------------------------------------
# restoration networks: one op pair per network class

def _net_op(prefix, doc):
    fwd_name, bwd_name = f"rr::{prefix}_forward", f"rr::{prefix}_backward"

    @torch.library.custom_op(fwd_name, mutates_args=(), device_types="cuda")
    def fwd(x: Tensor, params: List[Tensor], module: int,
            need_backward: bool) -> Tuple[Tensor, Tensor]:
        net = _module(module)
        out, S = net._rr_forward(x, need_bwd=need_backward)
        return out, (_stash(S) if need_backward else _no_state())

    @fwd.register_fake
    def _(x, params, module, need_backward):
        n, _, h, w = x.shape
        cout = 3
        if prefix == "resblock":
            cout = params[0].shape[0]
        return x.new_empty((n, cout, h, w)), torch.empty((), dtype=torch.int64)

    @torch.library.custom_op(bwd_name, mutates_args=(), device_types="cuda")
    def bwd(grad: Tensor, handle: Tensor, module: int) -> Tensor:
        """the reverse schedule; returns the flat fp32 gradient buffer in the
        module's grad_layout() order"""
        net = _module(module)
        return net._rr_backward(_unstash(handle), grad.contiguous())

    @bwd.register_fake
    def _(grad, handle, module):
        net = _module(module)
        return grad.new_empty((sum(p.numel() for p in net.grad_layout()),), dtype=torch.float32)

    def setup_context(ctx, inputs, output):
        _, params, module, need_backward = inputs
        ctx.module = module
        ctx.handle = output[1]
        ctx.n_params = len(params)
        ctx.params = params
        ctx.need = need_backward

    def backward(ctx, grad_out, grad_handle):
        if not ctx.need:
            raise RuntimeError(f"{fwd_name}: run with need_backward=True to differentiate")
        flat = getattr(torch.ops.rr, f"{prefix}_backward")(grad_out, ctx.handle, ctx.module)
        # per-parameter views of the one buffer (autograd adopts them as .grad)
        views = _flat_views(_module(ctx.module).grad_layout(), flat)
        return None, [views.get(id(p)) for p in ctx.params], None, None

    fwd.register_autograd(backward, setup_context=setup_context)
    fwd.__doc__ = doc
    return fwd, bwd


resunet_forward, resunet_backward = _net_op("resunet", "ResUNet fused schedule (14:117-186)")
simple_unet_forward, simple_unet_backward = _net_op("simple_unet",
                                                    "SimpleUNet fused schedule (07:75-120)")
resblock_forward, resblock_backward = _net_op("resblock",
                                              "standalone ResidualBlock (14:96-115), NCHW fp32")


# ---------------------------------------------------------------------------
# losses

@torch.library.custom_op("rr::pixel_loss", mutates_args=(), device_types="cuda")
def pixel_loss(a: Tensor, b: Tensor, kind: int) -> Tensor:
    """mean |a - b| (kind L1, 14:219) or mean (a - b)^2 (kind MSE, 07:142)"""
    return ops.loss_fwd(kind, a.contiguous(), b.contiguous())


@pixel_loss.register_fake
def _(a, b, kind):
    return a.new_empty(())


@torch.library.custom_op("rr::pixel_loss_backward", mutates_args=(), device_types="cuda")
def pixel_loss_backward(grad: Tensor, a: Tensor, b: Tensor, kind: int) -> Tensor:
    return ops.loss_bwd(kind, a, b, gscale=grad.contiguous())


@pixel_loss_backward.register_fake
def _(grad, a, b, kind):
    return torch.empty_like(a)


def _pix_setup(ctx, inputs, output):
    a, b, kind = inputs
    ctx.save_for_backward(a, b)
    ctx.kind = kind


def _pix_bwd(ctx, g):
    a, b = ctx.saved_tensors
    return torch.ops.rr.pixel_loss_backward(g, a, b, ctx.kind), None, None


pixel_loss.register_autograd(_pix_bwd, setup_context=_pix_setup)


@torch.library.custom_op("rr::unified_loss", mutates_args=(), device_types="cuda")
def unified_loss(out: Tensor, clean: Tensor, perceptual: int, w: float,
                 grad_scale: float, need_backward: bool) -> Tuple[Tensor, Tensor]:
    """L1(out, clean) + w * mean((F(out) - F(clean))^2), F = VGG16
    features[:16] (14:238-242), one fused node; with ``need_backward`` the
    handle carries the feature-stack state for rr::unified_loss_backward
    (without it -- the no-grad validation loss of 14:253-263 -- nothing is
    kept)"""
    perc = _module(perceptual)
    loss = ops.loss_fwd(ops.L1, out, clean)
    st = None
    if w != 0.0:
        fy = perc._target_features(clean)
        fx, S = engine.vgg_features_forward(perc.slice, out, perc._wc, perc.compute_dtype,
                                            need_bwd=need_backward)
        ops.loss_fwd(ops.MSE, fx, fy, scale=w, out=loss, accumulate=True)
        st = (S, fx, fy)
    else:
        perc._join()                 # a prefetched target is not needed, but joins the stream
    return loss, (_stash(st) if need_backward else _no_state())


@unified_loss.register_fake
def _(out, clean, perceptual, w, grad_scale, need_backward):
    return out.new_empty(()), torch.empty((), dtype=torch.int64)


@torch.library.custom_op("rr::unified_loss_backward", mutates_args=(), device_types="cuda")
def unified_loss_backward(grad: Tensor, out: Tensor, clean: Tensor, handle: Tensor, w: float,
                          grad_scale: float) -> Tensor:
    st = _unstash(handle)
    g = grad.contiguous()
    gout = ops.loss_bwd(ops.L1, out, clean, gscale=g, scale=grad_scale)
    if st is not None:
        S, fx, fy = st
        gpre = ops.loss_bwd(ops.MSE, fx, fy, gscale=g, scale=w * grad_scale, mask_a_pos=True)
        engine.vgg_features_backward_input(S, gpre, x_grad_out=gout, accumulate=True)
    return gout


@unified_loss_backward.register_fake
def _(grad, out, clean, handle, w, grad_scale):
    return torch.empty_like(out)


def _uni_setup(ctx, inputs, output):
    out, clean, _, w, gs, need = inputs
    ctx.save_for_backward(out, clean)
    ctx.handle, ctx.w, ctx.gs, ctx.need = output[1], w, gs, need


def _uni_bwd(ctx, g, g_handle):
    if not ctx.need:
        raise RuntimeError("rr::unified_loss: run with need_backward=True to differentiate")
    out, clean = ctx.saved_tensors
    return torch.ops.rr.unified_loss_backward(g, out, clean, ctx.handle, ctx.w, ctx.gs), None, \
        None, None, None, None


unified_loss.register_autograd(_uni_bwd, setup_context=_uni_setup)


@torch.library.custom_op("rr::perceptual_loss", mutates_args=(), device_types="cuda")
def perceptual_loss(x: Tensor, y: Tensor, perceptual: int, need_backward: bool) -> Tuple[Tensor, Tensor]:
    """VGGPerceptualLoss.forward (14:194-196)"""
    perc = _module(perceptual)
    loss, S, fx, fy = perc._rr_forward(x, y, 1.0, need_bwd=need_backward)
    return loss, (_stash((S, fx, fy)) if need_backward else _no_state())


@perceptual_loss.register_fake
def _(x, y, perceptual, need_backward):
    return x.new_empty(()), torch.empty((), dtype=torch.int64)


@torch.library.custom_op("rr::perceptual_loss_backward", mutates_args=(), device_types="cuda")
def perceptual_loss_backward(grad: Tensor, handle: Tensor, x: Tensor) -> Tensor:
    """dL/dx of VGGPerceptualLoss; ``x`` is the forward's input (its shape)"""
    S, fx, fy = _unstash(handle)
    gpre = ops.loss_bwd(ops.MSE, fx, fy, gscale=grad.contiguous(), scale=1.0, mask_a_pos=True)
    return engine.vgg_features_backward_input(S, gpre)


@perceptual_loss_backward.register_fake
def _(grad, handle, x):
    return torch.empty_like(x)


def _perc_setup(ctx, inputs, output):
    ctx.handle, ctx.need = output[1], inputs[3]
    ctx.save_for_backward(inputs[0])


def _perc_bwd(ctx, g, g_handle):
    if not ctx.need:
        raise RuntimeError("rr::perceptual_loss: run with need_backward=True to differentiate")
    x, = ctx.saved_tensors
    return torch.ops.rr.perceptual_loss_backward(g, ctx.handle, x), None, None, None


perceptual_loss.register_autograd(_perc_bwd, setup_context=_perc_setup)


# ---------------------------------------------------------------------------
# frozen judge and post-processing

@torch.library.custom_op("rr::vgg16_logits", mutates_args=(), device_types="cuda")
def vgg16_logits(x: Tensor, params: List[Tensor], module: int) -> Tensor:
    """eval-mode VGG16 logits (18:46), the classifier judge"""
    vgg = _module(module)
    logits = engine.vgg_classifier_forward(vgg, x.float().contiguous(), vgg._wc, vgg.compute_dtype)
    return logits if logits.dtype == torch.float32 else logits.float()


@vgg16_logits.register_fake
def _(x, params, module):
    return x.new_empty((x.shape[0], params[-1].shape[0]), dtype=torch.float32)


@torch.library.custom_op("rr::nearest_resize", mutates_args=(), device_types="cuda")
def nearest_resize(x: Tensor, h: int, w: int) -> Tensor:
    """F.interpolate(x, size=(h, w)) mode 'nearest' on NHWC (14:169-182)"""
    return ops.nearest_resize(x.contiguous(), h, w)


@nearest_resize.register_fake
def _(x, h, w):
    return x.new_empty((x.shape[0], h, w, x.shape[3]))


@torch.library.custom_op("rr::to_uint8_hwc", mutates_args=(), device_types="cuda")
def to_uint8_hwc(x: Tensor, bgr: bool = False) -> Tensor:
    """clamp(0, 1) * 255 truncated to uint8, NCHW fp32 -> NHWC, optionally
    RGB -> BGR channel order (17:84-92)"""
    return ops.to_uint8_hwc(x.contiguous(), bgr=bgr)


@to_uint8_hwc.register_fake
def _(x, bgr=False):
    n, c, h, w = x.shape
    return x.new_empty((n, h, w, c), dtype=torch.uint8)


@torch.library.custom_op("rr::psnr_u8", mutates_args=(), device_types="cuda")
def psnr_u8(a: Tensor, b: Tensor) -> Tensor:
    """per-image PSNR over uint8 HWC, data_range 255, fp64 (08:123)"""
    return ops.psnr_u8(a.contiguous(), b.contiguous())


@psnr_u8.register_fake
def _(a, b):
    return a.new_empty((a.shape[0],), dtype=torch.float64)


@torch.library.custom_op("rr::argmax_rows", mutates_args=(), device_types="cuda")
def argmax_rows(logits: Tensor) -> Tensor:
    """torch.max(logits, 1)[1]: first index on ties (18:47)"""
    return ops.argmax_rows(logits.contiguous())


@argmax_rows.register_fake
def _(logits):
    return logits.new_empty((logits.shape[0],), dtype=torch.int64)


OPS = ["resunet_forward", "resunet_backward", "simple_unet_forward", "simple_unet_backward",
       "resblock_forward", "resblock_backward", "pixel_loss", "pixel_loss_backward",
       "unified_loss", "unified_loss_backward", "perceptual_loss", "perceptual_loss_backward",
       "vgg16_logits", "nearest_resize", "to_uint8_hwc", "psnr_u8", "argmax_rows"]
