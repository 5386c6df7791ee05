"""Device-batched image I/O around the networks.

The reference runs these per image on the host (cv2 / PIL / skimage in
DataLoader workers and in the inference loop).  Here they take a whole
[n, h, w, c] uint8 batch resident on the GPU and run as HIP kernels
(csrc/imgproc.hip) behind the C ABI:

* ``Resize`` / ``ToTensor`` / ``Normalize`` / ``Compose`` -- torchvision's
  transform names and argument meaning (17:66, 18:28-32); ``Resize`` is
  PIL's bilinear resample bit for bit, and ``Compose([Resize, ToTensor,
  Normalize])`` runs as one fused pass.
* ``apply_random_distortions`` -- 14:31-64, the per-image random draws made
  with Python's ``random`` in the reference's order, the noise field drawn on
  device (Philox4x32-10) instead of ``np.random.normal``.
* ``apply_compound_distortion`` -- 16:14-37 (blur 10 @ 45 deg, fog 0.5, noise
  var 0.02).
* ``cv_resize`` -- ``cv2.resize(img, (224, 224))`` of the 08 PSNR leg's
  clean image (08:118-119): OpenCV's INTER_LINEAR, which is not PIL's.
* ``psnr`` / ``ssim`` -- 08:123-125 (skimage semantics, data_range 255).
"""
from __future__ import annotations

import ctypes as C
import os
import random as _random

import torch

from . import ops
from ._lib import (RR_DISTORT_BLUR, RR_DISTORT_FOG, RR_DISTORT_KMAX, RR_DISTORT_NOISE,
                   DistortParam, lib)

__all__ = ["Resize", "ToTensor", "Normalize", "Compose", "apply_random_distortions",
           "encode_png", "write_png",
           "RandomDistortion", "motion_blur_table",
           "apply_compound_distortion", "distortion_params", "psnr", "ssim", "cv_resize",
           "IMAGENET_MEAN", "IMAGENET_STD"]

IMAGENET_MEAN = (0.485, 0.456, 0.406)      # 18:31
IMAGENET_STD = (0.229, 0.224, 0.225)

# 14:23-25
PROB_NOISE = 0.5
PROB_BLUR = 0.5
PROB_FOG = 0.5


def _check_u8(x):
    if not isinstance(x, torch.Tensor) or x.dtype != torch.uint8 or x.dim() != 4:
        raise TypeError("expected a [n, h, w, c] uint8 device batch")


class Resize:
    """torchvision ``Resize((h, w))`` on PIL images (bilinear): u8 -> u8."""

    def __init__(self, size):
        if isinstance(size, int):
            raise NotImplementedError("Resize(int) (aspect-preserving) is not used by the reference")
        self.size = (int(size[0]), int(size[1]))

    def __call__(self, x):
        _check_u8(x)
        return ops.resize_bilinear_u8(x, self.size[0], self.size[1], out="u8")


class ToTensor:
    """u8 [n, h, w, c] -> fp32 [n, c, h, w] / 255."""

    def __call__(self, x):
        _check_u8(x)
        n, h, w, c = x.shape
        return ops.resize_bilinear_u8(x, h, w, out="f32")


class Normalize:
    """``(x - mean) / std`` per channel in fp32 (torchvision's
    ``sub_().div_()``).  It runs fused into the resample pass of
    ``Compose([Resize, ToTensor, Normalize])`` -- the only way the reference
    uses it (18:28-32); on its own it raises rather than fall back to ATen."""

    def __init__(self, mean, std):
        self.mean, self.std = tuple(mean), tuple(std)

    def __call__(self, x):
        raise NotImplementedError("Normalize runs fused: Compose([Resize(...), ToTensor(), "
                                  "Normalize(...)])")


class Compose:
    """Sequential transforms; ``[Resize, ToTensor]`` and ``[Resize, ToTensor,
    Normalize]`` prefixes fuse into one resample pass writing fp32 NCHW."""

    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, x):
        t = self.transforms
        i = 0
        if len(t) >= 2 and isinstance(t[0], Resize) and isinstance(t[1], ToTensor):
            mean = std = None
            i = 2
            if len(t) >= 3 and isinstance(t[2], Normalize):
                mean, std = t[2].mean, t[2].std
                i = 3
            _check_u8(x)
            x = ops.resize_bilinear_u8(x, t[0].size[0], t[0].size[1], out="f32", mean=mean, std=std)
        for tr in t[i:]:
            x = tr(x)
        return x


def distortion_params(n, rng=None):
    """Per-image draws of apply_random_distortions (14:36-58) in the
    reference's order with Python's ``random``: -> (params, taps [n, K, K])."""
    rng = rng or _random
    params, taps = [], torch.zeros(n, RR_DISTORT_KMAX, RR_DISTORT_KMAX)
    for i in range(n):
        p = DistortParam(0.0, 1.0, 0.0, 0, 0)
        if rng.random() < PROB_FOG:
            intensity = rng.uniform(0.3, 0.7)
            A = 0.9
            t = 1.0 - intensity * rng.uniform(0.8, 1.2)
            p.flags |= RR_DISTORT_FOG
            p.fog_mul, p.fog_add = t, A * (1 - t)          # stored as fp32, as numpy casts them
        if rng.random() < PROB_NOISE:
            var = rng.uniform(0.01, 0.03)
            p.flags |= RR_DISTORT_NOISE
            p.sigma = var ** 0.5
        if rng.random() < PROB_BLUR:
            degree = rng.randint(5, 15)
            angle = rng.randint(0, 360)
            if degree > 1:
                p.flags |= RR_DISTORT_BLUR
                p.ksize = degree
                taps[i] = ops.motion_blur_kernel(degree, angle)
        params.append(p)
    return params, taps


def apply_random_distortions(x, rng=None, seed=None, noise=None):
    """14:31-64 on a [n, h, w, c] uint8 device batch."""
    _check_u8(x)
    params, taps = distortion_params(x.shape[0], rng)
    if seed is None:
        seed = (rng or _random).getrandbits(64)
    return ops.distort_u8(x, params, taps, mode=0, noise=noise, seed=seed)


_TABLES = {}


def motion_blur_table(device):
    """Device copy of every motion-blur kernel the draws can pick (degree
    5..15 x angle 0..360, [11, 361, KMAX, KMAX] fp32), built once on the host
    by the same restatement of cv2 getRotationMatrix2D + warpAffine."""
    key = str(device)
    t = _TABLES.get(key)
    if t is None:
        import ctypes as C
        L = ops.lib()
        nf = L.rr_motion_blur_table_floats()
        host = torch.empty(nf, dtype=torch.float32)
        L.check(L.rr_motion_blur_table(C.c_void_p(host.data_ptr())), "rr_motion_blur_table")
        t = _TABLES[key] = host.view(11, 361, RR_DISTORT_KMAX, RR_DISTORT_KMAX).to(device)
    return t


class RandomDistortion:
    """apply_random_distortions (14:31-64) for a whole [n, h, w, c] uint8
    device batch with the per-image draws made ON DEVICE
    (rr_distort_random_u8): graph-capturable, so a captured training step
    re-draws on every replay.  The draws follow the reference's distributions
    (Philox4x32-10 keyed by (seed, step); the reference's stream is unseeded);
    the step counter lives in device memory and advances once per call.

    ``last_draws()`` reads the most recent draws back (tests)."""

    def __init__(self, device, seed=0):
        self.device = torch.device(device)
        self.seed = int(seed) & (2 ** 64 - 1)
        self.step = torch.zeros((), dtype=torch.int64, device=self.device)
        self.table = motion_blur_table(self.device)
        self._ws = None
        self._shape = None

    def __call__(self, x, out=None):
        _check_u8(x)
        ops._need_cuda(x)
        n, h, w, c = x.shape
        x = x.contiguous()
        L = ops.lib()
        if self._ws is None or self._shape != (n, h, w, c):
            self._ws = ops._ws(L.rr_distort_random_workspace(n, h, w, c), self.device)
            self._shape = (n, h, w, c)
        if out is None:
            out = torch.empty_like(x)
        L.check(L.rr_distort_random_u8(n, h, w, c, x.data_ptr(), out.data_ptr(), self.seed,
                                       self.step.data_ptr(), self.table.data_ptr(),
                                       self._ws.data_ptr(), self._ws.numel(), ops.stream()),
                "rr_distort_random_u8")
        return out

    def last_draws(self):
        """-> (params: list of DistortParam, table index [n] int32, noise seed)"""
        import ctypes as C
        n, h, w, c = self._shape
        po, io, so = C.c_size_t(), C.c_size_t(), C.c_size_t()
        L = ops.lib()
        L.check(L.rr_distort_random_draws(n, h, w, c, self._ws.data_ptr(), C.byref(po), C.byref(io),
                                          C.byref(so)), "rr_distort_random_draws")
        raw = self._ws.cpu()
        sz = C.sizeof(DistortParam)
        arr = (DistortParam * n).from_buffer_copy(bytes(raw[po.value:po.value + n * sz].numpy()))
        idx = raw[io.value:io.value + 4 * n].view(torch.int32).clone()
        seed = int(raw[so.value:so.value + 8].view(torch.int64).item()) & (2 ** 64 - 1)
        return list(arr), idx, seed


def apply_compound_distortion(x, seed=0, noise=None):
    """16:14-37 on a [n, h, w, c] uint8 device batch: blur (10, 45 deg) ->
    fog (intensity 0.5, A 0.9) -> noise (var 0.02)."""
    _check_u8(x)
    n = x.shape[0]
    t, A = 1.0 - 0.5, 0.9
    p = DistortParam(0.02 ** 0.5, t, A * (1 - t), RR_DISTORT_FOG | RR_DISTORT_NOISE | RR_DISTORT_BLUR, 10)
    taps = ops.motion_blur_kernel(10, 45).unsqueeze(0).expand(n, -1, -1).contiguous()
    return ops.distort_u8(x, [p] * n, taps, mode=1, noise=noise, seed=seed)


def cv_resize(x, size):
    """``cv2.resize(img, (w, h))`` (default INTER_LINEAR) of an [n, h, w, c]
    uint8 device batch (c <= 4): the clean image of the 08 PSNR leg
    (08:118-119; OpenCV's fixed-point bilinear, not PIL's, see
    rr_cv_resize_linear_u8).  ``size`` = (w, h) in cv2's order."""
    _check_u8(x)
    ow, oh = size
    n, h, w, c = x.shape
    x = x.contiguous()
    out = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
    lib().check(lib().rr_cv_resize_linear_u8(n, h, w, c, oh, ow, x.data_ptr(), out.data_ptr(),
                                              0, ops.stream()), "rr_cv_resize_linear_u8")
    return out


def psnr(a, b):
    """per-image PSNR (08:123, data_range 255) of [n, h, w, c] uint8 batches"""
    return ops.psnr_u8(a, b)


def ssim(a, b):
    """per-image SSIM (08:125, data_range 255, channel_axis=2)"""
    return ops.ssim_u8(a, b)


# ---------------------------------------------------------------------------
# PNG output (17:89-99)

def _host_u8(images):
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] not in (1, 3):
        raise ValueError("expected an [n, h, w, 1|3] uint8 tensor (rr_to_uint8_hwc layout)")
    return images.contiguous().cpu() if images.is_cuda else images.contiguous()


def encode_png(image, level=1):
    """One [h, w, c] uint8 RGB (or greyscale) image -> PNG bytes."""
    if image.dim() == 3:
        image = image.unsqueeze(0)
    host = _host_u8(image)
    _, h, w, c = host.shape
    need = lib().rr_png_encode(h, w, c, host.data_ptr(), int(level), None, 0)
    if need < 0:
        lib().check(int(need), "rr_png_encode")
    buf = (C.c_uint8 * need)()
    got = lib().rr_png_encode(h, w, c, host.data_ptr(), int(level), C.addressof(buf), need)
    if got != need:
        lib().check(int(got) if got < 0 else -1, "rr_png_encode")
    return bytes(buf)


def write_png(images, paths, level=1, threads=0):
    """Batched PNG writer for restored images (17:89-99).  ``images``: the
    [n, h, w, 3] uint8 RGB batch of ops.to_uint8_hwc (device or host).  The
    reference swaps to BGR and calls cv2.imwrite, which writes the RGB pixels
    back out; the files here hold the same RGB pixels.  Parent directories are
    created (17:96)."""
    host = _host_u8(images)
    n, h, w, c = host.shape
    paths = [os.fspath(p) for p in paths]
    if len(paths) != n:
        raise ValueError(f"{n} images, {len(paths)} paths")
    for p in paths:
        d = os.path.dirname(p)
        if d:
            os.makedirs(d, exist_ok=True)
    arr = (C.c_char_p * max(n, 1))(*[p.encode() for p in paths])
    lib().check(lib().rr_png_write_batch(n, h, w, c, host.data_ptr(), C.cast(arr, C.c_void_p),
                                         int(level), int(threads)), "rr_png_write_batch")
