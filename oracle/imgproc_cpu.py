"""CPU restatement of the image I/O around the networks -- TEST INFRASTRUCTURE
ONLY.

Only ``tests/`` (and ``bench.py``'s ``cpu_baseline`` leg) may import this
module, as the checker.  The product (``roadrestore``) never imports it.

* ``pil_resize_bilinear``  torchvision ``Resize((oh, ow))`` on a PIL image
  (17_run_unified_inference.py:66, 18_test_unified_benchmark.py:28-32), which
  is ``PIL.Image.resize(size, BILINEAR)``: Pillow's ``ImagingResample``
  (src/libImaging/Resample.c: ``precompute_coeffs``,
  ``normalize_coeffs_8bpc``, ``ImagingResampleHorizontal_8bpc`` /
  ``Vertical_8bpc``, ``ImagingResampleInner``).  Restated in numpy; pinned
  against the installed Pillow itself (tests/test_imgproc_cpu.py).
* ``cv_resize_linear``     ``cv2.resize(img, (224, 224))`` (default
  ``INTER_LINEAR``) on the uint8 clean image of the 08 PSNR leg
  (08_run_inference.py:118-119) -- OpenCV's OWN algorithm, not Pillow's:
  OpenCV 4.x ``imgproc/src/resize.cpp`` ``hal::resize`` -> ``resizeGeneric_``
  with ``HResizeLinear<uchar, int, short, 2048>`` and ``VResizeLinear<uchar,
  int, short, FixedPtCast<int, uchar, 22>>``: float source coordinates
  ``(d + 0.5) * scale - 0.5`` with ``scale = 1 / (dst / src)`` in double,
  border clamping, 11-bit coefficients ``saturate_cast<short>(c * 2048)``
  (round half to even), an exact int32 horizontal pass, and the vertical
  pass as the x86 SIMD body ``VResizeLinearVec_32s8u`` computes it
  (``((S0 >> 4) * b0 >> 16) + ((S1 >> 4) * b1 >> 16)``, then ``(v + 2) >> 2``
  saturated) for the elements it covers, the scalar ``(v + 2^21) >> 22`` for
  the row tail.  cv2 is not installed here: **parity vs cv2 is unpinned**
  (the IPP path, off by default for non-exact resizes, and other SIMD
  widths are not reproduced; at 224 x 3 = 672 row elements the scalar tail
  is empty for 16- and 32-lane vectors).
* ``to_tensor_normalize``  ``ToTensor`` (``.float().div(255)``) and
  ``Normalize`` (``sub_(mean).div_(std)``, fp32) (18:29-31).
* ``ssim``                 skimage ``structural_similarity(a, b,
  data_range=255, channel_axis=2)`` (08_run_inference.py:125): skimage is not
  installed here, so this restates its published algorithm (uniform 7x7
  window via ``scipy.ndimage.uniform_filter`` as skimage calls it, sample
  covariance, K1 .01, K2 .03, 3-pixel crop, per-channel mean).  Parity vs
  skimage itself is unpinned (no skimage, no reference fixture holds SSIM).
* ``distort``              the dynamic distortion generator 14:31-64 and the
  fixed compound variant 16:14-37 (fog, Gaussian noise, motion blur).  The
  random draws are inputs (the noise field and per-image parameters), so the
  arithmetic is checked bit-exactly; see that function for what of cv2 is
  restated and what is unpinned.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _precompute_coeffs(in_size: int, out_size: int):
    """Pillow precompute_coeffs (support 1.0, bilinear filter) followed by
    normalize_coeffs_8bpc: -> bounds [out][2] (xmin, count), kk [out][ksize]
    int64 fixed point."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = []
        ww = 0.0
        for x in range(xmax):
            t = abs((float(x + xmin) - center + 0.5) * ss)
            w = 1.0 - t if t < 1.0 else 0.0
            k.append(w)
            ww += w
        for x in range(xmax):
            v = k[x] / ww if ww != 0.0 else k[x]
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else \
                int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(s):
    return np.clip(s >> PRECISION_BITS, 0, 255).astype(np.uint8)


def _pass(img, bounds, kk, axis):
    """one 8bpc pass along ``axis`` (1 = horizontal, 0 = vertical) of a
    [H, W, C] uint8 image"""
    src = np.moveaxis(img.astype(np.int64), axis, 0)          # [in, other, C]
    out = np.empty((bounds.shape[0],) + src.shape[1:], np.int64)
    for o, (xmin, cnt) in enumerate(bounds):
        s = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for x in range(cnt):
            s += src[xmin + x] * kk[o, x]
        out[o] = s
    return np.moveaxis(_clip8(out), 0, axis)


def pil_resize_bilinear(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """[H, W, C] uint8 -> [oh, ow, C] uint8, as PIL Image.resize((ow, oh),
    Image.BILINEAR).  ImagingResampleInner: horizontal pass first over source
    rows [ybox_first, ybox_last), then the vertical pass with bounds shifted by
    ybox_first; a pass is skipped when its size is unchanged."""
    h, w = img.shape[:2]
    if (h, w) == (oh, ow):
        return img.copy()                                     # Image.resize: self.copy()
    bh, kh = _precompute_coeffs(w, ow)
    bv, kv = _precompute_coeffs(h, oh)
    out = img
    if ow != w:
        y0, y1 = bv[0, 0], bv[-1, 0] + bv[-1, 1]
        out = _pass(img[y0:y1], bh, kh, axis=1)
        bv = bv.copy()
        bv[:, 0] -= y0
    if oh != h:
        out = _pass(out, bv, kv, axis=0)
    return out


CV_COEF_BITS = 11
CV_COEF_SCALE = 1 << CV_COEF_BITS


def _cv_linear_coeffs(src: int, dst: int):
    """resize.cpp's per-output source index and 11-bit weights (xofs / ialpha,
    yofs / ibeta): (index [dst] int64, w0 [dst] int64, w1 [dst] int64).  The x
    axis clamps the index and zeroes the fraction at the borders; the y axis
    keeps the raw index (rows are clamped when fetched) and its weights."""
    scale = 1.0 / (float(dst) / float(src))          # hal::resize: 1. / inv_scale
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)  # (float)((dx+0.5)*scale_x - 0.5)
    i = np.floor(f).astype(np.int64)                  # cvFloor
    f = (f - i.astype(np.float32)).astype(np.float32)
    return i, f


def _cv_round_short(v: np.ndarray) -> np.ndarray:
    return np.rint(v.astype(np.float32)).astype(np.int64)   # cvRound: half to even


def cv_resize_linear(img: np.ndarray, oh: int, ow: int, simd_lanes: int = 16) -> np.ndarray:
    """[H, W, C] uint8 -> [oh, ow, C] uint8 as cv2.resize(img, (ow, oh))
    (INTER_LINEAR); see the module docstring.  ``simd_lanes``: the u8 vector
    width of the vertical pass (16 = SSE2/NEON baseline)."""
    h, w, cn = img.shape
    if (h, w) == (oh, ow):
        return img.copy()                                # cv::resize: same size -> copy
    sx, fx = _cv_linear_coeffs(w, ow)
    lo, hi = sx < 0, sx >= w - 1
    fx = np.where(lo | hi, np.float32(0), fx).astype(np.float32)
    sx = np.where(lo, 0, np.where(hi, w - 1, sx))
    a0 = _cv_round_short((np.float32(1) - fx) * np.float32(CV_COEF_SCALE))
    a1 = _cv_round_short(fx * np.float32(CV_COEF_SCALE))
    sx1 = np.minimum(sx + 1, w - 1)                      # weight 0 where clamped
    src = img.astype(np.int64)
    # horizontal: D[y][dx][c] = S[y][sx][c] * a0 + S[y][sx + 1][c] * a1 (int32)
    hz = src[:, sx, :] * a0[None, :, None] + src[:, sx1, :] * a1[None, :, None]
    sy, fy = _cv_linear_coeffs(h, oh)
    b0 = _cv_round_short((np.float32(1) - fy) * np.float32(CV_COEF_SCALE))
    b1 = _cv_round_short(fy * np.float32(CV_COEF_SCALE))
    r0 = np.clip(sy, 0, h - 1)
    r1 = np.clip(sy + 1, 0, h - 1)
    s0 = hz[r0].reshape(oh, ow * cn)
    s1 = hz[r1].reshape(oh, ow * cn)
    b0c, b1c = b0[:, None], b1[:, None]
    # VResizeLinearVec_32s8u: 16-bit fixed point (v_mul_hi = (a * b) >> 16)
    vec = ((((s0 >> 4) * b0c) >> 16) + (((s1 >> 4) * b1c) >> 16) + 2) >> 2
    # scalar tail: FixedPtCast<int, uchar, 22>
    sca = (s0 * b0c + s1 * b1c + (1 << 21)) >> 22
    width = ow * cn
    x = np.arange(width)
    nv = (width // simd_lanes) * simd_lanes              # x <= width - lanes loop
    half = simd_lanes // 2
    while nv < width - half:                             # x < width - lanes/2 loop
        nv += half
    out = np.where(x[None, :] < nv, vec, sca)
    return np.clip(out, 0, 255).astype(np.uint8).reshape(oh, ow, cn)


def to_tensor_normalize(img_u8: np.ndarray, mean=None, std=None) -> np.ndarray:
    """[H, W, C] uint8 -> [C, H, W] float32: ToTensor then Normalize, fp32."""
    x = np.transpose(img_u8, (2, 0, 1)).astype(np.float32) / np.float32(255)
    if mean is not None:
        m = np.asarray(mean, np.float32)[:, None, None]
        s = np.asarray(std, np.float32)[:, None, None]
        x = (x - m) / s
    return x


def ssim(a: np.ndarray, b: np.ndarray, data_range: float = 255.0) -> float:
    """skimage structural_similarity(a, b, data_range, channel_axis=2) for
    [H, W, C] uint8 images (defaults: win_size 7, uniform window,
    use_sample_covariance, K1 0.01, K2 0.03)."""
    from scipy.ndimage import uniform_filter
    win, K1, K2 = 7, 0.01, 0.03
    if min(a.shape[:2]) < win:
        raise ValueError("win_size exceeds image extent")
    res = []
    for ch in range(a.shape[2]):
        x = a[..., ch].astype(np.float64)
        y = b[..., ch].astype(np.float64)
        NP = win ** 2
        cov_norm = NP / (NP - 1)
        ux = uniform_filter(x, size=win)
        uy = uniform_filter(y, size=win)
        uxx = uniform_filter(x * x, size=win)
        uyy = uniform_filter(y * y, size=win)
        uxy = uniform_filter(x * y, size=win)
        vx = cov_norm * (uxx - ux * ux)
        vy = cov_norm * (uyy - uy * uy)
        vxy = cov_norm * (uxy - ux * uy)
        C1 = (K1 * data_range) ** 2
        C2 = (K2 * data_range) ** 2
        A1, A2 = 2 * ux * uy + C1, 2 * vxy + C2
        B1, B2 = ux ** 2 + uy ** 2 + C1, vx + vy + C2
        S = (A1 * A2) / (B1 * B2)
        pad = (win - 1) // 2
        res.append(S[pad:-pad, pad:-pad].mean(dtype=np.float64))
    return float(np.mean(res))


# ------------------------------------------------------------ distortion ----
KMAX = 15


def motion_blur_kernel(degree: int, angle: int) -> np.ndarray:
    """14:55-59 / 16:20-21: cv2.getRotationMatrix2D((d/2, d/2), angle, 1),
    cv2.warpAffine(np.diag(np.ones(d)), M, (d, d)), / d -- restated (cv2 is
    absent here): OpenCV getRotationMatrix2D (center as Point2f), warpAffine's
    matrix inversion, WarpAffineInvoker's 10-bit fixed-point coordinates
    (cvRound = half to even, +16 round delta, >> 5), remapBilinear over the
    1/32-pixel table of fp32 weights with BORDER_CONSTANT 0, the division by
    d in fp64, and filter2D's conversion of the kernel to fp32.  Returns the
    [d, d] float32 taps."""
    k = degree
    cx = cy = float(np.float32(k / 2))
    a = angle * math.pi / 180.0
    alpha, beta = math.cos(a) * 1.0, math.sin(a) * 1.0
    M = [alpha, beta, (1 - alpha) * cx - beta * cy, -beta, alpha, beta * cx + (1 - alpha) * cy]
    D = M[0] * M[4] - M[1] * M[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = M[4] * D, M[0] * D
    M[0] = A11
    M[1] *= -D
    M[3] *= -D
    M[4] = A22
    b1 = -M[0] * M[2] - M[1] * M[5]
    b2 = -M[3] * M[2] - M[4] * M[5]
    M[2], M[5] = b1, b2
    rnd = lambda v: int(np.rint(v))                                  # noqa: E731
    t1 = [(np.float32(1) - np.float32(i) * np.float32(1 / 32), np.float32(i) * np.float32(1 / 32))
          for i in range(32)]
    src = np.eye(k)
    out = np.zeros((k, k), np.float64)
    for y in range(k):
        for x in range(k):
            X0 = rnd((M[1] * y + M[2]) * 1024) + 16
            Y0 = rnd((M[4] * y + M[5]) * 1024) + 16
            X = (X0 + rnd(M[0] * x * 1024)) >> 5
            Y = (Y0 + rnd(M[3] * x * 1024)) >> 5
            sx, sy, fx, fy = X >> 5, Y >> 5, X & 31, Y & 31
            w = [float(t1[fy][0] * t1[fx][0]), float(t1[fy][0] * t1[fx][1]),
                 float(t1[fy][1] * t1[fx][0]), float(t1[fy][1] * t1[fx][1])]

            def s(xx, yy):
                return src[yy, xx] if 0 <= xx < k and 0 <= yy < k else 0.0
            if sx >= k or sx + 1 < 0 or sy >= k or sy + 1 < 0:
                v = 0.0
            else:
                v = s(sx, sy) * w[0] + s(sx + 1, sy) * w[1] + s(sx, sy + 1) * w[2] + s(sx + 1, sy + 1) * w[3]
            out[y, x] = v
    return (out / k).astype(np.float32)


def _reflect101(p, n):
    if n == 1:
        return 0
    while p < 0 or p >= n:
        p = -p if p < 0 else 2 * n - 2 - p
    return p


def filter2d_u8(img: np.ndarray, kern: np.ndarray) -> np.ndarray:
    """cv2.filter2D(img, -1, kern) for uint8 [H, W, C] and an fp32 kernel:
    anchor (k/2, k/2), BORDER_REFLECT_101, fp32 accumulation over the nonzero
    taps in row-major order (OpenCV Filter2D with preprocess2DKernel), then
    saturate_cast<uchar> (round half to even).  OpenCV switches to a DFT
    correlation for kernels of >= 130 taps on SSE3 builds (degree >= 12) and
    may fuse the multiply-add in its SIMD path; those can differ by one level
    from this direct form -- unpinned (cv2 is absent here)."""
    h, w, c = img.shape
    kh, kw = kern.shape
    ay, ax = kh // 2, kw // 2
    ys = np.array([[_reflect101(y + i - ay, h) for y in range(h)] for i in range(kh)])
    xs = np.array([[_reflect101(x + j - ax, w) for x in range(w)] for j in range(kw)])
    s = np.zeros((h, w, c), np.float32)
    src = img.astype(np.float32)
    for i in range(kh):
        for j in range(kw):
            kv = np.float32(kern[i, j])
            if kv == 0:
                continue
            s = (s + kv * src[ys[i]][:, xs[j]]).astype(np.float32)
    return np.clip(np.rint(s), 0, 255).astype(np.uint8)


def _trunc_u8(x):
    return np.clip(x * 255, 0, 255).astype(np.uint8)


def distort(img: np.ndarray, fog_t=None, noise=None, blur=None, A=0.9) -> np.ndarray:
    """apply_random_distortions 14:31-64 with its random draws as arguments:
    fog_t = t (1 - intensity * U(.8, 1.2)) or None; noise = the float64 noise
    field or None; blur = (degree, angle) or None.  numpy dtype semantics of
    the reference: fp32 image, fog in fp32 with the Python scalars cast to
    fp32, noise promotes to fp64, uint8 truncation."""
    out = img.astype(np.float32) / np.float32(255.0)
    if fog_t is not None:
        out = out * np.float32(fog_t) + np.float32(A * (1 - fog_t))
    if noise is not None:
        out = out + noise
    if blur is not None:
        temp = _trunc_u8(out)
        temp = filter2d_u8(temp, motion_blur_kernel(*blur))
        out = temp.astype(np.float32) / np.float32(255.0)
    return _trunc_u8(out)


def compound(img: np.ndarray, noise: np.ndarray, degree=10, angle=45, intensity=0.5, A=0.9):
    """apply_compound_distortion 16:14-37: blur -> fog -> noise."""
    x = img.astype(np.float32) / np.float32(255.0)
    temp = (x * np.float32(255)).astype(np.uint8)
    temp = filter2d_u8(temp, motion_blur_kernel(degree, angle))
    x = temp.astype(np.float32) / np.float32(255.0)
    t = 1.0 - intensity
    x = x * np.float32(t) + np.float32(A * (1 - t))
    x = x + noise
    return _trunc_u8(x)
