"""CPU: pin the image-I/O oracle (oracle/imgproc_cpu.py) to the libraries the
reference calls where they are installed here (Pillow for Resize, torch for
ToTensor/Normalize), and check the host-side pieces of the C ABI."""
import ctypes as C

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import imgproc_cpu as I

RESIZE_CASES = [
    (30, 30, 224, 224), (64, 64, 224, 224), (250, 180, 224, 224), (224, 224, 64, 64),
    (37, 53, 64, 64), (15, 17, 224, 224), (300, 41, 224, 224), (64, 64, 64, 32),
    (64, 64, 33, 64), (500, 500, 7, 9), (1, 1, 5, 3), (1, 40, 64, 64), (64, 64, 64, 64),
]


@pytest.mark.parametrize("h,w,oh,ow", RESIZE_CASES)
def test_resize_oracle_matches_pillow(h, w, oh, ow):
    rng = np.random.default_rng(h * 1000 + w)
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
    assert np.array_equal(I.pil_resize_bilinear(img, oh, ow), ref)


def test_resize_oracle_matches_pillow_gray():
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, (45, 33, 1), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(img[..., 0]).resize((224, 224), Image.BILINEAR))
    assert np.array_equal(I.pil_resize_bilinear(img, 224, 224)[..., 0], ref)


def test_to_tensor_normalize_matches_torch():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (20, 24, 3), dtype=np.uint8)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    # torchvision ToTensor: from_numpy.permute.contiguous().to(float).div(255);
    # Normalize: sub_(as_tensor(mean)[:, None, None]).div_(std...)
    t = torch.from_numpy(img).permute(2, 0, 1).contiguous().float().div(255)
    t = t.sub_(torch.as_tensor(mean)[:, None, None]).div_(torch.as_tensor(std)[:, None, None])
    assert np.array_equal(I.to_tensor_normalize(img, mean, std), t.numpy())


def test_ssim_oracle_properties():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (32, 40, 3), dtype=np.uint8)
    b = np.clip(a.astype(int) + rng.integers(-20, 21, a.shape), 0, 255).astype(np.uint8)
    assert I.ssim(a, a) == pytest.approx(1.0, abs=1e-12)
    s = I.ssim(a, b)
    assert 0.0 < s < 1.0
    assert I.ssim(b, a) == pytest.approx(s, abs=1e-12)
    with pytest.raises(ValueError):
        I.ssim(a[:6], b[:6])


def test_filter2d_and_distort_oracle_identities():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (19, 23, 3), dtype=np.uint8)
    one = np.ones((1, 1), np.float32)
    assert np.array_equal(I.filter2d_u8(img, one), img)
    # no distortion: (x / 255 * 255) truncated (a few values drop by one)
    plain = I.distort(img)
    assert np.all(plain <= img) and np.all(img.astype(int) - plain <= 1)
    k = I.motion_blur_kernel(10, 45)
    assert k.dtype == np.float32 and k.shape == (10, 10)
    assert 0.5 < float(k.sum()) <= 1.0 + 1e-6


def test_distort_param_layout():
    from roadrestore._lib import DistortParam
    assert C.sizeof(DistortParam) == 24
    assert [DistortParam.sigma.offset, DistortParam.fog_mul.offset, DistortParam.fog_add.offset,
            DistortParam.flags.offset, DistortParam.ksize.offset] == [0, 8, 12, 16, 20]


def test_motion_blur_kernel_host_abi_matches_oracle():
    """rr_motion_blur_kernel is host code (no GPU): every (degree, angle)
    the reference can draw (14:53-54 randint(5, 15), randint(0, 360)) plus
    the compound kernel (10, 45)."""
    import roadrestore
    lib = roadrestore.lib()
    buf = (C.c_float * 225)()
    for k in range(5, 16):
        for ang in range(0, 361, 7):
            assert lib.rr_motion_blur_kernel(k, ang, C.cast(buf, C.c_void_p)) == 0
            got = np.frombuffer(buf, np.float32).reshape(15, 15)
            assert np.array_equal(got[:k, :k], I.motion_blur_kernel(k, ang)), (k, ang)
            assert not got[k:, :].any() and not got[:, k:].any()
    assert lib.rr_motion_blur_kernel(16, 0, C.cast(buf, C.c_void_p)) == -1


def test_imgproc_workspace_queries():
    import roadrestore
    lib = roadrestore.lib()
    assert lib.rr_resize_workspace(4, 30, 30, 3, 224, 224) > 4 * 30 * 224 * 3
    assert lib.rr_resize_workspace(1, 30, 30, 5, 224, 224) == 0        # c > 4
    assert lib.rr_ssim_workspace(8, 3) == 8 * 3 * 8
    assert lib.rr_distort_workspace(2, 64, 64, 3) == 2 * 64 * 64 * 3


def test_distortion_params_follow_reference_draw_order():
    """imgproc.distortion_params draws exactly what 14:36-58 draws, in the
    same order, from the same Python `random` stream (host logic, no GPU)"""
    import random
    from roadrestore import imgproc
    from roadrestore._lib import RR_DISTORT_BLUR, RR_DISTORT_FOG, RR_DISTORT_NOISE
    n = 64
    params, taps = imgproc.distortion_params(n, random.Random(123))
    rng = random.Random(123)
    seen = set()
    for i in range(n):
        p = params[i]
        fog = rng.random() < 0.5
        if fog:
            intensity = rng.uniform(0.3, 0.7)
            t = 1.0 - intensity * rng.uniform(0.8, 1.2)
            assert p.fog_mul == np.float32(t) and p.fog_add == np.float32(0.9 * (1 - t))
        noise = rng.random() < 0.5
        if noise:
            assert p.sigma == rng.uniform(0.01, 0.03) ** 0.5
        blur = rng.random() < 0.5
        if blur:
            degree, angle = rng.randint(5, 15), rng.randint(0, 360)
            assert p.ksize == degree
            assert np.array_equal(taps[i][:degree, :degree].numpy(), I.motion_blur_kernel(degree, angle))
        else:
            assert not taps[i].any()
        assert bool(p.flags & RR_DISTORT_FOG) == fog
        assert bool(p.flags & RR_DISTORT_NOISE) == noise
        assert bool(p.flags & RR_DISTORT_BLUR) == blur
        seen.add((fog, noise, blur))
    assert len(seen) == 8                                    # every branch combination drawn


@pytest.mark.parametrize("shape", [(3, 64, 64, 3), (2, 224, 224, 3), (1, 37, 53, 3), (2, 5, 7, 1)])
def test_png_writer_roundtrip(tmp_path, shape):
    """17:89-99: the restored uint8 images written as PNG (host-side batched
    encoder in libroadrestore.so, no device needed) decode with Pillow to
    exactly the same pixels; cv2.imwrite of the BGR-swapped array stores the
    RGB pixels, so the files carry the RGB buffer."""
    import numpy as np
    from PIL import Image
    from roadrestore import imgproc
    g = np.random.default_rng(sum(shape))
    u8 = g.integers(0, 256, size=shape, dtype=np.uint8)
    u8[0, : shape[1] // 2] = 17                     # flat region: exercises the filters
    t = torch.from_numpy(u8)
    paths = [tmp_path / "sub" / f"img{i}.png" for i in range(shape[0])]
    imgproc.write_png(t, paths, level=1, threads=2)
    for i, p in enumerate(paths):
        with Image.open(p) as im:
            got = np.asarray(im)
        ref = u8[i, ..., 0] if shape[-1] == 1 else u8[i]
        assert got.shape == ref.shape and np.array_equal(got, ref)
    # single-image encoder: same bytes as the batch writer's file
    assert imgproc.encode_png(t[0], level=1) == paths[0].read_bytes()
