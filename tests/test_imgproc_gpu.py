"""GPU parity of the image-I/O kernels (csrc/imgproc.hip) against the CPU
oracle (oracle/imgproc_cpu.py, itself pinned to Pillow in
test_imgproc_cpu.py): bit-exact for the uint8 / fixed-point work, fp32
ToTensor/Normalize bit-exact, SSIM within 1e-10 (exact integer window sums
here vs scipy's running fp64 sums in the restatement)."""
import random

import numpy as np
import pytest
import torch

from oracle import imgproc_cpu as I
from rrpath import set_path  # noqa: E402

pytestmark = pytest.mark.gpu


def _batch(n, h, w, c=3, seed=0):
    return np.random.default_rng(seed).integers(0, 256, (n, h, w, c), dtype=np.uint8)


@pytest.mark.parametrize("h,w,oh,ow", [
    (30, 30, 224, 224), (250, 180, 224, 224), (224, 224, 64, 64), (37, 53, 64, 64),
    (300, 41, 224, 224), (64, 64, 64, 32), (64, 64, 33, 64), (500, 500, 7, 9), (1, 1, 5, 3),
    (64, 64, 64, 64)])
def test_resize_u8_bit_exact(dev, h, w, oh, ow):
    from roadrestore import ops
    x = _batch(3, h, w, seed=h + w)
    y = ops.resize_bilinear_u8(torch.from_numpy(x).to(dev), oh, ow).cpu().numpy()
    for i in range(3):
        assert np.array_equal(y[i], I.pil_resize_bilinear(x[i], oh, ow)), i


@pytest.mark.parametrize("c", [1, 4])
def test_resize_channels(dev, c):
    from roadrestore import ops
    x = _batch(2, 45, 33, c, seed=c)
    y = ops.resize_bilinear_u8(torch.from_numpy(x).to(dev), 224, 100).cpu().numpy()
    for i in range(2):
        assert np.array_equal(y[i], I.pil_resize_bilinear(x[i], 224, 100))


def test_compose_resize_totensor_normalize_bit_exact(dev):
    """18:28-32: Resize((224,224)) + ToTensor + Normalize(ImageNet) fused"""
    import roadrestore as rr
    T = rr.imgproc
    x = _batch(4, 48, 61, seed=9)
    tf = T.Compose([T.Resize((224, 224)), T.ToTensor(), T.Normalize(T.IMAGENET_MEAN, T.IMAGENET_STD)])
    y = tf(torch.from_numpy(x).to(dev)).cpu().numpy()
    assert y.shape == (4, 3, 224, 224) and y.dtype == np.float32
    for i in range(4):
        ref = I.to_tensor_normalize(I.pil_resize_bilinear(x[i], 224, 224), T.IMAGENET_MEAN, T.IMAGENET_STD)
        assert np.array_equal(y[i], ref), i
    # 17:66: Resize + ToTensor only
    y2 = T.Compose([T.Resize((64, 64)), T.ToTensor()])(torch.from_numpy(x).to(dev)).cpu().numpy()
    for i in range(4):
        assert np.array_equal(y2[i], I.to_tensor_normalize(I.pil_resize_bilinear(x[i], 64, 64)))
    # same size (the bench's ToTensor at 64x64): Pillow returns a copy -> the
    # single-pass copy / ToTensor (+ Normalize) path
    x3 = _batch(3, 64, 64, seed=10)
    for norm in (False, True):
        ops_ = [T.Resize((64, 64)), T.ToTensor()] + ([T.Normalize(T.IMAGENET_MEAN, T.IMAGENET_STD)] if norm else [])
        y3 = T.Compose(ops_)(torch.from_numpy(x3).to(dev)).cpu().numpy()
        for i in range(3):
            ref = I.pil_resize_bilinear(x3[i], 64, 64)
            assert np.array_equal(ref, x3[i])
            want = I.to_tensor_normalize(ref, T.IMAGENET_MEAN, T.IMAGENET_STD) if norm else I.to_tensor_normalize(ref)
            assert np.array_equal(y3[i], want), (norm, i)
    with pytest.raises(NotImplementedError):
        T.Normalize(T.IMAGENET_MEAN, T.IMAGENET_STD)(torch.zeros(1, 3, 2, 2, device=dev))


@pytest.mark.parametrize("h,w", [(224, 224), (64, 64), (7, 9), (31, 300)])
def test_ssim(dev, h, w):
    from roadrestore import imgproc
    a = _batch(3, h, w, seed=h)
    noise = np.random.default_rng(w).integers(-30, 31, a.shape)
    b = np.clip(a.astype(int) + noise, 0, 255).astype(np.uint8)
    b[2] = a[2]                                              # identical pair -> 1.0
    got = imgproc.ssim(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)).cpu().numpy()
    ref = np.array([I.ssim(a[i], b[i]) for i in range(3)])
    assert np.abs(got - ref).max() < 1e-10, (got, ref)
    assert got[2] == pytest.approx(1.0, abs=1e-12)


def test_ssim_rejects_small(dev):
    from roadrestore import ops
    z = torch.zeros(1, 6, 10, 3, dtype=torch.uint8, device=dev)
    with pytest.raises(RuntimeError):
        ops.ssim_u8(z, z)


def test_psnr_matches_formula(dev):
    from roadrestore import imgproc
    a = _batch(2, 224, 224, seed=1)
    b = _batch(2, 224, 224, seed=2)
    got = imgproc.psnr(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)).cpu().numpy()
    for i in range(2):
        mse = np.mean((a[i].astype(np.float64) - b[i].astype(np.float64)) ** 2)
        assert got[i] == pytest.approx(10 * np.log10(255.0 ** 2 / mse), abs=1e-9)


def _params_from_draws(rng, n):
    """mirror of the reference's draws, returned both as oracle kwargs and as
    the device parameters"""
    from roadrestore import imgproc
    state = rng.getstate()
    params, taps = imgproc.distortion_params(n, rng)
    rng.setstate(state)
    kw = []
    for _ in range(n):
        d = {}
        if rng.random() < 0.5:
            intensity = rng.uniform(0.3, 0.7)
            d["fog_t"] = 1.0 - intensity * rng.uniform(0.8, 1.2)
        sigma = None
        if rng.random() < 0.5:
            sigma = rng.uniform(0.01, 0.03) ** 0.5
        if rng.random() < 0.5:
            d["blur"] = (rng.randint(5, 15), rng.randint(0, 360))
        kw.append((d, sigma))
    return params, taps, kw


@pytest.mark.parametrize("h,w", [(64, 64), (31, 45)])
def test_random_distortions_bit_exact_given_noise(dev, h, w):
    """14:31-64 with the reference's random draws and an explicit fp64 noise
    field: the device generator equals the restatement byte for byte."""
    from roadrestore import ops
    n = 12
    rng = random.Random(5)
    params, taps, kw = _params_from_draws(rng, n)
    x = _batch(n, h, w, seed=11)
    noise = np.random.default_rng(12).normal(0, 1, x.shape)
    for i, (d, sigma) in enumerate(kw):
        noise[i] *= sigma if sigma is not None else 0.0
    y = ops.distort_u8(torch.from_numpy(x).to(dev), params, taps, mode=0,
                       noise=torch.from_numpy(noise)).cpu().numpy()
    kinds = set()
    for i, (d, sigma) in enumerate(kw):
        ref = I.distort(x[i], noise=noise[i] if sigma is not None else None, **d)
        assert np.array_equal(y[i], ref), (i, d, sigma)
        kinds.add((("fog_t" in d), sigma is not None, ("blur" in d)))
    assert len(kinds) >= 4                                    # several branch combinations


def test_compound_distortion_bit_exact_given_noise(dev):
    from roadrestore import imgproc
    x = _batch(3, 64, 64, seed=21)
    noise = np.random.default_rng(22).normal(0, 0.02 ** 0.5, x.shape)
    y = imgproc.apply_compound_distortion(torch.from_numpy(x).to(dev),
                                          noise=torch.from_numpy(noise)).cpu().numpy()
    for i in range(3):
        assert np.array_equal(y[i], I.compound(x[i], noise[i]))


def test_device_noise_statistics_and_determinism(dev):
    """Philox noise: N(0, sigma) per element, deterministic per seed"""
    from roadrestore import ops
    from roadrestore._lib import RR_DISTORT_NOISE, DistortParam
    n, h, w = 4, 128, 128
    x = torch.full((n, h, w, 3), 128, dtype=torch.uint8, device=dev)
    p = [DistortParam(0.1, 1.0, 0.0, RR_DISTORT_NOISE, 0)] * n
    taps = torch.zeros(n, 15, 15)
    y1 = ops.distort_u8(x, p, taps, seed=1234)
    y2 = ops.distort_u8(x, p, taps, seed=1234)
    y3 = ops.distort_u8(x, p, taps, seed=99)
    assert torch.equal(y1, y2) and not torch.equal(y1, y3)
    # v = trunc((128/255 + N(0, .1)) * 255): mean ~ 127.5 + E, std ~ 25.5
    v = y1.double().cpu()
    assert abs(v.std().item() - 25.5) < 0.5
    assert abs(v.mean().item() - 127.5) < 0.5


def test_random_distortions_entry_point(dev):
    from roadrestore import imgproc
    x = torch.from_numpy(_batch(8, 64, 64, seed=3)).to(dev)
    y = imgproc.apply_random_distortions(x, rng=random.Random(0))
    assert y.shape == x.shape and y.dtype == torch.uint8
    assert not torch.equal(x, y)


def test_random_distortion_draws_on_device(dev):
    """rr_distort_random_u8 (14:31-64 with the draws made on device): the
    draws follow the reference's distributions, the blur taps are the table
    entry of the drawn (degree, angle), the pixels equal rr_distort_u8 given
    the same draws byte for byte, and the step counter advances per call."""
    from roadrestore import imgproc, ops
    from roadrestore._lib import RR_DISTORT_BLUR, RR_DISTORT_FOG, RR_DISTORT_NOISE
    n = 512
    x = torch.from_numpy(_batch(n, 64, 64, seed=5)).to(dev)
    rd = imgproc.RandomDistortion(dev, seed=1234)
    y1 = rd(x)
    p1, idx1, s1 = rd.last_draws()
    y2 = rd(x)
    p2, idx2, s2 = rd.last_draws()
    assert rd.step.item() == 2 and s1 != s2 and not torch.equal(y1, y2)
    table = imgproc.motion_blur_table(dev).view(-1, 15, 15)
    for params, idx, seed, y in ((p1, idx1, s1, y1), (p2, idx2, s2, y2)):
        fog = np.array([bool(p.flags & RR_DISTORT_FOG) for p in params])
        noi = np.array([bool(p.flags & RR_DISTORT_NOISE) for p in params])
        blu = np.array([bool(p.flags & RR_DISTORT_BLUR) for p in params])
        for f in (fog, noi, blu):                       # p = 0.5 each: 3.5 sigma band
            assert abs(f.mean() - 0.5) < 3.5 * 0.5 / np.sqrt(n), f.mean()
        t = np.array([p.fog_mul for p in params])[fog]
        assert t.min() >= 1 - 0.7 * 1.2 - 1e-6 and t.max() <= 1 - 0.3 * 0.8 + 1e-6
        fa = np.array([p.fog_add for p in params])[fog]
        assert np.allclose(fa, 0.9 * (1 - t), atol=1e-6)
        sg = np.array([p.sigma for p in params])[noi]
        assert sg.min() >= 0.1 - 1e-12 and sg.max() <= 0.03 ** 0.5 + 1e-12
        k = np.array([p.ksize for p in params])[blu]
        assert k.min() >= 5 and k.max() <= 15 and len(set(k.tolist())) >= 9
        ang = idx.numpy()[blu] - (k - 5) * 361
        assert ang.min() >= 0 and ang.max() <= 360
        taps = table[idx.to(dev).long()]
        want = ops.distort_u8(x, params, taps, mode=0, seed=seed)
        assert torch.equal(y, want)


@pytest.mark.parametrize("mode", [0, 1])
def test_blur_tiled_equals_untiled(dev, mode, monkeypatch):
    """The LDS-compacted blur (h * w a multiple of 256: nonzero taps listed
    once per workgroup) is byte-identical to the per-pixel tap scan
    (RR_PATH blur_tiled=0) over every (degree, angle) the draws can produce."""
    from roadrestore import imgproc, ops
    from roadrestore._lib import RR_DISTORT_BLUR
    n = 11 * 24
    x = torch.from_numpy(_batch(n, 64, 64, seed=31)).to(dev)
    rd = imgproc.RandomDistortion(dev, seed=77)
    rd(x)
    params, _, seed = rd.last_draws()
    table = imgproc.motion_blur_table(dev).view(-1, 15, 15)
    idx = torch.tensor([(i % 11) * 361 + (i * 37) % 361 for i in range(n)], device=dev)
    for i, p in enumerate(params):
        p.flags |= RR_DISTORT_BLUR
        p.ksize = 5 + i % 11
    outs = []
    for tiled in ("1", "0"):
        set_path(monkeypatch, "blur_tiled", tiled)
        outs.append(ops.distort_u8(x, params, table[idx], mode=mode, seed=seed))
    assert torch.equal(outs[0], outs[1])


def test_random_distortion_in_hip_graph(dev):
    """Captured once, every replay re-draws (the counter is device state)."""
    from roadrestore import imgproc
    x = torch.from_numpy(_batch(64, 32, 32, seed=6)).to(dev)
    rd = imgproc.RandomDistortion(dev, seed=7)
    out = torch.empty_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        rd(x, out=out)                                  # warm-up: workspace allocated
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        rd(x, out=out)
    seen = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        seen.append(out.clone())
    assert rd.step.item() == 4
    assert not torch.equal(seen[0], seen[1]) and not torch.equal(seen[1], seen[2])


@pytest.mark.parametrize("h,w,oh,ow,c", [
    (41, 47, 224, 224, 3), (64, 58, 224, 224, 3), (30, 33, 224, 224, 3), (250, 180, 224, 224, 3),
    (224, 224, 64, 64, 3), (37, 53, 50, 61, 3), (9, 11, 5, 4, 1), (20, 30, 33, 47, 4),
    (64, 64, 64, 64, 3), (1, 1, 7, 5, 3)])
def test_cv_resize_linear_bit_exact(dev, h, w, oh, ow, c):
    """cv2.resize INTER_LINEAR (08:119, the PSNR leg's clean image) on device
    equals the oracle restatement bit for bit (up / down / anisotropic /
    1-pixel; 1, 3, 4 channels; scalar row tails at widths not a multiple of
    the vector width)."""
    import roadrestore as rr
    x = _batch(3, h, w, c, seed=h * w + c)
    y = rr.imgproc.cv_resize(torch.from_numpy(x).to(dev), (ow, oh)).cpu().numpy()
    assert y.shape == (3, oh, ow, c)
    for i in range(3):
        assert np.array_equal(y[i], I.cv_resize_linear(x[i], oh, ow)), i
