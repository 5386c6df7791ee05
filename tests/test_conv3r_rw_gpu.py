"""The register-weight K loop of the tap-reuse conv (conv3r RW, csrc/conv3r.hip):
every wave loads its A fragments from the weight tiles in global memory
into a 4-set register ring one stage ahead, the LDS holds only the
double-buffered halo, and a barrier ends each 32-channel chunk.  Per
accumulator the MFMA order is the LDS-weight loop's, so every output --
the conv, its BN statistics, every epilogue (bias / ReLU / accumulate / mask
/ concat split / fused BN-PReLU backward / PReLU / residual / pool) -- must be
BITWISE equal between RR_CONV3R_RW=1 and =0 on the same tile geometry, and
within bf16 rounding of fp32 torch (ResUNet 14:96-186 and VGG16 features,
14:189-196, at the cfg3 shapes and at small batches).  Shapes cover 2, 4, 6,
12 and 16 K chunks (the 4-chunk loop body, its 2-chunk tail, a concat source
switch mid-loop), every whole-row geometry (W = 32 / 16 / 8 pairs) and both
workgroup kinds and wave-tile widths."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


def nhwc(x, dev):
    return x.permute(0, 2, 3, 1).contiguous().to(dev, BF)


def nchw(y):
    return y.float().permute(0, 3, 1, 2).contiguous().cpu()


def rel(a, r):
    a, r = a.float().cpu(), r.float().cpu()
    return ((a - r).norm() / r.norm().clamp_min(1e-30)).item()


def _desc(n, w, c1, c2, co, **kw):
    from roadrestore._lib import RR_BF16, RR_CONV3X3, IgemmDesc
    return IgemmDesc(RR_BF16, RR_CONV3X3, n, w, w, c1, c2, co, kw.get("split", 0), kw.get("act", 0),
                     kw.get("acc", 0), kw.get("bias", 0), kw.get("mask", 0), kw.get("stats", 0), 0)


# (n, w, c1, c2, c_out)
SHAPES = [
    (4, 32, 64, 0, 128),     # res2.c1 / VGG conv2_1: 2 chunks (the tail only)
    (2, 32, 128, 0, 128),    # res2.c2: 4 chunks (one loop body)
    (4, 32, 128, 64, 64),    # dec2.c1 concat: 6 chunks, the source switch in the loop
    (2, 32, 128, 0, 256),    # two column blocks
    (8, 16, 128, 0, 256),    # res3.c1
    (4, 16, 256, 128, 128),  # dec3.c1 concat: 12 chunks
    (2, 16, 256, 0, 256),
    (64, 8, 512, 0, 512),    # bottleneck: 16 chunks
    (8, 8, 256, 0, 512),     # 128 x 32 wave tiles
    (8, 8, 128, 0, 128),
]
GEOMS = [("4", "64"), ("8", "64"), ("4", "32"), ("8", "32")]   # (RR_CONV3R_WG, RR_CONV3R_NW)


def _set(monkeypatch, geom, rw):
    monkeypatch.setenv("RR_CONV3R", "1")
    monkeypatch.setenv("RR_CONV3R_WG", geom[0])
    monkeypatch.setenv("RR_CONV3R_NW", geom[1])
    monkeypatch.setenv("RR_CONV3R_RW", rw)


def _both(monkeypatch, geom, desc, fn):
    """fn() under RW=0 and RW=1 on the same tile geometry -> (out0, out1, names)"""
    from roadrestore import ops
    res, names = {}, {}
    for rw in ("0", "1"):
        _set(monkeypatch, geom, rw)
        names[rw] = ops.igemm_kernel_name(desc)
        res[rw] = fn()
        torch.cuda.synchronize()
    return res["0"], res["1"], names


def _check_names(names):
    n0, n1 = names["0"], names["1"]
    assert n0.startswith("conv3r_kernel<") and "<s" not in n0, n0
    assert n1 == n0[:-1] + ",rw>", (n0, n1)


@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("shape", SHAPES)
def test_rw_fwd_bias_stats_relu_bitwise(dev, shape, geom, monkeypatch):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, w, c1, c2, co = shape
    cin = c1 + c2
    x = rnd(n, cin, w, w, seed=1).bfloat16().float()
    wt = (rnd(co, cin, 3, 3, seed=2) / (3 * cin ** 0.5)).bfloat16().float()
    b = rnd(co, seed=3)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    x1 = nhwc(x[:, :c1], dev)
    x2 = nhwc(x[:, c1:], dev) if c2 else None

    def run():
        y, _, st = rr.ops.igemm(RR_CONV3X3, x1, x2, n, w, w, wf, co, bias=b.to(dev), stats=True)
        yr, _, _ = rr.ops.igemm(RR_CONV3X3, x1, x2, n, w, w, wf, co, bias=b.to(dev), act=1)
        return y, st, yr
    o0, o1, names = _both(monkeypatch, geom, _desc(n, w, c1, c2, co, bias=1, stats=1), run)
    _check_names(names)
    for a, bb in zip(o0, o1):
        assert torch.equal(a, bb)
    ref = F.conv2d(x, wt, b, padding=1)
    assert rel(nchw(o1[0]), ref) < 4e-3
    assert rel(nchw(o1[2]), F.relu(ref)) < 4e-3


@pytest.mark.parametrize("geom", GEOMS[:2])
@pytest.mark.parametrize("shape", [(2, 32, 128, 0, 128), (8, 16, 256, 0, 256), (64, 8, 512, 0, 512),
                                   (4, 32, 128, 0, 64)])
def test_rw_dgrad_accumulate_mask_bitwise(dev, shape, geom, monkeypatch):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, w, c1, _, co = shape
    x = nhwc(rnd(n, c1, w, w, seed=11), dev)
    wt = (rnd(co, c1, 3, 3, seed=12) / (3 * c1 ** 0.5)).to(dev)
    y0 = nhwc(rnd(n, co, w, w, seed=13), dev)
    m = nhwc(rnd(n, co, w, w, seed=14), dev)
    wf, _ = rr.ops.pack_conv(wt, BF)

    def run():
        y, _, _ = rr.ops.igemm(RR_CONV3X3, x, None, n, w, w, wf, co, out=y0.clone(), accumulate=True,
                               mask=m)
        return y
    o0, o1, names = _both(monkeypatch, geom, _desc(n, w, c1, 0, co, acc=1, mask=1), run)
    _check_names(names)
    assert torch.equal(o0, o1)


@pytest.mark.parametrize("geom", GEOMS[:2])
@pytest.mark.parametrize("shape,split", [((4, 16, 128, 0, 384), 256), ((4, 32, 64, 0, 192), 64)])
def test_rw_concat_split_dgrad_bitwise(dev, shape, split, geom, monkeypatch):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, w, c1, _, co = shape
    x = nhwc(rnd(n, c1, w, w, seed=21), dev)
    wf, _ = rr.ops.pack_conv((rnd(co, c1, 3, 3, seed=22) / (3 * c1 ** 0.5)).to(dev), BF)

    def run():
        y1, y2, _ = rr.ops.igemm(RR_CONV3X3, x, None, n, w, w, wf, co, split=split)
        return y1, y2
    o0, o1, names = _both(monkeypatch, geom, _desc(n, w, c1, 0, co, split=split), run)
    _check_names(names)
    assert torch.equal(o0[0], o1[0]) and torch.equal(o0[1], o1[1])


@pytest.mark.parametrize("geom", GEOMS[:2])
@pytest.mark.parametrize("shape", [(2, 32, 128, 0, 128), (8, 16, 256, 0, 256), (64, 8, 512, 0, 512),
                                   (4, 32, 128, 0, 64)])
def test_rw_bnbwd_bitwise(dev, shape, geom, monkeypatch):
    """conv2 dgrad with the fused BN1 / PReLU backward epilogue (14:99-105)"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    ops = rr.ops
    n, w, cg, _, C = shape
    g2 = nhwc(rnd(n, cg, w, w, seed=51), dev)
    _, wd = ops.pack_conv((rnd(cg, C, 3, 3, seed=52) * (1.0 / (3 * C ** 0.5))).to(dev), BF)
    t1 = nhwc(rnd(n, C, w, w, seed=53) * 2 + 0.3, dev)
    tf = t1.float().reshape(-1, C)
    mean = tf.mean(0)
    inv = 1.0 / torch.sqrt(tf.var(0, unbiased=False) + 1e-5)
    gamma = (torch.rand(C, generator=torch.Generator().manual_seed(54)) + 0.5).to(dev)
    beta = (torch.rand(C, generator=torch.Generator().manual_seed(55)) - 0.5).to(dev)
    s1 = gamma * inv
    sh1 = beta - mean * s1
    alpha = torch.tensor([0.23], device=dev)

    def run():
        gm, part, rows, arows = ops.igemm_bnbwd(RR_CONV3X3, g2, n, w, w, wd, C, t1, mean, inv, s1,
                                                sh1, alpha)
        r = ops.bn_backward_rows(gm, part, rows, arows, t1, mean, inv, gamma)
        return gm, r["dgamma0"], r["dbeta0"], r["dalpha"], r["dt0"]
    o0, o1, _ = _both(monkeypatch, geom, _desc(n, w, cg, 0, C), run)
    # the masked grad bitwise; the per-row partial sums of the register-weight
    # loop (general epilogue, staged on the 4-wave tiles) and of the default
    # bnbwd-only instance (in registers) are laid out differently, so the
    # channel sums agree to fp32 rounding
    assert torch.equal(o0[0], o1[0])
    for a, b in zip(o0[1:4], o1[1:4]):
        assert ((a - b).norm() / b.norm().clamp_min(1e-30)).item() < 1e-5
    assert ((o0[4].float() - o1[4].float()).norm() / o1[4].float().norm()).item() < 1e-3


@pytest.mark.parametrize("shape", [(4, 16, 256, 0, 256), (8, 32, 128, 0, 128), (64, 8, 512, 0, 512)])
def test_rw_inference_epilogues_bitwise(dev, shape, monkeypatch):
    """rr_igemm_ex: PReLU, residual + ReLU, and the 2x2 max-pool from the
    registers (17:84-86 eval blocks; VGG conv + ReLU + MaxPool2d)"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, w, c1, _, co = shape
    x = nhwc(rnd(n, c1, w, w, seed=61), dev)
    wf, _ = rr.ops.pack_conv((rnd(co, c1, 3, 3, seed=62) / (3 * c1 ** 0.5)).to(dev), BF)
    b = rnd(co, seed=63).to(dev)
    res = nhwc(rnd(n, co, w, w, seed=64), dev)
    alpha = torch.tensor([0.2], device=dev)

    def run():
        a, _, _ = rr.ops.igemm(RR_CONV3X3, x, None, n, w, w, wf, co, bias=b, alpha=alpha)
        r, p, _ = rr.ops.igemm(RR_CONV3X3, x, None, n, w, w, wf, co, bias=b, res=res, act=1,
                               pool=True)
        return a, r, p
    o0, o1, _ = _both(monkeypatch, ("8", "64"), _desc(n, w, c1, 0, co, bias=1), run)
    for a, bb in zip(o0, o1):
        assert torch.equal(a, bb)
