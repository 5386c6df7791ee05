"""Tap-reuse 3x3 conv (csrc/conv3r.hip): the bf16 conv of the 64-512-channel
layers on 32x32 / 16x16 / 8x8 maps (ResUNet res2 / res3 / dec2 / dec3 /
bottleneck, VGG16 conv2_x / conv3_x; their dgrads with the concat split and
the fused BN/PReLU backward) vs fp32 torch and vs the LDS-halo kernel it
replaces (RR_PATH conv3r=0).  Inputs are bf16-exact, so against fp32 torch the
only error is the bf16 rounding of the output; vs the halo kernel the same
fp32 sums in another order, rounded once.  Shapes cover every tile geometry:
a tile inside an image (W = 32: 16 or 8 rows, top and bottom zero rows),
whole images (W = 16), image pairs (W = 8), several column blocks, concat
inputs."""
import pytest
import torch
import torch.nn.functional as F
from rrpath import set_path  # noqa: E402

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


def _desc(n, w, c1, c2, co, split=0, act=0, acc=0, bias=0, mask=0, stats=0, h=None):
    from roadrestore._lib import RR_BF16, RR_CONV3X3, IgemmDesc
    return IgemmDesc(RR_BF16, RR_CONV3X3, n, w if h is None else h, w, c1, c2, co, split, act, acc,
                     bias, mask, stats, 0)


# (n, w, c1, c2, c_out, kernel) -- 4-wave workgroups (2 per CU; RR_PATH conv3r_wg=4,
# the default where c_out % 128 != 0)
SHAPES = [
    (4, 32, 64, 0, 128, "conv3r_kernel<32,128>"),     # res2.c1 / VGG conv2_1
    (2, 32, 128, 0, 128, "conv3r_kernel<32,128>"),    # res2.c2 / conv2_2 (fwd + dgrad)
    (4, 32, 128, 64, 64, "conv3r_kernel<32,64>"),     # dec2.c1 (concat) fwd
    (2, 32, 128, 0, 256, "conv3r_kernel<32,128>"),    # 8-row tiles in a 32-row image, 2 blocks
    (8, 16, 128, 0, 256, "conv3r_kernel<16,128>"),    # res3.c1 / conv3_1
    (4, 16, 256, 128, 128, "conv3r_kernel<16,128>"),  # dec3.c1 (concat)
    (512, 8, 512, 0, 512, "conv3r_kernel<8,128>"),    # bottleneck at B = 512 (4 column blocks)
    (512, 8, 512, 0, 256, "conv3r_kernel<8,128,32>"), # 128 x 32 wave tiles: 512 workgroups
    (8, 8, 256, 0, 512, "conv3r_kernel<8,128,32>"),   # small batch: 128 x 32 tiles
    (8, 8, 128, 0, 128, "conv3r_kernel<8,128,32>"),
    (2, 64, 64, 64, 64, "conv3r_kernel<64,64>"),      # dec1.c1 (concat) fwd: 2-row wave tiles
    (2, 64, 128, 0, 128, "conv3r_kernel<64,128>"),
]
# the 8-wave, one-per-CU variant (RR_PATH conv3r_wg=8, the default where
# c_out % 128 == 0)
SHAPES_W8 = [
    (4, 32, 64, 0, 128, "conv3r_kernel<32,128,w8>"),
    (4, 32, 128, 64, 64, "conv3r_kernel<32,64,32,w8>"),
    (2, 32, 128, 0, 256, "conv3r_kernel<32,128,w8>"),
    (8, 16, 128, 0, 256, "conv3r_kernel<16,128,w8>"),
    (512, 8, 512, 0, 512, "conv3r_kernel<8,128,w8>"),
    (8, 8, 256, 0, 512, "conv3r_kernel<8,128,32,w8>"),
    (2, 64, 64, 0, 128, "conv3r_kernel<64,128,w8>"),  # dec1.c1 dgrad (64 -> 64 + 64)
    (2, 64, 64, 64, 64, "conv3r_kernel<64,64,32,w8>"),
]


@pytest.fixture(params=["4", "8"])
def wg(request, monkeypatch):
    set_path(monkeypatch, "conv3r_wg", request.param)
    return request.param


@pytest.mark.parametrize("shape", SHAPES + [s + ("w8",) for s in SHAPES_W8])
def test_conv3r_selected(dev, shape, monkeypatch):
    set_path(monkeypatch, "conv3r_wg", "4")
    if len(shape) == 7:
        set_path(monkeypatch, "conv3r_wg", "8")
        shape = shape[:6]
    from roadrestore import ops
    n, w, c1, c2, co, name = shape
    assert ops.igemm_kernel_name(_desc(n, w, c1, c2, co, bias=1, stats=1)) == name
    set_path(monkeypatch, "conv3r", "0")
    assert not ops.igemm_kernel_name(_desc(n, w, c1, c2, co, bias=1, stats=1)).startswith("conv3r")


@pytest.mark.parametrize("shape", SHAPES + SHAPES_W8)
def test_conv3r_fwd_bias_stats_relu(dev, shape, monkeypatch):
    set_path(monkeypatch, "conv3r_wg", "8" if shape in SHAPES_W8 else "4")
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, w, c1, c2, co, _ = shape
    cin = c1 + c2
    x = rnd(n, cin, w, w, seed=1).bfloat16().float()
    wt = (rnd(co, cin, 3, 3, seed=2) / (3 * cin ** 0.5)).bfloat16().float()
    b = rnd(co, seed=3)
    pre = F.conv2d(x, wt, None, padding=1)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    x1 = nhwc(x[:, :c1], dev)
    x2 = nhwc(x[:, c1:], dev) if c2 else None
    outs = {}
    for tag in ("1", "0"):
        set_path(monkeypatch, "conv3r", tag)
        y, _, st = rr.ops.igemm(RR_CONV3X3, x1, x2, n, w, w, wf, co, bias=b.to(dev), stats=True)
        yr, _, _ = rr.ops.igemm(RR_CONV3X3, x1, x2, n, w, w, wf, co, bias=b.to(dev), act=1)
        torch.cuda.synchronize()
        outs[tag] = (nchw(y), st.double().sum(0).cpu(), nchw(yr), st.shape[0])
    y, s, yr, rows = outs["1"]
    assert rows == n * w * w // 128
    ref = pre + b[None, :, None, None]
    assert rel(y, ref) < 4e-3
    assert rel(yr, F.relu(ref)) < 4e-3
    assert rel(s[:, 0], pre.double().sum((0, 2, 3))) < 1e-5
    assert rel(s[:, 1], (pre.double() ** 2).sum((0, 2, 3))) < 1e-5
    assert rel(y, outs["0"][0]) < 2e-3
    assert rel(s, outs["0"][1]) < 1e-5


@pytest.mark.parametrize("shape", [(2, 32, 128, 0, 128), (8, 16, 256, 0, 256), (8, 8, 512, 0, 512),
                                   (512, 8, 512, 0, 512), (4, 32, 128, 0, 64), (2, 64, 128, 0, 64),
                                   (2, 64, 64, 0, 128)])
@pytest.mark.parametrize("acc,msk", [(True, False), (False, True), (True, True)])
def test_conv3r_dgrad_epilogues(dev, shape, acc, msk, wg, monkeypatch):
    """dgrad epilogues: accumulate into y (the shortcut / identity grad), the
    ReLU-backward mask (VGG dgrads), both."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "conv3r", "1")
    n, w, c1, _, co = shape
    x = rnd(n, c1, w, w, seed=11).bfloat16().float()
    wt = (rnd(co, c1, 3, 3, seed=12) / (3 * c1 ** 0.5)).bfloat16().float()
    y0 = rnd(n, co, w, w, seed=13).bfloat16().float()
    m = rnd(n, co, w, w, seed=14).bfloat16().float()
    ref = F.conv2d(x, wt, None, padding=1) + (y0 if acc else 0)
    if msk:
        ref = torch.where(m > 0, ref, torch.zeros(()))
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    out = nhwc(y0, dev) if acc else None
    assert rr.ops.igemm_kernel_name(_desc(n, w, c1, 0, co, acc=int(acc), mask=int(msk))) \
        .startswith("conv3r")
    y, _, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, w, w, wf, co, out=out,
                           accumulate=acc, mask=nhwc(m, dev) if msk else None)
    assert rel(nchw(y), ref) < 4e-3


@pytest.mark.parametrize("shape,split", [((4, 16, 128, 0, 384), 256), ((4, 32, 64, 0, 192), 64),
                                         ((4, 32, 64, 0, 192), 128),
                                         ((2, 64, 64, 0, 128), 64)])
def test_conv3r_concat_split_dgrad(dev, shape, split, wg, monkeypatch):
    """the dgrad of a concat-input conv writes the two halves to two tensors
    (dec3.c1: 128 -> 256 + 128, dec2.c1: 64 -> 128 + 64 / 64 + 128)"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, w, c1, _, co = shape
    x = rnd(n, c1, w, w, seed=21).bfloat16().float()
    wt = (rnd(co, c1, 3, 3, seed=22) / (3 * c1 ** 0.5)).bfloat16().float()
    ref = F.conv2d(x, wt, None, padding=1)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    outs = {}
    for tag in ("1", "0"):
        set_path(monkeypatch, "conv3r", tag)
        y1, y2, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, w, w, wf, co, split=split)
        torch.cuda.synchronize()
        outs[tag] = torch.cat((nchw(y1), nchw(y2)), 1)
    assert rel(outs["1"], ref) < 4e-3
    assert rel(outs["1"], outs["0"]) < 2e-3


@pytest.mark.parametrize("shape", [(2, 32, 128, 0, 128), (8, 16, 256, 0, 256), (8, 8, 512, 0, 512),
                                   (4, 32, 128, 0, 64), (512, 8, 512, 0, 256), (2, 64, 128, 0, 64)])
def test_conv3r_bnbwd(dev, shape, wg, monkeypatch):
    """conv dgrad + BN/PReLU backward reduce fused in the staged epilogue ==
    the halo kernel's fused path == the unfused sequence."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    ops = rr.ops
    n, w, cg, _, C = shape
    g2 = nhwc(rnd(n, cg, w, w, seed=51), dev)
    wt = (rnd(cg, C, 3, 3, seed=52) * (1.0 / (3 * C ** 0.5))).to(dev)
    _, wd = ops.pack_conv(wt, BF)
    t1 = nhwc(rnd(n, C, w, w, seed=53) * 2 + 0.3, dev)
    tf = t1.float().reshape(-1, C)
    mean = tf.mean(0)
    inv = 1.0 / torch.sqrt(tf.var(0, unbiased=False) + 1e-5)
    gamma = (torch.rand(C, generator=torch.Generator().manual_seed(54)) + 0.5).to(dev)
    beta = (torch.rand(C, generator=torch.Generator().manual_seed(55)) - 0.5).to(dev)
    s1 = gamma * inv
    sh1 = beta - mean * s1
    alpha = torch.tensor([0.23], device=dev)
    set_path(monkeypatch, "conv3r", "0")
    da1, _, _ = ops.igemm(RR_CONV3X3, g2, None, n, w, w, wd, C)
    ref = ops.bn_backward(da1, t1, mean, inv, gamma, mask_kind=2, aux=t1, aff_s=s1, aff_b=sh1,
                          alpha=alpha)
    res = {}
    for tag in ("0", "1"):
        set_path(monkeypatch, "conv3r", tag)
        gm, part, rows, arows = ops.igemm_bnbwd(RR_CONV3X3, g2, n, w, w, wd, C, t1, mean, inv, s1,
                                                sh1, alpha)
        if tag == "1":
            assert rows == n * w * w // 128
            assert ops.igemm_kernel_name(_desc(n, w, cg, 0, C), bnbwd=True).startswith("conv3r")
        res[tag] = ops.bn_backward_rows(gm, part, rows, arows, t1, mean, inv, gamma)
    torch.cuda.synchronize()
    got, halo = res["1"], res["0"]
    assert rel(got["dt0"], ref["dt0"]) < 2e-2
    for k in ("dgamma0", "dbeta0", "dalpha"):
        assert rel(got[k], ref[k]) < 2e-2, k
        assert rel(got[k], halo[k]) < 1e-4, k
    assert rel(got["dt0"], halo["dt0"]) < 2e-3


@pytest.mark.parametrize("shape", [(2, 64, 64, 64, 64, 0), (2, 64, 64, 0, 128, 64)])
def test_conv3r_w64_rows_equal_segments(dev, shape, wg, monkeypatch):
    """64x64 maps: the whole-row tiles (2 output rows per wave) against the
    row-segment tiles they replace (RR_PATH conv3r_w64=0) -- dec1.c1 forward with
    BN statistics and its concat-split dgrad; the same fp32 sums per output
    (same K order), so bitwise-equal outputs; statistics rows differ only in
    which pixels share a partial row"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "conv3r", "1")
    n, w, c1, c2, co, split = shape
    x = rnd(n, c1 + c2, w, w, seed=41)
    wf, _ = rr.ops.pack_conv((rnd(co, c1 + c2, 3, 3, seed=42) / 24).to(dev), BF)
    x1 = nhwc(x[:, :c1], dev)
    x2 = nhwc(x[:, c1:], dev) if c2 else None
    res = {}
    for tag in ("1", "0"):
        set_path(monkeypatch, "conv3r_w64", tag)
        name = rr.ops.igemm_kernel_name(_desc(n, w, c1, c2, co, split=split, stats=int(not split)))
        assert name.startswith("conv3r_kernel<64," if tag == "1" else "conv3r_kernel<s2,"), name
        if split:
            y1, y2, _ = rr.ops.igemm(RR_CONV3X3, x1, x2, n, w, w, wf, co, split=split)
            res[tag] = (torch.cat((y1, y2), -1), None)
        else:
            y, _, st = rr.ops.igemm(RR_CONV3X3, x1, x2, n, w, w, wf, co, stats=True)
            res[tag] = (y, st.double().sum(0))
        torch.cuda.synchronize()
    assert torch.equal(res["1"][0], res["0"][0])
    if not split:
        assert rel(res["1"][1], res["0"][1]) < 1e-6


def test_conv3r_stats_rows_deterministic(dev, wg, monkeypatch):
    """fixed tile -> partial-row mapping: two launches give bitwise-equal
    outputs and statistics"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "conv3r", "1")
    n, w, c, co = 8, 16, 256, 256
    x = nhwc(rnd(n, c, w, w, seed=31), dev)
    wf, _ = rr.ops.pack_conv((rnd(co, c, 3, 3, seed=32) / 48).to(dev), BF)
    a = rr.ops.igemm(RR_CONV3X3, x, None, n, w, w, wf, co, stats=True)
    b = rr.ops.igemm(RR_CONV3X3, x, None, n, w, w, wf, co, stats=True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2])


# ---- row-segment tiles (any H x W): the reference's own geometry, 224^2 and
# its 112 / 56 / 28 / 14 maps (14:202-205, 17:66, 18:28-32), odd sizes,
# batches that do not fill whole-row tiles ----
# (n, h, w, c1, c2, c_out, kernel)
SHAPES_SEG = [
    (2, 224, 224, 64, 0, 64, "conv3r_kernel<s2,64>"),      # enc1.c2 / VGG conv1_2 at 224
    (2, 112, 112, 64, 0, 128, "conv3r_kernel<s2,128>"),    # enc2.c1 / conv2_1 (4th segment half out)
    (2, 56, 56, 128, 0, 256, "conv3r_kernel<s2,128>"),     # enc3.c1 / conv3_1
    (2, 28, 28, 256, 0, 512, "conv3r_kernel<s2,128,w8>"),  # bottleneck / conv4_1 (partial band)
    (2, 14, 14, 512, 0, 512, "conv3r_kernel<s1,128,w8>"),  # VGG conv5_x (8-wave, W <= 28)
    (4, 14, 14, 64, 0, 64, "conv3r_kernel<s1,64>"),
    (3, 36, 52, 64, 64, 128, "conv3r_kernel<s2,128>"),     # odd sizes, concat input
    (2, 60, 60, 64, 0, 64, "conv3r_kernel<s2,64>"),        # partial bands of 16 rows
    (1, 8, 8, 64, 0, 128, "conv3r_kernel<s1,128>"),        # B = 1 8x8: no whole-row tile
]


def _seg_rows(n, h, w, co, name):
    sg = int(name.split("<s")[1][0])
    bc = int(name.split(",")[1].rstrip(">"))
    w8 = ",w8" in name                          # conv3r_segwg=8: 8-wave workgroups
    nw = 64 if (sg == 2 and (bc == 128 or not w8)) else 32
    wp = (8 if w8 else 4) // (bc // nw)
    tr = wp * (8 // sg)
    return n * -(-w // (16 * sg)) * -(-h // tr) * wp


def _seg_name_ok(got, name):
    # RR_PATH conv3r_segwg=4 / 8 switches the workgroup kind
    base = name.replace(",w8", "")
    return got in (base, base[:-1] + ",w8>")


@pytest.mark.parametrize("shape", SHAPES_SEG)
def test_conv3r_seg_fwd_bias_stats_relu(dev, shape, monkeypatch):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, h, w, c1, c2, co, name = shape
    set_path(monkeypatch, "conv3r", "1")
    name_got = rr.ops.igemm_kernel_name(_desc(n, w, c1, c2, co, bias=1, stats=1, h=h))
    assert _seg_name_ok(name_got, name), name_got
    cin = c1 + c2
    x = rnd(n, cin, h, w, seed=1).bfloat16().float()
    wt = (rnd(co, cin, 3, 3, seed=2) / (3 * cin ** 0.5)).bfloat16().float()
    b = rnd(co, seed=3)
    pre = F.conv2d(x, wt, None, padding=1)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    x1 = nhwc(x[:, :c1], dev)
    x2 = nhwc(x[:, c1:], dev) if c2 else None
    outs = {}
    for tag in ("1", "0"):
        set_path(monkeypatch, "conv3r", tag)
        y, _, st = rr.ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), stats=True)
        yr, _, _ = rr.ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), act=1)
        torch.cuda.synchronize()
        outs[tag] = (nchw(y), st.double().sum(0).cpu(), nchw(yr), st.shape[0])
    y, s, yr, rows = outs["1"]
    assert rows == _seg_rows(n, h, w, co, name_got)
    ref = pre + b[None, :, None, None]
    assert rel(y, ref) < 4e-3
    assert rel(yr, F.relu(ref)) < 4e-3
    assert rel(s[:, 0], pre.double().sum((0, 2, 3))) < 1e-5
    assert rel(s[:, 1], (pre.double() ** 2).sum((0, 2, 3))) < 1e-5
    assert rel(y, outs["0"][0]) < 2e-3
    assert rel(s, outs["0"][1]) < 1e-5


@pytest.mark.parametrize("shape", [(2, 112, 112, 128, 0, 64), (2, 28, 28, 512, 0, 256),
                                   (4, 14, 14, 512, 0, 512), (3, 36, 52, 128, 0, 128)])
@pytest.mark.parametrize("acc,msk", [(True, False), (False, True), (True, True)])
def test_conv3r_seg_dgrad_epilogues(dev, shape, acc, msk, monkeypatch):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "conv3r", "1")
    n, h, w, c1, _, co = shape
    x = rnd(n, c1, h, w, seed=11).bfloat16().float()
    wt = (rnd(co, c1, 3, 3, seed=12) / (3 * c1 ** 0.5)).bfloat16().float()
    y0 = rnd(n, co, h, w, seed=13).bfloat16().float()
    m = rnd(n, co, h, w, seed=14).bfloat16().float()
    ref = F.conv2d(x, wt, None, padding=1) + (y0 if acc else 0)
    if msk:
        ref = torch.where(m > 0, ref, torch.zeros(()))
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    out = nhwc(y0, dev) if acc else None
    assert rr.ops.igemm_kernel_name(_desc(n, w, c1, 0, co, acc=int(acc), mask=int(msk), h=h)) \
        .startswith("conv3r_kernel<s")
    y, _, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, h, w, wf, co, out=out,
                           accumulate=acc, mask=nhwc(m, dev) if msk else None)
    assert rel(nchw(y), ref) < 4e-3


@pytest.mark.parametrize("shape,split", [((2, 56, 56, 128, 0, 384), 256),
                                         ((2, 224, 224, 64, 0, 128), 64)])
def test_conv3r_seg_concat_split_dgrad(dev, shape, split, monkeypatch):
    """dec3.c1 / dec1.c1 dgrads at the 224 geometry: two output tensors"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, h, w, c1, _, co = shape
    x = rnd(n, c1, h, w, seed=21).bfloat16().float()
    wt = (rnd(co, c1, 3, 3, seed=22) / (3 * c1 ** 0.5)).bfloat16().float()
    ref = F.conv2d(x, wt, None, padding=1)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    set_path(monkeypatch, "conv3r", "1")
    assert rr.ops.igemm_kernel_name(_desc(n, w, c1, 0, co, split=split, h=h)).startswith("conv3r_kernel<s")
    y1, y2, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, h, w, wf, co, split=split)
    torch.cuda.synchronize()
    assert rel(torch.cat((nchw(y1), nchw(y2)), 1), ref) < 4e-3


@pytest.mark.parametrize("shape", [(2, 56, 56, 256, 0, 128), (2, 28, 28, 512, 0, 256),
                                   (4, 14, 14, 512, 0, 512), (4, 14, 14, 128, 0, 64),
                                   (3, 36, 52, 128, 0, 64), (2, 112, 112, 64, 0, 128)])
def test_conv3r_seg_bnbwd(dev, shape, monkeypatch):
    """conv dgrad + BN/PReLU backward reduce in the row-segment kernel's
    register epilogue == the unfused sequence == the fallback kernel's fused
    path (partial rows in another grouping: sums to fp32 rounding)"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    ops = rr.ops
    n, h, w, cg, _, C = shape
    g2 = nhwc(rnd(n, cg, h, w, seed=51), dev)
    wt = (rnd(cg, C, 3, 3, seed=52) * (1.0 / (3 * C ** 0.5))).to(dev)
    _, wd = ops.pack_conv(wt, BF)
    t1 = nhwc(rnd(n, C, h, w, seed=53) * 2 + 0.3, dev)
    tf = t1.float().reshape(-1, C)
    mean = tf.mean(0)
    inv = 1.0 / torch.sqrt(tf.var(0, unbiased=False) + 1e-5)
    gamma = (torch.rand(C, generator=torch.Generator().manual_seed(54)) + 0.5).to(dev)
    beta = (torch.rand(C, generator=torch.Generator().manual_seed(55)) - 0.5).to(dev)
    s1 = gamma * inv
    sh1 = beta - mean * s1
    alpha = torch.tensor([0.23], device=dev)
    set_path(monkeypatch, "conv3r", "0")
    da1, _, _ = ops.igemm(RR_CONV3X3, g2, None, n, h, w, wd, C)
    ref = ops.bn_backward(da1, t1, mean, inv, gamma, mask_kind=2, aux=t1, aff_s=s1, aff_b=sh1,
                          alpha=alpha)
    res = {}
    for tag in ("0", "1"):
        set_path(monkeypatch, "conv3r", tag)
        gm, part, rows, arows = ops.igemm_bnbwd(RR_CONV3X3, g2, n, h, w, wd, C, t1, mean, inv, s1,
                                                sh1, alpha)
        if tag == "1":
            name = ops.igemm_kernel_name(_desc(n, w, cg, 0, C, h=h), bnbwd=True)
            assert name.startswith("conv3r_kernel<s"), name
            assert rows == _seg_rows(n, h, w, C, name)
        res[tag] = ops.bn_backward_rows(gm, part, rows, arows, t1, mean, inv, gamma)
    torch.cuda.synchronize()
    got, halo = res["1"], res["0"]
    assert rel(got["dt0"], ref["dt0"]) < 2e-2
    for k in ("dgamma0", "dbeta0", "dalpha"):
        assert rel(got[k], ref[k]) < 2e-2, k
        assert rel(got[k], halo[k]) < 1e-4, k
    assert rel(got["dt0"], halo["dt0"]) < 2e-3


def test_conv3r_seg_deterministic(dev, monkeypatch):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "conv3r", "1")
    n, h, w, c, co = 2, 56, 56, 128, 256
    x = nhwc(rnd(n, c, h, w, seed=31), dev)
    wf, _ = rr.ops.pack_conv((rnd(co, c, 3, 3, seed=32) / 48).to(dev), BF)
    a = rr.ops.igemm(RR_CONV3X3, x, None, n, h, w, wf, co, stats=True)
    b = rr.ops.igemm(RR_CONV3X3, x, None, n, h, w, wf, co, stats=True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2])


@pytest.mark.parametrize("shape", [(2, 224, 224, 64, 0, 64), (2, 56, 56, 128, 0, 256), (4, 16, 16, 256, 0, 256),
                                   (3, 36, 52, 64, 64, 128), (2, 32, 32, 128, 0, 128)])
def test_conv3r_ex_prelu_and_residual(dev, shape, monkeypatch):
    """rr_igemm_ex: the eval-mode residual block's epilogues (BN folded into
    the conv, 17:84-86) -- PReLU after conv1 (14:101-103) and the identity
    shortcut's relu(conv2 + x) (14:110-115) -- vs fp32 torch on bf16-exact
    inputs, and vs the unfused conv + activation pass."""
    import roadrestore as rr
    from roadrestore import ops
    from roadrestore._lib import RR_ACT_PRELU, RR_ACT_RES, RR_CONV3X3
    set_path(monkeypatch, "conv3r", "1")
    set_path(monkeypatch, "stream3", "0")       # (the 224 64 -> 64 maps: stream3's column strips)
    n, h, w, c1, c2, co = shape
    cin = c1 + c2
    x = rnd(n, cin, h, w, seed=61).bfloat16().float()
    wt = (rnd(co, cin, 3, 3, seed=62) / (3 * cin ** 0.5)).bfloat16().float()
    b = rnd(co, seed=63) * 0.3
    r = rnd(n, co, h, w, seed=64).bfloat16().float()
    alpha = torch.tensor([0.17], device=dev)
    pre = F.conv2d(x, wt, b, padding=1)
    wf, _ = ops.pack_conv(wt.to(dev), BF)
    x1 = nhwc(x[:, :c1], dev)
    x2 = nhwc(x[:, c1:], dev) if c2 else None
    assert ops.igemm_kernel_name(_desc(n, w, c1, c2, co, act=RR_ACT_PRELU, bias=1, h=h)).startswith("conv3r")
    y, _, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), alpha=alpha)
    ref = torch.where(pre > 0, pre, 0.17 * pre)
    assert rel(nchw(y), ref) < 4e-3
    t, _, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev))
    one, zero = torch.ones(co, device=dev), torch.zeros(co, device=dev)
    y0 = ops.affine_act(t, one, zero, alpha=alpha)
    assert rel(nchw(y), nchw(y0)) < 2e-3
    # residual + ReLU
    y, _, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), res=nhwc(r, dev), act=1)
    assert rel(nchw(y), F.relu(pre + r)) < 4e-3
    # residual + PReLU (both flags)
    y, _, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), res=nhwc(r, dev),
                        alpha=alpha)
    s = pre + r
    assert rel(nchw(y), torch.where(s > 0, s, 0.17 * s)) < 4e-3
    torch.cuda.synchronize()
    # the plain entry point refuses the fused activations
    from roadrestore._lib import lib
    import ctypes as C
    d = _desc(n, w, c1, c2, co, act=RR_ACT_PRELU | RR_ACT_RES, h=h)
    assert lib().rr_igemm(C.byref(d), None, None, None, None, None, None, None, None, None) != 0


@pytest.mark.parametrize("shape", [(2, 224, 224, 64, 0, 64), (2, 56, 56, 128, 0, 256), (3, 28, 28, 256, 0, 512),
                                   (2, 14, 14, 512, 0, 512), (4, 16, 16, 256, 0, 256), (8, 8, 8, 256, 0, 512),
                                   (2, 32, 32, 128, 0, 128), (3, 36, 52, 64, 64, 128), (2, 30, 22, 128, 0, 128),
                                   (2, 15, 17, 64, 0, 128), (3, 29, 13, 128, 0, 64)])
def test_conv3r_ex_pool(dev, shape, monkeypatch):
    """rr_igemm_ex RR_ACT_POOL: conv + bias + ReLU (+ residual) with the 2x2
    max-pool (MaxPool2d(2), floor sizes; the encoder's 14:127-131 and the VGG
    judge's pools) written from the epilogue, with and without the full-size
    output, vs fp32 torch on bf16-exact inputs"""
    from roadrestore import ops
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "conv3r", "1")
    set_path(monkeypatch, "stream3", "0")       # (the 224 64 -> 64 maps: stream3's column strips)
    n, h, w, c1, c2, co = shape
    cin = c1 + c2
    x = rnd(n, cin, h, w, seed=71).bfloat16().float()
    wt = (rnd(co, cin, 3, 3, seed=72) / (3 * cin ** 0.5)).bfloat16().float()
    b = rnd(co, seed=73) * 0.3
    r = rnd(n, co, h, w, seed=74).bfloat16().float()
    pre = F.conv2d(x, wt, b, padding=1)
    wf, _ = ops.pack_conv(wt.to(dev), BF)
    x1 = nhwc(x[:, :c1], dev)
    x2 = nhwc(x[:, c1:], dev) if c2 else None
    y, yp, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), act=1, pool=True)
    ref = F.relu(pre)
    assert rel(nchw(y), ref) < 4e-3
    # the pool of the rounded output equals the rounded pool (rounding is monotone)
    assert torch.equal(nchw(yp), F.max_pool2d(nchw(y), 2))
    y0, yp0, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), act=1, pool_only=True)
    assert y0 is None and torch.equal(yp0, yp)
    y, yp, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), act=1, res=nhwc(r, dev),
                         pool=True)
    assert rel(nchw(y), F.relu(pre + r)) < 4e-3
    assert torch.equal(nchw(yp), F.max_pool2d(nchw(y), 2))
    # accumulate + ReLU + pool (the eval BN-shortcut block: conv2 adds onto the
    # 1x1 shortcut's output, engine.resblock_forward_eval_folded)
    base = nhwc(r, dev)
    y, yp, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, co, bias=b.to(dev), out=base,
                         accumulate=True, act=1, pool=True)
    assert y.data_ptr() == base.data_ptr()
    assert rel(nchw(y), F.relu(pre + r)) < 4e-3
    assert torch.equal(nchw(yp), F.max_pool2d(nchw(y), 2))
