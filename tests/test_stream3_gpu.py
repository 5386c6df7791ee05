"""Row-streaming 3x3 conv (csrc/stream3.hip): the 64 -> 64 channel bf16 conv
at W = 64 / 32 (ResUNet res1 / dec1 / dec2, VGG16 conv1_2) vs fp32 torch and
vs the tiled halo kernel (RR_PATH stream3=0).  Shapes put workgroup row ranges
across image boundaries (uneven splits, short images) so the ring's
pre-load steps and zero-padding rows are exercised.  Inputs are bf16-exact,
so against fp32 torch the only error is the bf16 rounding of the output."""
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


# (n, h, w): >= one 256-pixel step per workgroup (P >= 65536, h % (256 / w) == 0);
# uneven splits and short images put workgroup ranges across image boundaries
SHAPES = [(16, 64, 64), (17, 64, 64), (65, 16, 64), (64, 32, 32), (81, 32, 32), (257, 8, 32)]


def _blocks(n, h, w):
    import ctypes as C
    import roadrestore as rr
    from roadrestore._lib import IgemmDesc, RR_BF16, RR_CONV3X3
    d = IgemmDesc(RR_BF16, RR_CONV3X3, n, h, w, 64, 0, 64, 0, 0, 0, 1, 0, 1, 0)
    return rr.lib().rr_igemm_stat_blocks(C.byref(d))


def _name(n, h, w):
    import roadrestore as rr
    from roadrestore._lib import IgemmDesc, RR_BF16, RR_CONV3X3
    return rr.ops.igemm_kernel_name(IgemmDesc(RR_BF16, RR_CONV3X3, n, h, w, 64, 0, 64, 0, 0, 0,
                                              1, 0, 1, 0))


@pytest.mark.parametrize("shape", SHAPES)
def test_stream3_selected(dev, shape, monkeypatch):
    """the streaming kernel owns these shapes (256 partial rows), and the
    RR_PATH stream3=0 switch hands them back to the tiled kernel"""
    n, h, w = shape
    assert _blocks(n, h, w) == 256 and _name(n, h, w).startswith("stream3")
    # too small for one step per workgroup / not whole steps: a tiled kernel
    assert not _name(n // 2 if n * h * w // 2 < 65536 else 1, h, w).startswith("stream3")
    set_path(monkeypatch, "stream3", "0")
    # the tap-reuse conv: 32x32 whole-row tiles (128-pixel partial rows),
    # else row-segment tiles (4 wave rows of 4 x 32 pixels per 16-row band)
    seg = n * -(-w // 32) * -(-h // 16) * 4
    whole = h == w and w in (32, 64)                 # (64x64: whole rows of 2-row wave tiles)
    assert _blocks(n, h, w) == ((n * h * w) // 128 if whole else seg)
    assert _name(n, h, w) == ("conv3r_kernel<%d,64>" % w if whole else "conv3r_kernel<s2,64>")


@pytest.mark.parametrize("shape", SHAPES)
def test_stream3_fwd_stats(dev, shape, monkeypatch):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, h, w = shape
    x = rnd(n, 64, h, w, seed=1).bfloat16().float()
    wt = (rnd(64, 64, 3, 3, seed=2) / 24.0).bfloat16().float()
    b = rnd(64, seed=3)
    pre = F.conv2d(x, wt, None, padding=1)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    outs = {}
    for tag in ("1", "0"):
        set_path(monkeypatch, "stream3", tag)
        y, _, st = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, h, w, wf, 64, bias=b.to(dev),
                                stats=True)
        yr, _, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, h, w, wf, 64, bias=b.to(dev),
                                act=1)
        torch.cuda.synchronize()
        outs[tag] = (nchw(y), st.double().sum(0).cpu(), nchw(yr))
    y, s, yr = outs["1"]
    assert rel(y, pre + b[None, :, None, None]) < 4e-3
    assert rel(yr, F.relu(pre + b[None, :, None, None])) < 4e-3
    assert rel(s[:, 0], pre.double().sum((0, 2, 3))) < 1e-5
    assert rel(s[:, 1], (pre.double() ** 2).sum((0, 2, 3))) < 1e-5
    # vs the tiled kernel: same bf16 rounding of the same fp32 sums
    assert rel(y, outs["0"][0]) < 1e-3
    assert rel(s, outs["0"][1]) < 1e-5


@pytest.mark.parametrize("shape", [(17, 64, 64), (81, 32, 32)])
@pytest.mark.parametrize("acc,msk,act", [(True, False, 0), (False, True, 0), (True, True, 0),
                                         (False, False, 1), (False, False, 0)])
def test_stream3_load_epilogue(dev, shape, acc, msk, act, monkeypatch):
    """dgrad epilogues: accumulate into y (identity-shortcut grad), relu
    backward mask (VGG conv1_2 dgrad), both; plain and ReLU without bias."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "stream3", "1")
    n, h, w = shape
    x = rnd(n, 64, h, w, seed=11).bfloat16().float()
    wt = (rnd(64, 64, 3, 3, seed=12) / 24.0).bfloat16().float()
    y0 = rnd(n, 64, h, w, seed=13).bfloat16().float()
    m = rnd(n, 64, h, w, seed=14).bfloat16().float()
    pre = F.conv2d(x, wt, None, padding=1)
    ref = pre + (y0 if acc else 0)
    if act:
        ref = F.relu(ref)
    if msk:
        ref = torch.where(m > 0, ref, torch.zeros(()))
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    out = nhwc(y0, dev) if acc else None
    y, _, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, h, w, wf, 64, out=out,
                           accumulate=acc, act=act, mask=nhwc(m, dev) if msk else None)
    assert rel(nchw(y), ref) < 4e-3


@pytest.mark.parametrize("shape", [(16, 64, 64), (17, 64, 64), (81, 32, 32)])
def test_stream3_bnbwd(dev, shape, monkeypatch):
    """conv dgrad + BN/PReLU backward reduce fused in the streaming epilogue
    == the tiled kernel's fused path == the unfused sequence."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    ops = rr.ops
    n, h, w = shape
    C = 64
    g2 = nhwc(rnd(n, C, h, w, seed=51), dev)
    wt = (rnd(C, C, 3, 3, seed=52) * (1.0 / (3 * C ** 0.5))).to(dev)
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
    set_path(monkeypatch, "stream3", "0")
    da1, _, _ = ops.igemm(RR_CONV3X3, g2, None, n, h, w, wd, C)
    ref = ops.bn_backward(da1, t1, mean, inv, gamma, mask_kind=2, aux=t1, aff_s=s1, aff_b=sh1,
                          alpha=alpha)
    res = {}
    for tag in ("0", "1"):
        set_path(monkeypatch, "stream3", tag)
        gm, part, rows, arows = ops.igemm_bnbwd(RR_CONV3X3, g2, n, h, w, wd, C, t1, mean, inv, s1,
                                                sh1, alpha)
        if tag == "1":
            assert rows == 256 and arows == 256
        res[tag] = ops.bn_backward_rows(gm, part, rows, arows, t1, mean, inv, gamma)
    torch.cuda.synchronize()
    got, tiled = res["1"], res["0"]
    assert rel(got["dt0"], ref["dt0"]) < 2e-2
    for k in ("dgamma0", "dbeta0", "dalpha"):
        assert rel(got[k], ref[k]) < 2e-2, k
        assert rel(got[k], tiled[k]) < 1e-4, k
    assert rel(got["dt0"], tiled["dt0"]) < 2e-3


@pytest.mark.parametrize("shape", [(16, 64, 64), (17, 64, 64), (81, 32, 32)])
@pytest.mark.parametrize("stats,bias,act", [(True, True, 0), (False, True, 1), (False, False, 0)])
def test_stream3_concat_one_pass(dev, shape, stats, bias, act, monkeypatch):
    """64 + 64-channel concat input (ResUNet dec1 conv1, 14:144,174-177):
    the tap-reuse conv in ONE pass (the K = 1152 sum in fp32, no bf16
    rounding of a half sum; the two-pass streaming form was removed in round
    6), against fp32 torch on the concatenation at the single-rounding bound;
    the statistics are of the pre-bias sum."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, h, w = shape
    x1 = rnd(n, 64, h, w, seed=61).bfloat16().float()
    x2 = rnd(n, 64, h, w, seed=62).bfloat16().float()
    wt = (rnd(64, 128, 3, 3, seed=63) / 34.0).bfloat16().float()
    b = rnd(64, seed=64) if bias else None
    pre = F.conv2d(torch.cat((x1, x2), 1), wt, None, padding=1)
    ref = pre + (b[None, :, None, None] if bias else 0)
    if act:
        ref = F.relu(ref)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    d = rr.ops.IgemmDesc(rr.ops.RR_BF16, RR_CONV3X3, n, h, w, 64, 64, 64, 0, act, 0,
                         int(bias), 0, int(stats), 0)
    one_pass = "conv3r_kernel<%d,64>" % w if h == w else "conv3r_kernel<s2,64>"
    assert rr.ops.igemm_kernel_name(d) == one_pass
    y, _, st = rr.ops.igemm(RR_CONV3X3, nhwc(x1, dev), nhwc(x2, dev), n, h, w, wf, 64,
                            bias=b.to(dev) if bias else None, act=act, stats=stats)
    torch.cuda.synchronize()
    y1 = nchw(y)
    assert rel(y1, ref) < 4e-3
    if stats:
        s1 = st.double().sum(0).cpu()
        assert rel(s1[:, 0], pre.double().sum((0, 2, 3))) < 1e-5
        assert rel(s1[:, 1], (pre.double() ** 2).sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize("shape", [(17, 64, 64), (65, 16, 64), (81, 32, 32)])
def test_dgrad_sc_equals_dgrad_plus_shortcut(dev, shape):
    """rr_igemm_dgrad_sc: per concat half, the 3x3 dgrad + the 1x1 shortcut
    dgrad in one pass (dec1's input grad, 14:99-115) vs fp32 torch
    (conv_transpose of both) and vs the two-step form it replaces (3x3 dgrad,
    then the 1x1 dgrad accumulated in bf16): the one-pass sum is rounded once,
    so it is at least as close to fp32."""
    import roadrestore as rr
    from roadrestore import ops
    from roadrestore._lib import RR_CONV1X1, RR_CONV3X3
    n, h, w = shape
    dt = rnd(n, 64, h, w, seed=71).bfloat16().float()
    dsc = rnd(n, 64, h, w, seed=72).bfloat16().float()
    wt = (rnd(64, 128, 3, 3, seed=73) / 24.0).bfloat16().float()      # dec1.conv_block[0]
    ws = (rnd(64, 128, 1, 1, seed=74) / 8.0).bfloat16().float()       # dec1.shortcut[0]
    ref = F.conv_transpose2d(dt, wt, padding=1) + F.conv_transpose2d(dsc, ws)
    _, wd = ops.pack_conv(wt.to(dev), BF)
    _, wsd = ops.pack_conv(ws.to(dev), BF)
    half, hs = 64 * 9 * 64, 64 * 64
    d = ops.dgrad_sc_desc(nhwc(dt, dev), n, h, w, 64)
    assert ops.igemm_dgrad_sc_kernel_name(d, 64) == "stream3_kernel<%d,sc>" % w
    assert ops.igemm_dgrad_sc_kernel_name(d, 32) == "unsupported"
    x, xs = nhwc(dt, dev), nhwc(dsc, dev)
    g1 = ops.igemm_dgrad_sc(x, n, h, w, wd[:half], 64, xs, wsd[:hs])
    g2 = ops.igemm_dgrad_sc(x, n, h, w, wd[half:], 64, xs, wsd[hs:])
    # the two-step form (RR_PATH sc_dgrad=0)
    t1, _, _ = ops.igemm(RR_CONV3X3, x, None, n, h, w, wd[:half], 64)
    t2, _, _ = ops.igemm(RR_CONV3X3, x, None, n, h, w, wd[half:], 64)
    ops.igemm(RR_CONV1X1, xs, None, n, h, w, wsd, 128, out=t1, out2=t2, split=64, accumulate=True)
    torch.cuda.synchronize()
    got = torch.cat((nchw(g1), nchw(g2)), 1)
    two = torch.cat((nchw(t1), nchw(t2)), 1)
    e_got, e_two = rel(got, ref), rel(two, ref)
    print(f"{shape}: one pass rel {e_got:.2e}, two-step rel {e_two:.2e}")
    assert e_got < 4e-3 and e_got <= e_two * 1.05
    assert rel(got, two) < 4e-3
    # deterministic
    g1b = ops.igemm_dgrad_sc(x, n, h, w, wd[:half], 64, xs, wsd[:hs])
    assert torch.equal(g1, g1b)
