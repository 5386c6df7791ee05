"""Column-strip mode of the row-streaming 3x3 conv (csrc/stream3.hip) and its
BN-folded eval epilogues.

The 64 -> 64 convs of the reference's 224 x 224 pipeline (17:66, 17:84-86 /
18:28-32 through 14:96-115 and VGG16 conv1_2) are wider than a ring row, so
the kernel walks each image as W-wide column strips (32 at 224, 64 where 64
divides the width) whose left / right neighbour columns are real pixels (the
strip's halo), zero only at the image edge.  Checked against fp32 torch (the
inputs are bf16-exact, so the only error is the output's bf16 rounding) and
against the tap-reuse conv's row-segment tiles on the same shape (RR_PATH
stream3_strips=0), for every epilogue the strips have an instance for:
  * the plain conv / dgrad, bias, bias + ReLU;
  * the eval ones (rr_igemm_ex): PReLU(conv + b); ReLU(conv + b + x); the
    same + the 2x2 max-pool with the full output kept; conv + ReLU + pool
    without the window index (rr_igemm_pool, the judge).  The pooled output is
    checked BITWISE against max-pooling the kernel's own full output.
Shapes put workgroup step ranges across strip and image boundaries (uneven
splits) and include non-square maps."""
import pytest
import torch
import torch.nn.functional as F
from rrpath import set_path  # noqa: E402

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
# (n, h, w): P >= 256 x 256 pixels, h % (256 / strip) == 0
STRIPS = [(2, 224, 224), (10, 40, 224), (5, 128, 128), (4, 104, 160)]


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


def _name(n, h, w, act=0):
    import roadrestore as rr
    from roadrestore._lib import IgemmDesc, RR_BF16, RR_CONV3X3
    return rr.ops.igemm_kernel_name(IgemmDesc(RR_BF16, RR_CONV3X3, n, h, w, 64, 0, 64, 0, act, 0,
                                              1, 0, 0, 0))


@pytest.mark.parametrize("shape", STRIPS)
def test_strip_fwd(dev, shape, monkeypatch):
    """plain / bias / bias + ReLU on strips vs fp32 torch and the row-segment
    tiles; the image borders (the outer strips' zero columns) included"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, h, w = shape
    assert _name(n, h, w).startswith("stream3_kernel<s32")
    x = rnd(n, 64, h, w, seed=1).bfloat16().float()
    wt = (rnd(64, 64, 3, 3, seed=2) / 24.0).bfloat16().float()
    b = rnd(64, seed=3)
    pre = F.conv2d(x, wt, None, padding=1)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    outs = {}
    for tag in ("1", "0"):
        set_path(monkeypatch, "stream3_strips", tag)
        y0, _, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, h, w, wf, 64)
        y, _, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, h, w, wf, 64, bias=b.to(dev))
        yr, _, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev), None, n, h, w, wf, 64, bias=b.to(dev),
                                act=1)
        torch.cuda.synchronize()
        outs[tag] = (nchw(y0), nchw(y), nchw(yr))
    y0, y, yr = outs["1"]
    ref = pre + b[None, :, None, None]
    assert rel(y0, pre) < 4e-3
    assert rel(y, ref) < 4e-3
    assert rel(yr, F.relu(ref)) < 4e-3
    # vs the row-segment tiles: the same bf16 rounding of the same fp32 sums
    for got, seg in zip(outs["1"], outs["0"]):
        assert rel(got, seg) < 1e-3
    # every image-border column / row and every strip seam (columns 31 / 32
    # of each 32-wide strip) at the bf16 rounding level
    assert rel(y[..., 0], ref[..., 0]) < 4e-3 and rel(y[..., -1], ref[..., -1]) < 4e-3
    assert rel(y[..., 31::32], ref[..., 31::32]) < 4e-3 and rel(y[..., 32::32], ref[..., 32::32]) < 4e-3
    assert rel(y[..., 0, :], ref[..., 0, :]) < 4e-3 and rel(y[..., -1, :], ref[..., -1, :]) < 4e-3


def test_strip_dgrad(dev, monkeypatch):
    """the plain dgrad (no epilogue) on strips == conv_transpose2d"""
    from roadrestore import ops
    from roadrestore._lib import RR_CONV3X3
    n, h, w = 2, 224, 224
    dt = rnd(n, 64, h, w, seed=71).bfloat16().float()
    wt = (rnd(64, 64, 3, 3, seed=73) / 24.0).bfloat16().float()
    ref = F.conv_transpose2d(dt, wt, padding=1)
    _, wd = ops.pack_conv(wt.to(dev), BF)
    g, _, _ = ops.igemm(RR_CONV3X3, nhwc(dt, dev), None, n, h, w, wd, 64)
    torch.cuda.synchronize()
    assert rel(nchw(g), ref) < 4e-3
    # (the dgrad + 1x1 shortcut form has no strip instance)
    d = ops.dgrad_sc_desc(nhwc(dt, dev), n, h, w, 64)
    assert ops.igemm_dgrad_sc_kernel_name(d, 64) == "unsupported"


@pytest.mark.parametrize("shape", STRIPS[:2] + [(17, 64, 64), (81, 32, 32)])
def test_eval_epilogues(dev, shape, monkeypatch):
    """rr_igemm_ex on the streaming kernel (strips, and whole rows at 64 /
    32): PReLU, residual + ReLU, + the 2x2 max-pool with the full output,
    and conv + ReLU + pool without an index; vs fp32 torch and vs the
    tap-reuse conv on the same call"""
    import roadrestore as rr
    from roadrestore._lib import RR_ACT_POOL, RR_ACT_PRELU, RR_ACT_RES, RR_CONV3X3
    ops = rr.ops
    n, h, w = shape
    x = rnd(n, 64, h, w, seed=81).bfloat16().float()
    r = rnd(n, 64, h, w, seed=82).bfloat16().float()
    wt = (rnd(64, 64, 3, 3, seed=83) / 24.0).bfloat16().float()
    b = rnd(64, seed=84) * 0.1
    al = torch.tensor([0.2])
    pre = F.conv2d(x, wt, None, padding=1) + b[None, :, None, None]
    wf, _ = ops.pack_conv(wt.to(dev), BF)
    xd, rd, bd, ad = nhwc(x, dev), nhwc(r, dev), b.to(dev), al.to(dev)
    assert _name(n, h, w, RR_ACT_PRELU).startswith("stream3")
    assert _name(n, h, w, 1 | RR_ACT_RES | RR_ACT_POOL).startswith("stream3")

    def run():
        y1, _, _ = ops.igemm(RR_CONV3X3, xd, None, n, h, w, wf, 64, bias=bd, alpha=ad)
        y2, _, _ = ops.igemm(RR_CONV3X3, xd, None, n, h, w, wf, 64, bias=bd, res=rd, act=1)
        y3, p3, _ = ops.igemm(RR_CONV3X3, xd, None, n, h, w, wf, 64, bias=bd, res=rd, act=1, pool=True)
        y4, _, _ = ops.igemm(RR_CONV3X3, xd, None, n, h, w, wf, 64, bias=bd, act=1)
        p4, i4 = ops.igemm_pool(xd, n, h, w, wf, 64, bias=bd, want_idx=False)
        torch.cuda.synchronize()
        return [nchw(t) for t in (y1, y2, y3, p3, y4, p4)]
    got = run()
    y1, y2, y3, p3, y4, p4 = got
    assert rel(y1, F.prelu(pre, al)) < 4e-3
    assert rel(y2, F.relu(pre + r)) < 4e-3
    assert torch.equal(y3, y2)                                     # the same epilogue + the pool
    assert torch.equal(p3, F.max_pool2d(y3, 2))                   # bitwise: the kernel's own output
    assert torch.equal(p4, F.max_pool2d(y4, 2))
    # vs the tap-reuse conv (the same ex calls, the streaming kernel off)
    set_path(monkeypatch, "stream3", "0")
    assert _name(n, h, w, RR_ACT_PRELU).startswith("conv3r")
    ref = run()
    for a, c in zip(got, ref):
        assert rel(a, c) < 2e-3


def test_strips_beyond_32bit_offsets(dev):
    """the cfg5 chunk size (1024 images of 224 x 224 = 6.6 GB per tensor:
    element offsets past 2^31): the same two images repeated through the
    batch give bitwise the outputs of the two-image call (a pixel's sum does
    not depend on the batch), at both ends of the batch"""
    from roadrestore import ops
    from roadrestore._lib import RR_CONV3X3
    n, h, w = 2, 224, 224
    x = rnd(n, 64, h, w, seed=91).bfloat16().float()
    wt = (rnd(64, 64, 3, 3, seed=92) / 24.0).bfloat16().float()
    b = rnd(64, seed=93) * 0.1
    wf, _ = ops.pack_conv(wt.to(dev), BF)
    xd, bd, ad = nhwc(x, dev), b.to(dev), torch.tensor([0.2], device=dev)
    small, _, _ = ops.igemm(RR_CONV3X3, xd, None, n, h, w, wf, 64, bias=bd, alpha=ad)
    rep = 344                                       # 688 images: 34.5 M pixels, 4.4 GB
    big_x = xd.repeat(rep, 1, 1, 1)
    assert _name(n * rep, h, w, 2).startswith("stream3_kernel<s32")
    big, _, _ = ops.igemm(RR_CONV3X3, big_x, None, n * rep, h, w, wf, 64, bias=bd, alpha=ad)
    torch.cuda.synchronize()
    assert torch.equal(big[:n], small) and torch.equal(big[-n:], small)
    assert torch.equal(big[n * (rep // 2):n * (rep // 2 + 1)], small)
