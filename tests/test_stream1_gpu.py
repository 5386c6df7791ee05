"""Wave-streaming 1x1 / convT GEMM (csrc/stream1.hip) vs fp32 torch and vs
the tiled igemm kernel (RR_PATH stream1=0), for every mode and epilogue the
ResUNet step routes through it: shortcut conv fwd with BN statistics
(14:109-112), its dgrad into a concat split with accumulate, the relu-mask
epilogue, the fp32 NCHW final conv (14:149), ConvTranspose2d(2, 2) fwd
(14:137-147) and its dgrad.  Inputs are bf16-exact, so against fp32 torch the
only error is the bf16 rounding of the output.  RR_PATH stream1_minp lowers the
pixel-count threshold so small shapes take the streaming path (uneven block
counts per wave, partial last rounds)."""
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


def _name(mode, n, h, w, c1, c2, co, split=0, act=0, acc=0, bias=0, mask=0, stats=0, nchw_=0):
    import roadrestore as rr
    d = rr.ops.IgemmDesc(rr.ops.RR_BF16, mode, n, h, w, c1, c2, co, split, act, acc, bias, mask,
                         stats, nchw_)
    return rr.ops.igemm_kernel_name(d)


# (n, h, w): P = 4096 .. 35200 pixels -> 256 .. 2200 16-pixel blocks over 2048 waves
SHAPES = [(4, 32, 32), (11, 16, 16), (137, 16, 16)]


@pytest.fixture
def small_ok(monkeypatch):
    set_path(monkeypatch, "stream1_minp", "1024")


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("c1,c2,co", [(64, 0, 128), (128, 0, 256), (64, 128, 64), (128, 256, 128),
                                      (64, 64, 64)])
def test_stream1_conv1x1_stats(dev, small_ok, shape, c1, c2, co, monkeypatch):
    """shortcut conv fwd: bias + BN partial statistics of the pre-bias sum"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV1X1
    n, h, w = shape
    x1 = rnd(n, c1, h, w, seed=1).bfloat16().float()
    x2 = rnd(n, c2, h, w, seed=2).bfloat16().float() if c2 else None
    wt = (rnd(co, c1 + c2, 1, 1, seed=3) / (c1 + c2) ** 0.5).bfloat16().float()
    b = rnd(co, seed=4)
    xin = torch.cat((x1, x2), 1) if c2 else x1
    pre = F.conv2d(xin, wt)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    # K = 192 with statistics stays on the tiled kernel (measured faster)
    want = "igemm_kernel" if c1 + c2 == 192 else "stream1_kernel"
    assert _name(RR_CONV1X1, n, h, w, c1, c2, co, bias=1, stats=1).startswith(want)
    res = {}
    for tag in ("1", "0"):
        set_path(monkeypatch, "stream1", tag)
        y, _, st = rr.ops.igemm(RR_CONV1X1, nhwc(x1, dev), nhwc(x2, dev) if c2 else None, n, h, w,
                                wf, co, bias=b.to(dev), stats=True)
        torch.cuda.synchronize()
        res[tag] = (nchw(y), st.double().sum(0).cpu())
    y, s = res["1"]
    assert rel(y, pre + b[None, :, None, None]) < 4e-3
    assert rel(s[:, 0], pre.double().sum((0, 2, 3))) < 1e-5
    assert rel(s[:, 1], (pre.double() ** 2).sum((0, 2, 3))) < 1e-5
    assert rel(y, res["0"][0]) < 1e-3
    assert rel(s, res["0"][1]) < 1e-5


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("cin,split,co", [(64, 64, 128), (64, 64, 192), (128, 128, 384),
                                          (128, 0, 64), (256, 0, 128)])
@pytest.mark.parametrize("acc", [True, False])
def test_stream1_dgrad_split_accumulate(dev, small_ok, shape, cin, split, co, acc):
    """shortcut dgrad: dx of the concat halves (column split), accumulated
    onto the conv1 dgrad already there (14:109-112 backward)"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV1X1
    n, h, w = shape
    g = rnd(n, cin, h, w, seed=11).bfloat16().float()
    wt = (rnd(co, cin, 1, 1, seed=12) / cin ** 0.5).bfloat16().float()
    ref = F.conv2d(g, wt)
    y0 = rnd(n, co, h, w, seed=13).bfloat16().float()
    if acc:
        ref = ref + y0
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    assert _name(RR_CONV1X1, n, h, w, cin, 0, co, split=split, acc=int(acc)).startswith("stream1")
    if split:
        o1, o2 = nhwc(y0[:, :split], dev), nhwc(y0[:, split:], dev)
        y1, y2, _ = rr.ops.igemm(RR_CONV1X1, nhwc(g, dev), None, n, h, w, wf, co, out=o1, out2=o2,
                                 split=split, accumulate=acc)
        got = torch.cat((nchw(y1), nchw(y2)), 1)
    else:
        y1, _, _ = rr.ops.igemm(RR_CONV1X1, nhwc(g, dev), None, n, h, w, wf, co,
                                out=nhwc(y0, dev) if acc else None, accumulate=acc)
        got = nchw(y1)
    assert rel(got, ref) < 4e-3


@pytest.mark.parametrize("shape", SHAPES[:2])
def test_stream1_relu_and_mask(dev, small_ok, shape):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV1X1
    n, h, w = shape
    x = rnd(n, 128, h, w, seed=21).bfloat16().float()
    wt = (rnd(64, 128, 1, 1, seed=22) / 11.0).bfloat16().float()
    m = rnd(n, 64, h, w, seed=23).bfloat16().float()
    b = rnd(64, seed=24)
    pre = F.conv2d(x, wt)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    y, _, _ = rr.ops.igemm(RR_CONV1X1, nhwc(x, dev), None, n, h, w, wf, 64, bias=b.to(dev), act=1)
    assert rel(nchw(y), F.relu(pre + b[None, :, None, None])) < 4e-3
    y, _, _ = rr.ops.igemm(RR_CONV1X1, nhwc(x, dev), None, n, h, w, wf, 64, mask=nhwc(m, dev))
    assert rel(nchw(y), torch.where(m > 0, pre, torch.zeros(()))) < 4e-3


@pytest.mark.parametrize("shape", SHAPES)
def test_stream1_final_conv_nchw(dev, small_ok, shape):
    """ResUNet final 1x1 conv 64 -> 3: fp32 NCHW output at the model boundary"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV1X1
    n, h, w = shape
    x = rnd(n, 64, h, w, seed=31).bfloat16().float()
    wt = (rnd(3, 64, 1, 1, seed=32) / 8.0).bfloat16().float()
    b = rnd(3, seed=33)
    wf, _ = rr.ops.pack_conv(wt.to(dev), BF)
    assert _name(RR_CONV1X1, n, h, w, 64, 0, 3, bias=1, nchw_=1) == "stream1_kernel<1,2>"
    y, _, _ = rr.ops.igemm(RR_CONV1X1, nhwc(x, dev), None, n, h, w, wf, 3, bias=b.to(dev),
                           out_nchw=True)
    assert y.dtype == torch.float32 and y.shape == (n, 3, h, w)
    ref = F.conv2d(x, wt, b)
    assert (y.cpu() - ref).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())


# the reference's 224-pipeline maps (14:202-205: 28 / 56 / 112 / 224) are not
# powers of two: image / row / column of a coarse pixel by invariant division
SHAPES_NP2 = [(8, 14, 14), (3, 28, 28), (2, 28, 56)]


@pytest.mark.parametrize("shape", SHAPES + SHAPES_NP2)
@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 64), (256, 128)])
def test_stream1_convT(dev, small_ok, shape, cin, cout, monkeypatch):
    """ConvTranspose2d(cin, cout, 2, stride=2) fwd (scatter by GEMM column)
    and its dgrad (4-tap gather from the fine grid, with a relu mask)"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONVT_DOWN, RR_CONVT_UP
    n, h, w = shape
    x = rnd(n, cin, h, w, seed=41).bfloat16().float()
    wt = (rnd(cin, cout, 2, 2, seed=42) / cin ** 0.5).bfloat16().float()
    b = rnd(cout, seed=43)
    g = rnd(n, cout, 2 * h, 2 * w, seed=44).bfloat16().float()
    m = rnd(n, cin, h, w, seed=45).bfloat16().float()
    wu, wdn = rr.ops.pack_convT(wt.to(dev), BF)
    b4 = rr.ops.bias_tile4(b.to(dev))
    kb_up, kb_dn = cin // 32, 4 * cout // 32
    if kb_up in (2, 4, 6, 8, 12):
        assert _name(RR_CONVT_UP, n, h, w, cin, 0, 4 * cout, bias=1).startswith("stream1")
    # the convT dgrad (2x2 gather) stays on the tiled kernel (measured faster)
    assert _name(RR_CONVT_DOWN, n, h, w, cout, 0, cin, mask=1).startswith("igemm_kernel")
    res = {}
    for tag in ("1", "0"):
        set_path(monkeypatch, "stream1", tag)
        y, _, _ = rr.ops.igemm(RR_CONVT_UP, nhwc(x, dev), None, n, h, w, wu, 4 * cout, bias=b4)
        gx, _, _ = rr.ops.igemm(RR_CONVT_DOWN, nhwc(g, dev), None, n, h, w, wdn, cin,
                                mask=nhwc(m, dev))
        torch.cuda.synchronize()
        res[tag] = (nchw(y), nchw(gx))
    y, gx = res["1"]
    assert rel(y, F.conv_transpose2d(x, wt, b, stride=2)) < 4e-3
    assert rel(gx, torch.where(m > 0, F.conv2d(g, wt, stride=2), torch.zeros(()))) < 4e-3
    assert rel(y, res["0"][0]) < 1e-3
    assert rel(gx, res["0"][1]) < 1e-3

