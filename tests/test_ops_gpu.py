"""Per-op parity of the HIP kernels against the CPU oracle (ATen fp32 ops the
reference dispatches), small shapes.  fp32 path: tight tolerances (the f32
MFMA is an exact fp32 FMA chain; only the summation order differs); bf16:
relative tolerances of bf16 storage."""
import pytest
import torch
import torch.nn.functional as F
from rrpath import set_path  # noqa: E402

pytestmark = pytest.mark.gpu

TOL = {torch.float32: (2e-4, 2e-5), torch.bfloat16: (3e-2, 3e-2)}


def nhwc(x, dev, dt):
    return x.permute(0, 2, 3, 1).contiguous().to(dev, dt)


def nchw(y):
    return y.float().permute(0, 3, 1, 2).contiguous().cpu()


def close(a, b, dt, scale=None):
    """fp32: max-abs error relative to the tensor scale.  bf16: relative L2
    error (bf16 storage flips a few ReLU/PReLU masks near 0, so a max-abs
    bound would test the rounding of single elements, not the kernel)."""
    a = a.float().cpu()
    b = b.float()
    if dt == torch.float32:
        rtol, atol = TOL[dt]
        s = scale if scale is not None else max(1.0, b.abs().max().item())
        err = (a - b).abs().max().item()
        assert err <= atol * s, (err, s)
    else:
        rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert rel <= 5e-2, rel


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 8, 8, 64, 64), (1, 5, 7, 128, 64), (2, 16, 16, 64, 256),
                                            (3, 9, 4, 192, 128)])
def test_conv3x3_fwd(dev, dt, n, h, w, cin, cout):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    x = rnd(n, cin, h, w, seed=1)
    wt = rnd(cout, cin, 3, 3, seed=2) * 0.05
    b = rnd(cout, seed=3)
    if dt == torch.bfloat16:
        x, wt = x.bfloat16().float(), wt.bfloat16().float()
    ref = F.relu(F.conv2d(x, wt, b, padding=1))
    wf, wd = rr.ops.pack_conv(wt.to(dev), dt)
    y, _, st = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev, dt), None, n, h, w, wf, cout,
                            bias=b.to(dev), act=1, stats=True)
    close(nchw(y), ref, dt)
    # stats of the pre-bias accumulator
    pre = F.conv2d(x, wt, None, padding=1)
    s = st.cpu().double().sum(0)
    mag = pre.abs().sum((0, 2, 3)).max().item()
    tol = (1e-5 if dt == torch.float32 else 1e-2) * mag
    assert (s[:, 0] - pre.double().sum((0, 2, 3))).abs().max().item() <= tol
    assert (s[:, 1] - (pre.double() ** 2).sum((0, 2, 3))).abs().max().item() <= \
        tol * pre.abs().max().item() * 2


# halo-eligible bf16 shapes: (n, h, w, c1, c2, cout, split) -- whole-row
# 256-pixel tiles (W in {8,16,32,64}), one tile spanning 4 images at 8x8,
# BC = 128 and 64 column tiles, concat sources and dgrad-style column split
HALO_SHAPES = [(4, 8, 8, 64, 64, 128, 0), (2, 16, 16, 64, 0, 64, 0), (1, 32, 32, 128, 0, 192, 0),
               (1, 8, 64, 64, 128, 128, 64), (8, 8, 8, 256, 0, 512, 256), (2, 16, 32, 64, 0, 256, 128)]


@pytest.mark.parametrize("halo", [True, False])
@pytest.mark.parametrize("shape", HALO_SHAPES)
def test_conv3x3_halo(dev, shape, halo, monkeypatch):
    """bf16 3x3 conv through the LDS-halo igemm (and the per-tap kernel for
    A/B): bias + ReLU + BN partial stats, concat input, column split with a
    relu-backward mask, accumulate.  Inputs bf16-exact, so vs fp32 torch the
    only error is the bf16 rounding of the output."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "igemm_halo", 1 if halo else 0)
    n, h, w, c1, c2, cout, split = shape
    cin = c1 + c2
    x = rnd(n, cin, h, w, seed=41).bfloat16().float()
    wt = (rnd(cout, cin, 3, 3, seed=42) * (1.0 / (3 * cin ** 0.5))).bfloat16().float()
    b = rnd(cout, seed=43)
    wf, _ = rr.ops.pack_conv(wt.to(dev), torch.bfloat16)
    bf = torch.bfloat16
    x1 = nhwc(x[:, :c1], dev, bf)
    x2 = nhwc(x[:, c1:], dev, bf) if c2 else None
    pre = F.conv2d(x, wt, None, padding=1)

    def rel(a, r):
        return ((a - r).norm() / r.norm()).item()

    if not split:
        y, _, st = rr.ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, cout, bias=b.to(dev), act=1,
                                stats=True)
        assert rel(nchw(y), F.relu(pre + b[None, :, None, None])) < 4e-3
        s = st.cpu().double().sum(0)
        assert rel(s[:, 0], pre.double().sum((0, 2, 3))) < 1e-5
        assert rel(s[:, 1], (pre.double() ** 2).sum((0, 2, 3))) < 1e-5
    else:
        # split columns [0, split) -> y1 (masked, accumulated), [split, cout) -> y2
        mask = rnd(n, split, h, w, seed=44)
        acc0 = rnd(n, split, h, w, seed=45).bfloat16().float()
        acc2 = rnd(n, cout - split, h, w, seed=46).bfloat16().float()
        y1, y2 = nhwc(acc0, dev, bf), nhwc(acc2, dev, bf)
        # accumulate applies to both column halves (the dgrad of a concat)
        y1, y2, _ = rr.ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf, cout, out=y1, out2=y2,
                                 split=split, accumulate=True, mask=None)
        assert rel(nchw(y1), pre[:, :split] + acc0) < 4e-3
        assert rel(nchw(y2), pre[:, split:] + acc2) < 4e-3
        # a plain masked conv over the first split columns
        wf2, _ = rr.ops.pack_conv(wt[:split].to(dev), bf)
        ym, _, _ = rr.ops.igemm(RR_CONV3X3, x1, x2, n, h, w, wf2, split, mask=nhwc(mask, dev, bf))
        refm = torch.where(mask.bfloat16().float() > 0, pre[:, :split], torch.zeros(()))
        assert rel(nchw(ym), refm) < 4e-3


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_concat_dgrad_split(dev, dt):
    """cat((up, skip), 1) read in place (07:112) and the dgrad split."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, h, w, c1, c2, cout = 2, 8, 8, 128, 64, 64
    x1, x2 = rnd(n, c1, h, w, seed=4), rnd(n, c2, h, w, seed=5)
    wt = rnd(cout, c1 + c2, 3, 3, seed=6) * 0.05
    if dt == torch.bfloat16:
        x1, x2, wt = x1.bfloat16().float(), x2.bfloat16().float(), wt.bfloat16().float()
    xc = torch.cat((x1, x2), 1).requires_grad_(True)
    ref = F.conv2d(xc, wt, None, padding=1)
    g = rnd(*ref.shape, seed=7)
    if dt == torch.bfloat16:
        g = g.bfloat16().float()
    ref.backward(g)
    wf, wd = rr.ops.pack_conv(wt.to(dev), dt)
    y, _, _ = rr.ops.igemm(RR_CONV3X3, nhwc(x1, dev, dt), nhwc(x2, dev, dt), n, h, w, wf, cout)
    close(nchw(y), ref.detach(), dt)
    g1, g2, _ = rr.ops.igemm(RR_CONV3X3, nhwc(g, dev, dt), None, n, h, w, wd, c1 + c2, split=c1)
    close(nchw(g1), xc.grad[:, :c1], dt)
    close(nchw(g2), xc.grad[:, c1:], dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("k", [3, 1])
def test_wgrad(dev, dt, k):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV1X1, RR_CONV3X3
    n, h, w, cin, cout = 3, 12, 10, 128, 64
    x = rnd(n, cin, h, w, seed=8)
    g = rnd(n, cout, h, w, seed=9)
    if dt == torch.bfloat16:
        x, g = x.bfloat16().float(), g.bfloat16().float()
    wt = torch.zeros(cout, cin, k, k, requires_grad=True)
    F.conv2d(x, wt, None, padding=k // 2).backward(g)
    dw = rr.ops.wgrad(RR_CONV3X3 if k == 3 else RR_CONV1X1, nhwc(g, dev, dt), nhwc(x, dev, dt),
                      None, n, h, w, cout, dw_shape=(cout, cin, k, k))
    close(dw.cpu(), wt.grad, dt, scale=wt.grad.abs().max().item())


@pytest.mark.parametrize("shape", [(3, 3, 12, 10, 128, 64), (1, 3, 16, 16, 64, 128), (1, 3, 64, 64, 64, 64),
                                   (1, 1, 32, 32, 64, 64), (2, 2, 8, 8, 128, 64)])
def test_wgrad_partial_reduce_on_another_stream(dev, shape):
    """rr_wgrad_partial + rr_wgrad_reduce, the reduce on a side stream
    (ops.wgrad(reduce_stream=...)), == rr_wgrad bit for bit, accumulate too
    (swgrad, halo, tiled and convT kernels)"""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV1X1, RR_CONV3X3, RR_CONVT_UP
    n, k, h, w, cin, cout = shape
    mode = {3: RR_CONV3X3, 1: RR_CONV1X1, 2: RR_CONVT_UP}[k]
    x = nhwc(rnd(n, cin, h, w, seed=61), dev, torch.bfloat16)
    gh, gw = (2 * h, 2 * w) if k == 2 else (h, w)
    g = nhwc(rnd(n, cout, gh, gw, seed=62), dev, torch.bfloat16)
    shp = (cin, cout, 2, 2) if k == 2 else (cout, cin, k, k)
    side = torch.cuda.Stream(dev)
    for acc in (False, True):
        base = rnd(*shp, seed=63).to(dev)
        ref = rr.ops.wgrad(mode, g, x, None, n, h, w, cout, dw=base.clone(), accumulate=acc)
        got = rr.ops.wgrad(mode, g, x, None, n, h, w, cout, dw=base.clone(), accumulate=acc,
                           reduce_stream=side)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        assert torch.equal(got, ref), (shape, acc)


@pytest.mark.parametrize("hw", [(8, 8), (16, 16), (12, 32), (2, 64), (1, 8, 8), (3, 8, 8), (1, 16, 16)])
@pytest.mark.parametrize("halo", [True, False])
def test_wgrad3_halo(dev, hw, halo, monkeypatch):
    """bf16 3x3 weight grad through the LDS-halo kernel (64-pixel stages of
    whole image rows, zero-padded halo) and through the per-tap kernel, with a
    concat second source (dec*.c1 shape), vs fp32 torch.  (n, h, w) cases
    give splits of 1-3 stages: the prefetching loop runs past a split's end
    with clamped loads and LDS writes no stage reads."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    set_path(monkeypatch, "wgrad_halo", 1 if halo else 0)
    n = 5
    if len(hw) == 3:
        n, hw = hw[0], hw[1:]
    h, w = hw
    c1, c2, cout = 64, 128, 128
    x = rnd(n, c1 + c2, h, w, seed=30).bfloat16().float()
    g = rnd(n, cout, h, w, seed=31).bfloat16().float()
    wt = torch.zeros(cout, c1 + c2, 3, 3, requires_grad=True)
    F.conv2d(x, wt, None, padding=1).backward(g)
    dw = rr.ops.wgrad(RR_CONV3X3, nhwc(g, dev, torch.bfloat16), nhwc(x[:, :c1], dev, torch.bfloat16),
                      nhwc(x[:, c1:], dev, torch.bfloat16), n, h, w, cout,
                      dw_shape=(cout, c1 + c2, 3, 3))
    # inputs are bf16-exact and products are exact in fp32: only the
    # summation order differs from torch
    rel = ((dw.cpu() - wt.grad).norm() / wt.grad.norm()).item()
    assert rel < 2e-5, rel


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,h,w,C", [(4, 8, 8, 128), (2, 16, 16, 64), (4, 8, 8, 256), (1, 8, 64, 64)])
def test_igemm_bnbwd_fused(dev, dt, n, h, w, C):
    """conv dgrad + BN/PReLU backward reduce fused in the epilogue
    (rr_igemm_bnbwd + rr_bn_bwd_finalize_rows) == the unfused sequence
    (rr_igemm, then rr_bn_bwd_reduce/finalize/apply with mask_kind 2)."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    ops = rr.ops
    g2 = nhwc(rnd(n, C, h, w, seed=51), dev, dt)
    wt = (rnd(C, C, 3, 3, seed=52) * (1.0 / (3 * C ** 0.5))).to(dev)
    _, wd = ops.pack_conv(wt, dt)
    t1 = nhwc(rnd(n, C, h, w, seed=53) * 2 + 0.3, dev, dt)
    tf = t1.float().reshape(-1, C)
    mean = tf.mean(0)
    inv = 1.0 / torch.sqrt(tf.var(0, unbiased=False) + 1e-5)
    gamma = (torch.rand(C, generator=torch.Generator().manual_seed(54)) + 0.5).to(dev)
    beta = (torch.rand(C, generator=torch.Generator().manual_seed(55)) - 0.5).to(dev)
    s1 = gamma * inv
    sh1 = beta - mean * s1
    alpha = torch.tensor([0.23], device=dev)
    da1, _, _ = ops.igemm(RR_CONV3X3, g2, None, n, h, w, wd, C)
    ref = ops.bn_backward(da1, t1, mean, inv, gamma, mask_kind=2, aux=t1, aff_s=s1, aff_b=sh1,
                          alpha=alpha)
    gm, part, rows, arows = ops.igemm_bnbwd(RR_CONV3X3, g2, n, h, w, wd, C, t1, mean, inv, s1, sh1,
                                            alpha)
    got = ops.bn_backward_rows(gm, part, rows, arows, t1, mean, inv, gamma)
    torch.cuda.synchronize()
    tol = 1e-5 if dt == torch.float32 else 2e-2   # bf16: the unfused path rounds da1 first

    def rel(a, b):
        a, b = a.float().cpu(), b.float().cpu()
        return ((a - b).norm() / b.norm()).item()
    assert rel(got["dt0"], ref["dt0"]) < tol
    for k in ("dgamma0", "dbeta0", "dalpha"):
        assert rel(got[k], ref[k]) < tol, k


@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("n,h,w", [(4, 8, 8), (2, 64, 64), (1, 16, 32), (1, 5, 7), (3, 40, 16),
                                   (1, 20, 112)])
def test_image_grad(dev, n, h, w, acc):
    """Image grad of the perceptual slice's conv1_1 (64 -> 3, 14:189): bf16
    dgrad into fp32 NCHW -- the narrow 16-column halo tile where eligible,
    the per-tap igemm otherwise -- with accumulate."""
    import roadrestore as rr
    ops = rr.ops
    g = rnd(n, 64, h, w, seed=71).bfloat16().float()
    wt = (rnd(64, 3, 3, 3, seed=72) * 0.1).bfloat16().float()
    x = torch.zeros(n, 3, h, w, requires_grad=True)
    F.conv2d(x, wt, None, padding=1).backward(g)
    base = rnd(n, 3, h, w, seed=73)
    _, wd = ops.pack_conv(wt.to(dev), torch.bfloat16)
    out = base.clone().to(dev) if acc else None
    y = ops.conv_in_dgrad(nhwc(g, dev, torch.bfloat16), wt.to(dev), 3, out=out, accumulate=acc,
                          wpack_dgrad=wd)
    ref = x.grad + (base if acc else 0)
    assert ((y.cpu() - ref).norm() / ref.norm()).item() < 1e-5


@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("n,h,w", [(33, 64, 64), (48, 64, 64), (97, 64, 64), (160, 32, 32)])
def test_image_grad_persistent(dev, n, h, w, acc):
    """The same image grad past 512 tiles of 256 pixels, where the kernel runs
    persistent (512 workgroups walking tiles with two tiles' halos in flight):
    1, 2 and 3 tiles per workgroup with ragged tails, against fp32 torch."""
    import roadrestore as rr
    ops = rr.ops
    g = rnd(n, 64, h, w, seed=74).bfloat16().float()
    wt = (rnd(64, 3, 3, 3, seed=75) * 0.1).bfloat16().float()
    x = torch.zeros(n, 3, h, w, requires_grad=True)
    F.conv2d(x, wt, None, padding=1).backward(g)
    base = rnd(n, 3, h, w, seed=76)
    _, wd = ops.pack_conv(wt.to(dev), torch.bfloat16)
    out = base.clone().to(dev) if acc else None
    y = ops.conv_in_dgrad(nhwc(g, dev, torch.bfloat16), wt.to(dev), 3, out=out, accumulate=acc,
                          wpack_dgrad=wd)
    ref = x.grad + (base if acc else 0)
    assert ((y.cpu() - ref).norm() / ref.norm()).item() < 1e-5
    # every image's grad matches on its own (no tile lost or written twice)
    per = ((y.cpu() - ref).flatten(1).norm(dim=1) / ref.flatten(1).norm(dim=1))
    assert per.max().item() < 1e-5


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("n,h,w", [(2, 16, 16), (1, 5, 7), (3, 64, 64)])
def test_first_conv_fused(dev, act, n, h, w):
    """bf16 fused first conv (rr_conv_in_mfma) vs the im2col + K=64 igemm
    path and vs fp32 torch on bf16-rounded inputs (07:78, 14:122, VGG f[0])."""
    import roadrestore as rr
    ops = rr.ops
    x = torch.rand(n, 3, h, w, generator=torch.Generator().manual_seed(61))
    wt = rnd(64, 3, 3, 3, seed=62) * 0.2
    b = rnd(64, seed=63) * 0.1
    alpha = torch.tensor([0.2])
    xb, wb = x.bfloat16().float(), wt.bfloat16().float()
    pre_ref = F.conv2d(xb, wb, b.bfloat16().float(), padding=1)
    ref = {0: pre_ref, 1: F.relu(pre_ref), 2: F.prelu(pre_ref, alpha)}[act]
    wp = ops.pack_conv_in(wt.to(dev), b.to(dev), torch.bfloat16)
    assert wp.numel() == 64 * ops.KPAD_MFMA
    y, pre = ops.first_conv_fwd(x.to(dev), wt.to(dev), b.to(dev), torch.bfloat16, wp, act=act,
                                alpha=alpha.to(dev), want_pre=True)

    def rel(a, r):
        return ((nchw(a) - r).norm() / r.norm()).item()
    assert rel(y, ref) < 4e-3
    assert rel(pre, pre_ref) < 4e-3
    # same math as the im2col + igemm (K = 64) path
    col = ops.im2col3(x.to(dev), torch.bfloat16)
    wp64 = ops.pack_conv_in(wt.to(dev), b.to(dev), torch.bfloat16, kpad=ops.KPAD_IN)
    from roadrestore._lib import RR_CONV1X1
    y64, _, _ = ops.igemm(RR_CONV1X1, col, None, n, h, w, wp64, 64)
    assert ((pre.float() - y64.float()).norm() / y64.float().norm()).item() < 1e-3


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_convT(dev, dt):
    import roadrestore as rr
    from roadrestore._lib import RR_CONVT_DOWN, RR_CONVT_UP
    n, h, w, cin, cout = 2, 4, 6, 128, 64
    x = rnd(n, cin, h, w, seed=10).requires_grad_(True)
    wt = (rnd(cin, cout, 2, 2, seed=11) * 0.05).requires_grad_(True)
    b = rnd(cout, seed=12)
    if dt == torch.bfloat16:
        with torch.no_grad():
            x.copy_(x.bfloat16().float()); wt.copy_(wt.bfloat16().float())
    ref = F.conv_transpose2d(x, wt, b, stride=2)
    g = rnd(*ref.shape, seed=13)
    if dt == torch.bfloat16:
        g = g.bfloat16().float()
    ref.backward(g)
    wu, wdn = rr.ops.pack_convT(wt.detach().to(dev), dt)
    y, _, _ = rr.ops.igemm(RR_CONVT_UP, nhwc(x.detach(), dev, dt), None, n, h, w, wu, 4 * cout,
                           bias=rr.ops.bias_tile4(b.to(dev)))
    close(nchw(y), ref.detach(), dt)
    gx, _, _ = rr.ops.igemm(RR_CONVT_DOWN, nhwc(g, dev, dt), None, n, h, w, wdn, cin)
    close(nchw(gx), x.grad, dt)
    dw = rr.ops.wgrad(RR_CONVT_UP, nhwc(g, dev, dt), nhwc(x.detach(), dev, dt), None, n, h, w,
                      cout, dw_shape=(cin, cout, 2, 2))
    close(dw.cpu(), wt.grad, dt, scale=wt.grad.abs().max().item())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bn_train_fwd_bwd(dev, dt):
    """BatchNorm2d train fwd (batch stats, running update) + PReLU, and the
    fused backward (mask kinds 1 and 2)."""
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    n, h, w, cin, C = 4, 8, 8, 64, 64
    x = rnd(n, cin, h, w, seed=14)
    wt = rnd(C, cin, 3, 3, seed=15) * 0.05
    b = rnd(C, seed=16)
    gamma, beta = rnd(C, seed=17).abs() + 0.5, rnd(C, seed=18) * 0.1
    alpha = torch.tensor([0.25])
    if dt == torch.bfloat16:
        x, wt = x.bfloat16().float(), wt.bfloat16().float()
    t = F.conv2d(x, wt, b, padding=1)
    tr = t.detach().requires_grad_(True)
    gam, bet, alp = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True), alpha.clone().requires_grad_(True)
    rm, rv = torch.zeros(C), torch.ones(C)
    u = F.batch_norm(tr, rm, rv, gam, bet, True, 0.1, 1e-5)
    a = F.prelu(u, alp)
    g = rnd(*a.shape, seed=19)
    a.backward(g)
    wf, _ = rr.ops.pack_conv(wt.to(dev), dt)
    tt, _, st = rr.ops.igemm(RR_CONV3X3, nhwc(x, dev, dt), None, n, h, w, wf, C, bias=b.to(dev), stats=True)
    rmd, rvd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    nbt = torch.zeros((), dtype=torch.long, device=dev)
    scale, shift, mean, inv = rr.ops.bn_finalize(st, n * h * w, b.to(dev), gamma.to(dev), beta.to(dev),
                                                 rmd, rvd, 0.1, 1e-5, nbt)
    aa = rr.ops.affine_act(tt, scale, shift, alpha=alpha.to(dev))
    close(nchw(aa), a.detach(), dt)
    torch.testing.assert_close(rmd.cpu(), rm, rtol=1e-4 if dt == torch.float32 else 3e-2, atol=1e-4)
    torch.testing.assert_close(rvd.cpu(), rv, rtol=1e-4 if dt == torch.float32 else 3e-2, atol=1e-4)
    assert nbt.item() == 1
    gd = nhwc(g, dev, dt)
    r = rr.ops.bn_backward(gd, tt, mean, inv, gamma.to(dev), mask_kind=2, aux=tt, aff_s=scale,
                           aff_b=shift, alpha=alpha.to(dev))
    close(nchw(r["dt0"]), tr.grad, dt)
    close(r["dgamma0"].cpu(), gam.grad, dt, scale=gam.grad.abs().max().item())
    close(r["dbeta0"].cpu(), bet.grad, dt, scale=bet.grad.abs().max().item())
    close(r["dalpha"].cpu(), alp.grad, dt, scale=alp.grad.abs().max().item())


@pytest.mark.parametrize("rows_a,rows_b,C", [(256, 8192, 64), (37, 2071, 128), (9001, 16, 32)])
def test_bn_finalize_pair_equals_two_launches(dev, rows_a, rows_b, C):
    """rr_bn_finalize_pair (tail BN + shortcut BN in one launch) == two
    rr_bn_finalize calls, bit for bit: scale / shift / mean / invstd, running
    stats and num_batches_tracked (and the > 8192-row fallback)."""
    import roadrestore as rr
    g = torch.Generator().manual_seed(rows_a + rows_b)

    def make(rows):
        st = torch.randn(rows, C, 2, generator=g)
        st[..., 1] = st[..., 1].abs() * 4.0 + 2.0
        return dict(st=st.to(dev), count=rows * 16, bias=torch.randn(C, generator=g).to(dev),
                    gamma=torch.randn(C, generator=g).to(dev), beta=torch.randn(C, generator=g).to(dev),
                    running_mean=torch.randn(C, generator=g).to(dev),
                    running_var=torch.rand(C, generator=g).to(dev) + 0.5, momentum=0.1, eps=1e-5,
                    num_batches_tracked=torch.zeros((), dtype=torch.long, device=dev))

    a, b = make(rows_a), make(rows_b)
    a2 = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in a.items()}
    b2 = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in b.items()}
    ra, rb = rr.ops.bn_finalize_pair(a, b)
    sa, sb = rr.ops.bn_finalize(**a2), rr.ops.bn_finalize(**b2)
    for got, want in ((ra, sa), (rb, sb)):
        for x, y in zip(got, want):
            assert torch.equal(x, y)
    for k in ("running_mean", "running_var", "num_batches_tracked"):
        assert torch.equal(a[k], a2[k]) and torch.equal(b[k], b2[k]), k
    assert a["num_batches_tracked"].item() == 1 and b["num_batches_tracked"].item() == 1


@pytest.mark.parametrize("rows,C", [(1, 64), (37, 64), (2071, 128), (8192, 64), (9001, 32)])
def test_bn_finalize_partials_and_pair_out(dev, rows, C):
    """Statistics finalize from raw per-tile partials [rows][C][2]: the direct
    path (<= 8192 rows) and the column-reduce path, with row counts that end
    inside and outside a batch of in-flight loads (rr_fixed_sum); against an
    fp64 torch sum, and ``out=`` rows of a [2, C] pair equal to the default
    outputs bit for bit."""
    import roadrestore as rr
    g = torch.Generator().manual_seed(rows * 7 + C)
    st = torch.randn(rows, C, 2, generator=g)
    st[..., 1] = st[..., 1].abs() * 4.0 + 2.0
    count = rows * 16
    bias, gamma, beta = (torch.randn(C, generator=g) for _ in range(3))
    s64 = st.double().sum(0)
    mean_acc = s64[:, 0] / count
    var = (s64[:, 1] / count - mean_acc ** 2).clamp_min(0)
    inv = 1.0 / torch.sqrt(var + 1e-5)
    want_scale = (gamma.double() * inv).float()
    want_shift = (beta.double() - (mean_acc + bias.double()) * gamma.double() * inv).float()
    mean = mean_acc + bias.double()
    want_rm = (0.1 * mean).float()                               # (1 - m) * 0 + m * mean
    want_rv = (0.9 + 0.1 * var * count / (count - 1)).float()    # unbiased update
    outs = []
    for pair in (None, (torch.empty(2, C, device=dev), torch.empty(2, C, device=dev))):
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.long, device=dev)
        o = (pair[0][1], pair[1][1]) if pair else None
        sc, sh, sm, si = rr.ops.bn_finalize(st.to(dev), count, bias.to(dev), gamma.to(dev),
                                            beta.to(dev), rm, rv, 0.1, 1e-5, nbt, out=o)
        if pair:
            assert sc.data_ptr() == pair[0][1].data_ptr() and sh.data_ptr() == pair[1][1].data_ptr()
        outs.append((sc.cpu(), sh.cpu()))
        torch.testing.assert_close(rm.cpu(), want_rm, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(rv.cpu(), want_rv, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(sm.cpu(), mean.float(), rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(si.cpu(), inv.float(), rtol=1e-6, atol=1e-6)
        assert nbt.item() == 1
    torch.testing.assert_close(outs[0][0], want_scale, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(outs[0][1], want_shift, rtol=1e-6, atol=1e-6)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,h,w", [(64, 8, 10), (12, 9, 11), (128, 7, 6)])
def test_maxpool(dev, dt, C, h, w):
    """8-channel (C % 8 == 0) and 4-channel kernels, floor mode on odd sizes"""
    import roadrestore as rr
    n = 2
    x = F.relu(rnd(n, C, h, w, seed=20))          # many exact-zero ties after ReLU
    x[0, 0, 0, :4] = 1.0                            # explicit ties inside a window
    if dt == torch.bfloat16:
        x = x.bfloat16().float()
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 2, 2)
    g = rnd(*y.shape, seed=21)
    if dt == torch.bfloat16:
        g = g.bfloat16().float()
    y.backward(g)
    yd, idx = rr.ops.maxpool2_fwd(nhwc(x, dev, dt))
    close(nchw(yd), y.detach(), dt)
    gx = rr.ops.maxpool2_bwd(nhwc(g, dev, dt), idx, h, w)
    assert torch.equal(nchw(gx) != 0, xr.grad != 0)
    close(nchw(gx), xr.grad, dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_first_last_layers(dev, dt):
    import roadrestore as rr
    n, h, w = 2, 12, 8
    x = torch.rand(n, 3, h, w)
    w0 = (rnd(64, 3, 3, 3, seed=22) * 0.2).requires_grad_(True)
    b0 = rnd(64, seed=23).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y0 = F.conv2d(xr, w0, b0, padding=1)
    y = rr.ops.conv_in_fwd(x.to(dev), w0.detach().to(dev), b0.detach().to(dev), dt, act=0)
    close(nchw(y), y0.detach(), dt)
    g = rnd(*y0.shape, seed=24)
    if dt == torch.bfloat16:
        g = g.bfloat16().float()
    y0.backward(g)
    dw, db = rr.ops.conv_in_wgrad(x.to(dev), nhwc(g, dev, dt), dw_shape=(64, 3, 3, 3))
    close(dw.cpu(), w0.grad, dt, scale=w0.grad.abs().max().item())
    close(db.cpu(), b0.grad, dt, scale=b0.grad.abs().max().item())
    gx = rr.ops.conv_in_dgrad(nhwc(g, dev, dt), w0.detach().to(dev), 3)
    close(gx.cpu(), xr.grad, dt, scale=xr.grad.abs().max().item())
    # last layer 64 -> 3 (1x1)
    a = F.relu(rnd(n, 64, h, w, seed=25))
    if dt == torch.bfloat16:
        a = a.bfloat16().float()
    ar = a.clone().requires_grad_(True)
    wl = (rnd(3, 64, 1, 1, seed=26) * 0.1).requires_grad_(True)
    bl = rnd(3, seed=27).requires_grad_(True)
    o = F.conv2d(ar, wl, bl)
    od = rr.ops.conv_out_fwd(nhwc(a, dev, dt), wl.detach().to(dev), bl.detach().to(dev))
    close(od.cpu(), o.detach(), dt)
    go = rnd(*o.shape, seed=28)
    o.backward(go)
    dx, dwl, dbl = rr.ops.conv_out_bwd(go.to(dev), nhwc(a, dev, dt), wl.detach().to(dev), mask_relu=True)
    close(nchw(dx), ar.grad * (a > 0), dt)
    close(dwl.cpu(), wl.grad, dt, scale=wl.grad.abs().max().item())
    close(dbl.cpu(), bl.grad, dt, scale=bl.grad.abs().max().item())


def test_losses_adamw_postproc(dev):
    import numpy as np
    import roadrestore as rr
    from oracle import reference_cpu as R
    a, b = torch.rand(2, 3, 16, 16), torch.rand(2, 3, 16, 16)
    l1 = rr.ops.loss_fwd(rr.ops.L1, a.to(dev), b.to(dev))
    mse = rr.ops.loss_fwd(rr.ops.MSE, a.to(dev), b.to(dev))
    assert abs(l1.item() - R.l1_loss(a, b).item()) < 1e-6
    assert abs(mse.item() - R.mse_loss(a, b).item()) < 1e-6
    ar = a.clone().requires_grad_(True)
    R.l1_loss(ar, b).backward()
    g = rr.ops.loss_bwd(rr.ops.L1, a.to(dev), b.to(dev))
    torch.testing.assert_close(g.cpu(), ar.grad)
    # AdamW vs the restated torch update order
    p = rnd(1000, seed=30)
    gr = rnd(1000, seed=31)
    pd, gd = p.to(dev), gr.to(dev)
    m, v = torch.zeros_like(pd), torch.zeros_like(pd)
    st = {}
    ref = {"p": p.clone()}
    for step in (1, 2, 3):
        rr.ops.adamw_(pd, gd, m, v, 2e-4, 0.9, 0.999, 1e-8, 1e-4, True, step)
        R.adamw_step(ref, {"p": gr}, st, 2e-4, weight_decay=1e-4)
    torch.testing.assert_close(pd.cpu(), ref["p"], rtol=1e-6, atol=1e-7)
    # uint8 truncation + PSNR (17:89-92, 08:123)
    o = torch.rand(2, 3, 16, 16) * 1.2 - 0.1
    u8 = rr.ops.to_uint8_hwc(o.to(dev)).cpu().numpy()
    assert np.array_equal(u8, R.to_uint8_image(o))
    c8 = R.to_uint8_image(torch.rand(2, 3, 16, 16))
    ps = rr.ops.psnr_u8(torch.from_numpy(u8).to(dev), torch.from_numpy(c8).to(dev)).cpu().numpy()
    for i in range(2):
        assert abs(ps[i] - R.psnr_u8(c8[i], u8[i])) < 1e-9
    lg = rnd(9, 43, seed=32)
    lg[3, 5] = lg[3, 7] = lg[3].max() + 1       # tie: first index wins (18:47)
    assert torch.equal(rr.ops.argmax_rows(lg.to(dev)).cpu(), R.top1(lg))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_pack_conv_batch_equals_single_packs(dev, dt):
    """rr_pack_conv_batch (one launch for a network's convs) == rr_pack_conv
    per weight, bitwise, including 1x1 and fwd-only entries"""
    from roadrestore import ops
    shapes = [(64, 3, 3, True), (64, 64, 3, True), (128, 64, 1, True), (3, 64, 1, False),
              (512, 256, 3, True), (7, 5, 3, False), (16, 12, 3, True), (128, 384, 3, True),
              (20, 24, 1, True)]
    ws = [rnd(co, ci, k, k, seed=i).to(dev) for i, (co, ci, k, _) in enumerate(shapes)]
    pb = ops.PackBatch([(w, dt, dg) for w, (_, _, _, dg) in zip(ws, shapes)])
    outs = pb.run()
    for w, (co, ci, k, dg), (bf, bd) in zip(ws, shapes, outs):
        sf, sd = ops.pack_conv(w, dt, True, dg)
        assert torch.equal(bf, sf)
        assert (bd is None) == (not dg)
        if dg:
            assert torch.equal(bd, sd)
    # in place: a weight update is picked up by the next run
    ws[1].mul_(2)
    outs = pb.run()
    assert torch.equal(outs[1][0], ops.pack_conv(ws[1], dt, True, True)[0])


@pytest.mark.parametrize("act", [1, 2])
@pytest.mark.parametrize("n,h,w", [(3, 16, 24), (2, 64, 64), (1, 8, 8)])
def test_first_conv_wgrad_act_fused(dev, act, n, h, w):
    """rr_conv_in_wgrad_act (ReLU/PReLU backward + first-conv wgrad from the
    image) against an fp64 CPU sum over the same bf16-rounded operands"""
    from roadrestore import ops
    x = torch.rand(n, 3, h, w, generator=torch.Generator().manual_seed(1))
    g = rnd(n, h, w, 64, seed=2).bfloat16()
    t = rnd(n, h, w, 64, seed=3).bfloat16()
    alpha = torch.tensor([0.25])
    dw = torch.full((64, 3, 3, 3), float("nan"), device=dev)
    db = torch.full((64,), float("nan"), device=dev)
    da = torch.full((1,), float("nan"), device=dev)
    ops.first_conv_wgrad_act(x.to(dev), g.to(dev), t.to(dev), act, alpha.to(dev), dw, db,
                             dalpha=da if act == 2 else None)
    gf, tf = g.float(), t.float()
    a = 0.25 if act == 2 else 0.0
    gp = torch.where(tf > 0, gf, a * gf).bfloat16().double()          # [n, h, w, 64]
    xb = x.bfloat16().double()
    xp = F.pad(xb, (1, 1, 1, 1))
    ref = torch.zeros(64, 3, 3, 3, dtype=torch.float64)
    for ky in range(3):
        for kx in range(3):
            patch = xp[:, :, ky:ky + h, kx:kx + w]                    # [n, 3, h, w]
            ref[:, :, ky, kx] = torch.einsum("nhwo,nchw->oc", gp, patch)
    refb = gp.sum((0, 1, 2))
    s = ref.abs().max().item()
    assert (dw.cpu().double() - ref).abs().max().item() <= 2e-4 * s
    assert (db.cpu().double() - refb).abs().max().item() <= 2e-4 * max(1.0, refb.abs().max().item())
    if act == 2:
        refa = (gf.double() * tf.double() * (tf <= 0)).sum().item()
        assert abs(da.item() - refa) <= 1e-4 * max(1.0, abs(refa))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shortcut", [False, True])
def test_affine_act_pool_equals_separate(dev, dt, shortcut):
    """rr_affine_act_pool == rr_affine_act then rr_maxpool2_fwd, bitwise
    (the pooling compares the stored, dtype-rounded values); ties included"""
    from roadrestore import ops
    n, h, w, C = 3, 8, 12, 64
    x = rnd(n, h, w, C, seed=1).to(dev, dt)
    x[:, 0::2, 0::2, :8] = x[:, 1::2, 1::2, :8]          # forced window ties
    res = rnd(n, h, w, C, seed=2).to(dev, dt)
    sc, sh = (rnd(C, seed=3) * 0.5 + 1).to(dev), rnd(C, seed=4).to(dev)
    rs, rb = ((rnd(C, seed=5) * 0.5 + 1).to(dev), rnd(C, seed=6).to(dev)) if shortcut else (None, None)
    y0 = ops.affine_act(x, sc, sh, res=res, res_scale=rs, res_shift=rb, relu=True)
    p0, i0 = ops.maxpool2_fwd(y0)
    y1, p1, i1 = ops.affine_act_pool(x, sc, sh, res=res, res_scale=rs, res_shift=rb, relu=True)
    assert torch.equal(y0, y1) and torch.equal(p0, p1) and torch.equal(i0, i1)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nbn", [1, 2])
def test_bn_backward_pool_fused(dev, dt, nbn):
    """mask kind 3 (the encoder max-pool backward inside the tail BN
    backward) == rr_maxpool2_bwd(accumulate) then mask kind 1; fp32 to
    rounding, bf16 within bf16 storage of the summed gradient"""
    from roadrestore import ops
    n, h, w, C = 2, 8, 12, 64
    g = rnd(n, h, w, C, seed=1).to(dev, dt)
    out = rnd(n, h, w, C, seed=2).to(dev, dt)
    t0 = rnd(n, h, w, C, seed=3).to(dev, dt)
    t1 = rnd(n, h, w, C, seed=4).to(dev, dt) if nbn == 2 else None
    _, idx = ops.maxpool2_fwd(out)
    pdy = rnd(n, h // 2, w // 2, C, seed=5).to(dev, dt)
    m0, i0 = rnd(C, seed=6).to(dev), (rnd(C, seed=7).abs() + 0.5).to(dev)
    m1, i1 = (rnd(C, seed=8).to(dev), (rnd(C, seed=9).abs() + 0.5).to(dev)) if nbn == 2 else (None, None)
    gam0 = rnd(C, seed=10).to(dev)
    gam1 = rnd(C, seed=11).to(dev) if nbn == 2 else None
    kw = dict(mask_kind=1, aux=out, t1=t1, mean1=m1, inv1=i1, gamma1=gam1, want_gm=True)
    fused = ops.bn_backward(g, t0, m0, i0, gam0, pool=(pdy, idx), **kw)
    g2 = g.clone()
    ops.maxpool2_bwd(pdy, idx, h, w, out=g2, accumulate=True)
    sep = ops.bn_backward(g2, t0, m0, i0, gam0, **kw)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    for k in ("dt0", "gm", "dgamma0", "dbeta0") + (("dt1", "dgamma1", "dbeta1") if nbn == 2 else ()):
        a, b = fused[k].float(), sep[k].float()
        rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert rel <= tol, (k, rel)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("C", [64, 512])
def test_bn_backward_gm_in_reduce(dev, dt, pool, C, monkeypatch):
    """identity-shortcut tail (one BN, gm wanted): the reduce that stores gm
    (rr_bn_bwd_reduce_gm) + the apply from gm alone == the apply that forms
    gm itself -- gm bit for bit, the rest within the rounding of gm to the
    storage dtype (fp32: to rounding); checked against fp64 torch too"""
    from roadrestore import ops
    n, h, w = 2, 8, 12
    g = rnd(n, h, w, C, seed=41).to(dev, dt)
    out = rnd(n, h, w, C, seed=42).to(dev, dt)
    t0 = rnd(n, h, w, C, seed=43).to(dev, dt)
    m0, i0 = rnd(C, seed=44).to(dev), (rnd(C, seed=45).abs() + 0.5).to(dev)
    gam0 = rnd(C, seed=46).to(dev)
    pl = None
    if pool:
        _, idx = ops.maxpool2_fwd(out)
        pl = (rnd(n, h // 2, w // 2, C, seed=47).to(dev, dt), idx)
    kw = dict(mask_kind=1, aux=out, want_gm=True, pool=pl)
    monkeypatch.setattr(ops, "_BN_GM_IN_REDUCE", False)
    ref = ops.bn_backward(g, t0, m0, i0, gam0, **kw)
    monkeypatch.setattr(ops, "_BN_GM_IN_REDUCE", True)
    got = ops.bn_backward(g, t0, m0, i0, gam0, **kw)
    assert torch.equal(got["gm"], ref["gm"])
    tol = 1e-5 if dt == torch.float32 else 1e-2
    for k in ("dt0", "dgamma0", "dbeta0"):
        a, b = got[k].float(), ref[k].float()
        rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert rel <= tol, (k, rel)
    # fp64: dt = gamma inv (gm - mean(gm) - xhat mean(gm xhat)) on the stored gm
    gm = got["gm"].double()
    xh = (t0.double() - m0.double()) * i0.double()
    P = n * h * w
    dt_ref = gam0.double() * i0.double() * (gm - gm.sum((0, 1, 2)) / P -
                                            xh * (gm * xh).sum((0, 1, 2)) / P)
    rel = ((got["dt0"].double() - dt_ref).norm() / dt_ref.norm()).item()
    assert rel <= (1e-5 if dt == torch.float32 else 1e-2), rel


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("C", [64, 256])
def test_bn_backward_recomputed_mask(dev, dt, pool, C):
    """mask kind 4 / 5: the BN-shortcut tail's ReLU mask recomputed from t0,
    t1 and the forward affines equals the mask read from the block output the
    forward kernels (rr_affine_act / rr_affine_act_pool) wrote -- every output
    bit for bit"""
    from roadrestore import ops
    n, h, w = 2, 8, 12
    t0 = rnd(n, h, w, C, seed=21).to(dev, dt)
    t1 = rnd(n, h, w, C, seed=22).to(dev, dt)
    s0, b0 = rnd(C, seed=23).to(dev), rnd(C, seed=24).to(dev)
    s1, b1 = rnd(C, seed=25).to(dev), rnd(C, seed=26).to(dev)
    if pool:
        out, pooled, idx = ops.affine_act_pool(t0, s0, b0, res=t1, res_scale=s1, res_shift=b1, relu=True)
        pl = (rnd(n, h // 2, w // 2, C, seed=27).to(dev, dt), idx)
    else:
        out = ops.affine_act(t0, s0, b0, res=t1, res_scale=s1, res_shift=b1, relu=True)
        pl = None
    assert 0.2 < (out.float() > 0).float().mean().item() < 0.8
    g = rnd(n, h, w, C, seed=28).to(dev, dt)
    m0, i0 = rnd(C, seed=29).to(dev), (rnd(C, seed=30).abs() + 0.5).to(dev)
    m1, i1 = rnd(C, seed=31).to(dev), (rnd(C, seed=32).abs() + 0.5).to(dev)
    gam0, gam1 = rnd(C, seed=33).to(dev), rnd(C, seed=34).to(dev)
    kw = dict(mask_kind=1, aux=out, t1=t1, mean1=m1, inv1=i1, gamma1=gam1, pool=pl)
    ref = ops.bn_backward(g, t0, m0, i0, gam0, **kw)
    got = ops.bn_backward(g, t0, m0, i0, gam0,
                          recompute=(torch.stack((s0, s1)), torch.stack((b0, b1))), **kw)
    for k in ("dt0", "dt1", "dgamma0", "dbeta0", "dgamma1", "dbeta1"):
        assert torch.equal(got[k], ref[k]), k


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("count", [4096, 4093])
@pytest.mark.parametrize("kind", [0, 1])
def test_loss_vector_and_scalar_paths(dev, dt, count, kind):
    """rr_loss_fwd / rr_loss_bwd: the 8-element vector kernels (count % 8 ==
    0) and the scalar ones agree with the torch formula (L1: mean |a-b|, MSE:
    mean (a-b)^2; grads incl. accumulate and the mask on a > 0)"""
    from roadrestore import ops
    a = rnd(count, seed=40).to(dev, dt)
    b = rnd(count, seed=41).to(dev, dt)
    af, bf = a.double().cpu(), b.double().cpu()
    ref = (af - bf).abs().mean() if kind == 0 else ((af - bf) ** 2).mean()
    got = ops.loss_fwd(kind, a, b).item()
    assert abs(got - ref.item()) <= 1e-5 * max(1.0, abs(ref.item()))
    d = af - bf
    gref = (torch.sign(d) if kind == 0 else 2 * d) / count
    gref = torch.where(af > 0, gref, torch.zeros_like(gref))
    base = rnd(count, seed=42).to(dev, dt)
    ga = ops.loss_bwd(kind, a, b, ga=base.clone(), accumulate=True, mask_a_pos=True)
    tol = 1e-6 if dt == torch.float32 else 1e-2
    err = (ga.double().cpu() - (base.double().cpu() + gref)).abs().max().item()
    assert err <= tol * max(1.0, base.abs().max().item()), err


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("src,dst", [((7, 7), (15, 15)), ((4, 6), (9, 13)), ((8, 8), (16, 16)),
                                     ((9, 13), (9, 13)), ((16, 16), (7, 11)), ((5, 3), (17, 10))])
def test_nearest_resize_fwd_bwd(dev, dt, src, dst):
    """F.interpolate(size=..., mode='nearest') as the ResUNet skip alignment
    calls it (14:169-182): forward equal to torch's CPU result bit for bit
    (a pure gather), backward equal to autograd's scatter-add (exact in fp32:
    at most 3 addends per source pixel for these ratios; bf16 within one
    rounding)."""
    import roadrestore as rr
    n, C = 3, 64
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, C, *src, generator=g)
    if dt == torch.bfloat16:
        x = x.bfloat16().float()
    xr = x.clone().requires_grad_(True)
    y = F.interpolate(xr, size=dst)
    dy = torch.randn(y.shape, generator=g)
    if dt == torch.bfloat16:
        dy = dy.bfloat16().float()
    y.backward(dy)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    yo = rr.ops.nearest_resize(xn, *dst)
    assert torch.equal(yo.float().permute(0, 3, 1, 2).cpu(), y.detach())
    dx = rr.ops.nearest_resize_bwd(dy.permute(0, 2, 3, 1).contiguous().to(dev, dt), *src)
    dxc = dx.float().permute(0, 3, 1, 2).cpu()
    if dt == torch.float32:
        assert (dxc - xr.grad).abs().max().item() <= 1e-6 * max(1.0, xr.grad.abs().max().item())
    else:
        assert (dxc - xr.grad).abs().max().item() <= 1e-2 * max(1.0, xr.grad.abs().max().item())
