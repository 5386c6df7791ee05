"""BN1 + PReLU folded into conv2 of a ResidualBlock (14:99-105; round 6,
VERDICT r5 item 3): rr_igemm_pre / rr_wgrad_pre take conv1's pre-BN output
t1 and turn every input row into a1 = PReLU(t1 * s + b) in LDS as it lands
in the row-streaming kernels' rings, so the a1 tensor is never written.

Bitwise checks: the folded forward (output + BN-statistics partials) and
weight grad equal the separate rr_affine_act pass followed by the plain
kernels on the stored a1 -- the same fp32 expression, the same bf16 rounding,
the same MFMA sums -- and a whole ResUNet training step (64x64, the maps
where the fold applies: res1 / dec1) gives bitwise the same output, loss,
gradients and running statistics with the fold on and off."""
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


# (n, h, w): whole-row streaming maps; uneven workgroup ranges start mid-image
SHAPES = [(16, 64, 64), (17, 64, 64), (64, 32, 32), (81, 32, 32)]


@pytest.mark.parametrize("shape", SHAPES)
def test_igemm_pre_and_wgrad_pre_bitwise(dev, shape):
    from roadrestore import ops
    from roadrestore._lib import RR_CONV3X3
    n, h, w = shape
    C = 64
    t1 = nhwc(rnd(n, C, h, w, seed=1) * 1.5 + 0.2, dev)
    wt = (rnd(C, C, 3, 3, seed=2) / 24.0).to(dev)
    wf, _ = ops.pack_conv(wt, BF)
    b2 = (rnd(C, seed=3) * 0.1).to(dev)
    s1 = (torch.rand(C, generator=torch.Generator().manual_seed(4)) + 0.5).to(dev)
    sh1 = (rnd(C, seed=5) * 0.3).to(dev)
    alpha = torch.tensor([0.23], device=dev)
    dy = nhwc(rnd(n, C, h, w, seed=6), dev)
    assert ops.igemm_pre_ok(BF, n, h, w, C, C) and ops.wgrad_pre_ok(BF, n, h, w, C, C)
    # the separate pass + plain kernels
    a1 = ops.affine_act(t1, s1, sh1, alpha=alpha)
    y0, _, st0 = ops.igemm(RR_CONV3X3, a1, None, n, h, w, wf, C, bias=b2, stats=True)
    dw0 = ops.wgrad(RR_CONV3X3, dy, a1, None, n, h, w, C, dw_shape=(C, C, 3, 3))
    # folded
    y1, _, st1 = ops.igemm_pre(t1, n, h, w, wf, C, b2, s1, sh1, alpha)
    dw1 = ops.wgrad_pre(dy, t1, n, h, w, C, s1, sh1, alpha,
                        dw=torch.empty((C, C, 3, 3), dtype=torch.float32, device=dev))
    torch.cuda.synchronize()
    assert ops.igemm_kernel_name(ops.IgemmDesc(ops.RR_BF16, RR_CONV3X3, n, h, w, C, 0, C, 0, 0, 0, 1, 0, 1,
                                               0)).startswith("stream3_kernel")
    assert torch.equal(y1, y0)
    assert torch.equal(st1, st0)
    assert torch.equal(dw1, dw0)
    # and against fp32 torch on the stored a1 (the fold changes nothing numerically)
    a1f = a1.float().permute(0, 3, 1, 2).cpu()
    ref = F.conv2d(a1f, wt.cpu(), b2.cpu(), padding=1)
    got = y1.float().permute(0, 3, 1, 2).cpu()
    assert ((got - ref).norm() / ref.norm()).item() < 4e-3


def test_unsupported_descriptors_refused(dev):
    from roadrestore import ops
    # strips, 16x16 (tap-reuse conv), concat second source: the separate pass
    assert not ops.igemm_pre_ok(BF, 2, 224, 224, 64, 64)
    assert not ops.igemm_pre_ok(BF, 64, 16, 16, 64, 64)
    assert not ops.igemm_pre_ok(torch.float32, 16, 64, 64, 64, 64)
    assert not ops.wgrad_pre_ok(BF, 64, 16, 16, 64, 64)


def test_resunet_step_bitwise_with_and_without_fold(dev, monkeypatch):
    """one ResUNet training forward + backward at 64x64 (res1 / dec1 take the
    fold, the others the separate pass): output, loss, every gradient and the
    running statistics bitwise equal with the fold on and off"""
    import roadrestore as rr
    from roadrestore import engine, ops
    from oracle import seeded as S
    sd = S.model_state_dict("resunet")
    B = 16
    g = torch.Generator().manual_seed(9)
    bad = torch.rand(B, 3, 64, 64, generator=g)
    clean = torch.rand(B, 3, 64, 64, generator=g)
    res = {}
    for fold in (True, False):
        monkeypatch.setattr(engine, "_FOLD_BN1", fold)
        m = rr.ResUNet().to(dev)
        m.load_state_dict(sd)
        m.compute_dtype = BF
        m.train()
        log = []
        ops.LAUNCH_LOG = log
        try:
            out = m(bad.to(dev))
            loss = F.l1_loss(out.float(), clean.to(dev))
            loss.backward()
            torch.cuda.synchronize()
        finally:
            ops.LAUNCH_LOG = None
        n_pre = sum(1 for _, t in log if t.endswith(" pre"))
        res[fold] = (out.detach().cpu(), loss.item(),
                     {k: p.grad.detach().cpu() for k, p in m.named_parameters()},
                     {k: b.detach().cpu() for k, b in m.named_buffers()}, n_pre)
        del m, out, loss
    on, off = res[True], res[False]
    assert on[4] == 4 and off[4] == 0, (on[4], off[4])      # res1 / dec1: conv2 fwd + wgrad each
    assert torch.equal(on[0], off[0])
    assert on[1] == off[1]
    for k in on[2]:
        assert torch.equal(on[2][k], off[2][k]), k
    for k in on[3]:
        assert torch.equal(on[3][k], off[3][k]), k
