"""Row-streaming bf16 3x3 weight gradient (csrc/swgrad.hip) for 64- and
128-channel output gradients (64-channel dy slices): eligibility mirror, parity against fp32 torch on
bf16-exact inputs (products exact in fp32, only the summation order
differs), concat second sources, accumulate, and agreement with the tiled
LDS-halo kernel (RR_PATH swgrad=0).  Shapes cover partial images per workgroup,
several images per workgroup and ragged step ranges."""
import pytest
import torch
import torch.nn.functional as F
from rrpath import set_path  # noqa: E402

pytestmark = pytest.mark.gpu

# (n, h, w, c1, c2, cout)
SHAPES = [(8, 64, 64, 64, 0, 64), (9, 64, 64, 64, 0, 64), (11, 64, 64, 64, 128, 64),
          (32, 32, 32, 64, 0, 64), (37, 32, 32, 64, 64, 64), (33, 32, 32, 128, 0, 64),
          (40, 32, 32, 64, 128, 64), (34, 32, 32, 64, 0, 128), (35, 32, 32, 128, 0, 128),
          (9, 64, 64, 64, 0, 128), (36, 32, 32, 64, 128, 128)]


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


def nhwc(x, dev):
    return x.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)


def run(dev, n, h, w, c1, c2, cout, seed, dw=None, accumulate=False):
    import roadrestore as rr
    from roadrestore._lib import RR_CONV3X3
    x = rnd(n, c1 + c2, h, w, seed=seed).bfloat16().float()
    g = rnd(n, cout, h, w, seed=seed + 1).bfloat16().float()
    x2 = nhwc(x[:, c1:], dev) if c2 else None
    out = rr.ops.wgrad(RR_CONV3X3, nhwc(g, dev), nhwc(x[:, :c1], dev), x2, n, h, w, cout,
                       dw=dw, accumulate=accumulate, dw_shape=(cout, c1 + c2, 3, 3))
    return x, g, out


@pytest.mark.parametrize("shape", SHAPES)
def test_swgrad_selected(shape):
    from roadrestore import ops
    from roadrestore._lib import RR_BF16, RR_CONV3X3, WgradDesc
    n, h, w, c1, c2, cout = shape
    d = WgradDesc(RR_BF16, RR_CONV3X3, n, h, w, c1, c2, cout, 0)
    assert ops.wgrad_kernel_name(d) == f"swgrad_kernel<{w}>"     # the library's own choice


@pytest.mark.parametrize("shape", SHAPES)
def test_swgrad_vs_torch(dev, shape):
    n, h, w, c1, c2, cout = shape
    x, g, dw = run(dev, n, h, w, c1, c2, cout, seed=70)
    wt = torch.zeros(cout, c1 + c2, 3, 3, requires_grad=True)
    F.conv2d(x, wt, None, padding=1).backward(g)
    rel = ((dw.cpu() - wt.grad).norm() / wt.grad.norm()).item()
    assert rel < 2e-5, rel


@pytest.mark.parametrize("shape", [SHAPES[1], SHAPES[4], SHAPES[8]])
def test_swgrad_accumulate_and_tiled(dev, shape, monkeypatch):
    n, h, w, c1, c2, cout = shape
    base = rnd(cout, c1 + c2, 3, 3, seed=9).to(dev)
    _, _, acc = run(dev, n, h, w, c1, c2, cout, seed=80, dw=base.clone(), accumulate=True)
    _, _, one = run(dev, n, h, w, c1, c2, cout, seed=80)
    torch.testing.assert_close(acc, base + one, rtol=0, atol=1e-4)
    set_path(monkeypatch, "swgrad", "0")
    _, _, tiled = run(dev, n, h, w, c1, c2, cout, seed=80)
    rel = ((one - tiled).norm() / tiled.norm()).item()
    assert rel < 2e-5, rel


def test_swgrad_deterministic(dev):
    _, _, a = run(dev, *SHAPES[10], seed=90)
    _, _, b = run(dev, *SHAPES[10], seed=90)
    assert torch.equal(a, b)
