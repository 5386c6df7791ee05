"""Leaf modules called on their own (roadrestore.layers): op registration,
fake shapes, shape gating and the no-CPU-fallback rule -- no GPU needed."""
import pytest
import torch

import roadrestore as rr
from roadrestore import layers


def test_layer_ops_registered_with_fake_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    assert all(hasattr(torch.ops.rr, n) for n in layers.OPS)
    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty(2, 64, 12, 20, device="cuda")
        w = torch.empty(128, 64, 3, 3, device="cuda")
        assert torch.ops.rr.conv2d(x, w, None, 1, 0).shape == (2, 128, 12, 20)
        wt = torch.empty(64, 128, 2, 2, device="cuda")
        assert torch.ops.rr.conv_transpose2d(x, wt, torch.empty(128, device="cuda"), 1).shape \
            == (2, 128, 24, 40)
        y, idx = torch.ops.rr.max_pool2d(torch.empty(2, 64, 13, 9, device="cuda"), 0)
        assert y.shape == (2, 64, 6, 4) and idx.shape == (2, 6, 4, 64) and idx.dtype == torch.uint8
        assert torch.ops.rr.adaptive_avg_pool2d(x, 7, 7, 0).shape == (2, 64, 7, 7)
        assert torch.ops.rr.linear(torch.empty(3, 128, device="cuda"), torch.empty(43, 128),
                                   torch.empty(43), 0).shape == (3, 43)


@pytest.mark.parametrize("cin,cout,k,pad,kind", [
    (3, 64, 3, 1, "in"), (64, 64, 3, 1, "igemm"), (384, 128, 3, 1, "igemm"),
    (64, 128, 1, 0, "igemm"), (64, 3, 1, 0, "out")])
def test_conv_kind(cin, cout, k, pad, kind):
    assert layers.conv_kind(cin, cout, k, pad) == kind


@pytest.mark.parametrize("cin,cout,k,pad", [(3, 64, 3, 0), (48, 64, 3, 1), (64, 40, 3, 1),
                                            (5, 3, 1, 0), (3, 64, 5, 2)])
def test_conv_kind_rejects_unserved_shapes(cin, cout, k, pad):
    with pytest.raises(NotImplementedError):
        layers.conv_kind(cin, cout, k, pad)


def test_leaf_modules_reject_cpu_input():
    """No CPU fallback: a leaf called on host tensors raises."""
    m = rr.ResUNet()
    x = torch.randn(1, 3, 8, 8)
    for f in (m.enc1, m.enc1[0], m.res1.conv_block[1], m.pool1, m.up1):
        with pytest.raises(RuntimeError, match="GPU only"):
            f(x if f is not m.up1 else torch.randn(1, 64, 4, 4))


def test_dropout_eval_identity_train_rejected():
    d = rr.nn.Dropout()
    x = torch.randn(4, 8)
    d.eval()
    assert d(x) is x
    d.train()
    with pytest.raises(NotImplementedError):
        d(x)
