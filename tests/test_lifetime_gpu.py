"""Boundary hygiene on the GPU:

* the forward state a network / loss op saves for its backward is freed with
  the autograd graph (50 grad-enabled forwards without a backward leave
  device memory flat), and the no-grad validation loss (14:253-263) saves
  nothing;
* the eval-mode conv+BN fold follows the running statistics after train-mode
  forwards that took no optimizer step (BN recalibration);
* ``torch.library.opcheck`` (schema, autograd registration, fake kernels) on
  every ``rr::`` op, with real inputs."""
import gc

import pytest
import torch

pytestmark = pytest.mark.gpu


def _mem(dev):
    gc.collect()
    torch.cuda.synchronize(dev)
    return torch.cuda.memory_allocated(dev)


def test_forward_without_backward_frees_state(dev):
    import roadrestore as rr
    from roadrestore import torch_ops as T
    torch.manual_seed(0)
    m = rr.ResUNet().to(dev)
    m.train()
    perc = rr.VGGPerceptualLoss().to(dev)
    x = torch.rand(8, 3, 32, 32, device=dev)
    n0 = T.saved_state_count()
    for _ in range(3):                           # warm the caches / allocator (the batched
        out = m(x)                               # weight re-pack is built on the 2nd forward)
        loss = rr.unified_loss(out, x, perc, 0.1)
        del out, loss
    base = _mem(dev)
    for _ in range(50):
        out = m(x)                               # grads enabled, output dropped
        loss = rr.unified_loss(out, x, perc, 0.1)
        del out, loss
    assert T.saved_state_count() == n0
    grown = _mem(dev) - base
    assert grown <= 4 << 20, grown               # flat (one step's state is ~100 MB here)
    with torch.no_grad():                        # the validation loss (14:253-263)
        for _ in range(10):
            rr.unified_loss(m(x), x, perc, 0.1)
    assert T.saved_state_count() == n0
    # an exception between forward and backward: the graph dies with the frame
    try:
        out = m(x)
        raise ValueError("boom")
    except ValueError:
        pass
    del out
    gc.collect()
    assert T.saved_state_count() == n0
    # the normal path still works and consumes its state
    out = m(x)
    rr.unified_loss(out, x, perc, 0.1).backward()
    assert T.saved_state_count() == n0


def test_eval_fold_follows_running_stats_without_optimizer_step(dev):
    """eval forward -> train-mode forwards with no optimizer step (the
    running statistics move) -> eval forward: the folded conv+BN weights
    must be re-made from the new statistics (keyed on tensor
    versions the finalize never bumped)."""
    import roadrestore as rr
    from oracle import reference_cpu as R
    from oracle import seeded as S
    sd = S.model_state_dict("resunet")
    m = rr.ResUNet().to(dev)
    m.load_state_dict(sd)
    x = S.fog_noise(S.image_batch(2, 32, 32, seed=3), seed=4)
    m.eval()
    with torch.no_grad():
        out0 = m(x.to(dev)).cpu()
    m.train()
    with torch.no_grad():
        for _ in range(3):
            m(x.to(dev) * 0.5)                   # BN recalibration, no step
    m.eval()
    with torch.no_grad():
        out1 = m(x.to(dev)).cpu()
    cur = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref = R.resunet_forward(cur, x, training=False)
    assert (out1 - ref).abs().mean().item() <= 1e-4
    assert (out0 - out1).abs().max().item() > 1e-3      # the statistics really moved


def _opcheck(op, args, utils=("test_schema", "test_autograd_registration", "test_faketensor")):
    torch.library.opcheck(op, args, test_utils=utils)


def test_opcheck_every_rr_op(dev):
    """torch.library.opcheck on every rr:: op with real device inputs."""
    import roadrestore as rr
    from roadrestore import ops
    torch.manual_seed(0)
    x = torch.rand(2, 3, 16, 16, device=dev)
    y = torch.rand(2, 3, 16, 16, device=dev)
    m = rr.ResUNet().to(dev).train()
    su = rr.SimpleUNet().to(dev).train()
    blk = rr.ResidualBlock(64, 128).to(dev).train()
    perc = rr.VGGPerceptualLoss().to(dev)
    vgg = rr.vgg16().to(dev).eval()
    o = torch.ops.rr
    # networks: forward (need_backward False: opcheck runs the op repeatedly)
    _opcheck(o.resunet_forward.default, (x, list(m.parameters()), m._op_key, False))
    _opcheck(o.simple_unet_forward.default, (x, list(su.parameters()), su._op_key, False))
    xb = torch.rand(2, 64, 8, 8, device=dev)
    _opcheck(o.resblock_forward.default, (xb, list(blk.parameters()), blk._op_key, False))
    # their backward ops consume a live forward handle: a fresh forward per
    # check (each opcheck utility runs the op for real)
    for util in ("test_schema", "test_faketensor"):
        for net, xin in ((m, x), (su, x), (blk, xb)):
            pre = net._op
            fwd = getattr(o, f"{pre}_forward").default
            bwd = getattr(o, f"{pre}_backward").default
            out, h = fwd(xin, list(net.parameters()), net._op_key, True)
            _opcheck(bwd, (torch.ones_like(out), h, net._op_key), utils=(util,))
        loss, h = o.unified_loss(x, y, perc._op_key, 0.1, 1.0, True)
        _opcheck(o.unified_loss_backward.default, (torch.ones((), device=dev), x, y, h, 0.1, 1.0),
                 utils=(util,))
        loss, h = o.perceptual_loss(x, y, perc._op_key, True)
        _opcheck(o.perceptual_loss_backward.default, (torch.ones((), device=dev), h, x),
                 utils=(util,))
    # losses
    _opcheck(o.pixel_loss.default, (x, y, ops.L1))
    _opcheck(o.pixel_loss_backward.default, (torch.ones((), device=dev), x, y, ops.MSE))
    _opcheck(o.unified_loss.default, (x, y, perc._op_key, 0.1, 1.0, False))
    _opcheck(o.perceptual_loss.default, (x, y, perc._op_key, False))
    # leaf layers called on their own (roadrestore.layers)
    from roadrestore import layers as L
    f32 = L.dtype_code(torch.float32)
    xc = torch.rand(2, 64, 8, 8, device=dev)
    w3 = torch.randn(64, 64, 3, 3, device=dev) * 0.05      # (64-multiple channels: layers.py)
    b3 = torch.randn(64, device=dev)
    _opcheck(o.conv2d.default, (xc, w3, b3, 1, f32))
    _opcheck(o.conv2d_backward.default, (torch.rand(2, 64, 8, 8, device=dev), xc, w3, 1, f32))
    wt = torch.randn(64, 64, 2, 2, device=dev) * 0.05
    bt = torch.randn(64, device=dev)
    _opcheck(o.conv_transpose2d.default, (xc, wt, bt, f32))
    _opcheck(o.conv_transpose2d_backward.default,
             (torch.rand(2, 64, 16, 16, device=dev), xc, wt, f32))
    bn = rr.BatchNorm2d(64).to(dev)
    for training in (True, False):
        _opcheck(o.batch_norm.default, (xc, bn.weight, bn.bias, bn._op_key, training, f32))
        yb, mean, inv = o.batch_norm(xc, bn.weight, bn.bias, bn._op_key, training, f32)
        _opcheck(o.batch_norm_backward.default,
                 (torch.rand_like(xc), xc, mean, inv, bn.weight, training, f32))
    alpha = torch.full((1,), 0.25, device=dev)
    _opcheck(o.prelu.default, (xc - 0.5, alpha, f32))
    _opcheck(o.prelu_backward.default, (torch.rand_like(xc), xc - 0.5, alpha, f32))
    _opcheck(o.relu.default, (xc - 0.5, f32))
    _opcheck(o.relu_backward.default, (torch.rand_like(xc), xc - 0.5, f32))
    _opcheck(o.max_pool2d.default, (xc, f32))
    _, idx = o.max_pool2d(xc, f32)
    _opcheck(o.max_pool2d_backward.default, (torch.rand(2, 64, 4, 4, device=dev), idx, 8, 8, f32))
    with torch.no_grad():
        _opcheck(o.adaptive_avg_pool2d.default, (torch.rand(2, 512, 2, 2, device=dev), 7, 7, f32))
        _opcheck(o.linear.default, (torch.rand(3, 64, device=dev), torch.randn(10, 64, device=dev),
                                    torch.randn(10, device=dev), f32))
    # judge and post-processing
    with torch.no_grad():
        _opcheck(o.vgg16_logits.default, (torch.rand(2, 3, 32, 32, device=dev),
                                          list(vgg.parameters()), vgg._op_key))
    _opcheck(o.nearest_resize.default, (torch.rand(2, 5, 7, 64, device=dev), 9, 13))
    _opcheck(o.to_uint8_hwc.default, (x, True))
    u8 = o.to_uint8_hwc(x, False)
    _opcheck(o.psnr_u8.default, (u8, o.to_uint8_hwc(y, False)))
    _opcheck(o.argmax_rows.default, (torch.rand(7, 43, device=dev),))


@pytest.mark.parametrize("nbytes", [16 * 1024, 4 * 1024 + 6, 3 << 20])
def test_library_zero_in_hip_graph_replays(dev, nbytes):
    """ops.zero_ (rr_zero, a library kernel) recorded in a HIP
    graph, alone and between torch / library nodes, zeroes its buffer on
    every replay (4 replays, the buffer refilled with garbage between them),
    and so does RunningLoss.reset() captured with an add."""
    import roadrestore as rr
    from roadrestore import ops
    n = nbytes
    for mode in ("alone", "between"):
        buf = torch.empty(n, dtype=torch.uint8, device=dev)
        other = torch.ones(1024, device=dev)
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(dev)
        with torch.cuda.graph(g):
            if mode == "between":
                other.mul_(2.0)
            ops.zero_(buf)
            if mode == "between":
                ops.zero_(other[:7])
                other.add_(1.0)
        for r in range(4):
            buf.fill_(0xA5)
            other.fill_(3.0)
            g.replay()
            torch.cuda.synchronize(dev)
            assert int(buf.count_nonzero()) == 0, (mode, r)
            if mode == "between":
                assert torch.all(other[:7] == 1.0) and torch.all(other[7:] == 7.0), (mode, r)
    run = rr.RunningLoss(dev)
    loss = torch.full((1,), 0.5, device=dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(g):
        run.reset()
        run.add(loss)
        run.add(loss)
    for r in range(4):
        run.acc.fill_(123.0)
        run.count.fill_(9)
        g.replay()
        assert run.steps() == 2 and run.total() == 1.0, r
