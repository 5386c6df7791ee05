"""Network executors: forward schedules and hand-written backward schedules.

Each reference network is run as one autograd node whose forward issues the
fused HIP kernels in order (NHWC activations kept resident in HBM, saved for
backward) and whose backward issues the reverse schedule: BN/PReLU/ReLU
backward reductions, dgrad implicit GEMMs and split-K wgrad GEMMs.  Parameter
gradients are written straight into one flat fp32 buffer laid out in the
order they become final (``GradSink``), so a data-parallel wrapper can
all-reduce finished buckets while the rest of the backward still runs, and a
fused optimizer can update every parameter with one launch.

Reference schedules mirrored (file:line in the reference repo):
  SimpleUNet.forward        07_train_restoration.py:99-120
  ResidualBlock.forward     14_train_unified_advanced.py:114-115
  ResUNet.forward           14_train_unified_advanced.py:151-186
  VGGPerceptualLoss.forward 14_train_unified_advanced.py:195-196
  VGG16 classifier          18_test_unified_benchmark.py:46 (torchvision cfg D)
"""
from __future__ import annotations


import torch

from . import ops
from ._lib import RR_CONV1X1, RR_CONV3X3, RR_CONVT_DOWN, RR_CONVT_UP, path_flag

RELU = 1


class Bag(dict):
    __getattr__ = dict.__getitem__

    def __setattr__(self, k, v):
        self[k] = v


# ---------------------------------------------------------------------------
# packed weights

class WeightCache:
    """Packed (compute layout / dtype) copies of fp32 weights, re-packed when
    the parameter's version counter moves (every optimizer step) and always
    while a HIP graph is being captured (so replays re-pack).

    Conv packs are batched: the convs a forward requests are recorded (the
    plan), and ``begin()`` at the start of every later forward re-packs all
    of them in ONE launch (ops.PackBatch) when any is stale or a graph is
    being captured; the per-layer ``conv()`` calls then hit those packs.

    ``static=True`` (the frozen perceptual VGG, 14:192-193): a capture uses the
    packs made by the eager forwards before it instead of re-packing in every
    replay -- weights changed after the capture need a new capture."""

    def __init__(self, static=False):
        self.static = static
        self._c = {}
        self._plan = {}          # id(w) -> [w, dtype, dgrad], first-request order
        self._batch = None
        self._fresh = {}         # key -> (ver, packed), set by begin()
        self._pending = None     # (event, fresh) of a prefetch() not yet joined
        self._misc = {}          # key -> (w, fn, also): the convT / first-conv / bias packs

    def _ver(self, w, also=None):
        # the fused optimizer's generation counts only for trained weights: a
        # static cache (the frozen VGG) keyed on it re-packed in every
        # captured step (2 x 12 us per replay, r5i trace)
        from .optim import GENERATION
        return (w.data_ptr(), w._version, 0 if self.static else GENERATION[0],
                None if also is None else (also.data_ptr(), also._version))

    def _get(self, w, dtype, kind, fn, also=None, record=True):
        cap = torch.cuda.is_current_stream_capturing()
        key = (id(w), dtype, kind)
        ver = self._ver(w, also)
        # the non-conv packs (re-)recorded by every use for the next
        # prefetch(); conv packs are the plan's (the batched re-pack), so a
        # conv reaching here (the first forward, before the plan exists) is
        # not recorded again as a per-layer pack
        if record and not self.static and w.is_cuda:
            self._misc[key] = (w, fn, also)
        f = self._fresh.get(key)
        if f is not None and f[0] == ver:
            return f[1]                  # made by a prefetch() of this forward
        e = None if cap and not self.static else self._c.get(key)
        if e is not None and e[0] == ver:
            return e[1]
        v = fn()
        if not cap:
            self._c[key] = (ver, v)
        return v

    def conv_bn_folded(self, conv, bn, dtype):
        """Eval: the BN after ``conv`` folded into it -- (packed fwd weights of
        w * s, fp32 bias b * s + t), s / t the BN eval affine (17:84-85).
        Cached on the versions of the conv and BN tensors."""
        deps = [t for t in (conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean,
                            bn.running_var) if t is not None]
        from .optim import GENERATION
        ver = tuple((t.data_ptr(), t._version) for t in deps) + (GENERATION[0], bn.eps)
        key = (id(conv.weight), dtype, "fold")
        cap = torch.cuda.is_current_stream_capturing()
        e = None if cap else self._c.get(key)
        if e is not None and e[0] == ver:
            return e[1]
        s, t = ops.bn_eval_affine(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps)
        wf, bf = ops.fold_conv_bn(conv.weight, conv.bias, s, t)
        pk, _ = ops.pack_conv(wf, dtype, fwd=True, dgrad=False)
        v = (pk, bf)
        if not cap:
            self._c[key] = (ver, v)
        return v

    def prefetch(self):
        """Fork the next forward's batched re-pack onto a side stream now --
        at the start of a training step, before the input pipeline (the
        distortion + ToTensor, 14:31-64 / 14:199-202) is enqueued: the packs
        depend on the weights only, so they overlap that work instead of
        sitting in front of the first conv.  The next begin() joins them.
        Only once the plan is known (after a first forward); False if nothing
        was forked.  The pack outputs are persistent buffers (PackBatch), so
        no allocation crosses streams."""
        if self._pending is not None or not self._plan:
            return False
        w0 = next(iter(self._plan.values()))[0]
        if not w0.is_cuda:
            return False
        side = _pack_stream(w0.device)
        side.wait_stream(torch.cuda.current_stream(w0.device))
        main = torch.cuda.current_stream(w0.device)
        # the packs are built into local dicts and published to _fresh / _c
        # only by the next begin(), after its wait on the side stream: until
        # then nothing on the main stream can see buffers still being written
        with torch.cuda.stream(side):
            fresh, cache = self._repack()
            # the small non-conv packs too (3 convT + 3 bias tiles + the
            # first conv: ~5 us launches each in front of their layers)
            misc, self._misc = self._misc, {}     # the packs the last forward asked for
            for key, (w, fn, also) in misc.items():
                v = fn()
                for t in (v if isinstance(v, (tuple, list)) else (v,)):
                    if isinstance(t, torch.Tensor):
                        t.record_stream(main)
                fresh[key] = (self._ver(w, also), v)
            ev = torch.cuda.Event()
            ev.record(side)
        self._pending = (ev, fresh, cache)
        return True

    def begin(self):
        """Start of a forward: one batched re-pack of every planned conv (or
        the join of a prefetch() of it)."""
        if self._pending is not None:
            ev, fresh, cache = self._pending
            self._pending = None
            torch.cuda.current_stream().wait_event(ev)
        else:
            fresh, cache = self._repack()
        self._fresh = fresh
        self._c.update(cache)

    def _repack(self):
        """The batched re-pack of every planned conv when any is stale or a
        graph is being captured: (fresh, cache) entries for the caller to
        publish (nothing is published here)."""
        fresh, cache = {}, {}
        if not self._plan:
            return fresh, cache
        cap = torch.cuda.is_current_stream_capturing()
        ent = list(self._plan.values())
        keys = [(id(w), dt, "conv+d" if dg else "conv") for w, dt, dg in ent]
        vers = [self._ver(w) for w, _, _ in ent]
        if cap and self.static and all(self._c.get(k, (None,))[0] == v for k, v in zip(keys, vers)):
            return fresh, cache                      # conv() hits the pre-capture packs
        ok = self._batch is not None and self._batch.valid() and \
            self._batch.entries == [tuple(e) for e in ent]
        if not ok and not cap and all(w.is_contiguous() for w, _, _ in ent) and \
                len({dt for _, dt, _ in ent}) == 1:
            # built eagerly (its job table is a host -> device copy, which a
            # capture does not allow), also when nothing is stale yet
            self._batch = ops.PackBatch([tuple(e) for e in ent])
            ok = True
        if not cap and all(self._c.get(k, (None,))[0] == v for k, v in zip(keys, vers)):
            return fresh, cache
        if not ok:
            return fresh, cache                      # per-layer packs instead
        outs = self._batch.run()
        for k, v, o in zip(keys, vers, outs):
            fresh[k] = (v, o)
            if not cap:
                cache[k] = (v, o)
        return fresh, cache

    def conv(self, w, dtype, dgrad):
        kind = "conv+d" if dgrad else "conv"
        ver = self._ver(w)
        for k in ((id(w), dtype, kind),) + (() if dgrad else ((id(w), dtype, "conv+d"),)):
            f = self._fresh.get(k)
            if f is not None and f[0] == ver:
                return f[1]
        p = self._plan.get(id(w))
        if p is None:
            self._plan[id(w)] = [w, dtype, dgrad]
        elif p[1] != dtype:
            self._plan = {id(w): [w, dtype, dgrad]}   # compute dtype changed: new plan
            self._batch = None
        elif dgrad and not p[2]:
            p[2] = True
        return self._get(w, dtype, kind, lambda: ops.pack_conv(w, dtype, True, dgrad), record=False)

    def convT(self, w, dtype, down):
        kind = "convT+d" if down else "convT"
        return self._get(w, dtype, kind, lambda: ops.pack_convT(w, dtype, True, down))

    def linear(self, w, dtype):
        return self._get(w, dtype, "linear", lambda: ops.pack_conv(
            w.view(w.shape[0], w.shape[1], 1, 1), dtype, True, False))

    def conv_in(self, w, b, dtype):
        return self._get(w, dtype, "conv_in", lambda: ops.pack_conv_in(w, b, dtype), also=b)

    def bias4(self, b):
        return self._get(b, torch.float32, "b4", lambda: ops.bias_tile4(b))

    def clear(self):
        self._c.clear()

    def drop_folds(self):
        """Forget the eval-mode folded conv+BN weights.  Called on every switch
        to eval mode: train-mode forwards (also HIP-graph replays, where no
        host code runs to bump version counters) may have moved the running
        statistics since the fold was made."""
        for k in [k for k in self._c if k[2] == "fold"]:
            del self._c[k]


# ---------------------------------------------------------------------------
# gradient sink

class GradSink:
    """Flat fp32 gradient buffer over ``params`` (in readiness order).

    ``zero_params`` are parameters whose gradient is exactly zero (a conv bias
    feeding a train-mode BatchNorm: the BN subtracts the batch mean, so
    d(loss)/d(bias) = sum_p dt_p = 0); they sit first and are cleared with one
    memset.  ``hook(sink, params)`` is called as groups become final.
    """

    def __init__(self, params, device, zero_params=(), hook=None):
        zp = [p for p in params if id(p) in {id(z) for z in zero_params}]
        rest = [p for p in params if id(p) not in {id(z) for z in zero_params}]
        self.order = zp + rest
        total = sum(p.numel() for p in self.order)
        self.flat = torch.empty(total, dtype=torch.float32, device=device)
        self.view = {}
        self.offset = {}
        off = 0
        for p in self.order:
            self.view[id(p)] = self.flat[off:off + p.numel()].view(p.shape)
            self.offset[id(p)] = off
            off += p.numel()
        nz = sum(p.numel() for p in zp)
        if nz:
            # the library's zero (rr_zero), graph-capturable: round 3's
            # garbage-after-a-second-replay observation does not reproduce
            # (tools/diag_memset*.py, test_library_zero_in_hip_graph_replays;
            # the zeros are checked after replays in
            # test_hip_graph_step_follows_cosine_lr_schedule)
            ops.zero_(self.flat[:nz])
        self.zero_count = nz
        self.hook = hook

    def __getitem__(self, p):
        return self.view[id(p)]

    def ready(self, params):
        if self.hook is not None:
            self.hook(self, params)

    def release(self):
        """Hand the per-parameter views over (the autograd engine then adopts
        them as .grad without a copy) and drop our references."""
        out = {k: v for k, v in self.view.items()}
        self.view = {}
        return out


# A/B switch for the fused conv-dgrad + BN/PReLU backward reduce (default on)
FUSE_BNBWD = path_flag("fuse_bnbwd", 1) != 0

def _params(*mods):
    out = []
    for m in mods:
        out.extend(m.parameters())
    return out


# ---------------------------------------------------------------------------
# SimpleUNet (07:75-120)

def _conv3(wc, dt, conv, x1, x2, n, h, w, act, need_bwd, stats=False):
    pk = wc.conv(conv.weight, dt, dgrad=need_bwd)
    y, _, st = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, pk[0], conv.weight.shape[0],
                         bias=conv.bias, act=act, stats=stats)
    return y, pk, st


def _convT_up(wc, dt, conv, x, n, h, w, need_bwd):
    pk = wc.convT(conv.weight, dt, down=need_bwd)
    cout = conv.weight.shape[1]
    y, _, _ = ops.igemm(RR_CONVT_UP, x, None, n, h, w, pk[0], 4 * cout, bias=wc.bias4(conv.bias))
    return y, pk


def simple_unet_forward(m, x, wc, dt, need_bwd):
    wc.begin()
    n, _, H, W = x.shape
    S = Bag(n=n, H=H, W=W, x=x)
    e1a, _ = ops.first_conv_fwd(x, m.enc1[0].weight, m.enc1[0].bias, dt,
                                wc.conv_in(m.enc1[0].weight, m.enc1[0].bias, dt), act=RELU)
    e1, pk12, _ = _conv3(wc, dt, m.enc1[2], e1a, None, n, H, W, RELU, need_bwd)
    p1, i1 = ops.maxpool2_fwd(e1)
    H2, W2 = H // 2, W // 2
    e2a, pk20, _ = _conv3(wc, dt, m.enc2[0], p1, None, n, H2, W2, RELU, need_bwd)
    e2, pk22, _ = _conv3(wc, dt, m.enc2[2], e2a, None, n, H2, W2, RELU, need_bwd)
    p2, i2 = ops.maxpool2_fwd(e2)
    H4, W4 = H2 // 2, W2 // 2
    ba, pkb0, _ = _conv3(wc, dt, m.bottleneck[0], p2, None, n, H4, W4, RELU, need_bwd)
    b, pkb2, _ = _conv3(wc, dt, m.bottleneck[2], ba, None, n, H4, W4, RELU, need_bwd)
    u2, pku2 = _convT_up(wc, dt, m.up2, b, n, H4, W4, need_bwd)
    d2a, pkd20, _ = _conv3(wc, dt, m.dec2[0], u2, e2, n, H2, W2, RELU, need_bwd)   # cat(up, skip)
    d2, pkd22, _ = _conv3(wc, dt, m.dec2[2], d2a, None, n, H2, W2, RELU, need_bwd)
    u1, pku1 = _convT_up(wc, dt, m.up1, d2, n, H2, W2, need_bwd)
    d1a, pkd10, _ = _conv3(wc, dt, m.dec1[0], u1, e1, n, H, W, RELU, need_bwd)
    d1, pkd12, _ = _conv3(wc, dt, m.dec1[2], d1a, None, n, H, W, RELU, need_bwd)
    out = ops.conv_out_fwd(d1, m.final.weight, m.final.bias,
                           wpack=wc.conv(m.final.weight, dt, dgrad=False)[0])
    if need_bwd:
        S.update(e1a=e1a, e1=e1, p1=p1, i1=i1, e2a=e2a, e2=e2, p2=p2, i2=i2, ba=ba, b=b, u2=u2,
                 d2a=d2a, d2=d2, u1=u1, d1a=d1a, d1=d1, pk12=pk12, pk20=pk20, pk22=pk22,
                 pkb0=pkb0, pkb2=pkb2, pku2=pku2, pkd20=pkd20, pkd22=pkd22, pku1=pku1,
                 pkd10=pkd10, pkd12=pkd12)
    return out, S


def simple_unet_grad_order(m):
    return _params(m.final, m.dec1, m.up1, m.dec2, m.up2, m.bottleneck, m.enc2, m.enc1)


def _conv3_bwd(conv, pk, gpre, xin1, xin2, n, h, w, sink, mask=None, want_dx=True, split=0):
    """grads of a 3x3 conv given the pre-activation grad: dW, db, dx."""
    cout = conv.weight.shape[0]
    ops.wgrad(RR_CONV3X3, gpre, xin1, xin2, n, h, w, cout, dw=sink[conv.weight])
    ops.channel_sum(gpre, out=sink[conv.bias])
    if not want_dx:
        return None, None
    cin = conv.weight.shape[1]
    y1, y2, _ = ops.igemm(RR_CONV3X3, gpre, None, n, h, w, pk[1], cin, mask=mask, split=split)
    return y1, y2


def _convT_bwd(conv, pk, gu, xin, n, h, w, sink, mask=None, side=False):
    """ConvTranspose2d(k2,s2) backward: gu on the (2h, 2w) grid; xin [n,h,w,cin].
    ``side``: the weight grad's reduce and the bias sum on the reduce stream
    (joined by join_wgrad_reduces)."""
    cin, cout = conv.weight.shape[0], conv.weight.shape[1]
    rs = reduce_stream(gu.device) if side else None
    ops.wgrad(RR_CONVT_UP, gu, xin, None, n, h, w, cout, dw=sink[conv.weight], reduce_stream=rs)
    if rs is None:
        ops.channel_sum(gu, out=sink[conv.bias])
    else:
        rs.wait_stream(torch.cuda.current_stream(gu.device))
        with torch.cuda.stream(rs):
            ops.channel_sum(gu, out=sink[conv.bias])
        gu.record_stream(rs)
    gx, _, _ = ops.igemm(RR_CONVT_DOWN, gu, None, n, h, w, pk[1], cin, mask=mask)
    return gx


def simple_unet_backward(m, S, g_out, sink):
    n, H, W = S.n, S.H, S.W
    H2, W2, H4, W4 = H // 2, W // 2, H // 4, W // 4
    g_d1, _, _ = ops.conv_out_bwd(g_out, S.d1, m.final.weight, mask_relu=True,
                                  dw=sink[m.final.weight], db=sink[m.final.bias])
    sink.ready(_params(m.final))
    g_d1a, _ = _conv3_bwd(m.dec1[2], S.pkd12, g_d1, S.d1a, None, n, H, W, sink, mask=S.d1a)
    g_u1, g_e1 = _conv3_bwd(m.dec1[0], S.pkd10, g_d1a, S.u1, S.e1, n, H, W, sink,
                            split=m.dec1[0].weight.shape[1] // 2)
    sink.ready(_params(m.dec1))
    g_d2 = _convT_bwd(m.up1, S.pku1, g_u1, S.d2, n, H2, W2, sink, mask=S.d2)
    sink.ready(_params(m.up1))
    g_d2a, _ = _conv3_bwd(m.dec2[2], S.pkd22, g_d2, S.d2a, None, n, H2, W2, sink, mask=S.d2a)
    g_u2, g_e2 = _conv3_bwd(m.dec2[0], S.pkd20, g_d2a, S.u2, S.e2, n, H2, W2, sink,
                            split=m.dec2[0].weight.shape[1] // 2)
    sink.ready(_params(m.dec2))
    g_b = _convT_bwd(m.up2, S.pku2, g_u2, S.b, n, H4, W4, sink, mask=S.b)
    sink.ready(_params(m.up2))
    g_ba, _ = _conv3_bwd(m.bottleneck[2], S.pkb2, g_b, S.ba, None, n, H4, W4, sink, mask=S.ba)
    g_p2, _ = _conv3_bwd(m.bottleneck[0], S.pkb0, g_ba, S.p2, None, n, H4, W4, sink)
    sink.ready(_params(m.bottleneck))
    ops.maxpool2_bwd(g_p2, S.i2, H2, W2, out=g_e2, accumulate=True, mask=S.e2)
    g_e2a, _ = _conv3_bwd(m.enc2[2], S.pk22, g_e2, S.e2a, None, n, H2, W2, sink, mask=S.e2a)
    g_p1, _ = _conv3_bwd(m.enc2[0], S.pk20, g_e2a, S.p1, None, n, H2, W2, sink)
    sink.ready(_params(m.enc2))
    ops.maxpool2_bwd(g_p1, S.i1, H, W, out=g_e1, accumulate=True, mask=S.e1)
    g_e1a, _ = _conv3_bwd(m.enc1[2], S.pk12, g_e1, S.e1a, None, n, H, W, sink, mask=S.e1a)
    # im2col of the input only here (the fused forward never materialises it)
    ops.first_conv_wgrad(ops.im2col3(S.x, g_e1a.dtype), g_e1a, sink[m.enc1[0].weight],
                         sink[m.enc1[0].bias])
    sink.ready(_params(m.enc1))


# ---------------------------------------------------------------------------
# ResidualBlock (14:96-115) and ResUNet (14:117-186)

def _bn_affine(bn, st, bias, count, training, out=None, need_bwd=False):
    """-> (scale, shift, mean, invstd).  Eval mode: the running statistics;
    mean / invstd only when a backward follows (eval-mode BN backward)."""
    if training:
        return ops.bn_finalize(st, count, bias, bn.weight, bn.bias, bn.running_mean,
                               bn.running_var, _momentum(bn), bn.eps, bn.num_batches_tracked,
                               out=out)
    s, b = ops.bn_eval_affine(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, out=out)
    if not need_bwd:
        return s, b, None, None
    inv, _ = ops.bn_eval_affine(None, None, bn.running_mean, bn.running_var, bn.eps)
    return s, b, bn.running_mean, inv


# A/B switch: the tail BN and the shortcut BN finalized by one launch
_PAIR_FINALIZE = path_flag("bn_pair_finalize", 1) != 0


def _momentum(bn):
    """BatchNorm2d(momentum=None) (cumulative moving average): -1, the
    finalize then reads the factor 1 / num_batches_tracked on the device (no
    host sync; as layers.batch_norm).  Without running statistics
    (track_running_stats=False: no counter, nothing updated) the momentum is
    never used: 0."""
    if bn.momentum is None:
        return -1.0 if bn.num_batches_tracked is not None else 0.0
    return bn.momentum


def _fin_args(bn, st, bias, count, out):
    return dict(st=st, count=count, bias=bias, gamma=bn.weight, beta=bn.bias,
                running_mean=bn.running_mean, running_var=bn.running_var, momentum=_momentum(bn),
                eps=bn.eps, num_batches_tracked=bn.num_batches_tracked, out=out)


def block_has_shortcut(blk):
    return len(blk.shortcut) > 0


# A/B switch: the training-step BN1 + PReLU applied inside conv2's streaming
# forward and weight grad instead of a separate affine pass over t1 (RR_PATH
# bn1_fold=0: the pass, as before round 6)
_FOLD_BN1 = path_flag("bn1_fold", 1) != 0

# A/B switch: eval-mode BN folded into the conv weights (RR_PATH fold_bn=0:
# conv + separate BN affine passes, as in training)
_FOLD_BN = path_flag("fold_bn", 1) != 0


def resblock_forward_eval_folded(blk, x1, x2, n, h, w, wc, dt, pool=False):
    """Inference (17:84-86): every BN folded into the conv before it, so
      a1  = PReLU(conv1'(x))                    conv1' = BN1 o conv1
      out = relu(conv2'(a1) + sc'(x))           the shortcut 1x1 accumulates onto
                                                conv2's output with the ReLU in
                                                its epilogue (no tail pass)
      out = relu(conv2'(a1) + x)                identity shortcut: one pass"""
    cb = blk.conv_block
    c1, bn1, pr, c2, bn2 = cb[0], cb[1], cb[2], cb[3], cb[4]
    cout = c1.weight.shape[0]
    c_in1, c_in2 = x1.shape[-1], (x2.shape[-1] if x2 is not None else 0)
    pk1, b1 = wc.conv_bn_folded(c1, bn1, dt)
    one, zero = _unit_affine(cout, x1.device)
    if _ex_fusable(x1.dtype, n, h, w, c_in1, c_in2, cout, ops.RR_ACT_PRELU):
        # PReLU in conv1's epilogue (rr_igemm_ex): no separate activation pass
        a1, _, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, pk1, cout, bias=b1, alpha=pr.weight)
    else:
        t1, _, _ = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, pk1, cout, bias=b1)
        a1 = ops.affine_act(t1, one, zero, alpha=pr.weight)
    pk2, b2 = wc.conv_bn_folded(c2, bn2, dt)
    S = Bag(x1=x1, x2=x2, n=n, h=h, w=w)
    pl = ops.RR_ACT_POOL if pool else 0
    if not block_has_shortcut(blk) and x2 is None and \
            _ex_fusable(a1.dtype, n, h, w, cout, 0, cout, RELU | ops.RR_ACT_RES | pl):
        # identity shortcut: relu(conv2'(a1) + x) in conv2's epilogue (+ the
        # encoder's MaxPool2d: no index, nothing runs backward)
        out, pooled, _ = ops.igemm(RR_CONV3X3, a1, None, n, h, w, pk2, cout, bias=b2, res=x1,
                                   act=RELU, pool=pool)
        return (out, S, (pooled, None)) if pool else (out, S)
    if block_has_shortcut(blk) and pool and _ex_fusable(a1.dtype, n, h, w, cout, 0, cout, RELU | pl):
        # the shortcut first, then conv2 accumulates onto it with the ReLU and
        # the max-pool in its epilogue (relu(sc'(x) + conv2'(a1)))
        pks, bs = wc.conv_bn_folded(blk.shortcut[0], blk.shortcut[1], dt)
        out, _, _ = ops.igemm(RR_CONV1X1, x1, x2, n, h, w, pks, cout, bias=bs)
        _, pooled, _ = ops.igemm(RR_CONV3X3, a1, None, n, h, w, pk2, cout, bias=b2, out=out,
                                 accumulate=True, act=RELU, pool=True)
        return out, S, (pooled, None)
    t2, _, _ = ops.igemm(RR_CONV3X3, a1, None, n, h, w, pk2, cout, bias=b2)
    if block_has_shortcut(blk):
        pks, bs = wc.conv_bn_folded(blk.shortcut[0], blk.shortcut[1], dt)
        out, _, _ = ops.igemm(RR_CONV1X1, x1, x2, n, h, w, pks, cout, bias=bs, out=t2,
                              accumulate=True, act=RELU)
    else:
        if x2 is not None:
            raise RuntimeError("identity shortcut with a concatenated input")
        out = ops.affine_act(t2, one, zero, res=x1, relu=True)
    if pool:
        return out, S, ops.maxpool2_fwd(out)
    return out, S


def _ex_fusable(dtype, n, h, w, c1, c2, cout, act):
    """rr_igemm_ex takes the epilogue ``act`` on this conv with the kernel the
    plain conv would run anyway: the tap-reuse conv, or the row-streaming
    kernel on the 64 -> 64 maps it takes (whole rows at 32 / 64, column strips
    at the reference's 224; its eval epilogues, stream3.hip F_PRELU / F_RES)."""
    if dtype != torch.bfloat16:
        return False
    if act & ops.RR_ACT_POOL and (h < 2 or w < 2):
        return False                       # (no 2x2 window: the unfused max-pool path)
    rd = ops.rr_dtype(dtype)
    fused = ops.igemm_kernel_name(ops.IgemmDesc(rd, RR_CONV3X3, n, h, w, c1, c2, cout, 0, act,
                                                0, 1, 0, 0, 0))
    plain = ops.igemm_kernel_name(ops.IgemmDesc(rd, RR_CONV3X3, n, h, w, c1, c2, cout, 0, 0,
                                                0, 1, 0, 0, 0))
    return (fused.startswith("conv3r") or fused.startswith("stream3")) and fused == plain


def resblock_forward(blk, x1, x2, n, h, w, wc, dt, training, need_bwd, pool=False):
    """-> (out, S), or (out, S, (pooled, idx)) with ``pool`` (the 2x2 max-pool
    that follows the encoder blocks, fused into the residual tail)."""
    if _FOLD_BN and not training and not need_bwd:
        return resblock_forward_eval_folded(blk, x1, x2, n, h, w, wc, dt, pool)
    cb = blk.conv_block
    c1, bn1, pr, c2, bn2 = cb[0], cb[1], cb[2], cb[3], cb[4]
    cout = c1.weight.shape[0]
    P = n * h * w
    pk1 = wc.conv(c1.weight, dt, dgrad=need_bwd)
    t1, _, st1 = ops.igemm(RR_CONV3X3, x1, x2, n, h, w, pk1[0], cout, bias=c1.bias, stats=training)
    s1, sh1, m1, i1 = _bn_affine(bn1, st1, c1.bias, P, training, need_bwd=need_bwd)
    pk2 = wc.conv(c2.weight, dt, dgrad=need_bwd)
    if _FOLD_BN1 and training and c2.bias is not None and ops.igemm_pre_ok(t1.dtype, n, h, w, cout, cout) and \
            (not need_bwd or ops.wgrad_pre_ok(t1.dtype, n, h, w, cout, cout)):
        # BN1 + PReLU applied to conv2's input rows as they land in the
        # streaming kernels' rings (rr_igemm_pre / rr_wgrad_pre): a1 is never
        # stored -- bitwise the a1 the affine pass would write
        a1 = None
        t2, _, st2 = ops.igemm_pre(t1, n, h, w, pk2[0], cout, c2.bias, s1, sh1, pr.weight)
    else:
        a1 = ops.affine_act(t1, s1, sh1, alpha=pr.weight)
        t2, _, st2 = ops.igemm(RR_CONV3X3, a1, None, n, h, w, pk2[0], cout, bias=c2.bias,
                               stats=training)
    has_sc = block_has_shortcut(blk)
    # (scale, shift) of bn2 and the shortcut BN as rows of two [2, C] buffers:
    # the backward's recomputed ReLU mask reads them as pairs (no stack copy)
    pair = None
    if has_sc and need_bwd and _RECOMPUTE_MASK:
        pair = (torch.empty(2, cout, dtype=torch.float32, device=x1.device),
                torch.empty(2, cout, dtype=torch.float32, device=x1.device))
    out2 = (pair[0][0], pair[1][0]) if pair else None
    S = Bag(x1=x1, x2=x2, n=n, h=h, w=w)
    if has_sc:
        sc0, sc1 = blk.shortcut[0], blk.shortcut[1]
        pks = wc.conv(sc0.weight, dt, dgrad=need_bwd)
        s, _, sts = ops.igemm(RR_CONV1X1, x1, x2, n, h, w, pks[0], cout, bias=sc0.bias,
                              stats=training)
        outs = (pair[0][1], pair[1][1]) if pair else None
        if training and _PAIR_FINALIZE:
            # both statistics are ready: the two finalizes as one launch
            (s2, sh2, m2, i2), (ss, shs, ms, is_) = ops.bn_finalize_pair(
                _fin_args(bn2, st2, c2.bias, P, out2), _fin_args(sc1, sts, sc0.bias, P, outs))
        else:
            s2, sh2, m2, i2 = _bn_affine(bn2, st2, c2.bias, P, training, out=out2, need_bwd=need_bwd)
            ss, shs, ms, is_ = _bn_affine(sc1, sts, sc0.bias, P, training, out=outs,
                                          need_bwd=need_bwd)
        res, rsc, rsh = s, ss, shs
        if need_bwd:
            S.update(s=s, ms=ms, is_=is_, pks=pks, s2=s2, sh2=sh2, ss=ss, shs=shs, pair=pair)
    else:
        if x2 is not None:
            raise RuntimeError("identity shortcut with a concatenated input")
        s2, sh2, m2, i2 = _bn_affine(bn2, st2, c2.bias, P, training, out=out2, need_bwd=need_bwd)
        res, rsc, rsh = x1, None, None
    pooled = None
    if pool and _FUSED_POOL and h % 2 == 0 and w % 2 == 0 and cout % 8 == 0:
        out, yp, idx = ops.affine_act_pool(t2, s2, sh2, res=res, res_scale=rsc, res_shift=rsh, relu=True)
        pooled = (yp, idx)
    else:
        out = ops.affine_act(t2, s2, sh2, res=res, res_scale=rsc, res_shift=rsh, relu=True)
        if pool:
            pooled = ops.maxpool2_fwd(out)
    if need_bwd:
        S.update(t1=t1, a1=a1, t2=t2, out=out, s1=s1, sh1=sh1, m1=m1, i1=i1, m2=m2, i2=i2,
                 pk1=pk1, pk2=pk2, eval=not training)
    return (out, S, pooled) if pool else (out, S)


def resblock_zero_grad_params(blk):
    """conv biases followed by a train-mode BN: exactly-zero gradients."""
    z = [blk.conv_block[0].bias, blk.conv_block[3].bias]
    if block_has_shortcut(blk):
        z.append(blk.shortcut[0].bias)
    return z


def resblock_backward(blk, S, g_out, sink, pool=None, convout=None, reduce_side=False):
    """``pool=(dy_pool, idx)``: the output also fed a 2x2 max-pool whose
    backward is fused into the tail BN backward (no separate pass).
    ``convout=(final, dy)``: the output fed the final 1x1 conv ``final`` and
    ``dy`` is that conv's output grad (``g_out`` None): its backward runs here,
    fused with the tail BN's reduce where the library takes it (the conv's
    input grad is then never stored)."""
    cb = blk.conv_block
    c1, bn1, pr, c2, bn2 = cb[0], cb[1], cb[2], cb[3], cb[4]
    n, h, w = S.n, S.h, S.w
    cout = c1.weight.shape[0]
    x1, x2 = S.x1, S.x2
    c_in1 = x1.shape[-1]
    c_in2 = x2.shape[-1] if x2 is not None else 0
    cin = c_in1 + c_in2
    has_sc = block_has_shortcut(blk)
    gx1 = gx2 = None
    # eval-mode BatchNorm: running statistics, no batch-statistic terms, and
    # the conv biases feeding the BNs get their (non-zero) grads
    ev = bool(S.get("eval"))
    # (reduce_side: the caller joins the reduce stream, join_wgrad_reduces)
    rs = reduce_stream(x1.device) if reduce_side and x1.is_cuda else None

    def wgrad(*args, **kw):
        ops.wgrad(*args, reduce_stream=rs, **kw)
    if has_sc:
        sc0, sc1 = blk.shortcut[0], blk.shortcut[1]
        # the ReLU mask from t2 and s as the forward formed the output (mask
        # kind 4/5): one tensor read fewer in both BN-backward passes
        rec = None
        if _RECOMPUTE_MASK and cout % 8 == 0 and 256 % (cout // 8) == 0:
            rec = S.pair if S.get("pair") is not None else (torch.stack((S.s2, S.ss)),
                                                             torch.stack((S.sh2, S.shs)))
        outs2 = dict(dgamma0=sink[bn2.weight], dbeta0=sink[bn2.bias], dgamma1=sink[sc1.weight],
                     dbeta1=sink[sc1.bias])
        r = None
        if convout is not None:
            final, dy = convout
            if _FUSED_CONVOUT_BN and rec is not None and not ev and pool is None:
                r = ops.bn_backward_convout(dy, S.out, final.weight, S.t2, S.m2, S.i2, bn2.weight,
                                            S.s, S.ms, S.is_, sc1.weight, rec, outs2,
                                            dw=sink[final.weight], db=sink[final.bias])
            if r is None:
                g_out, _, _ = ops.conv_out_bwd(dy, S.out, final.weight, mask_relu=False,
                                               dw=sink[final.weight], db=sink[final.bias])
            sink.ready(_params(final))
        if r is None:
            r = ops.bn_backward(g_out, S.t2, S.m2, S.i2, bn2.weight, mask_kind=1, aux=S.out,
                                pool=pool, recompute=rec, t1=S.s, mean1=S.ms, inv1=S.is_,
                                gamma1=sc1.weight, outs=outs2, eval_mode=ev,
                                dbias=(sink[c2.bias], sink[sc0.bias]) if ev else None)
        dt2, ds = r["dt0"], r["dt1"]
    else:
        if convout is not None:
            final, dy = convout
            g_out, _, _ = ops.conv_out_bwd(dy, S.out, final.weight, mask_relu=False,
                                           dw=sink[final.weight], db=sink[final.bias])
            sink.ready(_params(final))
        gx1 = torch.empty_like(x1)
        r = ops.bn_backward(g_out, S.t2, S.m2, S.i2, bn2.weight, mask_kind=1, aux=S.out, pool=pool,
                            want_gm=True, gm_out=gx1,
                            outs=dict(dgamma0=sink[bn2.weight], dbeta0=sink[bn2.bias]),
                            eval_mode=ev, dbias=(sink[c2.bias], None) if ev else None)
        dt2 = r["dt0"]
    if S.a1 is None:
        # (the forward folded BN1 + PReLU into conv2: its weight grad reads t1)
        ops.wgrad_pre(dt2, S.t1, n, h, w, cout, S.s1, S.sh1, pr.weight, dw=sink[c2.weight])
    else:
        wgrad(RR_CONV3X3, dt2, S.a1, None, n, h, w, cout, dw=sink[c2.weight])
    outs1 = dict(dgamma0=sink[bn1.weight], dbeta0=sink[bn1.bias], dalpha=sink[pr.weight])
    if FUSE_BNBWD:
        # conv2 dgrad whose epilogue applies the PReLU backward and reduces
        # BN1's backward sums (no separate pass over dL/d(PReLU out))
        gm1, part, rows, arows = ops.igemm_bnbwd(RR_CONV3X3, dt2, n, h, w, S.pk2[1], cout, S.t1,
                                                 S.m1, S.i1, S.s1, S.sh1, pr.weight)
        r1 = ops.bn_backward_rows(gm1, part, rows, arows, S.t1, S.m1, S.i1, bn1.weight,
                                  outs=outs1, eval_mode=ev, dbias=(sink[c1.bias],) if ev else None)
    else:
        da1, _, _ = ops.igemm(RR_CONV3X3, dt2, None, n, h, w, S.pk2[1], cout)
        r1 = ops.bn_backward(da1, S.t1, S.m1, S.i1, bn1.weight, mask_kind=2, aux=S.t1,
                             aff_s=S.s1, aff_b=S.sh1, alpha=pr.weight, outs=outs1,
                             eval_mode=ev, dbias=(sink[c1.bias], None) if ev else None)
    dt1 = r1["dt0"]
    wgrad(RR_CONV3X3, dt1, x1, x2, n, h, w, cout, dw=sink[c1.weight])
    split = c_in1 if c_in2 else 0
    if has_sc:
        wgrad(RR_CONV1X1, ds, x1, x2, n, h, w, cout, dw=sink[sc0.weight])
        if _SPLIT_DGRAD and split == 64 and cin == 128 and cout == 64 and \
                _streams_half(dt1.dtype, n, h, w):
            # dec1 (64 + 64 -> 64): each half of the concat grad is a 64 -> 64
            # dgrad over a contiguous slice of the packed weights, the shape
            # the row-streaming kernel serves (only there: a slice of the
            # [c_in][9][c_out] rows is not a pack the tap-reuse conv can
            # read -- its weight tiles sit behind the whole pack)
            half = 64 * 9 * cout
            if _FUSED_SC_DGRAD:
                # each half + the shortcut's 1x1 dgrad of it in the same pass
                # (no 1.3 GB accumulate pass over both halves)
                hs = 64 * cout
                gx1 = ops.igemm_dgrad_sc(dt1, n, h, w, S.pk1[1][:half], 64, ds, S.pks[1][:hs])
                gx2 = ops.igemm_dgrad_sc(dt1, n, h, w, S.pk1[1][half:], 64, ds, S.pks[1][hs:]) \
                    if gx1 is not None else None
                if gx2 is not None:
                    sink.ready(_params(blk))
                    return gx1, gx2
            gx1, _, _ = ops.igemm(RR_CONV3X3, dt1, None, n, h, w, S.pk1[1][:half], 64)
            gx2, _, _ = ops.igemm(RR_CONV3X3, dt1, None, n, h, w, S.pk1[1][half:], 64)
        else:
            gx1, gx2, _ = ops.igemm(RR_CONV3X3, dt1, None, n, h, w, S.pk1[1], cin, split=split)
        ops.igemm(RR_CONV1X1, ds, None, n, h, w, S.pks[1], cin, out=gx1, out2=gx2, split=split,
                  accumulate=True)
    else:
        ops.igemm(RR_CONV3X3, dt1, None, n, h, w, S.pk1[1], cin, out=gx1, accumulate=True)
    sink.ready(_params(blk))
    return gx1, gx2


def resunet_block_names():
    return ["res1", "res2", "res3", "bottleneck.0", "bottleneck.1", "bottleneck.2", "dec3", "dec2",
            "dec1"]


def _skip_align(u, h, w):
    """14:169-182: ``if d.size() != r.size(): d = F.interpolate(d, size=r.shape[2:])``.
    The reference compares full sizes (channels included), so the nearest
    resize always runs; at equal spatial sizes it is the identity (no launch
    here).  Returns (aligned, resized?)."""
    if u.shape[1] == h and u.shape[2] == w:
        return u, False
    return ops.nearest_resize(u, h, w), True


def resunet_forward(m, x, wc, dt, training, need_bwd):
    wc.begin()
    n, _, H, W = x.shape
    if H < 8 or W < 8:
        raise ValueError("ResUNet needs H, W >= 8 (three 2x2 max-pools, floor mode)")
    # floor-mode pool sizes (14:155-161)
    H2, W2 = H // 2, W // 2
    H3, W3 = H2 // 2, W2 // 2
    H4, W4 = H3 // 2, W3 // 2
    S = Bag(n=n, H=H, W=W, x=x, sizes=((H, W), (H2, W2), (H3, W3), (H4, W4)))
    pr = m.enc1[1]
    # conv + PReLU in one pass (the pre-activation kept for the PReLU backward)
    e1, e1pre = ops.first_conv_fwd(x, m.enc1[0].weight, m.enc1[0].bias, dt,
                                   wc.conv_in(m.enc1[0].weight, m.enc1[0].bias, dt), act=2,
                                   alpha=pr.weight, want_pre=need_bwd)
    if need_bwd:
        S.e1pre = e1pre
    r1, S.res1, (p1, i1) = resblock_forward(m.res1, e1, None, n, H, W, wc, dt, training, need_bwd,
                                            pool=True)
    r2, S.res2, (p2, i2) = resblock_forward(m.res2, p1, None, n, H2, W2, wc, dt, training,
                                            need_bwd, pool=True)
    r3, S.res3, (p3, i3) = resblock_forward(m.res3, p2, None, n, H3, W3, wc, dt, training,
                                            need_bwd, pool=True)
    b = p3
    for i in range(3):
        b, S[f"bottleneck.{i}"] = resblock_forward(m.bottleneck[i], b, None, n, H4, W4, wc,
                                                   dt, training, need_bwd)
    u3, pku3 = _convT_up(wc, dt, m.up3, b, n, H4, W4, need_bwd)
    u3, al3 = _skip_align(u3, H3, W3)
    d3, S.dec3 = resblock_forward(m.dec3, u3, r3, n, H3, W3, wc, dt, training, need_bwd)
    u2, pku2 = _convT_up(wc, dt, m.up2, d3, n, H3, W3, need_bwd)
    u2, al2 = _skip_align(u2, H2, W2)
    d2, S.dec2 = resblock_forward(m.dec2, u2, r2, n, H2, W2, wc, dt, training, need_bwd)
    u1, pku1 = _convT_up(wc, dt, m.up1, d2, n, H2, W2, need_bwd)
    u1, al1 = _skip_align(u1, H, W)
    d1, S.dec1 = resblock_forward(m.dec1, u1, r1, n, H, W, wc, dt, training, need_bwd)
    out = ops.conv_out_fwd(d1, m.final.weight, m.final.bias,
                           wpack=wc.conv(m.final.weight, dt, dgrad=False)[0])
    if need_bwd:
        S.update(e1=e1, r1=r1, r2=r2, r3=r3, i1=i1, i2=i2, i3=i3, b=b, d3=d3, d2=d2, d1=d1,
                 pku3=pku3, pku2=pku2, pku1=pku1, aligned=(al1, al2, al3))
    return out, S


_UNIT = {}


def _unit_affine(C, device):
    key = (C, str(device))
    if key not in _UNIT:
        _UNIT[key] = (torch.ones(C, device=device), torch.zeros(C, device=device))
    return _UNIT[key]


def resunet_grad_order(m):
    return _params(m.final, m.dec1, m.up1, m.dec2, m.up2, m.dec3, m.up3, m.bottleneck[2],
                   m.bottleneck[1], m.bottleneck[0], m.res3, m.res2, m.res1, m.enc1)


def resunet_zero_grad_params(m):
    z = []
    for name in resunet_block_names():
        z.extend(resblock_zero_grad_params(m.get_submodule(name)))
    return z


# A/B and test switches (RR_PATH, _lib.path_flag; the unfused forms are the
# paths of the shapes / dtypes the fused kernels do not take).  The fused
# first-conv backward (first_wgrad=0: the prelu_bwd + im2col + wgrad
# sequence)
_FUSED_FIRST_WGRAD = path_flag("first_wgrad", 1) != 0
# the residual tail + max-pool fusion (fused_pool=0: separate pool)
_FUSED_POOL = path_flag("fused_pool", 1) != 0
# A/B switch for the encoder max-pool backward fused into the tail BN backward
_FUSED_POOL_BWD = path_flag("fused_pool_bwd", 1) != 0
# A/B switch: dec1's concat dgrad as two 64 -> 64 row-streaming launches
_SPLIT_DGRAD = path_flag("split_dgrad", 1) != 0
# A/B switch: the final conv's backward fused with dec1's tail BN reduce, its
# input grad recomputed in the apply instead of stored (rr_conv_out_bwd_bnred)
_FUSED_CONVOUT_BN = path_flag("convout_bn", 1) != 0
# A/B switch: ... each with the shortcut's 1x1 dgrad summed in (rr_igemm_dgrad_sc)
_FUSED_SC_DGRAD = path_flag("sc_dgrad", 1) != 0


def _streams_half(dtype, n, h, w):
    """the 64 -> 64 dgrad of one concat half at n x h x w runs on the
    row-streaming kernel (which reads the [c_in][9][c_out] rows only)"""
    d = ops.IgemmDesc(ops.rr_dtype(dtype), RR_CONV3X3, n, h, w, 64, 0, 64, 0, 0, 0, 0, 0, 0, 0)
    return ops.igemm_kernel_name(d).startswith("stream3")
# A/B switch: the BN-shortcut tail's ReLU mask recomputed from t2 and the
# shortcut's pre-BN output (read anyway) instead of read from the block output
_RECOMPUTE_MASK = path_flag("recompute_mask", 1) != 0
# (a residual block's weight grads on a side stream, concurrent with the
# dgrad / BN-backward chain they do not feed, measured 29.2k vs 29.4k img/s
# in a same-box A/B -- the concurrent kernels contend for the CUs and L2 --
# and was removed in round 6)
# A/B switch: the weight grads' split-K reduces (rr_wgrad_reduce) and the
# convT bias sums on a side stream -- nothing in the backward reads them, so
# they run beside the next dgrad instead of between it and its producer;
# joined where the gradients are read (join_wgrad_reduces: the end of the
# backward, each data-parallel bucket).  Off: the graph step measured 2.2 %
# slower with it (14.52 vs 14.21 ms, 3 interleaved rounds,
# profiles/r5u_abstep_reduce_side.txt) -- the reduce workgroups take CUs the
# next dgrad's one-per-CU tiles are waiting for
_WGRAD_REDUCE_SIDE = path_flag("wgrad_reduce_side", 0) != 0
_REDUCE_SIDE = {}


def reduce_stream(device):
    """the stream the weight-grad reduces fork onto (one per device)"""
    s = _REDUCE_SIDE.get(device)
    if s is None:
        s = _REDUCE_SIDE[device] = torch.cuda.Stream(device)
    return s


def join_wgrad_reduces(stream=None, device=None):
    """``stream`` (default: the current one) waits for every weight-grad
    reduce forked so far"""
    for dev, s in _REDUCE_SIDE.items():
        if device is not None and dev != device:
            continue
        (stream or torch.cuda.current_stream(dev)).wait_stream(s)
_PACK_SIDE = {}


def _pack_stream(device):
    """the stream WeightCache.prefetch() forks its re-pack onto"""
    s = _PACK_SIDE.get(device)
    if s is None:
        s = _PACK_SIDE[device] = torch.cuda.Stream(device)
    return s


def resunet_backward(m, S, g_out, sink):
    n = S.n
    (H, W), (H2, W2), (H3, W3), (H4, W4) = S.sizes
    al1, al2, al3 = S.aligned
    sd = _WGRAD_REDUCE_SIDE and g_out.is_cuda
    # the final conv's backward runs inside dec1's (fused with its tail BN reduce)
    g_u1, g_r1 = resblock_backward(m.dec1, S.dec1, None, sink, convout=(m.final, g_out),
                                   reduce_side=sd)
    if al1:
        g_u1 = ops.nearest_resize_bwd(g_u1, 2 * H2, 2 * W2)
    g_d2 = _convT_bwd(m.up1, S.pku1, g_u1, S.d2, n, H2, W2, sink, side=sd)
    sink.ready(_params(m.up1))
    g_u2, g_r2 = resblock_backward(m.dec2, S.dec2, g_d2, sink, reduce_side=sd)
    if al2:
        g_u2 = ops.nearest_resize_bwd(g_u2, 2 * H3, 2 * W3)
    g_d3 = _convT_bwd(m.up2, S.pku2, g_u2, S.d3, n, H3, W3, sink, side=sd)
    sink.ready(_params(m.up2))
    g_u3, g_r3 = resblock_backward(m.dec3, S.dec3, g_d3, sink, reduce_side=sd)
    if al3:
        g_u3 = ops.nearest_resize_bwd(g_u3, 2 * H4, 2 * W4)
    g_b = _convT_bwd(m.up3, S.pku3, g_u3, S.b, n, H4, W4, sink, side=sd)
    sink.ready(_params(m.up3))
    for i in (2, 1, 0):
        g_b, _ = resblock_backward(m.bottleneck[i], S[f"bottleneck.{i}"], g_b, sink, reduce_side=sd)
    if _FUSED_POOL_BWD and g_b.dtype == torch.bfloat16 and H % 8 == 0 and W % 8 == 0:
        # each encoder block's output fed the skip concat and the pool: the
        # pool backward runs inside that block's tail BN backward
        g_p2, _ = resblock_backward(m.res3, S.res3, g_r3, sink, pool=(g_b, S.i3), reduce_side=sd)
        g_p1, _ = resblock_backward(m.res2, S.res2, g_r2, sink, pool=(g_p2, S.i2), reduce_side=sd)
        g_e1, _ = resblock_backward(m.res1, S.res1, g_r1, sink, pool=(g_p1, S.i1), reduce_side=sd)
    else:
        ops.maxpool2_bwd(g_b, S.i3, H3, W3, out=g_r3, accumulate=True)
        g_p2, _ = resblock_backward(m.res3, S.res3, g_r3, sink, reduce_side=sd)
        ops.maxpool2_bwd(g_p2, S.i2, H2, W2, out=g_r2, accumulate=True)
        g_p1, _ = resblock_backward(m.res2, S.res2, g_r2, sink, reduce_side=sd)
        ops.maxpool2_bwd(g_p1, S.i1, H, W, out=g_r1, accumulate=True)
        g_e1, _ = resblock_backward(m.res1, S.res1, g_r1, sink, reduce_side=sd)
    pr = m.enc1[1]
    if g_e1.dtype == torch.bfloat16 and W % 8 == 0 and _FUSED_FIRST_WGRAD:
        # PReLU backward + first-conv wgrad in one pass over the image
        ops.first_conv_wgrad_act(S.x, g_e1, S.e1pre, 2, pr.weight, sink[m.enc1[0].weight],
                                 sink[m.enc1[0].bias], dalpha=sink[pr.weight])
    else:
        g_e1pre, _ = ops.prelu_bwd(g_e1, S.e1pre, pr.weight, dalpha=sink[pr.weight])
        ops.first_conv_wgrad(ops.im2col3(S.x, g_e1pre.dtype), g_e1pre, sink[m.enc1[0].weight],
                             sink[m.enc1[0].bias])
    if sd:
        join_wgrad_reduces(device=g_out.device)
    sink.ready(_params(m.enc1))


# ---------------------------------------------------------------------------
# VGG16 features (torchvision cfg D) -- perceptual slice and classifier trunk

def _pool_2x2(mod):
    """MaxPool2d(2) / MaxPool2d(2, 2): the window the conv epilogue pools"""
    def two(v):
        return v == 2 or v == (2, 2)
    ks = getattr(mod, "kernel_size", None)
    st = getattr(mod, "stride", None)
    return (two(ks) and two(st if st is not None else ks)
            and getattr(mod, "padding", 0) in (0, (0, 0))
            and getattr(mod, "dilation", 1) in (1, (1, 1)) and not getattr(mod, "ceil_mode", False))


def vgg_layers(features, upto=None):
    """[(kind, module)] of features[:upto]; ReLU after each conv is fused."""
    mods = list(features)
    if upto is not None:
        mods = mods[:upto]
    out = []
    for mod in mods:
        name = type(mod).__name__
        if name == "Conv2d":
            out.append(("conv", mod))
        elif name == "MaxPool2d":
            out.append(("pool", mod))
        elif name == "ReLU":
            if not out or out[-1][0] != "conv":
                raise RuntimeError("unsupported VGG layer order")
            out[-1] = ("conv_relu", out[-1][1])
        else:
            raise RuntimeError(f"unsupported VGG feature layer {name}")
    return out


def vgg_features_forward(features, x, wc, dt, upto=None, need_bwd=False):
    """x: NCHW fp32 image.  Returns NHWC features and the saved state."""
    wc.begin()
    n, _, H, W = x.shape
    layers = vgg_layers(features, upto)
    S = Bag(n=n, H=H, W=W, acts=[], layers=layers)
    h, w = H, W
    cur = None
    skip_pool = False
    for li, (kind, mod) in enumerate(layers):
        if skip_pool:                    # (its max-pool ran in the conv's epilogue)
            skip_pool = False
            h, w = h // 2, w // 2
            continue
        if kind in ("conv", "conv_relu"):
            act = RELU if kind == "conv_relu" else 0
            nxt_pool = li + 1 < len(layers) and layers[li + 1][0] == "pool" and \
                _pool_2x2(layers[li + 1][1])
            cout = mod.weight.shape[0]
            pname = ops.igemm_pool_kernel_name(ops.igemm_pool_desc(cur, n, h, w, cout, mod.bias is not None)) \
                if cur is not None and kind == "conv_relu" and nxt_pool and cur.dtype == torch.bfloat16 \
                and h % 2 == 0 and w % 2 == 0 else "unsupported"
            if pname != "unsupported":
                # conv + ReLU + MaxPool2d in one pass (rr_igemm_pool), the
                # full-size map never written; with a backward the window
                # index is kept and the pool's backward takes its ReLU mask
                # from the pooled output ("pool_p", rr_maxpool2_bwd_pooled)
                pk = wc.conv(mod.weight, dt, dgrad=need_bwd)
                y, idx = ops.igemm_pool(cur, n, h, w, pk[0], cout, bias=mod.bias,
                                        want_idx=need_bwd or pname.startswith("stream3"))
                S.acts.append((kind, mod, cur, pk, h, w, None))
                S.acts.append(("pool_p", layers[li + 1][1], y, None, h, w, idx if need_bwd else None))
                cur = y
                skip_pool = True
                continue
            if cur is None:
                y, _ = ops.first_conv_fwd(x, mod.weight, mod.bias, dt,
                                          wc.conv_in(mod.weight, mod.bias, dt), act=act)
                pk = wc.conv(mod.weight, dt, dgrad=True) if need_bwd else None
            else:
                pk = wc.conv(mod.weight, dt, dgrad=need_bwd)
                y, _, _ = ops.igemm(RR_CONV3X3, cur, None, n, h, w, pk[0], mod.weight.shape[0],
                                    bias=mod.bias, act=act)
            S.acts.append((kind, mod, cur, pk, h, w, None))
            cur = y
        else:
            if not _pool_2x2(mod):
                raise NotImplementedError(f"VGG feature pool {mod}: only MaxPool2d(2, 2) (floor) "
                                          "is implemented")
            y, idx = ops.maxpool2_fwd(cur)
            S.acts.append((kind, mod, cur, None, h, w, idx))
            h, w = h // 2, w // 2
            cur = y
    S.out = cur
    return cur, S


def vgg_features_backward_input(S, g_pre_last, x_grad_out=None, accumulate=False):
    """Input (image) gradient of the frozen features: dgrad only, no wgrad.

    g_pre_last is the gradient at the PRE-activation of the last layer if it is
    a conv_relu (the caller folds the last ReLU mask in).  Returns the NCHW
    fp32 image grad (accumulated into x_grad_out if given)."""
    g = g_pre_last
    acts = S.acts
    for li in range(len(acts) - 1, -1, -1):
        kind, mod, xin, pk, h, w, idx = acts[li]
        if kind == "pool_p":
            # (fused conv + ReLU + pool: xin is the pooled output)
            g = ops.maxpool2_bwd_pooled(g, idx, xin, h, w)
            continue
        if kind == "pool":
            # input of the pool is the previous layer's (relu) output
            prev_relu = li > 0 and acts[li - 1][0] == "conv_relu"
            g = ops.maxpool2_bwd(g, idx, h, w, mask=xin if prev_relu else None)
            continue
        if xin is None:   # first layer: image grad
            cin = mod.weight.shape[1]
            return ops.conv_in_dgrad(g, mod.weight, cin, out=x_grad_out, accumulate=accumulate,
                                     wpack_dgrad=pk[1] if pk is not None else None)
        prev_relu = acts[li - 1][0] == "conv_relu"
        g, _, _ = ops.igemm(RR_CONV3X3, g, None, S.n, h, w, pk[1], mod.weight.shape[1],
                            mask=xin if prev_relu else None)
    raise RuntimeError("unreachable")


def vgg_classifier_forward(vgg, x, wc, dt):
    """Eval-mode VGG16 logits (Dropout = identity): 18:46."""
    f, _ = vgg_features_forward(vgg.features, x, wc, dt)
    n = x.shape[0]
    pooled = ops.adaptive_avgpool_flatten(f, 7, 7)        # [n, 25088] (NCHW flatten)
    h = pooled.view(n, 1, 1, -1)
    cls = [m for m in vgg.classifier if type(m).__name__ == "Linear"]
    for i, lin in enumerate(cls):
        pk = wc.linear(lin.weight, dt)
        last = i == len(cls) - 1
        h, _, _ = ops.igemm(RR_CONV1X1, h, None, n, 1, 1, pk[0], lin.weight.shape[0],
                            bias=lin.bias, act=0 if last else RELU)
    return h.view(n, -1)
