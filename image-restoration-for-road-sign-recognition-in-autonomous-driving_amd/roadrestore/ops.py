"""Tensor-level wrappers over the C ABI (one launch each, current HIP stream).

Activations are NHWC tensors ([N, H, W, C] contiguous) in the compute dtype
(torch.float32 or torch.bfloat16).  Every wrapper allocates its outputs from
the PyTorch caching allocator (PyTorch is plumbing here: device memory and
streams) and launches exactly one C-ABI entry point.  No op has a PyTorch or
CPU fallback: a missing library or device raises.
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import (path_flag, RR_ACT_NOFULL, RR_ACT_POOL, RR_ACT_PRELU, RR_ACT_RES, RR_BF16, RR_F32, RR_CONV1X1, RR_CONV3X3,
                   RR_CONVT_DOWN, RR_CONVT_UP, RR_DISTORT_KMAX, BnBwdDesc, DistortParam, IgemmDesc, PackJob, WgradDesc, lib)

__all__ = [
    "rr_dtype", "stream", "pack_conv", "pack_convT", "bias_tile4", "igemm", "wgrad",
    "bn_finalize", "bn_eval_affine", "affine_act", "bn_backward", "channel_sum",
    "maxpool2_fwd", "maxpool2_bwd", "conv_in_fwd", "conv_in_wgrad", "conv_in_dgrad",
    "prelu_bwd", "conv_out_fwd", "conv_out_bwd", "nchw_to_nhwc", "nhwc_to_nchw",
    "loss_fwd", "loss_bwd", "adamw_", "to_uint8_hwc", "psnr_u8", "argmax_rows",
    "adaptive_avgpool_flatten", "zero_", "resize_bilinear_u8", "ssim_u8", "distort_u8",
    "motion_blur_kernel", "first_conv_wgrad_act", "affine_act_pool", "nearest_resize",
    "nearest_resize_bwd", "fold_conv_bn", "bn_stats",
]


def rr_dtype(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return RR_F32
    if dt == torch.bfloat16:
        return RR_BF16
    raise TypeError(f"unsupported compute dtype {dt}")


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("roadrestore ops need device tensors (no CPU fallback)")


# Optional launch probe (bench.py): probe(kernel_symbol, algorithmic_flops, launch_fn, shape_tag)
PROBE = None
# Optional launch log (tests): a list that every igemm / wgrad launch appends
# (kernel_symbol, shape_tag) to -- the symbol is the library's own choice
# (rr_igemm_kernel_name / rr_wgrad_kernel_name), so a test can assert the
# schedule it exercises.
LAUNCH_LOG = None


def igemm_kernel_name(d, bnbwd=False):
    """The kernel rr_igemm / rr_igemm_bnbwd launches for descriptor ``d``."""
    return lib().rr_igemm_kernel_name(C.byref(d), int(bnbwd)).decode()


def wgrad_kernel_name(d):
    """The kernel rr_wgrad launches for descriptor ``d``."""
    return lib().rr_wgrad_kernel_name(C.byref(d)).decode()


def _launch(sym_fn, flops, launch, tag):
    if LAUNCH_LOG is not None:
        LAUNCH_LOG.append((sym_fn(), tag))
    if PROBE is None:
        launch()
    else:
        PROBE(sym_fn(), flops, launch, tag)


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# ---------------------------------------------------------------------------
# weights

def pack_conv(w: torch.Tensor, dtype: torch.dtype, fwd=True, dgrad=True):
    """fp32 [co][ci][k][k] -> (fwd [co][k*k][ci], dgrad [ci][k*k flipped][co]);
    bf16 3x3 packs carry the tap-reuse conv's weight tiles behind that
    layout (rr_pack_conv_elems)."""
    _need_cuda(w)
    co, ci, k, _ = w.shape
    ne = pack_elems(dtype, co, ci, k)
    wf = torch.empty(ne, dtype=dtype, device=w.device) if fwd else None
    wd = torch.empty(ne, dtype=dtype, device=w.device) if dgrad else None
    lib().check(lib().rr_pack_conv(rr_dtype(dtype), co, ci, k, _p(w.contiguous()), _p(wf),
                                   _p(wd), stream()), "rr_pack_conv")
    return wf, wd


def pack_elems(dtype, co, ci, k):
    """elements of one conv pack buffer (rr_pack_conv_elems)"""
    return int(lib().rr_pack_conv_elems(rr_dtype(dtype), co, ci, k))


class PackBatch:
    """All conv packs of a network as ONE launch (rr_pack_conv_batch): the
    packed outputs are allocated once and re-packed in place each call, from
    a job table kept in device memory.  ``entries``: [(w, dtype, dgrad)]."""

    def __init__(self, entries):
        dt = {e[1] for e in entries}
        if len(dt) != 1:
            raise ValueError("one compute dtype per pack batch")
        self.dtype = dt.pop()
        self.entries = list(entries)
        self.out = []
        jobs = (PackJob * len(entries))()
        begin = 0
        for j, (w, _, dgrad) in enumerate(entries):
            _need_cuda(w)
            if not w.is_contiguous():
                raise ValueError("pack batch needs contiguous weights")
            co, ci, k, _ = w.shape
            ne = pack_elems(self.dtype, co, ci, k)
            wf = torch.empty(ne, dtype=self.dtype, device=w.device)
            wd = torch.empty(ne, dtype=self.dtype, device=w.device) if dgrad else None
            self.out.append((wf, wd))
            jobs[j] = PackJob(_p(w), _p(wf), _p(wd), co, ci, k, 0, begin)
            begin += w.numel()
        self.total = begin
        self.sig = tuple(w.data_ptr() for w, _, _ in entries)
        self.table = torch.frombuffer(bytearray(jobs), dtype=torch.uint8).to(entries[0][0].device)

    def valid(self):
        return self.sig == tuple(w.data_ptr() for w, _, _ in self.entries)

    def run(self):
        lib().check(lib().rr_pack_conv_batch(rr_dtype(self.dtype), len(self.entries), _p(self.table),
                                             self.total, stream()), "rr_pack_conv_batch")
        return self.out


def pack_convT(w: torch.Tensor, dtype: torch.dtype, up=True, down=True):
    """fp32 [ci][co][2][2] -> (up [tap*co][ci], down [ci][tap][co])."""
    _need_cuda(w)
    ci, co = w.shape[0], w.shape[1]
    wu = torch.empty(4 * co * ci, dtype=dtype, device=w.device) if up else None
    wd = torch.empty(4 * co * ci, dtype=dtype, device=w.device) if down else None
    lib().check(lib().rr_pack_convT(rr_dtype(dtype), ci, co, _p(w.contiguous()), _p(wu), _p(wd),
                                    stream()), "rr_pack_convT")
    return wu, wd


def bias_tile4(b: torch.Tensor):
    out = torch.empty(4 * b.numel(), dtype=torch.float32, device=b.device)
    lib().check(lib().rr_bias_tile4(b.numel(), _p(b), _p(out), stream()), "rr_bias_tile4")
    return out


# ---------------------------------------------------------------------------
# implicit GEMM

def igemm(mode, x1, x2, n, h, w, wpack, cout, bias=None, act=0, out=None, out2=None,
          split=0, accumulate=False, mask=None, stats=False, out_nchw=False, alpha=None, res=None,
          pool=False, pool_only=False):
    """Run rr_igemm (rr_igemm_ex with ``alpha`` -- act RR_ACT_PRELU --,
    ``res`` added before the activation, or ``pool`` / ``pool_only``: the
    2x2 max-pool of the result).  Returns (y1, y2, stats_partial_or_None);
    with ``pool`` y2 is the pooled [n, h/2, w/2, cout] tensor (y1 None with
    ``pool_only``).

    mode RR_CONV3X3 / RR_CONV1X1: y [n, h, w, cout]
    mode RR_CONVT_UP: GEMM columns 4*cout_t, y [n, 2h, 2w, cout/4]
    mode RR_CONVT_DOWN: x1 on the (2h, 2w) grid, y [n, h, w, cout]
    """
    _need_cuda(x1, wpack)
    dt = x1.dtype
    c1 = x1.shape[-1]
    c2 = x2.shape[-1] if x2 is not None else 0
    pool = pool or pool_only
    ex = alpha is not None or res is not None or pool
    if alpha is not None:
        act = RR_ACT_PRELU
    if res is not None:
        act |= RR_ACT_RES
    if pool:
        act |= RR_ACT_POOL | (RR_ACT_NOFULL if pool_only else 0)
    d = IgemmDesc(rr_dtype(dt), mode, n, h, w, c1, c2, cout, split, act, int(accumulate),
                  int(bias is not None), int(mask is not None), int(stats), int(out_nchw))
    dev = x1.device
    if pool:
        if split or out2 is not None:
            raise ValueError("pool: no split output")
        out2 = torch.empty((n, h // 2, w // 2, cout), dtype=dt, device=dev)
    if out is None and pool_only:
        pass
    elif out is None:
        if out_nchw:
            out = torch.empty((n, cout, h, w), dtype=torch.float32, device=dev)
        elif mode == RR_CONVT_UP:
            out = torch.empty((n, 2 * h, 2 * w, cout // 4), dtype=dt, device=dev)
        elif split:
            out = torch.empty((n, h, w, split), dtype=dt, device=dev)
        else:
            out = torch.empty((n, h, w, cout), dtype=dt, device=dev)
    if split and out2 is None:
        out2 = torch.empty((n, h, w, cout - split), dtype=dt, device=dev)
    st = None
    if stats:
        blocks = lib().rr_igemm_stat_blocks(C.byref(d))
        st = torch.empty((blocks, cout, 2), dtype=torch.float32, device=dev)
    def launch():
        if ex:
            lib().check(lib().rr_igemm_ex(C.byref(d), _p(x1), _p(x2), _p(wpack), _p(bias),
                                          _p(alpha), _p(res), _p(out), _p(out2) if pool else None,
                                          _p(mask), _p(st), stream()), "rr_igemm_ex")
        else:
            lib().check(lib().rr_igemm(C.byref(d), _p(x1), _p(x2), _p(wpack), _p(bias), _p(out),
                                       _p(out2), _p(mask), _p(st), stream()), "rr_igemm")
    taps = 9 if mode == RR_CONV3X3 else (4 if mode == RR_CONVT_DOWN else 1)
    _launch(lambda: igemm_kernel_name(d), 2.0 * n * h * w * cout * taps * (c1 + c2), launch,
            f"fwd m{mode} {n}x{h}x{w} c{c1}+{c2}->{cout}" + (f" ex{act}" if ex else ""))
    return out, out2, st


def igemm_pre_ok(dtype, n, h, w, cin, cout):
    """rr_igemm_pre takes conv2's bias + statistics forward on t1 (BN1 + PReLU
    folded into the input); False on an older A/B build without it"""
    f = getattr(lib(), "rr_igemm_pre_ok", None)
    d = IgemmDesc(rr_dtype(dtype), RR_CONV3X3, n, h, w, cin, 0, cout, 0, 0, 0, 1, 0, 1, 0)
    return bool(f is not None and f(C.byref(d)))


def igemm_pre(t1, n, h, w, wpack, cout, bias, pre_scale, pre_shift, pre_alpha):
    """conv3x3 (+ bias, BN statistics) of a1 = PReLU(t1 * pre_scale + pre_shift)
    with a1 never stored (rr_igemm_pre): -> (y, None, stats_partial)"""
    _need_cuda(t1, wpack)
    d = IgemmDesc(rr_dtype(t1.dtype), RR_CONV3X3, n, h, w, t1.shape[-1], 0, cout, 0, 0, 0, 1, 0, 1, 0)
    out = torch.empty((n, h, w, cout), dtype=t1.dtype, device=t1.device)
    st = torch.empty((lib().rr_igemm_stat_blocks(C.byref(d)), cout, 2), dtype=torch.float32,
                     device=t1.device)

    def launch():
        lib().check(lib().rr_igemm_pre(C.byref(d), _p(t1), _p(wpack), _p(bias), _p(pre_scale),
                                       _p(pre_shift), _p(pre_alpha), _p(out), _p(st), stream()),
                    "rr_igemm_pre")
    _launch(lambda: igemm_kernel_name(d), 2.0 * n * h * w * cout * 9 * t1.shape[-1], launch,
            f"fwd m{RR_CONV3X3} {n}x{h}x{w} c{t1.shape[-1]}+0->{cout} pre")
    return out, None, st


def wgrad_pre_ok(dtype, n, h, w, cin, cout):
    f = getattr(lib(), "rr_wgrad_pre_ok", None)
    d = WgradDesc(rr_dtype(dtype), RR_CONV3X3, n, h, w, cin, 0, cout, 0)
    return bool(f is not None and f(C.byref(d)))


def wgrad_pre(dy, t1, n, h, w, cout, pre_scale, pre_shift, pre_alpha, dw):
    """conv2's weight grad on a1 = PReLU(t1 * pre_scale + pre_shift), a1 never
    stored (rr_wgrad_pre: partial + reduce on the current stream)"""
    _need_cuda(dy, t1)
    d = WgradDesc(rr_dtype(dy.dtype), RR_CONV3X3, n, h, w, t1.shape[-1], 0, cout, 0)
    ws = _ws(lib().rr_wgrad_workspace(C.byref(d)), dy.device)

    def launch():
        lib().check(lib().rr_wgrad_pre(C.byref(d), _p(dy), _p(t1), _p(pre_scale), _p(pre_shift),
                                       _p(pre_alpha), _p(dw), _p(ws), ws.numel(), stream()),
                    "rr_wgrad_pre")
    _launch(lambda: wgrad_kernel_name(d), 2.0 * cout * t1.shape[-1] * 9 * n * h * w, launch,
            f"wgrad m{RR_CONV3X3} {n}x{h}x{w} c{t1.shape[-1]}+0->{cout} pre")
    return dw


def wgrad(mode, dy, x1, x2, n, h, w, cout, dw=None, accumulate=False, dw_shape=None,
          reduce_stream=None):
    """Weight grad (fp32, torch layout) of a conv / convT; see rr_wgrad.

    ``reduce_stream``: the split-K reduce (rr_wgrad_reduce) runs there, after
    the partial launch (rr_wgrad_partial) on the current stream; ``dw`` is
    final once ``reduce_stream`` is joined."""
    _need_cuda(dy, x1)
    c1 = x1.shape[-1]
    c2 = x2.shape[-1] if x2 is not None else 0
    d = WgradDesc(rr_dtype(dy.dtype), mode, n, h, w, c1, c2, cout, int(accumulate))
    if dw is None:
        dw = torch.empty(dw_shape, dtype=torch.float32, device=dy.device)
    need = lib().rr_wgrad_workspace(C.byref(d))
    ws = _ws(need, dy.device)

    def launch():
        # (an A/B build loaded through RR_LIB_PATH may predate the split
        # entry points: the one-launch form then, on the current stream)
        if reduce_stream is None or not hasattr(lib(), "rr_wgrad_partial"):
            lib().check(lib().rr_wgrad(C.byref(d), _p(dy), _p(x1), _p(x2), _p(dw), _p(ws),
                                       ws.numel(), stream()), "rr_wgrad")
            return
        lib().check(lib().rr_wgrad_partial(C.byref(d), _p(dy), _p(x1), _p(x2), _p(ws),
                                           ws.numel(), stream()), "rr_wgrad_partial")
        reduce_stream.wait_stream(torch.cuda.current_stream(dy.device))
        with torch.cuda.stream(reduce_stream):
            lib().check(lib().rr_wgrad_reduce(C.byref(d), _p(ws), ws.numel(), _p(dw),
                                              reduce_stream.cuda_stream), "rr_wgrad_reduce")
        ws.record_stream(reduce_stream)
    taps = 9 if mode == RR_CONV3X3 else (4 if mode == RR_CONVT_UP else 1)
    convT = mode == RR_CONVT_UP
    CA = c1 if convT else cout
    CB = cout if convT else c1 + c2
    _launch(lambda: wgrad_kernel_name(d), 2.0 * CA * CB * taps * n * h * w, launch,
            f"wgrad m{mode} {n}x{h}x{w} c{c1}+{c2}->{cout}")
    return dw


# ---------------------------------------------------------------------------
# batch norm

def bn_finalize(st, count, bias, gamma, beta, running_mean, running_var, momentum=0.1,
                eps=1e-5, num_batches_tracked=None, out=None):
    """``out=(scale, shift)``: caller-provided fp32 [C] outputs (e.g. rows of
    one [2, C] buffer that a later kernel reads as a pair)."""
    blocks, Cc = st.shape[0], st.shape[1]
    dev = st.device
    if st.dtype != torch.float32 or not st.is_contiguous():
        raise ValueError("bn_finalize: st must be a contiguous fp32 [blocks, C, 2] tensor")
    if out is not None:
        scale, shift = out
        for o in (scale, shift):
            if (o.numel() != Cc or not o.is_contiguous() or o.dtype != torch.float32
                    or o.device != dev):
                raise ValueError("bn_finalize: out must be two contiguous fp32 [C] tensors "
                                 "on the device of st")
    else:
        scale = torch.empty(Cc, dtype=torch.float32, device=dev)
        shift = torch.empty(Cc, dtype=torch.float32, device=dev)
    for name, t in (("bias", bias), ("gamma", gamma), ("beta", beta),
                    ("running_mean", running_mean), ("running_var", running_var)):
        if t is not None and (t.dtype != torch.float32 or t.numel() != Cc or t.device != dev
                              or not t.is_contiguous()):
            raise ValueError(f"bn_finalize: {name} must be a contiguous fp32 [C] tensor on the "
                             "device of st")
    if num_batches_tracked is not None and (num_batches_tracked.dtype != torch.int64
                                            or num_batches_tracked.device != dev):
        raise ValueError("bn_finalize: num_batches_tracked must be an int64 tensor on the device")
    _need_cuda(st, scale, shift, bias, gamma, beta, running_mean, running_var, num_batches_tracked)
    mean = torch.empty(Cc, dtype=torch.float32, device=dev)
    inv = torch.empty(Cc, dtype=torch.float32, device=dev)
    ws = _ws(lib().rr_bn_finalize_workspace(Cc, blocks), dev)
    lib().check(lib().rr_bn_finalize(Cc, blocks, int(count), _p(st), _p(bias), _p(gamma), _p(beta),
                                     _p(running_mean), _p(running_var), float(momentum),
                                     float(eps), _p(scale), _p(shift), _p(mean), _p(inv),
                                     _p(num_batches_tracked), _p(ws), ws.numel(), stream()),
                "rr_bn_finalize")
    _bump_running(running_mean, running_var)
    return scale, shift, mean, inv


def _bump_running(*ts):
    """The finalize updated the running statistics through raw pointers: bump
    their version counters so caches keyed on them (the eval-mode conv+BN
    fold, engine.WeightCache.conv_bn_folded) see the update.  Under a HIP-graph
    capture nothing host-side runs on replay; nn._RRNet.train(False) drops the
    folds for that case."""
    ts = [t for t in ts if t is not None]
    inc = getattr(torch.autograd.graph, "increment_version", None)
    if ts and inc is not None and not torch.cuda.is_current_stream_capturing():
        inc(ts)


def bn_finalize_pair(a, b):
    """Two bn_finalize calls (keyword dicts of bn_finalize's arguments) as ONE
    launch (rr_bn_finalize_pair; the residual tail's BN and the shortcut BN).
    Falls back to two launches when either has > 8192 partial rows."""
    from ._lib import BnFinalizeDesc, RR_EUNSUPPORTED
    if a["st"].shape[0] > 8192 or b["st"].shape[0] > 8192:
        return bn_finalize(**a), bn_finalize(**b)
    descs, outs = [], []
    for k in (a, b):
        st = k["st"]
        Cc = st.shape[1]
        dev = st.device
        if st.dtype != torch.float32 or not st.is_contiguous():
            raise ValueError("bn_finalize_pair: st must be a contiguous fp32 [blocks, C, 2] tensor")
        o = k.get("out")
        scale, shift = o if o is not None else (torch.empty(Cc, dtype=torch.float32, device=dev),
                                                torch.empty(Cc, dtype=torch.float32, device=dev))
        mean = torch.empty(Cc, dtype=torch.float32, device=dev)
        inv = torch.empty(Cc, dtype=torch.float32, device=dev)
        for name in ("bias", "gamma", "beta", "running_mean", "running_var"):
            t = k.get(name)
            if t is not None and (t.dtype != torch.float32 or t.numel() != Cc or t.device != dev
                                  or not t.is_contiguous()):
                raise ValueError(f"bn_finalize_pair: {name} must be a contiguous fp32 [C] tensor")
        for t in (scale, shift):
            if t.numel() != Cc or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError("bn_finalize_pair: out must be two contiguous fp32 [C] tensors")
        _need_cuda(st, scale, shift, k.get("bias"), k.get("gamma"), k.get("beta"),
                   k.get("running_mean"), k.get("running_var"), k.get("num_batches_tracked"))
        descs.append(BnFinalizeDesc(Cc, st.shape[0], int(k["count"]), _p(st), _p(k.get("bias")),
                                    _p(k.get("gamma")), _p(k.get("beta")),
                                    _p(k.get("running_mean")), _p(k.get("running_var")),
                                    float(k.get("momentum", 0.1)), float(k.get("eps", 1e-5)),
                                    _p(scale), _p(shift), _p(mean), _p(inv),
                                    _p(k.get("num_batches_tracked"))))
        outs.append((scale, shift, mean, inv))
    rc = lib().rr_bn_finalize_pair(C.byref(descs[0]), C.byref(descs[1]), stream())
    if rc == RR_EUNSUPPORTED:
        return bn_finalize(**a), bn_finalize(**b)
    lib().check(rc, "rr_bn_finalize_pair")
    for k in (a, b):
        _bump_running(k.get("running_mean"), k.get("running_var"))
    return outs[0], outs[1]


def bn_eval_affine(gamma, beta, running_mean, running_var, eps=1e-5, out=None):
    """Eval-mode BN as scale / shift from the running statistics (gamma /
    beta None: 1 / 0, so scale = invstd); ``out=(scale, shift)``: fp32 [C]
    outputs to write."""
    Cc = running_mean.numel()
    if out is not None:
        scale, shift = out
    else:
        scale = torch.empty(Cc, dtype=torch.float32, device=running_mean.device)
        shift = torch.empty_like(scale)
    lib().check(lib().rr_bn_eval_affine(Cc, _p(gamma), _p(beta), _p(running_mean),
                                        _p(running_var), float(eps), _p(scale), _p(shift),
                                        stream()), "rr_bn_eval_affine")
    return scale, shift


def fold_conv_bn(w, b, scale, shift):
    """eval BN folded into the conv: (w * scale[c], b * scale + shift), fp32"""
    _need_cuda(w, scale, shift)
    co = w.shape[0]
    w = w.contiguous()
    wf = torch.empty_like(w)
    bf = torch.empty(co, dtype=torch.float32, device=w.device)
    lib().check(lib().rr_fold_conv_bn(co, w.numel() // co, _p(w), _p(b), _p(scale), _p(shift),
                                      _p(wf), _p(bf), stream()), "rr_fold_conv_bn")
    return wf, bf


def affine_act(x, scale, shift, alpha=None, res=None, res_scale=None, res_shift=None, relu=False,
               out=None):
    _need_cuda(x)
    Cc = x.shape[-1]
    P = x.numel() // Cc
    if out is None:
        out = torch.empty_like(x)
    lib().check(lib().rr_affine_act(rr_dtype(x.dtype), P, Cc, _p(x), _p(scale), _p(shift),
                                    _p(alpha), _p(res), _p(res_scale), _p(res_shift), int(relu),
                                    _p(out), stream()), "rr_affine_act")
    return out


def affine_act_pool(x, scale, shift, res=None, res_scale=None, res_shift=None, relu=True):
    """Residual tail fused with MaxPool2d(2, 2): -> (y, y_pool, idx)."""
    _need_cuda(x)
    n, h, w, Cc = x.shape
    y = torch.empty_like(x)
    yp = torch.empty((n, h // 2, w // 2, Cc), dtype=x.dtype, device=x.device)
    idx = torch.empty((n, h // 2, w // 2, Cc), dtype=torch.uint8, device=x.device)
    lib().check(lib().rr_affine_act_pool(rr_dtype(x.dtype), n, h, w, Cc, _p(x), _p(scale), _p(shift),
                                         _p(res), _p(res_scale), _p(res_shift), int(relu), _p(y),
                                         _p(yp), _p(idx), stream()), "rr_affine_act_pool")
    return y, yp, idx


# A/B switch: the identity-shortcut tail's BN backward stores gm in its
# reduce and applies from it (rr_bn_bwd_reduce_gm); 0: gm from the apply
_BN_GM_IN_REDUCE = path_flag("bn_gm_in_reduce", 1) != 0


def bn_backward(g, t0, mean0, inv0, gamma0, *, mask_kind=0, aux=None, aff_s=None, aff_b=None,
                alpha=None, t1=None, mean1=None, inv1=None, gamma1=None, want_gm=False,
                gm_out=None, outs=None, pool=None, recompute=None, eval_mode=False, dbias=None):
    """Full BN backward (reduce + finalize + apply) for one or two BNs that
    share the upstream gradient.  Returns dict with dt0, dt1, gm, dgamma0,
    dbeta0, dgamma1, dbeta1, dalpha.  ``pool=(dy_pool, idx)`` with
    mask_kind 1: the 2x2 max-pool backward is added to g before the ReLU mask
    (mask kind 3, g: [n, h, w, C]).  ``recompute=(aff_s2, aff_b2)`` with
    mask_kind 1 and two BNs: the ReLU mask is recomputed from t0, t1 with the
    forward affines ([2, C] each: BN0's then BN1's scale / shift) instead of
    read from ``aux`` (mask kind 4, or 5 with ``pool``).  ``eval_mode``:
    eval-mode BatchNorm (mean / inv = running statistics; no batch-statistic
    terms); ``dbias=(db0, db1)`` then receive the grads of the conv biases
    feeding the BNs."""
    Cc = g.shape[-1]
    P = g.numel() // Cc
    nbn = 2 if t1 is not None else 1
    dev = g.device
    d = BnBwdDesc(rr_dtype(g.dtype), P, Cc, mask_kind, nbn, 0, 0, None, None)
    _set_eval(d, eval_mode, dbias)
    if recompute is not None:
        if mask_kind != 1 or nbn != 2 or want_gm or gm_out is not None:
            raise ValueError("recomputed ReLU mask needs mask_kind 1, two BNs and no gm output")
        aff_s, aff_b = (x.contiguous() for x in recompute)
        aux = None
        d.mask_kind = 4
    if pool is not None:
        if mask_kind != 1 or g.dim() != 4:
            raise ValueError("pool backward fusion needs the ReLU mask and an [n, h, w, C] grad")
        pdy, pidx = pool
        d.mask_kind, d.h, d.w = 5 if recompute is not None else 3, g.shape[1], g.shape[2]
        d.pool_dy, d.pool_idx = _p(pdy.contiguous()), _p(pidx)
    blocks = lib().rr_bn_bwd_blocks(C.byref(d))
    part = torch.empty(blocks * Cc * 3 + blocks, dtype=torch.float32, device=dev)
    s = stream()
    # the identity-shortcut tail (gm is the block's input grad): the reduce
    # stores gm and the apply reads it alone (rr_bn_bwd_reduce_gm)
    gm_first = (_BN_GM_IN_REDUCE and (want_gm or gm_out is not None) and nbn == 1 and
                d.mask_kind in (1, 3) and Cc % 8 == 0 and 256 % (Cc // 8) == 0 and
                hasattr(lib(), "rr_bn_bwd_reduce_gm"))      # (absent from older A/B builds)
    if gm_first:
        if gm_out is None:
            gm_out = torch.empty_like(g)
        lib().check(lib().rr_bn_bwd_reduce_gm(C.byref(d), _p(g), _p(aux), _p(t0), _p(mean0),
                                              _p(inv0), _p(part), _p(gm_out), s),
                    "rr_bn_bwd_reduce_gm")
    else:
        lib().check(lib().rr_bn_bwd_reduce(C.byref(d), _p(g), _p(aux), _p(aff_s), _p(aff_b),
                                           _p(alpha), _p(t0), _p(mean0), _p(inv0), _p(t1),
                                           _p(mean1), _p(inv1), _p(part), s), "rr_bn_bwd_reduce")
    o = outs or {}
    dg0 = o.get("dgamma0")
    if dg0 is None:
        dg0 = torch.empty(Cc, dtype=torch.float32, device=dev)
    db0 = o.get("dbeta0")
    if db0 is None:
        db0 = torch.empty_like(dg0)
    dg1 = o.get("dgamma1")
    if dg1 is None and nbn == 2:
        dg1 = torch.empty_like(dg0)
    db1 = o.get("dbeta1")
    if db1 is None and nbn == 2:
        db1 = torch.empty_like(dg0)
    dal = o.get("dalpha")
    if dal is None and mask_kind == 2:
        dal = torch.empty(1, dtype=torch.float32, device=dev)
    coef = torch.empty(Cc * 6, dtype=torch.float32, device=dev)
    lib().check(lib().rr_bn_bwd_finalize(C.byref(d), _p(part), _p(gamma0), _p(inv0), _p(gamma1),
                                         _p(inv1), _p(dg0), _p(db0), _p(dg1), _p(db1), _p(dal),
                                         _p(coef), s), "rr_bn_bwd_finalize")
    dt0 = torch.empty_like(g)
    dt1 = torch.empty_like(g) if nbn == 2 else None
    if gm_first:
        da = BnBwdDesc(d.dtype, P, Cc, 0, 1, 0, 0, None, None)
        _set_eval(da, eval_mode, dbias)
        lib().check(lib().rr_bn_bwd_apply(C.byref(da), _p(gm_out), None, None, None, None,
                                          _p(t0), _p(mean0), _p(inv0), None, None, None,
                                          _p(coef), _p(dt0), None, None, s), "rr_bn_bwd_apply")
        return dict(dt0=dt0, dt1=None, gm=gm_out, dgamma0=dg0, dbeta0=db0, dgamma1=dg1,
                    dbeta1=db1, dalpha=dal)
    if want_gm and gm_out is None:
        gm_out = torch.empty_like(g)
    lib().check(lib().rr_bn_bwd_apply(C.byref(d), _p(g), _p(aux), _p(aff_s), _p(aff_b), _p(alpha),
                                      _p(t0), _p(mean0), _p(inv0), _p(t1), _p(mean1), _p(inv1),
                                      _p(coef), _p(dt0), _p(dt1), _p(gm_out), s),
                "rr_bn_bwd_apply")
    return dict(dt0=dt0, dt1=dt1, gm=gm_out, dgamma0=dg0, dbeta0=db0, dgamma1=dg1, dbeta1=db1,
                dalpha=dal)


def igemm_bnbwd(mode, dy, n, h, w, wpack, cout, t, mean, inv, aff_s, aff_b, alpha, out=None):
    """Conv dgrad fused with the BN -> PReLU backward reduce (rr_igemm_bnbwd).
    Returns (gm, partial, rows, arows): gm = dL/d(BN out) [n, h, w, cout] and
    the row partials for ``bn_backward_rows``."""
    _need_cuda(dy, wpack, t)
    dt = dy.dtype
    d = IgemmDesc(rr_dtype(dt), mode, n, h, w, dy.shape[-1], 0, cout, 0, 0, 0, 0, 0, 0, 0)
    if out is None:
        out = torch.empty((n, h, w, cout), dtype=dt, device=dy.device)
    rows = lib().rr_igemm_stat_blocks(C.byref(d))
    nbytes = lib().rr_igemm_bnbwd_workspace(C.byref(d))
    part = torch.empty(nbytes // 4, dtype=torch.float32, device=dy.device)

    def launch():
        lib().check(lib().rr_igemm_bnbwd(C.byref(d), _p(dy), _p(wpack), _p(t), _p(mean), _p(inv),
                                         _p(aff_s), _p(aff_b), _p(alpha), _p(out), _p(part),
                                         stream()), "rr_igemm_bnbwd")
    taps = 9 if mode == RR_CONV3X3 else 1
    _launch(lambda: igemm_kernel_name(d, bnbwd=True), 2.0 * n * h * w * cout * taps * dy.shape[-1],
            launch, f"bnbwd m{mode} {n}x{h}x{w} c{dy.shape[-1]}->{cout}")
    return out, part, rows, rows * (cout // 64)


def _set_eval(d, eval_mode, dbias):
    d.eval = int(bool(eval_mode))
    if eval_mode and dbias is not None:
        for i, t in enumerate(dbias[:2]):
            if t is not None:
                if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != d.C:
                    raise ValueError("dbias: contiguous fp32 [C] tensors")
                setattr(d, f"dbias{i}", _p(t))


def bn_backward_rows(gm, part, rows, arows, t0, mean0, inv0, gamma0, outs=None, eval_mode=False,
                     dbias=None):
    """BN backward from precomputed row partials (the rr_igemm_bnbwd epilogue):
    finalize (fp64 fixed order) + apply with gm already PReLU-masked
    (``eval_mode`` / ``dbias``: as bn_backward)."""
    Cc = gm.shape[-1]
    P = gm.numel() // Cc
    dev = gm.device
    d = BnBwdDesc(rr_dtype(gm.dtype), P, Cc, 0, 1)
    _set_eval(d, eval_mode, dbias)
    o = outs or {}
    dg0 = o.get("dgamma0")
    if dg0 is None:
        dg0 = torch.empty(Cc, dtype=torch.float32, device=dev)
    db0 = o.get("dbeta0")
    if db0 is None:
        db0 = torch.empty_like(dg0)
    dal = o.get("dalpha")
    if dal is None:
        dal = torch.empty(1, dtype=torch.float32, device=dev)
    coef = torch.empty(Cc * 6, dtype=torch.float32, device=dev)
    ws = _ws(lib().rr_bn_bwd_finalize_rows_workspace(Cc, rows), dev)
    apart = part[rows * Cc * 3:]
    s = stream()
    lib().check(lib().rr_bn_bwd_finalize_rows(C.byref(d), rows, _p(part), arows, _p(apart),
                                              _p(gamma0), _p(inv0), _p(dg0), _p(db0), _p(dal),
                                              _p(coef), _p(ws), ws.numel(), s),
                "rr_bn_bwd_finalize_rows")
    dt0 = torch.empty_like(gm)
    lib().check(lib().rr_bn_bwd_apply(C.byref(d), _p(gm), None, None, None, None, _p(t0), _p(mean0),
                                      _p(inv0), None, None, None, _p(coef), _p(dt0), None, None, s),
                "rr_bn_bwd_apply")
    return dict(dt0=dt0, dgamma0=dg0, dbeta0=db0, dalpha=dal)


def channel_sum(x, out=None, accumulate=False):
    Cc = x.shape[-1]
    P = x.numel() // Cc
    if out is None:
        out = torch.empty(Cc, dtype=torch.float32, device=x.device)
    ws = _ws(lib().rr_channel_sum_workspace(P, Cc), x.device)
    lib().check(lib().rr_channel_sum(rr_dtype(x.dtype), P, Cc, _p(x), _p(out), int(accumulate),
                                     _p(ws), ws.numel(), stream()), "rr_channel_sum")
    return out


def bn_stats(x):
    """(sum, sum of squares) partials [blocks, C, 2] of an NHWC tensor, for
    ``bn_finalize(st, count=P, ...)`` (a standalone BatchNorm2d)."""
    _need_cuda(x)
    Cc = x.shape[-1]
    P = x.numel() // Cc
    st = torch.empty((lib().rr_bn_stats_blocks(P), Cc, 2), dtype=torch.float32, device=x.device)
    lib().check(lib().rr_bn_stats(rr_dtype(x.dtype), P, Cc, _p(x), _p(st), stream()), "rr_bn_stats")
    return st


# ---------------------------------------------------------------------------
# pooling, first / last layers, layout

def maxpool2_fwd(x):
    n, h, w, Cc = x.shape
    y = torch.empty((n, h // 2, w // 2, Cc), dtype=x.dtype, device=x.device)
    idx = torch.empty((n, h // 2, w // 2, Cc), dtype=torch.uint8, device=x.device)
    lib().check(lib().rr_maxpool2_fwd(rr_dtype(x.dtype), n, h, w, Cc, _p(x), _p(y), _p(idx),
                                      stream()), "rr_maxpool2_fwd")
    return y, idx


def maxpool2_bwd_pooled(dy, idx, y_pool, h, w):
    """MaxPool2d(2, 2) backward through the ReLU before it, the mask taken
    from the pooled forward output (rr_maxpool2_bwd_pooled; bitwise
    maxpool2_bwd with mask = the full-size ReLU output)."""
    n, _, _, Cc = dy.shape
    out = torch.empty((n, h, w, Cc), dtype=dy.dtype, device=dy.device)
    lib().check(lib().rr_maxpool2_bwd_pooled(rr_dtype(dy.dtype), n, h, w, Cc, _p(dy), _p(idx),
                                             _p(y_pool), _p(out), stream()),
                "rr_maxpool2_bwd_pooled")
    return out


def igemm_pool_desc(x1, n, h, w, cout, has_bias):
    return IgemmDesc(rr_dtype(x1.dtype), RR_CONV3X3, n, h, w, x1.shape[-1], 0, cout, 0, 1, 0,
                     int(has_bias), 0, 0, 0)


def igemm_pool_kernel_name(d):
    """The kernel rr_igemm_pool launches for ``d`` ("unsupported": none, or
    an older build loaded for an A/B that lacks the entry point)."""
    fn = getattr(lib(), "rr_igemm_pool_kernel_name", None)
    return fn(C.byref(d)).decode() if fn is not None else "unsupported"


def igemm_pool(x1, n, h, w, wpack, cout, bias=None, want_idx=True):
    """conv3x3 (+ bias) + ReLU + MaxPool2d(2, 2) in one pass (rr_igemm_pool):
    -> (pooled [n, h/2, w/2, cout], first-max index or None); the full-size
    output is never written."""
    _need_cuda(x1, wpack)
    d = igemm_pool_desc(x1, n, h, w, cout, bias is not None)
    yp = torch.empty((n, h // 2, w // 2, cout), dtype=x1.dtype, device=x1.device)
    idx = torch.empty((n, h // 2, w // 2, cout), dtype=torch.uint8, device=x1.device) \
        if want_idx else None

    def launch():
        lib().check(lib().rr_igemm_pool(C.byref(d), _p(x1), None, _p(wpack), _p(bias), _p(yp),
                                        _p(idx), stream()), "rr_igemm_pool")
    _launch(lambda: igemm_pool_kernel_name(d), 2.0 * n * h * w * cout * 9 * x1.shape[-1], launch,
            f"fwd m{RR_CONV3X3} {n}x{h}x{w} c{x1.shape[-1]}+0->{cout} pool")
    return yp, idx


def igemm_dgrad_sc_kernel_name(d, c_sc):
    f = getattr(lib(), "rr_igemm_dgrad_sc_kernel_name", None)    # (older builds: A/B runs)
    return f(C.byref(d), c_sc).decode() if f is not None else "unsupported"


def dgrad_sc_desc(dy, n, h, w, cout):
    return IgemmDesc(rr_dtype(dy.dtype), RR_CONV3X3, n, h, w, dy.shape[-1], 0, cout, 0, 0, 0, 0, 0,
                     0, 0)


def igemm_dgrad_sc(dy, n, h, w, wpack, cout, dy_sc, wpack_sc):
    """the 3x3 dgrad of ``dy`` + the 1x1 dgrad of ``dy_sc`` (rows ``wpack_sc``
    of the 1x1 dgrad pack) into one [n, h, w, cout] output, one pass
    (rr_igemm_dgrad_sc); None where the library does not take the shape."""
    _need_cuda(dy, wpack, dy_sc, wpack_sc)
    d = dgrad_sc_desc(dy, n, h, w, cout)
    c_sc = dy_sc.shape[-1]
    if igemm_dgrad_sc_kernel_name(d, c_sc) == "unsupported":
        return None
    y = torch.empty((n, h, w, cout), dtype=dy.dtype, device=dy.device)

    def launch():
        lib().check(lib().rr_igemm_dgrad_sc(C.byref(d), _p(dy), _p(wpack), _p(dy_sc), _p(wpack_sc),
                                            c_sc, _p(y), stream()), "rr_igemm_dgrad_sc")
    _launch(lambda: igemm_dgrad_sc_kernel_name(d, c_sc),
            2.0 * n * h * w * cout * (9 * dy.shape[-1] + c_sc), launch,
            f"fwd m{RR_CONV3X3} {n}x{h}x{w} c{dy.shape[-1]}+0->{cout} sc{c_sc}")
    return y


def nearest_resize(x, ho, wo):
    """F.interpolate(x, size=(ho, wo)) mode 'nearest' (14:169-182), NHWC."""
    _need_cuda(x)
    n, hi, wi, Cc = x.shape
    y = torch.empty((n, ho, wo, Cc), dtype=x.dtype, device=x.device)
    lib().check(lib().rr_nearest_resize(rr_dtype(x.dtype), n, hi, wi, ho, wo, Cc, _p(x.contiguous()),
                                        _p(y), stream()), "rr_nearest_resize")
    return y


def nearest_resize_bwd(dy, hi, wi):
    """gradient of nearest_resize w.r.t. its [n, hi, wi, C] input"""
    _need_cuda(dy)
    n, ho, wo, Cc = dy.shape
    dx = torch.empty((n, hi, wi, Cc), dtype=dy.dtype, device=dy.device)
    lib().check(lib().rr_nearest_resize_bwd(rr_dtype(dy.dtype), n, hi, wi, ho, wo, Cc,
                                            _p(dy.contiguous()), _p(dx), stream()),
                "rr_nearest_resize_bwd")
    return dx


def maxpool2_bwd(dy, idx, h, w, out=None, accumulate=False, mask=None):
    n, _, _, Cc = dy.shape
    if out is None:
        out = torch.empty((n, h, w, Cc), dtype=dy.dtype, device=dy.device)
    lib().check(lib().rr_maxpool2_bwd(rr_dtype(dy.dtype), n, h, w, Cc, _p(dy), _p(idx), _p(out),
                                      int(accumulate), _p(mask), stream()), "rr_maxpool2_bwd")
    return out


KPAD_IN = 64      # K of the first-layer GEMM: 27 taps x channels + bias column, padded


def im2col3(x_nchw, dtype, kpad=KPAD_IN):
    n, cin, h, w = x_nchw.shape
    col = torch.empty((n, h, w, kpad), dtype=dtype, device=x_nchw.device)
    lib().check(lib().rr_im2col3(rr_dtype(dtype), n, h, w, cin, kpad, _p(x_nchw.contiguous()),
                                 _p(col), stream()), "rr_im2col3")
    return col


def pack_conv_in(wt, b, dtype, kpad=None):
    if kpad is None:
        kpad = conv_in_kpad(dtype, wt.shape[1], wt.shape[0])
    cout, cin = wt.shape[0], wt.shape[1]
    out = torch.empty(cout * kpad, dtype=dtype, device=wt.device)
    lib().check(lib().rr_pack_conv_in(rr_dtype(dtype), cout, cin, kpad, _p(wt.contiguous()), _p(b),
                                      _p(out), stream()), "rr_pack_conv_in")
    return out


KPAD_MFMA = 32    # K of the fused bf16 first conv (rr_conv_in_mfma): 27 taps + bias + pad


def conv_in_kpad(dtype, cin=3, cout=64):
    """K padding of the packed first-layer weights for ``first_conv_fwd``."""
    return KPAD_MFMA if (dtype == torch.bfloat16 and cin == 3 and cout == 64) else KPAD_IN


def first_conv_fwd(x_nchw, wt, b, dtype, wpack, act=0, alpha=None, want_pre=False):
    """First 3x3 conv (cin = 3), bias folded into the GEMM (07:78, 14:124,
    VGG16 features[0]).  act: 0 none, 1 ReLU, 2 PReLU(alpha).
    Returns (y, pre): y the activated NHWC output, pre the pre-activation
    (only when want_pre, else None).

    bf16 (3 -> 64): one fused launch (rr_conv_in_mfma: im2col in registers,
    K = 32 MFMA), pack with kpad 32.  fp32 (parity path): im2col + K = 64
    implicit GEMM (+ the activation pass)."""
    n, cin, h, w = x_nchw.shape
    cout = wt.shape[0]
    x_nchw = x_nchw.contiguous()
    if conv_in_kpad(dtype, cin, cout) == KPAD_MFMA:
        y = torch.empty((n, h, w, cout), dtype=dtype, device=x_nchw.device)
        pre = torch.empty_like(y) if (want_pre and act) else None
        lib().check(lib().rr_conv_in_mfma(n, h, w, _p(x_nchw), _p(wpack), act, _p(alpha),
                                          _p(pre), _p(y), stream()), "rr_conv_in_mfma")
        return y, (pre if act else (y if want_pre else None))
    col = im2col3(x_nchw, dtype)
    if act == 2:
        pre, _, _ = igemm(RR_CONV1X1, col, None, n, h, w, wpack, cout)
        one = torch.ones(cout, dtype=torch.float32, device=x_nchw.device)
        y = affine_act(pre, one, torch.zeros_like(one), alpha=alpha)
        return y, (pre if want_pre else None)
    if act == 1 and want_pre:
        pre, _, _ = igemm(RR_CONV1X1, col, None, n, h, w, wpack, cout)
        one = torch.ones(cout, dtype=torch.float32, device=x_nchw.device)
        y = affine_act(pre, one, torch.zeros_like(one), relu=True)
        return y, pre
    y, _, _ = igemm(RR_CONV1X1, col, None, n, h, w, wpack, cout, act=act)
    return y, (y if (want_pre and not act) else None)


def first_conv_wgrad(col, dy, dw, db):
    """Weight + bias grad of the first conv from its im2col matrix."""
    n, h, w, kpad = col.shape
    cout = dy.shape[-1]
    cin = dw.shape[1]
    g = wgrad(RR_CONV1X1, dy, col, None, n, h, w, cout, dw_shape=(cout, kpad, 1, 1))
    lib().check(lib().rr_unpack_conv_in_grad(cout, cin, kpad, _p(g), _p(dw), _p(db), stream()),
                "rr_unpack_conv_in_grad")
    return dw, db


def first_conv_wgrad_act(x_nchw, dy, t_pre, act, alpha, dw, db, dalpha=None):
    """First-conv weight/bias grad fused with its ReLU (act 1) / PReLU (act
    2) backward, from the NCHW fp32 image (rr_conv_in_wgrad_act)."""
    _need_cuda(x_nchw, dy, t_pre)
    n, cin, h, w = x_nchw.shape
    if cin != 3 or dy.shape[-1] != 64 or dy.dtype != torch.bfloat16 or t_pre.dtype != torch.bfloat16:
        raise ValueError("rr_conv_in_wgrad_act: 3 -> 64 channels, bf16 grads")
    L = lib()
    wsb = L.rr_conv_in_wgrad_act_workspace(n, h, w)
    ws = _ws(wsb, dy.device)
    L.check(L.rr_conv_in_wgrad_act(n, h, w, _p(x_nchw.contiguous()), _p(dy), _p(t_pre), int(act),
                                   _p(alpha), _p(dw), _p(db), _p(dalpha), _p(ws), wsb, stream()),
            "rr_conv_in_wgrad_act")
    return dw, db


def conv_in_fwd(x_nchw, wt, b, dtype, act=0, alpha=None):
    n, cin, h, w = x_nchw.shape
    cout = wt.shape[0]
    y = torch.empty((n, h, w, cout), dtype=dtype, device=x_nchw.device)
    lib().check(lib().rr_conv_in_fwd(rr_dtype(dtype), n, h, w, cin, cout, _p(x_nchw), _p(wt),
                                     _p(b), act, _p(alpha), _p(y), stream()), "rr_conv_in_fwd")
    return y


def conv_in_wgrad(x_nchw, dy, dw_shape=None, dw=None, db=None):
    n, cin, h, w = x_nchw.shape
    cout = dy.shape[-1]
    if dw is None:
        dw = torch.empty(dw_shape, dtype=torch.float32, device=dy.device)
    if db is None:
        db = torch.empty(cout, dtype=torch.float32, device=dy.device)
    ws = _ws(lib().rr_conv_in_wgrad_workspace(n, h, w, cin, cout), dy.device)
    lib().check(lib().rr_conv_in_wgrad(rr_dtype(dy.dtype), n, h, w, cin, cout, _p(x_nchw), _p(dy),
                                       _p(dw), _p(db), _p(ws), ws.numel(), stream()),
                "rr_conv_in_wgrad")
    return dw, db


def conv_in_dgrad(dy, wt, cin, out=None, accumulate=False, wpack_dgrad=None):
    """Image grad of the first 3x3 conv (cin = 3): an implicit GEMM with K =
    9*cout and cin GEMM columns, written straight into NCHW fp32.  Without
    a packed dgrad weight it uses the VALU kernel rr_conv_in_dgrad."""
    n, h, w, cout = dy.shape
    if wpack_dgrad is not None and cout % 64 == 0:
        y, _, _ = igemm(RR_CONV3X3, dy, None, n, h, w, wpack_dgrad, cin, out=out,
                        accumulate=accumulate, out_nchw=True)
        return y
    if out is None:
        out = torch.empty((n, cin, h, w), dtype=torch.float32, device=dy.device)
    lib().check(lib().rr_conv_in_dgrad(rr_dtype(dy.dtype), n, h, w, cin, cout, _p(dy), _p(wt),
                                       _p(out), int(accumulate), stream()), "rr_conv_in_dgrad")
    return out


def prelu_bwd(dy, y_pre, alpha, dalpha=None):
    count = dy.numel()
    blocks = max(1, min(1024, (count + 4095) // 4096))
    dx = torch.empty_like(dy)
    part = torch.empty(blocks, dtype=torch.float32, device=dy.device)
    if dalpha is None:
        dalpha = torch.empty(1, dtype=torch.float32, device=dy.device)
    lib().check(lib().rr_prelu_bwd(rr_dtype(dy.dtype), count, _p(dy), _p(y_pre), _p(alpha),
                                   _p(dx), _p(part), blocks, _p(dalpha), stream()),
                "rr_prelu_bwd")
    return dx, dalpha


def conv_out_fwd(x, wt, b, wpack=None):
    """Final 1x1 conv cin -> cout (3) into NCHW fp32: implicit GEMM with the
    NCHW epilogue when a packed weight is given, else the VALU kernel."""
    n, h, w, cin = x.shape
    cout = wt.shape[0]
    if wpack is not None and cin % 64 == 0:
        y, _, _ = igemm(RR_CONV1X1, x, None, n, h, w, wpack, cout, bias=b, out_nchw=True)
        return y
    y = torch.empty((n, cout, h, w), dtype=torch.float32, device=x.device)
    lib().check(lib().rr_conv_out_fwd(rr_dtype(x.dtype), n, h, w, cin, cout, _p(x),
                                      _p(wt.reshape(cout, cin)), _p(b), _p(y), stream()),
                "rr_conv_out_fwd")
    return y


def conv_out_bwd(dy_nchw, x, wt, mask_relu=False, want_dx=True, dw=None, db=None):
    n, h, w, cin = x.shape
    cout = wt.shape[0]
    dx = torch.empty_like(x) if want_dx else None
    if dw is None:
        dw = torch.empty(wt.shape, dtype=torch.float32, device=x.device)
    if db is None:
        db = torch.empty(cout, dtype=torch.float32, device=x.device)
    ws = _ws(lib().rr_conv_out_bwd_workspace(n, h, w, cin, cout), x.device)
    lib().check(lib().rr_conv_out_bwd(rr_dtype(x.dtype), n, h, w, cin, cout,
                                      _p(dy_nchw.contiguous()), _p(x), _p(wt.reshape(cout, cin)),
                                      _p(dx), int(mask_relu), _p(dw), _p(db), _p(ws), ws.numel(),
                                      stream()), "rr_conv_out_bwd")
    return dx, dw, db


def bn_backward_convout(dy_nchw, x, wt, t0, mean0, inv0, gamma0, t1, mean1, inv1, gamma1,
                        recompute, outs, dw, db):
    """The residual-tail BN backward (two BNs, recomputed ReLU mask: as
    ``bn_backward(g, ..., mask_kind=1, recompute=...)``) of the block whose
    output ``x`` feeds the final 1x1 conv, with g = that conv's input grad
    never materialised: rr_conv_out_bwd_bnred (the conv's dw / db + the BN
    reduce), rr_bn_bwd_finalize, rr_bn_bwd_apply_convout (g recomputed from
    ``dy_nchw``).  Train mode only.  Returns dict(dt0, dt1); None where the
    library does not take the shape (the caller runs conv_out_bwd +
    bn_backward)."""
    n, h, w, Cc = x.shape
    cout = wt.shape[0]
    if Cc != 64 or cout != 3 or not hasattr(lib(), "rr_conv_out_bwd_bnred"):
        return None
    P = n * h * w
    dev = x.device
    d = BnBwdDesc(rr_dtype(x.dtype), P, Cc, 4, 2, 0, 0, None, None)
    blocks = lib().rr_bn_bwd_blocks(C.byref(d))
    part = torch.empty(blocks * Cc * 3 + blocks, dtype=torch.float32, device=dev)
    ws = _ws(lib().rr_conv_out_bwd_bnred_workspace(P, Cc, cout), dev)
    dy = dy_nchw.contiguous()
    w2 = wt.reshape(cout, Cc)
    s = stream()
    lib().check(lib().rr_conv_out_bwd_bnred(C.byref(d), n, h, w, cout, _p(dy), _p(x), _p(w2), _p(t0),
                                            _p(mean0), _p(inv0), _p(t1), _p(mean1), _p(inv1), _p(dw),
                                            _p(db), _p(part), _p(ws), ws.numel(), s),
                "rr_conv_out_bwd_bnred")
    coef = torch.empty(Cc * 6, dtype=torch.float32, device=dev)
    lib().check(lib().rr_bn_bwd_finalize(C.byref(d), _p(part), _p(gamma0), _p(inv0), _p(gamma1),
                                         _p(inv1), _p(outs["dgamma0"]), _p(outs["dbeta0"]),
                                         _p(outs["dgamma1"]), _p(outs["dbeta1"]), None, _p(coef), s),
                "rr_bn_bwd_finalize")
    aff_s, aff_b = (q.contiguous() for q in recompute)
    dt0 = torch.empty_like(x)
    dt1 = torch.empty_like(x)
    lib().check(lib().rr_bn_bwd_apply_convout(C.byref(d), h, w, _p(dy), _p(w2), cout, _p(aff_s),
                                              _p(aff_b), _p(t0), _p(mean0), _p(inv0), _p(t1),
                                              _p(mean1), _p(inv1), _p(coef), _p(dt0), _p(dt1), s),
                "rr_bn_bwd_apply_convout")
    return dict(dt0=dt0, dt1=dt1)


def nchw_to_nhwc(x, dtype):
    n, c, h, w = x.shape
    y = torch.empty((n, h, w, c), dtype=dtype, device=x.device)
    lib().check(lib().rr_nchw_to_nhwc(rr_dtype(dtype), n, c, h, w, _p(x.contiguous()), _p(y),
                                      stream()), "rr_nchw_to_nhwc")
    return y


def nhwc_to_nchw(x):
    n, h, w, c = x.shape
    y = torch.empty((n, c, h, w), dtype=torch.float32, device=x.device)
    lib().check(lib().rr_nhwc_to_nchw(rr_dtype(x.dtype), n, c, h, w, _p(x), _p(y), stream()),
                "rr_nhwc_to_nchw")
    return y


# ---------------------------------------------------------------------------
# losses / optimiser / post-processing

L1, MSE = 0, 1


def loss_fwd(kind, a, b, scale=1.0, out=None, accumulate=False):
    count = a.numel()
    if out is None:
        out = torch.empty((), dtype=torch.float32, device=a.device)
    ws = _ws(lib().rr_loss_workspace(count), a.device)
    lib().check(lib().rr_loss_fwd(kind, rr_dtype(a.dtype), count, _p(a), _p(b), _p(out),
                                  float(scale), int(accumulate), _p(ws), ws.numel(), stream()),
                "rr_loss_fwd")
    return out


def loss_bwd(kind, a, b, gscale=None, scale=1.0, ga=None, accumulate=False, mask_a_pos=False):
    if ga is None:
        ga = torch.empty_like(a)
    lib().check(lib().rr_loss_bwd(kind, rr_dtype(a.dtype), a.numel(), _p(a), _p(b), _p(gscale),
                                  float(scale), _p(ga), None, int(accumulate), int(mask_a_pos),
                                  stream()), "rr_loss_bwd")
    return ga


def adamw_(param, grad, m, v, lr, beta1, beta2, eps, weight_decay, decoupled, step):
    lib().check(lib().rr_adamw(param.numel(), _p(param), _p(grad), _p(m), _p(v), float(lr),
                               float(beta1), float(beta2), float(eps), float(weight_decay),
                               int(decoupled), int(step), stream()), "rr_adamw")


def to_uint8_hwc(x_nchw, bgr=False):
    n, c, h, w = x_nchw.shape
    out = torch.empty((n, h, w, c), dtype=torch.uint8, device=x_nchw.device)
    lib().check(lib().rr_to_uint8_hwc(n, c, h, w, _p(x_nchw.contiguous()), _p(out), int(bgr),
                                      stream()), "rr_to_uint8_hwc")
    return out


def psnr_u8(a, b):
    n = a.shape[0]
    per = a.numel() // n
    out = torch.empty(n, dtype=torch.float64, device=a.device)
    lib().check(lib().rr_psnr_u8(n, per, _p(a.contiguous()), _p(b.contiguous()), _p(out),
                                 stream()), "rr_psnr_u8")
    return out


def argmax_rows(logits):
    n, k = logits.shape
    out = torch.empty(n, dtype=torch.int64, device=logits.device)
    lib().check(lib().rr_argmax_rows(n, k, _p(logits.contiguous()), _p(out), stream()),
                "rr_argmax_rows")
    return out


def adaptive_avgpool_flatten(x, oh=7, ow=7):
    n, h, w, Cc = x.shape
    y = torch.empty((n, Cc * oh * ow), dtype=x.dtype, device=x.device)
    lib().check(lib().rr_adaptive_avgpool_flatten(rr_dtype(x.dtype), n, h, w, Cc, oh, ow, _p(x),
                                                  _p(y), stream()), "rr_adaptive_avgpool_flatten")
    return y


def resize_bilinear_u8(x, oh, ow, out="u8", mean=None, std=None):
    """PIL-exact bilinear resize of a [n, h, w, c] uint8 batch (torchvision
    Resize((oh, ow)) on PIL images, 17:66 / 18:28-32).  out="u8": [n, oh, ow,
    c] uint8; out="f32": [n, c, oh, ow] fp32 ToTensor (+ Normalize(mean, std))."""
    _need_cuda(x)
    if x.dtype != torch.uint8 or x.dim() != 4:
        raise TypeError("resize_bilinear_u8 expects a [n, h, w, c] uint8 tensor")
    n, h, w, c = x.shape
    x = x.contiguous()
    if out == "u8":
        y = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
        kind = 0
    elif out == "f32":
        y = torch.empty((n, c, oh, ow), dtype=torch.float32, device=x.device)
        kind = 1
    else:
        raise ValueError(out)
    L = lib()
    wsb = L.rr_resize_workspace(n, h, w, c, oh, ow)
    if wsb == 0:
        raise RuntimeError(f"rr_resize_bilinear_u8: unsupported shape {tuple(x.shape)} -> {(oh, ow)}")
    ws = _ws(wsb, x.device)
    mp = sp = None
    if mean is not None:
        mp = (C.c_float * c)(*[float(v) for v in mean])
        sp = (C.c_float * c)(*[float(v) for v in std])
    L.check(L.rr_resize_bilinear_u8(n, h, w, c, oh, ow, _p(x), kind,
                                    C.cast(mp, C.c_void_p) if mp is not None else None,
                                    C.cast(sp, C.c_void_p) if sp is not None else None,
                                    _p(y), _p(ws), wsb, stream()), "rr_resize_bilinear_u8")
    return y


def ssim_u8(a, b):
    """per-image skimage SSIM (data_range 255, channel_axis=2) of two
    [n, h, w, c] uint8 batches (08:125) -> fp64 [n]"""
    _need_cuda(a, b)
    if a.shape != b.shape or a.dtype != torch.uint8 or a.dim() != 4:
        raise TypeError("ssim_u8 expects two equal [n, h, w, c] uint8 tensors")
    n, h, w, c = a.shape
    out = torch.empty(n, dtype=torch.float64, device=a.device)
    L = lib()
    wsb = L.rr_ssim_workspace(n, c)
    ws = _ws(wsb, a.device)
    L.check(L.rr_ssim_u8(n, h, w, c, _p(a.contiguous()), _p(b.contiguous()), _p(out), _p(ws), wsb,
                         stream()), "rr_ssim_u8")
    return out


def motion_blur_kernel(degree, angle):
    """host: the [KMAX, KMAX] fp32 taps of the 14:55-59 motion-blur kernel"""
    buf = (C.c_float * (RR_DISTORT_KMAX * RR_DISTORT_KMAX))()
    lib().check(lib().rr_motion_blur_kernel(int(degree), int(angle), C.cast(buf, C.c_void_p)),
                "rr_motion_blur_kernel")
    return torch.frombuffer(bytearray(buf), dtype=torch.float32).view(RR_DISTORT_KMAX, RR_DISTORT_KMAX)


def distort_u8(x, params, taps, mode=0, noise=None, seed=0):
    """distortion generator on a [n, h, w, c] uint8 batch: ``params`` is a
    list of n DistortParam, ``taps`` [n, KMAX, KMAX] fp32 (host or device),
    ``noise`` an optional fp64 [n, h, w, c] field (else Philox(seed))."""
    _need_cuda(x)
    n, h, w, c = x.shape
    x = x.contiguous()
    if len(params) != n:
        raise ValueError("one DistortParam per image")
    arr = (DistortParam * n)(*params)
    prm = torch.frombuffer(bytearray(arr), dtype=torch.uint8).to(x.device)
    taps = taps.to(x.device, torch.float32).contiguous()
    if tuple(taps.shape) != (n, RR_DISTORT_KMAX, RR_DISTORT_KMAX):
        raise ValueError("taps must be [n, KMAX, KMAX]")
    if noise is not None:
        noise = noise.to(x.device, torch.float64).contiguous()
        if tuple(noise.shape) != (n, h, w, c):
            raise ValueError("noise must match the image batch")
    y = torch.empty_like(x)
    L = lib()
    wsb = L.rr_distort_workspace(n, h, w, c)
    ws = _ws(wsb, x.device)
    L.check(L.rr_distort_u8(n, h, w, c, int(mode), _p(x), _p(y), _p(prm), _p(taps), _p(noise),
                            int(seed) & (2 ** 64 - 1), _p(ws), wsb, stream()), "rr_distort_u8")
    return y


def zero_(t):
    lib().check(lib().rr_zero(_p(t), t.numel() * t.element_size(), stream()), "rr_zero")
    return t


MODES = dict(conv3x3=RR_CONV3X3, conv1x1=RR_CONV1X1, convT_up=RR_CONVT_UP,
             convT_down=RR_CONVT_DOWN)
