"""Per-layer kernel times of one library build at the cfg3 shapes (B = 512),
one JSON line per layer (median of REPS HIP-event timings) with a SHA-1 of
the output bytes, so two builds run in alternating processes
(tools/gpu.sh ablayers:OTHER.so;SET) can be compared for time AND bitwise
equality.  SET=wgrad: every 3x3 / 1x1 / convT weight grad of the ResUNet
backward (14:96-186); SET=conv3r: the tap-reuse conv layers, fwd + dgrad;
SET=s3: the row-streaming conv's variants at 64x64 / 32x32.

    python tools/layer_times.py [SET]
"""
import hashlib
import json
import os
import sys

R_ = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch  # noqa: E402
from roadrestore import ops  # noqa: E402
from roadrestore._lib import RR_CONV1X1, RR_CONV3X3, RR_CONVT_UP  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 512))
REPS = int(os.environ.get("REPS", 10))
SET = sys.argv[1] if len(sys.argv) > 1 else "wgrad"

# (name, mode, H (input grid), c_in1, c_in2, c_out)
WGRAD = [("res1.c", RR_CONV3X3, 64, 64, 0, 64), ("dec1.c1", RR_CONV3X3, 64, 64, 64, 64),
         ("res2.c1", RR_CONV3X3, 32, 64, 0, 128), ("res2.c2", RR_CONV3X3, 32, 128, 0, 128),
         ("dec2.c1", RR_CONV3X3, 32, 128, 64, 64), ("dec2.c2", RR_CONV3X3, 32, 64, 0, 64),
         ("res3.c1", RR_CONV3X3, 16, 128, 0, 256), ("res3.c2", RR_CONV3X3, 16, 256, 0, 256),
         ("dec3.c1", RR_CONV3X3, 16, 256, 128, 128), ("dec3.c2", RR_CONV3X3, 16, 128, 0, 128),
         ("b0.c1", RR_CONV3X3, 8, 256, 0, 512), ("b.512", RR_CONV3X3, 8, 512, 0, 512),
         ("b2.c1", RR_CONV3X3, 8, 512, 0, 256), ("b2.c2", RR_CONV3X3, 8, 256, 0, 256),
         ("dec1.sc", RR_CONV1X1, 64, 64, 64, 64), ("res2.sc", RR_CONV1X1, 32, 64, 0, 128),
         ("dec2.sc", RR_CONV1X1, 32, 128, 64, 64), ("res3.sc", RR_CONV1X1, 16, 128, 0, 256),
         ("dec3.sc", RR_CONV1X1, 16, 256, 128, 128), ("b0.sc", RR_CONV1X1, 8, 256, 0, 512),
         ("b2.sc", RR_CONV1X1, 8, 512, 0, 256),
         ("up1", RR_CONVT_UP, 32, 64, 0, 64), ("up2", RR_CONVT_UP, 16, 128, 0, 64),
         ("up3", RR_CONVT_UP, 8, 256, 0, 128)]
CONV3R = [("res2.c1", 32, 64, 0, 128), ("res2.c2", 32, 128, 0, 128), ("dec2.c1", 32, 128, 64, 64),
          ("res3.c1", 16, 128, 0, 256), ("res3.c2", 16, 256, 0, 256), ("dec3.c1", 16, 256, 128, 128),
          ("dec3.c2", 16, 128, 0, 128), ("vgg2_2", 32, 128, 0, 128), ("vgg3_2", 16, 256, 0, 256),
          ("b0.c1", 8, 256, 0, 512), ("b.512", 8, 512, 0, 512), ("b2.c1", 8, 512, 0, 256)]


def timeit(fn):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(REPS):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    v = sorted(s.elapsed_time(e) for s, e in ts)
    return v[len(v) // 2]


def sha(*ts):
    h = hashlib.sha1()
    for t in ts:
        h.update(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()[:12]


tot_ms, tot_fl = 0.0, 0.0
g = torch.Generator(device=dev).manual_seed(7)
if SET == "wgrad":
    for name, mode, H, c1, c2, co in WGRAD:
        Ho = 2 * H if mode == RR_CONVT_UP else H
        x1 = torch.randn(B, H, H, c1, device=dev, generator=g).bfloat16()
        x2 = torch.randn(B, H, H, c2, device=dev, generator=g).bfloat16() if c2 else None
        dy = torch.randn(B, Ho, Ho, co, device=dev, generator=g).bfloat16()
        taps = {RR_CONV3X3: 9, RR_CONV1X1: 1, RR_CONVT_UP: 4}[mode]
        shape = (c1 + c2, co, 2, 2) if mode == RR_CONVT_UP else (co, c1 + c2, 3, 3) \
            if mode == RR_CONV3X3 else (co, c1 + c2, 1, 1)
        dw = torch.empty(shape, device=dev)
        fl = 2.0 * B * H * H * co * (c1 + c2) * taps
        ms = timeit(lambda: ops.wgrad(mode, dy, x1, x2, B, H, H, co, dw=dw))
        tot_ms += ms
        tot_fl += fl
        print(json.dumps({"layer": name, "kernel": ops.wgrad_kernel_name(
            ops.WgradDesc(ops.RR_BF16, mode, B, H, H, c1, c2, co, 0)), "ms": round(ms, 4),
            "tf": round(fl / ms / 1e9, 1), "sha": sha(dw)}), flush=True)
elif SET == "conv3r":
    for name, H, c1, c2, co in CONV3R:
        x1 = torch.randn(B, H, H, c1, device=dev, generator=g).bfloat16()
        x2 = torch.randn(B, H, H, c2, device=dev, generator=g).bfloat16() if c2 else None
        dy = torch.randn(B, H, H, co, device=dev, generator=g).bfloat16()
        wt = torch.randn(co, c1 + c2, 3, 3, device=dev, generator=g) * 0.05
        wf, wd = ops.pack_conv(wt, torch.bfloat16)
        bias = torch.randn(co, device=dev, generator=g)
        fl = 2.0 * B * H * H * co * (c1 + c2) * 9
        out = {}

        def fwd():
            out["f"] = ops.igemm(RR_CONV3X3, x1, x2, B, H, H, wf, co, bias=bias, stats=True)

        def dgr():
            out["d"] = ops.igemm(RR_CONV3X3, dy, None, B, H, H, wd, c1 + c2, split=c1 if c2 else 0)
        tf, td = timeit(fwd), timeit(dgr)
        tot_ms += tf + td
        tot_fl += 2 * fl
        d = ops.IgemmDesc(ops.RR_BF16, RR_CONV3X3, B, H, H, c1, c2, co, 0, 0, 0, 1, 0, 1, 0)
        outs = [out["f"][0], out["f"][2], out["d"][0]] + ([out["d"][1]] if c2 else [])
        print(json.dumps({"layer": name, "kernel": ops.igemm_kernel_name(d), "fwd_ms": round(tf, 4),
                          "dgrad_ms": round(td, 4), "tf": round(2 * fl / (tf + td) / 1e9, 1),
                          "sha": sha(*outs)}), flush=True)
elif SET == "epi":
    # conv3r dgrads with each epilogue operand set (the backward's variants):
    # plain, + accumulate (identity / shortcut grads), + ReLU mask (VGG), both
    for name, H, c1, co in [("res2.c2", 32, 128, 128), ("res2.c1", 32, 64, 128), ("res3.c2", 16, 256, 256),
                            ("vgg3_3", 16, 256, 256), ("b.512", 8, 512, 512)]:
        dy = torch.randn(B, H, H, co, device=dev, generator=g).bfloat16()
        _, wd = ops.pack_conv(torch.randn(co, c1, 3, 3, device=dev, generator=g) * 0.05, torch.bfloat16)
        y0 = torch.randn(B, H, H, c1, device=dev, generator=g).bfloat16()
        mk = torch.randn(B, H, H, c1, device=dev, generator=g).bfloat16()
        fl = 2.0 * B * H * H * co * c1 * 9
        row = {"layer": name}
        hs = []
        for tag, acc, msk in (("plain", False, False), ("acc", True, False), ("mask", False, True),
                              ("acc_mask", True, True)):
            out = {}
            yb = y0.clone()

            def run():
                out["y"] = ops.igemm(RR_CONV3X3, dy, None, B, H, H, wd, c1, out=yb if acc else None,
                                     accumulate=acc, mask=mk if msk else None)[0]
            ms = timeit(run)
            row[tag] = round(ms, 4)
            tot_ms += ms
            tot_fl += fl
            if not acc:
                hs.append(out["y"])
        d = ops.IgemmDesc(ops.RR_BF16, RR_CONV3X3, B, H, H, co, 0, c1, 0, 0, 0, 0, 0, 0, 0)
        row["kernel"] = ops.igemm_kernel_name(d)
        row["sha"] = sha(*hs)
        print(json.dumps(row), flush=True)
elif SET == "bnbwd":
    # conv2 dgrad with the fused BN1 -> PReLU backward epilogue (14:99-105):
    # (name, H, C) -- dy and t1 both C channels
    for name, H, C in [("res2.c2", 32, 128), ("res3.c2", 16, 256), ("dec3.c2", 16, 128),
                       ("b.512", 8, 512), ("b2.c2", 8, 256)]:
        g2 = torch.randn(B, H, H, C, device=dev, generator=g).bfloat16()
        _, wd = ops.pack_conv(torch.randn(C, C, 3, 3, device=dev, generator=g) / (3 * C ** 0.5),
                              torch.bfloat16)
        t1 = (torch.randn(B, H, H, C, device=dev, generator=g) * 2 + 0.3).bfloat16()
        tf = t1.float().reshape(-1, C)
        mean = tf.mean(0)
        inv = 1.0 / torch.sqrt(tf.var(0, unbiased=False) + 1e-5)
        s1 = torch.rand(C, device=dev, generator=g) + 0.5
        sh1 = torch.rand(C, device=dev, generator=g) - 0.5
        alpha = torch.tensor([0.23], device=dev)
        out = {}

        def run():
            out["r"] = ops.igemm_bnbwd(RR_CONV3X3, g2, B, H, H, wd, C, t1, mean, inv, s1, sh1, alpha)
        ms = timeit(run)
        fl = 2.0 * B * H * H * C * C * 9
        tot_ms += ms
        tot_fl += fl
        gm, part, rows, arows = out["r"]
        print(json.dumps({"layer": name, "kernel": ops.igemm_kernel_name(
            ops.IgemmDesc(ops.RR_BF16, RR_CONV3X3, B, H, H, C, 0, C, 0, 0, 0, 0, 0, 0, 0), bnbwd=True),
            "ms": round(ms, 4), "tf": round(fl / ms / 1e9, 1), "sha": sha(gm)}), flush=True)
elif SET == "s3":
    # the row-streaming conv's variants (64 -> 64 channels): fwd + BN stats
    # (res1 / dec1 / dec2 conv2), bias + ReLU (VGG conv1_2), plain / ReLU-mask /
    # accumulate dgrads, the fused BN -> PReLU backward dgrad
    for H in (64, 32):
        x = torch.randn(B, H, H, 64, device=dev, generator=g).bfloat16()
        wf, wd = ops.pack_conv(torch.randn(64, 64, 3, 3, device=dev, generator=g) / 24, torch.bfloat16)
        bias = torch.randn(64, device=dev, generator=g)
        mk = torch.randn(B, H, H, 64, device=dev, generator=g).bfloat16()
        y0 = torch.randn(B, H, H, 64, device=dev, generator=g).bfloat16()
        t1 = (torch.randn(B, H, H, 64, device=dev, generator=g) * 2 + 0.3).bfloat16()
        tf = t1.float().reshape(-1, 64)
        mean = tf.mean(0)
        inv = 1.0 / torch.sqrt(tf.var(0, unbiased=False) + 1e-5)
        s1 = torch.rand(64, device=dev, generator=g) + 0.5
        sh1 = torch.rand(64, device=dev, generator=g) - 0.5
        alpha = torch.tensor([0.23], device=dev)
        fl = 2.0 * B * H * H * 64 * 64 * 9
        row = {"layer": f"s3_{H}"}
        hs = []
        out = {}
        yb = y0.clone()
        cases = (("fwd_stats", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, 64, bias=bias, stats=True)),
                 ("fwd_relu", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, 64, bias=bias, act=1)),
                 ("dgrad", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wd, 64)),
                 ("dgrad_mask", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wd, 64, mask=mk)),
                 ("dgrad_acc", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wd, 64, out=yb, accumulate=True)),
                 ("bnbwd", lambda: ops.igemm_bnbwd(RR_CONV3X3, x, B, H, H, wd, 64, t1, mean, inv, s1, sh1, alpha)))
        for tag, fn in cases:
            def run(fn=fn, tag=tag):
                out[tag] = fn()
            ms = timeit(run)
            row[tag] = round(ms, 4)
            tot_ms += ms
            tot_fl += fl
            if tag != "dgrad_acc":
                hs.append(out[tag][0])
        row["sha"] = sha(*hs)
        print(json.dumps(row), flush=True)
print(json.dumps({"set": SET, "total_ms": round(tot_ms, 4),
                  "tflops": round(tot_fl / tot_ms / 1e9, 1)}), flush=True)
