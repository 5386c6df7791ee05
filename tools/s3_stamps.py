"""Where a row-streaming conv (stream3) step spends its cycles: the diagnostic
build (``make -C csrc s3stamps`` -> libroadrestore_s3stamps.so, stream3
compiled with RR_S3_STAMPS) sums per wave the s_memtime segments of every
step of the persistent loop:

  wait   the counted vmcnt wait + workgroup barrier at the step start
  issue  the epilogue operand loads + the DMA of the step D ahead
  mfma   the 18 (tap, k-half) groups of B reads and MFMAs
  epi    the epilogue (+ the wait for its operand loads)

per step (median over waves).  Read the SHARES: every stamp drains the LDS
reads in flight.  usage: python tools/s3_stamps.py  (cfg3 shapes, B = 512)"""
import ctypes as C
import json
import os
import sys

R_ = os.path.join(os.path.dirname(__file__), "..")
PKG = os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd")
os.environ["RR_LIB_PATH"] = os.path.join(PKG, "roadrestore", "libroadrestore_s3stamps.so")
sys.path.insert(0, PKG)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from roadrestore import ops  # noqa: E402
from roadrestore._lib import RR_CONV3X3, lib  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 512))
N = 256 * 8 * 8
fn = lib().dll.rr_s3_stamps_read
fn.argtypes = [C.c_void_p, C.c_int, C.c_int]
buf = np.zeros(N, dtype=np.uint64)


def stamps(run):
    run()
    torch.cuda.synchronize()
    fn(None, 0, 1)
    run()
    torch.cuda.synchronize()
    fn(buf.ctypes.data, N, 0)
    r = buf.reshape(-1, 8)
    r = r[r[:, 6] == 1].astype(np.float64)
    steps = np.maximum(r[:, 5], 1)
    tot = r[:, 0]
    seg = {"wait": r[:, 1], "issue": r[:, 2], "mfma": r[:, 3], "epi": r[:, 4]}
    per = {k: round(float(np.median(v / steps)), 1) for k, v in seg.items()}
    per["step"] = round(float(np.median(tot / steps)), 1)
    share = {k: round(float(np.sum(v) / np.sum(tot)), 3) for k, v in seg.items()}
    return {"waves": int(len(r)), "steps_per_wave": int(np.median(steps)), "cyc_per_step": per, "share": share}


for H in (64, 32):
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(B, H, H, 64, device=dev, generator=g).bfloat16()
    wf, wd = ops.pack_conv(torch.randn(64, 64, 3, 3, device=dev, generator=g) / 24, torch.bfloat16)
    bias = torch.randn(64, device=dev, generator=g)
    mk = torch.randn(B, H, H, 64, device=dev, generator=g).bfloat16()
    yb = torch.randn(B, H, H, 64, device=dev, generator=g).bfloat16()
    t1 = (torch.randn(B, H, H, 64, device=dev, generator=g) * 2 + 0.3).bfloat16()
    mean, inv = t1.float().reshape(-1, 64).mean(0), torch.ones(64, device=dev)
    s1, sh1 = torch.rand(64, device=dev, generator=g) + 0.5, torch.rand(64, device=dev, generator=g) - 0.5
    alpha = torch.tensor([0.23], device=dev)
    cases = [
        ("fwd_stats", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, 64, bias=bias, stats=True)),
        ("fwd_relu", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, 64, bias=bias, act=1)),
        ("dgrad", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wd, 64)),
        ("dgrad_mask", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wd, 64, mask=mk)),
        ("dgrad_acc", lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wd, 64, out=yb, accumulate=True)),
        ("bnbwd", lambda: ops.igemm_bnbwd(RR_CONV3X3, x, B, H, H, wd, 64, t1, mean, inv, s1, sh1, alpha)),
        ("pool", lambda: ops.igemm_pool(x, B, H, H, wf, 64, bias=bias)),
    ]
    for name, run in cases:
        print(json.dumps({"H": H, "case": name, **stamps(run)}), flush=True)
