"""Where a conv3r K-loop stage spends its cycles: the diagnostic build
(``make -C csrc stamps`` -> libroadrestore_stamps.so, conv3r compiled with
RR_CONV3R_STAMPS) sums per wave the s_memtime segments of every stage:

  row0  stage start -> row 0's fragments in registers (A + B reads)
  vm    the stage-end (or mid-stage) vmcnt wait for the DMA
  bar   the barrier after it
  rest  everything else in the loop (MFMA issue, B-row reads, DMA issue)

and per wave the prologue (kernel entry -> K loop: first halo + weights) and
the epilogue (K loop end -> return: statistics, bias, stores).

Read the SHARES, not the totals: every stamp drains the LDS reads in flight.
Usage: python tools/conv3r_stamps.py [NAME=v1,v2 ...] (env switches to sweep; cfg3 layers, B=512)."""
import ctypes as C
import itertools
import json
import os
import sys

R_ = os.path.join(os.path.dirname(__file__), "..")
PKG = os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd")
os.environ["RR_LIB_PATH"] = os.path.join(PKG, "roadrestore", "libroadrestore_stamps.so")
sys.path.insert(0, PKG)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from roadrestore import ops  # noqa: E402
from roadrestore._lib import RR_CONV3X3, lib  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 512))
LAYERS = [("res2.c1", 32, 64, 0, 128), ("res2.c2", 32, 128, 0, 128), ("dec2.c1", 32, 128, 64, 64),
          ("res3.c2", 16, 256, 0, 256), ("dec3.c1", 16, 256, 128, 128), ("bott.512", 8, 512, 0, 512)]
N = 1 << 18
fn = lib().dll.rr_conv3r_stamps
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
    r = r[r[:, 5] == 1].astype(np.float64)
    nst = r[:, 4]
    loop, row0, vm, bar = r[:, 0], r[:, 1], r[:, 2], r[:, 3]
    rest = loop - row0 - vm - bar
    per = lambda v: round(float(np.median(v / nst)), 1)   # noqa: E731
    tot = float(np.sum(loop))
    pro, epi = r[:, 6], r[:, 7]
    return {"waves": int(len(r)), "cyc_per_stage": per(loop), "row0": per(row0), "vm": per(vm),
            "bar": per(bar), "rest": per(rest), "stages": int(np.median(nst)),
            "loop_cyc": round(float(np.median(loop)), 0), "prologue_cyc": round(float(np.median(pro)), 0),
            "epilogue_cyc": round(float(np.median(epi)), 0),
            "share": {k: round(float(np.sum(v)) / tot, 3)
                      for k, v in (("row0", row0), ("vm", vm), ("bar", bar), ("rest", rest))}}


sweeps = [(k, v.split(",")) for k, v in (a.split("=", 1) for a in sys.argv[1:])]
combos = list(itertools.product(*[[(k, v) for v in vals] for k, vals in sweeps])) or [()]
for name, H, c1, c2, co in LAYERS:
    x1 = torch.randn(B, H, H, c1, device=dev).bfloat16()
    x2 = torch.randn(B, H, H, c2, device=dev).bfloat16() if c2 else None
    dy = torch.randn(B, H, H, co, device=dev).bfloat16()
    wt = torch.randn(co, c1 + c2, 3, 3, device=dev) * 0.05
    wf, wd = ops.pack_conv(wt, torch.bfloat16)
    bias = torch.randn(co, device=dev)
    for combo in combos:
        for k, v in combo:
            os.environ[k] = v
        tag = " ".join(f"{k}={v}" for k, v in combo)
        d = ops.IgemmDesc(ops.RR_BF16, RR_CONV3X3, B, H, H, c1, c2, co, 0, 0, 0, 1, 0, 1, 0)
        f = stamps(lambda: ops.igemm(RR_CONV3X3, x1, x2, B, H, H, wf, co, bias=bias, stats=True))
        print(json.dumps({"cfg": tag, "layer": name, "op": "fwd", "kernel": ops.igemm_kernel_name(d), **f}),
              flush=True)
        g = stamps(lambda: ops.igemm(RR_CONV3X3, dy, None, B, H, H, wd, c1 + c2, split=c1 if c2 else 0))
        print(json.dumps({"cfg": tag, "layer": name, "op": "dgrad", **g}), flush=True)
