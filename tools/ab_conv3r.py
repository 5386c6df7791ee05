"""Per-layer timing of the bf16 3x3 convs the tap-reuse kernel (conv3r) owns
at the cfg3 shapes (B = 512): fwd (bias + stats) and dgrad, TFLOP/s, for
every value of an environment switch given on the command line, e.g.

    python tools/ab_conv3r.py RR_PATH=conv3r=1,conv3r=0

(the library's one run-time knob, RR_PATH, csrc/common.h; the timing-only
switches of earlier rounds were removed in round 6)

(each NAME=v1,v2,... is swept; the first switch varies fastest; the values
alternate per layer, ROUNDS times, and each is reported as its median)."""
import itertools
import json
import os
import sys

R_ = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch  # noqa: E402
from roadrestore import ops  # noqa: E402
from roadrestore._lib import RR_CONV3X3  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 512))
LAYERS = [("res2.c1", 32, 64, 0, 128), ("res2.c2", 32, 128, 0, 128), ("dec2.c1", 32, 128, 64, 64),
          ("res3.c1", 16, 128, 0, 256), ("res3.c2", 16, 256, 0, 256), ("dec3.c1", 16, 256, 128, 128),
          ("bott.c1", 8, 256, 0, 512), ("bott.512", 8, 512, 0, 512)]
# SET=224: the cfg5 geometry (row-segment tiles), B = 64 by default
LAYERS_224 = [("enc.224", 224, 64, 0, 64), ("dec1.224", 224, 64, 64, 64), ("e2.112", 112, 64, 0, 128),
              ("r2.112", 112, 128, 0, 128), ("e3.56", 56, 128, 0, 256), ("r3.56", 56, 256, 0, 256),
              ("b.28", 28, 512, 0, 512), ("v5.14", 14, 512, 0, 512)]
if os.environ.get("SET") == "224":
    LAYERS = LAYERS_224
    B = int(os.environ.get("B", 64))
if os.environ.get("ONLY"):
    LAYERS = [l for l in LAYERS if l[0] in os.environ["ONLY"].split(",")]
REPS = int(os.environ.get("REPS", 10))


def timeit(fn, reps=None):
    reps = reps or REPS
    for _ in range(2):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    v = sorted(s.elapsed_time(e) for s, e in ts)
    return v[len(v) // 2]


sweeps = [(k, v.split(",")) for k, v in (a.split("=", 1) for a in sys.argv[1:])]
data = {}
for name, H, c1, c2, co in LAYERS:
    x1 = torch.randn(B, H, H, c1, device=dev).bfloat16()
    x2 = torch.randn(B, H, H, c2, device=dev).bfloat16() if c2 else None
    dy = torch.randn(B, H, H, co, device=dev).bfloat16()
    wt = torch.randn(co, c1 + c2, 3, 3, device=dev) * 0.05
    wf, wd = ops.pack_conv(wt, torch.bfloat16)
    bias = torch.randn(co, device=dev)
    data[name] = (H, c1, c2, co, x1, x2, dy, wf, wd, bias)
combos = list(itertools.product(*[[(k, v) for v in vals] for k, vals in sweeps])) or [()]
# the switch values alternate per layer, ROUNDS times (a box drifts by several
# per cent over a sweep: sequential sweeps are not an A/B); median per value
ROUNDS = int(os.environ.get("ROUNDS", 3))
tot = {}
for name, (H, c1, c2, co, x1, x2, dy, wf, wd, bias) in data.items():
    fl = 2.0 * B * H * H * co * (c1 + c2) * 9
    d = ops.IgemmDesc(ops.RR_BF16, RR_CONV3X3, B, H, H, c1, c2, co, 0, 0, 0, 1, 0, 1, 0)
    meas = {}
    for _ in range(ROUNDS):
        for combo in combos:
            for k, v in combo:
                os.environ[k] = v
            tag = " ".join(f"{k}={v}" for k, v in combo)
            tf = timeit(lambda: ops.igemm(RR_CONV3X3, x1, x2, B, H, H, wf, co, bias=bias, stats=True))
            td = timeit(lambda: ops.igemm(RR_CONV3X3, dy, None, B, H, H, wd, c1 + c2,
                                          split=c1 if c2 else 0))
            m = meas.setdefault(tag, ([], [], ops.igemm_kernel_name(d)))
            m[0].append(tf)
            m[1].append(td)
    for tag, (tfs, tds, kname) in meas.items():
        tf, td = sorted(tfs)[len(tfs) // 2], sorted(tds)[len(tds) // 2]
        t = tot.setdefault(tag, [0.0, 0.0])
        t[0] += 2 * fl
        t[1] += tf + td
        print(json.dumps({"cfg": tag, "layer": name, "kernel": kname,
                          "fwd_ms": round(tf, 4), "dgrad_ms": round(td, 4),
                          "fwd_tf": round(fl / tf / 1e9, 1), "dgrad_tf": round(fl / td / 1e9, 1)}),
              flush=True)
print(json.dumps({k: {"tflops": round(v[0] / v[1] / 1e9, 1), "ms": round(v[1], 3)}
                  for k, v in tot.items()}))
