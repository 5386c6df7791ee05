"""Time the 64 -> 64 channel bf16 3x3 conv at the cfg3 shapes (B=512) through
rr_igemm: the row-streaming kernel (RR_PATH=stream3=1) and the tap-reuse
kernel (RR_PATH=stream3=0), interleaved in one process.  Prints us / TFLOP/s / HBM GB/s
(algorithmic bytes: bf16 input + output (+ t or mask / accumulate reads))."""
import os
import sys

R_ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch  # noqa: E402
from roadrestore import ops  # noqa: E402
from roadrestore._lib import RR_CONV3X3  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 512))
reps = int(os.environ.get("REPS", 20))
variants = os.environ.get("VARIANTS", "stream3=1;stream3=0").split(";")
varenv = os.environ.get("VARENV", "RR_PATH")        # the env switch the variants set
only = os.environ.get("CASE")          # e.g. "64:fwd+stats"
rounds = int(os.environ.get("ROUNDS", 2))


def timeit(fn):
    for _ in range(3):
        fn()
    ev = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(e) for s, e in ev)
    return t[len(t) // 2]


res = {}
for H in ((64, 32) if not only else (int(only.split(":")[0]),)):
    x = torch.randn(B, H, H, 64, device=dev).bfloat16()
    y0 = torch.randn(B, H, H, 64, device=dev).bfloat16()
    t1 = torch.randn(B, H, H, 64, device=dev).bfloat16()
    wt = torch.randn(64, 64, 3, 3, device=dev) * 0.05
    wf, wd = ops.pack_conv(wt, torch.bfloat16)
    b = torch.randn(64, device=dev)
    mean = torch.zeros(64, device=dev)
    inv = torch.ones(64, device=dev)
    s1 = torch.ones(64, device=dev)
    sh1 = torch.zeros(64, device=dev)
    al = torch.tensor([0.25], device=dev)
    dwb = torch.empty(64, 64, 3, 3, device=dev)
    P = B * H * H
    fl = 2.0 * P * 64 * 576
    cases = {
        "fwd+stats": (lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, 64, bias=b, stats=True), 2),
        "fwd+relu": (lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, 64, bias=b, act=1), 2),
        "dgrad+acc": (lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wd, 64, out=y0, accumulate=True), 3),
        "wgrad": (lambda: ops.wgrad(RR_CONV3X3, y0, x, None, B, H, H, 64, dw=dwb), 2),
        "bnbwd": (lambda: ops.igemm_bnbwd(RR_CONV3X3, x, B, H, H, wd, 64, t1, mean, inv, s1, sh1, al), 3),
    }
    for _ in range(rounds):                  # interleaved rounds (rule 24)
        for name, (fn, passes) in cases.items():
            if only and name != only.split(":")[1]:
                continue
            for v in variants:
                os.environ[varenv] = v
                ms = timeit(fn)
                res.setdefault((H, name, v), []).append(ms)
for (H, name, v), ms in res.items():
    m = min(ms)
    P = B * H * H
    passes = 2 if name.startswith("fwd") or name == "wgrad" else 3
    print(f"W={H:2d} {name:10s} {varenv}={v}: {m * 1e3:7.1f} us  {2.0 * P * 64 * 576 / m / 1e9:7.1f} TF/s "
          f" {passes * P * 128 / m / 1e6:7.1f} GB/s")
