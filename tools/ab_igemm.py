"""A/B of the bf16 3x3 igemm paths (LDS-halo vs per-tap) at the cfg3 shapes:
fwd (bias+ReLU+stats) and dgrad (split for concat layers) time, TFLOP/s and
the relative difference between the two paths."""
import json, os, sys
R_ = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch
from roadrestore import ops
from roadrestore._lib import RR_CONV3X3

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 512))
LAYERS = [("res1.c", 64, 64, 0, 64), ("dec1.c1", 64, 64, 64, 64), ("res2.c1", 32, 64, 0, 128),
          ("res2.c2", 32, 128, 0, 128), ("dec2.c1", 32, 128, 64, 64), ("res3.c1", 16, 128, 0, 256),
          ("res3.c2", 16, 256, 0, 256), ("dec3.c1", 16, 256, 128, 128), ("bott.512", 8, 512, 0, 512),
          ("bott.c1", 8, 256, 0, 512), ("vgg3_x", 16, 256, 0, 256)]


def timeit(fn, reps=10):
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


tot = {}
for name, H, c1, c2, co in LAYERS:
    x1 = torch.randn(B, H, H, c1, device=dev).bfloat16()
    x2 = torch.randn(B, H, H, c2, device=dev).bfloat16() if c2 else None
    dy = torch.randn(B, H, H, co, device=dev).bfloat16()
    wt = torch.randn(co, c1 + c2, 3, 3, device=dev) * 0.05
    wf, wd = ops.pack_conv(wt, torch.bfloat16)
    bias = torch.randn(co, device=dev)
    fl = 2.0 * B * H * H * co * (c1 + c2) * 9
    row = {"layer": name}
    outs = {}
    for tag, env in (("halo", "0"), ("tap", "1")):
        os.environ["RR_IGEMM_NOHALO"] = env
        tf = timeit(lambda: ops.igemm(RR_CONV3X3, x1, x2, B, H, H, wf, co, bias=bias, act=1, stats=True))
        td = timeit(lambda: ops.igemm(RR_CONV3X3, dy, None, B, H, H, wd, c1 + c2, split=c1 if c2 else 0))
        y, _, st = ops.igemm(RR_CONV3X3, x1, x2, B, H, H, wf, co, bias=bias, act=1, stats=True)
        g1, g2, _ = ops.igemm(RR_CONV3X3, dy, None, B, H, H, wd, c1 + c2, split=c1 if c2 else 0)
        outs[tag] = (y.float(), st.sum(0), g1.float())
        row[f"{tag}_fwd_tf"] = round(fl / tf / 1e9, 1)
        row[f"{tag}_dgrad_tf"] = round(fl / td / 1e9, 1)
        row[f"{tag}_ms"] = [round(tf, 3), round(td, 3)]
        t = tot.setdefault(tag, [0.0, 0.0])
        t[0] += 2 * fl
        t[1] += tf + td
    for i, k in enumerate(("y", "stats", "dgrad")):
        a, b = outs["halo"][i], outs["tap"][i]
        row[f"rel_{k}"] = float((a - b).norm() / b.norm())
    print(json.dumps(row), flush=True)
print(json.dumps({k: round(v[0] / v[1] / 1e9, 1) for k, v in tot.items()}))
