"""A/B of the 3x3 bf16 wgrad paths (LDS-halo vs per-tap) at the cfg3 shapes:
per-layer time, TFLOP/s and max relative difference between the two."""
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


tot = {"halo": [0, 0], "tap": [0, 0]}
for name, H, c1, c2, co in LAYERS:
    x1 = torch.randn(B, H, H, c1, device=dev).bfloat16()
    x2 = torch.randn(B, H, H, c2, device=dev).bfloat16() if c2 else None
    dy = torch.randn(B, H, H, co, device=dev).bfloat16()
    fl = 2.0 * B * H * H * co * (c1 + c2) * 9
    res = {}
    for tag, env in (("halo", "0"), ("tap", "1")):
        os.environ["RR_WGRAD_NOHALO"] = env
        dw = torch.empty(co, c1 + c2, 3, 3, device=dev)
        t = timeit(lambda: ops.wgrad(RR_CONV3X3, dy, x1, x2, B, H, H, co, dw=dw))
        res[tag] = (t, dw.clone())
        tot[tag][0] += fl
        tot[tag][1] += t
    d = ((res["halo"][1] - res["tap"][1]).norm() / res["tap"][1].norm()).item()
    print(json.dumps(dict(layer=name, halo_ms=round(res["halo"][0], 3), tap_ms=round(res["tap"][0], 3),
                          halo_tf=round(fl / res["halo"][0] / 1e9, 1),
                          tap_tf=round(fl / res["tap"][0] / 1e9, 1), rel_diff=d)), flush=True)
print(json.dumps({k: round(v[0] / v[1] / 1e9, 1) for k, v in tot.items()}))
