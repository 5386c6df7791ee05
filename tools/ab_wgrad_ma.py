"""A/B of the halo wgrad variants: wave tiles (RR_WGRAD_HALO_MA = 2: 2 x 2
tiles of 16x16 MFMA blocks per wave, 4: all 64 dy channels x 16 x channels
per wave) and global prefetch depth (RR_WGRAD_HALO_PF = 1 / 2 stages)
at the cfg3 W <= 16 weight-grad shapes, B = 512: per-layer median time in
alternating rounds, TFLOP/s, and whether the two results are bitwise equal
(same pixel order per output element, same split-K partials)."""
import json, os, sys
R_ = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch
from roadrestore import ops
from roadrestore._lib import RR_CONV3X3

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 512))
# (name, W, c_in1, c_in2, c_out)
LAYERS = [("res3.c1", 16, 128, 0, 256), ("res3.c2", 16, 256, 0, 256), ("dec3.c1", 16, 256, 128, 128),
          ("dec3.c2", 16, 128, 0, 128), ("b0.c1", 8, 256, 0, 512), ("b.512", 8, 512, 0, 512),
          ("b2.c1", 8, 512, 0, 256), ("b2.c2", 8, 256, 0, 256)]


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


CFG = {"ma2": {"RR_WGRAD_HALO_MA": "2", "RR_WGRAD_HALO_PF": "1"},
       "ma4": {"RR_WGRAD_HALO_MA": "4", "RR_WGRAD_HALO_PF": "1"},
       "ma4pf2": {"RR_WGRAD_HALO_MA": "4", "RR_WGRAD_HALO_PF": "2"}}
tot = {k: [0.0, 0.0] for k in CFG}
for name, H, c1, c2, co in LAYERS:
    g = torch.Generator(device=dev).manual_seed(7)
    x1 = torch.randn(B, H, H, c1, device=dev, generator=g).bfloat16()
    x2 = torch.randn(B, H, H, c2, device=dev, generator=g).bfloat16() if c2 else None
    dy = torch.randn(B, H, H, co, device=dev, generator=g).bfloat16()
    fl = 2.0 * B * H * H * co * (c1 + c2) * 9
    res = {k: [] for k in CFG}
    outs = {}
    for rnd in range(3):
        for tag, env in CFG.items():
            os.environ.update(env)
            dw = torch.empty(co, c1 + c2, 3, 3, device=dev)
            res[tag].append(timeit(lambda: ops.wgrad(RR_CONV3X3, dy, x1, x2, B, H, H, co, dw=dw)))
            outs[tag] = dw.clone()
    t = {k: sorted(v)[1] for k, v in res.items()}
    for k in t:
        tot[k][0] += fl
        tot[k][1] += t[k]
    print(json.dumps(dict(layer=name, **{f"{k}_ms": round(t[k], 4) for k in CFG},
                          **{f"{k}_tf": round(fl / t[k] / 1e9, 1) for k in CFG},
                          bitwise_equal=all(torch.equal(outs["ma2"], outs[k]) for k in CFG))), flush=True)
for k in ("RR_WGRAD_HALO_MA", "RR_WGRAD_HALO_PF"):
    os.environ.pop(k)
print(json.dumps({"total_ms": {k: round(v[1], 4) for k, v in tot.items()},
                  "tflops": {k: round(v[0] / v[1] / 1e9, 1) for k, v in tot.items()}}))
