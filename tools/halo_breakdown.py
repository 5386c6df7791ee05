"""Time split of the halo igemm per layer: K loop (L), epilogue (E), fixed
per-tile cost (F, prologue + launch) from three timing-only variants
(RR_IGEMM_DBG: 0 normal, 1 no epilogue, 2 K loop twice):
T0 = F + L + E, T1 = F + L, T2 = F + 2L + E."""
import json, os, sys
R_ = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch
from roadrestore import ops
from roadrestore._lib import RR_CONV3X3

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 512))
LAYERS = [("dec1.c1", 64, 64, 64, 64), ("res2.c1", 32, 64, 0, 128), ("res2.c2", 32, 128, 0, 128),
          ("dec2.c1", 32, 128, 64, 64), ("res3.c1", 16, 128, 0, 256), ("res3.c2", 16, 256, 0, 256),
          ("dec3.c1", 16, 128, 256, 128), ("bott.256", 8, 256, 0, 512), ("bott.512", 8, 512, 0, 512)]
if os.environ.get("LAYERS"):
    LAYERS = [l for l in LAYERS if l[0] in os.environ["LAYERS"].split(",")]


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


for name, H, c1, c2, co in LAYERS:
    x1 = torch.randn(B, H, H, c1, device=dev).bfloat16()
    x2 = torch.randn(B, H, H, c2, device=dev).bfloat16() if c2 else None
    wt = torch.randn(co, c1 + c2, 3, 3, device=dev) * 0.05
    wf, _ = ops.pack_conv(wt, torch.bfloat16)
    fl = 2.0 * B * H * H * co * (c1 + c2) * 9
    bytes_ = B * H * H * (c1 + c2 + co) * 2
    for stats in (True, False):
        t = {}
        for dbg in (0, 1, 2):
            os.environ["RR_IGEMM_DBG"] = str(dbg)
            t[dbg] = timeit(lambda: ops.igemm(RR_CONV3X3, x1, x2, B, H, H, wf, co, stats=stats))
        os.environ["RR_IGEMM_DBG"] = "0"
        L = t[2] - t[0]
        E = t[0] - t[1]
        F = t[1] - L
        print(json.dumps(dict(layer=name, stats=stats, ms=round(t[0], 4), loop=round(L, 4), epi=round(E, 4),
                              fixed=round(F, 4), tflops=round(fl / t[0] / 1e9, 1),
                              loop_tflops=round(fl / L / 1e9, 1),
                              hbm_floor_ms=round(bytes_ / 5.3e12 * 1e3, 4))), flush=True)
