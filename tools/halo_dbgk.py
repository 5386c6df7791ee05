"""K-loop bounds of the halo igemm (timing only): the loop with the epilogue
skipped (RR_IGEMM_DBG=1) as built, without its barriers (RR_HALO_DBGK=1),
without its LDS fragment reads (2), without both (3); full time of the
unsplit staging (RR_HALO_DBGK=32) beside the weight/halo role split, and
of the next-chunk halo issued all at tap 0 (64) beside its spread over taps,
and weights 3 stages ahead (128) beside 2 (BC = 128 only; at BC = 64 these
select the same unsplit kernel, so their spread there is the noise).
DBGK_LIST=0,32,1,2,3 (env) picks the K-loop variants timed without the epilogue."""
import json, os, sys
R_ = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch
from roadrestore import ops
from roadrestore._lib import RR_CONV3X3

dev = torch.device("cuda:0")
B = 512
LAYERS = [("res2.c1", 32, 64, 0, 128), ("res2.c2", 32, 128, 0, 128), ("res3.c2", 16, 256, 0, 256),
          ("bott.512", 8, 512, 0, 512), ("res3.c1", 16, 128, 0, 256), ("bott.c1", 8, 256, 0, 512)]


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
    wt = torch.randn(co, c1 + c2, 3, 3, device=dev) * 0.05
    wf, _ = ops.pack_conv(wt, torch.bfloat16)
    fl = 2.0 * B * H * H * co * (c1 + c2) * 9
    r = {"layer": name, "kernel": ops.igemm_kernel_name(ops.IgemmDesc(ops.RR_BF16, RR_CONV3X3, B, H, H, c1, c2, co, 0, 0, 0, 0, 0, 1, 0))}
    os.environ["RR_IGEMM_DBG"] = "0"
    r["full_ms"] = round(timeit(lambda: ops.igemm(RR_CONV3X3, x1, None, B, H, H, wf, co, stats=True)), 4)
    for k, tag in ((32, "unsplit"), (64, "unsliced"), (128, "w3ahead")):
        os.environ["RR_HALO_DBGK"] = str(k)
        r[f"full_{tag}_ms"] = round(timeit(lambda: ops.igemm(RR_CONV3X3, x1, None, B, H, H, wf, co, stats=True)), 4)
    for k in [int(v) for v in os.environ.get("DBGK_LIST", "0").split(",")]:
        os.environ["RR_IGEMM_DBG"] = "1"
        os.environ["RR_HALO_DBGK"] = str(k)
        t = timeit(lambda: ops.igemm(RR_CONV3X3, x1, None, B, H, H, wf, co, stats=True))
        r[f"noepi_dbgk{k}_ms"] = round(t, 4)
        r[f"noepi_dbgk{k}_tf"] = round(fl / t / 1e9, 1)
    os.environ["RR_IGEMM_DBG"] = "0"
    os.environ["RR_HALO_DBGK"] = "0"
    print(json.dumps(r), flush=True)
