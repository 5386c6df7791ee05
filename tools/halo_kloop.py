"""K-loop share of the tiled halo conv on the deep cfg3 layers: time with
RR_IGEMM_DBG=0 / 2 (K loop run twice; results wrong) / 1 (no epilogue)."""
import os, sys
R_ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch
from roadrestore import ops
from roadrestore._lib import RR_CONV3X3
dev = torch.device("cuda:0")
B = 512
for H, ci, co in ((32, 128, 128), (16, 256, 256), (16, 128, 256), (8, 512, 512), (8, 256, 512)):
    x = torch.randn(B, H, H, ci, device=dev).bfloat16()
    wf, _ = ops.pack_conv(torch.randn(co, ci, 3, 3, device=dev) * 0.02, torch.bfloat16)
    b = torch.randn(co, device=dev)
    res = {}
    for rnd in range(3):
        for dbg in ("0", "2", "1"):
            os.environ["RR_IGEMM_DBG"] = dbg
            f = lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, co, bias=b, stats=True)
            for _ in range(2):
                f()
            ev = []
            for _ in range(8):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(); f(); e.record(); ev.append((s, e))
            torch.cuda.synchronize()
            res.setdefault(dbg, []).append(min(s.elapsed_time(e) for s, e in ev))
    t0, t2, t1 = (min(res[k]) * 1e3 for k in ("0", "2", "1"))
    fl = 2.0 * B * H * H * co * ci * 9
    print(f"{H}x{H} c{ci}->{co}: full {t0:6.1f} us ({fl / t0 / 1e6:6.0f} TF/s)  Kloop {t2 - t0:6.1f} us "
          f"({fl / (t2 - t0) / 1e6:6.0f} TF/s)  noepi {t1:6.1f} us")
