"""RR_S3_DBG ablations of the streaming conv (timing only; results wrong):
bit0 no MFMA, bit1 no row DMA, bit2 no stores.  fwd+stats at B=512."""
import os, sys
R_ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch
from roadrestore import ops
from roadrestore._lib import RR_CONV3X3
dev = torch.device("cuda:0")
B = 512
for H in (64, 32):
    x = torch.randn(B, H, H, 64, device=dev).bfloat16()
    wf, wd = ops.pack_conv(torch.randn(64, 64, 3, 3, device=dev) * 0.05, torch.bfloat16)
    b = torch.randn(64, device=dev)
    res = {}
    for rnd in range(3):
        for dbg in (0, 1, 2, 4, 3, 5, 6, 7):
            os.environ["RR_S3_DBG"] = str(dbg)
            f = lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, 64, bias=b, stats=True)
            for _ in range(3):
                f()
            ev = []
            for _ in range(10):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(); f(); e.record(); ev.append((s, e))
            torch.cuda.synchronize()
            res.setdefault(dbg, []).append(min(s.elapsed_time(e) for s, e in ev))
    for dbg, v in res.items():
        print(f"W={H} dbg={dbg} ({'noMFMA ' if dbg & 1 else ''}{'noDMA ' if dbg & 2 else ''}{'noST' if dbg & 4 else ''}): {min(v) * 1e3:.1f} us")
