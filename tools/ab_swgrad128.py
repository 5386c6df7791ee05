"""swgrad (row streaming) vs the tiled halo wgrad for 128-channel dy at the
cfg3 res2 shapes (B=512, 32x32, bf16), HIP events."""
import os, sys
R_ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch
from roadrestore import ops
from roadrestore._lib import RR_CONV3X3
dev = torch.device("cuda:0")
B = 512
for h, cin, cout in ((32, 64, 128), (32, 128, 128)):
    dy = torch.randn(B, h, h, cout, device=dev).bfloat16()
    x = torch.randn(B, h, h, cin, device=dev).bfloat16()
    dw = torch.empty(cout, cin, 3, 3, device=dev)
    res = {}
    for rnd_ in range(3):
        for sw in ("1", "0"):
            os.environ["RR_SWGRAD"] = sw
            f = lambda: ops.wgrad(RR_CONV3X3, dy, x, None, B, h, h, cout, dw=dw)
            f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                f()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(sw, []).append(s.elapsed_time(e) / 5 * 1e3)
    fl = 2.0 * B * h * h * cout * cin * 9
    t1, t0 = min(res["1"]), min(res["0"])
    print(f"{h}x{h} x{cin} dy{cout}: swgrad {t1:6.1f} us ({fl / t1 / 1e6:5.0f} TF/s)  "
          f"tiled {t0:6.1f} us ({fl / t0 / 1e6:5.0f} TF/s)", flush=True)
