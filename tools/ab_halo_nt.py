"""Per-layer A/B of the BC = 64 halo conv's workgroup shape (timing): 8 waves
of 64 x 32 tiles (default) vs 4 waves of 64 x 64 tiles (RR_HALO_NT=256) and
the 128-pixel tile (RR_HALO_BP=128) and BC = 128 (RR_HALO_BC64_MAXCIN=32, where Cout is a
multiple of 128), full kernel, B = 512 bf16, on the
BC = 64 layers of the cfg3 step (fwd shapes; dgrad shapes have Cin / Cout
swapped)."""
import json
import os
import sys

R_ = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch  # noqa: E402
from roadrestore import ops  # noqa: E402
from roadrestore._lib import RR_CONV3X3  # noqa: E402

dev = torch.device("cuda:0")
B = 512
LAYERS = [("res2.c1", 32, 64, 128), ("res2.c2", 32, 128, 128), ("res2.c2.dgrad", 32, 128, 128),
          ("dec2.c1", 32, 192, 64), ("vgg2_1", 32, 64, 128), ("res2.c1.dgrad", 32, 128, 64),
          ("res3.c1", 16, 128, 256), ("dec3.c2", 16, 128, 128)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    v = sorted(s.elapsed_time(e) for s, e in ts)
    return v[len(v) // 2]


for name, H, ci, co in LAYERS:
    x = torch.randn(B, H, H, ci, device=dev).bfloat16()
    wf, _ = ops.pack_conv(torch.randn(co, ci, 3, 3, device=dev) * 0.05, torch.bfloat16)
    fl = 2.0 * B * H * H * co * ci * 9
    r = {"layer": name, "shape": [H, ci, co]}
    for tag, env in (("nt512", {}), ("nt256", {"RR_HALO_NT": "256"}), ("bp128", {"RR_HALO_BP": "128"}),
                     ("bc128", {"RR_HALO_BC64_MAXCIN": "32"}), ("nt512_again", {})):
        for k in ("RR_HALO_NT", "RR_HALO_BP", "RR_HALO_BC64_MAXCIN"):
            os.environ.pop(k, None)
        os.environ.update(env)
        r["kernel_" + tag] = ops.igemm_kernel_name(ops.IgemmDesc(ops.RR_BF16, RR_CONV3X3, B, H, H, ci, 0, co,
                                                                 0, 0, 0, 0, 0, 1, 0))
        t = timeit(lambda: ops.igemm(RR_CONV3X3, x, None, B, H, H, wf, co, stats=True))
        r[tag + "_ms"] = round(t, 4)
        r[tag + "_tf"] = round(fl / t / 1e9, 1)
    print(json.dumps(r), flush=True)
