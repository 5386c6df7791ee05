"""Kernel times of the first conv at the cfg3 shape (B = 512, 64x64, bf16):
the fused backward (rr_conv_in_wgrad_act: PReLU backward + 3->64 weight grad
from the image) and the forward (rr_conv_in_mfma: conv + bias + PReLU, both
outputs), HIP events over 20 launches, median of 5, plus SHA-1s of the
outputs for a bitwise comparison of two builds.

    python tools/first_wgrad_time.py [other.so]   # alternates this build / other, 3 rounds"""
import hashlib
import json
import os
import statistics
import subprocess
import sys

R_ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def child():
    sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
    import torch
    from roadrestore import ops
    dev = torch.device("cuda:0")
    g0 = torch.Generator(device=dev).manual_seed(7)
    B, H = 512, 64
    x = torch.rand(B, 3, H, H, device=dev, generator=g0)
    g = torch.randn(B, H, H, 64, device=dev, generator=g0).bfloat16()
    t = torch.randn(B, H, H, 64, device=dev, generator=g0).bfloat16()
    alpha = torch.tensor([0.25], device=dev)
    dw = torch.empty(64, 3, 3, 3, device=dev)
    db = torch.empty(64, device=dev)
    da = torch.empty(1, device=dev)

    def timed(f):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        res = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                f()
            e.record()
            torch.cuda.synchronize()
            res.append(s.elapsed_time(e) / 20 * 1e3)
        return round(statistics.median(res), 1)

    def sha(*ts):
        h = hashlib.sha1()
        for v in ts:
            h.update(v.float().cpu().numpy().tobytes())
        return h.hexdigest()[:12]
    us = timed(lambda: ops.first_conv_wgrad_act(x, g, t, 2, alpha, dw, db, dalpha=da))
    w1 = torch.randn(64, 3, 3, 3, device=dev, generator=g0) * 0.2
    b1 = torch.randn(64, device=dev, generator=g0) * 0.1
    wp = ops.pack_conv_in(w1, b1, torch.bfloat16)
    out = {}

    def fwd():
        out["y"] = ops.first_conv_fwd(x, w1, b1, torch.bfloat16, wp, act=2, alpha=alpha, want_pre=True)
    us_f = timed(fwd)
    print(json.dumps({"lib": os.environ.get("RR_LIB_PATH", "cur"), "wgrad_us": us, "sha": sha(dw, db, da),
                      "fwd_us": us_f, "fwd_sha": sha(*out["y"])}), flush=True)


def main():
    if os.environ.get("_FW_CHILD"):
        child()
        return
    other = sys.argv[1] if len(sys.argv) > 1 else None
    for _ in range(3):
        for lib in ([None, other] if other else [None]):
            env = dict(os.environ, _FW_CHILD="1")
            env.pop("RR_LIB_PATH", None)
            if lib:
                env["RR_LIB_PATH"] = lib
            subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, check=True, timeout=300)


if __name__ == "__main__":
    main()
