"""Kernel time of the fused first-conv backward (rr_conv_in_wgrad_act: PReLU
backward + 3->64 weight grad from the image) at the cfg3 shape (B = 512, 64x64,
bf16), HIP events over 20 launches, median of 5, plus a SHA-1 of (dw, db,
dalpha) for a bitwise comparison of two builds.

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

    def f():
        ops.first_conv_wgrad_act(x, g, t, 2, alpha, dw, db, dalpha=da)
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
    h = hashlib.sha1()
    for v in (dw, db, da):
        h.update(v.cpu().numpy().tobytes())
    print(json.dumps({"lib": os.environ.get("RR_LIB_PATH", "cur"), "us": round(statistics.median(res), 1),
                      "sha": h.hexdigest()[:12]}), flush=True)


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
