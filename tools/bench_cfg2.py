"""cfg2 throughput: SimpleUNet (07_train_restoration.py:75-120) denoise
training step -- forward, MSE (07:142), backward, Adam lr 1e-3 (07:143) -- at
batch 256, 64x64, on one GPU, as a HIP graph.  fp32 (the BASELINE config) and
bf16.  Synthetic GTSRB-shaped data (clean U{0..255}/255, bad = clean +
N(0, 0.1) clipped), random-init weights.  FLOP/img: 9,495,379,968 (SURVEY
8d, hook-counted fwd+bwd).  usage: python tools/bench_cfg2.py [--steps 20]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"), REPO]

import torch  # noqa: E402

import roadrestore as rr  # noqa: E402
from roadrestore.optim import flatten_parameters  # noqa: E402

FLOP_IMG = 9495379968


def run(dt, B, H, steps, warmup):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = rr.SimpleUNet().to(dev)
    m.compute_dtype = dt
    m.train()
    flatten_parameters(m)
    opt = rr.Adam(m.parameters(), lr=1e-3, capturable=True)
    crit = rr.MSELoss()
    g = torch.Generator(device=dev).manual_seed(1)
    clean = torch.randint(0, 256, (B, 3, H, H), generator=g, device=dev, dtype=torch.uint8).float() / 255
    bad = (clean + 0.1 * torch.randn((B, 3, H, H), generator=g, device=dev)).clamp_(0, 1)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = crit(m(bad), clean)
        loss.backward()
        opt.step()
        return loss

    for _ in range(warmup):
        step()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        loss = step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        graph.replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    v = B * steps / el
    return {"config": "cfg2: SimpleUNet denoise fwd + MSE + bwd + Adam, 07_train_restoration.py",
            "dtype": "fp32" if dt == torch.float32 else "bf16", "batch": B, "image": [H, H, 3],
            "images_per_sec": round(v, 1), "ms_per_step": round(el / steps * 1e3, 3),
            "achieved_model_tflops": round(v * FLOP_IMG / 1e12, 2), "loss": round(loss.item(), 6),
            "data": "synthetic, random-init weights", "hip_graph": True}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    for dt in (torch.float32, torch.bfloat16):
        print(json.dumps(run(dt, a.batch, 64, a.steps, a.warmup)), flush=True)


if __name__ == "__main__":
    main()
