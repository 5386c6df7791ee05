"""Kernel times of the fused conv + ReLU + 2x2 max-pool (rr_igemm_pool) against
the plain conv + bias + ReLU and the separate pool, at the perceptual VGG's
conv1_2 / conv2_2 shapes of the cfg3 step (B = 512: 64x64x64 -> 64, 32x32x128
-> 128).  HIP events around 20 back-to-back launches each, median of 5.

    python tools/pool_bench.py [batch]"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"), REPO]

import torch  # noqa: E402

from roadrestore import ops  # noqa: E402
from roadrestore._lib import RR_CONV3X3  # noqa: E402

BF = torch.bfloat16


def timed(fn, reps=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / reps * 1e3)
    return round(statistics.median(res), 1)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dev = torch.device("cuda:0")
    for h, c in ((64, 64), (32, 128)):
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.randn(n, h, h, c, device=dev, generator=g).to(BF)
        wt = torch.randn(c, c, 3, 3, device=dev, generator=g) / (3 * c ** 0.5)
        b = torch.randn(c, device=dev, generator=g) * 0.1
        pk, _ = ops.pack_conv(wt, BF)
        y, _, _ = ops.igemm(RR_CONV3X3, x, None, n, h, h, pk, c, bias=b, act=1)
        d = ops.igemm_pool_desc(x, n, h, h, c, True)
        r = {"shape": [n, h, h, c], "pool_kernel": ops.igemm_pool_kernel_name(d),
             "conv_relu_us": timed(lambda: ops.igemm(RR_CONV3X3, x, None, n, h, h, pk, c, bias=b, act=1, out=y)),
             "maxpool_us": timed(lambda: ops.maxpool2_fwd(y)),
             "fused_us": timed(lambda: ops.igemm_pool(x, n, h, h, pk, c, bias=b)),
             "fused_noidx_us": timed(lambda: ops.igemm_pool(x, n, h, h, pk, c, bias=b, want_idx=False))}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
