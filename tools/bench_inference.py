"""cfg5: end-to-end inference on one GPU, every stage on device
(17_run_unified_inference.py + 18_test_unified_benchmark.py):

  GTSRB-sized uint8 crops [n, s, s, 3]
    -> Resize((224, 224)) + ToTensor                     (17:66, PIL-exact)
    -> ResUNet.eval() forward, clamp(0, 1)               (17:85-86)
    -> x255 -> uint8 HWC (truncation)                    (17:89-90)
    -> Resize((224, 224)) + ToTensor + Normalize(ImageNet) (18:28-32)
    -> VGG16 (43-class head) logits -> Top-1             (18:46-47)
  plus PSNR / SSIM of the restored vs the clean 224 images (08:123-125).

Synthetic data, random-init weights (no checkpoints ship with the reference).
Batch 8192 processed in chunks (``--chunk``).  usage:
  python tools/bench_inference.py [--images 8192] [--chunk 1024] [--size 48]
(chunk 256 / 512 / 1024 / 2048: 8,906 / 9,071 / 9,115 / 9,101 img/s bf16, profiles/r4zb_inference_chunks.txt)"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"), REPO]

import torch  # noqa: E402

import roadrestore as rr  # noqa: E402
from roadrestore import imgproc as T, ops  # noqa: E402
from roadrestore._lib import path_flag  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=8192)
    ap.add_argument("--chunk", type=int, default=1024)
    ap.add_argument("--size", type=int, default=48, help="source crop side (GTSRB ~30-250)")
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    net = rr.ResUNet().to(dev).eval()
    net.compute_dtype = dt
    judge = rr.vgg16().to(dev).eval()
    judge.compute_dtype = dt
    g = torch.Generator(device=dev).manual_seed(1)
    clean = torch.randint(0, 256, (a.images, a.size, a.size, 3), dtype=torch.uint8, device=dev, generator=g)
    bad = T.apply_compound_distortion(clean, seed=2)                       # 16:14-37 test set
    pre = T.Compose([T.Resize((a.res, a.res)), T.ToTensor()])
    judge_pre = T.Compose([T.Resize((224, 224)), T.ToTensor(), T.Normalize(T.IMAGENET_MEAN, T.IMAGENET_STD)])
    clean224 = T.Resize((a.res, a.res))
    stage_ms = {"restore": 0.0, "judge": 0.0, "metrics": 0.0}

    def run(count, timing):
        top1 = []
        ps, ss = [], []
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        with torch.no_grad():
            for i in range(0, count, a.chunk):
                xb, cb = bad[i:i + a.chunk], clean[i:i + a.chunk]
                ev[0].record()
                out = net(pre(xb)).clamp_(0, 1)
                u8 = ops.to_uint8_hwc(out)
                ev[1].record()
                logits = judge(judge_pre(u8))
                top1.append(ops.argmax_rows(logits))
                ev[2].record()
                c224 = clean224(cb)
                ps.append(T.psnr(c224, u8))
                ss.append(T.ssim(c224, u8))
                ev[3].record()
                if timing:
                    torch.cuda.synchronize()
                    stage_ms["restore"] += ev[0].elapsed_time(ev[1])
                    stage_ms["judge"] += ev[1].elapsed_time(ev[2])
                    stage_ms["metrics"] += ev[2].elapsed_time(ev[3])
        return torch.cat(top1), torch.cat(ps), torch.cat(ss)

    run(2 * a.chunk, False)                                               # warmup
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    top1, ps, ss = run(a.images, False)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    run(a.images, True)
    # roofline of the two compute stages: hook-counted conv/linear FLOP per
    # image at 224 over the HIP-event stage times, vs the dense
    # MFMA peak of the compute dtype (MI355X_MICROARCH.md)
    peak = 2516.6 if a.dtype == "bf16" else 157.3
    fl = {"restore": 55_991_599_104 * (a.res / 224) ** 2, "judge": 30_932_688_896}
    roof = {}
    for k in ("restore", "judge"):
        tf = fl[k] * a.images / (stage_ms[k] * 1e-3) / 1e12
        roof[k] = {"achieved_tflops": round(tf, 1), "peak_tflops": peak, "frac": round(tf / peak, 4)}
    print(json.dumps({
        "config": f"cfg5 end-to-end inference: {a.images} GTSRB-sized {a.size}x{a.size} crops, "
                  f"Resize({a.res}) + ResUNet eval + uint8 + Resize(224)/Normalize + VGG16 Top-1 + PSNR/SSIM",
        "dtype": a.dtype, "chunk": a.chunk, "images_per_sec": round(a.images / wall, 1),
        "wall_s": round(wall, 3),
        "stage_ms_per_1k_images": {k: round(v / a.images * 1000, 2) for k, v in stage_ms.items()},
        "data": "synthetic uint8 crops, compound distortion (16:14-37) on device, random-init weights",
        "mean_psnr_db": round(ps.mean().item(), 3), "mean_ssim": round(ss.mean().item(), 4),
        "top1_hist_max": int(torch.bincount(top1, minlength=43).max().item()),
        "top1_note": "random-init judge: Top-1 collapses to few classes; Top-1 parity with a "
                     "non-degenerate judge is tests/test_models_gpu.py::"
                     "test_inference_pipeline_fp32_end_to_end",
        "roofline": roof, "bn_folded": path_flag("fold_bn", 1) != 0,
    }))


if __name__ == "__main__":
    main()
