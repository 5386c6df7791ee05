"""Where does the bf16 training step's gradient error come from?  Per tensor
rel-L2 / cosine of (a) bf16 GPU, (b) fp32 GPU against the fp64 CPU oracle,
for the unified loss and for plain MSE (no sign discontinuity), at B=2 and
B=32 (diagnostic, not a test)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"), REPO]

import roadrestore as rr  # noqa: E402
from oracle import reference_cpu as R  # noqa: E402
from oracle import seeded as S  # noqa: E402

dev = torch.device("cuda:0")
sd = S.model_state_dict("resunet")
perc_sd = S.seeded_state_dict(S.load_manifest("perceptual"), seed=5)


def oracle(bad, clean, kind, dtype):
    p = {k: (v.detach().clone().to(dtype) if v.dtype.is_floating_point else v.clone()) for k, v in sd.items()}
    for k, v in p.items():
        if v.dtype.is_floating_point and "running" not in k:
            v.requires_grad_(True)
    out = R.resunet_forward(p, bad.to(dtype), True)
    if kind == "mse":
        loss = R.mse_loss(out, clean.to(dtype))
    else:
        loss = R.unified_loss(out, clean.to(dtype), {k: v.to(dtype) for k, v in perc_sd.items()})
    loss.backward()
    return out.detach().double(), {k: v.grad.double() for k, v in p.items() if v.requires_grad}


def ours(bad, clean, kind, dtype):
    m = rr.ResUNet().to(dev)
    m.load_state_dict(sd)
    m.compute_dtype = dtype
    m.train()
    out = m(bad.to(dev))
    if kind == "mse":
        loss = rr.MSELoss()(out, clean.to(dev))
    else:
        perc = rr.VGGPerceptualLoss().to(dev)
        perc.load_state_dict(perc_sd)
        perc.compute_dtype = dtype
        loss = rr.unified_loss(out, clean.to(dev), perc, 0.1)
    loss.backward()
    torch.cuda.synchronize()
    return out.detach().cpu().double(), {k: p.grad.cpu().double() for k, p in m.named_parameters()}


for B in (2, 32):
    clean = S.image_batch(B, 64, 64, seed=300)
    bad = S.fog_noise(clean, seed=400)
    for kind in ("mse", "unified"):
        o64, g64 = oracle(bad, clean, kind, torch.float64)
        res = {}
        for dt in (torch.float32, torch.bfloat16):
            o, g = ours(bad, clean, kind, dt)
            rows = []
            for k, t in g64.items():
                if t.norm() < 1e-9:
                    continue
                d = g[k] - t
                rows.append((d.norm().item() / t.norm().item(),
                             (g[k] * t).sum().item() / (g[k].norm() * t.norm()).item(), k))
            res[dt] = ((o - o64).norm().item() / o64.norm().item(), rows)
        e32, r32 = res[torch.float32]
        e16, r16 = res[torch.bfloat16]
        rel16 = np.array([r[0] for r in r16])
        cos16 = np.array([r[1] for r in r16])
        print(f"B={B} {kind}: out rel-L2 fp32 {e32:.2e} bf16 {e16:.2e}; grad rel-L2 bf16 median "
              f"{np.median(rel16):.3e} p90 {np.percentile(rel16, 90):.3e}; cos min {cos16.min():.4f} "
              f"median {np.median(cos16):.5f}; fp32 median {np.median([r[0] for r in r32]):.2e}")
        for e, c, k in sorted(r16, reverse=True)[:8]:
            print(f"    {k:45s} rel {e:.3e} cos {c:.4f}")
