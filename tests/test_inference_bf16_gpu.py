"""cfg5 on the bf16 throughput path at the reference's own geometry (224 x 224;
17:66, 17:84-86, 18:28-32, 18:46-47) -- the path tools/bench_inference.py
times:

  GTSRB-sized uint8 crops -> Resize((224, 224)) + ToTensor (PIL-exact)
    -> ResUNet.eval() in bf16: every BN folded into its conv, the 3x3 convs on
       the tap-reuse kernel's row-segment tiles -- the 64 -> 64 ones at 224 on
       the row-streaming kernel's 32-wide column strips -- with the
       rr_igemm_ex epilogues (PReLU, residual, fused 2x2 max-pool)
    -> clamp, x255, uint8 truncation
    -> Resize + ToTensor + Normalize(ImageNet) -> VGG16 in bf16 (conv + ReLU +
       max-pool in one epilogue, the full-size map never written) -> Top-1.

Bounds.  bf16 parity is not bitwise: each stage is held to the
error of an IDEAL bf16 implementation of that stage, measured by the
bf16-storage emulation (oracle/bf16_emulation.py: the reference arithmetic in
fp64, every tensor the HIP path stores rounded to bf16 at the same point,
including the folded weights), both against the fp64 oracle:
  restored image rel-L2      <= 2 x ideal + 2e-3   (as tests/test_fullsize_gpu.py)
  judge logits rel-L2        <= 2 x ideal + 2e-3   (same u8 input for both)
  Top-1 equal to the fp32 oracle (the reference's precision) on every image
  whose fp32 top-2 margin exceeds 2 x that image's measured max |logit error|
  (at least a quarter of the batch must be decided that way), and on the whole
  batch agreeing with fp32 at least as often as ideal bf16 does (less one).
Measured (round 4): restored 2.490e-2 vs ideal 2.491e-2; logits 7.50e-3 vs
7.66e-3; Top-1 16/16 equal to fp32.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 16
MEAN, STD = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]


def _images(n, s0=48):
    """GTSRB-sized uint8 crops with a per-image tint (so Top-1 varies)."""
    rng = np.random.Generator(np.random.PCG64([2024, 16]))
    out = []
    for i in range(n):
        base = rng.integers(0, 256, size=(s0, s0, 3)).astype(np.float64)
        tint = np.array([(i * 70) % 256, (i * 130 + 40) % 256, (255 - i * 40) % 256], dtype=np.float64)
        out.append(np.clip(0.35 * base + 0.65 * tint, 0, 255).astype(np.uint8))
    return np.stack(out)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _eval_state(seed=7):
    """ResUNet weights with non-trivial running statistics (so the fold is
    exercised: gamma / sqrt(var + eps) != 1, mean != 0)."""
    from oracle import seeded as S
    sd = S.model_state_dict("resunet")
    g = torch.Generator().manual_seed(seed)
    for k, v in sd.items():
        if k.endswith("running_var"):
            v.copy_(torch.rand(v.shape, generator=g) * 0.8 + 0.6)
        elif k.endswith("running_mean"):
            v.copy_(torch.randn(v.shape, generator=g) * 0.05)
    return sd


def test_inference_pipeline_bf16_224(dev):
    import roadrestore as rr
    from roadrestore import imgproc as T, ops
    from roadrestore._lib import RR_CONV3X3
    from oracle import reference_cpu as R
    from oracle import bf16_emulation as E
    from oracle import imgproc_cpu as I
    from oracle import seeded as S

    nt = torch.get_num_threads()
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    try:
        imgs = _images(B)
        sd = _eval_state()
        vsd = S.seeded_state_dict(S.load_manifest("vgg16"), seed=4)

        # ---- device pipeline, bf16 ----
        net = rr.ResUNet().to(dev).eval()
        net.load_state_dict(sd)
        net.compute_dtype = torch.bfloat16
        judge = rr.vgg16().to(dev).eval()
        judge.load_state_dict(vsd)
        judge.compute_dtype = torch.bfloat16
        pre = T.Compose([T.Resize((224, 224)), T.ToTensor()])
        judge_pre = T.Compose([T.Resize((224, 224)), T.ToTensor(), T.Normalize(MEAN, STD)])
        log = []
        ops.LAUNCH_LOG = log
        try:
            with torch.no_grad():
                x = pre(torch.from_numpy(imgs).to(dev))
                out = net(x).clamp_(0, 1)
                u8 = ops.to_uint8_hwc(out)
                n_restore = len(log)
                logits = judge(judge_pre(u8))
                pred = ops.argmax_rows(logits)
                torch.cuda.synchronize()
        finally:
            ops.LAUNCH_LOG = None

        # ---- the kernels: the 64 -> 64 3x3 convs at 224 run on the
        # row-streaming kernel's column strips (restore: res1 conv1 + PReLU,
        # res1 conv2 + residual + ReLU + pool, dec1 conv2; judge: conv1_2 +
        # ReLU + pool), every other 3x3 conv with >= 32 input channels on the
        # tap-reuse kernel's row-segment tiles (224 is not a whole-row map),
        # and the inference epilogues are taken ----
        conv3 = [(k, t) for k, t in log if t.startswith(f"fwd m{RR_CONV3X3} ")]
        wide = [(k, t) for k, t in conv3 if int(t.split(" c")[1].split("+")[0]) >= 32]
        assert wide, log

        def is64(t):
            return "x224x224 c64+0->64" in t
        strips = [(k, t) for k, t in wide if is64(t)]
        assert len(strips) == 4, strips                                        # 3 restore + judge conv1_2
        bad = [(k, t) for k, t in strips if not k.startswith("stream3_kernel<s32")]
        bad += [(k, t) for k, t in wide if not is64(t) and not k.startswith("conv3r_kernel<s")]
        assert not bad, bad
        ex_r = [t for _, t in log[:n_restore] if " ex" in t]
        # (the judge's conv + ReLU + MaxPool2d pairs: rr_igemm_pool, tag "... pool")
        ex_j = [t for _, t in log[n_restore:] if t.endswith(" pool")]
        acts = {int(t.rsplit(" ex", 1)[1]) for t in ex_r}
        print("restore ex epilogues:", sorted(acts), "judge conv+pool launches:", len(ex_j))
        assert any(a & ops.RR_ACT_PRELU == ops.RR_ACT_PRELU for a in acts)     # conv1 + PReLU
        assert any(a & ops.RR_ACT_RES for a in acts)                           # identity tail
        assert any(a & ops.RR_ACT_POOL for a in acts)                          # encoder pool
        assert len(ex_j) >= 4                                                  # conv + ReLU + pool

        # ---- restored image against fp64, bounded by ideal bf16 ----
        xc = x.cpu()
        x_ref = torch.from_numpy(np.stack([I.to_tensor_normalize(I.pil_resize_bilinear(im, 224, 224))
                                           for im in imgs]))
        assert torch.equal(xc, x_ref)                                          # PIL-exact resize
        p64 = {k: (v.double() if v.dtype.is_floating_point else v.clone()) for k, v in sd.items()}
        with torch.no_grad():
            o64 = R.resunet_forward(p64, xc.double(), training=False)
            oe = E.resunet_forward_eval_folded(p64, xc.double())
        o = out.float().cpu()
        e_out, e_ideal = _rel(o, o64.clamp(0, 1)), _rel(oe.clamp(0, 1), o64.clamp(0, 1))
        print(f"restored rel-L2 vs fp64: HIP bf16 {e_out:.3e}, ideal bf16 {e_ideal:.3e}")
        assert e_out <= 2.0 * e_ideal + 2e-3, (e_out, e_ideal)
        u8c = u8.cpu().numpy()
        u8_64 = R.to_uint8_image(o64.float())
        d = np.abs(u8c.astype(int) - u8_64.astype(int))
        print(f"u8 vs fp64 oracle: mean |d| {d.mean():.3f}, max {d.max()}")

        # ---- judge on the same u8 images: logits vs fp64, Top-1 vs fp32 ----
        xin = torch.from_numpy(np.stack([I.to_tensor_normalize(I.pil_resize_bilinear(u, 224, 224),
                                                               MEAN, STD) for u in u8c]))
        v64 = {k: v.double() for k, v in vsd.items()}
        with torch.no_grad():
            l64 = R.vgg16_forward(v64, xin.double())
            le = E.vgg16_forward(v64, xin.double())
            l32 = R.vgg16_forward({k: v.clone() for k, v in vsd.items()}, xin)
        lg = logits.float().cpu()
        e_lg, e_lg_i = _rel(lg, l64), _rel(le, l64)
        err = (lg.double() - l64).abs().max().item()
        print(f"logits rel-L2 vs fp64: HIP bf16 {e_lg:.3e}, ideal bf16 {e_lg_i:.3e}; max |err| {err:.3e}")
        assert e_lg <= 2.0 * e_lg_i + 2e-3, (e_lg, e_lg_i)
        top2 = l32.topk(2, dim=1).values
        margin = top2[:, 0] - top2[:, 1]
        e_img = (lg.double() - l64).abs().max(dim=1).values.float()     # per image
        decided = margin > 2.0 * e_img
        p32 = R.top1(l32)
        pc = pred.cpu()
        agree, agree_i = int((pc == p32).sum()), int((R.top1(le) == p32).sum())
        print(f"Top-1: {int(decided.sum())}/{B} decided (margin > 2 x the image's max |logit err|); "
              f"classes {sorted(set(p32.tolist()))}; agree with fp32 on {agree}/{B} "
              f"(ideal bf16: {agree_i}/{B})")
        assert int(decided.sum()) * 4 >= B, (margin, e_img)
        assert torch.equal(pc[decided], p32[decided]), (pc.tolist(), p32.tolist())
        assert agree >= agree_i - 1, (agree, agree_i)
        assert len(set(p32.tolist())) >= 2
    finally:
        torch.set_num_threads(nt)
