"""The CPU oracle (oracle/reference_cpu.py) against the golden fixtures the
REFERENCE classes produced (oracle/gen_golden.py).  Runs without a GPU."""
import os

import numpy as np
import pytest
import torch

from oracle import reference_cpu as R
from oracle import seeded as S


def gold(name):
    return np.load(os.path.join(S.GOLDEN_DIR, name + ".npz"))


def test_seeded_inputs_reproduce_fixtures():
    z = gold("resunet_64")
    clean = S.image_batch(2, 64, 64, seed=30 + 64)
    assert torch.equal(clean, torch.from_numpy(z["clean"]))
    assert torch.equal(S.fog_noise(clean, seed=40 + 64), torch.from_numpy(z["bad"]))
    z = gold("resunet_224")
    bad = S.fog_noise(S.image_batch(1, 224, 224, seed=30 + 224), seed=40 + 224)
    assert abs(bad.double().sum().item() - z["bad_sum"][0]) < 1e-6


def test_simpleunet_oracle_bitwise():
    z = gold("simpleunet_64")
    p = S.model_state_dict("simpleunet")
    out = R.simple_unet_forward(p, torch.from_numpy(z["bad"]))
    assert torch.equal(out, torch.from_numpy(z["out"]))


def test_resunet_oracle_eval_and_train():
    z = gold("resunet_64")
    sd = S.model_state_dict("resunet")
    bad = torch.from_numpy(z["bad"])
    with torch.no_grad():
        out = R.resunet_forward({k: v.clone() for k, v in sd.items()}, bad, training=False)
    assert torch.equal(out, torch.from_numpy(z["out_eval"]))
    p = {k: v.clone() for k, v in sd.items()}
    with torch.no_grad():
        out = R.resunet_forward(p, bad, training=True)
    assert torch.equal(out, torch.from_numpy(z["out_train"]))
    keys = [str(k) for k in z["running_keys"]]
    got = torch.cat([p[k].reshape(-1) for k in keys]).numpy()
    assert np.array_equal(got, z["running_vals"])
    assert p["res1.conv_block.1.num_batches_tracked"].item() == 1


def test_unified_loss_oracle():
    z = gold("resunet_64")
    sd = S.model_state_dict("resunet")
    perc = S.seeded_state_dict(S.load_manifest("perceptual"), seed=5)
    bad, clean = torch.from_numpy(z["bad"]), torch.from_numpy(z["clean"])
    with torch.no_grad():
        out = R.resunet_forward({k: v.clone() for k, v in sd.items()}, bad, True)
        assert abs(R.l1_loss(out, clean).item() - z["l_pix"][0]) == 0
        assert abs(R.perceptual_loss(perc, out, clean).item() - z["l_perc"][0]) <= 1e-6 * z["l_perc"][0]
        assert abs(R.perceptual_loss(perc, bad, clean).item() - z["perc_bad_clean"][0]) <= 1e-6


def test_postprocess_psnr_oracle():
    z = gold("resunet_64")
    u8 = R.to_uint8_image(torch.from_numpy(z["out_eval"]))
    assert np.array_equal(u8, z["out_u8"])
    for i in range(2):
        assert abs(R.psnr_u8(z["clean_u8"][i], z["out_u8"][i]) - z["psnr"][i]) < 1e-12
    a = np.zeros((4, 4, 3), np.uint8)
    assert R.psnr_u8(a, a) == float("inf")


@pytest.mark.parametrize("H", [64])
def test_vgg16_oracle_logits(H):
    z = gold(f"vgg16_{H}")
    sd = S.seeded_state_dict(S.load_manifest("vgg16"), seed=3)
    x = S.classifier_batch(8, H, seed=50 + H)
    assert torch.equal(x, torch.from_numpy(z["x"]))
    with torch.no_grad():
        lg = R.vgg16_forward(sd, x)
    # fp32 conv accumulation order depends on the host CPU's oneDNN kernels: the golden logits
    # (generated from the imported reference on one host) reproduce bit-for-bit there and to
    # ~1e-6 relative on another (AVX512 EPYC: max |diff| 1.9e-5 on logits of magnitude ~14)
    torch.testing.assert_close(lg, torch.from_numpy(z["logits"]), rtol=1e-5, atol=1e-4)
    assert np.array_equal(R.top1(lg).numpy(), z["pred"])


def test_adamw_restatement_matches_torch():
    p = torch.randn(100)
    g = torch.randn(100)
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=2e-4, weight_decay=1e-4)
    st = {}
    mine = {"p": p.clone()}
    for _ in range(3):
        ref.grad = g.clone()
        opt.step()
        R.adamw_step(mine, {"p": g}, st, 2e-4, weight_decay=1e-4)
    assert torch.equal(mine["p"], ref.detach())


def test_cosine_schedule():
    sch_lr = []
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=2e-4)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=25)
    for e in range(25):
        sch_lr.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    for e, lr in enumerate(sch_lr):
        assert abs(lr - R.cosine_lr(2e-4, e, 25)) < 1e-12


def test_bf16_emulation_is_the_reference_step_without_rounding(monkeypatch):
    """oracle/bf16_emulation.py is the reference restatement with bf16
    rounding points inserted: with the rounding switched off it reproduces
    reference_cpu's unified step exactly (same ops, same order)."""
    import torch
    from oracle import bf16_emulation as E, reference_cpu as R, seeded as S
    monkeypatch.setattr(E, "_rb", lambda x: x)
    sd = S.model_state_dict("resunet")
    perc = S.seeded_state_dict(S.load_manifest("perceptual"), seed=5)
    clean = S.image_batch(1, 32, 32, seed=3)
    bad = S.fog_noise(clean, seed=4)
    outs = []
    for M in (R, E):
        p = {k: v.clone().requires_grad_(v.dtype.is_floating_point and "running" not in k)
             for k, v in sd.items()}
        out = M.resunet_forward(p, bad, True)
        loss = M.unified_loss(out, clean, perc)
        loss.backward()
        outs.append((out.detach(), loss.item(), p["res2.conv_block.0.weight"].grad))
    assert torch.equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]
    assert torch.equal(outs[0][2], outs[1][2])
    # and with rounding on, it really rounds (differs from fp32)
    monkeypatch.undo()
    p = {k: v.clone() for k, v in sd.items()}
    assert not torch.equal(E.resunet_forward(p, bad, True), outs[0][0])


@pytest.mark.parametrize("hw", ["60x60", "36x52"])
def test_resunet_oracle_odd_sizes(hw):
    """The restatement reproduces the reference ResUNet bit for bit at input
    sizes that trigger the nearest interpolate (14:169-182): eval / train
    forward and the unified loss, from the committed fixtures."""
    from oracle import reference_cpu as R
    from oracle import seeded as S
    z = gold(f"resunet_{hw}")
    sd = S.model_state_dict("resunet")
    bad, clean = torch.from_numpy(z["bad"]), torch.from_numpy(z["clean"])
    with torch.no_grad():
        out = R.resunet_forward({k: v.clone() for k, v in sd.items()}, bad, training=False)
        assert torch.equal(out, torch.from_numpy(z["out_eval"]))
        p = {k: v.clone() for k, v in sd.items()}
        out = R.resunet_forward(p, bad, training=True)
        assert torch.equal(out, torch.from_numpy(z["out_train"]))
        perc_sd = S.seeded_state_dict(S.load_manifest("perceptual"), seed=5)
        loss = R.unified_loss(out, clean, perc_sd)
        assert abs(loss.item() - z["loss"][0]) <= 1e-6 * abs(z["loss"][0])


def test_08_psnr_leg_oracle():
    """cfg2's PSNR leg (08:86-125): the oracle chain -- Pillow Resize(224) +
    ToTensor, SimpleUNet batch-1 eval forward, uint8 truncation + BGR, the
    restated cv2.resize(INTER_LINEAR) of the clean image, PSNR / SSIM --
    reproduces the fixture the REFERENCE SimpleUNet (08:19-46) produced.
    The cv2 resize and skimage metrics are restatements (parity vs cv2 /
    skimage unpinned)."""
    from PIL import Image
    from oracle import imgproc_cpu as I
    z = gold("simpleunet_08")
    sd = S.model_state_dict("simpleunet")
    for i in range(len(z["sizes"])):
        dist = z[f"dist_{i}"]
        x = torch.from_numpy(np.asarray(Image.fromarray(dist, "RGB").resize((224, 224),
                                                                           Image.BILINEAR)).copy())
        assert np.array_equal(x.numpy(), I.pil_resize_bilinear(dist, 224, 224))
        x = x.permute(2, 0, 1).float().div(255).unsqueeze(0)
        with torch.no_grad():
            out = R.simple_unet_forward({k: v.clone() for k, v in sd.items()}, x)
        assert abs(out.double().sum().item() - z[f"out_sum_{i}"][0]) <= 1e-6 * out.numel()
        u8 = R.to_uint8_image(out)[0][:, :, ::-1]
        assert np.array_equal(u8, z["out_bgr"][i])
        c224 = I.cv_resize_linear(z[f"clean_bgr_{i}"], 224, 224)
        assert np.array_equal(c224, z["clean224"][i])
        assert abs(R.psnr_u8(c224, u8) - z["psnr"][i]) < 1e-12
        assert abs(I.ssim(c224, u8) - z["ssim"][i]) < 1e-12


def test_cv_resize_oracle_properties():
    """The OpenCV INTER_LINEAR restatement: same size = copy; a constant image
    stays constant (weights sum to 2048, both rounding paths exact there);
    upscaling by 2 keeps every source pixel's value on the grid where the
    source coordinate lands on it; the SIMD and scalar vertical roundings
    differ by at most one level."""
    from oracle import imgproc_cpu as I
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (13, 17, 3), dtype=np.uint8)
    assert np.array_equal(I.cv_resize_linear(img, 13, 17), img)
    for v in (0, 1, 128, 254, 255):
        c = np.full((9, 11, 3), v, np.uint8)
        assert np.all(I.cv_resize_linear(c, 224, 224) == v)
        assert np.all(I.cv_resize_linear(c, 4, 5) == v)
    a = I.cv_resize_linear(img, 50, 61, simd_lanes=16)
    b = I.cv_resize_linear(img, 50, 61, simd_lanes=10 ** 6)       # all scalar
    assert np.abs(a.astype(int) - b.astype(int)).max() <= 1


def test_07adv_step_oracle():
    """07adv:143-157 (SimpleUNet, L1 + 0.1 perceptual, Adam lr 2e-4): the
    oracle's loss and grads reproduce the reference's fixture."""
    z = gold("simpleunet_07adv")
    sd = S.model_state_dict("simpleunet")
    perc = S.seeded_state_dict(S.load_manifest("perceptual"), seed=5)
    p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    bad, clean = torch.from_numpy(z["bad"]), torch.from_numpy(z["clean"])
    out = R.simple_unet_forward(p, bad)
    assert abs(R.l1_loss(out, clean).item() - z["l_pix"][0]) <= 1e-7
    loss = R.unified_loss(out, clean, perc)
    assert abs(loss.item() - z["loss"][0]) <= 1e-6 * abs(z["loss"][0])
    loss.backward()
    for k, v in p.items():
        idx = z[f"grad:{k}|idx"]
        assert np.abs(v.grad.reshape(-1)[idx].numpy() - z[f"grad:{k}|val"]).max() <= \
            1e-5 * (v.grad.abs().max().item() + 1e-30), k
