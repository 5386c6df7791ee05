"""Generate tests/golden/* by importing the REFERENCE scripts -- TEST INFRA ONLY.

Run here (the survey container, where /root/reference exists):

    python oracle/gen_golden.py

The reference is a set of digit-prefixed scripts whose third-party imports
(torchvision, cv2, skimage) are not installed; those are replaced by empty
stub modules before each script is loaded with importlib.
``torchvision.models.vgg16`` is stubbed with the restated torchvision cfg-D
module (oracle.reference_cpu.TorchvisionVGG16) because the ImageNet weights are
a network download; the reference's own ``VGGPerceptualLoss`` slicing /
freezing / loss code then runs unchanged on seeded weights.

Every fixture is produced by the reference classes themselves; the functional
restatement (oracle/reference_cpu.py) is checked against them here and the
check is re-run from the committed fixtures by tests/test_oracle.py.
The reference itself never travels: only the .npz/.json data land in
tests/golden/.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

from oracle import reference_cpu as R          # noqa: E402
from oracle import seeded as S                 # noqa: E402

REF = os.environ.get("RR_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")


def _install_stubs():
    tv = types.ModuleType("torchvision")
    for sub in ("transforms", "models", "datasets"):
        m = types.ModuleType("torchvision." + sub)
        setattr(tv, sub, m)
        sys.modules["torchvision." + sub] = m
    sys.modules["torchvision"] = tv
    tv.models.vgg16 = lambda weights=None, **kw: R.TorchvisionVGG16(num_classes=1000)
    sys.modules["cv2"] = types.ModuleType("cv2")
    sk = types.ModuleType("skimage")
    skm = types.ModuleType("skimage.metrics")
    skm.peak_signal_noise_ratio = None
    skm.structural_similarity = None
    sk.metrics = skm
    sys.modules["skimage"] = sk
    sys.modules["skimage.metrics"] = skm


def _load(fname, modname):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, fname))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def manifest(module):
    return [[k, list(v.shape)] for k, v in module.state_dict().items()]


def digest(named, idx_seed=123, n_samples=8):
    """Per-tensor (sum, L2 norm, sampled elements at fixed flat indices)."""
    out = {}
    for i, (k, t) in enumerate(named.items()):
        t = t.detach().double().reshape(-1)
        rng = np.random.Generator(np.random.PCG64([idx_seed, i]))
        idx = rng.integers(0, t.numel(), size=n_samples)
        out[k + "|sum"] = np.array([t.sum().item()])
        out[k + "|norm"] = np.array([t.norm().item()])
        out[k + "|idx"] = idx.astype(np.int64)
        out[k + "|val"] = t[idx].numpy()
    return out


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path + ("" if path.endswith(".npz") else ".npz")))


def _close(a, b, tol=0.0):
    d = (a - b).abs().max().item()
    assert d <= tol, d
    return d


def main():
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    os.makedirs(OUT, exist_ok=True)
    _install_stubs()
    m07 = _load("07_train_restoration.py", "ref07")
    m14 = _load("14_train_unified_advanced.py", "ref14")
    m17 = _load("17_run_unified_inference.py", "ref17")
    m08 = _load("08_run_inference.py", "ref08")

    # ---- manifests (reference key trees) ----------------------------------
    su, ru = m07.SimpleUNet(), m14.ResUNet()
    assert manifest(su) == manifest(m08.SimpleUNet())        # 08:19-46 copy
    assert manifest(ru) == manifest(m17.ResUNet())           # 17:29-55 copy
    perc = m14.VGGPerceptualLoss()
    mans = {"simpleunet": manifest(su), "resunet": manifest(ru),
            "vgg16": manifest(R.TorchvisionVGG16(43)), "perceptual": manifest(perc)}
    for n, man in mans.items():
        with open(os.path.join(OUT, f"manifest_{n}.json"), "w") as f:
            json.dump(man, f)
        print(n, len(man), "keys")

    # ---- SimpleUNet: fwd + MSE train step (07:151-160) ---------------------
    for H, B, tag in ((64, 2, "64"), (224, 1, "224")):
        sd = S.model_state_dict("simpleunet", seed=0)
        clean = S.image_batch(B, H, H, seed=10 + H)
        bad = S.fog_noise(clean, seed=20 + H)
        m = m07.SimpleUNet()
        m.load_state_dict(sd)
        out = m(bad)
        p = {k: v.clone() for k, v in sd.items()}
        _close(R.simple_unet_forward(p, bad), out.detach())
        arrays = dict(bad=bad.numpy(), clean=clean.numpy(), out=out.detach().numpy())
        if H == 64:
            opt = torch.optim.Adam(m.parameters(), lr=1e-3)          # 07:143
            opt.zero_grad()
            loss = torch.nn.MSELoss()(m(bad), clean)                  # 07:154-156
            loss.backward()
            grads = {k: v.grad for k, v in m.named_parameters()}
            opt.step()
            arrays["loss"] = np.array([loss.item()])
            arrays.update({"grad:" + k: v for k, v in digest(grads).items()})
            arrays.update({"post:" + k: v for k, v in
                           digest(dict(m.named_parameters())).items()})
        if H == 224:
            arrays["bad_sum"] = np.array([bad.double().sum().item()])
            del arrays["bad"], arrays["clean"]
        save(f"simpleunet_{tag}.npz", **arrays)

    # ---- ResUNet ------------------------------------------------------------
    # Seeded running stats do not match the seeded conv statistics, so eval-mode
    # activations would grow through 10 blocks.  Calibrate them the way a
    # trained model's are (cumulative batch statistics of a calibration batch,
    # momentum=None) and commit them: S.model_state_dict("resunet") applies them.
    cal = m14.ResUNet()
    cal.load_state_dict(S.seeded_state_dict(mans["resunet"], 0, S.convT_prefixes(mans["resunet"])))
    for mod in cal.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.momentum = None
            mod.reset_running_stats()
    cal.train()
    with torch.no_grad():
        cal(S.fog_noise(S.image_batch(4, 64, 64, seed=99), seed=98))
    run = {k: v for k, v in cal.state_dict().items()
           if k.endswith("running_mean") or k.endswith("running_var")}
    save("resunet_calib.npz", keys=np.array(list(run)),
         vals=np.concatenate([v.numpy().ravel() for v in run.values()]))
    perc_sd = S.seeded_state_dict(mans["perceptual"], seed=5)
    perc.slice.load_state_dict({k[len("slice."):]: v for k, v in perc_sd.items()})
    for H, B, tag in ((64, 2, "64"), (224, 1, "224")):
        sd = S.model_state_dict("resunet", seed=0)
        clean = S.image_batch(B, H, H, seed=30 + H)
        bad = S.fog_noise(clean, seed=40 + H)
        m = m14.ResUNet()
        m.load_state_dict(sd)
        m.eval()
        with torch.no_grad():
            out_eval = m(bad)                       # 17:84-86 (running stats)
        p = {k: v.clone() for k, v in sd.items()}
        _close(R.resunet_forward(p, bad, training=False), out_eval)
        arrays = dict(bad=bad.numpy(), clean=clean.numpy(), out_eval=out_eval.numpy())
        u8 = R.to_uint8_image(out_eval)
        cu8 = R.to_uint8_image(clean)
        arrays["out_u8"] = u8
        arrays["clean_u8"] = cu8
        arrays["psnr"] = np.array([R.psnr_u8(cu8[i], u8[i]) for i in range(B)])
        if H == 64:
            m.train()
            out_train = m(bad)                      # 14:236 (batch stats)
            p = {k: v.clone() for k, v in sd.items()}
            _close(R.resunet_forward(p, bad, training=True), out_train.detach(), 0.0)
            arrays["out_train"] = out_train.detach().numpy()
            run = {k: v for k, v in m.state_dict().items()
                   if k.endswith("running_mean") or k.endswith("running_var")}
            arrays["running_keys"] = np.array(sorted(run))
            arrays["running_vals"] = np.concatenate(
                [run[k].numpy().ravel() for k in sorted(run)])
            # one unified train step (14:235-245) from the seeded state
            m.load_state_dict(sd)
            m.train()
            opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)  # 14:222
            crit_l1 = torch.nn.L1Loss()
            opt.zero_grad()
            out = m(bad)
            l_pix = crit_l1(out, clean)
            l_perc = perc(out, clean)
            loss = l_pix + 0.1 * l_perc
            loss.backward()
            grads = {k: v.grad for k, v in m.named_parameters()}
            # restatement check of the loss and a couple of grads
            p = {k: v.clone().requires_grad_(not ("running" in k or "num_batches" in k)) for k, v in sd.items()}
            lr_ = R.unified_loss(R.resunet_forward(p, bad, True), clean, perc_sd)
            lr_.backward()
            assert abs(lr_.item() - loss.item()) < 1e-6, (lr_.item(), loss.item())
            for k in ("enc1.0.weight", "res1.conv_block.0.weight", "final.bias"):
                _close(p[k].grad, grads[k], 1e-5)
            opt.step()
            arrays["loss"] = np.array([loss.item()])
            arrays["l_pix"] = np.array([l_pix.item()])
            arrays["l_perc"] = np.array([l_perc.item()])
            arrays.update({"grad:" + k: v for k, v in digest(grads).items()})
            arrays.update({"post:" + k: v for k, v in
                           digest(dict(m.named_parameters())).items()})
            # perceptual loss alone on (bad, clean)
            with torch.no_grad():
                arrays["perc_bad_clean"] = np.array([perc(bad, clean).item()])
                _close(R.perceptual_loss(perc_sd, bad, clean),
                       perc(bad, clean), 1e-6)
        if H == 224:   # regenerated from the seeded generator; keep a checksum
            arrays["bad_sum"] = np.array([bad.double().sum().item()])
            del arrays["bad"], arrays["clean"]
        save(f"resunet_{tag}.npz", **arrays)

    # ---- VGG16 classifier (18:43-49) ------------------------------------
    vsd = S.seeded_state_dict(mans["vgg16"], seed=3)
    vgg = R.TorchvisionVGG16(43)
    vgg.load_state_dict(vsd)
    vgg.eval()
    for H, B in ((224, 8), (64, 8)):
        x = S.classifier_batch(B, H, seed=50 + H)
        with torch.no_grad():
            logits = vgg(x)
        _close(R.vgg16_forward(vsd, x), logits, 0.0)
        top2 = torch.topk(logits, 2, dim=1).values
        xin = dict(x=x.numpy()) if H == 64 else dict(x_sum=np.array([x.double().sum().item()]))
        save(f"vgg16_{H}.npz", **xin, logits=logits.numpy(),
             pred=R.top1(logits).numpy(), margin=(top2[:, 0] - top2[:, 1]).numpy())
    print("done")


def odd_sizes(m14=None):
    """ResUNet at input sizes that are not multiples of 8 (14:169-182: the
    nearest interpolate really resizes the up-conv output), B = 2:
    eval / train forward, running stats, and one unified step (L1 + 0.1
    perceptual, 14:235-245) -- loss and grad digests.  60x60: 60 -> 30 -> 15
    -> 7, up3 14 -> 15; 36x52: 36x52 -> 18x26 -> 9x13 -> 4x6, up3 8x12 -> 9x13."""
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    if m14 is None:
        _install_stubs()
        m14 = _load("14_train_unified_advanced.py", "ref14")
    mans = {n: S.load_manifest(n) for n in ("resunet", "perceptual")}
    perc = m14.VGGPerceptualLoss()
    perc_sd = S.seeded_state_dict(mans["perceptual"], seed=5)
    perc.slice.load_state_dict({k[len("slice."):]: v for k, v in perc_sd.items()})
    for H, W in ((60, 60), (36, 52)):
        B = 2
        sd = S.model_state_dict("resunet", seed=0)
        clean = S.image_batch(B, H, W, seed=70 + H + W)
        bad = S.fog_noise(clean, seed=80 + H + W)
        m = m14.ResUNet()
        m.load_state_dict(sd)
        m.eval()
        with torch.no_grad():
            out_eval = m(bad)
        _close(R.resunet_forward({k: v.clone() for k, v in sd.items()}, bad, training=False), out_eval)
        arrays = dict(bad=bad.numpy(), clean=clean.numpy(), out_eval=out_eval.numpy())
        m.train()
        opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)   # 14:222
        opt.zero_grad()
        out = m(bad)
        l_pix = torch.nn.L1Loss()(out, clean)
        l_perc = perc(out, clean)
        loss = l_pix + 0.1 * l_perc
        loss.backward()
        p = {k: v.clone().requires_grad_(not ("running" in k or "num_batches" in k))
             for k, v in sd.items()}
        out_r = R.resunet_forward(p, bad, True)
        _close(out_r.detach(), out.detach(), 0.0)
        lr_ = R.unified_loss(out_r, clean, perc_sd)
        lr_.backward()
        assert abs(lr_.item() - loss.item()) < 1e-6, (lr_.item(), loss.item())
        grads = {k: v.grad for k, v in m.named_parameters()}
        for k in ("enc1.0.weight", "up3.weight", "final.bias"):
            _close(p[k].grad, grads[k], 1e-5)
        arrays["out_train"] = out.detach().numpy()
        run = {k: v for k, v in m.state_dict().items()
               if k.endswith("running_mean") or k.endswith("running_var")}
        arrays["running_keys"] = np.array(sorted(run))
        arrays["running_vals"] = np.concatenate([run[k].numpy().ravel() for k in sorted(run)])
        arrays["loss"] = np.array([loss.item()])
        arrays.update({"grad:" + k: v for k, v in digest(grads).items()})
        save(f"resunet_{H}x{W}.npz", **arrays)


# the 08 PSNR leg: GTSRB-like original sizes (distorted input, clean image)
SIZES_08 = ((41, 47), (64, 58), (30, 33))


def _u8_image(h, w, seed):
    """A smooth synthetic road-sign-like uint8 RGB image (gradients + a disc +
    mild noise) at an original (pre-resize) size."""
    rng = np.random.Generator(np.random.PCG64([seed, 13]))
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.stack([120 + 100 * np.sin(xx / 7 + c) * np.cos(yy / 9 - c) for c in range(3)], -1)
    disc = ((yy - h / 2) ** 2 + (xx - w / 2) ** 2) < (min(h, w) / 3) ** 2
    img[disc] = [200, 30, 40]
    img += rng.normal(0, 12, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def extra(m07adv=None, m08=None):
    """Round-3 fixtures.

    simpleunet_08.npz -- the cfg2 PSNR leg of 08_run_inference.py:86-125 on
    three images of GTSRB-like original sizes: PIL Resize(224) + ToTensor of
    the distorted RGB input (08:73-76, Pillow itself), the REFERENCE
    SimpleUNet (08:19-46) forward at batch 1 in eval mode (08:92-93),
    clamp / x255 / uint8 truncation / RGB->BGR (08:96-100); the clean image
    (BGR as cv2.imread gives it) resized with cv2.resize(224, 224)
    (08:118-119) -- restated (oracle.imgproc_cpu.cv_resize_linear; cv2 is not
    installed: parity vs cv2 unpinned) -- and PSNR / SSIM (08:123-125;
    skimage restated: unpinned vs skimage).

    simpleunet_07adv.npz -- one step of the perceptual U-Net trainer
    07_train_restoration_advanced.py:143-157: the REFERENCE SimpleUNet and
    VGGPerceptualLoss (07adv:95-112, slice on the seeded cfg-D weights),
    loss = L1 + 0.1 * perceptual, Adam lr 2e-4 (07adv:19, 23, 136): loss,
    its parts, grad digests, post-Adam digests."""
    from PIL import Image
    from oracle import imgproc_cpu as I
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    if m07adv is None or m08 is None:
        _install_stubs()
        m07adv = _load("07_train_restoration_advanced.py", "ref07adv")
        m08 = _load("08_run_inference.py", "ref08")
    sd = S.model_state_dict("simpleunet", seed=0)

    # ---- 08: SimpleUNet inference + PSNR/SSIM vs the cv2-resized clean ----
    m = m08.SimpleUNet()
    m.load_state_dict(sd)
    m.eval()
    arrays, outs, cleans, ps, ss = {}, [], [], [], []
    for i, (h, w) in enumerate(SIZES_08):
        clean_rgb = _u8_image(h, w, seed=200 + i)
        rng = np.random.Generator(np.random.PCG64([300 + i, 17]))
        dist = np.clip(clean_rgb.astype(np.float64) * 0.5 + 0.9 * 255 * 0.5 +
                       rng.normal(0, 0.14 * 255, clean_rgb.shape), 0, 255).astype(np.uint8)
        pil = Image.fromarray(dist, "RGB").resize((224, 224), Image.BILINEAR)   # Resize((224,224))
        x = torch.from_numpy(np.asarray(pil).copy()).permute(2, 0, 1).float().div(255)  # ToTensor
        with torch.no_grad():
            out = m(x.unsqueeze(0))                                               # 08:92-93
        _close(R.simple_unet_forward({k: v.clone() for k, v in sd.items()}, x.unsqueeze(0)), out)
        o = torch.clamp(out, 0, 1).squeeze().permute(1, 2, 0).numpy()            # 08:96-97
        out_bgr = np.ascontiguousarray((o * 255).astype(np.uint8)[:, :, ::-1])   # 08:98-100
        clean_bgr = np.ascontiguousarray(clean_rgb[:, :, ::-1])                  # cv2.imread
        clean224 = I.cv_resize_linear(clean_bgr, 224, 224)                       # 08:119
        arrays[f"dist_{i}"] = dist
        arrays[f"clean_bgr_{i}"] = clean_bgr
        arrays[f"out_sum_{i}"] = np.array([out.double().sum().item()])
        outs.append(out_bgr)
        cleans.append(clean224)
        ps.append(R.psnr_u8(clean224, out_bgr))                                  # 08:123
        ss.append(I.ssim(clean224, out_bgr))                                     # 08:125
    arrays.update(out_bgr=np.stack(outs), clean224=np.stack(cleans), psnr=np.array(ps),
                  ssim=np.array(ss), sizes=np.array(SIZES_08))
    save("simpleunet_08.npz", **arrays)
    print("08 leg: PSNR", ps, "SSIM", ss)

    # ---- 07adv: SimpleUNet + L1 + 0.1 perceptual, Adam lr 2e-4 -------------
    man = S.load_manifest("perceptual")
    perc_sd = S.seeded_state_dict(man, seed=5)
    perc = m07adv.VGGPerceptualLoss()
    perc.slice.load_state_dict({k[len("slice."):]: v for k, v in perc_sd.items()})
    assert [[k, list(v.shape)] for k, v in perc.state_dict().items()] == man
    B, H = 2, 64
    clean = S.image_batch(B, H, H, seed=400)
    bad = S.fog_noise(clean, seed=401)
    m = m07adv.SimpleUNet()
    m.load_state_dict(sd)
    m.train()
    opt = torch.optim.Adam(m.parameters(), lr=m07adv.LEARNING_RATE)          # 07adv:136
    opt.zero_grad()
    out = m(bad)                                                              # 07adv:147
    l_pix = torch.nn.L1Loss()(out, clean)                                     # 07adv:150
    l_perc = perc(out, clean)                                                 # 07adv:151
    loss = l_pix + m07adv.LAMBDA_PERCEPTUAL * l_perc                          # 07adv:154
    loss.backward()
    grads = {k: v.grad for k, v in m.named_parameters()}
    p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    lr_ = R.unified_loss(R.simple_unet_forward(p, bad), clean, perc_sd)
    lr_.backward()
    assert abs(lr_.item() - loss.item()) < 1e-6, (lr_.item(), loss.item())
    for k in ("enc1.0.weight", "up1.weight", "final.bias"):
        _close(p[k].grad, grads[k], 1e-5)
    opt.step()
    save("simpleunet_07adv.npz", bad=bad.numpy(), clean=clean.numpy(),
         loss=np.array([loss.item()]), l_pix=np.array([l_pix.item()]),
         l_perc=np.array([l_perc.item()]), lr=np.array([m07adv.LEARNING_RATE]),
         **{"grad:" + k: v for k, v in digest(grads).items()},
         **{"post:" + k: v for k, v in digest(dict(m.named_parameters())).items()})
    print("07adv step: loss", loss.item())


if __name__ == "__main__":
    if "--only-odd" in sys.argv:
        odd_sizes()
    elif "--only-extra" in sys.argv:
        extra()
    else:
        main()
        odd_sizes()
        extra()
