"""Seeded synthetic weights and inputs -- TEST INFRASTRUCTURE ONLY.

The reference's trained checkpoints are absent (.MISSING_LARGE_BLOBS:1-4) and
its ImageNet VGG16 weights are a network download (14:192), so every parity
case runs on seeded synthetic weights laid out in the reference's state_dict
key tree (manifests in tests/golden/manifest_*.json).  numpy PCG64 streams
keyed by (seed, key index) make the tensors identical on every machine.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import torch

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                          "tests", "golden")


def load_manifest(name):
    with open(os.path.join(GOLDEN_DIR, f"manifest_{name}.json")) as f:
        return json.load(f)   # [[key, [shape...]], ...] in state_dict order


def _kind(key):
    return key.rsplit(".", 1)[-1]


def seeded_state_dict(manifest, seed=0, module_kinds=None):
    """Build a state_dict for ``manifest``.

    Conv / linear weights: He-uniform U(-sqrt(6/fan_in), +) so activations stay
    O(1) through the deep stacks (meaningful absolute tolerances); biases
    U(-0.1, 0.1); BN gamma U(0.5, 1.5), beta U(-0.2, 0.2), running_mean
    U(-0.2, 0.2), running_var U(0.5, 1.5); PReLU alpha 0.25 + U(-0.05, 0.05).
    ``module_kinds`` maps a module prefix to "bn" / "prelu" / "conv" / "convT";
    by default it is inferred from shapes and key names.
    """
    sd = {}
    kinds = dict(module_kinds or {})
    keys = {k for k, _ in manifest}
    for key, shape in manifest:
        prefix, leaf = key.rsplit(".", 1)
        if prefix in kinds:
            continue
        if prefix + ".running_mean" in keys:
            kinds[prefix] = "bn"
        elif leaf == "weight" and list(shape) == [1] and prefix + ".bias" not in keys:
            kinds[prefix] = "prelu"
    for idx, (key, shape) in enumerate(manifest):
        rng = np.random.Generator(np.random.PCG64([seed, idx]))
        prefix, leaf = key.rsplit(".", 1)
        mk = kinds.get(prefix)
        shape = tuple(shape)
        if leaf == "num_batches_tracked":
            sd[key] = torch.zeros((), dtype=torch.long)
            continue
        if mk is None:
            if leaf in ("running_mean", "running_var"):
                mk = "bn"
            elif len(shape) == 1 and shape == (1,):
                mk = "prelu"
            elif leaf == "weight" and len(shape) == 1:
                mk = "bn"
            else:
                mk = "conv"
        if mk == "prelu":
            a = 0.25 + rng.uniform(-0.05, 0.05, size=shape)
        elif mk == "bn":
            lo, hi = {"weight": (0.5, 1.5), "bias": (-0.2, 0.2),
                      "running_mean": (-0.2, 0.2), "running_var": (0.5, 1.5)}[leaf]
            a = rng.uniform(lo, hi, size=shape)
        else:  # conv / convT / linear
            if leaf == "weight":
                if mk == "convT":           # [Cin, Cout, kh, kw]: fan_in seen by an output
                    fan_in = shape[0] * int(np.prod(shape[2:]))
                else:                       # [Cout, Cin, kh, kw] / [out, in]
                    fan_in = int(np.prod(shape[1:]))
                b = math.sqrt(6.0 / fan_in)
                a = rng.uniform(-b, b, size=shape)
            else:
                a = rng.uniform(-0.1, 0.1, size=shape)
        sd[key] = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    return sd


def convT_prefixes(manifest):
    """Module prefixes whose weights are ConvTranspose2d ([Cin, Cout, 2, 2])."""
    out = {}
    for key, shape in manifest:
        prefix, leaf = key.rsplit(".", 1)
        if leaf == "weight" and len(shape) == 4 and shape[2:] == [2, 2]:
            out[prefix] = "convT"
    return out


def model_state_dict(name, seed=0):
    """Seeded state_dict of a reference model; for ResUNet the BN running stats
    are replaced by the committed calibration (tests/golden/resunet_calib.npz)."""
    man = load_manifest(name)
    sd = seeded_state_dict(man, seed, convT_prefixes(man))
    cal = os.path.join(GOLDEN_DIR, f"{name}_calib.npz")
    if seed == 0 and os.path.exists(cal):
        z = np.load(cal)
        off = 0
        for k in z["keys"]:
            k = str(k)
            n = sd[k].numel()
            sd[k] = torch.from_numpy(z["vals"][off:off + n].reshape(sd[k].shape).copy())
            off += n
    return sd


def image_batch(n, h, w, seed=0):
    """ToTensor semantics: uint8 U{0..255} / 255, NCHW float32."""
    rng = np.random.Generator(np.random.PCG64([seed, 7]))
    u8 = rng.integers(0, 256, size=(n, 3, h, w), dtype=np.uint8)
    return torch.from_numpy(u8.astype(np.float32) / 255.0)


def fog_noise(clean, seed=1, t=0.5, A=0.9, var=0.02):
    """Synthetic distorted input: clip(clean*t + A(1-t) + N(0, var), 0, 1)
    (the fog + noise subset of 16_gen_compound_data.py:29-35)."""
    rng = np.random.Generator(np.random.PCG64([seed, 11]))
    noise = rng.normal(0.0, math.sqrt(var), size=tuple(clean.shape)).astype(np.float32)
    return torch.clamp(clean * t + A * (1 - t) + torch.from_numpy(noise), 0, 1)


def classifier_batch(n, h, seed=0):
    """ImageNet-normalised images (18:28-32) with a per-image contrast/brightness
    sweep so the seeded VGG16 head does not predict one class for every image."""
    x = imagenet_normalize(image_batch(n, h, h, seed=seed))
    return x * torch.linspace(0.5, 2.0, n).view(n, 1, 1, 1) + \
        torch.linspace(-1.0, 1.0, n).view(n, 1, 1, 1)


IMAGENET_MEAN = (0.485, 0.456, 0.406)   # 18:31
IMAGENET_STD = (0.229, 0.224, 0.225)


def imagenet_normalize(x):
    m = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    s = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    return (x - m) / s
