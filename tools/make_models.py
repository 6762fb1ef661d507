"""Build-defined model1/model2/model3 directories with seeded weights.

The real Cacophony CNNs are a Docker-time download (reference Dockerfile:33-37)
and are not in the tree, so this build defines the family:

    [magtransform]  (optional, only meaningful with db_scale=false)
    conv 3x3  ->32  BN LReLU     conv 3x3 ->32 BN LReLU    maxpool 3x3
    conv 3x3  ->64  BN LReLU     conv 3x3 ->64 BN LReLU
    conv 9x3  ->128 BN LReLU     maxpool 3x3
    conv 1x3  ->256 BN LReLU     conv 1x1 ->L (+bias)
    global max pool, sigmoid                      (all convs padding="valid")

Each directory mirrors the reference's model contract
(src/identify_tracks.py:291-299, src/analyse.py:414-418):
``<dir>/audioModel.safetensors`` (weights + ``__metadata__["arch"]``, taking the
place of ``audioModel.keras``) and ``<dir>/metadata.txt`` (front-end + label
JSON, same keys the reference reads at :466-497).

BatchNorm moving statistics are set from a calibration pass over dB-like
inputs, so activations stay O(1) like a trained network's; the final bias is
chosen so that some labels clear the 0.7 threshold.  Model creation is a
one-off tool, not part of the inference path.
"""
from __future__ import annotations

import json
import os
from pathlib import Path

import numpy as np

LABELS = [
    "bellbird", "bird", "fantail", "grey warbler", "human", "insect", "kea", "kiwi",
    "morepork", "noise", "robin", "saddleback", "silvereye", "sparrow", "song thrush",
    "tomtit", "tui", "whistler", "kaka", "weka", "blackbird", "chaffinch",
    "yellowhammer", "kokako",
]
EBIRD = {
    "bellbird": ["nezbel1"], "fantail": ["nezfan1"], "grey warbler": ["grywar1"],
    "kea": ["kea1"], "kiwi": ["nibkiw1", "liskiw1"], "morepork": ["morepo2"],
    "robin": ["nezrob2"], "saddleback": ["saddle2"], "silvereye": ["silver3"],
    "sparrow": ["houspa"], "song thrush": ["sonthr1"], "tomtit": ["tomtit1"],
    "tui": ["tui1"], "whistler": ["whiteh1"], "kaka": ["nezkak1"], "weka": ["weka1"],
    "blackbird": ["eurbla"], "chaffinch": ["comcha"], "yellowhammer": ["yellow2"],
    "kokako": ["kokako3"],
}

DEFAULT_META = {
    "segment_length": 3,
    "segment_stride": 1.5,
    "hop_length": 640,
    "n_fft": 4096,
    "n_mels": 160,
    "fmin": 50,
    "fmax": 11000,
    "break_freq": 1750,
    "htk": True,
    "power": 2,
    "db_scale": True,
    "normalize": True,
    "threshold": 0.7,
    "multi_label": True,
}


def arch_layers(widths=(32, 32, 64, 64, 128, 256), n_labels=len(LABELS), mag=None,
                alpha=0.3):
    c1, c2, c3, c4, c5, c6 = widths
    L = []
    if mag is not None:
        L.append({"type": "magtransform", "name": "mag", "version": int(mag)})
    def block(i, f, k):
        L.append({"type": "conv2d", "name": f"conv{i}", "filters": f, "kernel": list(k),
                  "use_bias": False})
        L.append({"type": "batchnorm", "name": f"bn{i}", "eps": 1e-3})
        L.append({"type": "leakyrelu", "alpha": alpha})
    block(1, c1, (3, 3))
    block(2, c2, (3, 3))
    L.append({"type": "maxpool2d", "pool": [3, 3]})
    block(3, c3, (3, 3))
    block(4, c4, (3, 3))
    block(5, c5, (9, 3))
    L.append({"type": "maxpool2d", "pool": [3, 3]})
    block(6, c6, (1, 3))
    L.append({"type": "conv2d", "name": "conv7", "filters": n_labels, "kernel": [1, 1],
              "use_bias": True})
    L.append({"type": "globalmaxpool2d"})
    L.append({"type": "activation", "fn": "sigmoid"})
    return L


def _init_weights(arch, in_ch, rng):
    import torch
    tensors = {}
    cin = in_ch
    for layer in arch:
        if layer["type"] == "magtransform":
            a0 = 0.0 if layer["version"] == 1 else -1.0
            shape = () if layer["version"] == 1 else (1,)
            tensors["mag.a"] = np.asarray(a0 + rng.uniform(-0.2, 0.2), np.float32).reshape(shape)
        elif layer["type"] == "conv2d":
            kh, kw = layer["kernel"]
            f = layer["filters"]
            std = np.sqrt(2.0 / (kh * kw * cin))
            tensors[layer["name"] + ".kernel"] = (rng.standard_normal((kh, kw, cin, f)) * std).astype(np.float32)
            if layer.get("use_bias"):
                tensors[layer["name"] + ".bias"] = (rng.standard_normal(f) * 0.1).astype(np.float32)
            cin = f
        elif layer["type"] == "batchnorm":
            tensors[layer["name"] + ".gamma"] = rng.uniform(0.7, 1.3, cin).astype(np.float32)
            tensors[layer["name"] + ".beta"] = rng.normal(0.0, 0.2, cin).astype(np.float32)
            tensors[layer["name"] + ".moving_mean"] = np.zeros(cin, np.float32)
            tensors[layer["name"] + ".moving_variance"] = np.ones(cin, np.float32)
    return tensors


def _calibrate(arch, tensors, x, rng):
    """Set BN moving stats to the calibration batch statistics and centre the
    final logits, layer by layer (torch CPU)."""
    import torch
    import torch.nn.functional as F
    t = lambda k: torch.from_numpy(tensors[k])
    h = torch.from_numpy(x).permute(0, 3, 1, 2).double()
    for i, layer in enumerate(arch):
        kind = layer["type"]
        if kind == "magtransform":
            h = torch.pow(h, torch.sigmoid(t("mag.a").double().reshape(-1)[0]))
        elif kind == "conv2d":
            w = t(layer["name"] + ".kernel").double().permute(3, 2, 0, 1)
            b = t(layer["name"] + ".bias").double() if layer.get("use_bias") else None
            h = F.conv2d(h, w, b)
        elif kind == "batchnorm":
            n = layer["name"]
            mu = h.mean(dim=(0, 2, 3))
            var = h.var(dim=(0, 2, 3), unbiased=False)
            tensors[n + ".moving_mean"] = mu.float().numpy()
            tensors[n + ".moving_variance"] = var.float().numpy()
            g, be = t(n + ".gamma").double(), t(n + ".beta").double()
            h = (h - mu[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + layer["eps"])
            h = h * g[None, :, None, None] + be[None, :, None, None]
        elif kind == "leakyrelu":
            h = F.leaky_relu(h, layer["alpha"])
        elif kind == "maxpool2d":
            h = F.max_pool2d(h, layer["pool"], layer["pool"])
        elif kind == "globalmaxpool2d":
            h = torch.amax(h, dim=(2, 3))
            # centre each label's logit, then give it a random offset so a few
            # labels clear the threshold on typical inputs
            last = [l for l in arch if l["type"] == "conv2d"][-1]["name"]
            shift = h.mean(dim=0) - torch.from_numpy(rng.normal(-0.8, 1.2, h.shape[1]))
            tensors[last + ".bias"] = (t(last + ".bias").double() - shift).float().numpy()
            h = h - shift
    return tensors


def calibration_input(n, n_mels, T, db_scale, rng):
    """dB-like inputs (or positive magnitudes when db_scale is false)."""
    base = rng.normal(-45.0, 10.0, size=(n, n_mels, 1, 1))
    x = base + rng.normal(0.0, 8.0, size=(n, n_mels, T, 1))
    x = np.clip(x, -80.0, 0.0)
    if not db_scale:
        x = 10.0 ** (x / 20.0)
    return x.astype(np.float32)


def make_chain(out_dir, blocks, seed=1, n_mels=160, T=226, alpha=0.3):
    """A conv chain ending in GlobalMaxPool2D (no 1x1 head): ``blocks`` =
    [(filters, (kh, kw), pool or None), ...], each conv + BN + LeakyReLU
    [+ MaxPooling2D]; the last conv carries the bias the calibration centres.
    For layer-by-layer checks of single conv kernels (tests/)."""
    from safetensors.numpy import save_file
    arch = []
    for i, (f, k, pool) in enumerate(blocks, 1):
        arch.append({"type": "conv2d", "name": f"conv{i}", "filters": f, "kernel": list(k),
                     "use_bias": i == len(blocks)})
        arch.append({"type": "batchnorm", "name": f"bn{i}", "eps": 1e-3})
        arch.append({"type": "leakyrelu", "alpha": alpha})
        if pool:
            arch.append({"type": "maxpool2d", "pool": list(pool)})
    arch.append({"type": "globalmaxpool2d"})
    rng = np.random.default_rng(seed)
    tensors = _init_weights(arch, 1, rng)
    tensors = _calibrate(arch, tensors, calibration_input(4, n_mels, T, True, rng), rng)
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    save_file({k: np.ascontiguousarray(v) for k, v in tensors.items()},
              str(out / "audioModel.safetensors"), metadata={"arch": json.dumps(arch)})
    meta = dict(DEFAULT_META)
    meta.update({"name": "chain", "labels": [f"c{i}" for i in range(blocks[-1][0])]})
    with open(out / "metadata.txt", "w") as f:
        json.dump(meta, f, indent=2)
    return out / "audioModel.safetensors"


def make_model(out_dir, name="model1", seed=1, widths=(32, 32, 64, 64, 128, 256),
               labels=None, mag=None, meta_overrides=None, pre_model=False, in_channels=None):
    """Create ``out_dir/audioModel.safetensors`` + ``out_dir/metadata.txt``.
    ``in_channels`` overrides the input channels (default: meta channels),
    e.g. 3 for an "efficientnet"-named model fed the repeated log-mel."""
    from safetensors.numpy import save_file
    labels = list(labels or LABELS)
    meta = dict(DEFAULT_META)
    if mag is not None:
        meta["db_scale"] = False
        meta["magv2"] = (int(mag) == 2)
    meta.update(meta_overrides or {})
    meta.update({
        "name": name,
        "labels": labels,
        "ebird_ids": [EBIRD.get(l, []) for l in labels],
        "pre_model": bool(pre_model),
    })
    rng = np.random.default_rng(seed)
    arch = arch_layers(widths, len(labels), mag)
    channels = int(in_channels or meta.get("channels", 1))
    tensors = _init_weights(arch, channels, rng)
    T = 1 + int(meta["segment_length"] * 48000) // int(meta["hop_length"])
    x = calibration_input(6, int(meta["n_mels"]), T, bool(meta["db_scale"]), rng)
    if channels > 1:
        x = np.repeat(x, channels, axis=3)
    tensors = _calibrate(arch, tensors, x, rng)
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    save_file({k: np.ascontiguousarray(v) for k, v in tensors.items()},
              str(out / "audioModel.safetensors"), metadata={"arch": json.dumps(arch)})
    with open(out / "metadata.txt", "w") as f:
        json.dump(meta, f, indent=2)
    return out / "audioModel.safetensors"


ENSEMBLE = {
    "model1": dict(seed=1),
    "model2": dict(seed=2),
    "model3": dict(seed=3),
}


def make_ensemble(root, names=("model1", "model2", "model3"), **kw):
    """Create the three-model ensemble under ``root``; returns model paths."""
    paths = []
    for n in names:
        d = Path(root) / n
        p = d / "audioModel.safetensors"
        if not (p.exists() and (d / "metadata.txt").exists()):
            make_model(d, name=n, **ENSEMBLE[n], **kw)
        paths.append(p)
    return paths


if __name__ == "__main__":
    import sys
    root = sys.argv[1] if len(sys.argv) > 1 else "models"
    for p in make_ensemble(root):
        print(p)
