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


def graph_arch(kind="effnet", n_labels=len(LABELS)):
    """Keras-Functional-style archs for the graph executor (aa_amd.graph):
    "effnet": an EfficientNet-like stem + three MBConv blocks (depthwise conv,
    squeeze-and-excite, residual add, ZeroPadding2D + valid stride-2 conv,
    swish) + head, global average pooling, Dense + sigmoid;
    "resnet": Rescaling + Normalization, "same" stride-2 convs, ReLU, max /
    average pools, a residual add, GlobalAveragePooling2D, Dense."""
    L = []

    def add(d):
        L.append(d)
        return d["name"]

    def bn(x, n):
        return add({"type": "batchnorm", "name": n, "eps": 1e-3, "inputs": [x]})

    def act(x, n, fn="swish"):
        return add({"type": "activation", "name": n, "fn": fn, "inputs": [x]})

    def conv(x, n, f, k, s=1, pad="same", bias=False, activation=None):
        d = {"type": "conv2d", "name": n, "filters": f, "kernel": list(k), "strides": [s, s], "padding": pad,
             "use_bias": bias, "inputs": [x]}
        if activation:
            d["activation"] = activation
        return add(d)

    def dw(x, n, k, s=1, pad="same"):
        return add({"type": "depthwise_conv2d", "name": n, "kernel": [k, k], "strides": [s, s], "padding": pad,
                    "use_bias": False, "inputs": [x]})

    def se(x, n, c, r):
        g = add({"type": "globalavgpool2d", "name": n + "_squeeze", "inputs": [x]})
        g = add({"type": "reshape", "name": n + "_reshape", "target": [1, 1, c], "inputs": [g]})
        g = conv(g, n + "_reduce", r, (1, 1), bias=True, activation="swish")
        g = conv(g, n + "_expand", c, (1, 1), bias=True, activation="sigmoid")
        return add({"type": "multiply", "name": n + "_excite", "inputs": [x, g]})

    if kind == "effnet":
        x = conv("input", "stem_conv", 32, (3, 3), s=2)
        x = act(bn(x, "stem_bn"), "stem_act")
        # block 1: depthwise 3x3, SE, project (no expansion)
        y = act(bn(dw(x, "b1_dw", 3), "b1_bn"), "b1_act")
        y = se(y, "b1_se", 32, 8)
        y = bn(conv(y, "b1_project", 16, (1, 1)), "b1_project_bn")
        y = add({"type": "maxpool2d", "name": "b1_pool", "pool": [3, 3], "strides": [1, 1], "padding": "same",
                 "inputs": [y]})
        # block 2: expand x4, ZeroPadding2D + valid 5x5 stride 2 (keras correct_pad), SE, project
        z = act(bn(conv(y, "b2_expand", 64, (1, 1)), "b2_expand_bn"), "b2_expand_act")
        z = add({"type": "zeropad2d", "name": "b2_pad", "pad": [[1, 2], [1, 2]], "inputs": [z]})
        z = act(bn(dw(z, "b2_dw", 5, s=2, pad="valid"), "b2_bn"), "b2_act")
        z = se(z, "b2_se", 64, 4)
        z = bn(conv(z, "b2_project", 24, (1, 1)), "b2_project_bn")
        # block 3: expand x4, depthwise 3x3, SE, project, dropout, residual add
        u = act(bn(conv(z, "b3_expand", 96, (1, 1)), "b3_expand_bn"), "b3_expand_act")
        u = act(bn(dw(u, "b3_dw", 3), "b3_bn"), "b3_act")
        u = se(u, "b3_se", 96, 6)
        u = bn(conv(u, "b3_project", 24, (1, 1)), "b3_project_bn")
        u = add({"type": "dropout", "name": "b3_drop", "inputs": [u]})
        u = add({"type": "add", "name": "b3_add", "inputs": [u, z]})
        h = act(bn(conv(u, "top_conv", 64, (1, 1)), "top_bn"), "top_act")
        h = add({"type": "globalavgpool2d", "name": "avg_pool", "inputs": [h]})
        h = add({"type": "dropout", "name": "top_dropout", "inputs": [h]})
        add({"type": "dense", "name": "predictions", "units": n_labels, "use_bias": True, "activation": "sigmoid",
             "inputs": [h]})
    elif kind == "effnetv2":
        # EfficientNetV2-B0's block table (Keras applications): stem 3x3/2 -> 32,
        # Fused-MBConv (expand conv 3x3 + project 1x1; no SE) x (1, 2, 2),
        # MBConv (expand 1x1, depthwise 3x3, SE 0.25 of the block input, project)
        # x (3, 5, 8), residual adds where stride 1 and widths match, head 1x1
        # -> 1280, global average pooling, Dense + sigmoid
        def fused(x, n, cin, cout, e, s):
            if e == 1:
                y = act(bn(conv(x, n + "_conv", cout, (3, 3), s=s), n + "_bn"), n + "_act")
            else:
                y = act(bn(conv(x, n + "_expand", cin * e, (3, 3), s=s), n + "_expand_bn"), n + "_expand_act")
                y = bn(conv(y, n + "_project", cout, (1, 1)), n + "_project_bn")
            if s == 1 and cin == cout:
                y = add({"type": "add", "name": n + "_add", "inputs": [y, x]})
            return y

        def mb(x, n, cin, cout, e, s):
            y = act(bn(conv(x, n + "_expand", cin * e, (1, 1)), n + "_expand_bn"), n + "_expand_act")
            y = act(bn(dw(y, n + "_dw", 3, s), n + "_bn"), n + "_act")
            y = se(y, n + "_se", cin * e, max(1, int(cin * 0.25)))
            y = bn(conv(y, n + "_project", cout, (1, 1)), n + "_project_bn")
            if s == 1 and cin == cout:
                y = add({"type": "add", "name": n + "_add", "inputs": [y, x]})
            return y

        x = act(bn(conv("input", "stem_conv", 32, (3, 3), s=2), "stem_bn"), "stem_act")
        table = [("f", 1, 3, 1, 32, 16, 1), ("f", 4, 3, 2, 16, 32, 2), ("f", 4, 3, 2, 32, 48, 2),
                 ("m", 4, 3, 2, 48, 96, 3), ("m", 6, 3, 1, 96, 112, 5), ("m", 6, 3, 2, 112, 192, 8)]
        for si, (typ, e, k, s, cin, cout, reps) in enumerate(table):
            for r in range(reps):
                n = f"block{si + 1}{chr(ord('a') + r)}"
                x = (fused if typ == "f" else mb)(x, n, cin if r == 0 else cout, cout, e, s if r == 0 else 1)
        h = act(bn(conv(x, "top_conv", 1280, (1, 1)), "top_bn"), "top_act")
        h = add({"type": "globalavgpool2d", "name": "avg_pool", "inputs": [h]})
        add({"type": "dense", "name": "predictions", "units": n_labels, "use_bias": True, "activation": "sigmoid",
             "inputs": [h]})
    elif kind == "resnet":
        x = add({"type": "rescaling", "name": "rescale", "scale": 1.0 / 80.0, "offset": 1.0, "inputs": ["input"]})
        x = add({"type": "normalization", "name": "norm", "inputs": [x]})
        x = conv(x, "conv1", 24, (5, 5), s=2, bias=True)
        x = add({"type": "relu", "name": "relu1", "inputs": [bn(x, "bn1")]})
        x = add({"type": "maxpool2d", "name": "pool1", "pool": [3, 3], "strides": [2, 2], "padding": "same",
                 "inputs": [x]})
        y = conv(x, "conv2a", 24, (3, 3), bias=False)
        y = add({"type": "relu", "name": "relu2a", "inputs": [bn(y, "bn2a")]})
        y = bn(conv(y, "conv2b", 24, (3, 3)), "bn2b")
        y = add({"type": "add", "name": "res2", "inputs": [x, y]})
        y = add({"type": "relu", "name": "relu2", "inputs": [y]})
        y = add({"type": "avgpool2d", "name": "pool2", "pool": [3, 3], "strides": [2, 2], "padding": "same",
                 "inputs": [y]})
        y = conv(y, "conv3", 48, (3, 1), s=2, bias=True, activation="relu")
        y = add({"type": "globalavgpool2d", "name": "gap", "inputs": [y]})
        add({"type": "dense", "name": "fc", "units": n_labels, "use_bias": True, "inputs": [y]})
        add({"type": "activation", "name": "out", "fn": "sigmoid", "inputs": ["fc"]})
    else:
        raise ValueError(kind)
    return L


def _graph_weights(arch, in_ch, rng):
    shapes = {"input": in_ch}
    tensors = {}
    for ly in arch:
        src = (ly.get("inputs") or ["input"])[0]
        c = shapes[src]
        n, kind = ly["name"], ly["type"]
        if kind == "conv2d":
            kh, kw = ly["kernel"]
            f = ly["filters"]
            tensors[n + ".kernel"] = (rng.standard_normal((kh, kw, c, f)) * np.sqrt(2.0 / (kh * kw * c))).astype(np.float32)
            if ly.get("use_bias"):
                tensors[n + ".bias"] = (rng.standard_normal(f) * 0.1).astype(np.float32)
            c = f
        elif kind == "depthwise_conv2d":
            kh, kw = ly["kernel"]
            tensors[n + ".kernel"] = (rng.standard_normal((kh, kw, c, 1)) * np.sqrt(2.0 / (kh * kw))).astype(np.float32)
        elif kind == "batchnorm":
            tensors[n + ".gamma"] = rng.uniform(0.7, 1.3, c).astype(np.float32)
            tensors[n + ".beta"] = rng.normal(0.0, 0.2, c).astype(np.float32)
            tensors[n + ".moving_mean"] = np.zeros(c, np.float32)
            tensors[n + ".moving_variance"] = np.ones(c, np.float32)
        elif kind == "normalization":
            tensors[n + ".mean"] = np.full(c, 0.45, np.float32)
            tensors[n + ".variance"] = np.full(c, 0.04, np.float32)
        elif kind == "dense":
            tensors[n + ".kernel"] = (rng.standard_normal((c, ly["units"])) * np.sqrt(1.0 / c)).astype(np.float32)
            tensors[n + ".bias"] = np.zeros(ly["units"], np.float32)
            c = ly["units"]
        shapes[n] = c
    return tensors


def make_graph(out_dir, kind="effnet", name=None, seed=1, in_channels=1, n_mels=160, T=226, labels=None,
               meta_overrides=None, calib=None, arch=None):
    """A graph model (graph_arch) with seeded weights, BatchNormalization
    statistics calibrated layer by layer on dB-like inputs (float64, through
    the oracle's graph semantics) and centred logits; writes
    audioModel.safetensors + metadata.txt like make_model.  ``calib``
    ([N][n_mels][T][C] log-mels, e.g. the front end's output on the inputs
    the model will see) replaces the synthetic dB-like calibration input: a
    deep network whose statistics were taken on another input distribution
    amplifies its activations layer after layer (logits in the thousands),
    which no trained network does.  ``arch`` (a graph_arch-style layer list
    ending in a Dense) replaces the named ``kind``."""
    import torch
    from safetensors.numpy import save_file
    from oracle.cnn_oracle import _forward_graph
    labels = list(labels or LABELS)
    arch = arch if arch is not None else graph_arch(kind, len(labels))
    rng = np.random.default_rng(seed)
    tensors = _graph_weights(arch, in_channels, rng)
    # (BatchNorm statistics are per channel: a deep network calibrates on a
    # shorter excerpt, each BN needs a forward of everything before it)
    if calib is not None:
        x = np.asarray(calib, np.float32)[:, :, :T]  # full windows: a crop's statistics do not carry over
        if x.shape[3] != in_channels:
            x = np.repeat(x[..., :1], in_channels, axis=3)
    else:
        x = calibration_input(6 if len(arch) < 80 else 3, n_mels, T if len(arch) < 80 else min(T, 160), True, rng)
        if in_channels > 1:
            x = np.repeat(x, in_channels, axis=3)
    xt = torch.from_numpy(x).double().permute(0, 3, 1, 2)
    for i, ly in enumerate(arch):
        if ly["type"] != "batchnorm":
            continue
        outs = {}
        _forward_graph(arch[:i], tensors, xt, torch.float64, capture=outs)
        h = outs[ly["inputs"][0]]
        tensors[ly["name"] + ".moving_mean"] = h.mean(dim=(0, 2, 3)).float().numpy()
        tensors[ly["name"] + ".moving_variance"] = h.var(dim=(0, 2, 3), unbiased=False).float().numpy()
    dense = [ly for ly in arch if ly["type"] == "dense"][-1]["name"]
    lg, _ = _forward_graph(arch, tensors, xt, torch.float64)
    if calib is not None:
        # logits of a trained classifier's scale (a few units): the Dense kernel
        # rescaled to a spread of about 2 on the calibration windows
        sd = float(np.std(lg - lg.mean(axis=0)))
        if sd > 2.0:
            tensors[dense + ".kernel"] = (tensors[dense + ".kernel"] * (2.0 / sd)).astype(np.float32)
            lg, _ = _forward_graph(arch, tensors, xt, torch.float64)
    shift = lg.mean(axis=0) - rng.normal(-0.8, 1.2, lg.shape[1])
    tensors[dense + ".bias"] = (tensors[dense + ".bias"] - shift).astype(np.float32)
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    save_file({k: np.ascontiguousarray(v) for k, v in tensors.items()},
              str(out / "audioModel.safetensors"), metadata={"arch": json.dumps(arch)})
    meta = dict(DEFAULT_META)
    meta.update({"name": name or f"{kind}-graph", "labels": labels,
                 "ebird_ids": [EBIRD.get(l, []) for l in labels], "channels": in_channels})
    meta.update(meta_overrides or {})
    with open(out / "metadata.txt", "w") as f:
        json.dump(meta, f, indent=2)
    return out / "audioModel.safetensors"
