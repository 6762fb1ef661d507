"""CPU fp32 oracle for the window classifier CNN.  TEST INFRASTRUCTURE ONLY.

Reference call site: ``model.predict(np.array(d))`` at
src/identify_tracks.py:544 (Keras / TF 2.19 on CPU), input ``[W, n_mels, T, C]``
(NHWC, produced by ``get_spect`` :267), output ``[W, n_labels]``.  The real
Cacophony weights/architecture are a Docker-time download (Dockerfile:33-37)
and TF is not installed, so the model family is defined by this build
 and stored as ``audioModel.safetensors`` whose
``__metadata__["arch"]`` is a Keras-style layer list.  This oracle evaluates
that layer list literally, un-fused, in torch-CPU float32 (or float64):

* ``magtransform``  -> ``x ** sigmoid(a)``   src/magtransform.py:17-19,
  src/magtransformv2.py:19-21
* ``conv2d``        -> Keras Conv2D, padding="valid", stride 1, HWIO kernel
* ``batchnorm``     -> inference BN with moving statistics (not folded)
* ``leakyrelu``     -> max(x, alpha*x)
* ``maxpool2d``     -> Keras MaxPooling2D(pool), strides = pool, valid (floor)
* ``globalmaxpool2d`` -> max over H, W
* ``activation``    -> sigmoid

``logits`` are the GlobalMaxPool outputs before the final sigmoid.
"""
from __future__ import annotations

import json

import numpy as np
import torch
import torch.nn.functional as F
from safetensors.numpy import load_file
from safetensors import safe_open


def load_arch(path):
    with safe_open(str(path), framework="np") as f:
        meta = f.metadata()
    return json.loads(meta["arch"]), load_file(str(path))


@torch.no_grad()
def forward(path_or_arch, x_nhwc: np.ndarray, dtype=torch.float32, tensors=None):
    """Run the CNN on ``x_nhwc`` [W, H, T, C]; returns (logits, probs) numpy."""
    if tensors is None:
        arch, tensors = load_arch(path_or_arch)
    else:
        arch = path_or_arch
    t = lambda k: torch.from_numpy(np.asarray(tensors[k])).to(dtype)
    x = torch.from_numpy(np.ascontiguousarray(x_nhwc)).to(dtype).permute(0, 3, 1, 2)
    logits = None
    for layer in arch:
        kind = layer["type"]
        name = layer.get("name")
        if kind == "magtransform":
            a = t(name + ".a").reshape(-1)[0]
            x = torch.pow(x, torch.sigmoid(a))
        elif kind == "conv2d":
            w = t(name + ".kernel").permute(3, 2, 0, 1)  # HWIO -> OIHW
            b = t(name + ".bias") if layer.get("use_bias", False) else None
            x = F.conv2d(x, w, b)
        elif kind == "batchnorm":
            g, be = t(name + ".gamma"), t(name + ".beta")
            mu, var = t(name + ".moving_mean"), t(name + ".moving_variance")
            eps = float(layer.get("eps", 1e-3))
            x = (x - mu[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + eps)
            x = x * g[None, :, None, None] + be[None, :, None, None]
        elif kind == "leakyrelu":
            x = F.leaky_relu(x, float(layer.get("alpha", 0.3)))
        elif kind == "maxpool2d":
            ph, pw = layer["pool"]
            x = F.max_pool2d(x, (ph, pw), (ph, pw))
        elif kind == "globalmaxpool2d":
            x = torch.amax(x, dim=(2, 3))
            logits = x
        elif kind == "activation":
            assert layer["fn"] == "sigmoid"
            x = torch.sigmoid(x)
        else:
            raise ValueError(f"unknown layer type {kind}")
    if logits is None:
        logits = x
    return logits.cpu().numpy(), x.cpu().numpy()


def ensemble_track_mean(probs_per_model):
    """np.mean over models then over windows (src/identify_tracks.py:548-551)."""
    p = np.mean(probs_per_model, axis=0)
    return np.mean(p, axis=0)
