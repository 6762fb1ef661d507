"""``.keras`` model files -> this build's layer list + weights.

The reference loads ``<dir>/audioModel.keras`` with ``tf.keras.models.load_model``
(src/identify_tracks.py:302-327; the AI-Model ``audio-v0.8`` release,
Dockerfile:33-37).  A ``.keras`` file is a zip of ``config.json`` (the
serialised model: Sequential or a single-chain Functional, one entry per
layer with ``class_name`` and ``config``), ``model.weights.h5`` (HDF5) and
``metadata.json``.  Keras 3 stores each layer's variables as datasets
``layers/<name>/vars/<i>`` of the weights file, ``<name>`` being the
snake_case class name with a per-class counter (``conv2d``, ``conv2d_1``,
...) in ``model.layers`` order, the variables in the layer's order
(trainable, then non-trainable: Conv2D kernel, bias; BatchNormalization
gamma, beta, moving_mean, moving_variance; Dense kernel, bias; MagTransform
a).  The HDF5 file is read by ``h5lite`` (no h5py in this stack).

Layers mapped onto the CNN planner (include/aa.h aa_op): InputLayer,
Conv2D (valid padding, stride 1, no dilation / groups; a fused activation
becomes its own layer), BatchNormalization (last axis), LeakyReLU, ReLU,
Activation (relu / sigmoid / linear), MaxPooling2D (valid, strides = pool),
GlobalMaxPooling2D, Dense after the global pooling, MagTransform (v1 scalar
or v2 [1] ``a``); Dropout-type layers are inference no-ops.  Any other layer
raises NotImplementedError naming it -- the planner has no kernel for it.

Parity: the HDF5 reader is pinned by files from the real HDF5 library
(tests/golden/h5); the zip/JSON layout follows Keras 3's saving_lib as
documented, and tests/golden/make_keras.py writes such files with h5py --
no Keras/TF exists in this image, so a file saved by Keras itself has not
been read (parity unpinned against Keras's writer).
"""
from __future__ import annotations

import io
import json
import re
import zipfile

import numpy as np

from . import h5lite

_NOOP = {"Dropout", "SpatialDropout2D", "GaussianNoise", "GaussianDropout", "AlphaDropout", "ActivityRegularization"}


def snake(name: str) -> str:
    """keras.src.utils.naming.to_snake_case."""
    name = re.sub(r"\W+", "", name)
    name = re.sub("(.)([A-Z][a-z]+)", r"\1_\2", name)
    name = re.sub("([a-z])([A-Z])", r"\1_\2", name)
    return name.lower()


def _class(layer):
    """Class of a serialised layer; registered custom layers appear as
    "Package>Name" (Keras 2 class_name, Keras 3 registered_name)."""
    return str(layer.get("class_name", "")).split(">")[-1]


def _pair(v):
    return list(v) if isinstance(v, (list, tuple)) else [v, v]


def _activation(act, out, where):
    if isinstance(act, dict):  # serialised activation object
        act = act.get("config", {}).get("name", act.get("class_name", ""))
    act = (act or "linear").lower()
    if act == "linear":
        return
    if act == "relu":
        out.append({"type": "relu"})
    elif act == "sigmoid":
        out.append({"type": "activation", "fn": "sigmoid"})
    elif act in ("leaky_relu", "leakyrelu"):
        out.append({"type": "leakyrelu", "alpha": 0.2})  # keras.activations.leaky_relu default slope
    else:
        raise NotImplementedError(f"{where}: activation {act!r}")


def model_layers(config: dict):
    """The layer list of a Sequential / single-chain Functional config."""
    cfg = config.get("config", config)
    layers = cfg.get("layers")
    if layers is None:
        raise ValueError("config.json has no layer list")
    if config.get("class_name") not in (None, "Sequential", "Functional", "Model"):
        raise NotImplementedError(f"model class {config.get('class_name')}")
    if config.get("class_name") in ("Functional", "Model"):
        prev = None
        for ly in layers:  # a chain: every layer's only input is the previous layer
            nodes = ly.get("inbound_nodes") or []
            names = re.findall(r'"keras_history": \["([^"]+)"', json.dumps(nodes))
            if prev is not None and names != [prev]:
                raise NotImplementedError(f"non-sequential Functional model at layer {ly['config'].get('name')}")
            prev = ly["config"].get("name")
    return layers


def convert(config: dict, weights: h5lite.H5File):
    """(arch list, {tensor name: float32 array}, input shape (H, W, C) or None)."""
    arch, tensors = [], {}
    counters = {}
    in_shape = None
    groups = set(weights.keys("layers")) if "layers" in weights.keys() else set()
    pooled = False

    def variables(ly, n_expected):
        cls = _class(ly)
        key = snake(cls)
        k = counters.get(key, -1) + 1
        counters[key] = k
        name = key if k == 0 else f"{key}_{k}"
        if name not in groups:
            name = ly["config"].get("name", name)
        if n_expected == 0:
            return []
        if name not in groups:
            raise ValueError(f"weights of layer {ly['config'].get('name')} ({cls}) not in model.weights.h5")
        path = f"layers/{name}/vars"
        return [weights.read(f"{path}/{i}").astype(np.float32) for i in range(len(weights.keys(path)))]

    for ly in model_layers(config):
        cls = _class(ly)
        c = ly.get("config", {})
        lname = c.get("name", cls)
        if cls == "InputLayer":
            shape = c.get("batch_shape") or c.get("batch_input_shape")
            if shape:
                in_shape = tuple(int(x) for x in shape[1:])
            continue
        if cls in _NOOP:
            variables(ly, 0)
            continue
        if cls == "Conv2D":
            if c.get("padding", "valid") != "valid" or _pair(c.get("strides", 1)) != [1, 1] or \
                    _pair(c.get("dilation_rate", 1)) != [1, 1] or c.get("groups", 1) != 1 or \
                    c.get("data_format", "channels_last") not in ("channels_last", None):
                raise NotImplementedError(f"{lname}: Conv2D other than valid / stride 1 / channels_last")
            v = variables(ly, 2)
            arch.append({"type": "conv2d", "name": lname, "filters": int(c["filters"]),
                         "kernel": _pair(c["kernel_size"]), "use_bias": bool(c.get("use_bias", True))})
            tensors[lname + ".kernel"] = v[0]
            if c.get("use_bias", True):
                tensors[lname + ".bias"] = v[1]
            _activation(c.get("activation"), arch, lname)
        elif cls == "BatchNormalization":
            ax = c.get("axis", -1)
            if ax not in (-1, 3, [3], [-1]):
                raise NotImplementedError(f"{lname}: BatchNormalization over axis {ax}")
            v = variables(ly, 4)
            i = 0
            n = v[-1].shape[0]
            g = v[i] if c.get("scale", True) else np.ones(n, np.float32)
            i += int(c.get("scale", True))
            b = v[i] if c.get("center", True) else np.zeros(n, np.float32)
            i += int(c.get("center", True))
            tensors.update({lname + ".gamma": g, lname + ".beta": b, lname + ".moving_mean": v[i],
                            lname + ".moving_variance": v[i + 1]})
            arch.append({"type": "batchnorm", "name": lname, "eps": float(c.get("epsilon", 1e-3))})
        elif cls == "LeakyReLU":
            variables(ly, 0)
            arch.append({"type": "leakyrelu", "alpha": float(c.get("negative_slope", c.get("alpha", 0.3)))})
        elif cls == "ReLU":
            variables(ly, 0)
            if c.get("max_value") is not None or c.get("negative_slope", 0) or c.get("threshold", 0):
                raise NotImplementedError(f"{lname}: ReLU with max_value / slope / threshold")
            arch.append({"type": "relu"})
        elif cls == "Activation":
            variables(ly, 0)
            _activation(c.get("activation"), arch, lname)
        elif cls == "MaxPooling2D":
            variables(ly, 0)
            pool = _pair(c.get("pool_size", 2))
            strides = c.get("strides") or pool
            if c.get("padding", "valid") != "valid" or _pair(strides) != pool:
                raise NotImplementedError(f"{lname}: MaxPooling2D other than valid with strides = pool")
            arch.append({"type": "maxpool2d", "pool": pool})
        elif cls == "GlobalMaxPooling2D":
            variables(ly, 0)
            if c.get("keepdims", False):
                raise NotImplementedError(f"{lname}: GlobalMaxPooling2D(keepdims=True)")
            arch.append({"type": "globalmaxpool2d"})
            pooled = True
        elif cls == "Dense":
            if not pooled:
                raise NotImplementedError(f"{lname}: Dense on a feature map (only after global pooling)")
            v = variables(ly, 2)
            arch.append({"type": "dense", "name": lname, "units": int(c["units"]),
                         "use_bias": bool(c.get("use_bias", True))})
            tensors[lname + ".kernel"] = v[0]
            if c.get("use_bias", True):
                tensors[lname + ".bias"] = v[1]
            _activation(c.get("activation"), arch, lname)
        elif cls == "MagTransform":
            v = variables(ly, 1)
            tensors[lname + ".a"] = np.asarray(v[0], np.float32).reshape(-1)[:1]
            arch.append({"type": "magtransform", "name": lname, "version": 2 if v[0].ndim else 1})
        else:
            raise NotImplementedError(f"layer {lname}: Keras {cls} has no kernel in this build")
    return arch, tensors, in_shape


def read_keras(path):
    """``.keras`` file -> (arch, tensors, input shape)."""
    with zipfile.ZipFile(path) as z:
        names = z.namelist()
        config = json.loads(z.read("config.json"))
        wname = "model.weights.h5" if "model.weights.h5" in names else next(
            (n for n in names if n.endswith(".weights.h5") or n.endswith(".h5")), None)
        if wname is None:
            raise ValueError(f"{path}: no weights file in the archive")
        weights = h5lite.open_h5(io.BytesIO(z.read(wname)).getvalue())
    return convert(config, weights)
