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

Layers: InputLayer, Conv2D (valid / same padding, any stride, no dilation /
groups; a fused activation becomes its own entry), DepthwiseConv2D (depth
multiplier 1), BatchNormalization (last axis), LeakyReLU, ReLU, Activation
(relu / sigmoid / swish / silu / leaky_relu / linear), MaxPooling2D and
AveragePooling2D (valid / same, any strides), GlobalMaxPooling2D,
GlobalAveragePooling2D, Add, Multiply, ZeroPadding2D, Reshape, Flatten,
Rescaling, Normalization, Dense, MagTransform (v1 scalar or v2 [1] ``a``),
nested Sequential / Functional models (weights under their own
``layers/<name>/layers/...`` path); Dropout-type layers are inference no-ops.
A chain of the first group maps onto the tuned sequential planner (aa_op
layer table); anything else becomes a graph (aa_amd.graph, aa_graph_*).  Any
other layer raises NotImplementedError naming it.

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


def _act_name(act):
    if isinstance(act, dict):  # serialised activation object
        act = act.get("config", {}).get("name", act.get("class_name", ""))
    return (act or "linear").lower()


def _activation(act, out, where, src=None):
    """Append the layer entry of a Keras activation (fused or standalone)."""
    act = _act_name(act)
    if act == "linear":
        return
    if act == "relu":
        e = {"type": "relu"}
    elif act in ("sigmoid", "swish", "silu"):
        e = {"type": "activation", "fn": "swish" if act == "silu" else act}
    elif act in ("leaky_relu", "leakyrelu"):
        e = {"type": "leakyrelu", "alpha": 0.2}  # keras.activations.leaky_relu default slope
    else:
        raise NotImplementedError(f"{where}: activation {act!r}")
    e["name"] = f"{where}/{act}"
    if src is not None:
        e["inputs"] = [src]
    out.append(e)


def _history(ly):
    """Names of the tensors a Functional layer reads (Keras 3 keras_history,
    or Keras 2 inbound_nodes [[name, node, tensor, kwargs], ...])."""
    nodes = ly.get("inbound_nodes") or []
    names = re.findall(r'"keras_history": \["([^"]+)"', json.dumps(nodes))
    if names or not nodes:
        return names
    out = []

    def walk(v):
        if isinstance(v, list) and len(v) >= 3 and isinstance(v[0], str) and isinstance(v[1], int):
            out.append(v[0])
        elif isinstance(v, list):
            for x in v:
                walk(x)
    walk(nodes)
    return out


_MODELS = ("Sequential", "Functional", "Model")


def model_layers(config: dict):
    """The layer list of a Sequential / Functional config."""
    cfg = config.get("config", config)
    layers = cfg.get("layers")
    if layers is None:
        raise ValueError("config.json has no layer list")
    if config.get("class_name") not in (None,) + _MODELS:
        raise NotImplementedError(f"model class {config.get('class_name')}")
    return layers


def _pad4(p):
    """ZeroPadding2D padding -> ((top, bottom), (left, right))."""
    if isinstance(p, int):
        return [[p, p], [p, p]]
    a, b = p
    a = [a, a] if isinstance(a, int) else list(a)
    b = [b, b] if isinstance(b, int) else list(b)
    return [a, b]


def convert(config: dict, weights: h5lite.H5File):
    """(arch list, {tensor name: float32 array}, input shape (H, W, C) or None).
    Sequential models and single-chain graphs become a plain layer chain (the
    tuned planner); any other Functional graph -- and nested models -- an arch
    whose entries name their inputs (aa_amd.graph)."""
    arch, tensors = [], {}
    state = {"in_shape": None, "pooled": False}

    def vars_at(path):
        if path not in _keys_cache:
            _keys_cache[path] = weights.keys(path) if _exists(path) else None
        ks = _keys_cache[path]
        if ks is None:
            return None
        return [weights.read(f"{path}/{i}").astype(np.float32) for i in range(len(ks))]

    _keys_cache = {}

    def _exists(path):
        parts = path.split("/")
        cur = ""
        for p_ in parts:
            try:
                ks = weights.keys(cur) if cur else weights.keys()
            except Exception:
                return False
            if p_ not in ks:
                return False
            cur = f"{cur}/{p_}" if cur else p_
        return True

    def walk(model_cfg, wprefix, nprefix, in_names, top):
        """Convert one (possibly nested) model; returns its output tensor name."""
        cls = model_cfg.get("class_name")
        c = model_cfg.get("config", model_cfg)
        layers = c.get("layers") or []
        sequential = cls in (None, "Sequential")
        counters = {}
        produced = {}
        prev = in_names[0] if in_names else "input"
        out_name = prev
        for ly in layers:
            lcls = _class(ly)
            lc = ly.get("config", {})
            lname = lc.get("name", lcls)
            full = nprefix + lname
            key = snake(lcls)
            k = counters.get(key, -1) + 1
            counters[key] = k
            wname = key if k == 0 else f"{key}_{k}"
            wpath = f"{wprefix}layers/{wname}"
            if not _exists(wpath) and _exists(f"{wprefix}layers/{lname}"):
                wpath = f"{wprefix}layers/{lname}"  # files written by layer name
            if lcls == "InputLayer":
                shape = lc.get("batch_shape") or lc.get("batch_input_shape")
                if shape and top and state["in_shape"] is None:
                    state["in_shape"] = tuple(int(x) for x in shape[1:])
                produced[lname] = prev if in_names else "input"
                continue
            if sequential:
                ins = [prev]
            else:
                hist = _history(ly)
                ins = [produced[h] for h in hist] if hist else [prev]
            if lcls in _MODELS:  # a nested model: its layers inline, under its weight path
                o = walk(ly, wpath + "/", full + "/", ins, False)
                produced[lname] = prev = out_name = o
                continue
            v = vars_at(wpath + "/vars") or []
            o = convert_layer(lcls, lc, full, ins, v)
            produced[lname] = prev = out_name = o
        if not sequential:
            outs = c.get("output_layers")
            if outs:
                names = re.findall(r'"([^"]+)"', json.dumps(outs))
                if names and names[0] in produced:
                    out_name = produced[names[0]]
        return out_name

    def convert_layer(cls, c, name, ins, v):
        """Arch entries of one layer; returns the name of its output tensor."""
        src = ins[0]

        def emit(e):
            e.setdefault("name", name)
            e["inputs"] = list(ins) if "inputs" not in e else e["inputs"]
            arch.append(e)
            return e["name"]

        if cls in _NOOP:
            return src
        if cls in ("Conv2D", "DepthwiseConv2D"):
            if _pair(c.get("dilation_rate", 1)) != [1, 1] or c.get("groups", 1) != 1 or \
                    c.get("data_format", "channels_last") not in ("channels_last", None):
                raise NotImplementedError(f"{name}: {cls} with dilation / groups / channels_first")
            if cls == "DepthwiseConv2D" and int(c.get("depth_multiplier", 1)) != 1:
                raise NotImplementedError(f"{name}: DepthwiseConv2D with depth_multiplier != 1")
            pad = c.get("padding", "valid")
            if pad not in ("valid", "same"):
                raise NotImplementedError(f"{name}: padding {pad!r}")
            bias = bool(c.get("use_bias", True))
            e = {"type": "conv2d" if cls == "Conv2D" else "depthwise_conv2d", "kernel": _pair(c["kernel_size"]),
                 "use_bias": bias}
            if cls == "Conv2D":
                e["filters"] = int(c["filters"])
            strides = _pair(c.get("strides", 1))
            if strides != [1, 1]:
                e["strides"] = strides
            if pad != "valid":
                e["padding"] = pad
            tensors[name + ".kernel"] = v[0]
            if bias:
                tensors[name + ".bias"] = v[1]
            o = emit(e)
            n0 = len(arch)
            _activation(c.get("activation"), arch, name, o)
            return arch[-1]["name"] if len(arch) > n0 else o
        if cls == "BatchNormalization":
            ax = c.get("axis", -1)
            if ax not in (-1, 3, [3], [-1]):
                raise NotImplementedError(f"{name}: BatchNormalization over axis {ax}")
            i = 0
            n = v[-1].shape[0]
            g = v[i] if c.get("scale", True) else np.ones(n, np.float32)
            i += int(c.get("scale", True))
            b = v[i] if c.get("center", True) else np.zeros(n, np.float32)
            i += int(c.get("center", True))
            tensors.update({name + ".gamma": g, name + ".beta": b, name + ".moving_mean": v[i],
                            name + ".moving_variance": v[i + 1]})
            return emit({"type": "batchnorm", "eps": float(c.get("epsilon", 1e-3))})
        if cls == "LeakyReLU":
            return emit({"type": "leakyrelu", "alpha": float(c.get("negative_slope", c.get("alpha", 0.3)))})
        if cls == "ReLU":
            if c.get("max_value") is not None or c.get("negative_slope", 0) or c.get("threshold", 0):
                raise NotImplementedError(f"{name}: ReLU with max_value / slope / threshold")
            return emit({"type": "relu"})
        if cls == "Activation":
            n0 = len(arch)
            _activation(c.get("activation"), arch, name, src)
            if len(arch) == n0:
                return src
            arch[-1]["name"] = name
            return name
        if cls in ("MaxPooling2D", "AveragePooling2D"):
            pool = _pair(c.get("pool_size", 2))
            strides = _pair(c.get("strides") or pool)
            pad = c.get("padding", "valid")
            e = {"type": "maxpool2d" if cls == "MaxPooling2D" else "avgpool2d", "pool": pool}
            if strides != pool:
                e["strides"] = strides
            if pad != "valid":
                e["padding"] = pad
            return emit(e)
        if cls in ("GlobalMaxPooling2D", "GlobalAveragePooling2D"):
            state["pooled"] = True
            return emit({"type": "globalmaxpool2d" if cls == "GlobalMaxPooling2D" else "globalavgpool2d"})
        if cls in ("Add", "Multiply"):
            if len(ins) != 2:
                raise NotImplementedError(f"{name}: {cls} of {len(ins)} tensors")
            return emit({"type": "add" if cls == "Add" else "multiply"})
        if cls == "ZeroPadding2D":
            return emit({"type": "zeropad2d", "pad": _pad4(c.get("padding", 1))})
        if cls == "Reshape":
            return emit({"type": "reshape", "target": list(c.get("target_shape", []))})
        if cls == "Flatten":
            return emit({"type": "flatten"})
        if cls == "Rescaling":
            sc, of = c.get("scale", 1.0), c.get("offset", 0.0)
            if not np.isscalar(sc) or not np.isscalar(of):
                raise NotImplementedError(f"{name}: per-channel Rescaling")
            return emit({"type": "rescaling", "scale": float(sc), "offset": float(of)})
        if cls == "Normalization":
            if c.get("invert", False):
                raise NotImplementedError(f"{name}: Normalization(invert=True)")
            mean = c.get("mean")
            var = c.get("variance")
            if mean is None:  # adapted: variables mean, variance (count)
                mean, var = v[0], v[1]
            tensors[name + ".mean"] = np.asarray(mean, np.float32).reshape(-1)
            tensors[name + ".variance"] = np.asarray(var, np.float32).reshape(-1)
            return emit({"type": "normalization"})
        if cls == "Dense":
            bias = bool(c.get("use_bias", True))
            tensors[name + ".kernel"] = v[0]
            if bias:
                tensors[name + ".bias"] = v[1]
            o = emit({"type": "dense", "units": int(c["units"]), "use_bias": bias})
            n0 = len(arch)
            _activation(c.get("activation"), arch, name, o)
            return arch[-1]["name"] if len(arch) > n0 else o
        if cls == "MagTransform":
            tensors[name + ".a"] = np.asarray(v[0], np.float32).reshape(-1)[:1]
            return emit({"type": "magtransform", "version": 2 if v[0].ndim else 1})
        raise NotImplementedError(f"layer {name}: Keras {cls} has no kernel in this build")

    if config.get("class_name") not in (None,) + _MODELS:
        raise NotImplementedError(f"model class {config.get('class_name')}")
    if (config.get("config", config).get("layers")) is None:
        raise ValueError("config.json has no layer list")
    walk(config, "", "", [], True)
    # a plain chain (every entry reads the previous one, no graph-only layer):
    # the tuned sequential planner's layer list, inputs implicit
    chain = all(e["inputs"] == [arch[i - 1]["name"] if i else "input"] for i, e in enumerate(arch))
    from .graph import GRAPH_ONLY
    if chain and not any(e["type"] in GRAPH_ONLY or e.get("padding", "valid") != "valid" or "strides" in e
                         for e in arch):
        for e in arch:
            e.pop("inputs", None)
            if e["type"] in ("relu", "leakyrelu", "maxpool2d", "globalmaxpool2d") or \
                    (e["type"] == "activation" and e.get("fn") == "sigmoid"):
                e.pop("name", None)
        if any(e["type"] == "dense" for e in arch) and not state["pooled"]:
            raise NotImplementedError("Dense on a feature map in a chain model (only after global pooling)")
    return arch, tensors, state["in_shape"]


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
