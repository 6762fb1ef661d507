"""Model loading and GPU inference (host side of aa_model_*).

Model contract (reference src/identify_tracks.py:291-327, src/analyse.py:414-418):
``--bird-model`` names ``<dir>/audioModel.keras`` (or the directory); the
JSON ``<dir>/metadata.txt`` beside it holds labels and front-end settings.
This build stores the network as ``<dir>/audioModel.safetensors`` (weights plus
``__metadata__["arch"]``, a Keras-style layer list); without one, the
reference's ``audioModel.keras`` itself is read (keras_import: zip + HDF5
through h5lite, no TF/h5py).  ``Model.predict`` replaces ``model.predict(np.array(d))`` (:544).
"""
from __future__ import annotations

import ctypes as C
import json
import logging
from pathlib import Path

import numpy as np
import torch

from . import _lib

WEIGHTS_NAME = "audioModel.safetensors"


def load_model_meta(model_path) -> dict:
    """metadata.txt next to a model file, or inside a model directory (:291-299)."""
    p = Path(model_path)
    meta_file = p.parent / "metadata.txt" if p.is_file() or p.suffix else p / "metadata.txt"
    with open(meta_file, "r") as f:
        return json.load(f)


def weights_path(model_path) -> Path:
    p = Path(model_path)
    if p.suffix == ".safetensors":
        return p
    if p.is_dir():
        return p / WEIGHTS_NAME
    return p.parent / WEIGHTS_NAME


def load_network(model_path):
    """(arch, tensors) of a model: this build's ``audioModel.safetensors`` when
    present, else the reference's ``audioModel.keras`` (keras_import)."""
    p = Path(model_path)
    wp = weights_path(p)
    if wp.exists():
        return read_arch(wp)
    kp = p if p.suffix == ".keras" else (p / "audioModel.keras" if p.is_dir() else p.with_name("audioModel.keras"))
    if kp.exists():
        from .keras_import import read_keras
        arch, tensors, _ = read_keras(kp)
        return arch, tensors
    raise FileNotFoundError(f"{model_path}: neither {wp.name} nor {kp.name}")


def read_arch(path):
    from safetensors import safe_open
    from safetensors.numpy import load_file
    with safe_open(str(path), framework="np") as f:
        meta = f.metadata() or {}
    if "arch" not in meta:
        raise ValueError(f"{path}: no arch metadata")
    return json.loads(meta["arch"]), load_file(str(path))


def layer_table(arch, tensors):
    """Keras-style layer list -> (aa_layer array, float32 blob)."""
    chunks, layers = [], []
    size = 0

    def put(name):
        nonlocal size
        a = np.ascontiguousarray(np.asarray(tensors[name], dtype=np.float32).reshape(-1))
        chunks.append(a)
        off = size
        size += a.size
        return off

    for ly in arch:
        kind = ly["type"]
        off = [-1, -1, -1, -1]
        kh = kw = filters = 0
        alpha = eps = 0.0
        if kind == "conv2d":
            kh, kw = ly["kernel"]
            filters = ly["filters"]
            off[0] = put(ly["name"] + ".kernel")
            if ly.get("use_bias", False):
                off[1] = put(ly["name"] + ".bias")
            op = "conv2d"
        elif kind == "batchnorm":
            n = ly["name"]
            off = [put(n + ".gamma"), put(n + ".beta"), put(n + ".moving_mean"),
                   put(n + ".moving_variance")]
            eps = float(ly.get("eps", 1e-3))
            op = "batchnorm"
        elif kind == "leakyrelu":
            alpha = float(ly.get("alpha", 0.3))
            op = "leakyrelu"
        elif kind == "relu":
            op = "relu"
        elif kind == "maxpool2d":
            kh, kw = ly["pool"]
            op = "maxpool2d"
        elif kind == "globalmaxpool2d":
            op = "globalmaxpool2d"
        elif kind == "activation":
            if ly["fn"] != "sigmoid":
                raise ValueError(f"unsupported activation {ly['fn']}")
            op = "sigmoid"
        elif kind == "magtransform":
            off[0] = put(ly["name"] + ".a")
            op = "magtransform"
        elif kind == "dense":
            filters = ly["units"]
            off[0] = put(ly["name"] + ".kernel")
            if ly.get("use_bias", True):
                off[1] = put(ly["name"] + ".bias")
            op = "dense"
        else:
            raise ValueError(f"unsupported layer type {kind}")
        L = _lib.Layer(op=_lib.AA_OP[op], kh=kh, kw=kw, filters=filters, alpha=alpha, eps=eps)
        for i in range(4):
            L.off[i] = off[i]
        layers.append(L)
    blob = np.concatenate(chunks).astype(np.float32) if chunks else np.zeros(1, np.float32)
    arr = (_lib.Layer * len(layers))(*layers)
    return arr, blob


class Model(_lib.StageTiming):
    """A loaded network on one device.  ``precision``: "bf16x3" (split-bf16,
    the default: ~17-bit products on bf16 MFMA, within the 1e-3 logit gate),
    "f32" (exact-f32 MFMA), "bf16" or "fp8" (throughput modes)."""
    _timing_prefix = "aa_model"

    def __init__(self, model_path, in_shape, precision="bf16x3", device=None, meta=None):
        self.path = Path(model_path)
        self.meta = meta if meta is not None else load_model_meta(model_path)
        self.device = torch.device(device or "cuda")
        self.precision = precision
        try:
            arch, tensors = load_network(model_path)
        except Exception:
            logging.info("Could not load model", exc_info=True)  # :324-326
            raise
        self.in_shape = tuple(int(v) for v in in_shape)  # (H, W, C)
        prec = {"f32": _lib.AA_PREC_F32, "bf16": _lib.AA_PREC_BF16, "fp8": _lib.AA_PREC_FP8,
                "bf16x3": _lib.AA_PREC_BF16X3}[precision]
        h = C.c_void_p()
        from .graph import graph_table, is_graph
        self.graph = is_graph(arch)
        with torch.cuda.device(self.device):
            if self.graph:
                # a Keras graph (residual / squeeze-excite / depthwise / strided
                # "same" convs): the node executor (aa_graph_*), split-bf16 or f32
                if prec not in (_lib.AA_PREC_BF16X3, _lib.AA_PREC_F32):
                    logging.info("%s: graph models run in split-bf16 (precision %s not served)", model_path,
                                 precision)
                    prec = _lib.AA_PREC_BF16X3
                nodes, blob, _ = graph_table(arch, tensors, self.in_shape)
                _lib.check(_lib.lib().aa_graph_create(nodes, len(nodes), blob.ctypes.data, blob.size,
                                                      *self.in_shape, prec, C.byref(h)), "aa_graph_create")
                self._timing_prefix = "aa_graph"
            else:
                layers, blob = layer_table(arch, tensors)
                _lib.check(_lib.lib().aa_model_create(layers, len(layers), blob.ctypes.data, blob.size,
                                                      *self.in_shape, prec, C.byref(h)), "aa_model_create")
        self._h = h
        self.n_labels = (_lib.lib().aa_graph_n_outputs if self.graph else _lib.lib().aa_model_n_outputs)(h)
        self._ws = None
        self._in_f16 = False

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            (_lib.lib().aa_graph_destroy if getattr(self, "graph", False) else _lib.lib().aa_model_destroy)(h)
            self._h = None

    def workspace_bytes(self, n: int) -> int:
        if self.graph:
            return int(_lib.lib().aa_graph_workspace_bytes(self._h, int(n)))
        return int(_lib.lib().aa_model_workspace_bytes(self._h, int(n)))

    def _workspace(self, n: int) -> torch.Tensor:
        need = self.workspace_bytes(n)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        return self._ws

    def forward(self, x: torch.Tensor, logits: torch.Tensor = None, probs: torch.Tensor = None,
                stream=None, workspace: torch.Tensor = None):
        """x: float32 (or float16: BASELINE configs[4]) [n, H, W, C] on device ->
        (logits, probs) float32 [n, L]."""
        n = int(x.shape[0])
        if tuple(x.shape[1:]) != self.in_shape:
            raise ValueError(f"input {tuple(x.shape)} != model input {self.in_shape}")
        if x.dtype not in (torch.float32, torch.float16):
            raise ValueError(f"input dtype {x.dtype}: float32 or float16")
        f16 = x.dtype == torch.float16
        if f16 and self.graph:
            x = x.float()  # (graphs read f32)
            f16 = False
        if f16 != self._in_f16:
            _lib.check(_lib.lib().aa_model_set_input_f16(self._h, int(f16)), "aa_model_set_input_f16")
            self._in_f16 = f16
        if logits is None:
            logits = torch.empty((n, self.n_labels), dtype=torch.float32, device=self.device)
        if probs is None:
            probs = torch.empty((n, self.n_labels), dtype=torch.float32, device=self.device)
        if n == 0:
            return logits, probs
        ws = workspace if workspace is not None else self._workspace(n)
        fwd = _lib.lib().aa_graph_forward if self.graph else _lib.lib().aa_model_forward
        _lib.check(fwd(self._h, _lib.dptr(x), n, _lib.dptr(logits), _lib.dptr(probs), _lib.dptr(ws),
                       int(ws.numel()), _lib.stream_ptr(stream)),
                   "aa_graph_forward" if self.graph else "aa_model_forward")
        return logits, probs

    def predict(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward(x)[1]


def track_mean(probs: torch.Tensor, win_begin: torch.Tensor, win_count: torch.Tensor,
               out: torch.Tensor = None, stream=None) -> torch.Tensor:
    """probs [M, n_win, L] -> per-track mean over models then windows [n_tracks, L]."""
    M, n_win, L = probs.shape
    nt = int(win_begin.numel())
    if out is None:
        out = torch.empty((nt, L), dtype=torch.float32, device=probs.device)
    if nt == 0:
        return out
    _lib.check(_lib.lib().aa_track_mean(_lib.dptr(probs), M, n_win * L, L, _lib.dptr(win_begin),
                                        _lib.dptr(win_count), nt, _lib.dptr(out),
                                        _lib.stream_ptr(stream)), "aa_track_mean")
    return out
