"""Keras-style layer graphs -> libaa's aa_node list (include/aa.h, aa_graph_*).

classify() loads whatever network ``audioModel.keras`` holds
(src/identify_tracks.py:302-327) and routes names containing "efficientnet"
to a 3-channel input (:539-540).  Networks that are not a single conv chain
-- residual ``Add``, squeeze-and-excite ``Multiply``, ``DepthwiseConv2D``,
strided / "same"-padded convs, ``GlobalAveragePooling2D`` -- run as a node
graph.  An arch entry may name its inputs (``"inputs": [layer names]``;
default: the previous entry; "input" is the model input).  Layer types:

  conv2d (kernel, strides, padding valid|same, filters, use_bias, activation)
  depthwise_conv2d (kernel, strides, padding, use_bias, activation)
  batchnorm, activation (fn relu|sigmoid|swish|silu|leaky_relu|linear),
  relu, leakyrelu, maxpool2d / avgpool2d (pool, strides, padding),
  globalmaxpool2d / globalavgpool2d, add, multiply, dense, zeropad2d
  (pad [[t, b], [l, r]]), rescaling (scale, offset), normalization (mean,
  variance), reshape / flatten / dropout (no-ops on NHWC), magtransform.

Host-side planning, as the sequential planner does in C++ for chains:
BatchNormalization is folded into the conv / depthwise conv it follows (in
float64) when that conv feeds nothing else, an activation joins its producer
when it is the producer's only consumer, ZeroPadding2D becomes the next
window's explicit padding, and TF's "same" padding (pad_total = max((ceil(n /
s) - 1) s + k - n, 0), the extra row / column at the bottom / right) is
resolved into explicit pads.
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib

GRAPH_ONLY = {"depthwise_conv2d", "add", "multiply", "globalavgpool2d", "avgpool2d", "zeropad2d", "rescaling",
              "normalization", "reshape", "flatten"}
_ACTS = {"relu": "relu", "sigmoid": "sigmoid", "swish": "swish", "silu": "swish", "leaky_relu": "leaky",
         "linear": None, None: None}


def is_graph(arch) -> bool:
    """True when the arch needs the graph executor (not a plain conv chain)."""
    for ly in arch:
        kind = ly["type"]
        if "inputs" in ly or kind in GRAPH_ONLY:
            return True
        if kind in ("conv2d", "maxpool2d") and ly.get("padding", "valid") != "valid":
            return True
        if kind == "conv2d" and (list(ly.get("strides", [1, 1])) != [1, 1] or
                                 ly.get("activation") not in (None, "linear")):
            return True
        if kind == "maxpool2d" and list(ly.get("strides") or ly["pool"]) != list(ly["pool"]):
            return True
        if kind == "activation" and ly.get("fn") not in ("sigmoid",):
            return True
    return False


def _same_pads(n, k, s):
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


class _Blob:
    def __init__(self):
        self.chunks, self.size = [], 0

    def put(self, a) -> int:
        a = np.ascontiguousarray(np.asarray(a, np.float32).reshape(-1))
        off = self.size
        self.chunks.append(a)
        self.size += a.size
        return off

    def array(self):
        return np.concatenate(self.chunks).astype(np.float32) if self.chunks else np.zeros(1, np.float32)


def graph_table(arch, tensors, in_shape):
    """(aa_node array, f32 blob, output size) for aa_graph_create."""
    H0, W0, C0 = (int(v) for v in in_shape)
    names = []
    for i, ly in enumerate(arch):
        names.append(ly.get("name") or f"_l{i}")
    inputs = []
    for i, ly in enumerate(arch):
        ins = ly.get("inputs")
        if ins is None:
            ins = ["input"] if i == 0 else [names[i - 1]]
        inputs.append(list(ins))
    index = {n: i for i, n in enumerate(names)}
    consumers = {n: 0 for n in names}
    for ins in inputs:
        for s in ins:
            if s != "input":
                consumers[s] += 1
    t = lambda k: np.asarray(tensors[k], np.float64)

    blob = _Blob()
    nodes = []              # dicts -> aa_node
    out_of = {"input": (-1, (H0, W0, C0), None)}  # layer name -> (node index, shape, pending pads)

    def node_of(name):
        return out_of[name]

    def new_node(op, src, shape, **kw):
        d = dict(op=_lib.AA_G[op], in0=src[0], in1=src[1] if len(src) > 1 else -1, kh=1, kw=1, sh=1, sw=1,
                 pt=0, pb=0, pl=0, pr=0, filters=0, act=0, alpha=0.0, off=[-1, -1])
        d.update(kw)
        nodes.append(d)
        return len(nodes) - 1

    def window(ly, n_in, shape, k, s, extra):
        H, W, _ = shape
        pad = ly.get("padding", "valid")
        pt = pb = pl = pr = 0
        if pad == "same":
            pt, pb = _same_pads(H + extra[0] + extra[1], k[0], s[0])
            pl, pr = _same_pads(W + extra[2] + extra[3], k[1], s[1])
        elif pad != "valid":
            raise NotImplementedError(f"{ly.get('name')}: padding {pad!r}")
        pt, pb, pl, pr = pt + extra[0], pb + extra[1], pl + extra[2], pr + extra[3]
        Ho = (H + pt + pb - k[0]) // s[0] + 1
        Wo = (W + pl + pr - k[1]) // s[1] + 1
        return dict(kh=k[0], kw=k[1], sh=s[0], sw=s[1], pt=pt, pb=pb, pl=pl, pr=pr), (Ho, Wo)

    def only_consumer(i, kinds):
        """index of the layer that is layer i's only consumer, if of a kind in kinds"""
        if consumers[names[i]] != 1:
            return None
        for j in range(i + 1, len(arch)):
            if names[i] in inputs[j]:
                return j if arch[j]["type"] in kinds else None
        return None

    def act_code(fn):
        a = _ACTS.get(fn if fn is None else str(fn).lower(), "?")
        if a == "?":
            raise NotImplementedError(f"activation {fn!r}")
        return _lib.AA_GACT[a]

    aliases = {}  # node index -> layer names that resolve to its output

    def bind(nm, entry):
        out_of[nm] = entry
        if entry[0] >= 0:
            aliases.setdefault(entry[0], set()).add(nm)

    def node_consumers(idx):
        return sum(consumers.get(nm, 0) for nm in aliases.get(idx, ()))

    skip = set()
    for i, ly in enumerate(arch):
        if i in skip:
            continue
        kind, name = ly["type"], names[i]
        srcs = [node_of(s) for s in inputs[i]]
        n0, shape0, extra0 = srcs[0]
        extra0 = extra0 or (0, 0, 0, 0)
        if kind not in ("conv2d", "depthwise_conv2d", "maxpool2d", "avgpool2d", "zeropad2d") and any(
                s[2] for s in srcs):
            raise NotImplementedError(f"{name}: ZeroPadding2D before a {kind}")
        H, W, C = shape0
        if kind in ("dropout", "reshape", "flatten", "input"):
            if kind == "reshape" and not (H == 1 and W == 1) and tuple(ly.get("target", ())) not in ((H, W, C),):
                raise NotImplementedError(f"{name}: Reshape of a {H}x{W}x{C} map")
            bind(name, srcs[0])
            continue
        if kind == "zeropad2d":
            (t_, b_), (l_, r_) = ly["pad"]
            e = extra0
            bind(name, (n0, shape0, (e[0] + t_, e[1] + b_, e[2] + l_, e[3] + r_)))
            continue
        if kind in ("conv2d", "depthwise_conv2d"):
            k = list(ly["kernel"])
            s = list(ly.get("strides", [1, 1]))
            if list(ly.get("dilation", [1, 1])) != [1, 1]:
                raise NotImplementedError(f"{name}: dilated conv")
            geo, (Ho, Wo) = window(ly, n0, shape0, k, s, extra0)
            kern = t(name + ".kernel")
            if kind == "conv2d":
                Co = int(ly["filters"])
                kern = kern.reshape(k[0], k[1], C, Co)
            else:
                if kern.size != k[0] * k[1] * C:
                    raise NotImplementedError(f"{name}: depth multiplier other than 1")
                Co = C
                kern = kern.reshape(k[0], k[1], C)
            bias = t(name + ".bias") if ly.get("use_bias", True) else np.zeros(Co)
            act = act_code(ly.get("activation"))
            end = i
            # fold a following BatchNormalization (sole consumer, no activation yet)
            if act == 0:
                j = only_consumer(end, ("batchnorm",))
                if j is not None:
                    bn, bnn = arch[j], names[j]
                    sc = t(bnn + ".gamma") / np.sqrt(t(bnn + ".moving_variance") + float(bn.get("eps", 1e-3)))
                    bias = (bias - t(bnn + ".moving_mean")) * sc + t(bnn + ".beta")
                    kern = kern * sc  # broadcast over the output-channel axis (last)
                    skip.add(j)
                    end = j
                j = only_consumer(end, ("activation", "relu", "leakyrelu"))
                alpha = 0.0
                if j is not None:
                    a = arch[j]
                    if a["type"] == "relu":
                        act = _lib.AA_GACT["relu"]
                    elif a["type"] == "leakyrelu":
                        act, alpha = _lib.AA_GACT["leaky"], float(a.get("alpha", 0.3))
                    else:
                        act = act_code(a["fn"])
                        alpha = 0.2 if act == _lib.AA_GACT["leaky"] else 0.0
                    skip.add(j)
                    end = j
            else:
                alpha = 0.2 if act == _lib.AA_GACT["leaky"] else 0.0
            op = "conv" if kind == "conv2d" else "dwconv"
            idx = new_node(op, [n0], None, filters=Co if kind == "conv2d" else 0, act=act, alpha=alpha,
                           off=[blob.put(kern), blob.put(bias)], **geo)
            out_of[names[end]] = (idx, (Ho, Wo, Co), None)
            bind(name, out_of[names[end]])
            continue
        if kind in ("maxpool2d", "avgpool2d"):
            k = list(ly["pool"])
            s = list(ly.get("strides") or k)
            geo, (Ho, Wo) = window(ly, n0, shape0, k, s, extra0)
            idx = new_node("maxpool" if kind == "maxpool2d" else "avgpool", [n0], None, **geo)
            bind(name, (idx, (Ho, Wo, C), None))
            continue
        if kind in ("globalmaxpool2d", "globalavgpool2d"):
            idx = new_node("gmaxpool" if kind == "globalmaxpool2d" else "gavgpool", [n0], None)
            bind(name, (idx, (1, 1, C), None))
            continue
        if kind in ("add", "multiply"):
            if len(srcs) != 2:
                raise NotImplementedError(f"{name}: {kind} of {len(srcs)} inputs")
            a_, b_ = srcs
            if kind == "multiply" and a_[1][:2] == (1, 1) and b_[1][:2] != (1, 1):
                a_, b_ = b_, a_  # the [1][1][C] operand second (broadcast)
            idx = new_node("add" if kind == "add" else "mul", [a_[0], b_[0]], None)
            bind(name, (idx, a_[1], None))
            continue
        if kind == "batchnorm":
            sc = t(name + ".gamma") / np.sqrt(t(name + ".moving_variance") + float(ly.get("eps", 1e-3)))
            sh = t(name + ".beta") - t(name + ".moving_mean") * sc
            idx = new_node("affine", [n0], None, off=[blob.put(sc), blob.put(sh)])
            bind(name, (idx, shape0, None))
            continue
        if kind in ("activation", "relu", "leakyrelu"):
            if kind == "relu":
                act, alpha = _lib.AA_GACT["relu"], 0.0
            elif kind == "leakyrelu":
                act, alpha = _lib.AA_GACT["leaky"], float(ly.get("alpha", 0.3))
            else:
                act = act_code(ly["fn"])
                alpha = 0.2 if act == _lib.AA_GACT["leaky"] else 0.0
            # fuse into the producer when it is a fresh node we own alone
            if n0 >= 0 and nodes[n0]["act"] == 0 and node_consumers(n0) == 1 and \
                    nodes[n0]["op"] != _lib.AA_G["pow"]:
                nodes[n0]["act"], nodes[n0]["alpha"] = act, alpha
                bind(name, (n0, shape0, None))
            else:
                idx = new_node("affine", [n0], None, act=act, alpha=alpha)
                bind(name, (idx, shape0, None))
            continue
        if kind == "rescaling":
            sc = np.broadcast_to(np.asarray(ly.get("scale", 1.0), np.float64), (C,))
            of = np.broadcast_to(np.asarray(ly.get("offset", 0.0), np.float64), (C,))
            idx = new_node("affine", [n0], None, off=[blob.put(sc), blob.put(of)])
            bind(name, (idx, shape0, None))
            continue
        if kind == "normalization":
            mean = np.broadcast_to(t(name + ".mean").reshape(-1), (C,))
            var = np.broadcast_to(t(name + ".variance").reshape(-1), (C,))
            sc = 1.0 / np.maximum(np.sqrt(var), 1e-7)  # keras: (x - mean) / max(sqrt(var), epsilon)
            idx = new_node("affine", [n0], None, off=[blob.put(sc), blob.put(-mean * sc)])
            bind(name, (idx, shape0, None))
            continue
        if kind == "magtransform":
            a = float(np.asarray(tensors[name + ".a"], np.float32).reshape(-1)[0])
            e = float(np.float32(1.0) / (np.float32(1.0) + np.exp(np.float32(-a))))
            idx = new_node("pow", [n0], None, alpha=e)
            bind(name, (idx, shape0, None))
            continue
        if kind == "dense":
            Co = int(ly["units"])
            kern = t(name + ".kernel").reshape(-1, Co)
            if kern.shape[0] != H * W * C:
                raise ValueError(f"{name}: Dense kernel for {kern.shape[0]} inputs, map has {H * W * C}")
            bias = t(name + ".bias") if ly.get("use_bias", True) else None
            act = act_code(ly.get("activation"))
            idx = new_node("dense", [n0], None, filters=Co, act=act, alpha=0.2 if act == 2 else 0.0,
                           off=[blob.put(kern), blob.put(bias) if bias is not None else -1])
            bind(name, (idx, (1, 1, Co), None))
            continue
        raise NotImplementedError(f"layer {name}: type {kind} has no graph kernel")
    last = out_of[names[-1]]
    if last[0] < 0:
        raise ValueError("the graph computes nothing")
    if last[0] != len(nodes) - 1:  # the output must be the last node
        nodes.append(dict(op=_lib.AA_G["affine"], in0=last[0], in1=-1, kh=1, kw=1, sh=1, sw=1, pt=0, pb=0, pl=0,
                          pr=0, filters=0, act=0, alpha=0.0, off=[-1, -1]))
    arr = (_lib.Node * len(nodes))()
    for k, d in enumerate(nodes):
        for f in ("op", "in0", "in1", "kh", "kw", "sh", "sw", "pt", "pb", "pl", "pr", "filters", "act"):
            setattr(arr[k], f, int(d[f]))
        arr[k].alpha = float(d["alpha"])
        arr[k].off[0], arr[k].off[1] = int(d["off"][0]), int(d["off"][1])
    H, W, C = last[1]
    return arr, blob.array(), H * W * C
