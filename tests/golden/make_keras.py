"""Write small Keras-3-layout ``.keras`` fixtures with the real HDF5 library,
to exercise aa_amd/keras_import.py (Keras/TF are not installed anywhere here;
h5py is, under /opt/conda/bin/python3.9):

    cd /tmp && /opt/conda/bin/python3.9 /root/repo/tests/golden/make_keras.py

Layout written (keras/src/saving/saving_lib.py of Keras 3): a zip with
metadata.json, config.json (Sequential: module / class_name / config /
registered_name per layer, InputLayer first) and model.weights.h5 with
layers/<snake_case class name>[_k]/vars/<i> datasets in model.layers order
(InputLayer excluded), plus an empty top-level vars/ group.  Outputs:
* keras/head1x1.keras  MagTransform(v2) conv3x3(1->8)+BN+LeakyReLU, MaxPool 2x2,
                       conv3x3(8->16, activation relu), Dropout, MaxPool 3x3,
                       conv1x1(16->5) + GlobalMaxPool2D + sigmoid
* keras/dense.keras    conv3x3(1->8, bias)+BN+ReLU, conv 5x3(8->12)+BN+LeakyReLU,
                       MaxPool 3x2, GlobalMaxPool2D, Dense(5, sigmoid)
* keras/expected.npz   every weight array by fixture and layer name
"""
import io
import json
import os
import zipfile

import h5py
import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "keras")
os.makedirs(OUT, exist_ok=True)
rng = np.random.default_rng(11)
expected = {}


def layer(cls, cfg, registered=None, module="keras.layers"):
    d = {"module": module, "class_name": cls, "config": cfg, "registered_name": registered}
    return d


def conv(name, f, k, act="linear", bias=False):
    return layer("Conv2D", {"name": name, "trainable": True, "dtype": "float32", "filters": f, "kernel_size": list(k),
                            "strides": [1, 1], "padding": "valid", "data_format": "channels_last",
                            "dilation_rate": [1, 1], "groups": 1, "activation": act, "use_bias": bias})


def bn(name):
    return layer("BatchNormalization", {"name": name, "axis": -1, "momentum": 0.99, "epsilon": 0.001,
                                        "center": True, "scale": True})


def write(fname, layers, weights, in_shape):
    cfg = {"module": "keras", "class_name": "Sequential",
           "config": {"name": "sequential", "trainable": True,
                      "layers": [layer("InputLayer", {"batch_shape": [None] + list(in_shape), "dtype": "float32",
                                                      "sparse": False, "name": "input_layer"})] + layers},
           "registered_name": None}
    h5 = io.BytesIO()
    with h5py.File(h5, "w") as f:
        f.create_group("vars")
        L = f.create_group("layers")
        used = {}
        for ly in layers:
            cls = ly["class_name"]
            snake = {"Conv2D": "conv2d", "BatchNormalization": "batch_normalization", "LeakyReLU": "leaky_re_lu",
                     "ReLU": "re_lu", "MaxPooling2D": "max_pooling2d", "GlobalMaxPooling2D": "global_max_pooling2d",
                     "Dense": "dense", "Dropout": "dropout", "Activation": "activation",
                     "MagTransform": "mag_transform"}[cls]
            k = used.get(snake, -1) + 1
            used[snake] = k
            path = snake if k == 0 else f"{snake}_{k}"
            v = L.create_group(path).create_group("vars")
            for i, a in enumerate(weights.get(ly["config"]["name"], [])):
                v.create_dataset(str(i), data=a)
                expected[f"{fname}|{ly['config']['name']}|{i}"] = a
    with zipfile.ZipFile(os.path.join(OUT, fname + ".keras"), "w") as z:
        z.writestr("metadata.json", json.dumps({"keras_version": "3.8.0", "date_saved": "2025-01-01@00:00:00"}))
        z.writestr("config.json", json.dumps(cfg))
        z.writestr("model.weights.h5", h5.getvalue())


def w(*shape, s=0.3):
    return (rng.standard_normal(shape) * s).astype(np.float32)


def bnw(c):
    return [1 + w(c, s=0.1), w(c, s=0.1), w(c, s=0.1), (0.5 + rng.random(c)).astype(np.float32)]


layers = [layer("MagTransform", {"name": "mag_transform", "trainable": True, "dtype": "float32"},
                registered="MyLayers>MagTransform", module=None),
          conv("c1", 8, (3, 3)), bn("bn1"), layer("LeakyReLU", {"name": "lr1", "negative_slope": 0.25}),
          layer("MaxPooling2D", {"name": "p1", "pool_size": [2, 2], "padding": "valid", "strides": [2, 2]}),
          conv("c2", 16, (3, 3), act="relu", bias=True),
          layer("Dropout", {"name": "drop", "rate": 0.3}),
          layer("MaxPooling2D", {"name": "p2", "pool_size": [3, 3], "padding": "valid", "strides": None}),
          conv("head", 5, (1, 1), bias=True),
          layer("GlobalMaxPooling2D", {"name": "gmp", "data_format": "channels_last", "keepdims": False}),
          layer("Activation", {"name": "act", "activation": "sigmoid"})]
weights = {"mag_transform": [np.array([-0.7], np.float32)], "c1": [w(3, 3, 1, 8)], "bn1": bnw(8),
           "c2": [w(3, 3, 8, 16), w(16, s=0.1)], "head": [w(1, 1, 16, 5), w(5, s=0.1)]}
write("head1x1", layers, weights, (40, 50, 1))

layers = [conv("c1", 8, (3, 3), bias=True), bn("bn1"), layer("ReLU", {"name": "r1"}),
          conv("c2", 12, (5, 3)), bn("bn2"), layer("LeakyReLU", {"name": "lr2", "negative_slope": 0.1}),
          layer("MaxPooling2D", {"name": "p", "pool_size": [3, 2], "padding": "valid", "strides": [3, 2]}),
          layer("GlobalMaxPooling2D", {"name": "gmp", "data_format": "channels_last", "keepdims": False}),
          layer("Dense", {"name": "dense", "units": 5, "activation": "sigmoid", "use_bias": True})]
weights = {"c1": [w(3, 3, 1, 8), w(8, s=0.1)], "bn1": bnw(8), "c2": [w(5, 3, 8, 12)], "bn2": bnw(12),
           "dense": [w(12, 5), w(5, s=0.1)]}
write("dense", layers, weights, (40, 50, 1))


# ---- graph.keras: a Keras 3 Functional DAG with a nested Sequential block --
def tensor(name):
    return {"class_name": "__keras_tensor__", "config": {"dtype": "float32", "keras_history": [name, 0, 0]}}


def node(cls, cfg, inputs, module="keras.layers"):
    d = layer(cls, cfg, module=module)
    d["name"] = cfg["name"]
    args = [[tensor(i) for i in inputs]] if len(inputs) > 1 else [tensor(i) for i in inputs]
    d["inbound_nodes"] = [{"args": args, "kwargs": {}}] if inputs else []
    return d


def gconv(name, f, k, strides=1, pad="valid", act="linear", bias=False):
    return {"name": name, "filters": f, "kernel_size": list(k), "strides": [strides, strides], "padding": pad,
            "data_format": "channels_last", "dilation_rate": [1, 1], "groups": 1, "activation": act,
            "use_bias": bias}


block = layer("Sequential", {"name": "block", "trainable": True, "layers": [
    layer("InputLayer", {"batch_shape": [None, 12, 15, 8], "dtype": "float32", "name": "block_in"}),
    layer("DepthwiseConv2D", {"name": "dw", "kernel_size": [3, 3], "strides": [1, 1], "padding": "same",
                              "depth_multiplier": 1, "data_format": "channels_last", "dilation_rate": [1, 1],
                              "activation": "linear", "use_bias": True}),
    bn("dw_bn"),
    layer("Activation", {"name": "dw_act", "activation": "silu"})]}, module="keras")
block["name"] = "block"
block["inbound_nodes"] = [{"args": [tensor("stem_act")], "kwargs": {}}]
glayers = [
    node("InputLayer", {"batch_shape": [None, 24, 30, 1], "dtype": "float32", "sparse": False, "name": "spec"}, []),
    node("Rescaling", {"name": "rescale", "scale": 1.0 / 40.0, "offset": 1.0}, ["spec"]),
    node("Conv2D", gconv("stem", 8, (3, 3), strides=2, pad="same"), ["rescale"]),
    node("BatchNormalization", bn("stem_bn")["config"], ["stem"]),
    node("Activation", {"name": "stem_act", "activation": "swish"}, ["stem_bn"]),
    block,
    node("GlobalAveragePooling2D", {"name": "se_squeeze", "data_format": "channels_last", "keepdims": True},
         ["block"]),
    node("Conv2D", gconv("se_reduce", 2, (1, 1), act="swish", bias=True), ["se_squeeze"]),
    node("Conv2D", gconv("se_expand", 8, (1, 1), act="sigmoid", bias=True), ["se_reduce"]),
    node("Multiply", {"name": "se_excite"}, ["block", "se_expand"]),
    node("ZeroPadding2D", {"name": "pad", "padding": [[0, 1], [0, 1]], "data_format": "channels_last"},
         ["se_excite"]),
    node("Conv2D", gconv("down", 12, (3, 3), strides=2), ["pad"]),
    node("BatchNormalization", bn("down_bn")["config"], ["down"]),
    node("ReLU", {"name": "down_relu"}, ["down_bn"]),
    node("Conv2D", gconv("proj", 12, (1, 1), bias=True), ["down_relu"]),
    node("Add", {"name": "res"}, ["down_relu", "proj"]),
    node("AveragePooling2D", {"name": "avg", "pool_size": [2, 2], "strides": [1, 1], "padding": "same"}, ["res"]),
    node("MaxPooling2D", {"name": "mx", "pool_size": [2, 2], "strides": [2, 2], "padding": "same"}, ["avg"]),
    node("GlobalAveragePooling2D", {"name": "gap", "data_format": "channels_last", "keepdims": False}, ["mx"]),
    node("Dropout", {"name": "drop", "rate": 0.2}, ["gap"]),
    node("Dense", {"name": "out", "units": 5, "activation": "sigmoid", "use_bias": True}, ["drop"]),
]
gweights = {"stem": [w(3, 3, 1, 8)], "stem_bn": bnw(8), "dw": [w(3, 3, 8, 1), w(8, s=0.1)], "dw_bn": bnw(8),
            "se_reduce": [w(1, 1, 8, 2), w(2, s=0.1)], "se_expand": [w(1, 1, 2, 8), w(8, s=0.1)],
            "down": [w(3, 3, 8, 12)], "down_bn": bnw(12), "proj": [w(1, 1, 12, 12), w(12, s=0.1)],
            "out": [w(12, 5), w(5, s=0.1)]}
cfg = {"module": "keras.src.models.functional", "class_name": "Functional",
       "config": {"name": "graph", "trainable": True, "layers": glayers, "input_layers": [["spec", 0, 0]],
                  "output_layers": [["out", 0, 0]]}, "registered_name": "Functional"}
h5 = io.BytesIO()
with h5py.File(h5, "w") as f:
    f.create_group("vars")

    def put_layers(grp, lys):
        used = {}
        for ly in lys:
            cls = ly["class_name"]
            if cls == "InputLayer":
                continue
            sn = {"Rescaling": "rescaling", "Conv2D": "conv2d", "BatchNormalization": "batch_normalization",
                  "Activation": "activation", "Sequential": "sequential", "DepthwiseConv2D": "depthwise_conv2d",
                  "GlobalAveragePooling2D": "global_average_pooling2d", "Multiply": "multiply",
                  "ZeroPadding2D": "zero_padding2d", "ReLU": "re_lu", "Add": "add",
                  "AveragePooling2D": "average_pooling2d", "MaxPooling2D": "max_pooling2d", "Dropout": "dropout",
                  "Dense": "dense"}[cls]
            k = used.get(sn, -1) + 1
            used[sn] = k
            g = grp.create_group(sn if k == 0 else f"{sn}_{k}")
            if cls == "Sequential":
                put_layers(g.create_group("layers"), ly["config"]["layers"])
                continue
            v = g.create_group("vars")
            for i, a in enumerate(gweights.get(ly["config"]["name"], [])):
                v.create_dataset(str(i), data=a)
                expected[f"graph|{ly['config']['name']}|{i}"] = a
    put_layers(f.create_group("layers"), glayers)
with zipfile.ZipFile(os.path.join(OUT, "graph.keras"), "w") as z:
    z.writestr("metadata.json", json.dumps({"keras_version": "3.8.0", "date_saved": "2025-01-01@00:00:00"}))
    z.writestr("config.json", json.dumps(cfg))
    z.writestr("model.weights.h5", h5.getvalue())

np.savez(os.path.join(OUT, "expected.npz"), **expected)
print("wrote", sorted(os.listdir(OUT)))
