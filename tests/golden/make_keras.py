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
np.savez(os.path.join(OUT, "expected.npz"), **expected)
print("wrote", sorted(os.listdir(OUT)))
