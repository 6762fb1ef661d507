"""``.keras`` import (aa_amd/keras_import.py) on fixtures whose HDF5 part was
written by the real HDF5 library in the Keras 3 layout
(tests/golden/make_keras.py).  CPU: layer mapping, weight placement and the
snake_case / counter naming of the weights file.  GPU: the imported networks
(generic-kernel shapes, MaxPool 2x2 / 3x2, a 5-label 1x1 head, a Dense head)
through libaa.so against the CPU oracle."""
import json
import shutil
from pathlib import Path

import numpy as np
import pytest

from aa_amd import keras_import

D = Path(__file__).parent / "golden" / "keras"
EXP = dict(np.load(D / "expected.npz"))


def _exp(fixture, layer, i):
    return EXP[f"{fixture}|{layer}|{i}"]


def test_snake_case_names():
    assert [keras_import.snake(c) for c in ("Conv2D", "BatchNormalization", "LeakyReLU", "MaxPooling2D",
                                             "GlobalMaxPooling2D", "MagTransform", "ReLU", "Dense")] == \
        ["conv2d", "batch_normalization", "leaky_re_lu", "max_pooling2d", "global_max_pooling2d", "mag_transform",
         "re_lu", "dense"]


def test_head1x1_mapping():
    arch, t, in_shape = keras_import.read_keras(D / "head1x1.keras")
    assert in_shape == (40, 50, 1)
    assert [a["type"] for a in arch] == ["magtransform", "conv2d", "batchnorm", "leakyrelu", "maxpool2d", "conv2d",
                                         "relu", "maxpool2d", "conv2d", "globalmaxpool2d", "activation"]
    assert arch[3]["alpha"] == 0.25 and arch[4]["pool"] == [2, 2] and arch[7]["pool"] == [3, 3]
    np.testing.assert_array_equal(t["mag_transform.a"], _exp("head1x1", "mag_transform", 0))
    np.testing.assert_array_equal(t["c1.kernel"], _exp("head1x1", "c1", 0))
    for i, k in enumerate(("gamma", "beta", "moving_mean", "moving_variance")):
        np.testing.assert_array_equal(t[f"bn1.{k}"], _exp("head1x1", "bn1", i))
    np.testing.assert_array_equal(t["c2.bias"], _exp("head1x1", "c2", 1))
    np.testing.assert_array_equal(t["head.kernel"], _exp("head1x1", "head", 0))


def test_dense_mapping_and_oracle():
    from oracle import cnn_oracle
    arch, t, _ = keras_import.read_keras(D / "dense.keras")
    assert [a["type"] for a in arch][-3:] == ["globalmaxpool2d", "dense", "activation"]
    assert arch[-2]["units"] == 5
    np.testing.assert_array_equal(t["dense.kernel"], _exp("dense", "dense", 0))
    x = np.random.default_rng(0).standard_normal((2, 40, 50, 1)).astype(np.float32)
    lg, pr = cnn_oracle.forward(arch, x, tensors=t)
    assert lg.shape == (2, 5) and np.all((pr > 0) & (pr < 1))
    np.testing.assert_allclose(pr, 1 / (1 + np.exp(-lg)), rtol=1e-6)


def test_unsupported_layer_named(tmp_path):
    import zipfile
    src = zipfile.ZipFile(D / "dense.keras")
    cfg = json.loads(src.read("config.json"))
    cfg["config"]["layers"].insert(2, {"class_name": "Conv2DTranspose", "config": {"name": "up"}})
    out = tmp_path / "m.keras"
    with zipfile.ZipFile(out, "w") as z:
        for n in src.namelist():
            z.writestr(n, json.dumps(cfg) if n == "config.json" else src.read(n))
    with pytest.raises(NotImplementedError, match="Conv2DTranspose"):
        keras_import.read_keras(out)


def test_functional_graph_mapping():
    """A Keras 3 Functional DAG (Rescaling, same / strided convs, a nested
    Sequential block, squeeze-excite Multiply, ZeroPadding2D, residual Add,
    average / max pools, GlobalAveragePooling2D, Dense): every layer names its
    inputs, the nested block's weights come from layers/sequential/layers/...,
    and the graph plan evaluates to the oracle's Keras semantics."""
    import torch
    from aa_amd.graph import graph_table, is_graph
    from oracle import cnn_oracle
    from test_graph import run_nodes
    arch, t, in_shape = keras_import.read_keras(D / "graph.keras")
    assert in_shape == (24, 30, 1) and is_graph(arch)
    types = [a["type"] for a in arch]
    assert types[:2] == ["rescaling", "conv2d"] and "depthwise_conv2d" in types and "multiply" in types
    by = {a["name"]: a for a in arch}
    assert by["block/dw"]["inputs"] == ["stem_act"] and by["se_excite"]["inputs"] == ["block/dw_act", "se_expand/sigmoid"]
    assert by["res"]["inputs"] == ["down_relu", "proj"] and by["stem"]["strides"] == [2, 2]
    assert by["pad"]["pad"] == [[0, 1], [0, 1]] and by["mx"]["padding"] == "same"
    np.testing.assert_array_equal(t["block/dw.kernel"], _exp("graph", "dw", 0))
    np.testing.assert_array_equal(t["block/dw_bn.moving_variance"], _exp("graph", "dw_bn", 3))
    np.testing.assert_array_equal(t["proj.bias"], _exp("graph", "proj", 1))
    np.testing.assert_array_equal(t["out.kernel"], _exp("graph", "out", 0))
    x = np.random.default_rng(2).normal(-40, 10, (3,) + in_shape).astype(np.float32)
    nodes, blob, L = graph_table(arch, t, in_shape)
    got = run_nodes(nodes, blob, torch.from_numpy(x).double().permute(0, 3, 1, 2))
    ref, _ = cnn_oracle.forward(arch, x, tensors=t, dtype=torch.float64)
    assert L == 5 and np.abs(got - ref).max() < 1e-6  # (folded weights stored as f32)


def _model_dir(tmp_path, fixture, labels):
    d = tmp_path / fixture
    d.mkdir()
    shutil.copy(D / f"{fixture}.keras", d / "audioModel.keras")
    (d / "metadata.txt").write_text(json.dumps({"name": fixture, "labels": labels}))
    return d / "audioModel.keras"


@pytest.mark.gpu
@pytest.mark.parametrize("fixture", ["head1x1", "dense", "graph"])
@pytest.mark.parametrize("precision", ["f32", "bf16x3", "bf16"])
def test_keras_model_on_gpu(gpu, tmp_path, fixture, precision):
    import torch
    from aa_amd.model import Model
    from oracle import cnn_oracle
    path = _model_dir(tmp_path, fixture, [f"l{i}" for i in range(5)])
    arch, t, in_shape = keras_import.read_keras(path)
    rng = np.random.default_rng(3)
    x = np.abs(rng.standard_normal((4,) + in_shape)).astype(np.float32)  # MagTransform needs x >= 0
    if fixture == "graph":
        x = (-80.0 * x / x.max()).astype(np.float32)  # dB-like
    m = Model(path, in_shape, precision=precision, device=gpu)
    lg, _ = m.forward(torch.from_numpy(x).to(gpu))
    torch.cuda.synchronize()
    ref, _ = cnn_oracle.forward(arch, x, tensors=t)
    d = float(np.abs(lg.cpu().numpy() - ref).max())
    print(f"{fixture} {precision}: stages {[m.stage_info(i)[0] for i in range(m.n_stages())]} max|dlogit| {d:.2e}")
    assert d <= (0.1 if precision == "bf16" and fixture != "graph" else 1e-3)  # (graphs run bf16 as split-bf16)
