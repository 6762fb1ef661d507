"""Graph planning (aa_amd.graph.graph_table) keeps the network's meaning:
the aa_node list it hands to aa_graph_create -- BatchNormalization folded
into convs, activations fused, ZeroPadding2D and TF "same" padding resolved
into explicit pads, squeeze-excite broadcast multiplies, residual adds --
evaluated here in float64 by a literal CPU reading of include/aa.h's node
semantics, equals the un-fused Keras-semantics oracle
(oracle/cnn_oracle.py) on the same input."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from aa_amd import _lib
from aa_amd.graph import graph_table, is_graph
from aa_amd.model import read_arch
from oracle import cnn_oracle
from tools.make_models import calibration_input, make_chain, make_graph

OPS = {v: k for k, v in _lib.AA_G.items()}


def _act(x, a, alpha):
    return [lambda v: v, F.relu, lambda v: F.leaky_relu(v, alpha), torch.sigmoid,
            lambda v: v * torch.sigmoid(v)][a](x)


def run_nodes(nodes, blob, x):
    """include/aa.h aa_node semantics in torch float64 (NCHW)."""
    b = torch.from_numpy(blob.astype(np.float64))
    outs = []
    for i, d in enumerate(nodes):
        op = OPS[d.op]
        a = x if d.in0 < 0 else outs[d.in0]
        act = 0 if (i == len(nodes) - 1 and d.act == 3) else d.act  # logits before the final sigmoid
        if op in ("conv", "dwconv", "maxpool", "avgpool"):
            p = F.pad(a, (d.pl, d.pr, d.pt, d.pb), value=-float("inf") if op == "maxpool" else 0.0)
            if op == "conv":
                C = a.shape[1]
                w = b[d.off[0]:d.off[0] + d.kh * d.kw * C * d.filters].reshape(d.kh, d.kw, C, d.filters)
                y = F.conv2d(p, w.permute(3, 2, 0, 1), b[d.off[1]:d.off[1] + d.filters] if d.off[1] >= 0 else None,
                             stride=(d.sh, d.sw))
            elif op == "dwconv":
                C = a.shape[1]
                w = b[d.off[0]:d.off[0] + d.kh * d.kw * C].reshape(d.kh, d.kw, C).permute(2, 0, 1)[:, None]
                y = F.conv2d(p, w, b[d.off[1]:d.off[1] + C] if d.off[1] >= 0 else None, stride=(d.sh, d.sw),
                             groups=C)
            elif op == "maxpool":
                y = F.max_pool2d(p, (d.kh, d.kw), (d.sh, d.sw))
            else:
                one = F.pad(torch.ones_like(a[:, :1]), (d.pl, d.pr, d.pt, d.pb))
                y = F.avg_pool2d(p, (d.kh, d.kw), (d.sh, d.sw), divisor_override=1) / \
                    F.avg_pool2d(one, (d.kh, d.kw), (d.sh, d.sw), divisor_override=1)
        elif op in ("gmaxpool", "gavgpool"):
            y = (a.mean(dim=(2, 3)) if op == "gavgpool" else a.amax(dim=(2, 3)))[:, :, None, None]
        elif op in ("add", "mul"):
            c = x if d.in1 < 0 else outs[d.in1]
            y = a + c if op == "add" else a * c
        elif op == "affine":
            C = a.shape[1]
            y = a
            if d.off[0] >= 0:
                y = y * b[d.off[0]:d.off[0] + C][None, :, None, None]
            if d.off[1] >= 0:
                y = y + b[d.off[1]:d.off[1] + C][None, :, None, None]
        elif op == "pow":
            y = torch.pow(a, d.alpha)
        elif op == "dense":
            flat = a.permute(0, 2, 3, 1).reshape(a.shape[0], -1)
            K = flat.shape[1]
            y = flat @ b[d.off[0]:d.off[0] + K * d.filters].reshape(K, d.filters)
            if d.off[1] >= 0:
                y = y + b[d.off[1]:d.off[1] + d.filters]
            y = y[:, :, None, None]
        y = _act(y, act, d.alpha)
        outs.append(y)
    o = outs[-1]
    return o.permute(0, 2, 3, 1).reshape(o.shape[0], -1).numpy()


@pytest.mark.parametrize("kind,ch", [("effnet", 1), ("effnet", 3), ("resnet", 3)])
def test_graph_plan_equals_keras_semantics(tmp_path, kind, ch):
    p = make_graph(tmp_path / kind, kind, in_channels=ch, T=113)
    arch, tensors = read_arch(p)
    assert is_graph(arch)
    x = calibration_input(3, 160, 113, True, np.random.default_rng(1))
    if ch > 1:
        x = np.repeat(x, ch, axis=3)
    nodes, blob, L = graph_table(arch, tensors, x.shape[1:])
    got = run_nodes(nodes, blob, torch.from_numpy(x).double().permute(0, 3, 1, 2))
    ref, _ = cnn_oracle.forward(p, x, dtype=torch.float64)
    assert got.shape == ref.shape == (3, L)
    assert np.abs(got - ref).max() < 1e-5 * max(1.0, np.abs(ref).max())
    ops = [OPS[n.op] for n in nodes]
    if kind == "effnet":
        assert ops.count("dwconv") == 3 and ops.count("mul") == 3 and ops.count("add") == 1
        assert "affine" not in ops  # every BatchNormalization folded, every activation fused


def test_chains_stay_on_the_tuned_planner(tmp_path):
    p = make_chain(tmp_path / "c", [(32, (3, 3), None), (64, (3, 3), (3, 3))])
    arch, _ = read_arch(p)
    assert not is_graph(arch)
