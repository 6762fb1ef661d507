"""Graph models on the GPU (aa_graph_*, csrc/aa_graph.hip): EfficientNet-like
(depthwise conv, squeeze-excite, residual add, ZeroPadding2D + stride-2 valid
conv, swish, global average pooling, Dense) and ResNet-like (Rescaling,
Normalization, "same" stride-2 convs, max / average pools, residual add)
networks against the fp32 oracle (oracle/cnn_oracle.py, Keras semantics),
in split-bf16 (convs with C_in >= 16 on the runtime-shaped MFMA kernel) and
exact f32; gate max |delta logit| <= 1e-3."""
import numpy as np
import pytest
import torch

from oracle import cnn_oracle
from tools.make_models import calibration_input, make_graph

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3


@pytest.mark.parametrize("kind,ch,T", [("effnet", 1, 226), ("effnet", 3, 513), ("resnet", 3, 226),
                                       ("effnetv2", 3, 226)])
@pytest.mark.parametrize("precision", ["bf16x3", "f32"])
def test_graph_model_matches_oracle(gpu, tmp_path, kind, ch, T, precision):
    from aa_amd.model import Model
    p = make_graph(tmp_path / kind, kind, in_channels=ch, T=T, seed=3)
    x = calibration_input(5, 160, T, True, np.random.default_rng(T))
    if ch > 1:
        x = np.repeat(x, ch, axis=3)
    m = Model(p, x.shape[1:], precision=precision)
    assert m.graph
    names = [m.stage_info(i)[0] for i in range(m.n_stages())]
    lg, pr = m.forward(torch.from_numpy(x).cuda())
    lg, pr = lg.cpu().numpy(), pr.cpu().numpy()
    rlg, rpr = cnn_oracle.forward(p, x)
    err = np.abs(lg - rlg).max()
    print(f"{kind} ch={ch} T={T} {precision}: max|dlogit| {err:.3e} (range {rlg.min():.2f}..{rlg.max():.2f}); "
          f"stages {names}")
    assert err <= LOGIT_TOL and np.abs(pr - rpr).max() <= LOGIT_TOL
    if precision == "bf16x3":
        assert any(n.startswith("conv_gx3_") for n in names)
    if kind == "effnet":
        assert sum(n.startswith("dwconv_") for n in names) == 3
    if kind == "effnetv2" and precision == "bf16x3":  # SE multiply / residual add fused into the convs
        assert any(n.endswith("+se") for n in names) and any("+add" in n for n in names)


def test_graph_fusions_are_bit_identical(gpu, tmp_path, monkeypatch):
    """The squeeze-excite Multiply and residual Add fused into the MFMA convs
    (graph_fuse) give exactly the unfused graph's logits."""
    from aa_amd.model import Model
    p = make_graph(tmp_path / "v2", "effnetv2", in_channels=3, T=160, seed=6)
    x = np.repeat(calibration_input(6, 160, 160, True, np.random.default_rng(2)), 3, axis=3)
    xt = torch.from_numpy(x).cuda()
    fused = Model(p, x.shape[1:])
    names = [fused.stage_info(i)[0] for i in range(fused.n_stages())]
    n_fused = sum(n.endswith("(fused)") for n in names)
    monkeypatch.setenv("AA_GRAPH_NOFUSE", "1")
    plain = Model(p, x.shape[1:])
    assert not any(plain.stage_info(i)[0].endswith("(fused)") for i in range(plain.n_stages()))
    a = fused.forward(xt)[0].cpu().numpy()
    b = plain.forward(xt)[0].cpu().numpy()
    print(f"{n_fused} nodes fused away")
    assert n_fused > 10 and np.array_equal(a, b)


def test_graph_model_large_batch_is_batch_invariant(gpu, tmp_path):
    from aa_amd.model import Model
    p = make_graph(tmp_path / "e", "effnet", in_channels=1, T=226, seed=4)
    x = calibration_input(40, 160, 226, True, np.random.default_rng(9))
    m = Model(p, x.shape[1:])
    xt = torch.from_numpy(x).cuda()
    a = m.forward(xt)[0].cpu().numpy()
    b = np.concatenate([m.forward(xt[i:i + 7])[0].cpu().numpy() for i in range(0, 40, 7)])
    assert np.array_equal(a, b)


def test_graph_capture_replay_matches_direct_launches(gpu, tmp_path):
    """aa_graph_forward replays a captured HIP graph of its launches (one per
    input / batch / workspace / output / stream); with node timing on it
    launches node by node.  Both give the same logits, and a replay after the
    input changed sees the new input."""
    from aa_amd.model import Model
    p = make_graph(tmp_path / "v2", "effnetv2", in_channels=3, T=160, seed=7)
    rng = np.random.default_rng(5)
    x = np.repeat(calibration_input(4, 160, 160, True, rng), 3, axis=3)
    m = Model(p, x.shape[1:])
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        xt = torch.from_numpy(x).cuda()
        lg = torch.empty((4, m.n_labels), dtype=torch.float32, device=xt.device)
        pr = torch.empty_like(lg)
        ws = m._workspace(4)
        run = lambda: m.forward(xt, lg, pr, workspace=ws)[0].cpu().numpy()
        a = run()      # node by node (first sight of these buffers)
        b = run()      # captured and launched
        b2 = run()     # replayed
        m.set_timing(True)
        c = run()      # node by node
        m.set_timing(False)
        xt.copy_(torch.from_numpy(np.repeat(calibration_input(4, 160, 160, True, rng), 3, axis=3)).cuda())
        d = run()      # replayed on the new input
        m.set_timing(True)
        e = run()
        m.set_timing(False)
    torch.cuda.synchronize()
    assert np.array_equal(a, b) and np.array_equal(a, b2) and np.array_equal(a, c)
    assert np.array_equal(d, e) and not np.array_equal(a, d)
