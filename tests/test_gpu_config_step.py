"""GPU parity of the exact step bench.py times (BASELINE.json configs[1]):
64 windows (39 of 60 s clip A + 25 of clip B, bench.make_batch), htk log-mel
n_fft 4096 / hop 640 / 160 bands, model1 -- every precision mode against the
CPU oracle (oracle.fe_oracle window_logmel + oracle.cnn_oracle fp32 forward on
the same PCM windows).

Gates: log-mel <= 1e-3 dB; logits <= 1e-3 in the gated modes (bf16x3, the
headline and classify() default, and f32).  bf16 / fp8 deltas are reported and
bounded loosely (they are throughput modes, BASELINE configs[1]/[4]).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3
DB_TOL = 1e-3
LOOSE = {"bf16": 0.25, "fp8": 2.0}


@pytest.fixture(scope="module")
def step(gpu, tmp_path_factory):
    import bench
    from aa_amd.frontend import FeSettings, FrontEnd
    from oracle import cnn_oracle, fe_oracle
    from tools.make_models import make_model

    fe_s = FeSettings(htk=True, hop_length=640, n_fft=4096, n_mels=160, break_freq=1750)
    pcm_np, rows_np, views = bench.make_batch(0, fe_s)
    assert rows_np.shape[0] == 64
    path = make_model(tmp_path_factory.mktemp("cfg1") / "model1", "model1", seed=1)
    fe = FrontEnd(fe_s, gpu)
    logmel = fe.run(torch.from_numpy(pcm_np).to(gpu), torch.from_numpy(rows_np).to(gpu))
    torch.cuda.synchronize()
    cfg = bench.fe_config(fe_s)
    ref_mel = np.stack([fe_oracle.window_logmel(bench.window_samples(pcm_np, v, fe_s.win_len), cfg)
                        for v in views])
    ref_logits, _ = cnn_oracle.forward(path, ref_mel)
    return dict(path=path, logmel=logmel, ref_mel=ref_mel, ref_logits=ref_logits)


def test_config1_logmel(step):
    err = float(np.abs(step["logmel"].cpu().numpy() - step["ref_mel"]).max())
    print(f"configs[1] log-mel max|d| = {err:.3e} dB")
    assert err <= DB_TOL


@pytest.mark.parametrize("precision", ["bf16x3", "f32", "bf16", "fp8"])
def test_config1_logits(step, gpu, precision):
    from aa_amd.model import Model
    m = Model(step["path"], step["logmel"].shape[1:], precision=precision, device=gpu)
    lg, _ = m.forward(step["logmel"])
    torch.cuda.synchronize()
    d = np.abs(lg.cpu().numpy() - step["ref_logits"])
    print(f"configs[1] {precision}: max|dlogit| = {d.max():.3e} (mean {d.mean():.3e})")
    assert np.isfinite(d).all()
    assert d.max() <= LOOSE.get(precision, LOGIT_TOL)


# ---- BASELINE configs[4]: fp16 log-mel + fp8 CNN (throughput-ceiling mode) ----

def test_config4_logmel_f16_is_rounded_f32(step, gpu):
    """aa_fe_config.out_f16: fe_db rounds the same f32 dB values to float16
    (round to nearest), so the fp16 log-mel is bit-identical to the f32 one
    cast to half."""
    import bench
    from aa_amd.frontend import FeSettings, FrontEnd
    fe_s = FeSettings(htk=True, hop_length=640, n_fft=4096, n_mels=160, break_freq=1750)
    pcm_np, rows_np, _ = bench.make_batch(0, fe_s)
    fe16 = FrontEnd(fe_s, gpu, out_dtype=torch.float16)
    lm16 = fe16.run(torch.from_numpy(pcm_np).to(gpu), torch.from_numpy(rows_np).to(gpu))
    torch.cuda.synchronize()
    assert lm16.dtype == torch.float16
    assert torch.equal(lm16, step["logmel"].half())


@pytest.mark.parametrize("precision", ["bf16x3", "fp8"])
def test_config4_f16_input_equals_f32_of_same_values(step, gpu, precision):
    """A float16 model input is widened to f32 exactly where the fused first
    conv stages it: logits equal those of the f32 tensor holding the same
    (half-rounded) values, bit for bit."""
    from aa_amd.model import Model
    lm16 = step["logmel"].half()
    m = Model(step["path"], lm16.shape[1:], precision=precision, device=gpu)
    a, _ = m.forward(lm16)
    b, _ = m.forward(lm16.float())
    c, _ = m.forward(lm16)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c)


def test_config4_step(step, gpu):
    """configs[4]'s step: fp16 log-mel -> fp8 CNN.  Against the fp8 CPU
    emulation fed the same half-rounded log-mel (gate: the fp8 bounds of
    test_gpu_cnn.py), and the delta to the fp32 oracle reported."""
    from aa_amd.model import Model
    from oracle import cnn_oracle
    from tests.test_gpu_cnn import FP8_EMU_MAX, FP8_EMU_MEAN, FP8_F32EMU_MAX, FP8_F32EMU_MEAN
    lm16 = step["logmel"].half()
    m = Model(step["path"], lm16.shape[1:], precision="fp8", device=gpu)
    lg, _ = m.forward(lm16)
    torch.cuda.synchronize()
    lg = lg.cpu().numpy()
    x16 = lm16.float().cpu().numpy()
    # all 64 windows against the f32-conv emulation, 3 against the MFMA-sum one
    elg, _ = cnn_oracle.forward_fp8_emulated(step["path"], x16, mfma=False)
    mlg, _ = cnn_oracle.forward_fp8_emulated(step["path"], x16[:3])
    d_emu, d_mfma = np.abs(lg - elg), np.abs(lg[:3] - mlg)
    d_ref = np.abs(lg - step["ref_logits"])
    print(f"configs[4] fp16 log-mel + fp8: max|dlogit| vs the MFMA emulation {d_mfma.max():.3e} (mean {d_mfma.mean():.3e}), "
          f"vs the f32-conv emulation {d_emu.max():.3e} (mean {d_emu.mean():.3e}), "
          f"vs fp32 oracle {d_ref.max():.3e} (mean {d_ref.mean():.3e})")
    assert np.isfinite(lg).all()
    assert d_mfma.max() <= FP8_EMU_MAX and d_mfma.mean() <= FP8_EMU_MEAN
    assert d_emu.max() <= FP8_F32EMU_MAX and d_emu.mean() <= FP8_F32EMU_MEAN
    assert d_ref.max() <= LOOSE["fp8"]


def test_f16_input_needs_fused_first_conv(gpu, tmp_path):
    """Only the fused first conv reads a float16 input: another first layer
    refuses it (AA_ERR_UNSUPPORTED) instead of misreading the buffer."""
    from aa_amd import _lib
    from aa_amd.model import Model
    from tools.make_models import make_model
    path = make_model(tmp_path / "m2", "model2", seed=2)  # C_in = 1 first conv, then a pooled 3x3/32: fused
    Model(path, (160, 226, 1), precision="fp8", device=gpu).forward(torch.zeros(1, 160, 226, 1, dtype=torch.float16,
                                                                             device=gpu))
    import json
    from safetensors.numpy import load_file, save_file
    from safetensors import safe_open
    with safe_open(str(path), "np") as f:
        meta = f.metadata()
    arch = json.loads(meta["arch"])
    # drop the fusing pattern: make the second conv unpooled
    for i, ly in enumerate(arch):
        if ly["type"] == "maxpool2d":
            del arch[i]
            break
    meta["arch"] = json.dumps(arch)
    p2 = tmp_path / "m3" / "audioModel.safetensors"
    p2.parent.mkdir()
    save_file(load_file(str(path)), str(p2), metadata=meta)
    for fn in ("metadata.txt",):
        if (path.parent / fn).exists():
            (p2.parent / fn).write_text((path.parent / fn).read_text())
    m = Model(p2, (160, 226, 1), precision="bf16x3", device=gpu)
    with pytest.raises(_lib.AAError):
        m.forward(torch.zeros(1, 160, 226, 1, dtype=torch.float16, device=gpu))
