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
