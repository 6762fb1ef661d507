"""Streamed multi-recording runner (aa_amd/stream.py, BASELINE.json configs[2])
against classifying each recording on its own through the same kernels:
per-track ensemble means must be bit-identical (every kernel works per window /
per track; the batch only changes which buffer a window lives in)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class T:
    def __init__(self, start, end, f0=0, f1=24000):
        self.start, self.end, self.freq_start, self.freq_end = start, end, f0, f1

    @property
    def length(self):
        return self.end - self.start


def test_stream_matches_per_recording(gpu, model_root):
    from aa_amd.frontend import FeSettings, FrontEnd, pack_windows
    from aa_amd.model import Model, track_mean
    from aa_amd.stream import Recording, StreamRunner
    from aa_amd.windows import schedule
    s = FeSettings(htk=True, hop_length=640, n_fft=4096, n_mels=160, break_freq=1750)
    paths = [model_root / m / "audioModel.safetensors" for m in ("model1", "model2", "model3")]
    rng = np.random.default_rng(5)
    recs = []
    for i in range(7):
        n = int(rng.integers(4, 12) * 48000 + rng.integers(0, 48000))
        pcm = (rng.standard_normal(n) * 0.1).astype(np.float32)
        secs = n / 48000
        tracks = [T(0, secs), T(secs * 0.25, secs * 0.6), T(secs * 0.9, secs)]
        recs.append(Recording(key=i, pcm=pcm, tracks=tracks))
    np.random.seed(3)  # short tracks draw a random offset, in recording order
    runner = StreamRunner(paths, s, precision="bf16", device=gpu, max_windows=40, max_samples=40 * 48000)
    got = {(k, t): v for k, t, v in runner.run(recs)}
    fe = FrontEnd(s, gpu)
    models = [Model(p, fe.out_shape(1)[1:], precision="bf16", device=gpu) for p in paths]
    np.random.seed(3)
    n_tracks = 0
    for r in recs:
        views = schedule(len(r.pcm), 48000, r.tracks, 3, 1.5, s.fmin, s.fmax, False)
        flat = [v for tv in views for v in tv]
        pcm = torch.from_numpy(r.pcm).to(gpu)
        lm = fe.run(pcm, torch.from_numpy(pack_windows(flat, len(r.pcm))).to(gpu))
        probs = torch.stack([m.forward(lm)[1] for m in models])
        counts = [len(tv) for tv in views]
        sel = [i for i, c in enumerate(counts) if c]
        begin = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
        means = track_mean(probs, torch.from_numpy(begin[sel]).to(gpu),
                           torch.from_numpy(np.asarray(counts, np.int32)[sel]).to(gpu)).cpu().numpy()
        for row, ti in enumerate(sel):
            assert np.array_equal(got[(r.key, ti)], means[row]), (r.key, ti)
            n_tracks += 1
    assert n_tracks == len(got) and n_tracks >= 14


def test_stream_matches_oracle(gpu, model_root):
    """BASELINE configs[2] against the CPU oracle: 8 full 60 s clips (39
    windows each) through StreamRunner with the model1+2+3 ensemble in the
    default (gated) split-bf16 precision; per-track means over models and
    windows within 1e-3 of oracle.fe_oracle + oracle.cnn_oracle (fp32)."""
    from oracle import cnn_oracle, fe_oracle
    from aa_amd.frontend import FeSettings
    from aa_amd.stream import Recording, StreamRunner
    from aa_amd.windows import schedule
    from tools import synth
    import bench
    s = FeSettings(htk=True, hop_length=640, n_fft=4096, n_mels=160, break_freq=1750)
    paths = [model_root / m / "audioModel.safetensors" for m in ("model1", "model2", "model3")]
    recs = [Recording(key=i, pcm=synth.clip(500 + i), tracks=[T(0, 60.0)]) for i in range(8)]
    runner = StreamRunner(paths, s, device=gpu, max_windows=4 * 39, max_samples=4 * 2_880_000)
    assert all(m.precision == "bf16x3" for m in runner.models)
    got = {k: v for k, _, v in runner.run(recs)}
    cfg = bench.fe_config(s)
    worst = 0.0
    for r in recs:
        (views,) = schedule(len(r.pcm), 48000, r.tracks, 3, 1.5, s.fmin, s.fmax, False)
        assert len(views) == 39
        mel = np.stack([fe_oracle.window_logmel(bench.window_samples(r.pcm, v, s.win_len), cfg) for v in views])
        probs = np.stack([cnn_oracle.forward(p, mel)[1] for p in paths])
        ref = np.mean(np.mean(probs, axis=0), axis=0)
        worst = max(worst, float(np.abs(got[r.key] - ref).max()))
    print(f"configs[2] 8 x 60 s, 3-model ensemble: max|d track mean| = {worst:.3e}")
    assert worst <= 1e-3
