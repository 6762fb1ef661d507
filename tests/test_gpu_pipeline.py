"""classify()'s model-group loop (aa_amd/pipeline.py, reference
src/identify_tracks.py:444-571) on the GPU against the CPU oracle, for the
routes beyond the plain one: band-pass filtered tracks (filter_freq /
filter_below, :152-162) and the efficientnet 3-channel repeat (:539-540).
Per-track means over models and windows within 1e-3 (default split-bf16)."""
from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _track(s, e, f0=0, f1=24000):
    return SimpleNamespace(start=s, end=e, freq_start=f0, freq_end=f1, length=e - s, results=[])


def _run(gpu, monkeypatch, frames, tracks, group, seed=5):
    from aa_amd import pipeline
    got = {}

    def capture(tr, sel, means, meta):
        for row, ti in enumerate(sel):
            got[ti] = means[row]
    monkeypatch.setattr(pipeline, "apply_group_scores", capture)
    np.random.seed(seed)
    pipeline.Classifier("bf16x3", device=gpu).classify_tracks(frames, 48000, tracks, [group])
    return got


def _oracle(frames, tracks, group, meta, channels_rep=1, seed=5):
    import bench
    from aa_amd.frontend import FeSettings
    from aa_amd.pipeline import fe_settings_from_meta
    from aa_amd.windows import filtered_sources, schedule
    from oracle import cnn_oracle, fe_oracle
    s = fe_settings_from_meta(meta, 48000)
    np.random.seed(seed)
    views, spans = schedule(len(frames), 48000, tracks, s.segment_length, 1.5, s.fmin, s.fmax, False,
                            return_spans=True)
    extra, views = filtered_sources(frames, 48000, tracks, views, spans, meta.get("filter_freq", False),
                                    meta.get("filter_below"), len(frames))
    buf = np.concatenate([frames, extra])
    cfg = bench.fe_config(s)
    out = {}
    for ti, tv in enumerate(views):
        if not tv:
            continue
        mel = np.stack([fe_oracle.window_logmel(bench.window_samples(buf, v, s.win_len), cfg) for v in tv])
        if channels_rep > 1:
            mel = np.repeat(mel, channels_rep, -1)
        probs = np.stack([cnn_oracle.forward(p.with_suffix(".safetensors"), mel)[1] for p, _ in group])
        out[ti] = np.mean(np.mean(probs, axis=0), axis=0)
    return out


def _model(tmp_path, name, **kw):
    import json
    from tools.make_models import make_model
    p = make_model(tmp_path / name, name=name, seed=4, **kw)
    meta = json.loads((p.parent / "metadata.txt").read_text())
    return p.with_suffix(".keras"), meta


@pytest.mark.parametrize("mode", ["filter_freq", "filter_below"])
def test_filtered_tracks_match_oracle(gpu, monkeypatch, tmp_path, mode):
    from tools import synth
    over = {"filter_freq": True} if mode == "filter_freq" else {"filter_below": 4000}
    path, meta = _model(tmp_path, "m_" + mode, meta_overrides=over)
    frames = synth.clip(21, seconds=12.0)
    tracks = [_track(0.5, 6.0, 800, 3000), _track(6.5, 11.0, 2000, 9000), _track(3.0, 4.0, 0, 2500)]
    group = [(path, meta)]
    got = _run(gpu, monkeypatch, frames, tracks, group)
    ref = _oracle(frames, tracks, group, meta)
    assert sorted(got) == sorted(ref) == [0, 1, 2]
    d = max(float(np.abs(got[k] - ref[k]).max()) for k in ref)
    print(f"{mode}: max|d track mean| = {d:.2e}")
    assert d <= 1e-3


def test_efficientnet_route_match_oracle(gpu, monkeypatch, tmp_path):
    from tools import synth
    path, meta = _model(tmp_path, "efficientnet_test", in_channels=3)
    frames = synth.clip(22, seconds=10.0)
    tracks = [_track(0.0, 10.0), _track(2.0, 4.5)]
    group = [(path, meta)]
    got = _run(gpu, monkeypatch, frames, tracks, group)
    ref = _oracle(frames, tracks, group, meta, channels_rep=3)
    d = max(float(np.abs(got[k] - ref[k]).max()) for k in ref)
    print(f"efficientnet route: max|d track mean| = {d:.2e}")
    assert sorted(got) == [0, 1] and d <= 1e-3
