"""configs[0] on the build side: the analyse.py CLI on a short recording
(reference src/analyse.py:434-470 -> species_identify :129-175) through the
GPU path, JSON out.  Checked: the reference's keys and version strings, the
-o output equals the sidecar the default mode writes, and every track's tags
agree with the same pipeline in exact f32 MFMA mode (labels identical,
confidences within 1 point: round(100 p) flips only where p sits on a
rounding boundary)."""
import io
import json
from contextlib import redirect_stdout

import pytest

pytestmark = pytest.mark.gpu


def _run(argv):
    import numpy as np
    from aa_amd import analyse
    np.random.seed(0)  # short tracks draw random window offsets (src/identify_tracks.py:132, :167)
    buf = io.StringIO()
    with redirect_stdout(buf):
        analyse.main(argv)
    return buf.getvalue()


def test_cli_json_on_short_wav(gpu, model_root, tmp_path):
    import os
    from tools import synth
    wav = tmp_path / "morepork.wav"
    synth.write_wav(wav, synth.clip(42, seconds=15.0))
    models = [str(model_root / m / "audioModel.keras") for m in ("model1", "model2")]
    argv = [str(wav)] + sum((["--bird-model", m] for m in models), [])
    out = json.loads(_run(argv + ["-o"]))
    for k in ("species_identify", "species_identify_version", "non_bird_tags", "duration",
              "cacophony_index", "cacophony_index_version", "chirps", "processing_time_seconds"):
        assert k in out, k
    assert out["species_identify_version"] == "2025-12-01"
    assert abs(out["duration"] - 15.0) < 1e-9
    assert out["species_identify"], "signals on the synthetic chirps give tracks"
    # default mode: the sidecar FILE.txt["analysis_result"]
    _run(argv)
    side = json.loads(wav.with_suffix(".txt").read_text())["analysis_result"]
    drop = lambda d: {k: v for k, v in d.items() if k != "processing_time_seconds"}
    assert drop(side) == drop(out)
    # the same recording with exact-f32 convolutions
    from aa_amd.pipeline import Classifier
    os.environ["AA_PRECISION"] = "f32"
    try:
        Classifier._shared.clear()
        ref = json.loads(_run(argv + ["-o"]))
    finally:
        os.environ.pop("AA_PRECISION")
        Classifier._shared.clear()
    assert len(ref["species_identify"]) == len(out["species_identify"])
    for a, b in zip(out["species_identify"], ref["species_identify"]):
        for ma, mb in zip(a["model_results"], b["model_results"]):
            pa = {p["label"]: p["confidence"] for p in ma.get("predictions", [])}
            pb = {p["label"]: p["confidence"] for p in mb.get("predictions", [])}
            assert pa.keys() == pb.keys()
            assert all(abs(pa[k] - pb[k]) <= 1 for k in pa)


def test_cli_track_scores_match_oracle(gpu, model_root, tmp_path, monkeypatch):
    """The per-track probabilities behind the CLI's JSON, in the default
    split-bf16 precision, against the CPU oracle: the same windows (the
    schedule the CLI drew, captured) through oracle.fe_oracle + cnn_oracle
    (fp32), np.mean over models then windows (src/identify_tracks.py:544-551),
    within the north-star 1e-3."""
    import numpy as np
    from pathlib import Path
    from oracle import cnn_oracle, fe_oracle
    from aa_amd import pipeline
    from tools import synth
    import bench
    wav = tmp_path / "morepork.wav"
    synth.write_wav(wav, synth.clip(43, seconds=20.0))
    models = [str(model_root / m / "audioModel.keras") for m in ("model1", "model2")]
    argv = [str(wav)] + sum((["--bird-model", m] for m in models), []) + ["-o"]
    seen = {"views": [], "scores": [], "pcm": [], "groups": []}
    sched, apply, batch = pipeline.schedule, pipeline.apply_group_scores, pipeline.Classifier.classify_batch

    def sched_w(*a, **k):
        out = sched(*a, **k)
        seen["views"].append(out[0] if k.get("return_spans") else out)
        return out

    def apply_w(tracks, idx, means, meta):
        seen["scores"].append((list(idx), np.array(means, np.float32)))
        return apply(tracks, idx, means, meta)

    def batch_w(self, pcm, sr, recs, groups, **k):
        seen["pcm"].append(pcm.cpu().numpy())
        seen["groups"].append(groups)
        return batch(self, pcm, sr, recs, groups, **k)

    monkeypatch.setattr(pipeline, "schedule", sched_w)
    monkeypatch.setattr(pipeline, "apply_group_scores", apply_w)
    monkeypatch.setattr(pipeline.Classifier, "classify_batch", batch_w)
    out = json.loads(_run(argv))
    assert out["species_identify"]
    assert len(seen["pcm"]) == 1 and len(seen["views"]) == 1 and len(seen["groups"][0]) == 1
    pcm, views, (group,) = seen["pcm"][0], seen["views"][0], seen["groups"][0]
    assert len(group) == 2  # model1 + model2: one mean ensemble
    s = pipeline.fe_settings_from_meta(group[0][1], 48000)
    cfg = bench.fe_config(s)
    paths = [Path(p).parent / "audioModel.safetensors" for p, _ in group]
    (idx, means), = seen["scores"]
    assert len(idx) >= 2
    worst = 0.0
    for row, ti in enumerate(idx):
        mel = np.stack([fe_oracle.window_logmel(bench.window_samples(pcm, v, s.win_len), cfg) for v in views[ti]])
        probs = np.stack([cnn_oracle.forward(p, mel)[1] for p in paths])
        ref = cnn_oracle.ensemble_track_mean(probs)
        worst = max(worst, float(np.abs(means[row] - ref).max()))
    print(f"CLI: {len(idx)} tracks, max|d track mean| vs oracle = {worst:.3e}")
    assert worst <= 1e-3
