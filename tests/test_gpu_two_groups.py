"""The CLI's default model layout: a mean-ensemble group plus a pre-model group
(reference src/analyse.py:414-418 runs `pre-model` + `bird-model-v2m`;
src/identify_tracks.py:444-465 splits the models on meta["pre_model"]).

The pre-model here asks for different STFT settings (hop 281) and has its own
labels, threshold and name.  The reference computes the windows once, with the
FIRST group's settings, and re-uses them for the pre-model group ("Re using
track data", :501-529); the pre-model then predicts on the mean group's
log-mel.  Through examine() (the GPU path: Classifier.classify_batch), checked:

* each group's per-track scores against the CPU oracle on the same windows
  (fe_oracle with the first group's settings, cnn_oracle fp32; np.mean over
  the group's models, then over windows, :544-551) within the north-star 1e-3;
* the JSON document against the one the post-processing (get_master_tag and
  species_identify, :580-647 and src/analyse.py:129-175; pinned byte for byte
  against the reference by tests/golden/postproc.json) gives on the ORACLE's
  scores: identical whenever no score sits within the tolerance of a
  threshold or a round(100 p) boundary.
"""
import copy
import json
import shutil

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pre_model_dir(model_root, tmp_path):
    """model3 re-labelled as the pre-model, with hop 281 in its metadata."""
    d = tmp_path / "pre-model"
    shutil.copytree(model_root / "model3", d)
    meta = json.loads((d / "metadata.txt").read_text())
    labels = list(meta["labels"])
    meta.update(name="pre-model", pre_model=True, hop_length=281, threshold=0.5,
                labels=labels[::-1])  # the same outputs under other names
    meta.pop("ebird_ids", None)
    (d / "metadata.txt").write_text(json.dumps(meta))
    return d


def _near_boundary(means, thr, tol=2e-3):
    p = np.asarray(means, np.float64)
    frac = 100 * p - np.floor(100 * p)
    return bool(np.any(np.abs(p - thr) < tol) or np.any(np.abs(frac - 0.5) < 100 * tol))


def test_mean_group_plus_pre_model(gpu, model_root, tmp_path, monkeypatch):
    from pathlib import Path
    from oracle import cnn_oracle, fe_oracle
    from aa_amd import analyse, pipeline
    from aa_amd import identify_tracks as it
    from tools import synth
    import bench
    wav = tmp_path / "rec.wav"
    synth.write_wav(wav, synth.clip(44, seconds=24.0))
    pre = _pre_model_dir(model_root, tmp_path)
    models = [str(model_root / "model1" / "audioModel.keras"), str(pre / "audioModel.keras"),
              str(model_root / "model2" / "audioModel.keras")]

    seen = {"views": [], "scores": [], "pcm": [], "groups": [], "res": []}
    sched, apply, batch, clf = (pipeline.schedule, pipeline.apply_group_scores,
                                pipeline.Classifier.classify_batch, analyse.classify)

    def sched_w(*a, **k):
        out = sched(*a, **k)
        seen["views"].append(out[0] if k.get("return_spans") else out)
        return out

    def apply_w(tracks, idx, means, meta):
        seen["scores"].append((list(idx), np.array(means, np.float32), meta))
        return apply(tracks, idx, means, meta)

    def batch_w(self, pcm, sr, recs, groups, **k):
        seen["pcm"].append(pcm.cpu().numpy())
        seen["groups"].append(groups)
        return batch(self, pcm, sr, recs, groups, **k)

    def classify_w(*a, **k):
        res = clf(*a, **k)
        # tracks before post-processing, without the GPU's model results
        tracks = []
        for t in res[0]:
            c = copy.copy(t)
            c.results = []
            tracks.append(c)
        seen["res"].append((tracks,) + tuple(res[1:]))
        return res

    monkeypatch.setattr(pipeline, "schedule", sched_w)
    monkeypatch.setattr(pipeline, "apply_group_scores", apply_w)
    monkeypatch.setattr(pipeline.Classifier, "classify_batch", batch_w)
    monkeypatch.setattr(analyse, "classify", classify_w)
    np.random.seed(0)
    doc = analyse.examine(str(wav), models, False)
    assert doc["species_identify"], "tracks from the synthetic chirps"

    # two groups: [model1, model2] (mean), then [pre-model]; the windows were
    # scheduled once, with the first group's settings
    (groups,) = seen["groups"]
    assert [len(g) for g in groups] == [2, 1] and groups[1][0][1]["pre_model"]
    assert len(seen["views"]) == 1 and len(seen["scores"]) == 2
    pcm, views = seen["pcm"][0], seen["views"][0]
    s = pipeline.fe_settings_from_meta(groups[0][0][1], 48000)
    assert s.hop_length == 640  # not the pre-model's 281
    cfg = bench.fe_config(s)
    oracle_means = []
    worst = 0.0
    for (idx, means, meta), group in zip(seen["scores"], groups):
        paths = [Path(p).parent / "audioModel.safetensors" for p, _ in group]
        ref_rows = []
        for row, ti in enumerate(idx):
            mel = np.stack([fe_oracle.window_logmel(bench.window_samples(pcm, v, s.win_len), cfg)
                            for v in views[ti]])
            probs = np.stack([cnn_oracle.forward(p, mel)[1] for p in paths])
            ref = cnn_oracle.ensemble_track_mean(probs)
            worst = max(worst, float(np.abs(means[row] - ref).max()))
            ref_rows.append(ref)
        oracle_means.append((idx, np.array(ref_rows, np.float32), meta))
    print(f"two groups: {len(seen['scores'][0][0])} tracks, max|d track mean| vs oracle = {worst:.3e}")
    assert worst <= 1e-3

    # the same post-processing on the oracle's scores
    (tracks, length, signals, raw_length, bird_labels), = seen["res"]
    for idx, ref, meta in oracle_means:
        apply(tracks, idx, ref, meta)
    ref_doc = analyse.species_result((tracks, length, signals, raw_length, bird_labels), None, False)
    drop = lambda d: {k: v for k, v in d.items() if k != "processing_time_seconds"}
    got, want = drop(doc), drop(ref_doc)
    masters = [t["master_tag"] if "master_tag" in t else None for t in want["species_identify"]]
    assert any(m is not None for m in masters)
    if not any(_near_boundary(m, meta.get("threshold", 0.7)) for _, m, meta in oracle_means):
        assert json.dumps(got, sort_keys=True) == json.dumps(want, sort_keys=True)
    else:  # a score on a boundary: same tracks, labels within one point
        assert len(got["species_identify"]) == len(want["species_identify"])
