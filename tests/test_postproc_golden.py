"""Result post-processing pinned against the reference itself.

tests/golden/make_golden.py runs the reference's species_identify
(src/analyse.py:129-175) through its real classify() tail
(src/identify_tracks.py:416-573) with decode, STFT and model.predict stubbed to
fixed per-window probabilities (stored in postproc_probs.npz).  Here the same
probabilities go through this build's host path -- window schedule, numpy's
model/window means (the GPU aa_track_mean is bit-identical to those, see
tests/test_gpu_cnn.py), apply_group_scores, region filtering, master tags --
and the JSON must match the reference's byte for byte.
"""
import json
from pathlib import Path

import numpy as np
import pytest

from aa_amd import analyse, pipeline
from aa_amd.identify_tracks import MAX_FRQUENCY, Signal, get_tracks_from_signals
from aa_amd.windows import schedule

G = Path(__file__).parent / "golden"
GOLD = json.load(open(G / "postproc.json"))
PROBS = np.load(G / "postproc_probs.npz")


def _classify_from_golden(name, case, metas):
    def fake(file_name, bird_models, analyse_tracks, meta_data=None):
        signals = [Signal(*x) for x in (case.get("signals") or [])]
        if analyse_tracks:
            tracks = []
            for t in meta_data["Tracks"]:
                s = Signal(t["start"], t["end"], t.get("minFreq", 0), t.get("maxFreq", MAX_FRQUENCY))
                s.track_id = t["id"]
                tracks.append(s)
        else:  # built from the signals exactly as classify() does (:434-437)
            tracks = get_tracks_from_signals([s.copy() for s in signals], 60.0)
        groups = [[metas[m] for m in case["models"] if not metas[m]["pre_model"]],
                  [metas[m] for m in case["models"] if metas[m]["pre_model"]]]
        np.random.seed(case["seed"])
        m0 = groups[0][0]
        views = schedule(60 * 48000, 48000, tracks, m0["segment_length"], m0["segment_stride"],
                         m0["fmin"], m0["fmax"], False)
        call = 0
        for g in groups:
            sel, rows = [], []
            for ti, tv in enumerate(views):
                if not tv:
                    continue
                per_model = []
                for _ in g:
                    per_model.append(PROBS[f"{name}__call{call}"])
                    call += 1
                sel.append(ti)
                rows.append(np.mean(np.mean(per_model, axis=0), axis=0))
            pipeline.apply_group_scores(tracks, sel, np.asarray(rows, np.float32), g[0])
        assert call == case["n_calls"]
        return tracks, 60.0, signals, 60.0, ["bird", "kiwi", "whistler", "morepork"]
    return fake


@pytest.mark.parametrize("name", sorted(GOLD["cases"]))
def test_species_identify_json_matches_reference(name, tmp_path, monkeypatch):
    case = GOLD["cases"][name]
    metas = GOLD["metas"]
    rec = tmp_path / "rec.wav"
    rec.write_bytes(b"")
    (tmp_path / "rec.txt").write_text(json.dumps(case["meta"]))
    monkeypatch.setenv("AA_EBIRD_SPECIES", str(G / "ebird_subset.json") if case["species_file"]
                       else str(tmp_path / "absent.json"))
    monkeypatch.setattr(analyse, "classify", _classify_from_golden(name, case, metas))
    got = analyse.species_identify(str(rec), ["m1", "m2", "m3"], case.get("signals") is None)
    assert json.dumps(got, sort_keys=True) == json.dumps(case["result"], sort_keys=True)


def test_cacophony_index_edge_cases():
    class T:
        def __init__(self, s, e):
            self.start, self.end = s, e
    p, v = analyse.calc_cacophony_index([T(1, 5), T(4, 25), T(59, 61)], 61.0)
    assert v == "1.0" and len(p) == 3 and p[-1]["end_s"] == 61.0
    assert p[0]["index_percent"] == 95.0
    p, _ = analyse.calc_cacophony_index([], 60.0)
    assert [x["index_percent"] for x in p] == [0, 0, 0]


def test_cli_parses_reference_flags():
    a = analyse.parse_args(["rec.wav", "--bird-model", "none", "-o", "--analyse-tracks", "true"])
    assert a.bird_model == [None] and a.meta_to_stdout == 1 and a.analyse_tracks is True
    b = analyse.parse_args(["rec.wav"])
    assert b.bird_model == ["/models/pre-model/audioModel.keras", "/models/bird-model-v2m/audioModel.keras"]
