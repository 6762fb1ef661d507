"""Band-pass filtered tracks (reference src/identify_tracks.py:152-162,
butter_bandpass_filter :1036-1056): the host builds each filtered track's
copy and remaps its windows onto it (aa_amd.windows.filtered_sources).

Pinned by tests/golden/filtered.json, made by running the reference's own
load_samples with filter_freqs / filter_below (tests/golden/make_golden.py):
every window's samples, rebuilt from the remapped views, match the
reference's (float64) windows to float32 rounding."""
import json
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest

from aa_amd.windows import filtered_sources, schedule

GOLD = json.loads((Path(__file__).parent / "golden" / "filtered.json").read_text())


def _clip(n, seed):
    rng = np.random.default_rng(seed)
    return (np.round(rng.standard_normal(n) * 0.1 * 32768) / 32768).astype(np.float32)


def _track(s, e, f0, f1):
    return SimpleNamespace(start=s, end=e, freq_start=f0, freq_end=f1, length=e - s)


@pytest.mark.parametrize("case", range(len(GOLD)))
def test_filtered_windows_match_reference(case):
    g = GOLD[case]
    sr = g["sr"]
    frames = _clip(g["clip_seconds"] * sr, g["clip_seed"])
    tracks = [_track(*t) for t in g["tracks"]]
    np.random.seed(g["seed"])
    views, spans = schedule(len(frames), sr, tracks, g["segment_length"], g["segment_stride"], g["fmin"],
                            g["fmax"], g["pad_short_tracks"], return_spans=True)
    extra, views = filtered_sources(frames, sr, tracks, views, spans, g["filter_freqs"], g["filter_below"],
                                    len(frames))
    buf = np.concatenate([frames, extra]).astype(np.float64)
    size = int(sr * g["segment_length"])
    assert [len(v) for v in views] == [len(w) for w in g["windows"]]
    n_filtered = 0
    for tv, (t, tw) in zip(views, zip(tracks, g["windows"])):
        for (src, n, p), ref in zip(tv, tw):
            w = np.zeros(size)
            w[p:p + n] = buf[src:src + n]
            n_filtered += src >= len(frames)
            assert ref["n"] == size
            np.testing.assert_allclose([w[i] for i in g["positions"]], ref["at"], rtol=1e-6, atol=1e-8)
            np.testing.assert_allclose(w.sum(), ref["sum"], rtol=1e-5, atol=1e-4)
            np.testing.assert_allclose((w * w).sum(), ref["sumsq"], rtol=1e-5)
    # filter_freqs filters every track; filter_below only the tracks ending below it
    expect = sum(len(tv) for tv, t in zip(views, tracks)
                 if g["filter_freqs"] or (g["filter_below"] and t.freq_end < g["filter_below"]))
    assert n_filtered == expect > 0


def test_use_mfcc_raises():
    """get_spect's MFCC branch (:269-280) is not built: a use_mfcc model must
    fail loudly instead of returning scores of a log-mel-only input."""
    import torch
    from aa_amd.pipeline import Classifier
    clf = Classifier("bf16x3", device="cpu")
    frames = _clip(4 * 48000, 1)
    meta = {"name": "m", "labels": ["a"], "use_mfcc": True}
    with pytest.raises(NotImplementedError, match="use_mfcc"):
        clf.classify_tracks(frames, 48000, [_track(0, 3, 0, 24000)], [[("m", meta)]],
                            pcm=torch.from_numpy(frames))
