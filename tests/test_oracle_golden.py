"""The CPU oracle pinned against golden vectors captured from the reference
itself (tests/golden/make_golden.py) and against analytic known answers for
the librosa pieces the reference does not ship (STFT, power_to_db)."""
import json
from pathlib import Path
import types

import numpy as np
import pytest

from oracle import cnn_oracle, fe_oracle, windows_oracle

G = Path(__file__).parent / "golden"


def test_custom_mel_bitexact_vs_reference():
    g = np.load(G / "mel_f.npz")
    for k in [k for k in g.files if not k.endswith("__cfg")]:
        sr, nm, fmin, fmax, nfft, brk = g[k + "__cfg"]
        w = fe_oracle.custom_mel_filterbank(int(sr), int(nm), fmin, fmax, int(nfft), brk)
        assert w.dtype == np.float32 and np.array_equal(w, g[k]), k


def test_normalize_bitexact_vs_reference():
    g = np.load(G / "normalize.npz")
    for i in range(3):
        out = fe_oracle.normalize_data(g[f"in{i}"])
        assert out.dtype == np.float32
        assert np.array_equal(out, g[f"out{i}"]), i


def _tracks(c):
    return [types.SimpleNamespace(start=s, end=e, length=e - s, freq_start=f0, freq_end=f1)
            for s, e, f0, f1 in c["tracks"]]


def test_windows_oracle_vs_reference():
    for c in json.load(open(G / "windows.json")):
        n = c["clip_samples"]
        frames = np.arange(1, n + 1, dtype=np.float32)
        np.random.seed(c["seed"])
        if "error" in c:
            with pytest.raises(AssertionError):  # the reference's :146 assert
                for t in _tracks(c):
                    windows_oracle.track_windows(frames, c["sr"], t, 3, 1.5, 50, 11000,
                                                 c["pad_short_tracks"])
            continue
        for t, want in zip(_tracks(c), c["windows"]):
            got = windows_oracle.track_windows(frames, c["sr"], t, 3, 1.5, 50, 11000,
                                               c["pad_short_tracks"])
            assert len(got) == len(want)
            for w, (src, nv, left) in zip(got, want):
                nz = np.flatnonzero(w)
                assert len(nz) == nv
                if nv:
                    assert nz[0] == left and w[nz[0]] == src + 1


# ---- analytic known answers for the librosa restatements ----
def test_stft_frame_count_and_pure_tone_bin():
    sr, n_fft, hop = 48000, 4096, 640
    k = 100
    t = np.arange(144000)
    x = np.cos(2 * np.pi * k * t / n_fft).astype(np.float32)
    mag = fe_oracle.stft_mag(x, n_fft, hop)
    assert mag.shape == (n_fft // 2 + 1, 1 + 144000 // hop)
    mid = mag[:, 100]
    assert np.argmax(mid) == k
    # periodic Hann: a bin-centred tone leaks only into k +- 1 (amplitude N/4)
    assert mid[k] == pytest.approx(n_fft / 4, rel=1e-5)
    assert mid[k + 1] == pytest.approx(n_fft / 8, rel=1e-4)
    assert mid[k + 3] < 1e-3


def test_hann_periodic_cola():
    w = fe_oracle.hann_periodic(4096)
    # overlap-add of hann^1 at hop N/4 is constant 2
    s = sum(np.roll(w, h) for h in range(0, 4096, 1024))
    assert np.allclose(s, 2.0)
    assert w[0] == 0.0 and w[2048] == 1.0


def test_power_to_db_known_answers():
    S = np.array([[1.0, 1e-3], [1e-12, 0.5]], dtype=np.float32)
    d = fe_oracle.power_to_db(S)
    assert d.dtype == np.float32
    assert d.max() == 0.0
    assert d[0, 1] == pytest.approx(-30.0, abs=1e-4)
    assert d[1, 0] == -80.0  # floor at max - top_db
    assert fe_oracle.power_to_db(np.zeros((3, 3), np.float32)).max() == 0.0


def test_stft_rejects_nonfinite():
    x = np.zeros(10000, np.float32)
    x[5] = np.nan
    with pytest.raises(ValueError):
        fe_oracle.stft_mag(x, 4096, 640)


def test_magtransform_known_answers(tmp_path):
    """x ** sigmoid(a): v1 init a=0 -> sqrt (src/magtransform.py:7-19),
    v2 init a=-1 -> x ** 0.2689 (src/magtransformv2.py:7-21)."""
    arch = [{"type": "magtransform", "name": "mag"}]
    x = np.array([[[[4.0]], [[0.25]]]], dtype=np.float32)
    for a, expo in [(0.0, 0.5), (-1.0, 1.0 / (1.0 + np.e))]:
        _, y = cnn_oracle.forward(arch, x, tensors={"mag.a": np.array([a], np.float32)})
        assert np.allclose(y.reshape(-1), np.array([4.0, 0.25]) ** expo, rtol=1e-6)
