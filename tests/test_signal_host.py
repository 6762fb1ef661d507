"""signal_noise's host-side pieces and its CPU oracle (no GPU).

* The oracle's cv2 restatement (oracle/signal_oracle.py) pinned by known
  answers of OpenCV's documented semantics (anchor, no kernel reflection,
  ignored borders, empty kernel, 8-connectivity, label order).
* The track builder (merge_signals / get_tracks_from_signals,
  src/identify_tracks.py:725-842) against tests/golden/tracks.json, made by
  running the reference's own function (tests/golden/make_golden.py).
"""
import json
from pathlib import Path

import numpy as np

from aa_amd.identify_tracks import Signal, get_tracks_from_signals
from oracle import signal_oracle as so

G = Path(__file__).parent / "golden"


def test_morph_opencv_anchor_semantics():
    img = np.zeros((12, 12), np.uint8)
    img[5, 5] = 1
    d = so.morph(img, 4, 4, False)
    # out(y, x) = max img(y + j - 2, x + i - 2), j, i in 0..3: the pixel reaches 4..7
    assert np.argwhere(d).min(0).tolist() == [4, 4] and np.argwhere(d).max(0).tolist() == [7, 7]
    # erode uses the same (unreflected) offsets, so dilate -> erode moves by +1
    assert np.argwhere(so.morph(d, 4, 4, True)).tolist() == [[6, 6]]
    # taps outside the image never change the result
    assert so.morph(np.ones((5, 9), np.uint8), 4, 4, True).all()
    assert not so.morph(np.zeros((5, 9), np.uint8), 10, 42, False).any()
    # an empty kernel is a 3x3 rectangle
    assert np.array_equal(so.morph(img, 0, 5, False), so.morph(img, 3, 3, False))


def test_components_8_connectivity_and_label_order():
    img = np.zeros((6, 10), np.uint8)
    img[0, 5] = 1
    img[1, 6] = 1    # diagonal neighbour: same component
    img[4, 0:3] = 1  # left 0, but its first 2x2 block comes later in raster order
    stats = so.connected_components_stats(img)
    assert stats.tolist() == [[5, 0, 2, 2, 2], [0, 4, 3, 1, 3]]
    assert so.connected_components_stats(np.zeros((3, 3), np.uint8)).shape == (0, 5)


def test_signal_geometry_48k():
    width, height, freqs = so.signal_geometry(48000, 281)
    assert (width, height) == (42, 10) and len(freqs) == 2049


def test_mask_even_and_odd_medians():
    rng = np.random.default_rng(3)
    for F in (7, 8):
        S = rng.random((5, F)).astype(np.float32)
        m = so.signal_mask(S)
        a = S.max()
        Sd = S / a
        ref = (Sd > 3 * np.median(Sd, axis=0)[None]) & (Sd > 3 * np.median(Sd, axis=1)[:, None])
        assert np.array_equal(m.astype(bool), ref)
    assert not so.signal_mask(np.zeros((4, 6), np.float32)).any()  # a == 0: NaN quotients


def test_track_builder_matches_reference():
    cases = json.load(open(G / "tracks.json"))
    assert len(cases) == 40
    for c in cases:
        got = get_tracks_from_signals([Signal(*a) for a in c["signals"]], c["end"])
        got = [[float(t.start), float(t.end), float(t.freq_start), float(t.freq_end)] for t in got]
        assert got == c["tracks"]


# ---- the native track builder (csrc/aa_tracks.cpp, aa_tracks_from_signals) ----
def _fields(tracks):
    """Every field a track's JSON or a later step reads, with its Python type
    (a JSON 0 and 0.0 differ)."""
    return [tuple((type(v) is int, float(v)) for v in (t.start, t.end, t.freq_start, t.freq_end))
            + (float(t.mel_freq_start), float(t.mel_freq_end)) for t in tracks]


def test_native_track_builder_matches_reference():
    from aa_amd.identify_tracks import tracks_from_signals
    for c in json.load(open(G / "tracks.json")):
        sig = [Signal(*a) for a in c["signals"]]
        got = tracks_from_signals(sig, c["end"])
        assert [[float(t.start), float(t.end), float(t.freq_start), float(t.freq_end)] for t in got] == c["tracks"]
        # the inputs are left as they were
        assert [[s.start, s.end, s.freq_start, s.freq_end] for s in sig] == c["signals"]


def _random_signals(rng, n, end, sr=48000):
    freqs = np.arange(2049) * sr / 4096
    sigs = []
    for _ in range(n):
        left = int(rng.integers(0, int(end * sr / 281)))
        if rng.random() < 0.2:
            left = int(rng.integers(0, 60))  # near 0: enlarge's max(start - pad, 0) gives the int 0
        width, top, height = int(rng.integers(1, 700)), int(rng.integers(0, 1500)), int(rng.integers(1, 500))
        if rng.random() < 0.35 and sigs:  # near-duplicates exercise every merge rule
            b = sigs[int(rng.integers(0, len(sigs)))]
            left = max(0, b[0] + int(rng.integers(-60, 60)))
            top = max(0, b[1] + int(rng.integers(-30, 30)))
        sigs.append((left, top, width, height))
    out = []
    for left, top, width, height in sigs:
        f0, f1 = freqs[top], freqs[min(2048, top + height)]
        if rng.random() < 0.1:  # integer frequencies (a sidecar's, or an earlier enlarge's)
            f0, f1 = int(f0), int(f1)
        out.append(Signal(left * 281 / sr, (left + width) * 281 / sr, f0, f1))
    return out


def test_native_track_builder_equals_python_builder():
    """Field for field and type for type against the Python restatement
    (itself pinned to the reference above) on 3,000 seeded signal sets:
    1-40 signals, near-duplicates, starts near 0, integer frequencies, float
    and int ends (get_end's truncated length is an int), other sample rates."""
    from aa_amd.identify_tracks import tracks_from_signals
    rng = np.random.default_rng(2024)
    n_tracks = n_int0 = 0
    for case in range(3000):
        sr = [48000, 44100, 16000, 96000][case % 4]
        end = [60.0, 59.7, 30.0, 60, 17][int(rng.integers(0, 5))]
        sig = _random_signals(rng, int(rng.integers(1, 41)), float(end), sr)
        want = get_tracks_from_signals([s.copy() for s in sig], end)
        got = tracks_from_signals(sig, end)
        assert _fields(got) == _fields(want), case
        n_tracks += len(got)
        n_int0 += sum(type(t.start) is int for t in got)
    assert n_tracks > 3000 and n_int0 > 100  # the int-0 starts did occur


def test_native_track_builder_edges():
    from aa_amd.identify_tracks import tracks_from_signals
    assert tracks_from_signals([], 60.0) == []
    # enlarged past the 2^17-entry mel table: the Python builder takes it, same result
    sig = [Signal(1.0, 2.0, 100000.0, 130000.0), Signal(1.2, 2.5, 101000.0, 131000.0)]
    assert _fields(tracks_from_signals(sig, 60.0)) == _fields(get_tracks_from_signals([s.copy() for s in sig], 60.0))
    # NaN anywhere: the Python builder's result (the native sorts need a strict weak order)
    sig = [Signal(1.0, 2.0, 500.0, 4000.0), Signal(float("nan"), 3.0, 600.0, 4500.0), Signal(1.5, 2.5, 550.0, 4200.0)]
    got, want = tracks_from_signals(sig, 60.0), get_tracks_from_signals([s.copy() for s in sig], 60.0)
    assert repr(_fields(got)) == repr(_fields(want)) and "nan" in repr(_fields(got))  # (nan != nan)
    # one signal shorter than min_length: no tracks; one clipped to an int end
    assert tracks_from_signals([Signal(1.0, 1.2, 500.0, 4000.0)], 60.0) == []
    got = tracks_from_signals([Signal(9.5, 10.0, 500.0, 4000.0)], 10)
    assert type(got[0].end) is int and got[0].end == 10


def test_mel_int_table_equals_scalar_mel():
    from aa_amd.identify_tracks import _mel_int_table
    t = _mel_int_table()
    assert t is not False
    f = np.arange(t.size)
    assert all(t[i] == 2595.0 * np.log10(1.0 + int(i) / 700.0) for i in f[::7])
