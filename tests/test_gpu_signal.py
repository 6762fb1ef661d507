"""signal_noise on the GPU (aa_sn_run, csrc/aa_signal.hip) against the CPU
oracle (oracle/signal_oracle.py, src/identify_tracks.py:650-706).

* |STFT| (aa_sn_spectrogram): the f64 transform rounded to complex64 and
  numpy's f32 magnitude give the oracle's S (numpy's own rfft + np.abs) bit for
  bit, on full 60 s recordings, ragged lengths and recordings shorter than one
  hop -- up to the rare value whose f64 transform lies within ~1e-16 of a
  complex64 rounding midpoint (two f64 FFTs, pocketfft's and this one, agree
  to that distance only): at most 4 values per recording may differ, by one
  float32 ulp (measured: 1 of 21,002,250 on a 60 s clip).
* The mask, the components and the Signal tuples: identical to the oracle's
  on full 60 s recordings (zero pixels differ), and so are the tracks built from
  those signals and their window start indices (the CLI default path,
  analyse_tracks=False, :435-437).
* Morphology + components + filter: bit-exact on identical masks
  (aa_sn_components_from_mask vs the oracle's cv2 restatement).
* Edge cases: silent input (max 0: no signals), non-finite input raises,
  recordings shorter than one frame hop, frame counts not a multiple of 64.
"""
import numpy as np
import pytest
import torch

from oracle import signal_oracle as so

pytestmark = pytest.mark.gpu
SR, HOP = 48000, 281


def _det(gpu):
    from aa_amd.signals import SignalDetector
    return SignalDetector(SR, HOP, gpu)


def _clip(seconds, seed, n_chirps=6):
    rng = np.random.default_rng(seed)
    n = int(seconds * SR)
    x = (rng.standard_normal(n) * 0.02).astype(np.float64)
    t = np.arange(n) / SR
    for _ in range(n_chirps):
        t0 = rng.uniform(0, max(seconds - 1.2, 0.1))
        dur = rng.uniform(0.3, 1.0)
        f0, f1 = rng.uniform(600, 6000), rng.uniform(600, 6000)
        m = (t >= t0) & (t < t0 + dur)
        tt = t[m] - t0
        x[m] += 0.3 * np.sin(2 * np.pi * (f0 * tt + (f1 - f0) * tt * tt / (2 * dur)))
    return np.round(np.clip(x, -1, 1) * 32767).astype(np.float32) / 32768


def _unpack(mask_words, n_frames):
    bits = np.unpackbits(mask_words.view(np.uint8).reshape(mask_words.shape[0], -1), axis=1,
                         bitorder="little")
    return bits[:, :n_frames]


def _pack(mask):
    H, F = mask.shape
    W = (F + 63) // 64
    pad = np.zeros((H, W * 64), np.uint8)
    pad[:, :F] = mask
    return np.packbits(pad, axis=1, bitorder="little").view(np.int64).reshape(H, W)


@pytest.mark.parametrize("F,seed", [(1, 0), (63, 1), (64, 2), (200, 3), (1000, 4), (1779, 5)])
def test_components_from_mask_bit_exact(gpu, F, seed):
    rng = np.random.default_rng(seed)
    m = (rng.random((2049, F)) < 0.002).astype(np.uint8)
    # blobs big enough to survive the opening and the size filter
    for _ in range(8):
        y, x = int(rng.integers(0, 2000)), int(rng.integers(0, F))
        m[y:y + int(rng.integers(3, 60)), x:x + int(rng.integers(3, 80))] = 1
    det = _det(gpu)
    got = det.components_from_mask(torch.from_numpy(_pack(m)).to(gpu), F)
    ref = so.signal_mask_to_stats(m, SR, HOP)
    assert got.tolist() == ref.tolist()


@pytest.mark.parametrize("n,seed", [(60 * SR, 30), (60 * SR, 31), (7 * SR + 12345, 32), (3000, 33), (0, 34)])
def test_spectrogram_bit_exact(gpu, n, seed):
    x = _clip(n / SR, seed) if n else np.zeros(0, np.float32)
    det = _det(gpu)
    got = det.spectrogram(torch.from_numpy(x).to(gpu)).cpu().numpy()
    from oracle.fe_oracle import stft_mag
    want = stft_mag(x, 4096, HOP)
    assert got.shape == want.shape
    _assert_s_equal(got, want)


@pytest.mark.parametrize("variant", ["base", "table"])
@pytest.mark.parametrize("n,seed", [(60 * SR, 35), (7 * SR + 999, 36), (5000, 37)])
def test_spectrogram_variants_bit_exact(gpu, monkeypatch, variant, n, seed):
    """sn_stft64 with its default W, W^2, W^4 twiddle ladders and with every
    twiddle from the tables (AA_SN_TW=table) gives the reference's
    magnitudes, and the detector built on either gives its mask."""
    if variant == "table":
        monkeypatch.setenv("AA_SN_TW", "table")
    x = _clip(n / SR, seed)
    det = _det(gpu)
    got = det.spectrogram(torch.from_numpy(x).to(gpu)).cpu().numpy()
    from oracle.fe_oracle import stft_mag
    _assert_s_equal(got, stft_mag(x, 4096, HOP))
    if n == 60 * SR:
        F = det.n_frames(len(x))
        mask_dev = torch.empty((2049, det.words(F)), dtype=torch.int64, device=gpu)
        stats = det.components(torch.from_numpy(x).to(gpu), mask_out=mask_dev)
        _, ref_mask, ref_stats = so.signal_noise(x, SR, HOP)
        assert int((_unpack(mask_dev.cpu().numpy(), F) != ref_mask).sum()) == 0
        assert stats.tolist() == ref_stats.tolist()


def test_twiddle_chain_vs_table_over_many_clips(gpu, monkeypatch):
    """the default chained twiddle powers (f64 products) against
    the table values, over 24 seeded clips of 2-20 s (about 45,000 frames x
    2,049 bins = 92 M magnitudes).  A product a few f64 ulps off a table value
    moves an f32 magnitude only where the f64 magnitude sits on an f32
    rounding tie: measured, 1 magnitude in 92 M differs (round 6,
    profiles/r06/pytest_gpu.log).  The tolerance, as for any two f64 FFT
    factorisations against numpy's pocketfft (_assert_s_equal): at most one
    differing magnitude per recording, one f32 ulp apart, and wherever the two
    differ the oracle's (numpy) value is one of them."""
    from oracle.fe_oracle import stft_mag
    rng = np.random.default_rng(77)
    clips = [_clip(float(rng.uniform(2.0, 20.0)), 100 + i) for i in range(24)]
    det_chain = _det(gpu)
    chain = [det_chain.spectrogram(torch.from_numpy(x).to(gpu)).cpu().numpy() for x in clips]
    monkeypatch.setenv("AA_SN_TW", "table")
    det_table = _det(gpu)
    total = 0
    for x, c in zip(clips, chain):
        t = det_table.spectrogram(torch.from_numpy(x).to(gpu)).cpu().numpy()
        bad = c.view(np.uint32) != t.view(np.uint32)
        n_bad = int(bad.sum())
        total += n_bad
        assert n_bad <= 1, n_bad
        if n_bad:
            ulp = np.abs(c.view(np.int32)[bad].astype(np.int64) - t.view(np.int32)[bad].astype(np.int64))
            assert int(ulp.max()) == 1
            ref = stft_mag(x, 4096, HOP)
            assert bool(np.all((ref[bad] == c[bad]) | (ref[bad] == t[bad])))
    print(f"chained vs table twiddles: {total} of {sum(c.size for c in chain)} magnitudes differ")
    assert total <= 4




def _assert_s_equal(got, want):
    d = got.view(np.uint32) != want.view(np.uint32)
    ulps = np.abs(got.view(np.int32)[d].astype(np.int64) - want.view(np.int32)[d].astype(np.int64))
    print(f"S: {int(d.sum())} of {want.size} magnitudes differ (ulps {sorted(set(ulps.tolist()))})")
    assert int(d.sum()) <= 4 and (ulps <= 1).all()


def test_spectrogram_tone(gpu):
    """A pure 1 kHz tone: most bins sit orders of magnitude below the peak.
    Bins above 1e-6 of their frame's maximum are the reference's values (up to
    rounding ties); below ~1e-9 of it a bin is f64 rounding noise in pocketfft
    itself (an exactly periodic int16 tone leaves bins at ~1e-16 of the peak),
    so there the two transforms agree to that noise level, not bit for bit."""
    t = np.arange(20 * SR) / SR
    x = (np.round(0.5 * np.sin(2 * np.pi * 1000.0 * t) * 32768) / 32768).astype(np.float32)
    got = _det(gpu).spectrogram(torch.from_numpy(x).to(gpu)).cpu().numpy()
    from oracle.fe_oracle import stft_mag
    want = stft_mag(x, 4096, HOP)
    top = want.max(axis=0, keepdims=True)
    big = want >= 1e-6 * top
    assert big.sum() > 20 * want.shape[1]
    _assert_s_equal(got[big], want[big])
    assert (np.abs(got - want) <= 1e-12 * top).all()


@pytest.mark.parametrize("seconds,seed", [(60.0, 10), (60.0, 11), (60.0, 12), (7.3, 13), (10.0, 14)])
def test_signal_noise_vs_oracle(gpu, seconds, seed):
    x = _clip(seconds, seed)
    x = x[:len(x) - seed]  # ragged lengths: frame counts off the 64-frame words
    det = _det(gpu)
    F = det.n_frames(len(x))
    mask_dev = torch.empty((2049, det.words(F)), dtype=torch.int64, device=gpu)
    stats = det.components(torch.from_numpy(x).to(gpu), mask_out=mask_dev)
    gmask = _unpack(mask_dev.cpu().numpy(), F)
    ref_sig, ref_mask, ref_stats = so.signal_noise(x, SR, HOP)
    assert int((gmask != ref_mask).sum()) == 0
    assert stats.tolist() == ref_stats.tolist() and len(stats) > 0
    assert det.to_tuples(stats) == ref_sig


def test_tracks_from_signals_window_indices(gpu):
    """The CLI default path (analyse_tracks=False, :435-437): the tracks built
    from the GPU's signals and their windows' start indices equal those built
    from the oracle's signals (same seeded np.random draws)."""
    from aa_amd.identify_tracks import Signal, get_tracks_from_signals
    from aa_amd import windows
    x = _clip(60.0, 15, n_chirps=10)
    det = _det(gpu)
    got_sig = det.signal_noise(pcm=torch.from_numpy(x).to(gpu))
    ref_sig, _, _ = so.signal_noise(x, SR, HOP)
    assert got_sig == ref_sig and len(got_sig) > 0

    def views(sig):
        tracks = get_tracks_from_signals([Signal(*s) for s in sig], 60.0)
        np.random.seed(1234)
        return [(t.start, t.end, t.freq_start, t.freq_end) for t in tracks], windows.schedule(
            len(x), SR, tracks, 3.0, 1.5, 50.0, 11000.0)

    got_tracks, got_views = views(got_sig)
    ref_tracks, ref_views = views(ref_sig)
    assert len(got_tracks) > 0 and sum(len(v) for v in got_views) > 0
    assert got_tracks == ref_tracks and got_views == ref_views


def test_signal_noise_edge_cases(gpu):
    det = _det(gpu)
    assert det.components(torch.zeros(5 * SR, device=gpu)).shape == (0, 5)
    assert det.components(torch.zeros(0, device=gpu)).shape == (0, 5)
    assert det.components(torch.ones(100, device=gpu) * 0.1).shape == (0, 5)
    x = torch.from_numpy(_clip(2.0, 3)).to(gpu)
    x[12345] = float("nan")
    with pytest.raises(ValueError):
        det.components(x)


def test_classify_builds_tracks_from_signals(gpu, model_root, tmp_path):
    """analyse_tracks=False (the CLI default): tracks come from the detected
    signals, every returned track carries model results."""
    import wave
    from aa_amd.identify_tracks import classify
    wav = tmp_path / "rec.wav"
    with wave.open(str(wav), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(SR)
        w.writeframes((_clip(12.0, 21, n_chirps=4) * 32768).astype("<i2").tobytes())
    models = [str(model_root / m / "audioModel.safetensors") for m in ("model1", "model2")]
    tracks, length, signals, raw_length, labels = classify(str(wav), models, False)
    assert raw_length == pytest.approx(12.0) and len(signals) > 0 and len(tracks) > 0
    for t in tracks:
        assert len(t.results) >= 1


def test_sn_run_batch_matches_single(gpu):
    """aa_sn_run_batch (the corpus path: per-recording STFT / medians / mask,
    one batched morphology + components pass) gives every recording exactly
    the components aa_sn_run gives it alone: lengths that differ (different
    frame counts and mask widths in one batch), an empty recording, unaligned
    offsets into one PCM buffer."""
    import ctypes as C
    from aa_amd import _lib
    det = _det(gpu)
    lens = [SR * 7 + 123, 0, SR * 3, HOP * 64 - 1, SR * 11 + 5, 4000]
    clips = [_clip(n / SR, 40 + i) if n else np.zeros(0, np.float32) for i, n in enumerate(lens)]
    offs, pos = [], 3  # unaligned start
    for c in clips:
        offs.append(pos)
        pos += len(c) + 17
    buf = np.zeros(pos, np.float32)
    for o, c in zip(offs, clips):
        buf[o:o + len(c)] = c
    pcm = torch.from_numpy(buf).to(gpu)
    K, cap = len(lens), 512
    L = _lib.lib()
    need = L.aa_sn_batch_workspace_bytes(det._h, max(lens), K)
    ws = torch.empty(need, dtype=torch.uint8, device=gpu)
    out = torch.zeros((K, cap + 1, 6), dtype=torch.int32, device=gpu)
    rc = L.aa_sn_run_batch(det._h, _lib.dptr(pcm), (C.c_int64 * K)(*offs), (C.c_int64 * K)(*lens), K, _lib.dptr(ws),
                           ws.numel(), _lib.dptr(out[0, 1:]), cap, cap + 1, _lib.dptr(out[0, 0]), (cap + 1) * 6, 0)
    _lib.check(rc, "aa_sn_run_batch")
    got = out.cpu().numpy()
    n_nonempty = 0
    for k in range(K):
        want = det.components(pcm[offs[k]:offs[k] + lens[k]])
        cnt, status = int(got[k, 0, 0]), int(got[k, 0, 1])
        assert status == 0 and cnt == len(want), (k, cnt, status, len(want))
        rows = got[k, 1:1 + cnt].astype(np.int64)
        rows = rows[np.lexsort((rows[:, 5], rows[:, 0]))][:, :5]
        assert np.array_equal(rows, want), k
        n_nonempty += cnt > 0
    assert n_nonempty >= 3
