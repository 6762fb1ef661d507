"""signal_noise on the GPU (aa_sn_run, csrc/aa_signal.hip) against the CPU
oracle (oracle/signal_oracle.py, src/identify_tracks.py:650-706).

* Morphology + components + filter: bit-exact on identical masks
  (aa_sn_components_from_mask vs the oracle's cv2 restatement).
* The mask: the GPU f32 FFT vs the oracle's f64 FFT (librosa 0.11) can flip
  pixels sitting on the 3x-median thresholds; the test bounds the disagreement
  (<= 1e-4 of the pixels) and requires the GPU components to equal the oracle's
  morphology of the GPU's own mask exactly, and the oracle's end result up to
  those flips (same count, boxes within 2 frames / 2 bins).
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


@pytest.mark.parametrize("seconds,seed", [(3.0, 10), (10.0, 11), (7.3, 12)])
def test_signal_noise_vs_oracle(gpu, seconds, seed):
    x = _clip(seconds, seed)
    det = _det(gpu)
    F = det.n_frames(len(x))
    mask_dev = torch.empty((2049, det.words(F)), dtype=torch.int64, device=gpu)
    stats = det.components(torch.from_numpy(x).to(gpu), mask_out=mask_dev)
    gmask = _unpack(mask_dev.cpu().numpy(), F)
    ref_sig, ref_mask, ref_stats = so.signal_noise(x, SR, HOP)
    diff = int((gmask != ref_mask).sum())
    assert diff <= max(2, 1e-4 * ref_mask.size), diff
    assert stats.tolist() == so.signal_mask_to_stats(gmask, SR, HOP).tolist()
    assert len(stats) == len(ref_stats) and len(stats) > 0
    assert np.abs(stats[:, :4] - ref_stats[:, :4]).max() <= 2
    got_sig = det.to_tuples(stats)
    if diff == 0:
        assert got_sig == ref_sig


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
