"""CPU oracle for the per-window log-mel front-end.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``audio-analysis_amd/aa_amd``) never imports it.

What it restates (reference = /root/reference, pinned librosa ~=0.11.0,
``requirements.txt:1``):

* ``normalize_data``            src/identify_tracks.py:202-209
* ``librosa.stft`` call          src/identify_tracks.py:243 (center=True,
  pad_mode="constant", periodic Hann, rfft in float64, stored as complex64)
* ``custommel.mel_f``/``mel_spec`` src/custommel.py:6-63  (HTK-style mel with a
  movable break frequency, Slaney area normalisation)
* ``librosa.filters.mel`` (htk=False, norm="slaney") for the non-htk branch
  src/identify_tracks.py:229-238
* ``librosa.power_to_db(S, ref=np.max)`` src/identify_tracks.py:266
* the ``get_spect`` tail (expand_dims, mean_sub, channels) :267-288

Parity status: ``mel_f`` and ``normalize_data`` are pinned bit-exactly against
golden vectors produced by importing the reference itself
(``tests/golden/make_golden.py``).  librosa is not installed in this image and
its source is not under /root/reference, so the STFT / power_to_db / Slaney
filterbank restatements are pinned only by analytic known-answer tests
(pure tones, COLA sums, frame counts, dB max/floor) -- "parity unpinned" for
those three against librosa itself.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


# --------------------------------------------------------------------------
# A3  normalize_data  (src/identify_tracks.py:202-209)
# --------------------------------------------------------------------------
def normalize_data(x: np.ndarray) -> np.ndarray:
    """Same float32 operation order as the reference: shift by the min, divide
    by the (shifted) max, add 1e-6 *after* the division, recentre, scale."""
    lo = np.min(x, -1, keepdims=True)
    shifted = x - lo
    hi = np.max(shifted, -1, keepdims=True)
    y = shifted / hi + 0.000001
    y = y - 0.5
    return y * 2


# --------------------------------------------------------------------------
# A4  librosa 0.11 stft, as called at src/identify_tracks.py:243
# --------------------------------------------------------------------------
def hann_periodic(n: int) -> np.ndarray:
    """scipy.signal.get_window('hann', n, fftbins=True) in float64 -- the call
    librosa 0.11's stft makes (filters.get_window); scipy is the reference's own
    pinned dependency (requirements.txt) and is present here."""
    from scipy.signal import get_window
    return get_window("hann", n, fftbins=True)


def n_frames(n_samples: int, hop: int) -> int:
    """center=True frame count: 1 + len // hop."""
    return 1 + n_samples // hop


def stft_mag(y: np.ndarray, n_fft: int, hop: int) -> np.ndarray:
    """|librosa.stft(y, n_fft, hop)| -> float32 [1 + n_fft//2, T].

    center=True with zero ("constant") padding of n_fft//2 on both sides,
    frames multiplied by the float64 periodic Hann window, rfft in float64,
    result stored as complex64 (dtype_r2c(float32)), magnitude in float32.
    """
    y = np.asarray(y)
    if not np.all(np.isfinite(y)):
        # librosa.util.valid_audio raises ParameterError on non-finite input
        raise ValueError("Audio buffer is not finite everywhere")
    half = n_fft // 2
    padded = np.zeros(len(y) + 2 * half, dtype=y.dtype)
    padded[half:half + len(y)] = y
    T = n_frames(len(y), hop)
    win = hann_periodic(n_fft)
    out = np.empty((1 + half, T), dtype=np.complex64)
    step = 64  # bound peak memory of the framed copy
    for t0 in range(0, T, step):
        t1 = min(T, t0 + step)
        idx = (np.arange(t0, t1) * hop)[:, None] + np.arange(n_fft)[None, :]
        frames = padded[idx].astype(np.float64) * win[None, :]
        out[:, t0:t1] = np.fft.rfft(frames, axis=-1).T.astype(np.complex64)
    return np.abs(out)


# --------------------------------------------------------------------------
# A5  custommel filterbank  (src/custommel.py:6-56)
# --------------------------------------------------------------------------
def _to_mel(f, brk):
    return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / brk)


def _from_mel(m, brk):
    return brk * (10.0 ** (np.asarray(m, dtype=np.float64) / 2595.0) - 1.0)


def custom_mel_filterbank(sr, n_mels, fmin, fmax, n_fft, break_freq) -> np.ndarray:
    """Triangles on a mel scale whose 700 Hz break is replaced by ``break_freq``.

    Rounding follows the reference: each triangle row is evaluated in float64
    and stored into a float32 matrix, then the float32 matrix is multiplied
    in place by the float64 Slaney factor 2/(f[i+2]-f[i]) (float64 multiply,
    float32 store).
    """
    n_bins = 1 + n_fft // 2
    bin_hz = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)  # librosa.fft_frequencies
    edges = _from_mel(np.linspace(_to_mel(fmin, break_freq), _to_mel(fmax, break_freq),
                                  int(n_mels) + 2), break_freq)
    width = np.diff(edges)
    dist = edges[:, None] - bin_hz[None, :]
    fb = np.zeros((int(n_mels), n_bins), dtype=F32)
    for m in range(int(n_mels)):
        rise = -dist[m] / width[m]
        fall = dist[m + 2] / width[m + 1]
        fb[m] = np.maximum(0.0, np.minimum(rise, fall))
    scale = 2.0 / (edges[2:int(n_mels) + 2] - edges[:int(n_mels)])
    fb *= scale[:, None]
    return fb


def mel_spec(mag: np.ndarray, fb: np.ndarray, power) -> np.ndarray:
    """custommel.mel_spec: fb . |S|**power (src/custommel.py:59-63)."""
    return fb.dot(np.abs(mag) ** power)


# --------------------------------------------------------------------------
# A7' librosa 0.11 filters.mel(htk=False, norm="slaney")  [ext, unpinned]
# --------------------------------------------------------------------------
def _slaney_hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz,
                    min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep,
                    mels)


def _slaney_mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def slaney_mel_filterbank(sr, n_fft, n_mels, fmin, fmax) -> np.ndarray:
    n_bins = 1 + n_fft // 2
    bin_hz = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    edges = _slaney_mel_to_hz(np.linspace(_slaney_hz_to_mel(fmin), _slaney_hz_to_mel(fmax),
                                          n_mels + 2))
    width = np.diff(edges)
    dist = edges[:, None] - bin_hz[None, :]
    fb = np.zeros((n_mels, n_bins), dtype=F32)
    for m in range(n_mels):
        rise = -dist[m] / width[m]
        fall = dist[m + 2] / width[m + 1]
        fb[m] = np.maximum(0.0, np.minimum(rise, fall))
    fb *= (2.0 / (edges[2:n_mels + 2] - edges[:n_mels]))[:, None]
    return fb


# --------------------------------------------------------------------------
# A7  librosa.power_to_db(S, ref=np.max, amin=1e-10, top_db=80)
# --------------------------------------------------------------------------
def power_to_db(S: np.ndarray, amin=1e-10, top_db=80.0) -> np.ndarray:
    S = np.asarray(S)
    ref = np.max(S)
    out = 10.0 * np.log10(np.maximum(amin, S))
    out -= 10.0 * np.log10(np.maximum(amin, ref))
    return np.maximum(out, out.max() - top_db)


# --------------------------------------------------------------------------
# get_spect  (src/identify_tracks.py:212-288), htk and non-htk branches
# --------------------------------------------------------------------------
def get_spect(data, sr, hop_length, n_mels, fmin, fmax, n_fft, power, db_scale,
              htk=True, break_freq=1750, mean_sub=False, channels=1) -> np.ndarray:
    mag = stft_mag(data, n_fft, hop_length)
    if htk:
        fb = custom_mel_filterbank(sr, n_mels, 50 if fmin is None else fmin,
                                   11000 if fmin is None else fmax, n_fft, break_freq)
        mel = mel_spec(mag, fb, power)
    else:
        # librosa.feature.melspectrogram: fixed fmin=50/fmax=11000, power 2.0
        fb = slaney_mel_filterbank(sr, n_fft, n_mels, 50, 11000)
        mel = fb.dot(mag ** 2.0).astype(F32)
    if db_scale:
        mel = power_to_db(mel)
    mel = mel[:, :, None]
    if mean_sub:
        mel = mel - np.mean(mel, axis=1, keepdims=True)
    if channels > 1:
        mel = np.repeat(mel, channels, axis=2)
    return mel.astype(F32)


def window_logmel(window: np.ndarray, cfg: dict) -> np.ndarray:
    """normalize (optional) + get_spect for one 1-D window -> [n_mels, T, C]."""
    x = np.asarray(window, dtype=F32)
    if cfg.get("normalize", True):
        x = normalize_data(x)
    return get_spect(x, cfg["sr"], cfg["hop_length"], cfg["n_mels"], cfg["fmin"], cfg["fmax"],
                     cfg["n_fft"], cfg["power"], cfg["db_scale"], htk=cfg["htk"],
                     break_freq=cfg["break_freq"], mean_sub=cfg.get("mean_sub", False),
                     channels=cfg.get("channels", 1))
