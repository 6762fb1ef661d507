"""Mel filterbanks, built once per front-end plan on the host.

* ``htk_break``: the custom HTK-style filterbank of src/custommel.py:6-56
  (mel = 2595 log10(1 + f / break_freq), Slaney area normalisation).  The
  reference rebuilds it on every window (src/custommel.py:62); here it is a
  per-plan constant.  Rounding matches the reference exactly: triangles in
  float64 stored to float32, then a float64 normalisation multiply stored to
  float32 (pinned bit-exactly by tests/golden/mel_f.npz).
* ``slaney``: librosa.filters.mel(htk=False, norm="slaney") used by the
  reference's non-htk branch (src/identify_tracks.py:229-238).
"""
from __future__ import annotations

import numpy as np


def _triangles(edges_hz: np.ndarray, sr: int, n_fft: int) -> np.ndarray:
    bins_hz = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    gaps = np.diff(edges_hz)
    d = edges_hz[:, None] - bins_hz[None, :]           # [n_mels + 2, n_bins]
    rising = -d[:-2] / gaps[:-1, None]
    falling = d[2:] / gaps[1:, None]
    tri = np.maximum(0.0, np.minimum(rising, falling)).astype(np.float32)
    norm = 2.0 / (edges_hz[2:] - edges_hz[:-2])
    return (tri.astype(np.float64) * norm[:, None]).astype(np.float32)


def htk_break(sr: int, n_mels: int, fmin: float, fmax: float, n_fft: int,
              break_freq: float) -> np.ndarray:
    def to_mel(f):
        return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / break_freq)

    mels = np.linspace(to_mel(fmin), to_mel(fmax), int(n_mels) + 2)
    edges = break_freq * (10.0 ** (mels / 2595.0) - 1.0)
    return _triangles(edges, sr, n_fft)


_F_SP = 200.0 / 3
_LOG_HZ = 1000.0
_LOG_MEL = _LOG_HZ / _F_SP
_LOG_STEP = np.log(6.4) / 27.0


def _slaney_mel(f):
    f = np.asarray(f, dtype=np.float64)
    lin = f / _F_SP
    return np.where(f >= _LOG_HZ, _LOG_MEL + np.log(np.maximum(f, _LOG_HZ) / _LOG_HZ) / _LOG_STEP, lin)


def _slaney_hz(m):
    m = np.asarray(m, dtype=np.float64)
    return np.where(m >= _LOG_MEL, _LOG_HZ * np.exp(_LOG_STEP * (m - _LOG_MEL)), _F_SP * m)


def slaney(sr: int, n_fft: int, n_mels: int, fmin: float, fmax: float) -> np.ndarray:
    edges = _slaney_hz(np.linspace(_slaney_mel(fmin), _slaney_mel(fmax), int(n_mels) + 2))
    return _triangles(edges, sr, n_fft)
