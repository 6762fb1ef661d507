"""CPU restatement of the reference's recording-end detector.  TEST INFRASTRUCTURE ONLY.

Follows ``get_end`` (src/identify_tracks.py:387-413) literally:

* ``np.abs(librosa.stft(frames, n_fft=sr // 10, hop_length=281))`` -- restated
  by ``fe_oracle.stft_mag`` (librosa 0.11: centred, zero padded, periodic
  Hann in float64, rfft stored as complex64);
* ``mel_spec(spectogram, sr, sr // 10, 281, 120, 50, 11000, 1750, power=1)``
  (src/custommel.py:59-63): ``mel_f(...) . |S| ** 1`` in float32, with the
  filterbank restated by ``fe_oracle.custom_mel_filterbank`` (pinned bit-exact
  to the reference's ``mel_f`` by tests/golden/mel_f.npz);
* the scan: 170-frame chunks (``sr // hop``), the first chunk whose mel block
  has ``amax == amin`` ends the recording at ``start * hop // sr`` seconds,
  only chunks that end before the last frame are examined (``while end <
  mel.shape[1]``), otherwise ``len(frames) / sr``.

librosa is absent here, so the STFT leg is the same restatement as the front
end's oracle (parity unpinned against librosa itself).
"""
from __future__ import annotations

import numpy as np

from . import fe_oracle


def mel_power1(frames: np.ndarray, sr: int) -> np.ndarray:
    n_fft = sr // 10
    mag = fe_oracle.stft_mag(np.asarray(frames, np.float32), n_fft, 281)
    fb = fe_oracle.custom_mel_filterbank(sr, 120, 50, 11000, n_fft, 1750)
    return fb.dot(np.abs(mag) ** 1)


def get_end(frames: np.ndarray, sr: int):
    hop_length = 281
    mel = mel_power1(frames, sr)
    start = 0
    chunk_length = sr // hop_length
    end = start + chunk_length
    file_length = len(frames) / sr
    while end < mel.shape[1]:
        data = mel[:, start:end]
        if np.amax(data) == np.amin(data):
            return start * hop_length // sr
        start = end
        end = start + chunk_length
    return file_length
