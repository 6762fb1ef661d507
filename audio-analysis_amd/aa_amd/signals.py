"""signal_noise (src/identify_tracks.py:650-706) on the GPU through libaa.so.

The reference takes |STFT| (n_fft 4096, hop 281) of the whole recording with
librosa, keeps the pixels above 3x both their row and their column median,
cleans that mask with cv2 morphology and returns each large enough 8-connected
component as Signal(start, end, freq_start, freq_end).  aa_sn_run
(csrc/aa_signal.hip) runs every step on the device and hands back the few kept
components; the host only orders them and converts them with the reference's
own arithmetic (:687-704).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib

SIGNAL_WIDTH = 0.25  # src/identify_tracks.py:21
N_FFT = 4096         # :652
FREQ_RANGE = 100.0   # :675
N_BINS = N_FFT // 2 + 1


def _config(sr, hop_length):
    return _lib.SnConfig(sr=int(sr), n_fft=N_FFT, hop_length=int(hop_length), signal_width=SIGNAL_WIDTH,
                         freq_range=FREQ_RANGE)


def geometry(sr, hop_length=281):
    """(dilate height, dilate width, erode height, erode width, min width, min
    height) that the plan derives from (sr, hop) (:673-691)."""
    g = (C.c_int32 * 6)()
    cfg = _config(sr, hop_length)
    _lib.check(_lib.lib().aa_sn_geometry(C.byref(cfg), g), "aa_sn_geometry")
    return tuple(g)


class SignalDetector(_lib.StageTiming):
    """One device plan per (sample rate, hop); the workspace grows with the
    longest recording seen.  Stage timing (aa_sn_stage_*): per-launch HIP
    events, an item being one STFT frame."""
    _timing_prefix = "aa_sn"

    def __init__(self, sr=48000, hop_length=281, device=None, max_components=65536):
        self.sr, self.hop = int(sr), int(hop_length)
        self.device = torch.device(device or "cuda")
        cfg = _config(self.sr, self.hop)
        h = C.c_void_p()
        _lib.check(_lib.lib().aa_sn_create(C.byref(cfg), C.byref(h)), "aa_sn_create")
        self._h = h
        self.freqs = np.fft.rfftfreq(n=N_FFT, d=1.0 / self.sr)  # librosa.fft_frequencies
        self.max_components = int(max_components)
        self._out = torch.empty((self.max_components, 6), dtype=torch.int32, device=self.device)
        self._n = torch.zeros(2, dtype=torch.int32, device=self.device)
        self._ws = None

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().aa_sn_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def n_frames(self, n_samples: int) -> int:
        return 1 + int(n_samples) // self.hop

    def words(self, n_frames: int) -> int:
        return (int(n_frames) + 63) // 64

    def _workspace(self, n_samples):
        need = _lib.lib().aa_sn_workspace_bytes(self._h, int(n_samples))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def components(self, pcm, mask_out=None, stream=None) -> np.ndarray:
        """Kept components of a device float32 recording: int64 rows (left,
        top, width, height, area), ordered like the reference's stable sort on
        left over OpenCV's label order (:687-691).  mask_out: optional device
        int64 [2049, words] tensor receiving the mask before morphology."""
        n = int(pcm.numel())
        ws = self._workspace(n)
        rc = _lib.lib().aa_sn_run(self._h, _lib.dptr(pcm) if n else 0, n, _lib.dptr(ws), ws.numel(),
                                  _lib.dptr(self._out), self.max_components, _lib.dptr(self._n),
                                  _lib.dptr(mask_out), _lib.stream_ptr(stream))
        _lib.check(rc, "aa_sn_run")
        return self._collect()

    def spectrogram(self, pcm, stream=None):
        """np.abs(librosa.stft(frames, n_fft=4096, hop_length=hop)) (:654) of a
        device float32 recording, in the reference's precision (f64 transform,
        complex64 rounding, numpy's magnitude): a device float32 [2049, F]
        view of a frame-major [F, 2049] tensor."""
        n = int(pcm.numel())
        F = self.n_frames(n)
        out = torch.empty((F, N_BINS), dtype=torch.float32, device=self.device)
        rc = _lib.lib().aa_sn_spectrogram(self._h, _lib.dptr(pcm) if n else 0, n, _lib.dptr(out), N_BINS,
                                          _lib.stream_ptr(stream))
        _lib.check(rc, "aa_sn_spectrogram")
        return out.t()

    def components_from_mask(self, mask, n_frames, stream=None) -> np.ndarray:
        """The same from a device int64 [2049, words] mask (aa_sn_run's
        mask_out layout): morphology, components, size filter."""
        ws = self._workspace((int(n_frames) - 1) * self.hop)
        rc = _lib.lib().aa_sn_components_from_mask(self._h, _lib.dptr(mask), int(n_frames), _lib.dptr(ws),
                                                   ws.numel(), _lib.dptr(self._out), self.max_components,
                                                   _lib.dptr(self._n), _lib.stream_ptr(stream))
        _lib.check(rc, "aa_sn_components_from_mask")
        return self._collect()

    def _collect(self) -> np.ndarray:
        cnt, status = (int(x) for x in self._n.cpu())
        if status & _lib.AA_SN_NONFINITE:
            raise ValueError("Audio buffer is not finite everywhere")  # librosa valid_audio
        if status & _lib.AA_SN_RUN_OVERFLOW:
            raise _lib.AAError("aa_sn_run: run table overflow")
        if cnt > self.max_components:
            raise _lib.AAError(f"aa_sn_run: {cnt} components > {self.max_components}")
        rows = self._out[:cnt].cpu().numpy().astype(np.int64)
        rows = rows[np.lexsort((rows[:, 5], rows[:, 0]))]  # left, then OpenCV label order
        return rows[:, :5]

    def to_tuples(self, stats):
        """(start, end, freq_start, freq_end) per component, as :698-704
        computes them (the 281 there is a literal)."""
        out = []
        for s in stats:
            left, top, width, height = (int(v) for v in s[:4])
            max_freq = min(len(self.freqs) - 1, top + height)
            out.append((left * 281 / self.sr, (left + width) * 281 / self.sr, self.freqs[top],
                        self.freqs[max_freq]))
        return out

    def signal_noise(self, frames=None, pcm=None):
        if pcm is None:
            pcm = torch.from_numpy(np.ascontiguousarray(frames, dtype=np.float32)).to(self.device)
        return self.to_tuples(self.components(pcm))


_detectors = {}


def detector(sr, hop_length=281, device=None) -> SignalDetector:
    key = (int(sr), int(hop_length), str(device or "cuda"))
    if key not in _detectors:
        _detectors[key] = SignalDetector(sr, hop_length, device)
    return _detectors[key]
