"""GPU log-mel front end (host side of aa_fe_*).

One ``FrontEnd`` per distinct front-end configuration (the first model of a
group configures it, src/identify_tracks.py:465-497).  ``run`` takes the whole
recording resident on the device plus a device table of window views and
returns ``[n_win, n_mels, T, channels]`` float32 -- the stack of what
``get_spect`` returns per window (src/identify_tracks.py:212-288).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, melbank


@dataclass(frozen=True)
class FeSettings:
    sr: int = 48000
    segment_length: float = 3
    n_fft: int = 4096
    hop_length: int = 640
    n_mels: int = 160
    fmin: float = 50
    fmax: float = 11000
    break_freq: float = 1750
    htk: bool = False
    power: float = 2
    db_scale: bool = True
    normalize: bool = True
    mean_sub: bool = False
    channels: int = 1

    @property
    def win_len(self) -> int:
        return int(self.sr * self.segment_length)

    @property
    def n_frames(self) -> int:
        return 1 + self.win_len // self.hop_length

    def filterbank(self) -> np.ndarray:
        if self.htk:
            # src/identify_tracks.py:254-264: fmax only honoured when fmin is set
            fmin = 50 if self.fmin is None else self.fmin
            fmax = 11000 if self.fmin is None else self.fmax
            return melbank.htk_break(self.sr, self.n_mels, fmin, fmax, self.n_fft, self.break_freq)
        # librosa.feature.melspectrogram branch: fixed 50..11000 Hz, power 2
        return melbank.slaney(self.sr, self.n_fft, self.n_mels, 50, 11000)

    @property
    def effective_power(self) -> float:
        return float(self.power) if self.htk else 2.0


class FrontEnd(_lib.StageTiming):
    _timing_prefix = "aa_fe"

    def __init__(self, s: FeSettings, device=None, out_dtype=torch.float32):
        """out_dtype: torch.float32 (what get_spect returns) or torch.float16
        (BASELINE configs[4]'s fp16 log-mel; aa_fe_config.out_f16)."""
        self.s = s
        self.device = torch.device(device or "cuda")
        if out_dtype not in (torch.float32, torch.float16):
            raise ValueError(f"log-mel dtype {out_dtype}: float32 or float16")
        self.out_dtype = out_dtype
        L = _lib.lib()
        cfg = _lib.FeConfig(
            win_len=s.win_len, n_fft=int(s.n_fft), hop=int(s.hop_length), n_mels=int(s.n_mels),
            normalize=int(bool(s.normalize)), db_scale=int(bool(s.db_scale)),
            power=float(s.effective_power), amin=1e-10, top_db=80.0,
            mean_sub=int(bool(s.mean_sub)), channels=int(s.channels),
            out_f16=int(out_dtype == torch.float16))
        fb = np.ascontiguousarray(s.filterbank(), dtype=np.float32)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(L.aa_fe_create(C.byref(cfg), fb.ctypes.data, C.byref(h)), "aa_fe_create")
        self._h = h
        self.T = L.aa_fe_n_frames(h)
        self._ws = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.lib().aa_fe_destroy(h)
            self._h = None

    def workspace_bytes(self, n_win: int) -> int:
        return int(_lib.lib().aa_fe_workspace_bytes(self._h, int(n_win)))

    def _workspace(self, n_win: int) -> torch.Tensor:
        need = self.workspace_bytes(n_win)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        return self._ws

    def out_shape(self, n_win: int):
        return (n_win, self.s.n_mels, self.T, self.s.channels)

    def run(self, pcm: torch.Tensor, windows: torch.Tensor, out: torch.Tensor = None,
            status: torch.Tensor = None, stream=None, workspace: torch.Tensor = None) -> torch.Tensor:
        """pcm: float32 [N] on device; windows: int64 [n_win, 2] packed aa_window
        rows (see ``pack_windows``) on device."""
        n_win = int(windows.shape[0])
        if out is None:
            out = torch.empty(self.out_shape(n_win), dtype=self.out_dtype, device=self.device)
        if n_win == 0:
            return out
        assert pcm.dtype == torch.float32 and windows.dtype == torch.int64
        assert tuple(out.shape) == self.out_shape(n_win) and out.dtype == self.out_dtype
        ws = workspace if workspace is not None else self._workspace(n_win)
        _lib.check(_lib.lib().aa_fe_run(
            self._h, _lib.dptr(pcm), int(pcm.numel()), _lib.dptr(windows), n_win, _lib.dptr(out),
            _lib.dptr(status), _lib.dptr(ws), int(ws.numel()), _lib.stream_ptr(stream)), "aa_fe_run")
        return out


def pack_windows(views, n_samples: int, offset: int = 0, win_len: int = None) -> np.ndarray:
    """(src, n_valid, pad_left) views -> int64 [n, 2] rows laid out like
    struct aa_window {int64 src; int32 n_valid; int32 pad_left;}.  ``offset``
    shifts ``src`` when several recordings share one PCM buffer."""
    arr = np.zeros((len(views), 2), dtype=np.int64)
    for i, (src, n_valid, pad_left) in enumerate(views):
        if n_valid < 0 or src < 0 or src + n_valid > n_samples or pad_left < 0:
            raise ValueError(f"window {i} outside the recording")
        if win_len is not None and pad_left + n_valid > win_len:
            raise ValueError(f"window {i} longer than {win_len} samples")
        arr[i, 0] = src + offset
        arr[i, 1] = (int(n_valid) & 0xFFFFFFFF) | (int(pad_left) << 32)
    return arr
