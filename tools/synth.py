"""Synthetic 48 kHz mono recordings for tests and benchmarks.

A clip is pink-ish noise at -30 dBFS plus 3-8 linear chirps (0.2-1.0 s,
500-8000 Hz, -12 dBFS, Hann-shaped), quantised to int16 and scaled by 1/32768
exactly like a decoded PCM16 file.  ``numpy.random.default_rng(seed)`` with
seed = clip index makes every clip reproducible on any host.
"""
from __future__ import annotations

import numpy as np

SR = 48000


def clip(seed: int, seconds: float = 60.0, sr: int = SR) -> np.ndarray:
    rng = np.random.default_rng(seed)
    n = int(round(seconds * sr))
    spec = np.fft.rfft(rng.standard_normal(n))
    hz = np.fft.rfftfreq(n, 1.0 / sr)
    spec[1:] /= np.sqrt(hz[1:])
    spec[0] = 0.0
    x = np.fft.irfft(spec, n)
    x *= 10 ** (-30 / 20) / max(np.std(x), 1e-12)
    t = np.arange(n) / sr
    for _ in range(int(rng.integers(3, 9))):
        dur = rng.uniform(0.2, 1.0)
        t0 = rng.uniform(0.0, max(seconds - dur, 0.0))
        f0, f1 = rng.uniform(500, 8000, size=2)
        i0, i1 = int(t0 * sr), min(n, int((t0 + dur) * sr))
        tt = t[i0:i1] - t0
        phase = 2 * np.pi * (f0 * tt + (f1 - f0) * tt * tt / (2 * dur))
        x[i0:i1] += 10 ** (-12 / 20) * np.sin(phase) * np.hanning(i1 - i0)
    q = np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16)
    return (q.astype(np.float32) / 32768.0).astype(np.float32)


def tone(freq: float = 1000.0, seconds: float = 60.0, amp: float = 0.5, sr: int = SR) -> np.ndarray:
    t = np.arange(int(round(seconds * sr))) / sr
    q = np.round(amp * np.sin(2 * np.pi * freq * t) * 32768.0).astype(np.int16)
    return (q.astype(np.float32) / 32768.0).astype(np.float32)


def write_wav(path, samples: np.ndarray, sr: int = SR) -> None:
    """Write float samples in [-1, 1) as a mono PCM16 WAV."""
    import wave
    q = np.clip(np.round(np.asarray(samples, dtype=np.float64) * 32768.0), -32768, 32767)
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(q.astype("<i2").tobytes())
