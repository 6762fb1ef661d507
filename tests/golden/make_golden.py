"""Generate golden fixtures by importing the REFERENCE itself (read-only, from
/root/reference/src) with small shims for the libraries this image lacks.

Run in the build container (the GPU box has no /root/reference):

    python tests/golden/make_golden.py

Shims (only what the import needs; none of them computes a pinned quantity):
* ``librosa``: ``fft_frequencies`` = np.fft.rfftfreq (the only librosa call in
  src/custommel.py:25).  STFT / power_to_db are NOT shimmed: nothing generated
  here goes through them.
* ``tensorflow``: a ``register_keras_serializable`` decorator and a ``Layer``
  base class so src/identify_tracks.py:26 imports; ``tf.expand_dims`` only in
  the stubbed-out get_spect.
* ``audioread``, ``cv2``: empty modules (decode / morphology are stubbed).

Outputs (all small, committed):
* mel_f.npz              custommel.mel_f for several configs (src/custommel.py:19)
* normalize.npz          identify_tracks.normalize_data on small arrays (:202)
* windows.json           load_samples window tables (:65-199), captured with
                         get_spect stubbed and normalize=False over a clip whose
                         samples are 1..N, so each window's samples name their
                         source indices exactly
* postproc.json          analyse.species_identify (src/analyse.py:129-175) for
                         fixed per-window probabilities, through the real
                         classify() tail (:416-573) with decode, end/signal
                         detection and model.predict stubbed
* ebird_subset.json      the reference's region species lists restricted to
                         the ebird codes the build's label sets use (data)
"""
from __future__ import annotations

import json
import os
import sys
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference/src")
OUT = Path(__file__).resolve().parent


def install_shims():
    sys.dont_write_bytecode = True
    lib = types.ModuleType("librosa")
    lib.fft_frequencies = lambda sr=22050, n_fft=2048: np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    sys.modules["librosa"] = lib

    tf = types.ModuleType("tensorflow")

    class _Layer:
        def __init__(self, **kw):
            pass

        def add_weight(self, **kw):
            return None

    keras = types.SimpleNamespace(
        utils=types.SimpleNamespace(register_keras_serializable=lambda **kw: (lambda c: c)),
        layers=types.SimpleNamespace(Layer=_Layer),
        initializers=types.SimpleNamespace(Constant=lambda value=0.0: None),
        constraints=types.SimpleNamespace(MinMaxNorm=lambda **kw: None),
    )
    tf.keras = keras
    tf.expand_dims = lambda x, axis: np.expand_dims(x, axis)
    sys.modules["tensorflow"] = tf
    ar = types.ModuleType("audioread")
    ar.ffdec = types.ModuleType("audioread.ffdec")
    sys.modules["audioread"] = ar
    sys.modules["audioread.ffdec"] = ar.ffdec
    sys.modules["cv2"] = types.ModuleType("cv2")
    sys.path.insert(0, str(REF))


def gen_mel():
    import custommel
    cfgs = {
        "htk160_4096": (48000, 160, 50, 11000, 4096, 1750),
        "htk120_4800": (48000, 120, 50, 11000, 4800, 1750),
        "htk80_4096_b1000": (48000, 80, 50, 11000, 4096, 1000),
        "htk96_2048": (48000, 96, 100, 8000, 2048, 1750),
    }
    arrays = {}
    for k, c in cfgs.items():
        arrays[k] = custommel.mel_f(*c)
        arrays[k + "__cfg"] = np.asarray(c, dtype=np.float64)
    np.savez_compressed(OUT / "mel_f.npz", **arrays)


def gen_normalize():
    import identify_tracks as it
    rng = np.random.default_rng(7)
    arrays = {}
    for i, n in enumerate([1000, 4097, 144000]):
        x = (rng.standard_normal(n) * 0.1).astype(np.float32)
        if i == 0:
            x[:100] = 0.0  # zero padding is normalised too (:165-170)
        if n == 144000:
            x = x[::48]  # keep the fixture small: 3000 samples
        arrays[f"in{i}"] = x
        arrays[f"out{i}"] = it.normalize_data(x)
    np.savez_compressed(OUT / "normalize.npz", **arrays)


def gen_windows():
    import identify_tracks as it
    captured = []
    it.get_spect = lambda data, *a, **k: captured.append(np.array(data)) or np.zeros(1)
    sr = 48000
    cases = [
        # (clip_seconds, [(start, end, fmin, fmax)], pad_short, seed)
        (60.0, [(0, 60, 0, 24000)], False, 0),
        (60.0, [(0, 3, 0, 24000), (0, 2.9, 0, 24000), (57.5, 60, 0, 24000)], False, 1),
        (60.0, [(1.0, 1.5, 0, 24000), (10.3, 17.77, 200, 5000), (55, 65, 0, 24000)], False, 2),
        (60.0, [(5, 9, 12000, 14000), (5, 9, 0, 40)], False, 3),
        (60.0, [(0.25, 2.0, 0, 24000), (30.1, 31.0, 0, 24000), (12.345, 20.0, 0, 24000)], True, 4),
        (2.0, [(0, 2.0, 0, 24000)], False, 5),
        (2.0, [(0.5, 1.0, 0, 24000)], True, 6),
        (37.3, [(0, 37.3, 0, 24000), (33.3, 37.3, 0, 24000)], False, 7),
        (61.0, [(58.9, 61.0, 100, 3000), (0.0, 0.1, 0, 24000)], False, 8),
    ]
    out = []
    for clip_s, tracks, pad_short, seed in cases:
        n = int(round(clip_s * sr))
        frames = np.arange(1, n + 1, dtype=np.float32)
        sigs = []
        for (s, e, f0, f1) in tracks:
            sigs.append(it.Signal(s, e, f0, f1))
        np.random.seed(seed)
        captured.clear()
        try:
            res = it.load_samples(frames, sr, sigs, 3, 1.5, 640, normalize=False,
                                  pad_short_tracks=pad_short, fmin=50, fmax=11000)
        except Exception as e:  # the reference's own failure mode is part of the contract
            out.append({"clip_samples": n, "sr": sr, "tracks": tracks,
                        "pad_short_tracks": pad_short, "seed": seed, "segment_length": 3,
                        "segment_stride": 1.5, "fmin": 50, "fmax": 11000,
                        "error": type(e).__name__})
            continue
        per_track = []
        k = 0
        for tr in res:
            wins = []
            for _ in tr:
                d = captured[k]
                k += 1
                nz = np.flatnonzero(d)
                if len(nz) == 0:
                    wins.append([0, 0, 0])
                    continue
                left = int(nz[0])
                vals = d[nz]
                assert np.all(np.diff(vals) == 1) and len(nz) == nz[-1] - nz[0] + 1
                wins.append([int(vals[0]) - 1, int(len(nz)), left])
            per_track.append(wins)
        out.append({"clip_samples": n, "sr": sr, "tracks": tracks, "pad_short_tracks": pad_short,
                    "seed": seed, "segment_length": 3, "segment_stride": 1.5,
                    "fmin": 50, "fmax": 11000, "windows": per_track})
    with open(OUT / "windows.json", "w") as f:
        json.dump(out, f, indent=1)


def main():
    install_shims()
    gen_mel()
    gen_normalize()
    gen_windows()
    print("wrote", sorted(p.name for p in OUT.glob("*.npz")) + sorted(p.name for p in OUT.glob("*.json")))


if __name__ == "__main__":
    main()
