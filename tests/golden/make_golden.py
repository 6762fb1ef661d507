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
* tracks.json            get_tracks_from_signals (:795-842) on seeded random
                         signal sets (the track builder of analyse_tracks=False)
* filtered.json          load_samples (:65-199) with filter_freqs / filter_below
                         (:152-162, butter_bandpass_filter :1053-1056, scipy),
                         normalize=False, on a seeded int16-quantised noise clip:
                         per window its length, sum, sum of squares and the
                         samples at 16 fixed positions (the windows themselves
                         are 144,000 samples each)
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


POSTPROC_CASES = [
    # name, location, species file present, tracks (id, start, end, minFreq, maxFreq), seed
    ("nz_default", None, True,
     [(1, 0.0, 12.0, None, None), (2, 3.2, 4.1, 800, 6000), (3, 20.0, 29.5, 12000, 15000),
      (4, 30.0, 45.0, 100, 9000), (5, 50.0, 60.0, None, None)], 11),
    ("auckland", {"lat": -36.85, "lng": 174.76}, True,
     [(7, 0.0, 9.0, None, None), (8, 10.5, 11.0, 500, 3000), (9, 40.0, 55.0, 200, 4000)], 12),
    ("no_species_file", {"lat": -43.5, "lng": 172.6}, False,
     [(3, 1.0, 7.0, None, None), (4, 8.0, 16.0, None, None)], 13),
]

# analyse_tracks=False: tracks built from these signals (start, end, f0, f1) by
# the reference's get_tracks_from_signals; the JSON carries chirps/signals
SIGNAL_CASES = [
    ("signals_nz", None, True,
     [(1.0, 1.6, 1500.0, 3000.0), (1.5, 2.2, 1600.0, 3200.0), (10.0, 10.4, 800.0, 900.0),
      (20.0, 21.5, 4000.0, 6000.0), (20.2, 21.0, 4100.0, 5500.0), (40.0, 43.0, 300.0, 2500.0),
      (55.0, 55.2, 100.0, 9000.0)], 21),
    ("signals_auckland", {"lat": -36.85, "lng": 174.76}, True,
     [(0.5, 1.5, 2000.0, 2600.0), (3.0, 5.0, 900.0, 4000.0), (30.0, 31.0, 6000.0, 9000.0)], 22),
]


def _model_metas():
    sys.path.insert(0, str(OUT.parents[1]))
    from tools.make_models import DEFAULT_META, EBIRD, LABELS
    def meta(name, labels, pre=False, thr=0.7):
        m = dict(DEFAULT_META)
        m.update(name=name, labels=labels, ebird_ids=[EBIRD.get(l, []) for l in labels],
                 pre_model=pre, threshold=thr)
        return m
    pre_labels = ["bird", "human", "insect", "morepork", "noise"]
    return {"model1": meta("model1", LABELS), "model2": meta("model2", LABELS),
            "premodel": meta("premodel", pre_labels, pre=True, thr=0.6)}


def _fake_probs(name, call, W, L, seed):
    rng = np.random.default_rng([seed, call, sum(map(ord, name))])
    p = rng.beta(0.6, 1.4, size=(W, L))
    hot = rng.choice(L, size=min(3, L), replace=False)
    p[:, hot] = rng.uniform(0.55, 1.0, size=(W, len(hot)))
    return p.astype(np.float32)


def gen_postproc():
    import tempfile
    import identify_tracks as it
    import analyse
    metas = _model_metas()
    out_json, arrays = {}, {}
    cases = [(c, None) for c in POSTPROC_CASES] + [((n, l, sf, [], sd), sig) for (n, l, sf, sig, sd) in SIGNAL_CASES]
    for (name, location, species_file, tracks, seed), signals in cases:
        calls = {"n": 0}
        class FakeModel:
            def __init__(self, mname):
                self.mname = mname
            def predict(self, x):
                probs = _fake_probs(self.mname, calls["n"], len(x), len(metas[self.mname]["labels"]), seed)
                arrays[f"{name}__call{calls['n']}"] = probs
                calls["n"] += 1
                return probs
        it.load_recording = lambda f, resample=48000: (np.ones(60 * 48000, np.float32) * 0.01, 48000)
        it.get_end = lambda frames, sr: 60.0
        it.signal_noise = (lambda frames, sr, hop=281, _s=signals: [it.Signal(*x) for x in (_s or [])])
        it.load_model_meta = lambda p: metas[Path(p).parent.name]
        it.load_model = lambda p, meta: FakeModel(Path(p).parent.name)
        it.get_spect = lambda data, *a, **k: np.zeros((1,), np.float32)
        analyse.classify = it.classify
        with tempfile.TemporaryDirectory() as d:
            rec = Path(d) / "rec.wav"
            rec.write_bytes(b"")
            meta = {"Tracks": []}
            for tid, s0, s1, f0, f1 in tracks:
                t = {"id": tid, "start": s0, "end": s1}
                if f0 is not None:
                    t["minFreq"], t["maxFreq"] = f0, f1
                meta["Tracks"].append(t)
            if location is not None:
                meta["location"] = location
            (Path(d) / "rec.txt").write_text(json.dumps(meta))
            models = [f"/m/{m}/audioModel.keras" for m in ("model1", "model2", "premodel")]
            cwd = os.getcwd()
            os.chdir(str(REF.parent) if species_file else d)
            try:
                np.random.seed(seed)
                res = analyse.species_identify(str(rec), models, signals is None)
            finally:
                os.chdir(cwd)
        out_json[name] = {"meta": meta, "models": ["model1", "model2", "premodel"], "seed": seed,
                          "signals": signals,
                          "species_file": species_file, "n_calls": calls["n"],
                          "result": json.loads(json.dumps(res, sort_keys=True))}
    with open(OUT / "postproc.json", "w") as f:
        json.dump({"metas": metas, "cases": out_json}, f, indent=1, sort_keys=True)
    np.savez_compressed(OUT / "postproc_probs.npz", **arrays)
    # species lists restricted to the codes the build's labels use (data only)
    codes = {c for m in metas.values() for ids in m["ebird_ids"] for c in ids}
    with open(REF / "ebird_species.json") as f:
        sp = json.load(f)
    subset = {k: {"region": {"info": v["region"]["info"]},
                  "species": [c for c in v["species"] if c in codes]} for k, v in sp.items()}
    with open(OUT / "ebird_subset.json", "w") as f:
        json.dump(subset, f, indent=1, sort_keys=True)


def gen_tracks():
    import identify_tracks as it
    freqs = np.fft.rfftfreq(n=4096, d=1.0 / 48000)
    cases = []
    for seed in range(40):
        rng = np.random.default_rng(1000 + seed)
        n = int(rng.integers(0, 30))
        end = float(rng.choice([60.0, 59.7, 30.0]))
        sigs = []
        for _ in range(n):
            left = int(rng.integers(0, int(end * 48000 / 281)))
            width = int(rng.integers(28, 600))
            top = int(rng.integers(0, 1200))
            height = int(rng.integers(10, 400))
            if rng.random() < 0.3 and sigs:  # near-duplicates exercise the merge rules
                b = sigs[int(rng.integers(0, len(sigs)))]
                left, top = b[0] + int(rng.integers(-40, 40)), max(0, b[1] + int(rng.integers(-20, 20)))
                left = max(0, left)
            sigs.append((left, top, width, height))
        inp = [[l * 281 / 48000, (l + w) * 281 / 48000, float(freqs[t]), float(freqs[min(2048, t + h)])]
               for (l, t, w, h) in sigs]
        tr = it.get_tracks_from_signals([it.Signal(*a) for a in inp], end)
        cases.append({"end": end, "signals": inp,
                      "tracks": [[float(x.start), float(x.end), float(x.freq_start), float(x.freq_end)]
                                 for x in tr]})
    with open(OUT / "tracks.json", "w") as f:
        json.dump(cases, f, indent=1)


FILTER_POS = [0, 1, 2, 3, 100, 1000, 5000, 20000, 47999, 48000, 72000, 100000, 120000, 143997, 143998, 143999]


def filter_clip(n, seed=11):
    rng = np.random.default_rng(seed)
    return (np.round(rng.standard_normal(n) * 0.1 * 32768) / 32768).astype(np.float32)


def gen_filtered():
    import identify_tracks as it
    captured = []
    it.get_spect = lambda data, *a, **k: captured.append(np.array(data)) or np.zeros(1)
    sr = 48000
    frames = filter_clip(20 * sr)
    cases = [
        # (tracks (start, end, fmin, fmax), filter_freqs, filter_below, pad_short, seed)
        ([(0.5, 7.2, 500, 4000), (9.0, 10.0, 0, 3000), (12.0, 19.0, 1500, 9000)], True, None, False, 0),
        ([(0.5, 7.2, 500, 4000), (9.0, 10.0, 0, 3000), (12.0, 19.0, 1500, 9000)], False, 5000, False, 1),
        ([(1.0, 2.0, 800, 2500), (3.0, 8.5, 100, 12000)], True, None, True, 2),
    ]
    out = []
    for tracks, ff, fb, pad_short, seed in cases:
        np.random.seed(seed)
        captured.clear()
        res = it.load_samples(frames, sr, [it.Signal(*t) for t in tracks], 3, 1.5, 640, normalize=False,
                              pad_short_tracks=pad_short, fmin=50, fmax=11000, filter_freqs=ff, filter_below=fb)
        per_track, k = [], 0
        for tr in res:
            wins = []
            for _ in tr:
                d = np.asarray(captured[k], dtype=np.float64)
                k += 1
                wins.append({"n": int(len(d)), "sum": float(d.sum()), "sumsq": float((d * d).sum()),
                             "at": [float(d[i]) for i in FILTER_POS]})
            per_track.append(wins)
        out.append({"sr": sr, "clip_seconds": 20, "clip_seed": 11, "tracks": tracks, "filter_freqs": ff,
                    "filter_below": fb, "pad_short_tracks": pad_short, "seed": seed, "segment_length": 3,
                    "segment_stride": 1.5, "fmin": 50, "fmax": 11000, "positions": FILTER_POS,
                    "windows": per_track})
    with open(OUT / "filtered.json", "w") as f:
        json.dump(out, f, indent=1)


def main():
    install_shims()
    gen_mel()
    gen_normalize()
    gen_windows()
    gen_postproc()
    gen_tracks()
    gen_filtered()
    print("wrote", sorted(p.name for p in OUT.glob("*.npz")) + sorted(p.name for p in OUT.glob("*.json")))


if __name__ == "__main__":
    main()
