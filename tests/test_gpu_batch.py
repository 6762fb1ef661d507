"""The batched corpus path (aa_amd.batch, K recordings per device pass) writes
exactly the documents the per-file path writes (analyse.examine, one
recording at a time: src/analyse.py:434-470), byte for byte, over a mixed set
of files: mono and stereo PCM16 WAV (the pinned int16 fast path and
aa_pcm_s16_to_f32), FLAC and 44.1 kHz WAV (the load_recording fallback with
resampling), a recording with a silent tail (get_end), one too short for a
window, an unreadable file (failed alone), and the analyse_tracks mode with
sidecar tracks."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, str(Path(__file__).resolve().parent))


def _docs(res):
    return json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "processing_time_seconds"}
                       for k, v in res.items()}, sort_keys=True)


def _corpus(tmp_path):
    import wave
    import flac_writer as fw
    from tools import synth
    files = []
    for i in range(6):  # plain mono PCM16, 20 s
        p = tmp_path / f"m{i}.wav"
        synth.write_wav(p, synth.clip(300 + i, seconds=20.0))
        files.append(p)
    # stereo PCM16: the device-side channel mean
    x = synth.clip(310, seconds=12.0)
    q = np.clip(np.round(np.stack([x, 0.5 * x[::-1]], 1) * 32768), -32768, 32767).astype("<i2")
    p = tmp_path / "stereo.wav"
    with wave.open(str(p), "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(48000)
        w.writeframes(q.tobytes())
    files.append(p)
    # silent tail: get_end stops at the first constant chunk
    x = synth.clip(311, seconds=15.0)
    x[8 * 48000:] = 0
    p = tmp_path / "tail.wav"
    synth.write_wav(p, x)
    files.append(p)
    # 44.1 kHz: resampled on the host (fallback path)
    p = tmp_path / "r44.wav"
    synth.write_wav(p, synth.clip(312, seconds=10.0, sr=44100), sr=44100)
    files.append(p)
    # FLAC (native decoder, fallback path)
    y = np.round(synth.clip(313, seconds=8.0) * 32768).astype(np.int64)
    blocks = [y[i:i + 4096] for i in range(0, len(y), 4096)]
    frames = [fw.frame([b], 16, 48000, k) for k, b in enumerate(blocks)]
    p = tmp_path / "f.flac"
    p.write_bytes(fw.stream(frames, 48000, 1, 16, len(y), 4096))
    files.append(p)
    # shorter than one 3 s window
    p = tmp_path / "short.wav"
    synth.write_wav(p, synth.clip(314, seconds=2.0))
    files.append(p)
    # not audio: this file fails alone
    p = tmp_path / "broken.wav"
    p.write_bytes(b"RIFF\x00\x00\x00\x00WAVEjunk")
    files.append(p)
    return [str(f) for f in files]


def test_batch_matches_per_file(gpu, model_root, tmp_path):
    from aa_amd import corpus
    files = _corpus(tmp_path)
    models = [str(model_root / m / "audioModel.keras") for m in ("model1", "model2")]
    per_file = corpus.run(files, models, False, batch=0)
    assert sum(1 for d in per_file.values() if d.get("species_identify")) >= 6
    assert corpus.FAILED in per_file[len(files) - 1]
    # k = 2 with the default 3 lanes: more files than pinned slots ((3 + 2) * 2 =
    # 10 < 13), the slot pool then bounds the decodes in flight
    for k in (2, 3, 5, 16):
        batched = corpus.run(files, models, False, batch=k)
        assert _docs(batched) == _docs(per_file), k


def test_batch_matches_per_file_analyse_tracks(gpu, model_root, tmp_path):
    """analyse_tracks: tracks from the FILE.txt sidecars (src/identify_tracks.py:422-433),
    short tracks placed by the seeded RandomState; a file without a sidecar
    returns None from classify()."""
    from aa_amd import corpus
    from tools import synth
    files = []
    for i in range(9):
        p = tmp_path / f"t{i}.wav"
        synth.write_wav(p, synth.clip(400 + i, seconds=14.0))
        if i != 4:
            tracks = [{"id": 10 * i + j, "start": 1.0 + 3.1 * j, "end": 1.0 + 3.1 * j + (0.8 if j % 2 else 3.6),
                       "minFreq": 300.0 + 100 * j, "maxFreq": 9000.0} for j in range(3)]
            p.with_suffix(".txt").write_text(json.dumps({"Tracks": tracks}))
        files.append(str(p))
    models = [str(model_root / "model1" / "audioModel.keras"), str(model_root / "model3" / "audioModel.keras")]
    per_file = corpus.run(files, models, True, batch=0)
    batched = corpus.run(files, models, True, batch=4)
    assert _docs(batched) == _docs(per_file)
    assert per_file[0]["species_identify"] and not per_file[4]["species_identify"]


def test_pcm_s16_to_f32_matches_host_decode(gpu):
    """aa_pcm_s16_to_f32 == audio._to_mono (ffmpeg s16 / 32768, channel mean) bit for bit."""
    import torch
    from aa_amd import _lib
    from aa_amd.audio import _to_mono
    rng = np.random.default_rng(0)
    for ch in (1, 2, 3, 6):
        q = rng.integers(-32768, 32768, size=(10007 * ch,)).astype(np.int16)
        q[:ch * 4] = [-32768] * (ch * 4)
        dev = torch.from_numpy(q).cuda()
        out = torch.empty(10007, dtype=torch.float32, device="cuda")
        _lib.check(_lib.lib().aa_pcm_s16_to_f32(_lib.dptr(dev), 10007, ch, _lib.dptr(out), _lib.stream_ptr()),
                   "aa_pcm_s16_to_f32")
        assert np.array_equal(out.cpu().numpy(), _to_mono(q.astype(np.int32), ch)), ch
