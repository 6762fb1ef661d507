"""Decode semantics of load_recording (reference src/identify_tracks.py:49-62):
ffmpeg -> interleaved s16 (libswresample, no dither) -> librosa buf_to_float
(int16 / 32768, float32) -> mono mean over channels.  Known-answer vectors
per WAV sample format: what ffmpeg's s16 conversion gives for each input
(u8 ``(x-128) << 8``; s24/s32 arithmetic ``>> 16`` of the 32-bit value; float
``av_clip_int16(lrint(x * 32768))``, round half to even)."""
import struct

import numpy as np
import pytest

from aa_amd.audio import decode


def _wav(path, tag, channels, sr, bits, payload):
    fmt = struct.pack("<HHIIHH", tag, channels, sr, sr * channels * bits // 8, channels * bits // 8, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(payload)) + payload
    if len(payload) % 2:
        body += b"\0"
    path.write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)
    return path


def _s16(vals):
    return np.asarray(vals, np.float32) / np.float32(32768)


def test_pcm16_exact(tmp_path):
    v = np.array([0, 1, -1, 32767, -32768, 12345], "<i2")
    x, sr = decode(_wav(tmp_path / "a.wav", 1, 1, 48000, 16, v.tobytes()))
    assert sr == 48000 and x.dtype == np.float32
    np.testing.assert_array_equal(x, _s16(v))


def test_pcm8(tmp_path):
    v = np.array([0, 1, 127, 128, 129, 255], np.uint8)
    x, _ = decode(_wav(tmp_path / "a.wav", 1, 1, 16000, 8, v.tobytes()))
    np.testing.assert_array_equal(x, _s16([-32768, -32512, -256, 0, 256, 32512]))


def test_pcm24_truncates_to_s16(tmp_path):
    vals = [0, 255, 256, -1, -256, -257, 0x7FFFFF, -0x800000, 0x123456]
    raw = b"".join(struct.pack("<i", v)[:3] for v in vals)
    x, _ = decode(_wav(tmp_path / "a.wav", 1, 1, 48000, 24, raw))
    np.testing.assert_array_equal(x, _s16([0, 0, 1, -1, -1, -2, 32767, -32768, 0x1234]))


def test_pcm32_truncates_to_s16(tmp_path):
    v = np.array([0, 65535, 65536, -1, -65537, 2**31 - 1, -2**31], "<i4")
    x, _ = decode(_wav(tmp_path / "a.wav", 1, 1, 48000, 32, v.tobytes()))
    np.testing.assert_array_equal(x, _s16([0, 0, 1, -1, -2, 32767, -32768]))


@pytest.mark.parametrize("bits", [32, 64])
def test_float_rounds_half_even_and_clips(tmp_path, bits):
    v = np.array([0.0, 0.5 / 32768, 1.5 / 32768, 2.5 / 32768, -1.5 / 32768, 0.25, 1.0, 1.7, -1.0, -2.0],
                 "<f4" if bits == 32 else "<f8")
    x, _ = decode(_wav(tmp_path / "a.wav", 3, 1, 48000, bits, v.tobytes()))
    np.testing.assert_array_equal(x, _s16([0, 0, 2, 2, -2, 8192, 32767, 32767, -32768, -32768]))


def test_stereo_mean_of_s16(tmp_path):
    v = np.array([[100, 201], [-32768, 32767], [3, -4]], "<i2")
    x, _ = decode(_wav(tmp_path / "a.wav", 1, 2, 44100, 16, v.tobytes()))
    f = _s16(v.reshape(-1)).reshape(-1, 2)
    np.testing.assert_array_equal(x, ((f[:, 0] + f[:, 1]) / np.float32(2)).astype(np.float32))


def test_rejects_non_wav(tmp_path):
    p = tmp_path / "a.mp3"
    p.write_bytes(b"ID3" + b"\0" * 64)
    with pytest.raises(ValueError):
        decode(p)
    p = tmp_path / "a.ogg"  # an Ogg capture pattern without a valid page / Vorbis stream
    p.write_bytes(b"OggS" + b"\0" * 64)
    with pytest.raises(RuntimeError):
        decode(p)
    p = tmp_path / "a.flac"  # a FLAC marker with a broken metadata chain
    p.write_bytes(b"fLaC" + b"\0" * 64)
    with pytest.raises(RuntimeError):
        decode(p)
