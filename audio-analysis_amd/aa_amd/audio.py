"""Recording decode (host side, outside the hot path).

The reference decodes with ffmpeg through audioread + librosa.load(sr=None)
(src/identify_tracks.py:49-62): ffmpeg converts every source to interleaved
signed 16-bit (``-f s16le``), librosa's ``buf_to_float`` scales by 1/32768 to
float32, and channels are averaged to mono.  This build reads RIFF/WAVE
directly (PCM 8/16/24/32-bit and IEEE float32/64) and applies the same s16
conversion ffmpeg's libswresample performs (no dither): u8 ``(x - 128) << 8``,
s24/s32 ``>> 16`` of the 32-bit value (truncation), float ``clip(lrint(x *
32768))`` -- so non-16-bit files give the reference's samples, not more
precise ones.  FLAC streams are decoded natively (``aa_flac_decode`` in
libaa.so, host code) and go through the same s16 conversion: ffmpeg's FLAC
decoder left-justifies a b-bit sample into s16 (b <= 16) or s32, so the s16
value is ``x << (16 - b)`` or ``x >> (b - 16)``.  Ogg Vorbis streams are
decoded natively too (``aa_vorbis_decode``, host code): ffmpeg's Vorbis decoder
outputs float, which libswresample converts to s16 as for float WAV
(``clip(lrint(x * 32768))``).  Other lossy containers (MP3, AAC/M4A, Opus)
need a codec this image does not have and are rejected.
Resampling to 48 kHz (librosa soxr_hq in the reference) runs on the GPU with
a filter designed to libsoxr's HQ specification (aa_amd.resample) -- parity
with libsoxr's samples unpinned: libsoxr is not available.
"""
from __future__ import annotations

import struct
import numpy as np


def _to_mono(q, channels):
    """ffmpeg s16 integers -> librosa.util.buf_to_float, then the channel mean."""
    x = q.astype(np.float32) / np.float32(32768.0)
    if channels > 1:
        x = x[: len(x) // channels * channels].reshape(-1, channels).mean(axis=1, dtype=np.float32)
    return np.ascontiguousarray(x, dtype=np.float32)


def _is_flac(data):
    if data[:3] == b"ID3" and len(data) >= 10:  # ID3v2 tag in front of the stream
        sz = (data[6] & 0x7F) << 21 | (data[7] & 0x7F) << 14 | (data[8] & 0x7F) << 7 | (data[9] & 0x7F)
        off = 10 + sz + (10 if data[5] & 0x10 else 0)
        return data[off:off + 4] == b"fLaC"
    return data[:4] == b"fLaC"


def decode_flac(data):
    """FLAC bytes -> (ffmpeg-s16 integers as int32 [frames * channels], channels, sr)."""
    import ctypes as C
    from ._lib import FlacInfo, check, lib
    buf = np.frombuffer(data, np.uint8)
    info = FlacInfo()
    check(lib().aa_flac_info(buf.ctypes.data, buf.size, C.byref(info)), "aa_flac_info")
    n = C.c_int64()
    # length not stated, or a header claiming more samples than any plausible
    # compression of this file holds (a bogus STREAMINFO must not size a huge
    # allocation): count the decodable frames first
    if info.total_frames == 0 or info.total_frames * info.channels > 64 * len(data) + (1 << 24):
        check(lib().aa_flac_decode(buf.ctypes.data, buf.size, None, 0, C.byref(n)), "aa_flac_decode")
        cap = n.value
    else:
        cap = info.total_frames
    out = np.empty(cap * info.channels, np.int32)
    check(lib().aa_flac_decode(buf.ctypes.data, buf.size, out.ctypes.data, cap, C.byref(n)), "aa_flac_decode")
    b = info.bits_per_sample
    q = out[: n.value * info.channels]
    q = q << (16 - b) if b <= 16 else q >> (b - 16)
    return q, info.channels, info.sample_rate


def _float_to_s16(f):
    """libswresample's packed float -> s16: av_clip_int16(lrint(x * 32768));
    a NaN converts to the integer indefinite (INT_MIN) and clips to -32768."""
    with np.errstate(invalid="ignore"):
        q = np.clip(np.rint(f.astype(np.float64) * 32768.0), -32768, 32767)
    return np.where(np.isnan(q), -32768.0, q)


def decode_vorbis(data):
    """Ogg Vorbis bytes -> (decoded float32 [frames * channels], channels, sr)."""
    import ctypes as C
    from ._lib import VorbisInfo, check, lib
    buf = np.frombuffer(data, np.uint8)
    info = VorbisInfo()
    check(lib().aa_vorbis_info(buf.ctypes.data, buf.size, C.byref(info)), "aa_vorbis_info")
    n = C.c_int64()
    # the last granule bounds the output; without one (or an implausible one:
    # Vorbis needs well over a bit per 64 samples) count the samples first
    if info.total_frames <= 0 or info.total_frames > 64 * 8 * len(data) + (1 << 20):
        check(lib().aa_vorbis_decode(buf.ctypes.data, buf.size, None, 0, C.byref(n)), "aa_vorbis_decode")
        cap = n.value
    else:
        cap = info.total_frames
    out = np.empty(max(cap, 1) * info.channels, np.float32)
    check(lib().aa_vorbis_decode(buf.ctypes.data, buf.size, out.ctypes.data, cap, C.byref(n)), "aa_vorbis_decode")
    return out[: n.value * info.channels], info.channels, info.sample_rate


def decode(path):
    with open(path, "rb") as f:
        data = f.read()
    if _is_flac(data):
        q, channels, sr = decode_flac(data)
        return _to_mono(q, channels), int(sr)
    if data[:4] == b"OggS":
        f, channels, sr = decode_vorbis(data)
        return _to_mono(_float_to_s16(f), channels), int(sr)
    if len(data) < 12 or data[:4] not in (b"RIFF", b"RF64") or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE, FLAC or Ogg Vorbis file")
    mv = memoryview(data)  # chunk bodies as views: no copy of the sample payload
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = mv[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", bytes(body[:16]))
            if fmt[0] == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: real tag in the GUID
                fmt = (struct.unpack("<H", bytes(body[24:26]))[0],) + fmt[1:]
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError(f"{path}: missing fmt/data chunk")
    tag, channels, sr, _, _, bits = fmt
    if tag == 1 and bits == 16:  # the common case in one pass: x = s16 * 2^-15 (== s16 / 32768 exactly)
        x = np.frombuffer(payload, "<i2", count=len(payload) // 2).astype(np.float32) * np.float32(1.0 / 32768.0)
        if channels > 1:
            x = x[: len(x) // channels * channels].reshape(-1, channels).mean(axis=1, dtype=np.float32)
        return np.ascontiguousarray(x, dtype=np.float32), int(sr)
    if tag == 1:  # PCM -> ffmpeg's s16
        if bits == 8:
            q = (np.frombuffer(payload, np.uint8).astype(np.int32) - 128) << 8
        elif bits == 16:
            q = np.frombuffer(payload[:len(payload) // 2 * 2], "<i2").astype(np.int32)
        elif bits == 24:
            b = np.frombuffer(payload[:len(payload) // 3 * 3], np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            q = v >> 8  # s24 -> s32 (<< 8) -> s16 (>> 16)
        elif bits == 32:
            q = np.frombuffer(payload[:len(payload) // 4 * 4], "<i4") >> 16
        else:
            raise ValueError(f"{path}: {bits}-bit PCM unsupported")
    elif tag == 3:  # IEEE float -> av_clip_int16(lrint(x * 32768))
        if bits not in (32, 64):
            raise ValueError(f"{path}: {bits}-bit IEEE float unsupported")
        f = np.frombuffer(payload[:len(payload) // (bits // 8) * (bits // 8)], "<f4" if bits == 32 else "<f8")
        q = _float_to_s16(f)
    else:
        raise ValueError(f"{path}: WAVE format tag {tag} unsupported")
    return _to_mono(q, channels), int(sr)


def resample(x, sr_in, sr_out):
    """librosa.resample(res_type="soxr_hq") to sr_out, on the GPU (aa_amd.resample)."""
    from .resample import resample as gpu_resample
    return gpu_resample(x, sr_in, sr_out)
