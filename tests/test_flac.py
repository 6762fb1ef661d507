"""FLAC decode (aa_flac_* in libaa.so, host code) for load_recording
(src/identify_tracks.py:49-62): every subframe / residual / stereo / header
feature of RFC 9639 round-trips bit-exactly through the test encoder
(tests/flac_writer.py), and a FLAC file decodes to the same samples as a WAV
of the same integers (the s16 conversion ffmpeg applies, then /32768 and the
channel mean).  Parity vs ffmpeg itself is unpinned (no codec in the image)."""
import struct

import numpy as np
import pytest

import flac_writer as fw
from aa_amd import audio
from aa_amd._lib import AAError


def _signal(rng, n, bps, kind="smooth"):
    lim = (1 << (bps - 1)) - 1
    if kind == "noise":
        x = rng.integers(-lim - 1, lim + 1, n)
    else:
        t = np.arange(n)
        x = 0.6 * lim * np.sin(2 * np.pi * t * rng.uniform(0.001, 0.05)) + rng.normal(0, lim * 0.01, n)
        x = np.clip(np.round(x), -lim - 1, lim)
    return x.astype(np.int64)


def _decode_ints(data):
    q, ch, sr = _raw(data)
    return q, ch, sr


def _raw(data):
    """decoded stream integers (before the s16 conversion)"""
    import ctypes as C
    from aa_amd._lib import FlacInfo, check, lib
    buf = np.frombuffer(data, np.uint8)
    info = FlacInfo()
    check(lib().aa_flac_info(buf.ctypes.data, buf.size, C.byref(info)), "info")
    n = C.c_int64()
    check(lib().aa_flac_decode(buf.ctypes.data, buf.size, None, 0, C.byref(n)), "count")
    out = np.empty(max(n.value, 1) * info.channels, np.int32)
    check(lib().aa_flac_decode(buf.ctypes.data, buf.size, out.ctypes.data, n.value, C.byref(n)), "decode")
    return out[: n.value * info.channels].reshape(-1, info.channels), info.channels, info.sample_rate


def test_crc_catalogue_values():
    # CRC-8 (poly 0x07) and CRC-16 (poly 0x8005, "BUYPASS") check values of "123456789"
    assert fw.crc8(b"123456789") == 0xF4
    assert fw.crc16(b"123456789") == 0xFEE8


SUBFRAMES = [
    {"kind": "verbatim"},
    {"kind": "fixed", "order": 0},
    {"kind": "fixed", "order": 1, "porder": 2},
    {"kind": "fixed", "order": 2, "method": 1, "porder": 3},
    {"kind": "fixed", "order": 3, "porder": 1, "escape_parts": (1,)},
    {"kind": "fixed", "order": 4},
    {"kind": "lpc", "order": 1, "prec": 5},
    {"kind": "lpc", "order": 8, "porder": 4, "escape_parts": (0, 5)},
    {"kind": "lpc", "order": 12, "prec": 15, "method": 1},
    {"kind": "lpc", "order": 32, "prec": 14, "porder": 2},
]


@pytest.mark.parametrize("bps", [8, 12, 16, 20, 24])
def test_subframe_kinds_roundtrip(bps):
    rng = np.random.default_rng(bps)
    frames, ref = [], []
    for i, kw in enumerate(SUBFRAMES):
        x = _signal(rng, 1024, bps, "noise" if i % 3 == 0 else "smooth")
        frames.append(fw.frame([x], bps, 48000, i, kinds=[kw]))
        ref.append(x)
    data = fw.stream(frames, 48000, 1, bps, 1024 * len(frames), 1024)
    q, ch, sr = _raw(data)
    assert ch == 1 and sr == 48000
    np.testing.assert_array_equal(q[:, 0], np.concatenate(ref))


def test_constant_and_wasted_bits():
    rng = np.random.default_rng(3)
    a = np.full(576, -1234, np.int64)
    b = _signal(rng, 576, 16) & ~np.int64(7)     # 3 wasted bits
    c = (_signal(rng, 576, 16) >> 4) << 4        # 4 wasted bits, LPC
    frames = [fw.frame([a], 16, 44100, 0, kinds=[{"kind": "constant"}]),
              fw.frame([b], 16, 44100, 1, kinds=[{"kind": "fixed", "order": 2, "wasted": 3}]),
              fw.frame([c], 16, 44100, 2, kinds=[{"kind": "lpc", "order": 6, "wasted": 4}]),
              fw.frame([a * 0 + 8], 16, 44100, 3, kinds=[{"kind": "constant", "wasted": 3}])]
    q, _, sr = _raw(fw.stream(frames, 44100, 1, 16, 576 * 4, 576))
    assert sr == 44100
    np.testing.assert_array_equal(q[:, 0], np.concatenate([a, b, c, a * 0 + 8]))


@pytest.mark.parametrize("stereo", ["indep", "left_side", "side_right", "mid_side"])
@pytest.mark.parametrize("bps", [16, 24, 32])
def test_stereo_decorrelation(stereo, bps):
    rng = np.random.default_rng(bps)
    n = 4096
    l = _signal(rng, n, bps)
    r = np.clip(l // 2 + _signal(rng, n, bps) // 4, -(1 << (bps - 1)), (1 << (bps - 1)) - 1)
    method = 1 if bps == 32 else 0  # 32-bit residuals need 5-bit Rice parameters
    kinds = [{"kind": "fixed", "order": 2, "method": method, "porder": 3},
             {"kind": "lpc", "order": 4, "method": method, "porder": 2}]
    frames = [fw.frame([l[:2048], r[:2048]], bps, 96000, 0, stereo, kinds),
              fw.frame([l[2048:], r[2048:]], bps, 96000, 1, stereo,
                       [{"kind": "verbatim"}, {"kind": "fixed", "order": 1, "method": method}])]
    q, ch, _ = _raw(fw.stream(frames, 96000, 2, bps, n, 2048))
    assert ch == 2
    np.testing.assert_array_equal(q, np.stack([l, r], 1))


def test_header_codes_variable_blocks_many_channels():
    rng = np.random.default_rng(11)
    sizes = [1, 17, 192, 256, 300, 576, 4608, 65536 - 1]
    modes = ["table", "khz", "dahz", "hz", "streaminfo"]
    frames, ref, pos = [], [], 0
    for i, bsz in enumerate(sizes):
        chans = [_signal(rng, bsz, 12) for _ in range(6)]
        kinds = [{"kind": "verbatim"} if bsz < 8 else {"kind": "fixed", "order": c % 5} for c in range(6)]
        frames.append(fw.frame(chans, 12, 32000, pos, kinds=kinds, sr_mode=modes[i % 5],
                               bps_mode="table" if i % 2 else "streaminfo",
                               bs_mode="16" if i == 2 else "table", variable=True))
        ref.append(np.stack(chans, 1))
        pos += bsz
    q, ch, sr = _raw(fw.stream(frames, 32000, 6, 12, pos, 65535))
    assert ch == 6 and sr == 32000
    np.testing.assert_array_equal(q, np.concatenate(ref))


def test_unknown_length_trailing_tag_and_id3():
    rng = np.random.default_rng(5)
    x = _signal(rng, 3000, 16)
    frames = [fw.frame([x[:1500]], 16, 48000, 0), fw.frame([x[1500:]], 16, 48000, 1)]
    id3 = b"ID3\x04\x00\x00\x00\x00\x00\x05" + b"\x00" * 5
    data = fw.stream(frames, 48000, 1, 16, 0, 1500, extra_blocks=[(4, b"\x00" * 12)], id3=id3)
    data += b"TAG" + b"\x00" * 125  # ID3v1 after the last frame
    q, _, _ = _raw(data)
    np.testing.assert_array_equal(q[:, 0], x)


def test_damage_is_an_error():
    rng = np.random.default_rng(6)
    x = _signal(rng, 1024, 16)
    good = fw.stream([fw.frame([x], 16, 48000, 0)], 48000, 1, 16, 1024, 1024)
    q, _, _ = _raw(good)
    np.testing.assert_array_equal(q[:, 0], x)
    frame_at = len(good) - len(fw.frame([x], 16, 48000, 0))
    for off, what in [(frame_at + 3, "header CRC"), (len(good) - 40, "frame CRC")]:
        bad = bytearray(good)
        bad[off] ^= 0x10
        with pytest.raises(AAError, match="CRC"):
            _raw(bytes(bad))
    with pytest.raises(AAError):
        _raw(good[:-300])   # truncated: fewer samples than STREAMINFO states
    with pytest.raises(AAError, match="not a FLAC"):
        _raw(b"RIFF" + good[4:])


def _wav(path, ints, channels, bits, sr):
    if bits == 16:
        payload = ints.astype("<i2").tobytes()
    else:  # 24-bit
        v = ints.astype(np.int64) & 0xFFFFFF
        payload = np.stack([v & 0xFF, (v >> 8) & 0xFF, v >> 16], 1).astype(np.uint8).tobytes()
    fmt = struct.pack("<HHIIHH", 1, channels, sr, sr * channels * bits // 8, channels * bits // 8, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(payload)) + payload
    path.write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)


@pytest.mark.parametrize("bits,channels", [(16, 1), (16, 2), (24, 2), (8, 1)])
def test_flac_file_decodes_like_wav(tmp_path, bits, channels):
    """audio.decode: the FLAC's samples reach the pipeline exactly as the WAV
    of the same integers does (ffmpeg's s16 conversion, /32768, channel mean)."""
    rng = np.random.default_rng(bits + channels)
    n = 9000
    chans = [_signal(rng, n, bits) for _ in range(channels)]
    stereo = "mid_side" if channels == 2 else "indep"
    frames = [fw.frame([c[i:i + 4500] for c in chans], bits, 22050, i // 4500, stereo,
                       [{"kind": "lpc", "order": 8, "porder": 2}] * channels) for i in range(0, n, 4500)]
    (tmp_path / "a.flac").write_bytes(fw.stream(frames, 22050, channels, bits, n, 4500))
    x, sr = audio.decode(str(tmp_path / "a.flac"))
    assert sr == 22050 and x.dtype == np.float32 and x.shape == (n,)
    ints = np.stack(chans, 1).reshape(-1)
    if bits == 8:  # 8-bit WAV is unsigned; FLAC's s8 goes to s16 by << 8
        s16 = ints << 8
        ref = s16.reshape(-1, channels).astype(np.float32) / np.float32(32768)
        np.testing.assert_array_equal(x, ref.mean(axis=1, dtype=np.float32))
        return
    _wav(tmp_path / "a.wav", ints, channels, bits, 22050)
    y, sr2 = audio.decode(str(tmp_path / "a.wav"))
    assert sr2 == 22050
    np.testing.assert_array_equal(x, y)
