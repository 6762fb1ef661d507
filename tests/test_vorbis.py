"""Ogg Vorbis decode (aa_vorbis_* in libaa.so, host code) for load_recording
(src/identify_tracks.py:49-62, which decodes through ffmpeg).

Every stream here is written by the test encoder tests/vorbis_writer.py, which
restates the Vorbis I specification's encoder side for the decoder's features:
floor 0 / floor 1, residues 0 / 1 / 2, coupling, submaps, short / long block
transitions, ordered / sparse / lookup-1 / lookup-2 / sequence_p codebooks, Ogg
lacing across pages, several packets per page, granule trims, a second logical
stream, a damaged page.  Checks:
- the library's samples equal the CPU restatement's (oracle/vorbis_oracle.py,
  O(N^2) inverse MDCT) to float rounding;
- decoding reconstructs the encoded signal (a round trip through the forward
  MDCT: SNR bounds that a wrong window, transform, floor or residue rule
  would miss by tens of dB);
- load_recording gives the oracle's samples after ffmpeg's float -> s16
  conversion, /32768 and the channel mean.
PARITY UNPINNED against ffmpeg/libvorbis (neither is in the image)."""
import ctypes as C

import numpy as np
import pytest

import vorbis_writer as vw
from aa_amd import audio
from aa_amd._lib import AAError, VorbisInfo, check, lib
from oracle import vorbis_oracle as vo

SR = 48000


def _lib_decode(data):
    buf = np.frombuffer(data, np.uint8)
    info = VorbisInfo()
    check(lib().aa_vorbis_info(buf.ctypes.data, buf.size, C.byref(info)), "info")
    n = C.c_int64()
    check(lib().aa_vorbis_decode(buf.ctypes.data, buf.size, None, 0, C.byref(n)), "count")
    out = np.empty(max(n.value, 1) * info.channels, np.float32)
    check(lib().aa_vorbis_decode(buf.ctypes.data, buf.size, out.ctypes.data, n.value, C.byref(n)), "decode")
    return out[: n.value * info.channels].reshape(-1, info.channels), info


def _signal(seconds=0.2, channels=1, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(int(seconds * SR)) / SR
    out = []
    for c in range(channels):
        f = rng.uniform(200, 6000, 3)
        x = sum(a * np.sin(2 * np.pi * fi * t + rng.uniform(0, 6)) for a, fi in zip((0.3, 0.15, 0.05), f))
        x *= np.minimum(1.0, t / 0.02)  # onset
        out.append(x + rng.normal(0, 0.002, len(t)))
    return np.stack(out, 1)


def _snr(x, y):
    n = min(len(x), len(y))
    e = y[:n] - x[:n]
    return 10 * np.log10((x[:n] ** 2).sum() / max((e ** 2).sum(), 1e-30))


STREAMS = {
    "mono_res1": dict(channels=1, kw=dict(schedule=[1, 1, 0, 0, 0, 1], residue_type=1)),
    "mono_res0_floor0_short": dict(channels=1, kw=dict(schedule=[1, 0, 0, 1, 1, 0], residue_type=0,
                                                      floor0_short=True)),
    "stereo_coupled_res2": dict(channels=2, kw=dict(schedule=[1, 0, 1, 1, 0, 0], residue_type=2)),
    "stereo_submaps_res1_res0": dict(channels=2, kw=dict(schedule=[0, 1, 1], residue_type=1, submaps=True,
                                                         coupling=False)),
    "stereo_coupled_submaps": dict(channels=2, kw=dict(schedule=[1, 1, 0], residue_type=1, submaps=True)),
}


@pytest.fixture(scope="module")
def streams():
    out = {}
    for name, s in STREAMS.items():
        x = _signal(channels=s["channels"], seed=len(name))
        out[name] = (x, vw.encode(x, sr=SR, **s["kw"]))
    return out


@pytest.mark.parametrize("name", list(STREAMS))
def test_library_matches_oracle(streams, name):
    x, data = streams[name]
    y, info = _lib_decode(data)
    ref, sr = vo.decode(data)
    assert info.sample_rate == sr == SR and info.channels == x.shape[1]
    assert info.total_frames == len(x) and y.shape == ref.shape == x.shape
    np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)


@pytest.mark.parametrize("name", list(STREAMS))
def test_round_trip_reconstructs_signal(streams, name):
    x, data = streams[name]
    y, _ = _lib_decode(data)
    for c in range(x.shape[1]):
        # an order-4 LSP curve follows the spectrum coarsely (more quantisation noise)
        assert _snr(x[:, c], y[:, c]) > (12 if "floor0" in name else 25), (name, c)


def test_imdct_matches_definition():
    """The library's FFT inverse MDCT against the O(N^2) definition: a single
    long block of a known spectrum, window flat in the middle -- checked
    through the round trip of an impulse train at every block size."""
    for bs in ((64, 128), (128, 512), (256, 2048), (512, 4096)):
        x = np.zeros((3 * bs[1], 1))
        x[::97, 0] = 0.5
        data = vw.encode(x, sr=SR, bs=bs, schedule=[1, 0, 1])
        y, _ = _lib_decode(data)
        ref, _ = vo.decode(data)
        np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)
        assert _snr(x[:, 0], y[:, 0]) > 15, bs


def test_ogg_paging_does_not_change_samples(streams):
    x, base = streams["stereo_coupled_res2"]
    y0, _ = _lib_decode(base)
    kw = STREAMS["stereo_coupled_res2"]["kw"]
    for extra in (dict(max_segs=3), dict(per_page=4), dict(per_page=3, max_segs=2), dict(extra_stream=True)):
        d = vw.encode(x, sr=SR, **kw, **extra)
        assert d != base
        y, _ = _lib_decode(d)
        np.testing.assert_array_equal(y, y0)


def test_granule_start_trim():
    x = _signal(0.15)
    data = vw.encode(x, sr=SR, schedule=[1, 0], start_trim=300)
    y, info = _lib_decode(data)
    ref, _ = vo.decode(data)
    assert len(y) == len(x) == info.total_frames
    np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)
    assert _snr(x[:, 0], y[:, 0]) > 25


def test_silent_blocks_unused_floors():
    x = _signal(0.2, channels=2)
    data = vw.encode(x, sr=SR, schedule=[1], residue_type=2, silent={2, 3})
    y, _ = _lib_decode(data)
    ref, _ = vo.decode(data)
    np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)
    # blocks 2 and 3 carry unused floors (zero spectra): output samples
    # [1024 k - 1024, 1024 k) come from blocks k-1 and k (long blocks, centre
    # of block 0 at sample 0), so [1024 * 2, 1024 * 3) is silent
    assert np.abs(y[2048:3072]).max() == 0.0
    assert np.abs(y[1024:2048]).max() > 0.0 and np.abs(y[3072:4096]).max() > 0.0


def test_damaged_page_is_skipped_like_the_oracle(streams):
    x, data = streams["mono_res1"]
    bad = vw.corrupt_page(data, 4)
    y, _ = _lib_decode(bad)
    ref, _ = vo.decode(bad)
    np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)
    assert len(y) <= len(x)


def test_bad_headers_are_errors():
    x = _signal(0.05)
    data = vw.encode(x, sr=SR)
    for bad in (data[:60], b"OggS" + b"\0" * 100, data.replace(b"vorbis", b"vorbiz", 1)):
        buf = np.frombuffer(bad, np.uint8)
        with pytest.raises(AAError):
            check(lib().aa_vorbis_info(buf.ctypes.data, buf.size, C.byref(VorbisInfo())), "info")


def test_fuzzed_streams_never_crash(streams):
    """Random byte damage to audio pages (CRCs re-stamped so the pages are
    accepted): the decoder returns samples or an error, never faults, and
    agrees with the oracle whenever both decode."""
    x, data = streams["stereo_coupled_res2"]
    rng = np.random.default_rng(7)
    pages, pos = [], 0
    while True:
        try:
            q = data.index(b"OggS", pos + 1)
        except ValueError:
            pages.append(data[pos:])
            break
        pages.append(data[pos:q])
        pos = q
    for trial in range(12):
        pg = [bytearray(p) for p in pages]
        k = int(rng.integers(3, len(pg)))
        body0 = 27 + pg[k][26]
        for _ in range(4):
            i = int(rng.integers(body0, len(pg[k])))
            pg[k][i] = int(rng.integers(0, 256))
        import struct
        pg[k][22:26] = b"\0\0\0\0"
        pg[k][22:26] = struct.pack("<I", vo.ogg_crc(bytes(pg[k])))
        d = b"".join(bytes(p) for p in pg)
        try:
            y, _ = _lib_decode(d)
        except AAError:
            continue
        ref, _ = vo.decode(d)
        assert y.shape == ref.shape
        np.testing.assert_allclose(y, ref, rtol=0, atol=1e-4 * max(1.0, float(np.abs(ref).max())))


@pytest.mark.parametrize("channels", [1, 2])
def test_load_recording_ogg_is_ffmpeg_s16_of_the_decode(tmp_path, channels):
    from aa_amd.identify_tracks import load_recording
    x = _signal(0.25, channels=channels, seed=3)
    p = tmp_path / "rec.ogg"
    p.write_bytes(vw.encode(x, sr=SR, schedule=[1, 1, 0, 0, 1], residue_type=2 if channels == 2 else 1))
    frames, sr = load_recording(p)
    assert sr == SR and frames.dtype == np.float32
    ref, _ = vo.decode(p.read_bytes())
    q = np.clip(np.rint(ref.astype(np.float64) * 32768), -32768, 32767).astype(np.float32) / np.float32(32768)
    want = q.mean(axis=1, dtype=np.float32) if channels > 1 else q[:, 0]
    # the library's float samples and the oracle's differ by float rounding, so
    # an s16 rounding may flip on a .5 boundary
    assert frames.shape == want.shape
    assert np.abs(frames - want).max() <= 1.0 / 32768 + 1e-9
    assert (frames != want).mean() < 1e-3


def test_load_recording_rejects_damage_the_reference_way(tmp_path):
    from aa_amd.identify_tracks import load_recording
    p = tmp_path / "bad.ogg"
    p.write_bytes(b"OggS" + b"\x00" * 200)
    with pytest.raises(Exception, match=f"Could not load {p}"):
        load_recording(p)
