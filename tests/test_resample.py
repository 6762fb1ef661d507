"""Resampling to 48 kHz (load_recording's librosa.resample(res_type="soxr_hq"),
src/identify_tracks.py:49-62), host side: the filter aa_amd.resample designs
against libsoxr's published HQ specification, and the float64 oracle
(oracle/resample_oracle.py) pinned by known answers.  Parity with libsoxr's
own samples is unpinned (libsoxr absent)."""
import numpy as np
import pytest

from aa_amd import resample as rs
from oracle import resample_oracle as ro

RATES = [44100, 32000, 22050, 16000, 8000, 96000, 88200, 24000]


@pytest.mark.parametrize("sr", RATES)
def test_output_length_is_librosa_fix_length(sr):
    for n in (0, 1, 2, 147, 160, 44099, 44100, 44101, 2646001):
        want = int(np.ceil(n * 48000 / sr))
        assert rs.out_length(n, sr, 48000) == want == ro.out_length(n, sr, 48000)


@pytest.mark.parametrize("sr", [44100, 32000, 16000, 96000])
def test_design_meets_the_hq_spec(sr):
    """Frequency response of the designed filter (upsampled grid, /L): flat to
    within 1e-4 dB up to 0.913 of the lower Nyquist, at least 120 dB down from
    1.0 of it, linear phase (symmetric taps)."""
    L, M, half, taps, bank = rs.design(sr, 48000)
    h = np.zeros(L * taps)
    for r in range(L):
        h[r::L] = bank[r]
    n = 2 * half + 1
    h = h[:n].astype(np.float64)
    assert np.allclose(h, h[::-1], atol=1e-12)  # linear phase
    fg = L * sr
    nyq = min(sr, 48000) / 2
    nfft = 1 << int(np.ceil(np.log2(n * 8)))
    H = np.abs(np.fft.rfft(h, nfft)) / L
    f = np.fft.rfftfreq(nfft, 1.0 / fg)
    pb = f <= rs.PASSBAND_END * nyq
    sb = f >= rs.STOPBAND_BEGIN * nyq
    assert np.max(np.abs(20 * np.log10(H[pb]))) < 1e-4
    assert 20 * np.log10(H[sb].max()) < -120


def test_attenuation_is_21_bits():
    assert abs(rs.ATTENUATION_DB - 126.43) < 0.01
    assert rs.PASSBAND_END == ro.PASSBAND_END and rs.STOPBAND_BEGIN == ro.STOPBAND_BEGIN


@pytest.mark.parametrize("sr", [44100, 32000, 16000, 96000])
def test_oracle_known_answers(sr):
    """DC stays DC, a 1 kHz tone is the same tone at 48 kHz (away from the
    zero-padded ends), a tone above the lower Nyquist vanishes when
    downsampling."""
    n = int(0.25 * sr)
    y = ro.resample(np.full(n, 0.5), sr, 48000)
    assert len(y) == ro.out_length(n, sr, 48000)
    mid = slice(len(y) // 4, 3 * len(y) // 4)
    assert np.max(np.abs(y[mid] - 0.5)) < 1e-6
    t = np.arange(n) / sr
    y = ro.resample(np.sin(2 * np.pi * 1000 * t), sr, 48000)
    tm = np.arange(len(y)) / 48000
    assert np.max(np.abs(y[mid] - np.sin(2 * np.pi * 1000 * tm[mid]))) < 1e-6
    if sr > 48000:
        y = ro.resample(np.sin(2 * np.pi * 30000 * t), sr, 48000)
        assert np.sqrt(np.mean(y[mid] ** 2)) < 10 ** (-118 / 20)


def test_host_design_matches_oracle_filter():
    """aa_amd.resample's bank and the oracle's firwin design are the same
    Kaiser filter up to firwin's DC normalisation (< 1e-6 relative)."""
    for sr in (44100, 16000):
        L, M, half, taps, bank = rs.design(sr, 48000)
        h, L2, M2 = ro.design(sr, 48000)
        assert (L, M) == (L2, M2) and len(h) == 2 * half + 1
        hb = np.zeros(L * taps)
        for r in range(L):
            hb[r::L] = bank[r]
        assert np.max(np.abs(hb[:len(h)] - h)) < 1e-6 * np.abs(h).max()
