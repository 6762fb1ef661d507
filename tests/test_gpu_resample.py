"""aa_resample_poly (csrc/aa_resample.hip) against the float64 oracle restating
libsoxr's HQ specification (oracle/resample_oracle.py), and load_recording's
use of it (src/identify_tracks.py:49-62).  f32 accumulation over ~190 taps:
max |delta| <= 1e-5 on full-scale noise.  Parity with libsoxr's samples is
unpinned (libsoxr absent)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.mark.parametrize("sr", [44100, 32000, 22050, 16000, 8000, 96000, 88200])
def test_gpu_resample_matches_oracle(gpu, sr):
    from aa_amd.resample import resample
    from oracle import resample_oracle as ro
    rng = np.random.default_rng(sr)
    x = np.clip(rng.standard_normal(int(0.3 * sr)) * 0.3, -1, 1).astype(np.float32)
    y = resample(x, sr, 48000)
    ref = ro.resample(x.astype(np.float64), sr, 48000)
    assert y.dtype == np.float32 and len(y) == len(ref) == ro.out_length(len(x), sr, 48000)
    err = np.abs(y - ref).max()
    print(f"{sr} -> 48000: {len(x)} -> {len(y)} samples, max|d| {err:.2e}")
    assert err <= TOL


def test_gpu_resample_edges_and_tiny_inputs(gpu):
    from aa_amd.resample import resample
    from oracle import resample_oracle as ro
    for n in (0, 1, 3, 160, 441):
        x = np.linspace(-0.5, 0.5, n).astype(np.float32)
        y = resample(x, 44100, 48000)
        assert len(y) == ro.out_length(n, 44100, 48000)
        if n:
            assert np.abs(y - ro.resample(x, 44100, 48000)).max() <= TOL


def test_load_recording_resamples_on_gpu(gpu, tmp_path):
    from aa_amd import identify_tracks as it
    from aa_amd.audio import decode
    from oracle import resample_oracle as ro
    from tools import synth
    p = tmp_path / "r.wav"
    synth.write_wav(p, synth.clip(7, seconds=3.0, sr=44100), sr=44100)
    frames, sr = it.load_recording(str(p))
    raw, sr0 = decode(str(p))
    assert sr == 48000 and sr0 == 44100 and len(frames) == 144000
    assert np.abs(frames - ro.resample(raw, 44100, 48000)).max() <= TOL
