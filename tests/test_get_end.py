"""get_end (reference src/identify_tracks.py:387-413) against its CPU
restatement (oracle/get_end_oracle.py: 4800-point STFT, hop 281, 120-band
mel at power 1, amax == amin per 170-frame chunk).

The build replaces the mel scan by a span scan (aa_amd.gpu_ops): a chunk's
mel block is constant exactly when every sample its frames cover is zero.
The CPU tests check that equivalence -- the spans of gpu_ops.get_end_spans
scanned with numpy -- on trailing silence, mid-clip gaps, DC stretches,
int16-LSB noise and lengths at chunk boundaries; the GPU tests run the
aa_span_nonzero kernel on the same cases.
"""
import numpy as np
import pytest

from oracle import get_end_oracle

SR = 48000
HOP = 281
CHUNK = SR // HOP  # 170 frames


def _noise(n, seed, amp=0.1):
    rng = np.random.default_rng(seed)
    x = np.round(rng.standard_normal(n) * amp * 32768) / 32768  # int16-quantised
    x[x == 0] = 1 / 32768
    return x.astype(np.float32)


def _cases():
    c = {}
    c["noise_5s"] = _noise(5 * SR, 1)
    x = _noise(12 * SR, 2)
    x[7 * SR:] = 0
    c["trailing_zeros"] = x
    x = _noise(12 * SR, 3)
    x[3 * SR:6 * SR] = 0  # a gap longer than a chunk plus its frames' reach
    c["mid_gap"] = x
    x = _noise(12 * SR, 4)
    x[4 * SR:4 * SR + SR // 2] = 0  # a gap shorter than a chunk: no end found there
    c["short_gap"] = x
    x = _noise(10 * SR, 5)
    x[5 * SR:] = 0.25  # DC stretch to the end
    c["dc_tail"] = x
    x = _noise(10 * SR, 6)
    x[3 * SR:8 * SR] = -1 / 32768  # one int16 LSB of DC
    c["lsb_dc"] = x
    c["lsb_noise"] = _noise(6 * SR, 7, amp=1 / 32768)
    # lengths that put the frame count at / around chunk multiples
    for k, extra in ((3, 0), (3, 1), (3, -1), (4, HOP)):
        n = (k * CHUNK - 1) * HOP + extra
        x = _noise(n, 10 + k)
        x[n // 2:] = 0
        c[f"len_{k}chunks_{extra:+d}"] = x
    c["all_zero_2s"] = np.zeros(2 * SR, np.float32)
    c["short_0.5s"] = _noise(SR // 2, 8)
    return c


CASES = _cases()


def _span_get_end(frames, sr):
    """gpu_ops.get_end with the kernel emulated by numpy (any nonzero sample)."""
    from aa_amd.gpu_ops import get_end_spans
    spans, starts, hop = get_end_spans(len(frames), sr)
    for (a, b), s in zip(spans, starts):
        if not np.any(frames[a:b] != 0):
            return s * hop // sr
    return len(frames) / sr


@pytest.mark.parametrize("name", sorted(CASES))
def test_span_scan_matches_mel_scan(name):
    x = CASES[name]
    ref = get_end_oracle.get_end(x, SR)
    got = _span_get_end(x, SR)
    assert got == ref, (name, got, ref)
    assert type(got) is type(ref)


def test_oracle_finds_trailing_silence():
    """Sanity of the restatement itself: the first all-silent chunk ends it."""
    x = CASES["trailing_zeros"]
    end = get_end_oracle.get_end(x, SR)
    assert isinstance(end, int) and 6 <= end <= 7


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_get_end(gpu, name):
    from aa_amd import gpu_ops
    x = CASES[name]
    assert gpu_ops.get_end(x, SR, device=gpu) == get_end_oracle.get_end(x, SR)


@pytest.mark.gpu
def test_gpu_get_end_unaligned_view(gpu):
    """Spans starting at any sample offset of a device view (16-B alignment
    of the float4 body is taken from the address, not the index)."""
    import torch
    from aa_amd import gpu_ops
    x = CASES["trailing_zeros"]
    big = torch.zeros(len(x) + 3, dtype=torch.float32, device=gpu)
    for off in range(4):
        big.zero_()
        big[off:off + len(x)] = torch.from_numpy(x).to(gpu)
        view = big[off:off + len(x)]
        assert gpu_ops.get_end(x, SR, device=gpu, pcm_dev=view) == get_end_oracle.get_end(x, SR)
