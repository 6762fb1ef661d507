"""CPU restatement of load_recording's resampling step (TEST INFRASTRUCTURE
ONLY -- tests/ are the only importers; the product path never imports this).

Reference: src/identify_tracks.py:49-62 resamples every non-48 kHz recording
with librosa 0.11's ``librosa.resample(..., res_type="soxr_hq")`` [ext: librosa
~=0.11.0, requirements.txt:1; python-soxr / libsoxr 0.1.3, neither in this
image nor under /root/reference] and ``fix_length``s it to ceil(n x ratio).
libsoxr's HQ recipe is published as: linear phase, 20-bit precision
(rejection (20 + 1) x 6.02 = 126.4 dB), pass band to 0.913 and stop band from
1.0 of the lower rate's Nyquist.  This oracle restates that specification
independently of aa_amd/resample.py: scipy.signal.firwin's Kaiser-window
design (DC gain normalised to exactly 1 per output sample) and scipy's
polyphase ``upfirdn``, in float64, with the same time alignment (output m at
input time m / fs_out, zero samples outside the recording).

**Parity with libsoxr's actual samples is unpinned** (no libsoxr here, and the
reference holds no resampled fixture); what is pinned is the specification:
pass-band flatness, stop-band rejection, DC and tone reconstruction, output
length -- tests/test_resample.py and tests/test_gpu_resample.py.
"""
from __future__ import annotations

from math import ceil, gcd, log10

import numpy as np

PASSBAND_END = 0.913
STOPBAND_BEGIN = 1.0
ATTENUATION_DB = 21 * 20 * log10(2.0)


def out_length(n_in, sr_in, sr_out):
    """librosa.resample(fix=True): ceil(n * target / orig)."""
    return int(ceil(n_in * float(sr_out) / sr_in))


def filter_spec(sr_in, sr_out):
    """(L, M, numtaps, cutoff Hz, beta, grid rate Hz) from the published HQ spec."""
    g = gcd(int(sr_in), int(sr_out))
    L, M = sr_out // g, sr_in // g
    nyq = min(sr_in, sr_out) / 2.0
    fg = float(L) * sr_in
    width = (STOPBAND_BEGIN - PASSBAND_END) * nyq
    A = ATTENUATION_DB
    numtaps = int(ceil((A - 7.95) / (2.285 * 2 * np.pi * width / fg))) + 1
    numtaps |= 1
    beta = 0.1102 * (A - 8.7)
    cutoff = 0.5 * (PASSBAND_END + STOPBAND_BEGIN) * nyq
    return L, M, numtaps, cutoff, beta, fg


def design(sr_in, sr_out):
    """Float64 low-pass on the L-times upsampled grid, gain L (firwin: unit DC gain, x L)."""
    from scipy.signal import firwin
    L, M, numtaps, cutoff, beta, fg = filter_spec(sr_in, sr_out)
    return L * firwin(numtaps, cutoff, window=("kaiser", beta), fs=fg), L, M


def resample(x, sr_in, sr_out):
    """float64 y[m] = sum_k x[k] h(m M - k L) with h centred at 0."""
    from scipy.signal import upfirdn
    x = np.asarray(x, np.float64)
    if sr_in == sr_out:
        return x.copy()
    h, L, M = design(sr_in, sr_out)
    half = (len(h) - 1) // 2
    s = (-half) % M  # pad h so that the centre lands on the decimation grid
    hp = np.concatenate([np.zeros(s), h])
    full = upfirdn(hp, x, up=L, down=M)
    d = (half + s) // M
    n_out = out_length(len(x), sr_in, sr_out)
    y = np.zeros(n_out)
    seg = full[d:d + n_out]
    y[:len(seg)] = seg
    return y
