// Rational polyphase resampling to the 48 kHz the reference analyses at.
//
// load_recording (reference src/identify_tracks.py:49-62) resamples any other
// rate with librosa.resample(res_type="soxr_hq"): libsoxr's high-quality
// recipe -- linear phase, 20-bit precision (stop band >= 126 dB down), pass
// band flat to 0.913 and stop band from 1.0 of the lower rate's Nyquist.
// libsoxr is not in this image; aa_amd/resample.py designs a filter to that
// published specification (Kaiser-windowed sinc on the L-times upsampled
// grid) and this kernel applies it.  Output sample m sits at time m / fs_out,
// i.e. grid index m M; with the filter's centre tap at half:
//   q = m M + half,  k0 = floor(q / L),  r = q - k0 L,
//   y[m] = sum_t bank[r][t] x[k0 - t]     (bank[r][t] = h[r + t L], x = 0 outside)
// One thread per output sample; the L x taps bank and the input window a
// block needs are served from L1/L2 (the kernel is FMA-bound: ~190 taps per
// output at 44.1 -> 48 kHz).
#include "aa_common.h"

namespace aa {

__global__ __launch_bounds__(256) void resample_poly(const float* __restrict__ x, long long n_in,
                                                     const float* __restrict__ bank, int L, int M, int taps,
                                                     int half, float* __restrict__ y, long long n_out) {
    const long long m = (long long)blockIdx.x * 256 + threadIdx.x;
    if (m >= n_out) return;
    const long long q = m * M + half;
    const long long k0 = q / L;
    const int r = (int)(q - k0 * L);
    const float* h = bank + (size_t)r * taps;
    float acc = 0.f;
    if (k0 - (taps - 1) >= 0 && k0 < n_in) {  // interior: no bounds checks
        const float* xp = x + k0;
        for (int t = 0; t < taps; ++t) acc = fmaf(h[t], xp[-t], acc);
    } else {
        for (int t = 0; t < taps; ++t) {
            const long long k = k0 - t;
            if (k >= 0 && k < n_in) acc = fmaf(h[t], x[k], acc);
        }
    }
    y[m] = acc;
}

}  // namespace aa

extern "C" int aa_resample_poly(const float* x, int64_t n_in, const float* bank, int32_t L, int32_t M, int32_t taps,
                                int32_t half, float* y, int64_t n_out, void* stream) {
    AA_CHECK(x && bank && y, AA_ERR_INVALID, "aa_resample_poly: null argument");
    AA_CHECK(n_in >= 0 && n_out >= 0 && L >= 1 && M >= 1 && taps >= 1 && half >= 0 && half < (int64_t)L * taps,
             AA_ERR_INVALID, "aa_resample_poly: bad sizes");
    if (n_out == 0) return AA_OK;
    hipLaunchKernelGGL(aa::resample_poly, dim3((unsigned)((n_out + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), x, (long long)n_in, bank, L, M, taps, half, y,
                       (long long)n_out);
    AA_LAUNCH_CHECK();
    return AA_OK;
}
