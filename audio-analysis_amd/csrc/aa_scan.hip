// Span scans over the PCM buffer, and the PCM16 -> f32 conversion of a batch
// of recordings.
//
// aa_span_nonzero backs get_end (reference src/identify_tracks.py:387-413):
// a 170-frame chunk of the 4800/281 STFT has a constant 120-band mel block
// exactly when every sample its frames see is zero, so the GPU reports, per
// sample span, whether any sample in it is nonzero (HBM-bound byte scan).
#include "aa_common.h"

namespace aa {

__global__ __launch_bounds__(256) void span_nonzero(const float* __restrict__ pcm,
                                                    const long long* __restrict__ spans,
                                                    int* __restrict__ flags) {
    const long long b = spans[2 * blockIdx.x], e = spans[2 * blockIdx.x + 1];
    int any = 0;
    // 16-byte body with scalar head/tail; the body starts at the first
    // 16-B-aligned ADDRESS (pcm may be an unaligned view)
    const long long mis = (long long)((reinterpret_cast<uintptr_t>(pcm) >> 2) & 3);  // pcm's float offset mod 4
    long long a4 = ((b + mis + 3) & ~3LL) - mis, e4 = ((e + mis) & ~3LL) - mis;
    if (a4 > e4) a4 = e4 = e;
    for (long long i = b + threadIdx.x; i < a4; i += 256) any |= pcm[i] != 0.f;
    const float4* q = reinterpret_cast<const float4*>(pcm + a4);
    const long long n4 = (e4 - a4) / 4;
    for (long long i = threadIdx.x; i < n4; i += 256) {
        const float4 v = q[i];
        any |= (v.x != 0.f) | (v.y != 0.f) | (v.z != 0.f) | (v.w != 0.f);
    }
    for (long long i = e4 + threadIdx.x; i < e; i += 256) any |= pcm[i] != 0.f;
    any = __syncthreads_or(any);
    if (threadIdx.x == 0) flags[blockIdx.x] = any;
}

// ffmpeg's s16 samples -> librosa's buf_to_float (x / 32768, exact) and
// load_recording's channel mean (numpy float32 sum in channel order, then one
// correctly rounded division; the sum of <= 8 multiples of 2^-15 is exact).
// One thread per output frame, 16-B stores of 4 frames where aligned.
__global__ __launch_bounds__(256) void pcm_s16_to_f32(const short* __restrict__ in, long long n_frames, int ch,
                                                      float* __restrict__ out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_frames) return;
    const short* q = in + i * ch;
    float s = (float)q[0] * (1.f / 32768.f);
    for (int c = 1; c < ch; ++c) s = __fadd_rn(s, (float)q[c] * (1.f / 32768.f));
    out[i] = ch == 1 ? s : __fdiv_rn(s, (float)ch);
}

}  // namespace aa

extern "C" int aa_pcm_s16_to_f32(const int16_t* in, int64_t n_frames, int32_t channels, float* out, void* stream) {
    AA_CHECK(in && out, AA_ERR_INVALID, "aa_pcm_s16_to_f32: null argument");
    AA_CHECK(n_frames >= 0 && channels >= 1 && channels <= 8, AA_ERR_INVALID, "aa_pcm_s16_to_f32: bad sizes");
    if (n_frames == 0) return AA_OK;
    hipLaunchKernelGGL(aa::pcm_s16_to_f32, dim3((unsigned)((n_frames + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), reinterpret_cast<const short*>(in), (long long)n_frames,
                       channels, out);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

extern "C" int aa_span_nonzero(const float* pcm, int64_t n, const int64_t* spans, int32_t n_spans,
                               int32_t* flags, void* stream) {
    AA_CHECK(pcm && spans && flags, AA_ERR_INVALID, "aa_span_nonzero: null argument");
    AA_CHECK(n_spans >= 0 && n >= 0, AA_ERR_INVALID, "aa_span_nonzero: bad sizes");
    if (n_spans == 0) return AA_OK;
    hipLaunchKernelGGL(aa::span_nonzero, dim3(n_spans), dim3(256), 0, static_cast<hipStream_t>(stream), pcm,
                       reinterpret_cast<const long long*>(spans), flags);
    AA_LAUNCH_CHECK();
    return AA_OK;
}
