// Per-window log-mel front end for gfx950.
//
// Replaces, per analysis window (reference /root/reference):
//   normalize_data                      src/identify_tracks.py:202-209
//   np.abs(librosa.stft(x, n_fft, hop))  src/identify_tracks.py:243
//   custommel.mel_spec (|S|**p, mel_f.)  src/custommel.py:59-63
//   librosa.power_to_db(ref=np.max)     src/identify_tracks.py:266
//   expand_dims / mean_sub / channels   src/identify_tracks.py:267-288
//
// Three launches per batch of windows (all on the caller's stream):
//   fe_stats    min/max/finite partials of every window (HBM stream of the PCM)
//   fe_stft_mel a block owns FPB consecutive frames of one window: the
//               overlapped PCM segment is loaded once (coalesced) and normalised
//               into LDS, each frame is windowed and transformed by an N/2-point
//               complex Stockham FFT (radix 8, LDS ping-pong, table twiddles),
//               split into the N-point real spectrum, |X|**power, and projected
//               on the sparse mel filterbank (CSR rows, contiguous bins).
//   fe_db       per-window max -> power_to_db, clamp, mean_sub, layout/channels.
#include "aa_common.h"
#include "aa_wavefft.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace aa {

constexpr int kStatSplit = 16;  // stats blocks per window
constexpr int kFpb = 6;         // frames per stft block

struct FePlan {
    aa_fe_config cfg;
    int T = 0;         // frames per window
    int kmin = 0;      // first filterbank bin with a nonzero weight
    int kmax = 0;      // last
    int nfblk = 0;     // frame blocks per window
    int nnz = 0;
    float* d_win = nullptr;   // periodic Hann, f32 [n_fft]
    float2* d_tw = nullptr;   // exp(-2 pi i m / Nc), m < Nc
    float2* d_tw2 = nullptr;  // exp(-2 pi i k / n_fft), k <= Nc
    int4* d_rows = nullptr;   // per band: (first bin, count, value offset, 0)
    float* d_vals = nullptr;  // CSR values
    char* d_cimg = nullptr;   // fe_stft_mel_4096 CSR image (rows | values), 1-KiB padded
    int cimg_bytes = 0;
    StageTimer timer;         // HIP events around the launches in timer.mask
};

enum { FE_STAGE_STATS = 0, FE_STAGE_STFT = 1, FE_STAGE_DB = 2, FE_N_STAGES = 3 };

// ---------------------------------------------------------------------------
// fe_stats: min / max / non-finite over each virtual window (zeros outside the
// valid view, exactly like np.pad before normalize_data).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fe_stats(const float* __restrict__ pcm,
                                                const aa_window* __restrict__ wins,
                                                int win_len, float4* __restrict__ stats) {
    const int w = blockIdx.y;
    const aa_window d = wins[w];
    const int chunk = (win_len + kStatSplit - 1) / kStatSplit;
    const int i0 = blockIdx.x * chunk;
    const int i1 = min(win_len, i0 + chunk);
    float mn = INFINITY, mx = -INFINITY;
    int bad = 0;
    // valid part of this chunk, in window coordinates; the rest is np.pad zeros
    const int v0 = max(i0, d.pad_left);
    const int v1 = min(i1, d.pad_left + d.n_valid);
    if (i0 < i1 && !(v0 == i0 && v1 >= i1)) { mn = 0.f; mx = 0.f; }
    if (v0 < v1) {
        const float* p = pcm + d.src + (v0 - d.pad_left);
        const int n = v1 - v0;
        // scalar head up to 16-byte alignment, float4 body, scalar tail
        const int head = min(n, (int)((16 - ((uintptr_t)p & 15)) & 15) / 4);
        for (int i = threadIdx.x; i < head; i += blockDim.x) {
            float x = p[i];
            bad |= !isfinite(x);
            mn = fminf(mn, x);
            mx = fmaxf(mx, x);
        }
        const int nb = (n - head) / 4;
        const float4* q = reinterpret_cast<const float4*>(p + head);
        // four independent loads in flight per thread before any is consumed
        // (past the end a lane re-reads the last float4: min / max / the
        // non-finite flag do not change under duplicates)
        constexpr int U = 4;
        for (int i = threadIdx.x; i < nb; i += U * blockDim.x) {
            float4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = q[min(i + u * (int)blockDim.x, nb - 1)];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                bad |= !isfinite(x[u].x) | !isfinite(x[u].y) | !isfinite(x[u].z) | !isfinite(x[u].w);
                mn = fminf(fminf(mn, x[u].x), fminf(x[u].y, fminf(x[u].z, x[u].w)));
                mx = fmaxf(fmaxf(mx, x[u].x), fmaxf(x[u].y, fmaxf(x[u].z, x[u].w)));
            }
        }
        for (int i = head + nb * 4 + threadIdx.x; i < n; i += blockDim.x) {
            float x = p[i];
            bad |= !isfinite(x);
            mn = fminf(mn, x);
            mx = fmaxf(mx, x);
        }
    }
    __shared__ float smn[4], smx[4];
    __shared__ int sbad[4];
    mn = wave_min(mn);
    mx = wave_max(mx);
    bad = wave_or(bad);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { smn[wv] = mn; smx[wv] = mx; sbad[wv] = bad; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
            mn = fminf(mn, smn[k]);
            mx = fmaxf(mx, smx[k]);
            bad |= sbad[k];
        }
        stats[w * kStatSplit + blockIdx.x] = make_float4(mn, mx, (float)bad, 0.f);
    }
}

// LDS index of complex point i: one float2 of padding per 8 keeps the radix-8
// scatter of pass 1 (stride 8) and the NS = 8 scatter of pass 2 conflict-free.
__device__ __forceinline__ int pidx(int i) { return i + (i >> 3); }

// One Stockham pass of radix R over NC points held in LDS (src -> dst), for
// sub-transform size NS (product of the earlier radices).  Thread handles
// butterflies j = tid + b*NT.  Its twiddles depend only on (j, NS), so they
// are loaded once per block into registers (load) and reused for every frame.
template <int NC, int R, int NT, int NS>
struct Pass {
    static constexpr int NB = NC / R;
    static constexpr int PER = (NB + NT - 1) / NT;
    float2 t[PER][R - 1];
    __device__ __forceinline__ void load(const float2* __restrict__ tw) {
#pragma unroll
        for (int b = 0; b < PER; ++b) {
            const int j = threadIdx.x + b * NT;
            const int k = j % NS;
#pragma unroll
            for (int r = 1; r < R; ++r)  // unconditional loads: all in flight together
                t[b][r - 1] = tw[(r * k * (NC / (NS * R))) & (NC - 1)];
        }
    }
    __device__ __forceinline__ void run(const float2* __restrict__ src, float2* __restrict__ dst) const {
#pragma unroll
        for (int b = 0; b < PER; ++b) {
            const int j = threadIdx.x + b * NT;
            if (NB % NT == 0 || j < NB) {
                float2 v[R];
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = src[pidx(j + r * NB)];
                if constexpr (NS > 1) {
#pragma unroll
                    for (int r = 1; r < R; ++r) v[r] = cmul(v[r], t[b][r - 1]);
                }
                if constexpr (R == 8) dft8(v);
                if constexpr (R == 4) dft4(v[0], v[1], v[2], v[3]);
                if constexpr (R == 2) dft2(v[0], v[1]);
                const int k = j % NS;
                const int o = (j / NS) * NS * R + k;
#pragma unroll
                for (int r = 0; r < R; ++r) dst[pidx(o + r * NS)] = v[r];
            }
        }
    }
};

// ---------------------------------------------------------------------------
// fe_stft_mel
// Transform plan for NC = NFFT/2 complex points with NT = NC/8 threads:
//   pass 1  radix 8, NS = 1   (input read from the windowed PCM segment)
//   pass 2  radix 8, NS = 8
//   pass 3  radix 8, NS = 64
//   pass 4  radix NC/512, NS = 512   (NC = 1024: 2, 2048: 4, 4096: 8)
// ---------------------------------------------------------------------------
// Correctly rounded (x - lo) / scale as three instructions: with
// y = RN(1/scale), q0 = RN(a y) is within an ulp of a/scale, the residual
// a - q0 scale is exact in one fma, and RN(q0 + r y) is the correctly rounded
// quotient (Markstein's theorem; tools/div_check.hip compares it with
// __fdiv_rn on 3.4e10 operand pairs: no mismatch).  Then normalize_data's
// remaining steps in reference order (src/identify_tracks.py:205-208).
__device__ __forceinline__ float normalize_sample(float x, float lo, float scale, float inv) {
    const float a = __fsub_rn(x, lo);
    const float q0 = __fmul_rn(a, inv);
    const float r = fmaf(-q0, scale, a);
    float y = fmaf(r, inv, q0);
    y = __fadd_rn(y, 0.000001f);
    y = __fsub_rn(y, 0.5f);
    return __fmul_rn(y, 2.0f);
}

// complex64 -> np.abs -> ** power.  The power mode is a template parameter:
// a runtime select between the three forms would make every bin pay for the
// inlined powf.  |X|^2 is formed directly (the reference squares a rounded
// hypot: the two differ by an ulp, far inside the f32-FFT tolerance), and the
// other modes use the hardware square root (v_sqrt_f32, 1 ulp) rather than the
// correctly rounded expansion.
enum { PM_GENERAL = 0, PM_ABS = 1, PM_SQUARE = 2 };
template <int PM>
__device__ __forceinline__ float pow_mag(float re, float im, float power) {
    const float m2 = fmaf(re, re, im * im);
    if constexpr (PM == PM_SQUARE) return m2;
    const float mag = __builtin_amdgcn_sqrtf(m2);
    if constexpr (PM == PM_ABS) return mag;
    else return powf(mag, power);
}

template <int NFFT, int PM>
__global__ __launch_bounds__(NFFT / 16) void fe_stft_mel(
    const float* __restrict__ pcm, const aa_window* __restrict__ wins, const float4* __restrict__ stats,
    const float* __restrict__ hann, const float2* __restrict__ tw, const float2* __restrict__ tw2,
    const int4* __restrict__ rows, const float* __restrict__ vals, int nnz, int win_len, int hop, int T,
    int n_mels, int kmin, int kmax, int normalize, float power, int nfblk, int n_items,
    float* __restrict__ melS, float* __restrict__ blkmax) {
    constexpr int NC = NFFT / 2;
    constexpr int NT = NC / 8;
    constexpr int R4 = NC / 512;
    static_assert(NC >= 1024 && NC <= 4096, "NFFT 2048..8192");
    constexpr int KREG = 4;  // post-processing bins per thread with register twiddles
    extern __shared__ float lds[];
    float* seg = lds;
    const int seg_cap = ((kFpb - 1) * hop + NFFT + 3) & ~3;
    float2* bufA = reinterpret_cast<float2*>(lds + seg_cap);
    constexpr int NCP = NC + NC / 8;  // padded buffer length (float2)
    float2* bufB = bufA + NCP;
    float* melT = reinterpret_cast<float*>(bufB + NCP);  // [n_mels][kFpb] staging
    int4* srows = reinterpret_cast<int4*>(melT + ((n_mels * kFpb + 3) & ~3));
    float* svals = reinterpret_cast<float*>(srows + n_mels);

    // --- per-thread constants, loaded once per block ---
    const int tid = threadIdx.x;
    float hw[8][2];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int n = tid + r * (NC / 8);
        const float2 h = reinterpret_cast<const float2*>(hann)[n];
        hw[r][0] = h.x;
        hw[r][1] = h.y;
    }
    Pass<NC, 8, NT, 8> p2;
    Pass<NC, 8, NT, 64> p3;
    Pass<NC, R4, NT, 512> p4;
    p2.load(tw);
    p3.load(tw);
    p4.load(tw);
    float2 w2r[KREG];
#pragma unroll
    for (int i = 0; i < KREG; ++i) {
        w2r[i] = tw2[min(kmin + tid + i * NT, kmax)];
    }
    for (int i = tid; i < n_mels; i += NT) srows[i] = rows[i];
    for (int i = tid; i < nnz; i += NT) svals[i] = vals[i];

    __syncthreads();
    // persistent loop over (window, frame block) items
    for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
    const int w = item / nfblk;
    const int fb = item - w * nfblk;
    const int f0 = fb * kFpb;
    const int nf = min(kFpb, T - f0);
    const int seg_len = (nf - 1) * hop + NFFT;
    // --- normalisation constants (normalize_data, :203-208) ---
    const aa_window d = wins[w];
    float lo = INFINITY, hi = -INFINITY;
#pragma unroll
    for (int s = 0; s < kStatSplit; ++s) {
        float4 st = stats[w * kStatSplit + s];
        lo = fminf(lo, st.x);
        hi = fmaxf(hi, st.y);
    }
    const float scale = __fsub_rn(hi, lo);  // == max(x - min) (monotone rounding)
    const float inv = __fdiv_rn(1.f, scale);

    // --- overlapped segment -> LDS, normalised; loads issued in batches of
    // SEGU per thread before any is consumed ---
    const int base = f0 * hop - NFFT / 2;  // window index of seg[0]
    constexpr int SEGU = 8;
    const long long safe = d.n_valid > 0 ? d.src : 0;  // any in-bounds sample
    for (int q0 = 0; q0 < seg_len; q0 += SEGU * NT) {
        float raw[SEGU];
        bool ok[SEGU];
#pragma unroll
        for (int u = 0; u < SEGU; ++u) {  // unconditional loads from clamped addresses
            const int q = q0 + u * NT + tid;
            const int i = base + q;
            const int rel = i - d.pad_left;
            ok[u] = q < seg_len && i >= 0 && i < win_len && rel >= 0 && rel < d.n_valid;
            raw[u] = pcm[ok[u] ? d.src + rel : safe];
        }
#pragma unroll
        for (int u = 0; u < SEGU; ++u) {
            const int q = q0 + u * NT + tid;
            const int i = base + q;
            if (q < seg_len) {
                float v = 0.f;
                if (i >= 0 && i < win_len) {
                    v = ok[u] ? raw[u] : 0.f;
                    if (normalize) v = normalize_sample(v, lo, scale, inv);
                }
                seg[q] = v;
            }
        }
    }
    __syncthreads();

    float bmax = 0.f;
    for (int f = 0; f < nf; ++f) {
        // pass 1 (NS = 1) straight from the segment: z[n] = xw[2n] + i xw[2n+1]
        {
            const float* x = seg + f * hop;
            float2 v[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int n = tid + r * NT;
                v[r] = make_float2(x[2 * n] * hw[r][0], x[2 * n + 1] * hw[r][1]);
            }
            dft8(v);
#pragma unroll
            for (int r = 0; r < 8; ++r) bufA[pidx(tid * 8 + r)] = v[r];
        }
        __syncthreads();
        p2.run(bufA, bufB);
        __syncthreads();
        p3.run(bufB, bufA);
        __syncthreads();
        p4.run(bufA, bufB);
        __syncthreads();
        const float2* Z = bufB;             // natural order
        float* Pf = reinterpret_cast<float*>(bufA);  // free scratch for |X|^p
        for (int i = 0; kmin + tid + i * NT <= kmax; ++i) {
            const int k = kmin + tid + i * NT;
            float re, im;
            if (k == 0 || k == NC) {
                const float2 z0 = Z[0];  // pidx(0) == 0
                re = (k == 0) ? z0.x + z0.y : z0.x - z0.y;
                im = 0.f;
            } else {
                const float2 a = Z[pidx(k)];
                const float2 b = Z[pidx(NC - k)];  // conj taken below
                // E = (a + conj b)/2 ; O = -i (a - conj b)/2 ; X = E + W^k O
                const float2 E = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
                const float2 O = make_float2(0.5f * (a.y + b.y), -0.5f * (a.x - b.x));
                float2 wk;
                if (i < KREG) {
                    wk = w2r[0];
#pragma unroll
                    for (int q = 1; q < KREG; ++q) if (i == q) wk = w2r[q];
                } else {
                    wk = tw2[k];
                }
                const float2 X = cadd(E, cmul(wk, O));
                re = X.x;
                im = X.y;
            }
            Pf[k - kmin] = pow_mag<PM>(re, im, power);
        }
        __syncthreads();
        for (int m = tid; m < n_mels; m += NT) {
            const int4 rw = srows[m];
            const float* wv = svals + rw.z;
            const float* pv = Pf + (rw.x - kmin);
            float s = 0.f;
            // predicated 16-wide chunks: all LDS reads of a chunk in flight at once
            for (int i0 = 0; i0 < rw.y; i0 += 16) {
                float a[16], b[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int ii = min(i0 + i, rw.y - 1);  // unconditional LDS reads
                    a[i] = (i0 + i < rw.y) ? wv[ii] : 0.f;
                    b[i] = pv[ii];
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) s = fmaf(a[i], b[i], s);
            }
            melT[m * kFpb + f] = s;
            bmax = fmaxf(bmax, s);
        }
        __syncthreads();  // P / buffers reused by the next frame
    }
    // staged [n_mels][nf] tile -> melS[w][m][f0 .. f0 + nf)
    const float inv_nm = 1.0f / (float)n_mels;  // exact row below 2^21 (as in fe_db)
    for (int idx = tid; idx < nf * n_mels; idx += NT) {  // frame-major rows
        const int f = (int)(((float)idx + 0.5f) * inv_nm), m = idx - f * n_mels;
        melS[((size_t)w * T + f0 + f) * n_mels + m] = melT[m * kFpb + f];
    }
    // item max -> blkmax[w][fb]
    __shared__ float red[NT / 64];
    bmax = wave_max(bmax);
    if ((tid & 63) == 0) red[tid >> 6] = bmax;
    __syncthreads();
    if (tid == 0) {
        for (int k = 1; k < NT / 64; ++k) bmax = fmaxf(bmax, red[k]);
        blkmax[w * nfblk + fb] = bmax;
    }
    }  // item loop
}

// ---------------------------------------------------------------------------
// fe_stft_mel_4096: the n_fft = 4096 path, one WAVE per frame, waves
// independent of each other (no block-level synchronisation after the
// prologue).
//
// normalize_data folded into the transform.  It is affine: inside the window
// y = a (x + beta) with a = 2 / scale, beta = scale (1e-6 - 0.5) - lo
// (src/identify_tracks.py:203-208), and the centre padding is y = 0.  The
// transform is linear, so a frame's spectrum is a * FFT(z) with z = x + beta on
// window samples and 0 on the padding, and |.|^p scales by a^p, applied to the
// mel sums.  In a frame without centre padding beta * 1 only reaches bin 0 of
// the unwindowed transform, i.e. bins -1..1 after the Hann convolution (step
// 7), so interior frames take z = x outright (the host keeps kmin >= 2); edge
// frames add beta and zero their padding.  The reference rounds y to f32
// before its f64 STFT; the two agree to f32 rounding (parity tolerance).
//
// z[n] = x[2n] + i x[2n+1] (2048 complex points) is loaded straight into
// registers: lane c holds n = c + 64 r, r = 0..31 (samples 2c + 128 r and +1),
// through a buffer resource spanning the window's view [src, src + n_valid),
// so np.pad zeros, centre padding and the ends of the recording all read as 0
// by the hardware range check (a negative offset wraps past num_records).
//   1. DFT-32 over r in registers                   -> Y[k1][c]
//   2. Y[k1][c] *= W2048^(c k1)                     (ladder from two table entries)
//   3. transpose through the wave's LDS buffer (two half passes, rows padded
//      to 66 float2 so the row writes and the strided reads are
//      conflict-free): lane L = 2 k1 + h gets Y[k1][h + 2m], m = 0..31
//   4. DFT-32 over m in registers -> E_h[k2']
//   5. radix-2 across the lane pair (DPP quad_perm swap):
//      Z[k1 + 32 k2'] = E0 + W64^k2' E1, Z[k1 + 32 (k2' + 32)] = E0 - W64^k2' E1
//   6. real split X[k] = E + W4096^k O from Z[k], conj Z[2048 - k] (both lanes
//      of a pair, 16 bins each), with
//      W4096^(k1 + 32 j) = W4096^k1 W128^j (one table entry per lane)
//   7. |X|^power into the wave's LDS buffer (the periodic Hann was applied to
//      the samples before step 1, by angle addition from two table values)
//   8. sparse mel rows (CSR in LDS, shared by the block), times a^p ->
//      melF[w][t][:] (frame-major: one contiguous row per frame) and the frame
//      maximum -> pmax[w][t]
// Block = 8 waves sharing one CSR image, 2 blocks per CU (16 waves: VGPRs
// capped at 128).  Each XCD (block b runs on XCD b % 8) owns a contiguous
// eighth of the frames -- neighbouring frames overlap by 4096 - hop samples
// and one L2 then serves the overlap -- and its waves take them round-robin,
// wave-major over its blocks, so the last partial round lands on every SIMD
// (block-major over the whole grid left that round to the first XCDs: 16 frames
// on their SIMDs against 12 elsewhere; 69.6 -> 64.0 us alone).
// ---------------------------------------------------------------------------
// band slots of the wave-per-frame kernel's CSR image: whole rounds of 64 lanes
__host__ __device__ constexpr int fe_mel_slots(int n_mels) { return (n_mels + 63) / 64 * 64; }

#ifndef AA_FE_WPB
#define AA_FE_WPB 8
#endif
#ifndef AA_FE_MEL_G
#define AA_FE_MEL_G 2  // mel rows: float4 groups whose loads are issued together (0: one per loop trip)
#endif
#ifndef AA_FE_MEL_P
#define AA_FE_MEL_P 1  // mel rows: slots (rounds of 64) whose first groups load together
#endif
constexpr int kWpb = AA_FE_WPB;         // waves per block (2 blocks per CU)

// DIAG (tools/fe_bench.hip only): 1 skip the PCM loads, 4 the FFT (steps 1-5),
// 8 the real split, 16 Hann and power, 32 the mel rows, 64 the output stores.
// DIAG & 128 (tools/fe_bench.hip): per-wave s_memtime totals of the frame's
// phases into fe_stamps[global wave][phase][lane] (every lane stores: vector
// stores only) -- 0 loads + Hann, 1 DFT-32 #1, 2 twiddles, 3 transpose,
// 4 DFT-32 #2, 5 radix-2, 6 split + power, 7 mel rows
constexpr int kFeStampPh = 8;
__device__ unsigned long long* fe_stamps = nullptr;
#define FE_STAMP(k)                                                              \
    if constexpr ((DIAG & 128) != 0) {                                           \
        const unsigned long long tn = __builtin_amdgcn_s_memtime();              \
        st_acc[k] += tn - st_prev;                                               \
        st_prev = tn;                                                            \
    }
template <int PM, int DIAG = 0>
__global__ __launch_bounds__(64 * kWpb) __attribute__((amdgpu_waves_per_eu(kWpb / 2, kWpb / 2))) void fe_stft_mel_4096(
    const float* __restrict__ pcm, const aa_window* __restrict__ wins, const float4* __restrict__ stats,
    const float2* __restrict__ tw, const float2* __restrict__ tw4096, const char* __restrict__ cimg,
    int cimg_bytes, int win_len, int hop, int T, int n_mels, int kmin, int kmax, int normalize, float power,
    int n_frames, float* __restrict__ melF, float* __restrict__ pmax) {
    constexpr int NC = 2048;
    extern __shared__ float lds[];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    char* cl = reinterpret_cast<char*>(lds);
    const int4* srows = reinterpret_cast<const int4*>(cl);  // CSR image (fe_cimg4096): rows | values
    const float* svals = reinterpret_cast<const float*>(srows + fe_mel_slots(n_mels));
    float2* wb = reinterpret_cast<float2*>(cl + cimg_bytes) + wave * kHalf;  // this wave's buffer

    for (int g = wave; g < cimg_bytes / 1024; g += kWpb)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(cimg + g * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(cl + g * 1024), 16, 0, 0);
    const int k1 = lane >> 1, h = lane & 1;
    float2 t1 = tw[lane];                // W2048^c
    float2 t8 = tw[(8 * lane) & (NC - 1)];  // W2048^(8c)
    const float2 wk1 = tw4096[k1];       // W4096^k1
    // (cos, sin) of 2 pi n / 4096 at the lane's first even / odd sample n = 2c, 2c + 1
    const float2 te = tw4096[2 * lane], to = tw4096[2 * lane + 1];
    const float2 hwe = make_float2(te.x, -te.y), hwo = make_float2(to.x, -to.y);
    __syncthreads();                     // vmcnt(0): the CSR image has landed
    unsigned long long st_acc[kFeStampPh] = {}, st_prev = 0;
    // the PCM samples of frame fl into yy (step 0): lane c gets z[c + 64 r]
    auto load_frame = [&](int fl, float2 (&yy)[32]) {
        const int wl = fl / T;
        const aa_window dl = wins[wl];
        const int i0l = (fl - wl * T) * hop - 2048;
        // per-lane sample index, opaque to the optimiser: otherwise it hoists the
        // 64 loop-invariant load offsets and edge masks out of the frame loop
        // and spills them
        int l2l = 2 * lane;
        __asm__ volatile("" : "+v"(l2l));
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(pcm + dl.src), 0, dl.n_valid * 4, 0x00020000);
        // even and odd samples through two address registers: the backend
        // must not fuse a pair into one 8-byte load, whose range check would
        // not zero the two samples independently
        const int offe = i0l - dl.pad_left + l2l;
        const int v0 = i0l - dl.pad_left;  // the frame's first sample in the view
        if (v0 >= 0 && v0 + 4096 <= dl.n_valid) {
            // frame inside the view (wave-uniform): no sample is range checked,
            // so a lane's pair comes in one 8-byte load (32 fully used 512-B
            // wave-instructions instead of 64 half-used)
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const uint2 v = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, (offe + 128 * r) * 4, 0, 0));
                yy[r] = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
            }
        } else {
            int offo = offe + 1;
            __asm__ volatile("" : "+v"(offo));
#pragma unroll
            for (int r = 0; r < 32; ++r) yy[r] = make_float2(load_view(rs, offe + 128 * r), load_view(rs, offo + 128 * r));
        }
    };

    // XCD x (block b runs on XCD b % 8) owns frames [x n / 8, (x + 1) n / 8);
    // its waves take them round-robin, wave-major over its blocks, so the last,
    // partial round is spread over every XCD, CU and SIMD (a block's waves w
    // and w + 4 share a SIMD) instead of filling the first XCDs only
    const int nbx = gridDim.x >> 3;  // blocks per XCD (grid a multiple of 8)
    const int xcd = blockIdx.x & 7;
    const int f_end = (int)((long long)(xcd + 1) * n_frames / 8);
    const int G = nbx * kWpb;
    const int f_first = (int)((long long)xcd * n_frames / 8) + wave * nbx + (blockIdx.x >> 3);
    for (int fi = f_first; fi < f_end; fi += G) {
        const int w = fi / T;
        const int t = fi - w * T;
        if constexpr ((DIAG & 128) != 0) st_prev = __builtin_amdgcn_s_memtime();
        float apow = 1.f, beta = 0.f;
        if (normalize) {
            float lo = INFINITY, hi = -INFINITY;
#pragma unroll
            for (int s = 0; s < kStatSplit; ++s) {
                const float4 st = stats[w * kStatSplit + s];
                lo = fminf(lo, st.x);
                hi = fmaxf(hi, st.y);
            }
            const float scale = __fsub_rn(hi, lo);  // == max(x - min) (monotone rounding)
            const float a = __fdiv_rn(2.f, scale);
            apow = PM == PM_SQUARE ? a * a : PM == PM_ABS ? a : powf(a, power);
            beta = fmaf(scale, 0.000001f - 0.5f, -lo);
        }
        const int i0 = t * hop - 2048;  // window index of the frame's first sample
        // per-lane sample index, opaque to the optimiser: otherwise it hoists the
        // 64 loop-invariant load offsets and edge masks out of the frame loop
        // and spills them
        int l2 = 2 * lane;
        __asm__ volatile("" : "+v"(l2));
        float2 wk = wk1;  // per frame, or W4096^k1 W128^j gets hoisted as 32 live twiddles
        __asm__ volatile("" : "+v"(wk.x), "+v"(wk.y));
        float2 u[32];
        {
            // ---- load (steps 0) ----
            float2 y[32];
            if constexpr ((DIAG & 1) != 0) {
#pragma unroll
                for (int r = 0; r < 32; ++r) y[r] = make_float2((float)(lane + r), (float)(t - r));
            } else {
                load_frame(fi, y);
            }
            if (normalize && (i0 < 0 || i0 + 4096 > win_len)) {  // edge frame: + beta, centre padding 0
#pragma unroll
                for (int r = 0; r < 32; ++r) {
                    const int i = i0 + l2 + 128 * r;
                    y[r].x = (i >= 0 && i < win_len) ? y[r].x + beta : 0.f;
                    y[r].y = (i + 1 >= 0 && i + 1 < win_len) ? y[r].y + beta : 0.f;
                }
            }
            // periodic Hann, w[n] = 1/2 - cos(2 pi n / 4096) / 2 at n = 2c + 128 r
            // (+1): cos(a + 2 pi r / 32) by angle addition from the lane's
            // cos/sin of a (table values; opaque per frame so the 64 products
            // are not hoisted into live registers)
            // The upper half-wave's (-1)^r input modulation of step 1 is folded
            // in as the sign of the odd-r weights: +-1/2 per lane.
            float2 he = hwe, ho = hwo;
            float hs = lane >= 32 ? -0.5f : 0.5f;
            __asm__ volatile("" : "+v"(he.x), "+v"(he.y), "+v"(ho.x), "+v"(ho.y), "+v"(hs));
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const float cr = kW32[r][0], sr = -kW32[r][1];  // cos, sin of 2 pi r / 32
                const float ce = fmaf(he.x, cr, -he.y * sr), co = fmaf(ho.x, cr, -ho.y * sr);
                const float a = (r & 1) ? hs : 0.5f;  // w = a (1 - cos)
                y[r].x *= fmaf(-a, ce, a);
                y[r].y *= fmaf(-a, co, a);
            }
            FE_STAMP(0)
            if constexpr ((DIAG & 4) != 0) {
#pragma unroll
                for (int j = 0; j < 32; ++j) u[j] = y[j];
            } else {
                // (the same steps as aa_wavefft.h's wave_hann + wave_fft_core,
                // kept inline here: called as functions, the register
                // allocation of this kernel spills 11 VGPRs)
                // The transpose (step 3) runs in two passes of 16 registers per
                // lane, each pass freeing 16 registers before it fills 16, so the
                // data never occupies more than 64 VGPRs.  For that, the upper
                // half-wave (columns c >= 32) works with its rows rotated by 16:
                // (-1)^r on the input gives DFT output X[(k + 16) % 32] in
                // register k (step 1), its twiddle ladder is rotated to match
                // (step 2), it reads its columns rotated by 16 (step 3), and
                // undoes that rotation of the second DFT by (-1)^k on the odd
                // outputs (step 4).
                const unsigned up = lane >= 32 ? 0x80000000u : 0u;  // sign mask of the upper half
                auto flip = [up](float2 v) {
                    return make_float2(__uint_as_float(__float_as_uint(v.x) ^ up),
                                       __uint_as_float(__float_as_uint(v.y) ^ up));
                };
                // ---- 1. DFT-32 over r ----
                // (the (-1)^r of the upper half rides on its Hann weights, above)
                dft32(y);
                FE_STAMP(1)
                // ---- 2. twiddle W2048^(c row) = (W^8c)^(row/8) (W^c)^(row%8),
                // row = k (+16 mod 32 in the upper half); ladders rebuilt per frame
                // (<= 4 roundings per twiddle; not kept live across the loop) ----
                __asm__ volatile("" : "+v"(t1.x), "+v"(t1.y), "+v"(t8.x), "+v"(t8.y));
                float2 p1[8], p8[4];
                p1[0] = make_float2(1.f, 0.f);
                p1[1] = t1;
#pragma unroll
                for (int i = 2; i < 8; ++i) p1[i] = cmul(p1[i - 1], t1);
                {
                    const float2 q1 = t8, q2 = cmul(t8, t8), q3 = cmul(q2, t8);
                    const bool hi = lane >= 32;
                    p8[0] = hi ? q2 : make_float2(1.f, 0.f);
                    p8[1] = hi ? q3 : q1;
                    p8[2] = hi ? make_float2(1.f, 0.f) : q2;
                    p8[3] = hi ? q1 : q3;
                }
#pragma unroll
                for (int k = 0; k < 32; ++k) {
                    const float2 tk = (k & 7) == 0 ? p8[k >> 3] : cmul(p8[k >> 3], p1[k & 7]);
                    y[dperm(k)] = cmul(y[dperm(k)], tk);
                }
                FE_STAMP(2)
                // ---- 3. transpose in two passes: pass p moves registers
                // 16p..16p+15 (rows (16p + 16 [c >= 32]) % 32 + 0..15 of column
                // c) and lane (k1, h) takes columns h + 2m, m in the 16-range
                // 16 ((k1 / 16) ^ p) of row k1, into u[16p ..] ----
#pragma unroll
                for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
                    for (int k = 0; k < 16; ++k) wb[k * kRow + lane] = y[dperm(16 * pass + k)];
                    wave_sync();
                    const float2* src = wb + (k1 & 15) * kRow + h + 32 * (((k1 >> 4) ^ pass) & 1);
#pragma unroll
                    for (int i = 0; i < 16; ++i) u[16 * pass + i] = src[2 * i];
                    wave_sync();
                }
                FE_STAMP(3)
                // ---- 4. DFT-32 over m (input rotated by 16 in the upper half:
                // output k times (-1)^k) ----
                dft32(u);
#pragma unroll
                for (int k = 1; k < 32; k += 2) u[dperm(k)] = flip(u[dperm(k)]);
                FE_STAMP(4)
                // ---- 5. radix-2 across the lane pair: lane h = 1 sends
                // W64^j E1, lane h = 0 sends E0; then Z = E0 + W E1 (h = 0) and
                // E0 - W E1 (h = 1) are recv +- own ----
                const float sg = h ? -1.f : 1.f;
#pragma unroll
                for (int j = 0; j < 32; ++j) {
                    const float2 e = u[dperm(j)];
                    const float2 wj = wconst64(j);
                    const float2 g = h ? cmul(wj, e) : e;
                    const float2 rv = make_float2(swap_pair(g.x), swap_pair(g.y));
                    u[dperm(j)] = make_float2(fmaf(sg, g.x, rv.x), fmaf(sg, g.y, rv.y));
                }
                FE_STAMP(5)
            }
        }
        // lane holds Z[k1 + 32 (32 h + j)] in u[dperm(j)]
        // ---- 6. real split and |X|^power ----
        if (h && !(DIAG & 8)) {
#pragma unroll
            for (int j = 0; j < 32; ++j) wb[k1 + 32 * j] = u[dperm(j)];  // Z[1024 + k1 + 32 j]
        }
        wave_sync();
        // Both lanes of a pair split: lane h takes the bins k = k1 + 32 (16 h +
        // i), i < 16 (all 1024 bins below NC/2 over the 64 lanes; bands above
        // take the generic kernel, see fe_fast4096).  Z[k] is the h = 0 lane's
        // u[dperm(16 h + i)] (the h = 1 lane swaps it over from its partner),
        // its mirror Z[2048 - k] the h = 1 lanes' LDS copy.  |X|^p is stored
        // reversed from the top of the wave's buffer (bin k at float Pt[-k],
        // Pt = float 2 kHalf - 1), where it overlaps mirrors that later
        // iterations still read, so the 16 values wait in registers until the
        // loop is done.
        float* Pt = reinterpret_cast<float*>(wb) + (2 * kHalf - 1);
        if (!(DIAG & 8)) {
            // mirror of bin k1 + 32 (16 h + i) at wb[1024 - k] = mb[32 (31 - i)]
            // (one base register, non-negative immediates; wb[1024], read for
            // k = 0, is in the buffer and unused)
            const float2* mb = wb + (32 - k1) - 512 * h;
            float* pk = Pt - k1 - 512 * h - 32 * 15;  // bin k at pk[32 (15 - i)] = Pt[-k]
            // W4096^k = W4096^k1 (W4096^512)^h W128^i, W4096^512 = (r, -r)
            const float r2 = 0.70710678118654752440f;
            const float2 wkh = h ? make_float2(r2 * (wk.x + wk.y), r2 * (wk.y - wk.x)) : wk;
            float pw[16];
            float2 zm[16];  // mirrors, read 8 ahead of their use
#pragma unroll
            for (int i = 0; i < 8; ++i) zm[i] = mb[32 * (31 - i)];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (i % 8 == 0 && i + 8 < 16) {
#pragma unroll
                    for (int k = i + 8; k < i + 16; ++k) zm[k] = mb[32 * (31 - k)];
                }
                const float2 hiv = u[dperm(16 + i)];
                const float2 oth = make_float2(swap_pair(hiv.x), swap_pair(hiv.y));
                const float2 a = h ? oth : u[dperm(i)];
                const float2 zb = zm[i];
                const float2 b = (i == 0 && k1 == 0 && !h) ? a : zb;  // Z[NC - k]; Z[0] for k = 0
                const float2 E = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
                const float2 O = make_float2(0.5f * (a.y + b.y), -0.5f * (a.x - b.x));
                float2 wj = cmul(wkh, wconst128(i));  // W4096^k
                __asm__ volatile("" : "+v"(wj.x), "+v"(wj.y));  // formed here, not hoisted
                const float2 X = cadd(E, cmul(wj, O));
                pw[i] = pow_mag<PM>(X.x, X.y, power);
            }
            if (!(DIAG & 16)) {
#pragma unroll
                for (int i = 0; i < 16; ++i) pk[32 * (15 - i)] = pw[i];
            }
        }
        wave_sync();
        FE_STAMP(6)
        // ---- 8. mel rows ----
        // rows of the CSR image are zero-padded to whole float4s (value
        // offsets 16-B aligned); the padding adds exact zeros
        float fmx = 0.f;
        float* orow = melF + (size_t)fi * n_mels;  // fi = w T + t
        const int nslot = fe_mel_slots(n_mels);
#if AA_FE_MEL_G > 0
        // the slot index opaque per frame: the rows' descriptors and value
        // addresses are frame-invariant, and hoisted out of the frame loop they
        // would stay live through the FFT (spills)
        int si0 = lane;
        __asm__ volatile("" : "+v"(si0));
#else
        const int si0 = lane;
#endif
        // slot si holds band rw.w (-1: empty, length 0) covering bins [x, x +
        // L): its values are stored reversed and front-padded to L4 = roundup(L,
        // 4) (fe_cimg4096), so with P reversed the row is an ascending run
        // pv[0 .. L4)
#if AA_FE_MEL_G > 0
        // P slots per trip, the first G float4 groups of each: every load issued
        // before the first FMA (one LDS round trip for P x G groups instead of
        // one per group), then each row's FMA chain in the order of the plain
        // loop (identical sums; fe_bench's hash, profiles/r06/fe_mel_groups.txt)
        constexpr int G = AA_FE_MEL_G, NP = AA_FE_MEL_P;
        for (int si = si0; si < ((DIAG & 32) ? 0 : nslot); si += 64 * NP) {
            int4 rw[NP];
            const float4* wv[NP];
            const float* pv[NP];
            float4 wa[NP][G];
            float pa[NP][G][4];
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const int sq = si + 64 * q;
                // a slot past the last round is an empty row (its loads stay
                // inside the wave's power buffer, as fe_cimg4096's empty slots)
                rw[q] = sq < nslot ? srows[sq] : make_int4(kmin + 3, 0, 0, -1);
                wv[q] = reinterpret_cast<const float4*>(svals + rw[q].z);
                pv[q] = Pt - rw[q].x - (rw[q].y - 1);  // bins x + L4 - 1 down to x
                // (groups past the row re-read its last group: in range, unused)
                const int glast = max((rw[q].y >> 2) - 1, 0);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int gi = min(g, glast);
                    wa[q][g] = wv[q][gi];
#pragma unroll
                    for (int e = 0; e < 4; ++e) pa[q][g][e] = pv[q][4 * gi + e];
                }
            }
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                float s = 0.f;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    if (4 * g < rw[q].y) {
                        s = fmaf(wa[q][g].x, pa[q][g][0], s);
                        s = fmaf(wa[q][g].y, pa[q][g][1], s);
                        s = fmaf(wa[q][g].z, pa[q][g][2], s);
                        s = fmaf(wa[q][g].w, pa[q][g][3], s);
                    }
                }
                for (int i = 4 * G; i < rw[q].y; i += 4) {
                    const float4 a = wv[q][i >> 2];
                    s = fmaf(a.x, pv[q][i], s);
                    s = fmaf(a.y, pv[q][i + 1], s);
                    s = fmaf(a.z, pv[q][i + 2], s);
                    s = fmaf(a.w, pv[q][i + 3], s);
                }
                s *= apow;
                if (!(DIAG & 64) && rw[q].w >= 0) orow[rw[q].w] = s;
                fmx = fmaxf(fmx, s);
            }
        }
#else
        for (int si = si0; si < ((DIAG & 32) ? 0 : nslot); si += 64) {
            const int4 rw = srows[si];
            const float4* wv = reinterpret_cast<const float4*>(svals + rw.z);
            const float* pv = Pt - rw.x - (rw.y - 1);  // bins x + L4 - 1 down to x
            float s = 0.f;
            for (int i = 0; i < rw.y; i += 4) {
                const float4 a = wv[i >> 2];
                s = fmaf(a.x, pv[i], s);
                s = fmaf(a.y, pv[i + 1], s);
                s = fmaf(a.z, pv[i + 2], s);
                s = fmaf(a.w, pv[i + 3], s);
            }
            s *= apow;
            if (!(DIAG & 64) && rw.w >= 0) orow[rw.w] = s;
            fmx = fmaxf(fmx, s);
        }
#endif
        fmx = wave_max(fmx);
        if (lane == 0 && !(DIAG & 64)) pmax[fi] = fmx;
        wave_sync();  // the buffer is rewritten by the next frame
        FE_STAMP(7)
    }
    if constexpr ((DIAG & 128) != 0) {
        const size_t gw = (size_t)blockIdx.x * kWpb + wave;
#pragma unroll
        for (int k = 0; k < kFeStampPh; ++k) fe_stamps[(gw * kFeStampPh + k) * 64 + lane] = st_acc[k];
    }
}

// ---------------------------------------------------------------------------
// fe_db: power_to_db(ref=max), clamp at -top_db, mean_sub, channel repeat,
// and the frame-major -> band-major transpose of the stft kernels' output.
// Block = (tile of `tile_t` frames, window): coalesced rows of melF in,
// dB in registers, transpose through LDS, contiguous band rows out.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float db_value(float v, float ref_db, int db_scale, float amin, float top_db) {
    if (db_scale) {
        v = __fsub_rn(__fmul_rn(10.0f, log10f(fmaxf(amin, v))), ref_db);
        v = fmaxf(v, -top_db);  // log_spec.max() == 0 exactly
    }
    return v;
}

// block-wide max of the window's partial maxima -> 10 log10(max(amin, S.max()))
__device__ __forceinline__ float window_ref_db(const float* __restrict__ pmax, int nparts, float amin, float* red) {
    float mx = 0.f;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) mx = fmaxf(mx, pmax[i]);
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    mx = red[0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) mx = fmaxf(mx, red[k]);
    return __fmul_rn(10.0f, log10f(fmaxf(amin, mx)));
}

// TO: float, or _Float16 for the fp16 log-mel of aa_fe_config.out_f16
template <typename TO>
__global__ __launch_bounds__(256) void fe_db(const float* __restrict__ melF, const float* __restrict__ pmax,
                                             int nparts, const float4* __restrict__ stats,
                                             const float* __restrict__ band_mean, int n_mels, int T, int tile_t,
                                             int db_scale, float amin, float top_db, int channels, int normalize,
                                             TO* __restrict__ out, int* __restrict__ status) {
    extern __shared__ float tile[];  // [tile_t][n_mels + 1]
    __shared__ float red[4];
    const int w = blockIdx.y;
    const int t0 = blockIdx.x * tile_t;
    const int nt = min(tile_t, T - t0);
    const int ld = n_mels + 1;
    const float* src = melF + ((size_t)w * T + t0) * n_mels;  // nt contiguous frame rows
    const int total = nt * n_mels;
    // row of element idx as a float product: exact while idx < 2^21 (the tile
    // holds at most 2^14 elements), ~35 VALU cheaper than an integer divide
    const float inv_nm = 1.0f / (float)n_mels;
    const int tsh = __builtin_ctz(tile_t);  // tile_t is a power of two (host)
#ifndef AA_FE_DB_U
#define AA_FE_DB_U 8
#endif
    constexpr int U = AA_FE_DB_U;  // loads in flight per thread before any is consumed
    // the first batch of rows is issued before the window's reference max
    // (independent loads: their latencies overlap instead of adding up)
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[min(u * 256 + (int)threadIdx.x, total - 1)];
    const float ref_db = window_ref_db(pmax + (size_t)w * nparts, nparts, amin, red);
    if (blockIdx.x == 0 && threadIdx.x == 0 && status) {
        float lo = INFINITY, hi = -INFINITY;
        int bad = 0;
        for (int s = 0; s < kStatSplit; ++s) {
            const float4 st = stats[w * kStatSplit + s];
            lo = fminf(lo, st.x);
            hi = fmaxf(hi, st.y);
            bad |= st.z != 0.f;
        }
        // normalize_data divides by max(x - min): 0 -> NaN -> librosa raises
        if (normalize && !(hi - lo > 0.f)) bad = 1;
        status[w] = bad ? AA_WIN_NONFINITE : AA_WIN_OK;
    }
    for (int i0 = 0; i0 < total; i0 += U * 256) {
        if (i0 > 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = src[min(i0 + u * 256 + (int)threadIdx.x, total - 1)];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int idx = i0 + u * 256 + threadIdx.x;
            if (idx < total) {
                const int tt = (int)(((float)idx + 0.5f) * inv_nm), m = idx - tt * n_mels;
                tile[tt * ld + m] = db_value(v[u], ref_db, db_scale, amin, top_db);
            }
        }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < n_mels * tile_t; idx += 256) {
        const int m = idx >> tsh, tt = idx & (tile_t - 1);
        if (tt < nt) {
            float v = tile[tt * ld + m];
            if (band_mean) v -= band_mean[(size_t)w * n_mels + m];
            TO* o = out + (((size_t)w * n_mels + m) * T + t0 + tt) * channels;
            for (int c = 0; c < channels; ++c) o[c] = (TO)v;
        }
    }
}

// mean_sub: per-band mean over time of the dB values, one block per window
__global__ __launch_bounds__(256) void fe_band_mean(const float* __restrict__ melF, const float* __restrict__ pmax,
                                                    int nparts, int n_mels, int T, int db_scale, float amin,
                                                    float top_db, float* __restrict__ band_mean) {
    __shared__ float red[4];
    const int w = blockIdx.x;
    const float ref_db = window_ref_db(pmax + (size_t)w * nparts, nparts, amin, red);
    const float* src = melF + (size_t)w * T * n_mels;
    for (int m = threadIdx.x; m < n_mels; m += 256) {
        float s = 0.f;
        for (int t = 0; t < T; ++t) s += db_value(src[(size_t)t * n_mels + m], ref_db, db_scale, amin, top_db);
        band_mean[(size_t)w * n_mels + m] = s / (float)T;
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static size_t fe_lds_bytes(const FePlan& p) {
    const int nc = p.cfg.n_fft / 2;
    const int seg_cap = ((kFpb - 1) * p.cfg.hop + p.cfg.n_fft + 3) & ~3;
    return sizeof(float) * ((size_t)seg_cap + 4 * (size_t)(nc + nc / 8) + (size_t)((p.cfg.n_mels * kFpb + 3) & ~3) + 4 * (size_t)p.cfg.n_mels +
                            (size_t)std::max(p.nnz, 1));
}

template <int NFFT, int PM>
static int launch_stft(const FePlan& p, const float* pcm, const aa_window* wins, int n_win,
                       const float4* stats, float* melS, float* blkmax, hipStream_t st) {
    const size_t lds = fe_lds_bytes(p);
    AA_CHECK(lds <= 150 * 1024, AA_ERR_UNSUPPORTED, "fe: hop %d needs %zu B of LDS", p.cfg.hop, lds);
    AA_DYN_LDS((fe_stft_mel<NFFT, PM>), lds);  // dynamic LDS opt-in (static LDS comes on top)
    const int n_items = p.nfblk * n_win;
    // persistent grid: as many blocks as fit (LDS-limited) on 256 CUs
    const int per_cu = std::max(1, (int)((160 * 1024) / (lds + 256)));
    const int grid = std::min(n_items, 256 * per_cu);
    hipLaunchKernelGGL((fe_stft_mel<NFFT, PM>), dim3(grid), dim3(NFFT / 16), lds, st, pcm, wins, stats, p.d_win,
                       p.d_tw, p.d_tw2, p.d_rows, p.d_vals, p.nnz, p.cfg.win_len, p.cfg.hop, p.T,
                       p.cfg.n_mels, p.kmin, p.kmax, p.cfg.normalize, p.cfg.power, p.nfblk, n_items,
                       melS, blkmax);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

// the wave-per-frame kernel covers n_fft 4096 whenever the kept band fits the
// per-wave buffer (15 bins per lane)
static bool fe_fast4096(const FePlan& p) {
    // kept band inside X[2..1022]: Hann neighbours in range and clear of the
    // bins -1..1 that the folded normalisation offset touches; padded rows
    // (+3 bins) inside the 15 x 64 power slots
    return p.cfg.n_fft == 4096 && p.kmin >= 2 && p.kmax <= 1022 && p.kmin + 64 * (kHalf / 64 - 1) < kHalf &&
           p.kmax - p.kmin + 1 + 3 <= (kHalf / 64 - 1) * 64;
}

static size_t fe_lds_bytes4096(const FePlan& p) {
    return (size_t)p.cimg_bytes + sizeof(float2) * (size_t)kWpb * kHalf;
}

template <int PM>
static int launch_stft4096(const FePlan& p, const float* pcm, const aa_window* wins, int n_win,
                           const float4* stats, float* melS, float* pmax, hipStream_t st) {
    const size_t lds = fe_lds_bytes4096(p);
    AA_CHECK(lds <= 160 * 1024, AA_ERR_UNSUPPORTED, "fe4096: %zu B of LDS", lds);
    AA_DYN_LDS(fe_stft_mel_4096<PM>, lds);
    const int n_frames = p.T * n_win;
    // persistent grid: blocks resident together (LDS-limited, 2 per CU at the
    // CFG filterbank), a multiple of 8 for the XCD renumbering
    // (1 block per CU measured -1.5 % on the two-stream step, profiles/r05/ab_fe_per_cu.txt)
    const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / lds)));
    int grid = std::min((n_frames + kWpb - 1) / kWpb, 256 * per_cu);
    grid = (grid + 7) & ~7;
    hipLaunchKernelGGL(fe_stft_mel_4096<PM>, dim3(grid), dim3(64 * kWpb), lds, st, pcm, wins, stats, p.d_tw,
                       p.d_tw2, p.d_cimg, p.cimg_bytes, p.cfg.win_len, p.cfg.hop, p.T, p.cfg.n_mels, p.kmin,
                       p.kmax, p.cfg.normalize, p.cfg.power, n_frames, melS, pmax);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

struct FeWs {
    float4* stats;
    float* melS;       // frame-major mel power [n_win][T][n_mels]
    float* blkmax;     // partial maxima [n_win][nparts]
    float* band_mean;  // mean_sub: [n_win][n_mels]
    size_t bytes;
};

static FeWs fe_ws_layout(const FePlan& p, int n_win, char* base) {
    FeWs w{};
    size_t off = 0;
    w.stats = reinterpret_cast<float4*>(base + off);
    off = align_up(off + sizeof(float4) * (size_t)n_win * kStatSplit, 256);
    w.melS = reinterpret_cast<float*>(base + off);
    off = align_up(off + sizeof(float) * (size_t)n_win * p.cfg.n_mels * p.T, 256);
    w.blkmax = reinterpret_cast<float*>(base + off);
    off = align_up(off + sizeof(float) * (size_t)n_win * p.nfblk, 256);
    w.band_mean = reinterpret_cast<float*>(base + off);
    if (p.cfg.mean_sub) off = align_up(off + sizeof(float) * (size_t)n_win * p.cfg.n_mels, 256);
    w.bytes = off;
    return w;
}

}  // namespace aa

using namespace aa;

extern "C" int aa_fe_create(const aa_fe_config* cfg, const float* melfb, void** plan) {
    AA_CHECK(cfg && melfb && plan, AA_ERR_INVALID, "aa_fe_create: null argument");
    const int n = cfg->n_fft;
    AA_CHECK(n == 2048 || n == 4096 || n == 8192, AA_ERR_UNSUPPORTED,
             "aa_fe_create: n_fft %d not supported (power of two 2048..8192)", n);
    AA_CHECK(cfg->hop > 0 && cfg->win_len > 0 && cfg->n_mels > 0 && cfg->channels >= 1 &&
                 (cfg->out_f16 == 0 || cfg->out_f16 == 1),
             AA_ERR_INVALID, "aa_fe_create: bad sizes");
    FePlan* p = new FePlan();
    p->cfg = *cfg;
    p->T = 1 + cfg->win_len / cfg->hop;

    const int nbins = n / 2 + 1;
    // CSR of the dense filterbank (rows are contiguous triangles; keep
    // [first nonzero, last nonzero] per row)
    std::vector<int4> rows(cfg->n_mels);
    std::vector<float> vals;
    int kmin = nbins, kmax = 0;
    for (int m = 0; m < cfg->n_mels; ++m) {
        const float* r = melfb + (size_t)m * nbins;
        int a = -1, b = -1;
        for (int k = 0; k < nbins; ++k)
            if (r[k] != 0.f) { if (a < 0) a = k; b = k; }
        if (a < 0) { a = 0; b = -1; }
        rows[m] = make_int4(a, b - a + 1, (int)vals.size(), 0);
        for (int k = a; k <= b; ++k) vals.push_back(r[k]);
        if (b >= a) { kmin = std::min(kmin, a); kmax = std::max(kmax, b); }
    }
    if (kmax < kmin) { kmin = 0; kmax = 0; }
    for (auto& r : rows) if (r.y == 0) r.x = kmin;
    p->kmin = kmin;
    p->kmax = kmax;
    p->nnz = (int)vals.size();
    // per-window partial maxima: one per frame block of whichever kernel runs
    p->nfblk = fe_fast4096(*p) ? p->T : (p->T + kFpb - 1) / kFpb;
    if (vals.empty()) vals.push_back(0.f);
    const int nc = n / 2;
    std::vector<float> win(n);
    for (int i = 0; i < n; ++i) win[i] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * i / n));
    std::vector<float2> tw(nc), tw2(nc + 1);
    for (int m = 0; m < nc; ++m) {
        const double a = -2.0 * M_PI * m / nc;
        tw[m] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    for (int k = 0; k <= nc; ++k) {
        const double a = -2.0 * M_PI * k / n;
        tw2[k] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    auto up = [](void** d, const void* h, size_t b) -> hipError_t {
        hipError_t e = hipMalloc(d, b);
        if (e != hipSuccess) return e;
        return hipMemcpy(*d, h, b, hipMemcpyHostToDevice);
    };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = up((void**)&p->d_win, win.data(), sizeof(float) * n);
    if (e == hipSuccess) e = up((void**)&p->d_tw, tw.data(), sizeof(float2) * nc);
    if (e == hipSuccess) e = up((void**)&p->d_tw2, tw2.data(), sizeof(float2) * (nc + 1));
    if (e == hipSuccess) e = up((void**)&p->d_rows, rows.data(), sizeof(int4) * rows.size());
    if (e == hipSuccess) e = up((void**)&p->d_vals, vals.data(), sizeof(float) * vals.size());
    if (e == hipSuccess && n == 4096) {
        // CSR image of the wave-per-frame kernel, byte-identical to its LDS
        // region: rows (first bin, padded length, value offset) | values, each
        // row zero-padded to whole float4s (value offsets 16-B aligned)
        // Rows sit in fe_mel_slots() slots, slot i served by lane i % 64 (the
        // .w field names the band): the longest row first goes to the
        // least-loaded lane with a free slot, so the lanes' loop trip counts
        // stay close (round-robin rows gave lane 31 the 3 widest-spaced rows:
        // 52 bins against a mean of 32).  Empty slots have length 0.
        const int nslot = fe_mel_slots(cfg->n_mels);
        // (an empty slot's first bin: kmin + 3, so that the grouped loads of an
        // empty row, AA_FE_MEL_G, read inside the wave's power buffer)
        std::vector<int4> prow(nslot, make_int4(kmin + 3, 0, 0, -1));
        std::vector<float> pval;
        std::vector<int> order(rows.size());
        for (size_t m = 0; m < rows.size(); ++m) order[m] = (int)m;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return rows[a].y > rows[b].y; });
        std::vector<int> load(64, 0), used(64, 0);
        for (int m : order) {
            int best = -1;
            for (int l = 0; l < 64; ++l)
                if (used[l] < nslot / 64 && (best < 0 || load[l] < load[best])) best = l;
            const int len = (rows[m].y + 3) & ~3, pad = len - rows[m].y;
            // (the kernel keeps the band power reversed: values are stored last
            // bin first, zero-padded at the front, so a row reads one ascending run)
            prow[best + 64 * used[best]] = make_int4(rows[m].x, len, (int)pval.size(), m);
            load[best] += len;
            ++used[best];
            for (int i = 0; i < len; ++i) pval.push_back(i < pad ? 0.f : vals[rows[m].z + rows[m].y - 1 - (i - pad)]);
        }
        const size_t raw = sizeof(int4) * prow.size() + sizeof(float) * pval.size();
        std::vector<char> img((raw + 1023) / 1024 * 1024, 0);
        memcpy(img.data(), prow.data(), sizeof(int4) * prow.size());
        memcpy(img.data() + sizeof(int4) * prow.size(), pval.data(), sizeof(float) * pval.size());
        p->cimg_bytes = (int)img.size();
        e = up((void**)&p->d_cimg, img.data(), img.size());
    }
    if (e != hipSuccess) {
        set_error("aa_fe_create: %s", hipGetErrorString(e));
        aa_fe_destroy(p);
        return AA_ERR_HIP;
    }
    AA_CHECK(fe_lds_bytes(*p) <= 150 * 1024, AA_ERR_UNSUPPORTED,
             "aa_fe_create: hop %d too large for the LDS segment", cfg->hop);
    *plan = p;
    return AA_OK;
}

extern "C" int aa_fe_destroy(void* plan) {
    FePlan* p = static_cast<FePlan*>(plan);
    if (!p) return AA_OK;
    (void)hipFree(p->d_win);
    (void)hipFree(p->d_tw);
    (void)hipFree(p->d_tw2);
    (void)hipFree(p->d_rows);
    (void)hipFree(p->d_vals);
    (void)hipFree(p->d_cimg);
    p->timer.release();
    delete p;
    return AA_OK;
}

extern "C" int aa_fe_n_frames(const void* plan) {
    return plan ? static_cast<const FePlan*>(plan)->T : -1;
}

extern "C" size_t aa_fe_workspace_bytes(const void* plan, int32_t max_windows) {
    if (!plan || max_windows < 0) return 0;
    return fe_ws_layout(*static_cast<const FePlan*>(plan), max_windows, nullptr).bytes;
}

extern "C" int aa_fe_run(void* plan, const float* pcm, int64_t pcm_len, const aa_window* windows,
                         int32_t n_win, void* out, int32_t* win_status, void* workspace,
                         size_t workspace_bytes, void* stream) {
    FePlan* p = static_cast<FePlan*>(plan);
    AA_CHECK(p && pcm && windows && out, AA_ERR_INVALID, "aa_fe_run: null argument");
    AA_CHECK(n_win >= 0, AA_ERR_INVALID, "aa_fe_run: n_win < 0");
    (void)pcm_len;  // window views are validated by the host against pcm_len
    if (n_win == 0) return AA_OK;
    // the per-window grids carry the window in blockIdx.y (at most 65,535):
    // larger batches run as consecutive chunks through the same workspace
    constexpr int32_t CHUNK = 32768;
    if (n_win > CHUNK) {
        const size_t ob = (size_t)p->cfg.n_mels * p->T * p->cfg.channels * (p->cfg.out_f16 ? 2 : 4);
        for (int32_t c0 = 0; c0 < n_win; c0 += CHUNK) {
            const int32_t nc = std::min(CHUNK, n_win - c0);
            const int rc = aa_fe_run(plan, pcm, pcm_len, windows + c0, nc, static_cast<char*>(out) + c0 * ob,
                                     win_status ? win_status + c0 : nullptr, workspace, workspace_bytes, stream);
            if (rc != AA_OK) return rc;
        }
        return AA_OK;
    }
    FeWs ws = fe_ws_layout(*p, n_win, static_cast<char*>(workspace));
    AA_CHECK(workspace && workspace_bytes >= ws.bytes, AA_ERR_WORKSPACE,
             "aa_fe_run: workspace %zu < %zu bytes", workspace_bytes, ws.bytes);
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipEvent_t e0;
    int rc = p->timer.begin(FE_STAGE_STATS, st, &e0);
    if (rc != AA_OK) return rc;
    hipLaunchKernelGGL(fe_stats, dim3(kStatSplit, n_win), dim3(256), 0, st, pcm, windows,
                       p->cfg.win_len, ws.stats);
    AA_LAUNCH_CHECK();
    if ((rc = p->timer.end(FE_STAGE_STATS, st, e0)) != AA_OK) return rc;
    if ((rc = p->timer.begin(FE_STAGE_STFT, st, &e0)) != AA_OK) return rc;
    const int pm = p->cfg.power == 2.f ? PM_SQUARE : p->cfg.power == 1.f ? PM_ABS : PM_GENERAL;
#define AA_FE_PM(PM)                                                                                    \
    if (fe_fast4096(*p)) {                                                                              \
        rc = launch_stft4096<PM>(*p, pcm, windows, n_win, ws.stats, ws.melS, ws.blkmax, st);            \
    } else switch (p->cfg.n_fft) {                                                                      \
        case 2048: rc = launch_stft<2048, PM>(*p, pcm, windows, n_win, ws.stats, ws.melS, ws.blkmax, st); break; \
        case 4096: rc = launch_stft<4096, PM>(*p, pcm, windows, n_win, ws.stats, ws.melS, ws.blkmax, st); break; \
        default: rc = launch_stft<8192, PM>(*p, pcm, windows, n_win, ws.stats, ws.melS, ws.blkmax, st); break;   \
    }
    if (pm == PM_SQUARE) { AA_FE_PM(PM_SQUARE) }
    else if (pm == PM_ABS) { AA_FE_PM(PM_ABS) }
    else { AA_FE_PM(PM_GENERAL) }
#undef AA_FE_PM
    if (rc != AA_OK) return rc;
    if ((rc = p->timer.end(FE_STAGE_STFT, st, e0)) != AA_OK) return rc;
    if ((rc = p->timer.begin(FE_STAGE_DB, st, &e0)) != AA_OK) return rc;
    if (p->cfg.mean_sub) {
        hipLaunchKernelGGL(fe_band_mean, dim3(n_win), dim3(256), 0, st, ws.melS, ws.blkmax, p->nfblk,
                           p->cfg.n_mels, p->T, p->cfg.db_scale, p->cfg.amin, p->cfg.top_db, ws.band_mean);
        AA_LAUNCH_CHECK();
    }
#ifndef AA_FE_DB_TILE
#define AA_FE_DB_TILE 8
#endif
    static_assert((AA_FE_DB_TILE & (AA_FE_DB_TILE - 1)) == 0, "fe_db indexes its tile by shifts");
    int tile_t = AA_FE_DB_TILE;  // frames per fe_db block (the [tile_t][n_mels + 1] tile within 64 KiB)
    while (tile_t > 1 && (size_t)tile_t * (p->cfg.n_mels + 1) * 4 > 65536) tile_t >>= 1;
    if (p->cfg.out_f16) {
        hipLaunchKernelGGL(fe_db<_Float16>, dim3((p->T + tile_t - 1) / tile_t, n_win), dim3(256),
                           (size_t)tile_t * (p->cfg.n_mels + 1) * 4, st, ws.melS, ws.blkmax, p->nfblk, ws.stats,
                           p->cfg.mean_sub ? ws.band_mean : nullptr, p->cfg.n_mels, p->T, tile_t, p->cfg.db_scale,
                           p->cfg.amin, p->cfg.top_db, p->cfg.channels, p->cfg.normalize, (_Float16*)out, win_status);
    } else {
        hipLaunchKernelGGL(fe_db<float>, dim3((p->T + tile_t - 1) / tile_t, n_win), dim3(256),
                           (size_t)tile_t * (p->cfg.n_mels + 1) * 4, st, ws.melS, ws.blkmax, p->nfblk, ws.stats,
                           p->cfg.mean_sub ? ws.band_mean : nullptr, p->cfg.n_mels, p->T, tile_t, p->cfg.db_scale,
                           p->cfg.amin, p->cfg.top_db, p->cfg.channels, p->cfg.normalize, (float*)out, win_status);
    }
    AA_LAUNCH_CHECK();
    return p->timer.end(FE_STAGE_DB, st, e0);
}

extern "C" int aa_fe_n_stages(const void* plan) { return plan ? FE_N_STAGES : -1; }

// Algorithmic work of one window through each launch:
//   stft_mel flops = T (2.5 N log2 N + N + 3 (N/2 + 1) + 2 nnz) + 5 L
//   (real FFT as an N/2 complex FFT + split, window, |.|^p, mel rows; the
//   normalisation pass), bytes = L f32 PCM in + n_mels T f32 mel power out.
extern "C" int aa_fe_stage_info(const void* plan, int32_t stage, char* name, int32_t name_len,
                                double* flops_per_item, double* bytes_per_item) {
    const FePlan* p = static_cast<const FePlan*>(plan);
    AA_CHECK(p && stage >= 0 && stage < FE_N_STAGES, AA_ERR_INVALID, "aa_fe_stage_info: bad stage");
    const double N = p->cfg.n_fft, L = p->cfg.win_len, T = p->T, M = p->cfg.n_mels;
    double fl = 0, by = 0;
    const char* nm = "";
    switch (stage) {
        case FE_STAGE_STATS: nm = "fe_stats"; fl = 2 * L; by = 4 * L; break;
        case FE_STAGE_STFT:
            nm = fe_fast4096(*p) ? "fe_stft_mel_4096" : "fe_stft_mel";
            fl = T * (2.5 * N * std::log2(N) + N + 3 * (N / 2 + 1) + 2.0 * p->nnz) + 5 * L;
            by = 4 * L + 4 * M * T;
            break;
        default: nm = "fe_db"; fl = 3 * M * T; by = M * T * (4 + (p->cfg.out_f16 ? 2 : 4) * p->cfg.channels); break;
    }
    if (name && name_len > 0) snprintf(name, name_len, "%s", nm);
    if (flops_per_item) *flops_per_item = fl;
    if (bytes_per_item) *bytes_per_item = by;
    return AA_OK;
}

extern "C" int aa_fe_set_timing(void* plan, uint32_t stage_mask) {
    FePlan* p = static_cast<FePlan*>(plan);
    AA_CHECK(p, AA_ERR_INVALID, "aa_fe_set_timing: null plan");
    p->timer.mask = stage_mask;
    return AA_OK;
}

extern "C" int aa_fe_stage_time(void* plan, int32_t stage, double* total_ms, int64_t* count) {
    FePlan* p = static_cast<FePlan*>(plan);
    AA_CHECK(p && stage >= 0 && stage < FE_N_STAGES, AA_ERR_INVALID, "aa_fe_stage_time: bad stage");
    return p->timer.collect(stage, total_ms, count);
}
