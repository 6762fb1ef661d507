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
    char* d_cimg = nullptr;   // fe_stft_mel_4096 block constants (W4096^k | rows | values), 1-KiB padded
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
        for (int i = threadIdx.x; i < nb; i += blockDim.x) {
            float4 x = q[i];
            bad |= !isfinite(x.x) | !isfinite(x.y) | !isfinite(x.z) | !isfinite(x.w);
            mn = fminf(fminf(mn, x.x), fminf(x.y, fminf(x.z, x.w)));
            mx = fmaxf(fmaxf(mx, x.x), fmaxf(x.y, fmaxf(x.z, x.w)));
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

// ---------------------------------------------------------------------------
// radix building blocks (forward transform, W = exp(-2 pi i / n))
// ---------------------------------------------------------------------------
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_negi(float2 a) { return make_float2(a.y, -a.x); }  // a * (-i)

__device__ __forceinline__ void dft2(float2& a, float2& b) {
    float2 t = csub(a, b);
    a = cadd(a, b);
    b = t;
}
// in: a,b,c,d = x0..x3 ; out in natural order X0..X3
__device__ __forceinline__ void dft4(float2& a, float2& b, float2& c, float2& d) {
    float2 t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = mul_negi(csub(b, d));
    a = cadd(t0, t2);
    c = csub(t0, t2);
    b = cadd(t1, t3);
    d = csub(t1, t3);
}
__device__ __forceinline__ void dft8(float2* v) {
    const float r = 0.70710678118654752440f;
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    // twiddles W8^k, k = 0..3
    float2 w1 = make_float2(r * (o1.x + o1.y), r * (o1.y - o1.x));   // * (r, -r)
    float2 w2 = mul_negi(o2);                                       // * (0, -1)
    float2 w3 = make_float2(r * (o3.y - o3.x), -r * (o3.x + o3.y));  // * (-r, -r)
    v[0] = cadd(e0, o0);
    v[4] = csub(e0, o0);
    v[1] = cadd(e1, w1);
    v[5] = csub(e1, w1);
    v[2] = cadd(e2, w2);
    v[6] = csub(e2, w2);
    v[3] = cadd(e3, w3);
    v[7] = csub(e3, w3);
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

// complex64 -> np.abs (hypot) -> ** power.  The power mode is a template
// parameter: a runtime select between the three forms would make every bin
// pay for the inlined powf.
enum { PM_GENERAL = 0, PM_ABS = 1, PM_SQUARE = 2 };
template <int PM>
__device__ __forceinline__ float pow_mag(float re, float im, float power) {
    const float mag = sqrtf(re * re + im * im);
    if constexpr (PM == PM_SQUARE) return mag * mag;
    else if constexpr (PM == PM_ABS) return mag;
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
    for (int idx = tid; idx < n_mels * nf; idx += NT) {
        const int m = idx / nf, f = idx - (idx / nf) * nf;
        melS[((size_t)w * n_mels + m) * T + f0 + f] = melT[m * kFpb + f];
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
// fe_stft_mel_4096: the n_fft = 4096 path, one WAVE per frame.
//
// z[n] = x[2n] + i x[2n+1] (2048 complex points), four-step FFT with 64 lanes:
//   n = c + 64 r (lane c holds r = 0..31 in registers)
//   1. DFT-32 over r in registers                   -> Y[k1][c]
//   2. Y[k1][c] *= W2048^(c k1)                     (per-lane register twiddles)
//   3. transpose through a per-wave LDS buffer (two half passes, rows padded
//      to 66 float2 so both the row writes and the strided reads are
//      conflict-free): lane L = 2 k1 + h gets Y[k1][h + 2m], m = 0..31
//   4. DFT-32 over m in registers -> E_h[k2']
//   5. radix-2 across the lane pair (DPP quad_perm swap):
//      Z[k1 + 32 k2'] = E0 + W64^k2' E1, Z[k1 + 32 (k2' + 32)] = E0 - W64^k2' E1
//   6. real split X[k] = E + W4096^k O from Z[k], conj Z[2048 - k]
//   7. periodic Hann applied in frequency: Xw[k] = X[k]/2 - (X[k-1] + X[k+1])/4,
//      |Xw|^power into LDS
//   8. sparse mel rows (CSR in LDS) -> block staging tile -> melS
// Block = 4 waves = 4 consecutive frames of one window sharing one normalised
// PCM segment; 2 blocks per CU.  Only wave-level synchronisation inside a frame.
// ---------------------------------------------------------------------------
#include "aa_twiddles.h"

constexpr int kFpg = 4;                 // frames (waves) per block
constexpr int kRow = 66;                // padded transpose row (float2)
constexpr int kHalf = 16 * kRow;        // per-wave buffer (float2)
constexpr int kCimgRows = 1026 * 8;     // byte offset of the CSR rows in the constant image

// PCM segment of one block, rounded to whole 64-sample global_load_lds rows
__host__ __device__ constexpr int fe4096_seg_cap(int hop) { return ((kFpg - 1) * hop + 4096 + 63) & ~63; }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float2 wconst32(int k) { return make_float2(kW32[k][0], kW32[k][1]); }
__device__ __forceinline__ float2 wconst64(int k) { return make_float2(kW64[k][0], kW64[k][1]); }

// 32-point DFT in registers, in place: 4 interleaved DFT-8s, twiddles, DFT-4s.
// Output X[k] is left in v[dperm(k)], dperm(k) = 4 (k % 8) + k / 8 (a
// compile-time permutation, so no data moves).
__device__ __forceinline__ constexpr int dperm(int k) { return 4 * (k & 7) + (k >> 3); }
__device__ __forceinline__ void dft32(float2* v) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        float2 t[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) t[m] = v[4 * m + p];
        dft8(t);
#pragma unroll
        for (int m = 0; m < 8; ++m) v[4 * m + p] = t[m];
    }
#pragma unroll
    for (int p = 1; p < 4; ++p)
#pragma unroll
        for (int k = 1; k < 8; ++k) v[4 * k + p] = cmul(v[4 * k + p], wconst32(p * k));
#pragma unroll
    for (int k = 0; k < 8; ++k) dft4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
}

__device__ __forceinline__ float swap_pair(float x) {  // value of lane ^ 1
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));
}

// DIAG (tools/fe_bench.hip only): 1 skip the global->LDS staging, 2 the
// normalisation pass, 4 the FFT (steps 1-5), 8 the real split, 16 Hann and
// power, 32 the mel rows, 64 the output stores.
template <int PM, int DIAG = 0>
__global__ __launch_bounds__(256) void fe_stft_mel_4096(
    const float* __restrict__ pcm, const aa_window* __restrict__ wins, const float4* __restrict__ stats,
    const float2* __restrict__ tw, const char* __restrict__ cimg, int cimg_bytes, int win_len, int hop, int T,
    int n_mels, int kmin, int kmax, int normalize, float power, int ngrp, int n_items, float* __restrict__ melS,
    float* __restrict__ blkmax) {
    constexpr int NC = 2048;
    extern __shared__ float lds[];
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int seg_cap = fe4096_seg_cap(hop);
    float* seg = lds;
    float2* wb = reinterpret_cast<float2*>(seg + seg_cap) + wave * kHalf;  // this wave's buffer
    // block constants, one contiguous image (fe4096_cimg): W4096^k | CSR rows | CSR values
    char* cl = reinterpret_cast<char*>(reinterpret_cast<float2*>(seg + seg_cap) + kFpg * kHalf);
    const float2* stw2 = reinterpret_cast<const float2*>(cl);
    const int4* srows = reinterpret_cast<const int4*>(cl + kCimgRows);
    const float* svals = reinterpret_cast<const float*>(srows + n_mels);
    float* melT = reinterpret_cast<float*>(cl + cimg_bytes);  // [n_mels][kFpg]

    // ---- block prologue: every global read is issued before the first wait.
    // The constant image and the overlapped PCM segment go global -> LDS by
    // global_load_lds (no registers, no per-iteration waits); the window
    // descriptor is the only dependent round trip. ----
    for (int g = wave; g < ((DIAG & 1) ? 0 : cimg_bytes / 1024); g += kFpg)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(cimg + g * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(cl + g * 1024), 16, 0, 0);
    // step-2 twiddles W2048^(c k1) = (W^8c)^(k1/8) (W^c)^(k1%8): two short power
    // ladders from two table entries (<= 4 roundings per twiddle)
    float2 p1[8], p8[4];
    p1[0] = make_float2(1.f, 0.f);
    p1[1] = tw[lane];
    p8[0] = make_float2(1.f, 0.f);
    p8[1] = tw[(8 * lane) & (NC - 1)];

    const int k1 = lane >> 1, h = lane & 1;
    {
        // XCD-aware item order: block b runs on XCD b % 8, so XCD x takes the
        // contiguous item range [x q + min(x, r), ...) (q, r = n_items / 8, % 8).
        // Consecutive frame groups of a window overlap by 4096 - 4 hop samples
        // and write the same 128-B lines of melS; keeping them on one XCD lets
        // its L2 serve the overlap and merge the partial-line stores.
        const int xcd = blockIdx.x & 7, q = n_items >> 3, r = n_items & 7;
        const int item = xcd * q + min(xcd, r) + (blockIdx.x >> 3);
        const int w = item / ngrp;
        const int g = item - w * ngrp;
        const int f0 = g * kFpg;
        const int nf = min(kFpg, T - f0);
        const int seg_len = (nf - 1) * hop + 4096;
        const aa_window d = wins[w];
        const int base = f0 * hop - 2048;
        const long long safe = d.n_valid > 0 ? d.src : 0;
        // raw segment: lane q of wave-instruction gg loads sample base + q (a
        // clamped in-bounds address where the window has no sample; the
        // normalisation pass below rewrites those)
        for (int gg = wave; gg * 64 < ((DIAG & 1) ? 0 : seg_len); gg += kFpg) {
            const int q = gg * 64 + lane;
            const int i = base + q;
            const int rel = i - d.pad_left;
            const bool ok = q < seg_len && i >= 0 && i < win_len && rel >= 0 && rel < d.n_valid;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(pcm + (ok ? d.src + rel : safe)),
                                             (__attribute__((address_space(3))) void*)(seg + gg * 64), 4, 0, 0);
        }
        float lo = INFINITY, hi = -INFINITY;
#pragma unroll
        for (int s = 0; s < kStatSplit; ++s) {
            const float4 st = stats[w * kStatSplit + s];
            lo = fminf(lo, st.x);
            hi = fmaxf(hi, st.y);
        }
        const float scale = __fsub_rn(hi, lo);
        const float inv = __fdiv_rn(1.f, scale);
#pragma unroll
        for (int i = 2; i < 8; ++i) p1[i] = cmul(p1[i - 1], p1[1]);
        p8[2] = cmul(p8[1], p8[1]);
        p8[3] = cmul(p8[2], p8[1]);
        __syncthreads();  // vmcnt(0): segment and constants have landed
        // ---- normalise in place (np.pad zeros, centre padding stays 0) ----
        {
            constexpr int U = 8;
            for (int q0 = 0; q0 < ((DIAG & 2) ? 0 : seg_len); q0 += U * 256) {
                float v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) v[u] = seg[min(q0 + u * 256 + tid, seg_cap - 1)];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int q = q0 + u * 256 + tid;
                    const int i = base + q;
                    const int rel = i - d.pad_left;
                    if (q < seg_len) {
                        float x = 0.f;
                        if (i >= 0 && i < win_len) {
                            x = (rel >= 0 && rel < d.n_valid) ? v[u] : 0.f;
                            if (normalize) x = normalize_sample(x, lo, scale, inv);
                        }
                        seg[q] = x;
                    }
                }
            }
        }
        __syncthreads();
        float bmax = 0.f;
        if (wave < nf) {
            float2 u[32];
            if constexpr ((DIAG & 4) != 0) {
#pragma unroll
                for (int j = 0; j < 32; ++j) u[j] = make_float2((float)j, seg[lane + j]);
            } else {
            // ---- 1. load + DFT-32 over r ----
            float2 y[32];
            const float* x = seg + wave * hop + 2 * lane;
#pragma unroll
            for (int r = 0; r < 32; ++r) y[r] = make_float2(x[128 * r], x[128 * r + 1]);
            dft32(y);
            // ---- 2. twiddle ----
#pragma unroll
            for (int k = 1; k < 32; ++k) {
                const float2 t = (k & 7) == 0 ? p8[k >> 3] : (k < 8 ? p1[k] : cmul(p8[k >> 3], p1[k & 7]));
                y[dperm(k)] = cmul(y[dperm(k)], t);
            }
            // ---- 3. transpose in two halves ----
#pragma unroll
            for (int half = 0; half < 2; ++half) {
#pragma unroll
                for (int k = 0; k < 16; ++k) wb[k * kRow + lane] = y[dperm(half * 16 + k)];
                wave_sync();
                if ((lane >> 5) == half) {
                    const float2* src = wb + (k1 - 16 * half) * kRow + h;
#pragma unroll
                    for (int m = 0; m < 32; ++m) u[m] = src[2 * m];
                }
                wave_sync();
            }
            // ---- 4. DFT-32 over m ----
            dft32(u);
            // ---- 5. radix-2 across the lane pair ----
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                const float2 e = u[dperm(j)];
                const float2 o = make_float2(swap_pair(e.x), swap_pair(e.y));
                const float2 E0 = h ? o : e, E1 = h ? e : o;
                const float2 t = cmul(wconst64(j), E1);
                u[dperm(j)] = h ? csub(E0, t) : cadd(E0, t);
            }
            }
            // lane holds Z[k1 + 32 (32 h + j)] in u[dperm(j)]
            // ---- 6. real split ----
            if (h && !(DIAG & 8)) {
#pragma unroll
                for (int j = 0; j < 32; ++j) wb[k1 + 32 * j] = u[dperm(j)];  // Z[1024 + k1 + 32 j]
            }
            wave_sync();
            // h = 0 lanes: X[k], k = k1 + 32 j < 1024 (bands above NC/2 take the
            // generic kernel, see fe_fast4096)
            if (!h && !(DIAG & 8)) {
#pragma unroll
                for (int j = 0; j < 32; ++j) {
                    const int k = k1 + 32 * j;
                    const float2 a = u[dperm(j)];
                    const float2 zb = wb[k == 0 ? 0 : 1024 - k];
                    const float2 b = (k == 0) ? a : zb;  // Z[NC - k]
                    const float2 E = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
                    const float2 O = make_float2(0.5f * (a.y + b.y), -0.5f * (a.x - b.x));
                    const float2 t = cmul(stw2[k], O);
                    u[dperm(j)] = cadd(E, t);
                }
            }
            wave_sync();
            if (!h) {  // X[0..1023] in natural order (the host keeps 1 <= kmin, kmax <= 1022)
#pragma unroll
                for (int j = 0; j < 32; ++j) wb[k1 + 32 * j] = u[dperm(j)];
            }
            wave_sync();
            // ---- 7. Hann in frequency, |.|^power ----
            constexpr int PT = kHalf / 64 - 1;  // 15 bins per lane: nb <= 960 (host-checked)
            float pw[PT];
            const int nb = kmax - kmin + 1;
#pragma unroll
            for (int t = 0; t < ((DIAG & 16) ? 0 : PT); ++t) {
                const int k = min(kmin + lane + 64 * t, kmax);  // clamped: unconditional LDS reads
                const float2 c0 = wb[k], cm = wb[k - 1], cp = wb[k + 1];
                const float re = 0.5f * c0.x - 0.25f * (cm.x + cp.x);
                const float im = 0.5f * c0.y - 0.25f * (cm.y + cp.y);
                pw[t] = pow_mag<PM>(re, im, power);
            }
            wave_sync();
            float* P = reinterpret_cast<float*>(wb);
#pragma unroll
            for (int t = 0; t < ((DIAG & 16) ? 0 : PT); ++t)
                if (lane + 64 * t < nb) P[lane + 64 * t] = pw[t];
            wave_sync();
            // ---- 8. mel rows ----
            // rows of the constant image are zero-padded to whole float4s
            // (value offsets 16-B aligned); the padding adds exact zeros
            for (int m = lane; m < ((DIAG & 32) ? 0 : n_mels); m += 64) {
                const int4 rw = srows[m];
                const float4* wv = reinterpret_cast<const float4*>(svals + rw.z);
                const float* pv = P + (rw.x - kmin);
                float s = 0.f;
                for (int i = 0; i < rw.y; i += 4) {
                    const float4 a = wv[i >> 2];
                    s = fmaf(a.x, pv[i], s);
                    s = fmaf(a.y, pv[i + 1], s);
                    s = fmaf(a.z, pv[i + 2], s);
                    s = fmaf(a.w, pv[i + 3], s);
                }
                melT[m * kFpg + wave] = s;
                bmax = fmaxf(bmax, s);
            }
        }
        __syncthreads();
        for (int idx = tid; idx < ((DIAG & 64) ? 0 : n_mels * nf); idx += 256) {
            const int m = idx / nf, f = idx - (idx / nf) * nf;
            melS[((size_t)w * n_mels + m) * T + f0 + f] = melT[m * kFpg + f];
        }
        __shared__ float red[kFpg];
        bmax = wave_max(bmax);
        if (lane == 0) red[wave] = bmax;
        __syncthreads();
        if (tid == 0) {
            for (int k = 1; k < kFpg; ++k) bmax = fmaxf(bmax, red[k]);
            blkmax[w * ngrp + g] = bmax;
        }
    }
}

// ---------------------------------------------------------------------------
// fe_db: power_to_db(ref=max), clamp at -top_db, mean_sub, channel repeat.
// One wave per mel band row.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fe_db(const float* __restrict__ melS, const float* __restrict__ blkmax,
                                             const float4* __restrict__ stats, int nfblk, int n_mels, int T,
                                             int db_scale, float amin, float top_db, int mean_sub,
                                             int channels, int normalize, float* __restrict__ out,
                                             int* __restrict__ status) {
    const int w = blockIdx.y;
    float smax = 0.f;
    for (int i = 0; i < nfblk; ++i) smax = fmaxf(smax, blkmax[w * nfblk + i]);
    const float ref_db = __fmul_rn(10.0f, log10f(fmaxf(amin, smax)));
    const int lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (blockIdx.x == 0 && threadIdx.x == 0 && status) {
        float lo = INFINITY, hi = -INFINITY;
        int bad = 0;
        for (int s = 0; s < kStatSplit; ++s) {
            float4 st = stats[w * kStatSplit + s];
            lo = fminf(lo, st.x);
            hi = fmaxf(hi, st.y);
            bad |= st.z != 0.f;
        }
        // normalize_data divides by max(x - min): 0 -> NaN -> librosa raises
        if (normalize && !(hi - lo > 0.f)) bad = 1;
        status[w] = bad ? AA_WIN_NONFINITE : AA_WIN_OK;
    }
    if (m >= n_mels) return;
    const float* row = melS + ((size_t)w * n_mels + m) * T;
    auto val = [&](int t) {
        float v = row[t];
        if (db_scale) {
            v = __fsub_rn(__fmul_rn(10.0f, log10f(fmaxf(amin, v))), ref_db);
            v = fmaxf(v, -top_db);  // log_spec.max() == 0 exactly
        }
        return v;
    };
    float mean = 0.f;
    if (mean_sub) {
        float s = 0.f;
        for (int t = lane; t < T; t += 64) s += val(t);
        mean = wave_sum(s) / (float)T;
    }
    float* o = out + ((size_t)w * n_mels + m) * T * channels;
    for (int t = lane; t < T; t += 64) {
        const float v = val(t) - mean;
        for (int c = 0; c < channels; ++c) o[t * channels + c] = v;
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
    static size_t attr_set = 0;  // dynamic LDS opt-in already granted (static LDS comes on top)
    if (lds > attr_set) {
        AA_HIP(hipFuncSetAttribute((const void*)fe_stft_mel<NFFT, PM>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr_set = lds;
    }
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
    // kept band inside X[1..1022] (Hann neighbours in range), padded rows
    // (+3 bins) inside the 15 x 64 power slots
    return p.cfg.n_fft == 4096 && p.kmin >= 1 && p.kmax <= 1022 &&
           p.kmax - p.kmin + 1 + 3 <= (kHalf / 64 - 1) * 64;
}

static size_t fe_lds_bytes4096(const FePlan& p) {
    return sizeof(float) * (size_t)fe4096_seg_cap(p.cfg.hop) + sizeof(float2) * (size_t)kFpg * kHalf +
           (size_t)p.cimg_bytes + sizeof(float) * (size_t)p.cfg.n_mels * kFpg;
}

template <int PM>
static int launch_stft4096(const FePlan& p, const float* pcm, const aa_window* wins, int n_win,
                           const float4* stats, float* melS, float* blkmax, hipStream_t st) {
    const size_t lds = fe_lds_bytes4096(p);
    AA_CHECK(lds <= 150 * 1024, AA_ERR_UNSUPPORTED, "fe4096: hop %d needs %zu B of LDS", p.cfg.hop, lds);
    static size_t attr_set = 0;
    if (lds > attr_set) {
        AA_HIP(hipFuncSetAttribute((const void*)fe_stft_mel_4096<PM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds));
        attr_set = lds;
    }
    const int ngrp = p.nfblk;
    const int n_items = ngrp * n_win;
    hipLaunchKernelGGL(fe_stft_mel_4096<PM>, dim3(n_items), dim3(256), lds, st, pcm, wins, stats, p.d_tw, p.d_cimg,
                       p.cimg_bytes, p.cfg.win_len, p.cfg.hop, p.T, p.cfg.n_mels, p.kmin, p.kmax,
                       p.cfg.normalize, p.cfg.power, ngrp, n_items, melS, blkmax);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

struct FeWs {
    float4* stats;
    float* melS;
    float* blkmax;
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
    AA_CHECK(cfg->hop > 0 && cfg->win_len > 0 && cfg->n_mels > 0 && cfg->channels >= 1,
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
    p->nfblk = fe_fast4096(*p) ? (p->T + kFpg - 1) / kFpg : (p->T + kFpb - 1) / kFpb;
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
        // constant image of the wave-per-frame kernel, byte-identical to its LDS region
        // CSR rows zero-padded to whole float4s, value offsets 16-B aligned
        std::vector<int4> prow(rows.size());
        std::vector<float> pval;
        for (size_t m = 0; m < rows.size(); ++m) {
            const int len = (rows[m].y + 3) & ~3;
            prow[m] = make_int4(rows[m].x, len, (int)pval.size(), 0);
            for (int i = 0; i < len; ++i) pval.push_back(i < rows[m].y ? vals[rows[m].z + i] : 0.f);
        }
        const size_t raw = kCimgRows + sizeof(int4) * prow.size() + sizeof(float) * pval.size();
        std::vector<char> img((raw + 1023) / 1024 * 1024, 0);
        memcpy(img.data(), tw2.data(), sizeof(float2) * 1025);
        memcpy(img.data() + kCimgRows, prow.data(), sizeof(int4) * prow.size());
        memcpy(img.data() + kCimgRows + sizeof(int4) * prow.size(), pval.data(), sizeof(float) * pval.size());
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
                         int32_t n_win, float* out, int32_t* win_status, void* workspace,
                         size_t workspace_bytes, void* stream) {
    FePlan* p = static_cast<FePlan*>(plan);
    AA_CHECK(p && pcm && windows && out, AA_ERR_INVALID, "aa_fe_run: null argument");
    AA_CHECK(n_win >= 0, AA_ERR_INVALID, "aa_fe_run: n_win < 0");
    (void)pcm_len;  // window views are validated by the host against pcm_len
    if (n_win == 0) return AA_OK;
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
    hipLaunchKernelGGL(fe_db, dim3((p->cfg.n_mels + 3) / 4, n_win), dim3(256), 0, st, ws.melS,
                       ws.blkmax, ws.stats, p->nfblk, p->cfg.n_mels, p->T, p->cfg.db_scale,
                       p->cfg.amin, p->cfg.top_db, p->cfg.mean_sub, p->cfg.channels,
                       p->cfg.normalize, out, win_status);
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
        default: nm = "fe_db"; fl = 3 * M * T; by = 4 * M * T * (1 + p->cfg.channels); break;
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
