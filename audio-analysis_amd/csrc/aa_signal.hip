// Signal detector of classify() for gfx950: signal_noise
// (reference src/identify_tracks.py:650-706), run on every recording (:420).
//
// Launches (one stream, no host synchronisation inside aa_sn_run):
//   sn_zero       the per-run counters (global max, run count, status) = 0
//   sn_stft64     |STFT| of the recording (n_fft 4096, centre zero padding,
//                 scipy's periodic Hann) in librosa's own precision: f64
//                 window x f32 frame, an f64 FFT (128 threads per frame,
//                 radix 16 x 16 x 8 through LDS, real split in registers),
//                 rounded to complex64 and np.abs'd with numpy's f32 formula,
//                 so S is the reference's S.  Writes the frame-major S[f][0..2048],
//                 the maximum, and the frame's median over bins (block radix
//                 select on the bit patterns)
//   sn_transpose  S -> ST[bin][frame] (64 x 64 tiles through LDS), and the
//                 frame thresholds c3 = 3 (colmed / a) (numpy's f32 steps)
//   sn_select     per-bin median over frames: radix select over the ST row
//                 (staged in LDS), both middle elements for an even count;
//                 then the row's threshold r3 = 3 rowmed / a and its mask bits
//                 (S/a > c3) & (S/a > r3) (:656-669) from the staged row,
//                 bit-packed along time by ballot
//   sn_morph      cv2 erode / dilate with a rectangle (:670-684): the
//                 vertical reduction of three neighbouring 64-frame words,
//                 then the horizontal one on the reduced words (a rectangle
//                 is separable and the two orders give the same bits), one
//                 launch per structuring element
//   sn_runs, sn_unite, sn_stats, sn_emit
//                 8-connected components over row runs (:686): union-find with
//                 atomicMin hooking, bounding box, area and OpenCV's label-order
//                 key per root, the size filter (:689-691), a compact list of
//                 kept components for the host (a few entries per recording).
#include "aa_common.h"
#include "aa_wavefft.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <climits>
#include <cmath>
#include <type_traits>

namespace aa {

constexpr int kSnBins = 2049;  // n_fft / 2 + 1
constexpr int kSnLd = 2080;    // S row stride in floats (128-B aligned rows)
constexpr int kSnHist = 256;   // radix-select buckets (8 bits per pass)
constexpr int kSnFields = 10;  // run table: x0 x1 y parent left right top bottom area key
enum { R_X0 = 0, R_X1, R_Y, R_P, R_LEFT, R_RIGHT, R_TOP, R_BOT, R_AREA, R_KEY };

// A batch of recordings for the launches that run once per batch (the
// counters, morphology and components): their frame counts, passed by value;
// recording k's buffers sit k * pf bytes after recording 0's (blockIdx.z or
// .y = k).
// launch stages (aa_sn_stage_*): per recording stft / transpose / select,
// per batch the four morphology launches and the component launches
enum { SN_STAGE_STFT = 0, SN_STAGE_TRANSPOSE, SN_STAGE_SELECT, SN_STAGE_MORPH, SN_STAGE_COMPONENTS, SN_STAGE_COLMED,
       SN_N_STAGES };
constexpr int kSnMaxBatch = 64;
struct SnBatch {
    int n;
    int nf[kSnMaxBatch];
};
template <typename T>
__host__ __device__ __forceinline__ T* sn_at(T* p, size_t pf, int k) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(const_cast<std::remove_const_t<T>*>(p)) + pf * k);
}

struct SnPlan {
    aa_sn_config cfg;
    int kh_d = 0, kw_d = 0;  // cv2.dilate(ones((height, width))) (:683)
    int kh_e = 0, kw_e = 0;  // cv2.erode(ones((height // 10, width))) (:684)
    int wmin = 0, hmin = 0;  // kept: width >= wmin, height >= hmin (:689-691)
    double2* d_tab = nullptr;  // sn_stft64's tables (kS64Tab*)
    StageTimer timer;          // HIP events around the launches of the stages in timer.mask
    bool tw_chain = true;      // sn_stft64's twiddle ladders from 7 table values (AA_SN_TW=table: all 22;
                               // 99 -> 94.5 us per 60 s clip, S bit-identical on the tests' clips)
};

__device__ __forceinline__ unsigned wave_incl_scan(unsigned v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// One histogram increment per active lane, wave-aggregated: the lanes that
// share the first active lane's bucket add their count with ONE atomic, the
// rest add one each.  A row of near-equal magnitudes (a quiet band: every
// value in one or two buckets, pass after pass) otherwise serialises 64 LDS
// atomics on one address per wave-instruction.
__device__ __forceinline__ void hist_add(unsigned* H, unsigned b, bool act) {
    const unsigned long long m = __ballot(act);
    if (m == 0) return;  // wave-uniform
    const int leader = __builtin_ctzll(m);
    const unsigned bl = __builtin_amdgcn_readlane(b, leader);
    const bool same = act && b == bl;
    const unsigned long long ms = __ballot(same);
    if ((threadIdx.x & 63) == leader) atomicAdd(&H[bl], (unsigned)__popcll(ms));
    if (act && !same) atomicAdd(&H[b], 1u);
}

// sn_zero: the counters a run accumulates into (atomicMax / atomicAdd), one
// launch for every recording of the batch instead of a memset per buffer
__global__ void sn_zero(unsigned* __restrict__ gmax, int* __restrict__ counters, size_t pf, int32_t* __restrict__ n_out,
                        int n_out_stride) {
    const int i = threadIdx.x, k = blockIdx.x;
    if (gmax && i < 16) sn_at(gmax, pf, k)[i] = 0u;
    if (i < 16) sn_at(counters, pf, k)[i] = 0;
    if (i < 2) n_out[(size_t)k * n_out_stride + i] = 0;
}

// ---------------------------------------------------------------------------
// signal_noise's |STFT| in the reference's own precision.  librosa 0.11 forms
// each frame as the f64 Hann window times the f32 samples, transforms it with
// numpy's f64 rfft and stores the result as complex64; np.abs of that array
// (numpy's SIMD complex absolute value, loops_unary_complex) is
// L * sqrtf(fmaf(r, r, 1)) with L = max(|re|, |im|), r = min / L, every step
// a correctly rounded f32 operation.  sn_stft64 does the same: the transform
// in f64 (its result agrees with pocketfft's to ~1e-16 relative, so the
// complex64 rounding of the two agree except on values within that distance
// of a rounding midpoint), then the f64 -> f32 rounding and numpy's
// magnitude formula bit for bit.  That makes S -- and the medians, the mask
// and the components built on it -- the reference's values, not an f32
// approximation of them.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double2 dadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 dsub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 dmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 dnegi(double2 a) { return make_double2(a.y, -a.x); }  // a * (-i)

constexpr double kCos8 = 0.92387953251128675613;  // cos(pi / 8)
constexpr double kSin8 = 0.38268343236508977173;  // sin(pi / 8)
constexpr double kRt2 = 0.70710678118654752440;   // sqrt(1 / 2)

// a * W16^E, W16 = exp(-2 pi i / 16), for the exponents a DFT-16 and the
// real split need (E in 0..9)
template <int E>
__device__ __forceinline__ double2 w16(double2 a) {
    static_assert(E >= 0 && E <= 9, "w16");
    if constexpr (E == 0) return a;
    else if constexpr (E == 1) return make_double2(a.x * kCos8 + a.y * kSin8, a.y * kCos8 - a.x * kSin8);
    else if constexpr (E == 2) return make_double2(kRt2 * (a.x + a.y), kRt2 * (a.y - a.x));
    else if constexpr (E == 3) return make_double2(a.x * kSin8 + a.y * kCos8, a.y * kSin8 - a.x * kCos8);
    else if constexpr (E == 4) return dnegi(a);
    else if constexpr (E == 5) return make_double2(a.y * kCos8 - a.x * kSin8, -(a.x * kCos8 + a.y * kSin8));
    else if constexpr (E == 6) return make_double2(kRt2 * (a.y - a.x), -kRt2 * (a.x + a.y));
    else if constexpr (E == 7) return make_double2(a.y * kSin8 - a.x * kCos8, -(a.x * kSin8 + a.y * kCos8));
    else if constexpr (E == 8) return make_double2(-a.x, -a.y);
    else return make_double2(-(a.x * kCos8 + a.y * kSin8), a.x * kSin8 - a.y * kCos8);  // E == 9
}

__device__ __forceinline__ void ddft4(double2& a, double2& b, double2& c, double2& d) {  // natural order out
    const double2 t0 = dadd(a, c), t1 = dsub(a, c), t2 = dadd(b, d), t3 = dnegi(dsub(b, d));
    a = dadd(t0, t2);
    c = dsub(t0, t2);
    b = dadd(t1, t3);
    d = dsub(t1, t3);
}
__device__ __forceinline__ void ddft8(double2 (&v)[8]) {  // natural order out
    double2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    double2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    ddft4(e0, e1, e2, e3);
    ddft4(o0, o1, o2, o3);
    o1 = w16<2>(o1);
    o2 = w16<4>(o2);
    o3 = w16<6>(o3);
    v[0] = dadd(e0, o0);
    v[4] = dsub(e0, o0);
    v[1] = dadd(e1, o1);
    v[5] = dsub(e1, o1);
    v[2] = dadd(e2, o2);
    v[6] = dsub(e2, o2);
    v[3] = dadd(e3, o3);
    v[7] = dsub(e3, o3);
}
// 16-point DFT in place (radix 4 x 4): X[k] is left in v[dp16(k)]
__device__ __forceinline__ constexpr int dp16(int k) { return 4 * (k & 3) + (k >> 2); }
__device__ __forceinline__ void ddft16(double2 (&v)[16]) {
#pragma unroll
    for (int b = 0; b < 4; ++b) ddft4(v[b], v[4 + b], v[8 + b], v[12 + b]);  // v[4c + b] = Y_b[c]
    v[5] = w16<1>(v[5]);
    v[9] = w16<2>(v[9]);
    v[13] = w16<3>(v[13]);
    v[6] = w16<2>(v[6]);
    v[10] = w16<4>(v[10]);
    v[14] = w16<6>(v[14]);
    v[7] = w16<3>(v[7]);
    v[11] = w16<6>(v[11]);
    v[15] = w16<9>(v[15]);
#pragma unroll
    for (int c = 0; c < 4; ++c) ddft4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);  // v[4c + d] = X[c + 4d]
}

// sqrtf correctly rounded for x in [1, 2]: v_sqrt_f32 (within 1 ulp), then
// the neighbour whose residual brackets x -- the IEEE sqrt sequence the
// compiler emits, without its denormal scaling and special-value checks
// (fmaf(r, r, 1) of a ratio r in [0, 1] is always in range)
__device__ __forceinline__ float sqrt_rn_1_2(float x) {
    float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = fmaf(-sd, s, x), ru = fmaf(-su, s, x);
    s = rd <= 0.f ? sd : s;
    s = ru > 0.f ? su : s;
    return s;
}

// np.abs of one complex64 value, numpy's SIMD formula (non-finite parts give
// a NaN / inf magnitude, which the host reports as non-finite input)
__device__ __forceinline__ float np_cabsf(double re64, double im64) {
    const float re = (float)re64, im = (float)im64;  // complex128 -> complex64 (round to nearest)
    const float x = fabsf(re), y = fabsf(im);
    const float L = fmaxf(x, y), s = fminf(x, y);
    const float r = (L == 0.f || s == __builtin_huge_valf()) ? 0.f : s / L;  // correctly rounded
    float m = sqrt_rn_1_2(fmaf(r, r, 1.f)) * L;
    if (re != re || im != im) m = __builtin_nanf("");
    return m;
}

// The bucket of a 256-bucket histogram that holds `rank` (0-based), found by
// one wave; c: the lane's buckets 4 lane .. 4 lane + 3.  *below: elements in
// lower buckets; *cnt: elements in the bucket.
__device__ __forceinline__ unsigned hist_pick4(uint4 c, unsigned rank, int lane, unsigned* below, unsigned* cnt) {
    const unsigned s = c.x + c.y + c.z + c.w;
    const unsigned incl = wave_incl_scan(s, lane);
    const unsigned excl = incl - s;
    const bool mine = excl <= rank && rank < incl;
    unsigned dig = 0, bl = 0, cn = 0;
    if (mine) {
        const unsigned r = rank - excl;
        if (r < c.x) { dig = 0; bl = 0; cn = c.x; }
        else if (r < c.x + c.y) { dig = 1; bl = c.x; cn = c.y; }
        else if (r < c.x + c.y + c.z) { dig = 2; bl = c.x + c.y; cn = c.z; }
        else { dig = 3; bl = c.x + c.y + c.z; cn = c.w; }
        dig += 4 * lane;
        bl += excl;
    }
    const int src = __builtin_ctzll(__ballot(mine));
    *below = __shfl(bl, src, 64);
    *cnt = __shfl(cn, src, 64);
    return __shfl(dig, src, 64);
}
__device__ __forceinline__ unsigned hist_pick(const unsigned* hist, unsigned rank, int lane, unsigned* below,
                                              unsigned* cnt) {
    return hist_pick4(reinterpret_cast<const uint4*>(hist)[lane], rank, lane, below, cnt);
}

// sn_stft64 geometry: 128 threads per frame; the 2048 complex points z[n] =
// x[2n] + i x[2n + 1] of the 4096-sample real frame, n = 128 n1 + 8 n2 + n3,
// bins k = k1 + 16 k2 + 256 k3, m = k1 + 16 k2:
//   1. thread (n2, n3): DFT-16 over n1, twiddle W256^(n2 k1)
//   2. thread (k1, n3): DFT-16 over n2 (the remaining twiddle W2048^(n3 m)
//      moves to step 3, where it is per-column)
//   3. thread j owns columns m = j and 256 - j (thread 0: 0 and 128):
//      twiddle W2048^(n3 m), DFT-8 over n3 gives Z[m + 256 k3].  The second
//      column's twiddle is W8^n3 conj(W2048^(n3 j)), and a W8^n3 factor on a
//      DFT-8's input shifts its output by one bin, so both columns use the same
//      7 twiddles.  Z[2048 - k] of every k the thread holds sits in its other
//      column, so the real split needs no exchange:
//      X[k] = E + W4096^k O, X[2048 - k] = conj(E - W4096^k O),
//      E = (Z[k] + conj Z[2048 - k]) / 2, O = -i (Z[k] - conj Z[2048 - k]) / 2.
// The step-1 twiddles depend on n2 only (a wave-instruction reads 8 distinct
// table entries), the step-3 ones on the thread: 7 x 16 B per thread and
// frame from L2, the window stays in registers.
// LDS: one 36,864-B buffer holds each exchange in turn (step-1 rows of 136
// double2 per k1, step-2 columns of 9 double2: both read conflict-free by
// ds_read_b128), then the frame's 2049 magnitudes.
// AA_SN_WIN_REG: the window in 64 VGPRs across frames (1) or read from L2
// per frame (0)
#ifndef AA_SN_WIN_REG
#define AA_SN_WIN_REG 0
#endif
constexpr int kS64T = 128;
constexpr int kS64R1 = 136;
constexpr int kS64C2 = 9;
constexpr int kS64Buf = 256 * kS64C2;  // double2
constexpr int kS64Mag = 64;            // float offset of the magnitudes (after column 0's 8 double2)
// SnPlan::d_tab: window pairs [2048] | tw1 [15][16] | tw3 [7][128] | split bases [128]
constexpr int kS64TabTw1 = 2048, kS64TabTw3 = kS64TabTw1 + 15 * 16, kS64TabTwS = kS64TabTw3 + 7 * kS64T,
              kS64TabN = kS64TabTwS + kS64T;
static_assert(16 * kS64R1 <= kS64Buf && (kS64Mag + 2049) * 4 <= kS64Buf * 16, "sn_stft64 LDS");

// sn_stft64: persistent blocks, XCD x (block b on XCD b % 8) owning frames
// [x F / 8, (x + 1) F / 8) (neighbouring frames share 4096 - hop samples
// through one L2).  Per frame: its S row (stride ld) and the running maximum
// (gmax: atomicMax on the bit patterns, may be null).  win2: the f64 Hann
// window (halved) as pairs (w[2n], w[2n + 1]); tw1: W256^(n2 k1) [k1 - 1][n2];
// tw3: W2048^(n3 j) [n3 - 1][j]; twS: W4096^t (thread 0: W4096^128), the
// split's per-thread base.
__device__ unsigned wave_median_2049(const unsigned (&v)[33], unsigned* hists, int lane);

// TWC (default; AA_SN_TW=table for all table values): per frame only W^1, W^2, W^4 (W^8) of each twiddle
// ladder come from the tables (L2); the other powers are their products in
// f64 (<= 3 roundings of 2^-53: the f32 magnitudes can move only on rounding
// ties, as between any two f64 FFT factorisations), so 7 instead of 22 table
// loads of 16 B per thread and frame
template <bool TWC>
__global__ __launch_bounds__(kS64T) __attribute__((amdgpu_waves_per_eu(2, 2))) void sn_stft64(
    const float* __restrict__ pcm, int n_samples, int hop, int n_frames, const double2* __restrict__ win2,
    const double2* __restrict__ tw1, const double2* __restrict__ tw3, const double2* __restrict__ twS,
    float* __restrict__ S, int ld, unsigned* __restrict__ gmax) {
    __shared__ double2 buf[kS64Buf];
    const int t = threadIdx.x;
    const bool z = t == 0;
    // the recording as a buffer view: centre padding and the ends read as 0
    // (a negative offset wraps past num_records)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)pcm, 0, n_samples * 4, 0x00020000);
#if AA_SN_WIN_REG
    double2 wv[16];  // the thread's window pairs, the same in every frame
#pragma unroll
    for (int n1 = 0; n1 < 16; ++n1) wv[n1] = win2[128 * n1 + t];
#endif
    const double2 tb = twS[t];
    const int n2a = t >> 3;                 // step 1
    const int k1b = t >> 3, n3b = t & 7;    // step 2
    // step 3 columns: j and 256 - j; thread 0: 0 and 128
    const int m1 = t, m2 = z ? 128 : 256 - t;
    float* mag = reinterpret_cast<float*>(buf) + kS64Mag;
    unsigned wmax = 0;
    const int nbx = gridDim.x >> 3;  // blocks per XCD (grid a multiple of 8)
    const int xcd = blockIdx.x & 7;
    const int f_end = (int)((long long)(xcd + 1) * n_frames / 8);
#pragma unroll 1
    for (int fi = (int)((long long)xcd * n_frames / 8) + (blockIdx.x >> 3); fi < f_end; fi += nbx) {
        // the twiddle tables are loop-invariant: opaque indices per frame keep
        // the compiler from hoisting their loads into live registers
        int i1 = n2a, i3 = t;
        __asm__ volatile("" : "+v"(i1), "+v"(i3));
#if !AA_SN_WIN_REG
        int iw = t;  // the window from L2 every frame (16 x 1 KiB per wave, coalesced)
        __asm__ volatile("" : "+v"(iw));
#endif
        double2 v[16];
        {
            const int off = fi * hop - 2048 + 2 * t;
            // the odd sample's offset in a register of its own: two adjacent
            // dword loads merged into one dwordx2 would be range-checked as a
            // unit, so the view's first / last sample would read as 0 / garbage
            int offo = off + 1;
            __asm__ volatile("" : "+v"(offo));
#pragma unroll
            for (int n1 = 0; n1 < 16; ++n1) {
                const float xe = load_view(rs, off + 256 * n1), xo = load_view(rs, offo + 256 * n1);
#if AA_SN_WIN_REG
                const double2 w = wv[n1];
#else
                const double2 w = win2[128 * n1 + iw];
#endif
                v[n1] = make_double2((double)xe * w.x, (double)xo * w.y);
            }
        }
        // ---- 1. DFT-16 over n1, twiddle, rows k1 ----
        if constexpr (TWC) {
            double2 w[16];
            w[1] = tw1[0 * 16 + i1];
            w[2] = tw1[1 * 16 + i1];
            w[4] = tw1[3 * 16 + i1];
            w[8] = tw1[7 * 16 + i1];
            ddft16(v);
            w[3] = dmul(w[2], w[1]);
            w[5] = dmul(w[4], w[1]);
            w[6] = dmul(w[4], w[2]);
            w[7] = dmul(w[4], w[3]);
#pragma unroll
            for (int k = 9; k < 16; ++k) w[k] = dmul(w[8], w[k - 8]);
#pragma unroll
            for (int k1 = 1; k1 < 16; ++k1) v[dp16(k1)] = dmul(v[dp16(k1)], w[k1]);
        } else {
            ddft16(v);
#pragma unroll
            for (int k1 = 1; k1 < 16; ++k1) v[dp16(k1)] = dmul(v[dp16(k1)], tw1[(k1 - 1) * 16 + i1]);
        }
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) buf[k1 * kS64R1 + t] = v[dp16(k1)];
        __syncthreads();
        // ---- 2. DFT-16 over n2, columns m = k1 + 16 k2 ----
#pragma unroll
        for (int n2 = 0; n2 < 16; ++n2) v[n2] = buf[k1b * kS64R1 + 8 * n2 + n3b];
        ddft16(v);
        __syncthreads();
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) buf[(k1b + 16 * k2) * kS64C2 + n3b] = v[dp16(k2)];
        __syncthreads();
        // ---- 3. twiddle and DFT-8 over n3 of the thread's two columns ----
        double2 c1[8], y2[8];
#pragma unroll
        for (int n3 = 0; n3 < 8; ++n3) {
            c1[n3] = buf[m1 * kS64C2 + n3];
            y2[n3] = buf[m2 * kS64C2 + n3];
        }
        __syncthreads();  // the buffer takes the magnitudes next
        // W16^n = (cos, -sin)(2 pi n / 16), n < 8
        constexpr double kW16r[8] = {1.0, kCos8, kRt2, kSin8, 0.0, -kSin8, -kRt2, -kCos8};
        constexpr double kW16i[8] = {0.0, -kSin8, -kRt2, -kCos8, -1.0, -kCos8, -kRt2, -kSin8};
        double2 w3c[8];
        if constexpr (TWC) {
            w3c[1] = tw3[0 * kS64T + i3];
            w3c[2] = tw3[1 * kS64T + i3];
            w3c[4] = tw3[3 * kS64T + i3];
            w3c[3] = dmul(w3c[2], w3c[1]);
            w3c[5] = dmul(w3c[4], w3c[1]);
            w3c[6] = dmul(w3c[4], w3c[2]);
            w3c[7] = dmul(w3c[4], w3c[3]);
        }
#pragma unroll
        for (int n3 = 1; n3 < 8; ++n3) {
            const double2 w = TWC ? w3c[n3] : tw3[(n3 - 1) * kS64T + i3];  // W2048^(n3 j)
            // thread 0's second column (128) takes W16^n3 = W8^n3 conj(W16^n3):
            // the same shift by one bin, times conj(W16^n3)
            const double2 b2 = z ? make_double2(kW16r[n3], kW16i[n3]) : w;
            c1[n3] = dmul(c1[n3], w);
            y2[n3] = dmul(y2[n3], make_double2(b2.x, -b2.y));
        }
        ddft8(c1);
        ddft8(y2);
        double2 c2[8];  // the second column: Z[m2 + 256 k] = y2[(k + 1) % 8]
#pragma unroll
        for (int k = 0; k < 8; ++k) c2[k] = y2[(k + 1) & 7];
        // ---- real split and magnitudes into the buffer (the window carries
        // the split's factor 1/2: Z here is half the transform of z).  Slot s
        // of thread j pairs a = Z[j + 256 s] with b = Z[2048 - j - 256 s]
        // (column 256 - j, entry 7 - s): X[k] = E + W4096^k O, X[2048 - k] =
        // conj(E - W4096^k O), E = a + conj b, O = -i (a - conj b).  Thread 0
        // re-seats its registers so the same slots pair column 128 with itself
        // (slots 0-3: bins 128 + 256 s) and column 0 with itself (slots 4-7:
        // bins 256 (s - 3)); Z[0] gives the DC and Nyquist bins. ----
        const double2 z0 = c1[0];
        if (z) {  // per-lane selects (no branch: one lane of one wave)
            const double2 a4 = c1[1], a5 = c1[2], a6 = c1[3], a7 = c1[4];
            const double2 b0 = c1[4], b1 = c1[5], b2 = c1[6], b3 = c1[7];
            c1[0] = c2[0];
            c1[1] = c2[1];
            c1[2] = c2[2];
            c1[3] = c2[3];
            c1[4] = a4;
            c1[5] = a5;
            c1[6] = a6;
            c1[7] = a7;
            c2[0] = b0;
            c2[1] = b1;
            c2[2] = b2;
            c2[3] = b3;
        }
        auto split = [&](double2 a, double2 b, double2 w, int ka) {
            const double2 E = make_double2(a.x + b.x, a.y - b.y);
            const double2 O = make_double2(a.y + b.y, b.x - a.x);
            const double2 q = dmul(w, O);
            mag[ka] = np_cabsf(E.x + q.x, E.y + q.y);
            mag[2048 - ka] = np_cabsf(E.x - q.x, q.y - E.y);
        };
        const int mA = z ? 128 : t;
        split(c1[0], c2[7], tb, mA);
        split(c1[1], c2[6], w16<1>(tb), mA + 256);
        split(c1[2], c2[5], w16<2>(tb), mA + 512);
        split(c1[3], c2[4], w16<3>(tb), mA + 768);
        split(c1[4], c2[3], z ? make_double2(kCos8, -kSin8) : w16<4>(tb), z ? 256 : t + 1024);
        split(c1[5], c2[2], z ? make_double2(kRt2, -kRt2) : w16<5>(tb), z ? 512 : t + 1280);
        split(c1[6], c2[1], z ? make_double2(kSin8, -kCos8) : w16<6>(tb), z ? 768 : t + 1536);
        split(c1[7], c2[0], z ? make_double2(0.0, -1.0) : w16<7>(tb), z ? 1024 : t + 1792);
        if (z) {  // rfft's DC and Nyquist bins: real
            mag[0] = fabsf((float)(2.0 * (z0.x + z0.y)));
            mag[2048] = fabsf((float)(2.0 * (z0.x - z0.y)));
        }
        __syncthreads();
        // ---- the frame's row of S and its maximum ----
        float* srow = S + (size_t)fi * ld;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float m = mag[t + 128 * i];
            srow[t + 128 * i] = m;
            // bit patterns of non-negative floats order like the values (NaN
            // and inf above every finite value: the host reads that as
            // non-finite input)
            wmax = max(wmax, __float_as_uint(m));
        }
        if (z) {
            const float m = mag[2048];
            srow[2048] = m;
            wmax = max(wmax, __float_as_uint(m));
        }
        __syncthreads();  // the buffer is rewritten by the next frame
    }
    if (gmax) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (unsigned)__shfl_xor((int)wmax, o, 64));
        if ((t & 63) == 0 && wmax) atomicMax(gmax, wmax);
    }
}


// ---------------------------------------------------------------------------
// The median over bins of one frame (numpy, odd count 2049: the middle
// element) by radix select on the bit patterns, by the wave that holds the
// frame: v[i] = bin lane + 64 i (i < 32), v[32] = bin 2048 (lane 0 only).
// 8-bit digits start below the bits the frame's min and max share (a
// spectrum spans a few binades: the first histogram then spreads over the
// exponents present instead of piling onto a handful of counters), counted
// in 4 LDS histogram copies (lane & 3 picks one: a frame's values crowd a
// few buckets, and same-address LDS atomics serialise).  hists: the wave's
// 4 x 256 unsigned.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned wave_median_2049(const unsigned (&v)[33], unsigned* hists, int lane) {
    unsigned* myh = hists + (lane & 3) * kSnHist;
    unsigned mn = v[0], mx = v[0];
#pragma unroll
    for (int i = 1; i < 32; ++i) {
        mn = min(mn, v[i]);
        mx = max(mx, v[i]);
    }
    if (lane == 0) {
        mn = min(mn, v[32]);
        mx = max(mx, v[32]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
        mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    }
    if (mn == mx) return mn;
    const int hb = 31 - __clz(mn ^ mx);
    unsigned pmask = hb == 31 ? 0u : (0xFFFFFFFFu << (hb + 1));
    unsigned prefix = mn & pmask, rank = kSnBins / 2;
#pragma unroll 1
    for (int sh = hb - 7;; sh -= 8) {
        const int shift = max(sh, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) reinterpret_cast<uint4*>(hists + q * kSnHist)[lane] = make_uint4(0u, 0u, 0u, 0u);
        wave_sync();
#pragma unroll
        for (int i = 0; i < 33; ++i)
            hist_add(myh, (v[i] >> shift) & 255u, (i < 32 || lane == 0) && (v[i] & pmask) == prefix);
        wave_sync();
        {  // fold the copies into copy 0 (lane owns buckets 4 lane .. 4 lane + 3)
            uint4 t = reinterpret_cast<uint4*>(hists)[lane];
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                const uint4 u = reinterpret_cast<uint4*>(hists + q * kSnHist)[lane];
                t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
            }
            reinterpret_cast<uint4*>(hists)[lane] = t;
        }
        wave_sync();
        unsigned below, cnt;
        const unsigned dig = hist_pick(hists, rank, lane, &below, &cnt);
        prefix = (prefix & ~(255u << shift)) | (dig << shift);
        pmask |= 255u << shift;
        rank -= below;
        wave_sync();
        if (shift == 0) break;
    }
    return prefix;
}


// sn_colmed: one wave per frame, the frame's S row (2049 floats, just
// written by sn_stft64: L2 / Infinity-Cache resident) into registers, its
// median over bins into colmed[f].  Four frames per 256-thread block, 4 KiB
// of histograms per wave.
__global__ __launch_bounds__(256) void sn_colmed(const float* __restrict__ S, int ld, int n_frames,
                                                 unsigned* __restrict__ colmed) {
    __shared__ unsigned hists[4][4 * kSnHist];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int f = blockIdx.x * 4 + wave;
    if (f >= n_frames) return;  // wave-uniform; no block barrier below
    const unsigned* row = reinterpret_cast<const unsigned*>(S) + (size_t)f * ld;
    unsigned v[33];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = row[lane + 64 * i];
    v[32] = lane == 0 ? row[2048] : 0u;
    const unsigned med = wave_median_2049(v, hists[wave], lane);
    if (lane == 0) colmed[f] = med;
}

// ---------------------------------------------------------------------------
// sn_transpose: S[f][b] (stride kSnLd) -> ST[b][f] (stride ldt)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sn_transpose(const float* __restrict__ S, int n_frames, int ldt,
                                                    float* __restrict__ ST, const unsigned* __restrict__ gmax,
                                                    const unsigned* __restrict__ colmed, float* __restrict__ c3) {
    __shared__ float tile[64][65];
    const int b0 = blockIdx.x * 64, f0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    // the first bin tile also forms its frames' thresholds c3 = 3 * (colmed /
    // a) in numpy's float32 steps (:656-667); division is monotone, so the
    // median of S / a is the quotient of S's middle element
    if (blockIdx.x == 0 && ty == 0 && f0 + tx < n_frames)
        c3[f0 + tx] = __fmul_rn(3.f, __fdiv_rn(__uint_as_float(colmed[f0 + tx]), __uint_as_float(*gmax)));
#pragma unroll 4
    for (int r = ty; r < 64; r += 4) {
        const int f = f0 + r, b = b0 + tx;
        tile[r][tx] = (f < n_frames && b < kSnBins) ? S[(size_t)f * kSnLd + b] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int r = ty; r < 64; r += 4) {
        const int b = b0 + r;
        if (b < kSnBins) ST[(size_t)b * ldt + f0 + tx] = tile[tx][r];
    }
}

// ---------------------------------------------------------------------------
// sn_select: numpy median of each row of X ([rows][ld], first n entries,
// non-negative f32) as bit patterns: lo = element of rank (n - 1) / 2, hi =
// element of rank n / 2 (equal for odd n); then the row's mask (below).  One
// block per row.  The row is
// staged in LDS when it fits (STAGE; otherwise every pass re-reads it from
// L2).  Radix select on the bit patterns: the bits above the highest bit where
// the row's min and max differ are common to every element, so the 8-bit
// digits start there (fewer passes, and the first digit spreads over the
// exponents actually present); one histogram per wave keeps the LDS atomics
// of different waves off each other's counters.
// ---------------------------------------------------------------------------
constexpr int kSnStageMax = 12288;  // values staged in LDS (48 KiB)

template <bool STAGE>
__global__ __launch_bounds__(256) void sn_select(const float* __restrict__ X, int ld, int n,
                                                 const unsigned* __restrict__ gmax, const float* __restrict__ c3,
                                                 int words, unsigned long long* __restrict__ M) {
    extern __shared__ unsigned srow[];
    __shared__ unsigned hist[4][kSnHist];
    __shared__ unsigned pick[3];
    __shared__ unsigned red[8];
    const unsigned* grow = reinterpret_cast<const unsigned*>(X) + (size_t)blockIdx.x * ld;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    unsigned mn = 0xFFFFFFFFu, mx = 0;
    for (int i = tid; i < n; i += 256) {
        const unsigned v = grow[i];
        if (STAGE) srow[i] = v;
        mn = min(mn, v);
        mx = max(mx, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
        mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    }
    if (lane == 0) { red[wv] = mn; red[4 + wv] = mx; }
    __syncthreads();
    mn = min(min(red[0], red[1]), min(red[2], red[3]));
    mx = max(max(red[4], red[5]), max(red[6], red[7]));
    const unsigned* row = STAGE ? srow : grow;
    unsigned rlo = mn, rhi = mn;  // a constant row (block-uniform): its value
    if (mn != mx) {
    const int hb = 31 - __clz(mn ^ mx);  // highest bit that differs
    unsigned pmask = hb == 31 ? 0u : (0xFFFFFFFFu << (hb + 1));
    unsigned prefix = mn & pmask, rank = (unsigned)(n - 1) / 2, cnt = 0;
    for (int s = hb - 7;; s -= 8) {
        const int shift = max(s, 0);  // a last digit may repeat known prefix bits: harmless
        reinterpret_cast<uint4*>(&hist[0][0])[tid] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        for (int i = tid; i < n; i += 256) {
            const unsigned v = row[i];
            hist_add(&hist[wv][0], (v >> shift) & 255u, i < n && (v & pmask) == prefix);
        }
        __syncthreads();
        hist[0][tid] += hist[1][tid] + hist[2][tid] + hist[3][tid];
        __syncthreads();
        if (tid < 64) {
            unsigned below, c;
            const unsigned dig = hist_pick(&hist[0][0], rank, lane, &below, &c);
            if (lane == 0) { pick[0] = dig; pick[1] = below; pick[2] = c; }
        }
        __syncthreads();
        prefix = (prefix & ~(255u << shift)) | (pick[0] << shift);
        pmask |= 255u << shift;
        rank -= pick[1];
        cnt = pick[2];
        if (shift == 0) break;
    }
    // prefix is the rank-(n-1)/2 element, `rank` its place among the cnt equal ones
    unsigned second = prefix;
    if ((n & 1) == 0 && rank + 1 >= cnt) {  // block-uniform: rank n/2 is the next larger value
        unsigned m2 = 0xFFFFFFFFu;
        for (int i = tid; i < n; i += 256) {
            const unsigned v = row[i];
            if (v > prefix) m2 = min(m2, v);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m2 = min(m2, (unsigned)__shfl_xor((int)m2, o, 64));
        __syncthreads();  // red[] reuse
        if (lane == 0) red[wv] = m2;
        __syncthreads();
        second = min(min(red[0], red[1]), min(red[2], red[3]));
    }
    rlo = prefix;
    rhi = second;
    }
    // ---- the row's mask: r3 = 3 * rowmed / a in numpy's float32 steps (an
    // even count takes the f32 mean of the two middle quotients), then bit
    // f % 64 of word (b, f / 64) = S[b][f] / a > c3[f] and > r3 (false
    // throughout when a == 0: NaN quotients, like numpy) ----
    const float a = __uint_as_float(*gmax);
    float dr = __fdiv_rn(__uint_as_float(rlo), a);
    if ((n & 1) == 0) dr = __fmul_rn(__fadd_rn(dr, __fdiv_rn(__uint_as_float(rhi), a)), 0.5f);
    const float rb = __fmul_rn(3.f, dr);
    for (int w = wv; w < words; w += 4) {
        const int f = 64 * w + lane;
        bool bit = false;
        if (f < n) {
            const float d = __fdiv_rn(__uint_as_float(row[f]), a);
            bit = d > c3[f] && d > rb;
        }
        const unsigned long long m = __ballot(bit);
        if (lane == 0) M[(size_t)blockIdx.x * words + w] = m;
    }
}


// ---------------------------------------------------------------------------
// sn_select_row: the row median and mask of sn_select with the row in
// registers: 256 threads x 41 values (rows of up to 10,496 frames -- a 58 s
// recording; sn_select above that) so that 6 blocks share a
// CU: the row's passes are latency chains (histogram, barrier, pick), and
// rows in flight are what hides them.  Per pass every wave counts its values
// into its own 256-bucket histogram (wave-aggregated atomics), then every
// wave folds the four copies and picks the same bucket (two barriers per
// pass, no broadcast).
// ---------------------------------------------------------------------------
constexpr int kRowT = 256, kRowPer = 41;  // 10,496 values

__global__ __launch_bounds__(kRowT) __attribute__((amdgpu_waves_per_eu(6))) void sn_select_row(
    const float* __restrict__ X, int ld, int n, const unsigned* __restrict__ gmax, const float* __restrict__ c3,
    int words, unsigned long long* __restrict__ M) {
    // slots past the row hold 0xFFFFFFFF: above every value (excluded from
    // the maximum by name), never matching a prefix (non-negative values have
    // bit 31 clear), a NaN quotient in the mask (bit 0) -- so no per-slot
    // validity predicate stays live across the kernel
    constexpr unsigned PAD = 0xFFFFFFFFu;
    __shared__ unsigned hist[2][4][256];  // two sets, one per pass parity
    __shared__ unsigned red[16];
    const unsigned* grow = reinterpret_cast<const unsigned*>(X) + (size_t)blockIdx.x * ld;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    unsigned v[kRowPer];
    {
        const int lim = n - 1 - tid;  // slot i holds frame tid + 256 i: valid while 256 i <= lim
#pragma unroll
        for (int i = 0; i < kRowPer; ++i) {
            const unsigned x = grow[tid + min(kRowT * i, max(lim, 0))];  // clamped: always in the row
            v[i] = kRowT * i <= lim ? x : PAD;
        }
    }
    unsigned mn = v[0], mx = 0;
#pragma unroll
    for (int i = 0; i < kRowPer; ++i) {
        mn = min(mn, v[i]);
        mx = max(mx, v[i] == PAD ? 0u : v[i]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
        mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    }
    if (lane == 0) {
        red[wv] = mn;
        red[4 + wv] = mx;
    }
    uint4* h4 = reinterpret_cast<uint4*>(&hist[0][0][0]);  // 512 uint4
    h4[tid] = make_uint4(0u, 0u, 0u, 0u);
    h4[tid + kRowT] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    mn = min(min(red[0], red[1]), min(red[2], red[3]));
    mx = max(max(red[4], red[5]), max(red[6], red[7]));
    unsigned rlo = mn, rhi = mn;  // a constant row (block-uniform): its value
    if (mn != mx) {
        const int hb = 31 - __clz(mn ^ mx);
        unsigned pmask = hb == 31 ? 0u : (0xFFFFFFFFu << (hb + 1));
        unsigned prefix = mn & pmask, rank = (unsigned)(n - 1) / 2, cnt = 0;
        int set = 0;
#pragma unroll 1
        for (int sh = hb - 7;; sh -= 8) {
            const int shift = max(sh, 0);  // a last digit may repeat known prefix bits: harmless
#pragma unroll
            for (int i = 0; i < kRowPer; ++i) hist_add(&hist[set][wv][0], (v[i] >> shift) & 255u, (v[i] & pmask) == prefix);
            __syncthreads();
            const uint4* hs = reinterpret_cast<const uint4*>(&hist[set][0][0]);
            uint4 c = hs[lane];
#pragma unroll
            for (int w = 1; w < 4; ++w) {
                const uint4 u = hs[64 * w + lane];
                c.x += u.x;
                c.y += u.y;
                c.z += u.z;
                c.w += u.w;
            }
            h4[(set ^ 1) * 256 + tid] = make_uint4(0u, 0u, 0u, 0u);  // the next pass's set
            unsigned below, cc;
            const unsigned dig = hist_pick4(c, rank, lane, &below, &cc);
            prefix = (prefix & ~(255u << shift)) | (dig << shift);
            pmask |= 255u << shift;
            rank -= below;
            cnt = cc;
            if (shift == 0) break;
            __syncthreads();  // every wave has read this set; the next set is zero
            set ^= 1;
        }
        rlo = rhi = prefix;
        if ((n & 1) == 0 && rank + 1 >= cnt) {  // block-uniform: rank n/2 is the next larger value
            unsigned m2 = PAD;
#pragma unroll
            for (int i = 0; i < kRowPer; ++i) m2 = min(m2, v[i] > prefix ? v[i] : PAD);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) m2 = min(m2, (unsigned)__shfl_xor((int)m2, o, 64));
            if (lane == 0) red[8 + wv] = m2;
            __syncthreads();
            rhi = min(min(red[8], red[9]), min(red[10], red[11]));
        }
    }
    // ---- the row's mask (sn_select's numpy f32 steps): bit f % 64 of word
    // f / 64; lane l of wave w holds frame 256 i + 64 w + l at iteration i ----
    const float a = __uint_as_float(*gmax);
    float dr = __fdiv_rn(__uint_as_float(rlo), a);
    if ((n & 1) == 0) dr = __fmul_rn(__fadd_rn(dr, __fdiv_rn(__uint_as_float(rhi), a)), 0.5f);
    const float rb = __fmul_rn(3.f, dr);
    constexpr int CH = 8;  // c3 loads in flight per chunk
    int t2 = tid;  // opaque: no frame index kept live from the load phase
    __asm__ volatile("" : "+v"(t2));
    const float* c3t = c3 + t2;
    const int lim2 = n - 1 - t2;
#pragma unroll
    for (int i0 = 0; i0 < kRowPer; i0 += CH) {
        float cv[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) cv[j] = c3t[min(kRowT * (i0 + j), max(lim2, 0))];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const int i = i0 + j;
            if (i >= kRowPer) break;
            const int w = 4 * i + wv;
            const float d = __fdiv_rn(__uint_as_float(v[i]), a);  // PAD: NaN, bit 0
            const unsigned long long m = __ballot(d > cv[j] && d > rb);
            if (lane == 0 && w < words) M[(size_t)blockIdx.x * words + w] = m;
        }
    }
}

// ---------------------------------------------------------------------------
// Morphology on the bit image (row = bin, bit = frame).  cv2's erode/dilate
// with a rectangle of ones and the default anchor (kw / 2, kh / 2): out(x, y)
// = min / max over the kernel of in(x + i - ax, y + j - ay), taps outside the
// image ignored.  Separable, one launch per rectangle: each thread reduces
// its word and the two neighbouring words over the rows y + vlo .. y + vhi
// (across bins), then along time over the offsets hlo .. hhi (|d| < 64) of
// the three reduced words -- the same bits as the horizontal pass followed by
// the vertical one (both are a min / max over the rectangle's in-image taps).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sn_morph(const unsigned long long* __restrict__ src,
                                                unsigned long long* __restrict__ dst, int rows, SnBatch nb, size_t pf,
                                                int vlo, int vhi, int hlo, int hhi, int erode) {
    // one thread per (row, word) of recording k = blockIdx.y, rows x words
    // flattened over the blocks (a row is ~160 words: a block per row would
    // idle a third of its lanes)
    const int k = blockIdx.y;
    const int n_frames = nb.nf[k], words = (n_frames + 63) / 64;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= rows * words) return;
    const int y = idx / words, w = idx - y * words;
    src = sn_at(src, pf, k);
    dst = sn_at(dst, pf, k);
    const unsigned long long ident = erode ? ~0ull : 0ull;
    // vertical: rows y + vlo .. y + vhi inside the image, words w - 1 .. w + 1
    unsigned long long vm = ident, v0 = ident, vp = ident;
    const int y0 = max(0, y + vlo), y1 = min(rows - 1, y + vhi);
    for (int yy = y0; yy <= y1; ++yy) {
        const unsigned long long* r = src + (size_t)yy * words;
        const unsigned long long a = w > 0 ? r[w - 1] : ident, b = r[w], c = w + 1 < words ? r[w + 1] : ident;
        if (erode) { vm &= a; v0 &= b; vp &= c; }
        else { vm |= a; v0 |= b; vp |= c; }
    }
    // bits past the image read as the identity (a frame position outside the
    // image is the identity in every row, so this commutes with the vertical pass)
    auto fix = [&](unsigned long long v, int i) -> unsigned long long {
        if (i < 0 || i >= words) return ident;
        const int valid = n_frames - 64 * i;
        if (valid >= 64) return v;
        const unsigned long long keep = (1ull << valid) - 1;
        return (v & keep) | (ident & ~keep);
    };
    const unsigned long long wm = fix(vm, w - 1), w0 = fix(v0, w), wp = fix(vp, w + 1);
    // horizontal: offsets hlo .. hhi (|d| < 64) from the word and its neighbours
    unsigned long long acc = ident;
    for (int d = hlo; d <= hhi; ++d) {
        unsigned long long s;  // bit i = in(64 w + i + d)
        if (d == 0) s = w0;
        else if (d > 0) s = (w0 >> d) | (wp << (64 - d));
        else s = (w0 << -d) | (wm >> (64 + d));
        acc = erode ? (acc & s) : (acc | s);
    }
    const int valid = n_frames - 64 * w;
    if (valid < 64) acc &= (1ull << valid) - 1;
    dst[(size_t)y * words + w] = acc;
}

// ---------------------------------------------------------------------------
// Connected components (8-connectivity) over row runs.
// Run table R (SoA, kSnFields arrays of max_runs ints).  sn_runs: one wave per
// row lists its runs [x0, x1] in order into one atomically allocated range,
// and initialises parents and statistics.  sn_unite: each run joins every run
// of the row above that touches it (x ranges within one frame).  sn_stats:
// bounding box, area and OpenCV's label-order key (the first 2x2 block of the
// component in block-raster order) accumulated on the root.  sn_emit: roots
// that pass the size filter.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int uf_load(const int* P, int i) {
    return __hip_atomic_load(P + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int uf_find(const int* P, int i) {
    int p = uf_load(P, i);
    while (p != i) {
        i = p;
        p = uf_load(P, i);
    }
    return i;
}
// Parents only ever decrease (atomicMin hooking of the larger root under the
// smaller), so every find terminates and the final root of a component is its
// smallest run index.
__device__ __forceinline__ void uf_union(int* P, int a, int b) {
    a = uf_find(P, a);
    b = uf_find(P, b);
    while (a != b) {
        if (a > b) { const int t = a; a = b; b = t; }
        const int old = atomicMin(P + b, a);
        if (old == b) return;  // b was still a root: hooked
        b = uf_find(P, old);   // b was hooked meanwhile: join a with b's new tree
        a = uf_find(P, a);
    }
}

__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(256) void sn_runs(const unsigned long long* __restrict__ M, int rows, SnBatch nb,
                                               size_t pf, int* __restrict__ R, int max_runs, int* __restrict__ row_off,
                                               int* __restrict__ row_cnt, int* __restrict__ counters) {
    const int lane = threadIdx.x & 63;
    const int y = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int k = blockIdx.y;
    if (y >= rows) return;
    const int words = (nb.nf[k] + 63) / 64;
    M = sn_at(M, pf, k);
    R = sn_at(R, pf, k);
    row_off = sn_at(row_off, pf, k);
    row_cnt = sn_at(row_cnt, pf, k);
    counters = sn_at(counters, pf, k);
    const unsigned long long* r = M + (size_t)y * words;
    auto starts_of = [&](int w) -> unsigned long long {
        const unsigned long long v = r[w], prev = w > 0 ? r[w - 1] : 0ull;
        return v & ~((v << 1) | (prev >> 63));
    };
    auto ends_of = [&](int w) -> unsigned long long {
        const unsigned long long v = r[w], next = w + 1 < words ? r[w + 1] : 0ull;
        return v & ~((v >> 1) | (next << 63));
    };
    int total = 0;
    for (int w0 = 0; w0 < words; w0 += 64) {
        const int w = w0 + lane;
        total += wave_sum_int(w < words ? __popcll(starts_of(w)) : 0);
    }
    int base = 0;
    if (lane == 0 && total > 0) base = atomicAdd(counters, total);
    base = __shfl(base, 0, 64);
    if (base + total > max_runs) {  // cannot happen within the host's bound; flagged, row dropped
        if (lane == 0) atomicOr(counters + 1, AA_SN_RUN_OVERFLOW);
        for (int i = base + lane; i < min(base + total, max_runs); i += 64) R[(size_t)R_Y * max_runs + i] = -1;
        total = 0;
    }
    if (lane == 0) {
        row_off[y] = base;
        row_cnt[y] = total;
    }
    if (total == 0) return;
    int* X0 = R + (size_t)R_X0 * max_runs;
    int* X1 = R + (size_t)R_X1 * max_runs;
    int* Y = R + (size_t)R_Y * max_runs;
    int* P = R + (size_t)R_P * max_runs;
    int ks0 = base, ke0 = base;
    for (int w0 = 0; w0 < words; w0 += 64) {
        const int w = w0 + lane;
        unsigned long long s = w < words ? starts_of(w) : 0ull;
        unsigned long long e = w < words ? ends_of(w) : 0ull;
        const unsigned cs = __popcll(s), ce = __popcll(e);
        const unsigned is = wave_incl_scan(cs, lane), ie = wave_incl_scan(ce, lane);
        int ks = ks0 + (int)(is - cs), ke = ke0 + (int)(ie - ce);
        while (s) {  // the k-th start and the k-th end of a row bound run k
            const int i = ks++;
            X0[i] = 64 * w + __builtin_ctzll(s);
            Y[i] = y;
            P[i] = i;
            R[(size_t)R_LEFT * max_runs + i] = INT_MAX;
            R[(size_t)R_RIGHT * max_runs + i] = -1;
            R[(size_t)R_TOP * max_runs + i] = INT_MAX;
            R[(size_t)R_BOT * max_runs + i] = -1;
            R[(size_t)R_AREA * max_runs + i] = 0;
            R[(size_t)R_KEY * max_runs + i] = INT_MAX;
            s &= s - 1;
        }
        while (e) {
            X1[ke++] = 64 * w + __builtin_ctzll(e);
            e &= e - 1;
        }
        ks0 += (int)__shfl(is, 63, 64);
        ke0 += (int)__shfl(ie, 63, 64);
    }
}

__global__ __launch_bounds__(256) void sn_unite(int* __restrict__ R, int max_runs, const int* __restrict__ row_off,
                                                const int* __restrict__ row_cnt, const int* __restrict__ counters,
                                                int rows, size_t pf) {
    const int k = blockIdx.y;
    R = sn_at(R, pf, k);
    row_off = sn_at(row_off, pf, k);
    row_cnt = sn_at(row_cnt, pf, k);
    counters = sn_at(counters, pf, k);
    const int nr = min(counters[0], max_runs);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < nr; i += gridDim.x * 256) {
    const int* X0 = R + (size_t)R_X0 * max_runs;
    const int* X1 = R + (size_t)R_X1 * max_runs;
    const int y = R[(size_t)R_Y * max_runs + i];
    if (y <= 0 || y >= rows) continue;  // row 0, or a slot of a dropped row (y = -1)
    int* P = R + (size_t)R_P * max_runs;
    const int a = X0[i] - 1, b = X1[i] + 1;  // 8-connectivity: diagonal neighbours touch
    const int first = row_off[y - 1], end = first + row_cnt[y - 1];
    int lo = first, hi = end;  // first run above that ends at or after a
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (X1[m] < a) lo = m + 1;
        else hi = m;
    }
    for (int j = lo; j < end && X0[j] <= b; ++j) uf_union(P, i, j);
    }
}

__global__ __launch_bounds__(256) void sn_stats(int* __restrict__ R, int max_runs, SnBatch nb,
                                                const int* __restrict__ counters, size_t pf) {
    const int k = blockIdx.y;
    const int kx = (nb.nf[k] + 1) / 2;  // 2x2 blocks per block row (OpenCV's label order)
    R = sn_at(R, pf, k);
    counters = sn_at(counters, pf, k);
    const int nr = min(counters[0], max_runs);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < nr; i += gridDim.x * 256) {
    const int y = R[(size_t)R_Y * max_runs + i];
    if (y < 0) continue;
    const int root = uf_find(R + (size_t)R_P * max_runs, i);
    const int x0 = R[(size_t)R_X0 * max_runs + i], x1 = R[(size_t)R_X1 * max_runs + i];
    atomicMin(R + (size_t)R_LEFT * max_runs + root, x0);
    atomicMax(R + (size_t)R_RIGHT * max_runs + root, x1);
    atomicMin(R + (size_t)R_TOP * max_runs + root, y);
    atomicMax(R + (size_t)R_BOT * max_runs + root, y);
    atomicAdd(R + (size_t)R_AREA * max_runs + root, x1 - x0 + 1);
    atomicMin(R + (size_t)R_KEY * max_runs + root, (y >> 1) * kx + (x0 >> 1));
    }
}

__global__ __launch_bounds__(256) void sn_emit(const int* __restrict__ R, int max_runs, int wmin, int hmin,
                                               const int* __restrict__ counters, const unsigned* __restrict__ gmax,
                                               size_t pf, aa_sn_component* __restrict__ out, int max_out,
                                               long long out_stride, int32_t* __restrict__ n_out, int n_out_stride) {
    const int k = blockIdx.y;
    R = sn_at(R, pf, k);
    counters = sn_at(counters, pf, k);
    if (gmax) gmax = sn_at(gmax, pf, k);
    out += k * out_stride;
    n_out += (size_t)k * n_out_stride;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int st = counters[1];
        if (gmax && (*gmax & 0x7FFFFFFFu) >= 0x7F800000u) st |= AA_SN_NONFINITE;
        n_out[1] = st;
    }
    const int nr = min(counters[0], max_runs);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < nr; i += gridDim.x * 256) {
    if (R[(size_t)R_Y * max_runs + i] < 0 || R[(size_t)R_P * max_runs + i] != i) continue;
    const int left = R[(size_t)R_LEFT * max_runs + i], top = R[(size_t)R_TOP * max_runs + i];
    const int w = R[(size_t)R_RIGHT * max_runs + i] - left + 1;
    const int hgt = R[(size_t)R_BOT * max_runs + i] - top + 1;
    if (w < wmin || hgt < hmin) continue;
    const int k = atomicAdd(n_out, 1);
    if (k < max_out) {
        aa_sn_component c;
        c.left = left;
        c.top = top;
        c.width = w;
        c.height = hgt;
        c.area = R[(size_t)R_AREA * max_runs + i];
        c.order = R[(size_t)R_KEY * max_runs + i];
        out[k] = c;
    }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct SnWs {
    // shared by the recordings of a batch (their per-recording launches run
    // one after another on the stream)
    float* S;
    float* ST;
    // recording 0's; recording k's sit k * pf bytes further
    unsigned* colmed;
    float* c3;
    unsigned* gmax;
    int* counters;  // [0] runs allocated, [1] status flags
    unsigned long long* M0;
    unsigned long long* M1;
    int* row_off;
    int* row_cnt;
    int* R;
    int max_runs;
    size_t pf;
    size_t bytes;
};

static int sn_frames(const SnPlan& p, int64_t n) { return 1 + (int)(n / p.cfg.hop_length); }

// After the final horizontal erosion of a horizontal dilation of the same
// width kw (and the row-wise AND of the vertical erosion), the runs of a row
// are separated by >= kw clear frames: at most (F + kw) / (kw + 1) per row.
static int sn_max_runs(const SnPlan& p, int F) {
    const long long per = (p.kw_e == p.kw_d && p.kw_e > 1) ? (F + p.kw_e) / (p.kw_e + 1) + 1 : F / 2 + 1;
    return (int)std::min<long long>(per * kSnBins, INT_MAX / kSnFields);
}

// F: the largest frame count of the batch; K recordings
static SnWs sn_ws_layout(const SnPlan& p, int F, int K, char* base) {
    SnWs w{};
    size_t off = 0;
    auto take = [&](size_t bytes) -> char* {
        char* q = base ? base + off : nullptr;
        off = align_up(off + bytes, 256);
        return q;
    };
    const int words = (F + 63) / 64, ldt = words * 64;
    w.S = reinterpret_cast<float*>(take(sizeof(float) * (size_t)F * kSnLd));
    w.ST = reinterpret_cast<float*>(take(sizeof(float) * (size_t)kSnBins * ldt));
    const size_t per0 = off;
    w.colmed = reinterpret_cast<unsigned*>(take(sizeof(unsigned) * (size_t)F));
    w.c3 = reinterpret_cast<float*>(take(sizeof(float) * (size_t)F));
    w.gmax = reinterpret_cast<unsigned*>(take(64));
    w.counters = reinterpret_cast<int*>(take(64));
    w.M0 = reinterpret_cast<unsigned long long*>(take(8 * (size_t)kSnBins * words));
    w.M1 = reinterpret_cast<unsigned long long*>(take(8 * (size_t)kSnBins * words));
    w.row_off = reinterpret_cast<int*>(take(sizeof(int) * kSnBins));
    w.row_cnt = reinterpret_cast<int*>(take(sizeof(int) * kSnBins));
    w.max_runs = sn_max_runs(p, F);
    w.R = reinterpret_cast<int*>(take(sizeof(int) * (size_t)kSnFields * w.max_runs));
    w.pf = off - per0;
    w.bytes = per0 + (size_t)K * w.pf;
    return w;
}

// morphology (:670-684), components (:686) and the size filter (:689-691)
// of every recording of the batch from its mask in M0, one launch per step
// for the whole batch
static int sn_components(SnPlan& p, const SnWs& ws, const SnBatch& nb, bool with_gmax, aa_sn_component* out,
                         int max_out, long long out_stride, int32_t* n_out, int n_out_stride, hipStream_t st) {
    int maxw = 1;
    for (int k = 0; k < nb.n; ++k) maxw = std::max(maxw, (nb.nf[k] + 63) / 64);
    const dim3 gm((kSnBins * maxw + 255) / 256, nb.n);
    unsigned long long* a = ws.M0;
    unsigned long long* b = ws.M1;
    // one launch per structuring element: rectangle kh x kw, anchor (kw / 2, kh / 2)
    auto morph = [&](int kh, int kw, int erode) -> int {
        const int ax = kw / 2, ay = kh / 2;
        hipEvent_t e0;
        int rc = p.timer.begin(SN_STAGE_MORPH, st, &e0);
        if (rc != AA_OK) return rc;
        hipLaunchKernelGGL(sn_morph, gm, dim3(256), 0, st, a, b, kSnBins, nb, ws.pf, -ay, kh - 1 - ay, -ax,
                           kw - 1 - ax, erode);
        AA_LAUNCH_CHECK();
        std::swap(a, b);
        return p.timer.end(SN_STAGE_MORPH, st, e0);
    };
    int rc = AA_OK;
    // MORPH_OPEN with ones(4, 4): erode, then dilate; dilate; erode
    if ((rc = morph(4, 4, 1)) || (rc = morph(4, 4, 0))) return rc;
    if ((rc = morph(p.kh_d, p.kw_d, 0)) || (rc = morph(p.kh_e, p.kw_e, 1))) return rc;
    // (counters were zeroed by sn_zero; sn_runs marks the slots of a dropped row)
    hipEvent_t e0;
    if ((rc = p.timer.begin(SN_STAGE_COMPONENTS, st, &e0)) != AA_OK) return rc;
    hipLaunchKernelGGL(sn_runs, dim3((kSnBins + 3) / 4, nb.n), dim3(256), 0, st, a, kSnBins, nb, ws.pf, ws.R,
                       ws.max_runs, ws.row_off, ws.row_cnt, ws.counters);
    AA_LAUNCH_CHECK();
    // grid-stride over the runs actually allocated (counters[0] of max_runs)
    const dim3 gr(std::min((ws.max_runs + 255) / 256, 512), nb.n);
    hipLaunchKernelGGL(sn_unite, gr, dim3(256), 0, st, ws.R, ws.max_runs, ws.row_off, ws.row_cnt, ws.counters, kSnBins,
                       ws.pf);
    AA_LAUNCH_CHECK();
    hipLaunchKernelGGL(sn_stats, gr, dim3(256), 0, st, ws.R, ws.max_runs, nb, ws.counters, ws.pf);
    AA_LAUNCH_CHECK();
    hipLaunchKernelGGL(sn_emit, gr, dim3(256), 0, st, ws.R, ws.max_runs, p.wmin, p.hmin, ws.counters,
                       with_gmax ? ws.gmax : nullptr, ws.pf, out, max_out, out_stride, n_out, n_out_stride);
    AA_LAUNCH_CHECK();
    return p.timer.end(SN_STAGE_COMPONENTS, st, e0);
}

// sn_stft64 over one recording: persistent blocks (4 per CU, the LDS limit),
// a multiple of 8 so every XCD owns an equal share of the blocks
static int sn_launch_stft(SnPlan& p, const float* pcm, int64_t n, int F, float* S, int ld, unsigned* gmax,
                          hipStream_t st) {
    int grid = std::min(F, 1024);  // 1024 = 4 resident blocks per CU, persistent
    grid = (grid + 7) & ~7;
    const double2* tab = p.d_tab;
    hipEvent_t e0;
    int rc = p.timer.begin(SN_STAGE_STFT, st, &e0);
    if (rc != AA_OK) return rc;
    if (p.tw_chain)
        hipLaunchKernelGGL(sn_stft64<true>, dim3(grid), dim3(kS64T), 0, st, pcm, (int)n, p.cfg.hop_length, F, tab,
                           tab + kS64TabTw1, tab + kS64TabTw3, tab + kS64TabTwS, S, ld, gmax);
    else
        hipLaunchKernelGGL(sn_stft64<false>, dim3(grid), dim3(kS64T), 0, st, pcm, (int)n, p.cfg.hop_length, F, tab,
                           tab + kS64TabTw1, tab + kS64TabTw3, tab + kS64TabTwS, S, ld, gmax);
    AA_LAUNCH_CHECK();
    return p.timer.end(SN_STAGE_STFT, st, e0);
}

// The whole detector over K recordings of one PCM buffer (recording k:
// offs[k], lens[k] samples, host arrays): per recording the STFT (+ column
// medians), transpose and row select (+ mask) into its own mask slot, then
// the morphology and components of the whole batch.
static int sn_run_impl(SnPlan* p, const float* pcm, const int64_t* offs, const int64_t* lens, int K,
                       void* workspace, size_t workspace_bytes, aa_sn_component* out, int max_out,
                       long long out_stride, int32_t* n_out, int n_out_stride, uint64_t* mask_out, hipStream_t st) {
    SnBatch nb{};
    nb.n = K;
    int Fmax = 1;
    for (int k = 0; k < K; ++k) {
        AA_CHECK(lens[k] >= 0 && lens[k] <= (int64_t(1) << 29) && offs[k] >= 0, AA_ERR_UNSUPPORTED,
                 "aa_sn_run: recording %d: %lld samples at %lld (at most 2^29)", k, (long long)lens[k],
                 (long long)offs[k]);
        AA_CHECK(pcm || lens[k] == 0, AA_ERR_INVALID, "aa_sn_run: null pcm");
        nb.nf[k] = sn_frames(*p, lens[k]);
        Fmax = std::max(Fmax, nb.nf[k]);
    }
    const SnWs ws = sn_ws_layout(*p, Fmax, K, static_cast<char*>(workspace));
    AA_CHECK(workspace && workspace_bytes >= ws.bytes, AA_ERR_WORKSPACE, "aa_sn_run: workspace %zu < %zu bytes",
             workspace_bytes, ws.bytes);
    hipLaunchKernelGGL(sn_zero, dim3(K), dim3(64), 0, st, ws.gmax, ws.counters, ws.pf, n_out, n_out_stride);
    AA_LAUNCH_CHECK();
    for (int k = 0; k < K; ++k) {
        const int F = nb.nf[k];
        unsigned* gmax = sn_at(ws.gmax, ws.pf, k);
        unsigned* colmed = sn_at(ws.colmed, ws.pf, k);
        float* c3 = sn_at(ws.c3, ws.pf, k);
        unsigned long long* M0 = sn_at(ws.M0, ws.pf, k);
        int rc = sn_launch_stft(*p, lens[k] ? pcm + offs[k] : pcm, lens[k], F, ws.S, kSnLd, gmax, st);
        if (rc != AA_OK) return rc;
        hipEvent_t e1;
        if ((rc = p->timer.begin(SN_STAGE_COLMED, st, &e1)) != AA_OK) return rc;
        hipLaunchKernelGGL(sn_colmed, dim3((F + 3) / 4), dim3(256), 0, st, ws.S, kSnLd, F, colmed);
        AA_LAUNCH_CHECK();
        if ((rc = p->timer.end(SN_STAGE_COLMED, st, e1)) != AA_OK) return rc;
        const int words = (F + 63) / 64, ldt = words * 64;
        hipEvent_t e0;
        if ((rc = p->timer.begin(SN_STAGE_TRANSPOSE, st, &e0)) != AA_OK) return rc;
        hipLaunchKernelGGL(sn_transpose, dim3((kSnBins + 63) / 64, words), dim3(256), 0, st, ws.S, F, ldt, ws.ST, gmax,
                           colmed, c3);
        AA_LAUNCH_CHECK();
        if ((rc = p->timer.end(SN_STAGE_TRANSPOSE, st, e0)) != AA_OK) return rc;
        if ((rc = p->timer.begin(SN_STAGE_SELECT, st, &e0)) != AA_OK) return rc;
        if (F <= kRowT * kRowPer)
            hipLaunchKernelGGL(sn_select_row, dim3(kSnBins), dim3(kRowT), 0, st, ws.ST, ldt, F, gmax, c3, words, M0);
        else if (F <= kSnStageMax)
            hipLaunchKernelGGL(sn_select<true>, dim3(kSnBins), dim3(256), sizeof(unsigned) * F, st, ws.ST, ldt, F, gmax,
                               c3, words, M0);
        else
            hipLaunchKernelGGL(sn_select<false>, dim3(kSnBins), dim3(256), 0, st, ws.ST, ldt, F, gmax, c3, words, M0);
        AA_LAUNCH_CHECK();
        if ((rc = p->timer.end(SN_STAGE_SELECT, st, e0)) != AA_OK) return rc;
    }
    if (mask_out)
        AA_HIP(hipMemcpyAsync(mask_out, ws.M0, 8 * (size_t)kSnBins * ((nb.nf[0] + 63) / 64), hipMemcpyDeviceToDevice,
                              st));
    return sn_components(*p, ws, nb, true, out, max_out, out_stride, n_out, n_out_stride, st);
}

}  // namespace aa

using namespace aa;

// cv2: an empty structuring element means a 3x3 rectangle
static void sn_kernel_dims(int kh, int kw, int* oh, int* ow) {
    if (kh <= 0 || kw <= 0) kh = kw = 3;
    *oh = kh;
    *ow = kw;
}

// kernel sizes and filter thresholds of src/identify_tracks.py:673-691, in
// the reference's arithmetic (host only)
static int sn_plan_geometry(const aa_sn_config& cfg, SnPlan* p) {
    AA_CHECK(cfg.n_fft == 4096, AA_ERR_UNSUPPORTED, "aa_sn: n_fft %d (signal_noise uses 4096)", cfg.n_fft);
    AA_CHECK(cfg.sr > 0 && cfg.hop_length > 0 && cfg.signal_width >= 0, AA_ERR_INVALID, "aa_sn: bad sizes");
    p->cfg = cfg;
    const int width = (int)(cfg.signal_width * cfg.sr / cfg.hop_length);
    const double bin_hz = 1.0 / (cfg.n_fft * (1.0 / cfg.sr));  // np.fft.rfftfreq: k / (n d)
    int height = 0;
    for (int k = 0; k <= cfg.n_fft / 2; ++k)
        if (k * bin_hz > cfg.freq_range) {
            height = k + 1;
            break;
        }
    sn_kernel_dims(height, width, &p->kh_d, &p->kw_d);
    sn_kernel_dims(height / 10, width, &p->kh_e, &p->kw_e);
    p->wmin = (int)std::floor(0.65 * width) + 1;  // s[2] > 0.65 * width
    p->hmin = height - height / 10 + 1;            // s[3] > height - height // 10
    AA_CHECK(p->kw_d <= 127 && p->kw_e <= 127, AA_ERR_UNSUPPORTED,
             "aa_sn: signal width %d frames exceeds the 127-frame morphology window", width);
    return AA_OK;
}

extern "C" int aa_sn_create(const aa_sn_config* cfg, void** plan) {
    AA_CHECK(cfg && plan, AA_ERR_INVALID, "aa_sn_create: null argument");
    SnPlan* p = new SnPlan();
    const int rc = sn_plan_geometry(*cfg, p);
    if (rc != AA_OK) {
        delete p;
        return rc;
    }
    if (const char* e = std::getenv("AA_SN_TW")) p->tw_chain = std::strcmp(e, "table") != 0;
    // sn_stft64's tables, rounded from long double
    auto wexp = [](long long e, long long m) {  // exp(-2 pi i e / m)
        const long double a = -2.0L * 3.141592653589793238462643383279502884L * (long double)(e % m) / (long double)m;
        return make_double2((double)cosl(a), (double)sinl(a));
    };
    std::vector<double2> tab(kS64TabN);
    {  // scipy.signal.get_window('hann', 4096, fftbins=True) (librosa 0.11's window, :654): general_cosine
       // over np.linspace(-pi, pi, 4097)[:4096], w = 0.5 + 0.5 cos(fac) in float64
        const double start = -M_PI, step = (M_PI - start) / 4096.0;
        std::vector<double> w(4096);
        for (int i = 0; i < 4096; ++i) {
            const double fac = (double)i * step + start;
            w[i] = 0.5 + 0.5 * std::cos(fac);
        }
        // halved (exact): the real split's factor 1/2 rides on the window
        for (int n = 0; n < 2048; ++n) tab[n] = make_double2(0.5 * w[2 * n], 0.5 * w[2 * n + 1]);
    }
    for (int k1 = 1; k1 < 16; ++k1)
        for (int n2 = 0; n2 < 16; ++n2) tab[kS64TabTw1 + (k1 - 1) * 16 + n2] = wexp((long long)n2 * k1, 256);
    for (int n3 = 1; n3 < 8; ++n3)
        for (int t = 0; t < kS64T; ++t) tab[kS64TabTw3 + (n3 - 1) * kS64T + t] = wexp((long long)n3 * t, 2048);
    for (int t = 0; t < kS64T; ++t) tab[kS64TabTwS + t] = wexp(t ? t : 128, 4096);
    hipError_t e = hipMalloc((void**)&p->d_tab, sizeof(double2) * tab.size());
    if (e == hipSuccess) e = hipMemcpy(p->d_tab, tab.data(), sizeof(double2) * tab.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_error("aa_sn_create: %s", hipGetErrorString(e));
        aa_sn_destroy(p);
        return AA_ERR_HIP;
    }
    *plan = p;
    return AA_OK;
}

extern "C" int aa_sn_destroy(void* plan) {
    SnPlan* p = static_cast<SnPlan*>(plan);
    if (!p) return AA_OK;
    (void)hipFree(p->d_tab);
    p->timer.release();
    delete p;
    return AA_OK;
}

extern "C" int aa_sn_geometry(const aa_sn_config* cfg, int32_t* out6) {
    AA_CHECK(cfg && out6, AA_ERR_INVALID, "aa_sn_geometry: null argument");
    SnPlan p;
    const int rc = sn_plan_geometry(*cfg, &p);
    if (rc != AA_OK) return rc;
    out6[0] = p.kh_d;
    out6[1] = p.kw_d;
    out6[2] = p.kh_e;
    out6[3] = p.kw_e;
    out6[4] = p.wmin;
    out6[5] = p.hmin;
    return AA_OK;
}

extern "C" int64_t aa_sn_n_frames(const void* plan, int64_t n_samples) {
    const SnPlan* p = static_cast<const SnPlan*>(plan);
    if (!p || n_samples < 0) return -1;
    return sn_frames(*p, n_samples);
}

extern "C" size_t aa_sn_workspace_bytes(const void* plan, int64_t max_samples) {
    const SnPlan* p = static_cast<const SnPlan*>(plan);
    if (!p || max_samples < 0) return 0;
    return sn_ws_layout(*p, sn_frames(*p, max_samples), 1, nullptr).bytes;
}

extern "C" size_t aa_sn_batch_workspace_bytes(const void* plan, int64_t max_samples, int32_t n_rec) {
    const SnPlan* p = static_cast<const SnPlan*>(plan);
    if (!p || max_samples < 0 || n_rec < 1 || n_rec > kSnMaxBatch) return 0;
    return sn_ws_layout(*p, sn_frames(*p, max_samples), n_rec, nullptr).bytes;
}

extern "C" int aa_sn_run(void* plan, const float* pcm, int64_t n_samples, void* workspace, size_t workspace_bytes,
                         aa_sn_component* out, int32_t max_out, int32_t* n_out, uint64_t* mask_out, void* stream) {
    SnPlan* p = static_cast<SnPlan*>(plan);
    AA_CHECK(p && out && n_out && (pcm || n_samples == 0), AA_ERR_INVALID, "aa_sn_run: null argument");
    const int64_t off = 0;
    return sn_run_impl(p, pcm, &off, &n_samples, 1, workspace, workspace_bytes, out, max_out, max_out, n_out, 2,
                       mask_out, static_cast<hipStream_t>(stream));
}

extern "C" int aa_sn_run_batch(void* plan, const float* pcm, const int64_t* offsets, const int64_t* lengths,
                               int32_t n_rec, void* workspace, size_t workspace_bytes, aa_sn_component* out,
                               int32_t max_out, int64_t out_stride, int32_t* n_out, int32_t n_out_stride,
                               void* stream) {
    SnPlan* p = static_cast<SnPlan*>(plan);
    AA_CHECK(p && offsets && lengths && out && n_out, AA_ERR_INVALID, "aa_sn_run_batch: null argument");
    AA_CHECK(n_rec >= 1 && n_rec <= kSnMaxBatch, AA_ERR_UNSUPPORTED, "aa_sn_run_batch: %d recordings (1..%d)", n_rec,
             kSnMaxBatch);
    AA_CHECK(out_stride >= max_out && n_out_stride >= 2, AA_ERR_INVALID, "aa_sn_run_batch: overlapping outputs");
    return sn_run_impl(p, pcm, offsets, lengths, n_rec, workspace, workspace_bytes, out, max_out, out_stride, n_out,
                       n_out_stride, nullptr, static_cast<hipStream_t>(stream));
}

extern "C" int aa_sn_components_from_mask(void* plan, const uint64_t* mask, int64_t n_frames, void* workspace,
                                          size_t workspace_bytes, aa_sn_component* out, int32_t max_out,
                                          int32_t* n_out, void* stream) {
    SnPlan* p = static_cast<SnPlan*>(plan);
    AA_CHECK(p && mask && out && n_out, AA_ERR_INVALID, "aa_sn_components_from_mask: null argument");
    AA_CHECK(n_frames >= 1 && n_frames <= (int64_t(1) << 28), AA_ERR_INVALID,
             "aa_sn_components_from_mask: %lld frames", (long long)n_frames);
    const int F = (int)n_frames;
    const SnWs ws = sn_ws_layout(*p, F, 1, static_cast<char*>(workspace));
    AA_CHECK(workspace && workspace_bytes >= ws.bytes, AA_ERR_WORKSPACE,
             "aa_sn_components_from_mask: workspace %zu < %zu bytes", workspace_bytes, ws.bytes);
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(sn_zero, dim3(1), dim3(64), 0, st, nullptr, ws.counters, ws.pf, n_out, 2);
    AA_LAUNCH_CHECK();
    AA_HIP(hipMemcpyAsync(ws.M0, mask, 8 * (size_t)kSnBins * ((F + 63) / 64), hipMemcpyDeviceToDevice, st));
    SnBatch nb{};
    nb.n = 1;
    nb.nf[0] = F;
    return sn_components(*p, ws, nb, false, out, max_out, max_out, n_out, 2, st);
}

extern "C" int aa_sn_spectrogram(void* plan, const float* pcm, int64_t n_samples, float* out, int64_t ld,
                                 void* stream) {
    SnPlan* p = static_cast<SnPlan*>(plan);
    AA_CHECK(p && out && (pcm || n_samples == 0), AA_ERR_INVALID, "aa_sn_spectrogram: null argument");
    AA_CHECK(n_samples >= 0 && n_samples < (int64_t(1) << 29), AA_ERR_UNSUPPORTED,
             "aa_sn_spectrogram: %lld samples (below 2^29)", (long long)n_samples);
    AA_CHECK(ld >= kSnBins && ld <= (int64_t(1) << 20), AA_ERR_INVALID, "aa_sn_spectrogram: ld %lld", (long long)ld);
    const int F = sn_frames(*p, n_samples);
    return sn_launch_stft(*p, pcm, n_samples, F, out, (int)ld, nullptr, static_cast<hipStream_t>(stream));
}

// Launch stages of aa_sn_run / aa_sn_run_batch and their timing (the
// aa_fe_stage_* contract); an item is one STFT frame of one recording.
//   stft: the f64 transform (2.5 N log2 N + the window's N), PCM read once
//         (hop samples per frame) + the S row written;
//   transpose: S read + ST written; select: ST read + the mask bits written;
//   morph: per launch the mask read and written (bits); components: the mask read.
extern "C" int aa_sn_n_stages(const void* plan) { return plan ? SN_N_STAGES : -1; }

extern "C" int aa_sn_stage_info(const void* plan, int32_t stage, char* name, int32_t name_len,
                                double* flops_per_item, double* bytes_per_item) {
    const SnPlan* p = static_cast<const SnPlan*>(plan);
    AA_CHECK(p && stage >= 0 && stage < SN_N_STAGES, AA_ERR_INVALID, "aa_sn_stage_info: bad stage");
    const double N = p->cfg.n_fft, B = kSnBins, hop = p->cfg.hop_length;
    double fl = 0, by = 0;
    const char* nm = "";
    switch (stage) {
        case SN_STAGE_STFT: nm = "sn_stft64"; fl = 2.5 * N * std::log2(N) + N; by = 4 * hop + 4 * B; break;
        case SN_STAGE_TRANSPOSE: nm = "sn_transpose"; by = 8 * B; break;
        case SN_STAGE_SELECT: nm = "sn_select"; by = 4 * B + B / 8; break;
        case SN_STAGE_MORPH: nm = "sn_morph"; by = B / 4; break;
        case SN_STAGE_COLMED: nm = "sn_colmed"; by = 4 * B; break;
        default: nm = "sn_components"; by = B / 8; break;
    }
    if (name && name_len > 0) snprintf(name, name_len, "%s", nm);
    if (flops_per_item) *flops_per_item = fl;
    if (bytes_per_item) *bytes_per_item = by;
    return AA_OK;
}

extern "C" int aa_sn_set_timing(void* plan, uint32_t stage_mask) {
    SnPlan* p = static_cast<SnPlan*>(plan);
    AA_CHECK(p, AA_ERR_INVALID, "aa_sn_set_timing: null plan");
    p->timer.mask = stage_mask;
    return AA_OK;
}

extern "C" int aa_sn_stage_time(void* plan, int32_t stage, double* total_ms, int64_t* count) {
    SnPlan* p = static_cast<SnPlan*>(plan);
    AA_CHECK(p && stage >= 0 && stage < SN_N_STAGES, AA_ERR_INVALID, "aa_sn_stage_time: bad stage");
    return p->timer.collect(stage, total_ms, count);
}
