// One-wave 4096-point real FFT for gfx950, shared by the log-mel front end
// (fe_stft_mel_4096, aa_frontend.hip) and the signal detector (sn_stft,
// aa_signal.hip).  The algorithm (a four-step FFT of the 2048 complex points
// z[n] = x[2n] + i x[2n+1]: DFT-32 in registers, twiddles, LDS transpose,
// DFT-32, DPP radix-2) is described in fe_stft_mel_4096's header comment; the
// real split that follows differs per caller and stays with the kernels.
#pragma once

#include "aa_common.h"
#include "aa_twiddles.h"

namespace aa {

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

// ---------------------------------------------------------------------------
// wave-level pieces
// ---------------------------------------------------------------------------
constexpr int kRow = 66;          // padded transpose row (float2)
constexpr int kHalf = 16 * kRow;  // per-wave LDS buffer (float2)

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float2 wconst32(int k) { return make_float2(kW32[k][0], kW32[k][1]); }
__device__ __forceinline__ float2 wconst64(int k) { return make_float2(kW64[k][0], kW64[k][1]); }
__device__ __forceinline__ float2 wconst128(int k) { return make_float2(kW128[k][0], kW128[k][1]); }

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

__device__ __forceinline__ float load_view(__amdgpu_buffer_rsrc_t rs, int i) {  // 0 outside the view
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, i * 4, 0, 0));
}

// Periodic Hann, w[n] = 1/2 - cos(2 pi n / 4096) / 2, on the lane's samples
// n = 2c + 128 r (+1 for the odd ones): cos(a + 2 pi r / 32) by angle addition
// from the lane's cos/sin of a (hwe / hwo: table values; made opaque per frame
// so the 64 products are not hoisted into live registers).  The upper
// half-wave's (-1)^r input modulation of step 1 (wave_fft_core) is folded in
// as the sign of the odd-r weights: +-1/2 per lane.
__device__ __forceinline__ void wave_hann(float2 (&y)[32], float2 hwe, float2 hwo, int lane) {
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
}

// Steps 1-5 of the 2048-point complex FFT of one frame.  In: lane c holds
// z[c + 64 r] in y[r] (windowed, upper half-wave modulated by wave_hann).
// t1 = W2048^c, t8 = W2048^(8c): the caller's loop-carried table values, made
// opaque here each frame.  wb: the wave's kHalf-float2 LDS buffer.
// Out: lane L = 2 k1 + h holds Z[k1 + 32 (32 h + j)] in u[dperm(j)].
__device__ __forceinline__ void wave_fft_core(float2 (&y)[32], float2 (&u)[32], float2* wb, int lane,
                                              float2& t1, float2& t8) {
    const int k1 = lane >> 1, h = lane & 1;
    // The transpose (step 3) runs in two passes of 16 registers per lane, each
    // pass freeing 16 registers before it fills 16, so the data never occupies
    // more than 64 VGPRs.  For that, the upper half-wave (columns c >= 32)
    // works with its rows rotated by 16: (-1)^r on the input gives DFT output
    // X[(k + 16) % 32] in register k (step 1), its twiddle ladder is rotated to
    // match (step 2), it reads its columns rotated by 16 (step 3), and undoes
    // that rotation of the second DFT by (-1)^k on the odd outputs (step 4).
    const unsigned up = lane >= 32 ? 0x80000000u : 0u;  // sign mask of the upper half
    auto flip = [up](float2 v) {
        return make_float2(__uint_as_float(__float_as_uint(v.x) ^ up), __uint_as_float(__float_as_uint(v.y) ^ up));
    };
    // ---- 1. DFT-32 over r ----
    dft32(y);
    // ---- 2. twiddle W2048^(c row) = (W^8c)^(row/8) (W^c)^(row%8), row = k
    // (+16 mod 32 in the upper half); ladders rebuilt per frame (<= 4 roundings
    // per twiddle; not kept live across the loop) ----
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
    // ---- 3. transpose in two passes: pass p moves registers 16p..16p+15
    // (rows (16p + 16 [c >= 32]) % 32 + 0..15 of column c) and lane (k1, h)
    // takes columns h + 2m, m in the 16-range 16 ((k1 / 16) ^ p) of row k1,
    // into u[16p ..] ----
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
    // ---- 4. DFT-32 over m (input rotated by 16 in the upper half: output k
    // times (-1)^k) ----
    dft32(u);
#pragma unroll
    for (int k = 1; k < 32; k += 2) u[dperm(k)] = flip(u[dperm(k)]);
    // ---- 5. radix-2 across the lane pair: lane h = 1 sends W64^j E1, lane
    // h = 0 sends E0; then Z = E0 + W E1 (h = 0) and E0 - W E1 (h = 1) are
    // recv +- own ----
    const float sg = h ? -1.f : 1.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const float2 e = u[dperm(j)];
        const float2 wj = wconst64(j);
        const float2 g = h ? cmul(wj, e) : e;
        const float2 rv = make_float2(swap_pair(g.x), swap_pair(g.y));
        u[dperm(j)] = make_float2(fmaf(sg, g.x, rv.x), fmaf(sg, g.y, rv.y));
    }
}

}  // namespace aa
