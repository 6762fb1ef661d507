// Split-bf16 convolution with a Winograd F(WO, 3) transform along W
// (AA_PREC_BF16X3, kernel width 3), included by aa_cnn.hip after
// aa_conv_x3.h (shares bf_hi/bf_lo, the grouped-split layout and x3_store).
//
// A kernel-width-3 conv computes, per output row, y_k = sum_t g_t d_{k+t}
// along W.  F(WO, 3) produces WO adjacent outputs from A = WO + 2 inputs with
// A products instead of 3 WO:
//   u = B^T d (A x A),   v = G g (A x 3),   m_e = u_e v_e,   y = A^T m (WO x A)
// (m_e summed over C_in and the KH rows), so the conv becomes A independent
// implicit GEMMs (one per plane e) over the output column GROUPS of WO, K =
// KH x C_in each: A / (3 WO) of the direct MFMA work -- 2/3 for F(2, 3), 1/2
// for F(4, 3), 4/9 for F(6, 3).  The input transform runs at staging (f32
// arithmetic, then the bf16 hi / lo split of u); the weights are transformed
// on the host in double and split there; the output transform runs in the
// epilogue on the f32 accumulators.  F(2, 3) is the form of rounds 2-4
// (u0 = d0 - d2, u1 = d1 + d2, u2 = d2 - d1, u3 = d1 - d3; v0 = g0, v1 =
// (g0 + g1 + g2) / 2, v2 = (g0 - g1 + g2) / 2, v3 = g2; y0 = m0 + m1 + m2,
// y1 = m1 - m2 - m3); F(4, 3) and F(6, 3) take the interpolation points
// {0, +-1, +-2} and {0, +-1, +-2, +-1/2} (and infinity).  The larger
// transforms amplify rounding, but split-bf16 keeps ~17 bits: emulated on the
// CPU (tools/wino_study.py), model1's max |delta logit| on the bench's 64
// windows stays 1.6-1.9e-4 for the 9x3 layer direct, F(2,3), F(4,3) or
// F(6,3) -- the other layers' rounding dominates.
//
// LDS: the A planes of the transformed patch, (TH + KH - 1) rows x TW / WO
// groups, 128 B per group-pixel (32-channel group, hi then lo), with the
// rotation swizzle of aa_conv_x3.h on the plane's linear group index v; staged
// NPASS planes-sets at a time (A / NPASS planes each) to bound the LDS.  A
// fragment's 16 lanes read 16 consecutive tile groups p, and at tap kh the
// group index is v = p + kh * TW/WO: consecutive for every tap with no row
// wrap (the planes have no halo along W), so the ds_read_b128 lane groups
// are conflict-free.  Weights come per step (group g, pass, row kh, plane) as
// [cout_pad][8 units] with aa_conv_x3.h's swizzle, loaded per wave straight
// from global (L2) one step ahead -- waves meet only at the barriers around
// each staging.
#pragma once

#include <type_traits>

namespace aa {

// transform coefficients (exact in f32): B^T [A][A], A^T [WO][A]
__host__ __device__ constexpr float wg_bt(int wo, int e, int t) {
    constexpr float b2[4][4] = {{1, 0, -1, 0}, {0, 1, 1, 0}, {0, -1, 1, 0}, {0, 1, 0, -1}};
    constexpr float b3[5][5] = {{2, -1, -2, 1, 0}, {0, -2, -1, 1, 0}, {0, 2, -3, 1, 0}, {0, -1, 0, 1, 0},
                                {0, 2, -1, -2, 1}};
    constexpr float b4[6][6] = {{4, 0, -5, 0, 1, 0},  {0, -4, -4, 1, 1, 0}, {0, 4, -4, -1, 1, 0},
                                {0, -2, -1, 2, 1, 0}, {0, 2, -1, -2, 1, 0}, {0, 4, 0, -5, 0, 1}};
    constexpr float b6[8][8] = {{-1, 0, 5.25f, 0, -5.25f, 0, 1, 0},         {0, 1, 1, -4.25f, -4.25f, 1, 1, 0},
                                {0, -1, 1, 4.25f, -4.25f, -1, 1, 0},        {0, 0.5f, 0.25f, -2.5f, -1.25f, 2, 1, 0},
                                {0, -0.5f, 0.25f, 2.5f, -1.25f, -2, 1, 0},  {0, 2, 4, -2.5f, -5, 0.5f, 1, 0},
                                {0, -2, 4, 2.5f, -5, -0.5f, 1, 0},          {0, -1, 0, 5.25f, 0, -5.25f, 0, 1}};
    return wo == 2 ? b2[e][t] : wo == 3 ? b3[e][t] : wo == 4 ? b4[e][t] : b6[e][t];
}
__host__ __device__ constexpr float wg_at(int wo, int k, int e) {
    constexpr float a2[2][4] = {{1, 1, 1, 0}, {0, 1, -1, -1}};
    constexpr float a3[3][5] = {{1, 1, 1, 1, 0}, {0, 1, -1, 2, 0}, {0, 1, 1, 4, 1}};
    constexpr float a4[4][6] = {{1, 1, 1, 1, 1, 0}, {0, 1, -1, 2, -2, 0}, {0, 1, 1, 4, 4, 0}, {0, 1, -1, 8, -8, 1}};
    constexpr float a6[6][8] = {{1, 1, 1, 1, 1, 1, 1, 0},
                                {0, 1, -1, 2, -2, 0.5f, -0.5f, 0},
                                {0, 1, 1, 4, 4, 0.25f, 0.25f, 0},
                                {0, 1, -1, 8, -8, 0.125f, -0.125f, 0},
                                {0, 1, 1, 16, 16, 0.0625f, 0.0625f, 0},
                                {0, 1, -1, 32, -32, 0.03125f, -0.03125f, 1}};
    return wo == 2 ? a2[k][e] : wo == 3 ? a3[k][e] : wo == 4 ? a4[k][e] : a6[k][e];
}
// G [A][3] (host, double): v_e = sum_k G[e][k] g_k
static inline double wg_g(int wo, int e, int k) {
    static const double g2[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    static const double g3[5][3] = {{0.5, 0, 0},
                                    {-0.5, -0.5, -0.5},
                                    {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                    {1.0 / 6, 1.0 / 3, 2.0 / 3},
                                    {0, 0, 1}};
    static const double g4[6][3] = {{0.25, 0, 0},
                                    {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                    {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                    {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                    {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                    {0, 0, 1}};
    static const double g6[8][3] = {{-1, 0, 0},
                                    {-2.0 / 9, -2.0 / 9, -2.0 / 9},
                                    {-2.0 / 9, 2.0 / 9, -2.0 / 9},
                                    {1.0 / 90, 1.0 / 45, 2.0 / 45},
                                    {1.0 / 90, -1.0 / 45, 2.0 / 45},
                                    {32.0 / 45, 16.0 / 45, 8.0 / 45},
                                    {32.0 / 45, -16.0 / 45, 8.0 / 45},
                                    {0, 0, 1}};
    return wo == 2 ? g2[e][k] : wo == 3 ? g3[e][k] : wo == 4 ? g4[e][k] : g6[e][k];
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename Fn>
__device__ __forceinline__ void wg_static_for(Fn&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        wg_static_for<B + 1, E>(f);
    }
}

template <int KH, int TH, int TW, int WO, int NPASS>
__host__ __device__ constexpr size_t wg_patch_bytes() {
    return (size_t)((WO + 2) / NPASS) * (TH + KH - 1) * (TW / WO) * 128;
}

// AA_WG_EPH: the epilogue's f32 tile holds BN / AA_WG_EPH channels at a time,
// the slices stored one after the other.  2 (default): the 9x3 layer's tile
// 60 -> 30 KiB, so its block's LDS is set by the 48 KiB of planes (72 -> 48
// KiB); the kernel alone is unchanged (115.5 -> 116 us, 2 waves/SIMD by its
// 180 VGPRs) but the other stream's blocks find room beside it: step 267.9k ->
// 270.6k audio-s/s, ahead in each of 3 alternating rounds
// (profiles/r05/ab_wg_eph.txt)
#ifndef AA_WG_EPH
#define AA_WG_EPH 2
#endif
// epilogue slices of a BN-channel block over WN waves: whole waves per slice,
// at least 32 channels (x3_store's 8 units) each
__host__ __device__ constexpr int wg_eph(int BN, int WN) {
    return (AA_WG_EPH > 1 && WN % AA_WG_EPH == 0 && BN / AA_WG_EPH >= 32) ? AA_WG_EPH : 1;
}
template <int KH, int BN, int TH, int TW, int WO, int NPASS, int WN = 1>
constexpr size_t wg_lds_bytes() {
    const size_t main = wg_patch_bytes<KH, TH, TW, WO, NPASS>();
    const size_t epi = (size_t)TH * TW * (BN / wg_eph(BN, WN)) * 4;
    return main > epi ? main : epi;
}

// epilogue pixel swizzle shift (x3_eoff): the WO outputs of a group land in
// distinct 16-B slots across a store's 8 lanes when WO >> PSH is odd
constexpr int wg_psh(int wo) { return wo == 4 ? 2 : wo == 3 ? 0 : 1; }

// Stage (group g, planes e0 .. e0 + PPS - 1) of the transformed patch: per
// (group-pixel v, channel quad cq) the A input columns WO jp .. WO jp + A - 1,
// transformed (u = B^T d, f32), split into bf16 hi / lo, into the planes
// (128 B per group-pixel, aa_conv_x3.h's rotation swizzle on v)
template <int WO, int PPS, int E0, int NP, int PV, int NTHR, int ITEMS, typename Load4>
__device__ __forceinline__ void wg_stage(char* patch, int oh0, int ow0, int Hin, int Win, int g, Load4&& load4) {
    constexpr int A = WO + 2;
    for (int idx = threadIdx.x; idx < ITEMS; idx += NTHR) {
        const int v = idx >> 3, cq = idx & 7;
        const int R = v / NP, jp = v - (v / NP) * NP;
        const int gh = min(oh0 + R, Hin - 1);
        float4 d[A];
#pragma unroll
        for (int c = 0; c < A; ++c) d[c] = load4(gh, min(ow0 + WO * jp + c, Win - 1), g, cq);
        const int unit = (((cq >> 1) + v) & 7) << 4;
        // F(6, 3): the factored input transform (shared partial sums,
        // 26 operations per channel instead of the 44 non-zeros of B^T)
        float4 u6[WO == 6 ? 8 : 1];
        if constexpr (WO == 6) {
            auto f = [&](auto get, auto put) {
                const float d0 = get(d[0]), d1 = get(d[1]), d2 = get(d[2]), d3 = get(d[3]);
                const float d4 = get(d[4]), d5 = get(d[5]), d6 = get(d[6]), d7 = get(d[7]);
                put(0, fmaf(5.25f, d2 - d4, d6 - d0));
                put(7, fmaf(5.25f, d3 - d5, d7 - d1));
                const float a12 = fmaf(-4.25f, d4, d2 + d6), b12 = fmaf(-4.25f, d3, d1 + d5);
                put(1, a12 + b12);
                put(2, a12 - b12);
                const float a34 = fmaf(-1.25f, d4, fmaf(0.25f, d2, d6));
                const float b34 = fmaf(2.f, d5, fmaf(-2.5f, d3, 0.5f * d1));
                put(3, a34 + b34);
                put(4, a34 - b34);
                const float a56 = fmaf(-5.f, d4, fmaf(4.f, d2, d6));
                const float b56 = fmaf(0.5f, d5, fmaf(-2.5f, d3, 2.f * d1));
                put(5, a56 + b56);
                put(6, a56 - b56);
            };
            f([](const float4& x) { return x.x; }, [&](int e, float y) { u6[e].x = y; });
            f([](const float4& x) { return x.y; }, [&](int e, float y) { u6[e].y = y; });
            f([](const float4& x) { return x.z; }, [&](int e, float y) { u6[e].z = y; });
            f([](const float4& x) { return x.w; }, [&](int e, float y) { u6[e].w = y; });
        }
#pragma unroll
        for (int el = 0; el < PPS; ++el) {
            float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (WO == 6) u = u6[E0 + el];
#pragma unroll
            for (int t = 0; t < (WO == 6 ? 0 : A); ++t) {
                const float b = wg_bt(WO, E0 + el, t);
                if (b == 0.f) continue;
                if (b == 1.f) {
                    u.x += d[t].x; u.y += d[t].y; u.z += d[t].z; u.w += d[t].w;
                } else if (b == -1.f) {
                    u.x -= d[t].x; u.y -= d[t].y; u.z -= d[t].z; u.w -= d[t].w;
                } else {
                    u.x = fmaf(b, d[t].x, u.x); u.y = fmaf(b, d[t].y, u.y);
                    u.z = fmaf(b, d[t].z, u.z); u.w = fmaf(b, d[t].w, u.w);
                }
            }
            uint32_t h0, l0, h1, l1;
            split2(u.x, u.y, h0, l0);
            split2(u.z, u.w, h1, l1);
            const int a = (el * PV + v) * 128 + unit + (cq & 1) * 8;
            *reinterpret_cast<uint2*>(patch + a) = make_uint2(h0, h1);
            *reinterpret_cast<uint2*>(patch + (a ^ 64)) = make_uint2(l0, l1);
        }
    }
}

// DIAG (tools/conv_bench_x3.hip only): bit 0 skips the staging, bit 1 the MFMA steps
template <int KH, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW, int OCC = 0,
          bool IN_SPLIT = false, bool OUT_SPLIT = false, int DIAG = 0, int WO = 2, int NPASS = 1, int BD = 2>
__global__ __launch_bounds__(WM * WN * 64)
__attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1, OCC ? OCC : 8)))
void conv_wg(const float* __restrict__ in, int Hin, int Win, const bf16* __restrict__ wt,
             const float* __restrict__ bias, float* __restrict__ out, int Hout, int Wout, int cout_store,
             int tiles_w, int act, float alpha) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    constexpr int A = WO + 2;                 // planes
    constexpr int PPS = A / NPASS;            // planes per staging pass
    static_assert(WO >= 2 && WO <= 6 && WO != 5, "F(2|3|4|6, 3)");
    static_assert(A % NPASS == 0, "whole passes");
    // BD: B fragment sets in flight (the next BD - 1 steps' weights load under
    // this step's MFMAs); a runtime row loop needs the set of a step fixed by
    // its plane slot
    static_assert(BD >= 2 && ((A / NPASS) % 2 != 0 || (A / NPASS) % BD == 0), "B ring depth divides the pass");
    static_assert(TW % WO == 0 && TH % POOL == 0 && TW % POOL == 0, "group- and pool-aligned tile");
    constexpr int NP = TW / WO;  // output column groups per tile row
    constexpr int TP = TH * NP;  // group-pixels per tile
    static_assert(TP <= WM * MF * 16, "tile covered by the waves' fragments");
    static_assert(CIN % 32 == 0, "C_in multiple of 32");
    constexpr int NTHR = WM * WN * 64;
    constexpr int BN = WN * NF * 16;
    constexpr int PH = TH + KH - 1;
    constexpr int PV = PH * NP;  // group-pixels per plane
    constexpr int NG = CIN / 32;
    constexpr int NSTEP = NG * NPASS * KH * PPS;  // (group, pass, kh, plane of the pass)
    constexpr int SLICE = BN * 64;      // bf16 elements of one step's slice
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* patch = smem;

    const BlockPos bp = x3_block<true>();
    const int n = bp.n, cb = bp.cb;
    const int th = bp.tile / tiles_w, tw = bp.tile - (bp.tile / tiles_w) * tiles_w;
    const int oh0 = th * TH, ow0 = tw * TW;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int wm = wave % WM, wn = wave / WM;
    const int q = lane >> 4;

    int abase[MF], aph[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        int p = (wm * MF + i) * 16 + (lane & 15);
        // padding rows (computed, never stored): the pixel 16 k rows back, whose
        // swizzle slot is the lane's own -- a padding lane reading pixel 0 put a
        // second address on a busy slot of its ds_read_b128 group (the 9x3
        // layer's MFMA loop: 6.5 M of its 7.5 M bank-conflict cycles per launch)
        if (p >= TP) p = max(p - 16 * ((p - TP) / 16 + 1), 0);
        abase[i] = p * 128;
        aph[i] = p + q;
    }
    int bofs[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const int row = wn * NF * 16 + j * 16 + (lane & 15);
        bofs[j] = row * 128 + (((q + row) & 7) << 4);
    }
    const size_t step_stride = (size_t)gridDim.y * SLICE;
    const __amdgpu_buffer_rsrc_t wrs = x3_wrsrc(wt);

    f32x4 acc[A][MF][NF];
#pragma unroll
    for (int e = 0; e < A; ++e)
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[e][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    struct BSet {
        bf16x8 h[NF], l[NF];
    };
    BSet Bq[BD];
    auto read_b = [&](BSet& b, int s) {
        const int soff = __builtin_amdgcn_readfirstlane((int)((cb * SLICE + s * step_stride) * 2));
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            b.h[j] = x3_wload(wrs, bofs[j], soff);
            b.l[j] = x3_wload(wrs, bofs[j] ^ 64, soff);
        }
    };
    // one step: plane e (slot el of the staged pass) at row offset kh, B of
    // this step in `cur`, the next step's B loaded into `nxt` under this
    // step's MFMAs; A fragments just in time, two in flight
    // bc: the step's B set (s % BD, known at compile time)
    auto step = [&](auto bc, int s, int kh, auto ec, auto elc) {
        constexpr int e = decltype(ec)::value;
        constexpr int el = decltype(elc)::value;
        constexpr int b = decltype(bc)::value;
        BSet& cur = Bq[b];
        if (s + BD - 1 < NSTEP) read_b(Bq[(b + BD - 1) % BD], s + BD - 1);
        const int pofs = el * PV * 128 + kh * NP * 128, tv = kh * NP;
        bf16x8 h2[2], l2[2];
        auto rd = [&](int i, int k) {
            const int a = pofs + abase[i] + (((aph[i] + tv) & 7) << 4);
            h2[k] = *reinterpret_cast<const bf16x8*>(patch + a);
            l2[k] = *reinterpret_cast<const bf16x8*>(patch + (a ^ 64));
        };
        rd(0, 0);
        if constexpr (AA_PIN_WG & 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            if (i + 1 < MF) rd(i + 1, (i + 1) & 1);
            if constexpr (AA_PIN_WG & 2) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                acc[e][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.h[j], h2[i & 1], acc[e][i][j], 0, 0, 0);
                acc[e][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.l[j], h2[i & 1], acc[e][i][j], 0, 0, 0);
                acc[e][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.h[j], l2[i & 1], acc[e][i][j], 0, 0, 0);
            }
        }
    };

    // one input value quad (4 channels of group g) of pixel (gh, gw), in f32
    // (buffer loads: the resource based at the window (64-bit), the pixel in the
    // lane's 32-bit offset -- any batch size, one window < 2 GiB)
    const __amdgpu_buffer_rsrc_t ars = x3_wrsrc(reinterpret_cast<const char*>(in) + (size_t)n * Hin * Win * CIN * 4);
    constexpr int wbase = 0;
    auto load4 = [&](int gh, int gw, int g, int cq) -> float4 {
        const int pix = gh * Win + gw;
        if constexpr (IN_SPLIT) {
            const int o = pix * (CIN * 4) + g * 128 + cq * 8;
            const bf16x4 h = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(ars, o, wbase, 0));
            const bf16x4 l = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(ars, o + 64, wbase, 0));
            return make_float4((float)h[0] + (float)l[0], (float)h[1] + (float)l[1], (float)h[2] + (float)l[2],
                               (float)h[3] + (float)l[3]);
        } else {
            return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ars, (pix * CIN + g * 32 + cq * 4) * 4,
                                                                                     wbase, 0));
        }
    };

#pragma unroll
    for (int k = 0; k < BD - 1; ++k)
        if (k < NSTEP) read_b(Bq[k], k);  // their latency hides behind the first staging
    wg_static_for<0, NG>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        wg_static_for<0, NPASS>([&](auto pc) {
            constexpr int pass = decltype(pc)::value;
            if (g > 0 || pass > 0) __syncthreads();  // every wave is done with the previous planes
            // ---- stage (group g, pass) ----
            wg_stage<WO, PPS, pass * PPS, NP, PV, NTHR, (DIAG & 1) ? 0 : PV * 8>(patch, oh0, ow0, Hin, Win, g, load4);
            __syncthreads();
            if constexpr (AA_WG_PRIO > 0) __builtin_amdgcn_s_setprio(AA_WG_PRIO);  // (A/B knob, as AA_X3_PRIO)
            if constexpr ((DIAG & 2) == 0) {
                if constexpr (PPS % 2 == 0) {
                    // an even count of steps per row: the B sets alternate the same way every row
                    for (int kh = 0; kh < KH; ++kh) {
                        const int s0 = ((g * NPASS + pass) * KH + kh) * PPS;
                        wg_static_for<0, PPS>([&](auto elc) {
                            constexpr int el = decltype(elc)::value;
                            constexpr std::integral_constant<int, pass * PPS + el> ec{};
                            // s0 is a multiple of PPS, hence of BD: the set is el % BD
                            step(std::integral_constant<int, el % BD>{}, s0 + el, kh, ec, elc);
                        });
                    }
                } else {
                    // odd: rows unrolled, the B set by the step's parity in the pass
                    // (KH * PPS steps per pass: even KH keeps passes aligned)
                    constexpr int sb = (g * NPASS + pass) * KH * PPS;
                    wg_static_for<0, KH * PPS>([&](auto sc) {
                        constexpr int si = decltype(sc)::value;
                        constexpr int kh = si / PPS, el = si % PPS;
                        constexpr std::integral_constant<int, pass * PPS + el> ec{};
                        constexpr std::integral_constant<int, el> elc{};
                        // the B set a step reads was loaded BD - 1 steps before
                        step(std::integral_constant<int, (sb + si) % BD>{}, sb + si, kh, ec, elc);
                    });
                }
            }
            if constexpr (AA_WG_PRIO > 0) __builtin_amdgcn_s_setprio(0);
        });
    });
    __syncthreads();  // planes no longer needed: the f32 tile reuses LDS

    // ---- epilogue: output transform into the f32 tile (x3_store's swizzled
    // layout: a store's 8 lanes hold pixels WO apart, PSH keeps their units in
    // distinct 16-B slots) ----
    constexpr int PSH = wg_psh(WO);
    constexpr int EH = wg_eph(BN, WN), WNE = WN / EH, BNE = BN / EH;  // channel slices of the epilogue tile
    float* E = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int h = 0; h < EH; ++h) {
        if (h > 0) __syncthreads();  // the previous slice's pooled reads are done
        if (wn / WNE == h) {
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                const int u = (wn % WNE) * NF * 4 + j * 4 + q;
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    const int p = (wm * MF + i) * 16 + (lane & 15);
                    if (p < TP) {
                        const int r = p / NP, jp = p - (p / NP) * NP;
                        const int px = r * TW + WO * jp;
#pragma unroll
                        for (int k = 0; k < WO; ++k) {
                            f32x4 y = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                            for (int e = 0; e < A; ++e) {
                                const float c = wg_at(WO, k, e);
                                if (c == 0.f) continue;
                                if (c == 1.f) y += acc[e][i][j];
                                else if (c == -1.f) y -= acc[e][i][j];
                                else y += c * acc[e][i][j];
                            }
                            *reinterpret_cast<float4*>(E + x3_eoff<BNE, PSH>(px + k, u)) =
                                make_float4(y[0], y[1], y[2], y[3]);
                        }
                    }
                }
            }
        }
        __syncthreads();
        // slice h of block cb: channels cb BN + h BNE .. (x3_store's channel base is its cb x its BN)
        x3_store<TH, TW, POOL, BNE, NTHR, OUT_SPLIT, false, PSH>(E, bias, out, n, cb * EH + h, oh0, ow0, Hout, Wout,
                                                                cout_store, act, alpha);
    }
}

}  // namespace aa
