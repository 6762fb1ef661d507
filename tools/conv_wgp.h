// conv_wgp: the 9x3 F(6,3) conv with the Winograd planes split over the
// waves instead of the output channels -- measured and rejected (bit-identical
// to conv_wg, 127-144 us against 115-124 us: its MFMA phase is ~7 % faster,
// the LDS-staged output transform ~7 us slower, and its 79 KiB / 219 VGPRs
// leave 2 waves per SIMD instead of 3; profiles/r06/wgp_rejected.txt).  Kept
// as a tools/ diagnostic for tools/conv_bench_x3.hip (modes 32-34).
#pragma once

namespace aa {

// ---------------------------------------------------------------------------
// conv_wgp: the same F(WO, 3) conv with the planes split over the waves
// instead of the output channels.  In conv_wg every wave multiplies the same
// A fragments (the staged planes) with its own 16 output channels, so each
// A byte is read from LDS by all four waves: at 3 MFMAs per 2 KiB of A the
// MFMA loop is LDS-bound (the 9x3 layer: MFMA pipe ~47 % busy, the LDS ~47 %,
// profiles/r06/pmc_sq_step_serial.txt).  Here wave w owns planes w WPL .. w WPL
// + WPL - 1 for all BN = NF x 16 channels: the A of a step is read once per
// block, its MFMAs per A fragment x4 (NF), and the block's B traffic (per-wave
// weight rows from L2, one step ahead) is unchanged.  The output transform
// needs all A planes of a (pixel, channel): the waves write their m planes
// to LDS (a 32-channel slice at a time), then every thread forms the WO
// outputs of its (group-pixel, 4-channel unit) items from the A planes in
// plane order -- the same f32 expression, on the same MFMA sums (each plane's
// steps accumulate in the same (group, row) order), as conv_wg's epilogue: the
// two kernels' outputs are bit-identical.
// LDS: the staged planes, then per slice M [A][MF 16][32 ch] f32 (16-B units
// rotated by the pixel: conflict-free writes and reads) and the E tile.
// ---------------------------------------------------------------------------
template <int KH, int TH, int TW, int WO, int MF>
__host__ __device__ constexpr size_t wgp_lds_bytes() {
    constexpr size_t planes = wg_patch_bytes<KH, TH, TW, WO, 1>();
    constexpr size_t epi = (size_t)(WO + 2) * MF * 16 * 32 * 4 + (size_t)TH * TW * 32 * 4;
    return planes > epi ? planes : epi;
}

template <int KH, int CIN, int NW, int MF, int NF, int POOL, int TH, int TW, int OCC = 0, bool IN_SPLIT = false,
          bool OUT_SPLIT = false, int DIAG = 0, int WO = 6, int BD = 2>
__global__ __launch_bounds__(NW * 64)
__attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1, OCC ? OCC : 8)))
void conv_wgp(const float* __restrict__ in, int Hin, int Win, const bf16* __restrict__ wt,
              const float* __restrict__ bias, float* __restrict__ out, int Hout, int Wout, int cout_store,
              int tiles_w, int act, float alpha) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    constexpr int A = WO + 2;    // planes
    constexpr int WPL = A / NW;  // planes per wave
    static_assert(A % NW == 0, "whole planes per wave");
    static_assert(WO >= 2 && WO <= 6 && WO != 5, "F(2|3|4|6, 3)");
    static_assert(TW % WO == 0 && TH % POOL == 0 && TW % POOL == 0, "group- and pool-aligned tile");
    constexpr int NP = TW / WO, TP = TH * NP;
    static_assert(TP <= MF * 16, "tile covered by the fragments");
    static_assert(CIN % 32 == 0, "C_in multiple of 32");
    constexpr int NTHR = NW * 64, BN = NF * 16, PH = TH + KH - 1, PV = PH * NP, NG = CIN / 32;
    static_assert(BN % 32 == 0, "32-channel epilogue slices");
    constexpr int EH = BN / 32;             // epilogue slices
    constexpr int NSW = NG * KH * WPL;      // steps per wave
    constexpr int SLICE = BN * 64;          // bf16 elements of one step's weight slice (all BN channels)
    constexpr int MP = MF * 16;             // m rows per plane (fragment pixels)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* patch = smem;

    const BlockPos bp = x3_block<true>();
    const int n = bp.n, cb = bp.cb;
    const int th = bp.tile / tiles_w, tw = bp.tile - (bp.tile / tiles_w) * tiles_w;
    const int oh0 = th * TH, ow0 = tw * TW;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4;
    const int ebase = wave * WPL;  // the wave's first plane

    int abase[MF], aph[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        int p = i * 16 + (lane & 15);
        if (p >= TP) p = 0;  // padding rows: computed, never stored
        abase[i] = p * 128;
        aph[i] = p + q;
    }
    int bofs[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const int row = j * 16 + (lane & 15);
        bofs[j] = row * 128 + (((q + row) & 7) << 4);
    }
    const size_t step_stride = (size_t)gridDim.y * SLICE;
    const __amdgpu_buffer_rsrc_t wrs = x3_wrsrc(wt);

    f32x4 acc[WPL][MF][NF];
#pragma unroll
    for (int e = 0; e < WPL; ++e)
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[e][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    struct BSet {
        bf16x8 h[NF], l[NF];
    };
    BSet Bq[BD];
    // the weight slice of the wave's step sw: (group, row, plane) -> conv_wg's
    // step index ((g KH + kh) A + plane) of the same host packing
    auto read_b = [&](BSet& b, int sw) {
        const int g = sw / (KH * WPL), r = sw - g * (KH * WPL), kh = r / WPL, el = r - kh * WPL;
        const int s = (g * KH + kh) * A + ebase + el;
        const int soff = __builtin_amdgcn_readfirstlane((int)((cb * SLICE + s * step_stride) * 2));
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            b.h[j] = x3_wload(wrs, bofs[j], soff);
            b.l[j] = x3_wload(wrs, bofs[j] ^ 64, soff);
        }
    };
    // one step: the wave's plane el at row kh; A fragments just in time, two in flight
    auto step = [&](auto bc, int sw, int kh, auto elc) {
        constexpr int el = decltype(elc)::value;
        constexpr int b = decltype(bc)::value;
        BSet& cur = Bq[b];
        if (sw + BD - 1 < NSW) read_b(Bq[(b + BD - 1) % BD], sw + BD - 1);
        const int pofs = (ebase + el) * PV * 128 + kh * NP * 128, tv = kh * NP;
        bf16x8 h2[2], l2[2];
        auto rd = [&](int i, int k) {
            const int a = pofs + abase[i] + (((aph[i] + tv) & 7) << 4);
            h2[k] = *reinterpret_cast<const bf16x8*>(patch + a);
            l2[k] = *reinterpret_cast<const bf16x8*>(patch + (a ^ 64));
        };
        rd(0, 0);
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            if (i + 1 < MF) rd(i + 1, (i + 1) & 1);
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                acc[el][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.h[j], h2[i & 1], acc[el][i][j], 0, 0, 0);
                acc[el][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.l[j], h2[i & 1], acc[el][i][j], 0, 0, 0);
                acc[el][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.h[j], l2[i & 1], acc[el][i][j], 0, 0, 0);
            }
        }
    };

    const __amdgpu_buffer_rsrc_t ars = x3_wrsrc(reinterpret_cast<const char*>(in) + (size_t)n * Hin * Win * CIN * 4);
    auto load4 = [&](int gh, int gw, int g, int cq) -> float4 {
        const int pix = gh * Win + gw;
        if constexpr (IN_SPLIT) {
            const int o = pix * (CIN * 4) + g * 128 + cq * 8;
            const bf16x4 h = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(ars, o, 0, 0));
            const bf16x4 l = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(ars, o + 64, 0, 0));
            return make_float4((float)h[0] + (float)l[0], (float)h[1] + (float)l[1], (float)h[2] + (float)l[2],
                               (float)h[3] + (float)l[3]);
        } else {
            return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ars, (pix * CIN + g * 32 + cq * 4) * 4,
                                                                                     0, 0));
        }
    };

#pragma unroll
    for (int k = 0; k < BD - 1; ++k)
        if (k < NSW) read_b(Bq[k], k);  // their latency hides behind the first staging
    wg_static_for<0, NG>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        if (g > 0) __syncthreads();  // every wave is done with the previous planes
        wg_stage<WO, A, 0, NP, PV, NTHR, (DIAG & 1) ? 0 : PV * 8>(patch, oh0, ow0, Hin, Win, g, load4);
        __syncthreads();
        if constexpr (AA_WG_PRIO > 0) __builtin_amdgcn_s_setprio(AA_WG_PRIO);
        if constexpr ((DIAG & 2) == 0) {
            if constexpr (WPL % BD == 0) {
                // the B sets alternate the same way every row: a runtime row loop
                for (int kh = 0; kh < KH; ++kh) {
                    const int s0 = (g * KH + kh) * WPL;
                    wg_static_for<0, WPL>([&](auto elc) {
                        constexpr int el = decltype(elc)::value;
                        step(std::integral_constant<int, el % BD>{}, s0 + el, kh, elc);
                    });
                }
            } else {
                // rows unrolled: the B set by the step's index
                constexpr int sb = g * KH * WPL;
                wg_static_for<0, KH * WPL>([&](auto sc) {
                    constexpr int si = decltype(sc)::value;
                    step(std::integral_constant<int, (sb + si) % BD>{}, sb + si, si / WPL,
                         std::integral_constant<int, si % WPL>{});
                });
            }
        }
        if constexpr (AA_WG_PRIO > 0) __builtin_amdgcn_s_setprio(0);
    });
    __syncthreads();  // planes no longer needed

    // ---- epilogue, per 32-channel slice h (fragments j = 2h, 2h + 1) ----
    constexpr int PSH = wg_psh(WO);
    float* M = reinterpret_cast<float*>(smem);             // [A][MP][32] f32, units rotated by the row
    float* E = M + (size_t)A * MP * 32;                    // [TH TW][32] f32 (x3_eoff layout)
#pragma unroll
    for (int h = 0; h < EH; ++h) {
        if (h > 0) __syncthreads();  // the previous slice's M and E reads are done
        // 1. the wave's planes: unit uq = 4 jj + q (channels 4 uq .. + 3 of the slice) of row p
#pragma unroll
        for (int el = 0; el < WPL; ++el)
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    const int p = i * 16 + (lane & 15), uq = 4 * jj + q;
                    const int row = (ebase + el) * MP + p;
                    *reinterpret_cast<f32x4*>(M + row * 32 + (((uq + p) & 7) << 2)) = acc[el][i][2 * h + jj];
                }
        __syncthreads();
        // 2. items (group-pixel p < TP, unit u): the WO outputs from the A planes in plane order
        for (int it = threadIdx.x; it < TP * 8; it += NTHR) {
            const int p = it >> 3, u = it & 7;
            f32x4 m[A];
#pragma unroll
            for (int e = 0; e < A; ++e) m[e] = *reinterpret_cast<const f32x4*>(M + (e * MP + p) * 32 + (((u + p) & 7) << 2));
            const int r = p / NP, jp = p - (p / NP) * NP;
            const int px = r * TW + WO * jp;
#pragma unroll
            for (int k = 0; k < WO; ++k) {
                f32x4 y = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int e = 0; e < A; ++e) {
                    const float c = wg_at(WO, k, e);
                    if (c == 0.f) continue;
                    if (c == 1.f) y += m[e];
                    else if (c == -1.f) y -= m[e];
                    else y += c * m[e];
                }
                *reinterpret_cast<float4*>(E + x3_eoff<32, PSH>(px + k, u)) = make_float4(y[0], y[1], y[2], y[3]);
            }
        }
        __syncthreads();
        x3_store<TH, TW, POOL, 32, NTHR, OUT_SPLIT, false, PSH>(E, bias, out, n, cb * EH + h, oh0, ow0, Hout, Wout,
                                                              cout_store, act, alpha);
    }
}

}  // namespace aa
