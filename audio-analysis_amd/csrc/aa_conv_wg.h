// Split-bf16 convolution with a Winograd F(2,3) transform along W
// (AA_PREC_BF16X3, kernel width 3), included by aa_cnn.hip after
// aa_conv_x3.h (shares bf_hi/bf_lo, the grouped-split layout and x3_store).
//
// A kernel-width-3 conv computes, per output row, y_k = sum_t g_t d_{k+t}
// along W.  F(2,3) produces two adjacent outputs from four inputs with four
// products instead of six:
//   u0 = d0 - d2   u1 = d1 + d2   u2 = d2 - d1   u3 = d1 - d3
//   v0 = g0        v1 = (g0 + g1 + g2) / 2       v2 = (g0 - g1 + g2) / 2   v3 = g2
//   m_e = u_e v_e  (summed over C_in and the KH rows)
//   y0 = m0 + m1 + m2      y1 = m1 - m2 - m3
// so the conv becomes four independent implicit GEMMs (one per e) over the
// output column PAIRS, K = KH x C_in each: 2/3 of the direct MFMA work.  The
// input transform runs at staging (f32 arithmetic, then the bf16 hi / lo
// split of u); the weights are transformed on the host in double and split
// there; the output transform runs in the epilogue on the f32 accumulators.
//
// LDS: four planes (e) of the transformed patch, (TH + KH - 1) rows x TW/2
// pairs, 128 B per pair-pixel (32-channel group, hi then lo), with the
// rotation swizzle of aa_conv_x3.h on the plane's linear pair index v.  A
// fragment's 16 lanes read 16 consecutive tile pairs p, and at tap kh the
// pair index is v = p + kh * TW/2: consecutive for every tap with no row
// wrap at all (the pair planes have no halo along W), so the ds_read_b128
// lane groups are conflict-free.  Weights come per step (group g, row kh,
// e) as [cout_pad][8 units] with aa_conv_x3.h's swizzle, loaded per wave
// straight from global (L2) one step ahead -- waves meet only at the
// barriers around each group's staging.
#pragma once

namespace aa {

template <int KH, int TH, int TW>
__host__ __device__ constexpr size_t wg_patch_bytes() {
    return (size_t)4 * (TH + KH - 1) * (TW / 2) * 128;
}

template <int KH, int BN, int TH, int TW>
constexpr size_t wg_lds_bytes() {
    const size_t main = wg_patch_bytes<KH, TH, TW>();
    const size_t epi = (size_t)TH * TW * BN * 4;
    return main > epi ? main : epi;
}

// DIAG (tools/conv_bench_x3.hip only): bit 0 skips the staging, bit 1 the MFMA steps
template <int KH, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW, int OCC = 0,
          bool IN_SPLIT = false, bool OUT_SPLIT = false, int DIAG = 0>
__global__ __launch_bounds__(WM * WN * 64)
__attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1, OCC ? OCC : 8)))
void conv_wg(const float* __restrict__ in, int Hin, int Win, const bf16* __restrict__ wt,
             const float* __restrict__ bias, float* __restrict__ out, int Hout, int Wout, int cout_store,
             int tiles_w, int act, float alpha) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    static_assert(TW % 2 == 0 && TH % POOL == 0 && TW % POOL == 0, "pair- and pool-aligned tile");
    constexpr int NP = TW / 2;  // output column pairs per tile row
    constexpr int TP = TH * NP;  // pair-pixels per tile
    static_assert(TP <= WM * MF * 16, "tile covered by the waves' fragments");
    static_assert(CIN % 32 == 0, "C_in multiple of 32");
    constexpr int NTHR = WM * WN * 64;
    constexpr int BN = WN * NF * 16;
    constexpr int PH = TH + KH - 1;
    constexpr int PV = PH * NP;  // pair-pixels per plane
    constexpr int NG = CIN / 32;
    constexpr int NSTEP = NG * KH * 4;  // (group, kh, e)
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
        if (p >= TP) p = 0;  // padding rows: computed, never stored
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

    f32x4 acc[4][MF][NF];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[e][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    struct BSet {
        bf16x8 h[NF], l[NF];
    };
    BSet B0, B1;
    auto read_b = [&](BSet& b, int s) {
        const int soff = __builtin_amdgcn_readfirstlane((int)((cb * SLICE + s * step_stride) * 2));
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            b.h[j] = x3_wload(wrs, bofs[j], soff);
            b.l[j] = x3_wload(wrs, bofs[j] ^ 64, soff);
        }
    };
    // one step: plane e at row offset kh, B of this step in `cur`, the next
    // step's B loaded into `nxt` under this step's MFMAs; A fragments just
    // in time, two in flight
    auto step = [&](BSet& cur, BSet& nxt, int s, int kh, auto ec) {
        constexpr int e = decltype(ec)::value;
        if (s + 1 < NSTEP) read_b(nxt, s + 1);
        const int pofs = e * PV * 128 + kh * NP * 128, tv = kh * NP;
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
            typedef __attribute__((ext_vector_type(2))) int i32x2;
            const bf16x4 h = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(ars, o, wbase, 0));
            const bf16x4 l = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(ars, o + 64, wbase, 0));
            return make_float4((float)h[0] + (float)l[0], (float)h[1] + (float)l[1], (float)h[2] + (float)l[2],
                               (float)h[3] + (float)l[3]);
        } else {
            return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ars, (pix * CIN + g * 32 + cq * 4) * 4,
                                                                                     wbase, 0));
        }
    };

    read_b(B0, 0);  // its latency hides behind the first staging
    for (int g = 0; g < NG; ++g) {
        if (g > 0) __syncthreads();  // every wave is done with group g-1's planes
        // ---- stage group g: per (pair-pixel v, channel quad cq) the four
        // input columns 2 jp .. 2 jp + 3, transformed, split, into the planes ----
        constexpr int ITEMS = (DIAG & 1) ? 0 : PV * 8;
        for (int idx = threadIdx.x; idx < ITEMS; idx += NTHR) {
            const int v = idx >> 3, cq = idx & 7;
            const int R = v / NP, jp = v - (v / NP) * NP;
            const int gh = min(oh0 + R, Hin - 1);
            float4 d[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) d[c] = load4(gh, min(ow0 + 2 * jp + c, Win - 1), g, cq);
            float4 u[4];
            u[0] = make_float4(d[0].x - d[2].x, d[0].y - d[2].y, d[0].z - d[2].z, d[0].w - d[2].w);
            u[1] = make_float4(d[1].x + d[2].x, d[1].y + d[2].y, d[1].z + d[2].z, d[1].w + d[2].w);
            u[2] = make_float4(d[2].x - d[1].x, d[2].y - d[1].y, d[2].z - d[1].z, d[2].w - d[1].w);
            u[3] = make_float4(d[1].x - d[3].x, d[1].y - d[3].y, d[1].z - d[3].z, d[1].w - d[3].w);
            const int unit = (((cq >> 1) + v) & 7) << 4;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                uint32_t h0, l0, h1, l1;
                split2(u[e].x, u[e].y, h0, l0);
                split2(u[e].z, u[e].w, h1, l1);
                const int a = (e * PV + v) * 128 + unit + (cq & 1) * 8;
                *reinterpret_cast<uint2*>(patch + a) = make_uint2(h0, h1);
                *reinterpret_cast<uint2*>(patch + (a ^ 64)) = make_uint2(l0, l1);
            }
        }
        __syncthreads();
        for (int kh = 0; kh < ((DIAG & 2) ? 0 : KH); ++kh) {
            const int s0 = (g * KH + kh) * 4;
            step(B0, B1, s0, kh, std::integral_constant<int, 0>{});
            step(B1, B0, s0 + 1, kh, std::integral_constant<int, 1>{});
            step(B0, B1, s0 + 2, kh, std::integral_constant<int, 2>{});
            step(B1, B0, s0 + 3, kh, std::integral_constant<int, 3>{});
        }
    }
    __syncthreads();  // planes no longer needed: the f32 tile reuses LDS

    // ---- epilogue: output transform into the f32 tile (x3_store's swizzled
    // layout, PSH = 1: a store's 8 lanes hold every other pixel) ----
    float* E = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const int u = wn * NF * 4 + j * 4 + q;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int p = (wm * MF + i) * 16 + (lane & 15);
            if (p < TP) {
                const int r = p / NP, jp = p - (p / NP) * NP;
                const f32x4 y0 = acc[0][i][j] + acc[1][i][j] + acc[2][i][j];
                const f32x4 y1 = acc[1][i][j] - acc[2][i][j] - acc[3][i][j];
                const int px = r * TW + 2 * jp;
                *reinterpret_cast<float4*>(E + x3_eoff<BN, 1>(px, u)) = make_float4(y0[0], y0[1], y0[2], y0[3]);
                *reinterpret_cast<float4*>(E + x3_eoff<BN, 1>(px + 1, u)) = make_float4(y1[0], y1[1], y1[2], y1[3]);
            }
        }
    }
    __syncthreads();
    x3_store<TH, TW, POOL, BN, NTHR, OUT_SPLIT, false, 1>(E, bias, out, n, cb, oh0, ow0, Hout, Wout, cout_store, act,
                                                         alpha);
}

}  // namespace aa
