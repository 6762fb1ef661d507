// conv_wgf: MEASURED AND REJECTED (round 5: 220 us against the fused
// conv_x3's 120 us in the pipeline, profiles/r05/wgf_ablations.txt), kept
// out of libaa.so as a diagnostic for tools/wgf_check.hip, which includes it
// after aa_cnn.hip.
#pragma once

namespace aa {

// ---------------------------------------------------------------------------
// conv_wgf: the fused first layer (C_in = 1, 3x3 -> 32, folded BN,
// activation; the log-mel never leaves LDS) and the next 3x3 32 -> 32 conv +
// 3x3 max pool as F(6, 3) along W -- 4/9 of conv_x3's MFMA work for the step's
// most expensive layer pair.
//
// The Winograd input transform needs 8 adjacent columns of one channel, but
// the first layer's MFMA leaves a pixel's channels in one lane.  So the first
// layer runs transposed (A = log-mel taps of 32 pixels, B = weights: D = 32
// pixels x 32 channels, a lane = one channel, its 16 registers = 16 pixels)
// and the transform is a second MFMA whose A operand is those registers as
// they stand: a "segment" is the 8 input columns of one group-pixel (patch
// row R, column group jp); a block of 4 segments = the 32 pixels of one
// first-layer MFMA, pixel label m -> segment 2 ((m >> 2) & 1) + (r >> 3),
// column r & 7 with r = 4 (m >> 3) + (m & 3), so register r of a k-group kg
// lane holds segment 2 kg + r / 8, column r % 8, and K chunk s of the
// transform MFMA (registers 8 s .. 8 s + 7) is segment 2 kg + s's 8 columns.
// B2 [k][n2] = B^T[e][col] on the diagonal blocks (n2 = 4 e + segment): D2 =
// 32 channels x (8 planes x 4 segments), a lane = one plane of one segment,
// 16 whole channels -- two 16-B units of the plane layout, written as
// ds_write_b128.  The activations enter the transform split (bf16 hi + lo:
// two MFMAs per chunk, products exact, f32 sums), u is split again for the
// main loop (tools/wino_study.py emulates both roundings: model1 max |delta
// logit| 2.1e-4 on the bench's 64 windows, 1.9e-4 with an exact f32 transform).
//
// Main loop and epilogue are conv_wg's (KH = 3, one 32-channel group, all 8
// planes staged at once).  Planes are PS = (PV | 1) x 128 B apart (an odd
// multiple of 128 B), so the 8-lane groups of a transform write (segments
// 4b .. 4b+3 of planes e, e + 1) land in distinct bank groups.
template <int TH, int TW>
__host__ __device__ constexpr int wgf_ps() {  // plane stride in 128-B group-pixels
    return ((TH + 2) * (TW / 6)) | 1;
}
template <int TH, int TW, int BN>
constexpr size_t wgf_lds_bytes() {
    const size_t planes = (size_t)8 * wgf_ps<TH, TW>() * 128;
    const size_t x = (size_t)(TH + 4) * (TW + 4) * 4;
    const size_t epi = (size_t)TH * TW * BN * 4;
    return (planes + x) > epi ? planes + x : epi;
}

// DIAG (tools/wgf_check.hip only): bit 0 skips the first layer + transform,
// bit 1 the main loop's MFMA steps, bit 2 its B loads after the first set
template <int TH, int TW, int WM, int WN, int MF, int NF, int OCC = 0, bool OUT_SPLIT = false, int BD = 2, int NU = 2,
          int DIAG = 0>
__global__ __launch_bounds__(WM * WN * 64)
__attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1, OCC ? OCC : 8)))
void conv_wgf(const float* __restrict__ in, int Hin, int Win, const bf16* __restrict__ wt,
              const float* __restrict__ bias, float* __restrict__ out, int Hout, int Wout, int cout_store,
              int tiles_w, int act, float alpha, FirstConv fc) {
    constexpr int WO = 6, A = 8, KH = 3, POOL = 3;
    static_assert(TW % WO == 0 && TH % POOL == 0, "group- and pool-aligned tile");
    constexpr int NP = TW / WO;
    constexpr int TP = TH * NP;
    static_assert(TP <= WM * MF * 16, "tile covered by the waves' fragments");
    constexpr int NTHR = WM * WN * 64, NW = WM * WN;
    constexpr int BN = WN * NF * 16;
    static_assert(BN == 32, "32 output channels per block");
    constexpr int PH = TH + 2;
    constexpr int PV = PH * NP;  // group-pixels (= segments) per plane
    constexpr int PS = wgf_ps<TH, TW>();
    constexpr int NSB = (PV + 3) / 4;  // 4-segment blocks (first-layer MFMAs)
    constexpr int NSTEP = KH * A;
    constexpr int SLICE = BN * 64;
    constexpr int XW = TW + 4, XH = TH + 4, XN = XH * XW;  // log-mel patch (f32 pre-split)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* patch = smem;
    uint32_t* Xs = reinterpret_cast<uint32_t*>(smem + (size_t)8 * PS * 128);

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
#pragma unroll
    for (int k = 0; k < BD - 1; ++k) read_b(Bq[k], k);  // their latency hides behind the first layer
    if constexpr (DIAG & 4) {
#pragma unroll
        for (int k = BD - 1; k < BD; ++k) read_b(Bq[k], 0);
    }

    // ---- the first layer's operands: weights (B, lane = channel label l32),
    // bias (C: the lane's channel in every register), the transform (B2) ----
    const int l32 = lane & 31, kg = lane >> 5;
    const int ch1 = 16 * ((l32 >> 2) & 1) + 4 * (l32 >> 3) + (l32 & 3);
    bf16x8 wa, wal, T2[2];
    {
        float w9[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) w9[t] = fc.w[ch1 * 9 + t];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            wa[j] = bf_hi(w9[j]);
            wal[j] = kg == 0 ? bf_lo(w9[j]) : j < 2 ? bf_hi(w9[8]) : j == 2 ? bf_lo(w9[8]) : (bf16)0.f;
        }
        const int e2 = l32 >> 2, sg2 = l32 & 3;  // this lane's column of D2: plane e2, segment sg2
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) T2[s][j] = sg2 == 2 * kg + s ? bf_hi(wg_bt(WO, e2, j)) : (bf16)0.f;
    }
    const float b1 = fc.b[ch1];
    const float ae = fc.alpha;  // host: act folded to a slope in [0, 1]

    // ---- the log-mel patch, split once per element (hi | lo << 16) ----
    {
        const int esz = fc.lm_f16 ? 2 : 4;
        const __amdgpu_buffer_rsrc_t lrs =
            x3_wrsrc(reinterpret_cast<const char*>(in) + (size_t)n * fc.H0 * fc.W0 * esz);
        for (int idx = threadIdx.x; idx < XN; idx += NTHR) {
            const int r = idx / XW, c = idx - (idx / XW) * XW;
            const int e = min(oh0 + r, fc.H0 - 1) * fc.W0 + min(ow0 + c, fc.W0 - 1);
            float v = fc.lm_f16 ? (float)__builtin_bit_cast(_Float16, __builtin_amdgcn_raw_buffer_load_b16(lrs, e * 2, 0, 0))
                                : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lrs, e * 4, 0, 0));
            if (fc.has_mag) v = powf(v, fc.mag_exp);
            uint32_t h, l;
            split2(v, 0.f, h, l);
            Xs[idx] = (h & 0xffffu) | (l << 16);
        }
    }
    __syncthreads();

    // ---- first layer + transform, 4 segments per MFMA pair ----
    {
        // this lane's pixel in the first-layer MFMA (A row m = l32)
        const int r1 = 4 * (l32 >> 3) + (l32 & 3);
        const int sg1 = 2 * ((l32 >> 2) & 1) + (r1 >> 3), col1 = r1 & 7;
        const int rmax = Hin - oh0;  // patch rows past the conv input feed no output
        const uint32_t psel = kg ? 0x07060302u : 0x05040100u;
        for (int b0 = wave; b0 < ((DIAG & 1) ? 0 : NSB); b0 += NW * NU) {
            bf16x8 xh[NU], xl[NU];
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int S = min((b0 + NW * u) * 4 + sg1, PV - 1);
                const int R = S / NP, jp = S - (S / NP) * NP;
                const uint32_t* xp = Xs + R * XW + WO * jp + col1;
                uint32_t xv[9];
#pragma unroll
                for (int j = 0; j < 9; ++j) xv[j] = xp[(j / 3) * XW + j % 3];
                uint4 p1, p2;
                p1.x = __builtin_amdgcn_perm(xv[1], xv[0], psel);
                p1.y = __builtin_amdgcn_perm(xv[3], xv[2], psel);
                p1.z = __builtin_amdgcn_perm(xv[5], xv[4], psel);
                p1.w = __builtin_amdgcn_perm(xv[7], xv[6], psel);
                p2.x = kg ? xv[8] : p1.x;
                p2.y = kg ? (xv[8] & 0xffffu) : p1.y;
                p2.z = kg ? 0u : p1.z;
                p2.w = kg ? 0u : p1.w;
                xh[u] = __builtin_bit_cast(bf16x8, p1);
                xl[u] = __builtin_bit_cast(bf16x8, p2);
            }
            f32x16 d[NU];
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                f32x16 c;
#pragma unroll
                for (int r = 0; r < 16; ++r) c[r] = b1;
                d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[u], wa, c, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < NU; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl[u], wal, d[u], 0, 0, 0);
            // activation, split: the transform's A operands (chunk s = registers 8 s ..)
            f32x16 t[NU];
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                uint4 ah[2], al[2];
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    uint32_t hw[4], lw[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) leaky_split2(d[u][8 * s + 2 * k], d[u][8 * s + 2 * k + 1], ae, hw[k], lw[k]);
                    ah[s] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                    al[s] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                }
                f32x16 z{};
                t[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ah[0]), T2[0], z, 0, 0, 0);
                t[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, al[0]), T2[0], t[u], 0, 0, 0);
                t[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ah[1]), T2[1], t[u], 0, 0, 0);
                t[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, al[1]), T2[1], t[u], 0, 0, 0);
            }
            // D2 lane (n2 = 4 e + segment, kg): channels 16 kg + r of plane e
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int S = (b0 + NW * u) * 4 + (l32 & 3), e = l32 >> 2;
                if (b0 + NW * u < NSB && S < PV && S / NP < rmax) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        uint32_t hw[4], lw[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) split2(t[u][8 * h + 2 * k], t[u][8 * h + 2 * k + 1], hw[k], lw[k]);
                        const int a = (e * PS + S) * 128 + (((2 * kg + h + S) & 7) << 4);
                        *reinterpret_cast<uint4*>(patch + a) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                        *reinterpret_cast<uint4*>(patch + (a ^ 64)) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                    }
                }
            }
        }
    }
    __syncthreads();

    // ---- main loop: conv_wg's steps (plane e at row offset kh) ----
    f32x4 acc[A][MF][NF];
#pragma unroll
    for (int e = 0; e < A; ++e)
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[e][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto step = [&](auto bc, int s, int kh, auto ec) {
        constexpr int e = decltype(ec)::value;
        constexpr int b = decltype(bc)::value;
        BSet& cur = Bq[b];
        if (!(DIAG & 4) && s + BD - 1 < NSTEP) read_b(Bq[(b + BD - 1) % BD], s + BD - 1);
        const int pofs = e * PS * 128 + kh * NP * 128, tv = kh * NP;
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
    // a wave whose fragments all lie in tile rows past the conv output (the
    // bottom tile of a tall tile) skips its MFMAs: those outputs are discarded
    const bool wave_idle = oh0 + (wm * MF * 16) / NP >= Hout * POOL || (DIAG & 2);
    if (!wave_idle) {
        if constexpr (AA_WG_PRIO > 0) __builtin_amdgcn_s_setprio(AA_WG_PRIO);
        for (int kh = 0; kh < KH; ++kh) {
            wg_static_for<0, A>([&](auto ec) {
                constexpr int e = decltype(ec)::value;
                // 8 steps per row: the B sets alternate the same way every row
                step(std::integral_constant<int, e % BD>{}, kh * A + e, kh, ec);
            });
        }
        if constexpr (AA_WG_PRIO > 0) __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();  // planes no longer needed: the f32 tile reuses LDS

    // ---- epilogue: output transform into the f32 tile, pool, bias, act, store ----
    constexpr int PSH = wg_psh(WO);
    float* E = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const int u = wn * NF * 4 + j * 4 + q;
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
                    *reinterpret_cast<float4*>(E + x3_eoff<BN, PSH>(px + k, u)) = make_float4(y[0], y[1], y[2], y[3]);
                }
            }
        }
    }
    __syncthreads();
    x3_store<TH, TW, POOL, BN, NTHR, OUT_SPLIT, false, PSH>(E, bias, out, n, cb, oh0, ow0, Hout, Wout, cout_store,
                                                           act, alpha);
}

}  // namespace aa
