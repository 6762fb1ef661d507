// conv_x3pc: the fused first conv pair (3x3 C_in = 1 -> 32, then 3x3 32 -> 32
// with the 3x3 max-pool; src/identify_tracks.py:544 model.predict, model1's
// first block) as a persistent producer / consumer kernel, split-bf16.
// Diagnostic only (tools/pc_check.hip includes it after aa_cnn.hip): MEASURED
// AND REJECTED, not part of libaa.so -- profiles/r06/pc_ablations.txt.
//
// conv_x3's fused form stages a tile (log-mel patch -> first layer -> split
// activations into the swizzled patch), then runs the tile's 9 taps of MFMAs,
// then its epilogue -- phases one block runs one after the other, so the
// matrix pipe of a CU idles whenever its co-resident blocks stage or store at
// the same time (round 5: 113 us for 51 us of MFMA issue; the staging alone
// ~33 us, `profiles/r05/fused_ablations_r05.txt`).  Here one 512-thread block
// per CU walks a strided list of (window, tile) items with two roles:
//
//  * 4 consumer waves (one per SIMD, 64 pixels x 32 channels each: conv_x3's
//    MFMA loop, with the whole weight set resident in registers and A
//    fragments two ahead from the patch -- no co-resident wave covers a
//    consumer's latencies) run item k out of patch buffer k % 2 and leave
//    their f32 accumulators in epilogue tile k % 2;
//  * 4 producer waves (one per SIMD) meanwhile stage item k + 1 into the
//    other patch buffer (each producer keeps its own copy of the log-mel
//    patch, so the first layer needs no block barrier) and pool, bias,
//    activate and store item k - 1 from the other epilogue tile.
//
// The first layer's VALU / LDS work and the stores issue in the slots the
// consumers' MFMAs leave (an MFMA 16x16x32 holds the SIMD's vector issue for
// 8 of its 16 cycles).  One s_barrier per item separates the roles' buffers:
// at barrier k patch k % 2 is complete, epilogue tile (k - 1) % 2 is written
// and epilogue tile k % 2 has been drained.  LDS: 2 patches (2 x 41,216 B) +
// 2 f32 tiles (2 x 32,256 B) + 4 log-mel patches (4 x 1,600 B) = 153,344 B.
//
// Per element the arithmetic is conv_x3's (same first-layer MFMAs, same
// activation split, same tap / MFMA order, same pool and store), so the
// outputs are bit-identical to the fused conv_x3 (tools/pc_check.hip,
// tests/test_gpu_cnn.py).
#pragma once

namespace aa {

constexpr int PC_TH = 12, PC_TW = 21;                       // output tile (pool-aligned)
constexpr int PC_PH = PC_TH + 2, PC_PW = PC_TW + 2;         // first-layer patch
constexpr int PC_XW = PC_PW + 2, PC_XN = (PC_PH + 2) * PC_XW;  // log-mel patch
constexpr int PC_BN = 32;                                   // output channels (cout_pad == 32)
constexpr size_t PC_PATCH = (size_t)PC_PH * PC_PW * 128;
constexpr size_t PC_ETILE = (size_t)PC_TH * PC_TW * PC_BN * 4;
constexpr size_t PC_XBYTES = (((size_t)PC_XN * 4) + 15) & ~(size_t)15;
constexpr size_t PC_BLDS = (size_t)9 * PC_BN * 128;          // the weights, all taps
constexpr size_t PC_LDS = 2 * PC_PATCH + PC_ETILE + PC_BLDS + 4 * PC_XBYTES;
static_assert(PC_LDS <= 160 * 1024, "conv_x3pc LDS");

// DIAG (diagnostic builds, tools/pc_check.hip): bit 1 the consumers skip
// their MFMA loop, bit 2 the producers skip the first layer (outputs wrong)
// WM consumer waves (WM / 4 per SIMD) of 256 / WM pixels x 32 channels, and
// 4 producer waves; AD: A fragments in flight ahead of the MFMAs using them
template <int WM>
constexpr int pc_threads() { return (WM + 4) * 64; }
constexpr int PC_WM = 8;
constexpr int PC_THREADS = pc_threads<PC_WM>();

template <bool OUT_SPLIT, int DIAG = 0, int AD = 2, int WM = PC_WM>
__global__ __launch_bounds__(pc_threads<WM>()) __attribute__((amdgpu_waves_per_eu(WM / 4 + 1, WM / 4 + 1)))
void conv_x3pc(const float* __restrict__ in, const bf16* __restrict__ wt, const float* __restrict__ bias,
               float* __restrict__ out, int Hout, int Wout, int cout_store, int tiles_w, int tiles_per_win,
               int n_items, int act, float alpha, FirstConv fc) {
    constexpr int TH = PC_TH, TW = PC_TW, PW = PC_PW, POOL = 3, MF = 16 / WM, NF = 2, NTAP = 9, NC = WM;
    static_assert(WM == 4 || WM == 8, "4 or 8 consumer waves");
    constexpr int SLICE = PC_BN * 64;  // bf16 elements of one tap's weight slice
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const P0 = smem;
    float* const E0 = reinterpret_cast<float*>(smem + 2 * PC_PATCH);
    char* const Bs = smem + 2 * PC_PATCH + PC_ETILE;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int G = gridDim.x, b0 = blockIdx.x;
    const int nk = b0 < n_items ? (n_items - b0 + G - 1) / G : 0;
    if (nk == 0) return;  // (uniform over the block)
    auto item_pos = [&](int k, int& n, int& oh0, int& ow0) {
        const int it = b0 + k * G;
        n = it / tiles_per_win;
        const int tile = it - n * tiles_per_win;
        const int th = tile / tiles_w;
        oh0 = th * TH;
        ow0 = (tile - th * tiles_w) * TW;
    };

    if (wave < NC) {
        // ------------------------------------------------------------ consumer
        const int wm = wave, q = lane >> 4;
        int aoff[MF][8];  // fragment i's patch byte offset per swizzle residue (taps add immediates)
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int p = (wm * MF + i) * 16 + (lane & 15);
            const int pp = p >= TH * TW ? 0 : p;  // padding rows: computed, never stored
            const int r = pp / TW, c = pp - (pp / TW) * TW;
            const int abase = (r * PW + c) * 128;
#pragma unroll
            for (int rr = 0; rr < 8; ++rr) aoff[i][rr] = abase + (((pp + q + rr) & 7) << 4);
        }
        int bofs[NF];
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            const int row = j * 16 + (lane & 15);
            bofs[j] = row * 128 + (((q + row) & 7) << 4);
        }
        // B: the block's weights (9 taps x 32 channels x hi / lo, 36 KiB)
        // copied into LDS once, read one tap ahead into a 2-set register ring
        // (per tap 16 KiB of L1 reads per block otherwise); A: a 3-slot ring
        // of AD + 1 fragments, AD ahead, over the item's 36 (tap, fragment) steps --
        // one consumer wave per SIMD has no co-resident wave to cover an LDS
        // read
        {
            const __amdgpu_buffer_rsrc_t wrs = x3_wrsrc(wt);
            constexpr int U = (int)(PC_BLDS / 16);  // 16-B units
#pragma unroll
            for (int u0 = 0; u0 < U; u0 += NC * 64) {
                const int u = u0 + wave * 64 + lane;
                if (u < U)
                    *reinterpret_cast<uint4*>(Bs + u * 16) =
                        __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, u * 16, 0, 0));
            }
        }
        bf16x8 bh[2][NF], bl[2][NF];
        auto read_b = [&](int set, int t) {
            const char* bt = Bs + t * (SLICE * 2);
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                bh[set][j] = *reinterpret_cast<const bf16x8*>(bt + bofs[j]);
                bl[set][j] = *reinterpret_cast<const bf16x8*>(bt + (bofs[j] ^ 64));
            }
        };
        constexpr int NS = NTAP * MF;  // (tap, fragment) steps per item
        bf16x8 ah[AD + 1], al[AD + 1];
        auto read_a = [&](const char* patch, int st) {
            const int t = st / MF, i = st % MF;
            const int kh = t / 3, kw = t - (t / 3) * 3;
            const int toff = (kh * PW + kw) * 128, tv = kh * TW + kw;
            ah[st % (AD + 1)] = *reinterpret_cast<const bf16x8*>(patch + toff + aoff[i][tv & 7]);
            al[st % (AD + 1)] = *reinterpret_cast<const bf16x8*>(patch + toff + aoff[i][(tv + 4) & 7]);
        };
        __syncthreads();  // prologue: item 0 staged
        for (int k = 0; k <= nk; ++k) {
            if (k < nk && !(DIAG & 2)) {
                int n, oh0, ow0;
                item_pos(k, n, oh0, ow0);
                (void)n;
                (void)ow0;
                const char* patch = P0 + (k & 1) * PC_PATCH;
                f32x4 acc[MF][NF];
#pragma unroll
                for (int i = 0; i < MF; ++i)
#pragma unroll
                    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                // a wave whose fragments all lie below the conv output skips its MFMAs
                const bool idle = oh0 + (wm * MF * 16) / TW >= Hout * POOL;
                if (!idle) {
                    read_b(0, 0);
#pragma unroll
                    for (int st = 0; st < AD; ++st) read_a(patch, st);
                    if (AA_X3_PRIO > 0) __builtin_amdgcn_s_setprio(AA_X3_PRIO);
#pragma unroll
                    for (int st = 0; st < NS; ++st) {
                        const int t = st / MF, i = st % MF, sa = st % (AD + 1), sb = t & 1;
                        if (i == 0 && t + 1 < NTAP) read_b(sb ^ 1, t + 1);
                        if (st + AD < NS) read_a(patch, st + AD);
                        if constexpr (AA_PIN_X3 & 2) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int j = 0; j < NF; ++j) {
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[sb][j], ah[sa], acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[sb][j], ah[sa], acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[sb][j], al[sa], acc[i][j], 0, 0, 0);
                        }
                    }
                }
                if (AA_X3_PRIO > 0) __builtin_amdgcn_s_setprio(0);
                __syncthreads();  // (M) the producers have drained item k - 1 from E
                float* E = E0;
#pragma unroll
                for (int j = 0; j < NF; ++j) {
                    const int u = j * 4 + q;
#pragma unroll
                    for (int i = 0; i < MF; ++i) {
                        const int p = (wm * MF + i) * 16 + (lane & 15);
                        if (p < TH * TW)
                            *reinterpret_cast<float4*>(E + x3_eoff<PC_BN, 0>(p, u)) =
                                make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
                    }
                }
            } else {
                __syncthreads();  // (M)
            }
            __syncthreads();  // (end of item k)
        }
        return;
    }

    // ---------------------------------------------------------------- producer
    const int pw = wave - NC, ptid = threadIdx.x - NC * 64;
    uint32_t* const Xs = reinterpret_cast<uint32_t*>(smem + 2 * PC_PATCH + PC_ETILE + PC_BLDS + pw * PC_XBYTES);
    const int l32 = lane & 31, kg = lane >> 5;
    // first-layer weights and bias (conv_x3's AA_F1_KPACK operand layout)
    bf16x8 wa{}, wal{};
    f32x16 cbias{};
    {
        const int ch1 = 16 * ((l32 >> 2) & 1) + 4 * (l32 >> 3) + (l32 & 3);
        float w9[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) w9[t] = fc.w[ch1 * 9 + t];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            wa[j] = bf_hi(w9[j]);
            wal[j] = kg == 0 ? bf_lo(w9[j]) : j < 2 ? bf_hi(w9[8]) : j == 2 ? bf_lo(w9[8]) : (bf16)0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) cbias[r] = fc.b[16 * kg + r];
    }
    const float ae = fc.alpha;  // host: act folded to a slope in [0, 1]
    const int esz = fc.lm_f16 ? 2 : 4;
    constexpr int XU = (PC_XN + 63) / 64;  // log-mel elements per lane (7)
    constexpr int NPX = PC_PH * PW, NGRP = (NPX + 31) / 32, NU = 3;
    static_assert(NGRP <= 4 * NU, "first-layer groups per producer wave");

    // the log-mel patch of an item -> registers (loads left in flight)
    typedef uint32_t XRegs[XU + 1];  // raw f32 (or f16) bits
    auto load_x = [&](int k, XRegs& xr) {
        int n, oh0, ow0;
        item_pos(k, n, oh0, ow0);
        const __amdgpu_buffer_rsrc_t lrs = x3_wrsrc(reinterpret_cast<const char*>(in) + (size_t)n * fc.H0 * fc.W0 * esz);
        int e[XU];
#pragma unroll
        for (int u = 0; u < XU; ++u) {
            const int idx = min(u * 64 + lane, PC_XN - 1);
            const int r = idx / PC_XW, c = idx - r * PC_XW;
            e[u] = min(oh0 + r, fc.H0 - 1) * fc.W0 + min(ow0 + c, fc.W0 - 1);
        }
        // the element type decided once per item (a per-element select made
        // the compiler wait for every f16 load at once)
        if (fc.lm_f16) {
#pragma unroll
            for (int u = 0; u < XU; ++u) xr[u] = __builtin_amdgcn_raw_buffer_load_b16(lrs, e[u] * 2, 0, 0);
        } else {
#pragma unroll
            for (int u = 0; u < XU; ++u) xr[u] = __builtin_amdgcn_raw_buffer_load_b32(lrs, e[u] * 4, 0, 0);
        }
        xr[XU] = 0u;
    };
    // registers -> this wave's split log-mel patch, then the first layer into patch buffer `buf`
    auto stage = [&](int buf, XRegs& xr) {
        float xv_[XU + 1];
#pragma unroll
        for (int u = 0; u <= XU; ++u)
            xv_[u] = fc.lm_f16 ? (float)__builtin_bit_cast(_Float16, (uint16_t)xr[u]) : __builtin_bit_cast(float, xr[u]);
        if (fc.has_mag) {
#pragma unroll
            for (int u = 0; u < XU; ++u) xv_[u] = powf(xv_[u], fc.mag_exp);
        }
#pragma unroll
        for (int u = 0; u < XU; u += 2) {
            uint32_t h, l;
            split2(xv_[u], xv_[u + 1], h, l);
            const int i0 = u * 64 + lane, i1 = i0 + 64;
            if (i0 < PC_XN) Xs[i0] = __builtin_amdgcn_perm(l, h, 0x05040100u);  // hi | lo << 16
            if (u + 1 < XU && i1 < PC_XN) Xs[i1] = __builtin_amdgcn_perm(l, h, 0x07060302u);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own writes, read back by other lanes
        char* patch = P0 + buf * PC_PATCH;
        bf16x8 xh[NU], xl[NU];
        int pix[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            pix[u] = min((pw + 4 * u) * 32 + l32, NPX - 1);
            const int r = pix[u] / PW, c = pix[u] - r * PW;
            const uint32_t* xp = Xs + r * PC_XW + c;
            uint32_t xv[9];
#pragma unroll
            for (int j = 0; j < 9; ++j) xv[j] = xp[(j / 3) * PC_XW + j % 3];
            const uint32_t psel = kg ? 0x07060302u : 0x05040100u;
            uint4 b1, b2;
            b1.x = __builtin_amdgcn_perm(xv[1], xv[0], psel);
            b1.y = __builtin_amdgcn_perm(xv[3], xv[2], psel);
            b1.z = __builtin_amdgcn_perm(xv[5], xv[4], psel);
            b1.w = __builtin_amdgcn_perm(xv[7], xv[6], psel);
            b2.x = kg ? xv[8] : b1.x;
            b2.y = kg ? (xv[8] & 0xffffu) : b1.y;
            b2.z = kg ? 0u : b1.z;
            b2.w = kg ? 0u : b1.w;
            xh[u] = __builtin_bit_cast(bf16x8, b1);
            xl[u] = __builtin_bit_cast(bf16x8, b2);
        }
        f32x16 d[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, xh[u], cbias, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < NU; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wal, xl[u], d[u], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            if ((pw + 4 * u) * 32 + l32 < NPX) {
                const int R = pix[u] / PW, C = pix[u] - R * PW;
#pragma unroll
                for (int h = 0; h < 2; ++h) {  // channels 16 kg + 8 h + e: unit 2 kg + h
                    uint32_t hw[4], lw[4];
#pragma unroll
                    for (int e = 0; e < 8; e += 2) leaky_split2(d[u][8 * h + e], d[u][8 * h + e + 1], ae, hw[e >> 1], lw[e >> 1]);
                    const int a = x3_addr(R, C, 2 * kg + h, PW, TW);
                    *reinterpret_cast<uint4*>(patch + a) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                    *reinterpret_cast<uint4*>(patch + (a ^ 64)) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                }
            }
        }
    };
    const float4 bv = x3_store_bias<PC_BN, 256>(bias, 0, ptid);
    auto drain = [&](int k) {  // pool, bias, activation, store of item k from epilogue tile k % 2
        int n, oh0, ow0;
        item_pos(k, n, oh0, ow0);
        const float* E = E0;
        x3_store<TH, TW, POOL, PC_BN, 256, OUT_SPLIT, false, 0>(E, bias, out, n, 0, oh0, ow0, Hout, Wout, cout_store,
                                                               act, alpha, ptid, &bv);
    };

    // iteration k: stage item k + 1 from the registers its loads filled,
    // drain item k - 1, then issue item k + 2's loads, whose latency runs
    // while this wave waits at the barrier for the consumers' MFMAs.  (The
    // loads go last: s_waitcnt vmcnt counts loads and stores together in
    // issue order, and with loads issued ahead of a stage in the same
    // iteration the compiler's count for the stage's registers came out as
    // vmcnt(0) -- a wait for the loads just issued.)
    XRegs xr;
    load_x(0, xr);
    stage(0, xr);
    load_x(min(1, nk - 1), xr);
    __syncthreads();  // prologue: item 0 staged
    for (int k = 0; k <= nk; ++k) {
        if (k >= 1) drain(k - 1);
        if (k + 1 < nk && !(DIAG & 4)) stage((k + 1) & 1, xr);
        if (k + 2 < nk) load_x(k + 2, xr);
        __syncthreads();  // (M) E free for item k, patch k + 1 staged
        __syncthreads();  // (end of item k) E holds item k
    }
}

}  // namespace aa
