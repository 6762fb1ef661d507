// The network's tail in one launch (AA_PREC_BF16X3): the last conv stage
// (kernel KH x KW, C_in = CIN, 256 output channels, bias + activation, no
// pool) and the 1x1 head that follows it (up to 32 labels) with its global
// max, for the reference family's model shape (src/identify_tracks.py:302-327:
// conv 1x3 -> 256, conv 1x1 -> labels, GlobalMaxPool2D, sigmoid).  Included
// by aa_cnn.hip after aa_conv_x3.h (shares its swizzle, weight packing, the
// grouped-split staging and x3_wload).
//
// Separately the conv writes 13 x 20 x 256 f32 per window to HBM and the head
// reads it back (two launches plus the head's partial-max pass); here:
//
//  * one block per (window, TH x TW tile), 8 waves; wave w owns output
//    channels 32 w .. 32 w + 31 (NF = 2 fragments of 16) for all MF pixel
//    fragments of the tile;
//  * all CIN / 32 channel groups of the input patch are staged at once by
//    global_load_lds from the grouped-split layout (one latency, not one
//    per group), each group in its own swizzled 128-B-per-pixel image;
//  * the conv: implicit GEMM on v_mfma_f32_16x16x32_bf16 x 3 (hi.hi, lo.hi,
//    hi.lo), B fragments per wave from L2 one step ahead, A just in time;
//  * the head straight from the accumulators: a lane holds channels
//    {4q..4q+3, 16+4q..16+4q+3} of its wave's 32 for one pixel, which after
//    bias, activation and the hi / lo split IS the B operand of a 16x16x32
//    MFMA whose K runs over those 32 channels (the head weights are packed
//    on the host in the same k order), so each wave forms its channels'
//    partial head logits for every label and pixel with 6 MFMAs per pixel
//    fragment;
//  * the 8 partial sums meet in LDS in a fixed order (waves 0-3 store, 4-7
//    add, then one pass sums the 4 slots): deterministic, no atomics; the
//    maximum over the tile's valid pixels goes to part[n][tile][32], which
//    head_final reduces over tiles (+ bias, activation, sigmoid) as for
//    conv_head.
#pragma once

namespace aa {

constexpr int TAIL_NW = 8;     // waves per block
constexpr int TAIL_COUT = 256;  // conv output channels (32 per wave)
#ifndef TAIL_BD
#define TAIL_BD 2  // B register sets in flight (prefetch distance + 1; 4 measured neutral)
#endif
constexpr int TAIL_SSTR = 36;   // floats per pixel row of a partial-sum slot (32 labels + 4: conflict-free)

template <int KH, int KW, int CIN, int TH, int TW>
__host__ __device__ constexpr size_t tail_lds_bytes() {
    const size_t patch = (size_t)(CIN / 32) * (TH + KH - 1) * (TW + KW - 1) * 128;
    const size_t slots = (size_t)4 * TH * TW * TAIL_SSTR * 4;
    return patch > slots ? patch : slots;
}

template <int KH, int KW, int CIN, int MF, int TH, int TW>
__global__ __launch_bounds__(TAIL_NW * 64) void conv_tail_x3(
    const float* __restrict__ in, int Hin, int Win, const bf16* __restrict__ wt, const float* __restrict__ bias,
    int Hc, int Wc, int tiles_w, int act, float alpha, const bf16* __restrict__ hw /*[8][2][64][8] hi then lo*/,
    float* __restrict__ part) {
    static_assert(TH * TW <= MF * 16, "tile covered by the pixel fragments");
    static_assert(CIN % 32 == 0 && (KW - 1) % 2 == 0, "C_in multiple of 32, odd kernel width");
    constexpr int NTHR = TAIL_NW * 64;
    constexpr int PH = TH + KH - 1, PW = TW + KW - 1;
    constexpr int NTAP = KH * KW, NG = CIN / 32, NSTEP = NTAP * NG;
    constexpr int GIMG = PH * PW * 128;                 // bytes of one group's patch image
    constexpr int SLICE = TAIL_COUT * 64;               // bf16 elements of one step's weights
    constexpr int TP = TH * TW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* patch = smem;

    const int tile = blockIdx.x, n = blockIdx.z;
    const int th = tile / tiles_w, tw = tile - (tile / tiles_w) * tiles_w;
    const int oh0 = th * TH, ow0 = tw * TW;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, q = lane >> 4;

    // ---- stage every channel group's patch image (grouped-split input) ----
    {
        const __amdgpu_buffer_rsrc_t ars = x3_wrsrc(reinterpret_cast<const char*>(in) + (size_t)n * Hin * Win * CIN * 4);
        constexpr int UNITS = PH * PW * 8;
        for (int i0 = wave * 64; i0 < UNITS; i0 += NTHR) {
            const int idx = i0 + lane;
            if (idx < UNITS) {
                const int pix = idx >> 3, slot = idx & 7;
                const int R = pix / PW, C = pix - R * PW;
                const int u = (slot - R * TW - C) & 7;
                const int gh = min(oh0 + R, Hin - 1), gw = min(ow0 + C, Win - 1);
#pragma unroll
                for (int g = 0; g < NG; ++g)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        ars, (__attribute__((address_space(3))) void*)(patch + g * GIMG + i0 * 16), 16,
                        (gh * Win + gw) * (CIN * 4) + u * 16, g * 128, 0, 0);
            }
        }
    }

    // per-lane fragment geometry (aa_conv_x3.h): pixel fragment i, B rows of this wave
    int abase[MF], aph[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        int p = i * 16 + (lane & 15);
        // padding rows (computed, never used): the pixel 16 k back, whose
        // swizzle slot is the lane's own (no second address on a busy slot)
        if (p >= TP) p = max(p - 16 * ((p - TP) / 16 + 1), 0);
        const int r = p / TW, c = p - (p / TW) * TW;
        abase[i] = (r * PW + c) * 128;
        aph[i] = p + q;
    }
    int bofs[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int row = wave * 32 + j * 16 + (lane & 15);
        bofs[j] = row * 128 + (((q + row) & 7) << 4);
    }
    const __amdgpu_buffer_rsrc_t wrs = x3_wrsrc(wt);
    struct BSet {
        bf16x8 h[2], l[2];
    };
    auto read_b = [&](BSet& b, int s) {
        const int soff = __builtin_amdgcn_readfirstlane(s * SLICE * 2);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            b.h[j] = x3_wload(wrs, bofs[j], soff);
            b.l[j] = x3_wload(wrs, bofs[j] ^ 64, soff);
        }
    };
    f32x4 acc[MF][2];
#pragma unroll
    for (int i = 0; i < MF; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};

    // B fragments BD - 1 steps ahead in a register ring (two waves per SIMD
    // leave few other waves to hide the L2 latency of the per-step loads)
    constexpr int BD = TAIL_BD;
    BSet Bq[BD];
#pragma unroll
    for (int s = 0; s < BD - 1; ++s)
        if (s < NSTEP) read_b(Bq[s], s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's patch pieces (and the first B sets) landed
    __syncthreads();

    auto step = [&](int s) {
        BSet& cur = Bq[s % BD];
        const int g = s / NTAP, t = s - (s / NTAP) * NTAP;
        if (s + BD - 1 < NSTEP) read_b(Bq[(s + BD - 1) % BD], s + BD - 1);
        const int kh = t / KW, kw = t - (t / KW) * KW;
        const int toff = g * GIMG + (kh * PW + kw) * 128, tv = kh * TW + kw;
        bf16x8 h2[2], l2[2];
        auto rd = [&](int i, int k) {
            const int a = abase[i] + toff + (((aph[i] + tv) & 7) << 4);
            h2[k] = *reinterpret_cast<const bf16x8*>(patch + a);
            l2[k] = *reinterpret_cast<const bf16x8*>(patch + (a ^ 64));
        };
        rd(0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            if (i + 1 < MF) rd(i + 1, (i + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.h[j], h2[i & 1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.l[j], h2[i & 1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.h[j], l2[i & 1], acc[i][j], 0, 0, 0);
            }
        }
    };
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) step(s);

    // ---- head: bias + activation + split of the accumulators = B operand ----
    // lane k-slot 8 q + e <-> channel 32 wave + (e < 4 ? 4 q + e : 16 + 4 q + e - 4)
    float bv[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        bv[e] = bias[wave * 32 + 4 * q + e];
        bv[4 + e] = bias[wave * 32 + 16 + 4 * q + e];
    }
    const __amdgpu_buffer_rsrc_t hrs = x3_wrsrc(hw);
    bf16x8 whh[2], whl[2];  // head weights of label fragments 0 / 1 (A operand), hi / lo
#pragma unroll
    for (int lf = 0; lf < 2; ++lf) {
        const int o = (((wave * 2 + lf) * 2) * 64 + lane) * 16;
        whh[lf] = x3_wload(hrs, o, 0);
        whl[lf] = x3_wload(hrs, o + 64 * 16, 0);
    }
    f32x4 D[MF][2];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        uint32_t h[4], l[4];
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
            split2(apply_act(acc[i][0][e] + bv[e], act, alpha), apply_act(acc[i][0][e + 1] + bv[e + 1], act, alpha),
                   h[e >> 1], l[e >> 1]);
            split2(apply_act(acc[i][1][e] + bv[4 + e], act, alpha),
                   apply_act(acc[i][1][e + 1] + bv[4 + e + 1], act, alpha), h[2 + (e >> 1)], l[2 + (e >> 1)]);
        }
        const bf16x8 xh = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
        const bf16x8 xl = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
#pragma unroll
        for (int lf = 0; lf < 2; ++lf) {
            f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whh[lf], xh, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whl[lf], xh, d, 0, 0, 0);
            D[i][lf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whh[lf], xl, d, 0, 0, 0);
        }
    }
    // ---- partial sums of the 8 waves in a fixed order ----
    __syncthreads();  // patch images no longer needed: the slots reuse LDS
    float* S = reinterpret_cast<float*>(smem);
    const int slot = wave & 3;
    if (wave >= 4) __syncthreads();
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        const int p = i * 16 + (lane & 15);
        if (p < TP) {
#pragma unroll
            for (int lf = 0; lf < 2; ++lf) {
                float4* d = reinterpret_cast<float4*>(S + ((size_t)slot * TP + p) * TAIL_SSTR + lf * 16 + 4 * q);
                const f32x4 v = D[i][lf];
                if (wave < 4) {
                    *d = make_float4(v[0], v[1], v[2], v[3]);
                } else {
                    const float4 a = *d;
                    *d = make_float4(a.x + v[0], a.y + v[1], a.z + v[2], a.w + v[3]);
                }
            }
        }
    }
    if (wave < 4) __syncthreads();
    __syncthreads();
    // ---- the tile's column maxima over its valid pixels ----
    const int lab = threadIdx.x & 31, strip = threadIdx.x >> 5;  // 16 strips of pixels
    constexpr int NSTRIP = NTHR / 32, PPS = (TP + NSTRIP - 1) / NSTRIP;
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < PPS; ++k) {
        const int p = strip * PPS + k;
        if (p < TP) {
            const int r = p / TW, c = p - (p / TW) * TW;
            if (oh0 + r < Hc && ow0 + c < Wc) {
                const float* sp = S + (size_t)p * TAIL_SSTR + lab;
                const float v = ((sp[0] + sp[(size_t)TP * TAIL_SSTR]) + sp[(size_t)2 * TP * TAIL_SSTR]) +
                                sp[(size_t)3 * TP * TAIL_SSTR];
                m = fmaxf(m, v);
            }
        }
    }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    __syncthreads();
    float* red = S;  // the slots are consumed
    if (lane < 32) red[wave * 32 + lab] = m;
    __syncthreads();
    if (threadIdx.x < 32) {
        float v = red[threadIdx.x];
#pragma unroll
        for (int w = 1; w < TAIL_NW; ++w) v = fmaxf(v, red[w * 32 + threadIdx.x]);
        part[((size_t)n * gridDim.x + tile) * 32 + threadIdx.x] = v;
    }
}

}  // namespace aa
