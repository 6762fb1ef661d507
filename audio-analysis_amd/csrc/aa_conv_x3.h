// Split-bf16 implicit-GEMM convolution (AA_PREC_BF16X3), included by
// aa_cnn.hip after conv_mfma (shares FirstConv, wait_vm_lgkm, bf_hi/bf_lo).
//
// Same GEMM as conv_mfma -- M = output pixels of a TH x TW tile, N = output
// channels, K = taps x C_in, D = W X^T on v_mfma_f32_16x16x32_bf16 -- with
// every operand split into bf16 hi + lo and each product formed as
// hi*hi + hi*lo + lo*hi (three MFMAs, f32 accumulation).  What differs is the
// LDS image, shaped by the split's doubled operand bytes:
//
//  * Channel groups.  C_in is consumed 32 channels at a time: the patch of
//    group g is staged, its KH*KW taps run, then group g+1 replaces it.  The
//    patch therefore holds 32 channels (hi + lo = 128 B per pixel) whatever
//    C_in is, so a block stays under 80 KiB and two blocks share a CU: one
//    block's staging overlaps the other's MFMAs.
//  * No padding, a rotation swizzle instead.  Pixel (R, C) of the patch is
//    stored at (R*PW + C) * 128 B; its 16-B unit u (hi: channels 8u..8u+7,
//    u = 0..3; lo: u = 4..7) sits in slot (u + R*TW + C) & 7.  A fragment's
//    16 lanes read 16 consecutive TILE pixels p, whose v = R*TW + C = p +
//    kh*TW + kw is consecutive even where the run wraps a tile row, and
//    whose pixel parity follows v (KW - 1 is even), so every ds_read_b128
//    lane group hits 16 distinct 4-bank groups for every tap and tile width
//    (a padded row only achieves that for runs that do not wrap).
//  * Weights packed per (group, tap) step as [cout][8 units] with unit u of
//    row o in slot (u + o) & 7: the same conflict-free read for B fragments;
//    a block's slice of a step is BN * 128 contiguous bytes, streamed by
//    global_load_lds through the LDS ring as in conv_mfma.
//  * Pre-split activations between conv_x3 stages (IN_SPLIT / OUT_SPLIT).
//    A stage whose consumer is another conv_x3 stage writes its output
//    already split, as the "grouped split" HBM layout: per pixel, per
//    32-channel group, 64 B of bf16 hi then 64 B of bf16 lo (the same 4 B per
//    element as f32).  The consumer then stages a group's patch with
//    global_load_lds alone -- lane i of a wave-instruction lands at LDS byte
//    16 i, and the per-lane GLOBAL address picks the unit that belongs in
//    that swizzled slot -- no VALU split, no ds_write, no register round trip.
#pragma once

namespace aa {

constexpr int X3_CG = 32;  // channels per staged group

// Build switches kept for in-pipeline A/B runs (tools/ab_build.py AB_DEFS):
// AA_X3_XSPLIT: the fused first layer's log-mel patch split into bf16 hi / lo
// once per element as it is staged, instead of once per tap read;
// AA_X3_REMAP: XCD-aware block order (x3_block) for conv_x3 as for conv_wg.
#ifndef AA_X3_XSPLIT
#define AA_X3_XSPLIT 1
#endif
#ifndef AA_X3_REMAP
#define AA_X3_REMAP 1
#endif
// AA_F1_KPACK: the fused first layer's 27 split products (hi.hi, hi.lo,
// lo.hi over 9 taps) in 2 MFMAs instead of 3; AA_X3_SCALAR_SPLIT: its
// activation / split in scalar f32 ops (packed f32 VALU costs extra issue
// beside MFMAs).  Together: fused conv 136 -> 126 us in the pipeline
// (harness 140 -> 132 us; each alone within the noise).
#ifndef AA_F1_KPACK
#define AA_F1_KPACK 1
#endif
#ifndef AA_X3_SCALAR_SPLIT
#define AA_X3_SCALAR_SPLIT 1
#endif

// Scheduling pins for the kernels whose waves load their own B fragments
// from global memory (conv_x3 with RING = false, conv_wg).  Bit 0: the next
// step's fragment loads are issued before this step's MFMAs; bit 1: fragment
// i+1's just-in-time A read before fragment i's MFMAs.  Without them the
// scheduler sinks the prefetches down to their first use and the wave waits
// out the L2 latency every step (s_waitcnt vmcnt(0) right after the issue,
// tools/isa_stats.py).  In-pipeline A/B: fused first conv 153 -> 147 us,
// Winograd 9x3 152 -> 138 us; the ring kernels (LDS-staged B, a barrier per
// step) lose with either pin (3x3/64: 52 -> 58 / 71 us), so they stay unpinned.
#ifndef AA_PIN_X3
#define AA_PIN_X3 3
#endif
// MFMA steps at issue priority 1 (s_setprio) in conv_x3 and conv_wg: in-pipeline
// A/B, 3 rounds on one box, step 259.2k -> 261.6k audio-s/s (both) -- the
// other batch's front end and the co-resident blocks' staging VALU fill the
// slots the matrix pipe leaves instead of delaying its issue
#ifndef AA_X3_PRIO
#define AA_X3_PRIO 1
#endif
#ifndef AA_WG_PRIO
#define AA_WG_PRIO 1
#endif
#ifndef AA_PIN_WG
#define AA_PIN_WG 3
#endif

template <int KH, int KW, int TH, int TW, bool FUSED>
__host__ __device__ constexpr size_t x3_patch_bytes() {
    size_t b = (size_t)(TH + KH - 1) * (TW + KW - 1) * 128;
    if (FUSED) b += ((sizeof(float) * (TH + KH + 1) * (TW + KW + 1)) + 15) & ~(size_t)15;
    return b;
}

template <int KH, int KW, int BN, int TH, int TW, bool FUSED>
constexpr size_t x3_lds_bytes_nb(int nb) {  // nb = 0: no LDS ring (B fragments from global)
    const size_t main = x3_patch_bytes<KH, KW, TH, TW, FUSED>() + (size_t)nb * BN * 128;
    const size_t epi = (size_t)TH * TW * BN * 4;
    return main > epi ? main : epi;
}

// ring depth: as in conv_ring, deepen while the blocks per CU a 3-deep ring
// allows stay resident (at most AA_X3_RING_MAX slices, one per step)
#ifndef AA_X3_RING_MAX
#define AA_X3_RING_MAX 8
#endif
template <int KH, int KW, int CIN, int BN, int TH, int TW, bool FUSED, bool RING = true>
constexpr int x3_ring() {
    if (!RING) return 0;
    constexpr size_t cap = 160 * 1024;
    constexpr int NSTEP = KH * KW * (CIN / X3_CG);
    const size_t blocks = cap / x3_lds_bytes_nb<KH, KW, BN, TH, TW, FUSED>(3);
    int nb = 3;  // the pipelined loop reads slice s+1 while s+NB-1 is issued
    while (nb < AA_X3_RING_MAX && nb < NSTEP && blocks * x3_lds_bytes_nb<KH, KW, BN, TH, TW, FUSED>(nb + 1) <= cap)
        ++nb;
    return nb;
}

template <int KH, int KW, int CIN, int BN, int TH, int TW, bool FUSED, bool RING = true>
constexpr size_t x3_lds_bytes() {
    return x3_lds_bytes_nb<KH, KW, BN, TH, TW, FUSED>(x3_ring<KH, KW, CIN, BN, TH, TW, FUSED, RING>());
}

template <int KH, int KW, int CIN, int WM, int WN, int NF, int TH, int TW, bool FUSED, bool RING>
constexpr int x3_waves_per_simd() {
    constexpr size_t lds = x3_lds_bytes<KH, KW, CIN, WN * NF * 16, TH, TW, FUSED, RING>();
    constexpr int blocks = (int)((160 * 1024) / lds);
    constexpr int w = (blocks * WM * WN + 3) / 4;
    return w < 1 ? 1 : (w > 8 ? 8 : w);
}

// Two f32 values as packed bf16 hi and lo words (5 VALU ops)
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& hi, uint32_t& lo) {
    typedef __attribute__((ext_vector_type(2))) float f2;
    typedef __attribute__((ext_vector_type(2))) __bf16 b2;
    const f2 o = f2{x0, x1};
    hi = __builtin_bit_cast(uint32_t, __builtin_convertvector(o, b2));
    const f2 hf = f2{__uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(o - hf, b2));
}

// Two activations max(x, a x) (0 <= a <= 1) as packed bf16 hi and lo
// words, in 8 VALU ops: two multiplies, two raw maxes, one packed conversion
// for hi, its two halves back to f32 (shift / mask), two subtracts, one
// packed conversion for lo.  The max is v_med3_f32(x, a x, +inf) through the
// builtin: max(x, a x) for every non-NaN x (the inputs are MFMA results),
// without the NaN canonicalisation a plain fmaxf adds, and -- unlike the
// inline-asm v_max_f32 of round 5 -- visible to the hazard recognizer, which
// pads the first VALU read of an MFMA result with the wait states the matrix
// pipe needs (an asm read right behind the MFMA took stale registers in
// the round-5 conv_wgf).  AA_X3_SCALAR_SPLIT 0: the multiply as one packed op.
__device__ __forceinline__ void leaky_split2(float x0, float x1, float a, uint32_t& hi, uint32_t& lo) {
    typedef __attribute__((ext_vector_type(2))) float f2;
    typedef __attribute__((ext_vector_type(2))) __bf16 b2;
    constexpr float inf = __builtin_inff();
#if AA_X3_SCALAR_SPLIT
    const float r0 = x0 * a, r1 = x1 * a;
#else
    const f2 r = f2{x0, x1} * a;
    const float r0 = r.x, r1 = r.y;
#endif
    const float o0 = __builtin_amdgcn_fmed3f(x0, r0, inf);
    const float o1 = __builtin_amdgcn_fmed3f(x1, r1, inf);
    hi = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{o0, o1}, b2));
    // (scalar subtracts: aa_cnn.hip is built with -fno-slp-vectorize, which
    // keeps them from being packed into v_pk_add_f32 -- an expensive issue
    // beside MFMAs: fused conv 127 -> 120 us, profiles/r06/ab_slp.txt)
    const float s0 = o0 - __uint_as_float(hi << 16);
    const float s1 = o1 - __uint_as_float(hi & 0xffff0000u);
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{s0, s1}, b2));
}

// byte offset of unit u of patch pixel (R, C)
__device__ __forceinline__ int x3_addr(int R, int C, int u, int PW, int TW) {
    return (R * PW + C) * 128 + (((u + R * TW + C) & 7) << 4);
}

// XCD-aware block order (split-bf16 kernels): the dispatcher places block L
// (linear id) on XCD L % 8, so consecutive linear ids land on different L2s.
// Renumber so each XCD works through a contiguous range of (window, tile,
// channel block) with the channel block fastest: the blocks that stage the
// same input patch (all channel blocks of a tile) and its neighbours (the
// next tiles, which share the halo) meet in the same L2.  In-pipeline A/B:
// the Winograd 9x3 kernel (two channel blocks per tile) gains a little; the
// conv_x3 kernels lost 0.8 % of the step with it at first and gained 0.3 %
// (3 of 3 rounds) after the later occupancy and first-layer changes, so they
// remap too (AA_X3_REMAP).
struct BlockPos {
    int tile, cb, n;
};
template <bool REMAP>
__device__ __forceinline__ BlockPos x3_block() {
    const int gx = gridDim.x, gy = gridDim.y, G = gx * gy * gridDim.z;
    int L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    if (REMAP && (G & 7) == 0) L = (L & 7) * (G >> 3) + (L >> 3);
    BlockPos b;
    b.cb = L % gy;
    const int r = L / gy;
    b.tile = r % gx;
    b.n = r / gx;
    return b;
}

// A weight fragment (16 B) through a buffer resource over the packed weights:
// the per-lane part of the address (row, swizzled unit) is a VGPR that stays
// fixed across steps, the step's slice base a wave-uniform SGPR offset -- no
// 64-bit address arithmetic per load in the unrolled step loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t x3_wrsrc(const void* wt) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(wt), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ bf16x8 x3_wload(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

// Epilogue shared by the split-bf16 kernels.  The f32 tile E holds TH*TW
// pixels of BN channels (bias not yet added), no padding: the 16-B unit u
// (channels 4u..4u+3) of pixel p sits in slot (u + (p >> PSH)) mod U of the
// pixel's row, U = BN / 4.  A producer lane writes one unit of 8 pixels p
// (PSH = 0: consecutive; PSH = 1: every other one, the Winograd pairs) per
// 8-lane ds_write_b128 group, so the 8 units land in 8 distinct 16-B bank
// groups.  The reader takes one (pooled pixel, unit) item per lane and lays
// the items out along ds_read_b128's 16-lane groups ({0-3,12-15,20-27},
// {4-11,16-19,28-31} and the same +32): one group reads U units of 16 / U
// pooled pixels whose rows alternate between the two 128-B halves of the
// 256-B bank space (their pixel indices differ by an odd count for POOL 1 and
// 3), so every read is conflict-free.  Then POOL x POOL max, bias,
// activation, and the NHWC store (f32, or the grouped-split layout when
// OUT_SPLIT).
template <int BN, int PSH>
__device__ __forceinline__ int x3_eoff(int p, int u) {  // float offset of unit u of pixel p
    constexpr int U = BN / 4;
    return p * BN + (((u + (p >> PSH)) & (U - 1)) << 2);
}

// the bias quad x3_store's thread tid applies (its channel unit is fixed)
template <int BN, int NTHR>
__device__ __forceinline__ float4 x3_store_bias(const float* __restrict__ bias, int cb, int tid) {
    constexpr int U = BN / 4, NG16 = NTHR / 16, GPP = U >= 16 ? U / 16 : 1;
    const int lane = tid & 63, wave = tid >> 6;
    const int a = (lane >> 2) & 7;
    const int gi = 4 * wave + (__builtin_popcount(a) & 1) + 2 * (lane >> 5);
    const int k = ((a >> 1) << 2) | (lane & 3);
    const int u = U >= 16 ? (gi % GPP) * 16 + k : (k & 7);
    (void)NG16;
    return *reinterpret_cast<const float4*>(bias + cb * BN + u * 4);
}

template <int TH, int TW, int POOL, int BN, int NTHR, bool OUT_SPLIT, bool NOSTORE, int PSH>
__device__ __forceinline__ void x3_store(const float* E, const float* __restrict__ bias, float* __restrict__ out, int n,
                                         int cb, int oh0, int ow0, int Hout, int Wout, int cout_store, int act,
                                         float alpha, int tid = -1, const float4* bias_pre = nullptr) {
    // tid: the thread's index among the NTHR storing threads (default: the
    // block's thread index; the producer waves of conv_x3pc pass their own,
    // with the thread's bias quad loaded once (bias_pre, x3_store_bias):
    // a bias load here would make the stores' s_waitcnt vmcnt also wait for
    // every load the wave issued before it)
    if (tid < 0) tid = threadIdx.x;
    constexpr int U = BN / 4;
    static_assert(U >= 8 && (U & (U - 1)) == 0, "a power-of-two count (>= 8) of units per pixel");
    static_assert(POOL == 1 || POOL % 2 == 1, "odd pool: neighbouring items alternate row parity");
    constexpr int PHo = TH / POOL, PWo = TW / POOL, NPO = PHo * PWo;
    // a 16-lane read group covers 2 pooled pixels x 8 units (U = 8) or 16
    // units of one pooled pixel (U >= 16: GPP groups per pooled pixel)
    constexpr int NG16 = NTHR / 16, GPP = U >= 16 ? U / 16 : 1;
    static_assert(NG16 % GPP == 0, "a lane keeps its unit across passes");
    const int lane = tid & 63, wave = tid >> 6;
    const int a = (lane >> 2) & 7;
    const int gi = 4 * wave + (__builtin_popcount(a) & 1) + 2 * (lane >> 5);
    const int k = ((a >> 1) << 2) | (lane & 3);
    const int u = U >= 16 ? (gi % GPP) * 16 + k : (k & 7);
    const int qo0 = U >= 16 ? gi / GPP : 2 * gi + (k >> 3);
    constexpr int QSTEP = U >= 16 ? NG16 / GPP : 2 * NG16;
    const int ch0 = cb * BN + u * 4;
    const float4 bv = bias_pre ? *bias_pre : *reinterpret_cast<const float4*>(bias + ch0);  // bias is padded to cout_pad
    const int oh0s = oh0 / POOL, ow0s = ow0 / POOL;
    for (int qo = qo0; qo < NPO; qo += QSTEP) {
        const int pr = qo / PWo, pc = qo - (qo / PWo) * PWo;
        const int gh = oh0s + pr, gw = ow0s + pc;
        // whole-vector max: per-component fmaxf lets the compiler scalarise
        // the loads into ds_read2_b32 pairs
        f32x4 m = *reinterpret_cast<const f32x4*>(E + x3_eoff<BN, PSH>(pr * POOL * TW + pc * POOL, u));
#pragma unroll
        for (int dy = 0; dy < POOL; ++dy)
#pragma unroll
            for (int dx = (dy == 0); dx < POOL; ++dx) {
                const int p = (pr * POOL + dy) * TW + pc * POOL + dx;
                m = __builtin_elementwise_max(m, *reinterpret_cast<const f32x4*>(E + x3_eoff<BN, PSH>(p, u)));
            }
        float4 v = make_float4(m[0], m[1], m[2], m[3]);
        if (gh >= Hout || gw >= Wout) continue;
        v.x = apply_act(v.x + bv.x, act, alpha);
        v.y = apply_act(v.y + bv.y, act, alpha);
        v.z = apply_act(v.z + bv.z, act, alpha);
        v.w = apply_act(v.w + bv.w, act, alpha);
        if constexpr (NOSTORE) {
            if (v.x != 12345.f) continue;  // keep the values live, store (almost) never
        }
        if constexpr (OUT_SPLIT) {
            // grouped split: 4 channels of group ch0 / 32 -> 8 B of the hi half
            // and 8 B of the lo half (cout_store % 32 == 0, planner-checked)
            if (ch0 < cout_store) {
                char* o = reinterpret_cast<char*>(out) + ((size_t)n * Hout * Wout + (size_t)gh * Wout + gw) * cout_store * 4 +
                          (ch0 >> 5) * 128 + (ch0 & 31) * 2;
                uint32_t h0, l0, h1, l1;
                split2(v.x, v.y, h0, l0);
                split2(v.z, v.w, h1, l1);
                *reinterpret_cast<uint2*>(o) = make_uint2(h0, h1);
                *reinterpret_cast<uint2*>(o + 64) = make_uint2(l0, l1);
            }
        } else {
            float* o = out + ((size_t)n * Hout * Wout + (size_t)gh * Wout + gw) * cout_store + ch0;
            if (ch0 + 4 <= cout_store) {
                *reinterpret_cast<float4*>(o) = v;
            } else {
                const float vv[4] = {v.x, v.y, v.z, v.w};
                for (int c = 0; c < 4 && ch0 + c < cout_store; ++c) o[c] = vv[c];
            }
        }
    }
}

// RING = false: no weight ring and no per-step barrier -- every wave loads
// its own B fragments (its NF x 16 output-channel rows of the step) straight
// from global memory (L2-resident weights) one step ahead, so waves only
// synchronise at the two barriers around each group's staging.
// AJIT: A fragments read just in time inside the step (fewer VGPRs) instead
// of a whole next-step set prefetched; OCC > 0 pins the waves per SIMD the
// compiler must fit (its VGPR budget), 0 leaves it free up to the LDS limit.
template <int KH, int KW, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW, bool FUSED = false,
          int DIAG = 0, bool RING = true, bool AJIT = false, int OCC = 0, bool IN_SPLIT = false,
          bool OUT_SPLIT = false>
__global__ __launch_bounds__(WM * WN * 64)
__attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1,
                                    OCC ? OCC : x3_waves_per_simd<KH, KW, CIN, WM, WN, NF, TH, TW, FUSED, RING>())))
void conv_x3(const float* __restrict__ in, int Hin, int Win, const bf16* __restrict__ wt,
             const float* __restrict__ bias, float* __restrict__ out, int Hout, int Wout, int cout_store,
             int tiles_w, int act, float alpha, FirstConv fc) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    static_assert(TH % POOL == 0 && TW % POOL == 0, "pool-aligned tile");
    static_assert(TH * TW <= WM * MF * 16, "tile covered by the waves' fragments");
    static_assert(CIN % X3_CG == 0, "C_in multiple of 32");
    static_assert((KW - 1) % 2 == 0, "odd kernel width (the swizzle needs even row jumps)");
    static_assert(!FUSED || CIN == 32, "fused first layer: 32 channels");
    static_assert(!(FUSED && IN_SPLIT), "the fused first layer reads the f32 log-mel");
    constexpr int NTHR = WM * WN * 64;
    constexpr int BN = WN * NF * 16;
    constexpr int PH = TH + KH - 1, PW = TW + KW - 1;
    constexpr int NTAP = KH * KW, NG = CIN / X3_CG, NSTEP = NTAP * NG;
    constexpr int NW = WM * WN;
    constexpr int NB = RING ? x3_ring<KH, KW, CIN, BN, TH, TW, FUSED, RING>() : 1;
    constexpr int SLICE = BN * 64;                  // bf16 elements of one step's slice
    constexpr int SLICE_LDS = BN * 128;             // bytes (a multiple of 1 KiB)
    constexpr int GPS = SLICE_LDS / 1024;           // global_load_lds wave-instructions per slice
    constexpr int GHI = (GPS + NW - 1) / NW, GLO = GPS / NW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* patch = smem;
    char* Bs = smem + x3_patch_bytes<KH, KW, TH, TW, FUSED>();

    // DIAG 4096 (tools/conv_bench_x3.hip): per-wave phase timestamps
    // (s_memtime) and hardware ids after the output, for timeline analysis
    unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (DIAG & 4096) ts[0] = __builtin_amdgcn_s_memtime();
    const BlockPos bp = x3_block<AA_X3_REMAP != 0>();
    const int n = bp.n, cb = bp.cb;
    const int th = bp.tile / tiles_w, tw = bp.tile - (bp.tile / tiles_w) * tiles_w;
    const int oh0 = th * TH, ow0 = tw * TW;
    const int wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;

    // weight ring: slice of step s = wt[s][cout_pad][64] rows of this block
    const size_t step_stride = (size_t)gridDim.y * SLICE;
    const __amdgpu_buffer_rsrc_t wrs = x3_wrsrc(wt);  // weight slices / fragments by buffer loads
#define X3_GLDS(s)                                                                                       \
    _Pragma("unroll") for (int u_ = 0; u_ < GHI; ++u_) {                                               \
        const int g_ = u_ * NW + wave0;                                                                  \
        if (GPS % NW == 0 || g_ < GPS)                                                                  \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                   \
                wrs, (__attribute__((address_space(3))) void*)(Bs + ((s) % NB) * SLICE_LDS + g_ * 1024), 16,   \
                lane * 16, __builtin_amdgcn_readfirstlane((int)((cb * SLICE + (s) * step_stride + g_ * 512) * 2)), 0, 0); \
    }
    if constexpr (RING && !(DIAG & 32)) {
#pragma unroll
        for (int s = 0; s < NB - 1; ++s)
            if (s < NSTEP) { X3_GLDS(s) }
    }

    // per-lane fragment geometry: tile pixel p of fragment i -> patch byte
    // base (tap 0) and its swizzle phase (p + q) for this lane's unit q
    const int wave = wave0, wm = wave % WM, wn = wave / WM;
    const int q = lane >> 4;
    int abase[MF], aph[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        int p = (wm * MF + i) * 16 + (lane & 15);
        // padding rows (computed, never stored): the pixel 16 k back, whose
        // swizzle slot is the lane's own (pixel 0 would put a second address on
        // a busy slot of the lane's ds_read_b128 group)
        if (p >= TH * TW) p = max(p - 16 * ((p - TH * TW) / 16 + 1), 0);
        if (DIAG & 8) p = 0;
        const int r = p / TW, c = p - (p / TW) * TW;
        abase[i] = (r * PW + c) * 128;
        aph[i] = p + q;  // v = r*TW + c = p
    }
    // AOFF (the fused first-layer kernel, which has VGPRs to spare): the
    // lane's fragment addresses for all 8 swizzle residues precomputed, so a
    // tap's A reads are a register plus an immediate offset (no per-read
    // address arithmetic in the fully unrolled tap loop)
#ifdef AA_NO_AOFF
    constexpr bool AOFF = false;
#else
    constexpr bool AOFF = FUSED;
#endif
    int aoff[AOFF ? MF : 1][8];
    if constexpr (AOFF) {
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int r = 0; r < 8; ++r) aoff[i][r] = abase[i] + (((aph[i] + r) & 7) << 4);
    }
    int bofs[NF];  // byte offset of the lane's hi unit in a slice (lo: ^ 64)
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const int row = wn * NF * 16 + j * 16 + (lane & 15);
        bofs[j] = row * 128 + (((q + row) & 7) << 4);
    }

    const bool hi_share = (GPS % NW == 0) || wave < GPS % NW;

    f32x4 acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    struct FragSet {
        bf16x8 ah[MF], al[MF], bh[NF], bl[NF];
    };
    FragSet F0, F1;
    auto read_a = [&](FragSet& f, int t) {
        if (DIAG & 128) return;
        const int kh = t / KW, kw = t - (t / KW) * KW;
        const int toff = (kh * PW + kw) * 128, tv = kh * TW + kw;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int a = abase[i] + toff + (((aph[i] + tv) & 7) << 4);
            f.ah[i] = *reinterpret_cast<const bf16x8*>(patch + a);
            f.al[i] = *reinterpret_cast<const bf16x8*>(patch + (a ^ 64));
        }
    };
    auto read_b = [&](FragSet& f, int s) {
        if (DIAG & 128) return;
        if constexpr (!RING) {
            const int soff = __builtin_amdgcn_readfirstlane((int)((cb * SLICE + ((DIAG & 16) ? 0 : s) * step_stride) * 2));
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                f.bh[j] = x3_wload(wrs, bofs[j], soff);
                f.bl[j] = x3_wload(wrs, bofs[j] ^ 64, soff);
            }
            return;
        }
        const char* bsl = Bs + ((DIAG & 16) ? 0 : (s % NB)) * SLICE_LDS;
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            f.bh[j] = *reinterpret_cast<const bf16x8*>(bsl + bofs[j]);
            f.bl[j] = *reinterpret_cast<const bf16x8*>(bsl + (bofs[j] ^ 64));
        }
    };
    auto step = [&](FragSet& cur, FragSet& nxt, int g, int t) {
        const int s = g * NTAP + t;
        // own share of slice s+1 landed (s+2 .. s+NB-2 may stay in flight), own LDS reads done
        if constexpr (RING) {
            const int ahead = s + 1 < NSTEP ? min(NB - 3, NSTEP - 2 - s) : 0;
            if (DIAG & 32) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            } else if (hi_share) {
                wait_vm_lgkm<GHI>(ahead);
            } else {
                wait_vm_lgkm<GLO>(ahead);
            }
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!(DIAG & 32)) {
                if (s + NB - 1 < NSTEP) { X3_GLDS(s + NB - 1) }  // into the buffer B(s-1) was read from
            }
        }
        if (s + 1 < NSTEP) read_b(nxt, s + 1);
        if constexpr (!AJIT) {
            if (t + 1 < NTAP) read_a(nxt, t + 1);
            if constexpr (!RING && (AA_PIN_X3 & 1)) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int j = 0; j < NF; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.bh[j], cur.ah[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.bl[j], cur.ah[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.bh[j], cur.al[i], acc[i][j], 0, 0, 0);
                }
        } else {
            // A fragments just in time, two in flight: fragment i+1's LDS read
            // under fragment i's MFMAs (2 x 16 VGPRs instead of 2 x MF x 8)
            const int kh = t / KW, kw = t - (t / KW) * KW;
            const int toff = (kh * PW + kw) * 128, tv = kh * TW + kw;
            bf16x8 h2[2], l2[2];
            auto rd = [&](int i, int k) {
                if constexpr (AOFF) {
                    h2[k] = *reinterpret_cast<const bf16x8*>(patch + toff + aoff[i][tv & 7]);
                    l2[k] = *reinterpret_cast<const bf16x8*>(patch + toff + aoff[i][(tv + 4) & 7]);
                } else {
                    const int a = abase[i] + toff + (((aph[i] + tv) & 7) << 4);
                    h2[k] = *reinterpret_cast<const bf16x8*>(patch + a);
                    l2[k] = *reinterpret_cast<const bf16x8*>(patch + (a ^ 64));
                }
            };
            rd(0, 0);
            if constexpr (!RING && (AA_PIN_X3 & 1)) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                if (i + 1 < MF) rd(i + 1, (i + 1) & 1);
                if constexpr (!RING && (AA_PIN_X3 & 2)) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < NF; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.bh[j], h2[i & 1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.bl[j], h2[i & 1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.bh[j], l2[i & 1], acc[i][j], 0, 0, 0);
                }
            }
        }
    };

    // The fused first layer's weights and bias (f32 -> bf16 hi / lo), loaded
    // before the log-mel staging so their L2 latency overlaps the log-mel's.
    // MFMA row m (A operand lane m) computes first-layer channel
    // 16 ((m >> 2) & 1) + 4 (m >> 3) + (m & 3), so that the D register r
    // of a k-group kg lane (row 8 (r / 4) + 4 kg + r % 4) holds channel
    // 16 kg + r: each lane owns two whole 8-channel units of its pixel
    // and writes them as ds_write_b128 (eight consecutive pixels per
    // lane group: conflict-free), not as eight half units
    bf16x8 f1_wa{}, f1_wal{};
    f32x16 f1_cb{};  // D register r: channel 16 kg + r
    if constexpr (FUSED) {
        const int l32 = lane & 31, kg = lane >> 5;
        const int ch1 = 16 * ((l32 >> 2) & 1) + 4 * (l32 >> 3) + (l32 & 3);
        if constexpr (AA_F1_KPACK) {
            // the 27 products of a pixel (hi.hi, hi.lo, lo.hi over 9 taps) in the
            // 32 k-slots of two MFMAs: MFMA 1 = wh.xh (k-group 0) and wh.xl
            // (k-group 1) over taps 0-7; MFMA 2 = wl.xh over taps 0-7 (k-group
            // 0) and wh8.xh8, wh8.xl8, wl8.xh8 (k-group 1)
            float w9[9];
#pragma unroll
            for (int t = 0; t < 9; ++t) w9[t] = fc.w[ch1 * 9 + t];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                f1_wa[j] = bf_hi(w9[j]);
                f1_wal[j] = kg == 0 ? bf_lo(w9[j]) : j < 2 ? bf_hi(w9[8]) : j == 2 ? bf_lo(w9[8]) : (bf16)0.f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int tap = 8 * kg + j;
                const float wv = fc.w[ch1 * 9 + min(tap, 8)];
                f1_wa[j] = tap < 9 ? bf_hi(wv) : (bf16)0.f;
                f1_wal[j] = tap < 9 ? bf_lo(wv) : (bf16)0.f;
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) f1_cb[r] = fc.b[16 * kg + r];
    }

    if constexpr (!RING) read_b(F0, 0);  // its latency hides behind the first staging
    for (int g = 0; g < NG; ++g) {
        // ---- stage channel group g of the patch (hi / lo planes, swizzled) ----
        if (g > 0) __syncthreads();  // every wave is done with group g-1's patch
        if constexpr (DIAG & 1) {
        } else if constexpr (IN_SPLIT) {
            // group g of the patch straight from the pre-split activations:
            // LDS unit index i = pixel * 8 + slot; slot holds unit
            // (slot - R*TW - C) & 7 of pixel (R, C).  Out-of-image pixels read a
            // clamped (finite) pixel: they only feed discarded outputs.
            constexpr int UNITS = PH * PW * 8;
            // buffer loads: the resource based at the window (64-bit, so any
            // batch size), the group's base in the SGPR offset, the pixel /
            // unit in the lane's VGPR offset
            const __amdgpu_buffer_rsrc_t ars =
                x3_wrsrc(reinterpret_cast<const char*>(in) + (size_t)n * Hin * Win * CIN * 4);
            const int abase_s = g * 128;
            for (int i0 = wave0 * 64; i0 < UNITS; i0 += NW * 64) {
                const int idx = i0 + lane;
                if (idx < UNITS) {
                    const int pix = idx >> 3, slot = idx & 7;
                    const int R = pix / PW, C = pix - R * PW;
                    const int u = (slot - R * TW - C) & 7;
                    const int gh = min(oh0 + R, Hin - 1), gw = min(ow0 + C, Win - 1);
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (__attribute__((address_space(3))) void*)(patch + i0 * 16),
                                                             16, (gh * Win + gw) * (CIN * 4) + u * 16, abase_s, 0, 0);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if constexpr (!FUSED) {
            constexpr int ITEMS = (PH * PW + 7) / 8 * 64;  // (pixel, channel quad), pixels in 8s
            constexpr int U = 4;
            const float* src = in + (size_t)n * Hin * Win * CIN + g * X3_CG;
            for (int i0 = 0; i0 < ITEMS; i0 += U * NTHR) {
                float4 v[U];
                bool ok[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int idx = i0 + u * NTHR + threadIdx.x;
                    // lanes 0-7 / 8-15 of a 16-lane store group take pixels 4 apart:
                    // their swizzle slots are disjoint
                    const int blk = idx >> 6, w8 = (idx >> 3) & 7;
                    const int pix = blk * 8 + ((w8 & 1) << 2) + (w8 >> 1), cq = idx & 7;
                    const int R = pix / PW, C = pix - R * PW;
                    const int gh = oh0 + R, gw = ow0 + C;
                    ok[u] = pix < PH * PW && gh < Hin && gw < Win;
                    const int ch = min(gh, Hin - 1), cw = min(gw, Win - 1);
                    v[u] = *reinterpret_cast<const float4*>(src + ((size_t)ch * Win + cw) * CIN + cq * 4);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int idx = i0 + u * NTHR + threadIdx.x;
                    const int blk = idx >> 6, w8 = (idx >> 3) & 7;
                    const int pix = blk * 8 + ((w8 & 1) << 2) + (w8 >> 1), cq = idx & 7;
                    if (pix < PH * PW) {
                        const int R = pix / PW, C = pix - R * PW;
                        const float4 x = ok[u] ? v[u] : make_float4(0.f, 0.f, 0.f, 0.f);
                        bf16x4 h, l;
                        h[0] = bf_hi(x.x); l[0] = bf_lo(x.x);
                        h[1] = bf_hi(x.y); l[1] = bf_lo(x.y);
                        h[2] = bf_hi(x.z); l[2] = bf_lo(x.z);
                        h[3] = bf_hi(x.w); l[3] = bf_lo(x.w);
                        const int a = x3_addr(R, C, cq >> 1, PW, TW) + (cq & 1) * 8;
                        *reinterpret_cast<bf16x4*>(patch + a) = h;
                        *reinterpret_cast<bf16x4*>(patch + (a ^ 64)) = l;
                    }
                }
            }
        } else {
            // fused first layer (C_in = 1, 3x3 -> 32): log-mel patch (PH+2) x (PW+2)
            // in LDS after the activation patch, then per 32 patch pixels three
            // v_mfma_f32_32x32x16_bf16 (weights hi/lo x log-mel hi/lo, the 9 taps
            // in k, the bias as C), activation, hi/lo into the swizzled patch
            constexpr int XW = PW + 2, XN = (PH + 2) * XW;
            // X: the log-mel patch split once per element, bf16 hi in the low and
            // bf16 lo in the high half of a dword (AA_X3_XSPLIT), else f32
            float* X = reinterpret_cast<float*>(smem + (size_t)PH * PW * 128);
            uint32_t* Xs = reinterpret_cast<uint32_t*>(X);
            // buffer loads: the resource based at the window (64-bit, so any
            // batch size), the element in the lane's offset
            const int esz = fc.lm_f16 ? 2 : 4;
            const __amdgpu_buffer_rsrc_t lrs =
                x3_wrsrc(reinterpret_cast<const char*>(in) + (size_t)n * fc.H0 * fc.W0 * esz);
            constexpr int lbase = 0;
            // XU elements per thread and pass (XN = 400 for 12x21 tiles: one
            // pass of 2 over 256 threads), split in pairs
            constexpr int XU = (XN + NTHR - 1) / NTHR <= 2 ? 2 : 4;
            for (int i0 = 0; i0 < ((DIAG & 512) ? 0 : XN); i0 += XU * NTHR) {
                float v[XU];
#pragma unroll
                for (int u = 0; u < XU; ++u) {
                    const int idx = min(i0 + u * NTHR + (int)threadIdx.x, XN - 1);
                    const int r = idx / XW, c = idx - r * XW;
                    const int e = min(oh0 + r, fc.H0 - 1) * fc.W0 + min(ow0 + c, fc.W0 - 1);
                    v[u] = fc.lm_f16 ? (float)__builtin_bit_cast(_Float16, __builtin_amdgcn_raw_buffer_load_b16(lrs, e * 2, lbase, 0))
                                     : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lrs, e * 4, lbase, 0));
                    if (fc.has_mag) v[u] = powf(v[u], fc.mag_exp);
                }
#pragma unroll
                for (int u = 0; u < XU; u += 2) {
                    const int idx = i0 + u * NTHR + threadIdx.x, idx2 = idx + NTHR;
                    if constexpr (AA_X3_XSPLIT) {
                        uint32_t h, l;
                        split2(v[u], v[u + 1], h, l);
                        if (idx < XN) Xs[idx] = __builtin_amdgcn_perm(l, h, 0x05040100u);     // hi | lo << 16
                        if (idx2 < XN) Xs[idx2] = __builtin_amdgcn_perm(l, h, 0x07060302u);
                    } else {
                        if (idx < XN) X[idx] = v[u];
                        if (idx2 < XN) X[idx2] = v[u + 1];
                    }
                }
            }
            const int l32 = lane & 31, kg = lane >> 5;
            const bf16x8 wa = f1_wa, wal = f1_wal;
            const f32x16 cb = f1_cb;
            const float ae = fc.alpha;  // host: act folded to a slope in [0, 1]
            const int off0 = kg ? 2 * XW + 2 : 0;  // k-group 1 only needs tap 8 (j = 0)
            if constexpr (DIAG & 4096) ts[4] = __builtin_amdgcn_s_memtime();
            __syncthreads();
            if constexpr (DIAG & 4096) ts[5] = __builtin_amdgcn_s_memtime();
            constexpr int NPX = PH * PW;
            constexpr int NGRP = (NPX + 31) / 32;
            // NU groups of 32 pixels per wave and pass (groups g0 + NW u): all
            // of them in one pass when that takes at most 3 (12x21 tiles on 4
            // waves: 322 patch pixels, 11 groups), else passes of 2
            constexpr int NU = (NGRP + NW - 1) / NW <= 3 ? (NGRP + NW - 1) / NW : 2;
            for (int g0 = wave0; g0 < ((DIAG & 64) ? 0 : NGRP); g0 += NW * NU) {
                bf16x8 xh[NU], xl[NU];
                int pix[NU];
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    pix[u] = min((g0 + NW * u) * 32 + l32, NPX - 1);
                    const int r = pix[u] / PW, c = pix[u] - r * PW;
                    if constexpr (AA_F1_KPACK) {
                        // taps 2k, 2k+1 -> one dword of MFMA 1's operand: their
                        // hi halves in k-group 0, lo halves in k-group 1; MFMA 2
                        // takes the same (k-group 0) or tap 8's hi, lo, hi
                        const uint32_t* xp = Xs + r * XW + c;
                        uint32_t xv[9];
#pragma unroll
                        for (int j = 0; j < 9; ++j) xv[j] = xp[(j / 3) * XW + j % 3];
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
                    } else if constexpr (AA_X3_XSPLIT) {
                        // taps 2k, 2k+1 of the pre-split patch -> one dword of
                        // the hi fragment (low halves) and one of the lo (high halves)
                        const uint32_t* xp = Xs + r * XW + c;
                        uint32_t xv[8];
                        xv[0] = xp[off0];
#pragma unroll
                        for (int j = 1; j < 8; ++j) xv[j] = xp[(j / 3) * XW + j % 3];
                        uint4 hh, ll;
                        hh.x = __builtin_amdgcn_perm(xv[1], xv[0], 0x05040100u);
                        hh.y = __builtin_amdgcn_perm(xv[3], xv[2], 0x05040100u);
                        hh.z = __builtin_amdgcn_perm(xv[5], xv[4], 0x05040100u);
                        hh.w = __builtin_amdgcn_perm(xv[7], xv[6], 0x05040100u);
                        ll.x = __builtin_amdgcn_perm(xv[1], xv[0], 0x07060302u);
                        ll.y = __builtin_amdgcn_perm(xv[3], xv[2], 0x07060302u);
                        ll.z = __builtin_amdgcn_perm(xv[5], xv[4], 0x07060302u);
                        ll.w = __builtin_amdgcn_perm(xv[7], xv[6], 0x07060302u);
                        xh[u] = __builtin_bit_cast(bf16x8, hh);
                        xl[u] = __builtin_bit_cast(bf16x8, ll);
                    } else {
                        const float* xp = X + r * XW + c;
                        float xv[8];
                        xv[0] = xp[off0];
#pragma unroll
                        for (int j = 1; j < 8; ++j) xv[j] = xp[(j / 3) * XW + j % 3];
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            xh[u][j] = bf_hi(xv[j]);
                            xl[u][j] = bf_lo(xv[j]);
                        }
                    }
                }
                f32x16 d[NU];
                if constexpr (DIAG & 8192) {  // ablation: no first-layer MFMAs
#pragma unroll
                    for (int u = 0; u < NU; ++u) {
                        d[u] = cb;
                        d[u][0] += __builtin_bit_cast(float, __builtin_bit_cast(uint4, xh[u]).x ^ __builtin_bit_cast(uint4, xl[u]).y);
                    }
                } else if constexpr (AA_F1_KPACK) {
#pragma unroll
                    for (int u = 0; u < NU; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, xh[u], cb, 0, 0, 0);
#pragma unroll
                    for (int u = 0; u < NU; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wal, xl[u], d[u], 0, 0, 0);
                } else {
#pragma unroll
                for (int u = 0; u < NU; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, xh[u], cb, 0, 0, 0);
#pragma unroll
                for (int u = 0; u < NU; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, xl[u], d[u], 0, 0, 0);
#pragma unroll
                for (int u = 0; u < NU; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wal, xh[u], d[u], 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    if ((g0 + NW * u) * 32 + l32 < NPX) {
                        const int R = pix[u] / PW, C = pix[u] - R * PW;
#pragma unroll
                        for (int h = 0; h < 2; ++h) {  // channels 16 kg + 8 h + e: unit 2 kg + h
                            uint32_t hw[4], lw[4];
#pragma unroll
                            for (int e = 0; e < 8; e += 2) {
                                if constexpr (DIAG & 16384) {  // ablation: no activation / split VALU
                                    hw[e >> 1] = __builtin_bit_cast(uint32_t, d[u][8 * h + e]);
                                    lw[e >> 1] = __builtin_bit_cast(uint32_t, d[u][8 * h + e + 1]);
                                } else {
                                    leaky_split2(d[u][8 * h + e], d[u][8 * h + e + 1], ae, hw[e >> 1], lw[e >> 1]);
                                }
                            }
                            const int a = x3_addr(R, C, 2 * kg + h, PW, TW);
                            if ((DIAG & 32768) && hw[0] != 0x12345u) continue;  // ablation: no patch writes
                            *reinterpret_cast<uint4*>(patch + a) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                            *reinterpret_cast<uint4*>(patch + (a ^ 64)) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                        }
                    }
                }
            }
        }
        if constexpr (DIAG & 4096) ts[6] = __builtin_amdgcn_s_memtime();

        // ---- the group's taps: one 32-deep K chunk each, through the ring.
        // Software-pipelined by one step: the barrier at the top of step s
        // publishes slice s+1, and B(s+1) / A(s+1) are read into the other
        // fragment set while step s's MFMAs run on operands already in
        // registers -- no wave waits out an LDS read after a barrier. ----
        if (g == 0) {  // slice 0: this wave's share landed before the barrier publishing the patch
            if constexpr (RING && !(DIAG & 32)) {
                if (hi_share) wait_vm_lgkm<GHI>(min(NB - 2, NSTEP - 1));
                else wait_vm_lgkm<GLO>(min(NB - 2, NSTEP - 1));
            }
        }
        __syncthreads();
        if (g == 0) {
            if constexpr (RING) read_b(F0, 0);  // (RING = false: issued before the first staging)
        }
        else if constexpr ((NTAP - 1) % 2 == 0) {  // the previous group's last step left B in F1
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                F0.bh[j] = F1.bh[j];
                F0.bl[j] = F1.bl[j];
            }
        }
        if (!(DIAG & 2) && !AJIT) read_a(F0, 0);
        // a wave whose fragments all lie in tile rows past the conv output
        // (the bottom tile row of a tall tile) skips its MFMAs: those outputs
        // are discarded by the epilogue
        const bool wave_idle = oh0 + (wm * MF * 16) / TW >= Hout * POOL;
        if constexpr (DIAG & 4096) ts[1] = __builtin_amdgcn_s_memtime();
        // AA_X3_PRIO (A/B knob): the wave's MFMA steps at a raised issue
        // priority, so waves of co-resident blocks still staging (VALU) fill
        // the slots the matrix pipe leaves instead of delaying its issue
        if constexpr (AA_X3_PRIO > 0) __builtin_amdgcn_s_setprio(AA_X3_PRIO);
#pragma unroll
        for (int t = 0; t < ((DIAG & 2) || wave_idle ? 0 : NTAP); t += 2) {
            step(F0, F1, g, t);
            if (t + 1 < NTAP) step(F1, F0, g, t + 1);
        }
        if constexpr (AA_X3_PRIO > 0) __builtin_amdgcn_s_setprio(0);
        if constexpr (DIAG & 4096) ts[2] = __builtin_amdgcn_s_memtime();
    }
#undef X3_GLDS
    __syncthreads();  // patch and ring no longer needed: the f32 tile reuses LDS

    // ---- epilogue: f32 tile (x3_store's swizzled layout), pool, bias, activation, store ----
    float* E = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const int u = wn * NF * 4 + j * 4 + q;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int p = (wm * MF + i) * 16 + (lane & 15);
            if (p < TH * TW)
                *reinterpret_cast<float4*>(E + x3_eoff<BN, 0>(p, u)) =
                    make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        }
    }
    __syncthreads();
    x3_store<TH, TW, POOL, BN, NTHR, OUT_SPLIT, (DIAG & 4) != 0, 0>(E, bias, out, n, cb, oh0, ow0, Hout, Wout,
                                                                  cout_store, act, alpha);
    if constexpr (DIAG & 4096) {
        ts[3] = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
            const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
            unsigned long long* d = reinterpret_cast<unsigned long long*>(out + (64u << 20)) + ((size_t)L * NW + wave0) * 10;
            for (int k = 0; k < 8; ++k) d[k] = ts[k];
            d[8] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
            d[9] = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
        }
    }
}

}  // namespace aa
