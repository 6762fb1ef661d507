// Window-classifier CNN for gfx950: MFMA implicit-GEMM convolutions.
//
// Replaces model.predict(np.array(d)) (reference src/identify_tracks.py:544,
// Keras on TF-CPU) for the layer family the build defines:
//   [MagTransform] conv-BN-act [maxpool] ... conv1x1 globalmax sigmoid
// Planner (aa_model_create) folds each BatchNormalization into the preceding
// conv, fuses the activation and a following 3x3/3 max-pool into the conv's
// epilogue, and the final 1x1 conv + GlobalMaxPool2D + sigmoid into one head
// kernel.  Stages:
//   conv_small  first layer (C_in = 1): VALU, f32 math, MagTransform prologue
//               (src/magtransformv2.py:19-21), writes NHWC activations.
//   conv_mfma   C_in % 32 == 0: implicit GEMM, M = output pixels of a
//               TH x TW tile, N = output channels, K = kh*kw*C_in.  The input
//               patch (TH+kh-1) x (TW+kw-1) x C_in is staged once in LDS
//               (16-B vector loads, +16 B channel pad per pixel); A fragments
//               come from LDS, B fragments (weights, [C_out][K], L2-resident)
//               from global.  bf16: v_mfma_f32_16x16x32_bf16; f32 parity mode:
//               v_mfma_f32_16x16x4_f32 (exact f32 fma chain), same fragment
//               layout with K permuted inside each 32-chunk.  Epilogue stages
//               the f32 tile in LDS, applies max-pool, bias (folded BN) and the
//               activation, and stores NHWC.
//   conv_head   1x1 conv + global max over all pixels + sigmoid, one block per
//               window, A fragments straight from global.
#include "aa_common.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

namespace aa {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __bf16 bf16;
// OCP e4m3fn byte (gfx950's fp8; not the MI300 fnuz encoding)
struct fp8 {
    uint8_t v;
};
// Split-bf16 precision tag (AA_PREC_BF16X3): activations stay f32 in HBM; at
// LDS staging every value x becomes bf16 hi = rn(x) and lo = rn(x - hi)
// (x - hi is exact in f32), weights likewise on the host, and each product
// is hi*hi + hi*lo + lo*hi on three bf16 MFMAs with f32 accumulation.  The
// representation error is <= 2^-18 |x| per operand and the dropped lo*lo
// term <= 2^-18 |x w|, so a MAC carries ~17 significant bits instead of
// bf16's 8 -- enough for the 1e-3 logit gate at 3/16 of the f32-MFMA cost.
struct bf16x3 {};

// Storage types of a precision: L = LDS / fragment element, G = HBM
// activation element.
template <typename T>
struct Prec {
    using L = T;
    using G = T;
};
template <>
struct Prec<bf16x3> {
    using L = bf16;
    using G = float;
};
template <typename T>
constexpr bool is_split() { return std::is_same<T, bf16x3>::value; }
template <typename T>
constexpr bool is_fp8() { return std::is_same<T, fp8>::value; }

// bf16 hi + lo of an f32 (round to nearest even both times)
__device__ __forceinline__ bf16 bf_hi(float x) { return (bf16)x; }
__device__ __forceinline__ bf16 bf_lo(float x) { return (bf16)(x - (float)(bf16)x); }

// 4 / 8 floats -> e4m3fn bytes, round to nearest even, saturated to +-448
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
    const float M = 448.f;
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a, -M), M), fminf(fmaxf(b, -M), M), 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c, -M), M), fminf(fmaxf(d, -M), M), w, true);
    return (uint32_t)w;
}

// ---- 8-element fragments and the MFMA step over one 32-deep K chunk -------
template <typename T>
struct Frag;
template <>
struct Frag<bf16> {
    bf16x8 v;
    __device__ __forceinline__ void load(const bf16* p) { v = *reinterpret_cast<const bf16x8*>(p); }
};
template <>
struct Frag<fp8> {
    long v;
    __device__ __forceinline__ void load(const fp8* p) { v = *reinterpret_cast<const long*>(p); }
};
template <>
struct Frag<float> {
    float v[8];
    __device__ __forceinline__ void load(const float* p) {
        const float4 a = reinterpret_cast<const float4*>(p)[0];
        const float4 b = reinterpret_cast<const float4*>(p)[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
};

// Lane l holds A[row l&15][k0 + 8(l>>4) + j] and B[k0 + 8(l>>4) + j][col l&15].
__device__ __forceinline__ f32x4 mfma_chunk(const Frag<bf16>& a, const Frag<bf16>& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}
// fp8: the same lane layout with 8 bytes per lane (non-scaled form: the bf16 rate,
// half the staging and fragment bytes)
__device__ __forceinline__ f32x4 mfma_chunk(const Frag<fp8>& a, const Frag<fp8>& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a.v, b.v, c, 0, 0, 0);
}
// f32: sub-step s feeds k = 8(l>>4) + s into the instruction's k slot (l>>4),
// identically for A and B, so the 8 instructions cover the 32-chunk exactly.
__device__ __forceinline__ f32x4 mfma_chunk(const Frag<float>& a, const Frag<float>& b, f32x4 c) {
#pragma unroll
    for (int s = 0; s < 8; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[s], b.v[s], c, 0, 0, 0);
    return c;
}

template <typename T>
__device__ __forceinline__ T to_t(float x);
template <>
__device__ __forceinline__ float to_t<float>(float x) { return x; }
template <>
__device__ __forceinline__ bf16 to_t<bf16>(float x) { return (bf16)x; }
template <>
__device__ __forceinline__ fp8 to_t<fp8>(float x) { return fp8{(uint8_t)(pack4_fp8(x, 0.f, 0.f, 0.f) & 0xff)}; }

enum { ACT_NONE = 0, ACT_LEAKY = 1, ACT_RELU = 2 };
__device__ __forceinline__ float apply_act(float v, int act, float alpha) {
    if (act == ACT_LEAKY) return v >= 0.f ? v : v * alpha;
    if (act == ACT_RELU) return fmaxf(v, 0.f);
    return v;
}

// ---------------------------------------------------------------------------
// conv_small: C_in == 1, VALU.  One thread per output pixel, all COUT channels.
// ---------------------------------------------------------------------------
template <typename TO, int KH, int KW, int COUT>
__global__ __launch_bounds__(256) void conv_small(const float* __restrict__ in, int Hin, int Win,
                                                  const float* __restrict__ wt /*[COUT][KH*KW]*/,
                                                  const float* __restrict__ bias, int has_mag,
                                                  float mag_exp, TO* __restrict__ out, int Hc, int Wc,
                                                  int act, float alpha) {
    __shared__ float sw[COUT * KH * KW];
    __shared__ float sb[COUT];
    for (int i = threadIdx.x; i < COUT * KH * KW; i += blockDim.x) sw[i] = wt[i];
    for (int i = threadIdx.x; i < COUT; i += blockDim.x) sb[i] = bias[i];
    __syncthreads();
    const int n = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= Hc * Wc) return;
    const int h = p / Wc, w = p - (p / Wc) * Wc;
    float x[KH * KW];
    const float* src = in + (size_t)n * Hin * Win;
#pragma unroll
    for (int i = 0; i < KH; ++i)
#pragma unroll
        for (int j = 0; j < KW; ++j) {
            float v = src[(h + i) * Win + w + j];
            if (has_mag) v = powf(v, mag_exp);
            x[i * KW + j] = v;
        }
    TO* o = out + ((size_t)n * Hc * Wc + p) * COUT;
#pragma unroll
    for (int c0 = 0; c0 < COUT; c0 += 8) {
        float r[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float s = 0.f;
#pragma unroll
            for (int t = 0; t < KH * KW; ++t) s = fmaf(x[t], sw[(c0 + c) * KH * KW + t], s);
            r[c] = apply_act(s + sb[c0 + c], act, alpha);
        }
        if constexpr (sizeof(TO) == 1) {
            *reinterpret_cast<uint2*>(o + c0) =
                make_uint2(pack4_fp8(r[0], r[1], r[2], r[3]), pack4_fp8(r[4], r[5], r[6], r[7]));
        } else if constexpr (sizeof(TO) == 2) {
            bf16x8 v;
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = (bf16)r[c];
            *reinterpret_cast<bf16x8*>(o + c0) = v;
        } else {
            reinterpret_cast<float4*>(o + c0)[0] = make_float4(r[0], r[1], r[2], r[3]);
            reinterpret_cast<float4*>(o + c0)[1] = make_float4(r[4], r[5], r[6], r[7]);
        }
    }
}

// ---------------------------------------------------------------------------
// conv_mfma: implicit-GEMM conv, C_in % 32 == 0, fused pool/bias/act.
// Block = 4 waves = WM (pixel) x WN (channel); wave = MF x NF 16x16 tiles.
// ---------------------------------------------------------------------------
// Padded row length (elements) of the staged patch and of the weight slices:
// bf16 rows padded by 32 B (stride = 2 mod 4 16-B units, which makes every
// ds_read_b128 lane group of the fragment reads conflict-free); fp8 rows
// padded by 16 B (48 / 80 / 144-B strides put the 16 rows of a ds_read_b64
// half-wave on distinct 4-bank groups); f32 (parity mode) keeps a 16-B pad.
template <typename T>
__host__ __device__ constexpr int conv_cstr(int cin) {
    return cin + (sizeof(T) == 1 ? 16 : sizeof(T) == 2 ? 16 : 4);
}

// LDS of one conv_mfma block: [staged patch][f32 log-mel patch if FUSED]
// [2 x weight slice], and afterwards the epilogue tile reusing it from 0.
template <typename T, int KH, int KW, int CIN, int TH, int TW, bool FUSED>
__host__ __device__ constexpr size_t conv_b_offset() {
    constexpr int CSTR = conv_cstr<T>(CIN);
    size_t off = ((size_t)(TH + KH - 1) * (TW + KW - 1) * CSTR * sizeof(typename Prec<T>::L) + 15) & ~(size_t)15;
    if (FUSED) off += ((sizeof(float) * (TH + KH + 1) * (TW + KW + 1)) + 15) & ~(size_t)15;
    return off;
}

// fp8 runs the block-scaled K = 128 MFMA (v_mfma_f32_16x16x128_f8f6f4, the
// scale operands literal 0 = unscaled, 2x the non-scaled fp8 rate): its K
// loop walks "super-steps" of four 32-deep chunks (chunk k = tap * C_in/32 +
// channel chunk), and its weights are packed per super-step as rows of
// 4 x 32 B (+16 B pad) instead of per tap.
// C_in = 32 layers keep the non-scaled K = 32 form: 9 taps are 9 chunks, and
// packed into K = 128 they would waste a quarter of the MFMA work (measured
// in the pipeline: fused first conv 64 -> 75 us, 3x3/32 19 -> 22 us).
constexpr int F8_BSTR = 144;  // bytes of one packed fp8 weight row (128 + pad)
template <typename T>
__host__ __device__ constexpr bool conv_k128(int cin) {
    return is_fp8<T>() && cin >= 64;
}
template <typename T>
__host__ __device__ constexpr int conv_bstr(int cin) {  // weight-row stride (elements) of one step's slice
    return conv_k128<T>(cin) ? F8_BSTR : conv_cstr<T>(cin);
}
template <typename T>
__host__ __device__ constexpr int conv_nstep(int ntap, int cin) {  // K-loop steps (= weight slices)
    return conv_k128<T>(cin) ? (ntap * (cin / 32) + 3) / 4 : ntap;
}

// One step's weight slice [BN][BSTR] in LDS, rounded up to whole 1-KiB
// wave-instructions of global_load_lds (the tail lanes land in the rounding).
template <typename T, int CIN, int BN>
__host__ __device__ constexpr int conv_slice_lds_bytes() {
    return (BN * conv_bstr<T>(CIN) * (int)sizeof(typename Prec<T>::L) + 1023) / 1024 * 1024;
}

template <typename T, int KH, int KW, int CIN, int BN, int TH, int TW, bool FUSED, bool EBF16>
constexpr size_t conv_lds_bytes_nb(int nb) {
    const size_t main = conv_b_offset<T, KH, KW, CIN, TH, TW, FUSED>() + (size_t)nb * conv_slice_lds_bytes<T, CIN, BN>();
    const size_t epi = (size_t)TH * TW * (BN + (EBF16 ? 8 : 4)) * (EBF16 ? 2 : 4);
    return main > epi ? main : epi;
}

// Depth of the LDS ring of weight slices: as many buffers (up to 8, at most
// one per tap) as fit without lowering the blocks per CU that a 2-deep ring
// allows.  Slices in flight = ring - 1.
template <typename T, int KH, int KW, int CIN, int BN, int TH, int TW, bool FUSED, bool EBF16>
constexpr int conv_ring() {
    constexpr size_t cap = 160 * 1024;
    // fp8: the loop reads slice s+1 while s+NB-1 is issued (one-step software pipeline): >= 3
    constexpr int NB0 = conv_k128<T>(CIN) ? 3 : 2;
    const size_t base = conv_lds_bytes_nb<T, KH, KW, CIN, BN, TH, TW, FUSED, EBF16>(NB0);
    const size_t blocks = cap / base;
    int nb = NB0;
    while (nb < 8 && nb < conv_nstep<T>(KH * KW, CIN) &&
           blocks * conv_lds_bytes_nb<T, KH, KW, CIN, BN, TH, TW, FUSED, EBF16>(nb + 1) <= cap)
        ++nb;
    return nb;
}

template <typename T, int KH, int KW, int CIN, int BN, int TH, int TW, bool FUSED, bool EBF16>
constexpr size_t conv_lds_bytes() {
    return conv_lds_bytes_nb<T, KH, KW, CIN, BN, TH, TW, FUSED, EBF16>(
        conv_ring<T, KH, KW, CIN, BN, TH, TW, FUSED, EBF16>());
}

// s_waitcnt vmcnt(N) with N = PER * k for a runtime k in [0, 7] (the
// immediate must be a literal), lgkmcnt(0) alongside.
template <int PER>
__device__ __forceinline__ void wait_vm_lgkm(int k) {
#define AA_W(K) case K: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER * K) : "memory"); break;
    switch (k) { AA_W(0) AA_W(1) AA_W(2) AA_W(3) AA_W(4) AA_W(5) AA_W(6) default: AA_W(7) }
#undef AA_W
}

// s_waitcnt vmcnt(N) alone (LDS reads stay in flight), N = PER * k
template <int PER>
__device__ __forceinline__ void wait_vm(int k) {
#define AA_W(K) case K: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER * K) : "memory"); break;
    switch (k) { AA_W(0) AA_W(1) AA_W(2) AA_W(3) AA_W(4) AA_W(5) AA_W(6) default: AA_W(7) }
#undef AA_W
}

// First layer fused into the next conv's patch staging (FUSED = true): the
// log-mel patch is staged in LDS and the C_in = 1, 3x3 conv (f32 VALU, folded
// BN, activation, optional MagTransform prologue) writes the activations the
// MFMA loop consumes straight into the LDS patch -- the first layer's output
// never reaches HBM.
struct FirstConv {
    const float* w;  // [32][9] folded
    const float* b;  // [32]
    int act;
    float alpha;
    int has_mag;
    float mag_exp;
    int H0, W0;      // log-mel image
    int lm_f16;      // log-mel stored as float16 (aa_model_set_input_f16)
};

// one log-mel value of the fused first conv's input (f32, or f16 when lm_f16)
__device__ __forceinline__ float load_lm(const void* in, size_t i, int lm_f16) {
    return lm_f16 ? (float)reinterpret_cast<const _Float16*>(in)[i] : reinterpret_cast<const float*>(in)[i];
}

// DIAG (diagnostic builds only, tools/conv_bench.hip): bit 0 skips the patch
// staging, bit 1 the MFMA loop, bit 2 the epilogue stores, bit 3 makes every
// lane read pixel 0 (no LDS bank conflicts), bit 4 re-reads chunk 0's weights
// (L1-resident, no L2 stream), bit 5 skips the weight loads in the loop, bit 7
// skips the fragment reads after the first (MFMA issue alone), bit 6 the
// fused first conv's compute, bit 9 its log-mel patch load.
// Waves per SIMD a conv_mfma block shape reaches (LDS-limited), told to the
// compiler so it schedules for latency at that occupancy instead of trimming
// registers for an occupancy the LDS footprint never allows.
template <typename T, int KH, int KW, int CIN, int WM, int WN, int NF, int TH, int TW, bool FUSED, bool EBF16>
constexpr int conv_waves_per_simd() {
    constexpr size_t lds = conv_lds_bytes<T, KH, KW, CIN, WN * NF * 16, TH, TW, FUSED, EBF16>();
    constexpr int blocks = (int)((160 * 1024) / lds);
    constexpr int w = blocks * WM * WN / 4;
    return w < 1 ? 1 : (w > 8 ? 8 : w);
}

template <typename T, int KH, int KW, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW,
          bool FUSED = false, int DIAG = 0, bool EBF16 = false, int OCC = 0>
__global__ __launch_bounds__(WM * WN * 64)
__attribute__((amdgpu_waves_per_eu(OCC ? OCC : conv_waves_per_simd<T, KH, KW, CIN, WM, WN, NF, TH, TW, FUSED, EBF16>(),
                                    OCC ? OCC : conv_waves_per_simd<T, KH, KW, CIN, WM, WN, NF, TH, TW, FUSED, EBF16>())))
void conv_mfma(const typename Prec<T>::G* __restrict__ in, int Hin, int Win,
                                                 const typename Prec<T>::L* __restrict__ wt, const float* __restrict__ bias,
                                                 typename Prec<T>::G* __restrict__ out, int Hout, int Wout, int cout_store,
                                                 int tiles_w, int act, float alpha, FirstConv fc) {
    using LT = typename Prec<T>::L;  // LDS / fragment element
    using GT = typename Prec<T>::G;  // HBM activation element
    constexpr bool F8 = is_fp8<T>();
    static_assert(!is_split<T>(), "split-bf16 runs conv_x3 (aa_conv_x3.h)");
    static_assert(TH % POOL == 0 && TW % POOL == 0, "pool-aligned tile");
    static_assert(TH * TW <= WM * MF * 16, "tile covered by the waves' fragments");
    constexpr int NTHR = WM * WN * 64;
    static_assert(CIN % 32 == 0, "C_in multiple of 32");
    constexpr int BN = WN * NF * 16;
    constexpr int VEC = 16 / sizeof(LT);
    constexpr int CSTR = conv_cstr<T>(CIN);  // padded pixel / weight-row stride
    // epilogue tile: f32, or bf16 with the bias already added (rounding is
    // monotone, so max-pooling the rounded values equals rounding the max)
    using ET = typename std::conditional<EBF16, bf16, float>::type;
    constexpr int ESTR = BN + (EBF16 ? 8 : 4);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LT* patch = reinterpret_cast<LT*>(smem);

    const int n = blockIdx.z;
    const int th = blockIdx.x / tiles_w, tw = blockIdx.x - (blockIdx.x / tiles_w) * tiles_w;
    const int oh0 = th * TH, ow0 = tw * TW;
    constexpr int PH = TH + KH - 1, PW = TW + KW - 1;

    // The first NB - 1 weight slices of the K loop's LDS ring (described
    // there) are issued before the patch is staged, so their L2 round trip
    // overlaps the staging instead of following it.
    const int wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int NTAP = KH * KW;
    constexpr int CPC = CIN / 32;
    constexpr int NW = WM * WN;
    constexpr int NB = conv_ring<T, KH, KW, CIN, BN, TH, TW, FUSED, EBF16>();
    constexpr int NSTEP = conv_nstep<T>(NTAP, CIN);                // K-loop steps / weight slices
    constexpr int SLICE = BN * conv_bstr<T>(CIN);                  // elements
    constexpr int SLICE_LDS = conv_slice_lds_bytes<T, CIN, BN>();  // bytes
    constexpr int GPS = SLICE_LDS / 1024;                          // wave-instructions per slice
    constexpr int GHI = (GPS + NW - 1) / NW, GLO = GPS / NW;       // this wave's share: GHI if wave < GPS % NW
    char* Bs = smem + conv_b_offset<T, KH, KW, CIN, TH, TW, FUSED>();
    const size_t tap_stride = (size_t)gridDim.y * SLICE;
    const LT* wsl = wt + (size_t)blockIdx.y * SLICE + (threadIdx.x & 63) * VEC;
#define AA_GLDS(t)                                                                                       \
    _Pragma("unroll") for (int u_ = 0; u_ < GHI; ++u_) {                                               \
        const int g_ = u_ * NW + wave0;                                                                  \
        if (GPS % NW == 0 || g_ < GPS)                                                                  \
            __builtin_amdgcn_global_load_lds(                                                           \
                (const __attribute__((address_space(1))) void*)(wsl + (size_t)(t) * tap_stride + g_ * (1024 / sizeof(LT))), \
                (__attribute__((address_space(3))) void*)(Bs + ((t) % NB) * SLICE_LDS + g_ * 1024), 16, 0, 0); \
    }
    if constexpr (!(DIAG & 32)) {
#pragma unroll
        for (int t = 0; t < NB - 1; ++t)
            if (t < NSTEP) { AA_GLDS(t) }
    }

    // ---- stage the input patch ----
    if constexpr (DIAG & 1) {
    } else if constexpr (!FUSED) {
        // batched, unconditional 16-B loads from clamped addresses (a
        // load-or-zero branch would serialise them); out-of-image pixels only
        // feed discarded outputs but are zeroed anyway
        constexpr int VPP = CIN / VEC;  // 16-B vectors per pixel
        constexpr int U = 4;
        const int total = PH * PW * VPP;
        const GT* src = in + (size_t)n * Hin * Win * CIN;
        for (int i0 = 0; i0 < total; i0 += U * NTHR) {
            uint4 v[U];
            bool ok[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int idx = i0 + u * NTHR + threadIdx.x;
                const int pix = idx / VPP, cv = idx - pix * VPP;
                const int r = pix / PW, c = pix - r * PW;
                const int gh = oh0 + r, gw = ow0 + c;
                ok[u] = idx < total && gh < Hin && gw < Win;
                const int ch = min(gh, Hin - 1), cw = min(gw, Win - 1);
                v[u] = *reinterpret_cast<const uint4*>(src + ((size_t)ch * Win + cw) * CIN + cv * VEC);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int idx = i0 + u * NTHR + threadIdx.x;
                if (idx < total) {
                    const int pix = idx / VPP, cv = idx - pix * VPP;
                    *reinterpret_cast<uint4*>(patch + pix * CSTR + cv * VEC) = ok[u] ? v[u] : make_uint4(0, 0, 0, 0);
                }
            }
        }
    } else {
        static_assert(CIN == 32, "fused first layer produces 32 channels");
        // (a) log-mel patch (PH+2) x (PW+2), f32, after the activation patch
        constexpr int XW = PW + 2, XN = (PH + 2) * XW;
        const size_t pbytes = ((size_t)PH * PW * CSTR * sizeof(LT) + 15) & ~(size_t)15;
        float* X = reinterpret_cast<float*>(smem + pbytes);
        const size_t lmo = (size_t)n * fc.H0 * fc.W0;
        for (int i0 = 0; i0 < ((DIAG & 512) ? 0 : XN); i0 += 4 * NTHR) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int idx = min(i0 + u * NTHR + (int)threadIdx.x, XN - 1);
                const int r = idx / XW, c = idx - r * XW;
                v[u] = load_lm(in, lmo + (size_t)min(oh0 + r, fc.H0 - 1) * fc.W0 + min(ow0 + c, fc.W0 - 1), fc.lm_f16);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int idx = i0 + u * NTHR + threadIdx.x;
                if (idx < XN) X[idx] = fc.has_mag ? powf(v[u], fc.mag_exp) : v[u];
            }
        }
        if constexpr (sizeof(LT) <= 2) {
            // (b) first conv on the matrix cores: per 32 patch pixels one
            // v_mfma_f32_32x32x16_bf16, D[32 ch][32 px] = W[32 ch][16 k] X[16 k][32 px]
            // with the 9 taps in k (0..8; weights 0 for k = 9..15, so those
            // B entries may hold any finite value), the bias as the C input,
            // then the activation, bf16, and 8-byte stores of 4 channels into
            // the patch.  Lane l: pixel l % 32, k-group / channel quad l / 32.
            const int wave1 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            const int l32 = threadIdx.x & 31, kg = (threadIdx.x >> 5) & 1;
            bf16x8 wa;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int tap = 8 * kg + j;
                wa[j] = tap < 9 ? (bf16)fc.w[l32 * 9 + tap] : (bf16)0.f;
            }
            f32x16 cb;  // D row (channel) of register r: 8 (r / 4) + 4 kg + r % 4
#pragma unroll
            for (int r = 0; r < 16; ++r) cb[r] = fc.b[8 * (r >> 2) + 4 * kg + (r & 3)];
            const float ae = fc.alpha;  // host: act folded to a slope in [0, 1]
            // tap offsets into X: k = 8 kg + j; k-group 1 only needs tap 8 (j = 0)
            const int off0 = kg ? 2 * XW + 2 : 0;
            __syncthreads();
            constexpr int NPX = PH * PW;
            // bf16: two pixel groups per iteration, so independent MFMA chains
            // (and their LDS reads) interleave instead of waiting out each
            // chain's latency (in-pipeline A/B: +0.7 % bench; fp8 -0.7 %, so one)
            constexpr int NG = (NPX + 31) / 32;
            constexpr int UG = std::is_same<T, bf16>::value ? 2 : 1;
            for (int g0 = wave1; g0 < ((DIAG & 64) ? 0 : NG); g0 += 4 * UG) {
                bf16x8 xh[UG], xl[UG];
                int pix[UG];
#pragma unroll
                for (int u = 0; u < UG; ++u) {
                    pix[u] = min((g0 + 4 * u) * 32 + l32, NPX - 1);
                    const int r = pix[u] / PW, c = pix[u] - r * PW;
                    const float* xp = X + r * XW + c;
                    float xv[8];
                    xv[0] = xp[off0];
#pragma unroll
                    for (int j = 1; j < 8; ++j) xv[j] = xp[(j / 3) * XW + j % 3];
                    // the log-mel as bf16 hi + lo (x - hi, exact in f32): two MFMAs
                    // keep ~16 significant bits of the input
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        xh[u][j] = (bf16)xv[j];
                        xl[u][j] = (bf16)(xv[j] - (float)xh[u][j]);
                    }
                }
                f32x16 d[UG];
#pragma unroll
                for (int u = 0; u < UG; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, xh[u], cb, 0, 0, 0);
#pragma unroll
                for (int u = 0; u < UG; ++u) d[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, xl[u], d[u], 0, 0, 0);
#pragma unroll
                for (int u = 0; u < UG; ++u) {
                    if ((g0 + 4 * u) * 32 + l32 < NPX) {
                        LT* dst = patch + pix[u] * CSTR + 4 * kg;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if constexpr (F8) {
                                float o[4];
#pragma unroll
                                for (int e = 0; e < 4; ++e) o[e] = fmaxf(d[u][4 * q + e], d[u][4 * q + e] * ae);
                                *reinterpret_cast<uint32_t*>(dst + 8 * q) = pack4_fp8(o[0], o[1], o[2], o[3]);
                            } else {
                                typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
                                bf16x4 o;
#pragma unroll
                                for (int e = 0; e < 4; ++e) o[e] = (bf16)fmaxf(d[u][4 * q + e], d[u][4 * q + e] * ae);
                                *reinterpret_cast<bf16x4*>(dst + 8 * q) = o;
                            }
                        }
                    }
                }
            }
        } else {
            // (b) first conv: wave -> 8 output channels (wave-uniform, so its 72
            // weights and 8 biases are scalar loads), lane -> one patch column; the
            // lane slides the 3x3 window down its column (3 new LDS reads per
            // output row) and computes channel pairs with packed FMAs, each f32
            // chain started at the bias (only the bf16 path fuses; the f32 parity
            // mode runs conv_small).  Activation as max(v, a v): the planner
            // fuses only when the activation has 0 <= a <= 1 (none: 1, relu: 0).
            static_assert(NTHR == 256 && PW <= 64, "fused first layer: 4 waves, patch width <= 64");
            const int cg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            const int col = threadIdx.x & 63;
            f32x2 w1[9][4];
            f32x2 b1[4];
    #pragma unroll
            for (int k = 0; k < 4; ++k) {
                b1[k] = f32x2{fc.b[cg * 8 + 2 * k], fc.b[cg * 8 + 2 * k + 1]};
    #pragma unroll
                for (int t = 0; t < 9; ++t)
                    w1[t][k] = f32x2{fc.w[(cg * 8 + 2 * k) * 9 + t], fc.w[(cg * 8 + 2 * k + 1) * 9 + t]};
            }
            const float ae = fc.alpha;  // host: act folded to a slope in [0, 1]
            __syncthreads();
            if (col < PW) {
                float xr[3][3];
    #pragma unroll
                for (int i = 0; i < 2; ++i)
    #pragma unroll
                    for (int j = 0; j < 3; ++j) xr[i][j] = X[i * XW + col + j];
    #pragma unroll
                for (int r = 0; r < PH; ++r) {
    #pragma unroll
                    for (int j = 0; j < 3; ++j) xr[(r + 2) % 3][j] = X[(r + 2) * XW + col + j];
                    f32x2 acc[4];  // the bias starts the chain (bf16 path only: f32 parity runs conv_small)
    #pragma unroll
                    for (int k = 0; k < 4; ++k) acc[k] = b1[k];
    #pragma unroll
                    for (int i = 0; i < 3; ++i)
    #pragma unroll
                        for (int j = 0; j < 3; ++j) {
                            const float xv = xr[(r + i) % 3][j];
    #pragma unroll
                            for (int k = 0; k < 4; ++k)
                                acc[k] = __builtin_elementwise_fma(f32x2{xv, xv}, w1[i * 3 + j][k], acc[k]);
                        }
                    float o[8];
    #pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const f32x2 v = acc[k];
                        const f32x2 sv = v * ae;
                        o[2 * k] = fmaxf(v.x, sv.x);
                        o[2 * k + 1] = fmaxf(v.y, sv.y);
                    }
                    LT* dst = patch + (r * PW + col) * CSTR + cg * 8;
                    if constexpr (sizeof(LT) == 2) {
                        bf16x8 v;
    #pragma unroll
                        for (int ch = 0; ch < 8; ++ch) v[ch] = (bf16)o[ch];
                        *reinterpret_cast<bf16x8*>(dst) = v;
                    } else {
                        reinterpret_cast<float4*>(dst)[0] = make_float4(o[0], o[1], o[2], o[3]);
                        reinterpret_cast<float4*>(dst)[1] = make_float4(o[4], o[5], o[6], o[7]);
                    }
                }
            }
        }
        }
    __syncthreads();

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int wm = wave % WM, wn = wave / WM;
    const int q8 = 8 * (lane >> 4);
    constexpr int TP = TH * TW;
    int abase[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        int p = (wm * MF + i) * 16 + (lane & 15);
        if (p >= TP || (DIAG & 8)) p = 0;  // padding rows: computed, never stored
        const int r = p / TW, c = p - (p / TW) * TW;
        abase[i] = (r * PW + c) * CSTR + q8;
    }
    f32x4 acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- K loop, one tap (kh, kw) at a time.  Weights are packed tap-major
    // with padded rows, [tap][cout_pad][CSTR], so a block's slice of one tap
    // is one contiguous [BN][CSTR] block whose bytes are exactly its LDS
    // image.  global_load_lds streams the slices through a ring of NB LDS
    // buffers, NB - 1 taps ahead of the one computing (an L2 round trip of
    // a slice outlasts one tap's MFMAs): at the top of tap t each wave waits
    // for its own loads of slice t with a counted vmcnt (later slices stay in
    // flight), one barrier publishes slice t to every wave and retires all
    // reads of the buffer slice t + NB - 1 will overwrite, then that slice is
    // issued.  A fragments come from the staged patch. ----
    const int brow = (wn * NF * 16 + (lane & 15)) * CSTR + q8;
    const bool hi_share = (GPS % NW == 0) || wave < GPS % NW;
    // Fragments are double-buffered in registers: while chunk q's MFMAs run,
    // chunk q+1's fragments are in flight.  Across a tap boundary only the A
    // fragments (from the static patch) can run ahead; the next slice's B
    // fragments follow the barrier that publishes it.
    Frag<LT> fa[MF], fb[NF], na[MF], nb[NF];
#define AA_LOAD_A(dst, tap, cc_)                                                             \
    if (!(DIAG & 128) || (tap) == 0)                                                         \
    {                                                                                        \
        const int kh_ = (tap) / KW, kw_ = (tap) - ((tap) / KW) * KW;                         \
        const int at_ = (kh_ * PW + kw_) * CSTR + (cc_) * 32;                                \
        _Pragma("unroll") for (int i = 0; i < MF; ++i) dst[i].load(patch + abase[i] + at_); \
    }
#define AA_LOAD_B(dst, buf, cc_)                                                             \
    if (!(DIAG & 128) || (buf) < 0)                                                          \
    {                                                                                        \
        const LT* bt_ = reinterpret_cast<const LT*>(Bs + (buf) * SLICE_LDS) + brow + (cc_) * 32; \
        _Pragma("unroll") for (int j = 0; j < NF; ++j) dst[j].load(bt_ + j * 16 * CSTR);   \
    }
    // f32 (parity mode) fragments are twice as wide: single-buffered there
    constexpr bool DB = !std::is_same<T, float>::value;
    if constexpr (conv_k128<T>(CIN)) {
        // ---- fp8, C_in >= 64: K = 128 per MFMA.  Super-step s covers chunks 4s .. 4s+3
        // (chunk k: tap k / CPC, channel chunk k % CPC); lane group q's 32
        // fragment bytes are its 8 bytes (channels 8q .. 8q+7) of each of the
        // four chunks, read as four ds_read_b64 from the patch (A, pixels)
        // and from the super-step's weight slice (B, rows of 4 x 32 B), in the
        // same order for both operands -- the instruction's k order is the
        // same permutation for A and B (tools/mfma_scale_probe.hip), so the
        // product is the sum over the four chunks.  Chunks past the last tap
        // have zero weights (their A reads re-read chunk 0: finite values).
        // Software-pipelined by one step: the barrier at the top of step s
        // publishes slice s+1, whose B fragments are read while step s's
        // MFMAs run; A fragments are read just in time, two in flight. ----
        typedef __attribute__((ext_vector_type(8))) int i32x8;
        typedef __attribute__((ext_vector_type(2))) int i32x2;
        constexpr int NCH = NTAP * CPC;
        const int browf = (wn * NF * 16 + (lane & 15)) * F8_BSTR + q8;
        auto choff = [&](int k) {
            k = k < NCH ? k : 0;
            const int t = k / CPC, cc = k - (k / CPC) * CPC;
            const int kh = t / KW, kw = t - (t / KW) * KW;
            return (kh * PW + kw) * CSTR + cc * 32;
        };
        auto rd4 = [](i32x8& v, const char* p0, const char* p1, const char* p2, const char* p3) {
            const i32x2 x0 = *reinterpret_cast<const i32x2*>(p0), x1 = *reinterpret_cast<const i32x2*>(p1);
            const i32x2 x2 = *reinterpret_cast<const i32x2*>(p2), x3 = *reinterpret_cast<const i32x2*>(p3);
            v = i32x8{x0[0], x0[1], x1[0], x1[1], x2[0], x2[1], x3[0], x3[1]};
        };
        auto read_b8 = [&](i32x8* b, int st) {
            const char* bt = Bs + (st % NB) * SLICE_LDS + browf;
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                const char* r = bt + j * 16 * F8_BSTR;
                rd4(b[j], r, r + 32, r + 64, r + 96);
            }
        };
        const char* pb = reinterpret_cast<const char*>(patch);
        auto f8step = [&](i32x8* bc, i32x8* bn, int st) {
            if (st + 1 < NSTEP && !(DIAG & 32)) {
                // own share of slice st+1 landed (st+2 .. st+NB-2 may stay in
                // flight); this wave's reads of slice st-1 (whose buffer the
                // next issue overwrites) were consumed by step st-1's MFMAs
                const int ahead = min(NB - 3, NSTEP - 2 - st);
                if (hi_share) wait_vm<GHI>(ahead);
                else wait_vm<GLO>(ahead);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                if (st + NB - 1 < NSTEP) { AA_GLDS(st + NB - 1) }  // into the buffer slice st-1 was read from
            }
            const int o0 = choff(4 * st), o1 = choff(4 * st + 1), o2 = choff(4 * st + 2), o3 = choff(4 * st + 3);
            // A fragments three deep (fragment i+2 in flight under fragment
            // i's MFMAs), the next step's B fragments issued after the first
            // two A reads so the first MFMAs do not wait behind them (LDS
            // reads retire in order)
            i32x8 a3[3];
            auto rda = [&](int i, int k) {
                if ((DIAG & 128) && st > 0) return;
                const char* a = pb + abase[i];
                rd4(a3[k], a + o0, a + o1, a + o2, a + o3);
            };
            rda(0, 0);
            if (MF > 1) rda(1, 1);
            if (st + 1 < NSTEP && !((DIAG & 128) && st > 0)) read_b8(bn, st + 1);
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                if (i + 2 < MF) rda(i + 2, (i + 2) % 3);
#pragma unroll
                for (int j = 0; j < NF; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bc[j], a3[i % 3], acc[i][j], 0, 0, 0, 0,
                                                                                 0, 0);
            }
        };
        i32x8 B0[NF], B1[NF];
        {  // slice 0: own share landed (later slices stay in flight), one barrier publishes it
            const int ahead = min(NB - 2, NSTEP - 1);
            if (hi_share) wait_vm_lgkm<GHI>(ahead);
            else wait_vm_lgkm<GLO>(ahead);
            __builtin_amdgcn_s_barrier();
            read_b8(B0, 0);
        }
        for (int st = 0; st < NSTEP; st += 2) {
            f8step(B0, B1, st);
            if (st + 1 < NSTEP) f8step(B1, B0, st + 1);
        }
    } else {
    if constexpr (DB) AA_LOAD_A(fa, 0, 0)
    for (int t = 0; t < ((DIAG & 2) ? 0 : NTAP); ++t) {
        // slices t+1 .. min(t+NB-2, NTAP-1) may stay in flight
        const int ahead = min(NB - 2, NTAP - 1 - t);
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
            if (t + NB - 1 < NTAP) { AA_GLDS(t + NB - 1) }
        }
        const int buf = (DIAG & 16) ? 0 : (t % NB);
        if constexpr (!DB) {
#pragma unroll
            for (int cc = 0; cc < CPC; ++cc) {
                AA_LOAD_A(fa, t, cc)
                AA_LOAD_B(fb, buf, cc)
#pragma unroll
                for (int i = 0; i < MF; ++i)
#pragma unroll
                    for (int j = 0; j < NF; ++j) acc[i][j] = mfma_chunk(fb[j], fa[i], acc[i][j]);
            }
            continue;
        }
        AA_LOAD_B(fb, buf, 0)
#pragma unroll
        for (int cc = 0; cc < CPC; ++cc) {
            if (cc + 1 < CPC) {
                AA_LOAD_A(na, t, cc + 1)
                AA_LOAD_B(nb, buf, cc + 1)
            } else if (t + 1 < NTAP) {
                AA_LOAD_A(na, t + 1, 0)
            }
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int j = 0; j < NF; ++j) acc[i][j] = mfma_chunk(fb[j], fa[i], acc[i][j]);
#pragma unroll
            for (int i = 0; i < MF; ++i) fa[i] = na[i];
            if (cc + 1 < CPC) {
#pragma unroll
                for (int j = 0; j < NF; ++j) fb[j] = nb[j];
            }
        }
    }
    }  // !K128
#undef AA_LOAD_A
#undef AA_LOAD_B
#undef AA_GLDS
    __syncthreads();  // patch no longer needed: reuse LDS for the f32 tile

    // The MFMAs compute D = W X^T (weights as the A operand): lane holds
    // output channels c0 .. c0 + 3 of pixel p, stored as one 8-byte (bf16) /
    // 16-byte (f32) vector per fragment
    ET* E = reinterpret_cast<ET*>(smem);
    // fp8: per-output-channel dequantisation scales follow the bias (both padded to cout_pad)
    const float* wscale = bias + gridDim.y * BN;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const int c0 = wn * NF * 16 + j * 16 + 4 * (lane >> 4);
        float bj[4], sj[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bj[r] = EBF16 ? bias[blockIdx.y * BN + c0 + r] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) sj[r] = (EBF16 && F8) ? wscale[blockIdx.y * BN + c0 + r] : 1.f;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int p = (wm * MF + i) * 16 + (lane & 15);
            if (p < TP) {
                ET* e = E + p * ESTR + c0;
                if constexpr (EBF16) {
                    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
                    bf16x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = (bf16)(F8 ? fmaf(acc[i][j][r], sj[r], bj[r]) : acc[i][j][r] + bj[r]);
                    *reinterpret_cast<bf16x4*>(e) = v;
                } else {
                    *reinterpret_cast<float4*>(e) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
                }
            }
        }
    }
    __syncthreads();

    // pooled outputs: each thread owns one 8-channel group (bias in registers)
    // and writes 16-B (bf16) / 32-B (f32) vectors
    constexpr int PHo = TH / POOL, PWo = TW / POOL;
    constexpr int G = BN / 8;
    static_assert(NTHR % G == 0, "fixed channel group per thread");
    const int oh0s = oh0 / POOL, ow0s = ow0 / POOL;
    const int col = (threadIdx.x % G) * 8;
    const int ch0 = blockIdx.y * BN + col;
    float bv[8], sv[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) bv[c] = EBF16 ? 0.f : bias[ch0 + c];  // bias is padded to cout_pad
#pragma unroll
    for (int c = 0; c < 8; ++c) sv[c] = (!EBF16 && F8) ? wscale[ch0 + c] : 1.f;
    GT* dst = out + (size_t)n * Hout * Wout * cout_store;
    for (int q = threadIdx.x / G; q < PHo * PWo; q += NTHR / G) {
        const int pr = q / PWo, pc = q - (q / PWo) * PWo;
        const int gh = oh0s + pr, gw = ow0s + pc;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = -INFINITY;
#pragma unroll
        for (int dy = 0; dy < POOL; ++dy)
#pragma unroll
            for (int dx = 0; dx < POOL; ++dx) {
                const ET* e = E + ((pr * POOL + dy) * TW + pc * POOL + dx) * ESTR + col;
                if constexpr (EBF16) {
                    const bf16x8 a = *reinterpret_cast<const bf16x8*>(e);
#pragma unroll
                    for (int c = 0; c < 8; ++c) v[c] = fmaxf(v[c], (float)a[c]);
                } else {
                    const float4 a = reinterpret_cast<const float4*>(e)[0], b = reinterpret_cast<const float4*>(e)[1];
                    v[0] = fmaxf(v[0], a.x); v[1] = fmaxf(v[1], a.y); v[2] = fmaxf(v[2], a.z); v[3] = fmaxf(v[3], a.w);
                    v[4] = fmaxf(v[4], b.x); v[5] = fmaxf(v[5], b.y); v[6] = fmaxf(v[6], b.z); v[7] = fmaxf(v[7], b.w);
                }
            }
        if (gh >= Hout || gw >= Wout) continue;
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = apply_act((!EBF16 && F8) ? fmaf(v[c], sv[c], bv[c]) : v[c] + bv[c], act, alpha);
        if constexpr ((DIAG & 4) != 0) {
            if (v[0] != 12345.f) continue;  // keep the values live, store (almost) never
        }
        GT* o = dst + ((size_t)gh * Wout + gw) * cout_store + ch0;
        if (ch0 + 8 <= cout_store) {
            if constexpr (F8) {
                *reinterpret_cast<uint2*>(o) = make_uint2(pack4_fp8(v[0], v[1], v[2], v[3]), pack4_fp8(v[4], v[5], v[6], v[7]));
            } else if constexpr (sizeof(GT) == 2) {
                bf16x8 pk;
#pragma unroll
                for (int c = 0; c < 8; ++c) pk[c] = (bf16)v[c];
                *reinterpret_cast<bf16x8*>(o) = pk;
            } else {
                reinterpret_cast<float4*>(o)[0] = make_float4(v[0], v[1], v[2], v[3]);
                reinterpret_cast<float4*>(o)[1] = make_float4(v[4], v[5], v[6], v[7]);
            }
        } else {
            for (int c = 0; c < 8 && ch0 + c < cout_store; ++c) o[c] = to_t<GT>(v[c]);
        }
    }
}

// ---------------------------------------------------------------------------
// conv_head: 1x1 conv (C_in % 32 == 0) + global max + sigmoid.  Pixel ranges
// of 64 per block (blockIdx.y), 32 labels per block (blockIdx.z: label group);
// 4 waves along pixels, MF tiles each per chunk, NF = 2 label tiles.
// ---------------------------------------------------------------------------
template <typename T, int MF, int NF>
__global__ __launch_bounds__(256) void conv_head(const T* __restrict__ in, int HW, int cin,
                                                 const T* __restrict__ wt, const float* __restrict__ bias,
                                                 int L, int act, float alpha, int sigmoid,
                                                 float* __restrict__ logits, float* __restrict__ probs,
                                                 float* __restrict__ part, const float* __restrict__ wscale) {
    const int n = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q8 = 8 * (lane >> 4);
    const int lg = blockIdx.z * 16 * NF;  // first label of this block's group
    const T* src = in + (size_t)n * HW * cin;
    const T* bptr[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) bptr[j] = wt + (size_t)(lg + j * 16 + (lane & 15)) * cin + q8;
    float rmax[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) rmax[j] = -INFINITY;
    constexpr int CHUNK = 4 * MF * 16;
    for (int p0 = blockIdx.y * CHUNK; p0 < HW; p0 += CHUNK * gridDim.y) {
        f32x4 acc[MF][NF];
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        int arow[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int p = p0 + (wave * MF + i) * 16 + (lane & 15);
            arow[i] = (p < HW ? p : 0) * cin + q8;
        }
#pragma unroll 2
        for (int k0 = 0; k0 < cin; k0 += 32) {
            Frag<T> b[NF];
#pragma unroll
            for (int j = 0; j < NF; ++j) b[j].load(bptr[j] + k0);
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                Frag<T> a;
                a.load(src + arow[i] + k0);
#pragma unroll
                for (int j = 0; j < NF; ++j) acc[i][j] = mfma_chunk(a, b[j], acc[i][j]);
            }
        }
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int prow = p0 + (wave * MF + i) * 16 + 4 * (lane >> 4);
#pragma unroll
            for (int j = 0; j < NF; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (prow + r < HW) rmax[j] = fmaxf(rmax[j], acc[i][j][r]);
        }
    }
    __shared__ float red[4][16 * NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        float v = rmax[j];
        v = fmaxf(v, __shfl_xor(v, 16, 64));
        v = fmaxf(v, __shfl_xor(v, 32, 64));
        if (lane < 16) red[wave][j * 16 + lane] = v;
    }
    __syncthreads();
    if (threadIdx.x < 16 * NF) {  // one of gridDim.y pixel ranges: its column maxima, finished by head_final
        const int lp = gridDim.z * 16 * NF;  // cout_pad
        part[((size_t)n * gridDim.y + blockIdx.y) * lp + lg + threadIdx.x] =
            fmaxf(fmaxf(red[0][threadIdx.x], red[1][threadIdx.x]), fmaxf(red[2][threadIdx.x], red[3][threadIdx.x]));
    }
}

// global max over the head's pixel ranges, bias, activation, sigmoid
__global__ __launch_bounds__(256) void head_final(const float* __restrict__ part, int nparts, int width,
                                                  const float* __restrict__ bias, int L, int act, float alpha,
                                                  int sigmoid, float* __restrict__ logits,
                                                  float* __restrict__ probs, const float* __restrict__ wscale) {
    const int n = blockIdx.x;
    for (int c = threadIdx.x; c < L; c += blockDim.x) {
        const float* p = part + (size_t)n * nparts * width + c;
        float v = p[0];
        for (int k = 1; k < nparts; ++k) v = fmaxf(v, p[(size_t)k * width]);
        v = apply_act(wscale ? fmaf(v, wscale[c], bias[c]) : v + bias[c], act, alpha);
        logits[(size_t)n * L + c] = v;
        if (probs) probs[(size_t)n * L + c] = sigmoid ? 1.f / (1.f + expf(-v)) : v;
    }
}

// ---------------------------------------------------------------------------
// Generic stages for layer shapes no tuned kernel covers (the planner's
// fallback, exact f32 arithmetic on the VALU): any kernel size, any C_in,
// any max-pool window, optional MagTransform prologue.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f(fp8 x) {  // OCP e4m3fn
    const int s = x.v >> 7, e = (x.v >> 3) & 15, m = x.v & 7;
    float v = e ? ldexpf(1.f + m / 8.f, e - 7) : ldexpf(m / 8.f, -6);
    if (e == 15 && m == 7) v = NAN;
    return s ? -v : v;
}

// one thread = one (pooled) output pixel x 8 output channels; weights
// [cout][kh][kw][cin] f32 (BN folded), bias f32
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void conv_generic(const TI* __restrict__ in, int Hin, int Win, int cin,
                                                    const float* __restrict__ w, const float* __restrict__ bias,
                                                    int kh, int kw, int cout, int ph, int pw, int Hout, int Wout,
                                                    int act, float alpha, int has_mag, float mag_exp,
                                                    TO* __restrict__ out) {
    const int n = blockIdx.z;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int c0 = blockIdx.y * 8;
    if (p >= Hout * Wout) return;
    const int oh = p / Wout, ow = p - (p / Wout) * Wout;
    const int K = kh * kw * cin;
    const int nc = min(8, cout - c0);
    float best[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) best[o] = -INFINITY;
    const TI* img = in + (size_t)n * Hin * Win * cin;
    for (int dy = 0; dy < ph; ++dy)
        for (int dx = 0; dx < pw; ++dx) {
            const int h = oh * ph + dy, x = ow * pw + dx;
            float acc[8];
#pragma unroll
            for (int o = 0; o < 8; ++o) acc[o] = 0.f;
            for (int i = 0; i < kh; ++i)
                for (int j = 0; j < kw; ++j) {
                    const TI* src = img + ((size_t)(h + i) * Win + x + j) * cin;
                    const float* wk = w + (size_t)c0 * K + (i * kw + j) * cin;
                    for (int c = 0; c < cin; ++c) {
                        float v = to_f(src[c]);
                        if (has_mag) v = powf(v, mag_exp);
#pragma unroll
                        for (int o = 0; o < 8; ++o)
                            if (o < nc) acc[o] = fmaf(v, wk[(size_t)o * K + c], acc[o]);
                    }
                }
#pragma unroll
            for (int o = 0; o < 8; ++o)
                if (o < nc) best[o] = fmaxf(best[o], apply_act(acc[o] + bias[c0 + o], act, alpha));
        }
    TO* dst = out + ((size_t)(n * Hout + oh) * Wout + ow) * cout + c0;
    for (int o = 0; o < nc; ++o) dst[o] = to_t<TO>(best[o]);
}

// GlobalMaxPool2D over a stage's output, then an optional Dense layer
// (weights [C][U] f32, bias [U]) and sigmoid; one block per window
template <typename TI>
__global__ __launch_bounds__(256) void pool_dense(const TI* __restrict__ in, int HW, int C,
                                                  const float* __restrict__ w, const float* __restrict__ b, int U,
                                                  int sigmoid, float* __restrict__ logits, float* __restrict__ probs) {
    extern __shared__ float mx[];
    const int n = blockIdx.x;
    const TI* src = in + (size_t)n * HW * C;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float m = -INFINITY;
        for (int p = 0; p < HW; ++p) m = fmaxf(m, to_f(src[(size_t)p * C + c]));
        mx[c] = m;
    }
    __syncthreads();
    for (int u = threadIdx.x; u < U; u += blockDim.x) {
        float v;
        if (w) {
            v = 0.f;
            for (int c = 0; c < C; ++c) v = fmaf(mx[c], w[(size_t)c * U + u], v);
            v += b[u];
        } else {
            v = mx[u];
        }
        logits[(size_t)n * U + u] = v;
        if (probs) probs[(size_t)n * U + u] = sigmoid ? 1.f / (1.f + expf(-v)) : v;
    }
}

// ---------------------------------------------------------------------------
// track mean: mean over models, then over the track's windows (f32,
// sequential, src/identify_tracks.py:547-551)
// ---------------------------------------------------------------------------
__global__ void track_mean(const float* __restrict__ probs, int n_models, long long model_stride, int L,
                           const int* __restrict__ wb, const int* __restrict__ wc,
                           float* __restrict__ out) {
    const int t = blockIdx.x;
    const int c = threadIdx.x;
    if (c >= L) return;
    constexpr int U = 40;  // loads in flight (a 60 s track has 39 windows); the adds stay in numpy's order
    float acc = 0.f;
    const int n = wc[t];
    const float* base = probs + (size_t)wb[t] * L + c;
    for (int w0 = 0; w0 < n; w0 += U) {
        float m[U];  // per window: ((0 + p_0) + p_1) + ..., numpy's axis-0 sum over models
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = 0.f;
        for (int k = 0; k < n_models; ++k) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = base[k * model_stride + (size_t)min(w0 + u, n - 1) * L];
#pragma unroll
            for (int u = 0; u < U; ++u) m[u] = __fadd_rn(m[u], v[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (w0 + u < n) acc = __fadd_rn(acc, __fdiv_rn(m[u], (float)n_models));
    }
    out[(size_t)t * L + c] = n > 0 ? __fdiv_rn(acc, (float)n) : NAN;
}

}  // namespace aa

#include "aa_conv_x3.h"
#include "aa_conv_wg.h"
#include "aa_gconv.h"
#include "aa_conv_tail.h"

namespace aa {

// ---------------------------------------------------------------------------
// host: planner, workspace, forward, timing
// ---------------------------------------------------------------------------
// ST_SMALL: C_in = 1 3x3 -> 32 first conv (VALU, fusable into the next
// stage); ST_MFMA: tuned matrix-core conv; ST_HEAD: 1x1 conv + global max;
// ST_GENERIC: any other conv shape / pool window (f32 VALU fallback);
// ST_POOLDENSE: GlobalMaxPool2D [+ Dense] [+ sigmoid] after a conv stage;
// ST_GCONV: split-bf16 mode, a conv with C_in >= 16 and no tuned tile: the
// runtime-shaped MFMA kernel gconv_x3 (aa_gconv.h) [+ gpool2d for the max pool]
enum StageKind { ST_SMALL = 0, ST_MFMA = 1, ST_HEAD = 2, ST_GENERIC = 3, ST_POOLDENSE = 4, ST_GCONV = 5 };

struct Stage {
    int kind = ST_MFMA;
    int kh = 1, kw = 1, cin = 0, cout = 0, cout_pad = 0;
    int pool = 1;        // square pool window of the tuned kernels (1 or 3), 0 otherwise
    int ph = 1, pw = 1;  // max-pool window (= strides)
    int act = ACT_NONE;
    float alpha = 0.f;
    int has_mag = 0;
    float mag_exp = 1.f;
    int sigmoid = 0;
    int Hin = 0, Win = 0, Hc = 0, Wc = 0, Hout = 0, Wout = 0;
    void* d_w = nullptr;
    float* d_b = nullptr;
    double flops = 0, bytes = 0;  // algorithmic per window
    std::string name;
    int skipped = 0;    // first layer computed inside the next stage
    int is_first = 0;   // reads the model input (f32 log-mel)
    int fused_first = 0;  // this stage computes the previous (first) layer itself
    int lm_f16 = 0;       // fused_first: the model input is float16
    int in_split = 0;     // split-bf16: input / output in the grouped-split layout (aa_conv_x3.h)
    int out_split = 0;
    int wg = 0;           // split-bf16 Winograd F(wg, 3)-along-W kernel (aa_conv_wg.h, wg = WO) and its weight packing
    int wg_npass = 1;     // its staging passes (planes per pass = (wg + 2) / wg_npass)
    int cin_pad = 0;      // ST_GCONV: C_in rounded up to 32
    int tail = 0;         // ST_HEAD, split-bf16: computes the previous conv stage itself (aa_conv_tail.h)
    void* d_tw = nullptr;  // tail: head weights packed per wave / label fragment, hi then lo
};

struct Model {
    int prec = AA_PREC_BF16;
    int in_h = 0, in_w = 0, in_c = 0;
    int L = 0;
    std::vector<Stage> st;
    size_t act_elems[2] = {0, 0};  // per-window elements of the ping-pong buffers
    size_t tmp_elems = 0;          // per-window f32 elements of an ST_GCONV stage's unpooled output
    StageTimer timer;  // HIP events around the stages in timer.mask
};


template <typename T, int KH, int KW, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW,
          bool FUSED = false, bool EBF16 = false, int OCC = 0>
static int launch_mfma(const Stage& s, const void* in, void* out, int n, hipStream_t st,
                       const Stage* first = nullptr) {
    auto k = conv_mfma<T, KH, KW, CIN, WM, WN, MF, NF, POOL, TH, TW, FUSED, 0, EBF16, OCC>;
    constexpr int BN = WN * NF * 16;
    const size_t lds = conv_lds_bytes<T, KH, KW, CIN, BN, TH, TW, FUSED, EBF16>();
    FirstConv fc{};
    if (FUSED) {
        const float slope = first->act == ACT_LEAKY ? first->alpha : first->act == ACT_RELU ? 0.f : 1.f;
        fc = FirstConv{(const float*)first->d_w, first->d_b, first->act, slope, first->has_mag,
                       first->mag_exp, first->Hin, first->Win, s.lm_f16};
    }
    AA_CHECK(lds <= 160 * 1024, AA_ERR_UNSUPPORTED, "conv %s: %zu B LDS", s.name.c_str(), lds);
    AA_DYN_LDS(k, lds);
    const int tiles_h = (s.Hout * POOL + TH - 1) / TH;
    const int tiles_w = (s.Wout * POOL + TW - 1) / TW;
    dim3 grid(tiles_h * tiles_w, s.cout_pad / BN, n);
    using GT = typename Prec<T>::G;
    using LT = typename Prec<T>::L;
    hipLaunchKernelGGL(k, grid, dim3(WM * WN * 64), lds, st, (const GT*)in, s.Hin, s.Win, (const LT*)s.d_w, s.d_b,
                       (GT*)out, s.Hout, s.Wout, s.cout, tiles_w, s.act, s.alpha, fc);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

// Tile configuration of every conv_mfma instantiation, one line per
// (dtype, kernel, C_in, pool): waves (WM x WN), 16x16 fragments per wave
// (MF x NF), output tile TH x TW, bf16 epilogue tile.  BN = WN * NF * 16
// output channels per block.  The f32 rows are the parity mode (smaller
// tiles: the same LDS budget holds half the elements).
#define AA_CONV_CFGS(X)                                     \
    X(bf16, 3, 3, 32, 3, 4, 1, 6, 2, 18, 21, true, 0)          \
    X(bf16, 3, 3, 32, 1, 2, 2, 4, 2, 8, 16, true, 0)           \
    X(bf16, 3, 3, 64, 1, 2, 2, 4, 2, 8, 16, true, 0)           \
    X(bf16, 9, 3, 64, 3, 4, 2, 6, 4, 39, 9, true, 0)           \
    X(bf16, 1, 3, 128, 1, 2, 4, 5, 2, 7, 20, false, 0)         \
    X(fp8, 3, 3, 32, 3, 4, 1, 6, 2, 12, 30, true, 0)           \
    X(fp8, 3, 3, 32, 1, 2, 2, 4, 2, 8, 16, true, 0)            \
    X(fp8, 3, 3, 64, 1, 4, 1, 3, 4, 12, 16, true, 0)           \
    X(fp8, 9, 3, 64, 3, 4, 2, 6, 4, 21, 18, true, 0)           \
    X(fp8, 1, 3, 128, 1, 2, 4, 5, 2, 7, 20, true, 0)           \
    X(float, 3, 3, 32, 3, 2, 2, 9, 1, 6, 48, false, 0)         \
    X(float, 3, 3, 32, 1, 1, 4, 9, 1, 6, 24, false, 0)         \
    X(float, 3, 3, 64, 1, 1, 4, 9, 1, 6, 24, false, 0)         \
    X(float, 9, 3, 64, 3, 1, 4, 7, 1, 3, 33, false, 0)         \
    X(float, 1, 3, 128, 1, 2, 2, 5, 1, 6, 24, false, 0)

// conv_x3 (split-bf16) instantiations: (kernel, C_in, pool) -> waves (WM x
// WN), fragments per wave (MF x NF), output tile TH x TW, weight ring in LDS
// (1) or per-wave B fragments from global (0), A fragments just in time (1)
// or a whole step ahead (0), pinned waves per SIMD (0: free); picked by
// tools/conv_bench_x3.hip sweeps
#ifdef AA_X3_ALT  // tools/ab_build.py: an alternative tile table for in-pipeline A/B runs
#define AA_X3_CFGS(X) AA_X3_ALT(X)
#else
#define AA_X3_CFGS(X)                                 \
    X(3, 3, 32, 3, 4, 1, 4, 2, 12, 21, 0, 1, 0)       \
    X(3, 3, 32, 1, 4, 2, 3, 2, 10, 18, 1, 0, 4)       \
    X(3, 3, 64, 1, 2, 2, 3, 2, 12, 8, 1, 1, 0)        \
    X(9, 3, 64, 3, 2, 2, 4, 2, 21, 6, 0, 1, 4)        \
    X(1, 3, 128, 1, 2, 2, 3, 2, 7, 12, 1, 1, 0)
#endif

// conv_wg (split-bf16, Winograd F(WO,3) along W) instantiations: (kh, C_in,
// pool) of kernel-width-3 convs -> waves (WM x WN), fragments per wave (MF x
// NF, each with WO + 2 accumulator sets), output tile TH x TW (TW a multiple
// of WO), pinned waves per SIMD (0: free), outputs per group WO, staging
// passes NPASS, B fragment sets in flight BD.  Preferred over conv_x3 where a row exists (the
// fused first-layer stage always runs conv_x3).  In-pipeline A/B (tools/ab.sh,
// same box): the 9x3 layer 187 -> 160 us, step 180k -> 193k audio-s/s; the
// small 3x3 / 1x3 layers lose on it (their transform-heavy staging outweighs
// the saved MFMAs: 3x3/32 36 -> 55 us, 3x3/64 52 -> 76 us, 1x3 22 -> 28 us).
#ifdef AA_WG_ALT
#define AA_WG_CFGS(X) AA_WG_ALT(X)
#else
// F(6,3) for the 9x3 layer (in-pipeline A/B, 3 rounds on one box: 9x3 131 ->
// 122 us, step 260k -> 264k; F(4,3) on 39x12 tiles 140 us, F(3,3) spills):
// 8 planes of the 39 x 6 tile's single column group, 4 waves of 16 output
// channels each, 96 accumulator VGPRs
#define AA_WG_CFGS(X) X(9, 64, 3, 1, 4, 3, 1, 39, 6, 0, 6, 1, 2)
#endif

static int wg_bn(int kh, int kw, int cin, int pool) {
#define AA_WBN(KH, CIN, POOL, WM, WN, MF, NF, TH, TW, OCC, WO, NPASS, BD) \
    if (kw == 3 && kh == KH && cin == CIN && pool == POOL) return WN * NF * 16;
    AA_WG_CFGS(AA_WBN)
#undef AA_WBN
    return 0;
}
// (WO, NPASS) of the Winograd instantiation serving a stage
static void wg_form(int kh, int cin, int pool, int* wo, int* npass) {
#define AA_WFORM(KH, CIN, POOL, WM, WN, MF, NF, TH, TW, OCC, WO, NPASS, BD) \
    if (kh == KH && cin == CIN && pool == POOL) { *wo = WO; *npass = NPASS; return; }
    AA_WG_CFGS(AA_WFORM)
#undef AA_WFORM
    *wo = 0;
    *npass = 1;
}

template <typename T>
constexpr int prec_of() {
    return is_split<T>() ? AA_PREC_BF16X3 : sizeof(T) == 1 ? AA_PREC_FP8 : sizeof(T) == 2 ? AA_PREC_BF16 : AA_PREC_F32;
}
// bytes of one stored activation (split-bf16 keeps f32 activations)
static size_t prec_bytes(int prec) { return prec == AA_PREC_FP8 ? 1 : prec == AA_PREC_BF16 ? 2 : 4; }

// output channels per block of the instantiation serving this stage (0: none)
static int mfma_bn(int prec, int kh, int kw, int cin, int pool) {
    if (prec == AA_PREC_BF16X3 && wg_bn(kh, kw, cin, pool)) return wg_bn(kh, kw, cin, pool);
#define AA_BN(T_, KH, KW, CIN, POOL, WM, WN, MF, NF, TH, TW, EB, OCC)                                       \
    if (prec_of<T_>() == prec && kh == KH && kw == KW && cin == CIN && pool == POOL) \
        return WN * NF * 16;
    AA_CONV_CFGS(AA_BN)
#undef AA_BN
#define AA_BN3(KH, KW, CIN, POOL, WM, WN, MF, NF, TH, TW, RING, AJIT, OCC)                                               \
    if (prec == AA_PREC_BF16X3 && kh == KH && kw == KW && cin == CIN && pool == POOL) return WN * NF * 16;
    AA_X3_CFGS(AA_BN3)
#undef AA_BN3
    return 0;
}

template <int KH, int KW, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW, bool RING, bool AJIT,
          int OCC, bool FUSED, bool IN_SPLIT, bool OUT_SPLIT>
static int launch_x3(const Stage& s, const void* in, void* out, int n, hipStream_t st, const Stage* first) {
    auto k = conv_x3<KH, KW, CIN, WM, WN, MF, NF, POOL, TH, TW, FUSED, 0, RING, AJIT, OCC, IN_SPLIT, OUT_SPLIT>;
    constexpr int BN = WN * NF * 16;
    // buffer-resource addressing: the resources are based at the window
    // (64-bit), offsets inside one window are 32-bit
    AA_CHECK((double)s.Hin * s.Win * s.cin * 4 < 2147483647.0, AA_ERR_UNSUPPORTED,
             "conv %s: one window's activations exceed 2 GiB", s.name.c_str());
    const size_t lds = x3_lds_bytes<KH, KW, CIN, BN, TH, TW, FUSED, RING>();
    FirstConv fc{};
    if (FUSED) {
        const float slope = first->act == ACT_LEAKY ? first->alpha : first->act == ACT_RELU ? 0.f : 1.f;
        fc = FirstConv{(const float*)first->d_w, first->d_b, first->act, slope, first->has_mag,
                       first->mag_exp, first->Hin, first->Win, s.lm_f16};
    }
    AA_CHECK(lds <= 160 * 1024, AA_ERR_UNSUPPORTED, "conv %s: %zu B LDS", s.name.c_str(), lds);
    AA_DYN_LDS(k, lds);
    const int tiles_h = (s.Hout * POOL + TH - 1) / TH;
    const int tiles_w = (s.Wout * POOL + TW - 1) / TW;
    dim3 grid(tiles_h * tiles_w, s.cout_pad / BN, n);
    hipLaunchKernelGGL(k, grid, dim3(WM * WN * 64), lds, st, (const float*)in, s.Hin, s.Win, (const bf16*)s.d_w,
                       s.d_b, (float*)out, s.Hout, s.Wout, s.cout, tiles_w, s.act, s.alpha, fc);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

template <int KH, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW, int OCC, int WO, int NPASS,
          int BD, bool IN_SPLIT, bool OUT_SPLIT>
static int launch_wg(const Stage& s, const void* in, void* out, int n, hipStream_t st) {
    auto k = conv_wg<KH, CIN, WM, WN, MF, NF, POOL, TH, TW, OCC, IN_SPLIT, OUT_SPLIT, 0, WO, NPASS, BD>;
    constexpr int BN = WN * NF * 16;
    AA_CHECK((double)s.Hin * s.Win * s.cin * 4 < 2147483647.0, AA_ERR_UNSUPPORTED,
             "conv %s: one window's activations exceed 2 GiB", s.name.c_str());
    const size_t lds = wg_lds_bytes<KH, BN, TH, TW, WO, NPASS, WN>();
    AA_CHECK(lds <= 160 * 1024, AA_ERR_UNSUPPORTED, "conv %s: %zu B LDS", s.name.c_str(), lds);
    AA_DYN_LDS(k, lds);
    const int tiles_h = (s.Hout * POOL + TH - 1) / TH;
    const int tiles_w = (s.Wout * POOL + TW - 1) / TW;
    dim3 grid(tiles_h * tiles_w, s.cout_pad / BN, n);
    hipLaunchKernelGGL(k, grid, dim3(WM * WN * 64), lds, st, (const float*)in, s.Hin, s.Win, (const bf16*)s.d_w,
                       s.d_b, (float*)out, s.Hout, s.Wout, s.cout, tiles_w, s.act, s.alpha);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

template <typename T>
static int launch_stage(const Model& m, const Stage& s, const void* in, void* out, float* logits,
                        float* probs, int n, hipStream_t st, const Stage* first, float* tmp) {
    using GT = typename Prec<T>::G;
    if (s.kind == ST_SMALL) {
        dim3 grid((s.Hc * s.Wc + 255) / 256, n);
        hipLaunchKernelGGL((conv_small<GT, 3, 3, 32>), grid, dim3(256), 0, st, (const float*)in, s.Hin,
                           s.Win, (const float*)s.d_w, s.d_b, s.has_mag, s.mag_exp, (GT*)out, s.Hc, s.Wc,
                           s.act, s.alpha);
        AA_LAUNCH_CHECK();
        return AA_OK;
    }
    if (s.kind == ST_GCONV) {
        if constexpr (!is_split<T>()) {
            set_error("%s: the runtime-shaped MFMA conv is split-bf16 only", s.name.c_str());
            return AA_ERR_UNSUPPORTED;
        } else {
            const ConvGeom g{s.Hin, s.Win, s.cin, s.Hc, s.Wc, s.cout, s.kh, s.kw, 1, 1, 0, 0, s.cin_pad};
            const bool pooled = s.ph > 1 || s.pw > 1;
            float* conv_out = pooled ? tmp : static_cast<float*>(out);
            const int gact_ = s.act == ACT_LEAKY ? GACT_LEAKY : s.act == ACT_RELU ? GACT_RELU : GACT_NONE;
            hipLaunchKernelGGL((gconv_x3t<2, 2, 2, 2>), dim3((s.Hc * s.Wc + 63) / 64, s.cout_pad / 64, n), dim3(256), 0, st,
                               (const float*)in, (const uint16_t*)s.d_w, s.d_b, conv_out, g, s.cout_pad, gact_,
                               s.alpha, nullptr, nullptr);
            AA_LAUNCH_CHECK();
            if (pooled) {  // max pool after the (monotonic) activation: the pool of the activated values
                const size_t items = (size_t)s.Hout * s.Wout * s.cout;
                hipLaunchKernelGGL(gpool2d, dim3((unsigned)((items + 255) / 256), n), dim3(256), 0, st, tmp,
                                   (float*)out, s.Hc, s.Wc, s.cout, s.Hout, s.Wout, s.ph, s.pw, s.ph, s.pw, 0, 0, 0,
                                   GACT_NONE, 0.f);
                AA_LAUNCH_CHECK();
            }
            return AA_OK;
        }
    }
    if (s.kind == ST_GENERIC) {
        if constexpr (is_fp8<T>()) {
            set_error("%s: no fp8 kernel for this shape", s.name.c_str());
            return AA_ERR_UNSUPPORTED;
        } else {
            dim3 grid((s.Hout * s.Wout + 255) / 256, (s.cout + 7) / 8, n);
            if (s.is_first) {  // reads the f32 model input (log-mel)
                hipLaunchKernelGGL((conv_generic<float, GT>), grid, dim3(256), 0, st, (const float*)in, s.Hin,
                                   s.Win, s.cin, (const float*)s.d_w, s.d_b, s.kh, s.kw, s.cout, s.ph, s.pw, s.Hout,
                                   s.Wout, s.act, s.alpha, s.has_mag, s.mag_exp, (GT*)out);
            } else {
                hipLaunchKernelGGL((conv_generic<GT, GT>), grid, dim3(256), 0, st, (const GT*)in, s.Hin, s.Win,
                                   s.cin, (const float*)s.d_w, s.d_b, s.kh, s.kw, s.cout, s.ph, s.pw, s.Hout,
                                   s.Wout, s.act, s.alpha, 0, 1.f, (GT*)out);
            }
            AA_LAUNCH_CHECK();
            return AA_OK;
        }
    }
    if (s.kind == ST_POOLDENSE) {
        hipLaunchKernelGGL((pool_dense<GT>), dim3(n), dim3(256), (size_t)s.cin * sizeof(float), st, (const GT*)in,
                           s.Hin * s.Win, s.cin, (const float*)s.d_w, s.d_b, s.cout, s.sigmoid, logits, probs);
        AA_LAUNCH_CHECK();
        return AA_OK;
    }
    if (s.kind == ST_HEAD && s.tail) {
        if constexpr (is_split<T>()) {
            // the last conv stage and the head in one launch (aa_conv_tail.h):
            // per-tile label maxima into `out`, then head_final over the tiles
            const Stage& c = *first;
#ifndef AA_TAIL_TW  // (A/B knobs: tile width and pixel fragments per wave)
#define AA_TAIL_TW 5
#define AA_TAIL_MF 5
#endif
            constexpr int TH = 13, TW = AA_TAIL_TW;
            const int tiles_h = (c.Hc + TH - 1) / TH, tiles_w = (c.Wc + TW - 1) / TW;
            auto k = conv_tail_x3<1, 3, 128, AA_TAIL_MF, TH, TW>;
            constexpr size_t lds = tail_lds_bytes<1, 3, 128, TH, TW>();
            AA_DYN_LDS(k, lds);
            float* part = static_cast<float*>(out);
            hipLaunchKernelGGL(k, dim3(tiles_h * tiles_w, 1, n), dim3(TAIL_NW * 64), lds, st, (const float*)in, c.Hin,
                               c.Win, (const bf16*)c.d_w, c.d_b, c.Hc, c.Wc, tiles_w, c.act, c.alpha,
                               (const bf16*)s.d_tw, part);
            AA_LAUNCH_CHECK();
            hipLaunchKernelGGL(head_final, dim3(n), dim3(64), 0, st, part, tiles_h * tiles_w, 32, s.d_b, s.cout, s.act,
                               s.alpha, s.sigmoid, logits, probs, (const float*)nullptr);
            AA_LAUNCH_CHECK();
            return AA_OK;
        } else {
            set_error("%s: the fused tail is split-bf16 only", s.name.c_str());
            return AA_ERR_UNSUPPORTED;
        }
    }
    if (s.kind == ST_HEAD) {
        // pixel ranges of 64 spread over blocks (a window alone is too little
        // work for one block's dependent load chain), 32 labels per block;
        // their column maxima go to the free ping-pong buffer `out` and
        // head_final reduces them
        const int HW = s.Hin * s.Win, parts = (HW + 63) / 64;
        float* part = static_cast<float*>(out);
        const float* hsc = is_fp8<T>() ? s.d_b + s.cout_pad : nullptr;  // fp8 dequantisation scales
        // split-bf16: the head reads f32 activations and runs the exact f32
        // MFMA (its 1x1 contraction is <1 % of the network's FLOPs)
        hipLaunchKernelGGL((conv_head<GT, 1, 2>), dim3(n, parts, s.cout_pad / 32), dim3(256), 0, st, (const GT*)in,
                           HW, s.cin, (const GT*)s.d_w, s.d_b, s.cout, s.act, s.alpha, s.sigmoid, logits, probs, part,
                           hsc);
        AA_LAUNCH_CHECK();
        hipLaunchKernelGGL(head_final, dim3(n), dim3(s.cout <= 64 ? 64 : 256), 0, st, part, parts, s.cout_pad, s.d_b,
                           s.cout, s.act, s.alpha, s.sigmoid, logits, probs, hsc);
        AA_LAUNCH_CHECK();
        return AA_OK;
    }
    if (s.fused_first) {
        AA_CHECK(s.kh == 3 && s.kw == 3 && s.cin == 32 && s.pool == 3, AA_ERR_UNSUPPORTED,
                 "no fused first-layer kernel for %s", s.name.c_str());
    }
    if constexpr (is_split<T>()) {
        if (s.wg) {
#define AA_LAUNCHW(KH, CIN, POOL, WM, WN, MF, NF, TH, TW, OCC, WO, NPASS, BD)                                       \
            if (s.kh == KH && s.cin == CIN && s.pool == POOL) {                                                   \
                if (s.in_split)                                                                                   \
                    return s.out_split ? launch_wg<KH, CIN, WM, WN, MF, NF, POOL, TH, TW, OCC, WO, NPASS, BD, true, true>(s, in, out, n, st) \
                                       : launch_wg<KH, CIN, WM, WN, MF, NF, POOL, TH, TW, OCC, WO, NPASS, BD, true, false>(s, in, out, n, st); \
                return s.out_split ? launch_wg<KH, CIN, WM, WN, MF, NF, POOL, TH, TW, OCC, WO, NPASS, BD, false, true>(s, in, out, n, st) \
                                   : launch_wg<KH, CIN, WM, WN, MF, NF, POOL, TH, TW, OCC, WO, NPASS, BD, false, false>(s, in, out, n, st); \
            }
            AA_WG_CFGS(AA_LAUNCHW)
#undef AA_LAUNCHW
            set_error("conv %dx%d cin %d pool %d: no Winograd kernel instantiation", s.kh, s.kw, s.cin, s.pool);
            return AA_ERR_UNSUPPORTED;
        }
#define AA_X3L(FU, IS, OS) launch_x3<KH_, KW_, CIN_, WM_, WN_, MF_, NF_, POOL_, TH_, TW_, RING_, AJIT_, OCC_, FU, IS, OS>(s, in, out, n, st, first)
#define AA_LAUNCH3(KH, KW, CIN, POOL, WM, WN, MF, NF, TH, TW, RING, AJIT, OCC)                            \
        if (s.kh == KH && s.kw == KW && s.cin == CIN && s.pool == POOL) {                                  \
            constexpr int KH_ = KH, KW_ = KW, CIN_ = CIN, WM_ = WM, WN_ = WN, MF_ = MF, NF_ = NF, POOL_ = POOL;  \
            constexpr int TH_ = TH, TW_ = TW, OCC_ = OCC;                                                  \
            constexpr bool RING_ = RING, AJIT_ = AJIT;                                                     \
            if (s.fused_first) {                                                                           \
                if constexpr (CIN == 32 && KH == 3 && KW == 3)                                             \
                    return s.out_split ? AA_X3L(true, false, true) : AA_X3L(true, false, false);          \
            } else if (s.in_split) {                                                                       \
                return s.out_split ? AA_X3L(false, true, true) : AA_X3L(false, true, false);              \
            } else {                                                                                       \
                return s.out_split ? AA_X3L(false, false, true) : AA_X3L(false, false, false);            \
            }                                                                                              \
        }
        AA_X3_CFGS(AA_LAUNCH3)
#undef AA_LAUNCH3
#undef AA_X3L
        set_error("conv %dx%d cin %d pool %d: no split-bf16 kernel instantiation", s.kh, s.kw, s.cin, s.pool);
        return AA_ERR_UNSUPPORTED;
    }
#define AA_LAUNCH(T_, KH, KW, CIN, POOL, WM, WN, MF, NF, TH, TW, EB, OCC)                                        \
    if constexpr (std::is_same<T, T_>::value) {                                                          \
        if (s.kh == KH && s.kw == KW && s.cin == CIN && s.pool == POOL) {                                \
            if (s.fused_first) {                                                                         \
                if constexpr (CIN == 32 && KH == 3 && KW == 3)                                           \
                    return launch_mfma<T, KH, KW, CIN, WM, WN, MF, NF, POOL, TH, TW, true, EB, OCC>(s, in, out, \
                                                                                              n, st, first); \
            } else {                                                                                     \
                return launch_mfma<T, KH, KW, CIN, WM, WN, MF, NF, POOL, TH, TW, false, EB, OCC>(s, in, out, n, st); \
            }                                                                                            \
        }                                                                                                \
    }
    AA_CONV_CFGS(AA_LAUNCH)
#undef AA_LAUNCH
    set_error("conv %dx%d cin %d pool %d: no kernel instantiation", s.kh, s.kw, s.cin, s.pool);
    return AA_ERR_UNSUPPORTED;
}

// a C_in = 1 first conv (3x3 -> 32) the next 3x3/32 pooled MFMA stage computes itself
static bool fusable_first(const Stage& a, const Stage& b) {
    return a.kind == ST_SMALL && a.kh == 3 && a.kw == 3 && a.cin == 1 && a.cout == 32 && b.kind == ST_MFMA &&
           b.cin == 32 && b.kh == 3 && b.kw == 3 && b.pool == 3 &&
           (a.act != ACT_LEAKY || (a.alpha >= 0.f && a.alpha <= 1.f));
}

static void free_model(Model* m) {
    if (!m) return;
    m->timer.release();
    for (auto& s : m->st) {
        (void)hipFree(s.d_w);
        (void)hipFree(s.d_b);
        (void)hipFree(s.d_tw);
    }
    delete m;
}

static uint16_t f2bf(float f) {  // round to nearest even
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
    u += 0x7fff + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t b) {
    const uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

// f32 -> OCP e4m3fn byte, round to nearest even, saturated to +-448 (the
// device's v_cvt_pk_fp8_f32 conversion of the same value)
static uint8_t f2fp8(float f) {
    const uint8_t sgn = std::signbit(f) ? 0x80 : 0;
    double a = std::fabs((double)f);
    if (std::isnan(f)) return 0x7f;
    if (a >= 448.0) return sgn | 0x7e;
    if (a < std::ldexp(1.0, -6)) {  // subnormal: multiples of 2^-9
        const int q = (int)std::nearbyint(a * 512.0);
        return sgn | (uint8_t)q;  // q == 8 is the smallest normal's encoding
    }
    int ex;
    std::frexp(a, &ex);  // a = m 2^ex, m in [0.5, 1)
    const int e = ex - 1;
    double q = std::nearbyint(std::ldexp(a, 3 - e));  // 8 .. 16
    int ee = e;
    if (q >= 16.0) { q = 8.0; ++ee; }
    if (ee > 8 || (ee == 8 && q > 14.0)) return sgn | 0x7e;
    return sgn | (uint8_t)(((ee + 7) << 3) | ((int)q - 8));
}

}  // namespace aa

using namespace aa;

extern "C" int aa_model_create(const aa_layer* layers, int32_t n_layers, const float* blob, int64_t blob_len,
                               int32_t in_h, int32_t in_w, int32_t in_c, int32_t precision, void** model) {
    AA_CHECK(layers && blob && model && n_layers > 0, AA_ERR_INVALID, "aa_model_create: null argument");
    AA_CHECK(precision == AA_PREC_F32 || precision == AA_PREC_BF16 || precision == AA_PREC_FP8 ||
                 precision == AA_PREC_BF16X3, AA_ERR_INVALID,
             "aa_model_create: precision %d", precision);
    auto get = [&](int64_t off, int64_t n) -> const float* {
        if (off < 0 || off + n > blob_len) return nullptr;
        return blob + off;
    };
    Model* m = new Model();
    m->prec = precision;
    m->in_h = in_h;
    m->in_w = in_w;
    m->in_c = in_c;
    int H = in_h, W = in_w, C = in_c;
    int has_mag = 0;
    float mag_exp = 1.f;
    int i = 0;
    int rc = AA_OK;
    auto fail = [&](int code, const char* msg) {
        set_error("aa_model_create: layer %d: %s", i, msg);
        rc = code;
    };
    auto upload = [&](Stage& s, const void* w, size_t wbytes, const std::vector<float>& bias) -> bool {
        hipError_t e = hipMalloc(&s.d_w, wbytes ? wbytes : 4);
        if (e == hipSuccess && wbytes) e = hipMemcpy(s.d_w, w, wbytes, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMalloc((void**)&s.d_b, sizeof(float) * std::max<size_t>(bias.size(), 1));
        if (e == hipSuccess && !bias.empty())
            e = hipMemcpy(s.d_b, bias.data(), sizeof(float) * bias.size(), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            m->st.push_back(s);
            fail(AA_ERR_HIP, hipGetErrorString(e));
            return false;
        }
        return true;
    };
    while (i < n_layers && rc == AA_OK) {
        const aa_layer& ly = layers[i];
        if (ly.op == AA_OP_MAGTRANSFORM) {
            const float* a = get(ly.off[0], 1);
            if (!a || !m->st.empty()) { fail(AA_ERR_UNSUPPORTED, "MagTransform must precede the first conv"); break; }
            has_mag = 1;
            mag_exp = 1.f / (1.f + expf(-a[0]));  // sigmoid(a) in f32 like tf.math.sigmoid
            ++i;
            continue;
        }
        if (ly.op == AA_OP_GLOBALMAXPOOL2D) {
            // GlobalMaxPool2D [+ Dense] [+ sigmoid] after a conv stage: one
            // pool_dense launch (the 1x1-conv head pattern is folded below)
            if (m->st.empty()) { fail(AA_ERR_UNSUPPORTED, "GlobalMaxPool2D before any conv"); break; }
            Stage s;
            s.kind = ST_POOLDENSE;
            s.Hin = H;
            s.Win = W;
            s.cin = C;
            s.cout = C;
            ++i;
            std::vector<float> wd, bias;
            if (i < n_layers && layers[i].op == AA_OP_DENSE) {
                const aa_layer& d = layers[i];
                s.cout = d.filters;
                const float* k = get(d.off[0], (int64_t)C * d.filters);
                if (!k || d.filters <= 0) { fail(AA_ERR_INVALID, "dense kernel outside the blob"); break; }
                wd.assign(k, k + (size_t)C * d.filters);
                bias.assign(d.filters, 0.f);
                if (d.off[1] >= 0) {
                    const float* bb = get(d.off[1], d.filters);
                    if (!bb) { fail(AA_ERR_INVALID, "dense bias outside the blob"); break; }
                    bias.assign(bb, bb + d.filters);
                }
                ++i;
            }
            if (i < n_layers && layers[i].op == AA_OP_SIGMOID) {
                s.sigmoid = 1;
                ++i;
            }
            if (i != n_layers) { fail(AA_ERR_UNSUPPORTED, "layers after the global pooling / dense"); break; }
            s.cout_pad = s.cout;
            if (!upload(s, wd.empty() ? nullptr : wd.data(), wd.size() * sizeof(float), bias)) break;
            if (wd.empty()) {  // no Dense: pool_dense reads a null weight pointer
                (void)hipFree(s.d_w);
                s.d_w = nullptr;
            }
            s.flops = 2.0 * C * (wd.empty() ? 0 : s.cout);
            s.bytes = (double)prec_bytes(precision) * H * W * C + 4.0 * s.cout;
            char nm[96];
            snprintf(nm, sizeof nm, "globalmax%s_%d_%d", wd.empty() ? "" : "_dense", C, s.cout);
            s.name = nm;
            m->st.push_back(s);
            m->L = s.cout;
            continue;
        }
        if (ly.op != AA_OP_CONV2D) { fail(AA_ERR_UNSUPPORTED, "expected Conv2D"); break; }
        Stage s;
        s.kh = ly.kh;
        s.kw = ly.kw;
        s.cin = C;
        s.cout = ly.filters;
        s.Hin = H;
        s.Win = W;
        s.Hc = H - ly.kh + 1;
        s.Wc = W - ly.kw + 1;
        s.is_first = m->st.empty();
        if (s.Hc <= 0 || s.Wc <= 0) { fail(AA_ERR_INVALID, "input smaller than the kernel"); break; }
        const int K = s.kh * s.kw * s.cin;
        const float* kern = get(ly.off[0], (int64_t)K * s.cout);
        if (!kern) { fail(AA_ERR_INVALID, "conv kernel outside the blob"); break; }
        std::vector<double> scale(s.cout, 1.0), shift(s.cout, 0.0);
        if (ly.off[1] >= 0) {
            const float* b = get(ly.off[1], s.cout);
            if (!b) { fail(AA_ERR_INVALID, "bias outside the blob"); break; }
            for (int c = 0; c < s.cout; ++c) shift[c] = b[c];
        }
        ++i;
        // absorb BN / activation / pool / head
        if (i < n_layers && layers[i].op == AA_OP_BATCHNORM) {
            const aa_layer& bn = layers[i];
            const float *g = get(bn.off[0], s.cout), *be = get(bn.off[1], s.cout), *mu = get(bn.off[2], s.cout),
                        *var = get(bn.off[3], s.cout);
            if (!g || !be || !mu || !var) { fail(AA_ERR_INVALID, "batchnorm params outside the blob"); break; }
            for (int c = 0; c < s.cout; ++c) {
                const double sc = (double)g[c] / std::sqrt((double)var[c] + (double)bn.eps);
                shift[c] = (shift[c] - mu[c]) * sc + be[c];
                scale[c] = sc;
            }
            ++i;
        }
        if (i < n_layers && (layers[i].op == AA_OP_LEAKYRELU || layers[i].op == AA_OP_RELU)) {
            s.act = layers[i].op == AA_OP_LEAKYRELU ? ACT_LEAKY : ACT_RELU;
            s.alpha = layers[i].alpha;
            if (s.act == ACT_LEAKY && s.alpha < 0.f) { fail(AA_ERR_UNSUPPORTED, "LeakyReLU with a negative slope"); break; }
            ++i;
        }
        if (i < n_layers && layers[i].op == AA_OP_MAXPOOL2D) {
            if (layers[i].kh <= 0 || layers[i].kw <= 0) { fail(AA_ERR_INVALID, "max-pool window"); break; }
            s.ph = layers[i].kh;
            s.pw = layers[i].kw;
            ++i;
        }
        s.pool = (s.ph == s.pw && (s.ph == 1 || s.ph == 3)) ? s.ph : 0;
        s.Hout = s.Hc / s.ph;
        s.Wout = s.Wc / s.pw;
        if (s.Hout <= 0 || s.Wout <= 0) { fail(AA_ERR_INVALID, "pool window larger than the conv output"); break; }
        const bool gpool = i < n_layers && layers[i].op == AA_OP_GLOBALMAXPOOL2D;
        const bool dense_next = gpool && i + 1 < n_layers && layers[i + 1].op == AA_OP_DENSE;
        // (the first stage reads the f32 model input: only ST_SMALL / ST_GENERIC do)
        if (!s.is_first && gpool && !dense_next && s.kh == 1 && s.kw == 1 && s.ph == 1 && s.pw == 1 &&
            s.cin % 32 == 0 && s.cout <= 1024) {
            // the reference family's head: 1x1 conv, global max, sigmoid
            s.kind = ST_HEAD;
            ++i;
            if (i < n_layers && layers[i].op == AA_OP_SIGMOID) {
                s.sigmoid = 1;
                ++i;
            }
            if (i != n_layers) { fail(AA_ERR_UNSUPPORTED, "layers after the 1x1 head"); break; }
        } else if (s.cin == 1 && s.kh == 3 && s.kw == 3 && s.cout == 32 && s.pool == 1) {
            s.kind = ST_SMALL;
        } else if (!s.is_first && s.pool && mfma_bn(precision, s.kh, s.kw, s.cin, s.pool)) {
            s.kind = ST_MFMA;
        } else if (precision == AA_PREC_BF16X3 && !s.is_first && s.cin >= 16) {
            s.kind = ST_GCONV;  // any other shape with a real contraction: the runtime-shaped MFMA kernel
        } else {
            s.kind = ST_GENERIC;
            if (precision == AA_PREC_FP8) {
                fail(AA_ERR_UNSUPPORTED, "no fp8 kernel for this conv shape (the f32 / bf16x3 / bf16 modes have one)");
                break;
            }
        }
        if (s.is_first) {
            s.has_mag = has_mag;
            s.mag_exp = mag_exp;
            if (has_mag && s.kind != ST_SMALL && s.kind != ST_GENERIC) {
                fail(AA_ERR_UNSUPPORTED, "MagTransform needs a C_in=1 first conv");
                break;
            }
        }
        int bn_tile = 32;
        if (s.kind == ST_MFMA) bn_tile = mfma_bn(precision, s.kh, s.kw, s.cin, s.pool);
        if (s.kind == ST_GCONV) {
            // [tap][cin_pad / 32][cout_pad][32 hi | 32 lo], BN folded (aa_gconv.h)
            s.cout_pad = (s.cout + 63) / 64 * 64;
            s.cin_pad = (s.cin + 31) / 32 * 32;
            const int ntap = s.kh * s.kw;
            std::vector<float> w_tco((size_t)ntap * s.cout * s.cin);
            for (int t = 0; t < ntap; ++t)
                for (int o = 0; o < s.cout; ++o)
                    for (int c = 0; c < s.cin; ++c)
                        w_tco[((size_t)t * s.cout + o) * s.cin + c] =
                            (float)(kern[((size_t)t * s.cin + c) * s.cout + o] * scale[o]);
            const std::vector<uint16_t> h = gconv_pack_x3(w_tco, ntap, s.cout, s.cin, s.cout_pad, s.cin_pad);
            std::vector<float> bias(s.cout_pad, 0.f);
            for (int o = 0; o < s.cout; ++o) bias[o] = (float)shift[o];
            if (!upload(s, h.data(), h.size() * 2, bias)) break;
            s.flops = 2.0 * s.Hc * s.Wc * K * s.cout;
            s.bytes = 4.0 * s.Hin * s.Win * s.cin + 4.0 * s.Hout * s.Wout * s.cout;
            char nm[96], pl[24] = "";
            if (s.ph > 1 || s.pw > 1) snprintf(pl, sizeof pl, s.ph == s.pw ? "_pool%d" : "_pool%dx%d", s.ph, s.pw);
            snprintf(nm, sizeof nm, "conv_gx3_%dx%d_%d_%d%s", s.kh, s.kw, s.cin, s.cout, pl);
            s.name = nm;
            if (s.ph > 1 || s.pw > 1) m->tmp_elems = std::max(m->tmp_elems, (size_t)s.Hc * s.Wc * s.cout);
            m->st.push_back(s);
            H = s.Hout;
            W = s.Wout;
            C = s.cout;
            continue;
        }
        s.wg = 0;
        if (precision == AA_PREC_BF16X3 && s.kind == ST_MFMA && wg_bn(s.kh, s.kw, s.cin, s.pool) > 0)
            wg_form(s.kh, s.cin, s.pool, &s.wg, &s.wg_npass);
        const bool rowmajor = s.kind == ST_SMALL || s.kind == ST_GENERIC;  // f32 [cout][K]
        s.cout_pad = rowmajor ? s.cout : (s.cout + bn_tile - 1) / bn_tile * bn_tile;
        // pack weights with the BN scale folded in: conv_small / generic
        // [cout][K] f32; MFMA stages tap-major with padded rows
        // [kh*KW + kw][cout_pad][cstr] (a block's per-tap slice is one
        // contiguous block, byte-identical to its LDS image) plus 1 KiB of
        // slack for the last slice's rounding; the 1x1 head [cout_pad][C_in]
        const bool bf = (precision == AA_PREC_BF16) && !rowmajor;
        const bool f8 = (precision == AA_PREC_FP8) && !rowmajor;
        // split-bf16: conv_x3 steps of hi/lo bf16 rows (packed below from the
        // compact f32 [tap][cout_pad][C_in] image); the head stays f32
        const bool sp = (precision == AA_PREC_BF16X3) && s.kind == ST_MFMA;
        const int wes = (bf || sp) ? 2 : f8 ? 1 : 4;
        const int cstr = s.kind == ST_MFMA ? (bf ? conv_cstr<bf16>(s.cin) : f8 ? conv_cstr<fp8>(s.cin)
                                              : sp ? s.cin : conv_cstr<float>(s.cin))
                                           : s.cin;
        const int ntap = s.kh * s.kw;
        const size_t slack = s.kind == ST_MFMA ? 1024 / wes : 0;
        std::vector<float> wpk(rowmajor ? (size_t)s.cout * K : (size_t)ntap * s.cout_pad * cstr + slack, 0.f);
        for (int o = 0; o < s.cout; ++o)
            for (int k = 0; k < K; ++k) {
                const double v = kern[(size_t)k * s.cout + o] * scale[o];
                if (rowmajor) {
                    wpk[(size_t)o * K + k] = (float)v;
                } else {
                    const int t = k / s.cin, c = k - t * s.cin;
                    wpk[((size_t)t * s.cout_pad + o) * cstr + c] = (float)v;
                }
            }
        // fp8: [bias | per-channel dequantisation scale], both cout_pad long
        std::vector<float> bias(f8 ? 2 * s.cout_pad : s.cout_pad, 0.f);
        for (int o = 0; o < s.cout; ++o) bias[o] = (float)shift[o];
        // split-bf16 stores hi + lo: twice the compact image's elements
        const size_t wbytes = (sp ? 2 * wpk.size() : wpk.size()) * wes;
        bool ok = true;
        if (f8) {
            // per output channel: the largest |w| maps to 240 (e4m3fn tops
            // out at 448), the kernel's epilogue multiplies by amax / 240.
            // conv stages: super-steps of four 32-channel chunks (chunk k =
            // tap k / (C_in/32), channels 32 (k % (C_in/32)) ..), each
            // [cout_pad][F8_BSTR] with chunk k % 4 at byte 32 (k % 4) of the
            // row (conv_mfma's K = 128 loop); the head keeps [cout_pad][cstr]
            const bool ss = s.kind == ST_MFMA && conv_k128<fp8>(s.cin);
            const int cpc = s.cin / 32, nch = ntap * cpc, nss = conv_nstep<fp8>(ntap, s.cin);
            std::vector<uint8_t> h(ss ? (size_t)nss * s.cout_pad * F8_BSTR + 1024 : wpk.size(), 0);
            for (int o = 0; o < s.cout_pad; ++o) {
                float amax = 0.f;
                for (int t = 0; t < ntap; ++t)
                    for (int c = 0; c < s.cin; ++c) amax = std::max(amax, std::fabs(wpk[((size_t)t * s.cout_pad + o) * cstr + c]));
                const float sc = amax > 0.f ? 240.f / amax : 1.f;
                bias[s.cout_pad + o] = 1.f / sc;
                if (ss) {
                    for (int k = 0; k < nch; ++k)
                        for (int c = 0; c < 32; ++c) {
                            const int t = k / cpc, cc = k % cpc;
                            h[((size_t)(k / 4) * s.cout_pad + o) * F8_BSTR + 32 * (k % 4) + c] =
                                f2fp8(wpk[((size_t)t * s.cout_pad + o) * cstr + 32 * cc + c] * sc);
                        }
                } else {
                    for (int t = 0; t < ntap; ++t)
                        for (int c = 0; c < s.cin; ++c) {
                            const size_t k = ((size_t)t * s.cout_pad + o) * cstr + c;
                            h[k] = f2fp8(wpk[k] * sc);
                        }
                }
            }
            ok = upload(s, h.data(), h.size(), bias);
        } else if (bf) {
            std::vector<uint16_t> h(wpk.size());
            for (size_t k = 0; k < wpk.size(); ++k) h[k] = f2bf(wpk[k]);
            ok = upload(s, h.data(), wbytes, bias);
        } else if (sp) {
            // conv_x3 steps (32-channel group g, tap t) in order s = g * ntap + t,
            // each [cout_pad][8 units of 8 bf16]: units 0-3 hi = rn_bf16(w) of
            // channels 32 g + 8 u .. + 7, units 4-7 lo = rn_bf16(w - hi), unit u
            // of row o stored in slot (u + o) & 7 (aa_conv_x3.h)
            std::vector<uint16_t> h(2 * wpk.size(), 0);
            const int ng = s.cin / 32;
            if (s.wg) {
                // conv_wg steps (group g, pass p, row kh, plane slot el) in order
                // ((g * npass + p) * kh + kh) * pps + el, each [cout_pad][8 units] as
                // above, holding the transformed weights v_e = sum_k G[e][k] w_k of
                // plane e = p * pps + el (w_kw = the folded kernel at (kh, kw);
                // F(2,3): v0 = w0, v1 = (w0 + w1 + w2) / 2, v2 = (w0 - w1 + w2) / 2,
                // v3 = w2), computed in double
                const int A = s.wg + 2, np = s.wg_npass, pps = A / np;
                h.assign((size_t)ng * s.kh * A * s.cout_pad * 64 * 2 + 1024, 0);
                for (int g = 0; g < ng; ++g)
                    for (int kh = 0; kh < s.kh; ++kh)
                        for (int o = 0; o < s.cout_pad; ++o)
                            for (int c = 0; c < 32; ++c) {
                                double w3[3];
                                for (int kw = 0; kw < 3; ++kw)
                                    w3[kw] = o < s.cout ? (double)kern[((size_t)(kh * 3 + kw) * s.cin + 32 * g + c) * s.cout + o] * scale[o] : 0.0;
                                for (int e = 0; e < A; ++e) {
                                    const double v = wg_g(s.wg, e, 0) * w3[0] + wg_g(s.wg, e, 1) * w3[1] + wg_g(s.wg, e, 2) * w3[2];
                                    const int p = e / pps, el = e % pps;
                                    const size_t row = ((size_t)(((g * np + p) * s.kh + kh) * pps + el) * s.cout_pad + o) * 64;
                                    const float w = (float)v;
                                    const uint16_t hi = f2bf(w);
                                    const int u = c / 8;
                                    h[row + ((u + o) & 7) * 8 + c % 8] = hi;
                                    h[row + ((u + 4 + o) & 7) * 8 + c % 8] = f2bf(w - bf2f(hi));
                                }
                            }
                ok = upload(s, h.data(), h.size() * 2, bias);
            } else {
            for (int g = 0; g < ng; ++g)
                for (int t = 0; t < ntap; ++t)
                    for (int o = 0; o < s.cout_pad; ++o) {
                        const size_t row = ((size_t)(g * ntap + t) * s.cout_pad + o) * 64;
                        for (int c = 0; c < 32; ++c) {
                            const float w = wpk[((size_t)t * s.cout_pad + o) * cstr + 32 * g + c];
                            const uint16_t hi = f2bf(w);
                            const int u = c / 8;
                            h[row + ((u + o) & 7) * 8 + c % 8] = hi;
                            h[row + ((u + 4 + o) & 7) * 8 + c % 8] = f2bf(w - bf2f(hi));
                        }
                    }
            ok = upload(s, h.data(), wbytes, bias);
            }
        } else {
            ok = upload(s, wpk.data(), wbytes, bias);
        }
        if (!ok) break;
        s.flops = 2.0 * s.Hc * s.Wc * K * s.cout;
        const double es = (double)prec_bytes(precision);
        s.bytes = (s.is_first ? 4.0 : es) * s.Hin * s.Win * s.cin +
                  (s.kind == ST_HEAD ? 4.0 * s.cout : es * s.Hout * s.Wout * s.cout);
        char nm[96], pl[24] = "";
        if (s.ph > 1 || s.pw > 1) snprintf(pl, sizeof pl, s.ph == s.pw ? "_pool%d" : "_pool%dx%d", s.ph, s.pw);
        snprintf(nm, sizeof nm, "%s%dx%d_%d_%d%s",
                 s.kind == ST_SMALL ? "conv_small_" : s.kind == ST_HEAD ? "head_" : s.kind == ST_GENERIC ? "conv_generic_" : "conv_",
                 s.kh, s.kw, s.cin, s.cout, pl);
        s.name = nm;
        m->st.push_back(s);
        H = s.Hout;
        W = s.Wout;
        C = s.cout;
        if (s.kind == ST_HEAD) m->L = s.cout;
    }
    if (rc == AA_OK && (m->st.empty() || (m->st.back().kind != ST_HEAD && m->st.back().kind != ST_POOLDENSE))) {
        set_error("aa_model_create: the model must end with GlobalMaxPool2D (after a 1x1 conv or before a Dense)");
        rc = AA_ERR_UNSUPPORTED;
    }
    if (rc != AA_OK) {
        free_model(m);
        return rc;
    }
    // fuse a C_in = 1 first conv (3x3 -> 32) into the following 3x3/32 pooled conv
    if (m->st.size() >= 2 && fusable_first(m->st[0], m->st[1])) {
        m->st[0].skipped = 1;
        m->st[1].fused_first = 1;
        m->st[1].flops += m->st[0].flops;
        // the fused pair reads the first conv's f32 input and writes the
        // second's output; the first conv's activations never reach HBM
        const double es1 = (double)prec_bytes(precision);
        m->st[1].bytes = 4.0 * m->st[0].Hin * m->st[0].Win * m->st[0].cin +
                         (m->st[1].bytes - es1 * m->st[1].Hin * m->st[1].Win * m->st[1].cin);
        m->st[1].name = m->st[0].name + "+" + m->st[1].name;
    }
    // split-bf16: a conv_x3 stage whose consumer is another conv_x3 stage
    // writes the grouped-split layout, and that consumer stages it by
    // global_load_lds alone (aa_conv_x3.h); heads / generic stages keep f32
    if (precision == AA_PREC_BF16X3) {
        for (size_t k = 0; k + 1 < m->st.size(); ++k) {
            Stage& a = m->st[k];
            Stage& b = m->st[k + 1];
            if (a.skipped || a.kind != ST_MFMA || b.kind != ST_MFMA || b.fused_first) continue;
            if (a.cout % 32 != 0 || b.cin != a.cout) continue;
            // a Winograd consumer transforms f32 values before it splits them: it
            // reads plain f32 (one 16-B load per 4 channels, not two 8-B loads and
            // a hi + lo sum); the split layout only pays for global_load_lds staging
            if (b.wg) continue;
            a.out_split = 1;
            b.in_split = 1;
        }
    }
    // split-bf16: the 1x3/128 -> 256 conv before a 1x1 head (<= 32 labels) and
    // the head in one kernel (aa_conv_tail.h); the conv's 13 x 20 x 256
    // activations never reach HBM.
    if (precision == AA_PREC_BF16X3 && m->st.size() >= 2) {
        Stage& h = m->st.back();
        Stage& c = m->st[m->st.size() - 2];
        if (h.kind == ST_HEAD && h.cout <= 32 && h.cout_pad == 32 && h.cin == 256 && c.kind == ST_MFMA && !c.skipped &&
            !c.fused_first && !c.wg && c.in_split && !c.out_split && c.kh == 1 && c.kw == 3 && c.cin == 128 &&
            c.cout == 256 && c.cout_pad == 256 && c.pool == 1 && c.ph == 1 && c.pw == 1) {
            // head weights f32 [cout_pad][256] -> per (wave w, label fragment lf,
            // hi / lo, lane l) 8 bf16: label 16 lf + (l & 15), k-slot e <-> channel
            // 32 w + (e < 4 ? 4 (l >> 4) + e : 16 + 4 (l >> 4) + e - 4)
            std::vector<float> hwf((size_t)h.cout_pad * h.cin);
            hipError_t e = hipMemcpy(hwf.data(), h.d_w, hwf.size() * 4, hipMemcpyDeviceToHost);
            std::vector<uint16_t> pk((size_t)TAIL_NW * 2 * 2 * 64 * 8, 0);
            for (int w = 0; w < TAIL_NW; ++w)
                for (int lf = 0; lf < 2; ++lf)
                    for (int l = 0; l < 64; ++l)
                        for (int k = 0; k < 8; ++k) {
                            const int lab = lf * 16 + (l & 15), qq = l >> 4;
                            const int co = 32 * w + (k < 4 ? 4 * qq + k : 16 + 4 * qq + k - 4);
                            const float v = lab < h.cout ? hwf[(size_t)lab * h.cin + co] : 0.f;
                            const uint16_t hi = f2bf(v);
                            pk[((((size_t)w * 2 + lf) * 2 + 0) * 64 + l) * 8 + k] = hi;
                            pk[((((size_t)w * 2 + lf) * 2 + 1) * 64 + l) * 8 + k] = f2bf(v - bf2f(hi));
                        }
            if (e == hipSuccess) e = hipMalloc(&h.d_tw, pk.size() * 2);
            if (e == hipSuccess) e = hipMemcpy(h.d_tw, pk.data(), pk.size() * 2, hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                set_error("aa_model_create: %s", hipGetErrorString(e));
                free_model(m);
                return AA_ERR_HIP;
            }
            c.skipped = 1;
            h.tail = 1;
            h.flops += c.flops;
            h.bytes = 4.0 * c.Hin * c.Win * c.cin + 4.0 * h.cout;
            h.name = c.name + "+" + h.name;
        }
    }
    // ping-pong activation buffers: stage s writes buffer s % 2
    for (size_t k = 0; k + 1 < m->st.size(); ++k) {
        const Stage& s = m->st[k];
        if (s.skipped || s.kind == ST_POOLDENSE) continue;
        const size_t e = (size_t)s.Hout * s.Wout * s.cout;
        m->act_elems[k % 2] = std::max(m->act_elems[k % 2], e);
    }
    if (!m->st.empty() && m->st.back().kind == ST_HEAD) {  // the head's partial maxima use its free buffer
        const Stage& h = m->st.back();
        const size_t es = prec_bytes(precision);
        const size_t parts = ((size_t)h.Hin * h.Win + 63) / 64;
        const size_t k = m->st.size() - 1;
        m->act_elems[k % 2] = std::max(m->act_elems[k % 2], (parts * h.cout_pad * sizeof(float) + es - 1) / es);
        if (h.tail) {  // the fused tail's per-tile maxima go to the skipped conv stage's buffer
            const Stage& c = m->st[k - 1];
            const size_t tiles = (size_t)((c.Hc + 12) / 13) * ((c.Wc + 4) / 5);
            m->act_elems[(k - 1) % 2] = std::max(m->act_elems[(k - 1) % 2], (tiles * 32 * sizeof(float) + es - 1) / es);
        }
    }
    *model = m;
    return AA_OK;
}

extern "C" int aa_model_destroy(void* model) {
    free_model(static_cast<Model*>(model));
    return AA_OK;
}

extern "C" int aa_model_n_outputs(const void* model) {
    return model ? static_cast<const Model*>(model)->L : -1;
}

extern "C" size_t aa_model_workspace_bytes(const void* model, int32_t max_batch) {
    if (!model || max_batch < 0) return 0;
    const Model* m = static_cast<const Model*>(model);
    const size_t es = prec_bytes(m->prec);
    return align_up(m->act_elems[0] * es * max_batch, 256) + align_up(m->act_elems[1] * es * max_batch, 256) +
           align_up(m->tmp_elems * 4 * max_batch, 256);
}

extern "C" int aa_model_set_input_f16(void* model, int32_t f16) {
    Model* m = static_cast<Model*>(model);
    AA_CHECK(m && (f16 == 0 || f16 == 1), AA_ERR_INVALID, "aa_model_set_input_f16: bad argument");
    AA_CHECK(!f16 || (m->st.size() >= 2 && m->st[1].fused_first), AA_ERR_UNSUPPORTED,
             "aa_model_set_input_f16: float16 input needs the fused first conv (3x3 C_in=1 -> 32 before a "
             "pooled 3x3/32 conv)");
    if (m->st.size() >= 2) m->st[1].lm_f16 = f16;
    return AA_OK;
}

extern "C" int aa_model_forward(void* model, const void* x, int32_t n, float* logits, float* probs,
                                void* workspace, size_t workspace_bytes, void* stream) {
    Model* m = static_cast<Model*>(model);
    AA_CHECK(m && x && logits, AA_ERR_INVALID, "aa_model_forward: null argument");
    if (n <= 0) return AA_OK;
    const size_t need = aa_model_workspace_bytes(m, n);
    AA_CHECK(workspace && workspace_bytes >= need, AA_ERR_WORKSPACE, "aa_model_forward: workspace %zu < %zu",
             workspace_bytes, need);
    const size_t es = prec_bytes(m->prec);
    char* buf[2] = {static_cast<char*>(workspace),
                    static_cast<char*>(workspace) + align_up(m->act_elems[0] * es * n, 256)};
    float* tmp = reinterpret_cast<float*>(buf[1] + align_up(m->act_elems[1] * es * n, 256));
    hipStream_t st = static_cast<hipStream_t>(stream);
    // launch grids carry the window index in blockIdx.z (at most 65,535):
    // larger batches run as consecutive chunks through the same workspace
    constexpr int32_t CHUNK = 32768;
    if (n > CHUNK) {
        const size_t in_bytes = (size_t)m->in_h * m->in_w * m->in_c *
                                (m->st.size() >= 2 && m->st[1].lm_f16 ? 2 : 4);
        for (int32_t c0 = 0; c0 < n; c0 += CHUNK) {
            const int32_t nc = std::min(CHUNK, n - c0);
            const int rc = aa_model_forward(model, static_cast<const char*>(x) + (size_t)c0 * in_bytes, nc,
                                            logits + (size_t)c0 * m->L, probs ? probs + (size_t)c0 * m->L : nullptr,
                                            workspace, workspace_bytes, stream);
            if (rc != AA_OK) return rc;
        }
        return AA_OK;
    }
    const void* in = x;
    for (size_t k = 0; k < m->st.size(); ++k) {
        Stage& s = m->st[k];
        if (s.skipped) continue;  // computed inside stage k + 1 (reads x directly)
        // (a fused tail writes its per-tile maxima into the skipped conv stage's
        // buffer: its own would be the one its input lives in)
        void* out = buf[(s.tail ? k - 1 : k) % 2];
        const Stage* first = (s.fused_first || s.tail) ? &m->st[k - 1] : nullptr;
        hipEvent_t e0;
        int rc = m->timer.begin((int)k, st, &e0);
        if (rc != AA_OK) return rc;
        rc = m->prec == AA_PREC_BF16     ? launch_stage<bf16>(*m, s, in, out, logits, probs, n, st, first, tmp)
             : m->prec == AA_PREC_FP8    ? launch_stage<fp8>(*m, s, in, out, logits, probs, n, st, first, tmp)
             : m->prec == AA_PREC_BF16X3 ? launch_stage<bf16x3>(*m, s, in, out, logits, probs, n, st, first, tmp)
                                         : launch_stage<float>(*m, s, in, out, logits, probs, n, st, first, tmp);
        if (rc != AA_OK) return rc;
        rc = m->timer.end((int)k, st, e0);
        if (rc != AA_OK) return rc;
        in = out;
    }
    return AA_OK;
}

extern "C" int aa_model_n_stages(const void* model) {
    return model ? (int)static_cast<const Model*>(model)->st.size() : -1;
}

extern "C" int aa_model_stage_info(const void* model, int32_t stage, char* name, int32_t name_len,
                                   double* flops_per_item, double* bytes_per_item) {
    const Model* m = static_cast<const Model*>(model);
    AA_CHECK(m && stage >= 0 && stage < (int)m->st.size(), AA_ERR_INVALID, "aa_model_stage_info: bad stage");
    const Stage& s = m->st[stage];
    if (name && name_len > 0) snprintf(name, name_len, "%s", s.name.c_str());
    if (flops_per_item) *flops_per_item = s.flops;
    if (bytes_per_item) *bytes_per_item = s.bytes;
    return AA_OK;
}

extern "C" int aa_model_set_timing(void* model, uint32_t stage_mask) {
    Model* m = static_cast<Model*>(model);
    AA_CHECK(m, AA_ERR_INVALID, "aa_model_set_timing: null model");
    m->timer.mask = stage_mask;
    return AA_OK;
}

extern "C" int aa_model_stage_time(void* model, int32_t stage, double* total_ms, int64_t* count) {
    Model* m = static_cast<Model*>(model);
    AA_CHECK(m && stage >= 0 && stage < (int)m->st.size(), AA_ERR_INVALID, "aa_model_stage_time: bad stage");
    return m->timer.collect(stage, total_ms, count);
}

extern "C" int aa_track_mean(const float* probs, int32_t n_models, int64_t model_stride, int32_t n_labels,
                             const int32_t* win_begin, const int32_t* win_count, int32_t n_tracks, float* out,
                             void* stream) {
    AA_CHECK(probs && win_begin && win_count && out, AA_ERR_INVALID, "aa_track_mean: null argument");
    AA_CHECK(n_models >= 1 && n_labels >= 1 && n_labels <= 1024, AA_ERR_INVALID, "aa_track_mean: bad sizes");
    if (n_tracks <= 0) return AA_OK;
    const int threads = (n_labels + 63) / 64 * 64;
    hipLaunchKernelGGL(track_mean, dim3(n_tracks), dim3(threads), 0, static_cast<hipStream_t>(stream), probs,
                       n_models, (long long)model_stride, n_labels, win_begin, win_count, out);
    AA_LAUNCH_CHECK();
    return AA_OK;
}
