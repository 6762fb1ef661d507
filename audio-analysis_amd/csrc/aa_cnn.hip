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
#include <cstring>
#include <string>
#include <vector>

namespace aa {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __bf16 bf16;

// ---- 8-element fragments and the MFMA step over one 32-deep K chunk -------
template <typename T>
struct Frag;
template <>
struct Frag<bf16> {
    bf16x8 v;
    __device__ __forceinline__ void load(const bf16* p) { v = *reinterpret_cast<const bf16x8*>(p); }
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
    TO* o = out + (size_t)(n * Hc * Wc + p) * COUT;
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
        if constexpr (sizeof(TO) == 2) {
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
template <typename T, int KH, int KW, int CIN, int WM, int WN, int MF, int NF, int POOL>
__global__ __launch_bounds__(256) void conv_mfma(const T* __restrict__ in, int Hin, int Win,
                                                 const T* __restrict__ wt, const float* __restrict__ bias,
                                                 T* __restrict__ out, int Hout, int Wout, int cout_store,
                                                 int TH, int TW, int tiles_w, int act, float alpha) {
    static_assert(WM * WN == 4, "4 waves");
    static_assert(CIN % 32 == 0, "C_in multiple of 32");
    constexpr int BN = WN * NF * 16;
    constexpr int VEC = 16 / sizeof(T);
    constexpr int CSTR = CIN + VEC;  // +16 B per pixel
    constexpr int KTOT = KH * KW * CIN;
    constexpr int ESTR = BN + 4;     // f32 epilogue row stride (conflict-free b32 writes)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* patch = reinterpret_cast<T*>(smem);

    const int n = blockIdx.z;
    const int th = blockIdx.x / tiles_w, tw = blockIdx.x - (blockIdx.x / tiles_w) * tiles_w;
    const int oh0 = th * TH, ow0 = tw * TW;
    const int PH = TH + KH - 1, PW = TW + KW - 1;

    // ---- stage the input patch ----
    {
        constexpr int VPP = CIN / VEC;  // 16-B vectors per pixel
        const int total = PH * PW * VPP;
        const T* src = in + (size_t)n * Hin * Win * CIN;
        for (int idx = threadIdx.x; idx < total; idx += 256) {
            const int pix = idx / VPP, cv = idx - pix * VPP;
            const int r = pix / PW, c = pix - r * PW;
            const int gh = oh0 + r, gw = ow0 + c;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (gh < Hin && gw < Win)
                v = *reinterpret_cast<const uint4*>(src + ((size_t)gh * Win + gw) * CIN + cv * VEC);
            *reinterpret_cast<uint4*>(patch + pix * CSTR + cv * VEC) = v;
        }
    }
    __syncthreads();

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave % WM, wn = wave / WM;
    const int q8 = 8 * (lane >> 4);
    const int TP = TH * TW;
    int abase[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        int p = (wm * MF + i) * 16 + (lane & 15);
        if (p >= TP) p = 0;  // padding rows: computed, never stored
        const int r = p / TW, c = p - (p / TW) * TW;
        abase[i] = (r * PW + c) * CSTR + q8;
    }
    const int nblk = blockIdx.y * BN + wn * NF * 16;
    const T* bptr[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) bptr[j] = wt + (size_t)(nblk + j * 16 + (lane & 15)) * KTOT + q8;

    f32x4 acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kh = 0; kh < KH; ++kh) {
#pragma unroll
        for (int kw = 0; kw < KW; ++kw) {
#pragma unroll
            for (int cc = 0; cc < CIN / 32; ++cc) {
                const int tap = (kh * PW + kw) * CSTR + cc * 32;
                const int koff = (kh * KW + kw) * CIN + cc * 32;
                Frag<T> b[NF];
#pragma unroll
                for (int j = 0; j < NF; ++j) b[j].load(bptr[j] + koff);
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    Frag<T> a;
                    a.load(patch + abase[i] + tap);
#pragma unroll
                    for (int j = 0; j < NF; ++j) acc[i][j] = mfma_chunk(a, b[j], acc[i][j]);
                }
            }
        }
    }
    __syncthreads();  // patch no longer needed: reuse LDS for the f32 tile

    float* E = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        const int prow = (wm * MF + i) * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            const int col = wn * NF * 16 + j * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (prow + r < TP) E[(prow + r) * ESTR + col] = acc[i][j][r];
        }
    }
    __syncthreads();

    const int PHo = TH / POOL, PWo = TW / POOL;
    const int oh0s = oh0 / POOL, ow0s = ow0 / POOL;
    const int items = PHo * PWo * BN;
    T* dst = out + (size_t)n * Hout * Wout * cout_store;
    for (int idx = threadIdx.x; idx < items; idx += 256) {
        const int col = idx % BN;
        const int q = idx / BN;
        const int pr = q / PWo, pc = q - (q / PWo) * PWo;
        const int gh = oh0s + pr, gw = ow0s + pc;
        const int ch = blockIdx.y * BN + col;
        if (gh >= Hout || gw >= Wout || ch >= cout_store) continue;
        float v = -INFINITY;
#pragma unroll
        for (int dy = 0; dy < POOL; ++dy)
#pragma unroll
            for (int dx = 0; dx < POOL; ++dx)
                v = fmaxf(v, E[((pr * POOL + dy) * TW + pc * POOL + dx) * ESTR + col]);
        v = apply_act(v + bias[ch], act, alpha);
        dst[((size_t)gh * Wout + gw) * cout_store + ch] = to_t<T>(v);
    }
}

// ---------------------------------------------------------------------------
// conv_head: 1x1 conv (C_in % 32 == 0, C_out <= 16*NF) + global max + sigmoid.
// One block per window; 4 waves along pixels, MF tiles each per chunk.
// ---------------------------------------------------------------------------
template <typename T, int CIN, int MF, int NF>
__global__ __launch_bounds__(256) void conv_head(const T* __restrict__ in, int HW,
                                                 const T* __restrict__ wt, const float* __restrict__ bias,
                                                 int L, int act, float alpha, int sigmoid,
                                                 float* __restrict__ logits, float* __restrict__ probs) {
    const int n = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q8 = 8 * (lane >> 4);
    const T* src = in + (size_t)n * HW * CIN;
    const T* bptr[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) bptr[j] = wt + (size_t)(j * 16 + (lane & 15)) * CIN + q8;
    float rmax[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) rmax[j] = -INFINITY;
    constexpr int CHUNK = 4 * MF * 16;
    for (int p0 = 0; p0 < HW; p0 += CHUNK) {
        f32x4 acc[MF][NF];
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        int arow[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int p = p0 + (wave * MF + i) * 16 + (lane & 15);
            arow[i] = (p < HW ? p : 0) * CIN + q8;
        }
#pragma unroll 2
        for (int k0 = 0; k0 < CIN; k0 += 32) {
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
    if (threadIdx.x < 16 * NF && (int)threadIdx.x < L) {
        const int c = threadIdx.x;
        float v = fmaxf(fmaxf(red[0][c], red[1][c]), fmaxf(red[2][c], red[3][c]));
        v = apply_act(v + bias[c], act, alpha);
        logits[(size_t)n * L + c] = v;
        if (probs) probs[(size_t)n * L + c] = sigmoid ? 1.f / (1.f + expf(-v)) : v;
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
    constexpr int U = 16;  // loads in flight; the adds stay in numpy's order
    float acc = 0.f;
    const int n = wc[t];
    const float* base = probs + (size_t)wb[t] * L + c;
    for (int w0 = 0; w0 < n; w0 += U) {
        float v[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[u][k] = base[min(k, n_models - 1) * model_stride + (size_t)min(w0 + u, n - 1) * L];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (w0 + u < n) {
                float m = 0.f;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < n_models) m = __fadd_rn(m, v[u][k]);
                for (int k = 4; k < n_models; ++k)
                    m = __fadd_rn(m, base[k * model_stride + (size_t)(w0 + u) * L]);
                acc = __fadd_rn(acc, __fdiv_rn(m, (float)n_models));
            }
        }
    }
    out[(size_t)t * L + c] = n > 0 ? __fdiv_rn(acc, (float)n) : NAN;
}

// ---------------------------------------------------------------------------
// host: planner, workspace, forward, timing
// ---------------------------------------------------------------------------
enum StageKind { ST_SMALL = 0, ST_MFMA = 1, ST_HEAD = 2 };

struct Stage {
    int kind = ST_MFMA;
    int kh = 1, kw = 1, cin = 0, cout = 0, cout_pad = 0;
    int pool = 1;
    int act = ACT_NONE;
    float alpha = 0.f;
    int has_mag = 0;
    float mag_exp = 1.f;
    int sigmoid = 0;
    int Hin = 0, Win = 0, Hc = 0, Wc = 0, Hout = 0, Wout = 0;
    int TH = 0, TW = 0;  // conv tile (ST_MFMA)
    void* d_w = nullptr;
    float* d_b = nullptr;
    double flops = 0, bytes = 0;  // algorithmic per window
    std::string name;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
};

struct Model {
    int prec = AA_PREC_BF16;
    int in_h = 0, in_w = 0, in_c = 0;
    int L = 0;
    std::vector<Stage> st;
    size_t act_elems[2] = {0, 0};  // per-window elements of the ping-pong buffers
    int timing = 0;
    std::vector<hipEvent_t> ev_pool;  // recycled timing events
};

// Tile configuration of each conv_mfma instantiation.
struct MfmaCfg {
    int kh, kw, cin, pool;
    int BN, TH, TW;
};
static const MfmaCfg kMfmaCfgs[] = {
    {3, 3, 32, 3, 32, 6, 48},   // conv2 + pool   : WM2 WN2 MF9 NF1
    {3, 3, 32, 1, 64, 6, 24},   // conv3          : WM1 WN4 MF9 NF1
    {3, 3, 64, 1, 64, 6, 24},   // conv4          : WM1 WN4 MF9 NF1
    {9, 3, 64, 3, 128, 3, 33},  // conv5 + pool   : WM1 WN4 MF7 NF2
    {1, 3, 128, 1, 128, 6, 24}, // conv6          : WM1 WN4 MF9 NF2
};

static const MfmaCfg* find_cfg(int kh, int kw, int cin, int pool) {
    for (const auto& c : kMfmaCfgs)
        if (c.kh == kh && c.kw == kw && c.cin == cin && c.pool == pool) return &c;
    return nullptr;
}

template <typename T, int KH, int KW, int CIN, int WM, int WN, int MF, int NF, int POOL>
static int launch_mfma(const Stage& s, const void* in, void* out, int n, hipStream_t st) {
    auto k = conv_mfma<T, KH, KW, CIN, WM, WN, MF, NF, POOL>;
    constexpr int BN = WN * NF * 16;
    constexpr int VEC = 16 / sizeof(T);
    const size_t patch = (size_t)(s.TH + KH - 1) * (s.TW + KW - 1) * (CIN + VEC) * sizeof(T);
    const size_t epi = (size_t)s.TH * s.TW * (BN + 4) * sizeof(float);
    const size_t lds = std::max(patch, epi);
    AA_CHECK(lds <= 160 * 1024, AA_ERR_UNSUPPORTED, "conv %s: %zu B LDS", s.name.c_str(), lds);
    static size_t attr = 0;
    if (lds > attr) {
        AA_HIP(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr = lds;
    }
    const int tiles_h = (s.Hout * POOL + s.TH - 1) / s.TH;
    const int tiles_w = (s.Wout * POOL + s.TW - 1) / s.TW;
    dim3 grid(tiles_h * tiles_w, s.cout_pad / BN, n);
    hipLaunchKernelGGL(k, grid, dim3(256), lds, st, (const T*)in, s.Hin, s.Win, (const T*)s.d_w, s.d_b,
                       (T*)out, s.Hout, s.Wout, s.cout, s.TH, s.TW, tiles_w, s.act, s.alpha);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

template <typename T>
static int launch_stage(const Model& m, const Stage& s, const void* in, void* out, float* logits,
                        float* probs, int n, hipStream_t st) {
    if (s.kind == ST_SMALL) {
        AA_CHECK(s.kh == 3 && s.kw == 3 && s.cout == 32 && s.cin == 1, AA_ERR_UNSUPPORTED,
                 "first conv %dx%d %d->%d unsupported", s.kh, s.kw, s.cin, s.cout);
        dim3 grid((s.Hc * s.Wc + 255) / 256, n);
        hipLaunchKernelGGL((conv_small<T, 3, 3, 32>), grid, dim3(256), 0, st, (const float*)in, s.Hin,
                           s.Win, (const float*)s.d_w, s.d_b, s.has_mag, s.mag_exp, (T*)out, s.Hc, s.Wc,
                           s.act, s.alpha);
        AA_LAUNCH_CHECK();
        return AA_OK;
    }
    if (s.kind == ST_HEAD) {
        AA_CHECK(s.cin == 256 && s.cout_pad == 32, AA_ERR_UNSUPPORTED, "head %d->%d unsupported", s.cin,
                 s.cout);
        hipLaunchKernelGGL((conv_head<T, 256, 4, 2>), dim3(n), dim3(256), 0, st, (const T*)in,
                           s.Hin * s.Win, (const T*)s.d_w, s.d_b, s.cout, s.act, s.alpha, s.sigmoid,
                           logits, probs);
        AA_LAUNCH_CHECK();
        return AA_OK;
    }
    if (s.kh == 3 && s.kw == 3 && s.cin == 32 && s.pool == 3)
        return launch_mfma<T, 3, 3, 32, 2, 2, 9, 1, 3>(s, in, out, n, st);
    if (s.kh == 3 && s.kw == 3 && s.cin == 32 && s.pool == 1)
        return launch_mfma<T, 3, 3, 32, 1, 4, 9, 1, 1>(s, in, out, n, st);
    if (s.kh == 3 && s.kw == 3 && s.cin == 64 && s.pool == 1)
        return launch_mfma<T, 3, 3, 64, 1, 4, 9, 1, 1>(s, in, out, n, st);
    if (s.kh == 9 && s.kw == 3 && s.cin == 64 && s.pool == 3)
        return launch_mfma<T, 9, 3, 64, 1, 4, 7, 2, 3>(s, in, out, n, st);
    if (s.kh == 1 && s.kw == 3 && s.cin == 128 && s.pool == 1)
        return launch_mfma<T, 1, 3, 128, 1, 4, 9, 2, 1>(s, in, out, n, st);
    set_error("conv %dx%d cin %d pool %d: no kernel instantiation", s.kh, s.kw, s.cin, s.pool);
    return AA_ERR_UNSUPPORTED;
}

static void free_model(Model* m) {
    if (!m) return;
    for (hipEvent_t e : m->ev_pool) (void)hipEventDestroy(e);
    for (auto& s : m->st) {
        (void)hipFree(s.d_w);
        (void)hipFree(s.d_b);
        for (auto& e : s.ev) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
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

}  // namespace aa

using namespace aa;

extern "C" int aa_model_create(const aa_layer* layers, int32_t n_layers, const float* blob, int64_t blob_len,
                               int32_t in_h, int32_t in_w, int32_t in_c, int32_t precision, void** model) {
    AA_CHECK(layers && blob && model && n_layers > 0, AA_ERR_INVALID, "aa_model_create: null argument");
    AA_CHECK(precision == AA_PREC_F32 || precision == AA_PREC_BF16, AA_ERR_INVALID,
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
            ++i;
        }
        if (i < n_layers && layers[i].op == AA_OP_MAXPOOL2D) {
            if (layers[i].kh != 3 || layers[i].kw != 3) { fail(AA_ERR_UNSUPPORTED, "only 3x3 max-pool is fused"); break; }
            s.pool = 3;
            ++i;
        }
        if (i < n_layers && layers[i].op == AA_OP_GLOBALMAXPOOL2D) {
            s.kind = ST_HEAD;
            ++i;
            if (i < n_layers && layers[i].op == AA_OP_SIGMOID) {
                s.sigmoid = 1;
                ++i;
            }
            if (i != n_layers || s.pool != 1 || s.kh != 1 || s.kw != 1) {
                fail(AA_ERR_UNSUPPORTED, "GlobalMaxPool2D must follow a final 1x1 conv");
                break;
            }
        } else if (s.cin <= 4) {
            s.kind = ST_SMALL;
        } else {
            s.kind = ST_MFMA;
        }
        s.Hout = s.pool > 1 ? s.Hc / s.pool : s.Hc;
        s.Wout = s.pool > 1 ? s.Wc / s.pool : s.Wc;
        if (s.kind == ST_SMALL) {
            s.has_mag = has_mag;
            s.mag_exp = mag_exp;
            if (s.pool != 1) { fail(AA_ERR_UNSUPPORTED, "pool after the first conv"); break; }
        } else if (has_mag && m->st.empty()) {
            fail(AA_ERR_UNSUPPORTED, "MagTransform needs a C_in=1 first conv");
            break;
        }
        int bn_tile = 32;
        if (s.kind == ST_MFMA) {
            const MfmaCfg* cfg = find_cfg(s.kh, s.kw, s.cin, s.pool);
            if (!cfg) { fail(AA_ERR_UNSUPPORTED, "no conv kernel for this shape"); break; }
            bn_tile = cfg->BN;
            s.TH = cfg->TH;
            s.TW = cfg->TW;
        }
        s.cout_pad = (s.kind == ST_SMALL) ? s.cout : (s.cout + bn_tile - 1) / bn_tile * bn_tile;
        // pack weights: HWIO -> [cout_pad][kh][kw][cin] with the BN scale folded in
        std::vector<float> wpk((size_t)s.cout_pad * K, 0.f);
        for (int o = 0; o < s.cout; ++o)
            for (int k = 0; k < K; ++k) wpk[(size_t)o * K + k] = (float)(kern[(size_t)k * s.cout + o] * scale[o]);
        std::vector<float> bias(s.cout_pad, 0.f);
        for (int o = 0; o < s.cout; ++o) bias[o] = (float)shift[o];
        const bool bf = (precision == AA_PREC_BF16) && s.kind != ST_SMALL;
        const size_t wbytes = wpk.size() * (bf ? 2 : 4);
        hipError_t e = hipMalloc(&s.d_w, wbytes);
        if (e == hipSuccess) {
            if (bf) {
                std::vector<uint16_t> h(wpk.size());
                for (size_t k = 0; k < wpk.size(); ++k) h[k] = f2bf(wpk[k]);
                e = hipMemcpy(s.d_w, h.data(), wbytes, hipMemcpyHostToDevice);
            } else {
                e = hipMemcpy(s.d_w, wpk.data(), wbytes, hipMemcpyHostToDevice);
            }
        }
        if (e == hipSuccess) e = hipMalloc((void**)&s.d_b, sizeof(float) * s.cout_pad);
        if (e == hipSuccess) e = hipMemcpy(s.d_b, bias.data(), sizeof(float) * s.cout_pad, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            m->st.push_back(s);
            fail(AA_ERR_HIP, hipGetErrorString(e));
            break;
        }
        s.flops = 2.0 * s.Hc * s.Wc * K * s.cout;
        const double es = (precision == AA_PREC_BF16) ? 2.0 : 4.0;
        s.bytes = (s.kind == ST_SMALL ? 4.0 : es) * s.Hin * s.Win * s.cin +
                  (s.kind == ST_HEAD ? 4.0 * s.cout : es * s.Hout * s.Wout * s.cout);
        char nm[96];
        snprintf(nm, sizeof nm, "%s%dx%d_%d_%d%s", s.kind == ST_SMALL ? "conv_small_" : s.kind == ST_HEAD ? "head_" : "conv_",
                 s.kh, s.kw, s.cin, s.cout, s.pool > 1 ? "_pool3" : "");
        s.name = nm;
        m->st.push_back(s);
        H = s.Hout;
        W = s.Wout;
        C = s.cout;
        if (s.kind == ST_HEAD) m->L = s.cout;
    }
    if (rc == AA_OK && (m->st.empty() || m->st.back().kind != ST_HEAD)) {
        set_error("aa_model_create: the model must end with conv1x1 + GlobalMaxPool2D");
        rc = AA_ERR_UNSUPPORTED;
    }
    if (rc != AA_OK) {
        free_model(m);
        return rc;
    }
    // ping-pong activation buffers: stage s writes buffer s % 2
    for (size_t k = 0; k + 1 < m->st.size(); ++k) {
        const Stage& s = m->st[k];
        const size_t e = (size_t)s.Hout * s.Wout * s.cout;
        m->act_elems[k % 2] = std::max(m->act_elems[k % 2], e);
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
    const size_t es = m->prec == AA_PREC_BF16 ? 2 : 4;
    return align_up(m->act_elems[0] * es * max_batch, 256) + align_up(m->act_elems[1] * es * max_batch, 256);
}

extern "C" int aa_model_forward(void* model, const float* x, int32_t n, float* logits, float* probs,
                                void* workspace, size_t workspace_bytes, void* stream) {
    Model* m = static_cast<Model*>(model);
    AA_CHECK(m && x && logits, AA_ERR_INVALID, "aa_model_forward: null argument");
    if (n <= 0) return AA_OK;
    const size_t need = aa_model_workspace_bytes(m, n);
    AA_CHECK(workspace && workspace_bytes >= need, AA_ERR_WORKSPACE, "aa_model_forward: workspace %zu < %zu",
             workspace_bytes, need);
    const size_t es = m->prec == AA_PREC_BF16 ? 2 : 4;
    char* buf[2] = {static_cast<char*>(workspace),
                    static_cast<char*>(workspace) + align_up(m->act_elems[0] * es * n, 256)};
    hipStream_t st = static_cast<hipStream_t>(stream);
    const void* in = x;
    for (size_t k = 0; k < m->st.size(); ++k) {
        Stage& s = m->st[k];
        void* out = buf[k % 2];
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (m->timing) {
            for (hipEvent_t* e : {&e0, &e1}) {
                if (!m->ev_pool.empty()) {
                    *e = m->ev_pool.back();
                    m->ev_pool.pop_back();
                } else {
                    AA_HIP(hipEventCreate(e));
                }
            }
            AA_HIP(hipEventRecord(e0, st));
        }
        int rc = (m->prec == AA_PREC_BF16) ? launch_stage<bf16>(*m, s, in, out, logits, probs, n, st)
                                           : launch_stage<float>(*m, s, in, out, logits, probs, n, st);
        if (rc != AA_OK) return rc;
        if (m->timing) {
            AA_HIP(hipEventRecord(e1, st));
            s.ev.emplace_back(e0, e1);
        }
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

extern "C" int aa_model_set_timing(void* model, int32_t enable) {
    Model* m = static_cast<Model*>(model);
    AA_CHECK(m, AA_ERR_INVALID, "aa_model_set_timing: null model");
    m->timing = enable;
    return AA_OK;
}

extern "C" int aa_model_stage_time(void* model, int32_t stage, double* total_ms, int64_t* count) {
    Model* m = static_cast<Model*>(model);
    AA_CHECK(m && stage >= 0 && stage < (int)m->st.size(), AA_ERR_INVALID, "aa_model_stage_time: bad stage");
    Stage& s = m->st[stage];
    double tot = 0;
    for (auto& e : s.ev) {
        AA_HIP(hipEventSynchronize(e.second));
        float ms = 0;
        AA_HIP(hipEventElapsedTime(&ms, e.first, e.second));
        tot += ms;
        m->ev_pool.push_back(e.first);
        m->ev_pool.push_back(e.second);
    }
    if (total_ms) *total_ms = tot;
    if (count) *count = (int64_t)s.ev.size();
    s.ev.clear();
    return AA_OK;
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
