// CNN graphs: Keras Functional models that are not one conv chain --
// residual Add, squeeze-and-excite Multiply, DepthwiseConv2D, strided and
// "same"-padded convs, global average pooling -- i.e. the layer set of the
// EfficientNet route of classify() (reference src/identify_tracks.py:539-540;
// the CLI's default models /models/*/audioModel.keras, src/analyse.py:414-418,
// are whatever Keras graph the AI-Model release holds).
//
// Execution: the node list (include/aa.h aa_node, topological order) runs
// node by node over a batch of windows, each node's output an NHWC f32
// tensor in a workspace region reused once its last consumer has run
// (first-fit over the freed intervals).  Kernels:
//   conv (C_in >= 16, split-bf16)  gconv_x3 (aa_gconv.h, MFMA)
//   conv (C_in < 16, or f32 mode)  gconv_f32 (exact f32 FMA chains)
//   depthwise conv                 gdwconv (one lane per output pixel and 4 channels)
//   max / avg pool, global pools   gpool2d / ggpool
//   add, broadcast multiply        gbinary
//   affine / activation / pow      gaffine / gpow
//   dense                          gdense
// every one with its activation fused.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>

#include "aa_common.h"
#include "aa_gconv.h"

namespace aa {

// depthwise conv: one lane per (output pixel, 4 channels) when C % 4 == 0
// (float4 taps and weights), else per (pixel, channel)
template <int V>
__global__ __launch_bounds__(256) void gdwconv(const float* __restrict__ in, const float* __restrict__ w,
                                               const float* __restrict__ bias, float* __restrict__ out, int Hin,
                                               int Win, int C, int Hout, int Wout, int kh, int kw, int sh, int sw,
                                               int pt, int pl, int act, float alpha) {
    typedef __attribute__((ext_vector_type(V))) float fv;
    const int CV = C / V;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const int n = blockIdx.y;
    if (i >= (size_t)Hout * Wout * CV) return;
    const int c = (int)(i % CV) * V;
    const int P = (int)(i / CV);
    const int oy = P / Wout, ox = P - (P / Wout) * Wout;
    const float* img = in + (size_t)n * Hin * Win * C;
    fv acc;
    for (int e = 0; e < V; ++e) acc[e] = bias ? bias[c + e] : 0.f;
    for (int ky = 0; ky < kh; ++ky) {
        const int iy = oy * sh - pt + ky;
        if (iy < 0 || iy >= Hin) continue;
        for (int kx = 0; kx < kw; ++kx) {
            const int ix = ox * sw - pl + kx;
            if (ix < 0 || ix >= Win) continue;
            const fv wv = *reinterpret_cast<const fv*>(w + (ky * kw + kx) * C + c);
            const fv xv = *reinterpret_cast<const fv*>(img + ((size_t)iy * Win + ix) * C + c);
            for (int e = 0; e < V; ++e) acc[e] = fmaf(wv[e], xv[e], acc[e]);
        }
    }
    fv o;
    for (int e = 0; e < V; ++e) o[e] = gact(acc[e], act, alpha);
    *reinterpret_cast<fv*>(out + (size_t)n * Hout * Wout * C + (size_t)P * C + c) = o;
}

// global pool over H x W: a block per (window, 64 channels), 16 pixel
// stripes of 64 lanes (coalesced channel reads), each stripe summed in pixel
// order, the stripes combined by a fixed tree (deterministic: the same sums
// whatever the batch; gdwconv_pool reproduces this order exactly)
constexpr int GP_STRIPES = 16;
__device__ __forceinline__ float gpool_combine(float (*part)[64], int lane, int avg) {
    float v[GP_STRIPES];
#pragma unroll
    for (int i = 0; i < GP_STRIPES; ++i) v[i] = part[i][lane];
#pragma unroll
    for (int w = GP_STRIPES / 2; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) v[i] = avg ? v[i] + v[i + w] : fmaxf(v[i], v[i + w]);
    return v[0];
}

__global__ __launch_bounds__(64 * GP_STRIPES) void ggpool(const float* __restrict__ in, float* __restrict__ out,
                                                          int HW, int C, int avg, int act, float alpha) {
    __shared__ float part[GP_STRIPES][64];
    const int lane = threadIdx.x & 63, s = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    const int n = blockIdx.y;
    float m = avg ? 0.f : -INFINITY;
    if (c < C) {
        const float* p = in + (size_t)n * HW * C + c;
        for (int i = s; i < HW; i += GP_STRIPES) m = avg ? m + p[(size_t)i * C] : fmaxf(m, p[(size_t)i * C]);
    }
    part[s][lane] = m;
    __syncthreads();
    if (s == 0 && c < C) {
        float r = gpool_combine(part, lane, avg);
        if (avg) r = r / (float)HW;
        out[(size_t)n * C + c] = gact(r, act, alpha);
    }
}

// depthwise conv fused with the global average pool that reads it (the
// squeeze of squeeze-and-excite): ggpool's block shape, each lane computing
// its stripe's output pixels of one channel (exactly gdwconv's chain), storing
// them and summing them in ggpool's order -- the map and the pooled vector
// equal the unfused pair bit for bit.
__global__ __launch_bounds__(64 * GP_STRIPES) void gdwconv_pool(
    const float* __restrict__ in, const float* __restrict__ w, const float* __restrict__ bias, float* __restrict__ out,
    float* __restrict__ pooled, int Hin, int Win, int C, int Hout, int Wout, int kh, int kw, int sh, int sw, int pt,
    int pl, int act, float alpha, int pact, float palpha) {
    __shared__ float part[GP_STRIPES][64];
    const int lane = threadIdx.x & 63, s = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    const int n = blockIdx.y;
    const int HW = Hout * Wout;
    float m = 0.f;
    if (c < C) {
        const float* img = in + (size_t)n * Hin * Win * C + c;
        float* o = out + (size_t)n * HW * C + c;
        const float b = bias ? bias[c] : 0.f;
        for (int P = s; P < HW; P += GP_STRIPES) {
            const int oy = P / Wout, ox = P - (P / Wout) * Wout;
            float acc = b;
            for (int ky = 0; ky < kh; ++ky) {
                const int iy = oy * sh - pt + ky;
                if (iy < 0 || iy >= Hin) continue;
                for (int kx = 0; kx < kw; ++kx) {
                    const int ix = ox * sw - pl + kx;
                    if (ix < 0 || ix >= Win) continue;
                    acc = fmaf(w[(ky * kw + kx) * C + c], img[((size_t)iy * Win + ix) * C], acc);
                }
            }
            const float y = gact(acc, act, alpha);
            o[(size_t)P * C] = y;
            m += y;
        }
    }
    part[s][lane] = m;
    __syncthreads();
    if (s == 0 && c < C) pooled[(size_t)n * C + c] = gact(gpool_combine(part, lane, 1) / (float)HW, pact, palpha);
}

constexpr int GP4_STRIPES = 32;
// The same two kernels 4 channels per lane (C % 4 == 0): thread t of a block
// owns channel quad t % Q of the block's 4 Q channels and stripe t / Q
// (GP4_STRIPES stripes: twice the scalar kernels', for twice the waves on
// the small maps of a network's last stages).  Per channel the sum order is
// fixed (pixel order within a stripe, a fixed combine tree), the same in the
// pool and in the fused dwconv + pool: float4 loads give 16 lanes 256
// contiguous bytes per pixel.
// Stripe s sums the pixels p = s, s + GP4_STRIPES, ... of the map in row-major
// order (the order gdwconv_pool4 produces its pixels in, so a fused depthwise
// conv + pool and the two separate nodes give the same bits; every stripe
// gets HW / GP4_STRIPES pixels within one, whatever the map's width).
template <int Q>
__global__ __launch_bounds__(Q * GP4_STRIPES) void ggpool4(const float* __restrict__ in, float* __restrict__ out,
                                                         int H, int W, int C, int avg, int act, float alpha) {
    __shared__ float part[GP4_STRIPES][4 * Q];
    const int cq = threadIdx.x % Q, s = threadIdx.x / Q;
    const int c = blockIdx.x * 4 * Q + 4 * cq;
    const int n = blockIdx.y;
    const int HW = H * W;
    float4 m = avg ? make_float4(0.f, 0.f, 0.f, 0.f) : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    if (c < C) {
        const float* p = in + (size_t)n * HW * C + c;
        for (int px = s; px < HW; px += GP4_STRIPES) {
            const float4 v = *reinterpret_cast<const float4*>(p + (size_t)px * C);
            if (avg) { m.x += v.x; m.y += v.y; m.z += v.z; m.w += v.w; }
            else { m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w); }
        }
    }
    part[s][4 * cq] = m.x; part[s][4 * cq + 1] = m.y; part[s][4 * cq + 2] = m.z; part[s][4 * cq + 3] = m.w;
    __syncthreads();
    const int k = threadIdx.x;  // one channel of the block per thread
    if (k < 4 * Q && blockIdx.x * 4 * Q + k < C) {
        float v[GP4_STRIPES];
#pragma unroll
        for (int i = 0; i < GP4_STRIPES; ++i) v[i] = part[i][k];
#pragma unroll
        for (int w = GP4_STRIPES / 2; w >= 1; w >>= 1)
#pragma unroll
            for (int i = 0; i < w; ++i) v[i] = avg ? v[i] + v[i + w] : fmaxf(v[i], v[i + w]);
        float r = v[0];
        if (avg) r = r / (float)HW;
        out[(size_t)n * C + blockIdx.x * 4 * Q + k] = gact(r, act, alpha);
    }
}

// KS = 3: a 3x3 kernel, the taps unrolled and their weights held in
// registers for every pixel; KS = 0: any kernel, weights re-read per tap.
// Thread = (channel quad, stripe s): it computes the pixels p = s, s +
// GP4_STRIPES, ... in row-major order, so every stripe has HW / GP4_STRIPES
// pixels within one.  S = 1 or 2 (KS = 3, both strides S): R of the thread's
// pixels at a time, their 9 R taps loaded unconditionally from clamped
// addresses and zeroed by a value select (R = 1 by default: the fewest
// registers).  Round 5's column walk with a sliding 3 x 3 window was
// latency-bound -- one round trip per output row, 0.69-0.86 of the wave
// cycles parked on loads, its padding zeros read through flat loads from
// scratch, and on a 33-column map stripe 0 walked two columns while the
// others walked one (profiles/r05/pmc_ev2_top.txt).
template <int Q, int KS, int S = 0, int R = 1>
__global__ __launch_bounds__(Q * GP4_STRIPES) void gdwconv_pool4(
    const float* __restrict__ in, const float* __restrict__ w, const float* __restrict__ bias, float* __restrict__ out,
    float* __restrict__ pooled, int Hin, int Win, int C, int Hout, int Wout, int kh, int kw, int sh, int sw, int pt,
    int pl, int act, float alpha, int pact, float palpha) {
    static_assert(S == 0 || KS == 3, "chunked rows: 3x3 kernels");
    __shared__ float part[GP4_STRIPES][4 * Q];
    const int cq = threadIdx.x % Q, s = threadIdx.x / Q;
    const int c = blockIdx.x * 4 * Q + 4 * cq;
    const int n = blockIdx.y;
    const int HW = Hout * Wout;
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < C) with_act(act, [&](auto actc) {
        constexpr int AV = decltype(actc)::value;
        const float* img = in + (size_t)n * Hin * Win * C + c;
        float* o = out + (size_t)n * HW * C + c;
        const float4 b = bias ? *reinterpret_cast<const float4*>(bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        constexpr int NW = KS ? KS * KS : 1;
        float4 wr[NW];  // the taps' weights of this lane's channels, held for every pixel
        if constexpr (KS > 0) {
#pragma unroll
            for (int t = 0; t < NW; ++t) wr[t] = *reinterpret_cast<const float4*>(w + t * C + c);
        }
        const int KH = KS ? KS : kh, KW = KS ? KS : kw;
        auto fma4 = [](float4& acc, const float4& wv, const float4& x) {
            acc.x = fmaf(wv.x, x.x, acc.x);
            acc.y = fmaf(wv.y, x.y, acc.y);
            acc.z = fmaf(wv.z, x.z, acc.z);
            acc.w = fmaf(wv.w, x.w, acc.w);
        };
        auto emit = [&](int oy, int ox, const float4& acc) {
            // no contraction of the activation's last product into the pool's
            // add: the pool sums the stored (rounded) outputs, as the unfused
            // ggpool4 does (with the activation a constant the compiler would
            // otherwise fuse swish's v * logistic(v) into an FMA with m)
#pragma clang fp contract(off)
            const float4 y = make_float4(gact(acc.x, AV, alpha), gact(acc.y, AV, alpha), gact(acc.z, AV, alpha),
                                         gact(acc.w, AV, alpha));
            *reinterpret_cast<float4*>(o + ((size_t)oy * Wout + ox) * C) = y;
            m.x += y.x; m.y += y.y; m.z += y.z; m.w += y.w;
        };
        if constexpr (S > 0) {
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            const float* imgw = in + (size_t)n * Hin * Win * C;
            for (int p0 = s; p0 < HW; p0 += GP4_STRIPES * R) {
                float4 x[R][9];
                int oyv[R], oxv[R];
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    const int p = p0 + u * GP4_STRIPES;
                    const bool pv = p < HW;
                    oyv[u] = pv ? p / Wout : 0;
                    oxv[u] = pv ? p - oyv[u] * Wout : 0;
#pragma unroll
                    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                        for (int kx = 0; kx < 3; ++kx) {
                            // a load from the clamped pixel, zeroed outside the image: a
                            // value select (a `cond ? *p : z` becomes a select of
                            // pointers -- flat loads, z in scratch)
                            const int iy = oyv[u] * S - pt + ky, ix = oxv[u] * S - pl + kx;
                            const int iyc = min(max(iy, 0), Hin - 1), ixc = min(max(ix, 0), Win - 1);
                            // (a 32-bit offset from the window's base: one VGPR per address)
                            const float4 t = *reinterpret_cast<const float4*>(
                                imgw + (uint32_t)((iyc * Win + ixc) * C + c));
                            x[u][ky * 3 + kx] = (pv && iy == iyc && ix == ixc) ? t : z;
                        }
                }
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (p0 + u * GP4_STRIPES >= HW) break;
                    float4 acc = b;
                    // padding taps add +0 * w: the same sum unless w is inf / nan
#pragma unroll
                    for (int t = 0; t < 9; ++t) fma4(acc, wr[t], x[u][t]);
                    emit(oyv[u], oxv[u], acc);
                }
            }
        } else {
            for (int p = s; p < HW; p += GP4_STRIPES) {
                const int oy = p / Wout, ox = p - oy * Wout;
                float4 acc = b;
                // (KS > 0: constant trip counts, unrolled by the compiler)
                for (int ky = 0; ky < KH; ++ky) {
                    const int iy = oy * sh - pt + ky;
                    if (iy < 0 || iy >= Hin) continue;
                    for (int kx = 0; kx < KW; ++kx) {
                        const int ix = ox * sw - pl + kx;
                        if (ix < 0 || ix >= Win) continue;
                        float4 wv;
                        if constexpr (KS > 0) wv = wr[ky * KS + kx];
                        else wv = *reinterpret_cast<const float4*>(w + (ky * kw + kx) * C + c);
                        fma4(acc, wv, *reinterpret_cast<const float4*>(img + ((size_t)iy * Win + ix) * C));
                    }
                }
                emit(oy, ox, acc);
            }
        }
    });
    part[s][4 * cq] = m.x; part[s][4 * cq + 1] = m.y; part[s][4 * cq + 2] = m.z; part[s][4 * cq + 3] = m.w;
    __syncthreads();
    const int k = threadIdx.x;
    if (k < 4 * Q && blockIdx.x * 4 * Q + k < C) {
        float v[GP4_STRIPES];
#pragma unroll
        for (int i = 0; i < GP4_STRIPES; ++i) v[i] = part[i][k];
#pragma unroll
        for (int ww = GP4_STRIPES / 2; ww >= 1; ww >>= 1)
#pragma unroll
            for (int i = 0; i < ww; ++i) v[i] = v[i] + v[i + ww];
        pooled[(size_t)n * C + blockIdx.x * 4 * Q + k] = gact(v[0] / (float)HW, pact, palpha);
    }
}

// [n][K] x W[Cout][K] + bias: one wave per (window, output), lanes striding
// K by float4s, a fixed-order butterfly reduction (deterministic).  Dense
// layers, and 1x1 convs on 1x1 maps (the squeeze-and-excite reduce / expand).
__global__ __launch_bounds__(256) void gmatvec(const float* __restrict__ in, const float* __restrict__ w,
                                               const float* __restrict__ bias, float* __restrict__ out, int K,
                                               int Cout, int act, float alpha) {
    const int lane = threadIdx.x & 63;
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int n = blockIdx.y;
    if (o >= Cout) return;  // wave-uniform
    const float* x = in + (size_t)n * K;
    const float* wr = w + (size_t)o * K;
    float acc = 0.f;
    if ((K & 3) == 0) {
#pragma unroll 4
        for (int k = 4 * lane; k < K; k += 256) {
            const float4 a = *reinterpret_cast<const float4*>(x + k);
            const float4 b = *reinterpret_cast<const float4*>(wr + k);
            acc = fmaf(a.x, b.x, acc);
            acc = fmaf(a.y, b.y, acc);
            acc = fmaf(a.z, b.z, acc);
            acc = fmaf(a.w, b.w, acc);
        }
    } else {
        for (int k = lane; k < K; k += 64) acc = fmaf(x[k], wr[k], acc);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
        if (bias) acc += bias[o];
        out[(size_t)n * Cout + o] = gact(acc, act, alpha);
    }
}

// a (+|*) b; b_bcast: b is [n][C] broadcast over the pixels
__global__ __launch_bounds__(256) void gbinary(const float* __restrict__ a, const float* __restrict__ b,
                                               float* __restrict__ out, size_t per_win, int C, int mul,
                                               int b_bcast, int act, float alpha) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const int n = blockIdx.y;
    if (i >= per_win) return;
    const size_t o = (size_t)n * per_win + i;
    const float y = b_bcast ? b[(size_t)n * C + (int)(i % C)] : b[o];
    out[o] = gact(mul ? a[o] * y : a[o] + y, act, alpha);
}

__global__ __launch_bounds__(256) void gaffine(const float* __restrict__ in, const float* __restrict__ scale,
                                               const float* __restrict__ shift, float* __restrict__ out,
                                               size_t total, int C, int act, float alpha) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int c = (int)(i % C);
    float v = in[i];
    if (scale) v = fmaf(v, scale[c], shift ? shift[c] : 0.f);
    else if (shift) v += shift[c];
    out[i] = gact(v, act, alpha);
}

__global__ __launch_bounds__(256) void gpow(const float* __restrict__ in, float* __restrict__ out, size_t total,
                                            float e) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < total) out[i] = powf(in[i], e);
}

// [n][K] x W[K][Cout] + bias for short K: one thread per (window, output),
// lanes along the outputs (coalesced weight rows), the K products summed in
// order
__global__ __launch_bounds__(256) void gmatvec_t(const float* __restrict__ in, const float* __restrict__ w,
                                                 const float* __restrict__ bias, float* __restrict__ out, int K,
                                                 int Cout, int act, float alpha) {
    const int o = blockIdx.x * 256 + threadIdx.x;
    const int n = blockIdx.y;
    if (o >= Cout) return;
    const float* x = in + (size_t)n * K;
    float acc = 0.f;
    // 16 products per round: all 32 loads issued (clamped indices, no
    // branches between them) before the round's FMAs -- one memory round trip
    // per 16 products instead of per 8; the same ordered chain
    for (int k0 = 0; k0 < K; k0 += 16) {
        float xv[16], wv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int k = min(k0 + u, K - 1);
            xv[u] = x[k];
            wv[u] = w[(size_t)k * Cout + o];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (k0 + u < K) acc = fmaf(xv[u], wv[u], acc);
    }
    if (bias) acc += bias[o];
    out[(size_t)n * Cout + o] = gact(acc, act, alpha);
}

__global__ __launch_bounds__(256) void gfinal(const float* __restrict__ x, float* __restrict__ logits,
                                              float* __restrict__ probs, size_t total, int sigmoid) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const float v = x[i];
    logits[i] = v;
    if (probs) probs[i] = sigmoid ? 1.f / (1.f + expf(-v)) : v;
}

struct GNode {
    aa_node d;
    int H = 0, W = 0, C = 0;  // output shape
    int mfma = 0;             // conv on gconv_x3t
    int bn = 64;              // its tile's output channels (16, 32, 64)
    int split = 1, cslice = 0;  // pointwise conv on a small map: K split into `split` slices of cslice chunks
    ConvGeom g{};
    int cout_pad = 0;
    void* d_w = nullptr;
    float* d_b = nullptr;
    float* d_b2 = nullptr;    // affine shift
    float* d_ws = nullptr;    // f32 stem: weights [C_out / 32][K][32] for the scalar path (gconv_f32_s)
    size_t off = 0;           // workspace offset (f32 elements per window)
    // fusions (graph_build): a skipped node launches nothing; a conv may read
    // a squeeze-and-excite scale [n][Cin] (the Multiply it replaces) and add a
    // residual map (the Add it replaces) in its epilogue
    bool skip = false;        // fused into a consumer: no launch, no buffer
    bool nolaunch = false;    // written by its producer's launch (a pool fused into a dwconv)
    int scale_src = -2, res_src = -2;
    int pool_into = -2;       // dwconv: the global average pool node it also writes
    int matvec = 0;           // 1x1 conv on a 1x1 map, or Dense: gmatvec on W[Cout][K]
    int last_use = 0;
    std::string name;
    double flops = 0, bytes = 0;
};

struct Graph {
    int prec = AA_PREC_BF16X3;
    int in_h = 0, in_w = 0, in_c = 0;
    std::vector<GNode> nodes;
    size_t per_win = 0;  // workspace f32 elements per window
    size_t part_off = 0; // split-K partial sums (per window, after the node buffers)
    int L = 0;
    int sigmoid_out = 0;
    // HIP events around node launches (aa_graph_set_timing / aa_graph_time_stage):
    // time_stage -1 every node, >= 0 that node only, -2 none
    int time_stage = -2;
    StageTimer timer;
    // the forward's launches captured into HIP graphs, one per (input,
    // batch, workspace, outputs, stream): a graph model issues one launch per
    // node (~180 for an EfficientNetV2-B0), which from the host costs about
    // as much as the kernels take on the device; a replay is one launch
    struct Captured {
        const float* x;
        int n;
        void* ws;
        float* logits;
        float* probs;
        hipStream_t st;
        hipGraphExec_t exec;
        hipEvent_t done;  // recorded after every launch of exec: it may still run when evicted
    };
    std::vector<Captured> captured;
    std::vector<Captured> seen;  // keys met once (captured the second time: a caller
                                 // that allocates its outputs per call never pays a capture)
    std::mutex cap_mu;
};

constexpr size_t AA_GRAPH_CAPTURES = 16;  // captured forwards kept per graph

// an instantiated forward that may still be executing from its last launch:
// wait for that launch before the executable goes
static void release_captured(Graph::Captured& c) {
    if (c.done) {
        (void)hipEventSynchronize(c.done);
        (void)hipEventDestroy(c.done);
    }
    if (c.exec) (void)hipGraphExecDestroy(c.exec);
    c.done = nullptr;
    c.exec = nullptr;
}

static void free_graph(Graph* g) {
    if (!g) return;
    for (auto& c : g->captured) release_captured(c);
    g->timer.release();
    for (auto& nd : g->nodes) {
        (void)hipFree(nd.d_w);
        (void)hipFree(nd.d_b);
        (void)hipFree(nd.d_b2);
        (void)hipFree(nd.d_ws);
    }
    delete g;
}

static int gupload(void** dst, const void* src, size_t bytes) {
    if (!bytes) return AA_OK;
    AA_HIP(hipMalloc(dst, bytes));
    AA_HIP(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
    return AA_OK;
}

static const char* gop_name(int op) {
    switch (op) {
        case AA_G_CONV: return "conv";
        case AA_G_DWCONV: return "dwconv";
        case AA_G_MAXPOOL: return "maxpool";
        case AA_G_AVGPOOL: return "avgpool";
        case AA_G_GMAXPOOL: return "gmaxpool";
        case AA_G_GAVGPOOL: return "gavgpool";
        case AA_G_ADD: return "add";
        case AA_G_MUL: return "mul";
        case AA_G_AFFINE: return "affine";
        case AA_G_DENSE: return "dense";
        case AA_G_POW: return "pow";
        default: return "?";
    }
}

// Fusions on the built node list (bit-identical to the unfused graph: the
// fused kernel computes the same f32 products and sums in the same order):
// * Multiply(x [H][W][C], s [1][1][C]) whose only consumer is an MFMA conv:
//   the conv scales its input channels while staging (squeeze-and-excite);
// * Add(conv, r) where the conv has no activation and no other consumer and r
//   is computed before the conv: the conv adds r in its epilogue and applies
//   the add's activation (the residual of an inverted-bottleneck block).
static void graph_fuse(Graph* G) {
    const int n = (int)G->nodes.size();
    std::vector<int> uses(n, 0);
    for (const GNode& N : G->nodes)
        for (int k : {N.d.in0, N.d.in1})
            if (k >= 0) ++uses[k];
    auto redirect = [&](int from, int to) {
        for (GNode& N : G->nodes) {
            if (N.d.in0 == from) N.d.in0 = to;
            if (N.d.in1 == from) N.d.in1 = to;
        }
    };
    for (int i = 0; i < n - 1; ++i) {
        GNode& M = G->nodes[i];
        if (M.d.op != AA_G_MUL || M.d.act != AA_GACT_NONE || uses[i] != 1 || M.d.in1 < 0) continue;
        const GNode& S = G->nodes[M.d.in1];
        if (!(S.H == 1 && S.W == 1 && (M.H != 1 || M.W != 1))) continue;
        for (int j = i + 1; j < n; ++j) {
            GNode& K = G->nodes[j];
            if (K.d.in0 != i && K.d.in1 != i) continue;
            if (K.d.op == AA_G_CONV && K.mfma && K.d.in0 == i && K.scale_src == -2) {
                K.d.in0 = M.d.in0;
                K.scale_src = M.d.in1;
                M.skip = true;
            }
            break;
        }
    }
    for (int i = 0; i < n - 1; ++i) {
        GNode& A = G->nodes[i];
        if (A.d.op != AA_G_ADD || A.d.in1 < 0) continue;
        for (int side = 0; side < 2; ++side) {
            const int x = side ? A.d.in1 : A.d.in0, r = side ? A.d.in0 : A.d.in1;
            if (x < 0) continue;
            GNode& X = G->nodes[x];
            if (X.d.op != AA_G_CONV || !X.mfma || X.skip || X.d.act != AA_GACT_NONE || uses[x] != 1 ||
                X.res_src != -2 || r >= x)
                continue;
            const bool same = r < 0 ? (G->in_h == X.H && G->in_w == X.W && G->in_c == X.C)
                                    : (G->nodes[r].H == X.H && G->nodes[r].W == X.W && G->nodes[r].C == X.C);
            if (!same || r < 0) continue;  // the graph input is not a workspace buffer
            X.res_src = r;
            X.d.act = A.d.act;
            X.d.alpha = A.d.alpha;
            X.bytes += 4.0 * X.H * X.W * X.C;
            X.name += "+add";
            A.skip = true;
            redirect(i, x);
            break;
        }
    }
    for (int i = 0; i + 1 < n; ++i) {
        GNode& D = G->nodes[i];
        GNode& P = G->nodes[i + 1];
        if (D.d.op == AA_G_DWCONV && P.d.op == AA_G_GAVGPOOL && P.d.in0 == i && i + 1 != n - 1) {
            D.pool_into = i + 1;
            P.nolaunch = true;
            D.name += "+gap";
        }
    }
    for (GNode& N : G->nodes) {
        if (N.scale_src >= 0) N.name += "+se";
        if (N.nolaunch) {
            N.name += "(fused)";
            N.flops = N.bytes = 0;
        }
        if (N.skip) {
            N.name += "(fused)";
            N.flops = N.bytes = 0;
        }
    }
}

// a pointwise conv over >= 384 channels on a small map (<= kSplitHW pixels
// per window) is a short grid of long K loops: its K is split over blocks
constexpr int kSplitHW = 128;

static int graph_build(Graph* G, const aa_node* nodes, int n_nodes, const float* blob, int64_t blob_len) {
    auto get = [&](int64_t off, int64_t n) -> const float* {
        if (off < 0 || n < 0 || off + n > blob_len) return nullptr;
        return blob + off;
    };
    G->nodes.resize(n_nodes);
    for (int i = 0; i < n_nodes; ++i) {
        GNode& N = G->nodes[i];
        N.d = nodes[i];
        const aa_node& d = N.d;
        AA_CHECK(d.in0 >= -1 && d.in0 < i && d.in1 >= -1 && d.in1 < i, AA_ERR_INVALID,
                 "aa_graph_create: node %d reads a later node", i);
        AA_CHECK(d.act >= AA_GACT_NONE && d.act <= AA_GACT_SWISH, AA_ERR_INVALID, "node %d: activation %d", i, d.act);
        auto shape = [&](int k, int& H, int& W, int& C) {
            if (k < 0) { H = G->in_h; W = G->in_w; C = G->in_c; }
            else { H = G->nodes[k].H; W = G->nodes[k].W; C = G->nodes[k].C; }
        };
        int H, W, C;
        shape(d.in0, H, W, C);
        const bool windowed = d.op == AA_G_CONV || d.op == AA_G_DWCONV || d.op == AA_G_MAXPOOL || d.op == AA_G_AVGPOOL;
        if (windowed) {
            AA_CHECK(d.kh >= 1 && d.kw >= 1 && d.sh >= 1 && d.sw >= 1 && d.pt >= 0 && d.pb >= 0 && d.pl >= 0 &&
                         d.pr >= 0, AA_ERR_INVALID, "node %d: window / strides / pads", i);
            N.H = (H + d.pt + d.pb - d.kh) / d.sh + 1;
            N.W = (W + d.pl + d.pr - d.kw) / d.sw + 1;
            AA_CHECK(H + d.pt + d.pb >= d.kh && W + d.pl + d.pr >= d.kw, AA_ERR_INVALID,
                     "node %d: input %dx%d smaller than the window", i, H, W);
        }
        char nm[96];
        switch (d.op) {
            case AA_G_CONV: {
                AA_CHECK(d.filters >= 1, AA_ERR_INVALID, "node %d: filters", i);
                N.C = d.filters;
                const int K = d.kh * d.kw * C;
                const float* k = get(d.off[0], (int64_t)K * d.filters);
                AA_CHECK(k, AA_ERR_INVALID, "node %d: conv kernel outside the blob", i);
                const float* b = d.off[1] >= 0 ? get(d.off[1], d.filters) : nullptr;
                AA_CHECK(d.off[1] < 0 || b, AA_ERR_INVALID, "node %d: bias outside the blob", i);
                N.g = ConvGeom{H, W, C, N.H, N.W, N.C, d.kh, d.kw, d.sh, d.sw, d.pt, d.pl, (C + 31) / 32 * 32};
                // a 1x1 conv on a 1x1 map is a matrix-vector product per window
                // (squeeze-and-excite): exact f32 on gmatvec, not a 64-pixel MFMA tile
                N.matvec = H == 1 && W == 1 && d.kh == 1 && d.kw == 1 && d.pt == 0 && d.pl == 0;
                N.mfma = G->prec == AA_PREC_BF16X3 && C >= 16 && !N.matvec;
                const int ntap = d.kh * d.kw;
                int rc;
                const bool pointwise = ntap == 1 && d.sh == 1 && d.sw == 1 && d.pt == 0 && d.pl == 0;
                if (N.mfma) {
                    N.bn = gconv_bn(N.C);
                    N.cout_pad = (N.C + N.bn - 1) / N.bn * N.bn;
                    std::vector<float> w_tco((size_t)ntap * N.C * C);
                    for (int t = 0; t < ntap; ++t)
                        for (int o = 0; o < N.C; ++o)
                            for (int c = 0; c < C; ++c) w_tco[((size_t)t * N.C + o) * C + c] = k[((size_t)t * C + c) * N.C + o];
                    const std::vector<uint16_t> h = gconv_pack_x3(w_tco, ntap, N.C, C, N.cout_pad, N.g.cin_pad);
                    if ((rc = gupload(&N.d_w, h.data(), h.size() * 2)) != AA_OK) return rc;
                    std::vector<float> bias(N.cout_pad, 0.f);
                    for (int o = 0; o < N.C; ++o) bias[o] = b ? b[o] : 0.f;
                    if ((rc = gupload((void**)&N.d_b, bias.data(), bias.size() * 4)) != AA_OK) return rc;
                } else {
                    // [Cout][K]; a matrix-vector product with K <= 64 keeps the
                    // Keras [K][Cout] order (gmatvec_t: one thread per output)
                    if (N.matvec && K <= 64) N.matvec = 2;
                    std::vector<float> w_ohwc((size_t)N.C * K);
                    for (int o = 0; o < N.C; ++o)
                        for (int kk = 0; kk < K; ++kk) w_ohwc[(size_t)o * K + kk] = k[(size_t)kk * N.C + o];
                    if ((rc = N.matvec == 2 ? gupload(&N.d_w, k, (size_t)K * N.C * 4)
                                            : gupload(&N.d_w, w_ohwc.data(), w_ohwc.size() * 4)) != AA_OK)
                        return rc;
                    if (d.kh == 3 && d.kw == 3 && C == 3) {  // the scalar-path stem layout
                        const int ng = (N.C + 31) / 32;
                        std::vector<float> wsl((size_t)ng * K * 32, 0.f);
                        for (int o = 0; o < N.C; ++o)
                            for (int kk = 0; kk < K; ++kk)
                                wsl[((size_t)(o / 32) * K + kk) * 32 + o % 32] = k[(size_t)kk * N.C + o];
                        if ((rc = gupload((void**)&N.d_ws, wsl.data(), wsl.size() * 4)) != AA_OK) return rc;
                    }
                    std::vector<float> bias(N.C, 0.f);
                    for (int o = 0; o < N.C; ++o) bias[o] = b ? b[o] : 0.f;
                    if ((rc = gupload((void**)&N.d_b, bias.data(), bias.size() * 4)) != AA_OK) return rc;
                }
                N.flops = 2.0 * N.H * N.W * K * N.C;
                N.bytes = 4.0 * (H * W * C + N.H * N.W * N.C);
                // split K over blocks on small maps (shape-only choice: the
                // sums do not depend on n)
                if (N.mfma && pointwise && N.H * N.W <= kSplitHW) {
                    const int ncc = N.g.cin_pad / 32;
                    for (int cs : {6, 7, 4, 5, 8, 9})
                        if (ncc >= 12 && ncc % cs == 0) {
                            N.split = ncc / cs;
                            N.cslice = cs;
                            break;
                        }
                }
                snprintf(nm, sizeof nm, "%s_%dx%d_s%d_%d_%d", N.mfma ? "conv_gx3" : N.matvec ? "matvec" : "conv_gf32",
                         d.kh, d.kw, d.sh, C, N.C);
                break;
            }
            case AA_G_DWCONV: {
                N.C = C;
                const float* k = get(d.off[0], (int64_t)d.kh * d.kw * C);
                AA_CHECK(k, AA_ERR_INVALID, "node %d: depthwise kernel outside the blob", i);
                const float* b = d.off[1] >= 0 ? get(d.off[1], C) : nullptr;
                AA_CHECK(d.off[1] < 0 || b, AA_ERR_INVALID, "node %d: bias outside the blob", i);
                int rc;
                if ((rc = gupload(&N.d_w, k, (size_t)d.kh * d.kw * C * 4)) != AA_OK) return rc;
                if (b && (rc = gupload((void**)&N.d_b, b, (size_t)C * 4)) != AA_OK) return rc;
                N.flops = 2.0 * N.H * N.W * d.kh * d.kw * C;
                N.bytes = 4.0 * (H * W * C + N.H * N.W * N.C);
                snprintf(nm, sizeof nm, "dwconv_%dx%d_s%d_%d", d.kh, d.kw, d.sh, C);
                break;
            }
            case AA_G_MAXPOOL:
            case AA_G_AVGPOOL:
                N.C = C;
                N.bytes = 4.0 * (H * W * C + N.H * N.W * N.C);
                snprintf(nm, sizeof nm, "%s_%dx%d_s%d_%d", gop_name(d.op), d.kh, d.kw, d.sh, C);
                break;
            case AA_G_GMAXPOOL:
            case AA_G_GAVGPOOL:
                N.H = N.W = 1;
                N.C = C;
                N.bytes = 4.0 * (H * W * C + C);
                snprintf(nm, sizeof nm, "%s_%d", gop_name(d.op), C);
                break;
            case AA_G_ADD:
            case AA_G_MUL: {
                int H1, W1, C1;
                shape(d.in1, H1, W1, C1);
                const bool same = H1 == H && W1 == W && C1 == C;
                const bool bc = d.op == AA_G_MUL && H1 == 1 && W1 == 1 && C1 == C;
                AA_CHECK(same || bc, AA_ERR_UNSUPPORTED, "node %d: %s of %dx%dx%d and %dx%dx%d", i, gop_name(d.op), H,
                         W, C, H1, W1, C1);
                N.H = H; N.W = W; N.C = C;
                N.bytes = 4.0 * (2 * H * W * C + H * W * C);
                snprintf(nm, sizeof nm, "%s_%d", gop_name(d.op), C);
                break;
            }
            case AA_G_AFFINE: {
                N.H = H; N.W = W; N.C = C;
                int rc;
                if (d.off[0] >= 0) {
                    const float* sc = get(d.off[0], C);
                    AA_CHECK(sc, AA_ERR_INVALID, "node %d: scale outside the blob", i);
                    if ((rc = gupload((void**)&N.d_b, sc, (size_t)C * 4)) != AA_OK) return rc;
                }
                if (d.off[1] >= 0) {
                    const float* sh = get(d.off[1], C);
                    AA_CHECK(sh, AA_ERR_INVALID, "node %d: shift outside the blob", i);
                    if ((rc = gupload((void**)&N.d_b2, sh, (size_t)C * 4)) != AA_OK) return rc;
                }
                N.bytes = 8.0 * H * W * C;
                snprintf(nm, sizeof nm, "affine_%d", C);
                break;
            }
            case AA_G_POW:
                N.H = H; N.W = W; N.C = C;
                N.bytes = 8.0 * H * W * C;
                snprintf(nm, sizeof nm, "pow_%d", C);
                break;
            case AA_G_DENSE: {
                AA_CHECK(d.filters >= 1, AA_ERR_INVALID, "node %d: units", i);
                const int K = H * W * C;
                const float* k = get(d.off[0], (int64_t)K * d.filters);
                AA_CHECK(k, AA_ERR_INVALID, "node %d: dense kernel outside the blob", i);
                const float* b = d.off[1] >= 0 ? get(d.off[1], d.filters) : nullptr;
                AA_CHECK(d.off[1] < 0 || b, AA_ERR_INVALID, "node %d: bias outside the blob", i);
                int rc;
                std::vector<float> w_ok((size_t)K * d.filters);  // [Cout][K] for gmatvec
                for (int kk = 0; kk < K; ++kk)
                    for (int o = 0; o < d.filters; ++o) w_ok[(size_t)o * K + kk] = k[(size_t)kk * d.filters + o];
                if ((rc = gupload(&N.d_w, w_ok.data(), w_ok.size() * 4)) != AA_OK) return rc;
                if (b && (rc = gupload((void**)&N.d_b, b, (size_t)d.filters * 4)) != AA_OK) return rc;
                N.matvec = 1;
                N.H = N.W = 1;
                N.C = d.filters;
                N.flops = 2.0 * K * d.filters;
                N.bytes = 4.0 * (K + (double)K * d.filters + d.filters);
                snprintf(nm, sizeof nm, "dense_%d_%d", K, d.filters);
                break;
            }
            default:
                AA_CHECK(false, AA_ERR_UNSUPPORTED, "node %d: op %d", i, d.op);
        }
        AA_CHECK(N.H >= 1 && N.W >= 1 && N.C >= 1, AA_ERR_INVALID, "node %d: empty output", i);
        N.name = nm;
    }
    const int last = n_nodes - 1;
    if (getenv("AA_GRAPH_NOFUSE") == nullptr) graph_fuse(G);
    // liveness: a node's buffer is free after its last consumer; first fit
    auto inputs = [&](const GNode& N) {
        return std::array<int, 4>{N.d.in0, N.d.in1, N.scale_src, N.res_src};
    };
    for (int i = 0; i < n_nodes; ++i) G->nodes[i].last_use = i;
    for (int i = 0; i < n_nodes; ++i) {
        if (G->nodes[i].skip || G->nodes[i].nolaunch) continue;
        for (int k : inputs(G->nodes[i]))
            if (k >= 0) G->nodes[k].last_use = std::max(G->nodes[k].last_use, i);
    }
    G->nodes[last].last_use = n_nodes;  // the output survives the forward
    std::vector<std::pair<size_t, size_t>> live;  // [begin, end) of buffers in use
    size_t peak = 0;
    std::vector<std::vector<int>> frees(n_nodes + 1);
    // per-window sizes rounded up to 16 floats: every buffer starts 64-B
    // aligned, so the float4 loads / stores of the kernels never straddle
    auto node_sz = [&](int k) { return align_up((size_t)G->nodes[k].H * G->nodes[k].W * G->nodes[k].C, 16); };
    auto alloc = [&](int k) {
        const size_t sz = node_sz(k);
        std::sort(live.begin(), live.end());
        size_t at = 0;
        for (auto& iv : live) {
            if (iv.first >= at + sz) break;
            at = std::max(at, iv.second);
        }
        G->nodes[k].off = at;
        peak = std::max(peak, at + sz);
        live.emplace_back(at, at + sz);
        return at;
    };
    for (int i = 0; i < n_nodes; ++i) {
        GNode& N = G->nodes[i];
        if (N.skip || N.nolaunch) continue;  // (a nolaunch node is allocated with its producer)
        const size_t sz = node_sz(i);
        const size_t at = alloc(i);
        if (N.pool_into >= 0) alloc(N.pool_into);
        // release the inputs whose last use is this node
        for (int k : inputs(N)) {
            if (k < 0 || G->nodes[k].last_use != i) continue;
            auto it = std::find(live.begin(), live.end(), std::make_pair(G->nodes[k].off, G->nodes[k].off + node_sz(k)));
            if (it != live.end()) live.erase(it);
        }
        // a node nobody reads (a dangling branch) frees itself
        if (N.last_use == i && i != last) {
            auto it = std::find(live.begin(), live.end(), std::make_pair(at, at + sz));
            if (it != live.end()) live.erase(it);
        }
    }
    G->part_off = (peak + 63) / 64 * 64;
    size_t part = 0;
    for (const GNode& N : G->nodes)
        if (N.split > 1 && !N.skip) part = std::max(part, (size_t)N.split * N.H * N.W * N.C);
    G->per_win = G->part_off + (part + 63) / 64 * 64;
    const GNode& O = G->nodes[last];
    G->L = O.H * O.W * O.C;
    G->sigmoid_out = O.d.act == AA_GACT_SIGMOID;
    return AA_OK;
}

// Tile and kernel choices of the graph's convs, fixed from in-pipeline A/B
// runs (rounds 4-5; the rejected alternatives are no longer built):
//  * 64 x 128 gconv_x3t tiles for short-K convs with C_out a multiple of 128,
//    1x1 and larger kernels (42.3k -> 43.2k audio-s/s on the EfficientNetV2
//    graph; 3x3 32->128 160 -> 147 us, profiles/r04/graph_ab_xcd.txt);
//    128 x 64 tiles measured slower;
//  * KC <= 2 chunks per K step (KC = 4 halves the blocks per CU);
//  * two K steps in flight in the one-chunk 64 x 64 launches over >= 8 chunks
//    (the 672 -> 112 project convs 46 -> 42 us; 3 steps and 64 / 128 x 224 /
//    192 / 112 pointwise tiles slower, profiles/r05/graph_ab_pw.txt);
//  * the depthwise conv + pool at 8 channel quads per 256-thread block and one
//    pixel's taps per load batch (dwconv stages 526 -> 363 us against round
//    5's column walk; 2 / 3 pixels 390 / 436 us, profiles/r05/graph_ab_dw.txt);
//  * XCD-aware block order (stage sum 3016 -> 2923 us, graph_ab_xcd.txt);
//  * gconv_x3p (patch-staged) for kernels > 1x1 at C_out <= 16 on 256-pixel
//    tiles (3x3/32->16 212 -> 149 us); 128-pixel tiles and the stride-1
//    patch + weight-ring kernel at 64 channels measured slower.
constexpr int kGxKcMax = 2;

static int graph_run_node(const Graph& G, const GNode& N, const float* x, float* ws, int n, hipStream_t st) {
    const aa_node& d = N.d;
    auto buf = [&](int k) -> const float* {
        return k < 0 ? x : ws + G.nodes[k].off * (size_t)n;
    };
    float* out = ws + N.off * (size_t)n;
    const float* a = buf(d.in0);
    int Hin, Win, Cin;
    if (d.in0 < 0) { Hin = G.in_h; Win = G.in_w; Cin = G.in_c; }
    else { Hin = G.nodes[d.in0].H; Win = G.nodes[d.in0].W; Cin = G.nodes[d.in0].C; }
    // the output node's sigmoid is applied by gfinal (logits before it)
    const bool last = &N == &G.nodes.back();
    const int act = last && G.sigmoid_out ? AA_GACT_NONE : d.act;
    const size_t per = (size_t)N.H * N.W * N.C;
    switch (d.op) {
        case AA_G_CONV:
            if (N.mfma) {
                ConvGeom g = N.g;
                int nz = n, scale_hw = 0;
                if (d.kh == 1 && d.kw == 1 && d.sh == 1 && d.sw == 1 && d.pt == 0 && d.pl == 0) {
                    // pointwise: the n windows' pixels are one [1][n H W] image
                    // (NHWC is [n][H][W][C] either way), so small maps fill whole
                    // tiles; a squeeze-and-excite scale is looked up per pixel's window
                    g.Hin = g.Hout = 1;
                    g.Win = g.Wout = N.H * N.W * n;
                    nz = 1;
                    scale_hw = N.H * N.W;
                }
                constexpr int xo = 1;  // XCD-aware block order (aa_gconv.h xcd_order)
                const float* scl = N.scale_src >= 0 ? buf(N.scale_src) : nullptr;
                const float* res = N.res_src >= 0 ? buf(N.res_src) : nullptr;
                const int HWo = g.Hout * g.Wout;
                // kernels larger than 1x1 with C_out <= 16: the patch-staged
                // kernel when its patch fits 64 KiB (two blocks per CU at least).
                // (Measured on the EfficientNetV2 graph: 3x3/32->16 212 -> 149
                // us; at 64 channels per block it lost -- 3x3/32->128 161 ->
                // 178, 3x3/2 16->64 97 -> 176 us -- its per-tap B loads from L2
                // stall the short tap loop: gconv_x3t keeps those.)
                int BM = 0, TW = 0;
                if (d.kh * d.kw > 1 && N.bn == 16) {
                    BM = 256;
                    TW = 16;
                    const int TH = BM / TW;
                    // every patch pixel staged (GX_P_STG items per thread) and the
                    // patch within 64 KiB; otherwise gconv_x3t
                    if (!gconv_x3p_fits((TH - 1) * d.sh + d.kh, (TW - 1) * d.sw + d.kw)) BM = 0;
                }
                if (BM) {
                    const int TH = BM / TW;
                    const int tiles_w = (N.W + TW - 1) / TW, tiles_h = (N.H + TH - 1) / TH;
                    const size_t lds = (size_t)((TH - 1) * d.sh + d.kh) * ((TW - 1) * d.sw + d.kw) * GX_ROW * 4;
                    const dim3 grid((unsigned)(tiles_w * tiles_h), N.cout_pad / N.bn, n);
                    if (N.bn == 16)
                        hipLaunchKernelGGL((gconv_x3p<4, 1, 4, 1, 16>), grid, dim3(256), lds, st, a,
                                           (const uint16_t*)N.d_w, N.d_b, out, g, N.cout_pad, act, d.alpha, TW, tiles_w,
                                           scl, res, xo);
                    else if (N.bn == 32)
                        hipLaunchKernelGGL((gconv_x3p<4, 1, 2, 2>), grid, dim3(256), lds, st, a, (const uint16_t*)N.d_w,
                                           N.d_b, out, g, N.cout_pad, act, d.alpha, TW, tiles_w, scl, res, xo);
                    else
                        hipLaunchKernelGGL((gconv_x3p<2, 2, 2, 2>), grid, dim3(256), lds, st, a, (const uint16_t*)N.d_w,
                                           N.d_b, out, g, N.cout_pad, act, d.alpha, TW, tiles_w, scl, res, xo);
                } else {
                    // gconv_x3t (64 x 64 by default)
#define AA_X3T(GRID, WM_, WN_, MF_, NF_, KC_, PD_, CS_, PART_)                                                     \
    hipLaunchKernelGGL((gconv_x3t<WM_, WN_, MF_, NF_, KC_, PD_>), GRID, dim3(256), 0, st, a, (const uint16_t*)N.d_w, \
                       N.d_b, out, g, N.cout_pad, act, d.alpha, scl, res, scale_hw, CS_, PART_, xo)
                    if (N.bn == 16)
                        AA_X3T(dim3((HWo + 255) / 256, N.cout_pad / 16, nz), 4, 1, 4, 1, 1, 1, 0, nullptr);
                    else if (N.bn == 32)
                        AA_X3T(dim3((HWo + 127) / 128, N.cout_pad / 32, nz), 4, 1, 2, 2, 1, 1, 0, nullptr);
                    else if (N.C >= 128 && N.g.cin_pad <= 256 && N.cout_pad % 128 == 0)
                        // 64 x 128 tiles: half the re-reads of the pixel tile
                        AA_X3T(dim3((HWo + 63) / 64, N.cout_pad / 128, nz), 2, 2, 2, 4, 1, 1, 0, nullptr);
                    else if (N.split > 1 && nz == 1) {
                        // split K: slices of cslice chunks on blockIdx.z, then the ordered sum
                        float* part = ws + G.part_off * (size_t)n;
                        const dim3 grid((HWo + 63) / 64, N.cout_pad / 64, N.split);
                        if (N.cslice % 2 == 0) AA_X3T(grid, 2, 2, 2, 2, 2, 1, N.cslice, part);
                        else AA_X3T(grid, 2, 2, 2, 2, 1, 1, N.cslice, part);
                        AA_LAUNCH_CHECK();
                        const size_t total = (size_t)HWo * N.C;
                        hipLaunchKernelGGL(gsplit_reduce, dim3((unsigned)((total / 4 + 255) / 256 + 1)), dim3(256), 0, st,
                                           part, N.split, total, N.C, N.d_b, res, out, act, d.alpha);
                    } else {
                        // 64 x 64 tiles, KC 32-channel chunks per K step (the same
                        // products summed in the same order whatever KC is)
                        const int ncc = N.g.cin_pad / 32;
                        const int KC = ncc % 2 == 0 && kGxKcMax >= 2 ? 2 : 1;
                        const dim3 grid((HWo + 63) / 64, N.cout_pad / 64, nz);
                        if (KC == 2) AA_X3T(grid, 2, 2, 2, 2, 2, 1, 0, nullptr);
                        else if (ncc >= 8) AA_X3T(grid, 2, 2, 2, 2, 1, 2, 0, nullptr);
                        else AA_X3T(grid, 2, 2, 2, 2, 1, 1, 0, nullptr);
                    }
#undef AA_X3T
                }
            } else if (N.matvec == 2) {
                hipLaunchKernelGGL(gmatvec_t, dim3((N.C + 255) / 256, n), dim3(256), 0, st, a, (const float*)N.d_w,
                                   N.d_b, out, Cin, N.C, act, d.alpha);
            } else if (N.matvec) {
                hipLaunchKernelGGL(gmatvec, dim3((N.C + 3) / 4, n), dim3(256), 0, st, a, (const float*)N.d_w, N.d_b,
                                   out, Cin, N.C, act, d.alpha);
            } else if (d.kh * d.kw * Cin <= GF32_KMAX) {
                const dim3 grid((N.H * N.W + 255) / 256, (N.C + 31) / 32, n);
                if (N.d_ws)  // an RGB-style stem, weights through the scalar cache
                    hipLaunchKernelGGL((gconv_f32_s<3, 3, 3>), grid, dim3(256), 0, st, a, (const float*)N.d_ws, N.d_b,
                                       out, N.g, act, d.alpha);
                else if (d.kh == 3 && d.kw == 3 && Cin == 3)
                    hipLaunchKernelGGL((gconv_f32_lds<3, 3, 3>), grid, dim3(256), 0, st, a, (const float*)N.d_w, N.d_b,
                                       out, N.g, act, d.alpha);
                else if (d.kh == 3 && d.kw == 3 && Cin == 1)
                    hipLaunchKernelGGL((gconv_f32_lds<3, 3, 1>), grid, dim3(256), 0, st, a, (const float*)N.d_w, N.d_b,
                                       out, N.g, act, d.alpha);
                else
                    hipLaunchKernelGGL((gconv_f32_lds<>), grid, dim3(256), 0, st, a, (const float*)N.d_w, N.d_b, out,
                                       N.g, act, d.alpha);
            } else {
                hipLaunchKernelGGL(gconv_f32, dim3((N.H * N.W + 255) / 256, (N.C + 7) / 8, n), dim3(256), 0, st, a,
                                   (const float*)N.d_w, N.d_b, out, N.g, act, d.alpha);
            }
            break;
        case AA_G_DWCONV:
            if (N.pool_into >= 0) {
                const GNode& P = G.nodes[N.pool_into];
                float* pooled = ws + P.off * (size_t)n;
                if ((Cin & 3) == 0) {
#define AA_DWP(Q, KS, S, R)                                                                                    \
    hipLaunchKernelGGL((gdwconv_pool4<Q, KS, S, R>), dim3((Cin + 4 * Q - 1) / (4 * Q), n), dim3(Q * GP4_STRIPES), 0, \
                       st, a, (const float*)N.d_w, N.d_b, out, pooled, Hin, Win, Cin, N.H, N.W, d.kh, d.kw, d.sh,    \
                       d.sw, d.pt, d.pl, act, d.alpha, P.d.act, P.d.alpha)
                    const bool k3 = d.kh == 3 && d.kw == 3;
                    const int cs = k3 && d.sh == d.sw && (d.sh == 1 || d.sh == 2) ? d.sh : 0;
                    if (cs == 1) AA_DWP(8, 3, 1, 1);
                    else if (cs == 2) AA_DWP(8, 3, 2, 1);
                    else if (k3) AA_DWP(8, 3, 0, 1);
                    else AA_DWP(8, 0, 0, 1);
#undef AA_DWP
                } else {
                    hipLaunchKernelGGL(gdwconv_pool, dim3((Cin + 63) / 64, n), dim3(64 * GP_STRIPES), 0, st, a,
                                       (const float*)N.d_w, N.d_b, out, pooled, Hin, Win, Cin, N.H, N.W, d.kh, d.kw,
                                       d.sh, d.sw, d.pt, d.pl, act, d.alpha, P.d.act, P.d.alpha);
                }
            } else if ((Cin & 3) == 0)
                hipLaunchKernelGGL(gdwconv<4>, dim3((unsigned)((per / 4 + 255) / 256), n), dim3(256), 0, st, a,
                                   (const float*)N.d_w, N.d_b, out, Hin, Win, Cin, N.H, N.W, d.kh, d.kw, d.sh, d.sw,
                                   d.pt, d.pl, act, d.alpha);
            else
                hipLaunchKernelGGL(gdwconv<1>, dim3((unsigned)((per + 255) / 256), n), dim3(256), 0, st, a,
                                   (const float*)N.d_w, N.d_b, out, Hin, Win, Cin, N.H, N.W, d.kh, d.kw, d.sh, d.sw,
                                   d.pt, d.pl, act, d.alpha);
            break;
        case AA_G_MAXPOOL:
        case AA_G_AVGPOOL:
            hipLaunchKernelGGL(gpool2d, dim3((unsigned)((per + 255) / 256), n), dim3(256), 0, st, a, out, Hin, Win, Cin,
                               N.H, N.W, d.kh, d.kw, d.sh, d.sw, d.pt, d.pl, d.op == AA_G_AVGPOOL ? 1 : 0, act,
                               d.alpha);
            break;
        case AA_G_GMAXPOOL:
        case AA_G_GAVGPOOL:
            if ((Cin & 3) == 0)
                hipLaunchKernelGGL((ggpool4<16>), dim3((Cin + 63) / 64, n), dim3(16 * GP4_STRIPES), 0, st, a, out,
                                   Hin, Win, Cin, d.op == AA_G_GAVGPOOL ? 1 : 0, act, d.alpha);
            else
                hipLaunchKernelGGL(ggpool, dim3((Cin + 63) / 64, n), dim3(64 * GP_STRIPES), 0, st, a, out, Hin * Win,
                                   Cin, d.op == AA_G_GAVGPOOL ? 1 : 0, act, d.alpha);
            break;
        case AA_G_ADD:
        case AA_G_MUL: {
            const GNode* B = d.in1 >= 0 ? &G.nodes[d.in1] : nullptr;
            const int bc = B ? (B->H == 1 && B->W == 1 && (N.H != 1 || N.W != 1)) : 0;
            hipLaunchKernelGGL(gbinary, dim3((unsigned)((per + 255) / 256), n), dim3(256), 0, st, a, buf(d.in1), out,
                               per, N.C, d.op == AA_G_MUL ? 1 : 0, bc, act, d.alpha);
            break;
        }
        case AA_G_AFFINE:
            hipLaunchKernelGGL(gaffine, dim3((unsigned)((per * n + 255) / 256)), dim3(256), 0, st, a, N.d_b, N.d_b2,
                               out, per * n, N.C, act, d.alpha);
            break;
        case AA_G_POW:
            hipLaunchKernelGGL(gpow, dim3((unsigned)((per * n + 255) / 256)), dim3(256), 0, st, a, out, per * n,
                               d.alpha);
            break;
        case AA_G_DENSE:
            hipLaunchKernelGGL(gmatvec, dim3((N.C + 3) / 4, n), dim3(256), 0, st, a, (const float*)N.d_w, N.d_b,
                               out, Hin * Win * Cin, N.C, act, d.alpha);
            break;
        default:
            return AA_ERR_UNSUPPORTED;
    }
    AA_LAUNCH_CHECK();
    return AA_OK;
}

}  // namespace aa

using namespace aa;

extern "C" int aa_graph_create(const aa_node* nodes, int32_t n_nodes, const float* blob, int64_t blob_len,
                               int32_t in_h, int32_t in_w, int32_t in_c, int32_t precision, void** graph) {
    AA_CHECK(nodes && blob && graph && n_nodes > 0, AA_ERR_INVALID, "aa_graph_create: null argument");
    AA_CHECK(precision == AA_PREC_BF16X3 || precision == AA_PREC_F32, AA_ERR_UNSUPPORTED,
             "aa_graph_create: graphs run in split-bf16 or f32 (precision %d)", precision);
    AA_CHECK(in_h >= 1 && in_w >= 1 && in_c >= 1, AA_ERR_INVALID, "aa_graph_create: input shape");
    Graph* G = new Graph();
    G->prec = precision;
    G->in_h = in_h;
    G->in_w = in_w;
    G->in_c = in_c;
    const int rc = graph_build(G, nodes, n_nodes, blob, blob_len);
    if (rc != AA_OK) {
        free_graph(G);
        return rc;
    }
    *graph = G;
    return AA_OK;
}

extern "C" int aa_graph_destroy(void* graph) {
    free_graph(static_cast<Graph*>(graph));
    return AA_OK;
}

extern "C" int aa_graph_n_outputs(const void* graph) { return graph ? static_cast<const Graph*>(graph)->L : -1; }

extern "C" size_t aa_graph_workspace_bytes(const void* graph, int32_t max_batch) {
    if (!graph || max_batch < 0) return 0;
    const Graph* G = static_cast<const Graph*>(graph);
    return align_up(G->per_win * 4 * (size_t)std::min<int32_t>(max_batch, 32768), 256);
}

// the forward's launches for n windows (<= 32768) on stream st
static int graph_enqueue(Graph* G, const float* x, int32_t n, float* logits, float* probs, float* ws,
                         hipStream_t st) {
    G->timer.mask = 0xFFFFFFFFu;  // the node filter is time_stage (graphs exceed 32 stages)
    for (size_t i = 0; i < G->nodes.size(); ++i) {
        if (G->nodes[i].skip || G->nodes[i].nolaunch) continue;
        const bool timed = G->time_stage == -1 || G->time_stage == (int)i;
        hipEvent_t e0 = nullptr;
        if (timed) {
            const int rc = G->timer.begin(0, st, &e0);
            if (rc != AA_OK) return rc;
        }
        const int rc = graph_run_node(*G, G->nodes[i], x, ws, n, st);
        if (rc != AA_OK) return rc;
        if (timed) {
            const int rc2 = G->timer.end((int)i, st, e0);
            if (rc2 != AA_OK) return rc2;
        }
    }
    const GNode& O = G->nodes.back();
    const size_t total = (size_t)G->L * n;
    hipLaunchKernelGGL(gfinal, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, ws + O.off * (size_t)n, logits,
                       probs, total, G->sigmoid_out);
    AA_LAUNCH_CHECK();
    return AA_OK;
}

extern "C" int aa_graph_forward(void* graph, const float* x, int32_t n, float* logits, float* probs, void* workspace,
                                size_t workspace_bytes, void* stream) {
    Graph* G = static_cast<Graph*>(graph);
    AA_CHECK(G && x && logits, AA_ERR_INVALID, "aa_graph_forward: null argument");
    if (n <= 0) return AA_OK;
    constexpr int32_t CHUNK = 32768;  // grids carry the window in blockIdx.y / z
    const int32_t nc0 = std::min(n, CHUNK);
    AA_CHECK(workspace && workspace_bytes >= aa_graph_workspace_bytes(G, nc0), AA_ERR_WORKSPACE,
             "aa_graph_forward: workspace %zu < %zu", workspace_bytes, aa_graph_workspace_bytes(G, nc0));
    hipStream_t st = static_cast<hipStream_t>(stream);
    float* ws = static_cast<float*>(workspace);
    const size_t in_per = (size_t)G->in_h * G->in_w * G->in_c;
    // replay a captured forward (not while timing nodes: the events would be
    // baked into the capture; not on the legacy null stream, which cannot capture)
    if (n <= CHUNK && G->time_stage == -2 && st != nullptr) {
        std::lock_guard<std::mutex> lk(G->cap_mu);
        auto same = [&](const Graph::Captured& c) {
            return c.x == x && c.n == n && c.ws == workspace && c.logits == logits && c.probs == probs && c.st == st;
        };
        for (const auto& c : G->captured)
            if (same(c)) {
                AA_HIP(hipGraphLaunch(c.exec, st));
                AA_HIP(hipEventRecord(c.done, st));
                return AA_OK;
            }
        bool again = false;
        for (auto it = G->seen.begin(); it != G->seen.end(); ++it)
            if (same(*it)) {
                again = true;
                G->seen.erase(it);
                break;
            }
        if (!again) {
            if (G->seen.size() >= AA_GRAPH_CAPTURES) G->seen.erase(G->seen.begin());
            G->seen.push_back(Graph::Captured{x, n, workspace, logits, probs, st, nullptr, nullptr});
            return graph_enqueue(G, x, n, logits, probs, ws, st);
        }
        // capture; if the stream cannot be captured (the runtime refuses, or the
        // caller's stream is itself capturing), launch node by node instead
        hipGraph_t hg = nullptr;
        if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            (void)hipGetLastError();
            return graph_enqueue(G, x, n, logits, probs, ws, st);
        }
        const int rc = graph_enqueue(G, x, n, logits, probs, ws, st);
        const hipError_t ec = hipStreamEndCapture(st, &hg);
        hipGraphExec_t exec = nullptr;
        const hipError_t ei = (rc == AA_OK && ec == hipSuccess) ? hipGraphInstantiate(&exec, hg, nullptr, nullptr, 0)
                                                                : hipErrorUnknown;
        if (hg) (void)hipGraphDestroy(hg);
        if (rc != AA_OK) return rc;  // a launch-configuration error: report it
        if (ei != hipSuccess) {
            (void)hipGetLastError();
            // (nothing ran during the capture attempt)
            return graph_enqueue(G, x, n, logits, probs, ws, st);
        }
        hipEvent_t done = nullptr;
        if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipGraphExecDestroy(exec);
            return graph_enqueue(G, x, n, logits, probs, ws, st);
        }
        if (G->captured.size() >= AA_GRAPH_CAPTURES) {  // bounded: the oldest goes
            release_captured(G->captured.front());
            G->captured.erase(G->captured.begin());
        }
        G->captured.push_back(Graph::Captured{x, n, workspace, logits, probs, st, exec, done});
        AA_HIP(hipGraphLaunch(exec, st));
        AA_HIP(hipEventRecord(done, st));
        return AA_OK;
    }
    for (int32_t c0 = 0; c0 < n; c0 += CHUNK) {
        const int32_t nc = std::min(CHUNK, n - c0);
        const int rc = graph_enqueue(G, x + (size_t)c0 * in_per, nc, logits + (size_t)c0 * G->L,
                                     probs ? probs + (size_t)c0 * G->L : nullptr, ws, st);
        if (rc != AA_OK) return rc;
    }
    return AA_OK;
}

extern "C" int aa_graph_n_stages(const void* graph) {
    return graph ? (int)static_cast<const Graph*>(graph)->nodes.size() : -1;
}

extern "C" int aa_graph_stage_info(const void* graph, int32_t stage, char* name, int32_t name_len,
                                   double* flops_per_item, double* bytes_per_item) {
    const Graph* G = static_cast<const Graph*>(graph);
    AA_CHECK(G && stage >= 0 && stage < (int)G->nodes.size(), AA_ERR_INVALID, "aa_graph_stage_info: bad stage");
    const GNode& N = G->nodes[stage];
    if (name && name_len > 0) snprintf(name, name_len, "%s", N.name.c_str());
    if (flops_per_item) *flops_per_item = N.flops;
    if (bytes_per_item) *bytes_per_item = N.bytes;
    return AA_OK;
}

// Node timing (the aa_model_stage_* contract, per node; a graph has more nodes
// than a 32-bit stage mask holds): set_timing(mask != 0) times every node,
// time_stage(k) only node k (-1 every node, -2 none).
extern "C" int aa_graph_set_timing(void* graph, uint32_t stage_mask) {
    Graph* G = static_cast<Graph*>(graph);
    AA_CHECK(G, AA_ERR_INVALID, "aa_graph_set_timing: null graph");
    G->time_stage = stage_mask ? -1 : -2;
    return AA_OK;
}

extern "C" int aa_graph_time_stage(void* graph, int32_t stage) {
    Graph* G = static_cast<Graph*>(graph);
    AA_CHECK(G && stage >= -2 && stage < (int)G->nodes.size(), AA_ERR_INVALID, "aa_graph_time_stage: bad stage");
    G->time_stage = stage;
    return AA_OK;
}

extern "C" int aa_graph_stage_time(void* graph, int32_t stage, double* total_ms, int64_t* count) {
    Graph* G = static_cast<Graph*>(graph);
    AA_CHECK(G && stage >= 0 && stage < (int)G->nodes.size(), AA_ERR_INVALID, "aa_graph_stage_time: bad stage");
    return G->timer.collect(stage, total_ms, count);
}
