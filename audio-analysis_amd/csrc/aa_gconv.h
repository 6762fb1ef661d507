// Runtime-shaped layers: the kernels behind any conv / pool / elementwise
// shape the tuned tables of aa_cnn.hip do not cover, and behind the graph
// (DAG) models of aa_graph.hip.  Included by both.
//
// gconv_x3: split-bf16 implicit GEMM on v_mfma_f32_16x16x32_bf16 for any
// kernel size, stride and padding (explicit top/left; the output size sets
// the bottom/right), C_in padded to 32 with zero weights, any C_out.  A
// 256-thread block computes 64 output pixels x 64 output channels: per
// K step (tap, 32 input channels) it gathers the 64 pixels' 32 channels
// (zero outside the image), splits them into bf16 hi / lo in LDS next to the
// step's pre-split weight slice, and each wave (2 x 2 over the tile) runs
// 2 x 2 fragments x 3 MFMAs (hi*hi + lo*hi + hi*lo, f32 accumulation, as
// conv_x3).  LDS rows are 96 B (32 bf16 + 16 B; per KC chunk 64 B more).
// Fused epilogue: bias,
// activation, NHWC f32 store (4 channels per lane).
//
// gconv_f32: the same geometry in exact f32 FMA chains (VALU), for C_in < 16
// and the f32 parity mode.
#pragma once

#include <type_traits>

#include "aa_common.h"

namespace aa {

enum GAct { GACT_NONE = 0, GACT_RELU = 1, GACT_LEAKY = 2, GACT_SIGMOID = 3, GACT_SWISH = 4 };

// The logistic of sigmoid / swish as v_exp_f32 (2^x) and v_rcp_f32, each
// within 1 ulp: 3 VALU instead of expf's range reduction and the IEEE
// division's scale / fixup sequence (~25), which made the epilogues of the
// graph's expand convs VALU-bound (112 -> 672: 21 VALU per MFMA).  Keras'
// own logistic (Eigen's rational approximation on the CPU) is no closer to
// the exact value than this.  Large -v: 2^x = inf, rcp(inf) = 0.
#ifndef AA_GACT_FAST
#define AA_GACT_FAST 1
#endif
__device__ __forceinline__ float glogistic(float v) {
#if AA_GACT_FAST
    return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(v * -1.44269504088896341f));
#else
    return 1.f / (1.f + expf(-v));
#endif
}
__device__ __forceinline__ float gact(float v, int act, float alpha) {
    switch (act) {
        case GACT_RELU: return fmaxf(v, 0.f);
        case GACT_LEAKY: return v >= 0.f ? v : v * alpha;
        case GACT_SIGMOID: return glogistic(v);
        case GACT_SWISH: return v * glogistic(v);
        default: return v;
    }
}

// f(integral_constant<int, act>): the activation resolved once, outside a
// kernel's per-element loops (a runtime `act` inside them is if-converted
// into every variant's instructions)
template <class F>
__device__ __forceinline__ void with_act(int act, F&& f) {
    switch (act) {
        case GACT_RELU: f(std::integral_constant<int, GACT_RELU>{}); break;
        case GACT_LEAKY: f(std::integral_constant<int, GACT_LEAKY>{}); break;
        case GACT_SIGMOID: f(std::integral_constant<int, GACT_SIGMOID>{}); break;
        case GACT_SWISH: f(std::integral_constant<int, GACT_SWISH>{}); break;
        default: f(std::integral_constant<int, GACT_NONE>{}); break;
    }
}

struct ConvGeom {
    int Hin, Win, Cin;   // input (NHWC)
    int Hout, Wout, Cout;
    int kh, kw, sh, sw;  // kernel, strides
    int pt, pl;          // top / left zero padding
    int cin_pad;         // Cin rounded up to 32 (gconv_x3 weight packing)
};

typedef __attribute__((ext_vector_type(8))) __bf16 gbf16x8;
typedef __attribute__((ext_vector_type(4))) float gf32x4;

// LDS rows of the patch-staged conv (gconv_x3p): 32 bf16 +
// GX_PAD.  8 (80 B rows, an odd multiple of 16 B, so the 16 rows of a
// fragment read sit on distinct banks) instead of round 4's 16 (96 B): the
// 3x3 32->16 patch kernel 125 -> 107 us -- the smaller patch (52 KiB) also
// fits three blocks per CU instead of two (profiles/r04/graph_ab_pad.txt).
#ifndef AA_GX_PAD
#define AA_GX_PAD 8
#endif
constexpr int GX_PAD = AA_GX_PAD;
constexpr int GX_ROW = 32 + GX_PAD;  // bf16 per LDS row (80 B)

// The block's (x, y, z) tile coordinates.  xord = 0: the launch grid's.
// xord = 1, XCD-aware order (as x3_block in aa_conv_x3.h): workgroup L (x
// fastest) is dispatched to XCD L % 8, so XCD x is given the contiguous
// logical range [x per, (x + 1) per) of an order with y (the channel blocks
// of a pixel tile) fastest, then x, then z: a tile's pixels -- and its
// neighbours' halo rows -- are read into one L2 once instead of once per
// channel block on every XCD.  Each block's arithmetic is unchanged
// (bit-identical results).
__device__ __forceinline__ void xcd_order(int xord, int& bx, int& by, int& bz) {
    bx = blockIdx.x;
    by = blockIdx.y;
    bz = blockIdx.z;
    if (!xord) return;
    const int X = gridDim.x, Y = gridDim.y;
    const int total = X * Y * (int)gridDim.z, per = total >> 3;
    const int L = blockIdx.x + X * (blockIdx.y + Y * blockIdx.z);
    const int lg = L < (per << 3) ? (L & 7) * per + (L >> 3) : L;
    by = lg % Y;
    const int rr = lg / Y;
    bx = rr % X;
    bz = rr / X;
}

// weights: [tap][cin_pad / 32][cout_pad][64] bf16, per row 32 hi then 32 lo.
// Tile: BM = WM MF 16 output pixels x BN = WN NF 16 output channels, the four
// waves WM x WN over it, each MF x NF fragments (64 x 64 by default; narrow
// layers take 128 x 32 or 256 x 16 so that C_out = 16 / 32 does not pay for 64
// padded channels).  cout_pad is a multiple of BN.
// Optional fusions (nullptr: off): in_scale [n][Cin] multiplies the input
// channels as they are staged (a squeeze-and-excite Multiply before the conv,
// the same f32 product the separate node computes), res [n][HWo][Cout] is
// added after the bias and before the activation (a residual Add after a
// conv without activation; the add's own activation is `act`).  The next K
// step's pixels and weights are loaded into registers before this step's
// MFMAs, so their latency hides behind the matrix work.
//
// KC: 32-channel chunks per K step (1, 2, 3 or 4; the layer's chunk count a
// multiple of it): KC x the MFMAs per barrier pair and per L2 round trip --
// a 1x1 conv over 1152 channels on a small map is otherwise 36 dependent
// steps of 12 MFMAs.  scale_hw > 0: the pixels of n windows run flattened as
// one image (pointwise convs) and pixel P's squeeze-and-excite scale is that
// of window P / scale_hw.
//
// PD: K steps whose loads are in flight at once (a register ring PD deep):
// step s's pixels and weights are loaded PD steps ahead.
template <int WM, int WN, int MF, int NF, int KC = 1, int PD = 1>
__global__ __launch_bounds__(256) void gconv_x3t(const float* __restrict__ in, const uint16_t* __restrict__ wpk,
                                                 const float* __restrict__ bias, float* __restrict__ out,
                                                 ConvGeom g, int cout_pad, int act, float alpha,
                                                 const float* __restrict__ in_scale, const float* __restrict__ res,
                                                 int scale_hw = 0, int cslice = 0, float* __restrict__ part = nullptr,
                                                 int xord = 0) {
    static_assert(WM * WN == 4, "four waves");
    constexpr int BM = WM * MF * 16, BN = WN * NF * 16, AI = BM / 64, BI = (BN + 63) / 64;
    // bf16 per LDS row: +32 B (the odd-multiple-of-16-B stride of GX_ROW
    // measured slower here: 3x3 48->192 96 -> 102 us, 16->64 81 -> 85 us,
    // 32->128 unchanged; profiles/r04/graph_ab_pad.txt)
    constexpr int ROW = KC * 32 + 16;
    __shared__ __attribute__((aligned(16))) uint16_t Ah[BM * ROW], Al[BM * ROW];
    __shared__ __attribute__((aligned(16))) uint16_t Bh[BN * ROW], Bl[BN * ROW];
    int bx, by, bz;
    xcd_order(xord, bx, by, bz);
    const int n = part ? 0 : bz;  // (split K: z is the slice)
    const int pix0 = bx * BM, ch0 = by * BN;
    const int HWo = g.Hout * g.Wout;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave % WM, wn = wave / WM;
    // staging role: rows r + 64 it (pixels) and r (weights, r < BN), 8-element quad q
    const int r = t >> 2, q = t & 3;
    int oy[AI], ox[AI];
    bool pv[AI];
    const float* sclp[AI];
#pragma unroll
    for (int it = 0; it < AI; ++it) {
        const int P = pix0 + r + 64 * it;
        pv[it] = P < HWo;
        oy[it] = pv[it] ? P / g.Wout : 0;
        ox[it] = pv[it] ? P - (P / g.Wout) * g.Wout : 0;
        sclp[it] = !in_scale ? nullptr
                   : scale_hw > 0 ? in_scale + (size_t)((pv[it] ? P : 0) / scale_hw) * g.Cin
                                  : in_scale + (size_t)n * g.Cin;
    }
    // weight rows r + 64 ib (ib < BI) of the block's BN
    const float* img = in + (size_t)n * g.Hin * g.Win * g.Cin;
    const int ncc = g.cin_pad / 32;
    // split K (part != nullptr, flattened pointwise convs): blockIdx.z = slice
    // of cslice chunks, raw sums to part[slice][pixel][Cout] (gsplit_reduce
    // adds the slices in order, then bias, residual and activation)
    const int cbase = part ? bz * cslice : 0;
    const int ngs = (part ? cslice : ncc) / KC;  // K steps per tap
    const int nsteps = g.kh * g.kw * ngs;
    gf32x4 acc[NF][MF];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j) acc[i][j] = gf32x4{0.f, 0.f, 0.f, 0.f};
    const bool vec = (g.Cin & 7) == 0;
    float v[PD][AI][KC][8];
    uint4 wh[PD][BI][KC], wl[PD][BI][KC];
#pragma unroll
    for (int u = 0; u < PD; ++u)
#pragma unroll
        for (int ib = 0; ib < BI; ++ib)
#pragma unroll
            for (int k = 0; k < KC; ++k) wh[u][ib][k] = wl[u][ib][k] = make_uint4(0, 0, 0, 0);
    // step s = (tap, chunks KC gs .. KC gs + KC - 1): this thread's 8 channels
    // of AI pixels per chunk and its 8 hi + 8 lo weights per chunk
    // the coordinates (kernel row, column, chunk group) of the next step to
    // load, stepped on by one per load (no integer divisions per step)
    int l_ky = 0, l_kx = 0, l_gs = 0;
    auto load = [&](float (&vb)[AI][KC][8], uint4 (&whb)[BI][KC], uint4 (&wlb)[BI][KC]) {
        const int ky = l_ky, kx = l_kx, gs = l_gs, tap = ky * g.kw + kx;
        if (++l_gs == ngs) {
            l_gs = 0;
            if (++l_kx == g.kw) {
                l_kx = 0;
                ++l_ky;
            }
        }
#pragma unroll
        for (int it = 0; it < AI; ++it) {
            const int iy = oy[it] * g.sh - g.pt + ky, ix = ox[it] * g.sw - g.pl + kx;
            const bool inside = pv[it] && iy >= 0 && iy < g.Hin && ix >= 0 && ix < g.Win;
            const float* px = img + ((size_t)(inside ? iy : 0) * g.Win + (inside ? ix : 0)) * g.Cin;
            const float* scl = sclp[it];
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const int c0 = (cbase + gs * KC + k) * 32 + 8 * q;
                if (vec && c0 >= g.Cin) {  // a padding chunk's quad: zeros, no loads
#pragma unroll
                    for (int e = 0; e < 8; ++e) vb[it][k][e] = 0.f;
                } else if (inside && vec && c0 + 8 <= g.Cin) {
                    const float4 a = *reinterpret_cast<const float4*>(px + c0);
                    const float4 b = *reinterpret_cast<const float4*>(px + c0 + 4);
                    vb[it][k][0] = a.x; vb[it][k][1] = a.y; vb[it][k][2] = a.z; vb[it][k][3] = a.w;
                    vb[it][k][4] = b.x; vb[it][k][5] = b.y; vb[it][k][6] = b.z; vb[it][k][7] = b.w;
                    if (scl) {
                        const float4 sa = *reinterpret_cast<const float4*>(scl + c0);
                        const float4 sb = *reinterpret_cast<const float4*>(scl + c0 + 4);
                        vb[it][k][0] *= sa.x; vb[it][k][1] *= sa.y; vb[it][k][2] *= sa.z; vb[it][k][3] *= sa.w;
                        vb[it][k][4] *= sb.x; vb[it][k][5] *= sb.y; vb[it][k][6] *= sb.z; vb[it][k][7] *= sb.w;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const bool ok = inside && c0 + e < g.Cin;
                        vb[it][k][e] = ok ? (scl ? px[c0 + e] * scl[c0 + e] : px[c0 + e]) : 0.f;
                    }
                }
            }
        }
#pragma unroll
        for (int ib = 0; ib < BI; ++ib) {
            if (r + 64 * ib >= BN) continue;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const uint16_t* wrow =
                    wpk + (((size_t)(tap * ncc + cbase + gs * KC + k) * cout_pad) + ch0 + r + 64 * ib) * 64;
                whb[ib][k] = *reinterpret_cast<const uint4*>(wrow + 8 * q);
                wlb[ib][k] = *reinterpret_cast<const uint4*>(wrow + 32 + 8 * q);
            }
        }
    };
#pragma unroll
    for (int u = 0; u < PD; ++u)
        if (u < nsteps) load(v[u], wh[u], wl[u]);
    for (int s0 = 0; s0 < nsteps; s0 += PD)
#pragma unroll
    for (int u = 0; u < PD; ++u) {
        const int s = s0 + u;
        if (s >= nsteps) break;  // block-uniform
        gbf16x8 h[AI][KC], l[AI][KC];
#pragma unroll
        for (int it = 0; it < AI; ++it)
#pragma unroll
            for (int k = 0; k < KC; ++k)
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    h[it][k][e] = (__bf16)v[u][it][k][e];
                    l[it][k][e] = (__bf16)(v[u][it][k][e] - (float)h[it][k][e]);
                }
        __syncthreads();  // the previous step's fragments are read
#pragma unroll
        for (int it = 0; it < AI; ++it)
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                *reinterpret_cast<gbf16x8*>(Ah + (r + 64 * it) * ROW + 32 * k + 8 * q) = h[it][k];
                *reinterpret_cast<gbf16x8*>(Al + (r + 64 * it) * ROW + 32 * k + 8 * q) = l[it][k];
            }
#pragma unroll
        for (int ib = 0; ib < BI; ++ib) {
            if (r + 64 * ib >= BN) continue;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                *reinterpret_cast<uint4*>(Bh + (r + 64 * ib) * ROW + 32 * k + 8 * q) = wh[u][ib][k];
                *reinterpret_cast<uint4*>(Bl + (r + 64 * ib) * ROW + 32 * k + 8 * q) = wl[u][ib][k];
            }
        }
        __syncthreads();
        if (s + PD < nsteps) load(v[u], wh[u], wl[u]);
#pragma unroll
        for (int k = 0; k < KC; ++k) {
            const int ko = 32 * k + 8 * (lane >> 4);
#pragma unroll
            for (int i = 0; i < NF; ++i) {
                const int wr = (wn * NF * 16 + i * 16 + (lane & 15)) * ROW + ko;
                const gbf16x8 w_h = *reinterpret_cast<const gbf16x8*>(Bh + wr);
                const gbf16x8 w_l = *reinterpret_cast<const gbf16x8*>(Bl + wr);
#pragma unroll
                for (int j = 0; j < MF; ++j) {
                    const int xr = (wm * MF * 16 + j * 16 + (lane & 15)) * ROW + ko;
                    const gbf16x8 x_h = *reinterpret_cast<const gbf16x8*>(Ah + xr);
                    const gbf16x8 x_l = *reinterpret_cast<const gbf16x8*>(Al + xr);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_h, x_h, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_l, x_h, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_h, x_l, acc[i][j], 0, 0, 0);
                }
            }
        }
    }
    // D[channel][pixel]: lane holds channels 4 (lane >> 4) .. + 3 of pixel lane & 15
    if (part) {
#pragma unroll
        for (int j = 0; j < MF; ++j) {
            const int Pj = pix0 + wm * MF * 16 + j * 16 + (lane & 15);
            if (Pj >= HWo) continue;
            float* o = part + ((size_t)bz * HWo + Pj) * g.Cout;
#pragma unroll
            for (int i = 0; i < NF; ++i) {
                const int c = ch0 + wn * NF * 16 + i * 16 + 4 * (lane >> 4);
                if (c + 4 <= g.Cout && (g.Cout & 3) == 0) {
                    *reinterpret_cast<float4*>(o + c) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
                } else {
                    for (int e = 0; e < 4 && c + e < g.Cout; ++e) o[c + e] = acc[i][j][e];
                }
            }
        }
        return;
    }
    float bv[NF][4];  // the lane's channels' biases, the same for every pixel fragment
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int c = ch0 + wn * NF * 16 + i * 16 + 4 * (lane >> 4);
        if (c + 4 <= g.Cout && (g.Cout & 3) == 0) {
            const float4 b4 = *reinterpret_cast<const float4*>(bias + c);
            bv[i][0] = b4.x; bv[i][1] = b4.y; bv[i][2] = b4.z; bv[i][3] = b4.w;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) bv[i][e] = c + e < g.Cout ? bias[c + e] : 0.f;
        }
    }
    // the activation resolved once per block (a per-element switch was
    // if-converted into every variant's instructions), the residual read as
    // float4 where the lane's 4 channels are whole
    const bool full4 = (g.Cout & 3) == 0;
    auto epi = [&](auto actc) {
        constexpr int A = decltype(actc)::value;
#pragma unroll
        for (int j = 0; j < MF; ++j) {
            const int Pj = pix0 + wm * MF * 16 + j * 16 + (lane & 15);
            if (Pj >= HWo) continue;
            float* o = out + ((size_t)n * HWo + Pj) * g.Cout;
            const float* rp = res ? res + ((size_t)n * HWo + Pj) * g.Cout : nullptr;
#pragma unroll
            for (int i = 0; i < NF; ++i) {
                const int c = ch0 + wn * NF * 16 + i * 16 + 4 * (lane >> 4);
                float y[4];
                if (full4 && c + 4 <= g.Cout) {
                    float z[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) z[e] = acc[i][j][e] + bv[i][e];
                    if (rp) {
                        const float4 r4 = *reinterpret_cast<const float4*>(rp + c);
                        z[0] += r4.x; z[1] += r4.y; z[2] += r4.z; z[3] += r4.w;
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e) y[e] = gact(z[e], A, alpha);
                    *reinterpret_cast<float4*>(o + c) = make_float4(y[0], y[1], y[2], y[3]);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float z = acc[i][j][e] + bv[i][e];
                        if (rp && c + e < g.Cout) z += rp[c + e];
                        y[e] = gact(z, A, alpha);
                    }
                    for (int e = 0; e < 4 && c + e < g.Cout; ++e) o[c + e] = y[e];
                }
            }
        }
    };
    with_act(act, epi);
}

// the split-K slices of a pointwise conv added in slice order, then the
// epilogue of gconv_x3t (bias, residual, activation); total = pixels x Cout
static __global__ __launch_bounds__(256) void gsplit_reduce(const float* __restrict__ part, int nslice, size_t total,
                                                     int Cout, const float* __restrict__ bias,
                                                     const float* __restrict__ res, float* __restrict__ out, int act,
                                                     float alpha) {
    const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i >= total) return;
    if ((Cout & 3) == 0) {
        float4 a = *reinterpret_cast<const float4*>(part + i);
        for (int s = 1; s < nslice; ++s) {
            const float4 b = *reinterpret_cast<const float4*>(part + (size_t)s * total + i);
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        const int c = (int)(i % Cout);
        float z[4] = {a.x + bias[c], a.y + bias[c + 1], a.z + bias[c + 2], a.w + bias[c + 3]};
        if (res) {
            const float4 r = *reinterpret_cast<const float4*>(res + i);
            z[0] += r.x; z[1] += r.y; z[2] += r.z; z[3] += r.w;
        }
        *reinterpret_cast<float4*>(out + i) =
            make_float4(gact(z[0], act, alpha), gact(z[1], act, alpha), gact(z[2], act, alpha), gact(z[3], act, alpha));
    } else {
        for (size_t k = i; k < i + 4 && k < total; ++k) {
            float a = part[k];
            for (int s = 1; s < nslice; ++s) a += part[(size_t)s * total + k];
            float z = a + bias[(int)(k % Cout)];
            if (res) z += res[k];
            out[k] = gact(z, act, alpha);
        }
    }
}

// gconv_x3p stages a chunk as (pixel, 8-channel quad) items, GX_P_STG per
// thread of its 256: patches of more than GX_P_STG * 64 pixels would leave
// pixels unwritten, so the host checks gconv_x3p_fits (patch pixels and the
// 64 KiB LDS cap) before it picks that kernel.
constexpr int GX_P_STG = 6;
static inline bool gconv_x3p_fits(int ph, int pw) {
    const long np = (long)ph * pw;
    return np * 4 <= (long)GX_P_STG * 256 && np * GX_ROW * 4 <= 65536;
}

// tile of a layer with C_out output channels: BN = 16, 32 or 64
static inline int gconv_bn(int cout) { return cout <= 16 ? 16 : cout <= 32 ? 32 : 64; }

// gconv_x3p: the same split-bf16 conv for kernels larger than 1x1, with the
// input patch of a TH x TW output tile staged once per 32-channel chunk (hi /
// lo planes in LDS, 96-B rows) and every tap's A fragments read from it --
// gconv_x3t gathers the tile's pixels again for every tap, i.e. reads its
// input kh kw times through L2.  B fragments come straight from L2 (16-B
// loads per lane), one tap ahead in registers, so the tap loop has no
// barrier.  TH = BM / TW; patch PH x PW = ((TH - 1) sh + kh) x ((TW - 1) sw +
// kw) pixels, dynamic LDS.  Accumulation runs chunk-major (all taps of chunk
// 0, then chunk 1, ...).
// TWC > 0: the tile width at compile time (divisions by it become shifts)
template <int WM, int WN, int MF, int NF, int TWC = 0>
__global__ __launch_bounds__(256) void gconv_x3p(const float* __restrict__ in, const uint16_t* __restrict__ wpk,
                                                 const float* __restrict__ bias, float* __restrict__ out,
                                                 ConvGeom g, int cout_pad, int act, float alpha, int TWr, int tiles_w,
                                                 const float* __restrict__ in_scale, const float* __restrict__ res,
                                                 int xord = 0) {
    static_assert(WM * WN == 4, "four waves");
    constexpr int BM = WM * MF * 16, BN = WN * NF * 16;
    extern __shared__ __attribute__((aligned(16))) uint16_t gsm[];
    int bx, by, bz;
    xcd_order(xord, bx, by, bz);
    const int TW = TWC ? TWC : TWr;
    const int TH = BM / TW;
    const int PH = (TH - 1) * g.sh + g.kh, PW = (TW - 1) * g.sw + g.kw, NP = PH * PW;
    uint16_t* Ph = gsm;
    uint16_t* Pl = gsm + NP * GX_ROW;
    const int n = bz;
    const int ty = bx / tiles_w, tx = bx - (bx / tiles_w) * tiles_w;
    const int oy0 = ty * TH, ox0 = tx * TW;
    const int ch0 = by * BN;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave % WM, wn = wave / WM;
    const int iy0 = oy0 * g.sh - g.pt, ix0 = ox0 * g.sw - g.pl;
    const float* img = in + (size_t)n * g.Hin * g.Win * g.Cin;
    const float* scl = in_scale ? in_scale + (size_t)n * g.Cin : nullptr;
    const int ncc = g.cin_pad / 32;
    const int ntap = g.kh * g.kw;
    // the lane's fragment pixels: patch index of tap (0, 0)
    int pb[MF];
#pragma unroll
    for (int j = 0; j < MF; ++j) {
        const int p = wm * MF * 16 + j * 16 + (lane & 15);
        const int py = p / TW, px = p - (p / TW) * TW;
        pb[j] = py * g.sh * PW + px * g.sw;
    }
    const int ko = 8 * (lane >> 4);
    gf32x4 acc[NF][MF];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j) acc[i][j] = gf32x4{0.f, 0.f, 0.f, 0.f};
    const bool vec = (g.Cin & 7) == 0;
    gbf16x8 b0h[NF], b0l[NF], b1h[NF], b1l[NF];  // B of this tap / the next (slots fixed by unrolling)
    auto load_b = [&](int s, gbf16x8 (&h)[NF], gbf16x8 (&l)[NF]) {
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const uint16_t* wrow = wpk + ((size_t)s * cout_pad + ch0 + wn * NF * 16 + i * 16 + (lane & 15)) * 64 + ko;
            h[i] = *reinterpret_cast<const gbf16x8*>(wrow);
            l[i] = *reinterpret_cast<const gbf16x8*>(wrow + 32);
        }
    };
    int tky = 0, tkx = 0;  // the tap's kernel row / column, stepped on per tap (no divisions)
    auto tap_step = [&](int tap, int cc, const gbf16x8 (&h)[NF], const gbf16x8 (&l)[NF], gbf16x8 (&nh)[NF],
                        gbf16x8 (&nl)[NF]) {
        if (tap + 1 < ntap) load_b((tap + 1) * ncc + cc, nh, nl);
        const int toff = tky * PW + tkx;
        if (++tkx == g.kw) {
            tkx = 0;
            ++tky;
        }
#pragma unroll
        for (int j = 0; j < MF; ++j) {
            const int xr = (pb[j] + toff) * GX_ROW + ko;
            const gbf16x8 x_h = *reinterpret_cast<const gbf16x8*>(Ph + xr);
            const gbf16x8 x_l = *reinterpret_cast<const gbf16x8*>(Pl + xr);
#pragma unroll
            for (int i = 0; i < NF; ++i) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h[i], x_h, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(l[i], x_h, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h[i], x_l, acc[i][j], 0, 0, 0);
            }
        }
    };
    for (int cc = 0; cc < ncc; ++cc) {
        load_b(cc, b0h, b0l);  // tap 0 of this chunk: in flight during the staging
        if (cc > 0) __syncthreads();  // every wave is done with the previous chunk's patch
        // ---- stage the chunk: item = (patch pixel, 8-channel quad); every
        // item's loads issued before any is split (GX_P_STG items per thread:
        // the host launches this kernel only for patches of <= GX_P_STG * 64
        // pixels, gconv_x3p_fits), the patch coordinates by
        // a float reciprocal (exact: (pix + 1/2) / PW stays >= 1/128 from an
        // integer for PW <= 64) ----
        constexpr int STG = GX_P_STG;
        const float inv_pw = 1.f / (float)PW;
        float v[STG][8];
        int pixs[STG];
#pragma unroll
        for (int u = 0; u < STG; ++u) {
            const int it = t + 256 * u;
            const int pix = it >> 2, q = it & 3;
            pixs[u] = it < NP * 4 ? pix : -1;
            const int R = (int)(((float)pix + 0.5f) * inv_pw), C = pix - R * PW;
            const int iy = iy0 + R, ix = ix0 + C;
            const bool inside = it < NP * 4 && iy >= 0 && iy < g.Hin && ix >= 0 && ix < g.Win;
            const int c0 = cc * 32 + 8 * q;
            const float* px = img + ((size_t)(inside ? iy : 0) * g.Win + (inside ? ix : 0)) * g.Cin;
            if (inside && vec && c0 + 8 <= g.Cin) {
                const float4 a = *reinterpret_cast<const float4*>(px + c0);
                const float4 b = *reinterpret_cast<const float4*>(px + c0 + 4);
                v[u][0] = a.x; v[u][1] = a.y; v[u][2] = a.z; v[u][3] = a.w;
                v[u][4] = b.x; v[u][5] = b.y; v[u][6] = b.z; v[u][7] = b.w;
                if (scl) {
                    const float4 sa = *reinterpret_cast<const float4*>(scl + c0);
                    const float4 sb = *reinterpret_cast<const float4*>(scl + c0 + 4);
                    v[u][0] *= sa.x; v[u][1] *= sa.y; v[u][2] *= sa.z; v[u][3] *= sa.w;
                    v[u][4] *= sb.x; v[u][5] *= sb.y; v[u][6] *= sb.z; v[u][7] *= sb.w;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const bool ok = inside && c0 + e < g.Cin;
                    v[u][e] = ok ? (scl ? px[c0 + e] * scl[c0 + e] : px[c0 + e]) : 0.f;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < STG; ++u) {
            if (pixs[u] < 0) continue;
            const int q = (t + 256 * u) & 3;
            gbf16x8 h, l;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                h[e] = (__bf16)v[u][e];
                l[e] = (__bf16)(v[u][e] - (float)h[e]);
            }
            *reinterpret_cast<gbf16x8*>(Ph + pixs[u] * GX_ROW + 8 * q) = h;
            *reinterpret_cast<gbf16x8*>(Pl + pixs[u] * GX_ROW + 8 * q) = l;
        }
        __syncthreads();
        // ---- the chunk's taps, two per iteration (B slots alternate) ----
        tky = tkx = 0;
        for (int tap = 0; tap < ntap; tap += 2) {
            tap_step(tap, cc, b0h, b0l, b1h, b1l);
            if (tap + 1 < ntap) tap_step(tap + 1, cc, b1h, b1l, b0h, b0l);
        }
    }
    const int HWo = g.Hout * g.Wout;
#pragma unroll
    for (int j = 0; j < MF; ++j) {
        const int p = wm * MF * 16 + j * 16 + (lane & 15);
        const int oy = oy0 + p / TW, ox = ox0 + p - (p / TW) * TW;
        if (oy >= g.Hout || ox >= g.Wout) continue;
        const int Pj = oy * g.Wout + ox;
        float* o = out + ((size_t)n * HWo + Pj) * g.Cout;
        const float* rp = res ? res + ((size_t)n * HWo + Pj) * g.Cout : nullptr;
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int c = ch0 + wn * NF * 16 + i * 16 + 4 * (lane >> 4);
            float y[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float z = acc[i][j][e] + (c + e < g.Cout ? bias[c + e] : 0.f);
                if (rp && c + e < g.Cout) z += rp[c + e];
                y[e] = gact(z, act, alpha);
            }
            if (c + 4 <= g.Cout && (g.Cout & 3) == 0) {
                *reinterpret_cast<float4*>(o + c) = make_float4(y[0], y[1], y[2], y[3]);
            } else {
                for (int e = 0; e < 4 && c + e < g.Cout; ++e) o[c + e] = y[e];
            }
        }
    }
}


// exact f32: one thread per (output pixel, 8 output channels); weights [Cout][kh][kw][Cin]
static __global__ __launch_bounds__(256) void gconv_f32(const float* __restrict__ in, const float* __restrict__ w,
                                                 const float* __restrict__ bias, float* __restrict__ out, ConvGeom g,
                                                 int act, float alpha) {
    const int n = blockIdx.z;
    const int P = blockIdx.x * 256 + threadIdx.x;
    const int c0 = blockIdx.y * 8;
    if (P >= g.Hout * g.Wout) return;
    const int oy = P / g.Wout, ox = P - (P / g.Wout) * g.Wout;
    const float* img = in + (size_t)n * g.Hin * g.Win * g.Cin;
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = c0 + c < g.Cout ? bias[c0 + c] : 0.f;
    for (int ky = 0; ky < g.kh; ++ky) {
        const int iy = oy * g.sh - g.pt + ky;
        if (iy < 0 || iy >= g.Hin) continue;
        for (int kx = 0; kx < g.kw; ++kx) {
            const int ix = ox * g.sw - g.pl + kx;
            if (ix < 0 || ix >= g.Win) continue;
            const float* px = img + ((size_t)iy * g.Win + ix) * g.Cin;
            const size_t wt = (size_t)(ky * g.kw + kx) * g.Cin;
            for (int ci = 0; ci < g.Cin; ++ci) {
                const float x = px[ci];
#pragma unroll
                for (int c = 0; c < 8; ++c)
                    if (c0 + c < g.Cout) acc[c] = fmaf(w[(size_t)(c0 + c) * g.kh * g.kw * g.Cin + wt + ci], x, acc[c]);
            }
        }
    }
    float* o = out + ((size_t)n * g.Hout * g.Wout + P) * g.Cout;
#pragma unroll
    for (int c = 0; c < 8; ++c)
        if (c0 + c < g.Cout) o[c0 + c] = gact(acc[c], act, alpha);
}

// exact f32 for small K = kh kw Cin (<= GF32_KMAX, e.g. a 3-channel stem):
// one thread per output pixel and 32 output channels (blockIdx.y), the
// group's weights staged once per block in LDS as [K][32] and read as
// broadcast float4s.  KH x KW x CI > 0: that shape at compile time -- the
// pixel's K inputs are all loaded up front (clamped addresses, zero outside
// the image), so their latency is paid once, not once per tap.  Each output is
// the same chain as gconv_f32 (bias, then fma over ky, kx, ci in order, taps
// outside the image skipped in both): the results are identical.
constexpr int GF32_KMAX = 96;  // 12 KiB of LDS
template <int KH = 0, int KW = 0, int CI = 0>
__global__ __launch_bounds__(256) void gconv_f32_lds(const float* __restrict__ in, const float* __restrict__ w,
                                                     const float* __restrict__ bias, float* __restrict__ out,
                                                     ConvGeom g, int act, float alpha) {
    __shared__ __attribute__((aligned(16))) float sw[GF32_KMAX * 32];
    const int n = blockIdx.z;
    const int c0 = blockIdx.y * 32;
    const int K = g.kh * g.kw * g.Cin;
    for (int i = threadIdx.x; i < K * 32; i += 256) {
        const int k = i >> 5, c = i & 31;
        sw[i] = c0 + c < g.Cout ? w[(size_t)(c0 + c) * K + k] : 0.f;
    }
    __syncthreads();
    const int P = blockIdx.x * 256 + threadIdx.x;
    if (P >= g.Hout * g.Wout) return;
    const int oy = P / g.Wout, ox = P - (P / g.Wout) * g.Wout;
    const float* img = in + (size_t)n * g.Hin * g.Win * g.Cin;
    float acc[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) acc[c] = c0 + c < g.Cout ? bias[c0 + c] : 0.f;
    auto fma32 = [&](float x, int k) {
        const float4* wk = reinterpret_cast<const float4*>(sw + k * 32);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float4 wv = wk[c];
            acc[4 * c + 0] = fmaf(wv.x, x, acc[4 * c + 0]);
            acc[4 * c + 1] = fmaf(wv.y, x, acc[4 * c + 1]);
            acc[4 * c + 2] = fmaf(wv.z, x, acc[4 * c + 2]);
            acc[4 * c + 3] = fmaf(wv.w, x, acc[4 * c + 3]);
        }
    };
    if constexpr (KH > 0) {
        float xv[KH * KW * CI];
        bool ok[KH * KW];
#pragma unroll
        for (int ky = 0; ky < KH; ++ky)
#pragma unroll
            for (int kx = 0; kx < KW; ++kx) {
                const int iy = oy * g.sh - g.pt + ky, ix = ox * g.sw - g.pl + kx;
                ok[ky * KW + kx] = iy >= 0 && iy < g.Hin && ix >= 0 && ix < g.Win;
                const int cy = min(max(iy, 0), g.Hin - 1), cx = min(max(ix, 0), g.Win - 1);
                const float* px = img + ((size_t)cy * g.Win + cx) * CI;
#pragma unroll
                for (int ci = 0; ci < CI; ++ci) xv[(ky * KW + kx) * CI + ci] = px[ci];
            }
#pragma unroll
        for (int t = 0; t < KH * KW; ++t)
            if (ok[t]) {
#pragma unroll
                for (int ci = 0; ci < CI; ++ci) fma32(xv[t * CI + ci], t * CI + ci);
            }
    } else {
        for (int ky = 0; ky < g.kh; ++ky) {
            const int iy = oy * g.sh - g.pt + ky;
            if (iy < 0 || iy >= g.Hin) continue;
            for (int kx = 0; kx < g.kw; ++kx) {
                const int ix = ox * g.sw - g.pl + kx;
                if (ix < 0 || ix >= g.Win) continue;
                const float* px = img + ((size_t)iy * g.Win + ix) * g.Cin;
                for (int ci = 0; ci < g.Cin; ++ci) fma32(px[ci], (ky * g.kw + kx) * g.Cin + ci);
            }
        }
    }
    float* o = out + ((size_t)n * g.Hout * g.Wout + P) * g.Cout;
    with_act(act, [&](auto actc) {
        constexpr int A = decltype(actc)::value;
        if ((g.Cout & 3) == 0 && c0 + 32 <= g.Cout) {
#pragma unroll
            for (int c = 0; c < 32; c += 4)
                *reinterpret_cast<float4*>(o + c0 + c) = make_float4(gact(acc[c], A, alpha), gact(acc[c + 1], A, alpha),
                                                                     gact(acc[c + 2], A, alpha),
                                                                     gact(acc[c + 3], A, alpha));
        } else {
#pragma unroll
            for (int c = 0; c < 32; ++c)
                if (c0 + c < g.Cout) o[c0 + c] = gact(acc[c], A, alpha);
        }
    });
}

// gconv_f32_s: the same conv for a compile-time KH x KW x CI (a 3-channel
// stem) with the weights in the scalar data path: ws = [C_out / 32][K][32]
// (zero-padded), read at wave-uniform addresses, so each FMA takes its weight
// from an SGPR -- no LDS staging, no LDS reads (gconv_f32_lds spends a
// ds_read_b128 per 4 FMAs).  The same chain per output as gconv_f32.
template <int KH, int KW, int CI>
__global__ __launch_bounds__(256) void gconv_f32_s(const float* __restrict__ in, const float* __restrict__ ws,
                                                   const float* __restrict__ bias, float* __restrict__ out,
                                                   ConvGeom g, int act, float alpha) {
    constexpr int K = KH * KW * CI;
    const int n = blockIdx.z;
    const int c0 = blockIdx.y * 32;
    const float* wq = ws + (size_t)blockIdx.y * K * 32;
    const int P = blockIdx.x * 256 + threadIdx.x;
    if (P >= g.Hout * g.Wout) return;
    const int oy = P / g.Wout, ox = P - (P / g.Wout) * g.Wout;
    const float* img = in + (size_t)n * g.Hin * g.Win * CI;
    float xv[K];
    bool ok[KH * KW];
#pragma unroll
    for (int ky = 0; ky < KH; ++ky)
#pragma unroll
        for (int kx = 0; kx < KW; ++kx) {
            const int iy = oy * g.sh - g.pt + ky, ix = ox * g.sw - g.pl + kx;
            ok[ky * KW + kx] = iy >= 0 && iy < g.Hin && ix >= 0 && ix < g.Win;
            const int cy = min(max(iy, 0), g.Hin - 1), cx = min(max(ix, 0), g.Win - 1);
            const float* px = img + ((size_t)cy * g.Win + cx) * CI;
#pragma unroll
            for (int ci = 0; ci < CI; ++ci) xv[(ky * KW + kx) * CI + ci] = px[ci];
        }
    float acc[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) acc[c] = c0 + c < g.Cout ? bias[c0 + c] : 0.f;
#pragma unroll
    for (int t = 0; t < KH * KW; ++t)
        if (ok[t]) {
#pragma unroll
            for (int ci = 0; ci < CI; ++ci)
#pragma unroll
                for (int c = 0; c < 32; ++c) acc[c] = fmaf(wq[(t * CI + ci) * 32 + c], xv[t * CI + ci], acc[c]);
        }
    float* o = out + ((size_t)n * g.Hout * g.Wout + P) * g.Cout;
    with_act(act, [&](auto actc) {
        constexpr int A = decltype(actc)::value;
        if ((g.Cout & 3) == 0 && c0 + 32 <= g.Cout) {
#pragma unroll
            for (int c = 0; c < 32; c += 4)
                *reinterpret_cast<float4*>(o + c0 + c) = make_float4(gact(acc[c], A, alpha), gact(acc[c + 1], A, alpha),
                                                                     gact(acc[c + 2], A, alpha),
                                                                     gact(acc[c + 3], A, alpha));
        } else {
#pragma unroll
            for (int c = 0; c < 32; ++c)
                if (c0 + c < g.Cout) o[c0 + c] = gact(acc[c], A, alpha);
        }
    });
}

// max / average pooling with explicit padding (average over the taps inside
// the image: TF's "same"-padded AvgPool excludes the padding); one thread per
// (output pixel, channel)
static __global__ __launch_bounds__(256) void gpool2d(const float* __restrict__ in, float* __restrict__ out, int Hin, int Win,
                                               int C, int Hout, int Wout, int kh, int kw, int sh, int sw, int pt,
                                               int pl, int avg, int act, float alpha) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const int n = blockIdx.y;
    if (i >= (size_t)Hout * Wout * C) return;
    const int c = (int)(i % C);
    const int P = (int)(i / C);
    const int oy = P / Wout, ox = P - (P / Wout) * Wout;
    const float* img = in + (size_t)n * Hin * Win * C;
    float m = avg ? 0.f : -INFINITY;
    int cnt = 0;
    for (int ky = 0; ky < kh; ++ky) {
        const int iy = oy * sh - pt + ky;
        if (iy < 0 || iy >= Hin) continue;
        for (int kx = 0; kx < kw; ++kx) {
            const int ix = ox * sw - pl + kx;
            if (ix < 0 || ix >= Win) continue;
            const float v = img[((size_t)iy * Win + ix) * C + c];
            m = avg ? m + v : fmaxf(m, v);
            ++cnt;
        }
    }
    if (avg) m = cnt ? m / (float)cnt : 0.f;
    out[(size_t)n * Hout * Wout * C + i] = gact(m, act, alpha);
}

// host: split-bf16 weight packing for gconv_x3 from a compact f32 [tap][Cout][Cin]
// image (BN already folded): [tap][cin_pad/32][cout_pad][32 hi | 32 lo]
static inline uint16_t g_f2bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
    u += 0x7fff + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}
static inline float g_bf2f(uint16_t b) {
    const uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static inline std::vector<uint16_t> gconv_pack_x3(const std::vector<float>& w_tco, int ntap, int cout, int cin,
                                                  int cout_pad, int cin_pad) {
    const int ncc = cin_pad / 32;
    std::vector<uint16_t> h((size_t)ntap * ncc * cout_pad * 64, 0);
    for (int t = 0; t < ntap; ++t)
        for (int o = 0; o < cout; ++o)
            for (int c = 0; c < cin; ++c) {
                const float w = w_tco[((size_t)t * cout + o) * cin + c];
                const uint16_t hi = g_f2bf(w);
                const size_t row = ((size_t)(t * ncc + c / 32) * cout_pad + o) * 64;
                h[row + c % 32] = hi;
                h[row + 32 + c % 32] = g_f2bf(w - g_bf2f(hi));
            }
    return h;
}

}  // namespace aa
