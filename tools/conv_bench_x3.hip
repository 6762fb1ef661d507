// Diagnostic harness: time split-bf16 (bf16x3) conv_x3 tilings of model1's
// layers at T = 226 on random f32 activations, 64 windows per launch.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include
//   tools/conv_bench_x3.hip audio-analysis_amd/csrc/aa_api.cpp -o tools/conv_bench_x3 ; run on the GPU box.
#include "../audio-analysis_amd/csrc/aa_cnn.hip"
#include "conv_wgp.h"  // the rejected plane-split Winograd conv (profiles/r06/wgp_rejected.txt)

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace aa;

template <int KH, int KW, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW, bool FUSED,
          int DIAG = 0, bool RING = true, bool AJIT = false, int OCC = 0, bool IS = false, bool OS = false>
static void time_one(const char* tag, int n, int Hin, int Win, int cout, const void* in, const void* w,
                     const float* b, void* out, FirstConv fc, int iters) {
    auto k = conv_x3<KH, KW, CIN, WM, WN, MF, NF, POOL, TH, TW, FUSED, DIAG, RING, AJIT, OCC, IS, OS>;
    constexpr int BN = WN * NF * 16;
    const size_t lds = x3_lds_bytes<KH, KW, CIN, BN, TH, TW, FUSED, RING>();
    if (lds > 160 * 1024) {
        printf("%-8s %dx%d cin %3d WM%d WN%d MF%2d NF%d %2dx%2d  LDS %zu: skip\n", tag, KH, KW, CIN, WM, WN, MF, NF,
               TH, TW, lds);
        return;
    }
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int Hc = Hin - KH + 1, Wc = Win - KW + 1;
    const int Hout = Hc / POOL, Wout = Wc / POOL;
    const int tiles_h = (Hout * POOL + TH - 1) / TH, tiles_w = (Wout * POOL + TW - 1) / TW;
    dim3 grid(tiles_h * tiles_w, cout / BN, n);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(k, grid, dim3(WM * WN * 64), lds, 0, (const float*)in, Hin, Win, (const bf16*)w, b,
                           (float*)out, Hout, Wout, cout, tiles_w, 1, 0.3f, fc);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(k, grid, dim3(WM * WN * 64), lds, 0, (const float*)in, Hin, Win, (const bf16*)w, b,
                           (float*)out, Hout, Wout, cout, tiles_w, 1, 0.3f, fc);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const float us = 1e3f * ms / iters;
    double fl = 2.0 * n * Hc * Wc * KH * KW * CIN * cout;
    if (FUSED) fl += 2.0 * n * (Hin) * (Win) * 9 * 32;
    printf("%-8s%s%s%s%d %dx%d cin %3d WM%d WN%d MF%2d NF%d %2dx%2d  LDS %6zu  grid %6d  %7.1f us  %6.1f TF (%.3f of 833)\n",
           tag, IS ? "S" : "", RING ? "" : "G", AJIT ? "J" : "", OCC, KH, KW, CIN, WM, WN, MF, NF, TH, TW, lds, grid.x * grid.y * grid.z, us, fl / us * 1e-6,
           fl / us * 1e-6 / 833.3);
}

template <int KH, int CIN, int WM, int WN, int MF, int NF, int POOL, int TH, int TW, int OCC, bool IS, bool OS,
          int DIAG = 0, int WO = 2, int NPASS = 1>
static void time_wg(const char* tag, int n, int Hin, int Win, int cout, const void* in, const void* w, const float* b,
                    void* out, int iters) {
    auto k = conv_wg<KH, CIN, WM, WN, MF, NF, POOL, TH, TW, OCC, IS, OS, DIAG, WO, NPASS>;
    constexpr int BN = WN * NF * 16;
    const size_t lds = wg_lds_bytes<KH, BN, TH, TW, WO, NPASS, WN>();
    if (lds > 160 * 1024) { printf("%s LDS %zu: skip\n", tag, lds); return; }
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int Hc = Hin - KH + 1, Wc = Win - 3 + 1;
    const int Hout = Hc / POOL, Wout = Wc / POOL;
    const int tiles_h = (Hout * POOL + TH - 1) / TH, tiles_w = (Wout * POOL + TW - 1) / TW;
    dim3 grid(tiles_h * tiles_w, cout / BN, n);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(k, grid, dim3(WM * WN * 64), lds, 0, (const float*)in, Hin, Win, (const bf16*)w, b,
                           (float*)out, Hout, Wout, cout, tiles_w, 1, 0.3f);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(k, grid, dim3(WM * WN * 64), lds, 0, (const float*)in, Hin, Win, (const bf16*)w, b,
                           (float*)out, Hout, Wout, cout, tiles_w, 1, 0.3f);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const float us = 1e3f * ms / iters;
    const double fl = 2.0 * n * Hc * Wc * KH * 3 * CIN * cout;
    printf("%-6s wg%d d%d %dx3 cin %3d WM%d WN%d MF%d NF%d %2dx%2d occ%d LDS %6zu grid %6d  %7.1f us  %6.1f TF (%.3f of 833)\n",
           tag, WO, DIAG, KH, CIN, WM, WN, MF, NF, TH, TW, OCC, lds, grid.x * grid.y * grid.z, us, fl / us * 1e-6,
           fl / us * 1e-6 / 833.3);
}

int main(int argc, char** argv) {
    const int n = 64, it = 20;
    std::vector<float> h(100u << 20);  // 400 MB of f32 activations: larger than every layer's input
    for (auto& x : h) x = 1.f + (rand() & 0xffff) / 65536.f;
    std::vector<uint16_t> hw(4u << 20);
    for (auto& x : hw) x = 0x3c00 + (rand() & 0x3ff);  // bf16 ~0.0078..0.0156
    void *in, *w, *out;
    float* b;
    (void)hipMalloc(&in, h.size() * 4);
    (void)hipMalloc(&w, hw.size() * 2);
    (void)hipMalloc(&out, 400u << 20);
    (void)hipMalloc(&b, 8192);
    (void)hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemset(b, 0, 8192);
    FirstConv fc{};
    float *w1, *b1;
    (void)hipMalloc(&w1, 32 * 9 * 4);
    (void)hipMalloc(&b1, 32 * 4);
    std::vector<float> hw1(32 * 9, 0.05f), hb1(32, 0.01f);
    (void)hipMemcpy(w1, hw1.data(), hw1.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(b1, hb1.data(), hb1.size() * 4, hipMemcpyHostToDevice);
    FirstConv f1{w1, b1, 1, 0.3f, 0, 1.f, 160, 226};
    const int which = argc > 1 ? atoi(argv[1]) : 0;  // 0: all layers, 9: ablations
    if (which == 9) {
        // DIAG bits (aa_cnn.hip): 1 no staging, 4 no stores, 32 no weight stream,
        // 128 no fragment reads after the first, 2 no MFMA loop
#define ABL5(D) time_one<9, 3, 64, 4, 2, 4, 4, 3, 39, 6, false, D, false, true, 2>("c5 d" #D, n, 48, 70, 128, in, w, b, out, fc, it);
#define ABL2(D) time_one<3, 3, 32, 4, 1, 4, 2, 3, 12, 21, true, D, false, true, 0>("c2 d" #D, n, 158, 224, 32, in, w, b, out, f1, it);
#define ABL4(D) time_one<3, 3, 64, 4, 2, 3, 2, 1, 12, 14, false, D, true, true, 4>("c4 d" #D, n, 50, 72, 64, in, w, b, out, fc, it);
#define ABL3(D) time_one<3, 3, 32, 4, 2, 3, 2, 1, 10, 18, false, D, true, false, 0>("c3 d" #D, n, 52, 74, 64, in, w, b, out, fc, it);
        ABL5(0) ABL5(1) ABL5(2) ABL5(4) ABL5(5) ABL5(33) ABL5(161) ABL5(165) ABL5(37)
        ABL2(0) ABL2(2) ABL2(64) ABL2(512) ABL2(576) ABL2(4) ABL2(1) ABL2(5)
        ABL4(0) ABL4(1) ABL4(2) ABL4(4) ABL4(5) ABL4(33) ABL4(161) ABL4(165)
        ABL3(0) ABL3(1) ABL3(2) ABL3(5) ABL3(165)
        return 0;
    }
    // model1 at T = 226: (Hin, Win) of each conv's input
#define C2(WM, WN, MF, NF, TH, TW) time_one<3, 3, 32, WM, WN, MF, NF, 3, TH, TW, true>("c1+c2", n, 158, 224, 32, in, w, b, out, f1, it);
#define C3(WM, WN, MF, NF, TH, TW) time_one<3, 3, 32, WM, WN, MF, NF, 1, TH, TW, false>("c3", n, 52, 74, 64, in, w, b, out, fc, it);
#define C4(WM, WN, MF, NF, TH, TW) time_one<3, 3, 64, WM, WN, MF, NF, 1, TH, TW, false>("c4", n, 50, 72, 64, in, w, b, out, fc, it);
#define C5(WM, WN, MF, NF, TH, TW) time_one<9, 3, 64, WM, WN, MF, NF, 3, TH, TW, false>("c5", n, 48, 70, 128, in, w, b, out, fc, it);
#define G2(WM, WN, MF, NF, TH, TW) time_one<3, 3, 32, WM, WN, MF, NF, 3, TH, TW, true, 0, false>("c1+c2", n, 158, 224, 32, in, w, b, out, f1, it);
#define G3(WM, WN, MF, NF, TH, TW) time_one<3, 3, 32, WM, WN, MF, NF, 1, TH, TW, false, 0, false>("c3", n, 52, 74, 64, in, w, b, out, fc, it);
#define G4(WM, WN, MF, NF, TH, TW) time_one<3, 3, 64, WM, WN, MF, NF, 1, TH, TW, false, 0, false>("c4", n, 50, 72, 64, in, w, b, out, fc, it);
#define G5(WM, WN, MF, NF, TH, TW) time_one<9, 3, 64, WM, WN, MF, NF, 3, TH, TW, false, 0, false>("c5", n, 48, 70, 128, in, w, b, out, fc, it);
#define G6(WM, WN, MF, NF, TH, TW) time_one<1, 3, 128, WM, WN, MF, NF, 1, TH, TW, false, 0, false>("c6", n, 13, 22, 256, in, w, b, out, fc, it);
#define J2(WM, WN, MF, NF, TH, TW, R, O) time_one<3, 3, 32, WM, WN, MF, NF, 3, TH, TW, true, 0, R, true, O>("c1+c2", n, 158, 224, 32, in, w, b, out, f1, it);
#define J3(WM, WN, MF, NF, TH, TW, R, O) time_one<3, 3, 32, WM, WN, MF, NF, 1, TH, TW, false, 0, R, true, O>("c3", n, 52, 74, 64, in, w, b, out, fc, it);
#define J4(WM, WN, MF, NF, TH, TW, R, O) time_one<3, 3, 64, WM, WN, MF, NF, 1, TH, TW, false, 0, R, true, O>("c4", n, 50, 72, 64, in, w, b, out, fc, it);
#define J5(WM, WN, MF, NF, TH, TW, R, O) time_one<9, 3, 64, WM, WN, MF, NF, 3, TH, TW, false, 0, R, true, O>("c5", n, 48, 70, 128, in, w, b, out, fc, it);
#define J6(WM, WN, MF, NF, TH, TW, R, O) time_one<1, 3, 128, WM, WN, MF, NF, 1, TH, TW, false, 0, R, true, O>("c6", n, 13, 22, 256, in, w, b, out, fc, it);
#define C6(WM, WN, MF, NF, TH, TW) time_one<1, 3, 128, WM, WN, MF, NF, 1, TH, TW, false>("c6", n, 13, 22, 256, in, w, b, out, fc, it);
    // pre-split input / output (IN_SPLIT, OUT_SPLIT): the shipped pipeline's c3..c6
#define S3(WM, WN, MF, NF, TH, TW, R, J, O) time_one<3, 3, 32, WM, WN, MF, NF, 1, TH, TW, false, 0, R, J, O, true, true>("c3", n, 52, 74, 64, in, w, b, out, fc, it);
#define S4(WM, WN, MF, NF, TH, TW, R, J, O) time_one<3, 3, 64, WM, WN, MF, NF, 1, TH, TW, false, 0, R, J, O, true, true>("c4", n, 50, 72, 64, in, w, b, out, fc, it);
#define S5(WM, WN, MF, NF, TH, TW, R, J, O) time_one<9, 3, 64, WM, WN, MF, NF, 3, TH, TW, false, 0, R, J, O, true, true>("c5", n, 48, 70, 128, in, w, b, out, fc, it);
#define S6(WM, WN, MF, NF, TH, TW, R, J, O) time_one<1, 3, 128, WM, WN, MF, NF, 1, TH, TW, false, 0, R, J, O, true, false>("c6", n, 13, 22, 256, in, w, b, out, fc, it);
    if (which == 11) {
        S5(4, 2, 4, 4, 39, 6, false, true, 2) S5(4, 1, 4, 4, 39, 6, false, true, 2) S5(4, 1, 4, 4, 39, 6, false, true, 0)
        S5(4, 1, 4, 4, 39, 6, true, true, 2) S5(4, 2, 4, 4, 39, 6, true, true, 2) S5(4, 2, 4, 2, 39, 6, false, true, 4)
        S5(4, 2, 4, 2, 39, 6, true, true, 4) S5(4, 1, 4, 2, 39, 6, false, true, 4) S5(2, 2, 4, 4, 21, 6, false, true, 2)
        S5(8, 2, 2, 4, 39, 6, false, true, 2) S5(4, 2, 4, 4, 42, 6, false, true, 2) S5(4, 2, 6, 4, 39, 9, false, true, 2)
        S4(4, 2, 3, 2, 12, 14, true, true, 4) S4(4, 2, 3, 2, 12, 14, false, true, 4) S4(4, 2, 4, 2, 16, 14, true, true, 4)
        S4(4, 2, 4, 2, 16, 14, true, true, 0) S4(4, 1, 3, 4, 12, 14, true, true, 4) S4(4, 2, 6, 2, 24, 14, true, true, 0)
        S4(4, 2, 3, 2, 8, 24, true, true, 4) S4(2, 2, 3, 2, 8, 12, true, true, 4)
        S3(4, 2, 3, 2, 10, 18, true, false, 0) S3(4, 2, 3, 2, 10, 18, true, true, 4) S3(4, 2, 4, 2, 10, 24, true, true, 4)
        S3(4, 2, 3, 2, 12, 16, true, true, 4) S3(4, 1, 3, 4, 12, 16, true, true, 4) S3(2, 2, 3, 2, 8, 12, true, true, 4)
        S6(4, 2, 3, 2, 7, 20, true, false, 0) S6(4, 2, 3, 2, 7, 20, true, true, 4) S6(4, 2, 5, 2, 13, 20, true, true, 0)
        S6(4, 1, 3, 4, 7, 20, true, false, 0) S6(2, 2, 3, 2, 7, 12, true, true, 4) S6(4, 2, 3, 2, 7, 20, false, true, 4)
        return 0;
    }
#define F2(WM, WN, MF, NF, TH, TW, R, O) time_one<3, 3, 32, WM, WN, MF, NF, 3, TH, TW, true, 0, R, true, O, false, true>("c1+c2", n, 158, 224, 32, in, w, b, out, f1, it);
#define W5(WM, WN, MF, NF, TH, TW, O, D) time_wg<9, 64, WM, WN, MF, NF, 3, TH, TW, O, true, true, D>("c5", n, 48, 70, 128, in, w, b, out, it);
#define W4(WM, WN, MF, NF, TH, TW, O, D) time_wg<3, 64, WM, WN, MF, NF, 1, TH, TW, O, true, true, D>("c4", n, 50, 72, 64, in, w, b, out, it);
#define W3(WM, WN, MF, NF, TH, TW, O, D) time_wg<3, 32, WM, WN, MF, NF, 1, TH, TW, O, true, true, D>("c3", n, 52, 74, 64, in, w, b, out, it);
#define W6(WM, WN, MF, NF, TH, TW, O, D) time_wg<1, 128, WM, WN, MF, NF, 1, TH, TW, O, true, false, D>("c6", n, 13, 22, 256, in, w, b, out, it);
    if (which == 19) {  // the shipped split-bf16 tiles (aa_cnn.hip AA_X3_CFGS / AA_WG_CFGS), then fused-kernel ablations
#define FS(D) time_one<3, 3, 32, 4, 1, 4, 2, 3, 12, 21, true, D, false, true, 0, false, true>("c1+c2 d" #D, n, 158, 224, 32, in, w, b, out, f1, it);
        FS(0) S3(4, 2, 3, 2, 10, 18, true, false, 4) S4(2, 2, 3, 2, 12, 8, true, true, 0)
        W5(2, 2, 4, 2, 39, 6, 2, 0) S6(2, 2, 3, 2, 7, 12, true, true, 0)
        FS(2) FS(64) FS(4) FS(128) FS(16) FS(512) FS(576) FS(0)
        return 0;
    }
    if (which == 30) {  // Winograd 9x3: F(2,3) (round 4) vs F(6,3) (round 5), ablations (1 no staging, 2 no MFMA)
#define W5O(WM, WN, MF, NF, TH, TW, O, D, WO) time_wg<9, 64, WM, WN, MF, NF, 3, TH, TW, O, true, true, D, WO>("c5", n, 48, 70, 128, in, w, b, out, it);
        W5O(2, 2, 4, 2, 39, 6, 2, 0, 2) W5O(1, 4, 3, 1, 39, 6, 2, 0, 6)
        W5O(2, 2, 4, 2, 39, 6, 2, 1, 2) W5O(1, 4, 3, 1, 39, 6, 2, 1, 6)
        W5O(2, 2, 4, 2, 39, 6, 2, 2, 2) W5O(1, 4, 3, 1, 39, 6, 2, 2, 6)
        W5O(2, 2, 4, 2, 39, 6, 2, 3, 2) W5O(1, 4, 3, 1, 39, 6, 2, 3, 6)
        W5O(1, 4, 3, 1, 39, 6, 0, 0, 6) W5O(1, 4, 3, 1, 39, 6, 3, 0, 6)
        return 0;
    }
    if (which == 31) {  // the shipped F(6,3) 9x3 tile (f32 in, split out): full, no staging, no MFMA steps (PMC)
#define W5S(D) time_wg<9, 64, 1, 4, 3, 1, 3, 39, 6, 0, false, true, D, 6>("c5", n, 48, 70, 128, in, w, b, out, 2);
        W5S(0) W5S(1) W5S(2) W5S(3)
        return 0;
    }
    if (which == 34) {  // conv_wg vs conv_wgp ablations: 1 no staging, 2 no MFMA steps
#define WGA(D) time_wg<9, 64, 1, 4, 3, 1, 3, 39, 6, 0, false, true, D, 6>("c5", n, 48, 70, 128, in, w, b, out, it);
#define WGPA(D) WGPX(4, 0, D)
#define WGPX(NWV, OCCV, D)                                                                                        \
        {                                                                                                         \
            auto k1 = conv_wgp<9, 64, NWV, 3, 4, 3, 39, 6, OCCV, false, true, D, 6, 2>;                          \
            const size_t l1 = wgp_lds_bytes<9, 39, 6, 6, 3>();                                                   \
            (void)hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l1);     \
            dim3 grid(11, 2, n);                                                                              \
            for (int i = 0; i < 3; ++i)                                                                           \
                hipLaunchKernelGGL(k1, grid, dim3(64 * NWV), l1, 0, (const float*)in, 48, 70, (const bf16*)w, b, (float*)out, 13, 22, 128, 11, 1, 0.3f); \
            hipEvent_t e0, e1;                                                                                    \
            (void)hipEventCreate(&e0);                                                                            \
            (void)hipEventCreate(&e1);                                                                            \
            (void)hipEventRecord(e0, 0);                                                                          \
            for (int i = 0; i < it; ++i)                                                                          \
                hipLaunchKernelGGL(k1, grid, dim3(64 * NWV), l1, 0, (const float*)in, 48, 70, (const bf16*)w, b, (float*)out, 13, 22, 128, 11, 1, 0.3f); \
            (void)hipEventRecord(e1, 0);                                                                          \
            (void)hipEventSynchronize(e1);                                                                        \
            float ms = 0;                                                                                         \
            (void)hipEventElapsedTime(&ms, e0, e1);                                                               \
            printf("wgp nw%d occ%d d%d %7.1f us\n", NWV, OCCV, D, 1e3f * ms / it);                                                      \
        }
        for (int r = 0; r < 2; ++r) {
            WGA(0) WGPA(0) WGPX(8, 0, 0) WGPX(8, 4, 0) WGA(1) WGPA(1) WGPX(8, 0, 1) WGA(2) WGPA(2) WGPX(8, 0, 2) WGA(3) WGPA(3)
        }
        return 0;
    }
    if (which == 32 || which == 33) {  // conv_wg (channel split) vs conv_wgp (plane split): outputs compared, then timed
        const int iters = which == 33 ? 2 : it;
        const int Hin = 48, Win = 70, cout = 128, Hc = Hin - 8, Wc = Win - 2, Hout = Hc / 3, Wout = Wc / 3;
        const int tiles_h = (Hout * 3 + 38) / 39, tiles_w = (Wout * 3 + 5) / 6;
        const size_t on = (size_t)n * Hout * Wout * cout;
        void* out2;
        (void)hipMalloc(&out2, on * 4);
        auto k0 = conv_wg<9, 64, 1, 4, 3, 1, 3, 39, 6, 0, false, true, 0, 6, 1, 2>;
        auto k1 = conv_wgp<9, 64, 4, 3, 4, 3, 39, 6, 0, false, true, 0, 6, 2>;
        const size_t l0 = wg_lds_bytes<9, 64, 39, 6, 6, 1, 4>(), l1 = wgp_lds_bytes<9, 39, 6, 6, 3>();
        (void)hipFuncSetAttribute((const void*)k0, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l0);
        (void)hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l1);
        dim3 grid(tiles_h * tiles_w, cout / 64, n);
        auto r0 = [&](void* o) { hipLaunchKernelGGL(k0, grid, dim3(256), l0, 0, (const float*)in, Hin, Win, (const bf16*)w, b, (float*)o, Hout, Wout, cout, tiles_w, 1, 0.3f); };
        auto r1 = [&](void* o) { hipLaunchKernelGGL(k1, grid, dim3(256), l1, 0, (const float*)in, Hin, Win, (const bf16*)w, b, (float*)o, Hout, Wout, cout, tiles_w, 1, 0.3f); };
        (void)hipMemset(out, 0xff, on * 4);
        (void)hipMemset(out2, 0xee, on * 4);
        r0(out);
        r1(out2);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 2; }
        std::vector<uint32_t> a(on), c(on);
        (void)hipMemcpy(a.data(), out, on * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(c.data(), out2, on * 4, hipMemcpyDeviceToHost);
        size_t nd = 0;
        for (size_t i = 0; i < on; ++i) nd += a[i] != c[i];
        printf("LDS wg %zu wgp %zu: %zu of %zu output words differ\n", l0, l1, nd, on);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        for (int round = 0; round < 3; ++round)
            for (int v = 0; v < 2; ++v) {
                for (int i = 0; i < 2; ++i) v ? r1(out2) : r0(out);
                (void)hipEventRecord(e0, 0);
                for (int i = 0; i < iters; ++i) v ? r1(out2) : r0(out);
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                printf("%s %7.1f us\n", v ? "conv_wgp (plane split)  " : "conv_wg (channel split) ", 1e3f * ms / iters);
            }
        return nd ? 1 : 0;
    }
    if (which == 21) {  // the shipped fused kernel, three timings (variant A/B across builds)
        FS(0) FS(0) FS(0)
        return 0;
    }
    if (which == 22) {  // per-wave phase timestamps of the shipped fused kernel -> gpurun_out/fused_ts.bin
        FS(0)
        const size_t cnt = (size_t)9152 * 4 * 10;
        std::vector<unsigned long long> ts(cnt);
#define TSD(D)                                                                                                        \
        time_one<3, 3, 32, 4, 1, 4, 2, 3, 12, 21, true, 4096 | D, false, true, 0, false, true>("c1+c2 ts" #D, n, 158, 224, 32, in, w, b, out, f1, 1); \
        (void)hipMemcpy(ts.data(), (char*)out + (64u << 22), cnt * 8, hipMemcpyDeviceToHost);                         \
        { FILE* f = fopen("gpurun_out/fused_ts_" #D ".bin", "wb"); fwrite(ts.data(), 8, cnt, f); fclose(f); }
        TSD(0) TSD(8192) TSD(16384) TSD(32768) TSD(57344) TSD(64) TSD(2)
        return 0;
    }
    if (which == 20) {  // the shipped fused kernel once (PMC passes)
        time_one<3, 3, 32, 4, 1, 4, 2, 3, 12, 21, true, 0, false, true, 0, false, true>("c1+c2", n, 158, 224, 32, in, w, b, out, f1, 1);
        W5(2, 2, 4, 2, 39, 6, 2, 0)
        return 0;
    }
    if (which == 18) {  // LDS bank conflicts of the fused kernel by phase (PMC): full, no conv1 compute, no MFMA loop
        ABL2(66) ABL2(70) ABL2(578) ABL2(582)
        return 0;
    }
    if (which == 17) {  // the shipped fused first conv and Winograd 9x3 once each (PMC passes)
        time_one<3, 3, 32, 4, 1, 3, 2, 3, 9, 21, true, 0, false, true, 4, false, true>("c2", n, 158, 224, 32, in, w, b, out, f1, 1);
        W5(2, 2, 4, 2, 39, 6, 2, 0)
        return 0;
    }
    if (which == 16) {  // the fused first conv: B latency (16: weights of step 0 re-read, L1-resident)
        ABL2(0) ABL2(16) ABL2(128) ABL2(144) ABL2(1) ABL2(17) ABL2(2)
        return 0;
    }
    if (which == 15) {  // the shipped 9x3 Winograd tile: staging / MFMA ablations
        W5(2, 2, 4, 2, 39, 6, 2, 0) W5(2, 2, 4, 2, 39, 6, 2, 1) W5(2, 2, 4, 2, 39, 6, 2, 2) W5(2, 2, 4, 2, 39, 6, 2, 3)
        C5(2, 2, 4, 2, 21, 6)
        return 0;
    }
    if (which == 14) {
        W5(2, 2, 2, 2, 21, 6, 0, 0) W5(2, 2, 2, 2, 21, 6, 0, 1) W5(2, 2, 2, 2, 21, 6, 0, 2) W5(2, 2, 2, 2, 21, 6, 0, 3)
        W5(2, 2, 4, 2, 39, 6, 0, 0) W5(2, 2, 4, 2, 39, 6, 2, 0) W5(4, 1, 2, 4, 21, 6, 0, 0) W5(2, 2, 2, 4, 21, 6, 0, 0)
        W5(1, 2, 4, 2, 21, 6, 0, 0) W5(2, 1, 2, 4, 21, 6, 0, 0) W5(2, 2, 2, 2, 21, 6, 2, 0) W5(2, 2, 2, 2, 21, 6, 4, 0)
        W5(4, 2, 2, 2, 39, 6, 0, 0) W5(2, 2, 3, 2, 15, 12, 0, 0)
        W4(2, 2, 2, 2, 8, 16, 0, 0) W4(2, 2, 2, 2, 8, 16, 0, 1) W4(2, 2, 2, 2, 8, 16, 0, 2) W4(2, 2, 3, 2, 12, 16, 0, 0)
        W4(2, 2, 4, 2, 16, 16, 0, 0) W4(2, 2, 2, 2, 4, 32, 0, 0) W4(4, 2, 2, 2, 16, 16, 0, 0) W4(2, 2, 4, 2, 8, 32, 0, 0)
        W3(2, 2, 2, 2, 8, 16, 0, 0) W3(2, 2, 2, 2, 8, 16, 0, 1) W3(2, 2, 2, 2, 8, 16, 0, 2) W3(2, 2, 3, 2, 12, 16, 0, 0)
        W3(2, 2, 4, 2, 16, 16, 0, 0) W3(4, 2, 2, 2, 16, 16, 0, 0) W3(2, 2, 4, 2, 8, 32, 0, 0)
        W6(2, 2, 2, 2, 13, 8, 0, 0) W6(2, 2, 5, 2, 13, 20, 0, 0) W6(2, 2, 3, 2, 13, 12, 0, 0) W6(1, 2, 4, 2, 13, 8, 0, 0)
        return 0;
    }
    if (which == 13) {
        // data dependence: the same tiles on random bit patterns (the default
        // fill) and on properly split N(0,1) activations / N(0,0.05) weights
        S5(2, 2, 4, 2, 21, 6, false, true, 4) S5(4, 2, 4, 4, 39, 6, false, true, 2) S4(2, 2, 3, 2, 12, 8, true, true, 4)
        F2(4, 1, 3, 2, 9, 21, false, 4)
        std::vector<uint16_t> hs(h.size() * 2), ws(hw.size());
        unsigned st = 1;
        auto gauss = [&]() {
            float a = 0;
            for (int k = 0; k < 4; ++k) { st = st * 1664525u + 1013904223u; a += (st >> 8) * (1.f / 16777216.f) - 0.5f; }
            return a * 1.7f;
        };
        auto split = [](float x, uint16_t& hi, uint16_t& lo) {
            uint32_t u; memcpy(&u, &x, 4);
            uint32_t r = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
            float hf; memcpy(&hf, &r, 4);
            float l = x - hf; uint32_t v; memcpy(&v, &l, 4);
            v = (v + 0x7fff + ((v >> 16) & 1)) >> 16;
            hi = (uint16_t)(r >> 16); lo = (uint16_t)v;
        };
        // grouped split: per 32 channels 32 hi then 32 lo
        for (size_t px = 0; px < hs.size() / 64; ++px)
            for (int c = 0; c < 32; ++c) split(gauss(), hs[px * 64 + c], hs[px * 64 + 32 + c]);
        for (size_t r = 0; r < ws.size() / 64; ++r)
            for (int c = 0; c < 32; ++c) split(0.05f * gauss(), ws[r * 64 + c], ws[r * 64 + 32 + c]);
        (void)hipMemcpy(in, hs.data(), std::min(hs.size() * 2, h.size() * 4), hipMemcpyHostToDevice);
        (void)hipMemcpy(w, ws.data(), ws.size() * 2, hipMemcpyHostToDevice);
        printf("-- split N(0,1) data --\n");
        S5(2, 2, 4, 2, 21, 6, false, true, 4) S5(4, 2, 4, 4, 39, 6, false, true, 2) S4(2, 2, 3, 2, 12, 8, true, true, 4)
        F2(4, 1, 3, 2, 9, 21, false, 4)
        return 0;
    }
    if (which == 12) {
        S5(2, 2, 4, 4, 21, 6, false, true, 2) S5(2, 2, 4, 4, 21, 6, false, true, 0) S5(2, 2, 4, 4, 21, 6, false, true, 3)
        S5(2, 2, 4, 4, 21, 6, true, true, 2) S5(2, 2, 5, 4, 24, 6, false, true, 2) S5(2, 2, 3, 4, 15, 6, false, true, 2)
        S5(2, 2, 4, 2, 21, 6, false, true, 4) S5(4, 1, 2, 4, 21, 6, false, true, 4) S5(2, 1, 4, 8, 21, 6, false, true, 2)
        S5(2, 2, 8, 4, 39, 6, false, true, 2) S5(2, 2, 8, 4, 39, 6, false, true, 1) S5(2, 1, 4, 4, 21, 6, false, true, 4)
        S5(1, 2, 8, 4, 21, 6, false, true, 2) S5(2, 2, 4, 4, 21, 6, false, false, 2) S5(2, 4, 4, 2, 21, 6, false, true, 2)
        S4(2, 2, 3, 2, 8, 12, true, true, 4) S4(2, 2, 3, 2, 8, 12, true, true, 0) S4(2, 2, 3, 2, 8, 12, false, true, 4)
        S4(2, 2, 4, 2, 8, 16, true, true, 4) S4(2, 2, 3, 2, 6, 16, true, true, 4) S4(2, 2, 2, 2, 4, 16, true, true, 4)
        S4(2, 1, 3, 4, 8, 12, true, true, 4) S4(2, 2, 3, 2, 12, 8, true, true, 4) S4(2, 2, 4, 2, 10, 12, true, true, 4)
        S3(2, 2, 3, 2, 8, 12, true, true, 0) S3(2, 2, 3, 2, 8, 12, true, false, 0) S3(2, 2, 4, 2, 8, 16, true, false, 0)
        S3(2, 2, 3, 2, 6, 16, true, false, 0) S3(2, 2, 2, 2, 4, 16, true, false, 0) S3(4, 2, 3, 2, 10, 18, true, false, 4)
        S3(2, 2, 4, 2, 10, 12, true, false, 0) S3(2, 1, 3, 4, 8, 12, true, false, 0)
        S6(2, 2, 3, 2, 7, 12, true, true, 4) S6(2, 2, 3, 2, 7, 12, true, false, 0) S6(2, 2, 2, 2, 4, 16, true, true, 4)
        S6(2, 1, 3, 4, 7, 12, true, true, 4) S6(2, 2, 3, 2, 7, 12, false, true, 4)
        F2(4, 1, 3, 2, 9, 21, false, 4) F2(4, 1, 3, 2, 9, 21, false, 0) F2(4, 1, 4, 2, 12, 21, false, 4)
        F2(4, 1, 6, 2, 12, 30, false, 3) F2(4, 1, 3, 2, 9, 21, true, 4) F2(4, 1, 2, 2, 6, 21, false, 4)
        return 0;
    }
    if (which == 10) {  // the shipped c5 / c2 tiles alone (PMC passes)
        C5(3, 2, 5, 2, 39, 6) C2(4, 1, 3, 2, 6, 30)
        return 0;
    }
    if (!which || which == 2) {
        G2(4, 1, 3, 2, 9, 21) G2(4, 1, 4, 2, 12, 21) G2(4, 1, 5, 2, 6, 48)
        J2(4, 1, 3, 2, 9, 21, false, 0) J2(4, 1, 4, 2, 12, 21, false, 0) J2(4, 1, 5, 2, 6, 48, false, 0)
        J2(4, 1, 6, 2, 12, 30, false, 0) J2(4, 1, 8, 2, 12, 42, false, 0) J2(4, 1, 6, 2, 18, 21, false, 0)
        J2(4, 1, 3, 2, 9, 21, false, 4) J2(4, 1, 4, 2, 12, 21, false, 4) J2(4, 1, 6, 2, 12, 30, false, 3)
        J2(4, 1, 4, 2, 12, 21, true, 0) J2(4, 1, 6, 2, 12, 30, true, 0)
    }
    if (!which || which == 3) {
        C3(4, 2, 3, 2, 10, 18) J3(4, 2, 3, 2, 10, 18, true, 0) J3(4, 2, 3, 2, 10, 18, true, 4)
        J3(4, 2, 4, 2, 10, 24, true, 0) J3(4, 2, 4, 2, 10, 24, true, 4) J3(4, 2, 3, 2, 10, 18, false, 4)
        J3(4, 2, 6, 2, 25, 12, true, 0) J3(4, 2, 5, 2, 25, 12, true, 0)
    }
    if (!which || which == 4) {
        C4(4, 2, 3, 2, 12, 14) J4(4, 2, 3, 2, 12, 14, true, 0) J4(4, 2, 3, 2, 12, 14, true, 4)
        J4(4, 2, 4, 2, 16, 14, true, 0) J4(4, 2, 4, 2, 16, 14, true, 4) J4(4, 2, 4, 2, 16, 14, false, 4)
        J4(4, 2, 6, 2, 24, 14, true, 0) J4(4, 2, 7, 2, 16, 28, true, 0) J4(2, 2, 7, 2, 16, 14, true, 0)
    }
    if (!which || which == 5) {
        G5(4, 2, 4, 2, 39, 6) J5(4, 2, 4, 2, 39, 6, false, 0) J5(4, 2, 4, 2, 39, 6, false, 4)
        J5(4, 2, 4, 2, 39, 6, true, 0) J5(4, 2, 4, 2, 39, 6, true, 4) J5(4, 1, 4, 4, 39, 6, false, 0)
        J5(4, 1, 4, 4, 39, 6, false, 4) J5(8, 2, 4, 2, 39, 12, false, 0) J5(8, 2, 4, 2, 39, 12, false, 4)
        J5(4, 2, 2, 2, 3, 33, false, 4) J5(2, 2, 4, 2, 3, 33, false, 4) J5(4, 2, 4, 2, 6, 33, false, 4)
        J5(4, 2, 4, 4, 39, 6, false, 0) J5(4, 2, 4, 4, 39, 6, false, 2)
    }
    if (!which || which == 6) {
        C6(4, 2, 3, 2, 7, 20) J6(4, 2, 3, 2, 7, 20, true, 0) J6(4, 2, 3, 2, 7, 20, true, 4)
        J6(4, 2, 5, 2, 13, 20, true, 0) J6(4, 1, 3, 4, 7, 20, true, 0)
    }
    hipError_t e = hipGetLastError();
    printf("last error: %s\n", hipGetErrorString(e));
    return 0;
}
