// Diagnostic harness: the persistent producer / consumer fused first conv
// (conv_x3pc, tools/conv_x3pc.h; measured and rejected, profiles/r06/pc_ablations.txt) against the fused conv_x3 it replaces, on the
// bench's shape (64 windows of a 160 x 226 log-mel, model1's first block):
// outputs compared bit for bit (f32 and grouped-split), then both timed,
// alternating, with HIP events.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -mllvm -amdgpu-mfma-vgpr-form
//   tools/pc_check.hip audio-analysis_amd/csrc/aa_api.cpp -o tools/pc_check ; run on the GPU box.
#include "../audio-analysis_amd/csrc/aa_cnn.hip"
#include "conv_x3pc.h"  // the rejected persistent producer / consumer form (profiles/r06/pc_ablations.txt)

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace aa;

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 64;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const int H0 = 160, W0 = 226, Hin = H0 - 2, Win = W0 - 2, Hout = Hin / 3, Wout = Win / 3, cout = 32;
    unsigned st = 12345;
    auto rnd = [&]() {
        st = st * 1664525u + 1013904223u;
        return (st >> 8) * (1.f / 16777216.f) - 0.5f;
    };
    std::vector<float> lm((size_t)n * H0 * W0);
    for (auto& v : lm) v = -40.f + 60.f * rnd();  // dB-like values
    std::vector<float> w1(32 * 9), b1(32), b2(cout);
    for (auto& v : w1) v = 0.05f * rnd();
    for (auto& v : b1) v = 0.2f * rnd();
    for (auto& v : b2) v = 0.2f * rnd();
    // packed weights [tap][cout][8 units] with unit u of row o in slot (u + o) & 7: hi units 0-3, lo 4-7
    std::vector<uint16_t> wp((size_t)9 * cout * 64);
    for (int t = 0; t < 9; ++t)
        for (int o = 0; o < cout; ++o)
            for (int c = 0; c < 32; ++c) {
                const float x = 0.08f * rnd();
                const uint16_t hi = f2bf(x);
                uint32_t hu = (uint32_t)hi << 16;
                float hf;
                memcpy(&hf, &hu, 4);
                const uint16_t lo = f2bf(x - hf);
                const int uh = c / 8, ul = 4 + c / 8;
                uint16_t* row = &wp[((size_t)t * cout + o) * 64];
                row[(((uh + o) & 7) * 8) + c % 8] = hi;
                row[(((ul + o) & 7) * 8) + c % 8] = lo;
            }
    float *d_lm, *d_w1, *d_b1, *d_b2, *d_o1, *d_o2;
    bf16* d_w;
    const size_t out_n = (size_t)n * Hout * Wout * cout;
    (void)hipMalloc(&d_lm, lm.size() * 4);
    (void)hipMalloc(&d_w1, w1.size() * 4);
    (void)hipMalloc(&d_b1, b1.size() * 4);
    (void)hipMalloc(&d_b2, 64 * 4);
    (void)hipMalloc(&d_w, wp.size() * 2);
    (void)hipMalloc(&d_o1, out_n * 4);
    (void)hipMalloc(&d_o2, out_n * 4);
    (void)hipMemcpy(d_lm, lm.data(), lm.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_w1, w1.data(), w1.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_b1, b1.data(), b1.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_b2, b2.data(), b2.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_w, wp.data(), wp.size() * 2, hipMemcpyHostToDevice);
    FirstConv fc{d_w1, d_b1, ACT_LEAKY, 0.3f, 0, 1.f, H0, W0, 0};

    // the shipped fused conv_x3 instantiation (AA_X3_CFGS row 1)
    auto k_old = conv_x3<3, 3, 32, 4, 1, 4, 2, 3, 12, 21, true, 0, false, true, 0, false, false>;
    const size_t lds_old = x3_lds_bytes<3, 3, 32, 32, 12, 21, true, false>();
    (void)hipFuncSetAttribute((const void*)k_old, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_old);
    const int tiles_h = (Hout * 3 + 11) / 12, tiles_w = (Wout * 3 + 20) / 21;
    auto run_old = [&](float* o) {
        hipLaunchKernelGGL(k_old, dim3(tiles_h * tiles_w, 1, n), dim3(256), lds_old, 0, (const float*)d_lm, Hin, Win,
                           (const bf16*)d_w, (const float*)d_b2, o, Hout, Wout, cout, tiles_w, ACT_LEAKY, 0.3f, fc);
    };
    auto k_new = conv_x3pc<false>;
    (void)hipFuncSetAttribute((const void*)k_new, hipFuncAttributeMaxDynamicSharedMemorySize, (int)PC_LDS);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int items = tiles_h * tiles_w * n;
    const int grid = items < cus ? items : cus;
    auto run_new = [&](float* o) {
        hipLaunchKernelGGL(k_new, dim3(grid), dim3(PC_THREADS), PC_LDS, 0, (const float*)d_lm, (const bf16*)d_w,
                           (const float*)d_b2, o, Hout, Wout, cout, tiles_w, tiles_h * tiles_w, items, ACT_LEAKY, 0.3f,
                           fc);
    };
    // ablations: producers alone (consumers skip their MFMA loop), consumers alone
    auto k_p = conv_x3pc<false, 0, 2, 4>;
    auto k_c = conv_x3pc<false, 0, 4, 8>;
    (void)hipFuncSetAttribute((const void*)k_p, hipFuncAttributeMaxDynamicSharedMemorySize, (int)PC_LDS);
    (void)hipFuncSetAttribute((const void*)k_c, hipFuncAttributeMaxDynamicSharedMemorySize, (int)PC_LDS);
    auto run_abl = [&](int which, float* o) {
        hipLaunchKernelGGL(which == 2 ? k_p : k_c, dim3(grid), dim3(which == 2 ? pc_threads<4>() : pc_threads<8>()), PC_LDS, 0, (const float*)d_lm,
                           (const bf16*)d_w, (const float*)d_b2, o, Hout, Wout, cout, tiles_w, tiles_h * tiles_w, items,
                           ACT_LEAKY, 0.3f, fc);
    };
    (void)hipMemset(d_o1, 0xff, out_n * 4);
    (void)hipMemset(d_o2, 0xee, out_n * 4);
    run_old(d_o1);
    run_new(d_o2);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        printf("kernel error: %s\n", hipGetErrorString(e));
        return 2;
    }
    std::vector<float> o1(out_n), o2(out_n);
    (void)hipMemcpy(o1.data(), d_o1, out_n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o2.data(), d_o2, out_n * 4, hipMemcpyDeviceToHost);
    size_t diff = 0, first = (size_t)-1;
    double maxd = 0, maxv = 0;
    for (size_t i = 0; i < out_n; ++i) {
        if (memcmp(&o1[i], &o2[i], 4) != 0) {
            if (first == (size_t)-1) first = i;
            ++diff;
            maxd = std::max(maxd, (double)fabsf(o1[i] - o2[i]));
        }
        maxv = std::max(maxv, (double)fabsf(o1[i]));
    }
    printf("n %d items %d grid %d LDS old %zu new %zu: %zu of %zu outputs differ (max |d| %.3g, max |out| %.3g)\n", n,
           items, grid, lds_old, (size_t)PC_LDS, diff, out_n, maxd, maxv);
    if (diff) {
        const size_t i = first, px = i / cout, c = i % cout;
        const size_t w = px / ((size_t)Hout * Wout), r = (px / Wout) % Hout, col = px % Wout;
        printf("first difference: window %zu row %zu col %zu ch %zu: old %.8g new %.8g\n", w, r, col, c, o1[i], o2[i]);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double fl = 2.0 * n * Hin * Win * 9 * 32 * cout + 2.0 * n * Hin * Win * 9 * 32;
    const char* names[4] = {"conv_x3 fused", "pc WM8 AD2   ", "pc WM4 AD2   ", "pc WM8 AD4   "};
    for (int round = 0; round < 3; ++round) {
        for (int which = 0; which < 4; ++which) {
            auto run = [&]() {
                if (which == 0) run_old(d_o1);
                else if (which == 1) run_new(d_o2);
                else run_abl(which == 2 ? 2 : 4, d_o1);
            };
            for (int i = 0; i < 3; ++i) run();
            (void)hipEventRecord(e0, 0);
            for (int i = 0; i < iters; ++i) run();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double us = 1e3 * ms / iters;
            printf("%s  %7.1f us  %6.1f TF (%.3f of 833)\n", names[which], us, fl / us * 1e-6,
                   fl / us * 1e-6 / 833.3);
        }
    }
    e = hipDeviceSynchronize();
    printf("last error: %s\n", hipGetErrorString(e));
    return diff ? 1 : 0;
}
