// Diagnostic harness: time fe_stft_mel_4096 with phases ablated (DIAG bits,
// see the kernel) on the config-2 shape: 64 windows of 144000 samples,
// n_fft 4096, hop 640, 160 triangular mel bands over bins 5..938.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I include
//   tools/fe_bench.hip audio-analysis_amd/csrc/aa_api.cpp -o tools/fe_bench
#include "../audio-analysis_amd/csrc/aa_frontend.hip"

#include <cstdio>
#include <cstdlib>
#include <string>

using namespace aa;

template <int DIAG>
static float time_diag(const FePlan& p, const float* pcm, const aa_window* wins, int n_win, const float4* stats,
                       float* melS, float* blkmax, int iters) {
    const size_t lds = fe_lds_bytes4096(p);
    (void)hipFuncSetAttribute((const void*)fe_stft_mel_4096<PM_SQUARE, DIAG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int n_frames = p.T * n_win;
    const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / lds)));
    int grid = std::min((n_frames + kWpb - 1) / kWpb, 256 * per_cu);
    grid = (grid + 7) & ~7;
    auto go = [&]() {
        hipLaunchKernelGGL((fe_stft_mel_4096<PM_SQUARE, DIAG>), dim3(grid), dim3(64 * kWpb), lds, 0, pcm, wins,
                           stats, p.d_tw, p.d_tw2, p.d_cimg, p.cimg_bytes, p.cfg.win_len, p.cfg.hop, p.T,
                           p.cfg.n_mels, p.kmin, p.kmax, p.cfg.normalize, p.cfg.power, n_frames, melS, blkmax);
    };
    for (int i = 0; i < 3; ++i) go();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i) go();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return 1e3f * ms / iters;
}

int main(int argc, char** argv) {
    const int n_win = 64, n_mels = 160, nbins = 2049;
    std::vector<float> fb((size_t)n_mels * nbins, 0.f);
    for (int m = 0; m < n_mels; ++m) {  // triangles with centres spread over bins 5..938
        const double a = 5 + 933.0 * m / (n_mels + 1), c = 5 + 933.0 * (m + 1) / (n_mels + 1),
                     b = 5 + 933.0 * (m + 2) / (n_mels + 1);
        for (int k = (int)a; k <= (int)b; ++k) {
            const double v = k < c ? (k - a) / (c - a) : (b - k) / (b - c);
            if (v > 0) fb[(size_t)m * nbins + k] = (float)v;
        }
    }
    aa_fe_config cfg{144000, 4096, 640, n_mels, 1, 1, 2.f, 1e-10f, 80.f, 0, 1};
    void* plan = nullptr;
    if (aa_fe_create(&cfg, fb.data(), &plan) != AA_OK) { printf("create: %s\n", aa_last_error()); return 1; }
    const FePlan& p = *static_cast<FePlan*>(plan);
    printf("nnz %d kmin %d kmax %d fast %d lds %zu\n", p.nnz, p.kmin, p.kmax, (int)fe_fast4096(p), fe_lds_bytes4096(p));
    const size_t n_pcm = 2 * 2880000;
    std::vector<float> h(n_pcm);
    uint32_t rs = 12345u;  // a local generator: the HIP runtime draws on rand() itself
    for (auto& x : h) {
        rs = rs * 1664525u + 1013904223u;
        x = (float)((int)(rs >> 16) - 32768) / 32768.f;
    }
    std::vector<aa_window> hw(n_win);
    for (int i = 0; i < n_win; ++i) hw[i] = aa_window{(int64_t)(i % 39) * 72000 + (i / 39) * 2880000, 144000, 0};
    float *pcm, *melS, *blkmax;
    aa_window* wins;
    float4* stats;
    (void)hipMalloc(&pcm, n_pcm * 4);
    (void)hipMalloc(&wins, n_win * sizeof(aa_window));
    (void)hipMalloc(&stats, n_win * kStatSplit * sizeof(float4));
    (void)hipMalloc(&melS, (size_t)n_win * n_mels * p.T * 4);
    (void)hipMalloc(&blkmax, (size_t)n_win * p.nfblk * 4);
    (void)hipMemcpy(pcm, h.data(), n_pcm * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(wins, hw.data(), n_win * sizeof(aa_window), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(fe_stats, dim3(kStatSplit, n_win), dim3(256), 0, 0, pcm, wins, cfg.win_len, stats);
    const int it = 20;
#define T_(D) printf("DIAG %3d: %7.1f us\n", D, time_diag<D>(p, pcm, wins, n_win, stats, melS, blkmax, it));
    if (argc > 1 && std::string(argv[1]) == "stamps") {  // per-phase s_memtime totals (DIAG 128)
        const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / fe_lds_bytes4096(p))));
        int grid = std::min((p.T * n_win + kWpb - 1) / kWpb, 256 * per_cu);
        grid = (grid + 7) & ~7;
        const size_t nw = (size_t)grid * kWpb;
        unsigned long long* d_st;
        (void)hipMalloc(&d_st, nw * kFeStampPh * 64 * 8);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(fe_stamps), &d_st, sizeof(d_st));
        T_(0)
        T_(128)
        std::vector<unsigned long long> hs(nw * kFeStampPh * 64);
        (void)hipMemcpy(hs.data(), d_st, hs.size() * 8, hipMemcpyDeviceToHost);
        const char* names[kFeStampPh] = {"loads+hann", "dft32 #1", "twiddles", "transpose", "dft32 #2", "radix-2",
                                         "split+power", "mel rows"};
        const double fpw = (double)p.T * n_win / nw;  // frames per wave
        double tot = 0;
        for (int k = 0; k < kFeStampPh; ++k) {
            double sum = 0;
            for (size_t w = 0; w < nw; ++w) sum += (double)hs[(w * kFeStampPh + k) * 64];
            tot += sum;
        }
        for (int k = 0; k < kFeStampPh; ++k) {
            double sum = 0;
            for (size_t w = 0; w < nw; ++w) sum += (double)hs[(w * kFeStampPh + k) * 64];
            printf("  %-12s %8.0f ticks per frame per wave  %5.1f %%\n", names[k], sum / nw / fpw, 100.0 * sum / tot);
        }
        printf("  (%zu waves, %.2f frames per wave; s_memtime ticks; the last iteration of 1 launch)\n", nw, fpw);
        return 0;
    }
    if (argc > 1) {  // PMC / A-B runs: the full kernel only, and a hash of its mel output
        T_(0)
        std::vector<uint32_t> hm((size_t)n_win * n_mels * p.T), h0;
        for (int rep = 0; rep < 2; ++rep) {  // the same launch twice: the hash of each
            if (rep) {
                (void)hipMemset(melS, 0xff, hm.size() * 4);
                time_diag<0>(p, pcm, wins, n_win, stats, melS, blkmax, 1);
            }
            (void)hipMemcpy(hm.data(), melS, hm.size() * 4, hipMemcpyDeviceToHost);
            uint64_t hsh = 1469598103934665603ull;
            for (uint32_t x : hm) hsh = (hsh ^ x) * 1099511628211ull;
            printf("mel hash %016llx ", (unsigned long long)hsh);
            if (rep) {
                size_t nd = 0, first = 0;
                for (size_t i = 0; i < hm.size(); ++i)
                    if (hm[i] != h0[i] && nd++ == 0) first = i;
                printf("(%zu differ from the first launch; first at frame %zu band %zu) ", nd, first / n_mels, first % n_mels);
            }
            h0 = hm;
        }
        uint64_t hp = 1469598103934665603ull;
        for (float x : h) hp = (hp ^ __builtin_bit_cast(uint32_t, x)) * 1099511628211ull;
        printf("pcm hash %016llx\n", (unsigned long long)hp);
        return 0;
    }
    T_(0) T_(1) T_(4) T_(8) T_(16) T_(32) T_(64) T_(4 | 8) T_(4 | 8 | 16) T_(4 | 8 | 16 | 32)
    T_(127) T_(1 | 32 | 64) T_(1 | 64)
#undef T_
    printf("last error: %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
