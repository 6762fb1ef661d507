// Accumulation precision of the fp8 MFMAs used by conv_mfma (AA_PREC_FP8):
// v_mfma_scale_f32_16x16x128_f8f6f4 (scales literal 0: unscaled) and
// v_mfma_f32_16x16x32_fp8_fp8, on random e4m3 operands and a random f32
// accumulator, against the exact dot product (double) rounded once to f32.
// Prints, per instruction, how many of the 16x16 outputs differ from
// fl32(C + exact) and the distribution of the difference in f32 ulps, plus
// how many match a few candidate rounding models, so the CPU emulation
// (oracle/cnn_oracle.py forward_fp8_emulated) can follow the hardware.
// Modes: (none) random operands; p: A >= 0; a: structured (one 2^e1 product
// and 127 products of 2^e2 per row, B = 1) to find the alignment window.
// Result (profiles/r03/fp8_mfma_precision.txt): the sum is NOT exact -- each
// group of 8 products (one lane's 8 bytes of a 32-deep chunk) is aligned to
// the largest exponent sum (ea + eb) of its products, every product truncated
// toward zero to 2^(that - 13).
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_fp8_precision.hip -o tools/mfma_fp8_precision
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef long v2l __attribute__((ext_vector_type(1)));
typedef float v4f __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__);               \
            return 1;                                                                \
        }                                                                            \
    } while (0)

// block b: A / B bytes of its own 16x16x128 tile (lane l: 32 bytes), C per lane
__global__ void k128(const uint8_t* A, const uint8_t* B, const float* C, float* out) {
    const int l = threadIdx.x, b = blockIdx.x;
    v8i av, bv;
    memcpy(&av, A + ((size_t)b * 64 + l) * 32, 32);
    memcpy(&bv, B + ((size_t)b * 64 + l) * 32, 32);
    v4f c;
    for (int r = 0; r < 4; ++r) c[r] = C[(size_t)b * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)];
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[(size_t)b * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

// the same tile as four K = 32 MFMAs (k group g = bytes 8g..8g+7 of each lane,
// the order conv_mfma's K = 32 path accumulates a 32-channel chunk in)
__global__ void k32x4(const uint8_t* A, const uint8_t* B, const float* C, float* out) {
    const int l = threadIdx.x, b = blockIdx.x;
    v4f c;
    for (int r = 0; r < 4; ++r) c[r] = C[(size_t)b * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)];
    for (int g = 0; g < 4; ++g) {
        long a, bb;
        memcpy(&a, A + ((size_t)b * 64 + l) * 32 + 8 * g, 8);
        memcpy(&bb, B + ((size_t)b * 64 + l) * 32 + 8 * g, 8);
        c = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, bb, c, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) out[(size_t)b * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

static double e4m3(uint8_t v) {
    const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
    const double f = e ? std::ldexp(1.0 + m / 8.0, e - 7) : std::ldexp(m / 8.0, -6);
    return s ? -f : f;
}

// hardware model under test: one group = 8 products; each truncated toward
// zero to a multiple of 2^(floor(log2(max |p|)) - WIN) of its group
static int WIN = 13;
static int e4m3_exp(uint8_t v) { const int e = (v >> 3) & 15; return e ? e - 7 : -6; }
static double group_sum(const double* p, const int* es) {
    int mx = -100;
    for (int t = 0; t < 8; ++t) mx = std::max(mx, es[t]);
    const double grid = std::ldexp(1.0, mx - WIN);
    double s = 0;
    for (int t = 0; t < 8; ++t) s += std::trunc(p[t] / grid) * grid;
    return s;
}

static long ulps(float a, float b) {
    int32_t ia, ib;
    memcpy(&ia, &a, 4);
    memcpy(&ib, &b, 4);
    if (ia < 0) ia = INT32_MIN - ia;
    if (ib < 0) ib = INT32_MIN - ib;
    return (long)ia - (long)ib;
}

int main(int argc, char** argv) {
    const int NB = 2048;
    const bool pos = argc > 1 && argv[1][0] == 'p';  // A >= 0 (post-activation inputs)
    if (argc > 2) WIN = atoi(argv[2]);
    std::mt19937 rng(7);
    std::vector<uint8_t> A((size_t)NB * 64 * 32), B(A.size());
    std::vector<float> C((size_t)NB * 256);
    auto rnd8 = [&](bool nonneg) {
        for (;;) {
            uint8_t v = (uint8_t)(rng() & 0xff);
            if ((v & 0x7f) == 0x7f) continue;           // NaN
            if (((v >> 3) & 15) < 3 && (rng() & 3)) continue;  // fewer tiny values
            if (nonneg) v &= 0x7f;
            return v;
        }
    };
    for (auto& v : A) v = rnd8(pos);
    for (auto& v : B) v = rnd8(false);
    const bool align = argc > 1 && argv[1][0] == 'a';
    const bool bits = argc > 1 && argv[1][0] == 'b';  // rounding window / grouping probes (row 0, B = 1)
    if (bits) {
        auto enc = [](double v) -> uint8_t {  // exact e4m3 code of a representable value
            for (int c = 0; c < 256; ++c)
                if ((c & 0x7f) != 0x7f && e4m3((uint8_t)c) == v) return (uint8_t)c;
            return 0;
        };
        std::fill(A.begin(), A.end(), 0);
        std::fill(B.begin(), B.end(), 0x38);
        for (int l = 0; l < 16; ++l) B[((size_t)514 * 64 + l) * 32 + 0] = enc(1.5);  // T6 t = 2
        for (int b = 0; b < NB; ++b) {
            uint8_t* a = &A[(size_t)b * 64 * 32];  // lane l's bytes at a[l * 32 ..]; row 0 = lanes 0, 16, 32, 48
            a[0] = enc(256.0);
            if (b < 256) {  // T1: one small product 2^(8-d) (1 + m/8) (sign s) beside 256 at byte 1
                const int d = 10 + b % 8, m = (b / 8) % 8, sg = (b / 64) % 2;
                double v = std::ldexp(1.0 + m / 8.0, 8 - d);
                if (8 - d < -6) v = std::ldexp(std::floor(std::ldexp(v, 9)), -9);  // subnormal grid
                a[1] = enc(sg ? -v : v);
            } else if (b >= 512 && b < 520) {  // T5 / T6
                const int t = b - 512;
                if (t == 0) { a[1] = enc(0.015625); a[2] = enc(0.015625); }          // two half-grid smalls
                if (t == 1) { a[1] = enc(0.015625); a[2] = enc(0.015625); a[3] = enc(0.015625); a[4] = enc(0.015625); }
                if (t == 2) { a[0] = enc(192.0); a[1] = enc(0.046875); }             // big 288 with B = 1.5 below
                if (t == 3) { a[0] = enc(192.0); a[1] = enc(0.046875); }             // same, B = 1 (big 192)
                if (t == 4) { a[1] = enc(-0.015625); a[2] = enc(0.046875); }          // mixed signs: -0.5 + 1.5 grid
                if (t == 5) { a[0] = enc(-256.0); a[1] = enc(0.046875); }             // negative big
                if (t == 6) { a[1] = enc(0.046875); a[32 * 16 + 0] = enc(0.046875); } // second group: 1.5 grid, own max
                if (t == 7) { a[0] = enc(256.0); a[8] = enc(0.046875); }              // byte 8: next chunk's group
            } else if (b < 512) {  // T3: 2^-6 (14 binades below) at lane group g, byte y
                const int q = b - 256, g = q % 4, y = (q / 4) % 32;
                if (g == 0 && y == 0) continue;
                a[g * 16 * 32 + y] = enc(std::ldexp(1.0, -6));
            }
        }
    }  // structured: one 2^e1 product + 127 of 2^e2
    if (align) {
        auto enc = [](int e) -> uint8_t { return e >= -6 ? (uint8_t)(((e + 7) << 3)) : (uint8_t)(1 << (e + 9)); };
        for (int b = 0; b < NB; ++b) {
            const int e1 = b % 16 - 6, e2 = -9 + (b / 16) % 16;  // e1 -6..9 (capped 8), e2 -9..6
            for (int l = 0; l < 64; ++l)
                for (int by = 0; by < 32; ++by) {
                    const bool first = (l >> 4) == 0 && by == 0;
                    A[((size_t)b * 64 + l) * 32 + by] = enc(std::min(first ? e1 : e2, 8));
                    B[((size_t)b * 64 + l) * 32 + by] = 0x38;  // 1.0
                }
        }
    }
    std::normal_distribution<float> nd(0.f, 40.f);
    for (auto& v : C) v = nd(rng);
    uint8_t *dA, *dB;
    float *dC, *dO;
    CK(hipMalloc(&dA, A.size()));
    CK(hipMalloc(&dB, B.size()));
    CK(hipMalloc(&dC, C.size() * 4));
    CK(hipMalloc(&dO, C.size() * 4));
    CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
    for (int zc = 0; zc < 2; ++zc) {
        std::vector<float> Cz(C.size(), 0.f);
        const std::vector<float>& Cu = zc ? C : Cz;
        CK(hipMemcpy(dC, Cu.data(), Cu.size() * 4, hipMemcpyHostToDevice));
        for (int kind = 0; kind < 2; ++kind) {
            if (kind == 0)
                hipLaunchKernelGGL(k128, dim3(NB), dim3(64), 0, 0, dA, dB, dC, dO);
            else
                hipLaunchKernelGGL(k32x4, dim3(NB), dim3(64), 0, 0, dA, dB, dC, dO);
            CK(hipDeviceSynchronize());
            std::vector<float> O(C.size());
            CK(hipMemcpy(O.data(), dO, O.size() * 4, hipMemcpyDeviceToHost));
            std::map<long, long> hist;
            long n = 0, eq_once = 0, eq_chunk = 0, eq_c_last = 0, eq_model = 0;
            for (int b = 0; b < NB; ++b)
                for (int i = 0; i < 16; ++i)
                    for (int j = 0; j < 16; ++j) {
                        double ex = 0, part[4] = {0, 0, 0, 0};
                        for (int g = 0; g < 4; ++g)
                            for (int by = 0; by < 32; ++by) {
                                const double p = e4m3(A[((size_t)b * 64 + i + 16 * g) * 32 + by]) *
                                                 e4m3(B[((size_t)b * 64 + j + 16 * g) * 32 + by]);
                                ex += p;
                                part[by / 8] += p;  // k32x4's chunk g' = bytes 8g'..8g'+7 of every lane group
                            }
                        const float c0 = Cu[(size_t)b * 256 + i * 16 + j];
                        const float once = (float)((double)c0 + ex);
                        float chunk = c0;  // four rounded partial adds
                        for (int g = 0; g < 4; ++g) chunk = (float)((double)chunk + part[g]);
                        const float tr = (float)(double)c0 + (float)ex;  // product sum rounded, then added
                        const float got = O[(size_t)b * 256 + i * 16 + j];
                        float model = c0;
                        {
                            double gs[4][4];  // [lane group g][chunk c]
                            for (int g = 0; g < 4; ++g)
                                for (int c = 0; c < 4; ++c) {
                                    double pp[8];
                                    int es[8];
                                    for (int t = 0; t < 8; ++t) {
                                        const uint8_t ua = A[((size_t)b * 64 + i + 16 * g) * 32 + 8 * c + t];
                                        const uint8_t ub = B[((size_t)b * 64 + j + 16 * g) * 32 + 8 * c + t];
                                        pp[t] = e4m3(ua) * e4m3(ub);
                                        es[t] = e4m3_exp(ua) + e4m3_exp(ub);
                                    }
                                    gs[g][c] = group_sum(pp, es);
                                }
                            if (kind == 0) {
                                double t = c0;
                                for (int g = 0; g < 4; ++g)
                                    for (int c = 0; c < 4; ++c) t += gs[g][c];
                                model = (float)t;
                            } else {
                                for (int c = 0; c < 4; ++c) {
                                    double t = model;
                                    for (int g = 0; g < 4; ++g) t += gs[g][c];
                                    model = (float)t;
                                }
                            }
                        }
                        eq_model += got == model;
                        ++n;
                        if (bits && zc == 0 && i == 0 && j == 0 && b >= 512 && b < 520)
                            printf("  %s T5/6 case %d: got %.9g exact %.9g\n", kind ? "k32" : "k128", b - 512, got, ex);
                        if (bits && zc == 0 && i == 0 && j == 0 && b < 512) {
                            if (b < 256)
                                printf("  %s T1 d=%d m=%d s=%d: got-256 %.9g small %.9g\n", kind ? "k32" : "k128", 10 + b % 8,
                                       (b / 8) % 8, (b / 64) % 2, got - 256.0, ex - 256.0);
                            else if (b >= 512)
                                ;
                            else if (got != once)
                                printf("  %s T3 dropped at lane group %d byte %d\n", kind ? "k32" : "k128", (b - 256) % 4,
                                       ((b - 256) / 4) % 32);
                        }
                        if (align && zc == 0 && kind == 0 && i == 0 && j == 0 && b < 256 && got != once)
                            printf("  big 2^%d + 127 x 2^%d: got %.9g exact %.9g\n", std::min(b % 16 - 6, 8), -9 + (b / 16) % 16, got, ex);
                        eq_once += got == once;
                        eq_chunk += got == chunk;
                                                eq_c_last += got == tr;
                        ++hist[std::max(-8L, std::min(8L, ulps(got, once)))];
                    }
            printf("%s C=%s A%s: n %ld  ==fl32(C+exact) %ld  ==4 chunk adds %ld  ==fl32(C)+fl32(exact) %ld  ==model(WIN %d) %ld\n",
                   kind ? "16x16x32 x4 " : "16x16x128  ", zc ? "rand" : "0   ", pos ? ">=0" : "+-", n, eq_once,
                   eq_chunk, eq_c_last, WIN, eq_model);
            printf("   ulps vs fl32(C+exact):");
            for (auto& kv : hist) printf(" %ld:%ld", kv.first, kv.second);
            printf("\n");
        }
    }
    return 0;
}
