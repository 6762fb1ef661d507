// Probe: issue rate of scalar vs packed f32 VALU on gfx950 (no MFMAs in
// flight): ITER iterations of 16 independent chains per lane, one kernel per
// form, W waves per SIMD, timed with HIP events.  The ratio of the packed and
// scalar forms' instruction rates answers whether a v_pk_* op issues as fast
// as its scalar counterpart (and so does twice the work per issue slot).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;

template <int FORM>
__global__ __launch_bounds__(256) void probe(float* out, float s) {
    // FORM 0: v_fma_f32 x16 chains; 1: v_pk_fma_f32 x8 pairs (same flops);
    // 2: v_add_f32 x16; 3: v_pk_add_f32 x8; 4: v_pk_fma_f32 x16 pairs (twice the flops of 0)
    float a[16];
    f2 p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        a[i] = threadIdx.x * 1e-3f + i;
        p[i] = f2{a[i], a[i] + 0.5f};
    }
    const f2 s2 = f2{s, s * 0.5f};
    // inline asm: exactly one instruction per chain step (the optimiser would
    // otherwise pack, fold or reassociate the chains)
    const f2 c2 = f2{0.25f, 0.25f};
    for (int it = 0; it < ITER; ++it) {
        if constexpr (FORM == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(a[i]) : "v"(s));
        } else if constexpr (FORM == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(s2), "v"(c2));
        } else if constexpr (FORM == 2) {
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
        } else if constexpr (FORM == 3) {
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(s2));
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(s2), "v"(c2));
        }
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) r += a[i] + p[i].x + p[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int FORM>
static void run(const char* name, int insts_per_iter, float* out, int waves_per_simd) {
    const int grid = 256 * waves_per_simd;  // 256 CUs x 4 SIMDs: 4 waves per block of 256 threads
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(probe<FORM>, dim3(grid), dim3(256), 0, 0, out, 0.999f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    const int reps = 5;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(probe<FORM>, dim3(grid), dim3(256), 0, 0, out, 0.999f);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double sec = ms * 1e-3 / reps;
    // instructions issued per SIMD: waves_per_simd * ITER * insts_per_iter
    const double ins = (double)waves_per_simd * ITER * insts_per_iter;
    const double ghz = 2.4;
    printf("%-28s W=%d  %8.1f us  %6.2f cycles per wave-instruction per SIMD (at %.1f GHz)\n", name, waves_per_simd,
           sec * 1e6, sec * ghz * 1e9 / ins, ghz);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 256 * 16 * 256 * sizeof(float));
    for (int w : {2, 4, 8}) {
        run<0>("v_fma_f32 x16", 16, out, w);
        run<1>("v_pk_fma_f32 x8", 8, out, w);
        run<4>("v_pk_fma_f32 x16", 16, out, w);
        run<2>("v_add_f32 x16", 16, out, w);
        run<3>("v_pk_add_f32 x8", 8, out, w);
    }
    printf("last error: %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
