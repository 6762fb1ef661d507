// Checks that the 3-instruction quotient used by the front end's
// normalisation, q1 = fma(fma(-q0, b, a), y, q0) with q0 = a*y and
// y = RN(1/b), equals the correctly rounded a/b (__fdiv_rn) on random
// operands: a in [0, b] (the normalisation's range) and a over wide ranges.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

__global__ void check(uint32_t seed, int mode, unsigned long long* bad, unsigned long long* tot) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    // divisor: random float in [2^-20, 2^20) with random mantissa
    const uint32_t hb = hash(seed * 0x9e3779b9u + t);
    const float b = __uint_as_float(((127 - 20 + (hb >> 27) % 40) << 23) | (hb & 0x7fffff));
    const float y = __fdiv_rn(1.f, b);
    unsigned long long nb = 0;
    for (int i = 0; i < 256; ++i) {
        const uint32_t ha = hash(hb ^ (i * 0x85ebca6bu) ^ seed);
        float a;
        if (mode == 0) a = __uint_as_float((ha >> 9) | 0x3f800000u) - 1.f;  // [0,1)
        else a = __uint_as_float(((127 - 30 + (ha >> 26) % 60) << 23) | (ha & 0x7fffff));
        if (mode == 0) a = a * b;  // [0, b)
        const float q = __fdiv_rn(a, b);
        const float q0 = a * y;
        const float r = fmaf(-q0, b, a);
        const float q1 = fmaf(r, y, q0);
        nb += (__float_as_uint(q) != __float_as_uint(q1));
    }
    atomicAdd(bad, nb);
    atomicAdd(tot, 256ull);
}

int main() {
    unsigned long long *bad, *tot;
    (void)hipMalloc(&bad, 16);
    (void)hipMalloc(&tot, 16);
    for (int mode = 0; mode < 2; ++mode) {
        (void)hipMemset(bad, 0, 16);
        (void)hipMemset(tot, 0, 16);
        for (uint32_t s = 1; s <= 64; ++s) hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, s, mode, bad, tot);
        unsigned long long hb = 0, ht = 0;
        (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&ht, tot, 8, hipMemcpyDeviceToHost);
        printf("mode %d: %llu mismatches of %llu quotients\n", mode, hb, ht);
    }
    return 0;
}
