// Shared helpers for libaa.so: error plumbing and small device utilities.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/aa.h"

namespace aa {

// Thread-local message behind aa_last_error().
void set_error(const char* fmt, ...);

#define AA_HIP(call)                                                                 \
    do {                                                                             \
        hipError_t e_ = (call);                                                      \
        if (e_ != hipSuccess) {                                                      \
            ::aa::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,               \
                            hipGetErrorString(e_));                                  \
            return AA_ERR_HIP;                                                       \
        }                                                                            \
    } while (0)

#define AA_CHECK(cond, code, ...)                                                    \
    do {                                                                             \
        if (!(cond)) {                                                               \
            ::aa::set_error(__VA_ARGS__);                                            \
            return (code);                                                           \
        }                                                                            \
    } while (0)

#define AA_LAUNCH_CHECK()                                                            \
    do {                                                                             \
        hipError_t e_ = hipGetLastError();                                           \
        if (e_ != hipSuccess) {                                                      \
            ::aa::set_error("%s:%d kernel launch: %s", __FILE__, __LINE__,           \
                            hipGetErrorString(e_));                                  \
            return AA_ERR_HIP;                                                       \
        }                                                                            \
    } while (0)

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- device helpers -------------------------------------------------------
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

}  // namespace aa
