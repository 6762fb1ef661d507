// Shared helpers for libaa.so: error plumbing and small device utilities.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

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

// Raise `kernel`'s dynamic-LDS limit to at least `bytes` (thread-safe, aa_api.cpp).
int ensure_dyn_lds(const void* kernel, size_t bytes);
#define AA_DYN_LDS(kernel, bytes)                                                    \
    do {                                                                             \
        const int rc_ = ::aa::ensure_dyn_lds((const void*)(kernel), (bytes));        \
        if (rc_ != AA_OK) return rc_;                                                \
    } while (0)

// HIP-event timing of selected launches (bench.py's roofline): a pair of
// events on the launch stream around each timed launch, recycled through a
// pool.  Only the stages named in `mask` are timed, so an untimed launch
// sequence carries no event records between its kernels.
struct StageTimer {
    uint32_t mask = 0;
    std::vector<hipEvent_t> pool;
    std::vector<std::vector<std::pair<hipEvent_t, hipEvent_t>>> ev;  // per stage

    bool on(int s) const { return s < 32 && (mask >> s) & 1u; }
    int begin(int s, hipStream_t st, hipEvent_t* e0) {
        *e0 = nullptr;
        if (!on(s)) return AA_OK;
        AA_HIP(take(e0));
        AA_HIP(hipEventRecord(*e0, st));
        return AA_OK;
    }
    int end(int s, hipStream_t st, hipEvent_t e0) {
        if (!e0) return AA_OK;
        hipEvent_t e1;
        AA_HIP(take(&e1));
        AA_HIP(hipEventRecord(e1, st));
        if ((int)ev.size() <= s) ev.resize(s + 1);
        ev[s].emplace_back(e0, e1);
        return AA_OK;
    }
    // sum and count of the recorded launches of stage s; clears them
    int collect(int s, double* total_ms, int64_t* count) {
        double tot = 0;
        int64_t n = 0;
        if (s < (int)ev.size()) {
            for (auto& e : ev[s]) {
                AA_HIP(hipEventSynchronize(e.second));
                float ms = 0;
                AA_HIP(hipEventElapsedTime(&ms, e.first, e.second));
                tot += ms;
                ++n;
                pool.push_back(e.first);
                pool.push_back(e.second);
            }
            ev[s].clear();
        }
        if (total_ms) *total_ms = tot;
        if (count) *count = n;
        return AA_OK;
    }
    void release() {
        for (auto& v : ev)
            for (auto& e : v) pool.push_back(e.first), pool.push_back(e.second);
        ev.clear();
        for (hipEvent_t e : pool) (void)hipEventDestroy(e);
        pool.clear();
    }

  private:
    hipError_t take(hipEvent_t* e) {
        if (!pool.empty()) {
            *e = pool.back();
            pool.pop_back();
            return hipSuccess;
        }
        return hipEventCreate(e);
    }
};

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
