// libaa.so: ABI version and the thread-local error string.
#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <unordered_map>

#include "aa_common.h"

namespace aa {
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// Per-kernel dynamic-LDS opt-in, raised to the largest size asked for.  Lane
// threads launch the same kernels concurrently, so the high-water marks sit
// behind one mutex (a plain static per call site would be a data race).
int ensure_dyn_lds(const void* kernel, size_t bytes) {
    static std::mutex mu;
    static std::unordered_map<const void*, size_t> granted;
    std::lock_guard<std::mutex> g(mu);
    size_t& have = granted[kernel];
    if (bytes > have) {
        AA_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
        have = bytes;
    }
    return AA_OK;
}
}  // namespace aa

extern "C" int aa_abi_version(void) { return AA_ABI_VERSION; }
extern "C" const char* aa_last_error(void) { return aa::g_err; }
