// libaa.so: ABI version, the thread-local error string, file input.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>
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

// One call per file for the corpus decoder threads: their Python wrapper
// holds the interpreter lock only around the call, not around each of the
// stat / open / read / close steps (with 8 lanes busy in Python, every
// re-acquisition of the lock could wait out a switch interval).
extern "C" int aa_read_file(const char* path, void* buf, int64_t cap, int64_t* size) {
    AA_CHECK(path && size && (buf || cap == 0), AA_ERR_INVALID, "aa_read_file: null argument");
    *size = 0;
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    AA_CHECK(fd >= 0, AA_ERR_INVALID, "aa_read_file: %s: %s", path, strerror(errno));
    struct stat st;
    if (fstat(fd, &st) != 0) {
        const int e = errno;
        close(fd);
        AA_CHECK(false, AA_ERR_INVALID, "aa_read_file: %s: %s", path, strerror(e));
    }
    *size = (int64_t)st.st_size;
    if ((int64_t)st.st_size > cap) {
        close(fd);
        aa::set_error("aa_read_file: %s: %lld bytes > %lld", path, (long long)st.st_size, (long long)cap);
        return AA_ERR_WORKSPACE;
    }
    char* p = static_cast<char*>(buf);
    int64_t got = 0;
    while (got < (int64_t)st.st_size) {
        const ssize_t r = read(fd, p + got, (size_t)(st.st_size - got));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
            const int e = r < 0 ? errno : 0;
            close(fd);
            AA_CHECK(false, AA_ERR_INVALID, "aa_read_file: %s: %s", path, e ? strerror(e) : "short read");
        }
        got += r;
    }
    close(fd);
    return AA_OK;
}
