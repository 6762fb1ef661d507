// libaa.so: ABI version and the thread-local error string.
#include <cstdarg>
#include <cstdio>

#include "aa_common.h"

namespace aa {
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace aa

extern "C" int aa_abi_version(void) { return AA_ABI_VERSION; }
extern "C" const char* aa_last_error(void) { return aa::g_err; }
