// Error reporting + version for the fdx C ABI.
#include <cstring>

#include "fdx_internal.h"

namespace fdx {
namespace {
thread_local char g_err[1024] = "";
}

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace fdx

extern "C" const char *fdx_last_error(void) { return fdx::g_err; }
extern "C" int fdx_abi_version(void) { return FDX_ABI_VERSION; }
