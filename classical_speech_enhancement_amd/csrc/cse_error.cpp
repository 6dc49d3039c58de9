// cse_last_error() / cse_version(): host-side bookkeeping of libcse.so.
#include <stdarg.h>
#include <stdio.h>

#include "cse_common.hpp"

namespace cse {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace cse

extern "C" const char* cse_last_error(void) { return cse::g_err; }
extern "C" int cse_version(void) { return 5; }
