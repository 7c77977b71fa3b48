// Host-side error reporting for the C ABI (thread-local last-error message).
#include <stdarg.h>
#include <stdio.h>
#include "../../include/dbsr_hip.h"

static thread_local char g_err[512];

void dbsr_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

extern "C" const char* dbsr_last_error(void) { return g_err; }
extern "C" int dbsr_abi_version(void) { return DBSR_ABI_VERSION; }
