// C-ABI runtime pieces: thread-local error string, version.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/rvc_amd.h"

static thread_local char g_err[512] = "";

void rvc_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

extern "C" const char* rvc_last_error(void) { return g_err; }
extern "C" int rvc_version(void) { return 1; }
