// C-ABI runtime pieces: thread-local error string, version, CU-masked streams.
#include <hip/hip_runtime.h>
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

// A stream whose kernels may only use the CUs set in mask (nwords 32-bit words; hipExtStreamCreateWithCUMask).
// Measured (scripts/cu_mask_probe.hip): bit i lands on XCD i mod 8, and a mask naming every CU of one XCD is not
// applied at all.  The clip stream can give its synthesizer stream one (VC.BACK_CU_MASK; off by default).
extern "C" int rvc_stream_create_cu_mask(const uint32_t* mask, int nwords, rvc_stream_t* out) {
    if (!mask || nwords <= 0 || !out) {
        rvc_set_error("stream_create_cu_mask: bad args");
        return RVC_EINVAL;
    }
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask);
    if (e != hipSuccess) {
        rvc_set_error("hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
        return RVC_EHIP;
    }
    *out = (rvc_stream_t)s;
    return RVC_OK;
}

extern "C" int rvc_stream_destroy(rvc_stream_t s) {
    const hipError_t e = hipStreamDestroy((hipStream_t)s);
    if (e != hipSuccess) {
        rvc_set_error("hipStreamDestroy: %s", hipGetErrorString(e));
        return RVC_EHIP;
    }
    return RVC_OK;
}
