// Shared device helpers for the RVC MI355X kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/rvc_amd.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define RVC_DEV __device__ __forceinline__

// MFMA f32 16x16x4 (exact f32 fma chain).  Lane l holds A[l&15][l>>4], B[l>>4][l&15];
// C/D: col = l&15, row = (l>>4)*4 + r.
RVC_DEV floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

RVC_DEV float act_apply(float v, int act, float slope) {
    switch (act) {
        case RVC_ACT_LRELU: return v >= 0.f ? v : v * slope;
        case RVC_ACT_RELU: return v > 0.f ? v : 0.f;
        case RVC_ACT_TANH: return tanhf(v);
        case RVC_ACT_GELU: return 0.5f * v * (1.f + erff(v * 0.70710678118654752440f));
        case RVC_ACT_SIGMOID: return 1.f / (1.f + expf(-v));
        case RVC_ACT_LOGCLAMP: return logf(fmaxf(v, slope));
        default: return v;
    }
}

RVC_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

RVC_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// thread-local error reporting for the C ABI
void rvc_set_error(const char* fmt, ...);

#define RVC_CHECK_ARG(cond, ...)            \
    do {                                    \
        if (!(cond)) {                      \
            rvc_set_error(__VA_ARGS__);     \
            return RVC_EINVAL;              \
        }                                   \
    } while (0)

#define RVC_HIP(call)                                                        \
    do {                                                                     \
        hipError_t e_ = (call);                                              \
        if (e_ != hipSuccess) {                                              \
            rvc_set_error("%s: %s", #call, hipGetErrorString(e_));          \
            return RVC_EHIP;                                                 \
        }                                                                    \
    } while (0)

static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }
