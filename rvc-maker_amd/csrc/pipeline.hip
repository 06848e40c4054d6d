// Glue kernels of VC.voice_conversion / VC.pipeline (main/inference/convert.py:328-458).
#include "rvc_common.h"

// phone[c][t] = f[c][t/2] * p + f0[c][t/2] * (1 - p),  p = pitchf[t] < 1 ? protect : 1
// F.interpolate(scale_factor=2, nearest) (convert.py:361-362) + protect blend (convert.py:372-378).
// With protect >= 0.5 (no blend) pass pitchf = NULL.  feats0 may alias feats (no index).
__global__ void phone_upsample_kernel(const float* feats, const float* feats0, const float* pitchf, float* out,
                                      int64_t Tf, int64_t T, float protect) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int c = blockIdx.y;
    if (t >= T) return;
    float v = feats[(int64_t)c * Tf + t / 2];
    if (pitchf) {
        float p = pitchf[t] < 1.f ? protect : 1.f;
        float v0 = feats0[(int64_t)c * Tf + t / 2];
        v = v * p + v0 * (1.f - p);
    }
    out[(int64_t)c * T + t] = v;
}

extern "C" int rvc_phone_upsample(const float* feats, const float* feats0, const float* pitchf, float* out, int64_t C,
                                  int64_t Tf, int64_t T, float protect, rvc_stream_t stream) {
    RVC_CHECK_ARG(feats && out && C > 0 && Tf > 0 && T > 0 && T <= 2 * Tf && (!pitchf || feats0),
                  "phone_upsample: bad args");
    hipLaunchKernelGGL(phone_upsample_kernel, dim3(cdiv(T, 256), (unsigned)C), dim3(256), 0, (hipStream_t)stream,
                       feats, feats0, pitchf, out, Tf, T, protect);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// peak normalisation (convert.py:450-451): m = max|x| / 0.99 (f32); if m > 1: x /= m.
__global__ void absmax_kernel(const float* x, int64_t n, unsigned* out) {
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = fmaxf(m, fabsf(x[i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

__global__ void peak_scale_kernel(float* x, int64_t n, const unsigned* mbits, float* scale_out) {
    const float m = __uint_as_float(*mbits) / 0.99f;
    if (blockIdx.x == 0 && threadIdx.x == 0 && scale_out) *scale_out = m;
    if (!(m > 1.f)) return;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        x[i] = x[i] / m;
}

extern "C" int rvc_peak_normalize(float* x, int64_t n, void* ws, float* scale_out, rvc_stream_t stream) {
    RVC_CHECK_ARG(x && ws && n > 0, "peak_normalize: bad args");
    hipStream_t s = (hipStream_t)stream;
    RVC_HIP(hipMemsetAsync(ws, 0, 16, s));
    unsigned grid = cdiv(n, 256) < 2048 ? cdiv(n, 256) : 2048;
    hipLaunchKernelGGL(absmax_kernel, dim3(grid), dim3(256), 0, s, x, n, (unsigned*)ws);
    RVC_HIP(hipGetLastError());
    hipLaunchKernelGGL(peak_scale_kernel, dim3(grid), dim3(256), 0, s, x, n, (const unsigned*)ws, scale_out);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
