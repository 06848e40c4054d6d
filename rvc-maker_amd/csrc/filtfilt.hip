// Zero-phase IIR high-pass (scipy.signal.filtfilt(bh, ah, x), padtype "odd", padlen 18) followed by
// the pipeline's reflect padding (convert.py:403, 416), in f64 on the device.
//
// lfilter is a linear recurrence on the 5-element transposed-direct-form-II state Z:
//   y = Z0 + b0 x ;  Z_i' = Z_{i+1} + b_{i+1} x - a_{i+1} y      (scipy's DOUBLE_filt order)
// i.e. s' = A s + B x.  One workgroup splits the (extended) signal into 256 chunks: each thread
// runs its chunk from a zero state (phase 1), thread 0 chains the chunk-boundary states with the
// host-precomputed A^c (phase 2), and each thread reruns its chunk from the true state writing y
// (phase 3).  Forward pass, then the backward pass on the reversed output with zi * y[-1].
// f64 throughout; FP contraction is off so every step rounds like the reference's C loop.
#include "rvc_common.h"

#pragma clang fp contract(off)

namespace {
constexpr int NS = 5;  // filter order
constexpr int NT = 256;
constexpr int PADLEN = 18;

struct FiltParams {
    double b[NS + 1], a[NS + 1], zi[NS];
    double Ac[NS * NS];  // A^c for the chunk length c
    int64_t N, L, c, tpad;
};

__device__ __forceinline__ double ext_in(const float* x, int64_t N, int64_t i) {
    if (i < PADLEN) return 2.0 * (double)x[0] - (double)x[PADLEN - i];
    if (i < PADLEN + N) return (double)x[i - PADLEN];
    return 2.0 * (double)x[N - 1] - (double)x[N - 2 - (i - PADLEN - N)];
}

__device__ __forceinline__ double step(const FiltParams& p, double* z, double xn) {
    const double yn = z[0] + p.b[0] * xn;
#pragma unroll
    for (int i = 0; i < NS - 1; ++i) z[i] = z[i + 1] + xn * p.b[i + 1] - yn * p.a[i + 1];
    z[NS - 1] = xn * p.b[NS] - yn * p.a[NS];
    return yn;
}

// one lfilter pass over L samples: in(i) -> out[i]; init state zi * in(0)-or-given scalar
template <typename In>
__device__ void lfilter_pass(const FiltParams& p, In in, double* out, double z0scale, double* states) {
    const int tid = threadIdx.x;
    const int64_t lo = (int64_t)tid * p.c, hi = lo + p.c < p.L ? lo + p.c : p.L;
    double z[NS];
    // phase 1: zero-state local run -> final local state
#pragma unroll
    for (int i = 0; i < NS; ++i) z[i] = 0.0;
    for (int64_t n = lo; n < hi; ++n) step(p, z, in(n));
#pragma unroll
    for (int i = 0; i < NS; ++i) states[(tid + 1) * NS + i] = z[i];
    __syncthreads();
    // phase 2: chain boundary states S_{t+1} = A^c S_t + F_t
    if (tid == 0) {
        double s[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) s[i] = p.zi[i] * z0scale;
#pragma unroll
        for (int i = 0; i < NS; ++i) states[i] = s[i];
        for (int t = 1; t < NT; ++t) {
            double ns[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                double v = 0.0;
#pragma unroll
                for (int j = 0; j < NS; ++j) v += p.Ac[i * NS + j] * s[j];
                ns[i] = v + states[t * NS + i];
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                s[i] = ns[i];
                states[t * NS + i] = ns[i];
            }
        }
    }
    __syncthreads();
    // phase 3: rerun from the true state
#pragma unroll
    for (int i = 0; i < NS; ++i) z[i] = states[tid * NS + i];
    for (int64_t n = lo; n < hi; ++n) out[n] = step(p, z, in(n));
    __syncthreads();
}

__global__ __launch_bounds__(NT) void filtfilt_kernel(FiltParams p, const float* x, double* work, float* out,
                                                      double* out64) {
    __shared__ double states[(NT + 1) * NS];
    double* y1 = work;
    double* y2 = work + p.L;
    const int64_t N = p.N, L = p.L;
    lfilter_pass(p, [&](int64_t i) { return ext_in(x, N, i); }, y1, ext_in(x, N, 0), states);
    const double ylast = y1[L - 1];
    lfilter_pass(p, [&](int64_t i) { return y1[L - 1 - i]; }, y2, ylast, states);
    // filtered[j] = y2[L - 1 - (PADLEN + j)]; out = reflect-pad(filtered, tpad)
    const int64_t M = N + 2 * p.tpad;
    for (int64_t k = threadIdx.x; k < M; k += NT) {
        int64_t j = k - p.tpad;
        if (j < 0) j = -j;
        if (j >= N) j = 2 * (N - 1) - j;
        const double v = y2[L - 1 - (PADLEN + j)];
        out[k] = (float)v;
        if (out64) out64[k] = v;
    }
}
}  // namespace

extern "C" int rvc_filtfilt_pad(const float* x, int64_t N, const double* b, const double* a, const double* zi,
                                const double* Ac, int64_t chunk, int64_t tpad, double* work, float* out,
                                double* out64, rvc_stream_t stream) {
    RVC_CHECK_ARG(x && b && a && zi && Ac && work && out, "filtfilt: null pointer");
    RVC_CHECK_ARG(N > PADLEN + 1 && tpad >= 0 && tpad < N, "filtfilt: N=%lld too short (needs > %d and > tpad)",
                  (long long)N, PADLEN + 1);
    FiltParams p;
    for (int i = 0; i <= NS; ++i) {
        p.b[i] = b[i];
        p.a[i] = a[i];
    }
    for (int i = 0; i < NS; ++i) p.zi[i] = zi[i];
    for (int i = 0; i < NS * NS; ++i) p.Ac[i] = Ac[i];
    p.N = N;
    p.L = N + 2 * PADLEN;
    p.c = chunk;
    p.tpad = tpad;
    RVC_CHECK_ARG(chunk * NT >= p.L && chunk > 0, "filtfilt: chunk %lld too small for L=%lld", (long long)chunk,
                  (long long)p.L);
    hipLaunchKernelGGL(filtfilt_kernel, dim3(1), dim3(NT), 0, (hipStream_t)stream, p, x, work, out, out64);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
