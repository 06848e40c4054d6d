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

// ------------------------------------------------------------------ quiet-point segmentation (convert.py:404-412)
// For inputs with n + window > t_max: audio_pad = reflect pad of the filtered f64 signal x by window/2;
// audio_sum[j] = sum_{i < window} audio_pad[j + i], accumulated in i order (numpy's `audio_sum +=
// audio_pad[i : i - window]` loop, f64); for each t in range(t_center, n, t_center) the quiet point is
// t - t_query + the first index of min |audio_sum[t - t_query : t + t_query]|.  Exact: the same f64 sums in
// the same order, the argmin's ties to the lower index.
constexpr int QP_CH = 1024;  // window positions per block
constexpr int QP_WMAX = 512;

__device__ __forceinline__ double qp_pad(const double* x, int64_t n, int64_t k, int half) {
    int64_t j = k - half;  // np.pad(x, (half, half), "reflect")
    if (j < 0) j = -j;
    if (j >= n) j = 2 * (n - 1) - j;
    return x[j];
}

// grid (cdiv(2 t_query, QP_CH), npts): partial (min |sum|, first index) per chunk of a point's window
__global__ __launch_bounds__(256) void quiet_partial_kernel(const double* x, int64_t n, int window, int64_t t_center,
                                                            int64_t t_query, double* pv, int64_t* pi) {
    __shared__ double tile[QP_CH + QP_WMAX];
    __shared__ double rv[256];
    __shared__ int64_t ri[256];
    const int64_t t = (int64_t)(blockIdx.y + 1) * t_center;
    const int64_t lo = t - t_query, hi = t + t_query < n ? t + t_query : n;  // numpy slice [lo, hi)
    const int64_t j0 = lo + (int64_t)blockIdx.x * QP_CH;
    const int span = QP_CH + window - 1;
    for (int i = threadIdx.x; i < span; i += 256) {
        const int64_t k = j0 + i;  // audio_pad index of sum j's i-th term: j + i
        tile[i] = k < n + window ? qp_pad(x, n, k, window / 2) : 0.0;
    }
    __syncthreads();
    double best = INFINITY;
    int64_t bi = INT64_MAX;
    for (int q = threadIdx.x; q < QP_CH; q += 256) {  // ascending j per thread: the first minimum wins
        const int64_t j = j0 + q;
        if (j >= hi) break;
        double s = 0.0;
        for (int i = 0; i < window; ++i) s += tile[q + i];
        const double a = fabs(s);
        if (a < best) {
            best = a;
            bi = j;
        }
    }
    rv[threadIdx.x] = best;
    ri[threadIdx.x] = bi;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            const double v2 = rv[threadIdx.x + o];
            const int64_t i2 = ri[threadIdx.x + o];
            if (v2 < rv[threadIdx.x] || (v2 == rv[threadIdx.x] && i2 < ri[threadIdx.x])) {
                rv[threadIdx.x] = v2;
                ri[threadIdx.x] = i2;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        pv[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = rv[0];
        pi[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = ri[0];
    }
}

__global__ void quiet_final_kernel(const double* pv, const int64_t* pi, int nchunk, int64_t t_query, int64_t t_center,
                                   int64_t* opt_ts) {
    const int p = blockIdx.x;
    double best = INFINITY;
    int64_t bi = INT64_MAX;
    for (int c = 0; c < nchunk; ++c) {  // chunks in window order: strict < keeps the first minimum
        const double v = pv[(int64_t)p * nchunk + c];
        if (v < best) {
            best = v;
            bi = pi[(int64_t)p * nchunk + c];
        }
    }
    if (threadIdx.x == 0) opt_ts[p] = bi;  // t - t_query + offset == the absolute index j of the minimum
}

extern "C" int64_t rvc_quiet_points_count(int64_t n, int window, int64_t t_center, int64_t t_max) {
    if (n <= 0 || window <= 0 || t_center <= 0) return -1;
    if (n + 2 * (window / 2) <= t_max) return 0;
    return n > t_center ? (n - 1) / t_center : 0;  // len(range(t_center, n, t_center))
}

extern "C" int64_t rvc_quiet_points_ws_bytes(int64_t n, int window, int64_t t_center, int64_t t_query, int64_t t_max) {
    const int64_t np = rvc_quiet_points_count(n, window, t_center, t_max);
    if (np < 0) return -1;
    return np * cdiv(2 * t_query, QP_CH) * 16;
}

extern "C" int rvc_quiet_points(const double* x, int64_t n, int window, int64_t t_center, int64_t t_query,
                                int64_t t_max, void* ws, int64_t ws_bytes, int64_t* opt_ts, rvc_stream_t stream) {
    const int64_t np = rvc_quiet_points_count(n, window, t_center, t_max);
    RVC_CHECK_ARG(x && opt_ts && np >= 0 && window >= 2 && window <= QP_WMAX && window % 2 == 0 && t_query > 0 &&
                      t_query <= t_center && n > window, "quiet_points: bad args");
    if (np == 0) return RVC_OK;
    const int nchunk = (int)cdiv(2 * t_query, QP_CH);
    RVC_CHECK_ARG(ws && ws_bytes >= np * nchunk * 16 && np < 65536, "quiet_points: workspace too small");
    double* pv = (double*)ws;
    int64_t* pi = (int64_t*)(pv + np * nchunk);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(quiet_partial_kernel, dim3(nchunk, (unsigned)np), dim3(256), 0, s, x, n, window, t_center,
                       t_query, pv, pi);
    hipLaunchKernelGGL(quiet_final_kernel, dim3((unsigned)np), dim3(64), 0, s, pv, pi, nchunk, t_query, t_center,
                       opt_ts);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
