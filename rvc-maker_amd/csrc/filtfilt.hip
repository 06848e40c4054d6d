// Zero-phase IIR high-pass (scipy.signal.filtfilt(bh, ah, x), padtype "odd", padlen 18) followed by
// the pipeline's reflect padding (convert.py:403, 416), in f64 on the device.
//
// lfilter is the transposed-direct-form-II recurrence of scipy's DOUBLE_filt:
//   y = Z0 + b0 x ;  Z_i' = Z_{i+1} + x b_{i+1} - y a_{i+1}
// It is sequential, so the (odd-extended) signal is cut into LC-sample chunks, one per lane, and
// each lane reconstructs its chunk's entry state by running the same recurrence over the WARM
// preceding samples from a zero state (the lane whose window reaches the start switches to
// zi * x0 at n = 0, exactly as scipy starts).  For this 5th-order 48 Hz Butterworth the zero-input
// transfer of the state a real signal carries has decayed below f64 resolution within a few
// thousand samples (3584 here: truncation < 1e-9 even for DC / 30 Hz content); what remains is
// rounding noise excited by the zero start (~3e-8 of full scale, measured).  A matrix-power
// or affine-scan chunk chaining is NOT used: the TDF-II
// transfer of these clustered poles is extremely non-normal (unit states peak at 1.7e7 before
// decaying), so a chained M * s amplifies rounding ~1e3x more.
//
// Memory: a wave owns 64 consecutive chunks and marches all 64 lanes through time in lockstep, so
// each PB-step tile of inputs (64 rows x PB samples) is read with coalesced row loads into LDS,
// issued one tile ahead; outputs leave through an LDS tile as coalesced row stores.  (Per-lane
// sequential loads touch 64 cache lines per instruction and serialise on vmcnt.)
#include "rvc_common.h"

#pragma clang fp contract(off)

namespace {
constexpr int NS = 5;  // filter order
constexpr int PADLEN = 18;
constexpr int LC = 512;     // output samples per lane
constexpr int WARM = 3584;  // warm-up samples per lane (multiple of PB; truncation < 1e-9 measured)
constexpr int PB = 32;      // time steps per staged tile
constexpr int RS = PB + 1;  // LDS row stride (elements)

struct FiltParams {
    double b[NS + 1], a[NS + 1], zi[NS];
    int N, L, tpad;
};

// fused multiply-adds (11 f64 ops per step instead of 21): scipy's DOUBLE_filt rounds each product
// separately, but the difference (~1e-16 per op, through the 1.7e7 state gain ~1e-9) is far below the
// chunking's own noise floor.  The recurrence is issue-bound on f64 VALU, so this halves the pass.
__device__ __forceinline__ double step(const FiltParams& p, double* z, double xn) {
    const double yn = fma(p.b[0], xn, z[0]);
#pragma unroll
    for (int i = 0; i < NS - 1; ++i) z[i] = fma(-yn, p.a[i + 1], fma(xn, p.b[i + 1], z[i + 1]));
    z[NS - 1] = fma(-yn, p.a[NS], xn * p.b[NS]);
    return yn;
}

// Pass 0 input: scipy odd_ext of the f32 signal, 2 * x[0] - x[k] evaluated in f32.  Split into a
// raw clamped load and the extension arithmetic at use time (arithmetic right after a load would
// make hipcc wait for it there).
struct ExtIn {
    const float* x;
    int N;
    float x0, xl;
    __device__ __forceinline__ float load(int n) const {
        const int k = n - PADLEN;
        int j = k < 0 ? -k : (k >= N ? 2 * (N - 1) - k : k);
        j = j < 0 ? 0 : (j >= N ? N - 1 : j);
        return x[j];
    }
    __device__ __forceinline__ double use(int n, float v) const {
        const int k = n - PADLEN;
        return (double)(k < 0 ? 2.0f * x0 - v : (k >= N ? 2.0f * xl - v : v));
    }
};

// Pass 1 input: the first pass's output reversed.
struct RevIn {
    const double* y1;
    int L;
    __device__ __forceinline__ double load(int n) const { return y1[L - 1 - (n < 0 ? 0 : (n >= L ? L - 1 : n))]; }
    __device__ __forceinline__ double use(int, double v) const { return v; }
};

// One lfilter pass over [0, L): lane r of block blk owns outputs [lo, lo + LC), lo = (blk*64 + r)*LC,
// and runs the recurrence from n = lo - WARM.
template <typename In>
__device__ __forceinline__ void pass(const FiltParams& p, const In& in, double x0, double* yout) {
    using V = decltype(in.load(0));
    __shared__ V tin[64 * RS];
    __shared__ double tout[64 * RS];
    const int lane = threadIdx.x;
    const int blo = blockIdx.x * 64 * LC;  // first output of the block
    const int lo = blo + lane * LC;
    const bool reset = blo < WARM;  // some lane's window contains n = 0 (block-uniform)
    double z[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) z[i] = 0.0;
    // staging slot: element i of a tile load covers row 2i + (lane >> 5), column lane & 31
    const int srow = lane >> 5, scol = lane & 31;
    V raw[PB];
    auto gload = [&](int t0) {
#pragma unroll
        for (int i = 0; i < PB; ++i) {
            const int row = 2 * i + srow;
            raw[i] = in.load(blo + row * LC - WARM + t0 + scol);
        }
    };
    auto sstore = [&]() {
#pragma unroll
        for (int i = 0; i < PB; ++i) tin[(2 * i + srow) * RS + scol] = raw[i];
    };
    constexpr int STEPS = WARM + LC;
    gload(0);
    sstore();
    __syncthreads();
    for (int t0 = 0; t0 < STEPS; t0 += PB) {
        const bool more = t0 + PB < STEPS;
        if (more) gload(t0 + PB);
        const bool out_phase = t0 >= WARM;
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            const int n = lo - WARM + t0 + j;
            double xn = in.use(n, tin[lane * RS + j]);
            xn = n < 0 ? 0.0 : xn;  // before the signal start: zero input, zero state
            if (reset && n == 0) {
#pragma unroll
                for (int i = 0; i < NS; ++i) z[i] = p.zi[i] * x0;
            }
            const double yn = step(p, z, xn);
            if (out_phase) tout[lane * RS + j] = yn;
        }
        __syncthreads();
        if (out_phase) {  // coalesced row stores of the tile's outputs
#pragma unroll
            for (int i = 0; i < PB; ++i) {
                const int row = 2 * i + srow;
                const int n = blo + row * LC + (t0 - WARM) + scol;
                if (n < p.L) yout[n] = tout[row * RS + scol];
            }
        }
        if (more) sstore();
        __syncthreads();
    }
}

__global__ __launch_bounds__(64) void filt_pass0(FiltParams p, const float* x, double* y1) {
    const ExtIn in{x, p.N, x[0], x[p.N - 1]};
    pass(p, in, in.use(0, in.load(0)), y1);
}

__global__ __launch_bounds__(64) void filt_pass1(FiltParams p, const double* y1, double* y2) {
    const RevIn in{y1, p.L};
    pass(p, in, y1[p.L - 1], y2);
}

// filtered[j] = y2[L - 1 - (PADLEN + j)]; out = numpy reflect-pad(filtered, tpad)
__global__ __launch_bounds__(256) void filt_reflect_pad(FiltParams p, const double* y2, float* out, double* out64) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t M = (int64_t)p.N + 2 * p.tpad;
    if (k >= M) return;
    int64_t j = k - p.tpad;
    if (j < 0) j = -j;
    if (j >= p.N) j = 2 * ((int64_t)p.N - 1) - j;
    const double v = y2[p.L - 1 - (PADLEN + j)];
    out[k] = (float)v;
    if (out64) out64[k] = v;
}
}  // namespace

extern "C" int64_t rvc_filtfilt_work_bytes(int64_t N) {
    if (N <= 0) return -1;
    return (int64_t)sizeof(double) * 2 * (N + 2 * PADLEN);
}

extern "C" int rvc_filtfilt_pad(const float* x, int64_t N, const double* b, const double* a, const double* zi,
                                int64_t tpad, double* work, float* out, double* out64, rvc_stream_t stream) {
    RVC_CHECK_ARG(x && b && a && zi && work && out, "filtfilt: null pointer");
    RVC_CHECK_ARG(N > PADLEN + 1 && tpad >= 0 && tpad < N, "filtfilt: N=%lld too short (needs > %d and > tpad)",
                  (long long)N, PADLEN + 1);
    RVC_CHECK_ARG(N + 2 * PADLEN + (int64_t)64 * LC < (1ll << 31), "filtfilt: N=%lld too long", (long long)N);
    FiltParams p;
    for (int i = 0; i <= NS; ++i) {
        p.b[i] = b[i];
        p.a[i] = a[i];
    }
    for (int i = 0; i < NS; ++i) p.zi[i] = zi[i];
    p.N = (int)N;
    p.L = (int)(N + 2 * PADLEN);
    p.tpad = (int)tpad;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(cdiv(p.L, 64 * LC));
    double* y1 = work;
    double* y2 = work + p.L;
    hipLaunchKernelGGL(filt_pass0, grid, dim3(64), 0, s, p, x, y1);
    hipLaunchKernelGGL(filt_pass1, grid, dim3(64), 0, s, p, y1, y2);
    hipLaunchKernelGGL(filt_reflect_pad, dim3(cdiv(N + 2 * tpad, 256)), dim3(256), 0, s, p, y2, out, out64);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
