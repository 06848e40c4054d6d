// pm f0 on the device: Praat's "To Pitch (ac)" as VC.get_f0_pm calls it (convert.py:206-213; time step
// 10 ms, floor 50 Hz, ceiling 1100 Hz, voicing threshold 0.6, the other arguments at parselmouth's defaults),
// then get_f0's padding / shift / autotune / f0-file / coarse steps (convert.py:304-323).  f64 throughout,
// as Praat.  Algorithm: Boersma (1993) as Praat implements it (Sound_to_Pitch_any with AC_HANNING,
// NUM_interpolate_sinc, NUMimproveMaximum's Brent search, Pitch_pathFinder); restated in oracle/pm.py --
// parity against Praat itself is unpinned (parselmouth is not installed).
//
//   pm_stats      one block: the signal mean and Praat's global peak max |x - mean|
//   pm_frames     one block per frame: local mean over +-1 longest period, Hann-windowed frame in LDS,
//                 local peak, linear autocorrelation over lags 0..479 (Praat zero-pads its FFT to 2048 >=
//                 958 + 479: the same linear correlation), normalised by the window's
//   pm_cands      one thread per frame: local maxima of r above half the voicing threshold, parabolic
//                 frequency, sinc-30 strength, the 15-slot candidate table with Praat's replacement rule
//   pm_refine     one thread per (frame, candidate): Brent maximisation of the sinc-70 interpolant
//   pm_path       one wave: the Viterbi path finder over the candidates (lanes = current candidates),
//                 then the backtrack (lane 0)
//   pm_post       get_f0_pm's zero padding to p_len, get_f0's autotune / shift / f0 file, the mel quantiser
#include "rvc_common.h"

namespace {

constexpr int PM_NCAND = 15;      // max_number_of_candidates
constexpr int PM_SR = 16000;
constexpr double PM_FLOOR = 50.0, PM_CEIL = 1100.0, PM_VOICING = 0.6, PM_SILENCE = 0.03;
constexpr double PM_OCTAVE = 0.01, PM_OCTJUMP = 0.35, PM_VUV = 0.14;
constexpr int PM_NSP = 320;       // nsamp_period = floor(sr / floor)
constexpr int PM_HP = PM_NSP / 2 + 1;
constexpr int PM_HW = 960 / 2 - 1;  // halfnsamp_window (nsamp_window = floor(0.06 sr) = 960)
constexpr int PM_NW = 2 * PM_HW;    // 958
constexpr int PM_BIX = PM_NW / 2;   // brent_ixmax = floor(958 * 0.5) = 479
constexpr int PM_MAXLAG = PM_NW / 3 + 2;  // floor(958 / 3) + 2 = 321
constexpr int PM_RY = 2 * PM_BIX + 1;     // Praat's r[-479..479] as a 1-based vector of 959

struct PmGeom {
    int64_t nx, nframes;
    double dx, x1, dt, t1;
};

// Praat's y[k] (1-based, k = lag + 480) of the mirrored correlation row r[0..479]
__device__ __forceinline__ double ry(const double* r, int k) {
    const int lag = k - PM_BIX - 1;
    return r[lag < 0 ? -lag : lag];
}

// NUM_interpolate_sinc over Praat's 1-based y[1..959]
__device__ double sinc_interp(const double* r, double x, int max_depth) {
    const int n = PM_RY;
    const int ix = (int)floor(x);
    if (x > n) return ry(r, n);
    if (x < 1) return ry(r, 1);
    if (x == ix) return ry(r, ix);
    const int midleft = ix, midright = ix + 1;
    max_depth = min(max_depth, min(midright - 1, n - midleft));
    const int left = midright - max_depth, right = midleft + max_depth;
    double result = 0.0;
    double a = M_PI * (x - midleft);
    double halfsina = 0.5 * sin(a);
    double aa = a / (x - left + 1.0);
    double daa = M_PI / (x - left + 1.0);
    for (int i = midleft; i >= left; --i) {
        result += ry(r, i) * (halfsina / a * (1.0 + cos(aa)));
        a += M_PI;
        aa += daa;
        halfsina = -halfsina;
    }
    a = M_PI * (midright - x);
    halfsina = 0.5 * sin(a);
    aa = a / (right - x + 1.0);
    daa = M_PI / (right - x + 1.0);
    for (int i = midright; i <= right; ++i) {
        result += ry(r, i) * (halfsina / a * (1.0 + cos(aa)));
        a += M_PI;
        aa += daa;
        halfsina = -halfsina;
    }
    return result;
}

__global__ __launch_bounds__(1024) void pm_stats_kernel(const double* x, int64_t n, double* stats) {
    __shared__ double red[1024];
    const int tid = threadIdx.x;
    double s = 0.0;
    for (int64_t i = tid; i < n; i += 1024) s += x[i];
    red[tid] = s;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    const double mean = red[0] / (double)n;
    __syncthreads();
    double m = 0.0;
    for (int64_t i = tid; i < n; i += 1024) m = fmax(m, fabs(x[i] - mean));
    red[tid] = m;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
        __syncthreads();
    }
    if (tid == 0) {
        stats[0] = mean;
        stats[1] = red[0];
    }
}

// r rows: [nframes][PM_BIX + 1]; intensity [nframes]
__global__ __launch_bounds__(256) void pm_frames_kernel(const double* x, PmGeom g, const double* window,
                                                        const double* window_r, const double* stats, double* r_out,
                                                        double* intensity) {
    __shared__ double fr[PM_NW];
    __shared__ double red[256];
    const int tid = threadIdx.x;
    const int64_t f = blockIdx.x;
    const double t = g.t1 + (double)f * g.dt;
    const int64_t left = (int64_t)floor((t - g.x1) / g.dx) + 1;  // Sampled_xToLowIndex (1-based)
    const int64_t right = left + 1;
    // local mean over the 1-based samples right - 320 .. left + 320
    double s = 0.0;
    for (int j = tid; j < 2 * PM_NSP; j += 256) s += x[right - PM_NSP - 1 + j];
    red[tid] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    const double mean = red[0] / (2.0 * PM_NSP);
    __syncthreads();
    const int64_t s0 = right - PM_HW - 1;  // 0-based first sample of the window
    for (int j = tid; j < PM_NW; j += 256) fr[j] = (x[s0 + j] - mean) * window[j];
    __syncthreads();
    // local peak over the frame's central +-half period (1-based j in [hw + 1 - hp, hw + hp])
    double pk = 0.0;
    for (int j = PM_HW - PM_HP + tid; j < PM_HW + PM_HP; j += 256) pk = fmax(pk, fabs(fr[j]));
    red[tid] = pk;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
        __syncthreads();
    }
    const double local_peak = red[0];
    __syncthreads();
    const double gp = stats[1];
    // (a constant signal has no global peak: Praat returns it all voiceless -- intensity 0 = no candidates)
    if (tid == 0) intensity[f] = gp == 0.0 ? 0.0 : (local_peak > gp ? 1.0 : local_peak / gp);
    // linear autocorrelation, lags 0..479, two per thread
    double* rr = r_out + f * (PM_BIX + 1);
    __shared__ double ac0;
    double acc[2] = {0.0, 0.0};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int lag = tid + 256 * u;
        if (lag <= PM_BIX) {
            double a = 0.0;
            for (int j = 0; j + lag < PM_NW; ++j) a += fr[j] * fr[j + lag];
            acc[u] = a;
        }
    }
    if (tid == 0) ac0 = acc[0];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int lag = tid + 256 * u;
        if (lag == 0) rr[0] = 1.0;
        else if (lag <= PM_BIX) rr[lag] = acc[u] / (ac0 * window_r[lag]);
    }
}

// candidate tables: cf / cs [nframes][PM_NCAND] (slot 0 = voiceless), imax [nframes][PM_NCAND], nc [nframes]
__global__ __launch_bounds__(64) void pm_cands_kernel(const double* r_all, const double* intensity, int64_t nframes,
                                                      double dx, double* cf, double* cs, int* imax, int* nc) {
    const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (f >= nframes) return;
    const double* r = r_all + f * (PM_BIX + 1);
    double* F = cf + f * PM_NCAND;
    double* S = cs + f * PM_NCAND;
    int* I = imax + f * PM_NCAND;
    int n = 1;
    F[0] = 0.0;
    S[0] = 0.0;
    I[0] = 0;
    if (intensity[f] == 0.0) {  // absolute silence: voiceless only
        nc[f] = 1;
        return;
    }
    const int offset = -PM_BIX - 1;
    for (int i = 2; i < PM_MAXLAG && i < PM_BIX; ++i) {
        const double rm = r[i - 1], r0 = r[i], rp = r[i + 1];
        if (!(r0 > 0.5 * PM_VOICING && r0 > rm && r0 >= rp)) continue;
        const double dr = 0.5 * (rp - rm), d2r = 2.0 * r0 - rm - rp;
        const double freq = 1.0 / dx / (i + dr / d2r);
        double strength = sinc_interp(r, 1.0 / dx / freq - offset, 30);
        if (strength > 1.0) strength = 1.0 / strength;
        int place = -1;
        if (n < PM_NCAND) {
            place = n++;
        } else {
            double weakest = 2.0;
            for (int iw = 1; iw < PM_NCAND; ++iw) {
                const double ls = S[iw] - PM_OCTAVE * log2(PM_FLOOR / F[iw]);
                if (ls < weakest) {
                    weakest = ls;
                    place = iw;
                }
            }
            if (strength - PM_OCTAVE * log2(PM_FLOOR / freq) <= weakest) place = -1;
        }
        if (place >= 0) {
            F[place] = freq;
            S[place] = strength;
            I[place] = i;
        }
    }
    nc[f] = n;
}

// NUMminimize_brent of -sinc_depth(r, x) over [a, b] -> (xmin, fmin)
__device__ void brent_max(const double* r, int depth, double a, double b, double& xo, double& fo) {
    const double golden = 0.3819660112501051;
    const double sqrt_eps = 1.4901161193847656e-08;  // sqrt(DBL_EPSILON)
    const double tol = 1e-10;
    double v = a + golden * (b - a);
    double fv = -sinc_interp(r, v, depth);
    double x = v, w = v, fx = fv, fw = fv;
    for (int iter = 0; iter < 60; ++iter) {
        const double middle = (a + b) / 2.0;
        const double tol_act = sqrt_eps * fabs(x) + tol / 3.0;
        if (fabs(x - middle) + (b - a) / 2.0 <= 2.0 * tol_act) break;
        double new_step = golden * (x < middle ? b - x : a - x);
        if (fabs(x - w) >= tol_act) {
            const double t = (x - w) * (fx - fv);
            double q = (x - v) * (fx - fw);
            double p = (x - v) * q - (x - w) * t;
            q = 2.0 * (q - t);
            if (q > 0.0) p = -p;
            else q = -q;
            if (fabs(p) < fabs(new_step * q) && p > q * (a - x + 2.0 * tol_act) && p < q * (b - x - 2.0 * tol_act))
                new_step = p / q;
        }
        if (fabs(new_step) < tol_act) new_step = new_step > 0.0 ? tol_act : -tol_act;
        const double t = x + new_step;
        const double ft = -sinc_interp(r, t, depth);
        if (ft <= fx) {
            if (t < x) b = x;
            else a = x;
            v = w; w = x; x = t;
            fv = fw; fw = fx; fx = ft;
        } else {
            if (t < x) a = t;
            else b = t;
            if (ft <= fw || w == x) {
                v = w; w = t;
                fv = fw; fw = ft;
            } else if (ft <= fv || v == x || v == w) {
                v = t;
                fv = ft;
            }
        }
    }
    xo = x;
    fo = fx;
}

__global__ __launch_bounds__(64) void pm_refine_kernel(const double* r_all, int64_t nframes, double dx, double* cf,
                                                       double* cs, const int* imax, const int* nc) {
    const int64_t idx = (int64_t)blockIdx.x * 64 + threadIdx.x;
    const int64_t f = idx / PM_NCAND;
    const int k = (int)(idx % PM_NCAND);
    if (f >= nframes || k == 0 || k >= nc[f]) return;
    double* F = cf + f * PM_NCAND;
    if (!(F[k] > 0.0)) return;
    const double* r = r_all + f * (PM_BIX + 1);
    const int offset = -PM_BIX - 1;
    const int depth = F[k] > 0.3 / dx ? 700 : 70;
    const double xm = (double)(imax[f * PM_NCAND + k] - offset);
    double xmid, fmin;
    brent_max(r, depth, xm - 1.0, xm + 1.0, xmid, fmin);
    double ymid = -fmin;
    xmid += offset;
    if (ymid > 1.0) ymid = 1.0 / ymid;
    F[k] = 1.0 / dx / xmid;
    cs[f * PM_NCAND + k] = ymid;
}

__device__ __forceinline__ bool pm_voiced(double f, double ceiling) { return f > 0.0 && f < ceiling; }

// One wave: delta of the current frame in registers (lane = candidate), the previous frame's in LDS;
// psi [nframes][PM_NCAND] in global memory; then lane 0 backtracks.
__global__ __launch_bounds__(64) void pm_path_kernel(const double* cf, const double* cs, const int* nc,
                                                     const double* intensity, int64_t nframes, double dt,
                                                     double ceiling, int* psi, double* f0) {
    __shared__ double prev_d[PM_NCAND], prev_f[PM_NCAND];
    const int lane = threadIdx.x;
    const double corr = 0.01 / dt;
    const double ojc = PM_OCTJUMP * corr, vuc = PM_VUV * corr;
    auto local_delta = [&](int64_t f, int k) -> double {
        double us = 2.0 - intensity[f] / (PM_SILENCE / (1.0 + PM_VOICING));
        us = PM_VOICING + (us > 0.0 ? us : 0.0);
        const double fr = cf[f * PM_NCAND + k];
        return pm_voiced(fr, ceiling) ? cs[f * PM_NCAND + k] - PM_OCTAVE * log2(ceiling / fr) : us;
    };
    if (lane < PM_NCAND) {
        prev_d[lane] = lane < nc[0] ? local_delta(0, lane) : -1e300;
        prev_f[lane] = cf[lane];
    }
    __syncthreads();
    for (int64_t f = 1; f < nframes; ++f) {
        const int n1 = nc[f - 1], n2 = nc[f];
        double best = -1e30;
        int place = 0;
        double f2 = 0.0;
        if (lane < n2) {
            f2 = cf[f * PM_NCAND + lane];
            const double cd = local_delta(f, lane);
            const bool v2 = pm_voiced(f2, ceiling);
            for (int j1 = 0; j1 < n1; ++j1) {
                const double f1 = prev_f[j1];
                const bool v1 = pm_voiced(f1, ceiling);
                double tc;
                if (!v2) tc = v1 ? vuc : 0.0;
                else tc = v1 ? ojc * fabs(log2(f1 / f2)) : vuc;
                const double v = prev_d[j1] - tc + cd;
                if (v > best) {
                    best = v;
                    place = j1;
                }
            }
            psi[f * PM_NCAND + lane] = place;
        }
        __syncthreads();
        if (lane < PM_NCAND) {
            prev_d[lane] = lane < n2 ? best : -1e300;
            prev_f[lane] = f2;
        }
        __syncthreads();
    }
    if (lane == 0) {
        const int nl = nc[nframes - 1];
        int place = 0;
        double mx = prev_d[0];
        for (int k = 1; k < nl; ++k)
            if (prev_d[k] > mx) {
                mx = prev_d[k];
                place = k;
            }
        for (int64_t f = nframes - 1; f >= 0; --f) {
            const double fr = cf[f * PM_NCAND + place];
            f0[f] = pm_voiced(fr, ceiling) ? fr : 0.0;
            if (f > 0) place = psi[f * PM_NCAND + place];
        }
    }
}

__global__ void pm_post_kernel(const double* f0, int64_t nf, int64_t nout, int64_t pad, double shift, double mel_min,
                               double mel_max, rvc_f0_post post, int64_t* coarse, float* pitchf) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nout) return;
    const int64_t s = t - pad;
    double v = (s >= 0 && s < nf) ? f0[s] : 0.0;
    v = f0_post_apply<double>(v, t, shift, post);
    double fm = 1127.0 * log(1.0 + v / 700.0);
    if (fm > 0) fm = (fm - mel_min) * 254.0 / (mel_max - mel_min) + 1.0;
    if (fm <= 1) fm = 1;
    if (fm > 255) fm = 255;
    coarse[t] = (int64_t)rint(fm);
    pitchf[t] = (float)v;
}

PmGeom pm_geom(int64_t nx) {
    PmGeom g;
    g.nx = nx;
    g.dx = 1.0 / PM_SR;
    g.x1 = 0.5 * g.dx;
    g.dt = 160.0 / 16000.0 * 1000.0 / 1000.0;  // convert.py:208's time_step expression
    const double duration = g.dx * (double)nx;
    const double dt_window = 3.0 / PM_FLOOR;
    g.nframes = duration < dt_window ? 0 : (int64_t)floor((duration - dt_window) / g.dt) + 1;
    const double mid = g.x1 - 0.5 * g.dx + 0.5 * duration;
    g.t1 = mid - 0.5 * (double)g.nframes * g.dt + 0.5 * g.dt;
    return g;
}

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

}  // namespace

extern "C" int64_t rvc_pm_frames(int64_t n) { return n > 0 ? pm_geom(n).nframes : -1; }

extern "C" int64_t rvc_pm_work_bytes(int64_t n) {
    const int64_t nf = rvc_pm_frames(n);
    if (nf <= 0) return -1;
    return (int64_t)(align256(64) + align256(sizeof(double) * PM_NW) + align256(sizeof(double) * (PM_BIX + 1)) +
                     align256(sizeof(double) * nf * (PM_BIX + 1)) + align256(sizeof(double) * nf) +
                     2 * align256(sizeof(double) * nf * PM_NCAND) + 2 * align256(sizeof(int) * nf * PM_NCAND) +
                     align256(sizeof(int) * nf));
}

extern "C" int rvc_pm_f0(const double* x, int64_t n, const double* window, const double* window_r, void* work,
                         int64_t work_bytes, double* f0, rvc_stream_t stream) {
    const int64_t nf = rvc_pm_frames(n);
    RVC_CHECK_ARG(x && window && window_r && work && f0 && n > 0, "pm_f0: bad args");
    RVC_CHECK_ARG(nf > 0, "pm_f0: %lld samples is shorter than one 60 ms analysis window", (long long)n);
    RVC_CHECK_ARG(work_bytes >= rvc_pm_work_bytes(n), "pm_f0: work buffer too small");
    const PmGeom g = pm_geom(n);
    char* w = (char*)work;
    double* stats = (double*)w; w += align256(64);
    w += align256(sizeof(double) * PM_NW) + align256(sizeof(double) * (PM_BIX + 1));  // (reserved)
    double* r = (double*)w; w += align256(sizeof(double) * nf * (PM_BIX + 1));
    double* inten = (double*)w; w += align256(sizeof(double) * nf);
    double* cf = (double*)w; w += align256(sizeof(double) * nf * PM_NCAND);
    double* cs = (double*)w; w += align256(sizeof(double) * nf * PM_NCAND);
    int* imax = (int*)w; w += align256(sizeof(int) * nf * PM_NCAND);
    int* psi = (int*)w; w += align256(sizeof(int) * nf * PM_NCAND);
    int* nc = (int*)w;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(pm_stats_kernel, dim3(1), dim3(1024), 0, s, x, n, stats);
    hipLaunchKernelGGL(pm_frames_kernel, dim3((unsigned)nf), dim3(256), 0, s, x, g, window, window_r, stats, r, inten);
    hipLaunchKernelGGL(pm_cands_kernel, dim3(cdiv(nf, 64)), dim3(64), 0, s, r, inten, nf, g.dx, cf, cs, imax, nc);
    hipLaunchKernelGGL(pm_refine_kernel, dim3(cdiv(nf * PM_NCAND, 64)), dim3(64), 0, s, r, nf, g.dx, cf, cs, imax, nc);
    hipLaunchKernelGGL(pm_path_kernel, dim3(1), dim3(64), 0, s, cf, cs, nc, inten, nf, g.dt, PM_CEIL, psi, f0);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_pm_post(const double* f0, int64_t nf, int64_t p_len, double shift, const rvc_f0_post* post,
                           int64_t* coarse, float* pitchf, rvc_stream_t stream) {
    RVC_CHECK_ARG(f0 && coarse && pitchf && nf > 0 && p_len > 0, "pm_post: bad args");
    RVC_CHECK_ARG(!post || !post->rep || (post->rep_off >= 0 && post->rep_len >= 0), "pm_post: bad f0 post");
    // get_f0_pm (convert.py:210-211): padded to p_len with (p_len - nf + 1) // 2 zero frames in front when
    // p_len > nf; a longer track is left as it is
    const bool padded = p_len > nf;
    const int64_t pad = padded ? (p_len - nf + 1) / 2 : 0;
    const int64_t nout = padded ? p_len : nf;
    const rvc_f0_post pp = f0_post_or_none(post);
    const double mel_min = 1127.0 * log(1.0 + 50.0 / 700.0), mel_max = 1127.0 * log(1.0 + 1100.0 / 700.0);
    hipLaunchKernelGGL(pm_post_kernel, dim3(cdiv(nout, 256)), dim3(256), 0, (hipStream_t)stream, f0, nf, nout,
                       pad, shift, mel_min, mel_max, pp, coarse, pitchf);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// Praat's Hanning window of Sound_to_Pitch_any (nsamp_window 958 at 16 kHz, pitch floor 50 Hz) and its
// normalised autocorrelation, on the host: window[i] = 0.5 - 0.5 cos((i + 1) 2 pi / 959), window_r[k] =
// sum_i w[i] w[i + k] / sum_i w[i]^2 for k <= 479 (sequential f64 sums, libm cos, contraction off).  The
// Python host (rvc_amd/pm.py) and the model-level C ABI (rvc_vc_convert_ex) both take them from here.
extern "C" int rvc_pm_windows(double* window, double* window_r) {
#pragma clang fp contract(off)
    RVC_CHECK_ARG(window && window_r, "pm_windows: null pointer");
    for (int i = 0; i < PM_NW; ++i) {
        const double a = (double)(i + 1) * 2.0 * M_PI / (double)(PM_NW + 1);
        window[i] = 0.5 - 0.5 * cos(a);
    }
    double r0 = 0.0;
    for (int k = 0; k <= PM_BIX; ++k) {
        double s = 0.0;
        for (int i = 0; i < PM_NW - k; ++i) s += window[i] * window[i + k];
        if (k == 0) r0 = s;
        window_r[k] = s;
    }
    for (int k = 0; k <= PM_BIX; ++k) window_r[k] /= r0;
    return RVC_OK;
}
