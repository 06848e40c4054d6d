// CREPE f0 (VC.get_f0_crepe, convert.py:230-237 -> main/library/predictors/CREPE.py) around the conv
// engine: framing/normalisation, BatchNorm + MaxPool, the masked softmax, librosa's Viterbi decode,
// bins -> Hz with dither, periodicity, the 3-tap mean / median smoothing and get_f0's coarse pitch.
#include <float.h>

#include "rvc_common.h"

#pragma clang fp contract(off)

namespace {
constexpr int WIN = 1024;
constexpr int NB = 360;  // pitch bins

// CREPE.py:151-171 (pad=True): frame f = padded[(f0 + f) * hop ...+1024], padded = 512 zeros | audio | 512
// zeros; x -= mean; x /= max(1e-10, std_unbiased).  One block per frame; f64 statistics.
__global__ __launch_bounds__(256) void crepe_frames_kernel(const float* audio, int64_t n, int hop, int64_t frame0,
                                                           float* out) {
    const int64_t f = frame0 + blockIdx.x;
    float v[4];
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = f * hop + threadIdx.x + 256 * j - WIN / 2;
        v[j] = (i >= 0 && i < n) ? audio[i] : 0.f;
        s += v[j];
    }
    __shared__ double red[4];
    auto bsum = [&](double x) {
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
        __syncthreads();
        return red[0] + red[1] + red[2] + red[3];
    };
    const float mean = (float)(bsum(s) / WIN);
    double ss = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = v[j] - mean;
        ss += (double)v[j] * v[j];
    }
    const float sd = (float)sqrt(bsum(ss) / (WIN - 1));
    const float den = sd > 1e-10f ? sd : 1e-10f;
    float* o = out + (int64_t)blockIdx.x * WIN;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[threadIdx.x + 256 * j] = v[j] / den;
}

// y [B][C][L] (ReLU already applied by the conv epilogue) -> BatchNorm(eval) + MaxPool(2): out[b][c][i] at
// out + b*obs + c*ocs + i*ois.  BN as torch's CPU eval path: alpha = w / sqrt(var + eps), beta = b - mean*alpha.
__global__ __launch_bounds__(256) void bn_maxpool_kernel(const float* y, int C, int L, const float* alpha,
                                                         const float* beta, float* out, int64_t obs, int64_t ocs,
                                                         int64_t ois) {
    const int Lo = L / 2;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (idx >= (int64_t)C * Lo) return;
    const int c = (int)(idx / Lo), i = (int)(idx - (int64_t)c * Lo);
    const float* yr = y + ((int64_t)b * C + c) * L;
    const float a = alpha[c], t = beta[c];
    const float v0 = yr[2 * i] * a + t, v1 = yr[2 * i + 1] * a + t;
    out[b * obs + c * ocs + (int64_t)i * ois] = fmaxf(v0, v1);
}

// CREPE.py:141-144 + viterbi's softmax (CREPE.py:85-86): p [360][T] sigmoid probabilities ->
// masked (bins < lo or >= hi set to -inf, in place: periodicity reads them) and softmax over bins.
__global__ __launch_bounds__(64) void crepe_softmax_kernel(float* p, int64_t T, int lo, int hi, float* sm) {
    const int64_t t = blockIdx.x;
    const int lane = threadIdx.x;
    float m = -INFINITY;
    for (int k = lane; k < NB; k += 64) {
        float v = p[(int64_t)k * T + t];
        if (k < lo || k >= hi) {
            v = -INFINITY;
            p[(int64_t)k * T + t] = v;
        }
        m = fmaxf(m, v);
    }
    m = wave_max(m);
    float s = 0.f;
    for (int k = lane; k < NB; k += 64) s += expf(p[(int64_t)k * T + t] - m);
    s = wave_sum(s);
    for (int k = lane; k < NB; k += 64) sm[(int64_t)k * T + t] = expf(p[(int64_t)k * T + t] - m) / s;
}

// librosa.sequence.viterbi(prob [360][T], transition) (restated: oracle/crepe.py) for one sequence per
// block.  value rows are f32 as in librosa (log_prob.dtype), trans_out in f64.  The CREPE transition
// max(12 - |i-j|, 0) / rowsum is zero off the band |i-j| < 12, where log(0 + tiny(f64)) is one constant:
// the off-band maximum is the global maximum of the previous row (its first index) plus that constant,
// so each state scans only its 23 in-band predecessors -- exact, including first-index tie-breaking.
__global__ __launch_bounds__(384) void crepe_viterbi_kernel(const float* sm, int64_t T, const int64_t* seq_off,
                                                            const double* log_trans, double log_off,
                                                            double log_p_init, uint16_t* ptr, int64_t* states) {
    const int64_t t0 = seq_off[blockIdx.x], t1 = seq_off[blockIdx.x + 1];
    const int j = threadIdx.x;
    __shared__ float val[2][NB];
    __shared__ float gmax_v[6];
    __shared__ int gmax_i[6];
    const float tiny = FLT_MIN;
    if (j < NB) val[0][j] = (float)((double)logf(sm[(int64_t)j * T + t0] + tiny) + log_p_init);
    __syncthreads();
    for (int64_t t = t0 + 1; t < t1; ++t) {
        const float* prev = val[(t - t0 - 1) & 1];
        float* cur = val[(t - t0) & 1];
        // global max of the previous row (first index)
        float gv = j < NB ? prev[j] : -INFINITY;
        int gi = j < NB ? j : NB;
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(gv, o, 64);
            const int oi = __shfl_xor(gi, o, 64);
            if (ov > gv || (ov == gv && oi < gi)) {
                gv = ov;
                gi = oi;
            }
        }
        if ((j & 63) == 0) {
            gmax_v[j >> 6] = gv;
            gmax_i[j >> 6] = gi;
        }
        __syncthreads();
        if (j < NB) {
            float bv = gmax_v[0];
            int bi = gmax_i[0];
            for (int w = 1; w < 6; ++w)
                if (gmax_v[w] > bv || (gmax_v[w] == bv && gmax_i[w] < bi)) {
                    bv = gmax_v[w];
                    bi = gmax_i[w];
                }
            double best = -INFINITY;
            int arg = NB;
            const int klo = j - 11 < 0 ? 0 : j - 11, khi = j + 11 > NB - 1 ? NB - 1 : j + 11;
            const bool g_in = bi >= klo && bi <= khi;
            if (!g_in && bi < klo) {  // off-band winner candidate before the band (first index)
                best = (double)bv + log_off;
                arg = bi;
            }
            for (int k = klo; k <= khi; ++k) {
                const double v = (double)prev[k] + log_trans[(int64_t)j * NB + k];  // [j][k] = log(A[k][j])
                if (v > best) {
                    best = v;
                    arg = k;
                }
            }
            if (!g_in && bi > khi) {
                const double v = (double)bv + log_off;
                if (v > best) {
                    best = v;
                    arg = bi;
                }
            }
            ptr[t * NB + j] = (uint16_t)arg;
            cur[j] = (float)((double)logf(sm[(int64_t)j * T + t] + tiny) + best);
        }
        __syncthreads();
    }
    if (j == 0) {
        const float* last = val[(t1 - 1 - t0) & 1];
        int s = 0;
        for (int k = 1; k < NB; ++k)
            if (last[k] > last[s]) s = k;
        states[t1 - 1] = s;
        for (int64_t t = t1 - 2; t >= t0; --t) {
            s = ptr[(t + 1) * NB + s];
            states[t] = s;
        }
    }
}

// bins -> Hz (CREPE.py:116-118) with dither cents, and periodicity = masked probability at the bin
__global__ __launch_bounds__(256) void crepe_freq_kernel(const int64_t* states, const float* dither, const float* p,
                                                         int64_t T, float* f0, float* pd) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    const int64_t b = states[t];
    const float cents = (float)(20 * b) + 1997.3794084376191f;
    f0[t] = 10.f * powf(2.f, (cents + dither[t]) / 1200.f);
    pd[t] = p[b * T + t];
}

// mean(f0, 3) (zero-padded, count-normalised), median(pd, 3) (reflect-padded values, zero-padded mask:
// the edge windows hold 2 valid values and take the smaller), f0[pd < 0.1] = 0  (CREPE.py:179-209,
// convert.py:235-236); then get_f0 (convert.py:310-323) in NumPy 2 semantics on the f32 f0:
// f0 *= 2^(pitch/12) (f32); mel = 1127 log(1 + f0/700) (f32); mel > 0 rescaled in f64 and stored f32;
// clamp [1, 255]; coarse = rint.
__global__ __launch_bounds__(256) void crepe_smooth_coarse_kernel(const float* f0r, const float* pd, int64_t T,
                                                                  float shift, double mel_min, double mel_max,
                                                                  rvc_f0_post post, int64_t* coarse, float* pitchf) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    const float a = t > 0 ? f0r[t - 1] : 0.f, c = t + 1 < T ? f0r[t + 1] : 0.f;
    const float cnt = (t > 0 ? 1.f : 0.f) + 1.f + (t + 1 < T ? 1.f : 0.f);
    float f = ((a + f0r[t]) + c) / cnt;
    // median of 3 over the valid window
    float med;
    if (T == 1) med = pd[0];
    else if (t == 0 || t == T - 1) med = fminf(pd[t], pd[t == 0 ? 1 : T - 2]);
    else {
        const float x = pd[t - 1], y = pd[t], z = pd[t + 1];
        med = fmaxf(fminf(x, y), fminf(fmaxf(x, y), z));
    }
    if (!isinf(med) && med < 0.1f) f = 0.f;  // an infinite median becomes NaN in the reference: kept
    f = f0_post_apply<float>(f, t, shift, post);
    float mel = 1127.f * logf(1.f + f / 700.f);
    if (mel > 0.f) mel = (float)(((double)mel - mel_min) * 254.0 / (mel_max - mel_min) + 1.0);
    if (mel <= 1.f) mel = 1.f;
    if (mel > 255.f) mel = 255.f;
    coarse[t] = (int64_t)rintf(mel);
    pitchf[t] = f;
}
}  // namespace

extern "C" int rvc_crepe_frames(const float* audio, int64_t n, int hop, int64_t frame0, int64_t nframes, float* out,
                                rvc_stream_t stream) {
    RVC_CHECK_ARG(audio && out && n > 0 && hop > 0 && frame0 >= 0 && nframes > 0 && nframes < (1 << 30),
                  "crepe_frames: bad args");
    hipLaunchKernelGGL(crepe_frames_kernel, dim3((unsigned)nframes), dim3(256), 0, (hipStream_t)stream, audio, n, hop,
                       frame0, out);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_bn_maxpool(const float* y, int64_t B, int64_t C, int64_t L, const float* alpha, const float* beta,
                              float* out, int64_t obs, int64_t ocs, int64_t ois, rvc_stream_t stream) {
    RVC_CHECK_ARG(y && alpha && beta && out && B > 0 && B < 65536 && C > 0 && L >= 2 && C * L < (1ll << 31),
                  "bn_maxpool: bad args");
    hipLaunchKernelGGL(bn_maxpool_kernel, dim3(cdiv(C * (L / 2), 256), (unsigned)B), dim3(256), 0, (hipStream_t)stream,
                       y, (int)C, (int)L, alpha, beta, out, obs, ocs, ois);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_crepe_decode(float* probs, int64_t T, int lo, int hi, const int64_t* seq_off, int nseq,
                                const double* log_trans, double log_off, double log_p_init, const float* dither,
                                void* ws, int64_t ws_bytes, float* f0_raw, float* pd_raw, rvc_stream_t stream) {
    RVC_CHECK_ARG(probs && seq_off && log_trans && dither && ws && f0_raw && pd_raw && T > 0 && nseq > 0 &&
                      0 <= lo && lo <= hi && hi <= NB, "crepe_decode: bad args");
    const int64_t need = T * NB * 4 + T * NB * 2 + T * 8;
    RVC_CHECK_ARG(ws_bytes >= need, "crepe_decode: workspace %lld < %lld", (long long)ws_bytes, (long long)need);
    float* sm = (float*)ws;
    uint16_t* ptr = (uint16_t*)(sm + T * NB);
    int64_t* states = (int64_t*)(((uintptr_t)(ptr + T * NB) + 7) & ~(uintptr_t)7);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(crepe_softmax_kernel, dim3((unsigned)T), dim3(64), 0, s, probs, T, lo, hi, sm);
    hipLaunchKernelGGL(crepe_viterbi_kernel, dim3((unsigned)nseq), dim3(384), 0, s, sm, T, seq_off, log_trans, log_off,
                       log_p_init, ptr, states);
    hipLaunchKernelGGL(crepe_freq_kernel, dim3(cdiv(T, 256)), dim3(256), 0, s, states, dither, probs, T, f0_raw,
                       pd_raw);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int64_t rvc_crepe_decode_ws_bytes(int64_t T) { return T * NB * 4 + T * NB * 2 + T * 8 + 16; }

extern "C" int rvc_crepe_smooth_coarse(const float* f0_raw, const float* pd_raw, int64_t T, float shift, double mel_min,
                                       double mel_max, const rvc_f0_post* post, int64_t* coarse, float* pitchf,
                                       rvc_stream_t stream) {
    RVC_CHECK_ARG(f0_raw && pd_raw && coarse && pitchf && T > 0, "crepe_smooth_coarse: bad args");
    RVC_CHECK_ARG(!post || !post->rep || (post->rep_off >= 0 && post->rep_len >= 0), "crepe_smooth_coarse: bad f0 post");
    const rvc_f0_post pp = f0_post_or_none(post);
    hipLaunchKernelGGL(crepe_smooth_coarse_kernel, dim3(cdiv(T, 256)), dim3(256), 0, (hipStream_t)stream, f0_raw,
                       pd_raw, T, shift, mel_min, mel_max, pp, coarse, pitchf);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
