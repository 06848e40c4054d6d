// Memory-bound kernels of the synthesizer path (HBM-bound; one pass each).
#include "rvc_common.h"

// ---------------------------------------------------------------- Philox4x32-10 + Box-Muller
RVC_DEV void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

// kind 0: standard normals (Box-Muller); kind 1: symmetric triangular on [lo, hi] (inverse CDF).
// seed_add (device, may be null) is added to the seed at run time, so that a captured graph draws
// fresh noise on every replay (graph.py).
__global__ void rand_kernel(float* out, int64_t n, uint64_t seed, uint64_t offset, const uint64_t* seed_add, int kind,
                            float lo, float hi) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one thread -> 4 draws
    int64_t base = i * 4;
    if (base >= n) return;
    if (seed_add) seed += *seed_add;
    uint64_t ctr = (uint64_t)i + offset;
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0x7A3Bu, 0x52u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    float r[4];
    if (kind == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float u1 = ((c[2 * j] >> 8) + 1) * (1.0f / 16777216.0f);  // (0, 1]
            float u2 = (c[2 * j + 1] >> 8) * (1.0f / 16777216.0f);
            float rad = sqrtf(-2.0f * logf(u1));
            float s, co;
            sincosf(6.2831853071795864f * u2, &s, &co);
            r[2 * j] = rad * co;
            r[2 * j + 1] = rad * s;
        }
    } else {
        const float w = hi - lo;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float u = ((c[j] >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
            r[j] = u < 0.5f ? lo + w * sqrtf(0.5f * u) : hi - w * sqrtf(0.5f * (1.0f - u));
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (base + j < n) out[base + j] = r[j];
}

static int launch_rand(float* out, int64_t n, uint64_t seed, uint64_t offset, const uint64_t* seed_add, int kind,
                       float lo, float hi, rvc_stream_t stream) {
    RVC_CHECK_ARG(out && n >= 0, "rand: bad args");
    if (n == 0) return RVC_OK;
    int64_t thr = (n + 3) / 4;
    hipLaunchKernelGGL(rand_kernel, dim3(cdiv(thr, 256)), dim3(256), 0, (hipStream_t)stream, out, n, seed, offset,
                       seed_add, kind, lo, hi);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_randn(float* out, int64_t n, uint64_t seed, uint64_t offset, rvc_stream_t stream) {
    return launch_rand(out, n, seed, offset, nullptr, 0, 0.f, 0.f, stream);
}

extern "C" int rvc_randn_ex(float* out, int64_t n, uint64_t seed, uint64_t offset, const uint64_t* seed_add,
                            rvc_stream_t stream) {
    return launch_rand(out, n, seed, offset, seed_add, 0, 0.f, 0.f, stream);
}

extern "C" int rvc_rand_triang(float* out, int64_t n, float lo, float hi, uint64_t seed, uint64_t offset,
                               const uint64_t* seed_add, rvc_stream_t stream) {
    RVC_CHECK_ARG(hi > lo, "rand_triang: hi <= lo");
    return launch_rand(out, n, seed, offset, seed_add, 1, lo, hi, stream);
}

// ---------------------------------------------------------------- TextEncoder input
// out[c][t] = lrelu((lin[c][t] + emb[pitch[t]][c]) * scale, slope)     (synthesizers.py:367)
// amax_out (or null): max |out| per batch element into a |max| cell (the first QKV projection's split-fp16 scale)
__global__ void textenc_embed_kernel(const float* lin, const float* emb, const int64_t* pitch, float* out, int C,
                                     int64_t T, float scale, float slope, unsigned* amax_out) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int c = blockIdx.y;
    int b = blockIdx.z;
    float m = 0.f;
    if (t < T) {
        int64_t o = ((int64_t)b * C + c) * T + t;
        float v = lin[o];
        if (emb) v += emb[pitch[(int64_t)b * T + t] * C + c];
        v *= scale;
        v = v >= 0.f ? v : v * slope;
        out[o] = v;
        m = fabsf(v);
    }
    if (amax_out) amax_publish_block(amax_out + (int64_t)b * RVC_AMAX_SHARDS, m);  // one atomic per block
}

extern "C" int rvc_textenc_embed_amax(const float* lin, const float* emb, const int64_t* pitch, float* out, int64_t B,
                                      int64_t C, int64_t T, float scale, float slope, unsigned* amax_out,
                                      rvc_stream_t stream) {
    RVC_CHECK_ARG(lin && out && (!emb || pitch) && B > 0 && C > 0 && T > 0, "textenc_embed: bad args");
    hipLaunchKernelGGL(textenc_embed_kernel, dim3(cdiv(T, 256), (unsigned)C, (unsigned)B), dim3(256), 0,
                       (hipStream_t)stream, lin, emb, pitch, out, (int)C, T, scale, slope, amax_out);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_textenc_embed(const float* lin, const float* emb, const int64_t* pitch, float* out, int64_t B,
                                 int64_t C, int64_t T, float scale, float slope, rvc_stream_t stream) {
    return rvc_textenc_embed_amax(lin, emb, pitch, out, B, C, T, scale, slope, nullptr, stream);
}

// ---------------------------------------------------------------- prior sample
// z_p[c][t] = (m[c][t] + exp(logs[c][t]) * noise[c][t] * 0.66666) * mask   (synthesizers.py:449)
// stats = [m; logs] stacked on channels ([2C][T]); mask is all ones at full length.
__global__ void prior_kernel(const float* stats, const float* noise, float* zp, int C, int64_t T, float nscale) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int c = blockIdx.y, b = blockIdx.z;
    if (t >= T) return;
    const float* sb = stats + (int64_t)b * 2 * C * T;
    float m = sb[(int64_t)c * T + t];
    float lg = sb[(int64_t)(c + C) * T + t];
    int64_t o = ((int64_t)b * C + c) * T + t;
    zp[o] = (m + expf(lg) * noise[o] * nscale);
}

extern "C" int rvc_prior_sample(const float* stats, const float* noise, float* zp, int64_t B, int64_t C, int64_t T,
                                float nscale, rvc_stream_t stream) {
    RVC_CHECK_ARG(stats && noise && zp && B > 0 && C > 0 && T > 0, "prior_sample: bad args");
    hipLaunchKernelGGL(prior_kernel, dim3(cdiv(T, 256), (unsigned)C, (unsigned)B), dim3(256), 0, (hipStream_t)stream,
                       stats, noise, zp, (int)C, T, nscale);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- WaveNet gate
// out[c][t] = tanh(a[c][t]) * sigmoid(a[c+H][t])     (commons.py:35-41; the cond term is
// already in a through the conv's bias2)
__global__ void gate_kernel(const float* a, float* out, int H, int64_t T) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int c = blockIdx.y, b = blockIdx.z;
    if (t >= T) return;
    const float* ab = a + (int64_t)b * 2 * H * T;
    float x0 = ab[(int64_t)c * T + t], x1 = ab[(int64_t)(c + H) * T + t];
    out[((int64_t)b * H + c) * T + t] = tanhf(x0) * (1.f / (1.f + expf(-x1)));
}

extern "C" int rvc_gate(const float* a, float* out, int64_t B, int64_t H, int64_t T, rvc_stream_t stream) {
    RVC_CHECK_ARG(a && out && B > 0 && H > 0 && T > 0, "gate: bad args");
    hipLaunchKernelGGL(gate_kernel, dim3(cdiv(T, 256), (unsigned)H, (unsigned)B), dim3(256), 0, (hipStream_t)stream,
                       a, out, (int)H, T);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- channel flip  (residuals.py:53-58)
__global__ void flip_kernel(const float* x, float* out, int C, int64_t T) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int c = blockIdx.y, b = blockIdx.z;
    if (t >= T) return;
    out[((int64_t)b * C + c) * T + t] = x[((int64_t)b * C + (C - 1 - c)) * T + t];
}

extern "C" int rvc_flip_channels(const float* x, float* out, int64_t B, int64_t C, int64_t T, rvc_stream_t stream) {
    RVC_CHECK_ARG(x && out && x != out && B > 0 && C > 0 && T > 0, "flip: bad args");
    hipLaunchKernelGGL(flip_kernel, dim3(cdiv(T, 256), (unsigned)C, (unsigned)B), dim3(256), 0, (hipStream_t)stream,
                       x, out, (int)C, T);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- 2-D transpose (batched)
__global__ void transpose_kernel(const float* in, float* out, int64_t R, int64_t C) {
    __shared__ float tile[32][33];
    int b = blockIdx.z;
    const float* ib = in + (int64_t)b * R * C;
    float* ob = out + (int64_t)b * R * C;
    int64_t c0 = (int64_t)blockIdx.x * 32, r0 = (int64_t)blockIdx.y * 32;
    int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
    for (int k = ty; k < 32; k += 8) {
        int64_t r = r0 + k, c = c0 + tx;
        tile[k][tx] = (r < R && c < C) ? ib[r * C + c] : 0.f;
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        int64_t c = c0 + k, r = r0 + tx;
        if (c < C && r < R) ob[c * R + r] = tile[tx][k];
    }
}

extern "C" int rvc_transpose(const float* in, float* out, int64_t B, int64_t R, int64_t C, rvc_stream_t stream) {
    RVC_CHECK_ARG(in && out && in != out && B > 0 && R > 0 && C > 0, "transpose: bad args");
    hipLaunchKernelGGL(transpose_kernel, dim3(cdiv(C, 32), cdiv(R, 32), (unsigned)B), dim3(256), 0,
                       (hipStream_t)stream, in, out, R, C);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- NSF source (SineGen + SourceModuleHnNSF)
// synthesizers.py:82-112, harmonic_num = 0.  Frame phase offsets follow torch-CPU's
// float32 cumsum exactly: f32 increments, f64 running sum, f32 per-element result,
// then fmodf (SURVEY §0 "CPU-only precision traps").
__global__ void sine_offsets_kernel(const float* f0, float* off, int64_t T, float sr, float upp) {
    // one block of 1024 per batch row: exclusive f64 prefix over frames
    __shared__ double part[1024];
    const int b = blockIdx.x;
    const float* fb = f0 + (int64_t)b * T;
    float* ob = off + (int64_t)b * T;
    const int tid = threadIdx.x;
    const int64_t per = (T + 1023) / 1024;
    const int64_t lo = tid * per, hi = lo + per < T ? lo + per : T;
    double s = 0.0;
    for (int64_t t = lo; t < hi; ++t) {
        if (t >= T - 1) break;  // increments exist for frames 0..T-2
        float r = (fb[t] / sr) * upp;
        float inc = fmodf(r + 0.5f, 1.0f) - 0.5f;
        s += (double)inc;
    }
    part[tid] = s;
    __syncthreads();
    // inclusive scan over 1024 partials (Hillis-Steele in f64)
    for (int o = 1; o < 1024; o <<= 1) {
        double v = tid >= o ? part[tid - o] : 0.0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    double run = tid > 0 ? part[tid - 1] : 0.0;
    for (int64_t t = lo; t < hi; ++t) {
        // offset for frame t = fmod(cum[t-1], 1) with cum[-1] := padded 0
        ob[t] = (t == 0) ? 0.f : fmodf((float)run, 1.0f);
        if (t < T - 1) {
            float r = (fb[t] / sr) * upp;
            float inc = fmodf(r + 0.5f, 1.0f) - 0.5f;
            run += (double)inc;
        }
    }
}

__global__ void sine_source_kernel(const float* f0, const float* off, const float* noise, float* har, int64_t T,
                                   int upp, float sr, float lw, float lb) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int b = blockIdx.y;
    int64_t L = T * upp;
    if (i >= L) return;
    int64_t t = i / upp;
    int j = (int)(i - t * upp);
    float f = f0[(int64_t)b * T + t];
    float rad = (f / sr) * (float)(j + 1) + off[(int64_t)b * T + t];
    float s = sinf(6.2831855f * rad) * 0.1f;
    float uv = f > 0.f ? 1.f : 0.f;
    float n = noise[(int64_t)b * L + i];
    float v = s * uv + ((uv * 0.003f + ((1.f - uv) * 0.1f) / 3.0f) * n);
    har[(int64_t)b * L + i] = tanhf(v * lw + lb);
}

extern "C" int rvc_sine_source(const float* f0, const float* noise, float* har, float* work, int64_t B, int64_t T,
                               int upp, float sr, float lin_w, float lin_b, rvc_stream_t stream) {
    RVC_CHECK_ARG(f0 && noise && har && work && B > 0 && T > 0 && upp > 0, "sine_source: bad args");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(sine_offsets_kernel, dim3((unsigned)B), dim3(1024), 0, s, f0, work, T, sr, (float)upp);
    RVC_HIP(hipGetLastError());
    hipLaunchKernelGGL(sine_source_kernel, dim3(cdiv(T * upp, 256), (unsigned)B), dim3(256), 0, s, f0, work, noise,
                       har, T, upp, sr, lin_w, lin_b);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- change_rms (convert.py:150-152)
// librosa.feature.rms(y, frame_length = 2*hop, hop_length = hop): centered frames over the zero-padded
// signal, mean of the f32 squares (librosa's abs2 dtype=float32), sqrt in f32.  One block per frame.
namespace {
__global__ __launch_bounds__(256) void rms_frames_kernel(const double* y64, const float* y32, int64_t n, int64_t hop,
                                                         float* out) {
    const int64_t f = blockIdx.x;
    const int64_t lo = f * hop - hop, hi = lo + 2 * hop;  // original-index window [lo, hi)
    const int64_t a = lo < 0 ? 0 : lo, b = hi > n ? n : hi;
    double acc = 0.0;
    for (int64_t i = a + threadIdx.x; i < b; i += 256) {
        const float v = y64 ? (float)y64[i] : y32[i];
        acc += (double)(v * v);
    }
    __shared__ double part[256];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[f] = sqrtf((float)(part[0] / (double)(2 * hop)));
}

// torch F.interpolate(mode="linear", align_corners=False) of r [m] to n points, at output index i.
__device__ __forceinline__ float interp_linear(const float* r, int64_t m, int64_t n, int64_t i) {
#pragma clang fp contract(off)
    const float scale = (float)m / (float)n;
    float src = scale * ((float)i + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    int64_t i0 = (int64_t)src;
    if (i0 > m - 1) i0 = m - 1;
    const int64_t i1 = i0 + (i0 < m - 1 ? 1 : 0);
    const float l1 = src - (float)i0, l0 = 1.f - l1;
    return l0 * r[i0] + l1 * r[i1];
}

__global__ __launch_bounds__(256) void rms_mix_kernel(float* y, int64_t n, const float* r1, int64_t n1, const float* r2,
                                                      int64_t n2, float e1, float e2) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float a = interp_linear(r1, n1, n, i);
    const float b = fmaxf(interp_linear(r2, n2, n, i), 1e-6f);
    y[i] = y[i] * powf(a, e1) * powf(b, e2);
}
}  // namespace

extern "C" int64_t rvc_rms_frames_len(int64_t n, int64_t hop) { return (n < 0 || hop <= 0) ? -1 : 1 + n / hop; }

extern "C" int rvc_rms_frames(const double* y64, const float* y32, int64_t n, int64_t hop, float* out,
                              rvc_stream_t stream) {
    RVC_CHECK_ARG((y64 || y32) && out && n > 0 && hop > 0, "rms_frames: bad args");
    hipLaunchKernelGGL(rms_frames_kernel, dim3((unsigned)(1 + n / hop)), dim3(256), 0, (hipStream_t)stream, y64, y32,
                       n, hop, out);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_rms_mix(float* y, int64_t n, const float* r1, int64_t n1, const float* r2, int64_t n2, double rate,
                           rvc_stream_t stream) {
    RVC_CHECK_ARG(y && r1 && r2 && n > 0 && n1 > 0 && n2 > 0, "rms_mix: bad args");
    // torch.pow(r, 1 - rate): the exponent is the python float 1 - rate, taken as f32 by the op
    const double rd = rate;
    hipLaunchKernelGGL(rms_mix_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, y, n, r1, n1, r2, n2,
                       (float)(1.0 - rd), (float)(rd - 1.0));
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
