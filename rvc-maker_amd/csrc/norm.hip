// Normalisations over the channels-first activations ([B][C][T], t contiguous).
#include "rvc_common.h"
#include <stdlib.h>

// ---------------------------------------------------------------- LayerNorm over channels
// out[c][t] = (v - mean_t) * rstd_t * gamma[c] + beta[c],  v = x[c][t] (+ res[c][t])
// A block owns 16 columns: the [C][16] tile is read once from HBM into LDS (64-B row
// segments), 16 threads reduce each column (two-pass mean / variance, as F.layer_norm),
// then the tile is written back.  Covers synthesizers.py:170-181 and the fairseq
// LayerNorms (fairseq.py:700, 1418, 1104) on this build's [C][T] layout.
// The staging loop issues LN_UNROLL rows' loads before it uses any (C is a runtime value, so an
// un-unrolled loop waited one HBM latency per row: 28 us for a 768 x 1599 tile set).
constexpr int LN_UNROLL = 24;

__global__ __launch_bounds__(256) void layernorm_cf_kernel(const float* x, const float* res, const float* gamma,
                                                           const float* beta, float* out, int C, int64_t T,
                                                           float eps, unsigned* amax_out) {
    extern __shared__ __attribute__((aligned(16))) float tile[];  // [C][17]
    const int tid = threadIdx.x;
    const int col = tid & 15, grp = tid >> 4;  // 16 columns x 16 channel groups
    const int b = blockIdx.y;
    const int64_t t0 = (int64_t)blockIdx.x * 16;
    const int64_t t = t0 + col;
    const bool ok = t < T;
    const int64_t tc = ok ? t : T - 1;  // clamped: every load is issued, masked at use
    const float* xb = x + (int64_t)b * C * T + tc;
    const float* rb = res ? res + (int64_t)b * C * T + tc : nullptr;
    float s = 0.f;
    for (int c0 = grp; c0 < C; c0 += 16 * LN_UNROLL) {
        float v[LN_UNROLL], r[LN_UNROLL];
#pragma unroll
        for (int u = 0; u < LN_UNROLL; ++u) {
            const int c = c0 + 16 * u;
            const int cc = c < C ? c : C - 1;
            v[u] = xb[(int64_t)cc * T];
            r[u] = rb ? rb[(int64_t)cc * T] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < LN_UNROLL; ++u) {
            const int c = c0 + 16 * u;
            if (c < C) {
                const float w = ok ? (rb ? v[u] + r[u] : v[u]) : 0.f;
                tile[c * 17 + col] = w;
                s += w;
            }
        }
    }
    float* red = tile + C * 17;  // [16][17]
    red[grp * 17 + col] = s;
    __syncthreads();
    float mean = 0.f;
    for (int g = 0; g < 16; ++g) mean += red[g * 17 + col];
    mean /= (float)C;
    float q = 0.f;
    for (int c = grp; c < C; c += 16) {
        float d = tile[c * 17 + col] - mean;
        q += d * d;
    }
    __syncthreads();
    red[grp * 17 + col] = q;
    __syncthreads();
    float var = 0.f;
    for (int g = 0; g < 16; ++g) var += red[g * 17 + col];
    const float rstd = 1.0f / sqrtf(var / (float)C + eps);
    float* ob = out + (int64_t)b * C * T;
    float amx = 0.f;  // amax_out: largest |stored value| of this thread
    if (ok) {
        for (int c = grp; c < C; c += 16) {
            const float y = (tile[c * 17 + col] - mean) * rstd * gamma[c] + beta[c];
            ob[(int64_t)c * T + t] = y;
            amx = fmaxf(amx, fabsf(y));
        }
    }
    if (amax_out) amax_publish_block(amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);  // one atomic per block
}

// Register-resident form for the path's small column counts (ContentVec: 1599 columns, TextEncoder: 3198):
// a block of 16 waves owns 16 columns, 64 channel groups of CPT channels each; every thread loads its CPT
// values (x + res) at once, keeps them in registers through the two-pass mean / variance (sums reduced over the
// wave's 4 groups by shuffles, then over the 16 waves through LDS) and writes the normalised values from
// them.  4x the waves of the LDS-tile form per column block, no tile round trip.
// amax_out (or null): max |out| folded into a |max| cell (rvc_conv1d_args.amax_in of the GEMM that reads out)
template <int CPT>
__global__ __launch_bounds__(1024) void layernorm_cf_reg_kernel(const float* x, const float* res, const float* gamma,
                                                                const float* beta, float* out, int C, int64_t T,
                                                                float eps, unsigned* amax_out) {
    const int tid = threadIdx.x;
    const int col = tid & 15, grp = tid >> 4, wv = tid >> 6;  // 16 columns x 64 channel groups
    const int b = blockIdx.y;
    const int64_t t = (int64_t)blockIdx.x * 16 + col;
    const bool ok = t < T;
    const int64_t tc = ok ? t : T - 1;
    const float* xb = x + (int64_t)b * C * T + tc;
    const float* rb = res ? res + (int64_t)b * C * T + tc : nullptr;
    float v[CPT], r[CPT];
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
        const int c = grp + 64 * u;
        const int cc = c < C ? c : C - 1;
        v[u] = xb[(int64_t)cc * T];
        r[u] = rb ? rb[(int64_t)cc * T] : 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
        v[u] = rb ? v[u] + r[u] : v[u];
        if (grp + 64 * u < C) s += v[u];
    }
    __shared__ float red[2][16][16];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if ((tid & 63) < 16) red[0][wv][col] = s;
    __syncthreads();
    float mean = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) mean += red[0][w][col];
    mean /= (float)C;
    float q = 0.f;
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
        const float d = v[u] - mean;
        if (grp + 64 * u < C) q += d * d;
    }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    if ((tid & 63) < 16) red[1][wv][col] = q;
    __syncthreads();
    float var = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) var += red[1][w][col];
    const float rstd = 1.0f / sqrtf(var / (float)C + eps);
    float* ob = out + (int64_t)b * C * T + tc;
    float amx = 0.f;
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
        const int c = grp + 64 * u;
        if (ok && c < C) {
            const float y = (v[u] - mean) * rstd * gamma[c] + beta[c];
            ob[(int64_t)c * T] = y;
            amx = fmaxf(amx, fabsf(y));
        }
    }
    if (amax_out) amax_publish_block(amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);  // one atomic per block
}

extern "C" int rvc_layernorm_cf(const float* x, const float* res, const float* gamma, const float* beta, float* out,
                                int64_t B, int64_t C, int64_t T, float eps, rvc_stream_t stream) {
    return rvc_layernorm_cf_amax(x, res, gamma, beta, out, B, C, T, eps, nullptr, stream);
}

extern "C" int rvc_layernorm_cf_amax(const float* x, const float* res, const float* gamma, const float* beta,
                                     float* out, int64_t B, int64_t C, int64_t T, float eps, unsigned* amax_out,
                                     rvc_stream_t stream) {
    RVC_CHECK_ARG(x && gamma && beta && out && B > 0 && C > 0 && T > 0, "layernorm_cf: bad args");
    RVC_CHECK_ARG(C <= 2048, "layernorm_cf: C=%lld > 2048", (long long)C);
    static const int reg = getenv("RVC_LN_REG") ? atoi(getenv("RVC_LN_REG")) : 1;
    // measured (scripts/micro.py norms): C=768 T=1599 19.6 -> 12.0 us, C=512 12.0 -> 9.0; C=192 T=3198 8.7 -> 9.2
    // (the LDS-tile form keeps C <= 256)
    if (reg && C > 256 && C <= 768) {
        const dim3 grid(cdiv(T, 16), (unsigned)B);
        hipStream_t s = (hipStream_t)stream;
        if (C <= 512)
            hipLaunchKernelGGL(layernorm_cf_reg_kernel<8>, grid, dim3(1024), 0, s, x, res, gamma, beta, out, (int)C, T,
                               eps, amax_out);
        else
            hipLaunchKernelGGL(layernorm_cf_reg_kernel<12>, grid, dim3(1024), 0, s, x, res, gamma, beta, out, (int)C,
                               T, eps, amax_out);
        RVC_HIP(hipGetLastError());
        return RVC_OK;
    }
    size_t lds = (size_t)(C + 16) * 17 * 4;
    hipLaunchKernelGGL(layernorm_cf_kernel, dim3(cdiv(T, 16), (unsigned)B), dim3(256), lds, (hipStream_t)stream, x,
                       res, gamma, beta, out, (int)C, T, eps, amax_out);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- per-channel norm (+GELU)
// GroupNorm(C, C) over time, affine, then exact GELU: the ContentVec conv feature
// extractor's first block (fairseq.py:1149-1155, 1183-1185).  One block per (b, c): the row's mean
// and variance in one pass over it (sums of x - x[0] and its square: the shift keeps the
// E[d^2] - E[d]^2 form well conditioned for a row whose mean is small against its spread), then the
// normalise + GELU pass; every pass issues CN_UNROLL loads per thread before using them.
constexpr int CN_UNROLL = 8;

__global__ __launch_bounds__(256) void chnorm_gelu_kernel(const float* x, const float* gamma, const float* beta,
                                                          float* out, int C, int64_t L, float eps, int gelu) {
    const int c = blockIdx.x, b = blockIdx.y;
    const float* xr = x + ((int64_t)b * C + c) * L;
    float* orow = out + ((int64_t)b * C + c) * L;
    __shared__ float red[2][4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float shift = xr[0];
    float s = 0.f, q = 0.f;
    for (int64_t i0 = tid; i0 < L; i0 += 256 * CN_UNROLL) {
        float v[CN_UNROLL];
#pragma unroll
        for (int u = 0; u < CN_UNROLL; ++u) {
            const int64_t i = i0 + 256 * u;
            v[u] = xr[i < L ? i : L - 1];
        }
#pragma unroll
        for (int u = 0; u < CN_UNROLL; ++u) {
            const float d = i0 + 256 * u < L ? v[u] - shift : 0.f;
            s += d;
            q += d * d;
        }
    }
    s = wave_sum(s);
    q = wave_sum(q);
    if (lane == 0) {
        red[0][w] = s;
        red[1][w] = q;
    }
    __syncthreads();
    const float ms = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / (float)L;  // mean of x - shift
    const float mq = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) / (float)L;
    const float mean = shift + ms;
    const float rstd = 1.0f / sqrtf(fmaxf(mq - ms * ms, 0.f) + eps);
    const float g = gamma[c], bt = beta[c];
    for (int64_t i0 = tid; i0 < L; i0 += 256 * CN_UNROLL) {
        float v[CN_UNROLL];
#pragma unroll
        for (int u = 0; u < CN_UNROLL; ++u) {
            const int64_t i = i0 + 256 * u;
            v[u] = xr[i < L ? i : L - 1];
        }
#pragma unroll
        for (int u = 0; u < CN_UNROLL; ++u) {
            const int64_t i = i0 + 256 * u;
            const float y = (v[u] - mean) * rstd * g + bt;
            if (i < L) orow[i] = gelu ? act_apply(y, RVC_ACT_GELU, 0.f) : y;
        }
    }
}

extern "C" int rvc_chnorm_gelu(const float* x, const float* gamma, const float* beta, float* out, int64_t B, int64_t C,
                               int64_t L, float eps, int gelu, rvc_stream_t stream) {
    RVC_CHECK_ARG(x && gamma && beta && out && B > 0 && C > 0 && L > 0, "chnorm_gelu: bad args");
    hipLaunchKernelGGL(chnorm_gelu_kernel, dim3((unsigned)C, (unsigned)B), dim3(256), 0, (hipStream_t)stream, x, gamma,
                       beta, out, (int)C, L, eps, gelu);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- ContentVec's first layer, fused (round 5)
// conv(1 -> C, k K, stride S) + GroupNorm(C, C) over time + affine + exact GELU (fairseq.py:1165-1195 layer 0) without
// the [C][T] conv output's HBM round trip: the conv (K FMAs per output) is cheap enough to compute twice.
//   fe0_stats:  per (time tile, channel) f64 sum / sum of squares of the conv outputs  -> ws partials
//   fe0_final:  per channel, the partials in tile order -> mean, 1 / sqrt(var + eps)
//   fe0_apply:  the conv again (the same fmaf chain, so the same bits), normalise, GELU, one coalesced write, and
//               (amax_out) the output's |max| into a cell for the split-fp16 conv of layer 1
// The separate conv + chnorm_gelu wrote the 210 MB output of a 32 s input at 0.4 TB/s and read it twice.
// Round 6: the tap loops are fully unrolled to FE0_KMAX with a uniform k < K guard -- with a run-time trip count the
// per-thread weight / sample arrays were indexed dynamically and lived in scratch (round 5: 273 + 389 us per 32 s
// input for stats + apply), and fe0_final issues its partial loads in batches (one dependent HBM round trip per tile
// made it 125 us).  w is the conv's K-major packed weight ([K][C], ops.Conv / ConvW); x the 16 kHz signal [B][N]
// (batch stride xbs).
// Round 6: tiles of 64 frames (not 256) and fe0_apply over channel groups of FE0_CG -- at 256 frames per tile one
// thread walked 256 frames serially and the launch had ~3 waves per SIMD; fe0_apply's threads each walked all C
// channels at ~1.5 waves per SIMD (stats + apply 0.18 + 0.21 ms per 30 s clip, r6f)
constexpr int FE0_TT = 64;    // frames per tile
constexpr int FE0_CG = 64;    // fe0_apply: channels per block
constexpr int FE0_KMAX = 16;  // taps (ContentVec: 10)
constexpr int FE0_CW = 20;    // fe0_apply's LDS record per channel: K_MAX taps, then mean, rstd, gamma, beta

__global__ __launch_bounds__(512) void fe0_stats_kernel(const float* x, int64_t xbs, int64_t T, const float* w, int C,
                                                        int K, int S, double* part) {
    __shared__ float xs[FE0_TT * 8 + FE0_KMAX];  // stride <= 8
    const int b = blockIdx.y, tile = blockIdx.x;
    const int64_t t0 = (int64_t)tile * FE0_TT;
    const int nt = (int)min((int64_t)FE0_TT, T - t0);
    const float* xb = x + b * xbs + t0 * S;
    const int nx = (nt - 1) * S + K;
    for (int i = threadIdx.x; i < nx; i += blockDim.x) xs[i] = xb[i];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float wr[FE0_KMAX];
#pragma unroll
        for (int k = 0; k < FE0_KMAX; ++k) wr[k] = k < K ? w[k * C + c] : 0.f;
        double s = 0.0, q = 0.0;
        for (int t = 0; t < nt; ++t) {
            float y = 0.f;
#pragma unroll
            for (int k = 0; k < FE0_KMAX; ++k)
                if (k < K) y = fmaf(wr[k], xs[t * S + k], y);
            s += y;
            q += (double)y * y;
        }
        double* pp = part + (((int64_t)b * gridDim.x + tile) * C + c) * 2;
        pp[0] = s;
        pp[1] = q;
    }
}

__global__ __launch_bounds__(256) void fe0_final_kernel(const double* part, int ntile, int C, int64_t T, float eps,
                                                        float* stat) {
    constexpr int U = 16;  // partial loads in flight per thread
    const int b = blockIdx.y;
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double2* pb = reinterpret_cast<const double2*>(part) + (int64_t)b * ntile * C + c;
    double s = 0.0, q = 0.0;
    for (int i0 = 0; i0 < ntile; i0 += U) {
        double2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = pb[(int64_t)min(i0 + u, ntile - 1) * C];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u < ntile) {  // tile order, as before
                s += v[u].x;
                q += v[u].y;
            }
    }
    const double mean = s / (double)T;
    const double var = fmax(q / (double)T - mean * mean, 0.0);
    stat[((int64_t)b * C + c) * 2] = (float)mean;
    stat[((int64_t)b * C + c) * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

__global__ __launch_bounds__(256) void fe0_apply_kernel(const float* x, int64_t xbs, int64_t T, const float* w, int C,
                                                        int K, int S, const float* stat, const float* gamma,
                                                        const float* beta, float* out, int gelu, unsigned* amax_out) {
    // per channel of the block's group [c0, c0 + nc): w[0..K_MAX), mean, rstd, gamma, beta
    __shared__ __attribute__((aligned(16))) float sm[FE0_CG * FE0_CW];
    const int b = blockIdx.z;
    const int c0 = blockIdx.y * FE0_CG, nc = min(FE0_CG, C - c0);
    for (int i = threadIdx.x; i < nc * FE0_KMAX; i += blockDim.x) {
        const int cl = i / FE0_KMAX, k = i - cl * FE0_KMAX;
        sm[cl * FE0_CW + k] = k < K ? w[k * C + c0 + cl] : 0.f;
    }
    for (int cl = threadIdx.x; cl < nc; cl += blockDim.x) {
        const int c = c0 + cl;
        sm[cl * FE0_CW + FE0_KMAX] = stat[((int64_t)b * C + c) * 2];
        sm[cl * FE0_CW + FE0_KMAX + 1] = stat[((int64_t)b * C + c) * 2 + 1];
        sm[cl * FE0_CW + FE0_KMAX + 2] = gamma[c];
        sm[cl * FE0_CW + FE0_KMAX + 3] = beta[c];
    }
    __syncthreads();
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool ok = t < T;
    const int64_t tc = ok ? t : T - 1;
    float xw[FE0_KMAX];
    const float* xb = x + b * xbs + tc * S;
#pragma unroll
    for (int k = 0; k < FE0_KMAX; ++k) xw[k] = k < K ? xb[k] : 0.f;
    float* ob = out + ((int64_t)b * C + c0) * T + tc;
    float amx = 0.f;
    for (int c = 0; c < nc; ++c) {
        const float4* rec = reinterpret_cast<const float4*>(sm + c * FE0_CW);  // same address in every lane: broadcast
        float wr[FE0_KMAX + 4];
#pragma unroll
        for (int i = 0; i < FE0_CW / 4; ++i) {
            const float4 v = rec[i];
            wr[4 * i] = v.x;
            wr[4 * i + 1] = v.y;
            wr[4 * i + 2] = v.z;
            wr[4 * i + 3] = v.w;
        }
        float y = 0.f;
#pragma unroll
        for (int k = 0; k < FE0_KMAX; ++k)
            if (k < K) y = fmaf(wr[k], xw[k], y);  // fe0_stats' chain
        const float v = (y - wr[FE0_KMAX]) * wr[FE0_KMAX + 1] * wr[FE0_KMAX + 2] + wr[FE0_KMAX + 3];
        const float o = gelu ? act_apply(v, RVC_ACT_GELU, 0.f) : v;
        if (ok) {
            ob[(int64_t)c * T] = o;
            amx = fmaxf(amx, fabsf(o));
        }
    }
    if (amax_out) amax_publish_block(amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);  // one atomic per block
}

extern "C" int64_t rvc_fe0_ws_bytes(int64_t B, int64_t C, int64_t T) {
    if (B <= 0 || C <= 0 || T <= 0) return -1;
    const int64_t ntile = (T + FE0_TT - 1) / FE0_TT;
    return B * ntile * C * 2 * 8 + B * C * 2 * 4 + 256;
}

extern "C" int rvc_fe0_gn_gelu_amax(const float* x, int64_t B, int64_t N, int64_t x_bstride, const float* w_km,
                                    int64_t C, int K, int stride, const float* gamma, const float* beta, float* out,
                                    float eps, int gelu, unsigned* amax_out, void* ws, int64_t ws_bytes,
                                    rvc_stream_t stream) {
    RVC_CHECK_ARG(x && w_km && gamma && beta && out && ws && B > 0 && C > 0 && K > 0 && K <= FE0_KMAX && stride > 0 &&
                      stride <= 8 && N >= K,
                  "fe0_gn_gelu: bad args");
    RVC_CHECK_ARG(C <= 65535 * FE0_CG, "fe0_gn_gelu: C=%lld too large", (long long)C);
    const int64_t T = (N - K) / stride + 1;
    RVC_CHECK_ARG(ws_bytes >= rvc_fe0_ws_bytes(B, C, T), "fe0_gn_gelu: workspace too small");
    RVC_CHECK_ARG(((uintptr_t)ws & 15) == 0, "fe0_gn_gelu: workspace must be 16-B aligned");
    const int64_t xbs = x_bstride ? x_bstride : N;
    const int ntile = (int)((T + FE0_TT - 1) / FE0_TT);
    double* part = (double*)ws;
    float* stat = (float*)((char*)ws + B * ntile * C * 2 * 8);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(fe0_stats_kernel, dim3(ntile, (unsigned)B), dim3(512), 0, s, x, xbs, T, w_km, (int)C, K, stride,
                       part);
    hipLaunchKernelGGL(fe0_final_kernel, dim3((unsigned)((C + 255) / 256), (unsigned)B), dim3(256), 0, s, part, ntile,
                       (int)C, T, eps, stat);
    hipLaunchKernelGGL(fe0_apply_kernel, dim3((unsigned)((T + 255) / 256), (unsigned)((C + FE0_CG - 1) / FE0_CG),
                                              (unsigned)B), dim3(256), 0, s, x, xbs, T, w_km, (int)C, K, stride, stat,
                       gamma, beta, out, gelu, amax_out);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_fe0_gn_gelu(const float* x, int64_t B, int64_t N, int64_t x_bstride, const float* w_km, int64_t C,
                               int K, int stride, const float* gamma, const float* beta, float* out, float eps,
                               int gelu, void* ws, int64_t ws_bytes, rvc_stream_t stream) {
    return rvc_fe0_gn_gelu_amax(x, B, N, x_bstride, w_km, C, K, stride, gamma, beta, out, eps, gelu, nullptr, ws,
                                ws_bytes, stream);
}
