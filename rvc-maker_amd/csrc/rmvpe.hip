// RMVPE f0 estimator kernels (main/library/predictors/RMVPE.py): STFT framing, magnitude,
// U-Net image staging / pooling / transposed-conv phase interleave, the bidirectional GRU
// recurrence, and the f64 salience decode + coarse pitch quantiser (convert.py:311-323).
// The 3x3 / 1x1 convolutions and the dense projections run on the implicit-GEMM MFMA
// engine (conv1d.hip) over zero-bordered images.
#include "rvc_common.h"
#include <stdlib.h>

// ---------------------------------------------------------------- STFT framing
// framesT[n][f] = xr[f*hop + n - nfft/2] * win[n], centred reflect padding (torch.stft center=True,
// pad_mode="reflect"; RMVPE.py:168).  Output is k-major for the DFT GEMM (K = 1 conv).
__global__ void stft_frames_kernel(const float* x, const float* win, float* out, int64_t N, int64_t F, int nfft,
                                   int hop) {
    int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int n = blockIdx.y;
    if (f >= F) return;
    int64_t j = f * hop + n - nfft / 2;
    if (j < 0) j = -j;
    if (j >= N) j = 2 * (N - 1) - j;
    out[(int64_t)n * F + f] = x[j] * win[n];
}

extern "C" int rvc_stft_frames(const float* x, const float* win, float* framesT, int64_t N, int64_t F, int nfft,
                               int hop, rvc_stream_t stream) {
    RVC_CHECK_ARG(x && win && framesT && N > nfft / 2 && F > 0 && nfft > 0 && hop > 0, "stft_frames: bad args");
    RVC_CHECK_ARG((F - 1) * hop <= N - 1 + nfft / 2 + (N - 1), "stft_frames: F too large");
    hipLaunchKernelGGL(stft_frames_kernel, dim3(cdiv(F, 256), (unsigned)nfft), dim3(256), 0, (hipStream_t)stream, x,
                       win, framesT, N, F, nfft, hop);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// mag[k][f] = sqrt(re^2 + im^2), spec = [re (K rows); im (K rows)]        (RMVPE.py:169)
__global__ void spec_mag_kernel(const float* spec, float* mag, int K, int64_t F) {
    int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int k = blockIdx.y;
    if (f >= F) return;
    float re = spec[(int64_t)k * F + f], im = spec[(int64_t)(k + K) * F + f];
    mag[(int64_t)k * F + f] = sqrtf(re * re + im * im);
}

extern "C" int rvc_spec_mag(const float* spec, float* mag, int64_t K, int64_t F, rvc_stream_t stream) {
    RVC_CHECK_ARG(spec && mag && K > 0 && F > 0, "spec_mag: bad args");
    hipLaunchKernelGGL(spec_mag_kernel, dim3(cdiv(F, 256), (unsigned)K), dim3(256), 0, (hipStream_t)stream, spec, mag,
                       (int)K, F);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- STFT magnitude in f64
// mag[b][k][f] = |sum_n xr[f*hop + n - nfft/2] win[n] e^{-2 pi i k n / nfft}| for k <= nfft/2, with centred
// reflect padding (torch.stft center=True, RMVPE.py:168-169), computed as an f64 radix-2 FFT in LDS and
// rounded to f32 once.  The reference evaluates this in f32 (torch.stft + sqrt(re^2 + im^2)); a bin far
// below the frame's energy then carries a relative error that log(clamp(mel, 1e-5)) turns into an absolute
// one (1e-3 on the synthetic weights with the f32 DFT GEMM this replaced, 2e-4 for torch's f32 FFT, ~1e-7
// here: scripts/rmvpe_prec.py).  STFT_FPB frames per block share the twiddle table; the bins of a block are
// stored STFT_FPB consecutive frames at a time.
constexpr int STFT_NMAX = 1024, STFT_FPB = 8;

template <typename TO>
__global__ __launch_bounds__(256) void stft_mag_kernel(const float* x, const float* win, TO* mag, int64_t N,
                                                       int64_t F, int nfft, int logn, int hop, int64_t x_bs,
                                                       int64_t m_bs) {
    __shared__ double2 a[STFT_FPB][STFT_NMAX];
    __shared__ double2 tw[STFT_NMAX / 2];
    const int b = blockIdx.y;
    const int64_t f0 = (int64_t)blockIdx.x * STFT_FPB;
    const float* xb = x + b * x_bs;
    for (int j = threadIdx.x; j < nfft / 2; j += blockDim.x) {
        double s, c;
        sincospi(-2.0 * (double)j / (double)nfft, &s, &c);
        tw[j] = make_double2(c, s);
    }
    for (int i = threadIdx.x; i < STFT_FPB * nfft; i += blockDim.x) {
        const int q = i / nfft, n = i - q * nfft;
        const int64_t f = f0 + q;
        double v = 0.0;
        if (f < F) {
            int64_t j = f * hop + n - nfft / 2;
            if (j < 0) j = -j;
            if (j >= N) j = 2 * (N - 1) - j;
            v = (double)xb[j] * (double)win[n];
        }
        a[q][__brev((unsigned)n) >> (32 - logn)] = make_double2(v, 0.0);
    }
    __syncthreads();
    for (int s = 1; s <= logn; ++s) {
        const int half = 1 << (s - 1);
        for (int j = threadIdx.x; j < nfft / 2; j += blockDim.x) {
            const int pos = j & (half - 1);
            const int i0 = ((j >> (s - 1)) << s) + pos, i1 = i0 + half;
            const double2 w = tw[pos << (logn - s)];
#pragma unroll
            for (int q = 0; q < STFT_FPB; ++q) {
                const double2 u = a[q][i0], v = a[q][i1];
                const double2 t = make_double2(w.x * v.x - w.y * v.y, w.x * v.y + w.y * v.x);
                a[q][i0] = make_double2(u.x + t.x, u.y + t.y);
                a[q][i1] = make_double2(u.x - t.x, u.y - t.y);
            }
        }
        __syncthreads();
    }
    const int K = nfft / 2 + 1;
    TO* mb = mag + b * m_bs;
    for (int i = threadIdx.x; i < K * STFT_FPB; i += blockDim.x) {
        const int k = i / STFT_FPB, q = i - k * STFT_FPB;
        const int64_t f = f0 + q;
        if (f < F) {
            const double2 v = a[q][k];
            mb[(int64_t)k * F + f] = (TO)sqrt(v.x * v.x + v.y * v.y);
        }
    }
}

template <typename TO>
static int stft_mag_launch(const float* x, const float* win, TO* mag, int64_t B, int64_t N, int64_t F, int nfft, int hop,
                           int64_t x_bstride, int64_t mag_bstride, rvc_stream_t stream) {
    int logn = 0;
    while ((1 << logn) < nfft) ++logn;
    RVC_CHECK_ARG(x && win && mag && B > 0 && N > nfft / 2 && F > 0 && hop > 0, "stft_mag: bad args");
    RVC_CHECK_ARG((1 << logn) == nfft && nfft >= 2 && nfft <= STFT_NMAX, "stft_mag: nfft must be a power of 2 <= 1024");
    RVC_CHECK_ARG((F - 1) * hop <= 2 * (N - 1), "stft_mag: F too large for reflect padding");
    RVC_CHECK_ARG(B == 1 || (x_bstride >= N && mag_bstride >= (int64_t)(nfft / 2 + 1) * F), "stft_mag: bad batch strides");
    hipLaunchKernelGGL(stft_mag_kernel<TO>, dim3(cdiv(F, STFT_FPB), (unsigned)B), dim3(256), 0, (hipStream_t)stream, x,
                       win, mag, N, F, nfft, logn, hop, x_bstride, mag_bstride);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_stft_mag(const float* x, const float* win, float* mag, int64_t B, int64_t N, int64_t F,
                            int nfft, int hop, int64_t x_bstride, int64_t mag_bstride, rvc_stream_t stream) {
    return stft_mag_launch<float>(x, win, mag, B, N, F, nfft, hop, x_bstride, mag_bstride, stream);
}

// the same magnitudes unrounded (the f64 RMVPE, rmvpe64.hip)
extern "C" int rvc_stft_mag64(const float* x, const float* win, double* mag, int64_t B, int64_t N, int64_t F,
                              int nfft, int hop, int64_t x_bstride, int64_t mag_bstride, rvc_stream_t stream) {
    return stft_mag_launch<double>(x, win, mag, B, N, F, nfft, hop, x_bstride, mag_bstride, stream);
}

// ---------------------------------------------------------------- U-Net input image
// img[(t+1)*(W+2) + m+1] = mel[m][src(t)] * scale + shift for t < Tp (reflect-padded frames,
// RMVPE.py:213) with the encoder's input BatchNorm2d(1) folded to (scale, shift) (RMVPE.py:64).
// The image border cells are left untouched (caller keeps them zero).
__global__ void mel_image_kernel(const float* mel, float* img, int M, int64_t F, int64_t Tp, float scale,
                                 float shift) {
    int64_t t = (int64_t)blockIdx.x;
    int m = threadIdx.x;
    if (t >= Tp || m >= M) return;
    int64_t s = t < F ? t : 2 * (F - 1) - t;
    img[(t + 1) * (M + 2) + m + 1] = mel[(int64_t)m * F + s] * scale + shift;
}

extern "C" int rvc_mel_image(const float* mel, float* img, int64_t M, int64_t F, int64_t Tp, float scale, float shift,
                             rvc_stream_t stream) {
    RVC_CHECK_ARG(mel && img && M > 0 && M <= 1024 && F > 1 && Tp >= F && Tp - F < F, "mel_image: bad args");
    hipLaunchKernelGGL(mel_image_kernel, dim3((unsigned)Tp), dim3((unsigned)((M + 63) / 64 * 64)), 0,
                       (hipStream_t)stream, mel, img, (int)M, F, Tp, scale, shift);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- AvgPool2d(2) on bordered images
// in [C][H+2][W+2] -> out [C][H/2+2][W/2+2]; ((a + b) + c) + d then / 4 as torch's CPU kernel.
__global__ void avgpool2_kernel(const float* in, float* out, int C, int H, int W) {
    const int Ho = H / 2, Wo = W / 2;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t n = (int64_t)C * Ho * Wo;
    if (i >= n) return;
    int x = (int)(i % Wo);
    int64_t r = i / Wo;
    int y = (int)(r % Ho);
    int c = (int)(r / Ho);
    const float* ib = in + (int64_t)c * (H + 2) * (W + 2);
    const int64_t a0 = (int64_t)(2 * y + 1) * (W + 2) + 2 * x + 1;
    float s = ib[a0];
    s += ib[a0 + 1];
    s += ib[a0 + W + 2];
    s += ib[a0 + W + 3];
    out[(int64_t)c * (Ho + 2) * (Wo + 2) + (int64_t)(y + 1) * (Wo + 2) + x + 1] = s / 4.0f;
}

extern "C" int rvc_avgpool2(const float* in, float* out, int64_t C, int64_t H, int64_t W, rvc_stream_t stream) {
    RVC_CHECK_ARG(in && out && C > 0 && H >= 2 && W >= 2, "avgpool2: bad args");
    int64_t n = C * (H / 2) * (W / 2);
    hipLaunchKernelGGL(avgpool2_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, in, out, (int)C, (int)H,
                       (int)W);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- ConvTranspose2d(3, s2, p1, op1) phases
// phases[py*2+px] are [C][H+2][W+2] bordered (computed on the input grid by the conv engine);
// out (bordered, [*][2H+2][2W+2], first C channels) gets out[c][2y+py][2x+px] = phase[c][y][x].
__global__ void interleave4_kernel(const float* ph, float* out, int C, int H, int W) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int Ho = 2 * H, Wo = 2 * W;
    int64_t n = (int64_t)C * Ho * Wo;
    if (i >= n) return;
    int xo = (int)(i % Wo);
    int64_t r = i / Wo;
    int yo = (int)(r % Ho);
    int c = (int)(r / Ho);
    int py = yo & 1, px = xo & 1, y = yo >> 1, x = xo >> 1;
    const int64_t plane = (int64_t)(H + 2) * (W + 2);
    float v = ph[((int64_t)(py * 2 + px) * C + c) * plane + (int64_t)(y + 1) * (W + 2) + x + 1];
    out[(int64_t)c * (Ho + 2) * (Wo + 2) + (int64_t)(yo + 1) * (Wo + 2) + xo + 1] = v;
}

extern "C" int rvc_interleave4(const float* phases, float* out, int64_t C, int64_t H, int64_t W,
                               rvc_stream_t stream) {
    RVC_CHECK_ARG(phases && out && C > 0 && H > 0 && W > 0, "interleave4: bad args");
    int64_t n = C * 4 * H * W;
    hipLaunchKernelGGL(interleave4_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, phases, out, (int)C,
                       (int)H, (int)W);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- cnn output -> GRU input
// x[c*W + f][t] = img[c][t+1][f+1]   (E2E.forward: .transpose(1, 2).flatten(-2), RMVPE.py:144)
__global__ void img_to_seq_kernel(const float* img, float* x, int C, int64_t H, int W) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int cf = blockIdx.y;
    if (t >= H) return;
    int c = cf / W, f = cf - c * W;
    x[(int64_t)cf * H + t] = img[(int64_t)c * (H + 2) * (W + 2) + (t + 1) * (W + 2) + f + 1];
}

extern "C" int rvc_img_to_seq(const float* img, float* x, int64_t C, int64_t H, int64_t W, rvc_stream_t stream) {
    RVC_CHECK_ARG(img && x && C > 0 && H > 0 && W > 0, "img_to_seq: bad args");
    hipLaunchKernelGGL(img_to_seq_kernel, dim3(cdiv(H, 256), (unsigned)(C * W)), dim3(256), 0, (hipStream_t)stream,
                       img, x, (int)C, H, (int)W);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

// ---------------------------------------------------------------- bidirectional GRU recurrence
// nn.GRU(384, 256, bidirectional) (RMVPE.py:254-260).  gi = W_ih x + b_ih is precomputed for
// all t by the MFMA engine ([2][3][256][T] channels-first); this kernel runs the sequential
// part: per step gh = W_hh h + b_hh, r/z/n gates, h' = (h - n) z + n (torch's GRU cell).
// 16 workgroups per direction, each owning 16 hidden units with its 48 rows of W_hh held in
// registers; hidden states are exchanged every step through 8-byte {tag, value} granules
// (agent-scope relaxed atomics; MI355X_MICROARCH "R2" granule hand-off), double-buffered by
// step parity.  Every spin is bounded; a timeout sets *err and the kernel drains.
constexpr int GRU_H = 256;
constexpr int GRU_WG_PER_DIR = 16;

// Batched form: blockIdx.y = sequence b (gi + b gi_bs, y + b y_bs, its own granule pair): B sequences
// advance in lockstep-free parallel at the latency of one (VC.pipeline_device_batch's equal-length chunks).
__global__ __launch_bounds__(256) void bigru_kernel(const float* gi, const float* whh, const float* bhh, float* y,
                                                    unsigned long long* gran, int* err, int64_t T,
                                                    unsigned spin_limit, int64_t gi_bs, int64_t y_bs) {
    gi += (int64_t)blockIdx.y * gi_bs;
    y += (int64_t)blockIdx.y * y_bs;
    gran += (int64_t)blockIdx.y * 2 * 2 * GRU_H;
    const int d = blockIdx.x / GRU_WG_PER_DIR;
    const int j = blockIdx.x % GRU_WG_PER_DIR;
    const int tid = threadIdx.x;
    const int ul = tid >> 4, s = tid & 15;
    const int u = j * 16 + ul;
    // h of the previous step, double-buffered by step parity: step t reads hs[t & 1] and the next step
    // writes hs[(t + 1) & 1], so one barrier per step orders both
    __shared__ float hs[2][GRU_H];
    __shared__ int abort_flag;
    if (tid == 0) abort_flag = 0;
    const float* W = whh + (int64_t)d * 3 * GRU_H * GRU_H;
    float wr[16], wz[16], wn[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        wr[i] = W[(int64_t)(u)*GRU_H + 16 * s + i];
        wz[i] = W[(int64_t)(GRU_H + u) * GRU_H + 16 * s + i];
        wn[i] = W[(int64_t)(2 * GRU_H + u) * GRU_H + 16 * s + i];
    }
    const float bhr = bhh[d * 3 * GRU_H + u], bhz = bhh[d * 3 * GRU_H + GRU_H + u],
                bhn = bhh[d * 3 * GRU_H + 2 * GRU_H + u];
    const float* G = gi + (int64_t)d * 3 * GRU_H * T;
    unsigned long long* GR = gran + (int64_t)d * 2 * GRU_H;
    float hprev = 0.f;
    // input projections of the current step, loaded one step ahead (after the poll, so that the poll's
    // wait does not queue behind them in vmcnt order)
    float gxr = 0.f, gxz = 0.f, gxn = 0.f;
    if (s == 0) {
        const int64_t tau0 = d ? T - 1 : 0;
        gxr = G[(int64_t)u * T + tau0];
        gxz = G[(int64_t)(GRU_H + u) * T + tau0];
        gxn = G[(int64_t)(2 * GRU_H + u) * T + tau0];
    }
    hs[0][tid] = 0.f;
    __syncthreads();
    for (int64_t t = 0; t < T; ++t) {
        const int64_t tau = d ? T - 1 - t : t;
        const int cur = (int)(t & 1);
        if (t > 0) {
            unsigned long long* g = GR + ((t - 1) & 1) * GRU_H + tid;
            unsigned long long v;
            unsigned spins = 0;
            for (;;) {
                v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(v >> 32) == (uint32_t)t) break;
                if (++spins > spin_limit) {
                    atomicExch(err, 1);
                    abort_flag = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            hs[cur][tid] = __uint_as_float((uint32_t)v);
            __syncthreads();
            if (abort_flag) break;
        }
        float nxr = 0.f, nxz = 0.f, nxn = 0.f;
        if (s == 0 && t + 1 < T) {
            const int64_t tn = d ? T - 2 - t : t + 1;
            nxr = G[(int64_t)u * T + tn];
            nxz = G[(int64_t)(GRU_H + u) * T + tn];
            nxn = G[(int64_t)(2 * GRU_H + u) * T + tn];
        }
        float pr = 0.f, pz = 0.f, pn = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float h = hs[cur][16 * s + i];
            pr += wr[i] * h;
            pz += wz[i] * h;
            pn += wn[i] * h;
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
            pr += __shfl_xor(pr, o, 64);
            pz += __shfl_xor(pz, o, 64);
            pn += __shfl_xor(pn, o, 64);
        }
        if (s == 0) {
            const float r = 1.f / (1.f + expf(-(gxr + (pr + bhr))));
            const float z = 1.f / (1.f + expf(-(gxz + (pz + bhz))));
            const float n = tanhf(gxn + r * (pn + bhn));
            const float h = (hprev - n) * z + n;
            hprev = h;
            const unsigned long long gv = ((unsigned long long)(uint32_t)(t + 1) << 32) | __float_as_uint(h);
            __hip_atomic_store(GR + (t & 1) * GRU_H + u, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            y[(int64_t)(d * GRU_H + u) * T + tau] = h;
        }
        gxr = nxr;
        gxz = nxz;
        gxn = nxn;
    }
}

static unsigned g_bigru_spin_limit = 1u << 22;

extern "C" unsigned rvc_bigru_set_spin_limit(unsigned limit) {
    const unsigned prev = g_bigru_spin_limit;
    if (limit) g_bigru_spin_limit = limit;
    return prev;
}

extern "C" int rvc_bigru(const float* gi, const float* whh, const float* bhh, float* y, void* gran_ws, int* err,
                         int64_t T, rvc_stream_t stream) {
    return rvc_bigru_batched(gi, 0, whh, bhh, y, 0, gran_ws, err, 1, T, stream);
}

// Sequences per launch: 32 workgroups each, all of which must be co-resident for the granule hand-off
// (2 per CU at 16 sequences); larger batches run as consecutive launches.
constexpr int GRU_B_MAX = 16;

extern "C" int rvc_bigru_batched(const float* gi, int64_t gi_bs, const float* whh, const float* bhh, float* y,
                                 int64_t y_bs, void* gran_ws, int* err, int64_t B, int64_t T, rvc_stream_t stream) {
    RVC_CHECK_ARG(gi && whh && bhh && y && gran_ws && err && T > 0 && T < (1ll << 31) && B > 0, "bigru: bad args");
    RVC_CHECK_ARG(B == 1 || (gi_bs >= 2 * 3 * GRU_H * T && y_bs >= 2 * GRU_H * T), "bigru: batch strides too small");
    hipStream_t s = (hipStream_t)stream;
    for (int64_t b0 = 0; b0 < B; b0 += GRU_B_MAX) {
        const int64_t nb = B - b0 < GRU_B_MAX ? B - b0 : GRU_B_MAX;
        RVC_HIP(hipMemsetAsync(gran_ws, 0, (size_t)nb * 2 * 2 * GRU_H * sizeof(unsigned long long), s));
        hipLaunchKernelGGL(bigru_kernel, dim3(2 * GRU_WG_PER_DIR, (unsigned)nb), dim3(256), 0, s, gi + b0 * gi_bs, whh,
                           bhh, y + b0 * y_bs, (unsigned long long*)gran_ws, err, T, g_bigru_spin_limit, gi_bs, y_bs);
        RVC_HIP(hipGetLastError());
    }
    return RVC_OK;
}

// ---------------------------------------------------------------- salience decode + coarse pitch
// RMVPE.decode / to_local_average_cents (RMVPE.py:217-252) in f64 with numpy's reduction
// order, then VC.get_f0's shift and mel quantiser (convert.py:311-323).  sal is [360][ld].
__device__ double np_pairwise9_d(const double* a) {
    return (((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]))) + a[8];
}
__device__ float np_pairwise9_f(const float* a) {
    return (((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]))) + a[8];
}

__global__ void rmvpe_decode_kernel(const float* sal, int64_t ld, int64_t F, double thred, double shift,
                                    double mel_min, double mel_max, rvc_f0_post post, double* f0_out, int64_t* coarse,
                                    float* pitchf) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= F) return;
    int am = 0;
    float mx = sal[t];
    for (int i = 1; i < 360; ++i) {
        float v = sal[(int64_t)i * ld + t];
        if (v > mx) {
            mx = v;
            am = i;
        }
    }
    double prod[9];
    float sv[9];
    for (int k = 0; k < 9; ++k) {
        int i = am - 4 + k;
        float v = (i >= 0 && i < 360) ? sal[(int64_t)i * ld + t] : 0.f;
        double cents = (i >= 0 && i < 360) ? 20.0 * i + 1997.3794084376191 : 0.0;
        sv[k] = v;
        prod[k] = (double)v * cents;
    }
    double dev = np_pairwise9_d(prod) / (double)np_pairwise9_f(sv);
    if ((double)fmaxf(mx, 0.f) <= thred) dev = 0.0;
    double f0 = 10.0 * pow(2.0, dev / 1200.0);
    if (f0 == 10.0) f0 = 0.0;
    f0 = f0_post_apply<double>(f0, t, shift, post);
    if (f0_out) f0_out[t] = f0;
    double fm = 1127.0 * log(1.0 + f0 / 700.0);
    if (fm > 0) fm = (fm - mel_min) * 254.0 / (mel_max - mel_min) + 1.0;
    if (fm <= 1) fm = 1;
    if (fm > 255) fm = 255;
    coarse[t] = (int64_t)rint(fm);
    pitchf[t] = (float)f0;
}

extern "C" int rvc_rmvpe_decode(const float* sal, int64_t ld, int64_t F, double thred, double shift,
                                const rvc_f0_post* post, double* f0, int64_t* coarse, float* pitchf,
                                rvc_stream_t stream) {
    RVC_CHECK_ARG(sal && coarse && pitchf && F > 0 && ld >= F, "rmvpe_decode: bad args");
    RVC_CHECK_ARG(!post || !post->rep || (post->rep_off >= 0 && post->rep_len >= 0), "rmvpe_decode: bad f0 post");
    const rvc_f0_post pp = f0_post_or_none(post);
    const double mel_min = 1127.0 * log(1.0 + 50.0 / 700.0), mel_max = 1127.0 * log(1.0 + 1100.0 / 700.0);
    hipLaunchKernelGGL(rmvpe_decode_kernel, dim3(cdiv(F, 128)), dim3(128), 0, (hipStream_t)stream, sal, ld, F, thred,
                       shift, mel_min, mel_max, pp, f0, coarse, pitchf);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
