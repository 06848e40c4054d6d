// Implicit-GEMM conv1d on f32 MFMA for gfx950.
//
// GEMM view per (batch, phase, group):  Y[m][n] = sum_k A[k][m] * B[k][n]
//   m = output channel, n = output column, k = (input channel c, tap t) -> c*K + t
//   A = packed weights (KM layout, k-major, m contiguous), B = im2col of x (never
//   materialised: x rows are staged once per channel chunk into LDS with their halo,
//   and B[k][n] is read at koff[k] + n*stride).
// Block = 256 threads = 4 wave64s arranged WAVES_M x WAVES_N; each wave owns a
// (16*FM) x (16*FN) output tile held in FM*FN MFMA accumulators (4 VGPRs each).
// The input transform (scale + leaky-relu, i.e. the reference's F.leaky_relu in
// front of every HiFiGAN conv) is applied once when the tile is staged, and the
// epilogue fuses bias, activation, residual add and accumulate.
#include "rvc_common.h"

namespace {

struct ConvParams {
    const float* x;
    const float* w;
    const float* bias;
    const float* bias2;
    const float* res;
    float* y;
    int64_t Ci, Co, Lin, Lout, ncols;
    int64_t x_bstride, y_bstride, res_bstride, w_bstride;
    int K, stride, dil, pad, groups;
    int nphase, ostride, ooffset;
    int in_act, out_act, accumulate;
    float in_scale, in_slope, out_slope, out_scale;
    int CK, KC, span, span_s;  // channels per chunk, padded k per chunk, staged row length / stride
    int mtiles_per_group;
    int ntoff, wrap;
    int toff[16];
};

template <int FM, int FN, int WM, int WN>
__global__ __launch_bounds__(256) void conv1d_mfma_kernel(ConvParams p) {
    constexpr int BM = 16 * FM * WM;
    constexpr int BN = 16 * FN * WN;
    constexpr int WS = BM + 16;  // A row stride (== 16 mod 32 -> conflict-free 2-row reads)
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Ws = smem;                          // [KC][WS]
    float* Xs = smem + p.KC * WS;              // [CK][span_s]
    int* koff = (int*)(Xs + p.CK * p.span_s);  // [KC]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;

    const int zb = blockIdx.z;
    const int b = zb / p.nphase;
    const int phase = zb % p.nphase;
    const int g = blockIdx.y / p.mtiles_per_group;
    const int Cog = (int)(p.Co / p.groups);
    const int Cig = (int)(p.Ci / p.groups);
    const int m0g = (blockIdx.y % p.mtiles_per_group) * BM;  // within group
    const int64_t n0 = (int64_t)blockIdx.x * BN;

    const float* xb = p.x + b * p.x_bstride + (int64_t)g * Cig * p.Lin;
    const float* wg = p.w + b * p.w_bstride + ((int64_t)phase * p.groups + g) * (int64_t)Cig * p.K * Cog;
    const int64_t base = n0 * p.stride - p.pad;
    const int kreal = p.CK * p.K;

    for (int i = tid; i < p.KC; i += 256) {
        int c = i / p.K, t = i - c * p.K;
        koff[i] = (i < kreal) ? c * p.span_s + (p.ntoff ? p.toff[t] : t * p.dil) : 0;
    }

    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int nchunks = (Cig + p.CK - 1) / p.CK;
    for (int ch = 0; ch < nchunks; ++ch) {
        const int c0 = ch * p.CK;
        __syncthreads();
        // stage A: Ws[kk][m] = Wt[(c0*K + kk)][m0g + m]
        {
            const int64_t krow0 = (int64_t)c0 * p.K;
            const int64_t kmax = (int64_t)Cig * p.K;
            for (int i = tid; i < p.KC * BM; i += 256) {
                int kk = i / BM, m = i - kk * BM;
                int64_t kr = krow0 + kk;
                float v = 0.f;
                if (kk < kreal && kr < kmax && m0g + m < Cog) v = wg[kr * Cog + m0g + m];
                Ws[kk * WS + m] = v;
            }
        }
        // stage B source rows: Xs[c][j] = pre(x[c0+c][base + j])
        {
            const int rows = p.CK;
            for (int i = tid; i < rows * p.span; i += 256) {
                int c = i / p.span, j = i - c * p.span;
                int64_t pos = base + j;
                float v = 0.f;
                if (c0 + c < Cig && pos >= 0 && pos < p.Lin) {
                    v = xb[(int64_t)(c0 + c) * p.Lin + pos] * p.in_scale;
                    if (p.in_act == RVC_ACT_LRELU) v = v >= 0.f ? v : v * p.in_slope;
                }
                Xs[c * p.span_s + j] = v;
            }
        }
        __syncthreads();
        const int lk = lane >> 4;
        const int ln = lane & 15;
        const float* wa = Ws + wm * (16 * FM) + ln;
        const int nb = (wn * 16 * FN + ln) * p.stride;
        for (int k0 = 0; k0 < p.KC; k0 += 4) {
            const int kk = k0 + lk;
            float a[FM], bv[FN];
#pragma unroll
            for (int i = 0; i < FM; ++i) a[i] = wa[kk * WS + i * 16];
            const float* xr = Xs + koff[kk] + nb;
#pragma unroll
            for (int j = 0; j < FN; ++j) bv[j] = xr[j * 16 * p.stride];
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(a[i], bv[j], acc[i][j]);
        }
    }

    // epilogue
    const int ln = lane & 15;
    const int lr = (lane >> 4) * 4;
    float* yb = p.y + b * p.y_bstride;
    const float* rb = p.res ? p.res + b * p.res_bstride : nullptr;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int mg = m0g + wm * 16 * FM + i * 16 + lr + r;
            if (mg >= Cog) continue;
            const int64_t m = (int64_t)g * Cog + mg;
            const float bs = p.bias ? p.bias[m] : 0.f;
            const float bs2 = p.bias2 ? p.bias2[m] : 0.f;
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int64_t n = n0 + wn * 16 * FN + j * 16 + ln;
                if (n >= p.ncols) continue;
                const int64_t t = n * p.ostride + p.ooffset + phase;
                if (t < 0 || t >= p.Lout) continue;
                if (p.wrap) {
                    const int64_t row = t / p.wrap, col = t - row * p.wrap;
                    if (col == 0 || col == p.wrap - 1 || row == 0 || row == p.Lout / p.wrap - 1) continue;
                }
                float v = acc[i][j][r] + bs;
                if (p.bias2) v += bs2;
                v = act_apply(v, p.out_act, p.out_slope) * p.out_scale;
                const int64_t o = m * p.Lout + t;
                if (rb) v += rb[o];
                if (p.accumulate) yb[o] += v;
                else yb[o] = v;
            }
        }
    }
}

struct Cfg {
    int FM, FN, WM, WN;
};

template <int FM, int FN, int WM, int WN>
hipError_t launch(const ConvParams& p, dim3 grid, size_t lds, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)conv1d_mfma_kernel<FM, FN, WM, WN>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL((conv1d_mfma_kernel<FM, FN, WM, WN>), grid, dim3(256), lds, s, p);
    return hipGetLastError();
}

}  // namespace

extern "C" int rvc_conv1d(const rvc_conv1d_args* a, rvc_stream_t stream) {
    RVC_CHECK_ARG(a && a->x && a->w && a->y, "conv1d: null pointer");
    RVC_CHECK_ARG(a->B > 0 && a->Ci > 0 && a->Co > 0 && a->K > 0 && a->Lin > 0 && a->Lout > 0,
                  "conv1d: bad sizes B=%lld Ci=%lld Co=%lld K=%d Lin=%lld Lout=%lld", (long long)a->B,
                  (long long)a->Ci, (long long)a->Co, a->K, (long long)a->Lin, (long long)a->Lout);
    RVC_CHECK_ARG(a->groups >= 1 && a->Ci % a->groups == 0 && a->Co % a->groups == 0, "conv1d: bad groups");
    RVC_CHECK_ARG(a->stride >= 1 && a->dil >= 1 && a->nphase >= 1 && a->ostride >= 1, "conv1d: bad stride/dil");
    const int64_t Cog = a->Co / a->groups;
    const int64_t ncols = a->ncols > 0 ? a->ncols : a->Lout;

    // tile config by output-channel count and column count
    Cfg cfg;
    if (Cog % 48 == 0 && Cog % 64 != 0) cfg = {3, 1, 1, 4};        // 48 x 64 (ContentVec pos_conv)
    else if (Cog <= 16) cfg = {1, 4, 1, 4};                         // 16 x 256
    else if (Cog <= 32) cfg = {2, 4, 1, 4};                         // 32 x 256
    else if (Cog <= 64) cfg = {2, 4, 2, 2};                         // 64 x 128
    else {
        int64_t tiles128 = ((Cog + 127) / 128) * a->groups * ((ncols + 127) / 128) * a->B * a->nphase;
        cfg = tiles128 >= 480 ? Cfg{4, 4, 2, 2} : Cfg{2, 2, 2, 2};  // 128x128 or 64x64
    }
    const int BM = 16 * cfg.FM * cfg.WM, BN = 16 * cfg.FN * cfg.WN;
    const int WS = BM + 16;

    ConvParams p;
    p.x = a->x; p.w = a->w; p.bias = a->bias; p.bias2 = a->bias2; p.res = a->res; p.y = a->y;
    p.w_bstride = a->w_bstride;
    p.Ci = a->Ci; p.Co = a->Co; p.Lin = a->Lin; p.Lout = a->Lout; p.ncols = ncols;
    p.x_bstride = a->x_bstride ? a->x_bstride : a->Ci * a->Lin;
    p.y_bstride = a->y_bstride ? a->y_bstride : a->Co * a->Lout;
    p.res_bstride = a->res_bstride ? a->res_bstride : a->Co * a->Lout;
    p.K = a->K; p.stride = a->stride; p.dil = a->dil; p.pad = a->pad; p.groups = a->groups;
    p.nphase = a->nphase; p.ostride = a->ostride; p.ooffset = a->ooffset;
    p.in_act = a->in_act; p.out_act = a->out_act; p.accumulate = a->accumulate;
    p.in_scale = a->in_scale; p.in_slope = a->in_slope; p.out_slope = a->out_slope; p.out_scale = a->out_scale;
    int maxoff = (a->K - 1) * a->dil;
    p.ntoff = a->ntoff;
    p.wrap = a->wrap;
    if (a->ntoff) {
        RVC_CHECK_ARG(a->ntoff == a->K && a->K <= 16, "conv1d: toff needs ntoff == K <= 16");
        maxoff = 0;
        for (int i = 0; i < a->K; ++i) {
            RVC_CHECK_ARG(a->toff[i] >= 0, "conv1d: negative tap offset");
            p.toff[i] = a->toff[i];
            if (a->toff[i] > maxoff) maxoff = a->toff[i];
        }
    }
    p.span = (BN - 1) * a->stride + maxoff + 1;
    p.span_s = p.span + 1;
    const int Cig = (int)(a->Ci / a->groups);
    // channels per chunk: aim for KC <= 128 and <= 56 KiB of LDS
    int ck = 128 / a->K;
    if (ck < 1) ck = 1;
    if (ck > Cig) ck = Cig;
    for (;;) {
        int kc = ((ck * a->K + 3) / 4) * 4;
        size_t lds = (size_t)kc * WS * 4 + (size_t)ck * p.span_s * 4 + (size_t)kc * 4;
        if (lds <= 56 * 1024 || ck == 1) break;
        --ck;
    }
    p.CK = ck;
    p.KC = ((ck * a->K + 3) / 4) * 4;
    size_t lds = (size_t)p.KC * WS * 4 + (size_t)p.CK * p.span_s * 4 + (size_t)p.KC * 4;
    RVC_CHECK_ARG(lds <= 160 * 1024, "conv1d: LDS %zu too large (K=%d dil=%d stride=%d)", lds, a->K, a->dil,
                  a->stride);
    p.mtiles_per_group = (int)((Cog + BM - 1) / BM);
    dim3 grid(cdiv(ncols, BN), (unsigned)(p.mtiles_per_group * a->groups), (unsigned)(a->B * a->nphase));
    RVC_CHECK_ARG(grid.y < 65536 && grid.z < 65536, "conv1d: grid too large");

    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (cfg.FM == 3) e = launch<3, 1, 1, 4>(p, grid, lds, s);
    else if (cfg.FM == 1) e = launch<1, 4, 1, 4>(p, grid, lds, s);
    else if (cfg.WM == 1) e = launch<2, 4, 1, 4>(p, grid, lds, s);
    else if (cfg.FM == 4) e = launch<4, 4, 2, 2>(p, grid, lds, s);
    else if (cfg.FN == 4) e = launch<2, 4, 2, 2>(p, grid, lds, s);
    else e = launch<2, 2, 2, 2>(p, grid, lds, s);
    RVC_HIP(e);
    return RVC_OK;
}
