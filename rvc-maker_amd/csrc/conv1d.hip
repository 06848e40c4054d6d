// Implicit-GEMM convolution engine on f32 MFMA for gfx950 (v_mfma_f32_16x16x4_f32).
//
// GEMM view per (batch, phase, group):  Y[m][n] = sum_k A[k][m] * B[k][n]
//   m = output channel, n = output column, k = c*K + tap (flattened input channel x tap)
//   A = packed weights (KM layout: k-major, m contiguous),
//   B = im2col of x, never materialised: for each 32-deep k chunk the <= ceil(32/K)+1 input rows it
//       touches are staged into LDS once with their halo (pre-activation applied on staging),
//       and B[k][n] is read at koff[k] + n*stride.
// Block = 256 threads = 4 wave64s (WM x WN); a wave owns a (16*FM) x (16*FN) tile in FM*FN
// accumulators.  Chunks are software-pipelined through registers: chunk i+1's global loads are
// issued before chunk i's MFMAs and written to LDS after them (one LDS buffer, two barriers).
// Small grids split the k range over blockIdx.z (split-K); partial tiles go to a workspace and
// conv_splitk_reduce applies the epilogue.  The epilogue fuses bias, a second bias (speaker
// conditioning), activation, residual add, accumulate, polyphase/strided stores (ConvTranspose)
// and border masking (2-D mode).
#include "rvc_common.h"

namespace {

constexpr int KCH = 32;     // flattened k per chunk
constexpr int NB_MAX = 16;  // staged B elements per thread (rows * span <= 256 * NB_MAX)

struct ConvParams {
    const float* x;
    const float* w;
    const float* bias;
    const float* bias2;
    const float* res;
    float* y;
    float* ws;  // split-K partials [ksplit][B*nphase][Co][ncols]
    int64_t B, Ci, Co, Lin, Lout, ncols;
    int64_t x_bstride, y_bstride, res_bstride, w_bstride;
    int K, stride, dil, pad, groups;
    int nphase, ostride, ooffset;
    int in_act, out_act, accumulate;
    float in_scale, in_slope, out_slope, out_scale;
    int span, span_s, rows_max;
    float inv_span;
    int mtiles_per_group, ksplit, chunks_per_split, avec;
    int ntoff, wrap;
    int toff[16];
};

__device__ __forceinline__ int tap_off(const ConvParams& p, int t) { return p.ntoff ? p.toff[t] : t * p.dil; }

// Output column n -> store position t (or -1 when the column is not stored: beyond ncols / Lout,
// or a border cell in 2-D mode).  32-bit math: every per-batch extent here is < 2^31.
__device__ __forceinline__ int out_pos(const ConvParams& p, int64_t n, int phase) {
    if (n >= p.ncols) return -1;
    const int t = (int)n * p.ostride + p.ooffset + phase;
    if (t < 0 || t >= (int)p.Lout) return -1;
    if (p.wrap) {
        const int row = t / p.wrap, col = t - row * p.wrap;
        if (col == 0 || col == p.wrap - 1 || row == 0 || row == (int)p.Lout / p.wrap - 1) return -1;
    }
    return t;
}

// Branch-free epilogue for one element: every load is issued unconditionally from a clamped
// address (a per-element guarded load makes hipcc branch and wait vmcnt(0) per element).
__device__ __forceinline__ void epilogue_store(const ConvParams& p, float acc, int b, int64_t m, int t) {
    const bool ok = t >= 0;
    const int64_t o = m * p.Lout + (ok ? t : 0);
    float v = acc;
    if (p.bias) v += p.bias[m];
    if (p.bias2) v += p.bias2[m];
    v = act_apply(v, p.out_act, p.out_slope) * p.out_scale;
    if (p.res) v += p.res[b * p.res_bstride + o];
    float* yb = p.y + b * p.y_bstride;
    if (p.accumulate) v += yb[o];
    if (ok) yb[o] = v;
}

template <int ACT, int FM, int FN>
__device__ __forceinline__ void apply_act(floatx4 (&acc)[FM][FN], float slope, float scale) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = act_apply(acc[i][j][r], ACT, slope) * scale;
}

template <int FM, int FN, int WM, int WN>
__global__ __launch_bounds__(256) void conv1d_mfma_kernel(ConvParams p) {
    constexpr int BM = 16 * FM * WM;
    constexpr int BN = 16 * FN * WN;
    constexpr int WS = (BM / 32) * 32 + 16 + ((BM % 32) ? 32 : 0);  // == 16 mod 32, >= BM
    constexpr int NA = KCH * BM / 256;                                // A elements per thread
    constexpr bool AVEC_OK = (NA % 4) == 0 && (BM % 4) == 0;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Ws = smem;                     // [KCH][WS]
    int* koff = (int*)(smem + KCH * WS);  // [KCH]
    float* Xs = smem + KCH * WS + KCH;    // [rows_max][span_s]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    int zb = blockIdx.z;
    const int split = zb % p.ksplit;
    zb /= p.ksplit;
    const int phase = zb % p.nphase;
    const int b = zb / p.nphase;
    const int g = blockIdx.y / p.mtiles_per_group;
    const int Cog = (int)(p.Co / p.groups);
    const int Cig = (int)(p.Ci / p.groups);
    const int m0g = (blockIdx.y % p.mtiles_per_group) * BM;
    const int64_t n0 = (int64_t)blockIdx.x * BN;

    const float* xb = p.x + b * p.x_bstride + (int64_t)g * Cig * p.Lin;
    const float* wg = p.w + b * p.w_bstride + ((int64_t)phase * p.groups + g) * (int64_t)Cig * p.K * Cog;
    const int64_t base = n0 * p.stride - p.pad;
    const int kmax = Cig * p.K;
    const int nch = (kmax + KCH - 1) / KCH;
    const int ch_beg = split * p.chunks_per_split;
    const int ch_end = min(nch, ch_beg + p.chunks_per_split);

    float ra[NA];
    float rb[NB_MAX];
    // Per-thread B staging slots are the same for every chunk: slot i covers idx = tid + 256 i of the
    // rows x span tile, i.e. (row, col) = divmod(idx, span).  Precompute them once, packed as
    // row << 16 | col, plus a bitmask of slots whose input position base + col lies inside [0, Lin).
    int bslot[NB_MAX];
    unsigned bcolok = 0;
    {
        const int lin = (int)p.Lin;
#pragma unroll
        for (int i = 0; i < NB_MAX; ++i) {
            const int idx = tid + 256 * i;
            int r = (int)((float)idx * p.inv_span);
            r -= (r * p.span > idx);
            r += ((r + 1) * p.span <= idx);
            const int j = idx - r * p.span;
            bslot[i] = (r << 16) | j;
            const int pos = (int)base + j;
            bcolok |= (unsigned)(pos >= 0 && pos < lin) << i;
        }
    }

    // gload issues raw loads only (clamped addresses, no arithmetic on the results), so the loads of
    // chunk i+1 stay in flight across chunk i's MFMAs; sstore masks, pre-activates and writes LDS.
    // Any use of a loaded value inside gload would make hipcc wait for it right there.
    auto gload = [&](int ch) {
        const int k0 = ch * KCH;
        if (AVEC_OK && p.avec) {
#pragma unroll
            for (int i = 0; i < NA / 4; ++i) {
                const int idx = tid + 256 * i;
                const int kk = idx / (BM / 4);
                const int m = (idx % (BM / 4)) * 4;
                const int kr = k0 + kk;
                const bool ok = kr < kmax && m0g + m < Cog;
                const float4 v = *reinterpret_cast<const float4*>(wg + (ok ? kr * Cog + m0g + m : 0));
                ra[4 * i] = v.x; ra[4 * i + 1] = v.y; ra[4 * i + 2] = v.z; ra[4 * i + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int idx = tid + 256 * i;
                const int kk = idx / BM, m = idx % BM;
                const int kr = k0 + kk;
                const bool ok = kr < kmax && m0g + m < Cog;
                ra[i] = wg[ok ? kr * Cog + m0g + m : 0];
            }
        }
        const int c_lo = k0 / p.K;
        const int c_hi = min((k0 + KCH - 1) / p.K, Cig - 1);
        const int rows = c_hi - c_lo + 1;
        const int n = rows * p.span;
        const int lin = (int)p.Lin;
        const int rbase = c_lo * lin + (int)base;
        // groups of 4 loads behind a block-uniform bound check: only the groups the tile needs are issued
#pragma unroll
        for (int gi = 0; gi < NB_MAX; gi += 4) {
            if (gi * 256 < n) {
#pragma unroll
                for (int i = gi; i < gi + 4; ++i) {
                    const int r = bslot[i] >> 16, j = bslot[i] & 0xffff;
                    const bool ok = r < rows && ((bcolok >> i) & 1u);
                    rb[i] = xb[ok ? rbase + r * lin + j : 0];
                }
            }
        }
    };
    auto sstore = [&](int ch) {
        const int k0 = ch * KCH;
        if (AVEC_OK && p.avec) {
#pragma unroll
            for (int i = 0; i < NA / 4; ++i) {
                const int idx = tid + 256 * i;
                const int kk = idx / (BM / 4);
                const int m = (idx % (BM / 4)) * 4;
                const bool ok = k0 + kk < kmax && m0g + m < Cog;
                *reinterpret_cast<float4*>(Ws + kk * WS + m) =
                    ok ? make_float4(ra[4 * i], ra[4 * i + 1], ra[4 * i + 2], ra[4 * i + 3]) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int idx = tid + 256 * i;
                const int kk = idx / BM, m = idx % BM;
                const bool ok = k0 + kk < kmax && m0g + m < Cog;
                Ws[kk * WS + m] = ok ? ra[i] : 0.f;
            }
        }
        const int c_lo = k0 / p.K;
        const int c_hi = min((k0 + KCH - 1) / p.K, Cig - 1);
        const int rows = c_hi - c_lo + 1;
        const int n = rows * p.span;
        const int dump = p.rows_max * p.span_s;  // scratch slot after the tile for idx >= n
#pragma unroll
        for (int gi = 0; gi < NB_MAX; gi += 4) {
            if (gi * 256 < n) {
#pragma unroll
                for (int i = gi; i < gi + 4; ++i) {
                    const int r = bslot[i] >> 16, j = bslot[i] & 0xffff;
                    const bool ok = r < rows && ((bcolok >> i) & 1u);
                    float v = rb[i] * p.in_scale;
                    if (p.in_act == RVC_ACT_LRELU) v = v >= 0.f ? v : v * p.in_slope;
                    Xs[tid + 256 * i < n ? r * p.span_s + j : dump] = ok ? v : 0.f;
                }
            }
        }
        if (tid < KCH) {
            const int kk = k0 + tid;
            const int c = kk / p.K, t = kk - c * p.K;
            koff[tid] = (kk < kmax) ? (c - c_lo) * p.span_s + tap_off(p, t) : 0;
        }
    };

    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int lk = lane >> 4, ln = lane & 15;
    const float* wa = Ws + wm * (16 * FM) + ln;
    const int nb = (wn * 16 * FN + ln) * p.stride;
    const int jstep = 16 * p.stride;

    if (ch_beg < ch_end) {
        gload(ch_beg);
        sstore(ch_beg);
    }
    __syncthreads();
    for (int ch = ch_beg; ch < ch_end; ++ch) {
        const bool more = ch + 1 < ch_end;
        if (more) gload(ch + 1);
#pragma unroll
        for (int ks = 0; ks < KCH / 4; ++ks) {
            const int kk = ks * 4 + lk;
            float a[FM], bv[FN];
#pragma unroll
            for (int i = 0; i < FM; ++i) a[i] = wa[kk * WS + i * 16];
            const float* xr = Xs + koff[kk] + nb;
#pragma unroll
            for (int j = 0; j < FN; ++j) bv[j] = xr[j * jstep];
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(a[i], bv[j], acc[i][j]);
        }
        __syncthreads();
        if (more) sstore(ch + 1);
        __syncthreads();
    }

    const int lr = (lane >> 4) * 4;
    if (p.ksplit > 1) {
        float* wsb = p.ws + (((int64_t)split * p.B * p.nphase + (int64_t)b * p.nphase + phase) * p.Co) * p.ncols;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mg = m0g + wm * 16 * FM + i * 16 + lr + r;
                const int64_t m = (int64_t)g * Cog + mg;
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int64_t n = n0 + wn * 16 * FN + j * 16 + ln;
                    if (mg < Cog && n < p.ncols) wsb[m * p.ncols + n] = acc[i][j][r];
                }
            }
        return;
    }
    // Epilogue one row fragment (16 channels x BN/WN columns) at a time, in passes so that hipcc
    // issues each class of loads together: bias + activation + scale in registers (activation
    // dispatched once per kernel, not per element), residual loads, accumulate loads -- all from
    // clamped addresses -- then masked stores.  Per-fragment (not whole-tile) passes bound the
    // epilogue's live registers, which would otherwise set the whole kernel's occupancy.
    int tcol[FN];  // store position per column fragment (shared by all rows)
#pragma unroll
    for (int j = 0; j < FN; ++j) tcol[j] = out_pos(p, n0 + wn * 16 * FN + j * 16 + ln, phase);
    float* yb = p.y + b * p.y_bstride;
    const float* rb2 = p.res ? p.res + b * p.res_bstride : nullptr;
    const int Lo = (int)p.Lout;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        floatx4 (&av)[1][FN] = *reinterpret_cast<floatx4 (*)[1][FN]>(&acc[i][0]);
        int mrow[4];  // channel index (clamped); m * Lout < 2^31 is checked on the host
        bool mok[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int mg = m0g + wm * 16 * FM + i * 16 + lr + r;
            mok[r] = mg < Cog;
            mrow[r] = g * Cog + (mg < Cog ? mg : 0);
            float bs = 0.f;
            if (p.bias) bs = p.bias[mrow[r]];
            if (p.bias2) bs += p.bias2[mrow[r]];
#pragma unroll
            for (int j = 0; j < FN; ++j) av[0][j][r] += bs;
        }
        switch (p.out_act) {
            case RVC_ACT_LRELU: apply_act<RVC_ACT_LRELU, 1, FN>(av, p.out_slope, p.out_scale); break;
            case RVC_ACT_RELU: apply_act<RVC_ACT_RELU, 1, FN>(av, p.out_slope, p.out_scale); break;
            case RVC_ACT_TANH: apply_act<RVC_ACT_TANH, 1, FN>(av, p.out_slope, p.out_scale); break;
            case RVC_ACT_GELU: apply_act<RVC_ACT_GELU, 1, FN>(av, p.out_slope, p.out_scale); break;
            case RVC_ACT_SIGMOID: apply_act<RVC_ACT_SIGMOID, 1, FN>(av, p.out_slope, p.out_scale); break;
            case RVC_ACT_LOGCLAMP: apply_act<RVC_ACT_LOGCLAMP, 1, FN>(av, p.out_slope, p.out_scale); break;
            default: apply_act<RVC_ACT_NONE, 1, FN>(av, p.out_slope, p.out_scale); break;
        }
        if (rb2) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < FN; ++j) av[0][j][r] += rb2[mrow[r] * Lo + (tcol[j] >= 0 ? tcol[j] : 0)];
        }
        if (p.accumulate) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < FN; ++j) av[0][j][r] += yb[mrow[r] * Lo + (tcol[j] >= 0 ? tcol[j] : 0)];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < FN; ++j)
                if (mok[r] && tcol[j] >= 0) yb[mrow[r] * Lo + tcol[j]] = av[0][j][r];
    }
}

__global__ void conv_splitk_reduce(ConvParams p) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t m = blockIdx.y;
    const int bp = blockIdx.z;
    if (n >= p.ncols) return;
    const int64_t sstride = p.B * p.nphase * p.Co * p.ncols;
    const float* src = p.ws + ((int64_t)bp * p.Co + m) * p.ncols + n;
    float s = 0.f;
    for (int k = 0; k < p.ksplit; ++k) s += src[k * sstride];
    epilogue_store(p, s, bp / p.nphase, m, out_pos(p, n, bp % p.nphase));
}

struct Cfg {
    int FM, FN, WM, WN;
};

template <int FM, int FN, int WM, int WN>
hipError_t launch(const ConvParams& p, dim3 grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((conv1d_mfma_kernel<FM, FN, WM, WN>), grid, dim3(256), lds, s, p);
    return hipGetLastError();
}

int plan(const rvc_conv1d_args* a, ConvParams& p, Cfg& cfg, dim3& grid, size_t& lds) {
    RVC_CHECK_ARG(a && a->x && a->w && a->y, "conv1d: null pointer");
    RVC_CHECK_ARG(a->B > 0 && a->Ci > 0 && a->Co > 0 && a->K > 0 && a->Lin > 0 && a->Lout > 0,
                  "conv1d: bad sizes B=%lld Ci=%lld Co=%lld K=%d Lin=%lld Lout=%lld", (long long)a->B,
                  (long long)a->Ci, (long long)a->Co, a->K, (long long)a->Lin, (long long)a->Lout);
    RVC_CHECK_ARG(a->groups >= 1 && a->Ci % a->groups == 0 && a->Co % a->groups == 0, "conv1d: bad groups");
    RVC_CHECK_ARG(a->stride >= 1 && a->dil >= 1 && a->nphase >= 1 && a->ostride >= 1, "conv1d: bad stride/dil");
    RVC_CHECK_ARG(a->Co * a->Lout < (1ll << 31) && a->Ci * a->Lin < (1ll << 31) && a->Lin + a->pad < (1ll << 30),
                  "conv1d: per-batch tensor exceeds 2^31 elements (use the batch dimension)");
    const int64_t Cog = a->Co / a->groups;
    const int64_t Cig = a->Ci / a->groups;
    const int64_t ncols = a->ncols > 0 ? a->ncols : a->Lout;

    if (Cog % 48 == 0 && Cog % 64 != 0) cfg = {3, 1, 1, 4};  // 48 x 64 (ContentVec pos_conv groups)
    else if (Cog <= 16) cfg = {1, 4, 1, 4};                  // 16 x 256
    else if (Cog <= 32) cfg = {2, 4, 1, 4};                  // 32 x 256
    else if (Cog <= 64 || Cog % 128 != 0) cfg = {2, 4, 2, 2}; // 64 x 128 (also 192: no half-empty M tile)
    else cfg = {4, 4, 2, 2};                                 // 128 x 128
    int BM = 16 * cfg.FM * cfg.WM, BN = 16 * cfg.FN * cfg.WN;

    int maxoff = (a->K - 1) * a->dil;
    if (a->ntoff) {
        RVC_CHECK_ARG(a->ntoff == a->K && a->K <= 16, "conv1d: toff needs ntoff == K <= 16");
        maxoff = 0;
        for (int i = 0; i < a->K; ++i) {
            RVC_CHECK_ARG(a->toff[i] >= 0, "conv1d: negative tap offset");
            if (a->toff[i] > maxoff) maxoff = a->toff[i];
        }
    }
    // rows touched by a chunk of KCH consecutive k starting at a multiple of KCH
    int rows_max = (KCH % a->K == 0) ? KCH / a->K : (KCH - 1) / a->K + 2;
    if (rows_max > Cig) rows_max = (int)Cig;
    int span = (BN - 1) * a->stride + maxoff + 1;
    // keep the staged B tile within the per-thread register budget by narrowing the N tile
    while ((int64_t)rows_max * span > 256 * NB_MAX && cfg.FN > 2) {
        cfg.FN /= 2;
        BN = 16 * cfg.FN * cfg.WN;
        span = (BN - 1) * a->stride + maxoff + 1;
    }
    RVC_CHECK_ARG((int64_t)rows_max * span <= 256 * NB_MAX, "conv1d: staged tile too large (rows %d x span %d)",
                  rows_max, span);

    p.x = a->x; p.w = a->w; p.bias = a->bias; p.bias2 = a->bias2; p.res = a->res; p.y = a->y; p.ws = nullptr;
    p.B = a->B; p.Ci = a->Ci; p.Co = a->Co; p.Lin = a->Lin; p.Lout = a->Lout; p.ncols = ncols;
    p.x_bstride = a->x_bstride ? a->x_bstride : a->Ci * a->Lin;
    p.y_bstride = a->y_bstride ? a->y_bstride : a->Co * a->Lout;
    p.res_bstride = a->res_bstride ? a->res_bstride : a->Co * a->Lout;
    p.w_bstride = a->w_bstride;
    p.K = a->K; p.stride = a->stride; p.dil = a->dil; p.pad = a->pad; p.groups = a->groups;
    p.nphase = a->nphase; p.ostride = a->ostride; p.ooffset = a->ooffset;
    p.in_act = a->in_act; p.out_act = a->out_act; p.accumulate = a->accumulate;
    p.in_scale = a->in_scale; p.in_slope = a->in_slope; p.out_slope = a->out_slope; p.out_scale = a->out_scale;
    p.ntoff = a->ntoff; p.wrap = a->wrap;
    for (int i = 0; i < 16; ++i) p.toff[i] = a->ntoff ? a->toff[i] : 0;
    p.span = span;
    p.span_s = span + 1;
    p.rows_max = rows_max;
    p.inv_span = 1.0f / (float)span;
    p.avec = (Cog % 4 == 0) && (((uintptr_t)a->w & 15) == 0) && (a->w_bstride % 4 == 0);
    p.mtiles_per_group = (int)((Cog + BM - 1) / BM);

    const int64_t tiles = (int64_t)p.mtiles_per_group * a->groups * ((ncols + BN - 1) / BN) * a->B * a->nphase;
    const int nch = (int)((Cig * a->K + KCH - 1) / KCH);
    int ks = 1;
    if (tiles < 512 && nch >= 4) {
        ks = (int)((512 + tiles - 1) / tiles);
        if (ks > 16) ks = 16;
        if (ks > nch / 2) ks = nch / 2;
        if (ks < 1) ks = 1;
    }
    p.chunks_per_split = (nch + ks - 1) / ks;
    ks = (nch + p.chunks_per_split - 1) / p.chunks_per_split;
    p.ksplit = ks;
    const int WS = (BM / 32) * 32 + 16 + ((BM % 32) ? 32 : 0);
    lds = (size_t)(KCH * WS + KCH) * 4 + ((size_t)rows_max * p.span_s + 4) * 4;  // +dump slot
    RVC_CHECK_ARG(lds <= 160 * 1024, "conv1d: LDS %zu too large", lds);
    grid = dim3(cdiv(ncols, BN), (unsigned)(p.mtiles_per_group * a->groups), (unsigned)(a->B * a->nphase * ks));
    RVC_CHECK_ARG(grid.y < 65536 && grid.z < 65536, "conv1d: grid too large");
    return RVC_OK;
}

}  // namespace

extern "C" int64_t rvc_conv1d_workspace_bytes(const rvc_conv1d_args* a) {
    ConvParams p;
    Cfg cfg;
    dim3 grid;
    size_t lds;
    if (plan(a, p, cfg, grid, lds) != RVC_OK) return -1;
    if (p.ksplit <= 1) return 0;
    return (int64_t)p.ksplit * p.B * p.nphase * p.Co * p.ncols * 4;
}

extern "C" int rvc_conv1d(const rvc_conv1d_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream) {
    ConvParams p;
    Cfg cfg;
    dim3 grid;
    size_t lds;
    int rc = plan(a, p, cfg, grid, lds);
    if (rc != RVC_OK) return rc;
    if (p.ksplit > 1) {
        const int64_t need = (int64_t)p.ksplit * p.B * p.nphase * p.Co * p.ncols * 4;
        RVC_CHECK_ARG(ws && ws_bytes >= need, "conv1d: split-K needs %lld B of workspace (got %lld)",
                      (long long)need, (long long)ws_bytes);
        p.ws = (float*)ws;
    }
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (cfg.FM == 3) e = launch<3, 1, 1, 4>(p, grid, lds, s);
    else if (cfg.FM == 1 && cfg.FN == 4) e = launch<1, 4, 1, 4>(p, grid, lds, s);
    else if (cfg.FM == 1) e = launch<1, 2, 1, 4>(p, grid, lds, s);
    else if (cfg.WM == 1 && cfg.FN == 4) e = launch<2, 4, 1, 4>(p, grid, lds, s);
    else if (cfg.WM == 1) e = launch<2, 2, 1, 4>(p, grid, lds, s);
    else if (cfg.FM == 4 && cfg.FN == 4) e = launch<4, 4, 2, 2>(p, grid, lds, s);
    else if (cfg.FM == 4) e = launch<4, 2, 2, 2>(p, grid, lds, s);
    else if (cfg.FN == 4) e = launch<2, 4, 2, 2>(p, grid, lds, s);
    else e = launch<2, 2, 2, 2>(p, grid, lds, s);
    RVC_HIP(e);
    if (p.ksplit > 1) {
        hipLaunchKernelGGL(conv_splitk_reduce, dim3(cdiv(p.ncols, 256), (unsigned)p.Co, (unsigned)(p.B * p.nphase)),
                           dim3(256), 0, s, p);
        RVC_HIP(hipGetLastError());
    }
    return RVC_OK;
}
