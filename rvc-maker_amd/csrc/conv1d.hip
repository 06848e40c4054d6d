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
#include "x6_common.h"
#include <stdlib.h>
#include <type_traits>
#include <algorithm>

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
    const uint4* wx;  // split-bf16 packed weights (x6 engine) or null
    int wx_nmf, wx_nch, wx_passes;
    int rot;  // x6: rotate each block's (chunk, tap) order so that the CUs of an XCD spread over the weight image
    int xcd;  // x6: XCD-aware tile order (each XCD takes a contiguous run of tiles: row tiles share weights in its L2)
    int dbg;  // RVC_CONV_DEBUG (profiling only): 1 = no epilogue, 2 = no MFMA, 4 = loaders skip global loads
    int tile_epi;  // x6: the tile epilogue through LDS (x6_tile_epilogue), set by plan() for plain stride-1 stores
    const unsigned* amax_in;  // |max| of x (f32 bits) or null: split-fp16 loaders take their scale from it
    int f16_fast;             // split-fp16 with amax_in: the fast loader form (RVC_X6_F16FAST, A/B switch)
    unsigned* amax_out;       // or null: max |y| over the stored values (atomic max of the f32 bits)
    int stagger;              // x6: the first round of blocks starts spread over this many shader cycles (0 = off)
    int stagger_blocks;       // ... the blocks of that round (one per CU)
    int swz;                  // x6: the 128-byte-row epilogue (conv_epilogue_swz; RVC_X6_SWZ, rvc_conv1d_set_swz)
    int gx6;                  // x6 grouped conv: the phase index is the group (Ci, Co per group; image packed per group)
#if RVC_CONV_STAMPS
    unsigned long long* stamps;  // diagnostic build only: [block][X6_STAMP_W] s_memtime stamps (rvc_conv1d_set_stamps)
    int64_t stamp_blocks;
#endif
};

// per-thread override of the split-fp16 fast loader form (rvc_conv1d_set_f16_fast; -1 = RVC_X6_F16FAST, default on)
static thread_local int g_f16_fast = -1;
// per-thread override of the 128-byte-row epilogue (rvc_conv1d_set_swz; -1 = RVC_X6_SWZ, default on)
static thread_local int g_swz = -1;

__device__ __forceinline__ int tap_off(const ConvParams& p, int t) { return p.ntoff ? p.toff[t] : t * p.dil; }

// Output column n -> store position t; -1 when the column is not stored (beyond ncols / Lout);
// -(t + 2) for a border cell of a 2-D image, which is stored as 0 (the bordered [C][H+2][W+2]
// images then need no zero-fill).  32-bit math: every per-batch extent here is < 2^31.
__device__ __forceinline__ int out_pos(const ConvParams& p, int64_t n, int phase) {
    if (n >= p.ncols) return -1;
    const int t = (int)n * p.ostride + p.ooffset + phase;
    if (t < 0 || t >= (int)p.Lout) return -1;
    if (p.wrap) {
        const int row = t / p.wrap, col = t - row * p.wrap;
        if (col == 0 || col == p.wrap - 1 || row == 0 || row == (int)p.Lout / p.wrap - 1) return -(t + 2);
    }
    return t;
}

// Branch-free epilogue for one element: every load is issued unconditionally from a clamped
// address (a per-element guarded load makes hipcc branch and wait vmcnt(0) per element).
// returns the value stored (0 when nothing is stored: a border cell stores 0, a column past the end nothing)
__device__ __forceinline__ float epilogue_store(const ConvParams& p, float acc, int b, int64_t m, int t) {
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
    else if (t <= -2) yb[m * p.Lout + (-t - 2)] = 0.f;  // 2-D border cell
    return ok ? v : 0.f;
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

// Shared epilogue of the conv engines (both produce the MFMA 16x16 C layout: lane l holds column
// l&15, rows (l>>4)*4 + r of each fragment).  Split-K partial tiles go to the workspace (summed in split
// order by conv_splitk_reduce); otherwise bias, 2nd bias, activation, scale, residual, accumulate and the
// (strided / polyphase / masked) store are fused here.
template <int FM, int FN, int WM, int WN>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, floatx4 (&acc)[FM][FN], int lane, int wm, int wn,
                                              int split, int phase, int b, int g, int Cog, int m0g, int64_t n0) {
    const int ln = lane & 15;
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
    float amx = 0.f;  // amax_out: largest |stored value| of this lane
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
            for (int j = 0; j < FN; ++j) {
                if (mok[r] && tcol[j] >= 0) {
                    yb[mrow[r] * Lo + tcol[j]] = av[0][j][r];
                    amx = fmaxf(amx, fabsf(av[0][j][r]));
                } else if (mok[r] && tcol[j] <= -2) {
                    yb[mrow[r] * Lo + (-tcol[j] - 2)] = 0.f;  // 2-D border cell
                }
            }
    }
    if (p.amax_out) amax_publish(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);  // the batch element's cell
}

// The same epilogue with 128-byte rows (round 6, x6 engine, even FN, no split-K): a 16x16 accumulator register holds 4
// rows x 16 columns (4 x 64-B segments per load / store instruction, a shape the guide leaves unmeasured); one
// v_permlane16_swap per register pair of two adjacent column fragments regroups them so that each register holds 2 rows
// x 32 consecutive columns -- 2 x 128-B segments, the access shape MI355X_MICROARCH.md rates at full rate -- for every
// residual / accumulate load and every store.  After the swap of fragments (2 jp, 2 jp + 1), register r of the first is
// row r + 8 h, of the second row 4 + r + 8 h (h = lane >> 5), both at column 32 jp + (lane & 31).  Same operations in
// the same order per element as conv_epilogue, so the same bits.
template <int FM, int FN, int WM, int WN>
__device__ __forceinline__ void conv_epilogue_swz(const ConvParams& p, floatx4 (&acc)[FM][FN], int lane, int wm, int wn,
                                                  int phase, int b, int g, int Cog, int m0g, int64_t n0) {
    static_assert(FN % 2 == 0, "column fragments in pairs");
    constexpr int NP = FN / 2;
    const int h = lane >> 5, lc = lane & 31;
    int tcol[NP];
#pragma unroll
    for (int jp = 0; jp < NP; ++jp) tcol[jp] = out_pos(p, n0 + wn * 16 * FN + jp * 32 + lc, phase);
    float* yb = p.y + b * p.y_bstride;
    const float* rb2 = p.res ? p.res + b * p.res_bstride : nullptr;
    const int Lo = (int)p.Lout;
    float amx = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int jp = 0; jp < NP; ++jp)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][r]),
                                                                 __float_as_uint(acc[i][2 * jp + 1][r]), false, false);
                acc[i][2 * jp][r] = __uint_as_float(sw[0]);
                acc[i][2 * jp + 1][r] = __uint_as_float(sw[1]);
            }
        // element (jp, k): k < 4 register k of fragment 2 jp, else register k - 4 of fragment 2 jp + 1; row k + 8 h
        floatx4 (&av)[1][FN] = *reinterpret_cast<floatx4 (*)[1][FN]>(&acc[i][0]);
        int mrow[8];
        bool mok[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int mg = m0g + wm * 16 * FM + i * 16 + 8 * h + k;
            mok[k] = mg < Cog;
            mrow[k] = g * Cog + (mg < Cog ? mg : 0);
            float bs = 0.f;
            if (p.bias) bs = p.bias[mrow[k]];
            if (p.bias2) bs += p.bias2[mrow[k]];
#pragma unroll
            for (int jp = 0; jp < NP; ++jp) av[0][2 * jp + (k >> 2)][k & 3] += bs;
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
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int jp = 0; jp < NP; ++jp)
                    av[0][2 * jp + (k >> 2)][k & 3] += rb2[mrow[k] * Lo + (tcol[jp] >= 0 ? tcol[jp] : 0)];
        }
        if (p.accumulate) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int jp = 0; jp < NP; ++jp)
                    av[0][2 * jp + (k >> 2)][k & 3] += yb[mrow[k] * Lo + (tcol[jp] >= 0 ? tcol[jp] : 0)];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int jp = 0; jp < NP; ++jp) {
                const float v = av[0][2 * jp + (k >> 2)][k & 3];
                if (mok[k] && tcol[jp] >= 0) {
                    yb[mrow[k] * Lo + tcol[jp]] = v;
                    amx = fmaxf(amx, fabsf(v));
                } else if (mok[k] && tcol[jp] <= -2) {
                    yb[mrow[k] * Lo + (-tcol[jp] - 2)] = 0.f;  // 2-D border cell
                }
            }
    }
    if (p.amax_out) amax_publish(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);
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

    conv_epilogue<FM, FN, WM, WN>(p, acc, lane, wm, wn, split, phase, b, g, Cog, m0g, n0);
}

// ------------------------------------------------------------------ split-bf16 ("x6") engine
// f32 convolution on the bf16 matrix cores: every f32 operand is split exactly into three bf16
// pieces (x = h + m + l, |x - (h+m+l)| <= 2^-27 |x|) and the product keeps the six terms down to
// the 2^-24 level: hH + hM + mH + hL + mM + lH (v_mfma_f32_16x16x32_bf16, f32 accumulation).
// That is f32-level accuracy at 6 x 16 cycles per 16x16x32 block against 8 x 32 for the f32 MFMA
// (2.7x the f32 matrix rate).  Stride-1, ungrouped 1-D convs (everything hot in the generator,
// flow, TextEncoder and the ContentVec linears).
//
// k-steps are (32-channel chunk, tap): a chunk's input rows are staged ONCE into LDS (split into
// h/m/l planes, channel-contiguous [pos][32 ch] rows, 16-B groups XOR-swizzled (x6_common.h x_slot) so
// both the staging writes and the operand reads are conflict-free) and reused by all K taps.
// B operands are one ds_read_b128 per plane per fragment; A operands (weights) come pre-split
// and pre-arranged per lane from global memory (L2-resident), prefetched one k-step ahead.
constexpr int X6_NI_MAX = 6;  // staged (position, 8-channel group) items per loader thread: 4 * span <= 256 NI
// Profiling ablations (RVC_CONV_DEBUG at run time) exist only in a -DRVC_CONV_ABLATIONS=1 build: a run-time
// test inside the k-loop made hipcc split every fragment's MFMAs into two paths with register copies,
// lgkmcnt(0) / vmcnt(0) waits in front of them and a branch per 6 MFMAs, and the loaders' per-element
// "load or zero" select serialised their loads.
#ifndef RVC_CONV_ABLATIONS
#define RVC_CONV_ABLATIONS 0
#endif
constexpr bool kAblations = RVC_CONV_ABLATIONS != 0;
#ifndef X6_BPIN
#define X6_BPIN 0
#endif
#ifndef X6_NOBAR
#define X6_NOBAR 0  // profiling ablation only: no per-chunk barrier (races, wrong results)
#endif
#if X6_NOBAR && !RVC_CONV_ABLATIONS
#error "X6_NOBAR races (wrong results): only in a -DRVC_CONV_ABLATIONS=1 profiling build"
#endif
#ifndef X6_PD8
#define X6_PD8 0
#endif
#ifndef X6_F16FAST
#define X6_F16FAST 0
#endif
// In-kernel stamps (diagnostic build -DRVC_CONV_STAMPS=1 only; scripts/conv_stamps.py): compute wave 0 and the first
// loader wave record s_memtime at the phase boundaries of each block into a buffer of their own (never an output),
// one lane, vector stores.  Layout per block (X6_STAMP_W words): 0 compute start, 1 memrealtime at start, 2 HW_ID,
// 3 compute: prefetch issued, 4 compute: F16 scale barrier passed, 5 compute: chunk 0 barrier passed,
// 6 compute: k-loop done, 7 compute: epilogue done, 8 loader start, 9 loader: F16 |max| published,
// 10 loader: chunk 0 staged, 11 loader: loop done, 12 number of chunks, 14 compute: epilogue stores issued; then per
// chunk c (< X6_STAMP_NC):
// 16 + 4c: compute arrives at chunk c's barrier, +1 released, +2 loader arrives, +3 released.
#ifndef RVC_CONV_STAMPS
#define RVC_CONV_STAMPS 0
#endif
constexpr int X6_STAMP_W = 256, X6_STAMP_NC = 60;
#if RVC_CONV_STAMPS
#define X6_STAMP(slot, val)                                                                                      \
    do {                                                                                                          \
        const int64_t sb_ = (int64_t)blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z); \
        if (p.stamps && lane == 0 && sb_ < p.stamp_blocks && (slot) < X6_STAMP_W)                                 \
            p.stamps[sb_ * X6_STAMP_W + (slot)] = (val);                                                         \
    } while (0)
#else
#define X6_STAMP(slot, val) \
    do {                    \
    } while (0)
#endif
#define X6_NOW() ((unsigned long long)__builtin_amdgcn_s_memtime())

// Block = 8 waves: waves 0-3 compute (WM x WN), waves 4-7 stage the input.  Each role keeps only its
// own loads in its vmcnt queue, so the compute waves' weight prefetch and the loaders' two-chunk-deep
// input prefetch never wait on each other.  One workgroup barrier per 32-channel chunk hands the
// next staged X buffer (double-buffered in LDS) to the compute waves.
// Small tiles (FM x FN <= 4 fragments per wave: <= 32-channel convs) are short blocks whose prologue
// and epilogue latencies dominate: they are built for 2 co-resident blocks per CU (<= 128 VGPRs,
// a 1-deep weight ring) so that one block's waits overlap the other's MFMAs.
// (measured on the 32-channel generator convs: -17..20 % at 6 and 3 passes, +8 % at 1 pass, which
// stays at one block).
template <int FM, int FN, int NCW, int NP>
constexpr int x6_min_blocks() { return (FM * FN <= 4 && NCW == 4 && NP >= 3) ? 2 : 1; }

// F16 (with NP = 3): the split-fp16 arithmetic (x6_common.h split2h): wx is an rvc_conv1d_pack_f16 image
// (h / l fp16 planes of per-row-scaled weights, then the rows' reciprocal scales); the loader waves first
// take the tile's |max| over every chunk of the block's k range (the chunks beyond the first two are
// loaded for it alone; they stay in L2 for the staging pass), agree on a power-of-2 scale through LDS, and
// stage the scaled activations as h / l planes; the epilogue multiplies by both reciprocal scales (exact).
// SA (with NP = 6): the five correction passes (hM mH hL mM lH, each <= 2^-8 of hH) accumulate apart from
// hH and the two sums are added once at the end: the f32 accumulator of the large terms is rounded once per
// 32 products instead of six times, the corrections' roundings are 2^-8 smaller (RMVPE, whose f0 is a
// per-frame decision: scripts/conv_prec.py).
// The loaders keep one chunk in flight in registers (chunk c + 2's loads are issued while chunk c computes, after
// chunk c + 1 was staged).  A 4-deep ring (with an L2 prefetch of the K = 1 weight panels by the loaders) measured
// no faster on ContentVec's K = 1 GEMMs and slower end to end: not kept.
// The x6 engine's tile epilogue (round 5).  The in-register epilogue (conv_epilogue) made each compute wave issue
// one dword load per residual / accumulate element and one dword store per output (64 stores per wave on the
// 128 x 256 tile), in FM passes, with the 4 loader waves idle: in-kernel stamps put it at 29k of a 154k-cycle block
// on the hottest conv (scripts/conv_stamps.py), the MFMA pipe idle throughout.  Here the compute waves finish
// bias / activation / scale in registers and write their fragments into the block's LDS (the X buffers are dead
// after the last chunk), then ALL waves of the block stream the tile row-major: every residual / accumulate load
// issued first (16 B per lane), then the adds and 16-B stores.  Same operations in the same order per element as
// conv_epilogue, so the outputs are the same bits.  Split-K blocks store their raw partial tile to the workspace
// the same way.  Only plain stores (one phase, output column = GEMM column): plan() sets p.tile_epi.
template <int BM, int BN, int NT>
__device__ __forceinline__ void x6_tile_epilogue(const ConvParams& p, const float* ot, int tid, int split, int b,
                                                 int m0g, int64_t n0) {
    constexpr int TS = BN + 4, C4 = BN / 4, NV = BM * C4, IT = (NV + NT - 1) / NT;
    const int Cog = (int)p.Co;
    const bool part = p.ksplit > 1;
    // destination rows and the columns valid in this tile
    float* dst;
    const float* rb = nullptr;
    const float* yb_in = nullptr;
    int64_t ld;
    int lim;
    if (part) {
        dst = p.ws + (((int64_t)split * p.B + b) * p.Co) * p.ncols;
        ld = p.ncols;
        lim = (int)min((int64_t)BN, p.ncols - n0);
    } else {
        dst = p.y + b * p.y_bstride;
        ld = p.Lout;
        lim = (int)min((int64_t)BN, min(p.ncols, p.Lout) - n0);
        if (p.res) rb = p.res + b * p.res_bstride;
        if (p.accumulate) yb_in = dst;
    }
    const bool vec = lim == BN && (ld & 3) == 0 && ((uintptr_t)dst & 15) == 0 && ((uintptr_t)rb & 15) == 0;
    float amx = 0.f;  // amax_out: largest |stored value| of this thread (final values only, not split-K partials)
    if (vec) {
        float4 rv[IT], av[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {  // every load first, from clamped addresses
            const int idx = tid + it * NT;
            const int row = idx / C4, c = (idx - row * C4) * 4;
            const int m = m0g + row;
            const int64_t o = (int64_t)(idx < NV && m < Cog ? m : 0) * ld + n0 + c;
            if (rb) rv[it] = *reinterpret_cast<const float4*>(rb + o);
            if (yb_in) av[it] = *reinterpret_cast<const float4*>(yb_in + o);
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int idx = tid + it * NT;
            const int row = idx / C4, c = (idx - row * C4) * 4;
            const int m = m0g + row;
            if (idx < NV && m < Cog) {
                float4 v = *reinterpret_cast<const float4*>(ot + row * TS + c);
                if (rb) {
                    v.x += rv[it].x;
                    v.y += rv[it].y;
                    v.z += rv[it].z;
                    v.w += rv[it].w;
                }
                if (yb_in) {
                    v.x += av[it].x;
                    v.y += av[it].y;
                    v.z += av[it].z;
                    v.w += av[it].w;
                }
                *reinterpret_cast<float4*>(dst + (int64_t)m * ld + n0 + c) = v;
                amx = fmaxf(amx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            }
        }
        if (p.amax_out && !part) amax_publish(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);
        return;
    }
    // edge tile (the last column tile) or unaligned rows: element by element, lanes along the row
    constexpr int NS = BM * BN, ITS = (NS + NT - 1) / NT;
#pragma unroll 4
    for (int it = 0; it < ITS; ++it) {
        const int idx = tid + it * NT;
        const int row = idx / BN, c = idx - row * BN;
        const int m = m0g + row;
        if (idx < NS && m < Cog && c < lim) {
            const int64_t o = (int64_t)m * ld + n0 + c;
            float v = ot[row * TS + c];
            if (rb) v += rb[o];
            if (yb_in) v += yb_in[o];
            dst[o] = v;
            amx = fmaxf(amx, fabsf(v));
        }
    }
    if (p.amax_out && !part) amax_publish(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);
}

// LF (split-fp16 on 8 compute waves, with the producer's |max|: amax_in): the loaders take ONLY the fast form (1: leaky
// ReLU pre-activation, 2: none) -- a kernel of its own, so the general form's registers are not allocated beside it
template <int FM, int FN, int WM, int WN, int X6_NI, int NP, bool F16, bool SA = false, int LF = 0>
__global__ __launch_bounds__(64 * (WM * WN + 4), (x6_min_blocks<FM, FN, WM * WN, NP>())) void conv_x6_kernel(ConvParams p) {
    static_assert(WM * WN == 4 || WM * WN == 8, "4 or 8 compute waves");
    constexpr int NCW = WM * WN;  // compute waves; 4 loader waves follow them
    static_assert(NP == 6 || NP == 3 || NP == 1, "6, 3 or 1 passes");
    static_assert(!F16 || NP == 3, "split-fp16: 3 passes");
    static_assert(!SA || (NP == 6 && !F16), "split accumulators: 6-pass split-bf16");
    static_assert(LF == 0 || (F16 && WM * WN == 8), "fast-only loaders: split-fp16 on 8 compute waves");
    constexpr int NPL = NP == 6 ? 3 : (NP == 3 ? 2 : 1);
    constexpr int BM = 16 * FM * WM;
    constexpr int BN = 16 * FN * WN;
    extern __shared__ uint4 xs[];  // [2 buffers][span][NPL planes][4 x 16 B]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // XCD-aware tile order (cdna_hip_programming.md T1, the bijective form): blocks are dealt round-robin over
    // the 8 XCDs, so block b serves tile t(b), which gives each XCD a contiguous run of the row-major tile
    // order -- whole rows of column tiles, which read the same weight fragments, share that XCD's L2 instead
    // of each XCD fetching every row's weights.  Speed only: every tile computes the same sums either way.
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (p.xcd) {
        const int nx = gridDim.x, ny = gridDim.y;
        const int nwg = nx * ny * (int)gridDim.z;
        const int orig = bx + nx * (by + ny * bz);
        const int q = nwg >> 3, r = nwg & 7, xc = orig & 7;
        const int t = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + (orig >> 3);
        bx = t % nx;
        by = (t / nx) % ny;
        bz = t / (nx * ny);
    }
    int zb = bz;
    const int split = zb % p.ksplit;
    zb /= p.ksplit;
    const int phase = zb % p.nphase;
    const int b = zb / p.nphase;
    // a grouped conv (gx6, ContentVec's pos_conv) runs its groups as phases: the phase selects the group's weight image,
    // input channel rows and output channel rows; its outputs are stored unphased
    const int grp = p.gx6 ? phase : 0;
    const int ophase = p.gx6 ? 0 : phase;
    const int Cog = (int)p.Co;
    const int Cig = (int)p.Ci;
    const int m0g = by * BM;
    const int64_t n0 = (int64_t)bx * BN;
    const int K = p.K, span = p.span;
    const int nch = p.wx_nch, nmf = p.wx_nmf;
    const int ch_beg = split * p.chunks_per_split;
    const int ch_end = min(nch, ch_beg + p.chunks_per_split);
    const int nck = ch_end - ch_beg;
    const int bufsz = NPL * span * 4;  // uint4 per buffer
    float* tmax = reinterpret_cast<float*>(xs + 2 * bufsz);  // F16: the 4 loader waves' tile |max|
    // Blocks co-resident on one XCD (ids = x mod 8) walk the k-steps from different starting
    // (chunk, tap): in lockstep they would all read the same few weight lines, i.e. the same L2 channels.
    const int rseed = p.rot ? (bx >> 3) : 0;
    const int rt = rseed % K, rc = (rseed / K) % max(nck, 1);
    // logical chunk i (clamped to the last) -> physical chunk; rc < nck, so one conditional subtract, no division
    auto pchunk = [&](int i) __attribute__((always_inline)) {
        const int c = min(i, nck - 1) + rc;
        return ch_beg + (c >= nck ? c - nck : c);
    };

    // Staggered start (p.stagger): the blocks of a launch all do the same work, so the first round's blocks -- and the
    // rounds that follow them on each CU -- reach their epilogues together, and the epilogue (residual loads, stores)
    // then runs HBM-bound chip-wide while HBM sits idle through the MFMA loops (stamps, rb128_k11: 34k cycles of a 147k
    // block with the residual, 16k without).  Delaying the first round's block i by a permutation of [0, stagger)
    // spreads every later round's epilogues over the block period.
    if (p.stagger) {
        const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if (lin < p.stagger_blocks) {
            const unsigned long long t0 = X6_NOW();
            const unsigned long long d = ((unsigned long long)((lin * 97) & 255) * (unsigned)p.stagger) >> 8;
            while (X6_NOW() - t0 < d) __builtin_amdgcn_s_sleep(2);
        }
    }
    if (wave == 0) {
        X6_STAMP(0, X6_NOW());
        X6_STAMP(1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
        X6_STAMP(2, (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));  // HW_ID
        X6_STAMP(12, (unsigned long long)(min(nch, ch_beg + p.chunks_per_split) - ch_beg));
        X6_STAMP(13, (unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)));  // XCC_ID
    }
    if (wave >= NCW) {
        // ---------------- loader waves: chunk c+1 split into LDS while chunk c computes
        const int ltid = tid - 64 * NCW;
        const bool lw0 = wave == NCW;
        if (lw0) X6_STAMP(8, X6_NOW());
        const int lin = (int)p.Lin;
        const float* xb = p.x + b * p.x_bstride + (int64_t)grp * Cig * p.Lin;
        const int base = (int)(n0 * p.stride - p.pad);
        int ipos[X6_NI], ig8[X6_NI];
        unsigned iok = 0;
#pragma unroll
        for (int it = 0; it < X6_NI; ++it) {
            const int idx = ltid + 256 * it;
            const int g8 = idx / span;
            ig8[it] = g8 < 4 ? g8 : 3;
            ipos[it] = idx - g8 * span;
            const int q = base + ipos[it];
            iok |= (unsigned)(idx < 4 * span && q >= 0 && q < lin) << it;
        }
      auto loader = [&](auto fast_c, auto lrelu_c) __attribute__((always_inline)) {
        // FASTL: every chunk holds 32 real channels (Ci % 32 == 0), no input scale, and the pre-activation is
        // fixed at compile time (LRELU: leaky ReLU, else none) -- the loads take a wave-uniform row base plus
        // one 32-bit per-lane offset (no per-element 64-bit address arithmetic or channel clamp) and the split
        // converts pairs (v_cvt_pk_bf16_f32); the general form handles everything else.  At K = 1 the loaders'
        // split is the per-chunk cost (one k-step of MFMAs per chunk), ~20 vector instructions per element in
        // the general form against ~7 here; the results are the same bits.
        constexpr bool FASTL = decltype(fast_c)::value;
        constexpr bool LRELU = decltype(lrelu_c)::value;
        uint32_t ioff[X6_NI];  // FASTL: element offset of (row 8 ig8, clamped position) within a chunk's rows
#pragma unroll
        for (int it = 0; it < X6_NI; ++it) {
            const int q = base + ipos[it];
            const int qc = q < 0 ? 0 : (q >= lin ? lin - 1 : q);
            ioff[it] = (uint32_t)(ig8[it] * 8 * lin + qc);
        }
        // General form: items are PAIRS of consecutive input positions (q, q + 1) with q even -- one 8-byte load per
        // channel, half the loads of one position per item, so that the ring (NI2 x 8 loads of a chunk in flight)
        // stays far below what vmcnt can count; with single positions the 6-item split-fp16 loaders kept 96 loads
        // in flight and waited vmcnt(0) per chunk.  Pair it covers staged positions ppos and ppos + 1 (the first
        // may be -1, unstaged); element j is always lane .x / .y of its load, so no per-element select -- a
        // select between two ring registers made hipcc keep the ring in scratch.  A pair starting below 0 is
        // wholly masked (q even), one past the end of a row reads the next row or 0 (buffer range): masked too.
        constexpr int NI2 = (X6_NI + 1) / 2;
        const int par = base & 1;
        const int npair = (span + par + 1) >> 1;
        int ppos[NI2], pg8[NI2], pq[NI2];
        unsigned pok = 0, pstage = 0;
#pragma unroll
        for (int it = 0; it < NI2; ++it) {
            const int idx = ltid + 256 * it;
            const int g8 = idx / npair;
            pg8[it] = g8 < 4 ? g8 : 3;
            ppos[it] = 2 * (idx - g8 * npair) - par;
            const int q0 = base + ppos[it];  // even
            pq[it] = q0 < 0 ? 0 : q0;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int bit = 2 * it + j, q = q0 + j, pos = ppos[it] + j;
                const bool staged = idx < 4 * npair && pos >= 0 && pos < span;
                pstage |= (unsigned)staged << bit;
                pok |= (unsigned)(staged && q >= 0 && q < lin) << bit;
            }
        }
        constexpr int NR = FASTL ? X6_NI : 2 * NI2;  // ring rows per chunk: items (fast form) or pair halves
        float xr[2][NR][8];  // slot 1: the chunk in flight; slot 0: chunk 0 and the split-fp16 |max| pass
        auto xload = [&](int ch, float (&r)[NR][8]) __attribute__((always_inline)) {
            // unconditional (clamped) loads so that the vmcnt bookkeeping is static
            if constexpr (FASTL) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float* xrow = xb + (int64_t)(ch * 32 + e) * lin;  // wave-uniform
#pragma unroll
                    for (int it = 0; it < X6_NI; ++it) r[it][e] = (kAblations && (p.dbg & 4)) ? 0.f : xrow[ioff[it]];
                }
            } else {
                // general form: position pairs, one 8-byte buffer load per channel (see the pair mapping above):
                // a per-chunk buffer resource over the chunk's (at most 32) real channel rows -- rows past Ci read
                // 0 by the range check, so the per-lane byte offsets are chunk-invariant (24 VGPRs, no 64-bit
                // address per load; Lin < 2^24: x6_eligible)
                const int c0 = __builtin_amdgcn_readfirstlane(ch * 32);
                const int nrow = Cig - c0 < 32 ? Cig - c0 : 32;
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    (void*)(xb + (int64_t)c0 * lin), (short)0, nrow * lin * 4, 0x00020000);
#pragma unroll
                for (int it = 0; it < NI2; ++it)
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int off = ((pg8[it] * 8 + e) * lin + pq[it]) * 4;
                        const rvc_f2 v = __builtin_bit_cast(rvc_f2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
                        r[2 * it][e] = (kAblations && (p.dbg & 4)) ? 0.f : v.x;
                        r[2 * it + 1][e] = (kAblations && (p.dbg & 4)) ? 0.f : v.y;
                    }
            }
        };
        float sc = 1.f;  // F16: the tile's activation scale (power of 2)
        auto xstore_fast = [&](int ch, const float (&r)[NR][8], uint4* dst) __attribute__((always_inline)) {
#pragma unroll
            for (int it = 0; it < X6_NI; ++it) {
                if (ltid + 256 * it < 4 * span) {
                    uint32_t hw[4], mw[4], lw[4];
                    {  // the fast form (FASTL; split-fp16 only with the producer's |max|, amax_in)
                        const bool ok = (iok >> it) & 1u;
#pragma unroll
                        for (int e2 = 0; e2 < 4; ++e2) {
                            float v0 = r[it][2 * e2], v1 = r[it][2 * e2 + 1];
                            if constexpr (LRELU) {
                                v0 = v0 >= 0.f ? v0 : v0 * p.in_slope;
                                v1 = v1 >= 0.f ? v1 : v1 * p.in_slope;
                            }
                            if constexpr (F16) split2h_pk(ok ? v0 * sc : 0.f, ok ? v1 * sc : 0.f, hw[e2], mw[e2]);
                            else split3_pk(ok ? v0 : 0.f, ok ? v1 : 0.f, hw[e2], mw[e2], lw[e2]);
                        }
                    }
                    const int pos = ipos[it];
                    dst[x_slot<NPL>(pos, 0, ig8[it])] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                    if constexpr (NPL >= 2) dst[x_slot<NPL>(pos, 1, ig8[it])] = make_uint4(mw[0], mw[1], mw[2], mw[3]);
                    if constexpr (NPL >= 3) dst[x_slot<NPL>(pos, 2, ig8[it])] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                }
            }
        };
        // general form: pair it's element j (position ppos + j) is lane .x (j = 0) / .y (j = 1) of its load
        auto xstore_gen = [&](int ch, const float (&r)[2 * NI2][8], uint4* dst) __attribute__((always_inline)) {
#pragma unroll
            for (int it = 0; it < NI2; ++it)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int bit = 2 * it + j;
                    if ((pstage >> bit) & 1u) {
                        uint32_t hw[4], mw[4], lw[4];
#pragma unroll
                        for (int e2 = 0; e2 < 4; ++e2) {
                            float v2[2];
#pragma unroll
                            for (int u = 0; u < 2; ++u) {
                                const int e = 2 * e2 + u;
                                const bool ok = ((pok >> bit) & 1u) && ch * 32 + pg8[it] * 8 + e < Cig;
                                float v = r[2 * it + j][e] * p.in_scale;
                                if (p.in_act == RVC_ACT_LRELU) v = v >= 0.f ? v : v * p.in_slope;
                                v2[u] = ok ? (F16 ? v * sc : v) : 0.f;
                            }
                            if constexpr (F16) split2h_pk(v2[0], v2[1], hw[e2], mw[e2]);
                            else split3_pk(v2[0], v2[1], hw[e2], mw[e2], lw[e2]);
                        }
                        const int pos = ppos[it] + j;
                        dst[x_slot<NPL>(pos, 0, pg8[it])] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                        if constexpr (NPL >= 2) dst[x_slot<NPL>(pos, 1, pg8[it])] = make_uint4(mw[0], mw[1], mw[2], mw[3]);
                        if constexpr (NPL >= 3) dst[x_slot<NPL>(pos, 2, pg8[it])] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                    }
                }
        };
        auto xstore = [&](int ch, const float (&r)[NR][8], uint4* dst) __attribute__((always_inline)) {
            if constexpr (FASTL) xstore_fast(ch, r, dst);
            else xstore_gen(ch, r, dst);
        };
        // prologue: chunk 0 -> LDS buffer 0, chunk 1 in flight in ring slot 1
        if constexpr (F16) {
            // tile |max| over the raw loads (clamped addresses read real elements of x, and lrelu only
            // shrinks: an upper bound of |pre(x)| over the staged tile); chunks 0 and 1 are loaded last and kept
            auto rmax = [&](const float (&r)[NR][8]) __attribute__((always_inline)) {
                float m = 0.f;
#pragma unroll
                for (int it = 0; it < NR; ++it)
#pragma unroll
                    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(r[it][e]));
                return m;
            };
            float am = 0.f;
            const bool cell = FASTL || p.amax_in;  // block-uniform
            if (cell) {
                // the producer published |max| of the whole input tensor (amax side channel): no pre-pass (the fast
                // form is only dispatched with amax_in, so its body never instantiates the pre-pass).  The chunk loads
                // go first: the cell is read through the scalar cache (its own counter), so its latency -- a line
                // the producer's atomics left at the memory side -- overlaps theirs
                xload(pchunk(0), xr[0]);
                xload(pchunk(1), xr[1]);
                am = amax_read(p.amax_in + (int64_t)b * RVC_AMAX_SHARDS) * fabsf(p.in_scale);  // the element's cell
            } else if constexpr (!FASTL) {
                for (int i = 2; i < nck; i += 2) {
                    xload(pchunk(i), xr[0]);
                    xload(pchunk(i + 1 < nck ? i + 1 : i), xr[1]);
                    am = fmaxf(am, fmaxf(rmax(xr[0]), rmax(xr[1])));
                }
                xload(pchunk(0), xr[0]);
                xload(pchunk(1), xr[1]);
                am = wave_max(fmaxf(am, fmaxf(rmax(xr[0]), rmax(xr[1])))) * fabsf(p.in_scale);
            }
            if (lane == 0) tmax[wave - NCW] = am;
            if (lw0) X6_STAMP(9, X6_NOW());
            if (cell) {
                // every loader wave read the same cell: the same scale, no agreement needed -- and the compute waves
                // need it only in the epilogue, so they take it from tmax after the chunk-0 barrier (one barrier less)
                sc = ldexpf(1.f, f16_exp(am));
            } else {
                __syncthreads();  // tile max published
                sc = ldexpf(1.f, f16_exp(fmaxf(fmaxf(tmax[0], tmax[1]), fmaxf(tmax[2], tmax[3]))));
            }
            xstore(pchunk(0), xr[0], xs);
        } else {
            xload(pchunk(0), xr[0]);
            xstore(pchunk(0), xr[0], xs);
            xload(pchunk(1), xr[1]);
        }
        if (lw0) X6_STAMP(10, X6_NOW());
        __syncthreads();
        // iteration i (chunk ch_beg + i computing): stage chunk i + 1 from ring slot 1 into the other LDS buffer
        // (released by chunk i - 1 at the last barrier), then load chunk i + 2 into the same slot -- one chunk of
        // registers in the steady state (the 2-slot ring of rounds 1-3 held two: ~96 VGPRs of loader state that
        // spilled), and the wait before each staging is on loads issued a whole chunk earlier, behind a barrier.
        // The loads are issued unconditionally (pchunk clamps past the last chunk) so that every path through the
        // loop issues the same loads and hipcc's vmcnt bookkeeping stays static; only the stores are guarded.
        for (int i = 0; i < nck; ++i) {
            if (i + 1 < nck) xstore(pchunk(i + 1), xr[1], xs + ((i + 1) & 1) * bufsz);
            xload(pchunk(i + 2), xr[1]);
            if (lw0 && i < X6_STAMP_NC) X6_STAMP(16 + 4 * i + 2, X6_NOW());
            if constexpr (!X6_NOBAR) __syncthreads();
            if (lw0 && i < X6_STAMP_NC) X6_STAMP(16 + 4 * i + 3, X6_NOW());
        }
        if (lw0) X6_STAMP(11, X6_NOW());
      };
        // the loader body, once per form (a wave-uniform choice made once per block); split-fp16 takes the fast form
        // only with the producer's |max| (amax_in): with the per-tile pre-pass instantiated in both forms the 128 x 256
        // kernel spilled 181 VGPRs (round 3)
        // (the 8-compute-wave tiles only: on the 4-wave small tiles the fast form took them from 3 to 2 waves per SIMD)
        // (X6_F16FAST=1 builds the split-fp16 fast form too: its loader registers pushed the 128 x 256 kernel's spills
        // from 34 to 93 VGPRs and its prologue, under the amax read, from 19k to 61k cycles -- end to end neutral,
        // r5f; off)
        if constexpr (LF == 1) {
            loader(std::true_type{}, std::true_type{});
        } else if constexpr (LF == 2) {
            loader(std::true_type{}, std::false_type{});
        } else if constexpr (!F16 || (NCW == 8 && X6_F16FAST)) {
            if ((!F16 || (p.amax_in && p.f16_fast)) && (Cig & 31) == 0 && p.in_scale == 1.f &&
                (p.in_act == RVC_ACT_NONE || p.in_act == RVC_ACT_LRELU)) {
                if (p.in_act == RVC_ACT_LRELU) loader(std::true_type{}, std::true_type{});
                else loader(std::true_type{}, std::false_type{});
            } else {
                loader(std::false_type{}, std::false_type{});
            }
        } else {
            loader(std::false_type{}, std::false_type{});
        }
        if (BN > 128) {  // (plan() never sets tile_epi on the 256-wide tile: not compiled there)
        } else if (p.tile_epi == 1) {  // the compute waves' tile is in LDS after this barrier
            __syncthreads();
            x6_tile_epilogue<BM, BN, 64 * (NCW + 4)>(p, reinterpret_cast<const float*>(xs), tid, split, b, m0g, n0);
        } else if (p.tile_epi == 2) {  // in two row halves (the tile is twice the X buffers' LDS)
            if constexpr (WM % 2 == 0) {
                __syncthreads();
                x6_tile_epilogue<BM / 2, BN, 64 * (NCW + 4)>(p, reinterpret_cast<const float*>(xs), tid, split, b, m0g,
                                                             n0);
                __syncthreads();
                __syncthreads();
                x6_tile_epilogue<BM / 2, BN, 64 * (NCW + 4)>(p, reinterpret_cast<const float*>(xs), tid, split, b,
                                                             m0g + BM / 2, n0);
            }
        }
        return;
    }

    // ---------------- compute waves
    const int wm = wave / WN, wn = wave % WN;
    const int s_beg = ch_beg * K, s_end = ch_end * K;
    const uint4* wxp = p.wx + (int64_t)phase * K * nch * nmf * 3 * 64;
    const int mf0 = m0g / 16 + wm * FM;
    // weight fragments of logical k-step (chunk index i, tap index tl) -- chunk-major from s_beg
    auto aload = [&](int i, int tl, uint4 (&a)[NPL][FM]) __attribute__((always_inline)) {
        // wave-uniform fragment base (scalar registers) + one per-lane offset: saddr loads, no
        // per-fragment 64-bit address registers
        const int ch = pchunk(i);
        const int t = tl + rt < K ? tl + rt : tl + rt - K;
        const int frag0 = __builtin_amdgcn_readfirstlane((t * nch + ch) * nmf + mf0);
        const uint4* src = wxp + (int64_t)frag0 * 3 * 64;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int q = 0; q < NPL; ++q) a[q][i] = src[(i * 3 + q) * 64 + lane];
    };
    floatx4 acc[FM][FN];
    floatx4 acc_lo[SA ? FM : 1][SA ? FN : 1];  // SA: the correction passes
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    if constexpr (SA) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc_lo[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    const int ln = lane & 15, lg = lane >> 4;
    const int pb = wn * 16 * FN + ln;
    // B operands are read from LDS one column fragment j at a time (NPL ds_read_b128 each), the next
    // fragment's reads issued before the current one's MFMAs: only 2 x NPL B registers stay live, which
    // leaves room for the PD-deep weight prefetch ring at 2 waves per SIMD.
    auto compute = [&](int t, const uint4* xbuf, const uint4 (&a)[NPL][FM]) __attribute__((always_inline)) {
        const int tof = tap_off(p, t);
        auto bload = [&](int j, uint4 (&bq)[NPL]) __attribute__((always_inline)) {
            const int pos = (pb + 16 * j) * p.stride + tof;
#pragma unroll
            for (int q = 0; q < NPL; ++q) bq[q] = xbuf[x_slot<NPL>(pos, q, lg)];
        };
        uint4 bb[2][NPL];
        bload(0, bb[0]);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            if (j + 1 < FN) bload(j + 1, bb[(j + 1) & 1]);
            if constexpr (X6_BPIN) __builtin_amdgcn_sched_barrier(0);
            const uint4 (&bq)[NPL] = bb[j & 1];
            if (kAblations && (p.dbg & 2)) {
#pragma unroll
                for (int i = 0; i < FM; ++i) acc[i][j][0] += __builtin_bit_cast(float, (a[0][i].x ^ bq[NPL - 1].y) & 0x3fffffu);
                continue;
            }
            // NP passes over the FM accumulators of this column fragment: hH hM mH hL mM lH
            constexpr int PA[6] = {0, 0, 1, 0, 1, 2};
            constexpr int PB[6] = {0, 1, 0, 2, 1, 0};
            if constexpr (SA) {
#pragma unroll
                for (int i = 0; i < FM; ++i) acc[i][j] = mfma_bf16(a[0][i], bq[0], acc[i][j]);
#pragma unroll
                for (int ps = 1; ps < 6; ++ps)
#pragma unroll
                    for (int i = 0; i < FM; ++i) acc_lo[i][j] = mfma_bf16(a[PA[ps]][i], bq[PB[ps]], acc_lo[i][j]);
            } else {
#pragma unroll
                for (int ps = 0; ps < NP; ++ps)
#pragma unroll
                    for (int i = 0; i < FM; ++i) {
                        if constexpr (F16) acc[i][j] = mfma_f16(a[PA[ps]][i], bq[PB[ps]], acc[i][j]);
                        else acc[i][j] = mfma_bf16(a[PA[ps]][i], bq[PB[ps]], acc[i][j]);
                    }
            }
        }
    };
    // Weight fragments are prefetched PD k-steps ahead through a ring of NB = PD + 1 register buffers
    // (the L2 latency must hide behind PD steps of MFMAs: 1 step of 6 passes, 2 of 3, 4 of 1).  The
    // sched_barrier pins each prefetch ahead of the MFMAs it must overlap (hipcc otherwise sinks the
    // independent loads below them and every k-step pays the full L2 round trip).
    // Every prefetch is issued unconditionally, past the last k-step too (pchunk clamps the chunk, the tap
    // stays in range: a valid fragment that is never used), and the k-step decode is a pair of counters
    // stepped once per k-step.  A prefetch under "if (s + PD < s_end)" made hipcc's vmcnt bookkeeping merge
    // the with- and without-load paths, and it then waited with vmcnt(0) -- on the prefetch just issued --
    // before each k-step's first MFMAs: the ring bought nothing and every k-step paid an L2 round trip.
    // The per-step divisions it replaces were ~80 scalar instructions per k-step.
    // depth: as many k-steps as fit a 24-uint4 (96-VGPR) ring, at most 4
    // (8 compute waves = 3 waves per SIMD: an 18-uint4 ring, at most 2 deep)
    // (a 256-column tile, FN = 8, keeps its 64 accumulators by giving the ring 12 uint4)
    constexpr int PD_FIT = ((FN == 8 ? 12 : (NCW == 8 ? 18 : 24)) - (SA ? FM * FN : 0)) / (NPL * FM) - 1;
    constexpr int PD_MAX = x6_min_blocks<FM, FN, NCW, NP>() == 2 ? 1 : (NCW == 8 ? 2 : 4);
    constexpr int PD_SEL = PD_FIT < 1 ? 1 : (PD_FIT > PD_MAX ? PD_MAX : PD_FIT);
    constexpr int PD = (FN == 8 && X6_PD8 > 0) ? X6_PD8 : PD_SEL;
    constexpr int NB = PD + 1;
    uint4 abuf[NB][NPL][FM];
    int li = 0, lt = 0;  // the next prefetch's logical (chunk index, tap index)
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        aload(li, lt, abuf[i]);
        if (++lt == K) { lt = 0; ++li; }
    }
    float tile_rs = 1.f;
    if (wave == 0) X6_STAMP(3, X6_NOW());
    if constexpr (F16) {
        if (!(LF || p.amax_in)) {  // the loaders' agreed pre-pass maximum (the cell case: after the chunk-0 barrier)
            __syncthreads();  // tile max published by the loaders
            tile_rs = ldexpf(1.f, -f16_exp(fmaxf(fmaxf(tmax[0], tmax[1]), fmaxf(tmax[2], tmax[3]))));
        }
        if (wave == 0) X6_STAMP(4, X6_NOW());
    }
    __syncthreads();  // chunk 0 staged
    if constexpr (F16) {
        if (LF || p.amax_in) tile_rs = ldexpf(1.f, -f16_exp(fmaxf(fmaxf(tmax[0], tmax[1]), fmaxf(tmax[2], tmax[3]))));
    }
    if (wave == 0) X6_STAMP(5, X6_NOW());
    const int nsteps = s_end - s_beg;
    int ci = 0, ct = 0;  // the computing k-step's logical (chunk index, tap index)
    for (int s0 = 0; s0 < nsteps; s0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            aload(li, lt, abuf[(u + PD) % NB]);
            if (++lt == K) { lt = 0; ++li; }
            __builtin_amdgcn_sched_barrier(0);
            if (s0 + u < nsteps) {
                const int t = ct + rt < K ? ct + rt : ct + rt - K;
                compute(t, xs + (ci & 1) * bufsz, abuf[u]);
                if (RVC_CONV_STAMPS && wave == 0 && ct == K - 1 && ci < X6_STAMP_NC) X6_STAMP(16 + 4 * ci, X6_NOW());
                if (!X6_NOBAR && ct == K - 1) __syncthreads();  // chunk done: hand the buffer back, take the next one
                if (RVC_CONV_STAMPS && wave == 0 && ct == K - 1 && ci < X6_STAMP_NC) X6_STAMP(16 + 4 * ci + 1, X6_NOW());
            }
            if (++ct == K) { ct = 0; ++ci; }
        }
    }
    if (wave == 0) X6_STAMP(6, X6_NOW());
    if constexpr (SA) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[i][j][r] += acc_lo[i][j][r];
    }
    if (kAblations && (p.dbg & 1)) {
        if (acc[0][0][0] == 1234.5f) p.y[lane] = acc[FM - 1][FN - 1][3];  // keep the loop live
        return;
    }
    if constexpr (F16) {
        // undo both scales: row m's reciprocal weight scale (stored after the image) x the tile's (exact:
        // powers of 2), before split-K partials or the epilogue see the sums
        const float* rs = reinterpret_cast<const float*>(p.wx + (int64_t)p.nphase * K * nch * nmf * 3 * 64);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float f = rs[m0g + wm * 16 * FM + i * 16 + lg * 4 + r] * tile_rs;
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j][r] *= f;
            }
    }
    if (BN <= 128 && p.tile_epi) {
        // bias, 2nd bias, activation and scale in registers (conv_epilogue's order), then the fragments into LDS: row
        // (wm * 16 FM + 16 i + 4 lg + r), column (wn * 16 FN + 16 j + ln); a row stride of BN + 4 floats puts the two
        // 16-lane halves of each ds_write_b32 on different banks
        float* ot = reinterpret_cast<float*>(xs);
        constexpr int TS = BN + 4;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            floatx4 (&av)[1][FN] = *reinterpret_cast<floatx4 (*)[1][FN]>(&acc[i][0]);
            if (p.ksplit == 1) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int mg = m0g + wm * 16 * FM + i * 16 + lg * 4 + r;
                    const int mr = mg < Cog ? mg : 0;
                    float bs = 0.f;
                    if (p.bias) bs = p.bias[mr];
                    if (p.bias2) bs += p.bias2[mr];
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
            }
        }
        // the fragments into LDS: the whole tile, or (tile_epi 2) the row half h of waves wm in [h WM / 2, (h + 1) WM / 2)
        auto put = [&](int row0) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        ot[(wm * 16 * FM - row0 + i * 16 + lg * 4 + r) * TS + wn * 16 * FN + j * 16 + ln] = acc[i][j][r];
        };
        if (p.tile_epi == 1) {
            put(0);
            __syncthreads();
            x6_tile_epilogue<BM, BN, 64 * (NCW + 4)>(p, ot, tid, split, b, m0g, n0);
        } else if constexpr (WM % 2 == 0) {
            if (wm < WM / 2) put(0);
            __syncthreads();
            x6_tile_epilogue<BM / 2, BN, 64 * (NCW + 4)>(p, ot, tid, split, b, m0g, n0);
            __syncthreads();  // half 0 read out: its LDS is free
            if (wm >= WM / 2) put(BM / 2);
            __syncthreads();
            x6_tile_epilogue<BM / 2, BN, 64 * (NCW + 4)>(p, ot, tid, split, b, m0g + BM / 2, n0);
        }
    } else if (p.swz && p.ksplit == 1) {
        conv_epilogue_swz<FM, FN, WM, WN>(p, acc, lane, wm, wn, ophase, b, grp, Cog, m0g, n0);
    } else {
        conv_epilogue<FM, FN, WM, WN>(p, acc, lane, wm, wn, split, ophase, b, grp, Cog, m0g, n0);
    }
#if RVC_CONV_STAMPS
    if (wave == 0) {
        X6_STAMP(14, X6_NOW());         // the epilogue's stores issued
        __builtin_amdgcn_s_waitcnt(0);  // ... and retired
        X6_STAMP(7, X6_NOW());
    }
#endif
}

// The split-K reduce: sums the ksplit partials in split order, then the epilogue.  (A last-arriving-block
// reduce inside the conv launch -- plain slab stores, an agent release per split block, an acquire in the
// last -- measured 11 % slower end to end, 780 vs 880 xRT on one box: each block's release writes back a
// 64 KB+ partial tile and the last arriver sums up to 16 of them alone; profiles/r3_ab_splitk_fused_rmvpe_sa.txt.)
// A block takes 256 columns x RED_ROWS rows (round 6: one row per block made a 576-row reduce 7k blocks, and with a
// |max| cell 30k atomics; now one per block, amax_publish_block).  Every load is issued ahead of the stores it could
// alias (the RED_ROWS rows' partials per split, then their residual / accumulate operands from clamped addresses): the
// per-element form waited one round trip per split and per row.  Same sums in the same split order, and the epilogue of
// epilogue_store per element.
constexpr int RED_ROWS = 8;
__global__ __launch_bounds__(256) void conv_splitk_reduce(ConvParams p) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int bp = blockIdx.z, b = bp / p.nphase;
    const int64_t m0 = (int64_t)blockIdx.y * RED_ROWS;
    const int nr = p.Co - m0 < RED_ROWS ? (int)(p.Co - m0) : RED_ROWS;
    const bool okn = n < p.ncols;
    const int t = okn ? out_pos(p, n, bp % p.nphase) : -1;
    const int64_t sstride = p.B * p.nphase * p.Co * p.ncols;
    const float* src = p.ws + ((int64_t)bp * p.Co + m0) * p.ncols + (okn ? n : 0);
    float s[RED_ROWS];
#pragma unroll
    for (int r = 0; r < RED_ROWS; ++r) s[r] = 0.f;
    for (int k = 0; k < p.ksplit; ++k) {
        float v[RED_ROWS];
#pragma unroll
        for (int r = 0; r < RED_ROWS; ++r) v[r] = src[k * sstride + (int64_t)(r < nr ? r : nr - 1) * p.ncols];
#pragma unroll
        for (int r = 0; r < RED_ROWS; ++r) s[r] += v[r];
    }
    const bool ok = t >= 0;
    const int64_t Lo = p.Lout;
    float v[RED_ROWS];
    int64_t o[RED_ROWS];
#pragma unroll
    for (int r = 0; r < RED_ROWS; ++r) {
        const int64_t m = m0 + (r < nr ? r : nr - 1);
        o[r] = m * Lo + (ok ? t : 0);
        float x = s[r];
        if (p.bias) x += p.bias[m];
        if (p.bias2) x += p.bias2[m];
        v[r] = act_apply(x, p.out_act, p.out_slope) * p.out_scale;
    }
    if (p.res) {
        float rr[RED_ROWS];
#pragma unroll
        for (int r = 0; r < RED_ROWS; ++r) rr[r] = p.res[b * p.res_bstride + o[r]];
#pragma unroll
        for (int r = 0; r < RED_ROWS; ++r) v[r] += rr[r];
    }
    float* yb = p.y + b * p.y_bstride;
    if (p.accumulate) {
        float aa[RED_ROWS];
#pragma unroll
        for (int r = 0; r < RED_ROWS; ++r) aa[r] = yb[o[r]];
#pragma unroll
        for (int r = 0; r < RED_ROWS; ++r) v[r] += aa[r];
    }
    float amx = 0.f;
#pragma unroll
    for (int r = 0; r < RED_ROWS; ++r) {
        if (r < nr) {
            if (ok) {
                yb[o[r]] = v[r];
                amx = fmaxf(amx, fabsf(v[r]));
            } else if (t <= -2) {
                yb[(m0 + r) * Lo + (-t - 2)] = 0.f;  // 2-D border cell
            }
        }
    }
    if (p.amax_out) amax_publish_block(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);
}

// The source-conv pass of a call with src_x (rvc_conv1d_args.src_*; the NSF generator's x = ups(x) + noise_convs(har),
// synthesizers.py:156): y[b][m][t] += sum_k src_w[k][m] * src[b][t * stride - pad + k] + src_b[m], the k-sum an fmaf chain
// in tap order from 0 -- the k order and roundings of that 1-input-channel conv on the f32 MFMA engine (whose
// v_mfma_f32_16x16x4_f32 is an exact fmaf chain) with accumulate, i.e. the same bits as the separate launch it replaces,
// as one HBM-bound read-modify-write of y (the engine's 1-channel conv was an implicit GEMM only K deep: 79-164 us per
// generator stage for 20-50 us of bytes).  A block takes SRC_T positions (lanes along t: coalesced y) x SRC_M channels;
// the signal span of its positions is staged in LDS once, the weights are wave-uniform (scalar loads).  Round 6 first
// fused this term into the conv epilogue: the extra live registers took the 128 x 256 tile's spills from 31 to 154 VGPRs
// in every instantiation (the epilogue is compiled into each), so it is a pass of its own.  It publishes amax_out (the
// conv itself then publishes nothing: its values are not the final ones).
struct SrcParams {
    float* y;
    const float* x;
    const float* w;  // KM [K][Co]
    const float* b;
    unsigned* amax_out;
    int64_t Co, Lout, len, xbs, ybs;
    int K, stride, pad, span;
};
constexpr int SRC_T = 256, SRC_M = 16;

__global__ __launch_bounds__(SRC_T) void src_add_kernel(SrcParams p) {
    // LDS: the block's channels' weights [K][SRC_M] (16-B aligned rows: broadcast ds_read_b128), then the signal span
    // (SRC_T - 1) * stride + K of its positions
    extern __shared__ __attribute__((aligned(16))) float smem_src[];
    float* sw = smem_src;
    float* sx = smem_src + p.K * SRC_M;
    const int b = blockIdx.z;
    const int64_t t0 = (int64_t)blockIdx.x * SRC_T;
    const int64_t q0 = t0 * p.stride - p.pad;
    const float* xb = p.x + b * p.xbs;
    const int m0 = blockIdx.y * SRC_M;
    const int nm = p.Co - m0 < SRC_M ? (int)(p.Co - m0) : SRC_M;  // block-uniform
    for (int i = threadIdx.x; i < p.K * SRC_M; i += SRC_T) {
        const int k = i / SRC_M, mi = i - k * SRC_M;
        sw[i] = mi < nm ? p.w[(int64_t)k * p.Co + m0 + mi] : 0.f;
    }
    for (int i = threadIdx.x; i < p.span; i += SRC_T) {
        const int64_t q = q0 + i;
        sx[i] = (q >= 0 && q < p.len) ? xb[q] : 0.f;
    }
    __syncthreads();
    const int64_t t = t0 + threadIdx.x;
    const bool ok = t < p.Lout;
    const float* xw = sx + threadIdx.x * p.stride;
    float* yb = p.y + b * p.ybs + (ok ? t : 0);
    // taps outer (one signal read per tap, shared by the block's channels; the 16 weights one broadcast), one fmaf chain
    // per channel in tap order
    float acc[SRC_M];
#pragma unroll
    for (int mi = 0; mi < SRC_M; ++mi) acc[mi] = 0.f;
    for (int k = 0; k < p.K; ++k) {
        const float xv = xw[k];
        const float4* wk = reinterpret_cast<const float4*>(sw + k * SRC_M);
#pragma unroll
        for (int q = 0; q < SRC_M / 4; ++q) {
            const float4 w4 = wk[q];
            acc[4 * q] = fmaf(w4.x, xv, acc[4 * q]);
            acc[4 * q + 1] = fmaf(w4.y, xv, acc[4 * q + 1]);
            acc[4 * q + 2] = fmaf(w4.z, xv, acc[4 * q + 2]);
            acc[4 * q + 3] = fmaf(w4.w, xv, acc[4 * q + 3]);
        }
    }
    // every y load first, then the stores: interleaved, hipcc kept each load behind the previous channel's store (it
    // cannot prove the rows apart) -- 16 dependent round trips per thread
    float yo[SRC_M];
#pragma unroll
    for (int mi = 0; mi < SRC_M; ++mi) yo[mi] = yb[(int64_t)(m0 + (mi < nm ? mi : 0)) * p.Lout];
    float amx = 0.f;
#pragma unroll
    for (int mi = 0; mi < SRC_M; ++mi) {
        if (mi < nm) {
            const int m = m0 + mi;
            const float v = (acc[mi] + (p.b ? p.b[m] : 0.f)) + yo[mi];
            if (ok) {
                yb[(int64_t)m * p.Lout] = v;
                amx = fmaxf(amx, fabsf(v));
            }
        }
    }
    if (p.amax_out) amax_publish_block(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);
}

struct Cfg {
    int FM, FN, WM, WN;
    bool x6;
};

template <int FM, int FN, int WM, int WN>
hipError_t launch(const ConvParams& p, dim3 grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((conv1d_mfma_kernel<FM, FN, WM, WN>), grid, dim3(256), lds, s, p);
    return hipGetLastError();
}

template <int FM, int FN, int WM, int WN, int NP, bool F16 = false, bool SA = false, int LF = 0>
void launch_x6_np(const ConvParams& p, dim3 grid, size_t lds, hipStream_t s) {
    // loader items per thread sized to the staged span (unused items would still issue loads)
    const dim3 blk(64 * (WM * WN + 4));
    if (4 * p.span <= 256 * 3)
        hipLaunchKernelGGL((conv_x6_kernel<FM, FN, WM, WN, 3, NP, F16, SA, LF>), grid, blk, lds, s, p);
    else hipLaunchKernelGGL((conv_x6_kernel<FM, FN, WM, WN, 6, NP, F16, SA, LF>), grid, blk, lds, s, p);
}

// the fast-only split-fp16 loaders apply (conv_x6_kernel's LF): 1 = leaky ReLU input, 2 = none, 0 = no
int x6_f16_fast_form(const ConvParams& p) {
    if (!p.amax_in || !p.f16_fast || (p.Ci & 31) != 0 || p.in_scale != 1.f) return 0;
    return p.in_act == RVC_ACT_LRELU ? 1 : (p.in_act == RVC_ACT_NONE ? 2 : 0);
}

// The tiles compiled with split accumulators (RVC_ARITH_FP32_SA): <= 64 rows on 4 / 8 waves and 128 x 128 on 8
// -- the ones plan() gives RMVPE's convs under the default engine switches.  A request on any other tile (e.g.
// RVC_X6_W8=0) is refused by plan() rather than run without the split accumulators.
constexpr bool x6_sa_tile(int FM, int FN, int WM, int WN) {
    return (WM * WN == 8 && FN == 4) || (WM * WN == 4 && FM <= 2 && FN == 2) || (WM == 2 && WN == 4);
}

template <int FM, int FN, int WM, int WN>
hipError_t launch_x6(const ConvParams& p, dim3 grid, size_t lds, hipStream_t s) {
    if (p.wx_passes == RVC_ARITH_F16X3) {
        const int lf = WM * WN == 8 ? x6_f16_fast_form(p) : 0;
        if constexpr (WM * WN == 8) {
            if (lf == 1) launch_x6_np<FM, FN, WM, WN, 3, true, false, 1>(p, grid, lds, s);
            else if (lf == 2) launch_x6_np<FM, FN, WM, WN, 3, true, false, 2>(p, grid, lds, s);
        }
        if (lf == 0) launch_x6_np<FM, FN, WM, WN, 3, true>(p, grid, lds, s);
    }
    else if (p.wx_passes == 1) launch_x6_np<FM, FN, WM, WN, 1>(p, grid, lds, s);
    else if (p.wx_passes == 3) launch_x6_np<FM, FN, WM, WN, 3>(p, grid, lds, s);
    else if (p.wx_passes == RVC_ARITH_FP32_SA) {
        // split accumulators: only the tiles RMVPE's convs take (x6_sa_tile; plan() refuses any other)
        if constexpr (x6_sa_tile(FM, FN, WM, WN)) launch_x6_np<FM, FN, WM, WN, 6, false, true>(p, grid, lds, s);
    }
    else launch_x6_np<FM, FN, WM, WN, 6>(p, grid, lds, s);
    return hipGetLastError();
}

#if RVC_CONV_STAMPS
unsigned long long* g_stamps = nullptr;
int64_t g_stamp_blocks = 0;
#endif

void fill_common(const rvc_conv1d_args* a, ConvParams& p) {
    p.x = a->x; p.w = a->w; p.bias = a->bias; p.bias2 = a->bias2; p.res = a->res; p.y = a->y; p.ws = nullptr;
    p.B = a->B; p.Ci = a->Ci; p.Co = a->Co; p.Lin = a->Lin; p.Lout = a->Lout;
    p.ncols = a->ncols > 0 ? a->ncols : a->Lout;
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
    p.wx = nullptr;
    p.wx_nmf = p.wx_nch = 0;
    p.wx_passes = a->wx_passes == 0 ? 6 : a->wx_passes;
    static const int dbg = getenv("RVC_CONV_DEBUG") ? atoi(getenv("RVC_CONV_DEBUG")) : 0;
    p.dbg = dbg;
    p.tile_epi = 0;
    p.amax_in = a->amax_in;
    p.amax_out = a->amax_out;
    static const int f16fast = getenv("RVC_X6_F16FAST") ? atoi(getenv("RVC_X6_F16FAST")) : 1;
    p.f16_fast = g_f16_fast >= 0 ? g_f16_fast : f16fast;
    p.stagger = 0;
    p.stagger_blocks = 0;
    static const int swz_env = getenv("RVC_X6_SWZ") ? atoi(getenv("RVC_X6_SWZ")) : 1;
    p.swz = g_swz >= 0 ? g_swz : swz_env;
    p.gx6 = 0;
#if RVC_CONV_STAMPS
    p.stamps = g_stamps;
    p.stamp_blocks = g_stamp_blocks;
#endif
    // k-step rotation (RVC_X6_ROT=1): +3 % on the conv suite, but it changes every output's
    // summation order, which moved one RMVPE voicing decision in the 45 s pipeline test past the 1e-4
    // waveform bar -- off, so the engine keeps the summation order the parity suite validated
    static const int rot = getenv("RVC_X6_ROT") ? atoi(getenv("RVC_X6_ROT")) : 0;
    p.rot = rot;
    static const int xcd = getenv("RVC_X6_XCD") ? atoi(getenv("RVC_X6_XCD")) : 1;
    p.xcd = xcd;
}

// compute units of the current device (read once per process: one device type per process)
int num_cus() {
    static const int n = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return cus;
    }();
    return n;
}

// split-K policy shared by both engines: split the chunk range when the tile grid underfills the chip
// per-thread override of the split-K target grid (rvc_conv1d_set_splitk_target; -1 = the process default)
static thread_local int g_splitk_target = -1;
// per-thread override of the x6 tile epilogue (rvc_conv1d_set_tile_epi; -1 = RVC_X6_TILE_EPI, default off)
static thread_local int g_tile_epi = -1;

void split_k(ConvParams& p, int64_t tiles, int nch, int per_cu = 2) {
    // target grid (RVC_SPLITK_TILES, 0 = never split): 256 tiles = 1 per CU (round 4, same box, alternated runs:
    // per call 720-723 xRT at 512 -> 731-732 at 256, clip stream 906-908 -> 907-912).  A kernel of which only one block fits
    // a CU (the 8-compute-wave x6 tiles: 768 threads) targets 256: past one round of blocks a split only adds
    // rounds (ContentVec's K = 1 GEMMs, 30 s: 2304 x 768 x 1599 76 -> 49 us unsplit, 3072 x 768 95 -> 89;
    // RVC_X6_SPLIT_OCC=0 restores 512 for every tile)
    static const int env_target = getenv("RVC_SPLITK_TILES") ? atoi(getenv("RVC_SPLITK_TILES")) : 256;
    static const int occ_aware = getenv("RVC_X6_SPLIT_OCC") ? atoi(getenv("RVC_X6_SPLIT_OCC")) : 1;
    int target = g_splitk_target >= 0 ? g_splitk_target : env_target;
    if (occ_aware && per_cu == 1 && g_splitk_target < 0) target /= 2;
    int ks = 1;
    if (tiles < target && nch >= 4) {
        ks = (int)((target + tiles - 1) / tiles);
        if (ks > 16) ks = 16;
        if (ks > nch / 2) ks = nch / 2;
        if (ks < 1) ks = 1;
    }
    p.chunks_per_split = (nch + ks - 1) / ks;
    p.ksplit = (nch + p.chunks_per_split - 1) / p.chunks_per_split;
}

constexpr int X6_BN = 128;

int max_tap_off(const rvc_conv1d_args* a) {
    if (!a->ntoff) return (a->K - 1) * a->dil;
    int m = 0;
    for (int i = 0; i < a->ntoff && i < 16; ++i) m = a->toff[i] > m ? a->toff[i] : m;
    return m;
}

// Taps per conv on the split-bf16 engine: CREPE's k=64 layers (CREPE.py:11-69) are the widest; the staged
// span (BN - 1) * stride + (K - 1) * dil + 1 is checked against the loader's item budget below.
constexpr int X6_K_MAX = 64;
// grouped convs (ContentVec's pos_conv: 16 groups of 48 channels, k = 128) run one group per phase (ConvParams.gx6): stride
// 1, plain stores, the image packed with the groups as phases (ops.Conv, make_images), no split-K, up to 128 taps
constexpr int X6_K_MAX_GROUPED = 128;

// stride 2 only with >= 32 input channels (ContentVec's feature extractor): the staged span doubles,
// and the operand reads of even positions are 2-way bank conflicted
bool x6_eligible(const rvc_conv1d_args* a) {
    static const int s2 = getenv("RVC_X6_STRIDE2") ? atoi(getenv("RVC_X6_STRIDE2")) : 1;
    // RVC_X6_K1=0: the K = 1 GEMMs (ContentVec / TextEncoder linears) on the f32 MFMA engine instead (A/B switch)
    static const int k1 = getenv("RVC_X6_K1") ? atoi(getenv("RVC_X6_K1")) : 1;
    if (a->K == 1 && !k1) return false;
    static const int grouped = getenv("RVC_X6_GROUPED") ? atoi(getenv("RVC_X6_GROUPED")) : 1;
    const bool grp_ok = a->groups == 1 ||
                        (grouped && a->stride == 1 && a->nphase == 1 && a->ostride == 1 && a->ooffset == 0 &&
                         !a->ntoff && !a->wrap && !a->src_x && a->Ci % a->groups == 0 && a->Co % a->groups == 0);
    return a->wx && a->Lin < (1 << 24) &&
           (a->stride == 1 || (s2 && a->stride == 2 && a->Ci >= 32 && !a->ntoff)) && grp_ok &&
           a->w_bstride == 0 && (!a->ntoff || a->ntoff == a->K) &&
           a->K <= (a->groups == 1 ? X6_K_MAX : X6_K_MAX_GROUPED) &&
           (X6_BN - 1) * a->stride + max_tap_off(a) + 1 <= 64 * X6_NI_MAX - 2 && a->wx_nmf % 8 == 0 &&
           (int64_t)a->wx_nmf * 16 >= a->Co / a->groups && (a->wx_passes == 0 || a->wx_passes == 6 ||
                                                a->wx_passes == RVC_ARITH_FP32_SA || a->wx_passes == 3 ||
                                                a->wx_passes == 1 || a->wx_passes == RVC_ARITH_F16X3);
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
    fill_common(a, p);
    RVC_CHECK_ARG(!a->src_x || (a->src_w && a->src_K > 0 && a->src_K <= 4096 && a->src_stride > 0 && a->src_pad >= 0 &&
                                a->src_len > 0 && a->src_bstride >= 0 && !a->wrap),
                  "conv1d: bad fused source conv (src_K=%d src_stride=%d src_pad=%d src_len=%lld)", a->src_K,
                  a->src_stride, a->src_pad, (long long)a->src_len);
    RVC_CHECK_ARG(!a->src_x || ((int64_t)255 * a->src_stride + 17 * a->src_K) * 4 <= 64 * 1024,
                  "conv1d: source conv span too large (stride %d, K %d)", a->src_stride, a->src_K);
    if (a->ntoff) {
        RVC_CHECK_ARG(a->ntoff == a->K && a->K <= 16, "conv1d: toff needs ntoff == K <= 16");
        for (int i = 0; i < a->K; ++i) RVC_CHECK_ARG(a->toff[i] >= 0, "conv1d: negative tap offset");
    }

    if (x6_eligible(a)) {
        cfg.x6 = true;
        // 8 compute waves (2 per SIMD beside 1 loader wave: one's MFMAs cover the other's waits) beat
        // 4 waves of twice the tile on every 128/256-channel shape, and on 64 channels at >= 3 passes
        static const int w8 = getenv("RVC_X6_W8") ? atoi(getenv("RVC_X6_W8")) : 1;
        const int np = a->wx_passes == 0 || a->wx_passes == RVC_ARITH_FP32_SA ? 6 : a->wx_passes;
        // 128 x 256 on 8 compute waves for the split-fp16 convs (RVC_X6_BN256: 1 = split-fp16 only, the
        // default; 2 = every pass set; 0 = off): half the blocks, so half the per-block prologue / epilogue
        // (~15-25 us each), and each weight fragment feeds twice the MFMAs; stride-1, short tap spans.
        // Measured (conv_bench, same box): split-fp16 C=128 K=11 762 -> 672 us, K=7 590 -> 534, C=256 K=11
        // 331 -> 307; end to end 820 -> 850 xRT.  The 6-pass form loses (its weight ring drops to 1 k-step
        // to fit 64 accumulators: C=128 K=11 883 -> 1113 us).
        static const int bn256 = getenv("RVC_X6_BN256") ? atoi(getenv("RVC_X6_BN256")) : 1;
        // ... unless the 256-wide grid quantises worse onto the chip's one block per CU: C=256 at 30 s (2 x 150
        // tiles, 1.17 rounds) runs 128-wide (2 x 300, 2.34 rounds): K=11 245-252 -> 226 us (conv_bench, round 4)
        auto round_eff = [](int64_t t) {
            const int64_t n = num_cus();
            return (double)t / (double)(((t + n - 1) / n) * n);
        };
        const int64_t rows128 = (Cog + 127) / 128, nb = a->B * a->nphase;
        const bool fills256 = round_eff(rows128 * ((ncols + 255) / 256) * nb) >=
                              round_eff(rows128 * ((ncols + 127) / 128) * nb) - 0.05;
        if (Cog > 64 && w8 && bn256 && a->stride == 1 && 255 + max_tap_off(a) + 1 <= 64 * X6_NI_MAX - 2 &&
            (bn256 == 2 || np == RVC_ARITH_F16X3) && (fills256 || bn256 == 3))
            cfg = {2, 8, 4, 2, true};
        else if (Cog > 64 && w8) cfg = {2, 4, 4, 2, true};  // 128 x 128 on 8 compute waves
        else if (Cog > 64) cfg = {4, 4, 2, 2, true};   // 128 x 128 on 4 compute waves
        else if (Cog > 32 && w8 && np >= 3) cfg = {2, 2, 2, 4, true};  // 64 x 128 on 8 compute waves
        else if (Cog > 32) cfg = {2, 4, 2, 2, true};   // 64 x 128
        else if (Cog > 16) cfg = {2, 2, 1, 4, true};   // 32 x 128
        else cfg = {1, 2, 1, 4, true};                 // 16 x 128
        RVC_CHECK_ARG(a->wx_passes != RVC_ARITH_FP32_SA || x6_sa_tile(cfg.FM, cfg.FN, cfg.WM, cfg.WN),
                      "conv1d: RVC_ARITH_FP32_SA has no split-accumulator kernel for the %dx%d tile on %d waves "
                      "(engine switches changed?)", 16 * cfg.FM * cfg.WM, 16 * cfg.FN * cfg.WN, cfg.WM * cfg.WN);
        const int BM = 16 * cfg.FM * cfg.WM, BN = 16 * cfg.FN * cfg.WN;
        p.span = (BN - 1) * a->stride + max_tap_off(a) + 1;
        p.span_s = p.span;
        p.rows_max = 0;
        p.inv_span = 1.0f / (float)p.span;
        p.avec = 0;
        p.wx = (const uint4*)a->wx;
        p.wx_nmf = a->wx_nmf;
        p.wx_nch = (int)((Cig + 31) / 32);
        p.mtiles_per_group = (int)((Cog + BM - 1) / BM);
        const int64_t tiles = (int64_t)p.mtiles_per_group * ((ncols + BN - 1) / BN) * a->B * a->nphase * a->groups;
        split_k(p, tiles, p.wx_nch, cfg.WM * cfg.WN == 8 ? 1 : 2);
        if (a->groups > 1) {  // groups as phases (gx6), each over its own Cig input / Cog output rows; never split-K
            p.gx6 = 1;
            p.nphase = a->groups;
            p.Ci = Cig;
            p.Co = Cog;
            p.chunks_per_split = p.wx_nch;
            p.ksplit = 1;
        }
        lds = (size_t)2 * (p.wx_passes == 6 || p.wx_passes == RVC_ARITH_FP32_SA ? 3 : (p.wx_passes == 1 ? 1 : 2)) *
              p.span * 64 + 16;  // + the split-fp16 tile |max|
        // the tile epilogue (x6_tile_epilogue) for plain stores: one phase, output column = GEMM column, no 2-D border;
        // its [BM][BN + 4] f32 tile reuses the X buffers' LDS (RVC_X6_TILE_EPI=0: the in-register epilogue, A/B switch)
        // Only where it needs no more LDS than the X buffers (whole, or in two row halves): a launch with a larger
        // LDS footprint leaves no room on its CUs for the concurrent front-end streams' blocks (round 5, the 128 x 256
        // tile with a 133 KB tile: its epilogue no faster -- every CU's blocks reach it at once and it is HBM-bound --
        // and the clip stream 928 -> 889 xRT); and not on the 256-wide tile, whose epilogue measured 29k -> 33k cycles.
        // Off by default: even LDS-neutral it measured slower end to end (893-899 vs 899-905 xRT, interleaved on one
        // box, r5c) -- kept as the RVC_X6_TILE_EPI=1 / rvc_conv1d_set_tile_epi(1) option, tested bit-identical.
        static const int tepi_env = getenv("RVC_X6_TILE_EPI") ? atoi(getenv("RVC_X6_TILE_EPI")) : 0;
        const int tepi = g_tile_epi >= 0 ? g_tile_epi : tepi_env;
        const size_t tile_bytes = (size_t)BM * (BN + 4) * 4;
        const bool plain = a->nphase == 1 && a->ostride == 1 && a->ooffset == 0 && !a->wrap && !(p.dbg & 1) &&
                           BN <= 128;
        p.tile_epi = !(tepi && plain && a->groups == 1) ? 0
                     : tile_bytes <= lds ? 1 : (cfg.WM % 2 == 0 && tile_bytes / 2 <= lds) ? 2 : 0;
        grid = dim3(cdiv(ncols, BN), (unsigned)p.mtiles_per_group, (unsigned)(a->B * p.nphase * p.ksplit));
        RVC_CHECK_ARG(grid.y < 65536 && grid.z < 65536, "conv1d: grid too large");
        // staggered start (RVC_X6_STAGGER shader cycles) when the launch runs more than one round of blocks per CU
        static const int stagger = getenv("RVC_X6_STAGGER") ? atoi(getenv("RVC_X6_STAGGER")) : 0;
        static const int stagger_rounds = getenv("RVC_X6_STAGGER_ROUNDS") ? atoi(getenv("RVC_X6_STAGGER_ROUNDS")) : 2;
        const int64_t nblk = (int64_t)grid.x * grid.y * grid.z;
        if (stagger > 0 && nblk >= stagger_rounds * (int64_t)num_cus()) {
            p.stagger = stagger;
            p.stagger_blocks = num_cus();
        }
        return RVC_OK;
    }

    if (Cog % 48 == 0 && Cog % 64 != 0) cfg = {3, 1, 1, 4, false};  // 48 x 64 (ContentVec pos_conv groups)
    else if (Cog <= 16) cfg = {1, 4, 1, 4, false};                  // 16 x 256
    else if (Cog <= 32) cfg = {2, 4, 1, 4, false};                  // 32 x 256
    else if (Cog <= 64 || Cog % 128 != 0) cfg = {2, 4, 2, 2, false}; // 64 x 128 (also 192: no half-empty M tile)
    else cfg = {4, 4, 2, 2, false};                                 // 128 x 128
    int BM = 16 * cfg.FM * cfg.WM, BN = 16 * cfg.FN * cfg.WN;

    const int maxoff = max_tap_off(a);
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
    p.span = span;
    p.span_s = span + 1;
    p.rows_max = rows_max;
    p.inv_span = 1.0f / (float)span;
    p.avec = (Cog % 4 == 0) && (((uintptr_t)a->w & 15) == 0) && (a->w_bstride % 4 == 0);
    p.mtiles_per_group = (int)((Cog + BM - 1) / BM);
    const int64_t tiles = (int64_t)p.mtiles_per_group * a->groups * ((ncols + BN - 1) / BN) * a->B * a->nphase;
    split_k(p, tiles, (int)((Cig * a->K + KCH - 1) / KCH));
    const int WS = (BM / 32) * 32 + 16 + ((BM % 32) ? 32 : 0);
    lds = (size_t)(KCH * WS + KCH) * 4 + ((size_t)rows_max * p.span_s + 4) * 4;  // +dump slot
    RVC_CHECK_ARG(lds <= 160 * 1024, "conv1d: LDS %zu too large", lds);
    grid = dim3(cdiv(ncols, BN), (unsigned)(p.mtiles_per_group * a->groups), (unsigned)(a->B * a->nphase * p.ksplit));
    RVC_CHECK_ARG(grid.y < 65536 && grid.z < 65536, "conv1d: grid too large");
    return RVC_OK;
}

// KM weights [nphase][Ci*K][Co] -> per-lane split-bf16 fragments [nphase][K][nch][nmf][3][64] x 16 B:
// lane l of (t, chunk, fragment mf, plane q) holds plane q of W[c = 32 chunk + 8 (l>>4) + e][m = 16 mf + (l&15)], e < 8.
__global__ __launch_bounds__(256) void pack_x6_kernel(const float* w, int64_t total, int Ci, int K, int Co, int nch,
                                                      int nmf, uint4* out) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    int64_t r = idx;
    const int lane = (int)(r % 64); r /= 64;
    const int q = (int)(r % 3); r /= 3;
    const int mf = (int)(r % nmf); r /= nmf;
    const int ch = (int)(r % nch); r /= nch;
    const int t = (int)(r % K); r /= K;
    const int64_t ph = r;
    const int m = mf * 16 + (lane & 15);
    uint32_t wd[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
        uint32_t hv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = ch * 32 + 8 * (lane >> 4) + 2 * e2 + u;
            const float v = (c < Ci && m < Co) ? w[((ph * Ci + c) * K + t) * Co + m] : 0.f;
            uint32_t h, mm, l;
            split3(v, h, mm, l);
            hv[u] = q == 0 ? h : (q == 1 ? mm : l);
        }
        wd[e2] = hv[0] | (hv[1] << 16);
    }
    out[idx] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
}

int64_t x6_nmf(int64_t Co) { return (Co + 127) / 128 * 8; }

// Split-fp16 image: per output row m, the power-of-2 scale 2^E_m that maps max |w[.][m]| (over every
// phase, input channel and tap) below 2^14; rs[m] = 2^-E_m.  Load time only: blocks of 64 columns x 4 row
// phases walk one row slice each and merge their |max| with an integer atomic max on the float bits
// (non-negative floats order as their bit patterns) into rs, zeroed before; rowscale_fin turns it into 2^-E.
__global__ __launch_bounds__(256) void rowscale_f16_kernel(const float* w, int64_t nrow, int Co, unsigned* amax) {
    const int m = blockIdx.x * 64 + (threadIdx.x & 63);
    const int64_t r0 = (int64_t)blockIdx.y * nrow / gridDim.y, r1 = (int64_t)(blockIdx.y + 1) * nrow / gridDim.y;
    float am = 0.f;
    if (m < Co)
        for (int64_t i = r0 + (threadIdx.x >> 6); i < r1; i += 4) am = fmaxf(am, fabsf(w[i * Co + m]));
    __shared__ float red[256];
    red[threadIdx.x] = am;
    __syncthreads();
    if (threadIdx.x < 64 && m < Co) {
        am = fmaxf(fmaxf(red[threadIdx.x], red[threadIdx.x + 64]), fmaxf(red[threadIdx.x + 128], red[threadIdx.x + 192]));
        atomicMax(amax + m, __float_as_uint(am));
    }
}

__global__ __launch_bounds__(256) void rowscale_fin_kernel(float* rs, int npad) {
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m < npad) rs[m] = ldexpf(1.f, -f16_exp(__uint_as_float(reinterpret_cast<const unsigned*>(rs)[m])));
}

// KM weights -> the x6 fragment layout [nphase][K][nch][nmf][3][64] x 16 B with plane 0 = fp16 h and
// plane 1 = fp16 l of w[.][m] / rs[m] (plane 2 zero: same strides as the bf16 image)
__global__ __launch_bounds__(256) void pack_f16_kernel(const float* w, int64_t total, int Ci, int K, int Co, int nch,
                                                       int nmf, const float* rs, uint4* out) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    int64_t r = idx;
    const int lane = (int)(r % 64); r /= 64;
    const int q = (int)(r % 3); r /= 3;
    const int mf = (int)(r % nmf); r /= nmf;
    const int ch = (int)(r % nch); r /= nch;
    const int t = (int)(r % K); r /= K;
    const int64_t ph = r;
    const int m = mf * 16 + (lane & 15);
    uint32_t wd[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
        uint32_t hv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = ch * 32 + 8 * (lane >> 4) + 2 * e2 + u;
            const float v = (c < Ci && m < Co) ? w[((ph * Ci + c) * K + t) * Co + m] / rs[m] : 0.f;
            uint32_t h, l;
            split2h(v, h, l);
            hv[u] = q == 0 ? h : (q == 1 ? l : 0u);
        }
        wd[e2] = hv[0] | (hv[1] << 16);
    }
    out[idx] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
}

}  // namespace

extern "C" int64_t rvc_conv1d_x6_bytes(int64_t nphase, int64_t Ci, int K, int64_t Co) {
    if (nphase <= 0 || Ci <= 0 || K <= 0 || Co <= 0) return -1;
    return nphase * K * ((Ci + 31) / 32) * x6_nmf(Co) * 3 * 64 * 16;
}

extern "C" int rvc_conv1d_pack_x6(const float* w_km, int64_t nphase, int64_t Ci, int K, int64_t Co, void* out,
                                  int* nmf_out, rvc_stream_t stream) {
    RVC_CHECK_ARG(w_km && out && nmf_out && nphase > 0 && Ci > 0 && K > 0 && Co > 0, "pack_x6: bad args");
    const int nch = (int)((Ci + 31) / 32), nmf = (int)x6_nmf(Co);
    const int64_t total = nphase * K * nch * nmf * 3 * 64;
    hipLaunchKernelGGL(pack_x6_kernel, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, w_km, total,
                       (int)Ci, K, (int)Co, nch, nmf, (uint4*)out);
    RVC_HIP(hipGetLastError());
    *nmf_out = nmf;
    return RVC_OK;
}

extern "C" int64_t rvc_conv1d_f16_bytes(int64_t nphase, int64_t Ci, int K, int64_t Co) {
    if (nphase <= 0 || Ci <= 0 || K <= 0 || Co <= 0) return -1;
    return nphase * K * ((Ci + 31) / 32) * x6_nmf(Co) * 3 * 64 * 16 + x6_nmf(Co) * 16 * 4;
}

extern "C" int rvc_conv1d_pack_f16(const float* w_km, int64_t nphase, int64_t Ci, int K, int64_t Co, void* out,
                                   int* nmf_out, rvc_stream_t stream) {
    RVC_CHECK_ARG(w_km && out && nmf_out && nphase > 0 && Ci > 0 && K > 0 && Co > 0, "pack_f16: bad args");
    const int nch = (int)((Ci + 31) / 32), nmf = (int)x6_nmf(Co);
    const int64_t total = nphase * K * nch * nmf * 3 * 64;
    float* rs = reinterpret_cast<float*>(reinterpret_cast<uint4*>(out) + total);
    hipStream_t s = (hipStream_t)stream;
    const int64_t nrow = nphase * Ci * K;
    RVC_HIP(hipMemsetAsync(rs, 0, (size_t)nmf * 16 * 4, s));
    hipLaunchKernelGGL(rowscale_f16_kernel, dim3(cdiv(Co, 64), (unsigned)std::min<int64_t>(64, cdiv(nrow, 64))),
                       dim3(256), 0, s, w_km, nrow, (int)Co, reinterpret_cast<unsigned*>(rs));
    hipLaunchKernelGGL(rowscale_fin_kernel, dim3(cdiv(nmf * 16, 256)), dim3(256), 0, s, rs, nmf * 16);
    hipLaunchKernelGGL(pack_f16_kernel, dim3(cdiv(total, 256)), dim3(256), 0, s, w_km, total, (int)Ci, K, (int)Co, nch,
                       nmf, (const float*)rs, (uint4*)out);
    RVC_HIP(hipGetLastError());
    *nmf_out = nmf;
    return RVC_OK;
}

extern "C" int rvc_conv1d_engine(const rvc_conv1d_args* a) {
    ConvParams p;
    Cfg cfg;
    dim3 grid;
    size_t lds;
    if (plan(a, p, cfg, grid, lds) != RVC_OK) return -1;
    return cfg.x6 ? 1 : 0;
}

extern "C" int64_t rvc_conv1d_workspace_bytes(const rvc_conv1d_args* a) {
    ConvParams p;
    Cfg cfg;
    dim3 grid;
    size_t lds;
    if (plan(a, p, cfg, grid, lds) != RVC_OK) return -1;
    if (p.ksplit <= 1) return 0;
    return (int64_t)p.ksplit * p.B * p.nphase * p.Co * p.ncols * 4;
}

extern "C" int rvc_conv1d_set_splitk_target(int target) {
    const int prev = g_splitk_target;
    g_splitk_target = target < 0 ? -1 : target;
    return prev;
}

static thread_local hipEvent_t g_probe_event = nullptr;

extern "C" void rvc_conv1d_set_probe_event(void* hip_event) { g_probe_event = (hipEvent_t)hip_event; }

extern "C" int rvc_conv1d_set_f16_fast(int on) {
    g_f16_fast = on < 0 ? -1 : (on ? 1 : 0);
    return RVC_OK;
}

extern "C" int rvc_conv1d_set_swz(int on) {
    g_swz = on < 0 ? -1 : (on ? 1 : 0);
    return RVC_OK;
}

extern "C" int rvc_conv1d_set_tile_epi(int on) {
    g_tile_epi = on < 0 ? -1 : (on ? 1 : 0);
    return RVC_OK;
}

// Diagnostic build only (-DRVC_CONV_STAMPS=1): the x6 engine's per-block phase stamps go to buf
// ([blocks][256] u64, blocks = bytes / 2048); returns -1 in a production build (no stamps compiled).
extern "C" int rvc_conv1d_set_stamps(void* buf, int64_t bytes) {
#if RVC_CONV_STAMPS
    g_stamps = (unsigned long long*)buf;
    g_stamp_blocks = buf ? bytes / (8 * X6_STAMP_W) : 0;
    return 0;
#else
    (void)buf;
    (void)bytes;
    return -1;
#endif
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
    if (a->src_x) p.amax_out = nullptr;  // the source pass publishes the final values' |max|
    hipError_t e;
    if (cfg.x6) {
        if (cfg.WM == 4 && cfg.FN == 8) e = launch_x6<2, 8, 4, 2>(p, grid, lds, s);
        else if (cfg.WM == 4) e = launch_x6<2, 4, 4, 2>(p, grid, lds, s);
        else if (cfg.WM == 2 && cfg.WN == 4) e = launch_x6<2, 2, 2, 4>(p, grid, lds, s);
        else if (cfg.FM == 4) e = launch_x6<4, 4, 2, 2>(p, grid, lds, s);
        else if (cfg.WM == 2) e = launch_x6<2, 4, 2, 2>(p, grid, lds, s);
        else if (cfg.FM == 2) e = launch_x6<2, 2, 1, 4>(p, grid, lds, s);
        else e = launch_x6<1, 2, 1, 4>(p, grid, lds, s);
    } else if (cfg.FM == 3) e = launch<3, 1, 1, 4>(p, grid, lds, s);
    else if (cfg.FM == 1 && cfg.FN == 4) e = launch<1, 4, 1, 4>(p, grid, lds, s);
    else if (cfg.FM == 1) e = launch<1, 2, 1, 4>(p, grid, lds, s);
    else if (cfg.WM == 1 && cfg.FN == 4) e = launch<2, 4, 1, 4>(p, grid, lds, s);
    else if (cfg.WM == 1) e = launch<2, 2, 1, 4>(p, grid, lds, s);
    else if (cfg.FM == 4 && cfg.FN == 4) e = launch<4, 4, 2, 2>(p, grid, lds, s);
    else if (cfg.FM == 4) e = launch<4, 2, 2, 2>(p, grid, lds, s);
    else if (cfg.FN == 4) e = launch<2, 4, 2, 2>(p, grid, lds, s);
    else e = launch<2, 2, 2, 2>(p, grid, lds, s);
    RVC_HIP(e);
    if (g_probe_event) RVC_HIP(hipEventRecord(g_probe_event, s));
    if (p.ksplit > 1) {
        hipLaunchKernelGGL(conv_splitk_reduce,
                           dim3(cdiv(p.ncols, 256), (unsigned)cdiv(p.Co, RED_ROWS), (unsigned)(p.B * p.nphase)),
                           dim3(256), 0, s, p);
        RVC_HIP(hipGetLastError());
    }
    if (a->src_x) {
        SrcParams q;
        q.y = a->y;
        q.x = a->src_x;
        q.w = a->src_w;
        q.b = a->src_b;
        q.amax_out = a->amax_out;
        q.Co = a->Co;
        q.Lout = a->Lout;
        q.len = a->src_len;
        q.xbs = a->src_bstride ? a->src_bstride : a->src_len;
        q.ybs = p.y_bstride;
        q.K = a->src_K;
        q.stride = a->src_stride;
        q.pad = a->src_pad;
        q.span = (SRC_T - 1) * a->src_stride + a->src_K;
        hipLaunchKernelGGL(src_add_kernel, dim3(cdiv(a->Lout, SRC_T), cdiv(a->Co, SRC_M), (unsigned)a->B), dim3(SRC_T),
                           (size_t)(q.span + q.K * SRC_M) * 4, s, q);
        RVC_HIP(hipGetLastError());
    }
    return RVC_OK;
}
