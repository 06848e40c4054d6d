// RMVPE in f64 (main/library/predictors/RMVPE.py): the f0 is a per-frame decision -- argmax over 360 salience
// bins and a 0.03 voicing threshold (RMVPE.py:217-252) -- and on real inputs a few frames per clip have their
// top two bins closer than any f32 evaluation of the network resolves (3.2e-6 apart on the headline clip, while
// f32 evaluations -- the reference's own at other thread counts among them -- err by up to 1.7e-4).  So the
// whole network runs in f64 here: mel (f64 STFT, f64 mel GEMM + log), the U-Net convs on the f64 matrix cores
// (v_mfma_f64_16x16x4_f64), pooling / transposed-conv phases / image->sequence in f64, W_ih, the BiGRU
// recurrence and the classifier in f64; only the salience is rounded to f32, once, for the decode (which is
// what the reference decodes: RMVPE.py:217).  Against the exact model the salience then errs by ~1e-13 and the
// only remaining difference is the f32 input rounding the reference itself applies (RMVPE.py:224: <= 1.4e-7 on
// the decision quantities of the headline clip).
//
// conv64_kernel: implicit GEMM Y[m][n] = sum_k W[k][m] X(k, n) over k = (input channel, tap), for the 3x3 /
// 1x1 convs on zero-bordered images ([C][H+2][W+2] flattened; tap offsets, border cells stored as 0) and the
// K = 1 GEMMs (mel basis, W_ih, fc).  A block is 4 waves; per 16-deep k chunk the weights [16][BM] and the
// input rows the chunk touches (with their tap halo) are staged into a double-buffered LDS tile, the next
// chunk's global loads in flight across the current chunk's MFMAs, one barrier per chunk.  An f64 MFMA is 64
// cycles, so the staging work per chunk is small beside the 4 x FM x FN MFMAs it feeds.
#include "rvc_common.h"
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <utility>

typedef double doublex4 __attribute__((ext_vector_type(4)));

namespace {

// v_mfma_f64_16x16x4_f64: lane l holds A[l&15][l>>4], B[l>>4][l&15]; C/D: col = l&15, row = (l>>4) + 4 r
RVC_DEV doublex4 mfma64(double a, double b, doublex4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// The same 16 x 16 x 4 product as four v_mfma_f64_4x4x4f64 (4 blocks of 4x4x4 per wave), 1.5x the f64 rate of the
// 16x16x4 form on gfx950 (72 against 47 TFLOP/s, scripts/bigru64_bench.hip).  Its lane layout, found by
// experiment (scripts/mfma64_layout.hip): block b = (l & 15) >> 2; A: row l & 3, k = l >> 4; B: col l & 3,
// k = l >> 4; D: col l & 3, row l >> 4.  With B as the 16x16x4 form's B (block b = columns 4b..4b+3) and, for
// component r, A = rows 4r..4r+3 replicated over the blocks (lane l: A[4r + (l & 3)][l >> 4]), D lane l is
// row 4r + (l >> 4), col l & 15: the 16x16x4 form's component r, so the epilogue is the same.  (The f64 form
// has no A broadcast: its CBSZ / ABID bits are modifiers, and ABID is ignored -- measured.)
RVC_DEV double mfma64q(double a, double b, double c) { return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0); }

// Measured (scripts/conv64_dbg.hip, round 4): no faster inside the conv engine than the 16x16x4 form (the MFMA-only
// loop 45-50 us either way on RMVPE's levels) while the 4 A values per fragment cost VGPRs and occupancy, so it
// is off; C64_M4=1 builds it.
#ifndef C64_M4
#define C64_M4 0
#endif

// the activations RMVPE's f64 network uses (plan64 refuses the others)
RVC_DEV double act64(double v, int act, double slope) {
    switch (act) {
        case RVC_ACT_RELU: return v > 0.0 ? v : 0.0;
        case RVC_ACT_SIGMOID: return 1.0 / (1.0 + exp(-v));
        case RVC_ACT_LOGCLAMP: return log(fmax(v, slope));
        default: return v;
    }
}


// scripts/conv64_dbg.hip builds this file with C64_DBG bits set to take parts of the main loop out (timing
// only; the results are then wrong): 1 = no global staging loads, 2 = no LDS staging stores, 4 = no barrier,
// 8 = no LDS operand reads
#ifndef C64_DBG
#define C64_DBG 0
#endif

// staged input doubles per thread (rows * span <= 256 * NB): 12 for the 512-column tile (3 channel rows of a
// 3x3 conv's 774-wide span), 8 otherwise (a K = 1 chunk's 16 rows of 128)
// (and 12 for the 256-column tiles of 32- / 36-deep chunks: 4 channel rows of a 3x3 conv's 518-wide span)
constexpr int nb64h(int BN, int KC) { return (BN >= 512 || (KC >= 32 && BN >= 256)) ? 12 : 8; }
template <int BN, int KC>
constexpr int nb64() { return nb64h(BN, KC); }

struct C64 {
    const double* x;
    const double* w;
    const double* bias;
    const double* res;
    double* y;
    float* yf;
    double* ws;  // split-K partials [ksplit][B][Co][nout]
    int64_t B, Ci, Co, Lin, Lout;
    int64_t x_bs, y_bs, res_bs;
    int K, pad, out_act, wrap;
    double out_slope;
    int ntoff;
    int toff[16];
    int span, span_s, rows_max, ksplit, cps;  // cps = chunks per split
    // compact form (2-D images with a narrow width): the GEMM's columns are the H x W interior cells only, not
    // the (H + 2) x (W + 2) bordered image (whose border columns are 2 / W of the work at W = 4, the 512-channel
    // layers); cw = W (0: bordered form), chh = H, nout = the column count either way
    int cw, chh, nout;
    // per-batch weights (the Winograd GEMMs): batch b uses w + (b % w_bmod) * w_bs (w_bmod 0: one weight)
    int64_t w_bs;
    int w_bmod;
};

RVC_DEV int tap64(const C64& p, int t) { return p.ntoff ? p.toff[t] : t; }

// output position n -> n, -1 (beyond Lout) or -(n + 2) for a border cell of a 2-D image (stored as 0)
RVC_DEV int opos64(const C64& p, int n) {
    if (n >= (int)p.Lout) return -1;
    if (p.wrap) {
        const int row = n / p.wrap, col = n - row * p.wrap;
        if (col == 0 || col == p.wrap - 1 || row == 0 || row == (int)p.Lout / p.wrap - 1) return -(n + 2);
    }
    return n;
}

RVC_DEV void store64(const C64& p, double acc, int b, int m, int t) {
    if (t == -1) return;
    const int64_t o = (int64_t)m * p.Lout + (t >= 0 ? t : -t - 2);
    double v = 0.0;
    if (t >= 0) {
        v = acc;
        if (p.bias) v += p.bias[m];
        v = act64(v, p.out_act, p.out_slope);
        if (p.res) v += p.res[b * p.res_bs + o];
    }
    if (p.yf) p.yf[b * p.y_bs + o] = (float)v;
    else p.y[b * p.y_bs + o] = v;
}

// compact form: interior cell n = h W + w sits at (h + 1)(W + 2) + w + 1 of the bordered image
RVC_DEV int cpos64(const C64& p, int n) { return n + 2 * (n / p.cw) + p.cw + 3; }

// ... and the cells on the image's edge also write the border cells beside them (0), corners included
RVC_DEV void border64(const C64& p, int b, int m, int n) {
    const int W = p.cw, R = W + 2;
    const int h = n / W, w = n - h * W;
    const int po = n + 2 * h + R + 1;
    const bool l = w == 0, r = w == W - 1;
    auto zero = [&](int o) { store64(p, 0.0, b, m, -o - 2); };
    if (l) zero(po - 1);
    if (r) zero(po + 1);
    if (h == 0) {
        zero(po - R);
        if (l) zero(po - R - 1);
        if (r) zero(po - R + 1);
    }
    if (h == p.chh - 1) {
        zero(po + R);
        if (l) zero(po + R - 1);
        if (r) zero(po + R + 1);
    }
}

template <int FM, int FN, int WM, int WN, bool CMP, int KC_>
__global__ __launch_bounds__(256, 2) void conv64_kernel(C64 p) {
    constexpr int KC = KC_;
    constexpr int BM = 16 * FM * WM;
    constexpr int BN = 16 * FN * WN;
    constexpr int NB64 = nb64<BN, KC>();
    constexpr int WS = BM + 4;            // weight tile row pitch (doubles)
    constexpr int NA = (KC * BM + 255) / 256;  // weight doubles staged per thread (the last slot partial at KC 36)
    constexpr bool NA_PART = (KC * BM) % 256 != 0;
    static_assert(WM * WN == 4 && NA >= 1 && KC % 4 == 0, "tile");
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int xs_n = p.rows_max * p.span_s + 1;  // + a dump cell
    double* Wsb = sm;                       // [2][KC][WS]
    double* Xsb = sm + 2 * KC * WS;         // [2][xs_n]
    int* koffb = (int*)(Xsb + 2 * xs_n);    // [2][KC]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int split = blockIdx.z % p.ksplit, b = blockIdx.z / p.ksplit;
    const int m0 = blockIdx.y * BM;
    const int n0 = blockIdx.x * BN;
    const int Co = (int)p.Co, Ci = (int)p.Ci, K = p.K;
    const double* xb = p.x + b * p.x_bs;
    const double* wb = p.w + (p.w_bmod ? (int64_t)(b % p.w_bmod) * p.w_bs : 0);
    const int kmax = Ci * K;
    const int nch = (kmax + KC - 1) / KC;
    const int ch_beg = split * p.cps;
    const int ch_end = min(nch, ch_beg + p.cps);
    const int h0 = CMP ? n0 / p.cw : 0;
    // the staged tile's first input position: column n0's (bordered) output position - pad
    const int base = CMP ? n0 + 2 * h0 + p.cw + 3 - p.pad : n0 - p.pad;
    const int lin = (int)p.Lin;
    const int lk = lane >> 4, ln = lane & 15;
    // this lane's B-operand column offsets into the staged tile (compact form: + 2 per image row crossed)
    int xo[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int nl = wn * 16 * FN + j * 16 + ln;
        xo[j] = CMP ? nl + 2 * ((n0 + nl) / p.cw - h0) : nl;
    }

    // per-thread staging slots of the rows x span input tile (the same for every chunk)
    int bslot[NB64];
    unsigned bok = 0;
#pragma unroll
    for (int i = 0; i < NB64; ++i) {
        const int idx = tid + 256 * i;
        const int r = idx / p.span, j = idx - r * p.span;
        bslot[i] = (r << 16) | j;
        bok |= (unsigned)(base + j >= 0 && base + j < lin) << i;
    }
    double ra[NA], rb[NB64];
    // raw loads only (clamped addresses): the values are first used by sstore, after the chunk's MFMAs
    auto gload = [&](int ch) {
        const int k0 = ch * KC;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int idx = tid + 256 * i;
            const int kk = idx / BM, m = idx % BM;
            const bool ok = k0 + kk < kmax && m0 + m < Co && (!NA_PART || idx < KC * BM);
            ra[i] = wb[ok ? (int64_t)(k0 + kk) * Co + m0 + m : 0];
        }
        const int c_lo = k0 / K;
        const int rows = min((k0 + KC - 1) / K, Ci - 1) - c_lo + 1;
        const int n = rows * p.span;
        const int rbase = c_lo * lin + base;
#pragma unroll
        for (int g = 0; g < NB64; g += 4) {
            if (g * 256 < n) {
#pragma unroll
                for (int i = g; i < g + 4; ++i) {
                    const int r = bslot[i] >> 16, j = bslot[i] & 0xffff;
                    const bool ok = r < rows && ((bok >> i) & 1u);
                    rb[i] = xb[ok ? rbase + r * lin + j : 0];
                }
            }
        }
    };
    auto sstore = [&](int ch, int buf) {
        const int k0 = ch * KC;
        double* Ws = Wsb + buf * KC * WS;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int idx = tid + 256 * i;
            const int kk = idx / BM, m = idx % BM;
            const bool ok = k0 + kk < kmax && m0 + m < Co;
            if (!NA_PART || idx < KC * BM) Ws[kk * WS + m] = ok ? ra[i] : 0.0;
        }
        const int c_lo = k0 / K;
        const int rows = min((k0 + KC - 1) / K, Ci - 1) - c_lo + 1;
        const int n = rows * p.span;
        double* Xs = Xsb + buf * xs_n;
#pragma unroll
        for (int g = 0; g < NB64; g += 4) {
            if (g * 256 < n) {  // block-uniform
#pragma unroll
                for (int i = g; i < g + 4; ++i) {
                    const int r = bslot[i] >> 16, j = bslot[i] & 0xffff;
                    const bool ok = r < rows && ((bok >> i) & 1u);
                    // slots past the tile go to the dump cell after it (no per-lane branch)
                    Xs[tid + 256 * i < n ? r * p.span_s + j : xs_n - 1] = ok ? rb[i] : 0.0;
                }
            }
        }
        if (tid < KC) {
            const int kk = k0 + tid;
            const int c = kk / K, t = kk - c * K;
            koffb[buf * KC + tid] = kk < kmax ? (c - c_lo) * p.span_s + tap64(p, t) : 0;
        }
    };

    doublex4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};

    if (ch_beg < ch_end) {
        gload(ch_beg);
        sstore(ch_beg, 0);
    }
    __syncthreads();
    for (int ch = ch_beg; ch < ch_end; ++ch) {
        const int cur = (ch - ch_beg) & 1;
        const bool more = ch + 1 < ch_end;
        if (more && !(C64_DBG & 1)) gload(ch + 1);
        // 16x16x4 form: lane reads A[m0 + (l & 15)][k]; 4x4x4 form: A[m0 + 4r + (l & 3)][k], r = 0..3
        const double* Ws = Wsb + cur * KC * WS + wm * 16 * FM + (C64_M4 ? (lane & 3) : ln);
        const double* Xs = Xsb + cur * xs_n;
        constexpr int NR = C64_M4 ? 4 : 1;
        // the chunk's tap offsets first (one LDS read per k-step, all issued together), then the operands
        // of k-step ks + 1 are read while k-step ks's MFMAs run (register double buffer)
        int ko[KC / 4];
#pragma unroll
        for (int ks = 0; ks < KC / 4; ++ks) ko[ks] = koffb[cur * KC + ks * 4 + lk];
        double a[2][FM][NR], bv[2][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < NR; ++r) a[0][i][r] = Ws[lk * WS + i * 16 + 4 * r];
#pragma unroll
        for (int j = 0; j < FN; ++j) bv[0][j] = Xs[ko[0] + xo[j]];
#pragma unroll
        for (int ks = 0; ks < KC / 4; ++ks) {
            const int q = (C64_DBG & 8) ? 0 : ks & 1;
            if (ks + 1 < KC / 4 && !(C64_DBG & 8)) {
                const int kk = (ks + 1) * 4 + lk;
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r = 0; r < NR; ++r) a[q ^ 1][i][r] = Ws[kk * WS + i * 16 + 4 * r];
#pragma unroll
                for (int j = 0; j < FN; ++j) bv[q ^ 1][j] = Xs[ko[ks + 1] + xo[j]];
            }
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    if constexpr (C64_M4) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[i][j][r] = mfma64q(a[q][i][r], bv[q][j], acc[i][j][r]);
                    } else {
                        acc[i][j] = mfma64(a[q][i][0], bv[q][j], acc[i][j]);
                    }
                }
        }
        if (more && !(C64_DBG & 2)) sstore(ch + 1, cur ^ 1);
        if (!(C64_DBG & 4)) __syncthreads();
    }

    if (p.ksplit > 1) {
        double* wsb = p.ws + ((int64_t)split * p.B + b) * p.Co * p.nout;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * 16 * FM + i * 16 + lk + 4 * r;
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int n = n0 + wn * 16 * FN + j * 16 + ln;
                    if (m < Co && n < p.nout) wsb[(int64_t)m * p.nout + n] = acc[i][j][r];
                }
            }
        return;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * 16 * FN + j * 16 + ln;
        const int t = CMP ? (n < p.nout ? cpos64(p, n) : -1) : opos64(p, n);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * 16 * FM + i * 16 + lk + 4 * r;
                if (m < Co) store64(p, acc[i][j][r], b, m, t);
            }
    }
    if (CMP) {  // the border cells beside this tile's edge cells (after the values: no accumulator is live)
        for (int j = 0; j < FN; ++j) {
            const int n = n0 + wn * 16 * FN + j * 16 + ln;
            if (n >= p.nout) continue;
            for (int i = 0; i < FM; ++i)
                for (int r = 0; r < 4; ++r) {
                    const int m = m0 + wm * 16 * FM + i * 16 + lk + 4 * r;
                    if (m < Co) border64(p, b, m, n);
                }
        }
    }
}

// split-K: the partials summed in split order, then the epilogue.  The partials' loads go out 8 at a time (the adds stay
// in split order): one dependent load per split made the 512-channel Winograd GEMMs' reduces (ksplit up to 32) ~75 us
// each, 2.4 ms per clip (kernel trace r6e)
__global__ void conv64_splitk_reduce(C64 p) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = blockIdx.y, b = blockIdx.z;
    if (n >= p.nout) return;
    const int64_t sstride = p.B * p.Co * p.nout;
    const double* src = p.ws + ((int64_t)b * p.Co + m) * p.nout + n;
    double s = 0.0;
    int k = 0;
    for (; k + 8 <= p.ksplit; k += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(k + u) * sstride];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < p.ksplit; ++k) s += src[k * sstride];
    if (p.cw) {
        store64(p, s, b, m, cpos64(p, n));
        border64(p, b, m, n);
    } else {
        store64(p, s, b, m, opos64(p, n));
    }
}

struct Cfg64 {
    int FM, FN, WM, WN, KC;
};

// the tiles the planner chooses from (BM x BN = 16 FM WM x 16 FN WN, k chunk KC): the 32-deep chunks halve the
// barriers and staging rounds per k and pay where the tile's registers and LDS leave room (scripts/conv64_dbg.hip:
// 32 x 128 tiles 15-20 % faster, 32 x 256 ones slower)
constexpr int N_TILES64 = 18;
constexpr Cfg64 kTiles64[N_TILES64] = {
    {1, 8, 1, 4, 16},  // 0: 16 x 512
    {1, 4, 1, 4, 16},  // 1: 16 x 256
    {2, 4, 1, 4, 16},  // 2: 32 x 256
    {2, 2, 1, 4, 16},  // 3: 32 x 128
    {2, 4, 2, 2, 16},  // 4: 64 x 128
    {2, 2, 2, 2, 16},  // 5: 64 x 64
    {4, 4, 2, 2, 16},  // 6: 128 x 128
    {4, 2, 2, 2, 16},  // 7: 128 x 64
    {1, 4, 1, 4, 32},  // 8: 16 x 256, KC 32
    {2, 2, 1, 4, 32},  // 9: 32 x 128, KC 32
    {2, 4, 2, 2, 32},  // 10: 64 x 128, KC 32
    {2, 2, 2, 2, 32},  // 11: 64 x 64, KC 32
    {4, 2, 2, 2, 32},  // 12: 128 x 64, KC 32
    {2, 1, 4, 1, 16},  // 13: 128 x 16 (the Winograd GEMMs of small images: a few dozen columns)
    {2, 1, 4, 1, 32},  // 14: 128 x 16, KC 32
    // 3x3 convs only: 36-deep chunks = 4 whole input channels, so each channel row is staged once per block
    // (16-deep chunks straddle channels and stage ~1.6 rows per channel)
    {1, 4, 1, 4, 36},  // 15: 16 x 256, KC 36
    {2, 2, 1, 4, 36},  // 16: 32 x 128, KC 36
    {2, 4, 1, 4, 36},  // 17: 32 x 256, KC 36
};

// the compact form of the 128 x 128 tile spills (its per-lane column offsets on top of 255 VGPRs): not built;
// with the 4x4x4 MFMA form (4 A values per fragment) the bordered one spills too and the planner skips it
constexpr bool has_cmp64(int t) { return t != 6; }

template <int T, bool CMP>
const void* kernel64() {
    constexpr Cfg64 c = kTiles64[T];
    if constexpr (CMP && !has_cmp64(T)) return nullptr;
    else return reinterpret_cast<const void*>(&conv64_kernel<c.FM, c.FN, c.WM, c.WN, CMP, c.KC>);
}

template <int T>
void launch64t(const C64& p, dim3 grid, size_t lds, hipStream_t s) {
    constexpr Cfg64 c = kTiles64[T];
    if constexpr (has_cmp64(T)) {
        if (p.cw) {
            hipLaunchKernelGGL((conv64_kernel<c.FM, c.FN, c.WM, c.WN, true, c.KC>), grid, dim3(256), lds, s, p);
            return;
        }
    }
    hipLaunchKernelGGL((conv64_kernel<c.FM, c.FN, c.WM, c.WN, false, c.KC>), grid, dim3(256), lds, s, p);
}

template <int... T>
void launch64_any(int tile, const C64& p, dim3 grid, size_t lds, hipStream_t s, std::integer_sequence<int, T...>) {
    ((tile == T ? launch64t<T>(p, grid, lds, s) : void()), ...);
}

void launch64(int tile, const C64& p, dim3 grid, size_t lds, hipStream_t s) {
    launch64_any(tile, p, grid, lds, s, std::make_integer_sequence<int, N_TILES64>{});
}

template <int... T>
const void* kernel64_any(int tile, bool cmp, std::integer_sequence<int, T...>) {
    const void* k = nullptr;
    ((tile == T ? (void)(k = cmp ? kernel64<T, true>() : kernel64<T, false>()) : void()), ...);
    return k;
}

// blocks of a tile resident per CU by its registers (the runtime's occupancy answer, asked once per tile)
int occ64(int tile, bool cmp) {
    static int cache[N_TILES64][2];
    int& o = cache[tile][cmp];
    if (o == 0) {
        const void* k = kernel64_any(tile, cmp, std::make_integer_sequence<int, N_TILES64>{});
        int n = 0;
        if (!k || hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, 0) != hipSuccess || n < 1) n = 1;
        o = n;
    }
    return o;
}

// forced plan (rvc_conv64_set_plan; diagnostics and sweeps): tile, split-K, compact (-1 = the planner's)
int g_force_tile = -1, g_force_ks = -1, g_force_cmp = -1;

struct Plan64 {
    int tile, ks, cmp;
    double cost_ns;
};

// The planner's time model (ns) of one (tile, split-K, form) choice, fitted (least squares weighted to the fast
// plans, median error 5.8 %) to every forced plan on RMVPE's U-Net shapes (scripts/conv64_sweep.py,
// profiles/r4_conv64_sweep.json): blocks are dealt evenly over 256 CUs and run `occ` at a time; a block's MFMAs
// (MFMA_NS each per SIMD, the chip's measured f64 rate) cost SHARED of that when its CU holds other blocks too
// and LONE when it runs alone; every k chunk of every block costs CHUNK_NS plus STAGE_NS per byte it stages
// (input rows with their halo, weights); a split adds the partials' round trip (RED_BPNS bytes per ns) and the
// reduce launch.  The fit leaves the MFMA terms small: on these shapes the staging, not the f64 MFMA rate, sets
// the time (scripts/conv64_dbg.hip: the MFMA-only loop runs 45-50 us where the whole kernel takes 55-60).
constexpr double MFMA_NS = 44.6, SHARED = 0.156, LONE = 0.247, CHUNK_NS = 287.6, STAGE_NS = 0.0247,
                 RED_BPNS = 8770.0, RED_FIX_NS = 7890.0;

double cost64(int FM, int FN, int KC, int64_t nblk, int cps, int occ, int64_t stage_bytes) {
    const double bt = cps * FM * FN * KC * MFMA_NS;
    const int64_t per_cu = (nblk + 255) / 256;
    const int64_t full = per_cu / occ, rem = per_cu % occ;
    const int64_t shared = (occ > 1 ? full * occ : 0) + (rem > 1 ? rem : 0);
    const int64_t lone = (occ == 1 ? full : 0) + (rem == 1 ? 1 : 0);
    return bt * (SHARED * shared + LONE * lone) + (CHUNK_NS + STAGE_NS * stage_bytes) * cps * per_cu;
}

// the staged tile's width (columns + tap halo) for a tile of BN columns
int span64(int BN, int maxoff, int cw) {
    return cw ? BN + 2 * ((cw + BN - 2) / cw) + maxoff : BN + maxoff;
}

int plan64(const rvc_conv64_args* a, C64& p, int& tile, dim3& grid, size_t& lds) {
    RVC_CHECK_ARG(a && a->x && a->w && a->y, "conv64: null pointer");
    RVC_CHECK_ARG(a->B > 0 && a->Ci > 0 && a->Co > 0 && a->K > 0 && a->Lin > 0 && a->Lout > 0,
                  "conv64: bad sizes B=%lld Ci=%lld Co=%lld K=%d Lin=%lld Lout=%lld", (long long)a->B,
                  (long long)a->Ci, (long long)a->Co, a->K, (long long)a->Lin, (long long)a->Lout);
    RVC_CHECK_ARG(a->Co * a->Lout < (1ll << 31) && a->Ci * a->Lin < (1ll << 31) && a->Lin + a->pad < (1ll << 30) &&
                      a->pad >= 0 && a->Ci * a->K < (1ll << 30),
                  "conv64: per-batch tensor exceeds 2^31 elements (use the batch dimension)");
    RVC_CHECK_ARG(a->ntoff == 0 || (a->ntoff == a->K && a->K <= 16), "conv64: toff needs ntoff == K <= 16");
    RVC_CHECK_ARG(a->out_act == RVC_ACT_NONE || a->out_act == RVC_ACT_RELU || a->out_act == RVC_ACT_SIGMOID ||
                      a->out_act == RVC_ACT_LOGCLAMP,
                  "conv64: out_act %d (NONE, RELU, SIGMOID, LOGCLAMP)", a->out_act);
    RVC_CHECK_ARG(a->wrap == 0 || (a->wrap >= 3 && a->Lout % a->wrap == 0 && a->Lout / a->wrap >= 3),
                  "conv64: Lout must be rows x wrap");
    int maxoff = a->ntoff ? 0 : a->K - 1;
    for (int i = 0; i < a->ntoff; ++i) {
        RVC_CHECK_ARG(a->toff[i] >= 0, "conv64: negative tap offset");
        maxoff = a->toff[i] > maxoff ? a->toff[i] : maxoff;
    }
    RVC_CHECK_ARG(a->w_bmod >= 0 && (a->w_bmod == 0 || a->w_bstride >= a->Ci * a->K * a->Co), "conv64: bad w_bmod / w_bstride");
    p.x = a->x; p.w = a->w; p.bias = a->bias; p.res = a->res;
    p.w_bs = a->w_bstride;
    p.w_bmod = a->w_bmod;
    p.y = a->y_f32 ? nullptr : (double*)a->y;
    p.yf = a->y_f32 ? (float*)a->y : nullptr;
    p.ws = nullptr;
    p.B = a->B; p.Ci = a->Ci; p.Co = a->Co; p.Lin = a->Lin; p.Lout = a->Lout;
    p.x_bs = a->x_bstride ? a->x_bstride : a->Ci * a->Lin;
    p.y_bs = a->y_bstride ? a->y_bstride : a->Co * a->Lout;
    p.res_bs = a->res_bstride ? a->res_bstride : a->Co * a->Lout;
    p.K = a->K; p.pad = a->pad; p.out_act = a->out_act; p.wrap = a->wrap; p.out_slope = a->out_slope;
    p.ntoff = a->ntoff;
    for (int i = 0; i < 16; ++i) p.toff[i] = a->ntoff && i < a->ntoff ? a->toff[i] : 0;

    auto rows_of = [&](int kc) {
        const int r = (kc % a->K == 0) ? kc / a->K : (kc - 1) / a->K + 2;
        return r > a->Ci ? (int)a->Ci : r;
    };
    const int W = a->wrap ? (int)a->wrap - 2 : 0, H = a->wrap ? (int)(a->Lout / a->wrap) - 2 : 0;
    const int64_t ncols[2] = {a->Lout, (int64_t)H * W};

    Plan64 best = {-1, 1, 0, 1e300};
    for (int cmp = 0; cmp < (a->wrap ? 2 : 1); ++cmp) {
        if (g_force_cmp >= 0 && cmp != g_force_cmp) continue;
        for (int t = 0; t < N_TILES64; ++t) {
            if ((g_force_tile >= 0 && t != g_force_tile) || (cmp && !has_cmp64(t)) || (C64_M4 && t == 6)) continue;
            // the 16 x 512 tile lost to 16 x 256 on every shape of the sweep (occupancy 2 against 4): forced only
            if (t == 0 && g_force_tile != 0) continue;
            const Cfg64 c = kTiles64[t];
            const int BM = 16 * c.FM * c.WM, BN = 16 * c.FN * c.WN, KC = c.KC;
            const int rows_max = rows_of(KC);
            const int nch = (int)((a->Ci * a->K + KC - 1) / KC);
            // the channel-aligned chunks: 3x3 convs only (RVC_C64_KC36=0: never)
            static const int kc36 = getenv("RVC_C64_KC36") ? atoi(getenv("RVC_C64_KC36")) : 1;
            // (and not at 16 input channels: 4 chunks leave the pipeline no steady state -- the sweep's 16 -> 16
            // level-0 conv ran 78.5 us with them against 74.7 with 16-deep chunks)
            if (KC % 16 != 0 && (a->K != 9 || !kc36 || a->Ci < 32)) continue;
            const int span = span64(BN, maxoff, cmp ? W : 0);
            if ((int64_t)rows_max * span > 256 * nb64h(BN, KC) || span >= 65536) continue;
            const size_t l = (size_t)(2 * KC * (BM + 4) + 2 * (rows_max * (span + 1) + 1)) * 8 + 2 * KC * 4;
            if (l > 160 * 1024) continue;
            const int occ = std::max(1, std::min(occ64(t, cmp), (int)(160 * 1024 / l)));
            const int64_t tiles = (a->Co + BM - 1) / BM * cdiv(ncols[cmp], BN) * a->B;
            const int ks_max = std::max(1, std::min(32, nch / 2));
            for (int ks = 1; ks <= ks_max; ++ks) {
                if (g_force_ks >= 1 && ks != std::min(g_force_ks, ks_max)) continue;
                const int cps = (nch + ks - 1) / ks;
                const int kse = (nch + cps - 1) / cps;
                if (kse != ks) continue;
                double cost = cost64(c.FM, c.FN, KC, tiles * kse, cps, occ, ((int64_t)rows_max * span + KC * BM) * 8);
                if (kse > 1) cost += (double)kse * a->B * a->Co * ncols[cmp] * 16 / RED_BPNS + RED_FIX_NS;
                if (cost < best.cost_ns) best = {t, kse, cmp, cost};
            }
        }
    }
    RVC_CHECK_ARG(best.tile >= 0, "conv64: no tile stages the rows x span of K %d (maxoff %d)", a->K, maxoff);
    tile = best.tile;
    const Cfg64 c = kTiles64[tile];
    const int BM = 16 * c.FM * c.WM, BN = 16 * c.FN * c.WN, KC = c.KC;
    const int rows_max = rows_of(KC);
    const int nch = (int)((a->Ci * a->K + KC - 1) / KC);
    p.cw = best.cmp ? W : 0;
    p.chh = best.cmp ? H : 0;
    p.nout = (int)ncols[best.cmp];
    p.span = span64(BN, maxoff, p.cw);
    p.span_s = p.span + 1;
    p.rows_max = rows_max;
    p.cps = (nch + best.ks - 1) / best.ks;
    p.ksplit = (nch + p.cps - 1) / p.cps;
    lds = (size_t)(2 * KC * (BM + 4) + 2 * (rows_max * p.span_s + 1)) * 8 + 2 * KC * 4;
    grid = dim3(cdiv(p.nout, BN), (unsigned)((a->Co + BM - 1) / BM), (unsigned)(a->B * p.ksplit));
    RVC_CHECK_ARG(grid.y < 65536 && grid.z < 65536, "conv64: grid too large");
    return RVC_OK;
}

// ---------------------------------------------------------------- f64 image / sequence glue (rmvpe.hip's f32 forms)
__global__ void mel_image64_kernel(const double* mel, double* img, int M, int64_t F, int64_t Tp, double scale,
                                   double shift, int64_t mel_bs, int64_t img_bs) {
    const int64_t t = blockIdx.x;
    const int m = threadIdx.x;
    mel += blockIdx.y * mel_bs;
    img += blockIdx.y * img_bs;
    if (t >= Tp || m >= M) return;
    const int64_t s = t < F ? t : 2 * (F - 1) - t;
    img[(t + 1) * (M + 2) + m + 1] = mel[(int64_t)m * F + s] * scale + shift;
    // the zero border too (the image needs no zero-fill launch before it)
    if (m == 0) {
        img[(t + 1) * (M + 2)] = 0.0;
        img[(t + 1) * (M + 2) + M + 1] = 0.0;
    }
    if (t == 0 || t == Tp - 1) {
        double* row = img + (t == 0 ? 0 : (Tp + 1) * (M + 2));
        row[m + 1] = 0.0;
        if (m == 0) {
            row[0] = 0.0;
            row[M + 1] = 0.0;
        }
    }
}

// the zero border cells beside interior cell (y, x) of a [H + 2][W + 2] plane (corners by the corner cells)
RVC_DEV void border_zero64(double* plane, int y, int x, int H, int W) {
    const int R = W + 2;
    if (x == 0) plane[(int64_t)(y + 1) * R] = 0.0;
    if (x == W - 1) plane[(int64_t)(y + 1) * R + W + 1] = 0.0;
    if (y == 0 || y == H - 1) {
        double* row = plane + (y == 0 ? 0 : (int64_t)(H + 1) * R);
        row[x + 1] = 0.0;
        if (x == 0) row[0] = 0.0;
        if (x == W - 1) row[W + 1] = 0.0;
    }
}

// AvgPool2d(2): ((a + b) + c) + d, / 4
__global__ void avgpool2_64_kernel(const double* in, double* out, int C, int H, int W, int64_t in_bs, int64_t out_bs) {
    const int Ho = H / 2, Wo = W / 2;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    in += blockIdx.y * in_bs;
    out += blockIdx.y * out_bs;
    if (i >= (int64_t)C * Ho * Wo) return;
    const int x = (int)(i % Wo);
    const int64_t r = i / Wo;
    const int y = (int)(r % Ho), c = (int)(r / Ho);
    const double* ib = in + (int64_t)c * (H + 2) * (W + 2);
    const int64_t a0 = (int64_t)(2 * y + 1) * (W + 2) + 2 * x + 1;
    double s = ib[a0];
    s += ib[a0 + 1];
    s += ib[a0 + W + 2];
    s += ib[a0 + W + 3];
    out[(int64_t)c * (Ho + 2) * (Wo + 2) + (int64_t)(y + 1) * (Wo + 2) + x + 1] = s / 4.0;
    border_zero64(out + (int64_t)c * (Ho + 2) * (Wo + 2), y, x, Ho, Wo);
}

__global__ void interleave4_64_kernel(const double* ph, double* out, int C, int H, int W, int64_t ph_bs,
                                      int64_t out_bs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int Ho = 2 * H, Wo = 2 * W;
    ph += blockIdx.y * ph_bs;
    out += blockIdx.y * out_bs;
    if (i >= (int64_t)C * Ho * Wo) return;
    const int xo = (int)(i % Wo);
    const int64_t r = i / Wo;
    const int yo = (int)(r % Ho), c = (int)(r / Ho);
    const int py = yo & 1, px = xo & 1, y = yo >> 1, x = xo >> 1;
    const int64_t plane = (int64_t)(H + 2) * (W + 2);
    out[(int64_t)c * (Ho + 2) * (Wo + 2) + (int64_t)(yo + 1) * (Wo + 2) + xo + 1] =
        ph[((int64_t)(py * 2 + px) * C + c) * plane + (int64_t)(y + 1) * (W + 2) + x + 1];
    border_zero64(out + (int64_t)c * (Ho + 2) * (Wo + 2), yo, xo, Ho, Wo);
}

__global__ void img_to_seq64_kernel(const double* img, double* x, int C, int64_t H, int W, int64_t img_bs,
                                    int64_t x_bs) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int cf = blockIdx.y;
    img += blockIdx.z * img_bs;
    x += blockIdx.z * x_bs;
    if (t >= H) return;
    const int c = cf / W, f = cf - c * W;
    x[(int64_t)cf * H + t] = img[(int64_t)c * (H + 2) * (W + 2) + (t + 1) * (W + 2) + f + 1];
}

// ---------------------------------------------------------------- f64 Winograd F(4x4, 3x3) for the deep U-Net levels
// The f64 matrix cores are power-bound chip-wide: the conv engine's MFMA-only loop runs ~36-39 TFLOP/s on every
// RMVPE level whatever the tile, split or MFMA form, and per SIMD at near the nominal rate only while <= ~96 CUs
// run (scripts/conv64_dbg.hip, round 4) -- so the lever is fewer MFMA FLOPs.  Winograd F(4x4, 3x3) (Lavin & Gray)
// computes each 4 x 4 output tile from a 6 x 6 input tile with 36 products per (ci, co) instead of 144:
//   Y = A^T [ sum_ci (G g G^T)[co][ci] (.) (B^T d B)[ci] ] A
// as (1) an input transform U[36][Ci][P] (P = output tiles), (2) 36 GEMMs M[x] = V[x]^T U[x] on the conv engine
// (K = 1, per-batch weights), (3) an output transform with the bias / activation / residual epilogue and the
// zero border.  In f64 the transforms cost ~1e-14 relative (numpy: 1.1e-14 at 512 channels vs 1e-15 direct),
// 7 orders below the f0 decisions' 1e-7 scale.  Used where the GEMMs dominate the transforms' HBM traffic
// (2.25x the input and output) and are wide enough: >= 64 channels in and out and >= 90 output tiles
// (rvc_wino64_use).  Measured (one box, RMVPE alone / the bench's clip stream): every >= 64-channel conv 15.64 ms /
// 925 xRT, >= 90 tiles (levels 2-4, not the 94 x 4 middle) 14.70 ms / 929, >= 300 15.05 / 926, none 15.52 / 907.
namespace {
// B^T d (6 -> 6) for one column / row
RVC_DEV void wbt(const double* d, double* o) {
    o[0] = 4.0 * d[0] - 5.0 * d[2] + d[4];
    o[1] = -4.0 * d[1] - 4.0 * d[2] + d[3] + d[4];
    o[2] = 4.0 * d[1] - 4.0 * d[2] - d[3] + d[4];
    o[3] = -2.0 * d[1] - d[2] + 2.0 * d[3] + d[4];
    o[4] = 2.0 * d[1] - d[2] - 2.0 * d[3] + d[4];
    o[5] = 4.0 * d[1] - 5.0 * d[3] + d[5];
}
// A^T m (6 -> 4)
RVC_DEV void wat(const double* m, double* o) {
    o[0] = m[0] + m[1] + m[2] + m[3] + m[4];
    o[1] = m[1] - m[2] + 2.0 * m[3] - 2.0 * m[4];
    o[2] = m[1] + m[2] + 4.0 * m[3] + 4.0 * m[4];
    o[3] = m[1] - m[2] + 8.0 * m[3] - 8.0 * m[4] + m[5];
}
// G g (3 -> 6)
RVC_DEV void wg(const double* g, double* o) {
    o[0] = g[0] / 4.0;
    o[1] = -(g[0] + g[1] + g[2]) / 6.0;
    o[2] = -(g[0] - g[1] + g[2]) / 6.0;
    o[3] = g[0] / 24.0 + g[1] / 12.0 + g[2] / 6.0;
    o[4] = g[0] / 24.0 - g[1] / 12.0 + g[2] / 6.0;
    o[5] = g[2];
}

// KM weights w[(ci * 9 + dy * 3 + dx)][co] -> V[36][ci][co]
__global__ void wino_w64_kernel(const double* w, double* v, int Ci, int Co) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Ci * Co) return;
    const int ci = (int)(i / Co), co = (int)(i - (int64_t)ci * Co);
    double g[3][3], t[6][3], col[3], o6[6];
    for (int k = 0; k < 9; ++k) g[k / 3][k % 3] = w[(int64_t)(ci * 9 + k) * Co + co];
    for (int c = 0; c < 3; ++c) {  // G g: columns
        for (int r = 0; r < 3; ++r) col[r] = g[r][c];
        wg(col, o6);
        for (int r = 0; r < 6; ++r) t[r][c] = o6[r];
    }
    for (int r = 0; r < 6; ++r) {  // (G g) G^T: rows
        wg(t[r], o6);
        for (int c = 0; c < 6; ++c) v[((int64_t)(r * 6 + c) * Ci + ci) * Co + co] = o6[c];
    }
}

// The output transform stages a band of RT tile rows through LDS (one block: 256 threads, one channel, RT tile
// rows, all tile columns): each thread transforms tiles into LDS, then the image rows are written whole and
// coalesced with the epilogue (L2-level shape 15.5 vs 20.1 us for one thread per tile writing its 4 x 4 block).
// RT = the tile rows that make ~256 tiles (rows of W / 4 tiles each).
inline int wino_rt(int W) {
    const int tw = (W + 3) / 4;
    return tw >= 256 ? 1 : 256 / tw;
}

// bordered x [B][C][(H+2)(W+2)] -> U [B][36][C][P], tile p = (th, tw): bordered rows 4 th .. 4 th + 5, cols 4 tw ..
// 4 tw + 5 (past the bordered image: 0).  One thread per tile, its patch read straight from global (the overlapping
// patches hit L1 / L2): 64-thread blocks, many of them, measured faster than banding the rows through LDS
// (L2-level shape 9.7 vs 14.1 us -- the banded form has 7x fewer blocks).
__global__ __launch_bounds__(64) void wino_in64_kernel(const double* x, double* u, int C, int H, int W, int TW, int P,
                                                       int64_t x_bs, int64_t u_bs) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int c = blockIdx.y, b = blockIdx.z;
    if (p >= P) return;
    const int th = p / TW, tw = p - th * TW;
    const int R = W + 2;
    const double* xc = x + b * x_bs + (int64_t)c * (H + 2) * R;
    double d[6][6], o6[6], col[6];
    for (int r = 0; r < 6; ++r) {
        const int y = 4 * th + r;
        for (int q = 0; q < 6; ++q) {
            const int xx = 4 * tw + q;
            d[r][q] = (y < H + 2 && xx < R) ? xc[(int64_t)y * R + xx] : 0.0;
        }
    }
    for (int r = 0; r < 6; ++r) {  // d B: rows, in place
        wbt(d[r], o6);
        for (int q = 0; q < 6; ++q) d[r][q] = o6[q];
    }
    double* ub = u + b * u_bs + (int64_t)c * P + p;
    for (int q = 0; q < 6; ++q) {  // B^T (d B): columns
        for (int r = 0; r < 6; ++r) col[r] = d[r][q];
        wbt(col, o6);
        for (int r = 0; r < 6; ++r) ub[(int64_t)(r * 6 + q) * C * P] = o6[r];
    }
}

// M [B][36][Co][P] -> bordered y [B][Co][(H+2)(W+2)]: act(A^T m A + bias) (+ res), the band's border cells 0
__global__ __launch_bounds__(256) void wino_out64_kernel(const double* m, double* y, float* yf, const double* bias,
                                                         const double* res, int Co, int H, int W, int TW, int P, int RT,
                                                         int act, int64_t m_bs, int64_t y_bs, int64_t res_bs) {
    extern __shared__ double band[];  // [4 RT][W] transformed outputs
    const int co = blockIdx.y, b = blockIdx.z;
    const int th0 = blockIdx.x * RT;
    const int TH = (H + 3) / 4;
    const int nth = min(RT, TH - th0);
    const int R = W + 2;
    const int W4 = 4 * TW;
    const double* mb = m + b * m_bs + (int64_t)co * P;
    for (int t = threadIdx.x; t < nth * TW; t += 256) {
        const int tr = t / TW, tw = t - tr * TW;
        const int p = (th0 + tr) * TW + tw;
        double mm[6][6], tt[4][6], col[6], o4[4];
        for (int r = 0; r < 6; ++r)
            for (int q = 0; q < 6; ++q) mm[r][q] = mb[(int64_t)(r * 6 + q) * Co * P + p];
        for (int q = 0; q < 6; ++q) {  // A^T m: columns
            for (int r = 0; r < 6; ++r) col[r] = mm[r][q];
            wat(col, o4);
            for (int r = 0; r < 4; ++r) tt[r][q] = o4[r];
        }
        for (int r = 0; r < 4; ++r) {  // (A^T m) A: rows
            wat(tt[r], o4);
            for (int q = 0; q < 4; ++q) band[(4 * tr + r) * W4 + 4 * tw + q] = o4[q];
        }
    }
    __syncthreads();
    const int64_t ybase = b * y_bs + (int64_t)co * (H + 2) * R;
    const double* rb = res ? res + b * res_bs + (int64_t)co * (H + 2) * R : nullptr;
    const double bv = bias ? bias[co] : 0.0;
    auto put = [&](int64_t o, double v) {
        if (yf) yf[ybase + o] = (float)v;
        else y[ybase + o] = v;
    };
    const int oy0 = 4 * th0, ny = min(4 * nth, H - oy0);
    // the band's output rows with their left / right border cells, row-contiguous
    for (int i = threadIdx.x; i < ny * R; i += 256) {
        const int r = i / R, q = i - r * R;
        const int64_t o = (int64_t)(oy0 + r + 1) * R + q;
        if (q == 0 || q == R - 1) {
            put(o, 0.0);
        } else {
            double v = act64(band[r * W4 + q - 1] + bv, act, 0.0);
            if (rb) v += rb[o];
            put(o, v);
        }
    }
    if (th0 == 0)
        for (int q = threadIdx.x; q < R; q += 256) put(q, 0.0);
    if (th0 + nth == TH)
        for (int q = threadIdx.x; q < R; q += 256) put((int64_t)(H + 1) * R + q, 0.0);
}

// Fused Winograd for the small-channel levels (Ci in {16, 32, 64}, Co in {16, 32}: U-Net levels 0-1), where the
// separate transforms' 2.25x HBM traffic would cost more than the 4x fewer MFMA FLOPs save.  Measured no faster
// than the direct engine (its per-thread 6x6 patch reads and 4-wide output writes are strided, 25 % of each
// access used), so off by default (RVC_RMVPE_WINO=3 turns it on; correct either way, tests/test_gpu_ops.py).  One block = 16
// consecutive output tiles (P order) of one image, all Co: per 16-channel input chunk the threads transform their
// (channel, tile) 6x6 patches (read from the bordered image, L1 / L2 resident across the overlapping patches)
// into U [36][16 ci][16 tiles] in LDS, and each wave accumulates XI of the 36 products M[x] += V[x]^T U[x]
// (v_mfma_f64_16x16x4: V from global, L2 resident, U from LDS); at the end M goes through LDS, 16 output
// channels at a time, to the output transform with the bias / activation / residual epilogue and the zero border.
// Nothing but x, v and y touches HBM.  Waves: 36 / XI (XI = 9 at Co 16: 4 waves; 6 at Co 32: 6 waves, which
// keeps the accumulators at 48 doubles per lane).
template <int CI, int CO>
__global__ __launch_bounds__(64 * (CO == 16 ? 4 : 6), CO == 16 ? 2 : 1) void wino_fused64_kernel(
    const double* x, const double* v, const double* bias, const double* res, double* y, float* yf, int H, int W,
    int TW, int P, int act, int64_t x_bs, int64_t y_bs, int64_t res_bs) {
    constexpr int XI = CO == 16 ? 9 : 6;  // products per wave
    constexpr int NW = 36 / XI;
    constexpr int NT = 64 * NW;
    constexpr int CB = CO / 16;           // 16-channel output blocks
    extern __shared__ double sm[];         // [36][16][16]: U chunk, then M (16 output channels at a time)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.y;
    const int p0 = blockIdx.x * 16;
    const int R = W + 2;
    const double* xb = x + b * x_bs;
    doublex4 acc[XI][CB];
#pragma unroll
    for (int i = 0; i < XI; ++i)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[i][c] = doublex4{0.0, 0.0, 0.0, 0.0};
    const int lk = lane >> 4, ln = lane & 15;
#pragma unroll 1
    for (int c0 = 0; c0 < CI; c0 += 16) {
        // input transform of (channel c0 + t / 16, tile p0 + t % 16)
        for (int t = tid; t < 256; t += NT) {
            const int cl = t >> 4, j = t & 15, p = p0 + j;
            double d[6][6];
            if (p < P) {
                const int th = p / TW, tw = p - th * TW;
                const double* xc = xb + (int64_t)(c0 + cl) * (H + 2) * R;
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    const int yy = 4 * th + r;
#pragma unroll
                    for (int q = 0; q < 6; ++q) {
                        const int xx = 4 * tw + q;
                        d[r][q] = (yy < H + 2 && xx < R) ? xc[(int64_t)yy * R + xx] : 0.0;
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < 6; ++r)
#pragma unroll
                    for (int q = 0; q < 6; ++q) d[r][q] = 0.0;
            }
            double o6[6], col[6];
#pragma unroll
            for (int r = 0; r < 6; ++r) {  // d B: rows, in place
                wbt(d[r], o6);
#pragma unroll
                for (int q = 0; q < 6; ++q) d[r][q] = o6[q];
            }
#pragma unroll
            for (int q = 0; q < 6; ++q) {  // B^T (d B): columns
#pragma unroll
                for (int r = 0; r < 6; ++r) col[r] = d[r][q];
                wbt(col, o6);
#pragma unroll
                for (int r = 0; r < 6; ++r) sm[((r * 6 + q) * 16 + cl) * 16 + j] = o6[r];
            }
        }
        __syncthreads();
        // products: M[x][co][tile] += sum_ci V[x][ci][co] U[x][ci][tile], 4 k-steps of 4 channels
#pragma unroll
        for (int i = 0; i < XI; ++i) {
            const int xi = wave * XI + i;
            const double* vx = v + ((int64_t)xi * CI + c0) * CO;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const double bop = sm[(xi * 16 + ks * 4 + lk) * 16 + ln];
#pragma unroll
                for (int c = 0; c < CB; ++c)
                    acc[i][c] = mfma64(vx[(ks * 4 + lk) * CO + c * 16 + ln], bop, acc[i][c]);
            }
        }
        __syncthreads();
    }
    const double* rb = res ? res + b * res_bs : nullptr;
    const int64_t ybase = b * y_bs;
    auto put = [&](int64_t o, double val) {
        if (yf) yf[ybase + o] = (float)val;
        else y[ybase + o] = val;
    };
    const int TH = (H + 3) / 4;
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        // this wave's M[x][co][tile] (D layout: col = tile = l & 15, row = co = (l >> 4) + 4 r) -> LDS
#pragma unroll
        for (int i = 0; i < XI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) sm[((wave * XI + i) * 16 + lk + 4 * r) * 16 + ln] = acc[i][c][r];
        __syncthreads();
        for (int t = tid; t < 256; t += NT) {
            const int cl = t >> 4, j = t & 15, p = p0 + j;
            if (p >= P) continue;
            const int co = c * 16 + cl;
            const int th = p / TW, tw = p - th * TW;
            double mm[6][6], o4[4], col[6];
#pragma unroll
            for (int r = 0; r < 6; ++r)
#pragma unroll
                for (int q = 0; q < 6; ++q) mm[r][q] = sm[((r * 6 + q) * 16 + cl) * 16 + j];
            double tt[4][6];
#pragma unroll
            for (int q = 0; q < 6; ++q) {  // A^T m: columns
#pragma unroll
                for (int r = 0; r < 6; ++r) col[r] = mm[r][q];
                wat(col, o4);
#pragma unroll
                for (int r = 0; r < 4; ++r) tt[r][q] = o4[r];
            }
            const int64_t cbase = (int64_t)co * (H + 2) * R;
            const double bv = bias ? bias[co] : 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // (A^T m) A: rows
                wat(tt[r], o4);
                const int oy = 4 * th + r;
                if (oy < H) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int ox = 4 * tw + q;
                        if (ox < W) {
                            const int64_t o = cbase + (int64_t)(oy + 1) * R + ox + 1;
                            double val = act64(o4[q] + bv, act, 0.0);
                            if (rb) val += rb[o];
                            put(o, val);
                        }
                    }
                }
            }
            // border cells beside this tile: top / bottom rows (with the corners) and left / right columns
            const int x0 = 4 * tw + 1, x1 = min(4 * tw + 4, W), y0 = 4 * th + 1, y1 = min(4 * th + 4, H);
            const int cx0 = tw == 0 ? 0 : x0, cx1 = tw == TW - 1 ? W + 1 : x1;
            if (th == 0)
                for (int xx = cx0; xx <= cx1; ++xx) put(cbase + xx, 0.0);
            if (th == TH - 1)
                for (int xx = cx0; xx <= cx1; ++xx) put(cbase + (int64_t)(H + 1) * R + xx, 0.0);
            if (tw == 0)
                for (int yy = y0; yy <= y1; ++yy) put(cbase + (int64_t)yy * R, 0.0);
            if (tw == TW - 1)
                for (int yy = y0; yy <= y1; ++yy) put(cbase + (int64_t)yy * R + W + 1, 0.0);
        }
        __syncthreads();
    }
}

template <int CI, int CO>
void launch_wino_fused(const rvc_wino64_args* a, int TW, int P, int64_t x_bs, int64_t y_bs, int64_t r_bs,
                       hipStream_t s) {
    constexpr int NT = 64 * (CO == 16 ? 4 : 6);
    hipLaunchKernelGGL((wino_fused64_kernel<CI, CO>), dim3(cdiv(P, 16), (unsigned)a->B), dim3(NT), 36 * 256 * 8, s,
                       a->x, a->v, a->bias, a->res, a->y_f32 ? nullptr : (double*)a->y,
                       a->y_f32 ? (float*)a->y : nullptr, (int)a->H, (int)a->W, TW, P, a->out_act, x_bs, y_bs, r_bs);
}

bool wino_fused_shape(int64_t Ci, int64_t Co) {
    return (Ci == 16 || Ci == 32 || Ci == 64) && (Co == 16 || Co == 32);
}
}  // namespace

// ---------------------------------------------------------------- f64 bidirectional GRU recurrence
// rmvpe.hip's bigru_kernel in f64: 16 workgroups per direction, 16 hidden units each, W_hh rows in registers
// (48 doubles per thread); h is exchanged every step as one 16-byte granule per unit {tag | lo, tag | hi}
// (each 8-byte half carries the step tag, so a read that straddles two steps is seen and retried), written and
// polled with one agent-coherent (sc1) dwordx4 access -- what the 8-byte atomics compile to, 16 bytes wide --
// double-buffered by step parity.  Every spin is bounded; a timeout sets *err and the kernel drains.
//
// The gate math is the step's critical path (scripts/bigru64_bench.hip: 1.45 of 3.3 us per step with ocml's f64
// exp / division / tanh), so: sigmoid(a) = 1 / (1 + e^-a) and tanh(a) = 1 - 2 / (1 + e^2a) on one short f64 exp
// (exp64: Cody-Waite reduction, degree-12 Taylor, ~1 ulp) and a Newton-refined reciprocal, and r and z are
// evaluated at once on two lanes of the unit's 16-lane group (lane 0: r, lane 1: z), n after r on lane 0.
constexpr int G_H = 256;

RVC_DEV double exp64(double x) {
    x = fmin(fmax(x, -700.0), 700.0);
    const double k = rint(x * 1.4426950408889634);
    double r = fma(-k, 6.93147180369123816490e-01, x);
    r = fma(-k, 1.90821492927058770002e-10, r);  // |r| <= 0.347
    double p = 2.08767569878680989792e-09;        // 1/12!
    p = fma(p, r, 2.50521083854417187751e-08);   // 1/11!
    p = fma(p, r, 2.75573192239858906526e-07);
    p = fma(p, r, 2.75573192239858906526e-06);
    p = fma(p, r, 2.48015873015873015873e-05);
    p = fma(p, r, 1.98412698412698412698e-04);
    p = fma(p, r, 1.38888888888888888889e-03);
    p = fma(p, r, 8.33333333333333333333e-03);
    p = fma(p, r, 4.16666666666666666667e-02);
    p = fma(p, r, 1.66666666666666666667e-01);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return ldexp(p, (int)k);
}

RVC_DEV double rcp64(double d) {  // 1 / d for d >= 1: hardware estimate + 2 Newton steps
    double y = __builtin_amdgcn_rcp(d);
    double e = fma(-d, y, 1.0);
    y = fma(y, e, y);
    e = fma(-d, y, 1.0);
    return fma(y, e, y);
}

// NWG workgroups per direction (16: 256 threads, 16 units each; 8: 512 threads, 32 units each -- half the CUs held
// for the whole recurrence; RVC_BIGRU64_WG=8).  Measured: 8 costs the clip stream 5 % (876 vs 921 xRT): 16.
template <int NWG>
__global__ __launch_bounds__(4096 / NWG) void bigru64_kernel(const double* gi, const double* whh, const double* bhh,
                                                             double* y, unsigned long long* gran, int* err, int64_t T,
                                                             unsigned spin_limit, int64_t gi_bs, int64_t y_bs,
                                                             int prio) {
    constexpr int UPW = G_H / NWG;  // hidden units per workgroup
    // the recurrence's waves first at their SIMDs' issue (s_setprio 3): they share CUs with the synthesizer's
    // blocks in the clip stream, and every step waits on the slowest of 32 workgroups (RVC_BIGRU64_PRIO=1;
    // measured neutral in the clip stream, 934 vs 932 xRT: off)
    if (prio) __builtin_amdgcn_s_setprio(3);
    gi += (int64_t)blockIdx.y * gi_bs;
    y += (int64_t)blockIdx.y * y_bs;
    gran += (int64_t)blockIdx.y * 2 * 2 * G_H * 2;
    const int d = blockIdx.x / NWG;
    const int j = blockIdx.x % NWG;
    const int tid = threadIdx.x;
    const int ul = tid >> 4, s = tid & 15;
    const int u = j * UPW + ul;
    __shared__ double hs[2][G_H];
    __shared__ int abort_flag;
    if (tid == 0) abort_flag = 0;
    const double* W = whh + (int64_t)d * 3 * G_H * G_H;
    double wr[16], wz[16], wn[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        wr[i] = W[(int64_t)u * G_H + 16 * s + i];
        wz[i] = W[(int64_t)(G_H + u) * G_H + 16 * s + i];
        wn[i] = W[(int64_t)(2 * G_H + u) * G_H + 16 * s + i];
    }
    // lane 0 of the group: r's input projection and bias (and n's); lane 1: z's
    const int gsel = s == 1 ? 1 : 0;
    const double bhg = bhh[d * 3 * G_H + gsel * G_H + u], bhn = bhh[d * 3 * G_H + 2 * G_H + u];
    const double* G = gi + (int64_t)d * 3 * G_H * T;
    unsigned long long* GR = gran + (int64_t)d * 2 * G_H * 2;  // [parity][unit][lo, hi]
    double hprev = 0.0;
    double gxg = 0.0, gxn = 0.0;  // the current step's input projections (lane 0: r and n, lane 1: z)
    if (s < 2) {
        const int64_t tau0 = d ? T - 1 : 0;
        gxg = G[(int64_t)(gsel * G_H + u) * T + tau0];
        gxn = G[(int64_t)(2 * G_H + u) * T + tau0];
    }
    if (tid < G_H) hs[0][tid] = 0.0;
    __syncthreads();
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    for (int64_t t = 0; t < T; ++t) {
        const int64_t tau = d ? T - 1 - t : t;
        const int cur = (int)(t & 1);
        if (t > 0) {
            if (tid < G_H) {  // (wave-uniform) one granule per thread of the first 4 waves
                const unsigned long long* g = GR + ((t - 1) & 1) * G_H * 2 + 2 * tid;
                u64x2 v;
                unsigned spins = 0;
                for (;;) {
                    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(g) : "memory");
                    if ((uint32_t)(v.x >> 32) == (uint32_t)t && (uint32_t)(v.y >> 32) == (uint32_t)t) break;
                    if (++spins > spin_limit) {
                        atomicExch(err, 1);
                        abort_flag = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                hs[cur][tid] = __hiloint2double((int)(uint32_t)v.y, (int)(uint32_t)v.x);
            }
            __syncthreads();
            if (abort_flag) break;
        }
        double nxg = 0.0, nxn = 0.0;
        if (s < 2 && t + 1 < T) {
            const int64_t tn = d ? T - 2 - t : t + 1;
            nxg = G[(int64_t)(gsel * G_H + u) * T + tn];
            nxn = G[(int64_t)(2 * G_H + u) * T + tn];
        }
        double pr = 0.0, pz = 0.0, pn = 0.0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const double h = hs[cur][16 * s + i];
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
        // lanes 0 / 1 of the group: r / z = sigmoid(gx + (W_h h + b_h)) in one evaluation
        const double sg = rcp64(1.0 + exp64(-(gxg + ((gsel ? pz : pr) + bhg))));
        const double zz = __shfl_down(sg, 1, 64);  // lane 0 <- lane 1's z
        if (s == 0) {
            const double n = 1.0 - 2.0 * rcp64(1.0 + exp64(2.0 * (gxn + sg * (pn + bhn))));
            const double h = (hprev - n) * zz + n;
            hprev = h;
            const unsigned long long tag = (unsigned long long)(uint32_t)(t + 1) << 32;
            unsigned long long* o = GR + (t & 1) * G_H * 2 + 2 * u;
            u64x2 gv;
            gv.x = tag | (uint32_t)__double2loint(h);
            gv.y = tag | (uint32_t)__double2hiint(h);
            asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(o), "v"(gv) : "memory");
            y[(int64_t)(d * G_H + u) * T + tau] = h;
        }
        gxg = nxg;
        gxn = nxn;
    }
}

// The recurrence in f32 behind the f64 interface (the default; RVC_BIGRU64_F32=0: bigru64_kernel, all f64): gi, W_hh, b_hh rounded to f32 on load, h in f32,
// y widened to f64.  The round-5 stage study (scripts/rmvpe_stage_prec.py, profiles/r5_rmvpe_stage_prec.json) put the
// f32 recurrence's decision noise at 1.8e-9 on the headline clip -- three orders below its smallest exact margin --
// where the input projection W_ih (2.4e-5) and every U-Net level (>= 4e-8) stay f64.  NWG workgroups per direction
// (4: 1024 threads, 64 units each, W_hh rows as 48 f32 registers per thread); with `spread`, the grid is 8 NWG blocks
// of which the NWG blocks b = d + 8 k (k < NWG) serve direction d and the rest leave at once: blocks b and b + 8 are
// dealt to the same XCD (MI355X_MICROARCH.md, dispatch; observed, speed only -- the hand-off is agent-scope either
// way).  8-byte {tag, f32} granules as rmvpe.hip's f32 kernel, double-buffered by step parity, bounded spins.
template <int NWG>
__global__ __launch_bounds__(4096 / NWG) void bigru_mx_kernel(const double* gi, const double* whh, const double* bhh,
                                                              double* y, unsigned long long* gran, int* err, int64_t T,
                                                              unsigned spin_limit, int64_t gi_bs, int64_t y_bs,
                                                              int spread) {
    constexpr int UPW = G_H / NWG;
    int d, j;
    if (spread) {
        const int slot = blockIdx.x & 7;
        if (slot >= 2) return;
        d = slot;
        j = blockIdx.x >> 3;
    } else {
        d = blockIdx.x / NWG;
        j = blockIdx.x % NWG;
    }
    gi += (int64_t)blockIdx.y * gi_bs;
    y += (int64_t)blockIdx.y * y_bs;
    gran += (int64_t)blockIdx.y * 2 * 2 * G_H;
    const int tid = threadIdx.x;
    const int ul = tid >> 4, s = tid & 15;
    const int u = j * UPW + ul;
    __shared__ float hs[2][G_H];
    __shared__ int abort_flag;
    if (tid == 0) abort_flag = 0;
    const double* W = whh + (int64_t)d * 3 * G_H * G_H;
    float wr[16], wz[16], wn[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        wr[i] = (float)W[(int64_t)u * G_H + 16 * s + i];
        wz[i] = (float)W[(int64_t)(G_H + u) * G_H + 16 * s + i];
        wn[i] = (float)W[(int64_t)(2 * G_H + u) * G_H + 16 * s + i];
    }
    // lane 0 of the unit's group: r's input projection and bias (and n's); lane 1: z's -- r and z in one evaluation
    const int gsel = s == 1 ? 1 : 0;
    const float bhg = (float)bhh[d * 3 * G_H + gsel * G_H + u], bhn = (float)bhh[d * 3 * G_H + 2 * G_H + u];
    const double* G = gi + (int64_t)d * 3 * G_H * T;
    unsigned long long* GR = gran + (int64_t)d * 2 * G_H;
    float hprev = 0.f;
    float gxg = 0.f, gxn = 0.f;
    if (s < 2) {
        const int64_t tau0 = d ? T - 1 : 0;
        gxg = (float)G[(int64_t)(gsel * G_H + u) * T + tau0];
        gxn = (float)G[(int64_t)(2 * G_H + u) * T + tau0];
    }
    if (tid < G_H) hs[0][tid] = 0.f;
    __syncthreads();
    for (int64_t t = 0; t < T; ++t) {
        const int64_t tau = d ? T - 1 - t : t;
        const int cur = (int)(t & 1);
        if (t > 0) {
            if (tid < G_H) {  // (wave-uniform) one granule per thread of the first 4 waves
                unsigned long long* g = GR + ((t - 1) & 1) * G_H + tid;
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
            }
            __syncthreads();
            if (abort_flag) break;
        }
        float nxg = 0.f, nxn = 0.f;
        if (s < 2 && t + 1 < T) {
            const int64_t tn = d ? T - 2 - t : t + 1;
            nxg = (float)G[(int64_t)(gsel * G_H + u) * T + tn];
            nxn = (float)G[(int64_t)(2 * G_H + u) * T + tn];
        }
        // two interleaved FMA chains per gate (half the dependent latency of one 16-deep chain)
        float pr = 0.f, pz = 0.f, pn = 0.f, qr = 0.f, qz = 0.f, qn = 0.f;
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            const float h0 = hs[cur][16 * s + i], h1 = hs[cur][16 * s + i + 1];
            pr = fmaf(wr[i], h0, pr);
            pz = fmaf(wz[i], h0, pz);
            pn = fmaf(wn[i], h0, pn);
            qr = fmaf(wr[i + 1], h1, qr);
            qz = fmaf(wz[i + 1], h1, qz);
            qn = fmaf(wn[i + 1], h1, qn);
        }
        pr += qr;
        pz += qz;
        pn += qn;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
            pr += __shfl_xor(pr, o, 64);
            pz += __shfl_xor(pz, o, 64);
            pn += __shfl_xor(pn, o, 64);
        }
        // hardware exp2 / reciprocal (~1 ulp each): far inside the stage's noise budget
        const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-(gxg + ((gsel ? pz : pr) + bhg))));
        const float zz = __shfl_down(sg, 1, 64);  // lane 0 <- lane 1's z
        if (s == 0) {
            const float n = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * (gxn + sg * (pn + bhn))));
            const float h = (hprev - n) * zz + n;
            hprev = h;
            const unsigned long long gv = ((unsigned long long)(uint32_t)(t + 1) << 32) | __float_as_uint(h);
            __hip_atomic_store(GR + (t & 1) * G_H + u, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            y[(int64_t)(d * G_H + u) * T + tau] = (double)h;
        }
        gxg = nxg;
        gxn = nxn;
    }
}

constexpr int G_B_MAX = 16;  // sequences per launch (32 co-resident workgroups each)

}  // namespace

extern "C" int64_t rvc_conv64_workspace_bytes(const rvc_conv64_args* a) {
    C64 p;
    int tile;
    dim3 grid;
    size_t lds;
    if (plan64(a, p, tile, grid, lds) != RVC_OK) return -1;
    return p.ksplit > 1 ? (int64_t)p.ksplit * p.B * p.Co * p.nout * 8 : 0;
}

extern "C" int rvc_conv64_set_plan(int tile, int ksplit, int compact) {
    RVC_CHECK_ARG(tile >= -1 && tile < N_TILES64 && ksplit >= -1 && ksplit <= 32 && compact >= -1 && compact <= 1,
                  "conv64_set_plan: tile %d (-1..%d), ksplit %d (-1..32), compact %d (-1..1)", tile, N_TILES64 - 1,
                  ksplit, compact);
    g_force_tile = tile;
    g_force_ks = ksplit;
    g_force_cmp = compact;
    return RVC_OK;
}

extern "C" int rvc_conv64_plan(const rvc_conv64_args* a, int* out) {
    C64 p;
    int tile;
    dim3 grid;
    size_t lds;
    const int rc = plan64(a, p, tile, grid, lds);
    if (rc != RVC_OK) return rc;
    RVC_CHECK_ARG(out, "conv64_plan: null out");
    out[0] = tile;
    out[1] = p.ksplit;
    out[2] = p.cw != 0;
    out[3] = (int)(grid.x * grid.y * grid.z);
    return RVC_OK;
}

extern "C" int rvc_conv64(const rvc_conv64_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream) {
    C64 p;
    int tile;
    dim3 grid;
    size_t lds;
    const int rc = plan64(a, p, tile, grid, lds);
    if (rc != RVC_OK) return rc;
    if (p.ksplit > 1) {
        const int64_t need = (int64_t)p.ksplit * p.B * p.Co * p.nout * 8;
        RVC_CHECK_ARG(ws && ws_bytes >= need, "conv64: split-K needs %lld B of workspace (got %lld)", (long long)need,
                      (long long)ws_bytes);
        p.ws = (double*)ws;
    }
    hipStream_t s = (hipStream_t)stream;
    // RVC_F64_ABLATE bit 1: no conv launches (timing ablation only: the output is then wrong)
    static const int ablate = getenv("RVC_F64_ABLATE") ? atoi(getenv("RVC_F64_ABLATE")) : 0;
    if (ablate & 2) return RVC_OK;
    launch64(tile, p, grid, lds, s);
    RVC_HIP(hipGetLastError());
    if (p.ksplit > 1) {
        hipLaunchKernelGGL(conv64_splitk_reduce, dim3(cdiv(p.nout, 256), (unsigned)p.Co, (unsigned)p.B), dim3(256), 0,
                           s, p);
        RVC_HIP(hipGetLastError());
    }
    return RVC_OK;
}

extern "C" int rvc_mel_image64(const double* mel, double* img, int64_t B, int64_t M, int64_t F, int64_t Tp,
                               double scale, double shift, int64_t mel_bstride, int64_t img_bstride,
                               rvc_stream_t stream) {
    RVC_CHECK_ARG(mel && img && B > 0 && M > 0 && M <= 1024 && F > 1 && Tp >= F && Tp - F < F, "mel_image64: bad args");
    RVC_CHECK_ARG(B == 1 || (mel_bstride >= M * F && img_bstride >= (Tp + 2) * (M + 2)), "mel_image64: bad strides");
    hipLaunchKernelGGL(mel_image64_kernel, dim3((unsigned)Tp, (unsigned)B), dim3((unsigned)((M + 63) / 64 * 64)), 0,
                       (hipStream_t)stream, mel, img, (int)M, F, Tp, scale, shift, mel_bstride, img_bstride);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_avgpool2_64(const double* in, double* out, int64_t B, int64_t C, int64_t H, int64_t W,
                               int64_t in_bstride, int64_t out_bstride, rvc_stream_t stream) {
    RVC_CHECK_ARG(in && out && B > 0 && C > 0 && H >= 2 && W >= 2, "avgpool2_64: bad args");
    RVC_CHECK_ARG(B == 1 || (in_bstride >= C * (H + 2) * (W + 2) && out_bstride >= C * (H / 2 + 2) * (W / 2 + 2)),
                  "avgpool2_64: bad strides");
    const int64_t n = C * (H / 2) * (W / 2);
    hipLaunchKernelGGL(avgpool2_64_kernel, dim3(cdiv(n, 256), (unsigned)B), dim3(256), 0, (hipStream_t)stream, in, out,
                       (int)C, (int)H, (int)W, in_bstride, out_bstride);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_interleave4_64(const double* phases, double* out, int64_t B, int64_t C, int64_t H, int64_t W,
                                  int64_t ph_bstride, int64_t out_bstride, rvc_stream_t stream) {
    RVC_CHECK_ARG(phases && out && B > 0 && C > 0 && H > 0 && W > 0, "interleave4_64: bad args");
    RVC_CHECK_ARG(B == 1 || (ph_bstride >= 4 * C * (H + 2) * (W + 2) && out_bstride >= C * (2 * H + 2) * (2 * W + 2)),
                  "interleave4_64: bad strides");
    const int64_t n = C * 4 * H * W;
    hipLaunchKernelGGL(interleave4_64_kernel, dim3(cdiv(n, 256), (unsigned)B), dim3(256), 0, (hipStream_t)stream,
                       phases, out, (int)C, (int)H, (int)W, ph_bstride, out_bstride);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_img_to_seq64(const double* img, double* x, int64_t B, int64_t C, int64_t H, int64_t W,
                                int64_t img_bstride, int64_t x_bstride, rvc_stream_t stream) {
    RVC_CHECK_ARG(img && x && B > 0 && B < 65536 && C > 0 && H > 0 && W > 0, "img_to_seq64: bad args");
    RVC_CHECK_ARG(B == 1 || (img_bstride >= C * (H + 2) * (W + 2) && x_bstride >= C * W * H),
                  "img_to_seq64: bad strides");
    hipLaunchKernelGGL(img_to_seq64_kernel, dim3(cdiv(H, 256), (unsigned)(C * W), (unsigned)B), dim3(256), 0,
                       (hipStream_t)stream, img, x, (int)C, H, (int)W, img_bstride, x_bstride);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" unsigned rvc_bigru_set_spin_limit(unsigned limit);

// per-thread override of the recurrence's arithmetic (rvc_bigru64_set_f32; -1 = RVC_BIGRU64_F32, default 1)
static thread_local int g_bigru64_f32 = -1;

extern "C" int rvc_bigru64_set_f32(int on) {
    g_bigru64_f32 = on < 0 ? -1 : (on ? 1 : 0);
    return RVC_OK;
}

extern "C" int rvc_bigru64_batched(const double* gi, int64_t gi_bs, const double* whh, const double* bhh, double* y,
                                   int64_t y_bs, void* gran_ws, int* err, int64_t B, int64_t T, rvc_stream_t stream) {
    RVC_CHECK_ARG(gi && whh && bhh && y && gran_ws && err && T > 0 && T < (1ll << 31) && B > 0, "bigru64: bad args");
    RVC_CHECK_ARG(B == 1 || (gi_bs >= 2 * 3 * G_H * T && y_bs >= 2 * G_H * T), "bigru64: batch strides too small");
    hipStream_t s = (hipStream_t)stream;
    const unsigned spin = rvc_bigru_set_spin_limit(0);
    // RVC_F64_ABLATE bit 0: a 1-step recurrence (timing ablation only: the output is then wrong)
    static const int ablate = getenv("RVC_F64_ABLATE") ? atoi(getenv("RVC_F64_ABLATE")) : 0;
    if (ablate & 1) T = 1;
    for (int64_t b0 = 0; b0 < B; b0 += G_B_MAX) {
        const int64_t nb = B - b0 < G_B_MAX ? B - b0 : G_B_MAX;
        RVC_HIP(hipMemsetAsync(gran_ws, 0, (size_t)nb * RVC_BIGRU64_GRAN_BYTES, s));
        static const int nwg_env = getenv("RVC_BIGRU64_WG") ? atoi(getenv("RVC_BIGRU64_WG")) : 16;
        static const int nwg = nwg_env == 8 || nwg_env == 4 ? nwg_env : 16;
        static const int prio = getenv("RVC_BIGRU64_PRIO") ? atoi(getenv("RVC_BIGRU64_PRIO")) : 0;
        // the f32 recurrence (bigru_mx_kernel): RVC_BIGRU64_F32=1, workgroups per direction RVC_BIGRU64_MXWG
        // (4 / 8 / 16), XCD-spread placement RVC_BIGRU64_SPREAD (NWG 4 only)
        static const int f32_env = getenv("RVC_BIGRU64_F32") ? atoi(getenv("RVC_BIGRU64_F32")) : 1;
        const int f32 = g_bigru64_f32 >= 0 ? g_bigru64_f32 : f32_env;
        static const int mxwg_env = getenv("RVC_BIGRU64_MXWG") ? atoi(getenv("RVC_BIGRU64_MXWG")) : 16;
        static const int mxwg = mxwg_env == 8 || mxwg_env == 4 ? mxwg_env : 16;
        static const int spread = getenv("RVC_BIGRU64_SPREAD") ? atoi(getenv("RVC_BIGRU64_SPREAD")) : 0;
        if (f32) {
            unsigned long long* gw = (unsigned long long*)gran_ws;
            if (mxwg == 4 && spread)
                hipLaunchKernelGGL(bigru_mx_kernel<4>, dim3(32, (unsigned)nb), dim3(1024), 0, s, gi + b0 * gi_bs, whh,
                                   bhh, y + b0 * y_bs, gw, err, T, spin, gi_bs, y_bs, 1);
            else if (mxwg == 4)
                hipLaunchKernelGGL(bigru_mx_kernel<4>, dim3(8, (unsigned)nb), dim3(1024), 0, s, gi + b0 * gi_bs, whh,
                                   bhh, y + b0 * y_bs, gw, err, T, spin, gi_bs, y_bs, 0);
            else if (mxwg == 8)
                hipLaunchKernelGGL(bigru_mx_kernel<8>, dim3(16, (unsigned)nb), dim3(512), 0, s, gi + b0 * gi_bs, whh,
                                   bhh, y + b0 * y_bs, gw, err, T, spin, gi_bs, y_bs, 0);
            else
                hipLaunchKernelGGL(bigru_mx_kernel<16>, dim3(32, (unsigned)nb), dim3(256), 0, s, gi + b0 * gi_bs, whh,
                                   bhh, y + b0 * y_bs, gw, err, T, spin, gi_bs, y_bs, 0);
            RVC_HIP(hipGetLastError());
            continue;
        }
        if (nwg == 4)
            hipLaunchKernelGGL(bigru64_kernel<4>, dim3(2 * 4, (unsigned)nb), dim3(1024), 0, s, gi + b0 * gi_bs, whh, bhh,
                               y + b0 * y_bs, (unsigned long long*)gran_ws, err, T, spin, gi_bs, y_bs, prio);
        else if (nwg == 8)
            hipLaunchKernelGGL(bigru64_kernel<8>, dim3(2 * 8, (unsigned)nb), dim3(512), 0, s, gi + b0 * gi_bs, whh, bhh,
                               y + b0 * y_bs, (unsigned long long*)gran_ws, err, T, spin, gi_bs, y_bs, prio);
        else
            hipLaunchKernelGGL(bigru64_kernel<16>, dim3(2 * 16, (unsigned)nb), dim3(256), 0, s, gi + b0 * gi_bs, whh,
                               bhh, y + b0 * y_bs, (unsigned long long*)gran_ws, err, T, spin, gi_bs, y_bs, prio);
        RVC_HIP(hipGetLastError());
    }
    return RVC_OK;
}

// ---------------------------------------------------------------- Winograd F(4x4, 3x3) entry points
extern "C" int rvc_wino64_use(int64_t Ci, int64_t Co, int64_t H, int64_t W) {
    static const int on = getenv("RVC_RMVPE_WINO") ? atoi(getenv("RVC_RMVPE_WINO")) : 1;
    // images of fewer output tiles than this run direct (the 36 GEMMs get too narrow; RVC_RMVPE_WINO_MINP)
    static const int64_t minp = getenv("RVC_RMVPE_WINO_MINP") ? atoll(getenv("RVC_RMVPE_WINO_MINP")) : 90;
    if (!on) return 0;
    // the fused small-channel form only on request (RVC_RMVPE_WINO=3): measured no faster than the direct engine
    // (16 -> 16 at 3232 x 128: 74 us vs 70-80; 32 -> 32 at 1616 x 64: 99 vs 57-81; clip stream 921 vs 927 xRT)
    if (wino_fused_shape(Ci, Co)) return on == 3;
    if (Ci < 64 || Co < 64) return 0;
    return H <= 0 || W <= 0 || ((H + 3) / 4) * ((W + 3) / 4) >= minp;
}

extern "C" int rvc_wino64_weights(const double* w, double* v, int64_t Ci, int64_t Co, rvc_stream_t stream) {
    RVC_CHECK_ARG(w && v && Ci > 0 && Co > 0 && Ci * Co * 36 < (1ll << 31), "wino64_weights: bad args");
    hipLaunchKernelGGL(wino_w64_kernel, dim3(cdiv(Ci * Co, 256)), dim3(256), 0, (hipStream_t)stream, w, v, (int)Ci,
                       (int)Co);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

namespace {
struct Wino64 {
    int64_t P, TW, u_n, m_n;  // tiles, tile columns, U / M doubles per image
    rvc_conv64_args g;        // the 36-batch GEMM
};

int wino64_plan(const rvc_wino64_args* a, Wino64& w) {
    RVC_CHECK_ARG(a && a->x && a->v && a->y && a->B > 0 && a->Ci > 0 && a->Co > 0 && a->H > 0 && a->W > 0,
                  "wino64: bad args");
    w.TW = (a->W + 3) / 4;
    w.P = ((a->H + 3) / 4) * w.TW;
    w.u_n = 36 * a->Ci * w.P;
    w.m_n = 36 * a->Co * w.P;
    RVC_CHECK_ARG(a->B * w.u_n < (1ll << 40) && w.P < (1 << 30), "wino64: too large");
    memset(&w.g, 0, sizeof(w.g));
    w.g.w = a->v;
    w.g.B = a->B * 36;
    w.g.Ci = a->Ci;
    w.g.Co = a->Co;
    w.g.Lin = w.P;
    w.g.Lout = w.P;
    w.g.K = 1;
    w.g.out_act = RVC_ACT_NONE;
    w.g.w_bstride = a->Ci * a->Co;
    w.g.w_bmod = 36;
    w.g.x = a->v;  // placeholders for planning (the workspace pointers are set at launch)
    w.g.y = (void*)a->v;
    return RVC_OK;
}
}  // namespace

extern "C" int64_t rvc_wino64_workspace_bytes(const rvc_wino64_args* a) {
    Wino64 w;
    if (wino64_plan(a, w) != RVC_OK) return -1;
    if (wino_fused_shape(a->Ci, a->Co)) return 0;
    const int64_t g = rvc_conv64_workspace_bytes(&w.g);
    if (g < 0) return -1;
    return (a->B * (w.u_n + w.m_n)) * 8 + g;
}

extern "C" int rvc_wino64_conv(const rvc_wino64_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream) {
    Wino64 w;
    const int rc = wino64_plan(a, w);
    if (rc != RVC_OK) return rc;
    if (wino_fused_shape(a->Ci, a->Co)) {
        const int64_t img_i = a->Ci * (a->H + 2) * (a->W + 2), img_o = a->Co * (a->H + 2) * (a->W + 2);
        const int64_t x_bs = a->x_bstride ? a->x_bstride : img_i, y_bs = a->y_bstride ? a->y_bstride : img_o;
        const int64_t r_bs = a->res_bstride ? a->res_bstride : img_o;
        RVC_CHECK_ARG(a->B < 65536, "wino64: too many images");
        hipStream_t s = (hipStream_t)stream;
        const int TW = (int)w.TW, P = (int)w.P;
        if (a->Co == 16) {
            if (a->Ci == 16) launch_wino_fused<16, 16>(a, TW, P, x_bs, y_bs, r_bs, s);
            else if (a->Ci == 32) launch_wino_fused<32, 16>(a, TW, P, x_bs, y_bs, r_bs, s);
            else launch_wino_fused<64, 16>(a, TW, P, x_bs, y_bs, r_bs, s);
        } else {
            if (a->Ci == 16) launch_wino_fused<16, 32>(a, TW, P, x_bs, y_bs, r_bs, s);
            else if (a->Ci == 32) launch_wino_fused<32, 32>(a, TW, P, x_bs, y_bs, r_bs, s);
            else launch_wino_fused<64, 32>(a, TW, P, x_bs, y_bs, r_bs, s);
        }
        RVC_HIP(hipGetLastError());
        return RVC_OK;
    }
    const int64_t g = rvc_conv64_workspace_bytes(&w.g);
    RVC_CHECK_ARG(g >= 0, "wino64: GEMM plan failed");
    const int64_t need = a->B * (w.u_n + w.m_n) * 8 + g;
    RVC_CHECK_ARG(ws && ws_bytes >= need, "wino64: needs %lld B of workspace (got %lld)", (long long)need,
                  (long long)ws_bytes);
    double* u = (double*)ws;
    double* m = u + a->B * w.u_n;
    void* gws = g ? (void*)(m + a->B * w.m_n) : nullptr;
    hipStream_t s = (hipStream_t)stream;
    const int64_t img_i = a->Ci * (a->H + 2) * (a->W + 2), img_o = a->Co * (a->H + 2) * (a->W + 2);
    const int64_t x_bs = a->x_bstride ? a->x_bstride : img_i, y_bs = a->y_bstride ? a->y_bstride : img_o;
    const int64_t r_bs = a->res_bstride ? a->res_bstride : img_o;
    RVC_CHECK_ARG(a->B < 65536 && a->Ci < 65536 && a->Co < 65536, "wino64: too many images / channels");
    const int RT = wino_rt((int)a->W);
    const unsigned nband = cdiv((a->H + 3) / 4, RT);
    const size_t lds_out = (size_t)(4 * RT) * (4 * w.TW) * 8;
    RVC_CHECK_ARG(lds_out <= 64 * 1024, "wino64: image too wide (W %lld)", (long long)a->W);
    hipLaunchKernelGGL(wino_in64_kernel, dim3(cdiv(w.P, 64), (unsigned)a->Ci, (unsigned)a->B), dim3(64), 0, s, a->x, u,
                       (int)a->Ci, (int)a->H, (int)a->W, (int)w.TW, (int)w.P, x_bs, w.u_n);
    RVC_HIP(hipGetLastError());
    w.g.x = u;
    w.g.y = m;
    w.g.x_bstride = a->Ci * w.P;
    w.g.y_bstride = a->Co * w.P;
    const int rg = rvc_conv64(&w.g, gws, g, stream);
    if (rg != RVC_OK) return rg;
    hipLaunchKernelGGL(wino_out64_kernel, dim3(nband, (unsigned)a->Co, (unsigned)a->B), dim3(256), lds_out, s, m,
                       a->y_f32 ? nullptr : (double*)a->y, a->y_f32 ? (float*)a->y : nullptr, a->bias, a->res,
                       (int)a->Co, (int)a->H, (int)a->W, (int)w.TW, (int)w.P, RT, a->out_act, w.m_n, y_bs, r_bs);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
