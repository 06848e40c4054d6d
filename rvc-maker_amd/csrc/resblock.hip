// Fused HiFiGAN ResBlock pair on the split-bf16 matrix cores:
//     y (+)= x + c2(lrelu(c1(lrelu(x), dilation d)))        (residuals.py:22-44, one (convs1[i], convs2[i]) pair)
// for the generator's small-channel stages (C = 32, 64: 13 of its 28.6 ms in the unfused engine, where a
// 32-channel conv is a GEMM only 96-352 deep and every launch pays its staging, epilogue and HBM latency).
//
// One persistent workgroup per CU walks time tiles of N outputs.  The tile's input span (N + halo) is
// staged ONCE into LDS as lrelu'd split-bf16 planes, c1's output T (N + K - 1 columns, lrelu'd, zero
// outside [0, L) = c2's zero padding) stays in LDS as split planes, and c2 reads it from there: the
// intermediate never touches HBM and each pair reads x once and writes y once.
//
// Roles (12 waves): 8 compute waves (row groups x column groups, 2 x 2 fragments each, so every B
// fragment read from LDS feeds 2 x NP MFMAs; weights streamed per lane from the x6 fragment image through
// an L2 prefetch ring that runs on across phases and tiles), 4 loader waves that fetch the NEXT tile's raw
// x into registers while the current tile's c1 runs, write it (lrelu'd, split) into X while c2 runs, and
// its raw residual rows into R at the next tile start.
// Two barriers per tile:  S0 (X of tile k staged) -> c1 -> T written -> S1 -> c2 -> S0 of tile k+1.
//
// Summation order, pass order and epilogue order are those of conv_x6_kernel (chunk-major (chunk, tap)
// k-steps; hH hM mH hL mM lH; acc + bias, + residual, + accumulate), so the result is bit-identical to the
// two-launch form.
#include "rvc_common.h"
#include "x6_common.h"
#include <stdlib.h>

namespace {

struct RbParams {
    const float* x;    // [B][C][L] chain state in (also the residual)
    float* y;          // [B][C][L] out (accumulated into when accumulate)
    const uint4* w1x;  // c1 split-bf16 image [K][C/32][nmf][3][64]
    const uint4* w2x;  // c2 image
    const float* b1;
    const float* b2;
    int L, K, dil, nmf1, nmf2, accumulate;
    int B;             // clips: tiles are numbered clip-major, tile g = clip g / ntc, time tile g % ntc
    float slope;
    int ylds;          // split-fp16 at C <= 64: c2's outputs go through R in LDS, the loader waves store them (RB_YLDS)
#if RVC_CONV_STAMPS
    unsigned long long* stamps;  // diagnostic build only: [block][RB_STAMP_W] s_memtime stamps (rvc_resblock_set_stamps)
    int64_t stamp_blocks;
#endif
};

// In-kernel stamps (diagnostic build -DRVC_CONV_STAMPS=1 only; scripts/rb_stamps.py): compute wave 0 and the first
// loader wave record s_memtime at each tile's phase boundaries into a buffer of their own (never an output), one lane,
// vector stores.  Per block (RB_STAMP_W words), tile k < RB_STAMP_NT at 8 k + : 0 S0 passed (tile start), 1 c1's last
// k-step issued, 2 B_T passed (split-fp16: T's |max| agreed), 3 S1 passed (T written), 4 c2's last k-step issued,
// 5 c2 epilogue issued, 6 loader: tile k+1's loads issued, 7 loader: tile k+1 staged into X; then 248 block start,
// 249 HW_ID, 250 XCC_ID, 251 tiles, 252 memrealtime at start, 253 compute done.
#ifndef RVC_CONV_STAMPS
#define RVC_CONV_STAMPS 0
#endif
constexpr int RB_STAMP_W = 256, RB_STAMP_NT = 31;
#if RVC_CONV_STAMPS
#define RB_STAMP(slot, val)                                                                       \
    do {                                                                                           \
        if (p.stamps && lane == 0 && (int64_t)blockIdx.x < p.stamp_blocks && (slot) < RB_STAMP_W) \
            p.stamps[(int64_t)blockIdx.x * RB_STAMP_W + (slot)] = (val);                           \
    } while (0)
#else
#define RB_STAMP(slot, val) \
    do {                    \
    } while (0)
#endif
#define RB_NOW() ((unsigned long long)__builtin_amdgcn_s_memtime())
static thread_local int g_rb_ylds = -1;  // rvc_resblock_set_ylds (-1 = RVC_RB_YLDS, default on)
#if RVC_CONV_STAMPS
unsigned long long* g_rb_stamps = nullptr;
int64_t g_rb_stamp_blocks = 0;
#endif

#ifndef RB_YREG
#define RB_YREG 1  // accumulate operands loaded at S1 into registers (else in the epilogue)
#endif
#ifndef RB_BPIN
#define RB_BPIN 1  // next fragment's B reads pinned ahead of this one's MFMAs (rb_bench: pairs -3.5 %)
#endif
#ifndef RB_FM_
#define RB_FM_ 1
#define RB_FN_ 4
#endif
constexpr int RB_FM = RB_FM_;  // row fragments per compute wave
constexpr int RB_FN = RB_FN_;  // column fragments per compute wave
constexpr int RB_MAXSPAN = 64; // (K - 1) * dil bound (generator: 10 * 5 = 50)

template <int C, bool WIDE = false>
struct RbGeom {
    // C = 128 (round 4): 2 row fragments per compute wave, so the 8 waves are 4 row groups x 2 column groups and
    // a tile is 112 outputs (not 48); its residual rows are read from x in the epilogue instead of LDS (the X and
    // T tiles alone take 157 KB at 2 split planes), and only the 1- and 2-plane pass sets fit (<= 3 passes)
    // WIDE (C = 64, round 6): the same 2 row fragments per wave -- 2 row groups x 4 column groups, 240 outputs per
    // tile (not 112) -- so each B fragment read from LDS feeds twice the MFMAs (at 1 row fragment the 8 waves' B reads,
    // 64 KB per k-step, outran the LDS's 128 B/clk: c1 / c2 ran at ~45 % of their MFMA bound, rb_stamps r6a) and the
    // per-tile barriers / epilogues are amortised over twice the outputs; the residual from x as at C = 128
    static constexpr int FM = (C >= 128 || WIDE) ? 2 : RB_FM;
    static constexpr bool RLDS = C <= 64 && !WIDE;  // residual rows staged in LDS
    static constexpr int RF = C / 16;            // row fragments
    static constexpr int NCH = C / 32;           // 32-channel chunks
    static constexpr int RG = RF / FM;           // row groups
    static constexpr int CG = 8 / RG;            // column groups (RG x CG = 8 compute waves)
    static constexpr int NF1 = CG * RB_FN;       // c1 column fragments: T holds 16 NF1 positions
    static constexpr int NF2 = NF1 - 1;          // c2 column fragments
    static constexpr int N = 16 * NF2;           // outputs per tile (240 at C = 32, 112 at C = 64)
    static constexpr int TW = 16 * NF1;
    static constexpr int RSTR = N + 4;           // residual row stride (floats): 4 rows apart = distinct banks
    static constexpr int NI = (NCH * (TW + RB_MAXSPAN) * 4 + 255) / 256;  // loader items per thread
};

// R buffers: C = 32 with 2 split planes (round 6) keeps two by tile parity, so the loader waves store tile k - 1's outputs
// (YLDS) after S1(k) instead of before the c1 epilogue's barrier -- there its 40 stores queued ahead of the next tile's
// 40 loads in vmcnt and the loaders reached B_T late (the K = 3 pair's critical path, rb_stamps r6f); 3 planes: no room
template <int C, int NP>
constexpr int rb_nr() { return C == 32 && NP == 3 ? 2 : 1; }

template <int C, int NP, bool WIDE = false>
size_t rb_lds_bytes(int K, int dil) {
    using G = RbGeom<C, WIDE>;
    constexpr int NPL = NP == 6 ? 3 : (NP == 3 ? 2 : 1);
    const int Wx = G::TW + (K - 1) * dil;
    return (size_t)G::NCH * (Wx + G::TW) * NPL * 64 + (G::RLDS ? (size_t)rb_nr<C, NP>() * C * G::RSTR * 4 : 0) + 64;  // + scales
}

// F16 (with NP = 3): split-fp16 operands (x6_common.h split2h).  The loader waves take each staged x tile's
// |max| (they hold the whole tile in registers) and publish it per wave in LDS (slots by tile parity); c1's
// epilogue takes the T tile's |max| over the 8 compute waves (one extra barrier per tile, B_T) before
// splitting T; the c1 / c2 epilogues undo the weight-row and tile scales (powers of 2: exact).
// x_ / y_: p.x / p.y again as __restrict__ kernel arguments (rb_check: x != y) -- so hipcc may issue the c2 epilogue's
// residual / accumulate loads from x / y ahead of its stores to y; through the struct's pointers it kept each load
// behind the previous store (32 dependent round trips per wave: 20k of a wide C = 64 tile's 85k cycles, r6e)
template <int C, int NP, bool F16, bool WIDE>
__global__ __launch_bounds__(768, 1) void resblock_x6_kernel(RbParams p, const float* __restrict__ x_,
                                                             float* __restrict__ y_) {
    using G = RbGeom<C, WIDE>;
    static_assert(!F16 || NP == 3, "split-fp16: 3 passes");
    constexpr int NPL = NP == 6 ? 3 : (NP == 3 ? 2 : 1);
    constexpr int N = G::N, TW = G::TW, NCH = G::NCH, NF1 = G::NF1, NF2 = G::NF2, RSTR = G::RSTR;
    constexpr int FM = G::FM, FN = RB_FN;
    constexpr bool YREG = RB_YREG && C <= 64 && !WIDE;  // 2 row fragments: no register room for the accumulate operands
    static_assert(G::RLDS || NP <= 3, "C = 128 / WIDE: at most 2 split planes fit LDS");
    extern __shared__ uint4 lds[];
    const int K = p.K, d = p.dil, L = p.L;
    const int hk = (K - 1) / 2;
    const int H = d * hk + hk;  // input halo per side
    const int Wx = TW + (K - 1) * d;
    uint4* Xs = lds;                          // [NCH][Wx][NPL][4]
    uint4* Ts = Xs + NCH * Wx * NPL * 4;      // [NCH][TW][NPL][4]
    float* Rs0 = reinterpret_cast<float*>(Ts + NCH * TW * NPL * 4);  // [NR][C][RSTR] (C <= 64)
    constexpr int NR = rb_nr<C, NP>();
    auto Rbuf = [&](int k) __attribute__((always_inline)) { return Rs0 + (NR == 2 ? (k & 1) * C * RSTR : 0); };
    float* xmax = Rs0 + (G::RLDS ? NR * C * RSTR : 0);  // F16: [2 tile parities][4 loader waves] x tile |max|
    float* tmaxs = xmax + 8;      // F16: [8 compute waves] T tile |max|
    const int ntc = (L + N - 1) / N;  // time tiles per clip
    const int ntiles = p.B * ntc;
    const int my_n = (int)blockIdx.x < ntiles ? (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave == 0) {
        RB_STAMP(248, RB_NOW());
        RB_STAMP(249, (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));   // HW_ID
        RB_STAMP(250, (unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)));  // XCC_ID
        RB_STAMP(251, (unsigned long long)my_n);
        RB_STAMP(252, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }

    if (wave >= 8) {
        // ---------------- loader waves.  Tile k+1's raw x is loaded into registers after S0(k) (while c1
        // runs), written to X as lrelu'd split planes after S1(k) (X free: c1 done), and its residual rows
        // to R after S0(k+1) (R free: tile k's c2 epilogue done), just before the registers are reloaded.
        const int ltid = threadIdx.x - 512;
        const int nitems = NCH * Wx * 4;
        float xr[G::NI][8];
        auto item = [&](int it, int& ch, int& g8, int& pos) __attribute__((always_inline)) {
            int idx = ltid + 256 * it;
            idx = idx < nitems ? idx : nitems - 1;
            ch = idx / (Wx * 4);
            const int rem = idx - ch * Wx * 4;
            g8 = rem / Wx;
            pos = rem - g8 * Wx;
        };
        auto xload = [&](int tile) __attribute__((always_inline)) {
            const int cb = tile / ntc;
            const int base = (tile - cb * ntc) * N - H;
            const float* xb = x_ + (int64_t)cb * C * L;
#pragma unroll
            for (int it = 0; it < G::NI; ++it) {
                int ch, g8, pos;
                item(it, ch, g8, pos);
                int q = base + pos;
                q = q < 0 ? 0 : (q >= L ? L - 1 : q);
                const float* src = xb + (int64_t)(ch * 32 + g8 * 8) * L + q;
#pragma unroll
                for (int e = 0; e < 8; ++e) xr[it][e] = src[(int64_t)e * L];
            }
        };
        float sc = 1.f;  // F16: the staged tile's activation scale
        auto publish_max = [&](int par) __attribute__((always_inline)) {  // F16: this wave's |max| of the tile
            float m = 0.f;
#pragma unroll
            for (int it = 0; it < G::NI; ++it)
#pragma unroll
                for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(xr[it][e]));
            m = wave_max(m);
            if (lane == 0) xmax[par * 4 + wave - 8] = m;
        };
        auto take_scale = [&](int par) __attribute__((always_inline)) {
            sc = ldexpf(1.f, f16_exp(fmaxf(fmaxf(xmax[par * 4], xmax[par * 4 + 1]),
                                           fmaxf(xmax[par * 4 + 2], xmax[par * 4 + 3]))));
        };
        auto xstore = [&](int tile) __attribute__((always_inline)) {
            const int base = (tile % ntc) * N - H;
#pragma unroll
            for (int it = 0; it < G::NI; ++it) {
                if (ltid + 256 * it < nitems) {
                    int ch, g8, pos;
                    item(it, ch, g8, pos);
                    const int q = base + pos;
                    const bool ok = q >= 0 && q < L;
                    uint32_t hw[4], mw[4], lw[4];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) {
                        float v2[2];
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const float v = ok ? xr[it][2 * e2 + u] : 0.f;
                            v2[u] = F16 ? (v >= 0.f ? v : v * p.slope) * sc : (v >= 0.f ? v : v * p.slope);
                        }
                        if constexpr (F16) split2h_pk(v2[0], v2[1], hw[e2], mw[e2]);
                        else split3_pk(v2[0], v2[1], hw[e2], mw[e2], lw[e2]);
                    }
                    uint4* dst = Xs + ch * Wx * NPL * 4;
                    dst[x_slot<NPL>(pos, 0, g8)] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                    if constexpr (NPL >= 2) dst[x_slot<NPL>(pos, 1, g8)] = make_uint4(mw[0], mw[1], mw[2], mw[3]);
                    if constexpr (NPL >= 3) dst[x_slot<NPL>(pos, 2, g8)] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                }
            }
        };
        auto rstore = [&](float* Rs) __attribute__((always_inline)) {  // raw residual rows of the staged tile
            if constexpr (!G::RLDS) return;
#pragma unroll
            for (int it = 0; it < G::NI; ++it) {
                if (ltid + 256 * it < nitems) {
                    int ch, g8, pos;
                    item(it, ch, g8, pos);
                    const int rc = pos - H;
                    if (rc >= 0 && rc < N) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) Rs[(ch * 32 + g8 * 8 + e) * RSTR + rc] = xr[it][e];
                    }
                }
            }
        };
        if (my_n > 0) xload(blockIdx.x);
        if constexpr (F16) {
            if (my_n > 0) publish_max(0);
            __syncthreads();  // B_pre: tile 0's x max published
            take_scale(0);
        }
        // YLDS: tile k's finished outputs sit in R (the compute waves' c2 epilogue wrote them in place of the residual
        // rows) until S0(k + 1); each loader thread stores exactly the R elements its own items cover and then writes
        // its next residual values to those same elements (no hazard between threads), rows coalesced over the lanes
        auto ystore = [&](int tile, const float* Rs) __attribute__((always_inline)) {
            if constexpr (G::RLDS && F16) {
                const int cb = tile / ntc;
                const int n0 = (tile - cb * ntc) * N;
                float* yb = y_ + (int64_t)cb * C * L;
                // (not unrolled over the items: unrolled, hipcc batched every item's LDS reads and store addresses and
                // the loader registers set the kernel's count -- 51 spilled VGPRs at C = 64)
#pragma unroll 1
                for (int it = 0; it < G::NI; ++it) {
                    if (ltid + 256 * it < nitems) {
                        int ch, g8, pos;
                        item(it, ch, g8, pos);
                        const int rc = pos - H;
                        if (rc >= 0 && rc < N && n0 + rc < L) {
                            const int row0 = ch * 32 + g8 * 8;
                            float v[8];
#pragma unroll
                            for (int e = 0; e < 8; ++e) v[e] = Rs[(row0 + e) * RSTR + rc];
                            float* dst = yb + (int64_t)row0 * L + n0 + rc;
#pragma unroll
                            for (int e = 0; e < 8; ++e) dst[(int64_t)e * L] = v[e];
                        }
                    }
                }
            }
        };
        const bool ylds = G::RLDS && F16 && p.ylds;  // block-uniform
        const bool ylate = ylds && NR == 2 && p.ylds == 2;  // two R buffers: tile k - 1's stores after S1(k)
        if (my_n > 0) xstore(blockIdx.x);
        for (int k = 0; k < my_n; ++k) {
            __syncthreads();  // S0(k): X(k) staged; R free (YLDS: R holds tile k - 1's outputs)
            if (ylds && !ylate && k > 0) ystore(blockIdx.x + (k - 1) * gridDim.x, Rbuf(k - 1));
            rstore(Rbuf(k));  // R(k) from the registers still holding tile k
            const bool more = k + 1 < my_n;
            // unconditional (the last tile reloads itself): every path issues the same loads, which keeps
            // hipcc's vmcnt bookkeeping exact across the loop (a guarded load made it wait vmcnt(0))
            xload(blockIdx.x + (more ? k + 1 : k) * gridDim.x);
            if (wave == 8 && k < RB_STAMP_NT) RB_STAMP(8 * k + 6, RB_NOW());
            if constexpr (F16) {
                __syncthreads();  // B_T(k): the compute waves' T max (c1 epilogue)
                if (more) publish_max((k + 1) & 1);
            }
            __syncthreads();  // S1(k): c1 of tile k done -> X free
            if constexpr (F16) take_scale((k + 1) & 1);
            if (more) xstore(blockIdx.x + (k + 1) * gridDim.x);
            // two R buffers: tile k - 1's outputs (its buffer is rewritten only by rstore(k + 1), after S0(k + 1))
            if (ylate && k > 0) ystore(blockIdx.x + (k - 1) * gridDim.x, Rbuf(k - 1));
            if (wave == 8 && k < RB_STAMP_NT) RB_STAMP(8 * k + 7, RB_NOW());
        }
        if (ylds) {
            __syncthreads();  // S_end: the last tile's outputs in R
            if (my_n > 0) ystore(blockIdx.x + (my_n - 1) * gridDim.x, Rbuf(my_n - 1));
        }
        return;
    }

    // ---------------- compute waves: row group rg (FM row fragments), column group cg (FN fragments)
    const int rg = wave % G::RG, cg = wave / G::RG;
    const int ln = lane & 15, lg = lane >> 4;
    const int SPH = NCH * K;      // k-steps per phase
    const int SPT = 2 * SPH;      // per tile
    const int S_end = my_n * SPT;
    // weight fragments of one k-step: conv two (c2) or c1, 32-channel chunk ch, tap t
    auto aload = [&](bool two, int ch, int t, uint4 (&a)[NPL][FM]) __attribute__((always_inline)) {
        const uint4* img = two ? p.w2x : p.w1x;
        const int nmf = two ? p.nmf2 : p.nmf1;
        const int frag = __builtin_amdgcn_readfirstlane((t * NCH + ch) * nmf + rg * FM);
        const uint4* src = img + (int64_t)frag * 3 * 64;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int q = 0; q < NPL; ++q) a[q][i] = src[(i * 3 + q) * 64 + lane];
    };
    floatx4 acc[FM][FN];
    // one k-step: B fragments from the LDS image (X for c1 with tap stride d, T for c2), NP passes
    auto compute = [&](const uint4* buf, int tof, int nfrag, const uint4 (&a)[NPL][FM]) __attribute__((always_inline)) {
        auto bload = [&](int j, uint4 (&bq)[NPL]) __attribute__((always_inline)) {
            const int pos = (cg * FN + j) * 16 + ln + tof;
#pragma unroll
            for (int q = 0; q < NPL; ++q) bq[q] = buf[x_slot<NPL>(pos, q, lg)];
        };
        uint4 bb[2][NPL];
        bload(0, bb[0]);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            if (j + 1 < FN && cg * FN + j + 1 < nfrag) bload(j + 1, bb[(j + 1) & 1]);
            if constexpr (RB_BPIN) __builtin_amdgcn_sched_barrier(0);
            if (cg * FN + j < nfrag) {
                const uint4 (&bq)[NPL] = bb[j & 1];
                constexpr int PA[6] = {0, 0, 1, 0, 1, 2};
                constexpr int PB[6] = {0, 1, 0, 2, 1, 0};
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
    // weight prefetch depth (k-steps): as many as fit the register budget of 3 waves per SIMD
#ifndef RB_PD3
#define RB_PD3 3
#endif
#ifndef RB_PD2
#define RB_PD2 2
#endif
    constexpr int PD = C >= 128 ? (NPL == 2 ? 1 : 2) : (NPL == 3 ? RB_PD3 : (NPL == 2 ? RB_PD2 : 4));
    constexpr int NB = PD + 1;            // ring slots: k-step S uses slot S % NB (compile-time below)
    uint4 abuf[NB][NPL][FM];
    // k-step decode by counters stepped once per k-step (tap, chunk, conv), for the prefetch (PD ahead) and the
    // computing step.  Every prefetch is issued, past the block's last k-step too (the counters wrap inside
    // the images, so the address stays valid): under "if (S + PD < S_end)" hipcc merged the with- and
    // without-load paths and waited vmcnt(0) on the prefetch it had just issued before each k-step's MFMAs;
    // the per-step divisions it replaces were ~80 scalar instructions per 12 MFMAs.
    bool l_two = false;
    int l_ch = 0, l_t = 0;
    auto lstep = [&]() __attribute__((always_inline)) {
        if (++l_t == K) {
            l_t = 0;
            if (++l_ch == NCH) { l_ch = 0; l_two = !l_two; }
        }
    };
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        aload(l_two, l_ch, l_t, abuf[i]);
        lstep();
    }
    bool two = false;  // the computing k-step: conv, chunk, tap, and its tile
    int ch = 0, t = 0, k = 0;
    float yold[YREG ? FM : 1][YREG ? FN : 1][4];
    int n0 = 0;
    float* yb = y_;  // the current tile's clip
    const float* xres = x_;  // C = 128 / WIDE: the current tile's clip of x, the residual
    // F16: row reciprocal scales of both images (after each image), the x tile's and T tile's reciprocals
    const float* rs1 = reinterpret_cast<const float*>(p.w1x + (int64_t)K * NCH * p.nmf1 * 3 * 64);
    const float* rs2 = reinterpret_cast<const float*>(p.w2x + (int64_t)K * NCH * p.nmf2 * 3 * 64);
    float t_rs = 1.f;
    const bool ylds_c = G::RLDS && F16 && p.ylds;  // block-uniform
    if constexpr (F16) __syncthreads();  // B_pre
    // One loop over the block's k-steps (tile k: c1 steps [k SPT, k SPT + SPH), c2 steps after), unrolled by
    // the ring size so every ring slot index is a compile-time constant; the tile / phase seams (barriers,
    // epilogues) are uniform branches inside it and the weight prefetch runs on across them.
    for (int S0 = 0; S0 < S_end; S0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int S = S0 + u;
            aload(l_two, l_ch, l_t, abuf[(u + PD) % NB]);
            lstep();
            __builtin_amdgcn_sched_barrier(0);
            if (S < S_end) {
                const bool last_ch = ch == NCH - 1 && t == K - 1;  // the conv's last k-step
                if (!two && ch == 0 && t == 0) {  // ---- tile start: X of tile k staged
                    const int g = (int)blockIdx.x + k * (int)gridDim.x;
                    const int cb = g / ntc;
                    n0 = (g - cb * ntc) * N;
                    yb = y_ + (int64_t)cb * C * L;
                    xres = x_ + (int64_t)cb * C * L;
                    __syncthreads();  // S0(k)
                    if (RVC_CONV_STAMPS && wave == 0 && k < RB_STAMP_NT) RB_STAMP(8 * k, RB_NOW());
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
                }
                if (!two) compute(Xs + ch * (Wx * NPL * 4), t * d, NF1, abuf[u]);  // c1 over X, tap stride d
                else compute(Ts + ch * (TW * NPL * 4), t, NF2, abuf[u]);        // c2 over T
                if (!two && last_ch) {
                    // ---- c1 epilogue: + bias, lrelu, zero outside [0, L) (c2's padding) -> T (split planes)
                    if (RVC_CONV_STAMPS && wave == 0 && k < RB_STAMP_NT) RB_STAMP(8 * k + 1, RB_NOW());
                    float tsc = 1.f;
                    if constexpr (F16) {
                        // T values in place (unscaled), their |max| over the 8 compute waves, T's scale
                        const int par = k & 1;
                        const float x_rs = ldexpf(1.f, -f16_exp(fmaxf(fmaxf(xmax[par * 4], xmax[par * 4 + 1]),
                                                                      fmaxf(xmax[par * 4 + 2], xmax[par * 4 + 3]))));
                        float m = 0.f;
#pragma unroll
                        for (int i = 0; i < FM; ++i) {
                            const int m0 = (rg * FM + i) * 16 + 4 * lg;
#pragma unroll
                            for (int j = 0; j < FN; ++j) {
                                const int q = n0 - hk + (cg * FN + j) * 16 + ln;
                                const bool ok = q >= 0 && q < L;
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    float v = acc[i][j][r] * (rs1[m0 + r] * x_rs) + p.b1[m0 + r];
                                    v = v >= 0.f ? v : v * p.slope;
                                    acc[i][j][r] = ok ? v : 0.f;
                                    m = fmaxf(m, fabsf(acc[i][j][r]));
                                }
                            }
                        }
                        m = wave_max(m);
                        if (lane == 0) tmaxs[wave] = m;
                        __syncthreads();  // B_T(k)
                        if (RVC_CONV_STAMPS && wave == 0 && k < RB_STAMP_NT) RB_STAMP(8 * k + 2, RB_NOW());
                        float tm = 0.f;
#pragma unroll
                        for (int w = 0; w < 8; ++w) tm = fmaxf(tm, tmaxs[w]);
                        const int Et = f16_exp(tm);
                        tsc = ldexpf(1.f, Et);
                        t_rs = ldexpf(1.f, -Et);
                    }
#pragma unroll
                    for (int i = 0; i < FM; ++i) {
                        const int mf = rg * FM + i;
                        const int m0 = mf * 16 + 4 * lg;  // this lane's 4 rows
                        const int tch = (mf * 16) / 32, tg8 = (mf & 1) * 2 + (lg >> 1), thalf = lg & 1;
                        uint4* tb = Ts + tch * TW * NPL * 4;
#pragma unroll
                        for (int j = 0; j < FN; ++j) {
                            const int it = (cg * FN + j) * 16 + ln;  // T position
                            const int q = n0 - hk + it;
                            const bool ok = q >= 0 && q < L;
                            uint32_t hw[2], mw[2], lw[2];
#pragma unroll
                            for (int r2 = 0; r2 < 2; ++r2) {
                                float v2[2];
#pragma unroll
                                for (int e = 0; e < 2; ++e) {
                                    if constexpr (F16) {
                                        v2[e] = acc[i][j][2 * r2 + e] * tsc;
                                    } else {
                                        float v = acc[i][j][2 * r2 + e] + p.b1[m0 + 2 * r2 + e];
                                        v = v >= 0.f ? v : v * p.slope;
                                        v2[e] = ok ? v : 0.f;
                                    }
                                }
                                if constexpr (F16) split2h_pk(v2[0], v2[1], hw[r2], mw[r2]);
                                else split3_pk(v2[0], v2[1], hw[r2], mw[r2], lw[r2]);
                            }
                            reinterpret_cast<uint2*>(tb + x_slot<NPL>(it, 0, tg8))[thalf] = make_uint2(hw[0], hw[1]);
                            if constexpr (NPL >= 2)
                                reinterpret_cast<uint2*>(tb + x_slot<NPL>(it, 1, tg8))[thalf] = make_uint2(mw[0], mw[1]);
                            if constexpr (NPL >= 3)
                                reinterpret_cast<uint2*>(tb + x_slot<NPL>(it, 2, tg8))[thalf] = make_uint2(lw[0], lw[1]);
                            acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
                        }
                    }
                    __syncthreads();  // S1(k): T written; X free for the loaders
                    if (RVC_CONV_STAMPS && wave == 0 && k < RB_STAMP_NT) RB_STAMP(8 * k + 3, RB_NOW());
                    if (YREG && p.accumulate) {
#pragma unroll
                        for (int i = 0; i < FM; ++i)
#pragma unroll
                            for (int j = 0; j < FN; ++j) {
                                int q = n0 + (cg * FN + j) * 16 + ln;
                                q = q < L ? q : L - 1;
#pragma unroll
                                for (int r = 0; r < 4; ++r)
                                    yold[i][j][r] = yb[(int64_t)((rg * FM + i) * 16 + 4 * lg + r) * L + q];
                            }
                    }
                }
                if (two && last_ch) {
                    if (RVC_CONV_STAMPS && wave == 0 && k < RB_STAMP_NT) RB_STAMP(8 * k + 4, RB_NOW());
                    // ---- c2 epilogue: + bias, + residual (from R) (+ accumulate) -> y
                    if constexpr (!G::RLDS) {
                        // residual from x (C = 128, WIDE): per row fragment, bias in place, then every residual (and
                        // accumulate) load at once from clamped addresses, then the masked stores -- the same
                        // operations per element in the same order.  The per-element form (guarded load, add, store)
                        // kept each load behind the previous store's branch: 32 dependent round trips per wave, 20k
                        // of a wide C = 64 tile's 85k cycles (rb_stamps r6e)
#pragma unroll
                        for (int i = 0; i < FM; ++i) {
                            const int m0 = (rg * FM + i) * 16 + 4 * lg;
                            int qc[FN];
#pragma unroll
                            for (int j = 0; j < FN; ++j) {
                                const int q = n0 + (cg * FN + j) * 16 + ln;
                                qc[j] = q < L ? q : L - 1;
                            }
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const float f = F16 ? rs2[m0 + r] * t_rs : 1.f, bb = p.b2[m0 + r];
#pragma unroll
                                for (int j = 0; j < FN; ++j) acc[i][j][r] = (F16 ? acc[i][j][r] * f : acc[i][j][r]) + bb;
                            }
                            float tmp[FN][4];
#pragma unroll
                            for (int j = 0; j < FN; ++j)
#pragma unroll
                                for (int r = 0; r < 4; ++r) tmp[j][r] = xres[(int64_t)(m0 + r) * L + qc[j]];
#pragma unroll
                            for (int j = 0; j < FN; ++j)
#pragma unroll
                                for (int r = 0; r < 4; ++r) acc[i][j][r] = acc[i][j][r] + tmp[j][r];
                            if (p.accumulate) {
#pragma unroll
                                for (int j = 0; j < FN; ++j)
#pragma unroll
                                    for (int r = 0; r < 4; ++r)
                                        tmp[j][r] = YREG ? yold[i][j][r] : yb[(int64_t)(m0 + r) * L + qc[j]];
#pragma unroll
                                for (int j = 0; j < FN; ++j)
#pragma unroll
                                    for (int r = 0; r < 4; ++r) acc[i][j][r] += tmp[j][r];
                            }
#pragma unroll
                            for (int j = 0; j < FN; ++j) {
                                const int col = (cg * FN + j) * 16 + ln;
                                const int q = n0 + col;
                                if (cg * FN + j < NF2 && col < N && q < L) {
#pragma unroll
                                    for (int r = 0; r < 4; ++r) yb[(int64_t)(m0 + r) * L + q] = acc[i][j][r];
                                }
                            }
                        }
                    } else {
#pragma unroll
                    for (int i = 0; i < FM; ++i) {
                        const int m0 = (rg * FM + i) * 16 + 4 * lg;
#pragma unroll
                        for (int j = 0; j < FN; ++j) {
                            const int col = (cg * FN + j) * 16 + ln;
                            const int q = n0 + col;
                            if (cg * FN + j < NF2 && col < N && q < L) {
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    float v = (F16 ? acc[i][j][r] * (rs2[m0 + r] * t_rs) : acc[i][j][r]) + p.b2[m0 + r];
                                    if constexpr (G::RLDS) v = v + Rbuf(k)[(m0 + r) * RSTR + col];
                                    else v = v + xres[(int64_t)(m0 + r) * L + q];
                                    if (p.accumulate) v += YREG ? yold[i][j][r] : yb[(int64_t)(m0 + r) * L + q];
                                    if (G::RLDS && F16 && ylds_c) Rbuf(k)[(m0 + r) * RSTR + col] = v;  // the loaders store it
                                    else yb[(int64_t)(m0 + r) * L + q] = v;
                                }
                            }
                        }
                    }
                    }
                    if (RVC_CONV_STAMPS && wave == 0 && k < RB_STAMP_NT) RB_STAMP(8 * k + 5, RB_NOW());
                }
            }
            if (++t == K) {  // step the computing k-step: tap, chunk, conv, tile
                t = 0;
                if (++ch == NCH) {
                    ch = 0;
                    if (two) ++k;
                    two = !two;
                }
            }
        }
    }
    if (ylds_c) __syncthreads();  // S_end: the last tile's outputs are in R for the loader waves
    if (wave == 0) RB_STAMP(253, RB_NOW());
}

template <int C, int NP, bool F16 = false, bool WIDE = false>
int launch_rb(const RbParams& p, hipStream_t s) {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (ncu <= 0) ncu = 256;
    }
    const size_t lds = rb_lds_bytes<C, NP, WIDE>(p.K, p.dil);
    static bool attr = false;
    if (!attr) {
        RVC_HIP(hipFuncSetAttribute((const void*)resblock_x6_kernel<C, NP, F16, WIDE>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    // workgroups per CU: 1 = persistent; more = shorter tile runs that the dispatcher hands to CUs as they free
    // up (a CU held by a concurrent stream's kernel then delays fewer tiles)
    static const int per_cu = getenv("RVC_RB_PER_CU") ? atoi(getenv("RVC_RB_PER_CU")) : 1;
    const int ntiles = p.B * ((p.L + RbGeom<C, WIDE>::N - 1) / RbGeom<C, WIDE>::N);
    const int nwg = ncu * (per_cu > 0 ? per_cu : 1);
    hipLaunchKernelGGL((resblock_x6_kernel<C, NP, F16, WIDE>), dim3(ntiles < nwg ? ntiles : nwg), dim3(768), lds, s, p,
                       p.x, p.y);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

int rb_check(const rvc_resblock_args* a) {
    RVC_CHECK_ARG(a && a->x && a->y && a->w1x && a->w2x && a->b1 && a->b2, "resblock: null pointer");
    RVC_CHECK_ARG(a->C == 32 || a->C == 64 || a->C == 128, "resblock: C must be 32, 64 or 128 (got %lld)", (long long)a->C);
    RVC_CHECK_ARG(a->C != 128 || a->passes != 6, "resblock: C = 128 takes at most 2 split planes (passes 3, 1, F16X3)");
    RVC_CHECK_ARG(a->L > 0 && a->C * a->L < (1ll << 31), "resblock: bad length");
    RVC_CHECK_ARG(a->B >= 0 && (int64_t)(a->B > 1 ? a->B : 1) * ((a->L + 15) / 16) < (1ll << 31), "resblock: bad B");
    RVC_CHECK_ARG(a->K >= 1 && a->K % 2 == 1 && a->K <= 15 && a->dil >= 1 && (a->K - 1) * a->dil <= RB_MAXSPAN,
                  "resblock: odd K <= 15 with (K-1)*dil <= %d expected", RB_MAXSPAN);
    RVC_CHECK_ARG(a->passes == 6 || a->passes == 3 || a->passes == 1 || a->passes == RVC_ARITH_F16X3,
                  "resblock: passes must be 6, 3, 1 or RVC_ARITH_F16X3");
    RVC_CHECK_ARG(a->nmf1 * 16 >= a->C && a->nmf2 * 16 >= a->C, "resblock: weight image too small");
    RVC_CHECK_ARG(a->x != a->y, "resblock: x and y must not alias (tiles read x halos other tiles overwrite)");
    return RVC_OK;
}

// the wide C = 64 geometry (RbGeom WIDE) for the <= 2-plane pass sets (RVC_RB_WIDE64=0: 1 row fragment per wave, the
// round-5 form; rvc_resblock_set_wide64)
static thread_local int g_rb_wide64 = -1;
bool rb_wide64(int passes) {
    static const int env = getenv("RVC_RB_WIDE64") ? atoi(getenv("RVC_RB_WIDE64")) : 1;
    return (g_rb_wide64 >= 0 ? g_rb_wide64 : env) && passes != 6;
}

}  // namespace

extern "C" int64_t rvc_resblock_lds_bytes(int64_t C, int K, int dil, int passes) {
    if (C == 64 && rb_wide64(passes))
        return passes == 1 ? rb_lds_bytes<64, 1, true>(K, dil) : rb_lds_bytes<64, 3, true>(K, dil);
    if (passes == RVC_ARITH_F16X3) passes = 3;  // same planes
    if (C == 32) return passes == 6 ? rb_lds_bytes<32, 6>(K, dil) : passes == 3 ? rb_lds_bytes<32, 3>(K, dil)
                                                                                : rb_lds_bytes<32, 1>(K, dil);
    if (C == 64) return passes == 6 ? rb_lds_bytes<64, 6>(K, dil) : passes == 3 ? rb_lds_bytes<64, 3>(K, dil)
                                                                                : rb_lds_bytes<64, 1>(K, dil);
    if (C == 128) return passes == 6 ? -1 : passes == 3 ? rb_lds_bytes<128, 3>(K, dil) : rb_lds_bytes<128, 1>(K, dil);
    return -1;
}

extern "C" int rvc_resblock_pair(const rvc_resblock_args* a, rvc_stream_t stream) {
    const int rc = rb_check(a);
    if (rc != RVC_OK) return rc;
    RbParams p;
    p.x = a->x;
    p.y = a->y;
    p.w1x = (const uint4*)a->w1x;
    p.w2x = (const uint4*)a->w2x;
    p.b1 = a->b1;
    p.b2 = a->b2;
    p.L = (int)a->L;
    p.K = a->K;
    p.dil = a->dil;
    p.nmf1 = a->nmf1;
    p.nmf2 = a->nmf2;
    p.accumulate = a->accumulate;
    p.slope = a->slope;
    p.B = a->B > 1 ? a->B : 1;
    // the outputs through LDS (split-fp16 at C <= 64; RVC_RB_YLDS=0: the compute waves' own global stores, A/B switch)
    // (2, the default: with C = 32's two R buffers the loaders store tile k - 1 after S1(k) -- 1 keeps them before the
    // c1 epilogue's barrier, the round-6 first form; same bits)
    static const int ylds = getenv("RVC_RB_YLDS") ? atoi(getenv("RVC_RB_YLDS")) : 2;
    p.ylds = g_rb_ylds >= 0 ? g_rb_ylds : ylds;
#if RVC_CONV_STAMPS
    p.stamps = g_rb_stamps;
    p.stamp_blocks = g_rb_stamp_blocks;
#endif
    hipStream_t s = (hipStream_t)stream;
    if (a->C == 32) {
        if (a->passes == RVC_ARITH_F16X3) return launch_rb<32, 3, true>(p, s);
        if (a->passes == 6) return launch_rb<32, 6>(p, s);
        if (a->passes == 3) return launch_rb<32, 3>(p, s);
        return launch_rb<32, 1>(p, s);
    }
    if (a->C == 128) {
        if (a->passes == RVC_ARITH_F16X3) return launch_rb<128, 3, true>(p, s);
        if (a->passes == 3) return launch_rb<128, 3>(p, s);
        return launch_rb<128, 1>(p, s);
    }
    if (rb_wide64(a->passes)) {
        if (a->passes == RVC_ARITH_F16X3) return launch_rb<64, 3, true, true>(p, s);
        if (a->passes == 3) return launch_rb<64, 3, false, true>(p, s);
        return launch_rb<64, 1, false, true>(p, s);
    }
    if (a->passes == RVC_ARITH_F16X3) return launch_rb<64, 3, true>(p, s);
    if (a->passes == 6) return launch_rb<64, 6>(p, s);
    if (a->passes == 3) return launch_rb<64, 3>(p, s);
    return launch_rb<64, 1>(p, s);
}

extern "C" int rvc_resblock_set_wide64(int on) {
    const int prev = g_rb_wide64;
    g_rb_wide64 = on < 0 ? -1 : (on ? 1 : 0);
    return prev;
}

extern "C" int rvc_resblock_set_ylds(int on) {
    g_rb_ylds = on < 0 ? -1 : (on > 2 ? 2 : on);
    return RVC_OK;
}

// Diagnostic build only (-DRVC_CONV_STAMPS=1): the fused pair's per-tile phase stamps go to buf ([bytes / 2048][256]
// u64, one row per workgroup); returns -1 in a production build (no stamps compiled).
extern "C" int rvc_resblock_set_stamps(void* buf, int64_t bytes) {
#if RVC_CONV_STAMPS
    g_rb_stamps = (unsigned long long*)buf;
    g_rb_stamp_blocks = buf ? bytes / (8 * RB_STAMP_W) : 0;
    return 0;
#else
    (void)buf;
    (void)bytes;
    return -1;
#endif
}
