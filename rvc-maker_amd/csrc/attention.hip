// Flash-style multi-head attention on f32 MFMA, channels-first activations.
//
// Q, K, V, O are [B][H][D][T] (any channel/head/batch strides; t contiguous), which is
// how this build keeps ContentVec (fairseq.py:204-225 via F.multi_head_attention_forward)
// and the TextEncoder (synthesizers.py:221-251) activations.  Nothing T x T is ever
// written to HBM.
//
// One wave owns 16 queries.  Scores are computed TRANSPOSED, S^T[key][q] =
// sum_c K[c][key] * (scale*Q[c][q]), so that a query is a lane column: the softmax
// column reductions are in-register + two shuffles, and the probability tile already sits
// in the B-operand layout of the next product O^T[c][q] += sum_key V[c][key] P^T[key][q]
// (k-step r uses keys {16f + 4i + r}), so P never goes through LDS.
// Optional relative-position band (TextEncoder, window W): S^T[key][q] += Rk[key-q+W][q]
// for |key - q| <= W (the reference's zero-padded rel embeddings contribute exactly 0
// elsewhere).  The matching value term is added by rvc_attn_relv_band afterwards, which
// needs the per-query softmax max / sum written to ML.
#include "rvc_common.h"
#include "x6_common.h"
#include <stdlib.h>

namespace {

struct AttnParams {
    const float* q;
    const float* k;
    const float* v;
    float* o;
    const float* rk;  // [B][H][2W+1][T] or null
    float* ml;        // [B][H][2][T] (max, sum) or null
    float* ws;        // split-KV partials: o [B*S][H][D][T], then ml [B*S][H][2][T]
    int64_t T;
    int64_t ldc;                     // channel stride of q/k/v/o (elements)
    int64_t q_hs, k_hs, v_hs, o_hs;  // head strides
    int64_t q_bs, k_bs, v_bs, o_bs;  // batch strides
    int H, W, S, kps;                // heads, rel window, KV splits, keys per split (multiple of 64)
    float scale;
    unsigned* amax_out;  // |max| cell of o (rvc_attention_amax) or null
    const unsigned* amax_in;  // |max| cell of q, k, v (rvc_attention_ex: the split-fp16 kernel) or null
};

// Grid (T/64, H, B*S).  The key range of a block is split blockIdx.z % S; with S > 1 the block
// writes its normalised partial output and (max, sum) to ws and attn_combine merges the splits.
// K/V tiles are software-pipelined through registers: tile i+1's raw loads are issued before tile
// i's MFMAs and written to LDS after them (no use of a loaded value in between, so the loads stay
// in flight).
template <int D>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnParams p) {
    constexpr int KT = 64;       // keys per tile
    constexpr int KS = KT + 16;  // Ks row stride (== 16 mod 32)
    constexpr int VS = D + 4;    // Vs row stride (== 4 mod 8)
    constexpr int NS = D / 4;    // k-steps over channels
    constexpr int NF = D / 16;   // output channel fragments
    constexpr int NE = D / 4;    // staged K (and V) elements per thread: D * KT / 256
    __shared__ __attribute__((aligned(16))) float Ks[D * KS];
    __shared__ __attribute__((aligned(16))) float Vs[KT * VS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = blockIdx.y;
    const int split = blockIdx.z % p.S, b = blockIdx.z / p.S;
    const int64_t T = p.T;
    const int lq = lane & 15, lg = lane >> 4;
    const int64_t q0 = (int64_t)blockIdx.x * 64 + wave * 16;
    const int64_t qa = q0 + lq;  // this lane's query
    const int64_t kbeg = (int64_t)split * p.kps;
    const int64_t kend = kbeg + p.kps < T ? kbeg + p.kps : T;

    const float* Q = p.q + b * p.q_bs + h * p.q_hs;
    const float* K = p.k + b * p.k_bs + h * p.k_hs;
    const float* V = p.v + b * p.v_bs + h * p.v_hs;

    float qreg[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) qreg[s] = Q[(int64_t)(4 * s + lg) * p.ldc + (qa < T ? qa : T - 1)] * p.scale;

    // staging slots: element e covers channel c = (tid >> 6) + 4 e, key j = tid & 63 (coalesced rows)
    const int sj = tid & 63, sc = tid >> 6;
    float kr[NE], vr[NE];
    auto gload = [&](int64_t kt) {
        const int64_t key = kt + sj < T ? kt + sj : T - 1;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            kr[e] = K[(int64_t)(sc + 4 * e) * p.ldc + key];
            vr[e] = V[(int64_t)(sc + 4 * e) * p.ldc + key];
        }
    };
    auto sstore = [&](int64_t kt) {
        const bool ok = kt + sj < kend;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            Ks[(sc + 4 * e) * KS + sj] = ok ? kr[e] : 0.f;
            Vs[sj * VS + sc + 4 * e] = ok ? vr[e] : 0.f;
        }
    };

    floatx4 acc_o[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) acc_o[f] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
    const float* RK = p.rk ? p.rk + ((int64_t)b * p.H + h) * (2 * p.W + 1) * T : nullptr;

    gload(kbeg);
    sstore(kbeg);
    __syncthreads();
    for (int64_t kt = kbeg; kt < kend; kt += KT) {
        const bool more = kt + KT < kend;
        if (more) gload(kt + KT);
        floatx4 s[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            floatx4 a4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int st = 0; st < NS; ++st) a4 = mfma16(Ks[(4 * st + lg) * KS + 16 * f + lq], qreg[st], a4);
            s[f] = a4;
        }
        // relative-position band: only tiles that meet the wave's band |key - q| <= W (wave-uniform)
        if (RK && kt - (q0 + 15) <= p.W && kt + KT - 1 - q0 >= -p.W) {
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t key = kt + 16 * f + lg * 4 + r;
                    const int64_t d = key - qa;
                    const bool in = d >= -p.W && d <= p.W && qa < T && key < T;
                    const float rv = RK[(in ? d + p.W : 0) * T + (qa < T ? qa : 0)];
                    s[f][r] += in ? rv : 0.f;
                }
        }
        float mloc = -INFINITY;
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t key = kt + 16 * f + lg * 4 + r;
                if (key >= kend) s[f][r] = -INFINITY;
                mloc = fmaxf(mloc, s[f][r]);
            }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = expf(m_run - m_new);
        float lsum = 0.f;
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = expf(s[f][r] - m_new);
                s[f][r] = e;
                lsum += e;
            }
        lsum += __shfl_xor(lsum, 16, 64);
        lsum += __shfl_xor(lsum, 32, 64);
        l_run = l_run * alpha + lsum;
        m_run = m_new;
#pragma unroll
        for (int f = 0; f < NF; ++f) acc_o[f] *= alpha;
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float* vrow = Vs + (16 * f + 4 * lg + r) * VS + lq;
#pragma unroll
                for (int fc = 0; fc < NF; ++fc) acc_o[fc] = mfma16(vrow[16 * fc], s[f][r], acc_o[fc]);
            }
        __syncthreads();
        if (more) sstore(kt + KT);
        __syncthreads();
    }

    float amx = 0.f;  // amax_out: largest |o| this lane stores (the final output only, S == 1)
    if (qa < T) {
        const float inv = 1.f / l_run;
        float* O;
        int64_t ldo;
        float* ML = nullptr;
        if (p.S > 1) {  // partial: ws o [b*S + split][h][D][T]
            const int64_t bs = (int64_t)b * p.S + split;
            O = p.ws + (bs * p.H + h) * D * T;
            ldo = T;
            ML = p.ws + (int64_t)gridDim.z * p.H * D * T + (bs * p.H + h) * 2 * T;
        } else {
            O = p.o + b * p.o_bs + h * p.o_hs;
            ldo = p.ldc;
            if (p.ml) ML = p.ml + ((int64_t)b * p.H + h) * 2 * T;
        }
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float o = acc_o[f][r] * inv;
                O[(int64_t)(16 * f + lg * 4 + r) * ldo + qa] = o;
                amx = fmaxf(amx, fabsf(o));
            }
        if (ML && lg == 0) {
            ML[qa] = m_run;
            ML[T + qa] = l_run;
        }
    }
    if (p.amax_out && p.S == 1) amax_publish(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);  // every lane (the wave's shuffles)
}

// ---------------------------------------------------------------- split-fp16 attention (round 6)
// The same flash attention with both products on the fp16 matrix cores (v_mfma_f32_16x16x32_f16, f32 accumulation)
// in the split-fp16 arithmetic of the conv engine (x6_common.h split2h): every operand is scaled by a power of 2 into
// fp16's range and split exactly into h + l (11 + 11 significant bits), and each product keeps hH + hL + lH (~2^-22
// relative).  The scales: q' = q * scale and k, v from the producer's published |max| of the QKV tensor (amax_in, the
// K = 1 GEMM's cell); the probabilities P in [0, 1] by 2^14 (their small values stay normal).  All undone exactly
// (powers of 2) before the softmax and in the epilogue.  32 fp16 MACs per MFMA lane-cycle against 1 for the f32 MFMA:
// at 3 passes the products cost ~1/10 of the f32 kernel's MFMA time.
// Layouts (conflict-free by the guide's bank rule for ds_read_b128 / ds_write_b128, scripts/attn_banks.py):
//   Ks [chunk of 32 channels][64 keys][2 planes][4 groups of 8 channels] (uint4): the A operand of S^T = K^T Q';
//   Vs [D channel rows][2 planes][8 octets of 8 keys] (uint4): the A operand of O^T = V P^T.
// The S^T fragment rows are assigned to keys so that P^T's C layout IS the next product's B operand: fragment f row
// m <-> key 32 (f >> 1) + 8 (m >> 2) + 4 (f & 1) + (m & 3), so lane (query, group g) holds keys 32 s + 8 g .. + 7 of
// key step s -- 8 consecutive keys, as Vs delivers them.
constexpr int AF_KT = 64;  // keys per tile

__device__ __forceinline__ int af_key(int f, int m) {
    return 32 * (f >> 1) + 8 * (m >> 2) + 4 * (f & 1) + (m & 3);
}
__device__ __forceinline__ int af_ks(int pos, int q, int g) {
    return pos * 8 + ((4 * q + g) ^ (((pos >> 1) & 1) | (((pos >> 3) & 3) << 1)));
}
__device__ __forceinline__ int af_vs(int r, int q, int u) {
    return r * 16 + 8 * (q ^ (r & 1)) + (u ^ (r & 7));
}

// Round 6, second form: at D = 64 each wave owns 32 queries as two 16-query fragments (af_qf), so every K / V operand
// read from LDS feeds both (the 16-query form read 32 KB of LDS per wave per key tile for 48 MFMAs: LDS-bound at 2
// waves per SIMD); a block is 4 waves = af_qb queries.  D = 96 keeps one fragment (two spill 37 VGPRs).
constexpr int af_qf(int D) { return D == 64 ? 2 : 1; }
constexpr int af_qb(int D) { return 64 * af_qf(D); }
template <int D>
__global__ __launch_bounds__(256, 2) void attn_f16_kernel(AttnParams p) {
    constexpr int NC = D / 32;        // 32-channel chunks: k-steps of S^T
    constexpr int NF = D / 16;        // output channel fragments
    constexpr int VI = D * 8 / 256;   // V staging items (channel row, key octet) per thread
    constexpr int QF = af_qf(D);      // query fragments per wave
    static_assert(D % 32 == 0 && (D * 8) % 256 == 0, "D = 64 or 96");
    __shared__ uint4 Ks[NC * AF_KT * 8];
    __shared__ uint4 Vs[D * 16];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = blockIdx.y;
    const int split = blockIdx.z % p.S, b = blockIdx.z / p.S;
    const int64_t T = p.T;
    const int lq = lane & 15, lg = lane >> 4;
    const int64_t q0 = (int64_t)blockIdx.x * af_qb(D) + wave * 16 * QF;
    int64_t qa[QF];  // this lane's query in fragment g
#pragma unroll
    for (int g = 0; g < QF; ++g) qa[g] = q0 + 16 * g + lq;
    const int64_t kbeg = (int64_t)split * p.kps;
    const int64_t kend = kbeg + p.kps < T ? kbeg + p.kps : T;
    const float* Q = p.q + b * p.q_bs + h * p.q_hs;
    const float* K = p.k + b * p.k_bs + h * p.k_hs;
    const float* V = p.v + b * p.v_bs + h * p.v_hs;

    // power-of-2 scales from the batch element's |max| cell (max |q|, |k|, |v| of the projection)
    const float amax = amax_read(p.amax_in + (int64_t)b * RVC_AMAX_SHARDS);
    const int eq = f16_exp(amax * p.scale), ek = f16_exp(amax), ev = f16_exp(amax);
    const float sq = ldexpf(1.f, eq), sk = ldexpf(1.f, ek), sv = ldexpf(1.f, ev);
    const float s_un = ldexpf(1.f, -(eq + ek));
    const float o_un = ldexpf(1.f, -(ev + 14));

    // Q' as the B operand of every S^T fragment (loop-invariant): fragment g, chunk c, lane (query lq, group lg) ->
    // channels 32 c + 8 lg .. + 7
    uint4 qh[QF][NC], ql[QF][NC];
#pragma unroll
    for (int g = 0; g < QF; ++g) {
        const int64_t qc = qa[g] < T ? qa[g] : T - 1;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = Q[(int64_t)(32 * c + 8 * lg + e) * p.ldc + qc] * p.scale * sq;
            uint32_t hw[4], lw[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) split2h_pk(v[2 * e2], v[2 * e2 + 1], hw[e2], lw[e2]);
            qh[g][c] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
            ql[g][c] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
        }
    }

    // staging: K item (key sj, group sg) of each chunk -- 8 channel rows, coalesced over the 64 keys of a wave; V item
    // (channel row, key octet) -- 8 consecutive keys of one row
    // The loads go through buffer resources over the head's D rows: K's channel row in the scalar offset and the key in
    // one 32-bit lane offset shared by every K load, V's row and key octet in one lane offset per item and the key in
    // the immediate -- no 64-bit address per load (those set the register count, not the tiles).  A V key past T reads
    // the next row (masked at the store) or 0 past the range.  (D ldc < 2^29: checked on the host.)
    const int sj = tid & 63, sg = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ldc = (int)p.ldc;
    const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)K, (short)0, D * ldc * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)V, (short)0, D * ldc * 4, 0x00020000);
    float kr[NC][8], vr[VI][8];
    auto gload = [&](int64_t kt) __attribute__((always_inline)) {
        const int ko = (int)(kt + sj < T ? kt + sj : T - 1) * 4;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int e = 0; e < 8; ++e)
                kr[c][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                         krs, ko, (32 * c + 8 * sg + e) * ldc * 4, 0));
#pragma unroll
        for (int it = 0; it < VI; ++it) {
            const int idx = tid + 256 * it, row = idx >> 3, u = idx & 7;
            const int vo = (row * ldc + (int)kt + 8 * u) * 4;
#pragma unroll
            for (int e = 0; e < 8; ++e)
                vr[it][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, vo + 4 * e, 0, 0));
        }
    };
    auto sstore = [&](int64_t kt) __attribute__((always_inline)) {
        const bool okk = kt + sj < kend;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            uint32_t hw[4], lw[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2)
                split2h_pk(okk ? kr[c][2 * e2] * sk : 0.f, okk ? kr[c][2 * e2 + 1] * sk : 0.f, hw[e2], lw[e2]);
            Ks[c * AF_KT * 8 + af_ks(sj, 0, sg)] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
            Ks[c * AF_KT * 8 + af_ks(sj, 1, sg)] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
        }
#pragma unroll
        for (int it = 0; it < VI; ++it) {
            const int idx = tid + 256 * it, row = idx >> 3, u = idx & 7;
            uint32_t hw[4], lw[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
                const bool o0 = kt + 8 * u + 2 * e2 < kend, o1 = kt + 8 * u + 2 * e2 + 1 < kend;
                split2h_pk(o0 ? vr[it][2 * e2] * sv : 0.f, o1 ? vr[it][2 * e2 + 1] * sv : 0.f, hw[e2], lw[e2]);
            }
            Vs[af_vs(row, 0, u)] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
            Vs[af_vs(row, 1, u)] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
        }
    };

    floatx4 acc_o[QF][NF];
#pragma unroll
    for (int g = 0; g < QF; ++g)
#pragma unroll
        for (int f = 0; f < NF; ++f) acc_o[g][f] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run[QF], l_run[QF];
#pragma unroll
    for (int g = 0; g < QF; ++g) {
        m_run[g] = -INFINITY;
        l_run[g] = 0.f;
    }
    const float* RK = p.rk ? p.rk + ((int64_t)b * p.H + h) * (2 * p.W + 1) * T : nullptr;

    gload(kbeg);
    sstore(kbeg);
    __syncthreads();
    for (int64_t kt = kbeg; kt < kend; kt += AF_KT) {
        const bool more = kt + AF_KT < kend;
        if (more) gload(kt + AF_KT);
        // S^T fragments: rows = keys af_key(f, .), columns = query fragment g's 16 queries; each K operand read once
        floatx4 s[QF][4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int krow = af_key(f, lq);
            floatx4 a4[QF];
#pragma unroll
            for (int g = 0; g < QF; ++g) a4[g] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const uint4 ah = Ks[c * AF_KT * 8 + af_ks(krow, 0, lg)];
                const uint4 al = Ks[c * AF_KT * 8 + af_ks(krow, 1, lg)];
#pragma unroll
                for (int g = 0; g < QF; ++g) {
                    a4[g] = mfma_f16(ah, qh[g][c], a4[g]);
                    a4[g] = mfma_f16(ah, ql[g][c], a4[g]);
                    a4[g] = mfma_f16(al, qh[g][c], a4[g]);
                }
            }
#pragma unroll
            for (int g = 0; g < QF; ++g)
#pragma unroll
                for (int r = 0; r < 4; ++r) s[g][f][r] = a4[g][r] * s_un;
        }
        // element (g, f, r) of this lane: key kt + af_key(f, 4 lg + r), query qa[g]
        if (RK && kt - (q0 + 16 * QF - 1) <= p.W && kt + AF_KT - 1 - q0 >= -p.W) {
#pragma unroll
            for (int g = 0; g < QF; ++g)
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int64_t key = kt + af_key(f, 4 * lg + r);
                        const int64_t d = key - qa[g];
                        const bool in = d >= -p.W && d <= p.W && qa[g] < T && key < T;
                        const float rv = RK[(in ? d + p.W : 0) * T + (qa[g] < T ? qa[g] : 0)];
                        s[g][f][r] += in ? rv : 0.f;
                    }
        }
        uint4 ph[QF][2], pl[QF][2];
        float alpha[QF];
#pragma unroll
        for (int g = 0; g < QF; ++g) {
            float mloc = -INFINITY;
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (kt + af_key(f, 4 * lg + r) >= kend) s[g][f][r] = -INFINITY;
                    mloc = fmaxf(mloc, s[g][f][r]);
                }
            mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
            mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
            const float m_new = fmaxf(m_run[g], mloc);
            alpha[g] = expf(m_run[g] - m_new);
            float lsum = 0.f;
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float e = expf(s[g][f][r] - m_new);
                    s[g][f][r] = e;
                    lsum += e;
                }
            lsum += __shfl_xor(lsum, 16, 64);
            lsum += __shfl_xor(lsum, 32, 64);
            l_run[g] = l_run[g] * alpha[g] + lsum;
            m_run[g] = m_new;
            // P^T as the B operand of key step st: keys 32 st + 8 lg + i = fragment 2 st (i < 4) / 2 st + 1 (i >= 4)
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                uint32_t hw[4], lw[4];
                split2h_pk(s[g][2 * st][0] * 16384.f, s[g][2 * st][1] * 16384.f, hw[0], lw[0]);
                split2h_pk(s[g][2 * st][2] * 16384.f, s[g][2 * st][3] * 16384.f, hw[1], lw[1]);
                split2h_pk(s[g][2 * st + 1][0] * 16384.f, s[g][2 * st + 1][1] * 16384.f, hw[2], lw[2]);
                split2h_pk(s[g][2 * st + 1][2] * 16384.f, s[g][2 * st + 1][3] * 16384.f, hw[3], lw[3]);
                ph[g][st] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                pl[g][st] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
            }
#pragma unroll
            for (int f = 0; f < NF; ++f) acc_o[g][f] *= alpha[g];
        }
        // O^T += V P^T: each V operand read once for both query fragments
#pragma unroll
        for (int fc = 0; fc < NF; ++fc) {
            const int row = 16 * fc + lq;
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                const uint4 ah = Vs[af_vs(row, 0, 4 * st + lg)];
                const uint4 al = Vs[af_vs(row, 1, 4 * st + lg)];
#pragma unroll
                for (int g = 0; g < QF; ++g) {
                    acc_o[g][fc] = mfma_f16(ah, ph[g][st], acc_o[g][fc]);
                    acc_o[g][fc] = mfma_f16(ah, pl[g][st], acc_o[g][fc]);
                    acc_o[g][fc] = mfma_f16(al, ph[g][st], acc_o[g][fc]);
                }
            }
        }
        __syncthreads();
        if (more) sstore(kt + AF_KT);
        __syncthreads();
    }

    float amx = 0.f;
#pragma unroll
    for (int g = 0; g < QF; ++g) {
        if (qa[g] < T) {
            const float inv = 1.f / l_run[g];
            float* O;
            int64_t ldo;
            float* ML = nullptr;
            if (p.S > 1) {
                const int64_t bs = (int64_t)b * p.S + split;
                O = p.ws + (bs * p.H + h) * D * T;
                ldo = T;
                ML = p.ws + (int64_t)gridDim.z * p.H * D * T + (bs * p.H + h) * 2 * T;
            } else {
                O = p.o + b * p.o_bs + h * p.o_hs;
                ldo = p.ldc;
                if (p.ml) ML = p.ml + ((int64_t)b * p.H + h) * 2 * T;
            }
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float o = acc_o[g][f][r] * o_un * inv;
                    O[(int64_t)(16 * f + lg * 4 + r) * ldo + qa[g]] = o;
                    amx = fmaxf(amx, fabsf(o));
                }
            if (ML && lg == 0) {
                ML[qa[g]] = m_run[g];
                ML[T + qa[g]] = l_run[g];
            }
        }
    }
    if (p.amax_out && p.S == 1) amax_publish(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);
}

// Merge S split-KV partials: o = sum_s o_s * l_s e^(m_s - m) / sum_s l_s e^(m_s - m).  Grid (T/64, H, B),
// block 256 = 64 queries (coalesced) x 4 channel groups; each thread keeps D/4 channel sums.
template <int D>
__global__ __launch_bounds__(256) void attn_combine_kernel(AttnParams p) {
    constexpr int NC = D / 4;
    const int h = blockIdx.y, b = blockIdx.z;
    const int64_t T = p.T;
    const int64_t qv = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int cg = threadIdx.x >> 6;
    const bool ok = qv < T;  // (no early return: the amax shuffles need the whole wave)
    const int64_t q = ok ? qv : T - 1;
    const int S = p.S;
    const float* wml = p.ws + (int64_t)gridDim.z * S * p.H * D * T;
    float m = -INFINITY;
    for (int s = 0; s < S; ++s) m = fmaxf(m, wml[(((int64_t)b * S + s) * p.H + h) * 2 * T + q]);
    float wsum = 0.f, acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[j] = 0.f;
    for (int s = 0; s < S; ++s) {
        const int64_t bsh = ((int64_t)b * S + s) * p.H + h;
        const float w = wml[bsh * 2 * T + T + q] * expf(wml[bsh * 2 * T + q] - m);
        wsum += w;
        const float* wo = p.ws + bsh * D * T + q;
#pragma unroll
        for (int j = 0; j < NC; ++j) acc[j] += w * wo[(int64_t)(cg + 4 * j) * T];
    }
    const float inv = 1.f / wsum;
    float* O = p.o + b * p.o_bs + h * p.o_hs;
    float amx = 0.f;
    if (ok) {
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            O[(int64_t)(cg + 4 * j) * p.ldc + q] = acc[j] * inv;
            amx = fmaxf(amx, fabsf(acc[j] * inv));
        }
    }
    if (p.amax_out) amax_publish(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);
    if (!ok) return;
    if (p.ml && cg == 0) {
        float* ML = p.ml + ((int64_t)b * p.H + h) * 2 * T;
        ML[q] = m;
        ML[T + q] = wsum;
    }
}

// out[c][q] += sum_{|j-q|<=W} softmax_p(q, j) * Ev[j-q+W][c]   (synthesizers.py:250, heads_share)
// p recomputed from scale*Q.K + Rk with the forward's saved (max, sum).  A block owns 32 queries:
// phase 1 computes the 32 x (2W+1) band probabilities (one dot product per thread-slot) into LDS,
// phase 2 applies them to Ev for the 32 x D outputs.  Round 6: the block's Q columns and the K columns its band
// touches (32 + 2W) are staged in LDS first by coalesced row loads -- each dot product had walked D strided global
// loads per operand, one latency each (84 us per TextEncoder layer, 30 s); same products in the same order.
constexpr int RELV_QB = 32, RELV_KW = RELV_QB + 2 * 15;  // W <= 15 (rvc_attention_ex)
__global__ __launch_bounds__(256) void attn_relv_band_kernel(AttnParams p, const float* ev, int D) {
    constexpr int QB = RELV_QB;
    __shared__ float pb[QB][32];
    __shared__ float evs[31 * 96];
    __shared__ float qs[96][QB + 1];
    __shared__ float ks[96][RELV_KW + 1];
    const int h = blockIdx.y, b = blockIdx.z;
    const int64_t T = p.T;
    const int64_t q0 = (int64_t)blockIdx.x * QB;
    const int tid = threadIdx.x;
    const int nb = 2 * p.W + 1, kw = QB + 2 * p.W;
    const float* Q = p.q + b * p.q_bs + h * p.q_hs;
    const float* K = p.k + b * p.k_bs + h * p.k_hs;
    const float* RK = p.rk + ((int64_t)b * p.H + h) * nb * T;
    const float* ML = p.ml + ((int64_t)b * p.H + h) * 2 * T;
    float* O = p.o + b * p.o_bs + h * p.o_hs;
    for (int i = tid; i < nb * D; i += 256) evs[i] = ev[i];
    for (int i = tid; i < D * QB; i += 256) {  // Q[c][q0 .. q0 + QB): lanes along t
        const int c = i / QB, qi = i - c * QB;
        const int64_t qa = q0 + qi;
        qs[c][qi] = qa < T ? Q[(int64_t)c * p.ldc + qa] : 0.f;
    }
    for (int i = tid; i < D * kw; i += 256) {  // K[c][q0 - W .. q0 + QB + W)
        const int c = i / kw, ji = i - c * kw;
        const int64_t j = q0 - p.W + ji;
        ks[c][ji] = (j >= 0 && j < T) ? K[(int64_t)c * p.ldc + j] : 0.f;
    }
    __syncthreads();
    for (int i = tid; i < QB * nb; i += 256) {
        const int qi = i % QB, r = i / QB;
        const int64_t qa = q0 + qi, j = qa + r - p.W;
        float pv = 0.f;
        if (qa < T && j >= 0 && j < T) {
            float sc = 0.f;
            for (int c = 0; c < D; ++c) sc += (qs[c][qi] * p.scale) * ks[c][qi + r];
            sc += RK[(int64_t)r * T + qa];
            pv = expf(sc - ML[qa]) / ML[T + qa];
        }
        pb[qi][r] = pv;
    }
    __syncthreads();
    float amx = 0.f;  // amax_out: max |o| of the final values (the band term is the last one added)
    for (int i = tid; i < QB * D; i += 256) {
        const int qi = i % QB, c = i / QB;
        const int64_t qa = q0 + qi;
        if (qa >= T) continue;
        float acc = 0.f;
        for (int r = 0; r < nb; ++r) acc += pb[qi][r] * evs[r * D + c];
        const float v = O[(int64_t)c * p.ldc + qa] + acc;
        O[(int64_t)c * p.ldc + qa] = v;
        amx = fmaxf(amx, fabsf(v));
    }
    if (p.amax_out) amax_publish_block(p.amax_out + (int64_t)b * RVC_AMAX_SHARDS, amx);  // one atomic per block
}

// Split-KV plan: enough blocks to cover the chip twice, at least 4 key tiles per split.
// qpb: queries per block (64: attn_fwd_kernel; af_qb(D): attn_f16_kernel)
void attn_plan(const rvc_attn_args* a, int& S, int& kps, int qpb = 64) {
    const int64_t blocks = (int64_t)cdiv(a->T, qpb) * a->H * a->B;
    int64_t s = (512 + blocks - 1) / blocks;
    const int64_t smax = a->T / 256;
    if (s > smax) s = smax;
    if (s > 32) s = 32;
    if (s < 1) s = 1;
    kps = (int)((a->T + s - 1) / s + 63) / 64 * 64;
    S = (int)((a->T + kps - 1) / kps);
}
}  // namespace

extern "C" int64_t rvc_attention_workspace_bytes(const rvc_attn_args* a) {
    if (!a || a->T <= 0 || a->H <= 0 || a->B <= 0 || (a->D != 64 && a->D != 96)) return -1;
    int S, kps, S16, kps16;
    attn_plan(a, S, kps);
    attn_plan(a, S16, kps16, af_qb(a->D));  // the split-fp16 kernel's plan (a call with a |max| cell): the larger
    S = S16 > S ? S16 : S;
    if (S <= 1) return 0;
    return (int64_t)4 * a->B * S * a->H * a->T * (a->D + 2);
}

extern "C" int rvc_attention(const rvc_attn_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream) {
    return rvc_attention_amax(a, nullptr, ws, ws_bytes, stream);
}

extern "C" int rvc_attention_amax(const rvc_attn_args* a, unsigned* amax_out, void* ws, int64_t ws_bytes,
                                  rvc_stream_t stream) {
    return rvc_attention_ex(a, nullptr, amax_out, ws, ws_bytes, stream);
}

// per-thread override of the split-fp16 kernel (rvc_attention_set_f16; -1 = RVC_ATTN_F16, default on)
static thread_local int g_attn_f16 = -1;

extern "C" int rvc_attention_set_f16(int on) {
    g_attn_f16 = on < 0 ? -1 : (on ? 1 : 0);
    return RVC_OK;
}

extern "C" int rvc_attention_ex(const rvc_attn_args* a, const unsigned* amax_in, unsigned* amax_out, void* ws,
                                int64_t ws_bytes, rvc_stream_t stream) {
    RVC_CHECK_ARG(a && a->q && a->k && a->v && a->o && a->T > 0 && a->H > 0 && a->B > 0, "attention: bad args");
    RVC_CHECK_ARG(!amax_out || !a->rk || a->ev, "attention: amax_out with the relative band needs its value term (ev)");
    RVC_CHECK_ARG(a->D == 64 || a->D == 96, "attention: head dim %d unsupported (64, 96)", a->D);
    RVC_CHECK_ARG(!a->rk || (a->ml && a->W >= 0 && a->W <= 15), "attention: rel band needs ml and W <= 15");
    RVC_CHECK_ARG(!a->ev || (a->rk && (2 * a->W + 1) * a->D <= 31 * 96), "attention: ev band too large");
    AttnParams p;
    p.q = a->q; p.k = a->k; p.v = a->v; p.o = a->o; p.rk = a->rk; p.ml = a->ml;
    p.T = a->T; p.ldc = a->ldc ? a->ldc : a->T;
    p.q_hs = a->q_hs; p.k_hs = a->k_hs; p.v_hs = a->v_hs; p.o_hs = a->o_hs;
    p.q_bs = a->q_bs; p.k_bs = a->k_bs; p.v_bs = a->v_bs; p.o_bs = a->o_bs;
    p.H = a->H; p.W = a->W; p.scale = a->scale;
    p.amax_out = (a->rk && a->ev) ? nullptr : amax_out;  // with the rel-v band its kernel publishes (final values)
    p.amax_in = amax_in;
    static const int f16_env = getenv("RVC_ATTN_F16") ? atoi(getenv("RVC_ATTN_F16")) : 1;
    const bool f16 = amax_in && (g_attn_f16 >= 0 ? g_attn_f16 : f16_env);
    attn_plan(a, p.S, p.kps, f16 ? af_qb(a->D) : 64);
    p.ws = nullptr;
    if (p.S > 1) {
        const int64_t need = (int64_t)4 * a->B * p.S * a->H * a->T * (a->D + 2);
        RVC_CHECK_ARG(ws && ws_bytes >= need, "attention: split-KV needs %lld B of workspace (got %lld)",
                      (long long)need, (long long)ws_bytes);
        p.ws = (float*)ws;
    }
    RVC_CHECK_ARG(a->B * p.S < 65536 && a->H < 65536, "attention: grid too large");
    RVC_CHECK_ARG(!f16 || (int64_t)a->D * p.ldc < (1ll << 29), "attention: split-fp16 needs D * ldc < 2^29");
    dim3 grid(cdiv(a->T, 64), (unsigned)a->H, (unsigned)(a->B * p.S));
    hipStream_t s = (hipStream_t)stream;
    if (f16) {
        const dim3 g16(cdiv(a->T, af_qb(a->D)), (unsigned)a->H, (unsigned)(a->B * p.S));
        if (a->D == 64) hipLaunchKernelGGL(attn_f16_kernel<64>, g16, dim3(256), 0, s, p);
        else hipLaunchKernelGGL(attn_f16_kernel<96>, g16, dim3(256), 0, s, p);
    } else if (a->D == 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(attn_fwd_kernel<96>, grid, dim3(256), 0, s, p);
    RVC_HIP(hipGetLastError());
    if (p.S > 1) {
        const dim3 cg(cdiv(a->T, 64), (unsigned)a->H, (unsigned)a->B);
        if (a->D == 64) hipLaunchKernelGGL(attn_combine_kernel<64>, cg, dim3(256), 0, s, p);
        else hipLaunchKernelGGL(attn_combine_kernel<96>, cg, dim3(256), 0, s, p);
        RVC_HIP(hipGetLastError());
    }
    if (a->rk && a->ev) {
        p.amax_out = amax_out;
        hipLaunchKernelGGL(attn_relv_band_kernel, dim3(cdiv(a->T, 32), (unsigned)a->H, (unsigned)a->B), dim3(256), 0,
                           s, p, a->ev, a->D);
        RVC_HIP(hipGetLastError());
    }
    return RVC_OK;
}
