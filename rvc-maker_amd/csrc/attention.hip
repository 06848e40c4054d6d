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
// phase 2 applies them to Ev for the 32 x D outputs.
__global__ __launch_bounds__(256) void attn_relv_band_kernel(AttnParams p, const float* ev, int D) {
    constexpr int QB = 32;
    __shared__ float pb[QB][32];
    __shared__ float evs[31 * 96];
    const int h = blockIdx.y, b = blockIdx.z;
    const int64_t T = p.T;
    const int64_t q0 = (int64_t)blockIdx.x * QB;
    const int tid = threadIdx.x;
    const int nb = 2 * p.W + 1;
    const float* Q = p.q + b * p.q_bs + h * p.q_hs;
    const float* K = p.k + b * p.k_bs + h * p.k_hs;
    const float* RK = p.rk + ((int64_t)b * p.H + h) * nb * T;
    const float* ML = p.ml + ((int64_t)b * p.H + h) * 2 * T;
    float* O = p.o + b * p.o_bs + h * p.o_hs;
    for (int i = tid; i < nb * D; i += 256) evs[i] = ev[i];
    for (int i = tid; i < QB * nb; i += 256) {
        const int qi = i % QB, r = i / QB;
        const int64_t qa = q0 + qi, j = qa + r - p.W;
        float pv = 0.f;
        if (qa < T && j >= 0 && j < T) {
            float sc = 0.f;
            for (int c = 0; c < D; ++c) sc += (Q[(int64_t)c * p.ldc + qa] * p.scale) * K[(int64_t)c * p.ldc + j];
            sc += RK[(int64_t)r * T + qa];
            pv = expf(sc - ML[qa]) / ML[T + qa];
        }
        pb[qi][r] = pv;
    }
    __syncthreads();
    for (int i = tid; i < QB * D; i += 256) {
        const int qi = i % QB, c = i / QB;
        const int64_t qa = q0 + qi;
        if (qa >= T) continue;
        float acc = 0.f;
        for (int r = 0; r < nb; ++r) acc += pb[qi][r] * evs[r * D + c];
        O[(int64_t)c * p.ldc + qa] += acc;
    }
}

// Split-KV plan: enough blocks to cover the chip twice, at least 4 key tiles per split.
void attn_plan(const rvc_attn_args* a, int& S, int& kps) {
    const int64_t blocks = (int64_t)cdiv(a->T, 64) * a->H * a->B;
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
    int S, kps;
    attn_plan(a, S, kps);
    if (S <= 1) return 0;
    return (int64_t)4 * a->B * S * a->H * a->T * (a->D + 2);
}

extern "C" int rvc_attention(const rvc_attn_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream) {
    return rvc_attention_amax(a, nullptr, ws, ws_bytes, stream);
}

extern "C" int rvc_attention_amax(const rvc_attn_args* a, unsigned* amax_out, void* ws, int64_t ws_bytes,
                                  rvc_stream_t stream) {
    RVC_CHECK_ARG(a && a->q && a->k && a->v && a->o && a->T > 0 && a->H > 0 && a->B > 0, "attention: bad args");
    RVC_CHECK_ARG(!amax_out || !a->rk, "attention: amax_out is not built for the relative band");
    RVC_CHECK_ARG(a->D == 64 || a->D == 96, "attention: head dim %d unsupported (64, 96)", a->D);
    RVC_CHECK_ARG(!a->rk || (a->ml && a->W >= 0 && a->W <= 15), "attention: rel band needs ml and W <= 15");
    RVC_CHECK_ARG(!a->ev || (a->rk && (2 * a->W + 1) * a->D <= 31 * 96), "attention: ev band too large");
    AttnParams p;
    p.q = a->q; p.k = a->k; p.v = a->v; p.o = a->o; p.rk = a->rk; p.ml = a->ml;
    p.T = a->T; p.ldc = a->ldc ? a->ldc : a->T;
    p.q_hs = a->q_hs; p.k_hs = a->k_hs; p.v_hs = a->v_hs; p.o_hs = a->o_hs;
    p.q_bs = a->q_bs; p.k_bs = a->k_bs; p.v_bs = a->v_bs; p.o_bs = a->o_bs;
    p.H = a->H; p.W = a->W; p.scale = a->scale;
    p.amax_out = amax_out;
    attn_plan(a, p.S, p.kps);
    p.ws = nullptr;
    if (p.S > 1) {
        const int64_t need = (int64_t)4 * a->B * p.S * a->H * a->T * (a->D + 2);
        RVC_CHECK_ARG(ws && ws_bytes >= need, "attention: split-KV needs %lld B of workspace (got %lld)",
                      (long long)need, (long long)ws_bytes);
        p.ws = (float*)ws;
    }
    RVC_CHECK_ARG(a->B * p.S < 65536 && a->H < 65536, "attention: grid too large");
    dim3 grid(cdiv(a->T, 64), (unsigned)a->H, (unsigned)(a->B * p.S));
    hipStream_t s = (hipStream_t)stream;
    if (a->D == 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(attn_fwd_kernel<96>, grid, dim3(256), 0, s, p);
    RVC_HIP(hipGetLastError());
    if (p.S > 1) {
        const dim3 cg(cdiv(a->T, 64), (unsigned)a->H, (unsigned)a->B);
        if (a->D == 64) hipLaunchKernelGGL(attn_combine_kernel<64>, cg, dim3(256), 0, s, p);
        else hipLaunchKernelGGL(attn_combine_kernel<96>, cg, dim3(256), 0, s, p);
        RVC_HIP(hipGetLastError());
    }
    if (a->rk && a->ev) {
        hipLaunchKernelGGL(attn_relv_band_kernel, dim3(cdiv(a->T, 32), (unsigned)a->H, (unsigned)a->B), dim3(256), 0,
                           s, p, a->ev, a->D);
        RVC_HIP(hipGetLastError());
    }
    return RVC_OK;
}
