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
    int64_t T;
    int64_t ldc;                     // channel stride of q/k/v/o (elements)
    int64_t q_hs, k_hs, v_hs, o_hs;  // head strides
    int64_t q_bs, k_bs, v_bs, o_bs;  // batch strides
    int H, W;
    float scale;
};

template <int D>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnParams p) {
    constexpr int KT = 64;       // keys per tile
    constexpr int KS = KT + 16;  // Ks row stride (== 16 mod 32)
    constexpr int VS = D + 4;    // Vs row stride (== 4 mod 8)
    constexpr int NS = D / 4;    // k-steps over channels
    constexpr int NF = D / 16;   // output channel fragments
    __shared__ __attribute__((aligned(16))) float Ks[D * KS];
    __shared__ __attribute__((aligned(16))) float Vs[KT * VS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = blockIdx.y, b = blockIdx.z;
    const int64_t T = p.T;
    const int lq = lane & 15, lg = lane >> 4;
    const int64_t q0 = (int64_t)blockIdx.x * 64 + wave * 16;
    const int64_t qa = q0 + lq;  // this lane's query

    const float* Q = p.q + b * p.q_bs + h * p.q_hs;
    const float* K = p.k + b * p.k_bs + h * p.k_hs;
    const float* V = p.v + b * p.v_bs + h * p.v_hs;

    float qreg[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) qreg[s] = qa < T ? Q[(int64_t)(4 * s + lg) * p.ldc + qa] * p.scale : 0.f;

    floatx4 acc_o[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) acc_o[f] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
    const float* RK = p.rk ? p.rk + ((int64_t)b * p.H + h) * (2 * p.W + 1) * T : nullptr;

    for (int64_t kt = 0; kt < T; kt += KT) {
        __syncthreads();
        for (int i = tid; i < D * KT; i += 256) {
            int c = i / KT, j = i - c * KT;
            int64_t key = kt + j;
            float kv = 0.f, vv = 0.f;
            if (key < T) {
                kv = K[(int64_t)c * p.ldc + key];
                vv = V[(int64_t)c * p.ldc + key];
            }
            Ks[c * KS + j] = kv;
            Vs[j * VS + c] = vv;
        }
        __syncthreads();

        floatx4 s[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            floatx4 a4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int st = 0; st < NS; ++st) a4 = mfma16(Ks[(4 * st + lg) * KS + 16 * f + lq], qreg[st], a4);
            s[f] = a4;
        }
        float mloc = -INFINITY;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int64_t key = kt + 16 * f + lg * 4 + r;
                float v = s[f][r];
                if (RK) {
                    int64_t d = key - qa;
                    if (d >= -p.W && d <= p.W && qa < T && key < T) v += RK[(d + p.W) * T + qa];
                }
                if (key >= T) v = -INFINITY;
                s[f][r] = v;
                mloc = fmaxf(mloc, v);
            }
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
                float e = expf(s[f][r] - m_new);
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
                const float* vr = Vs + (16 * f + 4 * lg + r) * VS + lq;
#pragma unroll
                for (int fc = 0; fc < NF; ++fc) acc_o[fc] = mfma16(vr[16 * fc], s[f][r], acc_o[fc]);
            }
    }

    if (qa < T) {
        float* O = p.o + b * p.o_bs + h * p.o_hs;
        const float inv = 1.f / l_run;
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) O[(int64_t)(16 * f + lg * 4 + r) * p.ldc + qa] = acc_o[f][r] * inv;
        if (p.ml && lg == 0) {
            float* ML = p.ml + ((int64_t)b * p.H + h) * 2 * T;
            ML[qa] = m_run;
            ML[T + qa] = l_run;
        }
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

}  // namespace

extern "C" int rvc_attention(const rvc_attn_args* a, rvc_stream_t stream) {
    RVC_CHECK_ARG(a && a->q && a->k && a->v && a->o && a->T > 0 && a->H > 0 && a->B > 0, "attention: bad args");
    RVC_CHECK_ARG(a->D == 64 || a->D == 96, "attention: head dim %d unsupported (64, 96)", a->D);
    RVC_CHECK_ARG(!a->rk || (a->ml && a->W >= 0 && a->W <= 15), "attention: rel band needs ml and W <= 15");
    RVC_CHECK_ARG(!a->ev || (a->rk && (2 * a->W + 1) * a->D <= 31 * 96), "attention: ev band too large");
    AttnParams p;
    p.q = a->q; p.k = a->k; p.v = a->v; p.o = a->o; p.rk = a->rk; p.ml = a->ml;
    p.T = a->T; p.ldc = a->ldc ? a->ldc : a->T;
    p.q_hs = a->q_hs; p.k_hs = a->k_hs; p.v_hs = a->v_hs; p.o_hs = a->o_hs;
    p.q_bs = a->q_bs; p.k_bs = a->k_bs; p.v_bs = a->v_bs; p.o_bs = a->o_bs;
    p.H = a->H; p.W = a->W; p.scale = a->scale;
    dim3 grid(cdiv(a->T, 64), (unsigned)a->H, (unsigned)a->B);
    hipStream_t s = (hipStream_t)stream;
    if (a->D == 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(attn_fwd_kernel<96>, grid, dim3(256), 0, s, p);
    RVC_HIP(hipGetLastError());
    if (a->rk && a->ev) {
        hipLaunchKernelGGL(attn_relv_band_kernel, dim3(cdiv(a->T, 32), (unsigned)a->H, (unsigned)a->B), dim3(256), 0,
                           s, p, a->ev, a->D);
        RVC_HIP(hipGetLastError());
    }
    return RVC_OK;
}
