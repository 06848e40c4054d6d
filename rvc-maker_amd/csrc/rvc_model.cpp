// Model-level C ABI (include/rvc_amd.h, "model-level API"): a per-device context that owns a
// voice model's weights and scratch and runs Synthesizer.infer (synthesizers.py:446-465) natively.
//
// Load (VoiceConverter.setup, convert.py:554-588): weight-norm folded on the host (torch._weight_norm,
// dim 0), weights transposed to the KM layout the conv engines read (ops.pack_km / pack_convT), uploaded, and
// split into the split-bf16 / split-fp16 operand images (rvc_conv1d_pack_x6 / _f16).
// Infer: the launch sequence of rvc_amd/synth.py -- TextEncoder (synthesizers.py:183-371), prior sample
// (:449), flow^-1 (residuals.py:87-137, modules.py:9-59), NSF-HiFiGAN (synthesizers.py:114-168) -- with the
// same pass-set choices (ops.conv_passes / rb_passes / resblock_fusable), so a model loaded from the same
// fp32 weights gives bit-identical output to SynthesizerAMD.
#include "model_common.h"

using namespace rvcm;

namespace synthm {

constexpr float kLreluSlope = 0.1f;  // synthesizers.py LRELU_SLOPE

struct Pair {
    int d;
    ConvW c1, c2;
};

struct Layer {
    ConvW qkv, relk, o, ffn1, ffn2;
    float *ev = nullptr, *ln1g = nullptr, *ln1b = nullptr, *ln2g = nullptr, *ln2b = nullptr;
};

struct Flow {
    ConvW pre, post;
    ConvW ins[3], rs_a[2], rs_b[3];
};

}  // namespace synthm

struct Synth : ModelBase {
    rvc_synth_cfg cfg{};
    int emb_dim = 0, upp = 1, kc = 0;
    ConvW emb_phone, proj, cond, conv_pre, conv_post;
    float *emb_pitch = nullptr, *emb_g = nullptr;
    int64_t n_spk = 0;
    std::vector<synthm::Layer> layers;
    synthm::Flow flows[4];
    float lin_w = 0, lin_b = 0;
    std::vector<ConvW> ups;
    std::vector<ConvW> noise;
    std::vector<int> noise_stride, noise_pad, chans;
    std::vector<std::vector<std::vector<synthm::Pair>>> res;  // [stage][block][pair]
};


void synth_delete(Synth* s) {
    if (!s) return;
    s->release();
    delete s;
}

namespace synthm {

int64_t convT_out_len(const ConvW& cw, int64_t Lin) { return (Lin - 1) * cw.u - 2 * cw.tpad + cw.Kfull; }

int rb_passes(const rvc_ctx* c, int K) {
    // the smallest split-fp16 kernel size (RVC_AMD_RB_F16_KMIN as ops.py, default 3)
    static const int kmin = getenv("RVC_AMD_RB_F16_KMIN") ? atoi(getenv("RVC_AMD_RB_F16_KMIN")) : 3;
    if (c->prec == RVC_PREC_FP32 && c->f16mix && K >= kmin) return RVC_ARITH_F16X3;
    return base_passes(c);
}

// the fused pair takes the pass sets ops.RB_PASSES lists (6, 3, 1, split-fp16); any other (FP32SA) runs as two
// rvc_conv1d launches, as ops.resblock_fusable decides
bool rb_pass_ok(int passes) { return passes == 6 || passes == 3 || passes == 1 || passes == RVC_ARITH_F16X3; }

bool resblock_fusable(const rvc_ctx* c, const ConvW& c1, const ConvW& c2, int d) {
    // the 128-channel pair only at <= 2 split planes (passes 3, 1, F16X3: what fits its LDS) and on request
    // (RVC_AMD_FUSED_RB128=1: measured slower in the clip stream), as ops.py
    static const bool rb128 = getenv("RVC_AMD_FUSED_RB128") && atoi(getenv("RVC_AMD_FUSED_RB128")) != 0;
    const int passes = rb_passes(c, c1.K);
    const bool chans = c1.Co == 32 || c1.Co == 64 || (c1.Co == 128 && rb128 && passes != 6);
    return c->fused_rb && rb_pass_ok(passes) && c1.wx_bf && c2.wx_bf && c1.Ci == c1.Co && c2.Ci == c2.Co &&
           c1.Co == c2.Co && chans && c1.K == c2.K && c1.K % 2 == 1 && c1.K <= 15 && (c1.K - 1) * d <= 64;
}



// |max| side-channel cells per generator stage (synth.py AMAX_PER_STAGE): y, then t1 / nxt of each unfused pair
constexpr int kAmaxPerStage = 16;

struct Bufs {
    int64_t phone_cf, lin, x, tmp, o, ml, qkv, rk, ffh, stats, znoise, zp, fb0, fb1, h, acts, outacc, xin, gc, har, work,
        snoise, xpre, amax, tcell, reg[2];
    std::vector<int64_t> Li;
    int64_t stage_floats = 0, total = 0;
};

Bufs plan_bufs(const Synth& S, int64_t T) {
    const rvc_synth_cfg& g = S.cfg;
    const int64_t H = g.hidden_channels, I = g.inter_channels, nh = g.n_heads, L = T * S.upp;
    Plan p;
    Bufs b;
    b.phone_cf = p.take(S.emb_dim * T);
    b.lin = p.take(H * T);
    b.x = p.take(H * T);
    b.tmp = p.take(H * T);
    b.o = p.take(H * T);
    b.ml = p.take(nh * 2 * T);
    b.qkv = p.take(3 * H * T);
    b.rk = p.take(nh * 21 * T);
    b.ffh = p.take((int64_t)g.filter_channels * T);
    b.stats = p.take(2 * I * T);
    b.znoise = p.take(I * T);
    b.zp = p.take(I * T);
    b.fb0 = p.take(I * T);
    b.fb1 = p.take(I * T);
    b.h = p.take(H * T);
    b.acts = p.take(H * T);
    b.outacc = p.take(H * T);
    b.xin = p.take(2 * H * T);
    b.gc = p.take(S.cond.Co);
    b.har = p.take(L);
    b.work = p.take(T);
    b.snoise = p.take(L);
    b.xpre = p.take((int64_t)g.upsample_initial_channel * T);
    // the |max| cells of the ResBlock stages, then one per stage output and one for conv_pre (synth.py generator)
    b.amax = p.take((kAmaxPerStage * 8 + 8 + 1) * RVC_AMAX_SHARDS);
    // the TextEncoder's |max| cells (embedding, then per layer qkv, o, ln1, ffn1, ln2) and the flow's (the constant 1.0
    // cell of the gate outputs, then per flow h0, h1, h2, the skip sum, post's x1): synth.py text_encoder / flow_reverse
    b.tcell = p.take((int64_t)(1 + 5 * S.layers.size() + 1 + 5 * 4) * RVC_AMAX_SHARDS);
    int64_t Lc = T;
    for (size_t i = 0; i < S.ups.size(); ++i) {
        Lc = convT_out_len(S.ups[i], Lc);
        b.Li.push_back(Lc);
        const int64_t f = 5 * ((S.chans[i] * Lc + 63) & ~int64_t(63));  // y, xa, xb, xs, t1
        if (f > b.stage_floats) b.stage_floats = f;
    }
    b.reg[0] = p.take(b.stage_floats);  // stages alternate regions: stage i reads stage i-1's xs
    b.reg[1] = p.take(b.stage_floats);
    b.total = p.off;
    return b;
}

// ------------------------------------------------------------------ one sequence (synth.py infer_cf)
int synth_one(rvc_ctx* c, const float* phone, const int64_t* pitch, const float* nsff0, int64_t T, int64_t sid,
              const float* z_noise, const float* sine_noise, uint64_t seed, float* wav, const Bufs& bf, hipStream_t s,
              bool phone_is_cf = false) {
    Synth& S = *c->syn;
    const rvc_synth_cfg& g = S.cfg;
    float* A = S.arena;
    const int64_t H = g.hidden_channels, I = g.inter_channels, half = I / 2, nh = g.n_heads, kc = S.kc, E = S.emb_dim;
    const int64_t L = T * S.upp;
    MCHECK(sid >= 0 && sid < S.n_spk, "rvc_synth_infer: sid %lld out of range [0, %lld)", (long long)sid, (long long)S.n_spk);

    // speaker conditioning: every cond conv stacked (synth.py speaker_cond)
    float* gc = A + bf.gc;
    {
        CallOpts o;
        MTRY(conv(c, S, S.cond, S.emb_g + sid * g.gin_channels, 1, gc, o, s));
    }
    // ---- TextEncoder (synthesizers.py:366-371)
    const float* phone_cf = phone;  // [E][T]
    if (!phone_is_cf) {             // [T][E] as Synthesizer.infer takes it
        MTRY(rvc_transpose(phone, A + bf.phone_cf, 1, T, E, s));
        phone_cf = A + bf.phone_cf;
    }
    float *lin = A + bf.lin, *x = A + bf.x, *tmp = A + bf.tmp, *ob = A + bf.o, *ml = A + bf.ml, *qkv = A + bf.qkv,
          *rk = A + bf.rk, *ffh = A + bf.ffh, *stats = A + bf.stats;
    {
        CallOpts o;
        MTRY(conv(c, S, S.emb_phone, phone_cf, T, lin, o, s));
    }
    // |max| cells (synth.py text_encoder / flow_reverse): the QKV projections' (attn_f16), the TextEncoder's others
    // (te_amax) and the flow's (flow_amax); one memset for all, then the flow's 1.0 cell
    const int64_t nl = (int64_t)S.layers.size();
    unsigned* cbase = reinterpret_cast<unsigned*>(A + bf.tcell);
    unsigned* tcells = c->te_amax ? cbase : nullptr;
    auto tcell = [&](int64_t k) { return tcells ? tcells + RVC_AMAX_SHARDS * k : nullptr; };
    auto fcell = [&](int64_t k) { return c->flow_amax ? cbase + RVC_AMAX_SHARDS * k : nullptr; };
    if (c->te_amax || c->flow_amax || c->attn_f16) {
        MHIP(hipMemsetAsync(cbase, 0, sizeof(unsigned) * RVC_AMAX_SHARDS * (1 + 5 * nl + 1 + 5 * 4), s));
        MHIP(hipMemsetD32Async((hipDeviceptr_t)(cbase + RVC_AMAX_SHARDS * (1 + 5 * nl)), 0x3F800000, 1, s));  // 1.0f
    }
    MTRY(rvc_textenc_embed_amax(lin, S.emb_pitch, pitch, x, 1, H, T, (float)sqrt((double)H), 0.1f, tcell(0), s));
    const unsigned* te_cell = tcell(0);  // the current x's
    const float scale = (float)(1.0 / sqrt((double)kc));
    for (int64_t li = 0; li < nl; ++li) {
        const Layer& Ly = S.layers[li];
        unsigned *c_qkv = c->attn_f16 ? cbase + RVC_AMAX_SHARDS * (1 + 5 * li) : nullptr, *c_o = tcell(2 + 5 * li),
                 *c_l1 = tcell(3 + 5 * li), *c_f1 = tcell(4 + 5 * li), *c_l2 = tcell(5 + 5 * li);
        CallOpts o;
        o.amax_in = te_cell;
        o.amax_out = c_qkv;
        MTRY(conv(c, S, Ly.qkv, x, T, qkv, o, s));
        o.amax_in = nullptr;
        o.amax_out = nullptr;
        CallOpts orl;
        orl.B = nh;
        orl.x_bstride = kc * T;
        orl.Lout = T;
        orl.out_scale = scale;
        MTRY(conv(c, S, Ly.relk, qkv, T, rk, orl, s));
        rvc_attn_args at;
        memset(&at, 0, sizeof(at));
        at.q = qkv;
        at.k = qkv + H * T;
        at.v = qkv + 2 * H * T;
        at.o = ob;
        at.rk = rk;
        at.ev = Ly.ev;
        at.ml = ml;
        at.B = 1;
        at.H = nh;
        at.D = kc;
        at.T = T;
        at.ldc = T;
        at.q_hs = at.k_hs = at.v_hs = at.o_hs = kc * T;
        at.W = 10;
        at.scale = scale;
        const int64_t need = rvc_attention_workspace_bytes(&at);
        MCHECK(need >= 0, "rvc_synth_infer: attention shape H=%lld D=%lld T=%lld unsupported", (long long)nh,
               (long long)kc, (long long)T);
        MTRY(ensure_ws(S, need, s));
        MTRY(rvc_attention_ex(&at, c_qkv, c_o, need ? S.ws : nullptr, need, s));
        CallOpts oo;
        oo.amax_in = c_o;
        MTRY(conv(c, S, Ly.o, ob, T, tmp, oo, s));
        MTRY(rvc_layernorm_cf_amax(x, tmp, Ly.ln1g, Ly.ln1b, x, 1, H, T, 1e-5f, c_l1, s));
        CallOpts f1;
        f1.pad = (g.kernel_size - 1) / 2;
        f1.out_act = RVC_ACT_RELU;
        f1.amax_in = c_l1;
        f1.amax_out = c_f1;
        MTRY(conv(c, S, Ly.ffn1, x, T, ffh, f1, s));
        CallOpts f2;
        f2.pad = (g.kernel_size - 1) / 2;
        f2.amax_in = c_f1;
        MTRY(conv(c, S, Ly.ffn2, ffh, T, tmp, f2, s));
        MTRY(rvc_layernorm_cf_amax(x, tmp, Ly.ln2g, Ly.ln2b, x, 1, H, T, 1e-5f, c_l2, s));
        te_cell = c_l2;
    }
    {
        CallOpts o;
        o.amax_in = te_cell;
        MTRY(conv(c, S, S.proj, x, T, stats, o, s));
    }
    // ---- prior sample (synthesizers.py:449)
    float* zp = A + bf.zp;
    if (!z_noise) {
        float* zn = A + bf.znoise;
        MTRY(rvc_randn_ex(zn, I * T, seed, 0, nullptr, s));
        z_noise = zn;
    }
    MTRY(rvc_prior_sample(stats, z_noise, zp, 1, I, T, 0.66666f, s));
    // ---- flow^-1 (synth.py flow_reverse)
    float *h = A + bf.h, *acts = A + bf.acts, *outacc = A + bf.outacc, *xin = A + bf.xin;
    float* bufs[2] = {A + bf.fb0, A + bf.fb1};
    float* xf_cur = zp;
    // the flow's |max| cells (synth.py flow_reverse): after the TextEncoder's, the 1.0 cell (|tanh * sigmoid| < 1) then
    // 5 per flow
    const unsigned* unit = fcell(1 + 5 * nl);
    const unsigned* post_cell = nullptr;
    for (int f = 3, n = 0; f >= 0; --f, ++n) {
        const Flow& F = S.flows[f];
        unsigned* c_h[3] = {fcell(2 + 5 * nl + 5 * n), fcell(3 + 5 * nl + 5 * n), fcell(4 + 5 * nl + 5 * n)};
        unsigned *c_acc = fcell(5 + 5 * nl + 5 * n), *c_post = fcell(6 + 5 * nl + 5 * n);
        float* xf = (xf_cur != bufs[0]) ? bufs[0] : bufs[1];
        MTRY(rvc_flip_channels(xf_cur, xf, 1, I, T, s));
        float *x0 = xf, *x1 = xf + half * T;
        {
            CallOpts o;
            o.amax_in = post_cell;
            o.amax_out = c_h[0];
            MTRY(conv(c, S, F.pre, x0, T, h, o, s));
        }
        for (int l = 0; l < 3; ++l) {
            CallOpts oi;
            oi.pad = (F.ins[l].K - 1) / 2;
            oi.bias2 = gc + (int64_t)f * 6 * H + (int64_t)l * 2 * H;
            oi.amax_in = c_h[l];
            MTRY(conv(c, S, F.ins[l], h, T, xin, oi, s));
            MTRY(rvc_gate(xin, acts, 1, H, T, s));
            if (l < 2) {
                CallOpts ra;
                ra.res = h;
                ra.amax_in = unit;
                ra.amax_out = c_h[l + 1];
                MTRY(conv(c, S, F.rs_a[l], acts, T, h, ra, s));
                CallOpts rb;
                rb.accumulate = l > 0;
                rb.amax_in = unit;
                MTRY(conv(c, S, F.rs_b[l], acts, T, outacc, rb, s));
            } else {
                CallOpts rb;
                rb.accumulate = 1;
                rb.amax_in = unit;
                rb.amax_out = c_acc;
                MTRY(conv(c, S, F.rs_b[l], acts, T, outacc, rb, s));
            }
        }
        CallOpts po;
        po.res = x1;
        po.out_scale = -1.f;
        po.amax_in = c_acc;
        po.amax_out = c_post;
        MTRY(conv(c, S, F.post, outacc, T, x1, po, s));
        post_cell = c_post;
        xf_cur = xf;
    }
    const float* z = xf_cur;
    // ---- NSF-HiFiGAN (synthesizers.py:144-161, synth.py generator)
    float *har = A + bf.har, *work = A + bf.work;
    if (!sine_noise) {
        float* sn = A + bf.snoise;
        MTRY(rvc_randn_ex(sn, L, seed, (uint64_t)1 << 40, nullptr, s));
        sine_noise = sn;
    }
    MTRY(rvc_sine_source(nsff0, sine_noise, har, work, 1, T, S.upp, (float)g.sr, S.lin_w, S.lin_b, s));
    float* xcur = A + bf.xpre;
    unsigned* amax = reinterpret_cast<unsigned*>(A + bf.amax);
    const bool use_amax = c->amax && (int64_t)S.ups.size() <= 8;
    const int64_t nst = (int64_t)S.ups.size();
    if (use_amax)
        MHIP(hipMemsetAsync(amax, 0, sizeof(unsigned) * RVC_AMAX_SHARDS * (kAmaxPerStage * nst + nst + 1), s));
    // the stage outputs' cells and conv_pre's, after the stages' own (synth.py's out_cell)
    auto out_cell = [&](int64_t k) { return use_amax ? amax + RVC_AMAX_SHARDS * (kAmaxPerStage * nst + k) : nullptr; };
    unsigned* x_cell = out_cell(nst);
    {
        CallOpts o;
        o.pad = 3;
        o.bias2 = gc + 4 * 6 * H;
        o.amax_out = x_cell;
        MTRY(conv(c, S, S.conv_pre, z, T, xcur, o, s));
    }
    int64_t Lcur = T;
    float scale_in = 1.f;
    const int nk = g.n_resblocks;
    for (size_t i = 0; i < S.ups.size(); ++i) {
        const int64_t Li = bf.Li[i], C = S.chans[i];
        const int64_t slab = (C * Li + 63) & ~int64_t(63);
        float* R = A + bf.reg[i & 1];
        float *y = R, *xa = R + slab, *xb = R + 2 * slab, *xs = R + 3 * slab, *t1 = R + 4 * slab;
        // the |max| side channel (synth.py generator): y, each unfused c1 output and each non-last c2 output publish
        // their |max|; the convs that read them take their split-fp16 scale from it
        unsigned* cell = use_amax ? amax + RVC_AMAX_SHARDS * kAmaxPerStage * i : nullptr;
        int ncell = 1;
        CallOpts ou;
        ou.in_act = RVC_ACT_LRELU;
        ou.in_slope = kLreluSlope;
        ou.in_scale = scale_in;
        ou.amax_in = c->amax_ups ? x_cell : nullptr;
        if (c->fused_noise) {  // y = ups(x) + noise_convs(har) in one launch (synth.py FUSED_NOISE)
            ou.src = &S.noise[i];
            ou.src_x = har;
            ou.src_stride = S.noise_stride[i];
            ou.src_pad = S.noise_pad[i];
            ou.src_len = L;
            ou.amax_out = cell;
        }
        MTRY(conv(c, S, S.ups[i], xcur, Lcur, y, ou, s));
        x_cell = nullptr;
        if (!c->fused_noise) {
            CallOpts on;
            on.Lout = Li;
            on.stride = S.noise_stride[i];
            on.pad = S.noise_pad[i];
            on.accumulate = 1;
            if (cell) on.amax_out = cell;
            MTRY(conv(c, S, S.noise[i], har, L, y, on, s));
        }
        for (int j = 0; j < nk; ++j) {
            const int kk = g.resblock_kernel_sizes[j];
            const std::vector<Pair>& pairs = S.res[i][j];
            float* cur = y;
            const unsigned* cur_cell = cell;
            for (size_t m = 0; m < pairs.size(); ++m) {
                const Pair& P = pairs[m];
                const bool last = m + 1 == pairs.size();
                if (resblock_fusable(c, P.c1, P.c2, P.d)) {
                    float* nxt = last ? xs : (cur != xa ? xa : xb);
                    rvc_resblock_args ra;
                    memset(&ra, 0, sizeof(ra));
                    const int passes = rb_passes(c, P.c1.K);
                    ra.x = cur;
                    ra.y = nxt;
                    ra.w1x = passes == RVC_ARITH_F16X3 ? P.c1.wx_hf : P.c1.wx_bf;
                    ra.w2x = passes == RVC_ARITH_F16X3 ? P.c2.wx_hf : P.c2.wx_bf;
                    ra.b1 = P.c1.b;
                    ra.b2 = P.c2.b;
                    ra.C = C;
                    ra.L = Li;
                    ra.K = P.c1.K;
                    ra.dil = P.d;
                    ra.nmf1 = P.c1.nmf;
                    ra.nmf2 = P.c2.nmf;
                    ra.passes = passes;
                    ra.accumulate = last && j > 0;
                    ra.slope = kLreluSlope;
                    MTRY(rvc_resblock_pair(&ra, s));
                    cur = nxt;
                    cur_cell = nullptr;
                    continue;
                }
                unsigned* t1_cell = cell && ncell < kAmaxPerStage ? cell + RVC_AMAX_SHARDS * ncell++ : nullptr;
                CallOpts o1;
                o1.pad = (kk * P.d - P.d) / 2;
                o1.dil = P.d;
                o1.in_act = RVC_ACT_LRELU;
                o1.in_slope = kLreluSlope;
                o1.amax_in = cur_cell;
                o1.amax_out = t1_cell;
                MTRY(conv(c, S, P.c1, cur, Li, t1, o1, s));
                CallOpts o2;
                o2.pad = (kk - 1) / 2;
                o2.res = cur;
                o2.in_act = RVC_ACT_LRELU;
                o2.in_slope = kLreluSlope;
                o2.amax_in = t1_cell;
                float* nxt;
                unsigned* nxt_cell = nullptr;
                if (last) {
                    nxt = xs;
                    o2.accumulate = j > 0;
                    if (j == nk - 1 && use_amax) {  // the stage output's final values: its |max| cell
                        o2.amax_out = out_cell((int64_t)i);
                        x_cell = o2.amax_out;
                    }
                } else {
                    nxt = cur != xa ? xa : xb;
                    nxt_cell = cell && ncell < kAmaxPerStage ? cell + RVC_AMAX_SHARDS * ncell++ : nullptr;
                    o2.amax_out = nxt_cell;
                }
                MTRY(conv(c, S, P.c2, t1, Li, nxt, o2, s));
                cur = nxt;
                cur_cell = nxt_cell;
            }
        }
        xcur = xs;
        Lcur = Li;
        scale_in = 1.f / nk;
    }
    CallOpts op;
    op.pad = 3;
    op.in_act = RVC_ACT_LRELU;
    op.in_slope = 0.01f;
    op.in_scale = scale_in;
    op.out_act = RVC_ACT_TANH;
    return conv(c, S, S.conv_post, xcur, Lcur, wav, op, s);
}

}  // namespace synthm

using namespace synthm;


// ------------------------------------------------------------------ C ABI
extern "C" int rvc_ctx_create(int hip_device, rvc_ctx** out) {
    MCHECK(out, "rvc_ctx_create: null out");
    *out = nullptr;
    MHIP(hipSetDevice(hip_device));
    rvc_ctx* c = new rvc_ctx();
    c->device = hip_device;
    c->x6 = env_on("RVC_AMD_X6");
    c->f16mix = env_on("RVC_AMD_F16MIX");
    c->fused_rb = env_on("RVC_AMD_FUSED_RB");
    c->amax = env_on("RVC_AMD_AMAX");
    c->amax_f16all = env_on("RVC_AMD_AMAX_F16ALL");
    c->cv_amax = env_on("RVC_AMD_CV_AMAX");
    c->amax_ups = env_on("RVC_AMD_AMAX_UPS");
    c->amax_s2 = env_on("RVC_AMD_AMAX_S2");
    c->fe_amax = env_on("RVC_AMD_FE_AMAX");
    c->fused_noise = env_set("RVC_AMD_FUSED_NOISE");
    c->attn_f16 = env_on("RVC_AMD_ATTN_F16");
    c->te_amax = env_set("RVC_AMD_TE_AMAX");
    c->flow_amax = env_set("RVC_AMD_FLOW_AMAX");
    *out = c;
    return RVC_OK;
}

extern "C" void rvc_ctx_destroy(rvc_ctx* c) {
    if (!c) return;
    if (hipSetDevice(c->device) == hipSuccess) {
        (void)hipDeviceSynchronize();
        synth_delete(c->syn);
        vc_delete(c->vc);
        contentvec_delete(c->cv);
        rmvpe_delete(c->rm);
        crepe_delete(c->cr);
    }
    delete c;
}

extern "C" int rvc_ctx_set_precision(rvc_ctx* c, int prec) {
    MCHECK(c, "rvc_ctx_set_precision: null ctx");
    MCHECK(prec == RVC_PREC_FP32 || prec == RVC_PREC_BF16 || prec == RVC_PREC_BF16X3 || prec == RVC_PREC_FP32X6 ||
               prec == RVC_PREC_FP32SA || prec == RVC_PREC_F16X3,
           "rvc_ctx_set_precision: unknown precision %d", prec);
    c->prec = prec;
    return RVC_OK;
}

extern "C" int64_t rvc_synth_out_len(const rvc_ctx* c, int64_t T) {
    if (!c || !c->syn || !c->syn->loaded || T <= 0) return -1;
    return T * c->syn->upp;
}

namespace {
// shape check of a loaded tensor: dims d0..d2 (-1 = any); a mismatch is a load error, not a device fault later
int expect(const HostT& t, const std::string& name, int64_t d0, int64_t d1 = -1, int64_t d2 = -1, int ndim = -1) {
    const int64_t want[3] = {d0, d1, d2};
    int64_t numel = 1;
    for (int64_t x : t.shape) numel *= x;
    MCHECK(numel == (int64_t)t.v.size(), "rvc_load_synth: %s: %zu values for its shape", name.c_str(), t.v.size());
    MCHECK(ndim < 0 || (int)t.shape.size() == ndim, "rvc_load_synth: %s must be %d-D", name.c_str(), ndim);
    for (int i = 0; i < 3; ++i)
        MCHECK(want[i] < 0 || t.dim(i) == want[i], "rvc_load_synth: %s dim %d is %lld, expected %lld", name.c_str(), i,
               (long long)t.dim(i), (long long)want[i]);
    return RVC_OK;
}
}  // namespace

extern "C" int rvc_load_synth(rvc_ctx* c, const rvc_param* params, int n, const rvc_synth_cfg* cfg) {
    MCHECK(c && params && n > 0 && cfg, "rvc_load_synth: null argument");
    const rvc_synth_cfg& g = *cfg;
    MCHECK(g.n_heads > 0 && g.hidden_channels % g.n_heads == 0 && g.n_layers > 0 && g.inter_channels % 2 == 0,
           "rvc_load_synth: bad TextEncoder config");
    MCHECK(g.n_upsamples >= 1 && g.n_upsamples <= 8 && g.n_resblocks >= 1 && g.n_resblocks <= 4 && g.n_dilations >= 1 &&
               g.n_dilations <= 4,
           "rvc_load_synth: bad generator config");
    MCHECK(g.hidden_channels > 0 && g.filter_channels > 0 && g.kernel_size > 0 && g.inter_channels > 0 &&
               g.gin_channels > 0 && g.upsample_initial_channel >> g.n_upsamples > 0,
           "rvc_load_synth: bad channel config");
    Params PM;  // x.weight folded from x.weight_g / x.weight_v (dim 0) when those are given
    MTRY(index_params(params, n, PM, "rvc_load_synth"));
    MHIP(hipSetDevice(c->device));
    synth_delete(c->syn);
    c->syn = new Synth();
    Synth& S = *c->syn;
    S.cfg = g;
    const int H = g.hidden_channels;
    S.kc = H / g.n_heads;
    S.upp = 1;
    for (int i = 0; i < g.n_upsamples; ++i) {
        MCHECK(g.upsample_rates[i] > 0 && g.upsample_rates[i] % 2 == 0,
               "rvc_load_synth: odd upsample rates (output_padding) are not used by any shipped config");
        S.upp *= g.upsample_rates[i];
    }
    HostT w, b, w2, b2;
#define GET(k, t) MCHECK(PM.get(k, t), "rvc_load_synth: missing %s", PM.missing.c_str())
    // ---- TextEncoder
    GET("enc_p.emb_phone.weight", w);
    GET("enc_p.emb_phone.bias", b);
    MTRY(expect(w, "enc_p.emb_phone.weight", H, -1, -1, 2));
    S.emb_dim = (int)w.dim(1);
    w.shape.push_back(1);
    MTRY(make_conv(c, S, w, &b, S.emb_phone));
    GET("enc_p.emb_pitch.weight", w);
    MTRY(expect(w, "enc_p.emb_pitch.weight", 256, H, -1, 2));
    MTRY(upload(S, w.v, &S.emb_pitch));
    for (int i = 0; i < g.n_layers; ++i) {
        Layer Ly;
        const std::string p = "enc_p.encoder.attn_layers." + std::to_string(i) + ".";
        HostT q, k, v, bq, bk, bv;
        GET(p + "conv_q.weight", q);
        GET(p + "conv_k.weight", k);
        GET(p + "conv_v.weight", v);
        GET(p + "conv_q.bias", bq);
        GET(p + "conv_k.bias", bk);
        GET(p + "conv_v.bias", bv);
        MTRY(expect(q, p + "conv_q.weight", H, H, 1));
        MTRY(expect(k, p + "conv_k.weight", H, H, 1));
        MTRY(expect(v, p + "conv_v.weight", H, H, 1));
        HostT wqkv = q, bqkv = bq;
        wqkv.v.insert(wqkv.v.end(), k.v.begin(), k.v.end());
        wqkv.v.insert(wqkv.v.end(), v.v.begin(), v.v.end());
        wqkv.shape[0] = q.dim(0) + k.dim(0) + v.dim(0);
        bqkv.v.insert(bqkv.v.end(), bk.v.begin(), bk.v.end());
        bqkv.v.insert(bqkv.v.end(), bv.v.begin(), bv.v.end());
        MTRY(make_conv(c, S, wqkv, &bqkv, Ly.qkv));
        GET(p + "emb_rel_k", w);  // [1][21][kc] -> relk conv weight [21][kc][1]
        MCHECK(w.dim(1) == 21 && w.dim(2) == S.kc, "rvc_load_synth: emb_rel_k must be [1][21][%d]", S.kc);
        HostT ek;
        ek.v = w.v;
        ek.shape = {21, S.kc, 1};
        MTRY(make_conv(c, S, ek, nullptr, Ly.relk));
        GET(p + "emb_rel_v", w);
        MTRY(expect(w, p + "emb_rel_v", 1, 21, S.kc));
        MTRY(upload(S, w.v, &Ly.ev));
        GET(p + "conv_o.weight", w);
        GET(p + "conv_o.bias", b);
        MTRY(expect(w, p + "conv_o.weight", H, H, 1));
        MTRY(make_conv(c, S, w, &b, Ly.o));
        const std::string si = std::to_string(i);
        GET("enc_p.encoder.norm_layers_1." + si + ".gamma", w);
        MTRY(expect(w, "norm_layers_1." + si + ".gamma", H, -1, -1, 1));
        MTRY(upload(S, w.v, &Ly.ln1g));
        GET("enc_p.encoder.norm_layers_1." + si + ".beta", w);
        MTRY(expect(w, "norm_layers_1." + si + ".beta", H, -1, -1, 1));
        MTRY(upload(S, w.v, &Ly.ln1b));
        GET("enc_p.encoder.ffn_layers." + si + ".conv_1.weight", w);
        GET("enc_p.encoder.ffn_layers." + si + ".conv_1.bias", b);
        MTRY(expect(w, "ffn_layers." + si + ".conv_1.weight", g.filter_channels, H, g.kernel_size));
        MTRY(make_conv(c, S, w, &b, Ly.ffn1));
        GET("enc_p.encoder.ffn_layers." + si + ".conv_2.weight", w);
        GET("enc_p.encoder.ffn_layers." + si + ".conv_2.bias", b);
        MTRY(expect(w, "ffn_layers." + si + ".conv_2.weight", H, g.filter_channels, g.kernel_size));
        MTRY(make_conv(c, S, w, &b, Ly.ffn2));
        GET("enc_p.encoder.norm_layers_2." + si + ".gamma", w);
        MTRY(expect(w, "norm_layers_2." + si + ".gamma", H, -1, -1, 1));
        MTRY(upload(S, w.v, &Ly.ln2g));
        GET("enc_p.encoder.norm_layers_2." + si + ".beta", w);
        MTRY(expect(w, "norm_layers_2." + si + ".beta", H, -1, -1, 1));
        MTRY(upload(S, w.v, &Ly.ln2b));
        S.layers.push_back(Ly);
    }
    GET("enc_p.proj.weight", w);
    GET("enc_p.proj.bias", b);
    MTRY(expect(w, "enc_p.proj.weight", 2 * g.inter_channels, H, 1));
    MTRY(make_conv(c, S, w, &b, S.proj));
    // ---- speaker conditioning: 4 flows' cond layers then dec.cond, stacked (synth.py)
    {
        HostT cw, cb;
        for (int f = 0; f <= 4; ++f) {
            const std::string p = f < 4 ? "flow.flows." + std::to_string(2 * f) + ".enc.cond_layer." : "dec.cond.";
            GET(p + "weight", w);
            GET(p + "bias", b);
            MTRY(expect(w, p + "weight", f < 4 ? 2 * H * 3 : g.upsample_initial_channel, g.gin_channels, 1));
            if (f == 0) {
                cw = w;
                cb = b;
            } else {
                cw.v.insert(cw.v.end(), w.v.begin(), w.v.end());
                cw.shape[0] += w.dim(0);
                cb.v.insert(cb.v.end(), b.v.begin(), b.v.end());
            }
        }
        MTRY(make_conv(c, S, cw, &cb, S.cond));
    }
    GET("emb_g.weight", w);
    MCHECK(w.dim(1) == g.gin_channels, "rvc_load_synth: emb_g width %lld != gin_channels %d", (long long)w.dim(1),
           g.gin_channels);
    S.n_spk = w.dim(0);  // convert.py:558 takes the speaker count from emb_g
    MTRY(upload(S, w.v, &S.emb_g));
    // ---- flow
    for (int f = 0; f < 4; ++f) {
        Flow& F = S.flows[f];
        const std::string p = "flow.flows." + std::to_string(2 * f) + ".";
        GET(p + "pre.weight", w);
        GET(p + "pre.bias", b);
        MTRY(expect(w, p + "pre.weight", H, g.inter_channels / 2, 1));
        MTRY(make_conv(c, S, w, &b, F.pre));
        GET(p + "post.weight", w);
        GET(p + "post.bias", b);
        MTRY(expect(w, p + "post.weight", g.inter_channels / 2, H, 1));
        MTRY(make_conv(c, S, w, &b, F.post));
        for (int l = 0; l < 3; ++l) {
            const std::string sl = std::to_string(l);
            GET(p + "enc.in_layers." + sl + ".weight", w);
            GET(p + "enc.in_layers." + sl + ".bias", b);
            MTRY(expect(w, p + "enc.in_layers." + sl + ".weight", 2 * H, H, 5));
            MTRY(make_conv(c, S, w, &b, F.ins[l]));
            GET(p + "enc.res_skip_layers." + sl + ".weight", w);
            GET(p + "enc.res_skip_layers." + sl + ".bias", b);
            MTRY(expect(w, p + "enc.res_skip_layers." + sl + ".weight", l < 2 ? 2 * H : H, H, 1));
            if (l < 2) {  // res half [:H], skip half [H:]
                const int64_t inner = (int64_t)w.v.size() / w.dim(0);
                HostT wa = w, wb = w, ba = b, bb = b;
                wa.v.assign(w.v.begin(), w.v.begin() + H * inner);
                wa.shape[0] = H;
                wb.v.assign(w.v.begin() + H * inner, w.v.end());
                wb.shape[0] = w.dim(0) - H;
                ba.v.assign(b.v.begin(), b.v.begin() + H);
                bb.v.assign(b.v.begin() + H, b.v.end());
                MTRY(make_conv(c, S, wa, &ba, F.rs_a[l]));
                MTRY(make_conv(c, S, wb, &bb, F.rs_b[l]));
            } else {
                MTRY(make_conv(c, S, w, &b, F.rs_b[l]));
            }
        }
    }
    // ---- generator
    GET("dec.m_source.l_linear.weight", w);
    GET("dec.m_source.l_linear.bias", b);
    MTRY(expect(w, "dec.m_source.l_linear.weight", 1, 1, -1, 2));
    MTRY(expect(b, "dec.m_source.l_linear.bias", 1, -1, -1, 1));
    S.lin_w = w.v[0];
    S.lin_b = b.v[0];
    GET("dec.conv_pre.weight", w);
    GET("dec.conv_pre.bias", b);
    MTRY(expect(w, "dec.conv_pre.weight", g.upsample_initial_channel, g.inter_channels, 7));
    MTRY(make_conv(c, S, w, &b, S.conv_pre));
    const int nup = g.n_upsamples;
    S.ups.resize(nup);
    S.noise.resize(nup);
    S.res.resize(nup);
    for (int i = 0; i < nup; ++i) {
        const int u = g.upsample_rates[i], k = g.upsample_kernel_sizes[i];
        S.chans.push_back(g.upsample_initial_channel >> (i + 1));
        const std::string si = std::to_string(i);
        GET("dec.ups." + si + ".weight", w);
        GET("dec.ups." + si + ".bias", b);
        const int ch = g.upsample_initial_channel >> (i + 1);
        MTRY(expect(w, "dec.ups." + si + ".weight", 2 * ch, ch, k));
        MTRY(expect(b, "dec.ups." + si + ".bias", ch, -1, -1, 1));
        MTRY(make_convT(c, S, w, b, u, (k - u) / 2, S.ups[i]));
        int st = 1;
        for (int j = i + 1; j < nup; ++j) st *= g.upsample_rates[j];
        const int kn = st == 1 ? 1 : st * 2 - st % 2;
        S.noise_stride.push_back(st);
        S.noise_pad.push_back(st == 1 ? 0 : (kn - st) / 2);
        GET("dec.noise_convs." + si + ".weight", w);
        GET("dec.noise_convs." + si + ".bias", b);
        MTRY(expect(w, "dec.noise_convs." + si + ".weight", ch, 1, kn));
        MTRY(make_conv(c, S, w, &b, S.noise[i]));
        S.res[i].resize(g.n_resblocks);
        for (int j = 0; j < g.n_resblocks; ++j) {
            const std::string rb = "dec.resblocks." + std::to_string(i * g.n_resblocks + j) + ".";
            for (int m = 0; m < g.n_dilations; ++m) {
                Pair P;
                P.d = g.resblock_dilation_sizes[j][m];
                const std::string sm = std::to_string(m);
                GET(rb + "convs1." + sm + ".weight", w);
                GET(rb + "convs1." + sm + ".bias", b);
                MTRY(expect(w, rb + "convs1." + sm + ".weight", ch, ch, g.resblock_kernel_sizes[j]));
                MTRY(make_conv(c, S, w, &b, P.c1));
                GET(rb + "convs2." + sm + ".weight", w2);
                GET(rb + "convs2." + sm + ".bias", b2);
                MTRY(expect(w2, rb + "convs2." + sm + ".weight", ch, ch, g.resblock_kernel_sizes[j]));
                MTRY(make_conv(c, S, w2, &b2, P.c2));
                S.res[i][j].push_back(P);
            }
        }
    }
    GET("dec.conv_post.weight", w);
    MTRY(expect(w, "dec.conv_post.weight", 1, g.upsample_initial_channel >> nup, 7));
    MTRY(make_conv(c, S, w, nullptr, S.conv_post));
#undef GET
    MHIP(hipDeviceSynchronize());
    S.loaded = true;
    return RVC_OK;
}

extern "C" int rvc_synth_infer(rvc_ctx* c, const float* phone, const int64_t* pitch, const float* pitchf, int64_t B,
                               int64_t T, const int64_t* sid, const float* z_noise, const float* sine_noise,
                               uint64_t seed, float* wav, rvc_stream_t stream) {
    MCHECK(c && c->syn && c->syn->loaded, "rvc_synth_infer: no synthesizer loaded");
    MCHECK(phone && pitch && pitchf && sid && wav, "rvc_synth_infer: null buffer");
    MCHECK(B >= 1 && T >= 1, "rvc_synth_infer: empty input (B=%lld, T=%lld)", (long long)B, (long long)T);
    hipStream_t s = (hipStream_t)stream;
    MHIP(hipSetDevice(c->device));
    const Bufs bf = plan_bufs(*c->syn, T);
    MTRY(ensure_arena(*c->syn, bf.total, s));
    const int64_t I = c->syn->cfg.inter_channels, L = T * c->syn->upp, E = c->syn->emb_dim;
    for (int64_t b = 0; b < B; ++b)  // sequences share the scratch in stream order
        MTRY(synth_one(c, phone + b * T * E, pitch + b * T, pitchf + b * T, T, sid[b], z_noise ? z_noise + b * I * T : nullptr,
                       sine_noise ? sine_noise + b * L : nullptr, seed + (uint64_t)b, wav + b * L, bf, s));
    return RVC_OK;
}

int synth_run_cf(rvc_ctx* c, const float* phone_cf, const int64_t* pitch, const float* pitchf, int64_t T, int64_t sid,
                 uint64_t seed, float* wav, hipStream_t s) {
    MCHECK(c && c->syn && c->syn->loaded, "rvc_vc_convert: no synthesizer loaded");
    const Bufs bf = plan_bufs(*c->syn, T);
    MTRY(ensure_arena(*c->syn, bf.total, s));
    return synth_one(c, phone_cf, pitch, pitchf, T, sid, nullptr, nullptr, seed, wav, bf, s, true);
}

bool synth_info(const rvc_ctx* c, int* emb_dim, int* upp) {
    if (!c || !c->syn || !c->syn->loaded) return false;
    *emb_dim = c->syn->emb_dim;
    *upp = c->syn->upp;
    return true;
}
