// Model-level C ABI, front end (include/rvc_amd.h): ContentVec (rvc_amd/contentvec.py) and
// RMVPE (rvc_amd/rmvpe.py) loaded from their checkpoints' named host arrays and run natively with the same
// launches, pass sets and order as the Python models -- bit-identical to them on the same weights and
// constants.  Scratch per model is sized by a dry run of the forward (Scratch / RUN in model_common.h).
#include "host_f0file.h"
#include "model_common.h"

using namespace rvcm;

namespace fem {

constexpr int kMels = 128, kClass = 360, kNfft = 1024, kHop = 160;
constexpr int kFeLayers[7][3] = {{512, 10, 5}, {512, 3, 2}, {512, 3, 2}, {512, 3, 2}, {512, 3, 2}, {512, 2, 2}, {512, 2, 2}};

struct CvLayer {
    ConvW qkv, o, fc1, fc2;
    float *ln1g = nullptr, *ln1b = nullptr, *ln2g = nullptr, *ln2b = nullptr;
};

// f64 KM weights [Ci*K][Co] (+ bias) for rvc_conv64: the f64 RMVPE (rmvpe.py with precision "f64")
struct W64 {
    int64_t Co = 0, Ci = 0;
    int K = 0;
    double* w = nullptr;
    double* b = nullptr;
    double* v = nullptr;  // the Winograd F(4x4, 3x3) weights [36][Ci][Co] (rvc_wino64_use), else null
};

// ConvBlockRes (RMVPE.py:11-44) with BatchNorm folded: conv.0 -> ReLU, conv.3 -> ReLU + shortcut
// (c* for the f32 form, d* for the f64 form: one of the two sets is loaded)
struct Cbr {
    ConvW c0, c3, sc;
    W64 d0, d3, dsc;
    bool has_sc = false;
};

struct ConvT2d {  // ConvTranspose2d(3, stride 2, pad 1, out pad 1) + BN + ReLU as 4 phase convs
    ConvW ph[4];
    W64 ph64[4];
    int ntap[4];
    int dy[4][4], dx[4][4];
    int64_t Co = 0;
};

}  // namespace fem

struct ContentVec : ModelBase {
    int E = 768, heads = 12;
    ConvW fe[7], proj, pos_conv, final_proj;
    float *gn_w = nullptr, *gn_b = nullptr, *ln_w = nullptr, *ln_b = nullptr, *enc_ln_w = nullptr, *enc_ln_b = nullptr;
    std::vector<fem::CvLayer> layers;
};

struct Rmvpe : ModelBase {
    bool f64 = true;  // the f64 network (rmvpe64.hip) or the f32 one at the context's rm_prec
    ConvW mel, cnn, w_ih, fc;
    fem::W64 mel64, cnn64, w_ih64, fc64;
    float in_scale = 1.f, in_shift = 0.f;
    double in_scale64 = 1.0, in_shift64 = 0.0;
    float *window = nullptr, *w_hh = nullptr, *b_hh = nullptr;
    double *w_hh64 = nullptr, *b_hh64 = nullptr;
    std::vector<std::vector<fem::Cbr>> enc, inter;  // [level][block]
    std::vector<fem::ConvT2d> dec_t;
    std::vector<std::vector<fem::Cbr>> dec;
    void* gran = nullptr;
    int* err = nullptr;
};

void contentvec_delete(ContentVec* m) {
    if (!m) return;
    m->release();
    delete m;
}

void rmvpe_delete(Rmvpe* m) {
    if (!m) return;
    m->release();
    delete m;
}

namespace fem {

using rvcm::HostT;

int64_t cv_frames(int64_t n) {
    for (auto& l : kFeLayers) n = (n - l[1]) / l[2] + 1;
    return n;
}

// ------------------------------------------------------------------ ContentVec forward, one sequence
int cv_one(rvc_ctx* c, ContentVec& M, Scratch& sc, const float* wav, int64_t N, int out_layer, int final_proj,
           float* feats, hipStream_t s, bool cf_out = false) {
    const int64_t E = M.E;
    // feature extractor (fairseq.py:1165-1195): conv(k10 s5) + GroupNorm + GELU, then conv + GELU
    int64_t L = N;
    const float* x = wav;
    float* bufs[2];
    const int64_t L0 = (N - kFeLayers[0][1]) / kFeLayers[0][2] + 1;
    bufs[0] = sc.take(512 * L0);
    bufs[1] = sc.take(512 * L0);
    float* fe0ws = sc.take((rvc_fe0_ws_bytes(1, 512, L0) + 3) / 4);
    // |max| cells as contentvec.py (cv_amax): cell 0 the FE LayerNorm's, 1 the encoder LayerNorm's, then per layer i
    // 4 i + 2 .. 5 (attention, ln1, fc1, ln2), then (fe_amax) the feature extractor's layers 0-5; one memset per forward
    const int nl = out_layer < (int)M.layers.size() ? out_layer : (int)M.layers.size();
    const int nfe = 6;
    unsigned* cells = nullptr;
    if (c->cv_amax) {  // (+ one QKV cell per layer: contentvec.py's ATTN_F16)
        cells = reinterpret_cast<unsigned*>(sc.take((int64_t)(2 + 5 * nl + nfe) * RVC_AMAX_SHARDS));
        RUN(hipMemsetAsync(cells, 0, sizeof(unsigned) * (2 + 5 * nl + nfe) * RVC_AMAX_SHARDS, s) == hipSuccess
                ? RVC_OK
                : RVC_EHIP);
    }
    auto cell = [&](int k) { return cells ? cells + (int64_t)k * RVC_AMAX_SHARDS : nullptr; };
    auto fe_cell = [&](int i) { return c->fe_amax ? cell(2 + 4 * nl + i) : nullptr; };
    for (int i = 0; i < 7; ++i) {
        const int k = kFeLayers[i][1], st = kFeLayers[i][2];
        const int64_t Lo = (L - k) / st + 1;
        float* y = bufs[i & 1];
        if (i == 0) {  // conv + GroupNorm + GELU fused (rvc_fe0_gn_gelu, as contentvec.py)
            RUN(rvc_fe0_gn_gelu_amax(x, 1, L, 0, M.fe[0].w, 512, k, st, M.gn_w, M.gn_b, y, 1e-5f, 1, fe_cell(0), fe0ws,
                                     rvc_fe0_ws_bytes(1, 512, Lo), s));
        } else {
            CallOpts o;
            o.stride = st;
            o.out_act = RVC_ACT_GELU;
            o.amax_in = fe_cell(i - 1);
            o.amax_out = i < nfe ? fe_cell(i) : nullptr;
            RUN(conv(c, M, M.fe[i], x, L, y, o, s));
        }
        x = y;
        L = Lo;
    }
    const int64_t T = L;
    float* x512 = bufs[(7 - 1) & 1];  // layer 6's output
    RUN(rvc_layernorm_cf_amax(x512, nullptr, M.ln_w, M.ln_b, x512, 1, 512, T, 1e-5f, cell(0), s));
    float* xp = sc.take(E * T);
    {
        CallOpts o;
        o.amax_in = cell(0);
        RUN(conv(c, M, M.proj, x512, T, xp, o, s));
    }
    float* xe = sc.take(E * T);
    {
        CallOpts o;  // pos_conv: SamePad drops the last column; GELU then + x (fairseq.py:585-592)
        o.pad = M.pos_conv.K / 2;
        o.Lout = T;
        o.out_act = RVC_ACT_GELU;
        o.res = xp;
        RUN(conv(c, M, M.pos_conv, xp, T, xe, o, s));
    }
    RUN(rvc_layernorm_cf_amax(xe, nullptr, M.enc_ln_w, M.enc_ln_b, xe, 1, E, T, 1e-5f, cell(1), s));
    const int64_t H = M.heads, D = E / H;
    float* qkv = sc.take(3 * E * T);
    float* ob = sc.take(E * T);
    float* yb = sc.take(E * T);
    float* hb = sc.take(M.layers[0].fc1.Co * T);
    for (int li = 0; li < nl; ++li) {
        const CvLayer& Ly = M.layers[li];
        unsigned *c_in = cell(4 * li + 1), *c_at = cell(4 * li + 2), *c_l1 = cell(4 * li + 3),
                 *c_f1 = cell(4 * li + 4), *c_l2 = cell(4 * li + 5);
        unsigned* c_qkv = c->attn_f16 ? cell(2 + 4 * nl + nfe + li) : nullptr;
        CallOpts oq;
        oq.amax_in = c_in;
        oq.amax_out = c_qkv;
        RUN(conv(c, M, Ly.qkv, xe, T, qkv, oq, s));
        rvc_attn_args at;
        memset(&at, 0, sizeof(at));
        at.q = qkv;
        at.k = qkv + E * T;
        at.v = qkv + 2 * E * T;
        at.o = ob;
        at.B = 1;
        at.H = H;
        at.D = D;
        at.T = T;
        at.ldc = T;
        at.q_hs = at.k_hs = at.v_hs = at.o_hs = D * T;
        at.q_bs = at.k_bs = at.v_bs = 3 * E * T;
        at.o_bs = E * T;
        at.scale = (float)pow((double)D, -0.5);
        if (!sc.dry) {
            const int64_t need = rvc_attention_workspace_bytes(&at);
            MCHECK(need >= 0, "rvc_contentvec_forward: attention shape H=%lld D=%lld T=%lld unsupported", (long long)H,
                   (long long)D, (long long)T);
            MTRY(ensure_ws(M, need, s));
            MTRY(rvc_attention_ex(&at, c_qkv, c_at, need ? M.ws : nullptr, need, s));
        }
        CallOpts oo;
        oo.amax_in = c_at;
        RUN(conv(c, M, Ly.o, ob, T, yb, oo, s));
        RUN(rvc_layernorm_cf_amax(xe, yb, Ly.ln1g, Ly.ln1b, xe, 1, E, T, 1e-5f, c_l1, s));
        CallOpts og;
        og.out_act = RVC_ACT_GELU;
        og.amax_in = c_l1;
        og.amax_out = c_f1;
        RUN(conv(c, M, Ly.fc1, xe, T, hb, og, s));
        CallOpts o2;
        o2.amax_in = c_f1;
        RUN(conv(c, M, Ly.fc2, hb, T, yb, o2, s));
        RUN(rvc_layernorm_cf_amax(xe, yb, Ly.ln2g, Ly.ln2b, xe, 1, E, T, 1e-5f, c_l2, s));
    }
    if (final_proj && cf_out) {  // VC.features_device: final_proj on the channels-first features
        CallOpts o;
        RUN(conv(c, M, M.final_proj, xe, T, feats, o, s));
    } else if (final_proj) {
        float* fp = sc.take(M.final_proj.Co * T);
        CallOpts o;
        RUN(conv(c, M, M.final_proj, xe, T, fp, o, s));
        RUN(rvc_transpose(fp, feats, 1, M.final_proj.Co, T, s));
    } else if (cf_out) {
        RUN(hipMemcpyAsync(feats, xe, E * T * 4, hipMemcpyDeviceToDevice, s) == hipSuccess ? RVC_OK : RVC_EHIP);
    } else {
        RUN(rvc_transpose(xe, feats, 1, E, T, s));
    }
    return RVC_OK;
}

// ------------------------------------------------------------------ RMVPE pieces
// _fold_bn (rmvpe.py): s = g / sqrt(v + eps), shift = b - m s, in f64
int fold_bn(Params& P, const std::string& name, std::vector<double>& sc, std::vector<double>& sh) {
    HostT g, b, m, v;
    MCHECK(P.get(name + ".weight", g) && P.get(name + ".bias", b) && P.get(name + ".running_mean", m) &&
               P.get(name + ".running_var", v),
           "rvc_load_rmvpe: missing %s", P.missing.c_str());
    sc.resize(g.v.size());
    sh.resize(g.v.size());
    for (size_t i = 0; i < g.v.size(); ++i) {
        sc[i] = (double)g.v[i] / sqrt((double)v.v[i] + 1e-5);
        sh[i] = (double)b.v[i] - (double)m.v[i] * sc[i];
    }
    return RVC_OK;
}

int upload64(ModelBase& m, const std::vector<double>& h, double** out) {
    MTRY(dev_alloc(m, h.size() * 8, (void**)out));
    MHIP(hipMemcpy(*out, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    return RVC_OK;
}

// f64 KM weights from w laid out [Co][Ci][K] (times scale[co] in f64 when given) + an f64 bias (ops.Conv64)
int make_w64(Rmvpe& M, const HostT& w, int64_t Co, int64_t Ci, int K, const std::vector<double>* scale,
             const std::vector<double>* bias, W64& cw) {
    MCHECK((int64_t)w.v.size() == Co * Ci * K, "rvc_load_rmvpe: weight of %zu values, expected %lld x %lld x %d",
           w.v.size(), (long long)Co, (long long)Ci, K);
    cw.Co = Co;
    cw.Ci = Ci;
    cw.K = K;
    std::vector<double> km((size_t)Co * Ci * K);
    for (int64_t co = 0; co < Co; ++co)
        for (int64_t ci = 0; ci < Ci; ++ci)
            for (int t = 0; t < K; ++t) {
                const double v = (double)w.v[(co * Ci + ci) * K + t];
                km[(ci * K + t) * Co + co] = scale ? v * (*scale)[co] : v;
            }
    MTRY(upload64(M, km, &cw.w));
    if (bias) {
        MCHECK((int64_t)bias->size() == Co, "rvc_load_rmvpe: bias size %zu != %lld", bias->size(), (long long)Co);
        MTRY(upload64(M, *bias, &cw.b));
    }
    // the deep levels' 3x3 convs as Winograd F(4x4, 3x3), the same rule and transform as rmvpe.py's _Conv2d
    if (K == 9 && rvc_wino64_use(Ci, Co, 0, 0)) {
        MTRY(dev_alloc(M, (size_t)36 * Ci * Co * 8, (void**)&cw.v));
        MTRY(rvc_wino64_weights(cw.w, cw.v, Ci, Co, nullptr));
        MHIP(hipStreamSynchronize(nullptr));
    }
    return RVC_OK;
}

std::vector<double> to_f64(const std::vector<float>& v) { return std::vector<double>(v.begin(), v.end()); }

// 3x3 / 1x1 Conv2d weight [Co][Ci][kh][kw] (optionally scaled per output channel) as a K = kh*kw conv
int make_conv2d(rvc_ctx* c, Rmvpe& M, const HostT& w, const std::vector<double>* scale, const std::vector<float>& bias,
                ConvW& cw) {
    HostT w3;
    w3.shape = {w.dim(0), w.dim(1), w.dim(2) * w.dim(3)};
    w3.v.resize(w.v.size());
    const int64_t inner = (int64_t)w.v.size() / w.dim(0);
    for (int64_t co = 0; co < w.dim(0); ++co)
        for (int64_t j = 0; j < inner; ++j)
            w3.v[co * inner + j] = scale ? (float)((double)w.v[co * inner + j] * (*scale)[co]) : w.v[co * inner + j];
    HostT b;
    b.v = bias;
    b.shape = {(int64_t)bias.size()};
    return make_conv(c, M, w3, &b, cw);
}

int make_cbr(rvc_ctx* c, Rmvpe& M, Params& P, const std::string& p, Cbr& blk) {
    const char* convs[2][2] = {{"conv.0", "conv.1"}, {"conv.3", "conv.4"}};
    for (int i = 0; i < 2; ++i) {
        std::vector<double> s, t;
        MTRY(fold_bn(P, p + "." + convs[i][1], s, t));
        HostT w;
        MCHECK(P.get(p + "." + convs[i][0] + ".weight", w), "rvc_load_rmvpe: missing %s", P.missing.c_str());
        if (M.f64) {
            MTRY(make_w64(M, w, w.dim(0), w.dim(1), (int)(w.dim(2) * w.dim(3)), &s, &t, i == 0 ? blk.d0 : blk.d3));
        } else {
            std::vector<float> bf(t.begin(), t.end());
            MTRY(make_conv2d(c, M, w, &s, bf, i == 0 ? blk.c0 : blk.c3));
        }
    }
    if (P.has(p + ".shortcut.weight")) {
        HostT w, b;
        MCHECK(P.get(p + ".shortcut.weight", w) && P.get(p + ".shortcut.bias", b), "rvc_load_rmvpe: missing %s",
               P.missing.c_str());
        if (M.f64) {
            const std::vector<double> bd = to_f64(b.v);
            MTRY(make_w64(M, w, w.dim(0), w.dim(1), (int)(w.dim(2) * w.dim(3)), nullptr, &bd, blk.dsc));
        } else {
            MTRY(make_conv2d(c, M, w, nullptr, b.v, blk.sc));
        }
        blk.has_sc = true;
    }
    return RVC_OK;
}

int make_convT2d(rvc_ctx* c, Rmvpe& M, Params& P, const std::string& p, ConvT2d& ct) {
    std::vector<double> s, t;
    MTRY(fold_bn(P, p + ".conv1.1", s, t));
    HostT w;
    MCHECK(P.get(p + ".conv1.0.weight", w), "rvc_load_rmvpe: missing %s", P.missing.c_str());
    const int64_t Ci = w.dim(0), Co = w.dim(1);
    ct.Co = Co;
    // per output parity: (kernel index, source offset) -- rmvpe.py _ConvT2d.TAPS
    const int tk[2][2] = {{1, -1}, {0, 2}}, td[2][2] = {{0, 0}, {1, 0}}, tn[2] = {1, 2};
    HostT bias;
    bias.v.assign(t.begin(), t.end());
    bias.shape = {Co};
    int ph = 0;
    for (int py = 0; py < 2; ++py)
        for (int px = 0; px < 2; ++px, ++ph) {
            int n = 0;
            const int nt = tn[py] * tn[px];
            std::vector<double> wd((size_t)Co * Ci * nt);  // [Co][Ci][ntap], BN scale folded in f64
            for (int a = 0; a < tn[py]; ++a)
                for (int b2 = 0; b2 < tn[px]; ++b2, ++n) {
                    const int ky = tk[py][a], kx = tk[px][b2];
                    ct.dy[ph][n] = td[py][a];
                    ct.dx[ph][n] = td[px][b2];
                    for (int64_t co = 0; co < Co; ++co)
                        for (int64_t ci = 0; ci < Ci; ++ci)
                            wd[(co * Ci + ci) * nt + n] = (double)w.v[((ci * Co + co) * 3 + ky) * 3 + kx] * s[co];
                }
            ct.ntap[ph] = nt;
            if (M.f64) {
                W64& cw = ct.ph64[ph];
                cw.Co = Co;
                cw.Ci = Ci;
                cw.K = nt;
                std::vector<double> km((size_t)Co * Ci * nt);
                for (int64_t co = 0; co < Co; ++co)
                    for (int64_t ci = 0; ci < Ci; ++ci)
                        for (int q = 0; q < nt; ++q) km[(ci * nt + q) * Co + co] = wd[(co * Ci + ci) * nt + q];
                MTRY(upload64(M, km, &cw.w));
                MTRY(upload64(M, t, &cw.b));
            } else {
                HostT wp;
                wp.shape = {Co, Ci, nt};
                wp.v.resize(wd.size());
                for (size_t i = 0; i < wd.size(); ++i) wp.v[i] = (float)wd[i];
                MTRY(make_conv(c, M, wp, &bias, ct.ph[ph]));
            }
        }
    return RVC_OK;
}

// _Conv2d.__call__ on bordered [C][H+2][W+2] images
int conv2d(rvc_ctx* c, Rmvpe& M, const ConvW& cw, const float* x, int64_t H, int64_t W, float* out, int out_act,
           const float* res, hipStream_t s) {
    const int64_t wrap = W + 2, L = (H + 2) * wrap;
    CallOpts o;
    o.Lout = L;
    o.wrap = (int)wrap;
    o.out_act = out_act;
    o.res = res;
    if (cw.K == 9) {
        o.ntoff = 9;
        for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx) o.toff[dy * 3 + dx] = (int)(dy * wrap + dx);
        o.pad = (int)(wrap + 1);
    } else {
        o.ntoff = 1;
        o.toff[0] = 0;
        o.pad = 0;
    }
    return conv(c, M, cw, x, L, out, o, s);
}

int cbr_run(rvc_ctx* c, Rmvpe& M, Scratch& sc, const Cbr& blk, const float* x, int64_t H, int64_t W, float* out,
            hipStream_t s) {
    const int64_t img = (H + 2) * (W + 2);
    float* h = sc.take(blk.c0.Co * img);
    RUN(conv2d(c, M, blk.c0, x, H, W, h, RVC_ACT_RELU, nullptr, s));
    const float* res = x;
    if (blk.has_sc) {
        float* scb = sc.take(blk.c0.Co * img);
        RUN(conv2d(c, M, blk.sc, x, H, W, scb, RVC_ACT_NONE, nullptr, s));
        res = scb;
    }
    RUN(conv2d(c, M, blk.c3, h, H, W, out, RVC_ACT_RELU, res, s));
    return RVC_OK;
}

// mel -> U-Net -> BiGRU -> fc for one sequence (rmvpe.py f0_device up to the decode)
int rm_one(rvc_ctx* c, Rmvpe& M, Scratch& sc, const float* wav, int64_t N, float* sal, hipStream_t s) {
    const int64_t F = 1 + N / kHop, Tp = 32 * ((F - 1) / 32 + 1);
    // MelSpectrogram.forward (RMVPE.py:162-181): |STFT| in f64 (rvc_stft_mag), then the mel GEMM + log
    float* mag = sc.take((int64_t)(kNfft / 2 + 1) * F);
    RUN(rvc_stft_mag(wav, M.window, mag, 1, N, F, kNfft, kHop, 0, 0, s));
    float* mel = sc.take((int64_t)kMels * F);
    {
        CallOpts o;
        o.out_act = RVC_ACT_LOGCLAMP;
        o.out_slope = 1e-5f;
        RUN(conv(c, M, M.mel, mag, F, mel, o, s));
    }
    // mel2hidden input image (RMVPE.py:210-213)
    int64_t H = Tp, W = kMels;
    float* x = sc.take((H + 2) * (W + 2));
    RUN(hipMemsetAsync(x, 0, (H + 2) * (W + 2) * 4, s) == hipSuccess ? RVC_OK : RVC_EHIP);
    RUN(rvc_mel_image(mel, x, kMels, F, Tp, M.in_scale, M.in_shift, s));
    // encoder (RMVPE.py:64-76): the last block of each level writes into the decoder's concat buffer
    struct Cat {
        float* buf;
        int64_t C, H, W;
    };
    std::vector<Cat> cats;
    int64_t C = M.enc[0][0].c0.Co;
    const int nb = (int)M.enc[0].size();
    for (size_t l = 0; l < M.enc.size(); ++l) {
        const int64_t img = (H + 2) * (W + 2);
        float* cat = sc.take(2 * C * img);
        RUN(hipMemsetAsync(cat, 0, 2 * C * img * 4, s) == hipSuccess ? RVC_OK : RVC_EHIP);
        for (int b = 0; b < nb; ++b) {
            float* out = b == nb - 1 ? cat + C * img : sc.take(C * img);
            MTRY(cbr_run(c, M, sc, M.enc[l][b], x, H, W, out, s));
            x = out;
        }
        cats.push_back({cat, C, H, W});
        float* pooled = sc.take(C * (H / 2 + 2) * (W / 2 + 2));
        RUN(hipMemsetAsync(pooled, 0, C * (H / 2 + 2) * (W / 2 + 2) * 4, s) == hipSuccess ? RVC_OK : RVC_EHIP);
        RUN(rvc_avgpool2(x, pooled, C, H, W, s));
        x = pooled;
        H /= 2;
        W /= 2;
        C *= 2;
    }
    for (auto& layer : M.inter)
        for (auto& blk : layer) {
            float* out = sc.take(blk.c0.Co * (H + 2) * (W + 2));
            MTRY(cbr_run(c, M, sc, blk, x, H, W, out, s));
            x = out;
        }
    // decoder (RMVPE.py:78-107)
    for (size_t i = 0; i < M.dec_t.size(); ++i) {
        const Cat& ct = cats[cats.size() - 1 - i];
        const ConvT2d& T2 = M.dec_t[i];
        const int64_t wrap = W + 2, Lc = (H + 2) * wrap;
        float* ph = sc.take(4 * T2.Co * Lc);
        for (int p = 0; p < 4; ++p) {
            CallOpts o;
            o.Lout = Lc;
            o.wrap = (int)wrap;
            o.out_act = RVC_ACT_RELU;
            o.ntoff = T2.ntap[p];
            for (int t = 0; t < T2.ntap[p]; ++t) o.toff[t] = (int)(T2.dy[p][t] * wrap + T2.dx[p][t]);
            RUN(conv(c, M, T2.ph[p], x, Lc, ph + p * T2.Co * Lc, o, s));
        }
        RUN(rvc_interleave4(ph, ct.buf, T2.Co, H, W, s));
        x = ct.buf;
        H = ct.H;
        W = ct.W;
        for (auto& blk : M.dec[i]) {
            float* out = sc.take(blk.c0.Co * (H + 2) * (W + 2));
            MTRY(cbr_run(c, M, sc, blk, x, H, W, out, s));
            x = out;
        }
    }
    float* img = sc.take(3 * (H + 2) * (W + 2));
    RUN(conv2d(c, M, M.cnn, x, H, W, img, RVC_ACT_NONE, nullptr, s));
    float* seq = sc.take(3 * W * H);
    RUN(rvc_img_to_seq(img, seq, 3, H, W, s));
    // BiGRU + Linear + sigmoid (RMVPE.py:254-260, 141)
    float* gi = sc.take(1536 * Tp);
    {
        CallOpts o;
        RUN(conv(c, M, M.w_ih, seq, Tp, gi, o, s));
    }
    float* y = sc.take(512 * Tp);
    RUN(rvc_bigru(gi, M.w_hh, M.b_hh, y, M.gran, M.err, Tp, s));
    CallOpts o;
    o.out_act = RVC_ACT_SIGMOID;
    RUN(conv(c, M, M.fc, y, Tp, sal, o, s));
    return RVC_OK;
}

// ------------------------------------------------------------------ the f64 network (rmvpe.py, precision "f64")
struct C64Opts {
    int64_t Lout = -1;
    int pad = 0, out_act = RVC_ACT_NONE, y_f32 = 0, ntoff = 0, wrap = 0;
    int toff[16] = {0};
    double out_slope = 0.0;
    const double* res = nullptr;
};

int conv64(Rmvpe& M, const W64& cw, const double* x, int64_t Lin, void* y, const C64Opts& o, hipStream_t s) {
    rvc_conv64_args a;
    memset(&a, 0, sizeof(a));
    a.x = x;
    a.w = cw.w;
    a.bias = cw.b;
    a.res = o.res;
    a.y = y;
    a.B = 1;
    a.Ci = cw.Ci;
    a.Co = cw.Co;
    a.Lin = Lin;
    a.Lout = o.Lout >= 0 ? o.Lout : Lin + 2 * o.pad - (cw.K - 1);
    a.K = cw.K;
    a.pad = o.pad;
    a.out_act = o.out_act;
    a.y_f32 = o.y_f32;
    a.out_slope = o.out_slope;
    a.ntoff = o.ntoff;
    a.wrap = o.wrap;
    for (int i = 0; i < o.ntoff; ++i) a.toff[i] = o.toff[i];
    const int64_t need = rvc_conv64_workspace_bytes(&a);
    if (need < 0) return RVC_EINVAL;
    MTRY(ensure_ws(M, need, s));
    return rvc_conv64(&a, need ? M.ws : nullptr, need, s);
}

// _Conv2d.__call__ (f64) on bordered [C][H+2][W+2] images
int conv2d64(Rmvpe& M, const W64& cw, const double* x, int64_t H, int64_t W, double* out, int out_act,
             const double* res, hipStream_t s) {
    if (cw.v && rvc_wino64_use(cw.Ci, cw.Co, H, W)) {
        rvc_wino64_args a;
        memset(&a, 0, sizeof(a));
        a.x = x;
        a.v = cw.v;
        a.bias = cw.b;
        a.res = res;
        a.y = out;
        a.B = 1;
        a.Ci = cw.Ci;
        a.Co = cw.Co;
        a.H = H;
        a.W = W;
        a.out_act = out_act;
        const int64_t need = rvc_wino64_workspace_bytes(&a);
        if (need < 0) return RVC_EINVAL;
        MTRY(ensure_ws(M, need, s));
        return rvc_wino64_conv(&a, M.ws, need, s);
    }
    const int64_t wrap = W + 2, L = (H + 2) * wrap;
    C64Opts o;
    o.Lout = L;
    o.wrap = (int)wrap;
    o.out_act = out_act;
    o.res = res;
    if (cw.K == 9) {
        o.ntoff = 9;
        for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx) o.toff[dy * 3 + dx] = (int)(dy * wrap + dx);
        o.pad = (int)(wrap + 1);
    } else {
        o.ntoff = 1;
    }
    return conv64(M, cw, x, L, out, o, s);
}

double* take64(Scratch& sc, int64_t n) { return (double*)sc.take(2 * n); }

int cbr_run64(Rmvpe& M, Scratch& sc, const Cbr& blk, const double* x, int64_t H, int64_t W, double* out,
              hipStream_t s) {
    const int64_t img = (H + 2) * (W + 2);
    double* h = take64(sc, blk.d0.Co * img);
    RUN(conv2d64(M, blk.d0, x, H, W, h, RVC_ACT_RELU, nullptr, s));
    const double* res = x;
    if (blk.has_sc) {
        double* scb = take64(sc, blk.d0.Co * img);
        RUN(conv2d64(M, blk.dsc, x, H, W, scb, RVC_ACT_NONE, nullptr, s));
        res = scb;
    }
    RUN(conv2d64(M, blk.d3, h, H, W, out, RVC_ACT_RELU, res, s));
    return RVC_OK;
}

// rm_one in f64: the same launch sequence as RMVPEAMD's f64 form, the salience rounded to f32 once
int rm_one64(rvc_ctx* c, Rmvpe& M, Scratch& sc, const float* wav, int64_t N, float* sal, hipStream_t s) {
    const int64_t F = 1 + N / kHop, Tp = 32 * ((F - 1) / 32 + 1);
    double* mag = take64(sc, (int64_t)(kNfft / 2 + 1) * F);
    RUN(rvc_stft_mag64(wav, M.window, mag, 1, N, F, kNfft, kHop, 0, 0, s));
    double* mel = take64(sc, (int64_t)kMels * F);
    {
        C64Opts o;
        o.out_act = RVC_ACT_LOGCLAMP;
        o.out_slope = 1e-5;
        RUN(conv64(M, M.mel64, mag, F, mel, o, s));
    }
    int64_t H = Tp, W = kMels;
    double* x = take64(sc, (H + 2) * (W + 2));
    RUN(rvc_mel_image64(mel, x, 1, kMels, F, Tp, M.in_scale64, M.in_shift64, 0, 0, s));
    struct Cat {
        double* buf;
        int64_t C, H, W;
    };
    std::vector<Cat> cats;
    int64_t C = M.enc[0][0].d0.Co;
    const int nb = (int)M.enc[0].size();
    for (size_t l = 0; l < M.enc.size(); ++l) {
        const int64_t img = (H + 2) * (W + 2);
        double* cat = take64(sc, 2 * C * img);
        for (int b = 0; b < nb; ++b) {
            double* out = b == nb - 1 ? cat + C * img : take64(sc, C * img);
            MTRY(cbr_run64(M, sc, M.enc[l][b], x, H, W, out, s));
            x = out;
        }
        cats.push_back({cat, C, H, W});
        double* pooled = take64(sc, C * (H / 2 + 2) * (W / 2 + 2));
        RUN(rvc_avgpool2_64(x, pooled, 1, C, H, W, 0, 0, s));
        x = pooled;
        H /= 2;
        W /= 2;
        C *= 2;
    }
    for (auto& layer : M.inter)
        for (auto& blk : layer) {
            double* out = take64(sc, blk.d0.Co * (H + 2) * (W + 2));
            MTRY(cbr_run64(M, sc, blk, x, H, W, out, s));
            x = out;
        }
    for (size_t i = 0; i < M.dec_t.size(); ++i) {
        const Cat& ct = cats[cats.size() - 1 - i];
        const ConvT2d& T2 = M.dec_t[i];
        const int64_t wrap = W + 2, Lc = (H + 2) * wrap;
        double* ph = take64(sc, 4 * T2.Co * Lc);
        for (int p = 0; p < 4; ++p) {
            C64Opts o;
            o.Lout = Lc;
            o.wrap = (int)wrap;
            o.out_act = RVC_ACT_RELU;
            o.ntoff = T2.ntap[p];
            for (int t = 0; t < T2.ntap[p]; ++t) o.toff[t] = (int)(T2.dy[p][t] * wrap + T2.dx[p][t]);
            RUN(conv64(M, T2.ph64[p], x, Lc, ph + p * T2.Co * Lc, o, s));
        }
        RUN(rvc_interleave4_64(ph, ct.buf, 1, T2.Co, H, W, 0, 0, s));
        x = ct.buf;
        H = ct.H;
        W = ct.W;
        for (auto& blk : M.dec[i]) {
            double* out = take64(sc, blk.d0.Co * (H + 2) * (W + 2));
            MTRY(cbr_run64(M, sc, blk, x, H, W, out, s));
            x = out;
        }
    }
    double* img = take64(sc, 3 * (H + 2) * (W + 2));
    RUN(conv2d64(M, M.cnn64, x, H, W, img, RVC_ACT_NONE, nullptr, s));
    double* seq = take64(sc, 3 * W * H);
    RUN(rvc_img_to_seq64(img, seq, 1, 3, H, W, 0, 0, s));
    double* gi = take64(sc, 1536 * Tp);
    {
        C64Opts o;
        RUN(conv64(M, M.w_ih64, seq, Tp, gi, o, s));
    }
    double* y = take64(sc, 512 * Tp);
    RUN(rvc_bigru64_batched(gi, 0, M.w_hh64, M.b_hh64, y, 0, M.gran, M.err, 1, Tp, s));
    C64Opts o;
    o.out_act = RVC_ACT_SIGMOID;
    o.y_f32 = 1;
    RUN(conv64(M, M.fc64, y, Tp, sal, o, s));
    return RVC_OK;
}

}  // namespace fem

using namespace fem;

// ------------------------------------------------------------------ C ABI
extern "C" int64_t rvc_contentvec_frames(int64_t n16k) { return n16k >= 400 ? cv_frames(n16k) : 0; }

extern "C" int rvc_load_contentvec(rvc_ctx* c, const rvc_param* params, int n, const rvc_contentvec_cfg* cfg) {
    MCHECK(c && params && n > 0 && cfg, "rvc_load_contentvec: null argument");
    MCHECK(cfg->encoder_embed_dim > 0 && cfg->encoder_attention_heads > 0 &&
               cfg->encoder_embed_dim % cfg->encoder_attention_heads == 0 && cfg->conv_pos_groups > 0,
           "rvc_load_contentvec: bad cfg");
    Params P;
    P.wn_dim = 2;  // encoder.pos_conv: weight_norm(dim=2) (fairseq.py:585-592)
    MTRY(index_params(params, n, P, "rvc_load_contentvec"));
    MHIP(hipSetDevice(c->device));
    contentvec_delete(c->cv);
    c->cv = new ContentVec();
    ContentVec& M = *c->cv;
    M.E = cfg->encoder_embed_dim;
    M.heads = cfg->encoder_attention_heads;
    HostT w, b;
#define GET(k, t) MCHECK(P.get(k, t), "rvc_load_contentvec: missing %s", P.missing.c_str())
    for (int i = 0; i < 7; ++i) {
        GET("feature_extractor.conv_layers." + std::to_string(i) + ".0.weight", w);
        MTRY(make_conv(c, M, w, nullptr, M.fe[i]));
    }
    GET("feature_extractor.conv_layers.0.2.weight", w);
    MTRY(upload(M, w.v, &M.gn_w));
    GET("feature_extractor.conv_layers.0.2.bias", w);
    MTRY(upload(M, w.v, &M.gn_b));
    GET("layer_norm.weight", w);
    MTRY(upload(M, w.v, &M.ln_w));
    GET("layer_norm.bias", w);
    MTRY(upload(M, w.v, &M.ln_b));
    GET("post_extract_proj.weight", w);
    GET("post_extract_proj.bias", b);
    w.shape.push_back(1);
    MTRY(make_conv(c, M, w, &b, M.proj));
    GET("encoder.pos_conv.0.weight", w);
    GET("encoder.pos_conv.0.bias", b);
    MTRY(make_conv(c, M, w, &b, M.pos_conv, cfg->conv_pos_groups));
    GET("encoder.layer_norm.weight", w);
    MTRY(upload(M, w.v, &M.enc_ln_w));
    GET("encoder.layer_norm.bias", w);
    MTRY(upload(M, w.v, &M.enc_ln_b));
    for (int i = 0; P.has("encoder.layers." + std::to_string(i) + ".fc1.weight"); ++i) {
        const std::string p = "encoder.layers." + std::to_string(i) + ".";
        CvLayer Ly;
        HostT wq, wk, wv, bq, bk, bv;
        GET(p + "self_attn.q_proj.weight", wq);
        GET(p + "self_attn.k_proj.weight", wk);
        GET(p + "self_attn.v_proj.weight", wv);
        GET(p + "self_attn.q_proj.bias", bq);
        GET(p + "self_attn.k_proj.bias", bk);
        GET(p + "self_attn.v_proj.bias", bv);
        wq.v.insert(wq.v.end(), wk.v.begin(), wk.v.end());
        wq.v.insert(wq.v.end(), wv.v.begin(), wv.v.end());
        wq.shape = {wq.dim(0) + wk.dim(0) + wv.dim(0), wq.dim(1), 1};
        bq.v.insert(bq.v.end(), bk.v.begin(), bk.v.end());
        bq.v.insert(bq.v.end(), bv.v.begin(), bv.v.end());
        MTRY(make_conv(c, M, wq, &bq, Ly.qkv));
        const char* lin[3][2] = {{"self_attn.out_proj", "o"}, {"fc1", "fc1"}, {"fc2", "fc2"}};
        ConvW* dst[3] = {&Ly.o, &Ly.fc1, &Ly.fc2};
        for (int j = 0; j < 3; ++j) {
            GET(p + lin[j][0] + ".weight", w);
            GET(p + lin[j][0] + ".bias", b);
            w.shape.push_back(1);
            MTRY(make_conv(c, M, w, &b, *dst[j]));
        }
        GET(p + "self_attn_layer_norm.weight", w);
        MTRY(upload(M, w.v, &Ly.ln1g));
        GET(p + "self_attn_layer_norm.bias", w);
        MTRY(upload(M, w.v, &Ly.ln1b));
        GET(p + "final_layer_norm.weight", w);
        MTRY(upload(M, w.v, &Ly.ln2g));
        GET(p + "final_layer_norm.bias", w);
        MTRY(upload(M, w.v, &Ly.ln2b));
        M.layers.push_back(Ly);
    }
    MCHECK(!M.layers.empty(), "rvc_load_contentvec: no encoder.layers.*");
    GET("final_proj.weight", w);
    GET("final_proj.bias", b);
    w.shape.push_back(1);
    MTRY(make_conv(c, M, w, &b, M.final_proj));
#undef GET
    MHIP(hipDeviceSynchronize());
    M.loaded = true;
    return RVC_OK;
}

extern "C" int rvc_contentvec_forward(rvc_ctx* c, const float* wav, int64_t B, int64_t N, int out_layer, int final_proj,
                                      float* feats, rvc_stream_t stream) {
    MCHECK(c && c->cv && c->cv->loaded, "rvc_contentvec_forward: no ContentVec loaded");
    MCHECK(wav && feats && B >= 1 && out_layer >= 1, "rvc_contentvec_forward: bad arguments");
    const int64_t T = rvc_contentvec_frames(N);
    MCHECK(T >= 1, "rvc_contentvec_forward: input of %lld samples is shorter than one frame", (long long)N);
    hipStream_t s = (hipStream_t)stream;
    MHIP(hipSetDevice(c->device));
    ContentVec& M = *c->cv;
    Scratch sc;
    MTRY(cv_one(c, M, sc, wav, N, out_layer, final_proj, feats, s));  // dry: size the scratch
    MTRY(ensure_arena(M, sc.off, s));
    const int64_t Cout = final_proj ? M.final_proj.Co : M.E;
    for (int64_t b = 0; b < B; ++b) {
        Scratch run;
        run.dry = false;
        run.base = M.arena;
        MTRY(cv_one(c, M, run, wav + b * N, N, out_layer, final_proj, feats + b * T * Cout, s));
    }
    return RVC_OK;
}

extern "C" int64_t rvc_rmvpe_frames(int64_t n16k) { return n16k >= 0 ? 1 + n16k / kHop : -1; }

extern "C" int64_t rvc_rmvpe_salience_ld(int64_t n16k) {
    const int64_t F = rvc_rmvpe_frames(n16k);
    return F > 0 ? 32 * ((F - 1) / 32 + 1) : -1;
}

extern "C" int rvc_load_rmvpe(rvc_ctx* c, const rvc_param* params, int n) {
    MCHECK(c && params && n > 0, "rvc_load_rmvpe: null argument");
    Params P;
    MTRY(index_params(params, n, P, "rvc_load_rmvpe"));
    MHIP(hipSetDevice(c->device));
    rmvpe_delete(c->rm);
    c->rm = new Rmvpe();
    Rmvpe& M = *c->rm;
    M.f64 = c->rm_prec == RVC_PREC_FP64;
    HostT w, b;
#define GET(k, t) MCHECK(P.get(k, t), "rvc_load_rmvpe: missing %s", P.missing.c_str())
    // constants: Hann window, mel basis (rmvpe.py __init__, melbasis.py)
    if (P.has("window")) {
        GET("window", w);
        MCHECK((int64_t)w.v.size() == kNfft, "rvc_load_rmvpe: window must have %d entries", kNfft);
    } else {
        w.v.resize(kNfft);  // torch.hann_window's float32 steps (periodic: n * 2 pi / N, cos, * -0.5, + 0.5)
        const float step = (float)(M_PI * 2.0 / kNfft);
        for (int i = 0; i < kNfft; ++i) {
#pragma clang fp contract(off)
            const float cs = (float)cos((double)((float)i * step));
            const float t = cs * -0.5f;
            w.v[i] = t + 0.5f;
        }
    }
    MTRY(upload(M, w.v, &M.window));
    HostT mb;
    if (P.has("mel_basis")) {
        GET("mel_basis", mb);
        MCHECK(mb.dim(0) == kMels && mb.dim(1) == kNfft / 2 + 1, "rvc_load_rmvpe: mel_basis must be [128][513]");
    } else {  // librosa.filters.mel(16000, 1024, 128, 30, 8000, htk=True), Slaney norm (melbasis.py)
        const int nb = kNfft / 2 + 1;
        auto hz2mel = [](double f) { return 2595.0 * log10(1.0 + f / 700.0); };
        auto mel2hz = [](double m) { return 700.0 * (pow(10.0, m / 2595.0) - 1.0); };
        const double m0 = hz2mel(30.0), m1 = hz2mel(8000.0), step = (m1 - m0) / (kMels + 1);
        std::vector<double> mf(kMels + 2), ff(nb);
        for (int i = 0; i < kMels + 2; ++i) mf[i] = mel2hz(i == kMels + 1 ? m1 : i * step + m0);
        const double val = 1.0 / (kNfft * (1.0 / 16000.0));
        for (int k = 0; k < nb; ++k) ff[k] = k * val;
        mb.shape = {kMels, nb};
        mb.v.resize((size_t)kMels * nb);
        for (int i = 0; i < kMels; ++i) {
            const double enorm = 2.0 / (mf[i + 2] - mf[i]);
            for (int k = 0; k < nb; ++k) {
                const double lower = -(mf[i] - ff[k]) / (mf[i + 1] - mf[i]);
                const double upper = (mf[i + 2] - ff[k]) / (mf[i + 2] - mf[i + 1]);
                const float wt = (float)fmax(0.0, fmin(lower, upper));
                mb.v[(size_t)i * nb + k] = (float)((double)wt * enorm);
            }
        }
    }
    mb.shape.push_back(1);
    if (M.f64) MTRY(make_w64(M, mb, kMels, kNfft / 2 + 1, 1, nullptr, nullptr, M.mel64));
    else MTRY(make_conv(c, M, mb, nullptr, M.mel));
    {
        std::vector<double> s, t;
        MTRY(fold_bn(P, "unet.encoder.bn", s, t));
        M.in_scale = (float)s[0];
        M.in_shift = (float)t[0];
        M.in_scale64 = s[0];
        M.in_shift64 = t[0];
    }
    const int nblk = 4;  // E2E(4, 1, (2, 2))
    for (int l = 0; P.has("unet.encoder.layers." + std::to_string(l) + ".conv.0.conv.0.weight"); ++l) {
        M.enc.emplace_back(nblk);
        for (int bb = 0; bb < nblk; ++bb)
            MTRY(make_cbr(c, M, P, "unet.encoder.layers." + std::to_string(l) + ".conv." + std::to_string(bb),
                          M.enc.back()[bb]));
    }
    for (int l = 0; P.has("unet.intermediate.layers." + std::to_string(l) + ".conv.0.conv.0.weight"); ++l) {
        M.inter.emplace_back(nblk);
        for (int bb = 0; bb < nblk; ++bb)
            MTRY(make_cbr(c, M, P, "unet.intermediate.layers." + std::to_string(l) + ".conv." + std::to_string(bb),
                          M.inter.back()[bb]));
    }
    for (int l = 0; P.has("unet.decoder.layers." + std::to_string(l) + ".conv1.0.weight"); ++l) {
        const std::string p = "unet.decoder.layers." + std::to_string(l);
        M.dec_t.emplace_back();
        MTRY(make_convT2d(c, M, P, p, M.dec_t.back()));
        M.dec.emplace_back(nblk);
        for (int bb = 0; bb < nblk; ++bb) MTRY(make_cbr(c, M, P, p + ".conv2." + std::to_string(bb), M.dec.back()[bb]));
    }
    MCHECK(M.enc.size() == 5 && M.dec.size() == 5 && (M.f64 ? M.enc[0][0].d0.Ci : M.enc[0][0].c0.Ci) == 1,
           "rvc_load_rmvpe: expected the E2E(4, 1, (2, 2)) U-Net (5 encoder / decoder levels)");
    GET("cnn.weight", w);
    GET("cnn.bias", b);
    if (M.f64) {
        const std::vector<double> bd = to_f64(b.v);
        MTRY(make_w64(M, w, w.dim(0), w.dim(1), (int)(w.dim(2) * w.dim(3)), nullptr, &bd, M.cnn64));
    } else {
        MTRY(make_conv2d(c, M, w, nullptr, b.v, M.cnn));
    }
    const std::string g = "fc.0.gru.";
    HostT wi, wir, bi, bir;
    GET(g + "weight_ih_l0", wi);
    GET(g + "weight_ih_l0_reverse", wir);
    GET(g + "bias_ih_l0", bi);
    GET(g + "bias_ih_l0_reverse", bir);
    MCHECK(wi.dim(0) == 768 && wi.dim(1) == 384, "rvc_load_rmvpe: GRU(384, 256) expected");
    wi.v.insert(wi.v.end(), wir.v.begin(), wir.v.end());
    wi.shape = {1536, 384, 1};
    bi.v.insert(bi.v.end(), bir.v.begin(), bir.v.end());
    if (M.f64) {
        const std::vector<double> bd = to_f64(bi.v);
        MTRY(make_w64(M, wi, 1536, 384, 1, nullptr, &bd, M.w_ih64));
    } else {
        MTRY(make_conv(c, M, wi, &bi, M.w_ih));
    }
    HostT wh, whr, bh, bhr;
    GET(g + "weight_hh_l0", wh);
    GET(g + "weight_hh_l0_reverse", whr);
    GET(g + "bias_hh_l0", bh);
    GET(g + "bias_hh_l0_reverse", bhr);
    wh.v.insert(wh.v.end(), whr.v.begin(), whr.v.end());
    bh.v.insert(bh.v.end(), bhr.v.begin(), bhr.v.end());
    if (M.f64) {
        MTRY(upload64(M, to_f64(wh.v), &M.w_hh64));
        MTRY(upload64(M, to_f64(bh.v), &M.b_hh64));
    } else {
        MTRY(upload(M, wh.v, &M.w_hh));
        MTRY(upload(M, bh.v, &M.b_hh));
    }
    GET("fc.1.weight", w);
    GET("fc.1.bias", b);
    MCHECK(w.dim(0) == kClass && w.dim(1) == 512, "rvc_load_rmvpe: fc.1 must be Linear(512, 360)");
    w.shape.push_back(1);
    if (M.f64) {
        const std::vector<double> bd = to_f64(b.v);
        MTRY(make_w64(M, w, kClass, 512, 1, nullptr, &bd, M.fc64));
    } else {
        MTRY(make_conv(c, M, w, &b, M.fc));
    }
#undef GET
    MTRY(dev_alloc(M, RVC_BIGRU64_GRAN_BYTES, &M.gran));
    MTRY(dev_alloc(M, 4, (void**)&M.err));
    MHIP(hipMemset(M.err, 0, 4));
    MHIP(hipDeviceSynchronize());
    M.loaded = true;
    return RVC_OK;
}

extern "C" int rvc_rmvpe_forward(rvc_ctx* c, const float* wav, int64_t B, int64_t N, float* salience,
                                 rvc_stream_t stream) {
    MCHECK(c && c->rm && c->rm->loaded, "rvc_rmvpe_forward: no RMVPE loaded");
    MCHECK(wav && salience && B >= 1 && N >= 1, "rvc_rmvpe_forward: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    MHIP(hipSetDevice(c->device));
    Rmvpe& M = *c->rm;
    const int prev = c->prec;
    // the f32 form runs at the RMVPE precision it was loaded for, whatever the context's conv precision
    // (rmvpe.py: self.precision); the f64 form has its own engine
    if (!M.f64) c->prec = c->rm_prec;
    auto one = [&](Scratch& scr, const float* x, float* sal) {
        return M.f64 ? rm_one64(c, M, scr, x, N, sal, s) : rm_one(c, M, scr, x, N, sal, s);
    };
    Scratch sc;
    int rc = one(sc, wav, salience);
    if (rc == RVC_OK) rc = ensure_arena(M, sc.off, s);
    const int64_t ld = rvc_rmvpe_salience_ld(N);
    for (int64_t b = 0; b < B && rc == RVC_OK; ++b) {
        Scratch run;
        run.dry = false;
        run.base = M.arena;
        rc = one(run, wav + b * N, salience + b * kClass * ld);
    }
    c->prec = prev;
    return rc;
}

extern "C" int rvc_ctx_set_rmvpe_precision(rvc_ctx* c, int prec) {
    MCHECK(c, "rvc_ctx_set_rmvpe_precision: null ctx");
    MCHECK(prec == RVC_PREC_FP64 || prec == RVC_PREC_FP32 || prec == RVC_PREC_BF16 || prec == RVC_PREC_BF16X3 ||
               prec == RVC_PREC_FP32X6 || prec == RVC_PREC_FP32SA || prec == RVC_PREC_F16X3,
           "rvc_ctx_set_rmvpe_precision: unknown precision %d", prec);
    c->rm_prec = prec;
    return RVC_OK;
}

extern "C" int rvc_rmvpe_check(rvc_ctx* c) {
    MCHECK(c && c->rm && c->rm->loaded, "rvc_rmvpe_check: no RMVPE loaded");
    MHIP(hipSetDevice(c->device));
    int e = 0;
    MHIP(hipMemcpy(&e, c->rm->err, 4, hipMemcpyDeviceToHost));
    if (e != 0) {
        MHIP(hipMemset(c->rm->err, 0, 4));
        rvc_set_error("rvc_rmvpe_check: bigru recurrence timed out (granule hand-off stalled); salience invalid");
        return RVC_EHIP;
    }
    return RVC_OK;
}

// ------------------------------------------------------------------ CREPE (rvc_amd/crepe.py)
struct Crepe : ModelBase {
    ConvW conv[6], classifier;
    float *alpha[6] = {nullptr}, *beta[6] = {nullptr};
    double* log_trans = nullptr;
    double log_off = 0, log_p_init = 0;
    int lo = 0, hi = 0;
    std::map<int64_t, int64_t*> seq_off;  // per length T: batch offsets, resident (uploaded once)
};

void crepe_delete(Crepe* m) {
    if (!m) return;
    m->release();
    delete m;
}

namespace fem {

constexpr int kCrepeBatch = 512;  // predict(batch_size=512): the Viterbi runs per batch

// _freq_to_bin (crepe.py, CREPE.py:120-121) in f32 steps: ((1200 log2(f / 10)) - 1997.379...) / 20
int crepe_bin(float f, bool up) {
#pragma clang fp contract(off)
    const float a = f / 10.f;
    const float l = log2f(a);
    const float c = 1200.f * l;
    const float d = c - (float)1997.3794084376191;
    const float e = d / 20.f;
    return (int)(up ? ceilf(e) : floorf(e));
}

// sigmoid outputs of frames [frame0, frame0 + nb) -> out [360][nb] (CrepeAMD.probabilities)
int crepe_batch(rvc_ctx* c, Crepe& M, Scratch& sc, const float* audio, int64_t N, int64_t frame0, int64_t nb, float* out,
                hipStream_t s) {
    float* frames = sc.take(nb * 1024);
    RUN(rvc_crepe_frames(audio, N, kHop, frame0, nb, frames, s));
    const float* x = frames;
    int64_t L = 1024;
    for (int i = 0; i < 6; ++i) {
        const ConvW& cw = M.conv[i];
        CallOpts o;
        o.B = nb;
        o.out_act = RVC_ACT_RELU;
        int64_t Lout;
        if (i == 0) {
            Lout = (L + 2 * 254 - 512) / 4 + 1;
            o.stride = 4;
            o.pad = 254;
            o.x_bstride = L;
        } else {
            Lout = L;  // pad (31, 32) with k = 64
            o.pad = 31;
            o.x_bstride = cw.Ci * L;
        }
        o.Lout = Lout;
        float* y = sc.take(nb * cw.Co * Lout);
        RUN(conv(c, M, cw, x, L, y, o, s));
        const int64_t Lp = Lout / 2;
        float* h = sc.take(nb * cw.Co * Lp);
        if (i < 5) {
            RUN(rvc_bn_maxpool(y, nb, cw.Co, Lout, M.alpha[i], M.beta[i], h, cw.Co * Lp, Lp, 1, s));
        } else {  // classifier input [c * Lp + h][frame]
            RUN(rvc_bn_maxpool(y, nb, cw.Co, Lout, M.alpha[i], M.beta[i], h, 1, Lp * nb, nb, s));
        }
        x = h;
        L = Lp;
    }
    CallOpts o;
    o.out_act = RVC_ACT_SIGMOID;
    RUN(conv(c, M, M.classifier, x, nb, out, o, s));
    return RVC_OK;
}

int crepe_run(rvc_ctx* c, Crepe& M, Scratch& sc, const float* audio, int64_t N, const float* dither, uint64_t seed,
              double pitch_shift, const rvc_f0_post* post, float* probs_out, int64_t* coarse, float* pitchf,
              const int64_t* seq_off, hipStream_t s) {
    const int64_t T = 1 + N / kHop;
    float* probs = sc.take(kClass * T);
    float* pb = sc.take(kClass * (T < kCrepeBatch ? T : kCrepeBatch));
    int nseq = 0;
    for (int64_t a = 0; a < T; a += kCrepeBatch, ++nseq) {
        const int64_t b = a + kCrepeBatch < T ? a + kCrepeBatch : T;
        MTRY(crepe_batch(c, M, sc, audio, N, a, b - a, pb, s));
        RUN(hipMemcpy2DAsync(probs + a, T * 4, pb, (b - a) * 4, (b - a) * 4, kClass, hipMemcpyDeviceToDevice, s) ==
                    hipSuccess
                ? RVC_OK
                : RVC_EHIP);
    }
    if (!dither) {
        float* d = sc.take(T);
        RUN(rvc_rand_triang(d, T, -20.f, 20.f, seed, 0, nullptr, s));
        dither = d;
    }
    const int64_t need = rvc_crepe_decode_ws_bytes(T);
    float* f0r = sc.take(T);
    float* pdr = sc.take(T);
    if (!sc.dry) {
        // the sigmoid outputs before the decode masks them in place outside [lo, hi)
        if (probs_out) MHIP(hipMemcpyAsync(probs_out, probs, kClass * T * 4, hipMemcpyDeviceToDevice, s));
        MTRY(ensure_ws(M, need, s));
        MTRY(rvc_crepe_decode(probs, T, M.lo, M.hi, seq_off, nseq, M.log_trans, M.log_off, M.log_p_init, dither, M.ws,
                              need, f0r, pdr, s));
    }
    const double mel_min = 1127 * log(1 + 50.0 / 700), mel_max = 1127 * log(1 + 1100.0 / 700);
    RUN(rvc_crepe_smooth_coarse(f0r, pdr, T, (float)pow(2.0, pitch_shift / 12), mel_min, mel_max, post, coarse, pitchf,
                                s));
    return RVC_OK;
}

}  // namespace fem

extern "C" int rvc_load_crepe(rvc_ctx* c, const rvc_param* params, int n) {
    MCHECK(c && params && n > 0, "rvc_load_crepe: null argument");
    Params P;
    MTRY(index_params(params, n, P, "rvc_load_crepe"));
    MHIP(hipSetDevice(c->device));
    crepe_delete(c->cr);
    c->cr = new Crepe();
    Crepe& M = *c->cr;
    HostT w, b;
#define GET(k, t) MCHECK(P.get(k, t), "rvc_load_crepe: missing %s", P.missing.c_str())
    const float eps = 0.0010000000474974513f;  // BatchNorm eps 1e-3 as f32 (crepe.py BN_EPS)
    for (int i = 0; i < 6; ++i) {
        const std::string si = std::to_string(i + 1);
        GET("conv" + si + ".weight", w);  // [Co][Ci][k][1]
        GET("conv" + si + ".bias", b);
        MCHECK(w.shape.size() == 4 && w.dim(3) == 1, "rvc_load_crepe: conv%s.weight must be [Co][Ci][k][1]", si.c_str());
        w.shape.pop_back();
        MTRY(make_conv(c, M, w, &b, M.conv[i]));
        HostT g, bb, mu, var;
        const std::string p = "conv" + si + "_BN.";
        GET(p + "weight", g);
        GET(p + "bias", bb);
        GET(p + "running_mean", mu);
        GET(p + "running_var", var);
        std::vector<float> al(g.v.size()), be(g.v.size());
        for (size_t k = 0; k < g.v.size(); ++k) {  // f32 like torch: invstd, alpha = w invstd, beta = b - mean alpha
#pragma clang fp contract(off)
            const float inv = 1.0f / sqrtf(var.v[k] + eps);
            al[k] = g.v[k] * inv;
            const float ma = mu.v[k] * al[k];
            be[k] = bb.v[k] - ma;
        }
        if (P.has(p + "alpha") && P.has(p + "beta")) {  // a host's own fold (torch's CPU sqrt is not IEEE-exact)
            HostT a2, b2;
            GET(p + "alpha", a2);
            GET(p + "beta", b2);
            MCHECK(a2.v.size() == al.size() && b2.v.size() == be.size(), "rvc_load_crepe: %salpha/beta size", p.c_str());
            al = a2.v;
            be = b2.v;
        }
        MTRY(upload(M, al, &M.alpha[i]));
        MTRY(upload(M, be, &M.beta[i]));
    }
    MCHECK(M.conv[0].K == 512 && M.conv[0].Ci == 1, "rvc_load_crepe: conv1 must be Conv2d(1, C, (512, 1), stride 4)");
    GET("classifier.weight", w);
    GET("classifier.bias", b);
    const int64_t nfeat = w.dim(1), c6 = M.conv[5].Co, Hh = nfeat / c6;
    MCHECK(w.dim(0) == kClass && nfeat == c6 * Hh, "rvc_load_crepe: classifier must be Linear(%lld, 360)", (long long)nfeat);
    {  // [360][h * c6 + c] -> the flatten order [c * H + h] of the strided bn_maxpool output
        HostT wp;
        wp.shape = {kClass, nfeat, 1};
        wp.v.resize(w.v.size());
        for (int64_t o = 0; o < kClass; ++o)
            for (int64_t cc = 0; cc < c6; ++cc)
                for (int64_t h = 0; h < Hh; ++h) wp.v[(o * c6 + cc) * Hh + h] = w.v[(o * Hh + h) * c6 + cc];
        MTRY(make_conv(c, M, wp, &b, M.classifier));
    }
    std::vector<double> lt((size_t)kClass * kClass);
    const double tiny = 2.2250738585072014e-308;  // np.finfo(np.float64).tiny
    if (P.has("log_trans")) {
        const rvc_param* q = P.by["log_trans"];
        MCHECK(q->dtype == RVC_DT_F64 && q->ndim == 2 && q->shape[0] == kClass && q->shape[1] == kClass,
               "rvc_load_crepe: log_trans must be f64 [360][360]");
        memcpy(lt.data(), q->data, lt.size() * 8);
    } else {  // tr[i][j] = max(12 - |i - j|, 0) / row sum; log_trans[j][k] = log(tr[k][j] + tiny)
        std::vector<double> rs(kClass, 0.0);
        for (int i = 0; i < kClass; ++i)
            for (int j = 0; j < kClass; ++j) rs[i] += fmax(12.0 - fabs((double)(j - i)), 0.0);
        for (int j = 0; j < kClass; ++j)
            for (int k = 0; k < kClass; ++k) lt[(size_t)j * kClass + k] = log(fmax(12.0 - fabs((double)(j - k)), 0.0) / rs[k] + tiny);
    }
#undef GET
    MTRY(dev_alloc(M, lt.size() * 8, (void**)&M.log_trans));
    MHIP(hipMemcpy(M.log_trans, lt.data(), lt.size() * 8, hipMemcpyHostToDevice));
    M.log_off = log(0.0 + tiny);
    M.log_p_init = log(1.0 / 360 + tiny);
    M.lo = crepe_bin(50.f, false);
    M.hi = crepe_bin(1100.f, true);
    MHIP(hipDeviceSynchronize());
    M.loaded = true;
    return RVC_OK;
}

extern "C" int rvc_crepe_f0(rvc_ctx* c, const float* audio, int64_t N, const float* dither, uint64_t seed,
                            double pitch_shift, const rvc_f0_post* post, float* probs, int64_t* coarse, float* pitchf,
                            rvc_stream_t stream) {
    MCHECK(c && c->cr && c->cr->loaded, "rvc_crepe_f0: no CREPE loaded");
    MCHECK(audio && coarse && pitchf && N >= 1, "rvc_crepe_f0: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    MHIP(hipSetDevice(c->device));
    Crepe& M = *c->cr;
    const int64_t T = 1 + N / kHop;
    int64_t*& so = M.seq_off[T];
    if (!so) {  // once per length, like crepe.py's resident offsets
        std::vector<int64_t> off;
        for (int64_t a = 0; a < T; a += kCrepeBatch) off.push_back(a);
        off.push_back(T);
        MTRY(dev_alloc(M, off.size() * 8, (void**)&so));
        MHIP(hipMemcpy(so, off.data(), off.size() * 8, hipMemcpyHostToDevice));
    }
    Scratch sc;
    MTRY(crepe_run(c, M, sc, audio, N, dither, seed, pitch_shift, post, probs, coarse, pitchf, so, s));
    MTRY(ensure_arena(M, sc.off, s));
    Scratch run;
    run.dry = false;
    run.base = M.arena;
    return crepe_run(c, M, run, audio, N, dither, seed, pitch_shift, post, probs, coarse, pitchf, so, s);
}

int contentvec_cf(rvc_ctx* c, const float* wav, int64_t N, int out_layer, int final_proj, float* feats_cf,
                  hipStream_t s) {
    MCHECK(c && c->cv && c->cv->loaded, "rvc_vc_convert: no ContentVec loaded");
    ContentVec& M = *c->cv;
    Scratch sc;
    MTRY(cv_one(c, M, sc, wav, N, out_layer, final_proj, feats_cf, s, true));
    MTRY(ensure_arena(M, sc.off, s));
    Scratch run;
    run.dry = false;
    run.base = M.arena;
    return cv_one(c, M, run, wav, N, out_layer, final_proj, feats_cf, s, true);
}

// ------------------------------------------------------------------ VC.pipeline (rvc_amd/pipeline.py pipeline_device)
// rvc_vc_convert_ex's scratch plus its f0 side stream: the f0 estimator runs there, concurrently with ContentVec on
// the caller's stream (as VC._pipeline_on_device does), joined by an event before the first phone upsample.
// the retrieval index (rvc_load_index): device copies, owned here and freed as a whole when replaced
struct IvfIndex : ModelBase {
    int64_t d = 0, nlist = 0, ntotal = 0;
    int nprobe = 1;
    float *centT = nullptr, *codes = nullptr, *big = nullptr;
    int64_t *list_off = nullptr, *ids = nullptr;
};

struct VcState : ModelBase {  // arena: the whole-input buffers (filtfilt, f0, quiet points, f0-file values)
    hipStream_t side = nullptr;
    hipEvent_t ev_in = nullptr, ev_f0 = nullptr;
    IvfIndex* ix = nullptr;
    void* ivf_ws = nullptr;
    int64_t ivf_ws_bytes = 0;
    ModelBase seg;  // arena: one segment's buffers (features, retrieval, phone, waveform), reused per segment
    double* pm_win = nullptr;  // Praat's window + its autocorrelation (rvc_pm_windows), uploaded once
};

void vc_delete(VcState* v) {
    if (!v) return;
    if (v->ix) {
        v->ix->release();
        delete v->ix;
    }
    if (v->ivf_ws) (void)hipFree(v->ivf_ws);
    if (v->side) (void)hipStreamDestroy(v->side);
    if (v->ev_in) (void)hipEventDestroy(v->ev_in);
    if (v->ev_f0) (void)hipEventDestroy(v->ev_f0);
    v->seg.release();
    v->release();
    delete v;
}

namespace {

// signal.butter(N=5, Wn=48, btype="high", fs=16000) (convert.py:30) and lfilter_zi of it, as scipy gives them
const double kBH[6] = {0.96996064518384473, -4.8498032259192234, 9.6996064518384468,
                       -9.6996064518384468, 4.8498032259192234, -0.96996064518384473};
const double kAH[6] = {1, -4.9390018191683636, 9.757863526739543, -9.6395448494134577, 4.7615067973562093,
                       -0.94082365320546057};
const double kZI[5] = {-0.96996047969958465, 3.8798419288925783, -5.8197629081730433, 3.879841948472456,
                       -0.96996048949233871};
constexpr int64_t kSr = 16000, kXQuery = 6, kXCenter = 38;  // Config (fp32): x_query 6, x_center 38

struct VcSeg {
    int64_t a, b, fa;  // padded-signal samples [a, b), f0 frames from fa
    int64_t Tf, T, L;  // ContentVec frames, synth frames (2 Tf), waveform samples (T upp)
};

struct VcPlan {
    int64_t tpad, Np, F, ld, p_len, C, tp, upp, emb;
    int64_t t_max, t_query, t_center;
    bool long_input;
};

int vc_basic(const rvc_ctx* c, int64_t N, const rvc_vc_args* a, const rvc_vc_opts* o, VcPlan& p) {
    int emb_dim = 0, upp = 0;
    MCHECK(c->cv && c->cv->loaded && synth_info(c, &emb_dim, &upp),
           "rvc_vc_convert: load ContentVec and the synthesizer first");
    const int f0m = o ? o->f0_method : RVC_F0_RMVPE;
    MCHECK(f0m == RVC_F0_RMVPE || f0m == RVC_F0_CREPE || f0m == RVC_F0_PM, "rvc_vc_convert: unknown f0 method %d", f0m);
    MCHECK(f0m != RVC_F0_RMVPE || (c->rm && c->rm->loaded), "rvc_vc_convert: f0 \"rmvpe\" needs rvc_load_rmvpe");
    MCHECK(f0m != RVC_F0_CREPE || (c->cr && c->cr->loaded), "rvc_vc_convert: f0 \"crepe\" needs rvc_load_crepe");
    MCHECK(a && (a->version == 1 || a->version == 2) && a->x_pad >= 0 && a->x_max > 0 && a->tgt_sr > 0,
           "rvc_vc_convert: bad args");
    MCHECK(N >= 1, "rvc_vc_convert: empty input");
    p.tpad = kSr * a->x_pad;
    p.Np = N + 2 * p.tpad;
    p.F = 1 + p.Np / kHop;
    p.ld = rvc_rmvpe_salience_ld(p.Np);
    p.p_len = p.Np / kHop;
    p.C = a->version == 1 ? c->cv->final_proj.Co : c->cv->E;
    MCHECK(p.C == emb_dim, "rvc_vc_convert: features of %lld channels, the synthesizer takes %d", (long long)p.C,
           emb_dim);
    MCHECK(a->index_rate == 0.0 || (c->vc && c->vc->ix && c->vc->ix->d == p.C),
           "rvc_vc_convert: index_rate %g needs an index of the features' width (rvc_load_index)", a->index_rate);
    p.upp = upp;
    p.emb = emb_dim;
    p.tp = (int64_t)a->tgt_sr * a->x_pad;
    p.t_max = kSr * a->x_max;
    p.t_query = kSr * kXQuery;
    p.t_center = kSr * kXCenter;
    p.long_input = N + kHop > p.t_max;  // convert.py:406 (audio padded by window / 2 on each side)
    return RVC_OK;
}

// one segment's sizes; `T <= frames available` as VC.voice_conversion needs (convert.py:364-370)
int vc_seg(const VcPlan& p, int64_t a, int64_t b, int64_t fa, int64_t fb, VcSeg& g) {
    g.a = a;
    g.b = b;
    g.fa = fa;
    const int64_t Ns = b - a;
    g.Tf = rvc_contentvec_frames(Ns);
    MCHECK(g.Tf >= 1 && 2 * g.Tf <= Ns / kHop, "rvc_vc_convert: segment of %lld samples too short", (long long)Ns);
    g.T = 2 * g.Tf;  // min(2 T_f, p_len)
    MCHECK(fa + g.T <= fb, "rvc_vc_convert: pitch shorter than the phone sequence");
    g.L = g.T * p.upp;
    MCHECK(g.L > 2 * p.tp, "rvc_vc_convert: input too short");
    return RVC_OK;
}

// Segments of convert.py:419-440 (VC._pipeline_on_device): [s, t + t_pad2 + w) for each quiet point t, then [t, end)
int vc_segments(const VcPlan& p, const std::vector<int64_t>& opt_ts, std::vector<VcSeg>& segs) {
    segs.clear();
    int64_t s = 0, last = 0;
    for (int64_t t : opt_ts) {
        t = t / kHop * kHop;
        VcSeg g;
        MTRY(vc_seg(p, s, t + 2 * p.tpad + kHop, s / kHop, (t + 2 * p.tpad) / kHop, g));
        segs.push_back(g);
        s = t;
        last = t;
    }
    VcSeg g;
    MTRY(vc_seg(p, last, p.Np, last / kHop, p.p_len, g));
    segs.push_back(g);
    return RVC_OK;
}

// convert.py:316-318 on the host (host_f0file.h, plain C++: also built with -fsanitize on the CPU by
// tests/test_c_host_cpu.py)
int f0_file_rep(const float* rows, int64_t nrows, std::vector<double>& rep) {
    MCHECK(rows && nrows >= 1, "rvc_vc_convert: empty f0 file");
    MCHECK(rvc_host::f0_file_interp(rows, nrows, rep) == 0, "rvc_vc_convert: f0 file times not finite or too long");
    return RVC_OK;
}

// a grow-only device buffer of a ModelBase-owned arena slice is not enough for the f0-file values: own buffer
int ensure_buf(void** buf, int64_t* cap, int64_t bytes, hipStream_t s) {
    if (bytes <= *cap) return RVC_OK;
    if (*buf) {
        MHIP(hipStreamSynchronize(s));
        MHIP(hipFree(*buf));
        *buf = nullptr;
        *cap = 0;
    }
    MHIP(hipMalloc(buf, bytes));
    *cap = bytes;
    return RVC_OK;
}

}  // namespace

extern "C" int64_t rvc_f0_file_resample(const float* rows, int64_t nrows, double* out, int64_t cap) {
    std::vector<double> rep;
    if (!rows || nrows < 1 || f0_file_rep(rows, nrows, rep) != RVC_OK) return -1;
    for (int64_t i = 0; i < (int64_t)rep.size() && i < cap && out; ++i) out[i] = rep[i];
    return (int64_t)rep.size();
}

extern "C" int64_t rvc_vc_out_len(const rvc_ctx* c, int64_t N, const rvc_vc_args* a) {
    VcPlan p;
    if (!c || !a || vc_basic(c, N, a, nullptr, p) != RVC_OK) return -1;
    if (!p.long_input) {
        std::vector<VcSeg> segs;
        if (vc_segments(p, {}, segs) != RVC_OK) return -1;
        return segs[0].L - 2 * p.tp;
    }
    // longer inputs: an upper bound (the quiet points are only known after the filtfilt; rvc_vc_convert_ex
    // reports the exact length).  Segments overlap by t_pad2 + window; each gives at most its frames * upp.
    const int64_t nq = rvc_quiet_points_count(N, (int)kHop, p.t_center, p.t_max);
    if (nq < 0) return -1;
    const int64_t nseg = nq + 1;
    return ((p.Np + nseg * (2 * p.tpad + kHop)) / kHop + nseg) * p.upp;
}

extern "C" int rvc_vc_convert_ex(rvc_ctx* c, const float* audio, int64_t N, const rvc_vc_args* a,
                                 const rvc_vc_opts* o, float* out, int64_t out_cap, int64_t* out_len,
                                 rvc_stream_t stream) {
    MCHECK(c && audio && out, "rvc_vc_convert: null argument");
    if (out_len) *out_len = 0;
    VcPlan p;
    MTRY(vc_basic(c, N, a, o, p));
    const int f0m = o ? o->f0_method : RVC_F0_RMVPE;
    const double venv = o ? o->volume_envelope : 1.0;
    MCHECK(!o || o->f0_file_rows == 0 || o->f0_file, "rvc_vc_convert: f0_file rows without data");
    hipStream_t s = (hipStream_t)stream;
    MHIP(hipSetDevice(c->device));
    if (!c->vc) c->vc = new VcState();
    VcState& V = *c->vc;
    if (!V.side) {  // high priority: the f0 branch is the longer one (RMVPE with the BiGRU recurrence)
        int least = 0, greatest = 0;
        MHIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        MHIP(hipStreamCreateWithPriority(&V.side, hipStreamNonBlocking, greatest));
        MHIP(hipEventCreateWithFlags(&V.ev_in, hipEventDisableTiming));
        MHIP(hipEventCreateWithFlags(&V.ev_f0, hipEventDisableTiming));
    }
    const bool need64 = p.long_input || venv != 1.0 || f0m == RVC_F0_PM;
    // f0 track length: RMVPE / CREPE 1 + Np / 160 frames; pm max(p_len, Praat frames) (get_f0_pm's padding)
    const int64_t nf_pm = f0m == RVC_F0_PM ? rvc_pm_frames(p.Np) : 0;
    MCHECK(f0m != RVC_F0_PM || nf_pm > 0, "rvc_vc_convert: pm: input shorter than one 60 ms window");
    const int64_t Ftr = f0m == RVC_F0_PM ? (p.p_len > nf_pm ? p.p_len : nf_pm) : p.F;
    const int64_t nq = rvc_quiet_points_count(N, (int)kHop, p.t_center, p.t_max);
    const int64_t qws = nq > 0 ? rvc_quiet_points_ws_bytes(N, (int)kHop, p.t_center, p.t_query, p.t_max) : 0;
    const int64_t pmw = f0m == RVC_F0_PM ? rvc_pm_work_bytes(p.Np) : 0;
    std::vector<double> rep;
    if (o && o->f0_file_rows > 0) MTRY(f0_file_rep(o->f0_file, o->f0_file_rows, rep));
    const int64_t fw = (rvc_filtfilt_work_bytes(N) + 7) / 8;
    MCHECK(fw > 0 && qws >= 0 && pmw >= 0, "rvc_vc_convert: work sizes");
    Plan pl;  // f32 slots; int64 / f64 buffers take two each
    const int64_t o_work = pl.take(2 * fw), o_xp = pl.take(p.Np), o_xp64 = pl.take(need64 ? 2 * p.Np : 0),
                  o_sal = pl.take(f0m == RVC_F0_RMVPE ? kClass * p.ld : 0), o_coarse = pl.take(2 * Ftr),
                  o_pitchf = pl.take(Ftr), o_opt = pl.take(2 * (nq > 0 ? nq : 1)), o_qws = pl.take((qws + 3) / 4),
                  o_pmw = pl.take((pmw + 3) / 4), o_pmf0 = pl.take(2 * (nf_pm > 0 ? nf_pm : 1)),
                  o_rep = pl.take(2 * (int64_t)rep.size()), o_ws = pl.take(16);
    if (pl.off > V.arena_floats && V.side) MHIP(hipStreamSynchronize(V.side));  // the old arena may be in use there
    MTRY(ensure_arena(V, pl.off, s));
    float* A = V.arena;
    float* xp = A + o_xp;
    double* xp64 = need64 ? (double*)(A + o_xp64) : nullptr;
    // filtfilt + reflect padding (convert.py:403, 416), f64 on the device
    MTRY(rvc_filtfilt_pad(audio, N, kBH, kAH, kZI, p.tpad, (double*)(A + o_work), xp, xp64, s));
    // quiet-point segmentation (convert.py:404-412): on the device, read back for the segment plan
    std::vector<int64_t> opt_ts;
    if (nq > 0) {
        int64_t* dopt = (int64_t*)(A + o_opt);
        MTRY(rvc_quiet_points(xp64 + p.tpad, N, (int)kHop, p.t_center, p.t_query, p.t_max, A + o_qws, qws, dopt,
                              (rvc_stream_t)s));
        opt_ts.resize(nq);
        MHIP(hipMemcpyAsync(opt_ts.data(), dopt, nq * 8, hipMemcpyDeviceToHost, s));
        MHIP(hipStreamSynchronize(s));
    }
    std::vector<VcSeg> segs;
    MTRY(vc_segments(p, opt_ts, segs));
    int64_t total = 0;
    for (const VcSeg& g : segs) total += g.L - 2 * p.tp;
    MCHECK(out_cap >= total, "rvc_vc_convert: output needs %lld samples, the buffer holds %lld", (long long)total,
           (long long)out_cap);
    MCHECK(out_len || !p.long_input, "rvc_vc_convert: inputs over x_max need rvc_vc_convert_ex's out_len");
    // get_f0's optional steps (convert.py:311-318) for the decode kernels
    rvc_f0_post post{};
    const rvc_f0_post* postp = nullptr;
    if ((o && o->f0_autotune) || !rep.empty()) {
        if (o && o->f0_autotune) {
            post.autotune = 1;
            post.strength = o->f0_autotune_strength;
        }
        const int64_t rep_off = (int64_t)a->x_pad * 100;
        if (!rep.empty() && rep_off < Ftr) {
            double* drep = (double*)(A + o_rep);
            MHIP(hipMemcpyAsync(drep, rep.data(), rep.size() * 8, hipMemcpyHostToDevice, s));
            post.rep = drep;
            post.rep_off = rep_off;
            post.rep_len = (int64_t)rep.size() < Ftr - rep_off ? (int64_t)rep.size() : Ftr - rep_off;
        }
        postp = &post;
    }
    if (f0m == RVC_F0_PM && !V.pm_win) {
        std::vector<double> w(958 + 480);
        MTRY(rvc_pm_windows(w.data(), w.data() + 958));
        MTRY(dev_alloc(V, w.size() * 8, (void**)&V.pm_win));
        MHIP(hipMemcpy(V.pm_win, w.data(), w.size() * 8, hipMemcpyHostToDevice));
    }
    // f0 over the whole padded input on the side stream (VC.get_f0, convert.py:304-323, 436)
    int64_t* coarse = (int64_t*)(A + o_coarse);
    float* pitchf = A + o_pitchf;
    const double shift = pow(2.0, a->pitch_shift / 12.0);
    MHIP(hipEventRecord(V.ev_in, s));
    MHIP(hipStreamWaitEvent(V.side, V.ev_in, 0));
    // from the fork on, every return joins the side stream back into s (its writes to the arenas must be
    // ordered before the next call's use of them on s)
    struct Join {
        hipStream_t s, side;
        hipEvent_t ev;
        bool armed = true;
        ~Join() {
            if (armed && hipEventRecord(ev, side) == hipSuccess) (void)hipStreamWaitEvent(s, ev, 0);
        }
    } join{s, V.side, V.ev_f0};
    const rvc_stream_t sd = (rvc_stream_t)V.side;
    if (f0m == RVC_F0_RMVPE) {
        float* sal = A + o_sal;
        MTRY(rvc_rmvpe_forward(c, xp, 1, p.Np, sal, sd));
        MTRY(rvc_rmvpe_decode(sal, p.ld, p.F, 0.03, shift, postp, nullptr, coarse, pitchf, sd));
    } else if (f0m == RVC_F0_CREPE) {
        MTRY(rvc_crepe_f0(c, xp, p.Np, o ? o->crepe_dither : nullptr, a->seed, a->pitch_shift, postp, nullptr, coarse,
                          pitchf, sd));
    } else {
        double* f0 = (double*)(A + o_pmf0);
        MTRY(rvc_pm_f0(xp64, p.Np, V.pm_win, V.pm_win + 958, A + o_pmw, pmw, f0, sd));
        MTRY(rvc_pm_post(f0, nf_pm, p.p_len, shift, postp, coarse, pitchf, sd));
    }
    MHIP(hipEventRecord(V.ev_f0, V.side));
    // per segment: features (convert.py:337-340), retrieval (:349-359), phone upsample + protect (:361-378),
    // Synthesizer.infer with the segment's noise seed, the x_pad trim -- in order into out
    int64_t Tf_max = 0, T_max = 0, L_max = 0;
    for (const VcSeg& g : segs) {
        Tf_max = g.Tf > Tf_max ? g.Tf : Tf_max;
        T_max = g.T > T_max ? g.T : T_max;
        L_max = g.L > L_max ? g.L : L_max;
    }
    const int nprobe = V.ix ? V.ix->nprobe : 1;
    Plan ps;
    const int64_t o_feats = ps.take(p.C * Tf_max), o_phone = ps.take(p.C * T_max), o_wav = ps.take(L_max),
                  o_blend = ps.take(a->index_rate != 0.0 ? p.C * Tf_max : 0), o_D = ps.take(8 * Tf_max),
                  o_I = ps.take(2 * 8 * Tf_max), o_probes = ps.take(2 * (int64_t)nprobe * Tf_max),
                  o_r1 = ps.take(venv != 1.0 ? N / 8000 + 2 : 0), o_r2 = ps.take(venv != 1.0 ? total / 8000 + 2 : 0);
    MTRY(ensure_arena(V.seg, ps.off, s));
    float* B = V.seg.arena;
    bool joined = false;
    int64_t off = 0;
    for (size_t k = 0; k < segs.size(); ++k) {
        const VcSeg& g = segs[k];
        float* feats = B + o_feats;
        MTRY(contentvec_cf(c, xp + g.a, g.b - g.a, a->version == 1 ? 9 : 12, a->version == 1, feats, s));
        const float* fb = feats;  // convert.py:347: the protect blend keeps the pre-retrieval features
        if (a->index_rate != 0.0) {
            const IvfIndex& X = *V.ix;
            const int64_t need = rvc_ivf_coarse_ws_bytes(g.Tf, X.nlist);
            MTRY(ensure_buf(&V.ivf_ws, &V.ivf_ws_bytes, need, s));
            float* D = B + o_D;
            int64_t* I = (int64_t*)(B + o_I);
            MTRY(rvc_ivf_search(feats, g.Tf, p.C, g.Tf, 1, X.centT, X.nlist, X.nprobe, X.list_off, X.codes, X.ids, 8,
                                V.ivf_ws, need, (int64_t*)(B + o_probes), D, I, (rvc_stream_t)s));
            MTRY(rvc_ivf_blend(feats, g.Tf, p.C, g.Tf, 1, D, I, 8, X.big, X.ntotal, a->index_rate, B + o_blend, g.Tf,
                               1, (rvc_stream_t)s));
            fb = B + o_blend;
        }
        if (!joined) {  // the upsample reads pitchf
            join.armed = false;
            MHIP(hipStreamWaitEvent(s, V.ev_f0, 0));
            joined = true;
        }
        float* phone = B + o_phone;
        MTRY(rvc_phone_upsample(fb, feats, a->protect < 0.5f ? pitchf + g.fa : nullptr, phone, p.C, g.Tf, g.T,
                                a->protect, (rvc_stream_t)s));
        float* wav = B + o_wav;
        MTRY(synth_run_cf(c, phone, coarse + g.fa, pitchf + g.fa, g.T, a->sid, a->seed + k, wav, s));
        MHIP(hipMemcpyAsync(out + off, wav + p.tp, (g.L - 2 * p.tp) * 4, hipMemcpyDeviceToDevice, s));
        off += g.L - 2 * p.tp;
    }
    if (venv != 1.0) {  // change_rms(audio, 16000, audio_opt, 16000, rate) (convert.py:449): hop 8000 for both
        const int64_t n1 = rvc_rms_frames_len(N, 8000), n2 = rvc_rms_frames_len(total, 8000);
        MCHECK(n1 > 0 && n1 <= N / 8000 + 2 && n2 > 0 && n2 <= total / 8000 + 2, "rvc_vc_convert: rms frames");
        float *r1 = B + o_r1, *r2 = B + o_r2;
        MTRY(rvc_rms_frames(xp64 + p.tpad, nullptr, N, 8000, r1, (rvc_stream_t)s));
        MTRY(rvc_rms_frames(nullptr, out, total, 8000, r2, (rvc_stream_t)s));
        MTRY(rvc_rms_mix(out, total, r1, n1, r2, n2, venv, (rvc_stream_t)s));
    }
    MTRY(rvc_peak_normalize(out, total, A + o_ws, nullptr, (rvc_stream_t)s));
    if (out_len) *out_len = total;
    return RVC_OK;
}

extern "C" int rvc_vc_convert(rvc_ctx* c, const float* audio, int64_t N, const rvc_vc_args* a, float* out,
                              rvc_stream_t stream) {
    const int64_t n = rvc_vc_out_len(c, N, a);
    if (n <= 0) return RVC_EINVAL;  // the message is set
    return rvc_vc_convert_ex(c, audio, N, a, nullptr, out, n, nullptr, stream);
}

extern "C" int rvc_load_index(rvc_ctx* c, const rvc_ivf_index* x) {
    MCHECK(c && x && x->centroids && x->list_off && x->big && x->codes && x->ids, "rvc_load_index: null array");
    // everything rvc_ivf_search / rvc_ivf_blend read on the device is validated here, on the host, so that a
    // malformed or foreign index is a load error instead of an out-of-bounds device read later
    MCHECK(x->d > 0 && x->d <= 1024 && x->d % 8 == 0, "rvc_load_index: d = %lld (1..1024, a multiple of 8)",
           (long long)x->d);
    MCHECK(x->nlist > 0 && x->ntotal > 0 && x->nprobe >= 1, "rvc_load_index: nlist %lld, ntotal %lld, nprobe %d",
           (long long)x->nlist, (long long)x->ntotal, x->nprobe);
    MCHECK(x->list_off[0] == 0 && x->list_off[x->nlist] == x->ntotal, "rvc_load_index: list_off must span [0, ntotal]");
    for (int64_t l = 0; l < x->nlist; ++l)
        MCHECK(x->list_off[l] <= x->list_off[l + 1], "rvc_load_index: list_off decreases at list %lld", (long long)l);
    for (int64_t i = 0; i < x->ntotal; ++i)
        MCHECK(x->ids[i] >= 0 && x->ids[i] < x->ntotal, "rvc_load_index: id %lld of entry %lld outside [0, ntotal)",
               (long long)x->ids[i], (long long)i);
    MHIP(hipSetDevice(c->device));
    if (!c->vc) c->vc = new VcState();
    VcState& V = *c->vc;
    if (V.ix) {  // replace: no call may still read the old arrays
        MHIP(hipDeviceSynchronize());
        V.ix->release();
        delete V.ix;
        V.ix = nullptr;
    }
    IvfIndex* X = new IvfIndex();
    X->d = x->d;
    X->nlist = x->nlist;
    X->ntotal = x->ntotal;
    X->nprobe = x->nprobe < x->nlist ? x->nprobe : (int)x->nlist;
    auto fail = [&](int rc) {
        X->release();
        delete X;
        return rc;
    };
    std::vector<float> ct((size_t)x->d * x->nlist);  // centroids transposed [d][nlist] (retrieval.py)
    for (int64_t l = 0; l < x->nlist; ++l)
        for (int64_t k = 0; k < x->d; ++k) ct[(size_t)k * x->nlist + l] = x->centroids[l * x->d + k];
    int rc = upload(*X, ct, &X->centT);
    auto up = [&](const void* src, size_t bytes, void** dst) -> int {
        MTRY(dev_alloc(*X, bytes, dst));
        MHIP(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
        return RVC_OK;
    };
    if (rc == RVC_OK) rc = up(x->list_off, (x->nlist + 1) * 8, (void**)&X->list_off);
    if (rc == RVC_OK) rc = up(x->codes, x->ntotal * x->d * 4, (void**)&X->codes);
    if (rc == RVC_OK) rc = up(x->ids, x->ntotal * 8, (void**)&X->ids);
    if (rc == RVC_OK) rc = up(x->big, x->ntotal * x->d * 4, (void**)&X->big);
    if (rc != RVC_OK) return fail(rc);
    V.ix = X;
    return RVC_OK;
}

extern "C" int64_t rvc_device_bytes_in_use(void) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return -1;
    return (int64_t)(total_b - free_b);
}
