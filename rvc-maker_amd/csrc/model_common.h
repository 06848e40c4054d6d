// Internal helpers of the model-level C ABI (rvc_model.cpp: synthesizer and context; rvc_frontend.cpp:
// ContentVec and RMVPE): host-side weight handling (fp16 -> f32, weight-norm folding, KM packing), the
// per-model device allocations and scratch, and the conv launch helper that mirrors ops.conv1d.
#pragma once
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/rvc_amd.h"

void rvc_set_error(const char* fmt, ...);

#define MCHECK(cond, ...)               \
    do {                                \
        if (!(cond)) {                  \
            rvc_set_error(__VA_ARGS__); \
            return RVC_EINVAL;          \
        }                               \
    } while (0)
#define MHIP(call)                                                  \
    do {                                                            \
        hipError_t e_ = (call);                                     \
        if (e_ != hipSuccess) {                                     \
            rvc_set_error("%s: %s", #call, hipGetErrorString(e_)); \
            return RVC_EHIP;                                        \
        }                                                           \
    } while (0)
#define MTRY(call)                     \
    do {                               \
        int rc_ = (call);              \
        if (rc_ != RVC_OK) return rc_; \
    } while (0)

struct Synth;
struct ContentVec;
struct Rmvpe;
struct Crepe;
struct VcState;

struct rvc_ctx {
    int device = 0;
    int prec = RVC_PREC_FP32;
    int rm_prec = RVC_PREC_FP64;  // RMVPE's arithmetic (rvc_ctx_set_rmvpe_precision), read by rvc_load_rmvpe
    bool x6 = true, f16mix = true, fused_rb = true;  // RVC_AMD_X6 / RVC_AMD_F16MIX / RVC_AMD_FUSED_RB as ops.py
    bool amax = true;  // RVC_AMD_AMAX as synth.py: the generator's |max| side channel
    bool amax_f16all = true;  // RVC_AMD_AMAX_F16ALL as ops.py
    bool cv_amax = true;      // RVC_AMD_CV_AMAX as contentvec.py: ContentVec's GEMMs take the producers' |max|
    bool amax_ups = true;     // RVC_AMD_AMAX_UPS as synth.py: the upsampling convs' inputs through |max| cells
    bool amax_s2 = true;      // RVC_AMD_AMAX_S2 as ops.py: stride-2 convs with a producer's |max| in split-fp16
    bool fe_amax = true;      // RVC_AMD_FE_AMAX as contentvec.py: the feature extractor's convs through |max| cells
    bool fused_noise = false; // RVC_AMD_FUSED_NOISE as synth.py: noise_convs fused into the upsampling convs (off)
    bool attn_f16 = true;     // RVC_AMD_ATTN_F16 as contentvec.py / synth.py: QKV |max| cells, split-fp16 attention
    bool te_amax = false;     // RVC_AMD_TE_AMAX as synth.py: the TextEncoder's GEMMs through |max| cells (default off)
    bool flow_amax = false;   // RVC_AMD_FLOW_AMAX as synth.py: the flow's (default off)
    Synth* syn = nullptr;
    ContentVec* cv = nullptr;
    Rmvpe* rm = nullptr;
    Crepe* cr = nullptr;
    VcState* vc = nullptr;  // rvc_vc_convert's own scratch
};

void synth_delete(Synth* s);
void contentvec_delete(ContentVec* m);
void rmvpe_delete(Rmvpe* m);
void crepe_delete(Crepe* m);
void vc_delete(VcState* v);

// internal entry points shared by the model files (rvc_vc_convert drives them)
int synth_run_cf(rvc_ctx* c, const float* phone_cf, const int64_t* pitch, const float* pitchf, int64_t T, int64_t sid,
                 uint64_t seed, float* wav, hipStream_t s);  // phone channels-first [E][T]
bool synth_info(const rvc_ctx* c, int* emb_dim, int* upp);  // loaded? + its phone width and upsampling
int contentvec_cf(rvc_ctx* c, const float* wav, int64_t N, int out_layer, int final_proj, float* feats_cf,
                  hipStream_t s);  // -> [C][T_f]

namespace rvcm {

// ------------------------------------------------------------------ host tensors
struct HostT {
    std::vector<float> v;
    std::vector<int64_t> shape;
    int64_t dim(int i) const { return i < (int)shape.size() ? shape[i] : 1; }
};

inline float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 31, m = h & 1023;
    uint32_t bits;
    if (e == 0) {
        if (m == 0) {
            bits = s;
        } else {  // subnormal: renormalise
            int ee = -1;
            uint32_t mm = m;
            do {
                ++ee;
                mm <<= 1;
            } while (!(mm & 1024));
            bits = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 1023) << 13);
        }
    } else if (e == 31) {
        bits = s | 0x7f800000u | (m << 13);
    } else {
        bits = s | ((e - 15 + 127) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

inline HostT to_host(const rvc_param& p) {
    HostT t;
    int64_t n = 1;
    for (int i = 0; i < p.ndim; ++i) {
        t.shape.push_back(p.shape[i]);
        n *= p.shape[i];
    }
    t.v.resize(n);
    if (p.dtype == RVC_DT_F16) {
        const uint16_t* s = (const uint16_t*)p.data;
        for (int64_t i = 0; i < n; ++i) t.v[i] = half_to_float(s[i]);
    } else if (p.dtype == RVC_DT_F64) {
        const double* s = (const double*)p.data;
        for (int64_t i = 0; i < n; ++i) t.v[i] = (float)s[i];
    } else {
        memcpy(t.v.data(), p.data, n * 4);
    }
    return t;
}

// torch._weight_norm(v, g, dim): w = v * (g / ||v||), the norm over every axis but `dim`
inline HostT fold_wn(const HostT& v, const HostT& g, int dim) {
    HostT w = v;
    int64_t outer = 1, inner = 1;
    for (int i = 0; i < dim; ++i) outer *= v.dim(i);
    for (int i = dim + 1; i < (int)v.shape.size(); ++i) inner *= v.dim(i);
    const int64_t n = v.dim(dim);
    for (int64_t k = 0; k < n; ++k) {
        double ss = 0;
        for (int64_t o = 0; o < outer; ++o)
            for (int64_t j = 0; j < inner; ++j) {
                const double e = v.v[(o * n + k) * inner + j];
                ss += e * e;
            }
        const float f = g.v[k] / (float)sqrt(ss);
        for (int64_t o = 0; o < outer; ++o)
            for (int64_t j = 0; j < inner; ++j) w.v[(o * n + k) * inner + j] = v.v[(o * n + k) * inner + j] * f;
    }
    return w;
}

// Named host arrays of a checkpoint; get("x.weight") folds x.weight_g / x.weight_v when x.weight is absent.
struct Params {
    std::map<std::string, const rvc_param*> by;
    std::string missing;
    int wn_dim = 0;
    bool has(const std::string& k) const { return by.count(k) > 0; }
    bool get(const std::string& k, HostT& out) {
        if (has(k)) {
            out = to_host(*by[k]);
            return true;
        }
        const std::string suf = ".weight";
        if (k.size() > suf.size() && k.compare(k.size() - suf.size(), suf.size(), suf) == 0) {
            const std::string base = k.substr(0, k.size() - suf.size());
            if (has(base + ".weight_g") && has(base + ".weight_v")) {
                out = fold_wn(to_host(*by[base + ".weight_v"]), to_host(*by[base + ".weight_g"]), wn_dim);
                return true;
            }
        }
        if (missing.empty()) missing = k;
        return false;
    }
};

inline int index_params(const rvc_param* params, int n, Params& P, const char* who) {
    for (int i = 0; i < n; ++i) {
        MCHECK(params[i].name && params[i].data && params[i].ndim >= 1 && params[i].ndim <= 4 &&
                   (params[i].dtype == RVC_DT_F32 || params[i].dtype == RVC_DT_F16 || params[i].dtype == RVC_DT_F64),
               "%s: bad param %d", who, i);
        P.by[params[i].name] = &params[i];
    }
    return RVC_OK;
}

// ------------------------------------------------------------------ per-model device state
struct ModelBase {
    std::vector<void*> allocs;  // weights
    void* ws = nullptr;         // split-K / split-KV scratch
    int64_t ws_bytes = 0;
    float* arena = nullptr;  // activations
    int64_t arena_floats = 0;
    bool loaded = false;
    void release() {
        for (void* p : allocs) (void)hipFree(p);
        allocs.clear();
        if (ws) (void)hipFree(ws);
        if (arena) (void)hipFree(arena);
        ws = nullptr;
        arena = nullptr;
        ws_bytes = arena_floats = 0;
    }
};

struct ConvW {
    int64_t Co = 0, Ci = 0;  // Ci: all input channels
    int K = 0;               // taps per phase (ConvT: ceil(K/u))
    int groups = 1;
    int nphase = 1;  // ConvT: u phases
    int Kfull = 0, u = 1, tpad = 0;
    float* w = nullptr;  // KM [nphase][groups][Ci/g*K][Co/g]
    float* b = nullptr;
    void* wx_bf = nullptr;  // split-bf16 image
    void* wx_hf = nullptr;  // split-fp16 image
    int nmf = 0;
};

inline int dev_alloc(ModelBase& m, size_t bytes, void** out) {
    MHIP(hipMalloc(out, bytes ? bytes : 4));
    m.allocs.push_back(*out);
    return RVC_OK;
}

inline int upload(ModelBase& m, const std::vector<float>& h, float** out) {
    MTRY(dev_alloc(m, h.size() * 4, (void**)out));
    MHIP(hipMemcpy(*out, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return RVC_OK;
}

// the split-operand images (ops.pack_x6): ungrouped convs with <= 64 taps, grouped ones (the groups packed as phases,
// conv1d.hip's gx6) with <= 128
inline int make_images(rvc_ctx* c, ModelBase& m, ConvW& cw) {
    if (!c->x6 || cw.K > (cw.groups == 1 ? 64 : 128) || (cw.groups > 1 && cw.nphase > 1)) return RVC_OK;
    const int64_t np = cw.nphase * cw.groups, Ci = cw.Ci / cw.groups, Co = cw.Co / cw.groups;
    const int64_t nb = rvc_conv1d_x6_bytes(np, Ci, cw.K, Co);
    const int64_t nh = rvc_conv1d_f16_bytes(np, Ci, cw.K, Co);
    MCHECK(nb > 0 && nh > 0, "model load: bad conv shape %lld x %lld x %d", (long long)cw.Co, (long long)cw.Ci, cw.K);
    MTRY(dev_alloc(m, nb, &cw.wx_bf));
    MTRY(dev_alloc(m, nh, &cw.wx_hf));
    int nmf = 0;
    MTRY(rvc_conv1d_pack_x6(cw.w, np, Ci, cw.K, Co, cw.wx_bf, &nmf, nullptr));
    MTRY(rvc_conv1d_pack_f16(cw.w, np, Ci, cw.K, Co, cw.wx_hf, &nmf, nullptr));
    cw.nmf = nmf;
    return RVC_OK;
}

// Conv1d weight [Co][Ci/g][K] (+ bias [Co]) -> KM [g][Ci/g*K][Co/g] (ops.pack_km)
inline int make_conv(rvc_ctx* c, ModelBase& m, const HostT& w, const HostT* b, ConvW& cw, int groups = 1) {
    MCHECK(w.shape.size() >= 2, "model load: conv weight must be 2- or 3-D");
    cw.groups = groups;
    cw.Co = w.dim(0);
    const int64_t Cig = w.dim(1), Cog = cw.Co / groups;
    cw.Ci = Cig * groups;
    cw.K = (int)w.dim(2);
    cw.Kfull = cw.K;
    std::vector<float> km((size_t)cw.Co * Cig * cw.K);
    for (int gi = 0; gi < groups; ++gi)
        for (int64_t mo = 0; mo < Cog; ++mo)
            for (int64_t ci = 0; ci < Cig; ++ci)
                for (int t = 0; t < cw.K; ++t)
                    km[((int64_t)gi * Cig * cw.K + ci * cw.K + t) * Cog + mo] =
                        w.v[((gi * Cog + mo) * Cig + ci) * cw.K + t];
    MTRY(upload(m, km, &cw.w));
    if (b) {
        MCHECK((int64_t)b->v.size() == cw.Co, "model load: bias size %zu != %lld", b->v.size(), (long long)cw.Co);
        MTRY(upload(m, b->v, &cw.b));
    }
    return make_images(c, m, cw);
}

// ConvTranspose1d weight [Ci][Co][K], stride u -> polyphase KM [u][Ci*T][Co] (ops.pack_convT)
inline int make_convT(rvc_ctx* c, ModelBase& m, const HostT& w, const HostT& b, int u, int pad, ConvW& cw) {
    cw.Ci = w.dim(0);
    cw.Co = w.dim(1);
    cw.Kfull = (int)w.dim(2);
    cw.u = u;
    cw.tpad = pad;
    cw.nphase = u;
    const int T = (cw.Kfull + u - 1) / u;
    cw.K = T;
    std::vector<float> km((size_t)u * cw.Ci * T * cw.Co, 0.f);
    for (int r = 0; r < u; ++r)
        for (int tp = 0; tp < T; ++tp) {
            const int j = r + (T - 1 - tp) * u;
            if (j >= cw.Kfull) continue;
            for (int64_t ci = 0; ci < cw.Ci; ++ci)
                for (int64_t mo = 0; mo < cw.Co; ++mo)
                    km[(((int64_t)r * cw.Ci + ci) * T + tp) * cw.Co + mo] = w.v[(ci * cw.Co + mo) * cw.Kfull + j];
        }
    MTRY(upload(m, km, &cw.w));
    MTRY(upload(m, b.v, &cw.b));
    return make_images(c, m, cw);
}

// ------------------------------------------------------------------ pass sets (ops.conv_passes / rb_passes)
inline int base_passes(const rvc_ctx* c) { return c->prec == RVC_PREC_FP32 ? 6 : c->prec; }

// amax: the input's |max| comes from its producer (the amax side channel): split-fp16 for every stride-1 1-D conv
inline int conv_passes(const rvc_ctx* c, int K, int64_t Cig, int stride, bool two_d, bool amax = false) {
    if (c->prec == RVC_PREC_FP32 && c->f16mix && !two_d &&
        ((stride == 1 && ((amax && c->amax_f16all) || (K >= 7 && Cig <= 256) || (K >= 3 && Cig >= 64 && Cig <= 128))) ||
         (stride == 2 && amax && c->amax_f16all && c->amax_s2)))
        return RVC_ARITH_F16X3;
    return base_passes(c);
}

inline int ensure_ws(ModelBase& m, int64_t need, hipStream_t s) {
    if (need <= m.ws_bytes) return RVC_OK;
    if (m.ws) {
        MHIP(hipStreamSynchronize(s));
        MHIP(hipFree(m.ws));
        m.ws = nullptr;
        m.ws_bytes = 0;
    }
    const int64_t bytes = need + (4 << 20);
    MHIP(hipMalloc(&m.ws, bytes));
    m.ws_bytes = bytes;
    return RVC_OK;
}

inline int ensure_arena(ModelBase& m, int64_t floats, hipStream_t s) {
    if (floats <= m.arena_floats) return RVC_OK;
    if (m.arena) {
        MHIP(hipStreamSynchronize(s));
        MHIP(hipFree(m.arena));
        m.arena = nullptr;
        m.arena_floats = 0;
    }
    MHIP(hipMalloc((void**)&m.arena, floats * 4));
    m.arena_floats = floats;
    return RVC_OK;
}

// ------------------------------------------------------------------ launch helper (ops.conv1d)
struct CallOpts {
    const float* bias2 = nullptr;
    const float* res = nullptr;
    int stride = 1, pad = 0, dil = 1;
    int64_t Lout = -1;
    int in_act = RVC_ACT_NONE, out_act = RVC_ACT_NONE, accumulate = 0;
    float in_slope = 0.f, in_scale = 1.f, out_slope = 0.f, out_scale = 1.f;
    int64_t B = 1, x_bstride = 0, y_bstride = 0, res_bstride = 0;
    int ntoff = 0, wrap = 0;  // 2-D mode (RMVPE): tap offsets and border masking
    int toff[16] = {0};
    const unsigned* amax_in = nullptr;  // the |max| side channel (rvc_conv1d_args.amax_in / amax_out)
    unsigned* amax_out = nullptr;
    // the fused 1-channel source conv (rvc_conv1d_args.src_*; ops.conv1d's src): its weights, signal and geometry
    const ConvW* src = nullptr;
    const float* src_x = nullptr;
    int src_stride = 1, src_pad = 0;
    int64_t src_len = 0;
};

inline int conv(rvc_ctx* c, ModelBase& m, const ConvW& cw, const float* x, int64_t Lin, float* y, const CallOpts& o,
                hipStream_t s) {
    rvc_conv1d_args a;
    memset(&a, 0, sizeof(a));
    a.x = x;
    a.w = cw.w;
    a.bias = cw.b;
    a.bias2 = o.bias2;
    a.res = o.res;
    a.y = y;
    a.B = o.B;
    a.Ci = cw.Ci;
    a.Co = cw.Co;
    a.Lin = Lin;
    a.x_bstride = o.x_bstride;
    a.y_bstride = o.y_bstride;
    a.res_bstride = o.res_bstride;
    a.groups = cw.groups;
    a.in_act = o.in_act;
    a.in_slope = o.in_slope;
    a.in_scale = o.in_scale;
    a.out_act = o.out_act;
    a.out_slope = o.out_slope;
    a.out_scale = o.out_scale;
    a.accumulate = o.accumulate;
    a.K = cw.K;
    a.ntoff = o.ntoff;
    a.wrap = o.wrap;
    for (int i = 0; i < o.ntoff; ++i) a.toff[i] = o.toff[i];
    a.amax_in = o.amax_in;
    a.amax_out = o.amax_out;
    if (o.src) {
        a.src_x = o.src_x;
        a.src_w = o.src->w;
        a.src_b = o.src->b;
        a.src_K = o.src->K;
        a.src_stride = o.src_stride;
        a.src_pad = o.src_pad;
        a.src_len = o.src_len;
        a.src_bstride = o.src_len;
    }
    int stride = o.stride;
    if (cw.nphase > 1) {  // ConvT as u phase convs (ops.ConvT.__call__)
        const int64_t Lout = (Lin - 1) * cw.u - 2 * cw.tpad + cw.Kfull;
        a.Lout = Lout;
        a.ncols = (Lout - 1 + cw.tpad) / cw.u + 1;
        a.stride = 1;
        a.pad = cw.K - 1;
        a.dil = 1;
        a.nphase = cw.u;
        a.ostride = cw.u;
        a.ooffset = -cw.tpad;
        stride = 1;
    } else {
        a.Lout = o.Lout >= 0 ? o.Lout : (Lin + 2 * o.pad - o.dil * (cw.K - 1) - 1) / o.stride + 1;
        a.stride = o.stride;
        a.pad = o.pad;
        a.dil = o.dil;
        a.nphase = 1;
        a.ostride = 1;
    }
    if (cw.wx_bf) {
        const int passes = conv_passes(c, cw.K, cw.Ci / cw.groups, stride, o.ntoff > 0, o.amax_in != nullptr);
        a.wx = passes == RVC_ARITH_F16X3 ? cw.wx_hf : cw.wx_bf;
        a.wx_nmf = cw.nmf;
        a.wx_passes = passes;
    }
    const int64_t need = rvc_conv1d_workspace_bytes(&a);
    if (need < 0) return RVC_EINVAL;
    MTRY(ensure_ws(m, need, s));
    return rvc_conv1d(&a, need ? m.ws : nullptr, need, s);
}

// ------------------------------------------------------------------ scratch: a bump allocator run twice per shape
// (dry: sizes only, no launches -- RUN() skips them; then for real on an arena of that size)
struct Scratch {
    float* base = nullptr;
    int64_t off = 0;
    bool dry = true;
    float* take(int64_t n) {  // 256-B aligned
        float* p = dry ? (float*)(uintptr_t)(256 + off * 4) : base + off;
        off += (n + 63) & ~int64_t(63);
        return p;
    }
};
#define RUN(call)              \
    do {                       \
        if (!sc.dry) MTRY(call); \
    } while (0)

// fixed layouts: 256-B aligned float offsets
struct Plan {
    int64_t off = 0;
    int64_t take(int64_t n) {  // 256-B aligned float offsets
        const int64_t o = off;
        off += (n + 63) & ~int64_t(63);
        return o;
    }
};

inline bool env_on(const char* name) {
    const char* v = getenv(name);
    return !(v && strcmp(v, "0") == 0);
}

// a switch that is off unless set to something other than "0"
inline bool env_set(const char* name) {
    const char* v = getenv(name);
    return v && strcmp(v, "0") != 0;
}

}  // namespace rvcm
