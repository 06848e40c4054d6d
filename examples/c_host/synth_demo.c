/*
 * A plain-C host of the model-level ABI (include/rvc_amd.h): loads a voice model's "weight" dict from a
 * safetensors file (the .pth exported unchanged -- fp16 weight_g / weight_v pairs included; the library
 * folds and packs them), runs Synthesizer.infer (synthesizers.py:446-465) once with device noise, and
 * writes the waveform.  No Python, no torch: the C ABI and the HIP runtime only.
 *
 *   synth_demo model.safetensors inputs.bin out.f32
 *
 * model.safetensors: the tensors plus __metadata__["rvc_synth_cfg"] = the rvc_synth_cfg ints in field order
 * (rvc_amd/native.py: export_synth_safetensors).  inputs.bin: int64 T, int64 E, int64 sid, uint64 seed,
 * then phone f32 [T][E], pitch int64 [T], pitchf f32 [T].  out.f32: wav f32 [rvc_synth_out_len(T)].
 * Build: make -C examples/c_host (gcc against include/rvc_amd.h, librvc_amd.so and libamdhip64.so)
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rvc_amd.h"

#define DIE(...)                      \
    do {                              \
        fprintf(stderr, __VA_ARGS__); \
        fputc('\n', stderr);          \
        exit(1);                      \
    } while (0)
#define HIPOK(x)                                                            \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) DIE("%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)
#define RVCOK(x)                                                 \
    do {                                                         \
        int rc_ = (x);                                           \
        if (rc_ != RVC_OK) DIE("%s -> %d: %s", #x, rc_, rvc_last_error()); \
    } while (0)

static char* slurp(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) DIE("cannot open %s", path);
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    char* b = (char*)malloc(*n + 1);
    if (!b || fread(b, 1, *n, f) != *n) DIE("cannot read %s", path);
    b[*n] = 0;
    fclose(f);
    return b;
}

/* ---- minimal safetensors header walk: {"name":{"dtype":"F16","shape":[..],"data_offsets":[a,b]}, ...} */
static const char* skip_ws(const char* p) {
    while (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r') ++p;
    return p;
}

static const char* read_str(const char* p, char* out, size_t cap) { /* p at '"' */
    size_t k = 0;
    for (++p; *p && *p != '"'; ++p) {
        if (*p == '\\' && p[1]) ++p;
        if (k + 1 < cap) out[k++] = *p;
    }
    out[k] = 0;
    return *p ? p + 1 : p;
}

static const char* skip_value(const char* p) { /* object, array, string or scalar */
    p = skip_ws(p);
    if (*p == '"') {
        char tmp[8];
        return read_str(p, tmp, sizeof(tmp));
    }
    if (*p == '{' || *p == '[') {
        int depth = 0;
        do {
            if (*p == '"') {
                char tmp[8];
                p = read_str(p, tmp, sizeof(tmp));
                continue;
            }
            if (*p == '{' || *p == '[') ++depth;
            if (*p == '}' || *p == ']') --depth;
            ++p;
        } while (*p && depth > 0);
        return p;
    }
    while (*p && *p != ',' && *p != '}') ++p;
    return p;
}

typedef struct {
    rvc_param* params;
    char** names;
    int n;
    int cfg[64];
    int ncfg;
} Model;

static void parse_tensor(const char* obj, const char* data, rvc_param* prm) {
    const char* d = strstr(obj, "\"dtype\"");
    const char* s = strstr(obj, "\"shape\"");
    const char* o = strstr(obj, "\"data_offsets\"");
    if (!d || !s || !o) DIE("bad tensor entry");
    char dt[16];
    read_str(skip_ws(strchr(d + 7, ':') + 1), dt, sizeof(dt));
    if (!strcmp(dt, "F16")) prm->dtype = RVC_DT_F16;
    else if (!strcmp(dt, "F32")) prm->dtype = RVC_DT_F32;
    else DIE("unsupported dtype %s", dt);
    const char* p = strchr(s, '[') + 1;
    prm->ndim = 0;
    while (*(p = skip_ws(p)) != ']') {
        if (prm->ndim == 4) DIE("more than 4 dims");
        prm->shape[prm->ndim++] = strtoll(p, (char**)&p, 10);
        p = skip_ws(p);
        if (*p == ',') ++p;
    }
    if (prm->ndim == 0) { /* a scalar: one element */
        prm->ndim = 1;
        prm->shape[0] = 1;
    }
    p = strchr(o, '[') + 1;
    const long long a = strtoll(p, (char**)&p, 10);
    prm->data = data + a;
}

static Model load_safetensors(const char* path, char** keep) {
    size_t n;
    char* buf = slurp(path, &n);
    *keep = buf;
    unsigned long long hlen;
    memcpy(&hlen, buf, 8);
    char* hdr = buf + 8;
    const char* data = hdr + hlen;
    char save = hdr[hlen];
    hdr[hlen] = 0;
    Model m = {0};
    m.params = (rvc_param*)calloc(4096, sizeof(rvc_param));
    m.names = (char**)calloc(4096, sizeof(char*));
    const char* p = skip_ws(hdr);
    if (*p != '{') DIE("bad safetensors header");
    ++p;
    for (;;) {
        p = skip_ws(p);
        if (*p == '}' || !*p) break;
        char key[256];
        p = read_str(p, key, sizeof(key));
        p = skip_ws(p);
        ++p; /* ':' */
        p = skip_ws(p);
        const char* end = skip_value(p);
        size_t len = (size_t)(end - p);
        char* obj = (char*)malloc(len + 1);
        memcpy(obj, p, len);
        obj[len] = 0;
        if (!strcmp(key, "__metadata__")) {
            const char* c = strstr(obj, "\"rvc_synth_cfg\"");
            if (c) {
                char val[1024];
                read_str(skip_ws(strchr(c + 15, ':') + 1), val, sizeof(val));
                char* q = val;
                while (*q && m.ncfg < 64) {
                    m.cfg[m.ncfg++] = (int)strtol(q, &q, 10);
                    while (*q == ' ') ++q;
                }
            }
        } else {
            if (m.n == 4096) DIE("too many tensors");
            m.names[m.n] = strdup(key);
            m.params[m.n].name = m.names[m.n];
            parse_tensor(obj, data, &m.params[m.n]);
            ++m.n;
        }
        free(obj);
        p = skip_ws(end);
        if (*p == ',') ++p;
    }
    hdr[hlen] = save;
    return m;
}

int main(int argc, char** argv) {
    if (argc != 4) DIE("usage: %s model.safetensors inputs.bin out.f32", argv[0]);
    char* keep;
    Model m = load_safetensors(argv[1], &keep);
    if (m.ncfg != (int)(sizeof(rvc_synth_cfg) / sizeof(int))) DIE("rvc_synth_cfg metadata: %d ints", m.ncfg);
    rvc_synth_cfg cfg;
    memcpy(&cfg, m.cfg, sizeof(cfg));

    size_t ni;
    char* in = slurp(argv[2], &ni);
    int64_t hdr[4];
    memcpy(hdr, in, sizeof(hdr));
    const int64_t T = hdr[0], E = hdr[1], sid = hdr[2];
    const uint64_t seed = (uint64_t)hdr[3];
    const size_t nphone = (size_t)(T * E) * 4, npitch = (size_t)T * 8, npf = (size_t)T * 4;
    if (ni != sizeof(hdr) + nphone + npitch + npf) DIE("inputs.bin: size mismatch");

    rvc_ctx* ctx;
    RVCOK(rvc_ctx_create(0, &ctx));
    RVCOK(rvc_load_synth(ctx, m.params, m.n, &cfg));
    const int64_t L = rvc_synth_out_len(ctx, T);
    void *phone, *pitch, *pitchf, *wav;
    HIPOK(hipMalloc(&phone, nphone));
    HIPOK(hipMalloc(&pitch, npitch));
    HIPOK(hipMalloc(&pitchf, npf));
    HIPOK(hipMalloc(&wav, (size_t)L * 4));
    HIPOK(hipMemcpy(phone, in + sizeof(hdr), nphone, hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(pitch, in + sizeof(hdr) + nphone, npitch, hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(pitchf, in + sizeof(hdr) + nphone + npitch, npf, hipMemcpyHostToDevice));
    hipStream_t s;
    HIPOK(hipStreamCreate(&s));
    RVCOK(rvc_synth_infer(ctx, (const float*)phone, (const int64_t*)pitch, (const float*)pitchf, 1, T, &sid, NULL, NULL,
                          seed, (float*)wav, (rvc_stream_t)s));
    HIPOK(hipStreamSynchronize(s));
    float* out = (float*)malloc((size_t)L * 4);
    HIPOK(hipMemcpy(out, wav, (size_t)L * 4, hipMemcpyDeviceToHost));
    FILE* f = fopen(argv[3], "wb");
    if (!f || fwrite(out, 4, (size_t)L, f) != (size_t)L) DIE("cannot write %s", argv[3]);
    fclose(f);
    double ss = 0, mx = 0;
    for (int64_t i = 0; i < L; ++i) {
        ss += (double)out[i] * out[i];
        if (out[i] > mx || -out[i] > mx) mx = out[i] > 0 ? out[i] : -out[i];
    }
    printf("synth_demo: %d tensors, T=%lld -> %lld samples, rms %.6f, peak %.6f\n", m.n, (long long)T, (long long)L,
           L ? sqrt(ss / L) : 0.0, mx);
    rvc_ctx_destroy(ctx);
    HIPOK(hipStreamDestroy(s));
    return 0;
}
