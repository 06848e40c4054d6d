/* Minimal safetensors reader for the plain-C hosts of the model-level ABI (synth_demo.c, vc_demo.c): the
 * header's tensor entries become rvc_param records pointing into the file image, and an optional
 * __metadata__ string of ints (key `meta_key`) is parsed into Model.cfg. */
#pragma once
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

static size_t dtype_size(int dt) { return dt == RVC_DT_F16 ? 2 : dt == RVC_DT_F32 ? 4 : 8; }

/* data_size: bytes after the header; every tensor's [a, b) must lie inside it and hold numel * dtype bytes */
static void parse_tensor(const char* obj, const char* data, size_t data_size, rvc_param* prm) {
    const char* d = strstr(obj, "\"dtype\"");
    const char* s = strstr(obj, "\"shape\"");
    const char* o = strstr(obj, "\"data_offsets\"");
    if (!d || !s || !o) DIE("bad tensor entry");
    const char* colon = strchr(d + 7, ':');
    if (!colon || *skip_ws(colon + 1) != '"') DIE("bad dtype");
    char dt[16];
    read_str(skip_ws(colon + 1), dt, sizeof(dt));
    if (!strcmp(dt, "F16")) prm->dtype = RVC_DT_F16;
    else if (!strcmp(dt, "F32")) prm->dtype = RVC_DT_F32;
    else if (!strcmp(dt, "F64")) prm->dtype = RVC_DT_F64;
    else DIE("unsupported dtype %s", dt);
    const char* p = strchr(s, '[');
    if (!p) DIE("bad shape");
    ++p;
    prm->ndim = 0;
    while (*(p = skip_ws(p)) != ']') {
        if (prm->ndim == 4) DIE("more than 4 dims");
        char* q;
        prm->shape[prm->ndim++] = strtoll(p, &q, 10);
        if (q == p) DIE("bad shape");
        p = q;
        p = skip_ws(p);
        if (*p == ',') ++p;
    }
    if (prm->ndim == 0) { /* a scalar: one element */
        prm->ndim = 1;
        prm->shape[0] = 1;
    }
    long long numel = 1;
    for (int i = 0; i < prm->ndim; ++i) {
        if (prm->shape[i] < 0 || (prm->shape[i] > 0 && numel > (1LL << 40) / prm->shape[i])) DIE("bad shape");
        numel *= prm->shape[i];
    }
    p = strchr(o, '[');
    if (!p) DIE("bad data_offsets");
    ++p;
    const long long a = strtoll(p, (char**)&p, 10);
    p = skip_ws(p);
    if (*p != ',') DIE("bad data_offsets");
    const long long b = strtoll(p + 1, (char**)&p, 10);
    if (a < 0 || a > b || (unsigned long long)b > (unsigned long long)data_size)
        DIE("data_offsets [%lld, %lld) outside the %zu data bytes", a, b, data_size);
    if ((unsigned long long)(b - a) != (unsigned long long)numel * dtype_size(prm->dtype))
        DIE("data_offsets span %lld bytes, shape x dtype needs %lld", b - a, numel * (long long)dtype_size(prm->dtype));
    prm->data = data + a;
}

static Model load_safetensors(const char* path, const char* meta_key, char** keep) {
    size_t n;
    char* buf = slurp(path, &n);
    *keep = buf;
    unsigned long long hlen;
    if (n < 8) DIE("%s: truncated safetensors file", path);
    memcpy(&hlen, buf, 8);
    if (hlen > n - 8) DIE("%s: header length %llu exceeds the file", path, hlen);
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
        if (*p != '"') DIE("bad safetensors header");
        p = read_str(p, key, sizeof(key));
        p = skip_ws(p);
        if (*p != ':') DIE("bad safetensors header");
        ++p;
        p = skip_ws(p);
        const char* end = skip_value(p);
        size_t len = (size_t)(end - p);
        char* obj = (char*)malloc(len + 1);
        memcpy(obj, p, len);
        obj[len] = 0;
        if (!strcmp(key, "__metadata__")) {
            char pat[128];
            snprintf(pat, sizeof(pat), "\"%s\"", meta_key ? meta_key : "");
            const char* c = meta_key ? strstr(obj, pat) : NULL;
            const char* colon = c ? strchr(c + strlen(pat), ':') : NULL;
            if (c && (!colon || *skip_ws(colon + 1) != '"')) DIE("bad metadata %s", meta_key);
            if (c) {
                char val[1024];
                read_str(skip_ws(colon + 1), val, sizeof(val));
                char* q = val;
                while (*q && m.ncfg < 64) {
                    char* e;
                    m.cfg[m.ncfg++] = (int)strtol(q, &e, 10);
                    if (e == q) DIE("bad metadata %s: not a list of ints", meta_key);
                    q = e;
                    while (*q == ' ') ++q;
                }
            }
        } else {
            if (m.n == 4096) DIE("too many tensors");
            m.names[m.n] = strdup(key);
            m.params[m.n].name = m.names[m.n];
            parse_tensor(obj, data, n - 8 - hlen, &m.params[m.n]);
            ++m.n;
        }
        free(obj);
        p = skip_ws(end);
        if (*p == ',') ++p;
    }
    hdr[hlen] = save;
    return m;
}

