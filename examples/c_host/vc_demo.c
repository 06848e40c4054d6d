/*
 * A plain-C host of the whole VC.pipeline (convert.py:388-458) through the model-level ABI: ContentVec, RMVPE and
 * the voice model loaded from safetensors exports of their checkpoints (rvc_amd/native.py: export_safetensors),
 * one rvc_vc_convert_ex call on a 16 kHz clip of any length (inputs over 41 s are segmented at quiet points by
 * the library), the waveform at tgt_sr written out.
 *
 *   vc_demo hubert.safetensors rmvpe.safetensors model.safetensors audio16k.f32 out.f32 [pitch protect seed]
 *
 * hubert.safetensors carries __metadata__["rvc_contentvec_cfg"] (embed dim, heads, pos_conv groups, 0),
 * model.safetensors __metadata__["rvc_synth_cfg"] (rvc_synth_cfg in field order, the last being sr); v1 / v2 is
 * read off the model's phone width.  Build: make -C examples/c_host.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>

#include "safetensors_min.h"

#define HIPOK(x)                                                            \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) DIE("%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)
#define RVCOK(x)                                                               \
    do {                                                                       \
        int rc_ = (x);                                                         \
        if (rc_ != RVC_OK) DIE("%s -> %d: %s", #x, rc_, rvc_last_error()); \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 6) DIE("usage: %s hubert.st rmvpe.st model.st audio16k.f32 out.f32 [pitch protect seed]", argv[0]);
    char *k1, *k2, *k3;
    Model hub = load_safetensors(argv[1], "rvc_contentvec_cfg", &k1);
    Model rm = load_safetensors(argv[2], NULL, &k2);
    Model syn = load_safetensors(argv[3], "rvc_synth_cfg", &k3);
    if (hub.ncfg != 4) DIE("rvc_contentvec_cfg metadata: %d ints", hub.ncfg);
    if (syn.ncfg != (int)(sizeof(rvc_synth_cfg) / sizeof(int))) DIE("rvc_synth_cfg metadata: %d ints", syn.ncfg);
    rvc_contentvec_cfg hc;
    memcpy(&hc, hub.cfg, sizeof(hc));
    rvc_synth_cfg sc;
    memcpy(&sc, syn.cfg, sizeof(sc));

    size_t na;
    float* audio = (float*)slurp(argv[4], &na);
    const int64_t N = (int64_t)(na / 4);
    rvc_vc_args va;
    memset(&va, 0, sizeof(va));
    va.sid = 0;
    va.pitch_shift = argc > 6 ? atof(argv[6]) : 0.0;
    va.protect = argc > 7 ? (float)atof(argv[7]) : 0.33f;
    va.seed = argc > 8 ? strtoull(argv[8], NULL, 10) : 0;
    va.version = 2; /* set below from the phone width */
    va.x_pad = 1;
    va.x_max = 41;
    va.tgt_sr = sc.sr;

    rvc_ctx* ctx;
    RVCOK(rvc_ctx_create(0, &ctx));
    RVCOK(rvc_load_contentvec(ctx, hub.params, hub.n, &hc));
    RVCOK(rvc_load_rmvpe(ctx, rm.params, rm.n));
    RVCOK(rvc_load_synth(ctx, syn.params, syn.n, &sc));
    /* v1 models take final_proj's 256-wide phone, v2 the 768-wide encoder output */
    for (int i = 0; i < syn.n; ++i)
        if (!strcmp(syn.params[i].name, "enc_p.emb_phone.weight"))
            va.version = syn.params[i].shape[1] == hc.encoder_embed_dim ? 2 : 1;
    const int64_t n_cap = rvc_vc_out_len(ctx, N, &va); /* exact for one segment, an upper bound beyond 41 s */
    if (n_cap <= 0) DIE("rvc_vc_out_len: %s", rvc_last_error());
    void *d_audio, *d_out;
    HIPOK(hipMalloc(&d_audio, (size_t)N * 4));
    HIPOK(hipMalloc(&d_out, (size_t)n_cap * 4));
    HIPOK(hipMemcpy(d_audio, audio, (size_t)N * 4, hipMemcpyHostToDevice));
    hipStream_t s;
    HIPOK(hipStreamCreate(&s));
    int64_t n_out = 0;
    RVCOK(rvc_vc_convert_ex(ctx, (const float*)d_audio, N, &va, NULL, (float*)d_out, n_cap, &n_out, (rvc_stream_t)s));
    HIPOK(hipStreamSynchronize(s));
    RVCOK(rvc_rmvpe_check(ctx));
    float* out = (float*)malloc((size_t)n_out * 4);
    HIPOK(hipMemcpy(out, d_out, (size_t)n_out * 4, hipMemcpyDeviceToHost));
    FILE* f = fopen(argv[5], "wb");
    if (!f || fwrite(out, 4, (size_t)n_out, f) != (size_t)n_out) DIE("cannot write %s", argv[5]);
    fclose(f);
    double ss = 0;
    for (int64_t i = 0; i < n_out; ++i) ss += (double)out[i] * out[i];
    printf("vc_demo: v%d, %lld samples at 16 kHz -> %lld at %d Hz, rms %.6f\n", va.version, (long long)N,
           (long long)n_out, va.tgt_sr, sqrt(ss / (double)n_out));
    rvc_ctx_destroy(ctx);
    HIPOK(hipStreamDestroy(s));
    return 0;
}
