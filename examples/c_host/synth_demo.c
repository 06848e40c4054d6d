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
#include "safetensors_min.h"

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

int main(int argc, char** argv) {
    if (argc != 4) DIE("usage: %s model.safetensors inputs.bin out.f32", argv[0]);
    char* keep;
    Model m = load_safetensors(argv[1], "rvc_synth_cfg", &keep);
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
