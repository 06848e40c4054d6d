/*
 * rvc_amd.h -- C ABI of librvc_amd.so, the MI355X (gfx950) kernels behind the
 * RVC-MAKER voice-conversion hot path (main/inference/convert.py:VC.pipeline).
 *
 * The reference is pure Python/PyTorch: it has no FFI of its own on this path
 * (SURVEY §0).  Every entry point below replaces the torch op(s) the reference
 * executes at the cited file:line; the Python host package (rvc-maker_amd/rvc_amd)
 * binds them with ctypes the way the reference's only native binding
 * (main/library/predictors/WORLD_WRAPPER.py:30-90: ctypes.CDLL, option structs,
 * caller-allocated outputs) does.  INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - All tensors are caller-owned DEVICE buffers (fp32 unless stated), dense,
 *     channels-first [B][C][L] like torch's NCL.  The library allocates nothing.
 *   - Every call is stream-ordered on the given hipStream_t and never
 *     synchronises; it returns RVC_OK or a negative code, with the message in
 *     rvc_last_error() (thread-local).
 *   - Weights are pre-packed by the host loader (weight-norm / BatchNorm folded,
 *     transposed to K-major "KM" = [groups][Cin/groups * K][Cout/groups]).
 */
#ifndef RVC_AMD_H
#define RVC_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* rvc_stream_t; /* == hipStream_t */

enum { RVC_OK = 0, RVC_EINVAL = -22, RVC_EHIP = -5 };

enum {
    RVC_ACT_NONE = 0,
    RVC_ACT_LRELU = 1,
    RVC_ACT_RELU = 2,
    RVC_ACT_TANH = 3,
    RVC_ACT_GELU = 4, /* exact erf GELU (torch.nn.GELU / F.gelu) */
    RVC_ACT_SIGMOID = 5,
    RVC_ACT_LOGCLAMP = 6, /* log(max(v, slope))  (RMVPE.py:181) */
};

const char* rvc_last_error(void);
int rvc_version(void);

/* ------------------------------------------------------------------ conv1d
 * Implicit-GEMM 1-D convolution on f32 MFMA (v_mfma_f32_16x16x4_f32).
 * Replaces every torch.nn.Conv1d / F.conv1d on the path:
 *   NSF-HiFiGAN conv_pre / noise_convs / ResBlock convs / conv_post
 *     (synthesizers.py:123,136,161; residuals.py:16-17,32-36),
 *   flow WaveNet + 1x1 convs (modules.py:27-44, residuals.py:120-129),
 *   TextEncoder FFN / q,k,v,o / proj (synthesizers.py:198-202,298-305,364),
 *   ContentVec conv feature extractor and pos_conv and every nn.Linear
 *     (fairseq.py:1165-1195, 585-592, 204-225, 778-814) as a K=1 conv,
 *   and, one phase per grid.z, ConvTranspose1d (synthesizers.py:133) through
 *   the polyphase weight packing done by the host.
 *
 *   v = out_scale * act(sum_{c,k} W[m][c][k] * pre(x[b][c][col*stride - pad + k*dil]) + bias[m] + bias2[m])
 *   v += res[b][m][t]                       (if res)
 *   y[b][m][t] = v  or  y[b][m][t] += v     (accumulate),   t = col*ostride + ooffset + phase
 *   pre(v) = in_act(v * in_scale)
 */
#define RVC_ARITH_F16X3 16 /* rvc_conv1d_args.wx_passes / rvc_resblock_args.passes: split-fp16, 3 passes */
#define RVC_AMAX_SHARDS 64 /* u32 words per |max| cell (rvc_conv1d_args.amax_in / amax_out) */
#define RVC_ARITH_FP32_SA 7 /* rvc_conv1d_args.wx_passes: 6-pass split-bf16 with the correction passes in their
                               own f32 accumulators (fewer roundings of the large sum; RMVPE) */

typedef struct rvc_conv1d_args {
    const float* x;    /* [B][Ci][Lin] with batch stride x_bstride           */
    const float* w;    /* KM packed: [nphase][groups][Ci/g*K][Co/g]            */
    const float* bias; /* [Co] or NULL                                          */
    const float* bias2;/* [Co] or NULL: second per-channel term added after bias
                          (speaker conditioning: synthesizers.py:147, modules.py:39-43) */
    const float* res;  /* [B][Co][Lout] residual added after the activation, or NULL */
    float* y;          /* [B][Co][Lout]                                         */
    int64_t B, Ci, Co, Lin, Lout;
    int64_t ncols;     /* GEMM columns per phase (== Lout for a plain conv)     */
    int64_t x_bstride, y_bstride, res_bstride, w_bstride; /* 0 = dense default; w: 0 = shared */
    int K, stride, dil, pad, groups;
    int nphase, ostride, ooffset;
    int in_act, out_act, accumulate, _pad0;
    float in_scale, in_slope, out_slope, out_scale;
    /* 2-D mode (RMVPE 3x3 convs on zero-bordered [C][H+2][W+2] images flattened to L):
       ntoff > 0 replaces tap*dil by toff[tap]; wrap > 0 skips stores to border cells
       (t % wrap in {0, wrap-1}, or t / wrap in {0, Lout/wrap - 1}). */
    int ntoff, wrap;
    int toff[16];
    /* Split-bf16 engine: wx = the same weights pre-split into bf16 h/m/l planes by
       rvc_conv1d_pack_x6 (NULL = f32 MFMA engine).  Used for stride-1 (and stride-2) 1-D convs --
       ungrouped (<= 64 taps), or grouped (<= 128 taps, nphase 1, stride 1, no src_*) with the image packed
       with the groups as phases: pack_x6(w, groups, Ci/g, K, Co/g); other shapes ignore it.
       wx_nmf = its padded 16-row fragment count.
       wx_passes: bf16 MFMA passes per product -- 0 or 6 = f32-accurate (hH+hM+mH+hL+mM+lH, products to
       2^-24), RVC_ARITH_FP32_SA = the same 6 passes with hH and the 5 corrections accumulated apart (RMVPE,
       whose f0 is a per-frame decision), 3 = hH+hM+mH (16-bit operand mantissas), 1 = hH (bf16 operands);
       f32 accumulation always.
       RVC_ARITH_F16X3: wx is an rvc_conv1d_pack_f16 image instead -- split-fp16 operands (per-row
       weight and per-tile activation power-of-2 scales, 11 + 11 significant bits each), hH + hL + lH
       on the fp16 MFMA: ~2^-20 relative per product, f32 accumulation. */
    const void* wx;
    int wx_nmf, wx_passes;
    /* Tensor |max| side channel (round 5): amax_out (or NULL) is a cell of RVC_AMAX_SHARDS u32 words that receives
       max |y| over every value the launch stores (atomic maxes of the f32 bits, spread over the words; the caller
       zeroes the cell before the producing launch), and amax_in (or NULL) is such a cell for x: a split-fp16
       launch (RVC_ARITH_F16X3) then takes its activation scale from the largest word (times |in_scale|: an upper
       bound of |pre(x)|) instead of a per-tile |max| pre-pass over its input.
       A batched launch (B > 1) takes B consecutive cells, one per batch element: element b's at
       amax + b * RVC_AMAX_SHARDS (round 6), so a clip's scale never depends on the other clips of its batch. */
    const unsigned* amax_in;
    unsigned* amax_out;
    /* Fused source conv (round 6; NULL src_x = none): every stored output y[b][m][t] also adds
       sum_k src_w[k][m] * src_x[b][t * src_stride - src_pad + k] + src_b[m] (zero outside [0, src_len)), after the
       residual and accumulate operands -- a 1-input-channel conv of src_K taps over a [B][src_len] signal (batch
       stride src_bstride, 0 = src_len; src_w KM-packed [src_K][Co] as a Ci = 1 conv weight, src_b [Co] or NULL).
       The NSF generator's x = ups(x) + noise_convs(har) (synthesizers.py:156) in the upsampling conv's call: a
       read-modify-write pass right after the conv (a direct kernel, HBM-bound, instead of the 1-channel conv as an
       implicit GEMM K deep); amax_out then receives the final values' |max|.  The k-sum is an fmaf chain in tap
       order from 0, then + src_b, so it equals the separate 1-channel conv on the f32 engine with accumulate. */
    const float* src_x;
    const float* src_w;
    const float* src_b;
    int src_K, src_stride, src_pad, _pad1;
    int64_t src_len, src_bstride;
} rvc_conv1d_args;

/* Split-K (chosen by the library when the tile grid would underfill the 256 CUs) needs a caller-owned
 * device workspace of rvc_conv1d_workspace_bytes(a) bytes (0 when not split; -1 on bad args).  Launches
 * that may run concurrently need separate workspaces. */
int64_t rvc_conv1d_workspace_bytes(const rvc_conv1d_args* a);
/* Which engine a call would run on: 0 = f32 MFMA, 1 = split-bf16 (x6); -1 on bad args. */
int rvc_conv1d_engine(const rvc_conv1d_args* a);
int rvc_conv1d(const rvc_conv1d_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream);
/* Profiling hook (this host thread): while set to a hipEvent_t, each rvc_conv1d call records it on its stream
 * right after the conv kernel, before any split-K reduce, so that a caller's events can bracket the conv
 * kernel alone (bench.py's roofline probe).  NULL (the default) turns it off. */
void rvc_conv1d_set_probe_event(void* hip_event);
/* Diagnostic build only (-DRVC_CONV_STAMPS=1, scripts/conv_stamps.py): the split-operand conv engine's per-block
 * phase stamps (s_memtime) go to buf ([bytes / 2048][256] u64); returns -1 in a production build. */
int rvc_conv1d_set_stamps(void* buf, int64_t bytes);
/* The same for the fused ResBlock pair (rvc_resblock_pair): per workgroup, per tile phase stamps (scripts/rb_stamps.py);
 * -1 in a production build. */
int rvc_resblock_set_stamps(void* buf, int64_t bytes);
/* The fused pair's output path for this thread's launches (round 6): 1 = split-fp16 pairs at C <= 64 write c2's results
 * into LDS (over the tile's residual rows) and the loader waves store them during the next tile (the compute waves go
 * straight on); 2 = the same, and at C = 32 (two R buffers by tile parity) after the next tile's c1 barriers instead of
 * before them; 0 = the compute waves' own global stores; -1 = RVC_RB_YLDS (default 2).  Same bits in every form. */
int rvc_resblock_set_ylds(int on);
/* The fused pair's C = 64 tiling for this thread's launches (round 6): 1 = 2 row fragments per compute wave, 240
 * outputs per tile (the <= 2-plane pass sets; 6-pass pairs keep the narrow form), 0 = 1 row fragment, 112 outputs,
 * -1 = RVC_RB_WIDE64 (default 1).  The same sums in the same order; split-fp16's power-of-2 tile scales follow the
 * tile, so results agree to that arithmetic's precision rather than bit for bit.  Returns the previous setting. */
int rvc_resblock_set_wide64(int on);
/* The split-operand engine's epilogue form for this thread's launches: 1 = the tile epilogue through LDS (on the
 * 128-wide tiles where it needs no extra LDS), 0 = the in-register epilogue, -1 = RVC_X6_TILE_EPI (default 0).  Both give the same bits (tests/test_gpu_ops.py);
 * an A/B switch for measurements in one process. */
int rvc_conv1d_set_tile_epi(int on);
/* The split-operand engine's in-register epilogue in 128-byte rows (round 6: a v_permlane16_swap per accumulator pair
 * regroups two 16-column fragments into 2 rows x 32 columns per register, so every residual / accumulate load and
 * store moves 2 x 128-B segments instead of 4 x 64 B): 1 on, 0 off, -1 RVC_X6_SWZ (default 1).  Same bits. */
int rvc_conv1d_set_swz(int on);
/* Per-thread override of the split-fp16 loaders' fast form (used with amax_in on the 8-compute-wave tiles; same
 * bits as the general form): 1 on, 0 off, -1 back to RVC_X6_F16FAST (default on).  Diagnostic / test knob. */
int rvc_conv1d_set_f16_fast(int on);
/* Split-K policy (this host thread): the library splits a conv's k range over blocks while its tile grid is
 * below `target` tiles (default 256 = 1 per CU, halved for tiles of which one block fills a CU; or
 * RVC_SPLITK_TILES); 0 = never split, -1 = back to the default.  Returns the previous setting.  Results depend on it at f32 rounding level (the split changes the
 * summation order). */
int rvc_conv1d_set_splitk_target(int target);
/* A stream restricted to the CUs set in mask (nwords 32-bit words, bit i = CU i), and its release. */
int rvc_stream_create_cu_mask(const uint32_t* mask, int nwords, rvc_stream_t* out);
int rvc_stream_destroy(rvc_stream_t stream);
/* Pack KM weights [nphase][Ci*K][Co] (one group) for the split-bf16 engine: out must hold
 * rvc_conv1d_x6_bytes(nphase, Ci, K, Co) bytes; *nmf_out receives wx_nmf. */
int64_t rvc_conv1d_x6_bytes(int64_t nphase, int64_t Ci, int K, int64_t Co);
int rvc_conv1d_pack_x6(const float* w_km, int64_t nphase, int64_t Ci, int K, int64_t Co, void* out, int* nmf_out,
                       rvc_stream_t stream);
/* The split-fp16 image (wx with wx_passes = RVC_ARITH_F16X3): the x6 fragment layout holding the fp16 h / l
 * planes of each output row's weights scaled by a power of 2 (max |w| below 2^14), followed by the rows'
 * reciprocal scales (f32 [wx_nmf * 16]); rvc_conv1d_f16_bytes(...) bytes, *nmf_out as for pack_x6. */
int64_t rvc_conv1d_f16_bytes(int64_t nphase, int64_t Ci, int K, int64_t Co);
int rvc_conv1d_pack_f16(const float* w_km, int64_t nphase, int64_t Ci, int K, int64_t Co, void* out, int* nmf_out,
                        rvc_stream_t stream);

/* ------------------------------------------------------------------ fused ResBlock pair
 * One (convs1[i], convs2[i]) pair of the NSF-HiFiGAN ResBlock (residuals.py:22-44) in one launch:
 *   y = x + c2(lrelu(c1(lrelu(x), dilation dil, pad dil*(K-1)/2)), pad (K-1)/2)   [+ y when accumulate]
 * on the split-bf16 engine, with c1's output kept in LDS (never written to HBM).  C = 32 or 64 channels
 * (the generator's last two stages, synthesizers.py:157-159), odd K <= 15, (K-1)*dil <= 64.
 * w1x / w2x: the convs' rvc_conv1d_pack_x6 images (nphase 1, Ci = Co = C; nmf1 / nmf2 their wx_nmf);
 * b1 / b2: f32 biases [C]; passes 6 / 3 / 1 as rvc_conv1d_args.wx_passes; slope: the lrelu slope (0.1).
 * x and y must not alias.  Bit-identical to the two rvc_conv1d launches it replaces.
 * B clips (0 = 1): x, y are [B][C][L] (dense); each clip's result is bit-identical to a B = 1 call on it. */
typedef struct rvc_resblock_args {
    const float* x;
    float* y;
    const void* w1x;
    const float* b1;
    const void* w2x;
    const float* b2;
    int64_t C, L;
    int K, dil, nmf1, nmf2, passes, accumulate;
    float slope;
    int B;
} rvc_resblock_args;

int64_t rvc_resblock_lds_bytes(int64_t C, int K, int dil, int passes);
int rvc_resblock_pair(const rvc_resblock_args* a, rvc_stream_t stream);

/* ------------------------------------------------------------------ attention
 * Flash-style multi-head attention on f32 MFMA over channels-first Q/K/V
 * ([B][H][D][T], channel stride ldc, t contiguous); O written in the same layout.
 * Replaces F.multi_head_attention_forward in ContentVec (fairseq.py:355-357,
 * D = 64, no mask: the single padded key of :1106-1111 has weight exactly 0) and
 * the TextEncoder's relative-position MHA (synthesizers.py:227-251, D = 96,
 * window W = 10): pass rk = scale * Q^T Ek as [B][H][2W+1][T], ev = Ev [2W+1][D]
 * and an ml scratch [B][H][2][T]; the value band term is added in a second pass.
 */
typedef struct rvc_attn_args {
    const float* q;
    const float* k;
    const float* v;
    float* o;
    const float* rk; /* NULL = no relative band                */
    const float* ev; /* [2W+1][D] (shared by heads) or NULL     */
    float* ml;       /* [B][H][2][T] scratch (required with rk) */
    int64_t B, H, D, T;
    int64_t ldc;                    /* channel stride (0 = T) */
    int64_t q_hs, k_hs, v_hs, o_hs; /* head strides           */
    int64_t q_bs, k_bs, v_bs, o_bs; /* batch strides          */
    int W, _pad0;
    float scale, _pad1;
} rvc_attn_args;

/* Long sequences are split over the keys (split-KV) to fill the chip; the partials need a
 * workspace of rvc_attention_workspace_bytes(a) bytes (0 when not split). */
int64_t rvc_attention_workspace_bytes(const rvc_attn_args* a);
int rvc_attention(const rvc_attn_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream);
/* the same, also folding max |o| into a |max| cell per batch element (amax_out as rvc_layernorm_cf_amax; with the
 * relative band only together with its value term ev, whose kernel publishes the final values) */
int rvc_attention_amax(const rvc_attn_args* a, unsigned* amax_out, void* ws, int64_t ws_bytes, rvc_stream_t stream);
/* Round 6: with amax_in (the |max| cell of q, k and v -- the QKV projection's published cell, one per batch element)
 * both products run in split-fp16 on the fp16 matrix cores (power-of-2 scaled operands split into 11 + 11 bit fp16
 * pieces, hH + hL + lH, f32 accumulation: ~2^-22 relative per product, the conv engine's arithmetic); NULL amax_in =
 * the f32-MFMA kernel.  amax_out as rvc_attention_amax. */
int rvc_attention_ex(const rvc_attn_args* a, const unsigned* amax_in, unsigned* amax_out, void* ws, int64_t ws_bytes,
                     rvc_stream_t stream);
/* This thread's choice for rvc_attention_ex with amax_in: 1 split-fp16, 0 the f32 kernel, -1 RVC_ATTN_F16 (default 1).
 * A/B and test knob. */
int rvc_attention_set_f16(int on);

/* ------------------------------------------------------------------ elementwise
 * Memory-bound pieces of Synthesizer.infer (synthesizers.py:446-465).  All
 * [B][C][T] channels-first.
 */
/* out = lrelu((lin + emb[pitch]) * scale, slope)       synthesizers.py:367 */
int rvc_textenc_embed(const float* lin, const float* emb, const int64_t* pitch, float* out, int64_t B, int64_t C,
                      int64_t T, float scale, float slope, rvc_stream_t stream);
/* the same, also folding max |out| into a |max| cell per batch element (round 6: the TextEncoder's first split-fp16
 * GEMM takes its scale from it) */
int rvc_textenc_embed_amax(const float* lin, const float* emb, const int64_t* pitch, float* out, int64_t B, int64_t C,
                           int64_t T, float scale, float slope, unsigned* amax_out, rvc_stream_t stream);
/* LayerNorm over channels of (x + res)                  synthesizers.py:170-181, fairseq.py:700 */
int rvc_layernorm_cf(const float* x, const float* res, const float* gamma, const float* beta, float* out, int64_t B,
                     int64_t C, int64_t T, float eps, rvc_stream_t stream);
/* the same, also folding max |out| into a |max| cell (amax_out: RVC_AMAX_SHARDS zeroed u32 words per batch element, the
 * amax_in of the GEMM that reads out; ContentVec's LayerNorms -- any C <= 2048, both LayerNorm forms) */
int rvc_layernorm_cf_amax(const float* x, const float* res, const float* gamma, const float* beta, float* out,
                          int64_t B, int64_t C, int64_t T, float eps, unsigned* amax_out, rvc_stream_t stream);
/* GroupNorm(C, C) over time + affine (+ exact GELU)      fairseq.py:1149-1155,1183-1185 */
int rvc_chnorm_gelu(const float* x, const float* gamma, const float* beta, float* out, int64_t B, int64_t C, int64_t L,
                    float eps, int gelu, rvc_stream_t stream);
/* ContentVec's first layer fused (fairseq.py:1165-1195, layer 0): conv(1 -> C, k K, stride) of the 16 kHz signal x
 * [B][N] (w_km: the K-major packed weight [K][C], no bias) + GroupNorm(C, C) over time + affine (+ exact GELU) ->
 * out [B][C][T], T = (N - K) / stride + 1; statistics in f64.  ws: rvc_fe0_ws_bytes(B, C, T) device bytes.
 * Replaces rvc_conv1d + rvc_chnorm_gelu for that layer (no HBM round trip of the conv output). */
int64_t rvc_fe0_ws_bytes(int64_t B, int64_t C, int64_t T);
int rvc_fe0_gn_gelu(const float* x, int64_t B, int64_t N, int64_t x_bstride, const float* w_km, int64_t C, int K,
                    int stride, const float* gamma, const float* beta, float* out, float eps, int gelu, void* ws,
                    int64_t ws_bytes, rvc_stream_t stream);
/* the same, also folding max |out| into a |max| cell per batch element (amax_out as rvc_layernorm_cf_amax): layer 1's
 * split-fp16 conv takes its activation scale from it (round 6).  C <= 819 (the per-channel LDS records), K <= 16. */
int rvc_fe0_gn_gelu_amax(const float* x, int64_t B, int64_t N, int64_t x_bstride, const float* w_km, int64_t C, int K,
                         int stride, const float* gamma, const float* beta, float* out, float eps, int gelu,
                         unsigned* amax_out, void* ws, int64_t ws_bytes, rvc_stream_t stream);
/* z_p = m + exp(logs) * noise * nscale, stats = [m; logs]  synthesizers.py:449 */
int rvc_prior_sample(const float* stats, const float* noise, float* zp, int64_t B, int64_t C, int64_t T, float nscale,
                     rvc_stream_t stream);
/* out = tanh(a[:H]) * sigmoid(a[H:])                    commons.py:35-41 */
int rvc_gate(const float* a, float* out, int64_t B, int64_t H, int64_t T, rvc_stream_t stream);
/* out[c] = x[C-1-c]                                      residuals.py:53-58 */
int rvc_flip_channels(const float* x, float* out, int64_t B, int64_t C, int64_t T, rvc_stream_t stream);
/* out[b][c][r] = in[b][r][c] */
int rvc_transpose(const float* in, float* out, int64_t B, int64_t R, int64_t C, rvc_stream_t stream);
/* standard normal noise, Philox4x32-10 counter stream (seed, offset) */
int rvc_randn(float* out, int64_t n, uint64_t seed, uint64_t offset, rvc_stream_t stream);
/* the same with seed += *seed_add read on the device (seed_add may be NULL): graph replays draw fresh noise */
int rvc_randn_ex(float* out, int64_t n, uint64_t seed, uint64_t offset, const uint64_t* seed_add,
                 rvc_stream_t stream);
/* symmetric triangular draws on [lo, hi] (CREPE's dither, scipy.stats.triang(c=0.5), CREPE.py:118),
 * same counter stream; used when the CREPE pass is graph-captured (host numpy draws cannot be) */
int rvc_rand_triang(float* out, int64_t n, float lo, float hi, uint64_t seed, uint64_t offset,
                    const uint64_t* seed_add, rvc_stream_t stream);
/* NSF harmonic source: SineGen + Linear(1,1) + tanh    synthesizers.py:69-112
 * f0 [B][T] -> har [B][T*upp]; noise [B][T*upp]; work: [B][T] floats scratch */
int rvc_sine_source(const float* f0, const float* noise, float* har, float* work, int64_t B, int64_t T, int upp,
                    float sr, float lin_w, float lin_b, rvc_stream_t stream);

/* ------------------------------------------------------------------ RMVPE (RMVPE.py)
 * framesT[n][f] = x[reflect(f*hop + n - nfft/2)] * win[n]               RMVPE.py:168 (torch.stft center)
 * mag[k][f] = |spec[k][f] + i spec[K+k][f]|                            RMVPE.py:169
 * img (bordered [Tp+2][M+2]) = BN(mel^T), frames reflect-padded to Tp     RMVPE.py:64,144,213
 * avgpool2 / interleave4 on bordered images                              RMVPE.py:35,93
 * img_to_seq: [C][H][W] image -> [C*W][H] sequence                       RMVPE.py:144
 * bigru: recurrence of nn.GRU(384, 256, bidirectional); gi = W_ih x + b_ih
 *        [2][768][T], whh [2][768][256], bhh [2][768], y [512][T];
 *        gran_ws: 8 KiB scratch (zeroed by the call), err: device int set to 1 when a step's hand-off wait
 *        exceeds the spin limit (the kernel then drains and y is incomplete); sticky until the caller clears it
 * bigru_set_spin_limit: polls per hand-off wait before the timeout fires (default 2^22); 0 only queries.
 *        Returns the previous limit.  For tests that force the timeout path.
 * rmvpe_decode: salience [360][ld] -> f0 (f64, optional), coarse (int64), pitchf (f32)
 *        RMVPE.py:217-252 + convert.py:311-323, f64, numpy's reduction order
 */
int rvc_stft_frames(const float* x, const float* win, float* framesT, int64_t N, int64_t F, int nfft, int hop,
                    rvc_stream_t stream);
int rvc_spec_mag(const float* spec, float* mag, int64_t K, int64_t F, rvc_stream_t stream);
/* stft_mag: B signals x [b * x_bstride + n] (n < N) -> mag [b * mag_bstride + k * F + f] = |STFT| (k <= nfft/2),
 *        reflect-centred frames x win (torch.stft center=True + sqrt(re^2 + im^2), RMVPE.py:168-169), an f64 FFT
 *        rounded to f32 once; nfft a power of 2 <= 1024.  Replaces stft_frames + the DFT GEMM + spec_mag. */
int rvc_stft_mag(const float* x, const float* win, float* mag, int64_t B, int64_t N, int64_t F, int nfft, int hop,
                 int64_t x_bstride, int64_t mag_bstride, rvc_stream_t stream);
int rvc_mel_image(const float* mel, float* img, int64_t M, int64_t F, int64_t Tp, float scale, float shift,
                  rvc_stream_t stream);
int rvc_avgpool2(const float* in, float* out, int64_t C, int64_t H, int64_t W, rvc_stream_t stream);
int rvc_interleave4(const float* phases, float* out, int64_t C, int64_t H, int64_t W, rvc_stream_t stream);
int rvc_img_to_seq(const float* img, float* x, int64_t C, int64_t H, int64_t W, rvc_stream_t stream);
int rvc_bigru(const float* gi, const float* whh, const float* bhh, float* y, void* gran_ws, int* err, int64_t T,
              rvc_stream_t stream);
unsigned rvc_bigru_set_spin_limit(unsigned limit);
/* bigru_batched: B independent sequences (gi + b*gi_bs, y + b*y_bs); gran_ws: 8192 B * min(B, 16) scratch. */
int rvc_bigru_batched(const float* gi, int64_t gi_bs, const float* whh, const float* bhh, float* y, int64_t y_bs,
                      void* gran_ws, int* err, int64_t B, int64_t T, rvc_stream_t stream);

/* ------------------------------------------------------------------ RMVPE in f64 (rmvpe64.hip)
 * RMVPE's f0 is a per-frame decision (argmax over 360 bins, 0.03 voicing threshold, RMVPE.py:217-252) and
 * some frames' top two bins lie closer than any f32 evaluation of the network resolves, so the f0 model runs
 * in f64 end to end (rvc_rmvpe_forward): the same steps as the f32 entry points above, on f64
 * buffers, with the salience rounded to f32 once.
 *
 * conv64: y[b][m][t] = act(sum_{c,k} w[c*K + k][m] x[b][c][t - pad + off(k)] + bias[m]) (+ res[b][m][t]),
 *   off(k) = toff[k] (ntoff == K) or k; x positions outside [0, Lin) read 0.  w is KM [Ci*K][Co] f64.
 *   wrap > 0: 2-D mode on zero-bordered images flattened to Lout = rows x wrap -- border cells are stored as 0.
 *   y is f64, or f32 (rounded once) when y_f32.  out_act: RVC_ACT_NONE / RELU / SIGMOID / LOGCLAMP (out_slope =
 *   the clamp).
 *   Stride 1, no groups.  Replaces torch.nn.Conv2d (3x3 pad 1 / 1x1) and nn.Linear in E2E / MelSpectrogram
 *   (RMVPE.py:11-44, 78-107, 141-144, 162-181), batch b in [0, B) with strides (0 = dense). */
typedef struct rvc_conv64_args {
    const double* x;
    const double* w;
    const double* bias;
    const double* res;
    void* y;
    int64_t B, Ci, Co, Lin, Lout;
    int64_t x_bstride, y_bstride, res_bstride;
    int K, pad, out_act, y_f32;
    double out_slope;
    int ntoff, wrap;
    int toff[16];
    /* per-batch weights: batch b uses w + (b % w_bmod) * w_bstride (w_bmod 0: every batch the same w) */
    int64_t w_bstride;
    int w_bmod, _pad0;
} rvc_conv64_args;
/* split-K workspace (bytes; 0 = none, -1 = bad args), as rvc_conv1d_workspace_bytes */
int64_t rvc_conv64_workspace_bytes(const rvc_conv64_args* a);
/* the planner's choice for a (diagnostics): out[0] tile (0..7: 16x512, 16x256, 32x256, 32x128, 64x128, 64x64,
 * 128x128, 128x64 with 16-deep k chunks; 8..12: 16x256, 32x128, 64x128, 64x64, 128x64 with 32-deep; 13, 14: 128x16
 * with 16- / 32-deep; 15..17: 16x256, 32x128, 32x256 with 36-deep = 4 whole channels of a 3x3 conv), out[1] split-K, out[2] compact form (wrap > 0: the H x W interior cells as the GEMM's
 * columns instead of the bordered image), out[3] blocks of the conv launch */
int rvc_conv64_plan(const rvc_conv64_args* a, int* out);
/* force the planner (process-wide; sweeps and tests): tile -1..17, ksplit -1..32, compact -1..1 (-1 = planner's) */
int rvc_conv64_set_plan(int tile, int ksplit, int compact);
int rvc_conv64(const rvc_conv64_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream);
/* Winograd F(4x4, 3x3) f64 conv for RMVPE's deep levels (3x3 pad 1 on bordered [C][H+2][W+2] images, as
 * conv64 with wrap): y = act(conv(x) + bias) (+ res), border cells 0.  v = rvc_wino64_weights(KM w [Ci*9][Co])
 * = the 36 transformed weight matrices [36][Ci][Co] (G g G^T).  rvc_wino64_use(Ci, Co, H, W): whether the f64
 * RMVPE takes this form for a Ci -> Co conv on an H x W image (>= 64 channels each and >= 90 4x4 output tiles,
 * RVC_RMVPE_WINO_MINP; H or W <= 0: the channel rule alone, whether to prepare v; RVC_RMVPE_WINO=0: never).
 * rvc_wino64_conv itself takes any channel counts: 16 / 32 / 64 -> 16 / 32 channels run one fused kernel (transforms
 * in LDS, no workspace; measured no faster than conv64, so rvc_wino64_use leaves those shapes to conv64 unless
 * RVC_RMVPE_WINO=3), the rest the three-step form with its workspace. */
typedef struct rvc_wino64_args {
    const double* x;
    const double* v;
    const double* bias;
    const double* res;
    void* y;
    int64_t B, Ci, Co, H, W;
    int64_t x_bstride, y_bstride, res_bstride;
    int out_act, y_f32;
} rvc_wino64_args;
int rvc_wino64_use(int64_t Ci, int64_t Co, int64_t H, int64_t W);
int rvc_wino64_weights(const double* w, double* v, int64_t Ci, int64_t Co, rvc_stream_t stream);
int64_t rvc_wino64_workspace_bytes(const rvc_wino64_args* a);
int rvc_wino64_conv(const rvc_wino64_args* a, void* ws, int64_t ws_bytes, rvc_stream_t stream);
/* stft_mag64: rvc_stft_mag with the f64 magnitudes unrounded */
int rvc_stft_mag64(const float* x, const float* win, double* mag, int64_t B, int64_t N, int64_t F, int nfft, int hop,
                   int64_t x_bstride, int64_t mag_bstride, rvc_stream_t stream);
/* f64 forms of rvc_mel_image / avgpool2 / interleave4 / img_to_seq over B images (batch strides, 0 = dense
 * unused when B == 1); mel_image64 writes only the interior (the caller keeps the border zero). */
int rvc_mel_image64(const double* mel, double* img, int64_t B, int64_t M, int64_t F, int64_t Tp, double scale,
                    double shift, int64_t mel_bstride, int64_t img_bstride, rvc_stream_t stream);
int rvc_avgpool2_64(const double* in, double* out, int64_t B, int64_t C, int64_t H, int64_t W, int64_t in_bstride,
                    int64_t out_bstride, rvc_stream_t stream);
int rvc_interleave4_64(const double* phases, double* out, int64_t B, int64_t C, int64_t H, int64_t W,
                       int64_t ph_bstride, int64_t out_bstride, rvc_stream_t stream);
int rvc_img_to_seq64(const double* img, double* x, int64_t B, int64_t C, int64_t H, int64_t W, int64_t img_bstride,
                     int64_t x_bstride, rvc_stream_t stream);
/* bigru64_batched: rvc_bigru_batched in f64 (gi [2][768][T], whh [2][768][256], bhh [2][768], y [512][T] per
 * sequence); gran_ws: RVC_BIGRU64_GRAN_BYTES * min(B, 16) scratch (zeroed by the call); err as rvc_bigru. */
#define RVC_BIGRU64_GRAN_BYTES 16384
/* The f64 BiGRU's recurrence arithmetic, per thread: 1 = W_hh h and the gates in f32 (the default: its decision noise
 * on the headline clip is 1.8e-9, three orders below the smallest exact margin; gi and y stay f64), 0 = all f64,
 * -1 = back to RVC_BIGRU64_F32 (default 1). */
int rvc_bigru64_set_f32(int on);
int rvc_bigru64_batched(const double* gi, int64_t gi_bs, const double* whh, const double* bhh, double* y,
                        int64_t y_bs, void* gran_ws, int* err, int64_t B, int64_t T, rvc_stream_t stream);
/* Optional steps of VC.get_f0 between the raw f0 and the mel quantiser (convert.py:311-318), in
 * the reference's order: autotune (Autotune.autotune_f0, convert.py:168-179: f += (nearest of the 54
 * reference notes - f) * strength, first note on ties, unvoiced frames included) on the raw f0, then
 * the pitch shift, then the f0-file override f0[rep_off + i] = rep[i] for i < rep_len (convert.py:314-318,
 * rep = the host's np.interp of the file, f64).  NULL = none of them.  Arithmetic is f64 on the RMVPE
 * path (its f0 is f64) and f32 on the CREPE path (its f0 is f32), as in NumPy 2. */
typedef struct rvc_f0_post {
    int autotune, _pad0;
    double strength;
    const double* rep; /* device f64 [rep_len] or NULL */
    int64_t rep_off, rep_len;
} rvc_f0_post;

int rvc_rmvpe_decode(const float* sal, int64_t ld, int64_t F, double thred, double shift, const rvc_f0_post* post,
                     double* f0, int64_t* coarse, float* pitchf, rvc_stream_t stream);

/* pm f0 (VC.get_f0_pm, convert.py:206-213): Praat's To Pitch (ac) with get_f0_pm's settings on the f64
 * 16 kHz signal x [n] -> f0 [rvc_pm_frames(n)] (0 = unvoiced); window [958] = Praat's Hann window
 * 0.5 - 0.5 cos(2 pi i / 959), i = 1..958, window_r [480] its normalised autocorrelation; work:
 * rvc_pm_work_bytes(n) bytes.  rvc_pm_post: get_f0_pm's zero padding to p_len (when p_len > nf), then
 * get_f0's autotune / shift / f0 file (post, as rvc_rmvpe_decode) and mel quantiser -> coarse, pitchf
 * [max(p_len, nf)].  Restated from Boersma (1993) / Praat: parity unpinned (no parselmouth here). */
int64_t rvc_pm_frames(int64_t n);
int64_t rvc_pm_work_bytes(int64_t n);
int rvc_pm_f0(const double* x, int64_t n, const double* window, const double* window_r, void* work,
              int64_t work_bytes, double* f0, rvc_stream_t stream);
/* rvc_pm_windows: the window [958] and window_r [480] rvc_pm_f0 takes, computed on the HOST (host pointers). */
int rvc_pm_windows(double* window, double* window_r);
int rvc_pm_post(const double* f0, int64_t nf, int64_t p_len, double shift, const rvc_f0_post* post,
                int64_t* coarse, float* pitchf, rvc_stream_t stream);

/* ------------------------------------------------------------------ VC.pipeline glue
 * phone_upsample: nearest x2 + protect blend (convert.py:361-378) -> phone [C][T]
 * peak_normalize: x /= max|x|/0.99 when > 1 (convert.py:450-451); ws: 16 B scratch;
 *                 scale_out (optional device float) receives max|x|/0.99
 */
/* filtfilt_pad: scipy.signal.filtfilt(b, a, x) (padtype odd, padlen 18; convert.py:403) in f64, then
 *   reflect padding by tpad (convert.py:416): x f32 [N] -> out f32 [N + 2*tpad] (+ optional f64 copy).
 *   b[6], a[6], zi[5] (= lfilter_zi(b, a)) are HOST arrays; work: device scratch of
 *   rvc_filtfilt_work_bytes(N) bytes (8-byte aligned). */
int64_t rvc_filtfilt_work_bytes(int64_t N);
int rvc_filtfilt_pad(const float* x, int64_t N, const double* b, const double* a, const double* zi, int64_t tpad,
                     double* work, float* out, double* out64, rvc_stream_t stream);
int rvc_phone_upsample(const float* feats, const float* feats0, const float* pitchf, float* out, int64_t C, int64_t Tf,
                       int64_t T, float protect, rvc_stream_t stream);
int rvc_peak_normalize(float* x, int64_t n, void* ws, float* scale_out, rvc_stream_t stream);
/* quiet_points: VC.pipeline's segmentation of inputs over x_max (convert.py:404-412) on the filtered f64 signal
 *   x [n] (before the t_pad reflect padding): for n + window > t_max, one quiet point per t in
 *   range(t_center, n, t_center): t - t_query + the first argmin of |moving window-sum| over [t - t_query,
 *   t + t_query) (the reference's f64 sums, in its order) -> opt_ts int64 [count] (device).  count =
 *   rvc_quiet_points_count(...) (0 for short inputs); ws: rvc_quiet_points_ws_bytes(...) bytes. */
int64_t rvc_quiet_points_count(int64_t n, int window, int64_t t_center, int64_t t_max);
int64_t rvc_quiet_points_ws_bytes(int64_t n, int window, int64_t t_center, int64_t t_query, int64_t t_max);
int rvc_quiet_points(const double* x, int64_t n, int window, int64_t t_center, int64_t t_query, int64_t t_max,
                     void* ws, int64_t ws_bytes, int64_t* opt_ts, rvc_stream_t stream);
/* change_rms (convert.py:150-152, VC.pipeline volume_envelope != 1, convert.py:449):
 *   rms_frames: librosa.feature.rms(y, frame_length = 2*hop, hop_length = hop) (center, zero pad)
 *     of y [n] (f64 when y64 != NULL, else f32 y32) -> out f32 [1 + n / hop] (mean square in f64).
 *   rms_mix: y[i] *= r1(i)^(1 - rate) * max(r2(i), 1e-6)^(rate - 1), r(i) = F.interpolate(r, n,
 *     "linear", align_corners=False) of the source (r1 [n1]) and output (r2 [n2]) envelopes, f32. */
int64_t rvc_rms_frames_len(int64_t n, int64_t hop);
int rvc_rms_frames(const double* y64, const float* y32, int64_t n, int64_t hop, float* out, rvc_stream_t stream);
int rvc_rms_mix(float* y, int64_t n, const float* r1, int64_t n1, const float* r2, int64_t n2, double rate,
                rvc_stream_t stream);

/* ------------------------------------------------------------------ spectral-gate denoise
 * Replaces main/tools/noisereduce.py:reduce_noise(y, sr, prop_decrease=clean_strength) as
 * VoiceConverter.convert_audio calls it for clean_audio (convert.py:514-516): the non-stationary TG
 * (noisereduce.py:124-180) over SpectralGate.get_traces' chunks (:96-122: chunk_size samples, each
 * zero-padded by `padding` both sides and gated independently), in f64 like the reference.
 *   window: device f64 [n_fft] = torch.hann_window(n_fft) (float32, promoted);
 *   filt:   device f64 [filt_h][filt_w] (TG._generate_mask_smoothing_filter, :144-154) or NULL
 *           with filt_h = filt_w = 0;
 *   n_movemean = int(time_constant_s / hop * sr) (:193); n_thresh = thresh_n_mult_nonstationary;
 *   temp_coeff = 1 / sigmoid_slope_nonstationary.
 * y f32 [n] -> out f32 [n]; work: rvc_denoise_work_bytes(n, a) bytes of device scratch. */
typedef struct rvc_denoise_args {
    int64_t chunk_size, padding;
    int n_fft, hop, n_movemean, filt_h, filt_w, _pad0;
    double prop_decrease, n_thresh, temp_coeff;
    const double* window;
    const double* filt;
} rvc_denoise_args;

int64_t rvc_denoise_work_bytes(int64_t n, const rvc_denoise_args* a);
int rvc_denoise(const float* y, int64_t n, const rvc_denoise_args* a, void* work, int64_t work_bytes, float* out,
                rvc_stream_t stream);

/* ------------------------------------------------------------------ FAISS IVF-Flat retrieval
 * Replaces faiss IndexIVFFlat(L2).search(feats, k=8) + the blend of convert.py:349-359.
 * Queries (query i, dim c) live at q[c*cs + i*qs] (channels-first [d][nq]: cs = nq, qs = 1).
 * centT: centroids transposed [d][nlist]; inverted lists in CSR form: list_off [nlist+1],
 * codes [ntotal][d] (list-major), ids [ntotal].  Results are D f32 [nq][k] (squared L2), I int64 [nq][k],
 * ascending by (distance, id), missing results (FLT_MAX, -1) as in faiss.
 * Arithmetic (rvc_ivf_search = RVC_IVF_FAISS): faiss's own f32 evaluation -- coarse ||x||^2 + ||c||^2 - 2<x,c>
 * clamped at 0 for nq >= 20 (knn_L2sqr's BLAS path), fvec_L2sqr below 20 and in the list scan, each f32 sum in
 * the structure of faiss's AVX2 kernels (d % 8 == 0); RVC_IVF_EXACT: f64 distances (a diagnostic).
 * ws: rvc_ivf_coarse_ws_bytes(nq, nlist) bytes; probes: int64 [nq][nprobe] scratch/out. */
enum { RVC_IVF_FAISS = 0, RVC_IVF_EXACT = 1 };
int64_t rvc_ivf_coarse_ws_bytes(int64_t nq, int64_t nlist);
int rvc_ivf_search(const float* q, int64_t nq, int64_t d, int64_t cs, int64_t qs, const float* centT, int64_t nlist,
                   int nprobe, const int64_t* list_off, const float* codes, const int64_t* ids, int k, void* ws,
                   int64_t ws_bytes, int64_t* probes, float* D, int64_t* I, rvc_stream_t stream);
int rvc_ivf_search_ex(const float* q, int64_t nq, int64_t d, int64_t cs, int64_t qs, const float* centT,
                      int64_t nlist, int nprobe, const int64_t* list_off, const float* codes, const int64_t* ids,
                      int k, void* ws, int64_t ws_bytes, int64_t* probes, float* D, int64_t* I, int arithmetic,
                      rvc_stream_t stream);
/* out = (sum_j big[I_j] * w_j / sum w) * index_rate + (1 - index_rate) * feats, w = (1/D)^2, in the
 * f32 operation order of the reference's numpy/torch code; big = reconstruct_n(0, ntotal) [ntotal][d]. */
int rvc_ivf_blend(const float* feats, int64_t nq, int64_t d, int64_t fcs, int64_t fqs, const float* D, const int64_t* I,
                  int k, const float* big, int64_t ntotal, double index_rate, float* out, int64_t ocs, int64_t oqs,
                  rvc_stream_t stream);

/* ------------------------------------------------------------------ CREPE f0 (VC.get_f0_crepe, convert.py:230-237)
 * crepe_frames: CREPE.py:151-171 framing (1024 @ hop, 512 zero pad) + per-frame zero-mean / unbiased-std
 *   normalisation of frames [frame0, frame0 + nframes) -> out [nframes][1024].
 * bn_maxpool: BatchNorm(eval, alpha/beta precomputed) + MaxPool(2) of y [B][C][L] into strided out.
 * crepe_decode: probs [360][T] sigmoid outputs (masked in place to -inf outside [lo, hi)), softmax,
 *   librosa Viterbi per sequence [seq_off[i], seq_off[i+1]) with log_trans[j][k] = log(A[k][j] + tiny),
 *   bins -> Hz with dither cents [T], periodicity -> f0_raw [T], pd_raw [T].
 * crepe_smooth_coarse: mean3(f0), median3(pd), f0[pd < 0.1] = 0, then get_f0's shift + coarse mel bins. */
int rvc_crepe_frames(const float* audio, int64_t n, int hop, int64_t frame0, int64_t nframes, float* out,
                     rvc_stream_t stream);
int rvc_bn_maxpool(const float* y, int64_t B, int64_t C, int64_t L, const float* alpha, const float* beta, float* out,
                   int64_t obs, int64_t ocs, int64_t ois, rvc_stream_t stream);
int64_t rvc_crepe_decode_ws_bytes(int64_t T);
int rvc_crepe_decode(float* probs, int64_t T, int lo, int hi, const int64_t* seq_off, int nseq, const double* log_trans,
                     double log_off, double log_p_init, const float* dither, void* ws, int64_t ws_bytes, float* f0_raw,
                     float* pd_raw, rvc_stream_t stream);
int rvc_crepe_smooth_coarse(const float* f0_raw, const float* pd_raw, int64_t T, float shift, double mel_min,
                            double mel_max, const rvc_f0_post* post, int64_t* coarse, float* pitchf,
                            rvc_stream_t stream);

/* ------------------------------------------------------------------ model-level API
 * A context per device that owns the weights of a voice model and its scratch, so that a non-Python
 * host can run Synthesizer.infer (synthesizers.py:446-465) through this header alone: the folding and
 * packing the Python loader does (rvc_amd/synth.py) and the launch sequence of its infer are native
 * (csrc/rvc_model.cpp), with the same kernels, pass sets and order -- bit-identical to the Python path
 * on the same fp32 weights.
 *   rvc_ctx_create / destroy   one context per HIP device (not re-entrant; calls are stream-ordered).
 *   rvc_ctx_set_precision      the conv engine's arithmetic: RVC_PREC_FP32 (default: 6-pass split-bf16
 *                              mixed with split-fp16 where measured faster), _FP32X6, _FP32SA, _F16X3,
 *                              _BF16X3, _BF16.  RMVPE has its own setting (below).
 *   rvc_ctx_set_rmvpe_precision RMVPE's arithmetic, read by the next rvc_load_rmvpe: RVC_PREC_FP64 (default: the
 *                              network in f64, rmvpe64.hip -- the f0 decisions of the exact model -- with ONE
 *                              exception: the BiGRU recurrence runs in f32 behind the f64 interface (f64 inputs, f64
 *                              output; its decision noise 1.8e-9, profiles/r5_rmvpe_stage_prec.json); all-f64 is
 *                              rvc_bigru64_set_f32(0) or RVC_BIGRU64_F32=0), or a conv precision above for the
 *                              f32 form (_FP32SA: round 3's split-accumulator convs).
 *   rvc_load_synth             params = the .pth "weight" dict (train.py:729-742) as named HOST arrays,
 *                              f32 or f16; weight-norm pairs (x.weight_g / x.weight_v) are folded at load
 *                              (torch._weight_norm, dim 0), already-folded x.weight is taken as is.
 *                              cfg = the .pth "config" list.  Synchronous; replaces a loaded model.
 *   rvc_synth_infer            phone f32 [B][T][E], pitch int64 [B][T], pitchf f32 [B][T] (device);
 *                              sid: HOST int64 [B]; z_noise [B][inter][T] / sine_noise [B][T*upp] device
 *                              or NULL (NULL = device Philox draws from seed + b, as the Python path);
 *                              wav f32 [B][rvc_synth_out_len(ctx, T)] device.  Scratch grows on demand
 *                              (a stream sync when it does); nothing else synchronises. */
typedef struct rvc_ctx rvc_ctx;

enum { RVC_DT_F32 = 0, RVC_DT_F16 = 1, RVC_DT_F64 = 2 };
enum { RVC_PREC_FP32 = 0, RVC_PREC_BF16 = 1, RVC_PREC_BF16X3 = 3, RVC_PREC_FP32X6 = 6, RVC_PREC_FP32SA = 7,
       RVC_PREC_F16X3 = 16, RVC_PREC_FP64 = 64 };

typedef struct rvc_param {
    const char* name;  /* state-dict key, e.g. "dec.ups.0.weight_v" */
    const void* data;  /* host, dense row-major                     */
    int dtype;         /* RVC_DT_F32 / RVC_DT_F16 (RVC_DT_F64: constants) */
    int ndim;
    int64_t shape[4];
} rvc_param;

typedef struct rvc_synth_cfg { /* the checkpoint's "config" list (train.py:729-742) */
    int inter_channels, hidden_channels, filter_channels, n_heads, n_layers, kernel_size;
    int n_resblocks, n_dilations;          /* len(resblock_kernel_sizes), len(resblock_dilation_sizes[0]) */
    int resblock_kernel_sizes[4];
    int resblock_dilation_sizes[4][4];
    int n_upsamples;
    int upsample_rates[8];
    int upsample_kernel_sizes[8];
    int upsample_initial_channel;
    int spk_embed_dim, gin_channels, sr;
} rvc_synth_cfg;

int rvc_ctx_create(int hip_device, rvc_ctx** out);
void rvc_ctx_destroy(rvc_ctx* ctx);
int rvc_ctx_set_precision(rvc_ctx* ctx, int prec);
int rvc_ctx_set_rmvpe_precision(rvc_ctx* ctx, int prec);
int rvc_load_synth(rvc_ctx* ctx, const rvc_param* params, int n, const rvc_synth_cfg* cfg);
int64_t rvc_synth_out_len(const rvc_ctx* ctx, int64_t T);
int rvc_synth_infer(rvc_ctx* ctx, const float* phone, const int64_t* pitch, const float* pitchf, int64_t B, int64_t T,
                    const int64_t* sid, const float* z_noise, const float* sine_noise, uint64_t seed, float* wav,
                    rvc_stream_t stream);

/* ContentVec / HuBERT-base (HubertModel.extract_features, fairseq.py:1459 -> :1412-1431; extractor "default",
 * post-LN).  params = the fairseq .pt "model" dict (floating entries); encoder.pos_conv's weight-norm pair
 * (dim 2) is folded at load.  cfg = the .pt "cfg"/"model" fields below.
 *   rvc_contentvec_forward: wav f32 [B][N] (16 kHz, device) -> feats f32 [B][T][C] time-major like
 *   extract_features' x (T = rvc_contentvec_frames(N)), after out_layer encoder layers (12 for v2, 9 for v1,
 *   convert.py:338); final_proj != 0 applies model.final_proj (convert.py:340) and C = its width. */
typedef struct rvc_contentvec_cfg {
    int encoder_embed_dim, encoder_attention_heads, conv_pos_groups, _pad0;
} rvc_contentvec_cfg;

int rvc_load_contentvec(rvc_ctx* ctx, const rvc_param* params, int n, const rvc_contentvec_cfg* cfg);
int64_t rvc_contentvec_frames(int64_t n16k);
int rvc_contentvec_forward(rvc_ctx* ctx, const float* wav, int64_t B, int64_t N, int out_layer, int final_proj,
                           float* feats, rvc_stream_t stream);

/* RMVPE (E2E(4, 1, (2, 2)), RMVPE.py:183-226 as VC.get_f0_rmvpe uses it, convert.py:248-255).
 * params = the rmvpe.pt state dict; BatchNorm folded at load.  Optional extra params: "mel_basis" f32 [128][513]
 * (librosa.filters.mel(16000, 1024, 128, 30, 8000, htk=True); default: restated natively, rvc_amd/melbasis.py)
 * and "window" f32 [1024] (torch.hann_window(1024); default: computed natively).
 *   rvc_rmvpe_forward: wav f32 [B][N] (device) -> salience f32 [B][360][Tp], Tp = rvc_rmvpe_salience_ld(N)
 *   (frames rounded up to 32); mel -> U-Net -> BiGRU -> Linear + sigmoid.  The first rvc_rmvpe_frames(N)
 *   columns decode with rvc_rmvpe_decode (ld = Tp) into f0 / coarse / pitchf.  Always f32-accurate arithmetic
 *   (the f0 is a per-frame decision, as rvc_amd/rmvpe.py).
 *   rvc_rmvpe_check: synchronises; returns RVC_EHIP (and clears the flag) if a BiGRU hand-off timed out since
 *   the last check (that salience is invalid), else RVC_OK. */
int rvc_load_rmvpe(rvc_ctx* ctx, const rvc_param* params, int n);
int64_t rvc_rmvpe_frames(int64_t n16k);
int64_t rvc_rmvpe_salience_ld(int64_t n16k);
int rvc_rmvpe_forward(rvc_ctx* ctx, const float* wav, int64_t B, int64_t N, float* salience, rvc_stream_t stream);
int rvc_rmvpe_check(rvc_ctx* ctx);

/* CREPE f0 (VC.get_f0_crepe, convert.py:230-237; CREPE.py, any capacity -- taken from the conv shapes).
 * params = the CREPE state dict (conv{1..6}, conv{1..6}_BN, classifier); BatchNorm (eps 1e-3) folded at load
 * in f32 as rvc_amd/crepe.py (or taken from optional "conv{i}_BN.alpha" / ".beta" f32 [C]); optional "log_trans"
 * f64 [360][360] (default: the 12-bin triangular transition matrix's log, computed natively).
 *   rvc_crepe_f0: the padded 16 kHz audio f32 [N] (device) -> coarse int64 [T], pitchf f32 [T],
 *   T = rvc_rmvpe_frames(N): 1024-sample frames at hop 160, the network in 512-frame batches, the librosa
 *   Viterbi per batch with the dither (device f32 cents [T], or NULL = the triangular law drawn on the device
 *   from seed), periodicity smoothing, then get_f0's pitch shift (semitones), `post` and the mel quantiser.
 *   probs (optional, device f32 [360][T]) receives the sigmoid outputs. */
int rvc_load_crepe(rvc_ctx* ctx, const rvc_param* params, int n);

/* VC.pipeline (convert.py:388-458) with inputs and output in device memory: filtfilt + reflect padding by
 * x_pad s; for inputs over x_max s the quiet-point segmentation (convert.py:404-412, rvc_quiet_points -- the
 * one device->host read-back: the segment plan needs the points); f0 over the whole padded input on a side
 * stream (RMVPE thred 0.03, CREPE or pm; pitch shift, then the optional autotune and f0-file override of
 * get_f0, convert.py:304-323); per segment ContentVec (v2: layer 12; v1: layer 9 + final_proj), the optional
 * FAISS retrieval (index_rate, rvc_load_index), phone upsample + protect, Synthesizer.infer with device noise
 * at seed + segment, the x_pad trim at tgt_sr; the optional volume envelope (change_rms, convert.py:449) and
 * the peak normalisation.  Needs ContentVec, the synthesizer and the chosen f0 model loaded on the context;
 * audio f32 [N] 16 kHz (device) -> out f32 (device).  Equal to rvc_amd.pipeline.VC.pipeline_device on the
 * same models, options and seed (tests/test_gpu_native.py).
 *   rvc_vc_out_len: the output length for inputs of one segment (N + 160 <= x_max s); for longer inputs an
 *   upper bound (the quiet points decide the exact length).  rvc_vc_convert_ex writes the exact length to
 *   *out_len; rvc_vc_convert = rvc_vc_convert_ex with default options and one-segment inputs only. */
typedef struct rvc_vc_args {
    int64_t sid;
    double pitch_shift; /* semitones */
    float protect;
    int version;        /* 1 or 2 */
    int x_pad, x_max;   /* Config: 1 and 41 at full precision */
    int tgt_sr, _pad0;
    double index_rate;  /* != 0: FAISS IVF-Flat retrieval + blend (convert.py:349-359), index from rvc_load_index */
    uint64_t seed;
} rvc_vc_args;

/* The retrieval index rvc_vc_convert blends with (a faiss IndexIVFFlat(L2) as create_index.py writes it; read
 * without faiss by rvc_amd.faiss_index): HOST arrays, copied to the device.  centroids [nlist][d]; inverted lists
 * in CSR form: list_off [nlist + 1], codes [ntotal][d] (list-major), ids [ntotal]; big = reconstruct_n(0, ntotal)
 * [ntotal][d]; nprobe as the index stores it.  Validated on the host (d a multiple of 8 up to 1024, ntotal > 0,
 * list_off non-decreasing from 0 to ntotal, every id in [0, ntotal)): a malformed index is a load error.
 * Loading again replaces the index and frees the previous one's device arrays (after a device sync). */
typedef struct rvc_ivf_index {
    int64_t d, nlist, ntotal;
    int nprobe, _pad0;
    const float* centroids;
    const int64_t* list_off;
    const float* codes;
    const int64_t* ids;
    const float* big;
} rvc_ivf_index;

int rvc_load_index(rvc_ctx* ctx, const rvc_ivf_index* index);
/* device memory in use on the current device (hipMemGetInfo total - free), for load / reload accounting */
int64_t rvc_device_bytes_in_use(void);

enum { RVC_F0_RMVPE = 0, RVC_F0_CREPE = 1, RVC_F0_PM = 2 };
typedef struct rvc_vc_opts {
    int f0_method;               /* RVC_F0_RMVPE (default), RVC_F0_CREPE (the model of rvc_load_crepe), RVC_F0_PM */
    int f0_autotune;             /* != 0: Autotune.autotune_f0 at f0_autotune_strength (convert.py:311-313) */
    double f0_autotune_strength;
    const float* f0_file;        /* HOST f32 [f0_file_rows][2] "time, f0" rows (read_f0_file, convert.py:425-436) */
    int64_t f0_file_rows;        /*   0 = none; resampled to 100 frames/s as np.interp (convert.py:316-318) */
    double volume_envelope;      /* != 1: change_rms of the output against the filtered input (convert.py:449) */
    const float* crepe_dither;   /* CREPE: device f32 [1 + (N + 2 x_pad 16000) / 160] cents, or NULL = drawn on the
                                    device from seed (the triangular law of CREPE.py:119) */
} rvc_vc_opts;

int64_t rvc_vc_out_len(const rvc_ctx* ctx, int64_t N, const rvc_vc_args* args);
/* the f0-file override values rvc_vc_convert_ex writes from opts.f0_file (host; convert.py:316-318's np.interp of
 * the rows at 100 frames/s): returns their count n and writes min(n, cap) of them to out (HOST f64); -1 on bad
 * input.  Exposed for the parity test against the reference's numpy. */
int64_t rvc_f0_file_resample(const float* rows, int64_t nrows, double* out, int64_t cap);
int rvc_vc_convert(rvc_ctx* ctx, const float* audio, int64_t N, const rvc_vc_args* args, float* out,
                   rvc_stream_t stream);
int rvc_vc_convert_ex(rvc_ctx* ctx, const float* audio, int64_t N, const rvc_vc_args* args, const rvc_vc_opts* opts,
                      float* out, int64_t out_cap, int64_t* out_len, rvc_stream_t stream);
int rvc_crepe_f0(rvc_ctx* ctx, const float* audio, int64_t N, const float* dither, uint64_t seed, double pitch_shift,
                 const rvc_f0_post* post, float* probs, int64_t* coarse, float* pitchf, rvc_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RVC_AMD_H */
