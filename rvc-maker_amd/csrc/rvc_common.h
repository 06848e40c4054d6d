// Shared device helpers for the RVC MI355X kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/rvc_amd.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define RVC_DEV __device__ __forceinline__

// MFMA f32 16x16x4 (exact f32 fma chain).  Lane l holds A[l&15][l>>4], B[l>>4][l&15];
// C/D: col = l&15, row = (l>>4)*4 + r.
RVC_DEV floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

RVC_DEV float act_apply(float v, int act, float slope) {
    switch (act) {
        case RVC_ACT_LRELU: return v >= 0.f ? v : v * slope;
        case RVC_ACT_RELU: return v > 0.f ? v : 0.f;
        case RVC_ACT_TANH: return tanhf(v);
        case RVC_ACT_GELU: return 0.5f * v * (1.f + erff(v * 0.70710678118654752440f));
        case RVC_ACT_SIGMOID: return 1.f / (1.f + expf(-v));
        case RVC_ACT_LOGCLAMP: return logf(fmaxf(v, slope));
        default: return v;
    }
}

RVC_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

RVC_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// amax_out: the wave's largest |stored value| folded into the tensor's cell (atomic max of the f32 bits: for values
// >= 0 the bit patterns order as the floats do).  A cell is RVC_AMAX_SHARDS words and each wave adds to one of them
// (by block and wave): thousands of waves on ONE address serialise at the memory side (round 5: the generator ran
// 904 -> 882 xRT with one word per tensor).  Called by every lane of a wave (the shuffles need them all).
RVC_DEV void amax_publish(unsigned* amax_out, float m) {
    m = wave_max(m);
    const unsigned shard = (blockIdx.x + 7u * blockIdx.y + 13u * blockIdx.z + (threadIdx.x >> 6)) % RVC_AMAX_SHARDS;
    if ((threadIdx.x & 63) == 0) atomicMax(amax_out + shard, __float_as_uint(m));
}

// The same from a whole block, for short, wide launches whose waves would all publish at once (the split-K reduce, the
// source pass, LayerNorms, the embedding): the block's largest value through LDS and ONE atomic per block.  Every
// thread of the (1-D, <= 1024-thread) block calls it, uniformly, as its last act.  Round 6: the split-K reduce of the
// TextEncoder's 576 x 3000 QKV projection took 144 us with a wave per 64 columns publishing (30k atomics on one cell,
// kernel trace r6d) against 9 us for the same reduce without a cell.
RVC_DEV void amax_publish_block(unsigned* amax_out, float m) {
    __shared__ float wmax_[16];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) wmax_[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float bm = 0.f;
        for (int w = 0; w < (int)((blockDim.x + 63) >> 6); ++w) bm = fmaxf(bm, wmax_[w]);
        const unsigned shard = (blockIdx.x + 7u * blockIdx.y + 13u * blockIdx.z) % RVC_AMAX_SHARDS;
        atomicMax(amax_out + shard, __float_as_uint(bm));
    }
}

// the |max| of a cell: the largest of its shards, read through the scalar cache (wave-uniform address, s_load: it does
// not queue behind the wave's vector loads in vmcnt order, and no shuffle)
typedef const __attribute__((address_space(4))) unsigned* amax_const_ptr;  // constant space: s_load
RVC_DEV float amax_read(const unsigned* cell) {
    const amax_const_ptr c = (amax_const_ptr)cell;  // read-only for the whole launch
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < RVC_AMAX_SHARDS; ++i) m = max(m, c[i]);
    return __uint_as_float(m);
}

// thread-local error reporting for the C ABI
void rvc_set_error(const char* fmt, ...);

#define RVC_CHECK_ARG(cond, ...)            \
    do {                                    \
        if (!(cond)) {                      \
            rvc_set_error(__VA_ARGS__);     \
            return RVC_EINVAL;              \
        }                                   \
    } while (0)

#define RVC_HIP(call)                                                        \
    do {                                                                     \
        hipError_t e_ = (call);                                              \
        if (e_ != hipSuccess) {                                              \
            rvc_set_error("%s: %s", #call, hipGetErrorString(e_));          \
            return RVC_EHIP;                                                 \
        }                                                                    \
    } while (0)

static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

// VC.get_f0's optional f0 steps (convert.py:311-318), shared by the RMVPE (f64) and CREPE (f32)
// decoders.  The 54 reference notes of VC.__init__ (convert.py:198).
static __device__ __constant__ double kRefNotes[54] = {
    49.00,  51.91,  55.00,  58.27,  61.74,  65.41,  69.30,  73.42,  77.78,  82.41,  87.31,  92.50,  98.00,  103.83,
    110.00, 116.54, 123.47, 130.81, 138.59, 146.83, 155.56, 164.81, 174.61, 185.00, 196.00, 207.65, 220.00, 233.08,
    246.94, 261.63, 277.18, 293.66, 311.13, 329.63, 349.23, 369.99, 392.00, 415.30, 440.00, 466.16, 493.88, 523.25,
    554.37, 587.33, 622.25, 659.25, 698.46, 739.99, 783.99, 830.61, 880.00, 932.33, 987.77, 1046.50};

// Autotune.autotune_f0 (convert.py:172-179): min(notes, key=|x - f|) keeps the first note on ties;
// F is the f0 array's dtype (NumPy 2: python-float note/strength operands take the array's dtype).
template <typename F>
RVC_DEV F autotune_note(F f, double strength) {
#pragma clang fp contract(off)
    F best = (F)kRefNotes[0];
    F bd = (F)fabs((double)((F)kRefNotes[0] - f));
    for (int i = 1; i < 54; ++i) {
        F d = (F)kRefNotes[i] - f;
        d = d < (F)0 ? -d : d;
        if (d < bd) {
            bd = d;
            best = (F)kRefNotes[i];
        }
    }
    return f + (best - f) * (F)strength;
}

// autotune -> * shift -> f0-file override, on frame t (kernels take the struct by value; the
// C entry points turn a NULL post into a zeroed one).
template <typename F>
RVC_DEV F f0_post_apply(F f, int64_t t, F shift, const rvc_f0_post& post) {
    if (post.autotune) f = autotune_note<F>(f, post.strength);
    f = f * shift;
    if (post.rep && t >= post.rep_off && t < post.rep_off + post.rep_len) f = (F)post.rep[t - post.rep_off];
    return f;
}

static inline rvc_f0_post f0_post_or_none(const rvc_f0_post* p) {
    rvc_f0_post z = {};
    return p ? *p : z;
}
