// Microbenchmark of the f64 BiGRU recurrence (rmvpe64.hip bigru64_kernel) and variants, to find where its
// per-step time goes.  One launch of 32 workgroups (2 directions x 16), T steps, timed with hip events.
//   hipcc --offload-arch=gfx950 -O3 scripts/bigru64_bench.hip -o /tmp/bigru64_bench && /tmp/bigru64_bench 3232
// Variants (template V):
//   0  the library kernel's structure (two 8-byte {tag, half} granules per unit)
//   1  0 with the gate transcendentals replaced by cheap f64 arithmetic (ablation: wrong results)
//   2  one 16-byte granule {tag, lo, tag, hi} per unit, one dwordx4 store / load
//   3  2 without the s_sleep in the poll loop
//   4  2 with the f32 kernel's 8-byte granule carrying an f32 value (the f32 kernel's exchange, f64 math)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));  \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int H = 256, WG = 16;

template <int V>
__device__ __forceinline__ double sig(double x) {
    if constexpr (V == 1) return 0.5 + 0.25 * x;
    return 1.0 / (1.0 + exp(-x));
}
template <int V>
__device__ __forceinline__ double th(double x) {
    if constexpr (V == 1) return x * (1.0 - 0.3 * x * x);
    return tanh(x);
}

template <int V>
__global__ __launch_bounds__(256) void bigru64(const double* gi, const double* whh, const double* bhh, double* y,
                                               unsigned long long* gran, int* err, int64_t T, unsigned spin_limit) {
    const int d = blockIdx.x / WG, j = blockIdx.x % WG, tid = threadIdx.x;
    const int ul = tid >> 4, s = tid & 15, u = j * 16 + ul;
    __shared__ double hs[2][H];
    __shared__ int abort_flag;
    if (tid == 0) abort_flag = 0;
    const double* W = whh + (int64_t)d * 3 * H * H;
    double wr[16], wz[16], wn[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        wr[i] = W[(int64_t)u * H + 16 * s + i];
        wz[i] = W[(int64_t)(H + u) * H + 16 * s + i];
        wn[i] = W[(int64_t)(2 * H + u) * H + 16 * s + i];
    }
    const double bhr = bhh[d * 3 * H + u], bhz = bhh[d * 3 * H + H + u], bhn = bhh[d * 3 * H + 2 * H + u];
    const double* G = gi + (int64_t)d * 3 * H * T;
    unsigned long long* GR = gran + (int64_t)d * 2 * H * 2;
    double hprev = 0.0, gxr = 0.0, gxz = 0.0, gxn = 0.0;
    if (s == 0) {
        const int64_t tau0 = d ? T - 1 : 0;
        gxr = G[(int64_t)u * T + tau0];
        gxz = G[(int64_t)(H + u) * T + tau0];
        gxn = G[(int64_t)(2 * H + u) * T + tau0];
    }
    hs[0][tid] = 0.0;
    __syncthreads();
    for (int64_t t = 0; t < T; ++t) {
        const int64_t tau = d ? T - 1 - t : t;
        const int cur = (int)(t & 1);
        if (t > 0) {
            unsigned long long* g = GR + ((t - 1) & 1) * H * 2 + 2 * tid;
            unsigned spins = 0;
            double hv = 0.0;
            if constexpr (V == 0 || V == 1) {
                unsigned long long v0 = 0, v1 = 0;
                bool ok0 = false, ok1 = false;
                for (;;) {
                    if (!ok0) {
                        v0 = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok0 = (uint32_t)(v0 >> 32) == (uint32_t)t;
                    }
                    if (!ok1) {
                        v1 = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok1 = (uint32_t)(v1 >> 32) == (uint32_t)t;
                    }
                    if (ok0 && ok1) break;
                    if (++spins > spin_limit) {
                        atomicExch(err, 1);
                        abort_flag = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                hv = __hiloint2double((int)(uint32_t)v1, (int)(uint32_t)v0);
            } else if constexpr (V == 4) {
                unsigned long long* g1 = GR + ((t - 1) & 1) * H * 2 + tid;
                unsigned long long v;
                for (;;) {
                    v = __hip_atomic_load(g1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((uint32_t)(v >> 32) == (uint32_t)t) break;
                    if (++spins > spin_limit) {
                        atomicExch(err, 1);
                        abort_flag = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                hv = (double)__uint_as_float((uint32_t)v);
            } else {
                // one 16-byte granule: {tag | lo} {tag | hi} read with one dwordx4 load (each 8-byte half carries
                // the step tag, so a read that mixes two steps is seen and retried)
                typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                u64x2 v;
                for (;;) {
                    // the agent-coherent load the 8-byte atomics compile to (sc1), 16 bytes wide
                    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(g) : "memory");
                    if ((uint32_t)(v.x >> 32) == (uint32_t)t && (uint32_t)(v.y >> 32) == (uint32_t)t) break;
                    if (++spins > spin_limit) {
                        atomicExch(err, 1);
                        abort_flag = 1;
                        break;
                    }
                    if constexpr (V != 3) __builtin_amdgcn_s_sleep(1);
                }
                hv = __hiloint2double((int)(uint32_t)v.y, (int)(uint32_t)v.x);
            }
            hs[cur][tid] = hv;
            __syncthreads();
            if (abort_flag) break;
        }
        double nxr = 0.0, nxz = 0.0, nxn = 0.0;
        if (s == 0 && t + 1 < T) {
            const int64_t tn = d ? T - 2 - t : t + 1;
            nxr = G[(int64_t)u * T + tn];
            nxz = G[(int64_t)(H + u) * T + tn];
            nxn = G[(int64_t)(2 * H + u) * T + tn];
        }
        double pr = 0.0, pz = 0.0, pn = 0.0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const double h = hs[cur][16 * s + i];
            pr += wr[i] * h;
            pz += wz[i] * h;
            pn += wn[i] * h;
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
            pr += __shfl_xor(pr, o, 64);
            pz += __shfl_xor(pz, o, 64);
            pn += __shfl_xor(pn, o, 64);
        }
        if (s == 0) {
            const double r = sig<V>(gxr + (pr + bhr));
            const double z = sig<V>(gxz + (pz + bhz));
            const double n = th<V>(gxn + r * (pn + bhn));
            const double h = (hprev - n) * z + n;
            hprev = h;
            const unsigned long long tag = (unsigned long long)(uint32_t)(t + 1) << 32;
            if constexpr (V == 0 || V == 1) {
                unsigned long long* o = GR + (t & 1) * H * 2 + 2 * u;
                __hip_atomic_store(o, tag | (uint32_t)__double2loint(h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(o + 1, tag | (uint32_t)__double2hiint(h), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            } else if constexpr (V == 4) {
                __hip_atomic_store(GR + (t & 1) * H * 2 + u, tag | __float_as_uint((float)h), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            } else {
                typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                unsigned long long* o = GR + (t & 1) * H * 2 + 2 * u;
                u64x2 v;
                v.x = tag | (uint32_t)__double2loint(h);
                v.y = tag | (uint32_t)__double2hiint(h);
                asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(o), "v"(v) : "memory");
            }
            y[(int64_t)(d * H + u) * T + tau] = h;
        }
        gxr = nxr;
        gxz = nxz;
        gxn = nxn;
    }
}

// f64 MFMA issue rate: every wave runs N x NA independent v_mfma_f64_16x16x4_f64
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NA>
__global__ __launch_bounds__(256) void mfma64_rate(double* out, int n) {
    d4 a[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) a[k] = d4{0, 0, 0, 0};
    double x = threadIdx.x * 1e-3, yv = 1.0 + blockIdx.x * 1e-6;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < NA; ++k) a[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(k & 1 ? x : yv, k & 2 ? yv : x, a[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) s += a[k][k & 3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
// v_mfma_f64_4x4x4f64 (16 independent 4x4 blocks per wave, one f64 accumulator per lane)
template <int NA>
__global__ __launch_bounds__(256) void mfma64_4x4_rate(double* out, int n) {
    double a[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) a[k] = 0;
    double x = threadIdx.x * 1e-3, yv = 1.0 + blockIdx.x * 1e-6;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < NA; ++k) a[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(k & 1 ? x : yv, k & 2 ? yv : x, a[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) s += a[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <typename Kern>
void rate(const char* name, Kern k, int nb, double flop_per_mfma, int na) {
    double* o2;
    const int n = 10000;
    CK(hipMalloc(&o2, (size_t)nb * 256 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, o2, 100);
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, o2, n);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double flop = (double)nb * 4 * n * na * flop_per_mfma;
    printf("%-40s %6.1f TFLOP/s\n", name, flop / ms / 1e9);
    CK(hipFree(o2));
}

template <int V>
double run(int64_t T, const double* gi, const double* whh, const double* bhh, double* y, unsigned long long* gran,
           int* err, std::vector<double>& out) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int it = 0; it < 4; ++it) {
        CK(hipMemset(gran, 0, 2 * 2 * H * 2 * 8));
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(bigru64<V>, dim3(2 * WG), dim3(256), 0, 0, gi, whh, bhh, y, gran, err, T, 1u << 22);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it && ms < best) best = ms;
    }
    out.resize(512 * T);
    CK(hipMemcpy(out.data(), y, 512 * T * 8, hipMemcpyDeviceToHost));
    return best;
}

int main(int argc, char** argv) {
    const int64_t T = argc > 1 ? atoll(argv[1]) : 3232;
    std::vector<double> hgi(1536 * T), hw(2 * 768 * 256), hb(1536);
    srand(1);
    for (auto& v : hgi) v = (rand() / (double)RAND_MAX - 0.5);
    for (auto& v : hw) v = (rand() / (double)RAND_MAX - 0.5) * 0.12;
    for (auto& v : hb) v = (rand() / (double)RAND_MAX - 0.5) * 0.2;
    double *gi, *whh, *bhh, *y;
    unsigned long long* gran;
    int* err;
    CK(hipMalloc(&gi, hgi.size() * 8));
    CK(hipMalloc(&whh, hw.size() * 8));
    CK(hipMalloc(&bhh, hb.size() * 8));
    CK(hipMalloc(&y, 512 * T * 8));
    CK(hipMalloc(&gran, 2 * 2 * H * 2 * 8));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    CK(hipMemcpy(gi, hgi.data(), hgi.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(whh, hw.data(), hw.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(bhh, hb.data(), hb.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> o0, o;
    const double t0 = run<0>(T, gi, whh, bhh, y, gran, err, o0);
    printf("V0 two granules         %8.3f ms  %.3f us/step\n", t0, t0 * 1e3 / T);
    const double t1 = run<1>(T, gi, whh, bhh, y, gran, err, o);
    printf("V1 no transcendentals   %8.3f ms  %.3f us/step\n", t1, t1 * 1e3 / T);
    const double t2 = run<2>(T, gi, whh, bhh, y, gran, err, o);
    double md = 0;
    for (size_t i = 0; i < o.size(); ++i) md = fmax(md, fabs(o[i] - o0[i]));
    printf("V2 one 16-B granule     %8.3f ms  %.3f us/step  (max |diff| vs V0 %.1e)\n", t2, t2 * 1e3 / T, md);
    const double t3 = run<3>(T, gi, whh, bhh, y, gran, err, o);
    printf("V3 V2 without s_sleep   %8.3f ms  %.3f us/step\n", t3, t3 * 1e3 / T);
    const double t4 = run<4>(T, gi, whh, bhh, y, gran, err, o);
    printf("V4 f32 exchange         %8.3f ms  %.3f us/step\n", t4, t4 * 1e3 / T);
    int e = 0;
    CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    rate("16x16x4 4 acc, 1 wave/SIMD", mfma64_rate<4>, 256, 2048.0, 4);
    rate("16x16x4 4 acc, 2 waves/SIMD", mfma64_rate<4>, 512, 2048.0, 4);
    rate("16x16x4 8 acc, 1 wave/SIMD", mfma64_rate<8>, 256, 2048.0, 8);
    rate("16x16x4 8 acc, 2 waves/SIMD", mfma64_rate<8>, 512, 2048.0, 8);
    rate("16x16x4 4 acc, 4 waves/SIMD", mfma64_rate<4>, 1024, 2048.0, 4);
    rate("4x4x4 (16 blocks) 8 acc, 2 waves/SIMD", mfma64_4x4_rate<8>, 512, 2048.0, 8);
    return 0;
}
