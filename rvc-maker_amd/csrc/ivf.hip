// FAISS IVF-Flat (L2) search + the reference's retrieval blend (convert.py:349-359, 392-399;
// index built by create_index.py:66-83 as IVF{n},Flat with nprobe 1, searched with k = 8).
//
// Arithmetic RVC_IVF_FAISS (the default) is faiss's own f32 evaluation as oracle/ivf.py restates it:
// the coarse step ||x||^2 + ||c||^2 - 2 <x, c> clamped at 0 for nq >= 20 (IndexFlatL2 -> knn_L2sqr's BLAS
// path), fvec_L2sqr(x, c) below that, fvec_L2sqr in the list scan; every f32 sum in the structure of
// faiss's AVX2 kernels (8 lane accumulators over consecutive 8-float chunks, multiply then add, then the
// ((m4+m0)+(m5+m1)) + ((m6+m2)+(m7+m3)) tree).  RVC_IVF_EXACT: f64 distances (diagnostic).
//
//   ivf_coarse_kernel   squared distances of every query to every centroid -> [nq][nlist] workspace
//   ivf_select_kernel   per query (one wave): the nprobe nearest lists, ties by list id (faiss keeps
//                       the first of equal distances in list order)
//   ivf_scan_kernel     per query (one wave): exhaustive L2 scan of the probed lists, top-k by
//                       (distance, id); missing results are (FLT_MAX, -1) as in faiss
//   ivf_blend_kernel    weight = (1/D)^2 normalised (numpy's 8-way pairwise row sum), then
//                       sum_j big[I_j] * w_j sequentially, times index_rate, plus (1 - rate) feats
//                       -- f32, contraction off, the operation order of the numpy/torch code
//
// Queries and features are addressed (query i, dim c) at base[c * cs + i * qs], so the
// channels-first [C][T] activations of the pipeline are read in place.
#include <float.h>

#include "rvc_common.h"

#pragma clang fp contract(off)

namespace {
constexpr int KMAX = 16;
constexpr int QB = 8;  // queries per coarse block

// the AVX2 horizontal reduction of 8 lane accumulators (extract-add, hadd, hadd)
__device__ __forceinline__ float hsum8(const float (&m)[8]) {
    return ((m[4] + m[0]) + (m[5] + m[1])) + ((m[6] + m[2]) + (m[7] + m[3]));
}

// faiss arithmetic: one thread per centroid, QB queries per block; lane a of the 8 accumulators takes the
// dims c = 8 j + a in order.  blas (nq >= 20): inner products + norms; else direct differences.
__device__ void coarse_faiss(const float* qsh, int d, const float* centT, int64_t nlist, int64_t l, bool blas,
                             const float* qn, float (&dis)[QB]) {
    float acc[QB][8], cn[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) {
        cn[a] = 0.f;
#pragma unroll
        for (int i = 0; i < QB; ++i) acc[i][a] = 0.f;
    }
    for (int c0 = 0; c0 < d; c0 += 8) {
#pragma unroll
        for (int a = 0; a < 8; ++a) {
            const float x = centT[(int64_t)(c0 + a) * nlist + l];
            if (blas) {
                cn[a] = cn[a] + x * x;
#pragma unroll
                for (int i = 0; i < QB; ++i) acc[i][a] = acc[i][a] + qsh[i * d + c0 + a] * x;
            } else {
#pragma unroll
                for (int i = 0; i < QB; ++i) {
                    const float t = qsh[i * d + c0 + a] - x;
                    acc[i][a] = acc[i][a] + t * t;
                }
            }
        }
    }
    const float cnorm = hsum8(cn);
#pragma unroll
    for (int i = 0; i < QB; ++i) {
        const float v = hsum8(acc[i]);
        if (blas) {
            const float t = (qn[i] + cnorm) - 2.0f * v;  // exhaustive_L2sqr_blas, then "if (dis < 0) dis = 0"
            dis[i] = t < 0.f ? 0.f : t;
        } else {
            dis[i] = v;
        }
    }
}

// grid (cdiv(nq, QB), cdiv(nlist, 256)); centT is [d][nlist] (transposed centroids, coalesced)
__global__ __launch_bounds__(256) void ivf_coarse_kernel(const float* q, int64_t nq, int d, int64_t cs, int64_t qs,
                                                         const float* centT, int64_t nlist, int arith, double* dist) {
    extern __shared__ float qsh[];  // [QB][d], then the QB query norms
    const int64_t q0 = (int64_t)blockIdx.x * QB;
    for (int i = threadIdx.x; i < QB * d; i += 256) {
        const int qi = i / d, c = i - qi * d;
        const int64_t qq = q0 + qi < nq ? q0 + qi : nq - 1;
        qsh[i] = q[c * cs + qq * qs];
    }
    __syncthreads();
    const bool blas = nq >= 20;  // faiss distance_compute_blas_threshold
    float* qn = qsh + QB * d;
    if (arith == RVC_IVF_FAISS && blas && threadIdx.x < QB) {  // fvec_norm_L2sqr per query
        float m[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) m[a] = 0.f;
        for (int c0 = 0; c0 < d; c0 += 8)
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                const float v = qsh[threadIdx.x * d + c0 + a];
                m[a] = m[a] + v * v;
            }
        qn[threadIdx.x] = hsum8(m);
    }
    __syncthreads();
    const int64_t l = (int64_t)blockIdx.y * 256 + threadIdx.x;
    if (l >= nlist) return;
    if (arith == RVC_IVF_FAISS) {
        float dis[QB];
        coarse_faiss(qsh, d, centT, nlist, l, blas, qn, dis);
#pragma unroll
        for (int i = 0; i < QB; ++i)
            if (q0 + i < nq) dist[(q0 + i) * nlist + l] = (double)dis[i];
        return;
    }
    double acc[QB];
#pragma unroll
    for (int i = 0; i < QB; ++i) acc[i] = 0.0;
    for (int c = 0; c < d; ++c) {
        const double x = (double)centT[(int64_t)c * nlist + l];
#pragma unroll
        for (int i = 0; i < QB; ++i) {
            const double t = (double)qsh[i * d + c] - x;
            acc[i] = fma(t, t, acc[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < QB; ++i)
        if (q0 + i < nq) dist[(q0 + i) * nlist + l] = acc[i];
}

// (d, id) lexicographic "a before b"
__device__ __forceinline__ bool before(double da, int64_t ia, double db, int64_t ib) {
    return da < db || (da == db && ia < ib);
}

// one wave per query: nprobe passes of a wave-wide argmin over the lists not yet taken
__global__ __launch_bounds__(64) void ivf_select_kernel(const double* dist, int64_t nq, int64_t nlist, int nprobe,
                                                        int64_t* probes) {
    const int64_t qi = blockIdx.x;
    const int lane = threadIdx.x;
    const double* row = dist + qi * nlist;
    double taken_d = -1.0;
    int64_t taken_i = -1;
    for (int p = 0; p < nprobe; ++p) {
        double bd = INFINITY;
        int64_t bi = INT64_MAX;
        for (int64_t l = lane; l < nlist; l += 64) {
            const double v = row[l];
            // strictly after the last taken (d, id) pair
            if (before(taken_d, taken_i, v, l) && before(v, l, bd, bi)) {
                bd = v;
                bi = l;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o, 64);
            const int64_t oi = __shfl_xor(bi, o, 64);
            if (before(od, oi, bd, bi)) {
                bd = od;
                bi = oi;
            }
        }
        if (lane == 0) probes[qi * nprobe + p] = bi < nlist ? bi : -1;
        taken_d = bd;
        taken_i = bi;
    }
}

// one wave per query, four list vectors per iteration (16 lanes each, lanes split the dimensions);
// every lane keeps the same top-k list.  Insertion by (distance, id) is order-independent.
// Arithmetic RVC_IVF_FAISS: eight list vectors per iteration, 8 lanes each -- lane a of a group is
// fvec_L2sqr's accumulator a (dims 8 j + a, in order), the group's butterfly (xor 4, 1, 2) is its
// horizontal tree (f32 addition commutes, so every lane holds the same value).
template <bool FAISS>
__global__ __launch_bounds__(64) void ivf_scan_kernel(const float* q, int64_t nq, int d, int64_t cs, int64_t qs,
                                                      const int64_t* probes, int nprobe, const int64_t* list_off,
                                                      const float* codes, const int64_t* ids, int k, float* D,
                                                      int64_t* I) {
    const int64_t qi = blockIdx.x;
    const int lane = threadIdx.x;
    constexpr int GL = FAISS ? 8 : 16;  // lanes per list vector
    constexpr int NG = 64 / GL;         // list vectors per iteration
    const int grp = lane / GL, r = lane % GL;
    constexpr int DPL = 1024 / GL;      // dims per lane (d <= 1024)
    float qv[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) {
        const int c = r + GL * j;
        qv[j] = c < d ? q[c * cs + qi * qs] : 0.f;
    }
    double td[KMAX];
    int64_t ti[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        td[j] = INFINITY;
        ti[j] = -1;
    }
    auto insert = [&](double dv, int64_t id) {
        if (!before(dv, id, td[k - 1], ti[k - 1])) return;
        double cd = dv;
        int64_t ci = id;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if (j < k && before(cd, ci, td[j], ti[j])) {
                const double sd = td[j];
                const int64_t si = ti[j];
                td[j] = cd;
                ti[j] = ci;
                cd = sd;
                ci = si;
            }
        }
    };
    for (int p = 0; p < nprobe; ++p) {
        const int64_t li = probes[qi * nprobe + p];
        if (li < 0) continue;
        const int64_t v0 = list_off[li], v1 = list_off[li + 1];
        for (int64_t v = v0; v < v1; v += NG) {
            const int64_t vv = v + grp < v1 ? v + grp : v1 - 1;
            const float* x = codes + vv * d;
            double part = 0.0;
            if constexpr (FAISS) {
                float acc = 0.f;
#pragma unroll
                for (int j = 0; j < DPL; ++j) {
                    const int c = r + GL * j;
                    if (c < d) {
                        const float t = qv[j] - x[c];
                        acc = acc + t * t;
                    }
                }
                acc = acc + __shfl_xor(acc, 4, 64);  // (m4 + m0) ...
                acc = acc + __shfl_xor(acc, 1, 64);  // (m4+m0) + (m5+m1), (m6+m2) + (m7+m3)
                acc = acc + __shfl_xor(acc, 2, 64);
                part = (double)acc;
            } else {
#pragma unroll
                for (int j = 0; j < DPL; ++j) {
                    const int c = r + GL * j;
                    if (c < d) {
                        const double t = (double)qv[j] - (double)x[c];
                        part = fma(t, t, part);
                    }
                }
#pragma unroll
                for (int o = 8; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
            }
            const int64_t myid = ids[vv];
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const double dv = __shfl(part, GL * g, 64);
                const int64_t id = __shfl(myid, GL * g, 64);
                if (v + g < v1) insert(dv, id);
            }
        }
    }
    if (lane < k) {
        double vd = 0.0;
        int64_t vi = -1;
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            if (j == lane) {
                vd = td[j];
                vi = ti[j];
            }
        D[qi * k + lane] = vi < 0 ? FLT_MAX : (float)vd;
        I[qi * k + lane] = vi;
    }
}

// numpy add.reduce over a contiguous row of n <= 8 f32 (pairwise: 8-way blocks, else sequential)
__device__ __forceinline__ float np_rowsum(const float* w, int n) {
    if (n < 8) {
        float s = 0.f;
        for (int j = 0; j < n; ++j) s += w[j];
        return s;
    }
    return ((w[0] + w[1]) + (w[2] + w[3])) + ((w[4] + w[5]) + (w[6] + w[7]));
}

// grid (cdiv(d, 256), nq): out[c][i] = (sum_j big[I_j][c] * wn_j) * rate + (1 - rate) * feats[c][i]
__global__ __launch_bounds__(256) void ivf_blend_kernel(const float* feats, int d, int64_t fcs, int64_t fqs,
                                                        const float* D, const int64_t* I, int k, const float* big,
                                                        int64_t ntotal, float rate, float rate1, float* out,
                                                        int64_t ocs, int64_t oqs) {
    const int64_t qi = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    float w[8];
    int64_t row[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j < k) {
            const float inv = 1.0f / D[qi * k + j];
            w[j] = inv * inv;
            const int64_t ix = I[qi * k + j];
            row[j] = ix < 0 ? ix + ntotal : ix;  // numpy negative indexing (-1 -> last row)
        } else {
            w[j] = 0.f;
            row[j] = 0;
        }
    }
    if (c >= d) return;
    const float s = np_rowsum(w, k);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j < k) {
            const float t = big[row[j] * d + c] * (w[j] / s);
            acc = j == 0 ? t : acc + t;
        }
    }
    out[c * ocs + qi * oqs] = acc * rate + rate1 * feats[c * fcs + qi * fqs];
}
}  // namespace

extern "C" int64_t rvc_ivf_coarse_ws_bytes(int64_t nq, int64_t nlist) {
    if (nq <= 0 || nlist <= 0) return -1;
    return nq * nlist * (int64_t)sizeof(double);
}

extern "C" int rvc_ivf_search_ex(const float* q, int64_t nq, int64_t d, int64_t cs, int64_t qs, const float* centT,
                                 int64_t nlist, int nprobe, const int64_t* list_off, const float* codes,
                                 const int64_t* ids, int k, void* ws, int64_t ws_bytes, int64_t* probes, float* D,
                                 int64_t* I, int arithmetic, rvc_stream_t stream) {
    RVC_CHECK_ARG(q && centT && list_off && codes && ids && ws && probes && D && I, "ivf_search: null pointer");
    RVC_CHECK_ARG(nq > 0 && d > 0 && d <= 1024 && nlist > 0 && nprobe >= 1 && nprobe <= nlist && k >= 1 &&
                      k <= KMAX, "ivf_search: bad sizes nq=%lld d=%lld nlist=%lld nprobe=%d k=%d", (long long)nq,
                  (long long)d, (long long)nlist, nprobe, k);
    RVC_CHECK_ARG(ws_bytes >= nq * nlist * (int64_t)sizeof(double), "ivf_search: workspace too small");
    RVC_CHECK_ARG((size_t)QB * (d + 1) * 4 <= 64 * 1024, "ivf_search: d too large");
    RVC_CHECK_ARG(arithmetic == RVC_IVF_FAISS || arithmetic == RVC_IVF_EXACT, "ivf_search: unknown arithmetic %d",
                  arithmetic);
    RVC_CHECK_ARG(arithmetic != RVC_IVF_FAISS || d % 8 == 0, "ivf_search: faiss arithmetic needs d %% 8 == 0");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(ivf_coarse_kernel, dim3(cdiv(nq, QB), cdiv(nlist, 256)), dim3(256), (size_t)QB * (d + 1) * 4, s,
                       q, nq, (int)d, cs, qs, centT, nlist, arithmetic, (double*)ws);
    hipLaunchKernelGGL(ivf_select_kernel, dim3((unsigned)nq), dim3(64), 0, s, (const double*)ws, nq, nlist, nprobe,
                       probes);
    if (arithmetic == RVC_IVF_FAISS)
        hipLaunchKernelGGL(ivf_scan_kernel<true>, dim3((unsigned)nq), dim3(64), 0, s, q, nq, (int)d, cs, qs,
                           (const int64_t*)probes, nprobe, list_off, codes, ids, k, D, I);
    else
        hipLaunchKernelGGL(ivf_scan_kernel<false>, dim3((unsigned)nq), dim3(64), 0, s, q, nq, (int)d, cs, qs,
                           (const int64_t*)probes, nprobe, list_off, codes, ids, k, D, I);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}

extern "C" int rvc_ivf_search(const float* q, int64_t nq, int64_t d, int64_t cs, int64_t qs, const float* centT,
                              int64_t nlist, int nprobe, const int64_t* list_off, const float* codes,
                              const int64_t* ids, int k, void* ws, int64_t ws_bytes, int64_t* probes, float* D,
                              int64_t* I, rvc_stream_t stream) {
    return rvc_ivf_search_ex(q, nq, d, cs, qs, centT, nlist, nprobe, list_off, codes, ids, k, ws, ws_bytes, probes, D,
                             I, RVC_IVF_FAISS, stream);
}

extern "C" int rvc_ivf_blend(const float* feats, int64_t nq, int64_t d, int64_t fcs, int64_t fqs, const float* D,
                             const int64_t* I, int k, const float* big, int64_t ntotal, double index_rate,
                             float* out, int64_t ocs, int64_t oqs, rvc_stream_t stream) {
    RVC_CHECK_ARG(feats && D && I && big && out, "ivf_blend: null pointer");
    RVC_CHECK_ARG(nq > 0 && d > 0 && k >= 1 && k <= 8 && ntotal > 0 && nq < 65536 * 32768ll, "ivf_blend: bad sizes");
    // torch: npy * index_rate + (1 - index_rate) * feats with the Python floats cast to f32
    const float r = (float)index_rate, r1 = (float)(1.0 - index_rate);
    hipLaunchKernelGGL(ivf_blend_kernel, dim3(cdiv(d, 256), (unsigned)nq), dim3(256), 0, (hipStream_t)stream, feats,
                       (int)d, fcs, fqs, D, I, k, big, ntotal, r, r1, out, ocs, oqs);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
