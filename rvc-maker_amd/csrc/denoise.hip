// Spectral-gate denoise (main/tools/noisereduce.py, the non-stationary TG that
// VoiceConverter.convert_audio runs for clean_audio, convert.py:514-516) in f64 on the device.
//
// The reference runs the whole gate in float64 (SpectralGate._read_chunk builds each chunk with
// np.zeros, noisereduce.py:76) over chunks of chunk_size samples, each zero-padded by `padding`
// on both sides and filtered independently (get_traces, :96-122).  All chunks of a signal are one
// batch here (grid.y = segment):
//   1. stft_fft       frame (centre zero padding) x window -> radix-2 FFT in LDS -> X [seg][bin][F] (complex)
//                     and |X| [seg][bin][F]
//   2. gate_mask      moving mean of |X| over n_movemean frames ("same" conv1d, :164), direct sums
//                     from an LDS row tile; sigmoid((|X|/mean - 1 - thresh) / temp) (:165);
//                     prop * (m - 1) + 1 (:176)
//   3. mask_smooth    "same" conv2d of the mask with the (2 nf + 1) x (2 nt + 1) triangle (:177) from an
//                     LDS tile; Y = X * mask in place
//   4. istft_frames   Hermitian spectrum -> inverse FFT -> x window -> frames [seg][F][n_fft]
//   5. ola_out        overlap-add / window-square envelope (torch.istft, centre trimmed; the envelope in
//                     f32 like torch with the reference's float32 window), the
//                     segment's kept range [padding, padding + len) -> f32 output
// HBM-bound bookkeeping around a few hundred MFLOP of f64 FFT work.
#include "rvc_common.h"

namespace {

constexpr int NFFT_MAX = 2048;
constexpr int MM_TILE = 256;     // frames per gate_mask block
constexpr int MM_MAX = 4096;     // longest moving-mean window staged in LDS
constexpr int SM_TK = 16, SM_TF = 64;  // mask_smooth output tile (bins x frames)
constexpr int SM_HALO_MAX = 48;  // nf, nt <= 48 (8 kHz: nf 32; 96 kHz: nt 18)
constexpr int SM_LDS_MAX = 64 * 1024;

struct DnParams {
    const float* y;
    int64_t n, chunk, pad, nseg, Ls, F;
    int nfft, hop, nbin, logn, n_mm, fh, fw;
    double prop, thresh, temp;
    const double* win;
    const double* filt;
    double2* X;  // [seg][nbin][F]
    double* A;   // [seg][nbin][F] |X|
    double* M;   // [seg][nbin][F] mask
    double* Fr;  // [seg][F][nfft] (aliases A/M after the mask is applied)
    float* out;
};

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// In-place iterative radix-2 DIT FFT (forward, e^{-2 pi i k n / N}) of N points in LDS `a`, input
// already in bit-reversed order.  Twiddles by sincospi in f64.
__device__ void fft_lds(double2* a, int N, int logn) {
    for (int s = 1; s <= logn; ++s) {
        const int half = 1 << (s - 1);
        for (int j = threadIdx.x; j < N / 2; j += blockDim.x) {
            const int pos = j & (half - 1);
            const int i0 = ((j >> (s - 1)) << s) + pos;
            const int i1 = i0 + half;
            double sn, cs;
            sincospi(-(double)pos / (double)half, &sn, &cs);
            const double2 t = cmul(make_double2(cs, sn), a[i1]);
            const double2 u = a[i0];
            a[i0] = make_double2(u.x + t.x, u.y + t.y);
            a[i1] = make_double2(u.x - t.x, u.y - t.y);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ int bitrev(int i, int logn) { return (int)(__brev((unsigned)i) >> (32 - logn)); }

// segment s covers input samples [s * chunk - pad, s * chunk - pad + Ls); outside [0, n) is zero
__global__ __launch_bounds__(256) void stft_fft_kernel(DnParams p) {
    __shared__ double2 a[NFFT_MAX];
    const int f = blockIdx.x, s = blockIdx.y;
    const int64_t seg0 = (int64_t)s * p.chunk - p.pad;
    for (int i = threadIdx.x; i < p.nfft; i += blockDim.x) {
        const int64_t loc = (int64_t)f * p.hop + i - p.nfft / 2;  // centre padding of torch.stft
        const int64_t g = seg0 + loc;
        const float v = (loc >= 0 && loc < p.Ls && g >= 0 && g < p.n) ? p.y[g] : 0.f;
        a[bitrev(i, p.logn)] = make_double2((double)v * p.win[i], 0.0);
    }
    __syncthreads();
    fft_lds(a, p.nfft, p.logn);
    for (int k = threadIdx.x; k < p.nbin; k += blockDim.x) {
        const int64_t o = ((int64_t)s * p.nbin + k) * p.F + f;
        const double2 v = a[k];
        p.X[o] = v;
        p.A[o] = sqrt(v.x * v.x + v.y * v.y);
    }
}

// moving mean ("same": (k-1)//2 zeros left, the rest right) -> gate mask
__global__ __launch_bounds__(256) void gate_mask_kernel(DnParams p) {
    __shared__ double row[MM_TILE + MM_MAX];
    const int k = blockIdx.y % p.nbin, s = blockIdx.y / p.nbin;
    const int64_t f0 = (int64_t)blockIdx.x * MM_TILE;
    const int left = (p.n_mm - 1) / 2;
    const double* ar = p.A + ((int64_t)s * p.nbin + k) * p.F;
    const int span = MM_TILE + p.n_mm - 1;
    for (int i = threadIdx.x; i < span; i += blockDim.x) {
        const int64_t f = f0 - left + i;
        row[i] = (f >= 0 && f < p.F) ? ar[f] : 0.0;
    }
    __syncthreads();
    const int64_t f = f0 + threadIdx.x;
    if (f >= p.F) return;
    double sum = 0.0;
    for (int j = 0; j < p.n_mm; ++j) sum += row[threadIdx.x + j];
    const double xs = sum / (double)p.n_mm;
    const double xa = row[threadIdx.x + left];
    const double z = (((xa - xs) / xs) - p.thresh) / p.temp;
    const double m = 1.0 / (1.0 + exp(-z));
    p.M[((int64_t)s * p.nbin + k) * p.F + f] = p.prop * (m * 1.0 - 1.0) + 1.0;
}

// "same" conv2d with the smoothing filter (zero padding), then Y = X * mask in place
__global__ __launch_bounds__(256) void mask_smooth_kernel(DnParams p) {
    extern __shared__ double t[];  // [SM_TK + 2 hk][SM_TF + 2 hf] mask tile, then the filter
    const int s = blockIdx.z;
    const int k0 = blockIdx.y * SM_TK;
    const int64_t f0 = (int64_t)blockIdx.x * SM_TF;
    const int hk = p.fh / 2, hf = p.fw / 2;
    const int th = SM_TK + 2 * hk, tw = SM_TF + 2 * hf;
    double* fl = t + th * tw;
    const double* mr = p.M + (int64_t)s * p.nbin * p.F;
    for (int i = threadIdx.x; i < th * tw; i += blockDim.x) {
        const int r = i / tw, c = i - r * tw;
        const int k = k0 - hk + r;
        const int64_t f = f0 - hf + c;
        t[i] = (k >= 0 && k < p.nbin && f >= 0 && f < p.F) ? mr[(int64_t)k * p.F + f] : 0.0;
    }
    for (int i = threadIdx.x; i < p.fh * p.fw; i += blockDim.x) fl[i] = p.filt[i];
    __syncthreads();
    for (int e = threadIdx.x; e < SM_TK * SM_TF; e += blockDim.x) {
        const int r = e / SM_TF, c = e - r * SM_TF;
        const int k = k0 + r;
        const int64_t f = f0 + c;
        if (k >= p.nbin || f >= p.F) continue;
        double acc = 0.0;
        for (int i = 0; i < p.fh; ++i)
            for (int j = 0; j < p.fw; ++j) acc += fl[i * p.fw + j] * t[(r + i) * tw + c + j];
        const int64_t o = ((int64_t)s * p.nbin + k) * p.F + f;
        const double2 x = p.X[o];
        p.X[o] = make_double2(x.x * acc, x.y * acc);
    }
}

// no smoothing filter: Y = X * mask
__global__ __launch_bounds__(256) void mask_apply_kernel(DnParams p) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= p.nseg * p.nbin * p.F) return;
    const double m = p.M[i];
    const double2 x = p.X[i];
    p.X[i] = make_double2(x.x * m, x.y * m);
}

// inverse real FFT of one frame (c2r: imaginary parts of DC / Nyquist ignored) x window
__global__ __launch_bounds__(256) void istft_frames_kernel(DnParams p) {
    __shared__ double2 a[NFFT_MAX];
    const int f = blockIdx.x, s = blockIdx.y;
    const int N = p.nfft;
    const double2* xr = p.X + (int64_t)s * p.nbin * p.F + f;
    // ifft(Z) = conj(fft(conj(Z))) / N; the real part needs only Re(fft(conj Z))
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        double2 z;
        if (i == 0 || i == N / 2) z = make_double2(xr[(int64_t)i * p.F].x, 0.0);
        else if (i < N / 2) z = xr[(int64_t)i * p.F];
        else {
            const double2 c = xr[(int64_t)(N - i) * p.F];
            z = make_double2(c.x, -c.y);
        }
        a[bitrev(i, p.logn)] = make_double2(z.x, -z.y);
    }
    __syncthreads();
    fft_lds(a, N, p.logn);
    double* fr = p.Fr + ((int64_t)s * p.F + f) * N;
    for (int i = threadIdx.x; i < N; i += blockDim.x) fr[i] = a[i].x / (double)N * p.win[i];
}

// overlap-add / envelope, centre-trimmed, segment s's kept samples -> out
__global__ __launch_bounds__(256) void ola_out_kernel(DnParams p) {
    const int s = blockIdx.y;
    const int64_t o = (int64_t)s * p.chunk + (int64_t)blockIdx.x * 256 + threadIdx.x;  // output sample
    const int64_t end = p.nseg > 1 ? min((int64_t)(s + 1) * p.chunk, p.n) : p.n;
    if (o >= end) return;
    const int64_t u = p.pad + (o - (int64_t)s * p.chunk) + p.nfft / 2;  // position in the un-trimmed OLA buffer
    int64_t fa = (u - p.nfft + p.hop) / p.hop;  // first frame with u - f hop < nfft
    if (fa < 0) fa = 0;
    int64_t fb = u / p.hop;
    if (fb > p.F - 1) fb = p.F - 1;
    // torch.istft builds the window-square envelope in the window's dtype: float32 (the reference's
    // torch.hann_window), squared and overlap-added in f32 in frame order -- no contraction
    double num = 0.0;
    float env = 0.f;
    for (int64_t f = fa; f <= fb; ++f) {
        const int i = (int)(u - f * p.hop);
        num += p.Fr[((int64_t)s * p.F + f) * p.nfft + i];
        const float wf = (float)p.win[i];
        env = __fadd_rn(env, __fmul_rn(wf, wf));
    }
    p.out[o] = (float)(num / (double)env);
}

size_t smooth_lds(const DnParams& p) {
    return (size_t)((SM_TK + 2 * (p.fh / 2)) * (SM_TF + 2 * (p.fw / 2)) + p.fh * p.fw) * sizeof(double);
}

int plan(const float* y, int64_t n, const rvc_denoise_args* a, DnParams& p) {
    RVC_CHECK_ARG(a && n > 0 && a->n_fft >= 64 && a->n_fft <= NFFT_MAX && (a->n_fft & (a->n_fft - 1)) == 0,
                  "denoise: n_fft must be a power of two in [64, %d]", NFFT_MAX);
    RVC_CHECK_ARG(a->hop > 0 && a->hop <= a->n_fft && a->padding >= 0 && a->n_movemean >= 1 &&
                      a->n_movemean <= MM_MAX, "denoise: bad hop / padding / moving-mean window");
    RVC_CHECK_ARG(a->filt_h >= 0 && a->filt_w >= 0 && a->filt_h <= 2 * SM_HALO_MAX + 1 &&
                      a->filt_w <= 2 * SM_HALO_MAX + 1 && (a->filt_h == 0 || (a->filt_h % 2 == 1 && a->filt_w % 2 == 1)),
                  "denoise: smoothing filter must be odd x odd, at most %d", 2 * SM_HALO_MAX + 1);
    p.y = y;
    p.n = n;
    const bool chunked = a->chunk_size > 0 && n > a->chunk_size;
    p.nseg = chunked ? (n - 1) / a->chunk_size + 1 : 1;
    p.chunk = chunked ? a->chunk_size : n;
    p.pad = a->padding;
    p.Ls = p.chunk + 2 * p.pad;
    RVC_CHECK_ARG(p.Ls >= 2 * a->n_fft, "denoise: chunk shorter than 2 * win_length (noisereduce.py:169)");
    p.nfft = a->n_fft;
    p.hop = a->hop;
    p.nbin = a->n_fft / 2 + 1;
    p.logn = 0;
    while ((1 << p.logn) < p.nfft) ++p.logn;
    p.F = 1 + p.Ls / p.hop;
    RVC_CHECK_ARG(p.pad + p.chunk <= p.hop * (p.F - 1), "denoise: istft output shorter than the kept range");
    p.n_mm = a->n_movemean;
    p.fh = a->filt_h;
    p.fw = a->filt_w;
    p.prop = a->prop_decrease;
    p.thresh = a->n_thresh;
    p.temp = a->temp_coeff;
    RVC_CHECK_ARG(smooth_lds(p) <= SM_LDS_MAX, "denoise: smoothing filter %d x %d too large", p.fh, p.fw);
    p.win = a->window;
    p.filt = a->filt;
    return RVC_OK;
}

}  // namespace

extern "C" int64_t rvc_denoise_work_bytes(int64_t n, const rvc_denoise_args* a) {
    DnParams p;
    if (plan(nullptr, n, a, p) != RVC_OK) return -1;
    const int64_t cells = p.nseg * p.nbin * p.F;
    const int64_t am = 2 * cells * 8, fr = p.nseg * p.F * p.nfft * 8;
    return cells * 16 + (am > fr ? am : fr);
}

extern "C" int rvc_denoise(const float* y, int64_t n, const rvc_denoise_args* a, void* work, int64_t work_bytes,
                           float* out, rvc_stream_t stream) {
    DnParams p;
    const int rc = plan(y, n, a, p);
    if (rc != RVC_OK) return rc;
    RVC_CHECK_ARG(y && out && a->window && (a->filt_h == 0 || a->filt), "denoise: null pointer");
    const int64_t need = rvc_denoise_work_bytes(n, a);
    RVC_CHECK_ARG(work && work_bytes >= need, "denoise: work needs %lld B", (long long)need);
    const int64_t cells = p.nseg * p.nbin * p.F;
    p.X = (double2*)work;
    p.A = (double*)((char*)work + cells * 16);
    p.M = p.A + cells;
    p.Fr = p.A;  // written after A and M are consumed
    p.out = out;
    hipStream_t s = (hipStream_t)stream;
    RVC_CHECK_ARG(p.F < (1 << 30) && p.nseg < 65536, "denoise: signal too long");
    hipLaunchKernelGGL(stft_fft_kernel, dim3((unsigned)p.F, (unsigned)p.nseg), dim3(256), 0, s, p);
    RVC_HIP(hipGetLastError());
    hipLaunchKernelGGL(gate_mask_kernel, dim3(cdiv(p.F, MM_TILE), (unsigned)(p.nseg * p.nbin)), dim3(256), 0, s, p);
    RVC_HIP(hipGetLastError());
    if (p.fh > 0) {
        hipLaunchKernelGGL(mask_smooth_kernel, dim3(cdiv(p.F, SM_TF), cdiv(p.nbin, SM_TK), (unsigned)p.nseg), dim3(256),
                           smooth_lds(p), s, p);
    } else {
        hipLaunchKernelGGL(mask_apply_kernel, dim3(cdiv(cells, 256)), dim3(256), 0, s, p);
    }
    RVC_HIP(hipGetLastError());
    hipLaunchKernelGGL(istft_frames_kernel, dim3((unsigned)p.F, (unsigned)p.nseg), dim3(256), 0, s, p);
    RVC_HIP(hipGetLastError());
    hipLaunchKernelGGL(ola_out_kernel, dim3(cdiv(p.chunk, 256), (unsigned)p.nseg), dim3(256), 0, s, p);
    RVC_HIP(hipGetLastError());
    return RVC_OK;
}
