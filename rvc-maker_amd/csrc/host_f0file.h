// Host-only C++ (no HIP): the f0-file resampling of VC.get_f0 (main/inference/convert.py:316-318), shared by
// rvc_frontend.cpp (rvc_vc_convert_ex, rvc_f0_file_resample) and the CPU sanitizer build in
// tests/test_c_host_cpu.py.
#pragma once
#include <cmath>
#include <cstdint>
#include <vector>

namespace rvc_host {

// rows: nrows x (time s, f0 Hz) f32 as read_f0_file gives them.  rep <- np.interp(range(n), t * 100, f0) in f64
// with numpy's branch structure, n = np.round((max t - min t) * 100 + 1).astype(np.int16) in f32 (x86 numpy
// casts through a 32-bit int, so an n past int16 wraps as there; n <= 0 gives no values).  Returns 0, or -1 for
// times that are not finite or whose frame count does not fit 32 bits (numpy's cast is undefined there).
inline int f0_file_interp(const float* rows, int64_t nrows, std::vector<double>& rep) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    rep.clear();
    if (!rows || nrows < 1) return -1;
    float tmin = rows[0], tmax = rows[0];
    for (int64_t i = 0; i < nrows; ++i) {
        if (!std::isfinite(rows[2 * i])) return -1;
        tmin = rows[2 * i] < tmin ? rows[2 * i] : tmin;
        tmax = rows[2 * i] > tmax ? rows[2 * i] : tmax;
    }
    const float span = tmax - tmin;
    const float v = span * 100.f + 1.f;
    if (!(std::fabs(v) < 2147483520.f)) return -1;
    const int64_t n = (int16_t)(int32_t)rintf(v);  // np.round (half to even), astype(np.int16)
    rep.assign(n > 0 ? n : 0, 0.0);
    std::vector<double> xp(nrows), fp(nrows);
    for (int64_t i = 0; i < nrows; ++i) {
        xp[i] = (double)(rows[2 * i] * 100.f);  // inp_f0[:, 0] * 100 is f32, np.interp takes it as f64
        fp[i] = (double)rows[2 * i + 1];
    }
    for (int64_t k = 0; k < (int64_t)rep.size(); ++k) {
        const double x = (double)k;
        if (x < xp[0]) {
            rep[k] = fp[0];
            continue;
        }
        if (x > xp[nrows - 1]) {
            rep[k] = fp[nrows - 1];
            continue;
        }
        int64_t lo = 0, hi = nrows - 1;  // xp[j] <= x < xp[j + 1] (binary search over a sorted xp)
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) / 2;
            if (xp[mid] <= x) lo = mid;
            else hi = mid - 1;
        }
        const int64_t j = lo;
        if (j == nrows - 1 || xp[j] == x) {
            rep[k] = fp[j];
            continue;
        }
        const double slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
        rep[k] = slope * (x - xp[j]) + fp[j];
    }
    return 0;
}

}  // namespace rvc_host
