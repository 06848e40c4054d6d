// Where does the f64 conv engine's time go?  rmvpe64.hip built with C64_DBG bits that take parts of the main
// loop out (timing only: results are wrong), on one RMVPE U-Net level (Ci = Co = 64, 752 x 32) with the plan
// forced.  Build each variant:
//   for d in 0 1 2 3 4 8 12 15; do hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Irvc-maker_amd/csrc \
//     -DC64_DBG=$d scripts/conv64_dbg.hip -Lrvc-maker_amd/lib -lrvc_amd -o scripts/conv64_dbg_$d; done
//   LD_LIBRARY_PATH=rvc-maker_amd/lib scripts/conv64_dbg_0 C H W tile ks cmp
#include "../rvc-maker_amd/csrc/rmvpe64.hip"
#include <stdio.h>
#include <vector>

int main(int argc, char** argv) {
    const int C = argc > 1 ? atoi(argv[1]) : 64, H = argc > 2 ? atoi(argv[2]) : 752, W = argc > 3 ? atoi(argv[3]) : 32;
    const int tile = argc > 4 ? atoi(argv[4]) : 2, ks = argc > 5 ? atoi(argv[5]) : 4, cmp = argc > 6 ? atoi(argv[6]) : 1;
    const int wrap = W + 2;
    const int64_t L = (int64_t)(H + 2) * wrap;
    double *x, *w, *y, *ws;
    hipMalloc(&x, C * L * 8);
    hipMalloc(&w, (int64_t)C * 9 * C * 8);
    hipMalloc(&y, C * L * 8);
    hipMalloc(&ws, (int64_t)64 << 20);
    hipMemset(x, 0, C * L * 8);
    hipMemset(w, 0, (int64_t)C * 9 * C * 8);
    rvc_conv64_args a = {};
    a.x = x; a.w = w; a.y = y;
    a.B = 1; a.Ci = C; a.Co = C; a.Lin = L; a.Lout = L;
    a.K = 9; a.pad = wrap + 1; a.out_act = RVC_ACT_RELU; a.ntoff = 9; a.wrap = wrap;
    for (int i = 0; i < 9; ++i) a.toff[i] = (i / 3) * wrap + i % 3;
    rvc_conv64_set_plan(tile, ks, cmp);
    int plan[4];
    if (rvc_conv64_plan(&a, plan) != RVC_OK) { printf("plan refused\n"); return 1; }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) rvc_conv64(&a, ws, (int64_t)64 << 20, nullptr);
    hipEventRecord(e0, nullptr);
    const int n = 50;
    for (int i = 0; i < n; ++i) rvc_conv64(&a, ws, (int64_t)64 << 20, nullptr);
    hipEventRecord(e1, nullptr);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / n, gf = 2.0 * C * C * 9 * H * W / 1e9;
    printf("dbg %2d  C %d %dx%d tile %d ks %d cmp %d blocks %d: %7.1f us  %5.1f TF\n", C64_DBG, C, H, W, plan[0], plan[1],
           plan[2], plan[3], us, gf / us * 1e3);
    return 0;
}
