// Operand / result lane layout of v_mfma_f64_4x4x4f64 (4 blocks of 4x4x4 per wave, one f64 per lane each of A,
// B, C/D), found by experiment, and its rate beside v_mfma_f64_16x16x4f64 at the conv engine's shapes.
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma64_layout.hip -o scripts/mfma64_layout && scripts/mfma64_layout
// Prints, for every lane, which (block, row, k) its A value is, which (block, k, col) its B value is and which
// (block, row, col) its D value is, and checks the hypothesis the conv engine uses:
//   A: lane = i + 4 k + 16 b,  B: lane = j + 4 k + 16 b,  D: lane = j + 4 i + 16 b.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void probe(const double* a, const double* b, const double* c, double* d) {
    const int l = threadIdx.x;
    d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 0);
}

typedef double doublex4 __attribute__((ext_vector_type(4)));

// the 16x16x4 product from four 4x4x4 ones with A broadcast from block r (CBSZ 2, ABID r): d16 / d4 [4][64]
__global__ void bcast(const double* a, const double* b, double* d16, double* d4) {
    const int l = threadIdx.x;
    doublex4 z = {0.0, 0.0, 0.0, 0.0};
    z = __builtin_amdgcn_mfma_f64_16x16x4f64(a[l], b[l], z, 0, 0, 0);
    double r0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, 0, 0);
    double r1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, 1, 0);
    double r2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, 2, 0);
    double r3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, 3, 0);
    for (int r = 0; r < 4; ++r) d16[r * 64 + l] = z[r];
    d4[l] = r0;
    d4[64 + l] = r1;
    d4[128 + l] = r2;
    d4[192 + l] = r3;
}

template <int CB, int AB>
__global__ void variant(const double* a, const double* b, double* d) {
    const int l = threadIdx.x;
    d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, CB, AB, 0);
}

int main() {
    double *a, *b, *c, *d;
    hipMalloc(&a, 512);
    hipMalloc(&b, 512);
    hipMalloc(&c, 512);
    hipMalloc(&d, 512);
    double ha[64], hb[64], hc[64], hd[64];
    int bad = 0;
    // hypothesis check with random-ish integers: D = A B per block, computed on the host from the hypothesis
    for (int l = 0; l < 64; ++l) {
        ha[l] = (l * 7 + 3) % 11 - 5;
        hb[l] = (l * 5 + 1) % 13 - 6;
        hc[l] = (l * 3) % 7;
    }
    hipMemcpy(a, ha, 512, hipMemcpyHostToDevice);
    hipMemcpy(b, hb, 512, hipMemcpyHostToDevice);
    hipMemcpy(c, hc, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, a, b, c, d);
    hipMemcpy(hd, d, 512, hipMemcpyDeviceToHost);
    for (int blk = 0; blk < 4; ++blk)
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double s = hc[j + 4 * i + 16 * blk];
                for (int k = 0; k < 4; ++k) s += ha[i + 4 * k + 16 * blk] * hb[j + 4 * k + 16 * blk];
                if (s != hd[j + 4 * i + 16 * blk]) ++bad;
            }
    printf("hypothesis A: i+4k+16b, B: j+4k+16b, D: j+4i+16b -> %s (%d of 64 outputs differ)\n", bad ? "WRONG" : "OK",
           bad);
    // experiments: A = 2^(lane%16) + 65536 * block-of-lane, B = ones -> D = sum over the lanes holding its row
    for (int e = 0; e < 2; ++e) {
        for (int l = 0; l < 64; ++l) {
            const double bits = (double)(1 << (l % 16)) + 65536.0 * (l / 16);
            ha[l] = e == 0 ? bits : 1.0;
            hb[l] = e == 0 ? 1.0 : bits;
            hc[l] = 0.0;
        }
        hipMemcpy(a, ha, 512, hipMemcpyHostToDevice);
        hipMemcpy(b, hb, 512, hipMemcpyHostToDevice);
        hipMemcpy(c, hc, 512, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, a, b, c, d);
        hipMemcpy(hd, d, 512, hipMemcpyDeviceToHost);
        printf("%s = bits, %s = 1: per output lane, the contributing lanes (mod 16) / block sum\n", e ? "B" : "A",
               e ? "A" : "B");
        for (int l = 0; l < 16; ++l) {
            const long long v = (long long)hd[l];
            printf("  D lane %2d: lanes", l);
            for (int q = 0; q < 16; ++q)
                if ((v & 0xffff) >> q & 1) printf(" %d", q);
            printf("  (block field %lld)\n", v >> 16);
        }
    }
    {
        double *d16, *d4, h16[256], h4[256];
        hipMalloc(&d16, 2048);
        hipMalloc(&d4, 2048);
        for (int l = 0; l < 64; ++l) {
            ha[l] = (l * 7 + 3) % 11 - 5;
            hb[l] = (l * 5 + 1) % 13 - 6;
        }
        hipMemcpy(a, ha, 512, hipMemcpyHostToDevice);
        hipMemcpy(b, hb, 512, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(bcast, dim3(1), dim3(64), 0, 0, a, b, d16, d4);
        hipMemcpy(h16, d16, 2048, hipMemcpyDeviceToHost);
        hipMemcpy(h4, d4, 2048, hipMemcpyDeviceToHost);
        int diff = 0;
        for (int i = 0; i < 256; ++i) diff += h16[i] != h4[i];
        printf("16x16x4 == four 4x4x4 (CBSZ 2, ABID r) -> %s (%d of 256 differ)\n", diff ? "NO" : "YES", diff);
        bad = diff;
        // raw dump for offline analysis: a, b, then D for (cbsz, abid) = (0,0) (1,0) (1,1) (2,0) (2,1) (2,2) (2,3)
        FILE* f = fopen("gpurun_out/mfma64_dump.txt", "w");
        double hv[64];
        auto dump = [&](const double* v) { for (int l = 0; l < 64; ++l) fprintf(f, "%g ", v[l]); fprintf(f, "\n"); };
        dump(ha);
        dump(hb);
#define V(CB, AB)                                                                   \
    hipLaunchKernelGGL((variant<CB, AB>), dim3(1), dim3(64), 0, 0, a, b, d);       \
    hipMemcpy(hv, d, 512, hipMemcpyDeviceToHost);                                   \
    dump(hv);
        V(0, 0) V(1, 0) V(1, 1) V(2, 0) V(2, 1) V(2, 2) V(2, 3)
        dump(h16);
        dump(h16 + 64);
        dump(h16 + 128);
        dump(h16 + 192);
        fclose(f);
    }
    return bad != 0;
}
