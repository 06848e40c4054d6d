// Which CUs does a CU-masked stream (hipExtStreamCreateWithCUMask, VC.BACK_CU_MASK) actually run on?  Launches
// many short blocks on a stream masked with "mod:m:r" (every CU whose mask index is r mod m left out) and on an
// unmasked stream; each block reads its XCC id (HW_REG_XCC_ID) and its SE / CU (HW_REG_HW_ID) and stores them.
// Prints, per XCC, how many distinct (SE, CU) slots each stream used.
//   hipcc --offload-arch=gfx950 -O2 scripts/cu_mask_probe.hip -o /tmp/cu_mask_probe && /tmp/cu_mask_probe 8 7
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <set>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void probe(unsigned* out) {
    if (threadIdx.x == 0) {
        // s_getreg_b32: XCC_ID (hwreg 20, bits 3:0) and HW_ID (hwreg 4, all bits)
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));
        const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
    // stay resident a little so that the blocks spread over the CUs the stream may use
    const long long t0 = clock64();
    while (clock64() - t0 < 200000) {
    }
}

static void run(hipStream_t s, const char* name, int nblk) {
    unsigned* d;
    CK(hipMalloc(&d, 8 * nblk));
    CK(hipMemsetAsync(d, 0xff, 8 * nblk, s));
    hipLaunchKernelGGL(probe, dim3(nblk), dim3(64), 0, s, d);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(s));
    std::vector<unsigned> h(2 * nblk);
    CK(hipMemcpy(h.data(), d, 8 * nblk, hipMemcpyDeviceToHost));
    CK(hipFree(d));
    std::set<unsigned> slots[16];
    for (int i = 0; i < nblk; ++i) {
        const unsigned xcc = h[2 * i] & 15, hw = h[2 * i + 1];
        const unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        slots[xcc].insert((se << 8) | (sh << 4) | cu);
    }
    printf("%-10s", name);
    int tot = 0;
    for (int x = 0; x < 8; ++x) {
        printf(" xcc%d:%2zu", x, slots[x].size());
        tot += (int)slots[x].size();
    }
    printf("  total %d\n", tot);
}

int main(int argc, char** argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 8, r = argc > 2 ? atoi(argv[2]) : 7;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0), top((ncu + 31) / 32, 0);
    for (int i = 0; i < ncu; ++i) {
        if (i % m != r) mask[i / 32] |= 1u << (i % 32);
        if (i < ncu - 32) top[i / 32] |= 1u << (i % 32);
    }
    hipStream_t plain, masked, topm;
    CK(hipStreamCreate(&plain));
    CK(hipExtStreamCreateWithCUMask(&masked, (uint32_t)mask.size(), mask.data()));
    CK(hipExtStreamCreateWithCUMask(&topm, (uint32_t)top.size(), top.data()));
    printf("%d CUs; mask mod:%d:%d keeps %d bits, top:32 keeps %d bits\n", ncu, m, r,
           ncu - (ncu + m - 1 - r) / m, ncu - 32);
    const int nblk = 8 * ncu;
    run(plain, "unmasked", nblk);
    char nm[32];
    snprintf(nm, sizeof nm, "mod:%d:%d", m, r);
    run(masked, nm, nblk);
    run(topm, "top:32", nblk);
    CK(hipStreamDestroy(masked));
    CK(hipStreamDestroy(topm));
    CK(hipStreamDestroy(plain));
    return 0;
}
