// Filter-bank lab: times each level kernel of filterbank.hip on 4096^2 db8 (cfg5 block size)
// against a plain copy of the same bytes.  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../wavelettransforms_amd/csrc fblab.hip -o fblab
#include <hip/hip_runtime.h>
__device__ unsigned long long g_fp[8];
#define WTP_FPROBE(i) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_fp[i] = wall_clock64(); } while (0)
#include "../../wavelettransforms_amd/csrc/filterbank.hip"
#include <cstdio>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace wtp;

__global__ void k_copy(const float4* __restrict__ p, float4* __restrict__ q, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) q[i] = p[i];
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1;
    const int N = 4096, L = 5, F = 16;
    Taps tp;
    memset(&tp, 0, sizeof tp);
    tp.F = F;
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < F; ++j) tp.f[k][j] = 0.1f * (j + 1) * (k % 2 ? -1.0f : 1.0f);
    wt_level_geom g;
    wt_geom(N, N, L, &g);
    const size_t n = (size_t)B * N * N;
    float *x, *P, *t0, *t1, *y;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&P, (size_t)B * g.PR * g.PC * 4));
    CK(hipMalloc(&t0, n * 4)); CK(hipMalloc(&t1, n * 4)); CK(hipMalloc(&y, n * 4));
    CK(hipMemset(x, 0, n * 4)); CK(hipMemset(P, 0, (size_t)B * g.PR * g.PC * 4));
    float thr = 0.001f, *dthr; CK(hipMalloc(&dthr, 4)); CK(hipMemcpy(dthr, &thr, 4, hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto bench = [&](const char* name, auto fn, double bytes) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipDeviceSynchronize());
        const int R = 20;
        CK(hipEventRecord(a));
        for (int i = 0; i < R; ++i) fn();
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / R;
        printf("%-40s %9.2f us  %7.0f GB/s\n", name, us, bytes / us / 1e3);
    };
    printf("B = %d, %dx%d, db8-like F=%d, L=%d\n", B, N, N, F, L);
    bench("copy 4096^2 x B", [&] { hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, (float4*)x, (float4*)y, (int64_t)n / 4); }, 8.0 * n);
    for (int k = 1; k <= L; ++k) {
        const int64_t R0 = g.R[k - 1], C0 = g.C[k - 1];
        const float* in = k == 1 ? x : t0;
        char nm[64];
        snprintf(nm, 64, "fwd level %d (%lldx%lld)", k, (long long)R0, (long long)C0);
        const double bytes = 4.0 * B * (R0 * C0 + 4 * g.R[k] * g.C[k]);
        bench(nm, [&] { launch_fwd_level(in, B, R0, C0, tp, t1, P, g.PR, g.PC, g.offR[k], g.offC[k], k == L, 0); }, bytes);
        unsigned long long fp[8]; CK(hipMemcpyFromSymbol(fp, HIP_SYMBOL(g_fp), sizeof(fp)));
        printf("    WG0 phases (us): load %.2f  colpass %.2f  rowpass %.2f\n", (fp[1] - fp[0]) / 100.0, (fp[2] - fp[1]) / 100.0, (fp[3] - fp[2]) / 100.0);
    }
    for (int k = L; k >= 1; --k) {
        const int64_t R = g.R[k], C = g.C[k];
        const bool fromP = k == L;
        char nm[64];
        snprintf(nm, 64, "inv level %d (%lldx%lld out)", k, (long long)(2 * R), (long long)(2 * C));
        const double bytes = 4.0 * B * (4 * R * C + 4 * R * C);
        bench(nm, [&] {
            launch_inv_level(fromP ? nullptr : t0, fromP ? 0 : 4 * g.R[k + 1] * g.C[k + 1], fromP ? 0 : 2 * g.C[k + 1],
                             fromP, P, g.PR, g.PC, g.offR[k], g.offC[k], B, R, C, tp, dthr, k == 1 ? y : t1, k == 1 ? N : 2 * R,
                             k == 1 ? N : 2 * C, nullptr, 0);
        }, bytes);
    }
    return 0;
}
