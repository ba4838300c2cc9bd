// VALU issue cost of packed FP32 (v_pk_mul_f32 + v_pk_add_f32) against scalar FP32 (v_mul_f32 +
// v_add_f32) on gfx950, no FMA contraction (the filter bank's bit-exactness contract).  Not
// part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off pkrate.hip -o pkrate
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;
__global__ void k_pk(float* out, float t0, float t1, unsigned long long* cyc) {
    f2 acc[8], v[8];
    for (int i = 0; i < 8; ++i) { acc[i] = f2{0.0f, 0.0f}; v[i] = f2{threadIdx.x * 1e-3f + i, i * 0.5f}; }
    const f2 t = {t0, t1};
    unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = acc[i] + t * v[i];
    }
    unsigned long long c1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = c1 - c0;
}
__global__ void k_sc(float* out, float t0, float t1, unsigned long long* cyc) {
    float acc[16], v[16];
    for (int i = 0; i < 16; ++i) { acc[i] = 0.0f; v[i] = threadIdx.x * 1e-3f + i; }
    unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = acc[i] + (i & 1 ? t1 : t0) * v[i];
    }
    unsigned long long c1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = c1 - c0;
}
int main() {
    float* out; unsigned long long* cyc; unsigned long long h[4096];
    hipMalloc(&out, 1 << 24); hipMalloc(&cyc, sizeof h);
    for (int wps = 1; wps <= 8; wps *= 2) { // waves per SIMD: one block per CU of 4*wps waves
        for (int kind = 0; kind < 2; ++kind) {
            const int threads = 256 * wps > 1024 ? 1024 : 256 * wps;
            const int blocks = 256 * (256 * wps / threads);
            for (int rep = 0; rep < 2; ++rep) {
                if (kind == 0) hipLaunchKernelGGL(k_pk, dim3(blocks), dim3(threads), 0, 0, out, 0.5f, 0.25f, cyc);
                else hipLaunchKernelGGL(k_sc, dim3(blocks), dim3(threads), 0, 0, out, 0.5f, 0.25f, cyc);
                hipDeviceSynchronize();
            }
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            hipEventRecord(a);
            if (kind == 0) hipLaunchKernelGGL(k_pk, dim3(blocks), dim3(threads), 0, 0, out, 0.5f, 0.25f, cyc);
            else hipLaunchKernelGGL(k_sc, dim3(blocks), dim3(threads), 0, 0, out, 0.5f, 0.25f, cyc);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            const int nw = blocks * threads / 64;
            hipMemcpy(h, cyc, sizeof(unsigned long long) * (nw < 4096 ? nw : 4096), hipMemcpyDeviceToHost);
            double avg = 0; for (int i = 0; i < 256; ++i) avg += h[i]; avg /= 256;
            const double ops = 16.0 * ITERS; // mul + add lane-ops per lane: 8 pk-pairs = 16 MACs... per iteration
            const double flop = 2.0 * 16 * ITERS * 64.0 * nw; // 16 MACs per lane per iteration
            printf("%s waves/SIMD %d: %.1f cycles per wave per iteration (%.2f per MAC-pair instr), %.1f TFLOP/s (no FMA)\n",
                   kind == 0 ? "packed" : "scalar", wps, avg / ITERS, avg / ITERS / (kind == 0 ? 16 : 32), flop / (ms * 1e-3) / 1e12);
            (void)ops;
        }
    }
    return 0;
}
