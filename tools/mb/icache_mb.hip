// Cost of executing straight-line code once per wave (instruction-cache misses) vs the same
// instruction count in a loop.  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
#pragma clang fp contract(off)
template <int N, bool UNROLL>
__global__ __launch_bounds__(512) void k_code(float* out, float a, float b) {
    float v = threadIdx.x * 1e-3f, w = v + 1.f;
    if (UNROLL) {
#pragma unroll
        for (int i = 0; i < N; ++i) { v = v * a + b; w = w * b + v; asm volatile("" : "+v"(v), "+v"(w)); }
    } else {
#pragma nounroll
        for (int i = 0; i < N; ++i) { v = v * a + b; w = w * b + v; asm volatile("" : "+v"(v), "+v"(w)); }
    }
    if (v + w == 1234.5f) out[blockIdx.x] = v;
}
template <int N, bool U>
void run(const char* name, float* out, int nb) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int r = 0; r < 30; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_code<N, U>), dim3(nb), dim3(512), 0, 0, out, 1.0001f, 0.5f);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms * 1000);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-40s %8.2f us\n", name, ts[ts.size() / 2]);
}
int main() {
    float* out; CK(hipMalloc(&out, 1 << 20));
    for (int k = 0; k < 2; ++k) {
        run<16, false>("empty-ish (16 iters loop)", out, 231);
        run<2000, false>("loop 2000 iters (4k fp ops/thread)", out, 231);
        run<2000, true>("straight-line 2000 iters (~32 KB code)", out, 231);
        run<4000, false>("loop 4000 iters", out, 231);
        run<4000, true>("straight-line 4000 iters (~64 KB code)", out, 231);
    }
}
