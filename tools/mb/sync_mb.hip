// Cost of a block-wide step (LDS write, __syncthreads, LDS read) at one 512-thread workgroup per
// CU, with and without ~96 live VGPRs of data per thread.  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
__device__ unsigned long long g_t[256][2];
template <int T, int STEPS, bool HEAVY>
__global__ __launch_bounds__(T) void k_sync(const float4* p, float* out) {
    __shared__ uint32_t buf[T * 4];
    float4 v[24];
    if (HEAVY) {
#pragma unroll
        for (int i = 0; i < 24; ++i) v[i] = p[(blockIdx.x * 24 + i) * T + threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x == 0) g_t[blockIdx.x][0] = wall_clock64();
    uint32_t a = threadIdx.x;
    for (int s = 0; s < STEPS; ++s) {
        buf[(threadIdx.x * 7 + s) % (T * 4)] = a;
        __syncthreads();
        a += buf[(threadIdx.x * 13 + s * 5) % (T * 4)];
        __syncthreads();
    }
    if (threadIdx.x == 0) g_t[blockIdx.x][1] = wall_clock64();
    float sx = a;
    if (HEAVY) {
#pragma unroll
        for (int i = 0; i < 24; ++i) sx += v[i].x + v[i].y;
    }
    if (sx == 1234.5f) out[blockIdx.x] = sx;
}
template <int T, int STEPS, bool HEAVY>
void run(const char* name, const float4* p, float* out, int nb) {
    std::vector<double> per;
    for (int r = 0; r < 20; ++r) {
        hipLaunchKernelGGL((k_sync<T, STEPS, HEAVY>), dim3(nb), dim3(T), 0, 0, p, out);
        CK(hipDeviceSynchronize());
        unsigned long long t[256][2];
        CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_t), sizeof t));
        std::vector<double> d;
        for (int i = 0; i < nb; ++i) d.push_back((double)(t[i][1] - t[i][0]) * 10.0 / (2.0 * STEPS)); /* ns per sync step */
        std::sort(d.begin(), d.end());
        per.push_back(d[d.size() / 2]);
    }
    std::sort(per.begin(), per.end());
    printf("%-40s %7.1f ns per (LDS op + __syncthreads)\n", name, per[per.size() / 2]);
}
int main() {
    float4* p; float* out;
    CK(hipMalloc(&p, 256ull * 24 * 1024 * 16)); CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(p, 0, 256ull * 24 * 1024 * 16));
    run<512, 200, false>("512 thr, 231 WG, light", p, out, 231);
    run<512, 200, true>("512 thr, 231 WG, 96 live regs", p, out, 231);
    run<256, 200, false>("256 thr, 231 WG, light", p, out, 231);
    run<1024, 200, false>("1024 thr, 231 WG, light", p, out, 231);
    run<64, 200, false>("64 thr, 231 WG, light", p, out, 231);
}
