// Streaming micro-benchmarks on the cfg2 footprint (11,166,912 floats = 44.7 MB), used to
// choose the shape of the selection passes.  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int T = 256;

template <int PER>  // PER float4 per thread, upfront
__global__ __launch_bounds__(T) void k_read(const float4* __restrict__ p, int64_t n4, float* out) {
    int64_t base = (int64_t)blockIdx.x * T * PER;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; v[i] = j < n4 ? p[j] : make_float4(0,0,0,0); }
    float s = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) s += v[i].x + v[i].y + v[i].z + v[i].w;
    if (s == 12345.f) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(T) void k_read_gs(const float4* __restrict__ p, int64_t n4, float* out) {
    float s = 0;
    for (int64_t j = (int64_t)blockIdx.x * T + threadIdx.x; j < n4; j += (int64_t)gridDim.x * T) {
        float4 v = p[j]; s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[blockIdx.x] = s;
}

template <int PER>
__global__ __launch_bounds__(T) void k_copy(const float4* __restrict__ p, float4* __restrict__ q, int64_t n4, float thr) {
    int64_t base = (int64_t)blockIdx.x * T * PER;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; if (j < n4) v[i] = p[j]; }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        int64_t j = base + i * T + threadIdx.x;
        float4 y = v[i];
        y.x = fabsf(y.x) < thr ? 0.f : y.x; y.y = fabsf(y.y) < thr ? 0.f : y.y;
        y.z = fabsf(y.z) < thr ? 0.f : y.z; y.w = fabsf(y.w) < thr ? 0.f : y.w;
        if (j < n4) q[j] = y;
    }
}

__global__ __launch_bounds__(T) void k_copy_gs(const float4* __restrict__ p, float4* __restrict__ q, int64_t n4, float thr) {
    for (int64_t j = (int64_t)blockIdx.x * T + threadIdx.x; j < n4; j += (int64_t)gridDim.x * T) {
        float4 y = p[j];
        y.x = fabsf(y.x) < thr ? 0.f : y.x; y.y = fabsf(y.y) < thr ? 0.f : y.y;
        y.z = fabsf(y.z) < thr ? 0.f : y.z; y.w = fabsf(y.w) < thr ? 0.f : y.w;
        q[j] = y;
    }
}

__device__ __forceinline__ int key_bin(uint32_t key) {
    if (key == 0) return 0;
    const uint32_t e = key >> 23;
    if (e < 101) return 1;
    if (e >= 133) return 4098;
    return 2 + (int)(((e - 101) << 7) | ((key >> 16) & 127));
}

template <int PER, bool MERGE>
__global__ __launch_bounds__(T) void k_hist(const float4* __restrict__ p, int64_t n4, uint32_t* g) {
    __shared__ uint32_t h[4099];
    for (int i = threadIdx.x; i < 4099; i += T) h[i] = 0;
    __syncthreads();
    int64_t base = (int64_t)blockIdx.x * T * PER;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; v[i] = j < n4 ? p[j] : make_float4(0,0,0,0); }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        atomicAdd(&h[key_bin(__float_as_uint(v[i].x) & 0x7fffffff)], 1u);
        atomicAdd(&h[key_bin(__float_as_uint(v[i].y) & 0x7fffffff)], 1u);
        atomicAdd(&h[key_bin(__float_as_uint(v[i].z) & 0x7fffffff)], 1u);
        atomicAdd(&h[key_bin(__float_as_uint(v[i].w) & 0x7fffffff)], 1u);
    }
    __syncthreads();
    if (MERGE) {
        for (int i = threadIdx.x; i < 4099; i += T) { uint32_t c = h[i]; if (c) atomicAdd(&g[i], c); }
    } else {
        if (h[threadIdx.x] == 0xffffffffu) g[0] = 1;
    }
}

// per-wave u16-packed sub-histograms (4 waves x 2050 words = 32.8 KB)
template <int PER, bool MERGE>
__global__ __launch_bounds__(T) void k_hist_w(const float4* __restrict__ p, int64_t n4, uint32_t* g) {
    __shared__ uint32_t h[4][2050];
    for (int i = threadIdx.x; i < 4 * 2050; i += T) (&h[0][0])[i] = 0;
    __syncthreads();
    uint32_t* hw = h[threadIdx.x >> 6];
    int64_t base = (int64_t)blockIdx.x * T * PER;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; v[i] = j < n4 ? p[j] : make_float4(0,0,0,0); }
    auto put = [&](float x) { int b = key_bin(__float_as_uint(x) & 0x7fffffff); atomicAdd(&hw[b >> 1], 1u << ((b & 1) * 16)); };
#pragma unroll
    for (int i = 0; i < PER; ++i) { put(v[i].x); put(v[i].y); put(v[i].z); put(v[i].w); }
    __syncthreads();
    if (MERGE) {
        for (int i = threadIdx.x; i < 2050; i += T) {
            uint32_t a = h[0][i] + h[1][i] + h[2][i] + h[3][i];  // no carry: each half < 65536
            uint32_t lo = (h[0][i] & 0xffff) + (h[1][i] & 0xffff) + (h[2][i] & 0xffff) + (h[3][i] & 0xffff);
            uint32_t hi = (h[0][i] >> 16) + (h[1][i] >> 16) + (h[2][i] >> 16) + (h[3][i] >> 16);
            (void)a;
            if (lo) atomicAdd(&g[2 * i], lo);
            if (hi && 2 * i + 1 < 4099) atomicAdd(&g[2 * i + 1], hi);
        }
    }
}

int main() {
    const int64_t n = 11166912, n4 = n / 4;
    float *x, *y, *o; uint32_t* g;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4)); CK(hipMalloc(&o, 1 << 20)); CK(hipMalloc(&g, 4099 * 4));
    std::vector<float> hx(n);
    uint64_t s = 1; for (int64_t i = 0; i < n; ++i) { s = s * 6364136223846793005ull + 1442695040888963407ull; hx[i] = ((int64_t)(s >> 40) - (1 << 23)) * 0x1p-30f; }
    CK(hipMemcpy(x, hx.data(), n * 4, hipMemcpyHostToDevice));
    float* flush; CK(hipMalloc(&flush, 512 << 20));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto bench = [&](const char* name, auto fn, double bytes) {
        for (int i = 0; i < 5; ++i) fn();
        CK(hipDeviceSynchronize());
        const int R = 200;
        CK(hipEventRecord(a));
        for (int i = 0; i < R; ++i) fn();
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        double us = ms * 1e3 / R;
        // cold: flush the Infinity Cache before each rep
        float tot = 0;
        for (int i = 0; i < 20; ++i) {
            CK(hipMemsetAsync(flush, i, 512 << 20));
            CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
            float m1; CK(hipEventElapsedTime(&m1, a, b)); tot += m1;
        }
        double cus = tot * 1e3 / 20;
        printf("%-28s warm %8.2f us %7.0f GB/s | cold %8.2f us %7.0f GB/s\n", name, us, bytes / us / 1e3, cus, bytes / cus / 1e3);
    };
    const double RB = n * 4.0, CB = n * 8.0;
    bench("read PER=16 (686 blk)", [&]{ hipLaunchKernelGGL(k_read<16>, dim3((n4 + T*16 - 1)/(T*16)), dim3(T), 0, 0, (float4*)x, n4, o); }, RB);
    bench("read PER=4 (2727 blk)", [&]{ hipLaunchKernelGGL(k_read<4>, dim3((n4 + T*4 - 1)/(T*4)), dim3(T), 0, 0, (float4*)x, n4, o); }, RB);
    bench("read PER=8", [&]{ hipLaunchKernelGGL(k_read<8>, dim3((n4 + T*8 - 1)/(T*8)), dim3(T), 0, 0, (float4*)x, n4, o); }, RB);
    bench("read grid-stride 1024", [&]{ hipLaunchKernelGGL(k_read_gs, dim3(1024), dim3(T), 0, 0, (float4*)x, n4, o); }, RB);
    bench("read grid-stride 2048", [&]{ hipLaunchKernelGGL(k_read_gs, dim3(2048), dim3(T), 0, 0, (float4*)x, n4, o); }, RB);
    bench("copy PER=16", [&]{ hipLaunchKernelGGL(k_copy<16>, dim3((n4 + T*16 - 1)/(T*16)), dim3(T), 0, 0, (float4*)x, (float4*)y, n4, 0.01f); }, CB);
    bench("copy PER=4", [&]{ hipLaunchKernelGGL(k_copy<4>, dim3((n4 + T*4 - 1)/(T*4)), dim3(T), 0, 0, (float4*)x, (float4*)y, n4, 0.01f); }, CB);
    bench("copy PER=2", [&]{ hipLaunchKernelGGL(k_copy<2>, dim3((n4 + T*2 - 1)/(T*2)), dim3(T), 0, 0, (float4*)x, (float4*)y, n4, 0.01f); }, CB);
    bench("copy grid-stride 2048", [&]{ hipLaunchKernelGGL(k_copy_gs, dim3(2048), dim3(T), 0, 0, (float4*)x, (float4*)y, n4, 0.01f); }, CB);
    bench("hist PER=16 nomerge", [&]{ hipLaunchKernelGGL((k_hist<16,false>), dim3((n4 + T*16 - 1)/(T*16)), dim3(T), 0, 0, (float4*)x, n4, g); }, RB);
    bench("hist PER=16 merge", [&]{ hipLaunchKernelGGL((k_hist<16,true>), dim3((n4 + T*16 - 1)/(T*16)), dim3(T), 0, 0, (float4*)x, n4, g); }, RB);
    bench("hist PER=4 merge", [&]{ hipLaunchKernelGGL((k_hist<4,true>), dim3((n4 + T*4 - 1)/(T*4)), dim3(T), 0, 0, (float4*)x, n4, g); }, RB);
    bench("hist_w PER=16 nomerge", [&]{ hipLaunchKernelGGL((k_hist_w<16,false>), dim3((n4 + T*16 - 1)/(T*16)), dim3(T), 0, 0, (float4*)x, n4, g); }, RB);
    bench("hist_w PER=16 merge", [&]{ hipLaunchKernelGGL((k_hist_w<16,true>), dim3((n4 + T*16 - 1)/(T*16)), dim3(T), 0, 0, (float4*)x, n4, g); }, RB);
    bench("hist_w PER=32 merge", [&]{ hipLaunchKernelGGL((k_hist_w<32,true>), dim3((n4 + T*32 - 1)/(T*32)), dim3(T), 0, 0, (float4*)x, n4, g); }, RB);
    // empty kernel: launch + dispatch floor
    bench("empty 1 block", [&]{ hipLaunchKernelGGL(k_read<1>, dim3(1), dim3(T), 0, 0, (float4*)x, 0, o); }, 1);
    return 0;
}
