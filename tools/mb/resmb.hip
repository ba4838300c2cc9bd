// Read / copy rates of one-shot register-resident chunk shapes on the cfg2 footprint (44.7 MB):
// how fast can a grid of ~1 workgroup per CU pull its whole chunk into VGPRs?  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int T, int PER, bool COPY>
__global__ __launch_bounds__(T) void k_res(const float4* __restrict__ p, float4* __restrict__ q, int64_t n4, float* out) {
    const int64_t base = (int64_t)blockIdx.x * T * PER;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; v[i] = j < n4 ? p[j] : make_float4(0, 0, 0, 0); }
    if (COPY) {
#pragma unroll
        for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; if (j < n4) q[j] = v[i]; }
    } else {
        float s = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) s += v[i].x + v[i].y + v[i].z + v[i].w;
        if (s == 12345.f) out[blockIdx.x] = s;
    }
}

/* read everything, grid barrier (per-shard arrival counters, sc1 polls), write everything */
__device__ __forceinline__ uint32_t ldc1(const uint32_t* p) { return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <int T, int PER, int MODE>
__global__ __launch_bounds__(T) void k_rbw(const float4* __restrict__ p, float4* __restrict__ q, int64_t n4, uint32_t* bar, uint32_t epoch) {
    const int64_t base = (int64_t)blockIdx.x * T * PER;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; v[i] = j < n4 ? p[j] : make_float4(0, 0, 0, 0); }
    if (MODE >= 1) {
        float s = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) s += v[i].x;
        if (s == 12345.f) q[0] = v[0];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int nblk = gridDim.x;
        if (threadIdx.x == 0) atomicAdd(&bar[(blockIdx.x & 7) * 32], 1u);
        if (threadIdx.x < 64) {
            const int lane = threadIdx.x;
            const uint32_t want = lane < 8 ? epoch * (uint32_t)((nblk - lane + 7) / 8) : 0u;
            while (true) {
                const uint32_t c = lane < 8 ? ldc1(&bar[lane * 32]) : 0u;
                if (__all(c >= want)) break;
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; if (j < n4) q[j] = make_float4(v[i].x * 2.f, v[i].y, v[i].z, v[i].w); }
}

/* read; (SPEC) store everything; a fake dependent chain of `chain_us` (s_sleep + one-lane loads);
 * store everything (no SPEC) or every 5th float4 (SPEC) */
template <int T, int PER, bool SPEC>
__global__ __launch_bounds__(T) void k_rcw(const float4* __restrict__ p, float4* __restrict__ q, int64_t n4, int chain_ticks,
                                           unsigned long long* tout) {
    const int64_t base = (int64_t)blockIdx.x * T * PER;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; v[i] = j < n4 ? p[j] : make_float4(0, 0, 0, 0); }
    float s = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) s += v[i].x;
    if (s == 12345.f) q[0] = v[0];
    if (SPEC) {
#pragma unroll
        for (int i = 0; i < PER; ++i) { int64_t j = base + i * T + threadIdx.x; if (j < n4) q[j] = v[i]; }
    }
    __syncthreads();
    if (threadIdx.x == 0) { /* the dependent chain: wall-clock spin */
        const unsigned long long t0 = wall_clock64();
        while (wall_clock64() - t0 < (unsigned long long)chain_ticks) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        int64_t j = base + i * T + threadIdx.x;
        if (j < n4 && (!SPEC || (i % 5) == 0)) q[j] = make_float4(v[i].x * 2.f, v[i].y, v[i].z, v[i].w);
    }
}

template <int T, int PER, bool SPEC>
void run_rcw(const char* name, const float4* p, float4* q, int64_t n4, int chain_us) {
    const int64_t per_blk = (int64_t)T * PER;
    const int nb = (int)((n4 + per_blk - 1) / per_blk);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int r = 0; r < 30; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_rcw<T, PER, SPEC>), dim3(nb), dim3(T), 0, 0, p, q, n4, chain_us * 100, nullptr);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-34s chain %2d us  %8.2f us\n", name, chain_us, ts[ts.size() / 2]);
}

template <int T, int PER, int MODE>
void run_rbw(const char* name, const float4* p, float4* q, int64_t n4, uint32_t* bar, int reps) {
    const int64_t per_blk = (int64_t)T * PER;
    const int nb = (int)((n4 + per_blk - 1) / per_blk);
    static uint32_t epoch = 0;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> ts;
    CK(hipMemset(bar, 0, 4096)); epoch = 0;
    for (int r = 0; r < reps; ++r) {
        ++epoch;
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_rbw<T, PER, MODE>), dim3(nb), dim3(T), 0, 0, p, q, n4, bar, epoch);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    printf("%-34s blocks %4d  %8.2f us  %7.0f GB/s\n", name, nb, us, 32.0 * n4 / us / 1e3);
}

template <int T, int PER, bool COPY>
void run(const char* name, const float4* p, float4* q, int64_t n4, float* out, int reps) {
    const int64_t per_blk = (int64_t)T * PER;
    const int nb = (int)((n4 + per_blk - 1) / per_blk);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_res<T, PER, COPY>), dim3(nb), dim3(T), 0, 0, p, q, n4, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    const double bytes = (COPY ? 32.0 : 16.0) * n4;
    printf("%-34s blocks %4d  %8.2f us  %7.0f GB/s\n", name, nb, us, bytes / us / 1e3);
}

int main() {
    const int64_t n = 11166912, n4 = n / 4;
    float4 *p, *q; float* out;
    CK(hipMalloc(&p, n * 4)); CK(hipMalloc(&q, n * 4)); CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(p, 0, n * 4));
    uint32_t* bar; CK(hipMalloc(&bar, 4096));
    for (int c : {0, 5, 10, 15}) {
        run_rcw<512, 24, false>("read, chain, store all", p, q, n4, c);
        run_rcw<512, 24, true>("read, spec store, chain, fix 20%", p, q, n4, c);
    }
    for (int k = 0; k < 2; ++k) {
        run_rbw<512, 24, 0>("read-all then write 512x24", p, q, n4, bar, 50);
        run_rbw<512, 24, 1>("read, grid barrier, write 512x24", p, q, n4, bar, 50);
        run_rbw<1024, 12, 1>("read, grid barrier, write 1024x12", p, q, n4, bar, 50);
        run<512, 24, false>("read 512x24 (resident)", p, q, n4, out, 50);
        run<1024, 12, false>("read 1024x12", p, q, n4, out, 50);
        run<256, 48, false>("read 256x48", p, q, n4, out, 50);
        run<256, 16, false>("read 256x16 (k_mask shape)", p, q, n4, out, 50);
        run<256, 8, false>("read 256x8", p, q, n4, out, 50);
        run<512, 24, true>("copy 512x24 (resident)", p, q, n4, out, 50);
        run<1024, 12, true>("copy 1024x12", p, q, n4, out, 50);
        run<256, 16, true>("copy 256x16 (k_mask shape)", p, q, n4, out, 50);
        run<256, 8, true>("copy 256x8", p, q, n4, out, 50);
    }
    return 0;
}
