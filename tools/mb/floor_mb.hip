// k_resident schedule lab on the cfg2 footprint (231 chunks of 49 152 floats, 20 segments with
// cfg2's workgroup counts, out of place): what a read -> [count] -> segment barrier -> select
// chain -> write schedule costs when the chain runs in the chunk-holding workgroups (as
// k_resident does) or on workgroups of otherwise idle CUs ("selectors"), with or without the
// decided float4s stored before the chain.  The chain is modelled by its dependent device reads
// (4 KB totals, 96 offsets, 264 keys, all sc1) and a 1.25 us LDS select (wall-clock spin).
// Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 floor_mb.hip -o floor_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int CT = 512, IT = 24, CHUNK = CT * IT * 4;
constexpr int NSEG = 20;
__constant__ int c_wgs[NSEG] = {1, 1, 1, 1, 1, 1, 2, 3, 3, 3, 1, 6, 12, 12, 12, 3, 24, 48, 48, 48};
constexpr uint64_t TMO = 2000000; /* 20 ms of the 100 MHz clock */

enum { SPEC = 1, REMOTE = 2, NOCHAIN = 4, COPY = 8, NOPUB = 16, SPECALL = 32, SAMPLE = 64, READONLY = 128 };

__device__ __forceinline__ uint32_t ldc(const uint32_t* p) { return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void stc(uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint64_t ticks() { return __builtin_amdgcn_s_memrealtime(); }

struct Ws {
    uint32_t bar[NSEG][32];   /* segment arrival counters (monotonic: epoch * nwg) */
    uint32_t flag[NSEG][32];  /* selector -> segment: the threshold granule (epoch) */
    uint32_t tot[NSEG][1024]; /* bucket totals */
    uint32_t err;
};

/* a lane-0 poll of a monotonic counter, bounded */
__device__ bool poll_ge(const uint32_t* p, uint32_t want, uint32_t* err) {
    __shared__ int ok;
    if (threadIdx.x == 0) {
        const uint64_t t0 = ticks();
        int o = 1;
        while (ldc(p) < want) {
            if (ticks() - t0 > TMO) { o = 0; atomicAdd(err, 1u); break; }
            __builtin_amdgcn_s_sleep(2);
        }
        ok = o;
    }
    __syncthreads();
    return ok;
}

/* the select chain: three dependent device reads of lines other CUs have just written (the
 * segment's atomic bucket totals, then its workgroups' sc1 publications: 2 offsets each, then
 * 264 keys), then the LDS select (a spin) */
__device__ uint32_t chain(const uint32_t* tot, const uint32_t* pub, int b0, int nwg, uint32_t* lds) {
    const int tid = threadIdx.x, lane = tid & 63;
    uint32_t a = ldc(tot + 2 * tid) + ldc(tot + 2 * tid + 1); /* 4 KB: the totals */
    lds[tid] = a;
    __syncthreads();
    uint32_t s = 0;
    if (tid < 64) {
        for (int i = 0; i < 8; ++i) s += lds[lane * 8 + i];
        s = __builtin_amdgcn_readfirstlane(s) & 0x10000u; /* 0 in practice, but a dependence */
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t* pw = pub + (int64_t)(b0 + lane % nwg) * 512;
        lds[600 + lane] = ldc(pw + s + (lane & 7)) + ldc(pw + s + 8 + (lane & 7)); /* offsets */
    }
    __syncthreads();
    const uint32_t o = lds[600] & 0x10000u;
    uint32_t k = tid < 264 ? ldc(pub + (int64_t)(b0 + tid % nwg) * 512 + o + tid / nwg) : 0u; /* the keys */
    lds[tid] = k;
    __syncthreads();
    if (tid == 0) {
        const uint64_t t0 = ticks();
        while (ticks() - t0 < 125) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
    return lds[0] & 0x10000u;
}

__global__ __launch_bounds__(CT) void k_sched(const float* __restrict__ x, float* __restrict__ y, Ws* ws,
                                              const uint32_t* __restrict__ tbl, uint32_t* __restrict__ pub, int mode,
                                              uint32_t epoch, int nchunks, unsigned long long* stamps) {
    extern __shared__ uint32_t lds[]; /* >= 96 KB: one workgroup per CU */
    const int tid = threadIdx.x;
    if (tid == 0) atomicMin(stamps, ticks());
    /* the segment and the workgroup's rank in it */
    int seg = 0, b0 = 0;
    const int b = blockIdx.x;
    if (b < nchunks) {
        while (b >= b0 + c_wgs[seg]) { b0 += c_wgs[seg]; ++seg; }
    }
    const bool selector = b >= nchunks;
    const int nwg = selector ? 0 : c_wgs[seg];
    if (selector) {
        /* selector of the multi-workgroup segment number (b - nchunks) */
        int m = b - nchunks, s = 0, sb = 0;
        for (; s < NSEG; ++s) { if (c_wgs[s] > 1 && m-- == 0) break; sb += c_wgs[s]; }
        if (!(mode & REMOTE) || s >= NSEG) return;
        if (poll_ge(&ws->bar[s][0], epoch * c_wgs[s], &ws->err)) {
            chain(&ws->tot[s][0], pub, sb, c_wgs[s], lds);
            if (tid == 0) stc(&ws->flag[s][0], epoch);
        }
        if (tid == 0) atomicMax(stamps + 1, ticks());
        return;
    }
    const float4* x4 = reinterpret_cast<const float4*>(x + (int64_t)b * CHUNK);
    float4* y4 = reinterpret_cast<float4*>(y + (int64_t)b * CHUNK);
    float4 v[IT];
    uint32_t smp = 0;
    if ((mode & SAMPLE) && tid < 256) {
        /* k_resident's sample: 16 loads a lane, groups of 16 contiguous floats spread over the
         * segment, issued ahead of the chunk */
        const float* sx = x + (int64_t)b0 * CHUNK;
        const int64_t n = (int64_t)nwg * CHUNK;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = j * 256 + tid;
            const int64_t pos = (int64_t)(i / 16) * ((n - 16) / 255) + (i % 16);
            smp += __float_as_uint(sx[pos]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < IT; ++it) v[it] = x4[it * CT + tid];
    if (mode & READONLY) {
        float sacc = 0.f;
#pragma unroll
        for (int it = 0; it < IT; ++it) sacc += v[it].x + v[it].y + v[it].z + v[it].w;
        if (sacc == 1234.5f + (float)smp) y[tid] = sacc;
    } else if (mode & COPY) {
#pragma unroll
        for (int it = 0; it < IT; ++it) y4[it * CT + tid] = v[it];
    } else {
        /* the count pass: max key, keys below a bound, each key into the thread's LDS column */
        uint32_t mx = 0, below = 0, cnt = 0;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const uint32_t k4[4] = {__float_as_uint(v[it].x) & 0x7fffffffu, __float_as_uint(v[it].y) & 0x7fffffffu,
                                    __float_as_uint(v[it].z) & 0x7fffffffu, __float_as_uint(v[it].w) & 0x7fffffffu};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                mx = max(mx, k4[c]);
                below += k4[c] < 0x3c000000u;
                lds[min(cnt, 30u) * CT + tid] = k4[c];
                cnt += (k4[c] >> 20) == 0x3c0u;
            }
        }
        __syncthreads();
        if (nwg > 1) {
            if (!(mode & NOPUB)) {
                /* the bucket totals (no-return atomics) and a 2 KB sc1 publication */
                for (int j = tid; j < 1024; j += CT) atomicAdd(&ws->tot[seg][j], lds[j] & 1u);
                stc(pub + (int64_t)b * 512 + tid, lds[tid] + below);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) atomicAdd(&ws->bar[seg][0], 1u);
        }
        uint32_t mk = mx;
        /* decided float4s go out before the chain (SPEC: 18 of 24; SPECALL: all) */
        if (mode & (SPEC | SPECALL)) {
#pragma unroll
            for (int it = 0; it < IT; ++it)
                if ((mode & SPECALL) || (it & 3) != 0) y4[it * CT + tid] = v[it];
        }
        if (nwg == 1) {
            if (tid == 0) { const uint64_t t0 = ticks(); while (ticks() - t0 < 250) __builtin_amdgcn_s_sleep(1); }
            __syncthreads();
        } else if (!(mode & NOCHAIN)) {
            if (mode & REMOTE) {
                poll_ge(&ws->flag[seg][0], epoch, &ws->err);
            } else if (poll_ge(&ws->bar[seg][0], epoch * nwg, &ws->err)) {
                mk += chain(&ws->tot[seg][0], pub, b0, nwg, lds);
            }
        } else {
            poll_ge(&ws->bar[seg][0], epoch * nwg, &ws->err);
        }
        const float t = __uint_as_float(mk & 1u);
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            if ((mode & SPECALL) || ((mode & SPEC) && (it & 3) != 0)) continue;
            float4 o = v[it];
            o.x = fabsf(o.x) < t ? 0.f : o.x;
            y4[it * CT + tid] = o;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) atomicMax(stamps + 1, ticks());
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    int nchunks = 0, nmulti = 0;
    const int wgs[NSEG] = {1, 1, 1, 1, 1, 1, 2, 3, 3, 3, 1, 6, 12, 12, 12, 3, 24, 48, 48, 48};
    for (int s = 0; s < NSEG; ++s) { nchunks += wgs[s]; nmulti += wgs[s] > 1; }
    const int64_t n = (int64_t)nchunks * CHUNK;
    float *x, *y;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4));
    std::vector<float> h(n);
    for (int64_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000003) * 1e-7f - 0.05f;
    CK(hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice));
    Ws* ws; CK(hipMalloc(&ws, sizeof(Ws))); CK(hipMemset(ws, 0, sizeof(Ws)));
    uint32_t *tbl, *pub; CK(hipMalloc(&tbl, 64 << 10)); CK(hipMemset(tbl, 0, 64 << 10));
    CK(hipMalloc(&pub, (size_t)nchunks * 512 * 4));
    unsigned long long* st; CK(hipMalloc(&st, (size_t)reps * 16));
    const size_t lds = 100 << 10;
    CK(hipFuncSetAttribute((const void*)k_sched, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    uint32_t epoch = 0;
    struct V { const char* name; int mode; };
    const V vs[] = {{"read only", READONLY},
                    {"read only, sample first", READONLY | SAMPLE},
                    {"copy (no barrier)", COPY},
                    {"copy, sample first", COPY | SAMPLE},
                    {"read, barrier, write, sample first", NOCHAIN | NOPUB | SAMPLE},
                    {"read, barrier, write (no chain)", NOCHAIN | NOPUB},
                    {"read, pub, barrier, write", NOCHAIN},
                    {"local chain (k_resident form)", 0},
                    {"local chain, 18/24 stored ahead", SPEC},
                    {"remote chain", REMOTE},
                    {"remote chain, 18/24 stored ahead", REMOTE | SPEC},
                    {"remote chain, all stored ahead", REMOTE | SPECALL},
                    {"local chain, all stored ahead", SPECALL}};
    for (int pass = 0; pass < 2; ++pass) {
        for (const V& vv : vs) {
            const int grid = nchunks + ((vv.mode & REMOTE) ? nmulti : 0);
            std::vector<unsigned long long> hs(2 * reps);
            for (int r = 0; r < reps; ++r) { hs[2 * r] = ~0ull; hs[2 * r + 1] = 0; }
            CK(hipMemcpy(st, hs.data(), reps * 16, hipMemcpyHostToDevice));
            hipEvent_t a, ev; CK(hipEventCreate(&a)); CK(hipEventCreate(&ev));
            CK(hipMemset(ws, 0, sizeof(Ws)));
            epoch = 0;
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < reps; ++r) {
                ++epoch;
                hipLaunchKernelGGL(k_sched, dim3(grid), dim3(CT), lds, 0, x, y, ws, tbl, pub, vv.mode, epoch, nchunks, st + 2 * r);
            }
            CK(hipEventRecord(ev));
            CK(hipEventSynchronize(ev));
            float ms; CK(hipEventElapsedTime(&ms, a, ev));
            CK(hipMemcpy(hs.data(), st, reps * 16, hipMemcpyDeviceToHost));
            std::vector<double> sp;
            for (int r = 0; r < reps; ++r) sp.push_back((double)(hs[2 * r + 1] - hs[2 * r]) * 0.01);
            std::sort(sp.begin(), sp.end());
            uint32_t err = 0; CK(hipMemcpy(&err, &ws->err, 4, hipMemcpyDeviceToHost));
            printf("%-36s grid %3d  span p10 %6.2f p50 %6.2f p90 %6.2f us   per launch %6.2f us  %s\n", vv.name, grid,
                   sp[reps / 10], sp[reps / 2], sp[reps * 9 / 10], ms * 1e3 / reps, err ? "TIMEOUTS" : "");
            if (err) return 1;
        }
    }
    return 0;
}
