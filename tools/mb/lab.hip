// Kernel lab: times each selection kernel of libwtprune in isolation on the cfg2 footprint
// (20 separately allocated ResNet-18 conv tensors), plus reference copy/read kernels.
// Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off lab.hip
#include <hip/hip_runtime.h>
__device__ unsigned long long g_probe[24][8];
#define WTP_PROBE(i) do { if (threadIdx.x == 0 && blockIdx.x < 24) g_probe[blockIdx.x][i] = wall_clock64(); } while (0)
__device__ unsigned long long g_cprobe[1024][8];
#define WTP_CPROBE(i) do { if (threadIdx.x == 0 && blockIdx.x < 1024) g_cprobe[blockIdx.x][i] = wall_clock64(); } while (0)
#include "../../wavelettransforms_amd/csrc/kernels.hip"
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <vector>
#include <cmath>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace wtp;

__global__ void k_dpp_test(const uint32_t* in, uint32_t* scan, uint32_t* mx, unsigned long long* sum64) {
    const uint32_t v = in[blockIdx.x * 256 + threadIdx.x];
    scan[blockIdx.x * 256 + threadIdx.x] = wave_scan_u32(v);
    mx[blockIdx.x * 256 + threadIdx.x] = wave_max_u32(v);
    sum64[blockIdx.x * 256 + threadIdx.x] = wave_sum_u64(((unsigned long long)v << 20) ^ v);
}

__global__ void k_ragged_test(const float* p, int len, float* out) {
    float4 v[16];
    load_chunk_ragged<16>(p, len, v);
    for (int it = 0; it < 16; ++it) reinterpret_cast<float4*>(out)[it * 256 + threadIdx.x] = v[it];
}

__global__ void k_copy16(const float4* __restrict__ p, float4* __restrict__ q, int64_t n4, float thr) {
    int64_t base = (int64_t)blockIdx.x * 256 * 16;
    float4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { int64_t j = base + i * 256 + threadIdx.x; if (j < n4) v[i] = p[j]; }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int64_t j = base + i * 256 + threadIdx.x;
        float4 y = v[i];
        y.x = fabsf(y.x) < thr ? 0.f : y.x; y.y = fabsf(y.y) < thr ? 0.f : y.y;
        y.z = fabsf(y.z) < thr ? 0.f : y.z; y.w = fabsf(y.w) < thr ? 0.f : y.w;
        if (j < n4) q[j] = y;
    }
}

// k_mask variants: SEG = find_seg over the SegTable (else: one flat buffer), THRG = threshold
// read from SelState in global memory (else: kernel argument), ZC = zero count reduction.
template <bool SEG, bool THRG, bool ZC, bool BLKTAB>
__global__ __launch_bounds__(256) void k_maskv(SegTable t, const SelState* __restrict__ sel, wtp_result* res,
                                                const float* flatp, float* flatq, float thr_arg) {
    const float* p;
    float* q;
    int64_t len;
    int si = 0;
    if (SEG) {
        if (BLKTAB) {
            si = 0;
#pragma unroll
            for (int i = 1; i < 20; ++i) si += (int)blockIdx.x >= t.s[i].blk_begin;
        } else {
            si = find_seg(t, blockIdx.x);
        }
        const SegDesc& sd = t.s[si];
        const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
        len = min((int64_t)CHUNK, sd.n - base);
        p = sd.data + base;
        q = sd.out + base;
    } else {
        p = flatp + (int64_t)blockIdx.x * CHUNK;
        q = flatq + (int64_t)blockIdx.x * CHUNK;
        len = CHUNK;
    }
    float thr = thr_arg;
    if (THRG) thr = sel[t.s[si].slot].thr32;
    unsigned long long z = 0;
    auto f = [&](float x) { const float y = (fabsf(x) < thr) ? 0.0f : x; z += (y == 0.0f); return y; };
    if (len == CHUNK) {
        float4 v[16];
        load_chunk<16>(p, v);
        float4* q4 = reinterpret_cast<float4*>(q);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            float4 y; y.x = f(v[it].x); y.y = f(v[it].y); y.z = f(v[it].z); y.w = f(v[it].w);
            q4[it * STREAM_THREADS + threadIdx.x] = y;
        }
    } else {
        for (int64_t i = threadIdx.x; i < len; i += STREAM_THREADS) q[i] = f(p[i]);
    }
    if (ZC) {
        const unsigned long long tot = block_sum_u64<STREAM_THREADS>(z);
        if (threadIdx.x == 0 && tot) atomicAdd((unsigned long long*)&res[t.s[si].res].zero_count, tot);
    } else if (z == 123456789ull) res[0].numel = 1;
}

int main() {
    {   // DPP wave primitives vs serial
        const int N = 4096;
        std::vector<uint32_t> h(N); uint64_t z = 88172645463325252ull;
        for (auto& v : h) { z ^= z << 13; z ^= z >> 7; z ^= z << 17; v = (uint32_t)(z >> ((z & 3) * 8)); }
        uint32_t *din, *dsc, *dmx; unsigned long long* ds64;
        CK(hipMalloc(&din, N * 4)); CK(hipMalloc(&dsc, N * 4)); CK(hipMalloc(&dmx, N * 4)); CK(hipMalloc(&ds64, N * 8));
        CK(hipMemcpy(din, h.data(), N * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_dpp_test, dim3(N / 256), dim3(256), 0, 0, din, dsc, dmx, ds64);
        std::vector<uint32_t> sc(N), mx(N); std::vector<unsigned long long> s64(N);
        CK(hipMemcpy(sc.data(), dsc, N * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(mx.data(), dmx, N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(s64.data(), ds64, N * 8, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int w = 0; w < N / 64; ++w) {
            uint32_t acc = 0, m = 0; unsigned long long a64 = 0;
            for (int l = 0; l < 64; ++l) { m = std::max(m, h[w * 64 + l]); a64 += ((unsigned long long)h[w * 64 + l] << 20) ^ h[w * 64 + l]; }
            for (int l = 0; l < 64; ++l) { acc += h[w * 64 + l]; bad += sc[w * 64 + l] != acc; bad += mx[w * 64 + l] != m; bad += s64[w * 64 + l] != a64; }
        }
        printf("DPP primitives: %d mismatches\n", bad);
        if (bad) return 1;
        // ragged buffer loads: values below len, zeros past it, for every len % 4
        float *src, *dst; CK(hipMalloc(&src, 16384 * 4 + 64)); CK(hipMalloc(&dst, 16384 * 4));
        std::vector<float> hsrc(16384 + 16); for (int i = 0; i < (int)hsrc.size(); ++i) hsrc[i] = 1.0f + i;
        CK(hipMemcpy(src, hsrc.data(), hsrc.size() * 4, hipMemcpyHostToDevice));
        int rbad = 0;
        for (int len : {1, 2, 3, 4, 5, 6, 7, 1001, 4097, 9407, 16383}) {
            hipLaunchKernelGGL(k_ragged_test, dim3(1), dim3(256), 0, 0, src + 3, len, dst);
            std::vector<float> hd(16384); CK(hipMemcpy(hd.data(), dst, 16384 * 4, hipMemcpyDeviceToHost));
            for (int i = 0; i < 16384; ++i) rbad += hd[i] != (i < len ? hsrc[i + 3] : 0.0f);
        }
        printf("ragged buffer loads: %d mismatches\n", rbad);
        if (rbad) return 1;
    }

    const int shapes[20] = {9408, 36864, 36864, 36864, 36864, 8192, 73728, 147456, 147456, 147456, 32768, 294912,
                            589824, 589824, 589824, 131072, 1179648, 2359296, 2359296, 2359296};
    std::vector<float*> xs(20), ys(20);
    int64_t tot = 0;
    for (int i = 0; i < 20; ++i) {
        CK(hipMalloc(&xs[i], shapes[i] * 4)); CK(hipMalloc(&ys[i], shapes[i] * 4));
        launch_synth(xs[i], shapes[i], 0, i, 30, 0); tot += shapes[i];
    }
    float *cx, *cy; CK(hipMalloc(&cx, tot * 4)); CK(hipMalloc(&cy, tot * 4));
    launch_synth(cx, tot, 0, 0, 30, 0);
    const size_t headb = sizeof(SelHeader) + 2 * SEL_REGION;
    SelHeader* head; CK(hipMalloc(&head, headb)); CK(hipMemset(head, 0, headb));
    uint32_t* cand; CK(hipMalloc(&cand, tot * 4));
    wtp_result* res; CK(hipMalloc(&res, 20 * sizeof(wtp_result)));
    float* thr; CK(hipMalloc(&thr, 20 * 4));
    SegTable t; memset(&t, 0, sizeof t);
    int blk = 0; int64_t coff = 0;
    for (int i = 0; i < 20; ++i) {
        SegDesc& sd = t.s[t.nseg++];
        sd.data = xs[i]; sd.out = ys[i]; sd.n = shapes[i]; sd.numel = shapes[i];
        double vi = (shapes[i] - 1) * 0.5; sd.r0 = (int64_t)floor(vi); sd.gamma = vi - floor(vi);
        sd.blk_begin = blk; t.blk_begin[i] = blk; sd.slot = i; sd.res = i; sd.flags = SEG_MASK | SEG_ALIGNED;
        { double ex = 0.05 * shapes[i]; int lg = 6; while (lg < 10 && (double)(1 << lg) * 1024.0 < ex) ++lg;
          int64_t bc = (int64_t)(4.0 * ex / (1 << lg)) + 1; bc = std::min<int64_t>(8192, std::max<int64_t>(256, bc));
          sd.nsub_log2 = lg; sd.bucket_cap = (int)bc; sd.cap = bc << lg; }
        sd.cand_off = coff; coff += sd.cap;
        blk += (shapes[i] + CHUNK - 1) / CHUNK;
    }
    t.nblk = blk;
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto bench = [&](const char* name, auto fn, double bytes) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipDeviceSynchronize());
        const int R = 100;
        CK(hipEventRecord(a));
        for (int i = 0; i < R; ++i) fn();
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        double us = ms * 1e3 / R;
        printf("%-34s %8.2f us  %7.0f GB/s\n", name, us, bytes / us / 1e3);
    };
    // full pipeline once to get state
    for (int i = t.nseg; i < SEG_PER_LAUNCH; ++i) t.blk_begin[i] = INT32_MAX;
    auto pipeline = [&]{ launch_collect(t, head, cand, res, 0); launch_mask_select(t, head, cand, res, thr, 0); };
    bench("pipeline (collect + mask_select)", pipeline, tot * 8.0);
    bench("copy16 contiguous", [&]{ hipLaunchKernelGGL(k_copy16, dim3((tot/4 + 4095)/4096), dim3(256), 0, 0, (float4*)cx, (float4*)cy, tot/4, 0.01f); }, tot * 8.0);
    bench("k_collect alone", [&]{ launch_collect(t, head, cand, res, 0); }, tot * 4.0);
    bench("k_window alone", [&]{ hipLaunchKernelGGL(k_window, dim3(t.nseg), dim3(WIN_THREADS), 0, 0, t, head); }, 0);
    bench("pipeline inline window", [&]{ hipLaunchKernelGGL((k_collect_t<0, 256, 16, true>), dim3(t.nblk), dim3(256), 0, 0, t, head, cand, res);
                                         launch_mask_select(t, head, cand, res, thr, 0); }, tot * 8.0);
    bench("pipeline k_window + collect", [&]{ hipLaunchKernelGGL(k_window, dim3(t.nseg), dim3(WIN_THREADS), 0, 0, t, head);
                                              hipLaunchKernelGGL((k_collect_t<0, 256, 16, false>), dim3(t.nblk), dim3(256), 0, 0, t, head, cand, res);
                                              launch_mask_select(t, head, cand, res, thr, 0); }, tot * 8.0);
    {   // collect block shapes (window from k_window): pipeline time and results vs production
        std::vector<wtp_result> r0(20), r1(20);
        pipeline(); CK(hipDeviceSynchronize());
        CK(hipMemcpy(r0.data(), res, 20 * sizeof(wtp_result), hipMemcpyDeviceToHost));
        auto run_shape = [&](const char* nm, auto kc) {
            auto pipe = [&] { hipLaunchKernelGGL(k_window, dim3(t.nseg), dim3(WIN_THREADS), 0, 0, t, head); kc();
                              launch_mask_select(t, head, cand, res, thr, 0); };
            bench(nm, pipe, tot * 8.0);
            pipe(); CK(hipDeviceSynchronize());
            CK(hipMemcpy(r1.data(), res, 20 * sizeof(wtp_result), hipMemcpyDeviceToHost));
            int bad = 0; for (int i = 0; i < 20; ++i) bad += r0[i].thr64 != r1[i].thr64 || r0[i].zero_count != r1[i].zero_count || r1[i].path == 3;
            printf("    mismatches/fallbacks vs production %d\n", bad);
        };
        run_shape("pipe collect CT256 IT16", [&] { hipLaunchKernelGGL((k_collect_t<0, 256, 16, false>), dim3(t.nblk), dim3(256), 0, 0, t, head, cand, res); });
        run_shape("pipe collect CT256 IT8", [&] { hipLaunchKernelGGL((k_collect_t<0, 256, 8, false>), dim3(t.nblk * 2), dim3(256), 0, 0, t, head, cand, res); });
        run_shape("pipe collect CT256 IT4", [&] { hipLaunchKernelGGL((k_collect_t<0, 256, 4, false>), dim3(t.nblk * 4), dim3(256), 0, 0, t, head, cand, res); });
        run_shape("pipe collect CT512 IT8", [&] { hipLaunchKernelGGL((k_collect_t<0, 512, 8, false>), dim3(t.nblk), dim3(512), 0, 0, t, head, cand, res); });
        run_shape("pipe collect CT128 IT16", [&] { hipLaunchKernelGGL((k_collect_t<0, 128, 16, false>), dim3(t.nblk * 2), dim3(128), 0, 0, t, head, cand, res); });
        run_shape("pipe collect CT1024 IT4", [&] { hipLaunchKernelGGL((k_collect_t<0, 1024, 4, false>), dim3(t.nblk), dim3(1024), 0, 0, t, head, cand, res); });
    }
    bench("collect LAB1 counters only", [&]{ hipLaunchKernelGGL((k_collect_t<1, 256, 16, COLLECT_WINDOW_INLINE>), dim3(t.nblk), dim3(256), 0, 0, t, head, cand, res); }, tot * 4.0);
    bench("collect LAB2 +staging", [&]{ hipLaunchKernelGGL((k_collect_t<2, 256, 16, COLLECT_WINDOW_INLINE>), dim3(t.nblk), dim3(256), 0, 0, t, head, cand, res); }, tot * 4.0);
    {
        // per-stage times of the real sequence (events between the kernels)
        hipEvent_t ev[3]; for (auto& evx : ev) CK(hipEventCreate(&evx));
        float* big; CK(hipMalloc(&big, 256 << 20));
        for (int mode = 0; mode < 2; ++mode) {
            double acc[2] = {0, 0};
            const int R = 20;
            for (int r = 0; r < R; ++r) {
                if (mode == 0) CK(hipMemsetAsync(big, r, 256 << 20));
                else hipLaunchKernelGGL(k_copy16, dim3((tot/4 + 4095)/4096), dim3(256), 0, 0, (float4*)cx, (float4*)cy, tot/4, 0.01f);
                CK(hipEventRecord(ev[0])); launch_collect(t, head, cand, res, 0);
                CK(hipEventRecord(ev[1])); launch_mask_select(t, head, cand, res, thr, 0);
                CK(hipEventRecord(ev[2])); CK(hipEventSynchronize(ev[2]));
                for (int i = 0; i < 2; ++i) { float ms; CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1])); acc[i] += ms * 1e3; }
            }
            printf("stages (%s): collect %.2f mask_select %.2f us\n", mode ? "warm" : "after 256MB memset", acc[0]/R, acc[1]/R);
        }
    }
    {   // collect phase timeline (100 MHz wall clock): per-phase distribution over blocks
        unsigned long long zero[1024][8] = {}; CK(hipMemcpyToSymbol(HIP_SYMBOL(g_cprobe), zero, sizeof(zero)));
        launch_collect(t, head, cand, res, 0); CK(hipDeviceSynchronize());
        static unsigned long long cp[1024][8];
        CK(hipMemcpyFromSymbol(cp, HIP_SYMBOL(g_cprobe), sizeof(cp)));
        const int nb = std::min(t.nblk, 1024);
        unsigned long long t0 = ~0ull, tend = 0; for (int b = 0; b < nb; ++b) { t0 = std::min(t0, cp[b][0]); tend = std::max(tend, cp[b][5]); }
        printf("  collect span (first start -> last end) %.2f us over %d blocks\n", (tend - t0) / 100.0, nb);
        std::vector<double> d[5];
        for (int b = 0; b < nb; ++b) for (int k = 0; k < 5; ++k) if (cp[b][k] && cp[b][k + 1]) d[k].push_back((cp[b][k + 1] - cp[b][k]) / 100.0);
        for (int k = 0; k < 5; ++k) { auto& v = d[k]; if (v.empty()) continue; std::sort(v.begin(), v.end());
            printf("  phase %d->%d: p50 %5.2f  p90 %5.2f  max %5.2f us\n", k, k + 1, v[v.size() / 2], v[v.size() * 9 / 10], v.back()); }
        // select timeline inside k_mask_select (blocks 0..23)
        launch_mask_select(t, head, cand, res, thr, 0); CK(hipDeviceSynchronize());
        unsigned long long hp[24][8];
        CK(hipMemcpyFromSymbol(hp, HIP_SYMBOL(g_probe), sizeof(hp)));
        for (int i = 0; i < 24; i += 4) { printf("  mask_select blk %2d select phases (us from its start):", i);
            for (int k = 1; k < 7; ++k) printf(" %6.2f", hp[i][k] ? (double)(hp[i][k] - hp[i][0]) / 100.0 : -1.0); printf("\n"); }
    }
    // print result info
    std::vector<wtp_result> hr(20);
    pipeline(); CK(hipDeviceSynchronize());
    CK(hipMemcpy(hr.data(), res, 20 * sizeof(wtp_result), hipMemcpyDeviceToHost));
    for (int i = 0; i < 20; i += 4) printf("seg %d zero %lld path %d thr %.9g\n", i, (long long)hr[i].zero_count, hr[i].path, hr[i].thr64);
    return 0;
}
