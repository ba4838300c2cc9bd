// Kernel lab: times each selection kernel of libwtprune in isolation on the cfg2 footprint
// (20 separately allocated ResNet-18 conv tensors), plus reference copy/read kernels.
// Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off lab.hip
#include "../../wavelettransforms_amd/csrc/kernels.hip"
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <vector>
#include <cmath>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace wtp;

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
        load_chunk(p, v);
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
    size_t selb = SEG_PER_LAUNCH * sizeof(SelState);
    SelState* sel; CK(hipMalloc(&sel, selb)); CK(hipMemset(sel, 0, selb));
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
    auto pipeline = [&]{ launch_sample(t, sel, 0); launch_collect(t, sel, cand, 0); launch_select(t, sel, cand, res, thr, 0); launch_mask(t, thr, 0); };
    bench("pipeline (4 kernels)", pipeline, tot * 8.0);
    bench("copy16 contiguous", [&]{ hipLaunchKernelGGL(k_copy16, dim3((tot/4 + 4095)/4096), dim3(256), 0, 0, (float4*)cx, (float4*)cy, tot/4, 0.01f); }, tot * 8.0);
    bench("k_mask", [&]{ launch_mask(t, thr, 0); }, tot * 8.0);
    const int fb = (int)(tot / CHUNK);
#define V(S, G, Z, B, nm) bench(nm, [&]{ hipLaunchKernelGGL((k_maskv<S, G, Z, B>), dim3(S ? t.nblk : fb), dim3(256), 0, 0, t, sel, res, cx, cy, 0.0015f); }, tot * 8.0);
    V(false, false, false, false, "maskv flat")
    V(false, false, true, false, "maskv flat +zc")
    V(true, false, false, false, "maskv seg")
    V(true, false, false, true, "maskv seg blktab")
    V(true, true, false, false, "maskv seg +thrg")
    V(true, true, true, false, "maskv seg +thrg +zc")
    V(true, true, true, true, "maskv seg blktab +thrg +zc")
    bench("k_sample", [&]{ launch_sample(t, sel, 0); }, 0);
    // collect + select must stay paired (select resets the counters)
    bench("k_collect+k_select", [&]{ launch_collect(t, sel, cand, 0); launch_select(t, sel, cand, res, thr, 0); }, tot * 4.0);
    {
        // per-stage times of the real sequence (events between the kernels, queue pre-filled)
        hipEvent_t ev[5]; for (auto& evx : ev) CK(hipEventCreate(&evx));
        float* big; CK(hipMalloc(&big, 256 << 20));
        double acc[4] = {0, 0, 0, 0};
        const int R = 20;
        for (int r = 0; r < R; ++r) {
            CK(hipMemsetAsync(big, r, 256 << 20));
            CK(hipEventRecord(ev[0])); launch_sample(t, sel, 0);
            CK(hipEventRecord(ev[1])); launch_collect(t, sel, cand, 0);
            CK(hipEventRecord(ev[2])); launch_select(t, sel, cand, res, thr, 0);
            CK(hipEventRecord(ev[3])); launch_mask(t, thr, 0);
            CK(hipEventRecord(ev[4])); CK(hipEventSynchronize(ev[4]));
            for (int i = 0; i < 4; ++i) { float ms; CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1])); acc[i] += ms * 1e3; }
        }
        printf("stages (after 256MB memset): sample %.2f collect %.2f select %.2f mask %.2f us\n", acc[0]/R, acc[1]/R, acc[2]/R, acc[3]/R);
        for (int i = 0; i < 4; ++i) acc[i] = 0;
        for (int r = 0; r < R; ++r) {
            hipLaunchKernelGGL(k_copy16, dim3((tot/4 + 4095)/4096), dim3(256), 0, 0, (float4*)cx, (float4*)cy, tot/4, 0.01f);
            CK(hipEventRecord(ev[0])); launch_sample(t, sel, 0);
            CK(hipEventRecord(ev[1])); launch_collect(t, sel, cand, 0);
            CK(hipEventRecord(ev[2])); launch_select(t, sel, cand, res, thr, 0);
            CK(hipEventRecord(ev[3])); launch_mask(t, thr, 0);
            CK(hipEventRecord(ev[4])); CK(hipEventSynchronize(ev[4]));
            for (int i = 0; i < 4; ++i) { float ms; CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1])); acc[i] += ms * 1e3; }
        }
        printf("stages (warm): sample %.2f collect %.2f select %.2f mask %.2f us\n", acc[0]/R, acc[1]/R, acc[2]/R, acc[3]/R);
        std::vector<SelState> hs(20);
        launch_sample(t, sel, 0); launch_collect(t, sel, cand, 0); CK(hipDeviceSynchronize());
        CK(hipMemcpy(hs.data(), sel, 20 * sizeof(SelState), hipMemcpyDeviceToHost));
        for (int i = 0; i < 20; i += 3) { unsigned long long nc = 0, mxb = 0; for (int b = 0; b < NSUB_MAX; ++b) { nc += hs[i].sub[b]; mxb = std::max<unsigned long long>(mxb, hs[i].sub[b]); }
            printf("  seg %2d n %8d below %8llu eql %llu eqh %llu cand %llu maxbucket %llu sh %u ovf %u\n", i, shapes[i], hs[i].below, hs[i].eq_lo, hs[i].eq_hi, nc, mxb, hs[i].shift, hs[i].overflow); }
        launch_select(t, sel, cand, res, thr, 0); CK(hipDeviceSynchronize());
    }
    bench("empty-ish: k_synth 1 elem", [&]{ launch_synth(cx, 1, 0, 0, 30, 0); }, 0);
    // print result info
    std::vector<wtp_result> hr(20);
    pipeline(); CK(hipDeviceSynchronize());
    CK(hipMemcpy(hr.data(), res, 20 * sizeof(wtp_result), hipMemcpyDeviceToHost));
    std::vector<SelState> hs(20);
    CK(hipMemcpy(hs.data(), sel, 20 * sizeof(SelState), hipMemcpyDeviceToHost));
    for (int i = 0; i < 20; i += 4) printf("seg %d zero %lld path %d thr %.9g kl %08x kh %08x\n", i, (long long)hr[i].zero_count, hr[i].path, hr[i].thr64, hs[i].kl, hs[i].kh);
    return 0;
}
