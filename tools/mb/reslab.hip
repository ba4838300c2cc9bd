// k_resident phase lab: the cfg2 footprint (20 ResNet-18 conv tensors, synthetic) through the
// real API (wtp_prune_layers_f32) with per-workgroup wall-clock probes at the phase boundaries
// of k_resident (WTP_RPROBE).  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off reslab.hip -o reslab
#include <hip/hip_runtime.h>
#define NWG 256
__device__ unsigned long long g_rprobe[NWG][20];
__device__ unsigned long long g_cyc[NWG][2];
__device__ unsigned long long g_sprobe[NWG][16];
#ifndef RESLAB_NOPROBE
#define WTP_RPROBE(i) do { if (threadIdx.x == 0) { g_rprobe[blockIdx.x][i] = wall_clock64(); \
    if ((i) == 0) g_cyc[blockIdx.x][0] = __builtin_amdgcn_s_memtime(); \
    if ((i) == 7) g_cyc[blockIdx.x][1] = __builtin_amdgcn_s_memtime(); } } while (0)
#define WTP_PROBE(i) do { if (threadIdx.x == 0) g_sprobe[blockIdx.x][i] = wall_clock64(); } while (0)
#define WTP_PROBE_T(i, t) do { if (threadIdx.x == (t)) g_sprobe[blockIdx.x][i] = wall_clock64(); } while (0)
#define WTP_WPROBE(i) WTP_RPROBE(12 + (i))
#define WTP_RTAG(tagv) do { if (threadIdx.x == 0) g_rprobe[blockIdx.x][19] = (unsigned long long)(tagv); } while (0)
#endif
#include "kernels.hip"  /* -I wavelettransforms_amd/csrc (or a variant copy) */
#include "filterbank.hip"  /* -I wavelettransforms_amd/csrc (or a variant copy) */
#include "small.hip"  /* -I wavelettransforms_amd/csrc (or a variant copy) */
#include "api.hip"  /* -I wavelettransforms_amd/csrc (or a variant copy) */
#include <cstdio>
#include <vector>
#include <algorithm>
/* cold-cache flushes between reps (argv[3]): 0 none (warm), 1 write 512 MiB (the bench's cold leg:
 * the Infinity Cache then holds dirty lines of another buffer), 2 read 512 MiB (clean lines of another
 * buffer), 3 write then read two other 512 MiB buffers (dirty lines written back before the call) */
__global__ void k_flush_read(const float4* __restrict__ p, size_t n4, float* __restrict__ sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i]; /* plain loads: they allocate in the Infinity Cache */
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) sink[0] = acc;
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    const int flush = argc > 3 ? atoi(argv[3]) : 0;
    const int64_t shapes[20][4] = {{64,3,7,7},{64,64,3,3},{64,64,3,3},{64,64,3,3},{64,64,3,3},{128,64,1,1},{128,64,3,3},
        {128,128,3,3},{128,128,3,3},{128,128,3,3},{256,128,1,1},{256,128,3,3},{256,256,3,3},{256,256,3,3},{256,256,3,3},
        {512,256,1,1},{512,256,3,3},{512,512,3,3},{512,512,3,3},{512,512,3,3}};
    std::vector<wtp_tensor> ts(20);
    int64_t nw = 0;
    for (int t = 0; t < 20; ++t) {
        memset(&ts[t], 0, sizeof ts[t]);
        int64_t n = 1;
        ts[t].ndim = 4;
        for (int d = 0; d < 4; ++d) { ts[t].shape[d] = shapes[t][d]; n *= shapes[t][d]; }
        float *x, *y;
        CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4));
        const double sig = sqrt(2.0 / (double)(shapes[t][0] * shapes[t][2] * shapes[t][3]));
        const int e = (int)std::lround(23 - std::log2(sig)); // ~kaiming scale
        wtp_synth_f32(x, n, t, t, e, 0);
        ts[t].in = x; ts[t].out = y;
        nw += n;
    }
    const int wid = wtp_wavelet_id("bior3.3");
    size_t wsb = wtp_workspace_size(ts.data(), 20, wid, 5);
    void* ws; CK(hipMalloc(&ws, wsb)); wtp_workspace_init(ws, wsb, 0);
    wtp_result* res; CK(hipMalloc(&res, 20 * sizeof(wtp_result)));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) if (wtp_prune_layers_f32(ts.data(), 20, wid, 5, 50.0, ws, wsb, res, 0)) { printf("err %s\n", wtp_last_error()); return 1; }
    CK(hipDeviceSynchronize());
    std::vector<float> tms;
    static unsigned long long pr[NWG][20];
    std::vector<std::vector<double>> ph(18), sel(15), phg[2];
    phg[0].resize(18); phg[1].resize(18);
    const size_t FL = (size_t)512 << 20;
    float *fw = nullptr, *fr = nullptr, *sink = nullptr;
    if (flush) { CK(hipMalloc(&fw, FL)); CK(hipMalloc(&fr, FL)); CK(hipMalloc(&sink, 64)); CK(hipMemset(fr, 0, FL)); }
    for (int r = 0; r < reps; ++r) {
        if (flush == 1 || flush == 3) CK(hipMemsetAsync(fw, r & 0xff, FL, 0));
        if (flush == 2 || flush == 3) hipLaunchKernelGGL(k_flush_read, dim3(4096), dim3(256), 0, 0, (const float4*)fr, FL / 16, sink);
        CK(hipEventRecord(a, 0));
        wtp_prune_layers_f32(ts.data(), 20, wid, 5, 50.0, ws, wsb, res, 0);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); tms.push_back(ms * 1000);
        CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_rprobe), sizeof pr));
        static unsigned long long sp[NWG][16];
        CK(hipMemcpyFromSymbol(sp, HIP_SYMBOL(g_sprobe), sizeof sp));
        int nb = 0; for (int t = 0; t < 20; ++t) { int64_t n = 1; for (int d = 0; d < 4; ++d) n *= shapes[t][d]; nb += (int)((n + RES_CHUNK - 1) / RES_CHUNK); }
        unsigned long long t0 = ~0ull;
        for (int i = 0; i < nb; ++i) t0 = std::min(t0, pr[i][0]);
        // per phase: median over workgroups of (probe_i - t0) in us (100 MHz clock)
        for (int p = 0; p < 15; ++p) { /* select_body probes 0..14 */
            std::vector<double> v;
            for (int i = 0; i < nb; ++i) if (sp[i][p] >= t0) v.push_back((double)(sp[i][p] - t0) / 100.0);
            std::sort(v.begin(), v.end());
            sel[p].push_back(v.empty() ? -1 : v[v.size() / 2]);
        }
        for (int p = 0; p < 18; ++p) {
            std::vector<double> v, vg[2];
            for (int i = 0; i < nb; ++i) {
                const double x = (double)(pr[i][p] - t0) / 100.0;
                v.push_back(x);
                vg[(pr[i][19] & 16) ? 1 : 0].push_back(x);
            }
            std::sort(v.begin(), v.end());
            ph[p].push_back(v[v.size() / 2]);
            ph[p].push_back(v.back());
            for (int g = 0; g < 2; ++g) {
                std::sort(vg[g].begin(), vg[g].end());
                phg[g][p].push_back(vg[g].empty() ? -1 : vg[g][vg[g].size() / 2]);
                phg[g][p].push_back(vg[g].empty() ? -1 : vg[g].back());
            }
        }
    }
    {   /* the last rep's probes of every workgroup, for offline analysis */
        FILE* f = fopen(argc > 2 ? argv[2] : "gpurun_out/reslab_probes.csv", "w");
        if (f) {
            int nb = 0; for (int t = 0; t < 20; ++t) { int64_t n = 1; for (int d = 0; d < 4; ++d) n *= shapes[t][d]; nb += (int)((n + RES_CHUNK - 1) / RES_CHUNK); }
            unsigned long long t0 = ~0ull;
            for (int i = 0; i < nb; ++i) t0 = std::min(t0, pr[i][0]);
            fprintf(f, "wg,late,start,window,counted,hist-pub,B1-arrive,B1-pass,selected,stored,sampled,sorted,issued,published\n");
            for (int i = 0; i < nb; ++i) {
                fprintf(f, "%d,%d", i, (int)((pr[i][19] >> 4) & 1));
                for (int p = 0; p < 12; ++p) fprintf(f, ",%.2f", (double)(pr[i][p] - t0) / 100.0);
                fprintf(f, "\n");
            }
            fclose(f);
        }
    }
    {
        static unsigned long long cy[NWG][2];
        CK(hipMemcpyFromSymbol(cy, HIP_SYMBOL(g_cyc), sizeof cy));
        int nb = 0; for (int t = 0; t < 20; ++t) { int64_t n = 1; for (int d = 0; d < 4; ++d) n *= shapes[t][d]; nb += (int)((n + RES_CHUNK - 1) / RES_CHUNK); }
        std::vector<double> f;
        for (int i = 0; i < nb; ++i) {
            const double dt = (double)(pr[i][7] - pr[i][0]) / 100e6;
            if (dt > 0) f.push_back((double)(cy[i][1] - cy[i][0]) / dt / 1e9);
        }
        std::sort(f.begin(), f.end());
        if (!f.empty()) printf("in-kernel shader clock (s_memtime / s_memrealtime): median %.2f GHz (min %.2f, max %.2f)\n", f[f.size() / 2], f[0], f.back());
    }
    std::sort(tms.begin(), tms.end());
    printf("flush mode %d\n", flush);
    printf("k_resident cfg2: median %.2f us (min %.2f) per call, %.1f GB/s algorithmic\n", tms[tms.size() / 2], tms[0],
           8.0 * nw / (tms[tms.size() / 2] * 1e-6) / 1e9);
    const char* names[18] = {"start", "window", "counted", "hist-pub", "B1-arrive", "B1-pass", "selected", "stored",
                             "sampled", "sorted", "issued", "published", "w:cleared", "w:histo", "w:scanned",
                             "w:found", "sc:placed", "sc:issued"};
    for (int p = 0; p < 18; ++p) {
        std::vector<double> med, mx;
        for (size_t i = 0; i < ph[p].size(); i += 2) { med.push_back(ph[p][i]); mx.push_back(ph[p][i + 1]); }
        std::sort(med.begin(), med.end()); std::sort(mx.begin(), mx.end());
        printf("  %-10s median WG %7.2f us   slowest WG %7.2f us", names[p], med[med.size() / 2], mx[mx.size() / 2]);
        for (int g = 0; g < 2; ++g) {
            std::vector<double> gm, gx;
            for (size_t i = 0; i < phg[g][p].size(); i += 2) { gm.push_back(phg[g][p][i]); gx.push_back(phg[g][p][i + 1]); }
            std::sort(gm.begin(), gm.end()); std::sort(gx.begin(), gx.end());
            printf("   | %s median %6.2f slowest %6.2f", g ? "late" : "early", gm[gm.size() / 2], gx[gx.size() / 2]);
        }
        printf("\n");
    }
    {   /* the selector workgroups (past the chunks) of the last rep: when each passed barrier 1,
         * read the totals, staged the keys and published the granule (us from the first start) */
        int nb = 0; for (int t = 0; t < 20; ++t) { int64_t n = 1; for (int d = 0; d < 4; ++d) n *= shapes[t][d]; nb += (int)((n + RES_CHUNK - 1) / RES_CHUNK); }
        unsigned long long t0 = ~0ull;
        for (int i = 0; i < nb; ++i) t0 = std::min(t0, pr[i][0]);
        static unsigned long long sp[NWG][16];
        CK(hipMemcpyFromSymbol(sp, HIP_SYMBOL(g_sprobe), sizeof sp));
        auto us = [&](unsigned long long x) { return x >= t0 && x - t0 < 100000000ull ? (double)(x - t0) / 100.0 : -1.0; };
        for (int i = nb; i < NWG; ++i) {
            if (pr[i][0] < t0 || pr[i][0] - t0 > 100000000ull) continue;
            printf("  selector %3d: start %6.2f  window %6.2f  B1-pass %6.2f  counters %6.2f  B2-pass %6.2f  staged %6.2f  ranks %6.2f  granule %6.2f\n",
                   i, us(pr[i][0]), us(pr[i][1]), us(pr[i][5]), us(sp[i][1]), us(sp[i][4]), us(sp[i][5]), us(sp[i][6]), us(pr[i][6]));
        }
    }
    const char* snames[15] = {"-", "counters", "buckets", "B2-wait", "B2-pass", "staged", "ranks", "-", "-", "-", "-", "-", "-", "-", "-"};
    for (int p = 0; p < 15; ++p) {
        if (p == 0 || p >= 7) continue;
        std::sort(sel[p].begin(), sel[p].end());
        printf("  select %-10s median WG %7.2f us\n", snames[p], sel[p][sel[p].size() / 2]);
    }
    return 0;
}
