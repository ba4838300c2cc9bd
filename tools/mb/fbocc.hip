// Filter-bank residency probe: every tile of one level launch records its start / end
// (100 MHz wall clock) and its CU (HW_ID + XCC_ID); prints the WG lifetime and how many
// workgroups each CU held at once (mean over the launch, max).  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off fbocc.hip -o fbocc
#include <hip/hip_runtime.h>
__device__ unsigned long long* g_occ;
#define WTP_FPROBE(i)                                                                              \
    do {                                                                                           \
        if (threadIdx.x == 0) {                                                                    \
            unsigned hw, xcc;                                                                      \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));                      \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));                    \
            const int slot_ = i == 0 ? 0 : (i == 3 ? 1 : 2 + i);                                   \
            g_occ[5 * gt + slot_] = wall_clock64();                                                \
            if (i == 0) g_occ[5 * gt + 2] = ((unsigned long long)(xcc & 15) << 32) | hw;           \
        }                                                                                          \
    } while (0)
#include "../../wavelettransforms_amd/csrc/filterbank.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace wtp;

static void report(const char* name, const unsigned long long* h, int nwg) {
    std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> ev; /* cu -> (t, +1/-1) */
    unsigned long long t0 = ~0ull, t1 = 0;
    std::vector<double> life, p1, p2;
    for (int b = 0; b < nwg; ++b) {
        const unsigned long long s = h[5 * b], e = h[5 * b + 1], id = h[5 * b + 2];
        p1.push_back((h[5 * b + 3] - s) / 100.0);
        p2.push_back((h[5 * b + 4] - s) / 100.0);
        const unsigned hw = (unsigned)id;
        const unsigned long long cu = ((id >> 32) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
        ev[cu].push_back({s, +1});
        ev[cu].push_back({e, -1});
        t0 = std::min(t0, s);
        t1 = std::max(t1, e);
        life.push_back((e - s) / 100.0);
    }
    std::sort(life.begin(), life.end());
    std::sort(p1.begin(), p1.end());
    std::sort(p2.begin(), p2.end());
    int mx = 0;
    double area = 0;
    for (auto& kv : ev) {
        auto v = kv.second;
        std::sort(v.begin(), v.end());
        int c = 0;
        unsigned long long last = v[0].first;
        for (auto& p : v) { area += (double)c * (p.first - last); last = p.first; c += p.second; mx = std::max(mx, c); }
    }
    printf("%-28s WGs %6d CUs %3zu span %8.2f us  life p10/50/90 %6.2f %6.2f %6.2f us  WGs per CU mean %.2f max %d\n",
           name, nwg, ev.size(), (t1 - t0) / 100.0, life[life.size() / 10], life[life.size() / 2], life[9 * life.size() / 10],
           area / ((t1 - t0) * (double)ev.size()), mx);
    printf("%-28s median probe 1 at %.2f us, probe 2 at %.2f us (from the tile's start)\n", "", p1[p1.size() / 2], p2[p2.size() / 2]);
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 8;
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
    const int MAXWG = 1 << 16;
    unsigned long long* occ; CK(hipMalloc(&occ, (size_t)5 * MAXWG * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_occ), &occ, sizeof(occ)));
    std::vector<unsigned long long> h(5 * MAXWG);
    auto run = [&](const char* name, auto fn, int nwg) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), occ, (size_t)5 * nwg * 8, hipMemcpyDeviceToHost));
        report(name, h.data(), nwg);
    };
    for (int k = 1; k <= 2; ++k) {
        const int64_t R0 = g.R[k - 1], C0 = g.C[k - 1];
        const float* in = k == 1 ? x : t0;
        const int nwg = (int)(B * ((g.R[k] + FR - 1) / FR) * ((g.C[k] + FC - 1) / FC));
        char nm[64];
        snprintf(nm, 64, "fwd level %d", k);
        run(nm, [&] { launch_fwd_level(in, B, R0, C0, tp, t1, P, g.PR, g.PC, g.offR[k], g.offC[k], k == L, 0); }, nwg);
    }
    for (int k = 2; k >= 1; --k) {
        const int64_t R = g.R[k], C = g.C[k];
        const int nwg = (int)(B * ((2 * R + IR - 1) / IR) * ((2 * C + IC - 1) / IC));
        char nm[64];
        snprintf(nm, 64, "inv level %d", k);
        run(nm, [&] {
            launch_inv_level(t0, 4 * g.R[k + 1] * g.C[k + 1], 2 * g.C[k + 1], 0, P, g.PR, g.PC, g.offR[k], g.offC[k], B, R, C, tp,
                             dthr, k == 1 ? y : t1, 2 * R, 2 * C, nullptr, 0);
        }, nwg);
    }
    return 0;
}
