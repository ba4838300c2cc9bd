// Host build of the product's filter-bank point evaluators (csrc/wt_dwt_core.h) so the CPU
// test suite can check the device index math against the oracle without a GPU.
// Built by tests/test_core_index.py with: g++ -O2 -ffp-contract=off -shared -fPIC
#include <cstring>
#include "../../wavelettransforms_amd/csrc/wt_dwt_core.h"

extern "C" void core_dwt1(const float* x, long long N, int F, const float* lo, const float* hi,
                          float* a, float* d) {
    const long long O = (N + 1) / 2;
    auto fetch = [&](int64_t k) { return x[k]; };
    for (long long o = 0; o < O; ++o) wt_ana_point(o, N, F, lo, hi, fetch, a[o], d[o]);
}

extern "C" void core_idwt1(const float* ca, const float* cd, long long N, int F, const float* rlo,
                           const float* rhi, float* out) {
    auto fa = [&](int64_t k) { return ca[k]; };
    auto fd = [&](int64_t k) { return cd[k]; };
    for (long long n = 0; n < 2 * N; ++n) out[n] = wt_syn_point(n, N, F, rlo, rhi, fa, fd);
}

extern "C" void core_geom(long long H, long long W, int L, long long* out /* PR, PC, R[L+1], C[L+1], offR[L+1], offC[L+1] */) {
    wt_level_geom g;
    wt_geom(H, W, L, &g);
    out[0] = g.PR;
    out[1] = g.PC;
    for (int k = 0; k <= L; ++k) {
        out[2 + 4 * k] = g.R[k];
        out[3 + 4 * k] = g.C[k];
        out[4 + 4 * k] = k ? g.offR[k] : 0;
        out[5 + 4 * k] = k ? g.offC[k] : 0;
    }
}
