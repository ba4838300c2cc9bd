/* Filter-bank point evaluators shared by the HIP kernels (device) and the host-side
 * index self-check (tests/native/corecheck.cpp).  They are GATHER forms of PyWavelets'
 * periodized float32 filter bank, each output sample summed in exactly the order the
 * reference's arithmetic produces it (separate multiply and add -- build with
 * -ffp-contract=off):
 *
 *  analysis (pywt float_downsampling_convolution_periodization, reached from
 *  pywt.wavedec2 at ResNet/dwt_pruning.py:67-68):
 *     i = F/2 + 2o;  i < N : taps j = 0..F-1 ascending
 *                    i >= N: taps with i-j >= N in descending j, then i-j < N ascending
 *     sample index (i-j) mod Ne, Ne = N + (N odd), index N (odd N) reads x[N-1]
 *
 *  synthesis (pywt float_upsampling_convolution_valid_sf, periodization branch, reached
 *  from pywt.waverec2 at dwt_pruning.py:77): output n of 2N receives H = F/2 terms of the
 *  rec_lo pass over cA, then H terms of the rec_hi pass over cD, all from one source
 *  position i and one tap parity (see wt_syn_site); the tap order rule is the same as above
 *  with the "special" first site (H even) wrapping at the left edge instead of the right.
 */
#ifndef WT_DWT_CORE_H
#define WT_DWT_CORE_H

#include <stdint.h>

#if defined(__HIPCC__)
#define WT_CORE __host__ __device__ __forceinline__
#else
#define WT_CORE static inline
#endif

#define WTP_MAX_F 102

WT_CORE int64_t wt_pmod(int64_t a, int64_t m) {
    int64_t r = a % m;
    return r < 0 ? r + m : r;
}

/* index into a periodized line of N samples extended to even length (odd N repeats x[N-1]) */
WT_CORE int64_t wt_ext_index(int64_t t, int64_t N) {
    const int64_t Ne = N + (N & 1);
    int64_t r = wt_pmod(t, Ne);
    return r < N ? r : N - 1;
}

/* One analysis output o (both bands).  Fetch(k) returns sample k, 0 <= k < N. */
template <class Fetch>
WT_CORE void wt_ana_point(int64_t o, int64_t N, int F, const float* lo, const float* hi,
                          const Fetch& fetch, float& sa, float& sd) {
    const int64_t i = F / 2 + 2 * o;
    float a = 0.0f, d = 0.0f;
    if (i < N) {
        for (int j = 0; j < F; ++j) {
            const float v = fetch(wt_ext_index(i - j, N));
            const float pa = lo[j] * v, pd = hi[j] * v;
            a = a + pa;
            d = d + pd;
        }
    } else {
        for (int j = F - 1; j >= 0; --j) {
            if (i - j >= N) {
                const float v = fetch(wt_ext_index(i - j, N));
                const float pa = lo[j] * v, pd = hi[j] * v;
                a = a + pa;
                d = d + pd;
            }
        }
        for (int j = 0; j < F; ++j) {
            if (i - j < N) {
                const float v = fetch(wt_ext_index(i - j, N));
                const float pa = lo[j] * v, pd = hi[j] * v;
                a = a + pa;
                d = d + pd;
            }
        }
    }
    sa = a;
    sd = d;
}

/* Which source position i, tap parity and ordering rule produce synthesis output n. */
struct wt_syn_site {
    int64_t i;
    int par;      /* 0: taps rec[2j], 1: taps rec[2j+1] */
    int special;  /* 1: the H-even first site (i = F/4 - 1), wrap at the left edge */
};

WT_CORE wt_syn_site wt_syn_locate(int64_t n, int64_t N, int F) {
    const int H = F / 2, start = F / 4;
    const int64_t M = 2 * N;
    wt_syn_site s;
    s.special = 0;
    if ((H & 1) == 0) {
        if (n == M - 1) { s.i = start - 1; s.par = 0; s.special = 1; }
        else if (n == 0) { s.i = start - 1; s.par = 1; s.special = 1; }
        else if (n & 1) { s.i = start + (n - 1) / 2; s.par = 0; }
        else { s.i = start + (n - 2) / 2; s.par = 1; }
    } else {
        if ((n & 1) == 0) { s.i = start + n / 2; s.par = 0; }
        else { s.i = start + (n - 1) / 2; s.par = 1; }
    }
    return s;
}

/* Accumulate one synthesis pass (H terms) for site s into acc.  Fetch(k), 0 <= k < N. */
template <class Fetch>
WT_CORE float wt_syn_pass(const wt_syn_site& s, int64_t N, int F, const float* rec,
                          const Fetch& fetch, float acc) {
    const int H = F / 2;
    const int64_t i = s.i;
    if (s.special) {
        for (int j = H - 1; j >= 0; --j)
            if (i - j >= 0) { const float p = rec[2 * j + s.par] * fetch(wt_pmod(i - j, N)); acc = acc + p; }
        for (int j = 0; j < H; ++j)
            if (i - j < 0) { const float p = rec[2 * j + s.par] * fetch(wt_pmod(i - j, N)); acc = acc + p; }
    } else if (i < N) {
        for (int j = 0; j < H; ++j) { const float p = rec[2 * j + s.par] * fetch(wt_pmod(i - j, N)); acc = acc + p; }
    } else {
        for (int j = H - 1; j >= 0; --j)
            if (i - j >= N) { const float p = rec[2 * j + s.par] * fetch(wt_pmod(i - j, N)); acc = acc + p; }
        for (int j = 0; j < H; ++j)
            if (i - j < N) { const float p = rec[2 * j + s.par] * fetch(wt_pmod(i - j, N)); acc = acc + p; }
    }
    return acc;
}

/* One synthesis output n of 2N: rec_lo pass over cA then rec_hi pass over cD. */
template <class FetchA, class FetchD>
WT_CORE float wt_syn_point(int64_t n, int64_t N, int F, const float* rlo, const float* rhi,
                           const FetchA& fa, const FetchD& fd) {
    const wt_syn_site s = wt_syn_locate(n, N, F);
    float acc = 0.0f;
    acc = wt_syn_pass(s, N, F, rlo, fa, acc);
    acc = wt_syn_pass(s, N, F, rhi, fd, acc);
    return acc;
}

/* ---- packed layout (pywt.coeffs_to_array for wavedec2 over axes (-2,-1)) ---- */
struct wt_level_geom {
    int64_t R[33], C[33];       /* R[0] = H; R[k] = ceil(R[k-1]/2) */
    int64_t offR[33], offC[33]; /* top-left of the level-k detail blocks in the packed image */
    int64_t PR, PC;             /* packed image size */
};

WT_CORE void wt_geom(int64_t H, int64_t W, int L, wt_level_geom* g) {
    g->R[0] = H;
    g->C[0] = W;
    for (int k = 1; k <= L; ++k) { g->R[k] = (g->R[k - 1] + 1) / 2; g->C[k] = (g->C[k - 1] + 1) / 2; }
    int64_t aR = g->R[L], aC = g->C[L];
    for (int k = L; k >= 1; --k) { g->offR[k] = aR; g->offC[k] = aC; aR += g->R[k]; aC += g->C[k]; }
    g->PR = (L == 0) ? H : aR;
    g->PC = (L == 0) ? W : aC;
}

#endif
