/* small_geom.h -- geometry of the one-launch small-population path (k_small, small.hip),
 * shared by the host planner (which checks every tile's LDS need before choosing a tiling) and
 * the device (every workgroup derives its own tile's windows with the same code).
 *
 * A tensor's level-L coefficient grid is cut into TR x TC tiles; a tile OWNS, at every level k,
 * the rows [tr*TR*2^(L-k), min((tr+1)*TR*2^(L-k), N_k)) (same for columns) -- a partition of
 * every level, so every packed coefficient and every output sample has exactly one owner.
 *
 * Forward (pywt.wavedec2, ResNet/dwt_pruning.py:67-68): to compute its owned coefficients the
 * tile needs, at each level k, the approximation samples of a WINDOW W_k (a circular interval of
 * real indices of level k): W_L = own_L, W_{k-1} = taps(W_k) u own_{k-1}, where the analysis
 * output o reads samples ext(F/2 + 2o - j), j < F (pywt's periodization with the odd-length
 * repeat).  Inverse (pywt.waverec2, :75-77): the owned outputs O_0 = own_0 need level-1
 * coefficients on S_1 = sources(O_0); the level-1 approximation is synthesised there, so
 * O_1 = S_1, S_2 = sources(O_1), ... where synthesis output n reads pmod(iu(n) - j, N), j < F/2.
 */
#ifndef WT_SMALL_GEOM_H
#define WT_SMALL_GEOM_H

#include <stdint.h>

#if defined(__HIPCC__)
#define WT_SM __host__ __device__ __forceinline__
#else
#define WT_SM static inline
#endif

#define SM_MAX_L 10

struct SmIvl { /* circular interval of real indices of a line of N: s in [0, N), 1 <= len <= N */
    int32_t s, len;
};

WT_SM int32_t sm_pm(int32_t a, int32_t m) { /* arguments within a few periods: no division */
    while (a < 0) a += m;
    while (a >= m) a -= m;
    return a;
}
WT_SM int32_t sm_ext(int32_t t, int32_t N) { /* wt_ext_index in 32 bits */
    const int32_t Ne = N + (N & 1);
    const int32_t r = sm_pm(t, Ne);
    return r < N ? r : N - 1;
}
WT_SM SmIvl sm_full(int32_t N) { return SmIvl{0, N}; }

/* smallest circular interval covering a and b (it starts at a.s or at b.s) */
WT_SM SmIvl sm_union(SmIvl a, SmIvl b, int32_t N) {
    if (a.len >= N || b.len >= N) return sm_full(N);
    const int32_t e1 = (sm_pm(b.s - a.s, N) + b.len > a.len) ? sm_pm(b.s - a.s, N) + b.len : a.len;
    const int32_t e2 = (sm_pm(a.s - b.s, N) + a.len > b.len) ? sm_pm(a.s - b.s, N) + a.len : b.len;
    SmIvl r = e1 <= e2 ? SmIvl{a.s, e1} : SmIvl{b.s, e2};
    if (r.len >= N) return sm_full(N);
    return r;
}

/* the real indices ext(t0 .. t0 + m) of a line of N (odd N: residue N repeats N - 1) */
WT_SM SmIvl sm_ext_image(int32_t t0, int32_t m, int32_t N) {
    if (m + 1 >= N) return sm_full(N);
    const int32_t Ne = N + (N & 1);
    const int32_t a = sm_pm(t0, Ne), b = sm_pm(a + m, Ne);
    const int32_t sa = a < N ? a : N - 1, sb = b < N ? b : N - 1;
    return SmIvl{sa, sm_pm(sb - sa, N) + 1};
}

/* analysis: the level-(k-1) samples (line length Np) read by the outputs W (line length N) */
WT_SM SmIvl sm_fwd_taps(SmIvl W, int32_t N, int32_t Np, int32_t F) {
    if (W.s + W.len <= N) return sm_ext_image(2 * W.s + 1 - F / 2, 2 * (W.len - 1) + F - 1, Np);
    const int32_t l1 = N - W.s, l2 = W.len - l1; /* [s, N-1] and [0, l2-1] */
    return sm_union(sm_ext_image(2 * W.s + 1 - F / 2, 2 * (l1 - 1) + F - 1, Np),
                    sm_ext_image(1 - F / 2, 2 * (l2 - 1) + F - 1, Np), Np);
}

/* synthesis site of output n of 2N (wt_syn_locate), as the unwrapped source position iu: the
 * H-even special last output n = 2N - 1 reads i - j + N */
WT_SM int32_t sm_iu(int32_t n, int32_t N, int32_t F) {
    const int32_t H = F / 2, start = F / 4, M = 2 * N;
    if ((H & 1) == 0) {
        if (n == M - 1) return start - 1 + N;
        if (n == 0) return start - 1;
        return (n & 1) ? start + (n - 1) / 2 : start + (n - 2) / 2;
    }
    return start + n / 2;
}

/* synthesis: the level-k coefficients (line length N) read by the outputs O (line length No) */
WT_SM SmIvl sm_inv_src(SmIvl O, int32_t No, int32_t N, int32_t F) {
    const int32_t H = F / 2;
    auto piece = [&](int32_t na, int32_t nb) {
        const int32_t a = sm_iu(na, N, F) - H + 1, m = sm_iu(nb, N, F) - a;
        return m + 1 >= N ? sm_full(N) : SmIvl{sm_pm(a, N), m + 1};
    };
    if (O.s + O.len <= No) return piece(O.s, O.s + O.len - 1);
    return sm_union(piece(O.s, No - 1), piece(0, O.s + O.len - No - 1), N);
}

/* owned range [lo, hi) of tile index t (tile size T at level L) at level k */
WT_SM void sm_own(int32_t t, int32_t T, int32_t L, int32_t k, const int32_t* N, int32_t* lo, int32_t* hi) {
    /* t * T < N_L < 2^20 and L - k <= 10: 32-bit products */
    const int32_t a = (t * T) << (L - k), b = ((t + 1) * T) << (L - k);
    *lo = a;
    *hi = b < N[k] ? b : N[k];
}

/* every window of one axis of one tile: fw[k] (k = 0..L) forward, sv[k] (k = 1..L) inverse
 * sources (= the synthesised approximation window of level k for k < L), ov0 = own_0 */
struct SmAxis {
    SmIvl fw[SM_MAX_L + 1];
    SmIvl sv[SM_MAX_L + 1];
    int32_t olo[SM_MAX_L + 1], ohi[SM_MAX_L + 1];
};

#if defined(__HIPCC__)
#define SM_NOUNROLL _Pragma("unroll 1")
#else
#define SM_NOUNROLL
#endif
WT_SM void sm_axis_fwd(int32_t t, int32_t T, int32_t L, const int32_t* N, int32_t F, SmAxis* a) {
    SM_NOUNROLL
    for (int k = 0; k <= L; ++k) sm_own(t, T, L, k, N, &a->olo[k], &a->ohi[k]);
    a->fw[L] = SmIvl{a->olo[L], a->ohi[L] - a->olo[L]};
    SM_NOUNROLL
    for (int k = L; k >= 1; --k) {
        const SmIvl own = SmIvl{a->olo[k - 1], a->ohi[k - 1] - a->olo[k - 1]};
        a->fw[k - 1] = sm_union(sm_fwd_taps(a->fw[k], N[k], N[k - 1], F), own, N[k - 1]);
    }
}
WT_SM void sm_axis_inv(int32_t t, int32_t T, int32_t L, const int32_t* N, int32_t F, SmAxis* a) {
    int32_t lo, hi;
    sm_own(t, T, L, 0, N, &lo, &hi);
    SmIvl o = SmIvl{lo, hi - lo};
    a->sv[0] = o;
    SM_NOUNROLL
    for (int k = 1; k <= L; ++k) {
        a->sv[k] = sm_inv_src(o, N[k - 1], N[k], F);
        o = a->sv[k];
    }
}
WT_SM void sm_axis(int32_t t, int32_t T, int32_t L, const int32_t* N, int32_t F, SmAxis* a) {
    sm_axis_fwd(t, T, L, N, F, a);
    sm_axis_inv(t, T, L, N, F, a);
}

/* LDS words one tile needs (the planner and the kernel lay out the arena the same way) */
struct SmNeed {
    int32_t fx, flh, fkeys;       /* forward: approximation window, column-pass rows, owned keys */
    int32_t ia, iwin, ilh;        /* inverse: synthesised cA window, the coefficient windows of every
                                     level (read from P ahead of the synthesis), row-pass rows, tables */
};

WT_SM SmNeed sm_need(const SmAxis& ar, const SmAxis& ac, int32_t L, int32_t F) {
    SmNeed n = {0, 0, 0, 0, 0, 0};
    for (int k = 0; k <= L; ++k) {
        const int32_t x = ar.fw[k].len * ac.fw[k].len;
        n.fx = x > n.fx ? x : n.fx;
    }
    for (int k = 1; k <= L; ++k) {
        const int32_t lh = 2 * ar.fw[k].len * ac.fw[k - 1].len;
        n.flh = lh > n.flh ? lh : n.flh;
        const int32_t h = ar.ohi[k] - ar.olo[k], w = ac.ohi[k] - ac.olo[k];
        n.fkeys += 3 * h * w + (k == L ? h * w : 0);
        const int32_t s = ar.sv[k].len * ac.sv[k].len;
        n.ia = s > n.ia ? s : n.ia;
        const int32_t lo = 2 * ar.sv[k].len * ac.sv[k - 1].len;
        n.ilh = lo > n.ilh ? lo : n.ilh;
    }
    for (int k = 1; k < L; ++k) { /* the synthesised approximation of level k covers sv[k] */
        const int32_t s = ar.sv[k].len * ac.sv[k].len;
        n.ia = s > n.ia ? s : n.ia;
    }
    for (int k = 1; k <= L; ++k) n.iwin += (3 + (k == L)) * ar.sv[k].len * ac.sv[k].len;
    return n;
}

/* regions start 16-byte aligned: up to 3 words of padding after each of the first three */
WT_SM int32_t sm_fwd_words(const SmNeed& n) { return n.fkeys + n.fx + n.flh + 12; }
/* the select gathers the segment's key slots (SM_SEG_WG_MAX x SM_SLOT_WORDS = 8192 words) at the
 * arena's tail while the windows are live */
WT_SM int32_t sm_inv_words(const SmNeed& n) { return n.fkeys + n.iwin + n.ia + n.ilh + 16 + 8192; }

#endif
