/*
 * wtprune_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
 * DWT -> percentile-threshold -> IDWT weight-pruning path, used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the CHECKER.  The product
 * (wavelettransforms_amd/, libwtprune.so) never links or calls this file.
 *
 * Reference path: ResNet/dwt_pruning.py:35-95 (multi_resolution_analysis), whose arithmetic
 * lives in two third-party libraries that are NOT part of /root/reference:
 *   - PyWavelets 1.1.1 (pinned "1.4.1" in requirements.txt:3; 1.1.1 is what this image has):
 *       wavedec2 pywt/_multilevel.py:179-253, dwt2/dwtn pywt/_multidim.py:24-74,121-192,
 *       coeffs_to_array :674-788, array_to_coeffs :791-877, waverec2 :256-337,
 *       idwt2/idwtn pywt/_multidim.py:77-118,222-311, C float_downsampling_convolution_
 *       periodization / float_upsampling_convolution_valid_sf (periodization branch).
 *   - NumPy 1.26.4: np.percentile numpy/lib/function_base.py:3993,4279 -> _quantile :4765-4870
 *       (linear method :109-112, _get_indexes :4730-4763, _lerp :4641-4662), and legacy
 *       value-based casting for `np.abs(arr) < threshold` (compare in float32).
 *
 * Parity pinning: tests/test_oracle_golden.py checks every function here bit for bit
 * against fixtures in tests/golden/ produced by tools/gen_golden.py, which runs the
 * reference's own call sequence (dwt_pruning.py:53-89) on PyWavelets 1.1.1 + NumPy 1.26.4.
 *
 * Arithmetic contract (verified against pywt for all 106 discrete wavelets, N = 1..70):
 *   A.1 analysis  : i = F/2 + 2o; taps ascending if i < N, else the wrapped taps (i-j >= N)
 *                   in descending j followed by the rest in ascending j; odd N is extended by
 *                   repeating x[N-1]; separate f32 multiply and add (no FMA).
 *   A.2 synthesis : the scatter loop of pywt's periodization synthesis, restated literally in
 *                   idwt1() below (rec_lo pass over cA, then rec_hi pass over cD).
 * Build: gcc -O2 -ffp-contract=off (never -ffast-math): the order of float ops is the oracle.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../wavelettransforms_amd/csrc/wt_filters.inc"
#include "../wavelettransforms_amd/csrc/wt_synth.h"
#include "../wavelettransforms_amd/csrc/wt_perm.h"

#define OR_OK 0
#define OR_EBADWAVELET (-1)  /* pywt.Wavelet(name) -> ValueError                      */
#define OR_EBADLEVEL (-2)    /* pywt _check_level -> ValueError (level < 0)            */
#define OR_EBADPCT (-3)      /* np.percentile -> ValueError (q outside [0, 100])       */
#define OR_EEMPTY (-4)       /* np.percentile on an empty array -> IndexError          */
#define OR_ECROP (-5)        /* dwt_pruning.py:79-82 4-index crop on a <4-D array -> IndexError */
#define OR_ENOMEM (-6)

typedef struct {
    int64_t numel;        /* weights in the tensor                                   */
    int64_t zero_count;   /* (pruned == 0).sum()            dwt_pruning.py:88        */
    int64_t nonzero;      /* pruned.nonzero().size(0)       dwt_pruning.py:119-120   */
    int64_t coeff_numel;  /* packed coefficient array size (percentile population)   */
    int64_t packed_rows, packed_cols; /* packed (rows, cols) per batch image         */
    double thr64;         /* np.percentile(|coeff_arr|, pct)                         */
    float thr32;          /* float32(thr64): the value the compare actually uses     */
    float max_abs;        /* np.max(np.abs(coeff_arr)) (debug print, :29-30)        */
    int32_t eff_level;    /* min(level, calculate_max_level(...))  :64-65            */
    int32_t status;
} or_result;

/* ------------------------------------------------------------------ wavelets --- */
static inline float tap(int wid, int k, int j) {
    const int F = wt_flen[wid];
    uint32_t b = wt_taps_bits[wt_foff[wid] + k * F + j];
    float f;
    memcpy(&f, &b, 4);
    return f;
}

int or_num_wavelets(void) { return WT_NUM_WAVELETS; }
const char* or_wavelet_name(int wid) { return (wid >= 0 && wid < WT_NUM_WAVELETS) ? wt_names[wid] : 0; }
int or_wavelet_id(const char* name) {
    for (int i = 0; i < WT_NUM_WAVELETS; ++i)
        if (strcmp(name, wt_names[i]) == 0) return i;
    return -1;
}
int or_dec_len(int wid) { return (wid >= 0 && wid < WT_NUM_WAVELETS) ? wt_flen[wid] : -1; }
void or_filters(int wid, float* out4F) {
    const int F = wt_flen[wid];
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < F; ++j) out4F[k * F + j] = tap(wid, k, j);
}

/* pywt.dwt_max_level (pywt/_dwt.py:18-80): 0 if n < F-1 else int(log2(n / (F-1))).
 * Restated as the exact integer: the largest L with (F-1) * 2^L <= n. */
int or_dwt_max_level(int64_t n, int F) {
    if (F < 2) return -1;
    if (n < F - 1) return 0;
    int L = 0;
    while ((int64_t)(F - 1) << (L + 1) <= n) ++L;
    return L;
}

/* --------------------------------------------------------------- 1-D kernels --- */
static inline int64_t pmod(int64_t a, int64_t m) { int64_t r = a % m; return r < 0 ? r + m : r; }

/* A.1: one level of periodized analysis along a strided line of N samples. */
static void dwt1(const float* x, int64_t xs, int64_t N, int wid, float* a, float* d, int64_t os) {
    const int F = wt_flen[wid];
    const int64_t Ne = N + (N & 1), O = Ne / 2;
    for (int64_t o = 0; o < O; ++o) {
        const int64_t i = F / 2 + 2 * o;
        float sa = 0.0f, sd = 0.0f;
#define OR_ACC(J)                                                        \
    do {                                                                 \
        int64_t t = pmod(i - (J), Ne);                                   \
        float v = x[(t < N ? t : N - 1) * xs];                           \
        float pa = tap(wid, 0, (J)) * v, pd = tap(wid, 1, (J)) * v;      \
        sa = sa + pa;                                                    \
        sd = sd + pd;                                                    \
    } while (0)
        if (i < N) {
            for (int j = 0; j < F; ++j) OR_ACC(j);
        } else {
            for (int j = F - 1; j >= 0; --j) if (i - j >= N) OR_ACC(j);
            for (int j = 0; j < F; ++j) if (i - j < N) OR_ACC(j);
        }
#undef OR_ACC
        a[o * os] = sa;
        d[o * os] = sd;
    }
}

/* A.2: one level of periodized synthesis (output 2N samples), the scatter loop of pywt's
 * float_upsampling_convolution_valid_sf periodization branch restated: each pass adds
 * rec[2j]*c[i-j] into out[o] and rec[2j+1]*c[i-j] into out[o+1]. */
static void idwt1(const float* ca, const float* cd, int64_t cs, int64_t N, int wid, float* out, int64_t os) {
    const int F = wt_flen[wid];
    const int H = F / 2, start = F / 4;
    const int64_t M = 2 * N;
    for (int64_t n = 0; n < M; ++n) out[n * os] = 0.0f;
    for (int pass = 0; pass < 2; ++pass) {
        const float* c = pass == 0 ? ca : cd;
        const int k = 2 + pass; /* rec_lo / rec_hi */
#define OR_ADD(OIDX, J)                                                                   \
    do {                                                                                  \
        float v = c[pmod(i - (J), N) * cs];                                               \
        int64_t o0 = pmod((OIDX), M) * os, o1 = pmod((OIDX) + 1, M) * os;                 \
        float p0 = tap(wid, k, 2 * (J)) * v, p1 = tap(wid, k, 2 * (J) + 1) * v;           \
        out[o0] = out[o0] + p0;                                                           \
        out[o1] = out[o1] + p1;                                                           \
    } while (0)
        if (H % 2 == 0) {
            const int64_t i = start - 1; /* writes out[2N-1] (even taps) and out[0] (odd taps) */
            for (int j = H - 1; j >= 0; --j) if (i - j >= 0) OR_ADD(M - 1, j);
            for (int j = 0; j < H; ++j) if (i - j < 0) OR_ADD(M - 1, j);
        }
        int64_t o = (H % 2 == 0) ? 1 : 0;
        const int64_t end = N + start - ((H % 2) ? 0 : 1);
        for (int64_t i = start; i < end; ++i, o += 2) {
            if (i < N) {
                for (int j = 0; j < H; ++j) OR_ADD(o, j);
            } else {
                for (int j = H - 1; j >= 0; --j) if (i - j >= N) OR_ADD(o, j);
                for (int j = 0; j < H; ++j) if (i - j < N) OR_ADD(o, j);
            }
        }
#undef OR_ADD
    }
}

void or_dwt1(const float* x, int64_t N, int wid, float* a, float* d) { dwt1(x, 1, N, wid, a, d, 1); }
void or_idwt1(const float* a, const float* d, int64_t N, int wid, float* out) { idwt1(a, d, 1, N, wid, out, 1); }

/* ------------------------------------------------------------ 2-D, one level --- */
/* pywt dwt2 -> dwtn (pywt/_multidim.py:183-191): axis -2 first, then axis -1 on both halves.
 * in: (B, R, C) with row stride ld; outputs aa/da/ad/dd: (B, Ro, Co) dense. */
static int dwt2_level(const float* in, int64_t B, int64_t R, int64_t C, int64_t ld, int wid,
                      float* aa, float* da, float* ad, float* dd) {
    const int64_t Ro = (R + 1) / 2, Co = (C + 1) / 2;
    float* L = (float*)malloc(sizeof(float) * (size_t)(Ro * C));
    float* Hh = (float*)malloc(sizeof(float) * (size_t)(Ro * C));
    if (!L || !Hh) { free(L); free(Hh); return OR_ENOMEM; }
    for (int64_t b = 0; b < B; ++b) {
        const float* X = in + b * R * ld;
        for (int64_t c = 0; c < C; ++c) dwt1(X + c, ld, R, wid, L + c, Hh + c, C);
        const int64_t ob = b * Ro * Co;
        for (int64_t r = 0; r < Ro; ++r) {
            dwt1(L + r * C, 1, C, wid, aa + ob + r * Co, ad + ob + r * Co, 1);
            dwt1(Hh + r * C, 1, C, wid, da + ob + r * Co, dd + ob + r * Co, 1);
        }
    }
    free(L);
    free(Hh);
    return OR_OK;
}

/* pywt idwt2 -> idwtn (pywt/_multidim.py:288-309): axis -1 first ((aa,ad)->a, (da,dd)->d),
 * then axis -2.  Inputs (B, R, C) each with their own row stride (the packed array), the
 * approximation may be a cropped view (lda).  out: (B, 2R, 2C) dense. */
static int idwt2_level(const float* aa, int64_t a_bs, int64_t lda, const float* da, const float* ad,
                       const float* dd, int64_t d_bs, int64_t ldd, int64_t B, int64_t R, int64_t C,
                       int wid, float* out) {
    const int64_t C2 = 2 * C, R2 = 2 * R;
    float* lo = (float*)malloc(sizeof(float) * (size_t)(R * C2));
    float* hi = (float*)malloc(sizeof(float) * (size_t)(R * C2));
    if (!lo || !hi) { free(lo); free(hi); return OR_ENOMEM; }
    for (int64_t b = 0; b < B; ++b) {
        for (int64_t r = 0; r < R; ++r) {
            idwt1(aa + b * a_bs + r * lda, ad + b * d_bs + r * ldd, 1, C, wid, lo + r * C2, 1);
            idwt1(da + b * d_bs + r * ldd, dd + b * d_bs + r * ldd, 1, C, wid, hi + r * C2, 1);
        }
        float* Y = out + b * R2 * C2;
        for (int64_t c = 0; c < C2; ++c) idwt1(lo + c, hi + c, C2, R, wid, Y + c, C2);
    }
    free(lo);
    free(hi);
    return OR_OK;
}

/* ---------------------------------------------------- multilevel + packing --- */
/* Packed layout of pywt.coeffs_to_array(wavedec2(...), axes=(-2,-1)) for one image:
 * cA_L at [0:R_L, 0:C_L]; then for k = L..1 with running (aR, aC) starting at (R_L, C_L):
 * 'da'(cH_k) at [aR:aR+R_k, 0:C_k], 'ad'(cV_k) at [0:R_k, aC:aC+C_k], 'dd'(cD_k) at
 * [aR:aR+R_k, aC:aC+C_k]; aR += R_k, aC += C_k.  Cells not covered stay 0 and ARE part of
 * the percentile population (pywt/_multilevel.py:747-755). */
void or_packed_shape(int64_t H, int64_t W, int L, int64_t* PR, int64_t* PC) {
    int64_t r = H, c = W, sr = 0, sc = 0;
    for (int k = 1; k <= L; ++k) { r = (r + 1) / 2; c = (c + 1) / 2; sr += r; sc += c; }
    *PR = (L == 0) ? H : sr + r;
    *PC = (L == 0) ? W : sc + c;
}

/* wavedec2(mode='periodization', axes=(-2,-1)) + coeffs_to_array: in (B,H,W) -> P (B,PR,PC). */
int or_wavedec2_packed(const float* in, int64_t B, int64_t H, int64_t W, int wid, int L, float* P) {
    int64_t PR, PC;
    or_packed_shape(H, W, L, &PR, &PC);
    if (L == 0) { memcpy(P, in, sizeof(float) * (size_t)(B * H * W)); return OR_OK; }
    memset(P, 0, sizeof(float) * (size_t)(B * PR * PC));
    int64_t Rk[64], Ck[64];
    Rk[0] = H; Ck[0] = W;
    for (int k = 1; k <= L; ++k) { Rk[k] = (Rk[k - 1] + 1) / 2; Ck[k] = (Ck[k - 1] + 1) / 2; }
    /* offsets of level-k detail blocks in the packed image */
    int64_t offR[64], offC[64];
    {
        int64_t aR = Rk[L], aC = Ck[L];
        for (int k = L; k >= 1; --k) { offR[k] = aR; offC[k] = aC; aR += Rk[k]; aC += Ck[k]; }
    }
    const float* cur = in;
    float* owned = NULL;
    int rc = OR_OK;
    for (int k = 1; k <= L && rc == OR_OK; ++k) {
        const int64_t R = Rk[k - 1], C = Ck[k - 1], Ro = Rk[k], Co = Ck[k], S = B * Ro * Co;
        float* buf = (float*)malloc(sizeof(float) * (size_t)(4 * S));
        if (!buf) { rc = OR_ENOMEM; break; }
        float *aa = buf, *da = buf + S, *ad = buf + 2 * S, *dd = buf + 3 * S;
        rc = dwt2_level(cur, B, R, C, C, wid, aa, da, ad, dd);
        for (int64_t b = 0; b < B; ++b) {
            float* Pb = P + b * PR * PC;
            for (int64_t r = 0; r < Ro; ++r)
                for (int64_t c = 0; c < Co; ++c) {
                    const int64_t s = b * Ro * Co + r * Co + c;
                    Pb[(offR[k] + r) * PC + c] = da[s];
                    Pb[r * PC + offC[k] + c] = ad[s];
                    Pb[(offR[k] + r) * PC + offC[k] + c] = dd[s];
                    if (k == L) Pb[r * PC + c] = aa[s];
                }
        }
        free(owned);
        /* keep only aa for the next level (move it to the front of buf) */
        owned = buf;
        cur = aa;
    }
    free(owned);
    return rc;
}

/* array_to_coeffs + waverec2 (pywt/_multilevel.py:314-337), optionally thresholding every
 * coefficient on load (|c| < thr32 -> +0, the np.where of dwt_pruning.py:31), then the crop to
 * (H, W).  P: (B, PR, PC) -> out: (B, H, W). */
static inline float thr_load(float c, int apply, float thr32) {
    return (apply && fabsf(c) < thr32) ? 0.0f : c;
}

int or_waverec2_packed(const float* P, int64_t B, int64_t H, int64_t W, int wid, int L,
                       int apply_thr, float thr32, float* out) {
    int64_t PR, PC;
    or_packed_shape(H, W, L, &PR, &PC);
    if (L == 0) {
        for (int64_t i = 0; i < B * H * W; ++i) out[i] = thr_load(P[i], apply_thr, thr32);
        return OR_OK;
    }
    int64_t Rk[64], Ck[64], offR[64], offC[64];
    Rk[0] = H; Ck[0] = W;
    for (int k = 1; k <= L; ++k) { Rk[k] = (Rk[k - 1] + 1) / 2; Ck[k] = (Ck[k - 1] + 1) / 2; }
    {
        int64_t aR = Rk[L], aC = Ck[L];
        for (int k = L; k >= 1; --k) { offR[k] = aR; offC[k] = aC; aR += Rk[k]; aC += Ck[k]; }
    }
    /* thresholded copy of the packed array (the pruned_coeff_arr of dwt_pruning.py:72-73) */
    float* Q = (float*)malloc(sizeof(float) * (size_t)(B * PR * PC));
    if (!Q) return OR_ENOMEM;
    for (int64_t i = 0; i < B * PR * PC; ++i) Q[i] = thr_load(P[i], apply_thr, thr32);
    /* a starts as cA_L, a view into Q */
    const float* a = Q;
    int64_t a_bs = PR * PC, lda = PC, aR = Rk[L], aC = Ck[L];
    float* abuf = NULL;
    int rc = OR_OK;
    for (int k = L; k >= 1; --k) {
        const int64_t R = Rk[k], C = Ck[k];
        /* waverec2 crop: drop the last row/col of a where a_len == d_len + 1 (:333-335) */
        (void)aR; (void)aC;
        float* y = (float*)malloc(sizeof(float) * (size_t)(B * 4 * R * C));
        if (!y) { rc = OR_ENOMEM; break; }
        rc = idwt2_level(a, a_bs, lda, Q + offR[k] * PC, Q + offC[k], Q + offR[k] * PC + offC[k],
                         PR * PC, PC, B, R, C, wid, y);
        free(abuf);
        abuf = y;
        a = y;
        a_bs = 4 * R * C;
        lda = 2 * C;
        aR = 2 * R;
        aC = 2 * C;
        if (rc != OR_OK) break;
    }
    if (rc == OR_OK) {
        /* final crop to the original (H, W): pruned_weight_np[..., :H, :W] (dwt_pruning.py:79-82) */
        for (int64_t b = 0; b < B; ++b)
            for (int64_t r = 0; r < H; ++r)
                memcpy(out + (b * H + r) * W, a + b * a_bs + r * lda, sizeof(float) * (size_t)W);
    }
    free(abuf);
    free(Q);
    return rc;
}

/* ------------------------------------------------------------- percentile --- */
static inline uint32_t abs_key(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return u & 0x7FFFFFFFu; /* |x| bit pattern: monotone in |x|; NaN sorts above +inf */
}
static inline float key_f(uint32_t k) { float f; memcpy(&f, &k, 4); return f; }

/* k-th smallest (0-based) of keys[0..n-1] by in-place quickselect (order statistics are
 * unique values, so ties need no special handling; equals np.partition's kth element). */
static uint32_t select_kth(uint32_t* a, int64_t n, int64_t k) {
    int64_t lo = 0, hi = n - 1;
    while (lo < hi) {
        int64_t mid = lo + (hi - lo) / 2;
        uint32_t x = a[lo], y = a[mid], z = a[hi];
        uint32_t piv = (x < y) ? ((y < z) ? y : (x < z ? z : x)) : ((x < z) ? x : (y < z ? z : y));
        int64_t i = lo, j = hi;
        while (i <= j) {
            while (a[i] < piv) ++i;
            while (a[j] > piv) --j;
            if (i <= j) { uint32_t t = a[i]; a[i] = a[j]; a[j] = t; ++i; --j; }
        }
        if (k <= j) hi = j;
        else if (k >= i) lo = i;
        else return a[k];
    }
    return a[k];
}

/* np.percentile(np.abs(arr), pct) with NumPy 1.26 'linear' semantics; returns the f64 value.
 * vi = (n-1)*q; lo = floor(vi); gamma = vi - lo; a = s[lo], b = s[lo+1] (s ascending);
 * vi >= n-1 -> a = b = max, gamma = vi + 1 (_get_indexes sets the index to -1);
 * _lerp: d = f32(b - a); thr = gamma >= 0.5 ? b - d*(1-gamma) : a + d*gamma   (in f64);
 * any NaN in arr -> NaN (_quantile slices_having_nans). */
int or_percentile_abs(const float* arr, int64_t n, double pct, double* thr64, float* max_abs) {
    if (!(pct >= 0.0 && pct <= 100.0)) return OR_EBADPCT;
    if (n <= 0) return OR_EEMPTY;
    uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
    if (!keys) return OR_ENOMEM;
    uint32_t kmax = 0;
    for (int64_t i = 0; i < n; ++i) { keys[i] = abs_key(arr[i]); if (keys[i] > kmax) kmax = keys[i]; }
    const double q = pct / 100.0;
    const double vi = (double)(n - 1) * q;
    double gamma;
    float a, b;
    if (vi >= (double)(n - 1)) {
        a = b = key_f(kmax);
        gamma = vi - (-1.0);
    } else {
        const double flo = floor(vi);
        const int64_t lo = (int64_t)flo;
        gamma = vi - flo;
        a = key_f(select_kth(keys, n, lo));
        b = key_f(select_kth(keys, n, lo + 1));
    }
    free(keys);
    const float d = b - a;
    double thr = (gamma >= 0.5) ? (double)b - (double)d * (1.0 - gamma) : (double)a + (double)d * gamma;
    if (kmax > 0x7F800000u) thr = (double)NAN;
    *thr64 = thr;
    if (max_abs) *max_abs = key_f(kmax);
    return OR_OK;
}

/* percentile_based_thresholding (dwt_pruning.py:25-32): out = where(|arr| < f32(thr), 0, arr) */
int or_percentile_threshold(const float* arr, int64_t n, double pct, float* out, double* thr64, float* max_abs) {
    int rc = or_percentile_abs(arr, n, pct, thr64, max_abs);
    if (rc != OR_OK) return rc;
    const float t = (float)*thr64;
    for (int64_t i = 0; i < n; ++i) out[i] = (fabsf(arr[i]) < t) ? 0.0f : arr[i];
    return OR_OK;
}

/* ------------------------------------------------ multi_resolution_analysis --- */
/* One tensor through dwt_pruning.py:53-89.  `level` is the level passed in (the caller
 * carries the clamped value across tensors exactly as :64-65 does); returns the status.
 * coeff_out (optional) receives the pre-threshold packed array. */
int or_prune_tensor(const float* in, float* out, int ndim, const int64_t* shape, int wid, int level,
                    double pct, or_result* res, float* coeff_out) {
    memset(res, 0, sizeof(*res));
    int64_t numel = 1;
    for (int i = 0; i < ndim; ++i) numel *= shape[i];
    res->numel = numel;
    int rc;
    if (ndim < 2) {
        /* :58-62 -- plain percentile mask, no wavelet validation */
        res->eff_level = level;
        res->coeff_numel = numel;
        res->packed_rows = 1;
        res->packed_cols = numel;
        rc = or_percentile_threshold(in, numel, pct, out, &res->thr64, &res->max_abs);
        if (rc != OR_OK) return res->status = rc;
        if (coeff_out) memcpy(coeff_out, in, sizeof(float) * (size_t)numel);
    } else {
        if (wid < 0 || wid >= WT_NUM_WAVELETS) return res->status = OR_EBADWAVELET;
        const int64_t H = shape[ndim - 2], W = shape[ndim - 1];
        const int64_t B = (H * W != 0) ? numel / (H * W) : 0;
        const int maxL = or_dwt_max_level(H < W ? H : W, wt_flen[wid]);
        const int L = level < maxL ? level : maxL;
        res->eff_level = L;
        if (L < 0) return res->status = OR_EBADLEVEL;
        int64_t PR, PC;
        or_packed_shape(H, W, L, &PR, &PC);
        res->packed_rows = PR;
        res->packed_cols = PC;
        res->coeff_numel = B * PR * PC;
        if (res->coeff_numel == 0) return res->status = OR_EEMPTY;
        float* P = (float*)malloc(sizeof(float) * (size_t)(B * PR * PC));
        if (!P) return res->status = OR_ENOMEM;
        rc = or_wavedec2_packed(in, B, H, W, wid, L, P);
        if (rc == OR_OK && coeff_out) memcpy(coeff_out, P, sizeof(float) * (size_t)(B * PR * PC));
        if (rc == OR_OK) rc = or_percentile_abs(P, B * PR * PC, pct, &res->thr64, &res->max_abs);
        /* waverec2 output is (B, 2R_1, 2C_1); it differs from (H, W) only for odd sizes, and the
         * reference's 4-index crop raises IndexError unless the tensor is 4-D (:79-82). */
        if (rc == OR_OK && L > 0) {
            const int hbad = 2 * ((H + 1) / 2) != H, wbad = 2 * ((W + 1) / 2) != W;
            /* ndim 2/3: the 4-index slice raises IndexError; ndim 4: crop succeeds; ndim 5: the
             * slice crops H but not W, so .view(original_shape) fails iff W mismatches;
             * ndim >= 6: neither is cropped. */
            if ((ndim < 4 && (hbad || wbad)) || (ndim == 5 && wbad) || (ndim >= 6 && (hbad || wbad)))
                rc = OR_ECROP;
        }
        if (rc == OR_OK) rc = or_waverec2_packed(P, B, H, W, wid, L, 1, (float)res->thr64, out);
        free(P);
        if (rc != OR_OK) return res->status = rc;
    }
    res->thr32 = (float)res->thr64;
    int64_t z = 0;
    for (int64_t i = 0; i < numel; ++i) z += (out[i] == 0.0f);
    res->zero_count = z;
    res->nonzero = numel - z;
    return res->status = OR_OK;
}

/* 1-D flattened mode (WTP_FLATTEN; an extension -- the reference transform is 2-D): tensors
 * with ndim >= 2 go through pywt.wavedec(w.ravel(), wavelet, 'periodization', L) with L =
 * min(level, dwt_max_level(numel, dec_len)) (pywt/_multilevel.py wavedec), coeffs_to_array
 * ([cA_L | cD_L | ... | cD_1]), the same percentile threshold as :25-32, array_to_coeffs,
 * waverec (its crop of a to len(d) when one longer, pywt/_multilevel.py waverec) and the cut
 * to numel; ndim < 2 keeps the plain-percentile branch (:58-62). */
int or_prune_tensor_flat(const float* in, float* out, int ndim, const int64_t* shape, int wid, int level,
                         double pct, or_result* res, float* coeff_out) {
    if (ndim < 2) return or_prune_tensor(in, out, ndim, shape, wid, level, pct, res, coeff_out);
    memset(res, 0, sizeof(*res));
    int64_t N = 1;
    for (int i = 0; i < ndim; ++i) N *= shape[i];
    res->numel = N;
    if (wid < 0 || wid >= WT_NUM_WAVELETS) return res->status = OR_EBADWAVELET;
    const int maxL = or_dwt_max_level(N, wt_flen[wid]);
    const int L = level < maxL ? level : maxL;
    res->eff_level = L;
    if (L < 0) return res->status = OR_EBADLEVEL;
    int64_t len[34];
    len[0] = N;
    for (int k = 1; k <= L; ++k) len[k] = (len[k - 1] + 1) / 2;
    int64_t pop = len[L];
    for (int k = 1; k <= L; ++k) pop += len[k];
    res->coeff_numel = pop;
    res->packed_rows = 1;
    res->packed_cols = pop;
    if (pop == 0) return res->status = OR_EEMPTY;
    float* P = (float*)malloc(sizeof(float) * (size_t)pop);
    float* A = (float*)malloc(sizeof(float) * (size_t)(N + 2));
    float* B = (float*)malloc(sizeof(float) * (size_t)(N + 2));
    if (!P || !A || !B) { free(P); free(A); free(B); return res->status = OR_ENOMEM; }
    /* wavedec: level k turns a_{k-1} (len[k-1]) into a_k, d_k; d_k lands at its packed offset */
    memcpy(A, in, sizeof(float) * (size_t)N);
    int64_t off = pop;
    for (int k = 1; k <= L; ++k) {
        off -= len[k]; /* cD_1 is last, cD_L right after cA_L */
        dwt1(A, 1, len[k - 1], wid, B, P + off, 1);
        float* t = A; A = B; B = t;
    }
    memcpy(P, A, sizeof(float) * (size_t)len[L]);
    if (coeff_out) memcpy(coeff_out, P, sizeof(float) * (size_t)pop);
    int rc = or_percentile_abs(P, pop, pct, &res->thr64, &res->max_abs);
    if (rc == OR_OK) {
        const float thr32 = (float)res->thr64;
        for (int64_t i = 0; i < pop; ++i) P[i] = thr_load(P[i], 1, thr32);
        if (L == 0) {
            memcpy(out, P, sizeof(float) * (size_t)N);
        } else {
            /* waverec: a starts as the packed cA_L; idwt(a[:len(d)], d) per level */
            memcpy(A, P, sizeof(float) * (size_t)len[L]);
            int64_t doff = len[L];
            for (int k = L; k >= 1; --k) {
                idwt1(A, P + doff, 1, len[k], wid, B, 1); /* 2 len[k] samples; A holds >= len[k] */
                doff += len[k];
                float* t = A; A = B; B = t;
            }
            memcpy(out, A, sizeof(float) * (size_t)N);
        }
    }
    free(P); free(A); free(B);
    if (rc != OR_OK) return res->status = rc;
    res->thr32 = (float)res->thr64;
    int64_t z = 0;
    for (int64_t i = 0; i < N; ++i) z += (out[i] == 0.0f);
    res->zero_count = z;
    res->nonzero = N - z;
    return res->status = OR_OK;
}

/* random_pruning (ResNet/random_pruning.py:49-56) restated: torch.randperm(n)[:k] with
 * Python's slice rule for k, the positions drawn from the keyed permutation of wt_perm.h
 * (torch's Philox stream is not reproduced), flatten_weights[idx] = 0, count_nonzero. */
int or_random_prune(const float* in, float* out, int64_t n, int64_t k, uint64_t seed, uint32_t tensor_id,
                    int64_t* zero_count) {
    if (n < 0) return OR_EEMPTY;
    const int64_t keff = k >= 0 ? (k < n ? k : n) : (n + k > 0 ? n + k : 0);
    if (n > 0 && out != in) memcpy(out, in, sizeof(float) * (size_t)n);
    const uint64_t key = wt_perm_key(seed, tensor_id);
    const int h = wt_perm_half_bits((uint64_t)n);
    for (int64_t j = 0; j < keff; ++j) out[wt_perm((uint64_t)j, (uint64_t)n, h, key)] = 0.0f;
    int64_t z = 0;
    for (int64_t i = 0; i < n; ++i) z += out[i] == 0.0f;
    *zero_count = z;
    return OR_OK;
}

/* A batch of independent tensors (one pruning "step" of the CPU baseline), threaded over
 * tensors with OpenMP when nthreads > 1 (the reference loop is sequential: 1 thread). */
int or_prune_batch(int ntensors, const float* const* ins, float* const* outs, const int* ndims,
                   const int64_t* shapes /* ntensors x 8 */, int wid, int level, double pct,
                   or_result* results, int nthreads) {
    int rc_all = OR_OK;
    (void)nthreads;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int t = 0; t < ntensors; ++t) {
        int rc = or_prune_tensor(ins[t], outs[t], ndims[t], shapes + 8 * t, wid, level, pct, &results[t], NULL);
        if (rc != OR_OK) rc_all = rc;
    }
    return rc_all;
}

/* ------------------------------------------------------------ synthetic data --- */
/* percentage_min_pruning (ResNet/min_weight_pruning.py:66-74): k = int(n * fraction) (C cast =
 * Python int() truncation); zero the k entries of smallest |x|; among |x| equal to the k-th
 * smallest the lowest indices go first (the rule the GPU path implements; torch.topk leaves it
 * unspecified).  Returns -6 on allocation failure, -7 when k is outside [0, n]. */
int or_min_prune(const float* in, float* out, int64_t n, double fraction, int64_t* zero_count, float* tval) {
    const double kd = (double)n * fraction;
    if (!(kd > -1.0 && kd < (double)n + 1.0)) return -7;
    const int64_t k = (int64_t)kd;
    if (out != in) memcpy(out, in, (size_t)n * sizeof(float));
    uint32_t t = 0xFFFFFFFFu;
    if (k > 0) {
        uint32_t* keys = (uint32_t*)malloc((size_t)n * sizeof(uint32_t));
        if (!keys) return -6;
        for (int64_t i = 0; i < n; ++i) keys[i] = abs_key(in[i]);
        t = select_kth(keys, n, k - 1);
        free(keys);
        int64_t below = 0;
        for (int64_t i = 0; i < n; ++i) below += abs_key(in[i]) < t;
        int64_t need = k - below;
        for (int64_t i = 0; i < n; ++i) {
            const uint32_t kk = abs_key(in[i]);
            if (kk < t) out[i] = 0.0f;
            else if (kk == t && need > 0) { out[i] = 0.0f; --need; }
        }
    }
    int64_t z = 0;
    for (int64_t i = 0; i < n; ++i) z += out[i] == 0.0f;
    *zero_count = z;
    *tval = k > 0 ? key_f(t) : 0.0f;
    return 0;
}

void or_synth_fill(float* out, int64_t n, uint64_t seed, uint32_t tensor_id, int e) {
    for (int64_t k = 0; k < n; ++k) out[k] = wt_synth_value(seed, tensor_id, (uint64_t)k, e);
}

int or_omp_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
