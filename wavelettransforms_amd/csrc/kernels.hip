/*
 * kernels.hip -- gfx950 kernels of the DWT -> percentile-threshold -> IDWT path.
 *
 * Selection (np.percentile(np.abs(coeff_arr), pct) + np.where(|c| < thr, 0, c),
 * ResNet/dwt_pruning.py:25-32) over grouped segments, one segment per tensor:
 *   k_hist     stream |x| once: 4099-bin LDS histogram of the |x| bit pattern + max key
 *   k_findbin  one block per segment: locate the bins of order statistics r0, r0+1
 *   k_compact  stream again (Infinity-Cache resident): gather the keys of those bins
 *   k_select   one block per segment: exact radix select among the candidates, NumPy 1.x
 *              linear interpolation in f64, float32 threshold
 *   k_mask     stream again: out = |x| < thr ? 0 : x, zero count        (level-0 segments)
 * Filter bank (pywt.wavedec2 / waverec2 periodization, :67-77): separable one-level passes
 * whose every output is summed in PyWavelets' exact order (csrc/wt_dwt_core.h); the
 * inverse thresholds coefficients as it loads them and the last pass crops and counts.
 * Built with -ffp-contract=off: the float32 operation order IS the parity contract.
 */
#include "wtp_internal.h"
#include "wt_synth.h"

#pragma clang fp contract(off)

namespace wtp {

/* ---------------------------------------------------------------- helpers --- */
__device__ __forceinline__ uint32_t abs_key(float x) { return __float_as_uint(x) & 0x7FFFFFFFu; }

__device__ __forceinline__ int find_seg(const SegTable& t, int b) {
    int s = 0;
    for (int i = 1; i < t.nseg; ++i)
        if (b >= t.s[i].blk_begin) s = i;
    return s;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

/* inclusive prefix sum across the 64 lanes of a wave */
__device__ __forceinline__ int64_t wave_incl_scan(int64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

/* block sum of an unsigned 64-bit value; result valid in thread 0 */
template <int THREADS>
__device__ __forceinline__ unsigned long long block_sum_u64(unsigned long long v) {
    __shared__ unsigned long long ws[THREADS / 64];
    v = wave_sum_u64(v);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned long long t = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < THREADS / 64; ++i) t += ws[i];
    return t;
}

/* 16 float4 per thread of one CHUNK (fully populated, 16-byte aligned) */
__device__ __forceinline__ void load_chunk(const float* p, float4 (&v)[16]) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int it = 0; it < 16; ++it) v[it] = p4[it * STREAM_THREADS + threadIdx.x];
}

/* ----------------------------------------------------------------- k_hist --- */
__global__ __launch_bounds__(STREAM_THREADS) void k_hist(SegTable t, uint32_t* __restrict__ hist,
                                                         SelState* __restrict__ sel) {
    __shared__ uint32_t h[NB];
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int64_t len = min((int64_t)CHUNK, sd.n - base);
    for (int i = threadIdx.x; i < NB; i += STREAM_THREADS) h[i] = 0;
    __syncthreads();
    uint32_t mx = 0;
    const float* p = sd.data + base;
    auto put = [&](float x) {
        const uint32_t k = abs_key(x);
        mx = max(mx, k);
        atomicAdd(&h[key_bin(k)], 1u);
    };
    if ((sd.flags & SEG_ALIGNED) && len == CHUNK) {
        float4 v[16];
        load_chunk(p, v);
#pragma unroll
        for (int it = 0; it < 16; ++it) { put(v[it].x); put(v[it].y); put(v[it].z); put(v[it].w); }
    } else {
        for (int64_t i = threadIdx.x; i < len; i += STREAM_THREADS) put(p[i]);
    }
    mx = wave_max_u32(mx);
    if ((threadIdx.x & 63) == 0) atomicMax(&sel[sd.slot].maxkey, mx);
    __syncthreads();
    uint32_t* g = hist + (size_t)sd.slot * NB_PAD;
    for (int i = threadIdx.x; i < NB; i += STREAM_THREADS) {
        const uint32_t c = h[i];
        if (c) atomicAdd(&g[i], c);
    }
}

/* -------------------------------------------------------------- k_findbin --- */
constexpr int FB_THREADS = 1024;
constexpr int FB_PER = (NB + FB_THREADS - 1) / FB_THREADS; /* 5 bins per thread */

__global__ __launch_bounds__(FB_THREADS) void k_findbin(SegTable t, uint32_t* __restrict__ hist,
                                                        SelState* __restrict__ sel, wtp_result* __restrict__ res) {
    __shared__ uint32_t h[FB_PER * FB_THREADS];
    __shared__ int64_t wtot[FB_THREADS / 64];
    __shared__ int64_t found[4]; /* bin0, before0, bin1, before1 */
    const SegDesc& sd = t.s[blockIdx.x];
    uint32_t* g = hist + (size_t)sd.slot * NB_PAD;
    if (threadIdx.x < 4) found[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < FB_PER * FB_THREADS; i += FB_THREADS) {
        uint32_t c = 0;
        if (i < NB) { c = g[i]; g[i] = 0; } /* read and leave the slot zeroed for the next call */
        h[i] = c;
    }
    __syncthreads();
    int64_t local = 0;
#pragma unroll
    for (int j = 0; j < FB_PER; ++j) local += h[threadIdx.x * FB_PER + j];
    const int64_t incl = wave_incl_scan(local);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    int64_t wbase = 0;
    for (int i = 0; i < wv; ++i) wbase += wtot[i];
    int64_t cum = wbase + incl - local;
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
#pragma unroll
    for (int j = 0; j < FB_PER; ++j) {
        const int b = threadIdx.x * FB_PER + j;
        const int64_t c = h[b];
        if (c) {
            if (r0 >= cum && r0 < cum + c) { found[0] = b; found[1] = cum; }
            if (r1 >= cum && r1 < cum + c) { found[2] = b; found[3] = cum; }
        }
        cum += c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        SelState& st = sel[sd.slot];
        const int bin0 = (int)found[0], bin1 = (int)found[2];
        st.a_zero = bin0 == BIN_ZERO;
        st.b_zero = bin1 == BIN_ZERO;
        if (bin1 == BIN_ZERO) {
            st.mode = MODE_ZERO;
            st.cb_lo = 1;
            st.cb_hi = 0;
            st.below = 0;
        } else {
            /* bins strictly between two adjacent order statistics are empty, so the
             * candidate range is [bin0, bin1] (or just bin1 when r0 is an exact zero) */
            const int lo = (bin0 == BIN_ZERO) ? bin1 : bin0;
            const int64_t below = (bin0 == BIN_ZERO) ? found[3] : found[1];
            const int64_t count = found[3] + (int64_t)h[bin1] - below;
            st.cb_lo = lo;
            st.cb_hi = bin1;
            st.below = below;
            st.mode = (count <= sd.cap) ? MODE_CAND : MODE_FULL;
        }
        res[sd.res].zero_count = 0;
    }
}

/* -------------------------------------------------------------- k_compact --- */
__global__ __launch_bounds__(STREAM_THREADS) void k_compact(SegTable t, SelState* __restrict__ sel,
                                                            uint32_t* __restrict__ cand) {
    __shared__ int wtot[STREAM_THREADS / 64];
    __shared__ uint32_t sbase;
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    SelState* st = sel + sd.slot;
    if (st->mode != MODE_CAND) return;
    const uint32_t blo = st->cb_lo, bhi = st->cb_hi;
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int64_t len = min((int64_t)CHUNK, sd.n - base);
    const float* p = sd.data + base;
    const bool full = (sd.flags & SEG_ALIGNED) && len == CHUNK;
    float4 v[16];
    int cnt = 0;
    auto hit = [&](float x) {
        const uint32_t b = (uint32_t)key_bin(abs_key(x));
        return b >= blo && b <= bhi;
    };
    if (full) {
        load_chunk(p, v);
#pragma unroll
        for (int it = 0; it < 16; ++it) cnt += hit(v[it].x) + hit(v[it].y) + hit(v[it].z) + hit(v[it].w);
    } else {
        for (int64_t i = threadIdx.x; i < len; i += STREAM_THREADS) cnt += hit(p[i]);
    }
    /* block exclusive scan of per-thread counts */
    const int incl = (int)wave_incl_scan(cnt);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    int off = incl - cnt, total = 0;
    for (int i = 0; i < STREAM_THREADS / 64; ++i) {
        if (i < wv) off += wtot[i];
        total += wtot[i];
    }
    if (threadIdx.x == 0) sbase = total ? atomicAdd(&st->cand_count, (uint32_t)total) : 0u;
    __syncthreads();
    if (!cnt) return;
    const int64_t cap = sd.cap;
    uint32_t* out = cand + sd.cand_off;
    int64_t pos = (int64_t)sbase + off;
    auto emit = [&](float x) {
        const uint32_t k = abs_key(x);
        const uint32_t b = (uint32_t)key_bin(k);
        if (b >= blo && b <= bhi) {
            if (pos < cap) out[pos] = k;
            ++pos;
        }
    };
    if (full) {
#pragma unroll
        for (int it = 0; it < 16; ++it) { emit(v[it].x); emit(v[it].y); emit(v[it].z); emit(v[it].w); }
    } else {
        for (int64_t i = threadIdx.x; i < len; i += STREAM_THREADS) emit(p[i]);
    }
}

/* --------------------------------------------------------------- k_select --- */
constexpr int SEL_THREADS = 1024;

/* Find the digit (8 bits) holding rank r in a 256-bin LDS histogram; one wave. */
__device__ __forceinline__ void wave_pick_digit(const uint32_t* hb, int64_t r, int* digit, int64_t* below) {
    const int lane = threadIdx.x & 63;
    const int64_t c0 = hb[4 * lane], c1 = hb[4 * lane + 1], c2 = hb[4 * lane + 2], c3 = hb[4 * lane + 3];
    const int64_t s = c0 + c1 + c2 + c3;
    const int64_t incl = wave_incl_scan(s);
    int64_t cum = incl - s;
    if (r >= cum && r < incl) {
        int d = 4 * lane;
        if (r >= cum + c0) { cum += c0; ++d;
            if (r >= cum + c1) { cum += c1; ++d;
                if (r >= cum + c2) { cum += c2; ++d; } } }
        *digit = d;
        *below = cum;
    }
}

/* Radix select of ranks ra / rb (0-based) among keys produced by get(i), i < m, one block. */
template <class Get>
__device__ void block_radix_select2(const Get& get, int64_t m, int64_t ra, int64_t rb, bool need_a, bool need_b,
                                    uint32_t* ka, uint32_t* kb) {
    __shared__ uint32_t ha[256], hb[256];
    __shared__ int dsel[2];
    __shared__ int64_t bsel[2];
    uint32_t pa = 0, pb = 0, mask = 0;
    for (int round = 0; round < 4; ++round) {
        const int shift = 24 - 8 * round;
        for (int i = threadIdx.x; i < 256; i += SEL_THREADS) { ha[i] = 0; hb[i] = 0; }
        __syncthreads();
        for (int64_t i = threadIdx.x; i < m; i += SEL_THREADS) {
            const uint32_t k = get(i);
            const uint32_t d = (k >> shift) & 255u;
            if (need_a && (k & mask) == pa) atomicAdd(&ha[d], 1u);
            if (need_b && (k & mask) == pb) atomicAdd(&hb[d], 1u);
        }
        __syncthreads();
        const int wv = threadIdx.x >> 6;
        if (wv == 0 && need_a) wave_pick_digit(ha, ra, &dsel[0], &bsel[0]);
        if (wv == 1 && need_b) wave_pick_digit(hb, rb, &dsel[1], &bsel[1]);
        __syncthreads();
        if (need_a) { pa |= (uint32_t)dsel[0] << shift; ra -= bsel[0]; }
        if (need_b) { pb |= (uint32_t)dsel[1] << shift; rb -= bsel[1]; }
        mask |= 255u << shift;
        __syncthreads();
    }
    *ka = pa;
    *kb = pb;
}

__global__ __launch_bounds__(SEL_THREADS) void k_select(SegTable t, SelState* __restrict__ sel,
                                                        const uint32_t* __restrict__ cand,
                                                        wtp_result* __restrict__ res) {
    const SegDesc& sd = t.s[blockIdx.x];
    SelState* st = sel + sd.slot;
    const int mode = st->mode;
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    uint32_t ka = 0, kb = 0;
    const bool need_a = !st->a_zero, need_b = !st->b_zero;
    int path = MODE_ZERO;
    if (mode == MODE_CAND) {
        const uint32_t* c = cand + sd.cand_off;
        const int64_t m = min((int64_t)st->cand_count, sd.cap);
        const int64_t below = st->below;
        block_radix_select2([&](int64_t i) { return c[i]; }, m, r0 - below, r1 - below, need_a, need_b, &ka, &kb);
        path = MODE_CAND;
    } else if (mode == MODE_FULL) {
        const float* x = sd.data;
        block_radix_select2([&](int64_t i) { return abs_key(x[i]); }, sd.n, r0, r1, need_a, need_b, &ka, &kb);
        path = MODE_FULL;
    }
    if (threadIdx.x == 0) {
        const uint32_t mk = st->maxkey;
        const float fa = __uint_as_float(ka), fb = __uint_as_float(kb);
        /* numpy/lib/function_base.py _lerp: diff in float32, the blend in float64 */
        const float diff = fb - fa;
        const double g = sd.gamma;
        double thr = (g >= 0.5) ? (double)fb - (double)diff * (1.0 - g) : (double)fa + (double)diff * g;
        if (mk > 0x7F800000u) thr = __longlong_as_double(0x7FF8000000000000ll); /* NaN present */
        const float thr32 = (float)thr;
        st->thr32 = thr32;
        st->key_a = ka;
        st->key_b = kb;
        st->cand_count = 0; /* leave the slot clean for the next call */
        st->maxkey = 0;
        wtp_result& r = res[sd.res];
        r.numel = sd.numel;
        r.coeff_numel = sd.n;
        r.thr64 = thr;
        r.thr32_bits = __float_as_uint(thr32);
        r.max_abs_bits = mk;
        r.eff_level = sd.eff_level;
        r.path = path;
    }
}

/* ----------------------------------------------------------------- k_mask --- */
__global__ __launch_bounds__(STREAM_THREADS) void k_mask(SegTable t, const SelState* __restrict__ sel,
                                                         wtp_result* __restrict__ res) {
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    if (!(sd.flags & SEG_MASK)) return;
    const float thr = sel[sd.slot].thr32;
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int64_t len = min((int64_t)CHUNK, sd.n - base);
    const float* p = sd.data + base;
    float* q = sd.out + base;
    unsigned long long z = 0;
    auto f = [&](float x) {
        const float y = (fabsf(x) < thr) ? 0.0f : x;
        z += (y == 0.0f);
        return y;
    };
    if ((sd.flags & SEG_ALIGNED) && len == CHUNK) {
        float4 v[16];
        load_chunk(p, v);
        float4* q4 = reinterpret_cast<float4*>(q);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            float4 y;
            y.x = f(v[it].x); y.y = f(v[it].y); y.z = f(v[it].z); y.w = f(v[it].w);
            q4[it * STREAM_THREADS + threadIdx.x] = y;
        }
    } else {
        for (int64_t i = threadIdx.x; i < len; i += STREAM_THREADS) q[i] = f(p[i]);
    }
    const unsigned long long tot = block_sum_u64<STREAM_THREADS>(z);
    if (threadIdx.x == 0 && tot) atomicAdd((unsigned long long*)&res[sd.res].zero_count, tot);
}

/* ------------------------------------------------------------ filter bank --- */
constexpr int DWT_THREADS = 256;

__device__ __forceinline__ float thr_load(float c, float thr) { return (fabsf(c) < thr) ? 0.0f : c; }

/* axis -2 analysis: in (B,R,C) -> L,H (B,Ro,C);  pywt dwtn first axis (_multidim.py:183-191) */
__global__ __launch_bounds__(DWT_THREADS) void k_dwt_cols(const float* __restrict__ in, int64_t B, int64_t R,
                                                          int64_t C, Taps tp, float* __restrict__ L,
                                                          float* __restrict__ H) {
    const int64_t Ro = (R + 1) / 2, total = B * Ro * C;
    for (int64_t idx = (int64_t)blockIdx.x * DWT_THREADS + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * DWT_THREADS) {
        const int64_t c = idx % C, t = idx / C, o = t % Ro, b = t / Ro;
        const float* x = in + b * R * C + c;
        float a, d;
        wt_ana_point(o, R, tp.F, tp.f[0], tp.f[1], [&](int64_t k) { return x[k * C]; }, a, d);
        L[idx] = a;
        H[idx] = d;
    }
}

/* axis -1 analysis of L and H -> aa (next level / packed cA), ad, da, dd into the packed array */
__global__ __launch_bounds__(DWT_THREADS) void k_dwt_rows(const float* __restrict__ L, const float* __restrict__ H,
                                                          int64_t B, int64_t Ro, int64_t C, Taps tp,
                                                          float* __restrict__ anext, float* __restrict__ P,
                                                          int64_t PR, int64_t PC, int64_t offR, int64_t offC,
                                                          int last) {
    const int64_t Co = (C + 1) / 2, total = B * Ro * Co;
    for (int64_t idx = (int64_t)blockIdx.x * DWT_THREADS + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * DWT_THREADS) {
        const int64_t o = idx % Co, t = idx / Co, r = t % Ro, b = t / Ro;
        const float* lrow = L + (b * Ro + r) * C;
        const float* hrow = H + (b * Ro + r) * C;
        float aa, ad, da, dd;
        wt_ana_point(o, C, tp.F, tp.f[0], tp.f[1], [&](int64_t k) { return lrow[k]; }, aa, ad);
        wt_ana_point(o, C, tp.F, tp.f[0], tp.f[1], [&](int64_t k) { return hrow[k]; }, da, dd);
        float* Pb = P + b * PR * PC;
        if (last) Pb[r * PC + o] = aa;
        else anext[idx] = aa;
        Pb[r * PC + offC + o] = ad;
        Pb[(offR + r) * PC + o] = da;
        Pb[(offR + r) * PC + offC + o] = dd;
    }
}

/* axis -1 synthesis: (aa,ad)->lo, (da,dd)->hi, each (B,R,2C); pywt idwtn (_multidim.py:288-309).
 * Every coefficient read from the packed array is thresholded on load (np.where of :31). */
__global__ __launch_bounds__(DWT_THREADS) void k_idwt_rows(const float* __restrict__ a, int64_t a_bs, int64_t lda,
                                                           int a_from_P, const float* __restrict__ P, int64_t PR,
                                                           int64_t PC, int64_t offR, int64_t offC, int64_t B,
                                                           int64_t R, int64_t C, Taps tp, const float* thrp,
                                                           float* __restrict__ lo, float* __restrict__ hi) {
    const float thr = thrp ? *thrp : 0.0f; /* |c| < 0 never holds: no threshold */
    const int64_t C2 = 2 * C, total = B * R * C2;
    for (int64_t idx = (int64_t)blockIdx.x * DWT_THREADS + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * DWT_THREADS) {
        const int64_t n = idx % C2, t = idx / C2, r = t % R, b = t / R;
        const float* Pb = P + b * PR * PC;
        const float* arow = a_from_P ? Pb + r * PC : a + b * a_bs + r * lda;
        const float* adr = Pb + r * PC + offC;
        const float* dar = Pb + (offR + r) * PC;
        const float* ddr = Pb + (offR + r) * PC + offC;
        const float* rlo = tp.f[2];
        const float* rhi = tp.f[3];
        float vlo, vhi;
        if (a_from_P)
            vlo = wt_syn_point(n, C, tp.F, rlo, rhi, [&](int64_t k) { return thr_load(arow[k], thr); },
                               [&](int64_t k) { return thr_load(adr[k], thr); });
        else
            vlo = wt_syn_point(n, C, tp.F, rlo, rhi, [&](int64_t k) { return arow[k]; },
                               [&](int64_t k) { return thr_load(adr[k], thr); });
        vhi = wt_syn_point(n, C, tp.F, rlo, rhi, [&](int64_t k) { return thr_load(dar[k], thr); },
                           [&](int64_t k) { return thr_load(ddr[k], thr); });
        lo[idx] = vlo;
        hi[idx] = vhi;
    }
}

/* axis -2 synthesis: lo,hi (B,R,C2) -> y (B,outH,outW) with outH <= 2R, outW <= C2 (crop);
 * optionally counts exact zeros of y (the final level writes the pruned weights). */
__global__ __launch_bounds__(DWT_THREADS) void k_idwt_cols(const float* __restrict__ lo, const float* __restrict__ hi,
                                                           int64_t B, int64_t R, int64_t C2, Taps tp,
                                                           float* __restrict__ y, int64_t outH, int64_t outW,
                                                           unsigned long long* zero_count) {
    const int64_t total = B * outH * outW;
    unsigned long long z = 0;
    for (int64_t idx = (int64_t)blockIdx.x * DWT_THREADS + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * DWT_THREADS) {
        const int64_t n = idx % outW, t = idx / outW, m = t % outH, b = t / outH;
        const float* lc = lo + b * R * C2 + n;
        const float* hc = hi + b * R * C2 + n;
        const float v = wt_syn_point(m, R, tp.F, tp.f[2], tp.f[3], [&](int64_t k) { return lc[k * C2]; },
                                     [&](int64_t k) { return hc[k * C2]; });
        y[idx] = v;
        z += (v == 0.0f);
    }
    if (zero_count) {
        const unsigned long long tot = block_sum_u64<DWT_THREADS>(z);
        if (threadIdx.x == 0 && tot) atomicAdd(zero_count, tot);
    }
}

__global__ __launch_bounds__(DWT_THREADS) void k_copy_threshold(const float* __restrict__ P, float* __restrict__ out,
                                                                int64_t n, const float* thrp,
                                                                unsigned long long* zero_count) {
    const float thr = thrp ? *thrp : 0.0f;
    unsigned long long z = 0;
    for (int64_t i = (int64_t)blockIdx.x * DWT_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * DWT_THREADS) {
        const float v = thr_load(P[i], thr);
        out[i] = v;
        z += (v == 0.0f);
    }
    if (zero_count) {
        const unsigned long long tot = block_sum_u64<DWT_THREADS>(z);
        if (threadIdx.x == 0 && tot) atomicAdd(zero_count, tot);
    }
}

__global__ __launch_bounds__(DWT_THREADS) void k_synth(float* __restrict__ out, int64_t n, uint64_t seed, uint32_t tid,
                                                       int e) {
    for (int64_t i = (int64_t)blockIdx.x * DWT_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * DWT_THREADS)
        out[i] = wt_synth_value(seed, tid, (uint64_t)i, e);
}

/* ---------------------------------------------------------------- launchers --- */
static inline unsigned grid_for(int64_t total) {
    int64_t g = (total + DWT_THREADS - 1) / DWT_THREADS;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (unsigned)g;
}

void launch_hist(const SegTable& t, uint32_t* hist, SelState* sel, hipStream_t s) {
    hipLaunchKernelGGL(k_hist, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, hist, sel);
}
void launch_findbin(const SegTable& t, uint32_t* hist, SelState* sel, wtp_result* res, hipStream_t s) {
    hipLaunchKernelGGL(k_findbin, dim3(t.nseg), dim3(FB_THREADS), 0, s, t, hist, sel, res);
}
void launch_compact(const SegTable& t, SelState* sel, uint32_t* cand, hipStream_t s) {
    hipLaunchKernelGGL(k_compact, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, sel, cand);
}
void launch_select(const SegTable& t, SelState* sel, const uint32_t* cand, wtp_result* res, hipStream_t s) {
    hipLaunchKernelGGL(k_select, dim3(t.nseg), dim3(SEL_THREADS), 0, s, t, sel, cand, res);
}
void launch_mask(const SegTable& t, const SelState* sel, wtp_result* res, hipStream_t s) {
    hipLaunchKernelGGL(k_mask, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, sel, res);
}
void launch_dwt_cols(const float* in, int64_t B, int64_t R, int64_t C, const Taps& tp, float* L, float* H,
                     hipStream_t s) {
    hipLaunchKernelGGL(k_dwt_cols, dim3(grid_for(B * ((R + 1) / 2) * C)), dim3(DWT_THREADS), 0, s, in, B, R, C, tp,
                       L, H);
}
void launch_dwt_rows(const float* L, const float* H, int64_t B, int64_t Ro, int64_t C, const Taps& tp, float* anext,
                     float* P, int64_t PR, int64_t PC, int64_t offR, int64_t offC, int last, hipStream_t s) {
    hipLaunchKernelGGL(k_dwt_rows, dim3(grid_for(B * Ro * ((C + 1) / 2))), dim3(DWT_THREADS), 0, s, L, H, B, Ro, C,
                       tp, anext, P, PR, PC, offR, offC, last);
}
void launch_idwt_rows(const float* a, int64_t a_bs, int64_t lda, int a_from_P, const float* P, int64_t PR, int64_t PC,
                      int64_t offR, int64_t offC, int64_t B, int64_t R, int64_t C, const Taps& tp, const float* thr,
                      float* lo, float* hi, hipStream_t s) {
    hipLaunchKernelGGL(k_idwt_rows, dim3(grid_for(B * R * 2 * C)), dim3(DWT_THREADS), 0, s, a, a_bs, lda, a_from_P,
                       P, PR, PC, offR, offC, B, R, C, tp, thr, lo, hi);
}
void launch_idwt_cols(const float* lo, const float* hi, int64_t B, int64_t R, int64_t C, const Taps& tp, float* y,
                      int64_t outH, int64_t outW, unsigned long long* zero_count, hipStream_t s) {
    hipLaunchKernelGGL(k_idwt_cols, dim3(grid_for(B * outH * outW)), dim3(DWT_THREADS), 0, s, lo, hi, B, R, 2 * C, tp,
                       y, outH, outW, zero_count);
}
void launch_copy_threshold(const float* P, float* out, int64_t n, const float* thr, unsigned long long* zc,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_copy_threshold, dim3(grid_for(n)), dim3(DWT_THREADS), 0, s, P, out, n, thr, zc);
}
void launch_synth(float* out, int64_t n, uint64_t seed, uint32_t tid, int e, hipStream_t s) {
    hipLaunchKernelGGL(k_synth, dim3(grid_for(n)), dim3(DWT_THREADS), 0, s, out, n, seed, tid, e);
}

}  // namespace wtp
