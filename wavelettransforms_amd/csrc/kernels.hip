/*
 * kernels.hip -- gfx950 kernels of the DWT -> percentile-threshold -> IDWT path.
 *
 * Selection (np.percentile(np.abs(coeff_arr), pct) + np.where(|c| < thr, 0, c),
 * ResNet/dwt_pruning.py:25-32) over grouped segments, one segment per tensor, on the float32
 * bit pattern of |x| (a key monotone in |x|; NaN sorts last as in np.partition):
 *   k_sample   one block per segment: 32768 sampled keys -> window [kl, kh] bracketing the
 *              order statistics r0, r0+1 (exact keys when the segment fits in the sample)
 *   k_collect  stream once: count keys < kl, == kl, == kh; gather keys inside (kl, kh)
 *              with a 256-bin sub-histogram; max key
 *   k_select   one block per segment: exact radix select of both ranks (inside candidates,
 *              or the whole segment if the window missed), NumPy 1.x _lerp in f64
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

/* --------------------------------------------------------- radix select --- */
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

/* Exact radix select (8-bit digits, MSB first) of ranks ra / rb (0-based, ascending) among
 * the keys get(i), i < m, that satisfy keep(key); one block of THREADS threads. */
template <int THREADS, class Get, class Keep>
__device__ void block_radix_select2(const Get& get, const Keep& keep, int64_t m, int64_t ra, int64_t rb,
                                    bool need_a, bool need_b, uint32_t* ka, uint32_t* kb) {
    __shared__ uint32_t ha[256], hb[256];
    __shared__ int dsel[2];
    __shared__ int64_t bsel[2];
    uint32_t pa = 0, pb = 0, mask = 0;
    for (int round = 0; round < 4; ++round) {
        const int shift = 24 - 8 * round;
        for (int i = threadIdx.x; i < 256; i += THREADS) { ha[i] = 0; hb[i] = 0; }
        __syncthreads();
        for (int64_t i = threadIdx.x; i < m; i += THREADS) {
            const uint32_t k = get(i);
            if (!keep(k)) continue;
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

/* --------------------------------------------------------------- k_sample --- */
constexpr int SAMPLE_THREADS = 1024;

__global__ __launch_bounds__(SAMPLE_THREADS) void k_sample(SegTable t, SelState* __restrict__ sel,
                                                           wtp_result* __restrict__ res) {
    __shared__ uint32_t sk[M_SAMPLE]; /* 128 KiB */
    const SegDesc& sd = t.s[blockIdx.x];
    const int64_t n = sd.n;
    const bool exact = n <= M_SAMPLE;
    const int m = exact ? (int)n : M_SAMPLE;
    const float* x = sd.data;
    if (exact) {
        for (int i = threadIdx.x; i < m; i += SAMPLE_THREADS) sk[i] = abs_key(x[i]);
    } else {
        constexpr int G = M_SAMPLE / SAMPLE_GROUP;
        for (int i = threadIdx.x; i < m; i += SAMPLE_THREADS) {
            const int64_t g = i / SAMPLE_GROUP, j = i % SAMPLE_GROUP;
            sk[i] = abs_key(x[g * (n - SAMPLE_GROUP) / (G - 1) + j]);
        }
    }
    __syncthreads();
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    int64_t sa, sb;
    bool lo_open = false, hi_open = false;
    if (exact) {
        sa = r0;
        sb = r1;
    } else {
        /* sample ranks bracketing r0 and r1 with a 6-sigma (+24) binomial margin */
        const double p = (double)r0 / (double)(n - 1);
        const double s0 = p * (double)(m - 1), s1 = (double)r1 / (double)(n - 1) * (double)(m - 1);
        const double d = 6.0 * sqrt((double)m * p * (1.0 - p)) + 24.0;
        sa = (int64_t)floor(s0 - d);
        sb = (int64_t)ceil(s1 + d);
        if (sa < 0) { lo_open = true; sa = 0; }
        if (sb > m - 1) { hi_open = true; sb = m - 1; }
    }
    uint32_t ka, kb;
    block_radix_select2<SAMPLE_THREADS>([&](int64_t i) { return sk[i]; }, [](uint32_t) { return true; }, m, sa, sb,
                                        !lo_open, !hi_open, &ka, &kb);
    if (threadIdx.x == 0) {
        SelState& st = sel[sd.slot];
        const uint32_t kl = lo_open ? 0u : ka;
        const uint32_t kh = hi_open ? 0xFFFFFFFFu : kb;
        st.kl = kl;
        st.kh = kh;
        uint32_t sh = 0;
        if (kh > kl + 1) {
            const uint32_t R = kh - kl - 1;
            const int bits = 32 - __clz(R);
            sh = bits > 8 ? bits - 8 : 0;
        }
        st.shift = sh;
        res[sd.res].zero_count = 0;
    }
}

/* -------------------------------------------------------------- k_collect --- */
__global__ __launch_bounds__(STREAM_THREADS) void k_collect(SegTable t, SelState* __restrict__ sel,
                                                            uint32_t* __restrict__ cand) {
    __shared__ uint32_t lsub[NSUB];
    __shared__ int wtot[STREAM_THREADS / 64];
    __shared__ uint32_t sbase;
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int64_t len = min((int64_t)CHUNK, sd.n - base);
    const float* p = sd.data + base;
    const bool full = (sd.flags & SEG_ALIGNED) && len == CHUNK;
    float4 v[16];
    if (full) load_chunk(p, v); /* issue the stream loads before the window state arrives */
    SelState* st = sel + sd.slot;
    const uint32_t kl = st->kl, kh = st->kh, sh = st->shift;
    for (int i = threadIdx.x; i < NSUB; i += STREAM_THREADS) lsub[i] = 0;
    __syncthreads();
    uint32_t below = 0, eql = 0, eqh = 0, mx = 0;
    int cnt = 0;
    auto tally = [&](float xv) {
        const uint32_t k = abs_key(xv);
        mx = max(mx, k);
        below += k < kl;
        if (k == kl) ++eql;
        else if (k == kh) ++eqh;
        else if (k > kl && k < kh) { ++cnt; atomicAdd(&lsub[(k - kl - 1) >> sh], 1u); }
    };
    if (full) {
#pragma unroll
        for (int it = 0; it < 16; ++it) { tally(v[it].x); tally(v[it].y); tally(v[it].z); tally(v[it].w); }
    } else {
        for (int64_t i = threadIdx.x; i < len; i += STREAM_THREADS) tally(p[i]);
    }
    /* counters: one atomic per block each */
    const unsigned long long tb = block_sum_u64<STREAM_THREADS>(below);
    const unsigned long long tl = block_sum_u64<STREAM_THREADS>(eql);
    const unsigned long long th = block_sum_u64<STREAM_THREADS>(eqh);
    mx = wave_max_u32(mx);
    if ((threadIdx.x & 63) == 0) atomicMax(&st->maxkey, mx);
    if (threadIdx.x == 0) {
        if (tb) atomicAdd(&st->below, tb);
        if (tl) atomicAdd(&st->eq_lo, tl);
        if (th) atomicAdd(&st->eq_hi, th);
    }
    /* inside keys: block exclusive scan, one returning atomic per block, then emit */
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
    for (int i = threadIdx.x; i < NSUB; i += STREAM_THREADS) {
        const uint32_t c = lsub[i];
        if (c) atomicAdd(&st->sub[i], c);
    }
    __syncthreads();
    if (!cnt) return;
    const int64_t cap = sd.cap;
    uint32_t* out = cand + sd.cand_off;
    int64_t pos = (int64_t)sbase + off;
    auto emit = [&](float xv) {
        const uint32_t k = abs_key(xv);
        if (k > kl && k < kh && k != kl && k != kh) {
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
constexpr int SEL_STAGE = 16384; /* filtered candidates staged in LDS */

__global__ __launch_bounds__(SEL_THREADS) void k_select(SegTable t, SelState* __restrict__ sel,
                                                        const uint32_t* __restrict__ cand,
                                                        wtp_result* __restrict__ res, float* __restrict__ thr_out) {
    __shared__ uint32_t stage[SEL_STAGE];
    __shared__ uint32_t nstage;
    __shared__ int sbin[2];
    __shared__ int64_t sbefore[2];
    const SegDesc& sd = t.s[blockIdx.x];
    SelState* st = sel + sd.slot;
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    const int64_t below = (int64_t)st->below, eql = (int64_t)st->eq_lo, eqh = (int64_t)st->eq_hi;
    const int64_t ncand = st->cand_count;
    const uint32_t kl = st->kl, kh = st->kh, sh = st->shift;
    /* class of a rank: 0 miss, 1 == kl, 2 inside, 3 == kh */
    auto classify = [&](int64_t r, int64_t* j) {
        if (r < below) return 0;
        r -= below;
        if (r < eql) return 1;
        r -= eql;
        if (r < ncand) { *j = r; return 2; }
        r -= ncand;
        if (r < eqh) return 3;
        return 0;
    };
    int64_t ja = 0, jb = 0;
    const int ca = classify(r0, &ja), cb = classify(r1, &jb);
    uint32_t ka = 0, kb = 0;
    int path;
    if (ca == 0 || cb == 0 || ncand > sd.cap) {
        /* the window missed (or overflowed): exact full radix select over the population */
        const float* x = sd.data;
        block_radix_select2<SEL_THREADS>([&](int64_t i) { return abs_key(x[i]); }, [](uint32_t) { return true; },
                                         sd.n, r0, r1, true, true, &ka, &kb);
        path = MODE_FULL;
    } else {
        ka = (ca == 1) ? kl : kh;
        kb = (cb == 1) ? kl : kh;
        path = MODE_WINDOW;
        if (ca == 2 || cb == 2) {
            path = MODE_CAND;
            /* sub-bins holding the inside ranks (bins between two adjacent ranks are empty) */
            if (threadIdx.x < 64) {
                if (ca == 2) wave_pick_digit(st->sub, ja, &sbin[0], &sbefore[0]);
                if (cb == 2) wave_pick_digit(st->sub, jb, &sbin[1], &sbefore[1]);
            }
            if (threadIdx.x == 0) nstage = 0;
            __syncthreads();
            const int blo = (ca == 2) ? sbin[0] : sbin[1];
            const int bhi = (cb == 2) ? sbin[1] : sbin[0];
            const int64_t before = (ca == 2) ? sbefore[0] : sbefore[1];
            int64_t nf = 0;
            for (int b = blo; b <= bhi; ++b) nf += st->sub[b];
            const uint32_t* c = cand + sd.cand_off;
            auto keep = [&](uint32_t k) {
                const int b = (int)((k - kl - 1) >> sh);
                return b >= blo && b <= bhi;
            };
            uint32_t xa, xb;
            if (nf <= SEL_STAGE) {
                for (int64_t i = threadIdx.x; i < ncand; i += SEL_THREADS) {
                    const uint32_t k = c[i];
                    if (keep(k)) stage[atomicAdd(&nstage, 1u)] = k;
                }
                __syncthreads();
                block_radix_select2<SEL_THREADS>([&](int64_t i) { return stage[i]; }, [](uint32_t) { return true; },
                                                 (int64_t)nstage, ja - before, jb - before, ca == 2, cb == 2, &xa, &xb);
            } else {
                block_radix_select2<SEL_THREADS>([&](int64_t i) { return c[i]; }, keep, ncand, ja - before,
                                                 jb - before, ca == 2, cb == 2, &xa, &xb);
            }
            if (ca == 2) ka = xa;
            if (cb == 2) kb = xb;
        }
    }
    __syncthreads();
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
        thr_out[sd.res] = thr32; /* per tensor, read by the inverse transform */
        st->key_a = ka;
        st->key_b = kb;
        st->mode = path;
        /* leave the slot clean for the next call */
        st->cand_count = 0;
        st->maxkey = 0;
        st->below = 0;
        st->eq_lo = 0;
        st->eq_hi = 0;
        wtp_result& r = res[sd.res];
        r.numel = sd.numel;
        r.coeff_numel = sd.n;
        r.thr64 = thr;
        r.thr32_bits = __float_as_uint(thr32);
        r.max_abs_bits = mk;
        r.eff_level = sd.eff_level;
        r.path = path;
    }
    for (int i = threadIdx.x; i < NSUB; i += SEL_THREADS) st->sub[i] = 0;
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

void launch_sample(const SegTable& t, SelState* sel, wtp_result* res, hipStream_t s) {
    hipLaunchKernelGGL(k_sample, dim3(t.nseg), dim3(SAMPLE_THREADS), 0, s, t, sel, res);
}
void launch_collect(const SegTable& t, SelState* sel, uint32_t* cand, hipStream_t s) {
    hipLaunchKernelGGL(k_collect, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, sel, cand);
}
void launch_select(const SegTable& t, SelState* sel, const uint32_t* cand, wtp_result* res, float* thr_out,
                   hipStream_t s) {
    hipLaunchKernelGGL(k_select, dim3(t.nseg), dim3(SEL_THREADS), 0, s, t, sel, cand, res, thr_out);
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
