/*
 * kernels.hip -- gfx950 kernels of the DWT -> percentile-threshold -> IDWT path.
 *
 * Selection (np.percentile(np.abs(coeff_arr), pct) + np.where(|c| < thr, 0, c),
 * ResNet/dwt_pruning.py:25-32) over grouped segments, one segment per tensor, on the float32
 * bit pattern of |x| (a key monotone in |x|; NaN sorts last as in np.partition):
 *   k_sample   one block per segment: 32768 sampled keys histogrammed into 1/128-octave
 *              bins -> window [kl, kh] bracketing the order statistics r0, r0+1
 *   k_collect  stream once: count keys < kl, == kl, == kh, == 0; scatter the keys inside
 *              (kl, kh) into key-range buckets (one run per bucket per block); max key
 *   k_select   one block per segment: exact radix select of both ranks (from the one or two
 *              buckets that hold them, or the whole segment if the window missed), NumPy 1.x
 *              _lerp in f64, and the
 *              exact zero count of the level-0 output (from the window counts)
 *   k_mask     stream again: out = |x| < thr ? 0 : x                    (level-0 segments)
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
    int s = 0; /* blk_begin[0] == 0; entries past nseg hold INT32_MAX */
#pragma unroll
    for (int i = 1; i < SEG_PER_LAUNCH; ++i) s += b >= t.blk_begin[i];
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

/* the float4 part of a ragged chunk (len4 float4s), all loads issued up front */
__device__ __forceinline__ void load_chunk_part(const float* p, int len4, float4 (&v)[16]) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int j = it * STREAM_THREADS + threadIdx.x;
        v[it] = j < len4 ? p4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
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

/* --------------------------------------------------------------- k_sample --- */
constexpr int SAMPLE_THREADS = 1024;
constexpr int SAMPLE_PER = M_SAMPLE / SAMPLE_THREADS; /* 32 */
constexpr int FB_PER = (NB + SAMPLE_THREADS - 1) / SAMPLE_THREADS; /* 5 bins per thread */

__global__ __launch_bounds__(SAMPLE_THREADS) void k_sample(SegTable t, SelState* __restrict__ sel) {
    __shared__ uint32_t h[FB_PER * SAMPLE_THREADS];
    __shared__ int64_t wtot[SAMPLE_THREADS / 64];
    __shared__ int64_t found[4]; /* bin(sa), bin(sb) */
    const SegDesc& sd = t.s[blockIdx.x];
    const int64_t n = sd.n;
    const bool exact = n <= M_SAMPLE;
    const int m = exact ? (int)n : M_SAMPLE;
    const float* x = sd.data;
    /* sampled keys: groups of SAMPLE_GROUP contiguous floats spread evenly over the segment */
    uint32_t k[SAMPLE_PER];
    const double step = exact ? 0.0 : (double)(n - SAMPLE_GROUP) / (double)(M_SAMPLE / SAMPLE_GROUP - 1);
#pragma unroll
    for (int j = 0; j < SAMPLE_PER; ++j) {
        const int i = j * SAMPLE_THREADS + threadIdx.x;
        int64_t pos = i;
        if (!exact) pos = (int64_t)((double)(i / SAMPLE_GROUP) * step) + (i % SAMPLE_GROUP);
        k[j] = (i < m) ? abs_key(x[pos]) : 0xFFFFFFFFu;
    }
    for (int i = threadIdx.x; i < FB_PER * SAMPLE_THREADS; i += SAMPLE_THREADS) h[i] = 0;
    if (threadIdx.x < 4) found[threadIdx.x] = -1;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SAMPLE_PER; ++j)
        if (k[j] != 0xFFFFFFFFu) atomicAdd(&h[key_bin(k[j])], 1u);
    __syncthreads();
    /* sample ranks bracketing r0 and r1 (exact ranks when the whole segment was sampled) */
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    int64_t sa, sb;
    if (exact) {
        sa = r0;
        sb = r1;
    } else {
        const double p = (double)r0 / (double)(n - 1);
        const double s0 = p * (double)(m - 1), s1 = (double)r1 / (double)(n - 1) * (double)(m - 1);
        const double d = 6.0 * sqrt((double)m * p * (1.0 - p)) + 24.0;
        sa = (int64_t)floor(s0 - d);
        sb = (int64_t)ceil(s1 + d);
    }
    int64_t local = 0;
#pragma unroll
    for (int j = 0; j < FB_PER; ++j) local += h[threadIdx.x * FB_PER + j];
    const int64_t incl = wave_incl_scan(local);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    int64_t cum = incl - local;
    for (int i = 0; i < wv; ++i) cum += wtot[i];
#pragma unroll
    for (int j = 0; j < FB_PER; ++j) {
        const int b = threadIdx.x * FB_PER + j;
        const int64_t c = h[b];
        if (c) {
            if (sa >= cum && sa < cum + c) found[0] = b;
            if (sb >= cum && sb < cum + c) found[1] = b;
        }
        cum += c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        SelState& st = sel[sd.slot];
        const uint32_t kl = (sa < 0 || found[0] < 0) ? 0u : bin_lo_key((int)found[0]);
        const uint32_t kh = (sb >= m || found[1] < 0) ? 0xFFFFFFFFu : bin_hi_key((int)found[1]);
        st.kl = kl;
        st.kh = kh;
        uint32_t sh = 0;
        if (kh > kl + 1) {
            const uint32_t R = kh - kl - 1; /* inside keys: (key - kl - 1) in [0, R) */
            const int bits = 32 - __clz(R);
            sh = bits > sd.nsub_log2 ? bits - sd.nsub_log2 : 0;
        }
        st.shift = sh;
    }
}

/* -------------------------------------------------------------- k_collect --- */
constexpr int STAGE_CAP = 4096; /* inside keys staged per block before the bucket scatter */

__global__ __launch_bounds__(STREAM_THREADS) void k_collect(SegTable t, SelState* __restrict__ sel,
                                                            uint32_t* __restrict__ cand) {
    __shared__ uint32_t lsub[NSUB_MAX];  /* this block's keys per bucket, then the running offset */
    __shared__ uint32_t lbase[NSUB_MAX]; /* reserved start of this block's run in each bucket     */
    __shared__ uint32_t stage[STAGE_CAP];
    __shared__ uint32_t wred[STREAM_THREADS / 64][5];
    __shared__ int wtot[STREAM_THREADS / 64];
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int len = (int)min((int64_t)CHUNK, sd.n - base);
    const float* p = sd.data + base;
    const bool vec = (sd.flags & SEG_ALIGNED) != 0;
    const int len4 = vec ? len >> 2 : 0;
    float4 v[16];
    if (vec) load_chunk_part(p, len4, v); /* stream loads first: the window state arrives meanwhile */
    SelState* st = sel + sd.slot;
    const uint32_t kl = st->kl, kh = st->kh, sh = st->shift;
    const int nsub = 1 << sd.nsub_log2;
    for (int i = threadIdx.x; i < nsub; i += STREAM_THREADS) lsub[i] = 0;
    uint32_t below = 0, eql = 0, eqh = 0, zer = 0, mx = 0;
    int cnt = 0;
    auto inside = [&](uint32_t k) { return k > kl && k < kh; };
    auto tally = [&](float xv) {
        const uint32_t k = abs_key(xv);
        mx = max(mx, k);
        below += k < kl;
        eql += k == kl;
        eqh += (k == kh) & (kh != kl);
        zer += k == 0;
        cnt += inside(k);
    };
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        if (it * STREAM_THREADS + (int)threadIdx.x < len4) {
            tally(v[it].x); tally(v[it].y); tally(v[it].z); tally(v[it].w);
        }
    }
    for (int i = len4 * 4 + threadIdx.x; i < len; i += STREAM_THREADS) tally(p[i]);
    /* one block reduction for the five counters */
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    {
        uint32_t r[5] = {below, eql, eqh, zer, mx};
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) r[q] += (uint32_t)__shfl_xor((int)r[q], o, 64);
            r[4] = max(r[4], (uint32_t)__shfl_xor((int)r[4], o, 64));
        }
        if (lane == 0)
            for (int q = 0; q < 5; ++q) wred[wv][q] = r[q];
    }
    const int incl = (int)wave_incl_scan(cnt);
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    int off = incl - cnt, total = 0;
    for (int i = 0; i < STREAM_THREADS / 64; ++i) {
        if (i < wv) off += wtot[i];
        total += wtot[i];
    }
    if (threadIdx.x == 0) {
        unsigned long long a[4] = {0, 0, 0, 0};
        uint32_t m2 = 0;
        for (int w = 0; w < STREAM_THREADS / 64; ++w) {
            for (int q = 0; q < 4; ++q) a[q] += wred[w][q];
            m2 = max(m2, wred[w][4]);
        }
        if (a[0]) atomicAdd(&st->below, a[0]);
        if (a[1]) atomicAdd(&st->eq_lo, a[1]);
        if (a[2]) atomicAdd(&st->eq_hi, a[2]);
        if (a[3]) atomicAdd(&st->zeros, a[3]);
        atomicMax(&st->maxkey, m2);
        if (total > STAGE_CAP) atomicOr(&st->overflow, 1u);
    }
    if (total == 0 || total > STAGE_CAP) return; /* uniform; an overflow sends k_select to the full scan */
    /* stage this block's inside keys, count them per bucket */
    if (cnt) {
        int pos = off;
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            if (it * STREAM_THREADS + (int)threadIdx.x < len4) {
                const uint32_t k4[4] = {abs_key(v[it].x), abs_key(v[it].y), abs_key(v[it].z), abs_key(v[it].w)};
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (inside(k4[c])) stage[pos++] = k4[c];
            }
        }
        for (int i = len4 * 4 + threadIdx.x; i < len; i += STREAM_THREADS) {
            const uint32_t k = abs_key(p[i]);
            if (inside(k)) stage[pos++] = k;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += STREAM_THREADS) atomicAdd(&lsub[(stage[i] - kl - 1) >> sh], 1u);
    __syncthreads();
    /* reserve one contiguous run per non-empty bucket (one returning atomic per bucket) */
    for (int b = threadIdx.x; b < nsub; b += STREAM_THREADS) {
        const uint32_t c = lsub[b];
        lbase[b] = c ? atomicAdd(&st->sub[b], c) : 0u;
        lsub[b] = 0;
    }
    __syncthreads();
    const int64_t bcap = sd.bucket_cap;
    uint32_t* out = cand + sd.cand_off;
    for (int i = threadIdx.x; i < total; i += STREAM_THREADS) {
        const uint32_t k = stage[i];
        const uint32_t b = (k - kl - 1) >> sh;
        const uint32_t at = lbase[b] + atomicAdd(&lsub[b], 1u);
        if (at < bcap) out[(int64_t)b * bcap + at] = k; /* counted beyond capacity: k_select sees it */
    }
}

/* --------------------------------------------------------------- k_select --- */
constexpr int SEL_THREADS = 1024;
constexpr int SEL_STAGE = 16384; /* filtered candidates staged in LDS */

/* Radix select of ranks ra / rb among keys that all lie in [lo, hi]: the bits above the
 * highest bit where lo and hi differ are common and skipped (concentrated digits are what
 * makes an MSB-first LDS histogram contend). */
template <int THREADS, class Get, class Keep>
__device__ void select_in_range(const Get& get, const Keep& keep, int64_t m, uint32_t lo, uint32_t hi, int64_t ra,
                                int64_t rb, bool need_a, bool need_b, uint32_t* ka, uint32_t* kb) {
    __shared__ uint32_t ha[256], hb[256];
    __shared__ int dsel[2];
    __shared__ int64_t bsel[2];
    const uint32_t diff = lo ^ hi;
    int top = diff ? 31 - __clz(diff) : -1; /* highest unknown bit */
    const uint32_t known = top >= 31 ? 0u : ~((2u << top) - 1u);
    uint32_t pa = lo & known, pb = lo & known, mask = known;
    while (top >= 0) {
        const int width = top + 1 < 8 ? top + 1 : 8;
        const int shift = top + 1 - width;
        const uint32_t dm = (1u << width) - 1u;
        for (int i = threadIdx.x; i < 256; i += THREADS) { ha[i] = 0; hb[i] = 0; }
        __syncthreads();
        for (int64_t i = threadIdx.x; i < m; i += THREADS) {
            const uint32_t k = get(i);
            if (!keep(k)) continue;
            const uint32_t d = (k >> shift) & dm;
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
        mask |= dm << shift;
        top = shift - 1;
        __syncthreads();
    }
    *ka = pa;
    *kb = pb;
}

/* count of keys < tk among get(i), block-wide; valid in every thread */
template <int THREADS, class Get>
__device__ int64_t block_count_below(const Get& get, int64_t m, uint32_t tk) {
    __shared__ unsigned long long acc;
    if (threadIdx.x == 0) acc = 0;
    __syncthreads();
    unsigned long long c = 0;
    for (int64_t i = threadIdx.x; i < m; i += THREADS) c += get(i) < tk;
    c = wave_sum_u64(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&acc, c);
    __syncthreads();
    const int64_t r = (int64_t)acc;
    __syncthreads();
    return r;
}

/* inclusive prefix over nsub bucket counts held in global memory; one wave.  Returns the
 * total and, for rank r (if found), its bucket and the count before it. */
__device__ __forceinline__ int64_t wave_bucket_total(const uint32_t* sub, int nsub) {
    const int lane = threadIdx.x & 63;
    unsigned long long s = 0;
    for (int b = lane; b < nsub; b += 64) s += sub[b];
    return (int64_t)wave_sum_u64(s);
}

__device__ __forceinline__ void wave_find_bucket(const uint32_t* sub, int nsub, int64_t r, int* bucket,
                                                 int64_t* before) {
    const int lane = threadIdx.x & 63;
    const int per = nsub / 64; /* 1..16 consecutive buckets per lane */
    int64_t s = 0;
    for (int j = 0; j < per; ++j) s += sub[lane * per + j];
    const int64_t incl = wave_incl_scan(s);
    int64_t cum = incl - s;
    if (r >= cum && r < incl) {
        for (int j = 0; j < per; ++j) {
            const int64_t c = sub[lane * per + j];
            if (r < cum + c) { *bucket = lane * per + j; *before = cum; break; }
            cum += c;
        }
    }
}

__global__ __launch_bounds__(SEL_THREADS) void k_select(SegTable t, SelState* __restrict__ sel,
                                                        const uint32_t* __restrict__ cand,
                                                        wtp_result* __restrict__ res, float* __restrict__ thr_out) {
    __shared__ uint32_t stage[SEL_STAGE];
    __shared__ int sbin[2];
    __shared__ int64_t sbefore[2];
    __shared__ int64_t s_ncand;
    const SegDesc& sd = t.s[blockIdx.x];
    SelState* st = sel + sd.slot;
    const int nsub = 1 << sd.nsub_log2;
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    const int64_t below = (int64_t)st->below, eql = (int64_t)st->eq_lo, eqh = (int64_t)st->eq_hi;
    const uint32_t kl = st->kl, kh = st->kh, sh = st->shift;
    if (threadIdx.x < 64) {
        const int64_t tot = wave_bucket_total(st->sub, nsub);
        if (threadIdx.x == 0) s_ncand = tot;
    }
    __syncthreads();
    const int64_t ncand = s_ncand;
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
    const float* x = sd.data;
    const int64_t bcap = sd.bucket_cap;
    uint32_t ka = 0, kb = 0;
    int path = MODE_WINDOW;
    int nst = 0;           /* staged keys (the buckets holding inside ranks) */
    int64_t before = 0;    /* inside keys in the buckets below the staged ones */
    bool full = ca == 0 || cb == 0 || st->overflow != 0;
    if (!full && (ca == 2 || cb == 2)) {
        if (threadIdx.x < 64) {
            if (ca == 2) wave_find_bucket(st->sub, nsub, ja, &sbin[0], &sbefore[0]);
            if (cb == 2) wave_find_bucket(st->sub, nsub, jb, &sbin[1], &sbefore[1]);
        }
        __syncthreads();
        const int blo = (ca == 2) ? sbin[0] : sbin[1];
        const int bhi = (cb == 2) ? sbin[1] : sbin[0];
        before = (ca == 2) ? sbefore[0] : sbefore[1];
        /* adjacent ranks: buckets strictly between blo and bhi are empty */
        const int64_t nlo = st->sub[blo], nhi = (bhi != blo) ? st->sub[bhi] : 0;
        if (nlo > bcap || nhi > bcap) {
            full = true;
        } else {
            const uint32_t* c = cand + sd.cand_off;
            for (int i = threadIdx.x; i < nlo; i += SEL_THREADS) stage[i] = c[(int64_t)blo * bcap + i];
            for (int i = threadIdx.x; i < nhi; i += SEL_THREADS) stage[nlo + i] = c[(int64_t)bhi * bcap + i];
            nst = (int)(nlo + nhi);
            __syncthreads();
            const uint64_t lo64 = (uint64_t)kl + 1 + ((uint64_t)blo << sh);
            const uint64_t hi64 = min((uint64_t)kh - 1, (uint64_t)kl + ((uint64_t)(bhi + 1) << sh));
            uint32_t xa = 0, xb = 0;
            select_in_range<SEL_THREADS>([&](int64_t i) { return stage[i]; }, [](uint32_t) { return true; },
                                         (int64_t)nst, (uint32_t)lo64, (uint32_t)hi64, ja - before, jb - before,
                                         ca == 2, cb == 2, &xa, &xb);
            ka = (ca == 2) ? xa : (ca == 1 ? kl : kh);
            kb = (cb == 2) ? xb : (cb == 1 ? kl : kh);
            path = MODE_CAND;
        }
    } else if (!full) {
        ka = (ca == 1) ? kl : kh;
        kb = (cb == 1) ? kl : kh;
    }
    if (full) {
        /* the window missed (or a block/bucket overflowed): exact radix select over the segment */
        select_in_range<SEL_THREADS>([&](int64_t i) { return abs_key(x[i]); }, [](uint32_t) { return true; }, sd.n, 0u,
                                     0xFFFFFFFFu, r0, r1, true, true, &ka, &kb);
        path = MODE_FULL;
    }
    __syncthreads();
    /* threshold: numpy/lib/function_base.py _lerp -- diff in float32, the blend in float64 */
    const uint32_t mk = st->maxkey;
    const float fa = __uint_as_float(ka), fb = __uint_as_float(kb);
    const float diff = fb - fa;
    const double g = sd.gamma;
    double thr = (g >= 0.5) ? (double)fb - (double)diff * (1.0 - g) : (double)fa + (double)diff * g;
    if (mk > 0x7F800000u) thr = __longlong_as_double(0x7FF8000000000000ll); /* NaN present */
    const float thr32 = (float)thr;
    /* level-0 segments: zeros of where(|x| < thr, 0, x) = #(|x| < thr) + [not (0 < thr)] * #(x == 0).
     * ka <= thr <= kb, so #(key < thr) = below + [thr > kl] eq_lo + before + #(staged < thr). */
    int64_t zc = 0;
    if (sd.flags & SEG_MASK) {
        if (thr32 > 0.0f) {
            const uint32_t tk = __float_as_uint(thr32);
            if (path == MODE_FULL)
                zc = block_count_below<SEL_THREADS>([&](int64_t i) { return abs_key(x[i]); }, sd.n, tk);
            else
                zc = below + (tk > kl ? eql : 0) + before +
                     block_count_below<SEL_THREADS>([&](int64_t i) { return stage[i]; }, nst, tk) +
                     (tk > kh ? eqh : 0);
        } else {
            zc = (int64_t)st->zeros;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        st->thr32 = thr32;
        thr_out[sd.res] = thr32; /* per tensor: read by k_mask and by the inverse transform */
        st->key_a = ka;
        st->key_b = kb;
        st->mode = path;
        /* leave the slot clean for the next call */
        st->overflow = 0;
        st->maxkey = 0;
        st->below = 0;
        st->eq_lo = 0;
        st->eq_hi = 0;
        st->zeros = 0;
        wtp_result& r = res[sd.res];
        r.numel = sd.numel;
        r.coeff_numel = sd.n;
        r.zero_count = zc; /* DWT segments: the inverse transform adds the zeros of its output */
        r.thr64 = thr;
        r.thr32_bits = __float_as_uint(thr32);
        r.max_abs_bits = mk;
        r.eff_level = sd.eff_level;
        r.path = path;
    }
    for (int i = threadIdx.x; i < nsub; i += SEL_THREADS) st->sub[i] = 0;
}

/* ----------------------------------------------------------------- k_mask --- */
/* out = where(|x| < thr, 0, x) for level-0 segments; the zero count came from k_select. */
__global__ __launch_bounds__(STREAM_THREADS) void k_mask(SegTable t, const float* __restrict__ thr_t) {
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    if (!(sd.flags & SEG_MASK)) return;
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int len = (int)min((int64_t)CHUNK, sd.n - base);
    const float* p = sd.data + base;
    float* q = sd.out + base;
    const bool vec = (sd.flags & SEG_ALIGNED) != 0;
    const int len4 = vec ? len >> 2 : 0;
    float4 v[16];
    if (vec) load_chunk_part(p, len4, v);
    const float thr = thr_t[sd.res];
    auto f = [&](float xv) { return (fabsf(xv) < thr) ? 0.0f : xv; };
    float4* q4 = reinterpret_cast<float4*>(q);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int j = it * STREAM_THREADS + threadIdx.x;
        if (j < len4) {
            float4 y;
            y.x = f(v[it].x); y.y = f(v[it].y); y.z = f(v[it].z); y.w = f(v[it].w);
            q4[j] = y;
        }
    }
    for (int i = len4 * 4 + threadIdx.x; i < len; i += STREAM_THREADS) q[i] = f(p[i]);
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

void launch_sample(const SegTable& t, SelState* sel, hipStream_t s) {
    hipLaunchKernelGGL(k_sample, dim3(t.nseg), dim3(SAMPLE_THREADS), 0, s, t, sel);
}
void launch_collect(const SegTable& t, SelState* sel, uint32_t* cand, hipStream_t s) {
    hipLaunchKernelGGL(k_collect, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, sel, cand);
}
void launch_select(const SegTable& t, SelState* sel, const uint32_t* cand, wtp_result* res, float* thr_out,
                   hipStream_t s) {
    hipLaunchKernelGGL(k_select, dim3(t.nseg), dim3(SEL_THREADS), 0, s, t, sel, cand, res, thr_out);
}
void launch_mask(const SegTable& t, const float* thr, hipStream_t s) {
    hipLaunchKernelGGL(k_mask, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, thr);
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
