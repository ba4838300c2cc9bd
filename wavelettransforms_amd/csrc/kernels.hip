/*
 * kernels.hip -- gfx950 kernels of the DWT -> percentile-threshold -> IDWT path.
 *
 * Selection (np.percentile(np.abs(coeff_arr), pct) + np.where(|c| < thr, 0, c),
 * ResNet/dwt_pruning.py:25-32) over grouped segments, one segment per tensor, on the float32
 * bit pattern of |x| (a key monotone in |x|; NaN sorts last as in np.partition):
 *   k_collect  every block first derives its segment's window [kl, kh] (bracketing the order
 *              statistics r0, r0+1) from the same deterministic sample of M_SAMPLE keys
 *              histogrammed into 1/128-octave bins; then it streams its chunk once: count
 *              keys < kl and == kl; scatter the keys inside (kl, kh] into key-range buckets
 *              (one run per bucket per block); max key
 *   k_mask_select  stream again: every block first resolves its segment's threshold (exact
 *              radix select of both ranks from the one or two buckets that hold them, or the
 *              whole segment if the window missed; NumPy 1.x _lerp in f64), then writes
 *              out = |x| < thr ? 0 : x (level-0 segments); the first
 *              block of a segment publishes the result and the exact zero count
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

/* Cross-lane primitives on DPP (GFX9 wave64: row_shr inside rows of 16 lanes, row_bcast:15/31
 * across rows): a few VALU cycles per step, where __shfl (ds_bpermute) pays an LDS round trip
 * per step.  Every lane of the wave must be active. */
template <int CTRL, int ROWM = 0xf, int BANKM = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWM, BANKM, false);
}

/* inclusive prefix sum across the 64 lanes */
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t v) {
    v += dpp_u32<0x111>(v); /* row_shr:1 */
    v += dpp_u32<0x112>(v); /* row_shr:2 */
    v += dpp_u32<0x114>(v); /* row_shr:4 */
    v += dpp_u32<0x118>(v); /* row_shr:8 */
    v += dpp_u32<0x142, 0xa>(v); /* row_bcast:15 into rows 1, 3 */
    v += dpp_u32<0x143, 0xc>(v); /* row_bcast:31 into rows 2, 3 */
    return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_u32(v), 63);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, dpp_u32<0x111>(v));
    v = max(v, dpp_u32<0x112>(v));
    v = max(v, dpp_u32<0x114>(v));
    v = max(v, dpp_u32<0x118>(v));
    v = max(v, dpp_u32<0x142, 0xa>(v));
    v = max(v, dpp_u32<0x143, 0xc>(v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

/* exact 64-bit sum (three 32-bit reductions of 16/16/32-bit fields) */
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    const uint32_t lo = wave_sum_u32((uint32_t)v & 0xFFFFu);
    const uint32_t mid = wave_sum_u32((uint32_t)(v >> 16) & 0xFFFFu);
    const uint32_t hi = wave_sum_u32((uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) + ((unsigned long long)mid << 16) + lo;
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

/* IT float4 per thread of one chunk (fully populated, 16-byte aligned) */
template <int IT, int CT = STREAM_THREADS>
__device__ __forceinline__ void load_chunk(const float* p, float4 (&v)[IT]) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int it = 0; it < IT; ++it) v[it] = p4[it * CT + threadIdx.x];
}

/* A ragged or unaligned chunk of len elements: element e of slot (it, c) is
 * 4 * (it * STREAM_THREADS + tid) + c, as in load_chunk.  Range-checked buffer loads: every
 * load is issued unconditionally (no per-load branch and wait) and reads 0 past len. */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ragged_rsrc(const float* p, int len) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* base = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, __builtin_amdgcn_readfirstlane(len * 4), 0x00020000);
}
template <int IT, int CT = STREAM_THREADS>
__device__ __forceinline__ void load_chunk_ragged(const float* p, int len, float4 (&v)[IT]) {
    const __amdgpu_buffer_rsrc_t r = ragged_rsrc(p, len);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = 4 * (it * CT + (int)threadIdx.x);
        v[it].x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * e, 0, 0));
        v[it].y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * e + 4, 0, 0));
        v[it].z = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * e + 8, 0, 0));
        v[it].w = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * e + 12, 0, 0));
    }
}
__device__ __forceinline__ float f4_get(const float4& v, int c) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); }

/* --------------------------------------------------------- radix select --- */
/* Find the digit (8 bits) holding rank r in a 256-bin LDS histogram; one wave. */
__device__ __forceinline__ void wave_pick_digit(const uint32_t* hb, int64_t r, int* digit, int64_t* below) {
    const int lane = threadIdx.x & 63;
    const uint32_t c0 = hb[4 * lane], c1 = hb[4 * lane + 1], c2 = hb[4 * lane + 2], c3 = hb[4 * lane + 3];
    const uint32_t s = c0 + c1 + c2 + c3; /* histograms count < 2^32 keys */
    const int64_t incl = wave_scan_u32(s);
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

/* timing probes for tools/mb/lab.hip (empty in the library) */
#ifndef WTP_PROBE
#define WTP_PROBE(i)
#endif
#ifndef WTP_CPROBE
#define WTP_CPROBE(i)
#endif

/* ------------------------------------------------------------ the window --- */
/* The selection window of a segment comes from a deterministic sample: MS keys in groups of
 * SAMPLE_GROUP contiguous floats spread evenly over the segment (the whole segment when
 * n <= MS).  Every block of the segment draws the same sample and so derives the same window,
 * which lets each k_collect block compute it for itself instead of waiting for a launch. */
template <int THREADS, int MS>
__device__ __forceinline__ void sample_keys(const SegDesc& sd, uint32_t (&k)[MS / THREADS]) {
    constexpr int PER = MS / THREADS;
    const int64_t n = sd.n;
    const bool exact = n <= MS;
    const double step = exact ? 0.0 : (double)(n - SAMPLE_GROUP) / (double)(MS / SAMPLE_GROUP - 1);
    /* all loads unconditional and issued before any use (indices clamped) */
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int i = j * THREADS + threadIdx.x;
        const int64_t pos = exact ? min((int64_t)i, n - 1)
                                  : (int64_t)((double)(i / SAMPLE_GROUP) * step) + (i % SAMPLE_GROUP);
        k[j] = abs_key(sd.data[pos]);
    }
}

/* LDS scratch of window_from_keys: the bin histogram plus a few words */
template <int THREADS>
struct WindowLds {
    static constexpr int FBP = (NB + THREADS - 1) / THREADS; /* bins per thread */
    uint32_t h[FBP * THREADS];
    uint32_t wtot[THREADS / 64];
    int found[2];
};

/* Histogram the sampled keys over the NB bins, locate the sample ranks bracketing r0 and r1
 * (6 sigma + 24 sample ranks of margin; exact ranks for a fully sampled segment) and return
 * the window: kl = low edge of the bin of the lower bracket (0: open), kh = high edge of the
 * bin of the upper bracket (0xFFFFFFFF: open), and the bucket shift for nsub buckets. */
template <int THREADS, int MS>
__device__ __forceinline__ void window_from_keys(const SegDesc& sd, const uint32_t (&k)[MS / THREADS],
                                                 WindowLds<THREADS>& L, uint32_t* kl_out, uint32_t* kh_out,
                                                 uint32_t* sh_out) {
    constexpr int PER = MS / THREADS, FBP = WindowLds<THREADS>::FBP;
    const int64_t n = sd.n;
    const bool exact = n <= MS;
    const int m = exact ? (int)n : MS;
    for (int i = threadIdx.x; i < FBP * THREADS; i += THREADS) L.h[i] = 0;
    if (threadIdx.x < 2) L.found[threadIdx.x] = -1;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j)
        if (j * THREADS + (int)threadIdx.x < m) atomicAdd(&L.h[key_bin(k[j])], 1u);
    __syncthreads();
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
    uint32_t local = 0;
#pragma unroll
    for (int j = 0; j < FBP; ++j) local += L.h[threadIdx.x * FBP + j];
    const uint32_t incl = wave_scan_u32(local);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) L.wtot[wv] = incl;
    __syncthreads();
    int64_t cum = (int64_t)incl - local;
    for (int i = 0; i < wv; ++i) cum += L.wtot[i];
#pragma unroll
    for (int j = 0; j < FBP; ++j) {
        const int b = threadIdx.x * FBP + j;
        const int64_t c = L.h[b];
        if (c) {
            if (sa >= cum && sa < cum + c) L.found[0] = b;
            if (sb >= cum && sb < cum + c) L.found[1] = b;
        }
        cum += c;
    }
    __syncthreads();
    const int f0 = L.found[0], f1 = L.found[1];
    const uint32_t kl = (sa < 0 || f0 < 0) ? 0u : bin_lo_key(f0);
    const uint32_t kh = (sb >= m || f1 < 0) ? 0xFFFFFFFFu : bin_hi_key(f1);
    uint32_t sh = 0;
    if (kh > kl + 1) {
        const uint32_t R = kh - kl - 1; /* inside keys kl < key <= kh: (key - kl - 1) in [0, R] */
        const int bits = 32 - __clz(R);
        sh = bits > sd.nsub_log2 ? bits - sd.nsub_log2 : 0;
    }
    *kl_out = kl;
    *kh_out = kh;
    *sh_out = sh;
}


/* -------------------------------------------------------------- k_collect --- */
/* LAB: 0 = the production kernel; 1 = stop after the counters; 2 = stop after the bucket
 * histogram (tools/mb/lab.hip ablations).  IT float4 per thread: a sub-chunk of IT * CT * 4
 * elements per block.  FULL: a whole 16-byte-aligned sub-chunk (unpredicated loads);
 * otherwise a ragged or unaligned one (range-checked buffer loads).
 *
 * One pass over the chunk: per key one unsigned compare each for "below" (k < kl), "equal to
 * kl" and "inside" (kl < k <= kh, as (k - kl - 1) < (kh - kl)), and the inside keys are staged
 * in the thread's own LDS column (stage[i * CT + tid], conflict-free, no scan).  A thread may
 * stage up to STG of its 4*IT keys; more sends the segment to the full-scan select. */
constexpr int STG = 24;
template <int CT, int IT, bool FULL, int LAB, bool WIN>
__device__ __forceinline__ void collect_body(const SegDesc& sd, SelState* __restrict__ st,
                                             uint32_t* __restrict__ cand, int64_t base, int len, bool first,
                                             uint32_t* lsub, uint32_t* lbase, uint32_t* stage,
                                             WindowLds<CT>* wl, uint32_t (*wred)[4], int* wtot) {
    const float* p = sd.data + base;
    WTP_CPROBE(0);
    uint32_t kl, kh, sh;
    float4 v[IT];
    if constexpr (WIN) {
        /* sample loads first, then the stream loads: the window is built while the chunk arrives */
        uint32_t ks[M_SAMPLE / CT];
        sample_keys<CT, M_SAMPLE>(sd, ks);
        if (FULL) load_chunk<IT, CT>(p, v);
        else load_chunk_ragged<IT, CT>(p, len, v);
        window_from_keys<CT, M_SAMPLE>(sd, ks, *wl, &kl, &kh, &sh);
        if (first && threadIdx.x == 0) { st->kl = kl; st->kh = kh; st->shift = sh; } /* for the select */
    } else {
        /* the window came from k_window; the stream loads go out first (the window words are
         * scalar loads, counted separately from the vector loads) */
        if (FULL) load_chunk<IT, CT>(p, v);
        else load_chunk_ragged<IT, CT>(p, len, v);
        kl = st->kl;
        kh = st->kh;
        sh = st->shift;
    }
    WTP_CPROBE(1);
    const int nsub = 1 << sd.nsub_log2;
    for (int i = threadIdx.x; i < nsub; i += CT) lsub[i] = 0;
    const uint32_t span = kh - kl; /* >= 1 */
    uint32_t below = 0, eql = 0, mx = 0, cnt = 0;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = 4 * (it * CT + (int)threadIdx.x);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t k = abs_key(f4_get(v[it], c));
            const bool valid = FULL || e + c < len;
            mx = max(mx, k); /* 0 past len: no effect */
            below += valid && k < kl;
            eql += valid && k == kl;
            if (valid && k - kl - 1u < span) {
                if (cnt < STG) stage[cnt * CT + threadIdx.x] = k;
                ++cnt;
            }
        }
    }
    /* one block reduction for the counters */
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    {
        const uint32_t r0 = wave_sum_u32(below), r1 = wave_sum_u32(eql), r2 = wave_max_u32(mx),
                       r3 = wave_max_u32(cnt);
        if (lane == 0) { wred[wv][0] = r0; wred[wv][1] = r1; wred[wv][2] = r2; wred[wv][3] = r3; }
    }
    const uint32_t tot_w = wave_sum_u32(cnt);
    if (lane == 0) wtot[wv] = (int)tot_w;
    __syncthreads();
    WTP_CPROBE(2);
    int total = 0;
    uint32_t cmax = 0;
    for (int w = 0; w < CT / 64; ++w) { total += wtot[w]; cmax = max(cmax, wred[w][3]); }
    const bool ovf = cmax > (uint32_t)STG;
    if (threadIdx.x == 0) {
        unsigned long long a0 = 0, a1 = 0;
        uint32_t m2 = 0;
        for (int w = 0; w < CT / 64; ++w) {
            a0 += wred[w][0];
            a1 += wred[w][1];
            m2 = max(m2, wred[w][2]);
        }
        const int sh8 = blockIdx.x & (NSHARD - 1);
        if (a0) atomicAdd(&st->below[sh8], a0);
        if (a1) atomicAdd(&st->eq_lo[sh8], a1);
        atomicMax(&st->maxkey[sh8], m2);
        if (ovf) atomicOr(&st->overflow, 1u);
    }
    /* uniform: nothing inside the window here, or a thread overflowed (full-scan select) */
    if (LAB == 1 || total == 0 || ovf) return;
    WTP_CPROBE(3);
    for (uint32_t i = 0; i < cnt; ++i) atomicAdd(&lsub[(stage[i * CT + threadIdx.x] - kl - 1) >> sh], 1u);
    __syncthreads();
    if (LAB == 2) return;
    /* reserve one contiguous run per non-empty bucket (one returning atomic per bucket) */
    for (int b = threadIdx.x; b < nsub; b += CT) {
        const uint32_t c = lsub[b];
        lbase[b] = c ? atomicAdd(&st->sub[b], c) : 0u;
        lsub[b] = 0;
    }
    __syncthreads();
    WTP_CPROBE(4);
    const int64_t bcap = sd.bucket_cap;
    uint32_t* out = cand + sd.cand_off;
    for (uint32_t i = 0; i < cnt; ++i) {
        const uint32_t k = stage[i * CT + threadIdx.x];
        const uint32_t b = (k - kl - 1) >> sh;
        const uint32_t at = lbase[b] + atomicAdd(&lsub[b], 1u);
        if (at < bcap) out[(int64_t)b * bcap + at] = k; /* counted beyond capacity: the select sees it */
    }
    WTP_CPROBE(5);
}

/* ------------------------------------------------------------- the select --- */
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
    uint32_t c = 0; /* per thread < 2^32 */
    for (int64_t i = threadIdx.x; i < m; i += THREADS) c += get(i) < tk;
    const unsigned long long w = wave_sum_u64(c);
    if ((threadIdx.x & 63) == 0 && w) atomicAdd(&acc, w);
    __syncthreads();
    const int64_t r = (int64_t)acc;
    __syncthreads();
    return r;
}

__device__ __forceinline__ void wave_find_bucket(const uint32_t* sub, int nsub, int64_t r, int* bucket,
                                                 int64_t* before) {
    const int lane = threadIdx.x & 63;
    const int per = nsub / 64; /* 1..16 consecutive buckets per lane */
    uint32_t s = 0; /* bucket counts of one segment: < 2^32 */
    for (int j = 0; j < per; ++j) s += sub[lane * per + j];
    const int64_t incl = wave_scan_u32(s);
    int64_t cum = incl - s;
    if (r >= cum && r < incl) {
        for (int j = 0; j < per; ++j) {
            const int64_t c = sub[lane * per + j];
            if (r < cum + c) { *bucket = lane * per + j; *before = cum; break; }
            cum += c;
        }
    }
}

/* Resolve the two order statistics of one segment from its counters and buckets, compute the
 * NumPy threshold and the level-0 zero count, publish the results, and leave the slot clean.
 * One block of THREADS threads; `stage` holds up to stage_cap keys in LDS. */
template <int THREADS>
__device__ float select_body(const SegDesc& sd, const SelState* __restrict__ st, const uint32_t* __restrict__ cand,
                             wtp_result* __restrict__ res, float* __restrict__ thr_out, uint32_t* stage,
                             int stage_cap, bool publish) {
    __shared__ int sbin[2];
    __shared__ int64_t sbefore[2];
    __shared__ uint32_t lsub[NSUB_MAX];
    __shared__ unsigned long long s_cnt[4]; /* below, eq_lo, eq_hi (unused: 0), inside */
    __shared__ uint32_t s_mk, s_ovf;
    const int nsub = 1 << sd.nsub_log2;
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    const uint32_t kl = st->kl, kh = st->kh, sh = st->shift;
    WTP_PROBE(0);
    /* one round trip: threads 0..4 gather the sharded counters, wave 1 the bucket counts (to LDS) */
    if (threadIdx.x < 64) {
        const int l = threadIdx.x;
        if (l < 3) {
            const unsigned long long* a = l == 0 ? st->below : (l == 1 ? st->eq_lo : st->eq_hi);
            unsigned long long v = 0;
#pragma unroll
            for (int i = 0; i < NSHARD; ++i) v += a[i];
            s_cnt[l] = v;
        } else if (l == 3) {
            uint32_t m = 0;
#pragma unroll
            for (int i = 0; i < NSHARD; ++i) m = max(m, st->maxkey[i]);
            s_mk = m;
        } else if (l == 4) {
            s_ovf = st->overflow;
        }
    } else if (threadIdx.x < 128) {
        const int l = threadIdx.x - 64;
        uint32_t sm = 0;
        for (int b = l; b < nsub; b += 64) { const uint32_t v = st->sub[b]; lsub[b] = v; sm += v; }
        sm = wave_sum_u32(sm);
        if (l == 0) s_cnt[3] = sm;
    }
    __syncthreads();
    WTP_PROBE(1);
    const int64_t below = (int64_t)s_cnt[0], eql = (int64_t)s_cnt[1], eqh = (int64_t)s_cnt[2];
    const int64_t ncand = (int64_t)s_cnt[3];
    uint32_t mk = s_mk;
    /* class of a rank: 0 miss, 1 == kl, 2 inside (kl, kh]  (eqh stays 0: keys == kh are inside) */
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
    const uint32_t* c = cand + sd.cand_off;
    uint32_t ka = 0, kb = 0;
    int path = MODE_WINDOW;
    int64_t nlo = 0, nhi = 0, before = 0;
    int blo = 0, bhi = 0;
    bool in_lds = false;
    bool full = ca == 0 || cb == 0 || s_ovf != 0;
    if (!full && (ca == 2 || cb == 2)) {
        if (threadIdx.x < 64 && ca == 2) wave_find_bucket(lsub, nsub, ja, &sbin[0], &sbefore[0]);
        if (threadIdx.x >= 64 && threadIdx.x < 128 && cb == 2) wave_find_bucket(lsub, nsub, jb, &sbin[1], &sbefore[1]);
        __syncthreads();
        WTP_PROBE(2);
        blo = (ca == 2) ? sbin[0] : sbin[1];
        bhi = (cb == 2) ? sbin[1] : sbin[0];
        before = (ca == 2) ? sbefore[0] : sbefore[1];
        /* adjacent ranks: buckets strictly between blo and bhi are empty */
        nlo = lsub[blo];
        nhi = (bhi != blo) ? lsub[bhi] : 0;
        if (nlo > bcap || nhi > bcap) {
            full = true;
        } else {
            in_lds = nlo + nhi <= stage_cap;
            if (in_lds) {
                for (int i = threadIdx.x; i < nlo; i += THREADS) stage[i] = c[(int64_t)blo * bcap + i];
                for (int i = threadIdx.x; i < nhi; i += THREADS) stage[nlo + i] = c[(int64_t)bhi * bcap + i];
                __syncthreads();
            }
            WTP_PROBE(3);
            const uint64_t lo64 = (uint64_t)kl + 1 + ((uint64_t)blo << sh);
            const uint64_t hi64 = min((uint64_t)kh, (uint64_t)kl + ((uint64_t)(bhi + 1) << sh));
            uint32_t xa = 0, xb = 0;
            auto getb = [&](int64_t i) {
                return in_lds ? stage[i] : (i < nlo ? c[(int64_t)blo * bcap + i] : c[(int64_t)bhi * bcap + i - nlo]);
            };
            select_in_range<THREADS>(getb, [](uint32_t) { return true; }, nlo + nhi, (uint32_t)lo64,
                                     (uint32_t)hi64, ja - before, jb - before, ca == 2, cb == 2, &xa, &xb);
            ka = (ca == 2) ? xa : (ca == 1 ? kl : kh);
            kb = (cb == 2) ? xb : (cb == 1 ? kl : kh);
            path = MODE_CAND;
            WTP_PROBE(4);
        }
    } else if (!full) {
        ka = (ca == 1) ? kl : kh;
        kb = (cb == 1) ? kl : kh;
    }
    if (full) {
        /* the window missed (or a block/bucket overflowed): exact radix select over the segment */
        select_in_range<THREADS>([&](int64_t i) { return abs_key(x[i]); }, [](uint32_t) { return true; }, sd.n, 0u,
                                 0xFFFFFFFFu, r0, r1, true, true, &ka, &kb);
        path = MODE_FULL;
    }
    __syncthreads();
    /* threshold: numpy/lib/function_base.py _lerp -- diff in float32, the blend in float64 */
    const float fa = __uint_as_float(ka), fb = __uint_as_float(kb);
    const float diff = fb - fa;
    const double g = sd.gamma;
    double thr = (g >= 0.5) ? (double)fb - (double)diff * (1.0 - g) : (double)fa + (double)diff * g;
    const bool minp = (sd.flags & SEG_MINPRUNE) != 0; /* rank select for min pruning: no NumPy NaN rule */
    if (mk > 0x7F800000u && !minp) thr = __longlong_as_double(0x7FF8000000000000ll); /* NaN present: np.percentile is NaN */
    const float thr32 = (float)thr;
    const bool nan = !minp && thr32 != thr32; /* also inf - inf inside the lerp */
    /* level-0 segments: zeros of where(|x| < thr, 0, x) = #(key < tk) with tk = bits(thr) when
     * thr > 0, else tk = 1 (only the zeros themselves).  ka <= thr <= kb and the two ranks are
     * adjacent, so #(key < tk) = below + [tk > kl] eq_lo + before + #(staged < tk).  A NaN
     * threshold prunes nothing: every k_mask_select block counts the zeros of its copy. */
    WTP_PROBE(5);
    if (!publish) return minp ? __uint_as_float(ka) : thr32; /* block-uniform */
    int64_t zc = 0;
    /* min pruning (k_minsel) wants #(key < t) for the exact key t = ka: none when t == 0 */
    if (((sd.flags & SEG_MASK) || (minp && ka > 0)) && !nan) {
        const uint32_t tk = minp ? ka : (thr32 > 0.0f ? __float_as_uint(thr32) : 1u);
        if (path == MODE_FULL)
            zc = block_count_below<THREADS>([&](int64_t i) { return abs_key(x[i]); }, sd.n, tk);
        else if (path == MODE_CAND)
            zc = below + (tk > kl ? eql : 0) + before +
                 block_count_below<THREADS>(
                     [&](int64_t i) {
                         return in_lds ? stage[i]
                                       : (i < nlo ? c[(int64_t)blo * bcap + i] : c[(int64_t)bhi * bcap + i - nlo]);
                     },
                     nlo + nhi, tk);
        else
            zc = below + (tk > kl ? eql : 0);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        thr_out[sd.res] = thr32; /* per tensor: read by the inverse transform */
        wtp_result& r = res[sd.res];
        r.numel = sd.numel;
        r.coeff_numel = sd.n;
        if (minp) r.zero_count = zc; /* k_minsel turns it into the tie budget; k_minmask counts */
        else if (zc) atomicAdd((unsigned long long*)&r.zero_count, (unsigned long long)zc); /* zeroed by k_collect */
        r.thr64 = thr;
        r.thr32_bits = __float_as_uint(thr32);
        r.max_abs_bits = mk;
        r.eff_level = sd.eff_level;
        r.path = path;
    }
    WTP_PROBE(6);
    return minp ? __uint_as_float(ka) : thr32;
}

/* k_window: one 1024-thread block per segment derives the window of the region k_collect is
 * about to fill (used when the window is not computed inline by every k_collect block) */
constexpr int WIN_THREADS = 1024;
__global__ __launch_bounds__(WIN_THREADS) void k_window(SegTable t, SelHeader* __restrict__ head) {
    __shared__ WindowLds<WIN_THREADS> wl;
    const SegDesc& sd = t.s[blockIdx.x];
    uint32_t ks[M_SAMPLE / WIN_THREADS];
    sample_keys<WIN_THREADS, M_SAMPLE>(sd, ks);
    uint32_t kl, kh, sh;
    window_from_keys<WIN_THREADS, M_SAMPLE>(sd, ks, wl, &kl, &kh, &sh);
    if (threadIdx.x == 0) {
        SelState* st = sel_region(head, head->parity) + sd.slot;
        st->kl = kl;
        st->kh = kh;
        st->shift = sh;
    }
}

/* one block per sub-chunk: block b takes sub-chunk (b % SPLIT) of table block (b / SPLIT).
 * The block also clears its share of the idle SelState region (the previous group's) and the
 * zero count of its segment's result; the last block to finish flips the region parity. */
template <int LAB, int CT, int IT, bool WIN>
__global__ __launch_bounds__(CT) void k_collect_t(SegTable t, SelHeader* __restrict__ head, uint32_t* __restrict__ cand,
                                                  wtp_result* __restrict__ res) {
    constexpr int SUB = IT * CT * 4, SPLIT = CHUNK / SUB;
    static_assert(CHUNK % SUB == 0, "sub-chunk size");
    __shared__ uint32_t lsub[NSUB_MAX];  /* this block's keys per bucket, then the running offset */
    __shared__ uint32_t lbase[NSUB_MAX]; /* reserved start of this block's run in each bucket     */
    __shared__ uint32_t stage[STG * CT];
    __shared__ WindowLds<WIN ? CT : 64> wl_; /* only the inline window uses it */
    WindowLds<CT>* wl = WIN ? reinterpret_cast<WindowLds<CT>*>(&wl_) : nullptr;
    __shared__ uint32_t wred[CT / 64][4];
    __shared__ int wtot[CT / 64];
    const uint32_t q = head->parity;
    {   /* clear this block's slice of the idle region */
        uint4* idle = reinterpret_cast<uint4*>(sel_region(head, q ^ 1u));
        constexpr int NV4 = (int)(SEL_REGION / 16);
        const int per = (NV4 + (int)gridDim.x - 1) / (int)gridDim.x;
        for (int i = threadIdx.x; i < per; i += CT) {
            const int j = (int)blockIdx.x * per + i;
            if (j < NV4) idle[j] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    const int tb = blockIdx.x / SPLIT;
    const int si = find_seg(t, tb);
    const SegDesc& sd = t.s[si];
    const int64_t base = (int64_t)(tb - sd.blk_begin) * CHUNK + (int64_t)(blockIdx.x % SPLIT) * SUB;
    const int len = (int)max((int64_t)0, min((int64_t)SUB, sd.n - base));
    SelState* st = sel_region(head, q) + sd.slot;
    const bool first = base == 0;
    if (first && threadIdx.x == 0) res[sd.res].zero_count = 0; /* k_mask_select and the inverse add */
    if (len > 0) {
        if ((sd.flags & SEG_ALIGNED) && len == SUB)
            collect_body<CT, IT, true, LAB, WIN>(sd, st, cand, base, len, first, lsub, lbase, stage, wl, wred, wtot);
        else
            collect_body<CT, IT, false, LAB, WIN>(sd, st, cand, base, len, first, lsub, lbase, stage, wl, wred, wtot);
    }
    __syncthreads(); /* every wave has read the parity */
    if (threadIdx.x == 0) {
        const uint32_t d = atomicAdd(&head->done, 1u);
        if (d == gridDim.x - 1) { /* last block: visible to the next kernel at the boundary */
            head->done = 0;
            head->parity = q ^ 1u;
        }
    }
}

/* ---------------------------------------------------------- k_mask_select --- */
/* out = where(|x| < thr, 0, x) over one chunk; returns the zeros written */
template <bool FULL>
__device__ __forceinline__ unsigned long long mask_body(const SegDesc& sd, int64_t base, int len, float thr) {
    const float* p = sd.data + base;
    float* q = sd.out + base;
    float4 v[16];
    if (FULL) load_chunk<16>(p, v);
    else load_chunk_ragged<16>(p, len, v);
    unsigned long long z = 0;
    auto f = [&](float xv) {
        const float y = (fabsf(xv) < thr) ? 0.0f : xv;
        z += y == 0.0f;
        return y;
    };
    if (FULL) {
        float4* q4 = reinterpret_cast<float4*>(q);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            float4 y;
            y.x = f(v[it].x); y.y = f(v[it].y); y.z = f(v[it].z); y.w = f(v[it].w);
            q4[it * STREAM_THREADS + threadIdx.x] = y;
        }
    } else {
        /* range-checked stores: writes past len are dropped, no per-store branch */
        const __amdgpu_buffer_rsrc_t r = ragged_rsrc(q, len);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int e = 4 * (it * STREAM_THREADS + (int)threadIdx.x);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float y = f(f4_get(v[it], c));
                if (e + c >= len) z -= y == 0.0f; /* the zeros read past the end */
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), r, 4 * (e + c), 0, 0);
            }
        }
    }
    return z;
}

/* The select and the level-0 mask in one launch.  Every block resolves its segment's
 * threshold itself from k_collect's counters and the one or two buckets holding the ranks
 * (a few thousand keys, read from L2), then streams its chunk: where(|x| < thr, 0, x).  The segment's first block also computes the exact zero count and
 * publishes the result record and the per-tensor threshold (read by the inverse transform).
 * A DWT segment needs one select (its first block), not one per chunk. */
constexpr int MS_STAGE = 4096;
__global__ __launch_bounds__(STREAM_THREADS) void k_mask_select(SegTable t, const SelHeader* __restrict__ head,
                                                                const uint32_t* __restrict__ cand,
                                                                wtp_result* __restrict__ res,
                                                                float* __restrict__ thr_out) {
    __shared__ uint32_t stage[MS_STAGE];
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const bool masked = (sd.flags & SEG_MASK) != 0;
    if (!masked && base != 0) return; /* block-uniform */
    const int len = (int)min((int64_t)CHUNK, sd.n - base);
    const bool full = (sd.flags & SEG_ALIGNED) && len == CHUNK;
    /* the select first: loads return in issue order (vmcnt), so chunk loads issued ahead of
     * the select's would only delay its round trips -- and the chunk's 64 registers would sit
     * live through it */
    const SelState* st = sel_region(const_cast<SelHeader*>(head), head->parity ^ 1u) + sd.slot;
    const float thr = select_body<STREAM_THREADS>(sd, st, cand, res, thr_out, stage, MS_STAGE, base == 0);
    if (!masked) return;
    float4 v[16];
    {
        const float* p = sd.data + base;
        if (full) load_chunk<16>(p, v);
        else load_chunk_ragged<16>(p, len, v);
    }
    float* q = sd.out + base;
    unsigned long long z = 0;
    auto f = [&](float xv) {
        const float y = (fabsf(xv) < thr) ? 0.0f : xv;
        z += y == 0.0f;
        return y;
    };
    if (full) {
        float4* q4 = reinterpret_cast<float4*>(q);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            float4 y;
            y.x = f(v[it].x); y.y = f(v[it].y); y.z = f(v[it].z); y.w = f(v[it].w);
            q4[it * STREAM_THREADS + threadIdx.x] = y;
        }
    } else {
        const __amdgpu_buffer_rsrc_t r = ragged_rsrc(q, len);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int e = 4 * (it * STREAM_THREADS + (int)threadIdx.x);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float y = f(f4_get(v[it], c));
                if (e + c >= len) z -= y == 0.0f; /* the zeros read past the end */
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), r, 4 * (e + c), 0, 0);
            }
        }
    }
    if (thr != thr) { /* uniform: a NaN threshold prunes nothing, the copy's zeros are counted */
        const unsigned long long tot = block_sum_u64<STREAM_THREADS>(z);
        if (threadIdx.x == 0 && tot) atomicAdd((unsigned long long*)&res[sd.res].zero_count, tot);
    }
}

/* -------------------------------------------------------- min-weight pruning --- */
/* percentage_min_pruning (ResNet/min_weight_pruning.py:66-74): zero the k smallest |w| of each
 * tensor.  The rank-(k-1) key t comes from the same window / collect / select machinery
 * (r0 = k-1, gamma 0).  Every |w| < t is pruned; of the |w| == t the lowest flat indices go
 * first until k are pruned (torch.topk's order among ties is unspecified).
 *   k_minsel   one block per segment: the exact t, and need = k - #(|w| < t)
 *   k_tiecount one block per chunk: #(|w| == t) in the chunk
 *   k_minmask  one block per chunk: its ties' global order = the counts of the segment's
 *              earlier chunks + an in-block scan in flat-index order; writes out, counts zeros */
struct MinPrune {
    uint32_t tkey;   /* |w| bit pattern of t (k = 0: 0, with need 0 nothing is pruned) */
    uint32_t pad;
    int64_t need;    /* ties to prune (lowest indices first) */
};

__global__ __launch_bounds__(STREAM_THREADS) void k_minsel(SegTable t, const SelHeader* __restrict__ head,
                                                           const uint32_t* __restrict__ cand,
                                                           wtp_result* __restrict__ res, float* __restrict__ thr_out,
                                                           MinPrune* __restrict__ mp) {
    __shared__ uint32_t stage[4096];
    const SegDesc& sd = t.s[blockIdx.x];
    const SelState* st = sel_region(const_cast<SelHeader*>(head), head->parity ^ 1u) + sd.slot;
    const int64_t k = (sd.flags & SEG_KZERO) ? 0 : sd.r0 + 1;
    float thr = 0.0f;
    if (k > 0) thr = select_body<STREAM_THREADS>(sd, st, cand, res, thr_out, stage, 4096, true);
    __syncthreads();
    if (threadIdx.x == 0) {
        wtp_result& r = res[sd.res];
        MinPrune m;
        m.pad = 0;
        if (k > 0) {
            m.tkey = __float_as_uint(thr) & 0x7FFFFFFFu;
            m.need = k - r.zero_count; /* select_body left #(|w| < t) there */
        } else { /* nothing to prune */
            r.numel = sd.numel;
            r.coeff_numel = sd.n;
            r.thr64 = 0.0;
            r.thr32_bits = 0;
            r.max_abs_bits = 0;
            r.eff_level = 0;
            r.path = MODE_WINDOW;
            m.tkey = 0; /* no key is below 0, and no tie is pruned */
            m.need = 0;
        }
        r.zero_count = 0; /* k_minmask adds the zeros it writes */
        mp[sd.res] = m;
    }
}

__global__ __launch_bounds__(STREAM_THREADS) void k_tiecount(SegTable t, const MinPrune* __restrict__ mp,
                                                             uint32_t* __restrict__ tiecnt) {
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    const MinPrune m = mp[sd.res];
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int len = (int)min((int64_t)CHUNK, sd.n - base);
    uint32_t c = 0;
    if (m.need > 0) { /* block-uniform */
        float4 v[16];
        if ((sd.flags & SEG_ALIGNED) && len == CHUNK) load_chunk<16>(sd.data + base, v);
        else load_chunk_ragged<16>(sd.data + base, len, v);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int e = 4 * (it * STREAM_THREADS + (int)threadIdx.x);
#pragma unroll
            for (int q = 0; q < 4; ++q) c += (e + q < len) && abs_key(f4_get(v[it], q)) == m.tkey;
        }
    }
    const unsigned long long tot = block_sum_u64<STREAM_THREADS>(c);
    if (threadIdx.x == 0) tiecnt[blockIdx.x] = (uint32_t)tot;
}

__global__ __launch_bounds__(STREAM_THREADS) void k_minmask(SegTable t, const MinPrune* __restrict__ mp,
                                                            const uint32_t* __restrict__ tiecnt,
                                                            wtp_result* __restrict__ res) {
    __shared__ uint32_t wsum[STREAM_THREADS / 64];
    __shared__ int64_t s_off;
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    const MinPrune m = mp[sd.res];
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int len = (int)min((int64_t)CHUNK, sd.n - base);
    const bool full = (sd.flags & SEG_ALIGNED) && len == CHUNK;
    float4 v[16];
    if (full) load_chunk<16>(sd.data + base, v);
    else load_chunk_ragged<16>(sd.data + base, len, v);
    /* ties of the segment's earlier chunks */
    const bool ties = m.need > 0 && tiecnt[blockIdx.x] > 0; /* block-uniform */
    if (ties && threadIdx.x < 64) {
        unsigned long long a = 0;
        for (int b = sd.blk_begin + (int)threadIdx.x; b < (int)blockIdx.x; b += 64) a += tiecnt[b];
        a = wave_sum_u64(a);
        if (threadIdx.x == 0) s_off = (int64_t)a;
    }
    __syncthreads();
    int64_t run = ties ? s_off : 0; /* ties before the current it-row */
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long z = 0;
    auto prune = [&](uint32_t k, int64_t rank) { return k < m.tkey || (k == m.tkey && rank < m.need); };
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = 4 * (it * STREAM_THREADS + (int)threadIdx.x);
        float4 y = v[it];
        if (ties) { /* flat-index order inside the block: it-row, then thread, then component */
            uint32_t c = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) c += (e + q < len) && abs_key(f4_get(v[it], q)) == m.tkey;
            const uint32_t incl = wave_scan_u32(c);
            if (lane == 63) wsum[wv] = incl;
            __syncthreads();
            int64_t before = run + (incl - c);
            uint32_t rowtot = 0;
            for (int w = 0; w < STREAM_THREADS / 64; ++w) {
                if (w < wv) before += wsum[w];
                rowtot += wsum[w];
            }
            __syncthreads();
            run += rowtot;
            float* yy = reinterpret_cast<float*>(&y);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t k = abs_key(yy[q]);
                if (prune(k, before)) yy[q] = 0.0f;
                before += (e + q < len) && k == m.tkey;
            }
        } else {
            float* yy = reinterpret_cast<float*>(&y);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (abs_key(yy[q]) < m.tkey) yy[q] = 0.0f;
        }
        v[it] = y;
#pragma unroll
        for (int q = 0; q < 4; ++q) z += (e + q < len) && f4_get(y, q) == 0.0f;
    }
    float* q = sd.out + base;
    if (full) {
        float4* q4 = reinterpret_cast<float4*>(q);
#pragma unroll
        for (int it = 0; it < 16; ++it) q4[it * STREAM_THREADS + threadIdx.x] = v[it];
    } else {
        const __amdgpu_buffer_rsrc_t r = ragged_rsrc(q, len);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int e = 4 * (it * STREAM_THREADS + (int)threadIdx.x);
#pragma unroll
            for (int c = 0; c < 4; ++c) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(f4_get(v[it], c)), r, 4 * (e + c), 0, 0);
        }
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

void launch_window(const SegTable& t, SelHeader* head, hipStream_t s) {
    if (!COLLECT_WINDOW_INLINE) hipLaunchKernelGGL(k_window, dim3(t.nseg), dim3(WIN_THREADS), 0, s, t, head);
}
void launch_collect(const SegTable& t, SelHeader* head, uint32_t* cand, wtp_result* res, hipStream_t s) {
    hipLaunchKernelGGL((k_collect_t<0, COLLECT_THREADS, COLLECT_IT, COLLECT_WINDOW_INLINE>),
                       dim3(t.nblk * (CHUNK / (COLLECT_IT * COLLECT_THREADS * 4))), dim3(COLLECT_THREADS), 0, s, t,
                       head, cand, res);
}
void launch_minprune(const SegTable& t, SelHeader* head, const uint32_t* cand, wtp_result* res, float* thr_out,
                     void* mp, uint32_t* tiecnt, hipStream_t s) {
    hipLaunchKernelGGL(k_minsel, dim3(t.nseg), dim3(STREAM_THREADS), 0, s, t, head, cand, res, thr_out,
                       reinterpret_cast<MinPrune*>(mp));
    hipLaunchKernelGGL(k_tiecount, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, reinterpret_cast<const MinPrune*>(mp),
                       tiecnt);
    hipLaunchKernelGGL(k_minmask, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, reinterpret_cast<const MinPrune*>(mp),
                       tiecnt, res);
}
void launch_mask_select(const SegTable& t, SelHeader* head, const uint32_t* cand, wtp_result* res, float* thr_out,
                        hipStream_t s) {
    hipLaunchKernelGGL(k_mask_select, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, head, cand, res, thr_out);
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
