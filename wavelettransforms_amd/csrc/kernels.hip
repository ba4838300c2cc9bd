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
#include "wt_perm.h"

#include <atomic>
#include <cstdlib>

#pragma clang fp contract(off)

namespace wtp {

/* ---------------------------------------------------------------- helpers --- */
__device__ __forceinline__ uint32_t abs_key(float x) { return __float_as_uint(x) & 0x7FFFFFFFu; }

/* Loads and stores of bytes handed between workgroups of ONE launch (k_resident): agent-scope
 * relaxed atomics lower to global_load/store ... sc1, which bypass the CU's L1 and write
 * through the XCD's L2 (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores + sc1 loads
 * + an agent-scope arrival counter, one workgroup per CU).  COH = false: plain accesses (the
 * data was produced by an earlier launch). */
template <bool COH, class T>
__device__ __forceinline__ T ldc(const T* p) {
    if constexpr (COH) return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <class T>
__device__ __forceinline__ void stc(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
/* a 16-byte write-through (sc1) vector store: MI355X_MICROARCH.md's hand-off form for tens of KB
 * per workgroup (drained by the storer's vmcnt(0) before its arrival, read with sc1 loads).  A
 * buffer store through the builtin (cache policy 16 = sc1), not inline asm: the compiler then
 * knows the store reads its data VGPRs late and keeps the wait state before they are rewritten
 * (an inline-asm dwordx4 store had its data registers overwritten by the next VALU op). */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t region_rsrc(const uint32_t* p, int words) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, words * 4, 0x00020000);
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, int word, uint4 v) {
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    const u4v x = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, 4 * word, 0, 16);
}

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

/* IT float4 per thread of one chunk (fully populated, 16-byte aligned).  NT: nontemporal loads
 * (the `nt` policy bit) -- k_resident's once-read chunk: measured neutral with warm caches and 7 us
 * shorter behind a 512 MiB write to another buffer (its reads then no longer evict that buffer's
 * dirty Infinity-Cache lines) */
template <int IT, int CT = STREAM_THREADS, bool NT = false>
__device__ __forceinline__ void load_chunk(const float* p, float4 (&v)[IT]) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
    typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        if (NT) {
            const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p4 + it * CT + threadIdx.x));
            v[it] = make_float4(t.x, t.y, t.z, t.w);
        } else {
            v[it] = p4[it * CT + threadIdx.x];
        }
    }
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
template <int IT, int CT = STREAM_THREADS, bool NT = false>
__device__ __forceinline__ void load_chunk_ragged(const float* p, int len, float4 (&v)[IT]) {
    const __amdgpu_buffer_rsrc_t r = ragged_rsrc(p, len);
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0 && (len & 3) == 0) { /* uniform */
        /* every float4 lies wholly inside or wholly past len: one 16-byte range-checked load
         * each (past len it reads as zeros) instead of four dword loads */
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const u4 q = __builtin_amdgcn_raw_buffer_load_b128(r, 16 * (it * CT + (int)threadIdx.x), 0, NT ? 2 : 0);
            v[it] = make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), __uint_as_float(q.w));
        }
        return;
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = 4 * (it * CT + (int)threadIdx.x);
        v[it].x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * e, 0, NT ? 2 : 0));
        v[it].y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * e + 4, 0, NT ? 2 : 0));
        v[it].z = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * e + 8, 0, NT ? 2 : 0));
        v[it].w = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * e + 12, 0, NT ? 2 : 0));
    }
}
/* range-checked float4 store: the dwords past the buffer's length are dropped */
__device__ __forceinline__ void store4_ragged(const float4& y, __amdgpu_buffer_rsrc_t r, int off) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y.x), r, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y.y), r, off + 4, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y.z), r, off + 8, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y.w), r, off + 12, 0, 0);
}
/* a copy the compiler cannot see through: keys derived from it are recomputed where needed
 * instead of being kept live beside the data (k_resident holds 96 floats per thread) */
__device__ __forceinline__ float opaque(float x) {
    asm volatile("" : "+v"(x));
    return x;
}
/* float4 slot j of a partial chunk of len elements: whole float4 stores where the slot is
 * complete and the buffer 16-byte aligned, range-checked dword stores otherwise */
__device__ __forceinline__ void store4_tail(const float4& y, float* q, __amdgpu_buffer_rsrc_t r, int j, int len,
                                            bool aligned) {
    if (aligned && 4 * j + 3 < len) reinterpret_cast<float4*>(q)[j] = y;
    else if (4 * j < len) store4_ragged(y, r, 16 * j);
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
#ifndef WTP_PROBE_T /* a probe taken by thread t */
#define WTP_PROBE_T(i, t)
#endif
#ifndef WTP_CPROBE
#define WTP_CPROBE(i)
#endif
#ifndef WTP_RPROBE
#define WTP_RPROBE(i)
#endif
#ifndef WTP_WPROBE
#define WTP_WPROBE(i)
#endif
#ifndef WTP_RTAG /* k_resident: the workgroup's segment flags, for the phase lab */
#define WTP_RTAG(tagv)
#endif
#ifndef WTP_GPROBE /* a probe taken by lane 0 of the executing wave */
#define WTP_GPROBE(i)
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
__device__ __forceinline__ void window_search(const SegDesc& sd, WindowLds<THREADS>& L, uint32_t* kl_out,
                                              uint32_t* kh_out, uint32_t* sh_out);
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
    WTP_WPROBE(0);
#pragma unroll
    for (int j = 0; j < PER; ++j)
        if (j * THREADS + (int)threadIdx.x < m) atomicAdd(&L.h[key_bin(k[j])], 1u);
    __syncthreads();
    WTP_WPROBE(1);
    window_search<THREADS, MS>(sd, L, kl_out, kh_out, sh_out);
}

/* the search half: L.h holds the histogram of the MS sampled keys (all n when n <= MS) */
template <int THREADS, int MS>
__device__ __forceinline__ void window_search(const SegDesc& sd, WindowLds<THREADS>& L, uint32_t* kl_out,
                                              uint32_t* kh_out, uint32_t* sh_out) {
    constexpr int FBP = WindowLds<THREADS>::FBP;
    const int64_t n = sd.n;
    const bool exact = n <= MS;
    const int m = exact ? (int)n : MS;
    /* sample ranks fit 32 bits; the bin counts stay in registers from the scan to the search */
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    int sa, sb;
    if (exact) {
        sa = (int)r0;
        sb = (int)r1;
    } else {
        const double p = (double)r0 / (double)(n - 1);
        const double s0 = p * (double)(m - 1), s1 = (double)r1 / (double)(n - 1) * (double)(m - 1);
        const double d = 6.0 * sqrt((double)m * p * (1.0 - p)) + 24.0;
        sa = (int)floor(s0 - d);
        sb = (int)ceil(s1 + d);
    }
    uint32_t c[FBP];
#pragma unroll
    for (int j = 0; j < FBP; ++j) c[j] = L.h[threadIdx.x * FBP + j];
    uint32_t local = 0;
#pragma unroll
    for (int j = 0; j < FBP; ++j) local += c[j];
    const uint32_t incl = wave_scan_u32(local);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) L.wtot[wv] = incl;
    __syncthreads();
    WTP_WPROBE(2);
    int cum = (int)(incl - local);
#pragma unroll
    for (int i = 0; i < THREADS / 64; ++i) cum += i < wv ? (int)L.wtot[i] : 0;
    if (sa >= cum || sb >= cum) { /* only threads at or below the ranks search their bins */
#pragma unroll
        for (int j = 0; j < FBP; ++j) {
            const int nx = cum + (int)c[j];
            if (sa >= cum && sa < nx) L.found[0] = threadIdx.x * FBP + j;
            if (sb >= cum && sb < nx) L.found[1] = threadIdx.x * FBP + j;
            cum = nx;
        }
    }
    __syncthreads();
    WTP_WPROBE(3);
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


/* window_from_keys for ONE wave (64 threads, no block barrier: the other waves of the block
 * are elsewhere).  Lane l owns the FBP consecutive bins from l * FBP (stride FBP odd: no bank
 * conflicts); the lane whose run holds a sample rank walks it. */
/* The search half of window_from_keys for ONE wave (no block barrier: the other waves are
 * issuing their loads meanwhile), over the block's histogram h of the MS sampled keys (NB bins)
 * and its coarse companion hc (bins of 128: WCB of them): one scan over the coarse bins finds
 * the 128 fine bins holding a sample rank, one more scan over those finds the bin. */
constexpr int WCB = (NB + 127) / 128; /* 33 <= 64 */
__device__ __forceinline__ int wave_find_bin(const uint32_t* h, const uint32_t* hc, int r) {
    const int lane = threadIdx.x & 63;
    if (r < 0) return -1;
    const uint32_t c = lane < WCB ? hc[lane] : 0u;
    const uint32_t incl = wave_scan_u32(c);
    const uint64_t m = __ballot((int)(incl - c) <= r && r < (int)incl);
    if (!m) return -1;
    const int cb = __ffsll((unsigned long long)m) - 1;
    const int before = __builtin_amdgcn_readlane((int)(incl - c), cb);
    const int b0 = cb * 128 + 2 * lane;
    const uint32_t f0 = b0 < NB ? h[b0] : 0u, f1 = b0 + 1 < NB ? h[b0 + 1] : 0u;
    const uint32_t s2 = f0 + f1;
    const int i2 = before + (int)wave_scan_u32(s2);
    const int e2 = i2 - (int)s2;
    const uint64_t m2 = __ballot(e2 <= r && r < i2);
    const int L = __ffsll((unsigned long long)m2) - 1;
    const int pick = (r < e2 + (int)f0) ? b0 : b0 + 1;
    return __builtin_amdgcn_readlane(pick, L);
}

template <int MS>
__device__ __forceinline__ void window_search_wave(const SegDesc& sd, const uint32_t* h, const uint32_t* hc,
                                                   uint32_t* kl_out, uint32_t* kh_out, uint32_t* sh_out,
                                                   double sig = 6.0, double add = 24.0) {
    const int64_t n = sd.n;
    const bool exact = n <= MS;
    const int m = exact ? (int)n : MS;
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    int sa, sb;
    if (exact) {
        sa = (int)r0;
        sb = (int)r1;
    } else {
        const double p = (double)r0 / (double)(n - 1);
        const double s0 = p * (double)(m - 1), s1 = (double)r1 / (double)(n - 1) * (double)(m - 1);
        const double d = sig * sqrt((double)m * p * (1.0 - p)) + add;
        sa = (int)floor(s0 - d);
        sb = (int)ceil(s1 + d);
    }
    const int f0 = wave_find_bin(h, hc, sa);
    const int f1 = sb < m ? wave_find_bin(h, hc, sb) : -1;
    const uint32_t kl = (sa < 0 || f0 < 0) ? 0u : bin_lo_key(f0);
    const uint32_t kh = (sb >= m || f1 < 0) ? 0xFFFFFFFFu : bin_hi_key(f1);
    uint32_t sh = 0;
    if (kh > kl + 1) {
        const uint32_t R = kh - kl - 1;
        const int bits = 32 - __clz(R);
        sh = bits > sd.nsub_log2 ? bits - sd.nsub_log2 : 0;
    }
    *kl_out = kl;
    *kh_out = kh;
    *sh_out = sh;
}

/* -------------------------------------------------------------- k_collect --- */
/* IT float4 per thread: a sub-chunk of IT * CT * 4
 * elements per block.  FULL: a whole 16-byte-aligned sub-chunk (unpredicated loads);
 * otherwise a ragged or unaligned one (range-checked buffer loads).
 *
 * One pass over the chunk: per key one unsigned compare each for "below" (k < kl), "equal to
 * kl" and "inside" (kl < k <= kh, as (k - kl - 1) < (kh - kl)), and the inside keys are staged
 * in the thread's own LDS column (stage[i * CT + tid], conflict-free, no scan).  A thread may
 * stage up to STG of its 4*IT keys; more sends the segment to the full-scan select. */
constexpr int STG = 24;

/* the counting pass over a thread's IT float4 (element e of slot (it, c) is 4 (it CT + tid) + c;
 * past len -- a ragged chunk -- nothing counts): below / equal-to-kl counts, the max key, and the
 * inside keys staged in the thread's LDS column; clears the block's bucket histogram */
template <int CT, int IT>
__device__ __forceinline__ void collect_count(const float4 (&v)[IT], bool full, int len, int nsub, uint32_t kl,
                                              uint32_t kh, uint32_t* lsub, uint32_t* stage, uint32_t& below,
                                              uint32_t& eql, uint32_t& mx, uint32_t& cnt) {
    for (int i = threadIdx.x; i < nsub; i += CT) lsub[i] = 0;
    const uint32_t span = kh - kl; /* >= 1 */
    below = 0; eql = 0; mx = 0; cnt = 0;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = 4 * (it * CT + (int)threadIdx.x);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t k = abs_key(f4_get(v[it], c));
            const bool valid = full || e + c < len;
            mx = max(mx, k); /* 0 past len: no effect */
            below += valid && k < kl;
            eql += valid && k == kl;
            if (valid && k - kl - 1u < span) {
                if (cnt < STG) stage[cnt * CT + threadIdx.x] = k;
                ++cnt;
            }
        }
    }
}

/* the rest of a chunk: the block's counters into the segment's (8-way sharded agent atomics), the
 * inside keys bucketed by key range (LDS histogram, the block's returning reservation atomics all
 * in flight at once) and scattered into the candidate buckets */
template <int CT, int STGN = STG>
__device__ __forceinline__ void collect_finish(const SegDesc& sd, SelState* __restrict__ st, uint32_t* __restrict__ cand,
                                               uint32_t kl, uint32_t sh, uint32_t below, uint32_t eql, uint32_t mx,
                                               uint32_t cnt, uint32_t* lsub, uint32_t* lbase, uint32_t* stage,
                                               uint32_t (*wred)[4], int* wtot) {
    const int nsub = 1 << sd.nsub_log2;
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
    const bool ovf = cmax > (uint32_t)STGN;
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
    if (total == 0 || ovf) return;
    WTP_CPROBE(3);
    for (uint32_t i = 0; i < cnt; ++i) atomicAdd(&lsub[(stage[i * CT + threadIdx.x] - kl - 1) >> sh], 1u);
    __syncthreads();
    /* reserve one contiguous run per non-empty bucket (one returning atomic per bucket, all of a
     * thread's in flight at once) */
    {
        constexpr int PER = NSUB_MAX / CT;
        uint32_t cj[PER], rj[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) cj[j] = (j * CT + (int)threadIdx.x < nsub) ? lsub[j * CT + threadIdx.x] : 0u;
#pragma unroll
        for (int j = 0; j < PER; ++j) rj[j] = cj[j] ? atomicAdd(&st->sub[j * CT + threadIdx.x], cj[j]) : 0u;
#pragma unroll
        for (int j = 0; j < PER; ++j)
            if (j * CT + (int)threadIdx.x < nsub) { lbase[j * CT + threadIdx.x] = rj[j]; lsub[j * CT + threadIdx.x] = 0; }
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

/* One chunk of a k_collect_t block: its loads (and with WIN the window from the block's own
 * sample), the counting pass, the rest.  FULL: a whole 16-byte-aligned chunk (unpredicated
 * loads); otherwise a ragged or unaligned one (range-checked buffer loads). */
template <int CT, int IT, bool FULL, bool WIN>
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
    uint32_t below, eql, mx, cnt;
    collect_count<CT, IT>(v, FULL, len, 1 << sd.nsub_log2, kl, kh, lsub, stage, below, eql, mx, cnt);
    collect_finish<CT>(sd, st, cand, kl, sh, below, eql, mx, cnt, lsub, lbase, stage, wred, wtot);
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

/* Rank r (0-based, ascending) among the m <= 64*KPL keys stage[0..m), all in [lo, hi]; one
 * wave, keys in registers.  Bit by bit below the common prefix of lo and hi, the result takes a
 * bit when at most r keys lie below it: it ends at the largest t with #(key < t) <= r, which is
 * the r-th key itself.  Every lane of the wave must be active. */
constexpr int WSEL_KPL = 16;
constexpr int STAGE_BATCH = 4;
template <int KPL>
__device__ __forceinline__ uint32_t wave_select_rank(const uint32_t* stage, int m, int64_t r, uint32_t lo, uint32_t hi) {
    const int lane = threadIdx.x & 63;
    uint32_t k[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int i = j * 64 + lane;
        k[j] = i < m ? stage[i] : 0xFFFFFFFFu; /* above every |x| key */
    }
    const uint32_t diff = lo ^ hi;
    const int top = diff ? 31 - __clz(diff) : -1;
    uint32_t res = top >= 31 ? 0u : (lo & ~((2u << top) - 1u));
    const uint32_t rr = (uint32_t)r; /* r < m */
    for (int b = top; b >= 0; --b) {
        const uint32_t cand = res | (1u << b);
        uint32_t c = 0; /* counted on the scalar unit: compare masks and popcounts, no DPP chain */
#pragma unroll
        for (int j = 0; j < KPL; ++j) c += (uint32_t)__popcll(__ballot(k[j] < cand));
        if (c <= rr) res = cand;
    }
    return res;
}

/* Ranks ra / rb among the m keys stage[0..m), all in [lo, lo + W), W <= HS_PER * THREADS:
 * one LDS histogram over the W key values, a block scan of per-thread runs of HS_PER bins kept
 * in registers, and the thread whose run holds a rank names its key.  out[] and wt[] are LDS. */
constexpr int HS_PER = 16;
template <int THREADS>
__device__ __forceinline__ void block_hist_select(const uint32_t* stage, int m, uint32_t lo, int W, int ra, int rb,
                                                  uint32_t* hist, uint32_t* out, uint32_t* wt) {
    const int per = (W + THREADS - 1) / THREADS;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    for (int i = tid; i < per * THREADS; i += THREADS) hist[i] = 0;
    __syncthreads();
    WTP_PROBE_T(12, 0);
    for (int i = tid; i < m; i += THREADS) atomicAdd(&hist[stage[i] - lo], 1u);
    __syncthreads();
    WTP_PROBE_T(13, 0);
    uint32_t c[HS_PER];
    uint32_t local = 0;
#pragma unroll
    for (int j = 0; j < HS_PER; ++j) {
        c[j] = j < per ? hist[tid * per + j] : 0u;
        local += c[j];
    }
    const uint32_t incl = wave_scan_u32(local);
    if (lane == 63) wt[wv] = incl;
    __syncthreads();
    WTP_PROBE_T(14, 0);
    int cum = (int)(incl - local);
#pragma unroll
    for (int i = 0; i < THREADS / 64; ++i) cum += i < wv ? (int)wt[i] : 0;
    if (local && ((ra >= cum && ra < cum + (int)local) || (rb >= cum && rb < cum + (int)local))) {
#pragma unroll
        for (int j = 0; j < HS_PER; ++j) {
            const int nx = cum + (int)c[j];
            if (ra >= cum && ra < nx) out[0] = lo + (uint32_t)(tid * per + j);
            if (rb >= cum && rb < nx) out[1] = lo + (uint32_t)(tid * per + j);
            cum = nx;
        }
    }
    __syncthreads();
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

/* The buckets holding ranks ra / rb from the counts in LDS: lane l takes the nsub/64
 * consecutive buckets from l * per (ds_read_b128), one wave scan of the lane sums, a ballot for
 * the lane, then a walk over that lane's buckets.  Writes bucket[i] and before[i] (the keys in
 * the buckets below it). */
__device__ __forceinline__ void wave_find_buckets(const uint32_t* lsub, int nsub, bool need_a, int64_t ra, bool need_b,
                                                  int64_t rb, int* bucket, int64_t* before) {
    const int lane = threadIdx.x & 63;
    const int per = nsub / 64; /* 1..16 */
    uint32_t c[16];
    const uint4* p4 = reinterpret_cast<const uint4*>(lsub + lane * per);
    if (per >= 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 t = q < per / 4 ? p4[q] : make_uint4(0u, 0u, 0u, 0u);
            c[4 * q] = t.x; c[4 * q + 1] = t.y; c[4 * q + 2] = t.z; c[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) c[q] = q < per ? lsub[lane * per + q] : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += c[q];
    const uint32_t incl = wave_scan_u32(s);
    const int64_t excl = (int64_t)(incl - s);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if (!(i == 0 ? need_a : need_b)) continue; /* uniform */
        const int64_t r = i == 0 ? ra : rb;
        const bool hit = excl <= r && r < (int64_t)incl;
        if (hit) { /* one lane: walk its buckets */
            int64_t cum = excl;
            int b = lane * per;
            bool go = true;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                go = go && q < per && r >= cum + (int64_t)c[q];
                if (go) { cum += c[q]; ++b; }
            }
            bucket[i] = b;
            before[i] = cum;
        }
    }
}

/* Resolve the two order statistics of one segment from its counters and buckets, compute the
 * NumPy threshold and the level-0 zero count, publish the results, and leave the slot clean.
 * One block of THREADS threads; `stage` holds up to stage_cap keys in LDS. */
template <int THREADS, bool COH = false>
__device__ float select_body(const SegDesc& sd, const SelState* __restrict__ st, const uint32_t* __restrict__ cand,
                             wtp_result* __restrict__ res, float* __restrict__ thr_out, uint32_t* stage,
                             int stage_cap, bool publish, uint32_t kl, uint32_t kh, uint32_t sh,
                             int* path_out = nullptr, uint32_t* hscratch = nullptr, bool prefer_wave = false) {
    __shared__ int sbin[2];
    __shared__ int64_t sbefore[2];
    __shared__ uint32_t lsub[NSUB_MAX];
    __shared__ unsigned long long s_cnt[4]; /* below, eq_lo, eq_hi (unused: 0), inside */
    __shared__ uint32_t s_mk, s_ovf;
    const int nsub = 1 << sd.nsub_log2;
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    WTP_PROBE(0);
    /* one round trip: threads 0..4 gather the sharded counters, wave 1 the bucket counts (to LDS) */
    if (threadIdx.x < 64) {
        const int l = threadIdx.x;
        if (l < 3) {
            const unsigned long long* a = l == 0 ? st->below : (l == 1 ? st->eq_lo : st->eq_hi);
            unsigned long long v = 0;
#pragma unroll
            for (int i = 0; i < NSHARD; ++i) v += ldc<COH>(a + i);
            s_cnt[l] = v;
        } else if (l == 3) {
            uint32_t m = 0;
#pragma unroll
            for (int i = 0; i < NSHARD; ++i) m = max(m, ldc<COH>(st->maxkey + i));
            s_mk = m;
        } else if (l == 4) {
            s_ovf = ldc<COH>(&st->overflow);
        }
    }
    /* wave 1: the bucket counts (bucket j * 64 + lane in sv[j]), every load issued before the
     * first is used -- 16 in flight per lane at nsub 1024, not 16 round trips in a row */
    uint32_t sv[NSUB_MAX / 64];
    if (threadIdx.x >= 64 && threadIdx.x < 128) {
        const int l = threadIdx.x - 64;
#pragma unroll
        for (int j = 0; j < NSUB_MAX / 64; ++j) sv[j] = (j * 64 + l < nsub) ? ldc<COH>(st->sub + j * 64 + l) : 0u;
        uint32_t sm = 0;
#pragma unroll
        for (int j = 0; j < NSUB_MAX / 64; ++j) {
            if (j * 64 + l < nsub) lsub[j * 64 + l] = sv[j];
            sm += sv[j];
        }
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
        WTP_PROBE_T(8, 64);
        if (threadIdx.x >= 64 && threadIdx.x < 128) /* wave 1: both ranks from one scan */
            wave_find_buckets(lsub, nsub, ca == 2, ja, cb == 2, jb, sbin, sbefore);
        WTP_PROBE_T(9, 64);
        __syncthreads();
        WTP_PROBE(2);
        blo = (ca == 2) ? sbin[0] : sbin[1];
        bhi = (cb == 2) ? sbin[1] : sbin[0];
        before = (ca == 2) ? sbefore[0] : sbefore[1];
        /* adjacent ranks: buckets strictly between blo and bhi are empty */
        nlo = lsub[blo];
        nhi = (bhi != blo) ? lsub[bhi] : 0;
        if (nlo > bcap || nhi > bcap) full = true;
        if (!full) {
            in_lds = nlo + nhi <= stage_cap;
            if (in_lds) { /* STAGE_BATCH loads in flight per thread before any is used */
                const int64_t m = nlo + nhi;
                for (int64_t i0 = 0; i0 < m; i0 += (int64_t)THREADS * STAGE_BATCH) {
                    uint32_t v[STAGE_BATCH];
#pragma unroll
                    for (int j = 0; j < STAGE_BATCH; ++j) {
                        const int64_t i = i0 + (int64_t)j * THREADS + threadIdx.x;
                        v[j] = i < m ? ldc<COH>(i < nlo ? c + (int64_t)blo * bcap + i : c + (int64_t)bhi * bcap + i - nlo)
                                     : 0u;
                    }
#pragma unroll
                    for (int j = 0; j < STAGE_BATCH; ++j) {
                        const int64_t i = i0 + (int64_t)j * THREADS + threadIdx.x;
                        if (i < m) stage[i] = v[j];
                    }
                }
                __syncthreads();
            }
            WTP_PROBE(3);
            const uint64_t lo64 = (uint64_t)kl + 1 + ((uint64_t)blo << sh);
            const uint64_t hi64 = min((uint64_t)kh, (uint64_t)kl + ((uint64_t)(bhi + 1) << sh));
            uint32_t xa = 0, xb = 0;
            const bool wave_ok = in_lds && nlo + nhi <= 64 * WSEL_KPL;
            if (in_lds && hscratch && hi64 - lo64 < (uint64_t)(HS_PER * THREADS) && !(prefer_wave && wave_ok)) {
                /* one LDS histogram over the bucket's key values: both ranks in one pass */
                __shared__ uint32_t sx[2], wt[THREADS / 64];
                block_hist_select<THREADS>(stage, (int)(nlo + nhi), (uint32_t)lo64, (int)(hi64 - lo64 + 1),
                                           (int)(ja - before), (int)(jb - before), hscratch, sx, wt);
                xa = sx[0];
                xb = sx[1];
            } else if (wave_ok) {
                /* a few hundred keys: one wave per rank, a bitwise search in registers */
                __shared__ uint32_t sx[2];
                const int wv = threadIdx.x >> 6;
                if (wv == 0 && ca == 2) {
                    const uint32_t k = wave_select_rank<WSEL_KPL>(stage, (int)(nlo + nhi), ja - before, (uint32_t)lo64, (uint32_t)hi64);
                    if ((threadIdx.x & 63) == 0) sx[0] = k;
                }
                if (wv == 1 && cb == 2) {
                    const uint32_t k = wave_select_rank<WSEL_KPL>(stage, (int)(nlo + nhi), jb - before, (uint32_t)lo64, (uint32_t)hi64);
                    if ((threadIdx.x & 63) == 0) sx[1] = k;
                }
                __syncthreads();
                xa = sx[0];
                xb = sx[1];
            } else {
                auto getb = [&](int64_t i) {
                    return in_lds ? stage[i]
                                  : ldc<COH>(i < nlo ? c + (int64_t)blo * bcap + i : c + (int64_t)bhi * bcap + i - nlo);
                };
                select_in_range<THREADS>(getb, [](uint32_t) { return true; }, nlo + nhi, (uint32_t)lo64,
                                         (uint32_t)hi64, ja - before, jb - before, ca == 2, cb == 2, &xa, &xb);
            }
            ka = (ca == 2) ? xa : (ca == 1 ? kl : kh);
            kb = (cb == 2) ? xb : (cb == 1 ? kl : kh);
            path = MODE_CAND;
            WTP_PROBE(4);
        }
    } else if (!full) {
        ka = (ca == 1) ? kl : kh;
        kb = (cb == 1) ? kl : kh;
    }
    if constexpr (!COH) { /* k_mask_select's select only (k_resident never sees a fused segment) */
        if (full && (sd.flags & SEG_FUSED)) {
            /* a fused segment: its window came from input patches; the retry launches take it
             * again from P (k_window / k_collect) -- nothing is published here */
            if (publish && threadIdx.x == 0) res[sd.res].path = MODE_RETRY;
            __syncthreads();
            return __uint_as_float(0x7FC00000u);
        }
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
    if (path_out) *path_out = path;
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
                                       : ldc<COH>(i < nlo ? c + (int64_t)blo * bcap + i
                                                          : c + (int64_t)bhi * bcap + i - nlo);
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
        if constexpr (COH) atomicMax(&r.path, path); /* a timed-out workgroup may raise it to MODE_FAULT */
        else r.path = r.path == MODE_RETRY ? path + MODE_RETRIED : path; /* the fused retry's select */
    }
    WTP_PROBE(6);
    return minp ? __uint_as_float(ka) : thr32;
}

/* k_window: one 1024-thread block per segment derives the window of the region k_collect is
 * about to fill (used when the window is not computed inline by every k_collect block) */
constexpr int WIN_THREADS = 1024;
__global__ __launch_bounds__(WIN_THREADS) void k_window(SegTable t, SelHeader* __restrict__ head,
                                                         const wtp_result* __restrict__ res) {
    __shared__ WindowLds<WIN_THREADS> wl;
    const SegDesc& sd = t.s[blockIdx.x];
    if (t.retry && res[sd.res].path != MODE_RETRY) return; /* block-uniform */
    /* the sample in passes of 16 keys a thread (groups of SAMPLE_GROUP contiguous keys spread
     * evenly over the segment, as sample_keys), histogrammed as they arrive */
    constexpr int PASS = 16 * WIN_THREADS, NPASS = M_SAMPLE_WIN / PASS;
    static_assert(M_SAMPLE_WIN % PASS == 0, "sample passes");
    for (int i = threadIdx.x; i < WindowLds<WIN_THREADS>::FBP * WIN_THREADS; i += WIN_THREADS) wl.h[i] = 0;
    if (threadIdx.x < 2) wl.found[threadIdx.x] = -1;
    __syncthreads();
    {
        const int64_t n = sd.n;
        const bool exact = n <= M_SAMPLE_WIN;
        const double step = exact ? 0.0 : (double)(n - SAMPLE_GROUP) / (double)(M_SAMPLE_WIN / SAMPLE_GROUP - 1);
        for (int ps = 0; ps < NPASS; ++ps) {
            uint32_t k[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int i = ps * PASS + j * WIN_THREADS + (int)threadIdx.x;
                const int64_t pos = exact ? min((int64_t)i, n - 1)
                                          : (int64_t)((double)(i / SAMPLE_GROUP) * step) + (i % SAMPLE_GROUP);
                k[j] = abs_key(sd.data[pos]);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (!exact || ps * PASS + j * WIN_THREADS + (int)threadIdx.x < n) atomicAdd(&wl.h[key_bin(k[j])], 1u);
        }
    }
    __syncthreads();
    uint32_t kl, kh, sh;
    window_search<WIN_THREADS, M_SAMPLE_WIN>(sd, wl, &kl, &kh, &sh);
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
template <int CT, int IT, bool WIN>
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
            collect_body<CT, IT, true, WIN>(sd, st, cand, base, len, first, lsub, lbase, stage, wl, wred, wtot);
        else
            collect_body<CT, IT, false, WIN>(sd, st, cand, base, len, first, lsub, lbase, stage, wl, wred, wtot);
    }
    __syncthreads(); /* every wave has read the parity */
    /* the grid's last block flips the parity (visible to the next kernel at the boundary).  Its
     * count is sharded (blockIdx % 8; the last block of a shard adds to the top counter, as in
     * k_small), so no single word takes a returning add from each of a cfg5 launch's ~25K blocks
     * (measured ~1 % of k_collect).  The counters sit in this region's BarState, zero at the
     * start of the launch (the previous launch cleared it as its idle region). */
    if (threadIdx.x == 0) {
        BarState* br = bar_region(head, q);
        const uint32_t sh = blockIdx.x & (NSHARD - 1);
        const uint32_t nsh = (gridDim.x - sh + NSHARD - 1) / NSHARD; /* blocks of this shard */
        const uint32_t nact = min((uint32_t)NSHARD, gridDim.x);     /* shards with blocks */
        if (atomicAdd(&br->arrive[sh][0], 1u) == nsh - 1u && atomicAdd(&br->arrive[0][16], 1u) == nact - 1u)
            head->parity = q + 1u;
    }
}

/* The fused selection's retry collect: k_collect_t over the chunks of the segments whose select
 * read MODE_RETRY only, as a grid-stride loop (a fixed small grid: when nothing missed, every block
 * reads the records and leaves); the housekeeping as k_collect_t (idle region, parity flip). */
template <int CT, int IT>
__global__ __launch_bounds__(CT) void k_collect_retry(SegTable t, SelHeader* __restrict__ head, uint32_t* __restrict__ cand,
                                                      wtp_result* __restrict__ res) {
    constexpr int SUB = IT * CT * 4, SPLIT = CHUNK / SUB;
    __shared__ uint32_t lsub[NSUB_MAX];
    __shared__ uint32_t lbase[NSUB_MAX];
    __shared__ uint32_t stage[STG * CT];
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
    const int total = t.nblk * SPLIT;
    for (int bb = blockIdx.x; bb < total; bb += gridDim.x) {
        const int tb = bb / SPLIT;
        const int si = find_seg(t, tb);
        const SegDesc& sd = t.s[si];
        if (res[sd.res].path != MODE_RETRY) continue; /* block-uniform */
        const int64_t base = (int64_t)(tb - sd.blk_begin) * CHUNK + (int64_t)(bb % SPLIT) * SUB;
        const int len = (int)max((int64_t)0, min((int64_t)SUB, sd.n - base));
        SelState* st = sel_region(head, q) + sd.slot;
        if (len > 0) {
            if ((sd.flags & SEG_ALIGNED) && len == SUB)
                collect_body<CT, IT, true, false>(sd, st, cand, base, len, false, lsub, lbase, stage, nullptr, wred, wtot);
            else
                collect_body<CT, IT, false, false>(sd, st, cand, base, len, false, lsub, lbase, stage, nullptr, wred, wtot);
        }
        __syncthreads(); /* LDS reused by the next chunk */
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        BarState* br = bar_region(head, q);
        const uint32_t sh = blockIdx.x & (NSHARD - 1);
        const uint32_t nsh = (gridDim.x - sh + NSHARD - 1) / NSHARD;
        const uint32_t nact = min((uint32_t)NSHARD, gridDim.x);
        if (atomicAdd(&br->arrive[sh][0], 1u) == nsh - 1u && atomicAdd(&br->arrive[0][16], 1u) == nact - 1u)
            head->parity = q + 1u;
    }
}

/* ------------------------------------------------------ fused selection --- */
/* k_fwin: the window of a fused segment before its forward (wtp_internal.h).  FWIN_NP blocks of
 * 1024 threads per segment, each transforming one patch of FWIN_PS^2 input samples in LDS --
 * pywt's periodization analysis at each level, the patch's own periodic extension -- and adding
 * the keys of every coefficient of every level to the segment's histogram (the FWIN_NP patches
 * give M_SAMPLE_WIN keys in the levels' population proportions); the segment's last block searches
 * the window as k_window does over its sample and leaves the histogram zeroed.  The sample is an
 * estimate: a window that misses the ranks is caught by the select, which then takes its exact
 * full-scan path, so the patches decide speed, never the result.  Patches sit at the centres of a
 * 4 x 4 Latin-square layout of the image (images b = patch % B).  Rows of the LDS images are
 * FWIN_PP = 129 floats apart: the row pass's lanes walk consecutive rows, conflict-free. */
constexpr int FWIN_RUN = 4; /* consecutive outputs per thread item: their samples shared in registers */
constexpr int FWIN_PP = FWIN_PS + 1;
template <int FT>
__global__ __launch_bounds__(FWIN_THREADS) void k_fwin(FwinTable t, SelHeader* __restrict__ head) {
    constexpr int PS = FWIN_PS, PP = FWIN_PP, NS = 2 * FWIN_RUN + FT - 2;
    __shared__ float A[PS * PP]; /* the patch, then each level's approximation */
    __shared__ float T[PS * PP]; /* a level's row-pass output: L | H halves of each row */
    __shared__ WindowLds<FWIN_THREADS> wl;
    __shared__ int s_last;
    const int si = blockIdx.x / FWIN_NP, pt = blockIdx.x - si * FWIN_NP;
    const FwinSeg& sg = t.s[si];
    for (int i = threadIdx.x; i < WindowLds<FWIN_THREADS>::FBP * FWIN_THREADS; i += FWIN_THREADS) wl.h[i] = 0;
    if (threadIdx.x < 2) wl.found[threadIdx.x] = -1;
    auto key = [&](float v) { atomicAdd(&wl.h[key_bin(abs_key(v))], 1u); };
    {
        /* eighths of the free range: rows 1, 3, 5, 7 against columns 3, 7, 1, 5 */
        const int lr = 1 + 2 * (pt & 3), lc = (0x5173 >> (4 * (pt & 3))) & 0xF;
        const int b = pt % sg.B;
        const int r0 = (int)((int64_t)(sg.R - PS) * lr / 8), c0 = (int)((int64_t)(sg.C - PS) * lc / 8);
        const float* x = sg.in + ((int64_t)b * sg.R + r0) * sg.C + c0;
        constexpr int PER = PS * PS / FWIN_THREADS; /* every load in flight before the first LDS write */
        float v[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = j * FWIN_THREADS + (int)threadIdx.x;
            v[j] = x[(int64_t)(i / PS) * sg.C + (i % PS)];
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = j * FWIN_THREADS + (int)threadIdx.x;
            A[(i / PS) * PP + (i % PS)] = v[j];
        }
    }
    __syncthreads();
    int N = PS; /* a power of two at every level: the periodic index is a mask */
    for (int k = 1; k <= sg.L; ++k) {
        const int h = N / 2, runs = (h + FWIN_RUN - 1) / FWIN_RUN; /* runs: a power of two or 1 */
        const int lN = __builtin_ctz(N);
        /* rows: output j of row r is sum_q f[q] x[(2j + 1 - q) mod N]; lanes take consecutive rows */
        for (int it = threadIdx.x; it < N * runs; it += FWIN_THREADS) {
            const int ru = it >> lN, r = it - (ru << lN), j0 = ru * FWIN_RUN;
            float v[NS];
#pragma unroll
            for (int m = 0; m < NS; ++m) v[m] = A[r * PP + ((2 * j0 + 2 - FT + m) & (N - 1))];
#pragma unroll
            for (int u = 0; u < FWIN_RUN; ++u) {
                float lo = 0.0f, hi = 0.0f;
#pragma unroll
                for (int q = 0; q < FT; ++q) {
                    lo += t.lo[q] * v[2 * u + FT - 1 - q];
                    hi += t.hi[q] * v[2 * u + FT - 1 - q];
                }
                if (j0 + u < h) { T[r * PP + j0 + u] = lo; T[r * PP + h + j0 + u] = hi; }
            }
        }
        __syncthreads();
        /* columns: lanes take consecutive columns */
        for (int it = threadIdx.x; it < N * runs; it += FWIN_THREADS) {
            const int ru = it >> lN, c = it - (ru << lN), i0 = ru * FWIN_RUN;
            float v[NS];
#pragma unroll
            for (int m = 0; m < NS; ++m) v[m] = T[((2 * i0 + 2 - FT + m) & (N - 1)) * PP + c];
#pragma unroll
            for (int u = 0; u < FWIN_RUN; ++u) {
                float lo = 0.0f, hi = 0.0f;
#pragma unroll
                for (int q = 0; q < FT; ++q) {
                    lo += t.lo[q] * v[2 * u + FT - 1 - q];
                    hi += t.hi[q] * v[2 * u + FT - 1 - q];
                }
                if (i0 + u < h) {
                    key(hi);
                    if (c >= h) key(lo);           /* a detail band */
                    else if (k == sg.L) key(lo);   /* the last level's approximation */
                    if (c < h) A[(i0 + u) * PP + c] = lo; /* the next level's input */
                }
            }
        }
        __syncthreads();
        N = h;
    }
    /* this patch's counts into the segment's histogram; the last patch block takes the window */
    uint32_t* gh = t.gh + (size_t)si * FWIN_HW;
    /* agent-scope atomics (performed at the coherence point), drained before the arrival -- no
     * release fence, whose L2 write-back per block cost ~0.6 us a block, serialised (MI355X_MICROARCH:
     * __threadfence); the last block reads the counts with sc1 loads */
    for (int i = threadIdx.x; i < NB; i += FWIN_THREADS)
        if (wl.h[i]) atomicAdd(&gh[i], wl.h[i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&gh[NB], 1u) == (uint32_t)(FWIN_NP - 1);
    __syncthreads();
    if (!s_last) return; /* block-uniform */
    for (int i = threadIdx.x; i < WindowLds<FWIN_THREADS>::FBP * FWIN_THREADS; i += FWIN_THREADS) {
        wl.h[i] = i < NB ? ldc<true>(gh + i) : 0u;
        if (i <= NB) gh[i] = 0; /* zero for the next launch (the counter too) */
    }
    if (threadIdx.x < 2) wl.found[threadIdx.x] = -1;
    __syncthreads();
    SegDesc sd = {};
    sd.n = sg.n;
    sd.r0 = sg.r0;
    sd.above = sg.above;
    sd.nsub_log2 = sg.nsub_log2;
    uint32_t kl, kh, sh;
    window_search<FWIN_THREADS, M_SAMPLE_WIN>(sd, wl, &kl, &kh, &sh);
    if (threadIdx.x == 0) { /* the window, and the forward's counters zeroed */
        FslHeader* hd = sg.hdr;
        hd->kl = kl;
        hd->kh = kh;
        hd->shift = sh;
        hd->overflow = 0;
    }
    if (threadIdx.x < NSHARD) {
        sg.hdr->maxkey[threadIdx.x] = 0;
        sg.hdr->be[threadIdx.x] = 0;
    }
}

/* k_fslot_collect: a fused group's bucket pass over its wave slots (k_fwd_int's inside keys).
 * A wave takes 64 slots, two per load: lanes 0-31 read words 0-31 of one slot and lanes 32-63 of
 * the next -- one 128-byte line per slot, which holds the count and up to 31 keys (a wave of the
 * forward classifies 768 coefficients, ~18 of them inside the window); a slot with more keys has
 * its second line read too.  Lane word j >= 1 holds key j - 1 and is kept when j <= the count.  The
 * keys are then bucketed as collect_finish buckets a chunk's (a block LDS histogram over the
 * window's buckets, one reservation per non-empty bucket, the scatter).  The forward already
 * counted the keys below and at kl and the largest key.  Housekeeping as k_collect: the idle region
 * cleared, the zero counts reset, the last block flips the parity. */
constexpr int FSC_SPW = FSC_SLOTS / (FSC_THREADS / 64); /* slots per wave */
constexpr int FSC_NP = FSC_SPW / 2;                     /* slot pairs per wave */
__global__ __launch_bounds__(FSC_THREADS) void k_fslot_collect(SegTable t, SelHeader* __restrict__ head,
                                                               uint32_t* __restrict__ cand, wtp_result* __restrict__ res) {
    static_assert(FSL_WORDS == 64 && FSC_NP <= 32, "two 32-word halves per slot, a pair bit per mask bit");
    __shared__ uint32_t lsub[NSUB_MAX];
    __shared__ uint32_t lbase[NSUB_MAX];
    __shared__ uint32_t s_any;
    const uint32_t q = head->parity;
    {   /* clear this block's slice of the idle region */
        uint4* idle = reinterpret_cast<uint4*>(sel_region(head, q ^ 1u));
        constexpr int NV4 = (int)(SEL_REGION / 16);
        const int per = (NV4 + (int)gridDim.x - 1) / (int)gridDim.x;
        for (int i = threadIdx.x; i < per; i += FSC_THREADS) {
            const int j = (int)blockIdx.x * per + i;
            if (j < NV4) idle[j] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    SelState* st = sel_region(head, q) + sd.slot;
    const FslHeader* hd = reinterpret_cast<const FslHeader*>(seg_fsl(sd));
    if ((int)blockIdx.x == sd.blk_begin) { /* the segment's first block: the head into the SelState */
        if (threadIdx.x == 0) {
            res[sd.res].zero_count = 0; /* the inverse adds */
            st->kl = hd->kl;
            st->kh = hd->kh;
            st->shift = hd->shift;
            if (hd->overflow) atomicOr(&st->overflow, 1u); /* other blocks may flag it too */
        }
        if (threadIdx.x < NSHARD) {
            const unsigned long long be = hd->be[threadIdx.x];
            st->below[threadIdx.x] = be & 0xFFFFFFFFull;
            st->eq_lo[threadIdx.x] = be >> 32;
            st->maxkey[threadIdx.x] = hd->maxkey[threadIdx.x];
        }
    }
    const int nsub = 1 << sd.nsub_log2;
    for (int i = threadIdx.x; i < nsub; i += FSC_THREADS) lsub[i] = 0;
    if (threadIdx.x == 0) s_any = 0;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, hl = lane >> 5, wj = lane & 31;
    const int s0 = ((int)blockIdx.x - sd.blk_begin) * FSC_SLOTS + wv * FSC_SPW;
    const int ns = max(0, min(FSC_SPW, seg_fsl_n(sd) - s0)); /* this wave's slots (uniform) */
    const uint32_t* base = seg_fsl(sd) + FSL_HDR_WORDS + (int64_t)s0 * FSL_WORDS;
    uint32_t w[FSC_NP];
#pragma unroll
    for (int p = 0; p < FSC_NP; ++p) w[p] = 2 * p + hl < ns ? base[(int64_t)(2 * p + hl) * FSL_WORDS + wj] : 0u;
    const uint32_t kl = hd->kl, sh = hd->shift;
    uint32_t keep = 0, ext = 0; /* bit p: this lane's first-line word of pair p is a key; pair p has a second line */
#pragma unroll
    for (int p = 0; p < FSC_NP; ++p) {
        const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)w[p], 0), c1 = (uint32_t)__builtin_amdgcn_readlane((int)w[p], 32);
        const uint32_t c = min(hl ? c1 : c0, (uint32_t)FSL_KEYS);
        if (2 * p + hl < ns && wj >= 1 && (uint32_t)wj <= c) keep |= 1u << p;
        if (max(c0, c1) > 31u) ext |= 1u << p; /* uniform */
    }
    /* a second-line word: key 31 + wj of its slot, kept when 32 + wj <= the count */
    auto second = [&](int p, uint32_t* kv) {
        const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)w[p], 0), c1 = (uint32_t)__builtin_amdgcn_readlane((int)w[p], 32);
        const uint32_t c = min(hl ? c1 : c0, (uint32_t)FSL_KEYS);
        const bool ok = 2 * p + hl < ns && (uint32_t)(32 + wj) <= c;
        *kv = ok ? base[(int64_t)(2 * p + hl) * FSL_WORDS + 32 + wj] : 0u;
        return ok;
    };
    /* a key's bucket; a key outside the window's buckets (never written by the forward, which
     * stores only inside keys) would mean a stale slot: dropped, and the segment retried */
    bool bad = false;
    auto bucket = [&](uint32_t k, uint32_t* b) {
        *b = (k - kl - 1) >> sh;
        const bool ok = *b < (uint32_t)nsub;
        bad = bad || !ok;
        return ok;
    };
    __syncthreads(); /* lsub cleared */
    if (keep || ext) {
        uint32_t b;
#pragma unroll
        for (int p = 0; p < FSC_NP; ++p)
            if (((keep >> p) & 1u) && bucket(w[p], &b)) atomicAdd(&lsub[b], 1u);
        for (uint32_t m = ext; m; m &= m - 1) { /* rare: a slot with more than 31 keys */
            uint32_t kv;
            if (second(__builtin_ctz(m), &kv) && bucket(kv, &b)) atomicAdd(&lsub[b], 1u);
        }
        if (keep) s_any = 1;
        if (bad) atomicOr(&st->overflow, 1u);
    }
    __syncthreads();
    if (!s_any && !__syncthreads_or(ext != 0)) goto done; /* uniform: no key in this block */
    {   /* one contiguous run per non-empty bucket (one returning atomic per bucket, all in flight) */
        constexpr int PER = NSUB_MAX / FSC_THREADS;
        uint32_t cj[PER], rj[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) cj[j] = (j * FSC_THREADS + (int)threadIdx.x < nsub) ? lsub[j * FSC_THREADS + threadIdx.x] : 0u;
#pragma unroll
        for (int j = 0; j < PER; ++j) rj[j] = cj[j] ? atomicAdd(&st->sub[j * FSC_THREADS + threadIdx.x], cj[j]) : 0u;
#pragma unroll
        for (int j = 0; j < PER; ++j)
            if (j * FSC_THREADS + (int)threadIdx.x < nsub) { lbase[j * FSC_THREADS + threadIdx.x] = rj[j]; lsub[j * FSC_THREADS + threadIdx.x] = 0; }
    }
    __syncthreads();
    {
        const int64_t bcap = sd.bucket_cap;
        uint32_t* out = cand + sd.cand_off;
        auto put = [&](uint32_t k) {
            const uint32_t b = (k - kl - 1) >> sh;
            if (b >= (uint32_t)nsub) return;
            const uint32_t at = lbase[b] + atomicAdd(&lsub[b], 1u);
            if (at < bcap) out[(int64_t)b * bcap + at] = k; /* counted beyond capacity: the select sees it */
        };
#pragma unroll
        for (int p = 0; p < FSC_NP; ++p)
            if ((keep >> p) & 1u) put(w[p]);
        for (uint32_t m = ext; m; m &= m - 1) {
            uint32_t kv;
            if (second(__builtin_ctz(m), &kv)) put(kv);
        }
    }
done:
    __syncthreads(); /* every wave has read the parity */
    if (threadIdx.x == 0) {
        BarState* br = bar_region(head, q);
        const uint32_t shd = blockIdx.x & (NSHARD - 1);
        const uint32_t nsh = (gridDim.x - shd + NSHARD - 1) / NSHARD;
        const uint32_t nact = min((uint32_t)NSHARD, gridDim.x);
        if (atomicAdd(&br->arrive[shd][0], 1u) == nsh - 1u && atomicAdd(&br->arrive[0][16], 1u) == nact - 1u)
            head->parity = q + 1u;
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
    if (t.retry && res[sd.res].path != MODE_RETRY) return;
    const int len = (int)min((int64_t)CHUNK, sd.n - base);
    const bool full = (sd.flags & SEG_ALIGNED) && len == CHUNK;
    /* the select first: loads return in issue order (vmcnt), so chunk loads issued ahead of
     * the select's would only delay its round trips -- and the chunk's 64 registers would sit
     * live through it */
    const SelState* st = sel_region(const_cast<SelHeader*>(head), head->parity ^ 1u) + sd.slot;
    int path = 0;
    const float thr = select_body<STREAM_THREADS>(sd, st, cand, res, thr_out, stage, MS_STAGE, base == 0, st->kl,
                                                  st->kh, st->shift, &path);
    if (!masked) return;
    /* a full-scan select reads the whole segment: in place, no block of it may write before
     * every block has scanned -- k_mask_inplace writes it in the next launch */
    if (path == MODE_FULL && sd.data == sd.out) return;
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

/* ------------------------------------------------------------- k_resident --- */
/* The level-0 prune of a whole launch group in ONE launch.  Every workgroup is resident (one per
 * CU; the host checks the grid against resident_capacity()) and holds its chunk in VGPRs from
 * the first read to the masked write, so HBM sees 4 B read + 4 B written per weight -- the
 * algorithmic minimum -- and the selection's two dependent steps run between them:
 *   P0  the sample loads, then the chunk's loads (RES_IT float4 per thread); the segment's
 *       window is built from the sample while the chunk is in flight (every workgroup of a
 *       segment draws the same sample and derives the same window)
 *   P1  from registers: count keys < kl and == kl, max key; histogram the keys inside (kl, kh]
 *       over the buckets in LDS, reserve one run per non-empty bucket (returning atomic), re-scan
 *       the registers and scatter the inside keys with write-through (sc1) stores
 *   --  grid barrier: each workgroup's waves drain their stores (vmcnt(0)), lane 0 adds to its
 *       shard's arrival counter (blockIdx % 8), wave 0 polls all shards with sc1 loads
 *   P2  every workgroup resolves its segment's threshold (select_body over sc1 loads); the
 *       segment's first workgroup publishes the record and the exact zero count
 *   P3  out = where(|x| < thr, 0, x) from registers
 * A segment whose window missed is re-scanned from memory (full radix select); when its input is
 * also its output (in place) its workgroups meet at a segment-wide barrier before any writes.
 * Every wait is bounded (RES_TIMEOUT of the 100 MHz wall clock): a grid that is not co-resident
 * after all drains instead of hanging, and its records read MODE_FAULT. */
/* The window search of k_resident for ONE wave over the flat NB-bin histogram h of the m sampled
 * keys: lane l owns the RES_BPL consecutive bins from l * RES_BPL (odd stride: no bank
 * conflicts); one scan of the lane sums finds the lane holding a sample rank, a second scan over
 * that lane's bins (RES_BPL - 1 by the lanes, the last one by elimination) finds the bin. */
constexpr int RES_BPL = 65;
constexpr int RES_HBINS = 64 * RES_BPL; /* >= NB; the bins past NB stay 0 */
static_assert(RES_HBINS >= NB, "flat window histogram");
__device__ __forceinline__ void wave_find_bins_flat(const uint32_t* h, int ra, int rb, int* fa, int* fb) {
    const int lane = threadIdx.x & 63;
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < RES_BPL; ++q) s += h[lane * RES_BPL + q];
    const int incl = (int)wave_scan_u32(s), excl = incl - (int)s;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = i == 0 ? ra : rb;
        int f = -1;
        const uint64_t msk = __ballot(r >= 0 && excl <= r && r < incl);
        if (msk) {
            const int L = __ffsll((unsigned long long)msk) - 1;
            const int before = __builtin_amdgcn_readlane(excl, L);
            const uint32_t c = h[L * RES_BPL + lane];
            const int i2 = before + (int)wave_scan_u32(lane < RES_BPL - 1 ? c : 0u);
            const int e2 = i2 - (int)(lane < RES_BPL - 1 ? c : 0u);
            const uint64_t m2 = __ballot(lane < RES_BPL - 1 && e2 <= r && r < i2);
            f = L * RES_BPL + (m2 ? __ffsll((unsigned long long)m2) - 1 : RES_BPL - 1);
        }
        if (i == 0) *fa = f; else *fb = f;
    }
}
__device__ __forceinline__ void window_search_flat(const SegDesc& sd, const uint32_t* h, int m, bool exact,
                                                   uint32_t* kl_out, uint32_t* kh_out, uint32_t* sh_out, double sig,
                                                   double add) {
    const int64_t n = sd.n;
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    int sa, sb;
    if (exact) {
        sa = (int)r0;
        sb = (int)r1;
    } else {
        const double p = (double)r0 / (double)(n - 1);
        const double s0 = p * (double)(m - 1), s1 = (double)r1 / (double)(n - 1) * (double)(m - 1);
        const double d = sig * sqrt((double)m * p * (1.0 - p)) + add;
        sa = (int)floor(s0 - d);
        sb = (int)ceil(s1 + d);
    }
    int f0, f1;
    wave_find_bins_flat(h, sa, sb < m ? sb : -1, &f0, &f1);
    const uint32_t kl = (sa < 0 || f0 < 0) ? 0u : bin_lo_key(f0);
    const uint32_t kh = (sb >= m || f1 < 0) ? 0xFFFFFFFFu : bin_hi_key(f1);
    uint32_t sh = 0;
    if (kh > kl + 1) {
        const uint32_t R = kh - kl - 1;
        const int bits = 32 - __clz(R);
        sh = bits > sd.nsub_log2 ? bits - sd.nsub_log2 : 0;
    }
    *kl_out = kl;
    *kh_out = kh;
    *sh_out = sh;
}


__device__ __forceinline__ uint64_t wall_ticks() { return __builtin_amdgcn_s_memrealtime(); }

/* Wait until the segment barrier counter reaches `want` arrivals (one lane polls with sc1 loads,
 * s_sleep between polls; the other waves wait at the workgroup barrier, then load).  A wait that
 * outlasts `timeout` ticks poisons the counter -- only while it is still short of `want`
 * (compare-and-swap) -- so every workgroup of the segment either passes the barrier or sees the
 * poison: all of them store, or none does.  Block-uniform result. */
__device__ __forceinline__ bool res_wait(uint32_t* ctr, uint32_t want, uint64_t timeout) {
    __shared__ int s_ok;
    if (threadIdx.x == 0) {
        const uint64_t t0 = wall_ticks();
        int ok = 0;
        while (true) {
            const uint32_t v = ldc<true>(ctr);
            if (v & RES_POISON) break;
            if (v >= want) { ok = 1; break; }
            if (wall_ticks() - t0 >= timeout) { /* >=: a zero bound poisons at the first incomplete look */
                if (atomicCAS(ctr, v, v | RES_POISON) == v) break;
                continue; /* it moved: look again */
            }
            __builtin_amdgcn_s_sleep(2);
        }
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

/* every wave drains its stores (vmcnt(0)), then lane 0 arrives: the sc1 hand-off form of
 * MI355X_MICROARCH.md (one arrival per workgroup for all its stores) */
__device__ __forceinline__ void res_arrive(uint32_t* ctr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(ctr, 1u);
}

/* the workspace parity, loaded at the kernel's start by a VECTOR load (qv) and made uniform only
 * where it is first needed, behind the chunk's loads: a scalar load of it is waited by the first
 * s_waitcnt lgkmcnt(0) -- every LDS barrier -- and put its device round trip (~1 us) ahead of
 * the sample's and the chunk's loads.  The asm keeps the read from being hoisted above the loads
 * (the wait the compiler inserts for it then counts only the older parity load). */
__device__ __forceinline__ uint32_t parity_late(uint32_t qv) {
    uint32_t q;
    asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(q) : "v"(qv) : "memory");
    return q;
}

/* k_resident's last pass: out = where(|x| < thr, 0, x) from registers; a NaN threshold prunes
 * nothing and the copy's zeros are counted (the pad slots read as +0.0 excluded) */
template <bool FULL>
__device__ __forceinline__ void res_final(const float4 (&v)[RES_IT], float thr, const SegDesc& sd,
                                          wtp_result* __restrict__ res, int64_t base, int len, bool al) {
    constexpr int CT = RES_THREADS, IT = RES_IT;
    const int tid = threadIdx.x;
    float* qo = sd.out + base;
    auto fin = [&](float xv) { return (fabsf(xv) < thr) ? 0.0f : xv; };
    if (FULL) {
        float4* q4 = reinterpret_cast<float4*>(qo);
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v yv = {fin(v[it].x), fin(v[it].y), fin(v[it].z), fin(v[it].w)};
            __builtin_nontemporal_store(yv, reinterpret_cast<f4v*>(q4 + it * CT + tid));
        }
    } else {
        const __amdgpu_buffer_rsrc_t rr = ragged_rsrc(qo, len);
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const float4 y = make_float4(fin(v[it].x), fin(v[it].y), fin(v[it].z), fin(v[it].w));
            store4_tail(y, qo, rr, it * CT + tid, len, al);
        }
    }
    if (thr != thr) { /* uniform */
        uint32_t z = 0;
#pragma unroll
        for (int it = 0; it < IT; ++it)
#pragma unroll
            for (int c = 0; c < 4; ++c) z += f4_get(v[it], c) == 0.0f;
        const unsigned long long tot = block_sum_u64<CT>(z) - (unsigned long long)(RES_CHUNK - len);
        if (tid == 0 && tot) atomicAdd((unsigned long long*)&res[sd.res].zero_count, tot);
    }
    WTP_RPROBE(7);
}

template <bool FULL>
__device__ __forceinline__ void res_body(const SegTable& t, const SegDesc& sd, SelHeader* __restrict__ head, uint32_t qv,
                                         uint32_t* __restrict__ cand, wtp_result* __restrict__ res,
                                         float* __restrict__ thr_out, int64_t base, int len, uint32_t* raw,
                                         uint32_t* lsub, uint32_t (*wred)[8], uint32_t* wstage, bool sel) {
    constexpr int CT = RES_THREADS, IT = RES_IT, NW = CT / 64;
    uint32_t q = 0;
    /* sel: this workgroup is its segment's selector (no chunk: len 0, its loads read nothing) */
    const bool first = base == 0 && !sel;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const uint64_t tmo = t.res_timeout;
    WTP_RPROBE(0);
    WTP_RTAG(sd.flags);
    __shared__ uint32_t s_win[3];
    __shared__ uint32_t s_sync; /* the sampling waves' LDS meeting counter */
    __shared__ uint32_t s_pubn; /* the storing waves drained (publication) */
    __shared__ uint32_t s_arr;  /* wave 7's first-level parity arrival */
    float4 v[IT];
    uint32_t arr1 = 0; /* wave 7 lane 0: the first-level parity arrival's result */
    /* ---- P0: the sample waves' loads go out before any chunk load of the workgroup (the barrier
     * below orders them), then every wave issues its chunk; the sample arrives first (a wave's
     * loads return in order) and is histogrammed while the chunk streams in; wave 0 searches the
     * histogram for the window [kl, kh] bracketing the segment's two ranks */
    {
        uint32_t ks[RES_SPL];
        const int64_t n = sd.n;
        const bool exact = n <= RES_MS;
        const int m = exact ? (int)n : RES_MS;
        if (wv < RES_SW) {
            /* group g = i / SAMPLE_GROUP starts at floor(g * (n - SAMPLE_GROUP) / (RES_MS / SAMPLE_GROUP - 1)),
             * in 32.32 fixed point from the host (res_step_fx): two 32-bit multiplies a load */
            const uint32_t sl = (uint32_t)sd.res_step_fx, shi = (uint32_t)(sd.res_step_fx >> 32);
#pragma unroll
            for (int j = 0; j < RES_SPL; ++j) {
                const int i = j * (64 * RES_SW) + tid;
                const uint32_t g = (uint32_t)i / SAMPLE_GROUP;
                const int pos = exact ? min(i, (int)n - 1)
                                      : (int)(__umulhi(g, sl) + g * shi) + (i % SAMPLE_GROUP);
                ks[j] = __float_as_uint(sd.data[pos]); /* raw bits: |x| at the histogram */
            }
        }
        for (int j = tid; j < RES_HBINS; j += CT) raw[j] = 0u;
        for (int j = tid; j < RES_NSUB; j += CT) lsub[j] = 0u;
        if (tid == 0) { s_sync = 0u; s_pubn = 0u; }
        if (first && tid == 0) { /* memory-side words: later adds come from other workgroups */
            stc(reinterpret_cast<unsigned long long*>(&res[sd.res].zero_count), 0ull);
            stc(&res[sd.res].path, 0);
        }
        __syncthreads(); /* the sample's loads are out before any chunk load of the workgroup */
        WTP_RPROBE(8);
        /* the sampling waves histogram their sample (it comes back ahead of the flood) and wave 0
         * searches the window; the other waves go straight to the loads.  The chunk is loaded at
         * ONE program point by every wave: a single definition of v[], so the compiler keeps the
         * loads' destination registers and nothing waits for the data before it is counted; the
         * sample's |x| is taken here, behind the barrier, by an AND the compiler cannot fold back
         * into the loads' block (it would make the sampling waves wait for the sample before the
         * barrier) */
        if (wv < RES_SW) {
#pragma unroll
            for (int j = 0; j < RES_SPL; ++j)
                if (j * (64 * RES_SW) + tid < m) {
                    uint32_t k;
                    asm volatile("v_and_b32 %0, 0x7fffffff, %1" : "=v"(k) : "v"(ks[j]));
                    atomicAdd(&raw[key_bin(k)], 1u);
                }
            /* the sampling waves meet on an LDS counter (the others do not wait for them) */
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) atomicAdd(&s_sync, 1u);
            if (wv == 0) {
                while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_sync, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_WORKGROUP)) < (uint32_t)RES_SW)
                    __builtin_amdgcn_s_sleep(1);
                asm volatile("" ::: "memory");
                uint32_t wkl, wkh, wsh;
                window_search_flat(sd, raw, m, exact, &wkl, &wkh, &wsh, RES_SIGMA_X100 * 0.01, 8.0);
                if (lane == 0) { s_win[0] = wkl; s_win[1] = wkh; s_win[2] = wsh; }
                WTP_RPROBE(1);
            }
        }
        /* a late workgroup (SEG_LATE: the group's small segments) issues its chunk only once
         * the window is known: the early group's chunks come off HBM first, and their counts,
         * barriers and selects run while the late group's chunks stream */
        if (sd.flags & SEG_LATE) __syncthreads(); /* block-uniform */
        if (FULL) load_chunk<IT, CT, true>(sd.data + base, v);
        else load_chunk_ragged<IT, CT, true>(sd.data + base, len, v);
        q = parity_late(qv);
        {   /* clear this workgroup's slice of the idle region (the previous launch's; the next
             * launch works in it): stores behind the chunk's loads */
            uint4* idle = reinterpret_cast<uint4*>(sel_region(head, q ^ 1u));
            constexpr int NV4 = (int)(SEL_REGION / 16);
            const int per = (NV4 + (int)gridDim.x - 1) / (int)gridDim.x;
            for (int i = tid; i < per; i += CT) {
                const int j = (int)blockIdx.x * per + i;
                if (j < NV4) idle[j] = make_uint4(0u, 0u, 0u, 0u);
            }
        }
        /* the parity flip's first-level arrival (the last reader of the parity in the grid flips
         * it): a returning add issued behind wave 7's chunk loads, its result used only at the
         * publication, so its queueing on the shard's counter costs no wave a wait */
        if (wv == NW - 1 && lane == 0) arr1 = atomicAdd(&bar_region(head, q)->arrive[blockIdx.x & (NSHARD - 1)][0], 1u);
        WTP_RPROBE(10);
    }
    __syncthreads();
    SelState* st = sel_region(head, q) + sd.slot;
    const uint32_t kl = s_win[0], kh = s_win[1];
    /* ---- P1: one branch-free pass over the registers, two classes per key from one difference
     * d = k - kl (keys and kl < 2^31): "below" (k < kl: bit 31 of d) and "inside" [kl, kh]
     * (d <= span; keys == kl belong to bucket 0), the max key, and the inside keys appended to the
     * thread's own LDS column (slot j of thread t at col[j * CT]; every key is written to the next
     * free slot and kept only if inside -- no branch, no atomic).  In a ragged chunk the slots
     * past len were loaded as +0.0: never inside, counted below (kl > 0) and dropped once. */
    const uint32_t span = kh - kl; /* >= 1 */
    uint32_t sh = 0; /* bucket of an inside key: (k - kl) >> sh, RES_NSUB buckets */
    if (span > 0) {
        const int bits = 32 - __clz(span);
        sh = bits > RES_NSUB_LOG2 ? bits - RES_NSUB_LOG2 : 0;
    }
    uint32_t wbelow = 0, mx = 0, cnt = 0;
    uint32_t* col = wstage + tid;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        uint32_t k4[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) k4[c] = abs_key(opaque(f4_get(v[it], c)));
        mx = max(mx, max(max(k4[0], k4[1]), max(k4[2], k4[3])));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t k = k4[c];
            const uint32_t d = k - kl;
            wbelow += d >> 31;
            col[min(cnt, (uint32_t)RES_STG) * CT] = k;
            const bool valid = FULL || 4 * (it * CT + tid) + c < len;
            cnt += (d <= span) & valid;
        }
    }
    {
        wbelow = wave_sum_u32(wbelow);
        const uint32_t r2 = wave_max_u32(mx), r4 = wave_max_u32(cnt);
        if (lane == 0) { wred[wv][0] = wbelow; wred[wv][2] = r2; wred[wv][5] = r4; }
    }
    __syncthreads();
    WTP_RPROBE(2);
    if (wv == NW - 1 && lane == 0) s_arr = arr1;
    uint32_t wmax = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) wmax = max(wmax, wred[w][5]);
    /* block-uniform: a thread's column overflowed -> the segment takes the full scan */
    const bool ovf = wmax > (uint32_t)RES_STG;
    /* a segment of ONE workgroup (solo) selects from its own LDS: no counter, bucket total,
     * publication or barrier touches memory -- under the launch's traffic every round trip costs
     * 1-3 us, and the solo segments were the launch's tail */
    const uint32_t nwg = (uint32_t)((sd.n + RES_CHUNK - 1) / RES_CHUNK);
    const bool solo = nwg == 1u; /* block-uniform */
    /* remote: a shared segment whose select runs on its selector workgroup (a CU that holds no
     * chunk: the select's dependent round trips start from an idle memory queue); its workgroups
     * only wait for the threshold granule */
    const bool remote = t.nsel > 0 && !solo; /* block-uniform */
    const bool al = (sd.flags & SEG_ALIGNED) != 0;
    __shared__ unsigned long long s_cnt[1];
    __shared__ uint32_t s_mk, s_ovf;
    if (tid == 0) {
        unsigned long long a0 = 0;
        uint32_t m2 = 0;
        for (int w = 0; w < NW; ++w) { a0 += wred[w][0]; m2 = max(m2, wred[w][2]); }
        if (kl > 0) a0 -= (unsigned long long)(RES_CHUNK - len);
        if (solo) {
            s_cnt[0] = a0;
            s_mk = m2;
            s_ovf = ovf;
        } else if (!sel) {
            const int sh8 = blockIdx.x & (NSHARD - 1);
            if (a0) atomicAdd(&st->below[sh8], a0);
            atomicMax(&st->maxkey[sh8], m2);
            if (ovf) atomicOr(&st->overflow, 1u);
        }
    }
    /* the inside keys' bucket histogram in LDS (eight column reads in flight per step), then the
     * segment's bucket totals as no-return atomic adds */
    constexpr int BPT = RES_NSUB / CT; /* buckets per thread */
    static_assert(BPT * CT == RES_NSUB, "buckets per thread");
    if (!ovf) { /* block-uniform */
        for (uint32_t j0 = 0; j0 < cnt; j0 += 8) {
            uint32_t kk[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) kk[u] = col[min(j0 + u, (uint32_t)RES_STG) * CT];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (j0 + u < cnt) atomicAdd(&lsub[(kk[u] - kl) >> sh], 1u);
        }
        __syncthreads();
        if (!solo && !sel) {
#pragma unroll
            for (int j = 0; j < BPT; ++j) { /* bucket j * CT + tid: 256 contiguous bytes per wave instruction */
                const uint32_t c = lsub[j * CT + tid];
                if (c) atomicAdd(&st->sub[j * CT + tid], c);
            }
        }
    }
    WTP_RPROBE(3);
    /* ---- segment barrier 1: every workgroup's counters and bucket totals are in */
    BarState* bar = bar_region(head, q);
    uint32_t* b0 = reinterpret_cast<uint32_t*>(&st->seg_bar[0]);
    uint32_t* b1 = reinterpret_cast<uint32_t*>(&st->seg_bar[1]);
    uint32_t* b2 = reinterpret_cast<uint32_t*>(&st->seg_bar[2]);
    if (!solo) {
        if (sel) __syncthreads(); /* orders s_arr for wave 6 (the selector has no publication) */
        else res_arrive(b1);
    }
    WTP_RPROBE(4);
    /* ---- publication, while the segment gathers at barrier 1: this workgroup's inside keys,
     * bucket-sorted in LDS, and the bucket offsets (exclusive prefix of its bucket histogram),
     * write-through (16-byte sc1 stores) to its region of the candidate area, then barrier 2's
     * arrival.  It depends on nothing global: waves 0-6 store and drain it while wave 7 polls
     * barrier 1, and after barrier 1 the select reads only the keys of the ranks' buckets from
     * the regions (offsets, then keys: two round trips) -- no slot round after the locate. */
    uint32_t* pub = cand + (int64_t)blockIdx.x * RES_PUB_WORDS;
    uint32_t* pos = raw;     /* bucket offsets (the window histogram is done with) */
    uint32_t* srt = wstage;  /* the sorted keys, over the columns */
    __shared__ uint32_t s_ok1;
    if (!ovf && !sel) { /* block-uniform */
        uint32_t kk[RES_STG];
#pragma unroll
        for (int j = 0; j < RES_STG; ++j) kk[j] = col[j * CT]; /* entries past cnt are not used */
        /* exclusive scan of the bucket counts, BPT buckets per thread */
        __shared__ uint32_t s_pw[NW];
        uint32_t c[BPT], cs = 0;
#pragma unroll
        for (int j = 0; j < BPT; ++j) { c[j] = lsub[BPT * tid + j]; cs += c[j]; }
        const uint32_t inc = wave_scan_u32(cs);
        if (lane == 63) s_pw[wv] = inc;
        __syncthreads(); /* also: every column is read into kk */
        uint32_t ex = inc - cs;
#pragma unroll
        for (int w = 0; w < NW; ++w) ex += w < wv ? s_pw[w] : 0u;
#pragma unroll
        for (int j = 0; j < BPT; ++j) { pos[BPT * tid + j] = ex; ex += c[j]; }
        __syncthreads();
        /* scatter, four keys at a time with no branch (a key past cnt counts into its lane's
         * spare counter pos[RES_NSUB + lane] -- one per lane: a shared one serialised every
         * atomic 64 ways -- and lands in the spare words past the sorted array): the four
         * returning atomics issue back to back; the trip count is the wave's largest cnt */
        const uint32_t wc = wred[wv][5];
#pragma unroll
        for (int j0 = 0; j0 < RES_STG; j0 += 4) {
            if ((uint32_t)j0 < wc) {
                uint32_t pp[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool ok = (uint32_t)(j0 + u) < cnt;
                    pp[u] = atomicAdd(&pos[ok ? (kk[j0 + u] - kl) >> sh : (uint32_t)(RES_NSUB + lane)], 1u);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool ok = (uint32_t)(j0 + u) < cnt;
                    srt[ok ? pp[u] : (uint32_t)(RES_STG * CT + lane)] = kk[j0 + u];
                }
            }
        }
        __syncthreads();
    }
    WTP_RPROBE(9);
    if (solo) {
        /* s_arr (wave 7's store after its returning add) must be visible to wave 6: on the
         * non-overflow path the publication's barriers order it; an overflowing solo segment has
         * none of them (block-uniform branch) */
        if (ovf) __syncthreads();
        /* the parity flip's second level (as the storing waves do it below) */
        if (tid == 64 * (NW - 2)) {
            const uint32_t sh8 = blockIdx.x & (NSHARD - 1);
            const uint32_t nsh = (gridDim.x - sh8 + NSHARD - 1) / NSHARD;
            const uint32_t nact = min((uint32_t)NSHARD, gridDim.x);
            if (s_arr == nsh - 1u && atomicAdd(&bar->arrive[0][16], 1u) == nact - 1u) stc(&head->parity, q + 1u);
        }
        if (tid == 0) s_ok1 = 1;
    } else if (wv == NW - 1 && remote && !sel) {
        if (lane == 0) s_ok1 = 1; /* a remote segment's workgroup does not wait at barrier 1 */
    } else if (wv == NW - 1) {
        /* ---- barrier 1, polled by wave 7 while the others store (the selector: by wave 7) */
        if (lane == 0) {
            const uint64_t t0 = wall_ticks();
            uint32_t ok = 0;
            while (true) {
                const uint32_t x = ldc<true>(b1);
                if (x & RES_POISON) break;
                if (x >= nwg) { ok = 1; break; }
                if (wall_ticks() - t0 >= tmo) {
                    if (atomicCAS(b1, x, x | RES_POISON) == x) break;
                    continue; /* it moved: look again */
                }
                __builtin_amdgcn_s_sleep(2);
            }
            s_ok1 = ok;
        }
    } else {
        constexpr int ST = CT - 64; /* the storing threads */
        if (!ovf && !sel) {
            /* offsets: pub[b] = start of bucket b (pos[b - 1] now), pub[RES_NSUB] = the total */
            const __amdgpu_buffer_rsrc_t prs = region_rsrc(pub, RES_PUB_WORDS);
            if (tid < RES_NSUB / 4) {
                const int b = 4 * tid;
                st16_sc1(prs, b, make_uint4(b ? pos[b - 1] : 0u, pos[b], pos[b + 1], pos[b + 2]));
            } else if (tid == RES_NSUB / 4) {
                stc(pub + RES_NSUB, pos[RES_NSUB - 1]);
            }
            const uint32_t nin = pos[RES_NSUB - 1];
            for (uint32_t i4 = tid; 4 * i4 < nin; i4 += ST)
                st16_sc1(prs, RES_PUB_KEYS + 4 * i4, *reinterpret_cast<const uint4*>(srt + 4 * i4));
        }
        /* every storing wave drains; the last one to do so arrives at barrier 2 for the
         * workgroup (its LDS add follows every other storing wave's drain) */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!sel && lane == 0 && atomicAdd(&s_pubn, 1u) == (uint32_t)(NW - 2)) atomicAdd(b2, 1u);
        /* the parity flip's second level: the last reader of a shard (blockIdx % 8) adds to the
         * top counter, whose last arrival flips the parity (every workgroup of the grid has read
         * it) -- wave 6, after its drain, off the barrier-1 poll */
        if (wv == NW - 2 && lane == 0) {
            const uint32_t sh8 = blockIdx.x & (NSHARD - 1);
            const uint32_t nsh = (gridDim.x - sh8 + NSHARD - 1) / NSHARD;
            const uint32_t nact = min((uint32_t)NSHARD, gridDim.x);
            if (s_arr == nsh - 1u && atomicAdd(&bar->arrive[0][16], 1u) == nact - 1u) stc(&head->parity, q + 1u);
        }
    }
    __syncthreads();
    WTP_RPROBE(11);
    uint64_t* gr = reinterpret_cast<uint64_t*>(&st->thr_gr);
    if (!s_ok1) {
        if (tid == 0) {
            atomicMax(&res[sd.res].path, (int32_t)MODE_FAULT);
            if (sel) atomicCAS(reinterpret_cast<unsigned long long*>(gr), 0ull, (unsigned long long)RES_GR_FAULT << 32);
        }
        return; /* nothing stored to the output: the caller's input and output are untouched */
    }
    WTP_RPROBE(5);
    if (remote && !sel) {
        /* ---- the threshold granule {thr bits, tag} from the segment's selector (one 8-byte sc1
         * word; the region is zero at the launch's start).  A wait that times out claims the
         * granule for FAULT by compare-and-swap, so every workgroup of the segment and the
         * selector agree: all store, or none does */
        __shared__ unsigned long long s_gr;
        if (wv == NW - 1 && lane == 0) {
            const uint64_t t0 = wall_ticks();
            unsigned long long x;
            while (true) {
                x = ldc<true>(reinterpret_cast<const unsigned long long*>(gr));
                if (x) break;
                if (wall_ticks() - t0 >= tmo) {
                    const unsigned long long f = (unsigned long long)RES_GR_FAULT << 32;
                    const unsigned long long o = atomicCAS(reinterpret_cast<unsigned long long*>(gr), 0ull, f);
                    x = o ? o : f;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            s_gr = x;
        }
        __syncthreads();
        const unsigned long long g = s_gr;
        const uint32_t tag = (uint32_t)(g >> 32);
        if (tag & RES_GR_FAULT) {
            if (tid == 0) atomicMax(&res[sd.res].path, (int32_t)MODE_FAULT);
            return;
        }
        const float thr = __uint_as_float((uint32_t)g);
        WTP_RPROBE(6);
        res_final<FULL>(v, thr, sd, res, base, len, al);
        return;
    }
    /* ---- P2: the segment's counters and bucket totals in one round trip (every load in
     * flight before any is used); a block scan of the totals names the bucket of each rank */
    __shared__ uint32_t s_wtot[NW], s_b2;
    __shared__ int s_bk[2];
    __shared__ uint32_t s_bef[2], s_bn[2];
    if (!solo) {
        if (tid == 0) {
            unsigned long long x[NSHARD];
#pragma unroll
            for (int i = 0; i < NSHARD; ++i) x[i] = ldc<true>(st->below + i);
            unsigned long long sum = 0;
#pragma unroll
            for (int i = 0; i < NSHARD; ++i) sum += x[i];
            s_cnt[0] = sum;
        } else if (tid == 2) {
            uint32_t x[NSHARD];
#pragma unroll
            for (int i = 0; i < NSHARD; ++i) x[i] = ldc<true>(st->maxkey + i);
            uint32_t mm = 0;
#pragma unroll
            for (int i = 0; i < NSHARD; ++i) mm = max(mm, x[i]);
            s_mk = mm;
        } else if (tid == 3) {
            s_ovf = ldc<true>(&st->overflow);
        } else if (tid == 4) {
            /* barrier 2's counter in the same round trip: its arrivals were made before barrier
             * 1's wait, so it is usually complete already and its poll round trip is skipped */
            s_b2 = ldc<true>(b2);
        }
    }
    if (tid < 2) { s_bk[tid] = -1; s_bef[tid] = 0; s_bn[tid] = 0; }
    uint32_t cb8[BPT]; /* buckets BPT * tid .. + BPT - 1, every load in flight before any is used */
#pragma unroll
    for (int j = 0; j < BPT; ++j) cb8[j] = solo ? lsub[BPT * tid + j] : ldc<true>(st->sub + BPT * tid + j);
    uint32_t cs = 0;
#pragma unroll
    for (int j = 0; j < BPT; ++j) cs += cb8[j];
    const uint32_t incl = wave_scan_u32(cs);
    if (lane == 63) s_wtot[wv] = incl;
    __syncthreads();
    WTP_PROBE(1);
    const int64_t sbelow = (int64_t)s_cnt[0];
    const uint32_t mk = s_mk;
    uint32_t excl = incl - cs, ninside = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) { const uint32_t x = s_wtot[w]; ninside += x; excl += w < wv ? x : 0u; }
    const int64_t r0 = sd.r0, r1 = sd.above ? sd.r0 : sd.r0 + 1;
    /* class of a rank: 0 outside the window, 2 inside [kl, kh] at inside-rank j */
    auto classify = [&](int64_t r, int64_t* j) {
        if (r < sbelow) return 0;
        r -= sbelow;
        if (r < (int64_t)ninside) { *j = r; return 2; }
        return 0;
    };
    int64_t ja = 0, jb = 0;
    const int ca = classify(r0, &ja), cb = classify(r1, &jb);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int64_t j = i == 0 ? ja : jb;
        if ((i == 0 ? ca : cb) == 2 && j >= (int64_t)excl && j < (int64_t)(excl + cs)) {
            uint32_t e = excl;
            int b = BPT * tid;
#pragma unroll
            for (int u = 0; u < BPT - 1; ++u) {
                const bool past = j >= (int64_t)(e + cb8[u]) && b == BPT * tid + u;
                e += past ? cb8[u] : 0u;
                b += past ? 1 : 0;
            }
            s_bk[i] = b;
            s_bef[i] = e;
            s_bn[i] = cb8[b - BPT * tid];
        }
    }
    __syncthreads();
    WTP_PROBE(2);
    bool full = ca == 0 || cb == 0 || s_ovf != 0;
    int path = MODE_WINDOW;
    uint32_t ka = kl, kb = kl;
    uint32_t before = 0;
    int m = 0;
    uint32_t* stage = raw; /* the window histogram is done with */
    const uint32_t* sel_keys = stage; /* the staged keys of the ranks' buckets */
    if (!full && (ca == 2 || cb == 2)) {
        const int ba = ca == 2 ? s_bk[0] : s_bk[1], bb = cb == 2 ? s_bk[1] : s_bk[0];
        before = ca == 2 ? s_bef[0] : s_bef[1];
        const uint32_t nlo = ca == 2 ? s_bn[0] : s_bn[1], nhi = (bb != ba) ? s_bn[1] : 0u;
        m = (int)(nlo + nhi);
        if (solo) {
            /* the ranks' buckets ba..bb are one run of this workgroup's sorted keys in LDS (the
             * buckets between are empty); pos[b] is the end of bucket b after the scatter */
            sel_keys = srt + (ba ? pos[ba - 1] : 0u);
            const uint32_t lo = (uint32_t)((uint64_t)kl + ((uint64_t)ba << sh));
            const uint32_t hi = (uint32_t)min((uint64_t)kh, (uint64_t)kl + ((uint64_t)(bb + 1) << sh) - 1);
            uint32_t xa = kl, xb = kl;
            select_in_range<CT>([&](int64_t i) { return sel_keys[i]; }, [](uint32_t) { return true; }, (int64_t)m, lo,
                                hi, ja - (int64_t)before, jb - (int64_t)before, ca == 2, cb == 2, &xa, &xb);
            ka = ca == 2 ? xa : kl;
            kb = cb == 2 ? xb : kl;
            path = MODE_CAND;
        } else if (m > RES_SEL_MAX) {
            full = true; /* uniform over the segment: the same totals everywhere */
        } else {
            /* ---- barrier 2: every region of the segment is published (its arrivals were made
             * before barrier 1's wait, so this wait is short) */
            WTP_PROBE(3);
            const uint32_t b2v = s_b2; /* block-uniform */
            if (!(b2v >= nwg && !(b2v & RES_POISON)) && !res_wait(b2, nwg, tmo)) {
                if (tid == 0) {
                    atomicMax(&res[sd.res].path, (int32_t)MODE_FAULT);
                    if (sel) atomicCAS(reinterpret_cast<unsigned long long*>(gr), 0ull, (unsigned long long)RES_GR_FAULT << 32);
                }
                return;
            }
            WTP_PROBE(4);
            /* ---- the segment's workgroups' offsets of buckets ba and bb + 1 (wave 0, every load
             * in flight at once), their key counts scanned; then the keys themselves, at most two
             * a thread (m <= RES_SEL_MAX), staged in LDS.  The buckets between ba and bb are
             * empty, so a workgroup's keys of ba..bb are one run of its sorted array. */
            const int wb = sd.blk_begin;
            __shared__ uint32_t s_so[RES_MAX_WG], s_ob[RES_MAX_WG];
            __shared__ uint32_t s_tot;
            if (wv == 0) {
                constexpr int WPL = RES_MAX_WG / 64;
                uint32_t ob[WPL], oe[WPL];
#pragma unroll
                for (int u = 0; u < WPL; ++u) {
                    const int w = lane + 64 * u;
                    const uint32_t* pw = cand + (int64_t)(wb + min(w, (int)nwg - 1)) * RES_PUB_WORDS;
                    ob[u] = ldc<true>(pw + ba);
                    oe[u] = ldc<true>(pw + bb + 1);
                }
                uint32_t base = 0;
#pragma unroll
                for (int u = 0; u < WPL; ++u) {
                    const int w = lane + 64 * u;
                    const uint32_t cw = w < (int)nwg ? oe[u] - ob[u] : 0u;
                    const uint32_t inc = wave_scan_u32(cw);
                    if (w < (int)nwg) { s_so[w] = base + inc - cw; s_ob[w] = ob[u]; }
                    base += __builtin_amdgcn_readlane(inc, 63);
                }
                if (lane == 0) s_tot = base;
            }
            __syncthreads();
            if ((int)s_tot != m) {
                full = true; /* uniform over the segment (the same regions everywhere) */
            } else {
                uint32_t kv[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int i = min(tid + u * CT, m - 1);
                    int lo_w = 0, hi_w = (int)nwg - 1; /* the last workgroup whose run starts <= i */
                    while (lo_w < hi_w) {
                        const int mid = (lo_w + hi_w + 1) >> 1;
                        if (s_so[mid] <= (uint32_t)i) lo_w = mid; else hi_w = mid - 1;
                    }
                    kv[u] = ldc<true>(cand + (int64_t)(wb + lo_w) * RES_PUB_WORDS + RES_PUB_KEYS + s_ob[lo_w] +
                                      ((uint32_t)i - s_so[lo_w]));
                }
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    if (tid + u * CT < m) stage[tid + u * CT] = kv[u];
                __syncthreads();
                WTP_PROBE(5);
                /* ---- the ranks among the staged keys (buckets ba..bb; buckets between are empty:
                 * the two ranks are adjacent): an LDS radix select of both at once */
                const uint32_t lo = (uint32_t)((uint64_t)kl + ((uint64_t)ba << sh));
                const uint32_t hi = (uint32_t)min((uint64_t)kh, (uint64_t)kl + ((uint64_t)(bb + 1) << sh) - 1);
                uint32_t xa = kl, xb = kl;
                select_in_range<CT>([&](int64_t i) { return stage[i]; }, [](uint32_t) { return true; }, (int64_t)m,
                                    lo, hi, ja - (int64_t)before, jb - (int64_t)before, ca == 2, cb == 2, &xa, &xb);
                ka = ca == 2 ? xa : kl;
                kb = cb == 2 ? xb : kl;
                path = MODE_CAND;
            }
        }
    }
    WTP_PROBE(6);
    if (full) {
        /* the window missed (or a column or slot overflowed): exact radix select over the
         * segment's input in memory -- every workgroup of the segment takes this branch */
        const float* x = sd.data;
        select_in_range<CT>([&](int64_t i) { return abs_key(x[i]); }, [](uint32_t) { return true; }, sd.n, 0u,
                            0xFFFFFFFFu, r0, r1, true, true, &ka, &kb);
        path = MODE_FULL;
    }
    /* threshold: numpy/lib/function_base.py _lerp -- diff in float32, the blend in float64 */
    const float fa = __uint_as_float(ka), fb = __uint_as_float(kb);
    const float diff = fb - fa;
    const double g = sd.gamma;
    double thr64 = (g >= 0.5) ? (double)fb - (double)diff * (1.0 - g) : (double)fa + (double)diff * g;
    if (mk > 0x7F800000u) thr64 = __longlong_as_double(0x7FF8000000000000ll); /* NaN present: np.percentile is NaN */
    const float thr = (float)thr64;
    const bool nan = thr != thr; /* also inf - inf inside the lerp */
    if (sel && tid == 0) {
        /* the threshold granule for the segment's workgroups, ahead of the record: {thr bits, tag},
         * claimed by compare-and-swap (a workgroup whose wait timed out may have claimed it for
         * FAULT) */
        const uint32_t tag = RES_GR_OK | (path == MODE_FULL ? RES_GR_ALL : 0u);
        const unsigned long long gv = ((unsigned long long)tag << 32) | __float_as_uint(thr);
        if (atomicCAS(reinterpret_cast<unsigned long long*>(gr), 0ull, gv) != 0ull)
            atomicMax(&res[sd.res].path, (int32_t)MODE_FAULT);
    }
    WTP_RPROBE(6);
    if (first || sel) {
        /* zeros of where(|x| < thr, 0, x) = #(key < tk), tk = bits(thr) when thr > 0, else 1 (only
         * the zeros themselves); ka <= thr <= kb and the ranks are adjacent, so #(key < tk) =
         * below + before + #(staged < tk).  A NaN threshold prunes nothing: every
         * workgroup counts the zeros of its copy below. */
        unsigned long long zc = 0;
        if (!nan) {
            const uint32_t tk = thr > 0.0f ? __float_as_uint(thr) : 1u;
            if (path == MODE_FULL) {
                /* a selector counts AFTER publishing the granule: in place, the segment's data
                 * workgroups may already be overwriting sd.data.  The count is unchanged by them:
                 * where(|x| < thr, 0, x) turns every key < tk into +0 (key 0 < tk) and leaves every
                 * other key as it was (tests/test_gpu_resident.py::
                 * test_cfg2_in_place_full_scan_with_selectors) */
                zc = (unsigned long long)block_count_below<CT>([&](int64_t i) { return abs_key(sd.data[i]); }, sd.n, tk);
            } else {
                uint32_t c = 0;
                if (path == MODE_CAND)
                    for (int i = tid; i < m; i += CT) c += sel_keys[i] < tk;
                const unsigned long long sc = block_sum_u64<CT>(c);
                zc = (unsigned long long)sbelow +
                     (path == MODE_CAND ? (unsigned long long)before : 0ull) + sc;
            }
        }
        if (tid == 0) {
            thr_out[sd.res] = thr; /* per tensor */
            wtp_result& r = res[sd.res];
            r.numel = sd.numel;
            r.coeff_numel = sd.n;
            if (zc) atomicAdd((unsigned long long*)&r.zero_count, zc);
            r.thr64 = thr64;
            r.thr32_bits = __float_as_uint(thr);
            r.max_abs_bits = mk;
            r.eff_level = sd.eff_level;
            atomicMax(&r.path, path);
        }
    }
    if (sel) return;
    if (path == MODE_FULL && sd.out == sd.data) { /* in place: nobody writes before the segment's scans end */
        res_arrive(b0);
        if (!res_wait(b0, nwg, tmo)) {
            if (tid == 0) atomicMax(&res[sd.res].path, (int32_t)MODE_FAULT);
            return;
        }
    }
    WTP_RPROBE(6);
    /* ---- P3: out = where(|x| < thr, 0, x) from registers (a NaN threshold prunes nothing) */
    res_final<FULL>(v, thr, sd, res, base, len, al);
    WTP_RPROBE(7);
}

__global__ __launch_bounds__(RES_THREADS) void k_resident(SegTable t, SelHeader* __restrict__ head,
                                                          uint32_t* __restrict__ cand, wtp_result* __restrict__ res,
                                                          float* __restrict__ thr_out) {
    __shared__ __attribute__((aligned(16))) uint32_t raw[RES_HBINS > RES_SEL_MAX ? RES_HBINS : RES_SEL_MAX];
    __shared__ uint32_t lsub[RES_NSUB];
    __shared__ uint32_t wred[RES_THREADS / 64][8];
    __shared__ __attribute__((aligned(16))) uint32_t wstage[(RES_STG + 1) * RES_THREADS]; /* 66 KB: RES_STG slots + the discard slot per thread */
    const uint32_t qv = ldc<true>(&head->parity); /* a vector load: see parity_late */
    if (t.stamps && threadIdx.x == 0) atomicMin(t.stamps, wall_ticks()); /* measurement only */
    /* workgroups past the chunks are selectors, one per shared segment (t.sel_seg) */
    const bool sel = (int)blockIdx.x >= t.nblk;
    const int si = sel ? t.sel_seg[blockIdx.x - t.nblk] : find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    const int64_t base = sel ? 0 : (int64_t)(blockIdx.x - sd.blk_begin) * RES_CHUNK;
    const int len = sel ? 0 : (int)min((int64_t)RES_CHUNK, sd.n - base);
    if ((sd.flags & SEG_ALIGNED) && len == RES_CHUNK)
        res_body<true>(t, sd, head, qv, cand, res, thr_out, base, len, raw, lsub, wred, wstage, false);
    else
        res_body<false>(t, sd, head, qv, cand, res, thr_out, base, len, raw, lsub, wred, wstage, sel);
    if (t.stamps) { /* measurement only: the workgroup's end, once its stores have completed */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(t.stamps + 1, wall_ticks());
    }
}

/* The in-place segments whose k_mask_select took the full-scan select: the mask pass that
 * k_mask_select skipped for them, with the threshold it published (launched only for groups
 * that hold an in-place level-0 segment; every other block returns at once). */
__global__ __launch_bounds__(STREAM_THREADS) void k_mask_inplace(SegTable t, const wtp_result* __restrict__ res,
                                                                 const float* __restrict__ thr_in) {
    const int si = find_seg(t, blockIdx.x);
    const SegDesc& sd = t.s[si];
    if (!(sd.flags & SEG_MASK) || sd.data != sd.out || res[sd.res].path != MODE_FULL) return;
    const int64_t base = (int64_t)(blockIdx.x - sd.blk_begin) * CHUNK;
    const int len = (int)min((int64_t)CHUNK, sd.n - base);
    const float thr = thr_in[sd.res];
    if ((sd.flags & SEG_ALIGNED) && len == CHUNK) (void)mask_body<true>(sd, base, len, thr);
    else (void)mask_body<false>(sd, base, len, thr);
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
    if (k > 0) thr = select_body<STREAM_THREADS>(sd, st, cand, res, thr_out, stage, 4096, true, st->kl, st->kh, st->shift);
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

/* ---- 1-D flattened mode: pywt.wavedec / waverec (periodization) of the flattened tensor ----
 * k_dwt1_level: one analysis level of a line of N samples -> a (ceil(N/2)) and d (ceil(N/2)),
 * one thread per output pair, summed in PyWavelets' order (wt_ana_point). */
__global__ __launch_bounds__(DWT_THREADS) void k_dwt1_level(const float* __restrict__ x, int64_t N, Taps tp,
                                                            float* __restrict__ a, float* __restrict__ d) {
    const int64_t M = (N + 1) / 2;
    for (int64_t o = (int64_t)blockIdx.x * DWT_THREADS + threadIdx.x; o < M; o += (int64_t)gridDim.x * DWT_THREADS) {
        float sa, sd;
        wt_ana_point(o, N, tp.F, tp.f[0], tp.f[1], [&](int64_t k) { return x[k]; }, sa, sd);
        a[o] = sa;
        d[o] = sd;
    }
}

/* One synthesis level (pywt.waverec's loop body): a cropped to len(d) = N when it is one longer,
 * idwt(a, d) -> 2N outputs, of which the first outN are written.  a_thr: threshold a on load
 * (the packed cA of the top level); d is always a packed detail band (thresholded on load).
 * thr == nullptr: no threshold.  The last level crops to the tensor and counts its zeros. */
__global__ __launch_bounds__(DWT_THREADS) void k_idwt1_level(const float* __restrict__ a, int a_thr,
                                                             const float* __restrict__ d, int64_t N, Taps tp,
                                                             const float* __restrict__ thr, float* __restrict__ y,
                                                             int64_t outN, unsigned long long* zero_count) {
    const float t = thr ? *thr : 0.0f;
    const bool ta = thr && a_thr, td = thr != nullptr;
    unsigned long long z = 0;
    for (int64_t n = (int64_t)blockIdx.x * DWT_THREADS + threadIdx.x; n < outN; n += (int64_t)gridDim.x * DWT_THREADS) {
        const float v = wt_syn_point(n, N, tp.F, tp.f[2], tp.f[3],
                                     [&](int64_t k) { return ta ? thr_load(a[k], t) : a[k]; },
                                     [&](int64_t k) { return td ? thr_load(d[k], t) : d[k]; });
        y[n] = v;
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

/* ------------------------------------------------------ random pruning --- */
/* random_pruning (ResNet/random_pruning.py:49-56): out = in with k distinct flat positions
 * zeroed -- perm(0..k-1) of the keyed permutation in wt_perm.h; zero_count = zeros(in) + the
 * chosen positions that held a non-zero (count_nonzero counts NaN as non-zero).
 *   k_rand_copy  out = in (unless in place), zeros(in) per block, the record's numel
 *   k_rand_zero  one thread per chosen position; block sums of the non-zeros it removed */
__device__ __forceinline__ int rand_seg(const int32_t* begin, int nseg, int b) {
    int s = 0;
    for (int i = 1; i < nseg; ++i) s += b >= begin[i];
    return s;
}

__global__ __launch_bounds__(STREAM_THREADS) void k_rand_copy(RandTable t, wtp_result* __restrict__ res) {
    const int si = rand_seg(t.copy_begin, t.nseg, blockIdx.x);
    const RandSeg& sg = t.s[si];
    const int64_t base = (int64_t)(blockIdx.x - t.copy_begin[si]) * CHUNK;
    const int64_t end = min(sg.numel, base + CHUNK);
    uint32_t z = 0;
    for (int64_t i = base + threadIdx.x; i < end; i += STREAM_THREADS) {
        const float v = sg.in[i];
        z += v == 0.0f;
        if (sg.out != sg.in) sg.out[i] = v;
    }
    const unsigned long long tot = block_sum_u64<STREAM_THREADS>(z);
    if (threadIdx.x == 0) {
        if (tot) atomicAdd((unsigned long long*)&res[sg.res].zero_count, tot);
        if (base == 0) res[sg.res].numel = sg.numel;
    }
}

__global__ __launch_bounds__(STREAM_THREADS) void k_rand_zero(RandTable t, wtp_result* __restrict__ res) {
    const int si = rand_seg(t.zero_begin, t.nseg, blockIdx.x);
    const RandSeg& sg = t.s[si];
    const int64_t j = (int64_t)(blockIdx.x - t.zero_begin[si]) * STREAM_THREADS + threadIdx.x;
    uint32_t hit = 0;
    if (j < sg.k) {
        const int64_t idx = (int64_t)wt_perm((uint64_t)j, (uint64_t)sg.numel, sg.h, sg.key);
        hit = sg.in[idx] != 0.0f; /* distinct positions: in place, nobody else has written idx */
        sg.out[idx] = 0.0f;
    }
    const unsigned long long tot = block_sum_u64<STREAM_THREADS>(hit);
    if (threadIdx.x == 0 && tot) atomicAdd((unsigned long long*)&res[sg.res].zero_count, tot);
}

/* calculate_sparsity (testing_suite/eval_model.py:7-20): #(|x| < thr) of one tensor */
__global__ __launch_bounds__(STREAM_THREADS) void k_count_small(const float* __restrict__ x, int64_t n, float thr,
                                                                unsigned long long* __restrict__ count) {
    uint32_t c = 0;
    for (int64_t i = (int64_t)blockIdx.x * STREAM_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * STREAM_THREADS)
        c += fabsf(x[i]) < thr;
    const unsigned long long tot = block_sum_u64<STREAM_THREADS>(c);
    if (threadIdx.x == 0 && tot) atomicAdd(count, tot);
}

/* ---------------------------------------------------------------- launchers --- */
static inline unsigned grid_for(int64_t total) {
    int64_t g = (total + DWT_THREADS - 1) / DWT_THREADS;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (unsigned)g;
}

static int collect_blocks(const SegTable& t) { return t.nblk * (CHUNK / (COLLECT_IT * COLLECT_THREADS * 4)); }
static bool window_inline(const SegTable& t) { return collect_blocks(t) <= WINDOW_INLINE_MAX_BLOCKS; }
void launch_window(const SegTable& t, SelHeader* head, hipStream_t s, const wtp_result* res) {
    if (!window_inline(t)) hipLaunchKernelGGL(k_window, dim3(t.nseg), dim3(WIN_THREADS), 0, s, t, head, res);
}
void launch_fused_retry(const SegTable& t, SelHeader* head, uint32_t* cand, wtp_result* res, float* thr_out,
                        hipStream_t s) {
    hipLaunchKernelGGL(k_window, dim3(t.nseg), dim3(WIN_THREADS), 0, s, t, head, (const wtp_result*)res);
    const int total = collect_blocks(t);
    hipLaunchKernelGGL((k_collect_retry<COLLECT_THREADS, COLLECT_IT>), dim3(total < 512 ? total : 512), dim3(COLLECT_THREADS), 0,
                       s, t, head, cand, res);
    launch_mask_select(t, head, cand, res, thr_out, s);
}
void launch_collect(const SegTable& t, SelHeader* head, uint32_t* cand, wtp_result* res, hipStream_t s) {
    if (window_inline(t))
        hipLaunchKernelGGL((k_collect_t<COLLECT_THREADS, COLLECT_IT, true>), dim3(collect_blocks(t)),
                           dim3(COLLECT_THREADS), 0, s, t, head, cand, res);
    else
        hipLaunchKernelGGL((k_collect_t<COLLECT_THREADS, COLLECT_IT, false>), dim3(collect_blocks(t)),
                           dim3(COLLECT_THREADS), 0, s, t, head, cand, res);
}
void launch_fwin(const FwinTable& t, SelHeader* head, hipStream_t s) {
    const dim3 g(t.nseg * FWIN_NP), b(FWIN_THREADS);
    switch (t.F) {
    case 2: hipLaunchKernelGGL(k_fwin<2>, g, b, 0, s, t, head); break;
    case 4: hipLaunchKernelGGL(k_fwin<4>, g, b, 0, s, t, head); break;
    case 6: hipLaunchKernelGGL(k_fwin<6>, g, b, 0, s, t, head); break;
    case 8: hipLaunchKernelGGL(k_fwin<8>, g, b, 0, s, t, head); break;
    case 10: hipLaunchKernelGGL(k_fwin<10>, g, b, 0, s, t, head); break;
    case 12: hipLaunchKernelGGL(k_fwin<12>, g, b, 0, s, t, head); break;
    case 16: hipLaunchKernelGGL(k_fwin<16>, g, b, 0, s, t, head); break;
    case 18: hipLaunchKernelGGL(k_fwin<18>, g, b, 0, s, t, head); break;
    default: break; /* the host fuses only k_fwd_int's filters */
    }
}
void launch_fslot_collect(const SegTable& t, SelHeader* head, uint32_t* cand, wtp_result* res, hipStream_t s) {
    hipLaunchKernelGGL(k_fslot_collect, dim3(t.nblk), dim3(FSC_THREADS), 0, s, t, head, cand, res);
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
    bool masked = false;
    for (int i = 0; i < t.nseg; ++i) masked = masked || (t.s[i].flags & SEG_MASK);
    if (masked) {
        hipLaunchKernelGGL(k_mask_select, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, head, cand, res, thr_out);
        return;
    }
    /* no segment to mask (the DWT segments: the inverse thresholds on load): only the select of
     * each segment's first block runs, so the grid is one block per segment */
    SegTable d = t;
    for (int i = 0; i < t.nseg; ++i) d.s[i].blk_begin = d.blk_begin[i] = i;
    d.nblk = t.nseg;
    hipLaunchKernelGGL(k_mask_select, dim3(d.nblk), dim3(STREAM_THREADS), 0, s, d, head, cand, res, thr_out);
}
void launch_mask_inplace(const SegTable& t, const wtp_result* res, const float* thr, hipStream_t s) {
    hipLaunchKernelGGL(k_mask_inplace, dim3(t.nblk), dim3(STREAM_THREADS), 0, s, t, res, thr);
}
int resident_capacity() {
    static std::atomic<int> cache[16];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
    if (dev < 16) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c) return c > 0 ? c : 0;
    }
    int per = 0, cus = 0;
    int cap = -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_resident, RES_THREADS, 0) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && per >= 1 && cus > 0)
        cap = cus; /* one workgroup per CU: the form the inter-workgroup hand-off is specified for */
    (void)hipGetLastError();
    if (dev < 16) cache[dev].store(cap, std::memory_order_relaxed);
    return cap > 0 ? cap : 0;
}
static std::atomic<uint32_t> g_res_timeout_us{RES_TIMEOUT_DEFAULT_US};
uint32_t set_resident_timeout_us(uint32_t us) { return g_res_timeout_us.exchange(std::min(us, RES_TIMEOUT_MAX_US)); }
static std::atomic<unsigned long long*> g_stamps{nullptr};
void set_kernel_stamps(unsigned long long* dev) { g_stamps.store(dev); }
uint32_t resident_timeout_us() { return g_res_timeout_us.load(std::memory_order_relaxed); }
unsigned long long* kernel_stamps() { return g_stamps.load(std::memory_order_relaxed); }
void launch_resident(const SegTable& t0, SelHeader* head, uint32_t* cand, wtp_result* res, float* thr_out,
                     hipStream_t s) {
    SegTable t = t0;
    t.res_timeout = g_res_timeout_us.load(std::memory_order_relaxed) * 100u; /* 100 MHz wall clock */
    t.stamps = g_stamps.load(std::memory_order_relaxed);
    /* one selector workgroup per shared segment when they fit beside the chunks (one per CU):
     * the segment's select runs on a CU that holds no chunk */
    int nshared = 0;
    for (int i = 0; i < t.nseg; ++i) nshared += t.s[i].n > RES_CHUNK;
    t.nsel = 0;
    if (nshared > 0 && t.nblk + nshared <= RES_MAX_WG && t.nblk + nshared <= resident_capacity())
        for (int i = 0; i < t.nseg; ++i)
            if (t.s[i].n > RES_CHUNK) t.sel_seg[t.nsel++] = i;
    hipLaunchKernelGGL(k_resident, dim3(t.nblk + t.nsel), dim3(RES_THREADS), 0, s, t, head, cand, res, thr_out);
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
void launch_dwt1_level(const float* x, int64_t N, const Taps& tp, float* a, float* d, hipStream_t s) {
    hipLaunchKernelGGL(k_dwt1_level, dim3(grid_for((N + 1) / 2)), dim3(DWT_THREADS), 0, s, x, N, tp, a, d);
}
void launch_idwt1_level(const float* a, int a_thr, const float* d, int64_t N, const Taps& tp, const float* thr,
                        float* y, int64_t outN, unsigned long long* zc, hipStream_t s) {
    hipLaunchKernelGGL(k_idwt1_level, dim3(grid_for(outN)), dim3(DWT_THREADS), 0, s, a, a_thr, d, N, tp, thr, y, outN,
                       zc);
}
void launch_copy_threshold(const float* P, float* out, int64_t n, const float* thr, unsigned long long* zc,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_copy_threshold, dim3(grid_for(n)), dim3(DWT_THREADS), 0, s, P, out, n, thr, zc);
}
void launch_random_prune(const RandTable& t, wtp_result* res, hipStream_t s) {
    if (t.copy_begin[t.nseg] > 0)
        hipLaunchKernelGGL(k_rand_copy, dim3(t.copy_begin[t.nseg]), dim3(STREAM_THREADS), 0, s, t, res);
    if (t.zero_begin[t.nseg] > 0)
        hipLaunchKernelGGL(k_rand_zero, dim3(t.zero_begin[t.nseg]), dim3(STREAM_THREADS), 0, s, t, res);
}
void launch_count_small(const float* x, int64_t n, float thr, unsigned long long* count, hipStream_t s) {
    int64_t g = (n + STREAM_THREADS * 16 - 1) / (STREAM_THREADS * 16);
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(k_count_small, dim3((unsigned)g), dim3(STREAM_THREADS), 0, s, x, n, thr, count);
}
void launch_synth(float* out, int64_t n, uint64_t seed, uint32_t tid, int e, hipStream_t s) {
    hipLaunchKernelGGL(k_synth, dim3(grid_for(n)), dim3(DWT_THREADS), 0, s, out, n, seed, tid, e);
}

}  // namespace wtp
