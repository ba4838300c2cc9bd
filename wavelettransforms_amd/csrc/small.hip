/*
 * small.hip -- the small-population path in ONE launch (k_small): pywt.wavedec2 of every level,
 * the exact np.percentile of |coeffs| and pywt.waverec2 of the thresholded coefficients
 * (ResNet/dwt_pruning.py:67-88) for calls whose tensors are a few hundred thousand coefficients
 * each -- the launch-latency regime of cfg3 (the MNIST MLP), where the per-level launches of
 * filterbank.hip spend more time filling and draining the chip than working.
 *
 * One workgroup per tile (one per CU: 144 KB of LDS), tiles of one tensor form its segment:
 *   F  the tile loads its level-0 window once and runs every analysis level in LDS
 *      (small_geom.h: the window of level k-1 holds every sample the tile's level-k window
 *      reads), writing the coefficients it owns to the packed array P (write-through sc1
 *      stores) and keeping their keys |c| in LDS;
 *   S  an exact three-digit radix select (10 + 10 + 11 bits of the key) over the segment: per
 *      digit the workgroups add their LDS histograms to the segment's (memory-side atomics),
 *      meet at a segment barrier and read the summed histogram (sc1 loads); the last digit's
 *      pass also reduces the smallest key above the rank's 21-bit group, so both order
 *      statistics of np.percentile come out of the same three passes (NumPy 1.x _lerp);
 *   I  the tile synthesises its owned output block from the coefficient windows of every level
 *      (thresholded as they are loaded: the np.where of :31), all in LDS, and counts its zeros.
 * Every output sample is summed in PyWavelets' exact order: the tap tables built per level list
 * each output's (tap, source) pairs in wt_dwt_core.h's order, so results are bit-identical to
 * the per-level kernels and the oracle.  A barrier whose wait times out poisons the segment's
 * counter (res_wait in kernels.hip semantics): the whole segment stores nothing to `out` and
 * records WTP_PATH_FAULT, and the caller re-runs it in the multi-launch form.
 */
#include "wtp_internal.h"
#include "small_geom.h"

#include <atomic>

static_assert(SM_MAX_L == wtp::SM_LMAX, "level bound");

#pragma clang fp contract(off)

namespace wtp {

/* phase stamps for tools/probe_small.py (a -DWTP_SM_PROBE build only): stamps[2 + 32 b + i] */
#ifdef WTP_SM_PROBE
#define SM_PROBE(i) \
    do { \
        if (t.stamps && threadIdx.x == 0) t.stamps[2 + 32 * blockIdx.x + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define SM_PROBE(i)
#endif

constexpr int SM_THREADS = 1024;
static_assert(SM_THREADS >= 256 && SM_THREADS <= 1024 && (SM_THREADS & (SM_THREADS - 1)) == 0, "k_small block");
constexpr int SM_NW = SM_THREADS / 64;
constexpr int SM_PF = 8; /* inverse-window words per thread prefetched in registers */
/* after the first barrier every workgroup publishes the keys of the rank's 12-bit bin in a slot
 * of its own: [0] count (bit 31: more than fit), [1] padding zeros it counts, [2] its smallest key
 * above the bin, then up to SM_SLOT_KEYS keys */
constexpr int SM_SLOT_KEYS = SM_SLOT_WORDS - 3;
constexpr int SM_GATHER = SM_SEG_WG_MAX * SM_SLOT_WORDS; /* LDS words of the gathered slots (arena tail) */
static_assert(SM_GATHER == 8192, "small_geom.h's sm_inv_words reserves 8192 words for the gathered slots");

/* per-segment selection state in the parity region (zero at the start of the launch) */
struct alignas(128) SmallState {
    uint32_t bar[4][32];   /* segment barrier counters, one 128-byte line each */
    uint32_t maxkey;       /* atomicMax of every key                           */
    uint32_t notmin;       /* fallback: atomicMax of ~key over the keys above the rank's group */
    uint32_t pad[30];
    uint32_t h1[4096];     /* key bits 30..19                                  */
    uint32_t h2[2048];     /* fallback: bits 18..8 of the keys in the rank's h1 bin */
    uint32_t h3[256];      /* fallback: bits 7..0 of the keys in the rank's 23-bit group */
};
static_assert(SM_MAX_SEG * sizeof(SmallState) <= SEG_PER_LAUNCH * sizeof(SelState), "small state fits the region");

__device__ __forceinline__ uint32_t sm_abs_key(float x) { return __float_as_uint(x) & 0x7FFFFFFFu; }
template <class T>
__device__ __forceinline__ void sm_stc(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T sm_ldc(const T* p) {
    return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t sm_ticks() { return __builtin_amdgcn_s_memrealtime(); }

/* a segment barrier: every wave drains its stores, lane 0 arrives with a returning add (its
 * own arrival is then performed, and the last arriver needs no poll); sm_wait polls (sc1) from
 * that value, with the poison-on-timeout rule of k_resident's res_wait (all-or-nothing over
 * the segment).  The arrival value lives in lane 0 of wave 0 only. */
__device__ __forceinline__ uint32_t sm_arrive(uint32_t* ctr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    return threadIdx.x == 0 ? atomicAdd(ctr, 1u) + 1u : 0u;
}
__device__ __forceinline__ bool sm_wait(uint32_t* ctr, uint32_t v0, uint32_t want, uint64_t timeout, int* s_ok) {
    if (threadIdx.x == 0) {
        const uint64_t t0 = sm_ticks();
        int ok = 0;
        uint32_t v = v0;
        while (true) {
            if (v & RES_POISON) break;
            if (v >= want) { ok = 1; break; }
            if (sm_ticks() - t0 >= timeout) { /* >=: a zero bound poisons at the first incomplete look */
                const uint32_t w = atomicCAS(ctr, v, v | RES_POISON);
                if (w == v) break;
                v = w; /* it moved: look again */
                continue;
            }
            __builtin_amdgcn_s_sleep(1);
            v = sm_ldc(ctr);
        }
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

/* two lanes of packed FP32 (v_pk_mul_f32 / v_pk_add_f32): the same IEEE operations per lane */
typedef float sf2 __attribute__((ext_vector_type(2)));

/* e / n and e % n for e < 2^24 without an integer division (n uniform, inv = 1.0f / n) */
__device__ __forceinline__ void sm_divmod(int e, int n, float inv, int* q, int* r) {
    int d = (int)((float)e * inv);
    int m = e - d * n;
    if (m < 0) { --d; m += n; }
    if (m >= n) { ++d; m -= n; }
    *q = d;
    *r = m;
}
__device__ __forceinline__ int sm_wrap(int a, int N) { return a < N ? a : a - N; } /* a < 2N */


__device__ __forceinline__ int sm_r4(int x) { return (x + 3) & ~3; } /* LDS regions start 16-byte aligned */

/* Cross-lane scan on DPP (row_shr inside rows of 16 lanes, row_bcast:15/31 across rows), as in
 * kernels.hip: a few VALU cycles per step where a shuffle pays an LDS round trip.  Whole wave. */
template <int CTRL, int ROWM = 0xf, int BANKM = 0xf>
__device__ __forceinline__ uint32_t sm_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWM, BANKM, false);
}
__device__ __forceinline__ uint32_t sm_wave_scan(uint32_t v) { /* inclusive */
    v += sm_dpp<0x111>(v);
    v += sm_dpp<0x112>(v);
    v += sm_dpp<0x114>(v);
    v += sm_dpp<0x118>(v);
    v += sm_dpp<0x142, 0xa>(v);
    v += sm_dpp<0x143, 0xc>(v);
    return v;
}

/* wave-wide min / max / or / sum on DPP (lanes without a source keep their own value), the
 * result read from lane 63; every lane of the wave must be active */
template <int CTRL, int ROWM = 0xf, int BANKM = 0xf>
__device__ __forceinline__ uint32_t sm_dppk(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROWM, BANKM, false);
}
template <class Op>
__device__ __forceinline__ uint32_t sm_wave_red(uint32_t v, const Op& op) {
    v = op(v, sm_dppk<0x111>(v));
    v = op(v, sm_dppk<0x112>(v));
    v = op(v, sm_dppk<0x114>(v));
    v = op(v, sm_dppk<0x118>(v));
    v = op(v, sm_dppk<0x142, 0xa>(v));
    v = op(v, sm_dppk<0x143, 0xc>(v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t sm_wave_min(uint32_t v) { return sm_wave_red(v, [](uint32_t a, uint32_t b) { return a < b ? a : b; }); }
__device__ __forceinline__ uint32_t sm_wave_max(uint32_t v) { return sm_wave_red(v, [](uint32_t a, uint32_t b) { return a > b ? a : b; }); }
__device__ __forceinline__ uint32_t sm_wave_or(uint32_t v) { return sm_wave_red(v, [](uint32_t a, uint32_t b) { return a | b; }); }
__device__ __forceinline__ uint32_t sm_wave_sum(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)sm_wave_scan(v), 63); }

/* block-wide exclusive scan of one u32 per thread (DPP inside the waves, one LDS exchange
 * across them); *tot the block total */
__device__ __forceinline__ uint32_t sm_scan(uint32_t v, uint32_t* wtot, uint32_t* tot) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t incl = sm_wave_scan(v);
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < SM_NW; ++w) {
        const uint32_t x = wtot[w];
        before += w < wv ? x : 0u;
        all += x;
    }
    __syncthreads();
    *tot = all;
    return before + incl - v;
}

/* Taps of one output, summed in PyWavelets' order (wt_dwt_core.h).  The interior form -- taps
 * j = 0, 1, ... ascending at consecutive descending window slots -- is recognised by its first
 * slot (the fast path: samples read back to back, taps from LDS by constant index); anything else
 * (the periodic wrap at the image edges, the split order of wt_ana_point / wt_syn_pass) walks
 * the taps one by one: tap q is j(q) = q < c1 ? c1 - 1 - q : q. */

__device__ __forceinline__ int sm_mod1(int a, int m) { /* a in [-m, 2m) */
    a += a < 0 ? m : 0;
    return a >= m ? a - m : a;
}

/* analysis output m of window W (line N) reading window Wp (line Np): when the samples of its
 * taps j sit at consecutive window slots s0 - j (always for an even line: the periodic wrap keeps
 * them contiguous; for an odd line only away from the repeated end), (s0 << 5) | c1, where c1 is
 * the count of taps wt_ana_point adds first in descending j (0 in the interior); else -1 */
__device__ __forceinline__ int sm_ana_fast(SmIvl W, int N, SmIvl Wp, int Np, int F, int m) {
    const int i = F / 2 + 2 * sm_wrap(W.s + m, N);
    const int s0 = sm_mod1(i - Wp.s, Np);
    const int c1 = min(max(i - Np + 1, 0), F);
    return (s0 >= F - 1 && ((Np & 1) == 0 || (i < Np && i - F + 1 >= 0))) ? (s0 << 5) | c1 : -1;
}
/* the general form: tap q's window slot and tap index */
struct SmAna {
    int i, c1, Ne;
};
__device__ __forceinline__ SmAna sm_ana_at(SmIvl W, int N, int Np, int F, int m) {
    SmAna a;
    a.i = F / 2 + 2 * sm_wrap(W.s + m, N);
    a.c1 = min(max(a.i - Np + 1, 0), F);
    a.Ne = Np + (Np & 1);
    return a;
}
__device__ __forceinline__ int sm_ana_tap(const SmAna& a, SmIvl Wp, int Np, int q, int* j) {
    const int jj = q < a.c1 ? a.c1 - 1 - q : q;
    int r = a.i - jj; /* in [-F, 2 Np): one period either way */
    r += r < 0 ? a.Ne : 0;
    r -= r >= a.Ne ? a.Ne : 0;
    const int src = r < Np ? r : Np - 1;
    *j = jj;
    return sm_mod1(src - Wp.s, Np);
}

/* synthesis site of output n of 2N (wt_syn_locate in 32 bits) */
struct SmSite {
    int i, par, special;
};
__device__ __forceinline__ SmSite sm_site(int n, int N, int F) {
    const int H = F / 2, start = F / 4;
    SmSite s;
    s.special = 0;
    if ((H & 1) == 0) {
        if (n == 2 * N - 1) { s.i = start - 1; s.par = 0; s.special = 1; }
        else if (n == 0) { s.i = start - 1; s.par = 1; s.special = 1; }
        else if (n & 1) { s.i = start + (n - 1) / 2; s.par = 0; }
        else { s.i = start + (n - 2) / 2; s.par = 1; }
    } else {
        s.i = start + n / 2;
        s.par = n & 1;
    }
    return s;
}
/* synthesis output m of window O (line No) reading window S (line N): the wrap is purely periodic,
 * so the sources of taps j sit at slots s0 - j whenever the window holds them:
 * (s0 << 6) | (parity << 5) | c1 (c1: the taps wt_syn_pass adds first in descending j), else -1 */
__device__ __forceinline__ int sm_syn_fast(SmIvl O, int No, SmIvl S, int N, int F, int m) {
    const int H = F / 2;
    const SmSite s = sm_site(sm_wrap(O.s + m, No), N, F);
    const int s0 = sm_mod1(s.i - S.s, N);
    const int c1 = s.special ? min(max(s.i + 1, 0), H) : (s.i < N ? 0 : min(max(s.i - N + 1, 0), H));
    return s0 >= H - 1 ? (s0 << 6) | (s.par << 5) | c1 : -1;
}

/* sum over T taps in PyWavelets' order: the c1 taps j = c1-1 .. 0 first, then j = c1 .. T-1;
 * v(j) the sample of tap j, c(j) its coefficient (compile-time j: registers, no indexing) */
template <int T, class V, class C, class A>
__device__ __forceinline__ void sm_order(int c1, bool plain, const V& v, const C& c, const A& acc) {
    if (plain) {
#pragma unroll
        for (int j = 0; j < T; ++j) acc(c(j), v(j));
    } else {
#pragma unroll
        for (int j = T - 1; j >= 0; --j)
            if (j < c1) acc(c(j), v(j));
#pragma unroll
        for (int j = 0; j < T; ++j)
            if (j >= c1) acc(c(j), v(j));
    }
}
struct SmSyn {
    int i, par, c1;
};
__device__ __forceinline__ SmSyn sm_syn_at(SmIvl O, int No, int N, int F, int m) {
    const int H = F / 2;
    const SmSite s = sm_site(sm_wrap(O.s + m, No), N, F);
    SmSyn y;
    y.i = s.i;
    y.par = s.par;
    y.c1 = s.special ? min(max(s.i + 1, 0), H) : (s.i < N ? 0 : min(max(s.i - N + 1, 0), H));
    return y;
}
__device__ __forceinline__ int sm_syn_tap(const SmSyn& y, SmIvl S, int N, int q, int* ci) {
    const int j = q < y.c1 ? y.c1 - 1 - q : q;
    *ci = 2 * j + y.par;
    return sm_mod1(sm_mod1(y.i - j, N) - S.s, N);
}

/* FT: the filter length as a compile-time constant (0: any, from the taps) -- the interior
 * outputs then read their FT samples back to back and take the taps from scalar registers */
template <int FT>
__global__ __launch_bounds__(SM_THREADS) void k_small(SmallTable t, SelHeader* __restrict__ head,
                                                      wtp_result* __restrict__ res) {
    __shared__ __attribute__((aligned(16))) float arena[SM_ARENA];
    __shared__ uint32_t hist[4096];
    __shared__ SmAxis axr, axc;
    __shared__ uint32_t wtot[SM_NW], wred[SM_NW];
    __shared__ int s_ok, s_dig[2];
    __shared__ uint32_t s_bef[2];
    __shared__ float staps[4][SM_F_MAX]; /* dec_lo, dec_hi, rec_lo, rec_hi */
    /* the inverse windows' per-level constants, for the window-word -> packed-offset map (win_src):
     * built once from the axes and the segment geometry, read from LDS at every word instead of
     * the kernel argument's per-level arrays indexed by a per-lane level */
    struct WinLvl { int base, ns, scl, srs, scs, R, C, offR, offC; float rns, rsc; int pad; };
    __shared__ WinLvl s_wl[SM_LMAX + 2];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t q = head->parity;
    if (t.stamps && tid == 0) atomicMin(t.stamps, sm_ticks()); /* measurement only */
    {   /* clear this workgroup's slice of the idle region (the previous launch's) */
        uint4* idle = reinterpret_cast<uint4*>(sel_region(head, q ^ 1u));
        constexpr int NV4 = (int)(SEL_REGION / 16);
        const int per = (NV4 + (int)gridDim.x - 1) / (int)gridDim.x;
        for (int i = tid; i < per; i += SM_THREADS) {
            const int j = (int)blockIdx.x * per + i;
            if (j < NV4) idle[j] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    SM_PROBE(6);
    int si = 0;
#pragma unroll
    for (int i = 1; i < SM_MAX_SEG; ++i) si += (int)blockIdx.x >= t.wg_begin[i];
    const SmallSeg& g = t.s[si];
    SmallState* st = reinterpret_cast<SmallState*>(sel_region(head, q)) + si;
    const int F = FT ? FT : t.tp.F;
    const int L = g.L;
    const int lt = (int)blockIdx.x - g.wg_begin;
    const int tpi = g.tilesR * g.tilesC;
    const int b = lt / tpi, tr = (lt - b * tpi) / g.tilesC, tc = (lt - b * tpi) - tr * g.tilesC;
    const uint64_t tmo = t.timeout;
    /* the tile's windows (computed by the host, small_geom.h) and the taps: one word per lane */
    {
        const int lw = 2 * (L + 1);
        const uint32_t* rw = t.win + g.win_off + tr * lw;
        const uint32_t* cw = t.win + g.win_off + g.tilesR * lw + tc * lw;
        if (tid < 2 * lw) {
            const bool cols = tid >= lw;
            const int x = cols ? tid - lw : tid, k = x >> 1;
            const uint32_t w = cols ? cw[x] : rw[x];
            SmAxis& ax = cols ? axc : axr;
            const int lo = (int)(w & 0xFFFFu), hi = (int)(w >> 16);
            if (x & 1) ax.sv[k] = SmIvl{lo, hi};
            else ax.fw[k] = SmIvl{lo, hi};
        } else if (tid >= 64 && tid < 64 + 2 * (L + 1)) { /* the owned ranges: shifts of the tile index */
            const bool cols = tid >= 64 + L + 1;
            const int k = tid - 64 - (cols ? L + 1 : 0);
            SmAxis& ax = cols ? axc : axr;
            sm_own(cols ? tc : tr, cols ? g.TC : g.TR, L, k, cols ? g.C : g.R, &ax.olo[k], &ax.ohi[k]);
        } else if (tid >= 128 && tid < 128 + 4 * SM_F_MAX) {
            const int i = (tid - 128) / SM_F_MAX, j = (tid - 128) - i * SM_F_MAX;
            staps[i][j] = t.tp.f[i][j];
        } else if (tid == SM_THREADS - 1 && lt == 0) { /* memory-side words: later adds come from other workgroups */
            sm_stc(reinterpret_cast<unsigned long long*>(&res[g.res].zero_count), 0ull);
            sm_stc(&res[g.res].path, 0);
        }
    }
    for (int i = tid; i < 4096; i += SM_THREADS) hist[i] = 0u;
    __syncthreads();
    SM_PROBE(0);

    if (tid == 0) {
        int base = 0;
        for (int k = 1; k <= L + 1; ++k) {
            WinLvl w{};
            w.base = base;
            if (k <= L) {
                const SmIvl sr = axr.sv[k], sc = axc.sv[k];
                w.ns = sr.len * sc.len;
                w.scl = sc.len;
                w.srs = sr.s;
                w.scs = sc.s;
                w.R = g.R[k];
                w.C = g.C[k];
                w.offR = g.offR[k];
                w.offC = g.offC[k];
                w.rns = 1.0f / (float)w.ns;
                w.rsc = 1.0f / (float)sc.len;
                base += (3 + (k == L)) * w.ns;
            }
            s_wl[k] = w;
        }
    }
    /* ---------------- F: every analysis level of the tile in LDS ---------------- */
    const int H0 = g.R[0], W0 = g.C[0];
    float* P = g.P + (int64_t)b * g.PR * g.PC;
    int fx = 0, flh = 0;
    for (int k = 0; k <= L; ++k) fx = max(fx, axr.fw[k].len * axc.fw[k].len);
    for (int k = 1; k <= L; ++k) flh = max(flh, 2 * axr.fw[k].len * axc.fw[k - 1].len);
    int nkeys = 0;
    for (int k = 1; k <= L; ++k)
        nkeys += (3 + (k == L)) * (axr.ohi[k] - axr.olo[k]) * (axc.ohi[k] - axc.olo[k]);
    /* arena: [owned keys | approximation window | column-pass rows]; the inverse reuses what
     * follows the keys */
    uint32_t* K = reinterpret_cast<uint32_t*>(arena);
    float* X = arena + sm_r4(nkeys);
    float2* LH = reinterpret_cast<float2*>(X + sm_r4(fx));
    uint32_t mx = 0;
    {   /* the level-0 window, all of a thread's loads in flight before the first LDS write */
        const SmIvl wr = axr.fw[0], wc = axc.fw[0];
        const float* img = g.in + (int64_t)b * H0 * W0;
        const int n = wr.len * wc.len;
        const float inv = 1.0f / (float)wc.len;
        auto src = [&](int e) {
            int mr, mc;
            sm_divmod(e, wc.len, inv, &mr, &mc);
            return img + (int64_t)sm_wrap(wr.s + mr, H0) * W0 + sm_wrap(wc.s + mc, W0);
        };
        for (int e0 = 0; e0 < n; e0 += SM_PF * SM_THREADS) {
            float v[SM_PF];
#pragma unroll
            for (int u = 0; u < SM_PF; ++u) {
                const int e = e0 + tid + u * SM_THREADS;
                v[u] = e < n ? *src(e) : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < SM_PF; ++u) {
                const int e = e0 + tid + u * SM_THREADS;
                if (e < n) X[e] = v[u];
            }
        }
    }
    __syncthreads();
    SM_PROBE(1);
    int kbase = 0;
    float* Xc = X;
    for (int k = 1; k <= L; ++k) {
        const SmIvl wr = axr.fw[k], wc = axc.fw[k], pr = axr.fw[k - 1], pc = axc.fw[k - 1];
        const int Nr = g.R[k], Nc = g.C[k], Npr = g.R[k - 1], Npc = g.C[k - 1];
        /* axis -2: (L, H) of every window column at the level-k window rows */
        {
            const int n = wr.len * pc.len;
            const float inv = 1.0f / (float)pc.len;
            for (int e = tid; e < n; e += SM_THREADS) {
                int mr, mc;
                sm_divmod(e, pc.len, inv, &mr, &mc);
                float a = 0.0f, d = 0.0f;
                const int fb = sm_ana_fast(wr, Nr, pr, Npr, F, mr);
                if (FT > 0 && __all(fb >= 0)) {
                    const int s0 = fb >> 5, c1 = fb & 31;
                    float v[FT > 0 ? FT : 1];
#pragma unroll
                    for (int qq = 0; qq < FT; ++qq) v[qq] = Xc[(s0 - qq) * pc.len + mc];
                    sf2 ad2 = {0.0f, 0.0f}; /* (a, d) packed */
                    sm_order<FT>(c1, __all(c1 == 0), [&](int j) { return v[j]; }, [&](int j) { return j; },
                                 [&](int j, float x) { ad2 = ad2 + sf2{staps[0][j], staps[1][j]} * sf2{x, x}; });
                    a = ad2.x;
                    d = ad2.y;
                } else {
                    const SmAna an = sm_ana_at(wr, Nr, Npr, F, mr);
                    for (int qq = 0; qq < F; ++qq) {
                        int j;
                        const int sl = sm_ana_tap(an, pr, Npr, qq, &j);
                        const float v = Xc[sl * pc.len + mc];
                        a = a + staps[0][j] * v;
                        d = d + staps[1][j] * v;
                    }
                }
                LH[e] = make_float2(a, d);
            }
            __syncthreads();
            if (k <= 3) SM_PROBE(14 + 2 * k); /* 16, 18, 20: level k's axis -2 pass */
        }
        /* axis -1: aa, ad from the L rows, da, dd from the H rows; aa is the next level's input */
        {
            const int n = wr.len * wc.len;
            const float inv = 1.0f / (float)wc.len;
            const int ohr = axr.ohi[k] - axr.olo[k], ohc = axc.ohi[k] - axc.olo[k];
            const int plane = ohr * ohc;
            const bool last = k == L;
            for (int e = tid; e < n; e += SM_THREADS) {
                int mr, mc;
                sm_divmod(e, wc.len, inv, &mr, &mc);
                const float2* row = LH + mr * pc.len;
                float aa = 0.0f, ad = 0.0f, da = 0.0f, dd = 0.0f;
                const int fb = sm_ana_fast(wc, Nc, pc, Npc, F, mc);
                if (FT > 0 && __all(fb >= 0)) {
                    const int s0 = fb >> 5, c1 = fb & 31;
                    float2 v[FT > 0 ? FT : 1];
#pragma unroll
                    for (int qq = 0; qq < FT; ++qq) v[qq] = row[s0 - qq];
                    sf2 lo2 = {0.0f, 0.0f}, hi2 = {0.0f, 0.0f}; /* (aa, da), (ad, dd) packed */
                    sm_order<FT>(c1, __all(c1 == 0), [&](int j) { return v[j]; }, [&](int j) { return j; },
                                 [&](int j, float2 x) {
                                     const float c0 = staps[0][j], c1v = staps[1][j];
                                     const sf2 xv = {x.x, x.y};
                                     lo2 = lo2 + sf2{c0, c0} * xv;
                                     hi2 = hi2 + sf2{c1v, c1v} * xv;
                                 });
                    aa = lo2.x;
                    da = lo2.y;
                    ad = hi2.x;
                    dd = hi2.y;
                } else {
                    const SmAna an = sm_ana_at(wc, Nc, Npc, F, mc);
                    for (int qq = 0; qq < F; ++qq) {
                        int j;
                        const int sl = sm_ana_tap(an, pc, Npc, qq, &j);
                        const float2 v = row[sl];
                        const float c0 = staps[0][j], c1 = staps[1][j];
                        aa = aa + c0 * v.x;
                        ad = ad + c1 * v.x;
                        da = da + c0 * v.y;
                        dd = dd + c1 * v.y;
                    }
                }
                if (!last) Xc[e] = aa;
                const int r = sm_wrap(wr.s + mr, Nr), c = sm_wrap(wc.s + mc, Nc);
                const int lr = r - axr.olo[k], lc = c - axc.olo[k];
                if (lr >= 0 && lr < ohr && lc >= 0 && lc < ohc) {
                    const int offR = g.offR[k], offC = g.offC[k];
                    sm_stc(P + (int64_t)r * g.PC + offC + c, ad);
                    sm_stc(P + (int64_t)(offR + r) * g.PC + c, da);
                    sm_stc(P + (int64_t)(offR + r) * g.PC + offC + c, dd);
                    const uint32_t k1 = sm_abs_key(ad), k2 = sm_abs_key(da), k3 = sm_abs_key(dd);
                    const int li = kbase + lr * ohc + lc;
                    K[li] = k1;
                    K[li + plane] = k2;
                    K[li + 2 * plane] = k3;
                    atomicAdd(&hist[k1 >> 19], 1u);
                    atomicAdd(&hist[k2 >> 19], 1u);
                    atomicAdd(&hist[k3 >> 19], 1u);
                    mx = max(mx, max(k1, max(k2, k3)));
                    if (last) {
                        sm_stc(P + (int64_t)r * g.PC + c, aa);
                        const uint32_t k0 = sm_abs_key(aa);
                        K[li + 3 * plane] = k0;
                        atomicAdd(&hist[k0 >> 19], 1u);
                        mx = max(mx, k0);
                    }
                }
            }
            kbase += (3 + last) * plane;
        }
        __syncthreads();
        if (k <= 3) SM_PROBE(15 + 2 * k); /* 17, 19, 21: level k's axis -1 pass */
    }
    /* the packed array's padding (non-tight layouts) holds zeros: keys 0, counted by tile 0 */
    const uint32_t npad = lt == 0 ? (uint32_t)g.npad : 0u;
    if (tid == 0 && npad) hist[0] += npad;
    {
        const uint32_t m = sm_wave_max(mx);
        if (lane == 0) wred[wv] = m;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t m = 0;
        for (int w = 0; w < SM_NW; ++w) m = max(m, wred[w]);
        atomicMax(&st->maxkey, m);
    }
    for (int i = tid; i < 4096; i += SM_THREADS)
        if (hist[i]) atomicAdd(&st->h1[i], hist[i]);
    const uint32_t nwg = (uint32_t)g.nwg;
    const uint32_t a0 = sm_arrive(&st->bar[0][0]);
    SM_PROBE(10);
    /* the grid's last arrival flips the region parity (every workgroup has read it by then): lane 0
     * of wave 1, off the polling lane's path, by per-XCD-shard counters (the last arriver of a
     * shard adds to the top counter) so no address takes more than ~gridDim / 8 returning adds */
    if (tid == 64) {
        BarState* br = bar_region(head, q);
        const uint32_t sh = blockIdx.x & (NSHARD - 1);
        const uint32_t nsh = (gridDim.x - sh + NSHARD - 1) / NSHARD; /* workgroups of this shard */
        const uint32_t nact = min((uint32_t)NSHARD, gridDim.x);     /* shards with workgroups */
        if (atomicAdd(&br->arrive[sh][0], 1u) == nsh - 1u && atomicAdd(&br->arrive[0][16], 1u) == nact - 1u)
            sm_stc(&head->parity, q + 1u);
    }
    /* inverse arena: [owned keys | coefficient windows of levels 1..L | synthesised cA | row-pass
     * rows | tap tables]; level k's windows: cV (ad), cH (da), cD (dd) planes, and cA at level L */
    float* WIN = reinterpret_cast<float*>(K) + sm_r4(nkeys);
    int nwin = 0;
    for (int k = 1; k <= L; ++k) nwin += (3 + (k == L)) * axr.sv[k].len * axc.sv[k].len;
    auto win_src = [&](int e) -> const float* { /* the packed coefficient behind window word e */
        int k = 1;
        while (k < L && e >= s_wl[k + 1].base) ++k;
        const WinLvl& w = s_wl[k];
        e -= w.base;
        int pl, idx, mr, mc;
        sm_divmod(e, w.ns, w.rns, &pl, &idx);
        sm_divmod(idx, w.scl, w.rsc, &mr, &mc);
        const int r = sm_wrap(w.srs + mr, w.R), c = sm_wrap(w.scs + mc, w.C);
        const int rr = pl == 1 || pl == 2 ? w.offR + r : r;
        const int cc = pl == 0 || pl == 2 ? w.offC + c : c;
        return P + (int64_t)rr * g.PC + cc;
    };

    /* this thread's prefetch words of the windows (see barrier 1), as element offsets from P: their
     * address arithmetic (a level search and two divisions a word) done while barrier 0 is awaited
     * -- done behind barrier 1's arrival it delayed that barrier's poll by ~1.5 us */
    uint32_t woff[SM_PF];
#pragma unroll
    for (int u = 0; u < SM_PF; ++u) {
        const int e = tid + u * SM_THREADS;
        woff[u] = e < nwin ? (uint32_t)(win_src(e) - P) : 0u;
    }
    bool ok = sm_wait(&st->bar[0][0], a0, nwg, tmo, &s_ok);
    SM_PROBE(11);

    /* ---------------- S: the two order statistics ---------------- */
    /* locate ranks ra <= rb in nb bins (get(i): count of bin i, every load of a thread issued
     * before the first is used): s_dig[x] = the bin holding rank x (-1: past the total),
     * s_bef[x] = keys in the bins before it */
    auto locate = [&](auto get, int nb, int64_t ra, int64_t rb) {
        constexpr int MAXP = 4096 / SM_THREADS;
        const int per = nb >= SM_THREADS ? nb / SM_THREADS : 1;
        uint32_t c[MAXP], cs = 0;
#pragma unroll
        for (int u = 0; u < MAXP; ++u) {
            const int i = tid * per + u;
            c[u] = (u < per && i < nb) ? get(i) : 0u;
        }
#pragma unroll
        for (int u = 0; u < MAXP; ++u) cs += c[u];
        if (tid < 2) s_dig[tid] = -1;
        uint32_t tot;
        const uint32_t ex = sm_scan(cs, wtot, &tot);
        uint32_t e = ex;
#pragma unroll
        for (int u = 0; u < MAXP; ++u) {
            if (ra >= (int64_t)e && ra < (int64_t)(e + c[u])) { s_dig[0] = tid * per + u; s_bef[0] = e; }
            if (rb >= (int64_t)e && rb < (int64_t)(e + c[u])) { s_dig[1] = tid * per + u; s_bef[1] = e; }
            e += c[u];
        }
        __syncthreads();
    };
    const int64_t ra0 = g.r0, rb0 = g.above ? g.r0 : g.r0 + 1;
    uint32_t ka = 0, kb = 0, mk = 0;
    int64_t rem = 0; /* ra inside the rank's 12-bit bin */
    uint32_t d1 = 0, cnt1 = 0;
    __shared__ uint32_t s_fill, s_min[2], s_lc, s_lk[2];
    __shared__ uint32_t s_list[64]; /* pass B's keys of digit da (the list form) */
    bool ovf = false;
    uint32_t* G = reinterpret_cast<uint32_t*>(arena + SM_ARENA - SM_GATHER);
    if (ok) {
        /* digit 1: the 12-bit bin of ra */
        if (tid == 0) { s_fill = 0; s_min[0] = 0xFFFFFFFFu; s_min[1] = 0xFFFFFFFFu; }
        locate([&](int i) { return sm_ldc(st->h1 + i); }, 4096, ra0, ra0);
        d1 = (uint32_t)s_dig[0];
        rem = ra0 - s_bef[0];
        SM_PROBE(2);
        /* this workgroup's keys of that bin into its slot, its smallest key above the bin */
        uint32_t* slot = t.slots + (int64_t)blockIdx.x * SM_SLOT_WORDS;
        uint32_t mn = 0xFFFFFFFFu;
        for (int i = tid; i < nkeys; i += SM_THREADS) {
            const uint32_t k = K[i];
            const uint32_t b12 = k >> 19;
            if (b12 == d1) {
                const uint32_t p = atomicAdd(&s_fill, 1u);
                if (p < (uint32_t)SM_SLOT_KEYS) sm_stc(slot + 3 + p, k);
            } else if (b12 > d1) {
                mn = min(mn, k);
            }
        }
        mn = sm_wave_min(mn);
        if (lane == 0 && mn != 0xFFFFFFFFu) atomicMin(&s_min[0], mn);
        __syncthreads();
        if (tid == 0) {
            const uint32_t f = s_fill;
            sm_stc(slot, min(f, (uint32_t)SM_SLOT_KEYS) | (f > (uint32_t)SM_SLOT_KEYS ? 0x80000000u : 0u));
            sm_stc(slot + 1, (npad && d1 == 0) ? npad : 0u);
            sm_stc(slot + 2, s_min[0]);
        }
        SM_PROBE(3);
        const uint32_t a1 = sm_arrive(&st->bar[1][0]);
        SM_PROBE(4);
        /* every level's coefficient windows of the inverse, from P (complete since barrier 0):
         * issued now, their round trip hidden behind this barrier's wait */
        float pv[SM_PF];
#pragma unroll
        for (int u = 0; u < SM_PF; ++u) {
            const int e = tid + u * SM_THREADS;
            pv[u] = e < nwin ? sm_ldc(P + woff[u]) : 0.0f;
        }
        ok = sm_wait(&st->bar[1][0], a1, nwg, tmo, &s_ok);
        SM_PROBE(5);
#pragma unroll
        for (int u = 0; u < SM_PF; ++u) {
            const int e = tid + u * SM_THREADS;
            if (e < nwin) WIN[e] = pv[u];
        }
        for (int e = tid + SM_PF * SM_THREADS; e < nwin; e += SM_THREADS) WIN[e] = sm_ldc(win_src(e));
        SM_PROBE(7);
    }
    if (ok) {
        /* every slot of the segment into LDS (and the segment's largest key, final since barrier 0) */
        mk = sm_ldc(&st->maxkey);
        const uint32_t* segs = t.slots + (int64_t)g.wg_begin * SM_SLOT_WORDS;
        const int nw = (int)nwg * SM_SLOT_WORDS;
        constexpr int GPT = SM_GATHER / SM_THREADS;
        uint32_t gv[GPT];
#pragma unroll
        for (int u = 0; u < GPT; ++u) {
            const int i = tid + u * SM_THREADS;
            gv[u] = i < nw ? sm_ldc(segs + i) : 0u;
        }
#pragma unroll
        for (int u = 0; u < GPT; ++u) {
            const int i = tid + u * SM_THREADS;
            if (i < nw) G[i] = gv[u];
        }
        for (int i = tid; i < 1536; i += SM_THREADS) hist[i] = 0u; /* pass A bins, then pass B's */
        if (tid == 0) { s_min[1] = 0xFFFFFFFFu; s_lc = 0u; }
        __syncthreads();
        SM_PROBE(8);
        /* the slot headers (wave 0 reduces them) */
        __shared__ uint32_t s_hdr[4];
        if (wv == 0) {
            uint32_t oo = 0, cc = 0, zz = 0, mw = 0xFFFFFFFFu;
            for (int w = lane; w < (int)nwg; w += 64) {
                const uint32_t c0 = G[w * SM_SLOT_WORDS];
                oo |= c0 & 0x80000000u;
                cc += c0 & 0x7FFFFFFFu;
                zz += G[w * SM_SLOT_WORDS + 1];
                mw = min(mw, G[w * SM_SLOT_WORDS + 2]);
            }
            const uint32_t o = sm_wave_or(oo), c = sm_wave_sum(cc);
            zz = sm_wave_sum(zz);
            mw = sm_wave_min(mw);
            if (lane == 0) { s_hdr[0] = o; s_hdr[1] = c; s_hdr[2] = zz; s_hdr[3] = mw; }
        }
        /* a thread's keys: entries tid + u * SM_THREADS of the slot array, read while wave 0 reduces */
        constexpr int KPT = SM_SEG_WG_MAX * SM_SLOT_KEYS / SM_THREADS + 1;
        uint32_t kk[KPT];
        bool kv[KPT];
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
            const int i = tid + u * SM_THREADS;
            const int w = i / SM_SLOT_KEYS, j = i - w * SM_SLOT_KEYS;
            const bool in = w < (int)nwg;
            const uint32_t c = in ? G[w * SM_SLOT_WORDS] & 0x7FFFFFFFu : 0u;
            kk[u] = in ? G[w * SM_SLOT_WORDS + 3 + j] : 0u;
            kv[u] = j < (int)c;
        }
        __syncthreads();
        const uint32_t z = s_hdr[2], mnab = s_hdr[3];
        cnt1 = s_hdr[1] + z;
        ovf = s_hdr[0] != 0;
        SM_PROBE(9);
        if (!ovf) {
            /* the exact ranks among the gathered keys: bits 18..9, then 8..0 (the padding zeros
             * carry zero digits) */
            const int64_t rbi = rb0 - (ra0 - rem); /* rb inside the bin */
#pragma unroll
            for (int u = 0; u < KPT; ++u)
                if (kv[u]) atomicAdd(&hist[(kk[u] >> 9) & 1023u], 1u);
            if (tid == 0 && z) hist[0] += z;
            __syncthreads();
            locate([&](int i) { return hist[i]; }, 1024, rem, min(rbi, (int64_t)cnt1 - 1));
            const uint32_t da = (uint32_t)s_dig[0], db = (uint32_t)s_dig[1];
            const int64_t ra2 = rem - s_bef[0], rb2 = rbi - s_bef[0];
            SM_PROBE(12);
            /* keys of digit da: hist[da] (the padding zeros included when da == 0) */
            const uint32_t nda = hist[da];
            if (nda <= 64u && !(z && da == 0)) { /* block-uniform: the usual case (cfg3: a handful) */
                /* pass B as a list: the digit's keys appended in LDS, then one wave ranks them by
                 * counting (rank = keys below + equal keys listed before), instead of a 512-bin
                 * histogram and a block scan (round 6: k_small 29.1 -> see DESIGN.md) */
                uint32_t mnA = 0xFFFFFFFFu;
#pragma unroll
                for (int u = 0; u < KPT; ++u) {
                    const uint32_t a = (kk[u] >> 9) & 1023u;
                    if (kv[u] && a == da) s_list[atomicAdd(&s_lc, 1u)] = kk[u];
                    else if (kv[u] && a > da) mnA = min(mnA, kk[u]);
                }
                mnA = sm_wave_min(mnA);
                if (lane == 0 && mnA != 0xFFFFFFFFu) atomicMin(&s_min[1], mnA);
                __syncthreads();
                if (wv == 0) {
                    const int n = (int)nda;
                    const uint32_t mine = lane < n ? s_list[lane] : 0xFFFFFFFFu;
                    int below = 0;
                    for (int j = 0; j < n; ++j) {
                        const uint32_t kj = s_list[j];
                        below += (kj < mine) | ((kj == mine) & (j < lane));
                    }
                    if (lane < n && below == (int)ra2) s_lk[0] = mine;
                    if (lane < n && below == (int)rb2) s_lk[1] = mine;
                }
                __syncthreads();
                ka = s_lk[0];
                if (rbi >= (int64_t)cnt1) kb = mnab;             /* rb past the bin: the next key above it */
                else if (rb2 >= (int64_t)nda) kb = s_min[1];     /* rb in a later 10-bit group of the bin */
                else kb = s_lk[1];
            } else {
            uint32_t* hb = hist + 1024;
            uint32_t mnA = 0xFFFFFFFFu;
#pragma unroll
            for (int u = 0; u < KPT; ++u) {
                const uint32_t a = (kk[u] >> 9) & 1023u;
                if (kv[u] && a == da) atomicAdd(&hb[kk[u] & 511u], 1u);
                else if (kv[u] && a > da) mnA = min(mnA, kk[u]);
            }
            mnA = sm_wave_min(mnA);
            if (lane == 0 && mnA != 0xFFFFFFFFu) atomicMin(&s_min[1], mnA);
            if (tid == 0 && z && da == 0) hb[0] += z;
            __syncthreads();
            locate([&](int i) { return hb[i]; }, 512, ra2, rb2);
            ka = (d1 << 19) | (da << 9) | (uint32_t)s_dig[0];
            if (rbi >= (int64_t)cnt1) kb = mnab;             /* rb past the bin: the next key above it */
            else if (db != da) kb = s_min[1];                /* rb in a later 10-bit group of the bin */
            else kb = (d1 << 19) | (da << 9) | (uint32_t)s_dig[1];
            }
        }
        SM_PROBE(13);
    }
    if (ok && ovf) {
        /* fallback (a workgroup held more keys of the bin than its slot): two more digits over the
         * segment, bits 18..8 and 7..0, each through the segment's histograms and a barrier */
        int64_t r = rem;
        uint32_t prefix = d1;
        __syncthreads();
        for (int i = tid; i < 2048; i += SM_THREADS) hist[i] = 0u;
        __syncthreads();
        for (int i = tid; i < nkeys; i += SM_THREADS) {
            const uint32_t k = K[i];
            if ((k >> 19) == prefix) atomicAdd(&hist[(k >> 8) & 2047u], 1u);
        }
        if (tid == 0 && npad && prefix == 0) hist[0] += npad;
        __syncthreads();
        for (int i = tid; i < 2048; i += SM_THREADS)
            if (hist[i]) atomicAdd(&st->h2[i], hist[i]);
        const uint32_t a2 = sm_arrive(&st->bar[2][0]);
        ok = sm_wait(&st->bar[2][0], a2, nwg, tmo, &s_ok);
        if (ok) {
            locate([&](int i) { return sm_ldc(st->h2 + i); }, 2048, r, r);
            r -= s_bef[0];
            prefix = (prefix << 11) | (uint32_t)s_dig[0];
            for (int i = tid; i < 256; i += SM_THREADS) hist[i] = 0u;
            if (tid == 0) s_min[0] = 0xFFFFFFFFu;
            __syncthreads();
            uint32_t mn = 0xFFFFFFFFu;
            for (int i = tid; i < nkeys; i += SM_THREADS) {
                const uint32_t k = K[i];
                if ((k >> 8) == prefix) atomicAdd(&hist[k & 255u], 1u);
                else if ((k >> 8) > prefix) mn = min(mn, k);
            }
            mn = sm_wave_min(mn);
            if (lane == 0 && mn != 0xFFFFFFFFu) atomicMin(&s_min[0], mn);
            if (tid == 0 && npad && prefix == 0) hist[0] += npad;
            __syncthreads();
            if (tid == 0 && s_min[0] != 0xFFFFFFFFu) atomicMax(&st->notmin, ~s_min[0]);
            for (int i = tid; i < 256; i += SM_THREADS)
                if (hist[i]) atomicAdd(&st->h3[i], hist[i]);
            const uint32_t a3 = sm_arrive(&st->bar[3][0]);
            ok = sm_wait(&st->bar[3][0], a3, nwg, tmo, &s_ok);
        }
        if (ok) {
            const int64_t rb = g.above ? r : r + 1;
            locate([&](int i) { return sm_ldc(st->h3 + i); }, 256, r, rb);
            ka = (prefix << 8) | (uint32_t)s_dig[0];
            kb = s_dig[1] >= 0 ? ((prefix << 8) | (uint32_t)s_dig[1]) : ~sm_ldc(&st->notmin);
        }
    }
    if (!ok) {
        if (tid == 0) atomicMax(&res[g.res].path, (int32_t)MODE_FAULT);
        return; /* nothing stored to `out`: the caller's input and output are untouched */
    }
    if (ovf) mk = sm_ldc(&st->maxkey);
    /* threshold: numpy/lib/function_base.py _lerp -- diff in float32, the blend in float64 */
    const float fa = __uint_as_float(ka), fb = __uint_as_float(kb);
    const float diff = fb - fa;
    const double gm = g.gamma;
    double thr = (gm >= 0.5) ? (double)fb - (double)diff * (1.0 - gm) : (double)fa + (double)diff * gm;
    if (mk > 0x7F800000u) thr = __longlong_as_double(0x7FF8000000000000ll); /* NaN present: np.percentile is NaN */
    const float thr32 = (float)thr;
    auto tl = [&](float c) { return (fabsf(c) < thr32) ? 0.0f : c; };

    /* ---------------- I: synthesis of the owned output block ---------------- */
    /* the np.where of :31 is applied as the packed coefficients are read below (tA: the cA plane
     * of level L, packed too; the synthesised ones are not thresholded) */
    int ia = 0, ilh = 0;
    for (int k = 1; k <= L; ++k) {
        ia = max(ia, axr.sv[k].len * axc.sv[k].len);
        ilh = max(ilh, 2 * axr.sv[k].len * axc.sv[k - 1].len);
    }
    float* A = WIN + sm_r4(nwin);
    float2* LoHi = reinterpret_cast<float2*>(A + sm_r4(ia));
    const int HH = F / 2;
    unsigned long long z = 0;
    int wb = nwin;
    for (int k = L; k >= 1; --k) {
        const SmIvl sr = axr.sv[k], sc = axc.sv[k], orr = axr.sv[k - 1], oc = axc.sv[k - 1];
        const int Nr = g.R[k], Nor = g.R[k - 1], Nc = g.C[k], Noc = g.C[k - 1];
        const int ns = sr.len * sc.len;
        wb -= (3 + (k == L)) * ns;
        const float* cV = WIN + wb;
        const float* cH = cV + ns;
        const float* cD = cH + ns;
        const float* cA = k == L ? cD + ns : A;
        const bool topA = k == L;
        auto tA = [&](float c) { return topA ? tl(c) : c; };
        constexpr int HT = FT / 2;
        if (k == L) SM_PROBE(14);
        /* axis -1: lo = rec(cA, cV), hi = rec(cH, cD) at every source row, output columns oc */
        {
            const int n = sr.len * oc.len;
            const float inv = 1.0f / (float)oc.len;
            for (int e = tid; e < n; e += SM_THREADS) {
                int mr, mc;
                sm_divmod(e, oc.len, inv, &mr, &mc);
                const int rb0 = mr * sc.len;
                float lo = 0.0f, hi = 0.0f;
                const int fb = sm_syn_fast(oc, Noc, sc, Nc, F, mc);
                if (FT > 0 && __all(fb >= 0)) {
                    const int b0 = rb0 + (fb >> 6), par = (fb >> 5) & 1, c1 = fb & 31;
                    const bool plain = __all(c1 == 0);
                    float va[HT > 0 ? HT : 1], vh[HT > 0 ? HT : 1], vv[HT > 0 ? HT : 1], vd[HT > 0 ? HT : 1];
#pragma unroll
                    for (int qq = 0; qq < HT; ++qq) {
                        va[qq] = tA(cA[b0 - qq]);
                        vv[qq] = tl(cV[b0 - qq]);
                        vh[qq] = tl(cH[b0 - qq]);
                        vd[qq] = tl(cD[b0 - qq]);
                    }
                    sf2 lh = {0.0f, 0.0f}; /* (lo, hi) packed */
                    sm_order<HT>(c1, plain, [&](int j) { return sf2{va[j], vh[j]}; },
                                 [&](int j) { return staps[2][2 * j + par]; },
                                 [&](float cf, sf2 x) { lh = lh + sf2{cf, cf} * x; });
                    sm_order<HT>(c1, plain, [&](int j) { return sf2{vv[j], vd[j]}; },
                                 [&](int j) { return staps[3][2 * j + par]; },
                                 [&](float cf, sf2 x) { lh = lh + sf2{cf, cf} * x; });
                    lo = lh.x;
                    hi = lh.y;
                } else {
                    const SmSyn sy = sm_syn_at(oc, Noc, Nc, F, mc);
                    for (int qq = 0; qq < HH; ++qq) {
                        int ci;
                        const int sl = sm_syn_tap(sy, sc, Nc, qq, &ci);
                        lo = lo + staps[2][ci] * tA(cA[rb0 + sl]);
                        hi = hi + staps[2][ci] * tl(cH[rb0 + sl]);
                    }
                    for (int qq = 0; qq < HH; ++qq) {
                        int ci;
                        const int sl = sm_syn_tap(sy, sc, Nc, qq, &ci);
                        lo = lo + staps[3][ci] * tl(cV[rb0 + sl]);
                        hi = hi + staps[3][ci] * tl(cD[rb0 + sl]);
                    }
                }
                LoHi[e] = make_float2(lo, hi);
            }
        }
        __syncthreads();
        if (L - k <= 2) SM_PROBE(22 + 2 * (L - k)); /* 22, 24, 26: synthesis level k's axis -1 pass */
        /* axis -2: y = rec_lo over lo, then rec_hi over hi, at the output rows orr */
        {
            const int n = orr.len * oc.len;
            const float inv = 1.0f / (float)oc.len;
            float* out = g.out + (int64_t)b * H0 * W0;
            for (int e = tid; e < n; e += SM_THREADS) {
                int mr, mc;
                sm_divmod(e, oc.len, inv, &mr, &mc);
                float y = 0.0f;
                const int fb = sm_syn_fast(orr, Nor, sr, Nr, F, mr);
                if (FT > 0 && __all(fb >= 0)) {
                    const int b0 = fb >> 6, par = (fb >> 5) & 1, c1 = fb & 31;
                    const bool plain = __all(c1 == 0);
                    float2 v[HT > 0 ? HT : 1];
#pragma unroll
                    for (int qq = 0; qq < HT; ++qq) v[qq] = LoHi[(b0 - qq) * oc.len + mc];
                    sm_order<HT>(c1, plain, [&](int j) { return v[j].x; }, [&](int j) { return staps[2][2 * j + par]; },
                                 [&](float cf, float x) { y = y + cf * x; });
                    sm_order<HT>(c1, plain, [&](int j) { return v[j].y; }, [&](int j) { return staps[3][2 * j + par]; },
                                 [&](float cf, float x) { y = y + cf * x; });
                } else {
                    const SmSyn sy = sm_syn_at(orr, Nor, Nr, F, mr);
                    for (int qq = 0; qq < HH; ++qq) {
                        int ci;
                        const int sl = sm_syn_tap(sy, sr, Nr, qq, &ci);
                        y = y + staps[2][ci] * LoHi[sl * oc.len + mc].x;
                    }
                    for (int qq = 0; qq < HH; ++qq) {
                        int ci;
                        const int sl = sm_syn_tap(sy, sr, Nr, qq, &ci);
                        y = y + staps[3][ci] * LoHi[sl * oc.len + mc].y;
                    }
                }
                if (k > 1) {
                    A[e] = y;
                } else {
                    out[(int64_t)(orr.s + mr) * W0 + oc.s + mc] = y;
                    z += y == 0.0f;
                }
            }
        }
        __syncthreads();
    }
    {
        const uint32_t zz = sm_wave_sum((uint32_t)z);
        if (lane == 0) wred[wv] = zz;
        __syncthreads();
        if (tid == 0) {
            unsigned long long s = 0;
            for (int w = 0; w < SM_NW; ++w) s += wred[w];
            if (s) atomicAdd(reinterpret_cast<unsigned long long*>(&res[g.res].zero_count), s);
            if (lt == 0) {
                wtp_result& r = res[g.res];
                r.numel = g.numel;
                r.coeff_numel = g.n;
                r.thr64 = thr;
                r.thr32_bits = __float_as_uint(thr32);
                r.max_abs_bits = mk;
                r.eff_level = L;
                atomicMax(&r.path, (int32_t)WTP_PATH_SMALL);
            }
        }
    }
    if (t.stamps) { /* measurement only: the workgroup's end, once its stores have completed */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) atomicMax(t.stamps + 1, sm_ticks());
        SM_PROBE(15);
    }
}

/* ------------------------------------------------------------------ host --- */
int small_capacity() {
    static std::atomic<int> cache[16];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
    if (dev < 16) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c) return c > 0 ? c : 0;
    }
    int cus = 0, cap = -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
        const void* ks[] = {(const void*)k_small<0>, (const void*)k_small<2>, (const void*)k_small<4>,
                            (const void*)k_small<6>, (const void*)k_small<8>, (const void*)k_small<10>,
                            (const void*)k_small<12>, (const void*)k_small<16>, (const void*)k_small<18>};
        cap = cus; /* one workgroup per CU, if every instance can hold one */
        for (const void* k : ks) {
            int per = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, SM_THREADS, 0) != hipSuccess || per < 1) cap = -1;
        }
    }
    (void)hipGetLastError();
    if (dev < 16) cache[dev].store(cap, std::memory_order_relaxed);
    return cap > 0 ? cap : 0;
}
void launch_small(const SmallTable& t0, SelHeader* head, wtp_result* res, hipStream_t s) {
    SmallTable t = t0;
    t.timeout = resident_timeout_us() * 100u; /* 100 MHz wall clock */
    t.stamps = kernel_stamps();
    switch (t.tp.F) {
    case 2: hipLaunchKernelGGL(k_small<2>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    case 4: hipLaunchKernelGGL(k_small<4>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    case 6: hipLaunchKernelGGL(k_small<6>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    case 8: hipLaunchKernelGGL(k_small<8>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    case 10: hipLaunchKernelGGL(k_small<10>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    case 12: hipLaunchKernelGGL(k_small<12>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    case 16: hipLaunchKernelGGL(k_small<16>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    case 18: hipLaunchKernelGGL(k_small<18>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    default: hipLaunchKernelGGL(k_small<0>, dim3(t.nblk), dim3(SM_THREADS), 0, s, t, head, res); break;
    }
}

}  // namespace wtp
