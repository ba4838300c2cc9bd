/*
 * filterbank.hip -- LDS-tiled, one-launch-per-level 2-D filter bank for gfx950.
 *
 * pywt.wavedec2 / waverec2 in periodization mode (ResNet/dwt_pruning.py:67-77) apply one
 * separable level at a time: analysis along axis -2 over the whole array, then along axis -1
 * (pywt/_multidim.py:183-191); synthesis along axis -1, then axis -2 (:288-309).  Each level
 * here is ONE kernel: a workgroup loads an input tile plus the filter halo into LDS once
 * (periodic / odd-length extension applied while loading), runs the first 1-D pass into LDS
 * and the second pass straight to HBM.  Every output sample is summed in PyWavelets' exact
 * order (csrc/wt_dwt_core.h: ascending taps in the interior, the split order at the right
 * edge, the special first synthesis site); only where the samples come from changes, so the
 * results are bit-identical to the two-pass kernels and to the oracle.  The two bands that
 * share a sample (lo/hi taps, or two subbands under one tap) are carried as a float2 so the
 * multiplies and adds issue as packed FP32 (v_pk_mul_f32 / v_pk_add_f32) -- still one
 * rounding per multiply and per add, as the contract requires (-ffp-contract=off).
 *
 * Forward tile: FR x FC outputs per subband; input tile (2 FR + F - 2) x (2 FC + F - 2).
 * Inverse tile: IR x IC outputs; coefficient tiles (IR/2 + F/2 + 1) x (IC/2 + F/2 + 1).
 */
#include "wtp_internal.h"
#include "wt_dwt_core.h"
#include "fb_index.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <type_traits>
#include <vector>

#pragma clang fp contract(off)

namespace wtp {

typedef float f2 __attribute__((ext_vector_type(2)));

/* timing probes for tools/mb/fblab.hip (empty in the library) */
#ifndef WTP_FPROBE
#define WTP_FPROBE(i)
#endif

/* waves per SIMD the filter-bank kernels are register-budgeted for (db8: 5 needs <= 96 VGPRs) */
#define WTP_FB_FWD_WPE __attribute__((amdgpu_waves_per_eu(5)))
#define WTP_FB_INV_WPE __attribute__((amdgpu_waves_per_eu(5)))

constexpr int FB_THREADS = 256;
/* forward output tile (per subband).  FC = 56: the axis -2 pass has 2 (2 FC + F - 2) column items,
 * <= 256 for F <= 18, so every thread of the workgroup takes exactly one (with FC = 64 and db8,
 * 284 items: wave 0 -- always on the same SIMD -- took a second one, doubling that SIMD's share
 * of the pass; cfg5 forward levels -5 %) */
constexpr int FR = 16, FC = 56;
constexpr int IR = 64, IC = 64;  /* inverse output tile */
constexpr int INV_RG = 2; /* synthesis row-pass rows interleaved per wave */
constexpr int FB_MAX_LDS = 64 * 1024;
/* the forward input tile in LDS (specialised filters): row pitch FWD_TP floats, the tile's first
 * column at FWD_S0 -- so that its column 0 - FWD_S0 is 16-byte aligned in the image (a tile's
 * first input column is 2 FC tc - F/2 + 1) and interior rows load as whole float4s */
template <int FT> constexpr int FWD_S0 = ((1 - FT / 2) % 4 + 4) % 4;
/* k_fwd_int's column-pass results in LDS: row o holds its even columns from o * 2 LHH, its odd ones
 * from o * 2 LHH + LHH (float2 units).  LHH = 8 (mod 16): a wave's float2 writes of consecutive
 * columns then put the even lanes on banks b .. b + 15 and the odd lanes on b + 16 .. b + 31 of
 * each 16-lane group (with LHH = (NC + 1) / 2 = 63 at db8 the two halves overlapped on 14 banks:
 * 0.69 bank-conflict cycles per LDS instruction, round-5 PMC); the row pass reads stay contiguous */
constexpr int fwd_lhh(int nc) { return (nc + 1) / 2 + ((8 - (nc + 1) / 2) % 16 + 16) % 16; }
template <int FT> constexpr int FWD_TP = (FWD_S0<FT> + 2 * FC + FT - 2 + 3) / 4 * 4;


__device__ __forceinline__ int ext_idx(int t, int N) { /* wt_ext_index in 32 bits */
    const int Ne = N + (N & 1);
    int r = t % Ne;
    r = r < 0 ? r + Ne : r;
    return r < N ? r : N - 1;
}
__device__ __forceinline__ int pmod32(int a, int m) {
    const int r = a % m;
    return r < 0 ? r + m : r;
}

/* analysis of one output (both bands) at site i = F/2 + 2o of a line of N samples;
 * get(g) returns the sample at unwrapped position g (the tile already holds the extension) */
template <int FT, class Get>
__device__ __forceinline__ f2 ana2(int i, int N, int Frt, const float* lo, const float* hi, const Get& get) {
    f2 acc = {0.0f, 0.0f};
    if constexpr (FT > 0) {
        /* every sample the output needs (positions i-j, j < F) is read into registers first,
         * so the LDS reads issue back to back; then the sum runs in pywt's order */
        float v[FT];
#pragma unroll
        for (int j = 0; j < FT; ++j) v[j] = get(i - j);
        if (i < N) {
#pragma unroll
            for (int j = 0; j < FT; ++j) { const f2 t = {lo[j], hi[j]}; acc = acc + t * v[j]; }
        } else {
#pragma unroll
            for (int j = FT - 1; j >= 0; --j)
                if (i - j >= N) { const f2 t = {lo[j], hi[j]}; acc = acc + t * v[j]; }
#pragma unroll
            for (int j = 0; j < FT; ++j)
                if (i - j < N) { const f2 t = {lo[j], hi[j]}; acc = acc + t * v[j]; }
        }
    } else {
        const int F = Frt;
        if (i < N) {
            for (int j = 0; j < F; ++j) { const f2 t = {lo[j], hi[j]}; acc = acc + t * get(i - j); }
        } else {
            for (int j = F - 1; j >= 0; --j)
                if (i - j >= N) { const f2 t = {lo[j], hi[j]}; acc = acc + t * get(i - j); }
            for (int j = 0; j < F; ++j)
                if (i - j < N) { const f2 t = {lo[j], hi[j]}; acc = acc + t * get(i - j); }
        }
    }
    return acc;
}

/* ana2 for specialised filters with the samples already in registers: samp(j) is the sample
 * at position i - j (a compile-time register index after unrolling) */
template <int FT, class Samp>
__device__ __forceinline__ f2 ana2_j(int i, int N, const float* lo, const float* hi, const Samp& samp) {
    f2 acc = {0.0f, 0.0f};
    if (__all(i < N)) { /* wave-uniform: the interior form, no predication */
#pragma unroll
        for (int j = 0; j < FT; ++j) { const f2 t = {lo[j], hi[j]}; acc = acc + t * samp(j); }
    } else if (i < N) {
#pragma unroll
        for (int j = 0; j < FT; ++j) { const f2 t = {lo[j], hi[j]}; acc = acc + t * samp(j); }
    } else {
#pragma unroll
        for (int j = FT - 1; j >= 0; --j)
            if (i - j >= N) { const f2 t = {lo[j], hi[j]}; acc = acc + t * samp(j); }
#pragma unroll
        for (int j = 0; j < FT; ++j)
            if (i - j < N) { const f2 t = {lo[j], hi[j]}; acc = acc + t * samp(j); }
    }
    return acc;
}

/* two analysis outputs at the same site sharing taps (e.g. the L and H rows): returns
 * (lo.x, hi.x) in r0 and (lo.y, hi.y) in r1, each band carried packed over the two rows */
template <int FT, class Get>
__device__ __forceinline__ void ana2x2(int i, int N, int Frt, const float* lo, const float* hi, const Get& get,
                                       f2& low, f2& high) {
    f2 a = {0.0f, 0.0f}, d = {0.0f, 0.0f};
    if constexpr (FT > 0) {
        f2 v[FT];
#pragma unroll
        for (int j = 0; j < FT; ++j) v[j] = get(i - j);
        auto term = [&](int j) { a = a + lo[j] * v[j]; d = d + hi[j] * v[j]; };
        if (__all(i < N)) { /* wave-uniform: the interior form, no predication */
#pragma unroll
            for (int j = 0; j < FT; ++j) term(j);
        } else if (i < N) {
#pragma unroll
            for (int j = 0; j < FT; ++j) term(j);
        } else {
#pragma unroll
            for (int j = FT - 1; j >= 0; --j)
                if (i - j >= N) term(j);
#pragma unroll
            for (int j = 0; j < FT; ++j)
                if (i - j < N) term(j);
        }
    } else {
        const int F = Frt;
        auto term = [&](int j) { const f2 v = get(i - j); a = a + lo[j] * v; d = d + hi[j] * v; };
        if (i < N) {
            for (int j = 0; j < F; ++j) term(j);
        } else {
            for (int j = F - 1; j >= 0; --j)
                if (i - j >= N) term(j);
            for (int j = 0; j < F; ++j)
                if (i - j < N) term(j);
        }
    }
    low = a;
    high = d;
}

/* synthesis site with an unwrapped source position: the H-even special last output n = 2N-1
 * reads positions i - j + N (== i - j mod N), so a tile's sites increase monotonically */
struct SiteU {
    int i, iu, par, special;
};
__device__ __forceinline__ SiteU site_u(int n, int N, int F) {
    const wt_syn_site s = wt_syn_locate(n, N, F);
    SiteU u;
    u.i = (int)s.i;
    u.par = s.par;
    u.special = s.special;
    u.iu = u.i + ((s.special && n == 2 * N - 1) ? N : 0);
    return u;
}

/* one synthesis pass (H terms) in wt_syn_pass's exact order; get(g) at unwrapped g = iu - j;
 * tap(j) = rec[2j + par] for this output's parity */
template <int FT, class T, class Tap, class Get>
__device__ __forceinline__ T syn_pass_u(const SiteU& s, int N, int Frt, const Tap& tap, const Get& get, T acc) {
    const int i = s.i;
    if constexpr (FT > 0) {
        constexpr int H = FT / 2;
        T v[H];
#pragma unroll
        for (int j = 0; j < H; ++j) v[j] = get(s.iu - j);
        if (s.special) {
#pragma unroll
            for (int j = H - 1; j >= 0; --j)
                if (i - j >= 0) acc = acc + tap(j) * v[j];
#pragma unroll
            for (int j = 0; j < H; ++j)
                if (i - j < 0) acc = acc + tap(j) * v[j];
        } else if (i < N) {
#pragma unroll
            for (int j = 0; j < H; ++j) acc = acc + tap(j) * v[j];
        } else {
#pragma unroll
            for (int j = H - 1; j >= 0; --j)
                if (i - j >= N) acc = acc + tap(j) * v[j];
#pragma unroll
            for (int j = 0; j < H; ++j)
                if (i - j < N) acc = acc + tap(j) * v[j];
        }
    } else {
        const int H = Frt / 2;
        if (s.special) {
            for (int j = H - 1; j >= 0; --j)
                if (i - j >= 0) acc = acc + tap(j) * get(s.iu - j);
            for (int j = 0; j < H; ++j)
                if (i - j < 0) acc = acc + tap(j) * get(s.iu - j);
        } else if (i < N) {
            for (int j = 0; j < H; ++j) acc = acc + tap(j) * get(s.iu - j);
        } else {
            for (int j = H - 1; j >= 0; --j)
                if (i - j >= N) acc = acc + tap(j) * get(s.iu - j);
            for (int j = 0; j < H; ++j)
                if (i - j < N) acc = acc + tap(j) * get(s.iu - j);
        }
    }
    return acc;
}

/* the interior form of syn_pass_u (not special, i < N): ascending taps */
template <int FT, class T, class Tap, class Get>
__device__ __forceinline__ T syn_pass_inner(const SiteU& s, int Frt, const Tap& tap, const Get& get, T acc) {
    if constexpr (FT > 0) {
        constexpr int H = FT / 2;
        T v[H];
#pragma unroll
        for (int j = 0; j < H; ++j) v[j] = get(s.iu - j);
#pragma unroll
        for (int j = 0; j < H; ++j) acc = acc + tap(j) * v[j];
    } else {
        for (int j = 0; j < Frt / 2; ++j) acc = acc + tap(j) * get(s.iu - j);
    }
    return acc;
}

/* ------------------------------------------------------------- analysis --- */
struct FwdArgs {
    const float* in;
    int64_t in_bs;       /* batch stride of the input level */
    int R, C;            /* input level dims (row pitch C) */
    int Ro, Co;          /* output dims per subband */
    float* P;
    int64_t P_bs;        /* packed image per batch item: PR * PC */
    int PC, offR, offC;  /* level-k detail origin in the packed image */
    float* anext;        /* (B, Ro, Co) next-level approximation; unused when last */
    int last, tilesC, tilesR;
    int al16;            /* in is 16-byte aligned and C % 4 == 0: interior tiles load float4 rows */
    /* the interior tiles (k_fwd_int): rows tr0 .. tr0 + nTR - 1, columns tc0 .. tc0 + nTC - 1 of
     * the tile grid; frame != 0: k_fwd_level runs only the tiles around that rectangle */
    int tr0, nTR, tc0, nTC, frame;
};

/* One launch covers the same level of up to FB_UNI items of the SAME geometry (same filter; the
 * cfg5 blocks of a call, the batch of one tensor): the geometry once, the pointers per item, and
 * a block's item is its tile / tiles-per-item.  The specialised kernels take their taps as a
 * SmallTaps (F <= 20): the whole argument stays near 2 KB. */
constexpr int FB_UNI = 64;
struct FwdGroup {
    FwdArgs geo;            /* the items' geometry; its pointers are unused */
    int n, tiles;           /* items; tiles per item */
    FastDiv dv_tiles, dv_per, dv_ntc; /* k_*_int: by tiles, by the rectangle's (or frame's) tiles, by nTC */
    FastDiv dv_tc, dv_side;           /* the frame's decode: by tilesC, by tilesC - nTC */
    const float* in[FB_UNI];
    float* anext[FB_UNI];
    float* P[FB_UNI];
};
template <int FT> using TapsT = typename std::conditional<FT == 0, Taps, SmallTaps>::type;


/* taps of the interior kernels: analysis {dec_lo[j], dec_hi[j]} adjacent, so one SGPR pair is
 * both bands' packed tap */
struct FwdIntTaps {
    f2 t[SM_F_MAX];
};
#define WTP_FB_INT_WPE __attribute__((amdgpu_waves_per_eu(EDGE ? 5 : 6))) /* EDGE: room for the edge forms */

template <int FT>
__global__ __launch_bounds__(FB_THREADS) WTP_FB_FWD_WPE void k_fwd_level(FwdGroup g, TapsT<FT> tp) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int F = FT ? FT : tp.F;
    const int NR = 2 * FR + F - 2, NC = 2 * FC + F - 2;
    float* T = lds;                /* NR x NC input tile */
    /* FR x NC: (L, H) column-pass outputs, even columns then odd (row-pass reads at stride 2
     * stay conflict-free).  Specialised filters hold their column results in registers across
     * a barrier and write them over the input tile: half the LDS, twice the workgroups per CU */
    float2* LH = reinterpret_cast<float2*>(FT > 0 ? lds : lds + NR * NC);
    const int HALF = (NC + 1) / 2;
    auto lhi = [&](int o, int cc) { return o * NC + (cc & 1) * HALF + (cc >> 1); };
    const int gt = xcd_tile(blockIdx.x, gridDim.x);
    const int item = gt / g.tiles;
    FwdArgs a = g.geo;
    a.in = g.in[item];
    a.anext = g.anext[item];
    a.P = g.P[item];
    const int tile = gt - item * g.tiles;
    int tc, tr, b;
    if (a.frame) {
        const int per = a.tilesR * a.tilesC - a.nTR * a.nTC;
        b = tile / per;
        frame_tile(tile - b * per, a.tilesC, a.tr0, a.nTR, a.tc0, a.nTC, &tr, &tc);
    } else {
        tc = tile % a.tilesC;
        tr = (tile / a.tilesC) % a.tilesR;
        b = tile / (a.tilesC * a.tilesR);
    }
    const int o0r = tr * FR, o0c = tc * FC;
    const int gr0 = 2 * o0r - F / 2 + 1, gc0 = 2 * o0c - F / 2 + 1;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const float* x = a.in + (int64_t)b * a.in_bs;
    WTP_FPROBE(0);
    /* 1. input tile with the periodic (odd: repeat-last) extension applied on load.  Rows
     *    go by wave (row index and extension are scalar work), columns by lane (a plain add
     *    except on edge tiles); for the specialised filters the trip counts are compile-time,
     *    so every load of a thread is issued before the first LDS write. */
    {
        const bool cin = gc0 >= 0 && gc0 + NC <= a.C; /* no column extension in this tile */
        auto rowptr = [&](int rr) {
            const int gr = gr0 + rr;
            return x + (int64_t)((gr >= 0 && gr < a.R) ? gr : ext_idx(gr, a.R)) * a.C;
        };
        auto colidx = [&](int cc) {
            const int gc = gc0 + cc;
            return cin ? gc : ((gc >= 0 && gc < a.C) ? gc : ext_idx(gc, a.C));
        };
        if constexpr (FT > 0) {
            constexpr int NRc = 2 * FR + FT - 2, NCc = 2 * FC + FT - 2;
            constexpr int S0 = FWD_S0<FT>, TP = FWD_TP<FT>, W4 = TP / 4;
            const int start = gc0 - S0; /* 16-byte aligned column of the tile's first float4 */
            if (a.al16 && gr0 >= 0 && gr0 + NRc <= a.R && start >= 0 && start + TP <= a.C) {
                /* interior tile: whole float4 rows [start, start + TP), every load of a thread in
                 * flight before its first LDS write (ds_write_b128) */
                constexpr int NE = NRc * W4, K = (NE + FB_THREADS - 1) / FB_THREADS;
                const float* x0 = x + (int64_t)gr0 * a.C + start;
                float4 q[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int e = min(k * FB_THREADS + (int)threadIdx.x, NE - 1);
                    const int rr = e / W4, j4 = e - rr * W4;
                    q[k] = *reinterpret_cast<const float4*>(x0 + (int64_t)rr * a.C + 4 * j4);
                }
                /* stored at the same clamped index it was loaded from (a duplicate of element
                 * NE - 1 rewrites its own value): no predicate, so the compiler cannot sink a
                 * load into a branch behind its own wait */
#pragma unroll
                for (int k = 0; k < K; ++k)
                    reinterpret_cast<float4*>(T)[min(k * FB_THREADS + (int)threadIdx.x, NE - 1)] = q[k];
            } else {
                constexpr int RW = (NRc + 3) / 4, CW = (NCc + 63) / 64; /* rows per wave, column chunks */
                int col[CW];
#pragma unroll
                for (int c = 0; c < CW; ++c) col[c] = colidx(min(lane + 64 * c, NCc - 1));
                float v[RW][CW];
#pragma unroll
                for (int k = 0; k < RW; ++k) {
                    const float* xr = rowptr(min(wv + 4 * k, NRc - 1));
#pragma unroll
                    for (int c = 0; c < CW; ++c) v[k][c] = xr[col[c]];
                }
#pragma unroll
                for (int k = 0; k < RW; ++k)
#pragma unroll
                    for (int c = 0; c < CW; ++c) /* clamped like the loads: duplicates rewrite their own value */
                        T[min(wv + 4 * k, NRc - 1) * TP + S0 + min(lane + 64 * c, NCc - 1)] = v[k][c];
            }
        } else {
            for (int rr = wv; rr < NR; rr += FB_THREADS / 64) {
                const float* xr = rowptr(rr);
                for (int cc = lane; cc < NC; cc += 64) T[rr * NC + cc] = xr[colidx(cc)];
            }
        }
    }
    __syncthreads();
    WTP_FPROBE(1);
    /* 2. axis -2 analysis of every tile column: L, H for the tile's output rows */
    const float* flo = tp.f[0];
    const float* fhi = tp.f[1];
    const int nrow = min(FR, a.Ro - o0r);
    if constexpr (FT > 0) {
        /* one tile column and FR/2 consecutive output rows per item: the column's
         * FR + F - 2 samples are read once into registers and shared by the rows */
        constexpr int RH = FR / 2, NV = 2 * RH + FT - 2, NCc = 2 * FC + FT - 2;
        constexpr int NIT = (2 * NCc + FB_THREADS - 1) / FB_THREADS;
        f2 res[NIT][RH];
#pragma unroll
        for (int q = 0; q < NIT; ++q) {
            const int it = threadIdx.x + q * FB_THREADS;
            if (it < 2 * NCc) {
                const int h = it >= NCc, cc = it - h * NCc;
                float v[NV];
#pragma unroll
                for (int k = 0; k < NV; ++k) v[k] = T[(2 * RH * h + k) * FWD_TP<FT> + FWD_S0<FT> + cc];
                const int i0 = FT / 2 + 2 * (o0r + RH * h);
                if (__all(i0 + 2 * (RH - 1) < a.R)) {
                    /* all RH outputs interior: tap-major, so the RH independent sums interleave */
#pragma unroll
                    for (int r = 0; r < RH; ++r) res[q][r] = f2{0.0f, 0.0f};
#pragma unroll
                    for (int j = 0; j < FT; ++j) {
                        const f2 t = {flo[j], fhi[j]};
#pragma unroll
                        for (int r = 0; r < RH; ++r) res[q][r] = res[q][r] + t * v[2 * r + FT - 1 - j];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < RH; ++r)
                        res[q][r] = ana2_j<FT>(i0 + 2 * r, a.R, flo, fhi, [&](int j) { return v[2 * r + FT - 1 - j]; });
                }
            }
        }
        __syncthreads(); /* every read of T is done: LH overwrites it */
#pragma unroll
        for (int q = 0; q < NIT; ++q) {
            const int it = threadIdx.x + q * FB_THREADS;
            if (it < 2 * NCc) {
                const int h = it >= NCc, cc = it - h * NCc;
#pragma unroll
                for (int r = 0; r < RH; ++r)
                    if (RH * h + r < nrow) LH[lhi(RH * h + r, cc)] = make_float2(res[q][r].x, res[q][r].y);
            }
        }
    } else {
        for (int o = wv; o < nrow; o += FB_THREADS / 64) {
            const int i = F / 2 + 2 * (o0r + o);
            for (int cc = lane; cc < NC; cc += 64) {
                const f2 r = ana2<FT>(i, a.R, F, flo, fhi, [&](int g) { return T[(g - gr0) * NC + cc]; });
                LH[lhi(o, cc)] = make_float2(r.x, r.y);
            }
        }
    }
    __syncthreads();
    WTP_FPROBE(2);
    /* 3. axis -1 analysis of the L and H rows -> aa, ad, da, dd (packed layout) */
    float* Pb = a.P + (int64_t)b * a.P_bs;
    const int oc = o0c + lane;
    if (lane < FC && oc < a.Co) {
        const int i = F / 2 + 2 * oc;
        auto put = [&](int o, f2 low, f2 high) { /* low = (aa, da), high = (ad, dd) */
            const int r = o0r + o;
            if (a.last) Pb[(int64_t)r * a.PC + oc] = low.x;
            else a.anext[((int64_t)b * a.Ro + r) * a.Co + oc] = low.x;
            Pb[(int64_t)r * a.PC + a.offC + oc] = high.x;
            Pb[(int64_t)(a.offR + r) * a.PC + oc] = low.y;
            Pb[(int64_t)(a.offR + r) * a.PC + a.offC + oc] = high.y;
        };
        bool done = false;
        if constexpr (FT > 0) {
            if (nrow == FR && __all(i < a.C)) {
                /* full tile, interior columns: two rows at a time, their four sums interleaved */
                constexpr int NW = FB_THREADS / 64;
                static_assert(FR % (2 * NW) == 0, "row pairs per wave");
#pragma unroll
                for (int pr = 0; pr < FR / (2 * NW); ++pr) {
                    const int oA = wv + 2 * NW * pr, oB = oA + NW;
                    f2 vA[FT], vB[FT];
#pragma unroll
                    for (int j = 0; j < FT; ++j) {
                        const float2 xa = LH[lhi(oA, i - j - gc0)], xb = LH[lhi(oB, i - j - gc0)];
                        vA[j] = f2{xa.x, xa.y};
                        vB[j] = f2{xb.x, xb.y};
                    }
                    f2 aA = {0.0f, 0.0f}, dA = {0.0f, 0.0f}, aB = {0.0f, 0.0f}, dB = {0.0f, 0.0f};
#pragma unroll
                    for (int j = 0; j < FT; ++j) {
                        aA = aA + flo[j] * vA[j];
                        dA = dA + fhi[j] * vA[j];
                        aB = aB + flo[j] * vB[j];
                        dB = dB + fhi[j] * vB[j];
                    }
                    put(oA, aA, dA);
                    put(oB, aB, dB);
                }
                done = true;
            }
        }
        for (int o = wv; !done && o < nrow; o += FB_THREADS / 64) {
            f2 low, high;
            ana2x2<FT>(i, a.C, F, flo, fhi,
                       [&](int g) {
                           const float2 v = LH[lhi(o, g - gc0)];
                           return f2{v.x, v.y};
                       },
                       low, high);
            put(o, low, high);
        }
    }
    WTP_FPROBE(3);
}

/* One analysis level over the INTERIOR tiles of a group (FwdGroup geo: tr0/nTR/tc0/nTC): every
 * tile's input window lies inside the image and its float4 rows are aligned, every output is a
 * full-tile interior site (i < N: ascending taps), so none of k_fwd_level's edge forms is compiled
 * in.  EDGE: the same kernel over the FRAME of tiles around that rectangle (FwdArgs.frame's decode):
 * the input tile gathered with the periodic (odd: repeat-last) extension as k_fwd_level loads it,
 * pywt's split order (wrapped terms first, wt_ana_point) only in the waves holding an output site
 * i >= N, stores masked to the level's extent.  Same sums in the same order (pywt's
 * ascending-tap interior form, every sum from 0 as pywt starts it, so even the sign of a zero
 * matches).  Instruction shape:
 *   column pass: a thread's column samples are read as PAIRS of consecutive rows into aligned
 *   register pairs, so the packed multiply broadcasts either sample by op_sel (no realigning
 *   move), against the {lo[j], hi[j]} tap pair in one SGPR pair;
 *   row pass: as k_fwd_level's interior form; stores by buffer instructions whose row offset is a
 *   scalar (the row is wave-uniform) and column offset the lane's -- no 64-bit address math. */
template <int FT, bool EDGE>
__global__ __launch_bounds__(FB_THREADS) WTP_FB_INT_WPE void k_fwd_int(FwdGroup g, FwdIntTaps tp, FwdSel fs) {
    static_assert(FT > 0 && FT % 2 == 0, "specialised even filters");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int NRc = 2 * FR + FT - 2, NCc = 2 * FC + FT - 2;
    constexpr int S0 = FWD_S0<FT>, TP = FWD_TP<FT>, W4 = TP / 4;
    constexpr int HALF = fwd_lhh(NCc);
    static_assert(HALF % 16 == 8 && HALF >= (NCc + 1) / 2, "LH half pitch");
    float* T = lds;
    float2* LH = reinterpret_cast<float2*>(lds);
    const int gt = xcd_tile(blockIdx.x, gridDim.x);
    const int item = fdiv(gt, g.dv_tiles);
    const FwdArgs& a = g.geo;
    const int tile = gt - item * g.tiles;
    int b, trow, tcol;
    if constexpr (EDGE) {
        const int per = a.tilesR * a.tilesC - a.nTR * a.nTC;
        b = fdiv(tile, g.dv_per);
        frame_tile_fd(tile - b * per, a.tilesC, a.tr0, a.nTR, a.tc0, a.nTC, g.dv_tc, g.dv_side, &trow, &tcol);
    } else {
        const int per = a.nTR * a.nTC;
        b = fdiv(tile, g.dv_per);
        const int t2 = tile - b * per, trr = fdiv(t2, g.dv_ntc);
        trow = a.tr0 + trr;
        tcol = a.tc0 + t2 - trr * a.nTC;
    }
    const int o0r = trow * FR, o0c = tcol * FC;
    const int gr0 = 2 * o0r - FT / 2 + 1, gc0 = 2 * o0c - FT / 2 + 1;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const float* x = g.in[item] + (int64_t)b * a.in_bs;
    /* fused selection (FwdSel): the window of the item's segment, by scalar loads in flight with
     * the tile's, and the wave's slot */
    const bool fsel = fs.on != 0;
    uint32_t skl = 0, sspan = 0;
    FslHeader* sst = nullptr;
    uint32_t* wslot = nullptr;
    if (fsel) {
        sst = fs.hdr[item];
        skl = sst->kl;
        sspan = sst->kh - skl;
        wslot = fs.slots[item] + ((int64_t)tile * (FB_THREADS / 64) + wv) * FSL_WORDS;
    }
    WTP_FPROBE(0);
    /* 1. the input tile; every load of a thread in flight before its first LDS write */
    if (EDGE && a.al16 && !(a.R & 1) && a.R >= NRc && a.C >= TP) {
        /* a frame tile of an even, aligned level: the interior kernel's float4 rows, each row and
         * each float4 wrapped once (C % 4 == 0 and the tile's first column is 16-byte aligned, so
         * a float4 lies wholly inside or wholly across the edge; periodic, no repeat-last) */
        constexpr int NE = NRc * W4, K = (NE + FB_THREADS - 1) / FB_THREADS;
        const int start = gc0 - S0;
        float4 q[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int e = min(k * FB_THREADS + (int)threadIdx.x, NE - 1);
            const int rr = e / W4, j4 = e - rr * W4;
            int r = gr0 + rr, c = start + 4 * j4;
            r = r < 0 ? r + a.R : (r >= a.R ? r - a.R : r);
            c = c < 0 ? c + a.C : (c >= a.C ? c - a.C : c);
            q[k] = *reinterpret_cast<const float4*>(x + (int64_t)r * a.C + c);
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            reinterpret_cast<float4*>(T)[min(k * FB_THREADS + (int)threadIdx.x, NE - 1)] = q[k];
    } else if constexpr (EDGE) {
        /* rows by wave (row index and extension are scalar work), columns by lane; clamped
         * duplicates rewrite their own value */
        constexpr int RW = (NRc + 3) / 4, CW = (NCc + 63) / 64;
        int col[CW];
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            const int gc = gc0 + min(lane + 64 * c, NCc - 1);
            col[c] = (gc >= 0 && gc < a.C) ? gc : ext_idx(gc, a.C);
        }
        float v[RW][CW];
#pragma unroll
        for (int k = 0; k < RW; ++k) {
            const int gr = gr0 + min(wv + 4 * k, NRc - 1);
            const float* xr = x + (int64_t)((gr >= 0 && gr < a.R) ? gr : ext_idx(gr, a.R)) * a.C;
#pragma unroll
            for (int c = 0; c < CW; ++c) v[k][c] = xr[col[c]];
        }
#pragma unroll
        for (int k = 0; k < RW; ++k)
#pragma unroll
            for (int c = 0; c < CW; ++c) T[min(wv + 4 * k, NRc - 1) * TP + S0 + min(lane + 64 * c, NCc - 1)] = v[k][c];
    } else {
        /* whole float4 rows from the aligned column gc0 - S0: buffer loads over the tile's rows, a
         * 32-bit offset each (fwd_interior bounds the tile's span below 2^31 bytes) */
        constexpr int NE = NRc * W4, K = (NE + FB_THREADS - 1) / FB_THREADS;
        const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(x) + (int64_t)gr0 * a.C + (gc0 - S0), 0, 4 * ((NRc - 1) * a.C + TP), 0x00020000);
        float4 q[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int e = min(k * FB_THREADS + (int)threadIdx.x, NE - 1);
            const int rr = e / W4, j4 = e - rr * W4;
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            const u4 w = __builtin_amdgcn_raw_buffer_load_b128(rX, 4 * (rr * a.C + 4 * j4), 0, 0);
            q[k] = make_float4(__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z), __uint_as_float(w.w));
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            reinterpret_cast<float4*>(T)[min(k * FB_THREADS + (int)threadIdx.x, NE - 1)] = q[k];
    }
    __syncthreads();
    WTP_FPROBE(1);
    /* 2. axis -2: one tile column and FR/2 consecutive output rows per item; item it = h HP + cc, with
     * HP a multiple of 64 when NC fits in 128 (F <= 18): no wave holds items of both halves, whose
     * column reads 2 RH rows apart would otherwise share LDS banks (round 6, with the LH pitch) */
    constexpr int RH = FR / 2, NV = 2 * RH + FT - 2, NP = NV / 2;
    constexpr int HP = NCc <= 128 ? 128 : NCc;
    constexpr int NIT = (2 * HP + FB_THREADS - 1) / FB_THREADS;
    static_assert(NV % 2 == 0, "sample pairs");
    f2 res[NIT][RH];
#pragma unroll
    for (int q = 0; q < NIT; ++q) {
        const int it = threadIdx.x + q * FB_THREADS;
        const int h = it >= HP, cc = it - h * HP;
        if (it < 2 * HP && cc < NCc) {
            const float* col = T + (2 * RH * h) * TP + S0 + cc;
            f2 P[NP];
#pragma unroll
            for (int m = 0; m < NP; ++m) P[m] = f2{col[(2 * m) * TP], col[(2 * m + 1) * TP]};
            auto smp = [&](int s) { return (s & 1) ? P[s >> 1].yy : P[s >> 1].xx; };
            const int i0 = FT / 2 + 2 * (o0r + RH * h); /* the site of the item's first output row */
            if (!EDGE || __all(i0 + 2 * (RH - 1) < a.R)) {
#pragma unroll
                for (int r = 0; r < RH; ++r) res[q][r] = f2{0.0f, 0.0f} + tp.t[0] * smp(2 * r + FT - 1);
#pragma unroll
                for (int j = 1; j < FT; ++j)
#pragma unroll
                    for (int r = 0; r < RH; ++r) res[q][r] = res[q][r] + tp.t[j] * smp(2 * r + FT - 1 - j);
            } else {
                /* wt_ana_point's order: the wrapped terms (i - j >= N) by descending j, then the
                 * rest ascending -- for a site i < N that is the ascending interior sum */
#pragma unroll
                for (int r = 0; r < RH; ++r) {
                    const int i = i0 + 2 * r;
                    f2 acc = {0.0f, 0.0f};
#pragma unroll
                    for (int j = FT - 1; j >= 0; --j)
                        if (i - j >= a.R) acc = acc + tp.t[j] * smp(2 * r + FT - 1 - j);
#pragma unroll
                    for (int j = 0; j < FT; ++j)
                        if (i - j < a.R) acc = acc + tp.t[j] * smp(2 * r + FT - 1 - j);
                    res[q][r] = acc;
                }
            }
        }
    }
    __syncthreads(); /* every read of T is done: LH overwrites it */
    auto lhi = [&](int o, int cc) { return o * (2 * HALF) + (cc & 1) * HALF + (cc >> 1); };
#pragma unroll
    for (int q = 0; q < NIT; ++q) {
        const int it = threadIdx.x + q * FB_THREADS;
        const int h = it >= HP, cc = it - h * HP;
        if (it < 2 * HP && cc < NCc) {
#pragma unroll
            for (int r = 0; r < RH; ++r) LH[lhi(RH * h + r, cc)] = make_float2(res[q][r].x, res[q][r].y);
        }
    }
    __syncthreads();
    WTP_FPROBE(2);
    /* 3. axis -1 of the L and H rows -> aa, ad, da, dd; two rows per step, four sums interleaved */
    constexpr int NW = FB_THREADS / 64, NPR = FR / (2 * NW);
    static_assert(FR % (2 * NW) == 0, "row pairs per wave");
    auto flo = [&](int k) { return (k & 1) ? tp.t[k >> 1].y : tp.t[k >> 1].x; };
    /* EDGE: the outputs whose site wraps past the row's end (ic >= C: the level's last F/4 or so
     * columns) are skipped by the uniform pass and computed in wt_ana_point's split order by a
     * compact fix-up: lane e of the wave = (its row e / nsc, the (e % nsc)-th such column) */
    uint64_t fxm = 0;
    if constexpr (EDGE) {
        const int ic = FT / 2 + 2 * (o0c + lane);
        fxm = __ballot(lane < FC && ic >= a.C && o0c + lane < a.Co);
    }
    /* fused selection: every coefficient the wave writes to P is classified against the window
     * [kl, kh] as k_collect classifies a chunk: keys < kl and == kl counted (ballot popcounts), the
     * largest key kept, the keys inside (kl, kh] appended to the wave's slot in write order.  Every
     * lane of the row pass takes every call (ok = the output exists), so the running count stays
     * the same in all of them. */
    uint32_t f_below = 0, f_eq = 0, f_cnt = 0, f_mx = 0;
    /* keys <= kl are counted together as "below" (one compare a key): the select then sees no key
     * at kl, so a rank at or under kl -- ties at the window's lower edge -- reads as a miss and is
     * retried over P, exactly.  The largest key is kept three at a time (fmax3). */
    auto fcls = [&](float v, bool ok) {
        const uint32_t k = __float_as_uint(v) & 0x7FFFFFFFu;
        f_below += (uint32_t)__popcll(__ballot(ok && k <= skl));
        const bool in = ok && k - skl - 1u < sspan;
        const uint64_t m = __ballot(in);
        if (m) {
            const uint32_t pos = f_cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (in && pos < (uint32_t)FSL_KEYS) wslot[1 + pos] = k;
            f_cnt += (uint32_t)__popcll(m);
        }
    };
    auto fmax3 = [&](float a, float b, float c, bool ok) {
        const uint32_t m3 = max(max(__float_as_uint(a) & 0x7FFFFFFFu, __float_as_uint(b) & 0x7FFFFFFFu),
                                __float_as_uint(c) & 0x7FFFFFFFu);
        f_mx = ok ? max(f_mx, m3) : f_mx;
    };
    if (lane < FC) {
        const __amdgpu_buffer_rsrc_t rP =
            __builtin_amdgcn_make_buffer_rsrc(g.P[item] + (int64_t)b * a.P_bs, 0, (int)(4 * a.P_bs), 0x00020000);
        const __amdgpu_buffer_rsrc_t rA = a.last ? rP
            : __builtin_amdgcn_make_buffer_rsrc(g.anext[item] + (int64_t)b * a.Ro * a.Co, 0, 4 * a.Ro * a.Co, 0x00020000);
        const int pitchA = a.last ? a.PC : a.Co;
        const int voff = 4 * (o0c + lane);
        const int ic = FT / 2 + 2 * (o0c + lane); /* the lane's output site along the row */
        const bool cin = !EDGE || (o0c + lane < a.Co && ic < a.C);
#pragma unroll
        for (int pr = 0; pr < NPR; ++pr) {
            const int oA = wv + 2 * NW * pr, oB = oA + NW;
            f2 vA[FT], vB[FT];
#pragma unroll
            for (int j = 0; j < FT; ++j) { /* sample cc = 2 lane + FT - 1 - j of the row */
                const float2 xa = LH[lhi(oA, 2 * lane + FT - 1 - j)], xb = LH[lhi(oB, 2 * lane + FT - 1 - j)];
                vA[j] = f2{xa.x, xa.y};
                vB[j] = f2{xb.x, xb.y};
            }
            const f2 z2 = {0.0f, 0.0f};
            f2 aA, dA, aB, dB;
            aA = z2 + flo(0) * vA[0];
            dA = z2 + flo(1) * vA[0];
            aB = z2 + flo(0) * vB[0];
            dB = z2 + flo(1) * vB[0];
#pragma unroll
            for (int j = 1; j < FT; ++j) {
                const float tl = flo(2 * j), th = flo(2 * j + 1);
                aA = aA + tl * vA[j];
                dA = dA + th * vA[j];
                aB = aB + tl * vB[j];
                dB = dB + th * vB[j];
            }
            /* low = (aa, da), high = (ad, dd) */
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int r = o0r + (u ? oB : oA);
                const bool ok = !EDGE || (cin && r < a.Ro);
                const f2 lw = u ? aB : aA, hg = u ? dB : dA;
                if (fsel) {
                    fcls(hg.x, ok);
                    fcls(lw.y, ok);
                    fcls(hg.y, ok);
                    fmax3(hg.x, lw.y, hg.y, ok);
                    if (a.last) { fcls(lw.x, ok); fmax3(lw.x, lw.x, lw.x, ok); }
                }
                if (!ok) continue;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lw.x), rA, voff, 4 * r * pitchA, 0);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hg.x), rP, voff, 4 * (r * a.PC + a.offC), 0);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lw.y), rP, voff, 4 * ((a.offR + r) * a.PC), 0);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hg.y), rP, voff, 4 * ((a.offR + r) * a.PC + a.offC), 0);
            }
        }
    }
    if (EDGE && fxm) { /* uniform */
        const int nsc = __builtin_popcountll(fxm);
        /* the fix-up lanes are row-pass lanes (lane < FC): their running slot count is current */
        static_assert(2 * NPR * (FT / 4 + 2) <= FC, "one fix-up pass per wave");
        if (lane < 2 * NPR * nsc) {
            const int rs = lane / nsc, ci = lane - rs * nsc;
            uint64_t mm = fxm;
            for (int t = 0; t < ci; ++t) mm &= mm - 1ull;
            const int cl = __builtin_ctzll(mm); /* the column's lane in the uniform pass */
            const int o = wv + NW * rs;       /* the wave's rows: wv + NW * (2 pr + u) */
            const int r = o0r + o;
            {
                const bool ok = r < a.Ro;
                const int ic = FT / 2 + 2 * (o0c + cl);
                f2 v[FT];
#pragma unroll
                for (int j = 0; j < FT; ++j) { const float2 xv = LH[lhi(o, 2 * cl + FT - 1 - j)]; v[j] = f2{xv.x, xv.y}; }
                f2 lw = {0.0f, 0.0f}, hg = {0.0f, 0.0f};
                auto term = [&](int j) { lw = lw + flo(2 * j) * v[j]; hg = hg + flo(2 * j + 1) * v[j]; };
#pragma unroll
                for (int j = FT - 1; j >= 0; --j)
                    if (ic - j >= a.C) term(j);
#pragma unroll
                for (int j = 0; j < FT; ++j)
                    if (ic - j < a.C) term(j);
                const __amdgpu_buffer_rsrc_t rP =
                    __builtin_amdgcn_make_buffer_rsrc(g.P[item] + (int64_t)b * a.P_bs, 0, (int)(4 * a.P_bs), 0x00020000);
                const __amdgpu_buffer_rsrc_t rA = a.last ? rP
                    : __builtin_amdgcn_make_buffer_rsrc(g.anext[item] + (int64_t)b * a.Ro * a.Co, 0, 4 * a.Ro * a.Co, 0x00020000);
                const int pitchA = a.last ? a.PC : a.Co;
                const int vo = 4 * (o0c + cl);
                if (fsel) {
                    fcls(hg.x, ok);
                    fcls(lw.y, ok);
                    fcls(hg.y, ok);
                    fmax3(hg.x, lw.y, hg.y, ok);
                    if (a.last) { fcls(lw.x, ok); fmax3(lw.x, lw.x, lw.x, ok); }
                }
                if (ok) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lw.x), rA, vo, 4 * r * pitchA, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hg.x), rP, vo, 4 * (r * a.PC + a.offC), 0);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lw.y), rP, vo, 4 * ((a.offR + r) * a.PC), 0);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hg.y), rP, vo, 4 * ((a.offR + r) * a.PC + a.offC), 0);
                }
            }
        }
    }
    if (fsel) { /* the wave's slot count (lane 0 took every call); the workgroup's counters */
        __shared__ uint32_t s_fc[FB_THREADS / 64][3];
        uint32_t mx = f_mx;
#pragma unroll
        for (int o = 32; o; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        if (lane == 0) {
            wslot[0] = f_cnt;
            s_fc[wv][0] = f_below;
            s_fc[wv][1] = f_eq;
            s_fc[wv][2] = mx;
            if (f_cnt > (uint32_t)FSL_KEYS) atomicOr(&sst->overflow, 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t b = 0, e = 0, m = 0;
#pragma unroll
            for (int w = 0; w < FB_THREADS / 64; ++w) { b += s_fc[w][0]; e += s_fc[w][1]; m = max(m, s_fc[w][2]); }
            const int sh8 = blockIdx.x & (NSHARD - 1);
            if (b | e) atomicAdd(&sst->be[sh8], ((unsigned long long)e << 32) | b);
            if (m) atomicMax(&sst->maxkey[sh8], m);
        }
    }
    WTP_FPROBE(3);
}

/* ------------------------------------------------------------ synthesis --- */
struct InvArgs {
    const float* a;      /* approximation (B, R, C) with row pitch lda, batch stride a_bs */
    int64_t a_bs;
    int lda, a_from_P;   /* a_from_P: the approximation is the packed cA (thresholded) */
    const float* P;
    int64_t P_bs;
    int PC, offR, offC;
    int R, C;            /* coefficient dims of this level */
    float* y;            /* output (B, outH, outW), row pitch outW */
    int outH, outW;
    const float* thr;    /* per-tensor float32 threshold applied to packed coefficients */
    unsigned long long* zc;
    int tilesC, tilesR;
    int tr0, nTR, tc0, nTC, frame; /* as FwdArgs: k_inv_int's rectangle, k_inv_level's frame */
};

/* the inverse's items of one geometry: per item its approximation source, packed array and output,
 * and its threshold / zero-count words as element offsets from the geometry's thr / zc (every
 * tensor of a call has them in one array) */
__host__ __device__ inline int thr_off_of(int32_t v) { return (int)(int16_t)(v & 0xFFFF); }
__host__ __device__ inline int zc_off_of(int32_t v) { return (int)(v >> 16); }
struct InvGroup {
    InvArgs geo;
    int n, tiles;
    FastDiv dv_tiles, dv_per, dv_ntc; /* as FwdGroup */
    FastDiv dv_tc, dv_side;
    const float* a[FB_UNI];
    const float* P[FB_UNI];
    float* y[FB_UNI];
    /* threshold (low 16 bits) and zero-count (high 16 bits) word offsets, signed, packed in one
     * 32-bit element: a scalar load (a 16-bit kernarg element is a vector load and a wait) */
    int32_t tz_off[FB_UNI];
};

template <int FT>
__global__ __launch_bounds__(FB_THREADS) WTP_FB_INV_WPE void k_inv_level(InvGroup g, TapsT<FT> tp) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int gt = xcd_tile(blockIdx.x, gridDim.x);
    const int F = FT ? FT : tp.F;
    const int H = F / 2;
    const int item = gt / g.tiles;
    InvArgs a = g.geo;
    a.a = g.a[item];
    a.P = g.P[item];
    a.y = g.y[item];
    a.thr = a.thr ? a.thr + thr_off_of(g.tz_off[item]) : nullptr;
    a.zc = a.zc ? a.zc + zc_off_of(g.tz_off[item]) : nullptr;
    const int tile = gt - item * g.tiles;
    int tc, tr, b;
    if (a.frame) {
        const int per = a.tilesR * a.tilesC - a.nTR * a.nTC;
        b = tile / per;
        frame_tile(tile - b * per, a.tilesC, a.tr0, a.nTR, a.tc0, a.nTC, &tr, &tc);
    } else {
        tc = tile % a.tilesC;
        tr = (tile / a.tilesC) % a.tilesR;
        b = tile / (a.tilesC * a.tilesR);
    }
    const int n0 = tr * IR, m0 = tc * IC;
    const int nl = min(n0 + IR, a.outH) - 1, ml = min(m0 + IC, a.outW) - 1;
    const int r_lo = site_u(n0, a.R, F).iu - H + 1, r_hi = site_u(nl, a.R, F).iu;
    const int c_lo = site_u(m0, a.C, F).iu - H + 1, c_hi = site_u(ml, a.C, F).iu;
    const int NRr = r_hi - r_lo + 1, NCc = c_hi - c_lo + 1;
    float2* Aq = reinterpret_cast<float2*>(lds);  /* (cA, cH=da) at each tile position  */
    float2* Dq = Aq + NRr * NCc;                  /* (cV=ad, cD=dd)                     */
    /* NRr x IC: (lo, hi) row-pass output; specialised filters keep their rows in registers
     * across a barrier and write them over Aq/Dq (half the LDS per workgroup) */
    float2* LoHi = FT > 0 ? Aq : Dq + NRr * NCc;
    const float thr = a.thr ? *a.thr : 0.0f;      /* |c| < 0 never holds: no threshold  */
    auto tl = [&](float c) { return (fabsf(c) < thr) ? 0.0f : c; };
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const float* Pb = a.P + (int64_t)b * a.P_bs;
    const float* ab = a.a + (int64_t)b * a.a_bs;
    WTP_FPROBE(0);
    /* 1. the four coefficient tiles (periodic wrap, thresholded on load); all loads of a
     *    thread issued before the LDS writes (compile-time trip count) */
    {
        /* a tile's coefficient rows / columns: NRr <= IR/2 + H, NCc <= IC/2 + H (its IR outputs sit on
         * IR/2 consecutive synthesis sites; the H-even special last output n = 2N - 1 included) */
        constexpr int NR_MAX = IR / 2 + (FT ? FT : 2) / 2, NC_MAX = IC / 2 + (FT ? FT : 2) / 2;
        const bool inner = r_lo >= 0 && r_hi < a.R && c_lo >= 0 && c_hi < a.C;
        auto load4 = [&](int rr, int cc, float4& q) {
            const int r = inner ? r_lo + rr : pmod32(r_lo + rr, a.R), c = inner ? c_lo + cc : pmod32(c_lo + cc, a.C);
            const float* prow = Pb + (int64_t)r * a.PC;
            const float* drow = Pb + (int64_t)(a.offR + r) * a.PC;
            const float va = a.a_from_P ? prow[c] : ab[(int64_t)r * a.lda + c];
            q = make_float4(va, prow[a.offC + c], drow[c], drow[a.offC + c]); /* cA, cV=ad, cH=da, cD=dd */
        };
        auto store4 = [&](int rr, int cc, float4 q) {
            const float va = a.a_from_P ? tl(q.x) : q.x;
            Aq[rr * NCc + cc] = make_float2(va, tl(q.z));
            Dq[rr * NCc + cc] = make_float2(tl(q.y), tl(q.w));
        };
        if (FT) {
            constexpr int K = (NR_MAX * NC_MAX + FB_THREADS - 1) / FB_THREADS;
            float4 q[K];
#pragma unroll
            for (int k = 0; k < K; ++k) { /* unconditional (clamped) loads: no per-load wait */
                const int e = k * FB_THREADS + threadIdx.x;
                const int rr = e / NC_MAX, cc = e - rr * NC_MAX;
                load4(min(rr, NRr - 1), min(cc, NCc - 1), q[k]);
            }
            /* stored at the clamped position it was loaded from (duplicates rewrite their own
             * value): no predicate, so no load is sunk into a branch behind its own wait */
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int e = k * FB_THREADS + threadIdx.x;
                const int rr = e / NC_MAX, cc = e - rr * NC_MAX;
                store4(min(rr, NRr - 1), min(cc, NCc - 1), q[k]);
            }
        } else {
            for (int e = threadIdx.x; e < NRr * NCc; e += FB_THREADS) {
                const int rr = e / NCc, cc = e - rr * NCc;
                float4 q;
                load4(rr, cc, q);
                store4(rr, cc, q);
            }
        }
    }
    __syncthreads();
    WTP_FPROBE(1);
    /* 2. axis -1 synthesis of every tile row: lo = rec(cA, cV), hi = rec(cH, cD), carried
     *    packed as (lo, hi): rec_lo over (cA, cH), then rec_hi over (cV, cD).  Each lane's
     *    taps (its output parity) are resolved into registers once. */
    const float* rlo = tp.f[2];
    const float* rhi = tp.f[3];
    constexpr int HM = FT ? FT / 2 : 1;
    const int m = m0 + lane;
    /* rows per wave: a tile's coefficient rows NRr = r_hi - r_lo + 1 <= IR/2 + H (the sites of
     * IR consecutive outputs span IR/2 positions; H even: exactly IR/2 + H) */
    constexpr int RRN = (IR / 2 + HM + 3) / 4;
    f2 rowres[FT ? RRN : 1];
    if (lane < IC && m <= ml) {
        const SiteU s = site_u(m, a.C, F);
        auto getA = [&](int rr) {
            return [&, rr](int g) { const float2 v = Aq[rr * NCc + (g - c_lo)]; return f2{v.x, v.y}; };
        };
        auto getD = [&](int rr) {
            return [&, rr](int g) { const float2 v = Dq[rr * NCc + (g - c_lo)]; return f2{v.x, v.y}; };
        };
        if (FT) {
            float tlo[HM], thi[HM];
#pragma unroll
            for (int j = 0; j < HM; ++j) {
                const float l0 = rlo[2 * j], l1 = rlo[2 * j + 1], h0 = rhi[2 * j], h1 = rhi[2 * j + 1];
                tlo[j] = s.par ? l1 : l0;
                thi[j] = s.par ? h1 : h0;
            }
            auto tl_ = [&](int j) { return tlo[j]; };
            auto th_ = [&](int j) { return thi[j]; };
            if (__all(!s.special && s.i < a.C)) {
                /* interior columns: no branch between the rows (rows past NRr are clamped, computed
                 * and dropped at the write), so their independent sums interleave */
                /* INV_RG rows at a time, tap-major: their chains are independent, so they
                 * interleave instead of running one 2H-long dependent chain after another */
                constexpr int G = INV_RG;
#pragma unroll
                for (int q0 = 0; q0 < RRN; q0 += G) {
                    f2 acc[G], v[G][HM];
                    int rb[G];
#pragma unroll
                    for (int gq = 0; gq < G; ++gq) {
                        acc[gq] = f2{0.0f, 0.0f};
                        rb[gq] = min(wv + 4 * min(q0 + gq, RRN - 1), NRr - 1) * NCc + s.iu - c_lo;
                    }
                    /* each row's HM samples from ONE base address (the lowest), so the reads take
                     * immediate offsets (ds_read2_b64 offset0 / offset1) instead of an address each */
                    const float2* pa[G];
#pragma unroll
                    for (int gq = 0; gq < G; ++gq) pa[gq] = Aq + (rb[gq] - (HM - 1));
#pragma unroll
                    for (int gq = 0; gq < G; ++gq)
#pragma unroll
                        for (int j = 0; j < HM; ++j) {
                            const float2 t = pa[gq][HM - 1 - j];
                            v[gq][j] = f2{t.x, t.y};
                        }
#pragma unroll
                    for (int j = 0; j < HM; ++j)
#pragma unroll
                        for (int gq = 0; gq < G; ++gq)
                            if (q0 + gq < RRN) acc[gq] = acc[gq] + tlo[j] * v[gq][j];
#pragma unroll
                    for (int gq = 0; gq < G; ++gq)
#pragma unroll
                        for (int j = 0; j < HM; ++j) {
                            const float2 t = (pa[gq] + (Dq - Aq))[HM - 1 - j];
                            v[gq][j] = f2{t.x, t.y};
                        }
#pragma unroll
                    for (int j = 0; j < HM; ++j)
#pragma unroll
                        for (int gq = 0; gq < G; ++gq)
                            if (q0 + gq < RRN) acc[gq] = acc[gq] + thi[j] * v[gq][j];
#pragma unroll
                    for (int gq = 0; gq < G; ++gq)
                        if (q0 + gq < RRN) rowres[q0 + gq] = acc[gq];
                }
            } else {
#pragma unroll
                for (int q = 0; q < RRN; ++q) {
                    const int rr = wv + 4 * q;
                    if (rr < NRr) {
                        f2 acc = {0.0f, 0.0f};
                        acc = syn_pass_u<FT>(s, a.C, F, tl_, getA(rr), acc);
                        acc = syn_pass_u<FT>(s, a.C, F, th_, getD(rr), acc);
                        rowres[q] = acc;
                    }
                }
            }
        } else {
            auto tl_ = [&](int j) { return rlo[2 * j + s.par]; };
            auto th_ = [&](int j) { return rhi[2 * j + s.par]; };
            for (int rr = wv; rr < NRr; rr += FB_THREADS / 64) {
                f2 acc = {0.0f, 0.0f};
                acc = syn_pass_u<FT>(s, a.C, F, tl_, getA(rr), acc);
                acc = syn_pass_u<FT>(s, a.C, F, th_, getD(rr), acc);
                LoHi[rr * IC + lane] = make_float2(acc.x, acc.y);
            }
        }
    }
    if constexpr (FT > 0) {
        __syncthreads(); /* every read of Aq/Dq is done: LoHi overwrites them */
        if (lane < IC && m <= ml) {
#pragma unroll
            for (int q = 0; q < RRN; ++q)
                if (wv + 4 * q < NRr) LoHi[(wv + 4 * q) * IC + lane] = make_float2(rowres[q].x, rowres[q].y);
        }
    }
    __syncthreads();
    WTP_FPROBE(2);
    /* 3. axis -2 synthesis: y = rec_lo over lo, then rec_hi over hi, down each column (the
     *    site of a row is wave-uniform: scalar taps) */
    unsigned long long z = 0;
    if (lane < IC && m <= ml) {
        float* yb = a.y + (int64_t)b * a.outH * a.outW;
        /* specialised filters: each wave owns RB consecutive rows.  Interior blocks run from
         * registers: outputs k and k + RB/2 share taps (same parity) and sit four sites apart,
         * so they are computed packed, and each LoHi row is read from LDS once for the block
         * (H + RB/2 - 1 + E rows instead of H per output) */
        constexpr int RB = IR / (FB_THREADS / 64);
        const int nf = FT ? n0 + RB * wv : n0 + wv;
        const int nend = FT ? min(nf + RB - 1, nl) : nl;
        const int nstep = FT ? 1 : FB_THREADS / 64;
        bool fast = false;
        if constexpr (FT > 0) {
            constexpr int H = FT / 2, E = (H & 1) ? 0 : 1, NV = H + RB / 2 - 1 + E, RB2 = RB / 2;
            static_assert(RB % 4 == 0, "packed column blocks pair rows k and k + RB/2, RB/4 sites apart");
            const SiteU s0 = site_u(nf, a.R, F);
            const int nlast = nf + RB - 1;
            fast = nlast <= nl && !s0.special && (E == 0 || nlast < 2 * a.R - 1) &&
                              s0.i + ((RB - 1 + E) >> 1) < a.R;
            if (fast) {
                const int g0 = s0.i - H + 1 - r_lo;
                float2 r[NV];
#pragma unroll
                for (int q = 0; q < NV; ++q) r[q] = LoHi[(g0 + q) * IC + lane];
                /* tap-major over the RB2 output pairs: RB2 independent chains interleave, and
                 * each tap is read once per j (two parities) instead of once per output */
                f2 acc[RB2];
#pragma unroll
                for (int k = 0; k < RB2; ++k) acc[k] = f2{0.0f, 0.0f};
#pragma unroll
                for (int j = 0; j < H; ++j) {
                    const float t0 = rlo[2 * j], t1 = rlo[2 * j + 1];
#pragma unroll
                    for (int k = 0; k < RB2; ++k) {
                        const int par = (k + E) & 1, base = ((k + E) >> 1) + H - 1;
                        const float t = par ? t1 : t0;
                        acc[k] = acc[k] + f2{t, t} * f2{r[base - j].x, r[base - j + RB2 / 2].x};
                    }
                }
#pragma unroll
                for (int j = 0; j < H; ++j) {
                    const float t0 = rhi[2 * j], t1 = rhi[2 * j + 1];
#pragma unroll
                    for (int k = 0; k < RB2; ++k) {
                        const int par = (k + E) & 1, base = ((k + E) >> 1) + H - 1;
                        const float t = par ? t1 : t0;
                        acc[k] = acc[k] + f2{t, t} * f2{r[base - j].y, r[base - j + RB2 / 2].y};
                    }
                }
#pragma unroll
                for (int k = 0; k < RB2; ++k) {
                    yb[(int64_t)(nf + k) * a.outW + m] = acc[k].x;
                    yb[(int64_t)(nf + k + RB2) * a.outW + m] = acc[k].y;
                    z += (acc[k].x == 0.0f) + (acc[k].y == 0.0f);
                }
            }
        }
        for (int n = nf; !fast && n <= nend; n += nstep) {
            const SiteU s = site_u(n, a.R, F);
            auto tl_ = [&](int j) { return rlo[2 * j + s.par]; };
            auto th_ = [&](int j) { return rhi[2 * j + s.par]; };
            auto gl = [&](int g) { return LoHi[(g - r_lo) * IC + lane].x; };
            auto gh = [&](int g) { return LoHi[(g - r_lo) * IC + lane].y; };
            float acc = 0.0f;
            if (!s.special && s.i < a.R) {
                acc = syn_pass_inner<FT>(s, F, tl_, gl, acc);
                acc = syn_pass_inner<FT>(s, F, th_, gh, acc);
            } else {
                acc = syn_pass_u<FT>(s, a.R, F, tl_, gl, acc);
                acc = syn_pass_u<FT>(s, a.R, F, th_, gh, acc);
            }
            yb[(int64_t)n * a.outW + m] = acc;
            z += acc == 0.0f;
        }
    }
    if (a.zc) {
        __shared__ unsigned long long zs;
        if (threadIdx.x == 0) zs = 0;
        __syncthreads();
        if (z) atomicAdd(&zs, z);
        __syncthreads();
        if (threadIdx.x == 0 && zs) atomicAdd(a.zc, zs);
    }
    WTP_FPROBE(3);
}

/* One synthesis level over the INTERIOR tiles of a group (InvGroup geo: tr0/nTR/tc0/nTC): every
 * output of the tile is a full-tile non-special site whose coefficient window lies inside the
 * level (no wrap), so the tile's coefficient rows / columns are exactly IR/2 + H - (H & 1) and
 * only wt_syn_pass's ascending interior order occurs.  EDGE: the same kernel over the FRAME of tiles
 * around that rectangle (InvArgs.frame's decode; the host runs it when the level is at least a
 * window tall and wide, so one wrap brings every coefficient position into range): the window
 * loaded with the periodic wrap, wt_syn_pass's special / wrapped-first orders only where a site
 * needs them (the samples and taps are the interior ones -- unwrapped positions stay monotonic),
 * stores and zero counts masked to the output extent.
 * Same sums in the same order as k_inv_level's interior forms (from 0, as pywt).  Instruction shape: coefficient loads are buffer loads
 * whose four subband offsets are scalars (one lane offset per element), the row pass's per-lane
 * taps are register pairs broadcast by op_sel, the output stores take the row as a scalar
 * offset, and zeros are counted by ballot. */
template <int FT, bool EDGE>
__global__ __launch_bounds__(FB_THREADS) WTP_FB_INT_WPE void k_inv_int(InvGroup g, SmallTaps tp) {
    static_assert(FT > 0 && FT % 2 == 0, "specialised even filters");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int H = FT / 2, HM = H;
    constexpr int NR = IR / 2 + H - (H & 1), NC = IC / 2 + H - (H & 1); /* coefficient rows / columns */
    const int gt = xcd_tile(blockIdx.x, gridDim.x);
    const int item = fdiv(gt, g.dv_tiles);
    const InvArgs& a = g.geo;
    const int tile = gt - item * g.tiles;
    int b, trow, tcol;
    if constexpr (EDGE) {
        const int per = a.tilesR * a.tilesC - a.nTR * a.nTC;
        b = fdiv(tile, g.dv_per);
        frame_tile_fd(tile - b * per, a.tilesC, a.tr0, a.nTR, a.tc0, a.nTC, g.dv_tc, g.dv_side, &trow, &tcol);
    } else {
        const int per = a.nTR * a.nTC;
        b = fdiv(tile, g.dv_per);
        const int t2 = tile - b * per, trr = fdiv(t2, g.dv_ntc);
        trow = a.tr0 + trr;
        tcol = a.tc0 + t2 - trr * a.nTC;
    }
    const int n0 = trow * IR, m0 = tcol * IC;
    const int nl = min(n0 + IR, a.outH) - 1, ml = min(m0 + IC, a.outW) - 1; /* EDGE: the last stored output */
    const int r_lo = site_u(n0, a.R, FT).iu - H + 1, c_lo = site_u(m0, a.C, FT).iu - H + 1;
    float2* Aq = reinterpret_cast<float2*>(lds); /* (cA, cH=da) */
    float2* Dq = Aq + NR * NC;                   /* (cV=ad, cD=dd) */
    float2* LoHi = Aq;                           /* NR x IC, written over Aq/Dq after the row pass */
    const float* thrp = a.thr ? a.thr + thr_off_of(g.tz_off[item]) : nullptr;
    const float thr = thrp ? *thrp : 0.0f; /* |c| < 0 never holds: no threshold */
    auto tl = [&](float c) { return (fabsf(c) < thr) ? 0.0f : c; };
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    WTP_FPROBE(0);
    /* 1. the four coefficient tiles, thresholded on load: element e of the NR x NC window at
     *    lane offset (r_lo + rr) * PC + c_lo + cc; the subbands differ by scalar offsets */
    {
        const __amdgpu_buffer_rsrc_t rP =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.P[item]) + (int64_t)b * a.P_bs, 0, (int)(4 * a.P_bs), 0x00020000);
        const __amdgpu_buffer_rsrc_t rA = a.a_from_P ? rP
            : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.a[item]) + (int64_t)b * a.a_bs, 0, (int)(4 * a.a_bs), 0x00020000);
        const int sV = 4 * a.offC, sH = 4 * a.offR * a.PC, sD = sH + sV;
        constexpr int NE = NR * NC, K = (NE + FB_THREADS - 1) / FB_THREADS;
        float4 q[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int e = min(k * FB_THREADS + (int)threadIdx.x, NE - 1);
            const int rr = e / NC, cc = e - rr * NC;
            int r = r_lo + rr, c = c_lo + cc;
            if constexpr (EDGE) { /* one wrap suffices: the level is at least NR x NC */
                r = r < 0 ? r + a.R : (r >= a.R ? r - a.R : r);
                c = c < 0 ? c + a.C : (c >= a.C ? c - a.C : c);
            }
            const int vo = 4 * (r * a.PC + c);
            const int va = a.a_from_P ? vo : 4 * (r * a.lda + c);
            q[k].x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rA, va, 0, 0));
            q[k].y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rP, vo, sV, 0));
            q[k].z = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rP, vo, sH, 0));
            q[k].w = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rP, vo, sD, 0));
        }
#pragma unroll
        for (int k = 0; k < K; ++k) { /* clamped duplicates rewrite their own value */
            const int e = min(k * FB_THREADS + (int)threadIdx.x, NE - 1);
            const float va = a.a_from_P ? tl(q[k].x) : q[k].x;
            Aq[e] = make_float2(va, tl(q[k].z));
            Dq[e] = make_float2(tl(q[k].y), tl(q[k].w));
        }
    }
    __syncthreads();
    WTP_FPROBE(1);
    /* 2. axis -1 synthesis of the NR coefficient rows.  Lane = (row ro = lane / 32 of a row pair,
     *    column slot c = lane % 32); sub-pass p computes output column m0 + 2c + p, so the output's
     *    parity -- its taps -- and its site offset are uniform: the taps stay scalar.  A wave takes
     *    the row pairs wv, wv + 4, ...; results wait in registers until every read of Aq/Dq is done
     *    (LoHi is written over them). */
    const int m = m0 + lane;
    constexpr int KP = (NR + 7) / 8; /* row pairs per wave */
    f2 rowres[KP][2];
    /* EDGE: the exact-order results of this lane's fix-up entry (row fxrow, column pair fxc) */
    f2 fx[2] = {f2{0.0f, 0.0f}, f2{0.0f, 0.0f}};
    int fxrow = -1, fxc = 0;
    {
        const int ro = lane >> 5, c = lane & 31;
        /* both sub-passes from one sample window: p's samples start at column c + pe(p), and the
         * two sums are independent chains that interleave */
        constexpr int PE1 = (H & 1) ? 0 : 1, NS = HM + PE1;
        constexpr int PAR0 = (H & 1) ? 0 : 1, PAR1 = 1 - PAR0;
        /* the two outputs of column pair cp at (unwrapped) sample row pa / pd in wt_syn_pass's
         * order: the terms with i - j >= T by descending j first (T = 0 at a special site, N past
         * the end), then the others ascending */
        auto exact_pair = [&](const float2* pa, const float2* pd, int cp, f2& a0, f2& a1) {
            const SiteU s0 = site_u(m0 + 2 * cp, a.C, FT), s1 = site_u(m0 + 2 * cp + 1, a.C, FT);
            const int i0 = s0.i, T0 = s0.special ? 0 : a.C, i1 = s1.i, T1 = s1.special ? 0 : a.C;
            f2 v[NS];
            auto sp = [&](int p, int j) { return v[(p ? PE1 : 0) + HM - 1 - j]; };
            a0 = f2{0.0f, 0.0f};
            a1 = f2{0.0f, 0.0f};
            auto pass = [&](const float* rec) {
#pragma unroll
                for (int j = HM - 1; j >= 0; --j) {
                    if (i0 - j >= T0) a0 = a0 + rec[2 * j + PAR0] * sp(0, j);
                    if (i1 - j >= T1) a1 = a1 + rec[2 * j + PAR1] * sp(1, j);
                }
#pragma unroll
                for (int j = 0; j < HM; ++j) {
                    if (i0 - j < T0) a0 = a0 + rec[2 * j + PAR0] * sp(0, j);
                    if (i1 - j < T1) a1 = a1 + rec[2 * j + PAR1] * sp(1, j);
                }
            };
#pragma unroll
            for (int q = 0; q < NS; ++q) { const float2 t = pa[q]; v[q] = f2{t.x, t.y}; }
            pass(tp.f[2]);
#pragma unroll
            for (int q = 0; q < NS; ++q) { const float2 t = pd[q]; v[q] = f2{t.x, t.y}; }
            pass(tp.f[3]);
        };
        /* EDGE: the column pairs whose sites are special or past the end get the exact order in
         * a compact fix-up after the uniform pass: lane e of this wave = (its row e / nsc, the
         * (e % nsc)-th such pair).  Such pairs within the stored extent are the first one (H
         * even: output 0) or the last F/4 + 1 of the level, never both in one tile (the host runs
         * the frame only when the level is >= NC coefficients wide, so 2N > IC): at most F/4 + 1
         * pairs, and the wave's 2 KP rows times that fit its 64 lanes. */
        static_assert(2 * KP * (FT / 4 + 1) <= 64, "one fix-up pass per wave");
        uint32_t fxmask = 0;
        int nsc = 0;
        if constexpr (EDGE) {
            const SiteU s0 = site_u(m0 + 2 * c, a.C, FT), s1 = site_u(m0 + 2 * c + 1, a.C, FT);
            /* pairs past the stored extent (a partial last tile) are never read: left out */
            const bool need = (s0.special || s0.i >= a.C || s1.special || s1.i >= a.C) && m0 + 2 * c <= ml;
            fxmask = (uint32_t)__ballot(need && ro == 0); /* lanes 0..31: bit c */
            nsc = __builtin_popcount(fxmask);
        }
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            const int row = min(2 * (wv + 4 * k) + ro, NR - 1);
            const float2* pa = Aq + row * NC + c;
            const float2* pd = Dq + row * NC + c;
            f2 a0, a1;
            {
                f2 v[NS];
                /* sample of sub-pass p at tap j: column c + pe(p) + HM - 1 - j */
                auto sp = [&](int p, int j) { return v[(p ? PE1 : 0) + HM - 1 - j]; };
#pragma unroll
                for (int q = 0; q < NS; ++q) { const float2 t = pa[q]; v[q] = f2{t.x, t.y}; }
                const f2 z2 = {0.0f, 0.0f};
                a0 = z2 + tp.f[2][PAR0] * sp(0, 0);
                a1 = z2 + tp.f[2][PAR1] * sp(1, 0);
#pragma unroll
                for (int j = 1; j < HM; ++j) {
                    a0 = a0 + tp.f[2][2 * j + PAR0] * sp(0, j);
                    a1 = a1 + tp.f[2][2 * j + PAR1] * sp(1, j);
                }
#pragma unroll
                for (int q = 0; q < NS; ++q) { const float2 t = pd[q]; v[q] = f2{t.x, t.y}; }
#pragma unroll
                for (int j = 0; j < HM; ++j) {
                    a0 = a0 + tp.f[3][2 * j + PAR0] * sp(0, j);
                    a1 = a1 + tp.f[3][2 * j + PAR1] * sp(1, j);
                }
            }
            /* computed HERE: without this the compiler sinks the sums past the barrier below
             * (their only use is the LoHi write) and keeps every sample alive across it */
            asm volatile("" : "+v"(a0), "+v"(a1));
            rowres[k][0] = a0;
            rowres[k][1] = a1;
        }
        if (EDGE && fxmask) { /* uniform */
            if (lane < 2 * KP * nsc) {
                const int rs = lane / nsc, ci = lane - rs * nsc;
                uint32_t mm = fxmask;
                for (int t = 0; t < ci; ++t) mm &= mm - 1u;
                const int cp = __builtin_ctz(mm);
                const int row = 2 * (wv + 4 * (rs >> 1)) + (rs & 1);
                if (row < NR) {
                    f2 a0, a1;
                    exact_pair(Aq + row * NC + cp, Dq + row * NC + cp, cp, a0, a1);
                    asm volatile("" : "+v"(a0), "+v"(a1));
                    fx[0] = a0;
                    fx[1] = a1;
                    fxrow = row;
                    fxc = cp;
                }
            }
        }
    }
    __syncthreads(); /* every read of Aq/Dq is done: LoHi overwrites them */
    {
        const int ro = lane >> 5, c = lane & 31;
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            const int row = 2 * (wv + 4 * k) + ro;
            if (row < NR) {
#pragma unroll
                for (int p = 0; p < 2; ++p) LoHi[row * IC + 2 * c + p] = make_float2(rowres[k][p].x, rowres[k][p].y);
            }
        }
        /* the fix-up's exact values over the uniform pass's (this wave's own rows; a wave's LDS
         * writes land in program order) */
        if (EDGE && fxrow >= 0) {
#pragma unroll
            for (int p = 0; p < 2; ++p) LoHi[fxrow * IC + 2 * fxc + p] = make_float2(fx[p].x, fx[p].y);
        }
    }
    __syncthreads();
    WTP_FPROBE(2);
    /* 3. axis -2: each wave owns RB consecutive output rows; outputs k and k + RB/2 share taps and
     *    sit four sites apart, computed packed from the block's LoHi rows held in registers */
    constexpr int RB = IR / (FB_THREADS / 64);
    constexpr int E = (H & 1) ? 0 : 1, NV = H + RB / 2 - 1 + E, RB2 = RB / 2;
    static_assert(RB % 4 == 0, "packed column blocks pair rows k and k + RB/2, RB/4 sites apart");
    const int nf = n0 + RB * wv;
    const int g0 = site_u(nf, a.R, FT).i - H + 1 - r_lo;
    float2 r[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) r[q] = LoHi[(g0 + q) * IC + lane];
    const __amdgpu_buffer_rsrc_t rY =
        __builtin_amdgcn_make_buffer_rsrc(g.y[item] + (int64_t)b * a.outH * a.outW, 0, 4 * a.outH * a.outW, 0x00020000);
    const int vy = 4 * m;
    uint32_t z = 0; /* wave-uniform: zeros of this wave's outputs */
    /* EDGE: rows whose site is special or wrapped (the image's first / last few) are computed
     * again one by one in wt_syn_pass's order after the packed pass, which skips storing them;
     * rows past the extent are not stored.  The row's site is wave-uniform, so are the masks. */
    uint32_t xmask = 0, smask = (1u << RB) - 1u;
    if constexpr (EDGE) {
        for (int k = 0; k < RB; ++k) {
            const SiteU s = site_u(nf + k, a.R, FT);
            if (s.special || s.i >= a.R) xmask |= 1u << k;
            if (nf + k > nl) smask &= ~(1u << k);
        }
    }
    const bool min_ = !EDGE || m <= ml; /* EDGE: a partial last tile column */
    {
        const uint32_t wmask = smask & ~xmask; /* the rows the packed pass stores */
        f2 acc[RB2];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const float t0 = tp.f[2][2 * j], t1 = tp.f[2][2 * j + 1];
#pragma unroll
            for (int k = 0; k < RB2; ++k) {
                const int par = (k + E) & 1, base = ((k + E) >> 1) + H - 1;
                const float t = par ? t1 : t0;
                const f2 p = f2{t, t} * f2{r[base - j].x, r[base - j + RB2 / 2].x};
                acc[k] = (j == 0 ? f2{0.0f, 0.0f} : acc[k]) + p;
            }
        }
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const float t0 = tp.f[3][2 * j], t1 = tp.f[3][2 * j + 1];
#pragma unroll
            for (int k = 0; k < RB2; ++k) {
                const int par = (k + E) & 1, base = ((k + E) >> 1) + H - 1;
                const float t = par ? t1 : t0;
                acc[k] = acc[k] + f2{t, t} * f2{r[base - j].y, r[base - j + RB2 / 2].y};
            }
        }
        if constexpr (!EDGE) {
#pragma unroll
            for (int k = 0; k < RB2; ++k) {
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[k].x), rY, vy, 4 * (nf + k) * a.outW, 0);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[k].y), rY, vy, 4 * (nf + k + RB2) * a.outW, 0);
                z += (uint32_t)__popcll(__ballot(acc[k].x == 0.0f)) + (uint32_t)__popcll(__ballot(acc[k].y == 0.0f));
            }
        } else {
#pragma unroll
            for (int k = 0; k < RB2; ++k) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int kk = k + u * RB2;
                    const float y = u ? acc[k].y : acc[k].x;
                    if ((wmask >> kk) & 1u) {
                        if (min_) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), rY, vy, 4 * (nf + kk) * a.outW, 0);
                        z += (uint32_t)__popcll(__ballot(min_ && y == 0.0f));
                    }
                }
            }
        }
    }
    if (EDGE && (xmask & smask)) { /* uniform */
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            if (!(((xmask & smask) >> k) & 1u)) continue;
            const int n = nf + k;
            const SiteU s = site_u(n, a.R, FT);
            const int Tn = s.special ? 0 : a.R;
            const int par = (k + E) & 1, base = ((k + E) >> 1) + H - 1;
            float y = 0.0f;
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
                const float* rec = tp.f[2 + pass];
#pragma unroll
                for (int j = H - 1; j >= 0; --j)
                    if (s.i - j >= Tn) y = y + rec[2 * j + par] * (pass ? r[base - j].y : r[base - j].x);
#pragma unroll
                for (int j = 0; j < H; ++j)
                    if (s.i - j < Tn) y = y + rec[2 * j + par] * (pass ? r[base - j].y : r[base - j].x);
            }
            if (min_) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), rY, vy, 4 * n * a.outW, 0);
            z += (uint32_t)__popcll(__ballot(min_ && y == 0.0f));
        }
    }
    if (a.zc) {
        /* 8 bytes: the dynamic LDS follows the static variables, and a 4-byte one would leave
         * every float2 of the tiles 4-byte misaligned (measured: k_inv_int 4x slower, LDS
         * instruction issue stalls) */
        __shared__ unsigned long long zs;
        if (threadIdx.x == 0) zs = 0;
        __syncthreads();
        if (lane == 0 && z) atomicAdd(&zs, (unsigned long long)z);
        __syncthreads();
        if (threadIdx.x == 0 && zs) atomicAdd(a.zc + zc_off_of(g.tz_off[item]), zs);
    }
    WTP_FPROBE(3);
}

/* ------------------------------------------------------------ launchers --- */
/* which kernels run a level's tiles: 3 (default) as 2, except that a level of at most
 * FB_ONE_LAUNCH_TILES tiles (all items of the launch) runs every tile in ONE launch of the EDGE
 * form; 2 the interior rectangle in k_fwd_int / k_inv_int and the frame around it in their EDGE
 * forms (two launches); 1 the frame in the general k_fwd_level / k_inv_level; 0 every tile in the
 * general kernels (A/B and parity cross-checks) */
constexpr int64_t FB_ONE_LAUNCH_TILES = 8192;
static std::atomic<int> g_fb_interior{3};
int fb_set_interior(int mode) { return g_fb_interior.exchange(mode < 0 ? 0 : (mode > 3 ? 3 : mode)); }


/* dynamic LDS per workgroup; `alias`: the specialised kernels write their second-pass input
 * over their first-pass input (k_fwd_level: LH over T; k_inv_level: LoHi over Aq/Dq) */
static size_t fwd_lds(int F, bool alias = false) {
    const size_t pitch = alias ? (size_t)(3 + 2 * FC + F - 2 + 3) / 4 * 4 : (size_t)(2 * FC + F - 2); /* >= FWD_TP */
    /* lh: k_level's FR x NC float2 rows, or k_fwd_int's FR rows of 2 fwd_lhh(NC) float2 (the larger) */
    const size_t t = (size_t)(2 * FR + F - 2) * pitch,
                 lh = 2 * (size_t)FR * std::max<size_t>(2 * FC + F - 2, 2 * (size_t)fwd_lhh(2 * FC + F - 2));
    return sizeof(float) * (alias ? std::max(t, lh) : t + lh);
}
/* k_fwd_int's exact dynamic LDS: its input tile at pitch FWD_TP (the tile's first column at FWD_S0),
 * then its column results over it at the fwd_lhh half pitch -- the occupancy is LDS-bound (db8:
 * 46 x 128 floats = 23 KB, six workgroups per CU) */
static size_t fwd_int_lds(int F) {
    const size_t s0 = (size_t)(((1 - F / 2) % 4 + 4) % 4), nc = (size_t)(2 * FC + F - 2);
    const size_t t = (size_t)(2 * FR + F - 2) * ((s0 + nc + 3) / 4 * 4), lh = 2 * (size_t)FR * 2 * (size_t)fwd_lhh((int)nc);
    return sizeof(float) * std::max(t, lh);
}
static size_t inv_lds(int F, bool alias = false) {
    /* the tile bounds of k_inv_level (IR/2 + H rows, IC/2 + H columns): db8 40 x 40, 25.6 KB aliased --
     * six workgroups per CU instead of five */
    const size_t nr = IR / 2 + F / 2, nc = IC / 2 + F / 2;
    return sizeof(float) * (alias ? std::max(4 * nr * nc, 2 * nr * IC) : 4 * nr * nc + 2 * nr * IC);
}

template <int FT>
static TapsT<FT> taps_of(const Taps& tp) {
    if constexpr (FT == 0) {
        return tp;
    } else {
        SmallTaps t;
        memset(&t, 0, sizeof t);
        t.F = tp.F;
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < FT; ++j) t.f[k][j] = tp.f[k][j];
        return t;
    }
}
template <int FT>
static void fwd_go(const FwdGroup& g, int grid, const Taps& tp, hipStream_t s) {
    static_assert(FT <= SM_F_MAX, "SmallTaps holds the specialised filters");
    hipLaunchKernelGGL(k_fwd_level<FT>, dim3(grid), dim3(FB_THREADS), fwd_lds(tp.F, FT > 0), s, g, taps_of<FT>(tp));
}
template <int FT, bool EDGE>
static void fwd_int_go(const FwdGroup& g, int grid, const Taps& tp, const FwdSel& fs, hipStream_t s) {
    FwdIntTaps t;
    memset(&t, 0, sizeof t);
    for (int j = 0; j < FT; ++j) t.t[j] = f2{tp.f[0][j], tp.f[1][j]};
    hipLaunchKernelGGL((k_fwd_int<FT, EDGE>), dim3(grid), dim3(FB_THREADS), fwd_int_lds(tp.F), s, g, t, fs);
}

/* The interior rectangle of a forward level's tile grid (k_fwd_int's tiles): a tile row is
 * interior when its input rows lie inside the image (no extension; then every output site of it
 * is interior too, i < R) and it is full; a tile column when its aligned float4 window
 * [gc0 - S0, gc0 - S0 + TP) lies inside the row and it is full.  Both conditions are intervals
 * of the tile index.  False: no interior tile (or offsets beyond the kernel's 32-bit buffer
 * offsets) -- k_fwd_level takes the whole grid. */
static bool fwd_interior(const FwdArgs& a, int F, int* r0, int* nr, int* c0, int* nc) {
    if (!a.al16 || (int64_t)4 * a.P_bs > INT32_MAX || (int64_t)4 * a.Ro * a.Co > INT32_MAX) return false;
    if ((int64_t)4 * (2 * FR + F) * a.C > INT32_MAX) return false; /* k_fwd_int's tile loads: 32-bit offsets */
    const int S0 = ((1 - F / 2) % 4 + 4) % 4, TP = (S0 + 2 * FC + F - 2 + 3) / 4 * 4, NR = 2 * FR + F - 2;
    int rlo = -1, rhi = -2, clo = -1, chi = -2;
    for (int tr = 0; tr < a.tilesR; ++tr) {
        const int gr0 = 2 * FR * tr - F / 2 + 1;
        if (gr0 >= 0 && gr0 + NR <= a.R && (tr + 1) * FR <= a.Ro) { if (rlo < 0) rlo = tr; rhi = tr; }
    }
    for (int tc = 0; tc < a.tilesC; ++tc) {
        const int st = 2 * FC * tc - F / 2 + 1 - S0;
        if (st >= 0 && st + TP <= a.C && (tc + 1) * FC <= a.Co) { if (clo < 0) clo = tc; chi = tc; }
    }
    if (rlo < 0 || clo < 0) return false;
    *r0 = rlo; *nr = rhi - rlo + 1; *c0 = clo; *nc = chi - clo + 1;
    return true;
}
static bool fwd_int_filter(int F) { return F == 2 || F == 4 || F == 6 || F == 8 || F == 10 || F == 12 || F == 16 || F == 18; }
template <int FT>
static void inv_go(const InvGroup& g, int grid, const Taps& tp, hipStream_t s) {
    hipLaunchKernelGGL(k_inv_level<FT>, dim3(grid), dim3(FB_THREADS), inv_lds(tp.F, FT > 0), s, g, taps_of<FT>(tp));
}
template <int FT, bool EDGE>
static void inv_int_go(const InvGroup& g, int grid, const Taps& tp, hipStream_t s) {
    hipLaunchKernelGGL((k_inv_int<FT, EDGE>), dim3(grid), dim3(FB_THREADS), inv_lds(tp.F, true), s, g, taps_of<FT>(tp));
}

/* The interior rectangle of a synthesis level's tile grid (k_inv_int's tiles): along each axis a
 * tile is interior when it is full, holds no special site (H even: outputs 0 and 2N - 1), its
 * last site is below N and its first site's window starts at or after 0 -- the sites grow with
 * the output index, so the interior tiles are an interval. */
static bool inv_axis(int tiles, int T, int out, int N, int F, int* lo, int* cnt) {
    const int H = F / 2;
    int a = -1, z = -2;
    for (int t = 0; t < tiles; ++t) {
        const int n0 = t * T, nl = n0 + T - 1;
        if (nl >= out) continue;
        const wt_syn_site s0 = wt_syn_locate(n0, N, F), s1 = wt_syn_locate(nl, N, F);
        if (s0.special || s1.special || (H % 2 == 0 && (n0 == 0 || nl >= 2 * N - 1))) continue;
        if (s1.i >= N || s0.i - H + 1 < 0) continue;
        if (a < 0) a = t;
        z = t;
    }
    if (a < 0) return false;
    *lo = a;
    *cnt = z - a + 1;
    return true;
}
static bool inv_interior(const InvArgs& a, int F, int* r0, int* nr, int* c0, int* nc) {
    if ((int64_t)4 * a.P_bs > INT32_MAX || (int64_t)4 * a.outH * a.outW > INT32_MAX) return false;
    if (!a.a_from_P && (int64_t)4 * a.a_bs > INT32_MAX) return false;
    return inv_axis(a.tilesR, IR, a.outH, a.R, F, r0, nr) && inv_axis(a.tilesC, IC, a.outW, a.C, F, c0, nc);
}
/* k_inv_int's EDGE form wraps a window coordinate once: the level spans a whole window */
static bool inv_frame_ok(const InvArgs& a, int F) {
    const int H = F / 2, NR = IR / 2 + H - (H & 1), NC = IC / 2 + H - (H & 1);
    return a.R >= NR && a.C >= NC;
}

/* The tiled path needs an even filter, the LDS budget, and images large enough that a tile
 * is mostly useful work (tiny conv kernels keep the per-point kernels). */
bool fb_tiled_ok(int64_t B, int64_t R, int64_t C, const Taps& tp) {
    if ((tp.F & 1) || fwd_lds(tp.F) > FB_MAX_LDS || inv_lds(tp.F) > FB_MAX_LDS) return false;
    if (R > (1 << 28) || C > (1 << 28) || B * R * C > ((int64_t)1 << 31)) return false;
    return R * C >= 512; /* at least a quarter of a forward tile of outputs */
}

static FwdArgs fwd_args(const FwdItem& x) {
    FwdArgs a;
    memset(&a, 0, sizeof a);
    a.in = x.in;
    a.in_bs = x.R * x.C;
    a.R = (int)x.R;
    a.C = (int)x.C;
    a.Ro = (int)((x.R + 1) / 2);
    a.Co = (int)((x.C + 1) / 2);
    a.P = x.P;
    a.P_bs = x.PR * x.PC;
    a.PC = (int)x.PC;
    a.offR = (int)x.offR;
    a.offC = (int)x.offC;
    a.anext = x.anext;
    a.last = x.last;
    a.tilesC = (a.Co + FC - 1) / FC;
    a.tilesR = (a.Ro + FR - 1) / FR;
    a.al16 = (reinterpret_cast<uintptr_t>(x.in) % 16) == 0 && (x.C % 4) == 0;
    return a;
}

static InvArgs inv_args(const InvItem& x) {
    InvArgs a;
    memset(&a, 0, sizeof a);
    a.a = x.a_src ? x.a_src : x.P;
    a.a_bs = x.a_bs;
    a.lda = (int)x.lda;
    a.a_from_P = x.a_from_P;
    a.P = x.P;
    a.P_bs = x.PR * x.PC;
    a.PC = (int)x.PC;
    a.offR = (int)x.offR;
    a.offC = (int)x.offC;
    a.R = (int)x.R;
    a.C = (int)x.C;
    a.y = x.y;
    a.outH = (int)x.outH;
    a.outW = (int)x.outW;
    a.thr = x.thr;
    a.zc = x.zc;
    a.tilesC = (int)((x.outW + IC - 1) / IC);
    a.tilesR = (int)((x.outH + IR - 1) / IR);
    return a;
}

static_assert(sizeof(FwdGroup) + sizeof(Taps) <= 3840 && sizeof(InvGroup) + sizeof(Taps) <= 3840,
              "filter-bank kernel arguments (plus the hidden ones) stay under 4 KB");

/* Items are grouped by geometry (their order does not matter: every item is independent); each
 * launch takes up to FB_UNI items of one geometry whose tiles sum below 2^31 (fb_tiled_ok bounds
 * every item's B * R * C below 2^31 elements, hence its tiles far below). */
template <class Arg, class Key>
static std::vector<std::vector<int>> uniform_groups(const std::vector<Arg>& args, const std::vector<int64_t>& tiles,
                                                    const Key& key, int cap) {
    std::vector<std::vector<int>> groups;
    std::vector<int> rep; /* a representative item of each group's geometry */
    for (int i = 0; i < (int)args.size(); ++i) {
        int gi = -1;
        for (int j = 0; j < (int)groups.size() && gi < 0; ++j) {
            const int r = rep[j];
            if ((int)groups[j].size() < cap && tiles[r] == tiles[i] && key(args[r], args[i]) &&
                tiles[i] * (int64_t)(groups[j].size() + 1) <= INT32_MAX)
                gi = j;
        }
        if (gi < 0) {
            groups.emplace_back();
            rep.push_back(i);
            gi = (int)groups.size() - 1;
        }
        groups[gi].push_back(i);
    }
    return groups;
}

/* one launch of the general (edge-capable) kernel, and one of the interior kernel, by filter */
static void fwd_general(const FwdGroup& g, int grid, const Taps& tp, hipStream_t s) {
    switch (tp.F) {
    case 2: fwd_go<2>(g, grid, tp, s); break;
    case 4: fwd_go<4>(g, grid, tp, s); break;
    case 6: fwd_go<6>(g, grid, tp, s); break;
    case 8: fwd_go<8>(g, grid, tp, s); break;
    case 10: fwd_go<10>(g, grid, tp, s); break;
    case 12: fwd_go<12>(g, grid, tp, s); break;
    case 16: fwd_go<16>(g, grid, tp, s); break;
    case 18: fwd_go<18>(g, grid, tp, s); break;
    default: fwd_go<0>(g, grid, tp, s); break;
    }
}
template <bool EDGE>
static void fwd_interior_go(const FwdGroup& g, int grid, const Taps& tp, const FwdSel& fs, hipStream_t s) {
    switch (tp.F) {
    case 2: fwd_int_go<2, EDGE>(g, grid, tp, fs, s); break;
    case 4: fwd_int_go<4, EDGE>(g, grid, tp, fs, s); break;
    case 6: fwd_int_go<6, EDGE>(g, grid, tp, fs, s); break;
    case 8: fwd_int_go<8, EDGE>(g, grid, tp, fs, s); break;
    case 10: fwd_int_go<10, EDGE>(g, grid, tp, fs, s); break;
    case 12: fwd_int_go<12, EDGE>(g, grid, tp, fs, s); break;
    case 16: fwd_int_go<16, EDGE>(g, grid, tp, fs, s); break;
    case 18: fwd_int_go<18, EDGE>(g, grid, tp, fs, s); break;
    default: break;
    }
}
static void inv_general(const InvGroup& g, int grid, const Taps& tp, hipStream_t s) {
    switch (tp.F) {
    case 2: inv_go<2>(g, grid, tp, s); break;
    case 4: inv_go<4>(g, grid, tp, s); break;
    case 6: inv_go<6>(g, grid, tp, s); break;
    case 8: inv_go<8>(g, grid, tp, s); break;
    case 10: inv_go<10>(g, grid, tp, s); break;
    case 12: inv_go<12>(g, grid, tp, s); break;
    case 16: inv_go<16>(g, grid, tp, s); break;
    case 18: inv_go<18>(g, grid, tp, s); break;
    default: inv_go<0>(g, grid, tp, s); break;
    }
}
template <bool EDGE>
static void inv_interior_go(const InvGroup& g, int grid, const Taps& tp, hipStream_t s) {
    switch (tp.F) {
    case 2: inv_int_go<2, EDGE>(g, grid, tp, s); break;
    case 4: inv_int_go<4, EDGE>(g, grid, tp, s); break;
    case 6: inv_int_go<6, EDGE>(g, grid, tp, s); break;
    case 8: inv_int_go<8, EDGE>(g, grid, tp, s); break;
    case 10: inv_int_go<10, EDGE>(g, grid, tp, s); break;
    case 12: inv_int_go<12, EDGE>(g, grid, tp, s); break;
    case 16: inv_int_go<16, EDGE>(g, grid, tp, s); break;
    case 18: inv_int_go<18, EDGE>(g, grid, tp, s); break;
    default: break;
    }
}

/* fused selection: a level of (B, R, C) images runs only in k_fwd_int (the interior rectangle and
 * the edge form, as launch_fwd_levels dispatches it with interior mode 2 or 3), whose waves classify
 * what they write; the slots are one per wave of every tile */
bool fwd_level_fused_ok(const FwdItem& x, const Taps& tp, int64_t* slots, bool any_mode) {
    const FwdArgs a = fwd_args(x);
    int r0, nr, c0, nc;
    if ((!any_mode && g_fb_interior.load(std::memory_order_relaxed) < 2) || !fwd_int_filter(tp.F) || !fb_tiled_ok(x.B, x.R, x.C, tp) ||
        !fwd_interior(a, tp.F, &r0, &nr, &c0, &nc))
        return false;
    *slots = (int64_t)a.tilesR * a.tilesC * x.B * (FB_THREADS / 64);
    return true;
}

void launch_fwd_levels(const FwdItem* it, int n, const Taps& tp, hipStream_t s, bool fused) {
    std::vector<FwdArgs> args(n);
    std::vector<int64_t> tiles(n);
    for (int i = 0; i < n; ++i) {
        args[i] = fwd_args(it[i]);
        tiles[i] = (int64_t)args[i].tilesC * args[i].tilesR * it[i].B;
    }
    auto same = [](const FwdArgs& x, const FwdArgs& y) {
        return x.in_bs == y.in_bs && x.R == y.R && x.C == y.C && x.Ro == y.Ro && x.Co == y.Co && x.P_bs == y.P_bs &&
               x.PC == y.PC && x.offR == y.offR && x.offC == y.offC && x.last == y.last && x.al16 == y.al16;
    };
    for (const auto& grp : uniform_groups(args, tiles, same, FB_UNI)) {
        FwdGroup g;
        memset(&g, 0, sizeof g);
        g.geo = args[grp[0]];
        g.n = (int)grp.size();
        g.tiles = (int)tiles[grp[0]];
        for (int m = 0; m < g.n; ++m) {
            g.in[m] = args[grp[m]].in;
            g.anext[m] = args[grp[m]].anext;
            g.P[m] = args[grp[m]].P;
        }
        /* fused selection: the items' slots (a fused launch group holds at most SEG_PER_LAUNCH
         * chains, so at most that many items of one level) */
        FwdSel fs;
        memset(&fs, 0, sizeof fs);
        if (fused && it[grp[0]].fslot && g.n <= SEG_PER_LAUNCH) {
            fs.on = 1;
            for (int m = 0; m < g.n; ++m) {
                fs.slots[m] = it[grp[m]].fslot;
                fs.hdr[m] = it[grp[m]].fhdr;
            }
        }
        int r0, nr, c0, nc;
        const int mode = g_fb_interior.load(std::memory_order_relaxed);
        if (mode && fwd_int_filter(tp.F) && fwd_interior(g.geo, tp.F, &r0, &nr, &c0, &nc)) {
            /* the interior tiles in k_fwd_int, then the frame around them (measured in round 4:
             * the frame on a stream of its own beside the interior launch gained nothing -- both
             * launches fill every CU, so the work only moved) */
            const int B = g.tiles / (g.geo.tilesR * g.geo.tilesC);
            g.geo.tr0 = r0; g.geo.nTR = nr; g.geo.tc0 = c0; g.geo.nTC = nc;
            FwdGroup gi = g;
            gi.tiles = nr * nc * B;
            gi.dv_tiles = make_fastdiv((uint32_t)gi.tiles);
            gi.dv_per = make_fastdiv((uint32_t)(nr * nc));
            gi.dv_ntc = make_fastdiv((uint32_t)nc);
            const int fr = g.geo.tilesR * g.geo.tilesC - nr * nc;
            if (mode == 3 && fr > 0 && (int64_t)g.n * g.tiles <= FB_ONE_LAUNCH_TILES) {
                /* a small level: every tile in ONE launch of the edge form (its decode with an empty
                 * rectangle walks the whole grid row-major; interior tiles take its interior paths),
                 * where the interior and the frame as two launches were latency cliffs (round 4: the
                 * frame's launch as long as the interior's at levels 3-5) */
                FwdGroup ga = g;
                ga.geo.tr0 = 0; ga.geo.nTR = 0; ga.geo.tc0 = 0; ga.geo.nTC = 0;
                ga.dv_tiles = make_fastdiv((uint32_t)ga.tiles);
                ga.dv_per = make_fastdiv((uint32_t)ga.tiles / (uint32_t)B);
                ga.dv_tc = make_fastdiv((uint32_t)g.geo.tilesC);
                ga.dv_side = make_fastdiv((uint32_t)g.geo.tilesC);
                fwd_interior_go<true>(ga, ga.n * ga.tiles, tp, fs, s);
                continue;
            }
            fwd_interior_go<false>(gi, gi.n * gi.tiles, tp, fs, s);
            if (fr == 0) continue;
            if (fs.on) /* the frame's slots follow the interior's */
                for (int m = 0; m < g.n; ++m) fs.slots[m] += (int64_t)gi.tiles * (FB_THREADS / 64) * FSL_WORDS;
            g.geo.frame = 1;
            g.tiles = fr * B;
            g.dv_tiles = make_fastdiv((uint32_t)g.tiles);
            g.dv_per = make_fastdiv((uint32_t)fr);
            g.dv_tc = make_fastdiv((uint32_t)g.geo.tilesC);
            g.dv_side = make_fastdiv((uint32_t)std::max(1, g.geo.tilesC - nc));
            if (mode >= 2) {
                fwd_interior_go<true>(g, g.n * g.tiles, tp, fs, s);
                continue;
            }
        }
        fwd_general(g, g.n * g.tiles, tp, s);
    }
}

void launch_inv_levels(const InvItem* it, int n, const Taps& tp, hipStream_t s) {
    std::vector<InvArgs> args(n);
    std::vector<int64_t> tiles(n);
    for (int i = 0; i < n; ++i) {
        args[i] = inv_args(it[i]);
        tiles[i] = (int64_t)args[i].tilesC * args[i].tilesR * it[i].B;
    }
    /* one geometry, and the threshold / zero-count words at whole-element offsets from the
     * group's first ones (or absent in all of them) */
    auto off_ok = [](const void* p, const void* q, size_t elem) {
        if ((p == nullptr) != (q == nullptr)) return false;
        if (!p) return true;
        const intptr_t d = reinterpret_cast<intptr_t>(q) - reinterpret_cast<intptr_t>(p);
        return d % (intptr_t)elem == 0 && d / (intptr_t)elem >= INT16_MIN && d / (intptr_t)elem <= INT16_MAX;
    };
    auto same = [&](const InvArgs& x, const InvArgs& y) {
        return x.a_bs == y.a_bs && x.lda == y.lda && x.a_from_P == y.a_from_P && x.P_bs == y.P_bs && x.PC == y.PC &&
               x.offR == y.offR && x.offC == y.offC && x.R == y.R && x.C == y.C && x.outH == y.outH &&
               x.outW == y.outW && off_ok(x.thr, y.thr, sizeof(float)) &&
               off_ok(x.zc, y.zc, sizeof(unsigned long long));
    };
    for (const auto& grp : uniform_groups(args, tiles, same, FB_UNI)) {
        InvGroup g;
        memset(&g, 0, sizeof g);
        g.geo = args[grp[0]];
        g.n = (int)grp.size();
        g.tiles = (int)tiles[grp[0]];
        for (int m = 0; m < g.n; ++m) {
            const InvArgs& x = args[grp[m]];
            g.a[m] = x.a;
            g.P[m] = x.P;
            g.y[m] = x.y;
            const int32_t to = x.thr ? (int32_t)(x.thr - g.geo.thr) : 0, zo = x.zc ? (int32_t)(x.zc - g.geo.zc) : 0;
            g.tz_off[m] = (int32_t)(((uint32_t)zo << 16) | ((uint32_t)to & 0xFFFFu)); /* off_ok: both within int16 */
        }
        int r0, nr, c0, nc;
        const int mode = g_fb_interior.load(std::memory_order_relaxed);
        if (mode && fwd_int_filter(tp.F) && inv_interior(g.geo, tp.F, &r0, &nr, &c0, &nc)) {
            /* the interior tiles in k_inv_int, then the frame around them (as the analysis) */
            const int B = g.tiles / (g.geo.tilesR * g.geo.tilesC);
            g.geo.tr0 = r0; g.geo.nTR = nr; g.geo.tc0 = c0; g.geo.nTC = nc;
            InvGroup gi = g;
            gi.tiles = nr * nc * B;
            gi.dv_tiles = make_fastdiv((uint32_t)gi.tiles);
            gi.dv_per = make_fastdiv((uint32_t)(nr * nc));
            gi.dv_ntc = make_fastdiv((uint32_t)nc);
            const int fr = g.geo.tilesR * g.geo.tilesC - nr * nc;
            const bool edge_ok = inv_frame_ok(g.geo, tp.F);
            if (mode == 3 && fr > 0 && edge_ok && (int64_t)g.n * g.tiles <= FB_ONE_LAUNCH_TILES) {
                /* a small level: every tile in one launch of the edge form (as the analysis) */
                InvGroup ga = g;
                ga.geo.tr0 = 0; ga.geo.nTR = 0; ga.geo.tc0 = 0; ga.geo.nTC = 0;
                ga.dv_tiles = make_fastdiv((uint32_t)ga.tiles);
                ga.dv_per = make_fastdiv((uint32_t)ga.tiles / (uint32_t)B);
                ga.dv_tc = make_fastdiv((uint32_t)g.geo.tilesC);
                ga.dv_side = make_fastdiv((uint32_t)g.geo.tilesC);
                inv_interior_go<true>(ga, ga.n * ga.tiles, tp, s);
                continue;
            }
            inv_interior_go<false>(gi, gi.n * gi.tiles, tp, s);
            if (fr == 0) continue;
            g.geo.frame = 1;
            g.tiles = fr * B;
            g.dv_tiles = make_fastdiv((uint32_t)g.tiles);
            g.dv_per = make_fastdiv((uint32_t)fr);
            g.dv_tc = make_fastdiv((uint32_t)g.geo.tilesC);
            g.dv_side = make_fastdiv((uint32_t)std::max(1, g.geo.tilesC - nc));
            if (mode >= 2 && edge_ok) {
                inv_interior_go<true>(g, g.n * g.tiles, tp, s);
                continue;
            }
        }
        inv_general(g, g.n * g.tiles, tp, s);
    }
}

void launch_fwd_level(const float* in, int64_t B, int64_t R, int64_t C, const Taps& tp, float* anext, float* P,
                      int64_t PR, int64_t PC, int64_t offR, int64_t offC, int last, hipStream_t s) {
    const FwdItem x{in, B, R, C, anext, P, PR, PC, offR, offC, last};
    launch_fwd_levels(&x, 1, tp, s);
}

void launch_inv_level(const float* a_src, int64_t a_bs, int64_t lda, int a_from_P, const float* P, int64_t PR,
                      int64_t PC, int64_t offR, int64_t offC, int64_t B, int64_t R, int64_t C, const Taps& tp,
                      const float* thr, float* y, int64_t outH, int64_t outW, unsigned long long* zc,
                      hipStream_t s) {
    const InvItem x{a_src, a_bs, lda, a_from_P, P, PR, PC, offR, offC, B, R, C, thr, y, outH, outW, zc};
    launch_inv_levels(&x, 1, tp, s);
}

}  // namespace wtp
