/* Internal types shared by the kernel and API translation units of libwtprune.so. */
#ifndef WTP_INTERNAL_H
#define WTP_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wtprune.h"
#include "wt_dwt_core.h"

#pragma clang fp contract(off)

namespace wtp {

/* ---- selection histogram: bins over the float32 bit pattern of |x| (monotone in |x|) ----
 * bin 0        : exact zeros (+0/-0)
 * bin 1        : 0 < |x| < 2^(WIN_E0-127)               (below the window)
 * bins 2..     : exponent window [WIN_E0, WIN_E0+WIN_EXP) x 2^MANT_BITS mantissa slices
 * bin NB-1     : |x| >= 2^(WIN_E0+WIN_EXP-127), inf, NaN
 * 1/128-octave slices keep the population of the bin holding the percentile at ~0.3-1% of a
 * weight tensor, which the candidate pass gathers and the select kernel resolves exactly. */
constexpr int WIN_EXP = 32;
constexpr int MANT_BITS = 7;
constexpr uint32_t WIN_E0 = 101; /* window = [2^-26, 2^6) */
constexpr int NB = 3 + (WIN_EXP << MANT_BITS); /* 4099 */
constexpr int BIN_ZERO = 0, BIN_UNDER = 1, BIN_OVER = NB - 1;
constexpr int NB_PAD = 4112; /* per-slot stride (16-word multiple) */

__host__ __device__ __forceinline__ int key_bin(uint32_t key) {
    if (key == 0) return BIN_ZERO;
    const uint32_t e = key >> 23;
    if (e < WIN_E0) return BIN_UNDER;
    if (e >= WIN_E0 + WIN_EXP) return BIN_OVER;
    return 2 + (int)(((e - WIN_E0) << MANT_BITS) | ((key >> (23 - MANT_BITS)) & ((1u << MANT_BITS) - 1)));
}

/* ---- grouped launches over segments (one segment = one selection population) ---- */
constexpr int CHUNK = 16384;        /* elements per block in the streaming passes */
constexpr int STREAM_THREADS = 256; /* 64 elements = 16 float4 per thread          */
constexpr int SEG_PER_LAUNCH = 24;

enum SegFlags : int32_t {
    SEG_MASK = 1,      /* level-0 / 1-D: the mask pass writes `out` from `data`   */
    SEG_ALIGNED = 2,   /* data (and out) 16-byte aligned: float4 path              */
};

struct SegDesc {
    const float* data; /* selection population: raw weights or the packed coefficients */
    float* out;        /* SEG_MASK: output weights                                       */
    int64_t n;         /* population size                                                */
    int64_t r0;        /* lower order statistic (0-based rank in ascending |x|)          */
    double gamma;      /* NumPy gamma = vi - previous_index                              */
    int64_t numel;     /* tensor numel (result field)                                    */
    int32_t blk_begin; /* first block of this segment in the grouped grid                */
    int32_t slot;      /* workspace selection slot                                       */
    int32_t res;       /* result index                                                   */
    int32_t flags;
    int32_t eff_level;
    int32_t above;     /* vi >= n-1: both order statistics are the maximum               */
    int64_t cand_off;  /* this segment's candidate buffer (elements into the workspace)  */
    int64_t cap;       /* its capacity                                                   */
};

struct SegTable {
    int32_t nseg;
    int32_t nblk;
    int32_t pad[2];
    SegDesc s[SEG_PER_LAUNCH];
};

/* per-slot selection state (workspace, zeroed once, left zeroed by every call) */
struct SelState {
    uint32_t maxkey;     /* atomicMax in k_hist; reset by k_select              */
    uint32_t cand_count; /* atomicAdd in k_compact; reset by k_select           */
    uint32_t cb_lo;      /* candidate bin range [cb_lo, cb_hi]                  */
    uint32_t cb_hi;
    int64_t below;       /* population in bins < cb_lo                          */
    int32_t mode;        /* MODE_*                                              */
    uint32_t key_a;      /* resolved order statistics (bit patterns of |x|)     */
    uint32_t key_b;
    float thr32;         /* the float32 threshold the compare uses              */
    int32_t a_zero;      /* lower statistic sits in the zero bin                */
    int32_t b_zero;
};

enum SelMode : int32_t { MODE_CAND = 1, MODE_ZERO = 2, MODE_FULL = 3 };

/* filter taps as a kernel argument (scalar-loaded, uniform across the wave) */
struct Taps {
    int32_t F;
    int32_t pad[3];
    float f[4][WTP_MAX_F]; /* dec_lo, dec_hi, rec_lo, rec_hi */
};

/* ---- launchers (kernels.hip) ---- */
void launch_hist(const SegTable& t, uint32_t* hist, SelState* sel, hipStream_t s);
void launch_findbin(const SegTable& t, uint32_t* hist, SelState* sel, wtp_result* res, hipStream_t s);
void launch_compact(const SegTable& t, SelState* sel, uint32_t* cand, hipStream_t s);
void launch_select(const SegTable& t, SelState* sel, const uint32_t* cand, wtp_result* res, hipStream_t s);
void launch_mask(const SegTable& t, const SelState* sel, wtp_result* res, hipStream_t s);

void launch_dwt_cols(const float* in, int64_t B, int64_t R, int64_t C, const Taps& tp, float* L, float* H,
                     hipStream_t s);
void launch_dwt_rows(const float* L, const float* H, int64_t B, int64_t Ro, int64_t C, const Taps& tp,
                     float* anext, float* P, int64_t PR, int64_t PC, int64_t offR, int64_t offC, int last,
                     hipStream_t s);
void launch_idwt_rows(const float* a, int64_t a_bs, int64_t lda, int a_from_P, const float* P, int64_t PR,
                      int64_t PC, int64_t offR, int64_t offC, int64_t B, int64_t R, int64_t C, const Taps& tp,
                      const float* thr, float* lo, float* hi, hipStream_t s);
void launch_idwt_cols(const float* lo, const float* hi, int64_t B, int64_t R, int64_t C, const Taps& tp,
                      float* y, int64_t outH, int64_t outW, unsigned long long* zero_count, hipStream_t s);
void launch_copy_threshold(const float* P, float* out, int64_t n, const float* thr, unsigned long long* zc,
                           hipStream_t s);
void launch_synth(float* out, int64_t n, uint64_t seed, uint32_t tid, int e, hipStream_t s);

}  // namespace wtp

#endif
