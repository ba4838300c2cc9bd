/* Internal types shared by the kernel and API translation units of libwtprune.so. */
#ifndef WTP_INTERNAL_H
#define WTP_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wtprune.h"
#include "wt_dwt_core.h"

#pragma clang fp contract(off)

namespace wtp {

/* ---- selection: sample window + one counting/collecting pass ----
 * k_sample brackets the two order statistics r0, r0+1 of |x| with a window [kl, kh] taken
 * from M_SAMPLE sampled keys (the exact values when the population fits in the sample);
 * k_collect streams the data once, counting keys below kl / equal to kl / equal to kh and
 * gathering the keys strictly inside (kl, kh) with a 256-bin sub-histogram; k_select
 * resolves both ranks exactly (or, if the window missed, by a full radix select). */
constexpr int M_SAMPLE = 32768;
constexpr int SAMPLE_GROUP = 16;   /* contiguous keys per sample group */
constexpr int NSUB = 256;          /* sub-histogram bins over (kl, kh) */

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

/* per-slot selection state.  Slots are the positions of a segment inside its launch group
 * (0..SEG_PER_LAUNCH-1); the SelState slots sit at the very start of every workspace
 * layout, so every call sees the same persistent region: zeroed once by wtp_workspace_init
 * and left zeroed (counters) by every call -- k_select clears what k_collect accumulated. */
struct SelState {
    uint32_t maxkey;             /* atomicMax (k_collect)                                 */
    uint32_t cand_count;         /* atomicAdd (k_collect): keys strictly inside (kl, kh)  */
    unsigned long long below;    /* atomicAdd (k_collect): keys < kl                       */
    unsigned long long eq_lo;    /* keys == kl                                            */
    unsigned long long eq_hi;    /* keys == kh (kh != kl)                                 */
    uint32_t kl, kh;             /* window (k_sample); kh = 0xFFFFFFFF: unbounded          */
    uint32_t shift;              /* sub-bin of an inside key = (key - kl - 1) >> shift     */
    int32_t mode;                /* MODE_* chosen by k_select (diagnostics)                */
    float thr32;                 /* the float32 threshold the compare uses                 */
    uint32_t key_a, key_b;       /* resolved order statistics                              */
    uint32_t pad[1];
    uint32_t sub[NSUB];          /* sub-histogram of inside keys (atomicAdd, k_collect)    */
};
static_assert(sizeof(SelState) % 64 == 0, "SelState padding");

enum SelMode : int32_t { MODE_CAND = 1, MODE_WINDOW = 2, MODE_FULL = 3 };

/* filter taps as a kernel argument (scalar-loaded, uniform across the wave) */
struct Taps {
    int32_t F;
    int32_t pad[3];
    float f[4][WTP_MAX_F]; /* dec_lo, dec_hi, rec_lo, rec_hi */
};

/* ---- launchers (kernels.hip) ---- */
void launch_sample(const SegTable& t, SelState* sel, wtp_result* res, hipStream_t s);
void launch_collect(const SegTable& t, SelState* sel, uint32_t* cand, hipStream_t s);
void launch_select(const SegTable& t, SelState* sel, const uint32_t* cand, wtp_result* res, float* thr_out,
                   hipStream_t s);
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
