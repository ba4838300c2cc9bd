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
 * Every k_collect block histograms the same M_SAMPLE sampled keys of its segment (the whole
 * segment when it fits) into 4099 bins of the float32 bit pattern of |x| (1/128 octave in
 * [2^-26, 2^6), plus zero / under / over bins) and takes a window [kl, kh] of bin edges that
 * brackets the order statistics r0, r0+1 with a 6-sigma binomial margin; it then streams its
 * chunk once, counting keys < kl and == kl and scattering the keys inside (kl, kh] into nsub
 * key-range buckets; k_select reads only the bucket(s) holding the two
 * ranks and resolves them exactly, or by a full radix select over the segment if the window
 * missed. */
constexpr int M_SAMPLE = 4096;      /* k_resident: every workgroup draws it before its chunk    */
/* k_window (three-launch form): one block per segment, 64 keys a thread in passes of 16; on cfg5
 * 65536 keys (window ~2.4 % of the segment) beat 16384 (~5 %: k_collect +55 us per 24-segment
 * launch) and 262144 (~1.2 %: k_window +47 us for 10 us less k_collect) */
constexpr int M_SAMPLE_WIN = 65536;
constexpr int SAMPLE_GROUP = 16;   /* contiguous keys per sample group */
constexpr int NSUB_MAX = 1024;     /* buckets over (kl, kh]: 64..1024 per segment (SegDesc) */
constexpr int RES_NSUB_LOG2 = 10;  /* k_resident: 1024 buckets over (kl, kh] (4096 measured slower: 8 KB more reads per
                                     * workgroup; 2048 with the selectors, round 5: 26.2 against 25.8 us) */
constexpr int RES_NSUB = 1 << RES_NSUB_LOG2;
constexpr int BUCKET_MAX = 8192;   /* keys per bucket (two buckets are staged in LDS)       */
constexpr int BUCKET_MAX_DWT = 1 << 16; /* DWT segments: 64 wide buckets, one select per segment */
constexpr int WIN_EXP = 32;
constexpr int MANT_BITS = 7;
constexpr uint32_t WIN_E0 = 101;   /* bin window = [2^-26, 2^6) */
constexpr int NB = 3 + (WIN_EXP << MANT_BITS); /* 4099 */
constexpr int BIN_ZERO = 0, BIN_UNDER = 1, BIN_OVER = NB - 1;

__host__ __device__ __forceinline__ int key_bin(uint32_t key) {
    if (key == 0) return BIN_ZERO;
    const uint32_t e = key >> 23;
    if (e < WIN_E0) return BIN_UNDER;
    if (e >= WIN_E0 + WIN_EXP) return BIN_OVER;
    return 2 + (int)(((e - WIN_E0) << MANT_BITS) | ((key >> (23 - MANT_BITS)) & ((1u << MANT_BITS) - 1)));
}
/* smallest key of bin b, and the smallest key of the bins above b */
__host__ __device__ __forceinline__ uint32_t bin_lo_key(int b) {
    if (b <= BIN_ZERO) return 0u;
    if (b == BIN_UNDER) return 1u;
    if (b == BIN_OVER) return (WIN_E0 + WIN_EXP) << 23;
    return ((WIN_E0 + ((uint32_t)(b - 2) >> MANT_BITS)) << 23) | (((uint32_t)(b - 2) & ((1u << MANT_BITS) - 1)) << (23 - MANT_BITS));
}
__host__ __device__ __forceinline__ uint32_t bin_hi_key(int b) { /* exclusive; 0xFFFFFFFF = unbounded */
    return b >= BIN_OVER ? 0xFFFFFFFFu : bin_lo_key(b + 1);
}

/* ---- grouped launches over segments (one segment = one selection population) ---- */
constexpr int CHUNK = 16384;        /* elements per block in the streaming passes */
constexpr int STREAM_THREADS = 256; /* 64 elements = 16 float4 per thread          */
constexpr int COLLECT_THREADS = 256; /* k_collect: 4 waves per block ...             */
constexpr int COLLECT_IT = 16;       /* ... of 16 float4 per thread: one CHUNK        */
/* launch groups of at most this many k_collect blocks derive the window inside every block (one
 * launch fewer: the launch-latency regime, e.g. cfg3); larger ones launch k_window once */
constexpr int WINDOW_INLINE_MAX_BLOCKS = 32;
constexpr int SEG_PER_LAUNCH = 24;

enum SegFlags : int32_t {
    SEG_MASK = 1,      /* level-0 / 1-D: the mask pass writes `out` from `data`   */
    SEG_ALIGNED = 2,   /* data (and out) 16-byte aligned: float4 path              */
    SEG_MINPRUNE = 4,  /* min-weight pruning: rank k-1 = r0 select, k_minmask writes */
    SEG_KZERO = 8,     /* min-weight pruning with k = 0: nothing pruned              */
    SEG_LATE = 16,     /* k_resident: the late group (window first, then the chunk's loads) */
    SEG_FUSED = 32,    /* fused selection: a window miss is retried (MODE_RETRY), not full-scanned */
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
    int64_t cand_off;  /* this segment's candidate buckets (elements into the workspace) */
    int64_t cap;       /* nsub * bucket_cap                                              */
    int32_t nsub_log2; /* 6..10                                                          */
    int32_t bucket_cap;
    uint64_t res_step_fx; /* k_resident: (n - SAMPLE_GROUP) / (RES_MS / SAMPLE_GROUP - 1) in 32.32 fixed point;
                           * SEG_FUSED (k_fslot_collect): the number of wave slots, whose area (FslHeader,
                           * then the slots) `out` points at -- the SegDesc stays 120 bytes (k_resident's
                           * kernel argument: a larger table measured +0.2 us there) */
};
__host__ __device__ inline const uint32_t* seg_fsl(const SegDesc& sd) { return reinterpret_cast<const uint32_t*>(sd.out); }
__host__ __device__ inline int32_t seg_fsl_n(const SegDesc& sd) { return (int32_t)sd.res_step_fx; }

struct SegTable {
    int32_t nseg;
    int32_t nblk;
    int32_t nsel;      /* k_resident: selector workgroups after the nblk chunks (0: every segment selects for itself) */
    int32_t retry;     /* fused selection's retry launches: only segments whose record reads MODE_RETRY */
    uint32_t res_timeout; /* k_resident: bound of every wait, in ticks of the 100 MHz wall clock */
    int32_t pad2;
    unsigned long long* stamps; /* k_resident: [0] min start, [1] max end (100 MHz ticks); null = off */
    int32_t blk_begin[SEG_PER_LAUNCH]; /* INT32_MAX past nseg: block -> segment in one scalar sweep */
    int32_t sel_seg[SEG_PER_LAUNCH];   /* k_resident: the segment of selector j */
    SegDesc s[SEG_PER_LAUNCH];
};
static_assert(sizeof(SegTable) <= 4096, "k_resident's kernel argument");


/* per-slot selection state.  Slots are the positions of a segment inside its launch group
 * (0..SEG_PER_LAUNCH-1); the SelState slots sit at the very start of every workspace
 * layout, so every call sees the same persistent region: zeroed once by wtp_workspace_init
 * and left zeroed (counters) by every call -- k_select clears what k_collect accumulated. */
constexpr int NSHARD = 8; /* k_collect's per-segment counters are sharded by block (contention) */
/* Field groups sit on separate 128-byte lines: counters (atomics), window parameters (read by
 * every k_collect block), bucket counts. */
struct alignas(128) SelState {
    unsigned long long below[NSHARD]; /* atomicAdd (k_collect): keys < kl                    */
    unsigned long long eq_lo[NSHARD]; /* keys == kl                                          */
    unsigned long long eq_hi[NSHARD]; /* unused (keys == kh are bucketed with the inside keys) */
    unsigned long long seg_bar[NSHARD]; /* k_resident: [0] = workgroups of the segment past a full-scan select */
    uint32_t maxkey[NSHARD];          /* atomicMax (k_collect)                               */
    uint32_t overflow;                /* a block had more inside keys than it can stage     */
    uint32_t pad0a;
    unsigned long long thr_gr;        /* k_resident: the selector's threshold granule {thr bits, RES_GR_* tag} */
    uint32_t pad0[20];
    uint32_t kl, kh;                  /* window (k_collect); kh = 0xFFFFFFFF: unbounded      */
    uint32_t shift;                   /* bucket of an inside key = (key - kl - 1) >> shift   */
    int32_t mode;                     /* MODE_* chosen by the select (diagnostics)           */
    float thr32;                      /* the float32 threshold the compare uses              */
    uint32_t key_a, key_b;            /* resolved order statistics                           */
    uint32_t pad1[25];
    uint32_t sub[RES_NSUB];           /* keys per bucket (atomicAdd; k_collect uses <= NSUB_MAX) */
};
static_assert(sizeof(SelState) % 128 == 0 && sizeof(SelState) == 512 + 4 * RES_NSUB, "SelState layout");

/* The persistent head of a workspace: two SelState regions used alternately by successive
 * launch groups.  A group's k_collect accumulates into region `parity`, zeroes the other
 * region (the previous group's, whose readers have finished) and its last block flips
 * `parity`; k_mask then reads region parity ^ 1.  So no kernel has to clear state that other
 * blocks of the same kernel may still be reading. */
struct alignas(128) SelHeader {
    uint32_t parity;
    uint32_t done; /* k_collect blocks finished (last one flips parity and clears this) */
    uint32_t pad[30];
};
/* k_resident's grid barrier: one arrival counter per shard (blockIdx % 8, i.e. per XCD under
 * the round-robin placement), each on its own 128-byte line; kept in the parity region so it is
 * zero at the start of every launch that uses the region. */
struct alignas(128) BarState {
    uint32_t arrive[NSHARD][32];
};
constexpr size_t SEL_REGION = SEG_PER_LAUNCH * sizeof(SelState) + sizeof(BarState);
/* the parity word counts selection launches (every launch's last arrival adds 1); its low bit
 * picks the region */
__host__ __device__ inline SelState* sel_region(void* head, uint32_t q) {
    return reinterpret_cast<SelState*>(reinterpret_cast<char*>(head) + sizeof(SelHeader) + (size_t)(q & 1u) * SEL_REGION);
}
__host__ __device__ inline BarState* bar_region(void* head, uint32_t q) {
    return reinterpret_cast<BarState*>(reinterpret_cast<char*>(sel_region(head, q)) + SEG_PER_LAUNCH * sizeof(SelState));
}

/* MODE_RETRY: a fused segment's window missed (or its slots overflowed); the retry launches
 * (window / collect / select over P) run it again and overwrite the record */
enum SelMode : int32_t { MODE_CAND = 1, MODE_WINDOW = 2, MODE_FULL = 3, MODE_RETRY = 5, MODE_RETRIED = 8,
                         MODE_FAULT = 99 };

/* ---- fused selection (large DWT segments, every forward level in k_fwd_int) ----
 * k_fwin derives each segment's window BEFORE its forward, from the periodized transform of
 * FWIN_NP patches of FWIN_PS^2 input samples (= M_SAMPLE_WIN coefficients in the population's
 * level proportions); every k_fwd_int wave then classifies the coefficients it writes to P against
 * it (counts below / equal to kl into the segment's SelState, the keys inside (kl, kh] into a slot
 * of its own: FSL_WORDS words, the count then up to FSL_KEYS keys; more sets the overflow flag and
 * sends the segment to the exact full-scan select), and k_fslot_collect buckets the slots' keys
 * as k_collect buckets a chunk's -- so P is never re-read for the selection. */
constexpr int FSL_WORDS = 64;
constexpr int FSL_KEYS = FSL_WORDS - 1;
constexpr int FWIN_PS = 128;
constexpr int FWIN_NP = 4;
constexpr int FWIN_THREADS = 1024;
constexpr int FSC_THREADS = 256; /* k_fslot_collect: 64 wave slots per wave, a slot word per lane */
constexpr int FSC_SLOTS = 64 * (FSC_THREADS / 64);
constexpr int FWIN_F_MAX = 18;   /* k_fwd_int's longest filter */
static_assert(FWIN_NP * FWIN_PS * FWIN_PS == M_SAMPLE_WIN, "k_fwin's sample is k_window's");
/* The head of a fused tensor's slot area: its window (k_fwin) and the forward's counters -- the
 * forward never touches the SelState regions, so a group's bucket pass and select can run on the
 * side stream while the next group's forward runs (the areas are double-buffered by group parity);
 * k_fslot_collect copies it into its SelState slot. */
struct alignas(256) FslHeader {
    /* the window on a line of its own: every forward workgroup reads it, and a line that also
     * took the counters' atomics would be re-fetched by each (measured: the level-1 forward
     * 785 -> 1361 us with window and counters on shared lines) */
    uint32_t kl, kh, shift;
    uint32_t pad0[29];
    /* per forward workgroup ONE 64-bit add of {keys == kl : keys < kl} (each < 2^32 per tensor)
     * and one max: per-wave adds of separate counters measured ~9 % of the level-1 forward (the
     * atomic units' queue on these few lines) */
    unsigned long long be[NSHARD];
    uint32_t maxkey[NSHARD];
    uint32_t overflow;
    uint32_t pad1[7];
    uint32_t pad2[32];
};
static_assert(sizeof(FslHeader) == 512, "FslHeader lines");
constexpr int FSL_HDR_WORDS = (int)(sizeof(FslHeader) / 4);
struct FwdSel { /* k_fwd_int's fused-selection argument (on = 0: off) */
    int32_t on, pad;
    FslHeader* hdr[SEG_PER_LAUNCH];    /* per item of the launch: its tensor's slot-area head */
    uint32_t* slots[SEG_PER_LAUNCH];   /* per item: its wave slots for this launch's tiles */
};
struct FwinSeg {
    const float* in; /* the segment's input images (B x R x C) */
    FslHeader* hdr;  /* the window goes here (its counters are zeroed) */
    int64_t n, r0;
    int32_t above, nsub_log2, B, R, C, L;
};
struct FwinTable {
    int32_t nseg, F;
    float lo[FWIN_F_MAX], hi[FWIN_F_MAX];
    uint32_t* gh; /* the per-segment histograms (Layout::fwh): zero when the launch starts */
    FwinSeg s[SEG_PER_LAUNCH];
};
/* k_fwin's per-segment histogram (NB bins) and arrival counter: zeroed once per call that has a
 * fused group (a memset), re-zeroed by each segment's last patch block for the next group */
constexpr int FWIN_HW = (NB + 1 + 31) / 32 * 32;
constexpr size_t FWIN_HIST_BYTES = (size_t)SEG_PER_LAUNCH * FWIN_HW * 4;

/* filter taps as a kernel argument (scalar-loaded, uniform across the wave) */
struct Taps {
    int32_t F;
    int32_t pad[3];
    float f[4][WTP_MAX_F]; /* dec_lo, dec_hi, rec_lo, rec_hi */
};

/* ---- launchers (kernels.hip) ---- */
void launch_window(const SegTable& t, SelHeader* head, hipStream_t s, const wtp_result* res = nullptr);
/* the fused selection's retry of the segments whose select read MODE_RETRY (t.retry = 1, chunk
 * units): k_window, a grid-stride k_collect over their chunks, k_mask_select -- a few us when
 * no segment missed */
void launch_fused_retry(const SegTable& t, SelHeader* head, uint32_t* cand, wtp_result* res, float* thr_out,
                        hipStream_t s);
void launch_collect(const SegTable& t, SelHeader* head, uint32_t* cand, wtp_result* res, hipStream_t s);
void launch_mask_select(const SegTable& t, SelHeader* head, const uint32_t* cand, wtp_result* res, float* thr_out,
                        hipStream_t s);
/* after launch_mask_select: the in-place level-0 segments whose select fell back to the full scan */
void launch_mask_inplace(const SegTable& t, const wtp_result* res, const float* thr, hipStream_t s);
/* one-launch level-0 prune (k_resident): every segment SEG_MASK, blk_begin in RES_CHUNK units,
 * t.nblk <= resident_capacity() */
constexpr int RES_THREADS = 512;
constexpr int RES_IT = 24;                          /* float4 per thread held in VGPRs */
constexpr int RES_CHUNK = RES_THREADS * RES_IT * 4; /* 49152 elements per workgroup   */
/* k_resident's window sample: RES_MS keys per segment, loaded by the first RES_SW waves of every
 * workgroup (RES_SPL per lane) ahead of the chunk's loads */
constexpr int RES_MS = 4096;
constexpr int RES_SW = 4;
constexpr int RES_SPL = RES_MS / (64 * RES_SW);
/* a wave may have at most 63 vector-memory instructions outstanding: the sample's loads and
 * the chunk's must all be in flight together */
static_assert(RES_SPL + RES_IT <= 63 && RES_SPL * 64 * RES_SW == RES_MS, "k_resident sample geometry");
/* k_resident's window margin in binomial sigmas x 100 (+ 8 sample ranks): a miss costs a full
 * scan of the segment, 4 sigma makes that ~1e-4 per segment; the three-launch form keeps 6 + 24 */
constexpr int RES_SIGMA_X100 = 400;
constexpr int RES_MAX_WG = 256;                     /* workgroups a resident launch may hold (<= CUs) */
/* the late group: the smallest segments of a launch group, together at most this percentage of
 * its workgroups; their workgroups issue their chunk's loads only once their window is known, so
 * the early group's chunks come off HBM first and its select overlaps the late group's stream
 * (round 5, with selector workgroups, cfg2: 0 / 25 / 45 / 60 / 80 / 99 % -> 28.1 / 27.8 / 26.1 /
 * 25.85 / 27.6 / 27.8 us, A/B on one box; 60 % puts one of the three 48-workgroup layers late) */
constexpr int RES_LATE_PCT = 60;
constexpr int RES_STG = 32;                         /* inside keys a thread may stage (of its 96; ~11 expected) */
/* After the first segment barrier every workgroup publishes the keys of the (one or two)
 * buckets holding the segment's ranks in a slot of its own: word 0 the count, then the keys */
/* one workgroup's published region in the candidate area: its bucket offsets (RES_NSUB + 1 words,
 * padded to 16 bytes), then its inside keys bucket-sorted (at most RES_STG per thread).  (Round 4
 * measured fixed per-bucket slots read in one round trip instead: the 16-byte granules scattered
 * over 1024 slots are partial-line write-through stores, k_resident 28.0 -> 30.5 us.) */
constexpr int RES_PUB_KEYS = (RES_NSUB + 1 + 3) / 4 * 4;
constexpr int RES_PUB_WORDS = RES_PUB_KEYS + RES_STG * RES_THREADS;
constexpr int RES_WG_WORDS = RES_PUB_WORDS;
constexpr int RES_SEL_MAX = 1024;                   /* keys the one-wave select takes (more: full scan) */
/* a wait this long means the grid is not co-resident: 2 ms, about 75x a cfg2 k_resident launch
 * (26 us) and 60x a cfg3 k_small launch -- every wait inside a co-resident launch ends in a few us.
 * A grid that is not co-resident (another stream's kernels hold CUs) costs at most this bound plus
 * the three-launch re-run of its tensors; the round-5 bound was 200 ms (tests/test_gpu_resident.py,
 * test_two_full_calls_on_two_streams / test_resident_beside_long_kernels measure the cases) */
constexpr uint32_t RES_TIMEOUT_DEFAULT_US = 2000;
int resident_capacity();
/* every resident wait's bound (k_resident, k_small), clamped to RES_TIMEOUT_MAX_US so that the
 * bound in 100 MHz ticks fits 32 bits; returns the previous one */
constexpr uint32_t RES_TIMEOUT_MAX_US = 40000000u;
uint32_t set_resident_timeout_us(uint32_t us);
void set_kernel_stamps(unsigned long long* dev); /* k_resident / k_small launch span stamps (measurement) */
uint32_t resident_timeout_us();
unsigned long long* kernel_stamps();
constexpr uint32_t RES_POISON = 0x80000000u; /* a segment barrier counter whose wait timed out */
/* the tag of a selector's threshold granule (SelState::thr_gr, high word; 0 = not yet) */
constexpr uint32_t RES_GR_OK = 1u;     /* the low word is the float32 threshold */
constexpr uint32_t RES_GR_ALL = 2u;    /* the window missed: every float4 is rewritten */
constexpr uint32_t RES_GR_FAULT = 4u;  /* a wait timed out: nobody stores */
void launch_resident(const SegTable& t, SelHeader* head, uint32_t* cand, wtp_result* res, float* thr_out,
                     hipStream_t s);
/* ---- the small-population path in one launch (small.hip, k_small) ----
 * every tensor of the call is a 2-D transform whose tiles fit one workgroup's LDS; one
 * workgroup per tile, the tiles of a tensor are its segment (small_geom.h) */
constexpr int SM_MAX_SEG = 4;       /* tensors per call */
constexpr int SM_SEG_WG_MAX = 128;  /* workgroups per tensor */
constexpr int SM_SLOT_WORDS = 64;   /* per workgroup in the candidate region: the keys of the rank's bin */
constexpr int SM_ARENA = 34 * 1024; /* LDS words of a workgroup's arena (136 KB) */
constexpr int SM_F_MAX = 20;        /* longest filter */
constexpr int SM_LMAX = 10;         /* = SM_MAX_L of small_geom.h */
constexpr int SM_WIN_WORDS = 480;   /* the tiles' windows, computed by the host (small_geom.h): per tile row
                                       and per tile column 2 (L + 1) words, level k's fw and sv */
constexpr int SM_LINE_MAX = 32767;  /* window ends packed in 16 bits */
struct SmallSeg {
    const float* in;
    float* out;
    float* P;         /* packed coefficients (workspace), B images of PR x PC */
    int64_t r0;       /* lower order statistic of the population          */
    double gamma;
    int64_t numel;
    int64_t n;        /* population: B * PR * PC                          */
    int32_t B, L, PR, PC;
    int32_t R[SM_LMAX + 1], C[SM_LMAX + 1], offR[SM_LMAX + 1], offC[SM_LMAX + 1];
    int32_t TR, TC, tilesR, tilesC; /* tile size at level L, tiles per image  */
    int32_t wg_begin, nwg, res, above, npad;
    int32_t win_off; /* this tensor's lines in SmallTable::win: tilesR row lines, then tilesC column lines */
};
struct SmallTaps { /* the filter in the kernel argument: only as many taps as the path takes */
    int32_t F;
    int32_t pad[3];
    float f[4][SM_F_MAX]; /* dec_lo, dec_hi, rec_lo, rec_hi */
};
struct SmallTable {
    int32_t nseg, nblk;
    uint32_t timeout; /* set by launch_small */
    int32_t pad;
    unsigned long long* stamps;
    uint32_t* slots;              /* SM_SLOT_WORDS per workgroup (the workspace's candidate region) */
    int32_t wg_begin[SM_MAX_SEG]; /* INT32_MAX past nseg */
    SmallSeg s[SM_MAX_SEG];
    SmallTaps tp;
    uint32_t win[SM_WIN_WORDS];
};
static_assert(sizeof(SmallTable) <= 4096, "k_small's kernel argument");
void launch_small(const SmallTable& t, SelHeader* head, wtp_result* res, hipStream_t s);
/* workgroups k_small may launch at once on the current device (one per CU, every F instance
 * checked by the occupancy query); 0: never used */
int small_capacity();

/* min-weight pruning after window + collect: mp = 16 B per tensor, tiecnt = one u32 per
 * streaming block */
void launch_minprune(const SegTable& t, SelHeader* head, const uint32_t* cand, wtp_result* res, float* thr_out,
                     void* mp, uint32_t* tiecnt, hipStream_t s);

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
/* filterbank.hip: one fused, LDS-tiled launch per level (and per group of images) */
bool fb_tiled_ok(int64_t B, int64_t R, int64_t C, const Taps& tp);
struct FwdItem { /* one image batch's analysis level k: (B, R, C) in -> P details, anext */
    const float* in;
    int64_t B, R, C;
    float* anext;
    float* P;
    int64_t PR, PC, offR, offC;
    int last;
    uint32_t* fslot = nullptr; /* fused selection: the item's wave slots for this level (null: off) */
    FslHeader* fhdr = nullptr; /* ... and its tensor's slot-area head */
};
/* fused selection: the wave slots one forward level of (B, R, C) images fills (k_fwd_int's tiles
 * x waves); false when some launch of that level would not be k_fwd_int (no classification) */
bool fwd_level_fused_ok(const FwdItem& x, const Taps& tp, int64_t* slots, bool any_mode = false);
void launch_fwin(const FwinTable& t, SelHeader* head, hipStream_t s);
void launch_fslot_collect(const SegTable& t, SelHeader* head, uint32_t* cand, wtp_result* res, hipStream_t s);
struct InvItem { /* one image batch's synthesis level k -> y (B, outH, outW) */
    const float* a_src; /* nullptr: the packed cA */
    int64_t a_bs, lda;
    int a_from_P;
    const float* P;
    int64_t PR, PC, offR, offC, B, R, C;
    const float* thr;
    float* y;
    int64_t outH, outW;
    unsigned long long* zc;
};
void launch_fwd_levels(const FwdItem* it, int n, const Taps& tp, hipStream_t s, bool fused = false);
void launch_inv_levels(const InvItem* it, int n, const Taps& tp, hipStream_t s);
int fb_set_interior(int mode); /* filter-bank kernel choice 0..2 (wtp_set_interior); returns the previous */
void launch_fwd_level(const float* in, int64_t B, int64_t R, int64_t C, const Taps& tp, float* anext, float* P,
                      int64_t PR, int64_t PC, int64_t offR, int64_t offC, int last, hipStream_t s);
void launch_inv_level(const float* a_src, int64_t a_bs, int64_t lda, int a_from_P, const float* P, int64_t PR,
                      int64_t PC, int64_t offR, int64_t offC, int64_t B, int64_t R, int64_t C, const Taps& tp,
                      const float* thr, float* y, int64_t outH, int64_t outW, unsigned long long* zc,
                      hipStream_t s);
void launch_copy_threshold(const float* P, float* out, int64_t n, const float* thr, unsigned long long* zc,
                           hipStream_t s);
/* random pruning: one segment per tensor, block ranges per kernel */
struct RandSeg {
    const float* in;
    float* out;
    int64_t numel;
    int64_t k;     /* positions to zero (torch.randperm(n)[:prune_count] semantics) */
    uint64_t key;  /* wt_perm_key(seed, tensor index) */
    int32_t h;     /* wt_perm_half_bits(numel) */
    int32_t res;
};
struct RandTable {
    int32_t nseg;
    int32_t pad;
    int32_t copy_begin[SEG_PER_LAUNCH + 1]; /* k_rand_copy blocks of CHUNK elements */
    int32_t zero_begin[SEG_PER_LAUNCH + 1]; /* k_rand_zero blocks of STREAM_THREADS positions */
    RandSeg s[SEG_PER_LAUNCH];
};
void launch_random_prune(const RandTable& t, wtp_result* res, hipStream_t s);
void launch_count_small(const float* x, int64_t n, float thr, unsigned long long* count, hipStream_t s);
/* 1-D flattened mode (one line per tensor) */
void launch_dwt1_level(const float* x, int64_t N, const Taps& tp, float* a, float* d, hipStream_t s);
void launch_idwt1_level(const float* a, int a_thr, const float* d, int64_t N, const Taps& tp, const float* thr,
                        float* y, int64_t outN, unsigned long long* zc, hipStream_t s);
void launch_synth(float* out, int64_t n, uint64_t seed, uint32_t tid, int e, hipStream_t s);

}  // namespace wtp

#endif
