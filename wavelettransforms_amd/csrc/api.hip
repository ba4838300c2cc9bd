/*
 * api.hip -- host side of libwtprune.so: validation in the reference's order, workspace
 * layout, segment tables and the launch sequence of one multi_resolution_analysis call
 * (ResNet/dwt_pruning.py:35-95).  No allocation, no synchronisation: everything is
 * stream-ordered and graph-capturable.
 */
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "wtp_internal.h"
#include "small_geom.h"
#include "wt_filters.inc"
#include "wt_perm.h"

using namespace wtp;

namespace {

thread_local std::string g_err;
thread_local int g_err_tensor = -1;
thread_local hipEvent_t g_stage_ev[8];
thread_local int g_stage_n = 0;
std::atomic<int> g_resident{1}; /* wtp_set_resident */
std::atomic<int> g_pipeline{1}; /* wtp_set_pipeline */
std::atomic<int> g_fused{1};    /* wtp_set_fused_select */

inline void stage(int i, hipStream_t s) {
    if (i < g_stage_n && g_stage_ev[i]) (void)hipEventRecord(g_stage_ev[i], s);
}

int fail(int code, int tensor, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(int code, int tensor, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    g_err_tensor = tensor;
    return code;
}

constexpr size_t ALIGN = 256;
inline size_t align_up(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

Taps make_taps(int wid) {
    Taps tp;
    memset(&tp, 0, sizeof tp);
    const int F = wt_flen[wid];
    tp.F = F;
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < F; ++j) {
            uint32_t b = wt_taps_bits[wt_foff[wid] + k * F + j];
            memcpy(&tp.f[k][j], &b, 4);
        }
    return tp;
}

int max_level(int64_t n, int F) {
    if (F < 2) return -1;
    if (n < F - 1) return 0;
    int L = 0;
    while (((int64_t)(F - 1) << (L + 1)) <= n && L < 62) ++L;
    return L;
}

/* One tensor of the call, as the reference would see it. */
struct TPlan {
    int ndim = 0;
    int64_t numel = 0;
    int64_t B = 1, H = 1, W = 1;
    int L = 0;
    bool dwt = false;     /* wavelet transform actually runs (ndim >= 2 and L >= 1)    */
    int64_t pop = 0;      /* selection population: numel, or the packed coefficient count */
    bool tight = true;
    wt_level_geom g;
    int64_t cap = 0;      /* candidate capacity                                         */
    size_t p_off = 0;     /* workspace byte offset of the packed array (dwt only)       */
    size_t cand_off = 0;  /* element offset into the candidate region                   */
    size_t t_off = 0;     /* workspace byte offset of this tensor's three level temps      */
    size_t t_elems = 0;   /* elements per temp                                              */
    bool flat = false;    /* 1-D flattened mode: pywt.wavedec / waverec of the flat tensor   */
    int64_t f_slots = 0;  /* fused selection: k_fwd_int wave slots of its forward (0: never fused) */
    size_t f_off = 0;     /* workspace byte offset of its slot area (per group parity and slot) */
    int64_t len[34] = {}; /* flat: len[0] = numel, len[k] = ceil(len[k-1] / 2)              */
};

struct Layout {
    size_t hist = 0, sel = 0, thr = 0, cand = 0, P = 0, total = 0;
    size_t fwh = 0; /* k_fwin's histograms (when some tensor can be fused) */
};

/* persistent slot region: identical position and size in every layout */
constexpr size_t PERSIST_BYTES = ((sizeof(SelHeader) + 2 * SEL_REGION) + 255) / 256 * 256;

bool pct_ok(double pct) { return pct >= 0.0 && pct <= 100.0; }

/* candidate buckets of the three-launch form: ~1000 keys of 5% of the population per bucket
 * (64..1024 buckets; the window holds ~5-6%) with capacity for 4x that (an overflowing bucket
 * sends the select to its exact full-scan path).  A DWT segment's select runs once (its first
 * k_mask_select block), so its buckets hold ~2000 keys -- still one LDS stage for the select
 * (MS_STAGE), twice as long runs per k_collect block (its ~900 inside keys are ~1 key per bucket
 * at 1024 buckets: partial-line stores, 4x the candidate bytes).  64 buckets cut those stores to
 * 1.2x but the select then radix-selects ~28K keys from L2 (+55 us per launch on cfg5, more
 * than k_collect saved).  The resident form always uses NSUB_MAX buckets: its runs are per
 * workgroup, and narrow buckets let one LDS histogram finish the select. */
void bucket_plan(int64_t n, int* nsub_log2, int* bucket_cap, bool dwt) {
    /* a segment too large for the inline window always gets k_window's M_SAMPLE_WIN-key window:
     * 2 (6 sigma + 24) sample ranks wide, plus the bins' outward rounding */
    const double m = (double)M_SAMPLE_WIN;
    const double wfrac = n > (int64_t)WINDOW_INLINE_MAX_BLOCKS * CHUNK ? (6.0 * sqrt(m) + 48.0) / m + 0.005 : 0.05;
    const double expect = wfrac * (double)n;
    int lg = 6;
    while (lg < 10 && (double)(1 << lg) * (dwt ? 2048.0 : 1024.0) < expect) ++lg;
    int64_t bc = (int64_t)(4.0 * expect / (double)(1 << lg)) + 1;
    if (bc < 256) bc = 256;
    if (bc > (dwt ? BUCKET_MAX_DWT : BUCKET_MAX)) bc = dwt ? BUCKET_MAX_DWT : BUCKET_MAX;
    *nsub_log2 = lg;
    *bucket_cap = (int)bc;
}

int64_t cap_for(int64_t n, bool dwt) {
    int lg, bc;
    bucket_plan(n, &lg, &bc, dwt);
    return (int64_t)bc << lg;
}

/* Validate and plan every tensor in the reference's order; returns WTP_OK or the first error. */
int plan_tensors(const wtp_tensor* ts, int n, int wid, int level, double pct, bool check_ptrs,
                 std::vector<TPlan>& out, bool carry = true, bool flat = false) {
    out.assign(n, TPlan());
    int cur_level = level;
    for (int t = 0; t < n; ++t) {
        if (!carry) cur_level = level;
        const wtp_tensor& x = ts[t];
        TPlan& p = out[t];
        if (x.ndim < 0 || x.ndim > WTP_MAX_DIMS) return fail(WTP_EARG, t, "tensor %d: ndim %d unsupported", t, x.ndim);
        p.ndim = x.ndim;
        p.numel = 1;
        for (int d = 0; d < x.ndim; ++d) {
            if (x.shape[d] < 0) return fail(WTP_EARG, t, "tensor %d: negative dimension", t);
            p.numel *= x.shape[d];
        }
        if (check_ptrs && p.numel > 0 && (!x.in || !x.out)) return fail(WTP_EARG, t, "tensor %d: null pointer", t);
        if (x.ndim < 2) {
            /* dwt_pruning.py:58-62 -- plain percentile, no wavelet lookup */
            if (!pct_ok(pct)) return fail(WTP_EBADPCT, t, "Percentiles must be in the range [0, 100]");
            if (p.numel == 0) return fail(WTP_EEMPTY, t, "index -1 is out of bounds for axis 0 with size 0");
            p.L = cur_level;
            p.pop = p.numel;
        } else if (flat) {
            /* 1-D flattened mode: pywt.wavedec(w.ravel(), wavelet, 'periodization', level) with
             * the level clamped as calculate_max_level clamps it for the 2-D path (:12-13, :64-65) */
            if (wid < 0 || wid >= WT_NUM_WAVELETS)
                return fail(WTP_EBADWAVELET, t, "Unknown wavelet name, check wavelist() for the list of available builtin wavelets.");
            p.flat = true;
            const int maxL = max_level(p.numel, wt_flen[wid]);
            if (maxL < cur_level) cur_level = maxL;
            p.L = cur_level;
            if (p.L < 0) return fail(WTP_EBADLEVEL, t, "Level value of %d is too low . Minimum level is 0.", p.L);
            if (p.L > 32) return fail(WTP_EARG, t, "tensor %d: level %d unsupported", t, p.L);
            if (!pct_ok(pct)) return fail(WTP_EBADPCT, t, "Percentiles must be in the range [0, 100]");
            p.len[0] = p.numel;
            for (int k = 1; k <= p.L; ++k) p.len[k] = (p.len[k - 1] + 1) / 2;
            p.pop = p.len[p.L];
            for (int k = 1; k <= p.L; ++k) p.pop += p.len[k];
            if (p.pop == 0) return fail(WTP_EEMPTY, t, "index -1 is out of bounds for axis 0 with size 0");
            p.dwt = p.L > 0;
        } else {
            if (wid < 0 || wid >= WT_NUM_WAVELETS)
                return fail(WTP_EBADWAVELET, t, "Unknown wavelet name, check wavelist() for the list of available builtin wavelets.");
            p.H = x.shape[x.ndim - 2];
            p.W = x.shape[x.ndim - 1];
            p.B = 1;
            for (int d = 0; d < x.ndim - 2; ++d) p.B *= x.shape[d];
            const int maxL = max_level(p.H < p.W ? p.H : p.W, wt_flen[wid]);
            if (maxL < cur_level) cur_level = maxL; /* :64-65, carried to later tensors */
            p.L = cur_level;
            if (p.L < 0) return fail(WTP_EBADLEVEL, t, "Level value of %d is too low . Minimum level is 0.", p.L);
            if (p.L > 32) return fail(WTP_EARG, t, "tensor %d: level %d unsupported", t, p.L);
            wt_geom(p.H, p.W, p.L, &p.g);
            p.pop = p.B * p.g.PR * p.g.PC;
            if (!pct_ok(pct)) return fail(WTP_EBADPCT, t, "Percentiles must be in the range [0, 100]");
            if (p.pop == 0) return fail(WTP_EEMPTY, t, "index -1 is out of bounds for axis 0 with size 0");
            p.dwt = p.L > 0;
            if (p.dwt) {
                int64_t nc = p.g.R[p.L] * p.g.C[p.L];
                for (int k = 1; k <= p.L; ++k) nc += 3 * p.g.R[k] * p.g.C[k];
                p.tight = nc == p.g.PR * p.g.PC;
                /* waverec2 yields (2R1, 2C1); the 4-index crop of :79-82 then fails for 2-D/3-D
                 * tensors (IndexError), cannot crop W for 5-D or anything for >= 6-D (the
                 * later .view(original_shape) raises RuntimeError) */
                const bool hbad = 2 * p.g.R[1] != p.H, wbad = 2 * p.g.C[1] != p.W;
                if ((x.ndim < 4 && (hbad || wbad)) || (x.ndim == 5 && wbad) || (x.ndim >= 6 && (hbad || wbad)))
                    return fail(WTP_ECROP, t, x.ndim < 4 ? "tuple index out of range"
                                                         : "shape is invalid for input of this size");
            }
        }
        /* selection counts are kept in 32 bits on the device (8 GiB of float32 per tensor) */
        if (p.pop > (int64_t)INT32_MAX) return fail(WTP_EARG, t, "tensor %d: more than 2^31-1 coefficients", t);
        p.cap = cap_for(p.pop, p.dwt);
    }
    return WTP_OK;
}

/* Elements one level temp of tensor p needs: the largest intermediate its forward and inverse
 * write to a temp, level by level, with the kernels forward_chains / inverse_chains pick (tiled:
 * the next approximation / the synthesis output below level 1; per-point: the column pass's two
 * outputs / the row pass's two outputs).  Level 1's synthesis writes the caller's output. */
size_t temp_elems(const TPlan& p, const Taps& tp) {
    if (p.flat) return (size_t)p.numel + 2; /* two ping-pong lines of up to numel + 1 samples */
    int64_t need = 0;
    for (int k = 1; k <= p.L; ++k) {
        const int64_t R0 = p.g.R[k - 1], C0 = p.g.C[k - 1], R = p.g.R[k], C = p.g.C[k];
        need = std::max(need, p.B * R * (fb_tiled_ok(p.B, R0, C0, tp) ? C : C0));
        if (!fb_tiled_ok(p.B, 2 * R, 2 * C, tp)) need = std::max(need, p.B * R * 2 * C);
        if (k >= 2) need = std::max(need, p.B * 4 * R * C);
    }
    return (size_t)need;
}

/* Fused selection (wtp_internal.h, FwdSel / k_fwin / k_fslot_collect): a tensor qualifies when
 * it is large (its window pass and bucket pass are then small beside the P re-read they replace),
 * tight (every packed coefficient is written by the forward: no padding zeros in the population),
 * its images hold k_fwin's patches and its level count leaves them at least 4 x 4, and every
 * forward level runs in k_fwd_int.  Returns the wave slots of its forward, 0 when it does not
 * qualify.  `sizing`: the workspace query -- the interior mode and the input's alignment are
 * not known yet, so the slots are reserved whenever the shape qualifies. */
constexpr int64_t FUSED_MIN_POP = (int64_t)1 << 22;
int64_t fused_slot_count(const TPlan& p, const float* in, const Taps& tp, bool sizing) {
    if (!p.dwt || p.flat || !p.tight || p.L < 1 || p.L > 6 || p.pop < FUSED_MIN_POP) return 0;
    if (p.g.R[0] < FWIN_PS || p.g.C[0] < FWIN_PS) return 0;
    int64_t tot = 0;
    for (int k = 1; k <= p.L; ++k) {
        /* level 1 reads the caller's input, the others a 256-byte aligned temp */
        const float* src = (k == 1 && !sizing) ? in : reinterpret_cast<const float*>((uintptr_t)ALIGN);
        const FwdItem x{src, p.B, p.g.R[k - 1], p.g.C[k - 1], nullptr, nullptr, p.g.PR, p.g.PC, p.g.offR[k], p.g.offC[k],
                        k == p.L};
        int64_t sl = 0;
        if (!fwd_level_fused_ok(x, tp, &sl, sizing)) return 0;
        tot += sl;
    }
    return tot;
}

Layout make_layout(std::vector<TPlan>& ps, const Taps& tp) {
    Layout L;
    L.hist = 0;
    L.sel = 0;
    size_t off = PERSIST_BYTES;
    L.thr = off;
    off = align_up(off + ps.size() * sizeof(float));
    L.cand = off;
    size_t ce = 0;
    for (auto& p : ps) { p.cand_off = ce; ce += (size_t)p.cap; }
    /* a resident launch (k_resident) keeps one published region of RES_WG_WORDS per workgroup there instead */
    int64_t rwg = 0;
    for (auto& p : ps)
        if (!p.dwt) rwg += (p.pop + RES_CHUNK - 1) / RES_CHUNK;
    ce = std::max(ce, (size_t)std::min<int64_t>(rwg, RES_MAX_WG) * RES_WG_WORDS);
    /* the one-launch small path keeps one slot of SM_SLOT_WORDS per workgroup there */
    ce = std::max(ce, (size_t)RES_MAX_WG * SM_SLOT_WORDS);
    off = align_up(off + ce * sizeof(uint32_t));
    L.P = off;
    for (auto& p : ps) {
        if (!p.dwt) continue;
        p.p_off = off;
        off = align_up(off + (size_t)p.pop * sizeof(float));
    }
    /* level temps per launch-group SLOT (tensor t uses slot t % SEG_PER_LAUNCH), not per tensor:
     * the same level of one launch group's tensors runs as one grouped launch, so their temps are
     * live together, but the groups' transforms run one group after another on the caller's
     * stream (prune_impl; the side stream only selects from P), so group g + 1 reuses group g's
     * temps.  cfg5 (64 x 4096^2, db8 L5): 24 slots x 3 x 16.8 MB instead of 64 x 3 x 67 MB */
    size_t slot_elems[SEG_PER_LAUNCH] = {};
    for (size_t t = 0; t < ps.size(); ++t)
        if (ps[t].dwt) slot_elems[t % SEG_PER_LAUNCH] = std::max(slot_elems[t % SEG_PER_LAUNCH], temp_elems(ps[t], tp));
    size_t slot_off[SEG_PER_LAUNCH] = {};
    for (int j = 0; j < SEG_PER_LAUNCH; ++j) {
        if (!slot_elems[j]) continue;
        slot_off[j] = off;
        off = align_up(off + 3 * align_up(slot_elems[j] * sizeof(float)));
    }
    for (size_t t = 0; t < ps.size(); ++t) {
        if (!ps[t].dwt) continue;
        ps[t].t_off = slot_off[t % SEG_PER_LAUNCH];
        ps[t].t_elems = slot_elems[t % SEG_PER_LAUNCH];
    }
    /* fused selection's wave slots, also per launch-group slot: a fused group's bucket pass reads
     * them before the next group's forward writes its own */
    size_t fsl_words[SEG_PER_LAUNCH] = {};
    for (size_t t = 0; t < ps.size(); ++t) {
        ps[t].f_slots = fused_slot_count(ps[t], nullptr, tp, true);
        if (ps[t].f_slots)
            fsl_words[t % SEG_PER_LAUNCH] =
                std::max(fsl_words[t % SEG_PER_LAUNCH], (size_t)FSL_HDR_WORDS + (size_t)ps[t].f_slots * FSL_WORDS);
    }
    /* two sets when the call has several groups: group g uses set g & 1, so group g + 1's forward
     * fills its slots while group g's bucket pass (side stream) still reads its own */
    const int nsets = ps.size() > (size_t)SEG_PER_LAUNCH ? 2 : 1;
    size_t fsl_off[2][SEG_PER_LAUNCH] = {};
    for (int k = 0; k < nsets; ++k)
        for (int j = 0; j < SEG_PER_LAUNCH; ++j) {
            if (!fsl_words[j]) continue;
            fsl_off[k][j] = off;
            off = align_up(off + fsl_words[j] * sizeof(uint32_t));
        }
    bool anyf = false;
    for (size_t t = 0; t < ps.size(); ++t)
        if (ps[t].f_slots) { ps[t].f_off = fsl_off[(t / SEG_PER_LAUNCH) & 1][t % SEG_PER_LAUNCH]; anyf = true; }
    if (anyf) {
        L.fwh = off;
        off = align_up(off + FWIN_HIST_BYTES);
    }
    L.total = off;
    return L;
}

void seg_ranks(int64_t n, double pct, SegDesc& sd) {
    /* numpy/lib/function_base.py: q = pct/100 (:4279); linear vi = (n-1)*q (:110);
     * _get_indexes (:4730-4763): vi >= n-1 -> index -1 (the max), gamma = vi - (-1) */
    const double q = pct / 100.0;
    const double vi = (double)(n - 1) * q;
    if (vi >= (double)(n - 1)) {
        sd.above = 1;
        sd.r0 = n - 1;
        sd.gamma = vi - (-1.0);
    } else {
        const double fl = std::floor(vi);
        sd.above = 0;
        sd.r0 = (int64_t)fl;
        sd.gamma = vi - fl;
    }
}

inline char* wsb(void* ws, size_t off) { return static_cast<char*>(ws) + off; }

int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WTP_EHIP, -1, "HIP: %s", hipGetErrorString(e));
    return WTP_OK;
}

/* one image batch's transform chain: its input / output, packed array and three level temps */
struct Chain {
    const TPlan* p;
    const float* in;   /* forward input */
    float* out;        /* inverse output */
    float* P;
    float* T[3];
    const float* thr;
    unsigned long long* zc;
    uint32_t* fsl = nullptr; /* fused selection: the tensor's slot area (null: not fused) */
};

/* pywt.wavedec2 (dwt_pruning.py:67-68) of every chain into its packed layout.  Level k of all
 * chains is ONE tiled launch (filterbank.hip) where the level is large enough, else the two
 * per-point passes of that chain.  Each approximation ping-pongs between the chain's own temps
 * so no launch reads what it writes. */
void forward_chains(const std::vector<Chain>& cs, const Taps& tp, hipStream_t s, bool fused = false) {
    int maxL = 0;
    for (const Chain& c : cs) maxL = std::max(maxL, c.p->L);
    std::vector<const float*> cur(cs.size());
    for (size_t j = 0; j < cs.size(); ++j) cur[j] = cs[j].in;
    std::vector<uint32_t*> fcur(cs.size()); /* fused selection: each chain's next level's slots */
    for (size_t j = 0; j < cs.size(); ++j) fcur[j] = (fused && cs[j].fsl) ? cs[j].fsl + FSL_HDR_WORDS : nullptr;
    std::vector<FwdItem> items;
    for (int k = 1; k <= maxL; ++k) {
        items.clear();
        for (size_t j = 0; j < cs.size(); ++j) {
            const TPlan& p = *cs[j].p;
            if (p.L < k) continue;
            float *tL = cs[j].T[0], *tH = cs[j].T[1], *tA = cs[j].T[2];
            const int64_t R0 = p.g.R[k - 1], C0 = p.g.C[k - 1];
            if (fb_tiled_ok(p.B, R0, C0, tp)) {
                float* an = (cur[j] == tA) ? tL : tA;
                items.push_back(FwdItem{cur[j], p.B, R0, C0, an, cs[j].P, p.g.PR, p.g.PC, p.g.offR[k], p.g.offC[k],
                                        k == p.L});
                int64_t sl = 0;
                if (fcur[j] && fwd_level_fused_ok(items.back(), tp, &sl)) { /* prune_impl checked every level */
                    items.back().fslot = fcur[j];
                    items.back().fhdr = reinterpret_cast<FslHeader*>(cs[j].fsl);
                    fcur[j] += sl * FSL_WORDS;
                }
                cur[j] = an;
            } else {
                float* t0 = (cur[j] == tL) ? tA : tL;
                float* t1 = (cur[j] == tH) ? tA : tH;
                float* an = (cur[j] == tL || cur[j] == tH || cur[j] == tA) ? const_cast<float*>(cur[j]) : tA;
                launch_dwt_cols(cur[j], p.B, R0, C0, tp, t0, t1, s);
                launch_dwt_rows(t0, t1, p.B, p.g.R[k], C0, tp, an, cs[j].P, p.g.PR, p.g.PC, p.g.offR[k], p.g.offC[k],
                                k == p.L, s);
                cur[j] = an;
            }
        }
        if (!items.empty()) launch_fwd_levels(items.data(), (int)items.size(), tp, s, fused);
    }
}

/* pywt.waverec2 (dwt_pruning.py:75-77) of every chain from its packed layout, thresholding the
 * packed coefficients as they are loaded (the np.where of :31), cropping and counting zeros on
 * the last level (:79-88).  Level k of all chains is one launch, as in forward_chains(). */
void inverse_chains(const std::vector<Chain>& cs, const Taps& tp, hipStream_t s) {
    int maxL = 0;
    for (const Chain& c : cs) maxL = std::max(maxL, c.p->L);
    std::vector<const float*> cur(cs.size(), nullptr); /* nullptr: the packed cA */
    std::vector<InvItem> items;
    for (int k = maxL; k >= 1; --k) {
        items.clear();
        for (size_t j = 0; j < cs.size(); ++j) {
            const TPlan& p = *cs[j].p;
            if (p.L < k) continue;
            float *tL = cs[j].T[0], *tH = cs[j].T[1], *tA = cs[j].T[2];
            const int64_t R = p.g.R[k], C = p.g.C[k];
            const bool fromP = k == p.L;
            const int64_t a_bs = fromP ? 0 : 4 * p.g.R[k + 1] * p.g.C[k + 1];
            const int64_t lda = fromP ? 0 : 2 * p.g.C[k + 1];
            const bool final = k == 1;
            const int64_t oH = final ? p.H : 2 * R, oW = final ? p.W : 2 * C;
            unsigned long long* zc = final ? cs[j].zc : nullptr;
            if (fb_tiled_ok(p.B, 2 * R, 2 * C, tp)) {
                float* y = final ? cs[j].out : ((cur[j] == tA) ? tL : tA);
                items.push_back(InvItem{cur[j], a_bs, lda, fromP, cs[j].P, p.g.PR, p.g.PC, p.g.offR[k], p.g.offC[k],
                                        p.B, R, C, cs[j].thr, y, oH, oW, zc});
                cur[j] = y;
            } else {
                float* t0 = (cur[j] == tL) ? tA : tL;
                float* t1 = (cur[j] == tH) ? tA : tH;
                launch_idwt_rows(cur[j], a_bs, lda, fromP, cs[j].P, p.g.PR, p.g.PC, p.g.offR[k], p.g.offC[k], p.B, R,
                                 C, tp, cs[j].thr, t0, t1, s);
                float* y = final ? cs[j].out : (cur[j] ? const_cast<float*>(cur[j]) : tA);
                launch_idwt_cols(t0, t1, p.B, R, C, tp, y, oH, oW, zc, s);
                cur[j] = y;
            }
        }
        if (!items.empty()) launch_inv_levels(items.data(), (int)items.size(), tp, s);
    }
}

/* ---- the one-launch small path (small.hip) ---- */
constexpr int64_t SM_POP_MAX = 1 << 20; /* population of a whole call taken by k_small */
constexpr int SM_TILES_MAX = SM_SEG_WG_MAX; /* workgroups per tensor */
constexpr int64_t SM_TILE_COST = 64;         /* tiling choice: LDS words a workgroup is worth */

/* Tile sizes (TR x TC at level L) for one tensor: every tile's forward and inverse arena must
 * fit; among those, the least per-workgroup level-0 window plus a charge per workgroup. */
bool small_tiling(const TPlan& p, int F, int budget, int words, SmallSeg& sg) {
    const int L = p.L;
    int32_t Rn[SM_LMAX + 1], Cn[SM_LMAX + 1];
    for (int k = 0; k <= L; ++k) { Rn[k] = (int32_t)p.g.R[k]; Cn[k] = (int32_t)p.g.C[k]; }
    const int RL = Rn[L], CL = Cn[L];
    int64_t best = INT64_MAX;
    std::vector<SmAxis> ar, ac;
    for (int TR = RL;; TR = (TR + 1) / 2) {
        const int tR = (RL + TR - 1) / TR;
        ar.resize(tR);
        for (int i = 0; i < tR; ++i) sm_axis(i, TR, L, Rn, F, &ar[i]);
        for (int TC = CL;; TC = (TC + 1) / 2) {
            const int tC = (CL + TC - 1) / TC;
            const int64_t tiles = p.B * tR * tC;
            if (tiles <= budget && 2 * (L + 1) * (tR + tC) <= words) {
                ac.resize(tC);
                for (int j = 0; j < tC; ++j) sm_axis(j, TC, L, Cn, F, &ac[j]);
                int64_t worst = 0;
                bool fits = true;
                for (int i = 0; i < tR && fits; ++i)
                    for (int j = 0; j < tC && fits; ++j) {
                        const SmNeed nd = sm_need(ar[i], ac[j], L, F);
                        fits = sm_fwd_words(nd) <= SM_ARENA && sm_inv_words(nd) <= SM_ARENA;
                        worst = std::max<int64_t>(worst, (int64_t)ar[i].fw[0].len * ac[j].fw[0].len + nd.fkeys / 2);
                    }
                const int64_t cost = worst + SM_TILE_COST * tiles;
                if (fits && cost < best) {
                    best = cost;
                    sg.TR = TR;
                    sg.TC = TC;
                    sg.tilesR = tR;
                    sg.tilesC = tC;
                }
            }
            if (TC == 1) break;
        }
        if (TR == 1) break;
    }
    return best != INT64_MAX;
}

/* k_small takes the whole call when every tensor is a 2-D transform, the call is small and
 * every tensor finds a tiling inside the co-resident grid */
bool plan_small(const std::vector<TPlan>& ps, const wtp_tensor* ts, int n, void* ws, double pct, const Taps& tp,
                uint32_t* slots, SmallTable& t) {
    if (n > SM_MAX_SEG || (tp.F & 1) || tp.F < 2 || tp.F > SM_F_MAX) return false;
    const int cap = std::min(small_capacity(), RES_MAX_WG);
    int64_t tot = 0;
    for (const TPlan& p : ps) {
        if (!p.dwt || p.flat || p.L > SM_LMAX || p.H > SM_LINE_MAX || p.W > SM_LINE_MAX) return false;
        tot += p.pop;
    }
    if (tot > SM_POP_MAX || cap < n) return false;
    memset(&t, 0, sizeof t);
    int wg = 0, words = 0;
    for (int i = 0; i < n; ++i) {
        const TPlan& p = ps[i];
        SmallSeg& sg = t.s[i];
        /* workgroups by share of the population, at least one per image */
        if (p.B > SM_SEG_WG_MAX) return false;
        const int budget = (int)std::max<int64_t>(p.B, std::min<int64_t>(std::min(SM_TILES_MAX, SM_SEG_WG_MAX),
                                                                         (int64_t)cap * p.pop / tot));
        if (!small_tiling(p, tp.F, budget, (SM_WIN_WORDS - words) / (n - i), sg)) return false;
        /* the windows of every tile row and tile column, packed (small_geom.h computes them) */
        {
            int32_t Rn[SM_LMAX + 1], Cn[SM_LMAX + 1];
            for (int k = 0; k <= p.L; ++k) { Rn[k] = (int32_t)p.g.R[k]; Cn[k] = (int32_t)p.g.C[k]; }
            sg.win_off = words;
            auto pack = [&](const SmAxis& a) {
                for (int k = 0; k <= p.L; ++k) {
                    t.win[words++] = (uint32_t)a.fw[k].s | ((uint32_t)a.fw[k].len << 16);
                    t.win[words++] = (uint32_t)a.sv[k].s | ((uint32_t)a.sv[k].len << 16);
                }
            };
            SmAxis a;
            for (int r = 0; r < sg.tilesR; ++r) { sm_axis(r, sg.TR, p.L, Rn, tp.F, &a); pack(a); }
            for (int c = 0; c < sg.tilesC; ++c) { sm_axis(c, sg.TC, p.L, Cn, tp.F, &a); pack(a); }
        }
        sg.in = ts[i].in;
        sg.out = ts[i].out;
        sg.P = reinterpret_cast<float*>(wsb(ws, p.p_off));
        SegDesc sd;
        memset(&sd, 0, sizeof sd);
        seg_ranks(p.pop, pct, sd);
        sg.r0 = sd.r0;
        sg.gamma = sd.gamma;
        sg.above = sd.above;
        sg.numel = p.numel;
        sg.n = p.pop;
        sg.B = (int32_t)p.B;
        sg.L = p.L;
        sg.PR = (int32_t)p.g.PR;
        sg.PC = (int32_t)p.g.PC;
        int64_t nc = p.g.R[p.L] * p.g.C[p.L];
        for (int k = 0; k <= p.L; ++k) {
            sg.R[k] = (int32_t)p.g.R[k];
            sg.C[k] = (int32_t)p.g.C[k];
            sg.offR[k] = k ? (int32_t)p.g.offR[k] : 0;
            sg.offC[k] = k ? (int32_t)p.g.offC[k] : 0;
            if (k) nc += 3 * p.g.R[k] * p.g.C[k];
        }
        sg.npad = (int32_t)(p.pop - p.B * nc);
        sg.res = i;
        sg.wg_begin = wg;
        sg.nwg = (int32_t)(p.B * sg.tilesR * sg.tilesC);
        t.wg_begin[i] = wg;
        wg += sg.nwg;
    }
    for (int i = n; i < SM_MAX_SEG; ++i) t.wg_begin[i] = INT32_MAX;
    if (wg > cap) return false;
    t.nseg = n;
    t.slots = slots;
    t.nblk = wg;
    t.tp.F = tp.F;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < SM_F_MAX; ++j) t.tp.f[i][j] = j < tp.F ? tp.f[i][j] : 0.0f;
    return true;
}

/* pywt.wavedec / waverec (periodization) of one flattened tensor (1-D mode): packed layout
 * [cA_L | cD_L | cD_L-1 | ... | cD_1] (pywt.coeffs_to_array of a 1-D list) */
int64_t flat_off_d(const TPlan& p, int k) {
    int64_t off = p.len[p.L];
    for (int j = p.L; j > k; --j) off += p.len[j];
    return off;
}

void forward_flat(const TPlan& p, const float* in, float* P, float* T0, float* T1, const Taps& tp, hipStream_t s) {
    const float* cur = in;
    for (int k = 1; k <= p.L; ++k) {
        float* a = (k == p.L) ? P : ((cur == T0) ? T1 : T0);
        launch_dwt1_level(cur, p.len[k - 1], tp, a, P + flat_off_d(p, k), s);
        cur = a;
    }
}

/* each level reads a (the packed cA at the top, thresholded on load; then the previous level's
 * output, of which the first len[k] samples are used -- waverec's crop) and the packed cD_k */
void inverse_flat(const TPlan& p, const float* P, float* out, float* T0, float* T1, const Taps& tp, const float* thr,
                  unsigned long long* zc, hipStream_t s) {
    const float* a = P;
    int a_thr = 1;
    for (int k = p.L; k >= 1; --k) {
        const bool final = k == 1;
        float* y = final ? out : ((a == T0) ? T1 : T0);
        launch_idwt1_level(a, a_thr, P + flat_off_d(p, k), p.len[k], tp, thr, y, final ? p.len[0] : 2 * p.len[k],
                           final ? zc : nullptr, s);
        a = y;
        a_thr = 0;
    }
}

}  // namespace

extern "C" {

int wtp_abi_version(void) { return WTP_ABI_VERSION; }
int wtp_wavelet_count(void) { return WT_NUM_WAVELETS; }
const char* wtp_wavelet_name(int wid) { return (wid >= 0 && wid < WT_NUM_WAVELETS) ? wt_names[wid] : nullptr; }
int wtp_wavelet_id(const char* name) {
    if (!name) return -1;
    for (int i = 0; i < WT_NUM_WAVELETS; ++i)
        if (strcmp(name, wt_names[i]) == 0) return i;
    return -1;
}
int wtp_dec_len(int wid) { return (wid >= 0 && wid < WT_NUM_WAVELETS) ? wt_flen[wid] : -1; }
int wtp_max_level(int64_t data_len, int dec_len) { return max_level(data_len, dec_len); }
int wtp_packed_shape(int64_t H, int64_t W, int level, int64_t* rows, int64_t* cols) {
    if (level < 0 || level > 32 || !rows || !cols) return fail(WTP_EARG, -1, "bad packed-shape request");
    wt_level_geom g;
    wt_geom(H, W, level, &g);
    *rows = g.PR;
    *cols = g.PC;
    return WTP_OK;
}
const char* wtp_last_error(void) { return g_err.c_str(); }
int wtp_set_stage_events(void* const* events, int n) {
    if (n < 0 || n > 8 || (n > 0 && !events)) return fail(WTP_EARG, -1, "bad stage events");
    for (int i = 0; i < 8; ++i) g_stage_ev[i] = (i < n) ? (hipEvent_t)events[i] : nullptr;
    g_stage_n = n;
    return WTP_OK;
}
int wtp_last_error_tensor(void) { return g_err_tensor; }
int wtp_set_resident(int mode) {
    if (mode < 0 || mode > 1) return fail(WTP_EARG, -1, "bad resident mode %d", mode);
    const int prev = g_resident.exchange(mode);
    return prev;
}
int wtp_resident_capacity(void) { return resident_capacity(); }
int wtp_set_interior(int mode) { return fb_set_interior(mode); }

int wtp_set_pipeline(int mode) {
    if (mode < 0 || mode > 1) return fail(WTP_EARG, -1, "bad pipeline mode %d", mode);
    return g_pipeline.exchange(mode);
}
int wtp_set_fused_select(int mode) {
    if (mode < 0 || mode > 1) return fail(WTP_EARG, -1, "bad fused-select mode %d", mode);
    return g_fused.exchange(mode);
}
unsigned wtp_set_resident_timeout_us(unsigned us) { return set_resident_timeout_us(us); }
int wtp_set_kernel_stamps(unsigned long long* stamps_dev) {
    set_kernel_stamps(stamps_dev);
    return WTP_OK;
}

size_t wtp_workspace_size(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level) {
    if (ntensors < 0 || (ntensors > 0 && !tensors)) return 0;
    /* large enough for both wtp_prune_f32 (level carried) and wtp_prune_layers_f32 */
    std::vector<TPlan> ps, pl;
    if (plan_tensors(tensors, ntensors, wavelet_id, level, 50.0, false, ps, true) != WTP_OK) return 0;
    if (plan_tensors(tensors, ntensors, wavelet_id, level, 50.0, false, pl, false) != WTP_OK) return 0;
    const Taps tp = (wavelet_id >= 0 && wavelet_id < WT_NUM_WAVELETS) ? make_taps(wavelet_id) : Taps{};
    return std::max(make_layout(ps, tp).total, make_layout(pl, tp).total);
}

int wtp_workspace_init(void* ws, size_t bytes, wtp_stream_t stream) {
    if (!ws && bytes) return fail(WTP_EARG, -1, "null workspace");
    if (bytes && hipMemsetAsync(ws, 0, bytes, (hipStream_t)stream) != hipSuccess)
        return fail(WTP_EHIP, -1, "hipMemsetAsync failed");
    return WTP_OK;
}

/* The selection pipeline's side stream (one per device and caller stream, non-blocking, created
 * on first use and kept) and its events: a call with several launch groups of DWT segments runs
 * group g's forward levels on the caller's stream and its selection (window / collect /
 * mask-select: HBM-bound) on the side stream, so it overlaps the next group's forward levels or
 * the previous group's inverse levels (VALU-bound); the caller's stream waits for every group's
 * selection before that group's inverse, which joins the side stream back (graph capture
 * included).  Selections stay serialised on the side stream (the SelHeader parity regions). */
struct SidePipe {
    hipStream_t side = nullptr;
    std::vector<hipEvent_t> ev;
};
std::mutex g_pipe_mu;
std::map<std::pair<int, hipStream_t>, SidePipe> g_pipes;
SidePipe* side_pipe(hipStream_t s, int nev) {
    /* the side stream must live on the caller's stream's device: when that is not the current
     * device (the caller set no device guard) the call keeps the single-stream form */
    int dev = 0, sdev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    if (hipStreamGetDevice(s, &sdev) != hipSuccess || sdev != dev) return nullptr;
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    SidePipe& sp = g_pipes[{dev, s}];
    if (!sp.side && hipStreamCreateWithFlags(&sp.side, hipStreamNonBlocking) != hipSuccess) {
        sp.side = nullptr;
        return nullptr;
    }
    while ((int)sp.ev.size() < nev) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        sp.ev.push_back(e);
    }
    return &sp;
}

static int prune_impl(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, double pct, void* ws,
                      size_t ws_bytes, wtp_result* results, wtp_stream_t stream, bool carry, bool flat = false,
                      bool no_resident = false) {
    g_err.clear();
    g_err_tensor = -1;
    if (ntensors < 0 || (ntensors > 0 && (!tensors || !results))) return fail(WTP_EARG, -1, "bad arguments");
    if (ntensors == 0) return WTP_OK;
    std::vector<TPlan> ps;
    int rc = plan_tensors(tensors, ntensors, wavelet_id, level, pct, true, ps, carry, flat);
    if (rc != WTP_OK) return rc;
    const Taps tp = (wavelet_id >= 0 && wavelet_id < WT_NUM_WAVELETS) ? make_taps(wavelet_id) : Taps{};
    Layout lay = make_layout(ps, tp);
    if (!ws || ws_bytes < lay.total)
        return fail(WTP_EWORKSPACE, -1, "workspace too small: need %zu bytes, got %zu", lay.total, ws_bytes);
    hipStream_t s = (hipStream_t)stream;
    SelHeader* head = reinterpret_cast<SelHeader*>(wsb(ws, lay.sel));
    uint32_t* cand = reinterpret_cast<uint32_t*>(wsb(ws, lay.cand));
    float* thr_t = reinterpret_cast<float*>(wsb(ws, lay.thr));

    stage(0, s);
    if (!no_resident && !flat && g_resident.load(std::memory_order_relaxed)) {
        /* a small call: the whole path in one launch (small.hip) */
        SmallTable st;
        if (plan_small(ps, tensors, ntensors, ws, pct, tp, cand, st)) {
            for (int i = 1; i <= 4; ++i) stage(i, s);
            launch_small(st, head, results, s);
            stage(5, s);
            return check_launch();
        }
    }
    /* 1. forward transforms into the packed arrays (pywt.wavedec2 + coeffs_to_array) */
    const int ngroups = (ntensors + SEG_PER_LAUNCH - 1) / SEG_PER_LAUNCH;
    std::vector<std::vector<Chain>> gchains(ngroups);
    for (int t = 0; t < ntensors; ++t) {
        const TPlan& p = ps[t];
        if (!p.dwt) continue;
        if (p.flat) {
            float* T = reinterpret_cast<float*>(wsb(ws, p.t_off));
            forward_flat(p, tensors[t].in, reinterpret_cast<float*>(wsb(ws, p.p_off)), T,
                         T + align_up(p.t_elems * sizeof(float)) / sizeof(float), tp, s);
            continue;
        }
        Chain c;
        c.p = &p;
        c.in = tensors[t].in;
        c.out = tensors[t].out;
        c.P = reinterpret_cast<float*>(wsb(ws, p.p_off));
        for (int i = 0; i < 3; ++i)
            c.T[i] = reinterpret_cast<float*>(wsb(ws, p.t_off + i * align_up(p.t_elems * sizeof(float))));
        c.thr = thr_t + t;
        c.zc = reinterpret_cast<unsigned long long*>(&results[t].zero_count);
        if (p.f_slots) c.fsl = reinterpret_cast<uint32_t*>(wsb(ws, p.f_off));
        gchains[t / SEG_PER_LAUNCH].push_back(c);
        if (!p.tight && hipMemsetAsync(c.P, 0, (size_t)p.pop * sizeof(float), s) != hipSuccess)
            return fail(WTP_EHIP, t, "hipMemsetAsync failed");
    }
    int dwt_groups = 0;
    for (const auto& gc : gchains) dwt_groups += !gc.empty();
    /* fused selection per launch group: every tensor of the group qualifies with its real input
     * pointer and the current interior mode (fused_slot_count) */
    std::vector<char> fused(ngroups, 0);
    bool any_fused = false;
    if (g_fused.load(std::memory_order_relaxed)) {
        for (int gi = 0; gi < ngroups; ++gi) {
            const int g0 = gi * SEG_PER_LAUNCH, g1 = std::min(ntensors, g0 + SEG_PER_LAUNCH);
            bool ok = true;
            for (int t = g0; t < g1 && ok; ++t)
                ok = ps[t].f_slots > 0 && fused_slot_count(ps[t], tensors[t].in, tp, false) == ps[t].f_slots;
            fused[gi] = ok;
            any_fused = any_fused || ok;
        }
    }
    const int pmode = dwt_groups > 1 ? g_pipeline.load(std::memory_order_relaxed) : 0;
    /* events 2g (group g's forward done) and 2g + 1 (its selection done); the last one joins the
     * side stream back on an error path.  (Round 5's mode 2 -- each group's levels on a lane
     * stream of its own -- measured slower and was removed in round 6; its capture-crash
     * bisection is kept in tools/lanes_capture_diag.py and DESIGN.md.) */
    /* ... and 2 ngroups + g (fused group g's window pass done), 3 ngroups (the call's start, on
     * the caller's stream) */
    const int nev = 3 * ngroups + 2;
    SidePipe* pipe = pmode ? side_pipe(s, nev) : nullptr;
    const hipStream_t ss = pipe ? pipe->side : s; /* the selection's stream */
    /* an error after the first fork still joins the side stream back into the caller's (an
     * unjoined fork invalidates a capture, and eagerly the caller may free what it still reads) */
    bool forked = false;
    auto fail_joined = [&](int t, const char* msg) {
        if (forked) {
            hipEvent_t e = pipe->ev[nev - 1];
            (void)hipEventRecord(e, ss);
            (void)hipStreamWaitEvent(s, e, 0);
        }
        return fail(WTP_EHIP, t, "%s", msg);
    };
    /* the fused groups' window passes (k_fwin); their histograms start at zero */
    if (any_fused && hipMemsetAsync(wsb(ws, lay.fwh), 0, FWIN_HIST_BYTES, s) != hipSuccess)
        return fail(WTP_EHIP, -1, "hipMemsetAsync failed");
    std::vector<FwinTable> fts(ngroups);
    for (int gi = 0; gi < ngroups; ++gi) {
        if (!fused[gi]) continue;
        FwinTable& ft = fts[gi];
        memset(&ft, 0, sizeof ft);
        const int g0 = gi * SEG_PER_LAUNCH, g1 = std::min(ntensors, g0 + SEG_PER_LAUNCH);
        ft.nseg = g1 - g0;
        ft.F = tp.F;
        ft.gh = reinterpret_cast<uint32_t*>(wsb(ws, lay.fwh));
        for (int j = 0; j < tp.F && j < FWIN_F_MAX; ++j) { ft.lo[j] = tp.f[0][j]; ft.hi[j] = tp.f[1][j]; }
        for (int t = g0; t < g1; ++t) {
            const TPlan& p = ps[t];
            FwinSeg& f = ft.s[t - g0];
            SegDesc sd;
            memset(&sd, 0, sizeof sd);
            seg_ranks(p.pop, pct, sd);
            bucket_plan(p.pop, &sd.nsub_log2, &sd.bucket_cap, true);
            f.in = tensors[t].in;
            f.hdr = reinterpret_cast<FslHeader*>(wsb(ws, p.f_off));
            f.n = p.pop;
            f.r0 = sd.r0;
            f.above = sd.above;
            f.nsub_log2 = sd.nsub_log2;
            f.B = (int32_t)p.B;
            f.R = (int32_t)p.g.R[0];
            f.C = (int32_t)p.g.C[0];
            f.L = p.L;
        }
    }
    if (!pipe) /* group by group: the groups share the level temps (make_layout); a fused group's
                * forward runs behind its window pass, in the selection loop below */
        for (int gi = 0; gi < ngroups; ++gi)
            if (!fused[gi]) forward_chains(gchains[gi], tp, s);
    /* pipelined: the first two fused groups' window passes on the side stream ahead of their
     * forwards (it reads the inputs: it waits for the caller's stream first); group g + 2's
     * follows group g's selection there, which has read the slot areas g + 2 reuses */
    auto fwin_side = [&](int gi) {
        if (gi >= ngroups || !fused[gi]) return true;
        launch_fwin(fts[gi], head, ss);
        return hipEventRecord(pipe->ev[2 * ngroups + gi], ss) == hipSuccess;
    };
    if (pipe && any_fused) {
        if (hipEventRecord(pipe->ev[3 * ngroups], s) != hipSuccess || hipStreamWaitEvent(ss, pipe->ev[3 * ngroups], 0) != hipSuccess)
            return fail_joined(-1, "hipEventRecord / hipStreamWaitEvent failed");
        forked = true;
        if (!fwin_side(0) || !fwin_side(1)) return fail_joined(-1, "hipEventRecord failed");
    }
    /* 2. exact percentile selection + level-0 mask, SEG_PER_LAUNCH segments per launch group:
     * one resident launch when every segment of the group is level-0 and the group's chunks fit
     * the co-resident grid, else window / collect / mask-select */
    for (int g0 = 0; g0 < ntensors; g0 += SEG_PER_LAUNCH) {
        const int g1 = std::min(ntensors, g0 + SEG_PER_LAUNCH);
        const int gi = g0 / SEG_PER_LAUNCH;
        bool all0 = true;
        int64_t rblk = 0;
        for (int t = g0; t < g1; ++t) {
            all0 = all0 && !ps[t].dwt;
            rblk += (ps[t].pop + RES_CHUNK - 1) / RES_CHUNK;
        }
        const bool fz = fused[gi] != 0;
        const bool resident = !fz && all0 && !no_resident && g_resident.load(std::memory_order_relaxed) &&
                              rblk <= RES_MAX_WG && rblk <= resident_capacity();
        const int64_t chunk = resident ? RES_CHUNK : CHUNK;
        SegTable tab;
        memset(&tab, 0, sizeof tab);
        /* the resident launch's late group: the smallest segments, together at most RES_LATE_PCT %
         * of the workgroups (at least one segment stays early) */
        bool late[SEG_PER_LAUNCH] = {};
        if (resident) {
            int by[SEG_PER_LAUNCH];
            for (int i = 0; i < g1 - g0; ++i) by[i] = g0 + i;
            std::stable_sort(by, by + (g1 - g0), [&](int a, int b) { return ps[a].pop < ps[b].pop; });
            int64_t lb = 0;
            for (int i = 0; i + 1 < g1 - g0; ++i) {
                const int64_t w = (ps[by[i]].pop + RES_CHUNK - 1) / RES_CHUNK;
                if (100 * (lb + w) > (int64_t)RES_LATE_PCT * rblk) break;
                lb += w;
                late[by[i] - g0] = true;
            }
        }
        int blk = 0;
        for (int t = g0; t < g1; ++t) {
            const TPlan& p = ps[t];
            SegDesc& sd = tab.s[tab.nseg++];
            sd.data = p.dwt ? reinterpret_cast<const float*>(wsb(ws, p.p_off)) : tensors[t].in;
            sd.out = p.dwt ? nullptr : tensors[t].out;
            sd.n = p.pop;
            seg_ranks(p.pop, pct, sd);
            sd.numel = p.numel;
            sd.blk_begin = blk;
            tab.blk_begin[tab.nseg - 1] = blk;
            sd.slot = t - g0;
            sd.res = t;
            sd.eff_level = p.L;
            sd.flags = p.dwt ? 0 : SEG_MASK;
            const uintptr_t a = reinterpret_cast<uintptr_t>(sd.data), o = reinterpret_cast<uintptr_t>(sd.out);
            if ((a % 16) == 0 && (o % 16) == 0) sd.flags |= SEG_ALIGNED;
            sd.cand_off = (int64_t)p.cand_off;
            sd.cap = p.cap;
            bucket_plan(p.pop, &sd.nsub_log2, &sd.bucket_cap, p.dwt);
            if (resident) {
                sd.nsub_log2 = RES_NSUB_LOG2;
                if (p.pop > RES_MS) /* rounded up: floor(g * step_fx / 2^32) is then the exact floor of
                                       * g (n - 16) / 255 for every group g <= 255 (the error stays
                                       * below 255 / 2^32, under the 1/255 gap to the next integer) */
                    sd.res_step_fx = (((uint64_t)(p.pop - SAMPLE_GROUP) << 32) + (uint64_t)(RES_MS / SAMPLE_GROUP - 2)) /
                                     (uint64_t)(RES_MS / SAMPLE_GROUP - 1);
            }
            if (late[t - g0]) sd.flags |= SEG_LATE;
            if (fz) { /* k_fslot_collect: one block per FSC_SLOTS wave slots (seg_fsl / seg_fsl_n) */
                sd.out = reinterpret_cast<float*>(wsb(ws, p.f_off));
                sd.res_step_fx = (uint64_t)p.f_slots;
                sd.flags |= SEG_FUSED;
                blk += (int)((p.f_slots + FSC_SLOTS - 1) / FSC_SLOTS);
            } else {
                blk += (int)((p.pop + chunk - 1) / chunk);
            }
        }
        tab.nblk = blk;
        for (int i = tab.nseg; i < SEG_PER_LAUNCH; ++i) tab.blk_begin[i] = INT32_MAX;
        const bool first = g0 == 0;
        if (pipe) { /* this group's forward levels on the caller's stream, its selection behind them */
            if (fz && hipStreamWaitEvent(s, pipe->ev[2 * ngroups + gi], 0) != hipSuccess) /* its window */
                return fail_joined(-1, "hipStreamWaitEvent failed");
            forward_chains(gchains[gi], tp, s, fz);
            if (hipEventRecord(pipe->ev[2 * gi], s) != hipSuccess) return fail_joined(-1, "hipEventRecord failed");
            if (hipStreamWaitEvent(ss, pipe->ev[2 * gi], 0) != hipSuccess)
                return fail_joined(-1, "hipStreamWaitEvent failed");
            forked = true;
        } else if (fz) {
            launch_fwin(fts[gi], head, s);
            forward_chains(gchains[gi], tp, s, true);
        }
        if (fz) {
            if (first) { stage(1, ss); stage(2, ss); }
            launch_fslot_collect(tab, head, cand, results, ss);
            /* group g + 2's window pass next on the side stream: it needs only the slot areas this
             * bucket pass has read, not this group's select and retry */
            if (pipe && !fwin_side(gi + 2)) return fail_joined(-1, "hipEventRecord failed");
            if (first) stage(3, ss);
            launch_mask_select(tab, head, cand, results, thr_t, ss);
            /* a segment whose patch window missed the ranks: the unfused window / collect / select
             * over P, for it alone (the same table in k_collect's chunk units) */
            SegTable rt = tab;
            rt.retry = 1;
            int rb = 0;
            for (int i = 0; i < rt.nseg; ++i) {
                SegDesc& sd = rt.s[i];
                sd.flags &= ~SEG_FUSED;
                sd.out = nullptr;
                sd.res_step_fx = 0;
                sd.blk_begin = rt.blk_begin[i] = rb;
                rb += (int)((sd.n + CHUNK - 1) / CHUNK);
            }
            rt.nblk = rb;
            launch_fused_retry(rt, head, cand, results, thr_t, ss);
        } else if (resident) {
            if (first) stage(1, ss);
            if (first) { stage(2, ss); stage(3, ss); }
            launch_resident(tab, head, cand, results, thr_t, ss);
        } else {
            if (first) stage(1, ss);
            launch_window(tab, head, ss);
            if (first) stage(2, ss);
            launch_collect(tab, head, cand, results, ss);
            if (first) stage(3, ss);
            launch_mask_select(tab, head, cand, results, thr_t, ss);
            bool inplace = false;
            for (int i = 0; i < tab.nseg; ++i) inplace = inplace || (tab.s[i].out && tab.s[i].out == tab.s[i].data);
            if (inplace) launch_mask_inplace(tab, results, thr_t, ss);
        }
        if (first) stage(4, ss);
        if (pipe && hipEventRecord(pipe->ev[2 * gi + 1], ss) != hipSuccess) {
            return fail_joined(-1, "hipEventRecord failed");
        }
        if (pipe && !fz && !fwin_side(gi + 2)) return fail_joined(-1, "hipEventRecord failed");
    }
    /* 3. inverse transforms with the threshold applied on load (array_to_coeffs + waverec2); in
     * the pipelined form group by group, each behind its selection (which joins the side stream) */
    if (pipe) {
        for (int gi = 0; gi < ngroups; ++gi) {
            if (hipStreamWaitEvent(s, pipe->ev[2 * gi + 1], 0) != hipSuccess) return fail_joined(-1, "hipStreamWaitEvent failed");
            inverse_chains(gchains[gi], tp, s);
        }
    } else {
        for (const auto& gc : gchains) inverse_chains(gc, tp, s);
    }
    for (int t = 0; t < ntensors; ++t) {
        const TPlan& p = ps[t];
        if (!p.flat || !p.dwt) continue;
        float* T = reinterpret_cast<float*>(wsb(ws, p.t_off));
        inverse_flat(p, reinterpret_cast<const float*>(wsb(ws, p.p_off)), tensors[t].out, T,
                     T + align_up(p.t_elems * sizeof(float)) / sizeof(float), tp, thr_t + t,
                     reinterpret_cast<unsigned long long*>(&results[t].zero_count), s);
    }
    stage(5, s);
    return check_launch();
}

int wtp_prune_f32(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, double pct, void* ws,
                  size_t ws_bytes, wtp_result* results, wtp_stream_t stream) {
    return prune_impl(tensors, ntensors, wavelet_id, level, pct, ws, ws_bytes, results, stream, true);
}

int wtp_prune_layers_f32(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, double pct, void* ws,
                         size_t ws_bytes, wtp_result* results, wtp_stream_t stream) {
    return prune_impl(tensors, ntensors, wavelet_id, level, pct, ws, ws_bytes, results, stream, false);
}

size_t wtp_workspace_size_ex(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, int flags) {
    if (ntensors < 0 || (ntensors > 0 && !tensors) || (flags & ~(WTP_CARRY_LEVEL | WTP_FLATTEN | WTP_NO_RESIDENT))) return 0;
    std::vector<TPlan> ps;
    if (plan_tensors(tensors, ntensors, wavelet_id, level, 50.0, false, ps, (flags & WTP_CARRY_LEVEL) != 0,
                     (flags & WTP_FLATTEN) != 0) != WTP_OK)
        return 0;
    const Taps tp = (wavelet_id >= 0 && wavelet_id < WT_NUM_WAVELETS) ? make_taps(wavelet_id) : Taps{};
    return make_layout(ps, tp).total;
}

int wtp_prune_ex_f32(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, double pct, int flags,
                     void* ws, size_t ws_bytes, wtp_result* results, wtp_stream_t stream) {
    if (flags & ~(WTP_CARRY_LEVEL | WTP_FLATTEN | WTP_NO_RESIDENT)) return fail(WTP_EARG, -1, "bad flags 0x%x", flags);
    return prune_impl(tensors, ntensors, wavelet_id, level, pct, ws, ws_bytes, results, stream,
                      (flags & WTP_CARRY_LEVEL) != 0, (flags & WTP_FLATTEN) != 0, (flags & WTP_NO_RESIDENT) != 0);
}

/* ---------------------------------------------------------- min pruning --- */
/* percentage_min_pruning (ResNet/min_weight_pruning.py:66-74): k = int(numel * fraction)
 * (Python int(): truncation toward zero); torch.topk rejects k outside [0, numel]. */
struct MinPlan {
    std::vector<TPlan> ps;
    std::vector<int64_t> k;
    Layout lay;
    size_t mp_off = 0, tie_off = 0, total = 0;
    int nblk = 0;
};

static int plan_min(const wtp_tensor* ts, int n, double fraction, bool check_ptrs, MinPlan& m) {
    m.ps.assign(n, TPlan());
    m.k.assign(n, 0);
    if (!(fraction == fraction)) return fail(WTP_EARG, -1, "cannot convert float NaN to integer");
    for (int t = 0; t < n; ++t) {
        const wtp_tensor& x = ts[t];
        TPlan& p = m.ps[t];
        if (x.ndim < 0 || x.ndim > WTP_MAX_DIMS) return fail(WTP_EARG, t, "tensor %d: ndim %d unsupported", t, x.ndim);
        p.ndim = x.ndim;
        p.numel = 1;
        for (int d = 0; d < x.ndim; ++d) {
            if (x.shape[d] < 0) return fail(WTP_EARG, t, "tensor %d: negative dimension", t);
            p.numel *= x.shape[d];
        }
        if (check_ptrs && p.numel > 0 && (!x.in || !x.out)) return fail(WTP_EARG, t, "tensor %d: null pointer", t);
        if (p.numel > (int64_t)INT32_MAX) return fail(WTP_EARG, t, "tensor %d: more than 2^31-1 elements", t);
        const double kd = (double)p.numel * fraction; /* min_weight_pruning.py:70 */
        if (!(kd > -1.0 && kd < (double)p.numel + 1.0))
            return fail(WTP_EARG, t, "selected index k out of range");
        m.k[t] = (int64_t)kd; /* C cast truncates toward zero, like int() */
        p.pop = p.numel;
        p.cap = p.numel ? cap_for(p.pop, false) : 0;
        m.nblk += (int)((p.pop + CHUNK - 1) / CHUNK);
    }
    m.lay = make_layout(m.ps, Taps{}); /* level-0 populations only: no temps */
    m.mp_off = align_up(m.lay.total);
    m.tie_off = align_up(m.mp_off + (size_t)n * 16);
    m.total = align_up(m.tie_off + (size_t)(m.nblk + 1) * sizeof(uint32_t));
    return WTP_OK;
}

size_t wtp_min_prune_workspace_size(const wtp_tensor* tensors, int ntensors, double fraction) {
    if (ntensors < 0 || (ntensors > 0 && !tensors)) return 0;
    MinPlan m;
    if (plan_min(tensors, ntensors, fraction, false, m) != WTP_OK) return 0;
    return m.total;
}

int wtp_min_prune_f32(const wtp_tensor* tensors, int ntensors, double fraction, void* ws, size_t ws_bytes,
                      wtp_result* results, wtp_stream_t stream) {
    g_err.clear();
    g_err_tensor = -1;
    if (ntensors < 0 || (ntensors > 0 && (!tensors || !results))) return fail(WTP_EARG, -1, "bad arguments");
    if (ntensors == 0) return WTP_OK;
    MinPlan m;
    int rc = plan_min(tensors, ntensors, fraction, true, m);
    if (rc != WTP_OK) return rc;
    if (!ws || ws_bytes < m.total)
        return fail(WTP_EWORKSPACE, -1, "workspace too small: need %zu bytes, got %zu", m.total, ws_bytes);
    hipStream_t s = (hipStream_t)stream;
    SelHeader* head = reinterpret_cast<SelHeader*>(wsb(ws, m.lay.sel));
    uint32_t* cand = reinterpret_cast<uint32_t*>(wsb(ws, m.lay.cand));
    float* thr_t = reinterpret_cast<float*>(wsb(ws, m.lay.thr));
    void* mp = wsb(ws, m.mp_off);
    uint32_t* tiecnt = reinterpret_cast<uint32_t*>(wsb(ws, m.tie_off));
    /* empty tensors: nothing to select; their records are zero */
    for (int t = 0; t < ntensors; ++t)
        if (m.ps[t].numel == 0 && hipMemsetAsync(results + t, 0, sizeof(wtp_result), s) != hipSuccess)
            return fail(WTP_EHIP, t, "hipMemsetAsync failed");
    std::vector<int> live;
    for (int t = 0; t < ntensors; ++t)
        if (m.ps[t].numel > 0) live.push_back(t);
    for (size_t g0 = 0; g0 < live.size(); g0 += SEG_PER_LAUNCH) {
        SegTable tab;
        memset(&tab, 0, sizeof tab);
        int blk = 0;
        for (size_t j = g0; j < live.size() && j < g0 + SEG_PER_LAUNCH; ++j) {
            const int t = live[j];
            const TPlan& p = m.ps[t];
            SegDesc& sd = tab.s[tab.nseg++];
            sd.data = tensors[t].in;
            sd.out = tensors[t].out;
            sd.n = p.pop;
            sd.above = 1; /* one rank: r1 = r0 */
            sd.gamma = 0.0;
            sd.r0 = m.k[t] > 0 ? m.k[t] - 1 : 0;
            sd.numel = p.numel;
            sd.blk_begin = blk;
            tab.blk_begin[tab.nseg - 1] = blk;
            sd.slot = (int)(j - g0);
            sd.res = t;
            sd.eff_level = 0;
            sd.flags = SEG_MINPRUNE | (m.k[t] == 0 ? SEG_KZERO : 0);
            const uintptr_t a = reinterpret_cast<uintptr_t>(sd.data), o = reinterpret_cast<uintptr_t>(sd.out);
            if ((a % 16) == 0 && (o % 16) == 0) sd.flags |= SEG_ALIGNED;
            sd.cand_off = (int64_t)p.cand_off;
            sd.cap = p.cap;
            bucket_plan(p.pop, &sd.nsub_log2, &sd.bucket_cap, false);
            blk += (int)((p.pop + CHUNK - 1) / CHUNK);
        }
        tab.nblk = blk;
        for (int i = tab.nseg; i < SEG_PER_LAUNCH; ++i) tab.blk_begin[i] = INT32_MAX;
        launch_window(tab, head, s);
        launch_collect(tab, head, cand, results, s);
        launch_minprune(tab, head, cand, results, thr_t, mp, tiecnt, s);
    }
    return check_launch();
}

/* ---------------------------------------------------------- random pruning --- */
int wtp_random_prune_f32(const wtp_tensor* tensors, int ntensors, const int64_t* prune_counts, uint64_t seed,
                         wtp_result* results, wtp_stream_t stream) {
    g_err.clear();
    g_err_tensor = -1;
    if (ntensors < 0 || (ntensors > 0 && (!tensors || !results || !prune_counts))) return fail(WTP_EARG, -1, "bad arguments");
    if (ntensors == 0) return WTP_OK;
    std::vector<int64_t> numel(ntensors), keff(ntensors);
    for (int t = 0; t < ntensors; ++t) {
        const wtp_tensor& x = tensors[t];
        if (x.ndim < 0 || x.ndim > WTP_MAX_DIMS) return fail(WTP_EARG, t, "tensor %d: ndim %d unsupported", t, x.ndim);
        int64_t n = 1;
        for (int d = 0; d < x.ndim; ++d) {
            if (x.shape[d] < 0) return fail(WTP_EARG, t, "tensor %d: negative dimension", t);
            n *= x.shape[d];
        }
        if (n > 0 && (!x.in || !x.out)) return fail(WTP_EARG, t, "tensor %d: null pointer", t);
        const int64_t k = prune_counts[t];
        numel[t] = n;
        keff[t] = k >= 0 ? std::min(k, n) : std::max<int64_t>(0, n + k); /* randperm(n)[:k], Python slicing */
    }
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(results, 0, sizeof(wtp_result) * (size_t)ntensors, s) != hipSuccess)
        return fail(WTP_EHIP, -1, "hipMemsetAsync failed");
    for (int g0 = 0; g0 < ntensors; g0 += SEG_PER_LAUNCH) {
        RandTable tab;
        memset(&tab, 0, sizeof tab);
        int cb = 0, zb = 0;
        for (int t = g0; t < ntensors && t < g0 + SEG_PER_LAUNCH; ++t) {
            RandSeg& sg = tab.s[tab.nseg];
            sg.in = tensors[t].in;
            sg.out = tensors[t].out;
            sg.numel = numel[t];
            sg.k = keff[t];
            sg.key = wt_perm_key(seed, (uint32_t)t);
            sg.h = wt_perm_half_bits((uint64_t)numel[t]);
            sg.res = t;
            tab.copy_begin[tab.nseg] = cb;
            tab.zero_begin[tab.nseg] = zb;
            cb += (int)((numel[t] + CHUNK - 1) / CHUNK);
            zb += (int)((keff[t] + STREAM_THREADS - 1) / STREAM_THREADS);
            ++tab.nseg;
        }
        tab.copy_begin[tab.nseg] = cb;
        tab.zero_begin[tab.nseg] = zb;
        for (int i = tab.nseg + 1; i <= SEG_PER_LAUNCH; ++i) { tab.copy_begin[i] = cb; tab.zero_begin[i] = zb; }
        launch_random_prune(tab, results, s);
    }
    return check_launch();
}

int wtp_count_small_f32(const float* x, int64_t n, float thr, unsigned long long* count_dev, wtp_stream_t stream) {
    if (n < 0 || (n > 0 && !x) || !count_dev) return fail(WTP_EARG, -1, "bad arguments");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(count_dev, 0, sizeof(unsigned long long), s) != hipSuccess)
        return fail(WTP_EHIP, -1, "hipMemsetAsync failed");
    if (n > 0) launch_count_small(x, n, thr, count_dev, s);
    return check_launch();
}

int wtp_threshold_f32(const float* in, float* out, int64_t n, double pct, void* ws, size_t ws_bytes,
                      wtp_result* result, wtp_stream_t stream) {
    wtp_tensor t;
    memset(&t, 0, sizeof t);
    t.in = in;
    t.out = out;
    t.ndim = 1;
    t.shape[0] = n;
    return wtp_prune_f32(&t, 1, -1, 0, pct, ws, ws_bytes, result, stream);
}

size_t wtp_dwt_workspace_size(int64_t B, int64_t H, int64_t W, int level) {
    if (level <= 0) return 0;
    wt_level_geom g;
    wt_geom(H, W, level, &g);
    const size_t a = (size_t)(B * g.R[1] * (W > 2 * g.C[1] ? W : 2 * g.C[1]));
    const size_t b = (size_t)(B * 2 * g.R[1] * 2 * g.C[1]);
    return 3 * align_up(std::max(a, b) * sizeof(float));
}

static int component_plan(int64_t B, int64_t H, int64_t W, int wid, int level, TPlan& p) {
    if (wid < 0 || wid >= WT_NUM_WAVELETS) return fail(WTP_EBADWAVELET, -1, "Unknown wavelet name");
    if (level < 0) return fail(WTP_EBADLEVEL, -1, "Level value of %d is too low . Minimum level is 0.", level);
    if (level > 32 || B < 0 || H <= 0 || W <= 0) return fail(WTP_EARG, -1, "bad component arguments");
    p.B = B;
    p.H = H;
    p.W = W;
    p.L = level;
    p.dwt = level > 0;
    wt_geom(H, W, level, &p.g);
    p.pop = B * p.g.PR * p.g.PC;
    int64_t nc = p.g.R[level] * p.g.C[level];
    for (int k = 1; k <= level; ++k) nc += 3 * p.g.R[k] * p.g.C[k];
    p.tight = nc == p.g.PR * p.g.PC;
    return WTP_OK;
}

int wtp_wavedec2_f32(const float* in, float* packed, int64_t B, int64_t H, int64_t W, int wid, int level, void* ws,
                     size_t ws_bytes, wtp_stream_t stream) {
    TPlan p;
    int rc = component_plan(B, H, W, wid, level, p);
    if (rc != WTP_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (level == 0) {
        if (hipMemcpyAsync(packed, in, (size_t)(B * H * W) * sizeof(float), hipMemcpyDeviceToDevice, s) != hipSuccess)
            return fail(WTP_EHIP, -1, "hipMemcpyAsync failed");
        return WTP_OK;
    }
    const size_t need = wtp_dwt_workspace_size(B, H, W, level);
    if (!ws || ws_bytes < need) return fail(WTP_EWORKSPACE, -1, "workspace too small: need %zu", need);
    const size_t one = need / 3;
    float* tL = reinterpret_cast<float*>(wsb(ws, 0));
    float* tH = reinterpret_cast<float*>(wsb(ws, one));
    float* tA = reinterpret_cast<float*>(wsb(ws, 2 * one));
    if (!p.tight && hipMemsetAsync(packed, 0, (size_t)p.pop * sizeof(float), s) != hipSuccess)
        return fail(WTP_EHIP, -1, "hipMemsetAsync failed");
    forward_chains({Chain{&p, in, nullptr, packed, {tL, tH, tA}, nullptr, nullptr}}, make_taps(wid), s);
    return check_launch();
}

int wtp_waverec2_f32(const float* packed, float* out, int64_t B, int64_t H, int64_t W, int wid, int level,
                     const float* thr32, void* ws, size_t ws_bytes, wtp_stream_t stream) {
    TPlan p;
    int rc = component_plan(B, H, W, wid, level, p);
    if (rc != WTP_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (level == 0) {
        launch_copy_threshold(packed, out, B * H * W, thr32, nullptr, s);
        return check_launch();
    }
    const size_t need = wtp_dwt_workspace_size(B, H, W, level);
    if (!ws || ws_bytes < need) return fail(WTP_EWORKSPACE, -1, "workspace too small: need %zu", need);
    const size_t one = need / 3;
    float* tL = reinterpret_cast<float*>(wsb(ws, 0));
    float* tH = reinterpret_cast<float*>(wsb(ws, one));
    float* tA = reinterpret_cast<float*>(wsb(ws, 2 * one));
    inverse_chains({Chain{&p, nullptr, out, const_cast<float*>(packed), {tL, tH, tA}, thr32, nullptr}}, make_taps(wid), s);
    return check_launch();
}

int wtp_synth_f32(float* out, int64_t n, uint64_t seed, uint32_t tensor_id, int e, wtp_stream_t stream) {
    if (n < 0 || (n > 0 && !out)) return fail(WTP_EARG, -1, "bad synth arguments");
    if (n == 0) return WTP_OK;
    launch_synth(out, n, seed, tensor_id, e, (hipStream_t)stream);
    return check_launch();
}

}  // extern "C"
