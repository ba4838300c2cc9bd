/*
 * wtprune.h -- C ABI of libwtprune.so, the MI355X (gfx950) implementation of the
 * DWT -> percentile-threshold -> IDWT weight-pruning path of iAmGiG/WaveletTransforms
 * (ResNet/dwt_pruning.py).  Plain pointers and sizes only; every device pointer is a HIP
 * device allocation owned by the caller; every entry point is stream-ordered on the given
 * hipStream_t (pass 0 for the null stream), never allocates, never synchronises, and is
 * safe to capture into a hipGraph.  Status: 0 = ok, < 0 = error (wtp_last_error() has the
 * message, phrased like the Python exception the reference would raise).
 *
 * Which reference interface each entry point replaces (file:line in /root/reference):
 *   wtp_wavelet_id / wtp_dec_len    pywt.Wavelet(name).dec_len        dwt_pruning.py:13
 *   wtp_max_level                   calculate_max_level               dwt_pruning.py:12-13
 *   wtp_prune_f32                   multi_resolution_analysis         dwt_pruning.py:35-95
 *                                   (per tensor of prune_layer_weights :98-127, which
 *                                    wavelet_pruning :130-174 calls per Conv2d)
 *   wtp_threshold_f32               percentile_based_thresholding     dwt_pruning.py:25-32
 *   wtp_wavedec2_f32                pywt.wavedec2 + coeffs_to_array   dwt_pruning.py:67-70
 *   wtp_waverec2_f32                array_to_coeffs + waverec2 + crop dwt_pruning.py:75-82
 *   wtp_synth_f32                   (test/bench input generator, no reference counterpart)
 */
#ifndef WTPRUNE_H
#define WTPRUNE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* wtp_stream_t; /* == hipStream_t */

#define WTP_MAX_DIMS 8
#define WTP_ABI_VERSION 1

/* error codes (mirroring the exception the reference path raises) */
#define WTP_OK 0
#define WTP_EBADWAVELET (-1) /* ValueError: Unknown wavelet name '...'                        */
#define WTP_EBADLEVEL (-2)   /* ValueError: Level value of L is too low . Minimum level is 0.  */
#define WTP_EBADPCT (-3)     /* ValueError: Percentiles must be in the range [0, 100]          */
#define WTP_EEMPTY (-4)      /* IndexError: percentile of an empty array                       */
#define WTP_ECROP (-5)       /* IndexError/RuntimeError: the 4-index crop at :79-82 fails      */
#define WTP_EARG (-6)        /* invalid argument (null pointer, too many dims, ...)           */
#define WTP_EWORKSPACE (-7)  /* workspace too small                                            */
#define WTP_EHIP (-8)        /* a HIP runtime call failed                                      */

typedef struct wtp_tensor {
    const float* in;                 /* device, contiguous C order                      */
    float* out;                      /* device, same shape; may alias `in` (in place)   */
    int32_t ndim;                    /* 0..8; >= 2 takes the wavelet path (:63-85)      */
    int32_t reserved;
    int64_t shape[WTP_MAX_DIMS];
} wtp_tensor;

/* Written by the device, one per tensor (copy back after the stream completes). */
typedef struct wtp_result {
    int64_t numel;          /* weights in the tensor                                 */
    int64_t zero_count;     /* (pruned == 0).sum()        dwt_pruning.py:88-89        */
    int64_t coeff_numel;    /* size of the packed coefficient array (percentile pop.)*/
    double thr64;           /* np.percentile(np.abs(coeff_arr), pct)      :27        */
    uint32_t thr32_bits;    /* float32(thr64): the compare of :31 runs in float32    */
    uint32_t max_abs_bits;  /* np.max(np.abs(coeff_arr)) as float32 bits  :29-30     */
    int32_t eff_level;      /* min(level, calculate_max_level(shape))     :64-65     */
    int32_t path;           /* selection: 1 window candidates, 2 window edges, 3 full scan,
                               4 the one-launch small path (exact three-digit radix select);
                               + 8 (9, 10, 11): the fused selection's patch window missed the ranks
                               and the segment was selected again over its coefficients;
                               99 = the resident launch's grid was not co-resident (results invalid) */
} wtp_result;

/* ---- wavelets ---- */
int wtp_abi_version(void);
int wtp_wavelet_count(void);
const char* wtp_wavelet_name(int wavelet_id);
int wtp_wavelet_id(const char* name);           /* -1 if pywt would reject the name */
int wtp_dec_len(int wavelet_id);
int wtp_max_level(int64_t data_len, int dec_len); /* pywt.dwt_max_level */
int wtp_packed_shape(int64_t H, int64_t W, int level, int64_t* rows, int64_t* cols);

/* ---- the path: multi_resolution_analysis over a list of tensors ----
 * Semantics per tensor t, in order (exactly dwt_pruning.py:53-89):
 *   ndim < 2 : percentile_based_thresholding on the raw values (no wavelet check)
 *   ndim >= 2: level = min(level, max_level(min(H, W), dec_len)) -- the clamped level
 *              carries over to later tensors; wavedec2(periodization, axes (-2,-1));
 *              coeffs_to_array; threshold at the pct-th percentile of |coeffs| (NumPy 1.x
 *              linear interpolation, float32 compare); waverec2; crop; zero count.
 * Validation happens for all tensors before any device work; on error nothing is written.
 * Results: results_dev[t] (device memory).  Workspace: wtp_workspace_size bytes of device
 * memory (enough for wtp_prune_f32 and wtp_prune_layers_f32 of the same tensors; 0 if the
 * request itself is invalid), zeroed ONCE with wtp_workspace_init before first use; the library leaves it in
 * that state after every call (it is reusable by any later call with a workspace-size
 * request no larger than it). */
size_t wtp_workspace_size(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level);
int wtp_workspace_init(void* workspace, size_t bytes, wtp_stream_t stream);
int wtp_prune_f32(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, double pct,
                  void* workspace, size_t workspace_bytes, wtp_result* results_dev, wtp_stream_t stream);

/* wavelet_pruning / prune_layer_weights semantics (dwt_pruning.py:98-174): every tensor is an
 * independent call of multi_resolution_analysis([weight], ...), so the requested level is NOT
 * carried from one tensor to the next; otherwise identical to wtp_prune_f32 (one batched
 * launch sequence for all layers). */
int wtp_prune_layers_f32(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, double pct,
                         void* workspace, size_t workspace_bytes, wtp_result* results_dev, wtp_stream_t stream);

/* The general entry: flags = WTP_CARRY_LEVEL (wtp_prune_f32's level carry) | WTP_FLATTEN.
 * WTP_FLATTEN is the 1-D flattened mode (an extension: the reference's transform is 2-D): every
 * tensor with ndim >= 2 is transformed as ONE line, pywt.wavedec(w.ravel(), wavelet,
 * 'periodization', level) with the level clamped to pywt.dwt_max_level(numel, dec_len) (carried
 * over the list under WTP_CARRY_LEVEL), packed by pywt.coeffs_to_array ([cA_L | cD_L | ... |
 * cD_1]), thresholded at the pct-th percentile of |coeffs| exactly as the 2-D path, rebuilt by
 * pywt.waverec and cut to numel; ndim < 2 tensors keep the plain-percentile branch (:58-62).
 * WTP_NO_RESIDENT forces the three-launch form of level-0 groups for this call only (the retry of
 * tensors whose resident launch recorded WTP_PATH_FAULT).
 * Workspace: wtp_workspace_size_ex with the same flags. */
#define WTP_CARRY_LEVEL 1
#define WTP_FLATTEN 2
#define WTP_NO_RESIDENT 4
size_t wtp_workspace_size_ex(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, int flags);
int wtp_prune_ex_f32(const wtp_tensor* tensors, int ntensors, int wavelet_id, int level, double pct, int flags,
                     void* workspace, size_t workspace_bytes, wtp_result* results_dev, wtp_stream_t stream);

/* percentile_based_thresholding(arr, pct) on n device floats: out = where(|in| < thr, 0, in) */
int wtp_threshold_f32(const float* in, float* out, int64_t n, double pct, void* workspace,
                      size_t workspace_bytes, wtp_result* result_dev, wtp_stream_t stream);

/* components: batch of B images of H x W (row-major), packed coefficient array (B, rows, cols)
 * as wtp_packed_shape; waverec2 optionally thresholds every coefficient on load with the
 * float32 threshold read from thr32_dev (device pointer; NULL = no threshold) and crops to H x W. */
size_t wtp_dwt_workspace_size(int64_t B, int64_t H, int64_t W, int level);
int wtp_wavedec2_f32(const float* in, float* packed, int64_t B, int64_t H, int64_t W, int wavelet_id,
                     int level, void* workspace, size_t workspace_bytes, wtp_stream_t stream);
int wtp_waverec2_f32(const float* packed, float* out, int64_t B, int64_t H, int64_t W, int wavelet_id,
                     int level, const float* thr32_dev, void* workspace, size_t workspace_bytes,
                     wtp_stream_t stream);

/* synthetic inputs (csrc/wt_synth.h): out[k] = wt_synth_value(seed, tensor_id, k, e) */
int wtp_synth_f32(float* out, int64_t n, uint64_t seed, uint32_t tensor_id, int e, wtp_stream_t stream);

/* percentage_min_pruning (ResNet/min_weight_pruning.py:66-74) for a batch of tensors (the
 * min_weight_pruning baseline of :77-139): in every tensor zero the k = int(numel * fraction)
 * entries of smallest |w| (flattened).  Among entries with |w| equal to the k-th smallest the
 * lowest flat indices are pruned first (torch.topk leaves that order unspecified; counts are
 * exact either way).  k outside [0, numel] is WTP_EARG ("selected index k out of range").
 * out may alias in.  Results: numel, zero_count (zeros of out), thr64/thr32_bits = the k-th
 * smallest |w| (0 when k = 0).  Workspace: wtp_min_prune_workspace_size bytes, zeroed once
 * with wtp_workspace_init. */
size_t wtp_min_prune_workspace_size(const wtp_tensor* tensors, int ntensors, double fraction);
int wtp_min_prune_f32(const wtp_tensor* tensors, int ntensors, double fraction, void* workspace,
                      size_t workspace_bytes, wtp_result* results_dev, wtp_stream_t stream);

/* random_pruning (ResNet/random_pruning.py:49-56) for a batch of tensors: in tensor t zero
 * prune_counts[t] (host array; torch.randperm(numel)[:k] slicing: k > numel takes all, k < 0
 * takes numel + k) distinct flat positions drawn by a keyed pseudo-random permutation of
 * [0, numel) (csrc/wt_perm.h; seed + tensor index).  torch's Philox stream is not reproduced:
 * the positions differ from the reference's, the counts follow the same rule.  out may alias
 * in.  Results: numel and zero_count (zeros of out, NaN counted as non-zero). */
int wtp_random_prune_f32(const wtp_tensor* tensors, int ntensors, const int64_t* prune_counts, uint64_t seed,
                         wtp_result* results_dev, wtp_stream_t stream);

/* calculate_sparsity's count (testing_suite/eval_model.py:7-20): *count_dev = #(|x| < thr) over n
 * device floats (NaN is not counted). */
int wtp_count_small_f32(const float* x, int64_t n, float thr, unsigned long long* count_dev, wtp_stream_t stream);

/* measurement hook (bench.py): hipEvent_t handles recorded on the call's stream at the stage
 * boundaries of later wtp_prune*_f32 calls on this thread -- [0] start, [1] forward DWT done,
 * [2] k_window, [3] k_collect, [4] k_mask_select, [5] inverse DWT done (first segment group).
 * n = 0 disables. */
int wtp_set_stage_events(void* const* events, int n);

/* Level-0 launch groups whose chunks fit the device's co-resident grid (wtp_resident_capacity
 * workgroups of 49152 weights, one per CU) run as ONE launch that keeps every weight in
 * registers between its read and its masked write (k_resident).  It needs the CUs to itself
 * while it runs; mode 0 always uses the three-launch form (window / collect / mask-select).
 * Returns the previous mode (process-wide). */
int wtp_set_resident(int mode);
int wtp_resident_capacity(void); /* 0 if the current device cannot host the resident launch */
/* Bound (microseconds) of every wait inside the resident launch; returns the previous bound.  A
 * launch whose workgroups were not all resident at once times out there and stores NOTHING for
 * the tensors concerned (inputs and outputs untouched): their records read path == 99
 * (WTP_PATH_FAULT), and the caller re-runs exactly those tensors with wtp_set_resident(0).
 * Default 2000 (about 75x a full ResNet-18 resident launch), at most 40000000 (larger values are clamped: the bound is kept in 32-bit
 * ticks of the 100 MHz wall clock); tests lower it to force the fault path. */
unsigned wtp_set_resident_timeout_us(unsigned us);
#define WTP_PATH_FAULT 99
/* A call with more than one launch group (24 tensors) of wavelet-transformed tensors runs each
 * group's percentile selection on a side stream of the library's (one per device and caller
 * stream, non-blocking, created on first use), overlapping the next group's forward transform;
 * the caller's stream waits for it before that group's inverse, so the call stays ordered on
 * the caller's stream (graph capture included).  Mode 0: everything on the caller's stream; any
 * other value is rejected (WTP_EARG).  Returns the previous mode (process-wide). */
int wtp_set_pipeline(int mode);
/* Fused selection for launch groups of large wavelet-transformed tensors (each >= 2^22 packed
 * coefficients, every forward level in the tiled interior kernels, at most 6 levels, images of at
 * least 128 x 128): the percentile window comes from a transform of four 128 x 128 input patches
 * before the forward, the forward classifies the coefficients as it writes them, and the packed
 * array is not read again for the selection (identical results: a window that misses the ranks is
 * caught by the select, which then takes its exact full scan).  Mode 1 (default) on, 0 off; any
 * other value is rejected (WTP_EARG).  Returns the previous mode (process-wide). */
int wtp_set_fused_select(int mode);
/* The filter-bank levels run their interior tiles (input window inside the image, full tile)
 * in kernels compiled without the edge forms and the frame of edge tiles in the same kernels'
 * edge-capable form (mode 2); mode 3 (default) as 2, but a small level (a few thousand tiles)
 * runs every tile in one launch of the edge-capable form; mode 1: the frame in the general
 * kernel; mode 0: every tile in the general kernel (identical results in every mode).  Returns the
 * previous mode (process-wide). */
int wtp_set_interior(int mode);
#define WTP_PATH_SMALL 4 /* every tensor of the call ran in one launch (2-D transforms, small population) */
/* measurement hook (bench.py): while set, every resident launch atomically lowers stamps_dev[0] to
 * its first workgroup's start and raises stamps_dev[1] to its last workgroup's end (after that
 * workgroup's stores completed), in ticks of the 100 MHz wall clock -- the launch's span on the
 * device, free of the host's dispatch gaps.  The caller initialises [0] = ~0, [1] = 0; NULL = off. */
int wtp_set_kernel_stamps(unsigned long long* stamps_dev);

const char* wtp_last_error(void);
int wtp_last_error_tensor(void); /* index of the tensor that failed validation, or -1 */

#ifdef __cplusplus
}
#endif
#endif
