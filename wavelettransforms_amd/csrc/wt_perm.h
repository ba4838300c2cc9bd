/* Keyed pseudo-random permutation of [0, n) for random pruning (ResNet/random_pruning.py:53-55
 * draws torch.randperm(numel)[:prune_count]).  The positions pruned are perm(0..k-1): k
 * distinct, uniformly spread indices, computed independently per j (no sort, no shuffle pass).
 * torch's Philox stream is not reproduced -- the reference's own logs pin only the counts.
 *
 *   b = bit width of n - 1, rounded up to an even number (>= 2); h = b / 2
 *   x -> four Feistel rounds on (hi h bits, lo h bits): (L, R) -> (R, L ^ (f_r(R) & mask_h)),
 *        f_r(R) = splitmix64(key + r * 0x9E3779B97F4A7C15 + R)
 *   cycle-walk: repeat while x >= n (2^b < 4n, so < 4 steps expected; every cycle of the
 *   permutation of [0, 2^b) that holds an index < n returns to [0, n))
 * Shared by the HIP library (device) and the C oracle (host).
 */
#ifndef WT_PERM_H
#define WT_PERM_H

#include <stdint.h>

#include "wt_synth.h"

#if defined(__HIPCC__)
#define WT_PD __host__ __device__ __forceinline__
#else
#define WT_PD static inline
#endif

WT_PD int wt_perm_half_bits(uint64_t n) {
    int b = 2;
    while (b < 64 && ((uint64_t)1 << b) < n) b += 2;
    return b / 2;
}

WT_PD uint64_t wt_perm_key(uint64_t seed, uint32_t tensor_id) {
    return wt_splitmix64(seed ^ ((uint64_t)tensor_id * 0xD1B54A32D192ED03ull));
}

WT_PD uint64_t wt_perm_round(uint64_t x, int h, uint64_t key) {
    const uint64_t mask = ((uint64_t)1 << h) - 1;
    for (int r = 0; r < 4; ++r) {
        const uint64_t L = x >> h, R = x & mask;
        const uint64_t f = wt_splitmix64(key + (uint64_t)r * 0x9E3779B97F4A7C15ull + R) & mask;
        x = (R << h) | (L ^ f);
    }
    return x;
}

/* perm(j) for 0 <= j < n */
WT_PD uint64_t wt_perm(uint64_t j, uint64_t n, int h, uint64_t key) {
    uint64_t x = wt_perm_round(j, h, key);
    while (x >= n) x = wt_perm_round(x, h, key);
    return x;
}

#endif
