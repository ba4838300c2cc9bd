/* Deterministic, NumPy-free synthetic weight generator shared by the HIP library (device),
 * the C oracle (host) and tools/gen_golden.py (NumPy restatement, checked by tests).
 *
 *   key  = (seed << 40) ^ (tensor_id << 32) ^ k                 (k < 2^32 element index)
 *   h_i  = splitmix64(key + i * 0x9E3779B97F4A7C15), i = 0..3
 *   z    = sum_i (h_i >> 42) - 2^23                               (Irwin-Hall, |z| <= 2^23)
 *   w    = ldexp((float)z, -e)                                    (exact: z fits in 24 bits)
 *
 * sigma(z) = 2^22 / sqrt(3); e = round(log2(sigma(z) / sigma_target)) is chosen on the host
 * (wt_synth_exponent) and passed in, so device and host agree bit for bit.  Integer-valued z
 * produces exact ties, which exercises np.partition tie semantics in the percentile.
 */
#ifndef WT_SYNTH_H
#define WT_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define WT_HD __host__ __device__ __forceinline__
#else
#define WT_HD static inline
#endif

WT_HD uint64_t wt_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

WT_HD float wt_synth_value(uint64_t seed, uint32_t tensor_id, uint64_t k, int e) {
    const uint64_t key = (seed << 40) ^ ((uint64_t)tensor_id << 32) ^ k;
    int64_t z = 0;
    for (int i = 0; i < 4; ++i)
        z += (int64_t)(wt_splitmix64(key + (uint64_t)i * 0x9E3779B97F4A7C15ull) >> 42);
    z -= (int64_t)1 << 23;
    /* ldexp by an integer power of two, exact for |z| < 2^24 and e < 100 */
    float v = (float)z;
    while (e > 60) { v *= 0x1p-60f; e -= 60; }
    union { uint32_t u; float f; } s;
    s.u = (uint32_t)(127 - e) << 23;
    return v * s.f;
}

#endif
