/* Tile-index arithmetic of the filter-bank kernels (filterbank.hip), shared with the host-compiled
 * CPU check tests/native/fbindex.cpp: the scalar-unit divisions by launch-invariant divisors, the
 * XCD-aware tile order and the decode of a level's frame of edge tiles. */
#ifndef WT_FB_INDEX_H
#define WT_FB_INDEX_H

#include <stdint.h>

#if defined(__HIPCC__)
#define WT_FB __host__ __device__ __forceinline__
#else
#define WT_FB inline
#endif

namespace wtp {

WT_FB uint32_t fb_umulhi(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

/* division by a launch-invariant d on the scalar unit (Granlund-Montgomery, exact for every 32-bit
 * n): the tile decode's quotients are uniform, and the compiler's own division expands to a
 * float reciprocal sequence on the VALU of every wave */
struct FastDiv {
    uint32_t m, sh; /* sh: first shift (0 or 1) | second shift << 8 */
};
WT_FB int fdiv(int n, const FastDiv& f) {
    const uint32_t u = (uint32_t)n, t = fb_umulhi(u, f.m);
    return (int)((t + ((u - t) >> (f.sh & 0xFFu))) >> (f.sh >> 8));
}
inline FastDiv make_fastdiv(uint32_t d) { /* host */
    int l = 0;
    while (l < 32 && (1ull << l) < d) ++l;
    FastDiv f;
    f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    f.sh = l ? (1u | ((uint32_t)(l - 1) << 8)) : 0u;
    return f;
}

/* XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (blocks b and b+8
 * share one L2), so tile t = xcd * per + b / 8 gives each XCD a contiguous run of tiles and the
 * halos neighbouring tiles re-read come from that XCD's L2 (MI355X_MICROARCH.md, XCD placement;
 * placement is a speed matter only, never correctness) */
WT_FB int xcd_tile(int b, int n) {
    const int per = (n + 7) / 8, x = b & 7, k = b >> 3;
    const int full = n - 8 * (per - 1); /* XCDs that get `per` tiles; the rest get per - 1 */
    return x < full ? x * per + k : full * per + (x - full) * (per - 1) + k;
}

/* frame index f -> tile (tr, tc) of a grid of tilesC columns around the interior rectangle
 * [r0, r0 + nr) x [c0, c0 + nc): the rows above it, then the side tiles of its rows, then the
 * rows below it (row-major inside each part) */
WT_FB void frame_tile(int f, int tilesC, int r0, int nr, int c0, int nc, int* tr, int* tc) {
    const int top = r0 * tilesC, side = tilesC - nc;
    if (f < top) {
        *tr = f / tilesC;
        *tc = f - *tr * tilesC;
        return;
    }
    f -= top;
    if (f < nr * side) {
        const int q = f / side, k = f - q * side;
        *tr = r0 + q;
        *tc = k < c0 ? k : k + nc;
        return;
    }
    f -= nr * side;
    *tr = r0 + nr + f / tilesC;
    *tc = f - (f / tilesC) * tilesC;
}

/* frame_tile with the divisions by tilesC and tilesC - nc on the scalar unit */
WT_FB void frame_tile_fd(int f, int tilesC, int r0, int nr, int c0, int nc, const FastDiv& dtc,
                                              const FastDiv& dside, int* tr, int* tc) {
    const int top = r0 * tilesC, side = tilesC - nc;
    if (f < top) {
        *tr = fdiv(f, dtc);
        *tc = f - *tr * tilesC;
        return;
    }
    f -= top;
    if (f < nr * side) {
        const int q = fdiv(f, dside), k = f - q * side;
        *tr = r0 + q;
        *tc = k < c0 ? k : k + nc;
        return;
    }
    f -= nr * side;
    const int q = fdiv(f, dtc);
    *tr = r0 + nr + q;
    *tc = f - q * tilesC;
}

}  // namespace wtp

#endif
