/* CPU check of csrc/fb_index.h (the filter-bank kernels' tile decode), compiled for the host:
 * the Granlund-Montgomery divisions against n / d, the XCD-aware tile order as a permutation, and
 * the frame decode listing every tile outside the interior rectangle exactly once.  Each entry
 * returns the number of mismatches (0 = pass). */
#include <cstdint>
#include <random>
#include <vector>

#include "../../wavelettransforms_amd/csrc/fb_index.h"

using namespace wtp;

static int check_div(uint32_t d, int n) { return fdiv(n, make_fastdiv(d)) != (int)((uint32_t)n / d); }

extern "C" int fb_check_fdiv(void) {
    int bad = 0;
    std::mt19937_64 rng(12345);
    for (uint32_t d = 1; d <= 65536; ++d) {
        const FastDiv f = make_fastdiv(d);
        auto one = [&](int64_t n) {
            if (n < 0 || n > INT32_MAX) return;
            bad += fdiv((int)n, f) != (int)((uint32_t)n / d);
        };
        for (int64_t n = 0; n < 64; ++n) one(n);
        for (int64_t k : {int64_t(1), int64_t(2), int64_t(3), int64_t(1000), int64_t(INT32_MAX / d)})
            for (int64_t e = -1; e <= 1; ++e) one(k * d + e);
        for (int64_t n : {int64_t(INT32_MAX), int64_t(INT32_MAX - 1), int64_t(1) << 30, (int64_t(1) << 30) - 1}) one(n);
        for (int r = 0; r < 16; ++r) one((int64_t)(rng() & 0x7FFFFFFF));
    }
    for (int r = 0; r < 200000; ++r) { /* random divisors up to 2^31, random and near-multiple dividends */
        const uint32_t d = (uint32_t)(rng() % 0x7FFFFFFFu) + 1u;
        bad += check_div(d, (int)(rng() & 0x7FFFFFFF));
        const uint64_t k = rng() % ((uint64_t)INT32_MAX / d + 1);
        const int64_t m = (int64_t)(k * d);
        if (m <= INT32_MAX) bad += check_div(d, (int)m);
        if (m >= 1) bad += check_div(d, (int)(m - 1));
    }
    return bad;
}

extern "C" int fb_check_xcd(void) {
    int bad = 0;
    for (int n = 1; n <= 3000; ++n) {
        std::vector<int> seen(n, 0);
        for (int b = 0; b < n; ++b) {
            const int t = xcd_tile(b, n);
            if (t < 0 || t >= n) { ++bad; continue; }
            ++seen[t];
        }
        for (int t = 0; t < n; ++t) bad += seen[t] != 1;
    }
    return bad;
}

/* every (tilesR, tilesC) up to 12 x 12 and every rectangle in it, empty ones (nr = 0) and
 * full-width ones (nc = tilesC) included */
extern "C" int fb_check_frame(void) {
    int bad = 0;
    for (int tilesR = 1; tilesR <= 12; ++tilesR)
        for (int tilesC = 1; tilesC <= 12; ++tilesC)
            for (int r0 = 0; r0 <= tilesR; ++r0)
                for (int nr = 0; r0 + nr <= tilesR; ++nr)
                    for (int c0 = 0; c0 < tilesC; ++c0)
                        for (int nc = 1; c0 + nc <= tilesC; ++nc) {
                            const int per = tilesR * tilesC - nr * nc;
                            const FastDiv dtc = make_fastdiv((uint32_t)tilesC);
                            const FastDiv dside = make_fastdiv((uint32_t)(tilesC - nc > 1 ? tilesC - nc : 1));
                            std::vector<int> seen(tilesR * tilesC, 0);
                            for (int f = 0; f < per; ++f) {
                                int tr, tc, tr2, tc2;
                                frame_tile(f, tilesC, r0, nr, c0, nc, &tr, &tc);
                                frame_tile_fd(f, tilesC, r0, nr, c0, nc, dtc, dside, &tr2, &tc2);
                                if (tr != tr2 || tc != tc2) ++bad;
                                if (tr < 0 || tr >= tilesR || tc < 0 || tc >= tilesC) { ++bad; continue; }
                                if (tr >= r0 && tr < r0 + nr && tc >= c0 && tc < c0 + nc) ++bad; /* inside */
                                ++seen[tr * tilesC + tc];
                            }
                            for (int t = 0; t < tilesR * tilesC; ++t) {
                                const int tr = t / tilesC, tc = t % tilesC;
                                const bool inside = tr >= r0 && tr < r0 + nr && tc >= c0 && tc < c0 + nc;
                                bad += seen[t] != (inside ? 0 : 1);
                            }
                        }
    return bad;
}
