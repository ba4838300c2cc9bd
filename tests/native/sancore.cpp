// Sanitizer driver for the product's host-compilable filter-bank core (csrc/wt_dwt_core.h, via
// corecheck.cpp): every filter length 2..20, line lengths 1..80 (odd and even), the packed
// geometry of every level up to the maximum.  Built and run by tests/test_sanitizers.py with
// -fsanitize=address,undefined -fno-sanitize-recover=all: any report aborts the run.
#include <cstdio>
#include <vector>

#include "corecheck.cpp"

int main() {
    long cases = 0;
    for (int F = 2; F <= 20; F += 2) {
        std::vector<float> lo(F), hi(F), rlo(F), rhi(F);
        for (int j = 0; j < F; ++j) {
            lo[j] = 0.1f * (j + 1);
            hi[j] = (j & 1) ? -lo[j] : lo[j];
            rlo[j] = lo[F - 1 - j];
            rhi[j] = hi[F - 1 - j];
        }
        for (long long N = 1; N <= 80; ++N) {
            std::vector<float> x(N), a((N + 1) / 2), d((N + 1) / 2), y(2 * ((N + 1) / 2));
            for (long long i = 0; i < N; ++i) x[i] = (float)((i * 37) % 11) - 5.0f;
            core_dwt1(x.data(), N, F, lo.data(), hi.data(), a.data(), d.data());
            core_idwt1(a.data(), d.data(), (N + 1) / 2, F, rlo.data(), rhi.data(), y.data());
            ++cases;
        }
    }
    for (long long H = 1; H <= 70; H += 3)
        for (long long W = 1; W <= 70; W += 5)
            for (int L = 0; L <= 6; ++L) {
                long long out[2 + 4 * 8];
                core_geom(H, W, L, out);
                ++cases;
            }
    std::printf("sancore: %ld cases clean\n", cases);
    return 0;
}
