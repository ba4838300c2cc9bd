/* Brute-force check of small_geom.h (the one-launch small path's tile windows): for every tile
 * of many shapes, filters and levels, every sample an owned (or window) output reads -- by the
 * analysis rule of wt_ana_point and the synthesis rule of wt_syn_pass -- must lie in the window
 * of the level below, and the owned ranges must partition every level.  Exit status 0 = pass. */
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../wavelettransforms_amd/csrc/wt_dwt_core.h"
#include "../../wavelettransforms_amd/csrc/small_geom.h"

static bool in_ivl(SmIvl w, int N, int x) { return sm_pm(x - w.s, N) < w.len; }

static int check_axis(int N0, int L, int F, int T) {
    int32_t N[SM_MAX_L + 1];
    N[0] = N0;
    for (int k = 1; k <= L; ++k) N[k] = (N[k - 1] + 1) / 2;
    const int tiles = (N[L] + T - 1) / T;
    std::vector<int> owner[SM_MAX_L + 1];
    for (int k = 0; k <= L; ++k) owner[k].assign(N[k], -1);
    int bad = 0;
    for (int t = 0; t < tiles; ++t) {
        SmAxis a;
        sm_axis(t, T, L, N, F, &a);
        for (int k = 0; k <= L; ++k) {
            if (a.ohi[k] <= a.olo[k]) { ++bad; continue; }
            for (int i = a.olo[k]; i < a.ohi[k]; ++i) {
                if (owner[k][i] != -1) ++bad;
                owner[k][i] = t;
            }
            if (a.fw[k].len < 1 || a.fw[k].len > N[k] || a.fw[k].s < 0 || a.fw[k].s >= N[k]) ++bad;
        }
        /* forward: outputs of window k read ext(F/2 + 2o - j) of level k-1, inside window k-1;
         * the owned outputs of every level are inside its window */
        for (int k = 1; k <= L; ++k) {
            for (int m = 0; m < a.fw[k].len; ++m) {
                const int o = (a.fw[k].s + m) % N[k];
                for (int j = 0; j < F; ++j) {
                    const int src = (int)wt_ext_index(F / 2 + 2 * (int64_t)o - j, N[k - 1]);
                    if (!in_ivl(a.fw[k - 1], N[k - 1], src)) ++bad;
                }
            }
            for (int i = a.olo[k]; i < a.ohi[k]; ++i)
                if (!in_ivl(a.fw[k], N[k], i)) ++bad;
        }
        /* inverse: outputs of window k-1 (sv[k-1], own_0 at k = 1) read pmod(i - j, N_k) of sv[k] */
        for (int i = a.olo[0]; i < a.ohi[0]; ++i)
            if (!in_ivl(a.sv[0], N[0], i)) ++bad;
        for (int k = 1; k <= L; ++k) {
            if (a.sv[k].len < 1 || a.sv[k].len > N[k] || a.sv[k].s < 0 || a.sv[k].s >= N[k]) ++bad;
            for (int m = 0; m < a.sv[k - 1].len; ++m) {
                const int n = (a.sv[k - 1].s + m) % N[k - 1];
                const wt_syn_site s = wt_syn_locate(n, N[k], F);
                for (int j = 0; j < F / 2; ++j)
                    if (!in_ivl(a.sv[k], N[k], (int)wt_pmod(s.i - j, N[k]))) ++bad;
            }
        }
    }
    for (int k = 0; k <= L; ++k)
        for (int i = 0; i < N[k]; ++i)
            if (owner[k][i] < 0) ++bad;
    if (bad) printf("FAIL N0=%d L=%d F=%d T=%d: %d\n", N0, L, F, T, bad);
    return bad;
}

int main() {
    int bad = 0, cases = 0;
    const int Fs[] = {2, 4, 6, 8, 10, 12, 16, 18, 20};
    for (int N0 = 1; N0 <= 140; N0 += (N0 < 40 ? 1 : 7))
        for (int F : Fs)
            for (int L = 1; L <= 6; ++L) {
                int n = N0;
                for (int k = 0; k < L; ++k) n = (n + 1) / 2;
                for (int T = 1; T <= n; T = T < 4 ? T + 1 : 2 * T) {
                    bad += check_axis(N0, L, F, T) != 0;
                    ++cases;
                }
            }
    bad += check_axis(784, 3, 6, 4) != 0;
    bad += check_axis(784, 3, 6, 2) != 0;
    bad += check_axis(128, 3, 6, 16) != 0;
    printf("%d cases, %d failing\n", cases + 3, bad);
    return bad ? 1 : 0;
}
