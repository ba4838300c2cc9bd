/* Sanitizer driver (ASan/UBSan for the CPU restatement): the C oracle
 * (oracle/wtprune_oracle.c, compiled into this program) over every wavelet, odd / even / tiny /
 * empty shapes, levels past the maximum, percentiles 0..100, NaN / inf / ties, the flattened mode,
 * min-weight and random pruning.  Built and run by tests/test_sanitizers.py with
 * -fsanitize=address,undefined -fno-sanitize-recover=all: any report aborts the run. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/wtprune_oracle.c"

static float* synth(int64_t n, uint32_t tid, int e, int special) {
    float* x = (float*)malloc((size_t)(n ? n : 1) * sizeof(float));
    or_synth_fill(x, n, 7, tid, e);
    if (special && n > 8) {
        x[1] = NAN;
        x[n / 2] = INFINITY;
        x[n - 1] = -INFINITY;
        x[3] = x[4];
    }
    return x;
}

static void run_tensor(int ndim, const int64_t* shape, int wid, int level, double pct, int special, int flat) {
    int64_t n = 1;
    for (int i = 0; i < ndim; ++i) n *= shape[i];
    float* x = synth(n, (uint32_t)(wid * 131 + level), 24, special);
    float* y = (float*)malloc((size_t)(n ? n : 1) * sizeof(float));
    or_result r;
    if (flat) (void)or_prune_tensor_flat(n ? x : 0, n ? y : 0, ndim, shape, wid, level, pct, &r, 0);
    else (void)or_prune_tensor(n ? x : 0, n ? y : 0, ndim, shape, wid, level, pct, &r, 0);
    free(x);
    free(y);
}

int main(void) {
    static const int64_t shapes[][4] = {{64, 3, 7, 7}, {8, 4, 3, 3}, {16, 8, 1, 1}, {2, 2, 9, 5},
                                        {96, 100, 0, 0}, {33, 65, 0, 0}, {1, 1, 1, 1}, {3, 130, 97, 0}};
    static const int ndims[] = {4, 4, 4, 4, 2, 2, 4, 3};
    static const double pcts[] = {0.0, 10.0, 23.599999999999998, 50.0, 61.8, 99.9, 100.0};
    const int nw = or_num_wavelets();
    long cases = 0;
    for (int w = 0; w < nw; ++w)
        for (int s = 0; s < 8; ++s)
            for (int level = 0; level <= 6; level += 3)
                for (int p = 0; p < 7; p += 2) {
                    run_tensor(ndims[s], shapes[s], w, level, pcts[p], (s + p) & 1, (w + s) % 3 == 0);
                    ++cases;
                }
    /* 1-D tensors, empty tensors, scalars */
    const int64_t v1000[1] = {1000}, v0[1] = {0}, e2[2] = {0, 5};
    for (int p = 0; p < 7; ++p) {
        run_tensor(1, v1000, 0, 5, pcts[p], p & 1, 0);
        run_tensor(1, v0, 0, 5, pcts[p], 0, 0);
        run_tensor(2, e2, 3, 2, pcts[p], 0, 0);
        run_tensor(0, v0, 0, 5, pcts[p], 0, 0);
        cases += 4;
    }
    /* min-weight and random pruning */
    for (int k = 0; k < 6; ++k) {
        const int64_t n = 1 + 997 * k;
        float* x = synth(n, (uint32_t)k, 20, k & 1);
        float* y = (float*)malloc((size_t)n * sizeof(float));
        int64_t zc;
        float t;
        (void)or_min_prune(x, y, n, 0.1 * k, &zc, &t);
        (void)or_random_prune(x, y, n, n / (k + 1), 99, (uint32_t)k, &zc);
        free(x);
        free(y);
        cases += 2;
    }
    printf("sancheck: %ld cases clean\n", cases);
    return 0;
}
