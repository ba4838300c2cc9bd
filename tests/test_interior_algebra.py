"""CPU check of the interior filter-bank kernels' index algebra (csrc/filterbank.hip k_fwd_int /
k_inv_int): their tile decomposition, sample offsets, tap parities and the interior rectangles the
host computes (fwd_interior / inv_interior), restated in float64 NumPy loop for loop and compared
with the C oracle's level-1 wavedec2 / waverec2 (pywt periodization) at every interior tile.  The
GPU suite checks the kernels themselves bit for bit (tests/test_gpu_large_levels.py); this test
catches an indexing slip without a GPU."""
import numpy as np
import pytest

from oracle import oracle as O

FR, FC, IR, IC = 16, 56, 64, 64  # filterbank.hip tile sizes


def _filters(wavelet):
    f = O.filters(wavelet)
    return [np.asarray(x, np.float64) for x in f]  # dec_lo, dec_hi, rec_lo, rec_hi


def _syn_locate(n, N, F):  # wt_dwt_core.h wt_syn_locate
    H, start = F // 2, F // 4
    M = 2 * N
    if H % 2 == 0:
        if n == M - 1:
            return start - 1, 0, True
        if n == 0:
            return start - 1, 1, True
        if n & 1:
            return start + (n - 1) // 2, 0, False
        return start + (n - 2) // 2, 1, False
    if n % 2 == 0:
        return start + n // 2, 0, False
    return start + (n - 1) // 2, 1, False


def _fwd_interior(R, C, F):  # filterbank.hip fwd_interior (al16 assumed)
    S0 = ((1 - F // 2) % 4 + 4) % 4
    TP = (S0 + 2 * FC + F - 2 + 3) // 4 * 4
    NR = 2 * FR + F - 2
    Ro, Co = (R + 1) // 2, (C + 1) // 2
    rows = [tr for tr in range((Ro + FR - 1) // FR)
            if 2 * FR * tr - F // 2 + 1 >= 0 and 2 * FR * tr - F // 2 + 1 + NR <= R and (tr + 1) * FR <= Ro]
    cols = [tc for tc in range((Co + FC - 1) // FC)
            if 2 * FC * tc - F // 2 + 1 - S0 >= 0 and 2 * FC * tc - F // 2 + 1 - S0 + TP <= C and (tc + 1) * FC <= Co]
    return rows, cols


def _inv_axis(out, N, F, T):  # filterbank.hip inv_axis
    H = F // 2
    ok = []
    for t in range((out + T - 1) // T):
        n0, nl = t * T, t * T + T - 1
        if nl >= out:
            continue
        i0, _, s0 = _syn_locate(n0, N, F)
        i1, _, s1 = _syn_locate(nl, N, F)
        if s0 or s1 or (H % 2 == 0 and (n0 == 0 or nl >= 2 * N - 1)):
            continue
        if i1 >= N or i0 - H + 1 < 0:
            continue
        ok.append(t)
    assert ok == list(range(ok[0], ok[-1] + 1)) if ok else True  # an interval
    return ok


@pytest.mark.parametrize("wavelet", ["db2", "rbio2.2", "bior3.3", "db5", "db8", "db9"])
def test_forward_interior_tiles(wavelet):
    lo, hi, _, _ = _filters(wavelet)
    F = len(lo)
    R, C = 200, 360
    rng = np.random.default_rng(F)
    x = rng.standard_normal((R, C)).astype(np.float32)
    P = O.wavedec2_packed(x, wavelet, 1).astype(np.float64)
    Ro, Co = R // 2, C // 2
    rows, cols = _fwd_interior(R, C, F)
    assert rows and cols
    xd = x.astype(np.float64)
    NCc = 2 * FC + F - 2
    for tr in rows:
        for tc in cols:
            o0r, o0c = tr * FR, tc * FC
            gr0, gc0 = 2 * o0r - F // 2 + 1, 2 * o0c - F // 2 + 1
            T = xd[gr0:gr0 + 2 * FR + F - 2, gc0:gc0 + NCc]
            Lr = np.zeros((FR, NCc)), np.zeros((FR, NCc))
            for h in range(2):  # column pass: item (h, cc), rows 8h + r from samples 16h + 2r + F - 1 - j
                for r in range(FR // 2):
                    for j in range(F):
                        s = T[FR * h + 2 * r + F - 1 - j]
                        Lr[0][FR // 2 * h + r] += lo[j] * s
                        Lr[1][FR // 2 * h + r] += hi[j] * s
            for o in range(FR):  # row pass: lane -> samples 2 lane + F - 1 - j
                for lane in range(FC):
                    idx = [2 * lane + F - 1 - j for j in range(F)]
                    aa = sum(lo[j] * Lr[0][o, idx[j]] for j in range(F))
                    ad = sum(hi[j] * Lr[0][o, idx[j]] for j in range(F))
                    da = sum(lo[j] * Lr[1][o, idx[j]] for j in range(F))
                    dd = sum(hi[j] * Lr[1][o, idx[j]] for j in range(F))
                    r, oc = o0r + o, o0c + lane
                    got = (aa, ad, da, dd)
                    want = (P[r, oc], P[r, Co + oc], P[Ro + r, oc], P[Ro + r, Co + oc])
                    assert np.allclose(got, want, rtol=1e-4, atol=1e-5), (tr, tc, o, lane)


@pytest.mark.parametrize("wavelet", ["db2", "rbio2.2", "bior3.3", "db5", "db8", "db9"])
def test_inverse_interior_tiles(wavelet):
    _, _, rlo, rhi = _filters(wavelet)
    F = len(rlo)
    H = F // 2
    R, C = 160, 200  # coefficients per subband; output 320 x 400
    rng = np.random.default_rng(100 + F)
    P = rng.standard_normal((2 * R, 2 * C)).astype(np.float32)
    y = O.waverec2_packed(P, (2 * R, 2 * C), wavelet, 1).astype(np.float64)
    Pd = P.astype(np.float64)
    outH, outW = 2 * R, 2 * C
    trs, tcs = _inv_axis(outH, R, F, IR), _inv_axis(outW, C, F, IC)
    assert trs and tcs
    NR = IR // 2 + H - (H & 1)
    NC = IC // 2 + H - (H & 1)
    PAR0 = 0 if H & 1 else 1
    PE1 = 0 if H & 1 else 1
    E = 0 if H & 1 else 1
    NV, RB, RB2 = H + 16 // 2 - 1 + E, 16, 8
    for tr in trs[:3]:
        for tc in tcs[:3]:
            n0, m0 = tr * IR, tc * IC
            r_lo = _syn_locate(n0, R, F)[0] - H + 1
            c_lo = _syn_locate(m0, C, F)[0] - H + 1
            assert _syn_locate(n0 + IR - 1, R, F)[0] - r_lo + 1 == NR
            A = np.stack([Pd[r_lo:r_lo + NR, c_lo:c_lo + NC], Pd[R + r_lo:R + r_lo + NR, c_lo:c_lo + NC]], -1)
            D = np.stack([Pd[r_lo:r_lo + NR, C + c_lo:C + c_lo + NC], Pd[R + r_lo:R + r_lo + NR, C + c_lo:C + c_lo + NC]], -1)
            LoHi = np.zeros((NR, IC, 2))
            for row in range(NR):  # row pass: lane = (row offset, column slot c), sub-pass p
                for c in range(32):
                    for p in range(2):
                        par = PAR0 if p == 0 else 1 - PAR0
                        pe = PE1 if p else 0
                        acc = np.zeros(2)
                        for j in range(H):
                            acc += rlo[2 * j + par] * A[row, c + pe + H - 1 - j]
                        for j in range(H):
                            acc += rhi[2 * j + par] * D[row, c + pe + H - 1 - j]
                        LoHi[row, 2 * c + p] = acc
            for wv in range(4):  # column pass: wave owns RB rows, outputs k and k + RB2 packed
                nf = n0 + RB * wv
                g0 = _syn_locate(nf, R, F)[0] - H + 1 - r_lo
                assert 0 <= g0 and g0 + NV <= NR
                rr = LoHi[g0:g0 + NV]
                for k in range(RB2):
                    par, base = (k + E) & 1, ((k + E) >> 1) + H - 1
                    for q, n in ((0, nf + k), (RB2 // 2, nf + k + RB2)):
                        acc = sum(rlo[2 * j + par] * rr[base - j + q, :, 0] for j in range(H))
                        acc = acc + sum(rhi[2 * j + par] * rr[base - j + q, :, 1] for j in range(H))
                        assert np.allclose(acc, y[n, m0:m0 + IC], rtol=1e-4, atol=1e-4), (tr, tc, n)
