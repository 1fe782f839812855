"""Pins the Soft-NMS kernel's exp (repurpose_amd/csrc/rp_infer.hip, np_expf) to numpy's float32 exp.

The reference decays scores with ``np.exp(-(overlap_ratio**2) / sigma)`` on float32 arrays
(models/softnms.py:35).  numpy runs its own SIMD float32 exp there on AVX2 / AVX512F hosts, which is
not correctly rounded: about 10 % of the float32 inputs in [-2, 0] come out one ulp away from the
correctly rounded value.  ``np_expf_restated`` is the algorithm the kernel implements (Cody-Waite
reduction with a two-part ln 2, [5/2] rational minimax polynomial by FMAs, IEEE division, 2^k
scale), evaluated here with exact FMAs (long-double products of float32 are exact).

    python tests/golden/np_exp_check.py [--all]

--all sweeps every float32 in [-2, 0] (1,073,741,825 values, ~6 min on 8 cores; the decay's domain
for the config's sigma = 0.5) — run on this container's numpy 2.2.6 (AVX512F dispatch): 0 mismatches.
Without --all a seeded 2^22-value sample (also run by tests/test_oracle.py).
"""
import sys

import numpy as np

F = np.float32
C1, C2 = F(-6.93145752e-1), F(-1.42860677e-6)
P = [F(9.999999999980870924916e-01), F(7.257664613233124478488e-01), F(2.473615434895520810817e-01),
     F(5.114512081637298353406e-02), F(6.757896990527504603057e-03), F(5.082762527590693718096e-04)]
Q = [F(1.0), F(-2.742335390411667452936e-01), F(2.159509375685829852307e-02)]
L2E = F(1.442695040888963407359924681001892137)


def _fma(a, b, c):
    r = np.asarray(a, np.longdouble) * np.asarray(b, np.longdouble) + np.asarray(c, np.longdouble)
    return r.astype(np.float32)


def np_expf_restated(x):
    x = np.asarray(x, np.float32)
    q = np.rint((x * L2E).astype(np.float32))
    y = _fma(q, C1, x)
    y = _fma(q, C2, y)
    num = _fma(P[5], y, P[4])
    for c in (P[3], P[2], P[1], P[0]):
        num = _fma(num, y, c)
    den = _fma(_fma(Q[2], y, Q[1]), y, Q[0])
    return np.ldexp((num / den).astype(np.float32), q.astype(np.int32)).astype(np.float32)


def sample_mismatches(n=1 << 22, seed=0):
    rs = np.random.RandomState(seed)
    x = -rs.uniform(0, 2, n).astype(np.float32)
    return int((np_expf_restated(x) != np.exp(x)).sum()), n


def sweep():
    lo, hi = 0x80000000, int(np.float32(-2.0).view(np.uint32))
    bad = n = 0
    for s in range(lo, hi + 1, 1 << 24):
        x = np.arange(s, min(s + (1 << 24), hi + 1), dtype=np.uint64).astype(np.uint32).view(np.float32)
        bad += int((np_expf_restated(x) != np.exp(x)).sum())
        n += len(x)
    return bad, n


if __name__ == "__main__":
    bad, n = sweep() if "--all" in sys.argv else sample_mismatches()
    cr = -np.random.RandomState(1).uniform(0, 2, 1 << 20).astype(np.float32)
    off = int((np.exp(cr) != np.exp(cr.astype(np.float64)).astype(np.float32)).sum())
    print(f"restated vs np.exp: {bad} mismatches of {n}; np.exp vs correctly rounded: {off} of {1 << 20} differ")
