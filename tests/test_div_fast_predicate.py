"""The predictor's proven fast division (cfd-simulations_amd/csrc/fields2d.hip,
div_fast): a quotient q1 is accepted only when |r| < RN(ub * kDivT) with
r = a - q1 b (one fma), ub = |b| 2^e (2^e: q1's power of two below its last
bit) and kDivT = RN((1/2 - 2^-20) 2^-23).  The acceptance must imply
q1 = RN(a / b).  These checks restate the predicate in NumPy float32 (every
product of two float32 is exact in float64, so one float64 product rounded to
float32 is the device's single rounding) and check

* the key inequality of the proof: the computed bound is strictly below
  |b| ulp(q1) / 2 for every |b|, q1 the guards admit, exponents swept;
* acceptance => correctly rounded, on random quotients and on quotients
  placed next to rounding midpoints, for the correctly rounded quotient and
  its two neighbours (the only candidates a one-Newton-step q1 can be).

This covers the predicate's arithmetic; the compiled kernel is pinned bit for
bit against the oracle by the -m gpu predictor tests.
"""
import numpy as np

F32, F64 = np.float32, np.float64
K_DIV_T = F32((0.5 - 2.0**-20) * 2.0**-23)


def _pow2_below(q):
    """2^e with e the exponent of bits(|q|) - 1 (the device's ulp base)."""
    b = (np.abs(q).view(np.uint32) - np.uint32(1)) & np.uint32(0x7F800000)
    return b.view(F32)


def _accept(a, b, q1):
    ab = np.abs(b)
    with np.errstate(over="ignore"):
        ub = (ab.astype(F64) * _pow2_below(q1).astype(F64)).astype(F32)
    thr = (ub.astype(F64) * F64(K_DIV_T)).astype(F32)
    r = (a.astype(F64) - q1.astype(F64) * b.astype(F64)).astype(F32)  # exact before the rounding
    with np.errstate(invalid="ignore"):
        return ((ab >= 2.0**-100) & (np.abs(q1) >= 2.0**-100) & (ub >= 2.0**-100) & (ub <= 2.0**100)
                & (np.abs(r) < thr))


def _rn_quotient(a, b):
    """RN(a / b) in float32 without double rounding: the float64 quotient's
    float32 rounding and its neighbours, the one with the smallest exact
    |a - c b| (b > 0 here)."""
    q = (a.astype(F64) / b.astype(F64)).astype(F32)
    cands = np.stack([np.nextafter(q, F32(-np.inf)), q, np.nextafter(q, F32(np.inf))])
    res = np.abs(a.astype(F64)[None] - cands.astype(F64) * b.astype(F64)[None])
    return cands[np.argmin(res, axis=0), np.arange(a.size)]


def test_bound_strictly_below_half_ulp():
    rng = np.random.default_rng(7)
    n = 400_000
    for eb in (-99, -60, -20, -1, 0, 1, 30, 60, 99):
        b = (rng.uniform(1.0, 2.0, n) * 2.0**eb).astype(F32)
        for eq in (-99, -40, -1, 0, 1, 40, 99):
            q1 = (rng.uniform(1.0, 2.0, n) * 2.0**eq).astype(F32)
            q1[:4] = F32(2.0**eq)  # powers of two: the lower binade's ulp
            ab = b.astype(F64)
            with np.errstate(over="ignore"):
                ub = (ab * _pow2_below(q1).astype(F64)).astype(F32)
            ok = (ub >= 2.0**-100) & (ub <= 2.0**100)
            thr = (ub.astype(F64) * F64(K_DIV_T)).astype(F32).astype(F64)
            half = ab * _pow2_below(q1).astype(F64) * 2.0**-23 / 2  # exact: |b| ulp / 2
            assert np.all(thr[ok] < half[ok]), (eb, eq)


def test_acceptance_implies_correct_rounding():
    rng = np.random.default_rng(11)
    n = 2_000_000
    b = (rng.uniform(1.0, 2.0, n) * 2.0 ** rng.integers(-30, 30, n)).astype(F32)
    a = (rng.uniform(1.0, 2.0, n) * 2.0 ** rng.integers(-30, 30, n)).astype(F32)
    q = _rn_quotient(a, b)
    for q1 in (np.nextafter(q, F32(-np.inf)), q, np.nextafter(q, F32(np.inf))):
        acc = _accept(a, b, q1)
        assert np.all(q1[acc] == q[acc])
    # the correctly rounded quotient is accepted almost always (the margin is 2^-20)
    assert _accept(a, b, q).mean() > 1 - 1e-4


def test_near_midpoint_quotients():
    # a = RN(m b) for the midpoint m between q and its successor: a / b lands
    # within an ulp of the midpoint, the near ones where the test must refuse
    rng = np.random.default_rng(13)
    n = 2_000_000
    q = rng.uniform(1.0, 2.0, n).astype(F32)
    b = rng.uniform(1.0, 2.0, n).astype(F32)
    m = (q.astype(F64) + np.nextafter(q, F32(np.inf)).astype(F64)) / 2
    a = (m * b.astype(F64)).astype(F32)
    rn = _rn_quotient(a, b)
    dist = np.abs(a.astype(F64) / b.astype(F64) - m) / (np.nextafter(q, F32(np.inf)) - q).astype(F64)
    assert (dist < 2.0**-16).sum() > 10  # the sample reaches the margin's neighbourhood
    for q1 in (np.nextafter(rn, F32(-np.inf)), rn, np.nextafter(rn, F32(np.inf))):
        acc = _accept(a, b, q1)
        assert np.all(q1[acc] == rn[acc])
