"""The bitset builder's draw ranges (gw_n2v_bitset.hip: bs_div32 / bs_draw_range).

A region entry's draw filter sets bucket floor(y * F / 2^32) for every 32-bit
draw word y whose index floor(y * d / 2^32) is a common position k, i.e. for
y in [floor(k * 2^32 / d), ceil((k + 1) * 2^32 / d) - 1].  The device computes
both ends from inv = 2^32 / d in double precision plus one integer correction
instead of two 64-bit divisions.  This restates that computation (IEEE double,
truncation like the C cast) and checks it against exact integer arithmetic on
random and extreme (k, d); the GPU side is covered by the walk-parity tests,
which read the filters.
"""
import numpy as np


def _div32(k, d, inv):
    q = np.trunc(k.astype(np.float64) * inv).astype(np.int64)
    r = (k << 32) - q * d
    lo, hi = r < 0, r >= d
    q = np.where(lo, q - 1, np.where(hi, q + 1, q))
    r = np.where(lo, r + d, np.where(hi, r - d, r))
    assert ((r >= 0) & (r < d)).all()  # one correction always suffices
    return q, r == 0


def _ranges(k, d):
    inv = 4294967296.0 / d.astype(np.float64)
    ylo, _ = _div32(k, d, inv)
    q1, exact = _div32(k + 1, d, inv)
    return ylo, q1 - exact.astype(np.int64)


def test_reciprocal_draw_range_is_exact():
    rng = np.random.default_rng(5)
    cases = []
    for lo, hi in ((353, 70000), (65536, 1 << 24), (1 << 24, (1 << 31) - 1)):
        d = rng.integers(lo, hi, 4000, dtype=np.int64)
        k = np.minimum((rng.random(4000) * d).astype(np.int64), d - 1)
        cases.append((k, d))
        cases.append((d - 1, d))          # last position
        cases.append((np.zeros_like(d), d))  # first position
    d = np.array([353, 354, 4096, 65535, 65536, (1 << 31) - 1], dtype=np.int64)
    cases.append((d - 1, d))
    for k, d in cases:
        ylo, yhi = _ranges(k, d)
        elo = np.array([(int(a) << 32) // int(b) for a, b in zip(k, d)])
        ehi = np.array([(((int(a) + 1) << 32) + int(b) - 1) // int(b) - 1 for a, b in zip(k, d)])
        np.testing.assert_array_equal(ylo, elo)
        np.testing.assert_array_equal(yhi, ehi)
