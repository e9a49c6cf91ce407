"""The row-minimum arithmetic of k_cosine_sym (cms_cosine_sym.hip), restated
on the host and checked against the reference's own fp64 expression.

DoubleCountMinSketch.cosine (T/impl/common/DoubleCountMinSketch.java:139-147)
forms each sketch row's value as valueAB / (sqrt(valueA) * sqrt(valueB)), both
operations rounded to double, and keeps the minimum over rows.  The kernel
decides "row r's value < the running minimum's" in two ways this file pins:

* near ties: exact_less compares the FMA-split cross products instead of the
  two quotients; wherever it answers "less" the reference's quotient is <=
  (equal only when both round to the same double), and wherever it answers
  "not less" the reference's quotient is >=;
* the estimate form of the running minimum: an fp32 estimate of AB/(sa*sb)
  with its low rbits mantissa bits replaced by the row; AB is recovered
  exactly as rint(est * sa * sb) while AB <= 0.5 / (2^-21 + 2^(rbits-23)).
"""
import math
import random
from fractions import Fraction

import numpy as np
import pytest


def _fma_err(a, b, p):
    """The exact error of the rounded product p = a * b (what __fma_rn(a, b, -p) returns)."""
    return float(Fraction(a) * Fraction(b) - Fraction(p))


def exact_less(ab, sa, sb, ab0, sa0, sb0):
    D, D0 = sa * sb, sa0 * sb0
    p1 = ab * D0
    e1 = _fma_err(ab, D0, p1)
    p2 = ab0 * D
    e2 = _fma_err(ab0, D, p2)
    return p1 < p2 or (p1 == p2 and e1 < e2)


def ref_value(ab, sa, sb):
    return ab / (sa * sb)


def _cases(rng, n):
    for _ in range(n):
        A = rng.randint(1, 1 << 27)
        B = rng.randint(1, 1 << 27)
        ab = rng.randint(0, 1 << 20)
        sa, sb = math.sqrt(A), math.sqrt(B)
        kind = rng.random()
        if kind < 0.3:  # the same row value (identical rows of the two owners)
            yield ab, sa, sb, ab, sa, sb
        elif kind < 0.6:  # a second row whose exact ratio is within a few ulps
            A0 = A + rng.randint(-3, 3) or 1
            B0 = B + rng.randint(-3, 3) or 1
            ab0 = ab + rng.randint(-1, 1)
            yield ab, sa, sb, max(0, ab0), math.sqrt(max(1, A0)), math.sqrt(max(1, B0))
        else:
            yield ab, sa, sb, rng.randint(0, 1 << 20), math.sqrt(rng.randint(1, 1 << 27)), math.sqrt(rng.randint(1, 1 << 27))


def test_exact_less_orders_like_the_reference_quotients():
    rng = random.Random(20261017)
    less = ties = 0
    for ab, sa, sb, ab0, sa0, sb0 in _cases(rng, 20000):
        v, v0 = ref_value(ab, sa, sb), ref_value(ab0, sa0, sb0)
        if exact_less(ab, sa, sb, ab0, sa0, sb0):
            assert v <= v0, (ab, sa, sb, ab0, sa0, sb0)
            less += 1
            ties += v == v0
        else:
            assert v >= v0, (ab, sa, sb, ab0, sa0, sb0)
    assert less > 1000 and ties >= 0


@pytest.mark.parametrize("rbits", [1, 2, 3, 4, 5])
def test_estimate_form_recovers_the_dot(rbits):
    """fp32 est = AB * rcp(sa) * rcp(sb) with relative error <= 2^-21 (two
    1-ulp reciprocals, two rounded products) and the low rbits mantissa bits
    cleared: AB = rint(est * sa * sb) for every AB up to the kernel's bound."""
    bound = math.floor(0.5 / (2.0 ** -21 + 2.0 ** (rbits - 23)))
    rng = np.random.default_rng(rbits)
    ab = np.concatenate([np.arange(0, 4096), rng.integers(0, bound + 1, 200000), [bound]]).astype(np.float64)
    A = rng.integers(1, 1 << 40, ab.size).astype(np.float64)
    B = rng.integers(1, 1 << 40, ab.size).astype(np.float64)
    sa, sb = np.sqrt(A), np.sqrt(B)
    f32 = np.float32
    # the worst 1-ulp reciprocal: the correctly rounded one pushed one ulp away
    ra = np.nextafter(f32(1.0) / sa.astype(f32), f32(np.inf) if rbits % 2 else f32(0))
    rb = np.nextafter(f32(1.0) / sb.astype(f32), f32(0) if rbits % 2 else f32(np.inf))
    est = (ab.astype(f32) * ra * rb).astype(f32)
    packed = (est.view(np.uint32) & np.uint32(~((1 << rbits) - 1) & 0xFFFFFFFF)).view(np.float32)
    rec = np.rint(packed.astype(np.float64) * sa * sb)
    assert np.array_equal(rec, ab)
