"""Integer SUM beyond 2^53: the oracle's default (exact 128-bit sum, rounded once — what the device
computes) against the reference's literal arithmetic (oracle literal_int_sum: values added into a
double in doc order per segment, SumAggregationFunction.java:80-92,190-200; segments merged as doubles).
At the bench's per-group scale (SUM of ~2.7M values below 2^40 per group, ~1.5e18, 170x past 2^53) the two
differ by rounding only: |exact - literal| / |literal| <= 1e-12, the north star's double tolerance."""
import numpy as np
import pytest

import oracle
from pinot_amd.segment import INT, LONG, build_segment

TOL = 1e-12


def _segments(n_seg, n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_seg):
        out.append(build_segment(f"lit{i}", {
            "g": (rng.integers(0, 3, n).astype(np.int32), INT, {}),
            "imp": (rng.integers(0, 1 << 40, n).astype(np.int64), LONG, {"dictionary": False}),
            "neg": (rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64), LONG, {"dictionary": False}),
            "c": (rng.integers(0, 1000, n).astype(np.int32), INT, {"dictionary": False}),
        }))
    return out


@pytest.mark.parametrize("query", [
    "SELECT COUNT(*), SUM(imp), SUM(neg), AVG(imp) FROM t WHERE c > 10",
    "SELECT g, COUNT(*), SUM(imp), SUM(neg), AVG(imp) FROM t WHERE c > 10 GROUP BY g",
])
def test_exact_vs_literal_double_sum(query):
    segs = _segments(3, 2_800_000, 7)
    n1, exact = oracle.execute(query, segs)
    n2, literal = oracle.execute(query, segs, literal_int_sum=True)
    assert n1 == n2 and set(exact) == set(literal)
    big = 0
    for k in exact:
        for e, l in zip(exact[k], literal[k]):
            if isinstance(e, tuple):  # AVG (sum, count)
                assert e[1] == l[1]
                e, l = e[0], l[0]
            if isinstance(e, int):
                assert e == l  # COUNT
                continue
            assert abs(e - l) <= TOL * abs(l), (k, e, l)
            big += abs(l) > 2.0 ** 53
    assert big > 0  # the regime past 2^53 is exercised


def test_literal_equals_exact_below_2_53():
    """Below 2^53 every partial sum is exact in double, so both modes agree bit for bit."""
    segs = _segments(2, 200_000, 11)
    q = "SELECT g, SUM(c), AVG(c), COUNT(*) FROM t GROUP BY g"
    assert oracle.execute(q, segs)[1] == oracle.execute(q, segs, literal_int_sum=True)[1]
