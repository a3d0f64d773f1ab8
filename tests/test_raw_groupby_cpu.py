"""GROUP BY on raw (no-dictionary) columns: the oracle's restatement of
NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator
(pinot-core/.../query/aggregation/groupby/NoDictionarySingleColumnGroupKeyGenerator.java:98-143:
one group per distinct value, fastutil key equality) checked against a plain numpy group-by of the
same values. No GPU needed."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle  # noqa: E402
from pinot_amd import segment as S  # noqa: E402


def numpy_groupby(keys, vals, mask):
    out = {}
    for k, v in zip(zip(*[k[mask] for k in keys]), vals[mask]):
        k = tuple(x.item() for x in k)
        c, s, mn = out.get(k, (0, 0, None))
        out[k] = (c + 1, s + int(v), int(v) if mn is None else min(mn, int(v)))
    return out


@pytest.mark.parametrize("t,comp", [(S.INT, S.PASS_THROUGH), (S.LONG, S.LZ4), (S.DOUBLE, S.SNAPPY), (S.FLOAT, S.PASS_THROUGH)])
def test_raw_group_by_matches_value_grouping(t, comp):
    rng = np.random.default_rng(5)
    n = 20_011
    base = rng.integers(-300, 300, n)
    npt = {S.INT: np.int32, S.LONG: np.int64, S.DOUBLE: np.float64, S.FLOAT: np.float32}[t]
    k = (base * (1 << 33)).astype(npt) if t == S.LONG else (base * 0.5).astype(npt) if t in (S.DOUBLE, S.FLOAT) else base.astype(npt)
    d = rng.integers(0, 7, n).astype(np.int32)
    v = rng.integers(0, 1000, n).astype(np.int32)
    bufs = S.build_segment("rg", {"k": (k, t, {"dictionary": False, "compression": comp}), "d": (d, S.INT, {}),
                                  "v": (v, S.INT, {"dictionary": False})})
    for q, keys, mask in [
        ("SELECT k, COUNT(*), SUM(v), MIN(v) FROM t GROUP BY k", [k], np.ones(n, bool)),
        ("SELECT k, d, COUNT(*), SUM(v), MIN(v) FROM t WHERE v < 500 GROUP BY k, d", [k, d], v < 500),
    ]:
        nm, groups = oracle.execute(q, [bufs])
        exp = numpy_groupby(keys, v, mask)
        assert nm == int(mask.sum())
        assert set(groups) == set(exp)
        for key, (c, s, mn) in exp.items():
            g = groups[key]
            assert g[0] == c and g[1] == s and g[2] == mn, (key, g, (c, s, mn))
