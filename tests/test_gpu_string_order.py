"""STRING dictionaries in Java String.compareTo order (UTF-16 code units) on the device path: values mixing
ASCII, BMP characters above U+E000 and supplementary characters (surrogate pairs in UTF-16, 4-byte UTF-8),
where UTF-8 byte order and UTF-16 order disagree. Two segments with different dictionaries (the merged
key space sorts their union), GROUP BY and range predicates on the column, against the oracle (which sorts
by UTF-16 code units itself), and the server table ordered by the key."""
import numpy as np
import pytest

import oracle
from oracle_reduce import server_table
from pinot_amd.query import parse_sql
from pinot_amd.segment import INT, STRING, build_segment

pytestmark = pytest.mark.gpu

VALUES = ["a", "b", "é", "", "x", "￯", "\U0001f600", "\U0001f600a", "\U00010000", "z\U0001f600",
          "z", "zz", "", "A"]


def _segments():
    rng = np.random.default_rng(5)
    out = []
    for i in range(2):
        vals = VALUES[i::2] + VALUES[: 3 + 4 * i]  # different dictionaries per segment
        n = 5000 + 777 * i
        s = np.array([vals[j] for j in rng.integers(0, len(vals), n)], dtype=object)
        out.append(build_segment(f"str{i}", {
            "s": (s, STRING, {}),
            "m": (rng.integers(0, 1000, n).astype(np.int32), INT, {"dictionary": False}),
        }))
    return out


@pytest.mark.parametrize("q", [
    "SELECT s, COUNT(*), SUM(m) FROM t GROUP BY s",
    "SELECT s, COUNT(*) FROM t WHERE s > '' GROUP BY s",
    "SELECT s, COUNT(*) FROM t WHERE s BETWEEN 'b' AND '\U0001f600' GROUP BY s",
    "SELECT s, COUNT(*) FROM t WHERE s < '￯' GROUP BY s",
])
def test_string_java_order_vs_oracle(q):
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    bufs = _segments()
    segs = [E.ImmutableSegment(b) for b in bufs]
    got = E.ServerQueryExecutor().execute(q, segs).groups()
    _, exp = oracle.execute(q, bufs)
    assert got == exp


def test_string_key_order_in_server_table():
    import torch
    assert torch.cuda.is_available()
    from pinot_amd import engine as E
    bufs = _segments()
    segs = [E.ImmutableSegment(b) for b in bufs]
    q = "SELECT s, COUNT(*) FROM t GROUP BY s ORDER BY s DESC LIMIT 6"
    got = E.ServerQueryExecutor(server_trim=True).execute(q, segs).groups()
    _, full = oracle.execute(q, bufs)
    exp = server_table(oracle.parse_sql(q), full)
    assert list(got) == list(exp) and got == exp
