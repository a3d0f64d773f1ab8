"""Diagnostic: the partitioned plan of tests/test_gpu_trim.py::test_int_sums_narrow_lds_partials (3 segments of
~120K rows, GROUP BY a, b over a 490K-key space, 16-byte records) executed many times against the oracle; prints
per execution the keys missing / extra / with wrong values. Usage:
  python scripts/repro_part_race.py [REPS] [ENV=VALUE ...]   (knobs read at plan time; PINOT_AMD_POOL_BYTES is read
  once per process, so set it in the process environment)"""
import os
import sys

import numpy as np

_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for _p in (_ROOT, os.path.join(_ROOT, "oracle"), os.path.join(_ROOT, "tests")):
    sys.path.insert(0, _p)

import oracle  # noqa: E402
from pinot_amd import segment as S  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    from pinot_amd import engine as E
    os.environ.setdefault("PINOT_AMD_NARROW_SUMS", "1")
    rng = np.random.default_rng(31)
    bufs = []
    for i in range(3):
        n = 120_000 + 17 * i
        iv = rng.choice(np.array([-(1 << 31), (1 << 31) - 1, 0, 5], dtype=np.int64), n).astype(np.int32)
        cols = {
            "g": (rng.integers(0, 50, n).astype(np.int32), S.INT, {}),
            "a": (rng.integers(0, 700, n).astype(np.int32), S.INT, {}),
            "b": (rng.integers(0, 700, n).astype(np.int32), S.INT, {}),
            "i": (iv, S.INT, {"dictionary": False}),
            "l44": (rng.integers((1 << 44) - 1000, 1 << 44, n, dtype=np.int64), S.LONG, {"dictionary": False}),
            "l60": (rng.integers(-(1 << 60), 1 << 60, n, dtype=np.int64), S.LONG, {"dictionary": False}),
            "dl": (rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64) // 4096 * 4096, S.LONG, {}),
        }
        bufs.append(S.build_segment(f"nw{i}", cols))
    segs = [E.ImmutableSegment(b) for b in bufs]
    q = ("SET numGroupsLimit = 1000000; SELECT a, b, COUNT(*), SUM(i), SUM(l44), SUM(l60) FROM t WHERE g < 40 "
         "GROUP BY a, b")
    _, og = oracle.execute(q, bufs)
    bad = 0
    for it in range(reps):
        res = E.ServerQueryExecutor().execute(q, segs)
        for again in range(3):
            if again:
                res.execute_again()
            got = res.groups()
            miss = [k for k in og if k not in got]
            extra = [k for k in got if k not in og]
            wrong = [k for k in og if k in got and got[k] != og[k]]
            ok = not (miss or extra or wrong)
            bad += not ok
            if not ok or (it == 0 and again == 0):
                print(f"rep {it}.{again} {res.kernel_info()} matched {res.num_docs_matched()} groups {len(got)}/{len(og)}"
                      f" missing {len(miss)} extra {len(extra)} wrong {len(wrong)} e.g. miss {miss[:3]} extra "
                      f"{[(k, (k[0] + 700 * k[1]) if len(k) == 2 else None) for k in extra[:3]]} wrong "
                      f"{[(k, got[k], og[k]) for k in wrong[:2]]}", flush=True)
        if it == 0:
            print("plan", {k: v for k, v in res.plan_timing().items() if not isinstance(v, dict)}, flush=True)
    print(f"SUMMARY env={sys.argv[2:]} pool={os.environ.get('PINOT_AMD_POOL_BYTES')} bad {bad}/{3 * reps}", flush=True)


if __name__ == "__main__":
    main()
