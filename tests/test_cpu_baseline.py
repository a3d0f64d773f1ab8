"""bench.py's cpu_baseline leg times oracle.cpu_plan (the oracle's C work for one segment, set up
once). Its matched-doc count must equal oracle.execute's on the same segment and query, and the
timed closure must be re-runnable (the inverted leaves' bitsets are rebuilt each call)."""
import numpy as np
import pytest

import oracle
from helpers import SV_FILTER, random_segment, sv_segment


@pytest.mark.parametrize("use_inverted", [True, False])
@pytest.mark.parametrize("query", [
    "SELECT COUNT(*), SUM(column1), MAX(column3) FROM t" + SV_FILTER,
    "SELECT column11, COUNT(*), SUM(column1) FROM t" + SV_FILTER + " GROUP BY column11",
    "SELECT column6, column7, SUM(column1) FROM t WHERE column17 IN (635553468, 1225000000) GROUP BY column6, column7",
])
def test_cpu_plan_matches_execute(query, use_inverted):
    seg = sv_segment()
    run = oracle.cpu_plan(query, seg, use_inverted)
    exp, _ = oracle.execute(query, [seg], use_inverted)
    assert run() == exp
    assert run() == exp


def test_cpu_plan_inverted_or():
    rng = np.random.default_rng(5)
    seg = random_segment(rng, 50_000, bits_cards=(300, 200, 100), inverted=("d0", "d1", "d2"))
    q = ("SELECT COUNT(*), SUM(r_int) FROM t WHERE d0 IN (3, 10, 17, 24, 500) AND "
         "(d1 IN (3, 52, 101) OR d2 IN (10, 17, 24, 31))")
    exp, _ = oracle.execute(q, [seg])
    run = oracle.cpu_plan(q, seg)
    assert exp > 0 and run() == exp and run() == exp


@pytest.mark.parametrize("info,want", [
    ("jit", "pinot_scan_jit"),
    ("jit-select", "pinot_select+pinot_gather"),
    ("jit-wselect", "pinot_select(word-level)+pinot_gather"),
    ("jit-fwselect", "roaring_select_kernel"),
    ("jit-partitioned+admit-seq", "pinot_admit_seq"),
    ("jit-partitioned+admit", "pinot_first_doc"),
    ("jit-hash-trim", "hash_merge_kernel"),
    ("jit x3", "(3 shape launches)"),
])
def test_bench_kernel_labels(info, want):
    """bench.py names the kernels a plan ran from its kernel_info (round-2 advisor: mislabelled lines)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert want in bench.plan_kernels(info), bench.plan_kernels(info)
