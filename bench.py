"""Benchmark: rows scanned/s + achieved HBM GB/s of a filter + group-by query (BASELINE.json metric).

Default workload (BASELINE.json configs[1], 1B rows in 100 segments per GPU): each rank holds
--segments immutable segments of --rows rows of the AdAnalytics-style table in HBM
(pinot_amd/datagen.py: two fixed-bit dictionary-encoded columns, raw INT/LONG/DOUBLE metrics) and
runs the filter + group-by query pinot_amd.datagen.BENCH_QUERY over all of them. A step is one full
execution of that query over the rank's segments (one batched scan kernel over 1B rows) plus, for
N > 1, the RCCL all-reduce of the dense group tables. Segments are independent, so per-GPU work is
fixed as N grows (weak scaling).

Other workloads (one JSON line per query; not the driver's headline line):
  --workload readme     configs[0]: the README's AdAnalytics query on one 10M-row segment (CPU baseline on
                        one thread: one segment is one Pinot worker's task)
  --workload highcard   configs[3]: GROUP BY two 1000-value dimensions (1M groups), numGroupsLimit raised
                        above the key space (every group kept): partitioned plan
  --workload highcard-default  configs[3]'s query at Pinot's default numGroupsLimit (100000 < 1M groups
                        per segment): exact first-seen trimming per segment (sequential admission pass,
                        then the partitioned plan over the admitted docs)
  --workload wide-keys  5-column GROUP BY past the dense key space: the hash-table plan with its LDS first level
  --workload wide-keys-uniform  the same over uniformly distributed entities (no hot keys)
  --workload inverted   configs[2]: inverted-index IN filters, AND/OR over 3 columns, selectivity sweep
  --workload ssb        configs[4]: SSB SF100 denormalized lineorder, Q1.1-Q4.3

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload readme|scan|highcard|highcard-default|inverted|ssb]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
METRIC = "rows scanned/sec + achieved HBM GB/s, filter+group-by query, 1/2/4/8 GPUs"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workloads():
    """name -> (segment generator, [queries], algorithmic HBM bytes per row, description, distinct segments)."""
    from pinot_amd import datagen, ssb
    return {
        "readme": (datagen.ad_segment, [datagen.README_QUERY], None,
                   "configs[0]: one 10M-row immutable segment of the AdAnalytics table, the reference README's "
                   "example query (8-day range AND IN filter, SUM clicks/impressions GROUP BY daysSinceEpoch)", None),
        "scan": (datagen.ad_segment, [datagen.BENCH_QUERY], datagen.BENCH_BYTES_PER_ROW,
                 "configs[1]: 1B rows in 100 segments per GPU, fixed-bit dict + raw INT/LONG/DOUBLE columns; "
                 "filter+group-by query", None),
        "highcard": (datagen.highcard_segment, [datagen.HIGHCARD_QUERY], datagen.HIGHCARD_BYTES_PER_ROW,
                     "configs[3]: high-cardinality GROUP BY on 2 dims (1M groups), SUM/COUNT/MIN/MAX, "
                     "100 segments x 10M rows per GPU (8B rows on 8 GPUs), RCCL merge of the group tables", None),
        "highcard-default": (datagen.highcard_segment, [datagen.HIGHCARD_DEFAULT_QUERY],
                             datagen.HIGHCARD_BYTES_PER_ROW,
                             "configs[3] at Pinot's default numGroupsLimit (100000): GROUP BY on 2 dims (1M keys), "
                             "each segment admits its first 100000 groups (DictionaryBasedGroupKeyGenerator), "
                             "100 segments x 10M rows per GPU", None),
        "wide-keys": (datagen.widekeys_segment, [datagen.WIDEKEYS_QUERY], datagen.WIDEKEYS_BYTES_PER_ROW,
                      "wide group keys: GROUP BY 5 dictionary columns (key space 4e18 > the 2^28 dense cap: the "
                      "hash-table plan, DictionaryBasedGroupKeyGenerator's map-based holders) over 1B rows in 100 "
                      "segments, ~1M groups of Zipf(1.1)-distributed entities, COUNT / SUM(INT) / MAX(DOUBLE)", None),
        "wide-keys-uniform": (datagen.widekeys_uniform_segment, [datagen.WIDEKEYS_QUERY], datagen.WIDEKEYS_BYTES_PER_ROW,
                              "wide group keys without skew: the wide-keys query over entities uniform over 1M ranks "
                              "(no hot key: every doc misses an on-die first level), 1B rows in 100 segments", None),
        "inverted": (datagen.inverted_segment, [datagen.inverted_query(s) for s in datagen.INVERTED_SELECTIVITIES],
                     None,
                     "configs[2]: inverted-index IN filters combined with AND/OR across 3 columns (10000-value "
                     "dictionaries, RoaringBitmap inverted indexes), selectivity sweep, 1B rows on 1 GPU", 4),
        "ssb": (ssb.lineorder_flat_segment, [sql for _, sql in ssb.SSB_QUERIES], None,
                "configs[4]: Star Schema Benchmark SF100 denormalized lineorder (600M rows per GPU in 60 segments), "
                "Q1.1-Q4.3 filter+group-by", None),
    }


def cpu_baseline(workload: str, query: str, seg_rows: int, seconds: float, threads: int, cache: dict):
    """Time the CPU oracle (scalar C restatement of the reference path) on the host cores: `threads`
    segments of the same workload, each with its query set up once (oracle.cpu_plan: predicates
    resolved, buffers laid out), run concurrently one per thread (the C calls release the GIL), round
    after round until `seconds` of wall time have passed — the shape of Pinot's server executing one
    segment per worker thread. Timed: inverted-index expansion + filter + aggregation / group-by."""
    import concurrent.futures as cf
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    gen, _, _, _, distinct = workloads()[workload]
    ndistinct = threads if distinct is None else min(threads, distinct)
    if "bufs" not in cache:  # host segments shared by every query of the workload
        cache["bufs"] = [gen(f"cpu{k}", seg_rows, seed=10_000 + k) for k in range(ndistinct)]
    bufs = cache["bufs"]
    runs = [oracle.cpu_plan(query, bufs[k % len(bufs)]) for k in range(threads)]
    rows = 0
    rounds = 0
    with cf.ThreadPoolExecutor(max_workers=threads) as pool:
        t0 = time.perf_counter()
        while rounds == 0 or time.perf_counter() - t0 < seconds:
            list(pool.map(lambda r: r(), runs))
            rows += threads * seg_rows
            rounds += 1
        wall = time.perf_counter() - t0
    del runs
    return {"value": rows / wall, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"{rounds} rounds x {threads} segments x {seg_rows} rows of the same table and query "
                      f"({ndistinct} distinct segments), one segment per thread, oracle/pinot_oracle.c (scalar C "
                      f"restatement of the reference Java path: inverted-index expansion, filter, aggregation / "
                      f"group-by), {wall:.1f} s wall"}


# kernels of each device plan (pinot_amd_result_kernel_info), dominant one first
PLAN_KERNELS = {
    "jit": "pinot_scan_jit",
    "jit-select": "pinot_select+pinot_gather",
    "jit-wselect": "pinot_select(word-level)+pinot_gather",
    "jit-fwselect": "roaring_select_kernel (inverted-index expansion + word-level select, one launch)+pinot_gather",
    "jit-partitioned": "pinot_part_scatter+pinot_part_agg (+pinot_part_count, or the direct-atomic pinot_scan_jit on handover)",
    "jit-hash": "pinot_scan_jit (LDS-privatised first level + HBM hash table)",
    "jit-hash-trim": "pinot_scan_jit (HBM hash table keyed by segment) + trim_* + hash_merge_kernel",
    "jit-hash+nolds": "pinot_scan_jit (no LDS level: every matching doc spilled to its block's region) + "
                      "spill_scatter_sorted_kernel + spill_agg_kernel",
    "jit-hash+direct": "pinot_scan_jit (no LDS level: records placed straight into their key-hash partitions) + "
                       "spill_agg_kernel",
}


def plan_kernels(info: str) -> str:
    base = info.split(" ")[0]
    admit = "+admit-seq" if "+admit-seq" in base else "+admit" if "+admit" in base else ""
    base = base.replace(admit, "")
    k = PLAN_KERNELS.get(base)
    if k is None:
        k = PLAN_KERNELS.get(base.replace("-fwselect", "").replace("-wselect", "").replace("-select", ""), base)
        k += " via " + PLAN_KERNELS["jit-fwselect" if base.endswith("-fwselect") else
                                    "jit-wselect" if base.endswith("-wselect") else "jit-select"]
    if admit == "+admit-seq":
        k += " + numGroupsLimit admission (pinot_admit_seq: one block per segment prefix, seen keys in LDS)"
    elif admit:
        k += (" + numGroupsLimit admission (pinot_first_doc over segment prefixes, admit_hist_kernel, trim_select, "
              "admit_bucket_kernel, trim_cutoff, admit_bits_kernel)")
    if " x" in info:
        k += f" ({info.split(' x')[1]} shape launches)"
    return k


def query_sha1(query: str) -> str:
    return hashlib.sha1(query.encode()).hexdigest()


def committed_traffic(query: str, kernel_info: str, rows: int):
    """HBM traffic per execution from the latest committed rocprofv3 PMC pass of this exact query (matched by
    the SHA-1 of its full text) on this exact device plan (pinot_amd_result_kernel_info): FETCH_SIZE x 2 (the
    gfx950 correction of MI355X_MICROARCH.md) + WRITE_SIZE, per row of the profiled run, scaled to `rows`.
    A record of another plan (a planner change since the pass) is not used: traffic is then None."""
    sha = query_sha1(query)
    for rnd in ("r06", "r05", "r04", "r03"):
        pmc = os.path.join(ROOT, "profiles", rnd, "pmc_index.json")
        if not os.path.exists(pmc):
            continue
        for key, d in json.load(open(pmc)).items():
            if not d.get("rows") or (d.get("query_sha1") or (query_sha1(d["query"]) if "query" in d else None)) != sha:
                continue
            if d.get("scan_kernel") != kernel_info:  # unrecorded plan (round 3 records): not evidence
                continue
            t = (d["hbm_read_bytes"] + d["hbm_write_bytes"]) / d["rows"] * rows
            src = (f"profiles/{rnd}/pmc_index.json[{key}] (rocprofv3 --pmc FETCH_SIZE x2, WRITE_SIZE per execution of "
                   f"this query on plan {d.get('scan_kernel', '?')} over {d['rows']:.0f} rows, commit "
                   f"{d.get('commit', '?')}, scaled per row; ROUND={rnd} profiles/profile.sh)")
            return t, src
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", default="scan", choices=["readme", "scan", "highcard", "highcard-default", "wide-keys", "wide-keys-uniform",
                                                           "inverted", "ssb"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--segments", type=int, default=None, help="segments per GPU (default 100; ssb: 60 = SF100)")
    ap.add_argument("--rows", type=int, default=10_000_000, help="rows per segment")
    ap.add_argument("--cpu-seconds", type=float, default=None,
                    help="CPU baseline wall time per query (default 12 s; 4 s per query for multi-query workloads)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads for the CPU baseline (the GPU box's CPU share per GPU is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify one segment against the oracle")
    ap.add_argument("--query-index", type=int, default=None, help="run only this query of the workload")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not under a launcher: start one rank per GPU as child processes (torchrun) before anything
        # touches the GPU, and exit with the launcher's status
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        log(f"spawning {args.gpus} ranks: {' '.join(cmd)}")
        import subprocess
        sys.exit(subprocess.call(cmd))

    import torch
    import torch.distributed as dist
    from pinot_amd import dist as pdist, engine
    from pinot_amd.query import parse_sql
    gen, queries, bytes_per_row, workload_desc, distinct = workloads()[args.workload]
    if args.query_index is not None:
        queries = [queries[args.query_index]]
    if args.segments is None:
        args.segments = {"ssb": 60, "readme": 1}.get(args.workload, 100)
    if args.workload == "readme":  # a single segment: one Pinot worker thread
        args.cpu_threads = min(args.cpu_threads, args.segments)
    if args.cpu_seconds is None:
        args.cpu_seconds = 12.0 if len(queries) == 1 else 4.0
    cpu_cache: dict = {}

    rank, world, local = pdist.init_distributed()
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE {world}")
        sys.exit(2)
    torch.cuda.set_device(local)
    if world > 1:
        if dist.get_world_size() != args.gpus:
            log(f"error: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
            sys.exit(2)
        if local >= torch.cuda.device_count():
            log(f"error: local rank {local} but only {torch.cuda.device_count()} visible GPUs")
            sys.exit(2)

    # ---- stage this rank's segments into HBM ----
    t0 = time.time()
    segs = []
    host_bufs = []
    for i in range(args.segments):
        if distinct is None or i < distinct:
            bufs = gen(f"{args.workload}_{rank}_{i}", args.rows, seed=rank * 100_003 + i)
            if distinct is not None:
                host_bufs.append(bufs)
        else:  # slow-to-build workloads: further segments are HBM copies of the first `distinct`
            bufs = host_bufs[i % distinct]
        segs.append(engine.ImmutableSegment(bufs))
        if i % 20 == 19:
            log(f"[rank {rank}] staged {i + 1}/{args.segments} segments ({time.time() - t0:.0f}s)")
    hbm = sum(s.device_bytes() for s in segs)
    log(f"[rank {rank}] {args.segments} segments, {hbm / 1e9:.1f} GB in HBM, staged in {time.time() - t0:.0f}s")
    data = "synthetic (device-generated segments in Pinot's on-disk formats)"
    if distinct is not None:
        data += f"; {distinct} distinct segments, each staged {args.segments // distinct}x"

    stream = torch.cuda.current_stream()
    ex = engine.ServerQueryExecutor()
    rows_per_rank = args.segments * args.rows
    outs = []
    for query in queries:
        # cold query latency: host planning + predicate resolution + hipRTC compile (first time this
        # shape is seen in the process) + first launch + result fetch; then the same with the
        # compiled kernel cached (a repeated query shape on a server)
        torch.cuda.synchronize()
        t_c = time.perf_counter()
        # every rank plans over the union of all ranks' group key values (one all-gather), so the dense
        # tables index the same groups and merge in place
        ks = pdist.global_key_space(segs, pdist.key_columns(parse_sql(query))) if world > 1 else None
        res = ex.execute(query, segs, stream=stream, key_space=ks)
        res.groups()
        torch.cuda.synchronize()
        cold_ms = (time.perf_counter() - t_c) * 1e3
        # the same query planned again while the first result is alive (compiled kernels cached, host planning
        # redone): the plan of a concurrent identical query
        t_c = time.perf_counter()
        res_b = ex.execute(query, segs, stream=stream, key_space=ks)
        res_b.groups()
        torch.cuda.synchronize()
        fresh_plan_ms = (time.perf_counter() - t_c) * 1e3
        res_b.destroy()  # idle: kept by the library's prepared-plan cache
        # a re-issued query (the earlier one finished): the prepared plan of its identity runs without planning.
        # Issued 5 times (once when the group conversion alone is slow, e.g. ~1M groups): the median is reported,
        # the spread beside it (a single sample caught host outliers: one SSB query at 2.5 ms for a 1.0-ms median)
        samples = []
        for _ in range(5 if cold_ms < 200 and world == 1 else 1):  # (the same count on every rank)
            t_c = time.perf_counter()
            res2 = ex.execute(query, segs, stream=stream, key_space=ks)
            torch.cuda.synchronize()
            t_f = time.perf_counter()
            arrays = res2.fetch_arrays() if hasattr(res2, "fetch_arrays") else None
            t_g = time.perf_counter()
            if arrays is not None:  # Python conversion of the arrays already fetched (no second fetch)
                res2.groups(arrays=arrays)
            else:
                res2.groups()
            t_e = time.perf_counter()
            samples.append({  # the re-issued query's host time: library execute (plan-cache lookup + launch),
                "total_ms": (t_e - t_c) * 1e3,  # library fetch (device compaction + copy of the groups), conversion
                "execute_ms": (t_f - t_c) * 1e3,
                "fetch_ms": (t_g - t_f) * 1e3 if arrays is not None else None,
                "python_groups_ms": (t_e - t_g) * 1e3,
                "plan_phases_ms": res2.plan_timing() if hasattr(res2, "plan_timing") else None,
            })
            del arrays
            res2.destroy()
        med = sorted(samples, key=lambda x: x["total_ms"])[len(samples) // 2]
        plan_ms = med["total_ms"]
        host_ms = {k: v for k, v in med.items() if k != "total_ms"}
        host_ms["fresh_plan_ms"] = fresh_plan_ms
        host_ms["reissued_ms_samples"] = [round(x["total_ms"], 3) for x in samples]
        scratch = None

        # device time of each step's plan: HIP events recorded on the plan's own stream around the execution
        # (no host sync inside the timed loop; read after it)
        ev_pairs = []
        merge_ev = []  # (N > 1) HIP events around each timed step's merge on the same stream

        def step(timed=False):
            nonlocal scratch
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            res.execute_again(stream)
            if timed:
                e1.record(stream)
                ev_pairs.append((e0, e1))
            if world > 1:
                scratch = pdist.merge_result(res, scratch, stream=stream)
                if timed:
                    e2 = torch.cuda.Event(enable_timing=True)
                    e2.record(stream)
                    merge_ev.append((e1, e2))

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()

        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(timed=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())

        total_rows = rows_per_rank * world * args.steps
        value = total_rows / elapsed
        merge = None
        if world > 1:
            # the cross-rank merge alone (the broker reduce's share of a step): HIP events around it inside the
            # timed steps, and, untimed afterwards, a few merges bracketed by device synchronisation (wall
            # clock, max over ranks) -- so a poor scaling curve says whether the scan or the merge is to blame
            ms_ev = sum(a.elapsed_time(b) for a, b in merge_ev) / max(len(merge_ev), 1)
            walls = []
            for _ in range(3):
                res.execute_again(stream)  # a fresh, unmerged table each time (a merge is not idempotent)
                torch.cuda.synchronize()
                dist.barrier()
                t_m = time.perf_counter()
                scratch = pdist.merge_result(res, scratch, stream=stream)
                torch.cuda.synchronize()
                walls.append(time.perf_counter() - t_m)
            w = torch.tensor([sum(walls) / len(walls)], dtype=torch.float64,
                             device="cuda" if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(w, op=dist.ReduceOp.MAX)
            st = (scratch or {}).get("stats", {}) if isinstance(scratch, dict) else {}
            merge = {"path": st.get("path"), "bytes_per_rank": st.get("bytes"), "ms_events": ms_ev,
                     "ms_wall_synchronized": float(w.item()) * 1e3, "backend": dist.get_backend(),
                     "source": "ms_events: HIP events on the step's stream around pdist.merge_result in the timed "
                               "steps; ms_wall_synchronized: 3 untimed merges between device synchronisations, "
                               "mean per rank, max over ranks"}
        kernel_ms = [a.elapsed_time(b) for a, b in ev_pairs]
        lib_kernel_ms = res.last_kernel_ms()  # the library's own events around the last execution (cross-check)
        avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
        # algorithmic bytes per execution, from the plan (pinot_amd_result_algorithmic_bytes): each
        # decoded column once at its stored width; under an inverted-index gate only the rows that
        # pass it, plus the selected bitmaps and the dense bitset written + read once
        alg_bytes = res.algorithmic_bytes()
        bpr = alg_bytes / rows_per_rank
        # the workload's own count of the query's column bytes (datagen); the roofline uses the plan's
        # figure, and a disagreement is reported on the line, not hidden in the log
        bpr_mismatch = None
        if bytes_per_row is not None and abs(alg_bytes - rows_per_rank * bytes_per_row) > 1e-6 * alg_bytes:
            bpr_mismatch = {"plan_bytes_per_row": bpr, "workload_bytes_per_row": bytes_per_row}
            log(f"warning: plan's algorithmic bytes {bpr:.4f} B/row != {bytes_per_row:.4f}")
        achieved = alg_bytes / avg_kernel_s / 1e9

        groups = res.groups()
        matched = res.num_docs_matched()
        if world > 1:
            m = torch.tensor([matched], dtype=torch.int64, device="cuda")
            dist.all_reduce(m)
            matched_all = int(m.item())
        else:
            matched_all = matched
        qc = parse_sql(query)
        # size-independent property: the merged group COUNTs add up to the docs that passed the filter
        # (diagnostic knobs that deliberately break results skip it; their lines say so in config)
        diag = sorted(k for k in os.environ if k.startswith("PINOT_AMD_DIAG_"))
        counts_first = bool(qc.aggregations) and qc.aggregations[0].func == "COUNT" and not diag
        if qc.group_by and counts_first:
            # numGroupsLimit trimming drops the docs of groups a segment did not admit (they were scanned)
            total = sum(p[0] for p in groups.values())
            if res.num_groups_limit_reached():
                assert total <= matched_all, "sum of group COUNTs > matched docs"
            else:
                assert total == matched_all, "sum of group COUNTs != matched docs"
        elif world == 1 and counts_first:
            assert groups[()][0] == matched, "COUNT(*) != matched docs"

        if args.check and rank == 0:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle
            one = gen("check", min(args.rows, 2_000_000), seed=424242)
            r1 = ex.execute(query, [engine.ImmutableSegment(one)]).groups()
            _, o1 = oracle.execute(query, [one])
            assert set(r1) == set(o1), "group keys differ"
            for k in o1:
                for i, a in enumerate(qc.aggregations):
                    g, e = r1[k][i], o1[k][i]
                    if a.func == "SUM" and isinstance(e, float) and e != int(e):
                        assert abs(g - e) <= 1e-12 * abs(e), (k, a.name, g, e)
                    else:
                        assert g == e, (k, a.name, g, e)
            log("[check] HIP result == oracle on a 2M-row segment")

        traffic, traffic_src = committed_traffic(query, res.kernel_info(), rows_per_rank)

        if rank == 0:
            cpu = None
            if not args.no_cpu_baseline and world == 1:
                log("[rank 0] timing the CPU baseline ...")
                cpu = cpu_baseline(args.workload, query, min(args.rows, 10_000_000), args.cpu_seconds,
                                   max(1, min(args.cpu_threads, os.cpu_count() or 1)), cpu_cache)
            out = {
                "metric": METRIC,
                "value": value,
                "unit": "rows/s",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": elapsed / args.steps * 1e3,
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": "int32/int64/f64",
                "data": data,
                "config": {
                    "workload": workload_desc,
                    "query": query if len(query) < 400 else query[:200] + " ... " + query[-120:],
                    "query_sha1": query_sha1(query),
                    "segments_per_gpu": args.segments,
                    "rows_per_segment": args.rows,
                    "rows_per_gpu": rows_per_rank,
                    "selectivity": matched / rows_per_rank,
                    "groups": len(groups),
                    "parallelism": f"segments sharded over {world} GPU(s), RCCL all-reduce merge" if world > 1
                                   else "1 GPU",
                    "hbm_bytes_per_gpu": hbm,
                    "scan_kernel": res.kernel_info(),
                    "diagnostic_knobs": diag or None,
                },
                "cold_ms": cold_ms,
                "cached_plan_ms": plan_ms,
                "cached_plan_breakdown": host_ms,
                "roofline": {
                    "bound": "hbm",
                    "achieved": achieved,
                    "peak": HBM_PEAK_GBS,
                    "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS,
                    "traffic": traffic,
                    "traffic_source": traffic_src,
                    "kernel": plan_kernels(res.kernel_info()),
                    "kernel_ms": avg_kernel_s * 1e3,
                    "kernel_ms_source": "mean of HIP events recorded on the plan's stream around each timed execution",
                    "library_last_kernel_ms": lib_kernel_ms,
                    "bytes_per_row": bpr,
                    "bytes_per_row_mismatch": bpr_mismatch,
                },
                "cpu_baseline": cpu,
            }
            if merge is not None:
                out["merge"] = merge
            print(json.dumps(out), flush=True)
            outs.append(out)
        res.destroy()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return outs[0] if len(outs) == 1 else outs


if __name__ == "__main__":
    main()
