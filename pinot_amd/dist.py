"""One process per GPU: segment sharding and the cross-GPU merge of group-by results.

Pinot combines per-segment results on a server (GroupByCombineOperator) and then across servers
in the broker (BrokerReduceService). Here every GPU executes its shard of segments into a dense
accumulator table over the query's merged key space (accumulation across its own segments happens
in-kernel), and the tables of all GPUs are merged in place with RCCL all-reduces over xGMI:
SUM/COUNT as int64 or fp64 sums, MIN/MAX as min/max of an order-preserving int64 encoding of the
double value. Small tables go through one all-gather reduced locally; no other data-path collective.
Results without a shared dense table (hash-table plans, numGroupsLimit trimming, DISTINCTCOUNT) merge
by value on the device, partitioned by key: every rank's compacted (key words, accumulator words) rows go
to the rank that owns their key hash (one all-to-all), each rank folds its 1/N share into a device hash
table (the library's merge), and the merged shares -- disjoint -- are all-gathered so every rank ends up
with the final groups (or only rank `root` receives them).

Every rank plans the query over the same group key space: ``global_key_space`` all-gathers each
rank's group-by column values and the union is installed on every rank
(``pinot_amd_query_set_group_key_values``), so dense tables index identical groups whatever each
rank's own dictionaries hold, and the by-value rows of every rank pack their keys identically.
"""
from __future__ import annotations

import hashlib
import os
from typing import List, Sequence

OP_SUM_I64, OP_SUM_F64, OP_MIN, OP_MAX, OP_SUM_I128, OP_HI = 0, 1, 2, 3, 4, 5
SIGN = -(1 << 63)  # 0x8000000000000000 as int64
MASK32 = 0xFFFFFFFF


def init_distributed():
    """torch.distributed from the launcher env (torchrun); returns (rank, world, local_rank)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        # rehearsal of the N-rank path on a one-GPU box: every rank on device 0, collectives over gloo
        # (RCCL needs a device per rank)
        backend = os.environ.get("PINOT_AMD_DIST_BACKEND", backend)
        if os.environ.get("PINOT_AMD_DIST_ONE_DEVICE") == "1":
            local = 0
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def shard(items: Sequence, rank: int, world: int) -> list:
    """Round-robin segment assignment (segments are independent units of work)."""
    return [x for i, x in enumerate(items) if i % world == rank]


def _limbs(lo, hi):
    """A 128-bit two's-complement (hi:lo) as four 32-bit limbs in int64 (the top one signed): summing
    them across up to 2^31 ranks cannot overflow, so an int64 all-reduce carries the exact sum."""
    import torch
    l0 = lo & MASK32
    l1 = (lo >> 32) & MASK32
    l2 = hi & MASK32
    l3 = hi >> 32
    return torch.stack([l0, l1, l2, l3])


def _from_limbs(l):
    """Carry-propagate summed limbs back into (lo, hi) int64 words."""
    c = l[0] >> 32
    w0 = l[0] & MASK32
    v1 = l[1] + c
    w1 = v1 & MASK32
    v2 = l[2] + (v1 >> 32)
    w2 = v2 & MASK32
    v3 = l[3] + (v2 >> 32)
    lo = w0 | (w1 << 32)
    hi = w2 | (v3 << 32)
    return lo, hi


def _reduce_gathered(g, ops):
    """[world, len(ops), num_keys] gathered tables -> the merged [len(ops), num_keys] table (the same
    reductions merge_tables' all-reduces perform)."""
    import torch
    out = g[0].clone()
    for i, op in enumerate(ops):
        if op == OP_SUM_I64:
            out[i] = g[:, i].sum(0)
        elif op == OP_SUM_F64:
            out[i] = g[:, i].contiguous().view(torch.float64).sum(0).view(torch.int64)
        elif op == OP_SUM_I128:
            lo, hi = _from_limbs(_limbs(g[:, i], g[:, i + 1]).sum(1))
            out[i] = lo
            out[i + 1] = hi
        elif op in (OP_MIN, OP_MAX):
            s_ = g[:, i] ^ SIGN
            out[i] = (s_.amin(0) if op == OP_MIN else s_.amax(0)) ^ SIGN
    return out


def merge_tables(table, ops: Sequence[int], num_keys: int, group=None, gather_max_bytes: int = 1 << 20,
                 check=None) -> int:
    """In-place merge across ranks of a [len(ops), num_keys] int64 tensor of accumulator words.

    ops per row: 0 = int64 sum, 1 = fp64 sum (words are double bits), 2/3 = min/max of the
    library's ordered-uint64 encoding (flipping the sign bit makes it an order-preserving int64),
    4/5 = low/high word of an exact 128-bit integer sum (reduced as 32-bit limbs).

    Tables up to gather_max_bytes: ONE all-gather of the whole table, reduced locally per row kind
    (a latency-bound exchange: one collective instead of one per reduction kind). Larger tables: one
    all-reduce per reduction kind (integer sums incl. the limbs of 128-bit rows in one int64 SUM, double
    sums in one fp64 SUM, one MIN, one MAX), each moving ~2x the table per rank on a ring.
    `check`: None, or a 1-element int64 tensor (the result's self-check word, engine.QueryResult.check_word)
    merged in the same collectives (max / sum, both nonzero iff some rank's is): a rank whose execution
    failed its self-check then voids every rank's merged table, with no extra collective and no host read.
    Returns the bytes this rank put into the collectives."""
    import torch
    import torch.distributed as dist
    t = table.view(len(ops), num_keys)
    ops = list(ops)
    world = dist.get_world_size(group)
    if world == 1:
        return 0
    if t.numel() * 8 <= gather_max_bytes:
        src = t.contiguous() if check is None else torch.cat([t.reshape(-1), check.reshape(1)])
        parts = [torch.empty_like(src) for _ in range(world)]
        dist.all_gather(parts, src, group=group)
        g = torch.stack(parts)
        if check is not None:
            check.copy_(g[:, -1].max().reshape(check.shape))
            g = g[:, :-1].reshape(world, len(ops), num_keys)
        t.copy_(_reduce_gathered(g, ops))
        return src.numel() * 8
    nbytes = 0
    i64 = [i for i, op in enumerate(ops) if op == OP_SUM_I64]
    i128 = [i for i, op in enumerate(ops) if op == OP_SUM_I128]
    f64 = [i for i, op in enumerate(ops) if op == OP_SUM_F64]
    parts = [t[i64]] if i64 else []
    parts += [_limbs(t[i], t[i + 1]) for i in i128]
    if parts or check is not None:
        rows = torch.cat(parts) if parts else t.new_empty((0, num_keys))
        # the self-check word rides the integer sum as one extra element: summed, it is nonzero iff some rank's is
        buf = rows.reshape(-1) if check is None else torch.cat([rows.reshape(-1), check.reshape(1)])
        nbytes += buf.numel() * 8
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        if check is not None:
            check.copy_(buf[-1:].reshape(check.shape))
        buf = buf[:rows.numel()].view(rows.shape)
        if i64:
            t[i64] = buf[:len(i64)]
        for j, i in enumerate(i128):
            lo, hi = _from_limbs(buf[len(i64) + 4 * j: len(i64) + 4 * j + 4])
            t[i] = lo
            t[i + 1] = hi
    if f64:
        f = t[f64].contiguous().view(torch.float64)
        nbytes += f.numel() * 8
        dist.all_reduce(f, op=dist.ReduceOp.SUM, group=group)
        t[f64] = f.view(torch.int64)
    for op, rop in ((OP_MIN, dist.ReduceOp.MIN), (OP_MAX, dist.ReduceOp.MAX)):
        rows = [i for i, o in enumerate(ops) if o == op]
        if rows:
            s_ = (t[rows] ^ SIGN).contiguous()
            nbytes += s_.numel() * 8
            dist.all_reduce(s_, op=rop, group=group)
            t[rows] = s_ ^ SIGN
    return nbytes


class _DeviceWords:
    """A library-owned HBM array seen by torch without a copy (__cuda_array_interface__)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False), "version": 2,
                                         "strides": None}


def merge_result(result, scratch=None, group=None, stream=None, gather_max_bytes: int = 1 << 20, root=None):
    """Merge a query result across ranks; afterwards every rank's result holds the merged groups (with
    `root` set, only that rank's; the others hold their key-partitioned share).

    The ranks first agree on HOW (one all-reduce of two flags: "some rank needs a merge by value" and
    numGroupsLimitReached, which the broker ORs over servers): when every rank's result keeps its groups in
    a dense accumulator table (identical key space via global_key_space) the tables are merged in place
    (merge_tables on a zero-copy torch view of the library's HBM table); when any rank ran a hash-table
    plan (large key spaces, numGroupsLimit trimming) or the query has DISTINCTCOUNT, grouped parts merge BY
    VALUE on the device, partitioned by key (merge_by_value); aggregation-only parts (DISTINCTCOUNT's base
    query without GROUP BY) still merge in place. A rank never decides alone, so ranks whose plans differ
    still run the same collectives.

    `stream`: the stream the result was executed on; torch's current stream waits for it first.
    `scratch`: None, or the dict an earlier merge_result of the SAME result object returned. The agreement
    (the flag all-reduce and its host read) is a property of the plan, which re-executions over the same
    immutable segments do not change: with the scratch of an earlier merge of this result the ranks skip it,
    so a dense merge enqueues its collectives without a host synchronisation. scratch["stats"] describes the
    last merge: its path ("dense-gather" / "dense-allreduce" / "by-value") and the bytes this rank put into
    the collectives."""
    import torch
    import torch.distributed as dist
    cur = torch.cuda.current_stream() if torch.cuda.is_available() else None
    if stream is not None and cur is not None:
        handle = int(getattr(stream, "cuda_stream", stream))
        if handle != cur.cuda_stream:
            ext = stream if isinstance(stream, torch.cuda.Stream) else torch.cuda.ExternalStream(handle)
            cur.wait_stream(ext)
    parts = result.results() if hasattr(result, "results") else [result]
    world = dist.get_world_size(group)
    if world == 1:
        return scratch
    if not isinstance(scratch, dict) or scratch.get("result") is not result:
        # DISTINCTCOUNT folds (group key, value) groups whose value column is not in the dense key space
        local_by_value = hasattr(result, "results") or any(not p.has_dense_table() for p in parts)
        reached = any(_limit_reached(p) for p in parts)
        dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
        flag = torch.tensor([1 if local_by_value else 0, 1 if reached else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        by_value, reached_any = (bool(x) for x in flag.tolist())
        scratch = {"result": result, "by_value": by_value, "reached": reached_any}
    by_value, reached_any = scratch["by_value"], scratch["reached"]
    if by_value:
        # the merge by value reads each rank's groups, and a result whose self-check failed refuses them: the ranks
        # agree first, so every rank fails together instead of some waiting in a collective for a rank that raised
        bad = any(p.self_check_failed() for p in parts if hasattr(p, "self_check_failed"))
        flag = torch.tensor([1 if bad else 0], dtype=torch.int64,
                            device="cuda" if dist.get_backend(group) == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag.item()):
            raise RuntimeError("merge_result: a rank's execution failed its partitioned self-check; the merged "
                               "result would be void on every rank")
    stats = {"path": None, "bytes": 0}
    for p in parts:
        if hasattr(p, "set_merged_limit_reached"):
            p.set_merged_limit_reached(reached_any)
        if by_value and _grouped(p):
            stats["path"] = "by-value"
            stats["bytes"] += merge_by_value(p, group, cur, root)
            continue
        ops, nk, ptrs = p.accumulators()
        if not ops:
            continue
        table = torch.as_tensor(_DeviceWords(ptrs[0], len(ops) * nk), device="cuda")
        assert table.data_ptr() == ptrs[0], "zero-copy view of the accumulator table failed"
        chk = torch.as_tensor(_DeviceWords(p.check_word(), 1), device="cuda") if hasattr(p, "check_word") else None
        stats["bytes"] += merge_tables(table, ops, nk, group, gather_max_bytes, check=chk)
        stats["path"] = stats["path"] or ("dense-gather" if len(ops) * nk * 8 <= gather_max_bytes else "dense-allreduce")
    scratch["stats"] = stats
    return scratch


def _grouped(p) -> bool:
    qc = getattr(p, "qc", None)
    return True if qc is None else bool(qc.group_by)


def _limit_reached(p) -> bool:
    f = getattr(p, "num_groups_limit_reached", None)
    return bool(f()) if f is not None else False


def key_owner(keys, world: int):
    """Rank owning each row's group: a multiplicative hash of its key words (int64 arithmetic wraps),
    high bits folded, modulo the world size. Identical on every rank for identical key words."""
    h = keys[:, 0] * -7046029254386353131
    for w in range(1, keys.shape[1]):
        h = (h ^ keys[:, w]) * -7046029254386353131
    return ((h >> 33) & 0x3FFFFFFF) % world


def exchange_rows(rows, dest, group=None):
    """All-to-all of [n, w] int64 rows: row i goes to rank dest[i]. Returns this rank's received rows (in
    source-rank order). One all-to-all of the counts, one of the rows."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    order = torch.argsort(dest, stable=True)
    send = rows[order].contiguous()
    send_counts = torch.bincount(dest, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    recv = rows.new_empty((sum(rc), rows.shape[1]))
    dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc, group=group)
    return recv


def merge_by_value(p, group=None, stream=None, root=None):
    """GroupByDataTableReducer's merge (GroupByDataTableReducer.java:258) across ranks, partitioned by key:
    export_groups -> all-to-all by key owner -> merge_groups of this rank's share (each group's partials
    meet on one rank, so 1/N of the rows per rank) -> the merged shares, disjoint, all-gathered (or
    gathered on `root`) -> merge_groups again, which only inserts them. Returns the bytes this rank put into
    the collectives (its exported rows, then its merged share)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    keys, acc = p.export_groups(stream=stream)
    kw = keys.shape[1]
    rows = torch.cat([keys, acc], dim=1)
    nbytes = rows.numel() * 8
    mine = exchange_rows(rows, key_owner(keys, world), group)
    p.merge_groups(mine[:, :kw].contiguous(), mine[:, kw:].contiguous(), stream=stream)
    mk, ma = p.export_groups(stream=stream)
    share = torch.cat([mk, ma], dim=1)
    nbytes += share.numel() * 8
    if root is None:
        allr = gather_rows(share, group)
    else:
        allr = gather_rows_to(share, root, group)
        if dist.get_rank(group) != root:
            return nbytes
    p.merge_groups(allr[:, :kw].contiguous(), allr[:, kw:].contiguous(), stream=stream)
    return nbytes


def gather_rows(rows, group=None, return_counts: bool = False):
    """All-gather every rank's [n_r, w] int64 rows (n_r may differ) into the concatenation in rank order:
    one all-gather of the row counts, one of the rows padded to the largest count."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    counts = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts)
    w = rows.shape[1]
    if m == 0:
        out = rows.new_empty((0, w))
        return (out, counts) if return_counts else out
    buf = rows.new_zeros((m, w))
    buf[:rows.shape[0]] = rows
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = torch.cat([p[:c] for p, c in zip(parts, counts)]).contiguous()
    return (out, counts) if return_counts else out


def gather_rows_to(rows, root: int, group=None):
    """gather_rows onto one rank (the broker's view): the rows of every rank in rank order on `root`, an
    empty tensor elsewhere. Counts travel by all-gather (tiny), rows by one gather."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    counts = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m, w = max(counts), rows.shape[1]
    if m == 0:
        return rows.new_empty((0, w))
    buf = rows.new_zeros((m, w))
    buf[:rows.shape[0]] = rows
    me = dist.get_rank(group)
    parts = [torch.empty_like(buf) for _ in range(world)] if me == root else None
    dist.gather(buf, parts, dst=root, group=group)
    if me != root:
        return rows.new_empty((0, w))
    return torch.cat([p[:c] for p, c in zip(parts, counts)]).contiguous()


def merge_groups(qc, groups: dict, group=None) -> dict:
    """Host merge by value of every rank's fetched groups (GroupByDataTableReducer.java:258 /
    AggregationFunction.merge) through all_gather_object: the reference semantics merge_result's device
    path implements, kept for callers holding groups() dicts (small results, tests)."""
    import torch.distributed as dist
    from .query import merge_partial
    world = dist.get_world_size(group)
    parts = [None] * world
    dist.all_gather_object(parts, groups, group=group)
    out: dict = {}
    for g in parts:
        for k, v in g.items():
            out[k] = [merge_partial(a.func, x, y) for a, x, y in zip(qc.aggregations, out[k], v)] if k in out else v
    return out


def local_key_values(segments, column: str, executor=None) -> list:
    """Distinct values of a group-by column over this rank's segments: the dictionaries of
    dictionary-encoded columns; raw columns' values through a device GROUP BY over all docs."""
    from .query import distinct_value
    vals = {}
    raw = []
    for s in segments:
        cb = s.columns[column]
        if cb.has_dictionary:
            for v in cb.dict_values.tolist():
                vals.setdefault(distinct_value(v), v)
        else:
            raw.append(s)
    if raw:
        from .engine import ServerQueryExecutor
        ex = executor or ServerQueryExecutor()
        res = ex.execute(f"SET numGroupsLimit = {1 << 40}; SELECT {column}, COUNT(*) FROM t GROUP BY {column}", raw)
        for (v,) in res.groups():
            vals.setdefault(distinct_value(v), v)
        res.destroy()
    return list(vals.values())


def key_columns(qc) -> list:
    """Columns whose key space must be global for a cross-rank merge: the GROUP BY columns, and the
    DISTINCTCOUNT columns (their device queries group by them too)."""
    cols = list(qc.group_by)
    for a in qc.aggregations:
        if a.func == "DISTINCTCOUNT" and a.column not in cols:
            cols.append(a.column)
    return cols


def _value_kind(vals) -> str:
    """'i' (all Python ints), 'f' (all floats), 's' (all strings), '-' (none), 'o' (mixed)."""
    if not vals:
        return "-"
    if all(isinstance(v, int) and not isinstance(v, bool) for v in vals):
        return "i"
    if all(isinstance(v, float) for v in vals):
        return "f"
    if all(isinstance(v, str) for v in vals):
        return "s"
    return "o"


def _gather_strings(vals, group=None) -> list:
    """Every rank's strings, concatenated in rank order, as tensors over the process group (no pickling):
    the UTF-8 byte lengths as [n, 1] int64 rows and the concatenated bytes packed 8 per int64 row, each
    through gather_rows (which also returns each rank's row counts, to cut the byte blob per rank)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    enc = [v.encode("utf-8") for v in vals]
    lens = np.asarray([len(b) for b in enc], dtype=np.int64)
    blob = b"".join(enc)
    blob += b"\0" * ((-len(blob)) % 8)
    words = np.frombuffer(blob, dtype=np.int64) if blob else np.zeros(0, dtype=np.int64)
    all_lens, nstr = gather_rows(torch.from_numpy(lens.reshape(-1, 1).copy()).to(dev), group, return_counts=True)
    all_words, _ = gather_rows(torch.from_numpy(words.reshape(-1, 1).copy()).to(dev), group, return_counts=True)
    all_lens = all_lens.cpu().numpy().reshape(-1)
    data = all_words.cpu().numpy().reshape(-1).tobytes()
    out, li, pos = [], 0, 0
    for c in nstr:  # rank by rank: its strings, then its blob padded to 8 bytes
        start = pos
        for n in all_lens[li:li + c].tolist():
            out.append(data[pos:pos + n].decode("utf-8"))
            pos += n
        li += c
        pos = start + ((pos - start + 7) // 8) * 8
    return out


def _gather_numeric(vals, kind: str, group=None) -> list:
    """Every rank's numeric values, concatenated in rank order, through gather_rows (two RCCL / gloo
    all-gathers of int64 tensors; doubles travel as their bit patterns, so -0.0 and NaN payloads
    arrive unchanged)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    arr = np.asarray(vals, dtype=np.int64) if kind == "i" else np.asarray(vals, dtype=np.float64).view(np.int64)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    rows = torch.from_numpy(arr.reshape(-1, 1).copy()).to(dev)
    out = gather_rows(rows, group).cpu().numpy().reshape(-1)
    return out.tolist() if kind == "i" else out.view(np.float64).tolist()


def global_key_space(segments, group_by: Sequence[str], group=None, executor=None) -> dict:
    """Union over all ranks of every group-by column's values, to install with
    ServerQueryExecutor.execute(..., key_space=...) so that every rank's dense group table indexes the
    same groups and merge_result can all-reduce them in place. Numeric columns travel as int64 tensors
    (one all-gather of counts, one of the padded values: million-value raw key columns never go through
    pickling), STRING columns as UTF-8 lengths + bytes packed in int64 tensors (_gather_strings); only ranks
    disagreeing on a column's value kind fall back to all_gather_object. The union keeps the first
    occurrence in rank order."""
    import torch.distributed as dist
    from .query import distinct_value
    mine = {g: local_key_values(segments, g, executor) for g in group_by}
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    gathered = {}
    if world > 1:
        kinds = [None] * world
        dist.all_gather_object(kinds, {g: _value_kind(mine[g]) for g in group_by}, group=group)
        objs = []
        for g in group_by:
            ks = {k[g] for k in kinds} - {"-"}
            if len(ks) == 1 and ks <= {"i", "f"}:
                gathered[g] = _gather_numeric(mine[g], ks.pop(), group)
            elif ks == {"s"}:
                gathered[g] = _gather_strings(mine[g], group)
            elif not ks:
                gathered[g] = []
            else:
                objs.append(g)
        if objs:
            parts = [None] * world
            dist.all_gather_object(parts, {g: mine[g] for g in objs}, group=group)
            for g in objs:
                gathered[g] = [v for p in parts for v in p[g]]
    else:
        gathered = mine
    out = {}
    for g in group_by:
        u = {}
        for v in gathered[g]:
            u.setdefault(distinct_value(v), v)
        out[g] = list(u.values())
    return out


def key_space_fingerprint(segments, group_by: Sequence[str]) -> str:
    """Hash of the merged dictionaries of the group-by columns (to check ranks agree)."""
    h = hashlib.sha256()
    for g in group_by:
        vals = set()
        for s in segments:
            vals.update(s.columns[g].dict_values.tolist())
        for v in sorted(vals, key=repr):
            h.update(repr(v).encode())
    return h.hexdigest()
