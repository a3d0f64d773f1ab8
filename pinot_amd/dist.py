"""One process per GPU: segment sharding and the cross-GPU merge of group-by results.

Pinot combines per-segment results on a server (GroupByCombineOperator) and then across servers
in the broker (BrokerReduceService). Here every GPU executes its shard of segments into a dense
accumulator table over the query's merged key space (accumulation across its own segments happens
in-kernel), and the tables of all GPUs are merged in place with RCCL all-reduces over xGMI:
SUM/COUNT as int64 or fp64 sums, MIN/MAX as min/max of an order-preserving int64 encoding of the
double value. One all-reduce per accumulator array; no other data-path collective.

The merge is valid when every rank's merged dictionaries of the group-by columns agree (the
segments share a table's dictionaries or the union is installed on all ranks);
``key_space_fingerprint`` lets callers assert that before merging.
"""
from __future__ import annotations

import ctypes as C
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


def merge_tables(table, ops: Sequence[int], num_keys: int, group=None) -> None:
    """In-place all-reduce of a [len(ops), num_keys] int64 tensor of accumulator words.

    ops per row: 0 = int64 sum, 1 = fp64 sum (words are double bits), 2/3 = min/max of the
    library's ordered-uint64 encoding (flipping the sign bit makes it an order-preserving int64),
    4/5 = low/high word of an exact 128-bit integer sum (all-reduced as 32-bit limbs).
    One collective per reduction kind: all integer sums (int64 rows and the limbs of 128-bit rows) in
    one int64 SUM, double sums in one fp64 SUM, and one MIN / one MAX."""
    import torch
    import torch.distributed as dist
    t = table.view(len(ops), num_keys)
    ops = list(ops)
    i64 = [i for i, op in enumerate(ops) if op == OP_SUM_I64]
    i128 = [i for i, op in enumerate(ops) if op == OP_SUM_I128]
    f64 = [i for i, op in enumerate(ops) if op == OP_SUM_F64]
    parts = [t[i64]] if i64 else []
    parts += [_limbs(t[i], t[i + 1]) for i in i128]
    if parts:
        buf = torch.cat(parts).contiguous()
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        if i64:
            t[i64] = buf[:len(i64)]
        for j, i in enumerate(i128):
            lo, hi = _from_limbs(buf[len(i64) + 4 * j: len(i64) + 4 * j + 4])
            t[i] = lo
            t[i + 1] = hi
    if f64:
        f = t[f64].contiguous().view(torch.float64)
        dist.all_reduce(f, op=dist.ReduceOp.SUM, group=group)
        t[f64] = f.view(torch.int64)
    for op, rop in ((OP_MIN, dist.ReduceOp.MIN), (OP_MAX, dist.ReduceOp.MAX)):
        rows = [i for i, o in enumerate(ops) if o == op]
        if rows:
            s_ = (t[rows] ^ SIGN).contiguous()
            dist.all_reduce(s_, op=rop, group=group)
            t[rows] = s_ ^ SIGN


_hip = None


def _hip_memcpy(dst: int, src: int, nbytes: int, stream=None) -> None:
    """Device-to-device copy through the process's (torch-loaded) HIP runtime."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so.7")
        _hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _hip.hipMemcpyAsync.restype = C.c_int
    rc = _hip.hipMemcpyAsync(dst, src, nbytes, 3, stream)  # hipMemcpyDeviceToDevice
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync failed: {rc}")


def merge_result(result, scratch=None, group=None, stream=None):
    """All-reduce a QueryResult's dense accumulators across ranks (in place). Returns the scratch
    tensor so callers can reuse it across steps."""
    import torch
    ops, nk, ptrs = result.accumulators()
    if not ops:
        return scratch
    n = len(ops) * nk
    if scratch is None or scratch.numel() != n:
        scratch = torch.empty(n, dtype=torch.int64, device="cuda")
    sh = None if stream is None else int(getattr(stream, "cuda_stream", stream))
    _hip_memcpy(scratch.data_ptr(), ptrs[0], n * 8, sh)  # rows are contiguous in one allocation
    merge_tables(scratch, ops, nk, group)
    _hip_memcpy(ptrs[0], scratch.data_ptr(), n * 8, sh)
    return scratch


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
