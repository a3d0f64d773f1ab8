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

OP_SUM_I64, OP_SUM_F64, OP_MIN, OP_MAX = 0, 1, 2, 3
SIGN = -(1 << 63)  # 0x8000000000000000 as int64


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


def merge_tables(table, ops: Sequence[int], num_keys: int, group=None) -> None:
    """In-place all-reduce of a [len(ops), num_keys] int64 tensor of accumulator words.

    ops per row: 0 = int64 sum, 1 = fp64 sum (words are double bits), 2/3 = min/max of the
    library's ordered-uint64 encoding (flipping the sign bit makes it an order-preserving int64)."""
    import torch
    import torch.distributed as dist
    t = table.view(len(ops), num_keys)
    for i, op in enumerate(ops):
        row = t[i]
        if op == OP_SUM_I64:
            dist.all_reduce(row, op=dist.ReduceOp.SUM, group=group)
        elif op == OP_SUM_F64:
            f = row.view(torch.float64)
            dist.all_reduce(f, op=dist.ReduceOp.SUM, group=group)
        else:
            s = row ^ SIGN
            dist.all_reduce(s, op=dist.ReduceOp.MIN if op == OP_MIN else dist.ReduceOp.MAX, group=group)
            row.copy_(s ^ SIGN)


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
