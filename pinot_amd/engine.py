"""Host-side mirror of pinot-core's server query execution for the HBM-resident hot path.

Class names follow the reference so that tests and callers read like Pinot:

* :class:`ImmutableSegment` — ``ImmutableSegmentLoader.load`` (pinot-segment-local/.../loader/
  ImmutableSegmentLoader.java): stages a segment's column buffers into HBM through
  ``pinot_amd_segment_add_column``.
* :class:`ServerQueryExecutor` — ``ServerQueryExecutorV1Impl.execute`` -> ``InstancePlanMakerImplV2``
  plan -> per-segment ``AggregationOperator`` / ``GroupByOperator`` -> ``*CombineOperator``
  (pinot-core/.../query/executor/ServerQueryExecutorV1Impl.java). All segments of the call are
  executed in one batched device pass.
* :class:`QueryResult` — ``AggregationGroupByResult`` / ``IntermediateResultsBlock``: per group the
  intermediate results of every aggregation (AVG as (sum, count)), mergeable across servers.

Every computation goes through libpinot_amd.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import gc
import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import ColumnSpec, PredicateSpec, check, lib
from .query import (JavaDouble, QueryContext, fold_distinct_count, parse_sql, reduce_rows, server_table,
                    split_distinct_count)
from .segment import ColumnBuffers, SegmentBuffers, DOUBLE, FLOAT, INT, LONG, STRING

TYPE_CODE = {INT: 0, LONG: 1, FLOAT: 2, DOUBLE: 3, STRING: 4}
ENC_CODE = {"FIXED_BIT": 0, "RAW": 1, "SORTED": 2}
PRED_CODE = {"EQ": 0, "NOT_EQ": 1, "IN": 2, "NOT_IN": 3, "RANGE": 4}
AGG_CODE = {"COUNT": 0, "SUM": 1, "MIN": 2, "MAX": 3, "SUMLONG": 4, "AVG": 5, "MINMAXRANGE": 6}
EXPR_CODE = {"MUL": 1, "SUB": 2, "ADD": 3}


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        return None
    return int(getattr(stream, "cuda_stream", stream))


class ImmutableSegment:
    """A segment whose forward indexes, dictionaries and inverted indexes live in HBM."""

    def __init__(self, buffers: SegmentBuffers):
        L = lib()
        self.name = buffers.name
        self.num_docs = buffers.num_docs
        self.columns: Dict[str, ColumnBuffers] = {}
        h = C.c_void_p()
        check(L.pinot_amd_segment_create(buffers.name.encode(), buffers.num_docs, C.byref(h)), "segment_create")
        self._h = h
        for cb in buffers.columns.values():
            self.add_column(cb)

    def add_column(self, cb: ColumnBuffers) -> None:
        spec = ColumnSpec()
        spec.name = cb.name.encode()
        spec.stored_type = TYPE_CODE[cb.stored_type]
        spec.encoding = ENC_CODE[cb.encoding]
        spec.cardinality = cb.cardinality
        spec.bits_per_element = cb.bits_per_element
        keep = [cb.fwd, cb.dictionary, cb.inverted]
        spec.h_fwd = C.cast(C.c_char_p(cb.fwd), C.c_void_p)
        spec.fwd_size = len(cb.fwd)
        if cb.dictionary:
            spec.h_dictionary = C.cast(C.c_char_p(cb.dictionary), C.c_void_p)
            spec.dictionary_size = len(cb.dictionary)
        if cb.inverted:
            spec.h_inverted = C.cast(C.c_char_p(cb.inverted), C.c_void_p)
            spec.inverted_size = len(cb.inverted)
        check(lib().pinot_amd_segment_add_column(self._h, C.byref(spec)), f"add_column({cb.name})")
        del keep
        self.columns[cb.name] = cb

    @property
    def handle(self):
        return self._h

    def device_bytes(self) -> int:
        return int(lib().pinot_amd_segment_device_bytes(self._h))

    def column_fwd_ptr(self, column: str) -> int:
        p = lib().pinot_amd_segment_column_fwd(self._h, column.encode())
        if not p:
            raise KeyError(column)
        return int(p)

    def destroy(self) -> None:
        if self._h:
            lib().pinot_amd_segment_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.destroy()
        except Exception:
            pass


def _coerce(value, stored_type: str):
    if stored_type == STRING:
        return str(value)
    if stored_type in (INT, LONG):
        if isinstance(value, float):
            if not value.is_integer():
                raise ValueError(f"non-integral literal {value} for {stored_type} column")
            value = int(value)
        if isinstance(value, str):
            value = int(value)
        return int(value)
    return float(value)


def _predicate_spec(pred, column: ColumnBuffers, use_inverted: bool, keep: list) -> PredicateSpec:
    s = PredicateSpec()
    s.column = pred.column.encode()
    s.type = PRED_CODE[pred.type]
    st = column.stored_type
    s.use_inverted_index = 1 if (use_inverted and column.inverted is not None and pred.type != "RANGE") else 0
    if pred.type == "RANGE":
        s.lower_unbounded = 1 if pred.lower is None else 0
        s.upper_unbounded = 1 if pred.upper is None else 0
        s.lower_inclusive = 1 if pred.lower_inclusive else 0
        s.upper_inclusive = 1 if pred.upper_inclusive else 0
        for side in ("lower", "upper"):
            v = getattr(pred, side)
            if v is None:
                continue
            v = _coerce(v, st)
            if st == STRING:
                b = v.encode()
                keep.append(b)
                setattr(s, side + "_s", b)
            elif st in (INT, LONG):
                setattr(s, side + "_i", v)
            else:
                setattr(s, side + "_d", v)
        return s
    s.num_values = len(pred.values)
    if st == STRING:
        vals = [_coerce(v, st) for v in pred.values]
        arr = (C.c_char_p * len(vals))(*[v.encode() for v in vals])
        keep.append(arr)
        s.h_values_s = arr
    elif st in (INT, LONG):
        # numpy buffers handed over by pointer: a ctypes array built element by element cost ~0.5 us per literal
        if all(type(v) is int for v in pred.values):
            arr = np.asarray(pred.values, dtype=np.int64)
        else:
            arr = np.asarray([_coerce(v, st) for v in pred.values], dtype=np.int64)
        keep.append(arr)
        s.h_values_i = arr.ctypes.data_as(C.POINTER(C.c_int64))
    else:
        arr = np.asarray([_coerce(v, st) for v in pred.values], dtype=np.float64)
        keep.append(arr)
        s.h_values_d = arr.ctypes.data_as(C.POINTER(C.c_double))
    return s


class DistinctCountResult:
    """Result of a query with DISTINCTCOUNT aggregations (query.split_distinct_count): the base
    result plus one grouped result per DISTINCTCOUNT, folded into per-group value sets."""

    def __init__(self, qc, base, subs, server_trim: bool = False):
        self.qc, self._base, self._subs = qc, base, subs
        self._server_trim = server_trim  # the server's combine table over the folded groups

    def num_docs_matched(self) -> int:
        return self._base.num_docs_matched()

    def num_groups_limit_reached(self) -> bool:
        return self._base.num_groups_limit_reached()

    def kernel_info(self) -> str:
        return self._base.kernel_info()

    def _all(self):
        return [self._base] + [r for _, r in self._subs]

    def groups(self):
        g = fold_distinct_count(self.qc, self._base.groups(), [(i, r.groups()) for i, r in self._subs])
        return server_table(self.qc, g) if self._server_trim else g

    def rows(self):
        return reduce_rows(self.qc, self.groups())

    def execute_again(self, stream=None) -> None:
        for r in self._all():
            r.execute_again(stream)

    def last_kernel_ms(self) -> float:
        return sum(r.last_kernel_ms() for r in self._all())

    def algorithmic_bytes(self) -> float:
        return sum(r.algorithmic_bytes() for r in self._all())

    def accumulators(self):
        raise NotImplementedError("DISTINCTCOUNT results merge by value (dist.merge_result merges each of "
                                  "results() with export_groups / merge_groups), not as one accumulator table")

    def results(self):
        """The device results this one folds: the base query, then one per DISTINCTCOUNT (each a GROUP BY
        whose groups are (group key, distinct value) pairs: merged by value across ranks, they union the
        value sets)."""
        return self._all()

    def destroy(self) -> None:
        for r in self._all():
            r.destroy()


class _DeviceWord:
    """One library-owned int64 in HBM seen by torch without a copy (__cuda_array_interface__)."""

    def __init__(self, ptr: int):
        self.__cuda_array_interface__ = {"shape": (1,), "typestr": "<i8", "data": (ptr, False), "version": 2,
                                         "strides": None}


def selfcheck_failures() -> int:
    """Executions of this process whose partitioned self-check failed (pinot_amd_selfcheck_failures)."""
    return int(lib().pinot_amd_selfcheck_failures())


class QueryResult:
    """Results of one executed query plan (kept in HBM until fetched)."""

    def __init__(self, handle, qc: QueryContext, agg_slots: List[tuple], key_types: List[str]):
        self._h = handle
        self.qc = qc
        self._agg_slots = agg_slots      # per qc aggregation: ('direct', native_idx) | ('avg', sum_idx)
        self._key_types = key_types
        self._merged_reached = None      # numGroupsLimitReached OR-ed over ranks by dist.merge_result

    def execute_again(self, stream=None) -> None:
        self._merged_reached = None
        check(lib().pinot_amd_execute_again(self._h, _stream_handle(stream)), "execute_again")

    def set_merged_limit_reached(self, reached: bool) -> None:
        """The broker ORs numGroupsLimitReached over servers (BrokerReduceService): after a cross-rank
        merge every rank reports the OR of all ranks' flags, until the next execution."""
        self._merged_reached = bool(reached)

    def num_docs_matched(self) -> int:
        out = C.c_int64()
        check(lib().pinot_amd_result_num_docs_matched(self._h, C.byref(out)), "num_docs_matched")
        return out.value

    def num_groups_limit_reached(self) -> bool:
        """GroupByResultsBlock.isNumGroupsLimitReached: more groups than the numGroupsLimit option (after
        dist.merge_result: the OR over every rank's)."""
        if self._merged_reached is not None:
            return self._merged_reached
        out = C.c_int32()
        check(lib().pinot_amd_result_num_groups_limit_reached(self._h, C.byref(out)), "num_groups_limit_reached")
        return bool(out.value)

    def kernel_info(self) -> str:
        """The device plan: 'jit' (fused scan), 'jit-select' / 'jit-wselect' (selection vector; the
        filter on 4-doc tiles / 64-doc bitset words), 'jit-partitioned', 'jit-hash', 'jit-hash-trim';
        ' xN' when the batch ran as N shape launches."""
        return lib().pinot_amd_result_kernel_info(self._h).decode()

    def last_kernel_ms(self) -> float:
        out = C.c_double()
        check(lib().pinot_amd_result_last_kernel_ms(self._h, C.byref(out)), "last_kernel_ms")
        return out.value

    def plan_timing(self) -> Dict[str, float]:
        """Host planning milliseconds per phase of the execute that built this result."""
        txt = lib().pinot_amd_result_plan_timing(self._h).decode()
        return {k: float(v) for k, v in (kv.split("=") for kv in txt.split(";") if kv)}

    def algorithmic_bytes(self) -> float:
        """Algorithmic HBM bytes of the last execution (pinot_amd_result_algorithmic_bytes)."""
        out = C.c_double()
        check(lib().pinot_amd_result_algorithmic_bytes(self._h, C.byref(out)), "algorithmic_bytes")
        return out.value

    def accumulators(self):
        """(ops, num_keys, [device pointers]) of the dense accumulators for a cross-GPU merge."""
        n = C.c_int32()
        nk = C.c_int64()
        check(lib().pinot_amd_result_accumulators(self._h, C.byref(n), C.byref(nk), None, None), "accumulators")
        ptrs = (C.c_void_p * n.value)()
        ops = (C.c_int32 * n.value)()
        check(lib().pinot_amd_result_accumulators(self._h, C.byref(n), C.byref(nk), ptrs, ops), "accumulators")
        return list(ops), nk.value, [int(p) for p in ptrs]

    def check_word(self) -> int:
        """Device address of the execution's self-check word (one int64, 0 = the check held; see
        pinot_amd_result_check_word): a cross-rank merge carries it through its collectives."""
        out = C.c_void_p()
        check(lib().pinot_amd_result_check_word(self._h, C.byref(out)), "check_word")
        return int(out.value)

    def self_check_failed(self) -> bool:
        """Whether the last execution's self-check failed (reads the word without raising: the ranks of a
        merge agree on it before anyone fails)."""
        import torch
        w = torch.as_tensor(_DeviceWord(self.check_word()), device="cuda")
        return bool(int(w.item()) != 0)

    def has_dense_table(self) -> bool:
        """True when the groups live in a dense accumulator table over the key space (mergeable in place
        across ranks with all-reduces); False for hash-table plans and merged results."""
        n = C.c_int32()
        nk = C.c_int64()
        return lib().pinot_amd_result_accumulators(self._h, C.byref(n), C.byref(nk), None, None) == 0

    def export_groups(self, stream=None):
        """This result's groups as device tensors for a cross-rank merge by value
        (pinot_amd_result_export_groups): keys [groups, key_words] and accumulator words [groups, num_acc],
        int64, written on `stream` (synchronised before returning)."""
        import torch
        L = lib()
        kw, na, ng = C.c_int32(), C.c_int32(), C.c_int64()
        sh = _stream_handle(stream)
        check(L.pinot_amd_result_export_groups(self._h, None, None, 0, C.byref(kw), C.byref(na), C.byref(ng), sh),
              "export_groups")
        keys = torch.empty((ng.value, kw.value), dtype=torch.int64, device="cuda")
        acc = torch.empty((ng.value, na.value), dtype=torch.int64, device="cuda")
        if ng.value:
            torch.cuda.current_stream().synchronize()  # the allocations are ordered on torch's stream
            check(L.pinot_amd_result_export_groups(self._h, keys.data_ptr(), acc.data_ptr(), ng.value, C.byref(kw),
                                                   C.byref(na), C.byref(ng), sh), "export_groups")
        return keys, acc

    def merge_groups(self, keys, acc, stream=None) -> None:
        """Fold gathered (keys, acc) rows of every rank into this result (pinot_amd_result_merge_groups):
        until the next execution, groups() are the merged groups. The tensors must be ready on `stream`."""
        assert keys.is_contiguous() and acc.is_contiguous() and keys.shape[0] == acc.shape[0]
        check(lib().pinot_amd_result_merge_groups(self._h, keys.data_ptr(), acc.data_ptr(), keys.shape[0],
                                                  _stream_handle(stream)), "merge_groups")

    def fetch_arrays(self):
        """The groups as flat arrays straight from the library (pinot_amd_result_fetch): (number of groups,
        keys [g * num_group_by + j], final values as double [g * num_aggs + a], exact int64 values, MINMAXRANGE
        pairs or None). groups() turns them into Python values."""
        L = lib()
        ng = C.c_int64()
        check(L.pinot_amd_result_num_groups(self._h, C.byref(ng)), "num_groups")
        n = max(ng.value, 1)
        nk = len(self.qc.group_by)
        nnat = max(len(self._native_aggs), 1)
        keys = np.zeros(n * max(nk, 1), dtype=np.int64)
        vals = np.zeros(n * nnat, dtype=np.float64)
        vals_i = np.zeros(n * nnat, dtype=np.int64)
        got = C.c_int64()
        check(L.pinot_amd_result_fetch(self._h, n, keys.ctypes.data_as(C.POINTER(C.c_int64)),
                                       vals.ctypes.data_as(C.POINTER(C.c_double)),
                                       vals_i.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(got)), "fetch")
        pairs = None
        if any(s[0] == "range" for s in self._agg_slots):
            pairs = np.zeros(n * nnat * 2, dtype=np.float64)
            got2 = C.c_int64()
            check(L.pinot_amd_result_fetch_intermediate(self._h, n, pairs.ctypes.data_as(C.POINTER(C.c_double)),
                                                        C.byref(got2)), "fetch_intermediate")
        return got, keys, vals, vals_i, pairs

    def groups(self, arrays=None) -> Dict[tuple, list]:
        """key tuple (group-by values; () for aggregation-only) -> intermediate result per aggregation.
        Converted column-wise (numpy -> Python lists, zipped), not group by group. `arrays`: the output of
        an earlier fetch_arrays() of this execution (not fetched again)."""
        L = lib()
        got, keys, vals, vals_i, pairs = self.fetch_arrays() if arrays is None else arrays
        n = got.value
        nk = len(self.qc.group_by)
        nnat = max(len(self._native_aggs), 1)
        kcols = []
        if nk:
            karr = keys[:n * nk].reshape(n, nk)
            for j in range(nk):
                t = self._key_types[j]
                col = karr[:, j]
                if t == STRING:
                    names = {int(i): L.pinot_amd_result_string_key(self._h, j, int(i)).decode() for i in np.unique(col)}
                    kcols.append([names[i] for i in col.tolist()])
                elif t in (FLOAT, DOUBLE):
                    kcols.append([JavaDouble(x) for x in col.view(np.float64).tolist()])
                else:
                    kcols.append(col.tolist())
            key_tuples = list(zip(*kcols))
        else:
            key_tuples = [()] * n
        v = vals[:n * nnat].reshape(n, nnat)
        vi = vals_i[:n * nnat].reshape(n, nnat)
        acols = []
        for a, slot in zip(self.qc.aggregations, self._agg_slots):
            if slot[0] == "avg":
                acols.append(list(zip(v[:, slot[1]].tolist(), vi[:, slot[2]].tolist())))
            elif slot[0] == "range":
                pr = pairs[:n * nnat * 2].reshape(n, nnat, 2)
                acols.append(list(zip(pr[:, slot[1], 0].tolist(), pr[:, slot[1], 1].tolist())))
            elif a.func in ("COUNT", "SUMLONG"):
                acols.append(vi[:, slot[1]].tolist())
            else:
                acols.append(v[:, slot[1]].tolist())
        # a million small containers would trigger the cyclic GC over and over (none of them is cyclic)
        was = gc.isenabled()
        gc.disable()
        try:
            parts = list(map(list, zip(*acols))) if acols else [[] for _ in range(n)]
            return dict(zip(key_tuples, parts))
        finally:
            if was:
                gc.enable()

    def rows(self) -> List[tuple]:
        return reduce_rows(self.qc, self.groups())

    def destroy(self) -> None:
        if self._h:
            lib().pinot_amd_result_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.destroy()
        except Exception:
            pass


class ServerQueryExecutor:
    """Compiles a QueryContext and runs it over a list of HBM-resident segments.

    server_trim: apply the server's combine table to GROUP BY results like GroupByCombineOperator's
    IndexedTable (LIMIT groups without ORDER BY; the top max(5 * LIMIT, minServerGroupTrimSize) by the
    ORDER BY otherwise; pinot_amd_query_set_result_limit). Off by default: every group is returned,
    which is what a multi-server broker reduce over exact partials wants."""

    def __init__(self, use_inverted_index: bool = True, server_trim: bool = False):
        self.use_inverted_index = use_inverted_index
        self.server_trim = server_trim

    def filter_doc_ids(self, query, segments: Sequence[ImmutableSegment], stream=None) -> List[np.ndarray]:
        """FilterPlanNode -> BlockDocIdSet: ascending matching docIds of each segment (the filter
        runs on the device into a dense bitset, compacted with ballot / prefix sums)."""
        import torch
        qc = parse_sql(query) if isinstance(query, str) else query
        L = lib()
        qh = self._compile(qc, segments)
        try:
            arr = (C.c_void_p * len(segments))(*[s.handle.value for s in segments])
            rh = C.c_void_p()
            check(L.pinot_amd_execute_filter(qh, arr, len(segments), _stream_handle(stream), C.byref(rh)),
                  "execute_filter")
        finally:
            L.pinot_amd_query_destroy(qh)
        out = []
        try:
            for i, seg in enumerate(segments):
                p = C.c_void_p()
                nw = C.c_int64()
                check(L.pinot_amd_result_bitset(rh, i, C.byref(p), C.byref(nw)), "result_bitset")
                ids = torch.empty(max(seg.num_docs, 1), dtype=torch.int32, device="cuda")
                cnt = C.c_int64()
                check(L.pinot_amd_bitset_to_doc_ids(p.value, seg.num_docs, ids.data_ptr(), C.byref(cnt),
                                                    _stream_handle(stream)), "bitset_to_doc_ids")
                out.append(ids[:cnt.value].cpu().numpy())
        finally:
            L.pinot_amd_result_destroy(rh)
        return out

    def _compile(self, qc: QueryContext, segments: Sequence[ImmutableSegment]):
        L = lib()
        first = segments[0]
        qh = C.c_void_p()
        check(L.pinot_amd_query_create(C.byref(qh)), "query_create")
        keep: list = []
        try:
            for ci, clause in enumerate(qc.cnf):
                for pred, neg in clause:
                    col = first.columns.get(pred.column)
                    if col is None:
                        raise _lib.PinotAmdError(f"unknown column {pred.column!r} in segment {first.name}")
                    spec = _predicate_spec(pred, col, self.use_inverted_index, keep)
                    check(L.pinot_amd_query_add_predicate(qh, ci, C.byref(spec), 1 if neg else 0), "add_predicate")
        except Exception:
            L.pinot_amd_query_destroy(qh)
            raise
        return qh

    def execute(self, query, segments: Sequence[ImmutableSegment], stream=None, key_space=None):
        """Run a query over HBM-resident segments. key_space (optional): group-by column -> the values of
        its global key space (dist.global_key_space: the union of every rank's dictionaries), so that
        every rank's dense group table indexes the same groups."""
        qc = parse_sql(query) if isinstance(query, str) else query
        if any(a.func == "DISTINCTCOUNT" for a in qc.aggregations):
            # the device queries run untrimmed (a result limit on a (group, value) sub-query would cut value
            # sets); the server's combine table applies to the folded groups (DistinctCountResult.groups)
            trim = self.server_trim and bool(qc.group_by)
            if trim and qc.safe_trim() and qc.limit >= qc.sort_aggregate_limit_threshold \
                    and not qc.server_return_final_result:
                raise _lib.PinotAmdError("DISTINCTCOUNT with a segment-level safe trim (ORDER BY = GROUP BY, LIMIT >= "
                                         "sortAggregateLimitThreshold) is not supported with server_trim")
            base, subs = split_distinct_count(qc)
            return DistinctCountResult(qc, self._execute(base, segments, stream, key_space, server_trim=False),
                                       [(i, self._execute(sq, segments, stream, key_space, server_trim=False))
                                        for i, sq in subs], server_trim=trim)
        return self._execute(qc, segments, stream, key_space)

    @staticmethod
    def _set_key_space(qh, column: str, stored_type: str, values) -> None:
        n = len(values)
        vi = vd = vs = None
        if stored_type == STRING:
            vs = (C.c_char_p * max(n, 1))(*[str(v).encode() for v in values])
        elif stored_type in (FLOAT, DOUBLE):
            vd = (C.c_double * max(n, 1))(*[float(v) for v in values])
        else:
            vi = (C.c_int64 * max(n, 1))(*[int(v) for v in values])
        check(lib().pinot_amd_query_set_group_key_values(qh, column.encode(), TYPE_CODE[stored_type], n, vi, vd, vs),
              f"set_group_key_values({column})")

    def _execute(self, qc, segments: Sequence[ImmutableSegment], stream=None, key_space=None,
                 server_trim=None) -> QueryResult:
        if not segments:
            raise ValueError("no segments")
        server_trim = self.server_trim if server_trim is None else server_trim
        L = lib()
        first = segments[0]
        qh = C.c_void_p()
        check(L.pinot_amd_query_create(C.byref(qh)), "query_create")
        keep: list = []
        try:
            for ci, clause in enumerate(qc.cnf):
                for pred, neg in clause:
                    col = first.columns.get(pred.column)
                    if col is None:
                        raise _lib.PinotAmdError(f"unknown column {pred.column!r} in segment {first.name}")
                    spec = _predicate_spec(pred, col, self.use_inverted_index, keep)
                    check(L.pinot_amd_query_add_predicate(qh, ci, C.byref(spec), 1 if neg else 0), "add_predicate")
            for g in qc.group_by:
                check(L.pinot_amd_query_add_group_by(qh, g.encode()), "add_group_by")
                if key_space is not None and g in key_space:
                    self._set_key_space(qh, g, first.columns[g].stored_type, key_space[g])
            check(L.pinot_amd_query_set_num_groups_limit(qh, qc.num_groups_limit), "set_num_groups_limit")
            if server_trim and qc.group_by:
                check(L.pinot_amd_query_set_result_limit(qh, qc.limit, qc.min_server_group_trim_size,
                                                         qc.group_trim_threshold), "set_result_limit")
                check(L.pinot_amd_query_set_server_options(qh, 1 if qc.server_return_final_result else 0,
                                                           qc.sort_aggregate_limit_threshold), "set_server_options")
                check(L.pinot_amd_query_set_segment_trim(qh, qc.min_segment_group_trim_size), "set_segment_trim")
            native = []
            agg_slots = []

            def add(func, column, expr=None):
                key = (func, column)
                if key in native:
                    return native.index(key)
                idx = C.c_int32()
                if expr is None:
                    check(L.pinot_amd_query_add_aggregation(qh, AGG_CODE[func], column.encode(), C.byref(idx)),
                          f"add_aggregation({func})")
                else:
                    check(L.pinot_amd_query_add_aggregation_expr(qh, AGG_CODE[func], EXPR_CODE[expr[0]],
                                                                 expr[1].encode(), expr[2].encode(), C.byref(idx)),
                          f"add_aggregation_expr({func} {column})")
                native.append(key)
                return idx.value

            for a in qc.aggregations:
                if a.func == "AVG":
                    agg_slots.append(("avg", add("SUM", a.column, a.expr), add("COUNT", "*")))
                elif a.func == "MINMAXRANGE":  # MinMaxRangePair (min, max), NaN-skipping, in the library
                    agg_slots.append(("range", add("MINMAXRANGE", a.column, a.expr)))
                else:
                    agg_slots.append(("direct", add(a.func, a.column, a.expr)))
            if not qc.aggregations and qc.group_by:
                add("COUNT", "*")  # DISTINCT-style group-by still needs the group presence count
            if server_trim and qc.group_by:
                for kind, idx, asc in qc.order_by_targets():
                    if kind == 1:  # the library aggregation whose final value orders (AVG: sum / count)
                        a = qc.aggregations[idx]
                        idx = add(a.func, a.column, a.expr)
                    check(L.pinot_amd_query_add_order_by(qh, kind, idx, 1 if asc else 0), "add_order_by")
            arr = (C.c_void_p * len(segments))(*[s.handle.value for s in segments])
            rh = C.c_void_p()
            check(L.pinot_amd_execute(qh, arr, len(segments), _stream_handle(stream), C.byref(rh)), "execute")
        finally:
            L.pinot_amd_query_destroy(qh)
        key_types = [first.columns[g].stored_type for g in qc.group_by]
        res = QueryResult(rh, qc, agg_slots, key_types)
        res._native_aggs = native
        return res
