"""pinot_amd — MI355X-native execution of Pinot's server-side segment scan / filter / group-by path.

Layers:
  segment.py  Pinot on-disk column formats (fixed-bit / sorted / raw forward index, dictionaries,
              roaring inverted index) — segment creation and parsing on the host
  query.py    QueryContext: SQL subset, filter CNF, broker reduce
  engine.py   ImmutableSegment (HBM staging) + ServerQueryExecutor over libpinot_amd.so
  dist.py     one process per GPU: segment sharding + RCCL merge of dense group tables
  csrc/       gfx950 HIP kernels and the C ABI (include/pinot_amd.h)
"""
from .query import parse_sql, QueryContext, Predicate, FilterContext  # noqa: F401

__all__ = ["parse_sql", "QueryContext", "Predicate", "FilterContext"]
