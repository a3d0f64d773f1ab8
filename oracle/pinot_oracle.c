/*
 * pinot_oracle.c — scalar CPU restatement of Pinot's segment scan / filter /
 * aggregation / group-by hot path. TEST INFRASTRUCTURE ONLY (see pinot_oracle.h).
 *
 * Reference paths are relative to the reference checkout root; "PDB" below is
 * pinot-segment-local/src/main/java/org/apache/pinot/segment/local/io/util/PinotDataBitSet.java.
 */
#include "pinot_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ helpers */
static uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
static uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
static uint16_t le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint64_t le64(const uint8_t* p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

/* ------------------------------------------------------------------ forward index */

/* PinotDataBitSet.readInt(int index, int numBitsPerValue) — PDB:80-102.
 * FixedBitIntReader.BitNReader.read / FixedBitSVForwardIndexReaderV2.getDictId return the
 * same value (they are unrolled specialisations of this stream layout). */
int32_t oracle_fixedbit_read(const uint8_t* buf, int32_t bits, int64_t index) {
  const uint32_t BYTE_MASK = 0xFF;
  int64_t bit_offset = index * (int64_t)bits;
  int64_t byte_offset = bit_offset / 8;
  int bit_in_first = (int)(bit_offset % 8);
  uint32_t current = buf[byte_offset] & (BYTE_MASK >> bit_in_first);
  int left = bits - (8 - bit_in_first);
  if (left <= 0) {
    return (int32_t)(current >> -left);
  }
  while (left > 8) {
    byte_offset++;
    current = (current << 8) | (buf[byte_offset] & BYTE_MASK);
    left -= 8;
  }
  return (int32_t)((current << left) | ((buf[byte_offset + 1] & BYTE_MASK) >> (8 - left)));
}

/* PinotDataBitSet.readInt(int startIndex, int numBitsPerValue, int length, int[] buffer) — PDB:104-141 */
void oracle_fixedbit_read_range(const uint8_t* buf, int32_t bits, int64_t start, int64_t n, int32_t* out) {
  for (int64_t i = 0; i < n; i++) out[i] = oracle_fixedbit_read(buf, bits, start + i);
}

/* PinotDataBitSet.writeInt(int index, int numBitsPerValue, int value) — PDB:143-170 */
void oracle_fixedbit_write(uint8_t* buf, int32_t bits, int64_t start, int64_t n, const int32_t* values) {
  for (int64_t k = 0; k < n; k++) {
    uint32_t value = (uint32_t)values[k];
    int64_t bit_offset = (start + k) * (int64_t)bits;
    int64_t byte_offset = bit_offset / 8;
    int bit_in_first = (int)(bit_offset % 8);
    uint32_t first = buf[byte_offset];
    uint32_t first_mask = 0xFFu >> bit_in_first;
    int left = bits - (8 - bit_in_first);
    if (left <= 0) {
      first_mask &= (0xFFu << -left) & 0xFFu;
      buf[byte_offset] = (uint8_t)((first & ~first_mask) | (value << -left));
    } else {
      buf[byte_offset] = (uint8_t)((first & ~first_mask) | ((value >> left) & first_mask));
      while (left > 8) {
        left -= 8;
        byte_offset++;
        buf[byte_offset] = (uint8_t)(value >> left);
      }
      byte_offset++;
      uint32_t last = buf[byte_offset];
      buf[byte_offset] = (uint8_t)((last & (0xFFu >> left)) | (value << (8 - left)));
    }
  }
}

/* SortedIndexReaderImpl.getDictId: binary search over (min,max) pairs
 * (pinot-segment-local/.../readers/sorted/SortedIndexReaderImpl.java:50-100). */
int32_t oracle_sorted_dict_id(const uint8_t* pairs, int32_t cardinality, int64_t doc) {
  int32_t lo = 0, hi = cardinality - 1;
  while (lo <= hi) {
    int32_t mid = (lo + hi) >> 1;
    int64_t start = (int32_t)be32(pairs + 8 * (int64_t)mid);
    if (start <= doc) {
      lo = mid + 1;
    } else {
      hi = mid - 1;
    }
  }
  return hi;
}

/* FixedBytePower2ChunkSVForwardIndexReader.getInt/getLong/getFloat/getDouble on a
 * PASS_THROUGH buffer: _rawData.getX(docId * size), big-endian
 * (.../readers/forward/FixedBytePower2ChunkSVForwardIndexReader.java:48-90). */
int64_t oracle_raw_read_i64(const uint8_t* raw, int32_t type, int64_t index) {
  switch (type) {
    case OR_INT: return (int32_t)be32(raw + 4 * index);
    case OR_LONG: return (int64_t)be64(raw + 8 * index);
    default: return 0;
  }
}
double oracle_raw_read_f64(const uint8_t* raw, int32_t type, int64_t index) {
  switch (type) {
    case OR_INT: return (double)(int32_t)be32(raw + 4 * index);
    case OR_LONG: return (double)(int64_t)be64(raw + 8 * index);
    case OR_FLOAT: {
      uint32_t u = be32(raw + 4 * index);
      float f;
      memcpy(&f, &u, 4);
      return (double)f;
    }
    case OR_DOUBLE: {
      uint64_t u = be64(raw + 8 * index);
      double d;
      memcpy(&d, &u, 8);
      return d;
    }
    default: return 0.0;
  }
}

static int32_t dict_id_of(const oracle_column* c, int64_t doc) {
  if (c->encoding == OR_ENC_IDS) return ((const int32_t*)c->fwd)[doc];
  if (c->encoding == OR_ENC_SORTED) return oracle_sorted_dict_id(c->fwd, c->cardinality, doc);
  return oracle_fixedbit_read(c->fwd, c->bits, doc);
}

void oracle_column_dict_ids(const oracle_column* col, int64_t start, int64_t n, int32_t* out) {
  for (int64_t i = 0; i < n; i++) out[i] = dict_id_of(col, start + i);
}

/* value of a column at doc as the stored type: dictionary lookup for dict columns
 * (Dictionary.readIntValues etc. behind BlockValSet.getXValuesSV) or raw read. */
static int is_float_type(int t) { return t == OR_FLOAT || t == OR_DOUBLE; }

static int64_t value_i64(const oracle_column* c, int64_t doc) {
  if (c->encoding == OR_ENC_RAW) return oracle_raw_read_i64(c->fwd, c->stored_type, doc);
  int32_t id = dict_id_of(c, doc);
  if (c->stored_type == OR_INT) return ((const int32_t*)c->dict)[id];
  return ((const int64_t*)c->dict)[id];
}
static double value_f64(const oracle_column* c, int64_t doc) {
  if (c->encoding == OR_ENC_RAW) return oracle_raw_read_f64(c->fwd, c->stored_type, doc);
  int32_t id = dict_id_of(c, doc);
  switch (c->stored_type) {
    case OR_INT: return (double)((const int32_t*)c->dict)[id];
    case OR_LONG: return (double)((const int64_t*)c->dict)[id];
    case OR_FLOAT: return (double)((const float*)c->dict)[id];
    default: return ((const double*)c->dict)[id];
  }
}

/* value of an aggregation's expression as the transform function yields it (double): the column
 * value, or MULT = 1.0 * a * b (MultiplicationTransformFunction.java: literal product, then each
 * argument in order), SUB = a - b (SubtractionTransformFunction.java), ADD = 0.0 + a + b
 * (AdditionTransformFunction.java) */
static double agg_f64(const oracle_column* cols, const oracle_agg* a, int64_t doc) {
  const double x = value_f64(&cols[a->column], doc);
  switch (a->expr) {
    case OR_EXPR_MUL: return 1.0 * x * value_f64(&cols[a->column2], doc);
    case OR_EXPR_SUB: return x - value_f64(&cols[a->column2], doc);
    case OR_EXPR_ADD: return 0.0 + x + value_f64(&cols[a->column2], doc);
    default: return x;
  }
}

/* Integer-valued SUM / AVG inputs (INT / LONG columns, and times/minus/plus of two INT columns) are
 * summed exactly in 128 bits and rounded to double once. SumAggregationFunction accumulates in double
 * (SumAggregationFunction.java:96-107,190-200); both agree whenever every partial sum stays below 2^53
 * (true of every reference golden value), and beyond that the exact sum is the value the north star's
 * "bit-exact integer SUM" pins (Pinot's own double accumulation then depends on the doc order). */
static int agg_is_int(const oracle_column* cols, const oracle_agg* a) {
  if (a->column < 0 || is_float_type(cols[a->column].stored_type)) return 0;
  if (a->expr == OR_EXPR_COL) return 1;
  return cols[a->column].stored_type == OR_INT && cols[a->column2].stored_type == OR_INT;
}
static __int128 agg_i128(const oracle_column* cols, const oracle_agg* a, int64_t doc) {
  const __int128 x = value_i64(&cols[a->column], doc);
  switch (a->expr) {
    case OR_EXPR_MUL: return x * value_i64(&cols[a->column2], doc);
    case OR_EXPR_SUB: return x - value_i64(&cols[a->column2], doc);
    case OR_EXPR_ADD: return x + value_i64(&cols[a->column2], doc);
    default: return x;
  }
}

/* LZ4 block decoding as lz4-java's LZ4FastDecompressor does it (org.lz4:lz4-java 1.11.0, pom.xml:186,
 * third-party): the chunk decompressor behind ChunkCompressionType.LZ4
 * (pinot-segment-local/.../io/compression/LZ4Decompressor.java). Returns bytes written or -1. */
int64_t oracle_lz4_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  int64_t ip = 0, op = 0;
  while (ip < n) {
    uint32_t token = src[ip++];
    int64_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do { if (ip >= n) return -1; b = src[ip++]; lit += b; } while (b == 255);
    }
    if (ip + lit > n || op + lit > cap) return -1;
    for (int64_t k = 0; k < lit; k++) dst[op++] = src[ip++];
    if (ip >= n) break;
    if (ip + 2 > n) return -1;
    int64_t off = src[ip] | (src[ip + 1] << 8);
    ip += 2;
    int64_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do { if (ip >= n) return -1; b = src[ip++]; ml += b; } while (b == 255);
    }
    ml += 4;
    if (off == 0 || off > op || op + ml > cap) return -1;
    for (int64_t k = 0; k < ml; k++, op++) dst[op] = dst[op - off];
  }
  return op;
}

/* Snappy raw block decoding (org.xerial.snappy:snappy-java 1.1.10.x, third-party: Snappy.uncompress,
 * the chunk decompressor behind ChunkCompressionType.SNAPPY, pinot-segment-local/.../io/compression/
 * SnappyDecompressor.java:40-44), restated from the published format: a varint uncompressed length,
 * then tagged elements -- 00 literal (length-1 in the tag's upper 6 bits, or 1-4 LE bytes after it
 * for 60..63), 01 copy (length 4..11, 11-bit offset), 10 copy (length 1..64, LE16 offset),
 * 11 copy (length 1..64, LE32 offset). Returns bytes written or -1. */
int64_t oracle_snappy_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  int64_t ip = 0, op = 0;
  uint64_t len = 0;
  for (int sh = 0;; sh += 7) {
    if (ip >= n || sh > 28) return -1;
    uint32_t b = src[ip++];
    len |= (uint64_t)(b & 0x7F) << sh;
    if (!(b & 0x80)) break;
  }
  if ((int64_t)len > cap) return -1;
  while (ip < n) {
    uint32_t tag = src[ip++];
    int64_t l, off;
    if ((tag & 3) == 0) {
      l = (tag >> 2) + 1;
      if (l > 60) {
        int nb = (int)l - 60;
        if (ip + nb > n) return -1;
        l = 0;
        for (int k = 0; k < nb; k++) l |= (int64_t)src[ip + k] << (8 * k);
        l += 1;
        ip += nb;
      }
      if (ip + l > n || op + l > (int64_t)len) return -1;
      for (int64_t k = 0; k < l; k++) dst[op++] = src[ip++];
      continue;
    }
    if ((tag & 3) == 1) {
      if (ip + 1 > n) return -1;
      l = 4 + ((tag >> 2) & 7);
      off = ((int64_t)(tag >> 5) << 8) | src[ip];
      ip += 1;
    } else if ((tag & 3) == 2) {
      if (ip + 2 > n) return -1;
      l = (tag >> 2) + 1;
      off = src[ip] | (src[ip + 1] << 8);
      ip += 2;
    } else {
      if (ip + 4 > n) return -1;
      l = (tag >> 2) + 1;
      off = (int64_t)le32(src + ip);
      ip += 4;
    }
    if (off == 0 || off > op || op + l > (int64_t)len) return -1;
    for (int64_t k = 0; k < l; k++, op++) dst[op] = dst[op - off];
  }
  return op == (int64_t)len ? op : -1;
}

static uint64_t rd_be(const uint8_t* p, int w) {
  uint64_t v = 0;
  for (int k = 0; k < w; k++) v = (v << 8) | p[k];
  return v;
}
static void wr_be(uint8_t* p, int w, uint64_t v) {
  for (int k = w - 1; k >= 0; k--, v >>= 8) p[k] = (uint8_t)v;
}

/* DELTA (dd = 0) / DELTADELTA (dd = 1) chunks (DeltaDecompressor.java:45-130,
 * DeltaDeltaDecompressor.java:45-140): flag byte (1 = LONG values, else INT), BE count, BE first
 * value, BE compressed size, then an LZ4 block of BE deltas (DELTADELTA: the first delta, then
 * deltas of deltas); values are rebuilt with Java's wrapping int/long arithmetic. */
int64_t oracle_delta_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t dd) {
  if (n < 5) return -1;
  const int w = src[0] == 1 ? 8 : 4;
  const int64_t cnt = (int32_t)rd_be(src + 1, 4);
  if (cnt < 0 || cnt * w > cap) return -1;
  if (cnt == 0) return 0;
  if (n < 5 + w) return -1;
  uint64_t prev = rd_be(src + 5, w);
  wr_be(dst, w, prev);
  if (cnt == 1) return w;
  if (n < 9 + w) return -1;
  const int64_t cs = (int32_t)rd_be(src + 5 + w, 4);
  if (cs < 0 || 9 + w + cs > n) return -1;
  const int64_t got = oracle_lz4_decompress(src + 9 + w, cs, dst + w, (cnt - 1) * w);
  if (got != (cnt - 1) * w) return -1;
  const uint64_t mask = w == 8 ? ~0ull : 0xFFFFFFFFull;
  uint64_t delta = 0;
  for (int64_t i = 1; i < cnt; i++) {
    const uint64_t e = rd_be(dst + i * w, w);
    delta = (dd && i > 1) ? (delta + e) & mask : e;
    prev = (prev + delta) & mask;
    wr_be(dst + i * w, w, prev);
  }
  return cnt * w;
}

/* ------------------------------------------------------------------ roaring */

/* RoaringBitmap 1.6.14 portable deserialisation (org.roaringbitmap.buffer.ImmutableRoaringBitmap,
 * third-party, not vendored): cookie 12346 = no run containers (int32 size follows),
 * 12347 | (size-1)<<16 = with run-container bitset; then (key u16, card-1 u16) per container;
 * offsets (int32) present unless (has runs && size < 4); then array (u16 x card), bitmap
 * (u64 x 1024) or run (nruns u16 + (start,len-1) u16 pairs) containers. Little-endian. */
int oracle_roaring_to_bitset(const uint8_t* buf, int64_t len, uint64_t* bitset, int64_t num_docs) {
  if (len < 4) return -1;
  uint32_t cookie = le32(buf);
  int64_t pos = 4;
  int32_t size;
  const uint8_t* runbits = NULL;
  int has_run = 0;
  if ((cookie & 0xFFFF) == 12347) {
    has_run = 1;
    size = (int32_t)(cookie >> 16) + 1;
    runbits = buf + pos;
    pos += (size + 7) / 8;
  } else if (cookie == 12346) {
    size = (int32_t)le32(buf + pos);
    pos += 4;
  } else {
    return -2;
  }
  const uint8_t* header = buf + pos;
  pos += 4 * (int64_t)size;
  if (!has_run || size >= 4) pos += 4 * (int64_t)size; /* skip offsets; containers are contiguous */
  for (int32_t i = 0; i < size; i++) {
    uint32_t key = le16(header + 4 * i);
    int32_t card = le16(header + 4 * i + 2) + 1;
    int64_t base = (int64_t)key << 16;
    int is_run = has_run && (runbits[i / 8] >> (i % 8)) & 1;
    if (is_run) {
      int32_t nruns = le16(buf + pos);
      pos += 2;
      for (int32_t r = 0; r < nruns; r++) {
        int64_t s = le16(buf + pos + 4 * r), l = le16(buf + pos + 4 * r + 2);
        for (int64_t d = base + s; d <= base + s + l; d++)
          if (d < num_docs) bitset[d >> 6] |= 1ull << (d & 63);
      }
      pos += 4 * (int64_t)nruns;
    } else if (card <= 4096) {
      for (int32_t j = 0; j < card; j++) {
        int64_t d = base + le16(buf + pos + 2 * j);
        if (d < num_docs) bitset[d >> 6] |= 1ull << (d & 63);
      }
      pos += 2 * (int64_t)card;
    } else {
      for (int32_t w = 0; w < 1024; w++) {
        uint64_t word = le64(buf + pos + 8 * w);
        while (word) {
          int b = __builtin_ctzll(word);
          int64_t d = base + 64 * w + b;
          if (d < num_docs) bitset[d >> 6] |= 1ull << (d & 63);
          word &= word - 1;
        }
      }
      pos += 8192;
    }
    if (pos > len) return -3;
  }
  return 0;
}

/* BitmapInvertedIndexReader.getDocIds(dictId) (.../readers/BitmapInvertedIndexReader.java:44-60)
 * OR-ed over the given dictIds, as BitmapBasedFilterOperator does for EQ/IN
 * (pinot-core/.../operator/filter/BitmapBasedFilterOperator.java). */
int oracle_inverted_to_bitset(const uint8_t* inv, int32_t cardinality, const int32_t* dict_ids, int32_t n,
                              uint64_t* bitset, int64_t num_docs) {
  uint32_t first = be32(inv);
  const uint8_t* bitmaps = inv + 4 * ((int64_t)cardinality + 1);
  for (int32_t k = 0; k < n; k++) {
    int32_t id = dict_ids[k];
    if (id < 0 || id >= cardinality) return -1;
    uint32_t s = be32(inv + 4 * (int64_t)id), e = be32(inv + 4 * ((int64_t)id + 1));
    int rc = oracle_roaring_to_bitset(bitmaps + (s - first), (int64_t)(e - s), bitset, num_docs);
    if (rc) return rc;
  }
  return 0;
}

/* ------------------------------------------------------------------ filter */

/* One predicate on one doc: PredicateEvaluator.applySV semantics
 * (RangePredicateEvaluatorFactory.java:221-224 dict range, :416-418 raw int range with
 * inclusive bounds; InPredicateEvaluatorFactory.java:188-190 dict set). */
static int leaf_match(const oracle_column* cols, const oracle_leaf* lf, int64_t doc) {
  int m = 0;
  switch (lf->kind) {
    case OR_PRED_DICT_RANGE: {
      int32_t id = dict_id_of(&cols[lf->column], doc);
      m = lf->lo_i <= id && lf->hi_i > id;
      break;
    }
    case OR_PRED_DICT_SET: {
      int32_t id = dict_id_of(&cols[lf->column], doc);
      m = lf->dict_mask[id] != 0;
      break;
    }
    case OR_PRED_RAW_RANGE: {
      const oracle_column* c = &cols[lf->column];
      if (is_float_type(c->stored_type)) {
        double v = value_f64(c, doc);
        m = v >= lf->lo_d && v <= lf->hi_d;
      } else {
        int64_t v = value_i64(c, doc);
        m = v >= lf->lo_i && v <= lf->hi_i;
      }
      break;
    }
    case OR_PRED_RAW_IN: {
      const oracle_column* c = &cols[lf->column];
      if (is_float_type(c->stored_type)) {
        double v = value_f64(c, doc);
        for (int32_t k = 0; k < lf->set_n && !m; k++) m = lf->set_d[k] == v;
      } else {
        int64_t v = value_i64(c, doc);
        for (int32_t k = 0; k < lf->set_n && !m; k++) m = lf->set_i[k] == v;
      }
      break;
    }
    case OR_PRED_DOC_BITSET:
      m = (lf->doc_bitset[doc >> 6] >> (doc & 63)) & 1;
      break;
  }
  return lf->negate ? !m : m;
}

/* Filter tree in conjunctive normal form, evaluated doc by doc like
 * ScanBasedFilterOperator/SVScanDocIdIterator (pinot-core/.../dociditerators/SVScanDocIdIterator.java:79-103)
 * under AndFilterOperator / OrFilterOperator. Returns the number of matching docs. */
int64_t oracle_filter(const oracle_column* cols, int64_t num_docs, const oracle_leaf* leaves, int32_t nleaves,
                      uint64_t* out_bitset) {
  int32_t nclauses = 0;
  for (int32_t i = 0; i < nleaves; i++)
    if (leaves[i].clause + 1 > nclauses) nclauses = leaves[i].clause + 1;
  memset(out_bitset, 0, sizeof(uint64_t) * (size_t)((num_docs + 63) / 64));
  int64_t count = 0;
  for (int64_t doc = 0; doc < num_docs; doc++) {
    int all = 1;
    for (int32_t c = 0; c < nclauses && all; c++) {
      int any = 0;
      for (int32_t i = 0; i < nleaves && !any; i++)
        if (leaves[i].clause == c) any = leaf_match(cols, &leaves[i], doc);
      all = any;
    }
    if (all) {
      out_bitset[doc >> 6] |= 1ull << (doc & 63);
      count++;
    }
  }
  return count;
}

/* BlockDocIdIterator order: ascending docIds */
int64_t oracle_bitset_to_doc_ids(const uint64_t* bitset, int64_t num_docs, int32_t* out) {
  int64_t n = 0;
  for (int64_t d = 0; d < num_docs; d++)
    if ((bitset[d >> 6] >> (d & 63)) & 1) out[n++] = (int32_t)d;
  return n;
}

/* ------------------------------------------------------------------ aggregation */

/* Integer SUM mode. 0 (default): the exact 128-bit integer sum, rounded to double once — what the
 * device computes, equal to Pinot's double accumulation while partial sums stay below 2^53. 1: Pinot's
 * literal arithmetic, the values added into a double in doc order (AggregationOperator: innerSum per
 * block of <= 10000 docs, then holder = innerSum + holder, SumAggregationFunction.java:80-92,179-188;
 * GROUP BY: holder + value per doc, :190-200). Tests bound the difference between the two. */
static int g_literal_int_sum = 0;
void oracle_set_literal_int_sum(int32_t on) { g_literal_int_sum = on != 0; }
int32_t oracle_literal_int_sum(void) { return g_literal_int_sum; }
static int exact_int_sum(const oracle_column* cols, const oracle_agg* a) {
  return !g_literal_int_sum && agg_is_int(cols, a);
}

#define MAX_DOC_PER_CALL 10000 /* pinot-core/.../plan/DocIdSetPlanNode.java:28 */

/* AggregationOperator over blocks of <= 10000 matching docs
 * (pinot-core/.../operator/query/AggregationOperator.java, DocIdSetOperator). Per block:
 * SUM: double innerSum over the block then holder += innerSum (SumAggregationFunction.java:84-136,160-170);
 * MIN/MAX: Math.min/Math.max of the block extreme into the holder, initial +/-inf
 * (MinAggregationFunction.java:38,83-135,175-185); COUNT: long; SUMLONG: long wrap
 * (SumLongAggregationFunction.java). */
int oracle_aggregate(const oracle_column* cols, int64_t num_docs, const uint64_t* bitset, const oracle_agg* aggs,
                     int32_t naggs, double* out, int64_t* out_i64, int64_t* out_hi64) {
  double* holder = (double*)malloc(sizeof(double) * (size_t)naggs);
  double* inner = (double*)malloc(sizeof(double) * (size_t)naggs);
  int64_t* li = (int64_t*)calloc((size_t)naggs, sizeof(int64_t));
  __int128* exact = (__int128*)calloc((size_t)naggs, sizeof(__int128));
  for (int32_t a = 0; a < naggs; a++) {
    const int f = aggs[a].func;
    holder[a] = (f == OR_AGG_MIN || f == OR_AGG_RMIN) ? INFINITY : (f == OR_AGG_MAX || f == OR_AGG_RMAX) ? -INFINITY : 0.0;
  }
  int64_t doc = 0;
  while (doc < num_docs) {
    /* gather the next block of up to MAX_DOC_PER_CALL matching docs */
    int64_t block[MAX_DOC_PER_CALL];
    int32_t len = 0;
    while (doc < num_docs && len < MAX_DOC_PER_CALL) {
      if (!bitset || ((bitset[doc >> 6] >> (doc & 63)) & 1)) block[len++] = doc;
      doc++;
    }
    if (len == 0) break;
    for (int32_t a = 0; a < naggs; a++) {
      const oracle_column* c = aggs[a].column >= 0 ? &cols[aggs[a].column] : NULL;
      switch (aggs[a].func) {
        case OR_AGG_COUNT:
          li[a] += len;
          break;
        case OR_AGG_SUM: {
          if (exact_int_sum(cols, &aggs[a])) {  /* exact, see agg_is_int */
            for (int32_t i = 0; i < len; i++) exact[a] += agg_i128(cols, &aggs[a], block[i]);
            break;
          }
          double s = 0;
          for (int32_t i = 0; i < len; i++) s += agg_f64(cols, &aggs[a], block[i]);
          holder[a] = s + holder[a];
          break;
        }
        case OR_AGG_SUMLONG: {
          uint64_t s = 0;
          for (int32_t i = 0; i < len; i++) s += (uint64_t)value_i64(c, block[i]);
          li[a] = (int64_t)((uint64_t)li[a] + s);
          break;
        }
        case OR_AGG_MIN: {
          double m = INFINITY;
          for (int32_t i = 0; i < len; i++) m = fmin(m, agg_f64(cols, &aggs[a], block[i]));
          /* Math.min propagates NaN; fmin does not */
          for (int32_t i = 0; i < len; i++)
            if (isnan(agg_f64(cols, &aggs[a], block[i]))) m = NAN;
          holder[a] = (isnan(m) || isnan(holder[a])) ? NAN : fmin(m, holder[a]);
          break;
        }
        case OR_AGG_MAX: {
          double m = -INFINITY;
          for (int32_t i = 0; i < len; i++) m = fmax(m, agg_f64(cols, &aggs[a], block[i]));
          for (int32_t i = 0; i < len; i++)
            if (isnan(agg_f64(cols, &aggs[a], block[i]))) m = NAN;
          holder[a] = (isnan(m) || isnan(holder[a])) ? NAN : fmax(m, holder[a]);
          break;
        }
        /* MinMaxRangeAggregationFunction.aggregateSV (:95-103): MinMaxRangePair.apply(value) compares
         * with < / > (MinMaxRangePair.java:37-48), so NaN never enters the pair */
        case OR_AGG_RMIN:
          for (int32_t i = 0; i < len; i++) {
            const double v = agg_f64(cols, &aggs[a], block[i]);
            if (v < holder[a]) holder[a] = v;
          }
          break;
        case OR_AGG_RMAX:
          for (int32_t i = 0; i < len; i++) {
            const double v = agg_f64(cols, &aggs[a], block[i]);
            if (v > holder[a]) holder[a] = v;
          }
          break;
      }
    }
  }
  for (int32_t a = 0; a < naggs; a++) {
    if (aggs[a].func == OR_AGG_COUNT || aggs[a].func == OR_AGG_SUMLONG) {
      out[a] = (double)li[a];
      out_i64[a] = li[a];
      out_hi64[a] = li[a] < 0 ? -1 : 0;
    } else if (aggs[a].func == OR_AGG_SUM && exact_int_sum(cols, &aggs[a])) {
      out[a] = (double)exact[a];
      out_i64[a] = (int64_t)(uint64_t)(unsigned __int128)exact[a];
      out_hi64[a] = (int64_t)(exact[a] >> 64);
    } else {
      out[a] = holder[a];
      out_i64[a] = 0;
      out_hi64[a] = 0;
    }
  }
  free(holder);
  free(inner);
  free(li);
  free(exact);
  return 0;
}

/* ------------------------------------------------------------------ group-by */

typedef struct {
  double h;        /* double holder (SUM on floating values, MIN, MAX) */
  int64_t li;      /* COUNT / SUMLONG */
  __int128 exact;  /* SUM on integer values */
} or_holder;

static void holder_init(or_holder* h, int func) {
  h->h = (func == OR_AGG_MIN || func == OR_AGG_RMIN) ? INFINITY : (func == OR_AGG_MAX || func == OR_AGG_RMAX) ? -INFINITY : 0.0;
  h->li = 0;
  h->exact = 0;
}

/* DefaultGroupByExecutor.process -> AggregationFunction.aggregateGroupBySV for one doc of a group:
 * SUM: holder + value (SumAggregationFunction.java:190-200), MIN: `value < holder`
 * (MinAggregationFunction.java:215-223), MAX: `value > holder`, COUNT: +1, SUMLONG: long wrap. */
static void holder_add(or_holder* h, const oracle_column* cols, const oracle_agg* a, int64_t doc) {
  const oracle_column* c = a->column >= 0 ? &cols[a->column] : NULL;
  switch (a->func) {
    case OR_AGG_COUNT: h->li += 1; break;
    case OR_AGG_SUM:
      if (exact_int_sum(cols, a)) h->exact += agg_i128(cols, a, doc);
      else h->h = h->h + agg_f64(cols, a, doc);
      break;
    case OR_AGG_SUMLONG: h->li = (int64_t)((uint64_t)h->li + (uint64_t)value_i64(c, doc)); break;
    case OR_AGG_MIN: { double v = agg_f64(cols, a, doc); if (v < h->h) h->h = v; break; }
    case OR_AGG_MAX: { double v = agg_f64(cols, a, doc); if (v > h->h) h->h = v; break; }
    /* MinMaxRangeAggregationFunction.setGroupByResult (:105-114): a group's first doc creates the pair
     * from its value (NaN included, which then stays: every later < / > against NaN is false); later
     * docs apply with < / >. li marks "pair created". */
    case OR_AGG_RMIN: { double v = agg_f64(cols, a, doc); if (!h->li || v < h->h) h->h = v; h->li = 1; break; }
    case OR_AGG_RMAX: { double v = agg_f64(cols, a, doc); if (!h->li || v > h->h) h->h = v; h->li = 1; break; }
  }
}

/* out: the double result; out_i / out_hi: COUNT / SUMLONG as int64 (sign-extended), and an integer
 * SUM's exact 128-bit value as (low, high) words, so the combine can carry it exactly */
static void holder_out(const or_holder* h, const oracle_column* cols, const oracle_agg* a, double* out, int64_t* out_i,
                       int64_t* out_hi) {
  *out_hi = 0;
  switch (a->func) {
    case OR_AGG_COUNT:
    case OR_AGG_SUMLONG: *out = (double)h->li; *out_i = h->li; *out_hi = h->li < 0 ? -1 : 0; break;
    case OR_AGG_SUM:
      if (exact_int_sum(cols, a)) {
        *out = (double)h->exact;
        *out_i = (int64_t)(uint64_t)(unsigned __int128)h->exact;
        *out_hi = (int64_t)(h->exact >> 64);
      } else {
        *out = h->h;
        *out_i = 0;
      }
      break;
    default: *out = h->h; *out_i = 0;
  }
}

static uint64_t mix_ids(const int32_t* ids, int32_t n) {
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int32_t j = 0; j < n; j++) {
    x ^= (uint64_t)(uint32_t)ids[j];
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
  }
  return x;
}

/* GroupByOperator + DefaultGroupByExecutor + DictionaryBasedGroupKeyGenerator over one segment.
 * Raw keys: key = sum_j dictId_j * prod_{i<j} card_i (the loop `rawKey = rawKey * card[j] + dictId[j]`
 * for j = n-1..0, DictionaryBasedGroupKeyGenerator.java:316-327,427-434); the holder is chosen as the
 * constructor does (:144-180):
 *   ARRAY_BASED when the key space is <= arrayBasedThreshold (10000) and <= numGroupsLimit: one slot
 *     per raw key, every key admitted (:304-342);
 *   otherwise a map holder (IntMapBasedHolder / LongMapBasedHolder / ArrayMapBasedHolder, :444-900),
 *     all with getGroupId(rawKey, numGroupsLimit) semantics: a key absent from the map gets the next
 *     group id while the map holds fewer than numGroupsLimit keys, and is dropped (INVALID_ID) after
 *     that (:651-659). Docs are visited in docId order, so a segment keeps the first numGroupsLimit
 *     keys its matching docs reach. Keyed here on the dictId tuple itself (the raw key is a bijection
 *     of it).
 * out_keys[g*ngroup + j] = dictId of group-by column j; groups in group-id order. *out_limit_reached =
 * numGroups >= numGroupsLimit (GroupByOperator.java:133). Returns groups, or -1 beyond max_groups. */
int64_t oracle_group_by(const oracle_column* cols, int64_t num_docs, const uint64_t* bitset,
                        const int32_t* group_cols, int32_t ngroup, const oracle_agg* aggs, int32_t naggs,
                        int64_t num_groups_limit, int64_t max_groups, int32_t* out_keys, double* out_vals,
                        int64_t* out_i64, int64_t* out_hi64, int32_t* out_limit_reached) {
  double prod = 1;
  for (int32_t j = 0; j < ngroup; j++) prod *= (double)cols[group_cols[j]].cardinality;
  const int array_based = prod <= 10000 && prod <= (double)num_groups_limit;
  int64_t nmatch = 0;
  for (int64_t d = 0; d < num_docs; d++)
    if (!bitset || ((bitset[d >> 6] >> (d & 63)) & 1)) nmatch++;
  /* group ids -> keys and holders */
  const int64_t max_ids = array_based ? (int64_t)prod : (nmatch < num_groups_limit ? nmatch : num_groups_limit);
  int32_t* gkeys = (int32_t*)malloc(sizeof(int32_t) * (size_t)(max_ids + 1) * (size_t)(ngroup ? ngroup : 1));
  or_holder* hold = (or_holder*)malloc(sizeof(or_holder) * (size_t)(max_ids + 1) * (size_t)(naggs ? naggs : 1));
  int64_t* array_gid = NULL;  /* ARRAY_BASED: raw key -> group id */
  int64_t* slots = NULL;      /* map holder: open addressing over group ids */
  int64_t cap = 16;
  if (array_based) {
    array_gid = (int64_t*)malloc(sizeof(int64_t) * (size_t)(prod > 0 ? prod : 1));
    for (int64_t k = 0; k < (int64_t)prod; k++) array_gid[k] = -1;
  } else {
    while (cap < 2 * max_ids + 16) cap <<= 1;
    slots = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    for (int64_t i = 0; i < cap; i++) slots[i] = -1;
  }
  int64_t ngroups = 0;
  int32_t ids[64];
  for (int64_t d = 0; d < num_docs; d++) {
    if (bitset && !((bitset[d >> 6] >> (d & 63)) & 1)) continue;
    for (int32_t j = 0; j < ngroup; j++) ids[j] = dict_id_of(&cols[group_cols[j]], d);
    int64_t gid = -1;
    if (array_based) {
      int64_t key = 0;
      for (int32_t j = ngroup - 1; j >= 0; j--) key = key * cols[group_cols[j]].cardinality + ids[j];
      gid = array_gid[key];
      if (gid < 0) gid = array_gid[key] = ngroups++;
      else goto have;
    } else {
      uint64_t i = mix_ids(ids, ngroup) & (uint64_t)(cap - 1);
      for (;; i = (i + 1) & (uint64_t)(cap - 1)) {
        if (slots[i] < 0) break;
        if (memcmp(&gkeys[slots[i] * ngroup], ids, sizeof(int32_t) * (size_t)ngroup) == 0) { gid = slots[i]; goto have; }
      }
      if (ngroups >= num_groups_limit) continue;  /* INVALID_ID: the doc's key is not admitted */
      gid = slots[i] = ngroups++;
    }
    memcpy(&gkeys[gid * ngroup], ids, sizeof(int32_t) * (size_t)ngroup);
    for (int32_t a = 0; a < naggs; a++) holder_init(&hold[gid * naggs + a], aggs[a].func);
  have:
    for (int32_t a = 0; a < naggs; a++) holder_add(&hold[gid * naggs + a], cols, &aggs[a], d);
  }
  if (out_limit_reached) *out_limit_reached = ngroups >= num_groups_limit;
  int64_t ret = ngroups;
  if (ngroups > max_groups) {
    ret = -1;
  } else {
    for (int64_t g = 0; g < ngroups; g++) {
      for (int32_t j = 0; j < ngroup; j++) out_keys[g * ngroup + j] = gkeys[g * ngroup + j];
      for (int32_t a = 0; a < naggs; a++)
        holder_out(&hold[g * naggs + a], cols, &aggs[a], &out_vals[g * naggs + a], &out_i64[g * naggs + a],
                   &out_hi64[g * naggs + a]);
    }
  }
  free(gkeys);
  free(hold);
  free(array_gid);
  free(slots);
  return ret;
}
