/*
 * row_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of java/fury-format's row writer
 * and reader semantics, used as the parity checker for the HIP path and as the `cpu_baseline`
 * ("port") leg of bench.py.  Nothing in fury_amd/ may include, link or call this file.
 *
 * Parity pinning: the reference's own known answers (ArrayEncoderTest lengths 224/1576/10824,
 * the C++ RowTest ToString answer, TypeInferenceTest order) and schema hashes produced by the
 * reference's python/pyfury/format/infer.py::compute_schema_hash, all under tests/golden/
 * (see DESIGN.md "Oracle").  The Java reference cannot be built here (no JDK) and the C++
 * sibling needs absl for its logging TU, so neither is executed.
 *
 * Every function names the reference file:line it restates.  Paths:
 *   FMT  = java/fury-format/src/main/java/org/apache/fury/format
 *   CORE = java/fury-core/src/main/java/org/apache/fury
 *
 * Structure mirrors the reference literally: a MemoryBuffer with a writer index (grow() hands
 * out zeroed bytes, like a fresh heap buffer), BinaryRowWriter / BinaryArrayWriter on top of it
 * sharing BinaryWriter's var-length append, and the generated toRow's per-field dispatch
 * (BaseBinaryEncoderBuilder.serializeFor) driven by Arrow-style input columns.
 *
 * Decode bounds (round 6, the reference's rule restated): every read of the batch is checked
 * against the batch buffer as MemoryBuffer does -- checkPosition(index, pos, length) throws
 * IndexOutOfBoundsException unless 0 <= index and index + length <= size
 * (CORE/memory/MemoryBuffer.java:303-309), get(index, dst, 0, size) / slice(offset, size) for a
 * payload (:311-325, :2515-2518), and copyToUnsafe's checkArgument over a primitive array's whole
 * element range (:2451-2455, reached from BinaryArray.toXxxArray, FMT/row/binary/BinaryArray.java:
 * 157-197, which the generated fromRow calls for primitive arrays, BaseBinaryEncoderBuilder.java:
 * 655-670).  Restated at container granularity, the way the device checks it: a row's / struct's
 * null bitmap + slots, an array's header + null bitmap + element slots, a map's key-size word and
 * both arrays, a STRING / BINARY payload, a DECIMAL's 16 bytes -- each checked whole when the decode
 * reaches it (a per-entry getter reads a subset of that range; a container that passes is read
 * without further checks).  A negative element count is an error too (BinaryArray.pointTo's
 * assert, :71; new byte[size] / new long[n] throw NegativeArraySizeException).  A value that fails
 * decodes as null and sets FO_ERR_OOB; map key / value arrays of different lengths set FO_ERR_MAP
 * (BinaryMap.pointTo, FMT/row/binary/BinaryMap.java:73-75, UnsupportedOperationException).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/fury_row.h"

/* ------------------------------------------------------------------------------------------
 * Errors
 * ---------------------------------------------------------------------------------------- */
static _Thread_local int g_err = 0;   /* per thread: bench.py's CPU baseline runs threads */
int fo_last_status(void) { return g_err; }

/* ------------------------------------------------------------------------------------------
 * Schema restatement: DataTypes.getTypeWidth (FMT/type/DataTypes.java:68-133) and
 * computeSchemaHash (FMT/type/DataTypes.java:499-544).
 * ---------------------------------------------------------------------------------------- */
int32_t fo_type_width(int32_t type_id) {
  switch (type_id) {
    case FURY_TYPE_BOOL: return 1;          /* visit(Bool) -> 1                 */
    case FURY_TYPE_INT8: return 1;          /* visit(Int)  -> bitWidth / 8      */
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: return 4;
    case FURY_TYPE_INT64: return 8;
    case FURY_TYPE_FLOAT32: return 4;       /* visit(FloatingPoint) SINGLE -> 4 */
    case FURY_TYPE_FLOAT64: return 8;
    case FURY_TYPE_DATE32: return 4;        /* visit(Date) -> 4                 */
    case FURY_TYPE_TIMESTAMP: return 8;     /* visit(Timestamp) -> 8            */
    default: return -1;                     /* Struct/List/Map/Binary/Decimal/Utf8 -> -1 */
  }
}

/* DataTypes.computeHash: Math.addExact(Math.multiplyExact(hash, 31), id); on
 * ArithmeticException hash >>= 2 (arithmetic shift) and retry; then recurse into
 * LIST element / MAP key,value / STRUCT children, depth first. */
static int64_t fo_hash_field(int64_t hash, const fury_field* f) {
  for (;;) {
    int64_t m, a;
    if (!__builtin_mul_overflow(hash, (int64_t)31, &m) &&
        !__builtin_add_overflow(m, (int64_t)f->type_id, &a)) {
      hash = a;
      break;
    }
    hash = hash >> 2;
  }
  for (int i = 0; i < f->num_children; i++) hash = fo_hash_field(hash, &f->children[i]);
  return hash;
}

int64_t fo_schema_hash(const fury_field* fields, int32_t n) {
  int64_t hash = 17;
  for (int i = 0; i < n; i++) hash = fo_hash_field(hash, &fields[i]);
  return hash;
}

/* BitUtils.calculateBitmapWidthInBytes (CORE/memory/BitUtils.java:175-177) */
static int32_t fo_bitmap_bytes(int64_t n) { return (int32_t)(((n + 63) / 64) * 8); }
/* BinaryWriter.roundNumberOfBytesToNearestWord (FMT/row/binary/writer/BinaryWriter.java:40-47) */
static int64_t fo_round8(int64_t n) { return (n & 7) ? n + (8 - (n & 7)) : n; }

/* ------------------------------------------------------------------------------------------
 * MemoryBuffer restatement (CORE/memory/MemoryBuffer.java): little-endian puts, grow() with
 * zero-filled new storage (growBuffer allocates a fresh byte[], :1221-1243).
 * ---------------------------------------------------------------------------------------- */
typedef struct fo_buf {
  uint8_t* data;
  int64_t size;
  int64_t writer_index;
} fo_buf;

static int fo_buf_init(fo_buf* b, int64_t cap) {
  b->data = (uint8_t*)calloc((size_t)(cap > 16 ? cap : 16), 1);
  b->size = cap > 16 ? cap : 16;
  b->writer_index = 0;
  return b->data ? 0 : -1;
}

/* MemoryBuffer.grow(neededSize) :1221-1243 */
static void fo_buf_grow(fo_buf* b, int64_t needed) {
  int64_t length = b->writer_index + needed;
  if (length > b->size) {
    int64_t nsize = length < (100LL << 20) ? length * 2 : length + (length >> 1);
    uint8_t* nd = (uint8_t*)realloc(b->data, (size_t)nsize);
    if (!nd) { g_err = FURY_ERR_ENCODER; return; }
    memset(nd + b->size, 0, (size_t)(nsize - b->size));
    b->data = nd;
    b->size = nsize;
  }
}

static void fo_put_i64(fo_buf* b, int64_t off, int64_t v) { memcpy(b->data + off, &v, 8); }
static int64_t fo_get_i64(const uint8_t* p) { int64_t v; memcpy(&v, p, 8); return v; }

/* ------------------------------------------------------------------------------------------
 * BinaryWriter / BinaryRowWriter / BinaryArrayWriter restatement.
 * ---------------------------------------------------------------------------------------- */
typedef struct fo_writer {
  fo_buf* buf;
  int64_t start;              /* BinaryWriter.startIndex                                  */
  int32_t bytes_before_bitmap;/* 0 for rows, 8 for arrays (numElements word)              */
  int32_t is_array;
  /* row */
  int32_t header_bytes;       /* bitmap bytes (row) / 8 + bitmap (array)                  */
  int32_t fixed_size;         /* row: bitmap + 8 * numFields                              */
  /* array */
  int32_t elem_size;
  int64_t num_elements;
} fo_writer;

/* BinaryRowWriter(Schema, ...) ctor :46-60 */
static void fo_row_writer_init(fo_writer* w, fo_buf* b, int32_t num_fields) {
  memset(w, 0, sizeof(*w));
  w->buf = b;
  w->header_bytes = fo_bitmap_bytes(num_fields);
  w->fixed_size = w->header_bytes + num_fields * 8;
}

/* BinaryArrayWriter(Field, ...) ctor :71-82: elementSize = width, or 8 when width < 0 */
static void fo_array_writer_init(fo_writer* w, fo_buf* b, const fury_field* elem) {
  memset(w, 0, sizeof(*w));
  w->buf = b;
  w->is_array = 1;
  w->bytes_before_bitmap = 8;
  int32_t width = fo_type_width(elem->type_id);
  w->elem_size = width < 0 ? 8 : width;
}

/* BinaryRowWriter.reset() :76-84 — startIndex = writerIndex, grow fixedSize, zero bitmap. */
static void fo_row_writer_reset(fo_writer* w) {
  fo_buf* b = w->buf;
  w->start = b->writer_index;
  fo_buf_grow(b, w->fixed_size);
  b->writer_index += w->fixed_size;
  for (int64_t i = w->start; i < w->start + w->header_bytes; i += 8) fo_put_i64(b, i, 0);
}

/* BinaryArrayWriter.reset(numElements) :91-118 */
static int fo_array_writer_reset(fo_writer* w, int64_t n) {
  fo_buf* b = w->buf;
  w->start = b->writer_index;
  w->num_elements = n;
  w->header_bytes = 8 + fo_bitmap_bytes(n);             /* BinaryArray.calculateHeaderInBytes */
  int64_t data_size = n * (int64_t)w->elem_size;
  if (data_size > (int64_t)(2147483647 - 15)) {          /* MAX_ROUNDED_ARRAY_LENGTH */
    g_err = FURY_ERR_UNSUPPORTED;
    return -1;
  }
  int64_t fixed_part = fo_round8(data_size);
  fo_buf_grow(b, w->header_bytes + fixed_part);
  fo_put_i64(b, w->start, n);                            /* numElements in an 8-byte word */
  for (int64_t i = w->start + 8; i < w->start + w->header_bytes; i += 8) fo_put_i64(b, i, 0);
  for (int64_t i = data_size; i < fixed_part; i++) b->data[w->start + w->header_bytes + i] = 0;
  b->writer_index += w->header_bytes + fixed_part;
  return 0;
}

/* getOffset: BinaryRowWriter.java:87-89 / BinaryArrayWriter.java:126-129 */
static int64_t fo_get_offset(const fo_writer* w, int64_t ordinal) {
  if (w->is_array) return w->start + w->header_bytes + ordinal * w->elem_size;
  return w->start + w->header_bytes + (ordinal << 3);
}

/* BitUtils.set / unset at startIndex + bytesBeforeBitMap (BinaryWriter.java:123-133) */
static void fo_set_null_at(fo_writer* w, int64_t ordinal) {
  w->buf->data[w->start + w->bytes_before_bitmap + (ordinal >> 3)] |= (uint8_t)(1u << (ordinal & 7));
}
static void fo_set_not_null_at(fo_writer* w, int64_t ordinal) {
  w->buf->data[w->start + w->bytes_before_bitmap + (ordinal >> 3)] &= (uint8_t)~(1u << (ordinal & 7));
}

/* BinaryWriter.write(int, long/double) :153-159 — 8-byte store, no null-bit change. */
static void fo_write_i64(fo_writer* w, int64_t ordinal, int64_t v) {
  fo_put_i64(w->buf, fo_get_offset(w, ordinal), v);
}

/* Narrow writes.  Row: putInt64(slot, 0) then the narrow put (BinaryRowWriter.java:92-124).
 * Array: setNotNullAt then the narrow put at elementSize stride (BinaryArrayWriter.java:131-163). */
static void fo_write_narrow(fo_writer* w, int64_t ordinal, const void* src, int width) {
  int64_t off = fo_get_offset(w, ordinal);
  if (w->is_array) {
    fo_set_not_null_at(w, ordinal);
  } else {
    fo_put_i64(w->buf, off, 0);
  }
  memcpy(w->buf->data + off, src, (size_t)width);
}

/* setOffsetAndSize(ordinal, absoluteOffset, size) :106-114 */
static void fo_set_offset_and_size(fo_writer* w, int64_t ordinal, int64_t abs, int64_t size) {
  int64_t rel = abs - w->start;
  int64_t v = (int64_t)(((uint64_t)rel << 32) | (uint64_t)(uint32_t)size);
  fo_write_i64(w, ordinal, v);
}

/* writeUnaligned(ordinal, bytes, 0, n) :187-194 — pad word zeroed before the copy. */
static void fo_write_unaligned(fo_writer* w, int64_t ordinal, const uint8_t* src, int64_t n) {
  fo_buf* b = w->buf;
  int64_t rounded = fo_round8(n);
  fo_buf_grow(b, rounded);
  if (n & 7) fo_put_i64(b, b->writer_index + ((n >> 3) << 3), 0);   /* zeroOutPaddingBytes */
  if (n) memcpy(b->data + b->writer_index, src, (size_t)n);
  fo_set_offset_and_size(w, ordinal, b->writer_index, n);
  b->writer_index += rounded;
}

/* writeDecimal :204-219 — 16 bytes (DecimalUtils.DECIMAL_BYTE_LENGTH) at the writer index. */
static void fo_write_decimal(fo_writer* w, int64_t ordinal, const uint8_t* src16) {
  fo_buf* b = w->buf;
  fo_buf_grow(b, 16);
  memcpy(b->data + b->writer_index, src16, 16);
  fo_set_offset_and_size(w, ordinal, b->writer_index, 16);
  b->writer_index += 16;
}

/* writeDirectly(long) :222-226 */
static void fo_write_directly(fo_writer* w, int64_t v) {
  fo_buf_grow(w->buf, 8);
  fo_put_i64(w->buf, w->buf->writer_index, v);
  w->buf->writer_index += 8;
}

/* ------------------------------------------------------------------------------------------
 * Column access helpers (Arrow layout: LSB validity bit = 1 valid).
 * ---------------------------------------------------------------------------------------- */
static int fo_col_valid(const fury_column* c, int64_t i) {
  return c->validity == NULL || ((c->validity[i >> 3] >> (i & 7)) & 1);
}

/* ------------------------------------------------------------------------------------------
 * Generated toRow restatement: BaseBinaryEncoderBuilder.serializeFor
 * (FMT/encoder/BaseBinaryEncoderBuilder.java:138-223) for a value at column index `i`.
 * ---------------------------------------------------------------------------------------- */
static void fo_serialize(fo_writer* w, int64_t ordinal, const fury_field* f,
                         const fury_column* c, int64_t i);

/* RowEncoderBuilder.buildEncodeExpression (FMT/encoder/RowEncoderBuilder.java:154-179):
 * one serializeFor per field, in schema order, for struct row `i` of `cols`. */
static void fo_to_row(fo_writer* w, const fury_field* fields, int32_t n,
                      const fury_column* cols, int64_t i) {
  for (int k = 0; k < n; k++) fo_serialize(w, k, &fields[k], &cols[k], i);
}

/* serializeForArrayByWriter (:225-278): reset(n) then serializeFor per element. */
static void fo_serialize_array(fo_writer* aw, const fury_field* elem, const fury_column* child,
                               int64_t begin, int64_t end) {
  if (fo_array_writer_reset(aw, end - begin)) return;
  for (int64_t j = begin; j < end; j++) fo_serialize(aw, j - begin, elem, child, j);
}

static void fo_serialize(fo_writer* w, int64_t ordinal, const fury_field* f,
                         const fury_column* c, int64_t i) {
  if (!fo_col_valid(c, i)) {            /* setValueOrNull / If(eqNull) -> setNullAt only */
    fo_set_null_at(w, ordinal);
    return;
  }
  int32_t width = fo_type_width(f->type_id);
  switch (f->type_id) {
    case FURY_TYPE_BOOL: {                /* write(ordinal, boolean) -> putBoolean 1/0 */
      const uint8_t* bits = (const uint8_t*)c->values;
      uint8_t v = (uint8_t)((bits[i >> 3] >> (i & 7)) & 1);
      fo_write_narrow(w, ordinal, &v, 1);
      return;
    }
    case FURY_TYPE_INT8:
    case FURY_TYPE_INT16:
    case FURY_TYPE_INT32:
    case FURY_TYPE_FLOAT32:
    case FURY_TYPE_DATE32:
      fo_write_narrow(w, ordinal, (const uint8_t*)c->values + i * width, width);
      return;
    case FURY_TYPE_INT64:
    case FURY_TYPE_FLOAT64:
    case FURY_TYPE_TIMESTAMP: {
      int64_t v;
      memcpy(&v, (const uint8_t*)c->values + i * 8, 8);
      fo_write_i64(w, ordinal, v);
      return;
    }
    case FURY_TYPE_STRING:                /* write(ordinal, String) -> getBytes(UTF_8) */
    case FURY_TYPE_BINARY: {
      int32_t b = c->offsets[i], e = c->offsets[i + 1];
      fo_write_unaligned(w, ordinal, (const uint8_t*)c->values + b, e - b);
      return;
    }
    case FURY_TYPE_DECIMAL:
      fo_write_decimal(w, ordinal, (const uint8_t*)c->values + i * 16);
      return;
    case FURY_TYPE_LIST: {                /* :198-215 offset / serializeArray / size */
      fo_writer aw;
      fo_array_writer_init(&aw, w->buf, &f->children[0]);
      int64_t offset = w->buf->writer_index;
      fo_serialize_array(&aw, &f->children[0], c->child, c->offsets[i], c->offsets[i + 1]);
      int64_t size = w->buf->writer_index - offset;
      fo_set_offset_and_size(w, ordinal, offset, size);
      return;
    }
    case FURY_TYPE_STRUCT: {              /* serializeForBean :363-417 */
      fo_writer rw;
      fo_row_writer_init(&rw, w->buf, f->num_children);
      int64_t offset = w->buf->writer_index;
      fo_row_writer_reset(&rw);
      fo_to_row(&rw, f->children, f->num_children, c->child, i);
      int64_t size = w->buf->writer_index - offset;
      fo_set_offset_and_size(w, ordinal, offset, size);
      return;
    }
    case FURY_TYPE_MAP: {                 /* serializeForMap :298-357 */
      /* children[0] = key field, children[1] = value field; c->child[0..1] = entry columns */
      int64_t offset = w->buf->writer_index;
      fo_write_directly(w, -1);
      fo_writer kw, vw;
      fo_array_writer_init(&kw, w->buf, &f->children[0]);
      fo_serialize_array(&kw, &f->children[0], &c->child[0], c->offsets[i], c->offsets[i + 1]);
      int64_t key_size = w->buf->writer_index - kw.start;
      fo_put_i64(w->buf, offset, key_size);   /* writeDirectly(offset, keyArray.size()) */
      fo_array_writer_init(&vw, w->buf, &f->children[1]);
      fo_serialize_array(&vw, &f->children[1], &c->child[1], c->offsets[i], c->offsets[i + 1]);
      int64_t size = w->buf->writer_index - offset;
      fo_set_offset_and_size(w, ordinal, offset, size);
      return;
    }
    default:
      g_err = FURY_ERR_UNSUPPORTED;
      (void)width;
      return;
  }
}

/* ------------------------------------------------------------------------------------------
 * Batch drivers.
 *
 * fo_encode_batch: RowEncoder.toRow per row (Encoders.java:88-93) — each row is written by a
 * BinaryRowWriter whose buffer starts zeroed, exactly the bytes of toRow(obj).toBytes().  Rows
 * are concatenated; row_offsets[0..n] receives the exclusive scan of row sizes.
 *
 * reuse != 0 restates RowEncoder.encode(obj) instead (Encoders.java:146,191-198): ONE buffer is
 * reused for all rows, so a null slot keeps whatever the previous row left there.
 * ---------------------------------------------------------------------------------------- */
int64_t fo_encode_batch(const fury_field* fields, int32_t nfields, const fury_column* cols,
                        int64_t nrows, uint8_t* out, int64_t out_cap, int64_t* row_offsets,
                        int32_t reuse) {
  g_err = 0;
  fo_buf b;
  if (fo_buf_init(&b, 1024)) return -FURY_ERR_ENCODER;
  fo_writer w;
  fo_row_writer_init(&w, &b, nfields);
  int64_t pos = 0;
  for (int64_t i = 0; i < nrows; i++) {
    b.writer_index = 0;
    if (!reuse) memset(b.data, 0, (size_t)b.size);      /* MemoryUtils.buffer(16): zeroed */
    fo_row_writer_reset(&w);
    fo_to_row(&w, fields, nfields, cols, i);
    if (g_err) { free(b.data); return -g_err; }
    int64_t size = b.writer_index - w.start;
    if (row_offsets) row_offsets[i] = pos;
    if (out) {
      if (pos + size > out_cap) { free(b.data); return -FURY_ERR_CAPACITY; }
      memcpy(out + pos, b.data + w.start, (size_t)size);
    }
    pos += size;
  }
  if (row_offsets) row_offsets[nrows] = pos;
  free(b.data);
  return pos;
}

/* ------------------------------------------------------------------------------------------
 * Reader restatement: BinaryRow / BinaryArray getters (FMT/row/binary/BinaryRow.java:79-123,
 * UnsafeTrait.java:68-197, BinaryArray.java:69-78,157-197) driving the generated fromRow
 * (RowEncoderBuilder.java:185-217: `if (!row.isNullAt(i)) bean.f = row.getX(i)`), with the
 * bean replaced by Arrow-style output columns.  A null leaves the value bytes 0 and clears
 * the validity bit; strings/binary of a null entry have zero length.
 *
 * Output variable-length buffers (values of STRING/BINARY, child columns of LIST/MAP) are
 * appended at the cursors in `cur` — one cursor per column node, depth first.
 * ---------------------------------------------------------------------------------------- */
/* Decode context: the batch (bounds), the errors found (FO_ERR_* bits), and the count walk's
 * per-row item budget (fo_count_walk). */
#define FO_ERR_OOB 1
#define FO_ERR_MAP 2
#define FO_ERR_BUDGET 4
static _Thread_local const uint8_t* g_rows;   /* batch base (per thread, as all decode state) */
static _Thread_local int64_t g_total;         /* batch bytes                */
static _Thread_local int32_t g_flags;         /* FO_ERR_* seen              */

/* MemoryBuffer.checkPosition / get / slice restated over [0, g_total): 0 <= p, 0 <= len,
 * p + len <= size (MemoryBuffer.java:303-309). */
static int fo_span_ok(int64_t p, int64_t len) { return p >= 0 && len >= 0 && len <= g_total - p; }

/* A BinaryArray at p with elements of es bytes: header word read (getInt64, BinaryArray.pointTo
 * :69-78), numElements >= 0, the null bitmap and the whole element range inside the batch
 * (copyToUnsafe :2451-2455).  Returns numElements, or -1 (and FO_ERR_OOB). */
static int64_t fo_array_ok(int64_t p, int32_t es) {
  if (!fo_span_ok(p, 8)) { g_flags |= FO_ERR_OOB; return -1; }
  int64_t m = (int32_t)fo_get_i64(g_rows + p);
  if (m < 0 || !fo_span_ok(p, 8 + fo_bitmap_bytes(m) + m * (int64_t)es)) {
    g_flags |= FO_ERR_OOB;
    return -1;
  }
  return m;
}

static int32_t fo_elem_size(const fury_field* f) {
  int32_t w = fo_type_width(f->type_id);
  return w < 0 ? 8 : w;
}

/* The checked position of a non-null non-scalar value of field f whose slot word is oas, in a
 * container starting at cont; *count = LIST / MAP elements.  -1: decode as null (the error is
 * recorded). */
static int64_t fo_value_pos(const fury_field* f, int64_t cont, int64_t oas, int64_t* count) {
  int64_t pos = cont + (int32_t)(oas >> 32);
  int32_t size = (int32_t)oas;
  *count = 0;
  switch (f->type_id) {
    case FURY_TYPE_STRING: case FURY_TYPE_BINARY:
      if (!fo_span_ok(pos, size)) { g_flags |= FO_ERR_OOB; return -1; }
      *count = size;
      return pos;
    case FURY_TYPE_DECIMAL:
      if (!fo_span_ok(pos, 16)) { g_flags |= FO_ERR_OOB; return -1; }
      return pos;
    case FURY_TYPE_STRUCT:
      if (!fo_span_ok(pos, fo_bitmap_bytes(f->num_children) + 8LL * f->num_children)) {
        g_flags |= FO_ERR_OOB;
        return -1;
      }
      return pos;
    case FURY_TYPE_LIST: {
      int64_t m = fo_array_ok(pos, fo_elem_size(&f->children[0]));
      if (m < 0) return -1;
      *count = m;
      return pos;
    }
    case FURY_TYPE_MAP: {        /* BinaryMap.pointTo :62-77 */
      if (!fo_span_ok(pos, 8)) { g_flags |= FO_ERR_OOB; return -1; }
      int64_t kb = (int32_t)fo_get_i64(g_rows + pos);
      int64_t nk = kb >= 0 ? fo_array_ok(pos + 8, fo_elem_size(&f->children[0])) : -1;
      int64_t nv = kb >= 0 ? fo_array_ok(pos + 8 + kb, fo_elem_size(&f->children[1])) : -1;
      if (kb < 0) g_flags |= FO_ERR_OOB;
      if (nk < 0 || nv < 0) return -1;
      if (nk != nv) { g_flags |= FO_ERR_MAP; return -1; }
      *count = nk;
      return pos;
    }
    default:
      return pos;
  }
}

typedef struct fo_view {          /* a BinaryRow or BinaryArray pointed at bytes */
  const uint8_t* base;
  int64_t header;                 /* bytes before the slots                   */
  int32_t bytes_before_bitmap;
  int32_t elem_size;              /* 8 for rows                               */
} fo_view;

static int fo_view_is_null(const fo_view* v, int64_t ordinal) {   /* BitUtils.isSet */
  return (v->base[v->bytes_before_bitmap + (ordinal >> 3)] >> (ordinal & 7)) & 1;
}
static const uint8_t* fo_view_slot(const fo_view* v, int64_t ordinal) {
  return v->base + v->header + ordinal * v->elem_size;
}

static void fo_set_valid(fury_column* c, int64_t i, int valid) {
  if (!c->validity) return;
  if (valid) c->validity[i >> 3] |= (uint8_t)(1u << (i & 7));
  else c->validity[i >> 3] &= (uint8_t)~(1u << (i & 7));
}

/* cursor per column node for appended outputs */
typedef struct fo_cursor {
  int64_t* pos;     /* array of cursors, indexed by node id */
  int32_t next_id;
} fo_cursor;

static int32_t fo_node_count(const fury_field* f) {
  int32_t n = 1;
  for (int i = 0; i < f->num_children; i++) n += fo_node_count(&f->children[i]);
  return n;
}

static void fo_read_value(const fo_view* v, int64_t ordinal, const fury_field* f,
                          fury_column* c, int64_t out_i, int64_t* cur, int32_t node);
static void fo_null_entry(const fury_field* f, fury_column* c, int64_t out_i, int64_t* cur,
                          int32_t node);

/* The n elements of a checked BinaryArray at batch position p (BinaryArray.pointTo :69-78). */
static void fo_read_array(int64_t p, int64_t n, const fury_field* elem, fury_column* child,
                          int64_t* cur, int32_t child_node, int32_t list_node) {
  fo_view av;
  av.base = g_rows + p;
  av.bytes_before_bitmap = 8;
  av.header = 8 + fo_bitmap_bytes(n);
  av.elem_size = fo_elem_size(elem);
  int64_t start = cur[list_node];
  for (int64_t j = 0; j < n; j++) fo_read_value(&av, j, elem, child, start + j, cur, child_node);
  cur[list_node] = start + n;
}

/* A null entry out_i of node `node` (ArrowWriter appendNull, FMT/vectorized/ArrowWriter.java:
 * 205-215 and the writers' appendNull): validity 0, values zeroed, a zero-length string / list /
 * map, and for a struct one null entry in EVERY child, recursively (StructWriter.appendNull
 * :577-584 calls each child writer's appendNull). */
static void fo_null_entry(const fury_field* f, fury_column* c, int64_t out_i, int64_t* cur,
                          int32_t node) {
  fo_set_valid(c, out_i, 0);
  const int32_t w = fo_type_width(f->type_id);
  switch (f->type_id) {
    case FURY_TYPE_BOOL:
      if (c->values) ((uint8_t*)c->values)[out_i >> 3] &= (uint8_t)~(1u << (out_i & 7));
      return;
    case FURY_TYPE_DECIMAL:
      if (c->values) memset((uint8_t*)c->values + out_i * 16, 0, 16);
      return;
    case FURY_TYPE_STRING: case FURY_TYPE_BINARY: case FURY_TYPE_LIST: case FURY_TYPE_MAP:
      if (c->offsets) {
        c->offsets[out_i] = (int32_t)cur[node];
        c->offsets[out_i + 1] = (int32_t)cur[node];
      }
      return;
    case FURY_TYPE_STRUCT: {
      int32_t child_node = node + 1;
      for (int k = 0; k < f->num_children; k++) {
        fo_null_entry(&f->children[k], &c->child[k], out_i, cur, child_node);
        child_node += fo_node_count(&f->children[k]);
      }
      return;
    }
    default:
      if (w > 0 && c->values) memset((uint8_t*)c->values + out_i * w, 0, (size_t)w);
      return;
  }
}

/* Entry `ordinal` of the checked container v (its null bit and slot lie inside it). */
static void fo_read_value(const fo_view* v, int64_t ordinal, const fury_field* f,
                          fury_column* c, int64_t out_i, int64_t* cur, int32_t node) {
  int is_null = fo_view_is_null(v, ordinal);
  int32_t width = fo_type_width(f->type_id);
  const uint8_t* slot = fo_view_slot(v, ordinal);
  if (width > 0) {
    fo_set_valid(c, out_i, !is_null);
    if (f->type_id == FURY_TYPE_BOOL) {      /* getBoolean: byte != 0 */
      uint8_t* bits = (uint8_t*)c->values;
      int bit = !is_null && slot[0] != 0;
      if (!bits) return;
      if (bit) bits[out_i >> 3] |= (uint8_t)(1u << (out_i & 7));
      else bits[out_i >> 3] &= (uint8_t)~(1u << (out_i & 7));
      return;
    }
    if (!c->values) return;
    uint8_t* dst = (uint8_t*)c->values + out_i * width;
    if (is_null) memset(dst, 0, (size_t)width);
    else memcpy(dst, slot, (size_t)width);
    return;
  }
  int64_t count = 0;
  int64_t pos = is_null ? -1 : fo_value_pos(f, v->base - g_rows, fo_get_i64(slot), &count);
  if (pos < 0) {                              /* null, or decoded as null after a failed check */
    fo_null_entry(f, c, out_i, cur, node);
    return;
  }
  fo_set_valid(c, out_i, 1);
  switch (f->type_id) {
    case FURY_TYPE_STRING: case FURY_TYPE_BINARY: {   /* getBinary :118-131 */
      int64_t start = cur[node];
      if (c->values) memcpy((uint8_t*)c->values + start, g_rows + pos, (size_t)count);
      if (c->offsets) {
        c->offsets[out_i] = (int32_t)start;
        c->offsets[out_i + 1] = (int32_t)(start + count);
      }
      cur[node] = start + count;
      return;
    }
    case FURY_TYPE_DECIMAL:
      if (c->values) memcpy((uint8_t*)c->values + out_i * 16, g_rows + pos, 16);
      return;
    case FURY_TYPE_LIST:                      /* getArray :168-178 */
      if (c->offsets) c->offsets[out_i] = (int32_t)cur[node];
      fo_read_array(pos, count, &f->children[0], c->child, cur, node + 1, node);
      if (c->offsets) c->offsets[out_i + 1] = (int32_t)cur[node];
      return;
    case FURY_TYPE_STRUCT: {                  /* getStruct :148-166 */
      /* child columns are row-aligned with the parent (Arrow struct) */
      int32_t child_node = node + 1;
      fo_view rv;
      rv.base = g_rows + pos;
      rv.bytes_before_bitmap = 0;
      rv.header = fo_bitmap_bytes(f->num_children);
      rv.elem_size = 8;
      for (int k = 0; k < f->num_children; k++) {
        fo_read_value(&rv, k, &f->children[k], &c->child[k], out_i, cur, child_node);
        child_node += fo_node_count(&f->children[k]);
      }
      return;
    }
    case FURY_TYPE_MAP: {                     /* getMap + BinaryMap.pointTo :62-77 */
      int32_t key_node = node + 1;
      int32_t val_node = key_node + fo_node_count(&f->children[0]);
      if (c->offsets) c->offsets[out_i] = (int32_t)cur[node];
      int64_t key_bytes = (int32_t)fo_get_i64(g_rows + pos);
      int64_t saved = cur[node];
      fo_read_array(pos + 8, count, &f->children[0], &c->child[0], cur, key_node, node);
      cur[node] = saved;
      fo_read_array(pos + 8 + key_bytes, count, &f->children[1], &c->child[1], cur, val_node, node);
      if (c->offsets) c->offsets[out_i + 1] = (int32_t)cur[node];
      return;
    }
    default:
      g_flags |= FO_ERR_OOB;
      g_err = FURY_ERR_UNSUPPORTED;
      return;
  }
}

/* ------------------------------------------------------------------------------------------
 * The device's two-phase nested decode (fury_decode_prepare, then fury_decode_execute) reports
 * the errors of its COUNT walk first: a walk of each row over the nodes that hold or contain a
 * counted slot (LIST / MAP elements, STRING / BINARY bytes -- walk.hip TNode.walk), with the same
 * container checks and an item budget of 2 x the row's bytes + 64 per top-level field of a row
 * (a row the encoder wrote holds every item in its own bytes; a corrupted row whose slots alias
 * other bytes would make the walk grow with the product of the aliased counts; per field since
 * round 6, when the device walks a wide bean's top-level fields in groups).  fo_count_walk restates that walk exactly
 * (walk.hip walk_row / wvalue / wcharge) so a test can predict which error the prepare reports;
 * FO_ERR_BUDGET is the device's own limit, not a reference exception.
 * ---------------------------------------------------------------------------------------- */
static int fo_walks(const fury_field* f) {
  if (f->type_id == FURY_TYPE_STRING || f->type_id == FURY_TYPE_BINARY ||
      f->type_id == FURY_TYPE_LIST || f->type_id == FURY_TYPE_MAP)
    return 1;
  for (int i = 0; i < f->num_children; i++)
    if (fo_walks(&f->children[i])) return 1;
  return 0;
}

static _Thread_local int64_t g_left;  /* the field's remaining item budget (-1: spent) */

static int fo_charge(const fury_field* f, int valid, int64_t m) {
  int64_t items = f->type_id == FURY_TYPE_MAP ? 2 * m
                  : (f->type_id == FURY_TYPE_STRUCT && !valid) ? 0 : m;
  int64_t left = g_left - items;
  int64_t was = g_left;
  g_left = left > -1 ? left : -1;
  if (left >= 0) return 1;
  if (was >= 0) g_flags |= FO_ERR_BUDGET;
  return 0;
}

static void fo_cwalk(const fury_field* f, int nul, int64_t oas, int64_t cont) {
  int64_t count = 0;
  int64_t pos = nul ? -1 : fo_value_pos(f, cont, oas, &count);
  int valid = pos >= 0;
  int ty = f->type_id;
  int strc = ty == FURY_TYPE_STRUCT;
  if (!strc && ty != FURY_TYPE_LIST && ty != FURY_TYPE_MAP) return;
  int64_t m = strc ? (valid ? f->num_children : 0) : count;
  if (!fo_charge(f, valid, m)) m = 0;
  int64_t hb = fo_bitmap_bytes(strc ? f->num_children : m);
  int sides = ty == FURY_TYPE_MAP ? 2 : 1;
  for (int sd = 0; sd < sides; sd++) {
    int64_t arr = pos;
    if (ty == FURY_TYPE_MAP && m > 0)
      arr = sd == 0 ? pos + 8 : pos + 8 + (int32_t)fo_get_i64(g_rows + pos);
    if (!strc && !fo_walks(&f->children[sd])) continue;
    for (int64_t j = 0; j < m; j++) {
      const fury_field* cf = strc ? &f->children[j] : &f->children[sd];
      if (fo_type_width(cf->type_id) > 0 || !fo_walks(cf)) continue;
      int64_t cbm = strc ? pos : arr + 8;
      int64_t cslot = strc ? pos + hb + 8 * j : arr + 8 + hb + 8 * j;
      int cnul = (g_rows[cbm + (j >> 3)] >> (j & 7)) & 1;
      fo_cwalk(cf, cnul, fo_get_i64(g_rows + cslot), strc ? pos : arr);
    }
  }
}

int32_t fo_count_walk(const fury_field* fields, int32_t nfields, const uint8_t* rows,
                      const int64_t* row_offsets, int64_t nrows) {
  g_rows = rows;
  g_total = row_offsets[nrows];
  g_flags = 0;
  int64_t hb = fo_bitmap_bytes(nfields);
  for (int64_t i = 0; i < nrows; i++) {
    int64_t base = row_offsets[i];
    int64_t budget = 2 * (row_offsets[i + 1] - base) + 64;
    if (budget > (1 << 30)) budget = 1 << 30;
    int rowok = fo_span_ok(base, hb + 8LL * nfields);
    if (!rowok) g_flags |= FO_ERR_OOB;
    for (int k = 0; k < nfields; k++) {
      if (fo_type_width(fields[k].type_id) > 0 || !fo_walks(&fields[k])) continue;
      g_left = budget;
      int nul = !rowok || ((rows[base + (k >> 3)] >> (k & 7)) & 1);
      fo_cwalk(&fields[k], nul, rowok ? fo_get_i64(rows + base + hb + 8 * k) : 0, base);
    }
  }
  return g_flags;
}

/* Decode rows [row_offsets[i], row_offsets[i+1]) (or i * fixed_size when row_offsets is NULL)
 * into columns.  Variable-length outputs must be large enough: callers size them from a first
 * pass over a column tree with every buffer NULL (nothing is written), whose final cursors
 * (cur_out, one per schema node in depth-first order) are the exact sizes -- STRING / BINARY:
 * payload bytes; LIST / MAP: child entries. */
int fo_decode_batch_cur(const fury_field* fields, int32_t nfields, const uint8_t* rows,
                        const int64_t* row_offsets, int64_t nrows, fury_column* cols,
                        int64_t* cur_out);
int fo_decode_batch(const fury_field* fields, int32_t nfields, const uint8_t* rows,
                    const int64_t* row_offsets, int64_t nrows, fury_column* cols) {
  return fo_decode_batch_cur(fields, nfields, rows, row_offsets, nrows, cols, NULL);
}

int fo_decode_batch_cur(const fury_field* fields, int32_t nfields, const uint8_t* rows,
                        const int64_t* row_offsets, int64_t nrows, fury_column* cols,
                        int64_t* cur_out) {
  g_err = 0;
  int32_t nodes = 0;
  for (int k = 0; k < nfields; k++) nodes += fo_node_count(&fields[k]);
  int64_t* cur = (int64_t*)calloc((size_t)(nodes + 1), sizeof(int64_t));
  if (!cur) return FURY_ERR_ENCODER;
  int32_t fixed = fo_bitmap_bytes(nfields) + 8 * nfields;
  g_rows = rows;
  g_total = row_offsets ? row_offsets[nrows] : nrows * (int64_t)fixed;
  g_flags = 0;
  for (int64_t i = 0; i < nrows; i++) {
    fo_view rv;
    int64_t base = row_offsets ? row_offsets[i] : i * (int64_t)fixed;
    rv.base = rows + base;
    rv.bytes_before_bitmap = 0;
    rv.header = fo_bitmap_bytes(nfields);
    rv.elem_size = 8;
    /* the row's null bitmap + slots inside the batch (getInt64 / isNullAt of every field) */
    int rowok = fo_span_ok(base, fixed);
    if (!rowok) g_flags |= FO_ERR_OOB;
    int32_t node = 0;
    for (int k = 0; k < nfields; k++) {
      if (rowok) fo_read_value(&rv, k, &fields[k], &cols[k], i, cur, node);
      else fo_null_entry(&fields[k], &cols[k], i, cur, node);
      node += fo_node_count(&fields[k]);
    }
  }
  if (cur_out) memcpy(cur_out, cur, (size_t)nodes * sizeof(int64_t));
  free(cur);
  if (g_err) return g_err;
  return (g_flags & FO_ERR_OOB) ? FURY_ERR_OUT_OF_BOUNDS
         : (g_flags & FO_ERR_MAP) ? FURY_ERR_UNSUPPORTED : 0;
}

/* FO_ERR_* bits of the last fo_decode_batch(_cur) / fo_count_walk call. */
int32_t fo_last_flags(void) { return g_flags; }

/* Convenience used by the CPU baseline: fixed-width schemas only, tight loop over the same
 * restated writer (toRow semantics, rows written straight into `out` which the caller zeroed).
 * Returns bytes written. */
int64_t fo_encode_fixed_inplace(const fury_field* fields, int32_t nfields, const fury_column* cols,
                                int64_t nrows, uint8_t* out) {
  g_err = 0;
  int32_t fixed = fo_bitmap_bytes(nfields) + 8 * nfields;
  fo_buf b;
  b.data = out;
  b.size = nrows * (int64_t)fixed;
  b.writer_index = 0;
  fo_writer w;
  fo_row_writer_init(&w, &b, nfields);
  for (int64_t i = 0; i < nrows; i++) {
    fo_row_writer_reset(&w);
    fo_to_row(&w, fields, nfields, cols, i);
  }
  return b.writer_index;
}
