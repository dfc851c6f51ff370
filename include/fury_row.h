/*
 * fury_row.h — C ABI of the MI355X-native Fury row-format codec.
 *
 * This is the drop-in boundary for the hot path named by BASELINE.json `north_star`:
 * java/fury-format's row encode/decode and row -> Arrow-column conversion.  Java objects
 * cannot cross onto the device, so the boundary is batches of Arrow-style columns <-> batches
 * of Fury rows; every row's bytes are identical to what the reference writes for the same
 * field values (see DESIGN.md "Parity").
 *
 * Reference interfaces each entry point replaces (paths relative to the reference root,
 * FMT = java/fury-format/src/main/java/org/apache/fury/format):
 *
 *   fury_schema_create      TypeInference.inferSchema + BinaryRowWriter ctor layout
 *                           (FMT/type/TypeInference.java:64-76,136-238,
 *                            FMT/row/binary/writer/BinaryRowWriter.java:46-52)
 *   fury_schema_hash        DataTypes.computeSchemaHash (FMT/type/DataTypes.java:499-544)
 *   fury_type_width         DataTypes.getTypeWidth (FMT/type/DataTypes.java:68-133,225-227)
 *   fury_row_measure        the writerIndex growth of generated toRow
 *                           (FMT/encoder/RowEncoderBuilder.java:154-179) — row sizes + scan
 *   fury_row_encode         RowEncoder.toRow over a batch: generated toRow + BinaryRowWriter /
 *                           BinaryWriter / BinaryArrayWriter (FMT/encoder/Encoders.java:88-93,
 *                           FMT/encoder/BaseBinaryEncoderBuilder.java:138-453,
 *                           FMT/row/binary/writer/BinaryWriter.java:106-194,
 *                           FMT/row/binary/writer/BinaryRowWriter.java:76-124,
 *                           FMT/row/binary/writer/BinaryArrayWriter.java:77-118)
 *   fury_row_encode_measured both in one call (toRow into a growable buffer, Encoders.java:88-93)
 *   fury_row_decode_measure the Arrow offsets fromRow/ArrowWriter would produce
 *   fury_row_decode         RowEncoder.fromRow over a batch: BinaryRow getters
 *                           (FMT/encoder/RowEncoderBuilder.java:185-217,
 *                            FMT/row/binary/UnsafeTrait.java:68-197,
 *                            FMT/row/binary/BinaryArray.java:69-78,157-197)
 *   fury_rows_to_arrow      ArrowWriter.write(row)* + finishAsRecordBatch
 *                           (FMT/vectorized/ArrowWriter.java:74-99,205-225,519-540)
 *   fury_arrow_append       ArrowWriter.write(row) appending at rowCount until finish() / reset()
 *                           (FMT/vectorized/ArrowWriter.java:74-99)
 *   fury_frame_rows /       RowEncoder.encode(MemoryBuffer, T) / decode(MemoryBuffer) stream
 *   fury_unframe_rows       framing [int32 len][int64 schemaHash][row]
 *                           (FMT/encoder/Encoders.java:165-182,201-213)
 *
 * Conventions
 *   - Every function returns an int status (FURY_OK == 0).  On failure a message is kept per
 *     thread and can be read with fury_last_error().  Status codes map 1:1 onto the
 *     reference's exception types (see fury_status).
 *   - Pointers passed to the fury_row_* / fury_rows_* / fury_*frame* functions are DEVICE
 *     pointers on the calling thread's current HIP device; `stream` is a hipStream_t (NULL =
 *     the legacy default stream).  Calls are asynchronous on `stream` unless documented.
 *   - Arrow layout: validity bitmaps are LSB-first with bit = 1 meaning VALID (Arrow); the row
 *     bitmap inside a Fury row is LSB-first with bit = 1 meaning NULL (BitUtils.set,
 *     fury-core memory/BitUtils.java:36-43,175-177).  All integers little-endian, floats as raw
 *     bits (MemoryBuffer.putFloat64 = doubleToRawLongBits).
 *   - Canonical bytes are the fresh-buffer bytes of RowEncoder.toRow(obj) (Encoders.java:88-93):
 *     a null field's slot is 0.  See DESIGN.md "Null slots" for RowEncoder.encode(obj)'s reused
 *     buffer.
 */
#ifndef FURY_ROW_H_
#define FURY_ROW_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FURY_ROW_ABI_VERSION 1

/* Status codes; the reference exception each one stands for is named. */
typedef enum fury_status {
  FURY_OK = 0,
  FURY_ERR_INVALID_ARGUMENT = 1,       /* IllegalArgumentException / checkArgument          */
  FURY_ERR_UNSUPPORTED = 2,            /* UnsupportedOperationException
                                          (TypeInference.java:233-237, BinaryArrayWriter.java:99-101) */
  FURY_ERR_CLASS_NOT_COMPATIBLE = 3,   /* ClassNotCompatibleException (Encoders.java:170-178) */
  FURY_ERR_OUT_OF_BOUNDS = 4,          /* IndexOutOfBoundsException (MemoryBuffer bounds)    */
  FURY_ERR_ENCODER = 5,                /* EncoderException (Encoders.java:215-218)          */
  FURY_ERR_DEVICE = 6,                 /* HIP runtime failure (no reference equivalent)     */
  FURY_ERR_CAPACITY = 7                /* output buffer too small for measured bytes        */
} fury_status;

/* Type ids = org.apache.fury.format.type.ArrowType ids (FMT/type/ArrowType.java:25-148);
 * they are also the ids hashed by DataTypes.computeSchemaHash. */
typedef enum fury_type_id {
  FURY_TYPE_BOOL = 1,
  FURY_TYPE_INT8 = 3,
  FURY_TYPE_INT16 = 5,
  FURY_TYPE_INT32 = 7,
  FURY_TYPE_INT64 = 9,
  FURY_TYPE_FLOAT32 = 11,
  FURY_TYPE_FLOAT64 = 12,
  FURY_TYPE_STRING = 13,   /* Arrow utf8  */
  FURY_TYPE_BINARY = 14,
  FURY_TYPE_DATE32 = 16,
  FURY_TYPE_TIMESTAMP = 18, /* microseconds */
  FURY_TYPE_DECIMAL = 23,  /* decimal128, 16 bytes */
  FURY_TYPE_LIST = 25,
  FURY_TYPE_STRUCT = 26,
  FURY_TYPE_MAP = 30
} fury_type_id;

/* A schema field (a node of org.apache.arrow.vector.types.pojo.Field as built by
 * TypeInference.inferField).  Fields are given in slot order, i.e. already sorted the way
 * Descriptor orders bean fields (lexicographic Java field name, Descriptor.java:324-332);
 * fury_sort_bean_fields() performs that ordering. */
typedef struct fury_field {
  const char* name;
  int32_t type_id;                  /* fury_type_id                                    */
  int32_t nullable;                 /* FieldType.nullable                              */
  int32_t num_children;             /* LIST: 1 (element), STRUCT: n, MAP: 2 (key, value) */
  const struct fury_field* children;
} fury_field;

typedef struct fury_schema fury_schema; /* opaque, immutable after creation, thread-safe */

/* Arrow-style column (one per top-level field, in schema order).  Array offset is 0.
 *   fixed width : values = n * width bytes (BOOL: bit-packed, Arrow), validity optional
 *   STRING/BINARY: offsets = n+1 int32, values = payload bytes
 *   DECIMAL     : values = n * 16 bytes (decimal128 little-endian)
 *   LIST        : offsets = n+1 int32 element offsets, child = element column (flattened)
 *   STRUCT      : child = array of the struct's field columns (entry-aligned with the parent)
 *   MAP         : offsets = n+1 int32 entry offsets, child = [keys column, values column]
 * validity: encode input NULL = all valid; decode output NULL = do not write validity.
 * capacity: decode output only — bytes available in `values` (STRING/BINARY payload; for a LIST,
 *   the child column's capacity bounds its element values).  Decode never writes past it.
 * Decode output bitmaps (validity, BOOL values) are written as 32-bit words: 4-byte aligned,
 *   padded to a multiple of 4 bytes. */
typedef struct fury_column {
  void* values;
  uint8_t* validity;
  int32_t* offsets;
  int64_t capacity;
  struct fury_column* child;
} fury_column;

/* Describes the computed layout of a schema (BinaryRowWriter ctor, BinaryRowWriter.java:46-52). */
typedef struct fury_schema_info {
  int32_t num_fields;
  int32_t bitmap_bytes;   /* BitUtils.calculateBitmapWidthInBytes(numFields) */
  int32_t fixed_size;     /* bitmap_bytes + 8 * num_fields                   */
  int32_t is_fixed;       /* 1 when every field is fixed width: rows are fixed_size bytes */
  int64_t schema_hash;    /* DataTypes.computeSchemaHash                     */
} fury_schema_info;

/* ---- version / errors ---------------------------------------------------------------- */
int32_t fury_abi_version(void);
/* Copies the calling thread's last error message (NUL-terminated, truncated to len). */
size_t fury_last_error(char* buf, size_t len);

/* ---- schema (host) --------------------------------------------------------------------- */
/* DataTypes.getTypeWidth: byte width of a fixed-width type, -1 for variable-length types. */
int32_t fury_type_width(int32_t type_id);
/* Sort `n` field indices by Java field name the way Descriptor does (String.compareTo on
 * UTF-16 code units); writes the permutation to order[0..n). */
int fury_sort_bean_fields(const char* const* java_names, int32_t n, int32_t* order);
/* StringUtils.lowerCamelToLowerUnderscore (fury-core util/StringUtils.java:252-271).
 * Returns the length written (excluding NUL); out must hold 2*strlen(in)+1 bytes. */
int32_t fury_lower_camel_to_lower_underscore(const char* in, char* out, size_t out_len);
/* Any number of fields; nested STRUCT / LIST / MAP up to 64 levels and 4096 nodes (a deeper or
 * larger schema is created, and its encode / decode calls return FURY_ERR_UNSUPPORTED).  Every
 * row of a schema within those limits encodes and decodes on the device, whatever its size. */
int fury_schema_create(const fury_field* fields, int32_t num_fields, fury_schema** out);
void fury_schema_destroy(fury_schema* schema);
int fury_schema_get_info(const fury_schema* schema, fury_schema_info* info);

/* ---- device batch codec ---------------------------------------------------------------- */
/* Row sizes and their exclusive scan: row_offsets[0..nrows] (int64, device); row i occupies
 * [row_offsets[i], row_offsets[i+1]) and row_offsets[nrows] is the batch's byte total.
 * For is_fixed schemas this is optional (rows sit at i * fixed_size). */
int fury_row_measure(const fury_schema* schema, const fury_column* columns, int64_t nrows,
                     int64_t* row_offsets, void* stream);
/* Encode nrows rows into `rows` (device, 8-byte aligned, row_offsets[nrows] bytes, or
 * nrows * fixed_size when row_offsets is NULL and the schema is fixed). */
int fury_row_encode(const fury_schema* schema, const fury_column* columns, int64_t nrows,
                    const int64_t* row_offsets, void* rows, void* stream);
/* Measure + encode in one call with no host synchronisation — the batch form of toRow writing
 * into a growable buffer: writes row_offsets[0..nrows] exactly as fury_row_measure and the rows
 * into `rows`
 * (capacity bytes).  Bytes at or past `capacity` are never written: when row_offsets[nrows] >
 * capacity, grow the buffer and call again.  Fixed schemas know their size up front and return
 * FURY_ERR_CAPACITY instead (row_offsets may be NULL for them). */
int fury_row_encode_measured(const fury_schema* schema, const fury_column* columns, int64_t nrows,
                             int64_t* row_offsets, void* rows, int64_t capacity, void* stream);
/* Decode pass 1 for variable-length outputs: writes columns[i].offsets (STRING/BINARY/LIST)
 * and, for LIST, nothing else.  The caller reads offsets[nrows] to size values/child buffers. */
int fury_row_decode_measure(const fury_schema* schema, const void* rows,
                            const int64_t* row_offsets, int64_t nrows, fury_column* columns,
                            void* stream);
/* Decode rows into columns (RowEncoder.fromRow semantics: a null field leaves 0 bytes and,
 * when validity != NULL, a cleared validity bit).  One device pass: the STRING/BINARY/LIST
 * offsets are computed here (fury_row_decode_measure is only needed to size the buffers); when
 * offsets[nrows] exceeds a column's capacity the payload past the capacity is not written —
 * grow the buffer and decode again.  Malformed rows are reported asynchronously, on `stream`
 * (fury_device_status below).  Nested schemas, and flat ones with more than 256 fields of which
 * some are variable-length (the generic engine), decode through fury_decode_prepare /
 * fury_decode_execute instead: these calls (and fury_row_decode_measure) return
 * FURY_ERR_INVALID_ARGUMENT for them, naming the plan API. */
int fury_row_decode(const fury_schema* schema, const void* rows, const int64_t* row_offsets,
                    int64_t nrows, fury_column* columns, void* stream);
/* ArrowWriter.write(row) for every row + finishAsRecordBatch: as fury_row_decode but every
 * column's validity is required (Arrow vectors always carry one) and null lists become
 * zero-length entries (ListVector fillHoles, ArrowWriter.java:539,223-225). */
int fury_rows_to_arrow(const fury_schema* schema, const void* rows, const int64_t* row_offsets,
                       int64_t nrows, fury_column* columns, void* stream);

/* Appends the Arrow columns `src` (src_rows top-level entries, e.g. fury_rows_to_arrow /
 * fury_decode_execute output) at entry dst_rows of the columns `dst` -- ArrowWriter.write(row)
 * appending at rowCount until finish() / reset() (FMT/vectorized/ArrowWriter.java:74-99): values
 * and STRING/BINARY payloads are copied after the destination's, offsets rebased on its end
 * (offsets[dst_rows]), validity / BOOL bits shifted to its bit position, LIST / MAP child entries
 * appended after its child entries, STRUCT children entry-aligned.  Every node's destination
 * buffers must hold the combined entries (validity / BOOL bitmaps as 32-bit words: 4-byte aligned,
 * padded to a multiple of 4 bytes; offsets entries + 1); fury_column.capacity, when > 0, bounds a
 * node's values / payload bytes (FURY_ERR_CAPACITY).  Child offsets of `src` must start at 0.
 * Reads the destination's and source's end offsets from the device, so the call synchronises
 * `stream`; the copies themselves are one launch on it. */
int fury_arrow_append(const fury_schema* schema, fury_column* dst, int64_t dst_rows,
                      const fury_column* src, int64_t src_rows, void* stream);

/* ---- ArrayEncoder / MapEncoder batches (Encoders.arrayEncoder / mapEncoder,
 *      FMT/encoder/Encoders.java:230-600, ArrayEncoderBuilder.java:118-140,
 *      MapEncoderBuilder.java:152-208) ----------------------------------------------------- */
/* A collection schema: its batch entries are top-level BinaryArrays (`field` of type LIST:
 * ArrayEncoder.toArray(obj)) or BinaryMaps (`field` of type MAP: [int64 keyArrayBytes][key
 * BinaryArray][value BinaryArray], MapEncoder.toMap(obj)) instead of rows.  The batch entry points
 * take it unchanged: fury_row_measure / fury_row_encode / fury_row_encode_measured write entry i
 * at row_offsets[i] (every entry a multiple of 8 bytes), fury_decode_prepare /
 * fury_decode_execute decode.  `columns` is ONE column, the collection column itself (LIST:
 * offsets + element child; MAP: offsets + child [keys, values]) with validity NULL: a collection
 * handed to toArray / toMap is never null.  schema_hash is 0 (these encoders carry no hash; their
 * encode(MemoryBuffer, T) frames [int32 size][bytes]), and the row framing entry points return
 * FURY_ERR_UNSUPPORTED for them. */
int fury_collection_schema_create(const fury_field* field, fury_schema** out);

/* ---- nested schemas: two-step decode --------------------------------------------------- */
/* Schemas with STRUCT / MAP / LIST-of-variable-length fields produce a TREE of Arrow columns whose
 * sizes depend on the data.  Nodes are the schema's fields at every level, numbered breadth-first:
 * top-level fields 0..n-1 first, then each node's children contiguously (LIST: element; STRUCT:
 * its fields; MAP: key, value).  fury_decode_prepare counts, for every node, the Arrow entries
 * (node_entries) and STRING/BINARY payload bytes (node_bytes) the batch produces and returns a
 * plan; the caller allocates every node's buffers (validity and BOOL value bitmaps ZEROED, offsets
 * entries+1, values entries*width / node_bytes / 16*entries) and runs fury_decode_execute on
 * the column tree (fury_column.child: LIST -> element column; STRUCT -> its field columns; MAP ->
 * [keys, values]).  Flat schemas may use it too.  Synchronises `stream` once (prepare). */
typedef struct fury_decode_plan fury_decode_plan;
int32_t fury_schema_num_nodes(const fury_schema* schema);
int fury_decode_prepare(const fury_schema* schema, const void* rows, const int64_t* row_offsets,
                        int64_t nrows, int64_t* node_entries, int64_t* node_bytes,
                        fury_decode_plan** plan, void* stream);
int fury_decode_execute(fury_decode_plan* plan, fury_column* columns, int32_t arrow, void* stream);
void fury_decode_plan_destroy(fury_decode_plan* plan);

/* ---- asynchronous device errors (no reference equivalent) ------------------------------- */
/* Decode kernels report what they find ASYNCHRONOUSLY: fury_row_decode,
 * fury_rows_to_arrow and fury_decode_execute return before their kernels run, so a malformed
 * batch is reported later --
 *   FURY_ERR_OUT_OF_BOUNDS  a variable-length value, array or map header outside the batch's row
 *                           bytes (MemoryBuffer's IndexOutOfBoundsException), or a nested row
 *                           whose slots alias other bytes so that its walk would visit more
 *                           items than twice its bytes (found by fury_decode_prepare);
 *   FURY_ERR_UNSUPPORTED    map key / value arrays of different lengths (BinaryMap.pointTo);
 *   FURY_ERR_DEVICE         a decoupled look-back that gave up waiting (by construction -- a
 *                           look-back computes a silent predecessor's aggregate itself -- never
 *                           raised on working hardware).
 * The report goes to the STREAM the call was launched on (the legacy null stream: per host
 * thread): fury_device_status(stream) synchronises that stream and returns it, and the next entry
 * point called on the same stream returns it before doing anything (without synchronising: it sees
 * the kernels that have finished).  Either clears it.  Calls on other streams never see it.  When
 * one is reported, every output of the failing call is invalid (the values that failed decode as
 * null; the rest may be incomplete).  fury_decode_prepare and the host-memory entry points
 * synchronise and report their own batch's errors directly.
 * Each stream that launched work holds one of 1024 error slots until it is released: call
 * fury_stream_release(stream) (it synchronises the stream and drops any unreported error) before
 * destroying a stream passed to this library; streams the library creates itself, and the
 * per-thread keys of the null stream / hipStreamPerThread, are released by the library.  With
 * every slot held, the next call on a new stream fails with FURY_ERR_DEVICE (slots are never
 * shared between streams). */
int fury_device_status(void* stream);
int fury_stream_release(void* stream);

/* ---- workspace (no reference equivalent) ------------------------------------------------- */
/* The library caches the device workspaces of its calls (scan scratch, decode plans, column
 * tables; at most 2 GB of idle blocks per process).  Releases every idle cached block of `device`
 * (after the work that last used it, so the call may wait for it) and trims the device's stream
 * memory pool.  An allocation that fails does the same by itself before it reports. */
int fury_trim_workspace(int32_t device);

/* ---- tuning (no reference equivalent) ---------------------------------------------------- */
/* Process-wide knobs for tests and A/B measurement (results are identical under every value,
 * except the diagnostic "walk_skip").
 * Key "lookback_help": 1 = every look-back of the variable-length decode computes a silent
 * predecessor tile's aggregate at once (the path a late-dispatched predecessor takes).
 * Key "unframe": 0 speculative parallel stream parse (a stream that does not verify -- a payload
 * spelling a plausible header -- is repaired in parallel; the sequential walk only reports
 * errors), 1 always the sequential walk.
 * Nested engines: "nested_decode" 2 row walk (default), 1 level engine (schemas past the walk's
 * limits -- 5 levels, 256 counted nodes -- use it by themselves), 3 row walk with the tile BFS past
 * its limits, 4 tile BFS ("bfs_threads" 64 / 128 / 256 / 512, "bfs_rows", "bfs_stage", "bfs_arena"
 * bytes, 0 = sized from the batch; fury_get_tuning "bfs_fallbacks" = batches whose tiles outgrew
 * the arena and went to the walk / level engine); nested encode is the row walk with an explicit-stack continuation
 * for deep schemas: "rowenc_rows" (128 / 256 / 512 threads per group), "rowenc_tile" (rows per group,
 * 0 = threads), "rowenc_img" (LDS image bytes); row-walk decode "walk_threads" /
 * "walk_threads_write" (128 / 256 / 512), "walk_stage" / "walk_stage_write" / "walk_pool" / "walk_out"
 * (LDS bytes), "walk_prefetch" (bit 0 write pass, bit 1 count pass), "walk_group_k" /
 * "walk_group_min" (a schema with more than walk_group_min counted nodes, default 16, walks its
 * top-level fields in groups of about walk_group_k counted nodes, default 8, a workgroup per tile
 * and group; 0 = one group); flat schemas of 17-256
 * fields: "var_wide" (1 wide tiles, default; 0 generic var tiles), "wide_engine" (the plan's engine
 * for them: 0 auto -- the row walk when the batch's average row exceeds "wide_walk_row" bytes,
 * default 896 --, 1 wide tiles, 2 row walk; "wide_enc_engine" the same for the encode, by the
 * columns' estimated row), "wide_threads" /
 * "wide_enc_threads" (256 / 512 / 1024); diagnostics "var_skip" (register-staged encode / decode phases
 * skipped: outputs WRONG, timing only),
 * "tree_debug" (phase clocks) and "walk_skip" (bitmask of write-pass phases skipped: outputs
 * WRONG, timing only).  Variable-length decode tile plan: "var_dec_cover" (percent of a tile's
 * row bytes the LDS stage must hold, default 95), "var_dec_rows" (forced tile rows, 0 = plan),
 * "var_dec_pipe" (0 one tile per workgroup, default; 1 / 2 persistent workgroups with two row
 * stages, the 3- and 6-column instances -- measured slower, kept for A/B).  Fixed-width encode:
 * "fixed_enc" (column loads per lane in flight: 2 = 16, default; 0 = 8; 3 = 32; 4 = 16 with 8
 * stores; 1 = 16-B pair loads).
 * Host path: "host_decode_inplace" (0 / 1).
 * fury_get_tuning only: "unframe_walks" = streams the walk parsed (wholly or from the first frame
 * the repair could not place), "unframe_repairs" = streams the parallel repair parsed,
 * "host_direct" = fury_row_encode_host / _decode_host calls that ran their kernels directly on
 * pinned host buffers (fixed-width and flat variable-length schemas, no staging),
 * "lookback_timeouts" = decoupled look-backs that gave up (must stay 0; synchronous device read),
 * "err_slots" = device error slots held by live streams (fury_stream_release),
 * "err_slots_quarantined" = slots of exited threads waiting for a device synchronisation,
 * "decode_budget_errors" = nested decodes refused by the item budget (a device limit),
 * "var_dec_rows_rejected" = forced "var_dec_rows" tiles whose images did not fit (planned tile used). */
int fury_set_tuning(const char* key, int32_t value);
int32_t fury_get_tuning(const char* key);

/* ---- measurement (no reference equivalent) ------------------------------------------------ */
/* Same-device streaming copy of `bytes` (a positive multiple of 16 KB) from src to dst (device,
 * 16-byte aligned) with 16-B non-temporal loads / stores, asynchronous on `stream`: the box's
 * achievable copy rate, which bench.py reports beside the codec's roofline fraction. */
int fury_hbm_copy(void* dst, const void* src, int64_t bytes, void* stream);

/* ---- framing (Encoders.java:201-213 / 165-182) ------------------------------------------ */
/* Writes the stream RowEncoder.encode(MemoryBuffer, T) produces for each row in turn:
 * [int32 len = 8 + rowSize][int64 schemaHash][row bytes].  frame_offsets (device, nrows+1)
 * receives where each frame starts; frame i starts at row_offsets[i] + 12 * i. */
int fury_frame_rows(const fury_schema* schema, const void* rows, const int64_t* row_offsets,
                    int64_t nrows, void* out, int64_t* frame_offsets, void* stream);
/* Parses such a stream back (RowEncoder.decode(MemoryBuffer) nrows times): writes
 * row_offsets[0..nrows] and the rows packed into `rows_out`, checking every schemaHash; a
 * mismatch returns FURY_ERR_CLASS_NOT_COMPATIBLE, a frame past the end FURY_ERR_OUT_OF_BOUNDS.
 * `stream_bytes` may start at any byte address.  Parallel on the device (speculative header scan
 * + verify, parallel repair when a payload spells a header).  Synchronises `stream`. */
int fury_unframe_rows(const fury_schema* schema, const void* stream_bytes, int64_t stream_len,
                      int64_t nrows, void* rows_out, int64_t* row_offsets, void* stream);

/* ---- host-memory batch path (the JNI boundary: DirectByteBuffer addresses) ---------------- */
/* The functions below take HOST pointers (a JVM's off-heap buffers) and run the device path
 * inside the call (synchronous): Encoders.bean(...).encode over a batch
 * (FMT/encoder/Encoders.java:185-213) and decode (:165-182), with the bytes crossing PCIe.
 * Fixed-width schemas whose buffers are ALL pinned (fury_host_alloc or fury_host_register) run
 * the kernel directly on host memory — loads and stores cross PCIe in both directions at once,
 * no HBM staging ("host_direct" counts these calls); otherwise they are staged through HBM
 * (chunked over three HIP streams).  Flat variable-length schemas on pinned buffers run direct
 * too (bitmaps through HBM), and so does the ENCODE of nested schemas (the column tree read and
 * the rows written in place); otherwise they are staged whole.  `device` is the
 * HIP device ordinal.  Buffers from fury_host_alloc (hipHostMalloc) run fastest; registering
 * ordinary 4 KB-page memory (fury_host_register, hipHostRegister) pins it in place but the GPU
 * then walks 4 KB translations (host path). */
int fury_host_alloc(int64_t bytes, void** out);  /* pinned host memory, freed by fury_host_free */
int fury_host_free(void* ptr);
int fury_host_register(void* ptr, int64_t bytes);
int fury_host_unregister(void* ptr);
/* Host columns (fury_column layout, host pointers) -> host rows.  Fixed-width: rows are
 * nrows * fixed_size bytes, row_offsets optional (filled with i * fixed_size when given).
 * Variable-length: row_offsets (host, nrows + 1) is required and filled.  *row_bytes = bytes
 * the rows need; FURY_ERR_CAPACITY (nothing written) when that exceeds rows_capacity. */
int fury_row_encode_host(const fury_schema* schema, const fury_column* columns, int64_t nrows,
                         void* rows, int64_t rows_capacity, int64_t* row_offsets,
                         int64_t* row_bytes, int32_t device);
/* Host rows -> host columns (fromRow semantics, like fury_row_decode).  Variable-length flat
 * schemas: STRING/BINARY payload capacity in fury_column.capacity, LIST element bytes in the
 * child's capacity (FURY_ERR_CAPACITY when short: staged calls size first and write nothing,
 * direct calls write nothing past a capacity and leave offsets[nrows] = the size needed); nested
 * schemas and flat ones with more than 256 fields of which some are variable-length:
 * FURY_ERR_UNSUPPORTED (their output sizes depend on the data: fury_decode_host_prepare /
 * fury_decode_host_execute below). */
int fury_row_decode_host(const fury_schema* schema, const void* rows, const int64_t* row_offsets,
                         int64_t nrows, fury_column* columns, int32_t device);

/* Host-memory decode of ANY schema (nested beans, maps, lists of structs / strings, collection
 * schemas), in the two steps of the device API (the output sizes depend on the data):
 * fury_decode_host_prepare stages the rows in HBM and returns every schema node's Arrow entries
 * and payload bytes (breadth-first node order, see fury_decode_prepare); the caller allocates the
 * host buffers from them (validity (entries + 7) / 8 bytes, offsets entries + 1 int32, values
 * entries * width / (entries + 7) / 8 for BOOL / node_bytes for STRING-BINARY (checked against
 * fury_column.capacity) / 16 * entries for DECIMAL) and calls fury_decode_host_execute, which
 * decodes in HBM and copies every buffer back (synchronous; with tuning "host_decode_inplace" the
 * values / offsets / payloads of pinned outputs are written in place -- slower).
 * The plan is freed by
 * fury_decode_plan_destroy.  Replaces generated fromRow + ArrowWriter for nested beans
 * (FMT/encoder/BaseBinaryEncoderBuilder.java:459-706, FMT/vectorized/ArrowWriter.java:519-640). */
int fury_decode_host_prepare(const fury_schema* schema, const void* rows, const int64_t* row_offsets,
                             int64_t nrows, int64_t* node_entries, int64_t* node_bytes,
                             fury_decode_plan** plan, int32_t device);
int fury_decode_host_execute(fury_decode_plan* plan, fury_column* columns);

/* ---- JNI core (java/.../GpuRowEncoder.java's native methods, minus the JNIEnv marshalling) ---
 * The exact arrays GpuRowEncoder builds, decoded in this library (fury_row_jni.cc only copies Java
 * arrays in and out and throws fury_jni_exception_class(status)).  Reference surface:
 * Encoders.bean(...) / RowEncoder (FMT/encoder/Encoders.java:60-219, RowEncoder.java:26-32).
 *   names / meta: flattenField in pre-order -- names[i] and meta[3 i .. 3 i + 2] = {typeId,
 *     nullable, numChildren} of node i (a MAP's children are key and value; `nodes` entries, the
 *     first `top` subtrees are the bean's fields in slot order);
 *   desc: describe() in pre-order -- 5 int64 per schema node {values address, validity address,
 *     offsets address, values capacity, numChildren} (host addresses); its child counts must
 *     match the schema's (FURY_ERR_INVALID_ARGUMENT otherwise);
 *   counts: 2 int64 per node (breadth-first, fury_decode_prepare order): entries, payload bytes;
 *   counts_len (the Java array's length) below 2 * fury_schema_num_nodes is
 *   FURY_ERR_INVALID_ARGUMENT, nothing written. */
const char* fury_jni_exception_class(int status);   /* Java class name of a status, NULL for OK */
int fury_jni_schema_create(const char* const* names, const int32_t* meta, int32_t nodes,
                           int32_t top, fury_schema** out);
int fury_jni_encode_host(const fury_schema* schema, const int64_t* desc, int64_t desc_len,
                         int64_t nrows, void* rows, int64_t rows_capacity, int64_t* row_offsets,
                         int64_t* row_bytes, int32_t device);
int fury_jni_decode_host(const fury_schema* schema, const void* rows, const int64_t* row_offsets,
                         int64_t nrows, const int64_t* desc, int64_t desc_len, int32_t device);
int fury_jni_decode_host_prepare(const fury_schema* schema, const void* rows,
                                 const int64_t* row_offsets, int64_t nrows, int64_t* counts,
                                 int64_t counts_len, fury_decode_plan** plan, int32_t device);
int fury_jni_decode_host_execute(const fury_schema* schema, fury_decode_plan* plan,
                                 const int64_t* desc, int64_t desc_len);

/* ---- Arrow IPC (ArrowUtils.serializeRecordBatch, FMT/vectorized/ArrowUtils.java:63-72;
 *      ArrowSerializers stream writers, FMT/vectorized/ArrowSerializers.java:128-167) --------- */
/* Encapsulated IPC Schema message of the schema, in HOST memory:
 * [0xFFFFFFFF][int32 metadata size][flatbuffer Message<Schema>][padding to 8].  *len receives
 * the size; out == NULL only sets *len, a too small cap returns FURY_ERR_CAPACITY.  An IPC
 * stream is this message, then record batch messages, then the 8-byte end-of-stream marker
 * [0xFFFFFFFF][0x00000000] (ArrowStreamWriter.writeEndOfStream). */
int fury_arrow_ipc_schema(const fury_schema* schema, uint8_t* out, int64_t cap, int64_t* len);
/* Encapsulated IPC RecordBatch message of device columns (fury_rows_to_arrow output, or any
 * columns in that layout) written to DEVICE memory `out` (16-byte aligned): flatbuffer metadata,
 * then the body = every Arrow buffer in pre-order (validity, offsets, values; children after
 * their parent; a MAP's "entries" struct node in between), each padded to 64 bytes.  Null
 * counts are computed on the device from the validity bitmaps.  The lengths of variable-size
 * buffers are read back from the device offsets, so the call is synchronous on `stream`.
 * out == NULL only sets *len. */
int fury_arrow_ipc_record_batch(const fury_schema* schema, const fury_column* columns,
                                int64_t nrows, void* out, int64_t cap, int64_t* len, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FURY_ROW_H_ */
