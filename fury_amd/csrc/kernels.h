// kernels.h — launch interfaces between the C-ABI layer (capi.cpp) and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "internal.h"

namespace fury {

// The same pointer in the global address space: accesses through it are global_load /
// global_store, not flat (a flat access also counts against lgkmcnt, so every later LDS or scalar
// wait waits for it too).  Pointers loaded from argument blocks or tables are generic to the
// compiler.  Only for pointers into device / host memory, never LDS.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gl(T* p) {
  return (__attribute__((address_space(1))) T*)(p);
}
// Pointer casts that keep the operand's address space (global via gl(), or a generic pointer the
// compiler resolves, e.g. into LDS), for code instantiated once per address space.
template <class T, class U>
__device__ __forceinline__ __attribute__((address_space(1))) T* cast_as(__attribute__((address_space(1))) U* p) {
  return (__attribute__((address_space(1))) T*)(p);
}
template <class T, class U>
__device__ __forceinline__ T* cast_as(U* p) {
  return (T*)(p);
}

// Columns per fixed-tile launch: the pointer table travels in the kernel argument block
// (scalar-loaded, no per-call device upload).  Wider schemas upload it (FixedArgs.tab).
constexpr int kMaxFixedCols = 128;

// Per-column record.  Every member is naturally aligned inside an 8-byte-aligned record: the
// kernels index this table with a wave-uniform column number, which the compiler turns into
// scalar (SMEM) loads; an int8 side array produced a byte-offset SMEM base that gfx950 masks
// to dword alignment (observed as an aperture fault), so keep all members >= 4 bytes.
struct FixedCol {
  const uint8_t* values;
  uint8_t* validity;                  // encode: input (NULL = all valid); decode: output or NULL
  int32_t width;                      // 1, 2, 4, 8; 0 = BOOL (bit-packed)
  int32_t pad_;
};

// Schemas wider than kMaxFixedCols take their column table from device memory (uploaded per
// call, FixedArgs.tab) and run the general tile kernel with 64-row tiles up to kMaxWideFixedCols
// (a 64-row tile, bitmap + 8 B per field per row, within the 160 KB of LDS); wider ones run the
// column-block kernels (64 rows x 64 fields per workgroup, no field limit).
constexpr int kMaxWideFixedCols = 315;

struct FixedArgs {
  FixedCol col[kMaxFixedCols];
  const FixedCol* tab;                // device table for > kMaxFixedCols fields, else NULL
  int32_t ncols;
  int32_t bitmap_bytes;
  int32_t row_size;
  int32_t pad_;
  int64_t nrows;
};

// Host-direct mode of the calling thread (hostpath.cpp): plain instead of non-temporal accesses.
void set_thread_host_direct(bool on);
int launch_encode_fixed(const FixedArgs& a, uint8_t* rows, hipStream_t stream, bool fast);
int launch_decode_fixed(const FixedArgs& a, const uint8_t* rows, hipStream_t stream, bool fast);

// ---- variable-length schemas ----------------------------------------------------------------
constexpr int kMaxVarCols = 64;
// Wider schemas: column table in device memory (VarArgs.tab), LDS-DMA / ticketed kernels.
constexpr int kMaxWideVarCols = 256;

// One top-level field as seen by the var kernels.
struct VarCol {
  const uint8_t* values;     // fixed values / bytes payload / decimal values / list child values
  uint8_t* validity;         // field validity (Arrow bits) or NULL
  int32_t* offsets;          // bytes / list offsets (n + 1)
  uint8_t* elem_validity;    // list element validity or NULL
  int32_t kind;              // FieldKind
  int32_t width;             // fixed: 1/2/4/8, 0 = bool; list: element width (0 = bool elements)
  int32_t var_slot;          // index among var fields (decode measure scratch), -1 otherwise
  int32_t nullable;
  int64_t capacity;          // decode: payload bytes (STRING/BINARY) / child elements (LIST)
};

struct VarArgs {
  VarCol col[kMaxVarCols];
  const VarCol* tab;         // device table for > kMaxVarCols fields, else NULL
  const VarCol* htab;        // its host copy (launchers only; never read on the device)
  int32_t ncols;
  int32_t bitmap_bytes;
  int32_t fixed_size;
  int32_t nvar;
  int64_t nrows;
  int32_t tile_rows;         // rows per encode tile (encode_tile_rows)
  int32_t help_now;          // look-backs help a silent predecessor at once (test hook, tuning
                             // "lookback_help"); 0 in production
  int32_t skip;              // diagnostics (tuning "var_skip"): phases skipped, outputs WRONG
  int32_t dec_pipe;          // decode_var_reg: persistent workgroups, two row stages (var_dec_pipe)
  uint32_t* err;             // the launch stream's device error slot (device_error_word) or NULL
};

// Host-visible device error words: host-pinned, mapped memory, one slot of kErrWords 32-bit words
// PER STREAM (capi.cpp), that kernels set with system-scope STORES (no read-modify-write over
// PCIe) when they cannot produce a valid result:
//   [kErrLookBack]            a look-back that gave up (FURY_ERR_DEVICE)
//   [kErrBounds], [+2, +3]    a decode read that would leave the batch, and where (one 64-bit
//                             word: a row, or bit 63 | node << 40 | entry) (FURY_ERR_OUT_OF_BOUNDS)
//   [kErrMapCount], [+2, +3]  map key / value arrays of different lengths (FURY_ERR_UNSUPPORTED)
//   [kErrTooDeep], [+2, +3]   encode: a row too large for on-chip assembly in a schema nested
//                             deeper than the row interpreter reaches (FURY_ERR_UNSUPPORTED)
//   [kErrInternal], [+2, +3]  a decode plan the device could not follow (tile BFS: a write tile
//                             whose records outgrew the arena its count pass fitted) (FURY_ERR_DEVICE)
//   [kErrBudget], [+2, +3]    nested decode: a row whose slots alias other bytes so that the row
//                             walk would visit more than 2 x its bytes + 64 items -- the DEVICE's
//                             limit, not a reference exception (FURY_ERR_UNSUPPORTED with its own
//                             message; tuning counter "decode_budget_errors")
// device_error_word(stream, &w) gives the slot kernels launched on `stream` raise into (NULL if the
// runtime cannot map host memory; FURY_ERR_DEVICE when every slot is held by a live stream);
// release_error_slot(stream) frees it before the stream is destroyed; take_device_error(stream) takes that slot only (flag exchanged first,
// then its location) and sets the thread's last error when one was raised.
constexpr int kErrWords = 24;
constexpr int kErrLookBack = 0, kErrBounds = 4, kErrMapCount = 8, kErrTooDeep = 12, kErrBudget = 16,
              kErrInternal = 20;
int device_error_word(hipStream_t stream, uint32_t** out);
void release_error_slot(hipStream_t stream, bool sync = true);
int error_slots_in_use();
int error_slots_quarantined();
int thread_key_exits();
int last_assigned_key_kind();
void drain_error_quarantine();
int take_device_error(hipStream_t stream);
int64_t device_error_count();        // failures raised so far (taken or pending), no sync
// The nested decode's item-budget error (device limit): the status and message every engine
// reports it with, counted by tuning "decode_budget_errors".
int budget_error(const std::string& where);
int64_t budget_errors();

// Cached device workspace (capi.cpp): stream-ordered like hipMallocAsync / hipFreeAsync, without
// their per-call host cost.
int dev_alloc(int64_t bytes, hipStream_t stream, void** out);
void dev_free(void* p, hipStream_t stream);

// Decode bounds (round 3).  Every byte a decode reads lies in [0, total) of the rows buffer, total
// = the batch's row bytes (row_offsets[nrows]): the reference's getters read through MemoryBuffer,
// whose slice / get throw IndexOutOfBoundsException for a range past the buffer (fury-core
// memory/MemoryBuffer.java:2500-2519, through UnsafeTrait.getBuffer / getBinary,
// format/row/binary/UnsafeTrait.java:44-51,118-129, and the getInt64 of an array header,
// BinaryArray.pointTo :69-78).  A value that fails decodes as null, the kernel records where in the
// error words and the call reports FURY_ERR_OUT_OF_BOUNDS; nothing outside the batch is read.
// A negative size or element count (NegativeArraySizeException / a failed assert there) fails too.
__device__ __forceinline__ bool span_ok(int64_t p, int64_t len, int64_t total) {
  return p >= 0 && len >= 0 && len <= total - p;
}
// A workgroup barrier that orders LDS only: every wave's LDS / scalar operations complete, then
// s_barrier.  __syncthreads() adds a workgroup-scope release / acquire fence, which also waits
// for every outstanding GLOBAL store and atomic of the wave -- a tile whose column stores are in
// flight then waits out their HBM write latency at the barrier.  Use this one where the barrier
// only hands LDS data between waves (never after LDS-DMA, whose completion is counted by vmcnt).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The location is one 64-bit store (concurrent raisers never mix halves), made visible before the
// flag by a release store of the flag; stores only -- no atomics over PCIe.
__device__ __forceinline__ void raise_at(uint32_t* err, int slot, uint64_t where) {
  if (!err) return;
  __hip_atomic_store(reinterpret_cast<uint64_t*>(err + slot + 2), where, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(err + slot, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void raise_oob(uint32_t* err, int64_t row) {
  raise_at(err, kErrBounds, static_cast<uint64_t>(row));
}
__device__ __forceinline__ uint64_t err_where_entry(int node, int64_t entry) {
  return (1ull << 63) | (static_cast<uint64_t>(node) << 40) | static_cast<uint64_t>(entry);
}

// Copies a host column table to device memory on `stream` (stream-ordered: through a pinned
// staging ring, no host synchronisation); the table is freed stream-ordered when the holder goes.
struct DeviceTable {
  void* dev = nullptr;
  hipStream_t stream = nullptr;
  std::vector<uint8_t> host;          // host copy of the table (for the launchers)
  DeviceTable() = default;
  DeviceTable(const DeviceTable&) = delete;
  DeviceTable& operator=(const DeviceTable&) = delete;
  ~DeviceTable();
};
int upload_table(const void* host, size_t bytes, hipStream_t stream, DeviceTable* out);

// Device scratch for scans; grown on demand (hipMalloc outside graph capture only).
struct Workspace {
  void* ptr = nullptr;
  size_t bytes = 0;
};
int workspace_reserve(size_t bytes, void** out);

// Rows per encode tile for this column set (the staged per-row inputs must fit the LDS pool).
int encode_tile_rows(const VarArgs& a);
int64_t lookback_timeouts();
void set_host_decode_inplace(int v);   // tuning "host_decode_inplace" (hostpath.cpp)
int host_decode_inplace();
int var_dec_rows();                   // tuning "var_dec_rows" (var.hip): 0 = planned
void set_var_dec_rows(int v);
int var_dec_rows_rejected();          // forced tiles whose images did not fit (plan used instead)
int fixed_enc();                      // tuning "fixed_enc" (fixed.hip)
void set_fixed_enc(int v);
int fixed_dec();                      // tuning "fixed_dec" (fixed.hip)
void set_fixed_dec(int v);
int var_dec_pipe();                   // tuning "var_dec_pipe" (var.hip)
void set_var_dec_pipe(int v);
int var_dec_cover();                  // tuning "var_dec_cover" (var.hip): stage coverage, percent
void set_var_dec_cover(int v);
int lookback_help_mode();
int var_wide_mode();                  // tuning "var_wide" (var.hip): 1 count + write passes, 0 look-back tiles
void set_var_wide_mode(int v);
int wide_threads(bool encode);        // tuning "wide_threads" / "wide_enc_threads" (var.hip)
void set_wide_threads(bool encode, int v);
// offsets_only: fury_row_decode_measure (the Arrow offsets of the variable-length fields only)
// Plan form of the wide decode (fury_decode_prepare / _execute): the count pass + scan once, the
// per-tile bases kept for the write pass.
struct WidePlan {
  int64_t* ws = nullptr;
  int64_t nt = 0;
  int nseq = 0;
  hipStream_t stream = nullptr;
};
int wide_prepare(const VarArgs& a, const uint8_t* rows, const int64_t* offs, hipStream_t stream,
                 WidePlan* wp, std::vector<int64_t>* seq_totals);
int wide_execute(const VarArgs& a, const uint8_t* rows, const int64_t* offs, hipStream_t stream,
                 const WidePlan& wp);
void wide_free(WidePlan* wp);
int launch_decode_wide(const VarArgs& a, const uint8_t* rows, const int64_t* offs, hipStream_t stream,
                       bool offsets_only);
int launch_encode_wide(const VarArgs& a, const int64_t* offs, uint8_t* rows, int64_t cap,
                       hipStream_t stream);
int var_skip();                       // tuning "var_skip" (diagnostics, timing only)
void set_var_skip(int v);
void set_lookback_help_mode(int v);
int launch_measure_rows(const VarArgs& a, int64_t* row_offsets, hipStream_t stream);
// Rows at the offsets fury_row_measure produced; never writes row bytes at or past `cap`.
int launch_encode_var(const VarArgs& a, const int64_t* row_offsets, uint8_t* rows, int64_t cap,
                      hipStream_t stream);
int launch_encode_measured_var(const VarArgs& a, int64_t* row_offsets, uint8_t* rows, int64_t cap,
                               hipStream_t stream);
int launch_decode_measure(const VarArgs& a, const uint8_t* rows, const int64_t* row_offsets,
                          hipStream_t stream);
// Single pass: computes the Arrow offsets itself (decoupled look-back scan across workgroups)
// and writes payloads clipped to each column's capacity.
int launch_decode_var(const VarArgs& a, const uint8_t* rows, const int64_t* row_offsets,
                      hipStream_t stream, bool arrow);
// ---- generic (nested) schema engine: generic.hip --------------------------------------------
constexpr int kGenMaxNodes = 48;      // schema tree nodes in the argument block
constexpr int kGenMaxWideNodes = 4096;  // beyond 48: node table uploaded per call (GenArgs.tab)

struct GenNode {
  const uint8_t* values;   // fixed values / bytes payload / decimal values (bool: bit-packed)
  uint8_t* validity;       // Arrow validity or NULL
  int32_t* offsets;        // STRING/BINARY byte offsets, LIST/MAP entry offsets
  int32_t type;            // fury_type_id
  int32_t first_child;     // node index of the first child (children are contiguous)
  int32_t num_children;
  int32_t row_aligned;     // reached from the top through STRUCTs only: Arrow entry index = row
};

struct GenArgs {
  GenNode node[kGenMaxNodes];
  int32_t nnodes;
  int32_t ntop;            // top-level fields = nodes [0, ntop)
  int64_t nrows;
  int32_t* err;            // optional device flag (never NULL when set by the host)
  int32_t root;            // fury_schema.root: 0 rows, 1 top-level arrays, 2 top-level maps
  int32_t pad_;
  const GenNode* tab;      // device node table for > kGenMaxNodes nodes, else NULL
  const GenNode* htab;     // its host copy (launchers only; never read on the device)
};

// Nested encode (rowenc.hip): measure pass (row sizes) / build pass at the given row offsets, for
// any nesting depth (kRowEncMaxDepth levels inlined, deeper ones on an explicit stack).
int launch_gen_measure(const GenArgs& g, int64_t* sizes, hipStream_t stream);
int launch_gen_encode(const GenArgs& g, const int64_t* offs, uint8_t* rows, int64_t cap,
                      hipStream_t stream);
constexpr int kRowEncMaxDepth = 5;
constexpr int kMaxNestLevels = 64;     // schema nesting limit (schema.cpp)
int rowenc_launch(const GenArgs& g, const int64_t* offs, int64_t* sizes, uint8_t* rows,
                  int64_t cap, hipStream_t stream);
void set_rowenc_tuning(int which, uint32_t v);   // 0 "rowenc_rows", 1 "rowenc_img", 2 "rowenc_tile"
uint32_t rowenc_tuning(int which);
// Level-by-level nested decode (levels.hip): prepare = per-level count / scan / expand passes
// (totals[2 i] entries, totals[2 i + 1] payload bytes of node i), execute = one write pass into
// the outputs of gen_args' node table.
struct LvPlan;
int lv_prepare(const fury_schema* s, const uint8_t* rows, const int64_t* offs, int64_t nrows,
               hipStream_t hs, LvPlan** out, std::vector<int64_t>* totals);
int lv_execute(const LvPlan* p, const GenNode* outs, const uint8_t* rows, const int64_t* offs,
               hipStream_t hs);
void lv_free(LvPlan* p);
// Row-walk nested decode (tree.hip / walk.hip): prepare = pass 1 + tile scan + one host sync (*out NULL:
// the batch needs the level engine above), execute = pass 2 into gen_args' node table.
struct TreePlan;
int tree_prepare(const fury_schema* s, const uint8_t* rows, const int64_t* offs, int64_t nrows,
                 hipStream_t hs, TreePlan** out, std::vector<int64_t>* totals);
int tree_execute(const TreePlan* p, const GenNode* outs, const uint8_t* rows, const int64_t* offs,
                 const std::vector<int64_t>& totals, hipStream_t hs);
void tree_free(TreePlan* p);
void set_tree_mode(int v);           // tuning "nested_decode": 1 levels, 2 row walk (default), 3 walk + BFS, 4 BFS
void set_bfs_tuning(int which, uint32_t v);   // bfs_threads / bfs_rows / bfs_stage / bfs_arena
int64_t bfs_tuning(int which);                // ... and 4: bfs_fallbacks
int tree_mode();
int set_tree_debug(int on);          // tuning "tree_debug": phase accumulators on / off
// tunings of the row-walk decode (walk.hip): 0 "walk_threads" (128 / 256 rows per tile),
// 1 "walk_stage" (LDS stage cap of the count pass, bytes), 2 "walk_pool" (LDS bitmap-window
// bytes), 3 "walk_stage_write" (LDS stage cap of the write pass), 4 "walk_prefetch" (bit 0 write pass, bit 1 count pass)
void set_walk_tuning(int which, uint32_t v);
uint32_t walk_tuning(int which);
uint64_t* tree_debug_buffer();
// Exclusive scan of s[0..n) with the total stored to *total (device); ws: scan_workspace(n).
int64_t scan_workspace(int64_t n);
void device_scan(int64_t* s, int64_t n, int64_t* total, int64_t* ws, hipStream_t stream);

int launch_frame_rows(const uint8_t* rows, const int64_t* row_offsets, int64_t nrows,
                      int64_t fixed_size, int64_t schema_hash, uint8_t* out,
                      int64_t* frame_offsets, hipStream_t stream);
// Unframe mode (tuning "unframe"): 0 speculative parallel parse (sequential walk on failure),
// 1 always the sequential walk; unframe_walk_count() = streams the walk has parsed.
int unframe_mode();
void set_unframe_mode(int v);
int64_t unframe_walk_count();
void keep_pool(int device);      // hostpath.cpp: keep freed stream-pool memory pooled
int64_t host_direct_count();     // hostpath.cpp: host calls run directly on pinned memory
int64_t unframe_repair_count();      // streams parsed by the parallel repair (pointer doubling)
int launch_unframe_rows(const uint8_t* in, int64_t in_len, int64_t nrows, int64_t schema_hash,
                        uint8_t* rows_out, int64_t* row_offsets, hipStream_t stream);

// Arrow IPC (ipc.hip): encapsulated Schema message (host bytes) and RecordBatch message of
// device columns written to device memory (out == NULL: *len only).
int type_width_of(int32_t type_id);
int ipc_schema_message(const fury_schema* s, std::vector<uint8_t>* out);
int ipc_record_batch(const fury_schema* s, const fury_column* cols, int64_t n, uint8_t* out,
                     int64_t cap, int64_t* len, hipStream_t stream);

}  // namespace fury
