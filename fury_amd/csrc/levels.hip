// levels.hip — decode of nested schemas level by level (the plan API: fury_decode_prepare /
// fury_decode_execute).  Reference semantics are those of generic.hip's row interpreter
// (FMT/encoder/BaseBinaryEncoderBuilder.java:459-706 getters, FMT/vectorized/ArrowWriter.java:
// 205-640): entries of a node in (parent entry, element) order, a null struct gives a null entry
// in every child, a null list / map a zero-length entry, null values zeroed.
//
// MI355X design.  One thread per Arrow ENTRY of one schema node (blockIdx.y = node), not per
// row: consecutive lanes own consecutive entries, so every output buffer is written by
// coalesced stores and every validity / bool bitmap by wave ballots (two whole 32-bit words per
// 64 entries, no atomics).  Each entry is described by its source: the container it lives in
// (row / nested struct row / BinaryArray) and its slot there.  Top-level fields read theirs
// straight from the row (entry = row); every other node that is not a fixed-width scalar gets a
// materialised source array (16 B per entry), written by its parent's level:
//   prepare, per nesting level L:  count   (elements of each LIST / MAP entry, payload bytes
//                                           of each STRING / BINARY entry)
//                                  scan    (exclusive starts = Arrow offsets)
//                                  expand  (sources of level L+1's entries)
//   execute, one launch:           write   (values, offsets, payloads, validity of every node)
// Fixed-width scalars below a STRUCT / LIST / MAP are written by their parent's thread (a
// struct child's entry index is the struct's; array elements are copied by the array's owner),
// so they need neither a source array nor a pass of their own.  The host synchronises once per
// level that holds lists or maps (their totals size the next level), and once at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

struct LvSrc {             // where an entry's slot is: rows + base + off; base < 0: null entry
  int64_t base;            // container start (byte offset into the rows buffer)
  int64_t off;             // slot offset inside the container; < 0: the value is AT base
};

enum : int32_t { kLvTop = 0, kLvInline = 1, kLvMat = 2 };

struct LvNode {
  const uint8_t* values;   // outputs (execute): values / payload / bool bitmap
  uint8_t* validity;
  int32_t* offsets;
  LvSrc* src;              // kLvMat: one source per entry
  int64_t* start;          // STRING / BINARY / LIST / MAP: exclusive starts [m + 1]
  int64_t m;               // Arrow entries
  int32_t type;
  int32_t first_child;
  int32_t num_children;
  int32_t kind;            // kLvTop / kLvInline / kLvMat
  int32_t slot;            // top-level field index (kLvTop)
};

struct LvPlan {
  std::vector<LvNode> nodes;        // device pointers (src, start) and entry counts
  int64_t nrows = 0;
  std::vector<void*> bufs;          // stream-pool allocations owned by the plan
  hipStream_t stream = nullptr;     // the stream they were allocated on (freed on it)
  int32_t ntop = 0;
  int32_t root = 0;
};

namespace {

constexpr int kLv = 256;                      // threads per workgroup (4 waves)

struct LvArgs {
  const LvNode* nodes;                        // device table
  const int32_t* list;                        // blockIdx.y -> node index
  const uint8_t* rows;
  const int64_t* offs;
  int64_t* out;                               // lv_gather output
  int64_t nrows;
  int32_t ntop;
  int32_t root;
  int32_t nlist;                              // row-major launches: nodes in the list
  int32_t pad_;
  uint32_t* err;                              // device error words (bounds, map counts)
};

// LvSrc records through the global address space (one 16-B load / store)
__device__ __forceinline__ LvSrc ld_src(const LvSrc* p, int64_t i) {
  const auto q = gl(reinterpret_cast<const int64_t*>(p + i));
  return LvSrc{q[0], q[1]};
}
__device__ __forceinline__ void st_src(LvSrc* p, int64_t i, int64_t base, int64_t off) {
  const auto q = gl(reinterpret_cast<int64_t*>(p + i));
  q[0] = base;
  q[1] = off;
}

__device__ __forceinline__ bool lbit(const uint8_t* b, int64_t i) { return (gl(b)[i >> 3] >> (i & 7)) & 1; }
__device__ __forceinline__ int64_t lbm(int64_t n) { return ((n + 63) >> 6) << 3; }
__device__ __forceinline__ uint64_t lld8(const uint8_t* p) { return *gl(reinterpret_cast<const uint64_t*>(p)); }

__device__ __forceinline__ int lwidth(int t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

__device__ __forceinline__ uint64_t load_w(const uint8_t* p, int w) {
  switch (w) {
    case 8: return lld8(p);
    case 4: return *gl(reinterpret_cast<const uint32_t*>(p));
    case 2: return *gl(reinterpret_cast<const uint16_t*>(p));
    default: return *gl(p);
  }
}

__device__ __forceinline__ void store_w(uint8_t* p, int w, uint64_t v) {
  switch (w) {
    case 8: *gl(reinterpret_cast<uint64_t*>(p)) = v; break;
    case 4: *gl(reinterpret_cast<uint32_t*>(p)) = static_cast<uint32_t>(v); break;
    case 2: *gl(reinterpret_cast<uint16_t*>(p)) = static_cast<uint16_t>(v); break;
    default: *gl(p) = static_cast<uint8_t>(v); break;
  }
}

// Bits of 64 consecutive entries (the wave's, starting at a multiple of 64) as two whole 32-bit
// words; words at or past m are not written.  Every lane of the wave calls it.
__device__ __forceinline__ void ballot_bits(uint8_t* bits, int64_t e, bool pred, int64_t m) {
  const uint64_t b = __ballot(pred);
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (e - lane) >> 5;
  if (lane < 2 && (w0 + lane) * 32 < m)
    gl(reinterpret_cast<uint32_t*>(bits))[w0 + lane] = static_cast<uint32_t>(b >> (32 * lane));
}

// One bit of a bitmap shared with other threads (array elements of different owners).
__device__ __forceinline__ void atomic_bit(uint8_t* bits, int64_t i) {
  uint32_t* wp = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(bits + (i >> 3)) & ~uintptr_t(3));
  const int sh = static_cast<int>((reinterpret_cast<uintptr_t>(bits + (i >> 3)) & 3) * 8 + (i & 7));
  atomicOr(wp, 1u << sh);
}

// len bytes from an 8-aligned source to any destination (only [dst, dst + len) written).
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, int64_t len) {
  if (len <= 0) return;
  const int64_t head = min<int64_t>(len, (8 - (reinterpret_cast<uintptr_t>(dst) & 7)) & 7);
  for (int64_t t = 0; t < head; t++) gl(dst)[t] = gl(src)[t];
  const int64_t body = (len - head) >> 3;
  const auto s64 = gl(reinterpret_cast<const uint64_t*>(src));
  const int sh = static_cast<int>(head) * 8;
  const auto d64 = gl(reinterpret_cast<uint64_t*>(dst + head));
  for (int64_t w = 0; w < body; w++) {
    const uint64_t lo = s64[w];
    d64[w] = sh ? (lo >> sh) | (s64[w + 1] << (64 - sh)) : lo;
  }
  for (int64_t t = head + 8 * body; t < len; t++) gl(dst)[t] = gl(src)[t];
}

// The value of entry e of node n: null flag, its container base, and for variable-length types
// the value's start (vp) and size (from the slot's (relOffset << 32) | size).
struct LvVal {
  bool null;
  int64_t base;            // container start
  int64_t slot;            // absolute slot offset (< 0: the value is at base)
};

// Slot width of a node's values inside a BinaryArray (BinaryArrayWriter elementSize: the type
// width, 8 for variable-length elements).
__device__ __forceinline__ int64_t elem_size(int t) {
  const int w = lwidth(t);
  return w > 0 ? w : 8;
}

// A BinaryArray at absolute byte p whose elements are of node `en`: its header, null bits and
// element slots lie inside the batch; returns numElements (-1: outside / negative).
__device__ __forceinline__ int64_t array_ok(const LvArgs& a, int64_t p, int en_type, int64_t total) {
  if (!span_ok(p, 8, total)) return -1;
  const int64_t m = static_cast<int32_t>(lld8(a.rows + p));
  if (m < 0 || !span_ok(p, 8 + lbm(m) + m * elem_size(en_type), total)) return -1;
  return m;
}

// Bounds check of a non-null value (the reference reads it through MemoryBuffer's bounds checks,
// see span_ok in kernels.h): STRING / BINARY bytes, DECIMAL's 16 bytes, a nested row's null bits
// and slots, a LIST's array, a MAP's [key bytes][key array][value array] with equal element counts
// (BinaryMap.pointTo, BinaryMap.java:62-77: UnsupportedOperationException otherwise).  Returns the
// value's absolute start, or -1 (the value decodes as null; the error words record where).
// Every pass (count, expand, write) checks through this one function, so they agree.
__device__ __forceinline__ int64_t lv_value(const LvArgs& a, const LvNode& n, const LvVal& v,
                                            int64_t total, uint32_t* size, uint64_t where) {
  int64_t vp;
  int64_t sz = 0;
  if (v.slot < 0) {
    vp = v.base;                                                // a top-level array / map
  } else {
    const uint64_t oas = lld8(a.rows + v.slot);
    sz = static_cast<int32_t>(oas);
    vp = v.base + static_cast<int32_t>(oas >> 32);
  }
  bool ok;
  switch (n.type) {
    case FURY_TYPE_STRING:
    case FURY_TYPE_BINARY:
      ok = span_ok(vp, sz, total);
      break;
    case FURY_TYPE_DECIMAL:
      ok = span_ok(vp, 16, total);
      break;
    case FURY_TYPE_STRUCT:
      ok = span_ok(vp, lbm(n.num_children) + 8 * n.num_children, total);
      break;
    case FURY_TYPE_LIST:
      ok = array_ok(a, vp, a.nodes[n.first_child].type, total) >= 0;
      break;
    case FURY_TYPE_MAP: {
      ok = span_ok(vp, 8, total);
      if (!ok) break;
      const int64_t kb = static_cast<int32_t>(lld8(a.rows + vp));   // getInt32 of the header
      const int64_t nk = kb >= 0 ? array_ok(a, vp + 8, a.nodes[n.first_child].type, total) : -1;
      const int64_t nv = kb >= 0 ? array_ok(a, vp + 8 + kb, a.nodes[n.first_child + 1].type, total) : -1;
      ok = nk >= 0 && nv >= 0;
      if (ok && nk != nv) {
        raise_at(a.err, kErrMapCount, where);
        *size = 0;
        return -1;
      }
      break;
    }
    default:
      ok = true;
  }
  if (!ok) {
    raise_at(a.err, kErrBounds, where);
    *size = 0;
    return -1;
  }
  *size = static_cast<uint32_t>(sz);
  return vp;
}

__device__ __forceinline__ int64_t lv_total(const LvArgs& a) { return gl(a.offs)[a.nrows]; }

__device__ __forceinline__ LvVal lv_source(const LvArgs& a, const LvNode& n, int64_t e,
                                           int64_t total) {
  if (n.kind == kLvTop) {
    const int64_t base = gl(a.offs)[e];
    if (a.root) return {false, base, -1};                       // a top-level array / map
    if (!span_ok(base, lbm(a.ntop) + 8 * a.ntop, total)) {      // the row itself is outside
      raise_oob(a.err, e);
      return {true, 0, -1};
    }
    return {lbit(a.rows + base, n.slot), base, base + lbm(a.ntop) + 8 * n.slot};
  }
  const LvSrc s = ld_src(n.src, e);
  return {s.base < 0, s.base, s.off < 0 ? -1 : s.base + s.off};
}

// Count of a checked non-null value at absolute vp: LIST elements, MAP entries (key array
// elements), STRING / BINARY bytes.
__device__ __forceinline__ int64_t value_count(const LvArgs& a, int type, int64_t vp, uint32_t size) {
  if (type == FURY_TYPE_LIST) return static_cast<int32_t>(lld8(a.rows + vp));
  if (type == FURY_TYPE_MAP) return static_cast<int32_t>(lld8(a.rows + vp + 8));
  return size;
}

// Pass 1 of a level: per entry, elements (LIST / MAP) or payload bytes (STRING / BINARY).
__device__ __forceinline__ void count_entry(const LvArgs& a, const LvNode& n, int ni, int64_t e,
                                            int64_t total) {
  const LvVal v = lv_source(a, n, e, total);
  int64_t c = 0;
  if (!v.null) {
    uint32_t size;
    const int64_t vp = lv_value(a, n, v, total, &size, err_where_entry(ni, e));
    if (vp >= 0) c = value_count(a, n.type, vp, size);
  }
  gl(n.start)[e] = c;
}

// Launch shapes: kRows = the listed nodes are top-level fields (entry = row) and one thread per
// row walks all of them, so a row's null bitmap and slots are fetched once for every field;
// otherwise blockIdx.y = node, a thread per entry.
template <bool kRows>
__global__ __launch_bounds__(kLv) void lv_count(LvArgs a) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * kLv + threadIdx.x;
  const int64_t total = lv_total(a);
  if (kRows) {
    if (e >= a.nrows) return;
    // batches of kB fields: all their loads are issued before any count is stored (a store to
    // the count buffers may alias the row bytes for the compiler, which would serialise them)
    constexpr int kB = 8;
    for (int j0 = 0; j0 < a.nlist; j0 += kB) {
      int64_t c[kB];
#pragma unroll
      for (int u = 0; u < kB; u++) {
        c[u] = 0;
        if (j0 + u >= a.nlist) continue;
        const int ni = a.list[j0 + u];
        const LvNode& n = a.nodes[ni];
        const LvVal v = lv_source(a, n, e, total);
        if (v.null) continue;
        uint32_t size;
        const int64_t vp = lv_value(a, n, v, total, &size, err_where_entry(ni, e));
        if (vp >= 0) c[u] = value_count(a, n.type, vp, size);
      }
#pragma unroll
      for (int u = 0; u < kB; u++)
        if (j0 + u < a.nlist) gl(a.nodes[a.list[j0 + u]].start)[e] = c[u];
    }
  } else {
    const int ni = a.list[blockIdx.y];
    const LvNode& n = a.nodes[ni];
    if (e < n.m) count_entry(a, n, ni, e, total);
  }
}

// Elements / payload bytes of a non-null variable-length value of node ci (entry q) whose slot is
// at rows + slot in the container at rows + base (what lv_count computes, here for the next
// level's entries; 0 when the value fails its bounds check).
__device__ __forceinline__ int64_t var_count(const LvArgs& a, int ci, int64_t q, int64_t base,
                                             int64_t slot, int64_t total) {
  const LvNode& c = a.nodes[ci];
  uint32_t size;
  const int64_t vp = lv_value(a, c, LvVal{false, base, slot}, total, &size, err_where_entry(ci, q));
  return vp >= 0 ? value_count(a, c.type, vp, size) : 0;
}

// The elements of the 64 entries of a wave (one LIST / MAP node) are one contiguous range of the
// child entries: [st[0], st[64]) with st = the entries' exclusive starts.  Lanes take the
// elements round-robin (q = st[0] + lane + 64 i), each finding its owner entry by a binary search
// over st in LDS, so element work is spread evenly over the lanes whatever the list lengths and
// consecutive lanes write consecutive child entries (coalesced stores, ballot-able bits).
struct WaveLists {
  int64_t st[65];          // exclusive starts of the wave's entries (clamped at m), st[64] = end
  int64_t arr[64];         // element array of the entry (LIST / MAP keys), rows-relative
  int64_t arr2[64];        // MAP values array
};

// The WaveLists of a wave are written and read by that wave only: a wave-scope LDS fence and a
// scheduling barrier order them (a workgroup barrier made all four waves wait for the slowest,
// twice per list / map node).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// (a value that fails its bounds check has no elements: its count and start range are empty)
__device__ __forceinline__ void wave_lists_fill(const LvArgs& a, const LvNode& n, int ni, int64_t e,
                                                int64_t total, WaveLists& W) {
  const int lane = threadIdx.x & 63;
  const bool live = e < n.m;
  LvVal v{true, 0, -1};
  if (live) v = lv_source(a, n, e, total);
  int64_t ab = -1, ab2 = -1;
  if (live && !v.null) {
    uint32_t size;
    const int64_t vp = lv_value(a, n, v, total, &size, err_where_entry(ni, e));
    if (vp < 0) {
    } else if (n.type == FURY_TYPE_LIST) {
      ab = vp;
    } else {                                             // MAP: [keyBytes][keys][values]
      ab = vp + 8;
      ab2 = vp + 8 + static_cast<int32_t>(lld8(a.rows + vp));
    }
  }
  W.st[lane] = gl(n.start)[live ? e : n.m];
  if (lane == 63) W.st[64] = gl(n.start)[min(e + 1, n.m)];
  W.arr[lane] = ab;
  W.arr2[lane] = ab2;
}

// Owner lane of child entry q: the last l with st[l] <= q.
__device__ __forceinline__ int wave_owner(const WaveLists& W, int64_t q) {
  int l = 0;
#pragma unroll
  for (int b = 32; b; b >>= 1)
    if (W.st[l + b] <= q && l + b < 64) l += b;
  return l;
}

// Sources (and, for counted element nodes, counts) of the elements of a wave's arrays, into the
// non-scalar element node c; `second` selects a MAP's values array.
__device__ __forceinline__ void expand_wave(const LvArgs& a, const LvNode& c, int ci,
                                            const WaveLists& W, bool second, int64_t total) {
  const int lane = threadIdx.x & 63;
  for (int64_t q = W.st[0] + lane; q < W.st[64]; q += 64) {
    const int l = wave_owner(W, q);
    const int64_t j = q - W.st[l];
    const int64_t m = W.st[l + 1] - W.st[l];
    const int64_t ab = second ? W.arr2[l] : W.arr[l];
    const int64_t hb = 8 + lbm(m);
    const bool nul = lbit(a.rows + ab + 8, j);
    st_src(c.src, q, nul ? -1 : ab, nul ? 0 : hb + 8 * j);
    if (c.start && !nul) gl(c.start)[q] = var_count(a, ci, q, ab, ab + hb + 8 * j, total);
  }
}

// Pass 3 of a level: the sources (and counts) of the next level's materialised entries.  Every
// lane of the wave calls it for the same node (per-wave LDS for lists / maps).
__device__ __forceinline__ void expand_node(const LvArgs& a, const LvNode& n, int ni, int64_t e,
                                            int64_t total, WaveLists& W) {
  if (n.type == FURY_TYPE_STRUCT) {
    if (e >= n.m) return;
    const LvVal v = lv_source(a, n, e, total);
    uint32_t size;
    const int64_t vb = v.null ? -1 : lv_value(a, n, v, total, &size, err_where_entry(ni, e));
    const int nc = n.num_children;
    for (int k = 0; k < nc; k++) {
      const int ci = n.first_child + k;
      const LvNode& c = a.nodes[ci];
      if (c.kind != kLvMat) continue;
      const bool nul = vb < 0 || lbit(a.rows + vb, k);
      st_src(c.src, e, nul ? -1 : vb, nul ? 0 : lbm(nc) + 8 * k);
      if (c.start && !nul) gl(c.start)[e] = var_count(a, ci, e, vb, vb + lbm(nc) + 8 * k, total);
    }
    return;
  }
  wave_lists_fill(a, n, ni, e, total, W);
  wave_sync();
  const LvNode& c0 = a.nodes[n.first_child];
  if (c0.kind == kLvMat) expand_wave(a, c0, n.first_child, W, false, total);
  if (n.type == FURY_TYPE_MAP) {
    const LvNode& c1 = a.nodes[n.first_child + 1];
    if (c1.kind == kLvMat) expand_wave(a, c1, n.first_child + 1, W, true, total);
  }
  wave_sync();
}

template <bool kRows>
__global__ __launch_bounds__(kLv) void lv_expand(LvArgs a) {
  __shared__ WaveLists wl[kLv / 64];
  WaveLists& W = wl[threadIdx.x >> 6];
  const int64_t e0 = static_cast<int64_t>(blockIdx.x) * kLv;
  const int64_t e = e0 + threadIdx.x;
  const int64_t total = lv_total(a);
  if (kRows) {
    if (e0 >= a.nrows) return;
    for (int j = 0; j < a.nlist; j++) expand_node(a, a.nodes[a.list[j]], a.list[j], e, total, W);
  } else {
    const int ni = a.list[blockIdx.y];
    const LvNode& n = a.nodes[ni];
    if (e0 < n.m) expand_node(a, n, ni, e, total, W);
  }
}

// start[m] of every listed node -> out[j] (the level's totals in one small copy).
__global__ void lv_gather(LvArgs a, int32_t count) {
  const int j = threadIdx.x + blockIdx.x * blockDim.x;
  if (j >= count) return;
  const LvNode& n = a.nodes[a.list[j]];
  a.out[j] = n.start[n.m];
}

// Segmented scan of a level's count buffer: after one exclusive scan over the concatenated
// segments ([m_j counts][0] per counted node j), every segment minus its first prefix.
__global__ void lv_seg_bases(const int64_t* __restrict__ buf, int64_t* tab, int32_t nseg) {
  const int j = threadIdx.x + blockIdx.x * blockDim.x;
  if (j < nseg) tab[nseg + 1 + j] = buf[tab[j]];          // tab = [offsets nseg + 1][bases nseg]
}

__global__ __launch_bounds__(kLv) void lv_seg_sub(int64_t* __restrict__ buf, const int64_t* tab,
                                                   int32_t nseg) {
  const int j = blockIdx.y;
  const int64_t i = tab[j] + static_cast<int64_t>(blockIdx.x) * kLv + threadIdx.x;
  if (i < tab[j + 1]) buf[i] -= tab[nseg + 1 + j];
}

// ORs a ballot (bit i = child entry base + i, base not aligned) into a bitmap whose words other
// waves share: at most three 32-bit atomics per 64 entries.
__device__ __forceinline__ void ballot_or(uint8_t* bits, int64_t base, bool pred) {
  const uint64_t b = __ballot(pred);
  if (!b) return;
  const int lane = threadIdx.x & 63;
  const int sh = static_cast<int>(base & 31);
  const uint64_t lo = b << sh;
  const uint32_t hi = sh ? static_cast<uint32_t>(b >> (64 - sh)) : 0u;
  if (lane < 3) {
    const uint32_t part = lane == 0 ? static_cast<uint32_t>(lo)
                        : lane == 1 ? static_cast<uint32_t>(lo >> 32) : hi;
    if (part)
      __hip_atomic_fetch_or(gl(reinterpret_cast<uint32_t*>(bits)) + (base >> 5) + lane, part,
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Scalar elements (node c, element width w) of a wave's arrays: lanes take consecutive child
// entries, so values are coalesced stores and bits one ballot per 64 entries.
__device__ __forceinline__ void write_wave(const LvArgs& a, const LvNode& c, const WaveLists& W,
                                           bool second) {
  const int lane = threadIdx.x & 63;
  const int w = lwidth(c.type);
  uint8_t* dst = const_cast<uint8_t*>(c.values);
  const int64_t end = W.st[64];
  for (int64_t base = W.st[0]; base < end; base += 64) {
    const int64_t q = base + lane;
    bool valid = false;
    uint64_t x = 0;
    if (q < end) {
      const int l = wave_owner(W, q);
      const int64_t j = q - W.st[l];
      const int64_t m = W.st[l + 1] - W.st[l];
      const uint8_t* arr = a.rows + (second ? W.arr2[l] : W.arr[l]);
      valid = !lbit(arr + 8, j);
      if (valid) x = load_w(arr + 8 + lbm(m) + j * w, w);
      if (dst && c.type != FURY_TYPE_BOOL) store_w(dst + q * w, w, x);
    }
    if (c.validity) ballot_or(c.validity, base, valid);
    if (dst && c.type == FURY_TYPE_BOOL) ballot_or(dst, base, valid && (x & 0xff));
  }
}

// The write pass: entry e of node n (kLvTop / kLvMat), plus the scalar children its thread
// owns.  Every lane of the wave calls it for the same node (the ballots below).
__device__ __forceinline__ void write_entry(const LvArgs& a, const LvNode& n, int ni, int64_t e,
                                            int64_t total, WaveLists& W) {
  const bool live = e < n.m;
  LvVal v{true, 0, -1};
  if (live) v = lv_source(a, n, e, total);
  const int t = n.type;
  const int w = lwidth(t);
  // a variable-length value that fails its bounds check is written as null (as in the count and
  // expand passes, which gave it no elements / bytes)
  uint32_t size = 0;
  int64_t vpa = -1;
  if (live && !v.null && w <= 0) vpa = lv_value(a, n, v, total, &size, err_where_entry(ni, e));
  const bool valid = live && !v.null && (w > 0 || vpa >= 0);
  if (n.validity) ballot_bits(n.validity, e, valid, n.m);
  if (w > 0) {                                           // a top-level scalar (slot of 8 B)
    const uint64_t x = valid ? load_w(a.rows + v.slot, w) : 0;
    uint8_t* dst = const_cast<uint8_t*>(n.values);
    if (t == FURY_TYPE_BOOL) {
      if (dst) ballot_bits(dst, e, valid && (x & 0xff), n.m);
    } else if (live && dst) {
      store_w(dst + e * w, w, x);
    }
    return;
  }
  const uint8_t* vp = valid ? a.rows + vpa : nullptr;
  switch (t) {
    case FURY_TYPE_STRING:
    case FURY_TYPE_BINARY: {
      if (!live) return;
      const int64_t pos = gl(n.start)[e];
      if (valid && n.values) copy_bytes(const_cast<uint8_t*>(n.values) + pos, vp, size);
      gl(n.offsets)[e + 1] = static_cast<int32_t>(pos + (valid ? size : 0));
      if (e == 0) gl(n.offsets)[0] = 0;
      return;
    }
    case FURY_TYPE_DECIMAL: {
      if (!live || !n.values) return;
      const auto d = gl(reinterpret_cast<uint64_t*>(const_cast<uint8_t*>(n.values) + 16 * e));
      d[0] = valid ? lld8(vp) : 0;
      d[1] = valid ? lld8(vp + 8) : 0;
      return;
    }
    case FURY_TYPE_LIST:
    case FURY_TYPE_MAP: {
      if (live) {
        gl(n.offsets)[e + 1] = static_cast<int32_t>(gl(n.start)[e + 1]);
        if (e == 0) gl(n.offsets)[0] = 0;
      }
      const LvNode& c0 = a.nodes[n.first_child];
      const bool s0 = c0.kind == kLvInline;
      const bool s1 = t == FURY_TYPE_MAP && a.nodes[n.first_child + 1].kind == kLvInline;
      if (!s0 && !s1) return;
      wave_lists_fill(a, n, ni, e, total, W);              // every lane of the wave
      wave_sync();
      if (s0) write_wave(a, c0, W, false);
      if (s1) write_wave(a, a.nodes[n.first_child + 1], W, true);
      wave_sync();
      return;
    }
    case FURY_TYPE_STRUCT: {                             // scalar fields: entry index = e
      const int nc = n.num_children;
      for (int k = 0; k < nc; k++) {
        const LvNode& c = a.nodes[n.first_child + k];
        if (c.kind != kLvInline) continue;
        const int cw = lwidth(c.type);
        const bool cv = valid && !lbit(vp, k);
        const uint64_t x = cv ? load_w(vp + lbm(nc) + 8 * k, cw) : 0;
        if (c.validity) ballot_bits(c.validity, e, cv, n.m);
        uint8_t* dst = const_cast<uint8_t*>(c.values);
        if (!dst) continue;
        if (c.type == FURY_TYPE_BOOL) ballot_bits(dst, e, cv && (x & 0xff), n.m);
        else if (live) store_w(dst + e * cw, cw, x);
      }
      return;
    }
    default:
      return;
  }
}

template <bool kRows>
__global__ __launch_bounds__(kLv) void lv_write(LvArgs a) {
  __shared__ WaveLists wl[kLv / 64];
  WaveLists& W = wl[threadIdx.x >> 6];
  const int64_t e0 = static_cast<int64_t>(blockIdx.x) * kLv;
  const int64_t e = e0 + threadIdx.x;
  const int64_t total = lv_total(a);
  if (kRows) {
    if (e0 >= a.nrows) return;
    for (int j = 0; j < a.nlist; j++) write_entry(a, a.nodes[a.list[j]], a.list[j], e, total, W);
  } else {
    const int ni = a.list[blockIdx.y];
    const LvNode& n = a.nodes[ni];
    if (e0 < n.m) write_entry(a, n, ni, e, total, W);
  }
}

bool counted(int32_t t) {
  return t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY || t == FURY_TYPE_LIST || t == FURY_TYPE_MAP;
}

int host_width(int32_t t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

// The node table + launch list for one kernel, uploaded stream-ordered (kept alive by dt until
// the launches before its release have run).
int upload_args(const LvPlan& p, const std::vector<int32_t>& list, const uint8_t* rows,
                const int64_t* offs, hipStream_t hs, DeviceTable* dt, LvArgs* a) {
  const size_t nb = p.nodes.size() * sizeof(LvNode);
  std::vector<uint8_t> buf(nb + list.size() * sizeof(int32_t));
  memcpy(buf.data(), p.nodes.data(), nb);
  if (!list.empty()) memcpy(buf.data() + nb, list.data(), list.size() * sizeof(int32_t));
  const int st = upload_table(buf.data(), buf.size(), hs, dt);
  if (st) return st;
  a->nodes = static_cast<const LvNode*>(dt->dev);
  a->list = reinterpret_cast<const int32_t*>(static_cast<const uint8_t*>(dt->dev) + nb);
  a->rows = rows;
  a->offs = offs;
  a->out = nullptr;
  a->ntop = p.ntop;
  a->root = p.root;
  a->nrows = p.nrows;
  a->nlist = static_cast<int32_t>(list.size());
  if (const int e = device_error_word(hs, &a->err)) return e;
  return FURY_OK;
}

int64_t max_m(const LvPlan& p, const std::vector<int32_t>& list) {
  int64_t m = 0;
  for (int i : list) m = std::max(m, p.nodes[i].m);
  return m;
}

dim3 grid_of(const LvPlan& p, const std::vector<int32_t>& list) {
  return dim3(static_cast<unsigned>((max_m(p, list) + kLv - 1) / kLv),
              static_cast<unsigned>(list.size()));
}

// Launches kernel K<true> row-major over the listed top-level nodes and K<false> node-major over
// the others (each with its own uploaded list).
template <typename F>
int launch_split(const LvPlan& p, const std::vector<int32_t>& list, const uint8_t* rows,
                 const int64_t* offs, hipStream_t hs, F launch) {
  std::vector<int32_t> top, deep;
  for (int i : list) (p.nodes[i].kind == kLvTop ? top : deep).push_back(i);
  for (int pass = 0; pass < 2; pass++) {
    const std::vector<int32_t>& l = pass == 0 ? top : deep;
    if (l.empty()) continue;
    DeviceTable dt;
    LvArgs a;
    int st = upload_args(p, l, rows, offs, hs, &dt, &a);
    if (st) return st;
    launch(pass == 0, a, pass == 0 ? dim3(static_cast<unsigned>((p.nrows + kLv - 1) / kLv))
                                   : grid_of(p, l));
    if ((st = check_hip(hipGetLastError(), "level kernel launch"))) return st;
  }
  return FURY_OK;
}

int pool_alloc(LvPlan* p, int64_t bytes, void** out) {
  *out = nullptr;
  const int st = dev_alloc(bytes > 0 ? bytes : 16, p->stream, out);
  if (!st) p->bufs.push_back(*out);
  return st;
}

// start[m] of the listed nodes -> host (one gather kernel, one copy, one sync).
// Pinned landing buffer of the level totals, per thread, grown on demand (a copy into pageable
// memory takes the runtime's staged path).
int64_t* pinned_totals(size_t n) {
  thread_local int64_t* buf = nullptr;
  thread_local size_t cap = 0;
  if (n > cap) {
    if (buf) (void)hipHostFree(buf);
    buf = nullptr;
    cap = 0;
    const size_t c = std::max<size_t>(n, 4096);
    void* p = nullptr;
    if (hipHostMalloc(&p, c * 8, hipHostMallocDefault) != hipSuccess) return nullptr;
    buf = static_cast<int64_t*>(p);
    cap = c;
  }
  return buf;
}

// *batch_bytes (when given): the batch's row bytes, offs[nrows], copied with the totals into the
// same pinned buffer (one word past them).
int level_totals(const LvPlan& p, const std::vector<int32_t>& list, const uint8_t* rows,
                 const int64_t* offs, hipStream_t hs, int64_t* dev_out, std::vector<int64_t>* out,
                 int64_t* batch_bytes) {
  out->assign(list.size(), 0);
  if (list.empty()) return FURY_OK;
  int64_t* host = pinned_totals(list.size() + 1);
  if (!host) return set_error(FURY_ERR_DEVICE, "hipHostMalloc (decode plan totals)");
  DeviceTable dt;
  LvArgs a;
  int st = upload_args(p, list, rows, offs, hs, &dt, &a);
  if (st) return st;
  a.out = dev_out;
  hipLaunchKernelGGL(lv_gather, dim3(static_cast<unsigned>((list.size() + 255) / 256)), dim3(256), 0,
                     hs, a, static_cast<int32_t>(list.size()));
  if ((st = check_hip(hipGetLastError(), "lv_gather launch"))) return st;
  if ((st = check_hip(hipMemcpyAsync(host, dev_out, list.size() * 8, hipMemcpyDeviceToHost, hs),
                      "hipMemcpyAsync totals")))
    return st;
  if (batch_bytes &&
      (st = check_hip(hipMemcpyAsync(host + list.size(), offs + p.nrows, 8, hipMemcpyDeviceToHost, hs),
                      "hipMemcpyAsync batch bytes")))
    return st;
  if ((st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize"))) return st;
  out->assign(host, host + list.size());
  if (batch_bytes) *batch_bytes = host[list.size()];
  return FURY_OK;
}

}  // namespace

void lv_free(LvPlan* p) {
  if (!p) return;
  for (void* b : p->bufs) dev_free(b, p->stream);
  delete p;
}

int lv_prepare(const fury_schema* s, const uint8_t* rows, const int64_t* offs, int64_t nrows,
               hipStream_t hs, LvPlan** out, std::vector<int64_t>* totals) {
  *out = nullptr;
  const int nn = static_cast<int>(s->nodes.size());
  int device = 0;
  (void)hipGetDevice(&device);
  keep_pool(device);                                // per-level syncs must not unmap the pool
  LvPlan* p = new LvPlan();
  p->stream = hs;
  p->ntop = s->num_fields;
  p->root = s->root;
  p->nodes.assign(nn, LvNode{});
  p->nrows = nrows;
  std::vector<int32_t> level(nn, 0);
  int maxl = 0;
  for (int i = 0; i < nn; i++) {
    const GenTpl& t = s->nodes[i];
    LvNode& n = p->nodes[i];
    n.type = t.type_id;
    n.first_child = t.first_child;
    n.num_children = t.num_children;
    if (i < s->num_fields) {
      n.kind = kLvTop;
      n.slot = i;
      n.m = nrows;
    } else {
      // scalars are written by their parent's thread (struct field) or wave (array element)
      n.kind = host_width(t.type_id) > 0 ? kLvInline : kLvMat;
    }
    for (int j = 0; j < t.num_children; j++) {
      level[t.first_child + j] = level[i] + 1;
      maxl = std::max(maxl, level[i] + 1);
    }
  }
  totals->assign(2 * nn, 0);
  int st = FURY_OK;
  int64_t* dev_tot = nullptr;
  if ((st = pool_alloc(p, 8 * (nn + 1), reinterpret_cast<void**>(&dev_tot)))) {
    lv_free(p);
    return st;
  }
  // The counted nodes of level L (m > 0) share one buffer of segments [m_j counts][0], zeroed:
  // lv_count (level 0) or the parent level's lv_expand fills the counts, one segmented scan
  // turns them into starts.
  auto counted_at = [&](int L) {
    std::vector<int32_t> v;
    for (int i = 0; i < nn; i++)
      if (level[i] == L && p->nodes[i].m > 0 && p->nodes[i].kind != kLvInline && counted(p->nodes[i].type))
        v.push_back(i);
    return v;
  };
  std::vector<int64_t> seg;                         // segment offsets of the current level
  auto alloc_level = [&](const std::vector<int32_t>& cnt) -> int {
    seg.assign(1, 0);
    for (int i : cnt) seg.push_back(seg.back() + p->nodes[i].m + 1);
    if (cnt.empty()) return FURY_OK;
    int64_t* buf = nullptr;
    int r = pool_alloc(p, 8 * (seg.back() + 1), reinterpret_cast<void**>(&buf));
    if (r) return r;
    for (size_t j = 0; j < cnt.size(); j++) p->nodes[cnt[j]].start = buf + seg[j];
    return check_hip(hipMemsetAsync(buf, 0, 8 * (seg.back() + 1), hs), "hipMemsetAsync counts");
  };
  auto scan_level = [&](const std::vector<int32_t>& cnt) -> int {
    if (cnt.empty()) return FURY_OK;
    int64_t* buf = p->nodes[cnt[0]].start;
    const int64_t len = seg.back();
    int64_t* ws = nullptr;
    int r = pool_alloc(p, 8 * scan_workspace(len), reinterpret_cast<void**>(&ws));
    if (r) return r;
    device_scan(buf, len, buf + len, ws, hs);
    if (cnt.size() == 1) return check_hip(hipGetLastError(), "scan launch");
    const int32_t nseg = static_cast<int32_t>(cnt.size());
    std::vector<int64_t> tab(seg.begin(), seg.end());
    tab.resize(2 * nseg + 1, 0);
    DeviceTable dt;
    if ((r = upload_table(tab.data(), tab.size() * 8, hs, &dt))) return r;
    int64_t* dtab = static_cast<int64_t*>(dt.dev);
    hipLaunchKernelGGL(lv_seg_bases, dim3(static_cast<unsigned>((nseg + 255) / 256)), dim3(256), 0, hs,
                       buf, dtab, nseg);
    int64_t maxlen = 0;
    for (int32_t j = 0; j < nseg; j++) maxlen = std::max(maxlen, seg[j + 1] - seg[j]);
    hipLaunchKernelGGL(lv_seg_sub, dim3(static_cast<unsigned>((maxlen + kLv - 1) / kLv), nseg),
                       dim3(kLv), 0, hs, buf, dtab, nseg);
    return check_hip(hipGetLastError(), "segmented scan launch");
  };
  // The batch's row bytes, read with every level's totals (one more word of the same pinned copy):
  // a node's elements each own at least one byte of some row, so more elements than row bytes means
  // slots that alias other bytes (a malformed batch whose level arrays would grow with the product
  // of the aliased counts).  Every non-zero total arrives through level_totals, so the check below
  // always has the byte count it needs.
  int64_t batch_bytes = -1;
  std::vector<int32_t> strings;                     // STRING / BINARY nodes: bytes at the end
  std::vector<int32_t> cnt = counted_at(0);
  if (!(st = alloc_level(cnt)) && !cnt.empty())
    st = launch_split(*p, cnt, rows, offs, hs, [&](bool by_row, const LvArgs& a, dim3 g) {
      if (by_row) hipLaunchKernelGGL(lv_count<true>, g, dim3(kLv), 0, hs, a);
      else hipLaunchKernelGGL(lv_count<false>, g, dim3(kLv), 0, hs, a);
    });
  for (int L = 0; L <= maxl && !st; L++) {
    if ((st = scan_level(cnt))) break;
    std::vector<int32_t> arrays, parents;
    for (int i : cnt)
      (p->nodes[i].type == FURY_TYPE_LIST || p->nodes[i].type == FURY_TYPE_MAP ? arrays : strings)
          .push_back(i);
    // sizes of the next level: a struct's children have its entries, an array's elements its total
    // one gather + copy + sync per level that holds lists / maps; string totals found so far
    // ride along (bytes), so the last sync is needed only for strings below the last array level
    std::vector<int64_t> tot;
    std::vector<int32_t> ask(arrays);
    if (!arrays.empty()) ask.insert(ask.end(), strings.begin(), strings.end());
    if ((st = level_totals(*p, ask, rows, offs, hs, dev_tot, &tot, &batch_bytes))) break;
    if (!arrays.empty()) {
      for (size_t j = 0; j < strings.size(); j++)
        (*totals)[2 * strings[j] + 1] = tot[arrays.size() + j];
      strings.clear();
    }
    for (size_t j = 0; j < arrays.size() && !st; j++) {
      if (tot[j] < 0 || tot[j] > batch_bytes)
        st = budget_error("nested decode (level engine): more elements of a node than the batch "
                          "has row bytes");
      const LvNode& n = p->nodes[arrays[j]];
      for (int c = 0; c < n.num_children; c++) p->nodes[n.first_child + c].m = tot[j];
    }
    if (st) break;
    for (int i = 0; i < nn; i++) {
      const LvNode& n = p->nodes[i];
      if (level[i] != L || n.type != FURY_TYPE_STRUCT) continue;
      for (int c = 0; c < n.num_children; c++) p->nodes[n.first_child + c].m = n.m;
    }
    if (L == maxl) break;
    cnt = counted_at(L + 1);
    if ((st = alloc_level(cnt))) break;
    for (int i = 0; i < nn; i++) {
      if (level[i] != L || p->nodes[i].m == 0 || p->nodes[i].kind == kLvInline) continue;
      const LvNode& n = p->nodes[i];
      bool has = false;
      for (int c = 0; c < n.num_children && !st; c++) {
        LvNode& ch = p->nodes[n.first_child + c];
        if (ch.kind != kLvMat || ch.m == 0) continue;
        st = pool_alloc(p, sizeof(LvSrc) * ch.m, reinterpret_cast<void**>(&ch.src));
        has = true;
      }
      if (has) parents.push_back(i);
    }
    if (st || parents.empty()) continue;
    st = launch_split(*p, parents, rows, offs, hs, [&](bool by_row, const LvArgs& a, dim3 g) {
      if (by_row) hipLaunchKernelGGL(lv_expand<true>, g, dim3(kLv), 0, hs, a);
      else hipLaunchKernelGGL(lv_expand<false>, g, dim3(kLv), 0, hs, a);
    });
  }
  std::vector<int64_t> bytes;
  if (!st) st = level_totals(*p, strings, rows, offs, hs, dev_tot, &bytes, &batch_bytes);
  if (st) {
    lv_free(p);
    return st;
  }
  for (int i = 0; i < nn; i++) (*totals)[2 * i] = p->nodes[i].m;
  for (size_t j = 0; j < strings.size(); j++) (*totals)[2 * strings[j] + 1] = bytes[j];
  // payload bytes past the batch's row bytes: strings that alias other bytes (as above)
  for (int i = 0; i < nn; i++)
    if ((*totals)[2 * i + 1] > std::max<int64_t>(batch_bytes, 0)) {
      lv_free(p);
      return budget_error("nested decode (level engine): more payload bytes of a node than the "
                          "batch has row bytes");
    }
  *out = p;
  return FURY_OK;
}

int lv_execute(const LvPlan* p, const GenNode* outs, const uint8_t* rows, const int64_t* offs,
               hipStream_t hs) {
  LvPlan q = *p;                                   // outputs of this call into a copy
  q.bufs.clear();
  std::vector<int32_t> list;
  for (size_t i = 0; i < q.nodes.size(); i++) {
    LvNode& n = q.nodes[i];
    n.values = outs[i].values;
    n.validity = outs[i].validity;
    n.offsets = outs[i].offsets;
    if (n.kind != kLvInline && n.m > 0) list.push_back(static_cast<int32_t>(i));
    if (n.m == 0 && n.offsets) {                   // no entries: the Arrow offsets are just [0]
      const int st = check_hip(hipMemsetAsync(n.offsets, 0, 4, hs), "hipMemsetAsync offsets");
      if (st) return st;
    }
  }
  if (list.empty()) return FURY_OK;
  return launch_split(q, list, rows, offs, hs, [&](bool by_row, const LvArgs& a, dim3 g) {
    if (by_row) hipLaunchKernelGGL(lv_write<true>, g, dim3(kLv), 0, hs, a);
    else hipLaunchKernelGGL(lv_write<false>, g, dim3(kLv), 0, hs, a);
  });
}

}  // namespace fury
