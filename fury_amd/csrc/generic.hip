// generic.hip — schema-interpreting kernels for ANY schema the reference row format supports:
// nested STRUCT (bean fields), LIST of any element type (incl. strings, structs, lists, maps),
// MAP (key / value arrays), plus every scalar type.  The specialised kernels in fixed.hip /
// var.hip cover flat schemas at full speed; this engine covers the rest of the type system.
//
// Reference semantics (FMT = java/fury-format/src/main/java/org/apache/fury/format):
//   encode   BaseBinaryEncoderBuilder.serializeFor (FMT/encoder/BaseBinaryEncoderBuilder.java:
//            138-453): primitives into 8-byte slots, var values appended at the writer index and
//            padded to 8 (BinaryWriter.java:106-121,187-194), List -> BinaryArrayWriter image
//            [int64 n][bitmap][n x elemSize, tail zeroed][var section] (BinaryArrayWriter.java:
//            91-163), bean -> child BinaryRowWriter row (:363-417), Map -> [int64 keyBytes]
//            [key array][value array] (:298-357); null -> setNullAt only.
//   decode   getters + ArrowWriter (FMT/vectorized/ArrowWriter.java:205-640): a null struct
//            appends a null to every child (StructWriter.appendNull :577-584), null lists/maps
//            are zero-length entries (ListWriter/MapWriter.appendNull no-op + fillHoles).
//
// MI355X design: the flattened schema and the per-call column pointers travel in the kernel
// argument block (scalar-loaded).  Encode is one thread per row (measure pass -> device scan ->
// build pass).  Decode counts, per row and per schema node, the Arrow entries and payload bytes
// the row contributes; device scans turn those into each row's starting positions in every
// output buffer, and a second thread-per-row pass writes them.  Validity bits go through 32-bit
// atomics on buffers the host zeroes; everything else is plain stores into disjoint ranges.
// Recursion is depth-unrolled (template<int D>), at most kMaxDepth levels of nesting.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

constexpr int kThreads = 64;          // decode keeps per-thread node counters in LDS
constexpr int kEncThreads = 256;

__device__ __forceinline__ bool gbit(const uint8_t* bits, int64_t i) {
  return (gl(bits)[i >> 3] >> (i & 7)) & 1;
}
__device__ __forceinline__ int64_t g8(int64_t n) { return (n + 7) & ~int64_t(7); }
__device__ __forceinline__ int64_t gbm(int64_t n) { return ((n + 63) >> 6) << 3; }

__device__ __forceinline__ int gwidth(int t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

// Typed accesses.  Row images are built in LDS (LdsU8) or, past the image, straight in HBM
// (uint8_t*: always device memory here); input columns and rows are device memory.  With the
// address space explicit the compiler emits ds_* / global_* instead of flat_* (a flat access
// counts against both vmcnt and lgkmcnt, so each wait waited for both).
template <class T>
using Lds = __attribute__((address_space(3))) T;
using LdsU8 = Lds<uint8_t>;

__device__ __forceinline__ void st8(uint8_t* p, uint64_t v) {   // p 8-aligned by construction
  *gl(reinterpret_cast<uint64_t*>(p)) = v;
}
__device__ __forceinline__ void st8(LdsU8* p, uint64_t v) { *reinterpret_cast<Lds<uint64_t>*>(p) = v; }
__device__ __forceinline__ void st4(uint8_t* p, uint32_t v) { *gl(reinterpret_cast<uint32_t*>(p)) = v; }
__device__ __forceinline__ void st4(LdsU8* p, uint32_t v) { *reinterpret_cast<Lds<uint32_t>*>(p) = v; }
__device__ __forceinline__ void st2(uint8_t* p, uint16_t v) { *gl(reinterpret_cast<uint16_t*>(p)) = v; }
__device__ __forceinline__ void st2(LdsU8* p, uint16_t v) { *reinterpret_cast<Lds<uint16_t>*>(p) = v; }
__device__ __forceinline__ void st1(uint8_t* p, uint8_t v) { *gl(p) = v; }
__device__ __forceinline__ void st1(LdsU8* p, uint8_t v) { *p = v; }
__device__ __forceinline__ void or1(uint8_t* p, uint8_t v) { *gl(p) |= v; }
__device__ __forceinline__ void or1(LdsU8* p, uint8_t v) { *p |= v; }
__device__ __forceinline__ uint64_t ld8(const uint8_t* p) {
  return *gl(reinterpret_cast<const uint64_t*>(p));
}

// Copies len bytes from an 8-byte aligned source (a row's var section) to any destination:
// bytes up to the destination's 8-byte boundary, then whole 8-byte stores of funnel-shifted
// source words, then the tail bytes.  Only [dst, dst + len) is written (neighbouring threads
// own the bytes around it).
__device__ __forceinline__ void copy_to_unaligned(uint8_t* dst, const uint8_t* src, int64_t len) {
  if (len <= 0) return;
  const int64_t head = min<int64_t>(len, (8 - (reinterpret_cast<uintptr_t>(dst) & 7)) & 7);
  for (int64_t t = 0; t < head; t++) dst[t] = src[t];
  const int64_t body = (len - head) >> 3;
  const uint64_t* s64 = reinterpret_cast<const uint64_t*>(src);
  const int sh = static_cast<int>(head) * 8;           // source bit offset of the body
  uint64_t* d64 = reinterpret_cast<uint64_t*>(dst + head);
  for (int64_t w = 0; w < body; w++) {
    const uint64_t lo = s64[w];
    const uint64_t v = sh ? (lo >> sh) | (s64[w + 1] << (64 - sh)) : lo;
    d64[w] = v;
  }
  for (int64_t t = head + 8 * body; t < len; t++) dst[t] = src[t];
}

// ---- encode ----------------------------------------------------------------------------------

template <class P>
__device__ __forceinline__ void zero_bytes(P p, int64_t n) {
  // 8-byte aligned start; n multiple of 8 in every use
  for (int64_t i = 0; i < n; i += 8) st8(p + i, 0);
}

// Appends len bytes (unaligned source) at dst (8-aligned), zero-padding to 8.
template <class P>
__device__ __forceinline__ void append_unaligned(P dst, const uint8_t* src, int64_t len) {
  // aligned source words funnel-shifted into place; no word past the last source byte is read
  const uintptr_t so = reinterpret_cast<uintptr_t>(src) & 7;
  const auto ap = gl(reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(src) - so));
  const int64_t nw = (len + 7) >> 3;
  const int64_t nsrc = (static_cast<int64_t>(so) + len + 7) >> 3;
  const int sh = static_cast<int>(so) * 8;
  uint64_t cur = nsrc > 0 ? ap[0] : 0;
  for (int64_t w = 0; w < nw; w++) {
    const uint64_t nxt = w + 1 < nsrc ? ap[w + 1] : 0;
    uint64_t x = sh ? (cur >> sh) | (nxt << (64 - sh)) : cur;
    const int64_t rem = len - 8 * w;
    if (rem < 8) x &= (~0ull) >> (8 * (8 - rem));
    st8(dst + 8 * w, x);
    cur = nxt;
  }
}

template <int D, bool W, class P, class NP>
__device__ void put_value(NP nodes, int ni, int64_t idx, P buf, int64_t container,
                          int64_t slot, int es, bool in_array, int64_t bitmap, int64_t ordinal,
                          int64_t& cursor);

// BinaryArrayWriter image of elements [b, b + m) of node `ei` at buf + cursor.
template <int D, bool W, class P, class NP>
__device__ void put_array(NP nodes, int ei, int64_t b, int64_t m, P buf,
                          int64_t& cursor) {
  const auto& e = nodes[ei];
  const int w = gwidth(e.type);
  const int es = w > 0 ? w : 8;
  const int64_t start = cursor;
  const int64_t hb = 8 + gbm(m);
  const int64_t fp = g8(m * es);
  if (W) {
    st8(buf + start, static_cast<uint64_t>(m));
    zero_bytes(buf + start + 8, hb - 8 + fp);     // bitmap, element slots, alignment tail
  }
  int64_t c2 = start + hb + fp;
  for (int64_t j = 0; j < m; j++)
    put_value<D + 1, W>(nodes, ei, b + j, buf, start, start + hb + j * es, es, true, start + 8, j, c2);
  cursor = c2;
}

template <int D, bool W, class P, class NP>
__device__ void put_value(NP nodes, int ni, int64_t idx, P buf, int64_t container,
                          int64_t slot, int es, bool in_array, int64_t bitmap, int64_t ordinal,
                          int64_t& cursor) {
  if constexpr (D >= kGenMaxDepth) {
    (void)nodes;
    return;
  } else {
    const auto& n = nodes[ni];
    if (n.validity && !gbit(n.validity, idx)) {      // setNullAt: bit only, slot stays 0
      if (W) or1(buf + bitmap + (ordinal >> 3), static_cast<uint8_t>(1u << (ordinal & 7)));
      return;
    }
    const int w = gwidth(n.type);
    if (w > 0) {
      if (W) {
        uint64_t v;
        if (n.type == FURY_TYPE_BOOL) v = gbit(n.values, idx);
        else if (w == 8) v = ld8(n.values + idx * 8);
        else if (w == 4) v = *gl(reinterpret_cast<const uint32_t*>(n.values + idx * 4));
        else if (w == 2) v = *gl(reinterpret_cast<const uint16_t*>(n.values + idx * 2));
        else v = gl(n.values)[idx];
        if (!in_array) {
          st8(buf + slot, v);                           // putInt64(0) + narrow put
        } else {
          switch (es) {
            case 8: st8(buf + slot, v); break;
            case 4: st4(buf + slot, static_cast<uint32_t>(v)); break;
            case 2: st2(buf + slot, static_cast<uint16_t>(v)); break;
            default: st1(buf + slot, static_cast<uint8_t>(v)); break;
          }
        }
      }
      return;
    }
    const int64_t start = cursor;
    switch (n.type) {
      case FURY_TYPE_STRING:
      case FURY_TYPE_BINARY: {
        const int64_t b = gl(n.offsets)[idx];
        const int64_t len = gl(n.offsets)[idx + 1] - b;
        if (W) append_unaligned(buf + start, n.values + b, len);
        cursor = start + g8(len);
        if (W) st8(buf + slot, (static_cast<uint64_t>(start - container) << 32) | static_cast<uint32_t>(len));
        return;
      }
      case FURY_TYPE_DECIMAL: {
        if (W) {
          st8(buf + start, ld8(n.values + 16 * idx));
          st8(buf + start + 8, ld8(n.values + 16 * idx + 8));
          st8(buf + slot, (static_cast<uint64_t>(start - container) << 32) | 16u);
        }
        cursor = start + 16;
        return;
      }
      case FURY_TYPE_LIST: {
        const int64_t b = gl(n.offsets)[idx];
        put_array<D, W>(nodes, n.first_child, b, gl(n.offsets)[idx + 1] - b, buf, cursor);
        break;
      }
      case FURY_TYPE_STRUCT: {
        const int nc = n.num_children;
        const int64_t bmb = gbm(nc);
        const int64_t fixed = bmb + 8 * nc;
        if (W) zero_bytes(buf + start, fixed);
        int64_t c2 = start + fixed;
        for (int k = 0; k < nc; k++)
          put_value<D + 1, W>(nodes, n.first_child + k, idx, buf, start, start + bmb + 8 * k, 8, false,
                              start, k, c2);
        cursor = c2;
        break;
      }
      case FURY_TYPE_MAP: {
        const int64_t b = gl(n.offsets)[idx];
        const int64_t m = gl(n.offsets)[idx + 1] - b;
        int64_t c2 = start + 8;                         // writeDirectly(-1) placeholder
        put_array<D, W>(nodes, n.first_child, b, m, buf, c2);
        if (W) st8(buf + start, static_cast<uint64_t>(c2 - (start + 8)));   // key array size
        put_array<D, W>(nodes, n.first_child + 1, b, m, buf, c2);
        cursor = c2;
        break;
      }
      default:
        
        return;
    }
    if (W) st8(buf + slot, (static_cast<uint64_t>(start - container) << 32) |
                               static_cast<uint32_t>(cursor - start));
  }
}

// Entry r of the batch: a row of the ntop top-level fields (root 0), or -- ArrayEncoder.toArray /
// MapEncoder.toMap (ArrayEncoderBuilder.java:118-140, MapEncoderBuilder.java:152-208) -- the
// top-level BinaryArray (root 1) / BinaryMap [int64 keyBytes][keys][values] (root 2) of node 0's
// entry r, written at the buffer start exactly as inside a row (element offsets are relative to
// the array itself).
template <bool W, int kRoot, class P, class NP>
__device__ int64_t put_row(NP nodes, int ntop, int64_t r, P buf) {
  constexpr int root = kRoot;
  if constexpr (kRoot != 0) {
    const auto& n = nodes[0];
    const int64_t b = gl(n.offsets)[r];
    const int64_t m = gl(n.offsets)[r + 1] - b;
    int64_t cursor = root == 2 ? 8 : 0;
    put_array<1, W>(nodes, n.first_child, b, m, buf, cursor);
    if (root == 2) {
      if (W) st8(buf, static_cast<uint64_t>(cursor - 8));      // key array bytes
      put_array<1, W>(nodes, n.first_child + 1, b, m, buf, cursor);
    }
    return cursor;
  }
  const int64_t bmb = gbm(ntop);
  const int64_t fixed = bmb + 8 * ntop;
  if (W) zero_bytes(buf, fixed);                       // fresh buffer: bitmap + slots zero
  int64_t cursor = fixed;
  for (int k = 0; k < ntop; k++)
    put_value<1, W>(nodes, k, r, buf, 0, bmb + 8 * k, 8, false, 0, k, cursor);
  return cursor;
}

// The node table is copied from the argument block into LDS once per workgroup and passed to
// the (non-inlined, recursive-by-depth) helpers as a pointer: taking the address of the kernel
// argument itself would make the compiler copy the whole block into per-lane scratch.  Schemas
// with more nodes than the argument block holds (kWide) read the table the host uploaded for the
// call straight from device memory (uniform indices: scalar loads).
template <bool kWide>
__device__ __forceinline__ const GenNode* stage_nodes(const GenArgs& g, GenNode* lds) {
  if (kWide) return g.tab;
  for (int i = threadIdx.x; i < g.nnodes; i += blockDim.x) lds[i] = g.node[i];
  __syncthreads();
  return lds;
}

// The encode side's node table with its address space explicit (LDS copy / uploaded table).
using GNodes = __attribute__((address_space(1))) const GenNode*;
using LNodes = Lds<const GenNode>*;
template <bool kWide>
__device__ __forceinline__ auto enc_nodes(const GenArgs& g, GenNode* lds) {
  const GenNode* p = stage_nodes<kWide>(g, lds);
  if constexpr (kWide) return (GNodes)(p);
  else return (LNodes)(p);
}

// kRoot (fury_schema.root) is a template parameter so the row kernels do not carry the
// collection code: inlining both into one kernel raised its scratch from 192 to 1200 B per lane
// and doubled the encode time.
template <bool kWide, int kRoot>
__global__ __launch_bounds__(kEncThreads) void gen_measure_kernel(GenArgs g, int64_t* __restrict__ sizes) {
  __shared__ GenNode sn[kWide ? 1 : kGenMaxNodes];
  const auto nodes = enc_nodes<kWide>(g, sn);
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kEncThreads + threadIdx.x;
  if (r < g.nrows) sizes[r] = put_row<false, kRoot>(nodes, g.ntop, r, static_cast<uint8_t*>(nullptr));
}

// The workgroup's 256 rows are one contiguous byte range of the output: each thread builds its
// row in an LDS image of that range (put_row writes every byte of a row: zeroed bitmaps and
// slots, zero-padded variable parts), then the workgroup stores the range with coalesced 8-byte
// stores.  Thread-per-row stores straight to HBM wrote ~5x the row bytes (WRITE_SIZE of the
// depth-3 schema at 4M rows: partial lines of 64 rows at a time, evicted before they filled).
// A tile larger than the image (or past `cap`) takes the direct path.
constexpr int64_t kGenImg = 76 * 1024;

template <bool kWide, int kRoot>
__global__ __launch_bounds__(kEncThreads, 2) void gen_encode_kernel(GenArgs g,
                                                                 const int64_t* __restrict__ offs,
                                                                 uint8_t* __restrict__ rows,
                                                                 int64_t cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t img[];
  __shared__ GenNode sn[kWide ? 1 : kGenMaxNodes];
  const auto nodes = enc_nodes<kWide>(g, sn);
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kEncThreads;
  const int64_t r = r0 + threadIdx.x;
  const int64_t rend = min(r0 + kEncThreads, g.nrows);
  const int64_t b0 = offs[r0], b1 = offs[rend];
  if (b1 - b0 <= kGenImg && b1 <= cap) {
    if (r < g.nrows) put_row<true, kRoot>(nodes, g.ntop, r, (LdsU8*)(img + (offs[r] - b0)));
    __syncthreads();
    const uint64_t* s = reinterpret_cast<const uint64_t*>(img);
    uint64_t* d = reinterpret_cast<uint64_t*>(rows + b0);
    for (int64_t i = threadIdx.x; i < (b1 - b0) >> 3; i += kEncThreads) d[i] = s[i];
    return;
  }
  if (r < g.nrows && offs[r + 1] <= cap) put_row<true, kRoot>(nodes, g.ntop, r, rows + offs[r]);
}

// ---- decode ----------------------------------------------------------------------------------
// Per thread, per node: running Arrow entry index and payload byte position -- in LDS (stride 1,
// bytes after the nnodes entries), or, for schemas wider than the LDS budget, in the plan's
// per-(node, row) count array itself (stride 2 * nrows: the row's own slots).
struct Cursors {
  int64_t* base;
  int64_t sn;        // stride between nodes
  int64_t ob;        // offset of the byte cursors
  uint64_t* vmask;   // row-aligned nodes: validity bit of this row's entry, by node index
  uint64_t* bmask;   // row-aligned BOOL nodes: value bit of this row's entry
  __device__ __forceinline__ int64_t& e(int ni) const { return base[ni * sn]; }
  __device__ __forceinline__ int64_t& b(int ni) const { return base[ni * sn + ob]; }
};

template <int D, bool W>
__device__ void get_value(const GenNode* nodes, int ni, bool present, const uint8_t* base,
                          int64_t slot_addr, int es, bool in_array, const uint8_t* bitmap,
                          int64_t ordinal, Cursors cur);

// Elements of a BinaryArray at `arr` into node ei's Arrow column (m entries).
template <int D, bool W>
__device__ void get_array(const GenNode* nodes, int ei, const uint8_t* arr, int64_t m, Cursors cur) {
  const GenNode& e = nodes[ei];
  const int w = gwidth(e.type);
  const int es = w > 0 ? w : 8;
  const int64_t hb = 8 + gbm(m);
  for (int64_t j = 0; j < m; j++)
    get_value<D + 1, W>(nodes, ei, true, arr, hb + j * es, es, true, arr + 8, j, cur);
}

// A null (or absent) entry for node ni and, for structs, one null entry in every child.
template <int D, bool W>
__device__ void null_entry(const GenNode* nodes, int ni, Cursors cur) {
  if constexpr (D >= kGenMaxDepth) {
    return;
  } else {
    const GenNode& n = nodes[ni];
    const int64_t e = cur.e(ni)++;
    if (W) {
      const int w = gwidth(n.type);
      if (w > 0 && n.type != FURY_TYPE_BOOL && n.values) {
        uint8_t* p = const_cast<uint8_t*>(n.values) + e * w;
        for (int t = 0; t < w; t++) p[t] = 0;
      } else if (n.type == FURY_TYPE_DECIMAL && n.values) {
        st8(const_cast<uint8_t*>(n.values) + 16 * e, 0);
        st8(const_cast<uint8_t*>(n.values) + 16 * e + 8, 0);
      } else if (n.offsets) {                          // zero-length string / list / map
        const int64_t pos = (n.type == FURY_TYPE_STRING || n.type == FURY_TYPE_BINARY)
                                ? cur.b(ni) : cur.e(n.first_child);
        n.offsets[e + 1] = static_cast<int32_t>(pos);
      }
    }
    if (n.type == FURY_TYPE_STRUCT)
      for (int k = 0; k < n.num_children; k++) null_entry<D + 1, W>(nodes, n.first_child + k, cur);
  }
}

__device__ __forceinline__ void set_valid_bit(uint8_t* bits, int64_t i) {
  uint32_t* wp = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(bits + (i >> 3)) & ~uintptr_t(3));
  const int sh = static_cast<int>((reinterpret_cast<uintptr_t>(bits + (i >> 3)) & 3) * 8 + (i & 7));
  atomicOr(wp, 1u << sh);
}

template <int D, bool W>
__device__ void get_value(const GenNode* nodes, int ni, bool present, const uint8_t* base,
                          int64_t slot_addr, int es, bool in_array, const uint8_t* bitmap,
                          int64_t ordinal, Cursors cur) {
  if constexpr (D >= kGenMaxDepth) {
    return;
  } else {
    const GenNode& n = nodes[ni];
    const bool isnull = !present || ((bitmap[ordinal >> 3] >> (ordinal & 7)) & 1);
    if (isnull) {
      null_entry<D, W>(nodes, ni, cur);
      return;
    }
    const int64_t e = cur.e(ni)++;
    if (W && n.validity) {
      if (n.row_aligned && ni < 64) *cur.vmask |= 1ull << ni;   // a wave ballot (entry = row)
      else set_valid_bit(n.validity, e);
    }
    const uint8_t* sp = base + slot_addr;
    const int w = gwidth(n.type);
    if (w > 0) {
      if (!W) return;
      uint64_t v;
      if (es == 8) v = ld8(sp);
      else if (es == 4) v = *reinterpret_cast<const uint32_t*>(sp);
      else if (es == 2) v = *reinterpret_cast<const uint16_t*>(sp);
      else v = *sp;
      uint8_t* dst = const_cast<uint8_t*>(n.values);
      if (!dst) return;
      if (n.type == FURY_TYPE_BOOL) {
        if (v & 0xff) {
          if (n.row_aligned && ni < 64) *cur.bmask |= 1ull << ni;
          else set_valid_bit(dst, e);
        }
      } else if (w == 8) {
        st8(dst + 8 * e, v);
      } else if (w == 4) {
        *reinterpret_cast<uint32_t*>(dst + 4 * e) = static_cast<uint32_t>(v);
      } else if (w == 2) {
        *reinterpret_cast<uint16_t*>(dst + 2 * e) = static_cast<uint16_t>(v);
      } else {
        dst[e] = static_cast<uint8_t>(v);
      }
      return;
    }
    const uint64_t oas = ld8(sp);
    const uint8_t* vp = base + static_cast<int32_t>(oas >> 32);
    const int64_t size = static_cast<uint32_t>(oas);
    switch (n.type) {
      case FURY_TYPE_STRING:
      case FURY_TYPE_BINARY: {
        const int64_t pos = cur.b(ni);
        cur.b(ni) = pos + size;
        if (W) {
          uint8_t* dst = const_cast<uint8_t*>(n.values);
          if (dst) copy_to_unaligned(dst + pos, vp, size);
          n.offsets[e + 1] = static_cast<int32_t>(pos + size);
        }
        return;
      }
      case FURY_TYPE_DECIMAL:
        if (W && n.values) {
          st8(const_cast<uint8_t*>(n.values) + 16 * e, ld8(vp));
          st8(const_cast<uint8_t*>(n.values) + 16 * e + 8, ld8(vp + 8));
        }
        return;
      case FURY_TYPE_LIST: {
        const int64_t m = static_cast<int32_t>(ld8(vp));
        get_array<D, W>(nodes, n.first_child, vp, m, cur);
        if (W) n.offsets[e + 1] = static_cast<int32_t>(cur.e(n.first_child));
        return;
      }
      case FURY_TYPE_STRUCT: {
        const int nc = n.num_children;
        const int64_t bmb = gbm(nc);
        for (int k = 0; k < nc; k++)
          get_value<D + 1, W>(nodes, n.first_child + k, true, vp, bmb + 8 * k, 8, false, vp, k, cur);
        return;
      }
      case FURY_TYPE_MAP: {
        const int64_t key_bytes = static_cast<int64_t>(ld8(vp));
        const uint8_t* ka = vp + 8;
        const uint8_t* va = vp + 8 + key_bytes;
        const int64_t m = static_cast<int32_t>(ld8(ka));
        get_array<D, W>(nodes, n.first_child, ka, m, cur);
        get_array<D, W>(nodes, n.first_child + 1, va, m, cur);
        if (W) n.offsets[e + 1] = static_cast<int32_t>(cur.e(n.first_child));
        return;
      }
      default:
        return;
    }
  }
}

// Pass 1 (W = false): per row, per node, Arrow entries and payload bytes -> cnt[2*node][row],
// cnt[2*node+1][row].  Pass 2 (W = true): cursors start at the scanned positions.
// The per-thread cursors live in dynamic LDS sized for the schema's node count (2 x 8 B x
// nnodes per thread), so small schemas keep many workgroups per CU (a fixed kGenMaxNodes-sized
// array held this latency-bound interpreter to 3 waves per CU).
template <bool W, bool kWide>
__global__ __launch_bounds__(kThreads) void gen_decode_kernel(GenArgs g, const uint8_t* __restrict__ rows,
                                                              const int64_t* __restrict__ offs,
                                                              int64_t* __restrict__ cnt) {
  static_assert(kThreads == 64, "one wave = 64 consecutive rows (ballot bitmap words)");
  extern __shared__ int64_t cur_lds[];
  __shared__ GenNode sn[kWide ? 1 : kGenMaxNodes];
  const GenNode* nodes = stage_nodes<kWide>(g, sn);
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  const bool live = r < g.nrows;
  uint64_t vmask = 0, bmask = 0;
  if (live) {
    Cursors cur;
    if (kWide) {             // cursors = the row's slots of the count array (see Cursors)
      cur = Cursors{cnt + r, 2 * g.nrows, g.nrows, &vmask, &bmask};
      if (!W)
        for (int i = 0; i < g.nnodes; i++) cur.e(i) = cur.b(i) = 0;
    } else {
      cur = Cursors{cur_lds + threadIdx.x * (2 * g.nnodes), 1, g.nnodes, &vmask, &bmask};
      for (int i = 0; i < g.nnodes; i++) {
        cur.e(i) = W ? cnt[(2 * i) * g.nrows + r] : 0;
        cur.b(i) = W ? cnt[(2 * i + 1) * g.nrows + r] : 0;
      }
    }
    int64_t* e = &cur.e(0);
    const uint8_t* row = rows + offs[r];
    const int64_t bmb = gbm(g.ntop);
    if (g.root) {        // a top-level BinaryArray / BinaryMap: node 0's entry r
      const GenNode& n = nodes[0];
      const int64_t en = cur.e(0)++;
      if (W && n.validity) vmask |= 1ull;
      const uint8_t* ka = g.root == 2 ? row + 8 : row;
      const int64_t m = static_cast<int32_t>(ld8(ka));
      get_array<1, W>(nodes, n.first_child, ka, m, cur);
      if (g.root == 2) get_array<1, W>(nodes, n.first_child + 1, row + 8 + static_cast<int64_t>(ld8(row)), m, cur);
      if (W) n.offsets[en + 1] = static_cast<int32_t>(cur.e(n.first_child));
    } else {
      for (int k = 0; k < g.ntop; k++)
        get_value<1, W>(nodes, k, true, row, bmb + 8 * k, 8, false, row, k, cur);
    }
    (void)e;
    if (!W && !kWide) {
      for (int i = 0; i < g.nnodes; i++) {
        cnt[(2 * i) * g.nrows + r] = cur.e(i);
        cnt[(2 * i + 1) * g.nrows + r] = cur.b(i);
      }
    }
  }
  if (!W) return;
  // row-aligned nodes: the wave's 64 rows are 64 consecutive Arrow entries, so their validity /
  // bool bits are two whole 32-bit words (no atomics; the host zeroes nothing for them)
  const int lane = threadIdx.x;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kThreads;
  const int64_t left = g.nrows - r0;
  const int nwords = left >= 64 ? 2 : static_cast<int>((left + 31) >> 5);
  for (int i = 0; i < g.nnodes; i++) {
    const GenNode& n = nodes[i];
    if (!n.row_aligned || i >= 64) continue;   // nodes >= 64: per-entry atomics (get_value)
    if (n.validity) {
      const uint64_t bits = __ballot(live && ((vmask >> i) & 1));
      if (lane < nwords)
        reinterpret_cast<uint32_t*>(n.validity)[(r0 >> 5) + lane] = static_cast<uint32_t>(bits >> (32 * lane));
    }
    if (n.type == FURY_TYPE_BOOL && n.values) {
      const uint64_t bits = __ballot(live && ((bmask >> i) & 1));
      if (lane < nwords)
        reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(n.values))[(r0 >> 5) + lane] =
            static_cast<uint32_t>(bits >> (32 * lane));
    }
  }
}

__global__ void seg_bases(const int64_t* __restrict__ s, int64_t nseq, int64_t len,
                          const int64_t* __restrict__ grand, int64_t* __restrict__ bases,
                          int64_t* __restrict__ totals) {
  const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= nseq) return;
  const int64_t b = s[q * len];
  const int64_t e = q + 1 < nseq ? s[(q + 1) * len] : *grand;
  bases[q] = b;
  totals[q] = e - b;
}

__global__ void seg_unbase(int64_t* __restrict__ s, int64_t n, int64_t len,
                           const int64_t* __restrict__ bases) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) s[i] -= bases[i / len];
}

size_t cursor_lds(const GenArgs& g) {
  return static_cast<size_t>(kThreads) * 2 * (g.nnodes > 0 ? g.nnodes : 1) * sizeof(int64_t);
}

// Arrow offsets start at 0 for every node that has them.
__global__ void gen_offsets_zero(GenArgs g) {
  for (int i = threadIdx.x; i < g.nnodes; i += blockDim.x) {
    const GenNode& n = g.tab ? g.tab[i] : g.node[i];
    if (n.offsets) n.offsets[0] = 0;
  }
}

}  // namespace

template <bool kWide, int kRoot>
void gen_encode_pass(const GenArgs& g, const int64_t* offs, int64_t* sizes, uint8_t* rows,
                     int64_t cap, hipStream_t stream) {
  const int64_t blocks = (g.nrows + kEncThreads - 1) / kEncThreads;
  if (sizes) {
    hipLaunchKernelGGL((gen_measure_kernel<kWide, kRoot>), dim3(blocks), dim3(kEncThreads), 0,
                       stream, g, sizes);
    return;
  }
  static const bool lds_ok = hipFuncSetAttribute(
      reinterpret_cast<const void*>(gen_encode_kernel<kWide, kRoot>),
      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kGenImg)) == hipSuccess;
  (void)lds_ok;
  hipLaunchKernelGGL((gen_encode_kernel<kWide, kRoot>), dim3(blocks), dim3(kEncThreads), kGenImg,
                     stream, g, offs, rows, cap);
}

template <bool kWide>
void gen_encode_root(const GenArgs& g, const int64_t* offs, int64_t* sizes, uint8_t* rows,
                     int64_t cap, hipStream_t stream) {
  switch (g.root) {
    case 1: return gen_encode_pass<kWide, 1>(g, offs, sizes, rows, cap, stream);
    case 2: return gen_encode_pass<kWide, 2>(g, offs, sizes, rows, cap, stream);
    default: return gen_encode_pass<kWide, 0>(g, offs, sizes, rows, cap, stream);
  }
}

int launch_gen_measure(const GenArgs& g, int64_t* sizes, hipStream_t stream) {
  if (g.tab) gen_encode_root<true>(g, nullptr, sizes, nullptr, 0, stream);
  else gen_encode_root<false>(g, nullptr, sizes, nullptr, 0, stream);
  return check_hip(hipGetLastError(), "gen_measure launch");
}

int launch_gen_encode(const GenArgs& g, const int64_t* offs, uint8_t* rows, int64_t cap,
                      hipStream_t stream) {
  if (g.tab) gen_encode_root<true>(g, offs, nullptr, rows, cap, stream);
  else gen_encode_root<false>(g, offs, nullptr, rows, cap, stream);
  return check_hip(hipGetLastError(), "gen_encode launch");
}

int launch_gen_count(const GenArgs& g, const uint8_t* rows, const int64_t* offs, int64_t* cnt,
                     hipStream_t stream) {
  const int64_t blocks = (g.nrows + kThreads - 1) / kThreads;
  if (g.tab)
    hipLaunchKernelGGL((gen_decode_kernel<false, true>), dim3(blocks), dim3(kThreads), 0, stream,
                       g, rows, offs, cnt);
  else
    hipLaunchKernelGGL((gen_decode_kernel<false, false>), dim3(blocks), dim3(kThreads),
                       cursor_lds(g), stream, g, rows, offs, cnt);
  return check_hip(hipGetLastError(), "gen_count launch");
}

// `cnt` holds the scanned start positions; a wide schema's write pass advances its cursors in
// place, so it runs on a copy (`scratch`, same size) and the plan stays reusable.
int launch_gen_decode(const GenArgs& g, const uint8_t* rows, const int64_t* offs, int64_t* cnt,
                      int64_t* scratch, hipStream_t stream) {
  hipLaunchKernelGGL(gen_offsets_zero, dim3(1), dim3(256), 0, stream, g);
  const int64_t blocks = (g.nrows + kThreads - 1) / kThreads;
  if (g.tab) {
    const int st = check_hip(hipMemcpyAsync(scratch, cnt, 2 * g.nnodes * g.nrows * 8,
                                            hipMemcpyDeviceToDevice, stream), "cursor copy");
    if (st) return st;
    hipLaunchKernelGGL((gen_decode_kernel<true, true>), dim3(blocks), dim3(kThreads), 0, stream,
                       g, rows, offs, scratch);
  } else {
    hipLaunchKernelGGL((gen_decode_kernel<true, false>), dim3(blocks), dim3(kThreads),
                       cursor_lds(g), stream, g, rows, offs, cnt);
  }
  return check_hip(hipGetLastError(), "gen_decode launch");
}

// nseq independent exclusive scans of len entries each (s[q * len + i]), totals[q] = sequence
// sums: ONE scan over the concatenation, then every sequence minus its starting prefix (instead
// of a 3-kernel scan per sequence: the nested decode has 2 x nodes sequences).
// ws: scan_workspace(nseq * len) + 2 * nseq + 1 entries.
int device_scan_batched(int64_t* s, int64_t nseq, int64_t len, int64_t* totals, int64_t* ws,
                        hipStream_t stream) {
  const int64_t n = nseq * len;
  int64_t* grand = ws;
  int64_t* bases = ws + 1;
  int64_t* sws = ws + 1 + nseq;
  device_scan(s, n, grand, sws, stream);
  hipLaunchKernelGGL(seg_bases, dim3(static_cast<unsigned>((nseq + 255) / 256)), dim3(256), 0, stream,
                     s, nseq, len, grand, bases, totals);
  hipLaunchKernelGGL(seg_unbase, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream,
                     s, n, len, bases);
  return check_hip(hipGetLastError(), "batched scan launch");
}

}  // namespace fury
