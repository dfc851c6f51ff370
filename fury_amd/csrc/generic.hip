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
// build pass).  Recursion is depth-unrolled (template<int D>), at most kMaxDepth levels of
// nesting.  Decode is levels.hip (level by level, a thread per Arrow entry); the round-1/2
// thread-per-row decode interpreter that lived here was removed in round 3.
#include <hip/hip_runtime.h>

#include <atomic>

#include <cstring>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

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

// ---- tree tiles: the encode walked level by level on chip ------------------------------------
// A workgroup owns a tile of consecutive rows.  Phase R: every node's Arrow entry range for the
// tile, top-down (a struct child's = its parent's, a list / map child's = the parent's element
// range from its offsets).  The tile's inputs -- each node's validity bits, offsets, values,
// string payload -- are then contiguous ranges, staged into LDS by LDS-DMA in ONE round trip.
// Phase S (bottom-up): the encoded size of every non-scalar entry (a struct's = its fixed part +
// its children's; a list's = header + element slots + its elements' var parts, read as a
// difference of the element node's in-tile prefix: one block scan per level over the nodes below a
// list / map).  The measure pass stops here (row sizes).  The encode pass then places every value
// top-down in a zeroed LDS image of the tile's output bytes: a row / struct thread writes its null
// bits and slots and gives each var child its position; an element finds its list by binary search
// over the staged offsets and writes its own slot and null bit; a string copies its staged payload.
// Every phase spreads ALL (node, entry) pairs of a level over the workgroup (node records in LDS).
// The image leaves as one contiguous range.  Tiles whose inputs + arrays + image do not fit the
// LDS budget are walked in halves; a single row that does not fit is encoded by the row
// interpreter above (te_fixup_kernel), straight to HBM.
struct TENode {
  const uint8_t* values;
  const uint8_t* validity;
  const int32_t* offsets;
  int32_t type;
  int32_t first_child;
  int32_t num_children;
  int32_t parent;           // -1: top-level field
  int32_t ord;              // index among the parent's children
  int32_t width;            // scalar bytes (BOOL: 1), -1 otherwise
  int32_t esize;            // slot bytes as an array element
  int32_t level;
};

constexpr int kTEMaxLevels = 64;
constexpr int kTEThreads = 256;

struct TEArgs {
  const TENode* nodes;
  const GenNode* gtab;      // the same schema for the row interpreter (single-row fallback)
  const int64_t* offs;      // encode: row offsets (input)
  int64_t* sizes;           // measure: row sizes (output)
  uint8_t* rows;
  int64_t nrows;
  int64_t cap;
  int32_t nn, ntop, root, nlevels;
  int32_t tile_rows;
  uint32_t lds_cap;
  uint32_t* fallback;       // bit r: row r is left to te_fixup_kernel (zeroed by the launcher)
  uint64_t* dbg;            // diagnostics (tuning "tree_debug"): phase times, or NULL
  uint32_t* err;            // the stream's device error slot
  int32_t deep;             // nested deeper than the row interpreter unrolls
  int32_t pad_;
  int32_t level_start[kTEMaxLevels + 1];
  int32_t nelem[kTEMaxLevels];   // per level: non-scalar LIST / MAP elements (first in `ord`)
};

#define TEMARK(sh, id)                                                             \
  do {                                                                             \
    if ((sh).tacc && threadIdx.x == 0) {                                           \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                        \
      (sh).tacc[id] += t_ - (sh).tacc[15];                                         \
      (sh).tacc[15] = t_;                                                          \
    }                                                                              \
  } while (0)

struct EMeta {
  int64_t lo;               // first Arrow entry of the node in the (sub-)tile
  int64_t plo;              // STRING / BINARY: first payload byte (offsets[lo])
  int64_t phi;              // STRING / BINARY: payload end (offsets[lo + cnt])
  uint32_t cnt;             // entries in the (sub-)tile
  uint32_t vst, ost, pst;   // LDS: validity byte lo / 8, offsets[lo], values / payload start
  uint32_t S;               // LDS: sizes -> prefixes -> positions (non-scalar nodes), cnt + 1
  uint32_t X;               // LDS: LIST: element var base; MAP: + value array pos, value var base
};

constexpr uint32_t kTNone = 0xffffffffu;
constexpr uint32_t kTDead = 0xffffffffu;

__device__ __forceinline__ bool te_scalar(int t) { return gwidth(t) > 0; }
__device__ __forceinline__ uint32_t r8u(uint32_t n) { return (n + 7) & ~7u; }
__device__ __forceinline__ uint32_t bmu(uint32_t n) { return ((n + 63) >> 6) << 3; }

// LDS-DMA of the 16-B pieces covering [gb, ge) at pool + at (at 16-aligned, advanced); returns the
// LDS offset of byte gb, or kTNone when the pieces do not fit below cap (nothing issued).
__device__ __forceinline__ uint32_t te_stage(uint8_t* pool, uint32_t& at, uint32_t cap,
                                             const uint8_t* gb, const uint8_t* ge) {
  if (ge <= gb) return at;
  const uint64_t lo = reinterpret_cast<uint64_t>(gb) & ~uint64_t(15);
  const uint64_t hi = (reinterpret_cast<uint64_t>(ge) + 15) & ~uint64_t(15);
  const uint64_t bytes = hi - lo;
  if (at + bytes > cap) return kTNone;
  const uint32_t nch = static_cast<uint32_t>(bytes >> 4);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t i0 = wave * 64; i0 < nch; i0 += kTEThreads)
    if (i0 + lane < nch)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(lo + 16ull * (i0 + lane)),
                                       pool + at + 16 * i0, 16, 0, 0);
  const uint32_t r = at + static_cast<uint32_t>(reinterpret_cast<uint64_t>(gb) - lo);
  at += static_cast<uint32_t>(bytes);
  return r;
}

__device__ __forceinline__ uint64_t te_wscan(uint64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Exclusive scan of uint32 a[0, m) (LDS) by the block (thread t owns a contiguous chunk).
__device__ void te_block_scan(uint32_t* a, uint32_t m, uint64_t* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t per = (m + kTEThreads - 1) / kTEThreads;
  const uint32_t b = min<uint32_t>(tid * per, m), e = min<uint32_t>(b + per, m);
  uint64_t s = 0;
  for (uint32_t i = b; i < e; i++) s += a[i];
  const uint64_t inc = te_wscan(s);
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint64_t pre = 0;
#pragma unroll
  for (int w = 0; w < kTEThreads / 64; w++) pre += w < wave ? wsum[w] : 0;
  uint64_t run = pre + inc - s;
  for (uint32_t i = b; i < e; i++) {
    const uint32_t v = a[i];
    a[i] = static_cast<uint32_t>(run);
    run += v;
  }
  __syncthreads();
}

__device__ __forceinline__ bool te_valid(const uint8_t* pool, const EMeta& m, int64_t q,
                                         const uint8_t* gvalid) {
  if (!gvalid) return true;
  const int64_t i = (m.lo & 7) + q;
  return (pool[m.vst + (i >> 3)] >> (i & 7)) & 1;
}
__device__ __forceinline__ int32_t te_off(const uint8_t* pool, const EMeta& m, int64_t q) {
  return reinterpret_cast<const int32_t*>(pool + m.ost)[q];
}
// Scalar value q of a node from its staged values (BOOL: bit-packed, as 0 / 1).
__device__ __forceinline__ uint64_t te_value(const uint8_t* pool, const EMeta& m, int t, int w, int64_t q) {
  if (t == FURY_TYPE_BOOL) {
    const int64_t i = (m.lo & 7) + q;
    return (pool[m.pst + (i >> 3)] >> (i & 7)) & 1;
  }
  const uint8_t* p = pool + m.pst + q * w;
  switch (w) {
    case 8: return *reinterpret_cast<const uint64_t*>(p);
    case 4: return *reinterpret_cast<const uint32_t*>(p);
    case 2: return *reinterpret_cast<const uint16_t*>(p);
    default: return *p;
  }
}

// Encoded size of entry q of non-scalar node n (children's sizes / prefixes already in place).
__device__ uint32_t te_size(const TENode* D, const uint8_t* pool, const EMeta* meta, int n, int64_t q) {
  const TENode& N = D[n];
  const EMeta& M = meta[n];
  if (!te_valid(pool, M, q, N.validity)) return 0;
  switch (N.type) {
    case FURY_TYPE_STRING:
    case FURY_TYPE_BINARY:
      return r8u(static_cast<uint32_t>(te_off(pool, M, q + 1) - te_off(pool, M, q)));
    case FURY_TYPE_DECIMAL:
      return 16;
    case FURY_TYPE_STRUCT: {
      const int nc = N.num_children;
      uint32_t sz = bmu(nc) + 8 * nc;
      for (int k = 0; k < nc; k++) {
        const int c = N.first_child + k;
        if (te_scalar(D[c].type)) continue;
        sz += reinterpret_cast<const uint32_t*>(pool + meta[c].S)[q];
      }
      return sz;
    }
    case FURY_TYPE_LIST:
    case FURY_TYPE_MAP: {
      const int32_t o0 = te_off(pool, M, q), o1 = te_off(pool, M, q + 1);
      const uint32_t m = static_cast<uint32_t>(o1 - o0);
      uint32_t sz = N.type == FURY_TYPE_MAP ? 8 : 0;
      for (int k = 0; k < (N.type == FURY_TYPE_MAP ? 2 : 1); k++) {
        const int c = N.first_child + k;
        const TENode& C = D[c];
        sz += 8 + bmu(m) + r8u(m * C.esize);
        if (!te_scalar(C.type)) {
          const uint32_t* P = reinterpret_cast<const uint32_t*>(pool + meta[c].S);
          const int64_t b = o0 - meta[c].lo;
          sz += P[b + m] - P[b];
        }
      }
      return sz;
    }
    default:
      return 0;
  }
}

// The unpadded size a slot records for a non-null value at entry q of node n with encoded size sz.
__device__ __forceinline__ uint32_t te_raw(const TENode* D, const uint8_t* pool, const EMeta* meta,
                                           int n, int64_t q, uint32_t sz) {
  const int t = D[n].type;
  if (t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY)
    return static_cast<uint32_t>(te_off(pool, meta[n], q + 1) - te_off(pool, meta[n], q));
  return sz;
}

// A struct-like container (a row: children = the top-level fields, or entry q of a STRUCT node)
// at image position pos: null bits and slots of its children; non-scalar children get their
// positions (in place of their sizes; kTDead when null / dead).  lim = image bytes (writes past it
// are dropped).
__device__ void te_put_struct(const TENode* D, uint8_t* pool, const EMeta* meta, uint8_t* img,
                              uint32_t lim, int fc, int nc, int64_t q, uint32_t pos, bool dead) {
  const uint32_t fixed = bmu(nc) + 8 * nc;
  uint32_t run = pos + fixed;
  if (!dead && pos + fixed > lim) dead = true;
  for (int w = 0; w < (nc + 63) / 64; w++) {
    uint64_t nulls = 0;
    for (int k = 64 * w; k < min(nc, 64 * w + 64); k++) {
      const int c = fc + k;
      const TENode& C = D[c];
      const bool valid = !dead && te_valid(pool, meta[c], q, C.validity);
      if (!valid) nulls |= 1ull << (k - 64 * w);
      uint64_t slot = 0;
      if (te_scalar(C.type)) {
        if (valid) slot = te_value(pool, meta[c], C.type, C.width, q);
      } else {
        uint32_t* S = reinterpret_cast<uint32_t*>(pool + meta[c].S);
        const uint32_t sz = S[q];
        if (valid) {
          slot = (static_cast<uint64_t>(run - pos) << 32) | te_raw(D, pool, meta, c, q, sz);
          S[q] = run;
          run += sz;
        } else {
          S[q] = kTDead;
        }
      }
      if (!dead) *reinterpret_cast<uint64_t*>(img + pos + bmu(nc) + 8 * k) = slot;
    }
    if (!dead) *reinterpret_cast<uint64_t*>(img + pos + 8 * w) = nulls;
  }
}

// Owner of child entry g (global Arrow index) among the nc entries of a LIST / MAP node whose
// staged offsets are O[0, nc]: the last e with O[e] <= g.
__device__ __forceinline__ uint32_t te_owner(const int32_t* O, uint32_t nc, int64_t g) {
  uint32_t lo = 0, hi = nc;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (O[mid] <= g) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void te_store_w(uint8_t* p, int w, uint64_t v) {
  switch (w) {
    case 8: *reinterpret_cast<uint64_t*>(p) = v; break;
    case 4: *reinterpret_cast<uint32_t*>(p) = static_cast<uint32_t>(v); break;
    case 2: *reinterpret_cast<uint16_t*>(p) = static_cast<uint16_t>(v); break;
    default: *p = static_cast<uint8_t>(v); break;
  }
}

// Slot k of a level's flattened (node, entry) list: cum[k] - cum[0] <= i < cum[k + 1] - cum[0].
__device__ __forceinline__ int te_item(const uint32_t* cum, int nk, uint32_t i) {
  const uint32_t x = i + cum[0];
  int lo = 0, hi = nk;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cum[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

// LDS working set of te_kernel: [node records][layout order][meta][wsum, wtot][ex][diag][pool].
constexpr int kTEScans = 7;
struct TEShared {
  TENode* D;
  int32_t* ord;             // layout order: level by level, each level's non-scalar elements of a
                            // LIST / MAP first (their size arrays are one scanned block), then its
                            // other non-scalar nodes, then its scalars
  EMeta* meta;
  uint64_t* wsum;
  uint32_t* wtot;
  uint32_t* ex;             // [kTEScans][nn + 1] layout scans over `ord`
  uint8_t* pool;
  uint64_t* tacc;           // diagnostics: 16 phase accumulators (NULL when off)
};

__host__ __device__ inline size_t te_lds_head(int nn) {
  size_t b = (sizeof(TENode) + 4 + sizeof(EMeta)) * static_cast<size_t>(nn);
  b = (b + 7) & ~size_t(7);
  b += 64 + 4 * kTEScans * (kTEThreads / 64);            // wsum, wtot
  b += 4 * kTEScans * static_cast<size_t>(nn + 1);        // ex
  b = (b + 7) & ~size_t(7);
  b += 128;                                               // diagnostics
  return (b + 15) & ~size_t(15);
}

// Walks rows [s0, s1).  Returns false when the LDS budget does not hold it (uniform).
template <bool kWrite>
__device__ bool te_walk(const TEArgs& a, const TEShared& sh, int64_t s0, int64_t s1) {
  const int tid = threadIdx.x;
  const uint32_t nr = static_cast<uint32_t>(s1 - s0);
  const TENode* D = sh.D;
  EMeta* meta = sh.meta;
  uint8_t* pool = sh.pool;
  const int nn = a.nn;
  TEMARK(sh, 7);
  // ---- R: entry ranges, top-down (a thread per node of the level)
  for (int L = 0; L < a.nlevels; L++) {
    const int nb = a.level_start[L], ne = a.level_start[L + 1];
    for (int n = nb + tid; n < ne; n += kTEThreads) {
      const TENode& N = D[n];
      int64_t lo, cnt;
      if (L == 0) {
        lo = s0;
        cnt = nr;
      } else {
        const EMeta& P = meta[N.parent];
        const TENode& PN = D[N.parent];
        if (PN.type == FURY_TYPE_STRUCT) {
          lo = P.lo;
          cnt = P.cnt;
        } else {
          lo = gl(PN.offsets)[P.lo];
          cnt = gl(PN.offsets)[P.lo + P.cnt] - lo;
        }
      }
      meta[n].lo = lo;
      meta[n].cnt = static_cast<uint32_t>(cnt);
      if (N.type == FURY_TYPE_STRING || N.type == FURY_TYPE_BINARY) {
        meta[n].plo = cnt ? gl(N.offsets)[lo] : 0;
        meta[n].phi = cnt ? gl(N.offsets)[lo + cnt] : 0;
      }
    }
    __syncthreads();
  }
  TEMARK(sh, 0);
  // ---- layout of everything the walk keeps in LDS: block scans over the nodes (in `ord`) of the
  // staged validity / offsets / values pieces, the size and LIST / MAP extra arrays, and each
  // level's size-phase (S) and position-phase (P) entries
  const uint32_t cap = a.lds_cap;
  const int32_t* ord = sh.ord;
  auto stage_span = [&](const uint8_t* gb, const uint8_t* ge) -> uint32_t {
    if (ge <= gb) return 0u;
    const uint64_t lo = reinterpret_cast<uint64_t>(gb) & ~uint64_t(15);
    const uint64_t hi = (reinterpret_cast<uint64_t>(ge) + 15) & ~uint64_t(15);
    return static_cast<uint32_t>(hi - lo);
  };
  auto value_span = [&](const TENode& N, const EMeta& M, const uint8_t** gb, const uint8_t** ge) {
    const int t = N.type;
    const int64_t lo = M.lo, cnt = M.cnt;
    *gb = *ge = nullptr;
    if (cnt == 0) return;
    if (t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY) {
      *gb = N.values + M.plo;
      *ge = N.values + M.phi;
    } else if (t == FURY_TYPE_BOOL) {
      *gb = N.values + (lo >> 3);
      *ge = N.values + ((lo + cnt + 7) >> 3);
    } else if (t == FURY_TYPE_DECIMAL) {
      *gb = N.values + 16 * lo;
      *ge = N.values + 16 * (lo + cnt);
    } else if (N.width > 0) {
      *gb = N.values + N.width * lo;
      *ge = N.values + N.width * (lo + cnt);
    }
  };
  uint32_t* ex = sh.ex;
  const int M1 = nn + 1;
  block_scan_k<kTEThreads, kTEScans>(nn, [&](int j, int k) -> uint32_t {
    const int n = ord[j];
    const TENode& N = D[n];
    const EMeta& M = meta[n];
    const int t = N.type;
    const uint32_t cnt = M.cnt;
    const bool sc = te_scalar(t);
    switch (k) {
      case 0:
        return cnt && N.validity ? stage_span(N.validity + (M.lo >> 3), N.validity + ((M.lo + cnt + 7) >> 3)) : 0u;
      case 1:
        return cnt && (t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY || t == FURY_TYPE_LIST ||
                       t == FURY_TYPE_MAP)
                   ? stage_span(reinterpret_cast<const uint8_t*>(N.offsets + M.lo),
                                reinterpret_cast<const uint8_t*>(N.offsets + M.lo + cnt + 1))
                   : 0u;
      case 2: {
        if (!kWrite) return 0u;
        const uint8_t *gb, *ge;
        value_span(N, M, &gb, &ge);
        return stage_span(gb, ge);
      }
      case 3:
        return sc ? 0u : 4 * (cnt + 1);
      case 4:
        return kWrite && (t == FURY_TYPE_LIST || t == FURY_TYPE_MAP) ? 4 * cnt * (t == FURY_TYPE_MAP ? 3 : 1) : 0u;
      case 5:
        return sc ? 0u : cnt;
      default: {
        const bool elem = N.parent >= 0 && (D[N.parent].type == FURY_TYPE_LIST || D[N.parent].type == FURY_TYPE_MAP);
        return (!sc || elem) ? cnt : 0u;
      }
    }
  }, ex, sh.wtot);
  const uint32_t vbase = 0, obase = ex[0 * M1 + nn], pbase = obase + ex[1 * M1 + nn];
  const uint32_t sbase = (pbase + ex[2 * M1 + nn] + 15) & ~15u;
  const uint32_t xbase = (sbase + ex[3 * M1 + nn] + 15) & ~15u;
  const uint32_t img_at = (xbase + ex[4 * M1 + nn] + 15) & ~15u;
  uint32_t lim = 0;
  if (kWrite) {
    const int64_t bytes = gl(a.offs)[s1] - gl(a.offs)[s0];
    if (bytes < 0 || img_at + bytes + 16 > cap) return false;
    lim = static_cast<uint32_t>(bytes);
  } else if (img_at > cap) {
    return false;
  }
  // meta of every node; its staged pieces issued by one wave
  const int wave = tid >> 6, lane = tid & 63;
  for (int j = tid; j < nn; j += kTEThreads) {
    const int n = ord[j];
    EMeta& M = meta[n];
    M.S = sbase + ex[3 * M1 + j];
    M.X = xbase + ex[4 * M1 + j];
  }
  for (int j = wave; j < nn; j += kTEThreads / 64) {
    const int n = ord[j];
    const TENode& N = D[n];
    EMeta& M = meta[n];
    const uint32_t off[3] = {vbase + ex[0 * M1 + j], obase + ex[1 * M1 + j], pbase + ex[2 * M1 + j]};
    const uint8_t* gb[3] = {nullptr, nullptr, nullptr};
    const uint8_t* ge[3] = {nullptr, nullptr, nullptr};
    if (M.cnt && N.validity) {
      gb[0] = N.validity + (M.lo >> 3);
      ge[0] = N.validity + ((M.lo + M.cnt + 7) >> 3);
    }
    if (M.cnt && (N.type == FURY_TYPE_STRING || N.type == FURY_TYPE_BINARY || N.type == FURY_TYPE_LIST ||
                  N.type == FURY_TYPE_MAP)) {
      gb[1] = reinterpret_cast<const uint8_t*>(N.offsets + M.lo);
      ge[1] = reinterpret_cast<const uint8_t*>(N.offsets + M.lo + M.cnt + 1);
    }
    if (kWrite) value_span(N, M, &gb[2], &ge[2]);
    uint32_t at3[3];
#pragma unroll
    for (int g = 0; g < 3; g++) {
      at3[g] = kTNone;
      if (!gb[g] || ge[g] <= gb[g]) {
        if (gb[g]) at3[g] = off[g];             // empty range: never read
        continue;
      }
      const uint64_t lo = reinterpret_cast<uint64_t>(gb[g]) & ~uint64_t(15);
      const uint32_t nch = stage_span(gb[g], ge[g]) >> 4;
      for (uint32_t i = lane; i < nch; i += 64)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(lo + 16ull * i),
                                         pool + off[g] + 16 * i, 16, 0, 0);
      at3[g] = off[g] + static_cast<uint32_t>(reinterpret_cast<uint64_t>(gb[g]) - lo);
    }
    if (lane == 0) {
      M.vst = at3[0];
      M.ost = at3[1];
      M.pst = at3[2];
    }
  }
  if (kWrite) {
    using v4 = __attribute__((ext_vector_type(4))) uint32_t;
    for (uint32_t i = 16 * tid; i < ((lim + 15) & ~15u); i += 16 * kTEThreads)
      *reinterpret_cast<v4*>(pool + img_at + i) = v4{0, 0, 0, 0};
  }
  TEMARK(sh, 1);
  __syncthreads();                               // staged inputs landed, meta and lists visible
  TEMARK(sh, 2);
  uint8_t* img = pool + img_at;
  // ---- S: sizes bottom-up (all non-scalar entries of a level at once); prefixes of the nodes
  // below a LIST / MAP (one scan per level)
  for (int L = a.nlevels - 1; L >= 0; L--) {
    const int j0 = a.level_start[L], j1 = a.level_start[L + 1];
    const uint32_t* cum = ex + 5 * M1;
    const uint32_t c0 = cum[j0], W = cum[j1] - c0;
    for (uint32_t i = tid; i < W; i += kTEThreads) {
      const int j = j0 + te_item(cum + j0, j1 - j0, i);
      const int n = ord[j];
      const uint32_t q = i + c0 - cum[j];
      uint32_t* S = reinterpret_cast<uint32_t*>(pool + meta[n].S);
      S[q] = te_size(D, pool, meta, n, q);
      if (q + 1 == meta[n].cnt) S[q + 1] = 0;
    }
    for (int j = j0 + tid; j < j1; j += kTEThreads) {
      const int n = ord[j];
      if (!te_scalar(D[n].type) && meta[n].cnt == 0) reinterpret_cast<uint32_t*>(pool + meta[n].S)[0] = 0;
    }
    __syncthreads();
    const int ne = a.nelem[L];                  // the level's first ne slots: elements, one block
    if (L > 0 && ne > 0) {
      const uint32_t b0 = ex[3 * M1 + j0], b1 = ex[3 * M1 + j0 + ne];
      if (b1 > b0) te_block_scan(reinterpret_cast<uint32_t*>(pool + sbase + b0), (b1 - b0) / 4, sh.wsum);
    }
  }
  TEMARK(sh, 3);
  // ---- row sizes (measure) / row containers (encode)
  for (uint32_t r = tid; r < nr; r += kTEThreads) {
    if (!kWrite) {
      uint64_t sz;
      if (a.root) {
        sz = reinterpret_cast<const uint32_t*>(pool + meta[0].S)[r];
      } else {
        sz = bmu(a.ntop) + 8ull * a.ntop;
        for (int k = 0; k < a.ntop; k++)
          if (!te_scalar(D[k].type)) sz += reinterpret_cast<const uint32_t*>(pool + meta[k].S)[r];
      }
      a.sizes[s0 + r] = static_cast<int64_t>(sz);
    } else {
      const int64_t b0 = gl(a.offs)[s0];
      const uint32_t pos = static_cast<uint32_t>(gl(a.offs)[s0 + r] - b0);
      if (a.root) reinterpret_cast<uint32_t*>(pool + meta[0].S)[r] = pos;
      else te_put_struct(D, pool, meta, img, lim, 0, a.ntop, r, pos, false);
    }
  }
  TEMARK(sh, 4);
  if (!kWrite) return true;
  __syncthreads();
  // ---- positions + contents, top-down (all element / non-scalar entries of a level at once)
  for (int L = 0; L < a.nlevels; L++) {
    const int j0 = a.level_start[L], j1 = a.level_start[L + 1];
    const uint32_t* cum = ex + 6 * M1;
    const uint32_t c0 = cum[j0], W = cum[j1] - c0;
    for (uint32_t i = tid; i < W; i += kTEThreads) {
      const int j = j0 + te_item(cum + j0, j1 - j0, i);
      const int n = ord[j];
      const uint32_t q = i + c0 - cum[j];
      const TENode& N = D[n];
      const EMeta& M = meta[n];
      const bool scalar = te_scalar(N.type);
      const int pt = L == 0 ? -1 : D[N.parent].type;
      const bool elem = pt == FURY_TYPE_LIST || pt == FURY_TYPE_MAP;
      uint32_t* S = scalar ? nullptr : reinterpret_cast<uint32_t*>(pool + M.S);
      uint32_t pos = scalar ? kTDead : S[q];
      if (elem) {                                // an element: its own slot in the parent array
        const EMeta& PM = meta[N.parent];
        const int32_t* O = reinterpret_cast<const int32_t*>(pool + PM.ost);
        const int64_t g = M.lo + q;
        const uint32_t e = te_owner(O, PM.cnt, g);
        const uint32_t j = static_cast<uint32_t>(g - O[e]);
        const uint32_t m = static_cast<uint32_t>(O[e + 1] - O[e]);
        const uint32_t ppos = reinterpret_cast<const uint32_t*>(pool + PM.S)[e];
        const uint32_t* PX = reinterpret_cast<const uint32_t*>(pool + PM.X);
        pos = kTDead;
        if (ppos != kTDead) {
          const uint32_t arr = pt == FURY_TYPE_LIST ? ppos : (N.ord == 0 ? ppos + 8 : PX[PM.cnt + e]);
          const bool valid = te_valid(pool, M, q, N.validity);
          const uint32_t sl = arr + 8 + bmu(m) + static_cast<uint32_t>(N.esize) * j;
          if (!valid) {
            if (arr + 8 + (j >> 3) < lim)
              atomicOr(reinterpret_cast<uint32_t*>(img + arr + 8) + (j >> 5), 1u << (j & 31));
          } else if (scalar) {
            if (sl + N.esize <= lim) te_store_w(img + sl, N.esize, te_value(pool, M, N.type, N.width, q));
          } else {
            const uint32_t base = N.ord == 0 ? PX[e] : PX[2 * PM.cnt + e];
            const uint32_t sz = te_size(D, pool, meta, n, q);
            pos = base + S[q];
            const uint64_t slot = (static_cast<uint64_t>(pos - arr) << 32) | te_raw(D, pool, meta, n, q, sz);
            if (sl + 8 <= lim) *reinterpret_cast<uint64_t*>(img + sl) = slot;
          }
        }
        if (scalar) continue;
        S[q] = pos;                              // (only this thread reads S[q] at this level)
      }
      if (pos == kTDead) {                       // a null / dead struct: its children are dead
        if (N.type == FURY_TYPE_STRUCT)
          te_put_struct(D, pool, meta, img, lim, N.first_child, N.num_children, q, 0, true);
        continue;
      }
      switch (N.type) {
        case FURY_TYPE_STRING:
        case FURY_TYPE_BINARY: {
          const int64_t o0 = te_off(pool, M, q), o1 = te_off(pool, M, q + 1);
          const uint8_t* src = pool + M.pst + (o0 - M.plo);
          const uint32_t len = static_cast<uint32_t>(o1 - o0);
          if (pos + len <= lim)
            for (uint32_t b = 0; b < len; b++) img[pos + b] = src[b];
          break;
        }
        case FURY_TYPE_DECIMAL: {
          const uint8_t* src = pool + M.pst + 16 * q;
          if (pos + 16 <= lim)
            for (int b = 0; b < 16; b++) img[pos + b] = src[b];
          break;
        }
        case FURY_TYPE_STRUCT:
          te_put_struct(D, pool, meta, img, lim, N.first_child, N.num_children, q, pos, false);
          break;
        case FURY_TYPE_LIST:
        case FURY_TYPE_MAP: {
          const int64_t o0 = te_off(pool, M, q), o1 = te_off(pool, M, q + 1);
          const uint32_t m = static_cast<uint32_t>(o1 - o0);
          uint32_t* X = reinterpret_cast<uint32_t*>(pool + M.X);
          uint32_t arr = N.type == FURY_TYPE_MAP ? pos + 8 : pos;
          for (int kk = 0; kk < (N.type == FURY_TYPE_MAP ? 2 : 1); kk++) {
            const int c = N.first_child + kk;
            const TENode& C = D[c];
            const uint32_t hdr = 8 + bmu(m) + r8u(m * C.esize);
            if (arr + 8 <= lim) *reinterpret_cast<uint64_t*>(img + arr) = m;
            uint32_t var = 0;
            if (!te_scalar(C.type)) {
              const uint32_t* P = reinterpret_cast<const uint32_t*>(pool + meta[c].S);
              const int64_t b = o0 - meta[c].lo;
              X[kk == 0 ? q : 2 * M.cnt + q] = arr + hdr - P[b];
              var = P[b + m] - P[b];
            }
            if (kk == 0 && N.type == FURY_TYPE_MAP) {
              const uint32_t kbytes = hdr + var;
              if (pos + 8 <= lim) *reinterpret_cast<uint64_t*>(img + pos) = kbytes;
              arr = pos + 8 + kbytes;
              X[M.cnt + q] = arr;
            }
          }
          break;
        }
        default:
          break;
      }
    }
    __syncthreads();
  }
  TEMARK(sh, 5);
  // ---- the image leaves as one contiguous range (bytes at or past cap are not written)
  const int64_t b0 = gl(a.offs)[s0];
  const int64_t end = min<int64_t>(static_cast<int64_t>(lim), a.cap - b0);
  const uint64_t* src = reinterpret_cast<const uint64_t*>(img);
  uint64_t* dst = reinterpret_cast<uint64_t*>(a.rows + b0);
  for (int64_t i = tid; i < (end >> 3); i += kTEThreads) __builtin_nontemporal_store(src[i], gl(dst) + i);
  TEMARK(sh, 6);
  return true;
}

// Rows the tree walk could not hold in LDS (one row beyond the budget): the row interpreter, in a
// kernel of its own (inlined into te_kernel it took 256 VGPRs and scratch from the whole walk).
template <bool kWrite, int kRoot>
__global__ __launch_bounds__(kTEThreads) void te_fixup_kernel(TEArgs a) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kTEThreads + threadIdx.x;
  if (r >= a.nrows || !((gl(a.fallback)[r >> 5] >> (r & 31)) & 1)) return;
  if (a.deep) {                                 // the interpreter cannot reach these levels
    raise_at(a.err, kErrTooDeep, static_cast<uint64_t>(r));
    if (!kWrite) a.sizes[r] = 0;
    return;
  }
  const GNodes gn = (GNodes)(a.gtab);
  if (!kWrite) a.sizes[r] = put_row<false, kRoot>(gn, a.ntop, r, static_cast<uint8_t*>(nullptr));
  else if (gl(a.offs)[r + 1] <= a.cap) put_row<true, kRoot>(gn, a.ntop, r, a.rows + gl(a.offs)[r]);
}

template <bool kWrite, int kRoot>
__global__ __launch_bounds__(kTEThreads) void te_kernel(TEArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tes[];
  TEShared sh;
  {
    const int nn = a.nn;
    uint8_t* p = tes;
    sh.D = reinterpret_cast<TENode*>(p);
    p += sizeof(TENode) * nn;
    sh.ord = reinterpret_cast<int32_t*>(p);
    p += 4 * nn;
    p = tes + ((p - tes + 7) & ~size_t(7));
    sh.meta = reinterpret_cast<EMeta*>(p);
    p += sizeof(EMeta) * nn;
    p = tes + ((p - tes + 7) & ~size_t(7));
    sh.wsum = reinterpret_cast<uint64_t*>(p);
    p += 64;
    sh.wtot = reinterpret_cast<uint32_t*>(p);
    p += 4 * kTEScans * (kTEThreads / 64);
    sh.ex = reinterpret_cast<uint32_t*>(p);
    p += 4 * kTEScans * (nn + 1);
    p = tes + ((p - tes + 7) & ~size_t(7));
    sh.tacc = a.dbg ? reinterpret_cast<uint64_t*>(p) : nullptr;
    sh.pool = tes + te_lds_head(nn);
  }
  if (sh.tacc && threadIdx.x < 16)
    sh.tacc[threadIdx.x] = threadIdx.x == 15 ? __builtin_amdgcn_s_memrealtime() : 0;
  {
    const int32_t* gord = reinterpret_cast<const int32_t*>(a.nodes + a.nn);
    for (int n = threadIdx.x; n < a.nn; n += kTEThreads) sh.ord[n] = gord[n];
  }
  for (int n = threadIdx.x; n < a.nn; n += kTEThreads) sh.D[n] = a.nodes[n];
  __syncthreads();
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * a.tile_rows;
  const int64_t r1 = min<int64_t>(r0 + a.tile_rows, a.nrows);
  // encode: sub-tiles whose OUTPUT bytes take at most ~40 % of the budget (inputs and arrays are
  // of the same order); the walk halves a sub-tile that still does not fit
  const int64_t img_budget = kWrite ? static_cast<int64_t>(a.lds_cap) * 2 / 5 : 0;
  int64_t s0 = r0;
  while (s0 < r1) {
    int64_t s1 = r1;
    if (kWrite) {                               // largest s1 with offs[s1] - offs[s0] <= budget
      const int64_t b0 = gl(a.offs)[s0];
      if (gl(a.offs)[s1] - b0 > img_budget) {
        int64_t lo = s0 + 1, hi = s1;            // offs[lo] may exceed it: at least one row
        while (hi - lo > 0) {
          const int64_t mid = (lo + hi + 1) >> 1;
          if (gl(a.offs)[mid] - b0 <= img_budget) lo = mid; else hi = mid - 1;
        }
        s1 = lo;
      }
    }
    bool ok = false;
    for (;;) {
      ok = te_walk<kWrite>(a, sh, s0, s1);
      if (!ok) TEMARK(sh, 9);
      __syncthreads();
      if (ok || s1 - s0 == 1) break;
      s1 = s0 + (s1 - s0 + 1) / 2;
    }
    if (!ok && threadIdx.x == 0)                 // one row beyond the budget: te_fixup_kernel
      atomicOr(a.fallback + (s0 >> 5), 1u << (s0 & 31));
    s0 = s1;
  }
  TEMARK(sh, 8);
  if (sh.tacc && threadIdx.x < 15)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg) + (kWrite ? 48 : 32) + threadIdx.x,
              static_cast<unsigned long long>(sh.tacc[threadIdx.x]));
  if (sh.tacc && threadIdx.x == 15)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg) + 66 + (kWrite ? 1 : 0), 1ull);
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

namespace {
// tuning "nested_encode": 0 tree tiles (measure + encode), 1 the row interpreter (both), 2 tree
// measure + interpreter encode, 3 tree measure + row-walk encode (rowenc.hip), 4 row walk (both).
// Schemas nested deeper than the interpreter unrolls (kGenMaxDepth) always take the tree tiles;
// the row walk covers up to kRowEncMaxDepth levels (deeper: the interpreter).
std::atomic<int> g_tree_encode = 4;
std::atomic<uint32_t> g_te_lds[2] = {24 * 1024, 60 * 1024};   // LDS budget: measure, encode
std::atomic<int> g_te_rows[2] = {256, 256};                   // rows per workgroup tile: measure, encode

int host_gwidth(int t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

// The tree-tile measure (sizes != NULL) or encode; returns 1 when the schema is left to the row
// interpreter (tables beyond the tree limits), else a status.
int launch_tree_encode(const GenArgs& g, const int64_t* offs, int64_t* sizes, uint8_t* rows,
                       int64_t cap, hipStream_t stream) {
  const int nn = g.nnodes;
  if (nn > 256 || nn <= 0) return 1;
  const GenNode* hn = g.htab ? g.htab : g.node;
  std::vector<TENode> tab(nn);
  std::vector<int32_t> level(nn, 0);
  for (int i = 0; i < nn; i++) {
    TENode& t = tab[i];
    t.values = hn[i].values;
    t.validity = hn[i].validity;
    t.offsets = hn[i].offsets;
    t.type = hn[i].type;
    t.first_child = hn[i].first_child;
    t.num_children = hn[i].num_children;
    if (i < g.ntop) {
      t.parent = -1;
      t.ord = i;
    }
    t.level = level[i];
    t.width = host_gwidth(t.type);
    t.esize = t.width > 0 ? t.width : 8;
    for (int j = 0; j < t.num_children; j++) {
      tab[t.first_child + j].parent = i;
      tab[t.first_child + j].ord = j;
      level[t.first_child + j] = level[i] + 1;
    }
  }
  const int nlev = level[nn - 1] + 1;
  if (nlev > kTEMaxLevels) return 1;
  const bool deep = nlev >= kGenMaxDepth;       // beyond the row interpreter
  if (!deep && (g_tree_encode == 1 || g_tree_encode == 4 || (g_tree_encode >= 2 && sizes == nullptr)))
    return 1;
  TEArgs a{};
  a.deep = deep ? 1 : 0;
  if (const int e = device_error_word(stream, &a.err)) return e;
  a.level_start[0] = 0;
  for (int L = 1; L <= nlev; L++) {
    int i = a.level_start[L - 1];
    while (i < nn && level[i] < L) i++;
    a.level_start[L] = i;
  }
  // layout order (TEShared.ord): per level, the non-scalar LIST / MAP elements first, then the
  // other non-scalar nodes, then the scalars (BFS: a level's nodes are contiguous)
  std::vector<int32_t> ord;
  for (int L = 0; L < nlev; L++) {
    const int b = a.level_start[L], e = a.level_start[L + 1];
    auto elem = [&](int i) {
      const int p = tab[i].parent;
      return p >= 0 && (tab[p].type == FURY_TYPE_LIST || tab[p].type == FURY_TYPE_MAP);
    };
    int ne = 0;
    for (int i = b; i < e; i++)
      if (tab[i].width < 0 && elem(i)) {
        ord.push_back(i);
        ne++;
      }
    for (int i = b; i < e; i++)
      if (tab[i].width < 0 && !elem(i)) ord.push_back(i);
    for (int i = b; i < e; i++)
      if (tab[i].width > 0) ord.push_back(i);
    a.nelem[L] = ne;
  }
  std::vector<uint8_t> blob(tab.size() * sizeof(TENode) + 4 * ord.size());
  memcpy(blob.data(), tab.data(), tab.size() * sizeof(TENode));
  memcpy(blob.data() + tab.size() * sizeof(TENode), ord.data(), 4 * ord.size());
  DeviceTable dt, dg;
  int st = upload_table(blob.data(), blob.size(), stream, &dt);
  if (st) return st;
  const GenNode* gtab = g.tab;
  if (!gtab) {
    st = upload_table(g.node, nn * sizeof(GenNode), stream, &dg);
    if (st) return st;
    gtab = static_cast<const GenNode*>(dg.dev);
  }
  const bool write = sizes == nullptr;
  a.nodes = static_cast<const TENode*>(dt.dev);
  a.gtab = gtab;
  a.offs = offs;
  a.sizes = sizes;
  a.rows = rows;
  a.nrows = g.nrows;
  a.cap = cap;
  a.nn = nn;
  a.ntop = g.ntop;
  a.root = g.root;
  a.nlevels = nlev;
  a.tile_rows = g_te_rows[write ? 1 : 0];
  a.dbg = tree_debug_buffer();
  a.lds_cap = g_te_lds[write ? 1 : 0];
  const size_t lds = te_lds_head(nn) + a.lds_cap;
  const dim3 grid(static_cast<unsigned>((g.nrows + a.tile_rows - 1) / a.tile_rows));
  const int64_t fb_bytes = ((g.nrows + 31) / 32) * 4;
  void* fb = nullptr;
  if ((st = dev_alloc(fb_bytes, stream, &fb))) return st;
  if ((st = check_hip(hipMemsetAsync(fb, 0, fb_bytes, stream), "hipMemsetAsync"))) return st;
  a.fallback = static_cast<uint32_t*>(fb);
  auto go = [&](auto kern, auto fix) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(kern, grid, dim3(kTEThreads), lds, stream, a);
    hipLaunchKernelGGL(fix, dim3(static_cast<unsigned>((g.nrows + kTEThreads - 1) / kTEThreads)),
                       dim3(kTEThreads), 0, stream, a);
  };
  switch ((write ? 3 : 0) + g.root) {
    case 0: go(te_kernel<false, 0>, te_fixup_kernel<false, 0>); break;
    case 1: go(te_kernel<false, 1>, te_fixup_kernel<false, 1>); break;
    case 2: go(te_kernel<false, 2>, te_fixup_kernel<false, 2>); break;
    case 3: go(te_kernel<true, 0>, te_fixup_kernel<true, 0>); break;
    case 4: go(te_kernel<true, 1>, te_fixup_kernel<true, 1>); break;
    default: go(te_kernel<true, 2>, te_fixup_kernel<true, 2>); break;
  }
  st = check_hip(hipGetLastError(), "tree encode launch");
  dev_free(fb, stream);
  return st;
}
}  // namespace

void set_tree_encode_mode(int v) { g_tree_encode = v; }
int tree_encode_mode() { return g_tree_encode; }
void set_tree_encode_lds(int which, uint32_t bytes) { g_te_lds[which ? 1 : 0] = (bytes + 15) & ~15u; }
uint32_t tree_encode_lds(int which) { return g_te_lds[which ? 1 : 0]; }
void set_tree_encode_rows(int which, int rows) { g_te_rows[which ? 1 : 0] = rows; }
int tree_encode_rows(int which) { return g_te_rows[which ? 1 : 0]; }

int launch_gen_measure(const GenArgs& g, int64_t* sizes, hipStream_t stream) {
  if (g.nrows > 0) {
    int t = launch_tree_encode(g, nullptr, sizes, nullptr, 0, stream);
    if (t == 1 && g_tree_encode == 4) t = rowenc_launch(g, nullptr, sizes, nullptr, 0, stream);
    if (t != 1) return t;
  }
  if (g.tab) gen_encode_root<true>(g, nullptr, sizes, nullptr, 0, stream);
  else gen_encode_root<false>(g, nullptr, sizes, nullptr, 0, stream);
  return check_hip(hipGetLastError(), "gen_measure launch");
}

int launch_gen_encode(const GenArgs& g, const int64_t* offs, uint8_t* rows, int64_t cap,
                      hipStream_t stream) {
  if (g.nrows > 0) {
    int t = launch_tree_encode(g, offs, nullptr, rows, cap, stream);
    if (t == 1 && g_tree_encode >= 3) t = rowenc_launch(g, offs, nullptr, rows, cap, stream);
    if (t != 1) return t;
  }
  if (g.tab) gen_encode_root<true>(g, offs, nullptr, rows, cap, stream);
  else gen_encode_root<false>(g, offs, nullptr, rows, cap, stream);
  return check_hip(hipGetLastError(), "gen_encode launch");
}

}  // namespace fury
