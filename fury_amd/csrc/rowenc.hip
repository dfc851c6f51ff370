// rowenc.hip — the encode (measure pass + build pass) of every schema the flat kernels do not
// take: nested STRUCT / LIST / MAP fields at any depth (up to 64 levels), flat variable-length
// schemas wider than 256 fields, and ArrayEncoder / MapEncoder collection batches.  A thread per
// ROW walks the schema, the first kRowEncMaxDepth levels inlined per depth, deeper levels with an
// explicit stack (rdeep).  (Round 5 removed the row interpreter and the tree-tile encode this
// replaced: one nested encode engine)
//
// Reference semantics: BaseBinaryEncoderBuilder
// .serializeFor (FMT/encoder/BaseBinaryEncoderBuilder.java:138-453) -- primitives in 8-byte slots
// (narrow in arrays), var values appended at the writer index and zero-padded to 8
// (BinaryWriter.java:106-121,187-194), List -> [int64 n][bitmap][n x elemSize, tail zeroed][var
// section] (BinaryArrayWriter.java:91-163), bean -> nested BinaryRowWriter row (:363-417), Map ->
// [int64 keyBytes][key array][value array] (:298-357), null -> setNullAt (bit only); the bytes are
// checked against the oracle (tests/test_tree.py, tests/test_reference_beans.py).
//
// MI355X design.  A row interpreter whose depth templates call each other keeps every level's
// registers live in a call frame (the round-2/3 engine: 256 VGPRs plus ~870 B of scratch per
// lane).  Here a container's children -- a STRUCT's fields, a LIST's elements, a
// MAP's keys then values -- go through ONE loop with ONE call of the next level, so the levels
// inline into straight code (as walk.hip's decode walk); scalar children are stored at the call
// site, so a schema of L levels needs L instances.  Every active lane of a wave is at the same
// schema node at the same time (the loops are schema-driven), so node records come from a device
// table through scalar loads (readfirstlane'd index).  The build pass writes a workgroup's rows
// (rowenc_rows) into an LDS image of their contiguous output range and stores it coalesced (as
// the interpreter's build kernel): thread-per-row stores straight to HBM wrote several times the
// row bytes (partial lines); only the rows past the image (rowenc_img) are built in HBM.
#include <hip/hip_runtime.h>

#include <atomic>

#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

constexpr int kRwThreads = 256;                 // measure pass rows per workgroup
std::atomic<int> g_rw_rows = 256;                            // tuning "rowenc_rows": build-pass rows per workgroup
                                                             // (512 with a 152 KB image: 1.31 vs 1.33 ms, not the default)
std::atomic<uint32_t> g_rw_img = 76 * 1024;                  // tuning "rowenc_img": its LDS image bytes
std::atomic<int> g_rw_tile = 0;                              // tuning "rowenc_tile": rows per workgroup (0: all)

template <class T>
using Lds = __attribute__((address_space(3))) T;
using LdsU8 = Lds<uint8_t>;
using CGNode = __attribute__((address_space(4))) const GenNode;

struct RwArgs {
  const GenNode* tab;       // device node table (scalar loads)
  int64_t img;              // build pass: LDS image bytes
  int64_t tile;             // build pass: rows per workgroup (<= its threads)
  const int64_t* offs;      // build pass: row offsets
  int64_t* sizes;           // measure pass: row sizes
  uint8_t* rows;
  int64_t nrows;
  int64_t cap;
  int32_t ntop;
};

__device__ __forceinline__ CGNode& rn(const RwArgs& a, int n) { return ((CGNode*)(a.tab))[n]; }

__device__ __forceinline__ int64_t r8(int64_t n) { return (n + 7) & ~int64_t(7); }
__device__ __forceinline__ int64_t rbm(int64_t n) { return ((n + 63) >> 6) << 3; }
__device__ __forceinline__ int rwidth(int t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

// Stores into the LDS image or (past it) HBM; every store is aligned to its width by the format.
__device__ __forceinline__ void s8(LdsU8* p, uint64_t v) { *reinterpret_cast<Lds<uint64_t>*>(p) = v; }
__device__ __forceinline__ void s8(uint8_t* p, uint64_t v) { *gl(reinterpret_cast<uint64_t*>(p)) = v; }
__device__ __forceinline__ void s4(LdsU8* p, uint32_t v) { *reinterpret_cast<Lds<uint32_t>*>(p) = v; }
__device__ __forceinline__ void s4(uint8_t* p, uint32_t v) { *gl(reinterpret_cast<uint32_t*>(p)) = v; }
__device__ __forceinline__ void s2(LdsU8* p, uint16_t v) { *reinterpret_cast<Lds<uint16_t>*>(p) = v; }
__device__ __forceinline__ void s2(uint8_t* p, uint16_t v) { *gl(reinterpret_cast<uint16_t*>(p)) = v; }
__device__ __forceinline__ void s1(LdsU8* p, uint8_t v) { *p = v; }
__device__ __forceinline__ void s1(uint8_t* p, uint8_t v) { *gl(p) = v; }
__device__ __forceinline__ void o1_(LdsU8* p, uint8_t v) { *p |= v; }
__device__ __forceinline__ void o1_(uint8_t* p, uint8_t v) { *gl(p) |= v; }

template <class P>
__device__ __forceinline__ void rzero(P p, int64_t n) {       // 8-aligned, n a multiple of 8
  for (int64_t i = 0; i < n; i += 8) s8(p + i, 0);
}

// len bytes from an unaligned source at dst (8-aligned), zero-padded to 8: aligned source words
// funnel-shifted into place; no word past the last source byte is read.
template <class P>
__device__ __forceinline__ void rappend(P dst, const uint8_t* src, int64_t len) {
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
    s8(dst + 8 * w, x);
    cur = nxt;
  }
}

template <int D, int MD, bool W, int DEEP, class P>
__device__ __forceinline__ void rvalue(const RwArgs& a, int ni, int ty, int64_t idx, int64_t o0,
                                       int64_t o1, P buf, int64_t container, int64_t slot,
                                       int64_t& cursor);
template <bool W, int SF, class P>
__device__ void rdeep(const RwArgs& a, int ni, int64_t idx, P buf, int64_t container, int64_t slot,
                      int es, bool in_array, int64_t bm, int64_t ord, int64_t& cursor);

// Entry idx of node ni at level D, in slot `slot` (es bytes; in_array: an array element) of a
// container starting at `container`, null bit `ord` of the bitmap at bm.  Every load of the entry
// -- its validity byte, its value or its offsets pair -- is issued before any branch on them: one
// memory round trip per entry instead of one per dependent read (the walk is latency-bound).
// (Issuing entry j + 1's loads before finishing entry j measured slower: more VGPRs, 1.34 ->
// 1.45 ms build at 4M depth-3 rows.)
template <int D, int MD, bool W, int DEEP, class P>
__device__ __forceinline__ void ritem(const RwArgs& a, int ni, int64_t idx, P buf,
                                      int64_t container, int64_t slot, int es, bool in_array,
                                      int64_t bm, int64_t ord, int64_t& cursor) {
  if constexpr (D >= MD) {
    // below the inlined levels: the explicit-stack walk (DEEP = its frames; instances for schemas
    // deeper than MD)
    if constexpr (DEEP > 0) rdeep<W, DEEP>(a, ni, idx, buf, container, slot, es, in_array, bm, ord, cursor);
    return;
  } else {
    CGNode& n = rn(a, ni);
    const int ty = n.type;
    const int w = rwidth(ty);
    const uint32_t vb = n.validity ? gl(n.validity)[idx >> 3] : 0xffu;
    uint64_t v = 0;
    int64_t o0 = 0, o1 = 0;
    if (w > 0) {
      if (W) {
        if (ty == FURY_TYPE_BOOL) v = gl(n.values)[idx >> 3];
        else if (w == 8) v = *gl(reinterpret_cast<const uint64_t*>(n.values + idx * 8));
        else if (w == 4) v = *gl(reinterpret_cast<const uint32_t*>(n.values + idx * 4));
        else if (w == 2) v = *gl(reinterpret_cast<const uint16_t*>(n.values + idx * 2));
        else v = gl(n.values)[idx];
      }
    } else if (n.offsets) {
      o0 = gl(n.offsets)[idx];
      o1 = gl(n.offsets)[idx + 1];
    }
    if (!((vb >> (idx & 7)) & 1)) {              // setNullAt: bit only, slot stays 0
      if (W) o1_(buf + bm + (ord >> 3), static_cast<uint8_t>(1u << (ord & 7)));
      return;
    }
    if (w > 0) {                                 // putInt64(0) + narrow put / element width
      if (W) {
        if (ty == FURY_TYPE_BOOL) v = (v >> (idx & 7)) & 1;
        if (!in_array || es == 8) s8(buf + slot, v);
        else if (es == 4) s4(buf + slot, static_cast<uint32_t>(v));
        else if (es == 2) s2(buf + slot, static_cast<uint16_t>(v));
        else s1(buf + slot, static_cast<uint8_t>(v));
      }
      return;
    }
    rvalue<D, MD, W, DEEP>(a, ni, ty, idx, o0, o1, buf, container, slot, cursor);
  }
}

// Elements [b, b + m) of a fixed-width node C (es bytes each) into an array's slots at buf + sp
// (null bits at buf + bm): validity bytes and values of four elements loaded together, then
// stored -- one memory round trip per four elements instead of one per element.
template <class P>
__device__ __forceinline__ void relems(CGNode& C, int es, int64_t b, int64_t m, P buf, int64_t sp,
                                       int64_t bm) {
  const bool boo = C.type == FURY_TYPE_BOOL;
  for (int64_t j0 = 0; j0 < m; j0 += 4) {
    uint64_t v[4];
    uint32_t vb[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t i = b + j0 + q;
      v[q] = 0;
      vb[q] = 0xffu;
      if (j0 + q < m) {
        if (C.validity) vb[q] = gl(C.validity)[i >> 3];
        if (boo) v[q] = gl(C.values)[i >> 3];
        else if (es == 8) v[q] = *gl(reinterpret_cast<const uint64_t*>(C.values + i * 8));
        else if (es == 4) v[q] = *gl(reinterpret_cast<const uint32_t*>(C.values + i * 4));
        else if (es == 2) v[q] = *gl(reinterpret_cast<const uint16_t*>(C.values + i * 2));
        else v[q] = gl(C.values)[i];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t j = j0 + q, i = b + j;
      if (j >= m) continue;
      if (!((vb[q] >> (i & 7)) & 1)) {
        o1_(buf + bm + (j >> 3), static_cast<uint8_t>(1u << (j & 7)));
        continue;
      }
      const uint64_t x = boo ? (v[q] >> (i & 7)) & 1 : v[q];
      if (es == 8) s8(buf + sp + 8 * j, x);
      else if (es == 4) s4(buf + sp + 4 * j, static_cast<uint32_t>(x));
      else if (es == 2) s2(buf + sp + 2 * j, static_cast<uint16_t>(x));
      else s1(buf + sp + j, static_cast<uint8_t>(x));
    }
  }
}

// The image of container entry idx of node ni (type ty: STRUCT, or LIST / MAP with elements
// [b, b + m) of its child nodes) at buf + start; returns the end of its bytes.  Children at level
// D + 1.
template <int D, int MD, bool W, int DEEP, class P>
__device__ __forceinline__ int64_t rcont(const RwArgs& a, int ni, int ty, int64_t idx, int64_t b,
                                         int64_t m, P buf, int64_t start) {
  CGNode& n = rn(a, ni);
  const bool strc = ty == FURY_TYPE_STRUCT;
  int64_t c2 = start + (ty == FURY_TYPE_MAP ? 8 : 0);   // a map's key-array size word first
  const int sides = ty == FURY_TYPE_MAP ? 2 : 1;
  for (int sd = 0; sd < sides; sd++) {
    int64_t arr, hb, items;
    int ces = 8;
    if (strc) {                                 // [bitmap][8-byte slots]
      items = n.num_children;
      arr = start;
      hb = rbm(items);
      if (W) rzero(buf + start, hb + 8 * items);
      c2 = start + hb + 8 * items;
    } else {                                    // [int64 m][bitmap][m x es, tail zeroed]
      if (sd == 1 && W) s8(buf + start, static_cast<uint64_t>(c2 - (start + 8)));
      CGNode& C = rn(a, n.first_child + sd);
      const int cw = rwidth(C.type);
      ces = cw > 0 ? cw : 8;
      arr = c2;
      hb = 8 + rbm(m);
      items = m;
      const int64_t fp = r8(m * ces);
      if (W) {
        s8(buf + arr, static_cast<uint64_t>(m));
        rzero(buf + arr + 8, hb - 8 + fp);
      }
      c2 = arr + hb + fp;
    }
    const int64_t bm = strc ? arr : arr + 8;
    if (!strc && ces == rwidth(rn(a, n.first_child + sd).type)) {
      // fixed-width elements: four at a time, every load of the four issued before any store
      if (W) relems(rn(a, n.first_child + sd), ces, b, items, buf, arr + hb, bm);
      continue;
    }
    for (int64_t j = 0; j < items; j++) {
      const int cn = __builtin_amdgcn_readfirstlane(
          strc ? n.first_child + static_cast<int>(j) : n.first_child + sd);
      ritem<D + 1, MD, W, DEEP>(a, cn, strc ? idx : b + j, buf, arr, arr + hb + (strc ? 8 : ces) * j,
                                strc ? 8 : ces, !strc, bm, j, c2);
    }
  }
  return c2;
}

// A non-null, non-scalar entry idx of node ni (level D; o0 / o1: its offsets pair): its bytes at
// the cursor, its slot (offset from the container, size).
template <int D, int MD, bool W, int DEEP, class P>
__device__ __forceinline__ void rvalue(const RwArgs& a, int ni, int ty, int64_t idx, int64_t o0,
                                       int64_t o1, P buf, int64_t container, int64_t slot,
                                       int64_t& cursor) {
  CGNode& n = rn(a, ni);
  const int64_t start = cursor;
  if (ty == FURY_TYPE_STRING || ty == FURY_TYPE_BINARY) {
    const int64_t len = o1 - o0;
    if (W) {
      rappend(buf + start, n.values + o0, len);
      s8(buf + slot, (static_cast<uint64_t>(start - container) << 32) | static_cast<uint32_t>(len));
    }
    cursor = start + r8(len);
    return;
  }
  if (ty == FURY_TYPE_DECIMAL) {
    if (W) {
      const auto v = gl(reinterpret_cast<const uint64_t*>(n.values + 16 * idx));
      s8(buf + start, v[0]);
      s8(buf + start + 8, v[1]);
      s8(buf + slot, (static_cast<uint64_t>(start - container) << 32) | 16u);
    }
    cursor = start + 16;
    return;
  }
  if (ty != FURY_TYPE_STRUCT && ty != FURY_TYPE_LIST && ty != FURY_TYPE_MAP) return;
  cursor = rcont<D, MD, W, DEEP>(a, ni, ty, idx, o0, o1 - o0, buf, start);
  if (W) s8(buf + slot, (static_cast<uint64_t>(start - container) << 32) |
                            static_cast<uint32_t>(cursor - start));
}

// Entry r of the batch (generic.hip put_row): a row of the ntop top-level fields, or the
// top-level BinaryArray / BinaryMap of node 0's entry r (ArrayEncoder.toArray / MapEncoder.toMap,
// ArrayEncoderBuilder.java:118-140, MapEncoderBuilder.java:152-208).  Returns its size.
template <bool W, int kRoot, int MD, int DEEP, class P>
__device__ __forceinline__ int64_t rrow(const RwArgs& a, int64_t r, P buf) {
  if constexpr (kRoot != 0) {
    const auto offs = gl(rn(a, 0).offsets);
    const int64_t b = offs[r];
    return rcont<0, MD, W, DEEP>(a, 0, kRoot == 1 ? FURY_TYPE_LIST : FURY_TYPE_MAP, r, b,
                                 offs[r + 1] - b, buf, 0);
  } else {
    const int ntop = a.ntop;
    const int64_t bmb = rbm(ntop);
    const int64_t fixed = bmb + 8 * static_cast<int64_t>(ntop);
    if (W) rzero(buf, fixed);
    int64_t cursor = fixed;
    for (int k = 0; k < ntop; k++)
      ritem<0, MD, W, DEEP>(a, k, r, buf, 0, bmb + 8 * static_cast<int64_t>(k), 8, false, 0, k, cursor);
    return cursor;
  }
}

template <int kRoot, int MD, int DEEP>
__global__ __launch_bounds__(kRwThreads) void rw_measure_kernel(RwArgs a) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kRwThreads + threadIdx.x;
  if (r < a.nrows) a.sizes[r] = rrow<false, kRoot, MD, DEEP>(a, r, static_cast<LdsU8*>(nullptr));
}

// Build pass: the workgroup's rows are built in the LDS image by whole waves as long as their
// bytes fit it (a.img), then stored with coalesced 8-byte stores; the waves past that build their
// rows straight in HBM in the same pass.  Per wave, not per row: a wave whose lanes took both
// paths ran both instruction streams one after the other (a 72 KB image on ~75 KB tiles: 2.1 ms
// per-row vs 1.33 ms when everything fit), and a second image round costs a whole walk latency.
// Rows past the capacity (encode_measured) are not written.
template <int NT, int kRoot, int MD, int DEEP>
__global__ __launch_bounds__(NT) void rw_encode_kernel(RwArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t img[];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * a.tile;
  const int64_t r = r0 + threadIdx.x;
  const int64_t rend = min(r0 + a.tile, a.nrows);
  const bool live = r < rend;
  const int64_t my0 = live ? a.offs[r] : 0, my1 = live ? a.offs[r + 1] : 0;
  const int64_t b0 = a.offs[r0];
  // rows whose end fits the image: a prefix of the tile (offsets ascend), cut to whole waves
  const int fit = __syncthreads_count(live && my1 - b0 <= a.img && my1 <= a.cap);
  const int64_t in_img = min<int64_t>(fit == rend - r0 ? fit : fit & ~63, rend - r0);
  if (live && my1 <= a.cap) {
    if (r < r0 + in_img) rrow<true, kRoot, MD, DEEP>(a, r, (LdsU8*)(img + (my0 - b0)));
    else rrow<true, kRoot, MD, DEEP>(a, r, a.rows + my0);
  }
  __syncthreads();
  const int64_t nw = (a.offs[r0 + in_img] - b0) >> 3;
  const uint64_t* s = reinterpret_cast<const uint64_t*>(img);
  uint64_t* d = reinterpret_cast<uint64_t*>(a.rows + b0);
  for (int64_t i = threadIdx.x; i < nw; i += NT) d[i] = s[i];
}

// ---- schemas nested deeper than kRowEncMaxDepth: the walk below the inlined levels with an
// explicit stack (per-lane frames in scratch) -- the same entries, in the same order, writing the
// same bytes as ritem / rvalue / rcont.  Lanes may sit at different depths here (a lane whose
// list is shorter pops while another pushes), so node records are plain per-lane loads.
struct RFrame {
  int64_t idx, b, m, start, slot, container, arr, hb, items, j;
  int32_t ni, sd;
};

// Header of side f.sd of the container of frame f at the cursor (a STRUCT: bitmap + slots; a LIST /
// MAP side: [int64 m][bitmap][m x elemSize, tail zeroed]); returns the items the walk visits (0:
// fixed-width elements, written here four at a time).
template <bool W, class P>
__device__ __forceinline__ int64_t rside(const RwArgs& a, RFrame& f, P buf, int64_t& cursor) {
  CGNode& n = rn(a, f.ni);
  if (n.type == FURY_TYPE_STRUCT) {
    const int64_t items = n.num_children;
    f.arr = f.start;
    f.hb = rbm(items);
    if (W) rzero(buf + f.start, f.hb + 8 * items);
    cursor = f.start + f.hb + 8 * items;
    return items;
  }
  if (f.sd == 1 && W) s8(buf + f.start, static_cast<uint64_t>(cursor - (f.start + 8)));
  CGNode& C = rn(a, n.first_child + f.sd);
  const int cw = rwidth(C.type);
  const int ces = cw > 0 ? cw : 8;
  f.arr = cursor;
  f.hb = 8 + rbm(f.m);
  const int64_t fp = r8(f.m * ces);
  if (W) {
    s8(buf + f.arr, static_cast<uint64_t>(f.m));
    rzero(buf + f.arr + 8, f.hb - 8 + fp);
  }
  cursor = f.arr + f.hb + fp;
  if (cw > 0) {
    if (W) relems(C, ces, f.b, f.m, buf, f.arr + f.hb, f.arr + 8);
    return 0;
  }
  return f.m;
}

// SF frames: one per container level below the inlined ones (rowenc_launch picks the smallest
// instance that holds the schema's depth, so a 6-level schema does not reserve 64 frames x 88 B of
// scratch per lane -- ADVICE r5).
template <bool W, int SF, class P>
__device__ void rdeep(const RwArgs& a, int ni0, int64_t idx0, P buf, int64_t container0,
                      int64_t slot0, int es0, bool in_array0, int64_t bm0, int64_t ord0,
                      int64_t& cursor) {
  RFrame st[SF];
  int sp = -1;
  // one entry (ritem + rvalue): leaves written at once, a container pushed with its first side
  auto enter = [&](int ni, int64_t idx, int64_t container, int64_t slot, int es, bool in_array,
                   int64_t bm, int64_t ord) {
    CGNode& n = rn(a, ni);
    const int ty = n.type;
    const int w = rwidth(ty);
    const uint32_t vb = n.validity ? gl(n.validity)[idx >> 3] : 0xffu;
    uint64_t v = 0;
    int64_t o0 = 0, o1 = 0;
    if (w > 0) {
      if (W) {
        if (ty == FURY_TYPE_BOOL) v = gl(n.values)[idx >> 3];
        else if (w == 8) v = *gl(reinterpret_cast<const uint64_t*>(n.values + idx * 8));
        else if (w == 4) v = *gl(reinterpret_cast<const uint32_t*>(n.values + idx * 4));
        else if (w == 2) v = *gl(reinterpret_cast<const uint16_t*>(n.values + idx * 2));
        else v = gl(n.values)[idx];
      }
    } else if (n.offsets) {
      o0 = gl(n.offsets)[idx];
      o1 = gl(n.offsets)[idx + 1];
    }
    if (!((vb >> (idx & 7)) & 1)) {
      if (W) o1_(buf + bm + (ord >> 3), static_cast<uint8_t>(1u << (ord & 7)));
      return;
    }
    if (w > 0) {
      if (W) {
        if (ty == FURY_TYPE_BOOL) v = (v >> (idx & 7)) & 1;
        if (!in_array || es == 8) s8(buf + slot, v);
        else if (es == 4) s4(buf + slot, static_cast<uint32_t>(v));
        else if (es == 2) s2(buf + slot, static_cast<uint16_t>(v));
        else s1(buf + slot, static_cast<uint8_t>(v));
      }
      return;
    }
    const int64_t start = cursor;
    if (ty == FURY_TYPE_STRING || ty == FURY_TYPE_BINARY) {
      const int64_t len = o1 - o0;
      if (W) {
        rappend(buf + start, n.values + o0, len);
        s8(buf + slot, (static_cast<uint64_t>(start - container) << 32) | static_cast<uint32_t>(len));
      }
      cursor = start + r8(len);
      return;
    }
    if (ty == FURY_TYPE_DECIMAL) {
      if (W) {
        const auto dv = gl(reinterpret_cast<const uint64_t*>(n.values + 16 * idx));
        s8(buf + start, dv[0]);
        s8(buf + start + 8, dv[1]);
        s8(buf + slot, (static_cast<uint64_t>(start - container) << 32) | 16u);
      }
      cursor = start + 16;
      return;
    }
    if (ty != FURY_TYPE_STRUCT && ty != FURY_TYPE_LIST && ty != FURY_TYPE_MAP) return;
    RFrame& f = st[++sp];
    f.ni = ni;
    f.idx = idx;
    f.b = o0;
    f.m = o1 - o0;
    f.start = start;
    f.slot = slot;
    f.container = container;
    f.sd = 0;
    f.j = 0;
    f.items = 0;
    cursor = start + (ty == FURY_TYPE_MAP ? 8 : 0);     // a map's key-array size word first
    f.items = rside<W>(a, f, buf, cursor);
  };
  enter(ni0, idx0, container0, slot0, es0, in_array0, bm0, ord0);
  while (sp >= 0) {
    RFrame& f = st[sp];
    CGNode& n = rn(a, f.ni);
    if (f.j < f.items) {
      const int64_t j = f.j++;
      if (n.type == FURY_TYPE_STRUCT)
        enter(n.first_child + static_cast<int>(j), f.idx, f.arr, f.arr + f.hb + 8 * j, 8, false, f.arr, j);
      else
        enter(n.first_child + f.sd, f.b + j, f.arr, f.arr + f.hb + 8 * j, 8, true, f.arr + 8, j);
      continue;
    }
    if (n.type == FURY_TYPE_MAP && f.sd == 0) {          // the value array after the keys
      f.sd = 1;
      f.j = 0;
      f.items = rside<W>(a, f, buf, cursor);
      continue;
    }
    if (W) s8(buf + f.slot, (static_cast<uint64_t>(f.start - f.container) << 32) |
                                static_cast<uint32_t>(cursor - f.start));
    sp--;
  }
}

}  // namespace

int rowenc_launch(const GenArgs& g, const int64_t* offs, int64_t* sizes, uint8_t* rows,
                  int64_t cap, hipStream_t stream) {
  const int nn = g.nnodes;
  const GenNode* hn = g.htab ? g.htab : g.node;
  if (nn <= 0 || !hn) return set_error(FURY_ERR_INVALID_ARGUMENT, "row-walk encode: empty schema");
  std::vector<int32_t> level(nn, 0);
  int nlev = 1;
  for (int i = 0; i < nn; i++)
    for (int j = 0; j < hn[i].num_children; j++) {
      level[hn[i].first_child + j] = level[i] + 1;
      nlev = std::max(nlev, level[i] + 2);
    }
  if (nlev > kMaxNestLevels) return set_error(FURY_ERR_UNSUPPORTED, "schema nested deeper than 64 levels");
  RwArgs a{};
  DeviceTable dt;
  const GenNode* tab = g.tab;
  if (!tab) {
    const int st = upload_table(g.node, nn * sizeof(GenNode), stream, &dt);
    if (st) return st;
    tab = static_cast<const GenNode*>(dt.dev);
  }
  a.tab = tab;
  a.offs = offs;
  a.sizes = sizes;
  a.rows = rows;
  a.nrows = g.nrows;
  a.cap = cap;
  a.ntop = g.ntop;
  a.img = g_rw_img;
  int nt = sizes ? kRwThreads : g_rw_rows.load();
  if (nlev > kRowEncMaxDepth && nt > 256) nt = 256;   // the explicit-stack instances: 128 / 256
  const int rt = g_rw_tile.load();
  a.tile = sizes ? nt : (rt > 0 && rt < nt ? rt : nt);
  const dim3 grid(static_cast<unsigned>((g.nrows + a.tile - 1) / a.tile));
  auto go = [&](auto meas, auto enc128, auto enc256, auto enc512) {
    if (sizes) {
      hipLaunchKernelGGL(meas, grid, dim3(nt), 0, stream, a);
      return;
    }
    auto run = [&](auto enc) {
      const size_t lds = a.img;
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(enc),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      hipLaunchKernelGGL(enc, grid, dim3(nt), lds, stream, a);
    };
    if (nt == 128) run(enc128);
    else if (nt == 512) run(enc512);
    else run(enc256);
  };
#define FURY_RW(R, MD)                                                                         \
  if (g.root == R && nlev <= MD) {                                                             \
    go(rw_measure_kernel<R, MD, 0>, rw_encode_kernel<128, R, MD, 0>,                           \
       rw_encode_kernel<256, R, MD, 0>, rw_encode_kernel<512, R, MD, 0>);                      \
    return check_hip(hipGetLastError(), "row-walk encode launch");                             \
  }
  // deeper schemas: kRowEncMaxDepth inlined levels, then the explicit stack (rdeep)
// (frames: the container levels below the inlined ones, at most nlev - kRowEncMaxDepth)
#define FURY_RW_DEEP(R, SF)                                                                    \
  if (g.root == R && nlev - kRowEncMaxDepth <= SF) {                                           \
    go(rw_measure_kernel<R, kRowEncMaxDepth, SF>,                                              \
       rw_encode_kernel<128, R, kRowEncMaxDepth, SF>, rw_encode_kernel<256, R, kRowEncMaxDepth, SF>, \
       rw_encode_kernel<256, R, kRowEncMaxDepth, SF>);                                         \
    return check_hip(hipGetLastError(), "row-walk encode launch");                             \
  }
  FURY_RW(0, 2) FURY_RW(0, 3) FURY_RW(0, 4) FURY_RW(0, 5)
  FURY_RW(1, 2) FURY_RW(1, 3) FURY_RW(1, 4) FURY_RW(1, 5)
  FURY_RW(2, 2) FURY_RW(2, 3) FURY_RW(2, 4) FURY_RW(2, 5)
  FURY_RW_DEEP(0, 16) FURY_RW_DEEP(1, 16) FURY_RW_DEEP(2, 16)
  FURY_RW_DEEP(0, kMaxNestLevels - kRowEncMaxDepth) FURY_RW_DEEP(1, kMaxNestLevels - kRowEncMaxDepth)
  FURY_RW_DEEP(2, kMaxNestLevels - kRowEncMaxDepth)
#undef FURY_RW_DEEP
#undef FURY_RW
  return set_error(FURY_ERR_UNSUPPORTED, "row-walk encode: collection root");
}

// fury_row_measure / fury_row_encode(_measured) of the schemas above (capi.cpp).
int launch_gen_measure(const GenArgs& g, int64_t* sizes, hipStream_t stream) {
  if (g.nrows == 0) return FURY_OK;
  return rowenc_launch(g, nullptr, sizes, nullptr, 0, stream);
}
int launch_gen_encode(const GenArgs& g, const int64_t* offs, uint8_t* rows, int64_t cap,
                      hipStream_t stream) {
  if (g.nrows == 0) return FURY_OK;
  return rowenc_launch(g, offs, nullptr, rows, cap, stream);
}

void set_rowenc_tuning(int which, uint32_t v) {
  if (which == 0) g_rw_rows = static_cast<int>(v);
  else if (which == 1) g_rw_img = (v + 15) & ~15u;
  else g_rw_tile = static_cast<int>(v);
}
uint32_t rowenc_tuning(int which) {
  return which == 0 ? static_cast<uint32_t>(g_rw_rows) : which == 1 ? g_rw_img.load()
         : static_cast<uint32_t>(g_rw_tile);
}

}  // namespace fury
