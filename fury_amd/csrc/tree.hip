// tree.hip — tile-staged codec of nested schemas ("tree tiles"): decode (rows -> the Arrow column
// tree) in two passes over LDS-staged row tiles.
//
// Reference semantics (FMT = java/fury-format/src/main/java/org/apache/fury/format): the getters
// of BinaryRow / BinaryArray / BinaryMap (FMT/row/binary/UnsafeTrait.java:68-197,
// BinaryArray.java:69-78, BinaryMap.java:62-77) as the generated fromRow and ArrowWriter walk
// them (FMT/encoder/BaseBinaryEncoderBuilder.java:459-706, FMT/vectorized/ArrowWriter.java:
// 205-640): entries of a node in (parent entry, element) order, a null struct gives a null entry
// in every child (StructWriter.appendNull :577-584), a null list / map a zero-length entry, null
// values zeroed; every read bounds-checked against the batch (MemoryBuffer, span_ok in kernels.h).
//
// MI355X design.  A workgroup owns a tile of consecutive rows = one contiguous byte range of the
// batch, staged into LDS by LDS-DMA (one round trip).  The schema tree is then walked level by
// level ON CHIP: a level's entries in the tile are laid out as per-node arrays in an LDS arena
// (source position of each non-scalar entry, count of each STRING / BINARY / LIST / MAP entry),
// filled from the previous level's arrays (a struct child's entry = its parent's; a list / map
// child's entries = the parent's elements, each finding its owner by binary search over the
// parent's in-tile count prefix), then one block scan per level turns the counts into in-tile
// prefixes.  Scalars (fixed-width / bool) are written while their parent level expands.
//   pass 1 (prepare): entries and payload bytes of every node per tile -> [node][tile] arrays;
//                     one scan kernel per batch turns them into each tile's output bases and the
//                     node totals the caller sizes its buffers from (the only host sync).
//   pass 2 (execute): the same walk, every output written at tile base + in-tile index: values
//                     and offsets by consecutive lanes (coalesced), validity / BOOL bits by wave
//                     ballots, string payloads copied from the staged rows.
// A tile whose arrays do not fit the arena is walked in halves (both passes split it the same
// way, deterministically); a single row that does not fit sends the whole batch to the
// level-by-level engine of levels.hip (fury_decode_prepare falls back).  Rows are read from the
// stage when the tile's bytes fit it, from HBM otherwise (skewed row sizes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

struct TNode {
  uint8_t* values;          // decode outputs (execute)
  uint8_t* validity;
  int32_t* offsets;
  int32_t type;
  int32_t first_child;
  int32_t num_children;
  int32_t parent;           // -1: top-level field
  int32_t ord;              // index among the parent's children (top-level: field index)
  int32_t width;            // fixed-width scalar: bytes (BOOL: 1); -1 otherwise
  int32_t esize;            // slot bytes as an array element (BinaryArrayWriter elementSize)
  int32_t pad_;
};

constexpr int kTreeMaxNodes = 512;
constexpr int kTreeMaxLevels = 64;
constexpr int kTreeThreads = 256;

struct TreeArgs {
  const TNode* nodes;       // device table (scalar loads: every use has a uniform index)
  const uint8_t* rows;
  const int64_t* offs;
  int64_t nrows;
  int64_t ntiles;
  int64_t* cnt;             // [nn][ntiles]: entries of node n in tile t (pass 1) / its base (pass 2)
  int64_t* byt;             // [nn][ntiles]: payload bytes of node n in tile t / its base
  uint32_t* err;            // the stream's device error slot
  int32_t* overflow;        // set when a single row does not fit the arena (pass 1)
  int32_t nn, ntop, root, nlevels;
  int32_t tile_rows;
  uint32_t stage_cap, arena_cap;
  int32_t level_start[kTreeMaxLevels + 1];
};

namespace {

constexpr int64_t kNullPos = -1;

// Per-node state of the tile being walked (LDS).
struct TMeta {
  uint32_t ecnt;            // entries of the node in the current (sub-)tile
  uint32_t src;             // arena byte offset of its int64 source array (non-scalar nodes)
  uint32_t cnt;             // arena byte offset of its uint32 count / prefix array (+1 slot)
  uint32_t tot;             // in-tile total of the counts (elements / payload bytes)
  int64_t run_e;            // pass 2: output entry base of the current sub-tile
  int64_t run_b;            // pass 2: payload byte base of the current sub-tile
};

__device__ __forceinline__ int64_t tbm(int64_t n) { return ((n + 63) >> 6) << 3; }

// Node records through the constant address space: every index is uniform, so scalar loads.
using CTNode = __attribute__((address_space(4))) const TNode;
__device__ __forceinline__ CTNode& tn(const TreeArgs& a, int n) {
  return ((CTNode*)(a.nodes))[n];
}

__device__ __forceinline__ bool is_scalar(int t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: case FURY_TYPE_INT16: case FURY_TYPE_INT32:
    case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64:
    case FURY_TYPE_TIMESTAMP:
      return true;
    default:
      return false;
  }
}
__device__ __forceinline__ bool is_counted(int t) {
  return t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY || t == FURY_TYPE_LIST || t == FURY_TYPE_MAP;
}

// Reads of the batch's row bytes: from the staged window when the bytes lie in it (naturally
// aligned LDS accesses only: the window starts at a 16-aligned address, so LDS and HBM alignment
// agree), else from HBM.  Positions are byte offsets into the batch.
struct Rows {
  const uint8_t* g;         // the batch (device memory)
  const uint8_t* stg;       // LDS copy of g[lo_al, hi)
  int64_t lo_al, lo, hi;    // staged: [lo, hi) of the batch, LDS byte 0 = batch byte lo_al
};

__device__ __forceinline__ uint64_t rd8(const Rows& R, int64_t p) {
  if (p >= R.lo && p + 8 <= R.hi && !((p - R.lo_al) & 7))
    return *reinterpret_cast<const uint64_t*>(R.stg + (p - R.lo_al));
  return *gl(reinterpret_cast<const uint64_t*>(R.g + p));
}
__device__ __forceinline__ uint8_t rd1(const Rows& R, int64_t p) {
  if (p >= R.lo && p < R.hi) return R.stg[p - R.lo_al];
  return gl(R.g)[p];
}
// w-byte little-endian value at p (w in 1, 2, 4, 8; p w-aligned in well-formed rows)
__device__ __forceinline__ uint64_t rdw(const Rows& R, int64_t p, int w) {
  if (p >= R.lo && p + w <= R.hi && !((p - R.lo_al) & (w - 1))) {
    const uint8_t* s = R.stg + (p - R.lo_al);
    switch (w) {
      case 8: return *reinterpret_cast<const uint64_t*>(s);
      case 4: return *reinterpret_cast<const uint32_t*>(s);
      case 2: return *reinterpret_cast<const uint16_t*>(s);
      default: return *s;
    }
  }
  const uint8_t* s = R.g + p;
  switch (w) {
    case 8: return *gl(reinterpret_cast<const uint64_t*>(s));
    case 4: return *gl(reinterpret_cast<const uint32_t*>(s));
    case 2: return *gl(reinterpret_cast<const uint16_t*>(s));
    default: return *gl(s);
  }
}
__device__ __forceinline__ bool rdbit(const Rows& R, int64_t p, int64_t i) {
  return (rd1(R, p + (i >> 3)) >> (i & 7)) & 1;
}

// A BinaryArray at p whose elements take es bytes: header, null bits and element slots inside the
// batch; returns numElements or -1 (the reference's BinaryArray.pointTo / getInt64 bounds).
__device__ __forceinline__ int64_t tarray_ok(const Rows& R, int64_t p, int es, int64_t total) {
  if (!span_ok(p, 8, total)) return -1;
  const int64_t m = static_cast<int32_t>(rd8(R, p));
  if (m < 0 || !span_ok(p, 8 + tbm(m) + m * es, total)) return -1;
  return m;
}

// Issues LDS-DMA copies of the 16-B pieces covering [gb, ge) to lds (16-aligned); returns nothing.
__device__ __forceinline__ void tstage(uint8_t* lds, const uint8_t* gb, const uint8_t* ge) {
  const uint64_t lo = reinterpret_cast<uint64_t>(gb) & ~uint64_t(15);
  const uint64_t hi = (reinterpret_cast<uint64_t>(ge) + 15) & ~uint64_t(15);
  const uint32_t nch = static_cast<uint32_t>((hi - lo) >> 4);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t i0 = wave * 64; i0 < nch; i0 += kTreeThreads)
    if (i0 + lane < nch)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(lo + 16ull * (i0 + lane)),
                                       lds + 16 * i0, 16, 0, 0);
}

__device__ __forceinline__ uint64_t tw_scan64(uint64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Exclusive scan of the uint32 array a[0, m) in LDS by the whole block (thread t owns a
// contiguous chunk).  Returns false when the sum does not fit 32 bits (every thread agrees).
__device__ bool block_scan_u32(uint32_t* a, uint32_t m, uint64_t* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t per = (m + kTreeThreads - 1) / kTreeThreads;
  const uint32_t b = min<uint32_t>(tid * per, m), e = min<uint32_t>(b + per, m);
  uint64_t s = 0;
  for (uint32_t i = b; i < e; i++) s += a[i];
  const uint64_t inc = tw_scan64(s);
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kTreeThreads / 64; w++) {
    const uint64_t v = wsum[w];
    pre += w < wave ? v : 0;
    tot += v;
  }
  uint64_t run = pre + inc - s;
  for (uint32_t i = b; i < e; i++) {
    const uint32_t v = a[i];
    a[i] = static_cast<uint32_t>(run);
    run += v;
  }
  __syncthreads();
  return tot < (1ull << 32);
}

// ORs the bits of 64 consecutive entries (lane l = output bit gbase + l, gbase = the wave's first
// entry, any alignment) into a bitmap shared with other waves / tiles: at most 3 atomics.
__device__ __forceinline__ void tballot_or(uint8_t* bits, int64_t gbase, bool pred) {
  const uint64_t b = __ballot(pred);
  if (!b) return;
  const int lane = threadIdx.x & 63;
  const int sh = static_cast<int>(gbase & 31);
  const uint64_t lo = b << sh;
  const uint32_t hi = sh ? static_cast<uint32_t>(b >> (64 - sh)) : 0u;
  if (lane < 3) {
    const uint32_t part = lane == 0 ? static_cast<uint32_t>(lo)
                        : lane == 1 ? static_cast<uint32_t>(lo >> 32) : hi;
    if (part)
      __hip_atomic_fetch_or(gl(reinterpret_cast<uint32_t*>(bits)) + (gbase >> 5) + lane, part,
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void tstore_w(uint8_t* p, int w, uint64_t v) {
  switch (w) {
    case 8: *gl(reinterpret_cast<uint64_t*>(p)) = v; break;
    case 4: *gl(reinterpret_cast<uint32_t*>(p)) = static_cast<uint32_t>(v); break;
    case 2: *gl(reinterpret_cast<uint16_t*>(p)) = static_cast<uint16_t>(v); break;
    default: *gl(p) = static_cast<uint8_t>(v); break;
  }
}

// len bytes of the batch at src -> dst (any alignment; only [dst, dst + len) written).
__device__ void tcopy_out(uint8_t* dst, const Rows& R, int64_t src, int64_t len) {
  if (len <= 0) return;
  int64_t i = 0;
  const int64_t head = min<int64_t>(len, (8 - (reinterpret_cast<uintptr_t>(dst) & 7)) & 7);
  for (; i < head; i++) gl(dst)[i] = rd1(R, src + i);
  const int64_t s = src + head;             // source of the first whole destination word
  const int o = static_cast<int>(s & 7);
  const int64_t nw = (len - head) >> 3;
  if (nw > 0) {
    const int64_t s0 = s - o;               // aligned source word
    uint64_t cur = rd8(R, s0);
    auto d64 = gl(reinterpret_cast<uint64_t*>(dst + head));
    for (int64_t w = 0; w < nw; w++) {
      uint64_t v;
      if (o == 0) {
        v = cur;
        if (w + 1 < nw) cur = rd8(R, s0 + 8 * (w + 1));
      } else {
        const uint64_t nxt = rd8(R, s0 + 8 * (w + 1));
        v = (cur >> (8 * o)) | (nxt << (64 - 8 * o));
        cur = nxt;
      }
      d64[w] = v;
    }
    i = head + 8 * nw;
  }
  for (; i < len; i++) gl(dst)[i] = rd1(R, src + i);
}

// Where an error of a nested entry is reported in pass 1: the node and the first row of the
// (sub-)tile walked (the entry's global index is not known before the scan).
__device__ __forceinline__ uint64_t err_where_tile(int node, int64_t row0) {
  return (1ull << 63) | (1ull << 62) | (static_cast<uint64_t>(node) << 40) |
         static_cast<uint64_t>(row0);
}

// Checked position (and count) of a non-null variable-length value at pos of node `n`
// (lv_value in levels.hip, the same checks in both passes).  Returns false: decode as null.
__device__ bool tcheck(const TreeArgs& a, const Rows& R, CTNode& n, int64_t pos,
                       int32_t size, int64_t total, uint32_t* count, uint64_t where) {
  bool ok = true;
  uint32_t c = 0;
  switch (n.type) {
    case FURY_TYPE_STRING:
    case FURY_TYPE_BINARY:
      ok = span_ok(pos, size, total);
      c = static_cast<uint32_t>(size);
      break;
    case FURY_TYPE_DECIMAL:
      ok = span_ok(pos, 16, total);
      break;
    case FURY_TYPE_STRUCT:
      ok = span_ok(pos, tbm(n.num_children) + 8 * n.num_children, total);
      break;
    case FURY_TYPE_LIST: {
      const int64_t m = tarray_ok(R, pos, tn(a, n.first_child).esize, total);
      ok = m >= 0;
      c = static_cast<uint32_t>(m);
      break;
    }
    case FURY_TYPE_MAP: {
      ok = span_ok(pos, 8, total);
      if (!ok) break;
      const int64_t kb = static_cast<int32_t>(rd8(R, pos));
      const int64_t nk = kb >= 0 ? tarray_ok(R, pos + 8, tn(a, n.first_child).esize, total) : -1;
      const int64_t nv = kb >= 0 ? tarray_ok(R, pos + 8 + kb, tn(a, n.first_child + 1).esize, total) : -1;
      ok = nk >= 0 && nv >= 0;
      if (ok && nk != nv) {
        raise_at(a.err, kErrMapCount, where);
        *count = 0;
        return false;
      }
      c = static_cast<uint32_t>(nk);
      break;
    }
    default:
      break;
  }
  if (!ok) {
    raise_at(a.err, kErrBounds, where);
    *count = 0;
    return false;
  }
  *count = c;
  return true;
}

// Owner of child entry q of a LIST / MAP node whose in-tile exclusive prefix is P[0, m]: the last
// e with P[e] <= q.
__device__ __forceinline__ uint32_t towner(const uint32_t* P, uint32_t m, uint32_t q) {
  uint32_t lo = 0, hi = m;                  // P[lo] <= q < P[hi] (P[m] = total > q)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P[mid] <= q) lo = mid; else hi = mid;
  }
  return lo;
}

// One walk of rows [s0, s1).  Returns false when the tile's arrays do not fit the arena.
template <bool kWrite>
__device__ bool tree_walk(const TreeArgs& a, TMeta* meta, uint64_t* wsum, uint8_t* stg,
                          uint8_t* arena, int64_t t, int64_t s0, int64_t s1, int64_t total) {
  const int tid = threadIdx.x;
  const int64_t nr = s1 - s0;
  // ---- stage the rows
  Rows R;
  R.g = a.rows;
  R.stg = stg;
  {
    const int64_t g0 = min<int64_t>(max<int64_t>(gl(a.offs)[s0], 0), total);
    const int64_t g1 = min<int64_t>(max<int64_t>(gl(a.offs)[s1], g0), total);
    // LDS byte 0 = the batch byte whose ADDRESS is the 16-aligned one at or below byte g0
    R.lo_al = g0 - static_cast<int64_t>((reinterpret_cast<uintptr_t>(a.rows) + g0) & 15);
    R.lo = g0;
    R.hi = min<int64_t>(g1, R.lo_al + a.stage_cap);
    if (R.hi > R.lo) tstage(stg, a.rows + R.lo_al, a.rows + R.hi);
    else R.hi = R.lo;
    __syncthreads();
  }
  uint32_t region_lo = 0, region_hi = 0;        // arena bytes of the previous level's arrays
  for (int L = 0; L < a.nlevels; L++) {
    const int nb = a.level_start[L], ne = a.level_start[L + 1];
    // ---- entries of this level's nodes and their arrays (uniform: every thread computes it)
    uint32_t need = 0;
    for (int n = nb; n < ne; n++) {
      CTNode& N = tn(a, n);
      uint32_t ec;
      if (L == 0) ec = static_cast<uint32_t>(nr);
      else if (tn(a, N.parent).type == FURY_TYPE_STRUCT) ec = meta[N.parent].ecnt;
      else ec = meta[N.parent].tot;
      if (!is_scalar(N.type)) need += 8 * ec;
      if (is_counted(N.type)) need += 4 * (ec + 1);
      if (tid == 0) meta[n].ecnt = ec;
    }
    need = (need + 15) & ~15u;
    uint32_t at;
    if (need <= region_lo) at = 0;
    else if (region_hi + need <= a.arena_cap) at = region_hi;
    else return false;                          // (uniform)
    __syncthreads();
    // (second uniform pass: array offsets; the SRC arrays first, then the contiguous count block)
    uint32_t p = at;
    for (int n = nb; n < ne; n++) {
      const uint32_t ec = meta[n].ecnt;
      if (!is_scalar(tn(a, n).type)) {
        if (tid == 0) meta[n].src = p;
        p += 8 * ec;
      }
    }
    const uint32_t cblk = p;
    for (int n = nb; n < ne; n++) {
      const uint32_t ec = meta[n].ecnt;
      if (is_counted(tn(a, n).type)) {
        if (tid == 0) meta[n].cnt = p;
        p += 4 * (ec + 1);
      }
    }
    const uint32_t cend = p;
    region_lo = at;
    region_hi = at + need;
    __syncthreads();
    // ---- expand: the entries of this level from the parent level (or the rows)
    for (int n = nb; n < ne; n++) {
      CTNode& N = tn(a, n);
      const uint32_t ec = meta[n].ecnt;
      const bool scalar = is_scalar(N.type);
      const bool counted = is_counted(N.type);
      int64_t* SRC = scalar ? nullptr : reinterpret_cast<int64_t*>(arena + meta[n].src);
      uint32_t* CNT = counted ? reinterpret_cast<uint32_t*>(arena + meta[n].cnt) : nullptr;
      const int32_t ptype = L == 0 ? -1 : tn(a, N.parent).type;
      const TMeta pm = L == 0 ? TMeta{} : meta[N.parent];
      const int64_t* PSRC = L == 0 ? nullptr : reinterpret_cast<const int64_t*>(arena + pm.src);
      const uint32_t* PP = (L == 0 || ptype == FURY_TYPE_STRUCT) ? nullptr
                           : reinterpret_cast<const uint32_t*>(arena + pm.cnt);
      const int es = N.esize;
      const int64_t gbase = kWrite ? meta[n].run_e : 0;
      for (uint32_t q0 = 0; q0 < ec; q0 += kTreeThreads) {
        const uint32_t q = q0 + tid;
        const bool live = q < ec;
        bool nul = true;
        int64_t slotp = 0, cont = 0;
        int64_t vpos = kNullPos;                // collection roots: the value at the row base
        int swid = 8;                           // bytes of the slot holding a scalar
        if (live) {
          if (L == 0) {
            const int64_t row = s0 + q;
            const int64_t base = gl(a.offs)[row];
            if (a.root) {
              nul = false;
              vpos = base;
            } else if (!span_ok(base, tbm(a.ntop) + 8 * a.ntop, total)) {
              if (N.ord == 0) raise_oob(a.err, row);
            } else {
              nul = rdbit(R, base, N.ord);
              slotp = base + tbm(a.ntop) + 8 * N.ord;
              cont = base;
            }
          } else if (ptype == FURY_TYPE_STRUCT) {
            const int64_t pb = PSRC[q];
            if (pb >= 0) {
              const int pnc = tn(a, N.parent).num_children;
              nul = rdbit(R, pb, N.ord);
              slotp = pb + tbm(pnc) + 8 * N.ord;
              cont = pb;
            }
          } else {                              // LIST / MAP element
            const uint32_t e = towner(PP, pm.ecnt, q);
            const uint32_t j = q - PP[e];
            const int64_t m = PP[e + 1] - PP[e];
            const int64_t pb = PSRC[e];
            int64_t arr = pb;
            if (ptype == FURY_TYPE_MAP)
              arr = N.ord == 0 ? pb + 8 : pb + 8 + static_cast<int32_t>(rd8(R, pb));
            nul = rdbit(R, arr + 8, j);
            slotp = arr + 8 + tbm(m) + static_cast<int64_t>(es) * j;
            cont = arr;
            swid = es;
          }
        }
        if (scalar) {
          if (kWrite) {
            const int w = N.width;
            uint64_t x = 0;
            if (live && !nul) x = rdw(R, slotp, swid == 8 ? w : es);
            const int64_t gi = gbase + q;
            if (N.type == FURY_TYPE_BOOL) {
              if (N.values) tballot_or(N.values, gbase + q0 + (tid & ~63), live && !nul && (x & 0xff));
            } else if (live && N.values) {
              tstore_w(N.values + gi * w, w, x);
            }
            if (N.validity) tballot_or(N.validity, gbase + q0 + (tid & ~63), live && !nul);
          }
          continue;
        }
        if (!live) continue;
        int64_t pos = kNullPos;
        uint32_t c = 0;
        if (!nul) {
          int32_t size = 0;
          if (vpos >= 0) {
            pos = vpos;
          } else {
            const uint64_t slot = rd8(R, slotp);
            pos = cont + static_cast<int32_t>(slot >> 32);
            size = static_cast<int32_t>(slot);
          }
          if (!tcheck(a, R, N, pos, size, total, &c, err_where_tile(n, s0))) pos = kNullPos;
        }
        SRC[q] = pos;
        if (counted) CNT[q] = c;
      }
      if (counted && tid == 0) CNT[ec] = 0;
    }
    __syncthreads();
    // ---- in-tile prefixes of the level's counts (one scan over the contiguous count block; a
    // node's prefix is relative to its first slot)
    if (cend > cblk) {
      uint32_t* blk = reinterpret_cast<uint32_t*>(arena + cblk);
      if (!block_scan_u32(blk, (cend - cblk) / 4, wsum)) return false;
      // rebase each node's segment to start at 0 and record its total
      for (int n = nb; n < ne; n++) {
        if (!is_counted(tn(a, n).type)) continue;
        uint32_t* P = reinterpret_cast<uint32_t*>(arena + meta[n].cnt);
        const uint32_t ec = meta[n].ecnt;
        const uint32_t b0 = P[0];
        const uint32_t tot = P[ec] - b0;
        __syncthreads();                        // every thread has read P[0] before it changes
        for (uint32_t i = tid; i <= ec; i += kTreeThreads) P[i] -= b0;
        if (tid == 0) meta[n].tot = tot;
      }
      __syncthreads();
    }
    // ---- pass 2: the level's non-scalar outputs (pass 1 only needed the counts)
    if (!kWrite) continue;
    for (int n = nb; n < ne; n++) {
      CTNode& N = tn(a, n);
      if (is_scalar(N.type)) continue;
      const uint32_t ec = meta[n].ecnt;
      const int64_t* SRC = reinterpret_cast<const int64_t*>(arena + meta[n].src);
      const uint32_t* P = is_counted(N.type) ? reinterpret_cast<const uint32_t*>(arena + meta[n].cnt) : nullptr;
      const int64_t gbase = meta[n].run_e;
      const int64_t bbase = meta[n].run_b;
      const int64_t cbase = (N.type == FURY_TYPE_LIST || N.type == FURY_TYPE_MAP)
                                ? meta[N.first_child].run_e : 0;
      for (uint32_t e0 = 0; e0 < ec; e0 += kTreeThreads) {
        const uint32_t e = e0 + tid;
        const bool live = e < ec;
        const int64_t pos = live ? SRC[e] : kNullPos;
        const bool valid = pos >= 0;
        if (N.validity) tballot_or(N.validity, gbase + e0 + (tid & ~63), valid);
        if (!live) continue;
        const int64_t gi = gbase + e;
        switch (N.type) {
          case FURY_TYPE_STRING:
          case FURY_TYPE_BINARY: {
            const uint32_t p0 = P[e], p1 = P[e + 1];
            if (N.offsets) {
              gl(N.offsets)[gi + 1] = static_cast<int32_t>(bbase + p1);
              if (gi == 0) gl(N.offsets)[0] = 0;
            }
            if (valid && N.values) tcopy_out(N.values + bbase + p0, R, pos, p1 - p0);
            break;
          }
          case FURY_TYPE_LIST:
          case FURY_TYPE_MAP:
            if (N.offsets) {
              gl(N.offsets)[gi + 1] = static_cast<int32_t>(cbase + P[e + 1]);
              if (gi == 0) gl(N.offsets)[0] = 0;
            }
            break;
          case FURY_TYPE_DECIMAL:
            if (N.values) {
              const auto d = gl(reinterpret_cast<uint64_t*>(N.values + 16 * gi));
              d[0] = valid ? rd8(R, pos) : 0;
              d[1] = valid ? rd8(R, pos + 8) : 0;
            }
            break;
          default:
            break;
        }
      }
    }
  }
  return true;
}

template <bool kWrite>
__global__ __launch_bounds__(kTreeThreads) void tree_dec_kernel(TreeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tsm[];
  TMeta* meta = reinterpret_cast<TMeta*>(tsm);
  uint64_t* wsum = reinterpret_cast<uint64_t*>(tsm + sizeof(TMeta) * a.nn);
  uint8_t* stg = tsm + ((sizeof(TMeta) * a.nn + 64 + 15) & ~size_t(15));
  uint8_t* arena = stg + a.stage_cap;
  const int tid = threadIdx.x;
  const int64_t t = blockIdx.x;
  const int64_t r0 = t * a.tile_rows, r1 = min<int64_t>(r0 + a.tile_rows, a.nrows);
  const int64_t total = gl(a.offs)[a.nrows];
  for (int n = tid; n < a.nn; n += kTreeThreads) {
    meta[n].run_e = kWrite ? a.cnt[static_cast<int64_t>(n) * a.ntiles + t] : 0;
    meta[n].run_b = kWrite ? a.byt[static_cast<int64_t>(n) * a.ntiles + t] : 0;
  }
  __syncthreads();
  int64_t s0 = r0, sub = r1 - r0;
  while (s0 < r1) {
    const int64_t s1 = min(s0 + sub, r1);
    if (!tree_walk<kWrite>(a, meta, wsum, stg, arena, t, s0, s1, total)) {
      __syncthreads();
      if (s1 - s0 == 1) {                       // one row does not fit: the level engine decodes
        if (!kWrite && tid == 0)
          __hip_atomic_store(a.overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      sub = (s1 - s0 + 1) / 2;                  // walk the tile in halves (deterministic: the
      continue;                                 // other pass splits it the same way)
    }
    __syncthreads();
    for (int n = tid; n < a.nn; n += kTreeThreads) {
      meta[n].run_e += meta[n].ecnt;
      const int ty = tn(a, n).type;
      if (ty == FURY_TYPE_STRING || ty == FURY_TYPE_BINARY) meta[n].run_b += meta[n].tot;
    }
    __syncthreads();
    s0 = s1;
  }
  if (!kWrite)
    for (int n = tid; n < a.nn; n += kTreeThreads) {
      a.cnt[static_cast<int64_t>(n) * a.ntiles + t] = meta[n].run_e;
      a.byt[static_cast<int64_t>(n) * a.ntiles + t] = meta[n].run_b;
    }
}

// Exclusive scan over the tiles of each [node] row of cnt (rows 0..nn-1) and byt (rows nn..2nn-1);
// tot[row] = the row's total.  One 1024-thread workgroup per row.
constexpr int kScanT = 1024;
__global__ __launch_bounds__(kScanT) void tree_tile_scan(int64_t* cnt, int64_t* byt, int64_t ntiles,
                                                         int32_t nn, int64_t* tot) {
  __shared__ int64_t ws[kScanT / 64];
  const int row = blockIdx.x;
  int64_t* v = row < nn ? cnt + static_cast<int64_t>(row) * ntiles : byt + static_cast<int64_t>(row - nn) * ntiles;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t per = (ntiles + kScanT - 1) / kScanT;
  const int64_t b = min<int64_t>(tid * per, ntiles), e = min<int64_t>(b + per, ntiles);
  int64_t s = 0;
  for (int64_t i = b; i < e; i++) s += v[i];
  int64_t x = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) ws[wave] = x;
  __syncthreads();
  int64_t pre = 0, all = 0;
  for (int w = 0; w < kScanT / 64; w++) {
    pre += w < wave ? ws[w] : 0;
    all += ws[w];
  }
  int64_t run = pre + x - s;
  for (int64_t i = b; i < e; i++) {
    const int64_t c = v[i];
    v[i] = run;
    run += c;
  }
  if (tid == 0) tot[row] = all;
}

int tree_host_width(int32_t t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

int g_tree_mode = 1;             // tuning "nested_decode": 0 tree tiles, 1 level engine
uint32_t g_tree_stage = 32 * 1024, g_tree_arena = 24 * 1024;

}  // namespace

void set_tree_mode(int v) { g_tree_mode = v; }
int tree_mode() { return g_tree_mode; }
void set_tree_lds(uint32_t stage, uint32_t arena) {
  if (stage) g_tree_stage = (stage + 15) & ~15u;
  if (arena) g_tree_arena = (arena + 15) & ~15u;
}
uint32_t tree_lds(int which) { return which ? g_tree_arena : g_tree_stage; }

struct TreePlan {
  std::vector<TNode> nodes;
  std::vector<int32_t> level_start;
  int64_t nrows = 0, ntiles = 0;
  int32_t tile_rows = 0, ntop = 0, root = 0;
  uint32_t stage_cap = 0, arena_cap = 0;
  int64_t* cnt = nullptr;          // scanned [nn][ntiles] bases (device, plan-owned)
  int64_t* byt = nullptr;
  hipStream_t stream = nullptr;
};

void tree_free(TreePlan* p) {
  if (!p) return;
  dev_free(p->cnt, p->stream);
  dev_free(p->byt, p->stream);
  delete p;
}

namespace {

int tree_launch(const TreePlan& p, bool write, const TNode* dev_nodes, const uint8_t* rows,
                const int64_t* offs, int32_t* overflow, hipStream_t hs) {
  TreeArgs a{};
  a.nodes = dev_nodes;
  a.rows = rows;
  a.offs = offs;
  a.nrows = p.nrows;
  a.ntiles = p.ntiles;
  a.cnt = p.cnt;
  a.byt = p.byt;
  a.err = device_error_word(hs);
  a.overflow = overflow;
  a.nn = static_cast<int32_t>(p.nodes.size());
  a.ntop = p.ntop;
  a.root = p.root;
  a.nlevels = static_cast<int32_t>(p.level_start.size()) - 1;
  a.tile_rows = p.tile_rows;
  a.stage_cap = p.stage_cap;
  a.arena_cap = p.arena_cap;
  for (int i = 0; i <= a.nlevels; i++) a.level_start[i] = p.level_start[i];
  const size_t lds = ((sizeof(TMeta) * a.nn + 64 + 15) & ~size_t(15)) + p.stage_cap + p.arena_cap;
  const void* fn = write ? reinterpret_cast<const void*>(tree_dec_kernel<true>)
                         : reinterpret_cast<const void*>(tree_dec_kernel<false>);
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  if (write)
    hipLaunchKernelGGL(tree_dec_kernel<true>, dim3(static_cast<unsigned>(p.ntiles)),
                       dim3(kTreeThreads), lds, hs, a);
  else
    hipLaunchKernelGGL(tree_dec_kernel<false>, dim3(static_cast<unsigned>(p.ntiles)),
                       dim3(kTreeThreads), lds, hs, a);
  return check_hip(hipGetLastError(), "tree decode launch");
}

}  // namespace

// Pass 1 + tile scan + the one host sync.  *out stays NULL (FURY_OK) when the batch needs the
// level engine: schema beyond the tree tables, or a row whose arrays do not fit the arena.
int tree_prepare(const fury_schema* s, const uint8_t* rows, const int64_t* offs, int64_t nrows,
                 hipStream_t hs, TreePlan** out, std::vector<int64_t>* totals) {
  *out = nullptr;
  const int nn = static_cast<int>(s->nodes.size());
  if (g_tree_mode != 0 || nn > kTreeMaxNodes || s->depth > kTreeMaxLevels || nrows <= 0)
    return FURY_OK;
  TreePlan* p = new TreePlan();
  p->stream = hs;
  p->nrows = nrows;
  p->ntop = s->num_fields;
  p->root = s->root;
  p->stage_cap = g_tree_stage;
  p->arena_cap = g_tree_arena;
  p->nodes.assign(nn, TNode{});
  std::vector<int32_t> level(nn, 0);
  for (int i = 0; i < nn; i++) {
    const GenTpl& g = s->nodes[i];
    TNode& n = p->nodes[i];
    n.type = g.type_id;
    n.first_child = g.first_child;
    n.num_children = g.num_children;
    if (i < s->num_fields) {
      n.parent = -1;
      n.ord = i;
    }
    n.width = tree_host_width(g.type_id);
    n.esize = n.width > 0 ? n.width : 8;
    for (int j = 0; j < g.num_children; j++) {
      TNode& c = p->nodes[g.first_child + j];
      c.parent = i;
      c.ord = j;
      level[g.first_child + j] = level[i] + 1;
    }
  }
  const int nlev = nn ? level[nn - 1] + 1 : 0;
  p->level_start.assign(nlev + 1, nn);
  for (int i = nn - 1; i >= 0; i--) p->level_start[level[i]] = i;
  p->level_start[0] = 0;
  for (int L = 1; L <= nlev; L++)               // BFS: levels are contiguous and increasing
    if (p->level_start[L] < p->level_start[L - 1]) p->level_start[L] = p->level_start[L - 1];
  // tile rows from the batch's average row size (one small read)
  int64_t* pin = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&pin), 8 * (2 * nn + 2), hipHostMallocDefault) != hipSuccess) {
    delete p;
    return set_error(FURY_ERR_DEVICE, "hipHostMalloc (tree plan)");
  }
  int st = check_hip(hipMemcpyAsync(pin, offs + nrows, 8, hipMemcpyDeviceToHost, hs), "hipMemcpyAsync");
  if (!st) st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize");
  if (st) {
    (void)hipHostFree(pin);
    delete p;
    return st;
  }
  const int64_t total = std::max<int64_t>(pin[0], 1);
  const double avg = std::max(8.0, static_cast<double>(total) / static_cast<double>(nrows));
  p->tile_rows = static_cast<int32_t>(std::clamp<double>(0.9 * p->stage_cap / avg, 1.0, 256.0));
  p->ntiles = (nrows + p->tile_rows - 1) / p->tile_rows;
  int32_t* overflow = nullptr;
  int64_t* tot = nullptr;
  DeviceTable dt;
  if (!st) st = dev_alloc(8 * nn * p->ntiles, hs, reinterpret_cast<void**>(&p->cnt));
  if (!st) st = dev_alloc(8 * nn * p->ntiles, hs, reinterpret_cast<void**>(&p->byt));
  if (!st) st = dev_alloc(8 * (2 * nn + 2), hs, reinterpret_cast<void**>(&tot));
  if (!st) {
    overflow = reinterpret_cast<int32_t*>(tot + 2 * nn);
    st = check_hip(hipMemsetAsync(overflow, 0, 8, hs), "hipMemsetAsync");
  }
  if (!st) st = upload_table(p->nodes.data(), p->nodes.size() * sizeof(TNode), hs, &dt);
  if (!st) st = tree_launch(*p, false, static_cast<const TNode*>(dt.dev), rows, offs, overflow, hs);
  if (!st) {
    hipLaunchKernelGGL(tree_tile_scan, dim3(static_cast<unsigned>(2 * nn)), dim3(kScanT), 0, hs,
                       p->cnt, p->byt, p->ntiles, nn, tot);
    st = check_hip(hipGetLastError(), "tree scan launch");
  }
  if (!st) st = check_hip(hipMemcpyAsync(pin, tot, 8 * (2 * nn + 1), hipMemcpyDeviceToHost, hs),
                          "hipMemcpyAsync totals");
  if (!st) st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize");
  const bool over = !st && reinterpret_cast<const int32_t*>(pin + 2 * nn)[0] != 0;
  if (!st && !over) {
    totals->assign(2 * nn, 0);
    for (int i = 0; i < nn; i++) {
      (*totals)[2 * i] = pin[i];
      (*totals)[2 * i + 1] = pin[nn + i];
    }
  }
  (void)hipHostFree(pin);
  dev_free(tot, hs);
  if (st || over) {
    tree_free(p);
    return st;
  }
  *out = p;
  return FURY_OK;
}

int tree_execute(const TreePlan* p, const GenNode* outs, const uint8_t* rows, const int64_t* offs,
                 const std::vector<int64_t>& totals, hipStream_t hs) {
  std::vector<TNode> nodes(p->nodes);
  for (size_t i = 0; i < nodes.size(); i++) {
    nodes[i].values = const_cast<uint8_t*>(outs[i].values);
    nodes[i].validity = outs[i].validity;
    nodes[i].offsets = outs[i].offsets;
  }
  DeviceTable dt;
  int st = upload_table(nodes.data(), nodes.size() * sizeof(TNode), hs, &dt);
  if (st) return st;
  // nodes without entries still get Arrow offsets [0]
  for (size_t i = 0; i < nodes.size() && !st; i++)
    if (totals[2 * i] == 0 && nodes[i].offsets)
      st = check_hip(hipMemsetAsync(nodes[i].offsets, 0, 4, hs), "hipMemsetAsync offsets");
  if (st) return st;
  return tree_launch(*p, true, static_cast<const TNode*>(dt.dev), rows, offs, nullptr, hs);
}

}  // namespace fury
