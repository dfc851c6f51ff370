// tree_dev.h — device side of the row-walk nested decode (walk.hip; tree.hip plans it).  Node records, the batch reader (LDS stage or HBM),
// the bounds checks every pass applies identically, block scans and bitmap helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

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
  int32_t k;                // walk.hip: counted slot (LIST / MAP elements, STRING / BINARY bytes), -1
  int32_t walk;             // walk.hip count pass: the node or a descendant has a counted slot
  int32_t ek;               // walk.hip: counted slot of the LIST / MAP whose elements hold this
                            // node's entries (through STRUCTs); -1: one entry per row
  int32_t top;              // the top-level field whose subtree holds the node
  int32_t pad_;
};

constexpr int kTreeMaxNodes = 512;
constexpr int kMaxLevels = 64;
constexpr int kMaxGroups = 32;

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
  uint32_t stage_cap;       // LDS bytes of the row stage (count / write pass)
  int32_t pad_;
  uint64_t* dbg;            // diagnostics (tuning "tree_debug"): phase times, or NULL
  int64_t stride;           // row stride of cnt / byt (ntiles + 1: [ntiles] = the node's total)
  uint32_t* rowpre;         // [K][nrows]: a row's in-tile exclusive prefix of counted slot k
  int32_t K;                // counted slots
  uint32_t pool_cap;        // LDS bytes of the bitmap windows (write pass)
  int32_t prefetch;         // write pass: each wave first pulls its rows' lines (tuning)
  int32_t skip;             // diagnostics (tuning "walk_skip", outputs wrong): 1 payload copies,
                            // 2 bitmaps, 4 scalar values, 8 offsets not written
  int32_t tmul;             // write pass: count tiles per write tile (1 or 2)
  int32_t ctr;              // rows per count tile
  int32_t knode[256];       // counted slot -> node (kWalkMaxK)
  uint32_t out_cap;         // write pass: LDS bytes of the output windows (tuning "walk_out")
  int32_t trows;            // bfs.hip: rows per tile
  uint32_t arena_cap;       // bfs.hip: LDS bytes of the per-node entry records
  int32_t pad2_;
  int32_t lvl[kMaxLevels + 1];  // bfs.hip: first node of each level (breadth-first numbering)
  // walk.hip field groups (round 6): group g walks top-level fields [gf[g], gf[g + 1]) of its tile's
  // rows and owns counted slots [gk[g], gk[g + 1]) (numbered subtree by subtree); Kl = the largest
  // group's slots (the LDS cursors are per group)
  int32_t ngrp, Kl;
  int32_t gf[kMaxGroups + 1];
  int32_t gk[kMaxGroups + 1];
};

constexpr int kWalkMaxK = 256;     // round 6: was 64 (wide nested beans went to the level engine)
constexpr int kWalkMaxDepth = 5;      // deeper: the level engine (register budget of the walk)

// walk.hip launchers (tree.hip owns the plan): LDS bytes of a pass, and the launch itself.
size_t walk_lds(const TreeArgs& a, int nt, bool write);
size_t walk_write_lds(int nn, int K, int nt, uint32_t stage, uint32_t pool, bool prefetch,
                      uint32_t out);
size_t walk_count_lds(int nn, int K, int nt, uint32_t stage, bool prefetch);
constexpr size_t kWalkLdsMax = 159 * 1024;   // LDS of one workgroup (160 KB, static arrays aside)
int walk_launch(const TreeArgs& a, int nt, bool write, hipStream_t hs);
// bfs.hip (tile BFS decode, the default): LDS bytes of a workgroup, and the launch itself.
size_t bfs_lds(int nn, int nt, uint32_t stage, uint32_t arena, int trows);
int bfs_launch(const TreeArgs& a, int nt, bool write, hipStream_t hs);

// Diagnostics: thread 0 of a workgroup adds the time since its previous mark to tacc[id]
// (s_memrealtime, 100 MHz); the kernel adds tacc to dbg at the end.
#define TMARK(sh, id)                                                              \
  do {                                                                             \
    if ((sh).tacc && threadIdx.x == 0) {                                           \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                        \
      (sh).tacc[id] += t_ - (sh).tacc[15];                                         \
      (sh).tacc[15] = t_;                                                          \
    }                                                                              \
  } while (0)

namespace {

constexpr int64_t kNullPos = -1;

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
template <int NT>
__device__ __forceinline__ void tstage(uint8_t* lds, const uint8_t* gb, const uint8_t* ge) {
  const uint64_t lo = reinterpret_cast<uint64_t>(gb) & ~uint64_t(15);
  const uint64_t hi = (reinterpret_cast<uint64_t>(ge) + 15) & ~uint64_t(15);
  const uint32_t nch = static_cast<uint32_t>((hi - lo) >> 4);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t i0 = wave * 64; i0 < nch; i0 += NT)
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
template <int NT>
__device__ __forceinline__ bool block_scan_u32(uint32_t* a, uint32_t m, uint64_t* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t per = (m + NT - 1) / NT;
  const uint32_t b = min<uint32_t>(tid * per, m), e = min<uint32_t>(b + per, m);
  uint64_t s = 0;
  for (uint32_t i = b; i < e; i++) s += a[i];
  const uint64_t inc = tw_scan64(s);
  if (lane == 63) wsum[wave] = inc;
  lds_barrier();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
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
  lds_barrier();
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

// Pointers into LDS with the address space explicit (ds_* instructions, never flat).
template <class T>
using LdsT = __attribute__((address_space(3))) T;
template <class T>
__device__ __forceinline__ LdsT<T>* lds_ptr(void* generic_lds) { return (LdsT<T>*)(generic_lds); }
// A w-byte store through a uint8_t pointer P of any address space: global (gl()), LDS (lds_ptr) or
// generic (flat: the write pass's output windows and HBM through one instruction stream).
template <class P, class T>
using SameAs = typename std::conditional<
    std::is_same<typename std::remove_pointer<P>::type, LdsT<uint8_t>>::value, LdsT<T>,
    typename std::conditional<std::is_same<typename std::remove_pointer<P>::type, uint8_t>::value, T,
                              __attribute__((address_space(1))) T>::type>::type;
template <class P>
__device__ __forceinline__ void tstore_wp(P p, int w, uint64_t v) {
  using AS16 = SameAs<P, uint16_t>;
  using AS32 = SameAs<P, uint32_t>;
  using AS64 = SameAs<P, uint64_t>;
  switch (w) {
    case 8: *reinterpret_cast<AS64*>(p) = v; break;
    case 4: *reinterpret_cast<AS32*>(p) = static_cast<uint32_t>(v); break;
    case 2: *reinterpret_cast<AS16*>(p) = static_cast<uint16_t>(v); break;
    default: *p = static_cast<uint8_t>(v); break;
  }
}

// len bytes of the batch at src -> dst (any alignment; only [dst, dst + len) written).  The source
// is read as aligned words (a word past the payload only when the payload reaches into it); the
// destination takes at most three stores of 1 / 2 / 4 bytes before its first 8-byte boundary and
// after its last, whole words in between (short strings: ~5 stores instead of ~15 byte stores).
// P: a global (gl()) or LDS (lds_ptr) uint8_t pointer -- the write pass assembles a tile's
// payload range in an LDS window (walk.hip) and stores it as whole lines.
template <class P>
__device__ void tcopy_to(P dst, const Rows& R, int64_t src, int64_t len) {
  if (len <= 0) return;
  const int64_t s0 = src & ~int64_t(7);
  const int o = static_cast<int>(src & 7);
  // 8 payload bytes from payload byte i (bytes past len are garbage, never stored)
  auto word_at = [&](int64_t i) -> uint64_t {
    const int64_t p = o + i;
    const int64_t q = s0 + (p & ~int64_t(7));
    const int sh = static_cast<int>(p & 7) * 8;
    const uint64_t a = rd8(R, q);
    if (!sh || (p & 7) + min<int64_t>(8, len - i) <= 8) return sh ? a >> sh : a;
    return (a >> sh) | (rd8(R, q + 8) << (64 - sh));
  };
  auto put_small = [&](P d, uint64_t v, int n) {   // n < 8 bytes, d + n 8-aligned or end
    int k = 0;
    while (k < n) {
      const uintptr_t ad = reinterpret_cast<uintptr_t>(d + k);
      if ((ad & 1) || n - k < 2) {
        tstore_wp(d + k, 1, v >> (8 * k));
        k += 1;
      } else if ((ad & 2) || n - k < 4) {
        tstore_wp(d + k, 2, v >> (8 * k));
        k += 2;
      } else {
        tstore_wp(d + k, 4, v >> (8 * k));
        k += 4;
      }
    }
  };
  const int64_t head = min<int64_t>(len, (8 - (reinterpret_cast<uintptr_t>(dst) & 7)) & 7);
  if (head > 0) put_small(dst, word_at(0), static_cast<int>(head));
  const int64_t nw = (len - head) >> 3;
  for (int64_t w = 0; w < nw; w++) tstore_wp(dst + head + 8 * w, 8, word_at(head + 8 * w));
  const int64_t t0 = head + 8 * nw;
  if (t0 < len) put_small(dst + t0, word_at(t0), static_cast<int>(len - t0));
}
__device__ __forceinline__ void tcopy_out(uint8_t* dst, const Rows& R, int64_t src, int64_t len) {
  tcopy_to(gl(dst), R, src, len);
}

// One wave stores bytes img[0, n) of an LDS window (16-aligned, >= 16 readable bytes past n) to
// g[0, n) (any alignment, every byte of the range this wave's): bytes up to g's 16-byte boundary,
// 16-B non-temporal stores funnel-shifted out of aligned window words, the byte tail.
__device__ __forceinline__ void wave_store_window(uint8_t* g, const uint8_t* img, int64_t n) {
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  if (n <= 0) return;
  const int lane = threadIdx.x & 63;
  const auto im = lds_ptr<const uint8_t>(const_cast<uint8_t*>(img));
  const auto i64 = lds_ptr<const uint64_t>(const_cast<uint8_t*>(img));
  const int64_t head = min<int64_t>(n, (16 - (reinterpret_cast<uintptr_t>(g) & 15)) & 15);
  const int64_t body = (n - head) >> 4;
  const int64_t t0 = head + 16 * body;
  if (lane < head) gl(g)[lane] = im[lane];
  if (lane < n - t0) gl(g)[t0 + lane] = im[t0 + lane];
  const int sh = static_cast<int>(head & 7) * 8;
  for (int64_t m = lane; m < body; m += 64) {
    const int64_t q = (head + 16 * m) >> 3;
    uint64_t x, y;
    if (sh == 0) {
      x = i64[q];
      y = i64[q + 1];
    } else {
      const uint64_t w0 = i64[q], w1 = i64[q + 1], w2 = i64[q + 2];
      x = (w0 >> sh) | (w1 << (64 - sh));
      y = (w1 >> sh) | (w2 << (64 - sh));
    }
    v4 vv;
    vv.x = static_cast<uint32_t>(x); vv.y = static_cast<uint32_t>(x >> 32);
    vv.z = static_cast<uint32_t>(y); vv.w = static_cast<uint32_t>(y >> 32);
    __builtin_nontemporal_store(vv, gl(reinterpret_cast<v4*>(g + head + 16 * m)));
  }
}

// Where an error of a nested entry is reported in pass 1: the node and the first row of the
// (sub-)tile walked (the entry's global index is not known before the scan).
__device__ __forceinline__ uint64_t err_where_tile(int node, int64_t row0) {
  return (1ull << 63) | (1ull << 62) | (static_cast<uint64_t>(node) << 40) |
         static_cast<uint64_t>(row0);
}

// Checked position (and count) of a non-null variable-length value at pos of node `n`
// (lv_value in levels.hip, the same checks in both passes).  Returns false: decode as null.
__device__ __forceinline__ bool tcheck(const TreeArgs& a, const Rows& R, CTNode& n, int64_t pos,
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

}  // namespace
}  // namespace fury
