// bfs.hip — nested decode, level-parallel inside a tile ("tile BFS"): the default engine of
// fury_decode_prepare / fury_decode_execute for nested schemas (tree.hip plans it; the row walk of
// walk.hip and the level engine of levels.hip take a batch whose tiles overflow the on-chip arena).
//
// Reference semantics are the row walk's (tree.hip header): the getters of BinaryRow / BinaryArray /
// BinaryMap as the generated fromRow and ArrowWriter walk them (FMT/encoder/
// BaseBinaryEncoderBuilder.java:459-706, FMT/vectorized/ArrowWriter.java:205-640), entries of a
// node in (parent entry, element) order, a null struct a null entry in every child (StructWriter.
// appendNull :577-584), a null list / map a zero-length entry, null values zeroed, every container
// checked against the batch when it is reached (tcheck, shared with the walk: MemoryBuffer's
// bounds).
//
// MI355X design.  The row walk gives each lane one row and walks it depth first:
// a chain of ~30 dependent reads per row, so it needs many rows in flight to hide latency -- more
// than L2 holds (the write pass re-fetched its rows 6x) or LDS holds (a staged walk ran at 1.5
// waves per SIMD, 53 us per 64-row tile: profiles/r06_phases.jsonl).  Here a workgroup stages the
// tile's rows in LDS ONCE and walks the SCHEMA, not the rows: nodes in breadth-first order (a parent
// before its children), and for each node all of the tile's entries of that node at once, one lane
// per entry, NT entries per step:
//   * an entry's slot is found from its parent's per-entry record in an LDS arena (a struct's
//     position; a list's / map's position, element count and in-tile element prefix) -- for a list
//     element, the owning parent entry comes from an owner array built once per list node by a
//     scatter of each entry's first element and a block max-scan (no per-element search);
//   * the node's entries of the tile are CONSECUTIVE in its Arrow column (their base is the tile
//     prefix the count pass's scan gives), so values and offsets leave as coalesced stores and
//     validity / BOOL bits as wave ballots -- no output windows, no per-row cursors (the walk's
//     rowpre array and its 4 B x counted nodes x rows are gone);
//   * every lane of a step runs the same node type: no divergence beyond null / invalid entries.
// Pass 1 (count) visits only the nodes that hold or contain a counted slot (TNode.walk: the same
// containers the walk's count pass checks) and writes each node's entries / payload bytes per tile;
// tree_tile_scan turns them into tile bases.  Pass 2 (write) visits every node.  A tile whose
// per-node records do not fit the arena sets the plan's overflow flag: the batch then decodes on
// the row walk (or the level engine), which bound aliasing rows by an item budget.
#include "tree_dev.h"

namespace fury {

namespace {

// Per-node table in LDS (thread 0 writes, the block reads after the node's closing barrier):
// [0] arena byte offset of the node's entry records (-1: none), [1] entries in the tile,
// [2] arena byte offset of its owner array (LIST / MAP: child entry -> parent entry), [3] child
// entries (LIST / MAP: the node's elements in the tile).
constexpr int kNt = 4;

struct BLayout {
  size_t stg, arena, ntab, rb, nbase, wsum, end;
};

// LDS: the staged rows, the arena, the node table, the tile's row bases (trows + 1: loaded once,
// not per top-level node) and every node's output bases of the tile (pass 2: one gather up front,
// not three dependent global loads per node).
__host__ __device__ inline BLayout bfs_layout(int nn, int nt, uint32_t stage, uint32_t arena,
                                              int trows) {
  BLayout l{};
  size_t b = 0;
  l.stg = b;
  b += (stage + 15) & ~15u;
  l.arena = b;
  b += (arena + 15) & ~15u;
  l.ntab = b;
  b += 4 * kNt * static_cast<size_t>(nn);
  b = (b + 15) & ~size_t(15);
  l.rb = b;
  b += 8 * static_cast<size_t>(trows + 1);
  l.nbase = b;
  b += 16 * static_cast<size_t>(nn);
  b = (b + 15) & ~size_t(15);
  l.wsum = b;
  b += 8 * static_cast<size_t>(nt / 64 + 2);
  l.end = (b + 15) & ~size_t(15);
  return l;
}

// Node boundaries and scans use lds_barrier() (kernels.h): __syncthreads() also waits for every
// outstanding global store -- each node boundary then paid the HBM write latency of the node's
// outputs (~2 us per node: profiles/r06_bfs_phases.jsonl).  No global location this kernel writes
// is read back by it, so only LDS needs ordering.
// Inclusive 32-bit wave scans by DPP (row shifts 1, 2, 4, 8 inside each 16-lane row, then the
// row broadcasts 15 / 31; lanes without a source take `old`: 0 for the sum, -1 for the max) --
// a few cycles per step where __shfl_up is an LDS permute round trip; the per-node chain of this
// kernel is latency-bound, so its scans must be short.
__device__ __forceinline__ uint32_t dpp_scan_add(uint32_t x) {
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x111, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x112, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x114, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x118, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x142, 0xa, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x143, 0xc, 0xf, false));
  return x;
}
__device__ __forceinline__ int32_t dpp_scan_max(int32_t x) {
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xa, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xc, 0xf, false));
  return x;
}

// Exclusive block scan of v (every thread calls it; the block's sum fits 32 bits: one tile's
// elements / payload bytes of one node in one chunk); *total = the block's sum.
template <int NT>
__device__ __forceinline__ uint64_t bscan(uint32_t v, uint64_t* wsum, uint64_t* total) {
  const int wave = threadIdx.x >> 6;
  const uint32_t inc = dpp_scan_add(v);
  const uint32_t wt = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(inc), 63));
  if constexpr (NT == 64) {
    *total = wt;
    return inc - v;
  } else {
    if ((threadIdx.x & 63) == 0) wsum[wave] = wt;
    lds_barrier();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
      const uint64_t s = wsum[w];
      pre += w < wave ? s : 0;
      tot += s;
    }
    lds_barrier();                        // wsum is reused by the next scan
    *total = tot;
    return pre + inc - v;
  }
}

// Inclusive block max-scan of v with a running carry (owner arrays); returns the scanned value and
// updates *carry to the block's maximum.
template <int NT>
__device__ __forceinline__ int32_t bmaxscan(int32_t v, int64_t* wsum, int32_t* carry) {
  const int wave = threadIdx.x >> 6;
  v = dpp_scan_max(v);
  const int32_t wmax = __builtin_amdgcn_readlane(v, 63);
  int32_t c = *carry;
  if constexpr (NT == 64) {
    v = max(v, c);
    *carry = max(c, wmax);
    return v;
  } else {
    const int lane = threadIdx.x & 63;
    (void)lane;
    if ((threadIdx.x & 63) == 0) wsum[wave] = wmax;
    lds_barrier();
    int32_t all = c;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
      const int32_t s = static_cast<int32_t>(wsum[w]);
      if (w < wave) c = max(c, s);
      all = max(all, s);
    }
    lds_barrier();
    *carry = all;
    return max(v, c);
  }
}

// Stages the bytes of rows [r0, r0 + nr) (as much as the stage holds) and returns the reader.
template <int NT>
__device__ __forceinline__ Rows bfs_stage(const TreeArgs& a, uint8_t* stg, int64_t r0, int64_t nr,
                                          int64_t total) {
  Rows R;
  R.g = a.rows;
  R.stg = stg;
  const int64_t g0 = min<int64_t>(max<int64_t>(gl(a.offs)[r0], 0), total);
  const int64_t g1 = min<int64_t>(max<int64_t>(gl(a.offs)[r0 + nr], g0), total);
  R.lo_al = g0 - static_cast<int64_t>((reinterpret_cast<uintptr_t>(a.rows) + g0) & 15);
  R.lo = g0;
  R.hi = min<int64_t>(g1, R.lo_al + a.stage_cap);
  if (R.hi > R.lo) tstage<NT>(stg, a.rows + R.lo_al, a.rows + R.hi);
  else R.hi = R.lo;
  return R;
}

// The arena: per container node, its entries' records (position, element count, in-tile element
// prefix) and, for a LIST / MAP, the owner array of its elements.
struct BArena {
  uint8_t* base;
  uint32_t cap, used;
  // reserves bytes (16-aligned) and returns the offset, or -1 (the tile overflows)
  __device__ __forceinline__ int32_t take(uint64_t bytes) {
    const uint64_t b = (bytes + 15) & ~uint64_t(15);
    if (used + b > cap) return -1;
    const int32_t off = static_cast<int32_t>(used);
    used += static_cast<uint32_t>(b);
    return off;
  }
};

template <class T>
__device__ __forceinline__ LdsT<T>* arr_at(uint8_t* arena, int32_t off) {
  return lds_ptr<T>(arena + off);
}

// Diagnostics (tuning "tree_debug", as walk.hip's): thread 0 adds the time between marks to
// acc[id]; flushed to a.dbg[base + id] (count pass base 0, write pass 16), workgroups counted at
// a.dbg[64 + base / 16].  Phases: 0 stage + row / node bases, 1 the top level, 2 the nested levels.
struct BClock {
  uint64_t* acc;
  __device__ __forceinline__ void mark(int id) const {
    if (acc && threadIdx.x == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      acc[id] += t - acc[15];
      acc[15] = t;
    }
  }
  __device__ __forceinline__ void start() const {
    if (acc && threadIdx.x < 16) acc[threadIdx.x] = threadIdx.x == 15 ? __builtin_amdgcn_s_memrealtime() : 0;
  }
  __device__ __forceinline__ void flush(uint64_t* dbg, int base) const {
    if (acc && threadIdx.x < 15)
      atomicAdd(reinterpret_cast<unsigned long long*>(dbg) + base + threadIdx.x,
                static_cast<unsigned long long>(acc[threadIdx.x]));
    if (acc && threadIdx.x == 15)
      atomicAdd(reinterpret_cast<unsigned long long*>(dbg) + 64 + base / 16, 1ull);
  }
};

// One node of the tile, processed by ONE wave (lane = entry, 64 entries per step, DPP wave scans:
// no block barrier inside).  Returns false when the arena overflows.
template <bool W>
__device__ __forceinline__ bool bfs_node(const TreeArgs& a, int n, const Rows& R, int32_t* ntab,
                                         const int64_t* rbs, const int64_t* nbase, uint8_t* arena,
                                         uint32_t* used, int64_t r0, int64_t nr, int64_t total,
                                         int64_t t) {
  const int lane = threadIdx.x & 63;
  n = __builtin_amdgcn_readfirstlane(n);
  CTNode& N = tn(a, n);
  const int ty = N.type;
  const int P = N.parent;
  const int ntop = a.ntop;
  const int64_t hbt = tbm(ntop);
  // entries of node n in the tile: the rows, the parent struct's entries, or the parent list's /
  // map's elements
  int64_t E = nr;
  int32_t poff = -1, pown = -1, pE = 0;
  int pty = 0;
  if (P >= 0) {
    CTNode& PN = tn(a, P);
    pty = PN.type;
    poff = ntab[kNt * P];
    pE = ntab[kNt * P + 1];
    pown = ntab[kNt * P + 2];
    E = pty == FURY_TYPE_STRUCT ? pE : ntab[kNt * P + 3];
  }
  const bool strc = ty == FURY_TYPE_STRUCT, coll = ty == FURY_TYPE_LIST || ty == FURY_TYPE_MAP;
  const bool bytes = ty == FURY_TYPE_STRING || ty == FURY_TYPE_BINARY;
  const bool scal = N.width > 0;
  const bool visit = (W || N.walk) && E > 0;
  // records of a container's entries: needed when its children are visited (pass 2: always;
  // pass 1: when a child holds a counted slot -- a list<int64> only counts its elements)
  bool kids = W;
  if (!W && (strc || coll))
    for (int c = 0; c < N.num_children; c++) kids |= tn(a, N.first_child + c).walk != 0;
  // arena: taken identically in both passes (records of every container with entries, the owner
  // array of every LIST / MAP with elements) -- pass 1 fills only what its walk needs, but a tile
  // that fits in pass 1 must fit in pass 2.  Waves allocate concurrently (LDS atomic bump).
  auto take = [&](uint64_t bytes_) -> int32_t {
    const uint32_t b = static_cast<uint32_t>((bytes_ + 15) & ~uint64_t(15));
    uint32_t off = 0;
    if (lane == 0) off = atomicAdd(used, b);
    off = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(off)));
    if (bytes_ > a.arena_cap || off + b > a.arena_cap) return -1;
    return static_cast<int32_t>(off);
  };
  int32_t noff = -1;
  if ((strc || coll) && E > 0) {
    noff = take(16 * static_cast<uint64_t>(E));
    if (noff < 0) return false;
  }
  const int64_t base = W ? nbase[n] : 0;                        // the tile's first entry of n
  const int64_t bbase = W && bytes ? nbase[a.nn + n] : 0;
  const int64_t cbase = W && coll ? nbase[N.first_child] : 0;
  uint64_t carry = 0;                             // elements / payload bytes of earlier steps
  if (visit) {
    const int hbp = P >= 0 && pty == FURY_TYPE_STRUCT ? static_cast<int>(tbm(tn(a, P).num_children)) : 0;
    for (int64_t c0 = 0; c0 < E; c0 += 64) {
      const int64_t i = c0 + lane;
      const bool live = i < E;
      // locate the entry: its null bit (bm, bit) and slot, and the container it is relative to
      bool can = false;
      int64_t bm = 0, slot = 0, cont = 0, bit = 0, row = r0;
      if (live) {
        if (P < 0) {
          row = r0 + i;
          const int64_t rb = rbs[i];
          can = span_ok(rb, hbt + 8 * ntop, total);    // (raised once, before the level loop)
          bm = rb;
          bit = N.ord;
          slot = rb + hbt + 8 * N.ord;
          cont = rb;
        } else if (pty == FURY_TYPE_STRUCT) {
          const int64_t pp = *arr_at<int64_t>(arena, poff + 8 * static_cast<int32_t>(i));
          can = pp >= 0;
          bm = pp;
          bit = N.ord;
          slot = pp + hbp + 8 * N.ord;
          cont = pp;
        } else {
          const int32_t e = *arr_at<int32_t>(arena, pown + 4 * static_cast<int32_t>(i));
          const uint32_t pm = *arr_at<uint32_t>(arena, poff + 8 * pE + 4 * e);
          const uint32_t pre = *arr_at<uint32_t>(arena, poff + 12 * pE + 4 * e);
          const int64_t pp = *arr_at<int64_t>(arena, poff + 8 * e);
          const int64_t j = i - pre;
          int64_t arr = pp;
          if (pty == FURY_TYPE_MAP)
            arr = N.ord == 0 ? pp + 8 : pp + 8 + static_cast<int32_t>(rd8(R, pp));
          can = true;
          bm = arr + 8;
          bit = j;
          slot = arr + 8 + tbm(pm) + static_cast<int64_t>(N.esize) * j;
          cont = arr;
        }
      }
      // the null bit and the slot / value together: one round trip
      uint32_t nb = 1;
      uint64_t sv = 0;
      if (can) {
        nb = rd1(R, bm + (bit >> 3)) >> (bit & 7);
        sv = scal ? rdw(R, slot, N.width) : rd8(R, slot);
      }
      const bool nul = !can || (nb & 1);
      if (scal) {                                 // (pass 2 only: scalars hold no counted slot)
        const uint64_t x = nul ? 0 : sv;
        if (ty == FURY_TYPE_BOOL) {
          if (N.values) tballot_or(N.values, base + c0, live && !nul && (x & 0xff));
        } else if (N.values && live) {
          tstore_w(N.values + (base + i) * N.width, N.width, x);
        }
        if (N.validity) tballot_or(N.validity, base + c0, live && !nul);
        continue;
      }
      // a non-scalar value: checked where it is (tcheck: the walk's rule), then by type
      int64_t pos = kNullPos;
      uint32_t cnt = 0;
      if (live && !nul) {
        pos = cont + static_cast<int32_t>(sv >> 32);
        const uint64_t where = P < 0 ? static_cast<uint64_t>(row) : err_where_tile(n, r0);
        if (!tcheck(a, R, N, pos, static_cast<int32_t>(sv), total, &cnt, where)) pos = kNullPos;
      }
      const bool valid = pos >= 0;
      if (W && N.validity) tballot_or(N.validity, base + c0, live && valid);
      if (bytes || coll) {
        const uint32_t v = valid ? cnt : 0u;
        // 32-bit wave scans: a count that could overflow one (a multi-GB payload or aliased
        // elements) sends the batch to the row walk
        if (!W && __ballot(v > 0xffffffffu / 64) && lane == 0)
          __hip_atomic_store(a.overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t inc = dpp_scan_add(v);
        const uint64_t pre = carry + (inc - v);
        if (coll && live && kids) {
          *arr_at<int64_t>(arena, noff + 8 * static_cast<int32_t>(i)) = valid ? pos : kNullPos;
          *arr_at<uint32_t>(arena, noff + 8 * static_cast<int32_t>(E) + 4 * static_cast<int32_t>(i)) = v;
          *arr_at<uint32_t>(arena, noff + 12 * static_cast<int32_t>(E) + 4 * static_cast<int32_t>(i)) =
              static_cast<uint32_t>(pre);
        }
        if (W && live && N.offsets) {
          const int64_t end = (bytes ? bbase : cbase) + static_cast<int64_t>(pre) + v;
          gl(N.offsets)[base + i + 1] = static_cast<int32_t>(end);
          if (base + i == 0) gl(N.offsets)[0] = 0;
        }
        if (W && bytes && valid && N.values && v) tcopy_out(N.values + bbase + pre, R, pos, v);
        carry += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(inc), 63));
      } else if (strc) {
        if (live && kids) *arr_at<int64_t>(arena, noff + 8 * static_cast<int32_t>(i)) = valid ? pos : kNullPos;
      } else if (W && ty == FURY_TYPE_DECIMAL && N.values && live) {
        const uint64_t lo = valid ? rd8(R, pos) : 0, hi = valid ? rd8(R, pos + 8) : 0;
        const auto d = gl(reinterpret_cast<uint64_t*>(N.values + 16 * (base + i)));
        d[0] = lo;
        d[1] = hi;
      }
    }
  }
  // a LIST / MAP's owner array (child entry -> parent entry), built by this wave alone
  int32_t own = -1;
  const uint64_t C = coll ? carry : 0;
  if (coll && C > 0) {
    own = take(4 * C);
    if (own < 0) return false;
  }
  if (visit && coll && kids && C > 0) {
    auto ow = arr_at<int32_t>(arena, own);
    for (uint64_t k = lane; k < C; k += 64) ow[k] = -1;
    for (int64_t e = lane; e < E; e += 64) {         // each non-empty entry marks its first element
      const uint32_t m = *arr_at<uint32_t>(arena, noff + 8 * static_cast<int32_t>(E) + 4 * static_cast<int32_t>(e));
      const uint32_t pr = *arr_at<uint32_t>(arena, noff + 12 * static_cast<int32_t>(E) + 4 * static_cast<int32_t>(e));
      if (m > 0) ow[pr] = static_cast<int32_t>(e);
    }
    int32_t mc = -1;
    for (uint64_t k0 = 0; k0 < C; k0 += 64) {      // max-scan: every element gets its owner
      const uint64_t k = k0 + lane;
      int32_t v = dpp_scan_max(k < C ? ow[k] : -1);
      v = max(v, mc);
      mc = __builtin_amdgcn_readlane(v, 63);
      if (k < C) ow[k] = v;
    }
  }
  if (lane == 0) {
    if (!W) {
      a.cnt[n * a.stride + t] = E;
      a.byt[n * a.stride + t] = bytes ? static_cast<int64_t>(carry) : 0;
    }
    ntab[kNt * n] = noff;
    ntab[kNt * n + 1] = static_cast<int32_t>(E);
    ntab[kNt * n + 2] = own;
    ntab[kNt * n + 3] = static_cast<int32_t>(C);
  }
  return true;
}

// Pass 1 (W false) / pass 2 (W true) over one tile: the schema's levels in order; inside a level
// the waves take its nodes round robin (the nodes of one level are independent: a wave per node
// overlaps their LDS round-trip chains), one LDS barrier per level.
template <int NT, bool W>
__global__ __launch_bounds__(NT) void bfs_kernel(TreeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t bsm[];
  const BLayout L = bfs_layout(a.nn, NT, a.stage_cap, a.arena_cap, a.trows);
  int32_t* ntab = reinterpret_cast<int32_t*>(bsm + L.ntab);
  uint32_t* ctl = reinterpret_cast<uint32_t*>(bsm + L.wsum);     // [0] arena used, [1] overflow
  int64_t* rbs = reinterpret_cast<int64_t*>(bsm + L.rb);
  int64_t* nbase = reinterpret_cast<int64_t*>(bsm + L.nbase);    // [n]: entries, [nn + n]: bytes
  __shared__ uint64_t tacc[16];
  const BClock clk{a.dbg ? tacc : nullptr};
  clk.start();
  const int tid = threadIdx.x, wave = tid >> 6;
  const int64_t t = blockIdx.x;
  const int64_t r0 = t * a.trows;
  const int64_t nr = min<int64_t>(a.trows, a.nrows - r0);
  const int64_t total = gl(a.offs)[a.nrows];
  const int ntop = a.ntop;
  const int64_t hbt = tbm(ntop);
  const Rows R = bfs_stage<NT>(a, bsm + L.stg, r0, nr, total);
  if (tid == 0) ctl[0] = ctl[1] = 0;
  // the rows' own null bitmaps and slots inside the batch (the walk's rowok, both passes)
  for (int64_t i = tid; i < nr; i += NT) {
    const int64_t rb = gl(a.offs)[r0 + i];
    rbs[i] = rb;
    if (!span_ok(rb, hbt + 8 * ntop, total)) raise_oob(a.err, r0 + i);
  }
  if (W)
    for (int i = tid; i < a.nn; i += NT) {
      nbase[i] = a.cnt[i * a.stride + t];
      nbase[a.nn + i] = a.byt[i * a.stride + t];
    }
  __syncthreads();                // (a full barrier: the stage's LDS-DMA and the global loads)
  clk.mark(0);
  for (int lv = 0; lv < a.nlevels; lv++) {
    for (int n = a.lvl[lv] + wave; n < a.lvl[lv + 1]; n += NT / 64)
      if (!bfs_node<W>(a, n, R, ntab, rbs, nbase, bsm + L.arena, ctl, r0, nr, total, t) &&
          (tid & 63) == 0)
        ctl[1] = 1;
    lds_barrier();
    clk.mark(lv == 0 ? 1 : 2);
    if (ctl[1]) {                 // uniform after the barrier: the tile's records outgrew the arena
      if (tid == 0) {
        if (!W) __hip_atomic_store(a.overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else raise_at(a.err, kErrInternal, static_cast<uint64_t>(r0));
      }
      return;
    }
  }
  clk.flush(a.dbg, W ? 16 : 0);
}

}  // namespace

size_t bfs_lds(int nn, int nt, uint32_t stage, uint32_t arena, int trows) {
  return bfs_layout(nn, nt, stage, arena, trows).end;
}

int bfs_launch(const TreeArgs& a, int nt, bool write, hipStream_t hs) {
  const size_t lds = bfs_lds(a.nn, nt, a.stage_cap, a.arena_cap, a.trows);
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(a.ntiles)), dim3(nt), lds, hs, a);
  };
  if (write) {
    if (nt == 64) go(bfs_kernel<64, true>);
    else if (nt == 128) go(bfs_kernel<128, true>);
    else if (nt == 256) go(bfs_kernel<256, true>);
    else go(bfs_kernel<512, true>);
  } else {
    if (nt == 64) go(bfs_kernel<64, false>);
    else if (nt == 128) go(bfs_kernel<128, false>);
    else if (nt == 256) go(bfs_kernel<256, false>);
    else go(bfs_kernel<512, false>);
  }
  return check_hip(hipGetLastError(), "tile BFS decode launch");
}

}  // namespace fury
