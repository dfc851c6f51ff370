// walk.hip — nested decode with a thread per ROW ("row walk"): the default engine of
// fury_decode_prepare / fury_decode_execute for schemas of up to kWalkMaxDepth levels and
// kWalkMaxK (256, round 6) counted nodes (tree.hip builds the plan; the level engine takes the rest).  A deeper
// walk on an explicit per-lane stack was built and measured 2.5-6.5x slower than the level
// engine on depth 6-20 schemas (profiles/r05_deep_walk_vs_levels.jsonl), so the level engine is
// the fallback.
//
// Reference semantics are tree.hip's (its header): the getters of BinaryRow / BinaryArray /
// BinaryMap as the generated fromRow and ArrowWriter walk them (FMT/encoder/
// BaseBinaryEncoderBuilder.java:459-706, FMT/vectorized/ArrowWriter.java:205-640), entries of a
// node in (parent entry, element) order, a null struct a null entry in every child, a null list /
// map a zero-length entry, null values zeroed, every read bounds-checked (tcheck, shared).
//
// MI355X design.  A workgroup owns NT consecutive rows, one per thread, whose bytes are staged in
// LDS by LDS-DMA (rows past the stage are read from HBM).  A thread walks its row depth first:
// inside one row, every node's entries come in (parent entry, element) order, so a row only needs
// one CURSOR per counted slot -- each LIST / MAP node (its elements) and each STRING / BINARY node
// (its payload bytes) -- to place everything it writes.
//   pass 1 (prepare): the walk adds up each row's counted slots (thread-private LDS counters), one
//     wave-scan per slot turns them into in-tile row prefixes -> rowpre[k][row] (4 B per row and
//     slot, coalesced), and the tile totals give every node's entries / payload bytes in the tile
//     (a node's entries are the rows, or the elements of its nearest LIST / MAP ancestor) ->
//     [node][tile], which tree_tile_scan turns into tile bases (the one host sync reads totals).
//   pass 2 (execute): cursors = tile base + rowpre; the walk writes values, offsets and payloads
//     at their final positions.  Validity / BOOL bits of row-aligned nodes (one entry per row) go
//     out by wave ballots; the other nodes' bits collect in LDS windows over the tile's entry range
//     (ds_or), flushed as whole words at the end (edge words, shared with the neighbouring tiles,
//     by atomic OR; a node whose window does not fit the pool ORs straight into HBM).
// Scalar subtrees are skipped by the counting walk (TNode.walk).  The per-row work is a serial
// chain of dependent LDS reads; occupancy, not bandwidth, bounds it.
#include "tree_dev.h"

namespace fury {

namespace {

// LDS working set (laid out by walk_layout).
struct WShared {
  uint32_t* cur;            // [K][NT]: a thread's cursor (pass 1: its row's totals)
  int64_t* kb;              // [K]: tile base of counted slot k (pass 2)
  int32_t* win;             // [2][nn]: LDS word of node n's validity / BOOL-value window, -1: none
  int64_t* w0;              // [nn]: first global bitmap word of node n's windows
  uint32_t* req;            // [2][nn + 1]: window words, scanned into window offsets
  uint64_t* wsum;           // [K][NT / 64] (pass 1) / [16] (pass 2) scan scratch
  uint32_t* pool;           // window words
  int32_t* ow;              // [3][nn]: output window (values / offsets / payload) of node n in
                            // opool, -1: stored straight to HBM
  uint32_t* olen;           // [3][nn]: its bytes
  int64_t* oe;              // [2][nn]: the tile's first entry (E0) / payload byte (B0) of node n
  uint32_t* oreq;           // [3 nn + 1]: window bytes, scanned into window offsets
  uint8_t* opool;           // output windows
  uint8_t* pf;              // prefetch landing zone
  uint8_t* stg;             // staged rows
};

struct WLayout {
  size_t cur, kb, win, w0, req, wsum, pool, ow, olen, oe, oreq, opool, pf, stg, end;
};

__host__ __device__ inline WLayout walk_layout(int nn, int K, int nt, uint32_t stage, uint32_t pool,
                                               bool write, bool prefetch, uint32_t out = 0) {
  WLayout l{};
  size_t b = 0;
  l.cur = b;
  b += 4 * static_cast<size_t>(K) * nt;
  b = (b + 15) & ~size_t(15);
  l.kb = b;
  b += 8 * static_cast<size_t>(K);
  l.w0 = b;
  b += write ? 8 * static_cast<size_t>(nn) : 0;
  l.win = b;
  b += write ? 4 * 2 * static_cast<size_t>(nn) : 0;
  l.req = b;
  b += write ? 4 * 2 * static_cast<size_t>(nn + 1) : 0;
  b = (b + 15) & ~size_t(15);
  l.wsum = b;
  b += 8 * static_cast<size_t>(write ? 16 : K * (nt / 64));
  b = (b + 15) & ~size_t(15);
  l.pool = b;
  b += write ? pool : 0;
  b = (b + 15) & ~size_t(15);
  const bool ow = write && out > 0;
  l.oe = b;
  b += ow ? 8 * 2 * static_cast<size_t>(nn) : 0;
  l.ow = b;
  b += ow ? 4 * 3 * static_cast<size_t>(nn) : 0;
  l.olen = b;
  b += ow ? 4 * 3 * static_cast<size_t>(nn) : 0;
  l.oreq = b;
  b += ow ? 4 * (3 * static_cast<size_t>(nn) + 1) : 0;
  b = (b + 15) & ~size_t(15);
  l.opool = b;
  b += ow ? out : 0;
  b = (b + 15) & ~size_t(15);
  l.pf = b;                                   // prefetch landing zone: 1 KB, shared by the waves
  b += prefetch ? 1024 : 0;                   // (the data is discarded: overlapping writes are harmless)
  l.stg = b;
  b += stage;
  l.end = (b + 15) & ~size_t(15);
  return l;
}

__device__ inline WShared walk_shared(uint8_t* base, const TreeArgs& a, int nt, bool write) {
  const WLayout l = walk_layout(a.nn, a.Kl, nt, a.stage_cap, a.pool_cap, write, a.prefetch != 0,
                                a.out_cap);
  WShared s;
  s.cur = reinterpret_cast<uint32_t*>(base + l.cur);
  s.kb = reinterpret_cast<int64_t*>(base + l.kb);
  s.win = reinterpret_cast<int32_t*>(base + l.win);
  s.w0 = reinterpret_cast<int64_t*>(base + l.w0);
  s.req = reinterpret_cast<uint32_t*>(base + l.req);
  s.wsum = reinterpret_cast<uint64_t*>(base + l.wsum);
  s.pool = reinterpret_cast<uint32_t*>(base + l.pool);
  s.ow = reinterpret_cast<int32_t*>(base + l.ow);
  s.olen = reinterpret_cast<uint32_t*>(base + l.olen);
  s.oe = reinterpret_cast<int64_t*>(base + l.oe);
  s.oreq = reinterpret_cast<uint32_t*>(base + l.oreq);
  s.opool = base + l.opool;
  s.pf = base + l.pf;
  s.stg = base + l.stg;
  return s;
}

// Stages the bytes of rows [r0, r0 + nr) (as much as the stage holds) and returns the reader.
template <int NT>
__device__ inline Rows walk_stage(const TreeArgs& a, uint8_t* stg, int64_t r0, int64_t nr,
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

// The wave's 64 rows are one contiguous byte range: pull its lines past the stage (from `from`)
// into the caches with coalesced 16-B LDS-DMA loads into a scratch zone (data discarded), so the
// walk's dependent reads hit L2 instead of each paying an HBM round trip.
__device__ inline void walk_prefetch(const TreeArgs& a, const WShared& sh, int64_t r0, int tid,
                                     int64_t total, int64_t from) {
  const int64_t wr0 = r0 + (tid & ~63);
  if (wr0 >= a.nrows) return;
  const int64_t wr1 = min<int64_t>(wr0 + 64, a.nrows);
  const int64_t g0 = min<int64_t>(max<int64_t>(max<int64_t>(gl(a.offs)[wr0], from), 0), total);
  const int64_t g1 = min<int64_t>(max<int64_t>(gl(a.offs)[wr1], g0), total);
  const uintptr_t lo = reinterpret_cast<uintptr_t>(a.rows + g0) & ~uintptr_t(15);
  const uintptr_t hi = (reinterpret_cast<uintptr_t>(a.rows + g1) + 15) & ~uintptr_t(15);
  uint8_t* land = sh.pf;
  for (uintptr_t q = lo + 16 * (tid & 63); q < hi; q += 1024)
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(q), land, 16, 0, 0);
}

// Walk context of one thread.
struct WCtx {
  const TreeArgs* a;
  const WShared* sh;
  const Rows* R;
  int64_t total;
  int64_t row;
  int64_t wave_row;         // the row of lane 0 of this wave (ballots of row-aligned nodes)
  int tid;
  // count pass: items (fields, elements, keys, values) the walk of the current top-level field
  // may still visit, 2 x the row's bytes + 64.  A row the encoder wrote holds every item in its
  // own bytes (an 8-B slot, or >= 1 B per fixed-width element), so only a malformed row whose slots
  // alias other bytes runs out -- its walk would otherwise grow with the product of the aliased
  // counts -- and is reported (the prepare fails, so the write pass, which visits the same items,
  // never meets such a row).  Per top-level field, so that field groups see the same budget.
  mutable int32_t left;
  int kg0;                  // the group's first counted slot (LDS cursors / bases are per group)
  int f0, f1;               // the group's top-level fields
};

// Tile t and field group g of this workgroup.  One group: t = blockIdx.x.  Several: the grid is
// ceil(tiles / 8) x 8 x ngrp blocks and the groups of a tile are consecutive blocks of ONE XCD
// (blocks go to the 8 XCDs round robin), so they read the tile's rows through the same L2 at about
// the same time.  Returns false for the padding blocks past the last tile.
__device__ __forceinline__ bool wgroup(const TreeArgs& a, int64_t* t, int* g) {
  const int64_t b = blockIdx.x;
  if (a.ngrp <= 1) {
    *t = b;
    *g = 0;
    return true;
  }
  const int64_t q = b >> 3;
  *g = static_cast<int>(q % a.ngrp);
  *t = (q / a.ngrp) * 8 + (b & 7);
  return *t < a.ntiles;
}

// Charges a container's items to the row's budget (count pass): false, and the row reported, when
// it is spent.  (Null structs are free: their fields read nothing.)  The level engine (deeper
// schemas) materialises every level instead: aliased counts there end in an allocation failure.
template <bool W>
__device__ __forceinline__ bool wcharge(const WCtx& c, int ty, bool valid, uint32_t m) {
  if constexpr (W) {
    return true;
  } else {
    const int64_t items = ty == FURY_TYPE_MAP ? 2 * static_cast<int64_t>(m)
                          : (ty == FURY_TYPE_STRUCT && !valid) ? 0 : m;
    const int64_t left = static_cast<int64_t>(c.left) - items;
    c.left = static_cast<int32_t>(max<int64_t>(left, -1));
    if (left >= 0) return true;
    if (left + items >= 0) raise_at(c.a->err, kErrBudget, static_cast<uint64_t>(c.row));
    return false;
  }
}

// Bit `e` of node n's validity (which = 0) / BOOL values (which = 1).  Row-aligned nodes (e = the
// row) take a wave ballot: every active lane calls this at the same node, pred or not.
__device__ __forceinline__ void wbit(const WCtx& c, CTNode& N, int n, int which, uint8_t* bits,
                                     int64_t e, bool pred) {
  if (N.ek < 0) {
    tballot_or(bits, c.wave_row, pred);
    return;
  }
  if (!pred) return;
  const int w = c.sh->win[which * c.a->nn + n];
  if (w >= 0) {
    const int64_t rel = e - (c.sh->w0[n] << 5);
    atomicOr(c.sh->pool + w + (rel >> 5), 1u << (rel & 31));
  } else {
    __hip_atomic_fetch_or(gl(reinterpret_cast<uint32_t*>(bits)) + (e >> 5), 1u << (e & 31),
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Bits of consecutive entries e0, e0 + 1, ... (mask bit q = entry e0 + q, q < 32) OR-ed into node
// n's window (or the bitmap in HBM): at most two words.  Not for row-aligned nodes.
__device__ __forceinline__ void wbits_run(const WCtx& c, int n, int which, uint8_t* bits,
                                          int64_t e0, uint32_t mask) {
  if (!mask) return;
  const int sh = static_cast<int>(e0 & 31);
  const uint32_t lo = mask << sh;
  const uint32_t hi = sh ? static_cast<uint32_t>(static_cast<uint64_t>(mask) >> (32 - sh)) : 0u;
  const int64_t w = e0 >> 5;
  const int wi = c.sh->win[which * c.a->nn + n];
  if (wi >= 0) {
    uint32_t* p = c.sh->pool + wi + (w - c.sh->w0[n]);
    if (lo) atomicOr(p, lo);
    if (hi) atomicOr(p + 1, hi);
  } else {
    auto g = gl(reinterpret_cast<uint32_t*>(bits)) + w;
    if (lo) __hip_atomic_fetch_or(g, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (hi) __hip_atomic_fetch_or(g + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Output windows (write pass, a.out_cap > 0): the tile's entries of a node that is not row-aligned
// (values of fixed-width / DECIMAL nodes, Arrow offsets of LIST / MAP / STRING / BINARY nodes) and
// the tile's payload bytes of every STRING / BINARY node (round 6; row-aligned ones too: a tile's
// payload range [B0, B1) is its own) are assembled in LDS and stored as whole lines at the end of
// the tile: per-lane 1-8 B stores straight to HBM left partial lines (WRITE_SIZE 1.98x the column
// bytes at 4M depth-3 rows).  A node whose window did not fit the
// pool (ow < 0), and the row-aligned ones (coalesced already), store to HBM.
__device__ __forceinline__ int32_t wwin(const WCtx& c, int which, int n) {
  return c.a->out_cap ? c.sh->ow[which * c.a->nn + n] : -1;
}
// The value x (w bytes) of entry e of fixed-width node n.
__device__ __forceinline__ void wput_val(const WCtx& c, CTNode& N, int n, int64_t e, int w,
                                         uint64_t x) {
  const int32_t o = N.ek >= 0 ? wwin(c, 0, n) : -1;
  if (o >= 0) tstore_wp(lds_ptr<uint8_t>(c.sh->opool + o + (e - c.sh->oe[n]) * w), w, x);
  else tstore_w(N.values + e * w, w, x);
}
// Arrow offset v of entry e + 1 of node n (offsets[0] = 0 by entry 0, straight to HBM).
__device__ __forceinline__ void wput_off(const WCtx& c, CTNode& N, int n, int64_t e, int32_t v) {
  const int32_t o = N.ek >= 0 ? wwin(c, 1, n) : -1;
  if (o >= 0) *lds_ptr<int32_t>(c.sh->opool + o + 4 * (e - c.sh->oe[n])) = v;
  else gl(N.offsets)[e + 1] = v;
  if (e == 0) gl(N.offsets)[0] = 0;
}
// cnt payload bytes of the batch at pos -> payload byte bp of STRING / BINARY node n: into the
// node's payload window when it has one, else straight to HBM.  (Round 4: a second, inlined
// instance of tcopy_to took the walk from 125 to 242 VGPRs; tcopy_to is out of line: the depth-3
// instance stays at 126.)
__device__ __forceinline__ void wput_bytes(const WCtx& c, CTNode& N, int n, int64_t bp, int64_t pos,
                                           uint32_t cnt) {
  const int32_t o = wwin(c, 2, n);
  if (o >= 0)
    tcopy_to(lds_ptr<uint8_t>(c.sh->opool + o + (bp - c.sh->oe[c.a->nn + n])), *c.R, pos, cnt);
  else
    tcopy_out(N.values + bp, *c.R, pos, cnt);
}

// m fixed-width elements of a LIST / MAP side (write pass) at entries cs, cs + 1, ...: values one
// by one, validity / BOOL bits batched 32 elements to an atomic pair, null bits read a word at a
// time.
__device__ __forceinline__ void welems(const WCtx& c, CTNode& C, int cn, int64_t cs, int64_t arr,
                                       int64_t hb, uint32_t m) {
  const Rows& R = *c.R;
  const int es = C.esize;
  const int64_t ev = arr + 8 + hb;
  const bool bits = !(c.a->skip & 2);
  uint64_t nb = 0;
  uint32_t vm = 0, bm = 0;
  int64_t eb = cs;
  for (uint32_t j = 0; j < m; j++) {
    if ((j & 63) == 0) nb = rd8(R, arr + 8 + (j >> 3));
    const bool cnul = (nb >> (j & 63)) & 1;
    uint64_t x = rdw(R, ev + static_cast<int64_t>(es) * j, es);   // in the array: load, then mask
    if (cnul) x = 0;
    const int q = static_cast<int>(j & 31);
    if (C.type == FURY_TYPE_BOOL) {
      if (!cnul && (x & 0xff)) bm |= 1u << q;
    } else if (C.values && !(c.a->skip & 4)) {
      wput_val(c, C, cn, cs + j, C.width, x);
    }
    if (!cnul) vm |= 1u << q;
    if (q == 31 || j + 1 == m) {
      if (bits) {
        if (C.validity) wbits_run(c, cn, 0, C.validity, eb, vm);
        if (C.type == FURY_TYPE_BOOL && C.values) wbits_run(c, cn, 1, C.values, eb, bm);
      }
      eb += q + 1;
      vm = bm = 0;
    }
  }
}

// A fixed-width entry (write pass): value sv (loaded with its null bit; 0 when null), BOOL bit,
// validity bit.
__device__ __forceinline__ void wscalar(const WCtx& c, CTNode& N, int n, int64_t e, bool nul,
                                        uint64_t sv) {
  const uint64_t x = nul ? 0 : sv;
  if (c.a->skip & 2) {
    if (N.type != FURY_TYPE_BOOL && N.values && !(c.a->skip & 4)) wput_val(c, N, n, e, N.width, x);
    return;
  }
  if (N.type == FURY_TYPE_BOOL) {
    if (N.values) wbit(c, N, n, 1, N.values, e, !nul && (x & 0xff));
  } else if (N.values) {
    if (!(c.a->skip & 4)) wput_val(c, N, n, e, N.width, x);
  }
  if (N.validity) wbit(c, N, n, 0, N.validity, e, !nul);
}

// The entry's own part of entry e of node n (non-scalar): its bounds check, validity bit, cursor
// of a counted slot, Arrow offset, payload / DECIMAL value.  Returns whether the value is valid;
// *m = the items a container's walk visits below it (STRUCT: fields, LIST / MAP: elements, 0 for
// a leaf) and *cs = a LIST / MAP's first element entry.
template <bool W>
__device__ __forceinline__ bool wentry(const WCtx& c, CTNode& N, int n, int64_t e, bool nul,
                                       uint64_t slot, int64_t cont, int64_t vpos, bool top,
                                       int64_t* ppos, uint32_t* pm, int64_t* pcs) {
  const TreeArgs& a = *c.a;
  const Rows& R = *c.R;
  const int ty = N.type;
  int64_t pos = kNullPos;
  uint32_t cnt = 0;
  if (!nul) {
    int32_t size = 0;
    if (vpos >= 0) {
      pos = vpos;
    } else {
      pos = cont + static_cast<int32_t>(slot >> 32);
      size = static_cast<int32_t>(slot);
    }
    if (!tcheck(a, R, N, pos, size, c.total, &cnt, static_cast<uint64_t>(c.row))) pos = kNullPos;
  }
  const bool valid = pos >= 0;
  *ppos = pos;
  *pm = 0;
  *pcs = 0;
  if (W && !top && N.validity && !(a.skip & 2)) wbit(c, N, n, 0, N.validity, e, valid);
  if (ty == FURY_TYPE_STRING || ty == FURY_TYPE_BINARY) {
    uint32_t* cu = c.sh->cur + (N.k - c.kg0) * static_cast<int>(blockDim.x) + c.tid;
    const uint32_t c0 = *cu;
    *cu = c0 + cnt;
    if (W) {
      const int64_t bp = c.sh->kb[N.k - c.kg0] + c0;
      if (N.offsets && !(a.skip & 8)) wput_off(c, N, n, e, static_cast<int32_t>(bp + cnt));
      if (valid && N.values && !(a.skip & 1)) wput_bytes(c, N, n, bp, pos, cnt);
    }
    return valid;
  }
  if (ty == FURY_TYPE_DECIMAL) {
    if (W && N.values) {
      const uint64_t lo = valid ? rd8(R, pos) : 0, hi = valid ? rd8(R, pos + 8) : 0;
      const int32_t o = N.ek >= 0 ? wwin(c, 0, n) : -1;
      if (o >= 0) {
        const auto d = lds_ptr<uint64_t>(c.sh->opool + o + 16 * (e - c.sh->oe[n]));
        d[0] = lo;
        d[1] = hi;
      } else {
        const auto d = gl(reinterpret_cast<uint64_t*>(N.values + 16 * e));
        d[0] = lo;
        d[1] = hi;
      }
    }
    return valid;
  }
  if (ty == FURY_TYPE_STRUCT) {
    *pm = (W || valid) ? static_cast<uint32_t>(N.num_children) : 0u;
  } else if (ty == FURY_TYPE_LIST || ty == FURY_TYPE_MAP) {
    uint32_t* cu = c.sh->cur + (N.k - c.kg0) * static_cast<int>(blockDim.x) + c.tid;
    const uint32_t c0 = *cu;
    *pm = cnt;
    *cu = c0 + cnt;
    if (W) {
      *pcs = c.sh->kb[N.k - c.kg0] + c0;
      if (N.offsets && !(a.skip & 8)) wput_off(c, N, n, e, static_cast<int32_t>(*pcs + cnt));
    }
  }
  return valid;
}

// Entry e of node n (non-scalar; scalars go through wscalar): slot word `slot` (loaded by the
// caller together with the null bit: one round trip) in a container that starts at cont (vpos >=
// 0: the value is AT vpos -- a collection batch's top-level entry).
// Returns whether the value is valid.  Top-level callers (D == 0) set the validity themselves.
// Every child item -- a STRUCT's fields, a LIST's elements, a MAP's keys then values -- goes
// through ONE loop with one call of the next level, so the levels inline into straight code (no
// call frames: a recursive call per level would keep every register of the walk live in scratch).
template <int D, bool W, int MD>
__device__ __forceinline__ bool wvalue(const WCtx& c, int n, int64_t e, bool nul, uint64_t slot,
                                       int64_t cont, int64_t vpos) {
  if constexpr (D >= MD) {
    return false;
  } else {
    n = __builtin_amdgcn_readfirstlane(n);      // every active lane is at the same node
    const TreeArgs& a = *c.a;
    const Rows& R = *c.R;
    CTNode& N = tn(a, n);
    const int ty = N.type;
    int64_t pos;
    uint32_t m;
    int64_t cs;
    const bool valid = wentry<W>(c, N, n, e, nul, slot, cont, vpos, D == 0, &pos, &m, &cs);
    const bool strc = ty == FURY_TYPE_STRUCT;
    if (!strc && ty != FURY_TYPE_LIST && ty != FURY_TYPE_MAP) return valid;
    if (!wcharge<W>(c, ty, valid, m)) m = 0;
    const int64_t hb = tbm(strc ? N.num_children : static_cast<int64_t>(m));
    const int sides = ty == FURY_TYPE_MAP ? 2 : 1;
    for (int sd = 0; sd < sides; sd++) {
      int64_t arr = pos;                          // LIST / MAP side: the BinaryArray
      if (ty == FURY_TYPE_MAP && m > 0)
        arr = sd == 0 ? pos + 8 : pos + 8 + static_cast<int32_t>(rd8(R, pos));
      if (!strc) {
        CTNode& C = tn(a, N.first_child + sd);
        if (!W && !C.walk) continue;              // nothing to count below
        if (W && C.width > 0) {                   // fixed-width elements: batched bits
          welems(c, C, N.first_child + sd, cs, arr, hb, m);
          continue;
        }
      }
      for (uint32_t j = 0; j < m; j++) {
        const int cn = strc ? N.first_child + static_cast<int>(j) : N.first_child + sd;
        CTNode& C = tn(a, __builtin_amdgcn_readfirstlane(cn));
        const int64_t ce = strc ? e : cs + static_cast<int64_t>(j);
        const int64_t cbm = strc ? pos : arr + 8;
        const int64_t cslot = strc ? pos + hb + 8 * static_cast<int64_t>(j)
                                   : arr + 8 + hb + static_cast<int64_t>(C.esize) * j;
        const int64_t ccont = strc ? pos : arr;
        const int crw = strc ? C.width : C.esize;
        const bool scal = C.width > 0;
        if (scal ? !W : !(W || C.walk)) continue;
        // the null bit and the slot / value together (inside the checked container: a struct's
        // fields only when it is valid, a list's elements only exist then)
        const bool can = !strc || valid;
        uint32_t nb = 1;
        uint64_t sv = 0;
        if (can) {
          nb = rd1(R, cbm + (j >> 3)) >> (j & 7);
          sv = scal ? rdw(R, cslot, crw) : rd8(R, cslot);
        }
        const bool cnul = !can || (nb & 1);
        if (scal) wscalar(c, C, cn, ce, cnul, sv);
        else wvalue<D + 1, W, MD>(c, cn, ce, cnul, sv, ccont, kNullPos);
      }
    }
    return valid;
  }
}

// The top level of one row, the group's fields (every thread of the workgroup, live or not:
// ballots).
template <bool W, int MD>
__device__ __forceinline__ void walk_row(const WCtx& c, bool live) {
  const TreeArgs& a = *c.a;
  const Rows& R = *c.R;
  const int64_t base = live ? gl(a.offs)[c.row] : 0;
  const int32_t budget =
      live ? static_cast<int32_t>(min<int64_t>(2 * (gl(a.offs)[c.row + 1] - base) + 64, 1 << 30)) : 0;
  if (!W) c.left = budget;
  if (a.root) {                                  // collection batch: the entry IS the value
    bool valid = false;
    if (live) valid = wvalue<0, W, MD>(c, 0, c.row, false, 0, 0, base);
    CTNode& N = tn(a, 0);
    if (W && N.validity) tballot_or(N.validity, c.wave_row, live && valid);
    return;
  }
  bool rowok = false;
  if (live) {
    rowok = span_ok(base, tbm(a.ntop) + 8 * a.ntop, c.total);
    if (!rowok) raise_oob(a.err, c.row);
  }
  const int64_t hb = tbm(a.ntop);
  for (int f = c.f0; f < c.f1; f++) {
    CTNode& N = tn(a, f);
    if (N.width > 0 ? !W : !(W || N.walk)) continue;
    if (!W) c.left = budget;
    const int64_t slotp = base + hb + 8 * f;
    // the null bit and the slot / value together: one round trip
    uint32_t nb = 1;
    uint64_t sv = 0;
    if (rowok) {
      nb = rd1(R, base + (f >> 3)) >> (f & 7);
      sv = N.width > 0 ? rdw(R, slotp, N.width) : rd8(R, slotp);
    }
    const bool nul = !rowok || (nb & 1);
    if (N.width > 0) {
      if (W) {
        const uint64_t x = (live && !nul) ? sv : 0;
        if (N.type == FURY_TYPE_BOOL) {
          if (N.values) tballot_or(N.values, c.wave_row, live && !nul && (x & 0xff));
        } else if (live && N.values) {
          tstore_w(N.values + c.row * N.width, N.width, x);
        }
        if (N.validity) tballot_or(N.validity, c.wave_row, live && !nul);
      }
      continue;
    }
    bool valid = false;
    if (live) valid = wvalue<0, W, MD>(c, f, c.row, nul, sv, base, kNullPos);
    if (W && N.validity) tballot_or(N.validity, c.wave_row, live && valid);
  }
}

// Diagnostics (tuning "tree_debug"): thread 0 adds the time between marks to acc[id]; the kernel
// adds acc to a.dbg[base + id] at the end (count pass base 0, write pass 16; see tree.hip).
struct WClock {
  uint64_t* acc;            // LDS [16] or NULL
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

// Pass 1: counted-slot totals of each row -> in-tile row prefixes (rowpre) and the tile's entries
// / payload bytes of every node (cnt / byt [node][tile]).  A tile whose slot totals do not fit 32
// bits sets *overflow (the level engine decodes the batch).
template <int NT, int MD>
__global__ __launch_bounds__(NT) void walk_count_kernel(TreeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];
  const WShared sh = walk_shared(wsm, a, NT, false);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int64_t t;
  int g;
  if (!wgroup(a, &t, &g)) return;                // (uniform: a padding block)
  const int kg0 = a.gk[g], kn = a.gk[g + 1] - kg0, f0 = a.gf[g], f1 = a.gf[g + 1];
  const int64_t r0 = t * NT;
  const int64_t nr = min<int64_t>(NT, a.nrows - r0);
  const int64_t total = gl(a.offs)[a.nrows];
  const bool live = tid < nr;
  __shared__ uint64_t tacc[16];
  const WClock clk{a.dbg ? tacc : nullptr};
  clk.start();
  for (int k = 0; k < kn; k++) sh.cur[k * NT + tid] = 0;
  const Rows R = walk_stage<NT>(a, sh.stg, r0, nr, total);
  if (a.prefetch) walk_prefetch(a, sh, r0, tid, total, R.hi);
  __syncthreads();
  clk.mark(0);
  WCtx c{&a, &sh, &R, total, r0 + tid, r0 + (tid & ~63), tid, 0, kg0, f0, f1};
  walk_row<false, MD>(c, live);
  clk.mark(1);
  // in-tile exclusive prefix of every slot of the group over the rows (row = thread)
  uint64_t* wsum = sh.wsum;
  for (int k = 0; k < kn; k++) {
    const uint64_t v = sh.cur[k * NT + tid];
    const uint64_t inc = tw_scan64(v);
    if (lane == 63) wsum[k * (NT / 64) + wave] = inc;
    sh.cur[k * NT + tid] = static_cast<uint32_t>(inc - v);   // wave-exclusive for now
  }
  lds_barrier();   // (LDS only)
  bool over = false;
  for (int k = 0; k < kn; k++) {
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
      const uint64_t s = wsum[k * (NT / 64) + w];
      pre += w < wave ? s : 0;
      tot += s;
    }
    over |= tot >= (1ull << 32);
    if (live) gl(a.rowpre)[static_cast<int64_t>(kg0 + k) * a.nrows + r0 + tid] =
        static_cast<uint32_t>(pre + sh.cur[k * NT + tid]);
    if (tid == 0) sh.kb[k] = static_cast<int64_t>(tot);
  }
  if (over && tid == 0) __hip_atomic_store(a.overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  lds_barrier();   // (LDS only: the rowpre stores need not land first)
  clk.mark(2);
  for (int n = tid; n < a.nn; n += NT) {
    CTNode& N = tn(a, n);
    if (N.top < f0 || N.top >= f1) continue;   // another group's node
    const int64_t ent = N.ek < 0 ? nr : sh.kb[N.ek - kg0];
    const int64_t byt = (N.type == FURY_TYPE_STRING || N.type == FURY_TYPE_BINARY) ? sh.kb[N.k - kg0] : 0;
    a.cnt[n * a.stride + t] = ent;
    a.byt[n * a.stride + t] = byt;
  }
  clk.mark(3);
  clk.flush(a.dbg, 0);
}

// Pass 2: the walk again, writing every output at its final position.
// STG false (no write stage, the default): the reader's window is the literal empty range, so every
// staged-or-HBM branch of the inlined reads folds to the HBM load at compile time (smaller code,
// fewer live scalars).
template <int NT, int MD, bool STG>
__global__ __launch_bounds__(NT) void walk_write_kernel(TreeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];
  const WShared sh = walk_shared(wsm, a, NT, true);
  const int tid = threadIdx.x;
  int64_t t;
  int g;
  if (!wgroup(a, &t, &g)) return;                // (uniform: a padding block)
  const int kg0 = a.gk[g], kn = a.gk[g + 1] - kg0, f0 = a.gf[g], f1 = a.gf[g + 1];
  const int64_t r0 = t * NT;
  const int64_t nr = min<int64_t>(NT, a.nrows - r0);
  const int64_t total = gl(a.offs)[a.nrows];
  const bool live = tid < nr;
  const int nn = a.nn;
  __shared__ uint64_t tacc[16];
  const WClock clk{a.dbg ? tacc : nullptr};
  clk.start();
  // A write tile spans tmul count tiles [tc0, tc1): a row's cursor = its in-count-tile prefix +
  // its count tile's base - the write tile's base (kb).
  const int64_t tc0 = t * a.tmul, tc1 = min<int64_t>(tc0 + a.tmul, a.stride - 1);
  const int64_t tcr = live ? (r0 + tid) / a.ctr : tc0;
  auto slot_base = [&](int k, int64_t tc) -> int64_t {
    const int n = a.knode[k];
    CTNode& N = tn(a, n);
    return (N.type == FURY_TYPE_STRING || N.type == FURY_TYPE_BINARY)
               ? a.byt[n * a.stride + tc] : a.cnt[N.first_child * a.stride + tc];
  };
  for (int k = 0; k < kn; k++) {
    uint32_t c = live ? gl(a.rowpre)[static_cast<int64_t>(kg0 + k) * a.nrows + r0 + tid] : 0u;
    if (tcr != tc0) c += static_cast<uint32_t>(slot_base(kg0 + k, tcr) - slot_base(kg0 + k, tc0));
    sh.cur[k * NT + tid] = c;
  }
  for (int k = tid; k < kn; k += NT) sh.kb[k] = slot_base(kg0 + k, tc0);
  // bitmap windows of the group's nodes that are not row-aligned: words covering the tile's entries
  // (another group's nodes get none: its flush must not store their words)
  for (int i = tid; i < 2 * nn; i += NT) {
    const int n = i < nn ? i : i - nn;
    CTNode& N = tn(a, n);
    const bool want = N.ek >= 0 && N.top >= f0 && N.top < f1 &&
                      (i < nn ? N.validity != nullptr
                              : (N.type == FURY_TYPE_BOOL && N.values != nullptr));
    uint32_t words = 0;
    if (want) {
      const int64_t e0 = a.cnt[n * a.stride + tc0], e1 = a.cnt[n * a.stride + tc1];
      if (e1 > e0) words = static_cast<uint32_t>(((e1 - 1) >> 5) - (e0 >> 5) + 1);
      if (i < nn) sh.w0[n] = e0 >> 5;
    }
    sh.req[i] = words;
  }
  if (tid == 0) sh.req[2 * nn] = 0;
  // output windows: the tile's range of each node's values / offsets / payload (wput_*)
  if (a.out_cap) {
    for (int i = tid; i < 3 * nn; i += NT) {
      const int which = i / nn, n = i - which * nn;
      CTNode& N = tn(a, n);
      int64_t bytes = 0;
      const bool grp = N.top >= f0 && N.top < f1;
      const bool mine = N.ek >= 0 && grp;
      if (which == 2) {                          // payload window: row-aligned nodes too
        if (grp && N.values && (N.type == FURY_TYPE_STRING || N.type == FURY_TYPE_BINARY) &&
            !(a.skip & 1)) {
          const int64_t b0 = a.byt[n * a.stride + tc0];
          sh.oe[nn + n] = b0;
          bytes = a.byt[n * a.stride + tc1] - b0;
        }
      } else {
        const int64_t e0 = a.cnt[n * a.stride + tc0], e1 = a.cnt[n * a.stride + tc1];
        if (which == 0) {
          if (mine && N.values && N.type != FURY_TYPE_BOOL &&
              (N.width > 0 || N.type == FURY_TYPE_DECIMAL))
            bytes = (e1 - e0) * (N.width > 0 ? N.width : 16);
        } else {
          sh.oe[n] = e0;
          if (mine && N.offsets) bytes = 4 * (e1 - e0);
        }
      }
      if (bytes > static_cast<int64_t>(a.out_cap)) bytes = 0;     // straight to HBM
      sh.olen[i] = static_cast<uint32_t>(bytes);
      sh.oreq[i] = bytes > 0 ? static_cast<uint32_t>((bytes + 31) & ~int64_t(15)) : 0u;
    }
    if (tid == 0) sh.oreq[3 * nn] = 0;
  }
  Rows R{a.rows, sh.stg, 0, 0, 0};
  if constexpr (STG) R = walk_stage<NT>(a, sh.stg, r0, nr, total);
  if (a.prefetch) walk_prefetch(a, sh, r0, tid, total, STG ? R.hi : int64_t(0));
  __syncthreads();
  block_scan_u32<NT>(sh.req, 2 * nn + 1, sh.wsum);   // (req[2nn] = 0 -> the total)
  if (a.out_cap) {
    block_scan_u32<NT>(sh.oreq, 3 * nn + 1, sh.wsum);
    for (int i = tid; i < 3 * nn; i += NT)
      sh.ow[i] = sh.olen[i] > 0 && sh.oreq[i + 1] <= a.out_cap ? static_cast<int32_t>(sh.oreq[i]) : -1;
  }
  const uint32_t pool_words = a.pool_cap / 4;
  for (int i = tid; i < 2 * nn; i += NT) {
    const uint32_t off = sh.req[i], end = sh.req[i + 1];
    sh.win[i] = (end > off && end <= pool_words) ? static_cast<int32_t>(off) : -1;
  }
  const uint32_t used = min(sh.req[2 * nn], pool_words);
  for (uint32_t i = tid; i < used; i += NT) sh.pool[i] = 0;
  lds_barrier();   // (LDS only)
  clk.mark(0);
  WCtx c{&a, &sh, &R, total, r0 + tid, r0 + (tid & ~63), tid, 0, kg0, f0, f1};
  walk_row<true, MD>(c, live);
  clk.mark(1);
  lds_barrier();   // (LDS only: the walk's column stores need not land before the flush)
  clk.mark(2);
  // flush the windows: whole words; the first and last of each (shared with the neighbouring
  // tiles) by atomic OR
  for (uint32_t i = tid; i < used; i += NT) {
    int lo = 0, hi = 2 * nn;                       // window: the last i0 with req[i0] <= i
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (sh.req[mid] <= i) lo = mid; else hi = mid;
    }
    while (lo + 1 < 2 * nn && sh.req[lo + 1] <= i) lo++;   // skip empty windows
    if (sh.win[lo] < 0) continue;
    const int n = lo < nn ? lo : lo - nn;
    CTNode& N = tn(a, n);
    uint8_t* bits = lo < nn ? N.validity : N.values;
    const uint32_t off = sh.req[lo], end = sh.req[lo + 1];
    const uint32_t v = sh.pool[i];
    auto g = gl(reinterpret_cast<uint32_t*>(bits)) + sh.w0[n] + (i - off);
    if (i == off || i + 1 == end) {
      if (v) __hip_atomic_fetch_or(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      *g = v;
    }
  }
  // output windows -> HBM, a wave per window: the range [E0, E1) / [B0, B1) is this tile's alone
  if (a.out_cap) {
    const int wave = tid >> 6;
    for (int i = wave; i < 3 * nn; i += NT / 64) {
      const int32_t o = sh.ow[i];
      if (o < 0) continue;
      const int which = i / nn, n = i - which * nn;
      CTNode& N = tn(a, n);
      uint8_t* dst = which == 0 ? N.values + sh.oe[n] * (N.width > 0 ? N.width : 16)
                   : which == 1 ? reinterpret_cast<uint8_t*>(N.offsets + sh.oe[n] + 1)
                                : N.values + sh.oe[nn + n];
      wave_store_window(dst, sh.opool + o, sh.olen[i]);
    }
  }
  clk.mark(3);
  clk.flush(a.dbg, 16);
}

}  // namespace

size_t walk_lds(const TreeArgs& a, int nt, bool write) {
  return walk_layout(a.nn, a.Kl, nt, a.stage_cap, a.pool_cap, write, a.prefetch != 0, a.out_cap).end;
}
size_t walk_write_lds(int nn, int K, int nt, uint32_t stage, uint32_t pool, bool prefetch,
                      uint32_t out) {
  return walk_layout(nn, K, nt, stage, pool, true, prefetch, out).end;
}
size_t walk_count_lds(int nn, int K, int nt, uint32_t stage, bool prefetch) {
  return walk_layout(nn, K, nt, stage, 0, false, prefetch, 0).end;
}

int walk_launch(const TreeArgs& a, int nt, bool write, hipStream_t hs) {
  const size_t lds = walk_lds(a, nt, write);
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    // field groups: ceil(tiles / 8) x 8 x groups blocks (wgroup)
    const int64_t blocks = a.ngrp <= 1 ? a.ntiles : (a.ntiles + 7) / 8 * 8 * a.ngrp;
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(nt), lds, hs, a);
  };
  // instances per schema depth (a level of the inlined walk keeps ~30 VGPRs live)
#define FURY_WALK(MD)                                                                        \
  if (a.nlevels <= MD) {                                                                     \
    if (!write) nt == 64 ? go(walk_count_kernel<64, MD>) : nt == 128 ? go(walk_count_kernel<128, MD>) \
                                                      : go(walk_count_kernel<256, MD>);       \
    else if (a.stage_cap)                                                                    \
      nt == 64 ? go(walk_write_kernel<64, MD, true>) : nt == 128 ? go(walk_write_kernel<128, MD, true>) \
                                                  : go(walk_write_kernel<256, MD, true>);     \
    else if (nt == 512) go(walk_write_kernel<512, MD, false>);                               \
    else nt == 64 ? go(walk_write_kernel<64, MD, false>) : nt == 128 ? go(walk_write_kernel<128, MD, false>) \
                                                      : go(walk_write_kernel<256, MD, false>); \
    return check_hip(hipGetLastError(), "walk decode launch");                               \
  }
  FURY_WALK(2)
  FURY_WALK(3)
  FURY_WALK(4)
  FURY_WALK(5)
#undef FURY_WALK
  return set_error(FURY_ERR_UNSUPPORTED, "walk decode: schema deeper than kWalkMaxDepth");
}

}  // namespace fury
