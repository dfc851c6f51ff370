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

#include <atomic>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "tree_dev.h"

namespace fury {

namespace {

// Per-node state of the tile being walked (LDS).
struct TMeta {
  uint32_t ecnt;            // entries of the node in the current (sub-)tile
  uint32_t src;             // arena byte offset of its int64 source array (non-scalar nodes)
  uint32_t cnt;             // arena byte offset of its uint32 count / prefix array (+1 slot)
  uint32_t tot;             // in-tile total of the counts (elements / payload bytes)
  uint32_t pad_;            // scanned count block value at the node's first slot (its base)
  int64_t run_e;            // pass 2: output entry base of the current sub-tile
  int64_t run_b;            // pass 2: payload byte base of the current sub-tile
};

// LDS working set of one workgroup (dynamic shared memory, laid out by tree_lds_head).
struct TShared {
  TNode* D;                 // node records (copied once)
  TMeta* meta;
  uint64_t* wsum;           // block scans of counts
  uint32_t* wtot;           // per-wave totals of the node-layout scans
  int64_t* roffs;           // row offsets of the (sub-)tile
  uint32_t* ex;             // node-layout scans, two levels' worth: [2][4][maxw + 1]
  uint8_t* stg;
  uint8_t* arena;
  uint64_t* tacc;           // diagnostics: 16 phase accumulators (NULL when off)
};

// One walk of rows [s0, s1), every level's (node, entry) pairs spread over the whole workgroup.
// Returns false when the tile's arrays do not fit the arena (uniform).
template <bool kWrite, int NT>
__device__ bool tree_walk(const TreeArgs& a, const TShared& sh, int64_t t, int64_t s0, int64_t s1,
                          int64_t total) {
  const int tid = threadIdx.x;
  const int64_t nr = s1 - s0;
  const TNode* D = sh.D;
  TMeta* meta = sh.meta;
  uint8_t* arena = sh.arena;
  TMARK(sh, 0);
  for (int64_t i = tid; i < nr; i += NT) sh.roffs[i] = gl(a.offs)[s0 + i];
  // ---- stage the rows
  Rows R;
  R.g = a.rows;
  R.stg = sh.stg;
  {
    const int64_t g0 = min<int64_t>(max<int64_t>(gl(a.offs)[s0], 0), total);
    const int64_t g1 = min<int64_t>(max<int64_t>(gl(a.offs)[s1], g0), total);
    // LDS byte 0 = the batch byte whose ADDRESS is the 16-aligned one at or below byte g0
    R.lo_al = g0 - static_cast<int64_t>((reinterpret_cast<uintptr_t>(a.rows) + g0) & 15);
    R.lo = g0;
    R.hi = min<int64_t>(g1, R.lo_al + a.stage_cap);
    if (R.hi > R.lo) tstage<NT>(sh.stg, a.rows + R.lo_al, a.rows + R.hi);
    else R.hi = R.lo;
  }
  uint32_t region_lo = 0, region_hi = 0;        // arena bytes of the previous level's arrays
  for (int L = 0; L < a.nlevels; L++) {
    const int nb = a.level_start[L], ne = a.level_start[L + 1], m = ne - nb;
    // ---- entries of this level's nodes (a thread per node), then their arrays and item lists
    // by block scans over the nodes: SRC bytes, CNT bytes, expansion entries (A), write entries (B)
    for (int j = tid; j < m; j += NT) {
      const TNode& N = D[nb + j];
      uint32_t ec;
      if (L == 0) ec = static_cast<uint32_t>(nr);
      else if (D[N.parent].type == FURY_TYPE_STRUCT) ec = meta[N.parent].ecnt;
      else ec = meta[N.parent].tot;
      meta[nb + j].ecnt = ec;
    }
    TMARK(sh, 1);
    __syncthreads();                             // (also: the stage and row offsets landed)
    uint32_t* ex = sh.ex + (L & 1) * 4 * (a.maxw + 1);
    block_scan_k<NT, 4>(m, [&](int j, int k) -> uint32_t {
      const int t = D[nb + j].type;
      const uint32_t ec = meta[nb + j].ecnt;
      switch (k) {
        case 0: return is_scalar(t) ? 0u : 8 * ec;
        case 1: return is_counted(t) ? 4 * (ec + 1) : 0u;
        case 2: return (kWrite || !is_scalar(t)) ? ec : 0u;
        default: return (kWrite && !is_scalar(t)) ? ec : 0u;
      }
    }, ex, sh.wtot);
    TMARK(sh, 2);
    const uint32_t* cumA = ex + 2 * (m + 1);
    const uint32_t* cumB = ex + 3 * (m + 1);
    const uint32_t srcb = ex[m], cntb = ex[(m + 1) + m];
    const uint32_t need = (srcb + cntb + 15) & ~15u;
    uint32_t at;
    if (need <= region_lo) at = 0;
    else if (region_hi + need <= a.arena_cap) at = region_hi;
    else return false;
    const uint32_t cblk = at + srcb, cend = cblk + cntb;
    for (int j = tid; j < m; j += NT) {
      meta[nb + j].src = at + ex[j];
      meta[nb + j].cnt = cblk + ex[(m + 1) + j];
    }
    region_lo = at;
    region_hi = at + need;
    __syncthreads();
    TMARK(sh, 3);
    // ---- expand: every (node, entry) of the level from the parent level (or the rows)
    {
      const uint32_t W = cumA[m];
      for (uint32_t i0 = 0; i0 < W; i0 += NT) {
        const uint32_t i = i0 + tid;
        const bool live = i < W;
        const int k = titem(cumA, m, live ? i : W - 1);
        const int n = nb + k;
        const uint32_t q = (live ? i : W - 1) - cumA[k];
        const TNode& N = D[n];
        const bool scalar = is_scalar(N.type);
        // (with every lane active: whether the wave's lanes are consecutive entries of one node)
        const bool uni = __all(n == __shfl(n, 0)) != 0;
        const int64_t gi = (kWrite ? meta[n].run_e : 0) + q;
        const int64_t gi0 = __shfl(gi, 0);
        bool nul = true;
        int64_t slotp = 0, cont = 0;
        int64_t vpos = kNullPos;                // collection roots: the value at the row base
        int rw = N.width;                       // bytes of a scalar's value in its slot
        if (live) {
          if (L == 0) {
            const int64_t base = sh.roffs[q];
            if (a.root) {
              nul = false;
              vpos = base;
            } else if (!span_ok(base, tbm(a.ntop) + 8 * a.ntop, total)) {
              if (N.ord == 0) raise_oob(a.err, s0 + q);
            } else {
              nul = rdbit(R, base, N.ord);
              slotp = base + tbm(a.ntop) + 8 * N.ord;
              cont = base;
            }
          } else {
            const TNode& P = D[N.parent];
            const TMeta& pm = meta[N.parent];
            const int64_t* PSRC = reinterpret_cast<const int64_t*>(arena + pm.src);
            if (P.type == FURY_TYPE_STRUCT) {
              const int64_t pb = PSRC[q];
              if (pb >= 0) {
                nul = rdbit(R, pb, N.ord);
                slotp = pb + tbm(P.num_children) + 8 * N.ord;
                cont = pb;
              }
            } else {                            // LIST / MAP element
              const uint32_t* PP = reinterpret_cast<const uint32_t*>(arena + pm.cnt);
              const uint32_t e = towner(PP, pm.ecnt, q + pm.pad_);
              const uint32_t j = q + pm.pad_ - PP[e];
              const int64_t m = PP[e + 1] - PP[e];
              const int64_t pb = PSRC[e];
              int64_t arr = pb;
              if (P.type == FURY_TYPE_MAP)
                arr = N.ord == 0 ? pb + 8 : pb + 8 + static_cast<int32_t>(rd8(R, pb));
              nul = rdbit(R, arr + 8, j);
              slotp = arr + 8 + tbm(m) + static_cast<int64_t>(N.esize) * j;
              cont = arr;
              rw = N.esize;
            }
          }
        }
        if (scalar) {                           // (pass 2 only: pass 1 lists no scalars)
          uint64_t x = 0;
          if (live && !nul) x = rdw(R, slotp, rw);
          if (N.type == FURY_TYPE_BOOL) {
            if (N.values) tbits(N.values, uni, gi0, gi, live && !nul && (x & 0xff));
          } else if (live && N.values) {
            tstore_w(N.values + gi * N.width, N.width, x);
          }
          if (N.validity) tbits(N.validity, uni, gi0, gi, live && !nul);
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
          if (!tcheck(a, R, tn(a, n), pos, size, total, &c, err_where_tile(n, s0))) pos = kNullPos;
        }
        reinterpret_cast<int64_t*>(arena + meta[n].src)[q] = pos;
        if (is_counted(N.type)) {
          uint32_t* CNT = reinterpret_cast<uint32_t*>(arena + meta[n].cnt);
          CNT[q] = c;
          if (q + 1 == meta[n].ecnt) CNT[q + 1] = 0;
        }
      }
      // counted nodes without entries still need their trailing slot
      for (int n = nb + tid; n < ne; n += NT)
        if (is_counted(D[n].type) && meta[n].ecnt == 0)
          reinterpret_cast<uint32_t*>(arena + meta[n].cnt)[0] = 0;
    }
    TMARK(sh, 4);
    __syncthreads();
    TMARK(sh, 5);
    // ---- in-tile prefixes of the level's counts: one scan over the contiguous count block; a
    // node's prefix is relative to its first slot (meta.pad_ = that base, meta.tot = its total)
    if (cend > cblk) {
      uint32_t* blk = reinterpret_cast<uint32_t*>(arena + cblk);
      if (!block_scan_u32<NT>(blk, (cend - cblk) / 4, sh.wsum)) return false;
      for (int n = nb + tid; n < ne; n += NT) {
        if (!is_counted(D[n].type)) continue;
        const uint32_t* P = reinterpret_cast<const uint32_t*>(arena + meta[n].cnt);
        meta[n].pad_ = P[0];
        meta[n].tot = P[meta[n].ecnt] - P[0];
      }
      __syncthreads();
    }
    TMARK(sh, 6);
    // ---- pass 2: the level's non-scalar outputs (pass 1 only needed the counts)
    if (!kWrite) continue;
    {
      const uint32_t W = cumB[m];
      for (uint32_t i0 = 0; i0 < W; i0 += NT) {
        const uint32_t i = i0 + tid;
        const bool live = i < W;
        const int k = titem(cumB, m, live ? i : W - 1);
        const int n = nb + k;
        const uint32_t e = (live ? i : W - 1) - cumB[k];
        const TNode& N = D[n];
        const TMeta& M = meta[n];
        const int64_t pos = live ? reinterpret_cast<const int64_t*>(arena + M.src)[e] : kNullPos;
        const bool valid = pos >= 0;
        const int64_t gi = M.run_e + e;
        const bool uni = __all(n == __shfl(n, 0)) != 0;
        const int64_t gi0 = __shfl(gi, 0);
        if (N.validity) tbits(N.validity, uni, gi0, gi, live && valid);
        if (!live) continue;
        const uint32_t* P = is_counted(N.type) ? reinterpret_cast<const uint32_t*>(arena + M.cnt) : nullptr;
        switch (N.type) {
          case FURY_TYPE_STRING:
          case FURY_TYPE_BINARY: {
            const uint32_t p0 = P[e] - M.pad_, p1 = P[e + 1] - M.pad_;
            if (N.offsets) {
              gl(N.offsets)[gi + 1] = static_cast<int32_t>(M.run_b + p1);
              if (gi == 0) gl(N.offsets)[0] = 0;
            }
            if (valid && N.values) tcopy_out(N.values + M.run_b + p0, R, pos, p1 - p0);
            break;
          }
          case FURY_TYPE_LIST:
          case FURY_TYPE_MAP:
            if (N.offsets) {
              gl(N.offsets)[gi + 1] = static_cast<int32_t>(meta[N.first_child].run_e + P[e + 1] - M.pad_);
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
    TMARK(sh, 7);
  }
  return true;
}

// Dynamic LDS of tree_dec_kernel: [node records][meta][wsum 64][row offsets][level lists][stage]
// [arena].
__host__ __device__ inline size_t tree_lds_head(int nn, int maxw, int nt) {
  size_t b = sizeof(TNode) * nn;
  b += sizeof(TMeta) * nn;
  b += 8 * 16 + 4 * 4 * 16;                      // wsum, wtot (up to 16 waves)
  b += 8 * static_cast<size_t>(nt);             // roffs
  b += 4 * 2 * 4 * static_cast<size_t>(maxw + 1);  // ex
  b += 128;                                      // diagnostics
  return (b + 15) & ~size_t(15);
}

template <bool kWrite, int NT>
__global__ __launch_bounds__(NT) void tree_dec_kernel(TreeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tsm[];
  TShared sh;
  {
    uint8_t* p = tsm;
    sh.D = reinterpret_cast<TNode*>(p);
    p += sizeof(TNode) * a.nn;
    sh.meta = reinterpret_cast<TMeta*>(p);
    p += sizeof(TMeta) * a.nn;
    sh.wsum = reinterpret_cast<uint64_t*>(p);
    p += 8 * 16;
    sh.wtot = reinterpret_cast<uint32_t*>(p);
    p += 4 * 4 * 16;
    sh.roffs = reinterpret_cast<int64_t*>(p);
    p += 8 * NT;
    sh.ex = reinterpret_cast<uint32_t*>(p);
    p += 4 * 2 * 4 * (a.maxw + 1);
    sh.tacc = a.dbg ? reinterpret_cast<uint64_t*>(p) : nullptr;
    sh.stg = tsm + tree_lds_head(a.nn, a.maxw, NT);
    sh.arena = sh.stg + a.stage_cap;
  }
  TMeta* meta = sh.meta;
  const int tid = threadIdx.x;
  const int64_t t = blockIdx.x;
  const int64_t r0 = t * a.tile_rows, r1 = min<int64_t>(r0 + a.tile_rows, a.nrows);
  const int64_t total = gl(a.offs)[a.nrows];
  if (sh.tacc && tid < 16) sh.tacc[tid] = tid == 15 ? __builtin_amdgcn_s_memrealtime() : 0;
  for (int n = tid; n < a.nn; n += NT) {
    sh.D[n] = a.nodes[n];
    meta[n].run_e = kWrite ? a.cnt[static_cast<int64_t>(n) * a.ntiles + t] : 0;
    meta[n].run_b = kWrite ? a.byt[static_cast<int64_t>(n) * a.ntiles + t] : 0;
  }
  __syncthreads();
  int64_t s0 = r0, sub = r1 - r0;
  while (s0 < r1) {
    const int64_t s1 = min(s0 + sub, r1);
    if (!tree_walk<kWrite, NT>(a, sh, t, s0, s1, total)) {
      TMARK(sh, 9);
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
    for (int n = tid; n < a.nn; n += NT) {
      meta[n].run_e += meta[n].ecnt;
      const int ty = sh.D[n].type;
      if (ty == FURY_TYPE_STRING || ty == FURY_TYPE_BINARY) meta[n].run_b += meta[n].tot;
    }
    __syncthreads();
    s0 = s1;
  }
  if (!kWrite)
    for (int n = tid; n < a.nn; n += NT) {
      a.cnt[static_cast<int64_t>(n) * a.ntiles + t] = meta[n].run_e;
      a.byt[static_cast<int64_t>(n) * a.ntiles + t] = meta[n].run_b;
    }
  TMARK(sh, 8);
  if (sh.tacc && tid < 15) atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg) + (kWrite ? 16 : 0) + tid,
                                     static_cast<unsigned long long>(sh.tacc[tid]));
  if (sh.tacc && tid == 15) atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg) + 64 + (kWrite ? 1 : 0), 1ull);
}

// Exclusive scan over the tiles of each [node] row of cnt (rows 0..nn-1) and byt (rows nn..2nn-1),
// rows `stride` apart; tot[row] = the row's total.  One 1024-thread workgroup per row.
constexpr int kScanT = 1024;
__global__ __launch_bounds__(kScanT) void tree_tile_scan(int64_t* cnt, int64_t* byt, int64_t ntiles,
                                                         int64_t stride, int32_t nn, int64_t* tot) {
  __shared__ int64_t ws[kScanT / 64];
  const int row = blockIdx.x;
  int64_t* v = row < nn ? cnt + static_cast<int64_t>(row) * stride : byt + static_cast<int64_t>(row - nn) * stride;
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
  if (tid == 0) {
    tot[row] = all;
    if (stride > ntiles) v[ntiles] = all;       // walk plans: [ntiles] = the total
  }
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

std::atomic<int> g_tree_mode = 2;             // tuning "nested_decode": 0 tree tiles, 1 level engine, 2 row walk
// Row-walk defaults from scripts/ab_generic.py legs at 4M depth-3 rows: 128-row count tiles with
// a 12 KB stage (prepare 1.35 -> 1.08 ms: more tiles resident), 256-row write tiles (1.87 -> 1.78
// ms) with the prefetch.
std::atomic<int> g_walk_threads = 128;        // tuning "walk_threads": rows (= threads) per count tile
std::atomic<int> g_walk_threads_w = 256;      // tuning "walk_threads_write": rows per write tile (a multiple)
std::atomic<uint32_t> g_walk_stage = 12 * 1024;  // tuning "walk_stage": LDS stage cap of a row-walk count tile
std::atomic<uint32_t> g_walk_stage_w = 0;        // tuning "walk_stage_write": the same for the write pass (its
                                    // LDS-bound occupancy costs more than HBM row reads save)
std::atomic<uint32_t> g_walk_pool = 8 * 1024;    // tuning "walk_pool": LDS bitmap-window bytes (write pass)
std::atomic<uint32_t> g_walk_out{16 * 1024};     // tuning "walk_out": LDS output-window bytes (write pass)
std::atomic<int> g_walk_prefetch = 1;            // tuning "walk_prefetch": waves pull their rows into L2 first
                                    // (bit 0: write pass, bit 1: count pass)
std::atomic<int> g_walk_skip = 0;                // tuning "walk_skip": diagnostics (TreeArgs.skip)
uint64_t* g_tree_dbg = nullptr;  // tuning "tree_debug": phase accumulators (device, 80 words)
std::atomic<uint32_t> g_tree_stage{32 * 1024}, g_tree_arena{24 * 1024};
std::atomic<int> g_tree_threads = 256;        // tuning "tree_threads": workgroup size of the decode (256/512/1024)

}  // namespace

void set_tree_mode(int v) { g_tree_mode = v; }
uint64_t* tree_debug_buffer() { return g_tree_dbg; }
int set_tree_debug(int on) {
  if (on && !g_tree_dbg) {
    if (hipMalloc(reinterpret_cast<void**>(&g_tree_dbg), 8 * 80) != hipSuccess) return FURY_ERR_DEVICE;
    if (hipMemset(g_tree_dbg, 0, 8 * 80) != hipSuccess) return FURY_ERR_DEVICE;
  } else if (!on && g_tree_dbg) {
    (void)hipFree(g_tree_dbg);
    g_tree_dbg = nullptr;
  }
  return FURY_OK;
}
int tree_mode() { return g_tree_mode; }
void set_tree_lds(uint32_t stage, uint32_t arena) {
  if (stage) g_tree_stage = (stage + 15) & ~15u;
  if (arena) g_tree_arena = (arena + 15) & ~15u;
}
uint32_t tree_lds(int which) { return which ? g_tree_arena : g_tree_stage; }
void set_tree_threads(int v) { g_tree_threads = v; }
int tree_threads() { return g_tree_threads; }
void set_walk_tuning(int which, uint32_t v) {
  if (which == 0) g_walk_threads = static_cast<int>(v);
  else if (which == 1) g_walk_stage = (v + 15) & ~15u;
  else if (which == 2) g_walk_pool = (v + 15) & ~15u;
  else if (which == 3) g_walk_stage_w = (v + 15) & ~15u;
  else if (which == 4) g_walk_prefetch = static_cast<int>(v);
  else if (which == 5) g_walk_skip = static_cast<int>(v);
  else if (which == 7) g_walk_out = (v + 15) & ~15u;
  else g_walk_threads_w = static_cast<int>(v);
}
uint32_t walk_tuning(int which) {
  return which == 0 ? static_cast<uint32_t>(g_walk_threads) : which == 1 ? g_walk_stage.load()
         : which == 2 ? g_walk_pool.load() : which == 3 ? g_walk_stage_w.load()
         : which == 4 ? static_cast<uint32_t>(g_walk_prefetch)
         : which == 5 ? static_cast<uint32_t>(g_walk_skip)
         : which == 7 ? g_walk_out.load() : static_cast<uint32_t>(g_walk_threads_w);
}

struct TreePlan {
  std::vector<TNode> nodes;
  std::vector<int32_t> level_start;
  int64_t nrows = 0, ntiles = 0;
  int32_t tile_rows = 0, ntop = 0, root = 0;
  uint32_t stage_cap = 0, arena_cap = 0;
  int64_t* cnt = nullptr;          // scanned [nn][stride] bases (device, plan-owned)
  int64_t* byt = nullptr;
  hipStream_t stream = nullptr;
  // row walk (walk.hip)
  bool walk = false;
  int64_t stride = 0;              // ntiles (tree tiles) / ntiles + 1 (row walk)
  uint32_t* rowpre = nullptr;      // [K][nrows]
  int32_t K = 0, nt = 0, ntw = 0;   // count / write tile rows
  uint32_t pool_cap = 0;
  int32_t knode[kWalkMaxK] = {};
};

void tree_free(TreePlan* p) {
  if (!p) return;
  dev_free(p->cnt, p->stream);
  dev_free(p->byt, p->stream);
  dev_free(p->rowpre, p->stream);
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
  if (const int e = device_error_word(hs, &a.err)) return e;
  a.overflow = overflow;
  a.nn = static_cast<int32_t>(p.nodes.size());
  a.ntop = p.ntop;
  a.root = p.root;
  a.nlevels = static_cast<int32_t>(p.level_start.size()) - 1;
  a.tile_rows = p.tile_rows;
  a.stage_cap = p.stage_cap;
  a.arena_cap = p.arena_cap;
  a.dbg = tree_debug_buffer();
  a.stride = p.stride;
  if (p.walk) {
    if (write) a.stage_cap = p.arena_cap;        // walk plans: the write pass's stage cap
    a.prefetch = (g_walk_prefetch >> (write ? 0 : 1)) & 1;
    a.skip = write ? g_walk_skip.load() : 0;
    a.rowpre = p.rowpre;
    a.K = p.K;
    a.pool_cap = p.pool_cap;
    a.out_cap = write ? g_walk_out.load() : 0;
    for (int k = 0; k < p.K; k++) a.knode[k] = p.knode[k];
    a.ctr = p.nt;
    a.tmul = write ? p.ntw / p.nt : 1;
    if (write) a.ntiles = (p.nrows + p.ntw - 1) / p.ntw;
    return walk_launch(a, write ? p.ntw : p.nt, write, hs);
  }
  for (int i = 0; i <= a.nlevels; i++) a.level_start[i] = p.level_start[i];
  int maxw = 0;
  for (int i = 0; i < a.nlevels; i++) maxw = std::max(maxw, p.level_start[i + 1] - p.level_start[i]);
  a.maxw = maxw;
  const int nt = g_tree_threads;
  const size_t lds = tree_lds_head(a.nn, maxw, nt) + p.stage_cap + p.arena_cap;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(p.ntiles)), dim3(nt), lds, hs, a);
  };
  if (nt == 1024) write ? go(tree_dec_kernel<true, 1024>) : go(tree_dec_kernel<false, 1024>);
  else if (nt == 512) write ? go(tree_dec_kernel<true, 512>) : go(tree_dec_kernel<false, 512>);
  else write ? go(tree_dec_kernel<true, 256>) : go(tree_dec_kernel<false, 256>);
  return check_hip(hipGetLastError(), "tree decode launch");
}

}  // namespace

// Pass 1 + tile scan + the one host sync.  *out stays NULL (FURY_OK) when the batch needs the
// level engine: schema beyond the tree tables, or a row whose arrays do not fit the arena.
int tree_prepare(const fury_schema* s, const uint8_t* rows, const int64_t* offs, int64_t nrows,
                 hipStream_t hs, TreePlan** out, std::vector<int64_t>* totals) {
  *out = nullptr;
  const int nn = static_cast<int>(s->nodes.size());
  if (g_tree_mode == 1 || nn > kTreeMaxNodes || s->depth > kTreeMaxLevels || nrows <= 0)
    return FURY_OK;
  // counted slots (row walk): LIST / MAP elements, STRING / BINARY payload bytes
  int K = 0;
  for (int i = 0; i < nn; i++) {
    const int t = s->nodes[i].type_id;
    if (t == FURY_TYPE_LIST || t == FURY_TYPE_MAP || t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY) K++;
  }
  const bool walk = g_tree_mode == 2;
  if (walk && (K > kWalkMaxK || s->depth > kWalkMaxDepth)) return FURY_OK;   // the level engine
  TreePlan* p = new TreePlan();
  p->walk = walk;
  p->K = K;
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
  {
    int k = 0;
    for (int i = 0; i < nn; i++) {               // breadth-first: a parent before its children
      TNode& n = p->nodes[i];
      const bool counted = n.type == FURY_TYPE_LIST || n.type == FURY_TYPE_MAP ||
                           n.type == FURY_TYPE_STRING || n.type == FURY_TYPE_BINARY;
      n.k = counted ? k++ : -1;
      if (counted) p->knode[n.k] = i;
      if (i < s->num_fields) n.ek = -1;
      for (int j = 0; j < n.num_children; j++)
        p->nodes[n.first_child + j].ek = n.type == FURY_TYPE_STRUCT ? n.ek : n.k;
    }
    for (int i = nn - 1; i >= 0; i--) {          // children first
      TNode& n = p->nodes[i];
      n.walk = n.k >= 0;
      for (int j = 0; j < n.num_children; j++) n.walk |= p->nodes[n.first_child + j].walk;
    }
  }
  const int nlev = nn ? level[nn - 1] + 1 : 0;
  p->level_start.assign(nlev + 1, nn);
  for (int i = nn - 1; i >= 0; i--) p->level_start[level[i]] = i;
  p->level_start[0] = 0;
  for (int L = 1; L <= nlev; L++)               // BFS: levels are contiguous and increasing
    if (p->level_start[L] < p->level_start[L - 1]) p->level_start[L] = p->level_start[L - 1];
  // pinned landing zone of the totals: one per host thread, kept (a hipHostMalloc / hipHostFree
  // pair per call cost more host time than the small kernels)
  static thread_local int64_t* pin = nullptr;
  static thread_local size_t pin_words = 0;
  if (pin_words < static_cast<size_t>(2 * nn + 2)) {
    if (pin) (void)hipHostFree(pin);
    pin = nullptr;
    pin_words = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&pin), 8 * (2 * kTreeMaxNodes + 2), hipHostMallocDefault) != hipSuccess) {
      pin = nullptr;
      delete p;
      return set_error(FURY_ERR_DEVICE, "hipHostMalloc (tree plan)");
    }
    pin_words = 2 * kTreeMaxNodes + 2;
  }
  int st = FURY_OK;
  double avg = 64.0;
  if (!walk) {
    // tile rows from the batch's average row size (one small read; the row walk's tiles are fixed)
    st = check_hip(hipMemcpyAsync(pin, offs + nrows, 8, hipMemcpyDeviceToHost, hs), "hipMemcpyAsync");
    if (!st) st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize");
    if (st) {
      delete p;
      return st;
    }
    const int64_t total = std::max<int64_t>(pin[0], 1);
    avg = std::max(8.0, static_cast<double>(total) / static_cast<double>(nrows));
  }
  // rows per tile: the tile's bytes fill ~90 % of the stage, its level arrays (~1.5 x the row
  // bytes at worst: 12 B per non-scalar entry, each behind an 8-byte slot) the arena
  if (walk) {
    // a thread per row; the stage holds the tile's rows up to walk_stage bytes (the rest are read
    // from HBM), the bitmap-window pool walk_pool bytes
    p->nt = g_walk_threads;
    const int tw = g_walk_threads_w.load();
    p->ntw = tw % p->nt == 0 && tw >= p->nt ? tw : p->nt;
    p->tile_rows = p->nt;
    p->stage_cap = (g_walk_stage + 15) & ~15u;
    p->arena_cap = (g_walk_stage_w + 15) & ~15u;
    p->pool_cap = g_walk_pool;
  } else {
    const double by_stage = 0.9 * p->stage_cap / avg, by_arena = 0.9 * p->arena_cap / (0.75 * avg);
    p->tile_rows = static_cast<int32_t>(std::clamp<double>(std::min(by_stage, by_arena), 1.0, 256.0));
  }
  p->ntiles = (nrows + p->tile_rows - 1) / p->tile_rows;
  p->stride = walk ? p->ntiles + 1 : p->ntiles;
  int32_t* overflow = nullptr;
  int64_t* tot = nullptr;
  DeviceTable dt;
  if (!st) st = dev_alloc(8 * nn * p->stride, hs, reinterpret_cast<void**>(&p->cnt));
  if (!st) st = dev_alloc(8 * nn * p->stride, hs, reinterpret_cast<void**>(&p->byt));
  if (!st && walk && K > 0)
    st = dev_alloc(4 * static_cast<size_t>(K) * nrows, hs, reinterpret_cast<void**>(&p->rowpre));
  if (!st) st = dev_alloc(8 * (2 * nn + 2), hs, reinterpret_cast<void**>(&tot));
  if (!st) {
    overflow = reinterpret_cast<int32_t*>(tot + 2 * nn);
    st = check_hip(hipMemsetAsync(overflow, 0, 8, hs), "hipMemsetAsync");
  }
  if (!st) st = upload_table(p->nodes.data(), p->nodes.size() * sizeof(TNode), hs, &dt);
  if (!st) st = tree_launch(*p, false, static_cast<const TNode*>(dt.dev), rows, offs, overflow, hs);
  if (!st) {
    hipLaunchKernelGGL(tree_tile_scan, dim3(static_cast<unsigned>(2 * nn)), dim3(kScanT), 0, hs,
                       p->cnt, p->byt, p->ntiles, p->stride, nn, tot);
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

// Diagnostics, not part of include/fury_row.h: copies the tree-tile phase accumulators (80 words:
// decode pass 1 [0, 16), pass 2 [16, 32), measure [32, 48), encode [48, 64) in 10 ns ticks, then
// workgroup counts [64, 68)) to out and zeroes them.  Synchronises the device.
extern "C" int fury_internal_tree_debug(int64_t* out, int32_t n) {
  uint64_t* d = fury::tree_debug_buffer();
  if (!d || !out || n < 1) return FURY_ERR_INVALID_ARGUMENT;
  if (hipDeviceSynchronize() != hipSuccess) return FURY_ERR_DEVICE;
  if (hipMemcpy(out, d, 8 * std::min(n, 80), hipMemcpyDeviceToHost) != hipSuccess) return FURY_ERR_DEVICE;
  return hipMemset(d, 0, 8 * 80) == hipSuccess ? FURY_OK : FURY_ERR_DEVICE;
}
