// tree.hip — the plan of the nested decode (fury_decode_prepare / fury_decode_execute): the row
// walk (walk.hip) for schemas of up to kWalkMaxDepth levels and kWalkMaxK counted nodes, the
// level-by-level engine (levels.hip) beyond them.  Round 5 removed the tile-level walk ("tree
// tiles") that lived here: one nested decode engine plus the level engine for depth
// (VERDICT r4 item 7).
//
// Reference semantics (FMT = java/fury-format/src/main/java/org/apache/fury/format): the getters
// of BinaryRow / BinaryArray / BinaryMap (FMT/row/binary/UnsafeTrait.java:68-197,
// BinaryArray.java:69-78, BinaryMap.java:62-77) as the generated fromRow and ArrowWriter walk
// them (FMT/encoder/BaseBinaryEncoderBuilder.java:459-706, FMT/vectorized/ArrowWriter.java:
// 205-640): entries of a node in (parent entry, element) order, a null struct gives a null entry
// in every child (StructWriter.appendNull :577-584), a null list / map a zero-length entry, null
// values zeroed; every read bounds-checked against the batch (MemoryBuffer, span_ok in kernels.h).
//
// The plan: pass 1 (walk_count_kernel) counts every node's entries / payload bytes per tile,
// tree_tile_scan turns them into each tile's output bases and the node totals the caller sizes
// its buffers from (the only host sync); pass 2 (walk_write_kernel) writes every output.
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

// Exclusive scan over the tiles of each [node] row of cnt (rows 0..nn-1) and byt (rows nn..2nn-1),
// rows `stride` apart; tot[row] = the row's total.  One 1024-thread workgroup per row walks it in
// chunks of 8192 tiles: a coalesced load into LDS, each thread's 8 consecutive entries scanned
// there, a block scan of the thread sums, a coalesced store.  (Per-thread contiguous runs read
// straight from HBM touched one line per lane per load: 72 us at 31k tiles x 40 rows.)
constexpr int kScanT = 1024;
constexpr int kScanPer = 8;
__global__ __launch_bounds__(kScanT) void tree_tile_scan(int64_t* cnt, int64_t* byt, int64_t ntiles,
                                                         int64_t stride, int32_t nn, int64_t* tot) {
  __shared__ int64_t buf[kScanT * kScanPer];
  __shared__ int64_t ws[kScanT / 64];
  const int row = blockIdx.x;
  int64_t* v = row < nn ? cnt + static_cast<int64_t>(row) * stride : byt + static_cast<int64_t>(row - nn) * stride;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int64_t carry = 0;
  for (int64_t c0 = 0; c0 < ntiles; c0 += kScanT * kScanPer) {
    const int64_t len = min<int64_t>(ntiles - c0, kScanT * kScanPer);
#pragma unroll
    for (int j = 0; j < kScanPer; j++) {
      const int64_t i = j * kScanT + tid;
      buf[i] = i < len ? v[c0 + i] : 0;
    }
    __syncthreads();
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanPer; j++) s += buf[tid * kScanPer + j];
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
    int64_t run = carry + pre + x - s;
#pragma unroll
    for (int j = 0; j < kScanPer; j++) {
      const int64_t c = buf[tid * kScanPer + j];
      buf[tid * kScanPer + j] = run;
      run += c;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kScanPer; j++) {
      const int64_t i = j * kScanT + tid;
      if (i < len) v[c0 + i] = buf[i];
    }
    carry += all;
    __syncthreads();                             // buf / ws are reused by the next chunk
  }
  if (tid == 0) {
    tot[row] = carry;
    if (stride > ntiles) v[ntiles] = carry;     // walk plans: [ntiles] = the total
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

// tuning "nested_decode": 1 level engine; 2 row walk, the level engine past its limits (default);
// 3 row walk, tile BFS (bfs.hip) past its limits; 4 tile BFS always (A/B, tests).  The BFS falls
// back to the walk / level engine for a batch whose tiles overflow its arena.  Measured round 6
// (profiles/r06_*): at depth 3 the walk decodes 4M rows in 2.53 ms, the BFS in 3.06 ms
// at best (its per-level chains of LDS round trips run at ~2 waves per SIMD, bounded by the LDS
// its staged tiles take); past the walk's limits the level engine beat the BFS too (depth 6-20,
// 128 counted nodes), so the BFS is not the default anywhere.
std::atomic<int> g_tree_mode = 2;
// Tile BFS defaults (tunings "bfs_threads", "bfs_rows", "bfs_stage" (0: sized from the batch's
// average row), "bfs_arena" (0: 60 % of the stage + 2 KB)).
std::atomic<int> g_bfs_threads = 128;
std::atomic<int> g_bfs_rows = 128;
std::atomic<uint32_t> g_bfs_stage{0};
std::atomic<uint32_t> g_bfs_arena{0};
std::atomic<int64_t> g_bfs_fallbacks{0};      // batches whose tiles overflowed the arena
// Row-walk defaults from scripts/ab_generic.py legs at 4M depth-3 rows: 128-row count tiles with
// a 12 KB stage (prepare 1.35 -> 1.08 ms: more tiles resident), 256-row write tiles (1.87 -> 1.78
// ms) with the prefetch; round 5: 512-row unstaged write tiles with 24 KB output windows (1.67 ->
// 1.62 ms: the tile prologue -- bases, window layout -- is ~16 % of a 256-row tile's time), then
// 40 KB windows (the same time, WRITE 1.34x -> 1.23x the column bytes).
std::atomic<int> g_walk_threads = 128;        // tuning "walk_threads": rows (= threads) per count tile
std::atomic<int> g_walk_threads_w = 512;      // tuning "walk_threads_write": rows per write tile (a multiple)
std::atomic<uint32_t> g_walk_stage = 12 * 1024;  // tuning "walk_stage": LDS stage cap of a row-walk count tile
std::atomic<uint32_t> g_walk_stage_w = 0;        // tuning "walk_stage_write": the same for the write pass (its
                                    // LDS-bound occupancy costs more than HBM row reads save)
std::atomic<uint32_t> g_walk_pool = 8 * 1024;    // tuning "walk_pool": LDS bitmap-window bytes (write pass)
std::atomic<uint32_t> g_walk_out{40 * 1024};     // tuning "walk_out": LDS output-window bytes (write pass)
std::atomic<int> g_walk_prefetch = 1;            // tuning "walk_prefetch": waves pull their rows into L2 first
                                    // (bit 0: write pass, bit 1: count pass)
std::atomic<int> g_walk_skip = 0;                // tuning "walk_skip": diagnostics (TreeArgs.skip)
// Field groups (round 6): a schema with more than "walk_group_min" counted slots walks its
// top-level fields in groups of about "walk_group_k" slots, a workgroup per (tile, group): the LDS
// cursors (4 B x slots x rows) of a 128-slot bean held one 64-row count tile per ~5 waves of a CU.
// 1M beans of 128 / 200 counted nodes (scripts/r06_group2.sh): one group 22.5 / 39.0 ms, groups
// of 16 / 8 / 4 / 2 slots 9.7 / 7.2 / 6.8 / 6.9 and 13.8 / 10.2 / 10.2 / 10.2 ms, the level engine
// 16.5 / 25.7 ms.  The depth-3 schema (9 slots) in groups of 4 / 2 / 1: 2.64 / 2.99 / 3.25 vs
// 2.53 ms -- at <= 16 slots the cursors do not limit the tiles per CU, so it stays one group.
// With the payload windows (late round 6, profiles/r06_walk_group_size_payload_windows.jsonl)
// groups of 8 took over: 128 counted nodes 6.52 vs 6.89 ms (4), flat id + 126 STRING fields 5.83
// vs 6.14; 200 counted nodes 9.47 (4 doubles to 8 there: at most 32 groups).
std::atomic<int> g_walk_group_k = 8;     // tuning "walk_group_k" (0 = one group)
std::atomic<int> g_walk_group_min = 16;  // tuning "walk_group_min"
uint64_t* g_tree_dbg = nullptr;  // tuning "tree_debug": phase accumulators (device, 80 words)

}  // namespace

void set_tree_mode(int v) { g_tree_mode = v; }
void set_bfs_tuning(int which, uint32_t v) {
  if (which == 0) g_bfs_threads = static_cast<int>(v);
  else if (which == 1) g_bfs_rows = static_cast<int>(v);
  else if (which == 2) g_bfs_stage = (v + 15) & ~15u;
  else g_bfs_arena = (v + 15) & ~15u;
}
int64_t bfs_tuning(int which) {
  return which == 0 ? g_bfs_threads.load() : which == 1 ? g_bfs_rows.load()
         : which == 2 ? static_cast<int64_t>(g_bfs_stage.load())
         : which == 3 ? static_cast<int64_t>(g_bfs_arena.load()) : g_bfs_fallbacks.load();
}
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
void set_walk_tuning(int which, uint32_t v) {
  if (which == 0) g_walk_threads = static_cast<int>(v);
  else if (which == 1) g_walk_stage = (v + 15) & ~15u;
  else if (which == 2) g_walk_pool = (v + 15) & ~15u;
  else if (which == 3) g_walk_stage_w = (v + 15) & ~15u;
  else if (which == 4) g_walk_prefetch = static_cast<int>(v);
  else if (which == 5) g_walk_skip = static_cast<int>(v);
  else if (which == 7) g_walk_out = (v + 15) & ~15u;
  else if (which == 8) g_walk_group_k = static_cast<int>(v);
  else if (which == 9) g_walk_group_min = static_cast<int>(v);
  else g_walk_threads_w = static_cast<int>(v);
}
uint32_t walk_tuning(int which) {
  return which == 0 ? static_cast<uint32_t>(g_walk_threads) : which == 1 ? g_walk_stage.load()
         : which == 2 ? g_walk_pool.load() : which == 3 ? g_walk_stage_w.load()
         : which == 4 ? static_cast<uint32_t>(g_walk_prefetch)
         : which == 5 ? static_cast<uint32_t>(g_walk_skip)
         : which == 7 ? g_walk_out.load()
         : which == 8 ? static_cast<uint32_t>(g_walk_group_k)
         : which == 9 ? static_cast<uint32_t>(g_walk_group_min) : static_cast<uint32_t>(g_walk_threads_w);
}

struct TreePlan {
  std::vector<TNode> nodes;
  int32_t nlevels = 0;
  int64_t nrows = 0, ntiles = 0;
  int32_t tile_rows = 0, ntop = 0, root = 0;
  uint32_t stage_cap = 0, stage_cap_w = 0;     // LDS stage bytes: count / write pass
  int64_t* cnt = nullptr;          // scanned [nn][stride] bases (device, plan-owned)
  int64_t* byt = nullptr;
  hipStream_t stream = nullptr;
  // row walk (walk.hip)
  int64_t stride = 0;              // ntiles + 1: [ntiles] holds the total
  uint32_t* rowpre = nullptr;      // [K][nrows]
  int32_t K = 0, nt = 0, ntw = 0;   // count / write tile rows
  uint32_t pool_cap = 0, out_cap = 0;  // write pass: bitmap-window / output-window LDS bytes
  int32_t knode[kWalkMaxK] = {};
  int32_t ngrp = 1, Kl = 0;           // field groups (TreeArgs)
  int32_t prefetch = 0;               // walk_prefetch bits of this plan
  int32_t gf[kMaxGroups + 1] = {}, gk[kMaxGroups + 1] = {};
  int32_t lvl[kMaxLevels + 1] = {};   // first node of each level
  // tile BFS (bfs.hip)
  bool bfs = false;
  int32_t bnt = 0;                 // threads per tile
  uint32_t arena_cap = 0;
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
  a.nlevels = p.nlevels;
  a.stage_cap = write ? p.stage_cap_w : p.stage_cap;
  a.dbg = tree_debug_buffer();
  a.stride = p.stride;
  a.prefetch = (p.prefetch >> (write ? 0 : 1)) & 1;
  a.skip = write ? g_walk_skip.load() : 0;
  a.rowpre = p.rowpre;
  a.K = p.K;
  a.pool_cap = p.pool_cap;
  a.out_cap = write ? p.out_cap : 0;
  for (int k = 0; k < p.K && k < kWalkMaxK; k++) a.knode[k] = p.knode[k];   // (the walk only)
  a.ngrp = p.ngrp;
  a.Kl = p.Kl;
  for (int g = 0; g <= p.ngrp && g <= kMaxGroups; g++) {
    a.gf[g] = p.gf[g];
    a.gk[g] = p.gk[g];
  }
  a.ctr = p.nt;
  if (p.bfs) {
    for (int L = 0; L <= p.nlevels && L <= kMaxLevels; L++) a.lvl[L] = p.lvl[L];
    a.trows = p.tile_rows;
    a.arena_cap = p.arena_cap;
    a.stage_cap = p.stage_cap;
    a.prefetch = 0;
    return bfs_launch(a, p.bnt, write, hs);
  }
  a.tmul = write ? p.ntw / p.nt : 1;
  if (write) a.ntiles = (p.nrows + p.ntw - 1) / p.ntw;
  return walk_launch(a, write ? p.ntw : p.nt, write, hs);
}

}  // namespace

// Tile BFS prepare: pass 1 + tile scan + the host sync for the totals.  p->bfs stays false (FURY_OK)
// when a tile's records outgrow the arena (the caller falls back to the row walk / level engine).
// The stage is sized from the batch's average row (one more 8-byte read: the batch's bytes).
int bfs_prepare(TreePlan* p, const uint8_t* rows, const int64_t* offs, int64_t nrows,
                hipStream_t hs, int64_t* pin, std::vector<int64_t>* totals) {
  const int nn = static_cast<int>(p->nodes.size());
  int st = check_hip(hipMemcpyAsync(pin + 2 * kTreeMaxNodes + 1, offs + nrows, 8,
                                    hipMemcpyDeviceToHost, hs), "hipMemcpyAsync batch bytes");
  if (!st) st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize");
  if (st) return st;
  const int64_t bytes = std::max<int64_t>(pin[2 * kTreeMaxNodes + 1], 0);
  const int nt = g_bfs_threads.load();
  const double avg = static_cast<double>(bytes) / static_cast<double>(nrows);
  DeviceTable dt;
  st = upload_table(p->nodes.data(), p->nodes.size() * sizeof(TNode), hs, &dt);
  if (st) return st;
  // A tile whose records outgrow the arena is retried with half the rows and a larger arena share
  // (container-heavy rows need ~16 B of records per container entry); after three tries the batch
  // goes to the row walk / level engine.
  for (int attempt = 0; attempt < 3; attempt++) {
    const int trows = std::max(1, g_bfs_rows.load() >> attempt);
    if (attempt > 0 && trows < 16) break;
    uint32_t stage = g_bfs_stage.load();
    if (!stage)
      stage = static_cast<uint32_t>(std::min<double>(std::max<double>(avg * trows * 1.05 + 64, 2048), 64 * 1024));
    stage = (stage + 15) & ~15u;
    uint32_t arena = g_bfs_arena.load();
    if (!arena)
      arena = ((static_cast<uint32_t>((attempt == 0 ? 0.6 : 1.5) * stage) + 2048) + 15) & ~15u;
    while (bfs_lds(nn, nt, stage, arena, trows) > kWalkLdsMax && arena > 1024) arena /= 2;
    while (bfs_lds(nn, nt, stage, arena, trows) > kWalkLdsMax && stage > 1024) stage /= 2;
    p->tile_rows = trows;
    p->bnt = nt;
    p->stage_cap = stage;
    p->arena_cap = arena;
    p->ntiles = (nrows + trows - 1) / trows;
    p->stride = p->ntiles + 1;
    int64_t* tot = nullptr;
    int32_t* overflow = nullptr;
    if (!st) st = dev_alloc(8 * nn * p->stride, hs, reinterpret_cast<void**>(&p->cnt));
    if (!st) st = dev_alloc(8 * nn * p->stride, hs, reinterpret_cast<void**>(&p->byt));
    if (!st) st = dev_alloc(8 * (2 * nn + 2), hs, reinterpret_cast<void**>(&tot));
    if (!st) {
      overflow = reinterpret_cast<int32_t*>(tot + 2 * nn);
      st = check_hip(hipMemsetAsync(overflow, 0, 8, hs), "hipMemsetAsync");
    }
    p->bfs = true;                          // (tree_launch dispatches on it)
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
    if (!st && !over) return FURY_OK;
    p->bfs = false;
    dev_free(p->cnt, hs);
    dev_free(p->byt, hs);
    p->cnt = p->byt = nullptr;
    if (st) return st;
  }
  return FURY_OK;                           // p->bfs false: the caller falls back
}

// Pass 1 + tile scan + the one host sync.  *out stays NULL (FURY_OK) when the batch needs the
// level engine: schema beyond the tree tables, or a row whose arrays do not fit the arena.
int tree_prepare(const fury_schema* s, const uint8_t* rows, const int64_t* offs, int64_t nrows,
                 hipStream_t hs, TreePlan** out, std::vector<int64_t>* totals) {
  *out = nullptr;
  const int nn = static_cast<int>(s->nodes.size());
  if (g_tree_mode == 1 || nn > kTreeMaxNodes || nrows <= 0)
    return FURY_OK;
  // counted slots (row walk): LIST / MAP elements, STRING / BINARY payload bytes
  int K = 0;
  for (int i = 0; i < nn; i++) {
    const int t = s->nodes[i].type_id;
    if (t == FURY_TYPE_LIST || t == FURY_TYPE_MAP || t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY) K++;
  }
  const bool walk_ok = K <= kWalkMaxK && s->depth <= kWalkMaxDepth;
  const bool bfs_ok = !s->root && (g_tree_mode == 4 || (g_tree_mode == 3 && !walk_ok));
  if (!walk_ok && !bfs_ok) return FURY_OK;                          // the level engine
  TreePlan* p = new TreePlan();
  p->K = K;
  p->stream = hs;
  p->nrows = nrows;
  p->ntop = s->num_fields;
  p->root = s->root;
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
    // counted slots numbered subtree by subtree (top-level field order), so that a field group's
    // slots are contiguous
    const int ntop = s->root ? 1 : s->num_fields;
    std::vector<int32_t> kf(std::max(ntop, 1), 0);
    for (int i = 0; i < nn; i++) {               // breadth-first: a parent before its children
      TNode& n = p->nodes[i];
      n.top = i < ntop ? i : p->nodes[n.parent].top;
      const bool counted = n.type == FURY_TYPE_LIST || n.type == FURY_TYPE_MAP ||
                           n.type == FURY_TYPE_STRING || n.type == FURY_TYPE_BINARY;
      if (counted) kf[n.top]++;
    }
    std::vector<int32_t> kn(kf.size() + 1, 0);  // first slot of each subtree
    for (size_t f = 0; f < kf.size(); f++) kn[f + 1] = kn[f] + kf[f];
    // field groups: consecutive top-level fields, about walk_group_k slots each, at most kMaxGroups
    const int gk0 = g_walk_group_k.load();
    p->ngrp = 1;
    p->gf[0] = p->gk[0] = 0;
    if (gk0 > 0 && K > g_walk_group_min.load() && ntop > 1 && !s->root) {
      for (int target = gk0;; target *= 2) {
        int g = 0, acc = 0;
        for (int f = 0; f < ntop && g < kMaxGroups; f++) {
          if (acc > 0 && acc + kf[f] > target) {
            g++;
            if (g >= kMaxGroups) break;
            p->gf[g] = f;
            p->gk[g] = kn[f];
            acc = 0;
          }
          acc += kf[f];
        }
        if (g < kMaxGroups) {
          p->ngrp = g + 1;
          break;
        }
      }
    }
    p->gf[p->ngrp] = ntop;
    p->gk[p->ngrp] = K;
    p->Kl = 0;
    for (int g = 0; g < p->ngrp; g++) p->Kl = std::max(p->Kl, p->gk[g + 1] - p->gk[g]);
    for (int i = 0; i < nn; i++) {               // breadth-first: a parent before its children
      TNode& n = p->nodes[i];
      const bool counted = n.type == FURY_TYPE_LIST || n.type == FURY_TYPE_MAP ||
                           n.type == FURY_TYPE_STRING || n.type == FURY_TYPE_BINARY;
      n.k = counted ? kn[n.top]++ : -1;
      if (counted && n.k < kWalkMaxK) p->knode[n.k] = i;
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
  for (int i = 0; i < nn; i++) p->nlevels = std::max(p->nlevels, level[i] + 1);
  // breadth-first numbering: each level's nodes are contiguous
  for (int L = 0, i = 0; L <= p->nlevels && L <= kMaxLevels; L++) {
    while (i < nn && level[i] < L) i++;
    p->lvl[L] = i;
  }
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
  if (bfs_ok) {
    st = bfs_prepare(p, rows, offs, nrows, hs, pin, totals);
    if (st || p->bfs) {                   // a plan, or an error
      if (st) tree_free(p);
      else *out = p;
      return st;
    }
    g_bfs_fallbacks.fetch_add(1);        // a tile overflowed the arena: the row walk / level engine
    if (!walk_ok) {
      tree_free(p);
      return FURY_OK;
    }
  }
  // a thread per row; the stage holds the tile's rows up to walk_stage bytes (the rest are read
  // from HBM), the bitmap-window pool walk_pool bytes
  p->nt = g_walk_threads;
  // Field groups read only their fields' slots and payloads: the L2 pull of whole rows (per group)
  // and the count stage cost more than they save (1M beans of 128 counted nodes, groups of 4:
  // 9.9 -> 7.1 ms without the pull, 6.9 ms without the stage too; scripts/r06_group2.sh)
  p->prefetch = p->ngrp > 1 ? 0 : g_walk_prefetch.load();
  const uint32_t cstage = p->ngrp > 1 ? 0u : (g_walk_stage + 15) & ~15u;
  // the count pass's per-row counters (4 B x counted nodes x rows) must fit one workgroup too:
  // a bean of ~200+ STRING fields counts on 64-row tiles
  while (p->nt > 64 &&
         walk_count_lds(nn, p->Kl, p->nt, cstage, (p->prefetch & 2) != 0) > kWalkLdsMax)
    p->nt /= 2;
  const int tw = g_walk_threads_w.load();
  p->ntw = tw % p->nt == 0 && tw >= p->nt ? tw : p->nt;
  p->tile_rows = p->nt;
  p->stage_cap = cstage;
  p->stage_cap_w = (g_walk_stage_w + 15) & ~15u;
  if (p->ntw > 256 && p->stage_cap_w) p->ntw = 256;   // 512-row write tiles: unstaged instance only
  p->pool_cap = g_walk_pool;
  p->out_cap = g_walk_out;
  // The write pass's LDS (cursors: K x rows, node tables, windows) must fit one workgroup: wide
  // schemas (many counted nodes / nodes) step down the tile rows, then the windows.
  const bool pfw = (p->prefetch & 1) != 0;
  for (;;) {
    if (walk_write_lds(nn, p->Kl, p->ntw, p->stage_cap_w, p->pool_cap, pfw, p->out_cap) <= kWalkLdsMax) break;
    if (p->ntw > p->nt) p->ntw /= 2;
    else if (p->out_cap > 0) p->out_cap = p->out_cap > 4096 ? p->out_cap / 2 : 0;
    else if (p->pool_cap > 0) p->pool_cap = p->pool_cap > 1024 ? p->pool_cap / 2 : 0;
    else if (p->stage_cap_w > 0) p->stage_cap_w = 0;
    else break;                                 // cannot happen for K <= kWalkMaxK, nn <= 512
  }
  if (walk_write_lds(nn, p->Kl, p->ntw, p->stage_cap_w, p->pool_cap, pfw, p->out_cap) > kWalkLdsMax) {
    tree_free(p);                               // (defensive) the level engine
    return FURY_OK;
  }
  p->ntiles = (nrows + p->tile_rows - 1) / p->tile_rows;
  p->stride = p->ntiles + 1;
  int32_t* overflow = nullptr;
  int64_t* tot = nullptr;
  DeviceTable dt;
  if (!st) st = dev_alloc(8 * nn * p->stride, hs, reinterpret_cast<void**>(&p->cnt));
  if (!st) st = dev_alloc(8 * nn * p->stride, hs, reinterpret_cast<void**>(&p->byt));
  if (!st && K > 0)
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

// Diagnostics, not part of include/fury_row.h: copies the row-walk phase accumulators (80 words:
// count pass [0, 16), write pass [16, 32) in 10 ns ticks, then
// workgroup counts [64, 68)) to out and zeroes them.  Synchronises the device.
extern "C" int fury_internal_tree_debug(int64_t* out, int32_t n) {
  uint64_t* d = fury::tree_debug_buffer();
  if (!d || !out || n < 1) return FURY_ERR_INVALID_ARGUMENT;
  if (hipDeviceSynchronize() != hipSuccess) return FURY_ERR_DEVICE;
  if (hipMemcpy(out, d, 8 * std::min(n, 80), hipMemcpyDeviceToHost) != hipSuccess) return FURY_ERR_DEVICE;
  return hipMemset(d, 0, 8 * 80) == hipSuccess ? FURY_OK : FURY_ERR_DEVICE;
}
