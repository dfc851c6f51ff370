// var.hip — host launchers of the variable-length kernels (schemas with STRING/BINARY, DECIMAL,
// LIST of fixed-width elements) and the kernels other than the register-staged ones; the device
// code is in var_dev.h, the register-staged template instances in var_reg_enc.hip and
// var_reg_dec_{lo,hi}.hip (separate translation units so they compile in parallel).
#define FURY_VAR_MAIN
#include <atomic>
#include "var_dev.h"

#include <algorithm>
#include <cstdlib>

namespace fury {

namespace {
// Column k on the host side of a launch: the argument block, or the host copy of a wide table.
const VarCol& hcol(const VarArgs& a, int k) { return a.htab ? a.htab[k] : a.col[k]; }

int64_t nblocks(int64_t n) { return (n + kThreads - 1) / kThreads; }

}  // namespace

// Device exclusive scan of s[0..n) (int64) with the total written to *total; `ws` needs
// scan_workspace(n) entries.  Hierarchical: levels of 256-entry group scans until one workgroup
// can finish, so no step is a long serial walk.
int64_t scan_workspace(int64_t n) {
  int64_t w = 0;
  while (n > kSmallScan) {
    n = (n + kThreads - 1) / kThreads;
    w += n;
  }
  return w + 1;
}

void device_scan(int64_t* s, int64_t n, int64_t* total, int64_t* ws, hipStream_t stream) {
  if (n <= kSmallScan) {
    hipLaunchKernelGGL(scan_small, dim3(1), dim3(kThreads), 0, stream, s, n, total);
    return;
  }
  const int64_t g = (n + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(scan_groups, dim3(g), dim3(kThreads), 0, stream, s, n, ws);
  device_scan(ws, g, total, ws + g, stream);
  hipLaunchKernelGGL(add_groups, dim3(g), dim3(kThreads), 0, stream, s, n, ws);
}

int launch_measure_rows(const VarArgs& a, int64_t* offs, hipStream_t stream) {
  const int64_t n = a.nrows;
  if (n == 0) return check_hip(hipMemsetAsync(offs, 0, 8, stream), "memset");
  const int64_t nb = (n + kMeasTile - 1) / kMeasTile;
  int64_t* ws = nullptr;          // [group sums x nb][total][scan scratch]
  const int64_t wsn = nb + 1 + scan_workspace(nb);
  int st = dev_alloc(wsn * 8, stream, reinterpret_cast<void**>(&ws));
  if (st) return st;
  hipLaunchKernelGGL(measure_kernel, dim3(nb), dim3(kThreads), 0, stream, a, offs, ws);
  device_scan(ws, nb, ws + nb, ws + nb + 1, stream);
  hipLaunchKernelGGL(add_group_prefix, dim3(nblocks(n)), dim3(kThreads), 0, stream, offs, n, ws,
                     ws + nb);
  st = check_hip(hipGetLastError(), "measure launch");
  dev_free(ws, stream);
  return st;
}

// Look-back spins abandoned so far (each one would have left wrong Arrow offsets behind; never
// observed: workgroups are dispatched in launch order).  Synchronous device read.
int64_t lookback_timeouts() { return device_error_count(); }

// Test hook (tuning "lookback_help"): every look-back computes a silent predecessor's aggregate
// at once -- the path a late-dispatched predecessor takes -- instead of polling first.
static std::atomic<int> g_help_now = 0;
int lookback_help_mode() { return g_help_now; }
void set_lookback_help_mode(int v) { g_help_now = v; }
// Rows per register-staged tile: the estimated tile bytes (row sizes from the input buffers' byte
// counts, as plan_encode_pipe) fit the LDS image with headroom.
int reg_tile_rows(const VarArgs& a) {
  double img_row = a.fixed_size;
  for (int k = 0; k < a.ncols; k++) {
    const VarCol& c = hcol(a, k);
    if (c.kind == kDecimal) img_row += 16;
    if (c.kind != kBytes && c.kind != kListFixed) continue;
    const double per = c.capacity > 0 && a.nrows > 0 ? static_cast<double>(c.capacity) / a.nrows : 32.0;
    img_row += c.kind == kBytes ? per + 7 : 16 + per * (c.width == 0 ? 1 : c.width) + 7;
  }
  for (int R = kEncRows; R > 64; R -= 64)
    if (R * img_row * 1.08 <= kRegImg) return R;
  return 64;
}

// Kind mode of a schema's register-staged instances (kind_of): strings-only, lists-only or all.
int reg_mode(const VarArgs& a) {
  bool bytes = false, lists = false, other = false;
  for (int k = 0; k < a.ncols; k++) {
    const int kd = hcol(a, k).kind;
    bytes |= kd == kBytes;
    lists |= kd == kListFixed;
    other |= kd != kFixed && kd != kBool && kd != kBytes && kd != kListFixed;
  }
  return other || (bytes && lists) ? kSeqAll : lists ? kSeqLists : kSeqBytes;
}

// fury_row_encode_measured for register-staged schemas (<= kRegCols fields): the byte totals of
// the encode's own tiles (measure_tiles, one wave per tile), their exclusive scan, then the encode
// scans each tile's row sizes itself and writes the final row offsets once (the row-sized measure
// wrote and the prefix pass re-read and re-wrote all 8 B/row of them).  -1: not this path.
int launch_encode_measured_var(const VarArgs& a, int64_t* offs, uint8_t* rows, int64_t cap,
                               hipStream_t stream) {
  if (a.ncols > kRegCols || a.nrows <= 0) return -1;
  VarArgs b = a;
  b.tile_rows = reg_tile_rows(a);
  const int64_t nt = (a.nrows + b.tile_rows - 1) / b.tile_rows;
  int64_t* ws = nullptr;          // [tile totals x nt][total][scan scratch]
  int st = dev_alloc((nt + 1 + scan_workspace(nt)) * 8, stream, reinterpret_cast<void**>(&ws));
  if (st) return st;
  st = launch_measure_tiles(b, ws, nt, stream);
  if (!st) {
    device_scan(ws, nt, ws + nt, ws + nt + 1, stream);
    st = launch_encode_var_reg(b, offs, rows, cap, nt, reg_mode(a), ws, stream);
  }
  dev_free(ws, stream);
  return st;
}

int launch_encode_var(const VarArgs& a, const int64_t* offs, uint8_t* rows, int64_t cap,
                      hipStream_t stream) {
  if (a.nrows == 0) return FURY_OK;
  const int64_t nb = (a.nrows + a.tile_rows - 1) / a.tile_rows;
  if (a.ncols <= kRegCols) {
    VarArgs b = a;
    b.tile_rows = reg_tile_rows(a);
    const int64_t nt = (a.nrows + b.tile_rows - 1) / b.tile_rows;
    return launch_encode_var_reg(b, const_cast<int64_t*>(offs), rows, cap, nt, reg_mode(a), nullptr,
                                 stream);
  } else if (var_wide_mode()) {   // 64-row tiles, fields round robin over the waves (wide.hip)
    return launch_encode_wide(a, offs, rows, cap, stream);
  } else if (a.tab) {          // wider than the argument block: column table in device memory
    hipLaunchKernelGGL(encode_var_kernel<MetaMapWide>, dim3(nb), dim3(kEncRows), 0, stream, a,
                       offs, rows, cap);
  } else {
    hipLaunchKernelGGL(encode_var_kernel<MetaMap>, dim3(nb), dim3(kEncRows), 0, stream, a, offs,
                       rows, cap);
  }
  return check_hip(hipGetLastError(), "encode_var launch");
}

// Rows per encode tile so that the staged per-row inputs of a tile fit kMetaPool; at 8 rows even
// kMaxWideVarCols columns of nullable decimals (~176 B of staged pieces each) stay within the
// kEncPool the LDS-DMA kernel stages them in.
int encode_tile_rows(const VarArgs& a) {
  for (int R = kEncRows; R >= 8; R >>= 1) {
    int64_t meta = 0;
    for (int k = 0; k < a.ncols; k++) {
      const VarCol& c = hcol(a, k);
      if (c.validity) meta += R / 8 + 32;
      if (c.kind == kFixed) meta += int64_t(R) * c.width + 32;
      else if (c.kind == kBool) meta += R / 8 + 32;
      else if (c.kind == kDecimal) meta += 16 * int64_t(R) + 32;
      else meta += 4 * int64_t(R + 1) + 32;
    }
    if (meta <= kMetaPool) return R;
  }
  return 8;
}

int launch_decode_measure(const VarArgs& a, const uint8_t* rows, const int64_t* offs,
                          hipStream_t stream) {
  int nseq = 0;
  for (int k = 0; k < a.ncols; k++)
    if (hcol(a, k).kind == kBytes || hcol(a, k).kind == kListFixed) nseq++;
  if (nseq == 0 || a.nrows == 0) return FURY_OK;
  if (a.ncols > kRegCols && var_wide_mode()) return launch_decode_wide(a, rows, offs, stream, true);
  const int64_t nb = nblocks(a.nrows);
  int64_t* ws = nullptr;
  const int64_t scr = scan_workspace(nb);
  int st = dev_alloc((nb * nseq + nseq + scr) * 8, stream, reinterpret_cast<void**>(&ws));
  if (st) return st;
  int64_t* totals = ws + nb * nseq;
  hipLaunchKernelGGL(decode_measure_kernel, dim3(nb), dim3(kThreads), 0, stream, a, rows, offs, ws,
                     nb);
  for (int q = 0; q < nseq; q++) device_scan(ws + q * nb, nb, totals + q, totals + nseq, stream);
  hipLaunchKernelGGL(decode_measure_fix, dim3(nb), dim3(kThreads), 0, stream, a, ws, totals, nb);
  st = check_hip(hipGetLastError(), "decode measure launch");
  dev_free(ws, stream);
  return st;
}

static std::atomic<int> g_dec_rows = 0;
// tuning "var_skip" (diagnostics: phases of encode_var_reg (1 / 2 / 4) and decode_var_reg (16 / 32 /
// 64 / 128) skipped, outputs WRONG; timing only)
static std::atomic<int> g_var_skip{0};
static std::atomic<int> g_var_wide{1};
// threads per 64-row tile of the wide kernels (ab_wide legs, 33 fields x 5M rows): decode 256
// (3.22 vs 3.37 ms at 512), encode 512 (2.20 vs 2.78 ms at 256)
static std::atomic<int> g_wide_threads[2] = {256, 512};
int wide_threads(bool encode) { return g_wide_threads[encode ? 1 : 0].load(); }
void set_wide_threads(bool encode, int v) { g_wide_threads[encode ? 1 : 0] = v; }
int var_wide_mode() { return g_var_wide.load(); }
void set_var_wide_mode(int v) { g_var_wide = v; }
int var_skip() { return g_var_skip.load(); }
void set_var_skip(int v) { g_var_skip = v; }
static std::atomic<int> g_dec_rows_rejected{0};
int var_dec_rows_rejected() { return g_dec_rows_rejected.load(); }
int var_dec_rows() { return g_dec_rows; }
void set_var_dec_rows(int v) { g_dec_rows = v; }
// tuning "var_dec_cover": percent of a tile's estimated row bytes the stage must hold (the rest
// is read from HBM by the rows' threads).  95 (scripts/ab_dec.py legs, interleaved): mixed 10M
// 0.542 -> 0.508 ms (its tiles grow 448 -> 512 rows), C4 4M unchanged (0.229 ms); 80 or less slows C4.
static std::atomic<int> g_dec_cover = 95;
// tuning "var_dec_pipe" (round 6): 0 one tile per workgroup; 1 persistent
// workgroups with two row stages of the planned size (fewer workgroups per CU); 2 the same with
// the planned LDS split into images + two half stages (the tile rows shrink to fit)
static std::atomic<int> g_dec_pipe = 0;
int var_dec_pipe() { return g_dec_pipe; }
void set_var_dec_pipe(int v) { g_dec_pipe = v; }
int var_dec_cover() { return g_dec_cover; }
void set_var_dec_cover(int v) { g_dec_cover = v; }

// Tile plan of decode_var_reg: rows per tile (a multiple of 64, <= kDecThreads), LDS bytes of the
// output images and of the row stage, within the LDS of two workgroups per CU.  Per-row sizes are
// estimated from the output capacities (exact after fury_row_decode_measure, an over-estimate under
// bound sizing); a tile whose payload outgrows its image stores that column straight to HBM and
// rows past the stage are read from HBM (both correct, slower), so the estimate only moves speed.
// mixed (C3): 512-row tiles.
void dec_tile_plan(const VarArgs& a, int* tile, uint32_t* img, uint32_t* stage, int pipe = 0) {
#ifndef FURY_DEC_BUDGET_KB
#define FURY_DEC_BUDGET_KB 80                     // (-D: A/B builds, scripts/r06_dec256.sh)
#endif
  constexpr int64_t kBudget = FURY_DEC_BUDGET_KB * 1024 - 1024;   // dynamic LDS per workgroup (+ static ~0.2 KB)
  double row = a.fixed_size, img_row = 0, img_fix = 0;
  for (int k = 0; k < a.ncols; k++) {
    const VarCol& c = hcol(a, k);
    const double per = a.nrows > 0 && c.capacity > 0 ? static_cast<double>(c.capacity) / a.nrows : 16.0;
    if (c.kind == kDecimal) row += 16;
    if (c.kind == kBytes) {
      row += per + 4;
      if (c.values) { img_row += per; img_fix += 80; }
    }
    if (c.kind == kListFixed) {
      row += 12 + per * (c.width == 0 ? 1 : c.width) + 4;
      if (c.values) {
        img_row += per * (c.width == 0 ? 0.125 : c.width) + (c.elem_validity ? per / 8 : 0);
        img_fix += c.elem_validity ? 160 : 80;
      }
    }
  }
  // headroom over the estimates: 8 % on the images, 2 % on the stage (a 512-row tile's bytes
  // vary by ~1 %; C4 0.252 -> 0.229 ms against 15 % / 5 %, mixed unchanged)
  const double mi = 1.08, mr = 1.02;
  if (g_dec_rows > 0) {                         // tuning "var_dec_rows": forced tile rows (A/B)
    const int R = g_dec_rows;
    const int64_t im = (static_cast<int64_t>(img_row * R * mi + img_fix) + 1023) & ~int64_t(1023);
    // a forced tile whose estimated images exceed half the budget is not run with clipped images
    // (that would change which overflow path an A/B leg measures): the plan below is used and the
    // rejection counted (fury_get_tuning "var_dec_rows_rejected")
    if (im <= kBudget / 2) {
      *tile = R;
      *img = static_cast<uint32_t>(im);
      *stage = static_cast<uint32_t>(((kBudget - *img) / (pipe == 2 ? 2 : 1)) & ~int64_t(15));
      return;
    }
    g_dec_rows_rejected.fetch_add(1);
  }
  for (int R = kDecThreads; R >= 64; R -= 64) {
    const int64_t im = (static_cast<int64_t>(img_row * R * mi + img_fix) + 1023) & ~int64_t(1023);
    const int64_t st = ((kBudget - im) / (pipe == 2 ? 2 : 1)) & ~int64_t(15);
    if (st >= static_cast<int64_t>(row * R * mr * g_dec_cover / 100.0) + 64 || R == 64) {
      *tile = R;
      *img = static_cast<uint32_t>(std::min<int64_t>(im, kBudget / 2));
      *stage = static_cast<uint32_t>(((kBudget - *img) / (pipe == 2 ? 2 : 1)) & ~int64_t(15));
      return;
    }
  }
}

int launch_decode_var(const VarArgs& a, const uint8_t* rows, const int64_t* offs,
                      hipStream_t stream, bool arrow) {
  (void)arrow;   // Arrow output differs only in requiring validity buffers (checked on host)
  if (a.nrows == 0) return FURY_OK;
  int nseq = 0;
  for (int k = 0; k < a.ncols; k++)
    if (hcol(a, k).kind == kBytes || hcol(a, k).kind == kListFixed) nseq++;
  const int mode = reg_mode(a);
  const int64_t nb = nblocks(a.nrows);
  if (a.ncols <= kRegCols) {
    VarArgs b = a;
    uint32_t img = 0, stage = 0;
    b.dec_pipe = dec_pipe_k(reg_dec_k(a.ncols)) ? g_dec_pipe.load() : 0;
    dec_tile_plan(a, &b.tile_rows, &img, &stage, b.dec_pipe);
    const int64_t nt = (a.nrows + b.tile_rows - 1) / b.tile_rows;
    // status words: tiles x K (the instance's column count), zeroed per launch
    const size_t wsb = static_cast<size_t>(nt) * reg_dec_k(a.ncols) * 8;
    uint64_t* ws = nullptr;
    int st = dev_alloc(wsb, stream, reinterpret_cast<void**>(&ws));
    if (st) return st;
    st = check_hip(hipMemsetAsync(ws, 0, wsb, stream), "memset");
    if (!st) st = launch_decode_var_reg(b, rows, offs, ws, img, stage, mode, nt, stream);
    dev_free(ws, stream);
    return st;
  }
  // wider than kRegCols: count pass + scan + write pass (wide.hip); tuning "var_wide" 0 = the
  // round-4 256-row look-back tile kernel below (A/B)
  if (var_wide_mode()) return launch_decode_wide(a, rows, offs, stream, false);
  // look-back status words (nb x nseq), zeroed per launch
  const size_t wsb = (nb * nseq + 1) * 8;
  uint64_t* ws = nullptr;
  int st = dev_alloc(wsb, stream, reinterpret_cast<void**>(&ws));
  if (st) return st;
  st = check_hip(hipMemsetAsync(ws, 0, wsb, stream), "memset");
  if (!st) {
    hipLaunchKernelGGL(decode_var_kernel, dim3(nb), dim3(kThreads), 0, stream, a, rows, offs,
                       ws, nseq);
    st = check_hip(hipGetLastError(), "decode_var launch");
  }
  dev_free(ws, stream);
  return st;
}

}  // namespace fury
