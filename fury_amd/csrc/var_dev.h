// var_dev.h -- device code of the variable-length kernels (var.hip, var_reg_enc.hip,
// var_reg_dec_lo.hip, var_reg_dec_hi.hip include it; each defines the FURY_VAR_* section it
// compiles, so the heavy register-staged template instances build in parallel).
#pragma once
// Original file comment (var.hip):
// var.hip — gfx950 kernels for schemas with variable-length fields (STRING/BINARY, DECIMAL,
// LIST of fixed-width elements): row-size measure + device scan, encode, decode-measure,
// decode / row->Arrow, and the [int32 len][int64 hash][row] stream framing.
//
// Reference semantics (FMT = java/fury-format/src/main/java/org/apache/fury/format):
//   var bytes  BinaryWriter.writeUnaligned: append at the writer index, pad to 8 with zeros
//              (pad word zeroed first), slot = (relativeOffset << 32) | unpaddedSize
//              (FMT/row/binary/writer/BinaryWriter.java:106-121,187-194)
//   decimal    BinaryWriter.writeDecimal: 16 bytes appended (BinaryWriter.java:204-219)
//   list       serializeFor(List) -> BinaryArrayWriter.reset(n) + per-element write, slot =
//              offset/size of [int64 n][bitmap][values, tail zeroed]
//              (FMT/encoder/BaseBinaryEncoderBuilder.java:198-278,
//               FMT/row/binary/writer/BinaryArrayWriter.java:91-163)
//   decode     UnsafeTrait.getBinary / getArray + BinaryArray.toXxxArray
//              (FMT/row/binary/UnsafeTrait.java:115-178, BinaryArray.java:69-78,157-197);
//   to Arrow   ArrowWriter StringWriter / ListWriter (FMT/vectorized/ArrowWriter.java:421-540)
//
// MI355X design: one workgroup of 256 threads owns 256 consecutive rows, i.e. one contiguous
// byte range of the row buffer (rows are packed by the exclusive scan of their sizes).  The
// group builds (encode) or reads (decode) its rows through an LDS image of that range so that
// global traffic is 16-byte-per-lane contiguous even though each row is built by one thread;
// ranges larger than the LDS budget fall back to direct 8-byte global accesses.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

constexpr int kThreads = 256;                 // = rows per workgroup
constexpr int kDecodeStage = 32 * 1024;       // LDS image of the group's row range (decode)
constexpr int kStrStage = 8 * 1024;           // LDS image of one column's Arrow payload range

// Column record k: from the kernel argument block, or -- schemas wider than kMaxVarCols -- from
// the device table the host uploaded for the call (VarArgs.tab).  Uniform branch, scalar loads.
// Both live in the constant address space (kernarg segment / a read-only device table), so the
// record's fields are scalar loads; a select of the kernarg and the table pointers as generic
// pointers compiled to flat (vector) loads, each waited with vmcnt and lgkmcnt.
using CVarCol = __attribute__((address_space(4))) const VarCol;
__device__ __forceinline__ CVarCol& vc(const VarArgs& a, int k) {
  CVarCol* base = a.tab ? (CVarCol*)(a.tab) : (CVarCol*)(a.col);
  return base[k];
}

__device__ __forceinline__ bool bit_at(const uint8_t* bits, int64_t i) {
  return (bits[i >> 3] >> (i & 7)) & 1;
}
// bit_at of a bitmap in device memory (global loads, never flat)
__device__ __forceinline__ bool bit_at_g(const uint8_t* bits, int64_t i) {
  return (gl(bits)[i >> 3] >> (i & 7)) & 1;
}
__device__ __forceinline__ int64_t rnd8(int64_t n) { return (n + 7) & ~int64_t(7); }
__host__ __device__ __forceinline__ int64_t r16(int64_t x) { return (x + 15) & ~int64_t(15); }
__device__ __forceinline__ int64_t bm_bytes(int64_t n) { return ((n + 63) >> 6) << 3; }

// Element i of a device-memory column (global loads).
__device__ __forceinline__ uint64_t load_fixed(const uint8_t* p, int64_t i, int w) {
  switch (w) {
    case 8: return *gl(reinterpret_cast<const uint64_t*>(p + i * 8));
    case 4: return *gl(reinterpret_cast<const uint32_t*>(p + i * 4));
    case 2: return *gl(reinterpret_cast<const uint16_t*>(p + i * 2));
    case 1: return gl(p)[i];
    default: return bit_at_g(p, i);
  }
}

// 64-lane block scan helpers -------------------------------------------------------------------
__device__ __forceinline__ int64_t wave_incl_scan(int64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Inclusive 32-bit scan over the 64 lanes of a wave by DPP: row shifts 1, 2, 4, 8 inside each
// 16-lane row, then the row broadcasts 15 / 31 carry rows 0 -> 1, 2 -> 3 and rows 0-1 -> 2-3
// (gfx9-family DPP; lanes without a source add the `old` operand, 0).
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t x) {
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x111, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x112, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x114, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x118, 0xf, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x142, 0xa, 0xf, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x143, 0xc, 0xf, false));
  return x;
}

// Exclusive scan over the NT threads of the block; *total gets the block sum.
template <int NT = kThreads>
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* total, int64_t* tmp) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t x = wave_incl_scan(v);
  if (lane == 63) tmp[wid] = x;
  __syncthreads();
  int64_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
    const int64_t s = tmp[w];
    pre += (w < wid) ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// --- encode side -------------------------------------------------------------------------------

// Copies len bytes from an unaligned source to an 8-byte aligned destination as whole 8-byte
// words, zero-filling the pad (writeUnaligned + zeroOutPaddingBytes).  Source words are read
// aligned; no word past the one holding the last source byte is touched.
__device__ __forceinline__ void copy_to_aligned(uint64_t* dst, const uint8_t* src, int64_t len) {
  if (len <= 0) return;
  const uintptr_t s = reinterpret_cast<uintptr_t>(src) & 7;
  const uint64_t* ap = reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(src) - s);
  if (len <= 32) {
    // short string: every source word is requested before any is used (one memory latency
    // instead of one per word); words past the last source byte are not read
    const int nsrc = static_cast<int>((s + len + 7) >> 3);       // <= 5
    uint64_t w[5];
#pragma unroll
    for (int j = 0; j < 5; j++) w[j] = j < nsrc ? ap[j] : 0;
    const int nw = static_cast<int>((len + 7) >> 3);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (k < nw) {
        uint64_t x = s ? (w[k] >> (8 * s)) | (w[k + 1] << (64 - 8 * s)) : w[k];
        const int64_t rem = len - 8 * k;
        if (rem < 8) x &= (~0ull) >> (8 * (8 - rem));
        dst[k] = x;
      }
    }
    return;
  }
  const int64_t nw = (len + 7) >> 3;
  const int64_t last_src_word = (static_cast<int64_t>(s) + len - 1) >> 3;
  uint64_t lo = ap[0];
  for (int64_t k = 0; k < nw; k++) {
    uint64_t w;
    if (s == 0) {
      w = (k == 0) ? lo : ap[k];
    } else {
      const uint64_t hi = (k + 1 <= last_src_word) ? ap[k + 1] : 0;
      w = (lo >> (8 * s)) | (hi << (64 - 8 * s));
      lo = hi;
    }
    const int64_t rem = len - 8 * k;
    if (rem < 8) w &= (~0ull) >> (8 * (8 - rem));
    dst[k] = w;
  }
}

// BinaryArrayWriter image of n elements of a fixed-width list column; returns its size.
// `vals` points at the first element's value bytes, `vbits`/`vbit0` at its Arrow validity bit
// (vbits == nullptr: no element nulls).  Sources may be global or an LDS staging copy.
__device__ int64_t write_array(uint8_t* dst, int width, const uint8_t* vals, const uint8_t* vbits,
                               int64_t vbit0, int64_t n) {
  const int ew = width == 0 ? 1 : width;
  const int64_t hb = 8 + bm_bytes(n);
  const int64_t data = n * ew;
  const int64_t fp = rnd8(data);
  uint64_t* d64 = reinterpret_cast<uint64_t*>(dst);
  d64[0] = static_cast<uint64_t>(n);                     // numElements as an 8-byte word
  for (int64_t w = 0; w < (hb - 8) >> 3; w++) {          // element null bits (bit = 1 null)
    uint64_t word = 0;
    if (vbits) {
      const int64_t lim = min<int64_t>(64, n - 64 * w);
      for (int64_t t = 0; t < lim; t++)
        if (!bit_at(vbits, vbit0 + 64 * w + t)) word |= 1ull << t;
    }
    d64[1 + w] = word;
  }
  uint64_t* out = reinterpret_cast<uint64_t*>(dst + hb);
  if (width == 8 && !vbits) {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(vals);
    for (int64_t j = 0; j < n; j++) out[j] = src[j];
    return hb + fp;
  }
  const int per = 8 / ew;
  for (int64_t q = 0; q < (fp >> 3); q++) {
    uint64_t word = 0;
    for (int t = 0; t < per; t++) {
      const int64_t j = q * per + t;
      if (j >= n) break;
      if (vbits && !bit_at(vbits, vbit0 + j)) continue;   // null element stays 0
      uint64_t v;
      switch (width) {
        case 8: v = reinterpret_cast<const uint64_t*>(vals)[j]; break;
        case 4: v = reinterpret_cast<const uint32_t*>(vals)[j]; break;
        case 2: v = reinterpret_cast<const uint16_t*>(vals)[j]; break;
        case 1: v = vals[j]; break;
        default: v = bit_at(vals, vbit0 + j); break;       // bool: bit-packed, same bit origin
      }
      word |= (ew == 8) ? v : (v << (8 * ew * t));
    }
    out[q] = word;
  }
  return hb + fp;
}

// Cooperative 8-byte-aligned copy of [0, bytes) between LDS and global (16 B per lane when the
// global side is 16-byte aligned).
template <bool kToGlobal, int NT = kThreads>
__device__ __forceinline__ void copy_range(uint8_t* g, uint8_t* l, int64_t bytes) {
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  int64_t head = 0;
  if ((reinterpret_cast<uintptr_t>(g) & 15) && bytes >= 8) head = 8;
  if (head && threadIdx.x == 0) {
    if (kToGlobal) *reinterpret_cast<uint64_t*>(g) = *reinterpret_cast<uint64_t*>(l);
    else *reinterpret_cast<uint64_t*>(l) = *reinterpret_cast<uint64_t*>(g);
  }
  const int64_t body = (bytes - head) >> 4;
  // LDS side may be only 8-aligned at g+head: move 2 x 8 bytes per lane on the LDS side.
  for (int64_t i = threadIdx.x; i < body; i += NT) {
    uint8_t* gp = g + head + 16 * i;
    uint8_t* lp = l + head + 16 * i;
    if (kToGlobal) {
      const uint64_t x = reinterpret_cast<uint64_t*>(lp)[0], y = reinterpret_cast<uint64_t*>(lp)[1];
      v4 v;
      v.x = static_cast<uint32_t>(x); v.y = static_cast<uint32_t>(x >> 32);
      v.z = static_cast<uint32_t>(y); v.w = static_cast<uint32_t>(y >> 32);
      __builtin_nontemporal_store(v, reinterpret_cast<v4*>(gp));
    } else {
      const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4*>(gp));
      reinterpret_cast<uint64_t*>(lp)[0] = (static_cast<uint64_t>(v.y) << 32) | v.x;
      reinterpret_cast<uint64_t*>(lp)[1] = (static_cast<uint64_t>(v.w) << 32) | v.z;
    }
  }
  const int64_t done = head + 16 * body;
  if (done < bytes && threadIdx.x == NT - 1) {    // one trailing 8-byte word
    if (kToGlobal) *reinterpret_cast<uint64_t*>(g + done) = *reinterpret_cast<uint64_t*>(l + done);
    else *reinterpret_cast<uint64_t*>(l + done) = *reinterpret_cast<uint64_t*>(g + done);
  }
}

// Exclusive scan of small arrays (<= kSmallScan entries): one workgroup, a few block scans.
constexpr int64_t kSmallScan = 16 * kThreads;
#ifdef FURY_VAR_MAIN
__global__ __launch_bounds__(kThreads) void scan_small(int64_t* __restrict__ s, int64_t n,
                                                       int64_t* __restrict__ total) {
  __shared__ int64_t tmp[kThreads / 64];
  int64_t carry = 0;
  for (int64_t base = 0; base < n; base += kThreads) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < n ? s[i] : 0;
    int64_t tot;
    const int64_t ex = block_excl_scan(v, &tot, tmp);
    if (i < n) s[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}
#endif  // FURY_VAR_MAIN

// One level of the hierarchical scan: each workgroup scans 256 entries in place (exclusive) and
// emits their total.
#ifdef FURY_VAR_MAIN
__global__ __launch_bounds__(kThreads) void scan_groups(int64_t* __restrict__ s, int64_t n,
                                                        int64_t* __restrict__ gsum) {
  __shared__ int64_t tmp[kThreads / 64];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  const int64_t v = i < n ? s[i] : 0;
  int64_t tot;
  const int64_t ex = block_excl_scan(v, &tot, tmp);
  if (i < n) s[i] = ex;
  if (threadIdx.x == 0) gsum[blockIdx.x] = tot;
}
#endif  // FURY_VAR_MAIN

#ifdef FURY_VAR_MAIN
__global__ __launch_bounds__(kThreads) void add_groups(int64_t* __restrict__ s, int64_t n,
                                                       const int64_t* __restrict__ gpre) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i < n) s[i] += gpre[blockIdx.x];
}
#endif  // FURY_VAR_MAIN

// --- cross-workgroup scan (decoupled look-back) ---------------------------------------------
constexpr int kSeqChunk = 8;                          // var outputs resolved per look-back round
constexpr uint64_t kAgg = 1ull << 62, kInc = 2ull << 62, kValMask = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t ld_status(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t wave_sum(int64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// One wave: exclusive prefix of logical group b in sequence q.  Status words pack a 2-bit flag
// (0 = not yet published, kAgg = group total, kInc = inclusive prefix) over a 62-bit value.
__device__ int64_t look_back(const uint64_t* status, int64_t b, int nseq, int q) {
  const int lane = threadIdx.x & 63;
  int64_t excl = 0;
  for (int64_t j = b - 1;; j -= 64) {
    const int64_t idx = j - lane;
    uint64_t v;
    for (;;) {
      v = idx >= 0 ? ld_status(status + idx * nseq + q) : kInc;
      if (__ballot((v >> 62) == 0) == 0) break;
      __builtin_amdgcn_s_sleep(1);
    }
    const uint64_t inc = __ballot((v >> 62) == 2);
    const int stop = inc ? __builtin_ctzll(inc) : 63;
    excl += wave_sum(lane <= stop ? static_cast<int64_t>(v & kValMask) : 0);
    if (inc) return excl;
  }
}

// ---- tile-staged encode ------------------------------------------------------------------------
// One workgroup of kEncRows threads owns kEncRows consecutive rows.  Every input the tile reads
// is a contiguous global range (a column's values / validity bytes / offsets for the tile, then
// each string column's payload bytes and each list column's element values + validity between
// the tile's first and last offsets), so the tile is staged in LDS by LDS-DMA
// (global_load_lds_dwordx4: 16-B pieces, no register round trip, all pieces of a phase in flight
// together): two dependent round trips to HBM per tile (meta, then payloads).  Each thread then
// builds its row from LDS into an LDS image of the tile's contiguous output range, which leaves
// with 16-B stores.
constexpr int kEncRows = 256;                 // threads per encode workgroup = max rows per tile
constexpr int kEncPool = 50 * 1024;           // LDS: staged inputs + row image (3 groups per CU)
constexpr int kMetaPool = 16 * 1024;          // bound on a tile's staged per-row inputs
constexpr uint32_t kNone = 0xffffffffu;

// LDS byte offsets of one tile's staged inputs, per column (kNone = not present / not staged).
template <int N>
struct MetaMapN {
  uint32_t fix[N];   // fixed values (row r0) / bool bits (byte r0/8) / decimal values
  uint32_t val[N];   // validity bits, byte r0/8
  uint32_t off[N];   // int32 offsets, entry r0
  uint32_t pay[N];   // payload bytes at offsets[r0] (bool elements: byte offsets[r0]/8)
  uint32_t pvb[N];   // list element validity, byte offsets[r0]/8
};
using MetaMap = MetaMapN<kMaxVarCols>;
using MetaMapWide = MetaMapN<kMaxWideVarCols>;

// Issues LDS-DMA copies of the 16-B-aligned pieces covering [gb, ge) into pool[at...]; returns
// the LDS offset of byte gb and advances `at` (kept 16-aligned).  Reading whole aligned pieces
// never leaves the pages holding the range.
template <int NT>
__device__ __forceinline__ uint32_t stage_range(uint8_t* pool, uint32_t& at, const uint8_t* gb,
                                                const uint8_t* ge, bool issue = true) {
  const uint64_t lo = reinterpret_cast<uint64_t>(gb) & ~uint64_t(15);
  const uint64_t hi = (reinterpret_cast<uint64_t>(ge) + 15) & ~uint64_t(15);
  const uint32_t nch = static_cast<uint32_t>((hi - lo) >> 4);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t i0 = wave * 64; issue && i0 < nch; i0 += NT) {
    if (i0 + lane < nch)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(lo + 16ull * (i0 + lane)),
                                       pool + at + 16 * i0, 16, 0, 0);
  }
  const uint32_t r = at + static_cast<uint32_t>(reinterpret_cast<uint64_t>(gb) - lo);
  at += nch * 16;
  return r;
}

__device__ __forceinline__ int32_t lds_i32(const uint8_t* pool, uint32_t off) {
  return *reinterpret_cast<const int32_t*>(pool + off);
}
__device__ __forceinline__ bool lds_bit(const uint8_t* pool, uint32_t off, int64_t i) {
  return (pool[off + (i >> 3)] >> (i & 7)) & 1;
}

// Phase A: stage every column's per-row inputs of rows [r0, r0 + nr).
template <int NT, class MM>
__device__ __forceinline__ uint32_t stage_meta(const VarArgs& a, int64_t r0, int64_t nr,
                                               uint8_t* pool, MM& mm, uint32_t at = 0) {
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    uint32_t fix = kNone, val = kNone, off = kNone;
    if (c.validity) val = stage_range<NT>(pool, at, c.validity + (r0 >> 3), c.validity + ((r0 + nr + 7) >> 3));
    switch (c.kind) {
      case kFixed:
        fix = stage_range<NT>(pool, at, c.values + r0 * c.width, c.values + (r0 + nr) * c.width);
        break;
      case kBool:
        fix = stage_range<NT>(pool, at, c.values + (r0 >> 3), c.values + ((r0 + nr + 7) >> 3));
        break;
      case kDecimal:
        fix = stage_range<NT>(pool, at, c.values + 16 * r0, c.values + 16 * (r0 + nr));
        break;
      default:      // kBytes, kListFixed
        off = stage_range<NT>(pool, at, reinterpret_cast<const uint8_t*>(c.offsets + r0),
                              reinterpret_cast<const uint8_t*>(c.offsets + r0 + nr + 1));
        break;
    }
    if (threadIdx.x == 0) {
      mm.fix[k] = fix;
      mm.val[k] = val;
      mm.off[k] = off;
      mm.pay[k] = kNone;
      mm.pvb[k] = kNone;
    }
  }
  return at;
}

// Row size of tile row t from the staged inputs (writerIndex growth of toRow).
template <class MM>
__device__ __forceinline__ int64_t tile_row_size(const VarArgs& a, const MM& mm,
                                                 const uint8_t* pool, int t) {
  int64_t sz = a.fixed_size;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (c.kind < kBytes) continue;
    if (mm.val[k] != kNone && !lds_bit(pool, mm.val[k], t)) continue;
    if (c.kind == kDecimal) {
      sz += 16;
      continue;
    }
    const int64_t n = lds_i32(pool, mm.off[k] + 4 * (t + 1)) - lds_i32(pool, mm.off[k] + 4 * t);
    if (c.kind == kBytes) sz += rnd8(n);
    else sz += 8 + bm_bytes(n) + rnd8(n * (c.width == 0 ? 1 : c.width));
  }
  return sz;
}

// Bytes the payload staging of the tile needs (uniform; from the staged offsets).
template <class MM>
__device__ __forceinline__ uint64_t payload_need(const VarArgs& a, const MM& mm,
                                                 const uint8_t* pool, int nr) {
  uint64_t need = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (c.kind != kBytes && c.kind != kListFixed) continue;
    const int64_t b = lds_i32(pool, mm.off[k]), e = lds_i32(pool, mm.off[k] + 4 * nr);
    if (e <= b) continue;
    int64_t bytes;
    if (c.kind == kBytes) bytes = e - b;
    else if (c.width == 0) bytes = ((e + 7) >> 3) - (b >> 3);
    else bytes = (e - b) * c.width;
    need += static_cast<uint64_t>(bytes) + 32;
    if (c.kind == kListFixed && c.elem_validity) need += static_cast<uint64_t>(((e + 7) >> 3) - (b >> 3)) + 32;
  }
  return need;
}

// Phase C: stage the payload ranges.
template <int NT, class MM>
__device__ __forceinline__ void stage_payloads(const VarArgs& a, MM& mm, uint8_t* pool,
                                               uint32_t at, int nr) {
  const bool iss = true;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (c.kind != kBytes && c.kind != kListFixed) continue;
    const int64_t b = lds_i32(pool, mm.off[k]), e = lds_i32(pool, mm.off[k] + 4 * nr);
    uint32_t pay = kNone, pvb = kNone;
    if (e > b) {
      if (c.kind == kBytes) pay = stage_range<NT>(pool, at, c.values + b, c.values + e, iss);
      else if (c.width == 0) pay = stage_range<NT>(pool, at, c.values + (b >> 3), c.values + ((e + 7) >> 3), iss);
      else pay = stage_range<NT>(pool, at, c.values + b * c.width, c.values + e * c.width, iss);
      if (c.kind == kListFixed && c.elem_validity)
        pvb = stage_range<NT>(pool, at, c.elem_validity + (b >> 3), c.elem_validity + ((e + 7) >> 3), iss);
    }
    if (threadIdx.x == 0) {
      mm.pay[k] = pay;
      mm.pvb[k] = pvb;
    }
  }
}

// Builds tile row t at dst (8-byte aligned) exactly as toRow does.  Per-row inputs come from the
// staged meta in `pool`; a column's payload from `pay` when it was staged (mm.pay[k] != kNone),
// else straight from global memory.
template <class MM>
__device__ __forceinline__ void build_tile_row(const VarArgs& a, const MM& mm,
                                               const uint8_t* pool, const uint8_t* pay, int t,
                                               uint8_t* dst) {
  uint64_t* d64 = reinterpret_cast<uint64_t*>(dst);
  const int nslot0 = a.bitmap_bytes >> 3;
  int64_t cursor = a.fixed_size;
  uint64_t nullbits = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    uint64_t slot = 0;
    if (mm.val[k] != kNone && !lds_bit(pool, mm.val[k], t)) {
      nullbits |= 1ull << (k & 63);
    } else {
      switch (c.kind) {
        case kFixed: {
          const uint8_t* p = pool + mm.fix[k] + t * c.width;
          switch (c.width) {
            case 8: slot = *reinterpret_cast<const uint64_t*>(p); break;
            case 4: slot = *reinterpret_cast<const uint32_t*>(p); break;
            case 2: slot = *reinterpret_cast<const uint16_t*>(p); break;
            default: slot = *p; break;
          }
          break;
        }
        case kBool:
          slot = lds_bit(pool, mm.fix[k], t);
          break;
        case kBytes: {
          const int64_t ob = lds_i32(pool, mm.off[k]);
          const int64_t o0 = lds_i32(pool, mm.off[k] + 4 * t);
          const int64_t len = lds_i32(pool, mm.off[k] + 4 * (t + 1)) - o0;
          const uint8_t* src = mm.pay[k] != kNone ? pay + mm.pay[k] + (o0 - ob) : c.values + o0;
          copy_to_aligned(d64 + (cursor >> 3), src, len);
          slot = (static_cast<uint64_t>(cursor) << 32) | static_cast<uint32_t>(len);
          cursor += rnd8(len);
          break;
        }
        case kDecimal: {
          const uint64_t* s = reinterpret_cast<const uint64_t*>(pool + mm.fix[k] + 16 * t);
          d64[cursor >> 3] = s[0];
          d64[(cursor >> 3) + 1] = s[1];
          slot = (static_cast<uint64_t>(cursor) << 32) | 16u;
          cursor += 16;
          break;
        }
        default: {   // kListFixed
          const int64_t ob = lds_i32(pool, mm.off[k]);
          const int64_t o0 = lds_i32(pool, mm.off[k] + 4 * t);
          const int64_t n = lds_i32(pool, mm.off[k] + 4 * (t + 1)) - o0;
          const uint8_t* vals;
          const uint8_t* vb = nullptr;
          if (c.width == 0)
            vals = mm.pay[k] != kNone ? pay + mm.pay[k] + ((o0 >> 3) - (ob >> 3)) : c.values + (o0 >> 3);
          else
            vals = mm.pay[k] != kNone ? pay + mm.pay[k] + (o0 - ob) * c.width : c.values + o0 * c.width;
          if (c.elem_validity)
            vb = mm.pvb[k] != kNone ? pay + mm.pvb[k] + ((o0 >> 3) - (ob >> 3)) : c.elem_validity + (o0 >> 3);
          const int64_t sz = write_array(dst + cursor, c.width, vals, vb, o0 & 7, n);
          slot = (static_cast<uint64_t>(cursor) << 32) | static_cast<uint32_t>(sz);
          cursor += sz;
          break;
        }
      }
    }
    d64[nslot0 + k] = slot;
    if ((k & 63) == 63) {                    // > 64 fields: one bitmap word per 64 fields
      d64[k >> 6] = nullbits;
      nullbits = 0;
    }
  }
  if (a.ncols & 63) d64[(a.ncols - 1) >> 6] = nullbits;
}

// Encode workgroup: rows [r0, r0 + R) at the offsets fury_row_measure produced.  Bytes at or
// past `cap` are never written.
template <int POOL, bool kStagePay, class MM>
__device__ __forceinline__ void encode_tile(const VarArgs& a, const int64_t* __restrict__ offs,
                                            uint8_t* __restrict__ rows, int64_t cap, int64_t tile,
                                            uint8_t* pool, MM& mm) {
  const int tid = threadIdx.x;
  const int R = a.tile_rows;                 // rows per tile (host-chosen so the meta fits)
  const int64_t r0 = tile * R;
  const int nr = static_cast<int>(min<int64_t>(R, a.nrows - r0));
  const bool live = tid < nr;
  // the offset loads go out together with the meta DMA
  const int64_t base = offs[r0];
  const int64_t bytes = offs[r0 + nr] - base;
  const int64_t ex = live ? offs[r0 + tid] - base : 0;
  const uint32_t img_at = stage_meta<kEncRows>(a, r0, nr, pool, mm);
  __syncthreads();
  const uint64_t img = static_cast<uint64_t>((bytes + 15) & ~int64_t(15));
  const bool img_fits = img_at + img <= POOL;
  const bool pay_fits =
      kStagePay && img_fits && img_at + img + payload_need(a, mm, pool, nr) <= POOL;
  if (pay_fits) {
    stage_payloads<kEncRows>(a, mm, pool, static_cast<uint32_t>(img_at + img), nr);
    __syncthreads();
  }
  const int64_t room = max<int64_t>(0, min<int64_t>(bytes, cap - base));
  if (img_fits) {
    uint8_t* image = pool + img_at;
    if (live) build_tile_row(a, mm, pool, pool, tid, image + ex);
    __syncthreads();
    copy_range<true, kEncRows>(rows + base, image, room);
  } else if (live && ex + tile_row_size(a, mm, pool, tid) <= room) {
    build_tile_row(a, mm, pool, pool, tid, rows + base + ex);    // oversized tile: straight to HBM
  }
}

#ifdef FURY_VAR_MAIN
template <class MM = MetaMap>
__global__ __launch_bounds__(kEncRows) void encode_var_kernel(VarArgs a,
                                                              const int64_t* __restrict__ offs,
                                                              uint8_t* __restrict__ rows,
                                                              int64_t cap) {
  __shared__ __attribute__((aligned(16))) uint8_t pool[kEncPool];
  __shared__ MM mm;
  encode_tile<kEncPool, true>(a, offs, rows, cap, blockIdx.x, pool, mm);
}
#endif  // FURY_VAR_MAIN

// Stores img[0, bytes) to g (any alignment): each wave writes a contiguous quarter of the 16-byte
// aligned body with 16-B non-temporal stores, wave 0 the unaligned head and wave 3 the tail by
// single-byte lanes.  Returns the number of store instructions this wave issued (uniform).
__device__ __forceinline__ int store_image(uint8_t* g, const uint8_t* img, int64_t bytes) {
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (bytes <= 0) return 0;
  const int64_t head = min<int64_t>(bytes, (16 - (reinterpret_cast<uintptr_t>(g) & 15)) & 15);
  const int64_t body = (bytes - head) >> 4;
  const int64_t tail = bytes - head - 16 * body;
  int cnt = 0;
  if (head > 0 && wave == 0) {
    if (lane < head) g[lane] = img[lane];
    cnt++;
  }
  const int64_t q = (body + 3) >> 2;
  const int64_t j0 = wave * q, j1 = min<int64_t>(body, j0 + q);
  for (int64_t j = j0; j < j1; j += 64) {
    const int64_t i = j + lane;
    if (i < j1) {
      const uint8_t* lp = img + head + 16 * i;
      const uint64_t x = reinterpret_cast<const uint64_t*>(lp)[0];
      const uint64_t y = reinterpret_cast<const uint64_t*>(lp)[1];
      v4 v;
      v.x = static_cast<uint32_t>(x); v.y = static_cast<uint32_t>(x >> 32);
      v.z = static_cast<uint32_t>(y); v.w = static_cast<uint32_t>(y >> 32);
      __builtin_nontemporal_store(v, reinterpret_cast<v4*>(g + head + 16 * i));
    }
    cnt++;
  }
  if (tail > 0 && wave == 3) {
    const int64_t t0 = head + 16 * body;
    if (lane < tail) g[t0 + lane] = img[t0 + lane];
    cnt++;
  }
  return cnt;
}

// ---- register-staged encode (schemas of <= kRegCols fields) -----------------------------------
// One workgroup builds one tile of R rows (thread = row) into an LDS image of the tile's
// contiguous output range, then stores it with 16-B stores.  The per-row inputs of every column
// are loaded straight into registers (the column count is a template parameter, so the per-column
// values live in VGPRs and all the loads are issued together: one HBM round trip), and the
// string / decimal / list bytes are then read from global memory by their row's thread (a second
// round trip, issued for all columns at once).  LDS holds only the image, so five workgroups
// share a CU.
constexpr int kRegCols = 16;
// kind modes of the register-staged instances (kind_of)
constexpr int kSeqBytes = 0, kSeqLists = 1, kSeqAll = 2;
// The kind of column k as a register-staged kernel instance sees it.  Instances for schemas of
// fixed-width, bool and STRING / BINARY fields only (kSeqBytes) or of fixed-width, bool and LIST
// fields (kSeqLists), as the host checks (reg_mode), map every kind onto those three, so the
// compiler drops the other kinds' code from the unrolled K-column bodies (mixed decode, K = 6:
// 7.1k instead of 18k instructions; the full body cost it ~10 % in instruction-cache misses).
template <int M>
__device__ __forceinline__ int kind_of(const VarCol& c) {
  const int kd = c.kind;
  if (M == kSeqAll) return kd;
  const int seq = M == kSeqBytes ? kBytes : kListFixed;
  return kd == seq ? seq : (kd == kBool ? kBool : kFixed);
}
// a sequence column's payload is bytes (else list elements)
template <int M>
__device__ __forceinline__ bool bytes_seq(const VarCol& c) {
  return M == kSeqBytes || (M == kSeqAll && c.kind == kBytes);
}
__device__ __forceinline__ bool seq_kind(int kd) { return kd == kBytes || kd == kListFixed; }

constexpr int kRegImg = 30 * 1024;

// Copies len bytes at global src to 8-byte aligned dst (LDS or global) as whole words, zero pad.
template <typename D>
__device__ __forceinline__ void put_string(D* dst, const uint8_t* src, int64_t len) {
  if (len <= 0) return;
  const uintptr_t s = reinterpret_cast<uintptr_t>(src) & 7;
  const auto ap = gl(reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(src) - s));
  const int64_t nw = (len + 7) >> 3;
  const int64_t nsrc = (static_cast<int64_t>(s) + len + 7) >> 3;
  for (int64_t k0 = 0; k0 < nw; k0 += 4) {
    uint64_t w[5];
#pragma unroll
    for (int j = 0; j < 5; j++) w[j] = k0 + j < nsrc ? ap[k0 + j] : 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int64_t k = k0 + j;
      if (k < nw) {
        uint64_t x = s ? (w[j] >> (8 * s)) | (w[j + 1] << (64 - 8 * s)) : w[j];
        const int64_t rem = len - 8 * k;
        if (rem < 8) x &= (~0ull) >> (8 * (8 - rem));
        dst[k] = x;
      }
    }
  }
}

// 64 bits of a bitmap starting at bit i, reading only the aligned words that hold wanted bits
// (bits past `lim` are garbage).
__device__ __forceinline__ uint64_t load_bits64(const uint8_t* bits, int64_t i, int lim) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(bits) + (i >> 3);
  const auto a = gl(reinterpret_cast<const uint64_t*>(addr & ~uintptr_t(7)));    // device memory
  const int sh = static_cast<int>((addr & 7) * 8 + (i & 7));
  const uint64_t lo = a[0];
  if (sh == 0) return lo;
  const uint64_t hi = sh + lim > 64 ? a[1] : 0;
  return (lo >> sh) | (hi << (64 - sh));
}

// BinaryArrayWriter image of n elements read from global memory (register-staged encode):
// element values and validity words are fetched in batches so their loads overlap.
template <typename D>
__device__ __forceinline__ int64_t put_array(D* d64, int width, const uint8_t* vals,
                                             const uint8_t* vbits, int64_t vbit0, int64_t n) {
  const int ew = width == 0 ? 1 : width;
  const int64_t nbw = (n + 63) >> 6;
  d64[0] = static_cast<uint64_t>(n);
  for (int64_t w = 0; w < nbw; w++) {
    const int lim = static_cast<int>(min<int64_t>(64, n - 64 * w));
    const uint64_t valid = vbits ? load_bits64(vbits, vbit0 + 64 * w, lim) : ~0ull;
    const uint64_t m = lim == 64 ? ~0ull : ((1ull << lim) - 1);
    d64[1 + w] = ~valid & m;                            // bit = 1 null
  }
  D* out = d64 + 1 + nbw;
  if (ew == 8) {
    const auto src = gl(reinterpret_cast<const uint64_t*>(vals));
    for (int64_t j0 = 0; j0 < n; j0 += 8) {
      const int lim = static_cast<int>(min<int64_t>(8, n - j0));
      const uint64_t vm = vbits ? load_bits64(vbits, vbit0 + j0, lim) : ~0ull;
      uint64_t x[8];
#pragma unroll
      for (int u = 0; u < 8; u++) x[u] = u < lim ? src[j0 + u] : 0;
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (u < lim) out[j0 + u] = ((vm >> u) & 1) ? x[u] : 0;
    }
    return 8 * (1 + nbw + n);
  }
  const int per = 8 / ew;
  const int64_t nw = (n * ew + 7) >> 3;
  for (int64_t q = 0; q < nw; q++) {
    const int lim = static_cast<int>(min<int64_t>(per, n - q * per));
    const uint64_t vm = vbits ? load_bits64(vbits, vbit0 + q * per, lim) : ~0ull;
    uint64_t word = 0;
    for (int t = 0; t < lim; t++) {
      const int64_t j = q * per + t;
      if (!((vm >> t) & 1)) continue;                  // null element stays 0
      uint64_t x;
      switch (width) {
        case 4: x = gl(reinterpret_cast<const uint32_t*>(vals))[j]; break;
        case 2: x = gl(reinterpret_cast<const uint16_t*>(vals))[j]; break;
        case 1: x = gl(vals)[j]; break;
        default: x = bit_at_g(vals, vbit0 + j); break;   // bool: bit-packed, same bit origin
      }
      word |= x << (8 * ew * t);
    }
    out[q] = word;
  }
  return 8 * (1 + nbw + nw);
}

// Builds row r (tile thread t) at d64 from the register-staged inputs.
template <int K, int M, typename D>
__device__ __forceinline__ void reg_build_row(const VarArgs& a, int64_t r, const uint64_t* v,
                                              uint64_t valid, D* d64) {
  const int nslot0 = a.bitmap_bytes >> 3;
  int64_t cursor = a.fixed_size;
  uint64_t nullbits = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    if (k >= a.ncols) continue;              // K rounded up past the schema's fields
    const VarCol& c = a.col[k];
    const int kd = kind_of<M>(c);
    uint64_t slot = 0;
    if (!((valid >> k) & 1)) {
      nullbits |= 1ull << k;
    } else if (kd == kFixed || kd == kBool) {
      slot = v[k];
    } else if (kd == kBytes) {
      const int32_t o0 = static_cast<int32_t>(v[k]), o1 = static_cast<int32_t>(v[k] >> 32);
      const int64_t len = o1 - o0;
      put_string(d64 + (cursor >> 3), c.values + o0, len);
      slot = (static_cast<uint64_t>(cursor) << 32) | static_cast<uint32_t>(len);
      cursor += rnd8(len);
    } else if (kd == kDecimal) {
      const auto s = gl(reinterpret_cast<const uint64_t*>(c.values)) + 2 * r;
      d64[cursor >> 3] = s[0];
      d64[(cursor >> 3) + 1] = s[1];
      slot = (static_cast<uint64_t>(cursor) << 32) | 16u;
      cursor += 16;
    } else {   // kListFixed
      const int32_t o0 = static_cast<int32_t>(v[k]), o1 = static_cast<int32_t>(v[k] >> 32);
      const int64_t n = o1 - o0;
      const uint8_t* vals = c.width == 0 ? c.values + (o0 >> 3) : c.values + int64_t(o0) * c.width;
      const uint8_t* vb = c.elem_validity ? c.elem_validity + (o0 >> 3) : nullptr;
      const int64_t sz = put_array(d64 + (cursor >> 3), c.width, vals, vb, o0 & 7, n);
      slot = (static_cast<uint64_t>(cursor) << 32) | static_cast<uint32_t>(sz);
      cursor += sz;
    }
    d64[nslot0 + k] = slot;
  }
  d64[0] = nullbits;
}

#ifdef FURY_VAR_ENC
// Size of the row whose per-column inputs are v / valid (encode_var_reg's registers): the same
// writerIndex growth as row_size_of.
template <int K, int M>
__device__ __forceinline__ int64_t reg_row_size(const VarArgs& a, const uint64_t* v, uint64_t valid) {
  int64_t sz = a.fixed_size;
#pragma unroll
  for (int k = 0; k < K; k++) {
    if (k >= a.ncols || !((valid >> k) & 1)) continue;
    const VarCol& c = a.col[k];
    const int kd = kind_of<M>(c);
    if (kd == kDecimal) {
      sz += 16;
    } else if (kd == kBytes || kd == kListFixed) {
      const int64_t n = static_cast<int64_t>(static_cast<int32_t>(v[k] >> 32)) - static_cast<int32_t>(v[k]);
      sz += kd == kBytes ? rnd8(n) : 8 + bm_bytes(n) + rnd8(n * (c.width == 0 ? 1 : c.width));
    }
  }
  return sz;
}

// Per-row inputs of row r, every column: K independent loads (values, offset pairs, validity).
template <int K, int M>
__device__ __forceinline__ void reg_load_meta(const VarArgs& a, int64_t r, uint64_t* v, uint64_t& valid) {
  valid = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    v[k] = 0;
    if (k >= a.ncols) continue;
    const VarCol& c = a.col[k];
    const bool ok = !c.validity || bit_at_g(c.validity, r);
    valid |= static_cast<uint64_t>(ok) << k;
    uint64_t x = 0;
    switch (kind_of<M>(c)) {
      case kFixed: x = load_fixed(c.values, r, c.width); break;
      case kBool: x = bit_at_g(c.values, r); break;
      case kBytes:
      case kListFixed:
        x = static_cast<uint32_t>(gl(c.offsets)[r]) |
            (static_cast<uint64_t>(static_cast<uint32_t>(gl(c.offsets)[r + 1])) << 32);
        break;
      default: break;
    }
    v[k] = x;
  }
}

// tbase == nullptr: rows at the given offs.  tbase != nullptr (fury_row_encode_measured): tbase[b]
// = the exclusive prefix of the tiles' byte totals (measure_tiles + scan); each tile scans its own
// rows' sizes and writes their final offs -- no per-row sizes pass, no prefix-add pass.
template <int K, int M>
__global__ __launch_bounds__(kEncRows) void encode_var_reg(VarArgs a, int64_t* __restrict__ offs,
                                                           uint8_t* __restrict__ rows, int64_t cap,
                                                           const int64_t* __restrict__ tbase) {
  __shared__ __attribute__((aligned(16))) uint64_t img[kRegImg / 8];
  __shared__ int64_t tmp[kEncRows / 64];
  const int tid = threadIdx.x;
  const int R = a.tile_rows;
  const int64_t b = blockIdx.x;
  const int64_t r0 = b * R;
  const int nr = static_cast<int>(min<int64_t>(R, a.nrows - r0));
  const bool live = tid < nr;
  const int64_t r = live ? r0 + tid : r0;
  // per-row inputs of every column: one batch of independent loads
  uint64_t v[K];
  uint64_t valid;
  reg_load_meta<K, M>(a, r, v, valid);
  int64_t base, bytes, ex, sz;
  if (tbase) {
    sz = live ? reg_row_size<K, M>(a, v, valid) : 0;
    base = tbase[b];
    ex = block_excl_scan<kEncRows>(sz, &bytes, tmp);
    if (live) offs[r] = base + ex;
    if (r0 + nr == a.nrows && tid == nr - 1) offs[a.nrows] = base + ex + sz;
  } else {
    base = offs[r0];
    bytes = offs[r0 + nr] - base;
    ex = offs[r] - base;
    sz = offs[r + 1] - offs[r];
  }
  const int64_t room = max<int64_t>(0, min<int64_t>(bytes, cap - base));
  if (bytes <= kRegImg) {
    // (a.skip, diagnostics: 1 no string bytes, 2 no row build, 4 no store)
    if (live && !(a.skip & 2)) reg_build_row<K, M>(a, r, v, (a.skip & 1) ? 0 : valid, img + (ex >> 3));
    lds_barrier();   // (LDS only: the offsets' stores need not land first)
    if (!(a.skip & 4)) store_image(rows + base, reinterpret_cast<const uint8_t*>(img), room);
  } else if (live) {        // oversized tile: rows straight to HBM (whole rows below the capacity)
    if (ex + sz <= room)
      reg_build_row<K, M>(a, r, v, valid, reinterpret_cast<uint64_t*>(rows + base + ex));
  }
}

#endif  // FURY_VAR_ENC

// ---- measure: row sizes (writerIndex growth of toRow) and their exclusive scan.  Each thread
// sizes 4 consecutive rows (one validity nibble and 5 consecutive offsets per column), so a
// 256-thread workgroup covers 1,024 rows and writes their group-relative exclusive offsets and its
// total; a device scan of the (few) group totals and one add pass finish the scan.  (A single
// pass with a decoupled look-back was measured slower: the ticket atomic that orders the
// workgroups serialises at this workgroup count.)
constexpr int kMeasRows = 4;                                   // rows per thread
constexpr int kMeasTile = kThreads * kMeasRows;                // rows per workgroup

__device__ __forceinline__ int64_t row_size_of(const VarArgs& a, int64_t r) {
  int64_t sz = a.fixed_size;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (c.kind < kBytes) continue;
    if (c.validity && !bit_at(c.validity, r)) continue;          // null: setNullAt only
    if (c.kind == kDecimal) {
      sz += 16;
      continue;
    }
    const int64_t n = c.offsets[r + 1] - c.offsets[r];
    if (c.kind == kBytes) sz += rnd8(n);
    else sz += 8 + bm_bytes(n) + rnd8(n * (c.width == 0 ? 1 : c.width));
  }
  return sz;
}

#ifdef FURY_VAR_ENC
// Byte totals of encode tiles of R rows (R a multiple of 64, <= 256): one wave per tile, each lane
// sizing R / 64 consecutive rows from one run of offsets and one or two validity bytes per column
// (fury_row_encode_measured; the measure_kernel pattern, without the per-row output).
__global__ __launch_bounds__(kThreads) void measure_tiles(VarArgs a, int64_t* __restrict__ tsum,
                                                          int R, int64_t nt) {
  const int lane = threadIdx.x & 63;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6);
  if (t >= nt) return;
  const int q = R >> 6;                               // rows per lane, 1..4
  const int64_t r = t * R + static_cast<int64_t>(lane) * q;
  int64_t s = 0;
  if (r + q <= a.nrows) {
    s = static_cast<int64_t>(q) * a.fixed_size;
    for (int k = 0; k < a.ncols; k++) {
      CVarCol& c = vc(a, k);
      if (c.kind < kBytes) continue;
      uint32_t vb = 0xffu;
      if (c.validity) {
        const int sh = static_cast<int>(r & 7);
        vb = c.validity[r >> 3];
        if (sh + q > 8) vb |= static_cast<uint32_t>(c.validity[(r >> 3) + 1]) << 8;
        vb >>= sh;
      }
      if (c.kind == kDecimal) {
        s += 16 * __builtin_popcount(vb & ((1u << q) - 1));
        continue;
      }
      int32_t o[5];
#pragma unroll
      for (int j = 0; j < 5; j++) o[j] = j <= q ? c.offsets[r + j] : 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if (j >= q || !((vb >> j) & 1)) continue;
        const int64_t n = o[j + 1] - o[j];
        s += c.kind == kBytes ? rnd8(n) : 8 + bm_bytes(n) + rnd8(n * (c.width == 0 ? 1 : c.width));
      }
    }
  } else {
    for (int j = 0; j < q; j++)
      if (r + j < a.nrows) s += row_size_of(a, r + j);
  }
  s = wave_sum(s);
  if (lane == 0) tsum[t] = s;
}
#endif  // FURY_VAR_ENC

#ifdef FURY_VAR_MAIN
__global__ __launch_bounds__(kThreads) void measure_kernel(VarArgs a, int64_t* __restrict__ offs,
                                                           int64_t* __restrict__ gsum) {
  __shared__ int64_t tmp[kThreads / 64];
  const int64_t b = blockIdx.x;
  const int64_t r = b * kMeasTile + kMeasRows * threadIdx.x;   // first of this thread's rows
  int64_t sz[kMeasRows];
  if (r + kMeasRows <= a.nrows) {                 // whole quad: vector-friendly straight line
#pragma unroll
    for (int j = 0; j < kMeasRows; j++) sz[j] = a.fixed_size;
    for (int k = 0; k < a.ncols; k++) {
      CVarCol& c = vc(a, k);
      if (c.kind < kBytes) continue;
      const uint32_t vb = c.validity ? (c.validity[r >> 3] >> (r & 7)) : 0xffu;
      if (c.kind == kDecimal) {
#pragma unroll
        for (int j = 0; j < kMeasRows; j++) sz[j] += ((vb >> j) & 1) ? 16 : 0;
        continue;
      }
      int32_t o[kMeasRows + 1];
#pragma unroll
      for (int j = 0; j <= kMeasRows; j++) o[j] = c.offsets[r + j];
#pragma unroll
      for (int j = 0; j < kMeasRows; j++) {
        const int64_t n = o[j + 1] - o[j];
        const int64_t add = c.kind == kBytes ? rnd8(n)
                                             : 8 + bm_bytes(n) + rnd8(n * (c.width == 0 ? 1 : c.width));
        sz[j] += ((vb >> j) & 1) ? add : 0;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kMeasRows; j++) sz[j] = r + j < a.nrows ? row_size_of(a, r + j) : 0;
  }
  int64_t loc[kMeasRows], run = 0;
#pragma unroll
  for (int j = 0; j < kMeasRows; j++) {
    loc[j] = run;
    run += sz[j];
  }
  int64_t total;
  const int64_t ex = block_excl_scan(run, &total, tmp);
#pragma unroll
  for (int j = 0; j < kMeasRows; j++)
    if (r + j < a.nrows) offs[r + j] = ex + loc[j];
  if (threadIdx.x == 0) gsum[b] = total;
}
#endif  // FURY_VAR_MAIN

// offs[r] += prefix of r's measure group; offs[n] = total.
#ifdef FURY_VAR_MAIN
__global__ __launch_bounds__(kThreads) void add_group_prefix(int64_t* __restrict__ offs, int64_t n,
                                                             const int64_t* __restrict__ prefix,
                                                             const int64_t* __restrict__ total) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (r < n) offs[r] += prefix[r / kMeasTile];
  if (r == n - 1) offs[n] = *total;
}
#endif  // FURY_VAR_MAIN

// --- decode side -------------------------------------------------------------------------------

// The count a variable-length value contributes to its Arrow column -- STRING / BINARY: the
// unpadded size (int)slot; LIST: numElements, (int) of the array's first 8 bytes
// (BinaryArray.pointTo, BinaryArray.java:69-78); DECIMAL and the rest: 0 -- for the slot of a
// non-null field of the row at absolute byte `base`.  A value any of whose bytes lie outside the
// batch [0, total) (string bytes, DECIMAL's 16, an array's header, null bits and elements), or with
// a negative size / count, sets *bad and counts 0 (span_ok, kernels.h).  Every decode kernel and
// the look-back's help (tile_count) count through this one function, so a helped aggregate equals
// the one its tile publishes.
__device__ __forceinline__ int64_t slot_count(int kind, int width, uint64_t slot, int64_t base,
                                              const uint8_t* rows, int64_t total, bool* bad) {
  const int64_t p = base + static_cast<int32_t>(slot >> 32);
  switch (kind) {
    case kBytes: {
      const int64_t n = static_cast<int32_t>(slot);
      if (span_ok(p, n, total)) return n;
      *bad = true;
      return 0;
    }
    case kDecimal:
      if (!span_ok(p, 16, total)) *bad = true;
      return 0;
    case kListFixed: {
      if (!span_ok(p, 8, total)) {
        *bad = true;
        return 0;
      }
      const int64_t n = static_cast<int32_t>(*gl(reinterpret_cast<const int64_t*>(rows + p)));
      const int64_t ew = width == 0 ? 1 : width;
      if (n >= 0 && span_ok(p, 8 + bm_bytes(n) + n * ew, total)) return n;
      *bad = true;
      return 0;
    }
    default:
      return 0;
  }
}

// Element count of a LIST whose array (header value n) starts at absolute byte p, bounds-checked as
// slot_count does.
__device__ __forceinline__ int64_t list_count(int64_t n, int width, int64_t p, int64_t total,
                                              bool* bad) {
  const int64_t ew = width == 0 ? 1 : width;
  if (n >= 0 && span_ok(p, 8 + bm_bytes(n) + n * ew, total)) return n;
  *bad = true;
  return 0;
}

// The row at absolute byte `base` is inside the batch: its null bitmap and slots can be read.
__device__ __forceinline__ bool row_ok(int64_t base, int fixed_size, int64_t total) {
  return span_ok(base, fixed_size, total);
}

// Null-or-bad test + count of field k of the row whose header bytes are at `hdr` (LDS or HBM) and
// which starts at absolute byte `base`.  Returns the count; *null = null field or bad value.
template <class Col>
__device__ __forceinline__ int64_t field_count(const Col& c, int k, const uint8_t* hdr,
                                               int bitmap_bytes, int64_t base, const uint8_t* rows,
                                               int64_t total, bool* null, bool* bad) {
  *bad = false;
  *null = (hdr[k >> 3] >> (k & 7)) & 1;
  if (*null || c.kind < kBytes) return 0;
  const uint64_t slot = *reinterpret_cast<const uint64_t*>(hdr + bitmap_bytes + 8 * k);
  const int64_t n = slot_count(c.kind, c.width, slot, base, rows, total, bad);
  if (*bad) *null = true;
  return n;
}

#ifdef FURY_VAR_MAIN
__global__ __launch_bounds__(kThreads) void decode_measure_kernel(VarArgs a,
                                                                  const uint8_t* __restrict__ rows,
                                                                  const int64_t* __restrict__ offs,
                                                                  int64_t* __restrict__ sums,
                                                                  int64_t nb) {
  __shared__ int64_t tmp[kThreads / 64];
  __shared__ __attribute__((aligned(16))) uint8_t stage[kDecodeStage];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kThreads;
  const int64_t nr = min<int64_t>(kThreads, a.nrows - r0);
  const int64_t total = offs[a.nrows];
  const int64_t rbeg = offs[r0];
  const int64_t bytes = offs[r0 + nr] - rbeg;
  const int64_t r = r0 + threadIdx.x;
  // stage the group's contiguous row range (LDS-DMA, 16-B pieces) so the per-row slot reads
  // below hit LDS instead of scattered HBM lines (only a range inside the batch)
  const bool staged = bytes >= 0 && bytes + 32 <= kDecodeStage && span_ok(rbeg, bytes, total);
  uint32_t d0 = 0;
  if (staged) {
    uint32_t at = 0;
    d0 = stage_range<kThreads>(stage, at, rows + rbeg, rows + rbeg + bytes);
    __syncthreads();
  }
  const int64_t base = r < a.nrows ? offs[r] : 0;
  const bool rok = r < a.nrows && row_ok(base, a.fixed_size, total);
  if (r < a.nrows && !rok) raise_oob(a.err, r);
  // a row header inside the staged range is read from LDS
  const bool in_stage = staged && rok && base >= rbeg && base + a.fixed_size <= rbeg + bytes;
  const uint8_t* row = rok ? (in_stage ? stage + d0 + (base - rbeg) : rows + base) : nullptr;
  int seq = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (c.kind != kBytes && c.kind != kListFixed) continue;
    bool nul = false, bad = false;
    const int64_t cnt = row ? field_count(c, k, row, a.bitmap_bytes, base, rows, total, &nul, &bad) : 0;
    if (bad) raise_oob(a.err, r);
    int64_t total;
    const int64_t ex = block_excl_scan(cnt, &total, tmp);
    if (row) c.offsets[r] = static_cast<int32_t>(ex);
    if (threadIdx.x == 0) sums[seq * nb + blockIdx.x] = total;
    seq++;
  }
}
#endif  // FURY_VAR_MAIN

#ifdef FURY_VAR_MAIN
__global__ __launch_bounds__(kThreads) void decode_measure_fix(VarArgs a,
                                                               const int64_t* __restrict__ sums,
                                                               const int64_t* __restrict__ totals,
                                                               int64_t nb) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  int seq = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (c.kind != kBytes && c.kind != kListFixed) continue;
    if (r < a.nrows) c.offsets[r] += static_cast<int32_t>(sums[seq * nb + blockIdx.x]);
    if (r == a.nrows - 1) c.offsets[a.nrows] = static_cast<int32_t>(totals[seq]);
    seq++;
  }
}
#endif  // FURY_VAR_MAIN

// Byte i (0 <= i < len) of an 8-byte-aligned source, read as whole aligned words.
__device__ __forceinline__ uint32_t src_byte(const uint8_t* src, int64_t i) {
  const uint64_t w = reinterpret_cast<const uint64_t*>(src)[i >> 3];
  return static_cast<uint32_t>((w >> (8 * (i & 7))) & 0xff);
}

// Writes src[0, len) (8-byte-aligned source: a row's var section) to dst + q (any alignment).
// 32-bit words wholly inside the destination range are written whole; the partial words at the
// two ends are written byte by byte, so neighbouring strings (other threads) are never touched
// and no atomics or pre-zeroing are needed (byte stores are masked in LDS and in HBM).
__device__ __forceinline__ void put_bytes(uint8_t* dst, int64_t q, const uint8_t* src, int64_t len) {
  if (len <= 0) return;
  const int64_t end = q + len;
  const int64_t w0 = (q + 3) >> 2;                 // first whole word
  const int64_t w1 = end >> 2;                     // one past the last whole word
  if (w0 >= w1) {
    for (int64_t i = 0; i < len; i++) dst[q + i] = static_cast<uint8_t>(src_byte(src, i));
    return;
  }
  for (int64_t i = q; i < 4 * w0; i++) dst[i] = static_cast<uint8_t>(src_byte(src, i - q));
  const int64_t d = 4 * w0 - q;                    // source index of the first whole word
  const uint64_t* s64 = reinterpret_cast<const uint64_t*>(src);
  uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
  for (int64_t w = w0; w < w1; w++) {
    const int64_t si = d + 4 * (w - w0);           // 4 source bytes [si, si + 4)
    const int64_t j = si >> 3;
    const int o = static_cast<int>(si & 7);
    uint64_t x = s64[j] >> (8 * o);
    if (o > 4) x |= s64[j + 1] << (64 - 8 * o);
    d32[w] = static_cast<uint32_t>(x);
  }
  for (int64_t i = 4 * w1; i < end; i++) dst[i] = static_cast<uint8_t>(src_byte(src, i - q));
}

template <bool kToGlobal>
__device__ __forceinline__ void copy_bytes_range(uint8_t* g, const uint8_t* l, int64_t p0, int64_t p1,
                                                 int64_t a0) {
  // [p0, p1) of g <- l[p - a0]: unaligned ends byte by byte, aligned middle 16 B per lane.
  const int64_t m0 = min<int64_t>((p0 + 15) & ~int64_t(15), p1);
  const int64_t m1 = max<int64_t>(p1 & ~int64_t(15), m0);
  for (int64_t i = p0 + threadIdx.x; i < m0; i += kThreads) g[i] = l[i - a0];
  for (int64_t i = m1 + threadIdx.x; i < p1; i += kThreads) g[i] = l[i - a0];
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  for (int64_t i = m0 + 16 * threadIdx.x; i < m1; i += 16 * kThreads)
    __builtin_nontemporal_store(*reinterpret_cast<const v4*>(l + (i - a0)),
                                reinterpret_cast<v4*>(g + i));
}

template <class Col>
__device__ __forceinline__ bool is_seq(const Col& c) {
  return c.kind == kBytes || c.kind == kListFixed;
}

// ---- row-staged decode (schemas of <= kRegCols fields) ---------------------------------------
// One 512-thread workgroup decodes a tile of up to 512 rows (thread = row; a.tile_rows rows, from
// dec_tile_plan).  The tile's contiguous row bytes arrive in LDS by coalesced LDS-DMA pieces
// (zeroing the output images meanwhile); each thread reads its row's null word and slots from
// there into registers.  STRING/BINARY/LIST counts are scanned in the workgroup (DPP wave scans,
// one barrier) and chained across workgroups by a decoupled look-back in launch order.  Each
// variable-length column's Arrow range for the tile is assembled in LDS (string bytes OR-ed at
// byte offsets into the zeroed image -- rows keep strings 8-byte aligned, so every source word is
// one aligned read; list elements at their element slots; validity / bool bits OR-ed into a bit
// image) and leaves with 16-B stores, byte-exact at the two ends and with atomic and/or on bitmap
// words shared with the neighbouring tiles; fixed-width fields leave as coalesced column stores
// while predecessors publish.
constexpr int kDecImg = 24 * 1024;
#ifndef FURY_DEC_THREADS
#define FURY_DEC_THREADS 512           // (-D: A/B builds of the tile shape, scripts/r06_dec256.sh)
#endif
constexpr int kDecThreads = FURY_DEC_THREADS;   // register-staged decode: threads (and maximum rows) per tile


// Count (string bytes / list elements) of column k summed over the rows of tile j, by one wave,
// straight from the rows: the aggregate tile j publishes, for a look-back that stopped waiting.
// Same counts (slot_count) and the same 32-bit truncation as the published aggregates.
template <int NT>
__device__ int64_t tile_count(const VarArgs& a, int k, const uint8_t* rows, const int64_t* offs,
                              int64_t j, int64_t tr = NT) {
  const int lane = threadIdx.x & 63;
  CVarCol& c = vc(a, k);
  const int64_t total = gl(offs)[a.nrows];
  int64_t sum = 0;
  const int64_t i1 = min<int64_t>((j + 1) * tr, a.nrows);
  for (int64_t i = j * tr + lane; i < i1; i += 64) {
    const int64_t base = gl(offs)[i];
    if (!row_ok(base, a.fixed_size, total)) continue;
    const uint8_t* row = rows + base;
    if ((gl(row)[k >> 3] >> (k & 7)) & 1) continue;
    const uint64_t slot = *gl(reinterpret_cast<const uint64_t*>(row + a.bitmap_bytes + 8 * k));
    bool bad = false;
    sum += slot_count(c.kind, c.width, slot, base, rows, total, &bad);
  }
  return static_cast<uint32_t>(wave_sum(sum));
}

// look_back_bounded for blockIdx-ordered tiles: when the nearest unpublished predecessor inside
// the window has not published for kHelpSpins polls, the wave computes that tile's aggregate
// itself (tile_count) and goes on, so the look-back finishes whatever the dispatch order.  The
// helped values are exactly what the tile publishes later.  Tuning "lookback_help" 1 helps at once
// (exercises this path in the tests; results are identical).
constexpr uint32_t kHelpSpins = 1u << 14;
// Column index of the q-th STRING / BINARY / LIST column (the kernels' sequence numbering).
__device__ __forceinline__ int seq_col(const VarArgs& a, int q) {
  int seq = 0;
  for (int k = 0; k < a.ncols; k++) {
    if (!is_seq(vc(a, k))) continue;
    if (seq++ == q) return k;
  }
  return 0;
}

template <int NT>
__device__ int64_t look_back_help(const VarArgs& a, int k, const uint8_t* rows,
                                  const int64_t* offs, const uint64_t* status, int64_t b, int nseq,
                                  int q, uint32_t* err, int64_t tr = NT) {
  const int lane = threadIdx.x & 63;
  const uint32_t limit = (a.help_now & 1) ? 0u : kHelpSpins;
  int64_t excl = 0;
  for (int64_t j = b - 1;; j -= 64) {
    const int64_t idx = j - lane;
    uint64_t v = idx >= 0 ? ld_status(status + idx * nseq + q) : kInc;
    uint64_t inc;
    int stop;
    uint32_t spins = 0, helped = 0;
    for (;;) {
      inc = __ballot((v >> 62) == 2);
      stop = inc ? __builtin_ctzll(inc) : 63;
      const uint64_t upto = stop == 63 ? ~0ull : ((2ull << stop) - 1);
      const uint64_t pend = __ballot((v >> 62) == 0) & upto;
      if (pend == 0) break;
      if (spins >= limit) {                      // help the nearest silent predecessor
        const int l = __builtin_ctzll(pend);
        const int64_t agg = tile_count<NT>(a, k, rows, offs, j - l, tr);
        if (lane == l) v = kAgg | static_cast<uint64_t>(agg);
        spins = 0;
        if (++helped > 64 && err) {              // cannot happen: at most 64 lanes to help
          if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return 0;
        }
        continue;
      }
      ++spins;
      __builtin_amdgcn_s_sleep(1);
      if ((v >> 62) == 0 && lane <= stop) v = ld_status(status + idx * nseq + q);
    }
    excl += wave_sum(lane <= stop ? static_cast<int64_t>(v & kValMask) : 0);
    if (inc) return excl;
  }
}

// Stores image bytes img[0, n) to g[0, n) (g any alignment, img 16-aligned LDS with >= 16 bytes
// of readable padding past n): byte stores up to g's 16-byte boundary, then 16-B non-temporal
// stores whose data is funnel-shifted out of aligned image words, then the byte tail.
template <int NT = kThreads>
__device__ __forceinline__ void store_shifted(uint8_t* g, const uint8_t* img, int64_t n) {
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  if (n <= 0) return;
  const int64_t head = min<int64_t>(n, (16 - (reinterpret_cast<uintptr_t>(g) & 15)) & 15);
  const int64_t body = (n - head) >> 4;
  const int64_t t0 = head + 16 * body;
  if (threadIdx.x < head) gl(g)[threadIdx.x] = img[threadIdx.x];
  if (threadIdx.x < n - t0) gl(g)[t0 + threadIdx.x] = img[t0 + threadIdx.x];
  const uint64_t* i64 = reinterpret_cast<const uint64_t*>(img);
  const int sh = static_cast<int>(head & 7) * 8;
  for (int64_t m = threadIdx.x; m < body; m += NT) {
    const int64_t off = head + 16 * m;
    const int64_t q = off >> 3;
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

// Stores a bit image (image bit i = global bit gbit0 + i, >= 1 word of padding) to the global
// bitmap bits [gbit0, gbit0 + n): whole words plainly, the words shared with neighbouring tiles
// with atomic and/or of exactly these bits.
template <int NT = kThreads>
__device__ __forceinline__ void store_bits_shifted(uint8_t* bits, const uint32_t* img, int64_t gbit0,
                                                   int64_t n) {
  if (n <= 0) return;
  const int64_t end = gbit0 + n;
  const int64_t w0 = gbit0 >> 5, w1 = (end + 31) >> 5;
  uint32_t* g = reinterpret_cast<uint32_t*>(bits);
  for (int64_t w = w0 + threadIdx.x; w < w1; w += NT) {
    const int64_t i0 = 32 * w - gbit0;
    uint32_t x;
    if (i0 < 0) {
      x = img[0] << (-i0);
    } else {
      const int64_t q = i0 >> 5;
      const int s = static_cast<int>(i0 & 31);
      x = s ? (img[q] >> s) | (img[q + 1] << (32 - s)) : img[q];
    }
    uint32_t m = ~0u;
    if (w == w0) m &= ~0u << (gbit0 & 31);
    if (w == w1 - 1 && (end & 31)) m &= (1u << (end & 31)) - 1;
    if (m == ~0u) {
      gl(g)[w] = x;
    } else {
      atomicAnd(g + w, ~m);
      atomicOr(g + w, x & m);
    }
  }
}

#ifdef FURY_VAR_DEC
// (K <= 4: at most 128 VGPRs, so two 512-thread workgroups share a CU -- the LDS plan assumes two)
template <int K, int M, bool PIPE = false>
__global__ __launch_bounds__(kDecThreads) __attribute__((amdgpu_waves_per_eu(K <= 4 ? 4 : 1))) void decode_var_reg(VarArgs a, const uint8_t* __restrict__ rows,
                                                              const int64_t* __restrict__ offs,
                                                              uint64_t* __restrict__ status,
                                                              uint32_t img_cap, uint32_t stage_cap) {
  constexpr int NT = kDecThreads;
  // dynamic LDS: [output images: img_cap][staged row bytes: stage_cap], both sized per launch
  // (dec_tile_plan) so that two workgroups fit a CU
  extern __shared__ __attribute__((aligned(16))) uint64_t oimg[];
  __shared__ uint32_t wtot[K][NT / 64];
  __shared__ int64_t sbase[K];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // Tile = blockIdx.  A ticket (tiles numbered in start order) made every look-back wait end by
  // construction, but its one device-scope atomic per tile serialises at the cross-XCD coherence
  // point (~12 ns each: the C4 decode's loads alone took 202 us with it, 83 us without).  Instead
  // the look-back helps itself (look_back_help): a predecessor that has published nothing for a
  // long time -- not dispatched yet, under any dispatch order -- has its aggregate computed from
  // its rows by the waiting wave, so no wait depends on a workgroup that is not running.
  const int64_t TR = a.tile_rows;                 // rows per tile (<= NT, a multiple of 64)
  const int64_t nb = (a.nrows + TR - 1) / TR;     // tiles
  constexpr int NW = NT / 64;
  const int64_t total = offs[a.nrows];            // the batch: every read stays in [0, total)
  // The tile's row bytes [offs[r0], offs[r0 + nr]) (up to stage_cap of them) are staged in LDS by
  // coalesced LDS-DMA pieces; header, string and list reads of rows inside the staged range read
  // LDS, the rest HBM.  (Per-lane row reads from HBM touched one cache line per lane per
  // instruction and fetched every line from L2 again for the header and for each value: 40M L1
  // misses vs 11.5M staged on 10M mixed rows, TCP_TCC_READ_REQ.)
  // PIPE (round 6, tuning "var_dec_pipe"; its own instances -- the loop costs the one-tile kernel
  // 30-50 VGPRs): a persistent grid whose workgroups take tiles blockIdx, + gridDim, ... with TWO
  // stages: the next tile's LDS-DMA is issued once the current
  // tile's prefixes are resolved (its last global loads), so it lands during the offsets and the
  // image store-out (vmcnt is in order: issued earlier, every wait on a load of the tile would wait
  // for it too).
  uint8_t* const stg0 = reinterpret_cast<uint8_t*>(oimg) + img_cap;
  uint8_t* const stg1 = stg0 + (PIPE ? stage_cap : 0u);
  auto stage_tile = [&](int64_t t, uint8_t* sp, uintptr_t* lo, uintptr_t* hi) {
    const int64_t t0 = t * TR;
    const int64_t tn = min<int64_t>(TR, a.nrows - t0);
    const int64_t tt = max<int64_t>(total, 0);
    const int64_t g0 = min<int64_t>(max<int64_t>(offs[t0], 0), tt);
    const int64_t g1 = min<int64_t>(max<int64_t>(offs[t0 + tn], g0), tt);
    *lo = reinterpret_cast<uintptr_t>(rows + g0) & ~uintptr_t(15);
    *hi = min<uintptr_t>(reinterpret_cast<uintptr_t>(rows + g1), *lo + stage_cap);
    uint32_t at = 0;
    if (*hi > *lo)
      stage_range<NT>(sp, at, reinterpret_cast<const uint8_t*>(*lo), reinterpret_cast<const uint8_t*>(*hi));
    else
      *hi = *lo;
  };
  auto zero_images = [&]() {
    for (uint32_t i = 16 * tid; i < img_cap; i += 16 * NT)
      *reinterpret_cast<__attribute__((ext_vector_type(4))) uint32_t*>(reinterpret_cast<uint8_t*>(oimg) + i) = 0;
  };
  uintptr_t nx_lo = 0, nx_hi = 0;                 // the next tile's staged range (dec_pipe)
  int64_t b = static_cast<int64_t>(blockIdx.x);
  for (int it = 0;; it++) {
  uint8_t* const stg = (it & 1) ? stg1 : stg0;
  const int64_t r0 = b * TR;
  const int nr = static_cast<int>(min<int64_t>(TR, a.nrows - r0));
  const bool live = tid < nr;
  const int64_t r = live ? r0 + tid : r0;
  uintptr_t sa_lo = nx_lo, sa_hi = nx_hi;         // absolute addresses held by stg
  const int64_t base0 = offs[r];                  // issued before the staging (its own round trip)
  if (it == 0) {
    stage_tile(b, stg, &sa_lo, &sa_hi);
    zero_images();                                // (while the pieces are in flight)
    __syncthreads();
  }
  const int64_t lim = total - a.fixed_size;       // last byte a row header may start at
  // the header is read at a clamped (always readable) start; a row outside the batch decodes as
  // all-null and is reported
  const int64_t base = min<int64_t>(max<int64_t>(base0, 0), max<int64_t>(lim, 0));
  const bool rok = lim >= 0 && base == base0;
  const uint8_t* row = rows + base;
  // null word + slots: the 16-byte aligned blocks covering them, from the stage (or HBM); rows
  // are only 8-aligned, the words are selected afterwards.  Blocks past the header's last word
  // are not read (the last block may extend 8 bytes past the header: inside the same 16-byte
  // block, never used).
  using u64x2 = __attribute__((ext_vector_type(2))) unsigned long long;
  constexpr int kNch = (K + 3) / 2;
  const uintptr_t ra = reinterpret_cast<uintptr_t>(row);
  const int mis = static_cast<int>((ra >> 3) & 1);
  // K may exceed the schema's field count (instances for K in {2, 4, 6, 8, 12, 16}): the columns
  // past a.ncols are zeroed records (no outputs, null) and their slots are not loaded
  const int need = lim >= 0 ? (mis + a.ncols + 2) / 2 : 0;
  const auto blk = gl(reinterpret_cast<const u64x2*>(ra & ~uintptr_t(15)));
  uint64_t hw[2 * kNch];
  const bool hin = ra >= sa_lo && ra + a.fixed_size <= sa_hi && !(ra & 7);
  if (hin) {
    const u64x2* lb = reinterpret_cast<const u64x2*>(stg + ((ra & ~uintptr_t(15)) - sa_lo));
#pragma unroll
    for (int c = 0; c < kNch; c++) {
      u64x2 x = {0, 0};
      if (c < need) x = lb[c];
      hw[2 * c] = x.x;
      hw[2 * c + 1] = x.y;
    }
  } else {
#pragma unroll
    for (int c = 0; c < kNch; c++) {
      u64x2 x = {0, 0};
      if (c < need) x = blk[c];
      hw[2 * c] = x.x;
      hw[2 * c + 1] = x.y;
    }
  }
  uint64_t nullw = live && rok ? (mis ? hw[1] : hw[0]) : ~0ull;
  nullw |= a.ncols >= 64 ? 0ull : (~0ull << a.ncols);
  uint64_t slot[K];
#pragma unroll
  for (int k = 0; k < K; k++) slot[k] = mis ? hw[k + 2] : hw[k + 1];
  // counts (LIST: the array header's element count), bounds-checked: a value outside the batch
  // decodes as null and is reported (slot_count / list_count)
  uint32_t cnt[K];
  uint64_t badw = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const VarCol& c = a.col[k];
    const int kd = kind_of<M>(c);
    cnt[k] = 0;
    if (((nullw >> k) & 1) || kd < kBytes) continue;
    bool bad = false;
    const int64_t p = base + static_cast<int32_t>(slot[k] >> 32);
    const uintptr_t pa = reinterpret_cast<uintptr_t>(rows + p);
    if (kd == kListFixed && span_ok(p, 8, total) && pa >= sa_lo && pa + 8 <= sa_hi && !(pa & 7))
      cnt[k] = static_cast<uint32_t>(list_count(
          static_cast<int32_t>(*reinterpret_cast<const int64_t*>(stg + (pa - sa_lo))), c.width, p,
          total, &bad));
    else
      cnt[k] = static_cast<uint32_t>(slot_count(kd, c.width, slot[k], base, rows, total, &bad));
    badw |= static_cast<uint64_t>(bad) << k;
  }
  nullw |= badw;
  if (live && (badw || !rok)) raise_oob(a.err, r);
  // in-tile exclusive scans of the STRING / BINARY / LIST counts (tile totals < 2^31: Arrow
  // offsets are int32): 32-bit DPP wave scans, wave totals exchanged through LDS behind ONE barrier
  uint32_t ex[K], tot[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    ex[k] = tot[k] = 0;
    if (!seq_kind(kind_of<M>(a.col[k]))) continue;
    const uint32_t inc = wave_scan_u32(cnt[k]);
    if (lane == 63) wtot[k][wave] = inc;
    ex[k] = inc - cnt[k];
  }
  lds_barrier();   // (LDS only)
#pragma unroll
  for (int k = 0; k < K; k++) {
    if (!seq_kind(kind_of<M>(a.col[k]))) continue;
    uint32_t pre = 0, t = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
      const uint32_t v = wtot[k][w];
      pre += w < wave ? v : 0;
      t += v;
    }
    ex[k] += pre;
    tot[k] = t;
  }
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < K; k++)
      if (seq_kind(kind_of<M>(a.col[k])))
        st_status(status + b * K + k, (b == 0 ? kInc : kAgg) | static_cast<uint64_t>(tot[k]));
  }
  // tile-relative LDS images of every variable-length column (image byte / bit i = the tile's
  // i-th output byte / element); laid out from the tile totals alone, so the rows are scattered
  // into them while the predecessors' prefixes are still being resolved
  uint32_t img_at[K];
  uint32_t used = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const VarCol& c = a.col[k];
    const int kd = kind_of<M>(c);
    img_at[k] = kNone;
    if (!seq_kind(kd) || !c.values || tot[k] == 0) continue;
    int64_t need;
    if (kd == kBytes) need = r16(tot[k] + 16);
    else if (c.width == 0) need = r16((((tot[k] + 31) >> 5) + 1) * 4);
    else need = r16(int64_t(tot[k]) * c.width + 16);
    if (kd == kListFixed && c.elem_validity) need += r16((((tot[k] + 31) >> 5) + 1) * 4);
    if (used + need <= img_cap) {
      img_at[k] = used;
      used += static_cast<uint32_t>(need);
    }
  }
  // (the images were zeroed while the rows were staged)
  // (a.skip, diagnostics -- outputs WRONG, timing only: 16 no image assembly, 32 no fixed-width /
  // validity stores, 64 no look-back, 128 no image store-out)
#pragma unroll
  for (int k = 0; k < K; k++) {
    const VarCol& c = a.col[k];
    if (img_at[k] == kNone || !live || cnt[k] == 0 || (a.skip & 16)) continue;
    if (static_cast<uint64_t>(ex[k]) + cnt[k] > tot[k]) {   // the tile's 32-bit total wrapped
      raise_oob(a.err, r);
      continue;
    }
    const uint8_t* src = row + static_cast<int32_t>(slot[k] >> 32);
    uint8_t* im = reinterpret_cast<uint8_t*>(oimg) + img_at[k];
    // (values are read from the stage when wholly there, else from HBM: the generic lambdas are
    // instantiated once per address space)
    const uintptr_t sa = reinterpret_cast<uintptr_t>(src);
    if (bytes_seq<M>(c)) {
      const int64_t len = cnt[k];
      const int64_t d = ex[k];
      uint64_t* iw = reinterpret_cast<uint64_t*>(im) + (d >> 3);
      const int sh = static_cast<int>(d & 7) * 8;
      const int64_t nw = (len + 7) >> 3;
      auto or_words = [&](auto s64) {
        for (int64_t j0 = 0; j0 < nw; j0 += 4) {
          uint64_t w[4];
#pragma unroll
          for (int u = 0; u < 4; u++) w[u] = j0 + u < nw ? s64[j0 + u] : 0;
#pragma unroll
          for (int u = 0; u < 4; u++) {
            const int64_t j = j0 + u;
            if (j >= nw) break;
            uint64_t x = w[u];
            const int64_t rem = len - 8 * j;
            if (rem < 8) x &= (~0ull) >> (8 * (8 - rem));
            atomicOr(reinterpret_cast<unsigned long long*>(iw + j), x << sh);
            if (sh && (x >> (64 - sh))) atomicOr(reinterpret_cast<unsigned long long*>(iw + j + 1), x >> (64 - sh));
          }
        }
      };
      if (sa >= sa_lo && sa + 8 * nw <= sa_hi && !(sa & 7))
        or_words(reinterpret_cast<const uint64_t*>(stg + (sa - sa_lo)));
      else
        or_words(gl(reinterpret_cast<const uint64_t*>(src)));
      continue;
    }
    // LIST of fixed-width elements: values at element slots, bits by OR
    const int64_t n = cnt[k];
    const int ew = c.width == 0 ? 1 : c.width;
    const int64_t vb = c.width == 0 ? r16((((tot[k] + 31) >> 5) + 1) * 4) : r16(int64_t(tot[k]) * c.width + 16);
    uint32_t* bimg = reinterpret_cast<uint32_t*>(im + vb);
    auto put_list = [&](auto arr) {
      const auto bw = cast_as<const uint64_t>(arr + 8);                    // 8-aligned bitmap
      const auto ev = arr + 8 + bm_bytes(n);
      for (int64_t j0 = 0; j0 < n; j0 += 8) {
        const int lim = static_cast<int>(min<int64_t>(8, n - j0));
        const int bsh = static_cast<int>(j0 & 63);
        const uint64_t nulls = bw[j0 >> 6] >> bsh;       // j0 % 8 == 0: the 8 bits share a word
        uint64_t x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          x[u] = 0;
          if (u < lim) {
            switch (ew) {
              case 8: x[u] = cast_as<const uint64_t>(ev)[j0 + u]; break;
              case 4: x[u] = cast_as<const uint32_t>(ev)[j0 + u]; break;
              case 2: x[u] = cast_as<const uint16_t>(ev)[j0 + u]; break;
              default: x[u] = ev[j0 + u]; break;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
          if (u >= lim) break;
          const bool valid = !((nulls >> u) & 1);
          const int64_t e = ex[k] + j0 + u;                     // tile-relative element
          const uint64_t val = valid ? x[u] : 0;
          if (c.width == 8) {
            reinterpret_cast<uint64_t*>(im)[e] = val;
          } else if (c.width == 0) {
            if (val & 0xff) atomicOr(reinterpret_cast<uint32_t*>(im) + (e >> 5), 1u << (e & 31));
          } else if (val) {
            const int64_t bo = e * ew;
            atomicOr(reinterpret_cast<uint32_t*>(im) + (bo >> 2), static_cast<uint32_t>(val << (8 * (bo & 3))));
          }
        }
        if (c.elem_validity) {                     // the chunk's validity bits as one run
          const uint32_t vb8 = static_cast<uint32_t>(~nulls) & ((1u << lim) - 1);
          const int64_t e0 = ex[k] + j0;
          const int s0 = static_cast<int>(e0 & 31);
          if (vb8) {
            atomicOr(bimg + (e0 >> 5), vb8 << s0);
            if (s0 + lim > 32) atomicOr(bimg + (e0 >> 5) + 1, vb8 >> (32 - s0));
          }
        }
      }
    };
    const int64_t abytes = 8 + bm_bytes(n) + n * ew;
    if (sa >= sa_lo && sa + abytes <= sa_hi && !(sa & 7))
      put_list(stg + (sa - sa_lo));
    else
      put_list(gl(src));
  }
  // fixed-width fields, decimals and every field's validity (no dependency on other tiles; stored
  // after the assembly: issued before the scans they slowed the tile, 0.62 vs 0.55 ms on mixed)
  const int64_t rbase = r0 + 64 * wave;
  const int64_t nvalid = r0 + nr - rbase;          // rows of this wave in this tile
  const int nwords = nvalid >= 64 ? 2 : nvalid <= 0 ? 0 : static_cast<int>((nvalid + 31) >> 5);
#pragma unroll
  for (int k = 0; k < K; k++) {
    const VarCol& c = a.col[k];
    const bool isnull = (nullw >> k) & 1;
    if (a.skip & 32) continue;
    if (c.validity) {
      const uint64_t ok = __ballot(live && !isnull);
      if (lane < nwords)
        reinterpret_cast<uint32_t*>(c.validity)[(rbase >> 5) + lane] = static_cast<uint32_t>(ok >> (32 * lane));
    }
    uint8_t* dst = const_cast<uint8_t*>(c.values);
    if (!dst) continue;
    const uint64_t x = isnull ? 0 : slot[k];
    if (kind_of<M>(c) == kFixed) {
      if (live) {
        switch (c.width) {
          case 8: __builtin_nontemporal_store(x, reinterpret_cast<uint64_t*>(dst) + r); break;
          case 4: __builtin_nontemporal_store(static_cast<uint32_t>(x), reinterpret_cast<uint32_t*>(dst) + r); break;
          case 2: reinterpret_cast<uint16_t*>(dst)[r] = static_cast<uint16_t>(x); break;
          default: dst[r] = static_cast<uint8_t>(x); break;
        }
      }
    } else if (kind_of<M>(c) == kBool) {
      const uint64_t bits = __ballot(live && (x & 0xff) != 0);
      if (lane < nwords)
        reinterpret_cast<uint32_t*>(dst)[(rbase >> 5) + lane] = static_cast<uint32_t>(bits >> (32 * lane));
    } else if (kind_of<M>(c) == kDecimal && live) {
      uint64_t lo = 0, hi = 0;
      if (!isnull) {
        const uint64_t* s = reinterpret_cast<const uint64_t*>(row + static_cast<int32_t>(x >> 32));
        lo = s[0];
        hi = s[1];
      }
      uint64_t* d = reinterpret_cast<uint64_t*>(dst + 16 * r);
      d[0] = lo;
      d[1] = hi;
    }
  }
  // prefixes of the variable-length columns: one wave per column (round robin)
  {
    int q = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      if (!seq_kind(kind_of<M>(a.col[k]))) continue;
      if ((q++ % (NT / 64)) != wave) continue;
      const int64_t pre = b == 0 || (a.skip & 64) ? 0 : look_back_help<NT>(a, k, rows, offs, status, b, K, k, a.err, TR);
      if (lane == 0) {
        sbase[k] = pre;
        if (b > 0) st_status(status + b * K + k, kInc | static_cast<uint64_t>(pre + tot[k]));
      }
    }
  }
  const int64_t nxt = b + static_cast<int64_t>(gridDim.x);
  const bool more = PIPE && nxt < nb;
  if (more) stage_tile(nxt, (it & 1) ? stg0 : stg1, &nx_lo, &nx_hi);
  lds_barrier();   // (LDS only: the column / status stores need not land first)
  // Arrow offsets; columns whose range did not fit the image go straight to HBM (rare)
#pragma unroll
  for (int k = 0; k < K; k++) {
    const VarCol& c = a.col[k];
    if (!seq_kind(kind_of<M>(c))) continue;
    const int64_t gb = sbase[k];
    if (live) c.offsets[r] = static_cast<int32_t>(gb + ex[k]);
    if (b == nb - 1 && tid == nr - 1) c.offsets[a.nrows] = static_cast<int32_t>(gb + tot[k]);
    if (img_at[k] != kNone || !c.values || !live || cnt[k] == 0) continue;
    uint8_t* dst = const_cast<uint8_t*>(c.values);
    const int64_t cap = c.capacity;
    const int64_t pos = gb + ex[k];
    const uint8_t* src = row + static_cast<int32_t>(slot[k] >> 32);
    if (bytes_seq<M>(c)) {
      put_bytes(dst, pos, src, max<int64_t>(0, min<int64_t>(cnt[k], cap - pos)));
      continue;
    }
    const int64_t n = cnt[k];
    const int ew = c.width == 0 ? 1 : c.width;
    const uint8_t* ev = src + 8 + bm_bytes(n);
    for (int64_t j = 0; j < n; j++) {
      const int64_t e = pos + j;
      if (e >= cap) break;
      const bool valid = !((src[8 + (j >> 3)] >> (j & 7)) & 1);
      uint64_t x = 0;
      if (valid) {
        switch (ew) {
          case 8: x = reinterpret_cast<const uint64_t*>(ev)[j]; break;
          case 4: x = reinterpret_cast<const uint32_t*>(ev)[j]; break;
          case 2: x = reinterpret_cast<const uint16_t*>(ev)[j]; break;
          default: x = ev[j]; break;
        }
      }
      switch (c.width) {
        case 8: reinterpret_cast<uint64_t*>(dst)[e] = x; break;
        case 4: reinterpret_cast<uint32_t*>(dst)[e] = static_cast<uint32_t>(x); break;
        case 2: reinterpret_cast<uint16_t*>(dst)[e] = static_cast<uint16_t>(x); break;
        case 1: dst[e] = static_cast<uint8_t>(x); break;
        default: {
          uint32_t* wd = reinterpret_cast<uint32_t*>(dst) + (e >> 5);
          const uint32_t m = 1u << (e & 31);
          if (valid && x) atomicOr(wd, m); else atomicAnd(wd, ~m);
        }
      }
      if (c.elem_validity) {
        uint32_t* wd = reinterpret_cast<uint32_t*>(c.elem_validity) + (e >> 5);
        const uint32_t m = 1u << (e & 31);
        if (valid) atomicOr(wd, m); else atomicAnd(wd, ~m);
      }
    }
  }
  // images -> HBM at the resolved positions
#pragma unroll
  for (int k = 0; k < K; k++) {
    const VarCol& c = a.col[k];
    if (img_at[k] == kNone || (a.skip & 128)) continue;
    const int64_t gb = sbase[k];
    uint8_t* dst = const_cast<uint8_t*>(c.values);
    const uint8_t* im = reinterpret_cast<const uint8_t*>(oimg) + img_at[k];
    const int64_t n = max<int64_t>(0, min<int64_t>(tot[k], c.capacity - gb));
    if (bytes_seq<M>(c)) {
      store_shifted<NT>(dst + gb, im, n);
      continue;
    }
    int64_t vb;
    if (c.width == 0) {
      vb = r16((((tot[k] + 31) >> 5) + 1) * 4);
      store_bits_shifted<NT>(dst, reinterpret_cast<const uint32_t*>(im), gb, n);
    } else {
      vb = r16(int64_t(tot[k]) * c.width + 16);
      store_shifted<NT>(dst + gb * c.width, im, n * c.width);
    }
    if (c.elem_validity)
      store_bits_shifted<NT>(c.elem_validity, reinterpret_cast<const uint32_t*>(im + vb), gb, n);
  }
  if constexpr (!PIPE) break;
  if (!more) break;
  __syncthreads();   // the images are read out, the next stage has landed (vmcnt)
  zero_images();
  lds_barrier();
  b = nxt;
  }
}
#endif  // FURY_VAR_DEC

// Decode / row->Arrow, single pass: 256 rows per workgroup.  Arrow offsets of STRING/BINARY and
// LIST fields are a scan over ALL rows, so groups chain their totals with a decoupled look-back
// (each group publishes its aggregate, then resolves its prefix from its predecessors' published
// words; groups take logical numbers from a ticket so every group they wait on is already
// running).  The group's row range is staged in LDS with 16-B loads; fixed fields leave as
// coalesced per-column stores with ballot-built validity while the look-back is in flight;
// string payloads are assembled in an LDS image of the group's output range; list elements are
// spread one per lane over the group's flat element range (row found by binary search over the
// group's element starts) so child values and validity bits leave coalesced.
// Last t in [0, nr) with pos[t] <= idx: the row holding element idx (empty rows share their
// successor's start and are skipped).
__device__ __forceinline__ int find_row(const int32_t* pos, int nr, int32_t idx) {
  int lo = 0, hi = nr;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (pos[mid] <= idx) lo = mid;
    else hi = mid;
  }
  return lo;
}

// 64 bits of an Arrow bitmap starting at 64-aligned bit gbit0: bits in `mask` get `val`.
// Words wholly owned by this group are stored; words shared with a neighbouring group are
// updated with atomic and/or of exactly these bits.
__device__ __forceinline__ void put_bits64(uint8_t* bits, int64_t gbit0, uint64_t val,
                                           uint64_t mask, int64_t cap) {
  if (gbit0 + 64 > cap) mask &= cap <= gbit0 ? 0 : (~0ull >> (64 - (cap - gbit0)));
  const int lane = threadIdx.x & 63;
  if (lane < 2) {
    const uint32_t m = static_cast<uint32_t>(mask >> (32 * lane));
    const uint32_t v = static_cast<uint32_t>(val >> (32 * lane)) & m;
    uint32_t* w = reinterpret_cast<uint32_t*>(bits) + (gbit0 >> 5) + lane;
    if (m == ~0u) {
      *w = v;
    } else if (m) {
      atomicAnd(w, ~m);
      atomicOr(w, v);
    }
  }
}

struct DecodeShared {
  int32_t pos[kSeqChunk][kThreads + 1];   // group-relative exclusive starts; [nr] = group total
  int64_t rowoff[kThreads];                // absolute row start; -1: the row is outside the batch
  int64_t base[kSeqChunk];                 // global start of the group's range, per sequence
  int64_t tmp[kThreads / 64];
};

// Where the group reads batch bytes [q, q + len) from: its staged row range in LDS when they lie
// inside it, else HBM (a slot may point at bytes of another row -- the reference reads them
// through the shared buffer, so this decode does too).
struct TileView {
  const uint8_t* rows;       // the batch (HBM)
  const uint8_t* stage;      // byte `lo` of the batch in LDS, or NULL (not staged)
  int64_t lo, hi;            // staged absolute range
  __device__ __forceinline__ const uint8_t* at(int64_t q, int64_t len) const {
    return (stage && q >= lo && q + len <= hi) ? stage + (q - lo) : rows + q;
  }
};

// Null-or-bad test + count of field k of the row at absolute byte `base` (-1: bad row).
__device__ __forceinline__ int64_t wide_count(const VarArgs& a, CVarCol& c, int k, const TileView& tv,
                                              int64_t base, int64_t total, bool* null, bool* bad) {
  if (base < 0) {
    *null = true;
    *bad = false;
    return 0;
  }
  return field_count(c, k, tv.at(base, a.fixed_size), a.bitmap_bytes, base, tv.rows, total, null,
                     bad);
}

// Counts + in-group scans of the sequences [cbase, cbase + nchunk); publishes the aggregates
// (32-bit, like tile_count).
__device__ __forceinline__ void chunk_count(const VarArgs& a, const TileView& tv, int64_t base,
                                            int64_t total, int64_t r, DecodeShared& sh, int cbase,
                                            int nchunk, int64_t b, uint64_t* status, int nseq) {
  int seq = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (!is_seq(c)) continue;
    const int q = seq++ - cbase;
    if (q < 0) continue;
    if (q >= nchunk) break;
    bool nul = false, bad = false;
    const int64_t cnt = wide_count(a, c, k, tv, base, total, &nul, &bad);
    if (bad) raise_oob(a.err, r);
    int64_t tot;
    const int64_t ex = block_excl_scan(cnt, &tot, sh.tmp);
    sh.pos[q][threadIdx.x] = static_cast<int32_t>(ex);
    if (threadIdx.x == 0) {
      sh.pos[q][kThreads] = static_cast<int32_t>(tot);
      st_status(status + b * nseq + cbase + q,
                (b == 0 ? kInc : kAgg) | static_cast<uint64_t>(static_cast<uint32_t>(tot)));
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void chunk_resolve(const VarArgs& a, DecodeShared& sh, int cbase,
                                              int nchunk, int64_t b, uint64_t* status, int nseq,
                                              const uint8_t* rows, const int64_t* offs) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int q = w; q < nchunk; q += kThreads / 64) {
    const int64_t ex = b == 0 ? 0
                       : look_back_help<kThreads>(a, seq_col(a, cbase + q), rows, offs, status, b,
                                                  nseq, cbase + q, a.err);
    if (lane == 0) {
      sh.base[q] = ex;
      if (b > 0)
        st_status(status + b * nseq + cbase + q,
                  kInc | static_cast<uint64_t>(ex + static_cast<uint32_t>(sh.pos[q][kThreads])));
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void decode_group(const VarArgs& a, const TileView& tv, int64_t total,
                                             uint8_t* oimg, DecodeShared& sh, int64_t b, int64_t nb,
                                             int nr, uint64_t* status, int nseq,
                                             const int64_t* offs) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t r0 = b * kThreads;
  const int64_t r = r0 + tid;
  const bool live = tid < nr;
  const int64_t base = live ? sh.rowoff[tid] : -1;
  const uint8_t* row = base >= 0 ? tv.at(base, a.fixed_size) : nullptr;
  const int64_t rbase = r - lane;                               // this wave's first row
  const int64_t nvalid = r0 + nr - rbase;          // rows of this wave in this tile
  const int nbytes = nvalid >= 64 ? 8 : static_cast<int>((nvalid + 7) >> 3);

  if (nseq > 0) chunk_count(a, tv, base, total, r, sh, 0, min(kSeqChunk, nseq), b, status, nseq);

  // fixed-width fields and every field's validity: no dependency on other groups
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    bool isnull = true, bad = false;
    if (row) (void)wide_count(a, c, k, tv, base, total, &isnull, &bad);
    const uint64_t slot =
        !isnull ? *reinterpret_cast<const uint64_t*>(row + a.bitmap_bytes + 8 * k) : 0;
    if (c.validity) {
      const uint64_t ok = __ballot(live && !isnull);
      if (lane < nbytes) c.validity[(rbase >> 3) + lane] = static_cast<uint8_t>(ok >> (8 * lane));
    }
    uint8_t* dst = const_cast<uint8_t*>(c.values);
    if (c.kind == kFixed) {
      if (live && dst) {
        switch (c.width) {
          case 8: __builtin_nontemporal_store(slot, reinterpret_cast<uint64_t*>(dst) + r); break;
          case 4: reinterpret_cast<uint32_t*>(dst)[r] = static_cast<uint32_t>(slot); break;
          case 2: reinterpret_cast<uint16_t*>(dst)[r] = static_cast<uint16_t>(slot); break;
          default: dst[r] = static_cast<uint8_t>(slot); break;
        }
      }
    } else if (c.kind == kBool) {
      const uint64_t bits = __ballot(live && (slot & 0xff) != 0);
      if (lane < nbytes && dst) dst[(rbase >> 3) + lane] = static_cast<uint8_t>(bits >> (8 * lane));
    } else if (c.kind == kDecimal) {
      if (live && dst) {
        uint64_t* d = reinterpret_cast<uint64_t*>(dst + 16 * r);
        uint64_t lo = 0, hi = 0;
        if (!isnull) {                                  // [p, p + 16) checked by wide_count
          const int64_t p = base + static_cast<int32_t>(slot >> 32);
          const uint8_t* s = tv.at(p, 16);
          lo = reinterpret_cast<const uint64_t*>(s)[0];
          hi = reinterpret_cast<const uint64_t*>(s)[1];
        }
        d[0] = lo;
        d[1] = hi;
      }
    }
  }

  for (int cbase = 0; cbase < nseq; cbase += kSeqChunk) {
    const int nchunk = min(kSeqChunk, nseq - cbase);
    if (cbase > 0) chunk_count(a, tv, base, total, r, sh, cbase, nchunk, b, status, nseq);
    chunk_resolve(a, sh, cbase, nchunk, b, status, nseq, tv.rows, offs);
    int seq = 0;
    for (int k = 0; k < a.ncols; k++) {
      CVarCol& c = vc(a, k);
      if (!is_seq(c)) continue;
      const int q = seq++ - cbase;
      if (q < 0) continue;
      if (q >= nchunk) break;
      const int64_t gb = sh.base[q];
      const int32_t tot = sh.pos[q][kThreads];
      if (live) c.offsets[r] = static_cast<int32_t>(gb + sh.pos[q][tid]);
      if (b == nb - 1 && tid == nr - 1) c.offsets[a.nrows] = static_cast<int32_t>(gb + tot);
      uint8_t* dst = const_cast<uint8_t*>(c.values);
      if (tot == 0 || !dst) continue;
      const int64_t cap = c.capacity;
      if (c.kind == kBytes) {
        const int64_t p0 = gb, p1 = gb + tot;
        bool isnull = true, bad = false;
        const int64_t len = row ? wide_count(a, c, k, tv, base, total, &isnull, &bad) : 0;
        const uint8_t* s = nullptr;
        if (!isnull && len > 0) {
          const uint64_t slot = *reinterpret_cast<const uint64_t*>(row + a.bitmap_bytes + 8 * k);
          const int64_t p = base + static_cast<int32_t>(slot >> 32);
          s = tv.at(p, len);
        }
        const int64_t pos = p0 + sh.pos[q][tid];
        // LDS byte i <-> global byte a0 + i, a0 = 16-aligned address of payload byte p0
        const int64_t a0 = p0 - static_cast<int64_t>(reinterpret_cast<uintptr_t>(dst + p0) & 15);
        if (p1 - a0 <= kStrStage) {
          if (s) put_bytes(oimg, pos - a0, s, len);
          __syncthreads();
          if (cap > p0) copy_bytes_range<true>(dst, oimg, p0, min<int64_t>(p1, cap), a0);
          __syncthreads();
        } else if (s) {
          put_bytes(dst, pos, s, max<int64_t>(0, min<int64_t>(len, cap - pos)));
        }
        continue;
      }
      // LIST of fixed-width elements -> Arrow child values + element validity.  A row owns
      // elements only when its array passed the bounds check (else its count is 0).
      const int ew = c.width == 0 ? 1 : c.width;
      const int sh0 = static_cast<int>(gb & 63);
      const int64_t span = sh0 + tot;
      for (int64_t u0 = 0; u0 < span; u0 += kThreads) {
        const int64_t i = u0 + tid - sh0;                       // element index in the group
        const bool act = i >= 0 && i < tot;
        bool valid = false;
        uint64_t v = 0;
        if (act) {
          const int t = find_row(sh.pos[q], nr, static_cast<int32_t>(i));
          const int64_t bt = sh.rowoff[t];
          const uint64_t sl = *reinterpret_cast<const uint64_t*>(tv.at(bt, a.fixed_size) +
                                                                 a.bitmap_bytes + 8 * k);
          const int64_t pa = bt + static_cast<int32_t>(sl >> 32);
          const int64_t n = static_cast<int32_t>(*gl(reinterpret_cast<const int64_t*>(tv.rows + pa)));
          const uint8_t* arr = tv.at(pa, 8 + bm_bytes(n) + n * ew);
          const int64_t j = i - sh.pos[q][t];
          valid = !((arr[8 + (j >> 3)] >> (j & 7)) & 1);
          if (valid) {
            const uint8_t* p = arr + 8 + bm_bytes(n) + j * ew;
            switch (ew) {
              case 8: v = *reinterpret_cast<const uint64_t*>(p); break;
              case 4: v = *reinterpret_cast<const uint32_t*>(p); break;
              case 2: v = *reinterpret_cast<const uint16_t*>(p); break;
              default: v = *p; break;
            }
          }
          const int64_t e = gb + i;
          if (e < cap) {
            switch (c.width) {
              case 8: __builtin_nontemporal_store(v, reinterpret_cast<uint64_t*>(dst) + e); break;
              case 4: reinterpret_cast<uint32_t*>(dst)[e] = static_cast<uint32_t>(v); break;
              case 2: reinterpret_cast<uint16_t*>(dst)[e] = static_cast<uint16_t>(v); break;
              case 1: dst[e] = static_cast<uint8_t>(v); break;
              default: break;                                 // bool elements: bits below
            }
          }
        }
        const uint64_t am = __ballot(act);
        const int64_t gbit0 = gb - sh0 + (u0 + tid - lane);     // 64-aligned
        if (c.elem_validity) put_bits64(c.elem_validity, gbit0, __ballot(act && valid), am, cap);
        if (c.width == 0) put_bits64(dst, gbit0, __ballot(act && valid && v != 0), am, cap);
      }
    }
  }
}

#ifdef FURY_VAR_MAIN
__global__ __launch_bounds__(kThreads) void decode_var_kernel(VarArgs a,
                                                              const uint8_t* __restrict__ rows,
                                                              const int64_t* __restrict__ offs,
                                                              uint64_t* __restrict__ status,
                                                              int nseq) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kDecodeStage];
  __shared__ __attribute__((aligned(16))) uint8_t oimg[kStrStage];
  __shared__ DecodeShared sh;
  // tile = blockIdx; the look-back helps itself (look_back_help), as in decode_var_reg.
  const int64_t b = static_cast<int64_t>(blockIdx.x);
  const int64_t r0 = b * kThreads;
  const int nr = static_cast<int>(min<int64_t>(kThreads, a.nrows - r0));
  const int64_t total = offs[a.nrows];
  const int64_t rbeg = offs[r0];
  const int64_t bytes = offs[r0 + nr] - rbeg;
  if (threadIdx.x < nr) {
    const int64_t base = offs[r0 + threadIdx.x];
    const bool ok = row_ok(base, a.fixed_size, total);
    if (!ok) raise_oob(a.err, r0 + threadIdx.x);
    sh.rowoff[threadIdx.x] = ok ? base : -1;
  }
  TileView tv{rows, nullptr, 0, 0};
  // LDS-DMA of the tile's row range (every piece in flight at once), when it is inside the batch
  if (bytes >= 0 && bytes + 32 <= kDecodeStage && span_ok(rbeg, bytes, total)) {
    uint32_t at = 0;
    const uint32_t d0 = stage_range<kThreads>(stage, at, rows + rbeg, rows + rbeg + bytes);
    tv = TileView{rows, stage + d0, rbeg, rbeg + bytes};
  }
  __syncthreads();
  decode_group(a, tv, total, oimg, sh, b, gridDim.x, nr, status, nseq, offs);
}
#endif  // FURY_VAR_MAIN

}  // namespace

// Dispatchers of the register-staged kernels (var_reg_enc.hip / var_reg_dec_*.hip).
int launch_encode_var_reg(const VarArgs& b, int64_t* offs, uint8_t* rows, int64_t cap,
                          int64_t ntiles, int mode, const int64_t* tbase, hipStream_t stream);
int launch_measure_tiles(const VarArgs& b, int64_t* tsum, int64_t ntiles, hipStream_t stream);
// The register-staged instances: K in {2, 3, 4, 6, 8, 12, 16} columns (the schema's fields rounded
// up; the decode's look-back status words are tiles x K) x mode (kind_of, from reg_mode).
// The instances with a persistent two-stage variant (VarArgs.dec_pipe): the C4 (3 columns) and
// C3 (6 columns) shapes -- an A/B, not every width.
constexpr bool dec_pipe_k(int k) { return k == 3 || k == 6; }

// Workgroups of a persistent decode_var_reg launch (VarArgs.dec_pipe): the resident count, at most
// the tiles.
inline int64_t dec_pipe_grid(const void* kern, int64_t nt, size_t lds) {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }();
  (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, kDecThreads, lds) != hipSuccess || per < 1) per = 1;
  return std::min<int64_t>(nt, static_cast<int64_t>(per) * cus);
}

inline int reg_dec_k(int ncols) {
  return ncols <= 4 ? (ncols < 2 ? 2 : ncols) : ncols <= 6 ? 6 : ncols <= 8 ? 8 : ncols <= 12 ? 12 : 16;
}
int launch_decode_var_reg(const VarArgs& a, const uint8_t* rows, const int64_t* offs,
                          uint64_t* status, uint32_t img, uint32_t stage, int mode, int64_t nt,
                          hipStream_t stream);
int launch_decode_var_reg_mid(const VarArgs& a, const uint8_t* rows, const int64_t* offs,
                              uint64_t* status, uint32_t img, uint32_t stage, int mode, int64_t nt,
                              hipStream_t stream);
int launch_decode_var_reg_hi(const VarArgs& a, const uint8_t* rows, const int64_t* offs,
                             uint64_t* status, uint32_t img, uint32_t stage, int mode, int64_t nt,
                             hipStream_t stream);

}  // namespace fury
