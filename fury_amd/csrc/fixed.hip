// fixed.hip — gfx950 kernels for schemas whose fields are all fixed width (every row is
// fixed_size = bitmap + 8 * numFields bytes; Struct-100 is the headline case).
//
// What the reference does per row (java/fury-format, FMT = .../org/apache/fury/format):
//   encode  BinaryRowWriter.reset() zeroes the null bitmap (FMT/row/binary/writer/
//           BinaryRowWriter.java:76-84); the generated toRow writes each field into its 8-byte
//           slot: 8-byte types as-is (BinaryWriter.java:153-159), narrow types as putInt64(0) +
//           narrow put (BinaryRowWriter.java:92-124); a null boxed field only sets its bitmap bit
//           (BaseBinaryEncoderBuilder.java:448-453) so its slot keeps the fresh buffer's 0.
//   decode  fromRow: `if (!row.isNullAt(i)) bean.f = row.getX(i)` (RowEncoderBuilder.java:185-217,
//           UnsafeTrait.java:68-111).
//
// MI355X design: a batch is an SoA <-> AoS transpose.  One workgroup owns a tile of R
// consecutive rows = ONE contiguous R * row_size byte range of the row buffer.
//   encode: coalesced column reads (a wave reads 64 consecutive values of one column) ->
//           LDS row image -> 16-byte-per-lane contiguous stores of the whole tile.
//   decode: 16-byte-per-lane contiguous loads of the tile -> LDS -> per-column coalesced stores;
//           Arrow validity / bool bits come from a 64-lane ballot (one 8-byte word per wave).
// No MFMA: the kernel is HBM-bound byte movement; LDS only re-shapes the access pattern.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 8;

__device__ __forceinline__ uint64_t load_value(const uint8_t* p, int64_t row, int width) {
  switch (width) {
    case 8: return *reinterpret_cast<const uint64_t*>(p + row * 8);
    case 4: return *reinterpret_cast<const uint32_t*>(p + row * 4);
    case 2: return *reinterpret_cast<const uint16_t*>(p + row * 2);
    case 1: return p[row];
    default: return (p[row >> 3] >> (row & 7)) & 1;   // 0 = Arrow bit-packed bool
  }
}

__device__ __forceinline__ void store_value(uint8_t* p, int64_t row, int width, uint64_t v) {
  switch (width) {
    case 8: *reinterpret_cast<uint64_t*>(p + row * 8) = v; break;
    case 4: *reinterpret_cast<uint32_t*>(p + row * 4) = static_cast<uint32_t>(v); break;
    case 2: *reinterpret_cast<uint16_t*>(p + row * 2) = static_cast<uint16_t>(v); break;
    case 1: p[row] = static_cast<uint8_t>(v); break;
    default: break;
  }
}

// Column of work item idx (= c * R + r).  R >= 64: a wave covers 64 rows of ONE column (wave
// uniform, scalar column record).  R == 32 (short tiles): lanes 0-31 take column c0 and lanes 32-63
// column c0 + 1 of the same wave.
template <int R>
__device__ __forceinline__ int col_of(int idx, int total, int lane) {
  if constexpr (R >= 64) {
    return __builtin_amdgcn_readfirstlane(min(idx, total - 1) / R);
  } else {
    static_assert(R == 32, "short tiles are 32 rows");
    return __builtin_amdgcn_readfirstlane(min(idx - lane, total - 1) / R) + (lane >> 5);
  }
}
template <int R>
__device__ __forceinline__ uint8_t* values_of(const FixedArgs& a, int c, int lane) {
  if constexpr (R >= 64) {
    return const_cast<uint8_t*>(a.col[c].values);
  } else {
    const int c0 = __builtin_amdgcn_readfirstlane(c);
    uint8_t* p0 = const_cast<uint8_t*>(a.col[c0].values);
    uint8_t* p1 = const_cast<uint8_t*>(a.col[min(c0 + 1, kMaxFixedCols - 1)].values);
    return lane >= 32 ? p1 : p0;
  }
}

// Column record c of the general path: argument block, or the device table of a wide schema.
// Both are constant address space (kernarg / read-only table): scalar loads of the record (as
// generic pointers, the select compiled to flat vector loads).
using CFixedCol = __attribute__((address_space(4))) const FixedCol;
__device__ __forceinline__ CFixedCol& fcol(const FixedArgs& a, int c) {
  CFixedCol* base = a.tab ? (CFixedCol*)(a.tab) : (CFixedCol*)(a.col);
  return base[c];
}

// Tile of workgroup b.  Workgroups are dealt round-robin to the 8 XCDs (b % 8); tile_order 1
// gives each XCD one contiguous eighth of the tiles (b -> (b % 8) * (nb / 8) + b / 8 on the
// largest multiple of 8, identity on the tail), so an XCD's L2 and TLB see one address range.
__device__ __forceinline__ int64_t tile_of(const FixedArgs& a) {
  const int64_t b = blockIdx.x, nb = gridDim.x;
  if (!a.tile_order) return b;
  const int64_t q = nb >> 3;
  return b < 8 * q ? (b & 7) * q + (b >> 3) : b;
}

// Global access helpers; NT bit 0 = non-temporal loads, bit 1 = non-temporal stores (streamed
// bytes are touched once, so keeping them out of L2/MALL leaves room for the other stream).
using v4u = __attribute__((ext_vector_type(4))) uint32_t;
template <int NT>
__device__ __forceinline__ uint64_t ld8(const uint8_t* p) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
  if (NT & 1) return __builtin_nontemporal_load(q);
  return *q;
}
template <int NT>
__device__ __forceinline__ void st8(uint8_t* p, uint64_t v) {
  uint64_t* q = reinterpret_cast<uint64_t*>(p);
  if (NT & 2) __builtin_nontemporal_store(v, q);
  else *q = v;
}
template <int NT>
__device__ __forceinline__ v4u ld16(const uint8_t* p) {
  const v4u* q = reinterpret_cast<const v4u*>(p);
  if (NT & 1) return __builtin_nontemporal_load(q);
  return *q;
}
template <int NT>
__device__ __forceinline__ void st16(uint8_t* p, const v4u& v) {
  v4u* q = reinterpret_cast<v4u*>(p);
  if (NT & 2) __builtin_nontemporal_store(v, q);
  else *q = v;
}

// Copies `bytes` (multiple of 8) between LDS and global, 16 B per lane where possible, with D
// 16-B accesses per lane in flight before the LDS side is touched (loads) / issued back to back
// (stores).
template <bool kToGlobal, int NT, int D = 4>
__device__ __forceinline__ void copy_tile(uint8_t* __restrict__ g, uint8_t* __restrict__ lds,
                                          int64_t bytes) {
  const int64_t n16 = bytes >> 4;
  v4u* l16 = reinterpret_cast<v4u*>(lds);
  int64_t i = threadIdx.x;
  for (; i + (D - 1) * kThreads < n16; i += D * kThreads) {
    v4u t[D];
    if (kToGlobal) {
#pragma unroll
      for (int k = 0; k < D; k++) t[k] = l16[i + k * kThreads];
#pragma unroll
      for (int k = 0; k < D; k++) st16<NT>(g + 16 * (i + k * kThreads), t[k]);
    } else {
#pragma unroll
      for (int k = 0; k < D; k++) t[k] = ld16<NT>(g + 16 * (i + k * kThreads));
#pragma unroll
      for (int k = 0; k < D; k++) l16[i + k * kThreads] = t[k];
    }
  }
  if (!kToGlobal) {     // remainder: all of this lane's loads first, then the LDS writes
    v4u t[D];
#pragma unroll
    for (int k = 0; k < D; k++)
      if (i + k * kThreads < n16) t[k] = ld16<NT>(g + 16 * (i + k * kThreads));
#pragma unroll
    for (int k = 0; k < D; k++)
      if (i + k * kThreads < n16) l16[i + k * kThreads] = t[k];
  } else {
    for (; i < n16; i += kThreads) st16<NT>(g + 16 * i, l16[i]);
  }
  if ((bytes & 15) && threadIdx.x == 0) {
    uint64_t* g8 = reinterpret_cast<uint64_t*>(g + (n16 << 4));
    uint64_t* l8 = reinterpret_cast<uint64_t*>(lds + (n16 << 4));
    if (kToGlobal) *g8 = *l8;
    else *l8 = *g8;
  }
}

// LDS row stride of the padded encode: an odd number of 8-B words.
__host__ __device__ __forceinline__ int lds_row_stride(int rs) { return ((rs >> 3) & 1) ? rs : rs + 8; }

// Row tile LDS -> global.  Unpadded: one contiguous copy.  Padded (LDS row stride ls != rs):
// each lane's 16-B output chunk is read as two 8-B words from their padded LDS rows; the chunk's
// (row, offset) advances incrementally by the loop stride, so there is no division per chunk.
template <int NT, int DS, bool PAD>
__device__ __forceinline__ void store_tile(uint8_t* __restrict__ g, uint8_t* __restrict__ lds,
                                           int nr, int rs, int ls) {
  const int64_t bytes = static_cast<int64_t>(nr) * rs;
  if (!PAD || ls == rs) {
    copy_tile<true, NT, DS>(g, lds, bytes);
    return;
  }
  const int n16 = static_cast<int>(bytes >> 4);
  constexpr int kStep = 16 * kThreads;
  const int q = kStep / rs, rm = kStep - q * rs;
  int o = 16 * threadIdx.x;
  int row = o / rs, w = o - row * rs;
  for (int i = threadIdx.x; i < n16; i += kThreads) {
    const uint64_t lo = *reinterpret_cast<const uint64_t*>(lds + row * ls + w);
    int row2 = row, w2 = w + 8;
    if (w2 >= rs) { w2 -= rs; row2++; }
    const uint64_t hi = *reinterpret_cast<const uint64_t*>(lds + row2 * ls + w2);
    st16<NT>(g + 16 * static_cast<int64_t>(i),
             v4u{static_cast<uint32_t>(lo), static_cast<uint32_t>(lo >> 32),
                 static_cast<uint32_t>(hi), static_cast<uint32_t>(hi >> 32)});
    row += q;
    w += rm;
    if (w >= rs) { w -= rs; row++; }
  }
  if ((bytes & 15) && threadIdx.x == 0) {       // a last 8-B word (rs % 16 == 8, nr odd)
    const int64_t o8 = static_cast<int64_t>(n16) << 4;
    const int r8 = static_cast<int>(o8 / rs);
    *reinterpret_cast<uint64_t*>(g + o8) =
        *reinterpret_cast<const uint64_t*>(lds + r8 * ls + (o8 - static_cast<int64_t>(r8) * rs));
  }
}

// kFast: every column is 8 bytes wide and no column carries validity.
// U = column loads per lane in flight in the gather (8 default, 16 "deep"); P = pair mode
// (fast path only): a lane moves rows 2q and 2q + 1 of one column with ONE 16-B load, so a
// wave-instruction covers 128 rows (R >= 128) or two columns x 64 rows (R = 64).
// PAD: LDS rows are laid out with an odd number of 8-B words (row size + 8 when row_size / 8 is
// even) so the 64 lanes of a column write hit 64 distinct LDS banks; the copy-out then maps
// each 16-B output chunk back to its padded LDS address.
template <int R, bool kFast, int NT, int U = kUnroll, int DS = 4, bool P = false, bool PAD = false>
__global__ __launch_bounds__(kThreads) void encode_fixed_kernel(FixedArgs a,
                                                                 uint8_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t r0 = tile_of(a) * R;
  const int nr = static_cast<int>(min(static_cast<int64_t>(R), a.nrows - r0));
  const int rs = a.row_size;
  const int bm = a.bitmap_bytes;
  const int bw = bm >> 3;
  const int ls = PAD ? lds_row_stride(rs) : rs;     // LDS bytes per row

  // BinaryRowWriter.reset(): zero the bitmap words of every row of the tile.
  for (int i = threadIdx.x; i < R * bw; i += kThreads) {
    const int r = i / bw, w = i - r * bw;
    *reinterpret_cast<uint64_t*>(lds + r * ls + 8 * w) = 0;
  }
  if (!kFast) __syncthreads();   // the null bits below are OR-ed into these words

  const int lane = threadIdx.x & 63;
  if constexpr (P) {
    static_assert(kFast, "pair mode is fast-path only");
    constexpr int H = R / 2;                       // row pairs per column of the tile
    const int total2 = a.ncols * H;
    for (int base = threadIdx.x; base < total2; base += kThreads * U) {
      v4u v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int idx = base + u * kThreads;
        const int c = col_of<H>(idx, total2, lane);
        const int r = 2 * (idx - c * H);
        if (idx < total2 && r < nr) {
          const uint8_t* src = values_of<H>(a, c, lane) + (r0 + r) * 8;
          if (r + 1 < nr) {
            v[u] = ld16<NT>(src);
          } else {
            const uint64_t x = ld8<NT>(src);
            v[u] = v4u{static_cast<uint32_t>(x), static_cast<uint32_t>(x >> 32), 0u, 0u};
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int idx = base + u * kThreads;
        const int c = col_of<H>(idx, total2, lane);
        const int r = 2 * (idx - c * H);
        if (idx < total2 && r < nr) {
          uint8_t* p = lds + r * ls + bm + 8 * c;
          *reinterpret_cast<uint64_t*>(p) = static_cast<uint64_t>(v[u].x) |
                                            (static_cast<uint64_t>(v[u].y) << 32);
          if (r + 1 < nr)
            *reinterpret_cast<uint64_t*>(p + ls) = static_cast<uint64_t>(v[u].z) |
                                                   (static_cast<uint64_t>(v[u].w) << 32);
        }
      }
    }
    __syncthreads();
    store_tile<NT, DS, PAD>(rows + r0 * rs, lds, nr, rs, ls);
    return;
  }

  // Gather: item = c * R + r; a wave covers 64 consecutive rows of ONE column (R % 64 == 0).
  const int total = a.ncols * R;
  for (int base = threadIdx.x; base < total; base += kThreads * U) {
    uint64_t v[U];
    bool isnull[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int idx = base + u * kThreads;
      const int c = col_of<R>(idx, total, lane);
      const int r = idx - c * R;
      v[u] = 0;
      isnull[u] = false;
      if (idx < total && r < nr) {
        const int64_t row = r0 + r;
        if (kFast) {
          v[u] = ld8<NT>(values_of<R>(a, c, lane) + row * 8);
        } else {
          CFixedCol& fc = fcol(a, c);
          const uint8_t* vb = fc.validity;
          if (vb && !((vb[row >> 3] >> (row & 7)) & 1)) {
            isnull[u] = true;
          } else {
            v[u] = load_value(fc.values, row, fc.width);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int idx = base + u * kThreads;
      const int c = col_of<R>(idx, total, lane);
      const int r = idx - c * R;
      if (idx < total && r < nr) {
        uint8_t* rowp = lds + r * ls;
        *reinterpret_cast<uint64_t*>(rowp + bm + 8 * c) = v[u];
        if (!kFast && isnull[u]) {
          atomicOr(reinterpret_cast<uint32_t*>(rowp) + (c >> 5), 1u << (c & 31));
        }
      }
    }
  }
  __syncthreads();
  store_tile<NT, DS, PAD>(rows + r0 * rs, lds, nr, rs, ls);
}

// D = 16-B row-tile loads per lane in flight (4 default, 16 "deep": the whole 64-row Struct-100
// tile in one round trip); P = pair mode (16-B column stores of rows 2q, 2q + 1).
template <int R, bool kFast, int NT, int D = 4, bool P = false>
__global__ __launch_bounds__(kThreads) void decode_fixed_kernel(FixedArgs a,
                                                                 const uint8_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t r0 = tile_of(a) * R;
  const int nr = static_cast<int>(min(static_cast<int64_t>(R), a.nrows - r0));
  const int rs = a.row_size;
  const int bm = a.bitmap_bytes;

  copy_tile<false, NT, D>(const_cast<uint8_t*>(rows + r0 * rs), lds, static_cast<int64_t>(nr) * rs);
  __syncthreads();

  const int lane = threadIdx.x & 63;
  if constexpr (P) {
    static_assert(kFast, "pair mode is fast-path only");
    constexpr int H = R / 2;
    const int total2 = a.ncols * H;
    for (int base = threadIdx.x; base < total2; base += kThreads * kUnroll) {
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const int idx = base + u * kThreads;
        if (__builtin_amdgcn_readfirstlane(idx - lane) >= total2) break;
        const int c = col_of<H>(idx, total2, lane);
        const int r = 2 * (idx - c * H);
        if (idx < total2 && r < nr) {
          const uint8_t* p = lds + r * rs + bm + 8 * c;
          const uint64_t x0 = *reinterpret_cast<const uint64_t*>(p);
          uint8_t* dst = values_of<H>(a, c, lane) + (r0 + r) * 8;
          if (r + 1 < nr) {
            const uint64_t x1 = *reinterpret_cast<const uint64_t*>(p + rs);
            st16<NT>(dst, v4u{static_cast<uint32_t>(x0), static_cast<uint32_t>(x0 >> 32),
                              static_cast<uint32_t>(x1), static_cast<uint32_t>(x1 >> 32)});
          } else {
            st8<NT>(dst, x0);
          }
        }
      }
    }
    return;
  }
  const int total = a.ncols * R;
  for (int base = threadIdx.x; base < total; base += kThreads * kUnroll) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
      const int idx = base + u * kThreads;
      if (__builtin_amdgcn_readfirstlane(idx - lane) >= total) break;   // wave-uniform exit
      const int c = col_of<R>(idx, total, lane);
      const int r = idx - c * R;
      const bool live = r < nr && idx < total;
      const uint8_t* rowp = lds + r * rs;
      const int64_t row = r0 + r;
      if (kFast) {
        if (live) {
          uint64_t v = *reinterpret_cast<const uint64_t*>(rowp + bm + 8 * c);
          st8<NT>(values_of<R>(a, c, lane) + row * 8, v);
        }
        continue;
      }
      bool isnull = live && ((rowp[c >> 3] >> (c & 7)) & 1);
      uint64_t v = 0;
      if (live && !isnull) v = *reinterpret_cast<const uint64_t*>(rowp + bm + 8 * c);
      CFixedCol& fc = fcol(a, c);
      const int w = fc.width;
      uint8_t* dst = const_cast<uint8_t*>(fc.values);
      // rows [rbase, rbase + 64) of this wave; rbase % 64 == 0 and R % 64 == 0
      const int64_t rbase = row - lane;
      const int64_t nvalid = a.nrows - rbase;                    // >= 1 for live waves
      const int nbytes = nvalid >= 64 ? 8 : static_cast<int>((nvalid + 7) >> 3);
      if (w == 0) {   // BOOL: getBoolean = byte != 0, bit-packed Arrow output
        uint64_t bitsv = __ballot(live && (v & 0xff) != 0);
        if (lane < nbytes) dst[(rbase >> 3) + lane] = static_cast<uint8_t>(bitsv >> (8 * lane));
      } else if (live) {
        store_value(dst, row, w, v);
      }
      uint8_t* vb = fc.validity;
      if (vb) {
        uint64_t ok = __ballot(live && !isnull);
        if (lane < nbytes) vb[(rbase >> 3) + lane] = static_cast<uint8_t>(ok >> (8 * lane));
      }
    }
  }
}

// ---- pipelined persistent variants (fast path: all 8-byte columns, no validity) ------------
// One workgroup walks tiles blockIdx.x, +gridDim.x, ...; while tile t's LDS image streams out to
// HBM, tile t+1's global loads are already in flight (register staging).  Barriers only order
// LDS (lgkmcnt(0) + s_barrier): no vmcnt(0) drain, so the prefetch survives them.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int MAXU, int NT>
__global__ __launch_bounds__(kThreads) void encode_fixed_pipe(FixedArgs a,
                                                              uint8_t* __restrict__ rows,
                                                              int64_t ntiles) {
  constexpr int R = 64;   // lane == row of the tile; wave w owns columns w, w+4, ...
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  const int rs = a.row_size;
  const int bm = a.bitmap_bytes;
  const int bw = bm >> 3;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ncols = a.ncols;
  for (int i = threadIdx.x; i < R * bw; i += kThreads) {
    const int r = i / bw, w = i - r * bw;
    *reinterpret_cast<uint64_t*>(lds + r * rs + 8 * w) = 0;   // never nulls on this path
  }
  // Column pointers are loop invariant and wave uniform: load them once into SGPRs (the
  // record table always has kMaxFixedCols entries, so reading past ncols is in bounds).
  static_assert(4 * MAXU <= kMaxFixedCols, "column table");
  const uint8_t* p[MAXU];
#pragma unroll
  for (int u = 0; u < MAXU; u++) p[u] = a.col[wid + 4 * u].values;
  uint64_t v[MAXU];
  int64_t tile = blockIdx.x;
  auto load = [&](int64_t t) {
    const int64_t row = t * R + lane;
    const bool ok = row < a.nrows;
#pragma unroll
    for (int u = 0; u < MAXU; u++) {
      const int c = wid + 4 * u;
      if (c < ncols && ok) v[u] = ld8<NT>(p[u] + row * 8);
    }
  };
  if (tile < ntiles) load(tile);
  while (tile < ntiles) {
    const int64_t r0 = tile * R;
    const int nr = static_cast<int>(min(static_cast<int64_t>(R), a.nrows - r0));
#pragma unroll
    for (int u = 0; u < MAXU; u++) {
      const int c = wid + 4 * u;
      if (c < ncols && lane < nr) *reinterpret_cast<uint64_t*>(lds + lane * rs + bm + 8 * c) = v[u];
    }
    lds_barrier();
    const int64_t next = tile + gridDim.x;
    if (next < ntiles) load(next);
    const int64_t bytes = static_cast<int64_t>(nr) * rs;
    uint8_t* g = rows + r0 * rs;
    const int n16 = static_cast<int>(bytes >> 4);
    for (int i = threadIdx.x; i < n16; i += kThreads)
      st16<NT>(g + 16 * i, *reinterpret_cast<const v4*>(lds + 16 * i));
    if ((bytes & 15) && threadIdx.x == 0)
      *reinterpret_cast<uint64_t*>(g + 16 * n16) = *reinterpret_cast<const uint64_t*>(lds + 16 * n16);
    lds_barrier();
    tile = next;
  }
}

template <int MAXL, int NT>
__global__ __launch_bounds__(kThreads) void decode_fixed_pipe(FixedArgs a,
                                                              const uint8_t* __restrict__ rows,
                                                              int64_t ntiles) {
  constexpr int R = 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  const int rs = a.row_size;
  const int bm = a.bitmap_bytes;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ncols = a.ncols;
  const uint8_t* q[32];
#pragma unroll
  for (int u = 0; u < 32; u++) q[u] = a.col[wid + 4 * u].values;
  v4 t16[MAXL];
  int64_t tile = blockIdx.x;
  auto load = [&](int64_t t) {
    const int64_t r0 = t * R;
    const int nr = static_cast<int>(min(static_cast<int64_t>(R), a.nrows - r0));
    const int n16 = (nr * rs) >> 4;
    const v4* g = reinterpret_cast<const v4*>(rows + r0 * rs);
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      const int i = threadIdx.x + k * kThreads;
      if (i < n16) t16[k] = ld16<NT>(reinterpret_cast<const uint8_t*>(g + i));
    }
  };
  if (tile < ntiles) load(tile);
  while (tile < ntiles) {
    const int64_t r0 = tile * R;
    const int nr = static_cast<int>(min(static_cast<int64_t>(R), a.nrows - r0));
    const int64_t bytes = static_cast<int64_t>(nr) * rs;
    const int n16 = static_cast<int>(bytes >> 4);
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      const int i = threadIdx.x + k * kThreads;
      if (i < n16) *reinterpret_cast<v4*>(lds + 16 * i) = t16[k];
    }
    if ((bytes & 15) && threadIdx.x == 0)
      *reinterpret_cast<uint64_t*>(lds + 16 * n16) =
          *reinterpret_cast<const uint64_t*>(rows + r0 * rs + 16 * n16);
    lds_barrier();
    const int64_t next = tile + gridDim.x;
    if (next < ntiles) load(next);
    const int64_t row = r0 + lane;
    if (lane < nr) {
#pragma unroll
      for (int u = 0; u < 32; u++) {
        const int c = wid + 4 * u;
        if (c < ncols) {
          const uint64_t x = *reinterpret_cast<const uint64_t*>(lds + lane * rs + bm + 8 * c);
          uint64_t* dst = reinterpret_cast<uint64_t*>(const_cast<uint8_t*>(q[u])) + row;
          st8<NT>(reinterpret_cast<uint8_t*>(dst), x);
        }
      }
    }
    lds_barrier();
    tile = next;
  }
}

}  // namespace

// Kernel variant for fixed-width fast-path schemas (fury_set_tuning("fixed_variant", v) or env
// FURY_FIXED_VARIANT), a bit set: 1 = pipelined persistent kernel, 2 = nt stores, 4 = nt loads.
static int g_variant = -1;
static thread_local int t_variant = -1;      // the calling thread's override (host direct path)

int fixed_variant() {
  if (t_variant >= 0) return t_variant;
  if (g_variant < 0) {
    const char* e = getenv("FURY_FIXED_VARIANT");
    // tile kernel + nt loads + nt stores + pair-mode deep decode (A/B: profiles/r01_ab_fixed*.json)
    g_variant = e ? atoi(e) : 54;
  }
  return g_variant;
}

void set_fixed_variant(int v) { g_variant = v; }
void set_thread_fixed_variant(int v) { t_variant = v; }

namespace {

template <typename K>
int launch_pipe(K kernel, int row_size, int64_t nrows, hipStream_t stream, const FixedArgs& a,
                uint8_t* rows) {
  const size_t lds = static_cast<size_t>(64) * row_size;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       static_cast<int>(lds));
    if (e != hipSuccess) return check_hip(e, "hipFuncSetAttribute");
  }
  const int64_t ntiles = (nrows + 63) / 64;
  int dev = 0, cus = 256, per_cu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kernel),
                                                     kThreads, lds);
  if (per_cu < 1) per_cu = 1;
  const int64_t cap = static_cast<int64_t>(cus) * per_cu;
  const int64_t grid = ntiles < cap ? ntiles : cap;
  hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(grid)), dim3(kThreads), lds, stream, a,
                     rows, ntiles);
  return check_hip(hipGetLastError(), "fixed pipelined kernel launch");
}

int pick_rows_per_tile(int row_size) {
  if (row_size * 256 <= 48 * 1024) return 256;
  if (row_size * 128 <= 64 * 1024) return 128;
  return 64;
}

template <typename K>
int launch_tile_kernel(K kernel, int R, int row_size, int64_t nrows, hipStream_t stream,
                       const FixedArgs& a, uint8_t* rows, int lds_row = 0) {
  const size_t lds = static_cast<size_t>(R) * (lds_row ? lds_row : row_size);
  static_assert(sizeof(FixedArgs) < 4096, "kernel argument block too large");
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       static_cast<int>(lds));
    if (e != hipSuccess) return check_hip(e, "hipFuncSetAttribute");
  }
  const int64_t blocks = (nrows + R - 1) / R;
  if (blocks > 0x7fffffff) return set_error(FURY_ERR_INVALID_ARGUMENT, "batch too large");
  hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(blocks)), dim3(kThreads), lds, stream, a,
                     rows);
  return check_hip(hipGetLastError(), "fixed kernel launch");
}

// Fast-path tile kernels (nt loads + stores) with the variant bits 3 (deep encode gather: 16
// column loads per lane in flight), 4 (pair mode: 16-B column accesses) and 5 (deep decode:
// 16 tile loads per lane in flight).
template <int R, bool kEnc, bool P>
int launch_fast_tile(const FixedArgs& a, uint8_t* rows, hipStream_t stream, bool deep, bool pad) {
  const int ls = lds_row_stride(a.row_size);
  if (kEnc) {
    if (pad)
      return deep ? launch_tile_kernel(encode_fixed_kernel<R, true, 3, 16, 4, P, true>, R,
                                       a.row_size, a.nrows, stream, a, rows, ls)
                  : launch_tile_kernel(encode_fixed_kernel<R, true, 3, 8, 4, P, true>, R,
                                       a.row_size, a.nrows, stream, a, rows, ls);
    return deep ? launch_tile_kernel(encode_fixed_kernel<R, true, 3, 16, 4, P>, R, a.row_size,
                                     a.nrows, stream, a, rows)
                : launch_tile_kernel(encode_fixed_kernel<R, true, 3, 8, 4, P>, R, a.row_size,
                                     a.nrows, stream, a, rows);
  }
  return deep ? launch_tile_kernel(decode_fixed_kernel<R, true, 3, 16, P>, R, a.row_size, a.nrows,
                                   stream, a, rows)
              : launch_tile_kernel(decode_fixed_kernel<R, true, 3, 4, P>, R, a.row_size, a.nrows,
                                   stream, a, rows);
}

template <bool kEnc>
int launch_fast_tile_variant(const FixedArgs& a0, uint8_t* rows, hipStream_t stream, int var) {
  FixedArgs a = a0;
  a.tile_order = (var & 512) ? 1 : 0;          // bit 9: XCD-contiguous tile ranges
  int R = pick_rows_per_tile(a.row_size);
  // bit 8: tall tiles (twice the rows: longer contiguous column runs, fewer workgroups per CU)
  if ((var & 256) && R < 256 && static_cast<int64_t>(2 * R) * a.row_size <= 160 * 1024) R *= 2;
  const bool deep = (var & (kEnc ? 8 : 32)) != 0;
  const bool pad = kEnc && (var & 128) != 0;
  // pad only where it fits the LDS budget of the unpadded tile's occupancy class
  const bool pad_ok = pad && static_cast<int64_t>(R) * lds_row_stride(a.row_size) <= 64 * 1024;
  bool pair = (var & (kEnc ? 64 : 16)) != 0;
  for (int c = 0; c < a.ncols && pair; c++)       // 16-B column accesses need 16-B aligned columns
    pair = (reinterpret_cast<uintptr_t>(a.col[c].values) & 15) == 0;
#define FURY_FT(RR)                                                              \
  if (R == RR)                                                                   \
    return pair ? launch_fast_tile<RR, kEnc, true>(a, rows, stream, deep, pad_ok) \
                : launch_fast_tile<RR, kEnc, false>(a, rows, stream, deep, pad_ok);
  FURY_FT(256)
  FURY_FT(128)
  FURY_FT(64)
#undef FURY_FT
  return set_error(FURY_ERR_UNSUPPORTED, "row size");
}

}  // namespace

// Variant bits (fury_set_tuning("fixed_variant")): bit 0 = pipelined persistent kernel,
// bit 1 = non-temporal stores, bit 2 = non-temporal loads, bit 3 = deep encode gather, bit 4 =
// pair-mode decode, bit 5 = deep decode loads, bit 6 = pair-mode encode, bit 7 = padded LDS rows
// in the encode, bit 8 = tall tiles (bits 3-8 with nt loads + stores only).  A column-strip
// encode (a workgroup per 256 rows x 20 columns: 2 KB contiguous column reads, 160-B strided row
// strips written) measured 2.77 vs 5.80 TB/s in one process and was removed: partial-row
// writes cost far more than the longer reads gain.  Only the fast path (8-byte columns,
// no validity) has variants; the general path always runs the tile kernel.
int launch_encode_fixed(const FixedArgs& a, uint8_t* rows, hipStream_t stream, bool fast) {
  if (a.nrows == 0) return FURY_OK;
  const int var = fixed_variant();
  const int nt = ((var >> 2) & 1) | (var & 2);          // NT bit0 loads, bit1 stores
  if (fast && (var & 1) && a.ncols <= 128) {
    switch (nt) {
      case 1: return launch_pipe(encode_fixed_pipe<32, 1>, a.row_size, a.nrows, stream, a, rows);
      case 2: return launch_pipe(encode_fixed_pipe<32, 2>, a.row_size, a.nrows, stream, a, rows);
      case 3: return launch_pipe(encode_fixed_pipe<32, 3>, a.row_size, a.nrows, stream, a, rows);
      default: return launch_pipe(encode_fixed_pipe<32, 0>, a.row_size, a.nrows, stream, a, rows);
    }
  }
  if (fast && (var & 1016) && nt == 3) return launch_fast_tile_variant<true>(a, rows, stream, var);
  const int R = pick_rows_per_tile(a.row_size);
#define FURY_ENC(RR)                                                                          \
  if (R == RR) {                                                                              \
    if (!fast)                                                                                \
      return launch_tile_kernel(encode_fixed_kernel<RR, false, 0>, RR, a.row_size, a.nrows,   \
                                stream, a, rows);                                             \
    switch (nt) {                                                                             \
      case 1: return launch_tile_kernel(encode_fixed_kernel<RR, true, 1>, RR, a.row_size,     \
                                        a.nrows, stream, a, rows);                            \
      case 2: return launch_tile_kernel(encode_fixed_kernel<RR, true, 2>, RR, a.row_size,     \
                                        a.nrows, stream, a, rows);                            \
      case 3: return launch_tile_kernel(encode_fixed_kernel<RR, true, 3>, RR, a.row_size,     \
                                        a.nrows, stream, a, rows);                            \
      default: return launch_tile_kernel(encode_fixed_kernel<RR, true, 0>, RR, a.row_size,    \
                                         a.nrows, stream, a, rows);                           \
    }                                                                                         \
  }
  FURY_ENC(256)
  FURY_ENC(128)
  FURY_ENC(64)
#undef FURY_ENC
  return set_error(FURY_ERR_UNSUPPORTED, "row size");
}

int launch_decode_fixed(const FixedArgs& a, const uint8_t* rows, hipStream_t stream, bool fast) {
  if (a.nrows == 0) return FURY_OK;
  uint8_t* r = const_cast<uint8_t*>(rows);
  const int var = fixed_variant();
  const int nt = ((var >> 2) & 1) | (var & 2);
  const int64_t tile_bytes = static_cast<int64_t>(a.row_size) * 64;
  if (fast && (var & 1) && tile_bytes <= 17 * 16 * kThreads) {
    if (tile_bytes <= 13 * 16 * kThreads) {
      switch (nt) {
        case 1: return launch_pipe(decode_fixed_pipe<13, 1>, a.row_size, a.nrows, stream, a, r);
        case 2: return launch_pipe(decode_fixed_pipe<13, 2>, a.row_size, a.nrows, stream, a, r);
        case 3: return launch_pipe(decode_fixed_pipe<13, 3>, a.row_size, a.nrows, stream, a, r);
        default: return launch_pipe(decode_fixed_pipe<13, 0>, a.row_size, a.nrows, stream, a, r);
      }
    }
    switch (nt) {
      case 1: return launch_pipe(decode_fixed_pipe<17, 1>, a.row_size, a.nrows, stream, a, r);
      case 2: return launch_pipe(decode_fixed_pipe<17, 2>, a.row_size, a.nrows, stream, a, r);
      case 3: return launch_pipe(decode_fixed_pipe<17, 3>, a.row_size, a.nrows, stream, a, r);
      default: return launch_pipe(decode_fixed_pipe<17, 0>, a.row_size, a.nrows, stream, a, r);
    }
  }
  if (fast && (var & 1016) && nt == 3) return launch_fast_tile_variant<false>(a, r, stream, var);
  const int R = pick_rows_per_tile(a.row_size);
#define FURY_DEC(RR)                                                                          \
  if (R == RR) {                                                                              \
    if (!fast)                                                                                \
      return launch_tile_kernel(decode_fixed_kernel<RR, false, 0>, RR, a.row_size, a.nrows,   \
                                stream, a, r);                                                \
    switch (nt) {                                                                             \
      case 1: return launch_tile_kernel(decode_fixed_kernel<RR, true, 1>, RR, a.row_size,     \
                                        a.nrows, stream, a, r);                               \
      case 2: return launch_tile_kernel(decode_fixed_kernel<RR, true, 2>, RR, a.row_size,     \
                                        a.nrows, stream, a, r);                               \
      case 3: return launch_tile_kernel(decode_fixed_kernel<RR, true, 3>, RR, a.row_size,     \
                                        a.nrows, stream, a, r);                               \
      default: return launch_tile_kernel(decode_fixed_kernel<RR, true, 0>, RR, a.row_size,    \
                                         a.nrows, stream, a, r);                              \
    }                                                                                         \
  }
  FURY_DEC(256)
  FURY_DEC(128)
  FURY_DEC(64)
#undef FURY_DEC
  return set_error(FURY_ERR_UNSUPPORTED, "row size");
}

}  // namespace fury
