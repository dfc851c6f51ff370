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
#include <atomic>
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

// kFast: every column is 8 bytes wide and no column carries validity.
// U = column loads per lane in flight in the gather (8 default, 16 "deep"); P = pair mode
// (fast path only): a lane moves rows 2q and 2q + 1 of one column with ONE 16-B load, so a
// wave-instruction covers 128 rows (R >= 128) or two columns x 64 rows (R = 64).
template <int R, bool kFast, int NT, int U = kUnroll, int DS = 4, bool P = false>
__global__ __launch_bounds__(kThreads) void encode_fixed_kernel(FixedArgs a,
                                                                 uint8_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  const int nr = static_cast<int>(min(static_cast<int64_t>(R), a.nrows - r0));
  const int rs = a.row_size;
  const int bm = a.bitmap_bytes;
  const int bw = bm >> 3;
  const int ls = rs;                                // LDS bytes per row

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
    copy_tile<true, NT, DS>(rows + r0 * rs, lds, static_cast<int64_t>(nr) * rs);
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
  copy_tile<true, NT, DS>(rows + r0 * rs, lds, static_cast<int64_t>(nr) * rs);
}

// D = 16-B row-tile loads per lane in flight (4 default, 16 "deep": the whole 64-row Struct-100
// tile in one round trip); P = pair mode (16-B column stores of rows 2q, 2q + 1).
template <int R, bool kFast, int NT, int D = 4, bool P = false, int SU = kUnroll>
__global__ __launch_bounds__(kThreads) void decode_fixed_kernel(FixedArgs a,
                                                                 const uint8_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
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
    for (int base = threadIdx.x; base < total2; base += kThreads * SU) {
#pragma unroll
      for (int u = 0; u < SU; u++) {
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
  for (int base = threadIdx.x; base < total; base += kThreads * SU) {
#pragma unroll
    for (int u = 0; u < SU; u++) {
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

// ---- schemas wider than kMaxWideFixedCols: column blocks -----------------------------------
// A 64-row tile of a very wide row no longer fits the LDS, so the grid is (row tile, column
// block): block b owns fields [64b, 64b + 64) of 64 rows, i.e. null-bitmap WORD b and 512 slot
// bytes of each row (BinaryRowWriter's bitmap is whole 64-bit words, so blocks never share a
// word).  LDS image: 64 rows x (1 + 64) words; a row's two pieces are stored as 8-byte runs.
constexpr int kBlkCols = 64;
constexpr int kBlkRows = 64;
constexpr int kBlkStride = kBlkCols + 1;        // LDS words per row: bitmap word + 64 slots

__global__ __launch_bounds__(kThreads) void encode_fixed_blocks(FixedArgs a, uint8_t* __restrict__ rows) {
  __shared__ uint64_t img[kBlkRows * kBlkStride];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kBlkRows;
  const int nr = static_cast<int>(min(static_cast<int64_t>(kBlkRows), a.nrows - r0));
  const int b = blockIdx.y, c0 = b * kBlkCols;
  const int nc = min(kBlkCols, a.ncols - c0);
  for (int r = threadIdx.x; r < kBlkRows; r += kThreads) img[r * kBlkStride] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < nc * kBlkRows; i += kThreads) {
    const int c = __builtin_amdgcn_readfirstlane(i / kBlkRows);   // a wave: 64 rows of one column
    const int r = i - c * kBlkRows;
    if (r >= nr) continue;
    CFixedCol& fc = fcol(a, c0 + c);
    const int64_t row = r0 + r;
    const uint8_t* vb = fc.validity;
    uint64_t v = 0;
    if (vb && !((vb[row >> 3] >> (row & 7)) & 1))
      atomicOr(reinterpret_cast<uint32_t*>(img + r * kBlkStride) + (c >> 5), 1u << (c & 31));
    else
      v = load_value(fc.values, row, fc.width);
    img[r * kBlkStride + 1 + c] = v;
  }
  __syncthreads();
  const int per = 1 + nc;
  for (int i = threadIdx.x; i < nr * per; i += kThreads) {
    const int r = i / per, j = i - r * per;
    uint8_t* rowp = rows + (r0 + r) * a.row_size;
    uint8_t* dst = j == 0 ? rowp + 8 * b : rowp + a.bitmap_bytes + 8 * (c0 + j - 1);
    *reinterpret_cast<uint64_t*>(dst) = img[r * kBlkStride + j];
  }
}

__global__ __launch_bounds__(kThreads) void decode_fixed_blocks(FixedArgs a,
                                                                const uint8_t* __restrict__ rows) {
  __shared__ uint64_t img[kBlkRows * kBlkStride];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kBlkRows;
  const int nr = static_cast<int>(min(static_cast<int64_t>(kBlkRows), a.nrows - r0));
  const int b = blockIdx.y, c0 = b * kBlkCols;
  const int nc = min(kBlkCols, a.ncols - c0);
  const int per = 1 + nc;
  for (int i = threadIdx.x; i < nr * per; i += kThreads) {
    const int r = i / per, j = i - r * per;
    const uint8_t* rowp = rows + (r0 + r) * a.row_size;
    const uint8_t* src = j == 0 ? rowp + 8 * b : rowp + a.bitmap_bytes + 8 * (c0 + j - 1);
    img[r * kBlkStride + j] = *reinterpret_cast<const uint64_t*>(src);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < nc * kBlkRows; i += kThreads) {
    const int c = __builtin_amdgcn_readfirstlane(i / kBlkRows);
    const int r = i - c * kBlkRows;                      // = lane
    const bool live = r < nr;
    const int64_t row = r0 + r;
    const bool isnull = live && ((img[r * kBlkStride] >> c) & 1);
    const uint64_t v = live && !isnull ? img[r * kBlkStride + 1 + c] : 0;
    CFixedCol& fc = fcol(a, c0 + c);
    const int w = fc.width;
    uint8_t* dst = const_cast<uint8_t*>(fc.values);
    const int64_t rbase = row - lane;                    // r0: the wave's 64 rows
    const int64_t nvalid = a.nrows - rbase;
    const int nbytes = nvalid >= 64 ? 8 : static_cast<int>((nvalid + 7) >> 3);
    if (w == 0) {                                        // BOOL: byte != 0, bit-packed
      const uint64_t bitsv = __ballot(live && (v & 0xff) != 0);
      if (lane < nbytes) dst[(rbase >> 3) + lane] = static_cast<uint8_t>(bitsv >> (8 * lane));
    } else if (live) {
      store_value(dst, row, w, v);
    }
    uint8_t* vb = fc.validity;
    if (vb) {
      const uint64_t ok = __ballot(live && !isnull);
      if (lane < nbytes) vb[(rbase >> 3) + lane] = static_cast<uint8_t>(ok >> (8 * lane));
    }
  }
}

int launch_blocks(bool encode, const FixedArgs& a, uint8_t* rows, hipStream_t stream) {
  const int64_t tiles = (a.nrows + kBlkRows - 1) / kBlkRows;
  const int blocks = (a.ncols + kBlkCols - 1) / kBlkCols;
  if (tiles > 0x7fffffff || blocks > 65535) return set_error(FURY_ERR_INVALID_ARGUMENT, "batch too large");
  const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(blocks));
  if (encode) hipLaunchKernelGGL(encode_fixed_blocks, grid, dim3(kThreads), 0, stream, a, rows);
  else hipLaunchKernelGGL(decode_fixed_blocks, grid, dim3(kThreads), 0, stream, a, rows);
  return check_hip(hipGetLastError(), "fixed column-block launch");
}

}  // namespace

// Host-direct mode of the calling thread (hostpath.cpp): the kernels run on pinned host memory
// over PCIe, where plain loads / stores measured faster than non-temporal ones (95 / 89 vs
// 92 / 88 GB/s encode / decode, profiles/r02_host_direct.json).
static thread_local bool t_host_direct = false;
void set_thread_host_direct(bool on) { t_host_direct = on; }
// tuning "fixed_enc" (round 6 A/B, scripts/r06_fixed_enc.sh, profiles/r06_fixed_enc_ab.txt): the
// fast-path encode's column gather with 0: 8 loads per lane in flight (rounds 1-5), 2: 16 (the
// default: Struct-100 encode 0.291 -> 0.286 ms, six alternating runs), 3: 32 (0.291), 4: 16 loads
// and 8 16-B stores (0.287); 1: pair mode, 16-B column loads of two rows per lane (0.320)
static std::atomic<int> g_fixed_enc{2};
// tuning "fixed_dec" (round 6 A/B): the fast-path decode's column stores per lane in flight, 0: 8
// (default), 1: 16, 2: 4; 3: 8 with 8 row loads per lane in flight instead of 16
static std::atomic<int> g_fixed_dec{0};
void set_fixed_dec(int v) { g_fixed_dec = v; }
int fixed_dec() { return g_fixed_dec; }
void set_fixed_enc(int v) { g_fixed_enc = v; }
int fixed_enc() { return g_fixed_enc; }

namespace {

int pick_rows_per_tile(int row_size) {
  if (row_size * 256 <= 48 * 1024) return 256;
  if (row_size * 128 <= 64 * 1024) return 128;
  return 64;
}

template <typename K>
int launch_tile_kernel(K kernel, int R, int row_size, int64_t nrows, hipStream_t stream,
                       const FixedArgs& a, uint8_t* rows) {
  const size_t lds = static_cast<size_t>(R) * row_size;
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

// 16-B column accesses of the pair mode need 16-B aligned columns.
bool pair_ok(const FixedArgs& a) {
  for (int c = 0; c < a.ncols; c++)
    if (reinterpret_cast<uintptr_t>(a.col[c].values) & 15) return false;
  return true;
}

}  // namespace

// Kernel choice (round-1/2 A/B sweeps, profiles/r01_ab_fixed*.json, r02_host_direct*.json; the
// measured-slower pipelined persistent kernels, padded LDS rows, deep encode gather, pair-mode
// encode and XCD-contiguous tile order were removed in round 3):
//   fast path (8-byte columns, no validity): non-temporal loads + stores; the encode gathers 16
//     column loads per lane (round 6: 1.7 % faster than 8 on this ROCm; tuning fixed_enc); the decode keeps the whole tile in flight (16 loads per lane) and
//     stores pairs of rows as 16-B column accesses;
//   general path (narrow types, validity, > 128 fields): the same tile kernels with per-column
//     width / validity handling;
//   host-direct calls: plain loads / stores (see t_host_direct).
int launch_encode_fixed(const FixedArgs& a, uint8_t* rows, hipStream_t stream, bool fast) {
  if (a.nrows == 0) return FURY_OK;
  if (a.ncols > kMaxWideFixedCols) return launch_blocks(true, a, rows, stream);
  const int R = pick_rows_per_tile(a.row_size);
#define FURY_ENC(RR)                                                                          \
  if (R == RR) {                                                                              \
    if (!fast)                                                                                \
      return launch_tile_kernel(encode_fixed_kernel<RR, false, 0>, RR, a.row_size, a.nrows,   \
                                stream, a, rows);                                             \
    if (t_host_direct)                                                                        \
      return launch_tile_kernel(encode_fixed_kernel<RR, true, 0>, RR, a.row_size, a.nrows,    \
                                stream, a, rows);                                             \
    if (g_fixed_enc == 1 && pair_ok(a))                                                       \
      return launch_tile_kernel(encode_fixed_kernel<RR, true, 3, kUnroll, 4, true>, RR,       \
                                a.row_size, a.nrows, stream, a, rows);                        \
    if (g_fixed_enc == 2)                                                                     \
      return launch_tile_kernel(encode_fixed_kernel<RR, true, 3, 16>, RR, a.row_size,         \
                                a.nrows, stream, a, rows);                                    \
    if (g_fixed_enc == 3)                                                                     \
      return launch_tile_kernel(encode_fixed_kernel<RR, true, 3, 32>, RR, a.row_size,         \
                                a.nrows, stream, a, rows);                                    \
    if (g_fixed_enc == 4)                                                                     \
      return launch_tile_kernel(encode_fixed_kernel<RR, true, 3, 16, 8>, RR, a.row_size,      \
                                a.nrows, stream, a, rows);                                    \
    return launch_tile_kernel(encode_fixed_kernel<RR, true, 3>, RR, a.row_size, a.nrows,      \
                              stream, a, rows);                                               \
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
  if (a.ncols > kMaxWideFixedCols) return launch_blocks(false, a, r, stream);
  const int R = pick_rows_per_tile(a.row_size);
  const bool pair = fast && !t_host_direct && pair_ok(a);
#define FURY_DEC(RR)                                                                          \
  if (R == RR) {                                                                              \
    if (!fast)                                                                                \
      return launch_tile_kernel(decode_fixed_kernel<RR, false, 0>, RR, a.row_size, a.nrows,   \
                                stream, a, r);                                                \
    if (t_host_direct)                                                                        \
      return launch_tile_kernel(decode_fixed_kernel<RR, true, 0>, RR, a.row_size, a.nrows,    \
                                stream, a, r);                                                \
    if (pair && g_fixed_dec == 1)                                                             \
      return launch_tile_kernel(decode_fixed_kernel<RR, true, 3, 16, true, 16>, RR,           \
                                a.row_size, a.nrows, stream, a, r);                           \
    if (pair && g_fixed_dec == 2)                                                             \
      return launch_tile_kernel(decode_fixed_kernel<RR, true, 3, 16, true, 4>, RR,            \
                                a.row_size, a.nrows, stream, a, r);                           \
    if (pair && g_fixed_dec == 3)                                                             \
      return launch_tile_kernel(decode_fixed_kernel<RR, true, 3, 8, true>, RR,                \
                                a.row_size, a.nrows, stream, a, r);                           \
    return pair ? launch_tile_kernel(decode_fixed_kernel<RR, true, 3, 16, true>, RR,          \
                                     a.row_size, a.nrows, stream, a, r)                       \
                : launch_tile_kernel(decode_fixed_kernel<RR, true, 3, 16, false>, RR,         \
                                     a.row_size, a.nrows, stream, a, r);                      \
  }
  FURY_DEC(256)
  FURY_DEC(128)
  FURY_DEC(64)
#undef FURY_DEC
  return set_error(FURY_ERR_UNSUPPORTED, "row size");
}

}  // namespace fury
