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

// Copies `bytes` (multiple of 8) between LDS and global, 16 B per lane where possible.
template <bool kToGlobal, int NT>
__device__ __forceinline__ void copy_tile(uint8_t* __restrict__ g, uint8_t* __restrict__ lds,
                                          int64_t bytes) {
  const int64_t n16 = bytes >> 4;
  v4u* l16 = reinterpret_cast<v4u*>(lds);
  int64_t i = threadIdx.x;
  for (; i + 3 * kThreads < n16; i += 4 * kThreads) {
    if (kToGlobal) {
      v4u a = l16[i], b = l16[i + kThreads], c = l16[i + 2 * kThreads], d = l16[i + 3 * kThreads];
      st16<NT>(g + 16 * i, a);
      st16<NT>(g + 16 * (i + kThreads), b);
      st16<NT>(g + 16 * (i + 2 * kThreads), c);
      st16<NT>(g + 16 * (i + 3 * kThreads), d);
    } else {
      v4u a = ld16<NT>(g + 16 * i), b = ld16<NT>(g + 16 * (i + kThreads));
      v4u c = ld16<NT>(g + 16 * (i + 2 * kThreads)), d = ld16<NT>(g + 16 * (i + 3 * kThreads));
      l16[i] = a; l16[i + kThreads] = b; l16[i + 2 * kThreads] = c; l16[i + 3 * kThreads] = d;
    }
  }
  for (; i < n16; i += kThreads) {
    if (kToGlobal) st16<NT>(g + 16 * i, l16[i]);
    else l16[i] = ld16<NT>(g + 16 * i);
  }
  if ((bytes & 15) && threadIdx.x == 0) {
    uint64_t* g8 = reinterpret_cast<uint64_t*>(g + (n16 << 4));
    uint64_t* l8 = reinterpret_cast<uint64_t*>(lds + (n16 << 4));
    if (kToGlobal) *g8 = *l8;
    else *l8 = *g8;
  }
}

// kFast: every column is 8 bytes wide and no column carries validity.
template <int R, bool kFast, int NT>
__global__ __launch_bounds__(kThreads) void encode_fixed_kernel(FixedArgs a,
                                                                 uint8_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  const int nr = static_cast<int>(min(static_cast<int64_t>(R), a.nrows - r0));
  const int rs = a.row_size;
  const int bm = a.bitmap_bytes;
  const int bw = bm >> 3;

  // BinaryRowWriter.reset(): zero the bitmap words of every row of the tile.
  for (int i = threadIdx.x; i < R * bw; i += kThreads) {
    const int r = i / bw, w = i - r * bw;
    *reinterpret_cast<uint64_t*>(lds + r * rs + 8 * w) = 0;
  }
  if (!kFast) __syncthreads();   // the null bits below are OR-ed into these words

  // Gather: item = c * R + r; a wave covers 64 consecutive rows of ONE column (R % 64 == 0).
  const int total = a.ncols * R;
  for (int base = threadIdx.x; base < total; base += kThreads * kUnroll) {
    uint64_t v[kUnroll];
    bool isnull[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
      const int idx = base + u * kThreads;
      const int c = __builtin_amdgcn_readfirstlane(min(idx, total - 1) / R);
      const int r = idx - c * R;
      v[u] = 0;
      isnull[u] = false;
      if (idx < total && r < nr) {
        const int64_t row = r0 + r;
        if (kFast) {
          v[u] = ld8<NT>(a.col[c].values + row * 8);
        } else {
          const uint8_t* vb = a.col[c].validity;
          if (vb && !((vb[row >> 3] >> (row & 7)) & 1)) {
            isnull[u] = true;
          } else {
            v[u] = load_value(a.col[c].values, row, a.col[c].width);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
      const int idx = base + u * kThreads;
      const int c = __builtin_amdgcn_readfirstlane(min(idx, total - 1) / R);
      const int r = idx - c * R;
      if (idx < total && r < nr) {
        uint8_t* rowp = lds + r * rs;
        *reinterpret_cast<uint64_t*>(rowp + bm + 8 * c) = v[u];
        if (!kFast && isnull[u]) {
          atomicOr(reinterpret_cast<uint32_t*>(rowp) + (c >> 5), 1u << (c & 31));
        }
      }
    }
  }
  __syncthreads();
  copy_tile<true, NT>(rows + r0 * rs, lds, static_cast<int64_t>(nr) * rs);
}

template <int R, bool kFast, int NT>
__global__ __launch_bounds__(kThreads) void decode_fixed_kernel(FixedArgs a,
                                                                 const uint8_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  const int nr = static_cast<int>(min(static_cast<int64_t>(R), a.nrows - r0));
  const int rs = a.row_size;
  const int bm = a.bitmap_bytes;

  copy_tile<false, NT>(const_cast<uint8_t*>(rows + r0 * rs), lds, static_cast<int64_t>(nr) * rs);
  __syncthreads();

  const int total = a.ncols * R;
  const int lane = threadIdx.x & 63;
  for (int base = threadIdx.x; base < total; base += kThreads * kUnroll) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
      const int idx = base + u * kThreads;
      if (__builtin_amdgcn_readfirstlane(idx - lane) >= total) break;   // wave-uniform exit
      const int c = __builtin_amdgcn_readfirstlane(idx / R);
      const int r = idx - c * R;
      const bool live = r < nr;
      const uint8_t* rowp = lds + r * rs;
      const int64_t row = r0 + r;
      if (kFast) {
        if (live) {
          uint64_t v = *reinterpret_cast<const uint64_t*>(rowp + bm + 8 * c);
          st8<NT>(const_cast<uint8_t*>(a.col[c].values) + row * 8, v);
        }
        continue;
      }
      bool isnull = live && ((rowp[c >> 3] >> (c & 7)) & 1);
      uint64_t v = 0;
      if (live && !isnull) v = *reinterpret_cast<const uint64_t*>(rowp + bm + 8 * c);
      const int w = a.col[c].width;
      uint8_t* dst = const_cast<uint8_t*>(a.col[c].values);
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
      uint8_t* vb = a.col[c].validity;
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

int fixed_variant() {
  if (g_variant < 0) {
    const char* e = getenv("FURY_FIXED_VARIANT");
    g_variant = e ? atoi(e) : 6;   // tile kernel + nt loads + nt stores (A/B: profiles/r01_ab_fixed.json)
  }
  return g_variant;
}

void set_fixed_variant(int v) { g_variant = v; }

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

}  // namespace

// Variant bits (fury_set_tuning("fixed_variant")): bit 0 = pipelined persistent kernel,
// bit 1 = non-temporal stores, bit 2 = non-temporal loads.  Only the fast path (8-byte columns,
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
