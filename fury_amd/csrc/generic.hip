// generic.hip — schema-interpreting kernels for ANY schema the reference row format supports:
// nested STRUCT (bean fields), LIST of any element type (incl. strings, structs, lists, maps),
// MAP (key / value arrays), plus every scalar type.  The specialised kernels in fixed.hip /
// var.hip cover flat schemas at full speed; this engine covers the rest of the type system.
//
// Reference semantics (FMT = java/fury-format/src/main/java/org/apache/fury/format):
//   encode   BaseBinaryEncoderBuilder.serializeFor (FMT/encoder/BaseBinaryEncoderBuilder.java:
//            138-453): primitives into 8-byte slots, var values appended at the writer index and
//            padded to 8 (BinaryWriter.java:106-121,187-194), List -> BinaryArrayWriter image
//            [int64 n][bitmap][n x elemSize, tail zeroed][var section] (BinaryArrayWriter.java:
//            91-163), bean -> child BinaryRowWriter row (:363-417), Map -> [int64 keyBytes]
//            [key array][value array] (:298-357); null -> setNullAt only.
//   decode   getters + ArrowWriter (FMT/vectorized/ArrowWriter.java:205-640): a null struct
//            appends a null to every child (StructWriter.appendNull :577-584), null lists/maps
//            are zero-length entries (ListWriter/MapWriter.appendNull no-op + fillHoles).
//
// MI355X design: the flattened schema and the per-call column pointers travel in the kernel
// argument block (scalar-loaded).  Encode is one thread per row (measure pass -> device scan ->
// build pass).  Recursion is depth-unrolled (template<int D>), at most kMaxDepth levels of
// nesting.  Decode is levels.hip (level by level, a thread per Arrow entry); the round-1/2
// thread-per-row decode interpreter that lived here was removed in round 3.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

constexpr int kEncThreads = 256;

__device__ __forceinline__ bool gbit(const uint8_t* bits, int64_t i) {
  return (gl(bits)[i >> 3] >> (i & 7)) & 1;
}
__device__ __forceinline__ int64_t g8(int64_t n) { return (n + 7) & ~int64_t(7); }
__device__ __forceinline__ int64_t gbm(int64_t n) { return ((n + 63) >> 6) << 3; }

__device__ __forceinline__ int gwidth(int t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

// Typed accesses.  Row images are built in LDS (LdsU8) or, past the image, straight in HBM
// (uint8_t*: always device memory here); input columns and rows are device memory.  With the
// address space explicit the compiler emits ds_* / global_* instead of flat_* (a flat access
// counts against both vmcnt and lgkmcnt, so each wait waited for both).
template <class T>
using Lds = __attribute__((address_space(3))) T;
using LdsU8 = Lds<uint8_t>;

__device__ __forceinline__ void st8(uint8_t* p, uint64_t v) {   // p 8-aligned by construction
  *gl(reinterpret_cast<uint64_t*>(p)) = v;
}
__device__ __forceinline__ void st8(LdsU8* p, uint64_t v) { *reinterpret_cast<Lds<uint64_t>*>(p) = v; }
__device__ __forceinline__ void st4(uint8_t* p, uint32_t v) { *gl(reinterpret_cast<uint32_t*>(p)) = v; }
__device__ __forceinline__ void st4(LdsU8* p, uint32_t v) { *reinterpret_cast<Lds<uint32_t>*>(p) = v; }
__device__ __forceinline__ void st2(uint8_t* p, uint16_t v) { *gl(reinterpret_cast<uint16_t*>(p)) = v; }
__device__ __forceinline__ void st2(LdsU8* p, uint16_t v) { *reinterpret_cast<Lds<uint16_t>*>(p) = v; }
__device__ __forceinline__ void st1(uint8_t* p, uint8_t v) { *gl(p) = v; }
__device__ __forceinline__ void st1(LdsU8* p, uint8_t v) { *p = v; }
__device__ __forceinline__ void or1(uint8_t* p, uint8_t v) { *gl(p) |= v; }
__device__ __forceinline__ void or1(LdsU8* p, uint8_t v) { *p |= v; }
__device__ __forceinline__ uint64_t ld8(const uint8_t* p) {
  return *gl(reinterpret_cast<const uint64_t*>(p));
}

// Copies len bytes from an 8-byte aligned source (a row's var section) to any destination:
// bytes up to the destination's 8-byte boundary, then whole 8-byte stores of funnel-shifted
// source words, then the tail bytes.  Only [dst, dst + len) is written (neighbouring threads
// own the bytes around it).
__device__ __forceinline__ void copy_to_unaligned(uint8_t* dst, const uint8_t* src, int64_t len) {
  if (len <= 0) return;
  const int64_t head = min<int64_t>(len, (8 - (reinterpret_cast<uintptr_t>(dst) & 7)) & 7);
  for (int64_t t = 0; t < head; t++) dst[t] = src[t];
  const int64_t body = (len - head) >> 3;
  const uint64_t* s64 = reinterpret_cast<const uint64_t*>(src);
  const int sh = static_cast<int>(head) * 8;           // source bit offset of the body
  uint64_t* d64 = reinterpret_cast<uint64_t*>(dst + head);
  for (int64_t w = 0; w < body; w++) {
    const uint64_t lo = s64[w];
    const uint64_t v = sh ? (lo >> sh) | (s64[w + 1] << (64 - sh)) : lo;
    d64[w] = v;
  }
  for (int64_t t = head + 8 * body; t < len; t++) dst[t] = src[t];
}

// ---- encode ----------------------------------------------------------------------------------

template <class P>
__device__ __forceinline__ void zero_bytes(P p, int64_t n) {
  // 8-byte aligned start; n multiple of 8 in every use
  for (int64_t i = 0; i < n; i += 8) st8(p + i, 0);
}

// Appends len bytes (unaligned source) at dst (8-aligned), zero-padding to 8.
template <class P>
__device__ __forceinline__ void append_unaligned(P dst, const uint8_t* src, int64_t len) {
  // aligned source words funnel-shifted into place; no word past the last source byte is read
  const uintptr_t so = reinterpret_cast<uintptr_t>(src) & 7;
  const auto ap = gl(reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(src) - so));
  const int64_t nw = (len + 7) >> 3;
  const int64_t nsrc = (static_cast<int64_t>(so) + len + 7) >> 3;
  const int sh = static_cast<int>(so) * 8;
  uint64_t cur = nsrc > 0 ? ap[0] : 0;
  for (int64_t w = 0; w < nw; w++) {
    const uint64_t nxt = w + 1 < nsrc ? ap[w + 1] : 0;
    uint64_t x = sh ? (cur >> sh) | (nxt << (64 - sh)) : cur;
    const int64_t rem = len - 8 * w;
    if (rem < 8) x &= (~0ull) >> (8 * (8 - rem));
    st8(dst + 8 * w, x);
    cur = nxt;
  }
}

template <int D, bool W, class P, class NP>
__device__ void put_value(NP nodes, int ni, int64_t idx, P buf, int64_t container,
                          int64_t slot, int es, bool in_array, int64_t bitmap, int64_t ordinal,
                          int64_t& cursor);

// BinaryArrayWriter image of elements [b, b + m) of node `ei` at buf + cursor.
template <int D, bool W, class P, class NP>
__device__ void put_array(NP nodes, int ei, int64_t b, int64_t m, P buf,
                          int64_t& cursor) {
  const auto& e = nodes[ei];
  const int w = gwidth(e.type);
  const int es = w > 0 ? w : 8;
  const int64_t start = cursor;
  const int64_t hb = 8 + gbm(m);
  const int64_t fp = g8(m * es);
  if (W) {
    st8(buf + start, static_cast<uint64_t>(m));
    zero_bytes(buf + start + 8, hb - 8 + fp);     // bitmap, element slots, alignment tail
  }
  int64_t c2 = start + hb + fp;
  for (int64_t j = 0; j < m; j++)
    put_value<D + 1, W>(nodes, ei, b + j, buf, start, start + hb + j * es, es, true, start + 8, j, c2);
  cursor = c2;
}

template <int D, bool W, class P, class NP>
__device__ void put_value(NP nodes, int ni, int64_t idx, P buf, int64_t container,
                          int64_t slot, int es, bool in_array, int64_t bitmap, int64_t ordinal,
                          int64_t& cursor) {
  if constexpr (D >= kGenMaxDepth) {
    (void)nodes;
    return;
  } else {
    const auto& n = nodes[ni];
    if (n.validity && !gbit(n.validity, idx)) {      // setNullAt: bit only, slot stays 0
      if (W) or1(buf + bitmap + (ordinal >> 3), static_cast<uint8_t>(1u << (ordinal & 7)));
      return;
    }
    const int w = gwidth(n.type);
    if (w > 0) {
      if (W) {
        uint64_t v;
        if (n.type == FURY_TYPE_BOOL) v = gbit(n.values, idx);
        else if (w == 8) v = ld8(n.values + idx * 8);
        else if (w == 4) v = *gl(reinterpret_cast<const uint32_t*>(n.values + idx * 4));
        else if (w == 2) v = *gl(reinterpret_cast<const uint16_t*>(n.values + idx * 2));
        else v = gl(n.values)[idx];
        if (!in_array) {
          st8(buf + slot, v);                           // putInt64(0) + narrow put
        } else {
          switch (es) {
            case 8: st8(buf + slot, v); break;
            case 4: st4(buf + slot, static_cast<uint32_t>(v)); break;
            case 2: st2(buf + slot, static_cast<uint16_t>(v)); break;
            default: st1(buf + slot, static_cast<uint8_t>(v)); break;
          }
        }
      }
      return;
    }
    const int64_t start = cursor;
    switch (n.type) {
      case FURY_TYPE_STRING:
      case FURY_TYPE_BINARY: {
        const int64_t b = gl(n.offsets)[idx];
        const int64_t len = gl(n.offsets)[idx + 1] - b;
        if (W) append_unaligned(buf + start, n.values + b, len);
        cursor = start + g8(len);
        if (W) st8(buf + slot, (static_cast<uint64_t>(start - container) << 32) | static_cast<uint32_t>(len));
        return;
      }
      case FURY_TYPE_DECIMAL: {
        if (W) {
          st8(buf + start, ld8(n.values + 16 * idx));
          st8(buf + start + 8, ld8(n.values + 16 * idx + 8));
          st8(buf + slot, (static_cast<uint64_t>(start - container) << 32) | 16u);
        }
        cursor = start + 16;
        return;
      }
      case FURY_TYPE_LIST: {
        const int64_t b = gl(n.offsets)[idx];
        put_array<D, W>(nodes, n.first_child, b, gl(n.offsets)[idx + 1] - b, buf, cursor);
        break;
      }
      case FURY_TYPE_STRUCT: {
        const int nc = n.num_children;
        const int64_t bmb = gbm(nc);
        const int64_t fixed = bmb + 8 * nc;
        if (W) zero_bytes(buf + start, fixed);
        int64_t c2 = start + fixed;
        for (int k = 0; k < nc; k++)
          put_value<D + 1, W>(nodes, n.first_child + k, idx, buf, start, start + bmb + 8 * k, 8, false,
                              start, k, c2);
        cursor = c2;
        break;
      }
      case FURY_TYPE_MAP: {
        const int64_t b = gl(n.offsets)[idx];
        const int64_t m = gl(n.offsets)[idx + 1] - b;
        int64_t c2 = start + 8;                         // writeDirectly(-1) placeholder
        put_array<D, W>(nodes, n.first_child, b, m, buf, c2);
        if (W) st8(buf + start, static_cast<uint64_t>(c2 - (start + 8)));   // key array size
        put_array<D, W>(nodes, n.first_child + 1, b, m, buf, c2);
        cursor = c2;
        break;
      }
      default:
        
        return;
    }
    if (W) st8(buf + slot, (static_cast<uint64_t>(start - container) << 32) |
                               static_cast<uint32_t>(cursor - start));
  }
}

// Entry r of the batch: a row of the ntop top-level fields (root 0), or -- ArrayEncoder.toArray /
// MapEncoder.toMap (ArrayEncoderBuilder.java:118-140, MapEncoderBuilder.java:152-208) -- the
// top-level BinaryArray (root 1) / BinaryMap [int64 keyBytes][keys][values] (root 2) of node 0's
// entry r, written at the buffer start exactly as inside a row (element offsets are relative to
// the array itself).
template <bool W, int kRoot, class P, class NP>
__device__ int64_t put_row(NP nodes, int ntop, int64_t r, P buf) {
  constexpr int root = kRoot;
  if constexpr (kRoot != 0) {
    const auto& n = nodes[0];
    const int64_t b = gl(n.offsets)[r];
    const int64_t m = gl(n.offsets)[r + 1] - b;
    int64_t cursor = root == 2 ? 8 : 0;
    put_array<1, W>(nodes, n.first_child, b, m, buf, cursor);
    if (root == 2) {
      if (W) st8(buf, static_cast<uint64_t>(cursor - 8));      // key array bytes
      put_array<1, W>(nodes, n.first_child + 1, b, m, buf, cursor);
    }
    return cursor;
  }
  const int64_t bmb = gbm(ntop);
  const int64_t fixed = bmb + 8 * ntop;
  if (W) zero_bytes(buf, fixed);                       // fresh buffer: bitmap + slots zero
  int64_t cursor = fixed;
  for (int k = 0; k < ntop; k++)
    put_value<1, W>(nodes, k, r, buf, 0, bmb + 8 * k, 8, false, 0, k, cursor);
  return cursor;
}

// The node table is copied from the argument block into LDS once per workgroup and passed to
// the (non-inlined, recursive-by-depth) helpers as a pointer: taking the address of the kernel
// argument itself would make the compiler copy the whole block into per-lane scratch.  Schemas
// with more nodes than the argument block holds (kWide) read the table the host uploaded for the
// call straight from device memory (uniform indices: scalar loads).
template <bool kWide>
__device__ __forceinline__ const GenNode* stage_nodes(const GenArgs& g, GenNode* lds) {
  if (kWide) return g.tab;
  for (int i = threadIdx.x; i < g.nnodes; i += blockDim.x) lds[i] = g.node[i];
  __syncthreads();
  return lds;
}

// The encode side's node table with its address space explicit (LDS copy / uploaded table).
using GNodes = __attribute__((address_space(1))) const GenNode*;
using LNodes = Lds<const GenNode>*;
template <bool kWide>
__device__ __forceinline__ auto enc_nodes(const GenArgs& g, GenNode* lds) {
  const GenNode* p = stage_nodes<kWide>(g, lds);
  if constexpr (kWide) return (GNodes)(p);
  else return (LNodes)(p);
}

// kRoot (fury_schema.root) is a template parameter so the row kernels do not carry the
// collection code: inlining both into one kernel raised its scratch from 192 to 1200 B per lane
// and doubled the encode time.
template <bool kWide, int kRoot>
__global__ __launch_bounds__(kEncThreads) void gen_measure_kernel(GenArgs g, int64_t* __restrict__ sizes) {
  __shared__ GenNode sn[kWide ? 1 : kGenMaxNodes];
  const auto nodes = enc_nodes<kWide>(g, sn);
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kEncThreads + threadIdx.x;
  if (r < g.nrows) sizes[r] = put_row<false, kRoot>(nodes, g.ntop, r, static_cast<uint8_t*>(nullptr));
}

// The workgroup's 256 rows are one contiguous byte range of the output: each thread builds its
// row in an LDS image of that range (put_row writes every byte of a row: zeroed bitmaps and
// slots, zero-padded variable parts), then the workgroup stores the range with coalesced 8-byte
// stores.  Thread-per-row stores straight to HBM wrote ~5x the row bytes (WRITE_SIZE of the
// depth-3 schema at 4M rows: partial lines of 64 rows at a time, evicted before they filled).
// A tile larger than the image (or past `cap`) takes the direct path.
constexpr int64_t kGenImg = 76 * 1024;

template <bool kWide, int kRoot>
__global__ __launch_bounds__(kEncThreads, 2) void gen_encode_kernel(GenArgs g,
                                                                 const int64_t* __restrict__ offs,
                                                                 uint8_t* __restrict__ rows,
                                                                 int64_t cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t img[];
  __shared__ GenNode sn[kWide ? 1 : kGenMaxNodes];
  const auto nodes = enc_nodes<kWide>(g, sn);
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kEncThreads;
  const int64_t r = r0 + threadIdx.x;
  const int64_t rend = min(r0 + kEncThreads, g.nrows);
  const int64_t b0 = offs[r0], b1 = offs[rend];
  if (b1 - b0 <= kGenImg && b1 <= cap) {
    if (r < g.nrows) put_row<true, kRoot>(nodes, g.ntop, r, (LdsU8*)(img + (offs[r] - b0)));
    __syncthreads();
    const uint64_t* s = reinterpret_cast<const uint64_t*>(img);
    uint64_t* d = reinterpret_cast<uint64_t*>(rows + b0);
    for (int64_t i = threadIdx.x; i < (b1 - b0) >> 3; i += kEncThreads) d[i] = s[i];
    return;
  }
  if (r < g.nrows && offs[r + 1] <= cap) put_row<true, kRoot>(nodes, g.ntop, r, rows + offs[r]);
}

}  // namespace

template <bool kWide, int kRoot>
void gen_encode_pass(const GenArgs& g, const int64_t* offs, int64_t* sizes, uint8_t* rows,
                     int64_t cap, hipStream_t stream) {
  const int64_t blocks = (g.nrows + kEncThreads - 1) / kEncThreads;
  if (sizes) {
    hipLaunchKernelGGL((gen_measure_kernel<kWide, kRoot>), dim3(blocks), dim3(kEncThreads), 0,
                       stream, g, sizes);
    return;
  }
  static const bool lds_ok = hipFuncSetAttribute(
      reinterpret_cast<const void*>(gen_encode_kernel<kWide, kRoot>),
      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kGenImg)) == hipSuccess;
  (void)lds_ok;
  hipLaunchKernelGGL((gen_encode_kernel<kWide, kRoot>), dim3(blocks), dim3(kEncThreads), kGenImg,
                     stream, g, offs, rows, cap);
}

template <bool kWide>
void gen_encode_root(const GenArgs& g, const int64_t* offs, int64_t* sizes, uint8_t* rows,
                     int64_t cap, hipStream_t stream) {
  switch (g.root) {
    case 1: return gen_encode_pass<kWide, 1>(g, offs, sizes, rows, cap, stream);
    case 2: return gen_encode_pass<kWide, 2>(g, offs, sizes, rows, cap, stream);
    default: return gen_encode_pass<kWide, 0>(g, offs, sizes, rows, cap, stream);
  }
}

int launch_gen_measure(const GenArgs& g, int64_t* sizes, hipStream_t stream) {
  if (g.tab) gen_encode_root<true>(g, nullptr, sizes, nullptr, 0, stream);
  else gen_encode_root<false>(g, nullptr, sizes, nullptr, 0, stream);
  return check_hip(hipGetLastError(), "gen_measure launch");
}

int launch_gen_encode(const GenArgs& g, const int64_t* offs, uint8_t* rows, int64_t cap,
                      hipStream_t stream) {
  if (g.tab) gen_encode_root<true>(g, offs, nullptr, rows, cap, stream);
  else gen_encode_root<false>(g, offs, nullptr, rows, cap, stream);
  return check_hip(hipGetLastError(), "gen_encode launch");
}

}  // namespace fury
