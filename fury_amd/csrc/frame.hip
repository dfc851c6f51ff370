// frame.hip — the row stream framing of RowEncoder.encode(MemoryBuffer, T) / decode(MemoryBuffer)
// (FMT/encoder/Encoders.java:165-182,201-213): every row travels as
//   [int32 len = 8 + rowSize][int64 schemaHash][row bytes]
// Frame i starts at rowOffset(i) + 12 * i, so frames are 4-byte aligned relative to the stream
// start and every Fury row size is a multiple of 8 (BinaryWriter pads to words).
//
// Parsing a stream back is inherently a chain (frame i's position depends on every earlier
// length); walking it with one lane costs one dependent HBM round trip per frame.  The device
// parse instead speculates and verifies:
//   mark    every 4-aligned stream position is tested as a frame header (schema hash at +4, length
//           >= 8, a multiple of 8, inside the stream): one coalesced read of the stream, one
//           candidate bit per word and a candidate count per workgroup;
//   scan    device exclusive scan of the counts;
//   emit    the first nrows candidate positions in stream order;
//   verify  candidate 0 is at 0 and candidate k + 1 is exactly where frame k ends, for all k
//           (then candidate k IS frame k, by induction); row offset k = position k - 12 k;
//   copy    rows, 8 B per lane, into the contiguous row buffer (skips itself unless verified).
// A stream that fails verification (payload bytes that happen to look like a header, a frame
// with the wrong schema hash, a truncated stream, an unaligned buffer) is re-parsed by the
// sequential walk, which reports exactly the errors Encoders.decode raises.  Results are
// therefore identical to the sequential walk's on every input.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

constexpr int kThreads = 256;
constexpr int kMarkWords = 8;                       // stream words (4 B) per lane in the mark pass
constexpr int kMarkSpan = kThreads * kMarkWords;    // words per workgroup
constexpr int kCopyFrames = 256;                    // frames per workgroup in the copy pass

// Encoders.encode(MemoryBuffer, T) for each row: a wave per row, 4-byte word copy.
__global__ __launch_bounds__(kThreads) void frame_kernel(const uint8_t* __restrict__ rows,
                                                         const int64_t* __restrict__ offs,
                                                         int64_t n, int64_t fixed,
                                                         int64_t hash, uint8_t* __restrict__ out,
                                                         int64_t* __restrict__ fo) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const int64_t b = offs ? offs[i] : i * fixed;
  const int64_t e = offs ? offs[i + 1] : (i + 1) * fixed;
  const int64_t start = b + 12 * i;
  uint32_t* o = reinterpret_cast<uint32_t*>(out + start);
  if (lane == 0) {
    o[0] = static_cast<uint32_t>(8 + (e - b));
    o[1] = static_cast<uint32_t>(hash);
    o[2] = static_cast<uint32_t>(static_cast<uint64_t>(hash) >> 32);
    if (fo) {
      fo[i] = start;
      if (i == n - 1) fo[n] = start + 12 + (e - b);
    }
  }
  const uint32_t* s = reinterpret_cast<const uint32_t*>(rows + b);
  for (int64_t w = lane; w < ((e - b) >> 2); w += 64) o[3 + w] = s[w];
}

// ---- sequential walk (reference semantics, fallback) -------------------------------------------
// Encoders.decode(MemoryBuffer): readInt32 len, readInt64 hash (ClassNotCompatibleException on a
// mismatch), row = next len - 8 bytes.  One lane.
__global__ void unframe_walk(const uint8_t* __restrict__ in, int64_t len, int64_t n, int64_t hash,
                             int64_t* __restrict__ frame_pos, int64_t* __restrict__ row_offs,
                             int32_t* __restrict__ err) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t pos = 0, out = 0;
  for (int64_t i = 0; i < n; i++) {
    if (pos + 12 > len) { *err = 2; return; }
    int32_t l;
    int64_t h;
    memcpy(&l, in + pos, 4);
    memcpy(&h, in + pos + 4, 8);
    if (h != hash) { *err = 1; return; }
    if (l < 8 || pos + 4 + l > len) { *err = 2; return; }
    frame_pos[i] = pos;
    row_offs[i] = out;
    out += l - 8;
    pos += 4 + l;
  }
  row_offs[n] = out;
}

__global__ __launch_bounds__(kThreads) void unframe_copy_walked(const uint8_t* __restrict__ in,
                                                                const int64_t* __restrict__ frame_pos,
                                                                const int64_t* __restrict__ row_offs,
                                                                int64_t n, uint8_t* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(in + frame_pos[i] + 12);
  uint32_t* d = reinterpret_cast<uint32_t*>(out + row_offs[i]);
  const int64_t words = (row_offs[i + 1] - row_offs[i]) >> 2;
  for (int64_t w = lane; w < words; w += 64) d[w] = s[w];
}

// ---- speculative parallel parse -----------------------------------------------------------------
__device__ __forceinline__ int block_sum(int x) {
  __shared__ int part[kThreads / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = x;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; w++) s += part[w];
  return s;
}

// Exclusive prefix of x over the workgroup (thread order).
__device__ __forceinline__ int block_excl_scan(int x) {
  __shared__ int part[kThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) part[wid] = inc;
  __syncthreads();
  int before = 0;
  for (int w = 0; w < wid; w++) before += part[w];
  return before + inc - x;
}

// Candidate bits: bit j of mask[g] = stream word kMarkWords * g + j starts a plausible header.
// The stream base is 16-byte aligned (checked on the host).
__global__ __launch_bounds__(kThreads) void unframe_mark(const uint32_t* __restrict__ in,
                                                         int64_t len, int64_t hash,
                                                         uint8_t* __restrict__ mask,
                                                         int64_t* __restrict__ counts) {
  const int64_t W = len >> 2;
  const int64_t g = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  const int64_t w0 = g * kMarkWords;
  uint32_t x[kMarkWords + 2];
  if (w0 + kMarkWords + 2 <= W) {
    using v4u = __attribute__((ext_vector_type(4))) uint32_t;
    const v4u a = *reinterpret_cast<const v4u*>(in + w0);
    const v4u b = *reinterpret_cast<const v4u*>(in + w0 + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
    x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    x[8] = in[w0 + 8];
    x[9] = in[w0 + 9];
  } else {
#pragma unroll
    for (int j = 0; j < kMarkWords + 2; j++) x[j] = w0 + j < W ? in[w0 + j] : 0u;
  }
  const uint32_t hlo = static_cast<uint32_t>(hash);
  const uint32_t hhi = static_cast<uint32_t>(static_cast<uint64_t>(hash) >> 32);
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < kMarkWords; j++) {
    const int64_t p = 4 * (w0 + j);
    const uint32_t l = x[j];
    const bool hdr = (w0 + j + 3 <= W) && x[j + 1] == hlo && x[j + 2] == hhi &&
                     static_cast<int32_t>(l) >= 8 && (l & 7) == 0 &&
                     p + 4 + static_cast<int64_t>(l) <= len;
    bits |= hdr ? (1u << j) : 0u;
  }
  mask[g] = static_cast<uint8_t>(bits);
  const int total = block_sum(__popc(bits));
  if (threadIdx.x == 0) counts[blockIdx.x] = total;
}

// The first n candidates' stream positions, in stream order (counts = exclusive prefix).
__global__ __launch_bounds__(kThreads) void unframe_emit(const uint8_t* __restrict__ mask,
                                                         const int64_t* __restrict__ counts,
                                                         int64_t n, int64_t* __restrict__ cand) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  uint32_t bits = mask[g];
  int64_t k = counts[blockIdx.x] + block_excl_scan(__popc(bits));
  const int64_t w0 = g * kMarkWords;
  while (bits && k < n) {
    const int j = __builtin_ctz(bits);
    cand[k++] = 4 * (w0 + j);
    bits &= bits - 1;
  }
}

// Candidate k is frame k iff candidate 0 is at 0 and each candidate ends where the next begins.
__global__ __launch_bounds__(kThreads) void unframe_verify(const uint8_t* __restrict__ in,
                                                           const int64_t* __restrict__ cand,
                                                           const int64_t* __restrict__ total,
                                                           int64_t n, int64_t* __restrict__ row_offs,
                                                           int32_t* __restrict__ err) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (k >= n) return;
  if (*total < n) {                  // fewer candidates than frames: not a clean stream
    if (k == 0) atomicOr(err, 4);
    return;
  }
  const int64_t p = cand[k];
  const int64_t end = p + 4 + *reinterpret_cast<const int32_t*>(in + p);
  bool ok = k != 0 || p == 0;
  if (k + 1 < n) ok = ok && cand[k + 1] == end;
  row_offs[k] = p - 12 * k;
  if (k == n - 1) row_offs[n] = end - 12 * n;
  if (!ok) atomicOr(err, 4);
}

// Rows out of a verified stream: each workgroup owns kCopyFrames frames = one contiguous range of
// the row buffer; a lane moves 8 B (its frame found by binary search over the range's row
// offsets in LDS), so the row-buffer stores are fully coalesced.
__global__ __launch_bounds__(kThreads) void unframe_copy(const uint8_t* __restrict__ in,
                                                         const int64_t* __restrict__ cand,
                                                         const int64_t* __restrict__ row_offs,
                                                         int64_t n, uint8_t* __restrict__ out,
                                                         const int32_t* __restrict__ err) {
  if (*err) return;                  // speculation failed: the sequential walk takes over
  __shared__ int64_t ro[kCopyFrames + 1];
  __shared__ int64_t src[kCopyFrames];
  const int64_t k0 = static_cast<int64_t>(blockIdx.x) * kCopyFrames;
  const int kn = static_cast<int>(min(static_cast<int64_t>(kCopyFrames), n - k0));
  for (int f = threadIdx.x; f <= kn; f += kThreads) {
    ro[f] = row_offs[k0 + f];
    if (f < kn) src[f] = cand[k0 + f] + 12;
  }
  __syncthreads();
  const int64_t base = ro[0];
  const int64_t words = (ro[kn] - base) >> 3;
  for (int64_t q = threadIdx.x; q < words; q += kThreads) {
    const int64_t d = base + 8 * q;
    int lo = 0, hi = kn - 1;
    while (lo < hi) {                 // last frame whose row starts at or before d
      const int mid = (lo + hi + 1) >> 1;
      if (ro[mid] <= d) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t* s = reinterpret_cast<const uint32_t*>(in + src[lo] + (d - ro[lo]));
    const uint64_t v = static_cast<uint64_t>(s[0]) | (static_cast<uint64_t>(s[1]) << 32);
    *reinterpret_cast<uint64_t*>(out + d) = v;
  }
}

std::atomic<int64_t> g_unframe_walks{0};   // streams parsed by the sequential walk
int g_unframe_mode = 0;                     // tuning "unframe": 0 speculative, 1 always walk

int unframe_walked(const uint8_t* in, int64_t len, int64_t n, int64_t hash, uint8_t* rows_out,
                   int64_t* row_offs, hipStream_t stream) {
  g_unframe_walks.fetch_add(1);
  int64_t* fp = nullptr;
  int st = check_hip(hipMallocAsync(reinterpret_cast<void**>(&fp), n * 8 + 8, stream),
                     "hipMallocAsync");
  if (st) return st;
  int32_t* err = reinterpret_cast<int32_t*>(fp + n);
  (void)hipMemsetAsync(err, 0, 4, stream);
  hipLaunchKernelGGL(unframe_walk, dim3(1), dim3(64), 0, stream, in, len, n, hash, fp, row_offs,
                     err);
  int32_t herr = 0;
  (void)hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, stream);
  st = check_hip(hipStreamSynchronize(stream), "unframe sync");
  if (!st && herr == 0 && n > 0) {
    const int64_t blocks = (n + (kThreads / 64) - 1) / (kThreads / 64);
    hipLaunchKernelGGL(unframe_copy_walked, dim3(blocks), dim3(kThreads), 0, stream, in, fp,
                       row_offs, n, rows_out);
    st = check_hip(hipGetLastError(), "unframe copy launch");
  }
  (void)hipFreeAsync(fp, stream);
  if (st) return st;
  if (herr == 1)
    return set_error(FURY_ERR_CLASS_NOT_COMPATIBLE,
                     "Schema is not consistent: peer schema hash differs from " +
                         std::to_string(hash));
  if (herr == 2) return set_error(FURY_ERR_OUT_OF_BOUNDS, "frame runs past the end of the stream");
  return FURY_OK;
}

}  // namespace

int unframe_mode() { return g_unframe_mode; }
void set_unframe_mode(int v) { g_unframe_mode = v; }
int64_t unframe_walk_count() { return g_unframe_walks.load(); }

int launch_frame_rows(const uint8_t* rows, const int64_t* offs, int64_t n, int64_t fixed,
                      int64_t hash, uint8_t* out, int64_t* fo, hipStream_t stream) {
  if (n == 0) return FURY_OK;
  const int64_t blocks = (n + (kThreads / 64) - 1) / (kThreads / 64);
  hipLaunchKernelGGL(frame_kernel, dim3(blocks), dim3(kThreads), 0, stream, rows, offs, n, fixed,
                     hash, out, fo);
  return check_hip(hipGetLastError(), "frame launch");
}

int launch_unframe_rows(const uint8_t* in, int64_t len, int64_t n, int64_t hash, uint8_t* rows_out,
                        int64_t* row_offs, hipStream_t stream) {
  const bool aligned = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
  if (n == 0 || len < 12 || !aligned || g_unframe_mode == 1)
    return unframe_walked(in, len, n, hash, rows_out, row_offs, stream);
  const int64_t W = len >> 2;
  const int64_t nb = (W + kMarkSpan - 1) / kMarkSpan;
  if (nb > 0x7fffffff) return set_error(FURY_ERR_INVALID_ARGUMENT, "stream too large");
  // workspace: [cand n][counts nb][total][scan ws][err (8 B)][mask nb * kThreads bytes]
  const int64_t ws_n = scan_workspace(nb);
  const int64_t words = n + nb + 1 + ws_n + 1;
  uint8_t* buf = nullptr;
  int st = check_hip(hipMallocAsync(reinterpret_cast<void**>(&buf), words * 8 + nb * kThreads,
                                    stream), "hipMallocAsync");
  if (st) return st;
  int64_t* cand = reinterpret_cast<int64_t*>(buf);
  int64_t* counts = cand + n;
  int64_t* total = counts + nb;
  int64_t* ws = total + 1;
  int32_t* err = reinterpret_cast<int32_t*>(ws + ws_n);
  uint8_t* mask = buf + words * 8;
  (void)hipMemsetAsync(err, 0, 4, stream);
  hipLaunchKernelGGL(unframe_mark, dim3(nb), dim3(kThreads), 0, stream,
                     reinterpret_cast<const uint32_t*>(in), len, hash, mask, counts);
  device_scan(counts, nb, total, ws, stream);
  hipLaunchKernelGGL(unframe_emit, dim3(nb), dim3(kThreads), 0, stream, mask, counts, n, cand);
  const int64_t vb = (n + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(unframe_verify, dim3(vb), dim3(kThreads), 0, stream, in, cand, total, n,
                     row_offs, err);
  const int64_t cb = (n + kCopyFrames - 1) / kCopyFrames;
  hipLaunchKernelGGL(unframe_copy, dim3(cb), dim3(kThreads), 0, stream, in, cand, row_offs, n,
                     rows_out, err);
  st = check_hip(hipGetLastError(), "unframe launch");
  int32_t herr = 0;
  if (!st) (void)hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, stream);
  (void)hipFreeAsync(buf, stream);
  const int st2 = check_hip(hipStreamSynchronize(stream), "unframe sync");
  if (st) return st;
  if (st2) return st2;
  if (herr == 0) return FURY_OK;
  return unframe_walked(in, len, n, hash, rows_out, row_offs, stream);
}

}  // namespace fury
