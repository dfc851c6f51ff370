// frame.hip — the row stream framing of RowEncoder.encode(MemoryBuffer, T) / decode(MemoryBuffer)
// (FMT/encoder/Encoders.java:165-182,201-213): every row travels as
//   [int32 len = 8 + rowSize][int64 schemaHash][row bytes]
// Frame i starts at rowOffset(i) + 12 * i, so frames are 4-byte aligned relative to the stream
// start and every Fury row size is a multiple of 8 (BinaryWriter pads to words).
//
// Parsing a stream back is inherently a chain (frame i's position depends on every earlier
// length); walking it with one lane costs one dependent HBM round trip per frame.  The device
// parse instead speculates and verifies:
//   scan    every 4-aligned stream position is tested as a frame header (schema hash at +4,
//           length >= 8, a multiple of 8, inside the stream): one coalesced read of the stream.
//           Each workgroup counts its candidates, takes its place among them by a decoupled
//           look-back over the workgroups before it (launch order, bounded spin), and writes the
//           positions and lengths of the first nrows candidates,
//           staged through LDS so the writes are coalesced;
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

// Encoders.encode(MemoryBuffer, T) for each row.  A workgroup owns kCopyFrames consecutive rows
// = one contiguous range of the row buffer and of the stream.  The stream side is written in
// 16-byte aligned chunks (non-temporal): a lane finds the frame under its chunk by binary search
// over the range's frame starts in LDS and assembles the chunk's four dwords from the 12-byte
// header and the row's 4-byte words (a chunk spans at most two frames: a frame is >= 20 bytes);
// the unaligned head and tail of the range go out as dwords.
__global__ __launch_bounds__(kThreads) void frame_kernel(const uint8_t* __restrict__ rows,
                                                         const int64_t* __restrict__ offs,
                                                         int64_t n, int64_t fixed,
                                                         int64_t hash, uint8_t* __restrict__ out,
                                                         int64_t* __restrict__ fo) {
  __shared__ int64_t ro[kCopyFrames + 1];   // row offsets of the range's rows (+ the end)
  __shared__ int64_t st[kCopyFrames + 1];   // their frame starts in the stream (+ the end)
  const int64_t k0 = static_cast<int64_t>(blockIdx.x) * kCopyFrames;
  const int kn = static_cast<int>(min(static_cast<int64_t>(kCopyFrames), n - k0));
  for (int f = threadIdx.x; f <= kn; f += kThreads) {
    const int64_t r = offs ? offs[k0 + f] : (k0 + f) * fixed;
    ro[f] = r;
    st[f] = r + 12 * (k0 + f);
  }
  __syncthreads();
  if (fo && threadIdx.x < kn) {
    fo[k0 + threadIdx.x] = st[threadIdx.x];
    if (k0 + threadIdx.x == n - 1) fo[n] = st[kn];
  }
  const uint32_t hlo = static_cast<uint32_t>(hash);
  const uint32_t hhi = static_cast<uint32_t>(static_cast<uint64_t>(hash) >> 32);
  // stream dword at byte position q of frame f (advanced while q is past its end)
  auto dword_at = [&](int64_t q, int& f) -> uint32_t {
    while (f + 1 < kn && st[f + 1] <= q) f++;
    const int64_t rel = q - st[f];
    if (rel < 12) {
      return rel == 0 ? static_cast<uint32_t>(8 + (ro[f + 1] - ro[f])) : rel == 4 ? hlo : hhi;
    }
    return *reinterpret_cast<const uint32_t*>(rows + ro[f] + rel - 12);
  };
  auto find = [&](int64_t q) {                 // last frame that starts at or before q
    int lo = 0, hi = kn - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (st[mid] <= q) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  const int64_t S = st[0], E = st[kn];
  const uintptr_t ob = reinterpret_cast<uintptr_t>(out);
  int64_t A = S + static_cast<int64_t>((16 - ((ob + S) & 15)) & 15);   // first 16-B aligned
  int64_t B = E - static_cast<int64_t>((ob + E) & 15);                   // last 16-B boundary
  if (A > B) A = B = E;                        // short range: dwords only
  for (int64_t q = S + 4 * threadIdx.x; q < A; q += 4 * kThreads) {
    int f = find(q);
    *reinterpret_cast<uint32_t*>(out + q) = dword_at(q, f);
  }
  for (int64_t q = B + 4 * threadIdx.x; q < E; q += 4 * kThreads) {
    int f = find(q);
    *reinterpret_cast<uint32_t*>(out + q) = dword_at(q, f);
  }
  using v4u = __attribute__((ext_vector_type(4))) uint32_t;
  for (int64_t q = A + 16 * threadIdx.x; q < B; q += 16 * kThreads) {
    int f = find(q);
    v4u v;
    v.x = dword_at(q, f);
    v.y = dword_at(q + 4, f);
    v.z = dword_at(q + 8, f);
    v.w = dword_at(q + 12, f);
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(out + q));
  }
}

// ---- stream words at any base alignment ---------------------------------------------------------
// The stream may start at any byte address (Java's encode(MemoryBuffer, T) frames at the buffer's
// writerIndex).  Frames are 4-byte aligned RELATIVE to the stream start, so the parse works on
// stream words (4 B).  A StreamView reads them from the 16-byte aligned buffer around the stream
// (abase = base rounded down to 16): word j = bytes [off + 4j, off + 4j + 4) of abase, assembled
// from the two aligned dwords it straddles (a funnel shift; one dword when off % 4 == 0).  Only
// aligned dwords holding stream bytes are read (and, on the bulk path, whole 16-B chunks holding
// them), so no access leaves the pages of the stream.
struct StreamView {
  const uint32_t* a;     // 16-byte aligned base (dwords)
  int32_t o4;            // (base & 15) >> 2: dword shift
  int32_t sh;            // (base & 3) * 8:   bit shift inside a dword
  int64_t adw;           // aligned dwords readable from a: to the end of the last 16-B chunk
};

StreamView make_view(const uint8_t* in, int64_t len) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(in);
  const uintptr_t off = p & 15;
  StreamView v;
  v.a = reinterpret_cast<const uint32_t*>(p - off);
  v.o4 = static_cast<int32_t>(off >> 2);
  v.sh = static_cast<int32_t>(off & 3) * 8;
  v.adw = static_cast<int64_t>((off + len + 15) & ~uintptr_t(15)) >> 2;
  return v;
}

// Stream word j (j < len / 4).
__device__ __forceinline__ uint32_t sword(const StreamView& v, int64_t j) {
  const int64_t q = j + v.o4;
  const uint32_t lo = v.a[q];
  return v.sh ? (lo >> v.sh) | (v.a[q + 1] << (32 - v.sh)) : lo;
}

// ---- sequential walk (reference semantics, fallback) -------------------------------------------
// Encoders.decode(MemoryBuffer): readInt32 len, readInt64 hash (ClassNotCompatibleException on a
// mismatch), row = next len - 8 bytes.  One lane.  Starts at frame i0; for i0 > 0 frames
// [0, i0) are already in frame_pos / row_offs (the path the parallel repair found) and the walk
// resumes where frame i0 - 1 ends.
__global__ void unframe_walk(const uint8_t* __restrict__ in, int64_t len, int64_t n, int64_t hash,
                             int64_t i0, int64_t* __restrict__ frame_pos,
                             int64_t* __restrict__ row_offs, int32_t* __restrict__ err) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t pos = 0, out = 0;
  if (i0 > 0) {
    int32_t l0;
    memcpy(&l0, in + frame_pos[i0 - 1], 4);
    pos = frame_pos[i0 - 1] + 4 + l0;
    out = row_offs[i0 - 1] + (l0 - 8);
  }
  for (int64_t i = i0; i < n; i++) {
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

// ---- speculative parallel parse -----------------------------------------------------------------
// Exclusive prefix of x over the workgroup (thread order) and the workgroup total, for packed
// 16-bit counters (no field overflows: at most kThreads * kMarkWords per field).
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t x, uint64_t* total) {
  __shared__ uint64_t part[kThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) part[wid] = inc;
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; w++) {
    before += w < wid ? part[w] : 0;
    all += part[w];
  }
  *total = all;
  return before + inc - x;
}

// Decoupled look-back status words: 2-bit flag (0 = not yet published, kAgg = the workgroup's
// own count, kInc = inclusive prefix) over a 62-bit value.
constexpr uint64_t kAgg = 1ull << 62, kInc = 2ull << 62, kValMask = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t ld_status(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave: exclusive prefix of piece b.  Pieces are numbered by a ticket in the order their
// workgroups start, so every predecessor is running and the wait ends; the spin is bounded all the
// same, and a workgroup that gives up flags the parse as failed (the stream is then re-parsed by
// the walk, so results never depend on it).  kWin predecessors per step; 64 measured faster than
// 256 (the polling traffic costs more than the shorter chain saves).
template <int kWin>
__device__ int64_t look_back(const uint64_t* status, int64_t b, int32_t* err) {
  constexpr int U = kWin / 64;            // predecessors per lane per step
  const int lane = threadIdx.x & 63;
  int64_t excl = 0;
  uint32_t spins = 0;
  for (int64_t j = b - 1;; j -= kWin) {
    uint64_t v[U];
    for (;;) {
      bool pend = false;
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t idx = j - 64 * u - lane;
        v[u] = idx >= 0 ? ld_status(status + idx) : kInc;
        pend |= (v[u] >> 62) == 0;
      }
      if (__ballot(pend) == 0) break;
      if (++spins > (1u << 22)) {
        if (lane == 0) atomicOr(err, 8);
        return 0;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    int stop = kWin;                      // nearest inclusive predecessor (distance - 1)
#pragma unroll
    for (int u = U - 1; u >= 0; u--) {
      const uint64_t inc = __ballot((v[u] >> 62) == 2);
      if (inc) stop = 64 * u + __builtin_ctzll(inc);
    }
    int64_t x = 0;
#pragma unroll
    for (int u = 0; u < U; u++)
      x += (64 * u + lane <= stop) ? static_cast<int64_t>(v[u] & kValMask) : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    excl += x;
    if (stop < kWin) return excl;
  }
}

// Candidates of the stream in order: position and length of candidate k < n go to cand[k] /
// clen[k]; *total = the number of candidates in the whole stream.  A workgroup covers kRounds
// consecutive 8-KB pieces (lane t of round r reads words r * kMarkSpan + 8 t .. + 8: coalesced),
// so the look-back chain has one link per 64 KB of stream.  Candidates are staged in LDS in
// stream order (at most kStage per workgroup: real frames are >= 20 B, so only a stream full of
// false candidates overflows; it is flagged and goes to the walk).  kAligned: the stream base
// is 16-byte aligned (stream words are aligned dwords); otherwise each lane loads the 16 aligned
// dwords around its 10 stream words and funnel-shifts them (StreamView).  ticket, status (nb
// words) and err are zero at launch.
constexpr int kRounds = 8;
constexpr int kStage = 4096;
template <int kWin, bool kAligned>
__global__ __launch_bounds__(kThreads) void unframe_scan(StreamView sv, int64_t len, int64_t hash,
                                                         int64_t n, uint32_t* __restrict__ ticket,
                                                         uint64_t* __restrict__ status,
                                                         int64_t* __restrict__ cand,
                                                         int32_t* __restrict__ clen,
                                                         int64_t* __restrict__ total,
                                                         int32_t* __restrict__ err) {
  __shared__ int64_t spre;
  __shared__ int64_t sb;
  __shared__ int32_t spos[kStage];        // candidate word index within the workgroup's span
  __shared__ int32_t slen[kStage];
  if (threadIdx.x == 0) sb = atomicAdd(ticket, 1u);
  __syncthreads();
  const int64_t b = sb;
  const int64_t W = len >> 2;
  const uint32_t hlo = static_cast<uint32_t>(hash);
  const uint32_t hhi = static_cast<uint32_t>(static_cast<uint64_t>(hash) >> 32);
  int tot = 0;                             // candidates staged so far (workgroup-uniform)
  bool overflow = false;
  using v4u = __attribute__((ext_vector_type(4))) uint32_t;
  // every round's words are loaded before any is tested: 64 KB per workgroup in flight
  uint32_t xs[kRounds][kMarkWords + 2];
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    const int64_t w0 = b * kRounds * kMarkSpan + r * kMarkSpan + threadIdx.x * kMarkWords;
    uint32_t* x = xs[r];
    if (kAligned) {
      const uint32_t* in = sv.a;
      if (w0 + kMarkWords + 2 <= W) {
        const v4u a = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(in + w0));
        const v4u c = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(in + w0 + 4));
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
        x[4] = c.x; x[5] = c.y; x[6] = c.z; x[7] = c.w;
        x[8] = in[w0 + 8];
        x[9] = in[w0 + 9];
      } else {
#pragma unroll
        for (int j = 0; j < kMarkWords + 2; j++) x[j] = w0 + j < W ? in[w0 + j] : 0u;
      }
    } else if (w0 + 16 <= sv.adw && w0 + kMarkWords + 2 <= W) {
      uint32_t d[16];                      // aligned dwords w0 .. w0 + 15 (w0 is 16-B aligned)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(sv.a + w0 + 4 * q));
        d[4 * q] = t.x; d[4 * q + 1] = t.y; d[4 * q + 2] = t.z; d[4 * q + 3] = t.w;
      }
      // word w0 + j = dwords o4 + j, o4 + j + 1 (o4 <= 3, j <= 9: index <= 13)
#pragma unroll
      for (int j = 0; j < kMarkWords + 2; j++) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int o = 0; o < 4; o++) {
          if (o == sv.o4) {
            lo = d[o + j];
            hi = d[o + j + 1];
          }
        }
        x[j] = sv.sh ? (lo >> sv.sh) | (hi << (32 - sv.sh)) : lo;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kMarkWords + 2; j++) x[j] = w0 + j < W ? sword(sv, w0 + j) : 0u;
    }
  }
  // candidate bits of every round, then ONE packed scan of the per-round counts (4 rounds of
  // 16-bit fields per 64-bit word) instead of a workgroup scan per round
  static_assert(kRounds == 8, "two packed words of four 16-bit round counters");
  uint32_t bits[kRounds];
  uint64_t packed[2] = {0, 0};
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    const int64_t w0 = b * kRounds * kMarkSpan + r * kMarkSpan + threadIdx.x * kMarkWords;
    const uint32_t* x = xs[r];
    uint32_t bb = 0;
#pragma unroll
    for (int j = 0; j < kMarkWords; j++) {
      const int64_t p = 4 * (w0 + j);
      const uint32_t l = x[j];
      const bool hdr = (w0 + j + 3 <= W) && x[j + 1] == hlo && x[j + 2] == hhi &&
                       static_cast<int32_t>(l) >= 8 && (l & 7) == 0 &&
                       p + 4 + static_cast<int64_t>(l) <= len;
      bb |= hdr ? (1u << j) : 0u;
    }
    bits[r] = bb;
    packed[r >> 2] |= static_cast<uint64_t>(__popc(bb)) << (16 * (r & 3));
  }
  uint64_t tlo, thi;
  const uint64_t elo = block_excl_scan64(packed[0], &tlo);
  __syncthreads();                         // block_excl_scan64's LDS reused
  const uint64_t ehi = block_excl_scan64(packed[1], &thi);
  int base = 0;                            // candidates of the earlier rounds (all threads)
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    const uint64_t e = r < 4 ? elo : ehi, t = r < 4 ? tlo : thi;
    const int sh = 16 * (r & 3);
    int local = base + static_cast<int>((e >> sh) & 0xffff);
    const int rel = r * kMarkSpan + threadIdx.x * kMarkWords;
#pragma unroll
    for (int j = 0; j < kMarkWords; j++) {
      if (bits[r] & (1u << j)) {
        if (local < kStage) {
          spos[local] = rel + j;
          slen[local] = static_cast<int32_t>(xs[r][j]);
        }
        local++;
      }
    }
    base += static_cast<int>((t >> sh) & 0xffff);
  }
  tot = base;
  overflow = tot > kStage;
  __syncthreads();
  if (overflow) {
    if (threadIdx.x == 0) atomicOr(err, 16);
    tot = kStage;                          // keep the chain consistent; the parse is discarded
  }
  if (threadIdx.x == 0 && b == 0) {
    st_status(status, kInc | static_cast<uint64_t>(tot));
    spre = 0;
  } else if (threadIdx.x == 0) {
    st_status(status + b, kAgg | static_cast<uint64_t>(tot));
  }
  if (b > 0 && threadIdx.x < 64) {
    const int64_t pre = look_back<kWin>(status, b, err);
    if (threadIdx.x == 0) {
      st_status(status + b, kInc | static_cast<uint64_t>(pre + tot));
      spre = pre;
    }
  }
  __syncthreads();
  const int64_t pre = spre;
  for (int i = threadIdx.x; i < tot; i += kThreads) {
    const int64_t k = pre + i;
    if (k < n) {
      cand[k] = 4 * (b * kRounds * kMarkSpan + spos[i]);
      clen[k] = slen[i];
    }
  }
  if (threadIdx.x == 0 && b == gridDim.x - 1) *total = pre + tot;
}

// Candidate k is frame k iff candidate 0 is at 0 and each candidate ends where the next begins.
__global__ __launch_bounds__(kThreads) void unframe_verify(const int64_t* __restrict__ cand,
                                                           const int32_t* __restrict__ clen,
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
  const int64_t end = p + 4 + clen[k];
  bool ok = k != 0 || p == 0;
  if (k + 1 < n) ok = ok && cand[k + 1] == end;
  row_offs[k] = p - 12 * k;
  if (k == n - 1) row_offs[n] = end - 12 * n;
  if (!ok) atomicOr(err, 4);
}

// ---- parallel repair: the frame chain through the candidates ------------------------------------
// When the candidates do not verify (a payload that spells a plausible header), the frames are
// still among them: frame 0 is the candidate at 0 and frame i + 1 the candidate where frame i
// ends.  succ[k] = the candidate where candidate k ends (-1: none), a forest whose path from
// candidate 0 is exactly the frame chain Encoders.decode walks (while its headers are valid).
// Pointer doubling marks that path in log2(candidates) passes: before pass r every node at
// distance < 2^r from candidate 0 is marked, and pass r marks jump_r(k) = succ^(2^r)(k) of every
// marked k, so after it every node at distance < 2^(r+1) is (marks only ever spread along succ,
// so nothing off the path is marked).  The marked candidates in stream order are frames 0, 1, ...
__global__ __launch_bounds__(kThreads) void repair_succ(const int64_t* __restrict__ cand,
                                                        const int32_t* __restrict__ clen, int64_t m,
                                                        int32_t* __restrict__ succ,
                                                        int64_t* __restrict__ mark) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (k >= m) return;
  const int64_t e = cand[k] + 4 + clen[k];
  int64_t found = -1;
  // the next frame usually is one of the next few candidates; else binary search (cand sorted)
  for (int64_t j = k + 1; j < m && j <= k + 3; j++) {
    const int64_t c = cand[j];
    if (c == e) { found = j; break; }
    if (c > e) break;
  }
  if (found < 0 && k + 4 < m && cand[k + 3] < e) {
    int64_t lo = k + 4, hi = m - 1;
    while (lo <= hi) {
      const int64_t mid = (lo + hi) >> 1;
      const int64_t c = cand[mid];
      if (c == e) { found = mid; break; }
      if (c < e) lo = mid + 1;
      else hi = mid - 1;
    }
  }
  succ[k] = static_cast<int32_t>(found);
  mark[k] = (k == 0 && cand[0] == 0) ? 1 : 0;
}

__global__ __launch_bounds__(kThreads) void repair_double(const int32_t* __restrict__ jump,
                                                          int32_t* __restrict__ next, int64_t m,
                                                          int64_t* __restrict__ mark) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (k >= m) return;
  const int32_t j = jump[k];
  if (j >= 0) {
    if (mark[k]) mark[j] = 1;
    next[k] = jump[j];
  } else {
    next[k] = -1;
  }
}

// rank = exclusive scan of the marks (count = their total): frame rank of every marked candidate.
__global__ __launch_bounds__(kThreads) void repair_gather(const int64_t* __restrict__ cand,
                                                          const int64_t* __restrict__ rank,
                                                          const int64_t* __restrict__ count,
                                                          int64_t m, int64_t n,
                                                          int64_t* __restrict__ frame_pos) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (k >= m) return;
  const int64_t r = rank[k];
  const int64_t nx = k + 1 < m ? rank[k + 1] : *count;
  if (nx > r && r < n) frame_pos[r] = cand[k];
}

// Row offsets of frames [0, L) (L = min(path length, n)) and, when the path covers all n frames,
// row_offs[n].
__global__ __launch_bounds__(kThreads) void repair_offsets(const uint8_t* __restrict__ in,
                                                           const int64_t* __restrict__ frame_pos,
                                                           int64_t L, int64_t n,
                                                           int64_t* __restrict__ row_offs) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= L) return;
  row_offs[i] = frame_pos[i] - 12 * i;
  if (i == n - 1) {
    int32_t l;
    memcpy(&l, in + frame_pos[i], 4);
    row_offs[n] = frame_pos[i] + 4 + l - 12 * n;
  }
}

// Rows out of a parsed stream: each workgroup owns kCopyFrames frames = one contiguous range of
// the row buffer, written in 16-byte aligned chunks (a lane finds its chunk's frame by binary
// search over the range's row offsets in LDS and reads the frame's stream words through the view).
__global__ __launch_bounds__(kThreads) void unframe_copy(StreamView sv,
                                                         const int64_t* __restrict__ cand,
                                                         const int64_t* __restrict__ row_offs,
                                                         int64_t n, uint8_t* __restrict__ out,
                                                         const int32_t* __restrict__ err) {
  if (err && *err) return;           // speculation failed: the repair / walk takes over
  __shared__ int64_t ro[kCopyFrames + 1];
  __shared__ int64_t src[kCopyFrames];
  const int64_t k0 = static_cast<int64_t>(blockIdx.x) * kCopyFrames;
  const int kn = static_cast<int>(min(static_cast<int64_t>(kCopyFrames), n - k0));
  for (int f = threadIdx.x; f <= kn; f += kThreads) {
    ro[f] = row_offs[k0 + f];
    if (f < kn) src[f] = cand[k0 + f] + 12;
  }
  __syncthreads();
  auto find = [&](int64_t d) {        // last frame whose row starts at or before d
    int lo = 0, hi = kn - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (ro[mid] <= d) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  // row-buffer dword at d (rows are whole 8-byte words, so a dword never straddles two rows)
  auto dword_at = [&](int64_t d, int& f) -> uint32_t {
    while (f + 1 < kn && ro[f + 1] <= d) f++;
    return sword(sv, (src[f] + (d - ro[f])) >> 2);
  };
  // 16-byte aligned chunks of the row buffer (non-temporal stores), dwords at the two ends
  const int64_t S = ro[0], E = ro[kn];
  const uintptr_t ob = reinterpret_cast<uintptr_t>(out);
  int64_t A = S + static_cast<int64_t>((16 - ((ob + S) & 15)) & 15);
  int64_t B = E - static_cast<int64_t>((ob + E) & 15);
  if (A > B) A = B = E;
  for (int64_t d = S + 4 * threadIdx.x; d < A; d += 4 * kThreads) {
    int f = find(d);
    *reinterpret_cast<uint32_t*>(out + d) = dword_at(d, f);
  }
  for (int64_t d = B + 4 * threadIdx.x; d < E; d += 4 * kThreads) {
    int f = find(d);
    *reinterpret_cast<uint32_t*>(out + d) = dword_at(d, f);
  }
  using v4u = __attribute__((ext_vector_type(4))) uint32_t;
  for (int64_t d = A + 16 * threadIdx.x; d < B; d += 16 * kThreads) {
    int f = find(d);
    v4u v;
    v.x = dword_at(d, f);
    v.y = dword_at(d + 4, f);
    v.z = dword_at(d + 8, f);
    v.w = dword_at(d + 12, f);
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(out + d));
  }
}

std::atomic<int64_t> g_unframe_walks{0};     // streams parsed (partly) by the sequential walk
std::atomic<int64_t> g_unframe_repairs{0};   // streams parsed by the parallel repair
std::atomic<int> g_unframe_mode = 0;   // tuning "unframe": 0 speculative, 1 always walk

struct DevBuf {                               // stream-ordered scratch freed on every exit
  void* p = nullptr;
  hipStream_t s;
  explicit DevBuf(hipStream_t st) : s(st) {}
  ~DevBuf() {
    if (p) dev_free(p, s);
  }
  int alloc(int64_t bytes) {
    return dev_alloc(bytes < 16 ? 16 : bytes, s, &p);
  }
};

int walk_status(int32_t herr, int64_t hash) {
  if (herr == 1)
    return set_error(FURY_ERR_CLASS_NOT_COMPATIBLE,
                     "Schema is not consistent: peer schema hash differs from " +
                         std::to_string(hash));
  if (herr == 2) return set_error(FURY_ERR_OUT_OF_BOUNDS, "frame runs past the end of the stream");
  return FURY_OK;
}

// Frames [i0, n) by the sequential walk (frames [0, i0) already in fp / row_offs), then the copy.
int unframe_walked(const uint8_t* in, int64_t len, int64_t n, int64_t hash, int64_t i0,
                   int64_t* fp, uint8_t* rows_out, int64_t* row_offs, hipStream_t stream) {
  g_unframe_walks.fetch_add(1);
  DevBuf eb(stream);
  int st = eb.alloc(8);
  if (st) return st;
  int32_t* err = static_cast<int32_t*>(eb.p);
  (void)hipMemsetAsync(err, 0, 4, stream);
  hipLaunchKernelGGL(unframe_walk, dim3(1), dim3(64), 0, stream, in, len, n, hash, i0, fp,
                     row_offs, err);
  int32_t herr = 0;
  (void)hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, stream);
  st = check_hip(hipStreamSynchronize(stream), "unframe sync");
  if (st) return st;
  if (herr) return walk_status(herr, hash);
  const int64_t cb = (n + kCopyFrames - 1) / kCopyFrames;
  hipLaunchKernelGGL(unframe_copy, dim3(cb), dim3(kThreads), 0, stream, make_view(in, len), fp,
                     row_offs, n, rows_out, nullptr);
  return check_hip(hipGetLastError(), "unframe copy launch");
}

int64_t scan_blocks(int64_t len) {
  return ((len >> 2) + kRounds * kMarkSpan - 1) / (kRounds * kMarkSpan);
}

// Launches the candidate scan over the whole stream: the first `want` candidates to cand / clen,
// the count of all of them to *total.  ws: ticket + status (scan_blocks + 1 words), zeroed here.
void launch_scan(const uint8_t* in, int64_t len, int64_t hash, int64_t want, uint64_t* ws,
                 int64_t* cand, int32_t* clen, int64_t* total, int32_t* err, hipStream_t stream) {
  const int64_t nb = scan_blocks(len);
  (void)hipMemsetAsync(ws, 0, (nb + 1) * 8, stream);
  const StreamView sv = make_view(in, len);
  uint32_t* ticket = reinterpret_cast<uint32_t*>(ws);
  if ((reinterpret_cast<uintptr_t>(in) & 15) == 0)
    hipLaunchKernelGGL((unframe_scan<64, true>), dim3(nb), dim3(kThreads), 0, stream, sv, len,
                       hash, want, ticket, ws + 1, cand, clen, total, err);
  else
    hipLaunchKernelGGL((unframe_scan<64, false>), dim3(nb), dim3(kThreads), 0, stream, sv, len,
                       hash, want, ticket, ws + 1, cand, clen, total, err);
}

// The candidates did not verify: find the frame chain among ALL candidates in parallel
// (pointer doubling), fall back to the walk only for what the chain does not cover (a frame the
// candidate test rejects: the error Encoders.decode reports, or a length that is not a multiple
// of 8, which Java never writes).
int unframe_repair(const uint8_t* in, int64_t len, int64_t n, int64_t hash, int64_t m,
                   int64_t* fp, uint8_t* rows_out, int64_t* row_offs, hipStream_t stream) {
  if (m <= 0 || m > 0x7fffffffLL)
    return unframe_walked(in, len, n, hash, 0, fp, rows_out, row_offs, stream);
  g_unframe_repairs.fetch_add(1);
  const int64_t nb = scan_blocks(len);
  // [cand m][mark m][scan ws][ticket+status nb+1][total][err][clen m][jump m][next m]
  const int64_t sw = scan_workspace(m);
  const int64_t w64 = m + m + sw + (nb + 1) + 2;
  DevBuf buf(stream);
  int st = buf.alloc(w64 * 8 + 3 * m * 4 + 64);
  if (st) return st;
  int64_t* cand = static_cast<int64_t*>(buf.p);
  int64_t* mark = cand + m;
  int64_t* sws = mark + m;
  uint64_t* ws = reinterpret_cast<uint64_t*>(sws + sw);
  int64_t* total = reinterpret_cast<int64_t*>(ws + nb + 1);
  int32_t* err = reinterpret_cast<int32_t*>(total + 1);
  int32_t* clen = reinterpret_cast<int32_t*>(cand + w64);
  int32_t* jump = clen + m;
  int32_t* next = jump + m;
  (void)hipMemsetAsync(err, 0, 8, stream);
  launch_scan(in, len, hash, m, ws, cand, clen, total, err, stream);
  const int64_t g = (m + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(repair_succ, dim3(g), dim3(kThreads), 0, stream, cand, clen, m, jump, mark);
  for (int64_t span = 1; span < m; span <<= 1) {
    hipLaunchKernelGGL(repair_double, dim3(g), dim3(kThreads), 0, stream, jump, next, m, mark);
    int32_t* t = jump;
    jump = next;
    next = t;
  }
  int64_t path = 0;                               // marked candidates = frames on the chain
  device_scan(mark, m, total, sws, stream);
  int32_t herr = 0;
  (void)hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, stream);
  (void)hipMemcpyAsync(&path, total, 8, hipMemcpyDeviceToHost, stream);
  if ((st = check_hip(hipGetLastError(), "unframe repair launch"))) return st;
  if ((st = check_hip(hipStreamSynchronize(stream), "unframe repair sync"))) return st;
  if (herr) return unframe_walked(in, len, n, hash, 0, fp, rows_out, row_offs, stream);
  hipLaunchKernelGGL(repair_gather, dim3(g), dim3(kThreads), 0, stream, cand, mark, total, m, n,
                     fp);
  const int64_t L = path < n ? path : n;
  if (L > 0)
    hipLaunchKernelGGL(repair_offsets, dim3((L + kThreads - 1) / kThreads), dim3(kThreads), 0,
                       stream, in, fp, L, n, row_offs);
  if ((st = check_hip(hipGetLastError(), "unframe repair launch"))) return st;
  if (L < n) return unframe_walked(in, len, n, hash, L, fp, rows_out, row_offs, stream);
  const int64_t cb = (n + kCopyFrames - 1) / kCopyFrames;
  hipLaunchKernelGGL(unframe_copy, dim3(cb), dim3(kThreads), 0, stream, make_view(in, len), fp,
                     row_offs, n, rows_out, nullptr);
  return check_hip(hipGetLastError(), "unframe copy launch");
}

}  // namespace

int unframe_mode() { return g_unframe_mode; }
void set_unframe_mode(int v) { g_unframe_mode = v; }
int64_t unframe_walk_count() { return g_unframe_walks.load(); }
int64_t unframe_repair_count() { return g_unframe_repairs.load(); }

int launch_frame_rows(const uint8_t* rows, const int64_t* offs, int64_t n, int64_t fixed,
                      int64_t hash, uint8_t* out, int64_t* fo, hipStream_t stream) {
  if (n == 0) return FURY_OK;
  const int64_t blocks = (n + kCopyFrames - 1) / kCopyFrames;
  hipLaunchKernelGGL(frame_kernel, dim3(blocks), dim3(kThreads), 0, stream, rows, offs, n, fixed,
                     hash, out, fo);
  return check_hip(hipGetLastError(), "frame launch");
}

// Any base alignment: the scan reads stream words through a StreamView.  A stream that does not
// verify is repaired in parallel (unframe_repair); the sequential walk only parses what the
// repair cannot (error reporting).
int launch_unframe_rows(const uint8_t* in, int64_t len, int64_t n, int64_t hash, uint8_t* rows_out,
                        int64_t* row_offs, hipStream_t stream) {
  if (n == 0) return check_hip(hipMemsetAsync(row_offs, 0, 8, stream), "memset");
  DevBuf fpb(stream);
  int st = fpb.alloc(n * 8);
  if (st) return st;
  int64_t* fp = static_cast<int64_t*>(fpb.p);       // frame positions
  if (len < 12 || g_unframe_mode == 1)
    return unframe_walked(in, len, n, hash, 0, fp, rows_out, row_offs, stream);
  const int64_t nb = scan_blocks(len);
  if (nb > 0x7fffffff) return set_error(FURY_ERR_INVALID_ARGUMENT, "stream too large");
  // workspace: [ticket + status (nb + 1)][total][err (8 B)][clen n x 4 B]
  const int64_t words = nb + 1 + 2;
  DevBuf buf(stream);
  if ((st = buf.alloc(words * 8 + n * 4))) return st;
  uint64_t* ws = static_cast<uint64_t*>(buf.p);
  int64_t* total = reinterpret_cast<int64_t*>(ws + nb + 1);
  int32_t* err = reinterpret_cast<int32_t*>(total + 1);
  int32_t* clen = reinterpret_cast<int32_t*>(ws + words);
  (void)hipMemsetAsync(total, 0, 16, stream);
  launch_scan(in, len, hash, n, ws, fp, clen, total, err, stream);
  const int64_t vb = (n + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(unframe_verify, dim3(vb), dim3(kThreads), 0, stream, fp, clen, total, n,
                     row_offs, err);
  const int64_t cb = (n + kCopyFrames - 1) / kCopyFrames;
  hipLaunchKernelGGL(unframe_copy, dim3(cb), dim3(kThreads), 0, stream, make_view(in, len), fp,
                     row_offs, n, rows_out, err);
  st = check_hip(hipGetLastError(), "unframe launch");
  int32_t herr = 0;
  int64_t m = 0;
  if (!st) {
    (void)hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, stream);
    (void)hipMemcpyAsync(&m, total, 8, hipMemcpyDeviceToHost, stream);
  }
  const int st2 = check_hip(hipStreamSynchronize(stream), "unframe sync");
  if (st) return st;
  if (st2) return st2;
  if (herr == 0) return FURY_OK;
  if (herr & (8 | 16))            // a look-back gave up / too many candidates in a piece
    return unframe_walked(in, len, n, hash, 0, fp, rows_out, row_offs, stream);
  return unframe_repair(in, len, n, hash, m, fp, rows_out, row_offs, stream);
}

}  // namespace fury
