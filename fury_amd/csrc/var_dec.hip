// var_dec.hip — rows -> Arrow columns for flat schemas with variable-length fields (STRING /
// BINARY, DECIMAL, LIST of fixed-width elements, any mix with fixed-width fields, 1..256 fields):
// fury_row_decode / fury_rows_to_arrow.
//
// Reference semantics (FMT = java/fury-format/src/main/java/org/apache/fury/format): the generated
// fromRow -- `if (!row.isNullAt(i)) bean.f = row.getX(i)` (FMT/encoder/RowEncoderBuilder.java:
// 185-217) over the BinaryRow getters (FMT/row/binary/UnsafeTrait.java:68-197: getBinary slices
// (relOffset << 32 | size) from the row base; getArray / BinaryArray.pointTo + toXxxArray,
// BinaryArray.java:69-78,157-197) -- and ArrowWriter's StringWriter / ListWriter
// (FMT/vectorized/ArrowWriter.java:421-540: int32 offsets, a null entry is zero-length).  Every
// read is bounds-checked against the batch (span_ok, kernels.h: MemoryBuffer's checks).
//
// MI355X design (round 3; replaces the register-staged thread-per-row decode, whose row-strided
// 16-B header loads touched 64 cache lines per wave instruction and held 127 VGPRs):
//   * a tile = NT rows = one workgroup of NT threads; every WAVE owns 64 consecutive rows, i.e.
//     one contiguous byte range of the rows buffer, and stages that range in its own LDS region
//     with LDS-DMA (global_load_lds_dwordx4: 1 KB per wave instruction, coalesced, no VGPRs);
//   * lane = row reads its null bits and slots from LDS, counts its STRING / LIST values, and the
//     wave scans the counts with cross-lane ops -- no workgroup barrier for in-wave positions;
//   * fixed-width fields leave as coalesced column stores, validity / bool bits as ballots (the
//     wave's 64 rows are two whole 32-bit words);
//   * the tile's totals chain across tiles by the decoupled look-back of var_dev.h (blockIdx
//     order, self-helping), resolved while the fixed-width stores drain;
//   * payloads: the wave's share of a column's Arrow range is contiguous, so lanes produce it as
//     16-byte chunks (one 16-B store per lane: a wave instruction writes 1 KB of consecutive
//     bytes) gathering bytes from the staged strings in LDS; list elements leave one per lane,
//     consecutive lanes = consecutive child entries.
// A wave whose range does not fit its stage (long strings / lists) or lies outside the batch reads
// HBM instead (same code, global accesses).
#define FURY_VAR_DEC2
#include "var_dev.h"

namespace fury {

namespace {

constexpr int kWs = 64;                 // rows per wave

__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Wave-only LDS-DMA of the 16-B-aligned pieces covering [gb, ge) into lds[0...); returns the LDS
// offset of byte gb.
__device__ __forceinline__ uint32_t stage_wave(uint8_t* lds, const uint8_t* gb, const uint8_t* ge) {
  const uint64_t lo = reinterpret_cast<uint64_t>(gb) & ~uint64_t(15);
  const uint64_t hi = (reinterpret_cast<uint64_t>(ge) + 15) & ~uint64_t(15);
  const uint32_t nch = static_cast<uint32_t>((hi - lo) >> 4);
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i0 = 0; i0 < nch; i0 += 64) {
    if (i0 + lane < nch)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(lo + 16ull * (i0 + lane)),
                                       lds + 16 * i0, 16, 0, 0);
  }
  return static_cast<uint32_t>(reinterpret_cast<uint64_t>(gb) - lo);
}

template <class T>
using Lds = __attribute__((address_space(3))) T;

// The bytes of the batch a wave reads: [lo, hi) staged in LDS at `st` (byte lo at st), the rest
// from HBM.  LDS and HBM accesses are typed (ds_* / global_*: never flat).
struct WaveView {
  const uint8_t* rows;
  Lds<const uint8_t>* st;   // byte lo of the batch
  int64_t lo, hi;           // staged range; empty when not staged
  __device__ __forceinline__ bool in(int64_t q, int64_t len) const { return q >= lo && q + len <= hi; }
  __device__ __forceinline__ uint8_t u8(int64_t q) const {
    return in(q, 1) ? st[q - lo] : *gl(rows + q);
  }
  __device__ __forceinline__ uint64_t u64(int64_t q) const {          // q 8-aligned
    return in(q, 8) ? *(Lds<const uint64_t>*)(st + (q - lo))
                    : *gl(reinterpret_cast<const uint64_t*>(rows + q));
  }
  __device__ __forceinline__ uint64_t load(int64_t q, int w) const {  // an element of width w
    if (in(q, w)) {
      Lds<const uint8_t>* p = st + (q - lo);
      switch (w) {
        case 8: return *(Lds<const uint64_t>*)(p);
        case 4: return *(Lds<const uint32_t>*)(p);
        case 2: return *(Lds<const uint16_t>*)(p);
        default: return *p;
      }
    }
    const uint8_t* p = rows + q;
    switch (w) {
      case 8: return *gl(reinterpret_cast<const uint64_t*>(p));
      case 4: return *gl(reinterpret_cast<const uint32_t*>(p));
      case 2: return *gl(reinterpret_cast<const uint16_t*>(p));
      default: return *gl(p);
    }
  }
};

// slot_count (var_dev.h) with the array header read through the wave's view.
__device__ __forceinline__ int64_t view_count(const WaveView& v, int kind, int width, uint64_t slot,
                                              int64_t base, int64_t total, bool* bad) {
  if (kind != kListFixed) return slot_count(kind, width, slot, base, v.rows, total, bad);
  const int64_t p = base + static_cast<int32_t>(slot >> 32);
  if (!span_ok(p, 8, total)) {
    *bad = true;
    return 0;
  }
  const int64_t n = static_cast<int32_t>(v.u64(p));
  const int64_t ew = width == 0 ? 1 : width;
  if (n >= 0 && span_ok(p, 8 + bm_bytes(n) + n * ew, total)) return n;
  *bad = true;
  return 0;
}

// dst bytes [pos, pos + len) <- batch bytes [src, src + len): one lane's string.  Staged 8-aligned
// sources (the writer's layout) are read as aligned LDS words and funnel-shifted into 4-byte
// destination words; the unaligned head / tail of the destination are byte stores, so strings of
// neighbouring lanes never share a store.  Anything else goes byte by byte.
__device__ __forceinline__ void copy_string(uint8_t* dst, int64_t pos, const WaveView& v,
                                            int64_t src, int64_t len) {
  if (len <= 0) return;
  if (!v.in(src, len) || (src & 7)) {
    for (int64_t t = 0; t < len; t++) gl(dst)[pos + t] = v.u8(src + t);
    return;
  }
  Lds<const uint8_t>* s = v.st + (src - v.lo);
  const int64_t head = min<int64_t>(len, (4 - (pos & 3)) & 3);
  for (int64_t t = 0; t < head; t++) gl(dst)[pos + t] = s[t];
  const int64_t nw = (len - head) >> 2;
  auto d32 = gl(reinterpret_cast<uint32_t*>(dst + pos + head));
  for (int64_t j = 0; j < nw; j++) {
    const int64_t q = head + 4 * j;                 // source byte of this destination word
    const int o = static_cast<int>(q & 7);
    Lds<const uint64_t>* w = (Lds<const uint64_t>*)(s + (q & ~int64_t(7)));
    uint64_t x = w[0] >> (8 * o);
    if (o > 4) x |= w[1] << (64 - 8 * o);
    d32[j] = static_cast<uint32_t>(x);
  }
  for (int64_t t = head + 4 * nw; t < len; t++) gl(dst)[pos + t] = s[t];
}

__device__ __forceinline__ int wave_max_scan(int x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x = max(x, y);
  }
  return x;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int64_t wave_excl_scan(int64_t x, int64_t* total) {
  const int64_t inc = wave_incl_scan(x);
  *total = __shfl(inc, 63, 64);
  return inc - x;
}

// Last t in [0, n) with ex[t] <= idx (ex: a wave's exclusive starts in LDS).
__device__ __forceinline__ int wave_find(const int32_t* ex, int n, int64_t idx) {
  int lo = 0, hi = n;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (ex[mid] <= idx) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Per-wave LDS: [stage: stage_bytes][ex: nc x 65 int32 -- per variable-length column of the
// chunk the wave's exclusive starts, [64] = the wave's total][rbase: 64 int64 -- each row's start]
// [own: 64 int32 -- list element owners].
__host__ __device__ __forceinline__ uint32_t ex_bytes(int nc) { return ((nc * (kWs + 1) * 4) + 15) & ~15u; }
__host__ __device__ __forceinline__ uint32_t wave_lds(uint32_t stage, int nc) {
  return stage + ex_bytes(nc) + kWs * 8 + kWs * 4;
}

// Decoupled look-back (var_dev.h look_back_help) with a window of 64 * NW tiles per round trip:
// lane l reads the status words of the NW consecutive predecessors b - 1 - (NW * l + u).  The
// inclusive prefix advances at most one window per status round trip (~1 us under load, the
// words live at the cross-XCD coherence point), so with the resident tiles several windows ahead
// of it a 64-tile window made every tile wait several round trips; NW words per lane, issued
// together, cover them in one.  Silent predecessors are helped exactly as in look_back_help.
__device__ __forceinline__ int wave_min_int(int x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x = min(x, __shfl_xor(x, d, 64));
  return x;
}

template <int NT, int NW>
__device__ int64_t look_back_wide(const VarArgs& a, int k, const uint8_t* rows, const int64_t* offs,
                                  const uint64_t* status, int64_t b, int nseq, int q,
                                  uint32_t* err) {
  const int lane = threadIdx.x & 63;
  const uint32_t limit = (a.help_now & 1) ? 0u : kHelpSpins;
  constexpr int W = 64 * NW;
  int64_t excl = 0;
  for (int64_t j = b - 1;; j -= W) {
    uint64_t v[NW];
#pragma unroll
    for (int u = 0; u < NW; u++) {
      const int64_t idx = j - (NW * lane + u);
      v[u] = idx >= 0 ? ld_status(status + idx * nseq + q) : kInc;
    }
    int stop;
    uint32_t spins = 0, helped = 0;
    for (;;) {
      int mine = W;                                      // nearest inclusive of this lane
#pragma unroll
      for (int u = NW - 1; u >= 0; u--)
        if ((v[u] >> 62) == 2) mine = NW * lane + u;
      stop = wave_min_int(mine);
      int pend = W;                                      // nearest unpublished at or before stop
#pragma unroll
      for (int u = NW - 1; u >= 0; u--)
        if ((v[u] >> 62) == 0 && NW * lane + u <= stop) pend = NW * lane + u;
      pend = wave_min_int(pend);
      if (pend == W) break;
      if (spins >= limit) {                              // help the nearest silent predecessor
        const int64_t agg = tile_count<NT>(a, k, rows, offs, j - pend);
#pragma unroll
        for (int u = 0; u < NW; u++)
          if (NW * lane + u == pend) v[u] = kAgg | static_cast<uint64_t>(agg);
        spins = 0;
        if (++helped > static_cast<uint32_t>(W) && err) {
          if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return 0;
        }
        continue;
      }
      ++spins;
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int u = 0; u < NW; u++) {
        const int64_t idx = j - (NW * lane + u);
        if ((v[u] >> 62) == 0 && NW * lane + u <= stop && idx >= 0)
          v[u] = ld_status(status + idx * nseq + q);
      }
    }
    int64_t part = 0;
#pragma unroll
    for (int u = 0; u < NW; u++)
      if (NW * lane + u <= stop) part += static_cast<int64_t>(v[u] & kValMask);
    excl += wave_sum(part);
    if (stop < W) return excl;
  }
}

template <int NT>
struct TileShared {
  int64_t wtot[kSeqChunk][NT / kWs];    // per column: each wave's total
  int64_t base[kSeqChunk];              // per column: the tile's global start
};

template <int NT>
__global__ __launch_bounds__(NT) void decode_var_ws(VarArgs a, const uint8_t* __restrict__ rows,
                                                   const int64_t* __restrict__ offs,
                                                   uint64_t* __restrict__ status, int nseq,
                                                   uint32_t stage_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ TileShared<NT> ts;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = blockIdx.x;
  const int64_t r0 = b * NT;
  const int nr = static_cast<int>(min<int64_t>(NT, a.nrows - r0));
  const int64_t rw0 = r0 + kWs * wave;
  const int nrw = max(0, min(kWs, nr - kWs * wave));
  const bool live = lane < nrw;
  const int64_t r = rw0 + lane;
  const int64_t total = offs[a.nrows];
  const int nc = max(1, min(nseq, kSeqChunk));
  uint8_t* wlds = lds + static_cast<size_t>(wave) * wave_lds(stage_bytes, nc);
  Lds<int32_t>* exb = (Lds<int32_t>*)(wlds + stage_bytes);
  Lds<int64_t>* rbase = (Lds<int64_t>*)(wlds + stage_bytes + ex_bytes(nc));
  Lds<int32_t>* own = (Lds<int32_t>*)(wlds + stage_bytes + ex_bytes(nc) + kWs * 8);

  // the wave's rows and its staged byte range
  const int64_t base = live ? offs[r] : 0;
  int64_t wbeg = 0, wend = 0;
  if (nrw > 0) {
    wbeg = offs[rw0];
    wend = offs[rw0 + nrw];
  }
  WaveView v{rows, (Lds<const uint8_t>*)(wlds), 0, 0};
  if (nrw > 0 && wend >= wbeg && span_ok(wbeg, wend - wbeg, total) &&
      (wend - wbeg) + 32 <= static_cast<int64_t>(stage_bytes)) {
    const uint32_t d0 = stage_wave(wlds, rows + wbeg, rows + wend);
    v = WaveView{rows, (Lds<const uint8_t>*)(wlds + d0), wbeg, wend};
  }
  const bool rok = live && row_ok(base, a.fixed_size, total);
  if (live && !rok) raise_oob(a.err, r);
  rbase[lane] = base;
  wait_vmem();                                   // this wave's stage has landed
  const int diag = a.help_now >> 8;
  if (diag & 8) {
    if (v.u64(wbeg) == 0x1234567812345678ull) status[0] = 1;
    return;
  }

  const int64_t vbase = r0 + kWs * wave;         // first row of the wave (64-aligned)
  const int64_t nleft = a.nrows - vbase;
  const int nwords = nleft >= 64 ? 2 : nleft <= 0 ? 0 : static_cast<int>((nleft + 31) >> 5);
  auto is_null = [&](int k) -> bool {
    if (!rok) return true;
    return (v.u8(base + (k >> 3)) >> (k & 7)) & 1;
  };
  auto slot_of = [&](int k) -> uint64_t { return v.u64(base + a.bitmap_bytes + 8 * k); };

  for (int cbase = 0; cbase < max(nseq, 1); cbase += kSeqChunk) {
    const int nchunk = nseq > 0 ? min(kSeqChunk, nseq - cbase) : 0;
    // ---- counts of this chunk's variable-length columns, scanned within the wave
    {
      int seq = 0;
      for (int k = 0; k < a.ncols; k++) {
        CVarCol& c = vc(a, k);
        if (!is_seq(c)) continue;
        const int q = seq++ - cbase;
        if (q < 0) continue;
        if (q >= nchunk) break;
        int64_t cnt = 0;
        if (rok && !is_null(k)) {
          bool bad = false;
          cnt = view_count(v, c.kind, c.width, slot_of(k), base, total, &bad);
          if (bad) raise_oob(a.err, r);
        }
        int64_t wt;
        const int64_t ex = wave_excl_scan(cnt, &wt);
        if (ex + cnt > INT32_MAX) raise_oob(a.err, r);     // int32 Arrow offsets
        exb[q * (kWs + 1) + lane] = static_cast<int32_t>(ex);
        if (lane == 63) {
          exb[q * (kWs + 1) + kWs] = static_cast<int32_t>(wt);
          ts.wtot[q][wave] = wt;
        }
      }
    }
    __syncthreads();
    if (diag & 16) return;
    // ---- publish the tile's aggregates (32-bit, as tile_count computes them)
    if (tid < nchunk) {
      int64_t t = 0;
      for (int w = 0; w < NT / kWs; w++) t += ts.wtot[tid][w];
      st_status(status + b * nseq + cbase + tid,
                (b == 0 ? kInc : kAgg) | static_cast<uint64_t>(static_cast<uint32_t>(t)));
    }
    // ---- fixed-width fields, decimals and every field's validity (first chunk only)
    if (cbase == 0 && !(diag & 2)) {
      for (int k = 0; k < a.ncols; k++) {
        CVarCol& c = vc(a, k);
        bool nul = !rok || is_null(k);
        uint64_t sl = 0;
        if (!nul && c.kind != kListFixed && c.kind != kBytes) sl = slot_of(k);
        if (!nul && c.kind >= kBytes) {               // a value outside the batch decodes as null
          bool bad = false;
          (void)view_count(v, c.kind, c.width, slot_of(k), base, total, &bad);
          nul = bad;
          if (bad && c.kind == kDecimal) raise_oob(a.err, r);
        }
        if (c.validity) {
          const uint64_t ok = __ballot(live && !nul);
          if (lane < nwords)
            gl(reinterpret_cast<uint32_t*>(c.validity))[(vbase >> 5) + lane] =
                static_cast<uint32_t>(ok >> (32 * lane));
        }
        uint8_t* dst = const_cast<uint8_t*>(c.values);
        if (!dst) continue;
        const uint64_t x = nul ? 0 : sl;
        if (c.kind == kFixed) {
          if (live) {
            switch (c.width) {
              case 8: __builtin_nontemporal_store(x, gl(reinterpret_cast<uint64_t*>(dst)) + r); break;
              case 4: __builtin_nontemporal_store(static_cast<uint32_t>(x), gl(reinterpret_cast<uint32_t*>(dst)) + r); break;
              case 2: gl(reinterpret_cast<uint16_t*>(dst))[r] = static_cast<uint16_t>(x); break;
              default: gl(dst)[r] = static_cast<uint8_t>(x); break;
            }
          }
        } else if (c.kind == kBool) {
          const uint64_t bits = __ballot(live && (x & 0xff) != 0);
          if (lane < nwords)
            gl(reinterpret_cast<uint32_t*>(dst))[(vbase >> 5) + lane] = static_cast<uint32_t>(bits >> (32 * lane));
        } else if (c.kind == kDecimal && live) {
          uint64_t lo = 0, hi = 0;
          if (!nul) {                                   // [p, p + 16) checked above
            const int64_t p = base + static_cast<int32_t>(x >> 32);
            lo = v.u64(p);
            hi = v.u64(p + 8);
          }
          auto d = gl(reinterpret_cast<uint64_t*>(dst + 16 * r));
          d[0] = lo;
          d[1] = hi;
        }
      }
    }
    // ---- the tile's global starts: one wave per column (decoupled look-back, var_dev.h)
    for (int q = wave; q < nchunk; q += NT / kWs) {
      const int64_t pre = (b == 0 || (diag & 4)) ? 0
                          : (diag & 32) ? look_back_help<NT>(a, seq_col(a, cbase + q), rows, offs,
                                                             status, b, nseq, cbase + q, a.err)
                          : look_back_wide<NT, 8>(a, seq_col(a, cbase + q), rows, offs, status, b,
                                                  nseq, cbase + q, a.err);
      if (lane == 0) {
        ts.base[q] = pre;
        if (b > 0) {
          int64_t t = 0;
          for (int w = 0; w < NT / kWs; w++) t += ts.wtot[q][w];
          st_status(status + b * nseq + cbase + q,
                    kInc | static_cast<uint64_t>(pre + static_cast<uint32_t>(t)));
        }
      }
    }
    __syncthreads();
    // ---- Arrow offsets and payloads / elements of the wave's rows
    {
      int seq = 0;
      for (int k = 0; k < a.ncols; k++) {
        CVarCol& c = vc(a, k);
        if (!is_seq(c)) continue;
        const int q = seq++ - cbase;
        if (q < 0) continue;
        if (q >= nchunk) break;
        int64_t cb = ts.base[q];
        for (int w = 0; w < wave; w++) cb += ts.wtot[q][w];
        Lds<const int32_t>* ex = exb + q * (kWs + 1);
        const int64_t wt = ex[kWs];
        if (live) gl(c.offsets)[r] = static_cast<int32_t>(cb + ex[lane]);
        if (r == a.nrows - 1) gl(c.offsets)[a.nrows] = static_cast<int32_t>(cb + wt);
        uint8_t* dst = const_cast<uint8_t*>(c.values);
        if (!dst || wt == 0 || nrw == 0 || (diag & 1)) continue;
        const int64_t cap = c.capacity;
        if (c.kind == kBytes && (diag & 64)) {
          // lane = row: its string at cb + ex[lane] (clipped to the capacity)
          const int64_t cnt = ex[lane + 1] - ex[lane];
          if (live && cnt > 0) {
            const int64_t pos = cb + ex[lane];
            const int64_t src = base + static_cast<int32_t>(slot_of(k) >> 32);
            copy_string(dst, pos, v, src, max<int64_t>(0, min<int64_t>(cnt, cap - pos)));
          }
          continue;
        }
        if (c.kind == kBytes) {
          // The wave's bytes [cb, cb + wt) of the payload as 16-B chunks of the destination's
          // alignment, one per lane: a wave instruction stores 1 KB of consecutive bytes.  The row
          // owning each chunk's first byte: rows mark the chunk index where they own the first
          // byte (atomic max: several short strings may start in one chunk), a wave max-scan
          // spreads it; lanes then walk their 16 bytes row by row.
          const int64_t end = min<int64_t>(cb + wt, cap);
          if (end <= cb) continue;
          const int64_t a0 = cb & ~int64_t(15);
          const int64_t nch = (end - a0 + 15) >> 4;
          const int64_t my_s = cb + ex[lane];
          const bool has = live && ex[lane + 1] > ex[lane];
          const int64_t my_c = (my_s - a0) >> 4;
          const int64_t my_m = my_s <= max<int64_t>(a0 + 16 * my_c, cb) ? my_c : my_c + 1;
          int carry = 0;
          for (int64_t w0 = 0; w0 < nch; w0 += kWs) {
            own[lane] = -1;
            wave_sync();
            if (has && my_m >= w0 && my_m < w0 + kWs) atomicMax((int*)(own + (my_m - w0)), lane);
            wave_sync();
            int t = max(wave_max_scan(own[lane]), carry);
            carry = __shfl(t, 63, 64);
            wave_sync();
            const int64_t ci = w0 + lane;
            if (ci >= nch) continue;
            const int64_t c0 = a0 + 16 * ci;
            const int64_t lo = max<int64_t>(c0, cb), hi = min<int64_t>(c0 + 16, end);
            uint32_t wd[4] = {0, 0, 0, 0};
            int64_t ts = cb + ex[t], te = cb + ex[t + 1];   // row t's bytes [ts, te)
            int64_t src = rbase[t] + static_cast<int32_t>(v.u64(rbase[t] + a.bitmap_bytes + 8 * k) >> 32);
            for (int64_t p = lo; p < hi; p++) {
              while (p >= te) {
                t++;
                ts = te;
                te = cb + ex[t + 1];
                src = rbase[t] + static_cast<int32_t>(v.u64(rbase[t] + a.bitmap_bytes + 8 * k) >> 32);
              }
              const uint32_t byte = v.u8(src + (p - ts));
              wd[(p - c0) >> 2] |= byte << (8 * ((p - c0) & 3));
            }
            if (lo == c0 && hi == c0 + 16) {
              using v4 = __attribute__((ext_vector_type(4))) uint32_t;
              __builtin_nontemporal_store(v4{wd[0], wd[1], wd[2], wd[3]},
                                          gl(reinterpret_cast<v4*>(dst + c0)));
            } else {
              for (int64_t p = lo; p < hi; p++)
                gl(dst)[p] = static_cast<uint8_t>(wd[(p - c0) >> 2] >> (8 * ((p - c0) & 3)));
            }
          }
          continue;
        }
        // LIST of fixed-width elements: child entries [cb, cb + wt), one per lane, 64-bit words
        // of the child bitmaps aligned to the destination (put_bits64).  The owner row of each
        // element: rows mark their first element's lane in `own`, a wave max-scan spreads it.
        const int ew = c.width == 0 ? 1 : c.width;
        const int sh0 = static_cast<int>(cb & 63);
        const int64_t span = sh0 + wt;
        const int32_t my_ex = ex[lane];
        const bool has = live && ex[lane + 1] > my_ex;
        int carry = 0;
        for (int64_t u0 = 0; u0 < span; u0 += kWs) {
          const int64_t i0 = u0 - sh0;                  // element index of lane 0
          const int64_t i = i0 + lane;                  // element index in the wave's range
          const bool act = i >= 0 && i < wt;
          own[lane] = -1;
          wave_sync();
          if (has && my_ex >= i0 && my_ex < i0 + kWs) own[my_ex - i0] = lane;
          wave_sync();
          const int t = max(wave_max_scan(own[lane]), carry);
          carry = __shfl(t, 63, 64);
          wave_sync();
          bool valid = false;
          uint64_t x = 0;
          if (act) {
            const int64_t rb = rbase[t];                // the array (checked by view_count)
            const int64_t p = rb + static_cast<int32_t>(v.u64(rb + a.bitmap_bytes + 8 * k) >> 32);
            const int64_t n = ex[t + 1] - ex[t];
            const int64_t j = i - ex[t];
            valid = !((v.u8(p + 8 + (j >> 3)) >> (j & 7)) & 1);
            if (valid) x = v.load(p + 8 + bm_bytes(n) + j * ew, ew);
            const int64_t e = cb + i;
            if (e < cap) {
              switch (c.width) {
                case 8: __builtin_nontemporal_store(x, gl(reinterpret_cast<uint64_t*>(dst)) + e); break;
                case 4: gl(reinterpret_cast<uint32_t*>(dst))[e] = static_cast<uint32_t>(x); break;
                case 2: gl(reinterpret_cast<uint16_t*>(dst))[e] = static_cast<uint16_t>(x); break;
                case 1: gl(dst)[e] = static_cast<uint8_t>(x); break;
                default: break;                           // bool elements: bits below
              }
            }
          }
          const uint64_t am = __ballot(act);
          const int64_t gbit0 = cb - sh0 + u0;            // 64-aligned
          if (c.elem_validity) put_bits64(c.elem_validity, gbit0, __ballot(act && valid), am, cap);
          if (c.width == 0) put_bits64(dst, gbit0, __ballot(act && valid && x != 0), am, cap);
        }
      }
    }
    if (nseq == 0) break;
    __syncthreads();                                      // ws / ts reused by the next chunk
  }
}

}  // namespace

// LDS per wave: the stage, sized from the batch's expected row bytes (row_hint: mean bytes per
// row, from the output capacities; 64 rows + 10 % + 512 B, 2 .. 16 KB) + the per-wave starts.  A
// wave whose rows exceed its stage reads HBM instead (correct, slower).
int launch_decode_var_ws(const VarArgs& a, const uint8_t* rows, const int64_t* offs,
                         uint64_t* status, int nseq, int64_t nb, int nt, double row_hint,
                         hipStream_t stream) {
  int64_t stage = static_cast<int64_t>(row_hint * kWs * 1.1) + 512;
  stage = (stage + 255) & ~int64_t(255);
  if (stage < 2048) stage = 2048;
  if (stage > 16384) stage = 16384;
  const int nc = nseq < 1 ? 1 : (nseq > kSeqChunk ? kSeqChunk : nseq);
  const size_t lds = static_cast<size_t>(nt / kWs) * wave_lds(static_cast<uint32_t>(stage), nc);
  auto launch = [&](auto kernel) -> int {
    static thread_local size_t raised = 0;
    if (lds > 64 * 1024 && lds > raised) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               static_cast<int>(lds));
      if (e != hipSuccess) return check_hip(e, "hipFuncSetAttribute");
      raised = lds;
    }
    hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(nb)), dim3(nt), lds, stream, a, rows,
                       offs, status, nseq, static_cast<uint32_t>(stage));
    return check_hip(hipGetLastError(), "decode_var_ws launch");
  };
  if (nt == 512) return launch(decode_var_ws<512>);
  return launch(decode_var_ws<256>);
}

}  // namespace fury
