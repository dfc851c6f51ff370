// var_lds.hip — LDS-staged single-pass decode / row->Arrow of flat schemas with variable-length
// fields (STRING/BINARY, DECIMAL, LIST of fixed-width elements), up to kLdsMaxSeq string / list
// columns.  Reference semantics as var_dev.h (UnsafeTrait.getBinary / getArray,
// BinaryArray.toXxxArray, ArrowWriter StringWriter / ListWriter:
// FMT/row/binary/UnsafeTrait.java:115-178, FMT/vectorized/ArrowWriter.java:421-540).
//
// Why a second decode: the register-staged decode_var_reg reads each row's null word and slots
// with row-strided 8-byte loads (thread = row), so every load instruction touches ~one cache line
// per lane and the vector-memory pipeline, not HBM, bounds it (its loads alone take 288 us of a
// 10M-row mixed decode).  Here a tile's rows -- one contiguous byte range -- arrive by LDS-DMA
// (global_load_lds, 16 B per lane, every piece in flight at once, no VGPRs), and everything after
// reads LDS:
//   1. ticket -> tile b (tiles numbered in start order, so every look-back wait ends);
//   2. DMA the tile's row range into LDS; zero the output images meanwhile;
//   3. per string / list column: counts, wave scans (32-bit), wave totals to LDS -- one barrier;
//   4. tile totals, aggregates published; fixed-width columns, validity, bool bits and decimals
//      leave as coalesced column stores; string bytes / list elements are OR-ed into LDS images
//      of the tile's output ranges (laid out from the tile totals alone);
//   5. decoupled look-back (a wave per column), one barrier;
//   6. Arrow offsets, then the images leave as 16-B stores at the resolved positions.
// Columns are walked in uniform loops over the argument block (scalar loads), so one instance
// serves every column count.  A tile whose rows exceed the stage reads them from HBM (same code,
// global pointer); a column whose tile payload exceeds its image is written directly.
#define FURY_VAR_LDS
#include "var_dev.h"

#include <algorithm>

namespace fury {

namespace {

constexpr int kLdsMaxSeq = 32;       // string / list columns this kernel chains
constexpr int kLdsMaxWaves = 8;      // NT <= 512

struct LdsDecShared {
  int64_t base[kLdsMaxSeq];                  // resolved global start of the tile's range
  uint32_t wtot[kLdsMaxSeq][kLdsMaxWaves];   // per-wave totals
  int64_t tile;
};

__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ uint32_t sgpr(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Decoupled look-back over one column's status words, laid out contiguously by tile (sq[t]), so
// a 64-lane window is 512 contiguous bytes -- 4 requests to the cross-XCD coherence point instead
// of 24 for the [tile][column] layout.  The first window is the 16 nearest tiles (lanes >= 16
// idle), since the nearest inclusive prefix is usually close; then 64-tile windows.  Only
// unpublished words nearer than the nearest inclusive are re-read while waiting.  A look-back that
// gives up raises the host-visible error word, as look_back_bounded.
constexpr int kLookFirst = 16;       // first look-back window (tiles)

__device__ __forceinline__ uint64_t look_first(const uint64_t* sq, int64_t b) {
  const int lane = threadIdx.x & 63;
  const int64_t idx = b - 1 - lane;
  return lane >= kLookFirst ? 0 : idx >= 0 ? ld_status(sq + idx) : kInc;
}

// first: the first window's words when the caller issued them early (look_first), else NULL.
__device__ int64_t look_back_col(const uint64_t* sq, int64_t b, uint32_t* err, const uint64_t* first) {
  const int lane = threadIdx.x & 63;
  int64_t excl = 0;
  uint32_t spins = 0;
  int width = kLookFirst;
  for (int64_t j = b - 1;; j -= width, width = 64) {
    const int64_t idx = j - lane;
    const bool in = lane < width;
    uint64_t v = (first && j == b - 1) ? *first : !in ? 0 : idx >= 0 ? ld_status(sq + idx) : kInc;
    uint64_t inc;
    int stop;
    for (;;) {
      inc = __ballot(in && (v >> 62) == 2);
      stop = inc ? __builtin_ctzll(inc) : width - 1;
      const uint64_t upto = stop == 63 ? ~0ull : ((2ull << stop) - 1);
      if ((__ballot(in && (v >> 62) == 0) & upto) == 0) break;
      if (++spins > (1u << 24)) {
        if (lane == 0 && err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return 0;
      }
      __builtin_amdgcn_s_sleep(1);
      if (in && (v >> 62) == 0 && lane <= stop) v = ld_status(sq + idx);
    }
    excl += wave_sum(lane <= stop ? static_cast<int64_t>(v & kValMask) : 0);
    if (inc) return excl;
  }
}

// LDS image bytes of a column's tile range of t entries (bytes / elements), + its bit image.
__device__ __forceinline__ uint32_t img_need(const VarCol& c, uint32_t t, uint32_t* vb) {
  uint32_t need;
  if (c.kind == kBytes) need = static_cast<uint32_t>(r16(int64_t(t) + 16));
  else if (c.width == 0) need = static_cast<uint32_t>(r16((((int64_t(t) + 31) >> 5) + 1) * 4));
  else need = static_cast<uint32_t>(r16(int64_t(t) * c.width + 16));
  *vb = need;
  if (c.kind == kListFixed && c.elem_validity)
    need += static_cast<uint32_t>(r16((((int64_t(t) + 31) >> 5) + 1) * 4));
  return need;
}

// Bits [j, j + 8) of a bitmap (j % 8 == 0), as the low bits.
__device__ __forceinline__ uint32_t bits8(const uint8_t* bm, int64_t j) {
  return bm[j >> 3];
}

template <int NT, bool kLds>
__device__ __forceinline__ void lds_tile(const VarArgs& a, const uint8_t* row, bool live,
                                         int64_t b, int64_t nb, int64_t r0, int nr, int nseq,
                                         uint32_t* pos, uint8_t* img, uint32_t img_cap,
                                         LdsDecShared& sh, uint64_t* status) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r = r0 + tid;
  const int bmb = a.bitmap_bytes;
  // 3. counts and wave-level scans of every string / list column
  {
    int q = 0;
    for (int k = 0; k < a.ncols; k++) {
      const VarCol& c = a.col[k];   // kernarg: scalar loads (never a.tab here)
      if (!is_seq(c)) continue;
      uint32_t cnt = 0;
      if (live && !((row[k >> 3] >> (k & 7)) & 1)) {
        const uint64_t slot = *reinterpret_cast<const uint64_t*>(row + bmb + 8 * k);
        cnt = c.kind == kBytes
                  ? static_cast<uint32_t>(slot)
                  : static_cast<uint32_t>(*reinterpret_cast<const int64_t*>(row + static_cast<int32_t>(slot >> 32)));
      }
      const uint32_t inc = wave_incl_scan32(cnt);
      pos[q * NT + tid] = inc - cnt;
      if (lane == 63) sh.wtot[q][wave] = inc;
      q++;
    }
  }
  __syncthreads();
  // 4a. tile totals -> aggregates published first, so successors can resolve early
  if (tid < nseq) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) t += sh.wtot[tid][w];
    st_status(status + tid * nb + b, (b == 0 ? kInc : kAgg) | static_cast<uint64_t>(t));
  }
  // 4b. every column: validity, fixed values, images of the string / list ranges
  const int64_t rbase = r0 + 64 * wave;
  const int64_t nvalid = a.nrows - rbase;
  const int nwords = nvalid >= 64 ? 2 : nvalid <= 0 ? 0 : static_cast<int>((nvalid + 31) >> 5);
  uint32_t used = 0;
  int q = 0;
  for (int k = 0; k < a.ncols; k++) {
    const VarCol& c = a.col[k];   // kernarg: scalar loads (never a.tab here)
    const bool isnull = !live || ((row[k >> 3] >> (k & 7)) & 1);
    if (c.validity && !(a.dbg & 8)) {
      const uint64_t ok = __ballot(!isnull);
      if (lane < nwords)
        gl(reinterpret_cast<uint32_t*>(c.validity))[(rbase >> 5) + lane] = static_cast<uint32_t>(ok >> (32 * lane));
    }
    uint8_t* dst = const_cast<uint8_t*>(c.values);
    const uint64_t slot = isnull ? 0 : *reinterpret_cast<const uint64_t*>(row + bmb + 8 * k);
    if (c.kind == kFixed) {
      if (live && dst && !(a.dbg & 8)) {
        switch (c.width) {
          case 8: __builtin_nontemporal_store(slot, gl(reinterpret_cast<uint64_t*>(dst)) + r); break;
          case 4: __builtin_nontemporal_store(static_cast<uint32_t>(slot), gl(reinterpret_cast<uint32_t*>(dst)) + r); break;
          case 2: gl(reinterpret_cast<uint16_t*>(dst))[r] = static_cast<uint16_t>(slot); break;
          default: gl(dst)[r] = static_cast<uint8_t>(slot); break;
        }
      }
      continue;
    }
    if (c.kind == kBool) {
      const uint64_t bits = __ballot((slot & 0xff) != 0);
      if (lane < nwords && dst)
        gl(reinterpret_cast<uint32_t*>(dst))[(rbase >> 5) + lane] = static_cast<uint32_t>(bits >> (32 * lane));
      continue;
    }
    if (c.kind == kDecimal) {
      if (live && dst) {
        uint64_t lo = 0, hi = 0;
        if (!isnull) {
          const uint64_t* s = reinterpret_cast<const uint64_t*>(row + static_cast<int32_t>(slot >> 32));
          lo = s[0];
          hi = s[1];
        }
        auto d = gl(reinterpret_cast<uint64_t*>(dst + 16 * r));
        d[0] = lo;
        d[1] = hi;
      }
      continue;
    }
    if (!is_seq(c)) continue;
    // string / list column q: final in-tile prefix, image slot
    uint32_t t = 0, wpre = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
      const uint32_t s = sh.wtot[q][w];
      t += s;
      wpre += w < wave ? s : 0;
    }
    t = sgpr(t);
    const uint32_t ex = pos[q * NT + tid] + wpre;
    pos[q * NT + tid] = ex;
    q++;
    if (!dst || t == 0 || (a.dbg & 16)) continue;
    uint32_t vb;
    const uint32_t need = img_need(c, t, &vb);    // uniform layout, as in step 6
    const uint32_t at = used;
    if (at + need > img_cap) continue;         // written directly after the look-back
    used += need;
    if (isnull) continue;
    const uint8_t* src = row + static_cast<int32_t>(slot >> 32);
    uint8_t* im = img + at;
    if (c.kind == kBytes) {
      const uint32_t len = static_cast<uint32_t>(slot);
      uint64_t* iw = reinterpret_cast<uint64_t*>(im) + (ex >> 3);
      const int sft = static_cast<int>(ex & 7) * 8;
      const uint64_t* s64 = reinterpret_cast<const uint64_t*>(src);
      const uint32_t nw = (len + 7) >> 3;
      for (uint32_t j = 0; j < nw; j++) {
        uint64_t x = s64[j];
        const uint32_t rem = len - 8 * j;
        if (rem < 8) x &= (~0ull) >> (8 * (8 - rem));
        atomicOr(reinterpret_cast<unsigned long long*>(iw + j), x << sft);
        if (sft && (x >> (64 - sft))) atomicOr(reinterpret_cast<unsigned long long*>(iw + j + 1), x >> (64 - sft));
      }
      continue;
    }
    // LIST of fixed-width elements: values at element slots, bits OR-ed
    const int64_t n = *reinterpret_cast<const int64_t*>(src);
    const int ew = c.width == 0 ? 1 : c.width;
    const uint8_t* bm = src + 8;
    const uint8_t* ev = src + 8 + bm_bytes(n);
    uint32_t* bimg = reinterpret_cast<uint32_t*>(im + vb);
    for (int64_t j0 = 0; j0 < n; j0 += 8) {
      const int lim = static_cast<int>(min<int64_t>(8, n - j0));
      const uint32_t nulls = bits8(bm, j0);
      for (int u = 0; u < lim; u++) {
        const int64_t j = j0 + u;
        const bool valid = !((nulls >> u) & 1);
        uint64_t x = 0;
        if (valid) {
          switch (ew) {
            case 8: x = reinterpret_cast<const uint64_t*>(ev)[j]; break;
            case 4: x = reinterpret_cast<const uint32_t*>(ev)[j]; break;
            case 2: x = reinterpret_cast<const uint16_t*>(ev)[j]; break;
            default: x = ev[j]; break;
          }
        }
        const int64_t e = ex + j;                 // tile-relative element
        if (c.width == 8) {
          reinterpret_cast<uint64_t*>(im)[e] = x;
        } else if (c.width == 0) {
          if (x & 0xff) atomicOr(reinterpret_cast<uint32_t*>(im) + (e >> 5), 1u << (e & 31));
        } else if (x) {
          const int64_t bo = e * ew;
          atomicOr(reinterpret_cast<uint32_t*>(im) + (bo >> 2), static_cast<uint32_t>(x << (8 * (bo & 3))));
        }
        if (c.elem_validity && valid) atomicOr(bimg + (e >> 5), 1u << (e & 31));
      }
    }
  }
  // 5. prefixes: one wave per column (round robin)
  for (int qq = wave; qq < nseq; qq += NT / 64) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) t += sh.wtot[qq][w];
    const int64_t pre = (b == 0 || (a.dbg & 32)) ? 0 : look_back_col(status + qq * nb, b, a.err, nullptr);
    if (lane == 0) {
      sh.base[qq] = pre;
      if (b > 0) st_status(status + qq * nb + b, kInc | static_cast<uint64_t>(pre + t));
    }
  }
  __syncthreads();
  // 6. Arrow offsets, direct writes of columns that missed their image, image stores
  used = 0;
  q = 0;
  for (int k = 0; k < a.ncols; k++) {
    const VarCol& c = a.col[k];   // kernarg: scalar loads (never a.tab here)
    if (!is_seq(c)) continue;
    const int64_t gb = sh.base[q];
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) t += sh.wtot[q][w];
    t = sgpr(t);
    const uint32_t ex = pos[q * NT + tid];
    q++;
    if (live) gl(c.offsets)[r] = static_cast<int32_t>(gb + ex);
    if (b == nb - 1 && tid == nr - 1) gl(c.offsets)[a.nrows] = static_cast<int32_t>(gb + t);
    uint8_t* dst = const_cast<uint8_t*>(c.values);
    if (!dst || t == 0 || (a.dbg & 16)) continue;
    uint32_t vb;
    const uint32_t need = img_need(c, t, &vb);
    const int64_t cap = c.capacity;
    if (used + need <= img_cap) {
      const uint8_t* im = img + used;
      used += need;
      const int64_t n = max<int64_t>(0, min<int64_t>(t, cap - gb));
      if (c.kind == kBytes) {
        store_shifted<NT>(dst + gb, im, n);
        continue;
      }
      if (c.width == 0) store_bits_shifted<NT>(dst, reinterpret_cast<const uint32_t*>(im), gb, n);
      else store_shifted<NT>(dst + gb * c.width, im, n * c.width);
      if (c.elem_validity)
        store_bits_shifted<NT>(c.elem_validity, reinterpret_cast<const uint32_t*>(im + vb), gb, n);
      continue;
    }
    // this tile's range did not fit the image: each thread writes its own entries
    if (!live || ((row[k >> 3] >> (k & 7)) & 1)) continue;
    const uint64_t slot = *reinterpret_cast<const uint64_t*>(row + bmb + 8 * k);
    const uint8_t* src = row + static_cast<int32_t>(slot >> 32);
    const int64_t p = gb + ex;
    if (c.kind == kBytes) {
      put_bytes(dst, p, src, max<int64_t>(0, min<int64_t>(static_cast<uint32_t>(slot), cap - p)));
      continue;
    }
    const int64_t n = *reinterpret_cast<const int64_t*>(src);
    const int ew = c.width == 0 ? 1 : c.width;
    const uint8_t* ev = src + 8 + bm_bytes(n);
    for (int64_t j = 0; j < n; j++) {
      const int64_t e = p + j;
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
}

// Dynamic LDS: [pos: nseq x NT int32][stage: stage_cap][images: img_cap].
template <int NT>
__global__ __launch_bounds__(NT) void decode_var_lds(VarArgs a, const uint8_t* __restrict__ rows,
                                                     const int64_t* __restrict__ offs,
                                                     uint64_t* __restrict__ status,
                                                     uint32_t* __restrict__ ticket, int nseq,
                                                     uint32_t stage_cap, uint32_t img_cap) {
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  extern __shared__ __attribute__((aligned(16))) uint64_t dyn[];
  __shared__ LdsDecShared sh;
  uint32_t* pos = reinterpret_cast<uint32_t*>(dyn);
  uint8_t* stage = reinterpret_cast<uint8_t*>(dyn) + static_cast<uint32_t>(nseq) * NT * 4;
  uint8_t* img = stage + stage_cap;
  const int tid = threadIdx.x;
  // tiles numbered by a ticket (start order), so every look-back wait ends; blockIdx order
  // (FURY_VAR_DBG 4096 | 128 with FURY_DIAGNOSTIC=1) is for timing only: this kernel's look-back
  // does not help itself
  const bool order = (a.dbg & 4096) && (a.dbg & 128);
  if (!order) {
    if (tid == 0) sh.tile = atomicAdd(ticket, 1u);
    __syncthreads();
  }
  const int64_t b = order ? static_cast<int64_t>(blockIdx.x) : sh.tile, nb = gridDim.x;
  const int64_t r0 = b * NT;
  const int nr = static_cast<int>(min<int64_t>(NT, a.nrows - r0));
  const bool live = tid < nr;
  const int64_t rbeg = offs[r0], rend = offs[r0 + nr];
  const int64_t myoff = offs[live ? r0 + tid : r0];
  const bool staged = rend - rbeg + 32 <= static_cast<int64_t>(stage_cap);
  uint32_t d0 = 0;
  if (staged) {
    uint32_t at = 0;
    d0 = stage_range<NT>(stage, at, rows + rbeg, rows + rend);
  }
  for (uint32_t i = 16 * tid; i < img_cap; i += 16 * NT) *reinterpret_cast<v4*>(img + i) = v4{0, 0, 0, 0};
  if (a.dbg & 128) {         // DIAGNOSTIC: the row staging only (a dependent store keeps it)
    if (staged) wait_dma();
    __syncthreads();
    const uint64_t x = staged ? *reinterpret_cast<const uint64_t*>(stage + 8 * tid) : 0;
    if (x == 0x123456789abcdefull) status[0] = x;
    return;
  }
  if (staged) {
    wait_dma();
    __syncthreads();
    lds_tile<NT, true>(a, stage + d0 + (myoff - rbeg), live, b, nb, r0, nr, nseq, pos, img, img_cap,
                       sh, status);
  } else {
    lds_tile<NT, false>(a, rows + myoff, live, b, nb, r0, nr, nseq, pos, img, img_cap, sh, status);
  }
}

}  // namespace

int lds_decode_max_seq() { return kLdsMaxSeq; }



// stage / img: LDS bytes for a tile's rows and output images (the launcher's estimates).
int launch_decode_var_lds(const VarArgs& a, const uint8_t* rows, const int64_t* offs,
                          uint64_t* status, uint32_t* ticket, int nseq, int nt, uint32_t stage,
                          uint32_t img, int64_t ntiles, hipStream_t stream) {
  const size_t lds = static_cast<size_t>(nseq) * nt * 4 + stage + img;
  static bool attr_set[3] = {false, false, false};
  const int which = nt == 512 ? 1 : nt == 128 ? 2 : 0;
  if (!attr_set[which]) {
    const void* fn = nt == 512 ? reinterpret_cast<const void*>(decode_var_lds<512>)
                     : nt == 128 ? reinterpret_cast<const void*>(decode_var_lds<128>)
                                 : reinterpret_cast<const void*>(decode_var_lds<256>);
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    if (e != hipSuccess) return check_hip(e, "hipFuncSetAttribute");
    attr_set[which] = true;
  }
  if (nt == 128)
    hipLaunchKernelGGL(decode_var_lds<128>, dim3(ntiles), dim3(128), lds, stream, a, rows, offs,
                       status, ticket, nseq, stage, img);
  else if (nt == 512)
    hipLaunchKernelGGL(decode_var_lds<512>, dim3(ntiles), dim3(512), lds, stream, a, rows, offs,
                       status, ticket, nseq, stage, img);
  else
    hipLaunchKernelGGL(decode_var_lds<256>, dim3(ntiles), dim3(256), lds, stream, a, rows, offs,
                       status, ticket, nseq, stage, img);
  return check_hip(hipGetLastError(), "decode_var_lds launch");
}

}  // namespace fury
