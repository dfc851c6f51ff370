// wide.hip — decode / row -> Arrow of flat variable-length schemas wider than kRegCols (16)
// fields, up to kMaxWideVarCols: a count pass, one device scan, a write pass.  No look-back.
//
// Reference semantics are the register-staged decode's (var_dev.h decode_var_reg): the getters of
// BinaryRow (UnsafeTrait.getBinary / getArray, FMT/row/binary/UnsafeTrait.java:115-178;
// BinaryArray.pointTo / toXxxArray, FMT/row/binary/BinaryArray.java:69-78,157-197) and ArrowWriter's
// StringWriter / ListWriter (FMT/vectorized/ArrowWriter.java:421-540): a null field is a null
// entry (value 0, zero-length range), a value any of whose bytes leave the batch decodes as null
// and is reported (IndexOutOfBoundsException, slot_count), payloads are clipped to the columns'
// capacities.
//
// MI355X design (the 256-row tile kernel this replaces ran 33 fields x 5M rows
// at 0.43 TB/s: its 148 KB tiles never fit the 32 KB stage, so every lane read its 581-B row
// from HBM field by field, and 33 look-back chains -- one per STRING / LIST column, in rounds of
// 8 with barriers -- serialised the tiles).  A tile is 64 rows: lane = row, the tile's contiguous
// row bytes staged in LDS by LDS-DMA (rows past the stage from HBM), its four waves taking the
// fields round robin, so there is one barrier per tile (after the stage) and none per field:
//   count pass  each wave sums its STRING / LIST fields' counts over the 64 rows (wave
//               reduction) -> counts[q][tile] (int64);
//   scan        one exclusive device scan of the flat [field][tile] array (field q's tile bases
//               are its entries minus the entry of tile 0);
//   write pass  per field: validity and BOOL values as ballot words, fixed-width values as
//               64-row coalesced stores, Arrow offsets = tile base + wave scan, and the tile's
//               payload / element range assembled in the wave's own LDS image and stored as
//               whole 16-B lines (byte-exact at the two ends; element bitmaps with atomic OR on
//               the two edge words they share with neighbouring tiles).
#include <algorithm>
#include <type_traits>

#include "var_dev.h"

namespace fury {

namespace {

constexpr int kWideRows = 64;                   // rows per tile (lane = row)
// Waves per tile (NT = 64 x waves threads) share its fields round robin: tuning "wide_threads"
// (256 / 512 / 1024).

// Typed reads through a pointer that keeps its address space (LDS stage or HBM rows): one
// instance per space, so no access is FLAT (a flat access counts against both the vector-memory
// and the LDS / scalar counters, and every later wait waits for it).
template <class P, class T>
using AsT = typename std::conditional<
    std::is_same<typename std::remove_pointer<P>::type,
                 __attribute__((address_space(3))) const uint8_t>::value,
    __attribute__((address_space(3))) const T, __attribute__((address_space(1))) const T>::type;
template <class T, class P>
__device__ __forceinline__ T ldv(P p) { return *reinterpret_cast<AsT<P, T>*>(p); }
// T in the address space of the (non-const) byte type D: global when D is, else generic (an LDS
// image derived from the kernel's shared array, which the compiler resolves)
template <class D, class T>
using DstT = typename std::conditional<
    std::is_same<D, __attribute__((address_space(1))) uint8_t>::value,
    __attribute__((address_space(1))) T, T>::type;
using LdsC = __attribute__((address_space(3))) const uint8_t;
using GlbC = __attribute__((address_space(1))) const uint8_t;

// The tile's row bytes [offs[r0], offs[r0 + nr]) (up to stage_cap of them) in LDS.
struct WideStage {
  const uint8_t* rows;
  LdsC* stg;
  uintptr_t lo, hi;                             // absolute addresses held by stg
  __device__ __forceinline__ bool staged(int64_t p, int64_t len) const {
    const uintptr_t q = reinterpret_cast<uintptr_t>(rows + p);
    return q >= lo && q + len <= hi;
  }
  // f(pointer to batch byte p): the LDS copy when [p, p + len) is staged (LDS keeps the batch's
  // alignment: the stage starts at a 16-aligned address), else HBM
  template <class F>
  __device__ __forceinline__ auto with(int64_t p, int64_t len, F f) const {
    if (staged(p, len)) return f(stg + (reinterpret_cast<uintptr_t>(rows + p) - lo));
    return f((GlbC*)(rows + p));
  }
};

template <int NT>
__device__ __forceinline__ WideStage wide_stage(uint8_t* stg, const uint8_t* rows, const int64_t* offs,
                                                int64_t r0, int nr, int64_t total, uint32_t cap) {
  const int64_t tt = max<int64_t>(total, 0);
  const int64_t g0 = min<int64_t>(max<int64_t>(gl(offs)[r0], 0), tt);
  const int64_t g1 = min<int64_t>(max<int64_t>(gl(offs)[r0 + nr], g0), tt);
  WideStage s{rows, (LdsC*)(stg), 0, 0};
  // 16-aligned start: LDS byte 0 = s.lo, so staged reads keep their HBM alignment.  With a rows
  // pointer that is not 16-aligned the first piece starts up to 15 bytes before the batch -- the
  // aligned 16-B piece holding its first byte, which never leaves that byte's page (the rule every
  // kernel's whole-word reads follow); those bytes are never used: staged() admits only [rows+p,..).
  s.lo = reinterpret_cast<uintptr_t>(rows + g0) & ~uintptr_t(15);
  s.hi = min<uintptr_t>(reinterpret_cast<uintptr_t>(rows + g1), s.lo + cap);
  uint32_t at = 0;
  if (s.hi > s.lo)
    stage_range<NT>(stg, at, reinterpret_cast<const uint8_t*>(s.lo),
                              reinterpret_cast<const uint8_t*>(s.hi));
  else
    s.hi = s.lo;
  return s;
}

// Null test + count of field k (STRING: payload bytes, LIST: elements) of the row at absolute
// byte `base` (rok: its header is inside the batch), exactly as slot_count counts; *slot = the
// slot word (0 when null).  A value outside the batch sets *bad and decodes as null.
template <class Col>
__device__ __forceinline__ int64_t wide_field(const Col& c, int k, const WideStage& S, int64_t base,
                                              bool rok, int bitmap_bytes, int64_t total,
                                              uint64_t* slot, bool* null, bool* bad) {
  *bad = false;
  *slot = 0;
  *null = true;
  if (!rok) return 0;
  const int64_t sp = base + bitmap_bytes + 8 * k;
  uint32_t nb = 0;
  uint64_t sv = 0;
  S.with(base, bitmap_bytes + 8 * (k + 1), [&](auto hp) {
    nb = ldv<uint8_t>(hp + (k >> 3));
    sv = ldv<uint64_t>(hp + (sp - base));
    return 0;
  });
  *null = (nb >> (k & 7)) & 1;
  if (*null) return 0;
  *slot = sv;
  if (c.kind < kBytes) return 0;
  const int64_t p = base + static_cast<int32_t>(sv >> 32);
  int64_t n = 0;
  if (c.kind == kListFixed) {
    if (!span_ok(p, 8, total)) {
      *bad = true;
    } else {
      const int64_t h = S.with(p, 8, [&](auto ap) { return ldv<int64_t>(ap); });
      n = list_count(static_cast<int32_t>(h), c.width, p, total, bad);
    }
  } else {
    n = slot_count(c.kind, c.width, sv, base, S.rows, total, bad);
  }
  if (*bad) {
    *null = true;
    *slot = 0;
    n = 0;
  }
  return n;
}

// len bytes of a source (LDS or HBM, P; 8-byte aligned in well-formed rows, any alignment in
// malformed ones) to byte q of dst (LDS image or HBM, any alignment): 32-bit words wholly inside
// the range written whole, the edges byte by byte (the neighbouring bytes belong to other lanes).
// The source is read as ABSOLUTELY aligned 8-byte words (the LDS stage keeps the batch's
// alignment), so every word read holds a byte of [src, src + len): a misaligned slot ending at the
// batch's end never reads past it.
template <class P, class D>
__device__ __forceinline__ void wcopy(D* dst, int64_t q, P src, int64_t len) {
  if (len <= 0) return;
  const int a = static_cast<int>(reinterpret_cast<uintptr_t>(src) & 7);
  src = src - a;                                 // aligned; source byte i = stream byte a + i
  auto sb = [&](int64_t i) -> uint32_t {
    const int64_t b = a + i;
    return static_cast<uint32_t>((ldv<uint64_t>(src + 8 * (b >> 3)) >> (8 * (b & 7))) & 0xff);
  };
  const int64_t end = q + len;
  const int64_t w0 = (q + 3) >> 2, w1 = end >> 2;
  if (w0 >= w1) {
    for (int64_t i = 0; i < len; i++) dst[q + i] = static_cast<uint8_t>(sb(i));
    return;
  }
  for (int64_t i = q; i < 4 * w0; i++) dst[i] = static_cast<uint8_t>(sb(i - q));
  const int64_t d = 4 * w0 - q;
  auto d32 = reinterpret_cast<DstT<D, uint32_t>*>(dst);
  for (int64_t w = w0; w < w1; w++) {
    const int64_t si = a + d + 4 * (w - w0);
    const int64_t j = si >> 3;
    const int o = static_cast<int>(si & 7);
    uint64_t x = ldv<uint64_t>(src + 8 * j) >> (8 * o);
    if (o > 4) x |= ldv<uint64_t>(src + 8 * (j + 1)) << (64 - 8 * o);
    d32[w] = static_cast<uint32_t>(x);
  }
  for (int64_t i = 4 * w1; i < end; i++) dst[i] = static_cast<uint8_t>(sb(i - q));
}

// Element j (ew bytes) of a BinaryArray of n elements at ap (LDS or HBM), 0 when null.
template <class P>
__device__ __forceinline__ uint64_t welem(P ap, int64_t n, int64_t j, int ew, bool* valid) {
  *valid = !((ldv<uint8_t>(ap + 8 + (j >> 3)) >> (j & 7)) & 1);
  if (!*valid) return 0;
  const P ev = ap + 8 + bm_bytes(n) + j * ew;
  switch (ew) {
    case 8: return ldv<uint64_t>(ev);
    case 4: return ldv<uint32_t>(ev);
    case 2: return ldv<uint16_t>(ev);
    default: return ldv<uint8_t>(ev);
  }
}

// Wave-level: bits [gbit0, gbit0 + n) of a bitmap from a bit image (LDS, image bit i = bit
// gbit0 + i, >= 1 word of padding): whole words stored, the edge words (shared with the
// neighbouring tiles) by atomic and/or of exactly these bits.
__device__ __forceinline__ void wave_store_bits(uint8_t* bits, const uint32_t* img, int64_t gbit0,
                                                int64_t n) {
  if (n <= 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t end = gbit0 + n;
  const int64_t w0 = gbit0 >> 5, w1 = (end + 31) >> 5;
  uint32_t* g = reinterpret_cast<uint32_t*>(bits);
  for (int64_t w = w0 + lane; w < w1; w += 64) {
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

// Stores bytes img[0, n) of the wave's LDS image (16-aligned, >= 16 readable bytes past n) to g
// (any alignment, every byte of [g, g + n) this tile's): bytes to g's 16-byte boundary, 16-B
// non-temporal stores funnel-shifted out of aligned image words, the byte tail.
__device__ __forceinline__ void wave_store_image(uint8_t* g, const uint8_t* img, int64_t n) {
  using v4 = __attribute__((ext_vector_type(4))) uint32_t;
  if (n <= 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t head = min<int64_t>(n, (16 - (reinterpret_cast<uintptr_t>(g) & 15)) & 15);
  const int64_t body = (n - head) >> 4;
  const int64_t t0 = head + 16 * body;
  if (lane < head) gl(g)[lane] = img[lane];
  if (lane < n - t0) gl(g)[t0 + lane] = img[t0 + lane];
  const uint64_t* i64 = reinterpret_cast<const uint64_t*>(img);
  const int sh = static_cast<int>(head & 7) * 8;
  for (int64_t m = lane; m < body; m += 64) {
    const int64_t q = (head + 16 * m) >> 3;
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

// Count pass: counts[q * ntiles + t] = STRING bytes / LIST elements of seq field q in tile t.
template <int NT>
__global__ __launch_bounds__(NT) void wide_count_kernel(VarArgs a, const uint8_t* __restrict__ rows,
                                                                  const int64_t* __restrict__ offs,
                                                                  int64_t* __restrict__ counts,
                                                                  int64_t ntiles, uint32_t stage_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t t = blockIdx.x;
  const int64_t r0 = t * kWideRows;
  const int nr = static_cast<int>(min<int64_t>(kWideRows, a.nrows - r0));
  const bool live = lane < nr;
  const int64_t r = live ? r0 + lane : r0;
  const int64_t total = gl(offs)[a.nrows];
  const int64_t base = gl(offs)[r];
  const WideStage S = wide_stage<NT>(wsm, rows, offs, r0, nr, total, stage_cap);
  __syncthreads();
  const bool rok = live && row_ok(base, a.fixed_size, total);
  if (live && !rok && wave == 0) raise_oob(a.err, r);
  int q = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (!is_seq(c)) continue;
    if (q % (NT / 64) == wave) {
      uint64_t slot;
      bool nul, bad;
      const int64_t n = wide_field(c, k, S, base, rok, a.bitmap_bytes, total, &slot, &nul, &bad);
      if (bad) raise_oob(a.err, r);
      const int64_t s = wave_sum(n);
      if (lane == 0) counts[q * ntiles + t] = s;
    }
    q++;
  }
}

// Write pass (images: per-wave LDS images of img_cap bytes + their bit images after the stage).
template <int NT>
__global__ __launch_bounds__(NT) void wide_write_kernel(VarArgs a, const uint8_t* __restrict__ rows,
                                                                  const int64_t* __restrict__ offs,
                                                                  const int64_t* __restrict__ bases,
                                                                  int64_t ntiles, uint32_t stage_cap,
                                                                  uint32_t img_cap, int offsets_only) {
  extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t t = blockIdx.x;
  const int64_t r0 = t * kWideRows;
  const int nr = static_cast<int>(min<int64_t>(kWideRows, a.nrows - r0));
  const bool live = lane < nr;
  const int64_t r = live ? r0 + lane : r0;
  const int64_t total = gl(offs)[a.nrows];
  const int64_t base = gl(offs)[r];
  const WideStage S = wide_stage<NT>(wsm, rows, offs, r0, nr, total, stage_cap);
  const uint32_t bit_cap = ((img_cap / 8 + 4 * 16) + 15) & ~15u;  // bit image bytes per wave
  uint8_t* img = wsm + ((stage_cap + 15) & ~15u) + wave * (img_cap + bit_cap);
  uint32_t* bimg = reinterpret_cast<uint32_t*>(img + img_cap);
  __syncthreads();
  const bool rok = live && row_ok(base, a.fixed_size, total);
  const int nwords = nr > 32 ? 2 : 1;                            // ballot words of the tile
  const bool last = t == ntiles - 1;
  int q = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    const bool seq = is_seq(c);
    const int qk = q;
    q += seq ? 1 : 0;
    if (k % (NT / 64) != wave) continue;
    if (offsets_only && !seq) continue;        // fury_row_decode_measure: the Arrow offsets only
    uint64_t slot;
    bool nul, bad;
    const int64_t n = wide_field(c, k, S, base, rok, a.bitmap_bytes, total, &slot, &nul, &bad);
    if (bad) raise_oob(a.err, r);
    if (c.validity && !offsets_only) {
      const uint64_t ok = __ballot(live && !nul);
      if (lane < nwords)
        gl(reinterpret_cast<uint32_t*>(c.validity))[(r0 >> 5) + lane] = static_cast<uint32_t>(ok >> (32 * lane));
    }
    uint8_t* dst = const_cast<uint8_t*>(c.values);
    if (c.kind == kBool) {
      const uint64_t bits = __ballot(live && !nul && (slot & 0xff) != 0);
      if (dst && lane < nwords)
        gl(reinterpret_cast<uint32_t*>(dst))[(r0 >> 5) + lane] = static_cast<uint32_t>(bits >> (32 * lane));
      continue;
    }
    if (c.kind == kFixed) {
      if (live && dst) {
        switch (c.width) {
          case 8: __builtin_nontemporal_store(slot, gl(reinterpret_cast<uint64_t*>(dst)) + r); break;
          case 4: __builtin_nontemporal_store(static_cast<uint32_t>(slot), gl(reinterpret_cast<uint32_t*>(dst)) + r); break;
          case 2: gl(reinterpret_cast<uint16_t*>(dst))[r] = static_cast<uint16_t>(slot); break;
          default: gl(dst)[r] = static_cast<uint8_t>(slot); break;
        }
      }
      continue;
    }
    if (c.kind == kDecimal) {
      if (live && dst) {
        uint64_t lo = 0, hi = 0;
        if (!nul) {
          S.with(base + static_cast<int32_t>(slot >> 32), 16, [&](auto dp) {
            lo = ldv<uint64_t>(dp);
            hi = ldv<uint64_t>(dp + 8);
            return 0;
          });
        }
        const auto d = gl(reinterpret_cast<uint64_t*>(dst + 16 * r));
        d[0] = lo;
        d[1] = hi;
      }
      continue;
    }
    if (!seq) continue;
    // STRING / BINARY / LIST: Arrow offsets from the tile base and a wave scan
    const int64_t inc = wave_incl_scan(n);
    const int64_t ex = inc - n;
    const int64_t tot = __shfl(inc, 63, 64);
    const int64_t gb = bases[qk * ntiles + t] - bases[qk * ntiles];
    if (live) gl(c.offsets)[r] = static_cast<int32_t>(gb + ex);
    if (last && lane == nr - 1) gl(c.offsets)[a.nrows] = static_cast<int32_t>(gb + ex + n);
    if (!dst || tot == 0 || offsets_only) continue;
    const int64_t cap = c.capacity;
    const int64_t p = base + static_cast<int32_t>(slot >> 32);   // the value (when not null)
    if (c.kind == kBytes) {
      const int64_t room = max<int64_t>(0, min<int64_t>(tot, cap - gb));
      if (tot + 16 <= img_cap) {
        if (n > 0) S.with(p, n, [&](auto sp) { wcopy(img, ex, sp, n); return 0; });
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        wave_store_image(dst + gb, img, room);
        __builtin_amdgcn_wave_barrier();
      } else if (n > 0) {                                          // a large tile range: direct
        const int64_t len = max<int64_t>(0, min<int64_t>(n, cap - (gb + ex)));
        auto gdst = gl(dst);
        S.with(p, n, [&](auto sp) { wcopy(gdst, gb + ex, sp, len); return 0; });
      }
      continue;
    }
    // LIST of fixed-width elements -> child values (nulls zero) + element validity bits
    const int ew = c.width == 0 ? 1 : c.width;
    const int64_t room = max<int64_t>(0, min<int64_t>(tot, cap - gb));   // elements that fit
    const int64_t vbytes = c.width == 0 ? 0 : tot * ew;
    const int64_t bwords = (tot + 31) / 32 + 1;                 // image bit i = global bit gb + i
    const bool fits = vbytes + 16 <= img_cap && 4 * bwords <= bit_cap;
    const int64_t abytes = 8 + bm_bytes(n) + n * ew;
    if (fits) {
      for (int64_t i = lane; i < bwords; i += 64) bimg[i] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (n > 0) S.with(p, abytes, [&](auto ap) {
        for (int64_t j = 0; j < n; j++) {
          bool valid;
          const uint64_t x = welem(ap, n, j, ew, &valid);
          const int64_t e = ex + j;
          switch (c.width) {
            case 8: reinterpret_cast<uint64_t*>(img)[e] = x; break;
            case 4: reinterpret_cast<uint32_t*>(img)[e] = static_cast<uint32_t>(x); break;
            case 2: reinterpret_cast<uint16_t*>(img)[e] = static_cast<uint16_t>(x); break;
            case 1: img[e] = static_cast<uint8_t>(x); break;
            default: break;                                    // bool elements: bits below
          }
          if (valid) atomicOr(bimg + (e >> 5), 1u << (e & 31));
        }
        return 0;
      });
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (c.width > 0) wave_store_image(dst + gb * ew, img, room * ew);
      if (c.elem_validity) wave_store_bits(c.elem_validity, bimg, gb, room);
      if (c.width == 0) {                                          // bool values: their own bits
        __builtin_amdgcn_wave_barrier();
        for (int64_t i = lane; i < bwords; i += 64) bimg[i] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (n > 0) S.with(p, abytes, [&](auto ap) {
          for (int64_t j = 0; j < n; j++) {
            bool valid;
            const uint64_t v = welem(ap, n, j, 1, &valid);
            const int64_t b = ex + j;
            if (valid && (v & 0xff)) atomicOr(bimg + (b >> 5), 1u << (b & 31));
          }
          return 0;
        });
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        wave_store_bits(dst, bimg, gb, room);
      }
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    // a large tile range: element by element straight to HBM (edge words of the bitmaps shared
    // with other lanes / tiles: atomics)
    for (int64_t j = 0; j < n; j++) {
      const int64_t e = gb + ex + j;
      if (e >= cap) break;
      bool valid = false;
      const uint64_t x = S.with(p, abytes, [&](auto ap) { return welem(ap, n, j, ew, &valid); });
      switch (c.width) {
        case 8: gl(reinterpret_cast<uint64_t*>(dst))[e] = x; break;
        case 4: gl(reinterpret_cast<uint32_t*>(dst))[e] = static_cast<uint32_t>(x); break;
        case 2: gl(reinterpret_cast<uint16_t*>(dst))[e] = static_cast<uint16_t>(x); break;
        case 1: gl(dst)[e] = static_cast<uint8_t>(x); break;
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

// The image img[0, bytes) -> g (any alignment) by the whole NT-thread block: the head to g's
// 16-byte boundary and the tail byte by byte, the body as 16-B non-temporal stores funnel-shifted
// out of aligned image words.
template <int NT>
__device__ __forceinline__ void store_image_nt(uint8_t* g, const uint8_t* img, int64_t bytes) {
  store_shifted<NT>(g, img, bytes);
}

// ---- encode ------------------------------------------------------------------------------------
// Column k of the row at dst (8-aligned; LDS image or HBM), variable-length values at `cursor`
// (the row's var-section position of this field, wide_encode_kernel phase 2): the slot word (0
// when null) and whether the field is null.  toRow's writes (BinaryWriter.write / writeUnaligned
// + zero pad / BinaryArrayWriter, BaseBinaryEncoderBuilder.java:138-453).
template <class Col, class D>
__device__ __forceinline__ uint64_t wide_put(const Col& c, int64_t r, D* dst, int64_t cursor,
                                             bool* nul) {
  using U64 = DstT<D, uint64_t>;
  *nul = c.validity && !bit_at_g(c.validity, r);
  if (*nul) return 0;
  switch (c.kind) {
    case kFixed: return load_fixed(c.values, r, c.width);
    case kBool: return bit_at_g(c.values, r);
    case kBytes: {
      const int32_t o0 = gl(c.offsets)[r], o1 = gl(c.offsets)[r + 1];
      const int64_t len = o1 - o0;
      put_string(reinterpret_cast<U64*>(dst + cursor), c.values + o0, len);
      return (static_cast<uint64_t>(cursor) << 32) | static_cast<uint32_t>(len);
    }
    case kDecimal: {
      const auto sv = gl(reinterpret_cast<const uint64_t*>(c.values)) + 2 * r;
      U64* d = reinterpret_cast<U64*>(dst + cursor);
      d[0] = sv[0];
      d[1] = sv[1];
      return (static_cast<uint64_t>(cursor) << 32) | 16u;
    }
    case kListFixed: {
      const int32_t o0 = gl(c.offsets)[r], o1 = gl(c.offsets)[r + 1];
      const int64_t n = o1 - o0;
      const uint8_t* vals = c.width == 0 ? c.values + (o0 >> 3) : c.values + int64_t(o0) * c.width;
      const uint8_t* vb = c.elem_validity ? c.elem_validity + (o0 >> 3) : nullptr;
      const int64_t sz = put_array(reinterpret_cast<U64*>(dst + cursor), c.width, vals, vb, o0 & 7, n);
      return (static_cast<uint64_t>(cursor) << 32) | static_cast<uint32_t>(sz);
    }
    default:
      return 0;
  }
}

// The var-section bytes field k (kind >= kBytes) takes in row r (0 when null).
template <class Col>
__device__ __forceinline__ int32_t wide_var_size(const Col& c, int64_t r) {
  if (c.validity && !bit_at_g(c.validity, r)) return 0;
  if (c.kind == kDecimal) return 16;
  const int32_t o0 = gl(c.offsets)[r], o1 = gl(c.offsets)[r + 1];
  const int64_t n = o1 - o0;
  if (c.kind == kBytes) return static_cast<int32_t>(rnd8(n));
  return static_cast<int32_t>(8 + bm_bytes(n) + rnd8(n * (c.width == 0 ? 1 : c.width)));
}

// Encode of flat schemas wider than kRegCols: rows at the offsets fury_row_measure produced, 64
// rows per tile (lane = row), the four waves taking the fields round robin (the 256-row tile
// kernel it replaces sized its tiles by a 16 KB staged-input pool: 64 rows of a 33-field schema
// on 256 threads, three quarters of them idle).  Phase 1: every variable-length field's bytes per
// row -> LDS; phase 2 (wave 0): their running sum = each field's var-section cursor in its row,
// and the rows' null bitmaps zeroed; phase 3: every field's slot, null bit (LDS atomic OR) and
// var bytes into the tile's LDS image; the image leaves as one contiguous range of 16-B stores.
// A tile whose rows do not fit the image is built row by row in HBM by wave 0.
template <int NT>
__global__ __launch_bounds__(NT) void wide_encode_kernel(VarArgs a, const int64_t* __restrict__ offs,
                                                                   uint8_t* __restrict__ rows,
                                                                   int64_t cap, uint32_t img_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t t = blockIdx.x;
  const int64_t r0 = t * kWideRows;
  const int nr = static_cast<int>(min<int64_t>(kWideRows, a.nrows - r0));
  const bool live = lane < nr;
  const int64_t r = live ? r0 + lane : r0;
  const int64_t base = gl(offs)[r0];
  const int64_t bytes = gl(offs)[r0 + nr] - base;
  const int64_t ex = live ? gl(offs)[r] - base : 0;
  const int64_t rsz = live ? gl(offs)[r + 1] - gl(offs)[r] : 0;
  const int64_t room = max<int64_t>(0, min<int64_t>(bytes, cap - base));
  int32_t* cur = reinterpret_cast<int32_t*>(wsm + img_cap);      // [var field][64]
  int v = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    if (c.kind < kBytes || c.kind > kListFixed) continue;
    if (v % (NT / 64) == wave) cur[v * kWideRows + lane] = live ? wide_var_size(c, r) : 0;
    v++;
  }
  __syncthreads();
  const bool fits = bytes + 16 <= static_cast<int64_t>(img_cap);
  const int nbw = a.bitmap_bytes >> 3;
  if (wave == 0) {
    int32_t cursor = a.fixed_size;
    for (int q = 0; q < v; q++) {
      const int32_t sz = cur[q * kWideRows + lane];
      cur[q * kWideRows + lane] = cursor;
      cursor += sz;
    }
    if (fits && live)
      for (int w = 0; w < nbw; w++) reinterpret_cast<uint64_t*>(wsm + ex)[w] = 0;
  }
  __syncthreads();
  if (fits) {
    uint8_t* row = wsm + ex;
    v = 0;
    for (int k = 0; k < a.ncols; k++) {
      CVarCol& c = vc(a, k);
      const bool var = c.kind >= kBytes && c.kind <= kListFixed;
      const int q = v;
      v += var ? 1 : 0;
      if (k % (NT / 64) != wave || !live) continue;
      bool nul;
      const uint64_t slot = wide_put(c, r, row, var ? cur[q * kWideRows + lane] : 0, &nul);
      reinterpret_cast<uint64_t*>(row + a.bitmap_bytes)[k] = slot;
      if (nul) atomicOr(reinterpret_cast<unsigned long long*>(row) + (k >> 6), 1ull << (k & 63));
    }
    __syncthreads();
    store_image_nt<NT>(rows + base, wsm, room);
    return;
  }
  if (wave != 0 || !live || ex + rsz > room) return;              // oversized tile: rows in HBM
  const auto row = gl(rows + base + ex);
  uint64_t nulls = 0;
  v = 0;
  for (int k = 0; k < a.ncols; k++) {
    CVarCol& c = vc(a, k);
    const bool var = c.kind >= kBytes && c.kind <= kListFixed;
    bool nul;
    const uint64_t slot = wide_put(c, r, row, var ? cur[v * kWideRows + lane] : 0, &nul);
    v += var ? 1 : 0;
    reinterpret_cast<__attribute__((address_space(1))) uint64_t*>(row + a.bitmap_bytes)[k] = slot;
    nulls |= static_cast<uint64_t>(nul) << (k & 63);
    if ((k & 63) == 63 || k == a.ncols - 1) {
      reinterpret_cast<__attribute__((address_space(1))) uint64_t*>(row)[k >> 6] = nulls;
      nulls = 0;
    }
  }
}

}  // namespace

int launch_encode_wide(const VarArgs& a, const int64_t* offs, uint8_t* rows, int64_t cap,
                       hipStream_t stream) {
  if (a.nrows == 0) return FURY_OK;
  int nvar = 0;
  for (int k = 0; k < a.ncols; k++) {
    const VarCol& c = a.htab ? a.htab[k] : a.col[k];
    if (c.kind >= kBytes && c.kind <= kListFixed) nvar++;
  }
  // the image holds 64 rows of up to ~600 B (three workgroups per CU); bigger tiles build in HBM
  const uint32_t img = 40 * 1024;
  const size_t lds = img + static_cast<size_t>(nvar) * kWideRows * 4;
  if (lds > 150 * 1024) return set_error(FURY_ERR_UNSUPPORTED, "wide encode: too many variable-length fields");
  const int64_t nt = (a.nrows + kWideRows - 1) / kWideRows;
  auto go = [&](auto kern, int threads) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nt)), dim3(threads), lds, stream, a, offs,
                       rows, cap, img);
  };
  const int th = wide_threads(true);
  if (th == 1024) go(wide_encode_kernel<1024>, 1024);
  else if (th == 512) go(wide_encode_kernel<512>, 512);
  else go(wide_encode_kernel<256>, 256);
  return check_hip(hipGetLastError(), "wide encode launch");
}

// LDS plan of the wide decode: the stage holds ~64 rows of the batch's estimated row size (from
// the output capacities, as dec_tile_plan) next to the four per-wave images.
namespace {
constexpr uint32_t kWideImg = 2048;
}  // namespace

namespace {
// The decode's LDS plan: the stage (~64 rows of the estimated row size) and the per-wave images.
struct WideGeom {
  int nseq = 0, th = 256;
  uint32_t stage = 0, imgs = 0;
  int64_t nt = 0;
};
WideGeom wide_geom(const VarArgs& a, double avg_row = -1);
}  // namespace

int launch_decode_wide(const VarArgs& a, const uint8_t* rows, const int64_t* offs, hipStream_t stream,
                       bool offsets_only) {
  if (a.nrows == 0) return FURY_OK;
  const WideGeom g = wide_geom(a);
  const int nseq = g.nseq;
  const uint32_t stage = g.stage, imgs = g.imgs;
  const int64_t nt = g.nt;
  const int th = g.th;
  int64_t* ws = nullptr;                   // [nseq x nt counts][total][scan scratch]
  const int64_t m = static_cast<int64_t>(nseq) * nt;
  int st = dev_alloc((m + 1 + scan_workspace(std::max<int64_t>(m, 1))) * 8, stream,
                     reinterpret_cast<void**>(&ws));
  if (st) return st;
  const size_t lds = static_cast<size_t>(stage) + imgs;
  auto go = [&](auto count, auto write, int threads) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(write),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(count),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(stage));
    if (nseq > 0) {
      hipLaunchKernelGGL(count, dim3(static_cast<unsigned>(nt)), dim3(threads), stage, stream, a,
                         rows, offs, ws, nt, stage);
      device_scan(ws, m, ws + m, ws + m + 1, stream);
    }
    hipLaunchKernelGGL(write, dim3(static_cast<unsigned>(nt)), dim3(threads), lds, stream, a, rows,
                       offs, ws, nt, stage, kWideImg, offsets_only ? 1 : 0);
  };
  if (th == 1024) go(wide_count_kernel<1024>, wide_write_kernel<1024>, 1024);
  else if (th == 512) go(wide_count_kernel<512>, wide_write_kernel<512>, 512);
  else go(wide_count_kernel<256>, wide_write_kernel<256>, 256);
  st = check_hip(hipGetLastError(), "wide decode launch");
  dev_free(ws, stream);
  return st;
}

// Plan form (fury_decode_prepare / fury_decode_execute): the count pass and the
// scan run once in the prepare, whose one host sync reads every sequence field's total (sizing the
// caller's buffers); the execute runs the write pass alone on the kept tile bases -- the rows are no
// longer counted twice (fury_row_decode_measure + fury_row_decode).
__global__ void wide_totals_kernel(const int64_t* ws, int64_t nt, int32_t nseq, int64_t* out) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q <= nseq) out[q] = ws[static_cast<int64_t>(q) * nt];      // q = nseq: the grand total
}

int wide_prepare(const VarArgs& a, const uint8_t* rows, const int64_t* offs, hipStream_t stream,
                 WidePlan* wp, std::vector<int64_t>* seq_totals) {
  // the stage is sized from the batch's average row (one 8-byte read)
  int64_t bytes = 0;
  if (a.nrows > 0) {
    int st = check_hip(hipMemcpyAsync(&bytes, offs + a.nrows, 8, hipMemcpyDeviceToHost, stream),
                       "hipMemcpyAsync batch bytes");
    if (!st) st = check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize");
    if (st) return st;
  }
  const WideGeom g = wide_geom(a, a.nrows > 0 ? static_cast<double>(bytes) / a.nrows : -1.0);
  wp->nt = g.nt;
  wp->nseq = g.nseq;
  wp->stream = stream;
  seq_totals->assign(g.nseq, 0);
  if (a.nrows == 0 || g.nseq == 0) return FURY_OK;
  const int64_t m = static_cast<int64_t>(g.nseq) * g.nt;
  int st = dev_alloc((m + 1 + scan_workspace(std::max<int64_t>(m, 1)) + g.nseq + 1) * 8, stream,
                     reinterpret_cast<void**>(&wp->ws));
  if (st) return st;
  int64_t* ws = wp->ws;
  int64_t* tot = ws + m + 1 + scan_workspace(std::max<int64_t>(m, 1));
  auto go = [&](auto count, int threads) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(count),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(g.stage));
    hipLaunchKernelGGL(count, dim3(static_cast<unsigned>(g.nt)), dim3(threads), g.stage, stream, a,
                       rows, offs, ws, g.nt, g.stage);
  };
  if (g.th == 1024) go(wide_count_kernel<1024>, 1024);
  else if (g.th == 512) go(wide_count_kernel<512>, 512);
  else go(wide_count_kernel<256>, 256);
  device_scan(ws, m, ws + m, ws + m + 1, stream);
  hipLaunchKernelGGL(wide_totals_kernel, dim3(static_cast<unsigned>((g.nseq + 256) / 256)), dim3(256),
                     0, stream, ws, g.nt, g.nseq, tot);
  if ((st = check_hip(hipGetLastError(), "wide prepare launch"))) return st;
  std::vector<int64_t> h(g.nseq + 1);
  if ((st = check_hip(hipMemcpyAsync(h.data(), tot, 8 * (g.nseq + 1), hipMemcpyDeviceToHost, stream),
                      "hipMemcpyAsync wide totals")))
    return st;
  if ((st = check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize"))) return st;
  for (int q = 0; q < g.nseq; q++) (*seq_totals)[q] = h[q + 1] - h[q];
  return FURY_OK;
}

int wide_execute(const VarArgs& a, const uint8_t* rows, const int64_t* offs, hipStream_t stream,
                 const WidePlan& wp) {
  if (a.nrows == 0) return FURY_OK;
  const WideGeom g = wide_geom(a);
  const size_t lds = static_cast<size_t>(g.stage) + g.imgs;
  auto go = [&](auto write, int threads) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(write),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(write, dim3(static_cast<unsigned>(g.nt)), dim3(threads), lds, stream, a, rows,
                       offs, wp.ws, g.nt, g.stage, kWideImg, 0);
  };
  if (g.th == 1024) go(wide_write_kernel<1024>, 1024);
  else if (g.th == 512) go(wide_write_kernel<512>, 512);
  else go(wide_write_kernel<256>, 256);
  return check_hip(hipGetLastError(), "wide execute launch");
}

void wide_free(WidePlan* wp) {
  if (!wp) return;
  dev_free(wp->ws, wp->stream);
  delete wp;
}

namespace {
// avg_row >= 0: the batch's average row bytes (the prepare, which has no output capacities to
// estimate it from)
WideGeom wide_geom(const VarArgs& a, double avg_row) {
  WideGeom g;
  int nseq = 0;
  double row = a.fixed_size;
  for (int k = 0; k < a.ncols; k++) {
    const VarCol& c = a.htab ? a.htab[k] : a.col[k];
    const double per = a.nrows > 0 && c.capacity > 0 ? static_cast<double>(c.capacity) / a.nrows : 16.0;
    if (c.kind == kBytes || c.kind == kListFixed) nseq++;
    if (c.kind == kDecimal) row += 16;
    if (c.kind == kBytes) row += per + 4;
    if (c.kind == kListFixed) row += 12 + per * (c.width == 0 ? 1 : c.width) + 4;
  }
  const uint32_t bit_cap = ((kWideImg / 8 + 4 * 16) + 15) & ~15u;
  const int th = wide_threads(false);
  const uint32_t imgs = static_cast<uint32_t>(th / 64) * (kWideImg + bit_cap);
  // the stage: the tile's estimated row bytes (+3 %), at least 1 KB, at most 96 KB (rows past it
  // are read from HBM)
  if (avg_row >= 0) row = avg_row;
  const uint32_t want = static_cast<uint32_t>(std::min<double>(row * kWideRows * 1.03 + 64, 96.0 * 1024));
  g.stage = (std::max<uint32_t>(want, 1024) + 15) & ~15u;
  g.nt = (a.nrows + kWideRows - 1) / kWideRows;
  g.nseq = nseq;
  g.th = th;
  g.imgs = imgs;
  return g;
}
}  // namespace

}  // namespace fury
