// hostpath.cpp — the host-memory batch path: columns and rows that live in host memory (a JVM's
// off-heap DirectByteBuffers, read from a socket or a file — the north-star boundary) go
// through HBM and back inside one call.  This is what the JNI glue calls with
// GetDirectBufferAddress pointers; the device entry points of capi.cpp do the work.
//
// Fixed-width schemas (Struct-100) whose buffers are all pinned run the kernel directly on the
// host memory (fixed_direct: both PCIe directions busy at once, no HBM staging).  Otherwise
// they are streamed in 64-row-aligned chunks on three HIP streams (chunk k's H2D copies, chunk
// k-1's kernel, chunk k-2's D2H copies).  Flat variable-length schemas on pinned buffers run
// their kernels on host memory too (var_encode_direct / var_decode_direct); otherwise they are
// staged whole: their row offsets are a scan over the whole batch.  Pinning (hipHostRegister) is the caller's choice
// (fury_host_register): pinned buffers DMA at the link rate, pageable ones are bounced through
// the runtime's staging buffers.
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {
namespace {

constexpr int kStages = 3;

// Stream-ordered device allocations on `stream` (pooled: keep_pool), freed on it when the arena
// goes — after the call's last use of them in stream order.
struct DeviceArena {
  hipStream_t stream;
  std::vector<void*> ptrs;
  explicit DeviceArena(hipStream_t s) : stream(s) {
    int device = 0;
    (void)hipGetDevice(&device);
    keep_pool(device);
  }
  ~DeviceArena() {
    for (void* p : ptrs) dev_free(p, stream);
  }
  int alloc(int64_t bytes, void** out) {
    *out = nullptr;
    if (bytes <= 0) bytes = 16;
    const int st = dev_alloc(bytes, stream, out);
    if (!st) ptrs.push_back(*out);
    return st;
  }
};

// The calling thread's HIP streams on `device`: created on its first host call and kept for the
// thread's lifetime (never destroyed: a thread_local destructor may run after the HIP runtime is
// gone at process exit).  Creating and destroying them per call was most of a small call's
// ~1.4 ms cost (scripts/ab_host_zc.py "api_tiny").  Every call ends with sync(), so a call
// finds its streams idle.
struct Streams {
  hipStream_t s[kStages] = {};
  int create(int device) {
    // the streams' error slots go back to the free list when the thread exits (the streams
    // themselves are idle: every call ends with sync())
    struct Pool : std::map<int, std::array<hipStream_t, kStages>> {
      ~Pool() {
        for (auto& kv : *this)
          for (hipStream_t x : kv.second) release_error_slot(x, false);
      }
    };
    thread_local Pool pool;
    auto it = pool.find(device);
    if (it == pool.end()) {
      std::array<hipStream_t, kStages> a{};
      for (auto& x : a) {
        const int st = check_hip(hipStreamCreateWithFlags(&x, hipStreamNonBlocking), "hipStreamCreate");
        if (st) {
          for (auto& y : a)
            if (y) (void)hipStreamDestroy(y);
          return st;
        }
      }
      it = pool.emplace(device, a).first;
    }
    for (int g = 0; g < kStages; g++) s[g] = it->second[g];
    return FURY_OK;
  }
  // Synchronous calls report what their kernels found (decode bounds, map counts) here.
  int sync() {
    int st = FURY_OK;
    for (auto& x : s) {
      const int e = check_hip(hipStreamSynchronize(x), "hipStreamSynchronize");
      if (!st) st = e;
    }
    for (auto& x : s) {                    // every stage stream's error slot (all are taken)
      const int e = take_device_error(x);
      if (!st) st = e;
    }
    return st;
  }
};

// Bytes of a fixed-width column's values for rows [0, n).
int64_t fixed_bytes(const FieldPlan& p, int64_t n) {
  return p.kind == kBool ? (n + 7) / 8 : n * p.width;
}
// Device bitmap buffers are written as 32-bit words (fury_row.h): pad to 4 bytes.
int64_t bitmap_alloc(int64_t n) { return ((n + 31) / 32) * 4 + 4; }

// Bytes one row occupies in a stage (row image + its column values + validity bits, rounded up).
int64_t stage_bytes_per_row(const fury_schema* s) {
  int64_t per_row = s->fixed_size;
  for (const auto& p : s->plan) per_row += p.width > 0 ? p.width : 1;
  return per_row + s->num_fields;             // validity bits, generously
}

// Rows per chunk: kTargetChunks chunks, 64-row aligned (bitmaps slice on
// 32-bit words), at most kMaxStageBytes of HBM per stage.  Measured on the MI355X box
// (scripts/ab_host.py, profiles/r01_host_path.json): the H2D and D2H copies of different
// streams did not overlap there, and every extra chunk adds one copy per column, so more chunks
// were slower (1: 42.6 GB/s, 3: 41.8, 6: 31.5, 12: 22.2 GB/s encode); the default is one chunk
// (whole batch staged), the pipeline stays for hosts whose copy engines do overlap.
constexpr int64_t kTargetChunks = 1;
constexpr int64_t kMaxStageBytes = 1ll << 30;
int64_t rows_per_chunk(const fury_schema* s, int64_t n) {
  const int64_t per_row = stage_bytes_per_row(s);
  int64_t chunks = kTargetChunks;
  int64_t c = (n + chunks - 1) / chunks;
  if (c * per_row > kMaxStageBytes) c = kMaxStageBytes / per_row;
  c = ((c + 63) / 64) * 64;
  return c < 64 ? 64 : c;
}

std::atomic<int64_t> g_host_direct{0};       // host calls run by fixed_direct

// Device address through which a kernel reaches host bytes [p, p + bytes): memory pinned by
// hipHostMalloc or hipHostRegister (fury_host_register) only — nullptr for pageable memory,
// which the GPU cannot address without XNACK.
uint8_t* device_view(const void* p, int64_t bytes) {
  if (!p || bytes <= 0) return nullptr;
  auto view = [](const uint8_t* q) -> uint8_t* {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, q) != hipSuccess) {
      (void)hipGetLastError();                  // pageable: not an error of the call
      return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return static_cast<uint8_t*>(a.devicePointer) + (q - static_cast<const uint8_t*>(a.hostPointer));
  };
  const uint8_t* b = static_cast<const uint8_t*>(p);
  uint8_t* d0 = view(b);
  uint8_t* d1 = d0 ? view(b + bytes - 1) : nullptr;   // the whole range is in one mapping
  return d1 == d0 + (bytes - 1) ? d0 : nullptr;
}

// Fixed-width schemas whose host buffers are all pinned: the encode / decode kernel reads and
// writes them directly over PCIe, with no HBM staging.  Loads of one direction and stores of
// the other are in flight together, so both directions of the link carry data at once — the
// staged copies did not overlap on the MI355X box (rows_per_chunk).  Measured Struct-100 1M rows
// (scripts/ab_host_zc.py, profiles/r02_host_direct.json): staged 58 GB/s, direct 92 GB/s
// encode / 88 GB/s decode (algorithmic column + row bytes).  The fixed kernels read their inputs
// and write value columns with exact-width accesses; decode output bitmaps (validity, BOOL
// values) are written as whole words and a host bitmap is only (n + 7) / 8 bytes, so those go to
// HBM and are copied back.  *used = false (and nothing ran) when any buffer is pageable.
int fixed_direct(const fury_schema* s, const fury_column* host, int64_t n, uint8_t* rows,
                 bool decode, int32_t device, bool* used) {
  *used = false;
  const int nf = s->num_fields;
  // the device entry points' alignment rules (16-B rows, width-aligned values) hold for the
  // staged buffers; host buffers that miss them are staged too
  auto aligned = [](const void* q, int64_t a) { return (reinterpret_cast<uintptr_t>(q) & (a - 1)) == 0; };
  uint8_t* drows = device_view(rows, n * s->fixed_size);
  if (!drows || !aligned(drows, 16)) return FURY_OK;
  std::vector<fury_column> dc(nf);
  std::vector<int64_t> bits(2 * nf, -1);               // decode: workspace offsets of bitmaps
  int64_t ws_bytes = 0;
  auto bitmap = [&](int64_t* off) {
    *off = ws_bytes;
    ws_bytes += ((bitmap_alloc(n) + 255) / 256) * 256;
  };
  for (int k = 0; k < nf; k++) {
    const FieldPlan& p = s->plan[k];
    dc[k] = fury_column{};
    if (decode && p.kind == kBool) {
      bitmap(&bits[2 * k]);
    } else {
      dc[k].values = device_view(host[k].values, fixed_bytes(p, n));
      if (!dc[k].values || (p.width > 1 && !aligned(dc[k].values, p.width))) return FURY_OK;
    }
    if (host[k].validity) {
      if (decode) {
        bitmap(&bits[2 * k + 1]);
      } else if (!(dc[k].validity = device_view(host[k].validity, (n + 7) / 8))) {
        return FURY_OK;
      }
    }
  }
  int st = check_hip(hipSetDevice(device), "hipSetDevice");
  if (st) return st;
  Streams ss;
  if ((st = ss.create(device))) return st;
  hipStream_t hs = ss.s[0];
  uint8_t* ws = nullptr;
  if (ws_bytes > 0) {
    keep_pool(device);
    if ((st = dev_alloc(ws_bytes, hs, reinterpret_cast<void**>(&ws))))
      return st;
    for (int k = 0; k < nf; k++) {
      if (bits[2 * k] >= 0) dc[k].values = ws + bits[2 * k];
      if (bits[2 * k + 1] >= 0) dc[k].validity = ws + bits[2 * k + 1];
    }
  }
  *used = true;
  g_host_direct.fetch_add(1);
  // Plain (not non-temporal) loads and stores: over PCIe the HBM-tuned kernels measured 92 / 88
  // GB/s, plain ones 95 / 89 (r02_host_direct.json sweep).
  struct DirectScope {
    DirectScope() { set_thread_host_direct(true); }
    ~DirectScope() { set_thread_host_direct(false); }
  } scope;
  st = decode ? fury_row_decode(s, drows, nullptr, n, dc.data(), hs)
              : fury_row_encode(s, dc.data(), n, nullptr, drows, hs);
  for (int k = 0; k < nf && !st; k++) {
    if (bits[2 * k] >= 0)
      (void)hipMemcpyAsync(host[k].values, dc[k].values, (n + 7) / 8, hipMemcpyDeviceToHost, hs);
    if (bits[2 * k + 1] >= 0)
      (void)hipMemcpyAsync(host[k].validity, dc[k].validity, (n + 7) / 8, hipMemcpyDeviceToHost, hs);
  }
  if (!st) st = check_hip(hipGetLastError(), "hipMemcpyAsync D2H bitmaps");
  if (ws) dev_free(ws, hs);
  const int st2 = ss.sync();
  return st ? st : st2;
}

int fixed_host(const fury_schema* s, const fury_column* host, int64_t n, uint8_t* rows, bool decode,
               int32_t device) {
  if (n == 0) return FURY_OK;
  bool used = false;
  int st = fixed_direct(s, host, n, rows, decode, device, &used);
  if (st || used) return st;
  if ((st = check_hip(hipSetDevice(device), "hipSetDevice"))) return st;
  const int64_t C = rows_per_chunk(s, n);
  const int nf = s->num_fields;
  Streams ss;
  if ((st = ss.create(device))) return st;
  // one stream-ordered workspace for all stages (pooled by the runtime across calls)
  std::vector<int64_t> col_off(nf), val_off(nf);
  int64_t stage = ((C * s->fixed_size + 255) / 256) * 256;
  for (int k = 0; k < nf; k++) {
    col_off[k] = stage;
    stage += ((fixed_bytes(s->plan[k], C) + 16 + 255) / 256) * 256;
    val_off[k] = -1;
    if (host[k].validity) {
      val_off[k] = stage;
      stage += ((bitmap_alloc(C) + 255) / 256) * 256;
    }
  }
  keep_pool(device);                          // keep the workspace pooled between calls
  uint8_t* ws = nullptr;
  if ((st = dev_alloc(stage * kStages, ss.s[0], reinterpret_cast<void**>(&ws))))
    return st;
  hipEvent_t ready;
  (void)hipEventCreateWithFlags(&ready, hipEventDisableTiming);
  (void)hipEventRecord(ready, ss.s[0]);
  for (int g = 1; g < kStages; g++) (void)hipStreamWaitEvent(ss.s[g], ready, 0);
  std::vector<std::vector<fury_column>> dcols(kStages, std::vector<fury_column>(nf));
  std::vector<void*> drows(kStages);
  for (int g = 0; g < kStages; g++) {
    uint8_t* base = ws + g * stage;
    drows[g] = base;
    for (int k = 0; k < nf; k++) {
      dcols[g][k] = fury_column{};
      dcols[g][k].values = base + col_off[k];
      if (val_off[k] >= 0) dcols[g][k].validity = base + val_off[k];
    }
  }
  for (int64_t r0 = 0, k = 0; r0 < n && !st; r0 += C, k++) {
    const int g = static_cast<int>(k % kStages);
    hipStream_t hs = ss.s[g];
    const int64_t nr = n - r0 < C ? n - r0 : C;
    uint8_t* hrows = rows + r0 * s->fixed_size;
    if (!decode) {
      for (int j = 0; j < nf; j++) {
        const FieldPlan& p = s->plan[j];
        const uint8_t* hv = static_cast<const uint8_t*>(host[j].values) +
                            (p.kind == kBool ? r0 / 8 : r0 * p.width);
        (void)hipMemcpyAsync(dcols[g][j].values, hv, fixed_bytes(p, nr), hipMemcpyHostToDevice, hs);
        if (host[j].validity)
          (void)hipMemcpyAsync(dcols[g][j].validity, host[j].validity + r0 / 8, (nr + 7) / 8,
                               hipMemcpyHostToDevice, hs);
      }
      st = fury_row_encode(s, dcols[g].data(), nr, nullptr, drows[g], hs);
      if (!st)
        st = check_hip(hipMemcpyAsync(hrows, drows[g], nr * s->fixed_size, hipMemcpyDeviceToHost,
                                      hs), "hipMemcpyAsync D2H rows");
    } else {
      (void)hipMemcpyAsync(drows[g], hrows, nr * s->fixed_size, hipMemcpyHostToDevice, hs);
      st = fury_row_decode(s, drows[g], nullptr, nr, dcols[g].data(), hs);
      for (int j = 0; j < nf && !st; j++) {
        const FieldPlan& p = s->plan[j];
        uint8_t* hv = static_cast<uint8_t*>(host[j].values) +
                      (p.kind == kBool ? r0 / 8 : r0 * p.width);
        (void)hipMemcpyAsync(hv, dcols[g][j].values, fixed_bytes(p, nr), hipMemcpyDeviceToHost, hs);
        if (host[j].validity)
          (void)hipMemcpyAsync(host[j].validity + r0 / 8, dcols[g][j].validity, (nr + 7) / 8,
                               hipMemcpyDeviceToHost, hs);
      }
      if (!st) st = check_hip(hipGetLastError(), "hipMemcpyAsync D2H columns");
    }
  }
  const int st2 = ss.sync();                  // every stage done before the workspace goes
  dev_free(ws, ss.s[0]);
  const int st3 = check_hip(hipStreamSynchronize(ss.s[0]), "hipStreamSynchronize");
  (void)hipEventDestroy(ready);
  return st ? st : st2 ? st2 : st3;
}

// ---- variable-length schemas: stage the whole batch ----------------------------------------
int host_offset(const int32_t* offs, int64_t i) { return offs ? offs[i] : 0; }

// Copies a host column tree (Arrow layout of fury_row.h) of `n` entries to the device.
int stage_column(const OwnedField& f, const fury_column& h, int64_t n, DeviceArena& arena,
                 std::deque<std::vector<fury_column>>& kids, fury_column* d, hipStream_t hs) {
  *d = fury_column{};
  auto copy = [&](const void* src, int64_t bytes, void** dst) {
    int st = arena.alloc(bytes + 16, dst);
    if (!st && bytes > 0 && src)
      st = check_hip(hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, hs), "H2D column");
    return st;
  };
  int st = FURY_OK;
  if (h.validity) {
    void* v = nullptr;
    if ((st = copy(h.validity, (n + 7) / 8, &v))) return st;
    d->validity = static_cast<uint8_t*>(v);
  }
  const int t = f.type_id;
  if (t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY || t == FURY_TYPE_LIST || t == FURY_TYPE_MAP) {
    if (n > 0 && !h.offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, f.name + ": offsets is null");
    void* o = nullptr;
    if ((st = copy(h.offsets, n > 0 ? (n + 1) * 4 : 0, &o))) return st;
    d->offsets = static_cast<int32_t*>(o);
  }
  const int64_t m = n > 0 ? host_offset(h.offsets, n) : 0;
  switch (t) {
    case FURY_TYPE_STRING: case FURY_TYPE_BINARY:
      return copy(h.values, m, &d->values);
    case FURY_TYPE_LIST: case FURY_TYPE_MAP: case FURY_TYPE_STRUCT: {
      const int64_t len = t == FURY_TYPE_STRUCT ? n : m;
      if (!h.child && len > 0) return set_error(FURY_ERR_INVALID_ARGUMENT, f.name + ": child is null");
      kids.emplace_back(f.children.size());
      std::vector<fury_column>& kc = kids.back();
      for (size_t i = 0; i < f.children.size(); i++) {
        static const fury_column empty{};
        if ((st = stage_column(f.children[i], h.child ? h.child[i] : empty, len, arena, kids,
                               &kc[i], hs)))
          return st;
      }
      d->child = kc.data();
      return FURY_OK;
    }
    case FURY_TYPE_BOOL:
      return copy(h.values, (n + 7) / 8, &d->values);
    default:
      return copy(h.values, n * type_width_of(t), &d->values);
  }
}

// ---- variable-length flat schemas on pinned buffers: kernels on host memory -----------------
// As fixed_direct: when every host buffer is pinned (fury_host_alloc / fury_host_register) and
// meets the device entry points' alignment, the measure / encode / decode kernels read and write
// host memory over PCIe, both link directions at once, instead of staging the batch through HBM.
// Every kernel read of an input is either exact or an aligned 8- or 16-byte word holding at least
// one byte of the buffer -- inside the same page, so inside the pinned mapping.  Outputs written
// as whole bitmap words or with atomics (validity, BOOL values, list element bitmaps) go to HBM
// and are copied back; Arrow offsets, payloads, element values and rows are written exactly.
bool aligned_to(const void* q, int64_t a) { return (reinterpret_cast<uintptr_t>(q) & (a - 1)) == 0; }

// Device views of a flat variable-length schema's host input columns (encode); false when a
// buffer is pageable or misaligned (the call is then staged).
bool view_inputs(const fury_schema* s, const fury_column* host, int64_t n,
                 std::vector<fury_column>& d, std::vector<fury_column>& dchild) {
  const int nf = s->num_fields;
  d.assign(nf, fury_column{});
  dchild.assign(nf, fury_column{});
  auto need = [](const void* p, int64_t bytes, uint8_t** out) {
    *out = nullptr;
    if (!p) return true;
    if (bytes <= 0) bytes = 1;
    *out = device_view(p, bytes);
    return *out != nullptr;
  };
  for (int k = 0; k < nf; k++) {
    const FieldPlan& p = s->plan[k];
    const fury_column& h = host[k];
    fury_column& c = d[k];
    if (!need(h.validity, (n + 7) / 8, &c.validity)) return false;
    uint8_t* v = nullptr;
    switch (p.kind) {
      case kFixed:
        if (!need(h.values, n * p.width, &v) || !aligned_to(v, p.width)) return false;
        c.values = v;
        break;
      case kBool:
        if (!need(h.values, (n + 7) / 8, &v)) return false;
        c.values = v;
        break;
      case kDecimal:
        if (!need(h.values, 16 * n, &v) || !aligned_to(v, 8)) return false;
        c.values = v;
        break;
      case kBytes:
      case kListFixed: {
        if (!h.offsets) return false;
        if (!need(h.offsets, (n + 1) * 4, &v) || !aligned_to(v, 4)) return false;
        c.offsets = reinterpret_cast<int32_t*>(v);
        const int64_t m = h.offsets[n];
        if (p.kind == kBytes) {
          if (!need(h.values, m, &v)) return false;
          c.values = v;
          break;
        }
        const fury_column* hc = h.child;
        if (!hc) return false;
        fury_column& e = dchild[k];
        const bool bits = p.elem_type == FURY_TYPE_BOOL;
        if (!need(hc->values, bits ? (m + 7) / 8 : m * p.elem_width, &v) ||
            (!bits && !aligned_to(v, p.elem_width)))
          return false;
        e.values = v;
        if (!need(hc->validity, (m + 7) / 8, &e.validity)) return false;
        c.child = &e;
        break;
      }
      default:
        return false;
    }
  }
  return true;
}

// Device views of a generic (nested / collection / very wide) schema's host input column tree,
// breadth-first like the schema nodes (a node's children contiguous: child = &d[first_child]);
// every node's entry count follows from its parent's (STRUCT: the same; LIST / MAP: the parent's
// offsets[m], read on the host).  False when a buffer is pageable, misaligned or missing (the call
// is then staged, which reports argument errors).
bool view_gen_inputs(const fury_schema* s, const fury_column* host, int64_t n,
                     std::vector<fury_column>& d) {
  const int nn = static_cast<int>(s->nodes.size());
  std::vector<const fury_column*> hc(nn, nullptr);
  std::vector<int64_t> m(nn, 0);
  d.assign(nn, fury_column{});
  for (int k = 0; k < s->num_fields; k++) {
    hc[k] = &host[k];
    m[k] = n;
  }
  for (int i = 0; i < nn; i++) {
    const GenTpl& t = s->nodes[i];
    if (!hc[i]) return false;
    const fury_column& h = *hc[i];
    fury_column& c = d[i];
    const int64_t mi = m[i];
    uint8_t* v = nullptr;
    if (h.validity) {
      if (!(v = device_view(h.validity, (mi + 7) / 8 > 0 ? (mi + 7) / 8 : 1))) return false;
      c.validity = v;
    }
    const int t_id = t.type_id;
    const bool var = t_id == FURY_TYPE_STRING || t_id == FURY_TYPE_BINARY ||
                     t_id == FURY_TYPE_LIST || t_id == FURY_TYPE_MAP;
    int64_t end = 0;                                    // offsets[m]: payload bytes / elements
    if (var) {
      if (!h.offsets) return false;
      if (!(v = device_view(h.offsets, (mi + 1) * 4)) || !aligned_to(v, 4)) return false;
      c.offsets = reinterpret_cast<int32_t*>(v);
      end = h.offsets[mi];
      if (end < 0) return false;
    }
    const int w = type_width_of(t_id);
    if (t_id == FURY_TYPE_BOOL) {
      if (h.values && !(c.values = device_view(h.values, std::max<int64_t>((mi + 7) / 8, 1)))) return false;
    } else if (w > 0) {
      if (mi > 0 && (!(v = device_view(h.values, mi * w)) || !aligned_to(v, w))) return false;
      c.values = v;
    } else if (t_id == FURY_TYPE_DECIMAL) {
      if (mi > 0 && (!(v = device_view(h.values, 16 * mi)) || !aligned_to(v, 8))) return false;
      c.values = v;
    } else if (t_id == FURY_TYPE_STRING || t_id == FURY_TYPE_BINARY) {
      if (end > 0 && !(c.values = device_view(h.values, end))) return false;
    }
    if (t.num_children > 0) {
      if (!h.child) return false;
      const int64_t cm = t_id == FURY_TYPE_STRUCT ? mi : end;
      for (int j = 0; j < t.num_children; j++) {
        hc[t.first_child + j] = &h.child[j];
        m[t.first_child + j] = cm;
      }
      c.child = &d[t.first_child];
    }
  }
  return true;
}

int var_encode_direct(const fury_schema* s, const fury_column* host, int64_t n, uint8_t* rows,
                      int64_t cap, int64_t* row_offsets, int64_t* row_bytes, int32_t device,
                      bool* used) {
  *used = false;
  if (n == 0 || cap <= 0) return FURY_OK;
  std::vector<fury_column> d, dchild;
  if (s->generic ? !view_gen_inputs(s, host, n, d) : !view_inputs(s, host, n, d, dchild))
    return FURY_OK;
  uint8_t* drows = device_view(rows, cap);
  if (!drows || !aligned_to(drows, 16) || !device_view(row_offsets, (n + 1) * 8)) return FURY_OK;
  int st = check_hip(hipSetDevice(device), "hipSetDevice");
  if (st) return st;
  Streams ss;
  if ((st = ss.create(device))) return st;
  hipStream_t hs = ss.s[0];
  DeviceArena arena(hs);
  void* doffs = nullptr;
  if ((st = arena.alloc((n + 1) * 8, &doffs))) return st;
  int64_t* dof = static_cast<int64_t*>(doffs);
  *used = true;
  g_host_direct.fetch_add(1);
  // the row offsets are a scan: measured into HBM (its passes re-read them), copied out once
  if ((st = fury_row_measure(s, d.data(), n, dof, hs))) return st;
  int64_t total = 0;
  if ((st = check_hip(hipMemcpyAsync(&total, dof + n, 8, hipMemcpyDeviceToHost, hs), "D2H total")))
    return st;
  if ((st = ss.sync())) return st;
  *row_bytes = total;
  if (total > cap)
    return set_error(FURY_ERR_CAPACITY, "rows need " + std::to_string(total) +
                                            " bytes, capacity is " + std::to_string(cap));
  if ((st = fury_row_encode(s, d.data(), n, dof, drows, hs))) return st;
  (void)hipMemcpyAsync(row_offsets, dof, (n + 1) * 8, hipMemcpyDeviceToHost, hs);
  return ss.sync();
}

// Host rows -> host columns with the decode kernel on host memory: payloads and offsets are
// written straight into the host buffers, bounded by their capacities (no sizing pass over the
// rows: the kernel never writes past a capacity and offsets[n] holds what a column needed, checked
// after the kernel -- FURY_ERR_CAPACITY when short, as the staged path reports).
int var_decode_direct(const fury_schema* s, const uint8_t* rows, const int64_t* row_offsets,
                      int64_t n, fury_column* host, int32_t device, bool* used) {
  *used = false;
  if (s->generic || n == 0) return FURY_OK;
  const int64_t total = row_offsets[n];
  const uint8_t* drows = total > 0 ? device_view(rows, total) : nullptr;
  const uint8_t* doff = device_view(row_offsets, (n + 1) * 8);
  if (!drows || !doff || !aligned_to(drows, 16) || !aligned_to(doff, 8)) return FURY_OK;
  const int nf = s->num_fields;
  std::vector<fury_column> d(nf, fury_column{}), dchild(nf, fury_column{});
  // HBM bitmaps: (host destination, device buffer, bits) -- copied back after the kernel
  struct Bits { uint8_t* host; int64_t off; int64_t bits; int64_t cap_bits; int kind; int k; };
  std::vector<Bits> bits;
  int64_t ws_bytes = 0;
  auto bitmap = [&](uint8_t* h, int64_t nb, int kind, int k) {
    bits.push_back(Bits{h, ws_bytes, nb, nb, kind, k});
    ws_bytes += ((bitmap_alloc(nb) + 255) / 256) * 256;
  };
  for (int k = 0; k < nf; k++) {
    const FieldPlan& p = s->plan[k];
    fury_column& h = host[k];
    fury_column& c = d[k];
    if (h.validity) bitmap(h.validity, n, 0, k);
    uint8_t* v = nullptr;
    switch (p.kind) {
      case kFixed:
        if (!(v = device_view(h.values, n * p.width)) || !aligned_to(v, p.width)) return FURY_OK;
        c.values = v;
        break;
      case kBool:
        bitmap(static_cast<uint8_t*>(h.values), n, 1, k);
        break;
      case kDecimal:
        if (!(v = device_view(h.values, 16 * n)) || !aligned_to(v, 8)) return FURY_OK;
        c.values = v;
        break;
      case kBytes:
      case kListFixed: {
        if (!h.offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, "output offsets is null");
        if (!(v = device_view(h.offsets, (n + 1) * 4)) || !aligned_to(v, 4)) return FURY_OK;
        c.offsets = reinterpret_cast<int32_t*>(v);
        if (p.kind == kBytes) {
          if (h.capacity > 0 && !(c.values = device_view(h.values, h.capacity))) return FURY_OK;
          c.capacity = c.values ? h.capacity : 0;
          break;
        }
        fury_column* hc = h.child;
        if (!hc) return set_error(FURY_ERR_INVALID_ARGUMENT, "output element column is null");
        fury_column& e = dchild[k];
        const bool bool_elems = p.elem_type == FURY_TYPE_BOOL;
        const int64_t cap_elems = bool_elems ? hc->capacity * 8 : hc->capacity / p.elem_width;
        if (bool_elems) {
          bitmap(static_cast<uint8_t*>(hc->values), cap_elems, 2, k);
        } else if (hc->capacity > 0) {
          if (!(e.values = device_view(hc->values, hc->capacity)) || !aligned_to(e.values, p.elem_width))
            return FURY_OK;
        }
        e.capacity = hc->capacity;
        if (hc->validity) bitmap(hc->validity, cap_elems, 3, k);
        c.child = &e;
        break;
      }
      default:
        return FURY_OK;
    }
  }
  int st = check_hip(hipSetDevice(device), "hipSetDevice");
  if (st) return st;
  Streams ss;
  if ((st = ss.create(device))) return st;
  hipStream_t hs = ss.s[0];
  DeviceArena arena(hs);
  uint8_t* ws = nullptr;
  if (ws_bytes > 0) {
    void* w = nullptr;
    if ((st = arena.alloc(ws_bytes, &w))) return st;
    ws = static_cast<uint8_t*>(w);
    if ((st = check_hip(hipMemsetAsync(ws, 0, ws_bytes, hs), "hipMemsetAsync bitmaps"))) return st;
  }
  for (const Bits& b : bits) {
    uint8_t* dv = ws + b.off;
    if (b.kind == 0) d[b.k].validity = dv;
    else if (b.kind == 1) d[b.k].values = dv;
    else if (b.kind == 2) dchild[b.k].values = dv;
    else dchild[b.k].validity = dv;
  }
  *used = true;
  g_host_direct.fetch_add(1);
  if ((st = fury_row_decode(s, drows, const_cast<int64_t*>(reinterpret_cast<const int64_t*>(doff)),
                            n, d.data(), hs)))
    return st;
  if ((st = ss.sync())) return st;
  // what each variable-length column needed (host offsets, now written)
  for (int k = 0; k < nf; k++) {
    const FieldPlan& p = s->plan[k];
    if (p.kind != kBytes && p.kind != kListFixed) continue;
    const int64_t m = host[k].offsets[n];
    const int64_t bytes = p.kind == kBytes ? m
                        : p.elem_type == FURY_TYPE_BOOL ? (m + 7) / 8 : m * p.elem_width;
    const int64_t have = p.kind == kBytes ? host[k].capacity : host[k].child->capacity;
    if (bytes > have)
      return set_error(FURY_ERR_CAPACITY, "column " + s->fields[k].name + " needs " +
                                              std::to_string(bytes) +
                                              (p.kind == kBytes ? " payload bytes" : " element bytes"));
  }
  for (const Bits& b : bits) {
    int64_t nb = b.bits;
    if (b.kind >= 2) nb = host[b.k].offsets[n];       // element bitmaps: the elements decoded
    if (nb > 0)
      (void)hipMemcpyAsync(b.host, ws + b.off, (nb + 7) / 8, hipMemcpyDeviceToHost, hs);
  }
  if ((st = check_hip(hipGetLastError(), "hipMemcpyAsync D2H bitmaps"))) return st;
  return ss.sync();
}

int var_encode_host(const fury_schema* s, const fury_column* host, int64_t n, uint8_t* rows,
                    int64_t cap, int64_t* row_offsets, int64_t* row_bytes, int32_t device) {
  int st = check_hip(hipSetDevice(device), "hipSetDevice");
  if (st) return st;
  {
    bool used = false;
    st = var_encode_direct(s, host, n, rows, cap, row_offsets, row_bytes, device, &used);
    if (st || used) return st;
  }
  Streams ss;
  if ((st = ss.create(device))) return st;
  hipStream_t hs = ss.s[0];
  DeviceArena arena(hs);
  std::deque<std::vector<fury_column>> kids;     // stable addresses: children point into it
  std::vector<fury_column> dcols(s->num_fields);
  for (int k = 0; k < s->num_fields; k++)
    if ((st = stage_column(s->fields[k], host[k], n, arena, kids, &dcols[k], hs))) return st;
  void* doffs = nullptr;
  if ((st = arena.alloc((n + 1) * 8, &doffs))) return st;
  int64_t* dof = static_cast<int64_t*>(doffs);
  if ((st = fury_row_measure(s, dcols.data(), n, dof, hs))) return st;
  int64_t total = 0;
  if ((st = check_hip(hipMemcpyAsync(&total, dof + n, 8, hipMemcpyDeviceToHost, hs), "D2H total")))
    return st;
  if ((st = ss.sync())) return st;
  *row_bytes = total;
  if (total > cap)
    return set_error(FURY_ERR_CAPACITY, "rows need " + std::to_string(total) +
                                            " bytes, capacity is " + std::to_string(cap));
  void* drows = nullptr;
  if ((st = arena.alloc(total, &drows))) return st;
  if ((st = fury_row_encode(s, dcols.data(), n, dof, drows, hs))) return st;
  (void)hipMemcpyAsync(rows, drows, total, hipMemcpyDeviceToHost, hs);
  (void)hipMemcpyAsync(row_offsets, dof, (n + 1) * 8, hipMemcpyDeviceToHost, hs);
  return ss.sync();
}

// Flat variable-length schemas: size the outputs on the device (decode measure), check them
// against the host buffers' capacities, decode, copy back.
int var_decode_host(const fury_schema* s, const uint8_t* rows, const int64_t* row_offsets,
                    int64_t n, fury_column* host, int32_t device) {
  if (s->generic)
    return set_error(FURY_ERR_UNSUPPORTED,
                     "host-memory decode of a nested schema: its output sizes depend on the data; "
                     "use fury_decode_host_prepare / fury_decode_host_execute");
  {
    bool used = false;
    const int st = var_decode_direct(s, rows, row_offsets, n, host, device, &used);
    if (st || used) return st;
  }
  int st = check_hip(hipSetDevice(device), "hipSetDevice");
  if (st) return st;
  Streams ss;
  if ((st = ss.create(device))) return st;
  hipStream_t hs = ss.s[0];
  DeviceArena arena(hs);
  const int64_t total = row_offsets[n];
  void *drows = nullptr, *doffs = nullptr;
  if ((st = arena.alloc(total, &drows)) || (st = arena.alloc((n + 1) * 8, &doffs))) return st;
  (void)hipMemcpyAsync(drows, rows, total, hipMemcpyHostToDevice, hs);
  (void)hipMemcpyAsync(doffs, row_offsets, (n + 1) * 8, hipMemcpyHostToDevice, hs);
  const int nf = s->num_fields;
  std::vector<fury_column> d(nf);
  std::vector<fury_column> dchild(nf);
  for (int k = 0; k < nf; k++) {
    const FieldPlan& p = s->plan[k];
    fury_column& c = d[k];
    c = fury_column{};
    void* v = nullptr;
    if (host[k].validity) {
      if ((st = arena.alloc(bitmap_alloc(n), &v))) return st;
      c.validity = static_cast<uint8_t*>(v);
    }
    if (p.kind == kBytes || p.kind == kListFixed) {
      if (!host[k].offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, "output offsets is null");
      if ((st = arena.alloc((n + 1) * 4, &v))) return st;
      c.offsets = static_cast<int32_t*>(v);
      if (p.kind == kListFixed) {           // element column, sized after the measure
        dchild[k] = fury_column{};
        c.child = &dchild[k];
      }
    } else {
      const int64_t bytes = p.kind == kDecimal ? n * 16 : p.kind == kBool ? bitmap_alloc(n)
                                                                          : n * p.width;
      if ((st = arena.alloc(bytes, &c.values))) return st;
    }
  }
  if ((st = fury_row_decode_measure(s, drows, static_cast<int64_t*>(doffs), n, d.data(), hs)))
    return st;
  std::vector<int32_t> need(nf, 0);
  for (int k = 0; k < nf; k++)
    if (d[k].offsets)
      (void)hipMemcpyAsync(&need[k], d[k].offsets + n, 4, hipMemcpyDeviceToHost, hs);
  if ((st = ss.sync())) return st;
  for (int k = 0; k < nf; k++) {
    const FieldPlan& p = s->plan[k];
    if (!d[k].offsets) continue;
    if (p.kind == kBytes) {
      if (host[k].capacity < need[k])
        return set_error(FURY_ERR_CAPACITY, "column " + s->fields[k].name + " needs " +
                                                std::to_string(need[k]) + " payload bytes");
      if ((st = arena.alloc(need[k], &d[k].values))) return st;
      d[k].capacity = need[k];
    } else {                                  // LIST of fixed-width elements
      const int64_t m = need[k];
      const int64_t eb = p.elem_type == FURY_TYPE_BOOL ? (m + 7) / 8 : m * type_width_of(p.elem_type);
      fury_column& e = dchild[k];
      e = fury_column{};
      const fury_column* he = host[k].child;
      if (!he || he->capacity < eb)
        return set_error(FURY_ERR_CAPACITY, "column " + s->fields[k].name + " needs " +
                                                std::to_string(eb) + " element bytes");
      if ((st = arena.alloc(eb + 8, &e.values))) return st;
      e.capacity = eb;
      if (he->validity) {
        void* v = nullptr;
        if ((st = arena.alloc(bitmap_alloc(m), &v))) return st;
        (void)hipMemsetAsync(v, 0, bitmap_alloc(m), hs);
        e.validity = static_cast<uint8_t*>(v);
      }
      d[k].child = &e;
    }
  }
  if ((st = fury_row_decode(s, drows, static_cast<int64_t*>(doffs), n, d.data(), hs))) return st;
  for (int k = 0; k < nf; k++) {
    const FieldPlan& p = s->plan[k];
    if (host[k].validity)
      (void)hipMemcpyAsync(host[k].validity, d[k].validity, (n + 7) / 8, hipMemcpyDeviceToHost, hs);
    if (d[k].offsets) {
      (void)hipMemcpyAsync(host[k].offsets, d[k].offsets, (n + 1) * 4, hipMemcpyDeviceToHost, hs);
      if (p.kind == kBytes) {
        (void)hipMemcpyAsync(host[k].values, d[k].values, need[k], hipMemcpyDeviceToHost, hs);
      } else {
        const int64_t m = need[k];
        const int64_t eb =
            p.elem_type == FURY_TYPE_BOOL ? (m + 7) / 8 : m * type_width_of(p.elem_type);
        (void)hipMemcpyAsync(host[k].child->values, dchild[k].values, eb, hipMemcpyDeviceToHost, hs);
        if (host[k].child->validity)
          (void)hipMemcpyAsync(host[k].child->validity, dchild[k].validity, (m + 7) / 8,
                               hipMemcpyDeviceToHost, hs);
      }
    } else {
      const int64_t bytes = p.kind == kDecimal ? n * 16 : p.kind == kBool ? (n + 7) / 8 : n * p.width;
      (void)hipMemcpyAsync(host[k].values, d[k].values, bytes, hipMemcpyDeviceToHost, hs);
    }
  }
  return ss.sync();
}

// Bytes of node buffers with m entries / b payload bytes (fury_row.h two-step decode contract).
int64_t node_values_bytes(int32_t t, int64_t m, int64_t b) {
  if (t == FURY_TYPE_BOOL) return (m + 7) / 8;
  if (t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY) return b;
  if (t == FURY_TYPE_DECIMAL) return 16 * m;
  const int w = type_width_of(t);
  return w > 0 ? m * w : 0;
}
bool node_has_offsets(int32_t t) {
  return t == FURY_TYPE_STRING || t == FURY_TYPE_BINARY || t == FURY_TYPE_LIST ||
         t == FURY_TYPE_MAP;
}

}  // namespace

int64_t host_direct_count() { return g_host_direct.load(); }
static std::atomic<int> g_host_decode_inplace{0};
void set_host_decode_inplace(int v) { g_host_decode_inplace.store(v); }
int host_decode_inplace() { return g_host_decode_inplace.load(); }

// The stream-ordered pool of `device` keeps freed workspace memory instead of returning it at
// every synchronisation (the default release threshold 0 re-mapped ~1.7 GB per call).  Once per
// device, thread-safe.
void keep_pool(int device) {
  static std::mutex mu;
  static std::set<int> done;
  std::lock_guard<std::mutex> lock(mu);
  if (!done.insert(device).second) return;
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
    uint64_t keep = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
  }
}

}  // namespace fury

using namespace fury;

extern "C" {

int fury_decode_host_prepare(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                             int64_t nrows, int64_t* node_entries, int64_t* node_bytes,
                             fury_decode_plan** plan, int32_t device) {
  if (!s || !plan) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_decode_host_prepare: null argument");
  *plan = nullptr;
  if (nrows < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "nrows < 0");
  if (nrows > 0 && (!rows || (!row_offsets && !s->is_fixed)))
    return set_error(FURY_ERR_INVALID_ARGUMENT, "rows / row_offsets is null");
  if (!s->device_ok) return set_error(FURY_ERR_UNSUPPORTED, "no device kernel for " + s->device_reason);
  int st = check_hip(hipSetDevice(device), "hipSetDevice");
  if (st) return st;
  hipStream_t hs = nullptr;
  if ((st = check_hip(hipStreamCreateWithFlags(&hs, hipStreamNonBlocking), "hipStreamCreate")))
    return st;
  const int64_t total = nrows == 0 ? 0 : s->is_fixed && !row_offsets ? nrows * s->fixed_size
                                                                      : row_offsets[nrows];
  // The rows are staged in HBM even when pinned: the decode walks read them twice (prepare and
  // execute) in dependent chains, which over PCIe ran at 7 GB/s (1M nested rows, kernels on the
  // pinned rows) against one DMA copy here; the execute writes its outputs in place instead.
  // stage the rows and their offsets (fixed-width rows: offsets i * fixed_size) in HBM
  uint8_t* d = nullptr;
  const int64_t rb = (total + 255) & ~int64_t(255);
  keep_pool(device);
  st = dev_alloc(rb + (nrows + 1) * 8 + 16, hs, reinterpret_cast<void**>(&d));
  if (st) {
    release_error_slot(hs);
    (void)hipStreamDestroy(hs);
    return st;
  }
  int64_t* doffs = reinterpret_cast<int64_t*>(d + rb);
  if (total > 0) (void)hipMemcpyAsync(d, rows, total, hipMemcpyHostToDevice, hs);
  if (nrows > 0) {
    if (row_offsets) {
      (void)hipMemcpyAsync(doffs, row_offsets, (nrows + 1) * 8, hipMemcpyHostToDevice, hs);
    } else {
      std::vector<int64_t> o(nrows + 1);
      for (int64_t i = 0; i <= nrows; i++) o[i] = i * s->fixed_size;
      (void)hipMemcpyAsync(doffs, o.data(), (nrows + 1) * 8, hipMemcpyHostToDevice, hs);
      if ((st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize"))) {
        dev_free(d, hs);
        release_error_slot(hs);
        (void)hipStreamDestroy(hs);
        return st;
      }
    }
  }
  fury_decode_plan* p = nullptr;
  st = fury_decode_prepare(s, d, doffs, nrows, node_entries, node_bytes, &p, hs);
  if (st) {
    dev_free(d, hs);
    release_error_slot(hs);
    (void)hipStreamDestroy(hs);
    return st;
  }
  p->owned = d;
  p->owned_stream = hs;
  p->device = device;
  *plan = p;
  return FURY_OK;
}

int fury_decode_host_execute(fury_decode_plan* p, fury_column* host) {
  if (!p || !p->owned_stream)
    return set_error(FURY_ERR_INVALID_ARGUMENT,
                     "fury_decode_host_execute: needs a plan from fury_decode_host_prepare");
  const fury_schema* s = p->schema;
  if (s->num_fields > 0 && !host) return set_error(FURY_ERR_INVALID_ARGUMENT, "columns is null");
  int st = check_hip(hipSetDevice(p->device), "hipSetDevice");
  if (st) return st;
  hipStream_t hs = static_cast<hipStream_t>(p->owned_stream);
  const int nn = static_cast<int>(s->nodes.size());
  // the host column tree in node (breadth-first) order
  std::vector<const fury_column*> hc(nn, nullptr);
  for (int k = 0; k < s->num_fields; k++) hc[k] = &host[k];
  for (int i = 0; i < nn; i++) {
    const GenTpl& t = s->nodes[i];
    if (!hc[i]) return set_error(FURY_ERR_INVALID_ARGUMENT, "node " + std::to_string(i) + ": missing column");
    if (t.num_children > 0) {
      if (!hc[i]->child) return set_error(FURY_ERR_INVALID_ARGUMENT, "node " + std::to_string(i) + ": child columns missing");
      for (int j = 0; j < t.num_children; j++) hc[t.first_child + j] = &hc[i]->child[j];
    }
  }
  DeviceArena arena(hs);
  std::vector<fury_column> dc(nn);
  // Tuning "host_decode_inplace": outputs the kernels write exactly (values, offsets, payloads)
  // go straight into pinned host buffers (bitmaps through HBM + a copy).  Off by default: the
  // decode's scattered 4-8 byte stores over PCIe ran at 27.5 GB/s end to end against 40.4 GB/s for
  // HBM outputs + copies (1M nested rows, scripts/ab_host_nested.py).
  std::vector<uint8_t> copy_off(nn, 1), copy_val(nn, 1);
  const bool inplace = host_decode_inplace();
  bool all_direct = inplace;
  for (int i = 0; i < nn; i++) {
    const GenTpl& t = s->nodes[i];
    const fury_column& h = *hc[i];
    const int64_t m = p->totals[2 * i], b = p->totals[2 * i + 1];
    fury_column& d = dc[i];
    d = fury_column{};
    void* v = nullptr;
    if (h.validity) {
      if ((st = arena.alloc(bitmap_alloc(m), &v))) return st;
      (void)hipMemsetAsync(v, 0, bitmap_alloc(m), hs);
      d.validity = static_cast<uint8_t*>(v);
    }
    if (node_has_offsets(t.type_id)) {
      if (!h.offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, "node " + std::to_string(i) + ": output offsets is null");
      uint8_t* view = inplace ? device_view(h.offsets, (m + 1) * 4) : nullptr;
      if (view && aligned_to(view, 4)) {
        d.offsets = reinterpret_cast<int32_t*>(view);
        copy_off[i] = 0;
      } else {
        all_direct = false;
        if ((st = arena.alloc((m + 1) * 4, &v))) return st;
        d.offsets = static_cast<int32_t*>(v);
      }
    }
    const int64_t vb = node_values_bytes(t.type_id, m, b);
    if (t.type_id != FURY_TYPE_LIST && t.type_id != FURY_TYPE_MAP && t.type_id != FURY_TYPE_STRUCT) {
      if (!h.values && vb > 0)
        return set_error(FURY_ERR_INVALID_ARGUMENT, "node " + std::to_string(i) + ": output values is null");
      if ((t.type_id == FURY_TYPE_STRING || t.type_id == FURY_TYPE_BINARY) && h.capacity < vb)
        return set_error(FURY_ERR_CAPACITY, "node " + std::to_string(i) + " needs " +
                                                std::to_string(vb) + " payload bytes");
      const int w = type_width_of(t.type_id);
      const int al = t.type_id == FURY_TYPE_DECIMAL ? 8 : w > 0 ? w : 1;
      uint8_t* view = inplace && t.type_id != FURY_TYPE_BOOL && vb > 0 ? device_view(h.values, vb) : nullptr;
      if (view && aligned_to(view, al)) {
        d.values = view;
        copy_val[i] = 0;
      } else {
        if (t.type_id != FURY_TYPE_BOOL && vb > 0) all_direct = false;
        const int64_t alloc = t.type_id == FURY_TYPE_BOOL ? bitmap_alloc(m) : vb + 16;
        if ((st = arena.alloc(alloc, &v))) return st;
        if (t.type_id == FURY_TYPE_BOOL) (void)hipMemsetAsync(v, 0, alloc, hs);
        d.values = v;
      }
      d.capacity = vb;
    }
    if (t.num_children > 0) d.child = &dc[t.first_child];
  }
  if ((st = fury_decode_execute(p, dc.data(), 0, hs))) return st;
  for (int i = 0; i < nn; i++) {
    const GenTpl& t = s->nodes[i];
    const fury_column& h = *hc[i];
    const fury_column& d = dc[i];
    const int64_t m = p->totals[2 * i], b = p->totals[2 * i + 1];
    if (h.validity && m > 0)
      (void)hipMemcpyAsync(h.validity, d.validity, (m + 7) / 8, hipMemcpyDeviceToHost, hs);
    if (d.offsets && copy_off[i])
      (void)hipMemcpyAsync(h.offsets, d.offsets, (m + 1) * 4, hipMemcpyDeviceToHost, hs);
    const int64_t vb = node_values_bytes(t.type_id, m, b);
    if (d.values && vb > 0 && copy_val[i])
      (void)hipMemcpyAsync(h.values, d.values, vb, hipMemcpyDeviceToHost, hs);
  }
  if (all_direct) g_host_direct.fetch_add(1);
  st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize");
  return st ? st : take_device_error(hs);
}

int fury_host_alloc(int64_t bytes, void** out) {
  if (!out || bytes <= 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_host_alloc: empty range");
  *out = nullptr;
  return check_hip(hipHostMalloc(out, static_cast<size_t>(bytes), hipHostMallocDefault),
                   "hipHostMalloc");
}

int fury_host_free(void* p) {
  if (!p) return FURY_OK;
  return check_hip(hipHostFree(p), "hipHostFree");
}

int fury_host_register(void* p, int64_t bytes) {
  if (!p || bytes <= 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_host_register: empty range");
  return check_hip(hipHostRegister(p, static_cast<size_t>(bytes), hipHostRegisterDefault),
                   "hipHostRegister");
}

int fury_host_unregister(void* p) {
  if (!p) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_host_unregister: null");
  return check_hip(hipHostUnregister(p), "hipHostUnregister");
}

int fury_row_encode_host(const fury_schema* s, const fury_column* columns, int64_t nrows,
                         void* rows, int64_t rows_capacity, int64_t* row_offsets,
                         int64_t* row_bytes, int32_t device) {
  if (!s || !row_bytes) return set_error(FURY_ERR_INVALID_ARGUMENT, "schema/row_bytes is null");
  if (nrows < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "nrows < 0");
  if (nrows > 0 && s->num_fields > 0 && !columns)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "columns is null");
  if (!s->device_ok) return set_error(FURY_ERR_UNSUPPORTED, "no device kernel for " + s->device_reason);
  if (s->is_fixed) {
    *row_bytes = nrows * s->fixed_size;
    if (*row_bytes > rows_capacity)
      return set_error(FURY_ERR_CAPACITY, "rows need " + std::to_string(*row_bytes) + " bytes");
    if (nrows > 0 && !rows) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows is null");
    if (row_offsets)
      for (int64_t i = 0; i <= nrows; i++) row_offsets[i] = i * s->fixed_size;
    return fixed_host(s, columns, nrows, static_cast<uint8_t*>(rows), false, device);
  }
  if (!row_offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, "row_offsets is null");
  if (nrows == 0) {
    row_offsets[0] = 0;
    *row_bytes = 0;
    return FURY_OK;
  }
  return var_encode_host(s, columns, nrows, static_cast<uint8_t*>(rows), rows_capacity, row_offsets,
                         row_bytes, device);
}

int fury_row_decode_host(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                         int64_t nrows, fury_column* columns, int32_t device) {
  if (!s) return set_error(FURY_ERR_INVALID_ARGUMENT, "schema is null");
  if (nrows < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "nrows < 0");
  if (nrows == 0) {            // an empty batch still yields valid Arrow offsets (offsets[0] = 0)
    for (int k = 0; columns && k < s->num_fields; k++)
      if (columns[k].offsets) columns[k].offsets[0] = 0;
    return FURY_OK;
  }
  if (!rows || (s->num_fields > 0 && !columns))
    return set_error(FURY_ERR_INVALID_ARGUMENT, "rows/columns is null");
  if (!s->device_ok) return set_error(FURY_ERR_UNSUPPORTED, "no device kernel for " + s->device_reason);
  if (s->is_fixed)
    return fixed_host(s, columns, nrows, static_cast<uint8_t*>(const_cast<void*>(rows)), true,
                      device);
  if (!row_offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, "row_offsets is null");
  return var_decode_host(s, static_cast<const uint8_t*>(rows), row_offsets, nrows, columns, device);
}

}  // extern "C"
