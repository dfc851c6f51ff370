// capi.cpp — the extern "C" device entry points of include/fury_row.h: argument checks, then
// dispatch to the fixed-width tile kernels (fixed.hip) or the variable-length kernels (var.hip).
// Error statuses mirror the reference's exceptions (see fury_status).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

int check_hip(int hip_status, const char* what) {
  if (hip_status == hipSuccess) return FURY_OK;
  return set_error(FURY_ERR_DEVICE, std::string(what) + ": " +
                                        hipGetErrorString(static_cast<hipError_t>(hip_status)));
}

// Device error words (kernels.h): one slot of kErrWords words per stream, in host-pinned mapped
// memory.  A kernel raises into the slot of the stream it was launched on, and a call takes (reads
// and clears) only the slot of its own stream, so a malformed decode on one stream is never
// reported by -- or swallowed into -- an unrelated call on another stream / thread.
// The legacy null stream and hipStreamPerThread are keyed per host thread (two keys per thread,
// released when the thread exits).  Slots are assigned on first launch and go back to a free list
// when their stream is released: by the library when it destroys a stream it created (decode
// plans, host-path plans), by the caller through fury_stream_release (which synchronises the
// stream first, the null stream and hipStreamPerThread included) before it destroys one of its
// own.  A thread that exits makes no HIP call, so work it launched on its null-stream /
// per-thread keys may still be running: those slots go to a QUARANTINE, not the free list, and
// become free only after a device synchronisation that covers them (when the free slots run out,
// or fury_trim_workspace) -- a late error lands in the quarantined slot and is dropped there, never
// on an unrelated stream.  A call that needs a slot when all kErrSlots are held fails
// with FURY_ERR_DEVICE -- slots are never shared, so an error is reported on its own stream or not
// at all.
namespace {
constexpr int kErrSlots = 1024;
uint32_t* g_err_host = nullptr;     // host view of the slots
uint32_t* g_err_dev = nullptr;      // the same memory as kernels address it
std::once_flag g_err_once;
std::mutex g_slot_mu;
std::unordered_map<uintptr_t, int> g_slot_of;
std::vector<int> g_slot_free;       // released slots (words cleared)
std::vector<int> g_slot_quarantine; // released at thread exit, their work maybe still running
int g_slot_next = 0;                // slots [0, g_slot_next) have been handed out at least once

void release_key(uintptr_t k, bool quarantine = false);

// Per-thread keys of the null stream and of hipStreamPerThread (odd: never a stream handle, which
// is aligned); their slots are quarantined when the thread exits.
std::atomic<int> g_thread_key_exits{0};   // ThreadKeys destructors run (diagnostics)
struct ThreadKeys {
  char null_key = 0, per_thread_key = 0;
  ~ThreadKeys() {
    g_thread_key_exits.fetch_add(1);
    release_key(reinterpret_cast<uintptr_t>(&null_key) | 1, true);
    release_key(reinterpret_cast<uintptr_t>(&per_thread_key) | 1, true);
  }
};

uintptr_t stream_key(hipStream_t s) {
  if (s && s != hipStreamPerThread) return reinterpret_cast<uintptr_t>(s);
  thread_local ThreadKeys keys;
  return reinterpret_cast<uintptr_t>(s ? &keys.per_thread_key : &keys.null_key) | 1;
}

void init_err() {
  std::call_once(g_err_once, [] {
    void* p = nullptr;
    const size_t bytes = size_t(kErrSlots) * kErrWords * 4;
    if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
      (void)hipHostFree(p);
      return;
    }
    std::memset(p, 0, bytes);
    g_err_host = static_cast<uint32_t*>(p);
    g_err_dev = static_cast<uint32_t*>(d);
  });
}

void clear_slot_words(int slot);
int assign_slot_locked(uintptr_t k);

// Every device synchronised: the quarantined slots' kernels have finished, so their words can be
// cleared (late errors dropped) and the slots reused.  Called without g_slot_mu held.
void drain_quarantine() {
  {
    std::lock_guard<std::mutex> lock(g_slot_mu);
    if (g_slot_quarantine.empty()) return;
  }
  int n = 0, cur = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return;
  (void)hipGetDevice(&cur);
  std::vector<int> q;
  {
    std::lock_guard<std::mutex> lock(g_slot_mu);
    q.swap(g_slot_quarantine);       // slots quarantined after this point wait for the next drain
  }
  for (int d = 0; d < n; d++)
    if (hipSetDevice(d) == hipSuccess) (void)hipDeviceSynchronize();
  (void)hipSetDevice(cur);
  std::lock_guard<std::mutex> lock(g_slot_mu);
  for (int slot : q) {
    clear_slot_words(slot);
    g_slot_free.push_back(slot);
  }
}

// The slot of stream key k: its own, else a free or never-used one; when none is left, the
// quarantine is drained first (-1: all kErrSlots held by live streams).
// `assign` false: lookup only (a stream that never launched has nothing to report).
int error_slot(uintptr_t k, bool assign) {
  {
    std::lock_guard<std::mutex> lock(g_slot_mu);
    auto it = g_slot_of.find(k);
    if (it != g_slot_of.end()) return it->second;
    if (!assign) return -1;
    if (g_slot_free.empty() && g_slot_next >= kErrSlots && !g_slot_quarantine.empty()) {
      // fall through to the drain below (it synchronises: no lock held)
    } else {
      return assign_slot_locked(k);
    }
  }
  drain_quarantine();
  std::lock_guard<std::mutex> lock(g_slot_mu);
  auto it = g_slot_of.find(k);
  if (it != g_slot_of.end()) return it->second;
  return assign_slot_locked(k);
}

std::atomic<uintptr_t> g_last_assigned_key{0};   // diagnostics ("err_slot_last_key")

int assign_slot_locked(uintptr_t k) {
  g_last_assigned_key = k;
  int slot = -1;
  if (!g_slot_free.empty()) {
    slot = g_slot_free.back();
    g_slot_free.pop_back();
  } else if (g_slot_next < kErrSlots) {
    slot = g_slot_next++;
  } else {
    return -1;
  }
  g_slot_of.emplace(k, slot);
  return slot;
}

std::atomic<int64_t> g_err_dropped{0};   // look-back flags cleared by a release, never taken

void clear_slot_words(int slot) {
  if (!g_err_host) return;
  uint32_t* w = g_err_host + size_t(kErrWords) * slot;
  if (__atomic_exchange_n(w + kErrLookBack, 0u, __ATOMIC_ACQ_REL)) g_err_dropped.fetch_add(1);
  for (int i = 0; i < kErrWords; i++) __atomic_store_n(w + i, 0u, __ATOMIC_RELEASE);
}

void release_key(uintptr_t k, bool quarantine) {
  std::lock_guard<std::mutex> lock(g_slot_mu);
  auto it = g_slot_of.find(k);
  if (it == g_slot_of.end()) return;
  const int slot = it->second;
  g_slot_of.erase(it);
  if (quarantine) {
    g_slot_quarantine.push_back(slot);
    return;
  }
  clear_slot_words(slot);
  g_slot_free.push_back(slot);
}
}  // namespace

int thread_key_exits() { return g_thread_key_exits.load(); }
// 0: a stream handle, 1: a thread's null-stream key, 2: a thread's hipStreamPerThread key
int last_assigned_key_kind() {
  const uintptr_t k = g_last_assigned_key.load();
  if (!(k & 1)) return 0;
  return 1;   // (both thread keys are odd; which one is not distinguished)
}
int error_slots_quarantined() {
  std::lock_guard<std::mutex> lock(g_slot_mu);
  return static_cast<int>(g_slot_quarantine.size());
}
void drain_error_quarantine() { drain_quarantine(); }

int device_error_word(hipStream_t stream, uint32_t** out) {
  *out = nullptr;
  init_err();
  if (!g_err_dev) return FURY_OK;     // no mapped memory: kernels run without error reporting
  const int slot = error_slot(stream_key(stream), true);
  if (slot < 0)
    return set_error(FURY_ERR_DEVICE,
                     "device error slots exhausted: " + std::to_string(kErrSlots) +
                         " streams hold one; call fury_stream_release(stream) before destroying a "
                         "stream passed to this library");
  *out = g_err_dev + size_t(kErrWords) * slot;
  return FURY_OK;
}

// Forgets `stream`'s slot after the work on it has finished (its pending errors are dropped);
// `sync` false: the caller knows the stream is idle (thread exit: no HIP call).
void release_error_slot(hipStream_t stream, bool sync) {
  if (sync) (void)hipStreamSynchronize(stream);   // NULL / hipStreamPerThread: this thread's
  release_key(stream_key(stream));
}

int error_slots_in_use() {
  std::lock_guard<std::mutex> lock(g_slot_mu);
  return static_cast<int>(g_slot_of.size());
}

std::atomic<int64_t> g_err_taken{0};

int64_t device_error_count() {
  int64_t pending = 0;
  if (g_err_host) {
    std::lock_guard<std::mutex> lock(g_slot_mu);
    for (int i = 0; i < g_slot_next; i++)
      pending += __atomic_load_n(g_err_host + size_t(kErrWords) * i + kErrLookBack, __ATOMIC_ACQUIRE) ? 1 : 0;
  }
  return g_err_taken.load() + g_err_dropped.load() + pending;
}

// Where a kernel found the problem: a row index, or (bit 63 set) a nested schema node and Arrow
// entry (err_where_entry).
static std::string where_text(uint64_t w) {
  if (!(w >> 63)) return "row " + std::to_string(w);
  if ((w >> 62) & 1)           // err_where_tile: a nested entry of the tile that starts at a row
    return "schema node " + std::to_string((w >> 40) & 0x3fffff) + " in the rows from row " +
           std::to_string(w & ((1ull << 40) - 1));
  return "schema node " + std::to_string((w >> 40) & 0x7fffff) + ", Arrow entry " +
         std::to_string(w & ((1ull << 40) - 1));
}

// Takes one flag of the slot: the flag is exchanged for 0 first, then its location word is read
// and cleared (raise_at stores the location before it releases the flag).
static bool take_flag(uint32_t* w, int flag, uint64_t* where) {
  if (!__atomic_exchange_n(w + flag, 0u, __ATOMIC_ACQ_REL)) return false;
  if (where) *where = __atomic_exchange_n(reinterpret_cast<uint64_t*>(w + flag + 2), 0ull, __ATOMIC_ACQ_REL);
  return true;
}

int take_device_error(hipStream_t stream) {
  if (!g_err_host) return FURY_OK;
  const int slot = error_slot(stream_key(stream), false);
  if (slot < 0) return FURY_OK;       // nothing was ever launched on this stream
  uint32_t* w = g_err_host + size_t(kErrWords) * slot;
  uint64_t oob_at = 0, map_at = 0;
  const bool lb = take_flag(w, kErrLookBack, nullptr);
  const bool oob = take_flag(w, kErrBounds, &oob_at);
  const bool map = take_flag(w, kErrMapCount, &map_at);
  uint64_t deep_at = 0, budget_at = 0;
  const bool deep = take_flag(w, kErrTooDeep, &deep_at);
  const bool budget = take_flag(w, kErrBudget, &budget_at);
  uint64_t internal_at = 0;
  const bool internal = take_flag(w, kErrInternal, &internal_at);
  if (!lb && !oob && !map && !deep && !budget && !internal) return FURY_OK;
  if (internal)
    return set_error(FURY_ERR_DEVICE, "decode: the tile from " + where_text(internal_at) +
                                          " outgrew its on-chip plan (internal error); the outputs "
                                          "of that call are invalid");
  if (lb) {
    g_err_taken.fetch_add(1);
    return set_error(FURY_ERR_DEVICE,
                     "an earlier asynchronous launch failed on the device (a decoupled look-back "
                     "gave up waiting): the outputs of that call are invalid");
  }
  if (oob)
    return set_error(FURY_ERR_OUT_OF_BOUNDS,
                     "decode: " + where_text(oob_at) +
                         " has a variable-length value, array or map header outside the batch's "
                         "row bytes (MemoryBuffer bounds check); the outputs of that call are "
                         "invalid");
  if (deep)
    return set_error(FURY_ERR_UNSUPPORTED,
                     "encode: " + where_text(deep_at) +
                         " is too large to assemble on chip and the schema is nested deeper than "
                         "the row interpreter reaches; the rows of that call are invalid");
  if (map)
    return set_error(FURY_ERR_UNSUPPORTED,
                     "decode: " + where_text(map_at) +
                         ": map key and value arrays have different element counts "
                         "(BinaryMap.pointTo); the outputs of that call are invalid");
  return budget_error(where_text(budget_at));
}

namespace {
std::atomic<int64_t> g_budget_errors{0};
}
int budget_error(const std::string& where) {
  g_budget_errors.fetch_add(1);
  return set_error(FURY_ERR_UNSUPPORTED,
                   "decode budget: " + where +
                       ": slots alias other bytes of the batch so that decoding would visit more "
                       "items than the rows hold (a device limit, not a reference exception: "
                       "the reference would decode such rows); the outputs of that call are "
                       "invalid");
}
int64_t budget_errors() { return g_budget_errors.load(); }

// Pinned staging ring for per-call column tables: the host table is copied into the ring, then
// DMA-ed to a stream-ordered device allocation on the caller's stream (no host synchronisation);
// a ring region is reused only after the event of the copy that read it has completed.
namespace {
std::mutex g_ring_mu;
uint8_t* g_ring = nullptr;
size_t g_ring_head = 0;
constexpr size_t kRingBytes = 4u << 20;
struct RingUse {
  size_t off, bytes;
  hipEvent_t ev;
};
std::vector<RingUse> g_ring_pending;
}  // namespace

// ---- device workspace cache -------------------------------------------------------------------
// Per-call workspaces (scan scratch, column tables, decode plans) come from size classes cached
// per device instead of hipMallocAsync / hipFreeAsync: on the box hipFreeAsync took ~110 us of
// host time per call (HIP API trace of scripts/ab_generic.py), more than most of the kernels it
// serves.  A freed block records an event on its stream; its next user's stream waits for that
// event on the device (hipStreamWaitEvent, no host sync) -- also when the handles are equal,
// since a destroyed stream's handle can be reused.  Classes: powers of two up to 64 MB, 2 MB
// multiples above (a 5.8 GB plan array is not rounded to 8 GB).  Cached free bytes are capped
// (kCacheCap, 2 GB: the cache exists for per-call workspaces, not for whole batches); beyond that
// blocks go back to the pool.  An allocation that fails releases every idle cached block and
// trims the stream pool, then retries once; fury_trim_workspace() does the same on request.
namespace {
struct CacheBlock {
  void* p;
  size_t cls;
  int device;
  hipEvent_t ev;
};
std::mutex g_cache_mu;
std::vector<CacheBlock> g_cache_free;
std::unordered_map<void*, std::pair<size_t, int>> g_cache_live;
size_t g_cache_bytes = 0;                     // bytes in g_cache_free
constexpr size_t kCacheCap = size_t(2) << 30;

size_t size_class(int64_t bytes) {
  const size_t b = static_cast<size_t>(bytes > 0 ? bytes : 1);
  constexpr size_t kBig = size_t(64) << 20, kStep = size_t(2) << 20;
  if (b > kBig) return (b + kStep - 1) / kStep * kStep;
  size_t cls = 4096;
  while (cls < b) cls <<= 1;
  return cls;
}

// Frees every idle cached block of `device` (after the work that last used it) and trims that
// device's stream pool.  Returns the bytes released.
size_t release_cached(int device) {
  std::vector<CacheBlock> drop;
  {
    std::lock_guard<std::mutex> lock(g_cache_mu);
    for (size_t i = 0; i < g_cache_free.size();) {
      if (g_cache_free[i].device == device) {
        drop.push_back(g_cache_free[i]);
        g_cache_bytes -= g_cache_free[i].cls;
        g_cache_free[i] = g_cache_free.back();
        g_cache_free.pop_back();
      } else {
        i++;
      }
    }
  }
  size_t bytes = 0;
  for (CacheBlock& b : drop) {
    (void)hipEventSynchronize(b.ev);
    (void)hipEventDestroy(b.ev);
    (void)hipFree(b.p);
    bytes += b.cls;
  }
  hipMemPool_t pool = nullptr;
  if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) (void)hipMemPoolTrimTo(pool, 0);
  return bytes;
}
}  // namespace

int dev_alloc(int64_t bytes, hipStream_t stream, void** out) {
  *out = nullptr;
  const size_t cls = size_class(bytes);
  int device = 0;
  (void)hipGetDevice(&device);
  {
    std::lock_guard<std::mutex> lock(g_cache_mu);
    for (size_t i = 0; i < g_cache_free.size(); i++) {
      CacheBlock b = g_cache_free[i];
      if (b.cls != cls || b.device != device) continue;
      g_cache_free[i] = g_cache_free.back();
      g_cache_free.pop_back();
      g_cache_bytes -= cls;
      // always wait on the device (free when already ordered): a stream handle can be reused
      // by a new stream after the old one is destroyed with work pending
      (void)hipStreamWaitEvent(stream, b.ev, 0);
      (void)hipEventDestroy(b.ev);
      g_cache_live[b.p] = {cls, device};
      *out = b.p;
      return FURY_OK;
    }
  }
  keep_pool(device);
  hipError_t e = hipMallocAsync(out, cls, stream);
  if (e != hipSuccess) {              // idle cached blocks may be what is missing: release, retry
    (void)hipGetLastError();
    release_cached(device);
    e = hipMallocAsync(out, cls, stream);
  }
  const int st = check_hip(e, "hipMallocAsync");
  if (st) return st;
  std::lock_guard<std::mutex> lock(g_cache_mu);
  g_cache_live[*out] = {cls, device};
  return FURY_OK;
}

void dev_free(void* p, hipStream_t stream) {
  if (!p) return;
  std::lock_guard<std::mutex> lock(g_cache_mu);
  auto it = g_cache_live.find(p);
  if (it == g_cache_live.end()) return;
  const size_t cls = it->second.first;
  const int device = it->second.second;
  g_cache_live.erase(it);
  hipEvent_t ev = nullptr;
  if (g_cache_bytes + cls > kCacheCap ||
      hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipFreeAsync(p, stream);
    return;
  }
  (void)hipEventRecord(ev, stream);
  g_cache_free.push_back(CacheBlock{p, cls, device, ev});
  g_cache_bytes += cls;
}

DeviceTable::~DeviceTable() {
  if (dev) dev_free(dev, stream);
}

int upload_table(const void* host, size_t bytes, hipStream_t stream, DeviceTable* out) {
  if (bytes == 0 || bytes > kRingBytes)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "column table size");
  std::lock_guard<std::mutex> lock(g_ring_mu);
  if (!g_ring) {
    void* p = nullptr;
    int st = check_hip(hipHostMalloc(&p, kRingBytes, hipHostMallocDefault), "hipHostMalloc");
    if (st) return st;
    g_ring = static_cast<uint8_t*>(p);
  }
  size_t off = (g_ring_head + 255) & ~size_t(255);
  if (off + bytes > kRingBytes) off = 0;
  for (size_t i = 0; i < g_ring_pending.size();) {   // wait for copies still reading the region
    RingUse& u = g_ring_pending[i];
    const bool overlap = u.off < off + bytes && off < u.off + u.bytes;
    if (overlap || hipEventQuery(u.ev) == hipSuccess) {
      if (overlap) (void)hipEventSynchronize(u.ev);
      (void)hipEventDestroy(u.ev);
      g_ring_pending[i] = g_ring_pending.back();
      g_ring_pending.pop_back();
    } else {
      i++;
    }
  }
  std::memcpy(g_ring + off, host, bytes);
  out->host.assign(static_cast<const uint8_t*>(host), static_cast<const uint8_t*>(host) + bytes);
  g_ring_head = off + bytes;
  int st = dev_alloc(static_cast<int64_t>(bytes), stream, &out->dev);
  if (st) return st;
  out->stream = stream;
  st = check_hip(hipMemcpyAsync(out->dev, g_ring + off, bytes, hipMemcpyHostToDevice, stream),
                 "hipMemcpyAsync column table");
  if (st) return st;
  hipEvent_t ev;
  if ((st = check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate")))
    return st;
  (void)hipEventRecord(ev, stream);
  g_ring_pending.push_back(RingUse{off, bytes, ev});
  return FURY_OK;
}

namespace {

bool misaligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) != 0; }

int common_checks(const fury_schema* s, const void* cols, int64_t nrows, const char* fn,
                  hipStream_t hs) {
  if (!s) return set_error(FURY_ERR_INVALID_ARGUMENT, std::string(fn) + ": schema is null");
  if (nrows < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, std::string(fn) + ": nrows < 0");
  if (nrows > 0 && s->num_fields > 0 && !cols)
    return set_error(FURY_ERR_INVALID_ARGUMENT, std::string(fn) + ": columns is null");
  if (!s->device_ok)
    return set_error(FURY_ERR_UNSUPPORTED,
                     std::string(fn) + ": no device kernel for " + s->device_reason);
  return take_device_error(hs);
}

int fixed_args(const fury_schema* s, const fury_column* cols, int64_t nrows, bool decode,
               bool need_validity, FixedArgs* a, bool* fast, DeviceTable* dt, hipStream_t hs) {
  *a = FixedArgs{};
  a->ncols = s->num_fields;
  a->bitmap_bytes = s->bitmap_bytes;
  a->row_size = s->fixed_size;
  a->nrows = nrows;
  const bool wide = s->num_fields > kMaxFixedCols;
  std::vector<FixedCol> tab(wide ? s->num_fields : 0);
  bool all8 = true, anyv = false;
  for (int k = 0; k < s->num_fields; k++) {
    const FieldPlan& p = s->plan[k];
    const fury_column& c = cols[k];
    if (nrows > 0 && !c.values)
      return set_error(FURY_ERR_INVALID_ARGUMENT,
                       "column " + std::to_string(k) + " (" + s->fields[k].name + "): values is null");
    const int w = p.kind == kBool ? 0 : p.width;
    if (w > 1 && misaligned(c.values, static_cast<uintptr_t>(w)))
      return set_error(FURY_ERR_INVALID_ARGUMENT,
                       "column " + std::to_string(k) + ": values not " + std::to_string(w) +
                           "-byte aligned");
    if (need_validity && !c.validity)
      return set_error(FURY_ERR_INVALID_ARGUMENT,
                       "column " + std::to_string(k) + ": Arrow output needs a validity buffer");
    FixedCol& fc = wide ? tab[k] : a->col[k];
    fc.values = static_cast<const uint8_t*>(c.values);
    fc.validity = c.validity;
    fc.width = w;
    if (w != 8) all8 = false;
    if (c.validity) anyv = true;
  }
  (void)decode;
  *fast = all8 && !anyv && !wide;         // wide tables run the general tile kernel only
  if (wide) {
    const int st = upload_table(tab.data(), tab.size() * sizeof(FixedCol), hs, dt);
    if (st) return st;
    a->tab = static_cast<const FixedCol*>(dt->dev);
  }
  return FURY_OK;
}

int var_args(const fury_schema* s, const fury_column* cols, int64_t nrows, bool decode,
             bool need_validity, VarArgs* a, DeviceTable* dt, hipStream_t hs,
             bool shape_only = false) {
  if (s->num_fields > kMaxWideVarCols)
    return set_error(FURY_ERR_UNSUPPORTED, "variable-length device path handles at most " +
                                               std::to_string(kMaxWideVarCols) + " fields");
  *a = VarArgs{};
  a->ncols = s->num_fields;
  a->bitmap_bytes = s->bitmap_bytes;
  a->fixed_size = s->fixed_size;
  a->nrows = nrows;
  const bool wide = s->num_fields > kMaxVarCols;
  std::vector<VarCol> tab(wide ? s->num_fields : 0);
  int nvar = 0;
  for (int k = 0; k < s->num_fields; k++) {
    const FieldPlan& p = s->plan[k];
    static const fury_column kNoColumn{};
    const fury_column& c = shape_only ? kNoColumn : cols[k];
    VarCol& v = wide ? tab[k] : a->col[k];
    const std::string who = "column " + std::to_string(k) + " (" + s->fields[k].name + ")";
    v.kind = p.kind;
    v.nullable = p.nullable;
    v.var_slot = -1;
    v.validity = c.validity;
    if (decode && c.validity && misaligned(c.validity, 4))
      return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": validity must be 4-byte aligned");
    if (need_validity && !c.validity)
      return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": Arrow output needs a validity buffer");
    switch (p.kind) {
      case kFixed:
      case kBool:
        v.width = p.kind == kBool ? 0 : p.width;
        v.values = static_cast<const uint8_t*>(c.values);
        if (!shape_only && nrows > 0 && !c.values) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": values is null");
        if (v.width > 1 && misaligned(c.values, v.width))
          return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": values misaligned");
        break;
      case kBytes:
        v.width = 1;
        v.values = static_cast<const uint8_t*>(c.values);
        v.offsets = c.offsets;
        v.var_slot = nvar++;
        v.capacity = c.values ? c.capacity : 0;
        if (!shape_only && nrows > 0 && !c.offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": offsets is null");
        break;
      case kDecimal:
        v.width = 16;
        v.values = static_cast<const uint8_t*>(c.values);
        v.var_slot = nvar++;
        if (!shape_only && nrows > 0 && !c.values) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": values is null");
        break;
      case kListFixed: {
        v.width = p.elem_type == FURY_TYPE_BOOL ? 0 : p.elem_width;
        v.offsets = c.offsets;
        v.var_slot = nvar++;
        if (!shape_only && nrows > 0 && !c.offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": offsets is null");
        if (!c.child) {
          if (!shape_only && (!decode || nrows > 0))
            return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": list needs a child column");
        } else {
          v.values = static_cast<const uint8_t*>(c.child->values);
          v.elem_validity = c.child->validity;
          // child capacity is in bytes of values; the kernels bound element indices by it
          v.capacity = !c.child->values ? 0
                       : v.width == 0   ? c.child->capacity * 8
                                        : c.child->capacity / v.width;
          if (decode && (misaligned(c.child->validity, 4) ||
                         (v.width == 0 && misaligned(c.child->values, 4))))
            return set_error(FURY_ERR_INVALID_ARGUMENT,
                             who + ": element bitmaps must be 4-byte aligned");
          if (need_validity && !c.child->validity)
            return set_error(FURY_ERR_INVALID_ARGUMENT,
                             who + ": Arrow output needs element validity");
          if (v.width > 1 && misaligned(v.values, v.width))
            return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": element values misaligned");
        }
        break;
      }
      default:
        return set_error(FURY_ERR_UNSUPPORTED, who + ": no device kernel");
    }
  }
  a->nvar = nvar;
  if (wide) {                      // wider than the argument block: the table goes to the device
    const int st = upload_table(tab.data(), tab.size() * sizeof(VarCol), hs, dt);
    if (st) return st;
    a->tab = static_cast<const VarCol*>(dt->dev);
    a->htab = reinterpret_cast<const VarCol*>(dt->host.data());
    a->tile_rows = encode_tile_rows(*a);
  } else {
    a->tile_rows = encode_tile_rows(*a);
  }
  if (const int e = device_error_word(hs, &a->err)) return e;
  a->help_now = lookback_help_mode();
  a->skip = var_skip();
  return FURY_OK;
}

// Generic engine arguments: schema nodes (breadth-first) + the column tree walked in the same
// order (LIST: child[0] = elements; STRUCT: child[0..n); MAP: child[0] keys, child[1] values).
int gen_args(const fury_schema* s, const fury_column* cols, int64_t nrows, bool decode,
             bool need_validity, GenArgs* g, DeviceTable* dt, hipStream_t hs) {
  const size_t nn = s->nodes.size();
  if (nn > static_cast<size_t>(kGenMaxWideNodes))
    return set_error(FURY_ERR_UNSUPPORTED, "nested schema has more than " +
                                               std::to_string(kGenMaxWideNodes) + " nodes");
  const bool wide = nn > static_cast<size_t>(kGenMaxNodes);
  std::vector<GenNode> tab(wide ? nn : 0);
  GenNode* nodes = nullptr;
  *g = GenArgs{};
  nodes = wide ? tab.data() : g->node;
  g->nnodes = static_cast<int32_t>(nn);
  g->ntop = s->num_fields;
  g->nrows = nrows;
  g->err = nullptr;
  g->root = s->root;
  if (s->root && !decode && cols && cols[0].validity)
    return set_error(FURY_ERR_INVALID_ARGUMENT,
                     "collection batch: the top-level column has no validity (toArray / toMap of a "
                     "null collection is not defined)");
  std::vector<const fury_column*> col(nn, nullptr);
  for (int k = 0; k < s->num_fields; k++) col[k] = &cols[k];
  for (size_t i = 0; i < nn; i++) {
    const GenTpl& t = s->nodes[i];
    const fury_column* c = col[i];
    const std::string who = "schema node " + std::to_string(i);
    if (!c) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": missing column");
    GenNode& n = nodes[i];
    n.values = static_cast<const uint8_t*>(c->values);
    n.validity = c->validity;
    n.offsets = c->offsets;
    n.type = t.type_id;
    n.first_child = t.first_child;
    n.num_children = t.num_children;
    // breadth-first order: a node's parent is set before it
    if (i < static_cast<size_t>(s->num_fields)) n.row_aligned = 1;
    if (n.row_aligned && t.type_id == FURY_TYPE_STRUCT)
      for (int j = 0; j < t.num_children; j++) nodes[t.first_child + j].row_aligned = 1;
    if (t.num_children > 0) {
      if (!c->child) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": child columns missing");
      for (int j = 0; j < t.num_children; j++) col[t.first_child + j] = &c->child[j];
    }
    const bool var = t.type_id == FURY_TYPE_STRING || t.type_id == FURY_TYPE_BINARY ||
                     t.type_id == FURY_TYPE_LIST || t.type_id == FURY_TYPE_MAP;
    if (nrows > 0 && var && !c->offsets)
      return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": offsets is null");
    if (need_validity && !c->validity)
      return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": Arrow output needs a validity buffer");
    if (decode && c->validity && misaligned(c->validity, 4))
      return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": validity must be 4-byte aligned");
    if (decode && t.type_id == FURY_TYPE_BOOL && c->values && misaligned(c->values, 4))
      return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": bool bitmap must be 4-byte aligned");
  }
  if (wide) {                      // more nodes than the argument block: table to the device
    const int st = upload_table(tab.data(), tab.size() * sizeof(GenNode), hs, dt);
    if (st) return st;
    g->tab = static_cast<const GenNode*>(dt->dev);
    g->htab = reinterpret_cast<const GenNode*>(dt->host.data());
  }
  return FURY_OK;
}

int gen_measure(const fury_schema* s, const fury_column* cols, int64_t nrows, int64_t* offs,
                hipStream_t stream) {
  GenArgs g;
  DeviceTable dt;
  int st = gen_args(s, cols, nrows, false, false, &g, &dt, stream);
  if (st) return st;
  if (nrows == 0) return check_hip(hipMemsetAsync(offs, 0, 8, stream), "memset");
  st = launch_gen_measure(g, offs, stream);
  if (st) return st;
  int64_t* ws = nullptr;
  st = dev_alloc(scan_workspace(nrows) * 8, stream, reinterpret_cast<void**>(&ws));
  if (st) return st;
  device_scan(offs, nrows, offs + nrows, ws, stream);
  st = check_hip(hipGetLastError(), "scan launch");
  dev_free(ws, stream);
  return st;
}

}  // namespace
}  // namespace fury

using namespace fury;

extern "C" {

// tuning "wide_enc_engine" (round 6): the encode of a 17-256-field flat variable-length schema -- 0
// auto, 1 the wide tiles (wide.hip), 2 the row-walk encode (rowenc.hip, as nested schemas).  Auto
// takes the row walk when the rows' estimated average (the header + each variable-length column's
// capacity / rows) exceeds "wide_walk_row" bytes, as the decode plan does.  The rows are the same
// bytes either way (the Java layout).  1M rows, wide vs walk (scripts/ab_wide.py --enc-engines,
// profiles/r06_wide_enc_engine.jsonl): id + 126 / 70 / 55 / 40 STRING fields (3.2 / 1.8 / 1.4 / 1.0
// KB rows) 9.56 / 5.22 / 4.10 / 2.59 vs 6.76 / 3.67 / 2.91 / 2.15 ms; the tests' 33-field schema
// (581 B rows) 0.51 vs 1.07 ms.
static std::atomic<int> g_wide_enc_engine{0};
static std::atomic<int> g_wide_walk_row{896};

static bool wide_encode_by_walk(const fury_schema* s, const fury_column* cols, int64_t nrows) {
  if (s->generic || s->is_fixed || s->num_fields <= 16 || s->num_fields > kMaxWideVarCols ||
      !var_wide_mode() || !cols || nrows <= 0)
    return false;
  const int mode = g_wide_enc_engine.load();
  if (mode != 0) return mode == 2;
  double row = s->fixed_size;
  for (int k = 0; k < s->num_fields; k++) {
    const int kind = s->plan[k].kind;
    if (kind == kBytes && cols[k].values) row += static_cast<double>(cols[k].capacity) / nrows + 4;
    if (kind == kDecimal) row += 16;
    if (kind == kListFixed && cols[k].child && cols[k].child->values)
      row += 16 + static_cast<double>(cols[k].child->capacity) / nrows;
  }
  return row > g_wide_walk_row.load();
}

int fury_row_measure(const fury_schema* s, const fury_column* cols, int64_t nrows,
                     int64_t* row_offsets, void* stream) {
  int st = common_checks(s, cols, nrows, "fury_row_measure", static_cast<hipStream_t>(stream));
  if (st) return st;
  if (!row_offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, "row_offsets is null");
  if (misaligned(row_offsets, 8)) return set_error(FURY_ERR_INVALID_ARGUMENT, "row_offsets misaligned");
  if (s->generic || wide_encode_by_walk(s, cols, nrows))
    return gen_measure(s, cols, nrows, row_offsets, static_cast<hipStream_t>(stream));
  VarArgs a;
  DeviceTable dt;
  st = var_args(s, cols, nrows, false, false, &a, &dt, static_cast<hipStream_t>(stream));
  if (st) return st;
  return launch_measure_rows(a, row_offsets, static_cast<hipStream_t>(stream));
}

int fury_row_encode(const fury_schema* s, const fury_column* cols, int64_t nrows,
                    const int64_t* row_offsets, void* rows, void* stream) {
  int st = common_checks(s, cols, nrows, "fury_row_encode", static_cast<hipStream_t>(stream));
  if (st) return st;
  if (nrows == 0) return FURY_OK;
  if (!rows) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows is null");
  if (misaligned(rows, 16)) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows must be 16-byte aligned");
  hipStream_t hs = static_cast<hipStream_t>(stream);
  if (s->is_fixed) {
    // Fixed schemas: rows are contiguous at i * fixed_size (row_offsets, when given, are those).
    FixedArgs a;
    bool fast = false;
    DeviceTable dt;
    st = fixed_args(s, cols, nrows, false, false, &a, &fast, &dt, hs);
    if (st) return st;
    return launch_encode_fixed(a, static_cast<uint8_t*>(rows), hs, fast);
  }
  if (!row_offsets)
    return set_error(FURY_ERR_INVALID_ARGUMENT,
                     "variable-length schema needs row_offsets from fury_row_measure");
  if (s->generic || wide_encode_by_walk(s, cols, nrows)) {
    GenArgs g;
    DeviceTable dt;
    st = gen_args(s, cols, nrows, false, false, &g, &dt, hs);
    if (st) return st;
    return launch_gen_encode(g, row_offsets, static_cast<uint8_t*>(rows), INT64_MAX, hs);
  }
  VarArgs a;
  DeviceTable dt;
  st = var_args(s, cols, nrows, false, false, &a, &dt, hs);
  if (st) return st;
  return launch_encode_var(a, row_offsets, static_cast<uint8_t*>(rows), INT64_MAX, hs);
}

int fury_row_encode_measured(const fury_schema* s, const fury_column* cols, int64_t nrows,
                             int64_t* row_offsets, void* rows, int64_t capacity, void* stream) {
  int st = common_checks(s, cols, nrows, "fury_row_encode_measured", static_cast<hipStream_t>(stream));
  if (st) return st;
  hipStream_t hs = static_cast<hipStream_t>(stream);
  if (capacity < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "capacity < 0");
  if (nrows > 0 && !rows) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows is null");
  if (misaligned(rows, 16)) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows must be 16-byte aligned");
  if (s->is_fixed) {
    if (nrows > 0 && nrows > capacity / s->fixed_size)
      return set_error(FURY_ERR_CAPACITY, "rows need " + std::to_string(nrows * s->fixed_size) +
                                              " bytes, capacity is " + std::to_string(capacity));
    if (row_offsets) {
      st = fury_row_measure(s, cols, nrows, row_offsets, stream);
      if (st) return st;
    }
    return fury_row_encode(s, cols, nrows, nullptr, rows, stream);
  }
  if (!row_offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, "row_offsets is null");
  if (misaligned(row_offsets, 8)) return set_error(FURY_ERR_INVALID_ARGUMENT, "row_offsets misaligned");
  if (s->generic || wide_encode_by_walk(s, cols, nrows)) {
    st = gen_measure(s, cols, nrows, row_offsets, hs);
    if (st || nrows == 0) return st;
    GenArgs g;
    DeviceTable dt;
    st = gen_args(s, cols, nrows, false, false, &g, &dt, hs);
    if (st) return st;
    return launch_gen_encode(g, row_offsets, static_cast<uint8_t*>(rows), capacity, hs);
  }
  VarArgs a;
  DeviceTable dt;
  st = var_args(s, cols, nrows, false, false, &a, &dt, hs);
  if (st) return st;
  const int one = launch_encode_measured_var(a, row_offsets, static_cast<uint8_t*>(rows), capacity, hs);
  if (one >= 0) return one;
  st = launch_measure_rows(a, row_offsets, hs);
  if (st || nrows == 0) return st;
  return launch_encode_var(a, row_offsets, static_cast<uint8_t*>(rows), capacity, hs);
}

// An empty batch still yields valid Arrow offsets (offsets[0] = 0) in every top-level column that
// has an offsets buffer; for n > 0 the decode kernels write them, for n = 0 none is launched.
static int zero_empty_offsets(const fury_schema* s, fury_column* cols, hipStream_t hs) {
  if (!cols) return FURY_OK;
  for (int k = 0; k < s->num_fields; k++) {
    if (!cols[k].offsets) continue;
    const int st = check_hip(hipMemsetAsync(cols[k].offsets, 0, 4, hs), "memset");
    if (st) return st;
  }
  return FURY_OK;
}

int fury_row_decode_measure(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                            int64_t nrows, fury_column* cols, void* stream) {
  int st = common_checks(s, cols, nrows, "fury_row_decode_measure", static_cast<hipStream_t>(stream));
  if (st) return st;
  if (nrows == 0) return zero_empty_offsets(s, cols, static_cast<hipStream_t>(stream));
  if (s->is_fixed) return FURY_OK;   // nothing variable to size
  if (s->generic)
    return set_error(FURY_ERR_INVALID_ARGUMENT,
                     "nested (or > 256-field variable-length) schema: size outputs with "
                     "fury_decode_prepare / fury_decode_execute");
  if (!rows || !row_offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows/row_offsets null");
  VarArgs a;
  DeviceTable dt;
  st = var_args(s, cols, nrows, true, false, &a, &dt, static_cast<hipStream_t>(stream));
  if (st) return st;
  return launch_decode_measure(a, static_cast<const uint8_t*>(rows), row_offsets,
                               static_cast<hipStream_t>(stream));
}

static int decode_impl(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                       int64_t nrows, fury_column* cols, void* stream, bool arrow,
                       const char* fn) {
  int st = common_checks(s, cols, nrows, fn, static_cast<hipStream_t>(stream));
  if (st) return st;
  if (nrows == 0) return zero_empty_offsets(s, cols, static_cast<hipStream_t>(stream));
  if (!rows) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows is null");
  hipStream_t hs = static_cast<hipStream_t>(stream);
  if (s->is_fixed) {
    if (misaligned(rows, 16)) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows must be 16-byte aligned");
    FixedArgs a;
    bool fast = false;
    DeviceTable dt;
    st = fixed_args(s, cols, nrows, true, arrow, &a, &fast, &dt, hs);
    if (st) return st;
    return launch_decode_fixed(a, static_cast<const uint8_t*>(rows), hs, fast);
  }
  if (!row_offsets)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "variable-length rows need row_offsets");
  if (misaligned(rows, 8)) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows must be 8-byte aligned");
  if (s->generic)
    return set_error(FURY_ERR_INVALID_ARGUMENT,
                     "nested (or > 256-field variable-length) schema: decode with "
                     "fury_decode_prepare / fury_decode_execute");
  VarArgs a;
  DeviceTable dt;
  st = var_args(s, cols, nrows, true, arrow, &a, &dt, hs);
  if (st) return st;
  return launch_decode_var(a, static_cast<const uint8_t*>(rows), row_offsets, hs, arrow);
}

int fury_row_decode(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                    int64_t nrows, fury_column* cols, void* stream) {
  return decode_impl(s, rows, row_offsets, nrows, cols, stream, false, "fury_row_decode");
}

int fury_rows_to_arrow(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                       int64_t nrows, fury_column* cols, void* stream) {
  return decode_impl(s, rows, row_offsets, nrows, cols, stream, true, "fury_rows_to_arrow");
}

// tuning "wide_engine" (round 6): the engine of a 17-256-field flat variable-length schema's plan --
// 0 auto (default), 1 the wide tiles (wide.hip), 2 the row walk (walk.hip, field groups past 16
// counted fields).  Auto takes the walk when the batch's average row (one 8-byte read) exceeds
// "wide_walk_row" bytes: the wide tiles stage 64 rows in at most 96 KB and read the rest from HBM
// lane by lane (1M rows, scripts/ab_deep.py --flat / --wide33, profiles/r06_wide_engine.jsonl; id +
// N STRING fields, wide vs walk: N = 126 / 2.45 KB rows 15.9 vs 6.1 ms, 90 / 1.75 KB 10.0 vs 4.3,
// 70 / 1.37 KB 5.45 vs 3.34, 55 / 1.07 KB 3.82 vs 2.65, 40 / 785 B 1.72 vs 1.95; the tests'
// 33-field schema, 520 B: 0.90 vs 1.70).
static std::atomic<int> g_wide_engine{0};

int fury_decode_prepare(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                        int64_t nrows, int64_t* node_entries, int64_t* node_bytes,
                        fury_decode_plan** plan, void* stream) {
  if (!s || !plan) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_decode_prepare: null argument");
  *plan = nullptr;
  if (nrows < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "nrows < 0");
  if (!s->device_ok) return set_error(FURY_ERR_UNSUPPORTED, "no device kernel for " + s->device_reason);
  if (nrows > 0 && (!rows || !row_offsets))
    return set_error(FURY_ERR_INVALID_ARGUMENT, "rows / row_offsets is null");
  hipStream_t hs = static_cast<hipStream_t>(stream);
  if (const int e = take_device_error(hs)) return e;
  const int nn = static_cast<int>(s->nodes.size());
  fury_decode_plan* p = new fury_decode_plan();
  p->schema = s;
  p->rows = static_cast<const uint8_t*>(rows);
  p->offs = row_offsets;
  p->nrows = nrows;
  std::vector<int64_t> totals(2 * nn, 0);
  // flat variable-length schemas of 17-256 fields: the wide kernels' count pass + scan, kept for
  // the execute (the tile bases), one host sync for the sequence fields' totals
  const bool wide_shape = nrows > 0 && !s->generic && !s->is_fixed && s->num_fields > 16 /* kRegCols: the register-staged kernels below */ &&
                          s->num_fields <= kMaxWideVarCols && var_wide_mode();
  int engine = g_wide_engine.load();
  if (wide_shape && engine == 0) {
    int64_t bytes = 0;
    int st = check_hip(hipMemcpyAsync(&bytes, row_offsets + nrows, 8, hipMemcpyDeviceToHost, hs),
                       "hipMemcpyAsync batch bytes");
    if (!st) st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize");
    if (st) {
      delete p;
      return st;
    }
    engine = bytes > static_cast<int64_t>(g_wide_walk_row.load()) * nrows ? 2 : 1;
  }
  const bool wide = wide_shape && engine != 2;
  if (wide) {
    VarArgs a;
    DeviceTable dt;
    std::vector<int64_t> seq;
    int st = var_args(s, nullptr, nrows, true, false, &a, &dt, hs, true);
    if (!st) {
      p->wide = new WidePlan();
      st = wide_prepare(a, p->rows, row_offsets, hs, p->wide, &seq);
    }
    if (!st) st = take_device_error(hs);
    if (st) {
      if (p->wide) wide_free(p->wide);
      delete p;
      return st;
    }
    int q = 0;
    for (int k = 0; k < s->num_fields; k++) {
      totals[2 * k] = nrows;
      const int kind = s->plan[k].kind;
      if (kind != kBytes && kind != kListFixed) continue;
      if (kind == kBytes) totals[2 * k + 1] = seq[q];
      else totals[2 * s->nodes[k].first_child] = seq[q];
      q++;
    }
  } else if (nrows > 0) {
    // both engines synchronise `stream`: rows whose values leave the batch are reported here.
    // The tile-staged engine first; the level engine when it declines the batch.
    int st = tree_prepare(s, p->rows, row_offsets, nrows, hs, &p->tree, &totals);
    if (!st && !p->tree) {
      if (const int e = take_device_error(hs)) {
        st = e;
      } else {
        totals.assign(2 * nn, 0);
        st = lv_prepare(s, p->rows, row_offsets, nrows, hs, &p->lv, &totals);
      }
    }
    if (!st) {
      st = take_device_error(hs);
    } else {
      // the engine failed on the host (the level engine's element bound): errors its finished
      // kernels raised on the device come first (out of bounds > map count > budget, as the row
      // walk reports them), and no flag is left behind for the stream's next call
      const int e = take_device_error(hs);
      if (e && st != FURY_ERR_DEVICE) st = e;
    }
    if (st) {
      if (p->lv) lv_free(p->lv);
      if (p->tree) tree_free(p->tree);
      delete p;
      return st;
    }
  }
  for (int i = 0; i < nn; i++) {
    if (node_entries) node_entries[i] = totals[2 * i];
    if (node_bytes) node_bytes[i] = totals[2 * i + 1];
  }
  p->totals = totals;
  *plan = p;
  return FURY_OK;
}

int fury_decode_execute(fury_decode_plan* p, fury_column* cols, int32_t arrow, void* stream) {
  if (!p) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_decode_execute: plan is null");
  GenArgs g;
  DeviceTable dt;
  hipStream_t hs = static_cast<hipStream_t>(stream);
  int st = gen_args(p->schema, cols, p->nrows, true, arrow != 0, &g, &dt, hs);
  if (st) return st;
  if (p->nrows == 0) {              // an empty batch still yields valid Arrow offsets ([0])
    const GenNode* nodes = g.tab ? reinterpret_cast<const GenNode*>(dt.host.data()) : g.node;
    for (int i = 0; i < g.nnodes && !st; i++)
      if (nodes[i].offsets)
        st = check_hip(hipMemsetAsync(nodes[i].offsets, 0, 4, hs), "hipMemsetAsync offsets");
    return st;
  }
  const GenNode* outs = g.tab ? reinterpret_cast<const GenNode*>(dt.host.data()) : g.node;
  if (p->wide) {
    VarArgs a;
    DeviceTable vdt;
    st = var_args(p->schema, cols, p->nrows, true, arrow != 0, &a, &vdt, hs);
    if (st) return st;
    return wide_execute(a, p->rows, p->offs, hs, *p->wide);
  }
  if (p->tree) return tree_execute(p->tree, outs, p->rows, p->offs, p->totals, hs);
  return lv_execute(p->lv, outs, p->rows, p->offs, hs);
}

void fury_decode_plan_destroy(fury_decode_plan* p) {
  if (!p) return;
  if (p->lv) lv_free(p->lv);
  if (p->tree) tree_free(p->tree);
  if (p->wide) wide_free(p->wide);
  if (p->owned) dev_free(p->owned, static_cast<hipStream_t>(p->owned_stream));
  if (p->owned_stream) {
    release_error_slot(static_cast<hipStream_t>(p->owned_stream));
    (void)hipStreamDestroy(static_cast<hipStream_t>(p->owned_stream));
  }
  delete p;
}

int fury_trim_workspace(int32_t device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_trim_workspace: no such device");
  int cur = 0;
  (void)hipGetDevice(&cur);
  int st = check_hip(hipSetDevice(device), "hipSetDevice");
  if (st) return st;
  release_cached(device);
  st = check_hip(hipSetDevice(cur), "hipSetDevice");
  if (!st) drain_error_quarantine();
  return st;
}

int fury_device_status(void* stream) {
  const int st = check_hip(hipStreamSynchronize(static_cast<hipStream_t>(stream)),
                           "hipStreamSynchronize");
  if (st) return st;
  return take_device_error(static_cast<hipStream_t>(stream));
}

int fury_stream_release(void* stream) {
  release_error_slot(static_cast<hipStream_t>(stream));
  return FURY_OK;
}

int fury_set_tuning(const char* key, int32_t value) {
  if (!key) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_set_tuning: key is null");
  if (std::string(key) == "lookback_help") {
    if (value < 0 || value > 1) return set_error(FURY_ERR_INVALID_ARGUMENT, "lookback_help: 0..1");
    set_lookback_help_mode(value);
    return FURY_OK;
  }
  if (std::string(key) == "unframe") {
    if (value < 0 || value > 1) return set_error(FURY_ERR_INVALID_ARGUMENT, "unframe: 0..1");
    set_unframe_mode(value);
    return FURY_OK;
  }
  if (std::string(key) == "nested_decode") {
    if (value < 1 || value > 4)
      return set_error(FURY_ERR_INVALID_ARGUMENT,
                       "nested_decode: 1 (level engine), 2 (row walk, level engine beyond it), 3 (row "
                       "walk, tile BFS beyond it) or 4 (tile BFS)");
    set_tree_mode(value);
    return FURY_OK;
  }
  if (std::string(key) == "bfs_threads") {
    if (value != 64 && value != 128 && value != 256 && value != 512)
      return set_error(FURY_ERR_INVALID_ARGUMENT, "bfs_threads: 64, 128, 256 or 512");
    set_bfs_tuning(0, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "bfs_rows") {
    if (value < 1 || value > 4096) return set_error(FURY_ERR_INVALID_ARGUMENT, "bfs_rows: 1..4096");
    set_bfs_tuning(1, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "bfs_stage" || std::string(key) == "bfs_arena") {
    if (value < 0 || value > 128 * 1024)
      return set_error(FURY_ERR_INVALID_ARGUMENT, std::string(key) + ": 0..131072 bytes (0: auto)");
    set_bfs_tuning(std::string(key) == "bfs_stage" ? 2 : 3, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "var_dec_cover") {
    if (value != 0 && (value < 50 || value > 100))
      return set_error(FURY_ERR_INVALID_ARGUMENT, "var_dec_cover: 50..100 (0 = default)");
    set_var_dec_cover(value ? value : 95);
    return FURY_OK;
  }
  if (std::string(key) == "var_wide") {
    if (value < 0 || value > 1) return set_error(FURY_ERR_INVALID_ARGUMENT, "var_wide: 0..1");
    set_var_wide_mode(value);
    return FURY_OK;
  }
  if (std::string(key) == "wide_threads" || std::string(key) == "wide_enc_threads") {
    if (value != 256 && value != 512 && value != 1024)
      return set_error(FURY_ERR_INVALID_ARGUMENT, std::string(key) + ": 256, 512 or 1024");
    set_wide_threads(std::string(key) == "wide_enc_threads", value);
    return FURY_OK;
  }
  if (std::string(key) == "var_skip") {
    if (value < 0 || value > 255) return set_error(FURY_ERR_INVALID_ARGUMENT, "var_skip: 0..255");
    set_var_skip(value);
    return FURY_OK;
  }
  if (std::string(key) == "fixed_dec") {
    if (value < 0 || value > 3) return set_error(FURY_ERR_INVALID_ARGUMENT, "fixed_dec: 0..3");
    set_fixed_dec(value);
    return FURY_OK;
  }
  if (std::string(key) == "fixed_enc") {
    if (value < 0 || value > 4) return set_error(FURY_ERR_INVALID_ARGUMENT, "fixed_enc: 0..4");
    set_fixed_enc(value);
    return FURY_OK;
  }
  if (std::string(key) == "wide_engine") {
    if (value < 0 || value > 2) return set_error(FURY_ERR_INVALID_ARGUMENT, "wide_engine: 0..2");
    g_wide_engine = value;
    return FURY_OK;
  }
  if (std::string(key) == "wide_enc_engine") {
    if (value < 0 || value > 2) return set_error(FURY_ERR_INVALID_ARGUMENT, "wide_enc_engine: 0..2");
    g_wide_enc_engine = value;
    return FURY_OK;
  }
  if (std::string(key) == "wide_walk_row") {
    if (value < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "wide_walk_row: bytes >= 0");
    g_wide_walk_row = value;
    return FURY_OK;
  }
  if (std::string(key) == "var_dec_pipe") {
    if (value < 0 || value > 2) return set_error(FURY_ERR_INVALID_ARGUMENT, "var_dec_pipe: 0..2");
    set_var_dec_pipe(value);
    return FURY_OK;
  }
  if (std::string(key) == "var_dec_rows") {
    if (value != 0 && (value < 64 || value > 512 || value % 64))
      return set_error(FURY_ERR_INVALID_ARGUMENT, "var_dec_rows: 0 or 64..512 in steps of 64");
    set_var_dec_rows(value);
    return FURY_OK;
  }
  if (std::string(key) == "walk_threads_write") {
    if (value != 64 && value != 128 && value != 256 && value != 512)
      return set_error(FURY_ERR_INVALID_ARGUMENT, "walk_threads_write: 64, 128, 256 or 512 (512: no write stage)");
    set_walk_tuning(6, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "walk_skip") {
    if (value < 0 || value > 15) return set_error(FURY_ERR_INVALID_ARGUMENT, "walk_skip: 0..15");
    set_walk_tuning(5, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "host_decode_inplace") {
    if (value < 0 || value > 1) return set_error(FURY_ERR_INVALID_ARGUMENT, "host_decode_inplace: 0..1");
    set_host_decode_inplace(value);
    return FURY_OK;
  }
  if (std::string(key) == "walk_prefetch") {
    if (value < 0 || value > 3) return set_error(FURY_ERR_INVALID_ARGUMENT, "walk_prefetch: 0..3 (bit 0 write pass, bit 1 count pass)");
    set_walk_tuning(4, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "walk_threads") {
    if (value != 64 && value != 128 && value != 256)
      return set_error(FURY_ERR_INVALID_ARGUMENT, "walk_threads: 64, 128 or 256");
    set_walk_tuning(0, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "walk_group_k" || std::string(key) == "walk_group_min") {
    if (value < 0 || value > 256) return set_error(FURY_ERR_INVALID_ARGUMENT, std::string(key) + ": 0..256");
    set_walk_tuning(std::string(key) == "walk_group_k" ? 8 : 9, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "walk_out") {
    if (value < 0 || value > 96 * 1024) return set_error(FURY_ERR_INVALID_ARGUMENT, "walk_out: 0..98304 bytes");
    set_walk_tuning(7, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "walk_stage" || std::string(key) == "walk_pool" ||
      std::string(key) == "walk_stage_write") {
    if (value < 0 || value > 96 * 1024)
      return set_error(FURY_ERR_INVALID_ARGUMENT, std::string(key) + ": 0..98304 bytes");
    set_walk_tuning(std::string(key) == "walk_stage" ? 1 : std::string(key) == "walk_pool" ? 2 : 3,
                    static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "tree_debug") {
    if (value < 0 || value > 1) return set_error(FURY_ERR_INVALID_ARGUMENT, "tree_debug: 0..1");
    return set_tree_debug(value) ? set_error(FURY_ERR_DEVICE, "tree_debug buffer") : FURY_OK;
  }
  if (std::string(key) == "rowenc_rows") {
    if (value != 128 && value != 256 && value != 512)
      return set_error(FURY_ERR_INVALID_ARGUMENT, "rowenc_rows: 128, 256 or 512");
    set_rowenc_tuning(0, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "rowenc_tile") {
    if (value < 0 || value > 256) return set_error(FURY_ERR_INVALID_ARGUMENT, "rowenc_tile: 0..256");
    set_rowenc_tuning(2, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  if (std::string(key) == "rowenc_img") {
    if (value < 1024 || value > 152 * 1024)
      return set_error(FURY_ERR_INVALID_ARGUMENT, "rowenc_img: 1024..155648 bytes");
    set_rowenc_tuning(1, static_cast<uint32_t>(value));
    return FURY_OK;
  }
  return set_error(FURY_ERR_INVALID_ARGUMENT, std::string("unknown tuning key ") + key);
}

int32_t fury_get_tuning(const char* key) {
  if (key && std::string(key) == "lookback_help") return lookback_help_mode();
  if (key && std::string(key) == "unframe") return unframe_mode();
  if (key && std::string(key) == "nested_decode") return tree_mode();
  if (key && std::string(key) == "bfs_threads") return static_cast<int32_t>(bfs_tuning(0));
  if (key && std::string(key) == "bfs_rows") return static_cast<int32_t>(bfs_tuning(1));
  if (key && std::string(key) == "bfs_stage") return static_cast<int32_t>(bfs_tuning(2));
  if (key && std::string(key) == "bfs_arena") return static_cast<int32_t>(bfs_tuning(3));
  if (key && std::string(key) == "bfs_fallbacks") return static_cast<int32_t>(bfs_tuning(4));
  if (key && std::string(key) == "rowenc_rows") return static_cast<int32_t>(rowenc_tuning(0));
  if (key && std::string(key) == "rowenc_img") return static_cast<int32_t>(rowenc_tuning(1));
  if (key && std::string(key) == "rowenc_tile") return static_cast<int32_t>(rowenc_tuning(2));
  if (key && std::string(key) == "walk_threads") return static_cast<int32_t>(walk_tuning(0));
  if (key && std::string(key) == "walk_stage") return static_cast<int32_t>(walk_tuning(1));
  if (key && std::string(key) == "walk_pool") return static_cast<int32_t>(walk_tuning(2));
  if (key && std::string(key) == "walk_stage_write") return static_cast<int32_t>(walk_tuning(3));
  if (key && std::string(key) == "walk_prefetch") return static_cast<int32_t>(walk_tuning(4));
  if (key && std::string(key) == "walk_threads_write") return static_cast<int32_t>(walk_tuning(6));
  if (key && std::string(key) == "walk_group_k") return static_cast<int32_t>(walk_tuning(8));
  if (key && std::string(key) == "walk_group_min") return static_cast<int32_t>(walk_tuning(9));
  if (key && std::string(key) == "walk_out") return static_cast<int32_t>(walk_tuning(7));
  if (key && std::string(key) == "walk_skip") return static_cast<int32_t>(walk_tuning(5));
  if (key && std::string(key) == "host_decode_inplace") return host_decode_inplace();
  if (key && std::string(key) == "var_dec_rows") return var_dec_rows();
  if (key && std::string(key) == "var_dec_pipe") return var_dec_pipe();
  if (key && std::string(key) == "wide_engine") return g_wide_engine.load();
  if (key && std::string(key) == "wide_walk_row") return g_wide_walk_row.load();
  if (key && std::string(key) == "wide_enc_engine") return g_wide_enc_engine.load();
  if (key && std::string(key) == "fixed_enc") return fixed_enc();
  if (key && std::string(key) == "fixed_dec") return fixed_dec();
  if (key && std::string(key) == "var_skip") return var_skip();
  if (key && std::string(key) == "var_wide") return var_wide_mode();
  if (key && std::string(key) == "wide_threads") return wide_threads(false);
  if (key && std::string(key) == "wide_enc_threads") return wide_threads(true);
  if (key && std::string(key) == "var_dec_cover") return var_dec_cover();
  if (key && std::string(key) == "lookback_timeouts")
    return static_cast<int32_t>(lookback_timeouts());
  if (key && std::string(key) == "unframe_walks")
    return static_cast<int32_t>(unframe_walk_count());
  if (key && std::string(key) == "host_direct")
    return static_cast<int32_t>(host_direct_count());
  if (key && std::string(key) == "err_slots") return error_slots_in_use();
  if (key && std::string(key) == "err_slots_quarantined") return error_slots_quarantined();
  if (key && std::string(key) == "thread_key_exits") return thread_key_exits();
  if (key && std::string(key) == "err_slot_last_key") return last_assigned_key_kind();
  if (key && std::string(key) == "decode_budget_errors") return static_cast<int32_t>(budget_errors());
  if (key && std::string(key) == "var_dec_rows_rejected") return var_dec_rows_rejected();
  if (key && std::string(key) == "unframe_repairs")
    return static_cast<int32_t>(unframe_repair_count());
  return -1;
}

int fury_frame_rows(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                    int64_t nrows, void* out, int64_t* frame_offsets, void* stream) {
  if (!s) return set_error(FURY_ERR_INVALID_ARGUMENT, "schema is null");
  if (s->root) return set_error(FURY_ERR_UNSUPPORTED, "row framing of a collection schema");
  if (nrows < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "nrows < 0");
  if (nrows == 0) return FURY_OK;
  if (!rows || !out) return set_error(FURY_ERR_INVALID_ARGUMENT, "rows/out is null");
  if (!s->is_fixed && !row_offsets)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "variable-length rows need row_offsets");
  return launch_frame_rows(static_cast<const uint8_t*>(rows), s->is_fixed ? nullptr : row_offsets,
                           nrows, s->fixed_size, s->schema_hash, static_cast<uint8_t*>(out),
                           frame_offsets, static_cast<hipStream_t>(stream));
}

int fury_unframe_rows(const fury_schema* s, const void* stream_bytes, int64_t stream_len,
                      int64_t nrows, void* rows_out, int64_t* row_offsets, void* stream) {
  if (!s) return set_error(FURY_ERR_INVALID_ARGUMENT, "schema is null");
  if (s->root) return set_error(FURY_ERR_UNSUPPORTED, "row framing of a collection schema");
  if (nrows < 0 || stream_len < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "negative size");
  if (nrows == 0) return FURY_OK;
  if (!stream_bytes || !rows_out || !row_offsets)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "null buffer");
  return launch_unframe_rows(static_cast<const uint8_t*>(stream_bytes), stream_len, nrows,
                             s->schema_hash, static_cast<uint8_t*>(rows_out), row_offsets,
                             static_cast<hipStream_t>(stream));
}

int fury_arrow_ipc_schema(const fury_schema* s, uint8_t* out, int64_t cap, int64_t* len) {
  if (!s || !len) return set_error(FURY_ERR_INVALID_ARGUMENT, "schema/len is null");
  std::vector<uint8_t> msg;
  const int st = ipc_schema_message(s, &msg);
  if (st) return st;
  *len = static_cast<int64_t>(msg.size());
  if (!out) return FURY_OK;
  if (cap < *len) return set_error(FURY_ERR_CAPACITY, "IPC schema message needs " +
                                                          std::to_string(*len) + " bytes");
  std::memcpy(out, msg.data(), msg.size());
  return FURY_OK;
}

int fury_arrow_ipc_record_batch(const fury_schema* s, const fury_column* columns, int64_t nrows,
                                void* out, int64_t cap, int64_t* len, void* stream) {
  if (!s || !len) return set_error(FURY_ERR_INVALID_ARGUMENT, "schema/len is null");
  if (nrows < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "nrows < 0");
  if (!columns && s->num_fields > 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "columns is null");
  return ipc_record_batch(s, columns, nrows, static_cast<uint8_t*>(out), cap, len,
                          static_cast<hipStream_t>(stream));
}

}  // extern "C"
