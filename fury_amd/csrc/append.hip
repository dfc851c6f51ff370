// append.hip — fury_arrow_append: appends one batch of device Arrow columns to another, so that
// ArrowWriter.write(batch) accumulates like the reference's write(row) loop.
//
// Reference: ArrowWriter.write(row) appends each row's values at the vectors' current rowCount
// (setSafe at rowCount, ListVector.startNewValue / endValue, StructVector setIndexDefined) and
// finish() / finishAsRecordBatch() set the value count of everything written since reset()
// (java/fury-format/src/main/java/org/apache/fury/format/vectorized/ArrowWriter.java:74-99,
// 205-225,519-540).  Here a whole batch is converted on the device (fury_rows_to_arrow /
// fury_decode_execute) and then appended to the accumulated columns: values and payloads are
// copied after the existing ones, offsets rebased on the destination's end, validity / BOOL bits
// shifted to the destination's bit position, child entries appended after the parent's.
//
// MI355X design: every buffer of every schema node becomes one "op" of a single launch (grid.y =
// op): 16-byte copies where both sides allow, one thread per destination 32-bit word for bitmaps
// (the word that also holds existing bits is merged by its one owner thread, no atomics), one
// thread per offset entry for rebasing.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

constexpr int kAppThreads = 256;

enum : int32_t { kOpCopy = 0, kOpBits = 1, kOpRebase = 2 };

struct AppendOp {
  uint8_t* dst;
  const uint8_t* src;
  int64_t n;          // copy: bytes; bits: bits; rebase: entries
  int64_t dst_at;     // bits: destination bit index; rebase: destination entry index
  int64_t base;       // rebase: added to every source offset (minus the source's first offset)
  int32_t kind;
  int32_t pad_;
};

__global__ __launch_bounds__(kAppThreads) void append_ops(const AppendOp* __restrict__ ops) {
  const AppendOp op = ops[blockIdx.y];
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * kAppThreads + threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kAppThreads;
  if (op.kind == kOpCopy) {
    const bool v16 = ((reinterpret_cast<uintptr_t>(op.dst) | reinterpret_cast<uintptr_t>(op.src)) & 15) == 0;
    using v4 = __attribute__((ext_vector_type(4))) uint32_t;
    const int64_t n16 = v16 ? op.n >> 4 : 0;
    for (int64_t i = tid; i < n16; i += stride)
      __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const v4*>(op.src) + i),
                                  reinterpret_cast<v4*>(op.dst) + i);
    for (int64_t i = 16 * n16 + tid; i < op.n; i += stride) op.dst[i] = op.src[i];
    return;
  }
  if (op.kind == kOpRebase) {
    // dst[at + 1 + i] = src[1 + i] - src[0] + base; dst[at] is the destination's end already
    const int32_t* s = reinterpret_cast<const int32_t*>(op.src);
    int32_t* d = reinterpret_cast<int32_t*>(op.dst);
    const int64_t s0 = s[0];
    for (int64_t i = tid; i < op.n; i += stride)
      d[op.dst_at + 1 + i] = static_cast<int32_t>(s[1 + i] - s0 + op.base);
    if (tid == 0 && op.dst_at == 0) d[0] = static_cast<int32_t>(op.base);
    return;
  }
  // bits: destination bits [at, at + n) <- source bits [0, n); one thread per destination word
  const uint32_t* s = reinterpret_cast<const uint32_t*>(op.src);
  uint32_t* d = reinterpret_cast<uint32_t*>(op.dst);
  const int64_t b0 = op.dst_at, b1 = op.dst_at + op.n;
  const int64_t w0 = b0 >> 5, w1 = (b1 + 31) >> 5;
  const int64_t nsw = (op.n + 31) >> 5;                         // source words
  for (int64_t w = w0 + tid; w < w1; w += stride) {
    const int64_t i0 = 32 * w - b0;                             // source bit of dst bit 32 w
    uint32_t x;
    if (i0 < 0) {
      x = s[0] << (-i0);
    } else {
      const int64_t q = i0 >> 5;
      const int sh = static_cast<int>(i0 & 31);
      const uint32_t lo = s[q];
      const uint32_t hi = (sh && q + 1 < nsw) ? s[q + 1] : 0u;
      x = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
    }
    uint32_t keep = 0;                                          // existing destination bits
    if (w == w0 && (b0 & 31)) keep = (1u << (b0 & 31)) - 1;
    uint32_t m = ~keep;
    if (w == w1 - 1 && (b1 & 31)) m &= (1u << (b1 & 31)) - 1;  // bits past the end: 0
    d[w] = (keep ? (d[w] & keep) : 0u) | (x & m);
  }
}

int read_i32(const int32_t* p, int64_t i, hipStream_t hs, int64_t* out) {
  int32_t v = 0;
  int st = check_hip(hipMemcpyAsync(&v, p + i, 4, hipMemcpyDeviceToHost, hs), "hipMemcpyAsync");
  if (!st) st = check_hip(hipStreamSynchronize(hs), "hipStreamSynchronize");
  *out = v;
  return st;
}

int width_of(int32_t t) {
  switch (t) {
    case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    case FURY_TYPE_DECIMAL: return 16;
    default: return 0;
  }
}

}  // namespace
}  // namespace fury

using namespace fury;

extern "C" int fury_arrow_append(const fury_schema* s, fury_column* dst, int64_t dst_rows,
                                 const fury_column* src, int64_t src_rows, void* stream) {
  if (!s) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_arrow_append: schema is null");
  if (dst_rows < 0 || src_rows < 0)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_arrow_append: negative row count");
  if (src_rows == 0) return FURY_OK;
  if (!dst || !src) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_arrow_append: columns is null");
  hipStream_t hs = static_cast<hipStream_t>(stream);
  if (int e = take_device_error(hs)) return e;
  const int nn = static_cast<int>(s->nodes.size());
  std::vector<const fury_column*> dc(nn, nullptr), sc(nn, nullptr);
  std::vector<int64_t> dm(nn, 0), sm(nn, 0);      // entries per node: destination, source
  for (int k = 0; k < s->num_fields; k++) {
    dc[k] = &dst[k];
    sc[k] = &src[k];
    dm[k] = dst_rows;
    sm[k] = src_rows;
  }
  std::vector<AppendOp> ops;
  auto add = [&](int32_t kind, void* d, const void* sp, int64_t n, int64_t at, int64_t base) {
    if (n <= 0) return;
    AppendOp o{};
    o.kind = kind;
    o.dst = static_cast<uint8_t*>(d);
    o.src = static_cast<const uint8_t*>(sp);
    o.n = n;
    o.dst_at = at;
    o.base = base;
    ops.push_back(o);
  };
  int st = FURY_OK;
  for (int i = 0; i < nn && !st; i++) {               // breadth-first: parents before children
    const GenTpl& t = s->nodes[i];
    const fury_column* d = dc[i];
    const fury_column* c = sc[i];
    const std::string who = "node " + std::to_string(i);
    if (!d || !c) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": missing column");
    const int64_t m0 = dm[i], m = sm[i];
    if (t.num_children > 0) {
      if (!d->child || !c->child) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": child columns missing");
      for (int j = 0; j < t.num_children; j++) {
        dc[t.first_child + j] = &d->child[j];
        sc[t.first_child + j] = &c->child[j];
      }
    }
    if ((d->validity != nullptr) != (c->validity != nullptr))
      return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": validity on one side only");
    if (d->validity) add(kOpBits, d->validity, c->validity, m, m0, 0);
    const int32_t ty = t.type_id;
    if (ty == FURY_TYPE_STRUCT) {
      for (int j = 0; j < t.num_children; j++) {
        dm[t.first_child + j] = m0;
        sm[t.first_child + j] = m;
      }
      continue;
    }
    if (ty == FURY_TYPE_BOOL) {
      if (!d->values || !c->values) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": values is null");
      add(kOpBits, d->values, c->values, m, m0, 0);
      continue;
    }
    const int w = width_of(ty);
    if (w > 0) {
      if (!d->values || !c->values) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": values is null");
      if (d->capacity > 0 && (m0 + m) * w > d->capacity)
        return set_error(FURY_ERR_CAPACITY, who + ": destination values need " +
                                                std::to_string((m0 + m) * w) + " bytes");
      add(kOpCopy, static_cast<uint8_t*>(d->values) + m0 * w, c->values, m * w, 0, 0);
      continue;
    }
    // STRING / BINARY / LIST / MAP: offsets, then payload or child entries
    if (!d->offsets || !c->offsets) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": offsets is null");
    int64_t dend = 0, s0 = 0, s1 = 0;
    if ((st = read_i32(d->offsets, m0, hs, &dend)) || (st = read_i32(c->offsets, 0, hs, &s0)) ||
        (st = read_i32(c->offsets, m, hs, &s1)))
      return st;
    if (m0 == 0) dend = 0;
    const int64_t cnt = s1 - s0;
    if (cnt < 0 || dend < 0) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": offsets decrease");
    if (dend + cnt > INT32_MAX)
      return set_error(FURY_ERR_CAPACITY, who + ": more than 2^31 - 1 entries / bytes (int32 offsets)");
    add(kOpRebase, d->offsets, c->offsets, m, m0, dend);
    if (ty == FURY_TYPE_STRING || ty == FURY_TYPE_BINARY) {
      if (cnt > 0 && (!d->values || !c->values))
        return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": payload is null");
      if (d->capacity > 0 && dend + cnt > d->capacity)
        return set_error(FURY_ERR_CAPACITY, who + ": destination payload needs " +
                                                std::to_string(dend + cnt) + " bytes");
      add(kOpCopy, static_cast<uint8_t*>(d->values) + dend, static_cast<const uint8_t*>(c->values) + s0,
          cnt, 0, 0);
      continue;
    }
    if (s0 != 0) return set_error(FURY_ERR_INVALID_ARGUMENT, who + ": source child entries must start at 0");
    for (int j = 0; j < t.num_children; j++) {
      dm[t.first_child + j] = dend;
      sm[t.first_child + j] = cnt;
    }
  }
  if (ops.empty()) return FURY_OK;
  int64_t maxw = 0;                                     // threads the largest op can use
  for (const AppendOp& o : ops) {
    const int64_t work = o.kind == kOpCopy ? (o.n + 15) / 16 : o.kind == kOpBits ? (o.n + 31) / 32 + 1 : o.n;
    maxw = std::max(maxw, work);
  }
  DeviceTable dt;
  if ((st = upload_table(ops.data(), ops.size() * sizeof(AppendOp), hs, &dt))) return st;
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>((maxw + kAppThreads - 1) / kAppThreads, 1), 4096);
  hipLaunchKernelGGL(append_ops, dim3(static_cast<unsigned>(blocks), static_cast<unsigned>(ops.size())),
                     dim3(kAppThreads), 0, hs, static_cast<const AppendOp*>(dt.dev));
  return check_hip(hipGetLastError(), "append launch");
}
