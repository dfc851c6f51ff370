// ipc.hip — Arrow IPC encapsulated messages of device-decoded columns: the device-side
// replacement of ArrowUtils.serializeRecordBatch (FMT/vectorized/ArrowUtils.java:63-72) and of
// ArrowSerializers' stream writers (FMT/vectorized/ArrowSerializers.java:128-167), which hand the
// columns ArrowWriter produced (ArrowWriter.java:89-99) to Arrow's MessageSerializer.
//
// A message is [0xFFFFFFFF][int32 metadata size][flatbuffer Message][padding][body].  The
// metadata is built here on the host (a small back-to-front flatbuffer builder over Arrow's
// Message.fbs / Schema.fbs tables); the body — every Arrow buffer of the batch in pre-order,
// each padded to 64 bytes — is gathered on the device by one kernel, which also counts the
// nulls of each validity buffer and subtracts them in place from the FieldNode.null_count the
// host wrote into the metadata (initialised to the node length), so no host round trip is
// needed for null counts.  Only the lengths of variable-size buffers (offsets[n] of
// STRING/BINARY/LIST/MAP columns) are read back to the host to lay the body out.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"

namespace fury {

namespace {

// ---- minimal flatbuffer builder (back to front, as the reference flatbuffers builder) --------
class FbBuilder {
 public:
  FbBuilder() : buf_(1 << 12), head_(buf_.size()) {}

  int64_t size() const { return static_cast<int64_t>(buf_.size() - head_); }

  void pad(int64_t n) {
    grow(n);
    for (int64_t i = 0; i < n; i++) buf_[--head_] = 0;
  }
  // Pads so that after writing `extra` more bytes the size is a multiple of `align`.
  void prep(int align, int64_t extra) {
    if (align > minalign_) minalign_ = align;
    const int64_t p = (~(size() + extra) + 1) & (align - 1);
    pad(p);
  }
  template <typename T>
  void push(T v) {
    grow(sizeof(T));
    head_ -= sizeof(T);
    std::memcpy(&buf_[head_], &v, sizeof(T));
  }
  template <typename T>
  void put(T v) {          // aligned scalar
    prep(sizeof(T), 0);
    push(v);
  }
  // uoffset to an object created earlier (its offset = size() right after it was written).
  void put_ref(int64_t target) {
    prep(4, 4);
    push(static_cast<uint32_t>(size() + 4 - target));
  }

  // -- tables --
  void start_table() {
    fields_.clear();
    table_start_ = size();
  }
  template <typename T>
  void field(int id, T v) {
    put(v);
    fields_.push_back({id, size()});
  }
  void field_ref(int id, int64_t target) {
    put_ref(target);
    fields_.push_back({id, size()});
  }
  int64_t end_table() {
    put<int32_t>(0);                   // soffset to the vtable, patched below
    const int64_t obj = size();
    int nslots = 0;
    for (auto& f : fields_) nslots = f.first + 1 > nslots ? f.first + 1 : nslots;
    std::vector<uint16_t> slot(nslots, 0);
    for (auto& f : fields_) slot[f.first] = static_cast<uint16_t>(obj - f.second);
    for (int i = nslots - 1; i >= 0; i--) push<uint16_t>(slot[i]);
    push<uint16_t>(static_cast<uint16_t>(obj - table_start_));
    push<uint16_t>(static_cast<uint16_t>(4 + 2 * nslots));
    const int64_t vt = size();
    const int32_t soff = static_cast<int32_t>(vt - obj);   // table address - vtable address
    std::memcpy(&buf_[buf_.size() - obj], &soff, 4);
    return obj;
  }

  // -- vectors --
  int64_t vector_of_refs(const std::vector<int64_t>& refs) {
    prep(4, 4 * static_cast<int64_t>(refs.size()));
    for (size_t i = refs.size(); i-- > 0;) put_ref(refs[i]);
    push(static_cast<uint32_t>(refs.size()));
    return size();
  }
  // Vector of 16-byte structs of two int64 {a, b}; *b_pos receives each element's b field
  // offset-from-end (final address = total - that) so it can be patched later.
  int64_t vector_of_pairs(const std::vector<std::pair<int64_t, int64_t>>& v,
                          std::vector<int64_t>* b_pos) {
    prep(8, 16 * static_cast<int64_t>(v.size()));      // elements 8-aligned; count follows
    if (b_pos) b_pos->assign(v.size(), 0);
    for (size_t i = v.size(); i-- > 0;) {
      push(v[i].second);
      if (b_pos) (*b_pos)[i] = size();
      push(v[i].first);
    }
    push(static_cast<uint32_t>(v.size()));
    return size();
  }
  int64_t string(const std::string& s) {
    prep(4, static_cast<int64_t>(s.size()) + 1);
    push<uint8_t>(0);
    grow(s.size());
    head_ -= s.size();
    if (!s.empty()) std::memcpy(&buf_[head_], s.data(), s.size());
    push(static_cast<uint32_t>(s.size()));
    return size();
  }
  int64_t empty_table() {
    start_table();
    return end_table();
  }

  // Root offset + final alignment; returns the finished bytes.
  std::vector<uint8_t> finish(int64_t root) {
    prep(minalign_ < 8 ? 8 : minalign_, 4);
    put_ref(root);
    return std::vector<uint8_t>(buf_.begin() + head_, buf_.end());
  }

 private:
  void grow(int64_t n) {
    if (static_cast<int64_t>(head_) >= n) return;
    const size_t used = buf_.size() - head_;
    size_t cap = buf_.size() * 2;
    while (cap - used < used + static_cast<size_t>(n)) cap *= 2;
    std::vector<uint8_t> nb(cap);
    std::memcpy(&nb[cap - used], &buf_[head_], used);
    buf_.swap(nb);
    head_ = cap - used;
  }

  std::vector<uint8_t> buf_;
  size_t head_;
  int minalign_ = 1;
  int64_t table_start_ = 0;
  std::vector<std::pair<int, int64_t>> fields_;
};

// Arrow format enums (format/Schema.fbs, format/Message.fbs).
enum : uint8_t { kTypeInt = 2, kTypeFloat = 3, kTypeBinary = 4, kTypeUtf8 = 5, kTypeBool = 6,
                 kTypeDecimal = 7, kTypeDate = 8, kTypeTimestamp = 10, kTypeList = 12,
                 kTypeStruct = 13, kTypeMap = 17 };
enum : uint8_t { kHeaderSchema = 1, kHeaderRecordBatch = 3 };
constexpr int16_t kMetadataV5 = 4;

// The Arrow type table of a field (ArrowType as TypeInference/DataTypes build it).
int64_t type_table(FbBuilder& b, int32_t type_id, uint8_t* tag) {
  switch (type_id) {
    case FURY_TYPE_BOOL: *tag = kTypeBool; return b.empty_table();
    case FURY_TYPE_INT8: case FURY_TYPE_INT16: case FURY_TYPE_INT32: case FURY_TYPE_INT64: {
      const int bits = type_id == FURY_TYPE_INT8 ? 8 : type_id == FURY_TYPE_INT16 ? 16
                       : type_id == FURY_TYPE_INT32 ? 32 : 64;
      *tag = kTypeInt;
      b.start_table();
      b.field<int32_t>(0, bits);
      b.field<uint8_t>(1, 1);            // is_signed
      return b.end_table();
    }
    case FURY_TYPE_FLOAT32: case FURY_TYPE_FLOAT64:
      *tag = kTypeFloat;
      b.start_table();
      b.field<int16_t>(0, type_id == FURY_TYPE_FLOAT32 ? 1 : 2);   // SINGLE / DOUBLE
      return b.end_table();
    case FURY_TYPE_STRING: *tag = kTypeUtf8; return b.empty_table();
    case FURY_TYPE_BINARY: *tag = kTypeBinary; return b.empty_table();
    case FURY_TYPE_DATE32:
      *tag = kTypeDate;
      b.start_table();
      b.field<int16_t>(0, 0);            // DateUnit.DAY
      return b.end_table();
    case FURY_TYPE_TIMESTAMP:
      *tag = kTypeTimestamp;
      b.start_table();
      b.field<int16_t>(0, 2);            // TimeUnit.MICROSECOND, no timezone
      return b.end_table();
    case FURY_TYPE_DECIMAL:              // DataTypes.decimal(): MAX_PRECISION 38, MAX_SCALE 18
      *tag = kTypeDecimal;
      b.start_table();
      b.field<int32_t>(0, 38);
      b.field<int32_t>(1, 18);
      b.field<int32_t>(2, 128);
      return b.end_table();
    case FURY_TYPE_LIST: *tag = kTypeList; return b.empty_table();
    case FURY_TYPE_STRUCT: *tag = kTypeStruct; return b.empty_table();
    case FURY_TYPE_MAP:
      *tag = kTypeMap;
      b.start_table();
      b.field<uint8_t>(0, 0);            // keysSorted = false
      return b.end_table();
    default: *tag = 0; return -1;
  }
}

int64_t field_table(FbBuilder& b, const std::string& name, int32_t type_id, bool nullable,
                    const std::vector<const OwnedField*>& kids, bool map_entries);

int64_t field_of(FbBuilder& b, const OwnedField& f) {
  std::vector<const OwnedField*> kids;
  for (const auto& c : f.children) kids.push_back(&c);
  return field_table(b, f.name, f.type_id, f.nullable != 0, kids, f.type_id == FURY_TYPE_MAP);
}

// Field table.  A MAP's children (key, value) sit under Arrow's non-null "entries" struct, the
// key being non-null (MapVector / DataTypes.mapField).
int64_t field_table(FbBuilder& b, const std::string& name, int32_t type_id, bool nullable,
                    const std::vector<const OwnedField*>& kids, bool map_entries) {
  std::vector<int64_t> child_refs;
  if (map_entries) {
    std::vector<int64_t> kv;
    for (size_t i = 0; i < kids.size(); i++) {
      std::vector<const OwnedField*> gk;
      for (const auto& c : kids[i]->children) gk.push_back(&c);
      kv.push_back(field_table(b, kids[i]->name, kids[i]->type_id,
                               i == 0 ? false : kids[i]->nullable != 0, gk,
                               kids[i]->type_id == FURY_TYPE_MAP));
    }
    const int64_t kvv = b.vector_of_refs(kv);
    const int64_t en = b.string("entries");
    uint8_t tag;
    const int64_t st = type_table(b, FURY_TYPE_STRUCT, &tag);
    b.start_table();
    b.field_ref(0, en);
    b.field<uint8_t>(1, 0);
    b.field<uint8_t>(2, tag);
    b.field_ref(3, st);
    b.field_ref(5, kvv);
    child_refs.push_back(b.end_table());
  } else {
    for (const OwnedField* k : kids) child_refs.push_back(field_of(b, *k));
  }
  const int64_t cv = b.vector_of_refs(child_refs);
  const int64_t nm = b.string(name);
  uint8_t tag;
  const int64_t ty = type_table(b, type_id, &tag);
  b.start_table();
  b.field_ref(0, nm);
  b.field<uint8_t>(1, nullable ? 1 : 0);
  b.field<uint8_t>(2, tag);
  b.field_ref(3, ty);
  b.field_ref(5, cv);
  return b.end_table();
}

std::vector<uint8_t> message(FbBuilder& b, uint8_t header_type, int64_t header, int64_t body_len) {
  b.start_table();
  b.field<int64_t>(3, body_len);
  b.field_ref(2, header);
  b.field<int16_t>(0, kMetadataV5);
  b.field<uint8_t>(1, header_type);
  return b.finish(b.end_table());
}

// Encapsulation: continuation marker, metadata size (flatbuffer + padding, so that the body
// starts `align`-aligned from the message start).
std::vector<uint8_t> encapsulate(const std::vector<uint8_t>& fb, int align, int64_t* fb_at) {
  int64_t meta = static_cast<int64_t>(fb.size());
  meta += (align - (8 + meta) % align) % align;
  std::vector<uint8_t> out(8 + meta, 0);
  const uint32_t cont = 0xFFFFFFFFu;
  const int32_t m = static_cast<int32_t>(meta);
  std::memcpy(&out[0], &cont, 4);
  std::memcpy(&out[4], &m, 4);
  std::memcpy(&out[8], fb.data(), fb.size());
  *fb_at = 8;
  return out;
}

// ---- record batch layout -----------------------------------------------------------------------
constexpr int64_t kBodyAlign = 64;
inline int64_t pad64(int64_t x) { return (x + kBodyAlign - 1) & ~(kBodyAlign - 1); }

struct IpcCopy {              // one body buffer
  const uint8_t* src;         // device source (NULL: zero fill)
  int64_t dst;                // offset in the message
  int64_t bytes;              // source bytes
  int64_t padded;             // bytes written (bytes rounded up to 64, zero tail)
  int64_t bits;               // > 0: validity bitmap of `bits` entries — count its set bits
  int64_t nc_at;              // message offset of the FieldNode.null_count to decrement
};

struct Layout {
  std::vector<std::pair<int64_t, int64_t>> nodes;    // FieldNode {length, null_count}
  std::vector<std::pair<int64_t, int64_t>> buffers;  // Buffer {offset, length} (body-relative)
  std::vector<IpcCopy> copies;
  std::vector<int> node_of_copy;                     // FieldNode index of a validity copy, or -1
  int64_t body = 0;
};

int read_offset(const int32_t* dev_offsets, int64_t i, int64_t* out) {
  int32_t v = 0;
  const int st = check_hip(hipMemcpy(&v, dev_offsets + i, 4, hipMemcpyDeviceToHost),
                           "hipMemcpy offsets");
  *out = v;
  return st;
}

void add_buffer(Layout& L, const void* src, int64_t bytes, int64_t bits, int node) {
  const int64_t at = L.body;
  L.buffers.push_back({at, bytes});
  if (bytes > 0) {
    L.copies.push_back({static_cast<const uint8_t*>(src), at, bytes, pad64(bytes), bits, -1});
    L.node_of_copy.push_back(node);
  }
  L.body += pad64(bytes);
}

int layout_column(Layout& L, int32_t type_id, const OwnedField* f, const fury_column& c,
                  int64_t len) {
  const int node = static_cast<int>(L.nodes.size());
  L.nodes.push_back({len, len});               // null_count = len - popcount(valid), on device
  const bool has_valid = c.validity != nullptr && len > 0;
  if (!has_valid) L.nodes[node].second = 0;
  add_buffer(L, c.validity, has_valid ? (len + 7) / 8 : 0, has_valid ? len : 0, node);
  switch (type_id) {
    case FURY_TYPE_BOOL:
      add_buffer(L, c.values, (len + 7) / 8, 0, -1);
      return FURY_OK;
    case FURY_TYPE_INT8: case FURY_TYPE_INT16: case FURY_TYPE_INT32: case FURY_TYPE_INT64:
    case FURY_TYPE_FLOAT32: case FURY_TYPE_FLOAT64: case FURY_TYPE_DATE32: case FURY_TYPE_TIMESTAMP:
    case FURY_TYPE_DECIMAL: {
      const int w = type_id == FURY_TYPE_DECIMAL ? 16 : type_width_of(type_id);
      add_buffer(L, c.values, len * w, 0, -1);
      return FURY_OK;
    }
    case FURY_TYPE_STRING: case FURY_TYPE_BINARY: {
      if (!c.offsets && len > 0) return set_error(FURY_ERR_INVALID_ARGUMENT, "column offsets missing");
      int64_t total = 0;
      if (len > 0) {
        const int st = read_offset(c.offsets, len, &total);
        if (st) return st;
      }
      add_buffer(L, c.offsets, len > 0 ? (len + 1) * 4 : 0, 0, -1);
      add_buffer(L, c.values, total, 0, -1);
      return FURY_OK;
    }
    case FURY_TYPE_LIST: case FURY_TYPE_MAP: {
      if ((!c.offsets || !c.child) && len > 0)
        return set_error(FURY_ERR_INVALID_ARGUMENT, "list/map column offsets/child missing");
      int64_t m = 0;
      if (len > 0) {
        const int st = read_offset(c.offsets, len, &m);
        if (st) return st;
      }
      add_buffer(L, c.offsets, len > 0 ? (len + 1) * 4 : 0, 0, -1);
      if (type_id == FURY_TYPE_LIST) {
        static const fury_column empty{};
        return layout_column(L, f->children[0].type_id, &f->children[0],
                             c.child ? c.child[0] : empty, m);
      }
      // MAP: the non-null "entries" struct node (no validity buffer), then keys and values
      L.nodes.push_back({m, 0});
      add_buffer(L, nullptr, 0, 0, -1);
      static const fury_column empty{};
      for (int k = 0; k < 2; k++) {
        const int st = layout_column(L, f->children[k].type_id, &f->children[k],
                                     c.child ? c.child[k] : empty, m);
        if (st) return st;
      }
      return FURY_OK;
    }
    case FURY_TYPE_STRUCT: {
      static const fury_column empty{};
      for (size_t k = 0; k < f->children.size(); k++) {
        const int st = layout_column(L, f->children[k].type_id, &f->children[k],
                                     c.child ? c.child[k] : empty, len);
        if (st) return st;
      }
      return FURY_OK;
    }
    default:
      return set_error(FURY_ERR_UNSUPPORTED, "no Arrow IPC layout for type " +
                                                 std::to_string(type_id));
  }
}

// ---- device body gather ------------------------------------------------------------------------
constexpr int kThreads = 256;
constexpr int64_t kChunk = 64 * 1024;     // body bytes per workgroup

struct IpcChunk {
  int32_t copy;
  int32_t pad_;
  int64_t off;                             // chunk start within the copy
};

// One workgroup per 64-KB chunk of one body buffer: 16-B copies (source and destination are
// 16-byte aligned: device allocations, 64-byte body padding), byte copies for a ragged tail,
// zeros up to the 64-byte padding; a validity chunk also counts its set bits below `bits` and
// subtracts them from its FieldNode.null_count (which the host set to the node length).
__global__ __launch_bounds__(kThreads) void ipc_gather(const IpcCopy* __restrict__ copies,
                                                       const IpcChunk* __restrict__ chunks,
                                                       uint8_t* __restrict__ out) {
  const IpcChunk ch = chunks[blockIdx.x];
  const IpcCopy cp = copies[ch.copy];
  const int64_t end = min(cp.padded, ch.off + kChunk);
  const bool aligned = ((reinterpret_cast<uintptr_t>(cp.src) | static_cast<uintptr_t>(cp.dst)) & 15) == 0;
  uint8_t* dst = out + cp.dst;
  int64_t ones = 0;
  for (int64_t p = ch.off + 16 * threadIdx.x; p < end; p += 16 * kThreads) {
    using v4u = __attribute__((ext_vector_type(4))) uint32_t;
    v4u v = {0u, 0u, 0u, 0u};
    if (cp.src && aligned && p + 16 <= cp.bytes) {
      v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(cp.src + p));
    } else if (cp.src) {
      uint8_t t[16];
#pragma unroll
      for (int i = 0; i < 16; i++) t[i] = p + i < cp.bytes ? cp.src[p + i] : 0;
      std::memcpy(&v, t, 16);
    }
    if (cp.bits > 0) {                     // set bits of entries [0, bits) in this piece
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int64_t b0 = 8 * (p + 4 * i);
        uint32_t x = w[i];
        if (b0 >= cp.bits) x = 0;
        else if (b0 + 32 > cp.bits) x &= (1u << (cp.bits - b0)) - 1u;
        ones += __popc(x);
      }
    }
    if (aligned) {
      __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(dst + p));
    } else {
      uint8_t t[16];
      std::memcpy(t, &v, 16);
      for (int i = 0; i < 16 && p + i < end; i++) dst[p + i] = t[i];
    }
  }
  if (cp.bits > 0) {
    __shared__ int64_t part[kThreads / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ones += __shfl_xor(ones, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = ones;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t s = 0;
      for (int w = 0; w < kThreads / 64; w++) s += part[w];
      if (s) atomicAdd(reinterpret_cast<unsigned long long*>(out + cp.nc_at),
                       static_cast<unsigned long long>(-s));
    }
  }
}

}  // namespace

int type_width_of(int32_t type_id) {
  switch (type_id) {
    case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: case FURY_TYPE_FLOAT32: case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT64: case FURY_TYPE_TIMESTAMP: return 8;
    case FURY_TYPE_DECIMAL: return 16;
    default: return 0;
  }
}

int ipc_schema_message(const fury_schema* s, std::vector<uint8_t>* out) {
  FbBuilder b;
  std::vector<int64_t> fields;
  for (const auto& f : s->fields) fields.push_back(field_of(b, f));
  const int64_t fv = b.vector_of_refs(fields);
  b.start_table();
  b.field_ref(1, fv);
  b.field<int16_t>(0, 0);                  // Endianness.Little
  const int64_t schema = b.end_table();
  int64_t at = 0;
  *out = encapsulate(message(b, kHeaderSchema, schema, 0), 8, &at);
  return FURY_OK;
}

int ipc_record_batch(const fury_schema* s, const fury_column* cols, int64_t n, uint8_t* out,
                     int64_t cap, int64_t* len, hipStream_t stream) {
  Layout L;
  for (size_t i = 0; i < s->fields.size(); i++) {
    const int st = layout_column(L, s->fields[i].type_id, &s->fields[i], cols[i], n);
    if (st) return st;
  }
  FbBuilder b;
  std::vector<int64_t> nc_pos;
  const int64_t bufv = b.vector_of_pairs(L.buffers, nullptr);
  const int64_t nodev = b.vector_of_pairs(L.nodes, &nc_pos);
  b.start_table();
  b.field<int64_t>(0, n);
  b.field_ref(2, bufv);
  b.field_ref(1, nodev);
  const int64_t rb = b.end_table();
  const std::vector<uint8_t> fb = message(b, kHeaderRecordBatch, rb, L.body);
  int64_t fb_at = 0;
  const std::vector<uint8_t> meta = encapsulate(fb, static_cast<int>(kBodyAlign), &fb_at);
  const int64_t body_at = static_cast<int64_t>(meta.size());
  *len = body_at + L.body;
  if (!out) return FURY_OK;
  if (cap < *len) return set_error(FURY_ERR_CAPACITY, "IPC record batch needs " +
                                                          std::to_string(*len) + " bytes");
  if (reinterpret_cast<uintptr_t>(out) & 15)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "IPC output must be 16-byte aligned");
  const int64_t fb_total = static_cast<int64_t>(fb.size());
  std::vector<IpcCopy> copies = L.copies;
  std::vector<IpcChunk> chunks;
  for (size_t k = 0; k < copies.size(); k++) {
    copies[k].dst += body_at;
    const int node = L.node_of_copy[k];
    // null_count of FieldNode `node`: its offset-from-end in the flatbuffer -> message offset
    copies[k].nc_at = node >= 0 ? fb_at + fb_total - nc_pos[node] : -1;
    for (int64_t o = 0; o < copies[k].padded; o += kChunk)
      chunks.push_back({static_cast<int32_t>(k), 0, o});
  }
  // table upload + metadata, then the gather; synchronous (the host vectors die on return)
  const size_t tb = copies.size() * sizeof(IpcCopy), cb = chunks.size() * sizeof(IpcChunk);
  uint8_t* tab = nullptr;
  int st = FURY_OK;
  if (!chunks.empty()) {
    st = dev_alloc(tb + cb, stream, reinterpret_cast<void**>(&tab));
    if (st) return st;
    (void)hipMemcpyAsync(tab, copies.data(), tb, hipMemcpyHostToDevice, stream);
    (void)hipMemcpyAsync(tab + tb, chunks.data(), cb, hipMemcpyHostToDevice, stream);
  }
  st = check_hip(hipMemcpyAsync(out, meta.data(), meta.size(), hipMemcpyHostToDevice, stream),
                 "hipMemcpyAsync metadata");
  if (!st && !chunks.empty()) {
    hipLaunchKernelGGL(ipc_gather, dim3(static_cast<unsigned>(chunks.size())), dim3(kThreads), 0,
                       stream, reinterpret_cast<const IpcCopy*>(tab),
                       reinterpret_cast<const IpcChunk*>(tab + tb), out);
    st = check_hip(hipGetLastError(), "ipc gather launch");
  }
  if (tab) dev_free(tab, stream);
  const int st2 = check_hip(hipStreamSynchronize(stream), "ipc sync");
  return st ? st : st2;
}

}  // namespace fury
