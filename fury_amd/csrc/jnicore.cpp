// jnicore.cpp — the JNI-free core of GpuRowEncoder's native methods
// (java/src/main/java/org/apache/fury/format/encoder/GpuRowEncoder.java): the descriptor arrays
// the Java side builds (flattenField's names + {typeId, nullable, numChildren} per node, describe()'s
// {values, validity, offsets, capacity, numChildren} per node, both in pre-order) are decoded into
// fury_field / fury_column trees HERE, in the tested library, so fury_row_jni.cc only marshals
// Java arrays and maps a status to an exception class (fury_jni_exception_class).
//
// Reference surface replaced: Encoders.bean(...) / RowEncoder encode + decode over batches
// (java/fury-format/src/main/java/org/apache/fury/format/encoder/Encoders.java:60-219,
// RowEncoder.java:26-32); exceptions as Encoders / MemoryBuffer throw them.
#include <cstdint>
#include <string>
#include <vector>

#include "internal.h"

namespace fury {
namespace {

// Pre-order names + {typeId, nullable, numChildren} x nodes -> fury_field tree.
struct JField {
  std::vector<std::vector<fury_field>> kids;     // children arrays (reserved: never move)
  int build(const char* const* names, const int32_t* meta, int32_t nodes, int32_t* at,
            fury_field* out) {
    const int32_t i = (*at)++;
    if (i >= nodes) return set_error(FURY_ERR_INVALID_ARGUMENT, "field descriptor: too few nodes");
    if (!names[i]) return set_error(FURY_ERR_INVALID_ARGUMENT, "field descriptor: null name");
    out->name = names[i];
    out->type_id = meta[3 * i];
    out->nullable = meta[3 * i + 1];
    out->num_children = meta[3 * i + 2];
    out->children = nullptr;
    if (out->num_children < 0 || out->num_children > nodes)
      return set_error(FURY_ERR_INVALID_ARGUMENT, "field descriptor: bad child count");
    if (out->num_children > 0) {
      const size_t slot = kids.size();
      kids.emplace_back(static_cast<size_t>(out->num_children));
      for (int c = 0; c < out->num_children; c++)
        if (int st = build(names, meta, nodes, at, &kids[slot][c])) return st;
      out->children = kids[slot].data();
    }
    return FURY_OK;
  }
};

// Pre-order {values, validity, offsets, capacity, numChildren} x nodes -> fury_column tree over
// the schema's node tree (a descriptor whose child counts differ from the schema is rejected).
struct JColumns {
  std::vector<std::vector<fury_column>> kids;
  std::vector<fury_column> top;
  int build_one(const fury_schema* s, int node, const int64_t* d, int64_t n, int64_t* at,
                fury_column* out) {
    if (*at + 5 > n) return set_error(FURY_ERR_INVALID_ARGUMENT, "column descriptor: too short");
    const int64_t* e = d + *at;
    *at += 5;
    out->values = reinterpret_cast<void*>(e[0]);
    out->validity = reinterpret_cast<uint8_t*>(e[1]);
    out->offsets = reinterpret_cast<int32_t*>(e[2]);
    out->capacity = e[3];
    out->child = nullptr;
    const GenTpl& t = s->nodes[node];
    if (e[4] != t.num_children)
      return set_error(FURY_ERR_INVALID_ARGUMENT,
                       "column descriptor: node " + std::to_string(node) + " has " +
                           std::to_string(e[4]) + " children, the schema " +
                           std::to_string(t.num_children));
    if (t.num_children > 0) {
      const size_t slot = kids.size();
      kids.emplace_back(static_cast<size_t>(t.num_children));
      for (int c = 0; c < t.num_children; c++)
        if (int st = build_one(s, t.first_child + c, d, n, at, &kids[slot][c])) return st;
      out->child = kids[slot].data();
    }
    return FURY_OK;
  }
  int build(const fury_schema* s, const int64_t* d, int64_t n) {
    if (!s) return set_error(FURY_ERR_INVALID_ARGUMENT, "schema is null");
    if (n > 0 && !d) return set_error(FURY_ERR_INVALID_ARGUMENT, "column descriptor is null");
    kids.reserve(static_cast<size_t>(s->nodes.size()) + 1);
    top.assign(static_cast<size_t>(s->num_fields), fury_column{});
    int64_t at = 0;
    for (int i = 0; i < s->num_fields; i++)
      if (int st = build_one(s, i, d, n, &at, &top[i])) return st;
    if (at != n)
      return set_error(FURY_ERR_INVALID_ARGUMENT, "column descriptor: " + std::to_string(n - at) +
                                                      " trailing entries");
    return FURY_OK;
  }
};

}  // namespace
}  // namespace fury

using namespace fury;

extern "C" {

const char* fury_jni_exception_class(int status) {
  switch (status) {
    case FURY_OK: return nullptr;
    case FURY_ERR_INVALID_ARGUMENT: return "java/lang/IllegalArgumentException";
    case FURY_ERR_UNSUPPORTED: return "java/lang/UnsupportedOperationException";
    case FURY_ERR_CLASS_NOT_COMPATIBLE: return "org/apache/fury/exception/ClassNotCompatibleException";
    case FURY_ERR_OUT_OF_BOUNDS: return "java/lang/IndexOutOfBoundsException";
    case FURY_ERR_ENCODER: return "org/apache/fury/format/encoder/EncoderException";
    case FURY_ERR_CAPACITY: return "java/lang/IndexOutOfBoundsException";
    default: return "java/lang/RuntimeException";       // FURY_ERR_DEVICE and unknown codes
  }
}

int fury_jni_schema_create(const char* const* names, const int32_t* meta, int32_t nodes,
                           int32_t top, fury_schema** out) {
  if (!out) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_jni_schema_create: out is null");
  *out = nullptr;
  if (nodes < 0 || top < 0 || top > nodes || (nodes > 0 && (!names || !meta)))
    return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_jni_schema_create: bad node counts");
  JField t;
  t.kids.reserve(static_cast<size_t>(nodes) + 1);
  std::vector<fury_field> fields(static_cast<size_t>(top));
  int32_t at = 0;
  for (int32_t i = 0; i < top; i++)
    if (int st = t.build(names, meta, nodes, &at, &fields[i])) return st;
  if (at != nodes)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_jni_schema_create: " +
                                                    std::to_string(nodes - at) + " unused nodes");
  return fury_schema_create(fields.data(), top, out);
}

int fury_jni_encode_host(const fury_schema* s, const int64_t* desc, int64_t desc_len,
                         int64_t nrows, void* rows, int64_t rows_capacity, int64_t* row_offsets,
                         int64_t* row_bytes, int32_t device) {
  JColumns c;
  if (int st = c.build(s, desc, desc_len)) return st;
  return fury_row_encode_host(s, c.top.data(), nrows, rows, rows_capacity, row_offsets, row_bytes,
                              device);
}

int fury_jni_decode_host(const fury_schema* s, const void* rows, const int64_t* row_offsets,
                         int64_t nrows, const int64_t* desc, int64_t desc_len, int32_t device) {
  JColumns c;
  if (int st = c.build(s, desc, desc_len)) return st;
  return fury_row_decode_host(s, rows, row_offsets, nrows, c.top.data(), device);
}

int fury_jni_decode_host_prepare(const fury_schema* s, const void* rows,
                                 const int64_t* row_offsets, int64_t nrows, int64_t* counts,
                                 int64_t counts_len, fury_decode_plan** plan, int32_t device) {
  if (!s || !counts) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_jni_decode_host_prepare: null");
  const size_t nn = s->nodes.size();
  if (counts_len < 0 || static_cast<uint64_t>(counts_len) < 2 * nn)
    return set_error(FURY_ERR_INVALID_ARGUMENT,
                     "fury_jni_decode_host_prepare: counts has " + std::to_string(counts_len) +
                         " entries, the schema needs " + std::to_string(2 * nn));
  std::vector<int64_t> e(nn + 1), b(nn + 1);
  const int st = fury_decode_host_prepare(s, rows, row_offsets, nrows, e.data(), b.data(), plan,
                                          device);
  if (st) return st;
  for (size_t i = 0; i < nn; i++) {
    counts[2 * i] = e[i];
    counts[2 * i + 1] = b[i];
  }
  return FURY_OK;
}

int fury_jni_decode_host_execute(const fury_schema* s, fury_decode_plan* plan, const int64_t* desc,
                                 int64_t desc_len) {
  JColumns c;
  if (int st = c.build(s, desc, desc_len)) return st;
  return fury_decode_host_execute(plan, c.top.data());
}

}  // extern "C"
