// schema.cpp — host-side schema/layout planner of libfury_row.
//
// Restates, for the C ABI:
//   DataTypes.getTypeWidth / computeSchemaHash   (java/fury-format/.../type/DataTypes.java:68-133,
//                                                 499-544)
//   BinaryRowWriter layout (bitmap + 8-byte slots) (.../row/binary/writer/BinaryRowWriter.java:46-52)
//   Descriptor field order                        (fury-core .../type/Descriptor.java:324-332)
//   StringUtils.lowerCamelToLowerUnderscore       (fury-core .../util/StringUtils.java:252-271)
#include <algorithm>
#include <cstring>
#include <new>
#include <numeric>

#include "internal.h"

namespace fury {

// keep in sync with kernels.h (this TU is host-only C++)
constexpr int kGenMaxNodesHost = 4096;   // = kGenMaxWideNodes
constexpr int kGenMaxDepthHost = 65;     // < : kMaxNestLevels = 64 levels (rowenc.hip rdeep stack)
constexpr int kMaxWideVarColsHost = 256; // = kMaxWideVarCols: the flat variable-length kernels

static thread_local std::string g_last_error;

int set_error(int status, const std::string& msg) {
  g_last_error = msg;
  return status;
}

static int32_t type_width(int32_t t) {
  switch (t) {
    case FURY_TYPE_BOOL: return 1;
    case FURY_TYPE_INT8: return 1;
    case FURY_TYPE_INT16: return 2;
    case FURY_TYPE_INT32: return 4;
    case FURY_TYPE_INT64: return 8;
    case FURY_TYPE_FLOAT32: return 4;
    case FURY_TYPE_FLOAT64: return 8;
    case FURY_TYPE_DATE32: return 4;
    case FURY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

static bool known_type(int32_t t) {
  switch (t) {
    case FURY_TYPE_BOOL: case FURY_TYPE_INT8: case FURY_TYPE_INT16: case FURY_TYPE_INT32:
    case FURY_TYPE_INT64: case FURY_TYPE_FLOAT32: case FURY_TYPE_FLOAT64: case FURY_TYPE_STRING:
    case FURY_TYPE_BINARY: case FURY_TYPE_DATE32: case FURY_TYPE_TIMESTAMP:
    case FURY_TYPE_DECIMAL: case FURY_TYPE_LIST: case FURY_TYPE_STRUCT: case FURY_TYPE_MAP:
      return true;
    default:
      return false;
  }
}

// Deep-copies and validates one field (DataTypes.computeHash's checkArgument on children).
static int copy_field(const fury_field& in, OwnedField* out, int depth) {
  if (depth > 64) return set_error(FURY_ERR_UNSUPPORTED, "schema nesting deeper than 64");
  if (!known_type(in.type_id)) {
    return set_error(FURY_ERR_UNSUPPORTED,
                     "Unsupported type id " + std::to_string(in.type_id) + " for field " +
                         (in.name ? in.name : "<null>"));
  }
  out->name = in.name ? in.name : "";
  out->type_id = in.type_id;
  out->nullable = in.nullable ? 1 : 0;
  int32_t want = -1;
  if (in.type_id == FURY_TYPE_LIST) want = 1;
  if (in.type_id == FURY_TYPE_MAP) want = 2;
  if (in.type_id != FURY_TYPE_STRUCT) {
    int32_t have = in.num_children;
    if (want < 0) want = 0;
    if (have != want) {
      return set_error(FURY_ERR_INVALID_ARGUMENT,
                       "field " + out->name + " of type id " + std::to_string(in.type_id) +
                           " needs " + std::to_string(want) + " children, got " +
                           std::to_string(have));
    }
  }
  if (in.num_children < 0 || (in.num_children > 0 && in.children == nullptr)) {
    return set_error(FURY_ERR_INVALID_ARGUMENT, "field " + out->name + ": bad children");
  }
  out->children.resize(in.num_children);
  for (int32_t i = 0; i < in.num_children; i++) {
    int st = copy_field(in.children[i], &out->children[i], depth + 1);
    if (st) return st;
  }
  return FURY_OK;
}

// DataTypes.computeHash (DataTypes.java:506-544): multiplyExact/addExact, h >>= 2 on overflow.
static int64_t hash_field(int64_t hash, const OwnedField& f) {
  for (;;) {
    int64_t m, a;
    if (!__builtin_mul_overflow(hash, int64_t{31}, &m) &&
        !__builtin_add_overflow(m, int64_t{f.type_id}, &a)) {
      hash = a;
      break;
    }
    hash >>= 2;
  }
  for (const auto& c : f.children) hash = hash_field(hash, c);
  return hash;
}

static FieldPlan plan_field(const OwnedField& f, std::string* why) {
  FieldPlan p{};
  p.type_id = f.type_id;
  p.width = type_width(f.type_id);
  p.nullable = f.nullable;
  p.elem_type = 0;
  p.elem_width = 0;
  p.elem_nullable = 0;
  switch (f.type_id) {
    case FURY_TYPE_BOOL: p.kind = kBool; break;
    case FURY_TYPE_STRING: case FURY_TYPE_BINARY: p.kind = kBytes; break;
    case FURY_TYPE_DECIMAL: p.kind = kDecimal; break;
    case FURY_TYPE_LIST: {
      const OwnedField& e = f.children[0];
      int32_t ew = type_width(e.type_id);
      p.elem_type = e.type_id;
      p.elem_width = ew < 0 ? 8 : ew;   // BinaryArrayWriter ctor :71-82
      p.elem_nullable = e.nullable;
      if (ew > 0) {
        p.kind = kListFixed;
      } else {
        p.kind = kOther;
        *why = "field " + f.name + ": list of variable-length elements";
      }
      break;
    }
    case FURY_TYPE_STRUCT:
      p.kind = kOther;
      *why = "field " + f.name + ": nested struct";
      break;
    case FURY_TYPE_MAP:
      p.kind = kOther;
      *why = "field " + f.name + ": map";
      break;
    default: p.kind = kFixed; break;
  }
  return p;
}

}  // namespace fury

using namespace fury;

extern "C" {

int32_t fury_abi_version(void) { return FURY_ROW_ABI_VERSION; }

size_t fury_last_error(char* buf, size_t len) {
  const std::string& e = g_last_error;
  if (buf && len) {
    size_t n = std::min(len - 1, e.size());
    std::memcpy(buf, e.data(), n);
    buf[n] = '\0';
  }
  return e.size();
}

int32_t fury_type_width(int32_t type_id) { return type_width(type_id); }

int fury_sort_bean_fields(const char* const* java_names, int32_t n, int32_t* order) {
  if (n < 0 || (n > 0 && (!java_names || !order)))
    return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_sort_bean_fields: null argument");
  // String.compareTo compares UTF-16 code units; for names given as UTF-8 we decode to code
  // points and compare the UTF-16 encodings (surrogates sort above the BMP range E000-FFFF).
  auto utf16 = [](const char* s) {
    std::vector<uint16_t> out;
    const unsigned char* p = reinterpret_cast<const unsigned char*>(s);
    while (*p) {
      uint32_t cp;
      int n = 1;
      if (*p < 0x80) cp = *p;
      else if ((*p >> 5) == 6) { cp = *p & 0x1F; n = 2; }
      else if ((*p >> 4) == 14) { cp = *p & 0x0F; n = 3; }
      else { cp = *p & 0x07; n = 4; }
      for (int i = 1; i < n && p[i]; i++) cp = (cp << 6) | (p[i] & 0x3F);
      p += n;
      if (cp >= 0x10000) {
        cp -= 0x10000;
        out.push_back(static_cast<uint16_t>(0xD800 + (cp >> 10)));
        out.push_back(static_cast<uint16_t>(0xDC00 + (cp & 0x3FF)));
      } else {
        out.push_back(static_cast<uint16_t>(cp));
      }
    }
    return out;
  };
  std::vector<std::vector<uint16_t>> keys(n);
  for (int32_t i = 0; i < n; i++) {
    if (!java_names[i]) return set_error(FURY_ERR_INVALID_ARGUMENT, "null field name");
    keys[i] = utf16(java_names[i]);
  }
  std::vector<int32_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(),
                   [&](int32_t a, int32_t b) { return keys[a] < keys[b]; });
  std::copy(idx.begin(), idx.end(), order);
  return FURY_OK;
}

int32_t fury_lower_camel_to_lower_underscore(const char* in, char* out, size_t out_len) {
  if (!in || !out || out_len == 0) return -1;
  size_t o = 0;
  for (const char* p = in; *p; ++p) {
    char c = *p;
    if (c >= 'A' && c <= 'Z') {
      if (o + 2 >= out_len) break;
      out[o++] = '_';
      out[o++] = static_cast<char>(c - 'A' + 'a');
    } else {
      if (o + 1 >= out_len) break;
      out[o++] = c;
    }
  }
  out[o] = '\0';
  return static_cast<int32_t>(o);
}

int fury_schema_create(const fury_field* fields, int32_t num_fields, fury_schema** out) {
  if (!out) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_schema_create: out is null");
  *out = nullptr;
  if (num_fields < 0 || (num_fields > 0 && !fields))
    return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_schema_create: bad field array");
  fury_schema* s = new (std::nothrow) fury_schema();
  if (!s) return set_error(FURY_ERR_ENCODER, "out of host memory");
  s->fields.resize(num_fields);
  for (int32_t i = 0; i < num_fields; i++) {
    int st = copy_field(fields[i], &s->fields[i], 0);
    if (st) {
      delete s;
      return st;
    }
  }
  s->num_fields = num_fields;
  s->bitmap_bytes = bitmap_bytes(num_fields);
  s->fixed_size = s->bitmap_bytes + 8 * num_fields;
  int64_t h = 17;
  for (const auto& f : s->fields) h = hash_field(h, f);
  s->schema_hash = h;
  s->is_fixed = 1;
  for (const auto& f : s->fields) {
    std::string why;
    FieldPlan p = plan_field(f, &why);
    if (p.width < 0) s->is_fixed = 0;
    if (p.kind == kOther && s->device_ok) {
      s->device_ok = 0;
      s->device_reason = why;
    }
    if (p.kind == kBytes || p.kind == kDecimal || p.kind == kListFixed) s->num_var++;
    s->plan.push_back(p);
  }
  // Flattened node tree (breadth-first) for the generic engine.
  {
    std::vector<const OwnedField*> q;
    std::vector<int32_t> depth;
    for (const auto& f : s->fields) {
      q.push_back(&f);
      depth.push_back(1);
    }
    for (size_t i = 0; i < q.size(); i++) {
      GenTpl t{q[i]->type_id, 0, static_cast<int32_t>(q[i]->children.size()), q[i]->nullable};
      t.first_child = static_cast<int32_t>(q.size());
      for (const auto& c : q[i]->children) {
        q.push_back(&c);
        depth.push_back(depth[i] + 1);
      }
      s->nodes.push_back(t);
      s->depth = std::max(s->depth, depth[i]);
    }
  }
  // flat variable-length schemas wider than the flat kernels: the generic engine (row
  // interpreter encode, plan-API decode), like nested ones
  if (s->device_ok && !s->is_fixed && num_fields > kMaxWideVarColsHost) {
    s->device_ok = 0;
    s->device_reason = "variable-length schema wider than " + std::to_string(kMaxWideVarColsHost) +
                       " fields";
  }
  if (!s->device_ok) {
    // nested fields: the generic engine handles them within its table limits
    if (s->nodes.size() <= static_cast<size_t>(kGenMaxNodesHost) && s->depth < kGenMaxDepthHost) {
      s->device_ok = 1;
      s->generic = 1;
      s->device_reason.clear();
    } else {
      s->device_reason += " (nested schema beyond " + std::to_string(kGenMaxNodesHost) +
                          " nodes / " + std::to_string(kGenMaxDepthHost - 1) + " levels)";
    }
  }
  *out = s;
  return FURY_OK;
}

int fury_collection_schema_create(const fury_field* field, fury_schema** out) {
  if (!out) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_collection_schema_create: out is null");
  *out = nullptr;
  if (!field) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_collection_schema_create: field is null");
  if (field->type_id != FURY_TYPE_LIST && field->type_id != FURY_TYPE_MAP)
    return set_error(FURY_ERR_INVALID_ARGUMENT,
                     "a collection schema's field must be a LIST (ArrayEncoder) or MAP (MapEncoder)");
  fury_schema* s = nullptr;
  int st = fury_schema_create(field, 1, &s);
  if (st) return st;
  // Every entry is one top-level BinaryArray / BinaryMap: always the generic engine, no row
  // header, no schema hash (these encoders frame [int32 size][bytes], Encoders.java:372-386).
  s->root = field->type_id == FURY_TYPE_LIST ? 1 : 2;
  s->is_fixed = 0;
  s->bitmap_bytes = 0;
  s->fixed_size = 0;
  s->schema_hash = 0;
  if (s->nodes.size() <= static_cast<size_t>(kGenMaxNodesHost) && s->depth < kGenMaxDepthHost) {
    s->device_ok = 1;
    s->generic = 1;
    s->device_reason.clear();
  } else {
    s->device_ok = 0;
    s->device_reason = "collection type beyond " + std::to_string(kGenMaxNodesHost) + " nodes / " +
                       std::to_string(kGenMaxDepthHost - 1) + " levels";
  }
  *out = s;
  return FURY_OK;
}

int32_t fury_schema_num_nodes(const fury_schema* s) {
  return s ? static_cast<int32_t>(s->nodes.size()) : -1;
}

void fury_schema_destroy(fury_schema* schema) { delete schema; }

int fury_schema_get_info(const fury_schema* s, fury_schema_info* info) {
  if (!s || !info) return set_error(FURY_ERR_INVALID_ARGUMENT, "fury_schema_get_info: null");
  info->num_fields = s->num_fields;
  info->bitmap_bytes = s->bitmap_bytes;
  info->fixed_size = s->fixed_size;
  info->is_fixed = s->is_fixed;
  info->schema_hash = s->schema_hash;
  return FURY_OK;
}

}  // extern "C"
