// internal.h — shared host-side structures of libfury_row (not part of the public ABI).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/fury_row.h"

namespace fury {

// How a top-level field is laid out in a row and moved by the device kernels.
enum FieldKind : int32_t {
  kFixed = 0,        // 1/2/4/8-byte scalar in its slot (zero-extended)
  kBool = 1,         // Arrow bit-packed input, putBoolean byte in the slot
  kBytes = 2,        // STRING / BINARY: writeUnaligned into the var section
  kDecimal = 3,      // 16 bytes in the var section (writeDecimal)
  kListFixed = 4,    // LIST of fixed-width (or bool) elements: BinaryArray in the var section
  kOther = 5         // STRUCT / MAP / LIST of var elements: not handled on device yet
};

struct FieldPlan {
  int32_t type_id;
  int32_t width;         // DataTypes.getTypeWidth (-1 for var)
  int32_t kind;          // FieldKind
  int32_t nullable;
  int32_t elem_type;     // LIST element type id
  int32_t elem_width;    // BinaryArrayWriter.elementSize
  int32_t elem_nullable;
};

// Node of the flattened schema tree used by the generic (nested) engine: breadth-first, the
// top-level fields first, every node's children contiguous.
struct GenTpl {
  int32_t type_id;
  int32_t first_child;
  int32_t num_children;
  int32_t nullable;
};

struct OwnedField {
  std::string name;
  int32_t type_id = 0;
  int32_t nullable = 1;
  std::vector<OwnedField> children;
};

}  // namespace fury

struct fury_schema {
  std::vector<fury::OwnedField> fields;
  std::vector<fury::FieldPlan> plan;
  int32_t num_fields = 0;
  int32_t bitmap_bytes = 0;
  int32_t fixed_size = 0;
  int32_t is_fixed = 0;
  int64_t schema_hash = 0;
  int32_t device_ok = 1;          // every field kind has a device kernel
  std::string device_reason;      // why not, when device_ok == 0
  int32_t num_var = 0;            // fields of kind kBytes / kDecimal / kListFixed
  int32_t generic = 0;            // nested schema: encode/decode run the generic engine
  int32_t root = 0;               // 0: rows of the fields; 1 / 2: batches of top-level
                                  // BinaryArrays / BinaryMaps (ArrayEncoder / MapEncoder)
  int32_t depth = 0;              // deepest nesting level (top-level fields = 1)
  std::vector<fury::GenTpl> nodes;
};

// Decode plan of the two-step (nested) decode, device and host-memory flavours.
namespace fury { struct LvPlan; struct TreePlan; struct WidePlan; }

struct fury_decode_plan {
  const fury_schema* schema = nullptr;
  const uint8_t* rows = nullptr;
  const int64_t* offs = nullptr;
  int64_t nrows = 0;
  fury::LvPlan* lv = nullptr;      // level-by-level engine state (levels.hip); NULL when nrows = 0
  fury::TreePlan* tree = nullptr;  // tile-staged engine state (tree.hip): used when set
  fury::WidePlan* wide = nullptr;  // flat schemas of 17-256 fields (wide.hip): used when set
  bool arrow = false;
  std::vector<int64_t> totals;     // per node: Arrow entries, payload bytes
  void* owned = nullptr;           // host flavour: the staged rows + offsets (device memory)
  void* owned_stream = nullptr;    // host flavour: its stream
  int32_t device = 0;
};

namespace fury {

// Per-thread last error (fury_last_error).
int set_error(int status, const std::string& msg);
int check_hip(int hip_status, const char* what);

inline int32_t bitmap_bytes(int64_t n) { return static_cast<int32_t>(((n + 63) / 64) * 8); }
inline int64_t round8(int64_t n) { return (n + 7) & ~int64_t(7); }

}  // namespace fury
