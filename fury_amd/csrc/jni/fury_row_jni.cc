// fury_row_jni.cc — JNI glue of java/src/main/java/org/apache/fury/format/encoder/
// GpuRowEncoder.java over the host-memory C ABI (include/fury_row.h: fury_schema_create,
// fury_row_encode_host, fury_row_decode_host).  Only addresses cross JNI: the Java side passes
// the off-heap addresses of Arrow buffers / MemoryBuffers (ArrowBuf.memoryAddress(),
// MemoryBuffer.getUnsafeAddress()), the bytes move over PCIe inside libfury_row.
//
// NOT BUILT BY DEFAULT: needs a JDK (jni.h), which this image lacks.  With one:
//   make -C fury_amd/csrc jni JAVA_HOME=/path/to/jdk      -> fury_amd/libfury_row_jni.so
// Status codes become the exceptions the reference throws (fury_status in fury_row.h).
#include <jni.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/fury_row.h"

namespace {

void throw_status(JNIEnv* env, int st) {
  static const char* cls[] = {
      nullptr,
      "java/lang/IllegalArgumentException",                      // FURY_ERR_INVALID_ARGUMENT
      "java/lang/UnsupportedOperationException",                 // FURY_ERR_UNSUPPORTED
      "org/apache/fury/exception/ClassNotCompatibleException",   // FURY_ERR_CLASS_NOT_COMPATIBLE
      "java/lang/IndexOutOfBoundsException",                     // FURY_ERR_OUT_OF_BOUNDS
      "org/apache/fury/format/encoder/EncoderException",         // FURY_ERR_ENCODER
      "java/lang/RuntimeException",                              // FURY_ERR_DEVICE
      "java/lang/IndexOutOfBoundsException"};                    // FURY_ERR_CAPACITY
  char msg[2048];
  fury_last_error(msg, sizeof msg);
  jclass k = env->FindClass(cls[st > 0 && st < 8 ? st : 6]);
  if (k) env->ThrowNew(k, msg);
}

// Pre-order field list {typeId, nullable, numChildren} x nodes -> fury_field tree.
struct FieldTree {
  std::vector<std::string> names;
  std::vector<std::vector<fury_field>> kids;   // children arrays, stable once built
  int build(const int* meta, int nodes, int* at, fury_field* out) {
    const int i = (*at)++;
    if (i >= nodes) return -1;
    out->name = names[i].c_str();
    out->type_id = meta[3 * i];
    out->nullable = meta[3 * i + 1];
    out->num_children = meta[3 * i + 2];
    out->children = nullptr;
    if (out->num_children > 0) {
      const size_t slot = kids.size();
      kids.emplace_back(out->num_children);
      for (int c = 0; c < out->num_children; c++)
        if (build(meta, nodes, at, &kids[slot][c])) return -1;
      out->children = kids[slot].data();
    }
    return 0;
  }
};

// Pre-order column descriptors {values, validity, offsets, capacity, numChildren} -> fury_column
// tree (host addresses).
struct ColumnTree {
  std::vector<std::vector<fury_column>> kids;
  int build(const jlong* d, jsize n, jsize* at, fury_column* out) {
    if (*at + 5 > n) return -1;
    const jlong* e = d + *at;
    *at += 5;
    out->values = reinterpret_cast<void*>(e[0]);
    out->validity = reinterpret_cast<uint8_t*>(e[1]);
    out->offsets = reinterpret_cast<int32_t*>(e[2]);
    out->capacity = e[3];
    out->child = nullptr;
    if (e[4] > 0) {
      const size_t slot = kids.size();
      kids.emplace_back(static_cast<size_t>(e[4]));
      for (jlong c = 0; c < e[4]; c++)
        if (build(d, n, at, &kids[slot][c])) return -1;
      out->child = kids[slot].data();
    }
    return 0;
  }
};

int columns_from(JNIEnv* env, const fury_schema* s, jlongArray desc, ColumnTree* tree,
                 std::vector<fury_column>* top) {
  fury_schema_info info;
  int st = fury_schema_get_info(s, &info);
  if (st) return st;
  const jsize n = env->GetArrayLength(desc);
  std::vector<jlong> d(n);
  env->GetLongArrayRegion(desc, 0, n, d.data());
  tree->kids.reserve(static_cast<size_t>(n / 5) + 1);    // no reallocation: children stay put
  top->assign(info.num_fields, fury_column{});
  jsize at = 0;
  for (int i = 0; i < info.num_fields; i++)
    if (tree->build(d.data(), n, &at, &(*top)[i])) return FURY_ERR_INVALID_ARGUMENT;
  return FURY_OK;
}

}  // namespace

extern "C" {

JNIEXPORT jlong JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeSchemaCreate(
    JNIEnv* env, jclass, jobjectArray names, jintArray meta, jint top) {
  const jsize nodes = env->GetArrayLength(names);
  FieldTree t;
  t.kids.reserve(static_cast<size_t>(nodes) + 1);
  for (jsize i = 0; i < nodes; i++) {
    jstring js = static_cast<jstring>(env->GetObjectArrayElement(names, i));
    const char* c = env->GetStringUTFChars(js, nullptr);
    t.names.emplace_back(c);
    env->ReleaseStringUTFChars(js, c);
  }
  std::vector<jint> m(env->GetArrayLength(meta));
  env->GetIntArrayRegion(meta, 0, static_cast<jsize>(m.size()), m.data());
  std::vector<fury_field> fields(top);
  int at = 0;
  for (jint i = 0; i < top; i++) {
    if (t.build(reinterpret_cast<const int*>(m.data()), nodes, &at, &fields[i])) {
      throw_status(env, FURY_ERR_INVALID_ARGUMENT);
      return 0;
    }
  }
  fury_schema* s = nullptr;
  const int st = fury_schema_create(fields.data(), top, &s);
  if (st) {
    throw_status(env, st);
    return 0;
  }
  return reinterpret_cast<jlong>(s);
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeSchemaDestroy(
    JNIEnv*, jclass, jlong schema) {
  fury_schema_destroy(reinterpret_cast<fury_schema*>(schema));
}

JNIEXPORT jlong JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeEncodeHost(
    JNIEnv* env, jclass, jlong schema, jlongArray desc, jlong nrows, jlong rows, jlong cap,
    jlong row_offsets, jint device) {
  const fury_schema* s = reinterpret_cast<const fury_schema*>(schema);
  ColumnTree tree;
  std::vector<fury_column> cols;
  int st = columns_from(env, s, desc, &tree, &cols);
  int64_t bytes = 0;
  if (!st)
    st = fury_row_encode_host(s, cols.data(), nrows, reinterpret_cast<void*>(rows), cap,
                              reinterpret_cast<int64_t*>(row_offsets), &bytes, device);
  if (st) throw_status(env, st);
  return bytes;
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeDecodeHost(
    JNIEnv* env, jclass, jlong schema, jlong rows, jlong row_offsets, jlong nrows,
    jlongArray desc, jint device) {
  const fury_schema* s = reinterpret_cast<const fury_schema*>(schema);
  ColumnTree tree;
  std::vector<fury_column> cols;
  int st = columns_from(env, s, desc, &tree, &cols);
  if (!st)
    st = fury_row_decode_host(s, reinterpret_cast<const void*>(rows),
                              reinterpret_cast<const int64_t*>(row_offsets), nrows, cols.data(),
                              device);
  if (st) throw_status(env, st);
}

JNIEXPORT jint JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeSchemaNumNodes(
    JNIEnv*, jclass, jlong schema) {
  return fury_schema_num_nodes(reinterpret_cast<const fury_schema*>(schema));
}

// Nested schemas, step 1: rows staged in HBM, per node (breadth-first) Arrow entries and payload
// bytes into counts[2 * i], counts[2 * i + 1]; returns the plan.
JNIEXPORT jlong JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeDecodeHostPrepare(
    JNIEnv* env, jclass, jlong schema, jlong rows, jlong row_offsets, jlong nrows,
    jlongArray counts, jint device) {
  const fury_schema* s = reinterpret_cast<const fury_schema*>(schema);
  const int nn = fury_schema_num_nodes(s);
  std::vector<int64_t> e(nn > 0 ? nn : 1), b(nn > 0 ? nn : 1);
  fury_decode_plan* plan = nullptr;
  const int st = fury_decode_host_prepare(s, reinterpret_cast<const void*>(rows),
                                          reinterpret_cast<const int64_t*>(row_offsets), nrows,
                                          e.data(), b.data(), &plan, device);
  if (st) {
    throw_status(env, st);
    return 0;
  }
  std::vector<jlong> c(2 * static_cast<size_t>(nn));
  for (int i = 0; i < nn; i++) {
    c[2 * i] = e[i];
    c[2 * i + 1] = b[i];
  }
  env->SetLongArrayRegion(counts, 0, static_cast<jsize>(c.size()), c.data());
  return reinterpret_cast<jlong>(plan);
}

// Step 2: decode into the host buffers the caller sized from the counts (descriptor tree as
// nativeDecodeHost), copy back.
JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeDecodeHostExecute(
    JNIEnv* env, jclass, jlong schema, jlong plan, jlongArray desc) {
  const fury_schema* s = reinterpret_cast<const fury_schema*>(schema);
  ColumnTree tree;
  std::vector<fury_column> cols;
  int st = columns_from(env, s, desc, &tree, &cols);
  if (!st) st = fury_decode_host_execute(reinterpret_cast<fury_decode_plan*>(plan), cols.data());
  if (st) throw_status(env, st);
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeDecodePlanDestroy(
    JNIEnv*, jclass, jlong plan) {
  fury_decode_plan_destroy(reinterpret_cast<fury_decode_plan*>(plan));
}

// Pinned host memory: GpuRowEncoder.allocatePinned / freePinned / pin / unpin and
// PinnedAllocationManager (Arrow buffers the GPU reaches directly).
JNIEXPORT jlong JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeHostAlloc(
    JNIEnv* env, jclass, jlong bytes) {
  void* p = nullptr;
  const int st = fury_host_alloc(bytes, &p);
  if (st) throw_status(env, st);
  return reinterpret_cast<jlong>(p);
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeHostFree(
    JNIEnv* env, jclass, jlong address) {
  const int st = fury_host_free(reinterpret_cast<void*>(address));
  if (st) throw_status(env, st);
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeHostRegister(
    JNIEnv* env, jclass, jlong address, jlong bytes) {
  const int st = fury_host_register(reinterpret_cast<void*>(address), bytes);
  if (st) throw_status(env, st);
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeHostUnregister(
    JNIEnv* env, jclass, jlong address) {
  const int st = fury_host_unregister(reinterpret_cast<void*>(address));
  if (st) throw_status(env, st);
}

}  // extern "C"
