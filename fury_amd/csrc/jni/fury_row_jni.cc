// fury_row_jni.cc — JNI glue of java/src/main/java/org/apache/fury/format/encoder/
// GpuRowEncoder.java.  Only JNIEnv marshalling lives here: Java arrays are copied in / out and a
// status becomes the exception fury_jni_exception_class names.  Decoding the descriptor arrays
// into fury_field / fury_column trees, the two-step nested decode and the status mapping are the
// library's fury_jni_* entry points (fury_amd/csrc/jnicore.cpp, include/fury_row.h), which the
// test suite exercises with GpuRowEncoder's exact array layouts (tests/test_jni_core.py).
//
// NOT BUILT BY DEFAULT: needs a JDK (jni.h), which this image lacks.  With one:
//   make -C fury_amd/csrc jni JAVA_HOME=/path/to/jdk      -> fury_amd/libfury_row_jni.so
#include <jni.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/fury_row.h"

namespace {

bool raise(JNIEnv* env, int st) {
  if (st == FURY_OK) return false;
  char msg[2048];
  fury_last_error(msg, sizeof msg);
  jclass k = env->FindClass(fury_jni_exception_class(st));
  if (k) env->ThrowNew(k, msg);
  return true;
}

std::vector<int64_t> longs(JNIEnv* env, jlongArray a) {
  std::vector<int64_t> v(a ? env->GetArrayLength(a) : 0);
  if (!v.empty()) env->GetLongArrayRegion(a, 0, static_cast<jsize>(v.size()),
                                          reinterpret_cast<jlong*>(v.data()));
  return v;
}

}  // namespace

extern "C" {

JNIEXPORT jlong JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeSchemaCreate(
    JNIEnv* env, jclass, jobjectArray names, jintArray meta, jint top) {
  const jsize nodes = env->GetArrayLength(names);
  std::vector<std::string> owned;
  owned.reserve(nodes);
  for (jsize i = 0; i < nodes; i++) {
    jstring js = static_cast<jstring>(env->GetObjectArrayElement(names, i));
    const char* c = env->GetStringUTFChars(js, nullptr);
    owned.emplace_back(c);
    env->ReleaseStringUTFChars(js, c);
  }
  std::vector<const char*> ptrs;
  for (const std::string& s : owned) ptrs.push_back(s.c_str());
  std::vector<int32_t> m(env->GetArrayLength(meta));
  env->GetIntArrayRegion(meta, 0, static_cast<jsize>(m.size()), reinterpret_cast<jint*>(m.data()));
  fury_schema* s = nullptr;
  if (static_cast<jsize>(m.size()) != 3 * nodes) {
    env->ThrowNew(env->FindClass("java/lang/IllegalArgumentException"), "meta length");
    return 0;
  }
  if (raise(env, fury_jni_schema_create(ptrs.data(), m.data(), nodes, top, &s))) return 0;
  return reinterpret_cast<jlong>(s);
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeSchemaDestroy(
    JNIEnv*, jclass, jlong schema) {
  fury_schema_destroy(reinterpret_cast<fury_schema*>(schema));
}

JNIEXPORT jint JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeSchemaNumNodes(
    JNIEnv*, jclass, jlong schema) {
  return fury_schema_num_nodes(reinterpret_cast<const fury_schema*>(schema));
}

JNIEXPORT jlong JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeEncodeHost(
    JNIEnv* env, jclass, jlong schema, jlongArray desc, jlong nrows, jlong rows, jlong cap,
    jlong row_offsets, jint device) {
  const std::vector<int64_t> d = longs(env, desc);
  int64_t bytes = 0;
  raise(env, fury_jni_encode_host(reinterpret_cast<const fury_schema*>(schema), d.data(),
                                  static_cast<int64_t>(d.size()), nrows,
                                  reinterpret_cast<void*>(rows), cap,
                                  reinterpret_cast<int64_t*>(row_offsets), &bytes, device));
  return bytes;
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeDecodeHost(
    JNIEnv* env, jclass, jlong schema, jlong rows, jlong row_offsets, jlong nrows,
    jlongArray desc, jint device) {
  const std::vector<int64_t> d = longs(env, desc);
  raise(env, fury_jni_decode_host(reinterpret_cast<const fury_schema*>(schema),
                                  reinterpret_cast<const void*>(rows),
                                  reinterpret_cast<const int64_t*>(row_offsets), nrows, d.data(),
                                  static_cast<int64_t>(d.size()), device));
}

JNIEXPORT jlong JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeDecodeHostPrepare(
    JNIEnv* env, jclass, jlong schema, jlong rows, jlong row_offsets, jlong nrows,
    jlongArray counts, jint device) {
  std::vector<int64_t> c(env->GetArrayLength(counts));
  fury_decode_plan* plan = nullptr;
  if (raise(env, fury_jni_decode_host_prepare(reinterpret_cast<const fury_schema*>(schema),
                                              reinterpret_cast<const void*>(rows),
                                              reinterpret_cast<const int64_t*>(row_offsets),
                                              nrows, c.data(), static_cast<int64_t>(c.size()),
                                              &plan, device)))
    return 0;
  env->SetLongArrayRegion(counts, 0, static_cast<jsize>(c.size()),
                          reinterpret_cast<const jlong*>(c.data()));
  return reinterpret_cast<jlong>(plan);
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeDecodeHostExecute(
    JNIEnv* env, jclass, jlong schema, jlong plan, jlongArray desc) {
  const std::vector<int64_t> d = longs(env, desc);
  raise(env, fury_jni_decode_host_execute(reinterpret_cast<const fury_schema*>(schema),
                                          reinterpret_cast<fury_decode_plan*>(plan), d.data(),
                                          static_cast<int64_t>(d.size())));
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
  raise(env, fury_host_alloc(bytes, &p));
  return reinterpret_cast<jlong>(p);
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeHostFree(
    JNIEnv* env, jclass, jlong address) {
  raise(env, fury_host_free(reinterpret_cast<void*>(address)));
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeHostRegister(
    JNIEnv* env, jclass, jlong address, jlong bytes) {
  raise(env, fury_host_register(reinterpret_cast<void*>(address), bytes));
}

JNIEXPORT void JNICALL Java_org_apache_fury_format_encoder_GpuRowEncoder_nativeHostUnregister(
    JNIEnv* env, jclass, jlong address) {
  raise(env, fury_host_unregister(reinterpret_cast<void*>(address)));
}

}  // extern "C"
