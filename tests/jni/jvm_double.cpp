// TEST DOUBLE — a minimal object model behind tests/jni/jni.h, so tests/test_jni.py
// can build NativeCodec-like objects (typed fields, direct ByteBuffers,
// ByteBuffer[] arrays) from Python and call the shim's Java_NativeCodec_*
// entry points. Field lookups check the JNI type signature the way a JVM does
// (GetFieldID with the wrong signature raises NoSuchFieldError).
#include "jni.h"

#include <map>
#include <memory>
#include <set>
#include <string>
#include <utility>
#include <vector>

namespace {

struct Obj : _jobject {
  std::string class_name;
  std::map<std::string, std::pair<std::string, long long>> prims;  // name -> (sig, value)
  std::map<std::string, Obj*> objs;                                // name -> object field
  void* addr = nullptr;                                            // direct buffer
  long long cap = -1;
  std::vector<Obj*> elems;                                         // object array
  bool is_array = false;
};

std::vector<std::unique_ptr<Obj>> g_heap;
std::set<std::pair<std::string, std::string>> g_fields;  // interned (name, sig): stable addresses
std::string g_exception;
long long g_live_refs = 0;

Obj* alloc(const std::string& cls) {
  g_heap.emplace_back(new Obj());
  g_heap.back()->class_name = cls;
  return g_heap.back().get();
}
Obj* as(jobject o) { return static_cast<Obj*>(o); }
Obj* as(void* o) { return static_cast<Obj*>(static_cast<_jobject*>(o)); }
const std::pair<std::string, std::string>& key(jfieldID f) {
  return *reinterpret_cast<const std::pair<std::string, std::string>*>(f);
}

jclass GetObjectClass(JNIEnv_*, jobject o) {
  ++g_live_refs;
  return o;  // the object doubles as its class: it knows its fields
}
jfieldID GetFieldID(JNIEnv_*, jclass c, const char* name, const char* sig) {
  Obj* o = as(c);
  const std::string n(name), s(sig);
  const bool prim = o->prims.count(n) && o->prims[n].first == s;
  const bool obj = o->objs.count(n) && s == "Ljava/nio/ByteBuffer;";
  if (!prim && !obj) {
    g_exception = "java/lang/NoSuchFieldError: " + n + " " + s;
    return nullptr;
  }
  auto it = g_fields.insert({n, s}).first;
  return reinterpret_cast<jfieldID>(const_cast<std::pair<std::string, std::string>*>(&*it));
}
long long prim(jobject o, jfieldID f) { return as(o)->prims.at(key(f).first).second; }
jint GetIntField(JNIEnv_*, jobject o, jfieldID f) { return static_cast<jint>(prim(o, f)); }
jchar GetCharField(JNIEnv_*, jobject o, jfieldID f) { return static_cast<jchar>(prim(o, f)); }
jboolean GetBooleanField(JNIEnv_*, jobject o, jfieldID f) { return static_cast<jboolean>(prim(o, f)); }
jobject GetObjectField(JNIEnv_*, jobject o, jfieldID f) {
  Obj* v = as(o)->objs.at(key(f).first);
  if (v) ++g_live_refs;
  return v;
}
void* GetDirectBufferAddress(JNIEnv_*, jobject b) { return as(b)->addr; }
jlong GetDirectBufferCapacity(JNIEnv_*, jobject b) { return as(b)->cap; }
jsize GetArrayLength(JNIEnv_*, jobjectArray a) { return static_cast<jsize>(as(a)->elems.size()); }
jobject GetObjectArrayElement(JNIEnv_*, jobjectArray a, jsize i) {
  Obj* arr = as(a);
  if (i < 0 || static_cast<size_t>(i) >= arr->elems.size()) {
    g_exception = "java/lang/ArrayIndexOutOfBoundsException";
    return nullptr;
  }
  if (arr->elems[i]) ++g_live_refs;
  return arr->elems[i];
}
void DeleteLocalRef(JNIEnv_*, jobject o) {
  if (o) --g_live_refs;
}
jclass FindClass(JNIEnv_*, const char* name) { return alloc(name); }
jint ThrowNew(JNIEnv_*, jclass c, const char* msg) {
  g_exception = as(c)->class_name + ": " + msg;
  return 0;
}
jboolean ExceptionCheck(JNIEnv_*) { return g_exception.empty() ? JNI_FALSE : JNI_TRUE; }

const JNIFunctionsDouble kFunctions = {
    GetObjectClass, GetFieldID, GetIntField, GetCharField, GetBooleanField, GetObjectField,
    GetDirectBufferAddress, GetDirectBufferCapacity, GetArrayLength, GetObjectArrayElement,
    DeleteLocalRef, FindClass, ThrowNew, ExceptionCheck,
};
JNIEnv_ g_env{&kFunctions};

}  // namespace

extern "C" {
void* jd_env() { return &g_env; }
void* jd_object(const char* cls) { return alloc(cls); }
// sig: "I", "C" or "Z"
void jd_set_prim(void* o, const char* name, const char* sig, long long v) { as(o)->prims[name] = {sig, v}; }
void jd_set_object(void* o, const char* name, void* v) { as(o)->objs[name] = as(v); }
void* jd_buffer(void* addr, long long cap) {
  Obj* b = alloc("java/nio/DirectByteBuffer");
  b->addr = addr;
  b->cap = cap;
  return b;
}
void* jd_array(int n) {
  Obj* a = alloc("[Ljava/nio/ByteBuffer;");
  a->is_array = true;
  a->elems.assign(n, nullptr);
  return a;
}
void jd_array_set(void* a, int i, void* v) { as(a)->elems.at(i) = as(v); }
const char* jd_exception() { return g_exception.c_str(); }
void jd_clear_exception() { g_exception.clear(); }
long long jd_live_refs() { return g_live_refs; }
}
