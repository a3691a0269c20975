/* TEST DOUBLE — the subset of the JNI interface that ecwide_amd/csrc/jni/ecw_jni.cpp
 * uses, with the same C++ member-call API as a JDK's <jni.h>, so the shim can be
 * compiled and driven without a JVM (this image has no JDK). Used only by
 * tests/test_jni.py together with tests/jni/jvm_double.cpp; the product
 * libcodec.so is built against $JAVA_HOME/include/jni.h (ecwide_amd/build.py).
 * The function table is this double's own layout, not the JNI ABI. */
#ifndef ECW_TEST_JNI_DOUBLE_H
#define ECW_TEST_JNI_DOUBLE_H

#include <cstdint>

typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef jint jsize;

struct _jobject {};
typedef _jobject* jobject;
typedef jobject jclass;
typedef jobject jobjectArray;
typedef jobject jthrowable;
struct _jfieldID;
typedef _jfieldID* jfieldID;

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1

struct JNIEnv_;
struct JNIFunctionsDouble {
  jclass (*GetObjectClass)(JNIEnv_*, jobject);
  jfieldID (*GetFieldID)(JNIEnv_*, jclass, const char*, const char*);
  jint (*GetIntField)(JNIEnv_*, jobject, jfieldID);
  jchar (*GetCharField)(JNIEnv_*, jobject, jfieldID);
  jboolean (*GetBooleanField)(JNIEnv_*, jobject, jfieldID);
  jobject (*GetObjectField)(JNIEnv_*, jobject, jfieldID);
  void* (*GetDirectBufferAddress)(JNIEnv_*, jobject);
  jlong (*GetDirectBufferCapacity)(JNIEnv_*, jobject);
  jsize (*GetArrayLength)(JNIEnv_*, jobjectArray);
  jobject (*GetObjectArrayElement)(JNIEnv_*, jobjectArray, jsize);
  void (*DeleteLocalRef)(JNIEnv_*, jobject);
  jclass (*FindClass)(JNIEnv_*, const char*);
  jint (*ThrowNew)(JNIEnv_*, jclass, const char*);
  jboolean (*ExceptionCheck)(JNIEnv_*);
};

struct JNIEnv_ {
  const JNIFunctionsDouble* functions;
  jclass GetObjectClass(jobject o) { return functions->GetObjectClass(this, o); }
  jfieldID GetFieldID(jclass c, const char* n, const char* s) { return functions->GetFieldID(this, c, n, s); }
  jint GetIntField(jobject o, jfieldID f) { return functions->GetIntField(this, o, f); }
  jchar GetCharField(jobject o, jfieldID f) { return functions->GetCharField(this, o, f); }
  jboolean GetBooleanField(jobject o, jfieldID f) { return functions->GetBooleanField(this, o, f); }
  jobject GetObjectField(jobject o, jfieldID f) { return functions->GetObjectField(this, o, f); }
  void* GetDirectBufferAddress(jobject b) { return functions->GetDirectBufferAddress(this, b); }
  jlong GetDirectBufferCapacity(jobject b) { return functions->GetDirectBufferCapacity(this, b); }
  jsize GetArrayLength(jobjectArray a) { return functions->GetArrayLength(this, a); }
  jobject GetObjectArrayElement(jobjectArray a, jsize i) { return functions->GetObjectArrayElement(this, a, i); }
  void DeleteLocalRef(jobject o) { functions->DeleteLocalRef(this, o); }
  jclass FindClass(const char* n) { return functions->FindClass(this, n); }
  jint ThrowNew(jclass c, const char* m) { return functions->ThrowNew(this, c, m); }
  jboolean ExceptionCheck() { return functions->ExceptionCheck(this); }
};
typedef JNIEnv_ JNIEnv;

#endif
