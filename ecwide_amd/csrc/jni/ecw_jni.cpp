// libcodec.so — ECWide-C's eight JNI natives over the C ABI of libecwide.so.
//
// Drop-in for the library `NativeCodec.java:213-215` loads
// (`System.loadLibrary("codec")`, built by `ECWide-C/src/native/makefile:12-14`):
// exports the symbols declared in `ECWide-C/src/native/NativeCodec.h:15-72`
// and reads the same `NativeCodec` fields the reference natives read
// (`NativeCodec.java:4-18`), so the Java side runs unchanged. The reference
// natives are `NativeCodec.cc:12-323`; what differs on purpose:
//
//  * the work runs on the MI355X (ecw_encode / ecw_decode / ... copy the
//    direct ByteBuffers through HBM in column slices, ecwide.h);
//  * by default every byte is the reference's, quirks included: local parities
//    are written as zeros (its XOR table is built from an all-zero matrix,
//    NativeCodec.cc:176-186) and the process's first xorIntemediate writes
//    zeros (its static `flag`, NativeCodec.cc:287-292). ECWIDE_LOCAL_MODE=xor
//    writes the group XOR the design intends (what CL repair needs), and
//    ECWIDE_XORI_LITERAL=0 XORs on every call;
//  * errors the reference never checked (short arrays, non-direct buffers,
//    device failures) raise a Java exception instead of crashing the JVM.
//
// Build against a JDK: see ecwide_amd/build.py:build_jni (needs
// $JAVA_HOME/include/jni.h). The codec for a NativeCodec instance is derived
// from its fields and cached per parameter set (codecs are reentrant; calls
// on one codec serialise on its own lock).
#include <jni.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "ecwide.h"

namespace {

// type, k, m, r, node, multinode, local mode, chunk
using Key = std::tuple<char, int, int, int, int, int, int, long long>;

// codecs are immutable after creation: one per parameter set for the life of
// the process. The cache is never destroyed: at JVM exit other Java threads
// may still be inside a native call on one of its codecs (System.exit does not
// wait for them), so releasing the codecs from a static destructor could free
// them under those calls. The map stays reachable through g_codecs, so leak
// checkers do not report it.
using Codecs = std::map<Key, ecw_codec*>;
std::mutex g_mu;
Codecs& g_codecs = *new Codecs();
std::atomic<bool> g_xori_called{false};

void throw_java(JNIEnv* e, const char* cls, const std::string& msg) {
  if (e->ExceptionCheck()) return;  // keep the first exception
  jclass c = e->FindClass(cls);
  if (c) e->ThrowNew(c, msg.c_str());
}

bool check(JNIEnv* e, int status, const char* what) {
  if (status >= 0) return true;
  throw_java(e, "java/lang/RuntimeException",
             std::string("ecwide: ") + what + ": " + ecw_status_string(status));
  return false;
}

// The NativeCodec fields the reference natives read (NativeCodec.java:4-18).
struct Fields {
  char code_type = 0;
  bool multinode = false;
  int chunk_size = 0, encode_data_num = 0, decode_data_num = 0, partial_decode_num = 0;
  int global_num = 0, group_num = 0, group_data_num = 0, node_index = 0;
};

bool field_id(JNIEnv* e, jclass c, const char* name, const char* sig, jfieldID* out) {
  *out = e->GetFieldID(c, name, sig);
  return *out != nullptr && !e->ExceptionCheck();
}

bool read_fields(JNIEnv* e, jobject o, Fields* f) {
  jclass c = e->GetObjectClass(o);
  if (!c) return false;
  jfieldID id;
  bool ok = true;
  auto int_field = [&](const char* name, int* dst) {
    if (ok && (ok = field_id(e, c, name, "I", &id))) *dst = e->GetIntField(o, id);
  };
  int_field("chunkSize", &f->chunk_size);
  int_field("encodeDataNum", &f->encode_data_num);
  int_field("decodeDataNum", &f->decode_data_num);
  int_field("partialDecodeNum", &f->partial_decode_num);
  int_field("globalNum", &f->global_num);
  int_field("groupNum", &f->group_num);
  int_field("groupDataNum", &f->group_data_num);
  int_field("nodeIndex", &f->node_index);
  if (ok && (ok = field_id(e, c, "codeType", "C", &id))) f->code_type = static_cast<char>(e->GetCharField(o, id));
  if (ok && (ok = field_id(e, c, "multiNodeEncode", "Z", &id))) f->multinode = e->GetBooleanField(o, id) != 0;
  e->DeleteLocalRef(c);
  return ok;
}

// k of the stripe. The Java object keeps k only as encodeDataNum, except for
// CL multi-node encode where encodeDataNum is the node's group size
// (NativeCodec.java:84-91): node 1 holds the last group, so k follows. Other
// nodes take k from the scheme file the Java side itself was built from --
// every ECWide-C process reads "config/scheme.ini" relative to its working
// directory (DataNode.java:48, MasterNode.java:64) -- or from ECWIDE_K, and
// the file's scheme must agree with the object's fields.
bool stripe_k(JNIEnv* e, const Fields& f, int* k) {
  if (f.code_type != 'C' || !f.multinode) {
    *k = f.encode_data_num;
    return true;
  }
  if (f.node_index == 1) {
    *k = (f.group_num - 1) * f.group_data_num + f.encode_data_num;
    return true;
  }
  auto fits = [&](int kk) {  // CodingScheme.java:24-40: groupNum = ceil(k / groupDataNum)
    return kk >= 1 && f.group_data_num >= 1 && (kk + f.group_data_num - 1) / f.group_data_num == f.group_num;
  };
  if (const char* env = std::getenv("ECWIDE_K")) {
    if (!fits(std::atoi(env))) {
      throw_java(e, "java/lang/IllegalStateException",
                 std::string("ecwide: ECWIDE_K=") + env + " disagrees with groupNum/groupDataNum");
      return false;
    }
    *k = std::atoi(env);
    return true;
  }
  const char* path = std::getenv("ECWIDE_SCHEME");
  if (!path) path = "config/scheme.ini";
  ecw_scheme s;
  if (ecw_scheme_from_ini(path, &s) != ECW_OK) {
    throw_java(e, "java/lang/IllegalStateException",
               std::string("ecwide: multi-node CL encode on node > 1 needs the stripe's k: ") + path +
                   " not readable (run from the ECWide-C directory, or set ECWIDE_SCHEME / ECWIDE_K)");
    return false;
  }
  if (s.code_type != 'C' || s.group_data_num != f.group_data_num || s.global_parity_num != f.global_num ||
      s.chunk_size != static_cast<size_t>(f.chunk_size) || !fits(s.k)) {
    throw_java(e, "java/lang/IllegalStateException",
               std::string("ecwide: ") + path + " does not describe this NativeCodec's scheme");
    return false;
  }
  *k = s.k;
  return true;
}

// Codec for this NativeCodec instance; checks that the counts the Java ctor
// allocated for agree with the codec's (they are the same formulas).
ecw_codec* codec_of(JNIEnv* e, jobject o, ecw_codec_info* info) {
  Fields f;
  if (!read_fields(e, o, &f)) {
    throw_java(e, "java/lang/IllegalStateException", "ecwide: NativeCodec fields not readable");
    return nullptr;
  }
  int k = 0;
  if (!stripe_k(e, f, &k)) return nullptr;
  const int r = (f.code_type == 'C' || f.code_type == 'L') ? f.group_data_num : -1;
  // The RS and LRC ctors never store nodeIndex (NativeCodec.java:20-31,56-73):
  // it stays 0. RS does not use it; LRC used it only for decodeDataNum, which
  // is r unless the node sits in group r-1 (sic, :62-66) — pick a node that
  // gives the object's value.
  int node = f.node_index;
  if (f.code_type == 'R') node = 1;
  if (f.code_type == 'L' && node < 1)
    node = f.decode_data_num == f.group_data_num ? 1 : (f.group_data_num - 1) * f.group_data_num + 1;
  const char* lm = std::getenv("ECWIDE_LOCAL_MODE");
  const int local_mode = lm && std::strcmp(lm, "xor") == 0 ? ECW_LOCAL_XOR : ECW_LOCAL_LITERAL;
  const Key key{f.code_type, k, f.global_num, r, node, f.multinode ? 1 : 0, local_mode, f.chunk_size};
  ecw_codec* cd = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_codecs.find(key);
    if (it != g_codecs.end()) {
      cd = it->second;
    } else {
      ecw_scheme s;
      if (!check(e, ecw_scheme_init(&s, f.code_type, k, f.global_num, r, static_cast<size_t>(f.chunk_size)),
                 "scheme"))
        return nullptr;
      const char* dev = std::getenv("ECW_DEVICE");
      if (!check(e, ecw_codec_create(&s, node, f.multinode ? 1 : 0, local_mode, dev ? std::atoi(dev) : 0, &cd),
                 "codec"))
        return nullptr;
      g_codecs[key] = cd;
    }
  }
  if (!check(e, ecw_codec_get_info(cd, info), "codec info")) return nullptr;
  if (info->encode_data_num != f.encode_data_num || info->decode_data_num != f.decode_data_num ||
      (f.code_type != 'R' && f.code_type != 'L' && info->partial_decode_num != f.partial_decode_num)) {
    throw_java(e, "java/lang/IllegalStateException",
               "ecwide: NativeCodec counts disagree with the codec geometry");
    return nullptr;
  }
  return cd;
}

// Address of a direct ByteBuffer field of the NativeCodec object.
uint8_t* buffer_field(JNIEnv* e, jobject o, const char* name, size_t need) {
  jclass c = e->GetObjectClass(o);
  jfieldID id;
  const bool ok = field_id(e, c, name, "Ljava/nio/ByteBuffer;", &id);
  e->DeleteLocalRef(c);
  if (!ok) return nullptr;
  jobject b = e->GetObjectField(o, id);
  void* p = b ? e->GetDirectBufferAddress(b) : nullptr;
  const jlong cap = b ? e->GetDirectBufferCapacity(b) : -1;
  if (b) e->DeleteLocalRef(b);
  if (!p || cap < static_cast<jlong>(need)) {
    throw_java(e, "java/lang/IllegalStateException", std::string("ecwide: ") + name + " is not a direct buffer of " +
                                                          std::to_string(need) + " bytes");
    return nullptr;
  }
  return static_cast<uint8_t*>(p);
}

uint8_t* buffer_addr(JNIEnv* e, jobject b, size_t need, const char* what) {
  void* p = b ? e->GetDirectBufferAddress(b) : nullptr;
  const jlong cap = b ? e->GetDirectBufferCapacity(b) : -1;
  if (!p || cap < static_cast<jlong>(need)) {
    throw_java(e, "java/lang/IllegalArgumentException",
               std::string("ecwide: ") + what + " is not a direct ByteBuffer of chunkSize bytes");
    return nullptr;
  }
  return static_cast<uint8_t*>(p);
}

// The first n direct-buffer addresses of a ByteBuffer[] (NativeCodec.cc:158-167).
bool buffer_array(JNIEnv* e, jobjectArray a, int n, size_t need, const char* what, std::vector<uint8_t*>* out) {
  if (!a || e->GetArrayLength(a) < n) {
    throw_java(e, "java/lang/IllegalArgumentException",
               std::string("ecwide: ") + what + " holds fewer than " + std::to_string(n) + " buffers");
    return false;
  }
  out->resize(n);
  for (int i = 0; i < n; ++i) {
    jobject b = e->GetObjectArrayElement(a, i);
    (*out)[i] = buffer_addr(e, b, need, what);
    if (b) e->DeleteLocalRef(b);
    if (!(*out)[i]) return false;
  }
  return true;
}

}  // namespace

extern "C" {

// NativeCodec.cc:12-64 (generateEncodeMatrix): the k x m Cauchy rows.
JNIEXPORT void JNICALL Java_NativeCodec_generateEncodeMatrix(JNIEnv* e, jobject o) {
  ecw_codec_info in;
  ecw_codec* cd = codec_of(e, o, &in);
  if (!cd) return;
  const size_t n = static_cast<size_t>(in.encode_data_num) * in.global_num;
  if (uint8_t* dst = buffer_field(e, o, "encodeMatrix", n)) check(e, ecw_codec_encode_matrix(cd, dst, n), "encodeMatrix");
}

// NativeCodec.cc:66-88 (initEncodeTable): ec_init_tables layout.
JNIEXPORT void JNICALL Java_NativeCodec_initEncodeTable(JNIEnv* e, jobject o) {
  ecw_codec_info in;
  ecw_codec* cd = codec_of(e, o, &in);
  if (!cd) return;
  const size_t n = 32 * static_cast<size_t>(in.encode_data_num) * in.global_num;
  if (uint8_t* dst = buffer_field(e, o, "encodeGftbl", n)) check(e, ecw_codec_encode_gftbl(cd, dst, n), "encodeGftbl");
}

// NativeCodec.cc:90-111 (initDecodeTable): all-ones row.
JNIEXPORT void JNICALL Java_NativeCodec_initDecodeTable(JNIEnv* e, jobject o) {
  ecw_codec_info in;
  ecw_codec* cd = codec_of(e, o, &in);
  if (!cd) return;
  const size_t n = 32 * static_cast<size_t>(in.decode_data_num);
  if (uint8_t* dst = buffer_field(e, o, "decodeGftbl", n)) check(e, ecw_codec_decode_gftbl(cd, dst, n), "decodeGftbl");
}

// NativeCodec.cc:113-135 (initPartialDecodeTable).
JNIEXPORT void JNICALL Java_NativeCodec_initPartialDecodeTable(JNIEnv* e, jobject o) {
  ecw_codec_info in;
  ecw_codec* cd = codec_of(e, o, &in);
  if (!cd) return;
  const size_t n = 32 * static_cast<size_t>(in.partial_decode_num);
  if (uint8_t* dst = buffer_field(e, o, "partialDecodeGftbl", n))
    check(e, ecw_codec_partial_decode_gftbl(cd, dst, n), "partialDecodeGftbl");
}

// NativeCodec.cc:137-219 (encodeData): parity = [G_0..G_{m-1}, L_0..] (BufferUnit.java:60-68).
JNIEXPORT void JNICALL Java_NativeCodec_encodeData(JNIEnv* e, jobject o, jobjectArray data, jobjectArray parity) {
  ecw_codec_info in;
  ecw_codec* cd = codec_of(e, o, &in);
  if (!cd) return;
  std::vector<uint8_t*> d, p;
  if (!buffer_array(e, data, in.encode_data_num, in.chunk_size, "data", &d) ||
      !buffer_array(e, parity, in.parity_num, in.chunk_size, "parity", &p))
    return;
  check(e, ecw_encode(cd, d.data(), p.data(), in.chunk_size), "encodeData");
}

// NativeCodec.cc:221-249 (decodeData): target = XOR of decodeDataNum buffers.
JNIEXPORT void JNICALL Java_NativeCodec_decodeData(JNIEnv* e, jobject o, jobjectArray data, jobject target) {
  ecw_codec_info in;
  ecw_codec* cd = codec_of(e, o, &in);
  if (!cd) return;
  std::vector<uint8_t*> d;
  if (!buffer_array(e, data, in.decode_data_num, in.chunk_size, "data", &d)) return;
  uint8_t* t = buffer_addr(e, target, in.chunk_size, "target");
  if (t) check(e, ecw_decode(cd, d.data(), t, in.chunk_size), "decodeData");
}

// NativeCodec.cc:251-282 (partialDecodeData): target = XOR of partialDecodeNum buffers.
JNIEXPORT void JNICALL Java_NativeCodec_partialDecodeData(JNIEnv* e, jobject o, jobjectArray data, jobject target) {
  ecw_codec_info in;
  ecw_codec* cd = codec_of(e, o, &in);
  if (!cd) return;
  std::vector<uint8_t*> d;
  if (!buffer_array(e, data, in.partial_decode_num, in.chunk_size, "data", &d)) return;
  uint8_t* t = buffer_addr(e, target, in.chunk_size, "target");
  if (t) check(e, ecw_partial_decode(cd, d.data(), t, in.chunk_size), "partialDecodeData");
}

// NativeCodec.cc:284-323 (xorIntemediate): target[i] ^= source[i], i < globalNum.
JNIEXPORT void JNICALL Java_NativeCodec_xorIntemediate(JNIEnv* e, jobject o, jobjectArray source, jobjectArray target) {
  ecw_codec_info in;
  ecw_codec* cd = codec_of(e, o, &in);
  if (!cd) return;
  std::vector<uint8_t*> s, t;
  if (!buffer_array(e, source, in.global_num, in.chunk_size, "source", &s) ||
      !buffer_array(e, target, in.global_num, in.chunk_size, "target", &t))
    return;
  const char* lit = std::getenv("ECWIDE_XORI_LITERAL");
  const bool first = !g_xori_called.exchange(true);
  if (first && !(lit && std::strcmp(lit, "0") == 0)) {
    // the reference's first call in the process runs with an all-zero table
    for (uint8_t* dst : t) std::memset(dst, 0, in.chunk_size);
    return;
  }
  check(e, ecw_xor_intermediate(cd, s.data(), t.data(), in.chunk_size), "xorIntemediate");
}

}  // extern "C"
