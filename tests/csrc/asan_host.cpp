// Host-side sanitizer driver (tests/test_sanitize.py): built with
// -fsanitize=address,undefined on the host side together with
// ecw_codec.cpp, the kernels' host stubs, the ISA-L shim, the JNI natives and
// the JNI test double, then run on a host WITHOUT a GPU. It drives every
// host-only path (scheme parsing, codec geometry and tables, repair fan-in,
// ISA-L matrix/table functions, the JNI natives' field handling) and every
// device entry point up to its ECW_EDEVICE return, plus the ISA-L shim's
// group-commit batcher from several threads. Exit status 0 = all checks held
// and the sanitizers stayed quiet.
#include <jni.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ecwide.h"
#include "../../ecwide_amd/csrc/ecw_internal.hpp"  // FastDiv (the kernels' tile -> stripe division)

extern "C" {
// libecw_isal.so (ecw_isal_shim.cpp), isal:include/erasure_code.h signatures
unsigned char gf_mul(unsigned char, unsigned char);
unsigned char gf_inv(unsigned char);
void gf_gen_rs_matrix(unsigned char*, int, int);
void gf_gen_cauchy1_matrix(unsigned char*, int, int);
int gf_invert_matrix(unsigned char*, unsigned char*, const int);
void gf_vect_mul_init(unsigned char, unsigned char*);
void ec_init_tables(int, int, unsigned char*, unsigned char*);
void ec_encode_data(int, int, int, unsigned char*, unsigned char**, unsigned char**);
int ecw_isal_last_status(void);
// tests/jni/jvm_double.cpp
void* jd_env();
void* jd_object(const char*);
void jd_set_prim(void*, const char*, const char*, long long);
void jd_set_object(void*, const char*, void*);
void* jd_buffer(void*, long long);
void* jd_array(int);
void jd_array_set(void*, int, void*);
const char* jd_exception();
void jd_clear_exception();
long long jd_live_refs();
// ecw_jni.cpp (NativeCodec.h:15-72)
JNIEXPORT void JNICALL Java_NativeCodec_generateEncodeMatrix(JNIEnv*, jobject);
JNIEXPORT void JNICALL Java_NativeCodec_initEncodeTable(JNIEnv*, jobject);
JNIEXPORT void JNICALL Java_NativeCodec_initDecodeTable(JNIEnv*, jobject);
JNIEXPORT void JNICALL Java_NativeCodec_initPartialDecodeTable(JNIEnv*, jobject);
JNIEXPORT void JNICALL Java_NativeCodec_encodeData(JNIEnv*, jobject, jobjectArray, jobjectArray);
JNIEXPORT void JNICALL Java_NativeCodec_decodeData(JNIEnv*, jobject, jobjectArray, jobject);
}

static int g_checks = 0, g_fail = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    ++g_checks;                                                           \
    if (!(c)) {                                                           \
      ++g_fail;                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
    }                                                                     \
  } while (0)

static void schemes() {
  ecw_scheme s;
  CHECK(ecw_scheme_from_ini_text("codeType = CL\nk = 32\ngroupDataNum = 11\nglobalParityNum = 3\n"
                                 "chunkSizeBits = 26\n",
                                 &s) == ECW_OK);
  CHECK(s.k == 32 && s.group_num == 3 && s.chunk_size == (size_t(1) << 26) && s.rack_nodes_num == 4);
  const char* bad[] = {"", "k = 3\n", "codeType = CL\nk = x\nchunkSizeBits = 3\nglobalParityNum = 1\n",
                       "k = 3\nchunkSizeBits = 40\nglobalParityNum = 1\n", "garbage line\n",
                       "codeType = CL\nk = 9\nchunkSizeBits = 3\nglobalParityNum = 1\n",
                       "k = 99999999999\nchunkSizeBits = 3\nglobalParityNum = 1\n"};
  for (const char* t : bad) CHECK(ecw_scheme_from_ini_text(t, &s) == ECW_EPARSE);
  CHECK(ecw_scheme_from_ini("/nonexistent/scheme.ini", &s) == ECW_EIO);
  CHECK(ecw_scheme_from_ini_text(nullptr, &s) == ECW_EINVAL);
  for (char t : {'R', 'T', 'L', 'C'}) CHECK(ecw_scheme_init(&s, t, 20, 3, 5, 4096) == ECW_OK);
  CHECK(ecw_scheme_init(&s, 'X', 20, 3, 5, 4096) == ECW_EINVAL);
  CHECK(ecw_scheme_init(&s, 'C', 250, 7, 5, 4096) == ECW_EINVAL);
  CHECK(ecw_scheme_init(&s, 'C', 20, 3, 0, 4096) == ECW_EINVAL);
  CHECK(ecw_scheme_init(&s, 'T', 20, 0, 0, 4096) == ECW_EINVAL);
}

static void codecs() {
  struct Case {
    char t;
    int k, m, r, node, multi;
  } cases[] = {{'C', 128, 3, 27, 1, 0}, {'C', 32, 3, 11, 4, 0}, {'C', 32, 3, 11, 2, 1}, {'C', 250, 6, 50, 1, 0},
               {'L', 12, 2, 4, 5, 0},   {'T', 12, 3, 0, 4, 0},   {'R', 11, 3, 0, 1, 0},   {'C', 3, 12, 2, 1, 0},
               {'C', 1, 1, 1, 1, 0},    {'R', 200, 56, 0, 1, 0}};
  for (const Case& c : cases) {
    ecw_scheme s;
    CHECK(ecw_scheme_init(&s, c.t, c.k, c.m, c.r, 8192) == ECW_OK);
    for (int mode : {ECW_LOCAL_XOR, ECW_LOCAL_LITERAL}) {
      ecw_codec* cd = nullptr;
      CHECK(ecw_codec_create(&s, c.node, c.multi, mode, 0, &cd) == ECW_OK && cd);
      if (!cd) continue;
      ecw_codec_info in;
      CHECK(ecw_codec_get_info(cd, &in) == ECW_OK);
      const int edn = in.encode_data_num, m = in.global_num;
      std::vector<uint8_t> mat(static_cast<size_t>(edn) * m), tb(32 * mat.size()), dt(32 * in.decode_data_num),
          pd(32 * static_cast<size_t>(in.partial_decode_num));
      CHECK(ecw_codec_encode_matrix(cd, mat.data(), mat.size()) == ECW_OK);
      CHECK(ecw_codec_encode_matrix(cd, mat.data(), mat.size() + 1) == ECW_EINVAL);
      CHECK(ecw_codec_encode_gftbl(cd, tb.data(), tb.size()) == ECW_OK);
      CHECK(ecw_codec_decode_gftbl(cd, dt.data(), dt.size()) == ECW_OK);
      if (c.t == 'C' || c.t == 'T') CHECK(ecw_codec_partial_decode_gftbl(cd, pd.data(), pd.size()) == ECW_OK);
      // the ISA-L layout of the codec's tables equals ec_init_tables of its matrix
      std::vector<uint8_t> tb2(tb.size());
      if (!mat.empty()) ec_init_tables(edn, m, mat.data(), tb2.data());
      CHECK(tb == tb2);
      int idx[256];
      const int nb = edn + in.parity_num;
      for (int b = 0; b < nb; ++b) {
        const int n = ecw_repair_sources(cd, b, idx, 256);
        if (c.multi || (c.t != 'C' && c.t != 'L')) {
          CHECK(n == ECW_EUNSUPPORTED);
        } else if (b >= edn && b < edn + m) {
          CHECK(n == ECW_EUNSUPPORTED);  // G repair: "not yet" in the reference
        } else {
          CHECK(n > 0);
          for (int i = 0; i < n; ++i) CHECK(idx[i] >= 0 && idx[i] < nb && idx[i] != b);
        }
      }
      CHECK(ecw_repair_sources(cd, nb, idx, 256) ==
            ((c.multi || (c.t != 'C' && c.t != 'L')) ? ECW_EUNSUPPORTED : ECW_EINVAL));
      CHECK(ecw_codec_set_xori_mode(cd, ECW_XORI_LITERAL) == ECW_OK);
      CHECK(ecw_codec_set_xori_mode(cd, 7) == ECW_EINVAL);
      // every device-side path stops at ECW_EDEVICE (no GPU here), after validation
      const size_t len = 4096 + 48;
      std::vector<std::vector<uint8_t>> blk(nb + 1, std::vector<uint8_t>(len, 0x5A));
      std::vector<const uint8_t*> ci(nb + 1);
      std::vector<uint8_t*> po(nb + 1);
      for (int i = 0; i <= nb; ++i) ci[i] = po[i] = blk[i].data();
      CHECK(ecw_encode(cd, ci.data(), po.data() + edn, len) == ECW_EDEVICE);
      CHECK(ecw_encode_stripes(cd, 1, ci.data(), po.data() + edn, len) == ECW_EDEVICE);
      CHECK(ecw_encode(cd, ci.data(), po.data() + edn, size_t(1) << 23) != ECW_OK);
      CHECK(ecw_decode(cd, ci.data(), po[nb], len) == ECW_EDEVICE);
      CHECK(ecw_xor_intermediate(cd, ci.data(), po.data(), len) == ECW_EDEVICE);
      if (!c.multi && (c.t == 'C' || c.t == 'L') && mode == ECW_LOCAL_XOR)
        CHECK(ecw_repair(cd, ci.data(), 0, po[nb], len) == ECW_EDEVICE);
      uint8_t* fake = reinterpret_cast<uint8_t*>(uintptr_t(1) << 40);
      CHECK(ecw_encode_batch_dev(cd, fake, 8192, 8192 * nb, 2, 8192, nullptr) == ECW_EDEVICE);
      CHECK(ecw_encode_batch_dev(cd, fake + 1, 8192, 8192 * nb, 2, 8192, nullptr) == ECW_EALIGN);
      CHECK(ecw_encode_batch_dev(cd, fake, 4096, 4096 * nb, 2, 8192, nullptr) == ECW_EINVAL);
      ecw_codec_destroy(cd);
    }
  }
  ecw_scheme s;
  ecw_codec* cd = nullptr;
  CHECK(ecw_scheme_init(&s, 'C', 8, 2, 4, 4096) == ECW_OK);
  CHECK(ecw_codec_create(&s, 0, 0, ECW_LOCAL_XOR, 0, &cd) == ECW_EINVAL && !cd);
  CHECK(ecw_codec_create(&s, 1, 0, 9, 0, &cd) == ECW_EINVAL && !cd);
  CHECK(ecw_device_count() == 0);
  uint8_t dst[64];
  CHECK(ecw_fill_random_pieces_dev(0, dst, 16, 16, 1, 1, 64, 16, 16, 0, 1, 0, 0, nullptr) == ECW_EDEVICE ||
        ecw_fill_random_pieces_dev(0, dst, 16, 16, 1, 1, 64, 16, 16, 0, 1, 0, 0, nullptr) == ECW_EALIGN);
  const uint8_t mat[6] = {1, 2, 3, 4, 5, 6};
  CHECK(ecw_matrix_codec_create(mat, 3, 2, 0, &cd) == ECW_OK && cd);
  ecw_codec_destroy(cd);
  CHECK(ecw_matrix_codec_create(mat, 0, 2, 0, &cd) == ECW_EINVAL);
}

static void isal_shim() {
  for (int a = 0; a < 256; ++a) {
    if (a) CHECK(gf_mul(static_cast<unsigned char>(a), gf_inv(static_cast<unsigned char>(a))) == 1);
  }
  const int k = 11, n = 14;
  std::vector<unsigned char> rs(n * k), ca(n * k), inv(k * k), sq(k * k);
  gf_gen_rs_matrix(rs.data(), n, k);
  gf_gen_cauchy1_matrix(ca.data(), n, k);
  // erase data rows 0..2, keep rows 3..13 of the Cauchy code: invertible
  for (int i = 0; i < k; ++i) std::memcpy(&sq[i * k], &ca[(i + 3) * k], k);
  CHECK(gf_invert_matrix(sq.data(), inv.data(), k) == 0);
  std::vector<unsigned char> z(k * k, 0);
  CHECK(gf_invert_matrix(z.data(), inv.data(), k) == -1);
  CHECK(gf_invert_matrix(z.data(), inv.data(), 0) == -1);
  unsigned char tbl[32];
  gf_vect_mul_init(0x53, tbl);
  CHECK(tbl[1] == 0x53);
  // ECWide-H's g_encode shape from 8 threads: the group-commit batcher hands
  // every caller the (device) failure of its batch, nobody hangs
  std::vector<unsigned char> g(32 * k * 3);
  ec_init_tables(k, 3, ca.data() + k * k, g.data());
  std::vector<std::thread> th;
  std::vector<int> st(8, 1);
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      std::vector<std::vector<unsigned char>> blk(k + 3, std::vector<unsigned char>(4096, static_cast<unsigned char>(t)));
      std::vector<unsigned char*> d(k), p(3);
      for (int i = 0; i < k; ++i) d[i] = blk[i].data();
      for (int i = 0; i < 3; ++i) p[i] = blk[k + i].data();
      for (int rep = 0; rep < 20; ++rep) ec_encode_data(4096, k, 3, g.data(), d.data(), p.data());
      st[t] = ecw_isal_last_status();
    });
  for (auto& x : th) x.join();
  for (int s : st) CHECK(s == ECW_EDEVICE);
}

static void jni() {
  JNIEnv* env = static_cast<JNIEnv*>(jd_env());
  // CL(k=32, r=11, m=3) at node 1, fields as NativeCodec.java:75-99 sets them
  const int edn = 32, m = 3, ddn = 5, pdn = 4;
  void* o = jd_object("NativeCodec");
  const struct {
    const char* name;
    long long v;
  } ints[] = {{"chunkSize", 4096}, {"encodeDataNum", edn}, {"decodeDataNum", ddn}, {"partialDecodeNum", pdn},
              {"globalNum", m},    {"groupNum", 3},        {"groupDataNum", 11}, {"rackPerGroup", 3},
              {"nodeIndex", 1}};
  for (const auto& f : ints) jd_set_prim(o, f.name, "I", f.v);
  jd_set_prim(o, "codeType", "C", 'C');
  jd_set_prim(o, "multiNodeEncode", "Z", 0);
  std::vector<uint8_t> mat(edn * m), tb(32 * edn * m), dt(32 * ddn), pd(32 * pdn);
  jd_set_object(o, "encodeMatrix", jd_buffer(mat.data(), static_cast<long long>(mat.size())));
  jd_set_object(o, "encodeGftbl", jd_buffer(tb.data(), static_cast<long long>(tb.size())));
  jd_set_object(o, "decodeGftbl", jd_buffer(dt.data(), static_cast<long long>(dt.size())));
  jd_set_object(o, "partialDecodeGftbl", jd_buffer(pd.data(), static_cast<long long>(pd.size())));
  jobject jo = static_cast<jobject>(o);
  jd_clear_exception();
  Java_NativeCodec_generateEncodeMatrix(env, jo);
  Java_NativeCodec_initEncodeTable(env, jo);
  Java_NativeCodec_initDecodeTable(env, jo);
  Java_NativeCodec_initPartialDecodeTable(env, jo);
  CHECK(std::string(jd_exception()).empty());
  ecw_scheme s;
  ecw_codec* cd = nullptr;
  CHECK(ecw_scheme_init(&s, 'C', 32, 3, 11, 4096) == ECW_OK);
  CHECK(ecw_codec_create(&s, 1, 0, ECW_LOCAL_XOR, 0, &cd) == ECW_OK);
  std::vector<uint8_t> want(mat.size());
  CHECK(ecw_codec_encode_matrix(cd, want.data(), want.size()) == ECW_OK && want == mat);
  ecw_codec_destroy(cd);
  // encodeData: device failure -> a Java exception, no crash; a short array too
  std::vector<std::vector<uint8_t>> blk(edn + 6, std::vector<uint8_t>(4096, 1));
  void* da = jd_array(edn);
  void* pa = jd_array(6);
  for (int i = 0; i < edn; ++i) jd_array_set(da, i, jd_buffer(blk[i].data(), 4096));
  for (int i = 0; i < 6; ++i) jd_array_set(pa, i, jd_buffer(blk[edn + i].data(), 4096));
  jd_clear_exception();
  Java_NativeCodec_encodeData(env, jo, static_cast<jobjectArray>(da), static_cast<jobjectArray>(pa));
  CHECK(!std::string(jd_exception()).empty());
  void* shorta = jd_array(2);
  jd_clear_exception();
  Java_NativeCodec_decodeData(env, jo, static_cast<jobjectArray>(shorta), static_cast<jobject>(jd_buffer(blk[0].data(), 4096)));
  CHECK(!std::string(jd_exception()).empty());
  CHECK(jd_live_refs() == 0);
}

// ecw::fast_div == n / d for divisors 1..2^16, powers of two, large and
// extreme divisors, against edge and pseudo-random numerators
static void fastdiv() {
  std::vector<uint32_t> ds;
  for (uint32_t d = 1; d <= 65536; ++d) ds.push_back(d);
  for (int b = 17; b < 32; ++b) {
    ds.push_back(1u << b);
    ds.push_back((1u << b) - 1);
    ds.push_back((1u << b) + 1);
  }
  for (uint32_t d : {0x7FFFFFFFu, 0x80000000u, 0x80000001u, 0xFFFFFFFEu, 0xFFFFFFFFu, 3000000019u, 1234567891u}) ds.push_back(d);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  int bad = 0;
  for (uint32_t d : ds) {
    const ecw::FastDiv f = ecw::make_fastdiv(d);
    const uint32_t edge[] = {0u, 1u, d - 1, d, d + 1, 2 * d - 1, 2 * d, 0x7FFFFFFFu, 0x80000000u, 0xFFFFFFFEu, 0xFFFFFFFFu};
    for (uint32_t n : edge)
      if (ecw::fast_div(n, f) != n / d) ++bad;
    for (int i = 0; i < 64; ++i) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      const uint32_t n = static_cast<uint32_t>(x >> (i & 31));
      if (ecw::fast_div(n, f) != n / d) ++bad;
    }
  }
  CHECK(bad == 0);
  // launch ranges of the 32-bit tile numbering
  CHECK(ecw::stripes_per_launch(1) == 0x7FFFFFFF);
  CHECK(ecw::stripes_per_launch(2) == (1 << 30) - 1);
  CHECK(ecw::stripes_per_launch(16384) == (1 << 17) - 1);
  CHECK(ecw::stripes_per_launch(1ull << 31) == 1);
  for (uint64_t t : {1ull, 2ull, 3ull, 4097ull, 1ull << 20})
    CHECK(static_cast<uint64_t>(ecw::stripes_per_launch(t)) * t < (1ull << 31) &&
          (static_cast<uint64_t>(ecw::stripes_per_launch(t)) + 1) * t >= (1ull << 31));
}

// ecw_set_schedule / ecw_get_schedule from 8 threads at once (the launchers
// take one copy per launch under the same lock), out-of-range values refused;
// ecw_host_alloc / ecw_host_free without a GPU: status codes, nothing leaked.
static void schedule_and_host() {
  std::vector<std::thread> th;
  std::atomic<int> bad{0};
  for (int t = 0; t < 8; ++t)
    th.emplace_back([t, &bad] {
      for (int i = 0; i < 200; ++i) {
        ecw_schedule s = {1 << (i % 3), t & 1, 10 + (i % 3), 32 * (i % 2), -1, i % 2 ? 0 : -1, (t + i) & 1};
        if (ecw_set_schedule(&s) != ECW_OK) ++bad;
        ecw_schedule g;
        if (ecw_get_schedule(&g) != ECW_OK || (g.xor_skew != 1 && g.xor_skew != 2 && g.xor_skew != 4)) ++bad;
      }
    });
  for (auto& x : th) x.join();
  CHECK(bad == 0);
  ecw_schedule s = {3, -1, -1, -1, -1, -1, -1};
  CHECK(ecw_set_schedule(&s) == ECW_EINVAL);
  s = ecw_schedule{-1, -1, 30, -1, -1, -1, -1};
  CHECK(ecw_set_schedule(&s) == ECW_EINVAL);
  CHECK(ecw_set_schedule(nullptr) == ECW_OK);
  CHECK(ecw_get_schedule(&s) == ECW_OK && s.xor_skew == -1 && s.enc_window_width == -1);
  CHECK(ecw_get_schedule(nullptr) == ECW_EINVAL);
  void* p = reinterpret_cast<void*>(1);
  int node = 5;
  CHECK(ecw_host_alloc(0, 1 << 20, &p, &node) == ECW_EDEVICE && p == nullptr && node == -1);
  CHECK(ecw_host_alloc(0, 0, &p, nullptr) == ECW_EINVAL);
  CHECK(ecw_host_free(nullptr) == ECW_OK);
  CHECK(ecw_host_free(&node) == ECW_EINVAL);
  CHECK(ecw_device_numa_node(0) == -1);
  CHECK(ecw_host_alloc_node(0, 5000, 4096, &p, &node) == ECW_EINVAL);
  CHECK(ecw_host_alloc_node(0, 0, 4096, &p, &node) == ECW_EDEVICE && p == nullptr);
}

int main() {
  fastdiv();
  schemes();
  codecs();
  schedule_and_host();
  isal_shim();
  jni();
  std::printf("asan_host: %d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
