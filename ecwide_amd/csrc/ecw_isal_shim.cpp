// libecw_isal.so — ISA-L erasure-code API on the MI355X engine.
//
// ECWide-H calls ISA-L directly (ECWide-H/proxy/encode.cpp:113-238:
// gf_gen_rs_matrix / gf_gen_cauchy1_matrix, ec_init_tables, ec_encode_data),
// as does ECWide-C's NativeCodec.cc. Linking this library instead of libisal
// moves those calls onto the GPU without touching the callers. Signatures
// follow isal:include/erasure_code.h (ISA-L 2.14.0).
//
// The matrix / table functions are pure host computations. ec_encode_data
// recovers the coefficient matrix from the 32-byte tables (entry 1 of each
// table is c*1 = c, exactly what ec_encode_data_base reads,
// isal:erasure_code/ec_base.c:290-305) and runs a cached matrix codec
// (ecw_matrix_codec_create) through the host-memory pipeline.
//
// ECWide-H calls ec_encode_data on 4 KiB chunks from four proxy threads
// (ECWide-H/proxy/proxy.cpp:2001-2012). Each call is one synchronous request
// to libecwide's resident request service (ecw_encode -> svc::serve), which
// serves concurrent callers on separate slots. With the service off
// (ECW_SERVICE=0) one GPU round trip costs far more than 4 KiB of work, so
// concurrent callers are batched instead (group commit): a call joins the
// pending list of its (codec, len); if no batch of that key is running, the
// caller runs everything pending as one ecw_encode_stripes call (one launch,
// packed copies); otherwise it waits and is picked up by the next batch. A
// lone caller runs at once -- there is no timer. ECW_ISAL_BATCH=1/0 forces
// batching on/off.
//
// The ISA-L functions return void; a failure is reported on stderr and by
// ecw_isal_last_status() (per thread), never by exit().
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ecwide.h"
#include "ecw_gf.hpp"

namespace {

// Pending calls of one (codec, len); see the group commit above.
struct Batcher {
  struct Req {
    unsigned char** data;
    unsigned char** coding;
    int status = ECW_OK;
    bool done = false;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Req*> pending;
  bool running = false;
};

struct Cache {
  std::mutex mu;
  std::map<std::string, ecw_codec*> codecs;  // key: k, rows, matrix bytes
  std::map<std::pair<ecw_codec*, int>, Batcher*> batchers;
  ~Cache() {
    for (auto& kv : batchers) delete kv.second;
    for (auto& kv : codecs) ecw_codec_destroy(kv.second);
  }
};

Cache& cache() {
  static Cache c;  // the only state: a lookup cache of immutable codecs
  return c;
}

thread_local int t_status = ECW_OK;

int device_from_env() {
  const char* e = std::getenv("ECW_DEVICE");
  return e ? std::atoi(e) : 0;
}

ecw_codec* codec_for(int k, int rows, const unsigned char* gftbls) {
  std::string key(reinterpret_cast<const char*>(&k), sizeof k);
  key.append(reinterpret_cast<const char*>(&rows), sizeof rows);
  std::vector<uint8_t> m(static_cast<size_t>(k) * rows);
  for (size_t i = 0; i < m.size(); ++i) m[i] = gftbls[i * 32 + 1];
  key.append(reinterpret_cast<const char*>(m.data()), m.size());
  Cache& c = cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.codecs.find(key);
  if (it != c.codecs.end()) return it->second;
  ecw_codec* cd = nullptr;
  t_status = ecw_matrix_codec_create(m.data(), k, rows, device_from_env(), &cd);
  if (t_status != ECW_OK) return nullptr;
  c.codecs.emplace(key, cd);
  return cd;
}

// Group commit pays off only without the resident request service: the
// service gives each concurrent caller a slot of its own (15 us per 4 KiB call
// from 4 threads at once, against 70 us when batched into launches; DESIGN.md
// section 8). ECW_ISAL_BATCH=1 / 0 forces it on / off.
bool batching_on() {
  static const bool on = [] {
    const char* e = std::getenv("ECW_ISAL_BATCH");
    if (e) return e[0] != '0';
    const char* s = std::getenv("ECW_SERVICE");
    return s && s[0] == '0';
  }();
  return on;
}

Batcher& batcher_for(ecw_codec* cd, int len) {
  Cache& c = cache();
  std::lock_guard<std::mutex> lk(c.mu);
  Batcher*& b = c.batchers[{cd, len}];
  if (!b) b = new Batcher();
  return *b;
}

int encode_batched(ecw_codec* cd, int len, int k, int rows, unsigned char** data, unsigned char** coding) {
  Batcher& b = batcher_for(cd, len);
  Batcher::Req r{data, coding};
  std::unique_lock<std::mutex> lk(b.mu);
  b.pending.push_back(&r);
  while (!r.done) {
    if (b.running) {
      b.cv.wait(lk);
      continue;
    }
    b.running = true;
    std::vector<Batcher::Req*> batch;
    batch.swap(b.pending);
    lk.unlock();
    std::vector<const uint8_t*> dp;
    std::vector<uint8_t*> pp;
    dp.reserve(batch.size() * k);
    pp.reserve(batch.size() * rows);
    for (const Batcher::Req* q : batch) {
      dp.insert(dp.end(), q->data, q->data + k);
      pp.insert(pp.end(), q->coding, q->coding + rows);
    }
    const int st = ecw_encode_stripes(cd, static_cast<int>(batch.size()), dp.data(), pp.data(),
                                      static_cast<size_t>(len));
    lk.lock();
    for (Batcher::Req* q : batch) {
      q->status = st;
      q->done = true;
    }
    b.running = false;
    b.cv.notify_all();
  }
  return r.status;
}

void report(const char* fn, int st) {
  t_status = st;
  if (st != ECW_OK) std::fprintf(stderr, "libecw_isal: %s failed: %s (%d)\n", fn, ecw_status_string(st), st);
}

}  // namespace

extern "C" {

int ecw_isal_last_status(void) { return t_status; }

unsigned char gf_mul(unsigned char a, unsigned char b) { return ecw::gf_mul(a, b); }

unsigned char gf_inv(unsigned char a) { return ecw::gf_inv(a); }

// isal:erasure_code/ec_base.c:62-79
void gf_gen_rs_matrix(unsigned char* a, int m, int k) {
  unsigned char p, gen = 1;
  std::memset(a, 0, static_cast<size_t>(k) * m);
  for (int i = 0; i < k; ++i) a[k * i + i] = 1;
  for (int i = k; i < m; ++i) {
    p = 1;
    for (int j = 0; j < k; ++j) {
      a[k * i + j] = p;
      p = ecw::gf_mul(p, gen);
    }
    gen = ecw::gf_mul(gen, 2);
  }
}

// isal:erasure_code/ec_base.c:81-97
void gf_gen_cauchy1_matrix(unsigned char* a, int m, int k) {
  std::memset(a, 0, static_cast<size_t>(k) * m);
  for (int i = 0; i < k; ++i) a[k * i + i] = 1;
  unsigned char* p = a + static_cast<size_t>(k) * k;
  for (int i = k; i < m; ++i)
    for (int j = 0; j < k; ++j) *p++ = ecw::gf_inv(static_cast<unsigned char>(i ^ j));
}

// isal:erasure_code/ec_base.c:99-155 — Gauss-Jordan inverse over GF(2^8);
// returns 0, or -1 when the matrix is singular (in_mat is destroyed, as in ISA-L)
int gf_invert_matrix(unsigned char* in_mat, unsigned char* out_mat, const int n) {
  if (n <= 0) return -1;
  std::memset(out_mat, 0, static_cast<size_t>(n) * n);
  for (int i = 0; i < n; ++i) out_mat[i * n + i] = 1;
  for (int i = 0; i < n; ++i) {
    if (in_mat[i * n + i] == 0) {  // find a row below with a non-zero pivot and swap
      int j = i + 1;
      while (j < n && in_mat[j * n + i] == 0) ++j;
      if (j == n) return -1;
      for (int c = 0; c < n; ++c) {
        std::swap(in_mat[i * n + c], in_mat[j * n + c]);
        std::swap(out_mat[i * n + c], out_mat[j * n + c]);
      }
    }
    const unsigned char inv = ecw::gf_inv(in_mat[i * n + i]);
    for (int c = 0; c < n; ++c) {
      in_mat[i * n + c] = ecw::gf_mul(in_mat[i * n + c], inv);
      out_mat[i * n + c] = ecw::gf_mul(out_mat[i * n + c], inv);
    }
    for (int j = 0; j < n; ++j) {
      if (j == i) continue;
      const unsigned char f = in_mat[j * n + i];
      if (!f) continue;
      for (int c = 0; c < n; ++c) {
        in_mat[j * n + c] ^= ecw::gf_mul(f, in_mat[i * n + c]);
        out_mat[j * n + c] ^= ecw::gf_mul(f, out_mat[i * n + c]);
      }
    }
  }
  return 0;
}

// isal:erasure_code/ec_base.c:157-262 (table layout)
void gf_vect_mul_init(unsigned char c, unsigned char* tbl) { ecw::vect_mul_table(c, tbl); }

// isal:erasure_code/ec_highlevel_func.c:33-43
void ec_init_tables(int k, int rows, unsigned char* a, unsigned char* g_tbls) {
  for (int i = 0; i < rows * k; ++i) ecw::vect_mul_table(a[i], g_tbls + 32 * static_cast<size_t>(i));
}

// isal:include/erasure_code.h:98 — on the GPU
void ec_encode_data(int len, int k, int rows, unsigned char* g_tbls, unsigned char** data,
                    unsigned char** coding) {
  if (len <= 0 || rows <= 0) return;
  ecw_codec* cd = codec_for(k, rows, g_tbls);
  if (!cd) return report("ec_encode_data", t_status);
  if (batching_on()) return report("ec_encode_data", encode_batched(cd, len, k, rows, data, coding));
  report("ec_encode_data", ecw_encode(cd, data, coding, static_cast<size_t>(len)));
}

// the dispatcher's explicit variants resolve to the same GPU path
void ec_encode_data_base(int len, int k, int rows, unsigned char* g_tbls, unsigned char** data,
                         unsigned char** coding) {
  ec_encode_data(len, k, rows, g_tbls, data, coding);
}

}  // extern "C"
