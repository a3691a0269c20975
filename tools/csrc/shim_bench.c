/* ECWide-H-style callers of ISA-L's API (tools only), on either backend:
 *   gpu: libecw_isal.so (the ISA-L-signature shim over the GPU engine)
 *   cpu: oracle/liboracle.so (the AVX2 nibble-pshufb port of ISA-L's
 *        gf_Nvect_dot_prod kernels; test infrastructure, the CPU baseline)
 * Build: gcc -O2 -o shim_bench shim_bench.c -ldl -lpthread
 * Run:   ./shim_bench BACKEND MODE THREADS CALLS     (from the repository root)
 * MODE
 *   calls  THREADS threads x CALLS synchronous ec_encode_data calls on 4 KiB
 *          chunks (g_encode's shape, ECWide-H/proxy/encode.cpp:145-175: GK=11,
 *          3 parities), tables made once
 *   seq    every iteration is ECWide-H's whole per-chunk mix
 *          (encode.cpp:113-238): l_encode (XOR of LK=11 through
 *          gf_gen_rs_matrix's all-ones row), g_encode (Cauchy 11 -> 3),
 *          l_middle (XOR of NODE=4), l_decode (XOR of 5), each rebuilding its
 *          matrix and tables as the reference does
 *   proxy  the proxy's own concurrency (ECWide-H/proxy/proxy.cpp:2001-2012,
 *          595, 766): THREADS threads per role, the roles running at once --
 *          the local_encode thread (l_encode), the global_encode thread
 *          (g_encode), the local_repair thread (l_decode) and the gather pool
 *          (l_middle) -- each making CALLS calls of its own function */
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef void (*gen_fn)(unsigned char*, int, int);
typedef void (*init_fn)(int, int, unsigned char*, unsigned char*);
typedef void (*enc_fn)(int, int, int, unsigned char*, unsigned char**, unsigned char**);
typedef int (*status_fn)(void);

static gen_fn gen_rs, gen_cauchy;
static init_fn init_tables;
static enc_fn encode_data;
static status_fn last_status;  /* gpu only */

enum { K = 11, M = 3, LEN = 4096 };
static unsigned char tbl[32 * K * M];
static int calls;

/* the four ECWide-H functions: sources, outputs, Cauchy (else the RS matrix's
 * all-ones row) */
static const struct {
  const char* name;
  int k, m, cauchy;
} kRole[4] = {{"l_encode", 11, 1, 0}, {"g_encode", 11, 3, 1}, {"l_middle", 4, 1, 0}, {"l_decode", 5, 1, 0}};

/* one ECWide-H call: matrix and tables rebuilt per call, as encode.cpp does */
static void call(int k, int m, int cauchy, unsigned char** d, unsigned char** p) {
  unsigned char mat[(11 + 3) * 11], t[32 * 11 * 3];
  if (cauchy)
    gen_cauchy(mat, k + m, k);
  else
    gen_rs(mat, k + m, k);
  init_tables(k, m, mat + k * k, t);
  encode_data(LEN, k, m, t, d, p);
}

static void check(void) {
  if (last_status && last_status() != 0) {
    fprintf(stderr, "call failed\n");
    exit(1);
  }
}

struct job {
  int mode;   /* 0 calls, 1 seq, 2 proxy */
  int role;   /* proxy: index into kRole */
  unsigned seed;
  double us;  /* per call, measured by the thread */
};

static double now(void) {
  struct timespec a;
  clock_gettime(CLOCK_MONOTONIC, &a);
  return a.tv_sec + a.tv_nsec * 1e-9;
}

static void* worker(void* arg) {
  struct job* j = arg;
  unsigned seed = j->seed;
  unsigned char* buf = malloc((size_t)(K + M) * LEN);
  unsigned char* d[K];
  unsigned char* p[M];
  for (int i = 0; i < K; ++i) d[i] = buf + (size_t)i * LEN;
  for (int i = 0; i < M; ++i) p[i] = buf + (size_t)(K + i) * LEN;
  for (size_t i = 0; i < (size_t)K * LEN; ++i) buf[i] = (unsigned char)rand_r(&seed);
  const double t0 = now();
  for (int c = 0; c < calls; ++c) {
    if (j->mode == 1) {
      for (int r = 0; r < 4; ++r) call(kRole[r].k, kRole[r].m, kRole[r].cauchy, d, p);
    } else if (j->mode == 2) {
      call(kRole[j->role].k, kRole[j->role].m, kRole[j->role].cauchy, d, p);
    } else {
      encode_data(LEN, K, M, tbl, d, p);
    }
    check();
  }
  j->us = (now() - t0) / calls * 1e6;
  free(buf);
  return NULL;
}

static void* sym(void* h, const char* name) {
  void* f = dlsym(h, name);
  if (!f) {
    fprintf(stderr, "missing symbol %s\n", name);
    exit(2);
  }
  return f;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s gpu|cpu calls|seq|proxy THREADS CALLS\n", argv[0]);
    return 2;
  }
  const int gpu = strcmp(argv[1], "gpu") == 0;
  const int mode = strcmp(argv[2], "seq") == 0 ? 1 : strcmp(argv[2], "proxy") == 0 ? 2 : 0;
  const int threads = atoi(argv[3]);
  calls = atoi(argv[4]);
  void* h = dlopen(gpu ? "ecwide_amd/libecw_isal.so" : "oracle/liboracle.so", RTLD_NOW);
  if (!h) {
    fprintf(stderr, "%s\n", dlerror());
    return 2;
  }
  gen_rs = (gen_fn)sym(h, gpu ? "gf_gen_rs_matrix" : "orc_gen_rs_matrix");
  gen_cauchy = (gen_fn)sym(h, gpu ? "gf_gen_cauchy1_matrix" : "orc_gen_cauchy1_matrix");
  init_tables = (init_fn)sym(h, gpu ? "ec_init_tables" : "orc_init_tables");
  encode_data = (enc_fn)sym(h, gpu ? "ec_encode_data" : "orc_encode_data_avx2");
  if (gpu) last_status = (status_fn)sym(h, "ecw_isal_last_status");
  unsigned char full[(K + M) * K];
  gen_cauchy(full, K + M, K);
  init_tables(K, M, full + K * K, tbl);
  const int n = mode == 2 ? 4 * threads : threads;
  pthread_t th[1024];
  struct job jobs[1024];
  if (n > 1024) return 2;
  {  /* warm-up: codecs, device, staging */
    struct job w = {mode == 2 ? 1 : mode, 0, 1, 0};
    int c = calls;
    calls = 50;
    worker(&w);
    if (mode == 2)
      for (int r = 0; r < 4; ++r) {
        w.role = r;
        worker(&w);
      }
    calls = c;
  }
  for (int t = 0; t < n; ++t) {
    jobs[t].mode = mode;
    jobs[t].role = t % 4;
    jobs[t].seed = (unsigned)t + 2;
  }
  const double a = now();
  for (int t = 0; t < n; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
  for (int t = 0; t < n; ++t) pthread_join(th[t], NULL);
  const double s = now() - a;
  const char* be = gpu ? "gpu (libecw_isal.so)" : "cpu (AVX2 port, oracle)";
  if (mode == 1) {
    printf("%s seq, %d threads x %d ECWide-H call sequences (4 calls, 37 x 4 KiB): %.2f GB/s, %.1f us per "
           "sequence per thread\n", be, threads, calls, (double)n * calls * 37 * LEN / s / 1e9, s / calls * 1e6);
  } else if (mode == 2) {
    double bytes = 0, us[4] = {0, 0, 0, 0};
    for (int t = 0; t < n; ++t) {
      bytes += (double)calls * (kRole[t % 4].k + kRole[t % 4].m) * LEN;
      us[t % 4] += jobs[t].us / threads;
    }
    printf("%s proxy, %d thread(s) per role, %d calls each: %.2f GB/s in all, %.0f calls/s; us per call: "
           "l_encode %.1f, g_encode %.1f, l_middle %.1f, l_decode %.1f\n", be, threads, calls, bytes / s / 1e9,
           n * (double)calls / s, us[0], us[1], us[2], us[3]);
  } else {
    printf("%s calls, %d threads x %d calls: %.0f stripes/s, %.2f GB/s of (k+m)*4 KiB, %.1f us per call per "
           "thread\n", be, threads, calls, n * (double)calls / s, (double)n * calls * (K + M) * LEN / s / 1e9,
           s / calls * 1e6);
  }
  return 0;
}
