/* ECWide-H-style concurrent callers of the ISA-L shim (libecw_isal.so):
 * T pthreads each issue N synchronous ec_encode_data calls on 4 KiB chunks
 * (g_encode's shape, ECWide-H/proxy/encode.cpp:145-175: GK=11, 3 parities).
 *   gcc -O2 -o shim_bench shim_bench.c -L../../ecwide_amd -lecw_isal -lpthread \
 *       -Wl,-rpath,$PWD/../../ecwide_amd
 *   ./shim_bench [threads] [calls per thread] [seq]
 * With "seq" every iteration is ECWide-H's whole per-chunk call mix
 * (encode.cpp:113-238): l_encode (XOR of LK=11 via gf_gen_rs_matrix's all-ones
 * row), g_encode (Cauchy 11 -> 3), l_middle (XOR of 4), l_decode (XOR of 5),
 * each rebuilding its matrix and tables as the reference does. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

void gf_gen_cauchy1_matrix(unsigned char* a, int m, int k);
void gf_gen_rs_matrix(unsigned char* a, int m, int k);
void ec_init_tables(int k, int rows, unsigned char* a, unsigned char* g_tbls);
void ec_encode_data(int len, int k, int rows, unsigned char* g_tbls, unsigned char** data, unsigned char** coding);
int ecw_isal_last_status(void);

enum { K = 11, M = 3, LEN = 4096 };
static unsigned char tbl[32 * K * M];
static int calls, seq;

/* one ECWide-H call: matrix and tables rebuilt per call, as encode.cpp does */
static void call(int k, int m, int cauchy, unsigned char** d, unsigned char** p) {
  unsigned char mat[(11 + 3) * 11], t[32 * 11 * 3];
  if (cauchy)
    gf_gen_cauchy1_matrix(mat, k + m, k);
  else
    gf_gen_rs_matrix(mat, k + m, k);
  ec_init_tables(k, m, mat + k * k, t);
  ec_encode_data(LEN, k, m, t, d, p);
}

static void* worker(void* arg) {
  unsigned seed = (unsigned)(size_t)arg;
  unsigned char* buf = malloc((size_t)(K + M) * LEN);
  unsigned char* d[K];
  unsigned char* p[M];
  for (int j = 0; j < K; ++j) d[j] = buf + (size_t)j * LEN;
  for (int i = 0; i < M; ++i) p[i] = buf + (size_t)(K + i) * LEN;
  for (size_t i = 0; i < (size_t)K * LEN; ++i) buf[i] = (unsigned char)rand_r(&seed);
  for (int c = 0; c < calls; ++c) {
    if (seq) {
      call(11, 1, 0, d, p);      /* l_encode */
      call(11, 3, 1, d, p);      /* g_encode */
      call(4, 1, 0, d, p + 1);   /* l_middle */
      call(5, 1, 0, d, p + 2);   /* l_decode */
    } else {
      ec_encode_data(LEN, K, M, tbl, d, p);
    }
    if (ecw_isal_last_status() != 0) {
      fprintf(stderr, "call failed\n");
      exit(1);
    }
  }
  free(buf);
  return NULL;
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 4;
  calls = argc > 2 ? atoi(argv[2]) : 500;
  seq = argc > 3 && strcmp(argv[3], "seq") == 0;
  unsigned char full[(K + M) * K];
  gf_gen_cauchy1_matrix(full, K + M, K);
  ec_init_tables(K, M, full + K * K, tbl);
  pthread_t th[256];
  worker((void*)1);  /* warm-up: codec, device, staging */
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, (void*)(size_t)(t + 2));
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &b);
  const double s = (b.tv_sec - a.tv_sec) + (b.tv_nsec - a.tv_nsec) * 1e-9;
  const double n = (double)threads * calls;
  if (seq)
    printf("shim, %d threads x %d ECWide-H call sequences (4 calls, 37 x 4 KiB): %.2f GB/s, %.1f us per sequence "
           "per thread\n", threads, calls, n * 37 * LEN / s / 1e9, s / calls * 1e6);
  else
    printf("shim, %d threads x %d calls: %.0f stripes/s, %.2f GB/s of (k+m)*4 KiB, %.1f us per call per thread\n",
           threads, calls, n / s, n * (K + M) * LEN / s / 1e9, s / calls * 1e6);
  return 0;
}
