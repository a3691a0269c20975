/* ECWide-H-style concurrent callers of the ISA-L shim (libecw_isal.so):
 * T pthreads each issue N synchronous ec_encode_data calls on 4 KiB chunks
 * (g_encode's shape, ECWide-H/proxy/encode.cpp:145-175: GK=11, 3 parities).
 *   gcc -O2 -o shim_bench shim_bench.c -L../../ecwide_amd -lecw_isal -lpthread \
 *       -Wl,-rpath,$PWD/../../ecwide_amd
 *   ./shim_bench [threads] [calls per thread] */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

void gf_gen_cauchy1_matrix(unsigned char* a, int m, int k);
void ec_init_tables(int k, int rows, unsigned char* a, unsigned char* g_tbls);
void ec_encode_data(int len, int k, int rows, unsigned char* g_tbls, unsigned char** data, unsigned char** coding);
int ecw_isal_last_status(void);

enum { K = 11, M = 3, LEN = 4096 };
static unsigned char tbl[32 * K * M];
static int calls;

static void* worker(void* arg) {
  unsigned seed = (unsigned)(size_t)arg;
  unsigned char* buf = malloc((size_t)(K + M) * LEN);
  unsigned char* d[K];
  unsigned char* p[M];
  for (int j = 0; j < K; ++j) d[j] = buf + (size_t)j * LEN;
  for (int i = 0; i < M; ++i) p[i] = buf + (size_t)(K + i) * LEN;
  for (size_t i = 0; i < (size_t)K * LEN; ++i) buf[i] = (unsigned char)rand_r(&seed);
  for (int c = 0; c < calls; ++c) {
    ec_encode_data(LEN, K, M, tbl, d, p);
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
  printf("shim, %d threads x %d calls: %.0f stripes/s, %.2f GB/s of (k+m)*4 KiB, %.1f us per call per thread\n",
         threads, calls, n / s, n * (K + M) * LEN / s / 1e9, s / calls * 1e6);
  return 0;
}
