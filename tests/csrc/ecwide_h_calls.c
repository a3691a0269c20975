/* Replays ECWide-H's ISA-L call sequence (ECWide-H/proxy/encode.cpp:113-238,
 * geometry common.hpp:21-32: GROUP 2, RACK 3, NODE 4, CHUNK_SIZE 4096)
 * against whichever library provides the ISA-L symbols; here libecw_isal.so
 * (the MI355X engine). Inputs: the ecwide.h counter PRNG (seeds 41..44 as in
 * tests/golden/gen_golden.py); output: the four results, raw, on stdout.
 * Prototypes as in isal:include/erasure_code.h (no ISA-L header needed). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void gf_gen_rs_matrix(unsigned char* a, int m, int k);
void gf_gen_cauchy1_matrix(unsigned char* a, int m, int k);
void ec_init_tables(int k, int rows, unsigned char* a, unsigned char* g_tbls);
void ec_encode_data(int len, int k, int rows, unsigned char* g_tbls, unsigned char** data, unsigned char** coding);

#define CHUNK_SIZE 4096
#define GROUP 2
#define RACK 3
#define NODE 4
#define LK (RACK * NODE - 1)
#define LN (LK + 1)
#define GK ((GROUP - 1) * (RACK * NODE - 1))
#define GN (GK + NODE - 1)

static uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 27; z *= 0x94D049BB133111EBull; z ^= z >> 31;
  return z;
}
static unsigned char* block(uint64_t seed, uint32_t j) {
  const uint64_t G = 0x9E3779B97F4A7C15ull;
  unsigned char* p = malloc(CHUNK_SIZE);
  uint64_t key = mix64(seed + G * (1ull + j));
  for (int w = 0; w < CHUNK_SIZE / 8; ++w) { uint64_t v = mix64(key + (uint64_t)w * G); memcpy(p + 8 * w, &v, 8); }
  return p;
}
/* encode.cpp's pattern: RS (or Cauchy) matrix n x k, tables of rows k..n-1, ec_encode_data */
static void run(int rs, int k, int n, uint64_t seed) {
  unsigned char mat[GN * GK > LN * LK ? GN * GK : LN * LK], tbl[32 * GK * (GN - GK) + 32 * LK];
  unsigned char* src[GN];
  for (int j = 0; j < k; ++j) src[j] = block(seed, j);
  for (int j = k; j < n; ++j) src[j] = calloc(CHUNK_SIZE, 1);
  if (rs) gf_gen_rs_matrix(mat, n, k); else gf_gen_cauchy1_matrix(mat, n, k);
  ec_init_tables(k, n - k, &mat[k * k], tbl);
  ec_encode_data(CHUNK_SIZE, k, n - k, tbl, src, &src[k]);
  for (int j = k; j < n; ++j) fwrite(src[j], 1, CHUNK_SIZE, stdout);
  for (int j = 0; j < n; ++j) free(src[j]);
}
int main(void) {
  run(1, LK, LN, 41);                 /* l_encode */
  run(0, GK, GN, 42);                 /* g_encode */
  run(1, NODE, NODE + 1, 43);         /* l_middle(count = NODE) */
  run(1, RACK - 1 + NODE - 1, RACK - 1 + NODE, 44); /* l_decode(need = RACK-1+NODE-1) */
  return 0;
}
