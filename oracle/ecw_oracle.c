/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's hot path, used exclusively by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker
 * (never as the product path: the ecwide_amd library neither links nor
 * loads this file).
 *
 * What is restated (paths relative to the reference root; `isal:` = file
 * inside ECWide-H/isa-l-2.14.0.tar.gz, under isa-l-2.14.0/):
 *   GF(2^8), poly 0x11D ............ isal:erasure_code/ec_base.c:36-60 (gf_mul, gf_inv)
 *   gf_gen_rs_matrix ............... isal:erasure_code/ec_base.c:62-79
 *   gf_gen_cauchy1_matrix .......... isal:erasure_code/ec_base.c:81-97
 *   gf_vect_mul_init (32-B table) .. isal:erasure_code/ec_base.c:157-262
 *   ec_init_tables ................. isal:erasure_code/ec_highlevel_func.c:33-43
 *   ec_encode_data_base ............ isal:erasure_code/ec_base.c:290-305
 *   ec_encode_data_avx2 dispatch ... isal:erasure_code/ec_highlevel_func.c:106-135
 *     + gf_Nvect_dot_prod_avx2 ..... isal:erasure_code/gf_3vect_dot_prod_avx2.asm:293-380
 *       (4-bit split vpshufb lookups; restated with intrinsics, same algorithm)
 *   ISA-L master's AVX-512 and AVX-512+GFNI kernels, which the reference's
 *   ECWide-C links (ECWide-C/makefile:12-14 -> /usr/lib/libisal.so, built from
 *   unpinned ISA-L master per ECWide-C/README.md:34-39). NOT in
 *   /root/reference: restated from ISA-L's published design (2.31+):
 *     ec_encode_data_avx512 ..... gf_{1..6}vect_dot_prod_avx512: the same
 *                                 4-bit split on 64-byte vectors, <= 6 rows a pass
 *     ec_init_tables_gfni ....... one 8x8 GF(2) matrix (8 bytes) per coefficient
 *     ec_encode_data_avx512_gfni  gf_Nvect_dot_prod_avx512_gfni: one
 *                                 vgf2p8affineqb per source byte and row
 *   Their arithmetic is pinned bit-exact against oracle/_ref (ISA-L 2.14's
 *   ec_encode_data_base) by tests/test_oracle.py; their pass schedule is not
 *   (no master source here) -- it only moves the CPU timing, not the bytes.
 *   NativeCodec field derivations .. ECWide-C/src/NativeCodec.java:20-109,145-195
 *   CodingScheme derivations ....... ECWide-C/src/CodingScheme.java:22-48
 *   generateEncodeMatrix ........... ECWide-C/src/native/NativeCodec.cc:12-64 (single-node branch)
 *   encodeData ..................... ECWide-C/src/native/NativeCodec.cc:137-219
 *   decodeData / partialDecodeData . ECWide-C/src/native/NativeCodec.cc:221-282
 *   xorIntemediate ................. ECWide-C/src/native/NativeCodec.cc:284-323
 *
 * Pinning: tests/golden/ holds vectors produced by oracle/_ref (ISA-L 2.14.0
 * ec_base.c compiled from the reference tarball, see oracle/Makefile) and
 * tests/test_oracle.py checks this file against them.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* ---------------- GF(2^8) ---------------- */
static uint8_t g_exp[256], g_log[256];

__attribute__((constructor)) static void orc_gf_build(void) {
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    g_exp[i] = (uint8_t)x;
    g_log[x] = (uint8_t)i;
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  g_exp[255] = g_exp[0];
  g_log[0] = 0; /* unused: gf_mul tests for zero first */
}

uint8_t orc_gf_mul(uint8_t a, uint8_t b) {
  if (a == 0 || b == 0) return 0;
  int i = g_log[a] + g_log[b];
  return g_exp[i > 254 ? i - 255 : i];
}

uint8_t orc_gf_inv(uint8_t a) {
  if (a == 0) return 0;
  return g_exp[255 - g_log[a]];
}

void orc_gen_rs_matrix(uint8_t* a, int m, int k) {
  uint8_t gen = 1;
  memset(a, 0, (size_t)k * m);
  for (int i = 0; i < k; ++i) a[k * i + i] = 1;
  for (int i = k; i < m; ++i) {
    uint8_t p = 1;
    for (int j = 0; j < k; ++j) {
      a[k * i + j] = p;
      p = orc_gf_mul(p, gen);
    }
    gen = orc_gf_mul(gen, 2);
  }
}

void orc_gen_cauchy1_matrix(uint8_t* a, int m, int k) {
  memset(a, 0, (size_t)k * m);
  for (int i = 0; i < k; ++i) a[k * i + i] = 1;
  uint8_t* p = a + (size_t)k * k;
  for (int i = k; i < m; ++i)
    for (int j = 0; j < k; ++j) *p++ = orc_gf_inv((uint8_t)(i ^ j));
}

/* tbl[0..15] = c*n, tbl[16..31] = c*(n<<4) */
void orc_vect_mul_init(uint8_t c, uint8_t* tbl) {
  for (int n = 0; n < 16; ++n) {
    tbl[n] = orc_gf_mul(c, (uint8_t)n);
    tbl[16 + n] = orc_gf_mul(c, (uint8_t)(n << 4));
  }
}

void orc_init_tables(int k, int rows, const uint8_t* a, uint8_t* g_tbls) {
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < k; ++j) {
      orc_vect_mul_init(*a++, g_tbls);
      g_tbls += 32;
    }
}

/* coefficient = v[..+1] (table entry c*1), as ec_encode_data_base reads it */
void orc_encode_data_base(int len, int srcs, int dests, const uint8_t* v, uint8_t** src,
                          uint8_t** dest) {
  for (int l = 0; l < dests; ++l)
    for (int i = 0; i < len; ++i) {
      uint8_t s = 0;
      for (int j = 0; j < srcs; ++j) s ^= orc_gf_mul(src[j][i], v[j * 32 + l * srcs * 32 + 1]);
      dest[l][i] = s;
    }
}

/* ---- AVX2 4-bit split port (the reference's actual CPU kernel family) ---- */
#if defined(__x86_64__)
/* rows is a compile-time constant at every call (dot_prod_avx2_rows below), so
 * the accumulators live in registers as in the asm kernels */
__attribute__((target("avx2"), always_inline)) static inline void dot_prod_avx2_n(int len, int srcs,
                                                                                 const int rows,
                                                                                 const uint8_t* v,
                                                                                 uint8_t** src,
                                                                                 uint8_t** dest) {
  /* rows <= 6 outputs per pass, as gf_{1..6}vect_dot_prod_avx2 */
  const __m256i mask = _mm256_set1_epi8(0x0f);
  int pos = 0;
  for (;;) {
    if (pos > len - 32) {
      if (pos == len) break;
      pos = len - 32; /* overlapping last vector, as the asm does */
    }
    __m256i acc[6];
    for (int l = 0; l < rows; ++l) acc[l] = _mm256_setzero_si256();
    for (int j = 0; j < srcs; ++j) {
      __m256i x = _mm256_loadu_si256((const __m256i*)(src[j] + pos));
      __m256i lo = _mm256_and_si256(x, mask);
      __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
      for (int l = 0; l < rows; ++l) {
        const uint8_t* t = v + (size_t)l * srcs * 32 + (size_t)j * 32;
        __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)t));
        __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)(t + 16)));
        acc[l] = _mm256_xor_si256(acc[l], _mm256_xor_si256(_mm256_shuffle_epi8(tl, lo),
                                                           _mm256_shuffle_epi8(th, hi)));
      }
    }
    for (int l = 0; l < rows; ++l) _mm256_storeu_si256((__m256i*)(dest[l] + pos), acc[l]);
    if (pos == len - 32) break;
    pos += 32;
  }
}

#define ORC_ROWS_SWITCH(fn, rows, ...)         \
  switch (rows) {                              \
    case 1: fn(__VA_ARGS__, 1, v, src, dest); break; \
    case 2: fn(__VA_ARGS__, 2, v, src, dest); break; \
    case 3: fn(__VA_ARGS__, 3, v, src, dest); break; \
    case 4: fn(__VA_ARGS__, 4, v, src, dest); break; \
    case 5: fn(__VA_ARGS__, 5, v, src, dest); break; \
    default: fn(__VA_ARGS__, 6, v, src, dest); break; \
  }

__attribute__((target("avx2"))) static void dot_prod_avx2_rows(int len, int srcs, int rows, const uint8_t* v,
                                                                uint8_t** src, uint8_t** dest) {
  ORC_ROWS_SWITCH(dot_prod_avx2_n, rows, len, srcs)
}

static int have_avx2(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2");
}
#endif

int orc_have_avx2(void) {
#if defined(__x86_64__)
  return have_avx2();
#else
  return 0;
#endif
}

/* ec_encode_data_avx2 dispatch: len < 32 -> base; rows in passes of <= 4
 * (gf_4vect first, then 3/2/1 for the remainder) */
void orc_encode_data_avx2(int len, int srcs, int dests, const uint8_t* v, uint8_t** src,
                          uint8_t** dest) {
#if defined(__x86_64__)
  if (len < 32 || !have_avx2()) {
    orc_encode_data_base(len, srcs, dests, v, src, dest);
    return;
  }
  while (dests >= 4) {
    dot_prod_avx2_rows(len, srcs, 4, v, src, dest);
    v += 4 * srcs * 32;
    dest += 4;
    dests -= 4;
  }
  if (dests > 0) dot_prod_avx2_rows(len, srcs, dests, v, src, dest);
#else
  orc_encode_data_base(len, srcs, dests, v, src, dest);
#endif
}

/* ---- ISA-L master kernel families (CPU baseline "as ECWide-C builds it") ----
 * kind: 0 = ec_encode_data_base, 1 = AVX2 (ISA-L 2.14's top), 2 = AVX-512BW
 * (4-bit split vpshufb, 64-byte vectors), 3 = AVX-512 + GFNI (vgf2p8affineqb).
 * Table format: 32 bytes per coefficient for kinds 0-2 (ec_init_tables), 8
 * bytes for kind 3 (ec_init_tables_gfni). */
enum { ORC_BASE = 0, ORC_AVX2 = 1, ORC_AVX512 = 2, ORC_GFNI = 3 };

/* the 8x8 GF(2) matrix of x -> c*x (poly 0x11D) in vgf2p8affineqb's layout:
 * result bit i = parity(x & byte[7 - i]) */
uint64_t orc_gfni_matrix(uint8_t c) {
  uint64_t m = 0;
  for (int i = 0; i < 8; ++i) {
    uint8_t row = 0;
    for (int j = 0; j < 8; ++j)
      if (orc_gf_mul(c, (uint8_t)(1u << j)) & (1u << i)) row |= (uint8_t)(1u << j);
    m |= (uint64_t)row << (8 * (7 - i));
  }
  return m;
}

void orc_init_tables_gfni(int k, int rows, const uint8_t* a, uint8_t* g_tbls) {
  for (int i = 0; i < rows * k; ++i) {
    uint64_t m = orc_gfni_matrix(a[i]);
    memcpy(g_tbls + 8 * (size_t)i, &m, 8);
  }
}

/* scalar model of vgf2p8affineqb (imm8 = 0) on one byte: the checker of the
 * matrix layout on a CPU without GFNI */
uint8_t orc_gfni_affine_byte(uint64_t m, uint8_t x) {
  uint8_t y = 0;
  for (int i = 0; i < 8; ++i) {
    uint8_t row = (uint8_t)(m >> (8 * (7 - i)));
    y |= (uint8_t)((__builtin_popcount(row & x) & 1) << i);
  }
  return y;
}

#if defined(__x86_64__)
__attribute__((target("avx512f,avx512bw"), always_inline)) static inline void dot_prod_avx512_n(
    int len, int srcs, const int rows, const uint8_t* v, uint8_t** src, uint8_t** dest) {
  const __m512i mask = _mm512_set1_epi8(0x0f);
  int pos = 0;
  for (;;) {
    if (pos > len - 64) {
      if (pos == len) break;
      pos = len - 64; /* overlapping last vector */
    }
    __m512i acc[6];
    for (int l = 0; l < rows; ++l) acc[l] = _mm512_setzero_si512();
    for (int j = 0; j < srcs; ++j) {
      __m512i x = _mm512_loadu_si512((const void*)(src[j] + pos));
      __m512i lo = _mm512_and_si512(x, mask);
      __m512i hi = _mm512_and_si512(_mm512_srli_epi64(x, 4), mask);
      for (int l = 0; l < rows; ++l) {
        const uint8_t* t = v + (size_t)l * srcs * 32 + (size_t)j * 32;
        __m512i tl = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)t));
        __m512i th = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)(t + 16)));
        acc[l] = _mm512_xor_si512(acc[l], _mm512_xor_si512(_mm512_shuffle_epi8(tl, lo),
                                                           _mm512_shuffle_epi8(th, hi)));
      }
    }
    for (int l = 0; l < rows; ++l) _mm512_storeu_si512((void*)(dest[l] + pos), acc[l]);
    if (pos == len - 64) break;
    pos += 64;
  }
}

__attribute__((target("avx512f,avx512bw,gfni"), always_inline)) static inline void dot_prod_gfni_n(
    int len, int srcs, const int rows, const uint8_t* v, uint8_t** src, uint8_t** dest) {
  int pos = 0;
  for (;;) {
    if (pos > len - 64) {
      if (pos == len) break;
      pos = len - 64;
    }
    __m512i acc[6];
    for (int l = 0; l < rows; ++l) acc[l] = _mm512_setzero_si512();
    for (int j = 0; j < srcs; ++j) {
      __m512i x = _mm512_loadu_si512((const void*)(src[j] + pos));
      for (int l = 0; l < rows; ++l) {
        uint64_t m;
        memcpy(&m, v + 8 * ((size_t)l * srcs + j), 8);
        acc[l] = _mm512_xor_si512(acc[l], _mm512_gf2p8affine_epi64_epi8(x, _mm512_set1_epi64((long long)m), 0));
      }
    }
    for (int l = 0; l < rows; ++l) _mm512_storeu_si512((void*)(dest[l] + pos), acc[l]);
    if (pos == len - 64) break;
    pos += 64;
  }
}

__attribute__((target("avx512f,avx512bw"))) static void dot_prod_avx512_rows(int len, int srcs, int rows,
                                                                             const uint8_t* v, uint8_t** src,
                                                                             uint8_t** dest) {
  ORC_ROWS_SWITCH(dot_prod_avx512_n, rows, len, srcs)
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void dot_prod_gfni_rows(int len, int srcs, int rows,
                                                                                const uint8_t* v, uint8_t** src,
                                                                                uint8_t** dest) {
  ORC_ROWS_SWITCH(dot_prod_gfni_n, rows, len, srcs)
}
#endif

int orc_have_kind(int kind) {
#if defined(__x86_64__)
  __builtin_cpu_init();
  switch (kind) {
    case ORC_BASE: return 1;
    case ORC_AVX2: return __builtin_cpu_supports("avx2");
    case ORC_AVX512: return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
    case ORC_GFNI:
      return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
             __builtin_cpu_supports("gfni");
  }
  return 0;
#else
  return kind == ORC_BASE;
#endif
}

/* the kernel family ISA-L master's ec_encode_data dispatch picks on this CPU
 * (ECWide-C as built): AVX-512 + GFNI, else AVX-512, else AVX2, else base */
int orc_isal_master_kind(void) {
  for (int kind = ORC_GFNI; kind > ORC_BASE; --kind)
    if (orc_have_kind(kind)) return kind;
  return ORC_BASE;
}

static void encode_data_base_gfni(int len, int srcs, int dests, const uint8_t* v, uint8_t** src, uint8_t** dest) {
  for (int l = 0; l < dests; ++l)
    for (int i = 0; i < len; ++i) {
      uint8_t s = 0;
      for (int j = 0; j < srcs; ++j) {
        uint64_t m;
        memcpy(&m, v + 8 * ((size_t)l * srcs + j), 8);
        s ^= orc_gfni_affine_byte(m, src[j][i]);
      }
      dest[l][i] = s;
    }
}

/* ec_encode_data of one kernel family; tables in that family's format */
void orc_encode_data_kind(int kind, int len, int srcs, int dests, const uint8_t* v, uint8_t** src,
                          uint8_t** dest) {
  if (!orc_have_kind(kind)) kind = kind == ORC_GFNI ? -1 : ORC_BASE; /* -1: scalar model of the gfni tables */
#if defined(__x86_64__)
  if (kind == ORC_AVX2) {
    orc_encode_data_avx2(len, srcs, dests, v, src, dest);
    return;
  }
  if ((kind == ORC_AVX512 || kind == ORC_GFNI) && len >= 64) {
    const int tb = kind == ORC_GFNI ? 8 : 32;
    while (dests > 0) {
      const int rows = dests < 6 ? dests : 6;
      if (kind == ORC_GFNI)
        dot_prod_gfni_rows(len, srcs, rows, v, src, dest);
      else
        dot_prod_avx512_rows(len, srcs, rows, v, src, dest);
      v += (size_t)rows * srcs * tb;
      dest += rows;
      dests -= rows;
    }
    return;
  }
#endif
  if (kind == ORC_GFNI || kind == -1)
    encode_data_base_gfni(len, srcs, dests, v, src, dest);
  else
    orc_encode_data_base(len, srcs, dests, v, src, dest);
}

void orc_init_tables_kind(int kind, int k, int rows, const uint8_t* a, uint8_t* g_tbls) {
  if (kind == ORC_GFNI)
    orc_init_tables_gfni(k, rows, a, g_tbls);
  else
    orc_init_tables(k, rows, a, g_tbls);
}

/* ---------------- NativeCodec restatement ---------------- */
typedef struct orc_codec {
  /* CodingScheme */
  char code_type;
  int k, m, group_data_num, group_num, rack_nodes_num, rack_num;
  int chunk_size;
  /* NativeCodec */
  int node_index, multinode;
  int encode_data_num, decode_data_num, partial_decode_num, rack_per_group;
  uint8_t* encode_matrix;   /* encode_data_num * m */
  uint8_t* encode_gftbl;    /* 32 * edn * m */
  uint8_t* decode_gftbl;    /* 32 * ddn */
  uint8_t* partial_gftbl;   /* 32 * pdn */
  int xori_called;          /* the reference's static `flag` (NativeCodec.cc:288) */
} orc_codec;

static int ceil_div(int a, int b) { return (a + b - 1) / b; }

/* CodingScheme ctors (CodingScheme.java:22-48) */
static void scheme_init(orc_codec* c, char t, int k, int m, int r, int chunk) {
  c->code_type = t;
  c->k = k;
  c->m = m;
  c->chunk_size = chunk;
  c->group_data_num = -1;
  c->group_num = 0;
  c->rack_nodes_num = 0;
  c->rack_num = 0;
  if (t == 'T') {
    c->rack_num = ceil_div(k, m) + 1;
    c->rack_nodes_num = m;
  } else if (t == 'L' || t == 'C') {
    c->group_data_num = r;
    c->group_num = ceil_div(k, r);
    if (t == 'C') {
      c->rack_nodes_num = m + 1;
      c->rack_num = ceil_div(k + c->group_num, m + 1) + 1;
    } else {
      c->rack_nodes_num = c->rack_num = -1;
    }
  }
}

/* NativeCodec.getClPartialDecodeNum (NativeCodec.java:175-183) */
static int cl_partial_decode_num(const orc_codec* c, int node) {
  int rack = (node - 1) / c->rack_nodes_num;
  if (rack != c->rack_num - 2) return c->rack_nodes_num;
  int last = (c->k - 1) % c->group_data_num + 1;
  return last % c->rack_nodes_num + 1;
}

/* NativeCodec.getTlPartialDecodeNum (NativeCodec.java:185-195) */
static int tl_partial_decode_num(int k, int m, int node) {
  int rn = m, rack = (node - 1) / rn, racks = ceil_div(k, m) + 1;
  if (rack == racks - 2) {
    int last = k - rack * rn;
    return (last - 1) % rn + 1;
  }
  return rn;
}

void orc_codec_free(orc_codec* c) {
  if (!c) return;
  free(c->encode_matrix);
  free(c->encode_gftbl);
  free(c->decode_gftbl);
  free(c->partial_gftbl);
  free(c);
}

/* NativeCodec ctors (NativeCodec.java:20-109) + the four init natives. */
orc_codec* orc_codec_new(char t, int k, int m, int r, int chunk, int node, int multinode) {
  orc_codec* c = (orc_codec*)calloc(1, sizeof(orc_codec));
  if (!c) return NULL;
  scheme_init(c, t, k, m, r, chunk);
  c->node_index = node;
  c->multinode = multinode;
  if (t == 'R') {
    c->decode_data_num = c->encode_data_num = k;
  } else if (t == 'T') {
    int racks = ceil_div(k, m) + 1;
    c->encode_data_num = k;
    c->partial_decode_num = tl_partial_decode_num(k, m, node);
    c->decode_data_num = c->partial_decode_num - 1 + racks - 1;
  } else if (t == 'L') {
    c->encode_data_num = k;
    int gi = (node - 1) / r;
    c->decode_data_num = (gi == r - 1) ? (k - 1) % r + 1 : r; /* sic, NativeCodec.java:63 */
  } else { /* 'C' */
    if (multinode)
      c->encode_data_num = (node == 1) ? (k - 1) % r + 1 : r;
    else
      c->encode_data_num = k;
    c->partial_decode_num = cl_partial_decode_num(c, node);
    c->rack_per_group = ceil_div(r + 1, c->rack_nodes_num);
    c->decode_data_num = c->partial_decode_num - 1 + c->rack_per_group - 1;
  }
  int edn = c->encode_data_num, ddn = c->decode_data_num, pdn = c->partial_decode_num;
  c->encode_matrix = (uint8_t*)calloc((size_t)edn * m + 1, 1);
  c->encode_gftbl = (uint8_t*)calloc((size_t)edn * m * 32 + 1, 1);
  c->decode_gftbl = (uint8_t*)calloc((size_t)ddn * 32 + 1, 1);
  c->partial_gftbl = (uint8_t*)calloc((size_t)pdn * 32 + 1, 1);
  /* generateEncodeMatrix, single-node branch (NativeCodec.cc:31-34,59-61) */
  int n = edn + m;
  uint8_t* tmp = (uint8_t*)calloc((size_t)edn * n, 1);
  orc_gen_cauchy1_matrix(tmp, n, edn);
  memcpy(c->encode_matrix, tmp + (size_t)edn * edn, (size_t)edn * m);
  free(tmp);
  orc_init_tables(edn, m, c->encode_matrix, c->encode_gftbl);
  uint8_t ones[256];
  memset(ones, 1, sizeof ones);
  orc_init_tables(ddn, 1, ones, c->decode_gftbl);
  if (t == 'T' || t == 'C') orc_init_tables(pdn, 1, ones, c->partial_gftbl);
  return c;
}

int orc_codec_field(const orc_codec* c, int which) {
  switch (which) {
    case 0: return c->encode_data_num;
    case 1: return c->decode_data_num;
    case 2: return c->partial_decode_num;
    case 3: return c->group_num;
    case 4: return c->rack_nodes_num;
    case 5: return c->rack_num;
    case 6: return c->rack_per_group;
    case 7: return c->group_data_num;
    default: return -1;
  }
}
const uint8_t* orc_codec_matrix(const orc_codec* c) { return c->encode_matrix; }
const uint8_t* orc_codec_gftbl(const orc_codec* c) { return c->encode_gftbl; }

/* encodeData (NativeCodec.cc:137-219), single-node, through the ec_encode_data
 * of kernel family `kind`. `literal` reproduces the zero local-parity tables
 * (NativeCodec.cc:181-186); otherwise the local tables are built from an
 * all-ones row (the CL code as designed). */
static void nc_encode(const orc_codec* c, uint8_t** data, uint8_t** parity, int literal, int kind, int off,
                      int len) {
  int k = c->encode_data_num, m = c->m;
  uint8_t* d[256];
  uint8_t* p[320];
  for (int j = 0; j < k; ++j) d[j] = data[j] + off;
  int np = m + ((c->code_type == 'C' || c->code_type == 'L') ? c->group_num : 0);
  for (int i = 0; i < np; ++i) p[i] = parity[i] + off;
  if (kind == ORC_GFNI) {
    uint8_t* g = (uint8_t*)malloc((size_t)8 * k * m + 8);
    orc_init_tables_gfni(k, m, c->encode_matrix, g);
    orc_encode_data_kind(kind, len, k, m, g, d, p);
    free(g);
  } else {
    orc_encode_data_kind(kind, len, k, m, c->encode_gftbl, d, p);
  }
  if (c->code_type != 'C' && c->code_type != 'L') return;
  int r = c->group_data_num;
  uint8_t row[256], *xor_tbl = (uint8_t*)malloc(32 * 256);
  memset(row, literal ? 0 : 1, sizeof row);
  orc_init_tables_kind(kind, r, 1, row, xor_tbl);
  int pos = m, offset = 0;
  for (int t = 0; t < c->group_num - 1; ++t, ++pos, offset += r)
    orc_encode_data_kind(kind, len, r, 1, xor_tbl, d + offset, p + pos);
  int last = (k - 1) % r + 1;
  orc_init_tables_kind(kind, last, 1, row, xor_tbl);
  orc_encode_data_kind(kind, len, last, 1, xor_tbl, d + offset, p + pos);
  free(xor_tbl);
}

void orc_nc_encode(const orc_codec* c, uint8_t** data, uint8_t** parity, int literal, int avx2) {
  nc_encode(c, data, parity, literal, avx2 ? ORC_AVX2 : ORC_BASE, 0, c->chunk_size);
}

void orc_nc_encode_len(const orc_codec* c, uint8_t** data, uint8_t** parity, int literal,
                       int avx2, int len) {
  nc_encode(c, data, parity, literal, avx2 ? ORC_AVX2 : ORC_BASE, 0, len);
}

/* the same with an explicit kernel family (0 base, 1 AVX2, 2 AVX-512, 3 GFNI) */
void orc_nc_encode_kind(const orc_codec* c, uint8_t** data, uint8_t** parity, int literal, int kind, int len) {
  nc_encode(c, data, parity, literal, kind, 0, len);
}

/* decodeData / partialDecodeData: ec_encode_data with the all-ones table */
void orc_nc_decode(const orc_codec* c, uint8_t** data, uint8_t* target, int len) {
  uint8_t* t[1] = {target};
  orc_encode_data_base(len, c->decode_data_num, 1, c->decode_gftbl, data, t);
}
void orc_nc_partial_decode(const orc_codec* c, uint8_t** data, uint8_t* target, int len) {
  uint8_t* t[1] = {target};
  orc_encode_data_base(len, c->partial_decode_num, 1, c->partial_gftbl, data, t);
}

/* xorIntemediate (NativeCodec.cc:284-323): first call -> zero tables */
void orc_nc_xor_intermediate(orc_codec* c, uint8_t** src, uint8_t** tgt, int len, int literal) {
  uint8_t tbl[64];
  memset(tbl, 0, sizeof tbl);
  if (!literal || c->xori_called) {
    uint8_t a[2] = {1, 1};
    orc_init_tables(2, 1, a, tbl);
  }
  for (int i = 0; i < c->m; ++i) {
    uint8_t* d[2] = {src[i], tgt[i]};
    uint8_t* o[1] = {tgt[i]};
    orc_encode_data_base(len, 2, 1, tbl, d, o);
  }
  c->xori_called = 1;
}

/* ---- multi-threaded CPU baseline: the same flow split by byte range ---- */
typedef struct {
  const orc_codec* c;
  uint8_t** data;
  uint8_t** parity;
  int literal, off, len, kind;
} mt_job;

static void* mt_run(void* arg) {
  mt_job* j = (mt_job*)arg;
  nc_encode(j->c, j->data, j->parity, j->literal, j->kind, j->off, j->len);
  return NULL;
}

void orc_nc_encode_mt_kind(const orc_codec* c, uint8_t** data, uint8_t** parity, int literal, int nthreads,
                           int len, int kind) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  mt_job jobs[256];
  int per = (len / nthreads) & ~63;
  if (nthreads == 1 || per < 64) {
    nc_encode(c, data, parity, literal, kind, 0, len);
    return;
  }
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].c = c;
    jobs[t].data = data;
    jobs[t].parity = parity;
    jobs[t].literal = literal;
    jobs[t].kind = kind;
    jobs[t].off = t * per;
    jobs[t].len = (t == nthreads - 1) ? len - t * per : per;
    pthread_create(&th[t], NULL, mt_run, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

void orc_nc_encode_mt(const orc_codec* c, uint8_t** data, uint8_t** parity, int literal, int nthreads, int len) {
  orc_nc_encode_mt_kind(c, data, parity, literal, nthreads, len, ORC_AVX2);
}

/* ec_encode_data (one kernel family) split by byte range over nthreads
 * threads: the multi-threaded form of decodeData / a CL repair
 * (NativeCodec.cc:237-248: ec_encode_data with the all-ones table) for the
 * CPU baseline; tables in that family's format. */
typedef struct {
  int len, k, rows, kind;
  const uint8_t* tbl;
  uint8_t* src[256];
  uint8_t* dst[256];
} ed_job;

static void* ed_run(void* arg) {
  ed_job* j = (ed_job*)arg;
  orc_encode_data_kind(j->kind, j->len, j->k, j->rows, j->tbl, j->src, j->dst);
  return NULL;
}

void orc_encode_data_mt_kind(int kind, int len, int k, int rows, const uint8_t* tbl, uint8_t** src,
                             uint8_t** dst, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  int per = (len / nthreads) & ~63;
  if (nthreads == 1 || per < 64 || k > 256 || rows > 256) {
    orc_encode_data_kind(kind, len, k, rows, tbl, src, dst);
    return;
  }
  pthread_t th[256];
  ed_job* jobs = (ed_job*)malloc(sizeof(ed_job) * nthreads);
  for (int t = 0; t < nthreads; ++t) {
    const int off = t * per;
    jobs[t].len = (t == nthreads - 1) ? len - off : per;
    jobs[t].k = k;
    jobs[t].rows = rows;
    jobs[t].kind = kind;
    jobs[t].tbl = tbl;
    for (int i = 0; i < k; ++i) jobs[t].src[i] = src[i] + off;
    for (int i = 0; i < rows; ++i) jobs[t].dst[i] = dst[i] + off;
    pthread_create(&th[t], NULL, ed_run, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(jobs);
}

void orc_encode_data_avx2_mt(int len, int k, int rows, const uint8_t* tbl, uint8_t** src, uint8_t** dst,
                             int nthreads) {
  orc_encode_data_mt_kind(ORC_AVX2, len, k, rows, tbl, src, dst, nthreads);
}

/* ---------------- synthetic data (ecwide.h, ecw_fill_random_dev) ---------------- */
static uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

/* bytes [off, off + len) of the stream of (seed, stripe, block); off % 8 == 0 */
void orc_fill_random_at(uint8_t* dst, size_t off, size_t len, uint64_t seed, uint32_t stripe, uint32_t block) {
  const uint64_t G = 0x9E3779B97F4A7C15ull;
  uint64_t key = mix64(seed + G * (1ull + (uint64_t)stripe * 65536ull + block));
  const uint64_t w0 = off / 8;
  size_t nw = len / 8;
  for (size_t w = 0; w < nw; ++w) {
    uint64_t v = mix64(key + (w0 + w) * G);
    memcpy(dst + 8 * w, &v, 8);
  }
  if (len % 8) {
    uint64_t v = mix64(key + (w0 + nw) * G);
    memcpy(dst + 8 * nw, &v, len % 8);
  }
}

void orc_fill_random(uint8_t* dst, size_t len, uint64_t seed, uint32_t stripe, uint32_t block) {
  orc_fill_random_at(dst, 0, len, seed, stripe, block);
}

/* XOR of n blocks (flat CL repair) */
void orc_xor_blocks(uint8_t** src, int n, uint8_t* dst, size_t len) {
  memset(dst, 0, len);
  for (int i = 0; i < n; ++i)
    for (size_t b = 0; b < len; ++b) dst[b] ^= src[i][b];
}
