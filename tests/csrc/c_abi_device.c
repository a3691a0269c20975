/* A plain C caller of the C ABI (include/ecwide.h) with no Python and no torch:
 * what a C/C++ host of ECWide-C's codec (or a JNI/cgo shim) links against.
 * HBM comes from the HIP runtime's C API; the engine fills a slab of CL
 * stripes, encodes them and repairs D0 of every stripe (ecw_fill_random_dev,
 * ecw_encode_batch_dev, ecw_repair_batch_dev: NativeCodec.cc:137-219 batched,
 * ClMetadataManager.java:137-257 flattened), and the host entry point
 * ecw_encode (encodeData) runs once on host buffers. Every byte is checked
 * against the oracle (oracle/liboracle.so: test infrastructure, the checker).
 *
 *   gcc -O2 -std=c11 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include tests/csrc/c_abi_device.c \
 *       -L ecwide_amd -lecwide -L oracle -loracle -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,... -o build/c_abi_device
 *   build/c_abi_device [k m r block_bytes stripes]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ecwide.h"

/* the checker's entry points (oracle/ecw_oracle.c) */
typedef struct orc_codec orc_codec;
orc_codec* orc_codec_new(char t, int k, int m, int r, int chunk, int node, int multinode);
void orc_codec_free(orc_codec* c);
void orc_nc_encode_len(const orc_codec* c, uint8_t** data, uint8_t** parity, int literal, int avx2, int len);
void orc_fill_random_at(uint8_t* dst, size_t off, size_t len, uint64_t seed, uint32_t stripe, uint32_t block);

#define ECW(x)                                                                     \
  do {                                                                             \
    int st_ = (x);                                                                 \
    if (st_ != ECW_OK) {                                                           \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, ecw_status_string(st_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)
#define HIP(x)                                                                     \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

static int same(const uint8_t* a, const uint8_t* b, size_t n, const char* what, int s, int i) {
  if (memcmp(a, b, n) == 0) return 1;
  size_t x = 0;
  while (a[x] == b[x]) ++x;
  fprintf(stderr, "mismatch: %s stripe %d block %d at byte %zu\n", what, s, i, x);
  return 0;
}

int main(int argc, char** argv) {
  const int k = argc > 1 ? atoi(argv[1]) : 32, m = argc > 2 ? atoi(argv[2]) : 2, r = argc > 3 ? atoi(argv[3]) : 8;
  const size_t B = argc > 4 ? strtoull(argv[4], NULL, 10) : (size_t)(1 << 20) + 4096 + 17; /* ragged on purpose */
  const int S = argc > 5 ? atoi(argv[5]) : 3;
  const uint64_t seed = 11;
  if (k < 2 || m < 1 || r < 1 || B < 1 || S < 1 || B > (1u << 30)) return 2;

  ecw_scheme sch;
  ecw_codec* c = NULL;
  ECW(ecw_scheme_init(&sch, 'C', k, m, r, B));
  ECW(ecw_codec_create(&sch, 1, 0, ECW_LOCAL_XOR, 0, &c));
  ecw_codec_info info;
  ECW(ecw_codec_get_info(c, &info));
  const int np = info.parity_num; /* m global + ceil(k / r) local */
  const size_t bstride = (B + 4096 + 255) & ~(size_t)255, sstride = (size_t)(k + np) * bstride;

  hipStream_t stream;
  uint8_t *d_slab = NULL, *d_out = NULL;
  HIP(hipStreamCreate(&stream));
  HIP(hipMalloc((void**)&d_slab, (size_t)S * sstride));
  HIP(hipMalloc((void**)&d_out, (size_t)S * bstride)); /* repaired blocks at a 16-byte-aligned stride */
  ECW(ecw_fill_random_dev(0, d_slab, bstride, sstride, S, k, B, seed, 0, 0, stream));
  ECW(ecw_encode_batch_dev(c, d_slab, bstride, sstride, S, B, stream));
  ECW(ecw_repair_batch_dev(c, d_slab, bstride, sstride, S, 0, d_out, bstride, B, stream));
  HIP(hipStreamSynchronize(stream));

  uint8_t* h_slab = malloc((size_t)S * sstride);
  uint8_t* h_out = malloc((size_t)S * bstride);
  uint8_t** data = malloc(sizeof(uint8_t*) * k);
  uint8_t** want = malloc(sizeof(uint8_t*) * np);
  uint8_t** got = malloc(sizeof(uint8_t*) * np);
  if (!h_slab || !h_out || !data || !want || !got) return 3;
  for (int j = 0; j < k; ++j) data[j] = malloc(B);
  for (int i = 0; i < np; ++i) {
    want[i] = malloc(B);
    got[i] = malloc(B);
  }
  HIP(hipMemcpy(h_slab, d_slab, (size_t)S * sstride, hipMemcpyDeviceToHost));
  HIP(hipMemcpy(h_out, d_out, (size_t)S * bstride, hipMemcpyDeviceToHost));

  orc_codec* oc = orc_codec_new('C', k, m, r, (int)B, 1, 0);
  if (!oc) return 3;
  int ok = 1;
  for (int s = 0; s < S && ok; ++s) {
    for (int j = 0; j < k; ++j) {
      orc_fill_random_at(data[j], 0, B, seed, (uint32_t)s, (uint32_t)j);
      ok &= same(h_slab + s * sstride + j * bstride, data[j], B, "fill", s, j);
    }
    orc_nc_encode_len(oc, data, want, 0, 0, (int)B);
    for (int i = 0; i < np && ok; ++i)
      ok &= same(h_slab + s * sstride + (size_t)(k + i) * bstride, want[i], B, "encode_batch_dev", s, k + i);
    ok &= same(h_out + s * bstride, data[0], B, "repair_batch_dev D0", s, 0);
  }
  /* the host-memory entry point on the last stripe's blocks */
  if (ok) {
    ECW(ecw_encode(c, (const uint8_t* const*)data, got, B));
    for (int i = 0; i < np && ok; ++i) ok &= same(got[i], want[i], B, "ecw_encode", S - 1, k + i);
  }
  orc_codec_free(oc);
  HIP(hipFree(d_slab));
  HIP(hipFree(d_out));
  HIP(hipStreamDestroy(stream));
  ecw_codec_destroy(c);
  if (!ok) return 1;
  printf("ok: CL(k=%d, r=%d, m=%d), %d stripes of %zu-byte blocks: fill, encode_batch_dev, repair_batch_dev, "
         "ecw_encode bit-exact vs the oracle\n", k, r, m, S, B);
  return 0;
}
