// GF(2^8) arithmetic for the host side of the codec (matrix + table
// construction). Polynomial x^8+x^4+x^3+x^2+1 (0x11D), the field ISA-L uses
// (isal:erasure_code/ec_base.c:36-60; tables ec_base.h:35,64).
//
// Everything here is constexpr / pure: no mutable static state (the
// reference keeps static tables in NativeCodec.cc:178-180,206,287-288).
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

namespace ecw {

struct GfTables {
  std::array<uint8_t, 256> exp{};
  std::array<uint8_t, 256> log{};
};

constexpr GfTables make_gf_tables() {
  GfTables t{};
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = static_cast<uint8_t>(x);
    t.log[x] = static_cast<uint8_t>(i);
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  t.exp[255] = t.exp[0];
  return t;
}

inline constexpr GfTables kGf = make_gf_tables();

constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
  if (a == 0 || b == 0) return 0;
  int i = kGf.log[a] + kGf.log[b];
  return kGf.exp[i > 254 ? i - 255 : i];
}

constexpr uint8_t gf_inv(uint8_t a) { return a == 0 ? 0 : kGf.exp[255 - kGf.log[a]]; }

// Rows k..n-1 of ISA-L's gf_gen_cauchy1_matrix(n, k): C[l][j] = 1/((k+l) ^ j)
// (isal:erasure_code/ec_base.c:81-97), i.e. what generateEncodeMatrix copies
// out for a single-node codec (NativeCodec.cc:31-34,59-61).
inline std::vector<uint8_t> cauchy_parity_rows(int k, int m) {
  std::vector<uint8_t> a(static_cast<size_t>(k) * m);
  for (int l = 0; l < m; ++l)
    for (int j = 0; j < k; ++j) a[static_cast<size_t>(l) * k + j] = gf_inv(static_cast<uint8_t>((k + l) ^ j));
  return a;
}

// ISA-L's 32-byte per-coefficient layout (gf_vect_mul_init,
// isal:erasure_code/ec_base.c:157-262): [c*0..c*15 | c*0x00,c*0x10..c*0xF0].
inline void vect_mul_table(uint8_t c, uint8_t* tbl) {
  for (int n = 0; n < 16; ++n) {
    tbl[n] = gf_mul(c, static_cast<uint8_t>(n));
    tbl[16 + n] = gf_mul(c, static_cast<uint8_t>(n << 4));
  }
}

// ec_init_tables (isal:erasure_code/ec_highlevel_func.c:33-43)
inline std::vector<uint8_t> isal_tables(int k, int rows, const uint8_t* a) {
  std::vector<uint8_t> g(static_cast<size_t>(32) * k * rows);
  for (int i = 0; i < rows * k; ++i) vect_mul_table(a[i], g.data() + 32 * static_cast<size_t>(i));
  return g;
}

// Device table image for one pass of up to 16 global rows:
// per data row j a record of 32 entries, entry type u32 (rows <= 4, NW = 1),
// u64 (rows <= 8, NW = 2) or 16 bytes (rows <= 16, NW = 4). The lo entry of
// nibble n packs c_l * n of every row l of the pass in byte l, the hi entry
// c_l * (n << 4). Record stride is 128 * NW bytes. NW = 1 and 4: lo entries
// first (address j * 128 * NW + n * 4 * NW), hi entries after them (+ 64 * NW).
// NW = 2: hi and lo entries interleaved, hi at n * 16 and lo at n * 16 + 8, so
// a hi address is the data byte's high nibble as it stands (W & 0xF0) and
// costs no shift.
inline std::vector<uint8_t> packed_pass_tables(const uint8_t* matrix, int k, int row0, int rows) {
  const int nw = rows <= 4 ? 1 : rows <= 8 ? 2 : 4;  // packed entry: 4, 8 or 16 bytes
  const size_t es = 4 * static_cast<size_t>(nw);
  std::vector<uint8_t> img(static_cast<size_t>(k) * 32 * es, 0);
  for (int j = 0; j < k; ++j) {
    uint8_t* rec = img.data() + static_cast<size_t>(j) * 32 * es;
    for (int n = 0; n < 16; ++n) {
      const size_t lo = nw == 2 ? (2 * n + 1) * es : n * es, hi = nw == 2 ? 2 * n * es : (16 + n) * es;
      for (int l = 0; l < rows; ++l) {
        const uint8_t c = matrix[static_cast<size_t>(row0 + l) * k + j];
        rec[lo + l] = gf_mul(c, static_cast<uint8_t>(n));
        rec[hi + l] = gf_mul(c, static_cast<uint8_t>(n << 4));
      }
    }
  }
  return img;
}

}  // namespace ecw
