// CPU self-test of tools/csrc/bitslice_math.hpp: transpose is an involution and
// bit-sliced c*x equals the table GF(2^8) product for every c and random x.
//   g++ -O2 -std=c++17 -DBS_HD=inline tools/csrc/bitslice_selftest.cpp -o /tmp/bs && /tmp/bs
#include <cstdio>
#include <cstring>
#include <random>

#include "bitslice_math.hpp"

static uint8_t gmul(uint8_t a, uint8_t b) {  // 0x11D, shift-and-add
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = static_cast<uint8_t>((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
    b >>= 1;
  }
  return r;
}

int main() {
  std::mt19937 rng(7);
  int bad = 0;
  for (int t = 0; t < 200; ++t) {
    uint32_t d[8], x[8];
    for (auto& w : d) w = rng();
    memcpy(x, d, sizeof x);
    bs::transpose(x);
    uint32_t y[8];
    memcpy(y, x, sizeof y);
    bs::transpose(y);
    if (memcmp(y, d, sizeof d)) ++bad;
    // plane i, byte p, bit q == bit i of byte p of d[q]
    for (int i = 0; i < 8; ++i)
      for (int p = 0; p < 4; ++p)
        for (int q = 0; q < 8; ++q)
          if (((x[i] >> (8 * p + q)) & 1) != ((d[q] >> (8 * p + i)) & 1)) ++bad;
    uint32_t qq[8][8];
    bs::powers(x, qq);
    for (int c = 0; c < 256; ++c) {
      uint32_t acc[8] = {0};
      bs::mul_acc(static_cast<uint32_t>(c), acc, qq);
      bs::transpose(acc);
      for (int q = 0; q < 8; ++q)
        for (int p = 0; p < 4; ++p) {
          const uint8_t in = static_cast<uint8_t>(d[q] >> (8 * p));
          const uint8_t out = static_cast<uint8_t>(acc[q] >> (8 * p));
          if (out != gmul(static_cast<uint8_t>(c), in)) ++bad;
        }
    }
  }
  printf(bad ? "FAIL %d\n" : "ok\n", bad);
  return bad != 0;
}
