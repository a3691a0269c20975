// Bit-sliced GF(2^8) products (prototype, tools/ only): the lane's 32 data
// bytes (8 dwords D0..D7) are transposed into 8 bit planes (plane i, byte p,
// bit q = bit i of byte p of D_q), multiplication by 2 is 3 XORs of planes
// (x^8 = x^4 + x^3 + x^2 + 1, ISA-L's 0x11D, isal:erasure_code/ec_base.c:159),
// and c*x = XOR over the set bits b of c of (2^b x). The coefficient is
// uniform over the wave, so the XOR network for each nibble of c is selected
// with a scalar branch instead of a table lookup: no LDS at all.
#pragma once
#include <cstdint>

#ifndef BS_HD
#define BS_HD __host__ __device__ __forceinline__
#endif

namespace bs {

// delta swap of an 8x8 bit block (per byte lane): a = row q, b = row q + d
template <int D>
BS_HD void dswap(uint32_t& a, uint32_t& b) {
  constexpr uint32_t m = D == 1 ? 0x55555555u : D == 2 ? 0x33333333u : 0x0F0F0F0Fu;
  const uint32_t na = (a & ~(m << D)) | ((b << D) & (m << D));
  const uint32_t nb = (b & ~m) | ((a >> D) & m);
  a = na;
  b = nb;
}

// 8x8 bit transpose of every byte position across the 8 registers (an involution)
BS_HD void transpose(uint32_t (&x)[8]) {
  dswap<1>(x[0], x[1]); dswap<1>(x[2], x[3]); dswap<1>(x[4], x[5]); dswap<1>(x[6], x[7]);
  dswap<2>(x[0], x[2]); dswap<2>(x[1], x[3]); dswap<2>(x[4], x[6]); dswap<2>(x[5], x[7]);
  dswap<4>(x[0], x[4]); dswap<4>(x[1], x[5]); dswap<4>(x[2], x[6]); dswap<4>(x[3], x[7]);
}

// q[b] = 2^b * p (bit planes)
BS_HD void powers(const uint32_t (&p)[8], uint32_t (&q)[8][8]) {
#pragma unroll
  for (int o = 0; o < 8; ++o) q[0][o] = p[o];
#pragma unroll
  for (int b = 0; b < 7; ++b) {
    const uint32_t* s = q[b];
    q[b + 1][0] = s[7];
    q[b + 1][1] = s[0];
    q[b + 1][2] = s[1] ^ s[7];
    q[b + 1][3] = s[2] ^ s[7];
    q[b + 1][4] = s[3] ^ s[7];
    q[b + 1][5] = s[4];
    q[b + 1][6] = s[5];
    q[b + 1][7] = s[6];
  }
}

// q[b] = 2^b * p for B0 <= b < B1 (q[B0 - 1] already computed when B0 > 0)
template <int B0, int B1>
BS_HD void powers_range(const uint32_t (&p)[8], uint32_t (&q)[8][8]) {
  if (B0 == 0) {
#pragma unroll
    for (int o = 0; o < 8; ++o) q[0][o] = p[o];
  }
#pragma unroll
  for (int b = (B0 == 0 ? 0 : B0 - 1); b < B1 - 1; ++b) {
    const uint32_t* s = q[b];
    q[b + 1][0] = s[7];
    q[b + 1][1] = s[0];
    q[b + 1][2] = s[1] ^ s[7];
    q[b + 1][3] = s[2] ^ s[7];
    q[b + 1][4] = s[3] ^ s[7];
    q[b + 1][5] = s[4];
    q[b + 1][6] = s[5];
    q[b + 1][7] = s[6];
  }
}

// 3-input XOR: v_bitop3_b32 (LUT 0x96) on the device
BS_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// acc ^= v * 16^H * p for the nibble value v (compile-time V inside the switch)
template <int H, int V>
BS_HD void nib(uint32_t (&acc)[8], const uint32_t (&q)[8][8]) {
  constexpr int n = (V & 1) + ((V >> 1) & 1) + ((V >> 2) & 1) + ((V >> 3) & 1);
  constexpr int b0 = (V & 1) ? 0 : (V & 2) ? 1 : (V & 4) ? 2 : 3;
  constexpr int b1 = (V >> (b0 + 1)) & 1 ? b0 + 1 : (V >> (b0 + 2)) & 1 ? b0 + 2 : b0 + 3;
  constexpr int b2 = (V >> (b1 + 1)) & 1 ? b1 + 1 : b1 + 2;
  constexpr int b3 = 3;
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    if (n == 1) acc[o] ^= q[4 * H + b0][o];
    if (n >= 2) acc[o] = xor3(acc[o], q[4 * H + b0][o], q[4 * H + b1][o]);
    if (n == 3) acc[o] ^= q[4 * H + b2][o];
    if (n == 4) acc[o] = xor3(acc[o], q[4 * H + 2][o], q[4 * H + b3][o]);
  }
}

template <int H>
BS_HD void apply(uint32_t v, uint32_t (&acc)[8], const uint32_t (&q)[8][8]) {
  switch (v) {
    case 1: nib<H, 1>(acc, q); break;
    case 2: nib<H, 2>(acc, q); break;
    case 3: nib<H, 3>(acc, q); break;
    case 4: nib<H, 4>(acc, q); break;
    case 5: nib<H, 5>(acc, q); break;
    case 6: nib<H, 6>(acc, q); break;
    case 7: nib<H, 7>(acc, q); break;
    case 8: nib<H, 8>(acc, q); break;
    case 9: nib<H, 9>(acc, q); break;
    case 10: nib<H, 10>(acc, q); break;
    case 11: nib<H, 11>(acc, q); break;
    case 12: nib<H, 12>(acc, q); break;
    case 13: nib<H, 13>(acc, q); break;
    case 14: nib<H, 14>(acc, q); break;
    case 15: nib<H, 15>(acc, q); break;
    default: break;
  }
}

// bit pair P of c (bits 2P, 2P+1): 4-way switch
template <int P>
BS_HD void apply_pair(uint32_t v, uint32_t (&acc)[8], const uint32_t (&q)[8][8]) {
  switch (v) {
    case 1:
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[o] ^= q[2 * P][o];
      break;
    case 2:
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[o] ^= q[2 * P + 1][o];
      break;
    case 3:
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[o] = xor3(acc[o], q[2 * P][o], q[2 * P + 1][o]);
      break;
    default: break;
  }
}

#ifndef BS_DISPATCH
#define BS_DISPATCH 0  // 0: 16-way switch per nibble, 1: one branch per bit, 2: 4-way switch per bit pair
#endif

// acc ^= c * p
BS_HD void mul_acc(uint32_t c, uint32_t (&acc)[8], const uint32_t (&q)[8][8]) {
#if BS_DISPATCH == 1
#pragma unroll
  for (int b = 0; b < 8; ++b)
    if ((c >> b) & 1u) {
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[o] ^= q[b][o];
    }
#elif BS_DISPATCH == 2
  apply_pair<0>(c & 3u, acc, q);
  apply_pair<1>((c >> 2) & 3u, acc, q);
  apply_pair<2>((c >> 4) & 3u, acc, q);
  apply_pair<3>((c >> 6) & 3u, acc, q);
#else
  apply<0>(c & 15u, acc, q);
  apply<1>((c >> 4) & 15u, acc, q);
#endif
}

}  // namespace bs
