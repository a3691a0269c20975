// Prototype (tools/ only, not the product): the encode tile of the bench's
// split/tiled geometry with bit-sliced GF(2^8) products (bitslice_math.hpp)
// instead of LDS table lookups. One 256-lane workgroup per 8 KiB unit (the
// tiled slab's column piece); lane t owns bytes [16t, 16t+16) and
// [4096+16t, 4096+16t+16) of every row (two coalesced 1 KiB runs per wave).
// Local (CL XOR) parities of finished groups are parked in LDS and stored at
// the end of the unit with the global rows.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC tools/csrc/bitslice.hip -o build/bitslice.so
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bitslice_math.hpp"

namespace {

constexpr uint32_t kPiece = 8192;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 ldv(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  // volatile raw buffer load: stays where it is written (the ring's prefetch)
  return __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(off), 0, static_cast<int>(0x80000000u));
}

#ifndef BS_NTLOAD
#define BS_NTLOAD 1
#endif
// Nontemporal ring loads (the product's flavour: volatile buffer loads come
// out as sc0 sc1, which the product measured 9 % slower). A compiler-level
// memory barrier after the issue keeps LLVM from sinking the prefetch down to
// its use; it does not make the wave wait for the load.
__device__ __forceinline__ u32x4 ldn(const uint8_t* base, uint32_t off) {
  const u32x4 v = __builtin_nontemporal_load((const gu32x4*)(base + off));
  asm volatile("" ::: "memory");
  return v;
}

__device__ __forceinline__ void stv(uint8_t* p, u32x4 v) { __builtin_nontemporal_store(v, (gu32x4*)p); }

#ifndef BS_SPLITQ
#define BS_SPLITQ 1
#endif
#ifndef BS_ABLATE
#define BS_ABLATE 0  // 1: no GF math (loads, local XOR, stores only): the structure's ceiling
#endif

template <int M>
__device__ __forceinline__ void row(const u32x4& a, const u32x4& b, const uint32_t (&cw)[4], uint32_t (&lacc)[8],
                                    uint32_t (&acc)[M][8]) {
  uint32_t x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) lacc[i] ^= x[i];
#if BS_ABLATE
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[r][i] += x[i] ^ cw[r >> 2];
#else
  bs::transpose(x);
  uint32_t q[8][8];
#if BS_SPLITQ
  // low nibbles of every row first (2^0..2^3 x live), then 2^4..2^7 x from
  // 2^3 x: fewer planes live at once than with all eight powers
  bs::powers_range<0, 4>(x, q);
#pragma unroll
  for (int r = 0; r < M; ++r) bs::apply<0>((cw[r >> 2] >> (8 * (r & 3))) & 15u, acc[r], q);
  bs::powers_range<4, 8>(x, q);
#pragma unroll
  for (int r = 0; r < M; ++r) bs::apply<1>((cw[r >> 2] >> (8 * (r & 3) + 4)) & 15u, acc[r], q);
#else
  bs::powers(x, q);
#pragma unroll
  for (int r = 0; r < M; ++r) bs::mul_acc((cw[r >> 2] >> (8 * (r & 3))) & 255u, acc[r], q);
#endif
#endif
}

#ifndef BS_MINB
#define BS_MINB 1
#endif
#ifndef BS_TPB
#define BS_TPB 256  // lanes per workgroup: a tile is BS_TPB x 32 bytes of one 8 KiB unit
#endif
constexpr uint32_t kTpb = BS_TPB, kTile = kTpb * 32, kHalf = kTpb * 16;
#ifdef BS_WPE
#define BS_WPE_ATTR __attribute__((amdgpu_waves_per_eu(BS_WPE, BS_WPE)))
#else
#define BS_WPE_ATTR
#endif
template <int M>
__global__ __launch_bounds__(BS_TPB, BS_MINB) BS_WPE_ATTR void bs_encode_kernel(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                                        const uint32_t* __restrict__ coef_t, int k, int r, int g) {
  extern __shared__ u32x4 park[];  // [group][half][lane]
  constexpr uint32_t kTiles = kPiece / kTile;  // tiles per unit
  const uint32_t u = blockIdx.x / kTiles, t = threadIdx.x;
  const uint32_t o1 = (blockIdx.x % kTiles) * kTile + t * 16, o2 = o1 + kHalf;
  const uint8_t* base = data + static_cast<size_t>(u) * k * kPiece;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, 0x7FFFFFFF, 0x00020000);
  uint32_t acc[M][8], lacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    lacc[i] = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) acc[j][i] = 0;
  }
  // one row in flight ahead of the one being consumed; the loop runs to k - 1
  // with unconditional next-row loads and the last row is peeled, which keeps
  // the compiler's waits counted (vmcnt(2)); copying the ring registers or
  // loading conditionally made them vmcnt(0)
#if BS_NTLOAD
#define BS_LD(off) ldn(base, (off))
#else
#define BS_LD(off) ldv(rs, (off))
#endif
  u32x4 ca = BS_LD(o1), cb = BS_LD(o2);
  int gend = r < k ? r : k, grp = 0;
  for (int j = 0; j < k - 1; ++j) {
    const u32x4 na = BS_LD((j + 1) * kPiece + o1), nb = BS_LD((j + 1) * kPiece + o2);
    uint32_t cw[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) cw[w] = w * 4 < M ? __builtin_amdgcn_readfirstlane(coef_t[j * 4 + w]) : 0u;
    row<M>(ca, cb, cw, lacc, acc);
    if (g > 0 && j + 1 == gend) {
      park[(grp * 2 + 0) * kTpb + t] = u32x4{lacc[0], lacc[1], lacc[2], lacc[3]};
      park[(grp * 2 + 1) * kTpb + t] = u32x4{lacc[4], lacc[5], lacc[6], lacc[7]};
#pragma unroll
      for (int i = 0; i < 8; ++i) lacc[i] = 0;
      ++grp;
      gend = gend + r < k ? gend + r : k;
    }
    ca = na;
    cb = nb;
  }
  {
    uint32_t cw[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) cw[w] = w * 4 < M ? __builtin_amdgcn_readfirstlane(coef_t[(k - 1) * 4 + w]) : 0u;
    row<M>(ca, cb, cw, lacc, acc);
  }
  uint8_t* pb = parity + static_cast<size_t>(u) * (M + g) * kPiece;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    bs::transpose(acc[j]);
    stv(pb + j * kPiece + o1, u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]});
    stv(pb + j * kPiece + o2, u32x4{acc[j][4], acc[j][5], acc[j][6], acc[j][7]});
  }
  if (g > 0) {
    for (int s = 0; s < g - 1; ++s) {
      stv(pb + (M + s) * kPiece + o1, park[(s * 2 + 0) * kTpb + t]);
      stv(pb + (M + s) * kPiece + o2, park[(s * 2 + 1) * kTpb + t]);
    }
    stv(pb + (M + g - 1) * kPiece + o1, u32x4{lacc[0], lacc[1], lacc[2], lacc[3]});
    stv(pb + (M + g - 1) * kPiece + o2, u32x4{lacc[4], lacc[5], lacc[6], lacc[7]});
  }
}

}  // namespace

// data: units x k rows of 8 KiB; parity: units x (m + g) rows of 8 KiB;
// coef_t (device): 4 words per source, byte (r & 3) of word 4j + (r >> 2) = matrix[r][j]
extern "C" int bs_encode_split(const uint8_t* data, uint8_t* parity, const uint32_t* coef_t, int k, int m, int r,
                               int g, int units, void* stream) {
  if (k < 1 || m < 1 || m > 16 || g < 0 || units < 1 || (g > 0 && r < 1)) return -1;
  const size_t lds = g > 1 ? static_cast<size_t>(g - 1) * 2 * kTpb * sizeof(u32x4) : 0;
  if (lds > 64 * 1024) return -2;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define BS_CASE(M_)                                                                                  \
  case M_:                                                                                           \
    hipLaunchKernelGGL(bs_encode_kernel<M_>, dim3(units * (kPiece / kTile)), dim3(kTpb), lds, s, data, parity, \
                       coef_t, k, r, g);                                                             \
    break;
  switch (m) {
    BS_CASE(1) BS_CASE(2) BS_CASE(3) BS_CASE(4) BS_CASE(5) BS_CASE(8) BS_CASE(10) BS_CASE(12) BS_CASE(16)
    default: return -4;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
