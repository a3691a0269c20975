// Device-side building blocks shared by the kernel translation units
// (ecw_kernels.hip: encode + fill, ecw_xor.hpp: XOR reduce, ecw_service.hip:
// the resident request service) and the launch helpers their host sides
// share. Everything here is internal (anonymous namespace: one copy per TU).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "ecw_internal.hpp"
#include "ecw_tuning.hpp"

namespace ecw {
namespace {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(3))) const unsigned long long lds_u64;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const u32x4_t lds_u128;

// Columns are 32-bit offsets from a wave-uniform row pointer, so loads and
// stores use the SGPR-base + VGPR-offset form (blocks are < 4 GiB; the host
// checks it).
//
// NT: plain nontemporal load (the XOR reduce: a straight stream, measured
// +4 % over the volatile buffer load the encode ring needs). Full tiles
// otherwise take a raw buffer load with the compiler-level volatile bit (aux
// bit 31): without it LLVM sinks the ring's prefetch loads down to their uses
// in the next iteration (re-rolling the software pipeline into "issue P
// loads, drain"); volatile loads stay where they are written, and their
// results are still tracked by the compiler's vmcnt bookkeeping (counted
// vmcnt(P-1..0), not vmcnt(0)). Codegen adds sc0 sc1 (L1 bypass, served from
// L2): fine for a stream every byte of which is read once.
template <bool TAIL, bool NT = false>
__device__ __forceinline__ uint4 ld16(const uint8_t* row, uint32_t col, uint32_t len) {
  if (NT && (!TAIL || col + 16 <= len)) {
    // global address space: a pointer loaded from a table would otherwise be
    // generic and get flat loads (which also count against lgkmcnt)
    typedef const __attribute__((address_space(1))) u32x4_t gu32x4;
    const u32x4_t v = __builtin_nontemporal_load((gu32x4*)(row + col));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  if (!TAIL) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(row), 0, 0x7FFFFFFF, 0x00020000);
    const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(col), 0, static_cast<int>(0x80000000u));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  if (col + 16 <= len) return *reinterpret_cast<const uint4*>(row + col);
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (col + i < len) w[i >> 2] |= static_cast<uint32_t>(row[col + i]) << (8 * (i & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <bool TAIL, bool NT = false>
__device__ __forceinline__ void st16(uint8_t* row, uint32_t col, uint32_t len, uint4 v) {
  if (!TAIL || col + 16 <= len) {
    if (NT) {
      typedef __attribute__((address_space(1))) u32x4_t gu32x4;
      const u32x4_t w = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(w, (gu32x4*)(row + col));
    } else {
      *reinterpret_cast<uint4*>(row + col) = v;
    }
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (col + i < len) row[col + i] = static_cast<uint8_t>(w[i >> 2] >> (8 * (i & 3)));
}

// First tile of this workgroup's grid-stride walk. Blocks are dealt round-robin
// over the 8 XCDs; with `remap` each XCD walks its own contiguous 1/8 of every
// grid-sized window (a permutation of [0, gridDim.x) when 8 divides it), so
// the workgroups resident on one CU take tiles 32 apart instead of 256 and
// share more address translations (EncodeGeom::remap, XorSched::remap).
__device__ __forceinline__ uint64_t wg_slot(uint32_t remap = 0) {
  const uint32_t G = gridDim.x, b = blockIdx.x;
  if (remap && (G & 7u) == 0) return static_cast<uint64_t>(b & 7u) * (G >> 3) + (b >> 3);
  return blockIdx.x;
}

__device__ __forceinline__ const uint8_t* uniform_ptr(const uint8_t* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
}

// Tile indices are 32-bit (FastDiv): one launch covers at most this many
// tiles; larger batches go in several launches over consecutive stripes.
constexpr uint64_t kMaxTilesPerLaunch = 1ull << 31;

// ECW_DEBUG_LAUNCH=1 (debugging aid, read once): every launch is printed with
// its grid and synchronised, so a faulting kernel names itself.
inline bool debug_launch() {
  static const bool on = [] {
    const char* e = std::getenv("ECW_DEBUG_LAUNCH");
    return e && e[0] == '1';
  }();
  return on;
}
inline hipError_t launched(const char* what, dim3 grid, size_t lds, hipStream_t s) {
  hipError_t e = hipGetLastError();
  if (debug_launch()) {
    std::fprintf(stderr, "ecw launch %s grid %u lds %zu: %s", what, grid.x, lds, hipGetErrorString(e));
    const hipError_t f = hipStreamSynchronize(s);
    std::fprintf(stderr, " -> %s\n", hipGetErrorString(f));
    if (e == hipSuccess) e = f;
  }
  return e;
}

inline unsigned grid_for(uint64_t tiles_total, uint64_t per_cu = kGridPerCu) {
  // memory-bound streaming: enough workgroups to fill 256 CUs many deep,
  // grid-stride beyond that (encode tables are staged once per workgroup)
  const uint64_t cap = 256ull * per_cu;
  return static_cast<unsigned>(tiles_total < cap ? (tiles_total ? tiles_total : 1) : cap);
}

}  // namespace
}  // namespace ecw
