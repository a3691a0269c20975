// HIP kernels for gfx950 (MI355X, CDNA4): wide-stripe GF(2^8) encode,
// XOR reduce (CL repair / decode / relayer stage) and the synthetic fill.
//
// Encode replaces ECWide-C encodeData (NativeCodec.cc:137-219), which makes
// two full passes over the k data blocks (ec_encode_data for the m global
// rows, then one pass per local group). Here ONE pass over HBM computes all
// global rows of a pass (<= 8) and every local XOR parity:
//
//   * one lane owns 16 consecutive byte columns (one dwordx4 per data row),
//     a 256-lane workgroup a 4 KiB column tile, rows streamed with a P-deep
//     register prefetch ring (coalesced 1 KiB per wave-instruction);
//   * GF(2^8) products use ISA-L's 4-bit split (c*x = c*lo ^ c*(hi<<4),
//     gf_vect_mul_init, isal:erasure_code/ec_base.c:157-262), but with the
//     tables of ALL rows of the pass packed into one LDS entry: entry n holds
//     byte l = c_l*n for every row l, so one ds_read per nibble serves up to
//     4 (u32) or 8 (u64) outputs. A table record of 16 entries spans 16
//     distinct banks: lookups are conflict-free whatever the data;
//   * LDS addresses are formed with v_perm_b32 from a pre-masked nibble word
//     (one v_and_or for four lookups, one v_perm per lookup); products are
//     folded with v_bitop3_b32 (xor3);
//   * local parities are a plain XOR of the dwordx4 rows, flushed at group
//     boundaries (all-zero in ECWide-C literal mode, still written).
//
// No MFMA: the work is byte-wise GF(2^8), not a dense FP contraction.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "ecw_internal.hpp"
#include "ecw_encode_asm.hpp"

namespace ecw {
namespace {

#ifndef ECW_ASM_PARK
#define ECW_ASM_PARK 1  // <= 5 local parities: store them at the end of the tile
#endif
constexpr int kPrefetchEncAsmTail = 2;
constexpr int kMaxParkedLocals = ECW_ASM_PARK ? 5 : 0;  // v[58:77] of the asm tile

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
#ifndef ECW_NT_STORES
#define ECW_NT_STORES 0
#endif
#ifndef ECW_NT_LOADS
#define ECW_NT_LOADS 0
#endif
#ifndef ECW_XOR_NT
#define ECW_XOR_NT 1  // XOR reduce: nontemporal loads and stores
#endif
#ifndef ECW_ABLATE
#define ECW_ABLATE 0  // tuning builds only: 1 = skip the GF lookups, 2 = skip the data loads
#endif

#ifndef ECW_BUFLOAD
#define ECW_BUFLOAD 1
#endif

// NT: plain nontemporal load (the XOR reduce: a straight stream, measured
// +4 % over the volatile buffer load the encode ring needs).
template <bool TAIL, bool NT = false>
__device__ __forceinline__ uint4 ld16(const uint8_t* row, uint32_t col, uint32_t len) {
  if (NT && (!TAIL || col + 16 <= len)) {
    // global address space: a pointer loaded from a table would otherwise be
    // generic and get flat loads (which also count against lgkmcnt)
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) u32x4 gu32x4;
    const u32x4 v = __builtin_nontemporal_load((gu32x4*)(row + col));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
#if ECW_BUFLOAD
  // Full tiles: a raw buffer load with the compiler-level volatile bit (aux
  // bit 31). Without it LLVM sinks the ring's prefetch loads down to their
  // uses in the next iteration (re-rolling the software pipeline into
  // "issue P loads, drain"); volatile loads stay where they are written, and
  // their results are still tracked by the compiler's vmcnt bookkeeping
  // (counted vmcnt(P-1..0), not vmcnt(0)). Codegen adds sc0 sc1 (L1 bypass,
  // served from L2): fine for a stream every byte of which is read once.
  if (!TAIL) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(row), 0, 0x7FFFFFFF, 0x00020000);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(col), 0, static_cast<int>(0x80000000u));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
#endif
#if ECW_ABLATE == 2
  if (!TAIL) return make_uint4(col ^ static_cast<uint32_t>(reinterpret_cast<uintptr_t>(row)), col * 3u, col + 7u, col >> 3);
#endif
#if ECW_NT_LOADS
  if (!TAIL || col + 16 <= len) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + col));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
#else
  if (!TAIL || col + 16 <= len) return *reinterpret_cast<const uint4*>(row + col);
#endif
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (col + i < len) w[i >> 2] |= static_cast<uint32_t>(row[col + i]) << (8 * (i & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <bool TAIL, bool NT = false>
__device__ __forceinline__ void st16(uint8_t* row, uint32_t col, uint32_t len, uint4 v) {
  if (!TAIL || col + 16 <= len) {
    if (NT || ECW_NT_STORES) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(1))) u32x4 gu32x4;
      const u32x4 w = {v.x, v.y, v.z, v.w};
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

// ---- row addressing (all wave-uniform) -------------------------------------
__device__ __forceinline__ const uint8_t* src_row(const PtrRows& r, const EncodeGeom&, int, int j) {
  return r.src[j];
}
__device__ __forceinline__ const uint8_t* src_row(const SlabRows& r, const EncodeGeom&, int s, int j) {
  return r.base + s * r.sstride + static_cast<uint64_t>(j) * r.bstride;
}
__device__ __forceinline__ const uint8_t* src_row(const PtrTabRows& r, const EncodeGeom& g, int s, int j) {
  return r.src[static_cast<uint64_t>(s) * g.k + j];
}
__device__ __forceinline__ uint8_t* glob_row(const PtrTabRows& r, const EncodeGeom& g, int s, int l) {
  return r.dst[static_cast<uint64_t>(s) * r.np + g.row0 + l];
}
__device__ __forceinline__ uint8_t* local_row(const PtrTabRows& r, const EncodeGeom& g, int s, int t) {
  return r.dst[static_cast<uint64_t>(s) * r.np + g.m + t];
}
__device__ __forceinline__ uint8_t* glob_row(const PtrRows& r, const EncodeGeom&, int, int l) {
  return r.dst[l];
}
__device__ __forceinline__ uint8_t* glob_row(const SlabRows& r, const EncodeGeom& g, int s, int l) {
  return r.pbase + s * r.psstride + static_cast<uint64_t>(g.row0 + l) * r.pbstride;
}
__device__ __forceinline__ uint8_t* local_row(const PtrRows& r, const EncodeGeom& g, int, int t) {
  return r.dst[g.nrows + t];
}
__device__ __forceinline__ uint8_t* local_row(const SlabRows& r, const EncodeGeom& g, int s, int t) {
  return r.pbase + s * r.psstride + static_cast<uint64_t>(g.m + t) * r.pbstride;
}

// ---- GF(2^8) multiply-accumulate of one 16-byte row slice -----------------
// acc[p] (NW=1) packs the running products of byte column p for up to 4
// rows; NW=2: acc[2p], acc[2p+1] pack 8 rows; NW=4: acc[4p..4p+3] pack 16
// rows (one 16-byte LDS entry per nibble, ds_read_b128). `rec` is the LDS
// byte address of row j's table record (a multiple of 128*NW): its bits 8..
// enter the address through v_perm (jhi), its low byte through the nibble
// mask (jlo).
template <int NW>
__device__ __forceinline__ void gf_row(const uint4 x, uint32_t (&acc)[16 * NW], uint32_t rec) {
  const uint32_t jhi = rec >> 8;
  const uint32_t jlo = (rec & 0xFFu) * 0x01010101u;
  const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t w = w4[d];
    // (nibble * entry size) in every byte, record low byte OR-ed in
    // (NW = 2: lo entries at +8 of the interleaved pairs, ecw_gf.hpp)
    const uint32_t lo = NW == 1 ? (((w << 2) & 0x3C3C3C3Cu) | jlo) : (((w << 4) & 0xF0F0F0F0u) | jlo);
    const uint32_t hi = NW == 1 ? (((w >> 2) & 0x3C3C3C3Cu) | jlo) : ((w & 0xF0F0F0F0u) | jlo);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      // address = jhi << 8 | byte b of lo/hi  (selector: S1.byte b, S0.byte0,
      // and S0.byte1 for the 16-row tables, which reach past 64 KiB at k > 128)
      const uint32_t sel = (NW == 4 ? 0x0C050400u : 0x0C0C0400u) | static_cast<uint32_t>(b);
      const uint32_t al = __builtin_amdgcn_perm(jhi, lo, sel);
      const uint32_t ah = __builtin_amdgcn_perm(jhi, hi, sel);
      const int p = 4 * d + b;
      if constexpr (NW == 1) {
        const uint32_t tl = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(al));
        const uint32_t th = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(ah + 64));
        acc[p] = xor3(acc[p], tl, th);
      } else if constexpr (NW == 2) {
        const unsigned long long tl = *reinterpret_cast<lds_u64*>(static_cast<uintptr_t>(al + 8));
        const unsigned long long th = *reinterpret_cast<lds_u64*>(static_cast<uintptr_t>(ah));
        acc[2 * p] = xor3(acc[2 * p], static_cast<uint32_t>(tl), static_cast<uint32_t>(th));
        acc[2 * p + 1] = xor3(acc[2 * p + 1], static_cast<uint32_t>(tl >> 32), static_cast<uint32_t>(th >> 32));
      } else {
        const u32x4_t tl = *reinterpret_cast<lds_u128*>(static_cast<uintptr_t>(al));
        const u32x4_t th = *reinterpret_cast<lds_u128*>(static_cast<uintptr_t>(ah + 256));
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[4 * p + e] = xor3(acc[4 * p + e], tl[e], th[e]);
      }
    }
  }
}

// byte l of the packed accumulators of columns 0..15 -> output row l
template <int NW>
__device__ __forceinline__ uint4 unpack_row(const uint32_t (&acc)[16 * NW], int l) {
  const int wsel = NW == 1 ? 0 : (l >> 2);
  const uint32_t bl = static_cast<uint32_t>(l & 3);
  const uint32_t s01 = 0x0C0C0000u | ((4 + bl) << 8) | bl;
  const uint32_t s23 = ((4 + bl) << 24) | (bl << 16) | 0x0C0Cu;
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t a0 = acc[NW * (4 * q + 0) + wsel], a1 = acc[NW * (4 * q + 1) + wsel];
    const uint32_t a2 = acc[NW * (4 * q + 2) + wsel], a3 = acc[NW * (4 * q + 3) + wsel];
    o[q] = __builtin_amdgcn_perm(a1, a0, s01) | __builtin_amdgcn_perm(a3, a2, s23);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
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
// ECW_XCD_REMAP = 0 | 1 (tuning; read per launch) overrides the launcher's
// choice of the per-XCD tile order above
inline uint32_t xcd_remap_env(uint32_t dflt) {
  const char* e = std::getenv("ECW_XCD_REMAP");
  if (!e || !e[0]) return dflt;
  return e[0] == '1' ? 1u : 0u;
}

// Column tile `tile` of the slab: stripe, this lane's column, whole tile in range?
struct TileAt {
  int s;
  uint32_t col;
  bool full;
};

__device__ __forceinline__ TileAt tile_at(const EncodeGeom& g, uint32_t tile) {
  const uint32_t s = fast_div(tile, g.per);
  const uint32_t col0 = (tile - s * g.per.d) * kTileBytes;
  return {static_cast<int>(s), col0 + threadIdx.x * kLaneBytes, static_cast<uint64_t>(col0) + kTileBytes <= g.len};
}

// rows 0..P-1 of tile t into the ring (clamped to k-1 when k < P)
template <int P, bool TAIL, class Rows>
__device__ __forceinline__ void ring_prologue(uint4 (&ring)[P], const Rows& rows, const EncodeGeom& g,
                                              const TileAt& t) {
#pragma unroll
  for (int p = 0; p < P; ++p)
    ring[p] = ld16<TAIL>(src_row(rows, g, t.s, p < g.k ? p : g.k - 1), t.col, static_cast<uint32_t>(g.len));
}

// One column tile: consumes the ring (rows 0..P-1 of `cur` already in flight)
// and streams rows P..k-1 through it. In the last round of the row loop the
// slots are refilled with rows 0..P-1 of the next tile when `pf`, so tiles
// follow each other without a load bubble and without redundant loads.
template <int NW, int P, int LOCAL, bool TAIL, class Rows>
__device__ __forceinline__ void encode_tile(const Rows& rows, const EncodeGeom& g, const TileAt& cur,
                                            uint4 (&ring)[P], bool pf, const TileAt& nxt, uint32_t lds_base) {
  const uint32_t len = static_cast<uint32_t>(g.len);
  const uint32_t col = cur.col;
  if (TAIL && col >= len) return;
  const int k = g.k;
  uint32_t acc[16 * NW];
#pragma unroll
  for (int i = 0; i < 16 * NW; ++i) acc[i] = 0;
  uint4 lacc = make_uint4(0, 0, 0, 0);
  int gend = g.r < k ? g.r : k;
  int t = 0;
  for (int j0 = 0; j0 < k; j0 += P) {
    const bool last_round = j0 + P >= k;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      // consume slot p, then refill it: the refill reuses the slot's
      // registers (no copy, so no early vmcnt wait)
      const int j = j0 + p;
      if (j < k) {
#if ECW_ABLATE == 1
        acc[0] ^= ring[p].x;
        acc[1] ^= ring[p].y;
#else
        gf_row<NW>(ring[p], acc, lds_base + static_cast<uint32_t>(j) * (128u * NW));
#endif
        if constexpr (LOCAL != kLocalNone) {
          lacc = xor4(lacc, ring[p]);
          if (j + 1 == gend) {
            // (this store makes LLVM put vmcnt(0) at the loop head; the slab
            // path avoids that with the asm tile, ecw_encode_asm.hpp)
            st16<TAIL>(local_row(rows, g, cur.s, t), col, len, LOCAL == kLocalXor ? lacc : make_uint4(0, 0, 0, 0));
            lacc = make_uint4(0, 0, 0, 0);
            ++t;
            gend = gend + g.r < k ? gend + g.r : k;
          }
        }
      }
      // exactly one load per visit (a conditional load would make the
      // compiler's vmcnt bookkeeping fall back to vmcnt(0)): the address
      // selects row j+P of this tile, row p of the next one, or a clamped
      // re-read of row k-1 when there is nothing left to prefetch
      const bool use_next = !TAIL && last_round && pf;
      const int row = use_next ? p : (j + P < k ? j + P : k - 1);
      ring[p] = ld16<TAIL>(src_row(rows, g, use_next ? nxt.s : cur.s, row), use_next ? nxt.col : col, len);
    }
  }
  if constexpr (NW == 4) {
    // unrolled over the 16 rows (constant accumulator indices: a runtime index
    // into 64 accumulators puts them in scratch)
#pragma unroll
    for (int l = 0; l < 4 * NW; ++l)
      if (l < g.nrows) st16<TAIL>(glob_row(rows, g, cur.s, l), col, len, unpack_row<NW>(acc, l));
  } else {
    for (int l = 0; l < g.nrows; ++l) st16<TAIL>(glob_row(rows, g, cur.s, l), col, len, unpack_row<NW>(acc, l));
  }
}

template <int NW, int P, int LOCAL, class Rows>
#ifndef ECW_ENC_MIN_WAVES
#define ECW_ENC_MIN_WAVES 6  // __launch_bounds__ min waves per SIMD: caps VGPRs at 80 (+1-4 %; spills only outside the row loop)
#endif
#ifndef ECW_ENC_MIN_WAVES_NW2
#define ECW_ENC_MIN_WAVES_NW2 4  // 5-8 rows: 128 VGPRs (at 80 the 32 accumulators spill inside the row loop)
#endif
#ifndef ECW_ENC_MIN_WAVES_NW4
#define ECW_ENC_MIN_WAVES_NW4 2  // 9-16 rows: 256 VGPRs for the 64 packed accumulators
#endif
__global__ __launch_bounds__(kBlock, NW == 1 ? ECW_ENC_MIN_WAVES : NW == 2 ? ECW_ENC_MIN_WAVES_NW2 : ECW_ENC_MIN_WAVES_NW4) void encode_kernel(const Rows rows, const EncodeGeom g,
                                                        const uint4* __restrict__ tbl) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  // workgroup b takes tiles begin + b, + grid, + 2 grid, ... (concurrently
  // resident workgroups then cover adjacent columns of the same rows; giving
  // each workgroup a contiguous run of tiles measured 6-10 % slower)
  uint32_t tile = g.tile_begin + blockIdx.x;
  const uint32_t tend = g.tile_end;
  const uint32_t tstep = gridDim.x;
  uint4 ring[P];
  // the first tile's row loads are issued before the table staging so the
  // two overlap
  bool have = false;
  if (tile < tend) {
    const TileAt t0 = tile_at(g, tile);
    if (t0.full) {
      ring_prologue<P, false>(ring, rows, g, t0);
      have = true;
    }
  }
  const int n16 = g.k * 8 * NW;
  for (int i = threadIdx.x; i < n16; i += kBlock) reinterpret_cast<uint4*>(lds)[i] = tbl[i];
  __syncthreads();
  // dynamic LDS starts at 0 (no static LDS in this kernel); records are
  // 128*NW-byte aligned relative to it
  const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds));
  const bool cross = g.k >= P;
  for (; tile < tend; tile += tstep) {
    const TileAt cur = tile_at(g, tile);
    if (!cur.full) {
      ring_prologue<P, true>(ring, rows, g, cur);
      encode_tile<NW, P, LOCAL, true>(rows, g, cur, ring, false, cur, lds_base);
      have = false;
      continue;
    }
    if (!have) ring_prologue<P, false>(ring, rows, g, cur);
    const uint32_t nt = tile + tstep;
    const TileAt nxt = tile_at(g, nt < tend ? nt : tile);
    const bool pf = cross && nt < tend && nxt.full;
    encode_tile<NW, P, LOCAL, false>(rows, g, cur, ring, pf, nxt, lds_base);
    have = pf;
  }
}

#ifndef ECW_ENC_ASM
#define ECW_ENC_ASM 1  // <= 4 global rows: hand-scheduled tile loop (ecw_encode_asm.hpp)
#endif
#ifndef ECW_ASM_MIN_WAVES
#define ECW_ASM_MIN_WAVES 6  // 80 VGPRs: the parked asm tile uses 77 (6 measured >= 8 also without parking)
#endif

__device__ __forceinline__ const uint8_t* uniform_ptr(const uint8_t* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
}

// Encode with <= 4 global rows (one u32 table entry per nibble) and k >= 2:
// full tiles through the hand-scheduled asm tile, the ragged last tile of a
// block through encode_tile<..., TAIL>. PARK (<= 5 groups): local parities
// are stored at the end of each tile (ecw_encode_asm.hpp). Pointer mode
// hands the asm the addresses of the pointer tables in the kernel
// arguments: `rows` is the first argument, so it sits at offset 0 of the
// kernarg segment (taking the address of the by-value argument itself
// would make the compiler copy all 3 KiB of it to scratch).
#ifndef ECW_ASM_MIN_WAVES_NW2
#define ECW_ASM_MIN_WAVES_NW2 4  // 128 VGPRs: the 8-row tile uses 110
#endif
#ifndef ECW_ASM_MIN_WAVES_NW4
#define ECW_ASM_MIN_WAVES_NW4 3  // 168 VGPRs: the 16-row tile uses 142
#endif
#ifndef ECW_ASM_TPB4
// 9-16 rows: workgroups of 2 tiles (512 threads) share one copy of the 64 KiB
// (k = 128) tables, so the LDS holds tables for 16 waves per CU instead of 8
#define ECW_ASM_TPB4 2
#endif
#ifndef ECW_ASM_TPB1
#define ECW_ASM_TPB1 1  // <= 4 rows (tuning: 2 = workgroups of two tiles sharing the 16 KiB of tables)
#endif
// column tiles per workgroup of the asm kernel (kBlock threads per tile)
template <int NW>
constexpr int asm_tpb() {
  return NW == 4 ? ECW_ASM_TPB4 : NW == 1 ? ECW_ASM_TPB1 : 1;
}

// Copy the packed tables (n16 x 16 B) into LDS, four loads in flight per lane
// (one at a time, each waited for before its LDS write, took four round trips
// at k = 128).
template <int NT = kBlock>
__device__ __forceinline__ void stage_tables(uint8_t* lds, const uint4* __restrict__ tbl, int n16) {
  uint4* l4 = reinterpret_cast<uint4*>(lds);
  int i = threadIdx.x;
  for (; i + 3 * NT < n16; i += 4 * NT) {
    const uint4 a = tbl[i], b = tbl[i + NT], c = tbl[i + 2 * NT], d = tbl[i + 3 * NT];
    l4[i] = a;
    l4[i + NT] = b;
    l4[i + 2 * NT] = c;
    l4[i + 3 * NT] = d;
  }
  for (; i < n16; i += NT) l4[i] = tbl[i];
}

// Next tile of a ticket-ordered launch (EncodeGeom::ticket): lane 0 of the
// workgroup takes a ticket, the slot after the LDS tables hands it to the rest.
__device__ __forceinline__ uint32_t take_ticket(const EncodeGeom& g, uint32_t* slot, uint32_t tiles = 1) {
  __syncthreads();  // every wave has read the previous ticket
  if (threadIdx.x == 0) *slot = g.tile_begin + static_cast<uint32_t>(atomicAdd(g.ticket, tiles));
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*slot);
}

template <int LOCAL, bool PARK, class Rows, int NW = 1>
__global__ __launch_bounds__(kBlock * asm_tpb<NW>(), NW == 1   ? ECW_ASM_MIN_WAVES
                                                   : NW == 2 ? ECW_ASM_MIN_WAVES_NW2
                                                             : ECW_ASM_MIN_WAVES_NW4) void encode_kernel_asm(
    const Rows rows, const EncodeGeom g, const uint4* __restrict__ tbl) {
  constexpr uint32_t TPB = asm_tpb<NW>();
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int n16 = g.k * 8 * NW;
#ifndef ECW_DIAG_NOSTAGE  // diagnostic builds only: time the encode without staging its tables
  stage_tables<kBlock * TPB>(lds, tbl, n16);
  __syncthreads();
#else
  (void)n16;
#endif
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds)));
  const int k = __builtin_amdgcn_readfirstlane(g.k);
  const int r = LOCAL == kLocalNone ? k : __builtin_amdgcn_readfirstlane(g.r);
  const int nrows = __builtin_amdgcn_readfirstlane(g.nrows);
  const uint32_t wmask = __builtin_amdgcn_readfirstlane(g.wmask), ww = __builtin_amdgcn_readfirstlane(g.wwidth);
  // TPB > 1: waves [4h, 4h + 4) take tile h of the workgroup's TPB consecutive
  // tiles (h is wave-uniform)
  const uint32_t lane_col = (threadIdx.x % kBlock) * kLaneBytes;
  const uint32_t half = __builtin_amdgcn_readfirstlane(threadIdx.x / kBlock);
  // the ticket slot sits after the tables: a static __shared__ variable would
  // shift the table records off the 64*NW alignment the LDS addressing relies on
  uint32_t* slot = reinterpret_cast<uint32_t*>(lds + static_cast<uint32_t>(g.k) * 128 * NW);
  const bool tickets = g.ticket != nullptr;
  // Full column tiles only (tile = stripe * per.d + column tile; the ragged
  // last tile of every block is encode_tail_kernel's): nothing but the asm
  // tile and a few scalar instructions per tile, so nothing lives in scratch
  // and no compiler-issued memory operation drains the ring between tiles.
  // Every wave runs every iteration (take_ticket holds a barrier); a wave whose
  // tile is past the end skips the work.
  for (uint32_t t0 = tickets ? take_ticket(g, slot, TPB) : g.tile_begin + static_cast<uint32_t>(wg_slot(g.remap)) * TPB;
       t0 < g.tile_end; t0 = tickets ? take_ticket(g, slot, TPB) : t0 + gridDim.x * TPB) {
    const uint32_t tile = t0 + half;
    if (tile >= g.tile_end) continue;
    const uint32_t s = fast_div(tile, g.per);
    if (s >= static_cast<uint32_t>(g.stripes)) continue;  // never past the batch, whatever the launch says
    const uint32_t col = (tile - s * g.per.d) * kTileBytes + lane_col;
    if constexpr (std::is_same<Rows, SlabRows>::value) {
      const uint64_t bs = rows.bstride, pbs = rows.pbstride;
      const uint8_t* sb = uniform_ptr(rows.base + static_cast<uint64_t>(s) * rows.sstride);
      const uint8_t* pb = uniform_ptr(rows.pbase + static_cast<uint64_t>(s) * rows.psstride);
      encode_tile_asm<LOCAL, PARK, false, NW>(sb, const_cast<uint8_t*>(pb + static_cast<uint64_t>(g.m) * pbs),
                                              const_cast<uint8_t*>(pb + static_cast<uint64_t>(g.row0) * pbs), bs,
                                              pbs, k, r, nrows, lds_base, col, wmask, ww);
    } else if constexpr (std::is_same<Rows, PtrTabRows>::value) {
      // this stripe's rows of the device pointer tables, read with s_load
      const uint8_t* st = uniform_ptr(reinterpret_cast<const uint8_t*>(rows.src + static_cast<uint64_t>(s) * k));
      const uint8_t* dt = uniform_ptr(reinterpret_cast<const uint8_t*>(rows.dst + static_cast<uint64_t>(s) * rows.np));
      encode_tile_asm<LOCAL, PARK, true, NW>(st, const_cast<uint8_t*>(dt + static_cast<uint64_t>(g.m) * sizeof(void*)),
                                             const_cast<uint8_t*>(dt + static_cast<uint64_t>(g.row0) * sizeof(void*)),
                                             0, 0, k, r, nrows, lds_base, col, wmask, ww);
    } else {
      const uint8_t* ka = uniform_ptr(reinterpret_cast<const uint8_t*>(
          reinterpret_cast<uintptr_t>(__builtin_amdgcn_kernarg_segment_ptr())));
      const uint8_t* dtab = ka + offsetof(PtrRows, dst);
      encode_tile_asm<LOCAL, PARK, true, NW>(ka + offsetof(PtrRows, src),
                                             const_cast<uint8_t*>(dtab + static_cast<uint64_t>(nrows) * sizeof(void*)),
                                             const_cast<uint8_t*>(dtab), 0, 0, k, r, nrows, lds_base, col, wmask, ww);
    }
  }
}

// The ragged last column tile of every stripe's blocks (len % kTileBytes != 0)
// for the asm launches, one workgroup per stripe: byte-granular loads and
// stores through the compiler-scheduled tile.
template <int NW, int LOCAL, class Rows>
__global__ __launch_bounds__(kBlock) void encode_tail_kernel(const Rows rows, const EncodeGeom g,
                                                             const uint4* __restrict__ tbl) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  stage_tables(lds, tbl, g.k * 8 * NW);
  __syncthreads();
  const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds));
  const uint32_t col0 = static_cast<uint32_t>(g.len / kTileBytes) * kTileBytes;
  for (int s = blockIdx.x; s < g.stripes; s += gridDim.x) {
    const TileAt cur{s, col0 + threadIdx.x * kLaneBytes, false};
    uint4 ring[kPrefetchEncAsmTail];
    ring_prologue<kPrefetchEncAsmTail, true>(ring, rows, g, cur);
    encode_tile<NW, kPrefetchEncAsmTail, LOCAL, true>(rows, g, cur, ring, false, cur, lds_base);
  }
}

// ---- XOR reduce: dst = src_0 ^ ... ^ src_{n-1} ----------------------------
__device__ __forceinline__ const uint8_t* xsrc(const XorPtr& a, int, int i) { return a.src[i]; }
__device__ __forceinline__ const uint8_t* xsrc(const XorSlab& a, int s, int i) {
  return a.base + s * a.sstride + static_cast<uint64_t>(a.idx[i]) * a.bstride;
}
__device__ __forceinline__ const uint8_t* xsrc(const XorSplit& a, int s, int i) {
  if (i < a.ndata) return a.base + s * a.sstride + static_cast<uint64_t>(a.idx[i]) * a.bstride;
  return a.pbase + s * a.psstride + static_cast<uint64_t>(a.idx[i]) * a.pbstride;
}
// Pointer tables are read through the constant address space at a uniform
// address, so the block pointers come in with scalar loads (batched by the
// compiler) instead of one vector load per lane and source, each of which the
// source's data loads had to wait for.
#ifndef ECW_XORTAB_SCALAR
#define ECW_XORTAB_SCALAR 1
#endif
template <class T>
__device__ __forceinline__ T* uniform_table_entry(T* const* table, uint64_t index) {
#if ECW_XORTAB_SCALAR
  const uint64_t a = reinterpret_cast<uint64_t>(table + index);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  const __attribute__((address_space(4))) uint64_t* c =
      reinterpret_cast<const __attribute__((address_space(4))) uint64_t*>((static_cast<uint64_t>(hi) << 32) | lo);
  return reinterpret_cast<T*>(*c);
#else
  return table[index];
#endif
}
__device__ __forceinline__ const uint8_t* xsrc(const XorTab& a, int s, int i) {
  return uniform_table_entry(a.src, static_cast<uint64_t>(s) * a.n + i);
}
__device__ __forceinline__ uint8_t* xdst(const XorTab& a, int s) { return uniform_table_entry(a.dst, static_cast<uint64_t>(s)); }
__device__ __forceinline__ uint8_t* xdst(const XorPtr& a, int) { return a.dst; }
__device__ __forceinline__ uint8_t* xdst(const XorSlab& a, int s) { return a.out + s * a.ostride; }
__device__ __forceinline__ uint8_t* xdst(const XorSplit& a, int s) { return a.out + s * a.ostride; }

template <int P, bool TAIL, class Args>
__device__ __forceinline__ void xor_tile(const Args& a, const XorGeom& g, int s, uint32_t col) {
  const uint32_t len = static_cast<uint32_t>(g.len);
  if (TAIL && col >= len) return;
  const int n = g.n;
  uint4 ring[P];
#pragma unroll
  for (int p = 0; p < P; ++p) ring[p] = ld16<TAIL, ECW_XOR_NT>(xsrc(a, s, p < n ? p : n - 1), col, len);
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int i0 = 0; i0 < n; i0 += P) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int i = i0 + p;
      if (i < n) acc = xor4(acc, ring[p]);
      ring[p] = ld16<TAIL, ECW_XOR_NT>(xsrc(a, s, i + P < n ? i + P : n - 1), col, len);
    }
  }
  st16<TAIL, ECW_XOR_NT>(xdst(a, s), col, len, acc);
}

template <int P, class Args>
__global__ __launch_bounds__(kBlock) void xor_kernel(const Args a, const XorGeom g, const FastDiv per) {
  const uint32_t total = static_cast<uint32_t>(g.stripes) * per.d;
  for (uint32_t tile = static_cast<uint32_t>(wg_slot()); tile < total; tile += gridDim.x) {
    const int s = static_cast<int>(fast_div(tile, per));
    const uint32_t col0 = (tile - static_cast<uint32_t>(s) * per.d) * kTileBytes;
    const uint32_t col = col0 + threadIdx.x * kLaneBytes;
    if (static_cast<uint64_t>(col0) + kTileBytes <= g.len)
      xor_tile<P, false>(a, g, s, col);
    else
      xor_tile<P, true>(a, g, s, col);
  }
}

// Source count known at compile time (n <= ECW_XOR_FIXED_MAX, every CL repair
// of a group of up to that many blocks): straight-line code, no loop. The
// runtime-n ring above compiles to a loop whose head waits vmcnt(0) (LLVM's
// waitcnt pass merges the prologue's and the back-edge's load orders), i.e.
// every wave drains its loads every P rows; straight-line code gets exact
// counted waits, and the source indices come in as one scalar batch.
// Loads are issued with at most W in flight per wave (W >= N: all at once).
#ifndef ECW_XOR_WINDOW
#define ECW_XOR_WINDOW 8
#endif
// Write window of the XOR reduce (XorSched::wwidth > 0): the output store
// waits until the chip-wide 100 MHz constant clock is in the first `wwidth`
// ticks of every `wmask + 1`, as the encode's asm tile does
// (ECW_WRITE_WINDOW, ecw_encode_asm.hpp); at most 16384 polls.
__device__ __forceinline__ void xor_write_window(uint32_t wmask, uint32_t wwidth) {
  if (wwidth == 0) return;
#pragma nounroll
  for (int n = 0; n < 16384; ++n) {
    const uint32_t t = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
    if ((t & wmask) < wwidth) break;
    __builtin_amdgcn_s_sleep(2);
  }
}

// One workgroup reduces K consecutive column tiles of one stripe. K = 1 is
// the plain tile. K > 1 skews the schedule diagonally: load t of the
// straight-line sequence reads source i = t % N at tile (t / N + i) % K, so
// the loads a wave has in flight (and the loads of the workgroups that run
// beside it) fall on K different column tiles of the sources instead of one.
// Blocks allocated separately start at the same offset modulo every large
// power of two, so one column of all n sources can sit on one HBM channel and
// bank, a row apart (SURVEY §7 "channel camping"; the slabs avoid it with a
// +4 KiB block stride, which the reference's per-block buffers,
// NativeCodec.cc:237-248, do not have).
template <int N, int K, bool TAIL, class Args>
__device__ __forceinline__ void xor_tiles_fixed(const Args& a, const XorGeom& g, const XorSched& sc, int s,
                                                uint32_t col) {
  const uint32_t len = static_cast<uint32_t>(g.len);
  if (TAIL && col >= len) return;
  constexpr int T = N * K;
  constexpr int W = ECW_XOR_WINDOW > 0 && ECW_XOR_WINDOW < T ? ECW_XOR_WINDOW : T;
  uint4 v[T];
  uint4 acc[K];
#pragma unroll
  for (int q = 0; q < K; ++q) acc[q] = make_uint4(0, 0, 0, 0);
  // every source pointer first (pointer tables: one batch of scalar loads)
  const uint8_t* sp[N];
#pragma unroll
  for (int i = 0; i < N; ++i) sp[i] = xsrc(a, s, i);
  // the scheduling barriers pin the issue order (the machine scheduler would
  // otherwise pull the first XORs up between the first loads: vmcnt(0) after two)
#pragma unroll
  for (int t = 0; t < T; ++t) {
    v[t] = ld16<TAIL, ECW_XOR_NT>(sp[t % N], col + ((t / N + t % N) % K) * kTileBytes, len);
    __builtin_amdgcn_sched_barrier(0);
    if (t >= W - 1) {
      const int u = t - W + 1;
      uint4& ac = acc[(u / N + u % N) % K];
      ac = xor4(ac, v[u]);
      if (W < T) asm volatile("" : "+v"(ac.x), "+v"(ac.y), "+v"(ac.z), "+v"(ac.w));  // keep the XOR here
    }
  }
#pragma unroll
  for (int u = T - W + 1; u < T; ++u) {
    uint4& ac = acc[(u / N + u % N) % K];
    ac = xor4(ac, v[u]);
  }
  xor_write_window(sc.wmask, sc.wwidth);
  uint8_t* d = xdst(a, s);
#pragma unroll
  for (int q = 0; q < K; ++q) st16<TAIL, ECW_XOR_NT>(d, col + q * kTileBytes, len, acc[q]);
}

// Groups of K column tiles, numbered stripe-major (order 0: group = stripe *
// per + column group) or column-major (order 1: group = column group *
// stripes + stripe, so the workgroups in flight spread over every stripe).
template <int N, int K, class Args>
__global__ __launch_bounds__(kBlock) void xor_kernel_fixed(const Args a, const XorGeom g, const XorSched sc) {
  const uint32_t total = static_cast<uint32_t>(g.stripes) * sc.per.d;
  for (uint32_t grp = static_cast<uint32_t>(wg_slot(sc.remap)); grp < total; grp += gridDim.x) {
    uint32_t s, c;
    if (sc.order) {
      c = fast_div(grp, sc.ns);
      s = grp - c * sc.ns.d;
    } else {
      s = fast_div(grp, sc.per);
      c = grp - s * sc.per.d;
    }
    const uint32_t col0 = c * (K * kTileBytes);
    const uint32_t col = col0 + threadIdx.x * kLaneBytes;
    if (static_cast<uint64_t>(col0) + K * kTileBytes <= g.len) {
      xor_tiles_fixed<N, K, false>(a, g, sc, static_cast<int>(s), col);
    } else {
      // the ragged last group of a stripe: its tiles one by one
      for (uint32_t q = 0; q < static_cast<uint32_t>(K); ++q) {
        const uint32_t c0 = col0 + q * kTileBytes;
        if (c0 >= g.len) break;
        if (static_cast<uint64_t>(c0) + kTileBytes <= g.len)
          xor_tiles_fixed<N, 1, false>(a, g, sc, static_cast<int>(s), col + q * kTileBytes);
        else
          xor_tiles_fixed<N, 1, true>(a, g, sc, static_cast<int>(s), col + q * kTileBytes);
      }
    }
  }
}

// ---- synthetic fill (ecwide.h: ecw_fill_random_dev) ------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

// Byte i of a block is byte (offset + i) of its generator stream; it lands at
// p + (i / piece) * pstride + i % piece (piece = len: one contiguous block; a
// tiled slab scatters the block's column pieces, so both layouts hold the same
// bytes). piece and offset are multiples of 16, so a 16-byte group never
// straddles a piece.
__global__ __launch_bounds__(kBlock) void fill_kernel(uint8_t* dst, uint64_t bstride, uint64_t sstride,
                                                      int stripes, int nblocks, uint64_t len, uint64_t piece,
                                                      uint64_t pstride, uint64_t offset, uint64_t seed, int s0,
                                                      int b0) {
  constexpr uint64_t G = 0x9E3779B97F4A7C15ull;
  const uint64_t npair = (len + 15) / 16;
  const uint64_t wbase = offset / 8;
  for (int y = blockIdx.y; y < stripes * nblocks; y += gridDim.y) {
    const int s = y / nblocks, b = y - s * nblocks;
    const uint64_t key = mix64(seed + G * (1ull + static_cast<uint64_t>(s0 + s) * 65536ull +
                                           static_cast<uint64_t>(b0 + b)));
    uint8_t* p = dst + s * sstride + static_cast<uint64_t>(b) * bstride;
    for (uint64_t q = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; q < npair;
         q += static_cast<uint64_t>(gridDim.x) * kBlock) {
      const uint64_t w0 = wbase + 2 * q;
      const uint64_t v0 = mix64(key + w0 * G), v1 = mix64(key + (w0 + 1) * G);
      const uint64_t i0 = 16 * q;
      const uint64_t pc = i0 / piece;
      uint8_t* o = p + pc * pstride + (i0 - pc * piece);
      if (i0 + 16 <= len) {
        *reinterpret_cast<uint4*>(o) = make_uint4(static_cast<uint32_t>(v0), static_cast<uint32_t>(v0 >> 32),
                                                  static_cast<uint32_t>(v1), static_cast<uint32_t>(v1 >> 32));
      } else {
        for (int i = 0; i < 16 && i0 + i < len; ++i)
          o[i] = static_cast<uint8_t>((i < 8 ? v0 >> (8 * i) : v1 >> (8 * (i - 8))));
      }
    }
  }
}

// Tunables (overridable with -D for tuning builds; tools/variants.py)
#ifndef ECW_PREFETCH_ENC
#define ECW_PREFETCH_ENC 2
#endif
#ifndef ECW_PREFETCH_XOR
#define ECW_PREFETCH_XOR 4  // repair ring depth: 4 vs 8 +2.6 % on the tiled slab, +0.3 % block slab (tools/layout_ab.py)
#endif
#ifndef ECW_GRID_PER_CU
#define ECW_GRID_PER_CU 256  // encode: workgroups per CU before tiles are grid-strided (256 vs 64: +2.7 %)
#endif
#ifndef ECW_XOR_FIXED_MAX
#define ECW_XOR_FIXED_MAX 32  // XOR reduce over n <= this many sources: straight-line kernel per n (0: off)
#endif
#ifndef ECW_GRID_PER_CU_XOR
#define ECW_GRID_PER_CU_XOR 2048  // XOR reduce: one workgroup per tile up to 512 Ki tiles (+8.6 % at the HBM-filling batch vs 512)
#endif
constexpr int kPrefetchEnc = ECW_PREFETCH_ENC;
constexpr int kPrefetchXor = ECW_PREFETCH_XOR;

// Tile indices are 32-bit (FastDiv): one launch covers at most this many
// tiles; larger batches go in several launches over consecutive stripes.
constexpr uint64_t kMaxTilesPerLaunch = 1ull << 31;

// The same rows from stripe s0 on (a batch split into several launches).
inline PtrRows offset_stripes(const PtrRows& r, int, int) { return r; }  // one stripe
inline SlabRows offset_stripes(const SlabRows& r, int s0, int) {
  SlabRows o = r;
  o.base += static_cast<uint64_t>(s0) * r.sstride;
  o.pbase += static_cast<uint64_t>(s0) * r.psstride;
  return o;
}
inline PtrTabRows offset_stripes(const PtrTabRows& r, int s0, int k) {
  PtrTabRows o = r;
  o.src += static_cast<uint64_t>(s0) * k;
  o.dst += static_cast<uint64_t>(s0) * r.np;
  return o;
}
inline XorPtr offset_stripes(const XorPtr& a, int) { return a; }  // one stripe
inline XorSlab offset_stripes(const XorSlab& a, int s0) {
  XorSlab o = a;
  o.base += static_cast<uint64_t>(s0) * a.sstride;
  o.out += static_cast<uint64_t>(s0) * a.ostride;
  return o;
}
inline XorSplit offset_stripes(const XorSplit& a, int s0) {
  XorSplit o = a;
  o.base += static_cast<uint64_t>(s0) * a.sstride;
  o.pbase += static_cast<uint64_t>(s0) * a.psstride;
  o.out += static_cast<uint64_t>(s0) * a.ostride;
  return o;
}
inline XorTab offset_stripes(const XorTab& a, int s0) {
  XorTab o = a;
  o.src += static_cast<uint64_t>(s0) * a.n;
  o.dst += s0;
  return o;
}

// ECW_DEBUG_LAUNCH=1 (debugging aid): every launch is printed with its grid
// and synchronised, so a faulting kernel names itself.
bool debug_launch() {
  static const bool on = [] {
    const char* e = std::getenv("ECW_DEBUG_LAUNCH");
    return e && e[0] == '1';
  }();
  return on;
}
hipError_t launched(const char* what, dim3 grid, size_t lds, hipStream_t s) {
  hipError_t e = hipGetLastError();
  if (debug_launch()) {
    std::fprintf(stderr, "ecw launch %s grid %u lds %zu: %s", what, grid.x, lds, hipGetErrorString(e));
    const hipError_t f = hipStreamSynchronize(s);
    std::fprintf(stderr, " -> %s\n", hipGetErrorString(f));
    if (e == hipSuccess) e = f;
  }
  return e;
}

unsigned grid_for(uint64_t tiles_total, uint64_t per_cu = ECW_GRID_PER_CU) {
  // memory-bound streaming: enough workgroups to fill 256 CUs many deep,
  // grid-stride beyond that (encode tables are staged once per workgroup)
  const uint64_t cap = 256ull * per_cu;
  return static_cast<unsigned>(tiles_total < cap ? (tiles_total ? tiles_total : 1) : cap);
}

// Launch with `lds` bytes of dynamic LDS; above 64 KiB (9-16-row tables of
// wide stripes: k * 512 B) the kernel's limit is raised first (160 KiB per CU).
template <class K, class... A>
void launch_lds(K kernel, dim3 grid, unsigned threads, size_t lds, hipStream_t s, const A&... a) {
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(lds));
  hipLaunchKernelGGL(kernel, grid, dim3(threads), lds, s, a...);
}

template <int NW, class Rows>
hipError_t launch_encode_nw(const Rows& rows, const EncodeGeom& g, const uint4* tbl, dim3 grid, hipStream_t s) {
  const size_t lds = static_cast<size_t>(g.k) * 128 * NW;
  switch (g.local_mode) {
    case kLocalXor:
      launch_lds(encode_kernel<NW, kPrefetchEnc, kLocalXor, Rows>, grid, kBlock, lds, s, rows, g, tbl);
      break;
    case kLocalZero:
      launch_lds(encode_kernel<NW, kPrefetchEnc, kLocalZero, Rows>, grid, kBlock, lds, s, rows, g, tbl);
      break;
    default:
      launch_lds(encode_kernel<NW, kPrefetchEnc, kLocalNone, Rows>, grid, kBlock, lds, s, rows, g, tbl);
  }
  return launched("encode_kernel", grid, lds, s);
}

template <class Rows, int NW>
hipError_t launch_encode_tail(const Rows& rows, const EncodeGeom& g, const uint4* tbl, hipStream_t s) {
  const size_t lds = static_cast<size_t>(g.k) * 128 * NW;
  const dim3 grid(static_cast<unsigned>(g.stripes < 65536 ? g.stripes : 65536));
  switch (g.local_mode) {
    case kLocalXor:
      launch_lds(encode_tail_kernel<NW, kLocalXor, Rows>, grid, kBlock, lds, s, rows, g, tbl);
      break;
    case kLocalZero:
      launch_lds(encode_tail_kernel<NW, kLocalZero, Rows>, grid, kBlock, lds, s, rows, g, tbl);
      break;
    default:
      launch_lds(encode_tail_kernel<NW, kLocalNone, Rows>, grid, kBlock, lds, s, rows, g, tbl);
  }
  return launched("encode_tail_kernel", grid, lds, s);
}

#ifndef ECW_ASM_LDS_PAD
#define ECW_ASM_LDS_PAD 0
#endif
template <class Rows, int NW>
hipError_t launch_encode_asm(const Rows& rows, const EncodeGeom& g, const uint4* tbl, dim3 grid, hipStream_t s) {
  // + ticket slot (+ ECW_ASM_LDS_PAD: tuning builds only, fewer workgroups per CU)
  const size_t lds = static_cast<size_t>(g.k) * 128 * NW + 16 + ECW_ASM_LDS_PAD;
  constexpr unsigned TPB = asm_tpb<NW>();
  const unsigned threads = kBlock * TPB;
  grid.x = (grid.x + TPB - 1) / TPB;  // the launch's tiles in workgroups of TPB
  switch (g.local_mode) {
    case kLocalXor:
      if (g.groups <= kMaxParkedLocals)
        launch_lds(encode_kernel_asm<kLocalXor, true, Rows, NW>, grid, threads, lds, s, rows, g, tbl);
      else
        launch_lds(encode_kernel_asm<kLocalXor, false, Rows, NW>, grid, threads, lds, s, rows, g, tbl);
      break;
    case kLocalZero:
      launch_lds(encode_kernel_asm<kLocalZero, false, Rows, NW>, grid, threads, lds, s, rows, g, tbl);
      break;
    default:
      launch_lds(encode_kernel_asm<kLocalNone, false, Rows, NW>, grid, threads, lds, s, rows, g, tbl);
  }
  return launched("encode_kernel_asm", grid, lds, s);
}

// The slab is encoded in launch windows of one grid's worth of tiles (256 CUs x
// ECW_GRID_PER_CU), one tile per workgroup, instead of one grid-strided launch:
// a grid-strided workgroup jumps a whole grid ahead when it finishes, spreading
// the in-flight tiles over several distant regions. Same allocation, interleaved:
// +3.5 % encode at the 272 GiB HBM-filling slab (8 windows), +0.3..1.5 % at the
// bench shape (2 windows) (profiles/r01_encode_launch_window_ab.log).
// ECW_COHORT_TILES > 0 sets another window, < 0 launches the slab at once.
#ifndef ECW_COHORT_TILES
#define ECW_COHORT_TILES 0
#endif
// Slabs of at least ECW_TICKET_MIN_TILES tiles (4 windows: 1 GiB of column per
// data row, e.g. the 272 GiB HBM-filling batch) run as ONE launch whose
// workgroups take tiles in order from a ticket counter: +2.9 % encode over the
// windows at 240 x 8 MiB stripes, but -1.4..-9 % on smaller slabs
// (profiles/r01_encode_ticket_ab.log). 0 disables.
#ifndef ECW_TICKET_MIN_TILES
#define ECW_TICKET_MIN_TILES (4ull * 256 * ECW_GRID_PER_CU)
#endif

// Write window of the asm tile (ECW_WRITE_WINDOW in ecw_encode_asm.hpp): every
// tile's parity stores wait for the first 64 of every 2048 ticks (0.64 us of
// 20.5 us) of the 100 MHz constant clock. It pays for whole-block layouts,
// where a column tile's parity stores go to m + g rows a block apart: encode
// +4..7 % on the block slab (5678 -> 5910, 5538 -> 5948 GB/s), +5.6 % pointer
// mode, +10 % pointer tables over separate allocations (5386 -> 5920)
// (profiles/r02_encode_write_window*.log; 2^10..2^12-tick periods within 1 %,
// 2^13 and longer lock the workgroups into generations that wait for the
// window: -6 %). Layouts whose parities sit in a region of their own gain
// nothing reliable: tiled slab -2.1 / +1.6 / -0.9 %, whole-block split slab +5 /
// -2.4 % on different boxes, so slabs use it only with in-slab parities.
// Launches under 8192 tiles go without (a window adds up to 20 us of latency).
// Narrow stripes lose: the window re-synchronises the resident workgroups into
// generations whose time is rounded up to whole periods, which costs more
// than it saves when a tile's reads take only a few periods (block slab k=32
// -4 %, pointer mode k=32 -8 %, k=8 -47 %; k=64 +5.5 %, k=96 +4.2 %, k=200 +7 %,
// RS(128, 3) +3.1 %; profiles/r02_encode_write_window_k*.log), so only k >= 64
// uses it, and not the 5-8-row tile (4 waves per SIMD: -1.2 %).
// ECW_WRITE_WINDOW = auto (default) | off | on | "LOG2P,W" overrides the choice
// (tuning; read per launch).
inline bool window_shape(const EncodeGeom& g) {
  return g.k >= 64 && g.nrows <= 4 && g.len >= 65536 && static_cast<uint64_t>(g.stripes) * g.tiles >= 8192;
}
// Slabs of whole blocks: the block slab (parity rows after each stripe's data
// rows) since round 2; the split slab (parities in a region of their own)
// since round 4, interleaved in one process: 5557 -> 6350 and 5846 -> 6285 GB/s
// (profiles/r04b_repair_ab_*.log; round 2 had measured +5.0 / -2.4 % on two
// boxes). The tiled slab's 8 KiB units are below window_shape's 64 KiB.
inline bool window_auto(const SlabRows&, const EncodeGeom& g) { return window_shape(g); }
inline bool window_auto(const PtrRows&, const EncodeGeom& g) { return window_shape(g); }
inline bool window_auto(const PtrTabRows&, const EncodeGeom& g) { return window_shape(g); }

// Tile order of the encode: the per-XCD contiguous order (wg_slot) for blocks
// behind pointers (the caller's own allocations). Their encode keeps the
// address-translation path busy (UTCL2 busy 96 % of the launch over 1088
// separate 64 MiB allocations, 93 % on the split slab, 4 % on the tiled slab;
// separate allocations take 2x the split slab's UTCL1 misses:
// profiles/r04b_repair_pmc_summary.txt); with the remap the workgroups
// resident on a CU take tiles 128 KiB apart instead of 1 MiB and share more
// translations. Interleaved (profiles/r04_remap_1/2.log): separate blocks
// 6012 -> 6211 and 5932 -> 6136 GB/s; slabs within +-1 %, so they keep the
// dispatch order.
inline uint32_t remap_auto(const SlabRows&) { return 0; }
inline uint32_t remap_auto(const PtrRows&) { return 1; }
inline uint32_t remap_auto(const PtrTabRows&) { return 1; }

template <class Rows>
void set_write_window(const Rows& rows, EncodeGeom& g) {
  uint32_t log2p = 11, w = 64;
  bool on = window_auto(rows, g);
  if (const char* e = std::getenv("ECW_WRITE_WINDOW")) {
    unsigned a = 0, b = 0;
    if (!std::strcmp(e, "off") || !std::strcmp(e, "0")) {
      on = false;
    } else if (!std::strcmp(e, "on")) {
      on = true;
    } else if (std::sscanf(e, "%u,%u", &a, &b) == 2 && a >= 4 && a <= 24 && b > 0) {
      on = true;
      log2p = a;
      w = b;
    }
  }
  g.wmask = (1u << log2p) - 1;
  g.wwidth = on ? w : 0;
}

// One launch range: stripes [0, g0.stripes) of `rows`, fewer than
// kMaxTilesPerLaunch tiles. The asm kernel covers the full column tiles (in
// launch windows, or in one ticket-ordered launch), encode_tail_kernel the
// ragged last tile of every block; k = 1 (or ECW_ENC_ASM=0) takes the
// compiler-scheduled kernel, which handles both.
template <class Rows>
hipError_t launch_encode_range(const Rows& rows, const EncodeGeom& g0, const uint4* tbl, hipStream_t s,
                               unsigned long long* ticket) {
  const bool asm_tile = ECW_ENC_ASM && g0.k >= 2;
  const uint64_t full = g0.len / kTileBytes;
  const uint64_t per = asm_tile ? full : g0.tiles;  // tiles per stripe in the launch's numbering
  const uint64_t total = static_cast<uint64_t>(g0.stripes) * per;
  // what the kernels' 32-bit tile numbering assumes (the grid never covers a
  // tile past the slab)
  if (g0.stripes < 0 || total >= kMaxTilesPerLaunch || per > 0xFFFFFFFFull) return hipErrorInvalidValue;
  EncodeGeom gw = g0;
  set_write_window(rows, gw);
  gw.remap = xcd_remap_env(remap_auto(rows));
  gw.per = make_fastdiv(static_cast<uint32_t>(per ? per : 1));
  gw.ticket = nullptr;
  const uint64_t win = ECW_COHORT_TILES > 0    ? static_cast<uint64_t>(ECW_COHORT_TILES)
                       : ECW_COHORT_TILES == 0 ? 256ull * ECW_GRID_PER_CU
                                               : total;
  if (asm_tile && ticket && total > 0 && encode_uses_ticket(total, g0.k)) {
    // one ticket-ordered launch; the caller zeroed the counter for it
    EncodeGeom g = gw;
    g.tile_begin = 0;
    g.tile_end = static_cast<uint32_t>(total);
    g.ticket = ticket;
    const dim3 grid(grid_for(total));
    const hipError_t e = g.nrows <= 4   ? launch_encode_asm<Rows, 1>(rows, g, tbl, grid, s)
                         : g.nrows <= 8 ? launch_encode_asm<Rows, 2>(rows, g, tbl, grid, s)
                                        : launch_encode_asm<Rows, 4>(rows, g, tbl, grid, s);
    if (e != hipSuccess) return e;
  } else {
    for (uint64_t t0 = 0; t0 < total; t0 += win) {
      EncodeGeom g = gw;
      g.tile_begin = static_cast<uint32_t>(t0);
      g.tile_end = static_cast<uint32_t>(t0 + win < total ? t0 + win : total);
      const dim3 grid(grid_for(g.tile_end - g.tile_begin));
      hipError_t e;
      if (asm_tile)
        e = g.nrows <= 4   ? launch_encode_asm<Rows, 1>(rows, g, tbl, grid, s)
            : g.nrows <= 8 ? launch_encode_asm<Rows, 2>(rows, g, tbl, grid, s)
                           : launch_encode_asm<Rows, 4>(rows, g, tbl, grid, s);
      else
        e = g.nrows <= 4   ? launch_encode_nw<1>(rows, g, tbl, grid, s)
            : g.nrows <= 8 ? launch_encode_nw<2>(rows, g, tbl, grid, s)
                           : launch_encode_nw<4>(rows, g, tbl, grid, s);
      if (e != hipSuccess) return e;
    }
  }
  if (asm_tile && full < g0.tiles)
    return g0.nrows <= 4   ? launch_encode_tail<Rows, 1>(rows, gw, tbl, s)
           : g0.nrows <= 8 ? launch_encode_tail<Rows, 2>(rows, gw, tbl, s)
                           : launch_encode_tail<Rows, 4>(rows, gw, tbl, s);
  return hipSuccess;
}

template <class Rows>
hipError_t launch_encode(const Rows& rows, const EncodeGeom& g0, const void* d_tbl, hipStream_t s,
                         unsigned long long* ticket) {
  if (static_cast<uint64_t>(g0.stripes) * g0.tiles == 0) return hipSuccess;
  if (g0.nrows < 1 || g0.nrows > kMaxPassRows || g0.k < 1 || g0.len > 0xFFFFFFF0ull ||
      g0.tiles != (g0.len + kTileBytes - 1) / kTileBytes || g0.tiles > kMaxTilesPerLaunch)
    return hipErrorInvalidValue;
  (void)hipGetLastError();  // report this call's launch errors, not an earlier one
  const uint4* tbl = static_cast<const uint4*>(d_tbl);
  const int per_launch = stripes_per_launch(g0.tiles);
  if (g0.stripes <= per_launch) return launch_encode_range(rows, g0, tbl, s, ticket);
  for (int64_t s0 = 0; s0 < g0.stripes; s0 += per_launch) {  // (no ticket: the counter serves one launch)
    EncodeGeom g = g0;
    g.stripes = static_cast<int>(g0.stripes - s0 < per_launch ? g0.stripes - s0 : per_launch);
    const hipError_t e = launch_encode_range(offset_stripes(rows, static_cast<int>(s0), g0.k), g, tbl, s, nullptr);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int N, int K, class Args>
hipError_t launch_xor_fixed(const Args& a, const XorGeom& g, const XorSched& sc, dim3 grid, hipStream_t s) {
  if constexpr (N >= 1) {
    if (g.n < N) return launch_xor_fixed<N - 1, K>(a, g, sc, grid, s);
    hipLaunchKernelGGL((xor_kernel_fixed<N, K, Args>), grid, dim3(kBlock), 0, s, a, g, sc);
    return launched("xor_kernel_fixed", grid, 0, s);
  }
  return hipErrorInvalidValue;
}

// Schedule of the straight-line XOR kernel: tiles per workgroup (skew K),
// group order, write window. ECW_XOR_SCHED = "K,ORDER[,LOG2P,W]" overrides
// the default (tuning; read per launch). K is 1 or ECW_XOR_SKEW_K (and 2, 4,
// 8 in builds with -DECW_XOR_SKEW_ALL=1).
#ifndef ECW_XOR_SKEW_K
#define ECW_XOR_SKEW_K 4
#endif
#ifndef ECW_XOR_SKEW_ALL
#define ECW_XOR_SKEW_ALL 0
#endif
struct XorChoice {
  int skew;
  uint32_t order, log2p, wwidth;
};
// Default, from interleaved A/Bs in one process over the same blocks
// (tools/repair_ab.py; profiles/r04_repair_ab_*.log, r04b_*, r04c_*; CL D0
// repair, 4 stripes of 64 MiB blocks):
//  * whole blocks (>= 64 KiB: the reference's per-block buffers, the split
//    and block slabs) take the diagonal skew, K = 4: blocks allocated one by
//    one start at the same offset modulo 2 MiB and beyond, so one column of
//    all n sources can sit on one HBM channel and bank a row apart; reading
//    the sources at K different column tiles at once spreads them. Separate
//    torch allocations 6008 -> 6248, one allocation at block stride B 5973 ->
//    6423 GB/s at n = 27; n = 4: 5950 -> 6540;
//  * ... and, from n >= 8 sources and 8192 column tiles per launch, the write
//    window (2^11 ticks, W = 64, as the encode's): n = 27 separate blocks 6612,
//    stride-B allocation 6734, split slab 5847 -> 6658 in a process where it
//    had landed slowly (+0.6 % where it had not), block slab 6658 -> 6765;
//    n = 9 6550-6558 against 6191-6320 without it. Below 8 sources a tile's
//    reads take too few window periods and the window locks the workgroups
//    into generations (n = 4: -2..-10 %; K = 1 with the window: -50..-70 %);
//  * the tiled slab's 8 KiB units keep K = 1 and no window (K = 4: -0.5..-8 %,
//    window -2..-70 %: its sources are one contiguous run already).
// Column-major group order and K = 2 / 8 gained less than K = 4 everywhere.
//  * round 4, later: the tiled slab's 16 KiB units (k <= 32, slab.default_chunk)
//    are one whole group of K = 4 tiles and take the same schedule: CL(32, 8, 2)
//    6240 -> 6379, CL(32, 11, 3) 6259 -> 6537 GB/s (profiles/r04_k32r_cfg1/0.log);
//    K = 2 on the 8 KiB units of k = 128: +0.5 % with the window, -2 % without
//    (r04_k128r_tiled.log), so they keep K = 1.
template <class Args>
inline XorChoice xor_choice(const XorGeom& g) {
  constexpr uint64_t group = static_cast<uint64_t>(ECW_XOR_SKEW_K) * kTileBytes;
  const bool whole = g.len >= 65536 || (g.len >= group && g.len % group == 0);
  XorChoice c{whole ? ECW_XOR_SKEW_K : 1, 0, 11, 0};
  if (whole && g.n >= 8 && static_cast<uint64_t>(g.stripes) * g.tiles >= 8192) c.wwidth = 64;
  if (const char* e = std::getenv("ECW_XOR_SCHED")) {
    int k = 1;
    unsigned o = 0, lp = 11, w = 0;
    const int got = std::sscanf(e, "%d,%u,%u,%u", &k, &o, &lp, &w);
    if (got >= 1) {  // an override names the whole schedule: no window unless given
      c.skew = k;
      c.wwidth = 0;
    }
    if (got >= 2) c.order = o ? 1 : 0;
    if (got >= 4 && lp >= 4 && lp <= 24) {
      c.log2p = lp;
      c.wwidth = w;
    }
  }
  return c;
}

template <int K, class Args>
hipError_t launch_xor_skew(const Args& a, const XorGeom& g, const XorChoice& c, hipStream_t s) {
  const uint64_t per = (g.tiles + K - 1) / K;
  const uint64_t total = static_cast<uint64_t>(g.stripes) * per;
  XorSched sc{};
  sc.per = make_fastdiv(static_cast<uint32_t>(per));
  sc.ns = make_fastdiv(static_cast<uint32_t>(g.stripes > 0 ? g.stripes : 1));
  sc.order = c.order;
  sc.remap = xcd_remap_env(0);  // the XOR: -0.4..-5 % with it (profiles/r04_remap_*.log)
  sc.wmask = (1u << c.log2p) - 1;
  sc.wwidth = c.wwidth;
  const dim3 grid(grid_for(total, ECW_GRID_PER_CU_XOR));
  return launch_xor_fixed<ECW_XOR_FIXED_MAX, K>(a, g, sc, grid, s);
}

template <class Args>
hipError_t launch_xor_range(const Args& a, const XorGeom& g, hipStream_t s) {
  const uint64_t total = static_cast<uint64_t>(g.stripes) * g.tiles;
  if (total == 0) return hipSuccess;
  if (g.stripes < 0 || total >= kMaxTilesPerLaunch) return hipErrorInvalidValue;  // 32-bit tile numbering
  // ring depth <= n: the ring refills past the last row re-read row n-1, so a
  // depth-8 ring over 1-2 sources would load every byte up to 8 times
  const dim3 grid(grid_for(total, ECW_GRID_PER_CU_XOR)), block(kBlock);
  const FastDiv per = make_fastdiv(static_cast<uint32_t>(g.tiles));
  if (g.n <= ECW_XOR_FIXED_MAX) {
    const XorChoice c = xor_choice<Args>(g);
#if ECW_XOR_SKEW_ALL
    if (c.skew == 2) return launch_xor_skew<2>(a, g, c, s);
    if (c.skew == 8) return launch_xor_skew<8>(a, g, c, s);
    if (c.skew == 4) return launch_xor_skew<4>(a, g, c, s);
#endif
    if (c.skew == ECW_XOR_SKEW_K) return launch_xor_skew<ECW_XOR_SKEW_K>(a, g, c, s);
    return launch_xor_skew<1>(a, g, c, s);
  }
  if (g.n <= 1)
    hipLaunchKernelGGL((xor_kernel<1, Args>), grid, block, 0, s, a, g, per);
  else if (g.n <= 2)
    hipLaunchKernelGGL((xor_kernel<2, Args>), grid, block, 0, s, a, g, per);
  else if (g.n <= 4)
    hipLaunchKernelGGL((xor_kernel<4, Args>), grid, block, 0, s, a, g, per);
  else
    hipLaunchKernelGGL((xor_kernel<kPrefetchXor, Args>), grid, block, 0, s, a, g, per);
  return launched("xor_kernel", grid, 0, s);
}

template <class Args>
hipError_t launch_xor(const Args& a, const XorGeom& g, hipStream_t s) {
  if (static_cast<uint64_t>(g.stripes) * g.tiles == 0) return hipSuccess;
  if (g.n < 1 || g.n > kMaxSrc || g.len > 0xFFFFFFF0ull || g.tiles > kMaxTilesPerLaunch) return hipErrorInvalidValue;
  (void)hipGetLastError();  // report this call's launch error, not an earlier one
  // tile indices are 32-bit: batches of more than kMaxTilesPerLaunch tiles go
  // in several launches over consecutive stripe ranges
  const int per_launch = stripes_per_launch(g.tiles);
  for (int64_t s0 = 0; s0 < g.stripes; s0 += per_launch) {
    XorGeom gs = g;
    gs.stripes = static_cast<int>(g.stripes - s0 < per_launch ? g.stripes - s0 : per_launch);
    const hipError_t e = launch_xor_range(offset_stripes(a, static_cast<int>(s0)), gs, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// ---- small-stripe request service (ecw_internal.hpp SvcCtl) ----------------
#ifndef ECW_SVC_TRACE
#define ECW_SVC_TRACE 0  // tools only: wall-clock stamps of each request's phases (ecw_codec.cpp svc::)
#endif
__device__ __forceinline__ unsigned long long sys_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long sys_load_relaxed(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The request as the workgroup sees it (copied from the slot by lane 0).
struct SvcReq {
  const uint4* tbl;
  uint8_t* data;
  uint8_t* out;
  unsigned long long len, cs;
  unsigned long long serial;
  int k, nrows, m, r, groups, local_mode, nw, flags;
};
constexpr int kSvcReqWords = 10;
static_assert(sizeof(SvcReq) == 8 * kSvcReqWords, "SvcReq mirrors the request words of SvcSlot");
static_assert(offsetof(SvcSlot, flags) + sizeof(int) - offsetof(SvcSlot, tbl) == sizeof(SvcReq), "SvcSlot request layout");

#ifndef ECW_SVC_ABLATE
#define ECW_SVC_ABLATE 0  // tuning only: 1 leaves the GF products out of served requests
#endif

// A part is a workgroup of kSvcThreads lanes, one dword (4 columns) each: a
// 1 KiB column unit per step. One wave alone was bound by its own issue: the
// GF products of a k=11 call (352 table lookups and ~1000 VALU per lane when
// each lane held 16 columns) took 2.6 us, more than its PCIe fetch (1.5 us);
// four waves of one dword per lane split that over the CU's four SIMDs.

// dword `col` of a row in pinned host memory: the volatile buffer load (all
// rows of a round are issued before the first use), bytes at the ragged end
template <bool TAIL>
__device__ __forceinline__ uint32_t svc_ld4(const uint8_t* row, uint32_t col, uint32_t len) {
  if (!TAIL || col + 4 <= len) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(row), 0, 0x7FFFFFFF, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(col), 0, static_cast<int>(0x80000000u));
  }
  uint32_t w = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (col + i < len) w |= static_cast<uint32_t>(row[col + i]) << (8 * i);
  return w;
}

// Store of a served parity dword: a buffer store (counted in vmcnt only; a
// flat store also counts in lgkmcnt, and the next LDS access would wait for
// it to reach host memory across PCIe), bytes at the ragged end.
template <bool TAIL>
__device__ __forceinline__ void svc_st4(uint8_t* row, uint32_t col, uint32_t len, uint32_t v) {
  if (!TAIL || col + 4 <= len) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(v, rs, static_cast<int>(col), 0, 0);
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (col + i < len) row[col + i] = static_cast<uint8_t>(v >> (8 * i));
}

// gf_row for one dword: acc[p] (NW = 1) / acc[2p], acc[2p+1] (NW = 2) pack the
// products of byte column p
template <int NW>
__device__ __forceinline__ void gf_dw(uint32_t w, uint32_t (&acc)[4 * NW], uint32_t rec) {
  const uint32_t jhi = rec >> 8;
  const uint32_t jlo = (rec & 0xFFu) * 0x01010101u;
  // NW = 2: hi / lo entries interleaved (ecw_gf.hpp packed_pass_tables)
  const uint32_t lo = NW == 1 ? (((w << 2) & 0x3C3C3C3Cu) | jlo) : (((w << 4) & 0xF0F0F0F0u) | jlo);
  const uint32_t hi = NW == 1 ? (((w >> 2) & 0x3C3C3C3Cu) | jlo) : ((w & 0xF0F0F0F0u) | jlo);
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const uint32_t sel = 0x0C0C0400u | static_cast<uint32_t>(b);
    const uint32_t al = __builtin_amdgcn_perm(jhi, lo, sel);
    const uint32_t ah = __builtin_amdgcn_perm(jhi, hi, sel);
    if constexpr (NW == 1) {
      const uint32_t tl = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(al));
      const uint32_t th = *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(ah + 64));
      acc[b] = xor3(acc[b], tl, th);
    } else {
      const unsigned long long tl = *reinterpret_cast<lds_u64*>(static_cast<uintptr_t>(al + 8));
      const unsigned long long th = *reinterpret_cast<lds_u64*>(static_cast<uintptr_t>(ah));
      acc[2 * b] = xor3(acc[2 * b], static_cast<uint32_t>(tl), static_cast<uint32_t>(th));
      acc[2 * b + 1] = xor3(acc[2 * b + 1], static_cast<uint32_t>(tl >> 32), static_cast<uint32_t>(th >> 32));
    }
  }
}

// byte l of the packed accumulators of columns 0..3 -> output row l's dword
template <int NW>
__device__ __forceinline__ uint32_t unpack_dw(const uint32_t (&acc)[4 * NW], int l) {
  const int wsel = NW == 1 ? 0 : (l >> 2);
  const uint32_t bl = static_cast<uint32_t>(l & 3);
  const uint32_t s01 = 0x0C0C0000u | ((4 + bl) << 8) | bl;
  const uint32_t s23 = ((4 + bl) << 24) | (bl << 16) | 0x0C0Cu;
  return __builtin_amdgcn_perm(acc[NW + wsel], acc[wsel], s01) |
         __builtin_amdgcn_perm(acc[3 * NW + wsel], acc[2 * NW + wsel], s23);
}

// One lane's dword of a served request. All input rows of a round of 16 are
// loaded before the first product (one PCIe round trip per 16 rows). The
// request's words are taken into registers first.
template <int NW, int LOCAL, bool TAIL, bool XORROW>
__device__ __forceinline__ void svc_dword(const SvcReq& q, uint32_t lds_base, uint32_t col) {
  const uint32_t len = static_cast<uint32_t>(q.len);
  const int k = q.k, r = q.r, m = q.m, nrows = q.nrows;
  const uint64_t cs = q.cs;
  const uint8_t* data = q.data;
  uint8_t* out = q.out;
  uint32_t acc[4 * NW];
#pragma unroll
  for (int i = 0; i < 4 * NW; ++i) acc[i] = 0;
  uint32_t lacc = 0;
  int gend = r < k ? r : k, t = 0;
  for (int j0 = 0; j0 < k; j0 += 16) {
    uint32_t v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (j0 + u < k) v[u] = svc_ld4<TAIL>(uniform_ptr(data + static_cast<uint64_t>(j0 + u) * cs), col, len);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = j0 + u;
      if (j >= k) continue;
#if ECW_SVC_ABLATE
      acc[0] ^= v[u];  // tuning only: the math left out
#else
      if constexpr (XORROW)
        acc[0] ^= v[u];  // coefficient 1 everywhere: the product is the byte itself
      else
        gf_dw<NW>(v[u], acc, lds_base + static_cast<uint32_t>(j) * (128u * NW));
#endif
      if constexpr (LOCAL != kLocalNone) {
        lacc ^= v[u];
        if (j + 1 == gend) {
          svc_st4<TAIL>(const_cast<uint8_t*>(uniform_ptr(out + static_cast<uint64_t>(m + t) * cs)), col, len,
                        LOCAL == kLocalXor ? lacc : 0u);
          lacc = 0;
          ++t;
          gend = gend + r < k ? gend + r : k;
        }
      }
    }
  }
  if constexpr (XORROW) {
    svc_st4<TAIL>(const_cast<uint8_t*>(uniform_ptr(out)), col, len, acc[0]);
  } else {
    for (int l = 0; l < nrows; ++l)
      svc_st4<TAIL>(const_cast<uint8_t*>(uniform_ptr(out + static_cast<uint64_t>(l) * cs)), col, len,
                    unpack_dw<NW>(acc, l));
  }
}

// This part's column units of a request: units of kSvcThreads dwords dealt
// round-robin over the parts.
template <int NW, int LOCAL, bool XORROW = false>
__device__ __forceinline__ void svc_local(const SvcReq& q, uint32_t lds_base, int part) {
  constexpr uint32_t kUnit = kSvcThreads * 4;
  for (unsigned long long u0 = static_cast<unsigned long long>(part) * kUnit; u0 < q.len;
       u0 += static_cast<unsigned long long>(kSvcParts) * kUnit) {
    const unsigned long long col = u0 + threadIdx.x * 4u;
    if (col + 4 <= q.len)
      svc_dword<NW, LOCAL, false, XORROW>(q, lds_base, static_cast<uint32_t>(col));
    else if (col < q.len)
      svc_dword<NW, LOCAL, true, XORROW>(q, lds_base, static_cast<uint32_t>(col));
  }
}

template <int NW>
__device__ __forceinline__ void svc_request(const SvcReq& q, uint32_t lds_base, int part) {
  // ECWide-H's l_encode / l_middle / l_decode: one all-ones row, no locals
  if (NW == 1 && (q.flags & kSvcXorRow) && q.local_mode == kLocalNone)
    svc_local<1, kLocalNone, true>(q, lds_base, part);
  else if (q.local_mode == kLocalXor)
    svc_local<NW, kLocalXor>(q, lds_base, part);
  else if (q.local_mode == kLocalZero)
    svc_local<NW, kLocalZero>(q, lds_base, part);
  else
    svc_local<NW, kLocalNone>(q, lds_base, part);
}

// Workgroup b is part b % kSvcParts of slot b / kSvcParts. Wave 0 of every
// part polls the slot's request word in host memory (relaxed system-scope
// loads: no cache invalidation per poll; a hand-off from one poller through
// device memory measured 2-6 us slower, the parts sitting on different XCDs)
// and hands it to the part's other waves through LDS; the part reads the
// request words when their generation changed, computes its column units,
// makes its parity stores visible (release, system scope) and publishes its
// own `done` word.
// Part 0 leaves on the stop flag, once NO slot has had a request for
// `idle_ticks`, or after `life_ticks` (checked every 64th poll), and tells its
// other parts so through device memory; the last workgroup out publishes
// exited_epoch. A request posted as part 0 leaves waits for the next epoch
// (the host relaunches on exited_epoch), which serves it whole. A request's
// tables stay staged in LDS while the next request uses the same codec (same
// codec serial: a destroyed codec's successor may get the same table address).
constexpr unsigned long long kSvcLeave = ~0ull;  // SvcDev::Slot::seq: part 0 has left
#ifndef ECW_SVC_COLD_SLEEPS
#define ECW_SVC_COLD_SLEEPS 2  // s_sleep 127 (~3.4 us each) after every poll of a cold slot
#endif

__global__ __launch_bounds__(kSvcThreads) void service_kernel(SvcCtl* ctl, SvcDev* st, unsigned long long epoch,
                                                              unsigned long long idle_ticks,
                                                              unsigned long long life_ticks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  SvcReq* req = reinterpret_cast<SvcReq*>(lds + kSvcLds);
  unsigned long long* bcast = reinterpret_cast<unsigned long long*>(lds + kSvcLds + 80);  // poller -> part: word, leave
  const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds));
  const int si = blockIdx.x / kSvcParts, part = blockIdx.x % kSvcParts;
  SvcSlot* slot = &ctl->slot[si];
  SvcDev::Slot* ds = &st->slot[si];
  const unsigned long long t0 = static_cast<unsigned long long>(wall_clock64());
  // the request word this part last served
  unsigned long long last = sys_load(&slot->done[part]);
  unsigned long long served = t0;      // wall clock of this part's latest request (polling speed)
  unsigned long long req_gen = ~0ull;  // generation of the request words held in LDS (none yet)
  unsigned long long staged = 0;       // serial of the codec whose tables are in LDS (serials start at 1)
  int staged_n16 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) sys_store(&ctl->started_epoch, epoch);
#if ECW_SVC_TRACE
  unsigned long long trace[5] = {0, 0, 0, 0, 0};  // tools only: detect, words, start, computed, fenced
#endif
  for (;;) {
    // --- wait for a request: wave 0 polls the slot's word in host memory
    // (the whole wave loads the same word: uniform control flow) ---
    if (threadIdx.x < kSvcWave) {
      unsigned long long seq = 0;
      bool leave = false;
      bool cold = false;
      for (int spin = 1;; ++spin) {
        seq = sys_load_relaxed(&slot->seq);
        if (seq != last) break;
        // a part without work for 1/20 of the idle exit polls less often:
        // every poll is a PCIe read, and the reads of 128 busy pollers slow
        // the hot slots' own polls and block reads (a caller gets its slot
        // back, so one busy caller keeps the parts of one slot hot)
        if (cold)
          for (int z = 0; z < ECW_SVC_COLD_SLEEPS; ++z) __builtin_amdgcn_s_sleep(127);
        if ((spin & 63) == 0) {
          // part 0 decides for its slot (idle, lifetime, stop) and tells the other
          // parts through device memory; they watch that, the stop flag and the
          // lifetime (plus a margin) only, as a safety net
          const unsigned long long now = static_cast<unsigned long long>(wall_clock64());
          cold = now - served > idle_ticks / 20;  // 1 ms at the default idle exit
          const unsigned long long act = __hip_atomic_load(&st->last_active, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const bool idle = part == 0 && now - (act > t0 ? act : t0) > idle_ticks;
          const bool told =
              part != 0 && __hip_atomic_load(&ds->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kSvcLeave;
          if (idle || told || sys_load_relaxed(&ctl->stop) || now - t0 > life_ticks + (part == 0 ? 0 : idle_ticks)) {
            leave = true;
            break;
          }
        }
      }
      if (threadIdx.x == 0) {
        bcast[0] = seq;
        bcast[1] = leave ? 1 : 0;
      }
    }
    __syncthreads();
    const unsigned long long seq = bcast[0];
    if (bcast[1]) {
      if (part == 0 && threadIdx.x == 0) __hip_atomic_store(&ds->seq, kSvcLeave, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    if (part >= svc_active_parts(seq)) {  // no column unit of this request: nothing to do, nobody waits
      last = seq;
      __syncthreads();  // bcast is rewritten next round
      continue;
    }
    // polling speed follows the requests this part had work in: with 4 KiB
    // calls only parts 0-3 stay hot
    served = static_cast<unsigned long long>(wall_clock64());
#if ECW_SVC_TRACE
    trace[0] = static_cast<unsigned long long>(wall_clock64());
#endif
    // activity counts from the request's arrival, so part 0 never leaves on
    // idle while one of its requests is still in flight
    if (part == 0 && threadIdx.x == 0)
      __hip_atomic_fetch_max(&st->last_active, static_cast<unsigned long long>(wall_clock64()), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the request and its blocks are visible
#if ECW_SVC_TRACE
    trace[1] = static_cast<unsigned long long>(wall_clock64());
#endif
    const unsigned long long gen = seq >> kSvcSeqBits;
    if (gen != req_gen) {  // new request words: 9 lanes read them at once
      if (threadIdx.x < kSvcReqWords)
        reinterpret_cast<unsigned long long*>(req)[threadIdx.x] =
            sys_load_relaxed(reinterpret_cast<const unsigned long long*>(&slot->tbl) + threadIdx.x);
      req_gen = gen;
      __syncthreads();
    }
    const SvcReq& q = *req;  // read from LDS (a private copy would live in scratch)
    const int n16 = q.k * 8 * q.nw;
    // a plain XOR (svc_request's XORROW path) reads no table: the staged ones stay
    const bool xor_only = (q.flags & kSvcXorRow) && q.local_mode == kLocalNone && q.nw == 1;
    if (!xor_only && (q.serial != staged || n16 != staged_n16)) {
      for (int i = threadIdx.x; i < n16; i += kSvcThreads) reinterpret_cast<uint4*>(lds)[i] = q.tbl[i];
      staged = q.serial;
      staged_n16 = n16;
      __syncthreads();
    }
#if ECW_SVC_TRACE
    trace[2] = static_cast<unsigned long long>(wall_clock64());
#endif
    if (q.nw == 2)
      svc_request<2>(q, lds_base, part);
    else
      svc_request<1>(q, lds_base, part);
#if ECW_SVC_TRACE
    trace[3] = static_cast<unsigned long long>(wall_clock64());
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this wave's parities are visible
    __syncthreads();                               // ... and every wave's, before this part's done
    last = seq;
    if (threadIdx.x == 0) {
#if ECW_SVC_TRACE
      trace[4] = static_cast<unsigned long long>(wall_clock64());
      if (part == svc_active_parts(seq) - 1)
        for (int i = 0; i < 5; ++i) __hip_atomic_store(&slot->trace[i], trace[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
      sys_store(&slot->done[part], seq);
      if (part == 0)
        __hip_atomic_fetch_max(&st->last_active, static_cast<unsigned long long>(wall_clock64()), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // req and bcast are rewritten next round
  }
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(&st->exited, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1 == gridDim.x)
    sys_store(&ctl->exited_epoch, epoch);  // the last workgroup out
}

}  // namespace

hipError_t launch_service(SvcCtl* d_ctl, SvcDev* d_state, unsigned long long epoch, unsigned long long idle_ticks,
                          unsigned long long life_ticks, hipStream_t s) {
  (void)hipGetLastError();
  hipLaunchKernelGGL(service_kernel, dim3(kSvcSlots * kSvcParts), dim3(kSvcThreads), kSvcLds + 128, s, d_ctl, d_state,
                     epoch, idle_ticks, life_ticks);
  return hipGetLastError();
}

hipError_t launch_encode_ptr(const PtrRows& rows, const EncodeGeom& g, const void* d_tbl, hipStream_t s,
                             unsigned long long* ticket) {
  return launch_encode(rows, g, d_tbl, s, ticket);
}
hipError_t launch_encode_slab(const SlabRows& slab, const EncodeGeom& g, const void* d_tbl, hipStream_t s,
                              unsigned long long* ticket) {
  return launch_encode(slab, g, d_tbl, s, ticket);
}
hipError_t launch_encode_tab(const PtrTabRows& rows, const EncodeGeom& g, const void* d_tbl, hipStream_t s,
                             unsigned long long* ticket) {
  return launch_encode(rows, g, d_tbl, s, ticket);
}
bool encode_uses_ticket(uint64_t tiles, int k) {
  return ECW_ENC_ASM && k >= 2 && ECW_TICKET_MIN_TILES > 0 && tiles >= ECW_TICKET_MIN_TILES;
}
hipError_t launch_xor_ptr(const XorPtr& p, const XorGeom& g, hipStream_t s) { return launch_xor(p, g, s); }
hipError_t launch_xor_slab(const XorSlab& p, const XorGeom& g, hipStream_t s) { return launch_xor(p, g, s); }
hipError_t launch_xor_split(const XorSplit& p, const XorGeom& g, hipStream_t s) { return launch_xor(p, g, s); }
hipError_t launch_xor_tab(const XorTab& p, const XorGeom& g, hipStream_t s) { return launch_xor(p, g, s); }

hipError_t launch_fill_random(uint8_t* dst, uint64_t bstride, uint64_t sstride, int stripes, int nblocks,
                              uint64_t len, uint64_t piece, uint64_t pstride, uint64_t offset, uint64_t seed,
                              int s0, int b0, hipStream_t s) {
  if (stripes <= 0 || nblocks <= 0 || len == 0) return hipSuccess;
  if (piece == 0 || offset % 16 || (piece < len && piece % 16)) return hipErrorInvalidValue;
  const uint64_t npair = (len + 15) / 16;
  uint64_t gx = (npair + kBlock - 1) / kBlock;
  if (gx > 1024) gx = 1024;
  const int rows = stripes * nblocks;
  const dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(rows < 65535 ? rows : 65535));
  (void)hipGetLastError();  // report this launch's error, not an earlier one
  hipLaunchKernelGGL(fill_kernel, grid, dim3(kBlock), 0, s, dst, bstride, sstride, stripes, nblocks, len,
                     piece, pstride, offset, seed, s0, b0);
  return launched("fill_kernel", grid, 0, s);
}

int stripes_per_launch(uint64_t tiles) {
  // stripes * tiles < kMaxTilesPerLaunch, what the launchers' range checks accept
  const uint64_t n = (kMaxTilesPerLaunch - 1) / (tiles ? tiles : 1);
  return n > 0x7FFFFFFFull ? 0x7FFFFFFF : n < 1 ? 1 : static_cast<int>(n);  // (a 2^31-tile stripe: rejected by the range check)
}

int device_cu_count(int device) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
  return n;
}

}  // namespace ecw
