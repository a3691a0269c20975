// HIP kernels for gfx950 (MI355X, CDNA4): wide-stripe GF(2^8) encode and the
// synthetic fill (the XOR reduce is ecw_xor.hpp, the request service
// ecw_service.hip).
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
#include "ecw_device.hpp"
#include "ecw_encode_asm.hpp"

namespace ecw {
namespace {

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
        gf_row<NW>(ring[p], acc, lds_base + static_cast<uint32_t>(j) * (128u * NW));
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

// __launch_bounds__ min waves per SIMD: the VGPR budget of each row count
// (ecw_tuning.hpp)
template <int NW, int P, int LOCAL, class Rows>
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

// Encode with <= 4 global rows (one u32 table entry per nibble) and k >= 2:
// full tiles through the hand-scheduled asm tile, the ragged last tile of a
// block through encode_tile<..., TAIL>. PARK (<= 5 groups): local parities
// are stored at the end of each tile (ecw_encode_asm.hpp). Pointer mode
// hands the asm the addresses of the pointer tables in the kernel
// arguments: `rows` is the first argument, so it sits at offset 0 of the
// kernarg segment (taking the address of the by-value argument itself
// would make the compiler copy all 3 KiB of it to scratch).
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
  stage_tables<kBlock * TPB>(lds, tbl, n16);
  __syncthreads();
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

template <class Rows, int NW>
hipError_t launch_encode_asm(const Rows& rows, const EncodeGeom& g, const uint4* tbl, dim3 grid, hipStream_t s) {
  const size_t lds = static_cast<size_t>(g.k) * 128 * NW + 16;  // + the ticket slot
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
// kGridPerCu), one tile per workgroup, instead of one grid-strided launch: a
// grid-strided workgroup jumps a whole grid ahead when it finishes, spreading
// the in-flight tiles over several distant regions; slabs of at least
// kTicketMinTiles tiles run as ONE ticket-ordered launch (ecw_tuning.hpp).

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
// Units of 8-64 KiB (the tiled slab's 8 KiB pieces at k = 128) take it too since
// round 5, with a 32-tick width: the window (and the three-slot ring it brings,
// ecw_encode_asm.hpp) narrows the encode's placement band from 5994-6391 to
// 6229-6304 GB/s over five slabs side by side, worst slab +0.2..4.5 % in six
// processes, median -1.4..+1.7 % (profiles/r05k_*, r05l_*, r05m_*: judged by the
// worst slab, as the repair's schedule).
// ecw_set_schedule (enc_window_*) overrides the choice for the process.
// Stripes of 24-63 data blocks take it too since round 5, at half the period
// (2^10 ticks): their tiles read a quarter of k = 128's rows, and at 2^11 the
// generations cost more than the window saves (the -4 / -8 % above), while at
// 2^10 the encode gains +4..6 % at k = 32 on the tiled, split and block slabs
// (worst slab and median) and +4.5 % over pointer tables, +3.6 % at k = 24,
// +1.5..2.3 % at k = 48; k = 16 loses 1 % (profiles/r05p_*, r05q_*, r05r_*);
// 2^9 gains nothing anywhere.
inline bool window_shape(const EncodeGeom& g) {
  return g.k >= 24 && g.nrows <= 4 && g.len >= 8192 && static_cast<uint64_t>(g.stripes) * g.tiles >= 8192;
}
inline uint32_t window_log2p(const EncodeGeom& g) { return g.k >= 64 ? 11u : 10u; }
inline uint32_t window_width(const EncodeGeom& g) { return g.len >= 65536 ? 64u : 32u; }
// Slabs of whole blocks: the block slab (parity rows after each stripe's data
// rows) since round 2; the split slab (parities in a region of their own)
// since round 4, interleaved in one process: 5557 -> 6350 and 5846 -> 6285 GB/s
// (profiles/r04b_repair_ab_*.log; round 2 had measured +5.0 / -2.4 % on two
// boxes); the tiled slab's 8 KiB units since round 5 (above).
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

// The launch's write window and tile order: the per-layout defaults above,
// or the process's schedule where it sets them (one copy per launch).
template <class Rows>
void set_schedule(const Rows& rows, EncodeGeom& g) {
  const Schedule sc = current_schedule();
  const bool on = sc.enc_width >= 0 ? sc.enc_width > 0 : window_auto(rows, g);
  const uint32_t log2p = sc.enc_log2p >= 0 ? static_cast<uint32_t>(sc.enc_log2p) : window_log2p(g);
  g.wmask = (1u << log2p) - 1;
  g.wwidth = on ? (sc.enc_width > 0 ? static_cast<uint32_t>(sc.enc_width) : window_width(g)) : 0u;
  g.remap = sc.xcd_remap >= 0 ? static_cast<uint32_t>(sc.xcd_remap) : remap_auto(rows);
}

// One launch range: stripes [0, g0.stripes) of `rows`, fewer than
// kMaxTilesPerLaunch tiles. The asm kernel covers the full column tiles (in
// launch windows, or in one ticket-ordered launch), encode_tail_kernel the
// ragged last tile of every block; k = 1 takes the compiler-scheduled kernel,
// which handles both.
template <class Rows>
hipError_t launch_encode_range(const Rows& rows, const EncodeGeom& g0, const uint4* tbl, hipStream_t s,
                               unsigned long long* ticket) {
  const bool asm_tile = g0.k >= 2;
  const uint64_t full = g0.len / kTileBytes;
  const uint64_t per = asm_tile ? full : g0.tiles;  // tiles per stripe in the launch's numbering
  const uint64_t total = static_cast<uint64_t>(g0.stripes) * per;
  // what the kernels' 32-bit tile numbering assumes (the grid never covers a
  // tile past the slab)
  if (g0.stripes < 0 || total >= kMaxTilesPerLaunch || per > 0xFFFFFFFFull) return hipErrorInvalidValue;
  EncodeGeom gw = g0;
  set_schedule(rows, gw);
  gw.per = make_fastdiv(static_cast<uint32_t>(per ? per : 1));
  gw.ticket = nullptr;
  const uint64_t win = kCohortTiles > 0    ? static_cast<uint64_t>(kCohortTiles)
                       : kCohortTiles == 0 ? 256ull * kGridPerCu
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

}  // namespace

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
  return k >= 2 && kTicketMinTiles > 0 && tiles >= kTicketMinTiles;
}
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
