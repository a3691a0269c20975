// HIP kernels for gfx950 (MI355X, CDNA4): the XOR reduce dst = src_0 ^ ...
// ^ src_{n-1} -- ECWide-C decodeData / partialDecodeData (NativeCodec.cc:
// 221-282: ec_encode_data with all-ones tables), xorIntemediate (:284-323)
// and the combined-locality single-block repair (the r surviving members of
// the lost block's group, ClMetadataManager.java:137-257), on every block
// layout: explicit pointers, the block / split / tiled slabs and device
// pointer tables. Byte-wise XOR: HBM-bound streaming, no MFMA.
//
// Kernels and launchers as templates over the source addressing (Args); the
// exported launchers are instantiated in two translation units,
// ecw_xor_ptr.hip (XorPtr, XorTab) and ecw_xor_slab.hip (XorSlab, XorSplit),
// which compile side by side (one straight-line kernel per source count,
// skew and addressing: 384 kernels in all).
#pragma once

#include "ecw_device.hpp"

namespace ecw {
namespace {

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
template <class T>
__device__ __forceinline__ T* uniform_table_entry(T* const* table, uint64_t index) {
  const uint64_t a = reinterpret_cast<uint64_t>(table + index);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  const __attribute__((address_space(4))) uint64_t* c =
      reinterpret_cast<const __attribute__((address_space(4))) uint64_t*>((static_cast<uint64_t>(hi) << 32) | lo);
  return reinterpret_cast<T*>(*c);
}
__device__ __forceinline__ const uint8_t* xsrc(const XorTab& a, int s, int i) {
  return uniform_table_entry(a.src, static_cast<uint64_t>(s) * a.n + i);
}
__device__ __forceinline__ uint8_t* xdst(const XorTab& a, int s) { return uniform_table_entry(a.dst, static_cast<uint64_t>(s)); }
__device__ __forceinline__ uint8_t* xdst(const XorPtr& a, int) { return a.dst; }
__device__ __forceinline__ uint8_t* xdst(const XorSlab& a, int s) { return a.out + s * a.ostride; }
__device__ __forceinline__ uint8_t* xdst(const XorSplit& a, int s) { return a.out + s * a.ostride; }

// Pairs of consecutive units of a split slab taken as one unit of 4 tiles, so
// that K = 4 can skew over the tiled slab's 2-tile (8 KiB) pieces: tile q of
// pair p is tile q % 2 of unit 2p + q / 2 (launch_xor_range). The units of a
// source are sstride (data) or psstride (parity) apart, the outputs ostride.
struct XorSplitPair {
  XorSplit a;
};
template <class Args>
struct is_pair : std::false_type {};
template <>
struct is_pair<XorSplitPair> : std::true_type {};
__device__ __forceinline__ const uint8_t* xsrc(const XorSplitPair& p, int s, int i) { return xsrc(p.a, 2 * s, i); }
__device__ __forceinline__ uint8_t* xdst(const XorSplitPair& p, int s) { return xdst(p.a, 2 * s); }
// byte offset of tile q of a pair from its first tile, in source i / the output
__device__ __forceinline__ uint64_t pair_src_off(const XorSplitPair& p, int i, int q) {
  return static_cast<uint64_t>(q >> 1) * (i < p.a.ndata ? p.a.sstride : p.a.psstride) +
         static_cast<uint64_t>(q & 1) * kTileBytes;
}
__device__ __forceinline__ uint64_t pair_dst_off(const XorSplitPair& p, int q) {
  return static_cast<uint64_t>(q >> 1) * p.a.ostride + static_cast<uint64_t>(q & 1) * kTileBytes;
}

// Loads and stores of the XOR reduce are nontemporal (+4-6 % at 4-64 MiB
// blocks; a straight stream, every byte touched once).
constexpr bool kXorNt = true;

template <int P, bool TAIL, class Args>
__device__ __forceinline__ void xor_tile(const Args& a, const XorGeom& g, int s, uint32_t col) {
  const uint32_t len = static_cast<uint32_t>(g.len);
  if (TAIL && col >= len) return;
  const int n = g.n;
  uint4 ring[P];
#pragma unroll
  for (int p = 0; p < P; ++p) ring[p] = ld16<TAIL, kXorNt>(xsrc(a, s, p < n ? p : n - 1), col, len);
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int i0 = 0; i0 < n; i0 += P) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int i = i0 + p;
      if (i < n) acc = xor4(acc, ring[p]);
      ring[p] = ld16<TAIL, kXorNt>(xsrc(a, s, i + P < n ? i + P : n - 1), col, len);
    }
  }
  st16<TAIL, kXorNt>(xdst(a, s), col, len, acc);
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

// Source count known at compile time (n <= kXorFixedMax, every CL repair
// of a group of up to that many blocks): straight-line code, no loop. The
// runtime-n ring above compiles to a loop whose head waits vmcnt(0) (LLVM's
// waitcnt pass merges the prologue's and the back-edge's load orders), i.e.
// every wave drains its loads every P rows; straight-line code gets exact
// counted waits, and the source indices come in as one scalar batch.
// Loads are issued with at most W = kXorWindow in flight per wave (W >= N:
// all at once).
// Write window of the XOR reduce (XorSched::wwidth > 0): the output store
// waits until the chip-wide 100 MHz constant clock is in the first `wwidth`
// ticks of every `wmask + 1`, as the encode's asm tile does
// (ECW_WRITE_WINDOW in ecw_encode_asm.hpp); at most 16384 polls.
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
  constexpr int W = kXorWindow > 0 && kXorWindow < T ? kXorWindow : T;
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
    if constexpr (is_pair<Args>::value)
      v[t] = ld16<TAIL, kXorNt>(sp[t % N] + pair_src_off(a, t % N, (t / N + t % N) % K), col, len);
    else
      v[t] = ld16<TAIL, kXorNt>(sp[t % N], col + ((t / N + t % N) % K) * kTileBytes, len);
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
  for (int q = 0; q < K; ++q) {
    if constexpr (is_pair<Args>::value)
      st16<TAIL, kXorNt>(d + pair_dst_off(a, q), col, len, acc[q]);
    else
      st16<TAIL, kXorNt>(d, col + q * kTileBytes, len, acc[q]);
  }
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

// The same sources from stripe s0 on (a batch split into several launches).
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
inline XorSplitPair offset_stripes(const XorSplitPair& p, int s0) { return XorSplitPair{offset_stripes(p.a, 2 * s0)}; }
inline XorTab offset_stripes(const XorTab& a, int s0) {
  XorTab o = a;
  o.src += static_cast<uint64_t>(s0) * a.n;
  o.dst += s0;
  return o;
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

// Schedule of the straight-line XOR kernel: tiles per workgroup (skew K, one
// of kXorSkews), group order, write window. The process's schedule
// (ecw_set_schedule: xor_skew / xor_order / xor_window_*) overrides each part
// it sets; the window, when not set, follows the default's rule below.
struct XorChoice {
  int skew;
  uint32_t order, log2p, wwidth, remap;
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
//  * column-major group order and K = 8 gained less than K = 4 for whole blocks;
//  * the tiled slab's 16 KiB units (k <= 32, slab.default_chunk) are one whole
//    group of K = 4 tiles and take the same schedule: CL(32, 8, 2) 6240 -> 6379,
//    CL(32, 11, 3) 6259 -> 6537 GB/s (profiles/r04_k32r_cfg1/0.log);
//  * round 5: the tiled slab's 8 KiB units (k = 128, the bench's headline) are
//    one whole group of K = 2 tiles and take K = 2 + the window, chosen by the
//    WORST of five tiled slabs allocated side by side in one process (where an
//    allocation lands sets +-3-6 %; tools/repair_placement.py, two processes,
//    profiles/r05_placement_1/2.log): worst slab 6145 / 6189 GB/s with round 4's
//    K = 1 and no window, 6467 / 6466 with K = 2 + window (median 6552 / 6592,
//    best 6594 / 6611 against 6637 / 6628), 0.983 / 0.987 of the split slab's
//    own default in the same process. K = 4 + window was the worst (6090 / 6167:
//    a 2-tile unit is a ragged group of 4, reduced tile by tile), K = 2 without
//    the window no better than K = 1, a 2^10 / 32 window between (6320 / 6340);
//  * ... and, later in round 5, K = 4 over PAIRS of those units (XorSplitPair:
//    the split / tiled slab's addressing, an even unit count) + the window beat
//    K = 2 + window on the worst slab in both processes: 6541 / 6373 against
//    6426 / 6318 GB/s (median 6578 / 6518 against 6487 / 6473; 0.998 / 0.995 of
//    the split slab's default; profiles/r05f_pair_placement_1/2.log). Units that
//    cannot be paired (odd count, pointer tables) keep K = 2 + window;
//  * the XOR keeps the dispatch tile order (the per-XCD order: -0.4..-5 %,
//    profiles/r04_remap_*.log).
// `pairable`: the launch can take pairs of 2-tile units (launch_xor_range).
inline XorChoice xor_choice(const XorGeom& g, bool pairable) {
  constexpr uint64_t group = static_cast<uint64_t>(kXorSkewWhole) * kTileBytes;
  const uint64_t tiles = static_cast<uint64_t>(g.stripes) * g.tiles;
  const bool whole = g.len >= 65536 || (g.len >= group && g.len % group == 0);
  // units of exactly two tiles (the tiled slab's 8 KiB pieces), wide enough
  // for the window
  const bool pair = !whole && g.len == 2 * kTileBytes && g.n >= 8 && tiles >= 8192;
  const Schedule sc = current_schedule();
  XorChoice c{whole ? kXorSkewWhole : pair ? (pairable ? 4 : 2) : 1, 0, 11, 0, 0};
  if ((whole || pair) && g.n >= 8 && tiles >= 8192) c.wwidth = 64;
  if (sc.xor_skew > 0) c.skew = sc.xor_skew;
  if (sc.xor_order >= 0) c.order = static_cast<uint32_t>(sc.xor_order);
  if (sc.xor_width >= 0) {
    c.wwidth = static_cast<uint32_t>(sc.xor_width);
    if (sc.xor_log2p >= 0) c.log2p = static_cast<uint32_t>(sc.xor_log2p);
  }
  if (sc.xcd_remap >= 0) c.remap = static_cast<uint32_t>(sc.xcd_remap);
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
  sc.remap = c.remap;
  sc.wmask = (1u << c.log2p) - 1;
  sc.wwidth = c.wwidth;
  const dim3 grid(grid_for(total, kGridPerCuXor));
  return launch_xor_fixed<kXorFixedMax, K>(a, g, sc, grid, s);
}

template <class Args>
hipError_t launch_xor_range(const Args& a, const XorGeom& g, hipStream_t s) {
  const uint64_t total = static_cast<uint64_t>(g.stripes) * g.tiles;
  if (total == 0) return hipSuccess;
  if (g.stripes < 0 || total >= kMaxTilesPerLaunch) return hipErrorInvalidValue;  // 32-bit tile numbering
  // ring depth <= n: the ring refills past the last row re-read row n-1, so a
  // depth-8 ring over 1-2 sources would load every byte up to 8 times
  const dim3 grid(grid_for(total, kGridPerCuXor)), block(kBlock);
  const FastDiv per = make_fastdiv(static_cast<uint32_t>(g.tiles));
  if (g.n <= kXorFixedMax) {
    const bool pairable = std::is_same<Args, XorSplit>::value && g.stripes % 2 == 0;
    const XorChoice c = xor_choice(g, pairable);
    static_assert(sizeof(kXorSkews) / sizeof(kXorSkews[0]) == 3 && kXorSkews[1] == 2 && kXorSkews[2] == 4,
                  "the skews instantiated here are the ones ecw_set_schedule accepts");
    static_assert(kXorSkewWhole == 4 || kXorSkewWhole == 2 || kXorSkewWhole == 1, "a built skew");
    if constexpr (std::is_same<Args, XorSplit>::value) {
      // K = 4 over 2-tile units (the tiled slab's 8 KiB pieces): pairs of units
      if (c.skew == 4 && g.len == 2 * kTileBytes && pairable) {
        const XorGeom gp{4 * kTileBytes, 4, g.stripes / 2, g.n};
        return launch_xor_skew<4>(XorSplitPair{a}, gp, c, s);
      }
    }
    if (c.skew == 4) return launch_xor_skew<4>(a, g, c, s);
    if (c.skew == 2) return launch_xor_skew<2>(a, g, c, s);
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

}  // namespace
}  // namespace ecw
