// Compile-time tunables of the kernels, in one place: each is a measured
// choice (the comment says where it was measured; DESIGN.md §4 has the
// numbers). A tuning build may override any of them with -D (tools/variants.py
// builds such variants under build/variants/ for interleaved A/Bs); the
// product build takes these defaults. Run-time launch choices (tile order,
// write windows, XOR skew) are not here: they are the launchers' per-layout
// defaults, overridable per process with ecw_set_schedule (ecwide.h).
#pragma once

#include <cstdint>

// ---- encode ------------------------------------------------------------------
#ifndef ECW_PREFETCH_ENC
#define ECW_PREFETCH_ENC 2  // compiler-scheduled tile (k = 1, ragged tails): register ring depth
#endif
#ifndef ECW_GRID_PER_CU
#define ECW_GRID_PER_CU 256  // encode: workgroups per CU before tiles are grid-strided (256 vs 64: +2.7 %)
#endif
#ifndef ECW_ENC_MIN_WAVES
#define ECW_ENC_MIN_WAVES 6  // compiler-scheduled tile, __launch_bounds__ min waves per SIMD: 80 VGPRs (+1-4 %)
#endif
#ifndef ECW_ENC_MIN_WAVES_NW2
#define ECW_ENC_MIN_WAVES_NW2 4  // 5-8 rows: 128 VGPRs (at 80 the 32 accumulators spill inside the row loop)
#endif
#ifndef ECW_ENC_MIN_WAVES_NW4
#define ECW_ENC_MIN_WAVES_NW4 2  // 9-16 rows: 256 VGPRs for the 64 packed accumulators
#endif
#ifndef ECW_ASM_MIN_WAVES
#define ECW_ASM_MIN_WAVES 6  // asm tile, <= 4 rows: 80 VGPRs (the parked tile uses 78)
#endif
#ifndef ECW_ASM_MIN_WAVES_NW2
#define ECW_ASM_MIN_WAVES_NW2 4  // 5-8-row asm tile: 128 VGPRs (it uses 110)
#endif
#ifndef ECW_ASM_MIN_WAVES_NW4
#define ECW_ASM_MIN_WAVES_NW4 3  // 9-16-row asm tile: 168 VGPRs (it uses 142)
#endif
#ifndef ECW_ASM_TPB4
// 9-16 rows: workgroups of 2 tiles (512 threads) share one copy of the 64 KiB
// (k = 128) tables, so the LDS holds tables for 16 waves per CU instead of 8
// (+3-5 %; +32 % at k = 200, profiles/r03_tpb_ab.log)
#define ECW_ASM_TPB4 2
#endif
#ifndef ECW_ASM_RING3
// <= 4-row asm tile: when it keeps 3 rows in flight per wave instead of 2 (slot C
// in v[36:39], no register cost). 0 never, 1 with the write window (the
// whole-block layouts at k >= 64: +0.8..1.8 % encode), 2 always (tiled slab
// -0.5..+0.5 % at k = 128, -1.2..-2.1 % at k = 32; profiles/r05h_*, r05i_*)
#define ECW_ASM_RING3 1
#endif
#ifndef ECW_ASM_RING3_NW2
// 5-8-row asm tile: three rows in flight per wave (slot C in v[36:39], same 110 /
// 90 VGPRs): +1.2..2.3 % over block slabs at k = 32 / 128, +3.6 % over pointer
// tables (profiles/r05u_nw2_ring3_*); 0 = the two-slot ring
#define ECW_ASM_RING3_NW2 1
#endif
#ifndef ECW_ASM_RING3_NW4
// 9-16-row asm tile: three rows in flight per wave (slot C in v[36:39], same 142 /
// 123 VGPRs): +0.3..1.2 % at k = 64 / 128, +4.4 % at k = 32 (profiles/r05v_ring3_*)
#define ECW_ASM_RING3_NW4 1
#endif
#ifndef ECW_ASM_TPB1
#define ECW_ASM_TPB1 1  // <= 4 rows (2: tiled +-0, block slab -1.2 %, profiles/r03_tpb1_ab.log; under the window tiled -0.5..-1.6 %, r05tp_*; pointer tables / block slab -0.6..-1.5 %, r05pt_*)
#endif
// The slab is encoded in launch windows of one grid's worth of tiles (256 CUs x
// ECW_GRID_PER_CU), one tile per workgroup (+3.5 % encode at the 272 GiB slab,
// +0.3..1.5 % at the bench shape, profiles/r01_encode_launch_window_ab.log).
// > 0 sets another window, < 0 launches the slab at once.
#ifndef ECW_COHORT_TILES
#define ECW_COHORT_TILES 0
#endif
// Slabs of at least this many tiles (4 windows: 1 GiB of column per data row,
// e.g. the 272 GiB HBM-filling batch) run as ONE launch whose workgroups take
// tiles in order from a ticket counter: +2.9 % encode over the windows at 240 x
// 8 MiB stripes, -1.4..-9 % on smaller slabs (profiles/r01_encode_ticket_ab.log).
// 0 disables.
#ifndef ECW_TICKET_MIN_TILES
#define ECW_TICKET_MIN_TILES (4ull * 256 * ECW_GRID_PER_CU)
#endif

// ---- XOR reduce ----------------------------------------------------------------
#ifndef ECW_PREFETCH_XOR
#define ECW_PREFETCH_XOR 4  // ring kernel (> 32 sources): depth 4 vs 8 +2.6 % tiled (tools/layout_ab.py)
#endif
#ifndef ECW_XOR_FIXED_MAX
#define ECW_XOR_FIXED_MAX 32  // straight-line kernel per source count up to this many sources
#endif
#ifndef ECW_GRID_PER_CU_XOR
#define ECW_GRID_PER_CU_XOR 2048  // one workgroup per tile up to 512 Ki tiles (+8.6 % at the HBM-filling batch vs 512)
#endif
#ifndef ECW_XOR_WINDOW
#define ECW_XOR_WINDOW 8  // straight-line kernel: loads in flight per wave (4..27 within +-0.5 % in round 4; round 5 at r = 8 / 11 / 27: 4 -0.1..-1.1 %, 16 -0.9..-3.9 %, profiles/r05xw_*)
#endif
#ifndef ECW_XOR_SKEW_K
#define ECW_XOR_SKEW_K 4  // diagonal skew of whole blocks; must be one of kXorSkews
#endif

// ---- host-memory pipeline -------------------------------------------------------
#ifndef ECW_HOST_IN_STREAMS
#define ECW_HOST_IN_STREAMS 2  // host -> HBM copy streams of the pipelined host calls (1 or 2)
#endif

// ---- request service -------------------------------------------------------------
#ifndef ECW_SVC_COLD_SLEEPS
#define ECW_SVC_COLD_SLEEPS 2  // s_sleep 127 (~3.4 us each) after every poll of a cold slot
#endif

namespace ecw {
constexpr int kPrefetchEnc = ECW_PREFETCH_ENC;
constexpr int kPrefetchEncAsmTail = 2;  // the asm launches' ragged-tail kernel
constexpr int kAsmRing3 = ECW_ASM_RING3;
static_assert(kAsmRing3 >= 0 && kAsmRing3 <= 2, "ECW_ASM_RING3: 0, 1 or 2");
constexpr int kAsmRing3Nw2 = ECW_ASM_RING3_NW2;
constexpr int kAsmRing3Nw4 = ECW_ASM_RING3_NW4;
constexpr uint64_t kGridPerCu = ECW_GRID_PER_CU;
constexpr uint64_t kGridPerCuXor = ECW_GRID_PER_CU_XOR;
constexpr int kPrefetchXor = ECW_PREFETCH_XOR;
constexpr int kXorFixedMax = ECW_XOR_FIXED_MAX;
constexpr int kXorWindow = ECW_XOR_WINDOW;
constexpr int kXorSkewWhole = ECW_XOR_SKEW_K;
constexpr int kMaxParkedLocals = 5;  // v[58:77] of the asm tile: <= 5 local parities stored at the end of the tile
constexpr int64_t kCohortTiles = ECW_COHORT_TILES;
constexpr unsigned long long kTicketMinTiles = ECW_TICKET_MIN_TILES;
constexpr int kSvcColdSleeps = ECW_SVC_COLD_SLEEPS;
constexpr int kHostInStreams = ECW_HOST_IN_STREAMS;
static_assert(kHostInStreams == 1 || kHostInStreams == 2, "ECW_HOST_IN_STREAMS: 1 or 2");
}  // namespace ecw
