// Internal interface between the host codec (ecw_codec.cpp) and the HIP
// kernels (ecw_kernels.hip: encode + fill, ecw_xor.hpp: XOR reduce,
// ecw_service.hip: request service). Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace ecw {

constexpr int kMaxSrc = 256;      // k + m <= 256 for a GF(2^8) Cauchy code
constexpr int kMaxPassRows = 16;  // global rows per encode pass (16-byte packed entries above 8)
constexpr int kMaxSvcRows = 8;    // global rows the resident request service encodes
constexpr int kMaxPtrLocals = 120;  // local outputs per pointer-mode encode pass
#ifndef ECW_BLOCK
#define ECW_BLOCK 256
#endif
constexpr int kBlock = ECW_BLOCK; // threads per workgroup
constexpr int kLaneBytes = 16;    // bytes per lane per row (dwordx4)
constexpr int kTileBytes = kBlock * kLaneBytes;

// Local-parity handling inside an encode pass.
enum LocalMode : int { kLocalNone = 0, kLocalXor = 1, kLocalZero = 2 };

// Addressing of rows: either explicit pointers (one stripe; pointers live
// in the kernel arguments) or a strided slab of `stripes` stripes.
struct PtrRows {
  const uint8_t* src[kMaxSrc];
  uint8_t* dst[kMaxPassRows + kMaxPtrLocals];  // [global rows of the pass..., locals...]
};

struct SlabRows {
  const uint8_t* base;   // data block 0 of stripe 0
  uint64_t bstride;      // bytes between data blocks of a stripe
  uint64_t sstride;      // bytes between stripes (data)
  uint8_t* pbase;        // parity block 0 (G0, then G1.., L0..) of stripe 0
  uint64_t pbstride;     // bytes between parity blocks of a stripe
  uint64_t psstride;     // bytes between stripes (parities)
};
// the slab layout proper: parities follow the k data blocks
inline SlabRows slab_rows(const uint8_t* base, uint64_t bstride, uint64_t sstride, int k) {
  return SlabRows{base, bstride, sstride, const_cast<uint8_t*>(base) + static_cast<uint64_t>(k) * bstride,
                  bstride, sstride};
}

// Pointer tables in device memory for a batch of stripes (ecw_encode_ptrs_dev):
// data block j of stripe s at src[s*k + j], output o of stripe s at
// dst[s*np + o] (o in [G_0..G_{m-1}, L_0..L_{g-1}] order).
struct PtrTabRows {
  const uint8_t* const* src;
  uint8_t* const* dst;
  int np;
};

// u32 division by a divisor fixed for a launch (Granlund-Montgomery, the
// round-down-and-fix-up form): q = fast_div(n, f) == n / f.d for every n < 2^32.
// The kernels map a tile index to (stripe, column tile) with it in a handful of
// scalar instructions; a 64-bit division by a kernel argument compiled to ~100
// instructions per tile whose hoisted reciprocals the encode kernel had to
// spill to scratch (and reload, behind vmcnt(0), at every tile).
struct FastDiv {
  uint32_t d, m, s1, s2;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while (l < 32 && (uint64_t(1) << l) < d) ++l;  // l = ceil(log2 d)
  FastDiv f;
  f.d = d;
  f.m = static_cast<uint32_t>(((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1);
  f.s1 = l < 1 ? l : 1;
  f.s2 = l > 1 ? l - 1 : 0;
  return f;
}
__host__ __device__ inline uint32_t fast_div(uint32_t n, const FastDiv& f) {
  const uint32_t t = static_cast<uint32_t>((static_cast<uint64_t>(n) * f.m) >> 32);
  return (t + ((n - t) >> f.s1)) >> f.s2;
}

struct EncodeGeom {
  uint64_t len;          // bytes per block
  uint64_t tiles;        // column tiles per stripe = ceil(len / kTileBytes)
  int stripes;
  int k, r, groups;      // data rows, group size, local groups
  int m;                 // total global rows (slab output indexing)
  int row0, nrows;       // global rows of this pass [row0, row0 + nrows)
  int local_mode;        // LocalMode
  // set by the launcher:
  uint32_t tile_begin;   // this launch covers tiles [tile_begin, tile_end) of its numbering:
  uint32_t tile_end;     //   tile = stripe * per.d + column tile (the asm kernel numbers full tiles only)
  FastDiv per;           // column tiles per stripe in that numbering
  unsigned long long* ticket;  // non-null: workgroups take tiles in order from this counter (zeroed before the launch)
  uint32_t wmask, wwidth;      // write window (asm tile): store when (clock & wmask) < wwidth; 0 = off
  uint32_t remap;              // 1: per-XCD contiguous tile order (wg_slot)
};

// Launchers return hipSuccess or the launch error (an earlier, unrelated HIP
// error of the calling thread is cleared first, not reported). The encode
// launchers run a slab of >= kTicketMinTiles tiles as one ticket-ordered
// launch when `ticket` is given (an 8-byte device counter the caller has
// zeroed on stream `s` and keeps for this launch alone), else in launch windows.
hipError_t launch_encode_ptr(const PtrRows& rows, const EncodeGeom& g, const void* d_tbl,
                             hipStream_t s, unsigned long long* ticket);
hipError_t launch_encode_slab(const SlabRows& slab, const EncodeGeom& g, const void* d_tbl,
                              hipStream_t s, unsigned long long* ticket);
hipError_t launch_encode_tab(const PtrTabRows& rows, const EncodeGeom& g, const void* d_tbl,
                             hipStream_t s, unsigned long long* ticket);
// true when an encode of `tiles` column tiles at k data rows would use a ticket counter
bool encode_uses_ticket(uint64_t tiles, int k);

struct XorPtr {
  const uint8_t* src[kMaxSrc];
  uint8_t* dst;
};
struct XorSlab {
  const uint8_t* base;           // block j of stripe s at base + s*sstride + j*bstride
  uint64_t bstride, sstride;
  uint8_t* out;
  uint64_t ostride;
  int idx[kMaxSrc];              // source block indices within a stripe
};
// Split layout (ecw_*_batch_split_dev): sources [0, ndata) are data blocks,
// the rest parity blocks, each region with its own strides.
struct XorSplit {
  const uint8_t* base;
  uint64_t bstride, sstride;
  const uint8_t* pbase;
  uint64_t pbstride, psstride;
  uint8_t* out;
  uint64_t ostride;
  int ndata;
  int idx[kMaxSrc];              // block index of source i within its region
};
// Device pointer tables (ecw_xor_reduce_ptrs_dev): source i of stripe s at
// src[s*n + i], its output at dst[s].
struct XorTab {
  const uint8_t* const* src;
  uint8_t* const* dst;
  int n;
};
struct XorGeom {
  uint64_t len, tiles;
  int stripes, n;
};
// Set by the XOR launcher (ecw_xor.hpp launch_xor_range): the kernel's
// unit is a group of K column tiles (K a template argument of the kernel).
struct XorSched {
  FastDiv per;            // column groups per stripe
  FastDiv ns;             // stripes (order 1)
  uint32_t order;         // 0: groups numbered stripe-major, 1: column-major
  uint32_t wmask, wwidth; // write window: store when (clock & wmask) < wwidth; 0 = off
  uint32_t remap;         // 1: per-XCD contiguous group order (wg_slot)
};
hipError_t launch_xor_ptr(const XorPtr& p, const XorGeom& g, hipStream_t s);
hipError_t launch_xor_slab(const XorSlab& p, const XorGeom& g, hipStream_t s);
hipError_t launch_xor_split(const XorSplit& p, const XorGeom& g, hipStream_t s);
hipError_t launch_xor_tab(const XorTab& p, const XorGeom& g, hipStream_t s);

hipError_t launch_fill_random(uint8_t* dst, uint64_t bstride, uint64_t sstride, int stripes,
                              int nblocks, uint64_t len, uint64_t piece, uint64_t pstride,
                              uint64_t offset, uint64_t seed, int s0, int b0, hipStream_t s);

int device_cu_count(int device);

// Process-wide launch schedule (ecwide.h ecw_schedule; -1 = the launcher's
// own choice). Seeded once from ECW_XOR_SCHED / ECW_WRITE_WINDOW /
// ECW_XCD_REMAP at first use, then changed only by ecw_set_schedule; the
// launchers take one copy per launch (ecw_codec.cpp), never the environment.
struct Schedule {
  int xor_skew, xor_order, xor_log2p, xor_width;
  int enc_log2p, enc_width;
  int xcd_remap;
};
Schedule current_schedule();
// XOR skews compiled into the library (xor_kernel_fixed<N, K>)
constexpr int kXorSkews[] = {1, 2, 4};

// Stripes one launch may cover when each has `tiles` column tiles: the
// kernels number tiles in 32 bits, so a launch covers fewer than 2^31 tiles
// and a larger batch goes in several launches over consecutive stripes.
int stripes_per_launch(uint64_t tiles);

// ---- small-stripe request service (ecw_codec.cpp: svc::) -------------------
// A resident kernel serves synchronous small encodes (ECWide-H encodes one
// 4 KiB chunk per ec_encode_data call, ECWide-H/proxy/encode.cpp:145-175)
// without a launch or a stream synchronisation per call: the workgroups of
// slot i poll slot i of a control block in coherent pinned host memory, read
// the request's blocks from pinned staging over PCIe, write the parities back
// there and publish `done`. Every workgroup leaves the loop on the stop flag,
// once NO slot has had a request for `idle_ticks` of wall clock, or after
// `life_ticks`; the last one out publishes exited_epoch = epoch, and the host
// launches the next epoch when a request finds the service gone.
#ifndef ECW_SVC_SLOTS
#define ECW_SVC_SLOTS 16
#endif
constexpr int kSvcSlots = ECW_SVC_SLOTS;  // concurrent callers served at once
constexpr size_t kSvcMaxLen = size_t(64) << 10;   // bytes per block served (larger: launch path)
constexpr size_t kSvcLds = size_t(60) << 10;       // LDS for the packed tables: k * 128 * nw bytes

// `seq` and `done` hold a request word: the request number in the low 32
// bits, the number of parts with work (one per 1 KiB column unit, at most
// kSvcParts) in bits 32..39, the generation of the request words below in the
// bits from kSvcSeqBits. The host bumps the generation only when the request
// words change (another codec, length or staging), so a workgroup that
// already holds that generation skips reading them: one PCIe round trip less
// per call. Parts without work only note the word; the host waits for the
// others' done words.
constexpr int kSvcSeqBits = 40;
constexpr int kSvcXorRow = 1;  // request flag: one global row, all coefficients 1 (a plain XOR)
constexpr unsigned long long kSvcReqMask = 0xFFFFFFFFull;
__host__ __device__ inline int svc_active_parts(unsigned long long seq) { return static_cast<int>((seq >> 32) & 0xFF); }

// Each slot is served by kSvcParts workgroups of kSvcThreads lanes, each
// taking every kSvcParts-th 1 KiB column unit (one dword per lane): the
// blocks of a call come in through several CUs at once (one wave reads pinned
// host memory at ~2 GB/s) and its GF products run on four SIMDs per part.
// Wave 0 of every part polls the slot; every part publishes its own `done`
// word, and the call is finished when all of them hold its request word.
#ifndef ECW_SVC_PARTS
#define ECW_SVC_PARTS 8
#endif
constexpr int kSvcParts = ECW_SVC_PARTS;
static_assert(kSvcParts >= 1 && kSvcParts <= 8, "one done word per part in the slot's second line");
constexpr int kSvcWave = 64;       // wave size
constexpr int kSvcThreads = 256;   // threads per service workgroup (four waves)

struct alignas(64) SvcSlot {
  unsigned long long seq;    // host: word of the latest request
  unsigned long long pad0[7];
  unsigned long long done[8];  // device: word of the latest request part p finished
  // the request words (written by the host before `seq` when they change)
  const void* tbl;           // packed tables of the codec's pass 0 (device memory)
  uint8_t* data;             // k input rows, `cs` bytes apart (device view of pinned staging)
  uint8_t* out;              // parity rows [G.., L..], `cs` bytes apart
  unsigned long long len, cs;
  unsigned long long serial;  // the codec's unique serial: tables staged in LDS are its tables
  int k, nrows, m, r, groups, local_mode, nw, flags;  // flags: kSvcXorRow
};

struct SvcCtl {
  unsigned long long stop;          // host: leave now
  unsigned long long exited_epoch;  // device: the epoch that last left the loop
  unsigned long long started_epoch; // device: the epoch whose first workgroup is running
  unsigned long long pad[5];
  SvcSlot slot[kSvcSlots];
};

// device-memory state of one service launch (zeroed before every launch)
struct SvcDev {
  unsigned long long last_active;  // wall clock of the latest request served by any workgroup
  unsigned int exited;             // workgroups that left the loop
  unsigned int pad;
  struct Slot {
    unsigned long long seq;        // kSvcLeave once part 0 has left (tells the other parts)
    unsigned long long pad[7];
  } slot[kSvcSlots];
};

hipError_t launch_service(SvcCtl* d_ctl, SvcDev* d_state, unsigned long long epoch, unsigned long long idle_ticks,
                          unsigned long long life_ticks, hipStream_t s);

}  // namespace ecw
