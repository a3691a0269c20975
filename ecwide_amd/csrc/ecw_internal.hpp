// Internal interface between the host codec (ecw_codec.cpp) and the HIP
// kernels (ecw_kernels.hip). Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace ecw {

constexpr int kMaxSrc = 256;      // k + m <= 256 for a GF(2^8) Cauchy code
constexpr int kMaxPassRows = 8;   // global rows per encode pass (u64 packed entries)
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

struct EncodeGeom {
  uint64_t len;          // bytes per block
  uint64_t tiles;        // column tiles per stripe = ceil(len / kTileBytes)
  int stripes;
  int k, r, groups;      // data rows, group size, local groups
  int m;                 // total global rows (slab output indexing)
  int row0, nrows;       // global rows of this pass [row0, row0 + nrows)
  int local_mode;        // LocalMode
  uint64_t tile_begin;   // this launch covers slab tiles [tile_begin, tile_end)
  uint64_t tile_end;     //   (tile = stripe * tiles + column tile)
  unsigned long long* ticket;  // non-null: workgroups take tiles in order from this counter
  uint64_t ticket_base;        //   whose value at this launch's start is ticket_base
};

// Device counter of ticket-ordered encode launches, one per (codec, stream).
// It is never reset: a launch whose grid has G workgroups over T tiles takes
// exactly T + G tickets (every workgroup draws one past the end to stop), so
// the host knows the counter's value at the start of the next launch on the
// same stream. The owner serialises launches that use one counter.
struct TicketCounter {
  unsigned long long* ptr = nullptr;
  uint64_t next = 0;
};

// Launchers return hipSuccess or the launch error (an earlier, unrelated HIP
// error of the calling thread is cleared first, not reported). The encode
// launchers run a slab of >= ECW_TICKET_MIN_TILES tiles as one ticket-ordered
// launch when `tc` is given, else in launch windows.
hipError_t launch_encode_ptr(const PtrRows& rows, const EncodeGeom& g, const void* d_tbl,
                             hipStream_t s, TicketCounter* tc);
hipError_t launch_encode_slab(const SlabRows& slab, const EncodeGeom& g, const void* d_tbl,
                              hipStream_t s, TicketCounter* tc);
hipError_t launch_encode_tab(const PtrTabRows& rows, const EncodeGeom& g, const void* d_tbl,
                             hipStream_t s, TicketCounter* tc);
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
struct XorGeom {
  uint64_t len, tiles;
  int stripes, n;
};
hipError_t launch_xor_ptr(const XorPtr& p, const XorGeom& g, hipStream_t s);
hipError_t launch_xor_slab(const XorSlab& p, const XorGeom& g, hipStream_t s);
hipError_t launch_xor_split(const XorSplit& p, const XorGeom& g, hipStream_t s);

hipError_t launch_fill_random(uint8_t* dst, uint64_t bstride, uint64_t sstride, int stripes,
                              int nblocks, uint64_t len, uint64_t piece, uint64_t pstride,
                              uint64_t offset, uint64_t seed, int s0, int b0, hipStream_t s);

int device_cu_count(int device);

}  // namespace ecw
