// The resident small-stripe request service for gfx950 (ecw_internal.hpp
// SvcCtl, host side ecw_codec.cpp svc::): synchronous small host-memory
// encodes and XORs (ECWide-H encodes one 4 KiB chunk per ec_encode_data call,
// ECWide-H/proxy/encode.cpp:145-175) served by a persistent kernel that polls
// request words in coherent pinned host memory -- no launch, DMA or stream
// synchronisation per call. The same packed-table GF(2^8) products as the
// encode kernels (ecw_kernels.hip).
#include "ecw_device.hpp"

namespace ecw {
namespace {

// ---- small-stripe request service (ecw_internal.hpp SvcCtl) ----------------
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
      if constexpr (XORROW)
        acc[0] ^= v[u];  // coefficient 1 everywhere: the product is the byte itself
      else
        gf_dw<NW>(v[u], acc, lds_base + static_cast<uint32_t>(j) * (128u * NW));
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
          for (int z = 0; z < kSvcColdSleeps; ++z) __builtin_amdgcn_s_sleep(127);
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
    // activity counts from the request's arrival, so part 0 never leaves on
    // idle while one of its requests is still in flight
    if (part == 0 && threadIdx.x == 0)
      __hip_atomic_fetch_max(&st->last_active, static_cast<unsigned long long>(wall_clock64()), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the request and its blocks are visible
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
    if (q.nw == 2)
      svc_request<2>(q, lds_base, part);
    else
      svc_request<1>(q, lds_base, part);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this wave's parities are visible
    __syncthreads();                               // ... and every wave's, before this part's done
    last = seq;
    if (threadIdx.x == 0) {
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

}  // namespace ecw
