// Store flavours against the WRITE_SIZE counter and the clock (tools only;
// VERDICT r02 item 7). Known byte counts, the bench's tiled geometry:
//   store_only<F>:   every workgroup writes one 4 KiB column tile of 8 parity
//                    pieces (8 KiB apart inside a 64 KiB run per unit), the
//                    encode's parity-store pattern without any reads
//   mix<F, WIN>:     the encode's byte mix: 128 data rows of a (stripe, piece)
//                    unit read with nontemporal loads (XOR instead of GF math),
//                    then the same 8 stores; WIN = the asm tile's write window
//                    (first 64 of every 2048 ticks of s_memrealtime)
// F: 0 plain, 1 nt, 2 nt sc0 sc1 (the encode's current stores), 3 sc0 sc1,
//    4 nt sc1, 5 sc1.
// Build: hipcc --offload-arch=gfx950 -O3 tools/csrc/storebench.hip -o build/storebench
// Run:   build/storebench ITERS      (rocprofv3 --pmc WRITE_SIZE -- build/storebench 1)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kK = 128;           // data rows per unit
constexpr int kOut = 8;           // parity rows per unit
constexpr uint64_t kPiece = 8192; // tiled slab piece

template <int F>
__device__ __forceinline__ void st(uint8_t* p, u32x4 v) {
  if constexpr (F == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
  if constexpr (F == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  if constexpr (F == 2) asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (F == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (F == 4) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (F == 5) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ uint8_t* out_at(uint8_t* pbase, uint64_t t, int i) {
  const uint64_t u = t >> 1, h = t & 1;
  return pbase + u * (kOut * kPiece) + (uint64_t)i * kPiece + h * 4096 + threadIdx.x * 16;
}

template <int F>
__global__ __launch_bounds__(256) void store_only(uint8_t* pbase) {
  const uint64_t t = blockIdx.x;
  const u32x4 v = {(uint32_t)t, threadIdx.x, 0x5a5a5a5au, (uint32_t)(t >> 7)};
#pragma unroll
  for (int i = 0; i < kOut; ++i) st<F>(out_at(pbase, t, i), v ^ (u32x4){(uint32_t)i, 0, 0, 0});
}

template <int F, bool WIN>
__global__ __launch_bounds__(256) void mix(const uint8_t* base, uint8_t* pbase) {
  extern __shared__ u32x4 lds_occ[];  // dynamic LDS only sets the occupancy
  const uint64_t t = blockIdx.x, u = t >> 1, h = t & 1;
  const uint8_t* p = base + u * (kK * kPiece) + h * 4096 + threadIdx.x * 16;
  u32x4 acc[kOut];
#pragma unroll
  for (int i = 0; i < kOut; ++i) acc[i] = (u32x4){0, 0, 0, 0};
  u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + kPiece));
  for (int j = 0; j < kK - 2; j += 2) {
    acc[j & 7] ^= a;
    a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + 2) * kPiece));
    acc[(j + 1) & 7] ^= b;
    b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + 3) * kPiece));
  }
  acc[6] ^= a;
  acc[7] ^= b;
  if (WIN) {
    for (int n = 0; n < 16384 && (unsigned)(wall_clock64() & 2047) >= 64u; ++n) __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_s_waitcnt(0);  // every load consumed before the asm stores (vmcnt counts both)
#pragma unroll
  for (int i = 0; i < kOut; ++i) st<F>(out_at(pbase, t, i), acc[i]);
  if (t == ~0ull) lds_occ[threadIdx.x] = acc[0];
}

__global__ void fill_random(uint64_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

template <class L>
static double time_ms(L launch, int iters) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / iters;
}

static const char* kName[] = {"plain", "nt", "nt sc0 sc1", "sc0 sc1", "nt sc1", "sc1"};

template <int F>
static void one(const uint8_t* base, uint8_t* pbase, unsigned ntiles, int iters, int lds) {
  const double wbytes = (double)ntiles * kOut * 4096, mbytes = (double)ntiles * (kK + kOut) * 4096;
  const double so = time_ms([&] { store_only<F><<<ntiles, 256>>>(pbase); }, iters);
  const double mx = time_ms([&] { mix<F, false><<<ntiles, 256, lds>>>(base, pbase); }, iters);
  const double mw = time_ms([&] { mix<F, true><<<ntiles, 256, lds>>>(base, pbase); }, iters);
  std::printf("F=%d %-11s store-only %7.1f GB/s | mix %7.1f GB/s, with write window %7.1f GB/s (%d B LDS/WG)\n", F,
              kName[F], wbytes / so / 1e6, mbytes / mx / 1e6, mbytes / mw / 1e6, lds);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 5;
  const int lds = argc > 2 ? std::atoi(argv[2]) : 24576;  // 6 WG/CU, the asm encode's occupancy
  const unsigned ntiles = 131072;  // 8 stripes x 64 MiB / 4 KiB: the bench's tiles
  const uint64_t units = ntiles / 2;
  uint8_t *base, *pbase;
  CHECK(hipMalloc(&base, units * kK * kPiece));
  CHECK(hipMalloc(&pbase, units * kOut * kPiece));
  fill_random<<<65536, 256>>>(reinterpret_cast<uint64_t*>(base), units * kK * kPiece / 8);
  CHECK(hipDeviceSynchronize());
  std::printf("tiled geometry: %u tiles, stores %.3f GB per launch, mix %.3f GB per launch\n", ntiles,
              ntiles * kOut * 4096.0 / 1e9, ntiles * (kK + kOut) * 4096.0 / 1e9);
  for (int rep = 0; rep < 2; ++rep) {
    one<0>(base, pbase, ntiles, iters, lds);
    one<1>(base, pbase, ntiles, iters, lds);
    one<2>(base, pbase, ntiles, iters, lds);
    one<3>(base, pbase, ntiles, iters, lds);
    one<4>(base, pbase, ntiles, iters, lds);
    one<5>(base, pbase, ntiles, iters, lds);
  }
  CHECK(hipFree(base));
  CHECK(hipFree(pbase));
  return 0;
}
