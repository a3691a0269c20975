// Read-only HBM stream rates for the encode's access pattern (tools only).
//   rows:  a 4 KiB column tile of K rows, rows BSTRIDE apart (the encode ring)
//   flat:  the same bytes read as one contiguous run per workgroup
// U = 16-byte loads in flight per lane. Prints GB/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void rows_kernel(const uint8_t* base, uint64_t bstride, uint64_t sstride,
                                                   int k, uint64_t tiles_per_stripe, uint32_t* sink) {
  const uint64_t tile = blockIdx.x;
  const uint64_t s = tile / tiles_per_stripe, c = tile % tiles_per_stripe;
  const uint8_t* p = base + s * sstride + c * 4096 + threadIdx.x * 16;
  u32x4 acc = {0, 0, 0, 0};
  for (int j = 0; j < k; j += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + u) * bstride))
                : *reinterpret_cast<const u32x4*>(p + (uint64_t)(j + u) * bstride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = 1;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void flat_kernel(const uint8_t* base, int k, uint32_t* sink) {
  const uint8_t* p = base + (uint64_t)blockIdx.x * k * 4096 + threadIdx.x * 16;
  u32x4 acc = {0, 0, 0, 0};
  for (int j = 0; j < k; j += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + u) * 4096))
                : *reinterpret_cast<const u32x4*>(p + (uint64_t)(j + u) * 4096);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = 1;
}

// the encode kernel's shape: stage n16 x 16 B of tables into LDS, then
// grid-stride over tiles (dynamic LDS size sets the occupancy)
template <int U>
__global__ __launch_bounds__(256) void rows_lds_kernel(const uint8_t* base, uint64_t bstride, uint64_t sstride,
                                                       int k, uint64_t tiles_per_stripe, uint64_t ntiles,
                                                       const u32x4* tbl, int n16, uint32_t* sink) {
  extern __shared__ u32x4 lds[];
  for (int i = threadIdx.x; i < n16; i += 256) lds[i] = tbl[i];
  __syncthreads();
  u32x4 acc = lds[threadIdx.x % (n16 ? n16 : 1)];
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t s = tile / tiles_per_stripe, c = tile % tiles_per_stripe;
    const uint8_t* p = base + s * sstride + c * 4096 + threadIdx.x * 16;
    for (int j = 0; j < k; j += U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + u) * bstride));
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u];
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = 1;
}

// 128 row reads + 8 output rows per tile (the CL(128,27,3) encode's byte
// mix, math replaced by XOR). ST: store the outputs; PF: issue the next
// tile's first two row loads before this tile's stores.
// SM: 0 nontemporal stores into the stripe's 8 output rows, 1 plain stores
// there, 2 nontemporal stores into one contiguous 32 KiB run per tile of a
// separate buffer (out)
template <bool ST, bool PF, int SM = 0, int NST = 8>
__global__ __launch_bounds__(256) void rows_st_kernel(uint8_t* base, uint64_t bstride, uint64_t sstride, int k,
                                                      uint64_t tiles_per_stripe, uint64_t ntiles, uint32_t* sink,
                                                      uint8_t* out = nullptr) {
  u32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = u32x4{0, 0, 0, 0};
  uint64_t tile = blockIdx.x;
  if (tile >= ntiles) return;
  auto rowp = [&](uint64_t t, int j) {
    const uint64_t s = t / tiles_per_stripe, c = t % tiles_per_stripe;
    return base + s * sstride + c * 4096 + threadIdx.x * 16 + (uint64_t)j * bstride;
  };
  u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(tile, 0)));
  u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(tile, 1)));
  for (; tile < ntiles; tile += gridDim.x) {
    const uint8_t* p = rowp(tile, 0);
    for (int j = 0; j < k - 2; j += 2) {
      acc[j & 7] ^= a;
      a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + 2) * bstride));
      acc[(j + 1) & 7] ^= b;
      b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + 3) * bstride));
    }
    acc[6] ^= a;
    acc[7] ^= b;
    const uint64_t nt = tile + gridDim.x;
    if (PF && nt < ntiles) {
      a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(nt, 0)));
      b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(nt, 1)));
    }
    if (ST) {
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        if (SM == 0)
          __builtin_nontemporal_store(acc[i], reinterpret_cast<u32x4*>(const_cast<uint8_t*>(p) + (uint64_t)(k + i) * bstride));
        else if (SM == 1)
          *reinterpret_cast<u32x4*>(const_cast<uint8_t*>(p) + (uint64_t)(k + i) * bstride) = acc[i];
        else if (SM >= 3) {
          u32x4* q = reinterpret_cast<u32x4*>(const_cast<uint8_t*>(p) + (uint64_t)(k + i) * bstride);
          if (SM == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q), "v"(acc[i]) : "memory");
          if (SM == 4) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(q), "v"(acc[i]) : "memory");
          if (SM == 5) asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1" ::"v"(q), "v"(acc[i]) : "memory");
          if (SM == 6) asm volatile("global_store_dwordx4 %0, %1, off nt sc0" ::"v"(q), "v"(acc[i]) : "memory");
          if (SM == 7) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(q), "v"(acc[i]) : "memory");
        } else
          __builtin_nontemporal_store(acc[i], reinterpret_cast<u32x4*>(out + tile * 32768 + (threadIdx.x / 64) * 8192 +
                                                                         i * 1024 + (threadIdx.x % 64) * 16));
      }
    }
    if (!PF && nt < ntiles) {
      a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(nt, 0)));
      b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(nt, 1)));
    }
  }
  if (!ST) {
    u32x4 x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3] ^ acc[4] ^ acc[5] ^ acc[6] ^ acc[7];
    if ((x.x ^ x.y ^ x.z ^ x.w) == 0x12345678u) sink[threadIdx.x] = 1;
  }
}

// Same bytes as rows_st<true,false,0,8>, but the 4 reading waves hand their 8
// output rows to a 5th (writer) wave through LDS, so no reading wave ever
// has a store outstanding (vmcnt is in order: a load issued after a store
// cannot be consumed before the store is acknowledged).
__global__ __launch_bounds__(320) void rows_wr_kernel(uint8_t* base, uint64_t bstride, uint64_t sstride, int k,
                                                      uint64_t tiles_per_stripe, uint64_t ntiles, uint32_t* sink) {
  __shared__ u32x4 stage[8][256];  // 32 KiB: [output row][lane of the 4 reading waves]
  const int tid = threadIdx.x;
  const bool writer = tid >= 256;
  auto rowp = [&](uint64_t t, int j, int lane) {
    const uint64_t s = t / tiles_per_stripe, c = t % tiles_per_stripe;
    return base + s * sstride + c * 4096 + lane * 16 + (uint64_t)j * bstride;
  };
  if (writer) {
    const int l = tid - 256;  // 64 writer lanes cover the 4 KiB tile row in 4 steps
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      __syncthreads();  // A: previous stage consumed (by us)
      __syncthreads();  // B: stage holds this tile
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          __builtin_nontemporal_store(stage[i][q * 64 + l],
                                      reinterpret_cast<u32x4*>(rowp(tile, k + i, q * 64 + l)));
    }
    return;
  }
  u32x4 acc[8];
  uint64_t tile = blockIdx.x;
  if (tile >= ntiles) return;  // grid <= ntiles on the host side, so never taken
  u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(tile, 0, tid)));
  u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(tile, 1, tid)));
  for (; tile < ntiles; tile += gridDim.x) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = u32x4{0, 0, 0, 0};
    const uint8_t* p = rowp(tile, 0, tid);
    for (int j = 0; j < k - 2; j += 2) {
      acc[j & 7] ^= a;
      a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + 2) * bstride));
      acc[(j + 1) & 7] ^= b;
      b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + 3) * bstride));
    }
    acc[6] ^= a;
    acc[7] ^= b;
    const uint64_t nt = tile + gridDim.x;
    if (nt < ntiles) {
      a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(nt, 0, tid)));
      b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp(nt, 1, tid)));
    }
    __syncthreads();  // A
#pragma unroll
    for (int i = 0; i < 8; ++i) stage[i][tid] = acc[i];
    __syncthreads();  // B
  }
}

// flat reads (each tile's 128 x 4 KiB contiguous) + NST output rows into a
// separate contiguous region; and a plain 16 B/lane copy
template <int NST, bool INPLACE = false>
__global__ __launch_bounds__(256) void flat_st_kernel(const uint8_t* in, uint8_t* out, int k, uint64_t ntiles) {
  u32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = u32x4{0, 0, 0, 0};
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint8_t* p = in + tile * (INPLACE ? k + 8 : k) * 4096 + threadIdx.x * 16;
    for (int j = 0; j < k; j += 2) {
      u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)j * 4096));
      u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (uint64_t)(j + 1) * 4096));
      acc[j & 7] ^= a;
      acc[(j + 1) & 7] ^= b;
    }
#pragma unroll
    for (int i = 0; i < NST; ++i)
      __builtin_nontemporal_store(acc[i], reinterpret_cast<u32x4*>(
          INPLACE ? const_cast<uint8_t*>(p) + (uint64_t)(k + i) * 4096 : out + (tile * NST + i) * 4096 + threadIdx.x * 16));
  }
}

__global__ __launch_bounds__(256) void copy_kernel(const u32x4* in, u32x4* out, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

__global__ void fill_random(uint64_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

template <class F>
static double time_ms(F launch, int iters) {
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
  return ms / iters;
}

int main(int argc, char** argv) {
  const int k = 128, S = 8;
  const uint64_t B = 64ull << 20, bstride = B + 4096, sstride = (uint64_t)(k + 8) * bstride;
  const uint64_t bytes = (uint64_t)S * k * B;
  uint8_t* buf;
  uint32_t* sink;
  CHECK(hipMalloc(&buf, S * sstride));
  CHECK(hipMalloc(&sink, 4096));
  const bool rnd = argc > 2 && std::atoi(argv[2]);
  if (rnd)
    fill_random<<<65536, 256>>>(reinterpret_cast<uint64_t*>(buf), S * sstride / 8);
  else
    CHECK(hipMemset(buf, 0x5a, S * sstride));
  CHECK(hipDeviceSynchronize());
  std::printf("data: %s\n", rnd ? "random" : "constant 0x5a");
  const uint64_t tps = B / 4096, ntiles = S * tps;
  const int iters = argc > 1 ? std::atoi(argv[1]) : 5;
#define ROWS(U, NT)                                                                                          \
  {                                                                                                          \
    double ms = time_ms([&] { rows_kernel<U, NT><<<ntiles, 256>>>(buf, bstride, sstride, k, tps, sink); }, iters); \
    std::printf("rows U=%d nt=%d  %8.1f GB/s\n", U, NT, bytes / ms / 1e6);                                  \
  }
#define FLAT(U, NT)                                                                                          \
  {                                                                                                          \
    double ms = time_ms([&] { flat_kernel<U, NT><<<ntiles, 256>>>(buf, k, sink); }, iters);                  \
    std::printf("flat U=%d nt=%d  %8.1f GB/s\n", U, NT, bytes / ms / 1e6);                                  \
  }
  u32x4* tbl;
  CHECK(hipMalloc(&tbl, 1 << 16));
  CHECK(hipMemset(tbl, 0, 1 << 16));
#define RL(U, GRID, N16, LDSB)                                                                                \
  {                                                                                                          \
    const unsigned grid = GRID ? GRID : (unsigned)ntiles;                                                    \
    double ms = time_ms([&] { rows_lds_kernel<U><<<grid, 256, LDSB>>>(buf, bstride, sstride, k, tps, ntiles, tbl, N16, sink); }, iters); \
    std::printf("rows_lds U=%d grid=%u stage=%d lds=%d  %8.1f GB/s\n", U, grid, N16 * 16, LDSB, bytes / ms / 1e6); \
  }
  const uint64_t sbytes = (uint64_t)S * (k + 8) * B;
#define RS(ST, PF, GRID)                                                                                       \
  {                                                                                                          \
    const unsigned grid = GRID ? GRID : (unsigned)ntiles;                                                    \
    double ms = time_ms([&] { rows_st_kernel<ST, PF><<<grid, 256>>>(buf, bstride, sstride, k, tps, ntiles, sink); }, iters); \
    std::printf("rows_st st=%d pf=%d grid=%u  %8.1f GB/s (136 rows counted)\n", ST, PF, grid, sbytes / ms / 1e6); \
  }
  uint8_t* out;
  CHECK(hipMalloc(&out, ntiles * 32768));
#define RSM(SM, GRID)                                                                                        \
  {                                                                                                          \
    const unsigned grid = GRID ? GRID : (unsigned)ntiles;                                                    \
    double ms = time_ms([&] { rows_st_kernel<true, false, SM><<<grid, 256>>>(buf, bstride, sstride, k, tps, ntiles, sink, out); }, iters); \
    std::printf("rows_st sm=%d grid=%u  %8.1f GB/s (136 rows counted)\n", SM, grid, sbytes / ms / 1e6);     \
  }
#define RSN(NST)                                                                                             \
  {                                                                                                          \
    double ms = time_ms([&] { rows_st_kernel<true, false, 0, NST><<<65536, 256>>>(buf, bstride, sstride, k, tps, ntiles, sink, out); }, iters); \
    const double by = (double)S * (k + NST) * B;                                                             \
    std::printf("rows_st stores=%d grid=65536  %8.1f GB/s (128+%d rows counted)\n", NST, by / ms / 1e6, NST);  \
  }
  if (argc > 6) {
    const uint64_t n16 = (uint64_t)S * k * B / 16 / 2;
    for (int rep = 0; rep < 2; ++rep) {
      for (unsigned grid : {65536u, 262144u}) {
        double ms = time_ms([&] { copy_kernel<<<grid, 256>>>(reinterpret_cast<const u32x4*>(buf),
                                                             reinterpret_cast<u32x4*>(buf) + n16, n16); }, iters);
        std::printf("copy grid=%u  %8.1f GB/s (read + write)\n", grid, 2.0 * n16 * 16 / ms / 1e6);
      }
#define FST(NST)                                                                                             \
  {                                                                                                          \
    double ms = time_ms([&] { flat_st_kernel<NST><<<65536, 256>>>(buf, out, k, ntiles); }, iters);           \
    std::printf("flat_st stores=%d  %8.1f GB/s (128+%d rows counted)\n", NST, (double)S * (k + NST) * B / ms / 1e6, NST); \
  }
      FST(1) FST(8)
      {
        double ms = time_ms([&] { flat_st_kernel<8, true><<<65536, 256>>>(buf, out, k, ntiles); }, iters);
        std::printf("flat_st in-place (4 KiB chunk layout) stores=8  %8.1f GB/s (136 rows counted)\n", (double)S * (k + 8) * B / ms / 1e6);
      }
      for (unsigned grid : {65536u, 131072u}) {
        double ms = time_ms([&] { rows_st_kernel<true, false, 0, 8><<<grid, 256>>>(buf, bstride, sstride, k, tps, ntiles, sink, out); }, iters);
        std::printf("rows_st stores=8 grid=%u  %8.1f GB/s (136 rows counted)\n", grid, (double)S * (k + 8) * B / ms / 1e6);
      }
    }
    return 0;
  }
  if (argc > 5) {
    for (int rep = 0; rep < 2; ++rep) {
      RS(false, false, 65536) RSN(1) RSN(8)
      for (unsigned grid : {16384u, 32768u, 65536u}) {
        double ms = time_ms([&] { rows_wr_kernel<<<grid, 320>>>(buf, bstride, sstride, k, tps, ntiles, sink); }, iters);
        std::printf("rows_wr (writer wave) grid=%u  %8.1f GB/s (136 rows counted)\n", grid, sbytes / ms / 1e6);
      }
    }
    return 0;
  }
  for (int rep = 0; rep < 2; ++rep) {
    RSM(0, 65536) RSM(1, 65536) RSM(3, 65536) RSM(4, 65536) RSM(5, 65536) RSM(6, 65536) RSM(7, 65536)
  }
  if (argc > 4) return 0;
  for (int rep = 0; rep < 2; ++rep) {
    RS(false, false, 65536) RS(true, false, 65536) RS(true, true, 65536)
    RS(false, false, 0) RS(true, false, 0)
    RS(false, false, 16384) RS(true, false, 16384) RS(true, true, 16384)
    RS(true, false, 4096) RS(true, true, 4096)
  }
  if (argc > 3) return 0;
  for (int rep = 0; rep < 2; ++rep) {
    RL(2, 0, 0, 0) RL(2, 0, 1024, 16384) RL(2, 0, 1024, 20480) RL(2, 0, 1024, 26624) RL(2, 0, 1024, 40960)
    RL(2, 65536, 1024, 16384) RL(2, 65536, 1024, 26624) RL(2, 16384, 1024, 26624) RL(4, 65536, 1024, 26624)
  }
  for (int rep = 0; rep < 1; ++rep) {
    ROWS(2, true) ROWS(4, true) ROWS(8, true) ROWS(16, true) ROWS(4, false)
    FLAT(2, true) FLAT(4, true) FLAT(8, true) FLAT(16, true) FLAT(4, false)
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
