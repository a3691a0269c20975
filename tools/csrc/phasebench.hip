// Does the encode's write cost come from reads and writes interleaving at the
// memory? (tools only). The CL(128,27,3) byte mix (128 row reads + 8 output
// rows per 4 KiB column tile, math replaced by XOR) run three ways:
//   inter:  every workgroup stores its tile's 8 rows as soon as it has them
//           (the encode kernel's pattern)
//   phased: a persistent grid; in each phase every workgroup reads T tiles and
//           keeps their outputs in registers, a grid barrier, then everyone
//           stores, optionally a second barrier before the next phase's reads
//   read-only / barrier-only controls
// Build: hipcc --offload-arch=gfx950 -O3 tools/csrc/phasebench.hip -o build/phasebench
// Run:   build/phasebench ITERS
// The barrier spins are bounded: a barrier that does not complete within
// ~2^22 polls gives up (and the run reports it), so a grid that is not fully
// resident cannot hang.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ldnt(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ void stnt(uint8_t* p, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// Grid barrier, two levels: a workgroup arrives on the counter of its group
// (blockIdx % 8, one counter per 256 B line), the last arrival of a group on
// the top counter, and the last group's last arrival publishes the barrier's
// generation, which every workgroup polls. Targets grow monotonically (the
// counters are zeroed before each launch). Gives up after ~2^22 polls.
__device__ int g_sleep = 1;
__device__ __forceinline__ void grid_sync(unsigned* ctr, unsigned gen, unsigned* fail) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned G = gridDim.x, grp = blockIdx.x & 7;
    const unsigned in_grp = G / 8 + (grp < G % 8 ? 1 : 0);
    const unsigned ngrp = G < 8 ? G : 8;
    unsigned* sub = ctr + 64 * (1 + grp);
    unsigned* top = ctr + 64 * 9;
    unsigned* flag = ctr;
    const unsigned old = __hip_atomic_fetch_add(sub, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == gen * in_grp) {
      const unsigned t = __hip_atomic_fetch_add(top, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (t + 1 == gen * ngrp) __hip_atomic_store(flag, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned n = 0;
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < gen) {
      if (g_sleep > 1) __builtin_amdgcn_s_sleep(8); else __builtin_amdgcn_s_sleep(1);
      if (++n > (1u << 22)) {
        __hip_atomic_fetch_add(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

struct Geo {
  uint8_t* base;
  uint64_t bstride, sstride, tps, ntiles;
  int k;
  uint8_t* pbase = nullptr;  // non-null: output rows in a region of their own
  uint64_t pbstride = 0, psstride = 0;
};

__device__ __forceinline__ uint8_t* rowp(const Geo& g, uint64_t t, int j) {
  const uint64_t s = t / g.tps, c = t % g.tps;
  return g.base + s * g.sstride + c * 4096 + threadIdx.x * 16 + (uint64_t)j * g.bstride;
}

__device__ __forceinline__ void read_tile(const Geo& g, uint64_t t, u32x4* acc) {
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = u32x4{0, 0, 0, 0};
  const uint8_t* p = rowp(g, t, 0);
  u32x4 a = ldnt(p), b = ldnt(p + g.bstride);
  for (int j = 0; j < g.k - 2; j += 2) {
    acc[j & 7] ^= a;
    a = ldnt(p + (uint64_t)(j + 2) * g.bstride);
    acc[(j + 1) & 7] ^= b;
    b = ldnt(p + (uint64_t)(j + 3) * g.bstride);
  }
  acc[6] ^= a;
  acc[7] ^= b;
}

template <int NOUT = 8>
__device__ __forceinline__ void write_tile(const Geo& g, uint64_t t, const u32x4* acc) {
  if (g.pbase) {
    const uint64_t su = t / g.tps, c = t % g.tps;
    uint8_t* q = g.pbase + su * g.psstride + c * 4096 + threadIdx.x * 16;
#pragma unroll
    for (int i = 0; i < NOUT; ++i) stnt(q + (uint64_t)i * g.pbstride, acc[i]);
    return;
  }
  uint8_t* p = rowp(g, t, g.k);
#pragma unroll
  for (int i = 0; i < NOUT; ++i) stnt(p + (uint64_t)i * g.bstride, acc[i]);
}

// read ring of depth D (loads in flight per lane)
template <int D>
__device__ __forceinline__ void read_tile_d(const Geo& g, uint64_t t, u32x4* acc) {
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = u32x4{0, 0, 0, 0};
  const uint8_t* p = rowp(g, t, 0);
  u32x4 v[D];
#pragma unroll
  for (int d = 0; d < D; ++d) v[d] = ldnt(p + (uint64_t)d * g.bstride);
  for (int j = 0; j < g.k - D; j += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[(j + d) & 7] ^= v[d];
      v[d] = ldnt(p + (uint64_t)(j + D + d) * g.bstride);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) acc[d & 7] ^= v[d];
}

// one tile per workgroup, stores right after the reads (the encode's pattern);
// dynamic LDS (unused) sets the occupancy; D = read ring depth
template <bool ST, int D = 2>
__global__ __launch_bounds__(256) void inter_kernel(Geo g, uint32_t* sink) {
  extern __shared__ u32x4 lds_occ[];
  u32x4 acc[8];
  if (D == 2) read_tile(g, blockIdx.x, acc); else read_tile_d<D>(g, blockIdx.x, acc);
  if (g.k < 0) lds_occ[threadIdx.x] = acc[0];
  if (ST) {
    write_tile(g, blockIdx.x, acc);
  } else {
    u32x4 x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3] ^ acc[4] ^ acc[5] ^ acc[6] ^ acc[7];
    if ((x.x ^ x.y ^ x.z ^ x.w) == 0x12345678u) sink[threadIdx.x] = 1;
  }
}

// MODE 0: phased (reads | barrier | writes), 1: phased + barrier after the
// writes, 2: barrier only (reads, writes, barrier), 3: interleaved, persistent
// grid without barriers, 5: the barriers alone. T tiles per workgroup per phase.
template <int MODE, int T>
__global__ __launch_bounds__(256) void phased_kernel(Geo g, unsigned* ctr, unsigned* fail) {
  const uint64_t G = gridDim.x;
  const uint64_t nphase = (g.ntiles + G * T - 1) / (G * T);
  unsigned gen = 0;
  for (uint64_t ph = 0; ph < nphase; ++ph) {
    u32x4 acc[T][8];
#pragma unroll
    for (int u = 0; u < T; ++u) {
      const uint64_t t = (ph * T + u) * G + blockIdx.x;
      if (t < g.ntiles) read_tile(g, t, acc[u]);
      if (MODE == 3 && t < g.ntiles) write_tile(g, t, acc[u]);
    }
    if (MODE == 0 || MODE == 1 || MODE == 5) {
      grid_sync(ctr, ++gen, fail);
    }
    if (MODE != 3 && MODE != 5) {
#pragma unroll
      for (int u = 0; u < T; ++u) {
        const uint64_t t = (ph * T + u) * G + blockIdx.x;
        if (t < g.ntiles) write_tile(g, t, acc[u]);
      }
    }
    if (MODE == 1 || MODE == 2) {
      __builtin_amdgcn_s_waitcnt(0);
      grid_sync(ctr, ++gen, fail);
    }
  }
}

// one tile per workgroup; the stores wait for the chip-wide write window:
// the first W ticks of every P ticks of the 100 MHz constant clock
// WAVE: every wave polls the clock itself (no workgroup barrier); P a power
// of two then (mask). LDS: dynamic LDS bytes, to set the occupancy.
template <bool WAVE, int NOUT = 8>
__global__ __launch_bounds__(256) void window_kernel(Geo g, unsigned P, unsigned W) {
  extern __shared__ u32x4 lds_pad[];
  u32x4 acc[8];
  read_tile(g, blockIdx.x, acc);
  if (WAVE) {
    while ((unsigned)(wall_clock64() & (P - 1)) >= W) __builtin_amdgcn_s_sleep(2);
  } else {
    if (threadIdx.x == 0) {
      while ((unsigned)(wall_clock64() % P) >= W) __builtin_amdgcn_s_sleep(2);
    }
    __syncthreads();
  }
  if (NOUT == 1) acc[0] ^= acc[1] ^ acc[2] ^ acc[3] ^ acc[4] ^ acc[5] ^ acc[6] ^ acc[7];
  write_tile<NOUT>(g, blockIdx.x, acc);
  if (g.k < 0) lds_pad[threadIdx.x] = acc[0];
}

// persistent workgroups, tiles i*G + blockIdx.x; a tile's outputs stay
// pending while the next tile is read and are stored at the first write
// window (checked every CHK rows); the wait is only for the last tile.
// P a power of two (ticks), W the window; W >= P: store at once (no window).
template <int CHK>
__global__ __launch_bounds__(256) void pipelined_kernel(Geo g, unsigned P, unsigned W) {
  u32x4 pend[8];
  bool has = false;
  uint64_t pt = 0;
  const bool nowin = W >= P;
  auto in_win = [&]() { return nowin || (unsigned)(wall_clock64() & (P - 1)) < W; };
  for (uint64_t t = blockIdx.x; t < g.ntiles; t += gridDim.x) {
    u32x4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = u32x4{0, 0, 0, 0};
    const uint8_t* p = rowp(g, t, 0);
    u32x4 a = ldnt(p), b = ldnt(p + g.bstride);
    for (int j = 0; j < g.k - 2; j += 2) {
      acc[j & 7] ^= a;
      a = ldnt(p + (uint64_t)(j + 2) * g.bstride);
      acc[(j + 1) & 7] ^= b;
      b = ldnt(p + (uint64_t)(j + 3) * g.bstride);
      if (has && (j % CHK) == 0 && in_win()) {
        write_tile(g, pt, pend);
        has = false;
      }
    }
    acc[6] ^= a;
    acc[7] ^= b;
    if (has) {
      while (!in_win()) __builtin_amdgcn_s_sleep(2);
      write_tile(g, pt, pend);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) pend[i] = acc[i];
    has = true;
    pt = t;
  }
  if (has) {
    while (!in_win()) __builtin_amdgcn_s_sleep(2);
    write_tile(g, pt, pend);
  }
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
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / iters;
}

template <int MODE, int T>
static void run_phased(const Geo& g, unsigned* ctr, unsigned* fail, int per_cu_div, int iters, double sbytes) {
  int dev = 0, ncu = 0, per_cu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, phased_kernel<MODE, T>, 256, 0));
  const int use = per_cu / per_cu_div > 0 ? per_cu / per_cu_div : 1;
  const unsigned grid = (unsigned)(ncu * use);
  CHECK(hipMemset(fail, 0, 4));
  double ms = time_ms([&] {
    CHECK(hipMemsetAsync(ctr, 0, 4096));
    phased_kernel<MODE, T><<<grid, 256>>>(g, ctr, fail);
  }, iters);
  unsigned f = 0;
  CHECK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
  std::printf("phased mode=%d T=%d grid=%u (%d/CU of %d)  %8.1f GB/s (136 rows counted)%s\n", MODE, T, grid, use,
              per_cu, sbytes / ms / 1e6, f ? "  BARRIER TIMEOUTS" : "");
}

int main(int argc, char** argv) {
  const int k = 128, S = 8;
  const uint64_t B = 64ull << 20, bstride = B + 4096, sstride = (uint64_t)(k + 8) * bstride;
  uint8_t* buf;
  uint32_t* sink;
  unsigned *ctr, *fail;
  CHECK(hipMalloc(&buf, S * sstride));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMalloc(&ctr, 4096));
  CHECK(hipMalloc(&fail, 256));
  fill_random<<<65536, 256>>>(reinterpret_cast<uint64_t*>(buf), S * sstride / 8);
  CHECK(hipDeviceSynchronize());
  const int iters = argc > 1 ? std::atoi(argv[1]) : 5;
  Geo g{buf, bstride, sstride, B / 4096, (uint64_t)S * (B / 4096), k};
  if (argc > 3 && std::atoi(argv[3]) == 1) {
    // the tiled slab's geometry: 8 KiB pieces, piece c of a stripe's 136 rows one
    // 1.06 MiB run (parities after the data here), two 4 KiB tiles per piece
    g.bstride = 8192;
    g.sstride = (uint64_t)(k + 8) * 8192;  // one (stripe, piece) unit
    g.tps = 2;
    g.ntiles = (uint64_t)S * (B / 4096);
    std::printf("geometry: tiled (rows 8 KiB apart)\n");
  }
  if (argc > 3 && std::atoi(argv[3]) == 2) {
    // the bench's tiled slab: (stripe, piece) units of k x 8 KiB data, their 8
    // parity pieces one 64 KiB run in a region after all the data
    g.bstride = 8192;
    g.sstride = (uint64_t)k * 8192;
    g.tps = 2;
    g.ntiles = (uint64_t)S * (B / 4096);
    g.pbase = buf + (uint64_t)S * k * B;
    g.pbstride = 8192;
    g.psstride = 8 * 8192;
    std::printf("geometry: tiled, parities in their own region (the bench's slab)\n");
  }
  const double sbytes = (double)S * (k + 8) * B;
  const bool sweep_barriers = argc > 2 && std::atoi(argv[2]) == 1;
  for (int rep = 0; rep < 2; ++rep) {
    double ms = time_ms([&] { inter_kernel<false><<<(unsigned)g.ntiles, 256>>>(g, sink); }, iters);
    std::printf("read-only one tile/WG          %8.1f GB/s (136 rows counted)\n", sbytes / ms / 1e6);
    ms = time_ms([&] { inter_kernel<true><<<(unsigned)g.ntiles, 256>>>(g, sink); }, iters);
    std::printf("interleaved one tile/WG        %8.1f GB/s (136 rows counted)\n", sbytes / ms / 1e6);
    for (int sl : {1, 2}) {
      if (!sweep_barriers) break;
      CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_sleep), &sl, sizeof(int)));
      std::printf("-- barrier poll sleep %s\n", sl > 1 ? "8" : "1");
      // barriers alone: report us per barrier
      {
        int dev = 0, ncu = 0, per_cu = 0;
        CHECK(hipGetDevice(&dev));
        CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, phased_kernel<5, 1>, 256, 0));
        const unsigned grid = ncu * per_cu;
        const uint64_t nph = (g.ntiles + grid - 1) / grid;
        double bms = time_ms([&] {
          CHECK(hipMemsetAsync(ctr, 0, 4096));
          phased_kernel<5, 1><<<grid, 256>>>(g, ctr, fail);
        }, iters);
        std::printf("barrier only grid=%u: %.2f us per barrier\n", grid, bms * 1e3 / nph);
      }
      run_phased<3, 1>(g, ctr, fail, 1, iters, sbytes);
      run_phased<2, 1>(g, ctr, fail, 1, iters, sbytes);
      run_phased<0, 1>(g, ctr, fail, 1, iters, sbytes);
      run_phased<1, 1>(g, ctr, fail, 1, iters, sbytes);
      run_phased<0, 1>(g, ctr, fail, 2, iters, sbytes);
      run_phased<0, 1>(g, ctr, fail, 4, iters, sbytes);
    }
    for (unsigned P : {2048u, 4096u, 8192u}) {
      const unsigned W = P / 32;
      double wms = time_ms([&] { window_kernel<true><<<(unsigned)g.ntiles, 256>>>(g, P, W); }, iters);
      double w6 = time_ms([&] { window_kernel<true><<<(unsigned)g.ntiles, 256, 24576>>>(g, P, W); }, iters);
      std::printf("wave window %4u of %5u ticks   %8.1f GB/s, at 6 WG/CU %8.1f (136 rows counted)\n", W, P,
                  sbytes / wms / 1e6, sbytes / w6 / 1e6);
    }
    // read-only and interleaved rates against occupancy (dynamic LDS) and ring depth
    for (int lds : {0, 24576, 36864}) {
      double r2 = time_ms([&] { inter_kernel<false, 2><<<(unsigned)g.ntiles, 256, lds>>>(g, sink); }, iters);
      double r4 = time_ms([&] { inter_kernel<false, 4><<<(unsigned)g.ntiles, 256, lds>>>(g, sink); }, iters);
      double s2 = time_ms([&] { inter_kernel<true, 2><<<(unsigned)g.ntiles, 256, lds>>>(g, sink); }, iters);
      double s4 = time_ms([&] { inter_kernel<true, 4><<<(unsigned)g.ntiles, 256, lds>>>(g, sink); }, iters);
      std::printf("lds %5d: read-only ring2 %7.1f ring4 %7.1f | with stores ring2 %7.1f ring4 %7.1f (136 rows counted)\n",
                  lds, sbytes / r2 / 1e6, sbytes / r4 / 1e6, sbytes / s2 / 1e6, sbytes / s4 / 1e6);
    }
    // the repair's mix: 27 rows -> 1 row
    if (argc > 4) {
      Geo r = g;
      r.k = 27;  // same geometry (rows 0..27 of each unit: inside it in both layouts)
      const double rbytes = (double)S * 28 * B;
      double a1 = time_ms([&] { window_kernel<true, 1><<<(unsigned)r.ntiles, 256>>>(r, 4096, 4096); }, iters);
      std::printf("repair mix 27+1, no window        %8.1f GB/s\n", rbytes / a1 / 1e6);
      for (unsigned W : {32u, 64u, 128u, 256u}) {
        double a2 = time_ms([&] { window_kernel<true, 1><<<(unsigned)r.ntiles, 256>>>(r, 4096, W); }, iters);
        std::printf("repair mix 27+1, window %3u/4096  %8.1f GB/s\n", W, rbytes / a2 / 1e6);
      }
    }
  }
  CHECK(hipFree(buf));
  return 0;
}
