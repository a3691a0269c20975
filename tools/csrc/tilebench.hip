// Layout / tile-width experiments for the block (pointer-interface) layout
// (tools only). The encode's byte mix with the math replaced by XOR: each
// workgroup reads k = 128 data rows of a column tile through a 2-deep ring and
// writes 8 output rows, like CL(128, 27, 3). Variants:
//   blocks W  : rows B + 4 KiB apart (the block slab / separate blocks), each
//               lane W x 16 B per row (W loads 4 KiB apart: a W x 4 KiB tile),
//               outputs in rows k..k+7 of the stripe
//   tiled     : the tiled slab (8 KiB column pieces; a unit's 128 data pieces
//               contiguous, its 8 parity pieces contiguous in a separate region)
//   outputs=1  : block rows for the reads, outputs 8 rows x tile contiguous per
//               tile in a separate region (separates read and write layout)
//   outputs=2  : outputs in separate 64 MiB parity blocks (pointer mode)
//   st=0       : reads only
// argv: iters, block-stride padding (bytes)
// Prints GB/s counted over 136 rows. hipcc --offload-arch=gfx950 -O3
// tools/csrc/tilebench.hip -o build/tilebench && build/tilebench [iters]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Geo {
  uint8_t* base;      // data
  uint64_t bstride;   // between rows of a unit
  uint64_t ustride;   // between units
  uint64_t tpu;       // tiles per unit
  uint64_t tbytes;    // column bytes per tile (W * 4 KiB)
  uint8_t* pbase;     // outputs: tile t writes row i at
  uint64_t pbstride;  //   pbase + (t / ptpu) * pustride + (t % ptpu) * tbytes + i * pbstride
  uint64_t pustride;
  uint64_t ptpu;
  uint64_t ntiles;
  int k;
};

// the encode ring's load: a raw buffer load with the volatile bit, so the
// compiler keeps the 2-deep ring as written (ecw_kernels.hip ld16); the row
// address is wave-uniform (SGPRs), the lane's column the buffer offset
__device__ __forceinline__ u32x4 ldrow(const uint8_t* row, uint32_t off) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(row), 0, 0x7FFFFFFF, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(off), 0, static_cast<int>(0x80000000u));
}

template <int W, bool ST>
__global__ __launch_bounds__(256) void tile_kernel(Geo g, uint32_t* sink) {
  const uint64_t tile = blockIdx.x;
  if (tile >= g.ntiles) return;
  const uint64_t u = tile / g.tpu, c = tile % g.tpu;
  const uint8_t* p = g.base + u * g.ustride + c * g.tbytes;  // wave-uniform
  const uint32_t lane = threadIdx.x * 16;
  u32x4 acc[8][W];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int w = 0; w < W; ++w) acc[i][w] = u32x4{0, 0, 0, 0};
  u32x4 a[W], b[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    a[w] = ldrow(p, lane + w * 4096);
    b[w] = ldrow(p + g.bstride, lane + w * 4096);
  }
  // 8 rows per trip, unrolled, so acc[] is indexed by constants (k % 8 == 0);
  // the last trip loads nothing past row k-1
  for (int j0 = 0; j0 < g.k; j0 += 8) {
    const bool last = j0 + 8 >= g.k;
#pragma unroll
    for (int jj = 0; jj < 8; jj += 2) {
      const int j = j0 + jj;
      const bool more = !last || jj < 6;
      const uint8_t* ra = p + (uint64_t)(j + 2) * g.bstride;
      const uint8_t* rb = ra + g.bstride;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        acc[jj][w] ^= a[w];
        if (more) a[w] = ldrow(ra, lane + w * 4096);
      }
#pragma unroll
      for (int w = 0; w < W; ++w) {
        acc[jj + 1][w] ^= b[w];
        if (more) b[w] = ldrow(rb, lane + w * 4096);
      }
    }
  }
  if (ST) {
    uint8_t* q = g.pbase + (tile / g.ptpu) * g.pustride + (tile % g.ptpu) * g.tbytes + lane;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int w = 0; w < W; ++w)
        __builtin_nontemporal_store(acc[i][w], reinterpret_cast<u32x4*>(q + (uint64_t)i * g.pbstride + w * 4096));
  } else {
    u32x4 x = u32x4{0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int w = 0; w < W; ++w) x ^= acc[i][w];
    if ((x.x ^ x.y ^ x.z ^ x.w) == 0x12345678u) sink[threadIdx.x] = 1;
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
  return ms / iters;
}

int main(int argc, char** argv) {
  const int k = 128, S = 8;
  const uint64_t B = 64ull << 20, pad = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 4096;
  const uint64_t bstride = B + pad, sstride = (uint64_t)(k + 8) * bstride;
  const int iters = argc > 1 ? std::atoi(argv[1]) : 5;
  // one allocation: the block slab, and the tiled slab carved from the same memory
  const uint64_t bytes = S * sstride;
  uint8_t* buf;
  uint32_t* sink;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&sink, 4096));
  fill_random<<<65536, 256>>>(reinterpret_cast<uint64_t*>(buf), bytes / 8);
  CHECK(hipDeviceSynchronize());
  const double counted = (double)S * (k + 8) * B;
  const uint64_t units_t = S * (B / 8192);
  const uint64_t poff = (units_t * k * 8192 + 4095) / 4096 * 4096;

  // block rows; outputs in rows k.. of the stripe (mode 0), 8 rows of one
  // tile's width contiguous per tile in a separate region (mode 1), or
  // separate 64 MiB parity blocks in a separate region (mode 2: pointer mode
  // with parity buffers of their own)
  auto blocks = [&](uint64_t W, int mode) {
    const uint64_t tpu = B / (W * 4096);
    if (mode == 1)
      return Geo{buf, bstride, sstride, tpu, W * 4096, buf + poff, W * 4096, 8 * W * 4096, 1, S * tpu, k};
    if (mode == 2)
      return Geo{buf, bstride, sstride, tpu, W * 4096, buf + poff, B, 8 * B, tpu, S * tpu, k};
    return Geo{buf, bstride, sstride, tpu, W * 4096, buf + (uint64_t)k * bstride, bstride, sstride, tpu, S * tpu, k};
  };
  for (int rep = 0; rep < 2; ++rep) {
    {
      Geo g{buf, 8192, (uint64_t)k * 8192, 2, 4096, buf + poff, 8192, 8 * 8192, 2, units_t * 2, k};
      double ms = time_ms([&] { tile_kernel<1, true><<<g.ntiles, 256>>>(g, sink); }, iters);
      std::printf("tiled 8K pieces            %8.1f GB/s\n", counted / ms / 1e6);
    }
#define BL(W, ST, MODE)                                                                             \
  {                                                                                                 \
    Geo g = blocks(W, MODE);                                                                        \
    double ms = time_ms([&] { tile_kernel<W, ST><<<g.ntiles, 256>>>(g, sink); }, iters);           \
    std::printf("blocks W=%d st=%d outputs=%d  %8.1f GB/s\n", W, ST, MODE, counted / ms / 1e6);      \
  }
    BL(1, true, 0) BL(2, true, 0) BL(4, true, 0)
    BL(1, true, 1) BL(2, true, 1)
    BL(1, true, 2) BL(2, true, 2)
    BL(1, false, 0) BL(2, false, 0)
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
