// Issue rates of the encode tile's instruction mix on gfx950 (tools only):
// how many wave-instructions per CU-cycle the VALU sustains for v_perm_b32 /
// v_bitop3_b32, the LDS for conflict-free ds_read_b32 nibble lookups, and
// both interleaved in the asm tile's ratio (2 VALU : 1 LDS). Cycles are the
// waves' own s_memtime deltas (shader clock), so DVFS does not enter.
// Build: hipcc --offload-arch=gfx950 -O3 tools/csrc/valubench.hip -o build/valubench
// Run:   build/valubench [ITERS]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int kChains = 16;

#define PERM1(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(sel));
#define BOP1(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(sel));
// lookup: address = low 6 bits of a[i] (dword aligned) within a 64 B table, as
// the nibble lookups (16 entries x 4 B, distinct banks)
#define LDS1(i) asm volatile("v_and_b32 %0, 0x3c, %0\n\tds_read_b32 %0, %0" : "+v"(a[i]));
#define WAITL asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#define SDWA1(i) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(a[i]) : "v"(b));
#define ANDOR1(i) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(sel));
#define SHL1(i) asm volatile("v_lshlrev_b32 %0, 2, %0" : "+v"(a[i]));
// wide lookups: 16 entries of W bytes at a stride of S bytes (ds_read_b64 /
// b96 / b128), eight in flight per wave, the next address from the result
#define WIDE8(INS, MASK, T)                                                                         \
  {                                                                                                 \
    T t0, t1, t2, t3, t4, t5, t6, t7;                                                               \
    asm volatile("v_and_b32 %8, " MASK ", %8\n\t" INS " %0, %8\n\t"                                \
                 "v_and_b32 %9, " MASK ", %9\n\t" INS " %1, %9\n\t"                                \
                 "v_and_b32 %10, " MASK ", %10\n\t" INS " %2, %10\n\t"                             \
                 "v_and_b32 %11, " MASK ", %11\n\t" INS " %3, %11\n\t"                             \
                 "v_and_b32 %12, " MASK ", %12\n\t" INS " %4, %12\n\t"                             \
                 "v_and_b32 %13, " MASK ", %13\n\t" INS " %5, %13\n\t"                             \
                 "v_and_b32 %14, " MASK ", %14\n\t" INS " %6, %14\n\t"                             \
                 "v_and_b32 %15, " MASK ", %15\n\t" INS " %7, %15\n\t"                             \
                 "s_waitcnt lgkmcnt(0)"                                                             \
                 : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7), \
                   "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),   \
                   "+v"(a[7])                                                                       \
                 :                                                                                  \
                 : "memory");                                                                       \
    a[0] ^= t0.x; a[1] ^= t1.x; a[2] ^= t2.x; a[3] ^= t3.x;                                          \
    a[4] ^= t4.x; a[5] ^= t5.x; a[6] ^= t6.x; a[7] ^= t7.x;                                          \
  }
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef unsigned int v3u __attribute__((ext_vector_type(3)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define X16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

// MODE 0: v_perm_b32 only; 1: v_bitop3_b32 only; 2: ds_read_b32 (+ the
// v_and forming its address); 3: the tile's mix per chain: 2 v_perm + 1 bitop3
// + 1 ds_read_b32 (+ its v_and); 4: v_or_b32_sdwa (byte select); 5:
// v_and_or_b32; 6: v_lshlrev_b32; 7: ds_read_b64 (16 x 8 B); 8: ds_read_b96
// (16 entries at a 16 B stride: the 9-16-row tile's record, 12 bytes used);
// 9: ds_read_b128 (16 x 16 B) -- 7-9 each with a v_and and a v_xor per lookup
template <int MODE>
__global__ __launch_bounds__(256) void bench(uint32_t* out, int iters, uint32_t seed) {
  __shared__ uint32_t tab[64];
  if (threadIdx.x < 64) tab[threadIdx.x] = MODE >= 7 ? (threadIdx.x * 0x01010101u) & 0xF0F0F0F0u : threadIdx.x * 0x01010101u;
  __syncthreads();
  uint32_t a[kChains];
  const uint32_t b = seed ^ threadIdx.x, sel = 0x07050301u ^ (seed & 0x03030303u);
#pragma unroll
  for (int i = 0; i < kChains; ++i)
    a[i] = MODE == 7 ? (threadIdx.x * 8 + i * 24) & 0x78 : MODE >= 8 ? (threadIdx.x * 16 + i * 48) & 0xf0 : (threadIdx.x * 4 + i * 8) & 0x3c;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
      PERM1(0) PERM1(1) PERM1(2) PERM1(3) PERM1(4) PERM1(5) PERM1(6) PERM1(7)
      PERM1(8) PERM1(9) PERM1(10) PERM1(11) PERM1(12) PERM1(13) PERM1(14) PERM1(15)
    } else if constexpr (MODE == 1) {
      BOP1(0) BOP1(1) BOP1(2) BOP1(3) BOP1(4) BOP1(5) BOP1(6) BOP1(7)
      BOP1(8) BOP1(9) BOP1(10) BOP1(11) BOP1(12) BOP1(13) BOP1(14) BOP1(15)
    } else if constexpr (MODE == 2) {
      LDS1(0) LDS1(1) LDS1(2) LDS1(3) LDS1(4) LDS1(5) LDS1(6) LDS1(7)
      WAITL
      LDS1(8) LDS1(9) LDS1(10) LDS1(11) LDS1(12) LDS1(13) LDS1(14) LDS1(15)
      WAITL
    } else if constexpr (MODE == 4) {
      X16(SDWA1)
    } else if constexpr (MODE == 5) {
      X16(ANDOR1)
    } else if constexpr (MODE == 6) {
      X16(SHL1)
    } else if constexpr (MODE == 7) {
      WIDE8("ds_read_b64", "0x78", v2u)
      WIDE8("ds_read_b64", "0x78", v2u)
    } else if constexpr (MODE == 8) {
      WIDE8("ds_read_b96", "0xf0", v3u)
      WIDE8("ds_read_b96", "0xf0", v3u)
    } else if constexpr (MODE == 9) {
      WIDE8("ds_read_b128", "0xf0", v4u)
      WIDE8("ds_read_b128", "0xf0", v4u)
    } else {
      LDS1(0) LDS1(1) LDS1(2) LDS1(3) LDS1(4) LDS1(5) LDS1(6) LDS1(7)
      PERM1(8) PERM1(9) PERM1(10) PERM1(11) PERM1(12) PERM1(13) PERM1(14) PERM1(15)
      PERM1(8) PERM1(9) PERM1(10) PERM1(11) PERM1(12) PERM1(13) PERM1(14) PERM1(15)
      BOP1(8) BOP1(9) BOP1(10) BOP1(11) BOP1(12) BOP1(13) BOP1(14) BOP1(15)
      WAITL
      LDS1(8) LDS1(9) LDS1(10) LDS1(11) LDS1(12) LDS1(13) LDS1(14) LDS1(15)
      PERM1(0) PERM1(1) PERM1(2) PERM1(3) PERM1(4) PERM1(5) PERM1(6) PERM1(7)
      PERM1(0) PERM1(1) PERM1(2) PERM1(3) PERM1(4) PERM1(5) PERM1(6) PERM1(7)
      BOP1(0) BOP1(1) BOP1(2) BOP1(3) BOP1(4) BOP1(5) BOP1(6) BOP1(7)
      WAITL
#pragma unroll
      for (int i = 0; i < kChains; ++i) a[i] &= 0x3c;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = tab[threadIdx.x & 63];  // the table stays allocated
#pragma unroll
  for (int i = 0; i < kChains; ++i) x ^= a[i];
  const unsigned wave = (blockIdx.x * 256 + threadIdx.x) / 64;
  // per wave: shader cycles, 100 MHz ticks (the wave's own clock = their ratio)
  if ((threadIdx.x & 63) == 0) {
    out[2 * wave] = static_cast<uint32_t>(t1 - t0);
    out[2 * wave + 1] = static_cast<uint32_t>(r1 - r0) | (x == 0x12345678u ? 0x80000000u : 0u);
  }
}

// wave-instructions per iteration and mode: {VALU, LDS}
static const int kValu[10] = {16, 16, 16, 16 + 32 + 16 + 16, 16, 16, 16, 32, 32, 32};  // mix: 16 v_and + 32 perm + 16 bitop3 + 16 re-masks
static const int kLds[10] = {0, 0, 16, 16, 0, 0, 0, 16, 16, 16};
static const char* kName[10] = {"v_perm_b32", "v_bitop3_b32", "ds_read_b32 (+v_and)", "mix 2 perm : 1 bitop3 : 1 lds",
                                "v_or_b32_sdwa (BYTE_1)", "v_and_or_b32", "v_lshlrev_b32",
                                "ds_read_b64 (+v_and, v_xor)", "ds_read_b96 16B-stride (+2)", "ds_read_b128 (+2)"};

template <int MODE>
static void run(int blocks_per_cu, int cus, int iters) {
  const int blocks = blocks_per_cu * cus, waves = blocks * 4;
  uint32_t* out;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * 2 * waves));
  hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(256), 0, 0, out, 8, 1u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint32_t> h(2 * waves);
  CHECK(hipMemcpy(h.data(), out, sizeof(uint32_t) * 2 * waves, hipMemcpyDeviceToHost));
  std::vector<double> clk;
  for (int w = 0; w < waves; ++w) clk.push_back(h[2 * w] / ((h[2 * w + 1] & 0x7fffffffu) * 10e-9) / 1e9);
  std::sort(clk.begin(), clk.end());
  const double ghz = clk[clk.size() / 2];  // the waves' own clock
  // whole-chip rates over the launch's wall time at that clock
  const double cu_cycles = static_cast<double>(cus) * ms * 1e-3 * ghz * 1e9;
  const double valu = static_cast<double>(kValu[MODE]) * iters * waves / cu_cycles;
  const double lds = static_cast<double>(kLds[MODE]) * iters * waves / cu_cycles;
  std::printf("%-30s %2d waves/SIMD: %.3f ms, clock %.2f GHz; VALU %.3f, LDS %.3f wave-instr per CU-cycle\n",
              kName[MODE], blocks_per_cu, ms, ghz, valu, lds);
  CHECK(hipFree(out));
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  std::printf("%d CUs, %d iterations\n", cus, iters);
  if (argc > 2 && std::atoi(argv[2]) == 1) {  // the wide lookups only
    for (int bpc : {1, 2, 4, 8}) {
      run<2>(bpc, cus, iters);
      run<7>(bpc, cus, iters);
      run<8>(bpc, cus, iters);
      run<9>(bpc, cus, iters);
    }
    return 0;
  }
  for (int bpc : {1, 2, 4, 8}) {
    run<0>(bpc, cus, iters);
    run<1>(bpc, cus, iters);
    run<2>(bpc, cus, iters);
    run<3>(bpc, cus, iters / 4);
    run<4>(bpc, cus, iters);
    run<5>(bpc, cus, iters);
    run<6>(bpc, cus, iters);
  }
  return 0;
}
