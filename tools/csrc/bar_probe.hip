// Can the host write device memory directly (large BAR), and how fast?
// Allocates fine-grained device memory, asks the runtime whether the host
// may touch it, and only then writes it from the CPU: write rate for small
// (45 KiB) and large copies, and the round trip of a flag written by the CPU
// and echoed by a polling kernel. Tuning probe for the request service.
//
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/bar_probe tools/csrc/bar_probe.hip && /tmp/bar_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <csetjmp>
#include <csignal>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// echo: wait for flag[0] == i, write ack (host memory) = i; n rounds; every
// wave leaves after n rounds or a bounded number of polls
__global__ void echo(const unsigned long long* flag, unsigned long long* ack, int n) {
  for (int i = 1; i <= n; ++i) {
    long spins = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != static_cast<unsigned long long>(i))
      if (++spins > 3000000L) return;  // a few seconds: the host gave up
    if (threadIdx.x == 0) __hip_atomic_store(ack, static_cast<unsigned long long>(i), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// one wave: `rows` loads of 16 B per lane (1 KiB per row, rows `stride`
// bytes apart) from pinned host memory, cache-bypassing, all in flight at
// once; wall-clock ticks from issue to the last return, `iters` times
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// fence = 1: a system-scope acquire before each fetch (what the service
// does after seeing a request), so the rows come over PCIe, not from L2;
// ticks[2] accumulates the fence's own time
__global__ void fetch(const uint8_t* src, size_t stride, int rows, int iters, unsigned long long* ticks, int fence) {
  unsigned long long total = 0, ftot = 0;
  uint32_t sink = 0;
  for (int it = 0; it < iters; ++it) {
    const uint8_t* base = src + static_cast<size_t>(it % 16) * stride * 16;
    if (fence) {
      const unsigned long long f0 = wall_clock64();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      ftot += wall_clock64() - f0;
    }
    const unsigned long long t0 = wall_clock64();
    u32x4 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (r < rows) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + r * stride) + threadIdx.x);
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (r < rows) sink ^= v[r].x ^ v[r].w;
    __builtin_amdgcn_s_waitcnt(0);
    total += wall_clock64() - t0;
  }
  if (threadIdx.x == 0) {
    ticks[0] = total;
    ticks[2] = ftot;
  }
  if (sink == 0x12345678u) ticks[1] = sink;
}

// the service's own access: volatile raw buffer loads (sc0 sc1), `waves`
// workgroups at once each on its own 1 KiB column, after a system acquire;
// then (stores = 1) 3 buffer stores of 1 KiB back and a wait for them
__global__ void fetch_svc(uint8_t* src, size_t stride, int rows, int iters, unsigned long long* ticks, int stores) {
  unsigned long long total = 0, stot = 0;
  uint32_t sink = 0;
  for (int it = 0; it < iters; ++it) {
    uint8_t* base = src + static_cast<size_t>(it % 16) * stride * 16 + blockIdx.x * 1024;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const unsigned long long t0 = wall_clock64();
    u32x4 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (r < rows) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + r * stride, 0, 0x7FFFFFFF, 0x00020000);
        v[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(threadIdx.x * 16), 0, static_cast<int>(0x80000000u));
      }
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (r < rows) acc ^= v[r];
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = wall_clock64();
    total += t1 - t0;
    if (stores) {
      for (int l = 0; l < 3; ++l) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + (12 + l) * stride, 0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(acc + static_cast<unsigned>(l), rs, static_cast<int>(threadIdx.x * 16), 0, 0);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      stot += wall_clock64() - t1;
    }
    sink ^= acc.x;
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    ticks[0] = total;
    ticks[2] = stot;
  }
  if (sink == 0x12345678u) ticks[1] = sink;
}

static hsa_status_t find_cpu(hsa_agent_t a, void* out) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(out) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

// one CPU store and load at p; false if the CPU has no mapping there
static bool cpu_can_touch(volatile uint64_t* p) {
  struct sigaction sa {}, old {};
  sa.sa_handler = on_segv;
  sigaction(SIGSEGV, &sa, &old);
  sigaction(SIGBUS, &sa, nullptr);
  bool ok = false;
  if (sigsetjmp(g_jb, 1) == 0) {
    *p = 0x1234;
    ok = *p == 0x1234;
  }
  sigaction(SIGSEGV, &old, nullptr);
  signal(SIGBUS, SIG_DFL);
  return ok;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  CK(hipSetDevice(0));
  {
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    uint8_t* hs = nullptr;
    const size_t stride = 4096;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hs), stride * 16 * 16, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(hs, 1, stride * 16 * 16);
    void* dhs = nullptr;
    CK(hipHostGetDevicePointer(&dhs, hs, 0));
    unsigned long long* tk = nullptr;
    CK(hipMalloc(reinterpret_cast<void**>(&tk), 32));
    for (int fence : {0, 1})
      for (int rows : {1, 4, 11, 16}) {
        const int iters = 2000;
        hipLaunchKernelGGL(fetch, dim3(1), dim3(64), 0, 0, static_cast<const uint8_t*>(dhs), stride, rows, iters, tk,
                           fence);
        CK(hipGetLastError());
        unsigned long long t[3] = {};
        CK(hipMemcpy(t, tk, 24, hipMemcpyDeviceToHost));
        std::printf("one wave, %2d x 1 KiB rows from pinned host memory, %s: %.2f us per fetch (fence %.2f us)\n", rows,
                    fence ? "after a system acquire" : "no fence", static_cast<double>(t[0]) / iters * 1e3 / khz,
                    static_cast<double>(t[2]) / iters * 1e3 / khz);
      }
  }
  {
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    uint8_t* hs = nullptr;
    const size_t stride = 4096;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hs), stride * 16 * 16, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(hs, 1, stride * 16 * 16);
    void* dhs = nullptr;
    CK(hipHostGetDevicePointer(&dhs, hs, 0));
    unsigned long long* tk = nullptr;
    CK(hipMalloc(reinterpret_cast<void**>(&tk), 32));
    for (int stores : {0, 1})
      for (int waves : {1, 4}) {
        const int iters = 2000, rows = 11;
        hipLaunchKernelGGL(fetch_svc, dim3(waves), dim3(64), 0, 0, static_cast<uint8_t*>(dhs), stride, rows, iters, tk,
                           stores);
        CK(hipGetLastError());
        unsigned long long t[3] = {};
        CK(hipMemcpy(t, tk, 24, hipMemcpyDeviceToHost));
        std::printf("service access, %d wave(s), 11 x 1 KiB volatile buffer loads: %.2f us per fetch; 3 stores + release: %.2f us\n",
                    waves, static_cast<double>(t[0]) / iters * 1e3 / khz, static_cast<double>(t[2]) / iters * 1e3 / khz);
      }
  }
  void* d = nullptr;
  CK(hipExtMallocWithFlags(&d, 1 << 20, hipDeviceMallocFinegrained));
  hipPointerAttribute_t at{};
  CK(hipPointerGetAttributes(&at, d));
  std::printf("fine-grained device memory %p: type %d, hostPointer %p, devicePointer %p\n", d,
              static_cast<int>(at.type), at.hostPointer, at.devicePointer);
  uint8_t* h = static_cast<uint8_t*>(at.hostPointer);
  if (!h) {
    // ask ROCr for CPU access to the allocation (large-BAR mapping), then
    // check that the CPU agent is now listed as an accessor
    hsa_agent_t cpu{};
    if (hsa_init() != HSA_STATUS_SUCCESS) return std::printf("hsa_init failed\n"), 1;
    hsa_iterate_agents(find_cpu, &cpu);
    const hsa_status_t st = hsa_amd_agents_allow_access(1, &cpu, nullptr, d);
    std::printf("hsa_amd_agents_allow_access(cpu): %d\n", static_cast<int>(st));
    hsa_amd_pointer_info_t pi{};
    pi.size = sizeof(pi);
    uint32_t na = 0;
    hsa_agent_t* acc = nullptr;
    if (hsa_amd_pointer_info(d, &pi, malloc, &na, &acc) != HSA_STATUS_SUCCESS) return std::printf("pointer_info failed\n"), 1;
    bool cpu_ok = false;
    for (uint32_t i = 0; i < na; ++i) cpu_ok |= acc[i].handle == cpu.handle;
    std::printf("pointer info: type %d, hostBaseAddress %p, agentBaseAddress %p, %u accessors, cpu %s\n",
                static_cast<int>(pi.type), pi.hostBaseAddress, pi.agentBaseAddress, na, cpu_ok ? "yes" : "no");
    h = static_cast<uint8_t*>(pi.hostBaseAddress);
    if (st != HSA_STATUS_SUCCESS || !h || !cpu_can_touch(reinterpret_cast<volatile uint64_t*>(h))) {
      std::printf("no host mapping: the host cannot write device memory directly\n");
      return 0;
    }
    std::printf("the CPU can store to and load from the allocation\n");
  }
  std::vector<uint8_t> src(45056, 7);
  // small copies (one 4 KiB k=11 call's blocks)
  for (int rep = 0; rep < 3; ++rep) {
    const double t0 = now_us();
    for (int i = 0; i < 1000; ++i) std::memcpy(h + (i & 7) * 65536, src.data(), src.size());
    const double t1 = now_us();
    std::printf("host -> device memory, 44 KiB memcpy: %.2f us each (%.2f GB/s)\n", (t1 - t0) / 1000,
                src.size() * 1000 / (t1 - t0) / 1e3);
  }
  // flag round trip: host writes the flag into device memory, kernel echoes into host memory
  unsigned long long* ack = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&ack), 64, hipHostMallocCoherent | hipHostMallocMapped));
  void* dack = nullptr;
  CK(hipHostGetDevicePointer(&dack, ack, 0));
  auto* flag = reinterpret_cast<volatile unsigned long long*>(h);
  *flag = 0;
  *ack = 0;
  const int n = 20000;
  hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, 0, static_cast<const unsigned long long*>(d),
                     static_cast<unsigned long long*>(dack), n);
  CK(hipGetLastError());
  double t0 = 0;
  for (int i = 1; i <= n; ++i) {
    if (i == 1001) t0 = now_us();
    __atomic_store_n(const_cast<unsigned long long*>(flag), static_cast<unsigned long long>(i), __ATOMIC_RELEASE);
    const double w = now_us();
    while (__atomic_load_n(ack, __ATOMIC_ACQUIRE) != static_cast<unsigned long long>(i))
      if (now_us() - w > 1e6) {
        std::printf("no echo at round %d\n", i);
        (void)hipDeviceSynchronize();  // the kernel leaves on its own spin bound
        return 1;
      }
  }
  std::printf("flag in device memory -> kernel echo in host memory: %.2f us round trip\n", (now_us() - t0) / (n - 1000));
  CK(hipDeviceSynchronize());
  // the same with the flag in host memory (what the service does today)
  unsigned long long* hflag = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&hflag), 64, hipHostMallocCoherent | hipHostMallocMapped));
  void* dflag = nullptr;
  CK(hipHostGetDevicePointer(&dflag, hflag, 0));
  *hflag = 0;
  *ack = 0;
  hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, 0, static_cast<const unsigned long long*>(dflag),
                     static_cast<unsigned long long*>(dack), n);
  CK(hipGetLastError());
  for (int i = 1; i <= n; ++i) {
    if (i == 1001) t0 = now_us();
    __atomic_store_n(hflag, static_cast<unsigned long long>(i), __ATOMIC_RELEASE);
    const double w = now_us();
    while (__atomic_load_n(ack, __ATOMIC_ACQUIRE) != static_cast<unsigned long long>(i))
      if (now_us() - w > 1e6) {
        std::printf("no echo at round %d\n", i);
        (void)hipDeviceSynchronize();  // the kernel leaves on its own spin bound
        return 1;
      }
  }
  std::printf("flag in host memory -> kernel echo in host memory: %.2f us round trip\n", (now_us() - t0) / (n - 1000));
  CK(hipDeviceSynchronize());
  return 0;
}
