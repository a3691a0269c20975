// Host side of the engine: scheme geometry, the codec object and every
// C-ABI entry point declared in include/ecwide.h. The arithmetic itself runs
// in the HIP kernels (ecw_kernels.hip); nothing here computes parity on the
// CPU, and every device call fails loudly (ECW_EDEVICE) without a GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <mutex>
#include <new>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/ecwide.h"
#include "ecw_gf.hpp"
#include "ecw_internal.hpp"
#include "ecw_tuning.hpp"

using namespace ecw;

namespace {

int ceil_div(int a, int b) { return (a + b - 1) / b; }

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Restores the caller's current device on scope exit (the C ABI must not
// change thread state behind the caller's back).
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int status_of(hipError_t e) { return e == hipSuccess ? ECW_OK : ECW_EDEVICE; }

}  // namespace

namespace svc {
bool busy(int device);  // the request service's resident kernel is (or may be) running on `device`
// Launch-path work is about to be queued on `device`: ask a running resident
// kernel to leave, so the work is not queued behind it on a shared hardware
// queue. hold: keep it from relaunching until release_hold (the caller waits
// for its own work in between).
void yield(int device, bool hold);
void release_hold(int device);
constexpr int kNotServed = 1;  // not an error: the caller takes the launch path
// serve one small request through the resident kernel (below), or kNotServed
int serve(ecw_codec* c, const uint8_t* const* data, int nsrc, uint8_t* const* parity, size_t len, bool xor_only);
// RAII form for the blocking host-memory entry points
struct Hold {
  int device;
  bool on;
  explicit Hold(int d, bool take = true) : device(d), on(take) {
    if (on) yield(d, true);
  }
  ~Hold() {
    if (on) release_hold(device);
  }
};
}  // namespace svc

// ---- deferred release of device resources -----------------------------------
// hipFree / hipHostFree / hipStreamDestroy can wait for the device to go idle,
// which it does not while the request service's resident kernel serves other
// threads (up to its lifetime). Codec teardown and staging growth therefore
// hand their old allocations to this list while the service runs; they are
// released by the next release that finds the service gone, and by the
// service itself whenever an epoch has left and before it launches the next
// (svc::Service::ensure_running), so the list holds at most what one epoch's
// lifetime (100 ms) of teardowns deferred.
namespace grave {

enum Kind { kDevice, kHost, kStream, kEvent };
struct Item {
  void* p;
  Kind kind;
  int device;
};
std::mutex mu;
std::vector<Item> items;

void release_now(const Item& it) {
  DeviceGuard g(it.device);
  switch (it.kind) {
    case kDevice: (void)hipFree(it.p); break;
    case kHost: (void)hipHostFree(it.p); break;
    case kStream: (void)hipStreamDestroy(static_cast<hipStream_t>(it.p)); break;
    case kEvent: (void)hipEventDestroy(static_cast<hipEvent_t>(it.p)); break;
  }
}

// release everything of devices whose service is not running (svc::busy takes
// the service's lock: never called with `mu` held, the service calls
// reap_device with its own lock held)
void reap() {
  std::vector<Item> all, keep, now;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (items.empty()) return;
    all.swap(items);
  }
  for (const Item& it : all) (svc::busy(it.device) ? keep : now).push_back(it);
  if (!keep.empty()) {
    std::lock_guard<std::mutex> lk(mu);
    items.insert(items.end(), keep.begin(), keep.end());
  }
  for (const Item& it : now) release_now(it);
}

// release everything of `device`: its service has left and is not relaunched
// meanwhile (the caller holds the service's lock)
void reap_device(int device) {
  std::vector<Item> now;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto mid = std::stable_partition(items.begin(), items.end(), [&](const Item& it) { return it.device != device; });
    now.assign(mid, items.end());
    items.erase(mid, items.end());
  }
  for (const Item& it : now) release_now(it);
}

// release `p` now, or later if the service on its device is running
void release(void* p, Kind kind, int device) {
  if (!p) return;
  if (svc::busy(device)) {
    std::lock_guard<std::mutex> lk(mu);
    items.push_back(Item{p, kind, device});
    return;
  }
  release_now(Item{p, kind, device});
  reap();
}

}  // namespace grave

// Ticket counters of ticket-ordered encode launches: a ring of 8-byte device
// counters, one per launch. The host zeroes the slot's counter on the launch's
// stream right before the launch and records an event after it; a slot is
// reused only once that event has completed (the host waits for it in the rare
// case that kTicketSlots launches later it has not). So no two launches share
// a counter whatever their streams are (hipStreamPerThread from several
// threads, a destroyed stream's handle reused, ...). Launches on a capturing
// stream take the launch windows instead (no counter in a graph).
constexpr int kTicketSlots = 64;
struct TicketRing {
  unsigned long long* d = nullptr;
  hipEvent_t ev[kTicketSlots] = {};
  bool used[kTicketSlots] = {};
  unsigned next = 0;
};

std::atomic<unsigned long long> g_codec_serial{0};

struct ecw_codec {
  ecw_scheme scheme{};
  ecw_codec_info info{};
  int device = 0;
  int xori_mode = ECW_XORI_XOR;
  unsigned long long serial = ++g_codec_serial;  // unique per codec (the service's LDS table cache key)
  std::vector<uint8_t> matrix;        // m x edn, row-major (encodeMatrix)
  std::vector<uint8_t> gftbl;         // 32 * edn * m (encodeGftbl, ISA-L layout)
  std::vector<uint8_t> dtbl, pdtbl;   // decode / partial-decode tables (all ones)
  std::vector<std::vector<uint8_t>> pass_img;  // packed device tables per pass of <= 16 rows
  bool xor_row = false;               // m == 1 and every coefficient 1: the global parity is a plain XOR

  std::mutex mu;                      // guards everything below
  bool dev_ready = false;
  std::vector<void*> d_pass;          // device copies of pass_img
  bool xori_called = false;           // per-codec replacement of the static `flag`
  // staging for the host-memory entry points
  hipStream_t stream = nullptr;
  struct HostPipe* pipe = nullptr;    // streams/events of the host-memory pipeline
  uint8_t* d_stage = nullptr;
  size_t stage_bytes = 0;
  uint8_t* h_stage = nullptr;         // pinned host staging of the small-block path
  size_t h_stage_bytes = 0;

  std::mutex ticket_mu;               // guards `tickets`
  TicketRing tickets;

  ~ecw_codec() {
    // every allocation goes through grave::release: freed now, or once the
    // request service on this device has left (a destroy never waits for it)
    for (int i = 0; i < kTicketSlots; ++i) grave::release(tickets.ev[i], grave::kEvent, device);
    grave::release(tickets.d, grave::kDevice, device);
    for (void* p : d_pass) grave::release(p, grave::kDevice, device);
    grave::release(d_stage, grave::kDevice, device);
    grave::release(h_stage, grave::kHost, device);
    grave::release(stream, grave::kStream, device);
    destroy_pipe();
  }
  void destroy_pipe();

  bool has_local() const { return info.code_type == 'C' || info.code_type == 'L'; }
  int k() const { return info.encode_data_num; }
  int m() const { return info.global_num; }
  // a multi-node codec encodes one data group: one local parity over all its rows
  int groups() const { return has_local() ? (info.multinode ? 1 : info.group_num) : 0; }
  int r() const { return info.multinode ? info.encode_data_num : info.group_data_num; }

  // lazily upload the packed tables (first device call)
  int ensure_device() {
    if (dev_ready) return ECW_OK;
    DeviceGuard g(device);
    if (!g.ok) return ECW_EDEVICE;
    auto fail = [&](int st) {  // leave nothing half-initialised: a later call retries from scratch
      for (void* q : d_pass) grave::release(q, grave::kDevice, device);
      d_pass.clear();
      return st;
    };
    for (const auto& img : pass_img) {
      void* p = nullptr;
      if (hipMalloc(&p, img.size()) != hipSuccess) return fail(ECW_ENOMEM);
      d_pass.push_back(p);
      if (hipMemcpy(p, img.data(), img.size(), hipMemcpyHostToDevice) != hipSuccess) return fail(ECW_EDEVICE);
    }
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return fail(ECW_EDEVICE);
    dev_ready = true;
    return ECW_OK;
  }

  // A zeroed counter for one ticket-ordered launch on stream s (caller holds
  // ticket_mu and calls ticket_done after the launch), or null: the encode
  // then runs in launch windows.
  unsigned long long* ticket_take(hipStream_t s, int* slot) {
    *slot = -1;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
      (void)hipGetLastError();
      return nullptr;
    }
    TicketRing& t = tickets;
    if (!t.d) {
      void* p = nullptr;
      if (hipMalloc(&p, sizeof(unsigned long long) * kTicketSlots) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
      }
      t.d = static_cast<unsigned long long*>(p);
    }
    const int i = static_cast<int>(t.next++ % kTicketSlots);
    if (!t.ev[i] && hipEventCreateWithFlags(&t.ev[i], hipEventDisableTiming) != hipSuccess) {
      t.ev[i] = nullptr;
      (void)hipGetLastError();
      return nullptr;
    }
    if (t.used[i] && hipEventSynchronize(t.ev[i]) != hipSuccess) {  // launched kTicketSlots ago and still running
      (void)hipGetLastError();
      return nullptr;
    }
    t.used[i] = false;
    if (hipMemsetAsync(t.d + i, 0, sizeof(unsigned long long), s) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    *slot = i;
    return t.d + i;
  }
  void ticket_done(int slot, hipStream_t s) {
    if (slot < 0) return;
    if (hipEventRecord(tickets.ev[slot], s) == hipSuccess) {
      tickets.used[slot] = true;
    } else {  // no event to wait for: make sure the launch is over before the slot is reused
      (void)hipGetLastError();
      (void)hipStreamSynchronize(s);
    }
  }

  int ensure_stage(size_t bytes) {
    if (stage_bytes >= bytes) return ECW_OK;
    grave::release(d_stage, grave::kDevice, device);
    d_stage = nullptr;
    stage_bytes = 0;
    if (hipMalloc(&d_stage, bytes) != hipSuccess) return ECW_ENOMEM;
    stage_bytes = bytes;
    return ECW_OK;
  }
  int ensure_host_stage(size_t bytes) {
    if (h_stage_bytes >= bytes) return ECW_OK;
    grave::release(h_stage, grave::kHost, device);
    h_stage = nullptr;
    h_stage_bytes = 0;
    // coherent: the zero-copy path (encode_stripes_packed) has kernels read and
    // write this memory directly
    if (hipHostMalloc(reinterpret_cast<void**>(&h_stage), bytes, hipHostMallocCoherent) != hipSuccess)
      return ECW_ENOMEM;
    h_stage_bytes = bytes;
    return ECW_OK;
  }
};

namespace {

int local_mode_of(const ecw_codec* c) {
  if (!c->has_local()) return kLocalNone;
  return c->info.local_mode == ECW_LOCAL_LITERAL ? kLocalZero : kLocalXor;
}

// Encode through the kernels. `src(j)` / `dst(o)` give device row pointers for
// pointer mode; for slab mode `slab` is set. Handles m > 8 (several passes),
// m == 0 and > kMaxPtrLocals locals (XOR-reduce launches per group).
struct EncodeTarget {
  const uint8_t* const* src = nullptr;  // pointer mode
  uint8_t* const* dst = nullptr;
  const SlabRows* slab = nullptr;       // slab mode
  int stripes = 1;
};

// Pointer-mode rows that are really a strided layout (data blocks at one
// stride, parity blocks -- globals then locals -- at one stride of their own,
// e.g. two [k, B] / [m+g, B] tensors): describe them as a one-stripe slab, so
// the encode takes the slab kernel (asm tile) instead of the pointer kernel.
bool as_slab(const uint8_t* const* src, int k, uint8_t* const* dst, int np, SlabRows* out) {
  auto at = [](const void* p) { return static_cast<uint64_t>(reinterpret_cast<uintptr_t>(p)); };
  if (k < 2 || np < 1 || at(src[1]) <= at(src[0])) return false;
  const uint64_t bs = at(src[1]) - at(src[0]);
  for (int j = 2; j < k; ++j)
    if (at(src[j]) != at(src[0]) + j * bs) return false;
  uint64_t pbs = bs;
  if (np > 1) {
    if (at(dst[1]) <= at(dst[0])) return false;
    pbs = at(dst[1]) - at(dst[0]);
    for (int i = 2; i < np; ++i)
      if (at(dst[i]) != at(dst[0]) + i * pbs) return false;
  }
  *out = SlabRows{src[0], bs, 0, dst[0], pbs, 0};
  return true;
}

int run_encode(ecw_codec* c, const EncodeTarget& t0, size_t len, hipStream_t s) {
  const int k = c->k(), m = c->m(), ng = c->groups();
  svc::yield(c->device, false);  // not queued behind the request service's resident kernel
  EncodeTarget t = t0;
  SlabRows strided;
  if (!t.slab && t.stripes == 1 && as_slab(t.src, k, t.dst, c->info.parity_num, &strided)) t.slab = &strided;
  const int lmode = local_mode_of(c);
  if (len == 0 || t.stripes == 0) return ECW_OK;
  EncodeGeom g{};
  g.len = len;
  g.tiles = (len + kTileBytes - 1) / kTileBytes;
  g.stripes = t.stripes;
  g.k = k;
  g.r = c->has_local() ? c->r() : k;
  g.groups = ng;
  g.m = m;
  const int npass = (m + kMaxPassRows - 1) / kMaxPassRows;
  // locals ride in the first pass when they fit in the pointer-mode args
  const bool locals_inline = lmode != kLocalNone && m > 0 && (t.slab || ng <= kMaxPtrLocals);
  for (int q = 0; q < npass; ++q) {
    g.row0 = q * kMaxPassRows;
    g.nrows = std::min(kMaxPassRows, m - g.row0);
    g.local_mode = (q == 0 && locals_inline) ? lmode : kLocalNone;
    hipError_t e;
    if (t.slab) {
      if (encode_uses_ticket(g.tiles * static_cast<uint64_t>(t.stripes), k)) {
        std::lock_guard<std::mutex> lk(c->ticket_mu);
        int slot;
        unsigned long long* tk = c->ticket_take(s, &slot);
        e = launch_encode_slab(*t.slab, g, c->d_pass[q], s, tk);
        c->ticket_done(slot, s);
      } else {
        e = launch_encode_slab(*t.slab, g, c->d_pass[q], s, nullptr);
      }
    } else {
      PtrRows rows;
      std::memset(&rows, 0, sizeof rows);
      for (int j = 0; j < k; ++j) rows.src[j] = t.src[j];
      for (int l = 0; l < g.nrows; ++l) rows.dst[l] = t.dst[g.row0 + l];
      if (g.local_mode != kLocalNone)
        for (int i = 0; i < ng; ++i) rows.dst[g.nrows + i] = t.dst[m + i];
      if (encode_uses_ticket(g.tiles, k)) {
        std::lock_guard<std::mutex> lk(c->ticket_mu);
        int slot;
        unsigned long long* tk = c->ticket_take(s, &slot);
        e = launch_encode_ptr(rows, g, c->d_pass[q], s, tk);
        c->ticket_done(slot, s);
      } else {
        e = launch_encode_ptr(rows, g, c->d_pass[q], s, nullptr);
      }
    }
    if (e != hipSuccess) return ECW_EDEVICE;
  }
  if (lmode != kLocalNone && !locals_inline) {
    // m == 0 or very many local groups: one XOR reduce per group
    for (int i = 0; i < ng; ++i) {
      const int j0 = i * g.r, n = std::min(g.r, k - j0);
      XorGeom xg{len, (len + kTileBytes - 1) / kTileBytes, t.stripes, n};
      hipError_t e;
      if (t.slab) {
        XorSlab xs;
        std::memset(&xs, 0, sizeof xs);
        xs.base = t.slab->base;
        xs.bstride = t.slab->bstride;
        xs.sstride = t.slab->sstride;
        xs.out = t.slab->pbase + static_cast<uint64_t>(m + i) * t.slab->pbstride;
        xs.ostride = t.slab->psstride;
        for (int u = 0; u < n; ++u) xs.idx[u] = j0 + u;
        if (lmode == kLocalZero) {
          for (int st = 0; st < t.stripes; ++st)
            if (hipMemsetAsync(xs.out + st * xs.ostride, 0, len, s) != hipSuccess) return ECW_EDEVICE;
          continue;
        }
        e = launch_xor_slab(xs, xg, s);
      } else {
        if (lmode == kLocalZero) {
          if (hipMemsetAsync(t.dst[m + i], 0, len, s) != hipSuccess) return ECW_EDEVICE;
          continue;
        }
        XorPtr xp;
        std::memset(&xp, 0, sizeof xp);
        for (int u = 0; u < n; ++u) xp.src[u] = t.src[j0 + u];
        xp.dst = t.dst[m + i];
        e = launch_xor_ptr(xp, xg, s);
      }
      if (e != hipSuccess) return ECW_EDEVICE;
    }
  }
  return ECW_OK;
}

int run_xor_ptr(const uint8_t* const* src, int n, uint8_t* dst, size_t len, hipStream_t s) {
  if (n < 1 || n > kMaxSrc) return ECW_EINVAL;
  if (len == 0) return ECW_OK;
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) svc::yield(dev, false);
  XorPtr xp;
  std::memset(&xp, 0, sizeof xp);
  for (int i = 0; i < n; ++i) xp.src[i] = src[i];
  xp.dst = dst;
  XorGeom xg{len, (len + kTileBytes - 1) / kTileBytes, 1, n};
  return status_of(launch_xor_ptr(xp, xg, s));
}

bool check_len(size_t len) { return len <= 0xFFFFFFF0ull; }

// The `rows` blocks of `stripes` stripes at s * sstride + j * bstride, each
// `len` bytes, never overlap: stripes one after another (stripe-major), or
// the stripes interleaved inside every block (block-major: e.g. the column
// pieces of one block-layout stripe taken as stripes of their own).
bool disjoint_units(size_t bstride, size_t sstride, size_t rows, int stripes, size_t len) {
  if (stripes <= 1 || len == 0) return true;
  const size_t S = static_cast<size_t>(stripes);
  if (sstride >= (rows - 1) * bstride + len) return true;
  return sstride >= len && (rows <= 1 || bstride >= (S - 1) * sstride + len);
}

template <class P>
bool all_aligned(P const* ptrs, int n) {
  for (int i = 0; i < n; ++i)
    if (!ptrs[i] || !aligned16(ptrs[i])) return false;
  return true;
}

// ---- launch schedule (ecw_set_schedule) ------------------------------------
constexpr int kWindowLog2p = 11, kWindowWidth = 64;  // a window with one field given: the other's default

bool skew_built(int k) {
  for (int s : kXorSkews)
    if (s == k) return true;
  return false;
}

// every field -1 or in range; windows completed with the defaults
bool normalise(Schedule& s) {
  auto in = [](int v, int lo, int hi) { return v == -1 || (v >= lo && v <= hi); };
  if (!(s.xor_skew == -1 || skew_built(s.xor_skew)) || !in(s.xor_order, 0, 1) || !in(s.xcd_remap, 0, 1) ||
      !in(s.xor_log2p, 4, 24) || !in(s.enc_log2p, 4, 24) || !in(s.xor_width, 0, 1 << 24) ||
      !in(s.enc_width, 0, 1 << 24))
    return false;
  for (auto w : {std::make_pair(&s.xor_log2p, &s.xor_width), std::make_pair(&s.enc_log2p, &s.enc_width)}) {
    if (*w.first == -1 && *w.second > 0) *w.first = kWindowLog2p;
    if (*w.first != -1 && *w.second == -1) *w.second = kWindowWidth;
  }
  return true;
}

// The environment's overrides, read once (tuning runs that predate the API):
// ECW_XOR_SCHED = "K,ORDER[,LOG2P,W]" names the whole XOR schedule (no window
// unless given), ECW_WRITE_WINDOW = off | on | "LOG2P,W" the encode's window,
// ECW_XCD_REMAP = 0 | 1 the tile order of both. A malformed or out-of-range
// value is reported on stderr and ignored.
Schedule schedule_from_env() {
  Schedule s{-1, -1, -1, -1, -1, -1, -1};
  auto warn = [](const char* var, const char* v) {
    std::fprintf(stderr, "libecwide: ignoring %s=%s (out of range or not built)\n", var, v);
  };
  if (const char* e = std::getenv("ECW_XOR_SCHED")) {
    Schedule t = s;
    int k = 1;
    unsigned o = 0, lp = 0, w = 0;
    const int got = std::sscanf(e, "%d,%u,%u,%u", &k, &o, &lp, &w);
    if (got >= 1) {
      t.xor_skew = k;
      t.xor_width = 0;
      if (got >= 2) t.xor_order = static_cast<int>(o);
      if (got >= 4) {
        t.xor_log2p = static_cast<int>(lp);
        t.xor_width = static_cast<int>(w);
      }
    }
    if (got >= 1 && got != 3 && normalise(t))
      s = t;
    else
      warn("ECW_XOR_SCHED", e);
  }
  if (const char* e = std::getenv("ECW_WRITE_WINDOW")) {
    Schedule t = s;
    unsigned a = 0, b = 0;
    if (!std::strcmp(e, "off") || !std::strcmp(e, "0")) {
      t.enc_width = 0;
    } else if (!std::strcmp(e, "on")) {
      t.enc_log2p = kWindowLog2p;
      t.enc_width = kWindowWidth;
    } else if (std::sscanf(e, "%u,%u", &a, &b) == 2) {
      t.enc_log2p = static_cast<int>(a);
      t.enc_width = static_cast<int>(b);
    } else if (e[0]) {
      t.enc_log2p = -2;  // rejected below
    }
    if (normalise(t))
      s = t;
    else
      warn("ECW_WRITE_WINDOW", e);
  }
  if (const char* e = std::getenv("ECW_XCD_REMAP")) {
    if (e[0] == '0' || e[0] == '1')
      s.xcd_remap = e[0] - '0';
    else if (e[0])
      warn("ECW_XCD_REMAP", e);
  }
  return s;
}

std::mutex g_sched_mu;
Schedule g_sched;
bool g_sched_init = false;

Schedule& schedule_locked() {
  if (!g_sched_init) {
    g_sched = schedule_from_env();
    g_sched_init = true;
  }
  return g_sched;
}

// ---- NUMA-local pinned host staging (ecw_host_alloc) ------------------------
// The GPU's NUMA node from sysfs (-1: unknown, e.g. a host without NUMA).
int device_numa_node(int device) {
  char bdf[64] = {};
  if (hipDeviceGetPCIBusId(bdf, sizeof bdf, device) != hipSuccess) return -1;
  for (char* p = bdf; *p; ++p) *p = static_cast<char>(std::tolower(static_cast<unsigned char>(*p)));
  std::ifstream f(std::string("/sys/bus/pci/devices/") + bdf + "/numa_node");
  int node = -1;
  if (!(f >> node)) return -1;
  return node;
}

// Node of the pages of [p, p + n) by sampling up to 64 of them (move_pages
// with no target nodes only reports): the node they all sit on, -1 if they
// are spread or the kernel does not tell.
int pages_node(void* p, size_t n) {
  const size_t pg = 4096, npages = (n + pg - 1) / pg, samples = std::min<size_t>(64, npages);
  std::vector<void*> pages(samples);
  std::vector<int> status(samples, -1);
  for (size_t i = 0; i < samples; ++i)
    pages[i] = static_cast<char*>(p) + (npages * i / samples) * pg;
  if (syscall(SYS_move_pages, 0, samples, pages.data(), nullptr, status.data(), 0) != 0) return -1;
  for (size_t i = 1; i < samples; ++i)
    if (status[i] != status[0]) return -1;
  return status[0] >= 0 ? status[0] : -1;
}

std::mutex g_host_mu;
std::map<void*, size_t> g_host_allocs;  // ecw_host_alloc'd regions (mapped bytes)

}  // namespace

Schedule ecw::current_schedule() {
  std::lock_guard<std::mutex> lk(g_sched_mu);
  return schedule_locked();
}

// =====================================================================
extern "C" {

int ecw_abi_version(void) { return ECW_ABI_VERSION; }

int ecw_set_schedule(const ecw_schedule* in) {
  Schedule s{-1, -1, -1, -1, -1, -1, -1};
  if (in)
    s = Schedule{in->xor_skew,         in->xor_order,        in->xor_window_log2p, in->xor_window_width,
                 in->enc_window_log2p, in->enc_window_width, in->xcd_remap};
  if (!normalise(s)) return ECW_EINVAL;
  std::lock_guard<std::mutex> lk(g_sched_mu);
  schedule_locked() = s;
  return ECW_OK;
}

int ecw_get_schedule(ecw_schedule* out) {
  if (!out) return ECW_EINVAL;
  const Schedule s = current_schedule();
  *out = ecw_schedule{s.xor_skew, s.xor_order, s.xor_log2p, s.xor_width, s.enc_log2p, s.enc_width, s.xcd_remap};
  return ECW_OK;
}

const char* ecw_status_string(int status) {
  switch (status) {
    case ECW_OK: return "ok";
    case ECW_EINVAL: return "invalid argument";
    case ECW_ENOMEM: return "out of memory";
    case ECW_EDEVICE: return "HIP device error";
    case ECW_EALIGN: return "pointer or stride not 16-byte aligned";
    case ECW_EUNSUPPORTED: return "unsupported operation";
    case ECW_EPARSE: return "malformed scheme.ini";
    case ECW_EIO: return "file could not be read";
    default: return "unknown status";
  }
}

int ecw_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// CodingScheme ctors (CodingScheme.java:22-48)
int ecw_scheme_init(ecw_scheme* out, char code_type, int k, int m, int group_data_num, size_t chunk_size) {
  if (!out) return ECW_EINVAL;
  if (code_type != 'R' && code_type != 'T' && code_type != 'L' && code_type != 'C') return ECW_EINVAL;
  if (k < 1 || m < 0 || k + m > 256) return ECW_EINVAL;
  ecw_scheme s{};
  s.code_type = code_type;
  s.k = k;
  s.global_parity_num = m;
  s.chunk_size = chunk_size;
  s.chunk_size_bits = -1;
  s.group_data_num = -1;
  if (code_type == 'T') {
    if (m < 1) return ECW_EINVAL;
    s.rack_num = ceil_div(k, m) + 1;
    s.rack_nodes_num = m;
  } else if (code_type == 'L' || code_type == 'C') {
    if (group_data_num < 1) return ECW_EINVAL;
    s.group_data_num = group_data_num;
    s.group_num = ceil_div(k, group_data_num);
    if (code_type == 'C') {
      s.rack_nodes_num = m + 1;
      s.rack_num = ceil_div(k + s.group_num, m + 1) + 1;
    } else {
      s.rack_nodes_num = s.rack_num = -1;
    }
  }
  *out = s;
  return ECW_OK;
}

// CodingScheme.getFromConfig (CodingScheme.java:66-113): "key = value" lines;
// codeType CL/LRC/TL, anything else RS; the other values parseInt'ed.
// Blank lines are skipped (the Java would throw on them); any other line
// without '=' or with a non-integer value is ECW_EPARSE.
int ecw_scheme_from_ini_text(const char* text, ecw_scheme* out) {
  if (!text || !out) return ECW_EINVAL;
  std::istringstream in(text);
  std::string line;
  std::map<std::string, long long> kv;
  char code = 'C';
  auto trim = [](std::string x) {
    size_t a = 0, b = x.size();
    while (a < b && std::isspace(static_cast<unsigned char>(x[a]))) ++a;
    while (b > a && std::isspace(static_cast<unsigned char>(x[b - 1]))) --b;
    return x.substr(a, b - a);
  };
  while (std::getline(in, line)) {
    if (trim(line).empty()) continue;
    const size_t eq = line.find('=');
    if (eq == std::string::npos) return ECW_EPARSE;
    const std::string key = trim(line.substr(0, eq));
    std::string val = trim(line.substr(eq + 1));
    const size_t eq2 = val.find('=');  // Java split("=")[1] drops the rest
    if (eq2 != std::string::npos) val = trim(val.substr(0, eq2));
    if (key == "codeType") {
      code = val == "CL" ? 'C' : val == "LRC" ? 'L' : val == "TL" ? 'T' : 'R';
      continue;
    }
    char* end = nullptr;
    errno = 0;
    const long long v = std::strtoll(val.c_str(), &end, 10);
    if (val.empty() || *end != '\0' || errno || v < INT32_MIN || v > INT32_MAX) return ECW_EPARSE;
    kv[key] = v;
  }
  for (const char* key : {"k", "chunkSizeBits", "globalParityNum"})
    if (!kv.count(key)) return ECW_EPARSE;
  if ((code == 'C' || code == 'L') && !kv.count("groupDataNum")) return ECW_EPARSE;
  const long long bits = kv["chunkSizeBits"];
  if (bits < 0 || bits > 31) return ECW_EPARSE;  // Java: 1 << bits on an int
  const int r = (code == 'C' || code == 'L') ? static_cast<int>(kv["groupDataNum"]) : -1;
  const int st = ecw_scheme_init(out, code, static_cast<int>(kv["k"]), static_cast<int>(kv["globalParityNum"]),
                                 r, static_cast<size_t>(1) << bits);
  if (st == ECW_OK) out->chunk_size_bits = static_cast<int>(bits);
  return st;
}

int ecw_scheme_from_ini(const char* path, ecw_scheme* out) {
  if (!path || !out) return ECW_EINVAL;
  std::ifstream f(path);
  if (!f) return ECW_EIO;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  return ecw_scheme_from_ini_text(text.c_str(), out);
}

// NativeCodec ctors (NativeCodec.java:20-109) and the four init natives
// (NativeCodec.cc:12-135).
int ecw_codec_create(const ecw_scheme* sch, int node_index, int multinode, int local_mode, int device,
                     ecw_codec** out) {
  if (!sch || !out) return ECW_EINVAL;
  *out = nullptr;
  if (local_mode != ECW_LOCAL_XOR && local_mode != ECW_LOCAL_LITERAL) return ECW_EINVAL;
  const char t = sch->code_type;
  const int k = sch->k, m = sch->global_parity_num, r = sch->group_data_num;
  if (k < 1 || m < 0 || k + m > 256) return ECW_EINVAL;
  if ((t == 'C' || t == 'L') && (r < 1 || sch->rack_nodes_num == 0)) return ECW_EINVAL;
  if ((t == 'T' || t == 'C') && node_index < 1) return ECW_EINVAL;
  if (t == 'L' && node_index < 1) return ECW_EINVAL;
  if (multinode && t != 'C') return ECW_EINVAL;
  ecw_codec* c = new (std::nothrow) ecw_codec();
  if (!c) return ECW_ENOMEM;
  c->scheme = *sch;
  c->device = device;
  ecw_codec_info& in = c->info;
  in.code_type = t;
  in.node_index = node_index;
  in.multinode = multinode ? 1 : 0;
  in.local_mode = local_mode;
  in.global_num = m;
  in.chunk_size = sch->chunk_size;
  in.group_num = sch->group_num;
  in.group_data_num = sch->group_data_num;
  if (t == 'R') {
    in.decode_data_num = in.encode_data_num = k;
  } else if (t == 'T') {
    const int racks = ceil_div(k, m) + 1, rn = m, rack = (node_index - 1) / rn;
    in.encode_data_num = k;
    in.partial_decode_num = rack == racks - 2 ? ((k - rack * rn) - 1) % rn + 1 : rn;
    in.decode_data_num = in.partial_decode_num - 1 + racks - 1;
  } else if (t == 'L') {
    in.encode_data_num = k;
    const int gi = (node_index - 1) / r;
    in.decode_data_num = gi == r - 1 ? (k - 1) % r + 1 : r;  // sic: NativeCodec.java:63
  } else {
    in.encode_data_num = multinode ? (node_index == 1 ? (k - 1) % r + 1 : r) : k;
    const int rn = sch->rack_nodes_num, rack = (node_index - 1) / rn;
    in.partial_decode_num = rack != sch->rack_num - 2 ? rn : ((k - 1) % r + 1) % rn + 1;
    in.rack_per_group = ceil_div(r + 1, rn);
    in.decode_data_num = in.partial_decode_num - 1 + in.rack_per_group - 1;
  }
  in.parity_num = m + ((t == 'C' || t == 'L') ? (multinode ? 1 : in.group_num) : 0);
  const int edn = in.encode_data_num;
  if (multinode) {
    // Multi-node CL encode (ECTaskProcessor.java:267-291, paper p.240 Fig. 6):
    // node i (1-based) holds data group g-i ("data group 1 - l => node l | ...
    // | 1", NativeCodec.cc:47) and computes the partial global parities over
    // that group's columns of the stripe's Cauchy matrix, plus the group's
    // XOR local parity; xorIntemediate merges partials along the chain. The
    // reference slices a Cauchy matrix of the GROUP size at a misaligned
    // offset (NativeCodec.cc:31,46-58: out of bounds for most nodes), so its
    // partials do not add up to the single-node parities; this implements
    // the intended columns, whose XOR over all nodes equals encodeData's G.
    const int c0 = (sch->group_num - node_index) * r;
    if (c0 < 0) {
      delete c;
      return ECW_EINVAL;
    }
    const std::vector<uint8_t> full = cauchy_parity_rows(k, m);
    c->matrix.resize(static_cast<size_t>(edn) * m);
    for (int l = 0; l < m; ++l)
      for (int j = 0; j < edn; ++j) c->matrix[static_cast<size_t>(l) * edn + j] = full[static_cast<size_t>(l) * k + c0 + j];
  } else {
    c->matrix = cauchy_parity_rows(edn, m);
  }
  c->gftbl = isal_tables(edn, m, c->matrix.data());
  std::vector<uint8_t> ones(256, 1);
  c->dtbl = isal_tables(in.decode_data_num, 1, ones.data());
  if (t == 'T' || t == 'C') c->pdtbl = isal_tables(in.partial_decode_num, 1, ones.data());
  for (int row0 = 0; row0 < m; row0 += kMaxPassRows)
    c->pass_img.push_back(packed_pass_tables(c->matrix.data(), edn, row0, std::min(kMaxPassRows, m - row0)));
  *out = c;
  return ECW_OK;
}

void ecw_codec_destroy(ecw_codec* codec) {
  delete codec;
  grave::reap();  // what earlier teardowns deferred, if the service has left since
}

int ecw_matrix_codec_create(const uint8_t* matrix, int k, int rows, int device, ecw_codec** out) {
  if (!matrix || !out || k < 1 || rows < 1 || k > kMaxSrc || rows > 255) return ECW_EINVAL;
  *out = nullptr;
  ecw_codec* c = new (std::nothrow) ecw_codec();
  if (!c) return ECW_ENOMEM;
  c->device = device;
  c->scheme.code_type = 'M';
  c->scheme.k = k;
  c->scheme.global_parity_num = rows;
  c->scheme.group_data_num = -1;
  c->scheme.chunk_size_bits = -1;
  ecw_codec_info& in = c->info;
  in.code_type = 'M';
  in.node_index = 1;
  in.encode_data_num = k;
  in.decode_data_num = k;
  in.global_num = rows;
  in.group_data_num = -1;
  in.parity_num = rows;
  c->matrix.assign(matrix, matrix + static_cast<size_t>(k) * rows);
  c->xor_row = rows == 1 && std::all_of(c->matrix.begin(), c->matrix.end(), [](uint8_t v) { return v == 1; });
  c->gftbl = isal_tables(k, rows, c->matrix.data());
  std::vector<uint8_t> ones(256, 1);
  c->dtbl = isal_tables(k, 1, ones.data());
  for (int row0 = 0; row0 < rows; row0 += kMaxPassRows)
    c->pass_img.push_back(packed_pass_tables(c->matrix.data(), k, row0, std::min(kMaxPassRows, rows - row0)));
  *out = c;
  return ECW_OK;
}

int ecw_codec_get_info(const ecw_codec* c, ecw_codec_info* out) {
  if (!c || !out) return ECW_EINVAL;
  *out = c->info;
  return ECW_OK;
}

int ecw_codec_set_xori_mode(ecw_codec* c, int mode) {
  if (!c || (mode != ECW_XORI_XOR && mode != ECW_XORI_LITERAL)) return ECW_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  c->xori_mode = mode;
  return ECW_OK;
}

static int copy_out(const std::vector<uint8_t>& v, uint8_t* out, size_t len) {
  if (!out || len != v.size()) return ECW_EINVAL;
  if (len) std::memcpy(out, v.data(), len);
  return ECW_OK;
}
int ecw_codec_encode_matrix(const ecw_codec* c, uint8_t* out, size_t len) {
  return c ? copy_out(c->matrix, out, len) : ECW_EINVAL;
}
int ecw_codec_encode_gftbl(const ecw_codec* c, uint8_t* out, size_t len) {
  return c ? copy_out(c->gftbl, out, len) : ECW_EINVAL;
}
int ecw_codec_decode_gftbl(const ecw_codec* c, uint8_t* out, size_t len) {
  return c ? copy_out(c->dtbl, out, len) : ECW_EINVAL;
}
int ecw_codec_partial_decode_gftbl(const ecw_codec* c, uint8_t* out, size_t len) {
  return c ? copy_out(c->pdtbl, out, len) : ECW_EINVAL;
}

// ---- device entry points ----------------------------------------------------
int ecw_encode_dev(ecw_codec* c, const uint8_t* const* d_data, uint8_t* const* d_parity, size_t len,
                   void* stream) {
  if (!c || !d_data || !d_parity || !check_len(len)) return ECW_EINVAL;
  const int k = c->k(), np = c->info.parity_num;
  if (!all_aligned(d_data, k) || !all_aligned(d_parity, np)) return ECW_EALIGN;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    const int st = c->ensure_device();
    if (st) return st;
  }
  DeviceGuard g(c->device);
  if (!g.ok) return ECW_EDEVICE;
  EncodeTarget t;
  t.src = d_data;
  t.dst = d_parity;
  return run_encode(c, t, len, static_cast<hipStream_t>(stream));
}

int ecw_encode_ptrs_dev(ecw_codec* c, int stripes, const uint8_t* const* d_data_ptrs, uint8_t* const* d_parity_ptrs,
                        size_t len, void* stream) {
  if (!c || !d_data_ptrs || !d_parity_ptrs || stripes < 0 || !check_len(len)) return ECW_EINVAL;
  if (reinterpret_cast<uintptr_t>(d_data_ptrs) % 8 || reinterpret_cast<uintptr_t>(d_parity_ptrs) % 8)
    return ECW_EALIGN;
  const int k = c->k(), m = c->m(), ng = c->groups();
  if (m < 1 && local_mode_of(c) != kLocalNone) return ECW_EUNSUPPORTED;  // locals ride in a global-row pass
  if (len == 0 || stripes == 0 || m < 1) return ECW_OK;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    const int st = c->ensure_device();
    if (st) return st;
  }
  DeviceGuard g(c->device);
  if (!g.ok) return ECW_EDEVICE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  EncodeGeom eg{};
  eg.len = len;
  eg.tiles = (len + kTileBytes - 1) / kTileBytes;
  eg.stripes = stripes;
  eg.k = k;
  eg.r = c->has_local() ? c->r() : k;
  eg.groups = ng;
  eg.m = m;
  const PtrTabRows rows{d_data_ptrs, d_parity_ptrs, c->info.parity_num};
  const int npass = (m + kMaxPassRows - 1) / kMaxPassRows;
  svc::yield(c->device, false);
  for (int q = 0; q < npass; ++q) {
    eg.row0 = q * kMaxPassRows;
    eg.nrows = std::min(kMaxPassRows, m - eg.row0);
    eg.local_mode = q == 0 ? local_mode_of(c) : kLocalNone;
    hipError_t e;
    if (encode_uses_ticket(eg.tiles * static_cast<uint64_t>(stripes), k)) {
      std::lock_guard<std::mutex> lk(c->ticket_mu);
      int slot;
      unsigned long long* tk = c->ticket_take(s, &slot);
      e = launch_encode_tab(rows, eg, c->d_pass[q], s, tk);
      c->ticket_done(slot, s);
    } else {
      e = launch_encode_tab(rows, eg, c->d_pass[q], s, nullptr);
    }
    if (e != hipSuccess) return ECW_EDEVICE;
  }
  return ECW_OK;
}

int ecw_xor_reduce_dev(int device, const uint8_t* const* d_src, int n, uint8_t* d_dst, size_t len, void* stream) {
  if (!d_src || !d_dst || n < 1 || n > kMaxSrc || !check_len(len)) return ECW_EINVAL;
  if (!all_aligned(d_src, n) || !aligned16(d_dst)) return ECW_EALIGN;
  DeviceGuard g(device);
  if (!g.ok) return ECW_EDEVICE;
  return run_xor_ptr(d_src, n, d_dst, len, static_cast<hipStream_t>(stream));
}

int ecw_xor_reduce_ptrs_dev(int device, int stripes, int n, const uint8_t* const* d_src_ptrs,
                            uint8_t* const* d_dst_ptrs, size_t len, void* stream) {
  if (!d_src_ptrs || !d_dst_ptrs || stripes < 0 || n < 1 || n > kMaxSrc || !check_len(len)) return ECW_EINVAL;
  if (reinterpret_cast<uintptr_t>(d_src_ptrs) % 8 || reinterpret_cast<uintptr_t>(d_dst_ptrs) % 8) return ECW_EALIGN;
  if (len == 0 || stripes == 0) return ECW_OK;
  DeviceGuard g(device);
  if (!g.ok) return ECW_EDEVICE;
  svc::yield(device, false);
  const XorTab t{d_src_ptrs, d_dst_ptrs, n};
  const XorGeom xg{len, (len + kTileBytes - 1) / kTileBytes, stripes, n};
  return status_of(launch_xor_tab(t, xg, static_cast<hipStream_t>(stream)));
}

int ecw_decode_dev(ecw_codec* c, const uint8_t* const* d_data, uint8_t* d_target, size_t len, void* stream) {
  if (!c) return ECW_EINVAL;
  return ecw_xor_reduce_dev(c->device, d_data, c->info.decode_data_num, d_target, len, stream);
}

int ecw_partial_decode_dev(ecw_codec* c, const uint8_t* const* d_data, uint8_t* d_target, size_t len,
                           void* stream) {
  if (!c) return ECW_EINVAL;
  if (c->info.partial_decode_num < 1) return ECW_EUNSUPPORTED;  // RS/LRC codecs have no partial decode
  return ecw_xor_reduce_dev(c->device, d_data, c->info.partial_decode_num, d_target, len, stream);
}

int ecw_xor_intermediate_dev(ecw_codec* c, const uint8_t* const* d_src, uint8_t* const* d_tgt, size_t len,
                             void* stream) {
  if (!c || !d_src || !d_tgt || !check_len(len)) return ECW_EINVAL;
  const int m = c->m();
  if (!all_aligned(d_src, m) || !all_aligned(d_tgt, m)) return ECW_EALIGN;
  bool zero_first;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    zero_first = c->xori_mode == ECW_XORI_LITERAL && !c->xori_called;
    c->xori_called = true;
  }
  DeviceGuard g(c->device);
  if (!g.ok) return ECW_EDEVICE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int i = 0; i < m; ++i) {
    if (zero_first) {
      if (len && hipMemsetAsync(d_tgt[i], 0, len, s) != hipSuccess) return ECW_EDEVICE;
      continue;
    }
    const uint8_t* two[2] = {d_src[i], d_tgt[i]};
    const int st = run_xor_ptr(two, 2, d_tgt[i], len, s);
    if (st) return st;
  }
  return ECW_OK;
}

int ecw_encode_batch_dev(ecw_codec* c, uint8_t* d_slab, size_t block_stride, size_t stripe_stride, int stripes,
                         size_t len, void* stream) {
  if (!c || !d_slab || stripes < 0 || !check_len(len) || len > block_stride) return ECW_EINVAL;
  if (!aligned16(d_slab) || block_stride % 16 || stripe_stride % 16) return ECW_EALIGN;
  const size_t nblk = static_cast<size_t>(c->k()) + c->info.parity_num;
  if (stripes > 1 && stripe_stride < nblk * block_stride) return ECW_EINVAL;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    const int st = c->ensure_device();
    if (st) return st;
  }
  DeviceGuard g(c->device);
  if (!g.ok) return ECW_EDEVICE;
  const SlabRows slab = slab_rows(d_slab, block_stride, stripe_stride, c->k());
  EncodeTarget t;
  t.slab = &slab;
  t.stripes = stripes;
  return run_encode(c, t, len, static_cast<hipStream_t>(stream));
}

int ecw_encode_batch_split_dev(ecw_codec* c, const uint8_t* d_data, size_t data_block_stride,
                               size_t data_stripe_stride, uint8_t* d_parity, size_t parity_block_stride,
                               size_t parity_stripe_stride, int stripes, size_t len, void* stream) {
  if (!c || !d_data || !d_parity || stripes < 0 || !check_len(len)) return ECW_EINVAL;
  const size_t k = static_cast<size_t>(c->k()), np = static_cast<size_t>(c->info.parity_num);
  if ((k > 1 && len > data_block_stride) || (np > 1 && len > parity_block_stride)) return ECW_EINVAL;
  if (!aligned16(d_data) || !aligned16(d_parity) || data_block_stride % 16 || data_stripe_stride % 16 ||
      parity_block_stride % 16 || parity_stripe_stride % 16)
    return ECW_EALIGN;
  if (!disjoint_units(data_block_stride, data_stripe_stride, k, stripes, len) ||
      !disjoint_units(parity_block_stride, parity_stripe_stride, np, stripes, len))
    return ECW_EINVAL;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    const int st = c->ensure_device();
    if (st) return st;
  }
  DeviceGuard g(c->device);
  if (!g.ok) return ECW_EDEVICE;
  const SlabRows slab{d_data, data_block_stride, data_stripe_stride, d_parity, parity_block_stride,
                      parity_stripe_stride};
  EncodeTarget t;
  t.slab = &slab;
  t.stripes = stripes;
  return run_encode(c, t, len, static_cast<hipStream_t>(stream));
}

// a10: flat CL single-block repair = XOR of the surviving members of the lost
// block's local group (ClMetadataManager.java:161-183 takes the group's
// positions; XOR is associative, so the two-stage relay of
// ECTaskProcessor.java:293-332 gives the identical bytes).
int ecw_repair_sources(const ecw_codec* c, int lost, int* out, int cap) {
  if (!c || !out) return ECW_EINVAL;
  if (!c->has_local() || c->info.multinode) return ECW_EUNSUPPORTED;
  const int k = c->k(), m = c->m(), r = c->r(), ng = c->groups();
  if (lost < 0 || lost >= k + m + ng) return ECW_EINVAL;
  if (lost >= k && lost < k + m) return ECW_EUNSUPPORTED;  // G repair: "not yet" (ClMetadataManager.java:179-182)
  const int t = lost < k ? lost / r : lost - k - m;
  const int j0 = t * r, n = std::min(r, k - j0);
  if (cap < n) return ECW_EINVAL;
  int w = 0;
  for (int j = j0; j < j0 + n; ++j)
    if (j != lost) out[w++] = j;
  if (lost < k) out[w++] = k + m + t;  // the group's local parity
  return w;
}

// lost_block's sources as XOR sources over `rows`; a standard slab (parities
// right after the data blocks, same strides) runs as one region
static int repair_rows(ecw_codec* c, const SlabRows& rows, int stripes, int lost_block, uint8_t* d_out,
                       size_t out_stride, size_t len, hipStream_t stream) {
  if (c->info.local_mode == ECW_LOCAL_LITERAL) return ECW_EUNSUPPORTED;  // literal L blocks are zeros
  int idx[kMaxSrc];
  const int n = ecw_repair_sources(c, lost_block, idx, kMaxSrc);
  if (n < 0) return n;
  if (n == 0) return ECW_EUNSUPPORTED;
  DeviceGuard g(c->device);
  if (!g.ok) return ECW_EDEVICE;
  XorGeom xg{len, (len + kTileBytes - 1) / kTileBytes, stripes, n};
  if (len == 0 || stripes == 0) return ECW_OK;
  svc::yield(c->device, false);
  const int k = c->k();
  const bool one_region = rows.pbase == rows.base + static_cast<uint64_t>(k) * rows.bstride &&
                          rows.pbstride == rows.bstride && rows.psstride == rows.sstride;
  if (one_region) {
    XorSlab xs;
    std::memset(&xs, 0, sizeof xs);
    xs.base = rows.base;
    xs.bstride = rows.bstride;
    xs.sstride = rows.sstride;
    xs.out = d_out;
    xs.ostride = out_stride;
    for (int i = 0; i < n; ++i) xs.idx[i] = idx[i];
    return status_of(launch_xor_slab(xs, xg, stream));
  }
  XorSplit xs;
  std::memset(&xs, 0, sizeof xs);
  xs.base = rows.base;
  xs.bstride = rows.bstride;
  xs.sstride = rows.sstride;
  xs.pbase = rows.pbase;
  xs.pbstride = rows.pbstride;
  xs.psstride = rows.psstride;
  xs.out = d_out;
  xs.ostride = out_stride;
  for (int i = 0; i < n; ++i) {
    if (idx[i] < k) {
      if (xs.ndata != i) return ECW_EINVAL;  // ecw_repair_sources lists the data blocks first
      ++xs.ndata;
      xs.idx[i] = idx[i];
    } else {
      xs.idx[i] = idx[i] - k;
    }
  }
  return status_of(launch_xor_split(xs, xg, stream));
}

int ecw_repair_batch_dev(ecw_codec* c, const uint8_t* d_slab, size_t block_stride, size_t stripe_stride,
                         int stripes, int lost_block, uint8_t* d_out, size_t out_stride, size_t len, void* stream) {
  if (!c || !d_slab || !d_out || stripes < 0 || !check_len(len) || len > block_stride) return ECW_EINVAL;
  if (!aligned16(d_slab) || !aligned16(d_out) || block_stride % 16 || stripe_stride % 16 || out_stride % 16)
    return ECW_EALIGN;
  return repair_rows(c, slab_rows(d_slab, block_stride, stripe_stride, c->k()), stripes, lost_block, d_out,
                     out_stride, len, static_cast<hipStream_t>(stream));
}

int ecw_repair_batch_split_dev(ecw_codec* c, const uint8_t* d_data, size_t data_block_stride,
                               size_t data_stripe_stride, const uint8_t* d_parity, size_t parity_block_stride,
                               size_t parity_stripe_stride, int stripes, int lost_block, uint8_t* d_out,
                               size_t out_stride, size_t len, void* stream) {
  if (!c || !d_data || !d_parity || !d_out || stripes < 0 || !check_len(len)) return ECW_EINVAL;
  if (!aligned16(d_data) || !aligned16(d_parity) || !aligned16(d_out) || data_block_stride % 16 ||
      data_stripe_stride % 16 || parity_block_stride % 16 || parity_stripe_stride % 16 || out_stride % 16)
    return ECW_EALIGN;
  const SlabRows rows{d_data, data_block_stride, data_stripe_stride, const_cast<uint8_t*>(d_parity),
                      parity_block_stride, parity_stripe_stride};
  return repair_rows(c, rows, stripes, lost_block, d_out, out_stride, len, static_cast<hipStream_t>(stream));
}

int ecw_fill_random_dev(int device, uint8_t* d_dst, size_t block_stride, size_t stripe_stride, int stripes,
                        int nblocks, size_t len, uint64_t seed, int s0, int b0, void* stream) {
  if (!d_dst || stripes < 0 || nblocks < 0 || s0 < 0 || b0 < 0) return ECW_EINVAL;
  if (nblocks > 1 && block_stride < len) return ECW_EINVAL;
  if (!aligned16(d_dst) || block_stride % 16 || stripe_stride % 16) return ECW_EALIGN;
  DeviceGuard g(device);
  if (!g.ok) return ECW_EDEVICE;
  return status_of(launch_fill_random(d_dst, block_stride, stripe_stride, stripes, nblocks, len, len ? len : 1, 0,
                                      0, seed, s0, b0, static_cast<hipStream_t>(stream)));
}

int ecw_fill_random_pieces_dev(int device, uint8_t* d_dst, size_t block_stride, size_t stripe_stride, int stripes,
                               int nblocks, size_t len, size_t piece, size_t piece_stride, size_t offset,
                               uint64_t seed, int s0, int b0, void* stream) {
  if (!d_dst || stripes < 0 || nblocks < 0 || s0 < 0 || b0 < 0 || piece == 0) return ECW_EINVAL;
  if (!aligned16(d_dst) || block_stride % 16 || stripe_stride % 16 || piece % 16 || piece_stride % 16 ||
      offset % 16)
    return ECW_EALIGN;
  if (len > piece && piece_stride < piece) return ECW_EINVAL;
  DeviceGuard g(device);
  if (!g.ok) return ECW_EDEVICE;
  return status_of(launch_fill_random(d_dst, block_stride, stripe_stride, stripes, nblocks, len, piece,
                                      piece_stride, offset, seed, s0, b0, static_cast<hipStream_t>(stream)));
}

// ---- host-memory entry points (blocking) ------------------------------------
// The blocks stay in host memory (files / Java direct ByteBuffers in the
// reference). Columns are independent, so the call is pipelined over column
// slices of kHostChunk bytes through kSlots HBM staging slots on three
// streams: H2D copies of slice i+1 overlap the kernel on slice i and the D2H
// copies of slice i-1. With pinned (hipHostMalloc / registered) buffers the
// copies are DMA at PCIe rate; pageable buffers work too (HIP stages them).
// Serialised per codec (the staging slots are per codec).
constexpr size_t kHostChunk = size_t(8) << 20;
constexpr size_t kSmallBlock = size_t(256) << 10;  // blocks up to this size take the packed path
constexpr int kSlots = 3;

// Host -> HBM copies of a slice go out on kHostInStreams streams (block b on
// stream b % kHostInStreams): one copy queue moves 8 MiB copies at ~53.5 GB/s,
// two together at ~57 GB/s, PCIe Gen5 x16's practical rate
// (profiles/r05h2d_probe.log).
struct HostPipe {
  hipStream_t s_in[kHostInStreams] = {}, s_run = nullptr, s_out = nullptr;
  hipEvent_t ev_in[kHostInStreams][kSlots] = {}, ev_run[kSlots] = {}, ev_out[kSlots] = {};
  bool ok = false;
  int init() {
    if (ok) return ECW_OK;
    for (hipStream_t& st : s_in)
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return ECW_EDEVICE;
    for (hipStream_t* st : {&s_run, &s_out})
      if (hipStreamCreateWithFlags(st, hipStreamNonBlocking) != hipSuccess) return ECW_EDEVICE;
    for (int i = 0; i < kSlots; ++i) {
      for (auto& q : ev_in)
        if (hipEventCreateWithFlags(&q[i], hipEventDisableTiming) != hipSuccess) return ECW_EDEVICE;
      for (hipEvent_t* e : {&ev_run[i], &ev_out[i]})
        if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return ECW_EDEVICE;
    }
    ok = true;
    return ECW_OK;
  }
  void destroy(int device) {
    for (hipStream_t st : s_in) grave::release(st, grave::kStream, device);
    for (hipStream_t st : {s_run, s_out}) grave::release(st, grave::kStream, device);
    for (int i = 0; i < kSlots; ++i) {
      for (auto& q : ev_in) grave::release(q[i], grave::kEvent, device);
      for (hipEvent_t e : {ev_run[i], ev_out[i]}) grave::release(e, grave::kEvent, device);
    }
  }
  hipStream_t in(size_t b) const { return s_in[b % kHostInStreams]; }
  // slot `slot` may be refilled once its previous D2H copies are done
  bool wait_slot_free(int slot) const {
    for (hipStream_t st : s_in)
      if (hipStreamWaitEvent(st, ev_out[slot], 0) != hipSuccess) return false;
    return true;
  }
  // the kernel on slot `slot` waits for every input stream's copies into it
  bool inputs_ready(int slot) {
    for (int q = 0; q < kHostInStreams; ++q)
      if (hipEventRecord(ev_in[q][slot], s_in[q]) != hipSuccess || hipStreamWaitEvent(s_run, ev_in[q][slot], 0) != hipSuccess)
        return false;
    return true;
  }
};

// error exit of a pipelined call: let the copies already queued on the
// pipeline's streams finish before the caller may free its buffers
static int drain(HostPipe& P, int st) {
  for (hipStream_t x : P.s_in)
    if (x) (void)hipStreamSynchronize(x);
  for (hipStream_t x : {P.s_run, P.s_out})
    if (x) (void)hipStreamSynchronize(x);
  return st;
}

typedef int (*host_op)(ecw_codec*, uint8_t* const*, int, uint8_t* const*, int, size_t, hipStream_t);
static int op_xor(ecw_codec*, uint8_t* const* din, int nin, uint8_t* const* dout, int, size_t len, hipStream_t s);

static int host_roundtrip(ecw_codec* c, const uint8_t* const* in, int nin, uint8_t* const* out, int nout,
                          size_t len, host_op op) {
  for (int i = 0; i < nin; ++i)
    if (!in[i]) return ECW_EINVAL;
  for (int i = 0; i < nout; ++i)
    if (!out[i]) return ECW_EINVAL;
  if (len == 0) return ECW_OK;
  // a small XOR (decodeData / partialDecodeData / repair / xorIntemediate of
  // blocks up to 64 KiB): the resident request service, no launch
  const bool offered = len <= kSvcMaxLen && op == op_xor && nout == 1;
  if (offered) {
    const int sst = svc::serve(c, in, nin, out, len, true);
    if (sst != svc::kNotServed) return sst;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  int st = c->ensure_device();
  if (st) return st;
  DeviceGuard g(c->device);
  if (!g.ok) return ECW_EDEVICE;
  // bulk work is not queued behind the request service's resident kernel (its
  // launches also ask a running epoch to leave). A small XOR the service
  // declined (it was held off or stopping) does not hold it off in turn;
  // every other call -- bulk, a small op_zero, an XOR of more sources than
  // the service takes -- does, so it never waits out a running epoch on a
  // shared hardware queue.
  svc::Hold hold(c->device, !offered);
  if (offered) svc::yield(c->device, false);
  if (!c->pipe) {
    c->pipe = new (std::nothrow) HostPipe();
    if (!c->pipe) return ECW_ENOMEM;
  }
  HostPipe& P = *c->pipe;
  if ((st = P.init())) return st;
  const size_t chunk = std::min(len, kHostChunk);
  const size_t cstride = (chunk + 255) & ~static_cast<size_t>(255);
  const size_t slot_bytes = cstride * (nin + nout);
  if ((st = c->ensure_stage(slot_bytes * kSlots))) return st;
  std::vector<uint8_t*> din(nin), dout(nout);
  size_t i = 0;
  for (size_t c0 = 0; c0 < len; c0 += chunk, ++i) {
    const int slot = static_cast<int>(i % kSlots);
    const size_t n = std::min(chunk, len - c0);
    uint8_t* base = c->d_stage + slot * slot_bytes;
    for (int b = 0; b < nin; ++b) din[b] = base + b * cstride;
    for (int b = 0; b < nout; ++b) dout[b] = base + (nin + b) * cstride;
    if (i >= kSlots && !P.wait_slot_free(slot)) return drain(P, ECW_EDEVICE);
    for (int b = 0; b < nin; ++b)
      if (hipMemcpyAsync(din[b], in[b] + c0, n, hipMemcpyHostToDevice, P.in(b)) != hipSuccess) return drain(P, ECW_EDEVICE);
    if (!P.inputs_ready(slot)) return drain(P, ECW_EDEVICE);
    if ((st = op(c, din.data(), nin, dout.data(), nout, n, P.s_run))) return drain(P, st);
    if (hipEventRecord(P.ev_run[slot], P.s_run) != hipSuccess) return drain(P, ECW_EDEVICE);
    if (hipStreamWaitEvent(P.s_out, P.ev_run[slot], 0) != hipSuccess) return drain(P, ECW_EDEVICE);
    for (int b = 0; b < nout; ++b)
      if (hipMemcpyAsync(out[b] + c0, dout[b], n, hipMemcpyDeviceToHost, P.s_out) != hipSuccess) return drain(P, ECW_EDEVICE);
    if (hipEventRecord(P.ev_out[slot], P.s_out) != hipSuccess) return drain(P, ECW_EDEVICE);
  }
  if (hipStreamSynchronize(P.s_out) != hipSuccess) return drain(P, ECW_EDEVICE);
  return hipStreamSynchronize(P.s_run) == hipSuccess ? ECW_OK : ECW_EDEVICE;
}

void ecw_codec::destroy_pipe() {
  if (pipe) {
    pipe->destroy(device);
    delete pipe;
    pipe = nullptr;
  }
}

static int op_zero(ecw_codec*, uint8_t* const*, int, uint8_t* const* dout, int nout, size_t len, hipStream_t s) {
  for (int b = 0; b < nout; ++b)
    if (hipMemsetAsync(dout[b], 0, len, s) != hipSuccess) return ECW_EDEVICE;
  return ECW_OK;
}

static int op_encode(ecw_codec* c, uint8_t* const* din, int, uint8_t* const* dout, int, size_t len, hipStream_t s) {
  EncodeTarget t;
  t.src = din;
  t.dst = dout;
  return run_encode(c, t, len, s);
}
static int op_xor(ecw_codec*, uint8_t* const* din, int nin, uint8_t* const* dout, int, size_t len, hipStream_t s) {
  return run_xor_ptr(din, nin, dout[0], len, s);
}

// ---- small-stripe request service (ecw_internal.hpp SvcCtl) -----------------
// One synchronous small encode = copy the blocks into a slot's pinned staging,
// bump the slot's `seq`, spin on `done`, copy the parities out: no launch, no
// stream synchronisation, no DMA setup. The resident kernel is (re)launched on
// demand and leaves by itself after ECW_SERVICE_IDLE_MS (default 20) ms with no
// request on any slot. ECW_SERVICE=0 turns the service off.
namespace svc {

bool enabled() {
  static const bool on = [] {
    const char* e = std::getenv("ECW_SERVICE");
    return !(e && e[0] == '0');
  }();
  return on;
}

struct Service {
  int device = -1;
  std::mutex mu;  // everything below
  std::condition_variable cv;
  bool broken = false;
  SvcCtl* ctl = nullptr;    // coherent pinned host memory (host view)
  SvcCtl* d_ctl = nullptr;  // its device view
  SvcDev* d_state = nullptr;
  hipStream_t stream = nullptr;
  unsigned long long epoch = 0;  // last epoch launched (0: none yet)
  unsigned long long idle_ticks = 0, life_ticks = 0;
  std::vector<int> free_slots;
  // blocking launch-path calls in flight on this device (svc::Hold): while
  // any, the resident kernel is not relaunched and new small calls take the
  // launch path, so that work never queues behind it
  std::atomic<int> holds{0};
  std::atomic<unsigned long long> n_served{0}, n_declined{0};  // ecw_service_counters
  uint8_t* stage[kSvcSlots] = {};
  uint8_t* d_stage[kSvcSlots] = {};
  size_t stage_bytes[kSvcSlots] = {};

  int init() {
    DeviceGuard g(device);
    if (!g.ok) return ECW_EDEVICE;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0)
      return ECW_EDEVICE;
    const char* e = std::getenv("ECW_SERVICE_IDLE_MS");
    const unsigned long long idle_ms = e ? std::strtoull(e, nullptr, 10) : 20;
    // A lifetime bounds how long the resident kernel holds the device while
    // callers keep it busy: device-wide synchronisation (hipDeviceSynchronize,
    // hipFree) and other kernels sharing its hardware queue wait for it to
    // leave. 100 ms costs a relaunch (~10 us) per 100 ms of service.
    const char* l = std::getenv("ECW_SERVICE_LIFE_MS");
    const unsigned long long life_ms = l ? std::strtoull(l, nullptr, 10) : 100;
    idle_ticks = idle_ms * static_cast<unsigned long long>(khz);
    life_ticks = (life_ms ? life_ms : 1) * static_cast<unsigned long long>(khz);
    void* h = nullptr;
    if (hipHostMalloc(&h, sizeof(SvcCtl), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
      return ECW_ENOMEM;
    std::memset(h, 0, sizeof(SvcCtl));
    void* dv = nullptr;
    if (hipHostGetDevicePointer(&dv, h, 0) != hipSuccess || hipMalloc(&d_state, sizeof(SvcDev)) != hipSuccess ||
        hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
      (void)hipHostFree(h);
      if (d_state) (void)hipFree(d_state);
      d_state = nullptr;
      return ECW_EDEVICE;
    }
    ctl = static_cast<SvcCtl*>(h);
    d_ctl = static_cast<SvcCtl*>(dv);
    for (int i = kSvcSlots - 1; i >= 0; --i) free_slots.push_back(i);
    return ECW_OK;
  }

  // launch the next epoch unless the current one is still serving, or a
  // launch-path call holds it off (under mu; ECW_OK either way)
  int ensure_running() {
    if (epoch != 0 && __atomic_load_n(&ctl->exited_epoch, __ATOMIC_ACQUIRE) != epoch) return ECW_OK;
    if (holds.load(std::memory_order_acquire) > 0) return ECW_OK;  // relaunched once the hold ends
    grave::reap_device(device);  // what teardowns deferred while the last epoch ran
    __atomic_store_n(&ctl->stop, 0ull, __ATOMIC_RELEASE);  // a yield asked the previous epoch to leave
    DeviceGuard g(device);
    if (!g.ok || hipMemsetAsync(d_state, 0, sizeof(SvcDev), stream) != hipSuccess) return ECW_EDEVICE;
    if (launch_service(d_ctl, d_state, epoch + 1, idle_ticks, life_ticks, stream) != hipSuccess) return ECW_EDEVICE;
    ++epoch;
    return ECW_OK;
  }

  // A slot's staging only grows (at least 1 MiB, doubling), and a replaced
  // one is retired, not freed: freeing pinned memory can wait for the device
  // to go idle, which the resident kernel does not while other callers keep
  // it busy.
  std::vector<void*> retired;

  int ensure_stage(int slot, size_t bytes) {
    if (stage_bytes[slot] >= bytes) return ECW_OK;
    const size_t want = std::max({bytes, 2 * stage_bytes[slot], size_t(1) << 20});
    void* h = nullptr;
    void* dv = nullptr;
    if (hipHostMalloc(&h, want, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return ECW_ENOMEM;
    if (hipHostGetDevicePointer(&dv, h, 0) != hipSuccess) {
      retired.push_back(h);
      return ECW_EDEVICE;
    }
    if (stage[slot]) retired.push_back(stage[slot]);
    stage[slot] = static_cast<uint8_t*>(h);
    d_stage[slot] = static_cast<uint8_t*>(dv);
    stage_bytes[slot] = want;
    return ECW_OK;
  }

  void stop() {
    std::lock_guard<std::mutex> lk(mu);
    if (!ctl || epoch == 0) return;
    __atomic_store_n(&ctl->stop, 1ull, __ATOMIC_RELEASE);
    DeviceGuard g(device);
    (void)hipStreamSynchronize(stream);
    __atomic_store_n(&ctl->stop, 0ull, __ATOMIC_RELEASE);
  }
};

std::mutex g_mu;
std::map<int, Service*> g_services;  // one per device, kept for the life of the process

Service* find(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_services.find(device);
  return it == g_services.end() ? nullptr : it->second;
}

// (declared at the top)
extern "C++" void yield(int device, bool hold) {
  Service* sv = find(device);
  if (!sv) return;
  if (hold) sv->holds.fetch_add(1, std::memory_order_acq_rel);
  std::lock_guard<std::mutex> lk(sv->mu);
  // every part watches the stop flag; the next epoch starts with it cleared
  if (sv->ctl && sv->epoch != 0 && __atomic_load_n(&sv->ctl->exited_epoch, __ATOMIC_ACQUIRE) != sv->epoch)
    __atomic_store_n(&sv->ctl->stop, 1ull, __ATOMIC_RELEASE);
}
extern "C++" void release_hold(int device) {
  Service* sv = find(device);
  if (sv) sv->holds.fetch_sub(1, std::memory_order_acq_rel);
}

// (declared at the top) the resident kernel has been launched and has not
// published its exit yet
extern "C++" bool busy(int device) {
  Service* sv;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_services.find(device);
    if (it == g_services.end()) return false;
    sv = it->second;
  }
  std::lock_guard<std::mutex> lk(sv->mu);
  return sv->ctl && sv->epoch != 0 && __atomic_load_n(&sv->ctl->exited_epoch, __ATOMIC_ACQUIRE) != sv->epoch;
}

void stop_all() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& kv : g_services) kv.second->stop();
}

Service* service_for(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  Service*& sv = g_services[device];
  if (!sv) {
    if (g_services.size() == 1) std::atexit(stop_all);  // leave every resident kernel before the runtime goes
    sv = new Service();
    sv->device = device;
  }
  return sv;
}

// Serve one request, or return kNotServed (shape or state not suitable): the
// codec's encode of one stripe (xor_only false: k data blocks -> its parity
// blocks), or the XOR of `nsrc` blocks into one (xor_only true: decodeData /
// partialDecodeData / a CL repair / xorIntemediate on host memory; no tables).
extern "C++" int serve(ecw_codec* c, const uint8_t* const* data, int nsrc, uint8_t* const* parity, size_t len,
                       bool xor_only) {
  const int k = xor_only ? nsrc : c->k(), m = xor_only ? 1 : c->m(), np = xor_only ? 1 : c->info.parity_num;
  const int nw = m <= 4 ? 1 : 2;
  if (!enabled() || m < 1 || m > kMaxSvcRows || len == 0 || len > kSvcMaxLen || k < 1 || k > kMaxSrc ||
      (!xor_only && static_cast<size_t>(k) * 128 * nw > kSvcLds))
    return kNotServed;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->ensure_device() != ECW_OK) return kNotServed;  // the launch path reports the error
  }
  Service* sv = service_for(c->device);
  auto decline = [&] {
    sv->n_declined.fetch_add(1, std::memory_order_relaxed);
    return kNotServed;
  };
  if (sv->holds.load(std::memory_order_acquire) > 0) return decline();  // launch-path work in flight
  const size_t cs = (len + 255) & ~static_cast<size_t>(255);
  int slot;
  {
    std::unique_lock<std::mutex> lk(sv->mu);
    if (sv->broken) return decline();
    if (!sv->ctl && sv->init() != ECW_OK) {
      sv->broken = true;
      return decline();
    }
    sv->cv.wait(lk, [&] { return !sv->free_slots.empty() || sv->broken; });
    if (sv->broken) return decline();
    // a thread keeps the slot it had last time when it is free: its parts
    // poll at full speed (a slot idle for 1 ms polls slowly) and may still
    // hold the thread's request words and tables
    thread_local int t_slot = -1;
    auto it = std::find(sv->free_slots.begin(), sv->free_slots.end(), t_slot);
    if (it == sv->free_slots.end()) it = sv->free_slots.end() - 1;
    slot = *it;
    sv->free_slots.erase(it);
    t_slot = slot;
    if (sv->ensure_stage(slot, cs * (k + np)) != ECW_OK) {
      sv->free_slots.push_back(slot);
      sv->cv.notify_one();
      return decline();
    }
  }
  // give the slot back (takes mu: never call it with mu held)
  auto release = [&](int st) {
    std::lock_guard<std::mutex> lk(sv->mu);
    sv->free_slots.push_back(slot);
    sv->cv.notify_all();
    return st;
  };
  uint8_t* h = sv->stage[slot];
  for (int j = 0; j < k; ++j) std::memcpy(h + j * cs, data[j], len);
  SvcSlot& q = sv->ctl->slot[slot];
  // only this thread writes the slot while it holds it
  const SvcSlot want = [&] {
    SvcSlot w = q;
    w.tbl = c->d_pass[0];
    w.data = sv->d_stage[slot];
    w.out = sv->d_stage[slot] + static_cast<size_t>(k) * cs;
    w.len = len;
    w.cs = cs;
    w.k = k;
    w.nrows = m;
    w.m = m;
    w.r = !xor_only && c->has_local() ? c->r() : k;
    w.groups = xor_only ? 0 : c->groups();
    w.local_mode = xor_only ? kLocalNone : local_mode_of(c);
    w.nw = nw;
    w.flags = xor_only || c->xor_row ? kSvcXorRow : 0;  // a plain XOR: no tables staged
    w.serial = c->serial;
    return w;
  }();
  unsigned long long gen = q.seq >> kSvcSeqBits;
  const size_t words = offsetof(SvcSlot, flags) + sizeof(int) - offsetof(SvcSlot, tbl);
  if (q.seq == 0 || std::memcmp(&want.tbl, &q.tbl, words) != 0) {  // new request words: a new generation
    std::memcpy(&q.tbl, &want.tbl, words);
    gen = (gen + 1) & ((1ull << (64 - kSvcSeqBits)) - 1);
  }
  const unsigned long long units = (len + kSvcThreads * 4 - 1) / (kSvcThreads * 4);
  const int active = static_cast<int>(std::min<unsigned long long>(units, kSvcParts));
  const unsigned long long seq = (gen << kSvcSeqBits) | (static_cast<unsigned long long>(active) << 32) |
                                 (((q.seq & kSvcReqMask) + 1) & kSvcReqMask);
  __atomic_store_n(&q.seq, seq, __ATOMIC_RELEASE);
  bool up;
  {
    std::lock_guard<std::mutex> lk(sv->mu);
    up = sv->ensure_running() == ECW_OK;
    if (!up) sv->broken = true;  // the launch path takes this call and every later one
  }
  if (!up) {
    release(0);
    return decline();
  }
  const auto t0 = std::chrono::steady_clock::now();
  int failed = ECW_OK;
  bool timed_out = false, held_off = false;
  // every part with work publishes its own done word (one cache line)
  auto finished = [&] {
    for (int p = 0; p < active; ++p)
      if (__atomic_load_n(&q.done[p], __ATOMIC_ACQUIRE) != seq) return false;
    return true;
  };
  for (unsigned spins = 1; !finished(); ++spins) {
    if (spins % 1024) {
      __builtin_ia32_pause();
      continue;
    }
    std::lock_guard<std::mutex> lk(sv->mu);
    if (finished()) break;
    // the epoch this request was posted to left before serving it: start the next one
    if (sv->ensure_running() != ECW_OK) {  // a HIP error: the launch path takes this call and every later one
      sv->broken = true;
      failed = ECW_EDEVICE;
      break;
    }
    // The epoch left without serving this request (a launch-path call asked it
    // to) and a hold keeps the next one from starting: take the launch path
    // now instead of waiting for every hold to end. The service stays on. No
    // kernel polls while the epoch is gone and none starts while mu is held,
    // so the request is withdrawn before the slot is given back -- by a NEW
    // request word with no active part (the parts only note it), never by
    // restoring the previous word: some parts may have finished this request
    // and published its word in their `done`, and a later request posted with
    // that same word again would find them "finished" with this one's
    // results. Request numbers only ever advance.
    if (sv->holds.load(std::memory_order_acquire) > 0 &&
        __atomic_load_n(&sv->ctl->exited_epoch, __ATOMIC_ACQUIRE) == sv->epoch) {
      const unsigned long long withdrawn =
          (seq & ~((static_cast<unsigned long long>(0xFF) << 32) | kSvcReqMask)) | (((seq & kSvcReqMask) + 1) & kSvcReqMask);
      __atomic_store_n(&q.seq, withdrawn, __ATOMIC_RELEASE);
      held_off = true;
      break;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
      // Not served in 10 s. An epoch that has not started is queued behind
      // other work on the device (contention): this call takes the launch path
      // (the slot is given back; a late serve only rewrites its own staging).
      // An epoch that runs and does not serve is broken: the launch path takes
      // every later call too.
      if (__atomic_load_n(&sv->ctl->started_epoch, __ATOMIC_ACQUIRE) == sv->epoch) sv->broken = true;
      timed_out = true;
      break;
    }
  }
  if (failed) return release(failed);
  if (timed_out || held_off) {
    release(0);
    return decline();
  }
  for (int i = 0; i < np; ++i) std::memcpy(parity[i], h + static_cast<size_t>(k + i) * cs, len);
  sv->n_served.fetch_add(1, std::memory_order_relaxed);
  return release(ECW_OK);
}

extern "C++" int counters(int device, unsigned long long out[4]) {
  Service* sv = find(device);
  if (!sv) {
    for (int i = 0; i < 4; ++i) out[i] = 0;
    return ECW_OK;
  }
  std::lock_guard<std::mutex> lk(sv->mu);
  out[0] = sv->n_served.load(std::memory_order_relaxed);
  out[1] = sv->n_declined.load(std::memory_order_relaxed);
  out[2] = sv->epoch;
  out[3] = sv->broken ? 1 : 0;
  return ECW_OK;
}

}  // namespace svc

int ecw_host_alloc(int device, size_t bytes, void** out, int* numa_node) {
  return ecw_host_alloc_node(device, -1, bytes, out, numa_node);
}

int ecw_host_alloc_node(int device, int node, size_t bytes, void** out, int* numa_node) {
  if (!out || bytes == 0 || device < 0 || node < -1 || node >= 1024) return ECW_EINVAL;
  *out = nullptr;
  if (numa_node) *numa_node = -1;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) return ECW_EDEVICE;
  if (node < 0) node = device_numa_node(device);
  const size_t n = (bytes + 4095) & ~static_cast<size_t>(4095);
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return ECW_ENOMEM;
  if (node >= 0 && node < 1024) {
    // preferred (not bound): a full node falls back to another instead of failing
    unsigned long mask[16] = {};
    mask[node / 64] = 1ul << (node % 64);
    (void)syscall(SYS_mbind, p, n, 1 /* MPOL_PREFERRED */, mask, 1024ul, 0u);
  }
  // fault every page in (on the preferred node) from several threads
  const unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  const size_t per = (n / nt + 4095) & ~static_cast<size_t>(4095);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) {
    const size_t o = t * per;
    if (o >= n) break;
    th.emplace_back([=] { std::memset(static_cast<char*>(p) + o, 0, std::min(per, n - o)); });
  }
  for (auto& x : th) x.join();
  {
    DeviceGuard g(device);
    if (!g.ok || hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) {
      munmap(p, n);
      return ECW_EDEVICE;
    }
  }
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_allocs[p] = n;
  }
  if (numa_node) *numa_node = pages_node(p, n);
  *out = p;
  return ECW_OK;
}

int ecw_host_free(void* p) {
  if (!p) return ECW_OK;
  size_t n = 0;
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_allocs.find(p);
    if (it == g_host_allocs.end()) return ECW_EINVAL;
    n = it->second;
    g_host_allocs.erase(it);
  }
  const int st = hipHostUnregister(p) == hipSuccess ? ECW_OK : ECW_EDEVICE;
  munmap(p, n);
  return st;
}

int ecw_device_numa_node(int device) {
  int ndev = 0;
  if (device < 0 || hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) return -1;
  return device_numa_node(device);
}

int ecw_service_counters(int device, unsigned long long out[4]) {
  if (!out || device < 0) return ECW_EINVAL;
  return svc::counters(device, out);
}

int ecw_encode(ecw_codec* c, const uint8_t* const* data, uint8_t* const* parity, size_t len) {
  if (!c || !data || !parity || !check_len(len)) return ECW_EINVAL;
  for (int j = 0; j < c->k(); ++j)
    if (!data[j]) return ECW_EINVAL;
  for (int i = 0; i < c->info.parity_num; ++i)
    if (!parity[i]) return ECW_EINVAL;
  // small blocks: the resident request service, else one packed stripe (two
  // copy calls instead of one per block)
  if (len > 0 && len <= kSmallBlock) return ecw_encode_stripes(c, 1, data, parity, len);
  return host_roundtrip(c, data, c->k(), parity, c->info.parity_num, len, op_encode);
}

int ecw_decode(ecw_codec* c, const uint8_t* const* data, uint8_t* target, size_t len) {
  if (!c || !data || !target || !check_len(len)) return ECW_EINVAL;
  uint8_t* const out[1] = {target};
  return host_roundtrip(c, data, c->info.decode_data_num, out, 1, len, op_xor);
}

int ecw_partial_decode(ecw_codec* c, const uint8_t* const* data, uint8_t* target, size_t len) {
  if (!c || !data || !target || !check_len(len)) return ECW_EINVAL;
  if (c->info.partial_decode_num < 1) return ECW_EUNSUPPORTED;
  uint8_t* const out[1] = {target};
  return host_roundtrip(c, data, c->info.partial_decode_num, out, 1, len, op_xor);
}

// Many stripes from host memory: batches of stripes x column slices go
// through the same 3-slot / 3-stream pipeline as host_roundtrip, each slot
// laid out as a slab ([D.., G.., L..] per stripe) so one launch encodes the
// whole batch.
namespace {

// Small blocks (ECWide-H's 4 KiB chunks): one copy call per block would cost
// more than the block (~5 us of API time each), so a batch of stripes is
// packed by the CPU into pinned host memory laid out like the device slab,
// crosses PCIe as one 2-D copy each way, and is encoded in one launch. Two
// staging slots: the CPU packs batch b+1 (and unpacks batch b-1) while the
// GPU copies and encodes batch b.
constexpr size_t kPackBytes = size_t(32) << 20;  // host + device slot size
// A batch whose packed image is at most this many bytes skips both copies:
// the kernel reads the pinned image over PCIe and writes the parities back
// into it (zero-copy). For a handful of 4 KiB stripes the two DMA transfers
// are most of the round trip. ECW_ZERO_COPY_BYTES overrides (0 = off).
size_t zero_copy_bytes() {
  static const size_t v = [] {
    const char* e = std::getenv("ECW_ZERO_COPY_BYTES");
    return e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : size_t(1) << 20;
  }();
  return v;
}

void copy_blocks(size_t n, size_t len, const std::function<void(size_t, size_t)>& fn) {
  // parallel memcpy loop for big batches only: a thread costs tens of us to
  // start, one core copies ~8 MiB in about a millisecond
  const size_t nt = std::min<size_t>(8, std::max<unsigned>(1, std::thread::hardware_concurrency()));
  if (n * len < (size_t(8) << 20) || nt < 2) return fn(0, n);
  std::vector<std::thread> th;
  const size_t per = (n + nt - 1) / nt;
  for (size_t t = 1; t < nt && t * per < n; ++t) th.emplace_back(fn, t * per, std::min(n, (t + 1) * per));
  fn(0, std::min(n, per));
  for (auto& x : th) x.join();
}

int encode_stripes_packed(ecw_codec* c, HostPipe& P, int stripes, const uint8_t* const* data,
                          uint8_t* const* parity, size_t len) {
  const int k = c->k(), np = c->info.parity_num, nb = k + np;
  const size_t cs = (len + 255) & ~static_cast<size_t>(255);  // block stride in the slot
  const size_t sb_bytes = cs * nb;
  const int per = static_cast<int>(std::max<size_t>(1, std::min<size_t>(stripes, kPackBytes / sb_bytes)));
  const size_t slot = sb_bytes * per;
  int st;
  if ((st = c->ensure_stage(slot * 2)) || (st = c->ensure_host_stage(slot * 2))) return st;
  if (per >= stripes && sb_bytes * stripes <= zero_copy_bytes()) {
    uint8_t* h = c->h_stage;
    copy_blocks(static_cast<size_t>(stripes) * k, len, [&](size_t a, size_t e) {
      for (size_t x = a; x < e; ++x) std::memcpy(h + (x / k) * sb_bytes + (x % k) * cs, data[x], len);
    });
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, h, 0) != hipSuccess) return drain(P, ECW_EDEVICE);
    const SlabRows slab = slab_rows(static_cast<uint8_t*>(dp), cs, sb_bytes, k);
    EncodeTarget t;
    t.slab = &slab;
    t.stripes = stripes;
    if ((st = run_encode(c, t, len, P.s_run))) return drain(P, st);
    if (hipStreamSynchronize(P.s_run) != hipSuccess) return drain(P, ECW_EDEVICE);
    for (size_t x = 0; x < static_cast<size_t>(stripes) * np; ++x)
      std::memcpy(parity[x], h + (x / np) * sb_bytes + (k + x % np) * cs, len);
    return ECW_OK;
  }
  int first[2] = {-1, -1}, count[2] = {0, 0};  // batch held by each slot, awaiting unpack
  auto unpack = [&](int q) -> int {
    if (first[q] < 0) return ECW_OK;
    if (hipEventSynchronize(P.ev_out[q]) != hipSuccess) return drain(P, ECW_EDEVICE);
    const uint8_t* h = c->h_stage + q * slot;
    const int s0 = first[q];
    copy_blocks(static_cast<size_t>(count[q]) * np, len, [&](size_t a, size_t b) {
      for (size_t x = a; x < b; ++x)
        std::memcpy(parity[static_cast<size_t>(s0) * np + x], h + (x / np) * sb_bytes + (k + x % np) * cs, len);
    });
    first[q] = -1;
    return ECW_OK;
  };
  int b = 0;
  for (int s0 = 0; s0 < stripes; s0 += per, ++b) {
    const int q = b & 1, ns = std::min(per, stripes - s0);
    if ((st = unpack(q))) return drain(P, st);
    uint8_t* h = c->h_stage + q * slot;
    uint8_t* d = c->d_stage + q * slot;
    copy_blocks(static_cast<size_t>(ns) * k, len, [&](size_t a, size_t e) {
      for (size_t x = a; x < e; ++x)
        std::memcpy(h + (x / k) * sb_bytes + (x % k) * cs, data[static_cast<size_t>(s0) * k + x], len);
    });
    if (hipMemcpy2DAsync(d, sb_bytes, h, sb_bytes, k * cs, ns, hipMemcpyHostToDevice, P.s_run) != hipSuccess)
      return drain(P, ECW_EDEVICE);
    const SlabRows slab = slab_rows(d, cs, sb_bytes, k);
    EncodeTarget t;
    t.slab = &slab;
    t.stripes = ns;
    if ((st = run_encode(c, t, len, P.s_run))) return drain(P, st);
    if (hipMemcpy2DAsync(h + k * cs, sb_bytes, d + k * cs, sb_bytes, np * cs, ns, hipMemcpyDeviceToHost,
                         P.s_run) != hipSuccess ||
        hipEventRecord(P.ev_out[q], P.s_run) != hipSuccess)
      return drain(P, ECW_EDEVICE);
    first[q] = s0;
    count[q] = ns;
  }
  if ((st = unpack(b & 1)) || (st = unpack((b + 1) & 1))) return st;
  return ECW_OK;
}

}  // namespace

int ecw_encode_stripes(ecw_codec* c, int stripes, const uint8_t* const* data, uint8_t* const* parity,
                       size_t len) {
  if (!c || stripes < 0 || !data || !parity || !check_len(len)) return ECW_EINVAL;
  const int k = c->k(), np = c->info.parity_num, nb = k + np;
  for (size_t i = 0; i < static_cast<size_t>(stripes) * k; ++i)
    if (!data[i]) return ECW_EINVAL;
  for (size_t i = 0; i < static_cast<size_t>(stripes) * np; ++i)
    if (!parity[i]) return ECW_EINVAL;
  if (len == 0 || stripes == 0) return ECW_OK;
  if (stripes == 1 && len <= kSvcMaxLen) {
    const int sst = svc::serve(c, data, c->k(), parity, len, false);
    if (sst != svc::kNotServed) return sst;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  int st = c->ensure_device();
  if (st) return st;
  DeviceGuard g(c->device);
  if (!g.ok) return ECW_EDEVICE;
  // bulk work is not queued behind the request service's resident kernel; a
  // single small stripe that the service did not take (it is held off, or
  // stopping) does not hold it off in turn
  svc::Hold hold(c->device, !(stripes == 1 && len <= kSvcMaxLen));
  if (!c->pipe) {
    c->pipe = new (std::nothrow) HostPipe();
    if (!c->pipe) return ECW_ENOMEM;
  }
  HostPipe& P = *c->pipe;
  if ((st = P.init())) return st;
  if (len <= kSmallBlock) return encode_stripes_packed(c, P, stripes, data, parity, len);
  const size_t chunk = std::min(len, kHostChunk);
  const size_t cstride = (chunk + 255) & ~static_cast<size_t>(255);
  const size_t stripe_bytes = cstride * nb;
  // stripes per batch: fill a slot of ~ (k + np) * 8 MiB
  const int sb = static_cast<int>(std::max<size_t>(1, std::min<size_t>(stripes, (kHostChunk * nb) / stripe_bytes)));
  const size_t slot_bytes = stripe_bytes * sb;
  if ((st = c->ensure_stage(slot_bytes * kSlots))) return st;
  size_t step = 0;
  for (int s0 = 0; s0 < stripes; s0 += sb) {
    const int ns = std::min(sb, stripes - s0);
    for (size_t c0 = 0; c0 < len; c0 += chunk, ++step) {
      const int slot = static_cast<int>(step % kSlots);
      const size_t n = std::min(chunk, len - c0);
      uint8_t* base = c->d_stage + slot * slot_bytes;
      if (step >= kSlots && !P.wait_slot_free(slot)) return drain(P, ECW_EDEVICE);
      for (int s = 0; s < ns; ++s)
        for (int j = 0; j < k; ++j)
          if (hipMemcpyAsync(base + s * stripe_bytes + j * cstride, data[static_cast<size_t>(s0 + s) * k + j] + c0, n,
                             hipMemcpyHostToDevice, P.in(static_cast<size_t>(s) * k + j)) != hipSuccess)
            return drain(P, ECW_EDEVICE);
      if (!P.inputs_ready(slot)) return drain(P, ECW_EDEVICE);
      const SlabRows slab = slab_rows(base, cstride, stripe_bytes, k);
      EncodeTarget t;
      t.slab = &slab;
      t.stripes = ns;
      if ((st = run_encode(c, t, n, P.s_run))) return drain(P, st);
      if (hipEventRecord(P.ev_run[slot], P.s_run) != hipSuccess) return drain(P, ECW_EDEVICE);
      if (hipStreamWaitEvent(P.s_out, P.ev_run[slot], 0) != hipSuccess) return drain(P, ECW_EDEVICE);
      for (int s = 0; s < ns; ++s)
        for (int i = 0; i < np; ++i)
          if (hipMemcpyAsync(parity[static_cast<size_t>(s0 + s) * np + i] + c0, base + s * stripe_bytes + (k + i) * cstride,
                             n, hipMemcpyDeviceToHost, P.s_out) != hipSuccess)
            return drain(P, ECW_EDEVICE);
      if (hipEventRecord(P.ev_out[slot], P.s_out) != hipSuccess) return drain(P, ECW_EDEVICE);
    }
  }
  if (hipStreamSynchronize(P.s_out) != hipSuccess) return drain(P, ECW_EDEVICE);
  return hipStreamSynchronize(P.s_run) == hipSuccess ? ECW_OK : ECW_EDEVICE;
}

int ecw_repair(ecw_codec* c, const uint8_t* const* blocks, int lost, uint8_t* out, size_t len) {
  if (!c || !blocks || !out || !check_len(len)) return ECW_EINVAL;
  if (c->info.local_mode == ECW_LOCAL_LITERAL) return ECW_EUNSUPPORTED;  // literal L blocks are zeros
  int idx[kMaxSrc];
  const int n = ecw_repair_sources(c, lost, idx, kMaxSrc);
  if (n < 0) return n;
  if (n == 0) return ECW_EUNSUPPORTED;
  std::vector<const uint8_t*> src(n);
  for (int i = 0; i < n; ++i) src[i] = blocks[idx[i]];
  uint8_t* const o[1] = {out};
  return host_roundtrip(c, src.data(), n, o, 1, len, op_xor);
}

int ecw_xor_intermediate(ecw_codec* c, const uint8_t* const* source, uint8_t* const* target, size_t len) {
  if (!c || !source || !target || !check_len(len)) return ECW_EINVAL;
  const int m = c->m();
  bool zero_first;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    zero_first = c->xori_mode == ECW_XORI_LITERAL && !c->xori_called;
    c->xori_called = true;
  }
  for (int i = 0; i < m; ++i) {
    if (!source[i] || !target[i]) return ECW_EINVAL;
    if (zero_first) {  // the reference's first-call output (NativeCodec.cc:287-292), made on the device
      const uint8_t* in1[1] = {source[i]};
      uint8_t* const out1[1] = {target[i]};
      const int st = host_roundtrip(c, in1, 0, out1, 1, len, op_zero);
      if (st) return st;
      continue;
    }
    const uint8_t* in[2] = {source[i], target[i]};
    uint8_t* const out[1] = {target[i]};
    const int st = host_roundtrip(c, in, 2, out, 1, len, op_xor);
    if (st) return st;
  }
  return ECW_OK;
}

}  // extern "C"
