// C ABI of the MI355X Reed-Solomon path (include/callfs_rs.h).
//
// Host side of the drop-in for erasure/codec.go. The control flow and error precedence
// follow codec.go:21-78 and the upstream reedsolomon methods it calls (Split/Encode at
// :31/:36, Reconstruct at :55, Verify at :59); every byte of GF(2^8) arithmetic over
// shard data runs in the HIP kernels of rs_kernels.hip.
//
// Structure
//  * rs_ctx     — selected devices, each with a pool of Lanes and a cache of decode
//                 tables keyed by (k, m, presence mask).
//  * Lane       — one HIP stream plus grow-only device/pinned buffers: the pitched
//                 shard workspace used by the host-memory entry points, pointer
//                 tables and coefficient tables for one-shot launches.
//  * rs_plan    — device-resident tables for repeated, graph-capturable launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/callfs_rs.h"
#include "bitslice.hpp"
#include "copy_pool.hpp"
#include "dispatch.hpp"
#include "gf256.hpp"
#include "rs_kernels.hpp"
#include "sha256.hpp"
#include "tune_table.hpp"

using namespace callfs;

namespace {

#define HIPCHK(x)                           \
  do {                                      \
    if ((x) != hipSuccess) return RS_E_HIP; \
  } while (0)

// Restores the calling thread's current HIP device on scope exit: entry points select
// the device they work on, and a caller's later default-device work (torch, HIP) must
// not land on another GPU because of a codec call.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

constexpr size_t kPitchAlign = 256;
constexpr int kMaxLanesPerDevice = 8;

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int check_profile(int k, int m) {
  if (k < 1 || m < 1) return RS_E_INVALID_PROFILE;
  if (k + m > 256) return RS_E_UNSUPPORTED;
  return RS_OK;
}

// ---- coefficient tables -----------------------------------------------------------

// One launch group: up to kMaxRowsPerLaunch output rows over the same k inputs.
struct Group {
  std::vector<int> shard;     // shard index per row
  uint32_t verify_mask = 0;   // bit r: compare row r (Verify) instead of storing it
  std::vector<uint32_t> tabs; // [k][R][5] v_perm tables
  std::vector<uint8_t> ltabs;  // [k][32][W] LDS nibble tables (used for R >= 5)
  // the group's bit-sliced kernel (bitslice.hpp; compiled on demand), R >= kBitsliceMinRows
  std::shared_ptr<bs::Kernel> bsk;
};

struct Tables {
  int k = 0, m = 0;
  std::vector<int> valid;
  std::vector<int> missing;
  std::vector<int> check;
  std::vector<Group> groups;
};

// verify=false drops the check rows (plain Reconstruct).
std::shared_ptr<const Tables> build_tables(int k, int m, const uint8_t* present, bool verify) {
  DecodePlan dp;
  if (!decode_plan(k, m, present, dp)) return nullptr;
  auto t = std::make_shared<Tables>();
  t->k = k;
  t->m = m;
  t->valid = dp.valid;
  t->missing = dp.missing;
  if (verify) t->check = dp.check;
  const int nrows = static_cast<int>(t->missing.size() + t->check.size());
  for (int g0 = 0; g0 < nrows; g0 += kMaxRowsPerLaunch) {
    Group g;
    const int R = std::min(kMaxRowsPerLaunch, nrows - g0);
    g.tabs.assign(static_cast<size_t>(k) * R * kTabWords, 0);
    for (int r = 0; r < R; ++r) {
      const int row = g0 + r;
      const bool is_check = row >= static_cast<int>(t->missing.size());
      g.shard.push_back(is_check ? t->check[row - t->missing.size()] : t->missing[row]);
      if (is_check) g.verify_mask |= 1u << r;
      for (int i = 0; i < k; ++i)
        perm_tables(dp.rows.at(row, i), &g.tabs[(static_cast<size_t>(i) * R + r) * kTabWords]);
    }
    const size_t per_shard = 32u * nibble_width(R);
    g.ltabs.assign(static_cast<size_t>(k) * per_shard, 0);
    for (int i = 0; i < k; ++i) {
      uint8_t col[kMaxRowsPerLaunch] = {0};
      for (int r = 0; r < R; ++r) col[r] = dp.rows.at(g0 + r, i);
      nibble_tables(col, R, &g.ltabs[static_cast<size_t>(i) * per_shard]);
    }
    if (R >= kBitsliceMinRows && bs::mode() != bs::Mode::kOff) {
      std::vector<uint8_t> coef(static_cast<size_t>(R) * k);
      for (int r = 0; r < R; ++r)
        for (int i = 0; i < k; ++i) coef[static_cast<size_t>(r) * k + i] = dp.rows.at(g0 + r, i);
      g.bsk = bs::kernel_for(k, R, coef.data());
    }
    t->groups.push_back(std::move(g));
  }
  return t;
}

class TableCache {
 public:
  std::shared_ptr<const Tables> get(int k, int m, const uint8_t* present, bool verify) {
    std::string key;
    key.reserve(k + m + 8);
    key.append(reinterpret_cast<const char*>(&k), sizeof k);
    key.append(reinterpret_cast<const char*>(&m), sizeof m);
    key.push_back(verify ? 'v' : 'r');
    for (int i = 0; i < k + m; ++i) key.push_back(present[i] ? '1' : '0');
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = map_.find(key);
      if (it != map_.end()) return it->second;
    }
    auto t = build_tables(k, m, present, verify);
    if (!t) return nullptr;
    std::lock_guard<std::mutex> g(mu_);
    if (map_.size() >= kCap) map_.clear();
    map_.emplace(key, t);
    return t;
  }

 private:
  static constexpr size_t kCap = 4096;
  std::mutex mu_;
  std::unordered_map<std::string, std::shared_ptr<const Tables>> map_;
};

// ---- device buffers ------------------------------------------------------------------

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return RS_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, n) != hipSuccess) return RS_E_NOMEM;
    cap = n;
    return RS_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return RS_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    // Non-coherent: DMA into the default (coherent, fine-grained) pinned memory ran at
    // 9 GB/s for 4 MiB D2H copies and 34-41 GB/s at 64 MiB, against 50 / 57 GB/s here
    // (tools/host_ceilings.cpp). The host reads staging only after the
    // slot's event has completed, so coherence during the copy is never needed.
    static const unsigned flags =
        std::getenv("CALLFS_RS_PINNED_COHERENT") ? hipHostMallocDefault : hipHostMallocNonCoherent;
    if (hipHostMalloc(&p, n, flags) != hipSuccess) return RS_E_NOMEM;
    cap = n;
    return RS_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Host-coherent pinned memory that kernels read and write in place (the one-dispatch
// small-call path): the CPU fills it between calls, so device caches must not keep its
// lines across launches (as for rs_host_alloc buffers).
struct CoherentBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return RS_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    n = std::max<size_t>(n, 64u << 10);
    if (hipHostMalloc(&p, n, hipHostMallocCoherent) != hipSuccess) return RS_E_NOMEM;
    cap = n;
    return RS_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Layout facts the kernel dispatch keys its tile order on (ApplyArgs addr_tz,
// stripe_stride).
struct LayoutHint {
  int addr_tz = 0;
  uint64_t stripe_stride = 0;
  uint32_t in_misalign = 0;
  uint32_t out_misalign = 0;  // over every launch group's output pointers
};

// One pipeline stage of the host-memory path: a stream, a pinned chunk buffer and its
// device mirror ([n][cpitch]), and the pointer/coefficient tables for launches on it.
struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  DevBuf dev;
  HostBuf host;
  DevBuf meta;
  HostBuf hmeta;
  std::shared_ptr<const Tables> meta_tables;  // what `meta` currently holds
  size_t meta_pitch = 0;
  int meta_spc = 0;
  LayoutHint meta_hint;  // of the pointers in `meta`
  void* meta_base = nullptr;
  HostBuf hstat;         // per-stripe verify flags of the chunk in flight
  // one-dispatch small calls: staging the kernel works on in place (+ status words),
  // and the v_perm tables of the tables set it was last used with, per launch group
  CoherentBuf small;
  DevBuf small_counter;  // finished-block counter of the completion flag
  int small_seq = 0;     // sequence number of the last small call on this slot
  DevBuf small_tabs;
  std::shared_ptr<const Tables> small_tables;
  std::vector<size_t> small_tab_off;
  bool pending = false;  // a chunk's outputs wait in `host`
  int b0 = 0, count = 0;  // its stripes
  size_t off = 0, width = 0;  // and columns
};

constexpr int kMaxSlots = 6;
// Pipeline depth (slots per lane): CALLFS_RS_SLOTS overrides, 2..kMaxSlots.
int pipeline_slots() {
  static const int v = [] {
    const char* e = std::getenv("CALLFS_RS_SLOTS");
    const int x = e ? std::atoi(e) : 3;
    return std::max(2, std::min(kMaxSlots, x));
  }();
  return v;
}
// Column chunk: about this many bytes over all n shards per pipeline step
// (CALLFS_RS_CHUNK_BYTES overrides; DESIGN.md §7.4 has the sweep).
size_t chunk_bytes() {
  static const size_t v = [] {
    const char* e = std::getenv("CALLFS_RS_CHUNK_BYTES");
    const long long x = e ? std::atoll(e) : 0;
    return x >= (64 << 10) ? static_cast<size_t>(x) : (16u << 20);
  }();
  return v;
}

// Calls moving at most this many staging bytes (n shards rounded to 16 B, all stripes)
// take the one-dispatch small path (CALLFS_RS_SMALL_MAX_BYTES overrides; 0 turns it off).
size_t small_max_bytes() {
  static const size_t v = [] {
    const char* e = std::getenv("CALLFS_RS_SMALL_MAX_BYTES");
    return e ? static_cast<size_t>(std::strtoull(e, nullptr, 0)) : (2u << 20);
  }();
  return v;
}

// CALLFS_RS_INPLACE_PIPELINE=1: calls above the small limit run the chunk pipeline with
// in-place kernels on host-coherent staging instead of H2D / kernel / D2H (A/B)
bool inplace_pipeline() {
  static const bool on = [] {
    const char* e = std::getenv("CALLFS_RS_INPLACE_PIPELINE");
    return e && *e == '1';
  }();
  return on;
}

// Host spin on a flag a kernel releases with a system-scope store (rs_apply_small):
// true once *flag == want, false after `us` microseconds.
constexpr int kSmallSpinUs = 2000;
bool spin_until(const int* flag, int want, int us) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0;; ++i) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == want) return true;
    if ((i & 63u) == 63u &&
        std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(us))
      return false;
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#else
    std::this_thread::yield();
#endif
  }
}

struct Lane {
  Slot slot[kMaxSlots];
};

struct Device {
  int id = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::unique_ptr<Lane>> lanes;
  std::vector<Lane*> free_lanes;
};

// Device-side layout of everything one set of launches needs, packed into one buffer.
struct MetaLayout {
  size_t in_off = 0, status_off = 0, total = 0;
  std::vector<size_t> out_off, tab_off, ltab_off;
};

MetaLayout meta_layout(const Tables& t, int batch) {
  MetaLayout L;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off = round_up(off + bytes, 256);
    return o;
  };
  L.status_off = take(sizeof(int) * static_cast<size_t>(batch));
  L.in_off = take(sizeof(void*) * static_cast<size_t>(batch) * t.k);
  for (const Group& g : t.groups) {
    L.out_off.push_back(take(sizeof(void*) * static_cast<size_t>(batch) * g.shard.size()));
    L.tab_off.push_back(take(sizeof(uint32_t) * g.tabs.size()));
    L.ltab_off.push_back(take(g.ltabs.size()));
  }
  L.total = off;
  return L;
}

// Fill host staging for the meta buffer. shard_ptr(b, i) gives stripe b's shard i.
// Returns the layout hint: shard_addr_tz over the shards stripe 0's launches touch, and
// the stripe stride when every stripe sits at the same distance from the previous one.
template <class F>
LayoutHint fill_meta(const Tables& t, const MetaLayout& L, int batch, uint8_t* h, F shard_ptr) {
  std::memset(h + L.status_off, 0, sizeof(int) * static_cast<size_t>(batch));
  auto* in = reinterpret_cast<const uint8_t**>(h + L.in_off);
  uint32_t misalign = 0, out_misalign = 0;
  for (int b = 0; b < batch; ++b)
    for (int i = 0; i < t.k; ++i) {
      const uint8_t* p = shard_ptr(b, t.valid[i]);
      in[static_cast<size_t>(b) * t.k + i] = p;
      misalign |= static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)) & 15u;
    }
  for (size_t gi = 0; gi < t.groups.size(); ++gi) {
    const Group& g = t.groups[gi];
    auto* out = reinterpret_cast<uint8_t**>(h + L.out_off[gi]);
    const size_t R = g.shard.size();
    for (int b = 0; b < batch; ++b)
      for (size_t r = 0; r < R; ++r) {
        out[b * R + r] = const_cast<uint8_t*>(shard_ptr(b, g.shard[r]));
        out_misalign |= static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out[b * R + r])) & 15u;
      }
    std::memcpy(h + L.tab_off[gi], g.tabs.data(), g.tabs.size() * sizeof(uint32_t));
    std::memcpy(h + L.ltab_off[gi], g.ltabs.data(), g.ltabs.size());
  }
  std::vector<const void*> s0;
  for (int i : t.valid) s0.push_back(shard_ptr(0, i));
  for (const Group& g : t.groups)
    for (int i : g.shard) s0.push_back(shard_ptr(0, i));
  LayoutHint hint;
  hint.in_misalign = misalign;
  hint.out_misalign = out_misalign;
  hint.addr_tz = shard_addr_tz(s0.data(), static_cast<int>(s0.size()));
  if (batch > 1) {
    const int v = t.valid[0];
    auto addr = [&](int b) { return reinterpret_cast<uintptr_t>(shard_ptr(b, v)); };
    const uint64_t stride = addr(1) - addr(0);
    bool regular = true;
    for (int b = 2; b < batch && regular; ++b) regular = addr(b) - addr(b - 1) == stride;
    if (regular) hint.stripe_stride = stride;
  }
  return hint;
}

ApplyArgs group_args(const Tables& t, const MetaLayout& L, size_t gi, int batch, uint8_t* d,
                     size_t S, int status_stride, const LayoutHint& hint) {
  const Group& g = t.groups[gi];
  ApplyArgs a{};
  a.in_tab = reinterpret_cast<const uint8_t* const*>(d + L.in_off);
  a.out_tab = reinterpret_cast<uint8_t* const*>(d + L.out_off[gi]);
  a.tabs = reinterpret_cast<const uint32_t*>(d + L.tab_off[gi]);
  a.ltabs = d + L.ltab_off[gi];
  a.S = S;
  a.verify_mask = g.verify_mask;
  a.status = reinterpret_cast<int*>(d + L.status_off);
  a.status_stride = status_stride;
  a.K = t.k;
  a.R = static_cast<int>(g.shard.size());
  a.batch = batch;
  a.addr_tz = hint.addr_tz;
  a.stripe_stride = hint.stripe_stride;
  a.in_misalign = hint.in_misalign;
  a.out_misalign = hint.out_misalign;
  a.bs = g.bsk.get();
  return a;
}

// orders: per launch group, a TileOrder from rs_plan_tune or -1 (the rule); null = rule.
// ev: the first group's first dispatch records ev.start, the last group's last ev.stop.
hipError_t launch_groups(const Tables& t, const MetaLayout& L, int batch, uint8_t* d, size_t S,
                         hipStream_t s, int status_stride, const LayoutHint& hint,
                         const std::vector<int>* orders = nullptr, LaunchEvents ev = {}) {
  const size_t ng = t.groups.size();
  for (size_t gi = 0; gi < ng; ++gi) {
    const ApplyArgs a = group_args(t, L, gi, batch, d, S, status_stride, hint);
    // a plan's pinned or tuned order; else what rs_plan_tune measured for this shape on the
    // device (tune_table.hpp); else the rule
    int order = orders && gi < orders->size() ? (*orders)[gi] : -1;
    if (order < 0) order = tuned_order(a);
    LaunchEvents g;
    g.start = gi == 0 ? ev.start : nullptr;
    g.stop = gi + 1 == ng ? ev.stop : nullptr;
    hipError_t e = launch_apply(a, s, /*bytes_only=*/false, order, g);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

uint64_t algo_bytes(const Tables& t, size_t S, int batch) {
  // reads: k valid shards + compared parity; writes: missing shards.
  return static_cast<uint64_t>(batch) * S * (t.k + t.check.size() + t.missing.size());
}

}  // namespace

// ---- context ------------------------------------------------------------------------

// Allocations made by rs_host_alloc: [base, base+size) ranges the host path may DMA
// from / to directly.
class PinnedRegistry {
 public:
  void add(void* p, size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    ranges_[reinterpret_cast<uintptr_t>(p)] = n;
  }
  bool remove(void* p) {
    std::lock_guard<std::mutex> g(mu_);
    return ranges_.erase(reinterpret_cast<uintptr_t>(p)) == 1;
  }
  // size of the allocation starting at p (0 when p is not one)
  size_t size_of(void* p) const {
    std::lock_guard<std::mutex> g(mu_);
    auto it = ranges_.find(reinterpret_cast<uintptr_t>(p));
    return it == ranges_.end() ? 0 : it->second;
  }
  // true when [p, p+n) lies inside one registered allocation
  bool contains(const void* p, size_t n) const {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> g(mu_);
    auto it = ranges_.upper_bound(a);
    if (it == ranges_.begin()) return false;
    --it;
    return a >= it->first && a + n <= it->first + it->second;
  }
  bool empty() const {
    std::lock_guard<std::mutex> g(mu_);
    return ranges_.empty();
  }
  std::vector<void*> all() const {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<void*> v;
    for (const auto& r : ranges_) v.push_back(reinterpret_cast<void*>(r.first));
    return v;
  }

 private:
  mutable std::mutex mu_;
  std::map<uintptr_t, size_t> ranges_;
};

// Idle rs_host_alloc buffers kept for reuse. Page-locking a fresh buffer costs about
// 0.2 s per 384 MiB, so a server that allocates a pinned body per request and frees it
// after the call ran 25-30x slower than one that reuses buffers (RS(4,2) 256 MiB,
// zero-copy: 1.6 vs 48 GiB/s encode). rs_host_free parks a buffer here;
// rs_host_alloc takes the smallest parked buffer that fits without wasting more than a
// quarter of it, both sides counted in 2 MiB granules. Parked bytes are capped by
// CALLFS_RS_HOST_POOL_BYTES (default 4 GiB;
// 0 disables parking): beyond it the largest parked buffers are released.
class HostPool {
 public:
  struct Buf {
    void* p;
    size_t cap;
  };
  // a parked buffer of at least n bytes, or {nullptr, 0}
  Buf take(size_t n) {
    // compare in allocation granules: a 4 KiB or 1 MiB request was allocated as one
    // 2 MiB granule, and that buffer must serve the next request of the same size
    const size_t want = granule(n);
    std::lock_guard<std::mutex> g(mu_);
    auto it = idle_.lower_bound(want);
    if (it == idle_.end() || it->first - want > it->first / 4) return {nullptr, 0};
    Buf b{it->second, it->first};
    idle_bytes_ -= it->first;
    idle_.erase(it);
    return b;
  }
  // park a buffer; returns the buffers to release now (over the cap)
  std::vector<void*> put(void* p, size_t cap) {
    std::vector<void*> drop;
    std::lock_guard<std::mutex> g(mu_);
    if (cap > limit()) {
      drop.push_back(p);
      return drop;
    }
    idle_.emplace(cap, p);
    idle_bytes_ += cap;
    while (idle_bytes_ > limit() && !idle_.empty()) {
      auto last = std::prev(idle_.end());
      idle_bytes_ -= last->first;
      drop.push_back(last->second);
      idle_.erase(last);
    }
    return drop;
  }
  std::vector<void*> drain() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<void*> all;
    for (auto& kv : idle_) all.push_back(kv.second);
    idle_.clear();
    idle_bytes_ = 0;
    return all;
  }
  size_t idle_bytes() {
    std::lock_guard<std::mutex> g(mu_);
    return idle_bytes_;
  }
  // capacity rs_host_alloc gives a fresh buffer of n bytes (2 MiB granules, so buffers
  // freed by one request fit the next request of similar size)
  static size_t granule(size_t n) { return (n + kGranule - 1) / kGranule * kGranule; }
  static constexpr size_t kGranule = 2u << 20;

 private:
  static size_t limit() {
    static const size_t v = [] {
      const char* e = std::getenv("CALLFS_RS_HOST_POOL_BYTES");
      return e ? static_cast<size_t>(std::strtoull(e, nullptr, 0)) : (4ull << 30);
    }();
    return v;
  }
  std::mutex mu_;
  std::multimap<size_t, void*> idle_;
  size_t idle_bytes_ = 0;
};

struct rs_ctx {
  std::vector<std::unique_ptr<Device>> devs;
  std::atomic<unsigned> rr{0};
  TableCache cache;
  CopyPool pool;
  PinnedRegistry pinned;
  HostPool host_pool;

  ~rs_ctx() {
    for (void* p : pinned.all()) (void)hipHostFree(p);  // buffers the caller did not free
    for (void* p : host_pool.drain()) (void)hipHostFree(p);
    for (auto& d : devs) {
      (void)hipSetDevice(d->id);
      for (auto& l : d->lanes) {
        for (Slot& sl : l->slot) {
          if (sl.stream) (void)hipStreamSynchronize(sl.stream);
          sl.dev.release();
          sl.host.release();
          sl.meta.release();
          sl.hmeta.release();
          sl.hstat.release();
          sl.small.release();
          sl.small_tabs.release();
          sl.small_counter.release();
          if (sl.done) (void)hipEventDestroy(sl.done);
          if (sl.stream) (void)hipStreamDestroy(sl.stream);
        }
      }

    }
  }

  Device* device(int id) {
    for (auto& d : devs)
      if (d->id == id) return d.get();
    return nullptr;
  }

  Lane* acquire(Device* d) {
    std::unique_lock<std::mutex> g(d->mu);
    for (;;) {
      if (!d->free_lanes.empty()) {
        Lane* l = d->free_lanes.back();
        d->free_lanes.pop_back();
        return l;
      }
      if (static_cast<int>(d->lanes.size()) < kMaxLanesPerDevice) {
        auto l = std::make_unique<Lane>();
        if (hipSetDevice(d->id) != hipSuccess) return nullptr;
        for (Slot& sl : l->slot)
          if (hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess ||
              hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess) {
            for (Slot& s : l->slot) {  // a partly built lane is not kept: free what exists
              if (s.done) (void)hipEventDestroy(s.done);
              if (s.stream) (void)hipStreamDestroy(s.stream);
            }
            return nullptr;
          }
        d->lanes.push_back(std::move(l));
        return d->lanes.back().get();
      }
      d->cv.wait(g);
    }
  }

  void release(Device* d, Lane* l) {
    {
      std::lock_guard<std::mutex> g(d->mu);
      d->free_lanes.push_back(l);
    }
    d->cv.notify_one();
  }
};

namespace {

struct LaneGuard {
  rs_ctx* ctx;
  Device* dev;
  Lane* lane;
  ~LaneGuard() {
    if (lane) ctx->release(dev, lane);
  }
};

// Host-memory path (Codec.Encode/Decode ends, codec.go:21-78) over `batch` stripes that
// share one table set and one shard size S. Work is cut into chunks that rotate through
// the lane's kSlots slots: a chunk is a block of whole stripes when a stripe is small
// (many stripes per H2D / launch / D2H), otherwise one column range [off, off+w) of a
// single stripe. Per chunk: copy-pool copies of the input shards into pinned memory
// ([stripe][n][cpitch]), H2D, the kernel groups, D2H of the written shards (and of the
// per-stripe status words when there are verify rows) on the slot's stream; the CPU
// copies chunk j in while the GPU/DMA work on chunks j-1 and j-2, and copies chunk
// j-kSlots out. in(b, i)/out(b, i) give host buffers by stripe and shard index.
// stripe_status (nullable, `batch` ints) receives 1 for stripes whose verify rows
// mismatched. Returns RS_OK, RS_E_CORRUPT (some stripe mismatched) or an error.
// Decode's join/trim target (codec.go:67-77): data shard i's column c belongs at
// out[i*S + c] when that is below len (= min(originalSize, k*S)). The single-stripe
// host path writes it while the columns pass through the copy pool (a tee on the
// staging copies), instead of a separate k*S pass after the pipeline.
struct Join {
  uint8_t* out;
  size_t len;
  size_t S;  // full shard size (a column part's offset is added per part)
  int k;
  bool done = false;  // set when the pipeline wrote every join byte
};

// Tee target for shard i's columns [col, col+w) or {nullptr, 0}.
std::pair<uint8_t*, size_t> join_span(const Join* j, int i, size_t col, size_t w) {
  if (!j || i >= j->k) return {nullptr, 0};
  const size_t pos = static_cast<size_t>(i) * j->S + col;
  if (pos >= j->len) return {nullptr, 0};
  return {j->out + pos, std::min(w, j->len - pos)};
}

template <class InF, class OutF>
int run_host_impl(rs_ctx* ctx, Lane& L, int device, const std::shared_ptr<const Tables>& tp,
                  size_t S, int batch, InF host_in, OutF host_out, int* stripe_status,
                  const Join* join, size_t col0);

template <class InF, class OutF>
int run_on(rs_ctx* ctx, Device* dev, const std::shared_ptr<const Tables>& tp, size_t S,
           int batch, InF host_in, OutF host_out, int* stripe_status,
           const Join* join = nullptr, size_t col0 = 0) {
  LaneGuard lg{ctx, dev, ctx->acquire(dev)};
  if (!lg.lane) return RS_E_HIP;
  const int rc =
      run_host_impl(ctx, *lg.lane, dev->id, tp, S, batch, host_in, host_out, stripe_status,
                    join, col0);
  if (rc != RS_OK && rc != RS_E_CORRUPT) {
    // never hand a lane with work in flight to the next caller
    for (Slot& sl : lg.lane->slot) {
      if (sl.stream) (void)hipStreamSynchronize(sl.stream);
      sl.pending = false;
    }
  }
  return rc;
}

// Ways to split one large object's columns over (device, lane) pairs (dispatch.hpp):
// objects of at least CALLFS_RS_SPLIT_MIN_BYTES over all n shards (default 256 MiB)
// are split CALLFS_RS_SPLIT_WAYS ways (default: one per device), each way on its own
// lane, so a multi-GPU host moves one object over every GPU's PCIe link at once.
int split_ways(const rs_ctx* ctx, size_t S, int n, int batch) {
  // read per call (cheap next to a >= 256 MiB object; tests change them in-process)
  const char* e = std::getenv("CALLFS_RS_SPLIT_MIN_BYTES");
  const unsigned long long min_bytes = e ? std::strtoull(e, nullptr, 0) : (256ull << 20);
  const char* w = std::getenv("CALLFS_RS_SPLIT_WAYS");
  const int ways_req = split_ways_request(w);  // unset: one per device; <= 1: no split
  return callfs::split_ways(ctx->devs.size(), kMaxLanesPerDevice, S, n, batch, min_bytes,
                            ways_req);
}

template <class InF, class OutF>
int run_host(rs_ctx* ctx, const std::shared_ptr<const Tables>& tp, size_t S, int batch,
             InF host_in, OutF host_out, int* stripe_status = nullptr,
             const Join* join = nullptr) {
  if (ctx->devs.empty()) return RS_E_HIP;
  const size_t nd = ctx->devs.size();
  const unsigned base = ctx->rr.fetch_add(1);
  const int ways = split_ways(ctx, S, tp->k + tp->m, batch);
  if (ways == 1)
    return run_on(ctx, ctx->devs[device_slot(base, 0, nd)].get(), tp, S, batch, host_in,
                  host_out, stripe_status, join, 0);
  const std::vector<size_t> c = column_parts(S, ways);  // parts [c[p], c[p+1])
  std::vector<int> rc(ways, RS_OK), flag(ways, 0);
  std::vector<std::thread> th;
  for (int p = 0; p < ways; ++p)
    th.emplace_back([&, p] {
      const size_t c0 = c[p];
      if (c[p + 1] <= c0) return;
      rc[p] = run_on(ctx, ctx->devs[device_slot(base, p, nd)].get(), tp, c[p + 1] - c0, 1,
                     [&](int b, int i) { return host_in(b, i) + c0; },
                     [&](int b, int i) { return host_out(b, i) + c0; }, &flag[p], join, c0);
    });
  for (auto& t : th) t.join();
  int out = RS_OK;
  for (int p = 0; p < ways; ++p) {
    if (rc[p] != RS_OK && rc[p] != RS_E_CORRUPT) return rc[p];
    if (rc[p] == RS_E_CORRUPT) out = RS_E_CORRUPT;
  }
  if (out == RS_E_CORRUPT && stripe_status) stripe_status[0] = 1;
  return out;
}

// Single-stripe form used by the per-object entry points.
template <class InF, class OutF>
int run_host1(rs_ctx* ctx, const std::shared_ptr<const Tables>& tp, size_t S, InF in, OutF out,
              const Join* join = nullptr) {
  return run_host(ctx, tp, S, 1, [&](int, int i) { return in(i); },
                  [&](int, int i) { return out(i); }, nullptr, join);
}

// Runs [first, last] of consecutive values in an index list (sorted here).
std::vector<std::pair<int, int>> index_runs(std::vector<int> v) {
  std::sort(v.begin(), v.end());
  std::vector<std::pair<int, int>> runs;
  for (int x : v) {
    if (!runs.empty() && runs.back().second + 1 == x) runs.back().second = x;
    else runs.push_back({x, x});
  }
  return runs;
}

// In-place kernels on host-coherent staging (rs_apply_small): make `sl` ready for
// tables `tp` with `bytes` of staging -- the v_perm tables and shard indices of every
// launch group uploaded to device memory once per (slot, tables), and the finished-block
// counter of the completion flag.
int prep_inplace(Slot& sl, const std::shared_ptr<const Tables>& tp, size_t bytes) {
  int rc;
  if ((rc = sl.small.ensure(bytes))) return rc;
  if (!sl.small_counter.p) {
    if ((rc = sl.small_counter.ensure(256))) return rc;
    HIPCHK(hipMemset(sl.small_counter.p, 0, 256));
  }
  if (sl.small_tables == tp) return RS_OK;
  const Tables& t = *tp;
  // per launch group: [v_perm tables][idx: 256 input + 16 row shard indices]
  std::vector<size_t> off;
  size_t tot = 0;
  for (const Group& g : t.groups) {
    off.push_back(tot);
    tot = round_up(tot + g.tabs.size() * sizeof(uint32_t) + 272, 256);
  }
  sl.small_tables = nullptr;
  if ((rc = sl.small_tabs.ensure(tot))) return rc;
  std::vector<uint8_t> h(tot, 0);
  for (size_t gi = 0; gi < t.groups.size(); ++gi) {
    const Group& g = t.groups[gi];
    const size_t tb = g.tabs.size() * sizeof(uint32_t);
    std::memcpy(h.data() + off[gi], g.tabs.data(), tb);
    uint8_t* ix = h.data() + off[gi] + tb;
    for (int i = 0; i < t.k; ++i) ix[i] = static_cast<uint8_t>(t.valid[i]);
    for (size_t r = 0; r < g.shard.size(); ++r) ix[256 + r] = static_cast<uint8_t>(g.shard[r]);
  }
  HIPCHK(hipMemcpy(sl.small_tabs.p, h.data(), tot, hipMemcpyHostToDevice));
  sl.small_tables = tp;
  sl.small_tab_off = off;
  return RS_OK;
}

// One chunk in place: `cnt` stripes at base + b*sp, shard i at + i*cp, w bytes per shard;
// the last launch group releases `seq` into *done when all its blocks have finished.
hipError_t launch_inplace(Slot& sl, const Tables& t, uint8_t* base, size_t sp, size_t cp,
                          size_t w, int cnt, int* st, int* done, int seq) {
  for (size_t gi = 0; gi < t.groups.size(); ++gi) {
    const Group& g = t.groups[gi];
    SmallArgs A{};
    A.base = base;
    A.spitch = sp;
    A.cpitch = cp;
    A.nvec = static_cast<uint32_t>((w + 15) / 16);
    A.S = static_cast<uint32_t>(w);
    A.K = t.k;
    A.R = static_cast<int>(g.shard.size());
    A.batch = cnt;
    A.verify_mask = g.verify_mask;
    const uint8_t* tb = static_cast<uint8_t*>(sl.small_tabs.p) + sl.small_tab_off[gi];
    A.tabs = reinterpret_cast<const uint32_t*>(tb);
    A.idx = tb + g.tabs.size() * sizeof(uint32_t);
    for (int i = 0; i < std::min(t.k, 16); ++i)
      A.idx_in[i >> 2] |= static_cast<uint32_t>(t.valid[i]) << (8 * (i & 3));
    for (size_t r = 0; r < g.shard.size(); ++r)
      A.idx_out[r >> 2] |= static_cast<uint32_t>(g.shard[r]) << (8 * (r & 3));
    A.status = st;
    A.done = gi + 1 == t.groups.size() ? done : nullptr;
    A.counter = static_cast<unsigned*>(sl.small_counter.p);
    A.seq = seq;
    const hipError_t e = launch_small(A, sl.stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <class InF, class OutF>
int run_host_impl(rs_ctx* ctx, Lane& L, int device, const std::shared_ptr<const Tables>& tp,
                  size_t S, int batch, InF host_in, OutF host_out, int* stripe_status,
                  const Join* join, size_t col0) {
  if (batch != 1) join = nullptr;  // only single-object decodes join
  const Tables& t = *tp;
  HIPCHK(hipSetDevice(device));
  const int n = t.k + t.m;
  const bool verify = !t.check.empty();

  std::vector<int> ins(t.valid);
  ins.insert(ins.end(), t.check.begin(), t.check.end());
  const std::vector<int>& outs = t.missing;
  const int in_lo = *std::min_element(ins.begin(), ins.end());
  const int in_hi = *std::max_element(ins.begin(), ins.end());
  const int out_lo = outs.empty() ? 0 : *std::min_element(outs.begin(), outs.end());
  const int out_hi = outs.empty() ? -1 : *std::max_element(outs.begin(), outs.end());

  // chunk shape: cw bytes per shard (a multiple of 4 KiB unless the whole shard) and
  // spc stripes per chunk (>1 only when a whole stripe fits several times in a chunk)
  size_t cw = S;
  int spc = 1;
  const size_t cb = chunk_bytes();
  if (S * n > cb) {
    cw = std::max<size_t>(4096, cb / n / 4096 * 4096);
  } else {
    const size_t per = round_up(S, kPitchAlign) * n;
    spc = static_cast<int>(std::min<size_t>(static_cast<size_t>(batch), std::max<size_t>(1, cb / per)));
  }
  const size_t cpitch = round_up(cw, kPitchAlign);
  const size_t spitch = cpitch * n;  // one stripe in a slot's staging buffer
  const size_t ncol = (S + cw - 1) / cw;
  const size_t nblk = (static_cast<size_t>(batch) + spc - 1) / spc;
  const size_t nchunks = ncol * nblk;
  const int kSlots = pipeline_slots();
  const int nslots = static_cast<int>(std::min<size_t>(nchunks, kSlots));
  const MetaLayout ML = meta_layout(t, spc);
  // Small stripes move as one contiguous row range (rows that are not inputs ride
  // along). Larger chunks move one copy per run of consecutive shard indices: each copy
  // on a stream costs ~9 us of gap, so one copy per shard was much slower than one per
  // run.
  const bool coalesce = spitch <= (4u << 20);
  const std::vector<std::pair<int, int>> in_runs = index_runs(ins), out_runs = index_runs(outs);

  // Zero-copy: when every caller buffer lies in rs_host_alloc memory (page-locked and
  // mapped into the device's address space at the same address), the kernels read and
  // write the caller's bytes over PCIe in one launch set over the whole call -- no
  // staging copies, no chunk pipeline, nothing for the CPU but the join of present
  // data shards. RS(10,4) 64 MiB: 43.7 GiB/s vs 36.7 for H2D + launch + D2H
  // (tests/perf/zerocopy_probe.py).
  // Threshold: 48 KiB per shard over the call (S x batch), i.e. 48 KiB x n over all n
  // shards. Below it the one-dispatch path on the library's coherent staging is faster;
  // tools/jobs.sh zc_threshold (profiles/r04/zc_threshold/zc.jsonl, GiB/s enc / dec, 1 thread,
  // zero-copy vs one-dispatch): RS(4,2) 128 KiB objects 4.6 / 4.2 vs 6.2 / 5.9, 256 KiB
  // 8.7 / 7.7 vs 5.3 / 5.3; RS(10,4) 384 KiB 9.6 / 8.9 vs 9.0 / 9.1, 512 KiB 11.7 / 11.4 vs
  // 8.0 / 10.0; RS(16,4) 512 KiB 11.2 / 9.1 vs 10.9 / 9.2, 1 MiB 20.9 / 17.1 vs 10.8 / 14.6.
  // (Round 2's 128 KiB over all shards predates the one-dispatch path.)
  // CALLFS_RS_ZERO_COPY_MIN_BYTES sets it in bytes over all n shards instead.
  static const long long zc_env = [] {
    const char* e = std::getenv("CALLFS_RS_ZERO_COPY_MIN_BYTES");
    return e ? static_cast<long long>(std::strtoull(e, nullptr, 0)) : -1LL;
  }();
  const unsigned long long zc_min =
      zc_env >= 0 ? static_cast<unsigned long long>(zc_env) : (48ull << 10) * static_cast<unsigned long long>(n);
  bool direct = !ctx->pinned.empty() &&
                static_cast<unsigned long long>(S) * n * batch >= zc_min;
  for (int b = 0; direct && b < batch; ++b) {
    for (int i : ins) direct = direct && ctx->pinned.contains(host_in(b, i), S);
    for (int i : outs) direct = direct && ctx->pinned.contains(host_out(b, i), S);
  }
  if (direct && join) direct = ctx->pinned.contains(join->out, join->len);
  if (direct) {
    Slot& sl = L.slot[0];
    const MetaLayout DL = meta_layout(t, batch);
    int rc;
    if ((rc = sl.meta.ensure(DL.total)) || (rc = sl.hmeta.ensure(DL.total)) ||
        (rc = sl.hstat.ensure(sizeof(int) * batch)))
      return rc;
    sl.meta_tables = nullptr;  // the staged path refills its tables next time
    std::vector<char> is_out(n, 0);
    for (int i : outs) is_out[i] = 1;
    const LayoutHint hint = fill_meta(t, DL, batch, static_cast<uint8_t*>(sl.hmeta.p), [&](int b, int i) {
      return is_out[i] ? static_cast<const uint8_t*>(host_out(b, i)) : host_in(b, i);
    });
    auto* meta = static_cast<uint8_t*>(sl.meta.p);
    HIPCHK(hipMemcpyAsync(meta, sl.hmeta.p, DL.total, hipMemcpyHostToDevice, sl.stream));
    HIPCHK(launch_groups(t, DL, batch, meta, S, sl.stream, 1, hint));
    if (verify)
      HIPCHK(hipMemcpyAsync(sl.hstat.p, meta + DL.status_off, sizeof(int) * batch,
                            hipMemcpyDeviceToHost, sl.stream));
    HIPCHK(hipEventRecord(sl.done, sl.stream));
    // decode's join: present data shards go to `out` while the kernels run,
    // reconstructed ones once they have landed
    auto join_segs = [&](bool present) {
      std::vector<CopyPool::Seg> js_segs;
      for (int i = 0; join && i < t.k; ++i) {
        if (static_cast<bool>(is_out[i]) == present) continue;
        const auto js = join_span(join, i, col0, S);
        if (js.first)
          js_segs.push_back({js.first, present ? host_in(0, i) : host_out(0, i), js.second});
      }
      ctx->pool.run(js_segs);
    };
    join_segs(true);
    HIPCHK(hipEventSynchronize(sl.done));
    join_segs(false);
    bool corrupt = false;
    if (verify) {
      const int* st = static_cast<const int*>(sl.hstat.p);
      for (int b = 0; b < batch; ++b)
        if (st[b]) {
          corrupt = true;
          if (stripe_status) stripe_status[b] = 1;
        }
    }
    return corrupt ? RS_E_CORRUPT : RS_OK;
  }

  // In-place kernels on host-coherent staging (rs_apply_small): the kernel reads the
  // inputs and writes the outputs over PCIe, one dispatch per chunk and launch group, and
  // the host spins on the kernel's completion flag. The staged path spends three dependent
  // dispatches (H2D, kernel, D2H) per chunk, which bound 4 KiB calls at ~29 us
  // (DESIGN.md §7.4). Calls of at most CALLFS_RS_SMALL_MAX_BYTES of staging run as one
  // chunk on slot 0; with CALLFS_RS_INPLACE_PIPELINE=1 (A/B) larger calls run the staged
  // path's chunk pipeline with in-place kernels instead of H2D / kernel / D2H.
  const size_t cp16 = round_up(S, 16), sp16 = cp16 * n;
  const bool one_chunk = sp16 * static_cast<size_t>(batch) <= small_max_bytes() &&
                         batch <= 65535 && S <= 0xFFFFFFF0u;
  if (one_chunk || (inplace_pipeline() && cw <= 0xFFFFFFF0u && spc <= 65535)) {
    // chunk geometry: the whole call, or the staged path's chunks
    const size_t icw = one_chunk ? S : cw, icp = round_up(icw, 16), isp = icp * n;
    const int ispc = one_chunk ? batch : spc;
    const size_t incol = one_chunk ? 1 : ncol, inblk = one_chunk ? 1 : nblk;
    const size_t ichunks = incol * inblk;
    const int islots = one_chunk ? 1 : static_cast<int>(std::min<size_t>(ichunks, kSlots));
    const size_t stat_off = round_up(isp * ispc, 256);
    const size_t done_off = round_up(stat_off + sizeof(int) * ispc, 256);
    for (int si = 0; si < islots; ++si) {
      int rc = prep_inplace(L.slot[si], tp, done_off + 256);
      if (rc) return rc;
      L.slot[si].pending = false;
    }
    bool corrupt = false;
    std::vector<CopyPool::Seg> segs;
    // waits for the slot's chunk and appends its output copies to `segs`
    auto drain = [&](Slot& sl) -> int {
      if (!sl.pending) return RS_OK;
      auto* base = static_cast<uint8_t*>(sl.small.p);
      const int* done = reinterpret_cast<const int*>(base + done_off);
      // ~5 us sooner than the runtime's completion signal; past kSmallSpinUs the stream
      // wait, which also reports a faulted kernel
      if (!spin_until(done, sl.small_seq, kSmallSpinUs)) HIPCHK(hipStreamSynchronize(sl.stream));
      if (verify) {
        const int* st = reinterpret_cast<const int*>(base + stat_off);
        for (int b = 0; b < sl.count; ++b)
          if (st[b]) {
            corrupt = true;
            if (stripe_status) stripe_status[sl.b0 + b] = 1;
          }
      }
      for (int b = 0; b < sl.count; ++b)
        for (int i : outs) {
          const auto tee = join_span(join, i, col0 + sl.off, sl.width);
          segs.push_back({host_out(sl.b0 + b, i) + sl.off, base + isp * b + icp * i, sl.width,
                          tee.first, tee.second});
        }
      sl.pending = false;
      return RS_OK;
    };
    for (size_t j = 0; j < ichunks; ++j) {
      Slot& sl = L.slot[j % islots];
      segs.clear();
      int rc = drain(sl);
      if (rc) return rc;
      const int b0 = static_cast<int>(j / incol) * ispc;
      const int cnt = std::min(ispc, batch - b0);
      const size_t off = (j % incol) * icw, w = std::min(icw, S - off);
      auto* base = static_cast<uint8_t*>(sl.small.p);
      for (int b = 0; b < cnt; ++b)
        for (int i : ins) {
          const auto tee = join_span(join, i, col0 + off, w);
          segs.push_back({base + isp * b + icp * i, host_in(b0 + b, i) + off, w, tee.first,
                          tee.second});
        }
      ctx->pool.run(segs);
      int* st = reinterpret_cast<int*>(base + stat_off);
      int* done = reinterpret_cast<int*>(base + done_off);
      sl.small_seq = sl.small_seq >= 0x3fffffff ? 1 : sl.small_seq + 1;  // never 0
      // a fresh or moved buffer holds whatever it held: clear the flag before the launch
      __atomic_store_n(done, 0, __ATOMIC_RELEASE);
      if (verify) std::memset(st, 0, sizeof(int) * cnt);
      HIPCHK(launch_inplace(sl, t, base, isp, icp, w, cnt, st, done, sl.small_seq));
      sl.pending = true;
      sl.b0 = b0;
      sl.count = cnt;
      sl.off = off;
      sl.width = w;
    }
    for (size_t j = ichunks > static_cast<size_t>(islots) ? ichunks - islots : 0; j < ichunks; ++j) {
      segs.clear();
      int rc = drain(L.slot[j % islots]);
      if (rc) return rc;
      ctx->pool.run(segs);
    }
    return corrupt ? RS_E_CORRUPT : RS_OK;
  }

  for (int si = 0; si < nslots; ++si) {
    Slot& sl = L.slot[si];
    int rc;
    if ((rc = sl.dev.ensure(spitch * spc)) || (rc = sl.host.ensure(spitch * spc)) ||
        (rc = sl.meta.ensure(ML.total)) || (rc = sl.hmeta.ensure(ML.total)) ||
        (rc = sl.hstat.ensure(sizeof(int) * spc)))
      return rc;
    if (sl.meta_tables != tp || sl.meta_pitch != cpitch || sl.meta_spc != spc ||
        sl.meta_base != sl.dev.p) {
      auto* base = static_cast<uint8_t*>(sl.dev.p);
      sl.meta_hint = fill_meta(t, ML, spc, static_cast<uint8_t*>(sl.hmeta.p),
                             [&](int b, int i) { return base + spitch * b + cpitch * i; });
      HIPCHK(hipMemcpyAsync(sl.meta.p, sl.hmeta.p, ML.total, hipMemcpyHostToDevice, sl.stream));
      sl.meta_tables = tp;
      sl.meta_pitch = cpitch;
      sl.meta_spc = spc;
      sl.meta_base = sl.dev.p;
    }
    sl.pending = false;
  }

  bool corrupt = false;
  std::vector<CopyPool::Seg> segs;
  // Waits for the slot's chunk and appends its output copies to `segs` (run by the
  // caller together with the next chunk's input copies: one pool job per step; the
  // slot's input and output rows are disjoint).
  auto drain = [&](Slot& sl) -> int {
    if (!sl.pending) return RS_OK;
    HIPCHK(hipEventSynchronize(sl.done));
    auto* h = static_cast<uint8_t*>(sl.host.p);
    for (int b = 0; b < sl.count; ++b)
      for (int i : outs) {
        const auto tee = join_span(join, i, col0 + sl.off, sl.width);
        segs.push_back({host_out(sl.b0 + b, i) + sl.off, h + spitch * b + cpitch * i, sl.width,
                        tee.first, tee.second});
      }
    if (verify) {
      const int* st = static_cast<const int*>(sl.hstat.p);
      for (int b = 0; b < sl.count; ++b)
        if (st[b]) {
          corrupt = true;
          if (stripe_status) stripe_status[sl.b0 + b] = 1;
        }
    }
    sl.pending = false;
    return RS_OK;
  };

  int* dstatus = nullptr;
  for (size_t j = 0; j < nchunks; ++j) {
    Slot& sl = L.slot[j % kSlots];
    segs.clear();
    int rc = drain(sl);
    if (rc) return rc;
    const int b0 = static_cast<int>(j / ncol) * spc;
    const int cnt = std::min(spc, batch - b0);
    const size_t off = (j % ncol) * cw, w = std::min(cw, S - off);
    auto* h = static_cast<uint8_t*>(sl.host.p);
    auto* d = static_cast<uint8_t*>(sl.dev.p);
    auto* meta = static_cast<uint8_t*>(sl.meta.p);
    dstatus = reinterpret_cast<int*>(meta + ML.status_off);
    for (int b = 0; b < cnt; ++b)
      for (int i : ins) {
        const auto tee = join_span(join, i, col0 + off, w);
        segs.push_back({h + spitch * b + cpitch * i, host_in(b0 + b, i) + off, w, tee.first,
                        tee.second});
      }
    ctx->pool.run(segs);
    if (coalesce) {
      const size_t bytes = spitch * (cnt - 1) + cpitch * (in_hi - in_lo) + w;
      HIPCHK(hipMemcpyAsync(d + cpitch * in_lo, h + cpitch * in_lo, bytes,
                            hipMemcpyHostToDevice, sl.stream));
    } else {
      // one copy per run of consecutive shard indices of every stripe in the chunk
      for (int b = 0; b < cnt; ++b)
        for (const auto& r : in_runs) {
          const size_t o = spitch * b + cpitch * r.first;
          HIPCHK(hipMemcpyAsync(d + o, h + o, cpitch * (r.second - r.first) + w,
                                hipMemcpyHostToDevice, sl.stream));
        }
    }
    if (verify) HIPCHK(hipMemsetAsync(dstatus, 0, sizeof(int) * cnt, sl.stream));
    HIPCHK(launch_groups(t, ML, cnt, meta, w, sl.stream, 1, sl.meta_hint));
    if (!outs.empty()) {
      if (coalesce) {
        const size_t bytes = spitch * (cnt - 1) + cpitch * (out_hi - out_lo) + w;
        HIPCHK(hipMemcpyAsync(h + cpitch * out_lo, d + cpitch * out_lo, bytes,
                              hipMemcpyDeviceToHost, sl.stream));
      } else {
        for (int b = 0; b < cnt; ++b)
          for (const auto& r : out_runs) {
            const size_t o = spitch * b + cpitch * r.first;
            HIPCHK(hipMemcpyAsync(h + o, d + o, cpitch * (r.second - r.first) + w,
                                  hipMemcpyDeviceToHost, sl.stream));
          }
      }
    }
    if (verify)
      HIPCHK(hipMemcpyAsync(sl.hstat.p, dstatus, sizeof(int) * cnt, hipMemcpyDeviceToHost,
                            sl.stream));
    HIPCHK(hipEventRecord(sl.done, sl.stream));
    sl.pending = true;
    sl.b0 = b0;
    sl.count = cnt;
    sl.off = off;
    sl.width = w;
  }
  for (size_t j = nchunks > static_cast<size_t>(kSlots) ? nchunks - kSlots : 0; j < nchunks; ++j) {
    segs.clear();
    int rc = drain(L.slot[j % kSlots]);
    if (rc) return rc;
    ctx->pool.run(segs);
  }
  return corrupt ? RS_E_CORRUPT : RS_OK;
}

// Reconstruct's argument checks (upstream checkShards(shards, true)).
int check_lens(int n, const size_t* lens, bool nilok, size_t* S, int* npresent) {
  size_t size = 0;
  for (int i = 0; i < n; ++i)
    if (lens[i]) {
      size = lens[i];
      break;
    }
  if (size == 0) return RS_E_NO_DATA;
  int np = 0;
  for (int i = 0; i < n; ++i) {
    if (lens[i] != size && (lens[i] != 0 || !nilok)) return RS_E_SHARD_SIZE;
    np += lens[i] != 0;
  }
  *S = size;
  *npresent = np;
  return RS_OK;
}

// Shared by rs_reconstruct / rs_codec_decode. verify=true fuses upstream Verify.
int reconstruct_host(rs_ctx* ctx, int k, int m, uint8_t* const* shards, size_t* lens,
                     bool verify, Join* join = nullptr) {
  const int n = k + m;
  size_t S = 0;
  int np = 0;
  int rc = check_lens(n, lens, true, &S, &np);
  if (rc) return rc;
  if (np < k) return RS_E_TOO_FEW_SHARDS;
  if (np == n && !verify) return RS_OK;
  for (int i = 0; i < n; ++i)
    if (!shards[i]) return RS_E_ARG;
  uint8_t present[256];
  for (int i = 0; i < n; ++i) present[i] = lens[i] != 0;
  auto t = ctx->cache.get(k, m, present, verify);
  if (!t) return RS_E_SINGULAR;
  if (t->groups.empty()) return RS_OK;
  if (join) {
    join->S = S;
    join->len = std::min(join->len, S * k);
  }
  rc = run_host1(ctx, t, S, [&](int i) { return shards[i]; }, [&](int i) { return shards[i]; },
                 join);
  if (rc == RS_OK || rc == RS_E_CORRUPT) {
    for (int i : t->missing) lens[i] = S;
    if (join) join->done = true;
  }
  return rc;
}

}  // namespace

// ---- exported -------------------------------------------------------------------------

extern "C" {

int rs_abi_version(void) { return RS_ABI_VERSION; }

const char* rs_strerror(int code) {
  switch (code) {
    case RS_OK: return "ok";
    case RS_E_INVALID_PROFILE: return "erasure: invalid erasure profile parameters (code 3054)";
    case RS_E_SHORT_DATA: return "not enough data to fill the number of requested shards";
    case RS_E_TOO_FEW_SHARDS: return "too few shards given";
    case RS_E_SHARD_SIZE: return "shard sizes do not match";
    case RS_E_NO_DATA: return "no shard data";
    case RS_E_CORRUPT: return "erasure: shard checksum mismatch (code 3051)";
    case RS_E_INSUFFICIENT: return "erasure: insufficient shards for reconstruction (code 3050)";
    case RS_E_UNSUPPORTED: return "profile needs the GF(2^16) (Leopard) codec: k+m > 256";
    case RS_E_HIP: return "HIP runtime error or no usable device";
    case RS_E_ARG: return "invalid argument";
    case RS_E_SINGULAR: return "matrix is singular";
    case RS_E_NOMEM: return "out of memory";
    default: return "unknown error";
  }
}

int rs_init(rs_ctx** out, unsigned device_mask) {
  if (!out) return RS_E_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return RS_E_HIP;
  auto ctx = std::make_unique<rs_ctx>();
  for (int d : select_devices(count, device_mask)) {
    auto dev = std::make_unique<Device>();
    dev->id = d;
    ctx->devs.push_back(std::move(dev));
  }
  if (ctx->devs.empty()) return RS_E_HIP;
  // (the wide kernels' > 64 KiB dynamic-LDS opt-in is a per-device attribute: launch_apply
  // issues it once per (device, R) before the first such launch on a device, so rs_init
  // touches no device -- a process per GPU must not load code onto all eight)
  *out = ctx.release();
  return RS_OK;
}

void rs_shutdown(rs_ctx* ctx) {
  DeviceGuard dg;
  delete ctx;
}

int rs_device_count(const rs_ctx* ctx) { return ctx ? static_cast<int>(ctx->devs.size()) : 0; }

int rs_host_alloc(rs_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out || bytes == 0) return RS_E_ARG;
  *out = nullptr;
  HostPool::Buf b = ctx->host_pool.take(bytes);
  if (!b.p) {
    b.cap = HostPool::granule(bytes);
    // portable: every device of the context may use it. Coherent: the kernels read and
    // write it in place (zero-copy), and the caller refills the same buffer between
    // calls, so device caches must not keep its lines across launches.
    if (hipHostMalloc(&b.p, b.cap, hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess)
      return RS_E_NOMEM;
  }
  ctx->pinned.add(b.p, b.cap);
  *out = b.p;
  return RS_OK;
}

int rs_host_free(rs_ctx* ctx, void* p) {
  if (!ctx || !p) return RS_E_ARG;
  const size_t cap = ctx->pinned.size_of(p);
  if (!cap || !ctx->pinned.remove(p)) return RS_E_ARG;
  int rc = RS_OK;
  for (void* q : ctx->host_pool.put(p, cap))
    if (hipHostFree(q) != hipSuccess) rc = RS_E_HIP;
  return rc;
}

int rs_shard_size(int k, int m, int64_t len, int64_t* shard_size) {
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!shard_size || len < 0) return RS_E_ARG;
  if (len == 0) return RS_E_SHORT_DATA;
  *shard_size = (len + k - 1) / k;
  return RS_OK;
}

int rs_encode_matrix(int k, int m, uint8_t* out) {
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!out) return RS_E_ARG;
  Mat E;
  if (!encode_matrix(k, m, E)) return RS_E_SINGULAR;
  std::memcpy(out, E.v.data(), E.v.size());
  return RS_OK;
}

int rs_decode_rows(int k, int m, const uint8_t* present, int* valid_out, int* missing_out,
                   int* n_missing, uint8_t* rows_out) {
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!present || !valid_out || !missing_out || !n_missing || !rows_out) return RS_E_ARG;
  int np = 0;
  for (int i = 0; i < k + m; ++i) np += present[i] != 0;
  if (np < k) return RS_E_TOO_FEW_SHARDS;
  DecodePlan dp;
  if (!decode_plan(k, m, present, dp)) return RS_E_SINGULAR;
  std::copy(dp.valid.begin(), dp.valid.end(), valid_out);
  std::copy(dp.missing.begin(), dp.missing.end(), missing_out);
  *n_missing = static_cast<int>(dp.missing.size());
  std::memcpy(rows_out, dp.rows.v.data(), dp.missing.size() * static_cast<size_t>(k));
  return RS_OK;
}

int rs_encode(rs_ctx* ctx, int k, int m, size_t S, const uint8_t* const* data,
              uint8_t* const* parity) {
  DeviceGuard dg;
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!ctx || !data || !parity) return RS_E_ARG;
  if (S == 0) return RS_E_NO_DATA;  // upstream Encode: checkShards -> ErrShardNoData
  uint8_t present[256];
  for (int i = 0; i < k + m; ++i) present[i] = i < k;
  auto t = ctx->cache.get(k, m, present, false);
  if (!t) return RS_E_SINGULAR;
  return run_host1(ctx, t, S, [&](int i) { return data[i]; },
                  [&](int i) { return parity[i - k]; });
}

int rs_codec_encode(rs_ctx* ctx, int k, int m, const uint8_t* data, size_t len,
                    uint8_t* shards_out, size_t out_cap, size_t* shard_size) {
  DeviceGuard dg;
  // codec.go:22-24 profile check, :26 New, :31 Split, :36 Encode. Upstream New accepts
  // k+m > 256 (Leopard), so an empty object fails in Split before the profile is
  // found unsupported here.
  if (k < 1 || m < 1) return RS_E_INVALID_PROFILE;
  if (!ctx || !shard_size || (len && (!data || !shards_out))) return RS_E_ARG;
  if (len == 0) return RS_E_SHORT_DATA;
  int rc = check_profile(k, m);
  if (rc) return rc;
  const size_t S = (len + k - 1) / k;
  const int n = k + m;
  if (out_cap < S * n) return RS_E_ARG;
  uint8_t present[256];
  for (int i = 0; i < n; ++i) present[i] = i < k;
  auto t = ctx->cache.get(k, m, present, false);
  if (!t) return RS_E_SINGULAR;
  *shard_size = S;
  const bool overlap = shards_out != data && shards_out < data + len && data < shards_out + S * n;
  if (shards_out == data || overlap) {
    if (overlap) std::memmove(shards_out, data, len);
    std::memset(shards_out + len, 0, S * k - len);  // Split zero padding
    return run_host1(ctx, t, S, [&](int i) { return shards_out + S * i; },
                    [&](int i) { return shards_out + S * i; });
  }
  // Disjoint buffers: the partial last shard and its zero padding go to shards_out first;
  // the full data shards are staged straight from `data`, and the staging copies tee
  // them into shards_out (no separate object-sized copy).
  const size_t full = len / S;
  std::memcpy(shards_out + full * S, data + full * S, len - full * S);
  std::memset(shards_out + len, 0, S * k - len);  // Split zero padding
  Join tee{shards_out, full * S, S, k};
  return run_host1(ctx, t, S,
                   [&](int i) {
                     return static_cast<size_t>(i) < full ? data + S * i : shards_out + S * i;
                   },
                   [&](int i) { return shards_out + S * i; }, &tee);
}

int rs_reconstruct(rs_ctx* ctx, int k, int m, uint8_t* const* shards, size_t* lens) {
  DeviceGuard dg;
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!ctx || !shards || !lens) return RS_E_ARG;
  return reconstruct_host(ctx, k, m, shards, lens, false);
}

int rs_verify(rs_ctx* ctx, int k, int m, const uint8_t* const* shards, const size_t* lens,
              int* ok) {
  DeviceGuard dg;
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!ctx || !shards || !lens || !ok) return RS_E_ARG;
  const int n = k + m;
  size_t S = 0;
  int np = 0;
  if ((rc = check_lens(n, lens, false, &S, &np))) return rc;
  uint8_t present[256];
  for (int i = 0; i < n; ++i) present[i] = 1;
  auto t = ctx->cache.get(k, m, present, true);
  if (!t) return RS_E_SINGULAR;
  rc = run_host1(ctx, t, S, [&](int i) { return shards[i]; },
                 [&](int) { return static_cast<uint8_t*>(nullptr); });
  if (rc == RS_OK || rc == RS_E_CORRUPT) {
    *ok = rc == RS_OK;
    return RS_OK;
  }
  return rc;
}

int rs_codec_decode(rs_ctx* ctx, int k, int m, uint8_t* const* shards, size_t* lens,
                    uint8_t* out, int64_t original_size) {
  DeviceGuard dg;
  // codec.go:46-48 profile, :50 New, :55 Reconstruct, :59-65 Verify, :67-77 join/trim
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!ctx || !shards || !lens || original_size < 0 || (original_size && !out)) return RS_E_ARG;
  Join join{out, static_cast<size_t>(original_size), 0, k};
  rc = reconstruct_host(ctx, k, m, shards, lens, true, &join);
  if (rc) return rc;
  const size_t S = lens[0];
  if (static_cast<uint64_t>(S) * k < static_cast<uint64_t>(original_size))
    return RS_E_INSUFFICIENT;
  if (join.done) return RS_OK;  // joined on the way through the pipeline
  size_t left = static_cast<size_t>(original_size);
  std::vector<CopyPool::Seg> segs;
  for (int i = 0; i < k && left; ++i) {
    const size_t c = std::min(S, left);
    segs.push_back({out + S * i, shards[i], c});
    left -= c;
  }
  ctx->pool.run(segs);
  return RS_OK;
}

// ---- batched host-memory calls ---------------------------------------------------------

namespace {

// Stripes grouped by (S, presence): each group shares one table set and one pipeline.
struct BatchGroups {
  std::map<std::string, std::vector<int>> by_key;
  void add(size_t S, const uint8_t* present, int n, int b) {
    std::string key(reinterpret_cast<const char*>(&S), sizeof S);
    key.append(reinterpret_cast<const char*>(present), n);
    by_key[key].push_back(b);
  }
  static size_t shard_size(const std::string& key) {
    size_t S;
    std::memcpy(&S, key.data(), sizeof S);
    return S;
  }
};

int first_error(const int* status, int batch) {
  for (int b = 0; b < batch; ++b)
    if (status[b]) return status[b];
  return RS_OK;
}

}  // namespace

int rs_encode_batch(rs_ctx* ctx, int k, int m, int batch, const size_t* sizes,
                    const uint8_t* const* data, uint8_t* const* parity, int* status) {
  DeviceGuard dg;
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!ctx || batch < 0 || (batch && (!sizes || !data || !parity || !status))) return RS_E_ARG;
  const int n = k + m;
  uint8_t present[256];
  for (int i = 0; i < n; ++i) present[i] = i < k;
  BatchGroups groups;
  for (int b = 0; b < batch; ++b) {
    status[b] = sizes[b] ? RS_OK : RS_E_NO_DATA;  // upstream Encode: ErrShardNoData
    if (sizes[b]) groups.add(sizes[b], present, n, b);
  }
  auto t = ctx->cache.get(k, m, present, false);
  if (!t) return RS_E_SINGULAR;
  for (auto& kv : groups.by_key) {
    const std::vector<int>& ids = kv.second;
    const size_t S = BatchGroups::shard_size(kv.first);
    rc = run_host(ctx, t, S, static_cast<int>(ids.size()),
                  [&](int b, int i) { return data[static_cast<size_t>(ids[b]) * k + i]; },
                  [&](int b, int i) { return parity[static_cast<size_t>(ids[b]) * m + i - k]; });
    if (rc) return rc;
  }
  return first_error(status, batch);
}

int rs_reconstruct_batch(rs_ctx* ctx, int k, int m, int batch, uint8_t* const* shards,
                         size_t* lens, int verify, int* status) {
  DeviceGuard dg;
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!ctx || batch < 0 || (batch && (!shards || !lens || !status))) return RS_E_ARG;
  const int n = k + m;
  BatchGroups groups;
  uint8_t present[256];
  for (int b = 0; b < batch; ++b) {
    uint8_t* const* sh = shards + static_cast<size_t>(b) * n;
    const size_t* ln = lens + static_cast<size_t>(b) * n;
    size_t S = 0;
    int np = 0;
    status[b] = check_lens(n, ln, true, &S, &np);
    if (status[b]) continue;
    if (np < k) {
      status[b] = RS_E_TOO_FEW_SHARDS;
      continue;
    }
    if (np == n && !verify) continue;
    bool ok = true;
    for (int i = 0; i < n; ++i) {
      ok &= sh[i] != nullptr;
      present[i] = ln[i] != 0;
    }
    if (!ok) {
      status[b] = RS_E_ARG;
      continue;
    }
    groups.add(S, present, n, b);
  }
  std::vector<int> flags;
  for (auto& kv : groups.by_key) {
    const std::vector<int>& ids = kv.second;
    const size_t S = BatchGroups::shard_size(kv.first);
    const uint8_t* pres = reinterpret_cast<const uint8_t*>(kv.first.data() + sizeof(size_t));
    auto t = ctx->cache.get(k, m, pres, verify != 0);
    if (!t) return RS_E_SINGULAR;
    if (!t->groups.empty()) {
      flags.assign(ids.size(), 0);
      rc = run_host(ctx, t, S, static_cast<int>(ids.size()),
                    [&](int b, int i) { return shards[static_cast<size_t>(ids[b]) * n + i]; },
                    [&](int b, int i) { return shards[static_cast<size_t>(ids[b]) * n + i]; },
                    flags.data());
      if (rc != RS_OK && rc != RS_E_CORRUPT) return rc;
      for (size_t j = 0; j < ids.size(); ++j)
        if (flags[j]) status[ids[j]] = RS_E_CORRUPT;
    }
    for (int b : ids)
      for (int i : t->missing) lens[static_cast<size_t>(b) * n + i] = S;
  }
  return first_error(status, batch);
}

// ---- device-resident ----------------------------------------------------------------

struct rs_plan {
  int device = 0;
  size_t S = 0;
  int batch = 0;
  std::shared_ptr<const Tables> tables;
  MetaLayout layout;
  void* dmeta = nullptr;
  uint64_t bytes = 0;
  LayoutHint hint;
  std::vector<int> orders;  // per launch group: tile order from rs_plan_tune, -1 = rule
  std::mutex mu;            // orders are written by rs_plan_tune, read by rs_plan_launch
};

int rs_plan_create(rs_ctx* ctx, int device, int k, int m, size_t S, int batch,
                   const uint8_t* present, uint8_t* const* shards, rs_plan** out) {
  DeviceGuard dg;
  int rc = check_profile(k, m);
  if (rc) return rc;
  if (!ctx || !shards || !out || batch < 1) return RS_E_ARG;
  *out = nullptr;
  Device* dev = ctx->device(device);
  if (!dev) return RS_E_ARG;
  const int n = k + m;
  uint8_t pres[256];
  int np = 0;
  for (int i = 0; i < n; ++i) {
    pres[i] = present ? (present[i] != 0) : (i < k);
    np += pres[i];
  }
  if (np < k) return RS_E_TOO_FEW_SHARDS;
  auto t = ctx->cache.get(k, m, pres, true);
  if (!t) return RS_E_SINGULAR;
  auto plan = std::make_unique<rs_plan>();
  plan->device = device;
  plan->S = S;
  plan->batch = batch;
  plan->tables = t;
  plan->layout = meta_layout(*t, batch);
  plan->bytes = algo_bytes(*t, S, batch);
  std::vector<uint8_t> h(plan->layout.total);
  plan->hint = fill_meta(*t, plan->layout, batch, h.data(), [&](int b, int i) {
    return static_cast<const uint8_t*>(shards[static_cast<size_t>(b) * n + i]);
  });
  HIPCHK(hipSetDevice(device));
  if (hipMalloc(&plan->dmeta, plan->layout.total) != hipSuccess) return RS_E_NOMEM;
  if (hipMemcpy(plan->dmeta, h.data(), h.size(), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(plan->dmeta);
    return RS_E_HIP;
  }
  // plans are launched many times: the launch groups the rule gives the bit-sliced kernel have
  // it compiled (or loaded from the code cache) here, so every launch runs it; a compile that
  // fails leaves them on the nibble-table kernels. A plan waits for at most kSyncCompileKR
  // coefficients' worth of compiles (about 4 s on the GPU box); its other blocks compile in
  // the background (RS(200,16) alone: 8 s there, RS(240,16) 48 s on a build host; the 8 groups
  // of an RS(128,128) decode: 30 s) and run the nibble-table kernels until they are ready.
  constexpr int kSyncCompileKR = 2048;
  int sync_kr = 0;
  for (size_t gi = 0; gi < t->groups.size(); ++gi) {
    const Group& g = t->groups[gi];
    if (!g.bsk || !bitslice_wanted(group_args(*t, plan->layout, gi, batch,
                                              static_cast<uint8_t*>(plan->dmeta), S, 1, plan->hint)))
      continue;
    const int kr = k * static_cast<int>(g.shard.size());
    const bool wait = sync_kr + kr <= kSyncCompileKR;
    if (wait) sync_kr += kr;
    (void)g.bsk->function(device, wait);
  }
  *out = plan.release();
  return RS_OK;
}

// A timed launch that dispatches no kernel still records both events on the stream, so
// the caller's elapsed time is this launch's (zero), never a stale earlier interval.
static int record_empty(void* stream, void* start_event, void* stop_event) {
  const auto s = static_cast<hipStream_t>(stream);
  if (start_event) HIPCHK(hipEventRecord(static_cast<hipEvent_t>(start_event), s));
  if (stop_event) HIPCHK(hipEventRecord(static_cast<hipEvent_t>(stop_event), s));
  return RS_OK;
}

int rs_plan_launch(rs_plan* plan, void* stream) {
  return rs_plan_launch_timed(plan, stream, nullptr, nullptr);
}

int rs_plan_launch_timed(rs_plan* plan, void* stream, void* start_event, void* stop_event) {
  DeviceGuard dg;
  if (!plan) return RS_E_ARG;
  HIPCHK(hipSetDevice(plan->device));
  std::vector<int> orders;
  {
    std::lock_guard<std::mutex> g(plan->mu);
    orders = plan->orders;
  }
  if (plan->S == 0)  // nothing dispatches: the events still bracket this (empty) launch
    return record_empty(stream, start_event, stop_event);
  LaunchEvents ev;
  ev.start = static_cast<hipEvent_t>(start_event);
  ev.stop = static_cast<hipEvent_t>(stop_event);
  HIPCHK(launch_groups(*plan->tables, plan->layout, plan->batch,
                       static_cast<uint8_t*>(plan->dmeta), plan->S,
                       static_cast<hipStream_t>(stream), /*status_stride=*/1, plan->hint,
                       &orders, ev));
  return RS_OK;
}

int rs_plan_launch_ceiling(rs_plan* plan, void* stream, int mode) {
  return rs_plan_launch_ceiling_timed(plan, stream, mode, nullptr, nullptr);
}

int rs_plan_launch_ceiling_timed(rs_plan* plan, void* stream, int mode, void* start_event,
                                 void* stop_event) {
  DeviceGuard dg;
  if (!plan || mode < 0 || mode > 8) return RS_E_ARG;
  // the product implements RS_CEIL_READ / RS_CEIL_WRITE; the other modes are the A/B build's
  // (tools/callfs_rs_ab.h)
  if (!kAbInstances && mode != RS_CEIL_READ && mode != RS_CEIL_WRITE) return RS_E_ARG;
  HIPCHK(hipSetDevice(plan->device));
  std::vector<int> orders;
  {
    std::lock_guard<std::mutex> g(plan->mu);
    orders = plan->orders;
  }
  if (plan->S < 16)  // the ceilings cover whole 16-B vectors only: nothing dispatches
    return record_empty(stream, start_event, stop_event);
  const Tables& t = *plan->tables;
  auto* d = static_cast<uint8_t*>(plan->dmeta);
  const size_t ng = t.groups.size();
  for (size_t gi = 0; gi < ng; ++gi) {
    const int order = gi < orders.size() ? orders[gi] : -1;
    LaunchEvents ev;
    ev.start = gi == 0 ? static_cast<hipEvent_t>(start_event) : nullptr;
    ev.stop = gi + 1 == ng ? static_cast<hipEvent_t>(stop_event) : nullptr;
    HIPCHK(launch_ceiling(group_args(t, plan->layout, gi, plan->batch, d, plan->S, 1, plan->hint),
                          static_cast<hipStream_t>(stream), order, mode, ev));
  }
  return RS_OK;
}

// Times every tile order each launch group's kernel offers and keeps the fastest. Which
// order HBM serves best varies between MI355X boxes by 1-2 points on the same shape
// (DESIGN.md §6.2 "Tile order"), so a plan that is launched many times measures it on the
// box it runs on, like a library autotuner, instead of trusting the rule alone. Each
// candidate gets `reps` back-to-back launches between two events, in three rounds with the
// candidate order rotated; the per-launch mean of the best round counts, and the rule's
// order is kept unless another is faster by more than 1 % (with 0.3 % the tuner sometimes
// left the rule for an order that then timed 0.5-1 % slower, round 3).
namespace {
constexpr int kTuneRounds = 3;
constexpr float kTuneWarmMs = 150.0f;
constexpr int kTuneWarmBatches = 400;
// CALLFS_RS_TUNE_BAR=<percent>: how much faster than the rule's order another order must
// time to replace it (default 1)
float tune_bar() {
  static const float v = [] {
    const char* e = std::getenv("CALLFS_RS_TUNE_BAR");
    if (e && *e) {
      const float x = std::strtof(e, nullptr);
      if (x >= 0.0f && x < 50.0f) return x;
    }
    return 1.0f;
  }();
  return v;
}

// CALLFS_RS_TUNE_LOG=1: rs_plan_tune prints each candidate's time per launch to stderr
bool tune_log() {
  static const bool on = [] {
    const char* e = std::getenv("CALLFS_RS_TUNE_LOG");
    return e && *e && *e != '0';
  }();
  return on;
}
}  // namespace

int rs_plan_tune(rs_plan* plan, void* stream, int reps, int* orders, int max_groups) {
  DeviceGuard dg;
  if (!plan || reps < 1 || max_groups < 0 || (max_groups > 0 && !orders)) return RS_E_ARG;
  HIPCHK(hipSetDevice(plan->device));
  auto s = static_cast<hipStream_t>(stream);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIPCHK(hipStreamIsCapturing(s, &cap));
  if (cap != hipStreamCaptureStatusNone) return RS_E_ARG;  // synchronous: not in a capture
  const Tables& t = *plan->tables;
  auto* d = static_cast<uint8_t*>(plan->dmeta);
  std::vector<int> chosen(t.groups.size(), -1);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIPCHK(hipEventCreate(&e0));
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return RS_E_HIP;
  }
  int rc = RS_OK;
  for (size_t gi = 0; gi < t.groups.size() && rc == RS_OK; ++gi) {
    const ApplyArgs a = group_args(t, plan->layout, gi, plan->batch, d, plan->S, 1, plan->hint);
    std::vector<int> cand = order_candidates(a);
    // the bit-sliced orders only when the group's kernel compiles and loads here: a hiprtc
    // that fails on some box leaves the tuner (and the bench) on the nibble-table forms
    const Group& grp = t.groups[gi];
    const auto bs_order = [](int o) { return o >= kOrderBitslice; };
    if (std::any_of(cand.begin(), cand.end(), bs_order) &&
        (!grp.bsk || !grp.bsk->function(plan->device, /*wait=*/true)))
      cand.erase(std::remove_if(cand.begin(), cand.end(), bs_order), cand.end());
    if (cand.size() < 2) continue;
    std::vector<float> best(cand.size(), 1e30f);
    // warm-up in the rule's order first, by time: a chip that has just come out of other
    // (or no) work runs the bench shape up to 4 % slow for ~100 ms (bench.py at 5 vs 100
    // warm-up steps, profiles/r02/warmup/), and candidates timed during that ramp favour
    // whichever is timed last. Batches of `reps` launches until kTuneWarmMs of device
    // time have passed (at most kTuneWarmBatches batches).
    {
      float warm = 0;
      for (int b = 0; b < kTuneWarmBatches && warm < kTuneWarmMs && rc == RS_OK; ++b) {
        bool ok = hipEventRecord(e0, s) == hipSuccess;
        for (int r = 0; r < reps && ok; ++r) ok = launch_apply(a, s, false, cand[0]) == hipSuccess;
        float ms = 0;
        ok = ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
             hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
        if (!ok) rc = RS_E_HIP;
        warm += ms;
      }
    }
    for (int round = 0; round < kTuneRounds && rc == RS_OK; ++round) {
      for (size_t j = 0; j < cand.size() && rc == RS_OK; ++j) {
        const size_t c = (j + round) % cand.size();
        // one untimed launch, then `reps` timed ones
        bool ok = launch_apply(a, s, false, cand[c]) == hipSuccess && hipEventRecord(e0, s) == hipSuccess;
        for (int r = 0; r < reps && ok; ++r) ok = launch_apply(a, s, false, cand[c]) == hipSuccess;
        ok = ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess;
        float ms = 0;
        ok = ok && hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
        if (!ok) {
          rc = RS_E_HIP;
          break;
        }
        best[c] = std::min(best[c], ms / static_cast<float>(reps));
      }
    }
    if (rc != RS_OK) break;
    size_t win = 0;  // cand[0] is the rule's order
    for (size_t c = 1; c < cand.size(); ++c)
      if (best[c] < best[win] * (win == 0 ? 1.0f - tune_bar() / 100.0f : 1.0f)) win = c;
    chosen[gi] = cand[win];
    record_tuned(a, chosen[gi]);  // later untuned launches of this shape take it
    if (tune_log()) {
      std::fprintf(stderr, "rs_plan_tune: group %zu (K=%d R=%d S=%zu batch=%d):", gi, a.K, a.R,
                   static_cast<size_t>(a.S), a.batch);
      for (size_t c = 0; c < cand.size(); ++c)
        std::fprintf(stderr, " order %d %.1f us%s", cand[c], best[c] * 1e3f, c == win ? " *" : "");
      std::fprintf(stderr, "\n");
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc != RS_OK) return rc;
  {
    std::lock_guard<std::mutex> g(plan->mu);
    plan->orders = chosen;
  }
  for (int i = 0; i < max_groups; ++i)
    orders[i] = static_cast<size_t>(i) < chosen.size() ? chosen[i] : -1;
  return RS_OK;
}

// Pins launch group i to orders[i] (-1: the rule), as rs_plan_tune would: the order must
// be one order_candidates offers for that group's kernel (RS_E_ARG otherwise, and nothing
// changes). For orders tuned once and kept (a deployment's own shard layout), and for
// tests that run every instance.
int rs_plan_set_orders(rs_plan* plan, const int* orders, int n) {
  if (!plan || n < 0 || (n > 0 && !orders)) return RS_E_ARG;
  const Tables& t = *plan->tables;
  if (static_cast<size_t>(n) > t.groups.size()) return RS_E_ARG;
  auto* d = static_cast<uint8_t*>(plan->dmeta);
  std::vector<int> next(t.groups.size(), -1);
  for (int gi = 0; gi < n; ++gi) {
    if (orders[gi] == -1) continue;
    const ApplyArgs a = group_args(t, plan->layout, gi, plan->batch, d, plan->S, 1, plan->hint);
    const std::vector<int> cand = order_candidates(a, /*every_instance=*/true);
    if (std::find(cand.begin(), cand.end(), orders[gi]) == cand.end()) return RS_E_ARG;
    next[gi] = orders[gi];
  }
  std::lock_guard<std::mutex> g(plan->mu);
  plan->orders = next;
  return RS_OK;
}

int rs_tune_table_reset(const char* path) {
  tune_table().reset(path);
  return RS_OK;
}

int rs_tune_table_entries(void) { return static_cast<int>(tune_table().size()); }

int rs_plan_forms(const rs_plan* plan, int* forms, int max_groups) {
  if (!plan || max_groups < 0 || (max_groups > 0 && !forms)) return RS_E_ARG;
  auto* p = const_cast<rs_plan*>(plan);
  std::vector<int> orders;
  {
    std::lock_guard<std::mutex> g(p->mu);
    orders = p->orders;
  }
  const Tables& t = *plan->tables;
  auto* d = static_cast<uint8_t*>(plan->dmeta);
  const int ng = static_cast<int>(t.groups.size());
  for (int gi = 0; gi < ng && gi < max_groups; ++gi) {
    const int order = static_cast<size_t>(gi) < orders.size() ? orders[gi] : -1;
    forms[gi] = launch_form(group_args(t, plan->layout, gi, plan->batch, d, plan->S, 1, plan->hint), order);
  }
  return ng;
}

int rs_plan_stripe_status(rs_plan* plan, void* stream, int* flags) {
  DeviceGuard dg;
  if (!plan || !flags) return RS_E_ARG;
  HIPCHK(hipSetDevice(plan->device));
  auto s = static_cast<hipStream_t>(stream);
  auto* st = static_cast<uint8_t*>(plan->dmeta) + plan->layout.status_off;
  const size_t bytes = sizeof(int) * static_cast<size_t>(plan->batch);
  HIPCHK(hipMemcpyAsync(flags, st, bytes, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemsetAsync(st, 0, bytes, s));
  HIPCHK(hipStreamSynchronize(s));
  return RS_OK;
}

int rs_plan_status(rs_plan* plan, void* stream, int* corrupt) {
  if (!plan || !corrupt) return RS_E_ARG;
  std::vector<int> flags(static_cast<size_t>(plan->batch));
  const int rc = rs_plan_stripe_status(plan, stream, flags.data());
  if (rc) return rc;
  *corrupt = std::any_of(flags.begin(), flags.end(), [](int f) { return f != 0; });
  return RS_OK;
}

uint64_t rs_plan_bytes(const rs_plan* plan) { return plan ? plan->bytes : 0; }

int rs_plan_groups(const rs_plan* plan) {
  return plan ? static_cast<int>(plan->tables->groups.size()) : 0;
}

void rs_plan_destroy(rs_plan* plan) {
  DeviceGuard dg;
  if (!plan) return;
  (void)hipSetDevice(plan->device);
  if (plan->dmeta) (void)hipFree(plan->dmeta);
  delete plan;
}

static int one_shot(rs_ctx* ctx, int device, int k, int m, size_t S, int batch,
                    const uint8_t* present, uint8_t* const* shards, void* stream) {
  rs_plan* p = nullptr;
  int rc = rs_plan_create(ctx, device, k, m, S, batch, present, shards, &p);
  if (rc) return rc;
  rc = rs_plan_launch(p, stream);
  int corrupt = 0;
  if (!rc) rc = rs_plan_status(p, stream, &corrupt);
  rs_plan_destroy(p);
  if (!rc && corrupt) rc = RS_E_CORRUPT;
  return rc;
}

int rs_encode_dev(rs_ctx* ctx, int device, int k, int m, size_t S, int batch,
                  uint8_t* const* shards, void* stream) {
  return one_shot(ctx, device, k, m, S, batch, nullptr, shards, stream);
}

int rs_decode_dev(rs_ctx* ctx, int device, int k, int m, size_t S, int batch,
                  const uint8_t* present, uint8_t* const* shards, void* stream) {
  if (!present) return RS_E_ARG;
  return one_shot(ctx, device, k, m, S, batch, present, shards, stream);
}

// ---- batched SHA-256 (ShardChecksum) ------------------------------------------------

struct rs_hash_plan {
  int device = 0;
  int count = 0;
  int mpw = 1;
  void* dtab = nullptr;  // [count] pointers then [count] lengths
};

int rs_sha256_plan_create(rs_ctx* ctx, int device, const uint8_t* const* msgs,
                          const uint64_t* lens, int count, rs_hash_plan** out) {
  DeviceGuard dg;
  if (!ctx || !out || count < 0 || (count && (!msgs || !lens))) return RS_E_ARG;
  *out = nullptr;
  if (!ctx->device(device)) return RS_E_ARG;
  auto plan = std::make_unique<rs_hash_plan>();
  plan->device = device;
  plan->count = count;
  plan->mpw = default_msgs_per_wave(count);
  if (const char* e = kAbInstances ? std::getenv("CALLFS_SHA_MSGS_PER_WAVE") : nullptr)
    plan->mpw = std::atoi(e);
  HIPCHK(hipSetDevice(device));
  const size_t bytes = static_cast<size_t>(count) * (sizeof(void*) + sizeof(uint64_t));
  if (count) {
    std::vector<uint8_t> h(bytes);
    std::memcpy(h.data(), msgs, count * sizeof(void*));
    std::memcpy(h.data() + count * sizeof(void*), lens, count * sizeof(uint64_t));
    if (hipMalloc(&plan->dtab, bytes) != hipSuccess) return RS_E_NOMEM;
    if (hipMemcpy(plan->dtab, h.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(plan->dtab);
      return RS_E_HIP;
    }
  }
  *out = plan.release();
  return RS_OK;
}

int rs_sha256_plan_launch(rs_hash_plan* plan, uint8_t* digests, void* stream) {
  DeviceGuard dg;
  if (!plan || (plan->count && !digests)) return RS_E_ARG;
  if ((reinterpret_cast<uintptr_t>(digests) & 3u) != 0) return RS_E_ARG;
  HIPCHK(hipSetDevice(plan->device));
  Sha256Args a{};
  a.msgs = static_cast<const uint8_t* const*>(plan->dtab);
  a.lens = reinterpret_cast<const uint64_t*>(static_cast<uint8_t*>(plan->dtab) +
                                             plan->count * sizeof(void*));
  a.digests = reinterpret_cast<uint32_t*>(digests);
  a.count = plan->count;
  HIPCHK(launch_sha256(a, plan->mpw, static_cast<hipStream_t>(stream)));
  return RS_OK;
}

void rs_sha256_plan_destroy(rs_hash_plan* plan) {
  DeviceGuard dg;
  if (!plan) return;
  (void)hipSetDevice(plan->device);
  if (plan->dtab) (void)hipFree(plan->dtab);
  delete plan;
}

int rs_sha256_dev(rs_ctx* ctx, int device, const uint8_t* const* msgs, const uint64_t* lens,
                  int count, uint8_t* digests, void* stream) {
  rs_hash_plan* p = nullptr;
  int rc = rs_sha256_plan_create(ctx, device, msgs, lens, count, &p);
  if (rc) return rc;
  rc = rs_sha256_plan_launch(p, digests, stream);
  if (!rc && hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess) rc = RS_E_HIP;
  rs_sha256_plan_destroy(p);
  return rc;
}

}  // extern "C"
