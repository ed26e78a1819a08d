// Host-memory call placement over the devices of an rs_ctx: which devices a mask
// selects, on which device a call runs, and how one large object's columns are split
// over devices. Plain C++ with no HIP dependence, so tests/native/host_test.cpp checks
// it against mocked device lists on the CPU; rs_capi.cpp is the only product user.
//
// Every output byte depends only on the same column of the inputs (codec.go:36 ->
// upstream Encode), so column ranges of one object are independent: the in-process form
// of bench.py's column_slices.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace callfs {

constexpr int kMaxDevices = 32;

// rs_init's device selection: bit d of mask selects HIP device d; 0 selects all of the
// `count` visible devices. Devices beyond 32 are never selected.
inline std::vector<int> select_devices(int count, unsigned mask) {
  std::vector<int> out;
  for (int d = 0; d < count && d < kMaxDevices; ++d)
    if (!mask || ((mask >> d) & 1u)) out.push_back(d);
  return out;
}

// Index into the selected-device list for part p of the call that drew ticket `base`
// from the context's round-robin counter: consecutive calls land on consecutive
// devices, and the parts of one split call on consecutive devices from there.
inline size_t device_slot(unsigned base, int part, size_t ndev) {
  return ndev ? (static_cast<size_t>(base) + static_cast<size_t>(part)) % ndev : 0;
}

// Ways to split one object's columns: only single-stripe calls of at least `min_bytes`
// over all n shards; `ways_req` (<= 0: one per device) capped by the lanes available
// (ndev * lanes_per_device) and by 4 MiB of columns per way.
inline int split_ways(size_t ndev, int lanes_per_device, size_t S, int n, int batch,
                      unsigned long long min_bytes, int ways_req) {
  if (batch != 1 || ndev == 0) return 1;
  if (static_cast<unsigned long long>(S) * static_cast<unsigned>(n) < min_bytes) return 1;
  long ways = ways_req > 0 ? ways_req : static_cast<long>(ndev);
  ways = std::max(1L, std::min(ways, static_cast<long>(ndev) * lanes_per_device));
  return static_cast<int>(std::max<size_t>(1, std::min<size_t>(static_cast<size_t>(ways), S >> 22)));
}

// ways_req for split_ways from CALLFS_RS_SPLIT_WAYS: unset (nullptr) = one way per
// device; an explicit value <= 1 (0, negative, not a number) keeps every object on one
// device, which is what 0 meant before the per-device default existed.
inline int split_ways_request(const char* env) {
  if (!env) return 0;
  const long v = std::strtol(env, nullptr, 10);
  return v > 1 ? static_cast<int>(std::min(v, 1L << 20)) : 1;
}

// One-time setup per (device, key), e.g. the > 64 KiB dynamic-LDS opt-in of the wide
// kernels (launch_apply, key R - 9): hipFuncSetAttribute applies to the calling thread's
// current device only, so a once-flag per kernel would leave every device but the first
// without it. `run`
// calls f() the first time a (device, key) pair is seen and returns whether it did;
// concurrent callers of one pair wait until f() has returned. Devices outside
// [0, kMaxDevices) and keys outside [0, 64) run f() every time.
class DeviceOnce {
 public:
  template <class F>
  bool run(int device, int key, F&& f) {
    if (device < 0 || device >= kMaxDevices || key < 0 || key >= 64) {
      f();
      return true;
    }
    const uint64_t bit = 1ull << key;
    if (done_[device].load(std::memory_order_acquire) & bit) return false;
    std::lock_guard<std::mutex> g(mu_);
    if (done_[device].load(std::memory_order_relaxed) & bit) return false;
    f();
    done_[device].fetch_or(bit, std::memory_order_release);
    return true;
  }
  bool done(int device, int key) const {
    return device >= 0 && device < kMaxDevices && key >= 0 && key < 64 &&
           (done_[device].load(std::memory_order_acquire) >> key) & 1u;
  }

 private:
  std::atomic<uint64_t> done_[kMaxDevices] = {};
  std::mutex mu_;
};

// Column boundaries c[0..ways] of an S-byte shard: c[0] = 0, c[ways] = S, interior
// boundaries 4 KiB aligned (parts may be empty only when S is tiny).
inline std::vector<size_t> column_parts(size_t S, int ways) {
  std::vector<size_t> c(static_cast<size_t>(ways) + 1, 0);
  for (int p = 1; p < ways; ++p) {
    const size_t at = (S / static_cast<size_t>(ways) * static_cast<size_t>(p) + 4095) / 4096 * 4096;
    c[static_cast<size_t>(p)] = std::min(S, at);
  }
  c[static_cast<size_t>(ways)] = S;
  return c;
}

}  // namespace callfs
