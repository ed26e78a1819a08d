// Measured kernel forms per launch shape: what rs_plan_tune chose, kept per
// device and consulted by every launch that has no order of its own (untuned plans and the
// host-memory calls) before the fitted rule of tile_order.hpp. The rule stays the fallback
// for shapes nobody has tuned on the device. Plain C++ (no HIP): tests/native/host_test.cpp
// checks lookup, fallback, persistence and concurrent use under ASan / TSan.
//
// Key: (device, K inputs, R rows, tiles-per-stripe bucket, address-alignment class, written /
// mixed / read-only rows, input and output misalignment). Shapes in one key share the traffic
// pattern the tile orders respond to: tiles per stripe in powers of two (the rule's bands are
// powers of two as well), and the shard addresses' alignment in the classes the rule keys on
// (pitches that are multiples of 128 KiB, of 256 B, or less).
//
// Persistence: CALLFS_RS_TUNE_TABLE names a text file, one entry per line
// ("device K R tps_log2 align kind mis order"), read on first use and rewritten whole (temp
// file + rename) after each change, merged with what other processes wrote to it meanwhile, so
// a deployment tunes once per box and every later process starts from the measured forms.
// Unset: the table lives for the process.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <unistd.h>

namespace callfs {

struct TuneKey {
  int device = 0;
  int K = 0, R = 0;
  int tps_log2 = 0;  // floor(log2(tiles per stripe)), tiles of 8 KiB
  int align = 0;     // 0: shard addresses differ by multiples of 128 KiB; 1: of 256 B; 2: less
  int kind = 0;      // 0: every row written; 1: written and compared rows; 2: only compared
  int mis = 0;       // bit 0: an input shard is not 16-B aligned; bit 1: an output row
  uint64_t packed() const {
    return (static_cast<uint64_t>(device & 0xff) << 40) | (static_cast<uint64_t>(K & 0x1ff) << 31) |
           (static_cast<uint64_t>(R & 0x1f) << 26) | (static_cast<uint64_t>(tps_log2 & 0x3f) << 20) |
           (static_cast<uint64_t>(align & 3) << 18) | (static_cast<uint64_t>(kind & 3) << 16) |
           static_cast<uint64_t>(mis & 3);
  }
};

// The key of a launch: `tps` = 8 KiB tiles per stripe, `addr_tz` as ApplyArgs::addr_tz.
inline TuneKey tune_key(int device, int K, int R, uint64_t tps, int addr_tz, bool verify,
                        bool read_only, bool in_mis, bool out_mis) {
  TuneKey k;
  k.device = device;
  k.K = K;
  k.R = R;
  int l = 0;
  while (l < 63 && (tps >> (l + 1)) != 0) ++l;
  k.tps_log2 = l;
  k.align = addr_tz >= 17 ? 0 : (addr_tz >= 8 ? 1 : 2);
  k.kind = read_only ? 2 : (verify ? 1 : 0);
  k.mis = (in_mis ? 1 : 0) | (out_mis ? 2 : 0);
  return k;
}

class TuneTable {
 public:
  // The measured order for `k`, or -1 (then the rule decides).
  int lookup(const TuneKey& k) {
    std::lock_guard<std::mutex> g(mu_);
    load_locked();
    auto it = map_.find(k.packed());
    return it == map_.end() ? -1 : it->second.order;
  }
  bool empty() {
    std::lock_guard<std::mutex> g(mu_);
    load_locked();
    return map_.empty();
  }
  // Records rs_plan_tune's choice (order >= 0) for `k`, replacing an earlier one, and
  // rewrites the file when one is configured.
  void record(const TuneKey& k, int order) {
    if (order < 0) return;
    std::lock_guard<std::mutex> g(mu_);
    load_locked();
    auto& e = map_[k.packed()];
    if (e.order == order && e.key.K == k.K) return;
    e.key = k;
    e.order = order;
    e.ours = true;
    save_locked();
  }
  // Forgets every entry (and the file's path: tests point tables at their own files).
  void reset(const char* path) {
    std::lock_guard<std::mutex> g(mu_);
    map_.clear();
    path_ = path ? path : "";
    loaded_ = false;
  }
  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    load_locked();
    return map_.size();
  }

 private:
  struct Entry {
    TuneKey key;
    int order = -1;
    bool ours = false;  // recorded by this process (else read from the file)
  };
  void load_locked() {
    if (loaded_) return;
    loaded_ = true;
    if (path_.empty()) {
      const char* e = std::getenv("CALLFS_RS_TUNE_TABLE");
      if (e) path_ = e;
    }
    read_file(false);
  }
  // Adds the file's entries; `keep_ours`: an entry this process recorded wins over the file's
  // (an entry it only read is replaced by the file's, which may be newer).
  void read_file(bool keep_ours) {
    if (path_.empty()) return;
    FILE* f = std::fopen(path_.c_str(), "r");
    if (!f) return;
    TuneKey k;
    int order = -1;
    while (std::fscanf(f, "%d %d %d %d %d %d %d %d", &k.device, &k.K, &k.R, &k.tps_log2, &k.align,
                       &k.kind, &k.mis, &order) == 8) {
      if (k.K < 1 || k.K > 256 || k.R < 1 || k.R > 16 || order < 0) continue;
      auto it = map_.find(k.packed());
      if (keep_ours && it != map_.end() && it->second.ours) continue;
      map_[k.packed()] = Entry{k, order};
    }
    std::fclose(f);
  }
  void save_locked() {
    if (path_.empty()) return;
    // what other processes recorded since this one read the file is kept, not overwritten
    read_file(true);
    // one temp file per process: processes sharing a table file never write the same temp
    const std::string tmp = path_ + "." + std::to_string(static_cast<long>(getpid())) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "w");
    if (!f) return;
    bool ok = true;
    for (const auto& kv : map_) {
      const TuneKey& k = kv.second.key;
      ok &= std::fprintf(f, "%d %d %d %d %d %d %d %d\n", k.device, k.K, k.R, k.tps_log2, k.align,
                         k.kind, k.mis, kv.second.order) > 0;
    }
    ok &= std::fclose(f) == 0;
    if (!ok || std::rename(tmp.c_str(), path_.c_str()) != 0) (void)std::remove(tmp.c_str());
  }

  std::mutex mu_;
  std::map<uint64_t, Entry> map_;
  std::string path_;
  bool loaded_ = false;
};

// The process's table (never destroyed: launches may run during static teardown).
inline TuneTable& tune_table() {
  static TuneTable* t = new TuneTable;
  return *t;
}

}  // namespace callfs
