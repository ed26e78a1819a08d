// Parallel memcpy pool for the host-memory path's pinned staging (rs_capi.cpp).
// Header-only so tests/native/host_test.cpp can run it under ASan/TSan on the CPU.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace callfs {

// Parallel memcpy for pageable <-> pinned staging. A job's segments are cut into
// pieces; the calling thread and the pool's workers take pieces until none are left.
// Threads: CALLFS_RS_COPY_THREADS, default min(8, hardware threads).
class CopyPool {
 public:
  // n bytes src -> dst; with dst2, the first n2 (<= n) of them also go to dst2 (a tee:
  // the second copy reads the piece while it is still in cache).
  struct Seg {
    void* dst;
    const void* src;
    size_t n;
    void* dst2 = nullptr;
    size_t n2 = 0;
  };

  CopyPool() {
    int n = std::min(8u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("CALLFS_RS_COPY_THREADS")) n = std::max(1, std::atoi(e));
    for (int i = 1; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }

  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  void run(const std::vector<Seg>& segs) {
    size_t total = 0;
    for (const Seg& s : segs) total += s.n;
    if (workers_.empty() || total < kInline) {
      for (const Seg& s : segs) copy(s);
      return;
    }
    Job job;
    for (const Seg& s : segs)
      for (size_t o = 0; o < s.n; o += kPiece) {
        const size_t len = std::min(kPiece, s.n - o);
        const size_t len2 = s.dst2 && s.n2 > o ? std::min(len, s.n2 - o) : 0;
        job.pieces.push_back({static_cast<uint8_t*>(s.dst) + o,
                              static_cast<const uint8_t*>(s.src) + o, len,
                              len2 ? static_cast<uint8_t*>(s.dst2) + o : nullptr, len2});
      }
    {
      std::lock_guard<std::mutex> g(mu_);
      queue_.push_back(&job);
    }
    cv_.notify_all();
    work(job);
    std::unique_lock<std::mutex> lk(mu_);
    unlink(&job);
    done_.wait(lk, [&] { return job.users == 0; });
  }

 private:
  static constexpr size_t kPiece = 1u << 20;
  static constexpr size_t kInline = 256u << 10;
  struct Job {
    std::vector<Seg> pieces;
    std::atomic<size_t> next{0};
    int users = 0;  // workers inside work(); guarded by mu_
  };

  static void copy(const Seg& s) {
    if (s.n) std::memcpy(s.dst, s.src, s.n);
    if (s.dst2 && s.n2) std::memcpy(s.dst2, s.src, std::min(s.n, s.n2));
  }

  static void work(Job& j) {
    for (size_t i; (i = j.next.fetch_add(1)) < j.pieces.size();) copy(j.pieces[i]);
  }

  void unlink(Job* j) {
    for (auto it = queue_.begin(); it != queue_.end(); ++it)
      if (*it == j) {
        queue_.erase(it);
        return;
      }
  }

  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
      if (stop_) return;
      Job* j = queue_.front();
      ++j->users;
      lk.unlock();
      work(*j);
      lk.lock();
      unlink(j);  // every piece is taken
      if (--j->users == 0) done_.notify_all();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::deque<Job*> queue_;
  std::vector<std::thread> workers_;
  bool stop_ = false;
};

}  // namespace callfs
