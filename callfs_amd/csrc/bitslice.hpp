// Bit-sliced GF(2^8) kernels compiled at plan time: the runtime around
// bitslice_gen.hpp. One Kernel per distinct coefficient block (K inputs x R rows), compiled
// once per process by hiprtc for the device's gfx target (and kept in an on-disk cache of code
// objects), loaded into each device on first use. tests/native/bs_worker.cpp drives the
// compile state machine from eight threads under ThreadSanitizer.
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "bitslice_gen.hpp"
#include "dispatch.hpp"

namespace callfs {
namespace bs {

class Kernel : public std::enable_shared_from_this<Kernel> {
 public:
  enum class State { kIdle, kQueued, kCompiling, kReady, kFailed };
  Kernel(int K, int R, const uint8_t* coef);
  ~Kernel();
  Kernel(const Kernel&) = delete;
  Kernel& operator=(const Kernel&) = delete;

  int K() const { return net_.K; }
  int R() const { return net_.R; }
  int block_threads() const { return opt_.block; }
  int tile_vecs() const { return opt_.tile_vecs(); }
  State state() const;
  // Queues the compile on the background worker (no-op once queued or done). The worker is
  // drained at exit before hiprtc's own teardown; requests made while exiting, or in a fork's
  // child, are dropped (the kernel then stays on the nibble-table forms).
  void compile_async();
  // Compiles on the calling thread if nobody has (waits for a compile in flight); true when
  // the code object exists.
  bool compile_now();
  // The kernel for HIP device `device` (the caller's current device), loading the module on
  // first use; null when not compiled or the load failed. wait: compile first if needed.
  hipFunction_t function(int device, bool wait);
  // Compiler-reported resources of the code object (0 before it exists).
  int vgprs() const { return vgprs_; }
  int waves_floor() const { return waves_; }
  int spills() const { return spills_; }
  double compile_seconds() const { return compile_s_; }
  const std::string& error() const { return error_; }

 private:
  friend class Worker;
  void compile_locked(std::unique_lock<std::mutex>& lk);

  Network net_;
  std::string arch_;  // the gfx target the code object is compiled for
  GenOptions opt_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  State state_ = State::kIdle;
  std::vector<char> code_;
  std::string error_;
  int vgprs_ = 0;
  int waves_ = 0;
  int spills_ = -1;
  double compile_s_ = 0;
  hipModule_t mod_[kMaxDevices] = {};
  hipFunction_t fn_[kMaxDevices] = {};
};

// The process-wide kernel for a coefficient block (coef: [R][K] row-major); never null.
std::shared_ptr<Kernel> kernel_for(int K, int R, const uint8_t* coef);

// CALLFS_RS_BITSLICE: 0 = never, 1 / auto (default) = the rule's launch groups once their
// kernel is compiled (plans compile it at creation), sync = compile on first use and wait.
enum class Mode { kOff, kAuto, kSync };
Mode mode();

// Launches rs_bs over `tiles` tiles starting at a.t_base (`block` threads per tile);
// ev_start / ev_stop as hipExtModuleLaunchKernel takes them.
hipError_t launch(hipFunction_t fn, const Args& a, uint32_t tiles, int block, hipStream_t stream,
                  hipEvent_t ev_start, hipEvent_t ev_stop);

}  // namespace bs
}  // namespace callfs
