// The bit-sliced kernels' compile state machine under concurrency (bitslice.hpp Kernel,
// Worker, kernel_for), on the CPU: hiprtc compiles without a GPU, and nothing here loads a
// module. Built by tests/test_native_host.py with ThreadSanitizer on the host code.
//
// Eight threads ask for kernels of four coefficient blocks (two of them the same block under
// different vectors, which must map to one Kernel), queue background compiles, wait on
// synchronous ones and poll states in every interleaving; every kernel must end Ready exactly
// once with a code object, a forked child must exit cleanly, and the process must exit with
// the worker joined.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include <sys/wait.h>
#include <unistd.h>

#include "bitslice.hpp"

using namespace callfs;

int main() {
  std::vector<std::vector<uint8_t>> blocks;
  const int shapes[4][2] = {{10, 9}, {12, 9}, {10, 9}, {6, 12}};  // K, R; [2] repeats [0]
  for (int s = 0; s < 4; ++s) {
    const int K = shapes[s][0], R = shapes[s][1];
    std::vector<uint8_t> c(static_cast<size_t>(K) * R);
    for (size_t i = 0; i < c.size(); ++i) c[i] = static_cast<uint8_t>((i * 37 + (s == 2 ? 0 : s) * 11 + 1) & 0xff);
    blocks.push_back(c);
  }
  std::atomic<int> bad{0};
  std::vector<std::shared_ptr<bs::Kernel>> seen(8 * 4);
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      for (int rep = 0; rep < 4; ++rep) {
        const int s = (t + rep) % 4;
        auto k = bs::kernel_for(shapes[s][0], shapes[s][1], blocks[s].data());
        seen[t * 4 + rep] = k;
        if ((t + rep) & 1) {
          k->compile_async();
          (void)k->state();
        }
        if (!k->compile_now()) bad++;
        if (k->state() != bs::Kernel::State::kReady) bad++;
      }
    });
  for (auto& x : th) x.join();
  // one Kernel per coefficient block: blocks 0 and 2 are the same bytes
  std::shared_ptr<bs::Kernel> k0, k2;
  for (int t = 0; t < 8; ++t)
    for (int rep = 0; rep < 4; ++rep) {
      const int s = (t + rep) % 4;
      if (s == 0) k0 = k0 ? k0 : seen[t * 4 + rep];
      if (s == 2) k2 = k2 ? k2 : seen[t * 4 + rep];
      if (s == 0 && seen[t * 4 + rep] != k0) bad++;
    }
  if (!k0 || k0 != k2) bad++;
  // a fork's child (the worker thread is the parent's): a compile request is ignored and
  // exit's drain does not join a thread the child does not have
  const pid_t pid = fork();
  if (pid == 0) {
    std::vector<uint8_t> c(11 * 9, 3);
    bs::kernel_for(11, 9, c.data())->compile_async();
    std::exit(0);
  }
  int status = -1;
  if (pid < 0 || waitpid(pid, &status, 0) != pid || !WIFEXITED(status) || WEXITSTATUS(status) != 0) {
    std::printf("forked child: status %d\n", status);
    bad++;
  }
  // a queued compile of a fresh block still in the worker's queue at exit is dropped, the
  // compile in flight finishes and the worker is joined (static teardown)
  std::vector<uint8_t> late(14 * 9, 7);
  bs::kernel_for(14, 9, late.data())->compile_async();
  std::printf(bad ? "bs_worker FAILED %d\n" : "bs_worker ok\n", bad.load());
  return bad ? 1 : 0;
}
