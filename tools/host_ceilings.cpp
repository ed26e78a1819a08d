// Host-side transfer ceilings for the host-memory RS path (development tool, not
// product): pinned H2D / D2H / both directions at once, H2D straight from pageable
// memory, hipHostRegister cost, and pageable<->pinned memcpy with T threads.
// They bound tools/e2e_native's end-to-end rates.
//
// build: hipcc -O2 -std=c++17 tools/host_ceilings.cpp -lpthread -o tools/host_ceilings
// run:   tools/host_ceilings [MiB=64] [reps=20]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,           \
                   hipGetErrorString(e_));                                     \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

using clk = std::chrono::steady_clock;

static double secs(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

static void line(const char* what, double bytes, double s, const char* note = "") {
  std::printf("{\"what\": \"%s\", \"GB/s\": %.2f, \"bytes\": %.0f, \"s\": %.6f%s%s}\n", what,
              bytes / s / 1e9, bytes, s, *note ? ", \"note\": " : "", note);
}

int main(int argc, char** argv) {
  const size_t MiB = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 64;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  const size_t n = MiB << 20;
  void *pin_a, *pin_b, *dev_a, *dev_b;
  CK(hipHostMalloc(&pin_a, n, hipHostMallocDefault));
  CK(hipHostMalloc(&pin_b, n, hipHostMallocDefault));
  CK(hipMalloc(&dev_a, n));
  CK(hipMalloc(&dev_b, n));
  std::vector<uint8_t> page_a(n, 1), page_b(n, 2);  // touched pageable buffers
  std::memset(pin_a, 3, n);
  std::memset(pin_b, 4, n);
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));

  auto timed = [&](auto&& body) {
    body();  // warm
    CK(hipDeviceSynchronize());
    const auto t0 = clk::now();
    for (int r = 0; r < reps; ++r) body();
    CK(hipDeviceSynchronize());
    return secs(t0, clk::now()) / reps;
  };
  line("pinned H2D", n, timed([&] { CK(hipMemcpyAsync(dev_a, pin_a, n, hipMemcpyHostToDevice, s1)); }));
  line("pinned D2H", n, timed([&] { CK(hipMemcpyAsync(pin_b, dev_b, n, hipMemcpyDeviceToHost, s1)); }));
  line("pinned H2D + D2H concurrent (sum)", 2.0 * n, timed([&] {
         CK(hipMemcpyAsync(dev_a, pin_a, n, hipMemcpyHostToDevice, s1));
         CK(hipMemcpyAsync(pin_b, dev_b, n, hipMemcpyDeviceToHost, s2));
       }));
  line("pageable H2D (runtime-staged)", n, timed([&] {
         CK(hipMemcpyAsync(dev_a, page_a.data(), n, hipMemcpyHostToDevice, s1));
       }));
  line("pageable D2H (runtime-staged)", n, timed([&] {
         CK(hipMemcpyAsync(page_b.data(), dev_b, n, hipMemcpyDeviceToHost, s1));
       }));
  {
    // register + H2D + unregister of a pageable buffer, as a zero-staging alternative
    const double t = timed([&] {
      CK(hipHostRegister(page_a.data(), n, hipHostRegisterDefault));
      CK(hipMemcpyAsync(dev_a, page_a.data(), n, hipMemcpyHostToDevice, s1));
      CK(hipStreamSynchronize(s1));
      CK(hipHostUnregister(page_a.data()));
    });
    line("hipHostRegister + H2D + unregister", n, t);
    const double tr = timed([&] {
      CK(hipHostRegister(page_a.data(), n, hipHostRegisterDefault));
      CK(hipHostUnregister(page_a.data()));
    });
    line("hipHostRegister + unregister only", n, tr);
  }
  {
    // fresh (never registered) pageable buffers each rep: what a request's Go heap buffer is
    std::vector<std::vector<uint8_t>> fresh(reps + 1);
    for (auto& f : fresh) f.assign(n, 5);
    int i = 0;
    const double t = timed([&] {
      void* p = fresh[i++ % fresh.size()].data();
      CK(hipHostRegister(p, n, hipHostRegisterDefault));
      CK(hipMemcpyAsync(dev_a, p, n, hipMemcpyHostToDevice, s1));
      CK(hipStreamSynchronize(s1));
      CK(hipHostUnregister(p));
    });
    line("fresh buffer: hipHostRegister + H2D + unregister", n, t);
    int j = 0;
    const double t2 = timed([&] {
      void* p = fresh[j++ % fresh.size()].data();
      CK(hipMemcpyAsync(dev_a, p, n, hipMemcpyHostToDevice, s1));
      CK(hipStreamSynchronize(s1));
    });
    line("fresh buffer: pageable H2D (runtime-staged)", n, t2);
    int q = 0;
    const double t3 = timed([&] {
      void* p = fresh[q++ % fresh.size()].data();
      CK(hipMemcpyAsync(p, dev_b, n, hipMemcpyDeviceToHost, s1));
      CK(hipStreamSynchronize(s1));
    });
    line("fresh buffer: pageable D2H (runtime-staged)", n, t3);
    // host-side blocking of a pageable async H2D: time until hipMemcpyAsync returns
    const auto a0 = clk::now();
    CK(hipMemcpyAsync(dev_a, fresh[0].data(), n, hipMemcpyHostToDevice, s1));
    const auto a1 = clk::now();
    CK(hipStreamSynchronize(s1));
    const auto a2 = clk::now();
    std::printf("{\"what\": \"pageable H2D async: call returns after\", \"s\": %.6f, \"total_s\": %.6f}\n",
                secs(a0, a1), secs(a0, a2));
  }
  {
    void* nc;
    CK(hipHostMalloc(&nc, n, hipHostMallocNonCoherent));
    std::memset(nc, 6, n);
    line("non-coherent pinned H2D", n, timed([&] { CK(hipMemcpyAsync(dev_a, nc, n, hipMemcpyHostToDevice, s1)); }));
    line("non-coherent pinned D2H", n, timed([&] { CK(hipMemcpyAsync(nc, dev_b, n, hipMemcpyDeviceToHost, s1)); }));
    CK(hipHostFree(nc));
    std::vector<uint8_t> reg(n, 7);
    CK(hipHostRegister(reg.data(), n, hipHostRegisterDefault));
    line("registered pageable D2H", n, timed([&] { CK(hipMemcpyAsync(reg.data(), dev_b, n, hipMemcpyDeviceToHost, s1)); }));
    CK(hipHostUnregister(reg.data()));
  }
  for (int T : {1, 2, 4, 8, 16}) {
    auto par_copy = [&](void* dst, const void* src) {
      std::vector<std::thread> th;
      const size_t per = (n + T - 1) / T;
      for (int t = 0; t < T; ++t)
        th.emplace_back([=] {
          const size_t o = per * t;
          if (o < n) std::memcpy(static_cast<uint8_t*>(dst) + o, static_cast<const uint8_t*>(src) + o, std::min(per, n - o));
        });
      for (auto& x : th) x.join();
    };
    char what[96];
    std::snprintf(what, sizeof what, "memcpy pageable->pinned, %d threads", T);
    line(what, n, timed([&] { par_copy(pin_a, page_a.data()); }));
    std::snprintf(what, sizeof what, "memcpy pinned->pageable, %d threads", T);
    line(what, n, timed([&] { par_copy(page_b.data(), pin_b); }));
  }
  std::printf("{\"what\": \"hardware_concurrency\", \"value\": %u}\n", std::thread::hardware_concurrency());
  return 0;
}
