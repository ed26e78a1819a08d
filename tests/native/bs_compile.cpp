// Compiles the bit-sliced kernels of a few coefficient blocks with hiprtc on the CPU (no GPU
// needed; built by tests/test_native_host.py with hipcc): every generated source compiles for
// gfx950 and the occupancy search ends with at most 16 spilled VGPRs.
// usage: bs_compile k,m [k,m ...]   (the encode matrix's parity rows, at most 16 of them)
#include <cstdio>
#include <cstdlib>
#include <string>

#include "bitslice.hpp"

using namespace callfs;

int main(int argc, char** argv) {
  int bad = 0;
  for (int a = 1; a < argc; ++a) {
    int k = 0, m = 0;
    if (std::sscanf(argv[a], "%d,%d", &k, &m) != 2) return 2;
    Mat E;
    if (!encode_matrix(k, m, E)) return 2;
    const int R = m < 16 ? m : 16;
    std::vector<uint8_t> coef(static_cast<size_t>(R) * k);
    for (int r = 0; r < R; ++r)
      for (int i = 0; i < k; ++i) coef[static_cast<size_t>(r) * k + i] = E.at(k + r, i);
    auto kern = bs::kernel_for(k, R, coef.data());
    const bool ok = kern->compile_now();
    std::printf("RS(%d,%d) ok=%d waves=%d spills=%d %.2f s%s%.400s\n", k, m, ok, kern->waves_floor(),
                kern->spills(), kern->compile_seconds(), ok ? "" : " ", ok ? "" : kern->error().c_str());
    bad |= !ok || kern->spills() > 16;
  }
  std::printf(bad ? "bs_compile FAILED\n" : "bs_compile ok\n");
  return bad;
}
