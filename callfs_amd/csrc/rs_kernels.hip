// Kernel instantiations and launch dispatch for the RS path (device code in
// rs_apply.hpp). The production policy is chosen from tools/kbench.hip measurements
// on MI355X (DESIGN.md "Kernel tuning log").
#include <algorithm>
#include <array>
#include <mutex>
#include <utility>

#include "rs_apply.hpp"

namespace callfs {

namespace {

using dev::kBlock;

// Production policy (tools/kbench.hip on MI355X, RS(10,4) 1 MiB shards x 256 stripes,
// DESIGN.md "Kernel tuning log"): runtime-K pair loop, non-temporal loads and stores,
// 512-thread blocks, two input pairs in flight = 6118-6168 GB/s (76.5-77.1 % of
// 8 TB/s) vs 5457 GB/s for the first compile-time-K / plain-load version and
// 5957 GB/s for an XOR-only kernel with the same loads and stores.
using ProdPolicy = dev::Policy<4, 1, true, true, false, 512, 2, 0>;

// Row groups of 5..16 use the LDS nibble-table kernel: its cost does not grow with the
// row count (RS(10,8): 5,749 vs 4,887 GB/s; RS(32,8): 4,783 vs 3,948; RS(12,6): 5,318
// vs 5,118 — tools/kbench.hip), while for R <= 4 the v_perm kernel is faster.
using LdsPolicy = dev::Policy<2, 1, true, true, false, 512, 2, 0>;
constexpr int kLdsMinRows = 5;
constexpr int kPermMaxRows = 8;  // v_perm kernel instantiations (production uses <= 4)

using VecFn = void (*)(ApplyArgs);
using ByteFn = void (*)(ApplyArgs, uint64_t);

template <int... Rs>
constexpr auto vec_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_vec<0, Rs + 1, ProdPolicy>...};
}

template <int... Rs>
constexpr auto lds_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, LdsPolicy>...};
}

template <int... Rs>
constexpr auto byte_table(std::integer_sequence<int, Rs...>) {
  return std::array<ByteFn, sizeof...(Rs)>{&dev::rs_apply_bytes<Rs + 1>...};
}

const auto kVec = vec_table(std::make_integer_sequence<int, kPermMaxRows>{});
// R 1..8 exact; R 9..16 share the 16-row instance (rs_apply_lds: b128 table reads).
const auto kLds = lds_table(std::make_integer_sequence<int, kPermMaxRows>{});
const VecFn kLdsWide = &dev::rs_apply_lds<kMaxRowsPerLaunch, LdsPolicy>;
const auto kByte = byte_table(std::make_integer_sequence<int, kMaxRowsPerLaunch>{});

}  // namespace

hipError_t launch_apply(ApplyArgs a, bool aligned, hipStream_t stream) {
  if (a.R < 1 || a.R > kMaxRowsPerLaunch || a.K < 1 || a.K > kMaxK || a.batch < 1)
    return hipErrorInvalidValue;
  if (a.S == 0) return hipSuccess;
  uint64_t tail0 = 0;
  if (aligned) {
    a.nvec = a.S / 16;
    tail0 = a.nvec * 16;
    if (a.nvec) {
      if (a.R >= kLdsMinRows || a.R > kPermMaxRows) {
        if (!a.ltabs) return hipErrorInvalidValue;
        const size_t lds = dev::lds_bytes(a.K, a.R);
        const int fi = a.R > kPermMaxRows ? kPermMaxRows : a.R - 1;
        VecFn fn = a.R > kPermMaxRows ? kLdsWide : kLds[fi];
        if (lds > (64u << 10)) {  // wide groups with many shards: opt in once per kernel
          static std::once_flag once[kPermMaxRows + 1];
          std::call_once(once[fi], [fn] {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10);
          });
        }
        const unsigned gx = dev::vec_grid<LdsPolicy>(a.nvec, a.batch);
        hipLaunchKernelGGL(fn, dim3(gx), dim3(LdsPolicy::BS), lds, stream, a);
      } else {
        const unsigned gx = dev::vec_grid<ProdPolicy>(a.nvec, a.batch);
        hipLaunchKernelGGL(kVec[a.R - 1], dim3(gx), dim3(ProdPolicy::BS), 0, stream, a);
      }
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  } else {
    a.nvec = 0;
  }
  if (tail0 < a.S) {
    const unsigned gy = static_cast<unsigned>(std::min(a.batch, 65535));
    const uint64_t gx = (a.S - tail0 + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(kByte[a.R - 1], dim3(static_cast<unsigned>(gx), gy), dim3(kBlock), 0,
                       stream, a, tail0);
    return hipGetLastError();
  }
  return hipSuccess;
}

}  // namespace callfs
