// Kernel instantiations and launch dispatch for the RS path (device code in
// rs_apply.hpp). The production policy is chosen from tools/kbench.hip measurements
// on MI355X (DESIGN.md "Kernel tuning log").
#include <algorithm>
#include <array>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <string>
#include <type_traits>
#include <utility>

#include <hip/hip_ext.h>

#include "bitslice.hpp"
#include "bitslice_rule.hpp"
#include "dispatch.hpp"
#include "rs_apply.hpp"
#include "tile_order.hpp"
#include "tune_table.hpp"

namespace callfs {

namespace {

using dev::kBlock;

// v_perm kernel policy (tools/kbench.hip on MI355X, RS(10,4) 1 MiB shards x 256 stripes,
// DESIGN.md "Kernel tuning log"): runtime-K pair loop, non-temporal loads and stores,
// 512-thread blocks, two input pairs in flight = 6118-6168 GB/s (76.5-77.1 % of
// 8 TB/s) vs 5457 GB/s for the first compile-time-K / plain-load version and
// 5957 GB/s for an XOR-only kernel with the same loads and stores. Used for k <= 3.
using ProdPolicy = dev::Policy<4, 1, true, true, false, 512, 2, 0>;
using ProdG2Policy = dev::Policy<4, 1, true, true, false, 512, 2, 5>;
using ProdQ16Policy = dev::Policy<4, 1, true, true, false, 512, 2, 8>;

// The LDS nibble-table kernel takes every launch with k >= 4 inputs or R >= 5 rows. Its
// cost per data byte barely grows with R, and with all 8 lookups of a dword in flight it
// also beats the v_perm kernel at R <= 4 (tools/kbench.hip, rotated order, 5 rounds,
// % of 8 TB/s): RS(10,4) 78.6 vs 73.0-75.7, RS(16,4) 77.4 vs 72.2-73.2, RS(20,4) 75.9
// vs 70.2-71.2, RS(4,2) 78.6 vs 76.6, RS(10,8) 71-72 vs 62, RS(32,8) 69.7 vs 49.3.
// With k <= 3 the per-block table prologue does not pay (RS(3,2): 73.3 vs 77.5-79.9),
// so those launches keep the v_perm kernel. One instance per R.
using LdsPolicy = dev::Policy<2, 1, true, true, false, 512, 2, 0>;
// Row groups of 9..16 (16-byte table entries, 100-127 VGPRs, 4 waves/SIMD): fewer waves
// hold fewer loads in flight, so they prefetch 4 input shards ahead through an unrolled
// 5-slot ring. RS(10,12) 61.5 -> 68.0 %, RS(10,16) 63.2 -> 69.3 %, RS(20,16) 59.3 ->
// 60.7 % of 8 TB/s (tools/kbench.hip, KB_RING). For R <= 8 the unrolled ring measured
// 1-3 % slower than the shifted ring of three, so those keep LdsPolicy.
// Their table addresses are formed by v_or_b32_sdwa (byte select + OR with an SGPR
// base) instead of v_perm_b32: same issue rate (tools/valu_rates.hip, 0.24 per SIMD
// clock), but no VGPR for the table base, which keeps R = 16 at 125 VGPRs (4 waves per
// SIMD; the v_perm form had grown to 129 = 3 waves once the ragged tail moved into the
// kernel). profiles/r02/sdwa/, % of 8 TB/s, v_perm -> SDWA:
// RS(10,16) 58.3 -> 66.8, RS(20,16) 52.2 -> 59.3, RS(32,16) 49.0 -> 55.0, RS(10,12)
// 65.9 -> 66.5.
using LdsWidePolicy = dev::Policy<2, 1, true, true, false, 512, 4, 0, 1, false, false, true>;
using LdsWideQ8Policy = dev::Policy<2, 1, true, true, false, 512, 4, 6, 1, false, false, true>;
template <int R>
using LdsPolicyFor = typename std::conditional<(R > 8), LdsWidePolicy, LdsPolicy>::type;
using LdsG8Policy = dev::Policy<2, 1, true, true, false, 512, 2, 2>;
using LdsG2Policy = dev::Policy<2, 1, true, true, false, 512, 2, 5>;
using LdsQ8Policy = dev::Policy<2, 1, true, true, false, 512, 2, 6>;
using LdsQ16Policy = dev::Policy<2, 1, true, true, false, 512, 2, 8>;
using LdsX8Policy = dev::Policy<2, 1, true, true, false, 512, 2, 10>;
using LdsX32Policy = dev::Policy<2, 1, true, true, false, 512, 2, 11>;
// Launch groups of R <= 4 rows with Verify rows load the compared vectors 4 shards before
// the end of the input loop (rs_apply.hpp Policy::VPF):
// profiles/r02/verify_prefetch/, RS(10,4) 1 MiB x 256, % of 8 TB/s, after the loop ->
// prefetch distance 2 / 4 / 6 / 8: one write + three compare rows 71.6 -> 72.7 / 74.1 /
// 73.7 / 73.3, four compare rows 78.0 -> 79.3 / 80.9 / 80.8 / 79.5. Without Verify rows
// the same code measured 0.4 points slower (the extra registers), so encode launches keep
// the policies above: one instance per tile order.
template <int ORD>
using LdsVerifyPolicy = dev::Policy<2, 1, true, true, false, 512, 2, ORD, 0, false, 0, false, 0, 4>;
// Misaligned shards (upstream Split layout of contiguous objects at odd S) with R <= 8:
// loads from aligned addresses realigned in registers, and parity stores to aligned
// addresses realigned the same way (62 vectors per wave; the bytes no aligned block
// covers are written by each stripe's first tile; rs_apply.hpp REALIGN 2). Round 1's
// form realigned only the loads (REALIGN 1, 63 vectors per wave, k >= 8; kept in
// tools/kbench for comparison). Round 2,
// profiles/r02/realign_out/, % of 8 TB/s, unaligned -> loads realigned -> loads and stores
// realigned: RS(10,4) 64 MiB objects (S = 6,710,887) 67.6 -> 68.1 -> 69.5, RS(10,8)
// 1,048,577 B 63.9 -> 65.3 -> 67.0, RS(6,3) 65.6 -> 67.0 -> 71.5, RS(5,3) 68.7 -> 66.7
// -> 72.2, RS(4,2) 69.0 -> 69.1 -> 69.8; RS(12,4) S = 5,592,406 ran 71.2 unaligned and
// 68.9 realigned, so rs_plan_tune offers the unaligned kernel as an alternative.
// (R <= 4 asks for 8 waves per SIMD: left alone the compiler used 106 SGPRs, 7 waves)
// One instance per tile order it runs in: consecutive, X8, X32 (tile_order.hpp block_tile).
// R <= 4 with 6-bit lookups over shard triples (rs_apply.hpp Policy::WIX): 4 lookups per
// byte position of three shards instead of 6; one instance per tile order.
template <int ORD>
using LdsWixPolicy = dev::Policy<8, 1, true, true, false, 512, 2, ORD, 0, false, 0, false, 0, 0, 1>;
// The triple loop with nibble lookups, R <= 8 (the rule's triple form, tile_order.hpp
// tri_rule_order; orders kOrderTri + TileOrder)
template <int R, int ORD>
using LdsTriPolicy = dev::Policy<(R <= 4 ? 8 : 2), 1, true, true, false, 512, 2, ORD, 0, false, 0, false, 0, 0, 2>;
// The triple loop with the Verify rows' compare loads issued with the triple that reaches
// K - 4 (Policy::VPF, as LdsVerifyPolicy): launches of R <= 4 rows that mix written and
// Verify rows (the one-erasure decode of a download) when they take triples
template <int ORD>
using LdsTriVerifyPolicy = dev::Policy<2, 1, true, true, false, 512, 2, ORD, 0, false, 0, false, 0, 4, 2>;
// The realigning kernel with its aligned loads issued in triples (rs_apply.hpp REALIGN
// with WIX 2)
template <int R, int ORD>
using LdsRealignTriPolicy =
    dev::Policy<(R <= 4 ? 7 : 2), 1, true, true, false, 512, 2, ORD, 0, false, 2, false, 0, 0, 2>;
// Misaligned inputs with 16-B-aligned outputs (upstream Split of an io.ReadAll body: the
// data shards inside the body, the parity in reedsolomon's AllocAligned buffers): 64-vector
// waves, lane 63's neighbour vector from one single-lane load per shard (rs_apply.hpp
// REALIGN 5), so the parity stores fill whole 1 KiB windows
template <int R, int ORD>
using LdsRealign64Policy =
    dev::Policy<6, 1, true, true, false, 512, 2, ORD, 0, false, 5>;
// ... and the realigning kernel's aligned loads double-buffered in two triple sets
// (rs_apply.hpp WIX 3 with REALIGN 2), R <= 4 and K >= 6 (kTriDbMinK): A/B instances
// behind the realign-tri orders
template <int ORD>
using LdsRealignTriDbPolicy = dev::Policy<5, 1, true, true, false, 512, 2, ORD, 0, false, 2, false, 0, 0, 3>;
template <int ORD>
using LdsRealignOutPolicy = dev::Policy<2, 1, true, true, false, 512, 2, ORD, 0, false, 2>;
// Input vectors staged through an LDS-DMA ring of kDmaDepth shards per wave (rs_apply.hpp
// Policy::DMA): R <= 8, aligned shards, at most 64 KiB of LDS (K <= 64); A/B build
constexpr int kDmaDepth = 6;
template <int R, int ORD>
using LdsDmaPolicy = dev::Policy<(R <= 4 ? 8 : 6), 1, true, true, false, 512, 2, ORD, 0, false, 0,
                                 false, 0, 0, 0, kDmaDepth>;
template <int ORD>
using LdsRealignOut8Policy = dev::Policy<8, 1, true, true, false, 512, 2, ORD, 0, false, 2>;
template <int R, int ORD>
using LdsRealignOutPolicyFor =
    typename std::conditional<(R <= 4), LdsRealignOut8Policy<ORD>, LdsRealignOutPolicy<ORD>>::type;
// CALLFS_RS_TILE_ORDER=consecutive|g8|g2|q8|q16|x8|x32 overrides the rule for every LDS-kernel
// launch with R <= 8 (A/B on a deployment's own shard layout; unset = the rule).
int tile_order_override() {
  static const int v = [] {
    const char* e = std::getenv("CALLFS_RS_TILE_ORDER");
    if (!e) return -1;
    const std::string o(e);
    if (o == "consecutive") return static_cast<int>(TileOrder::kConsecutive);
    if (o == "g8") return static_cast<int>(TileOrder::kGroup8);
    if (o == "g2") return static_cast<int>(TileOrder::kGroup2);
    if (o == "q8") return static_cast<int>(TileOrder::kSeg8);
    if (o == "q16") return static_cast<int>(TileOrder::kSeg16);
    if (o == "x8") return static_cast<int>(TileOrder::kXcd8);
    if (o == "x32") return static_cast<int>(TileOrder::kXcd32);
    return -1;
  }();
  return v;
}
// Tiles per kernel launch. Blocks are dealt to the 8 XCDs round-robin and each XCD runs
// its share in order, so over a long grid the XCDs drift apart and the tiles in flight
// spread over more of the address space than the tile order intends. Grids of more than
// twice about 4 GiB of shard traffic are cut into equal consecutive slices of at most
// that much (one launch each, same tile order), which resets the drift. Round 2 sweep
// (profiles/r02/slice_rule/, % of 8 TB/s, unsliced / 2 GiB /
// 4 GiB slices): RS(10,4) 64 MiB objects x 256 (24 GiB) 73.1 / 77.5 / 77.4, 1 MiB x 1,024
// 77.9 / 79.2 / 79.4, RS(4,2) 1 MiB x 2,048 76.8 / 79.2 / 79.3: long memory-bound grids
// need slices, and 4 GiB ones keep the gain. Every slice boundary drains the machine,
// which costs the grids of 4.5-12 GiB that 2 GiB slices used to cut: RS(10,8) 73.9 / 73.4
// / 74.0, RS(10,16) 69.3 / 68.0 / 69.2 (unsliced at 4 GiB), RS(20,4) 77.4 / 75.9 / 75.8
// (unsliced at 4 GiB), RS(32,8) 70.1 / 68.4 / 69.6, RS(32,16) 56.0 / 54.6 / 55.8; the
// bench grid (3.5 GiB) stays whole either way. CALLFS_RS_MAX_TILES_PER_LAUNCH sets the
// slice in tiles instead.
std::atomic<long long> g_slice_tiles_override{-1};

uint32_t slice_tiles(int streams) {
  static const long forced = [] {
    const char* e = std::getenv("CALLFS_RS_MAX_TILES_PER_LAUNCH");
    return e ? std::atol(e) : 0L;
  }();
  const long long ov = g_slice_tiles_override.load(std::memory_order_relaxed);
  if (ov == 0) return ~0u;  // never slice
  if (ov > 0) return static_cast<uint32_t>(std::min<long long>(std::max<long long>(ov, 1024), 1LL << 30));
  if (forced >= 1024) return static_cast<uint32_t>(std::min<long>(forced, 1L << 30));
  const uint64_t tile_bytes = 8192ull * static_cast<uint64_t>(std::max(1, streams));
  return static_cast<uint32_t>(std::max<uint64_t>(4096, (4ull << 30) / tile_bytes));
}

// Launches `grid` blocks of one kernel as consecutive slices (see slice_tiles). Launches
// that only compare (every row a Verify row, no stores) stay whole: read-only streams
// lose ≈ 1 point to the slice drains and gain nothing (configs[2] shape with nothing
// erased: 79.0-79.4 % whole vs 78.0-78.4 % sliced).
// launch(blocks, first, last): first / last = this is the launch's first / last slice.
template <class Launch>
void launch_sliced(uint32_t grid, int streams, ApplyArgs& a, Launch&& launch) {
  const uint32_t all_rows = a.R >= 32 ? ~0u : (1u << a.R) - 1;
  const bool read_only = (a.verify_mask & all_rows) == all_rows;
  const uint32_t lim = read_only ? grid : slice_tiles(streams);
  const uint32_t nsl = grid / 2 > lim ? (grid + lim - 1) / lim : 1;
  const uint32_t per = (grid + nsl - 1) / nsl;
  for (uint32_t t0 = 0; t0 < grid; t0 += per) {
    a.t_base = t0;
    launch(std::min(per, grid - t0), t0 == 0, t0 + per >= grid);
  }
  a.t_base = 0;
}

// One dispatch of kernel fn; with events, the first dispatch of a launch records ev.start
// at its start and the last records ev.stop at its end (hipExtLaunchKernel).
template <class... Args>
void dispatch(void (*fn)(Args...), dim3 grid, dim3 block, size_t lds, hipStream_t stream,
              const LaunchEvents& ev, bool first, bool last, Args... args) {
  if (ev.start || ev.stop)
    hipExtLaunchKernelGGL(fn, grid, block, static_cast<uint32_t>(lds), stream,
                          first ? ev.start : nullptr, last ? ev.stop : nullptr, 0, args...);
  else
    hipLaunchKernelGGL(fn, grid, block, lds, stream, args...);
}
constexpr int kLdsMinRows = 5;
constexpr int kLdsMinK = 4;
constexpr int kPermMaxRows = 4;  // v_perm kernel: k <= 3 and R <= 4 (takes_lds sends the rest to LDS)

using VecFn = void (*)(ApplyArgs);
using ByteFn = void (*)(ApplyArgs, uint64_t);

template <int... Rs>
constexpr auto vec_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_vec<0, Rs + 1, ProdPolicy>...};
}

template <int... Rs>
constexpr auto lds_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, LdsPolicyFor<Rs + 1>>...};
}

template <class P, int... Rs>
constexpr auto lds_order_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, P>...};
}

template <int... Rs>
constexpr auto byte_table(std::integer_sequence<int, Rs...>) {
  return std::array<ByteFn, sizeof...(Rs)>{&dev::rs_apply_bytes<Rs + 1>...};
}

const auto kVec = vec_table(std::make_integer_sequence<int, kPermMaxRows>{});
template <class P, int... Rs>
constexpr auto vec_order_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_vec<0, Rs + 1, P>...};
}
const auto kVecG2 = vec_order_table<ProdG2Policy>(std::make_integer_sequence<int, 4>{});
const auto kVecQ16 = vec_order_table<ProdQ16Policy>(std::make_integer_sequence<int, 4>{});
const auto kLds = lds_table(std::make_integer_sequence<int, kMaxRowsPerLaunch>{});
const auto kLdsG8 = lds_order_table<LdsG8Policy>(std::make_integer_sequence<int, 8>{});
const auto kLdsG2 = lds_order_table<LdsG2Policy>(std::make_integer_sequence<int, 8>{});
const auto kLdsQ8 = lds_order_table<LdsQ8Policy>(std::make_integer_sequence<int, 8>{});
const auto kLdsQ16 = lds_order_table<LdsQ16Policy>(std::make_integer_sequence<int, 8>{});
const auto kLdsX8 = lds_order_table<LdsX8Policy>(std::make_integer_sequence<int, 8>{});
const auto kLdsX32 = lds_order_table<LdsX32Policy>(std::make_integer_sequence<int, 8>{});
// [tile order][R - 1] for R <= 4 with Verify rows (TileOrder values index the first level)
const std::array<std::array<VecFn, 4>, kTileOrders> kLdsVerify = {
    lds_order_table<LdsVerifyPolicy<0>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsVerifyPolicy<2>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsVerifyPolicy<5>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsVerifyPolicy<6>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsVerifyPolicy<8>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsVerifyPolicy<10>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsVerifyPolicy<11>>(std::make_integer_sequence<int, 4>{})};
#if CALLFS_RS_AB_INSTANCES
// [tile order][R - 1] for R <= 4, 6-bit triple lookups (A/B build)
const std::array<std::array<VecFn, 4>, kTileOrders> kLdsWix = {
    lds_order_table<LdsWixPolicy<0>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsWixPolicy<2>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsWixPolicy<5>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsWixPolicy<6>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsWixPolicy<8>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsWixPolicy<10>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsWixPolicy<11>>(std::make_integer_sequence<int, 4>{})};
#endif
template <int ORD, int... Rs>
constexpr auto lds_tri_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, LdsTriPolicy<Rs + 1, ORD>>...};
}
// [consecutive, G2, X32, Q8, Q16, X8][R - 1] (tri_index)
const std::array<std::array<VecFn, 8>, 6> kLdsTri = {
    lds_tri_table<0>(std::make_integer_sequence<int, 8>{}),
    lds_tri_table<5>(std::make_integer_sequence<int, 8>{}),
    lds_tri_table<11>(std::make_integer_sequence<int, 8>{}),
    lds_tri_table<6>(std::make_integer_sequence<int, 8>{}),
    lds_tri_table<8>(std::make_integer_sequence<int, 8>{}),
    lds_tri_table<10>(std::make_integer_sequence<int, 8>{})};
// The triple loop double-buffered in two register sets with no conditional loads
// (rs_apply.hpp Policy::WIX 3): the compiler's waits then leave six loads in flight where
// the rotating form waited for the next triple inside each iteration. 81 VGPRs (5 waves
// per SIMD) at R <= 4; at R = 8 it needs 131 and lost (3 waves). Launches with R <= 4 and
// K >= 6 that take the triple form run it. profiles/r04/tridb/,
// % of 8 TB/s, rotating -> double-buffered triples in the same order: RS(10,4) 1 MiB 76.6
// -> 80.0 (G2), RS(8,4) 2 MiB 77.4 -> 80.5 (X32), RS(12,4) 1 MiB 79.4 -> 80.9 (G2),
// RS(6,3) 1 MiB 75.6 -> 78.4, 4 MiB 75.8 -> 78.1 (X32), RS(6,3) 174,763 B 72.2 -> 75.9,
// RS(10,4) 16 MiB 77.7 -> 77.9 (Q16); with K = 4 (no loop iteration) it lost 0.5-7 points.
template <int ORD>
using LdsTriDbPolicy = dev::Policy<2, 1, true, true, false, 512, 2, ORD, 0, false, 0, false, 0, 0, 3>;
// [consecutive, G2, X32, Q8, Q16, X8][R - 1] (tri_index), R <= 4
const std::array<std::array<VecFn, 4>, 6> kLdsTriDb = {
    lds_order_table<LdsTriDbPolicy<0>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbPolicy<5>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbPolicy<11>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbPolicy<6>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbPolicy<8>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbPolicy<10>>(std::make_integer_sequence<int, 4>{})};
// ... with the Verify rows' compare loads issued with the last groups' loads (Policy::VPF):
// R <= 4 launches that mix written and Verify rows (one-erasure decodes), K >= 6; 92-96
// VGPRs at 5 waves per SIMD
template <int ORD>
using LdsTriDbVerifyPolicy = dev::Policy<5, 1, true, true, false, 512, 2, ORD, 0, false, 0, false, 0, 4, 3>;
const std::array<std::array<VecFn, 4>, 6> kLdsTriDbVerify = {
    lds_order_table<LdsTriDbVerifyPolicy<0>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbVerifyPolicy<5>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbVerifyPolicy<11>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbVerifyPolicy<6>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbVerifyPolicy<8>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbVerifyPolicy<10>>(std::make_integer_sequence<int, 4>{})};
// CALLFS_RS_TRIDB=0 keeps R <= 4 triple launches on the rotating loop (A/B build only)
bool tridb_enabled() {
  static const bool on = [] {
    const char* e = kAbInstances ? std::getenv("CALLFS_RS_TRIDB") : nullptr;
    return !(e && *e == '0');
  }();
  return on;
}
constexpr int kTriDbMinK = 6;
// Ragged-tail placement (ApplyArgs::tail_in_vec, rs_apply.hpp tail_lane) for a kernel of
// TV-vector tiles and BS-thread blocks: the idle last wave of each stripe's last tile for
// stripes of at most kTailLastMaxTps tiles whose last tile leaves that wave idle, else wave
// 0 of the first tile. Round 4 moved every tail to the last tile (1 MiB-object shards, 7-22
// tiles per stripe, gained 0.4-1.3 points); on long stripes that put the grid's last tile
// behind the tail's load chain (profiles/r04/tail_ab: RS(20,4) S =
// 3,355,444, 410 tiles, first tile 73.8 %, last tile 72.6). CALLFS_RS_TAIL_LAST_TPS
// overrides the bound (A/B build only; clamped so that (tps - 1) << 2 fits the 32-bit code).
// Every LDS policy that takes this code tiles as LdsPolicy does (static_assert in
// launch_apply); the realigning forms place their edges themselves (tail_in_vec = 1).
uint32_t tail_code(uint64_t nvec, uint64_t TV, uint64_t BS) {
  static const uint64_t max_tps = [] {
    const char* e = kAbInstances ? std::getenv("CALLFS_RS_TAIL_LAST_TPS") : nullptr;
    return std::min<uint64_t>(e && *e ? std::strtoull(e, nullptr, 10) : 32ull, 1ull << 29);
  }();
  const uint64_t tps = (nvec + TV - 1) / TV, last = nvec - (tps - 1) * TV;
  if (tps <= max_tps && last + 64 <= BS) return static_cast<uint32_t>(((tps - 1) << 2) | 3u);
  return 1u;
}
// [consecutive, G2, X32, Q8, Q16][R - 1] for R <= 4 with Verify rows (tri_index)
const std::array<std::array<VecFn, 4>, 5> kLdsTriVerify = {
    lds_order_table<LdsTriVerifyPolicy<0>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriVerifyPolicy<5>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriVerifyPolicy<11>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriVerifyPolicy<6>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriVerifyPolicy<8>>(std::make_integer_sequence<int, 4>{})};
template <int ORD, int... Rs>
constexpr auto lds_realign_tri_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, LdsRealignTriPolicy<Rs + 1, ORD>>...};
}
#if CALLFS_RS_AB_INSTANCES
template <int ORD, int... Rs>
constexpr auto lds_dma_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, LdsDmaPolicy<Rs + 1, ORD>>...};
}
// [consecutive, G2, Q8, X32][R - 1] (A/B build)
const std::array<std::array<VecFn, 8>, 4> kLdsDma = {
    lds_dma_table<0>(std::make_integer_sequence<int, 8>{}), lds_dma_table<5>(std::make_integer_sequence<int, 8>{}),
    lds_dma_table<6>(std::make_integer_sequence<int, 8>{}), lds_dma_table<11>(std::make_integer_sequence<int, 8>{})};
int dma_index(TileOrder o) {
  switch (o) {
    case TileOrder::kGroup2: return 1;
    case TileOrder::kSeg8: return 2;
    case TileOrder::kXcd32: return 3;
    default: return 0;
  }
}
// [G4, G8][R - 1]: the double-buffered triples with 4 / 8 stripes interleaved (A/B build)
const std::array<std::array<VecFn, 4>, 2> kLdsTriDbG = {
    lds_order_table<LdsTriDbPolicy<4>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsTriDbPolicy<2>>(std::make_integer_sequence<int, 4>{})};
#endif
bool can_tridb_g(const ApplyArgs& a) {
  const uint32_t rows = a.R >= 32 ? ~0u : (1u << a.R) - 1;
  return kAbInstances && a.R <= 4 && a.K >= kTriDbMinK && !(a.in_misalign | a.out_misalign) &&
         (a.verify_mask & rows) == 0;
}
bool can_dma(const ApplyArgs& a) {
  return kAbInstances && a.R <= 8 && a.K >= 2 && !(a.in_misalign | a.out_misalign) &&
         dev::lds_bytes_dma(a.K, a.R, kDmaDepth) <= (64u << 10);
}
#if CALLFS_RS_AB_INSTANCES
// [consecutive, X8, X32][R - 1], R <= 4 (A/B build)
const std::array<std::array<VecFn, 4>, 3> kLdsRealignTriDb = {
    lds_order_table<LdsRealignTriDbPolicy<0>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsRealignTriDbPolicy<10>>(std::make_integer_sequence<int, 4>{}),
    lds_order_table<LdsRealignTriDbPolicy<11>>(std::make_integer_sequence<int, 4>{})};
#endif
// [consecutive, X8, X32][R - 1]
const std::array<std::array<VecFn, 8>, 3> kLdsRealignTri = {
    lds_realign_tri_table<0>(std::make_integer_sequence<int, 8>{}),
    lds_realign_tri_table<10>(std::make_integer_sequence<int, 8>{}),
    lds_realign_tri_table<11>(std::make_integer_sequence<int, 8>{})};
#if CALLFS_RS_AB_INSTANCES
template <int ORD, int... Rs>
constexpr auto lds_realign64_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, LdsRealign64Policy<Rs + 1, ORD>>...};
}
// [consecutive, X8, X32][R - 1] (A/B build)
const std::array<std::array<VecFn, 8>, 3> kLdsRealign64 = {
    lds_realign64_table<0>(std::make_integer_sequence<int, 8>{}),
    lds_realign64_table<10>(std::make_integer_sequence<int, 8>{}),
    lds_realign64_table<11>(std::make_integer_sequence<int, 8>{})};
#endif
template <int ORD, int... Rs>
constexpr auto lds_realign_out_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, LdsRealignOutPolicyFor<Rs + 1, ORD>>...};
}
// [consecutive, X8, X32][R - 1]
const std::array<std::array<VecFn, 8>, 3> kLdsRealignOut = {
    lds_realign_out_table<0>(std::make_integer_sequence<int, 8>{}),
    lds_realign_out_table<10>(std::make_integer_sequence<int, 8>{}),
    lds_realign_out_table<11>(std::make_integer_sequence<int, 8>{})};
template <class P, int... Rs>
constexpr auto lds_wide_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 9, P>...};
}
const auto kLdsWideQ8 = lds_wide_table<LdsWideQ8Policy>(std::make_integer_sequence<int, 8>{});
const auto kByte = byte_table(std::make_integer_sequence<int, kMaxRowsPerLaunch>{});

// Row groups of 9..16 with more than 64 KiB of tables (k > 128) need the dynamic-LDS
// opt-in, which hipFuncSetAttribute sets for the current device only: one flag per
// (device, R), key R - 9 (dispatch.hpp DeviceOnce). Both tile-order instances of an R
// opt in together.
DeviceOnce g_wide_lds;

void wide_lds_opt_in(int R) {
  for (VecFn f : {kLds[R - 1], kLdsWideQ8[R - 9]})
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(f),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10);
}

}  // namespace

namespace {
using SmallFn = void (*)(SmallArgs);
template <int... Rs>
constexpr auto small_table(std::integer_sequence<int, Rs...>) {
  return std::array<SmallFn, sizeof...(Rs)>{&dev::rs_apply_small<Rs + 1>...};
}
const auto kSmall = small_table(std::make_integer_sequence<int, kMaxRowsPerLaunch>{});
}  // namespace

hipError_t launch_small(const SmallArgs& a, hipStream_t stream) {
  if (a.R < 1 || a.R > kMaxRowsPerLaunch || a.K < 1 || a.K > kMaxK || a.batch < 1 ||
      a.batch > 65535 || a.nvec == 0 || !a.base || !a.tabs || !a.idx || !a.status)
    return hipErrorInvalidValue;
  const unsigned gx = (a.nvec + 255u) / 256u;
  hipLaunchKernelGGL(kSmall[a.R - 1], dim3(gx, static_cast<unsigned>(a.batch)), dim3(256), 0,
                     stream, a);
  return hipGetLastError();
}


void set_slice_tiles_for_tuning(long long tiles) {
  g_slice_tiles_override.store(tiles, std::memory_order_relaxed);
}

namespace {

TileOrder lds_rule(const ApplyArgs& a) {
  const int forced = tile_order_override();
  if (forced >= 0) return static_cast<TileOrder>(forced);
  const uint32_t rows = a.R >= 32 ? ~0u : (1u << a.R) - 1;
  return lds_tile_order(a.S, (a.nvec + LdsPolicy::BS - 1) / LdsPolicy::BS, a.addr_tz, a.K + a.R,
                        a.stripe_stride, (a.verify_mask & rows) != 0,
                        (a.verify_mask & rows) == rows, a.R);
}

TileOrder wide_rule(const ApplyArgs& a) {
  return wide_tile_order((a.nvec + LdsWidePolicy::BS - 1) / LdsWidePolicy::BS);
}

TileOrder vec_rule(const ApplyArgs& a) {
  return vec_tile_order(a.S, (a.nvec + ProdPolicy::BS - 1) / ProdPolicy::BS, a.addr_tz);
}

// CALLFS_RS_REALIGN=0 sends misaligned launches to the plain kernel (unaligned 16-B
// loads and stores; A/B)
bool realign_out_enabled() {
  static const bool on = [] {
    const char* e = kAbInstances ? std::getenv("CALLFS_RS_REALIGN") : nullptr;
    return !(e && *e == '0');
  }();
  return on;
}

bool takes_lds(const ApplyArgs& a) { return a.R >= kLdsMinRows || a.K >= kLdsMinK; }
// Misaligned R <= 8 launches can take the realigning kernel; by default they do when some
// shard sits at an odd byte offset. Shards misaligned only by even offsets (even S) ran
// the plain kernel 2.3-4.3 points faster (RS(12,4), S = 5,592,406, two boxes), odd ones
// mostly slower (RS(6,3) -6, RS(5,3) -4, RS(10,8) -1.7; RS(10,4) and RS(4,2) within
// +-1.4 depending on the box). rs_plan_tune times both.
bool can_realign(const ApplyArgs& a) {
  return a.R <= 8 && (a.in_misalign || a.out_misalign) && realign_out_enabled();
}
// 6-bit triple lookups (Policy::WIX): R <= 4, 3 <= K <= 96 (tables within the 64 KiB of
// dynamic LDS a launch gets without the opt-in), aligned shards
bool can_wix(const ApplyArgs& a) {
  return a.R <= 4 && a.K >= 3 && a.K <= 96 && !(a.in_misalign | a.out_misalign);
}
// CALLFS_RS_WIX=0 keeps every launch on the ring-of-three nibble kernel (A/B build only)
bool wix_enabled() {
  static const bool on = [] {
    const char* e = kAbInstances ? std::getenv("CALLFS_RS_WIX") : nullptr;
    return !(e && *e == '0');
  }();
  return on;
}
// Since the triple-load form (below) measured equal or faster than WIX everywhere, the
// rule no longer takes WIX: its instances remain for rs_plan_set_orders (A/B).
// profiles/r03/wix/: WIX in the nibble rule's order vs the nibble kernel's best order, 1 MiB shards: RS(4,2) 72.3 -> 79.0, RS(4,4) 75.0 -> 81.5, RS(5,3) 74.5 -> 79.9,
// RS(8,4) 76.5 -> 80.1; RS(10,4) equal, RS(16,4) / RS(20,4) / RS(32,4) -1.2 ... -1.5.

// Triple loads (Policy::WIX 2): tile_order.hpp tri_rule. profiles/r03/wix/ab4_tri_verify.jsonl, % of 8 TB/s, nibble (best order) -> triples in
// the rule's order: RS(4,2) 71.8 -> 80.6, RS(5,3) 74.6 -> 80.3, RS(8,4) 76.3 -> 80.2,
// RS(10,4) 75.8 -> 76.6, RS(6,6) 74.6 -> 75.7, RS(8,8) 75.4 -> 76.3, RS(10,8) 74.1 -> 77.4;
// read-only (download Verify): RS(4,2) 82.5 -> 88.4, RS(10,4) 83.8 -> 86.0 (X32). Second
// box (profiles/r03/tri1/ab.jsonl), the rule itself: RS(4,2) 72.5 -> 80.6, 1 MiB objects
// 71.9 -> 77.9, RS(8,8) 75.6 -> 77.6, RS(10,8) 74.4 -> 78.2, RS(4,2) read-only 82.8 ->
// 88.0, RS(6,3) 1 MiB objects 71.4 -> 73.2, RS(10,4) 76.5 -> 75.9-76.1 (the tuner keeps
// whichever is faster), RS(12,4) 77.2 -> 80.3 (G2).
// The rule's triple-form order (tile_order.hpp tri_rule_order: round 4 adds X32 for K <= 4,
// X32 / Q16 for K 5..6 and Q16 on 16-32 MiB power-of-two pitches), or -1. With
// CALLFS_RS_TILE_ORDER set, the triple form follows the forced order with round 3's bounds.
// Misaligned inputs with 16-B-aligned outputs (upstream Split of an io.ReadAll body: the
// data shards inside the body, the parity in AllocAligned buffers): the triple form with
// unaligned 16-B loads, X32 up to 256 tiles per stripe and X8 above, not the realigning
// kernel. profiles/r04/utri1/readall_enc.jsonl (% of 8 TB/s,
// realigning kernel (rule) -> triples in X32 / X8): RS(10,4) 104,858 B 69.5 -> 76.7 (G2
// 77.5), RS(12,4) 87,382 B 69.0 -> 75.7, RS(5,3) 209,716 B 71.0 -> 78.3, RS(6,3) 174,763 B
// 70.6 -> 74.4, RS(10,8) 1,048,577 B 68.8 -> 70.9, RS(10,4) 6,710,887 B 71.2 -> 72.8 (X8),
// RS(12,4) 5,592,406 B 71.8 -> 74.2 (X8), RS(4,2) 1,048,577 B 71.0 -> 71.9. With unaligned
// stores as well (the contiguous Split layout) the same forms lost 1-6 points
// (split_enc.jsonl), so misaligned outputs keep the realigning kernel.
// (Measured for K <= 12 only; wider launches above 256 KiB shards keep the realigning
// kernel, as the aligned rule keeps K > 12 off the triples there.)
int tri_unaligned_order(const ApplyArgs& a, uint64_t tps) {
  if (a.R > 8 || a.K < 4 || !a.in_misalign || a.out_misalign || tile_order_override() >= 0)
    return -1;
  // More than 12 inputs above 256 KiB: the realigning ring, except for R <= 4 launches that
  // also compare rows (one-shard decodes), where the unaligned triples lead it (round 5, 40
  // seeded object sizes in the readall layout, profiles/r05/tiles/random_readall_*: RS(16,4)
  // 2.3 MB decode {1} 70.9 -> 73.6; its encodes split, 3.9 MB 73.4 -> 69.9)
  const uint32_t rows = (1u << a.R) - 1;
  const bool verify = (a.verify_mask & rows) != 0;
  if (a.K > 12 && tps > 32 && !(a.R <= 4 && verify)) return -1;
  // R 5..8 launches that compare rows take a ring, as the aligned rule gives them the ring
  // (the plain one on unaligned loads, takes_realign): the rotating unaligned triples ran
  // 3-7 points behind the ring forms (RS(8,8) /
  // RS(10,8) {1}, 122 KB - 24 MB: 62-64 vs 65.7-71.0; after: those 8 cells 63.7 -> 66.4
  // on average, random_readall_dec1_after.jsonl)
  if (a.R > 4 && verify) return -1;
  // round 5 (tools/jobs.sh readall_rule_sweep, profiles/r05/readall_rule/): Q8 from 1 to 2 MiB,
  // X32 -> Q8: RS(10,4) 1.68 MB 74.9 -> 76.6, RS(12,4) 1.4 MB 75.1 -> 76.3, RS(8,8) 2 MiB
  // 75.0 -> 76.3, RS(10,8) 1.68 MB 70.4 -> 71.7
  if (tps > 128 && tps <= 256) return static_cast<int>(TileOrder::kSeg8);
  return static_cast<int>(tps <= 256 ? TileOrder::kXcd32 : TileOrder::kXcd8);
}

int tri_rule_of(const ApplyArgs& a) {
  if (!wix_enabled() || !takes_lds(a)) return -1;
  const uint32_t rows = (1u << a.R) - 1;
  const uint64_t tps = (a.nvec + LdsPolicy::BS - 1) / LdsPolicy::BS;
  if (a.in_misalign && !a.out_misalign) return tri_unaligned_order(a, tps);
  const bool mis = (a.in_misalign | a.out_misalign) != 0, verify = (a.verify_mask & rows) != 0,
             read_only = (a.verify_mask & rows) == rows;
  if (tile_order_override() >= 0)
    return tri_rule(a.K, a.R, mis, verify, read_only, tps) &&
                   (tps <= 256 || (tps <= 512 && a.K <= 6))
               ? static_cast<int>(tri_order(lds_rule(a)))
               : -1;
  return tri_rule_order(a.K, a.R, mis, verify, read_only, tps, a.addr_tz, a.S, lds_rule(a));
}
bool takes_tri(const ApplyArgs& a) { return tri_rule_of(a) >= 0; }
bool tri_tunable_launch(const ApplyArgs& a) {
  const uint32_t rows = (1u << a.R) - 1;
  return wix_enabled() && tri_tunable(a.K, a.R, (a.in_misalign | a.out_misalign) != 0,
                                      (a.verify_mask & rows) != 0, (a.verify_mask & rows) == rows);
}
// kLdsTri's first index; G8 has no triple instance (tri_order maps it to X32)
int tri_index(TileOrder o) {
  switch (o) {
    case TileOrder::kGroup2: return 1;
    case TileOrder::kXcd32: return 2;
    case TileOrder::kSeg8: return 3;
    case TileOrder::kSeg16: return 4;
    case TileOrder::kXcd8: return 5;
    default: return 0;
  }
}
bool takes_realign(const ApplyArgs& a) {
  // (round 5: R 5..8 launches with misaligned inputs, aligned outputs and compared rows run
  // the plain ring on unaligned loads 3.2-4.5 points ahead of the realigning form, RS(8,8)
  // 23.8 MB {1} readall 67.8 -> 72.3, RS(10,8) 161,009 B 62.1 -> 66.6;
  // profiles/r05/tiles/random_readall_dec1_after.jsonl)
  const uint32_t rows = (1u << a.R) - 1;
  if (a.R > 4 && (a.verify_mask & rows) != 0 && a.in_misalign && !a.out_misalign) return false;
  return can_realign(a) && ((a.in_misalign | a.out_misalign) & 1u) && !takes_tri(a);
}
// the 64-vector realigning form: misaligned inputs, every output 16-B aligned
bool can_realign64(const ApplyArgs& a) {
  return kAbInstances && can_realign(a) && a.in_misalign && !a.out_misalign;
}

// The rule's realigning launches with triple loads (tile_order.hpp realign_tri_rule);
// CALLFS_RS_WIX=0 keeps them on the ring of three
bool takes_realign_tri(const ApplyArgs& a) {
  const uint32_t rows = (1u << a.R) - 1;
  return wix_enabled() && realign_tri_rule(a.K, a.R, (a.verify_mask & rows) != 0,
                                           (a.verify_mask & rows) == rows);
}

// The realigning kernel's tile order (index into kLdsRealignOut): a tuned realign code
// (kOrderRealign + TileOrder) names it; otherwise CALLFS_RS_TILE_ORDER=consecutive / x8
// / x32, else X32 (tools/order_ab.py, Split
// layout, % of 8 TB/s, two runs, consecutive -> X32: RS(10,4) 64 MiB objects 68.3 /
// 68.6 -> 69.5 / 69.9, RS(4,2) 1,048,577 B 67.1 / 66.8 -> 68.6 / 68.3, RS(12,4) S =
// 5,592,406 65.5 / 65.9 -> 66.9 / 66.9, the other five shapes -0.2 ... +0.9).
int realign_order_index(int order) {
  const int o = order >= kOrderRealign ? order - kOrderRealign : tile_order_override();
  if (o == static_cast<int>(TileOrder::kConsecutive)) return 0;
  return o == static_cast<int>(TileOrder::kXcd8) ? 1 : 2;
}

}  // namespace

namespace {
std::vector<int> nibble_candidates(const ApplyArgs& a0, bool every_instance);
bool can_bitslice(const ApplyArgs& a);

// The bit-sliced kernel's orders: launch groups of kBitsliceMinRows or more
// rows whose plan carries a kernel handle (ApplyArgs::bs), unless CALLFS_RS_BITSLICE=0.
bool can_bitslice(const ApplyArgs& a) {
  return a.bs && a.R >= kBitsliceMinRows && a.K >= 1 && a.S >= 16 && bs::mode() != bs::Mode::kOff;
}
// The rule's bit-sliced launches and their order (tile_order.hpp bitslice_rule)
bool takes_bitslice(const ApplyArgs& a) {
  const uint32_t rows = a.R >= 32 ? ~0u : (1u << a.R) - 1;
  return can_bitslice(a) &&
         bitslice_rule(a.K, a.R, (a.S / 16 + bs::kTileVecs - 1) / bs::kTileVecs, a.in_misalign != 0,
                       a.out_misalign != 0, (a.verify_mask & rows) != 0,
                       (a.verify_mask & rows) == rows);
}
TileOrder bitslice_rule_order(const ApplyArgs& a) {
  const uint32_t rows = a.R >= 32 ? ~0u : (1u << a.R) - 1;
  return bitslice_tile_order((a.S / 16 + bs::kTileVecs - 1) / bs::kTileVecs,
                             (a.in_misalign | a.out_misalign) != 0, (a.verify_mask & rows) != 0,
                             (a.verify_mask & rows) == rows);
}
// bs::Args::order of a TileOrder (-1: no generated form)
int bitslice_order(TileOrder o) {
  switch (o) {
    case TileOrder::kConsecutive: return 0;
    case TileOrder::kSeg8: return 1;
    case TileOrder::kXcd32: return 2;
    case TileOrder::kGroup2: return 3;
    case TileOrder::kXcd8: return 4;
    case TileOrder::kGroup8: return 5;
    case TileOrder::kSeg16: return 6;
  }
  return -1;  // not a TileOrder (a code outside 256 + [0, kTileOrders))
}
}  // namespace

bool bitslice_wanted(const ApplyArgs& a) { return takes_bitslice(a); }

namespace {
TuneKey key_of(const ApplyArgs& a) {
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) device = 0;
  const uint32_t rows = a.R >= 32 ? ~0u : (1u << a.R) - 1;
  return tune_key(device, a.K, a.R, (a.S / 16 + LdsPolicy::BS - 1) / LdsPolicy::BS, a.addr_tz,
                  (a.verify_mask & rows) != 0, (a.verify_mask & rows) == rows, a.in_misalign != 0,
                  a.out_misalign != 0);
}
}  // namespace

int tuned_order(const ApplyArgs& a) {
  TuneTable& t = tune_table();
  if (t.empty()) return -1;
  const int o = t.lookup(key_of(a));
  if (o < 0) return -1;
  const std::vector<int> c = order_candidates(a, /*every_instance=*/true);
  if (std::find(c.begin(), c.end(), o) == c.end()) return -1;
  if (o >= kOrderBitslice) {  // host calls never wait for a compile: the rule until it is ready
    auto* k = static_cast<bs::Kernel*>(const_cast<void*>(a.bs));
    if (k->state() != bs::Kernel::State::kReady) {
      k->compile_async();
      return -1;
    }
  }
  return o;
}

void record_tuned(const ApplyArgs& a, int order) { tune_table().record(key_of(a), order); }

int launch_form(const ApplyArgs& a, int order) {
  if (order < 0) order = tuned_order(a);
  if (order >= 0) return order;
  if (takes_bitslice(a) && static_cast<const bs::Kernel*>(a.bs)->state() == bs::Kernel::State::kReady)
    return kOrderBitslice + static_cast<int>(bitslice_rule_order(a));
  const std::vector<int> c = nibble_candidates(a, false);
  return c.empty() ? -1 : c[0];
}

std::vector<int> order_candidates(const ApplyArgs& a, bool every_instance) {
  std::vector<int> c = nibble_candidates(a, every_instance);
  // the rule's kernel first (rs_plan_tune's bar favours cand[0])
  if (!c.empty() && takes_bitslice(a)) c.insert(c.begin(), kOrderBitslice + static_cast<int>(bitslice_rule_order(a)));
  if (!c.empty() && can_bitslice(a)) {
    const uint64_t tps = (a.S / 16 + bs::kTileVecs - 1) / bs::kTileVecs;
    auto add = [&c](TileOrder o) {
      const int v = kOrderBitslice + static_cast<int>(o);
      if (std::find(c.begin(), c.end(), v) == c.end()) c.push_back(v);
    };
    add(bitslice_rule_order(a));
    add(TileOrder::kConsecutive);
    add(TileOrder::kGroup2);
    if (tps <= 32 || every_instance) add(TileOrder::kGroup8);
    if (tps >= 64 || every_instance) add(TileOrder::kSeg8);
    if (tps >= 256 || every_instance) add(TileOrder::kSeg16);
    if (every_instance) {
      add(TileOrder::kXcd8);
      add(TileOrder::kXcd32);
    }
  }
  return c;
}

namespace {
std::vector<int> nibble_candidates(const ApplyArgs& a0, bool every_instance) {
  ApplyArgs a = a0;
  a.nvec = a.S / 16;
  std::vector<int> c;
  auto add = [&c](TileOrder o) {
    const int v = static_cast<int>(o);
    if (std::find(c.begin(), c.end(), v) == c.end()) c.push_back(v);
  };
  if (a.nvec == 0 || a.R < 1 || a.R > kMaxRowsPerLaunch || a.K < 1) return c;
  const uint64_t tps = (a.nvec + LdsPolicy::BS - 1) / LdsPolicy::BS;
  if (takes_lds(a)) {
    if (a.R > 8) {
      add(wide_rule(a));
      add(TileOrder::kConsecutive);
      add(TileOrder::kSeg8);
      return c;
    }
    const auto realign_in = [](TileOrder o) {
      return static_cast<TileOrder>(kOrderRealign + static_cast<int>(o));
    };
    const auto rtri_in = [](TileOrder o) {
      return static_cast<TileOrder>(kOrderRealignTri + static_cast<int>(o));
    };
    const auto r64_in = [](TileOrder o) {
      return static_cast<TileOrder>(kOrderRealign64 + static_cast<int>(o));
    };
    const auto wix_in = [](TileOrder o) {
      return static_cast<TileOrder>(kOrderWix + static_cast<int>(o));
    };
    // the rule's kernel first (rs_plan_tune's bar favours cand[0]): the realign order the
    // rule itself runs (realign_order_index(-1) follows CALLFS_RS_TILE_ORDER)
    static constexpr TileOrder kRealignRule[3] = {TileOrder::kConsecutive, TileOrder::kXcd8,
                                                  TileOrder::kXcd32};
    if (takes_realign(a)) add(realign_in(kRealignRule[realign_order_index(-1)]));
    const auto tri_in = [](TileOrder o) {
      return static_cast<TileOrder>(kOrderTri + static_cast<int>(o));
    };
    if (takes_tri(a)) add(tri_in(static_cast<TileOrder>(tri_rule_of(a))));  // the rule's kernel first
    add(lds_rule(a));
    if (can_realign(a)) {
      add(realign_in(TileOrder::kXcd32));
      add(realign_in(TileOrder::kConsecutive));
      if (every_instance) add(realign_in(TileOrder::kXcd8));
      if (every_instance && can_realign64(a)) {  // (A/B build)
        add(r64_in(TileOrder::kXcd32));
        add(r64_in(TileOrder::kConsecutive));
        add(r64_in(TileOrder::kXcd8));
      }
      if (a.K >= 3) {  // the realigning kernel with triple loads
        add(rtri_in(TileOrder::kXcd32));
        add(rtri_in(TileOrder::kConsecutive));
        if (every_instance) add(rtri_in(TileOrder::kXcd8));
      }
    }
    add(TileOrder::kConsecutive);
    add(TileOrder::kGroup2);
    if (tps <= 32 || every_instance) add(TileOrder::kGroup8);
    // Q8 from 64 tiles per stripe (8 segments of >= 8 tiles): at 1 MiB shards it ran within
    // a point of the best order and ahead of the rule's on some boxes (RS(16,4) 77.7 vs 76.8,
    // profiles/r04/tri_sweep1); Q16 above 8 MiB as before
    if (tps >= 64) add(TileOrder::kSeg8);
    if (tps > 1024 || (every_instance && tps >= 64)) add(TileOrder::kSeg16);
    if (every_instance) {  // on aligned shards never faster than the rule's order, which
                           // is X32 itself for read-only launches
      add(TileOrder::kXcd8);
      add(TileOrder::kXcd32);
    }
    // (on misaligned shards the triple forms are the plain kernel's unaligned 16-B
    // accesses: A/B instances for rs_plan_set_orders)
    // (misaligned launches: the tuner also times the triple forms' unaligned accesses,
    // which the rule takes for aligned outputs only)
    if ((every_instance && a.K >= 3) || tri_tunable_launch(a) ||
        (a.in_misalign && a.R <= 8 && a.K >= 4 && wix_enabled())) {
      add(tri_in(TileOrder::kConsecutive));
      add(tri_in(TileOrder::kGroup2));
      add(tri_in(TileOrder::kXcd32));
      // tri-Q8 from 64 tiles per stripe (RS(10,4) 1 MiB 77.5 / 77.3 against 76.3 / 76.2 for
      // tri-G2, profiles/r04/tri_sweep1, tri_sweep2); tri-Q16 above 8 MiB
      if (tps >= 64) add(tri_in(TileOrder::kSeg8));
      if (tps > 1024 || (every_instance && tps >= 64)) add(tri_in(TileOrder::kSeg16));
      if (tps > 1024 || every_instance) add(tri_in(TileOrder::kXcd8));
    }
    if (every_instance && can_tridb_g(a)) {  // G4 / G8 double-buffered triples: A/B build only
      add(static_cast<TileOrder>(kOrderTriDbG));
      add(static_cast<TileOrder>(kOrderTriDbG + 1));
    }
    if (every_instance && can_dma(a)) {  // the LDS-DMA ring: A/B build only
      for (TileOrder o : {TileOrder::kConsecutive, TileOrder::kGroup2, TileOrder::kSeg8, TileOrder::kXcd32})
        add(static_cast<TileOrder>(kOrderDma + static_cast<int>(o)));
    }
    if (kAbInstances && every_instance && can_wix(a)) {  // WIX: A/B build only
      const int n0 = static_cast<int>(c.size());
      for (int i = 0; i < n0; ++i)
        if (c[i] >= 0 && c[i] < kTileOrders) add(wix_in(static_cast<TileOrder>(c[i])));
    }
    return c;
  }
  add(vec_rule(a));
  add(TileOrder::kConsecutive);
  add(TileOrder::kGroup2);
  if (tps > 1024) add(TileOrder::kSeg16);
  return c;
}
}  // namespace

namespace {
// One launch of the group's bit-sliced kernel in tile order `ord` (plus the byte kernel for
// the S % 16 tail). Returns false, launching nothing, when the kernel is not compiled yet and
// `wait` is false (the caller then runs the nibble-table kernel); with `wait` a kernel that
// cannot be compiled or loaded returns true with *err set.
bool launch_bitslice(ApplyArgs a, hipStream_t stream, TileOrder ord, LaunchEvents ev, bool wait,
                     hipError_t* err) {
  *err = hipSuccess;
  const int bo = bitslice_order(ord);
  if (!can_bitslice(a) || bo < 0) {
    if (wait) *err = hipErrorInvalidValue;
    return wait;
  }
  int device = -1;
  if (hipGetDevice(&device) != hipSuccess) {
    *err = hipErrorInvalidDevice;
    return true;
  }
  auto* k = static_cast<bs::Kernel*>(const_cast<void*>(a.bs));
  const hipFunction_t fn = k->function(device, wait);
  if (!fn) {
    if (wait) *err = hipErrorNoBinaryForGpu;
    return wait;
  }
  bs::Args b{};
  b.in_tab = a.in_tab;
  b.out_tab = a.out_tab;
  b.status = a.status;
  b.nvec = a.S / 16;
  b.tps = static_cast<uint32_t>((b.nvec + k->tile_vecs() - 1) / k->tile_vecs());
  b.ntiles = b.tps * static_cast<uint32_t>(a.batch);
  b.verify_mask = a.verify_mask;
  b.status_stride = a.status_stride;
  b.order = bo;
  const bool tail_after = b.nvec * 16 < a.S;
  launch_sliced(b.ntiles, a.K + a.R, a, [&](uint32_t blocks, bool first, bool last) {
    b.t_base = a.t_base;
    const hipError_t e = bs::launch(fn, b, blocks, k->block_threads(), stream,
                                    first ? ev.start : nullptr, last && !tail_after ? ev.stop : nullptr);
    if (e != hipSuccess && *err == hipSuccess) *err = e;
  });
  if (*err != hipSuccess) return true;
  if (tail_after) {
    const uint64_t tail0 = b.nvec * 16;
    const unsigned gy = static_cast<unsigned>(std::min(a.batch, 65535));
    const uint64_t gx = (a.S - tail0 + kBlock - 1) / kBlock;
    dispatch(kByte[a.R - 1], dim3(static_cast<unsigned>(gx), gy), dim3(kBlock), 0, stream, ev,
             /*first=*/false, /*last=*/true, a, tail0);
    *err = hipGetLastError();
  }
  return true;
}
}  // namespace

hipError_t launch_apply(ApplyArgs a, hipStream_t stream, bool bytes_only, int order,
                        LaunchEvents ev) {
  if (a.R < 1 || a.R > kMaxRowsPerLaunch || a.K < 1 || a.K > kMaxK || a.batch < 1)
    return hipErrorInvalidValue;
  if (a.S == 0) return hipSuccess;
  // the bit-sliced kernel: a pinned kOrderBitslice order waits for its compile; the rule's
  // choice runs it once compiled and the nibble-table kernel until then
  if (!bytes_only && (order >= kOrderBitslice || (order < 0 && takes_bitslice(a)))) {
    const bool pinned = order >= kOrderBitslice;
    if (pinned && order >= kOrderBitslice + kTileOrders) return hipErrorInvalidValue;
    const TileOrder bo = pinned ? static_cast<TileOrder>(order - kOrderBitslice) : bitslice_rule_order(a);
    hipError_t e = hipSuccess;
    if (launch_bitslice(a, stream, bo, ev, pinned || bs::mode() == bs::Mode::kSync, &e)) return e;
    order = -1;
  }
  // (A/B) the double-buffered triples in G4 / G8: the nibble instances' G8 order underneath
  int tdg = -1;
  if (order >= kOrderTriDbG) {
    tdg = can_tridb_g(a) ? order - kOrderTriDbG : -1;
    order = tdg >= 0 ? static_cast<int>(TileOrder::kGroup8) : -1;
  }
  const bool dma = order >= kOrderDma && can_dma(a);
  if (order >= kOrderDma) order = dma ? order - kOrderDma : -1;
  // realigning kernel with triple loads: kOrderRealignTri + its order -> kOrderRealign + it
  const bool r64 = order >= kOrderRealign64 && can_realign64(a);
  if (order >= kOrderRealign64) order = r64 ? order - kOrderRealign64 + kOrderRealign : -1;
  const bool rtri = order >= kOrderRealignTri && a.K >= 3 && can_realign(a);
  if (order >= kOrderRealignTri) order = rtri ? order - kOrderRealignTri + kOrderRealign : -1;
  bool tri = order >= kOrderTri && a.R <= 8 && a.K >= 3;
  if (order >= kOrderTri) order = tri ? order - kOrderTri : -1;
  const bool wix = kAbInstances && order >= kOrderWix && can_wix(a);
  if (order >= kOrderWix) order -= kOrderWix;
  uint64_t tail0 = 0;
  a.tail_in_vec = 0;
  if (!bytes_only) {
    a.nvec = a.S / 16;
    tail0 = a.nvec * 16;
    if (a.nvec) {
      if (takes_lds(a)) {
        // the LDS kernel's first tile per stripe computes the S % 16 tail itself: an odd-S
        // launch (Split layout) is one kernel, not two back to back
        a.tail_in_vec = tail0 < a.S ? tail_code(a.nvec, LdsPolicy::TILE_VECS, LdsPolicy::BS) : 0u;
        if (a.tail_in_vec) tail0 = a.S;
        if (!a.ltabs) return hipErrorInvalidValue;
        size_t lds = dev::lds_bytes(a.K, a.R);
        VecFn fn = kLds[a.R - 1];
        if (a.R <= 8) {  // (8-byte entries: at most 64 KiB of tables, no opt-in needed)
          const TileOrder ord =
              order >= 0 && order < kOrderRealign ? static_cast<TileOrder>(order) : lds_rule(a);
          switch (ord) {
            case TileOrder::kGroup8: fn = kLdsG8[a.R - 1]; break;
            case TileOrder::kGroup2: fn = kLdsG2[a.R - 1]; break;
            case TileOrder::kSeg8: fn = kLdsQ8[a.R - 1]; break;
            case TileOrder::kSeg16: fn = kLdsQ16[a.R - 1]; break;
            case TileOrder::kXcd8: fn = kLdsX8[a.R - 1]; break;
            case TileOrder::kXcd32: fn = kLdsX32[a.R - 1]; break;
            case TileOrder::kConsecutive: break;
          }
          const uint32_t rows = (1u << a.R) - 1;
          const int oi = static_cast<int>(ord);
          if (a.R <= 4 && (a.verify_mask & rows) && oi >= 0 && oi < kTileOrders)
            fn = kLdsVerify[oi][a.R - 1];
#if CALLFS_RS_AB_INSTANCES
          if (wix && oi >= 0 && oi < kTileOrders) {  // (at most 56 KiB of tables at K = 96)
            fn = kLdsWix[oi][a.R - 1];
            lds = dev::lds_bytes_wix(a.K);
          }
#else
          (void)wix;
#endif
          if (!tri && order < 0 && takes_tri(a)) tri = true;  // the rule: ord is the nibble rule's
          if (tri) {
            const int ti = tri_index(order < 0 ? static_cast<TileOrder>(tri_rule_of(a)) : ord);
            const bool mixed = (a.verify_mask & rows) && (a.verify_mask & rows) != rows;
            const bool db = a.K >= kTriDbMinK && tridb_enabled();
            if (a.R <= 4 && mixed)  // written + Verify rows: early compares
              fn = db ? kLdsTriDbVerify[ti][a.R - 1] : kLdsTriVerify[ti == 5 ? 2 : ti][a.R - 1];
            else if (a.R <= 4 && db)
              fn = kLdsTriDb[ti][a.R - 1];
            else
              fn = kLdsTri[ti][a.R - 1];
          }
#if CALLFS_RS_AB_INSTANCES
          if (dma) {
            fn = kLdsDma[dma_index(ord)][a.R - 1];
            lds = dev::lds_bytes_dma(a.K, a.R, kDmaDepth);
          }
          if (tdg >= 0) fn = kLdsTriDbG[tdg][a.R - 1];
#else
          (void)tdg;
#endif
        } else if ((order >= 0 ? static_cast<TileOrder>(order) : wide_rule(a)) == TileOrder::kSeg8) {
          fn = kLdsWideQ8[a.R - 9];
        }
        if (lds > (64u << 10)) {  // wide groups with many shards (only R > 8 gets here):
          // the opt-in is a per-device attribute: once per (device, R), before the first
          // such launch on each device (a once-flag per kernel left devices 1..7 without it)
          int device = -1;
          if (hipGetDevice(&device) != hipSuccess) return hipErrorInvalidDevice;
          g_wide_lds.run(device, a.R - 9, [&a] { wide_lds_opt_in(a.R); });
        }
        static_assert(LdsPolicy::BS == LdsWidePolicy::BS && LdsPolicy::U == LdsWidePolicy::U &&
                          LdsG8Policy::BS == LdsPolicy::BS && LdsG2Policy::BS == LdsPolicy::BS &&
                          LdsQ8Policy::BS == LdsPolicy::BS && LdsQ16Policy::BS == LdsPolicy::BS &&
                          LdsX8Policy::BS == LdsPolicy::BS && LdsX32Policy::BS == LdsPolicy::BS &&
                          LdsWideQ8Policy::BS == LdsPolicy::BS &&
                          LdsVerifyPolicy<0>::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsRealignOutPolicy<0>::BS == LdsPolicy::BS &&
                          LdsRealignOut8Policy<0>::TILE_VECS == LdsRealignOutPolicy<0>::TILE_VECS &&
                          LdsRealignOutPolicy<10>::TILE_VECS == LdsRealignOutPolicy<0>::TILE_VECS &&
                          LdsTriPolicy<1, 0>::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsTriPolicy<8, 10>::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsTriPolicy<8, 10>::BS == LdsPolicy::BS &&
                          LdsTriDbPolicy<0>::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsTriDbPolicy<0>::BS == LdsPolicy::BS &&
                          LdsTriVerifyPolicy<0>::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsTriVerifyPolicy<0>::BS == LdsPolicy::BS &&
                          LdsTriDbVerifyPolicy<0>::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsTriDbVerifyPolicy<0>::BS == LdsPolicy::BS &&
                          LdsVerifyPolicy<0>::BS == LdsPolicy::BS &&
                          LdsWixPolicy<0>::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsWidePolicy::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsWideQ8Policy::TILE_VECS == LdsPolicy::TILE_VECS &&
                          LdsDmaPolicy<8, 0>::TILE_VECS == LdsPolicy::TILE_VECS,
                      "one grid shape and tail placement (tail_code) for every LDS policy");
        unsigned gx = dev::vec_grid<LdsPolicy>(a.nvec, a.batch);
        // misaligned shards: the realigning form, unless a tuned order names a plain kernel
        if (r64) {  // 512-vector tiles and the ragged tail as the plain kernel's
          static_assert(LdsRealign64Policy<1, 0>::TILE_VECS == LdsPolicy::TILE_VECS &&
                            LdsRealign64Policy<8, 0>::TILE_VECS == LdsPolicy::TILE_VECS,
                        "REALIGN 5 tiles as the plain kernel's");
#if CALLFS_RS_AB_INSTANCES
          fn = kLdsRealign64[realign_order_index(order)][a.R - 1];
#endif
        } else if (can_realign(a) && (order >= kOrderRealign || (order < 0 && takes_realign(a)))) {
          const bool rt = rtri || (order < 0 && takes_realign_tri(a));
          fn = (rt ? kLdsRealignTri : kLdsRealignOut)[realign_order_index(order)][a.R - 1];
#if CALLFS_RS_AB_INSTANCES
          if (rt && a.R <= 4 && a.K >= kTriDbMinK && tridb_enabled())
            fn = kLdsRealignTriDb[realign_order_index(order)][a.R - 1];
#endif
          gx = dev::vec_grid<LdsRealignOutPolicy<0>>(a.nvec, a.batch);
          a.tail_in_vec = 1;  // its first tile writes every edge byte, the tail included
          tail0 = a.S;
        }
        const bool tail_after = tail0 < a.S;  // a byte-kernel launch follows: it ends the launch
        launch_sliced(gx, a.K + a.R, a, [&](uint32_t blocks, bool first, bool last) {
          dispatch(fn, dim3(blocks), dim3(LdsPolicy::BS), lds, stream, ev, first,
                   last && !tail_after, a);
        });
      } else {
        a.tail_in_vec = tail0 < a.S ? tail_code(a.nvec, ProdPolicy::TILE_VECS, ProdPolicy::BS) : 0u;
        if (a.tail_in_vec) tail0 = a.S;
        VecFn fn = kVec[a.R - 1];  // R <= 4 here (R >= kLdsMinRows takes the LDS kernel)
        switch (order >= 0 ? static_cast<TileOrder>(order) : vec_rule(a)) {
          case TileOrder::kGroup2: fn = kVecG2[a.R - 1]; break;
          case TileOrder::kSeg16: fn = kVecQ16[a.R - 1]; break;
          default: break;
        }
        static_assert(ProdG2Policy::BS == ProdPolicy::BS && ProdQ16Policy::BS == ProdPolicy::BS &&
                          ProdG2Policy::U == ProdPolicy::U && ProdQ16Policy::U == ProdPolicy::U,
                      "one grid shape for every v_perm policy");
        const unsigned gx = dev::vec_grid<ProdPolicy>(a.nvec, a.batch);
        const bool tail_after = tail0 < a.S;
        launch_sliced(gx, a.K + a.R, a, [&](uint32_t blocks, bool first, bool last) {
          dispatch(fn, dim3(blocks), dim3(ProdPolicy::BS), 0, stream, ev, first,
                   last && !tail_after, a);
        });
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
    dispatch(kByte[a.R - 1], dim3(static_cast<unsigned>(gx), gy), dim3(kBlock), 0, stream, ev,
             /*first=*/a.nvec == 0, /*last=*/true, a, tail0);
    return hipGetLastError();
  }
  return hipSuccess;
}

// ---- no-lookup ceiling (measurement only; rs_plan_launch_ceiling) ----------------------
// Policy::NOMATH turns the LDS kernel into the memory ceiling of its own traffic shape:
// the same loads, stores, grid, block size, tile order and table prologue, with the
// lookups replaced by one XOR per input dword.
// bench.py times it in the same process as the plan it bounds.
namespace {
#if CALLFS_RS_AB_INSTANCES
template <int ORD, int R>
using NomathPolicy = dev::Policy<2, 1, true, true, false, 512, (R > 8 ? 4 : 2), ORD, (R > 8 ? 1 : 0), true>;
template <int ORD, int... Rs>
constexpr auto nomath_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 1, NomathPolicy<ORD, Rs + 1>>...};
}
template <int ORD, int... Rs>
constexpr auto nomath_wide_table(std::integer_sequence<int, Rs...>) {
  return std::array<VecFn, sizeof...(Rs)>{&dev::rs_apply_lds<Rs + 9, NomathPolicy<ORD, Rs + 9>>...};
}
// [TileOrder][R - 1] for R <= 8; wide groups: consecutive and Q8 (the orders they run)
const std::array<std::array<VecFn, 8>, kTileOrders> kNomath = {
    nomath_table<0>(std::make_integer_sequence<int, 8>{}), nomath_table<2>(std::make_integer_sequence<int, 8>{}),
    nomath_table<5>(std::make_integer_sequence<int, 8>{}), nomath_table<6>(std::make_integer_sequence<int, 8>{}),
    nomath_table<8>(std::make_integer_sequence<int, 8>{}), nomath_table<10>(std::make_integer_sequence<int, 8>{}),
    nomath_table<11>(std::make_integer_sequence<int, 8>{})};
const auto kNomathWide = nomath_wide_table<0>(std::make_integer_sequence<int, 8>{});
const auto kNomathWideQ8 = nomath_wide_table<6>(std::make_integer_sequence<int, 8>{});
static_assert(NomathPolicy<0, 4>::TILE_VECS == LdsPolicy::TILE_VECS &&
                  NomathPolicy<0, 16>::TILE_VECS == LdsPolicy::TILE_VECS && LdsPolicy::BS == 512,
              "the ceilings run the production grid");
#endif

const std::array<VecFn, kTileOrders> kStreamRead = {
    &dev::rs_stream_read<0>, &dev::rs_stream_read<2>, &dev::rs_stream_read<5>, &dev::rs_stream_read<6>,
    &dev::rs_stream_read<8>, &dev::rs_stream_read<10>, &dev::rs_stream_read<11>};
const std::array<VecFn, kTileOrders> kStreamWrite = {
    &dev::rs_stream_write<0>, &dev::rs_stream_write<2>, &dev::rs_stream_write<5>,
    &dev::rs_stream_write<6>, &dev::rs_stream_write<8>, &dev::rs_stream_write<10>,
    &dev::rs_stream_write<11>};

#if CALLFS_RS_AB_INSTANCES
// modes 3..5 (probe): the write streams alone from each row's first 64 / 128 / 256-B
// boundary, consecutive tiles
const std::array<VecFn, 3> kStreamWriteAligned = {
    &dev::rs_stream_write<0, 64>, &dev::rs_stream_write<0, 128>, &dev::rs_stream_write<0, 256>};
// modes 6..8 (probe): the read streams alone from each shard's first 64 / 128 / 256-B boundary
const std::array<VecFn, 3> kStreamReadAligned = {
    &dev::rs_stream_read<0, 64>, &dev::rs_stream_read<0, 128>, &dev::rs_stream_read<0, 256>};
#endif
}  // namespace

hipError_t launch_ceiling(ApplyArgs a, hipStream_t stream, int order, int mode, LaunchEvents ev) {
  if (a.R < 1 || a.R > kMaxRowsPerLaunch || a.K < 1 || a.K > kMaxK || a.batch < 1 || !a.ltabs ||
      mode < 0 || mode > 8)
    return hipErrorInvalidValue;
  if (!kAbInstances && mode != 1 && mode != 2) return hipErrorNotSupported;
  a.nvec = a.S / 16;
  if (a.nvec == 0) return hipSuccess;
  a.tail_in_vec = a.nvec * 16 < a.S ? tail_code(a.nvec, LdsPolicy::TILE_VECS, LdsPolicy::BS) : 0u;
  if (order >= kOrderBitslice) order -= kOrderBitslice;  // (bit-sliced: its tile order)
  else if (order >= kOrderTriDbG) order = static_cast<int>(TileOrder::kGroup8);  // (A/B forms:
  else if (order >= kOrderDma) order -= kOrderDma;                          //  their tile order)
  else if (order >= kOrderRealign64) order = order - kOrderRealign64 + kOrderRealign;
  else if (order >= kOrderRealignTri) order = order - kOrderRealignTri + kOrderRealign;
  else if (order >= kOrderTri) order -= kOrderTri;
  if (order >= kOrderWix) order -= kOrderWix;  // bounded by the nibble kernel's traffic
  // the order the production launch would take (a tuned order, else the rule; the
  // realigning and v_perm launches are bounded by the plain kernel's traffic)
  static constexpr TileOrder kRealignOrders[3] = {TileOrder::kConsecutive, TileOrder::kXcd8,
                                                 TileOrder::kXcd32};
  const bool realign = a.R <= 8 && can_realign(a) &&
                       (order >= kOrderRealign || (order < 0 && takes_realign(a)));
  const TileOrder ord =
      realign    ? kRealignOrders[realign_order_index(order)]
      : a.R <= 8 ? (order >= 0   ? static_cast<TileOrder>(order)
                    : takes_tri(a) ? static_cast<TileOrder>(tri_rule_of(a))
                                   : lds_rule(a))
                 : (order >= 0 ? static_cast<TileOrder>(order) : wide_rule(a));
  const unsigned grid = dev::vec_grid<LdsPolicy>(a.nvec, a.batch);
  if (mode > 0) {  // the read streams alone / the write streams alone
#if CALLFS_RS_AB_INSTANCES
    const VecFn fn = mode >= 6   ? kStreamReadAligned[mode - 6]
                     : mode >= 3 ? kStreamWriteAligned[mode - 3]
                               : (mode == 1 ? kStreamRead : kStreamWrite)[static_cast<int>(ord)];
#else
    const VecFn fn = (mode == 1 ? kStreamRead : kStreamWrite)[static_cast<int>(ord)];
#endif
    a.tail_in_vec = 0;
    launch_sliced(grid, a.K + a.R, a, [&](uint32_t blocks, bool first, bool last) {
      dispatch(fn, dim3(blocks), dim3(LdsPolicy::BS), 0, stream, ev, first, last, a);
    });
    return hipGetLastError();
  }
#if CALLFS_RS_AB_INSTANCES
  VecFn fn;
  if (a.R <= 8)
    fn = kNomath[static_cast<int>(ord)][a.R - 1];
  else
    fn = ord == TileOrder::kSeg8 ? kNomathWideQ8[a.R - 9] : kNomathWide[a.R - 9];
  const size_t lds = dev::lds_bytes(a.K, a.R);
  if (lds > (64u << 10))
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10);
  launch_sliced(grid, a.K + a.R, a, [&](uint32_t blocks, bool first, bool last) {
    dispatch(fn, dim3(blocks), dim3(LdsPolicy::BS), lds, stream, ev, first, last, a);
  });
  return hipGetLastError();
#else
  return hipErrorNotSupported;
#endif
}

}  // namespace callfs
