// Launch interface of the GF(2^8) shard-matrix kernels (rs_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <vector>
#include <cstdint>

// 1: also build the measurement-only kernel forms (the 6-bit triple lookups, the 64-vector
// and double-buffered realigning forms, the no-lookup and aligned-window ceilings) and honour
// the A/B environment toggles (CALLFS_RS_WIX, _TRIDB, _REALIGN, _TAIL_LAST_TPS). The
// product library is built with 0: `python callfs_amd/build.py --ab` writes the A/B build to
// libcallfs_rs_ab.so, which the development tools load through CALLFS_RS_LIB.
#ifndef CALLFS_RS_AB_INSTANCES
#define CALLFS_RS_AB_INSTANCES 0
#endif

namespace callfs {

constexpr bool kAbInstances = CALLFS_RS_AB_INSTANCES != 0;

constexpr int kMaxRowsPerLaunch = 16;  // output rows per launch group (LDS kernel above 4)
constexpr int kMaxK = 256;

// One launch applies an R x K coefficient block to every stripe of a batch:
//   out[b][r][x] = XOR_i coef[r][i] * in[b][i][x]      for x in [0, S)
// Rows with bit r of verify_mask set are compared against out[b][r] instead of
// stored; any mismatch ORs 1 into *status (upstream Verify, codec.go:59).
struct ApplyArgs {
  const uint8_t* const* in_tab;  // [batch][K] device pointers (k valid shards)
  uint8_t* const* out_tab;       // [batch][R] device pointers (written or compared)
  const uint32_t* tabs;          // [K][R][5] v_perm tables (gf256.hpp perm_tables)
  const uint8_t* ltabs;          // [K][32][W] nibble tables for rs_apply_lds (gf256.hpp nibble_tables)
  uint64_t S;                    // shard bytes
  uint64_t nvec;                 // 16-byte vectors per shard handled by the vector kernel
  uint32_t verify_mask;
  int* status;                   // mismatch flag; stripe b uses status[b * status_stride]
  int status_stride;
  int K;
  int R;
  int batch;
  // log2 of the largest power of two dividing every difference between the shard
  // addresses of a stripe (shard_addr_tz); picks the LDS kernel's tile order. 0 = odd
  // or unknown.
  int addr_tz;
  // byte distance between consecutive stripes' shards when it is the same for every
  // stripe (0 = one stripe or irregular); also keys the tile order.
  uint64_t stripe_stride;
  // first tile of this launch (launch_apply cuts grids of many tiles into consecutive
  // slices; a kernel's block b works on tile t_base + b of the whole tile order)
  uint32_t t_base;
  // OR of (address & 15) over every input shard pointer of every stripe: nonzero when
  // some input shard is not 16-B aligned (upstream Split layout of a contiguous object
  // at odd S); selects the LDS kernel's realigning form (rs_apply.hpp REALIGN)
  uint32_t in_misalign;
  // the same over the launch group's output (written or compared) shard pointers; with
  // in_misalign it selects the form that also aligns the parity stores (REALIGN 2)
  uint32_t out_misalign;
  // set by launch_apply: nonzero when the vector kernel also computes the ragged tail S % 16
  // (no separate byte-kernel launch): (tile << 2) | (last wave << 1) | 1, the tile of each
  // stripe and the wave (0 or the block's last) that take it (rs_apply.hpp tail_lane)
  uint32_t tail_in_vec;
  // host-side handle of the launch group's bit-sliced kernel (bitslice.hpp bs::Kernel, compiled
  // at plan time for this coefficient block) or null; the device kernels never read it
  const void* bs;
};

// One-dispatch small host calls (rs_apply_small): stripe b's shard i lives at
// base + b*spitch + i*cpitch in host-coherent pinned staging that the kernel reads and
// writes over PCIe; one launch group (R <= 16 rows) per launch.
struct SmallArgs {
  const uint8_t* base;
  uint64_t spitch;       // bytes per stripe in staging
  uint64_t cpitch;       // bytes per shard (S rounded up to 16)
  uint32_t nvec;         // 16-B vectors per shard, ceil(S / 16)
  uint32_t S;
  int K;
  int R;
  int batch;
  uint32_t verify_mask;
  // device memory, uploaded once per (lane, tables): [K][R][5] v_perm tables of the group,
  // then idx: the shard index of input i (idx[i], the k valid shards) and of row r
  // (idx[256 + r]). Kept out of the kernel arguments: 272 B of arguments cost the launch
  // ~2 us (profiles/r03/small_path/r03_smalltrace2)
  const uint32_t* tabs;
  const uint8_t* idx;
  // idx[0..15] and idx[256..271] again, as kernel arguments: the data loads of a k <= 16
  // call need no dependent device-memory read first
  uint32_t idx_in[4];
  uint32_t idx_out[4];
  int* status;           // host-coherent: status[b] = 1 when stripe b's Verify rows mismatch
  // completion flag (last launch of a call only, else null): when every block of the launch
  // has finished, the last one stores `seq` into *done (host-coherent) with a system-scope
  // release; `counter` (device memory, 0 between launches) counts finished blocks
  int* done;
  unsigned* counter;
  int seq;
};

// Enqueues rs_apply_small for one launch group on `stream`.
hipError_t launch_small(const SmallArgs& a, hipStream_t stream);

// addr_tz for a set of shard addresses: trailing zeros of the OR of their differences
// from the first (63 for a single address).
inline int shard_addr_tz(const void* const* p, int count) {
  uint64_t d = 0;
  for (int i = 1; i < count; ++i)
    d |= reinterpret_cast<uintptr_t>(p[i]) ^ reinterpret_cast<uintptr_t>(p[0]);
  return d ? __builtin_ctzll(d) : 63;
}

// [0, 16*floor(S/16)) runs on a vector kernel and the ragged tail on the byte kernel,
// whatever the pointers' alignment: gfx950 under ROCm (SH_MEM_CONFIG alignment mode
// "unaligned") serves 16-byte global accesses at any byte address, and at odd shard
// offsets (upstream Split layout of a contiguous object) that ran 4.7x the byte kernel
// (DESIGN.md §5). bytes_only forces the byte kernel over all of [0, S) (kbench A/B).
// Returns hipSuccess or the launch error.
// order_candidates / launch_apply code for the realigning kernel of misaligned launches
// (tile orders are TileOrder values 0..4, which on a misaligned launch select the plain
// kernel with unaligned accesses)
// (kOrderRealign + the TileOrder it runs in: consecutive, X8 or X32)
constexpr int kOrderRealign = 32;
// (kOrderWix + a TileOrder: the R <= 4 LDS kernel with 6-bit lookups over shard triples,
// rs_apply.hpp Policy::WIX; aligned launches without Verify rows, K >= 3)
constexpr int kOrderWix = 64;
// (kOrderTri + consecutive / G2 / X32 / Q8 / Q16: the triple loop with nibble lookups)
constexpr int kOrderTri = 96;
// (kOrderRealignTri + consecutive / X8 / X32: the realigning kernel with its aligned loads
// issued in triples)
constexpr int kOrderRealignTri = 128;
// (kOrderRealign64 + consecutive / X8 / X32: misaligned inputs with 16-B-aligned outputs --
// upstream Split of an io.ReadAll body, whose parity reedsolomon allocates aligned -- in
// 64-vector waves: aligned loads realigned in registers, lane 63's neighbour vector from
// one extra single-lane load, stores unshifted in 1 KiB wave windows; rs_apply.hpp
// REALIGN 5)
constexpr int kOrderRealign64 = 160;
// (kOrderDma + consecutive / G2 / Q8 / X32: aligned R <= 8 launches with their input vectors
// staged through an LDS-DMA ring, rs_apply.hpp Policy::DMA; A/B build)
constexpr int kOrderDma = 192;
// (kOrderTriDbG + 0 / 1: R <= 4, K >= 6 double-buffered triples with the tiles of 4 / 8 stripes
// interleaved (G4 / G8); A/B build)
constexpr int kOrderTriDbG = 224;
// (kOrderBitslice + any TileOrder: the launch group's bit-sliced kernel, ApplyArgs::bs,
// DESIGN.md §5.7; every launch group gets one: the rule takes it for wide groups and
// rs_plan_tune times it for every group)
constexpr int kOrderBitslice = 256;
constexpr int kBitsliceMinRows = 1;

// `order` >= 0 (a TileOrder) replaces the measured rule for this launch where the
// chosen kernel has an instance in that order (order_candidates lists them); -1 = the
// rule (or CALLFS_RS_TILE_ORDER).
// ev_start / ev_stop (optional, created by the caller): recorded by the launch's first
// kernel dispatch when it starts and by its last when it ends (hipExtLaunchKernel), so
// their interval is the kernels' own time without the stream's gaps before and after.
struct LaunchEvents {
  hipEvent_t start = nullptr;
  hipEvent_t stop = nullptr;
};
hipError_t launch_apply(ApplyArgs a, hipStream_t stream, bool bytes_only = false, int order = -1,
                        LaunchEvents ev = {});

// Tile orders worth timing for launch `a` (rs_plan_tune): the rule's choice first, then
// the alternatives that have kernel instances for this path. Empty when the launch has
// no choice (byte kernel, realigning kernel, S < 16). every_instance: also the orders
// that have an instance but never measured faster (rs_plan_set_orders accepts them).
std::vector<int> order_candidates(const ApplyArgs& a, bool every_instance = false);

// True when the rule runs launch `a` on its bit-sliced kernel (ApplyArgs::bs) once that is
// compiled (rs_plan_create compiles it up front for such launches).
bool bitslice_wanted(const ApplyArgs& a);

// The form (an order code as order_candidates lists them) launch_apply runs for `order`
// (-1 = the tune table's entry for the launch's shape, else the rule, whose bit-sliced choice
// counts once its kernel is compiled).
int launch_form(const ApplyArgs& a, int order);

// The tune table (tune_table.hpp): the order rs_plan_tune measured for launch `a`'s shape on
// the current device, when it is one `a` offers and (for a bit-sliced order) its kernel is
// compiled -- else -1, and the rule decides. record_tuned stores a tuner's choice.
int tuned_order(const ApplyArgs& a);
void record_tuned(const ApplyArgs& a, int order);

// Measurement only (rs_plan_launch_ceiling), for launch `a` in the order the production
// launch takes (`order` as for launch_apply), on the production grid and slicing:
//   mode 0  the no-lookup form of the LDS kernel: same loads, stores and table prologue,
//           one XOR per input dword instead of the lookups (outputs junk, Verify rows may
//           flag status);
//   mode 1  the launch's read streams alone (inputs + Verify rows; writes nothing);
//   mode 2  its write streams alone (junk into the written rows);
//   modes 3..8 (probes) the write / read streams from each row's first 64 / 128 / 256-B
//           boundary.
// Modes 0 and 3..8 exist in the A/B build only (hipErrorNotSupported otherwise).
hipError_t launch_ceiling(ApplyArgs a, hipStream_t stream, int order, int mode,
                          LaunchEvents ev = {});


// Tuning hook for tools/kbench.hip (not part of the C ABI): tiles per launch slice for
// every later launch_apply in the process; 0 = never slice, < 0 = the built-in rule
// (CALLFS_RS_MAX_TILES_PER_LAUNCH or ~4 GiB of traffic per slice).
void set_slice_tiles_for_tuning(long long tiles);

}  // namespace callfs
