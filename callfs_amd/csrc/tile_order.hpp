// Tile order of the RS kernels (DESIGN.md §6.2 "Tile order"): which column tile of which
// stripe block t works on (map_tile, host and device), and the measured rules that pick
// the order for a launch (lds_tile_order, wide_tile_order, vec_tile_order; host).
// Plain C++ apart from the __host__ __device__ marker, so tests/native/host_test.cpp
// builds it with g++ and checks that every order is a bijection and the rules' choices.
#pragma once

#include <algorithm>
#include <cstdint>

#if defined(__HIPCC__)
#define CALLFS_HD __host__ __device__
#else
#define CALLFS_HD
#endif

namespace callfs {

// Block t -> (stripe, column tile) for tile order ORD (Policy::ORD; LDS kernel and the
// tools/kbench read probe). tps = tiles per stripe; t < tps * batch.
template <int ORD>
CALLFS_HD inline void map_tile(uint32_t t, uint32_t tps, uint32_t batch, uint32_t& stripe,
                               uint32_t& tile) {
  if constexpr (ORD == 0 || ORD >= 10) {  // 10, 11: consecutive after block_tile (below)
    stripe = t / tps;
    tile = t - stripe * tps;
  } else if constexpr (ORD >= 6) {
    // one stripe at a time, its columns cut into Q segments; neighbouring blocks take
    // the same position of different segments (tiles past the last full round of Q
    // keep their place, so the map stays a bijection)
    constexpr uint32_t Q = ORD == 6 ? 8 : (ORD == 7 ? 32 : (ORD == 8 ? 16 : 64));
    stripe = t / tps;
    const uint32_t r = t - stripe * tps, seg = tps / Q;
    tile = r < seg * Q ? (r % Q) * seg + r / Q : r;
  } else {
    // groups of G stripes whose tiles interleave (neighbouring blocks: same offset of
    // different stripes)
    constexpr uint32_t G = ORD == 2 ? 8 : (ORD == 3 ? 32 : (ORD == 4 ? 4 : 2));
    const uint32_t per_group = G * tps;
    const uint32_t g = t / per_group, r = t - g * per_group;
    const uint32_t gsz = std::min<uint32_t>(G, batch - g * G);
    tile = r / gsz;
    stripe = g * G + (r - tile * gsz);
  }
}

// XCD-grouped consecutive orders (ORD 10: X8, 11: X32). A dispatch deals its blocks to the
// 8 XCDs round-robin (block b of the launch runs on XCD b % 8), so in consecutive order
// neighbouring tiles of a row run on different XCDs, each with its own L2. X8 / X32 give
// the blocks b, b+8, b+16, ... of every group of 8*J blocks J consecutive tiles (J = 8 /
// 32): the tiles in flight are those of consecutive order, permuted within the group, and
// each XCD streams runs of J neighbouring tiles. Measured: write streams
// unchanged, read streams of 6.7 MB shards 6 % shorter; adopted for the realigning kernel
// and for read-only launches (lds_tile_order). Blocks past the last full group keep their
// place. Host-side as well: host_test checks that the map is a bijection.
template <int ORD>
CALLFS_HD inline uint32_t block_tile(uint32_t b, uint32_t nblocks) {
  if constexpr (ORD >= 10) {
    constexpr uint32_t J = ORD == 10 ? 8 : 32, G = 8 * J;
    if (b >= nblocks / G * G) return b;
    const uint32_t g = b / G, r = b - g * G;
    return g * G + (r & 7u) * J + (r >> 3);
  } else {
    return b;
  }
}

// Launch-time choice; Policy::ORD of each: consecutive 0, G8 2, G2 5, Q8 6, Q16 8, X8 10,
// X32 11.
enum class TileOrder { kConsecutive, kGroup8, kGroup2, kSeg8, kSeg16, kXcd8, kXcd32 };
constexpr int kTileOrders = 7;


// Tile order for R <= 8 (Policy::ORD; tools/kbench.hip KB_ORD, profiles/r01/tile_order/,
// 5-15 rounds, % of 8 TB/s, DESIGN.md "Tile order"). Neighbouring blocks normally take
// neighbouring column tiles of one stripe (consecutive). For small shards it pays to
// interleave the same column tile of G stripes instead: G8 up to 256 KiB (RS(10,4)
// 256 KiB 70.8 -> 73.3-74.0, RS(16,4) 64 KiB 70.9 -> 73.5), G2 up to 1 MiB (512 KiB
// 72.6 -> 77.6, RS(6,3) 1 MiB 73.7 -> 79.3, RS(10,4) 1 MiB 78.8 -> 79.7) and, for 14 or
// more shard streams per stripe, up to 8 MiB (RS(16,4) 4 MiB 69.5 -> 75.2, 64 MiB
// objects 74.6 -> 76.5); with fewer streams G2 loses 1-3.5 points at 4 MiB (RS(4,2)
// 79.1 -> 75.6), so those keep consecutive tiles. Above 8 MiB, shards whose addresses
// differ by multiples of 8 MiB (addr_tz >= 23: power-of-two pitches, 24/48 MiB) lose
// 5-13 points in consecutive order once a stripe has 12 or more streams; interleaving
// Q column segments of the stripe recovers it: Q16 for 16-32 MiB (RS(10,4) 16 MiB 67.6
// -> 75.6, RS(16,4) 16 MiB 64.4 -> 77.6, RS(8,4) 32 MiB 71.5 -> 80.1), Q8 otherwise
// below 128 MiB (24 MiB 70.9 -> 75.8, 48 MiB 68.9 -> 75.1, 64 MiB 69.3 -> 77.2). With
// fewer streams Q16 hurts at 16 MiB (RS(4,2) 75.7 -> 67.9), so 6-11 streams keep
// consecutive tiles up to 16 MiB and take Q8 above (RS(6,3) 32 MiB 75.1 -> 79.0).
// Pitches with few trailing zeros (the 13-107 MB column slices of 1 GiB objects) and
// >= 128 MiB keep consecutive tiles.
//
// Launch groups with Verify rows (the decodes of a download, codec.go:59) keep G2 only up
// to 1 MiB: from 1 to 8 MiB consecutive tiles ran 0.2-1.9 points faster on every decode
// pattern (configs[2] shape, S = 6,710,887: one erasure {5} 73.9 -> 75.2, {13} 74.3 ->
// 75.9, nothing erased 77.4 -> 78.1; tools/ceiling_sweep.py, profiles/r03/ceil1,
// profiles/r02/decode_order_sweep).
//
// Launch groups that only compare (every row a Verify row: the download with nothing
// lost, codec.go:59, read-only) take X32 above 256 KiB shards: tools/order_ab.py,
// profiles/r03/dec3, dec4 (three runs, two boxes), % of 8 TB/s, rule -> X32: RS(10,4)
// 1 MiB 85.0 / 85.4 / 85.1 -> 85.8 / 86.4 / 85.5, 6.7 MB 83.3 / 84.4 / 83.2 -> 84.0 /
// 84.0 / 84.5, RS(4,2) 1 MiB 82.3 / 82.3 -> 82.9 / 83.5, RS(16,4) 4 MiB 80.2 / 80.3 ->
// 81.2 / 81.4, RS(6,3) 2.8 MB 84.8 / 84.6 -> 85.3 / 85.3; at 105 KB shards all orders
// within 0.3.
//
// Round 4 re-measured G2 for many streams above 1 MiB on the current kernels (every order,
// interleaved, tools/order_ab.py; profiles/r04/tri_sweep1-3, tridb_wide, wide_db, % of
// 8 TB/s, G2 -> consecutive, runs averaged): with R <= 4 consecutive tiles won on every
// shape, RS(16,4) 4 MiB 74.2 -> 75.7, RS(14,4) 4.8 MB 71.7 -> 73.6, RS(20,4) 3.4 MB 72.8 ->
// 74.0, RS(24,4) 2.8 MB 71.0 -> 71.8, RS(12,4) 5.6 MB 74.0 -> 74.9, RS(10,4) 4 MiB 74.3 ->
// 75.0, RS(16,4) 2 MiB 75.2 -> 75.6; with R = 8 G2 kept its lead (RS(10,8) 6.7 MB 71.5 vs
// 70.9, RS(8,8) 8 MiB 71.7 vs 69.0). So G2 above 1 MiB only for launches of 5-8 rows.
//
// tps = tiles of 512 16-B vectors (8 KiB) per stripe; streams = K + R of the launch;
// addr_tz / stripe_stride as in ApplyArgs; verify = the launch compares some rows,
// read_only = it compares every row (writes nothing); rows = R.
inline TileOrder lds_tile_order(uint64_t S, uint64_t tps, int addr_tz, int streams,
                                uint64_t stripe_stride, bool verify = false,
                                bool read_only = false, int rows = 8) {
  if (read_only && tps > 32) return TileOrder::kXcd32;
  // (round 5, planar: read-only launches of 5-8 rows up to 256 KiB run the ring fastest in
  // consecutive order, RS(10,8) 104,858 B 76.5; profiles/r05/decode_rule/)
  if (read_only && rows >= 5) return TileOrder::kConsecutive;
  // stripes exactly 2 MiB apart: interleaving stripes costs 2-12 points (RS(8,8) 128 KiB
  // 72.4 -> 60.6 with G8, RS(4,4) 256 KiB 77.9 -> 65.8, RS(6,2) 256 KiB 81.5 -> 78.4);
  // strides of 1, 4, 8 or 16 MiB interleave fine (profiles/r01/tile_order/segments/
  // ord_stride*). Consecutive tiles there.
  if (stripe_stride == (2ull << 20) && tps <= 1024) return TileOrder::kConsecutive;
  // exactly 1 MiB apart: G2 beats G8 (RS(4,4) 128 KiB 61.2 -> 68.7, RS(8,8) 64 KiB 64.2
  // -> 67.7, RS(12,4) 64 KiB equal)
  if (stripe_stride == (1ull << 20) && tps <= 32) return TileOrder::kGroup2;
  // round 5, planar layout (tools/jobs.sh rule_sweep, profiles/r05/rule/): more than 16 inputs
  // with R <= 4 on 256 KiB - 1 MiB shards run the ring faster in consecutive order
  // (RS(20,4) 838,861 B G2 73.9 / 73.4 -> consecutive 74.9 / 74.7); the same from 13 inputs
  // and down to the smallest shards, where tri_rule_order leaves these launches to the ring
  // (RS(16,4) 300,000-1,000,000 B, RS(20,4) / RS(24,4) 40-224 KiB; profiles/r05/tiles/)
  if (tps <= 128 && streams - rows > 12 && rows <= 4 && !verify) return TileOrder::kConsecutive;
  if (tps <= 32) return TileOrder::kGroup8;  // S <= 256 KiB
  // (round 5, planar: not for more than 16 inputs, RS(32,8) 2 MiB G2 69.3 / 69.2 ->
  // consecutive 70.4 / 70.7)
  if (tps <= 128 || (tps <= 1024 && streams >= 14 && rows >= 5 && !verify && streams - rows <= 16))
    return TileOrder::kGroup2;
  if (tps <= 1024) return TileOrder::kConsecutive;  // S <= 8 MiB, few streams
  if (addr_tz >= 23 && S < (128ull << 20)) {
    if (streams >= 12)
      return addr_tz >= 24 && S <= (32ull << 20) ? TileOrder::kSeg16 : TileOrder::kSeg8;
    return S <= (16ull << 20) ? TileOrder::kConsecutive : TileOrder::kSeg8;
  }
  return TileOrder::kConsecutive;
}

// The triple form's tile order for the order the nibble rule (or CALLFS_RS_TILE_ORDER)
// picks: G8 (shards up to 256 KiB) -> X32, which ran within 0.6 points of G8 for the 6-bit
// form at 1 MiB objects; every other order has its own triple instance.
inline TileOrder tri_order(TileOrder nibble) {
  return nibble == TileOrder::kGroup8 ? TileOrder::kXcd32 : nibble;
}

// Triple-load form of an aligned R <= 8 LDS launch (rs_kernels.hip takes_tri; DESIGN.md §5
// "Shard triples", "Round 4"): the loads of three input shards issued together, then their
// nibble lookups; with R <= 4 and K >= 6 double-buffered in two register sets
// (Policy::WIX 3), else rotating (WIX 2). Returns the triple form's tile order (instances:
// consecutive, G2, X32, Q8, Q16, X8), or -1 for the ring of three in the nibble rule's
// order `nibble`. % of 8 TB/s below, the previous rule -> this one:
//  * round 3 (profiles/r03/r03s5, r03s6): launches that write every row or compare every
//    row, shards up to 2 MiB (4 MiB with K <= 6), at <= 256 KiB only K <= 6 or R >= 5, in
//    the nibble rule's order (G8 -> X32): RS(4,2) 1 MiB 72 -> 80.6, RS(10,8) 74.4 -> 78.2;
//  * round 4, rotating form (profiles/r04/tri_sweep1, tri_sweep2,
//    tri_validate, triord): K <= 5 in X32 up to 8 MiB and X8 above (RS(4,2) 8 MiB 70.0 ->
//    79.6, 16 MiB 69.9 -> 81.1, 32 MiB 69.8 -> 81.4); R 5..8 with K = 6 in X32 / Q16;
//    read-only launches in X32 at every size (RS(6,3) 16 MiB 85.7 -> 90.0, RS(10,4) 4 MiB
//    84.9 -> 86.3); Q16 on 16-32 MiB power-of-two pitches for K 7..12;
//  * round 4, double-buffered form, R <= 4 and K >= 6 (profiles/r04/tri_sweep3,
//    tridb_wide): X32 up to 256 KiB (RS(12,4) 87 KB 70.9 -> 75.6, RS(32,4) 32 KiB 67.8 ->
//    79.3, RS(20,4) 52 KB 68.1 -> 72.2); K = 6 in X32 to 8 MiB, X8 above (RS(6,3) 1 MiB 74.5
//    -> 78.7, 8 MiB 73.0 -> 78.0, 16 MiB 72.8 -> 77.7); K >= 7 in G2 to 1 MiB (RS(10,4)
//    76.5 -> 80.0, RS(16,4) 76.5 -> 78.4, RS(32,4) 74.2 -> 76.0), Q8 to 2 MiB (RS(8,4) 77.0
//    -> 80.7, RS(10,4) 1.68 MB 74.4 -> 78.8), Q8 to 8 MiB for K <= 12 (RS(10,4) 6.7 MB 73.0
//    -> 76.9, RS(12,4) 5.6 MB 73.8 -> 76.2, RS(8,4) 8 MiB 74.4 -> 75.0), Q16 on 16-32 MiB
//    power-of-two pitches (RS(10,4) 73.8 -> 78.7); K > 12 above 2 MiB keeps the ring
//    (RS(16,4) 4 MiB: consecutive 76.0 vs 72.5), and so does K > 16 from 256 KiB to 1 MiB
//    unless the shards sit 64 KiB-aligned apart (profiles/r04/wide_db, regress: RS(20,4)
//    S = 838,861 at a 256-B pitch, ring in G2 73.2 / 72.9 vs 71.1 / 71.0; RS(24,4) 699,051 B
//    72.0 vs 70.9; at a 1 MiB pitch the form leads, RS(20,4) 78.1 vs 74.8);
//  * written + Verify rows (the one-erasure decode), R <= 4, the early-compare forms: K <= 4
//    in X32 (RS(4,2) erase {1} 76.2 -> 80.1); K = 5 up to 1 MiB in the nibble rule's order;
//    K 6..16 double-buffered in G2 to 1 MiB and X32 above (profiles/r04/tri_verify_ab2:
//    RS(10,4) {5} 75.0 -> 77.2, RS(12,4) {7} 74.4 -> 77.3, RS(16,4) {3} 74.6 -> 77.5,
//    RS(10,4) 6.7 MB {5} 73.8 -> 75.9).
inline int tri_rule_order(int K, int R, bool misaligned, bool verify, bool read_only,
                          uint64_t tps, int addr_tz, uint64_t S, TileOrder nibble) {
  if (R > 8 || K < 4 || misaligned) return -1;
  const int x32 = static_cast<int>(TileOrder::kXcd32), q16 = static_cast<int>(TileOrder::kSeg16),
            q8 = static_cast<int>(TileOrder::kSeg8), x8 = static_cast<int>(TileOrder::kXcd8),
            g2 = static_cast<int>(TileOrder::kGroup2);
  const bool pow2_16_32 = addr_tz >= 24 && S >= (16ull << 20) && S <= (32ull << 20);
  // R <= 4 with K >= 6 runs the double-buffered form (rs_kernels.hip kTriDbMinK)
  const bool db = R <= 4 && K >= 6;
  const int cons = static_cast<int>(TileOrder::kConsecutive);
  if (verify && !read_only) {  // written + Verify rows: only the R <= 4 early-compare forms
    if (R > 4) return -1;
    if (K <= 4) return x32;
    if (db) {  // round 4 (profiles/r04/tri_verify_ab2): G2 up to 1 MiB, X32 above
      // round 5, planar (tools/jobs.sh decode_rule_sweep, profiles/r05/decode_rule/): up to 256 KiB
      // the early-compare triples for K >= 7, where the ring ran (in G2: RS(10,4) 104,858 B
      // erase {1} 71.0 -> 75.7, {10} 72.0 -> 76.9; RS(12,4) 87,382 B {1} 69.3 -> 75.2; RS(8,4)
      // 128 KiB {1} 74.6 -> 77.6; RS(16,4) 64 KiB {1} 70.5 -> 77.3)
      // Between those cells G2 collapses on shards of at most 10 tiles that are not a power of
      // two: 2-7 points behind X32 (RS(10,4) 75,550 B {1} 67.8 vs 73.9, 45,000 B 70.0 vs 74.4;
      // 40 sizes x K = 8..16, profiles/r05/tiles/mixed_small_band.jsonl); from 11 to 32 tiles
      // the two tie on average and the cells above keep G2 (X32 there lost 1.5-2.7 points,
      // profiles/r05/decode_rule/after3_x32small.jsonl)
      if (tps <= 32) return K <= 6 || tps <= 10 ? x32 : g2;
      if (K > 16) return -1;
      // (round 5: G2 to 2 MiB, RS(10,4) 1.68 MB {1} X32 74.7 -> G2 75.5, RS(12,4) 1.4 MB
      // {12} 73.4 -> 74.5; but below 1 MiB X32 leads G2 by 0.6-1.0 on average and up to 3.6,
      // RS(16,4) 832,781 B {1} 72.3 -> 75.9, RS(10,4) 1,111,633 B 74.9 -> 78.2; 8 sizes x
      // K = 6 / 10 / 16, profiles/r05/tiles/mixed_mid_band.jsonl; pitches that are multiples
      // of 128 KiB keep G2, RS(16,4) 1 MiB {1} 76.7 with the tuner finding nothing better)
      return tps <= 128 && addr_tz < 17 ? x32 : tps <= 256 ? g2 : x32;
    }
    if (tps <= 32) return x32;
    return tps <= 128 ? static_cast<int>(tri_order(nibble)) : -1;
  }
  if (db && !read_only) {  // round 4, double-buffered (profiles/r04/tri_sweep3, tridb_wide)
    // (round 5, planar: G2 for K > 16, RS(20,4) 52 KB X32 69.8 / 70.0 -> G2 72.5.) A sweep of
    // shard sizes between 40 and 96 KiB (tile fills 0.0-0.8; tools/ceiling_sweep.py pinned
    // orders, profiles/r05/tiles/) then put the ring in consecutive order ahead for K > 12
    // whenever the pitch is not 64 KiB-aligned: K = 20 / 24 tri-G2 -> ring by 0-6 points
    // (RS(20,4) 57,344 B 70.7 -> 73.9, 45,875 B 66.4 -> 71.3; 52,429 B equal), K = 16
    // tri-X32 -> ring by 0.3-1.8 on 6 of 8 sizes. On power-of-two shards of at most 64 KiB
    // tri-X32 leads the ring by 2.5-3.1 (RS(20,4) 64 KiB 76.6 vs 74.1, RS(16,4) 77.5 vs 74.4;
    // 32 KiB equal or ahead), while at 128 KiB the ring leads by 1.7-3.9 and at 192 KiB
    // (64 KiB-aligned) by 3-4 (rule_after*.jsonl there, K = 14..32)
    if (tps <= 32) return K > 12 && ((S & (S - 1)) != 0 || tps > 8) ? -1 : x32;
    if (K == 6) return tps <= 1024 ? x32 : x8;
    // 256 KiB - 1 MiB (round 5, pinned orders at 9 sizes, profiles/r05/tiles/mid_band.jsonl):
    // G2 only where the pitch is a multiple of 128 KiB (512 KiB: X32 collapses to 70-73);
    // elsewhere X32 for K <= 12 (K = 8 / 10 tri-G2 -> tri-X32 by 1-3.4 on every size, RS(8,4)
    // 464,531 B 75.7 -> 78.1, RS(10,4) 655,000 B 75.8 -> 78.9; K = 12 all forms within ~1)
    // and the ring in consecutive order above (RS(16,4) 8 of 9 sizes, 832,781 B 69.2 -> 74.3)
    if (tps <= 128) return addr_tz >= 17 ? g2 : K > 12 ? -1 : x32;
    // K >= 10 on 1-8 MiB shards at pitches that are not a power of two: the ring of three in
    // consecutive order (round 4, fourth session,
    // profiles/r04/mid1/, two passes, one-block layout, tri-Q8 -> ring: RS(10,4) 1.68 MB
    // 74.2 -> 75.2, 6.7 MB 73.2 -> 74.0, RS(12,4) 1.4 MB 73.2 -> 75.2, 5.6 MB 71.4 -> 74.9;
    // power-of-two pitches keep tri-Q8: RS(8,4) 2 MiB 77.2 vs 75.0, 4 MiB 74.9 vs 72.2)
    // round 5, planar (tools/jobs.sh rule_sweep, tools/jobs.sh cfg12_orders, profiles/r05/): above 1 MiB
    // the ring in consecutive order for K >= 10 at every pitch (RS(10,4) 2 MiB tri-Q8 72.9 ->
    // ring 76.9, 4 MiB 74.8 -> 75.4, 8 MiB 72.6 -> 75.6; round 4 kept tri-Q8 on power-of-two
    // pitches in the one-block layout), except Q16 on 16-32 MiB power-of-two pitches (round 4,
    // RS(10,4) 16 MiB 73.8 -> 78.7); K 7..9 in G2 to 2 MiB (RS(8,4) 2 MiB Q8 75.1 / 74.1 -> G2
    // 77.6 / 76.9) and the ring to 8 MiB (RS(8,4) 8 MiB Q8 73.6 / 72.6 -> ring 74.2 / 75.4)
    if (K >= 10) return K <= 12 && pow2_16_32 ? q16 : -1;
    if (tps <= 256) return g2;
    // K 7..9 from 2 to ~6.5 MiB in Q8 (round 5, pinned orders at 6 sizes,
    // profiles/r05/tiles/r8_small_k79_mid.jsonl: ring -> tri-Q8 RS(8,4) 2.5 MB 74.0 -> 77.4,
    // 4.39 MB 74.2 -> 78.7, 6.5 MB 74.7 -> 77.8; at 7.5 MB every triple form drops below the
    // ring, 69.5-72.5 vs 73.7, as round 4 found at 8 MiB)
    if (tps <= 800) return q8;
    if (tps <= 1024) return -1;
    return pow2_16_32 ? q16 : -1;
  }
  // Read-only launches (every row compared: the download with nothing lost), round 5, planar
  // (tools/jobs.sh decode_rule_sweep, profiles/r05/decode_rule/): R 5..8 keep the ring, which
  // runs 5-7 points ahead of the rotating triples there (RS(10,8) 104,858 B tri-X32 71.6 ->
  // ring 76.5, 1.68 MB 71.1 -> 78.3, 6.7 MB 72.1 -> 78.1); R <= 4 take the triples up to 256
  // KiB in consecutive order (RS(16,4) 64 KiB ring 78.3 -> 83.7, RS(12,4) 87,382 B 78.2 ->
  // 81.5, RS(10,4) 104,858 B 79.5 -> 82.3, RS(8,4) 128 KiB 83.1 -> 84.9) and with K > 12 above
  // it too, in Q8 to 1 MiB and X32 above (RS(16,4) 1 MiB ring 78.5 -> tri-Q8 83.3, 4 MiB 77.9
  // -> tri-X32 81.0)
  if (read_only) {
    if (R > 4) return -1;
    if (tps <= 32) return cons;
    if (K > 12) return tps <= 128 ? q8 : x32;
    // K 10..12 above 2 MiB in Q8 (RS(10,4) 6.7 MB X32 82.9 / 81.9 -> 83.9 / 83.4, RS(12,4)
    // 5.6 MB 82.3 / 81.1 -> 82.8 / 82.1)
    if (K >= 10 && tps > 256) return q8;
  }
  // R 5..8 on shards up to 256 KiB: the rotating triples in X32 for any K (round 4,
  // planar 1 MiB objects, profiles/r04/smallr8/ab.jsonl: RS(32,8)
  // 32 KiB 65.9 -> 69.3, one-block layout 66.9 -> 68.7; RS(16,8) 64 KiB 69.8 -> 73.2)
  // (round 5, planar: G2 for K <= 12 where the pitch is a multiple of 128 KiB, RS(8,8) 128 KiB
  // X32 75.4 / 75.5 -> G2 76.3 / 76.5; elsewhere X32, which leads G2 on 23 of 30 sizes from
  // 33 to 250 KB for K = 8..12 by up to 5 points, RS(10,8) 125,000 B 72.4 -> 77.5, RS(12,8)
  // 75,628 B 70.6 -> 75.9; profiles/r05/tiles/r8_small_k79_mid.jsonl)
  if (tps <= 32 && R >= 5 && !read_only) return K <= 12 && addr_tz >= 17 ? g2 : x32;
  if (K > 12) return -1;
  if (tps <= 32) return K <= 6 || R >= 5 ? x32 : -1;
  if (read_only) return x32;
  // K <= 5 above 8 MiB: X8 (profiles/r04/triord/: RS(4,2) 16 MiB
  // 71.7 -> 81.1, 32 MiB 77.5 -> 81.4, 16 MiB at a padded pitch 76.6 -> 80.4; 8 MiB X32
  // 80.9 vs X8 79.4)
  if (K <= 5) return tps > 1024 ? x8 : x32;
  if (K == 6) return tps <= 256 ? x32 : q16;
  if (pow2_16_32) return q16;
  // R 5..8 above 1 MiB (round 5, planar, profiles/r05/rule/): to 2 MiB consecutive for K < 10
  // and Q8 from K = 10 (RS(8,8) 2 MiB tri-G2 73.0 / 73.3 -> tri 74.8 / 74.3, RS(10,8) 1.68 MB
  // 74.3 -> tri-Q8 74.9), to 8 MiB X32 (RS(10,8) 6.7 MB ring G2 70.2 / 70.2 -> tri-X32 72.3,
  // RS(8,8) 8 MiB ring 72.6 = tri-X32 72.6 / 72.8)
  if (R >= 5 && tps > 128)
    return tps <= 256 ? (K < 10 ? static_cast<int>(TileOrder::kConsecutive) : q8) : tps <= 1024 ? x32 : -1;
  if (tps <= 256) return static_cast<int>(tri_order(nibble));
  return -1;
}
inline bool tri_rule(int K, int R, bool misaligned, bool verify, bool read_only, uint64_t tps,
                     int addr_tz = 0, uint64_t S = 0) {
  return tri_rule_order(K, R, misaligned, verify, read_only, tps, addr_tz, S,
                        TileOrder::kConsecutive) >= 0;
}
// Triple loads in the realigning kernel (misaligned shards, upstream Split layout):
// measured in round 4; until then only rs_plan_tune and
// rs_plan_set_orders take it.
inline bool realign_tri_rule(int K, int R, bool verify, bool read_only) {
  (void)K; (void)R; (void)verify; (void)read_only;
  return false;
}
// rs_plan_tune also times the triple form up to K = 16
// (R <= 4 launches that mix written and Verify rows take the triple loop with early
// compare loads, Policy::VPF)
inline bool tri_tunable(int K, int R, bool misaligned, bool verify, bool read_only) {
  return R <= 8 && K >= 3 && (K <= 16 || R <= 4) && !misaligned && (!verify || read_only || R <= 4);
}
// Wide groups hold 19-32 shard streams per stripe; from 2 MiB shards on, 8 interleaved
// column segments beat consecutive tiles (tools/kbench.hip KB_ORD, 9 rounds, % of
// 8 TB/s: RS(10,12) 4 MiB 60.3 -> 66.9, RS(10,16) 16 MiB 58.0 -> 66.7; at 1 MiB all
// orders are within 0.6 of each other, profiles/r01/tile_order/segments/ord_wide).
inline TileOrder wide_tile_order(uint64_t tps) {
  return tps >= 256 ? TileOrder::kSeg8 : TileOrder::kConsecutive;  // S >= 2 MiB
}

// Tile order of the v_perm kernel (k <= 3: at most 7 shard streams per stripe;
// tools/kbench.hip KB_ORD "vperm ord", 7 rounds, % of 8 TB/s,
// profiles/r01/tile_order/segments/ord_vperm): 2-stripe interleave up to 8 MiB shards
// (RS(3,2) 1 MiB 74.9 -> 77.6, 5.6 MB 75.6 -> 80.6, RS(2,1) 64 KiB 74.9 -> 78.2, RS(2,2)
// 4 MiB 75.9 -> 77.6; RS(1,1) 1 MiB 79.2 -> 78.4), 16 column segments above 8 MiB when
// the shards sit at multiples of 8 MiB (RS(3,2) 16 MiB 72.7 -> 77.7), else consecutive.
inline TileOrder vec_tile_order(uint64_t S, uint64_t tps, int addr_tz) {
  if (tps <= 1024) return TileOrder::kGroup2;
  if (addr_tz >= 23 && S < (128ull << 20)) return TileOrder::kSeg16;
  return TileOrder::kConsecutive;
}

}  // namespace callfs
