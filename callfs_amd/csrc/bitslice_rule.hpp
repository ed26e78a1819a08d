// Which launch groups run the bit-sliced kernels (rs_kernels.hip
// launch_bitslice) and in which tile order: the form rule beside tile_order.hpp's order rules.
// Plain C++: tests/native/host_test.cpp checks its choices.
#pragma once

#include <cstdint>

#include "tile_order.hpp"

namespace callfs {

// Launch groups that take the bit-sliced kernel (rs_kernels.hip launch_bitslice, DESIGN.md
// §5.7) once it is compiled, and its tile order. tps = its 8 KiB tiles per stripe.
// tools/bs_probe.py, profiles/r06/sweep1 (% of 8 TB/s, nibble rule -> bit-sliced, best order):
//  * R 9..16, every size: the nibble tables bind the LDS array there. RS(32,16) 64 KiB 55.6 ->
//    74.2 (G8), 1 MiB 55.7 -> 75.1 (G2), 4 MiB 55.7 -> 72.3 (Q8); RS(20,16) 60.3 -> 74.3,
//    RS(20,9) 58.3 -> 75.3, RS(10,16) 256 KiB 67.1 -> 73.7, RS(10,12) 1 MiB 68.4 -> 70.8;
//  * R 5..8 with K >= 20 inputs: RS(32,8) 512 KiB 69.4 -> 75.3, 2 MiB 69.6 -> 78.1 (G2); with
//    K = 16 it wins at 1 MiB (74.2 -> 78.8, profiles/r06/bs1) and loses at 256 KiB (73.4 ->
//    72.2), ties at 4 MiB; K <= 12 loses (RS(12,8) 1 MiB 76.5 -> 74.8, RS(10,8) 77.3 -> 73.1);
//  * R 5..8 with compared rows on misaligned inputs (one-shard decodes of the io.ReadAll
//    layout, rebuilt into fresh buffers): RS(10,8) 553,574 B {1} 65.1 -> 74.9, 122,190 B 66.2
//    -> 74.8, RS(8,8) 312,855 B 65.8 -> 74.3 (X32 / G8), RS(16,8) 1 MiB 73.7 -> 77.0;
//  * R <= 4: the nibble tables run at the HBM ceiling, except for K >= 24 inputs at 0.5 - 1 MiB
//    shards (G2), on two boxes: RS(32,4) 1 MiB 72.7 -> 74.7 / 72.4 -> 74.8, RS(24,4) 74.1 ->
//    75.5 / 74.0 -> 75.6 (profiles/r06/sweep1, sweep2); RS(20,4) 3.4 MB and RS(16,4) 4 MiB
//    lose 2-3 points.
//  * every read-only launch (a download's Verify with nothing lost, codec.go:59, paid on every
//    download): the bit-sliced form reads 32 B per lane per shard and compares in registers
//    at 85-91 % of 8 TB/s where the nibble rule ran 77-88 (profiles/r06/readonly*, readall_ro:
//    RS(10,4) 1 MiB 85.6 -> 89.6, RS(16,4) 83.7 -> 89.8, RS(12,8) 77.3 -> 89.8, RS(6,6) 81.8 ->
//    91.4; io.ReadAll layout RS(10,8) 553,574 B 73.0 -> 90.5, RS(4,2) 1 MiB + 1 74.4 -> 88.7).
//    Launches that write a row and compare the others keep the nibble kernels at R <= 4
//    (RS(10,4) {5} 77.6 against 72.7).
inline bool bitslice_rule(int K, int R, uint64_t tps, bool in_misaligned, bool out_misaligned,
                          bool verify, bool read_only) {
  if (R > 8 || read_only) return true;
  if (R <= 4) return K >= 24 && tps >= 64 && tps <= 128 && !verify && !in_misaligned && !out_misaligned;
  // R 5..8 launches that compare rows (one-shard decodes: a row written, the rest compared)
  // on aligned outputs, misaligned inputs or not (profiles/r06/mixed_r8, nibble rule ->
  // bit-sliced: RS(10,8) 256 KiB {1} 69.1 -> 74.6, 64 KiB 67.9 -> 72.5, RS(12,6) 1 MiB {2}
  // 71.8 -> 75.4, RS(10,8) 6.7 MB {1} 71.7 -> 73.6, RS(8,8) 8 MiB 76.7 -> 78.1; one cell
  // equal, RS(10,8) 1 MiB {0,5} 74.0 / 73.9)
  if (verify && !out_misaligned) return true;
  if (K >= 20) return true;
  return K >= 16 && tps >= 64 && tps <= 256;
}
inline TileOrder bitslice_tile_order(uint64_t tps, bool misaligned, bool verify, bool read_only) {
  if (misaligned && verify) return TileOrder::kXcd32;
  if (read_only) return TileOrder::kGroup8;  // within a point of the best order 64 KiB - 6.7 MB
  // written + compared rows: X32 up to 256 KiB and above 2 MiB, G2 between (mixed_r8: 1 MiB
  // G2 ahead of X32 by 0.7-4.3 on 4 of 5 cells; 64 KiB, 6.7 MB and 8 MiB X32 ahead by 0.4-5.6)
  if (verify) return tps <= 32 || tps > 256 ? TileOrder::kXcd32 : TileOrder::kGroup2;
  if (tps <= 32) return TileOrder::kGroup8;
  if (tps <= 256) return TileOrder::kGroup2;
  // above 2 MiB shards 16 column segments (profiles/r06/long1, % of 8 TB/s, Q8 -> Q16):
  // RS(32,16) 4 MiB 70.4 -> 72.3, 16 MiB 71.6 -> 73.3, RS(20,16) 4 MiB 68.9 -> 71.3,
  // RS(10,16) 4 MiB 70.2 -> 72.7, RS(32,8) 8 MiB 72.2 -> 73.1
  return TileOrder::kSeg16;
}

}  // namespace callfs
