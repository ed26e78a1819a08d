// Host-side C++ of the RS path under sanitizers (built by tests/test_native_host.py
// with g++ -fsanitize=address,undefined and -fsanitize=thread; no GPU needed).
//  1. GF(2^8) field + matrices (gf256.hpp) against upstream known-answer values
//  2. v_perm_b32 table packing: emulate the instruction on the CPU and check c*x for
//     every (c, x), i.e. what rs_apply.hpp's gf_mul4 computes
//  3. decode_plan rows reproduce erased shards for every 1..m erasure pattern subset
//  4. CopyPool under concurrent callers
//  5. tile orders (tile_order.hpp): every block -> (stripe, tile) map is a bijection, and
//     the launch rules pick the measured orders for known layouts
//  6. multi-device placement (dispatch.hpp) over mocked device lists: mask selection,
//     round-robin device slots, split ways and column part boundaries
//  7. per-device kernel setup (DeviceOnce): the wide kernels' dynamic-LDS opt-in is issued
//     once per (device, R), before the first such launch on each device
//  9. the tune table (tune_table.hpp): shape keys, lookup and rule fallback, replacement,
//     persistence through a file, and concurrent recording and lookups
//  8. the bit-sliced kernels' generator (bitslice_gen.hpp): the bit transpose against its
//     definition, each coefficient's GF(2) matrix against the field, the XOR network of
//     random coefficient blocks (zeros included) against a scalar GF multiply, the rule
//     and order bounds, and that the generated source declares every accumulator
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <random>
#include <cstring>
#include <thread>
#include <vector>
#include <string>
#include <unistd.h>

#include "bitslice_gen.hpp"
#include "bitslice_rule.hpp"
#include "copy_pool.hpp"
#include "dispatch.hpp"
#include "gf256.hpp"
#include "tile_order.hpp"
#include "tune_table.hpp"

using namespace callfs;

static int fails = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
      ++fails;                                                    \
    }                                                             \
  } while (0)

// ISA semantics of v_perm_b32 D = perm(S0, S1, sel), bytes of {S0,S1} (S1 low).
static uint32_t v_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t v = (static_cast<uint64_t>(s0) << 32) | s1;
  uint32_t d = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t s = (sel >> (8 * i)) & 0xff;
    uint32_t b;
    if (s >= 13) b = 0xff;
    else if (s == 12) b = 0;
    else if (s >= 8) b = 0;  // sign-extension selects: never produced by the kernel
    else b = (v >> (8 * s)) & 0xff;
    d |= b << (8 * i);
  }
  return d;
}

int main() {
  const GF& g = gf();
  CHECK(g.mul[3][4] == 12 && g.mul[7][7] == 21 && g.mul[23][45] == 41);
  CHECK(g.pow(2, 2) == 4 && g.pow(5, 20) == 235 && g.pow(13, 7) == 43 && g.pow(0, 0) == 1);
  Mat E;
  CHECK(encode_matrix(10, 4, E));
  const uint8_t row0[10] = {129, 150, 175, 184, 210, 196, 254, 232, 3, 2};
  for (int i = 0; i < 10; ++i) CHECK(E.at(10, i) == row0[i]);
  CHECK(encode_matrix(5, 5, E));
  {  // TestOneEncode RS(5,5)
    const uint8_t d[5][2] = {{0, 1}, {4, 5}, {2, 3}, {6, 7}, {8, 9}};
    const uint8_t want[5][2] = {{12, 13}, {10, 11}, {14, 15}, {90, 91}, {94, 95}};
    for (int j = 0; j < 5; ++j)
      for (int b = 0; b < 2; ++b) {
        uint8_t v = 0;
        for (int i = 0; i < 5; ++i) v ^= g.mul[E.at(5 + j, i)][d[i][b]];
        CHECK(v == want[j][b]);
      }
  }
  // 2. v_perm tables: every coefficient, every byte value, 4 lanes of a dword
  for (int c = 0; c < 256; ++c) {
    uint32_t t[kTabWords];
    perm_tables(static_cast<uint8_t>(c), t);
    for (int x0 = 0; x0 < 256; x0 += 1) {
      const uint32_t x = static_cast<uint32_t>(x0) | (static_cast<uint32_t>(255 - x0) << 8) |
                         (static_cast<uint32_t>((x0 * 7) & 255) << 16) |
                         (static_cast<uint32_t>((x0 ^ 0x5a)) << 24);
      const uint32_t i0 = x & 0x07070707u, i1 = (x >> 3) & 0x07070707u, i2 = (x >> 6) & 0x03030303u;
      const uint32_t p = v_perm(t[1], t[0], i0) ^ v_perm(t[3], t[2], i1) ^ v_perm(t[4], t[4], i2);
      for (int b = 0; b < 4; ++b)
        CHECK(((p >> (8 * b)) & 0xff) == g.mul[c][(x >> (8 * b)) & 0xff]);
    }
  }
  // 2b. LDS nibble-table kernel math (rs_apply.hpp lds_mac / lds_row) emulated on the
  // CPU: table layout, v_perm address formation (W = 8 and 16), per-position
  // accumulation and the final byte transpose, for R = 1..16 rows and K = 3 shards.
  for (int R = 1; R <= 16; ++R) {
    const int K = 3, W = nibble_width(R);
    std::mt19937 rng(R);
    std::vector<uint8_t> coef(static_cast<size_t>(K) * R);
    for (auto& c : coef) c = static_cast<uint8_t>(rng());
    std::vector<uint8_t> lds(static_cast<size_t>(K) * 32 * W);
    for (int i = 0; i < K; ++i) {
      uint8_t col[16] = {0};
      for (int r = 0; r < R; ++r) col[r] = coef[static_cast<size_t>(r) * K + i];
      nibble_tables(col, R, &lds[static_cast<size_t>(i) * 32 * W]);
    }
    for (int trial = 0; trial < 64; ++trial) {
      uint32_t x[3];
      for (auto& v : x) v = static_cast<uint32_t>(rng());
      uint8_t T[4][16] = {};  // per byte position j: products for all rows
      for (int i = 0; i < K; ++i) {
        const uint32_t base = static_cast<uint32_t>(i) * 32u * W;
        uint32_t xl, xh, base_hi;
        if (W == 8) {
          xl = (x[i] << 3) & 0x78787878u;
          xh = ((x[i] >> 1) & 0x78787878u) | 0x80808080u;
          base_hi = base;
        } else {
          xl = (x[i] << 4) & 0xf0f0f0f0u;
          xh = x[i] & 0xf0f0f0f0u;
          base_hi = base + 256u;
        }
        for (int j = 0; j < 4; ++j) {
          const uint32_t sel = 0x07060500u | static_cast<uint32_t>(j);
          const uint32_t alo = v_perm(base, xl, sel), ahi = v_perm(base_hi, xh, sel);
          for (int b = 0; b < W; ++b) T[j][b] ^= lds[alo + b] ^ lds[ahi + b];
        }
      }
      for (int r = 0; r < R; ++r) {
        // lds_row: byte r of T[0..3] via two v_perm on the dwords holding row r
        auto dw = [&](int j) {
          const int d = r >> 2;
          return static_cast<uint32_t>(T[j][4 * d]) | (static_cast<uint32_t>(T[j][4 * d + 1]) << 8) |
                 (static_cast<uint32_t>(T[j][4 * d + 2]) << 16) | (static_cast<uint32_t>(T[j][4 * d + 3]) << 24);
        };
        const int rr = r & 3;
        const uint32_t lo = v_perm(dw(1), dw(0), 0x0c0c0400u | (0x0101u * rr));
        const uint32_t hi = v_perm(dw(3), dw(2), 0x04000c0cu | (0x01010000u * rr));
        const uint32_t got = lo | hi;
        for (int j = 0; j < 4; ++j) {
          uint8_t want = 0;
          for (int i = 0; i < K; ++i)
            want ^= g.mul[coef[static_cast<size_t>(r) * K + i]][(x[i] >> (8 * j)) & 0xff];
          CHECK(((got >> (8 * j)) & 0xff) == want);
        }
      }
    }
  }
  // 3. decode rows: every erasure pattern of RS(6,3) up to 3 erasures
  {
    const int k = 6, m = 3, n = 9, S = 64;
    std::mt19937 rng(1);
    Mat E2;
    encode_matrix(k, m, E2);
    std::vector<std::vector<uint8_t>> sh(n, std::vector<uint8_t>(S));
    for (int i = 0; i < k; ++i)
      for (auto& b : sh[i]) b = rng() & 0xff;
    for (int j = 0; j < m; ++j)
      for (int b = 0; b < S; ++b) {
        uint8_t v = 0;
        for (int i = 0; i < k; ++i) v ^= g.mul[E2.at(k + j, i)][sh[i][b]];
        sh[k + j][b] = v;
      }
    int patterns = 0;
    for (int mask = 0; mask < (1 << n); ++mask) {
      if (__builtin_popcount(mask) > m) continue;
      uint8_t present[16];
      for (int i = 0; i < n; ++i) present[i] = !((mask >> i) & 1);
      DecodePlan dp;
      CHECK(decode_plan(k, m, present, dp));
      for (size_t r = 0; r < dp.missing.size() + dp.check.size(); ++r) {
        const int idx = r < dp.missing.size() ? dp.missing[r] : dp.check[r - dp.missing.size()];
        for (int b = 0; b < S; ++b) {
          uint8_t v = 0;
          for (int i = 0; i < k; ++i) v ^= g.mul[dp.rows.at(static_cast<int>(r), i)][sh[dp.valid[i]][b]];
          CHECK(v == sh[idx][b]);
        }
      }
      ++patterns;
    }
    CHECK(patterns == 1 + 9 + 36 + 84);
  }
  // 4. copy pool: 6 concurrent callers, ragged segments, tee prefixes
  {
    CopyPool pool;
    std::vector<std::thread> ts;
    std::atomic<int> bad{0};
    for (int t = 0; t < 6; ++t)
      ts.emplace_back([&, t] {
        std::mt19937 rng(100 + t);
        for (int it = 0; it < 20; ++it) {
          const size_t nseg = 1 + rng() % 7;
          std::vector<std::vector<uint8_t>> src(nseg), dst(nseg), dst2(nseg);
          std::vector<size_t> n2(nseg, 0);
          std::vector<CopyPool::Seg> segs;
          for (size_t s = 0; s < nseg; ++s) {
            const size_t len = rng() % (3u << 20);
            src[s].resize(len);
            for (size_t b = 0; b < len; b += 4093) src[s][b] = static_cast<uint8_t>(rng());
            dst[s].assign(len, 0xEE);
            // every other segment tees a prefix (decode's join) into a second buffer
            if (s % 2 && len) n2[s] = 1 + rng() % len;
            dst2[s].assign(n2[s] + 64, 0xDD);
            segs.push_back({dst[s].data(), src[s].data(), len, n2[s] ? dst2[s].data() : nullptr,
                            n2[s]});
          }
          pool.run(segs);
          for (size_t s = 0; s < nseg; ++s) {
            if (src[s] != dst[s]) bad++;
            if (std::memcmp(dst2[s].data(), src[s].data(), n2[s]) != 0) bad++;
            for (size_t b = n2[s]; b < dst2[s].size(); ++b) bad += dst2[s][b] != 0xDD;
          }
        }
      });
    for (auto& th : ts) th.join();
    CHECK(bad == 0);
  }
  // 5. tile orders
  {
    auto bijective = [](auto map, uint32_t tps, uint32_t batch) {
      std::vector<uint8_t> seen(static_cast<size_t>(tps) * batch, 0);
      for (uint32_t t = 0; t < tps * batch; ++t) {
        uint32_t stripe = ~0u, tile = ~0u;
        map(t, tps, batch, stripe, tile);
        if (stripe >= batch || tile >= tps) return false;
        uint8_t& c = seen[static_cast<size_t>(stripe) * tps + tile];
        if (c++) return false;
      }
      return true;
    };
    const uint32_t tpss[] = {1, 2, 7, 8, 13, 16, 31, 32, 33, 63, 64, 100, 128, 129, 1023,
                             1024, 1025, 1537, 2048, 2561, 4100};
    const uint32_t batches[] = {1, 2, 3, 5, 7, 8, 9, 31, 33};
    for (uint32_t tps : tpss)
      for (uint32_t b : batches) {
        CHECK(bijective(map_tile<0>, tps, b));
        CHECK(bijective(map_tile<2>, tps, b));
        CHECK(bijective(map_tile<3>, tps, b));
        CHECK(bijective(map_tile<4>, tps, b));
        CHECK(bijective(map_tile<5>, tps, b));
        CHECK(bijective(map_tile<6>, tps, b));
        CHECK(bijective(map_tile<7>, tps, b));
        CHECK(bijective(map_tile<8>, tps, b));
        CHECK(bijective(map_tile<9>, tps, b));
      }
    // XCD-grouped orders: block -> tile index is a bijection on every launch (slice) size,
    // and blocks b, b + 8 of a full group take neighbouring tiles
    auto block_bijective = [](auto fn, uint32_t nb) {
      std::vector<uint8_t> seen(nb, 0);
      for (uint32_t b = 0; b < nb; ++b) {
        const uint32_t t = fn(b, nb);
        if (t >= nb || seen[t]++) return false;
      }
      return true;
    };
    for (uint32_t nb : {1u, 7u, 8u, 63u, 64u, 65u, 255u, 256u, 257u, 1000u, 4096u, 65536u, 70001u}) {
      CHECK(block_bijective(block_tile<10>, nb));
      CHECK(block_bijective(block_tile<11>, nb));
      CHECK(block_bijective(block_tile<0>, nb));
    }
    CHECK(block_tile<10>(3, 64) == 24 && block_tile<10>(11, 64) == 25 && block_tile<10>(64, 128) == 64);
    CHECK(block_tile<11>(1, 256) == 32 && block_tile<11>(9, 256) == 33 && block_tile<11>(5, 255) == 5);
    // rules, on layouts measured in DESIGN.md §5 (tps = S / 8 KiB)
    auto tps_of = [](uint64_t S) { return (S / 16 + 511) / 512; };
    const uint64_t MiB = 1ull << 20;
    // bench shape RS(10,4) 1 MiB, contiguous stripes 14 MiB apart: G2
    CHECK(lds_tile_order(MiB, tps_of(MiB), 20, 14, 14 * MiB) == TileOrder::kGroup2);
    // 64 MiB objects, S = 6,710,887 (pitch 2^8 * odd), 14 streams: G2
    CHECK(lds_tile_order(6710887, tps_of(6710887), 8, 14, 14 * 6711040ull) == TileOrder::kGroup2);
    // decodes with Verify rows: consecutive from 1 to 8 MiB, G2 up to 1 MiB
    CHECK(lds_tile_order(6710887, tps_of(6710887), 8, 14, 14 * 6711040ull, true) == TileOrder::kConsecutive);
    CHECK(lds_tile_order(MiB, tps_of(MiB), 20, 14, 14 * MiB, true) == TileOrder::kGroup2);
    // read-only (every row compared: the download with nothing lost) above 256 KiB: X32
    CHECK(lds_tile_order(MiB, tps_of(MiB), 20, 14, 14 * MiB, true, true) == TileOrder::kXcd32);
    CHECK(lds_tile_order(6710887, tps_of(6710887), 8, 14, 14 * 6711040ull, true, true) == TileOrder::kXcd32);
    CHECK(lds_tile_order(104858, tps_of(104858), 8, 14, 14 * 105216ull, true, true, 4) == TileOrder::kGroup8);
    // RS(4,2) 4 MiB: consecutive (few streams); RS(12,8) 4 MiB: G2; RS(16,4) 4 MiB:
    // consecutive (round 4: G2 above 1 MiB only for 5-8 rows)
    CHECK(lds_tile_order(4 * MiB, tps_of(4 * MiB), 22, 6, 24 * MiB) == TileOrder::kConsecutive);
    CHECK(lds_tile_order(4 * MiB, tps_of(4 * MiB), 22, 20, 80 * MiB) == TileOrder::kGroup2);
    CHECK(lds_tile_order(4 * MiB, tps_of(4 * MiB), 22, 20, 80 * MiB, false, false, 4) ==
          TileOrder::kConsecutive);
    // (round 5: more than 12 inputs with R <= 4 up to 1 MiB run the ring in consecutive order)
    CHECK(lds_tile_order(MiB, tps_of(MiB), 20, 20, 20 * MiB, false, false, 4) == TileOrder::kConsecutive);
    CHECK(lds_tile_order(MiB, tps_of(MiB), 20, 16, 16 * MiB, false, false, 4) == TileOrder::kGroup2);
    // power-of-two 16 MiB shards: Q16 with 14 streams, consecutive with 6
    CHECK(lds_tile_order(16 * MiB, tps_of(16 * MiB), 24, 14, 224 * MiB) == TileOrder::kSeg16);
    CHECK(lds_tile_order(16 * MiB, tps_of(16 * MiB), 24, 6, 96 * MiB) == TileOrder::kConsecutive);
    // 64 MiB shards, 14 streams: Q8; 1 GiB column slices (pitch 2^8 * odd): consecutive
    CHECK(lds_tile_order(64 * MiB, tps_of(64 * MiB), 26, 14, 0) == TileOrder::kSeg8);
    CHECK(lds_tile_order(13421824, tps_of(13421824), 10, 14, 0) == TileOrder::kConsecutive);
    // small shards: G8, unless stripes sit exactly 2 MiB (consecutive) or 1 MiB (G2) apart
    CHECK(lds_tile_order(256 << 10, tps_of(256 << 10), 18, 14, 3584 << 10) == TileOrder::kGroup8);
    CHECK(lds_tile_order(128 << 10, tps_of(128 << 10), 17, 16, 2 * MiB) == TileOrder::kConsecutive);
    CHECK(lds_tile_order(128 << 10, tps_of(128 << 10), 17, 8, 1 * MiB) == TileOrder::kGroup2);
    // wide groups: Q8 from 2 MiB; v_perm kernel: G2 up to 8 MiB, Q16 for aligned 16 MiB
    CHECK(wide_tile_order(tps_of(4 * MiB)) == TileOrder::kSeg8);
    CHECK(wide_tile_order(tps_of(MiB)) == TileOrder::kConsecutive);
    CHECK(vec_tile_order(349526, tps_of(349526), 8) == TileOrder::kGroup2);
    CHECK(vec_tile_order(16 * MiB, tps_of(16 * MiB), 24) == TileOrder::kSeg16);
    CHECK(vec_tile_order(107374183, tps_of(107374183), 8) == TileOrder::kConsecutive);
    // triple loads (tri_rule_order): aligned R <= 8 launches with 4..12 inputs that write
    // every row or compare every row; round 3's bounds (shards up to 2 MiB, 4 MiB with
    // K <= 6) in the nibble rule's order, and since round 4 K <= 4 at any size in X32, K 5..6
    // in X32 / Q16, K 7..12 on 16-32 MiB power-of-two pitches in Q16
    const uint64_t t1 = tps_of(MiB);
    const int X32 = static_cast<int>(TileOrder::kXcd32), Q16 = static_cast<int>(TileOrder::kSeg16),
              G2 = static_cast<int>(TileOrder::kGroup2);
    auto tro = [](int K, int R, uint64_t S, int tz, bool verify = false, bool ro = false,
                  TileOrder nib = TileOrder::kGroup2) {
      return tri_rule_order(K, R, false, verify, ro, (S / 16 + 511) / 512, tz, S, nib);
    };
    CHECK(tri_rule(4, 2, false, false, false, t1));   // CallFS default RS(4,2) encode
    CHECK(tri_rule(10, 4, false, false, false, t1));  // the bench shape
    CHECK(tri_rule(8, 8, false, false, false, t1));   // 8-byte entries too
    CHECK(tri_rule(4, 2, false, true, true, t1));     // download Verify (read-only)
    CHECK(!tri_rule(3, 2, false, false, false, t1));  // k = 3: the v_perm kernel
    CHECK(tri_rule(12, 4, false, false, false, t1));
    CHECK(tri_rule(16, 4, false, false, false, t1, 20));  // double-buffered from K = 6 at R <= 4
    CHECK(!tri_rule(16, 4, false, false, false, tps_of(1000000), 8));  // ... the ring off 128 KiB pitches
    CHECK(!tri_rule(16, 8, false, false, false, t1)); // rotating form: K <= 12
    CHECK(tri_rule(32, 8, false, false, false, tps_of(32768)));   // ... any K up to 256 KiB
    CHECK(tri_rule(16, 8, false, false, false, tps_of(65536)));
    CHECK(!tri_rule(4, 2, true, false, false, t1));   // Split layout: realigning kernel
    CHECK(tri_rule(6, 3, false, true, false, t1));    // written + Verify rows: early compares
    CHECK(!tri_rule(6, 6, false, true, false, t1));   // ... at R <= 4 only
    CHECK(!tri_rule(10, 9, false, false, false, t1)); // 16-byte entries
    CHECK(tri_rule(8, 8, false, false, false, tps_of(8 * MiB), 23));  // 8 MiB, R = 8: X32 (round 5)
    CHECK(tri_rule(8, 4, false, false, false, tps_of(2 * MiB)));      // 2 MiB: gained
    CHECK(tri_rule(4, 2, false, false, false, tps_of(256 << 10)));    // small S, few inputs
    CHECK(tri_rule(10, 4, false, false, false, tps_of(104858)));      // small S, double-buffered
    CHECK(tri_rule(10, 8, false, false, false, tps_of(104858)));      // small S, R = 8
    CHECK(!tri_rule(10, 4, false, false, false, tps_of(4 * MiB), 22)); // K >= 10 above 1 MiB: ring
    CHECK(!tri_rule(10, 4, false, false, false, tps_of(6710887), 8));  // configs[2] shards: ring
    CHECK(!tri_rule(8, 4, false, false, false, tps_of(6710887), 8));   // K 7..9 above 2 MiB: ring
    CHECK(!tri_rule(16, 4, false, false, false, tps_of(4 * MiB)));    // K > 12 above 2 MiB
    // round 4: K <= 5 in X32 up to 8 MiB (RS(4,2) 8 MiB 70.0 -> 79.6), X8 above (16 MiB
    // 71.7 -> 81.1, 32 MiB 77.5 -> 81.4)
    const int X8 = static_cast<int>(TileOrder::kXcd8);
    CHECK(tro(4, 2, MiB, 20) == X32 && tro(4, 2, 8 * MiB, 23) == X32 && tro(4, 2, 5592406, 8) == X32);
    CHECK(tro(4, 2, 16 * MiB, 24) == X8 && tro(4, 2, 64 * MiB, 26) == X8 && tro(5, 3, 16 * MiB, 24) == X8);
    // K 5..6: X32 up to 2 MiB, Q16 above (RS(6,3) 4 MiB 71.7 -> 77.3, 16 MiB 73.2 -> 76.5)
    CHECK(tro(6, 3, MiB, 20) == X32 && tro(6, 3, 2796203, 8) == X32 && tro(6, 3, 16 * MiB, 24) == X8);
    CHECK(tro(6, 6, 2796203, 8) == Q16);  // R 5..8: the rotating form's K = 6 rule
    CHECK(tro(10, 4, 104858, 8) == X32 && tro(10, 4, 1677722, 8) == -1 && tro(10, 4, 2 * MiB, 21) == -1);
    // round 5, planar layout: K 7..9 in G2 to 2 MiB, the ring to 8 MiB; R 5..8: G2 to
    // 256 KiB (K <= 12), consecutive / Q8 to 2 MiB, X32 to 8 MiB
    const int Q8 = static_cast<int>(TileOrder::kSeg8), CONS = static_cast<int>(TileOrder::kConsecutive);
    CHECK(tro(8, 4, 2 * MiB, 21) == G2 && tro(8, 4, 8 * MiB, 23) == -1);
    CHECK(tro(8, 4, 4389515, 8) == Q8 && tro(7, 4, 2500000, 8) == Q8 && tro(9, 4, 7500000, 8) == -1);
    CHECK(tro(10, 8, 75628, 8) == X32 && tro(12, 8, 125000, 8) == X32);
    CHECK(tro(8, 8, 131072, 17) == G2 && tro(32, 8, 32768, 15) == X32 && tro(8, 8, 2 * MiB, 21) == CONS);
    CHECK(tro(10, 8, 1677722, 8) == Q8 && tro(10, 8, 6710887, 8) == X32 && tro(8, 8, 8 * MiB, 23) == X32);
    CHECK(tro(10, 8, 16 * MiB, 8) == -1);
    CHECK(lds_tile_order(838861, tps_of(838861), 8, 24, 0, false, false, 4) == TileOrder::kConsecutive);
    CHECK(lds_tile_order(2 * MiB, tps_of(2 * MiB), 21, 40, 0, false, false, 8) == TileOrder::kConsecutive);
    CHECK(lds_tile_order(524288, tps_of(524288), 19, 40, 0, false, false, 8) == TileOrder::kGroup2);
    // K 7..12: Q16 on 16-32 MiB power-of-two pitches, round 3's rule elsewhere
    CHECK(tro(10, 4, 16 * MiB, 24) == Q16 && tro(12, 4, 32 * MiB, 25) == Q16);
    CHECK(tro(10, 4, 16 * MiB, 8) == -1 && tro(10, 4, 64 * MiB, 26) == -1);
    CHECK(tro(10, 4, MiB, 20) == G2);  // the nibble rule's order (G2 for the bench shape)
    // K > 16 from 256 KiB to 1 MiB: the ring on unaligned pitches, G2 on 64 KiB-aligned ones
    CHECK(tro(20, 4, 838861, 8) == -1 && tro(20, 4, MiB, 20) == G2 && tro(16, 4, 838861, 8) == -1);
    // 256 KiB - 1 MiB off 128 KiB-multiple pitches: X32 for K <= 12 (round 5, mid_band.jsonl)
    CHECK(tro(8, 4, 464531, 8) == X32 && tro(10, 4, 655000, 8) == X32 && tro(12, 4, 720000, 8) == X32);
    CHECK(tro(8, 4, 524288, 19) == G2 && tro(12, 4, 524288, 19) == G2);
    CHECK(tro(16, 4, 65536, 16) == X32 && tro(20, 4, 65536, 16) == X32);
    // up to 256 KiB, K > 12 on shards that are not a power of two: the ring (round 5,
    // profiles/r05/tiles/)
    CHECK(tro(20, 4, 52429, 8) == -1 && tro(24, 4, 57344, 13) == -1 && tro(16, 4, 40960, 13) == -1);
    CHECK(tro(16, 4, 196608, 16) == -1 && tro(32, 4, 32768, 15) == X32 && tro(20, 4, 131072, 17) == -1);
    CHECK(tro(8, 4, 131072, 17) == X32);  // K <= 12 keep the triples
    CHECK(tro(12, 4, 87382, 8) == X32 && tro(10, 4, 57344, 13) == X32);
    CHECK(lds_tile_order(52429, tps_of(52429), 8, 24, 0, false, false, 4) == TileOrder::kConsecutive);
    CHECK(lds_tile_order(65536, tps_of(65536), 16, 20, 0, false, false, 4) == TileOrder::kConsecutive);
    CHECK(lds_tile_order(65536, tps_of(65536), 16, 16, 0, false, false, 4) == TileOrder::kGroup8);
    // read-only launches: X32 at every size above 256 KiB (RS(6,3) 16 MiB 85.7 -> 90.0)
    CHECK(tro(4, 2, 16 * MiB, 24, true, true) == X32 && tro(10, 4, MiB, 20, true, true, TileOrder::kXcd32) == X32);
    // written + Verify rows (R <= 4, early compares): K <= 4 in X32, K 5..12 up to 1 MiB
    CHECK(tro(4, 2, MiB, 20, true, false) == X32 && tro(4, 2, 4 * MiB, 22, true, false) == X32);
    CHECK(tro(10, 4, MiB, 20, true, false) == G2 && tro(10, 4, 6710887, 8, true, false) == X32);
    CHECK(tro(5, 3, 6710887, 8, true, false) == -1 && tro(20, 4, MiB, 20, true, false) == -1);
    CHECK(tro(10, 4, 104858, 8, true, false) == G2 && tro(6, 3, 174763, 8, true, false) == X32);
    CHECK(tro(10, 4, 75550, 8, true, false) == X32 && tro(16, 4, 60287, 8, true, false) == X32);
    // round 5, planar: mixed decodes up to 256 KiB in G2 for K >= 7; read-only launches: R 5..8
    // keep the ring (consecutive up to 256 KiB), R <= 4 take consecutive triples up to 256 KiB
    // and, with K > 12, Q8 to 1 MiB and X32 above
    CHECK(tro(16, 4, 65536, 16, true, false) == X32 && tro(20, 4, MiB, 20, true, false) == -1);
    CHECK(tro(10, 8, 104858, 8, true, true) == -1 && tro(10, 8, 1677722, 8, true, true) == -1);
    CHECK(tro(10, 4, 104858, 8, true, true) == CONS && tro(16, 4, 65536, 16, true, true) == CONS);
    CHECK(tro(16, 4, MiB, 20, true, true) == Q8 && tro(16, 4, 4 * MiB, 22, true, true) == X32);
    CHECK(tro(10, 4, 1677722, 8, true, true) == X32 && tro(10, 4, 6710887, 8, true, true) == Q8);
    CHECK(tro(10, 4, 1677722, 8, true, false) == G2 && tro(12, 4, 5592406, 8, true, false) == X32);
    CHECK(tro(16, 4, 832781, 8, true, false) == X32 && tro(6, 3, 413283, 8, true, false) == X32);
    CHECK(lds_tile_order(104858, tps_of(104858), 8, 18, 0, true, true, 8) == TileOrder::kConsecutive);
    CHECK(tri_tunable(16, 4, false, false, false) && tri_tunable(20, 4, false, false, false) &&
          !tri_tunable(20, 8, false, false, false));  // R <= 4: the double-buffered form at any K
    CHECK(tri_order(TileOrder::kGroup8) == TileOrder::kXcd32);
    CHECK(tri_order(TileOrder::kGroup2) == TileOrder::kGroup2);
    CHECK(tri_order(TileOrder::kConsecutive) == TileOrder::kConsecutive);
    CHECK(tri_order(TileOrder::kSeg16) == TileOrder::kSeg16 && tri_order(TileOrder::kXcd8) == TileOrder::kXcd8);
  }
  // 6. multi-device placement (dispatch.hpp), mocked device counts
  {
    // rs_init's mask: 0 = all, bit d = device d, bits beyond the visible count ignored
    CHECK((select_devices(8, 0) == std::vector<int>{0, 1, 2, 3, 4, 5, 6, 7}));
    CHECK((select_devices(8, 0x81u) == std::vector<int>{0, 7}));
    CHECK((select_devices(2, 0xFCu).empty()));
    CHECK((select_devices(40, 0).size() == 32));
    CHECK((select_devices(1, 1u) == std::vector<int>{0}));
    // round robin: consecutive tickets walk the devices; parts of one call start at the
    // call's device and take consecutive ones
    for (size_t nd : {1u, 2u, 3u, 8u}) {
      std::vector<int> hits(nd, 0);
      for (unsigned t = 0; t < 8 * nd; ++t) hits[device_slot(t, 0, nd)]++;
      for (size_t d = 0; d < nd; ++d) CHECK(hits[d] == 8);
      for (int p = 0; p < 8; ++p) CHECK(device_slot(5, p, nd) == (5 + static_cast<size_t>(p)) % nd);
    }
    CHECK(device_slot(~0u, 1, 8) == (static_cast<size_t>(~0u) + 1) % 8);  // ticket wrap
    // split ways: single-stripe calls of >= min bytes, one way per device by default,
    // capped by lanes and by 4 MiB of columns per way
    const unsigned long long min_b = 256ull << 20;
    const size_t S1g = 107374183;  // 1 GiB RS(10,4)
    CHECK(split_ways(8, 8, S1g, 14, 1, min_b, 0) == 8);
    CHECK(split_ways(1, 8, S1g, 14, 1, min_b, 0) == 1);
    CHECK(split_ways(8, 8, S1g, 14, 2, min_b, 0) == 1);          // batches never split
    CHECK(split_ways(8, 8, 1 << 20, 14, 1, min_b, 0) == 1);      // 14 MiB < 256 MiB
    CHECK(split_ways(2, 8, S1g, 14, 1, min_b, 5) == 5);          // explicit ways
    CHECK(split_ways(1, 8, S1g, 14, 1, min_b, 100) == 8);        // lane cap
    CHECK(split_ways(8, 8, 20u << 20, 14, 1, 1u << 20, 64) == 5);  // 4 MiB per way
    CHECK(split_ways(0, 8, S1g, 14, 1, min_b, 0) == 1);
    // column parts: cover [0, S) exactly, interior boundaries 4 KiB aligned, in order
    for (size_t S : {S1g, static_cast<size_t>(13000002), static_cast<size_t>(4096 * 8 + 5)})
      for (int w : {1, 2, 3, 5, 8}) {
        const std::vector<size_t> c = column_parts(S, w);
        CHECK(c.size() == static_cast<size_t>(w) + 1 && c.front() == 0 && c.back() == S);
        for (int p = 1; p <= w; ++p) CHECK(c[p] >= c[p - 1]);
        for (int p = 1; p < w; ++p) CHECK(c[p] % 4096 == 0 || c[p] == S);
      }
    // the 8-way split of a 1 GiB object over 8 devices: one part per device, each a
    // nonempty column range of about S/8
    const std::vector<size_t> c8 = column_parts(S1g, 8);
    for (int p = 0; p < 8; ++p) {
      const size_t w = c8[p + 1] - c8[p];
      CHECK(w > 0 && w <= S1g / 8 + 4096);
      CHECK(device_slot(0, p, 8) == static_cast<size_t>(p));
    }
    // CALLFS_RS_SPLIT_WAYS: unset = one per device; explicit <= 1 keeps one device
    CHECK(split_ways_request(nullptr) == 0);
    CHECK(split_ways_request("0") == 1 && split_ways_request("-3") == 1);
    CHECK(split_ways_request("1") == 1 && split_ways_request("x") == 1);
    CHECK(split_ways_request("5") == 5);
    CHECK(split_ways(8, 8, S1g, 14, 1, min_b, split_ways_request("0")) == 1);
    CHECK(split_ways(8, 8, S1g, 14, 1, min_b, split_ways_request(nullptr)) == 8);
  }
  // 7. per-device kernel setup (the wide kernels' > 64 KiB dynamic-LDS opt-in is a
  // per-device attribute): launch_apply issues it once per (device, R) before the first
  // such launch on a device -- every device of a mocked 8-device context gets it before its
  // first launch whatever the launch order, exactly once, with the device current; other
  // keys and devices stay untouched; concurrent first launches issue it once
  {
    for (unsigned mask : {0u, 0x81u, 0x0Eu}) {
      DeviceOnce once;
      const std::vector<int> devs = select_devices(8, mask);
      std::vector<std::vector<int>> issued(8, std::vector<int>(8, 0));  // [device][R - 9]
      int current = -1;
      auto launch = [&](int d, int R) {  // what launch_apply does for a wide launch on d
        current = d;
        once.run(d, R - 9, [&] {
          CHECK(current == d);
          issued[d][R - 9]++;
        });
        CHECK(once.done(d, R - 9));  // issued before the launch proceeds
      };
      for (int rep = 0; rep < 3; ++rep)
        for (size_t j = 0; j < devs.size(); ++j) {
          const int d = devs[(j * 5 + rep) % devs.size()];  // scrambled device order
          for (int R : {16, 9, 12}) launch(d, R);
        }
      for (int d = 0; d < 8; ++d) {
        const bool sel = std::find(devs.begin(), devs.end(), d) != devs.end();
        for (int R = 9; R <= 16; ++R) {
          const bool used = sel && (R == 16 || R == 9 || R == 12);
          CHECK(issued[d][R - 9] == (used ? 1 : 0));
          CHECK(once.done(d, R - 9) == used);
        }
      }
    }
    // concurrent first use of one (device, key): one call
    DeviceOnce once2;
    std::atomic<int> calls{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&] {
        for (int d = 0; d < 8; ++d) once2.run(d, 2, [&] { calls++; });
      });
    for (auto& t : th) t.join();
    CHECK(calls.load() == 8);
    // out-of-range devices / keys run every time (never silently skipped)
    int n = 0;
    once2.run(40, 0, [&] { n++; });
    once2.run(40, 0, [&] { n++; });
    once2.run(0, 70, [&] { n++; });
    CHECK(n == 3);
  }
  // 8. bit-sliced kernels (bitslice_gen.hpp)
  {
    std::mt19937 rng(0xB175);
    // tr8: bit i of byte p of out[k] == bit k of byte p of in[i]; an involution
    for (int t = 0; t < 64; ++t) {
      uint32_t in[8], d[8];
      for (int i = 0; i < 8; ++i) in[i] = d[i] = rng();
      bs::tr8(d);
      bool ok = true;
      for (int k = 0; k < 8; ++k)
        for (int i = 0; i < 8; ++i)
          for (int p = 0; p < 4; ++p)
            ok &= ((d[k] >> (8 * p + i)) & 1u) == ((in[i] >> (8 * p + k)) & 1u);
      CHECK(ok);
      bs::tr8(d);
      CHECK(std::equal(d, d + 8, in));
    }
    // M_c: c*x == XOR over set bits j of x of column j, for every (c, x)
    {
      const GF& g = gf();
      bool ok = true;
      for (int c = 0; c < 256; ++c) {
        uint8_t rows[8];
        bs::mul_matrix(static_cast<uint8_t>(c), rows);
        for (int x = 0; x < 256; ++x) {
          uint8_t y = 0;
          for (int k = 0; k < 8; ++k)
            y |= static_cast<uint8_t>((__builtin_popcount(rows[k] & x) & 1) << k);
          ok &= y == g.mul[c][x];
        }
      }
      CHECK(ok);
    }
    // the network: random blocks (a third of the coefficients zero), 32 random bytes per
    // input and lane, against the scalar multiply byte by byte
    const GF& g = gf();
    for (int t = 0; t < 40; ++t) {
      const int K = 1 + static_cast<int>(rng() % 40), R = 1 + static_cast<int>(rng() % 16);
      std::vector<uint8_t> coef(static_cast<size_t>(K) * R);
      for (auto& c : coef) c = rng() % 3 == 0 ? 0 : static_cast<uint8_t>(rng());
      const bs::Network net = bs::build_network(K, R, coef.data());
      std::vector<std::array<uint32_t, 8>> in(K), out;
      for (auto& v : in)
        for (auto& w : v) w = rng();
      bs::evaluate(net, in, out);
      bool ok = static_cast<int>(out.size()) == R;
      for (int r = 0; r < R && ok; ++r)
        for (int w = 0; w < 8; ++w)
          for (int p = 0; p < 4; ++p) {
            uint8_t want = 0;
            for (int i = 0; i < K; ++i)
              want ^= g.mul[coef[static_cast<size_t>(r) * K + i]][(in[i][w] >> (8 * p)) & 0xffu];
            ok &= ((out[r][w] >> (8 * p)) & 0xffu) == want;
          }
      CHECK(ok);
      // the generated kernel: every used accumulator declared, one pin per shard group
      const std::string src = bs::kernel_source(net, "rs_bs", bs::GenOptions{}, 56);
      CHECK(src.find("void rs_bs(const Args a)") != std::string::npos);
      CHECK(src.find("static_assert(sizeof(Args) == 56") != std::string::npos);
      for (int r = 0; r < R; ++r) {
        char nm[32];
        std::snprintf(nm, sizeof nm, " a%d_7", r);
        CHECK(src.find(nm) != std::string::npos);
      }
    }
    // the rule: every wide group; R 5..8 for many inputs or misaligned one-shard decodes;
    // never R <= 4 or read-only launches; orders by tiles per stripe
    CHECK(bitslice_rule(10, 9, 128, false, false, false, false));
    CHECK(bitslice_rule(2, 16, 1, true, true, true, true));
    CHECK(bitslice_rule(32, 8, 256, false, false, false, false));
    CHECK(!bitslice_rule(10, 8, 128, false, false, false, false));
    CHECK(bitslice_rule(10, 8, 68, true, false, true, false));
    CHECK(!bitslice_rule(10, 8, 68, true, true, true, false));  // misaligned outputs: nibble
    CHECK(bitslice_rule(10, 8, 128, false, false, true, false));  // aligned mixed R 5..8
    CHECK(bitslice_tile_order(128, false, true, false) == TileOrder::kGroup2);
    CHECK(bitslice_tile_order(8, false, true, false) == TileOrder::kXcd32);
    CHECK(bitslice_tile_order(820, false, true, false) == TileOrder::kXcd32);
    CHECK(bitslice_rule(10, 8, 68, true, false, true, true));   // read-only: every R
    CHECK(bitslice_rule(10, 4, 128, false, false, true, true));
    CHECK(!bitslice_rule(10, 4, 128, false, false, true, false));  // mixed R <= 4: nibble
    CHECK(bitslice_rule(32, 4, 128, false, false, false, false));
    CHECK(!bitslice_rule(32, 4, 256, false, false, false, false));
    CHECK(!bitslice_rule(16, 4, 128, false, false, false, false));
    CHECK(!bitslice_rule(10, 4, 128, false, false, false, false));
    CHECK(bitslice_rule(16, 8, 128, false, false, false, false));
    CHECK(!bitslice_rule(16, 8, 32, false, false, false, false));
    CHECK(bitslice_tile_order(8, false, false, false) == TileOrder::kGroup8);
    CHECK(bitslice_tile_order(128, false, false, false) == TileOrder::kGroup2);
    CHECK(bitslice_tile_order(512, false, false, false) == TileOrder::kSeg16);
    CHECK(bitslice_tile_order(256, false, false, false) == TileOrder::kGroup2);
    CHECK(bitslice_tile_order(512, true, true, false) == TileOrder::kXcd32);
    CHECK(bitslice_tile_order(512, false, true, true) == TileOrder::kGroup8);
    CHECK(bitslice_tile_order(512, true, true, true) == TileOrder::kXcd32);
  }

  // 9. the tune table
  {
    TuneTable t;
    char path[] = "/tmp/callfs_tune_XXXXXX";
    const int fd = mkstemp(path);
    CHECK(fd >= 0);
    if (fd >= 0) close(fd);
    t.reset(path);
    // keys: tiles per stripe bucketed by powers of two, alignment classes by addr_tz
    const TuneKey a = tune_key(0, 10, 4, 128, 20, false, false, false, false);
    CHECK(a.tps_log2 == 7 && a.align == 0 && a.kind == 0 && a.mis == 0);
    CHECK(tune_key(0, 10, 4, 255, 20, false, false, false, false).packed() == a.packed());
    CHECK(tune_key(0, 10, 4, 256, 20, false, false, false, false).packed() != a.packed());
    CHECK(tune_key(0, 10, 4, 128, 10, false, false, false, false).align == 1);
    CHECK(tune_key(0, 10, 4, 128, 4, true, false, true, false).packed() != a.packed());
    CHECK(tune_key(1, 10, 4, 128, 20, false, false, false, false).packed() != a.packed());
    CHECK(tune_key(0, 10, 4, 128, 20, true, true, false, true).kind == 2);
    CHECK(tune_key(0, 10, 4, 128, 20, true, true, false, true).mis == 2);
    CHECK(tune_key(0, 10, 4, 0, 20, false, false, false, false).tps_log2 == 0);
    // empty: every lookup falls back to the rule (-1)
    CHECK(t.empty() && t.lookup(a) == -1);
    t.record(a, 98);
    t.record(a, -1);  // no choice: ignored
    CHECK(t.lookup(a) == 98 && t.size() == 1);
    t.record(a, 258);  // a later tune replaces it
    CHECK(t.lookup(a) == 258 && t.size() == 1);
    const TuneKey b = tune_key(0, 32, 16, 8, 63, true, false, true, false);
    t.record(b, 257);
    CHECK(t.lookup(b) == 257 && t.lookup(a) == 258 && t.size() == 2);
    // persistence: a new table bound to the same file reads both entries back
    TuneTable u;
    u.reset(path);
    CHECK(u.size() == 2 && u.lookup(a) == 258 && u.lookup(b) == 257);
    // two processes' tables on one file: each rewrite keeps the entries the other recorded
    const TuneKey c = tune_key(0, 6, 3, 64, 20, false, false, false, false);
    const TuneKey d = tune_key(0, 8, 4, 64, 20, false, false, false, false);
    u.record(c, 3);        // u read the file before t recorded d
    t.record(d, 5);        // t's rewrite merges u's c
    CHECK(t.lookup(c) == 3 && t.lookup(d) == 5);
    u.record(a, 96);       // u's own newer choice for a wins over the file's 258
    TuneTable v;
    v.reset(path);
    CHECK(v.size() == 4 && v.lookup(a) == 96 && v.lookup(b) == 257 && v.lookup(c) == 3 &&
          v.lookup(d) == 5);
    // an entry a table only read is not written back over a newer one: u read b = 257 and
    // never recorded it; v re-tunes b, and u's next rewrite (for another key) keeps v's 99
    v.record(b, 99);
    u.record(tune_key(0, 5, 2, 64, 20, false, false, false, false), 1);
    TuneTable w;
    w.reset(path);
    CHECK(w.lookup(b) == 99 && w.size() == 5);
    u.reset(nullptr);  // memory only (CALLFS_RS_TUNE_TABLE unset in this test)
    CHECK(u.empty());
    // concurrent tuners and launches
    std::vector<std::thread> ths;
    for (int w = 0; w < 4; ++w)
      ths.emplace_back([&t, w] {
        for (int i = 0; i < 200; ++i) {
          const TuneKey k = tune_key(w, 4 + i % 20, 1 + i % 16, 1u << (i % 12), i % 24, i & 1,
                                     false, i & 2, false);
          t.record(k, i % 7);
          (void)t.lookup(k);
        }
      });
    for (auto& x : ths) x.join();
    CHECK(t.size() > 2);
    std::remove(path);
  }

  std::printf(fails ? "FAILED %d\n" : "host_test ok\n", fails);
  return fails ? 1 : 0;
}
