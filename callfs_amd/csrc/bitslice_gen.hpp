// Source generator of the bit-sliced GF(2^8) kernels: one straight-line
// HIP kernel per coefficient block, compiled at plan time by hiprtc (bitslice.cpp).
//
// Why: a launch group of R rows over K inputs is, over GF(2), an (8R x 8K) bit matrix. The
// LDS nibble-table kernel (rs_apply.hpp) reads 2R bytes of table per input byte, which
// binds the LDS array once R > 8. Here the matrix is baked into the code:
//  * each lane owns 32 column bytes of a stripe (two 16-B vectors 1 KiB apart, so a wave
//    still loads whole 1 KiB windows) and transposes the 8 dwords of every input shard
//    into 8 bit planes (plane j = bit j of the 32 bytes; 3 stages of masked swaps, tr8);
//  * multiplying by a plan-time constant c is the 8x8 GF(2) matrix M_c (column j =
//    c * 2^j): output plane k of a row gets the XOR of the input planes j with
//    M_c[k][j] = 1. Four Russians: the XORs of planes 0..3 (L[s], s = 1..15) and of
//    planes 4..7 (H[s]) are formed once per shard, so each (row, output plane) costs one
//    v_bitop3 XOR3: acc ^= L[row k & 15] ^ H[row k >> 4] -- 8 VALU per (shard, row) per
//    32 bytes, 0.25 VALU per byte per row, against 2R LDS bytes per byte for the tables;
//  * the R rows' 8 accumulator planes are transposed back and stored (or, for Verify
//    rows, compared) once.
// Plain C++ (no HIP): tests/native/host_test.cpp runs `evaluate`, the same network on the
// host, against a scalar GF multiply, and checks tr8 against its definition.
#pragma once

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "gf256.hpp"

namespace callfs {
namespace bs {

// Rows per launch group the generator accepts (kMaxRowsPerLaunch) and input shards.
constexpr int kMaxRows = 16;
constexpr int kMaxInputs = 256;
// 16-B vectors per wave-tile: lane l owns vectors base + l and base + 64 + l
constexpr int kWaveVecs = 128;
constexpr int kBlockThreads = 256;  // default block (GenOptions::block)
constexpr int kTileVecs = kWaveVecs * (kBlockThreads / 64);  // 512 vectors = 8 KiB per shard

// Kernel arguments. The generated source declares the same struct (kArgsDecl); bitslice.cpp
// static_asserts the host layout and the source checks sizeof.
struct Args {
  const uint8_t* const* in_tab;  // [batch][K] input shard pointers
  uint8_t* const* out_tab;       // [batch][R] output (written or compared) shard pointers
  int* status;                   // stripe b ORs 1 into status[b * status_stride] on a mismatch
  uint64_t nvec;                 // 16-B vectors per shard the kernel covers (S / 16)
  uint32_t tps;                  // tiles per stripe: ceil(nvec / kTileVecs)
  uint32_t ntiles;               // tps * batch
  uint32_t t_base;               // first tile of this dispatch (sliced grids)
  uint32_t verify_mask;          // bit r: compare row r instead of storing it
  int status_stride;
  int order;                     // tile order: 0 consecutive, 1 Q8, 2 X32, 3 G2, 4 X8, 5 G8, 6 Q16
};

inline const char* args_decl() {
  return "struct Args {\n"
         "  const unsigned char* const* in_tab;\n"
         "  unsigned char* const* out_tab;\n"
         "  int* status;\n"
         "  unsigned long long nvec;\n"
         "  unsigned int tps;\n"
         "  unsigned int ntiles;\n"
         "  unsigned int t_base;\n"
         "  unsigned int verify_mask;\n"
         "  int status_stride;\n"
         "  int order;\n"
         "};\n";
}

// Rows of the GF(2) matrix of x -> c*x: bit j of rows[k] = bit k of c * 2^j.
inline void mul_matrix(uint8_t c, uint8_t rows[8]) {
  const GF& g = gf();
  for (int k = 0; k < 8; ++k) rows[k] = 0;
  for (int j = 0; j < 8; ++j) {
    const uint8_t col = g.mul[c][1u << j];
    for (int k = 0; k < 8; ++k)
      if ((col >> k) & 1u) rows[k] |= static_cast<uint8_t>(1u << j);
  }
}

// The 8x8 bit transpose of every byte position of 8 dwords (an involution): afterwards bit
// i of byte p of d[k] is bit k of byte p of the input d[i]. Host copy of the device tr8.
inline void tr8(uint32_t d[8]) {
  auto stage = [&d](int dist, int sh, uint32_t m) {
    for (int i = 0; i < 8; ++i) {
      if (i & dist) continue;
      const uint32_t a = d[i], b = d[i + dist];
      d[i] = (a & m) | ((b << sh) & ~m);
      d[i + dist] = ((a >> sh) & m) | (b & ~m);
    }
  };
  stage(4, 4, 0x0f0f0f0fu);
  stage(2, 2, 0x33333333u);
  stage(1, 1, 0x55555555u);
}

// The network of one launch group: for input shard i the plane combos it needs (bit s of
// lo_used / hi_used: L[s] / H[s] is read by some row), and per (row r, plane k) the pair of
// combo indices (lo, hi) XORed into acc[r][k] (0 = no term).
struct Network {
  int K = 0, R = 0;
  std::vector<uint8_t> coef;                // [R][K]
  std::vector<uint32_t> lo_used, hi_used;   // [K]
  std::vector<uint8_t> lo, hi;              // [K][R][8]
  uint8_t term_lo(int i, int r, int k) const { return lo[(static_cast<size_t>(i) * R + r) * 8 + k]; }
  uint8_t term_hi(int i, int r, int k) const { return hi[(static_cast<size_t>(i) * R + r) * 8 + k]; }
};

inline Network build_network(int K, int R, const uint8_t* coef) {
  Network n;
  n.K = K;
  n.R = R;
  n.coef.assign(coef, coef + static_cast<size_t>(K) * R);
  n.lo_used.assign(K, 0);
  n.hi_used.assign(K, 0);
  n.lo.assign(static_cast<size_t>(K) * R * 8, 0);
  n.hi.assign(static_cast<size_t>(K) * R * 8, 0);
  for (int i = 0; i < K; ++i)
    for (int r = 0; r < R; ++r) {
      const uint8_t c = coef[static_cast<size_t>(r) * K + i];
      if (!c) continue;
      uint8_t rows[8];
      mul_matrix(c, rows);
      for (int k = 0; k < 8; ++k) {
        const uint8_t l = rows[k] & 15u, h = rows[k] >> 4;
        n.lo[(static_cast<size_t>(i) * R + r) * 8 + k] = l;
        n.hi[(static_cast<size_t>(i) * R + r) * 8 + k] = h;
        if (l) n.lo_used[i] |= 1u << l;
        if (h) n.hi_used[i] |= 1u << h;
      }
    }
  return n;
}

// Host evaluation of the network on 32 column bytes per lane: in[i] = the 8 dwords of shard
// i (dwords 0..3 = the lane's first vector, 4..7 its second), out[r] likewise.
inline void evaluate(const Network& n, const std::vector<std::array<uint32_t, 8>>& in,
                     std::vector<std::array<uint32_t, 8>>& out) {
  std::vector<std::array<uint32_t, 8>> acc(n.R);
  for (auto& a : acc) a.fill(0);
  for (int i = 0; i < n.K; ++i) {
    uint32_t p[8];
    for (int j = 0; j < 8; ++j) p[j] = in[i][j];
    tr8(p);
    uint32_t L[16] = {0}, H[16] = {0};
    for (int s = 1; s < 16; ++s)
      for (int j = 0; j < 4; ++j)
        if ((s >> j) & 1) {
          L[s] ^= p[j];
          H[s] ^= p[4 + j];
        }
    for (int r = 0; r < n.R; ++r)
      for (int k = 0; k < 8; ++k) acc[r][k] ^= L[n.term_lo(i, r, k)] ^ H[n.term_hi(i, r, k)];
  }
  out.assign(n.R, {});
  for (int r = 0; r < n.R; ++r) {
    uint32_t o[8];
    for (int k = 0; k < 8; ++k) o[k] = acc[r][k];
    tr8(o);
    for (int k = 0; k < 8; ++k) out[r][k] = o[k];
  }
}

// ---- device source ------------------------------------------------------------------------

struct GenOptions {
  int prefetch = 2;  // input shards whose loads are in flight while one is computed
  int min_waves = 2; // amdgpu_waves_per_eu lower bound (bitslice.cpp: 0 = auto_waves)
  int block = kBlockThreads;  // threads per block: a tile is block / 64 * kWaveVecs vectors
  int tile_vecs() const { return block / 64 * kWaveVecs; }
};

namespace detail {
inline std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
inline std::string fmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  std::vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return buf;
}

// Emits the definitions of the used combos of one group (planes 0..3 -> prefix L, 4..7 ->
// H; variable names <P><i>_<s>), cheapest first: pairs and triples from the planes, quads
// from a pair already formed when there is one.
inline void emit_combos(std::string& o, char P, int i, uint32_t used, int plane0) {
  auto name = [&](int s) {
    if (__builtin_popcount(s) == 1) return fmt("p%d_%d", i, plane0 + __builtin_ctz(s));
    return fmt("%c%d_%d", P, i, s);
  };
  uint32_t have = 0x2 | 0x4 | 0x10 | 0x100;  // the single planes
  for (int pc = 2; pc <= 4; ++pc)
    for (int s = 1; s < 16; ++s) {
      if (__builtin_popcount(s) != pc || !((used >> s) & 1u)) continue;
      std::vector<int> bits;
      for (int j = 0; j < 4; ++j)
        if ((s >> j) & 1) bits.push_back(1 << j);
      std::string e;
      if (pc == 2) {
        e = fmt("x2(%s, %s)", name(bits[0]).c_str(), name(bits[1]).c_str());
      } else if (pc == 3) {
        e = fmt("x3(%s, %s, %s)", name(bits[0]).c_str(), name(bits[1]).c_str(), name(bits[2]).c_str());
      } else {
        int pair = 0;
        for (int q : {3, 5, 6, 9, 10, 12})
          if ((have >> q) & 1u) { pair = q; break; }
        if (pair) {
          const int rest = 15 & ~pair;
          const int r0 = rest & -rest, r1 = rest & ~r0;
          e = fmt("x3(%s, %s, %s)", name(pair).c_str(), name(r0).c_str(), name(r1).c_str());
        } else {
          e = fmt("x2(x3(%s, %s, %s), %s)", name(1).c_str(), name(2).c_str(), name(4).c_str(),
                  name(8).c_str());
        }
      }
      o += fmt("    const u32 %s = %s;\n", name(s).c_str(), e.c_str());
      have |= 1u << s;
    }
}
}  // namespace detail

// The HIP source of the kernel `name` for network n.
inline std::string kernel_source(const Network& n, const std::string& name, const GenOptions& opt,
                                 size_t args_size) {
  using detail::fmt;
  std::string o;
  o.reserve(static_cast<size_t>(n.K) * n.R * 8 * 48 + 16384);
  o += "// generated by callfs_amd/csrc/bitslice_gen.hpp\n";
  o += "typedef unsigned int u32;\ntypedef unsigned long long u64;\n";
  o += args_decl();
  o += fmt("static_assert(sizeof(Args) == %zu, \"Args layout\");\n", args_size);
  o += R"SRC(
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <class T> using cptr = const __attribute__((address_space(4))) T*;
// every XOR through v_bitop3: opaque to LLVM's reassociation, which otherwise regroups the
// XOR chains across shards and keeps every shard's planes alive to the end (spills)
__device__ __forceinline__ u32 x3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ u32 x2(u32 a, u32 b) { return __builtin_amdgcn_bitop3_b32(a, b, 0u, 0x3C); }
// (m & a) | (~m & b)
__device__ __forceinline__ u32 sel(u32 m, u32 a, u32 b) { return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA); }
__device__ __forceinline__ void tr8(u32 (&d)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) if (!(i & 4)) { const u32 a = d[i], b = d[i + 4]; d[i] = sel(0x0f0f0f0fu, a, b << 4); d[i + 4] = sel(0x0f0f0f0fu, a >> 4, b); }
#pragma unroll
  for (int i = 0; i < 8; ++i) if (!(i & 2)) { const u32 a = d[i], b = d[i + 2]; d[i] = sel(0x33333333u, a, b << 2); d[i + 2] = sel(0x33333333u, a >> 2, b); }
#pragma unroll
  for (int i = 0; i < 8; ++i) if (!(i & 1)) { const u32 a = d[i], b = d[i + 1]; d[i] = sel(0x55555555u, a, b << 1); d[i + 1] = sel(0x55555555u, a >> 1, b); }
}
__device__ __forceinline__ void load_pair(u32 (&x)[8], const unsigned char* p, u64 va, bool lb) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  // no branch: a lane whose second vector lies past the shard reloads its first (the bit
  // planes keep byte positions apart, so those bytes only reach outputs it does not store)
  const u32x4 a = __builtin_nontemporal_load(q + va);
  const u32x4 b = __builtin_nontemporal_load(q + va + (lb ? 64 : 0));
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}
__device__ __forceinline__ void map_tile(const Args& a, u32 b, u32& stripe, u32& tile) {
  // a.order: 0 consecutive, 1 Q8, 2 X32, 3 G2, 4 X8, 5 G8, 6 Q16 (tile_order.hpp map_tile /
  // block_tile: the same bijections the nibble-table kernels use)
  u32 t = a.t_base + b;
  if (a.order == 2 || a.order == 4) {  // X32 / X8: each XCD takes runs of J neighbouring tiles
    const u32 J = a.order == 2 ? 32u : 8u, G = 8u * J, nb = gridDim.x;
    if (b < nb / G * G) { const u32 g = b / G, r = b - g * G; t = a.t_base + g * G + (r & 7u) * J + (r >> 3); }
  }
  if (a.order == 3 || a.order == 5) {  // G2 / G8: the same tile of G stripes on neighbouring blocks
    const u32 G = a.order == 3 ? 2u : 8u;
    const u32 per = G * a.tps, g = t / per, r = t - g * per;
    const u32 bt = a.ntiles / a.tps, gsz = bt - g * G < G ? bt - g * G : G;
    tile = r / gsz; stripe = g * G + (r - tile * gsz);
    return;
  }
  stripe = t / a.tps;
  const u32 r = t - stripe * a.tps;
  if (a.order == 1 || a.order == 6) {  // Q8 / Q16: the same position of Q column segments
    const u32 Q = a.order == 1 ? 8u : 16u, seg = a.tps / Q;
    tile = r < seg * Q ? (r % Q) * seg + r / Q : r;
  } else {
    tile = r;
  }
}
)SRC";
  o += fmt("extern \"C\" __global__ __launch_bounds__(%d) __attribute__((amdgpu_waves_per_eu(%d, 8)))\n",
           opt.block, opt.min_waves);
  o += fmt("void %s(const Args a) {\n", name.c_str());
  o += "  u32 stripe, tile;\n  map_tile(a, blockIdx.x, stripe, tile);\n";
  o += "  if (stripe * a.tps + tile >= a.ntiles) return;\n";
  o += fmt("  const u64 va = (u64)tile * %d + (threadIdx.x >> 6) * %d + (threadIdx.x & 63u);\n",
           opt.tile_vecs(), kWaveVecs);
  o += "  if (va >= a.nvec) return;\n  const bool lb = va + 64 < a.nvec;\n";
  o += fmt("  const cptr<const unsigned char*> in = (cptr<const unsigned char*>)(a.in_tab) + (u64)stripe * %d;\n", n.K);
  o += fmt("  const cptr<unsigned char*> out = (cptr<unsigned char*>)(a.out_tab) + (u64)stripe * %d;\n", n.R);
  const int D = std::max(1, std::min(opt.prefetch, n.K));
  std::vector<std::vector<bool>> init(n.R, std::vector<bool>(8, false));
  auto acc = [](int r, int k) { return fmt("a%d_%d", r, k); };
  for (int r = 0; r < n.R; ++r) {
    o += "  u32";
    for (int k = 0; k < 8; ++k) o += fmt("%s %s", k ? "," : "", acc(r, k).c_str());
    o += ";\n";
  }
  for (int i = 0; i < D; ++i) o += fmt("  u32 sh%d[8]; load_pair(sh%d, in[%d], va, lb);\n", i, i, i);
  for (int i = 0; i < n.K; ++i) {
    if (i + D < n.K)
      o += fmt("  u32 sh%d[8]; load_pair(sh%d, in[%d], va, lb);\n", i + D, i + D, i + D);
    o += "  asm volatile(\"\" ::: \"memory\");\n  __builtin_amdgcn_sched_barrier(0);\n  {\n";
    o += fmt("    tr8(sh%d);\n", i);
    for (int j = 0; j < 8; ++j) o += fmt("    const u32 p%d_%d = sh%d[%d];\n", i, j, i, j);
    detail::emit_combos(o, 'L', i, n.lo_used[i], 0);
    detail::emit_combos(o, 'H', i, n.hi_used[i], 4);
    auto cname = [&](char P, int s, int plane0) {
      if (__builtin_popcount(s) == 1) return fmt("p%d_%d", i, plane0 + __builtin_ctz(s));
      return fmt("%c%d_%d", P, i, s);
    };
    for (int r = 0; r < n.R; ++r)
      for (int k = 0; k < 8; ++k) {
        const int l = n.term_lo(i, r, k), h = n.term_hi(i, r, k);
        if (!l && !h) continue;
        std::string t1 = l ? cname('L', l, 0) : cname('H', h, 4);
        std::string t2 = l && h ? cname('H', h, 4) : "";
        const std::string a = acc(r, k);
        if (!init[r][k]) {
          o += t2.empty() ? fmt("    %s = %s;\n", a.c_str(), t1.c_str())
                          : fmt("    %s = x2(%s, %s);\n", a.c_str(), t1.c_str(), t2.c_str());
          init[r][k] = true;
        } else {
          o += t2.empty() ? fmt("    %s = x2(%s, %s);\n", a.c_str(), a.c_str(), t1.c_str())
                          : fmt("    %s = x3(%s, %s, %s);\n", a.c_str(), a.c_str(), t1.c_str(), t2.c_str());
        }
      }
    // pin: every accumulator this shard wrote is an in/out operand of an empty volatile asm,
    // so no update of shard i moves past it (the SelectionDAG scheduler orders pure
    // arithmetic freely inside a block: without this it deferred most of shard 0's updates
    // to the end and spilled the planes they read)
    std::vector<std::string> pins;
    for (int r = 0; r < n.R; ++r)
      for (int k = 0; k < 8; ++k)
        if (init[r][k] && (n.term_lo(i, r, k) || n.term_hi(i, r, k))) pins.push_back(acc(r, k));
    for (size_t p0 = 0; p0 < pins.size(); p0 += 16) {
      o += "    asm volatile(\"\" :";
      for (size_t q = p0; q < pins.size() && q < p0 + 16; ++q)
        o += fmt("%s \"+v\"(%s)", q > p0 ? "," : "", pins[q].c_str());
      o += ");\n";
    }
    o += "  }\n";
  }
  o += "  __builtin_amdgcn_sched_barrier(0);\n  bool bad = false;\n";
  for (int r = 0; r < n.R; ++r) {
    o += "  {\n    u32 o[8] = {";
    for (int k = 0; k < 8; ++k) o += fmt("%s%s", k ? ", " : "", init[r][k] ? acc(r, k).c_str() : "0u");
    o += "};\n    tr8(o);\n";
    o += fmt("    u32x4* q = reinterpret_cast<u32x4*>(out[%d]) + va;\n", r);
    o += "    const u32x4 v0 = {o[0], o[1], o[2], o[3]}, v1 = {o[4], o[5], o[6], o[7]};\n";
    o += fmt("    if ((a.verify_mask >> %d) & 1u) {\n", r);
    o += "      const u32x4 y0 = __builtin_nontemporal_load(q);\n";
    o += "      u32x4 y1 = v1;\n      if (lb) y1 = __builtin_nontemporal_load(q + 64);\n";
    o += "      const u32x4 z = (y0 ^ v0) | (y1 ^ v1);\n";
    o += "      bad |= (z.x | z.y | z.z | z.w) != 0u;\n";
    o += "    } else {\n      __builtin_nontemporal_store(v0, q);\n";
    o += "      if (lb) __builtin_nontemporal_store(v1, q + 64);\n    }\n  }\n";
  }
  o += "  if (bad) atomicOr(a.status + (u64)stripe * a.status_stride, 1);\n}\n";
  return o;
}

}  // namespace bs
}  // namespace callfs
