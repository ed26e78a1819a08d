// Device code of the GF(2^8) shard-matrix kernels for gfx950 (MI355X, CDNA4).
//
// Replaces the SIMD kernels of github.com/klauspost/reedsolomon v1.13.3 (go.mod:13)
// behind erasure/codec.go:36 (Encode), :55 (Reconstruct) and :59 (Verify).
//
// Two kernels (DESIGN.md "Kernels"); launch_apply in rs_kernels.hip picks one per launch:
//  * rs_apply_lds — every launch with k >= 4 inputs or R >= 5 rows (the bench's kernel).
//    Per data byte, two LDS lookups into per-shard nibble tables return the products for
//    all R rows at once. Table addresses are formed by v_perm_b32 (R <= 8) or
//    v_or_b32_sdwa (R 9..16: no VGPR for the table base, 4 waves per SIMD), and partial
//    products are combined by v_bitop3 as a three-input XOR. The tables are staged into
//    LDS once per block. Misaligned shards (upstream Split layout at odd S) take its
//    REALIGN form: aligned loads and stores, realigned in registers by DPP + v_alignbyte.
//  * rs_apply_vec — k <= 3 with R <= 4. GF multiply by a wave-uniform coefficient c on 4
//    packed bytes = three v_perm_b32 byte-selects from 8-byte tables:
//    c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6] (gf256.hpp perm_tables). The tables arrive
//    through the constant address space (s_load into SGPRs): no LDS.
// Both stream each lane's 16-byte column vectors through all K input shards with
// global_load_dwordx4 (non-temporal), keep the R outputs in registers and write (or,
// for Verify rows, compare) them once: (K + R) * 16 bytes of compulsory HBM traffic per
// vector, nothing re-read (rocprofv3 FETCH/WRITE_SIZE = algorithmic bytes).
// Ragged tails (S % 16) are computed by each stripe's first tile, one byte per thread
// (the byte kernel rs_apply_bytes remains for S < 16). Shard pointers need no alignment:
// 16-B global accesses at any byte address are legal on gfx950 (rs_kernels.hpp).
#pragma once

#include <algorithm>
#include <type_traits>

#include "rs_kernels.hpp"
#include "tile_order.hpp"

namespace callfs {
namespace dev {

constexpr int kBlock = 256;



template <class T>
using cptr = const __attribute__((address_space(4))) T*;

template <class T>
__device__ __forceinline__ cptr<T> as_const(const T* p) {
  return (cptr<T>)(p);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

struct Sel {
  uint32_t i0, i1, i2;
};

__device__ __forceinline__ Sel selectors(uint32_t x) {
  return Sel{x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// c*x for 4 packed bytes, as three partial products (XOR them to finish).
struct Prod {
  uint32_t p0, p1, p2;
};

__device__ __forceinline__ Prod gf_mul4(const Sel& s, cptr<uint32_t> t) {
  return Prod{__builtin_amdgcn_perm(t[1], t[0], s.i0), __builtin_amdgcn_perm(t[3], t[2], s.i1),
              __builtin_amdgcn_perm(t[4], t[4], s.i2)};
}

// acc ^ a ^ b with three v_bitop3 for the six partial products.
__device__ __forceinline__ uint32_t fma2(uint32_t acc, const Prod& a, const Prod& b) {
  acc = xor3(acc, a.p0, a.p1);
  acc = xor3(acc, a.p2, b.p0);
  return xor3(acc, b.p1, b.p2);
}

__device__ __forceinline__ uint32_t fma1(uint32_t acc, const Prod& a) {
  return xor3(acc, a.p0, xor3(a.p1, a.p2, 0u));
}

__device__ __forceinline__ uint32_t word(const uint4& v, int w) {
  return w == 0 ? v.x : (w == 1 ? v.y : (w == 2 ? v.z : v.w));
}

// Compile-time launch policy of the vector kernel.
//   WPE      minimum waves per SIMD the register allocation must allow
//   U        16-B column vectors per lane (tile = 256*U vectors of a stripe)
//   NT_LOAD  / NT_STORE: non-temporal (streaming) global loads / stores
//   PERSIST  grid-stride over tiles with a fixed grid instead of one tile per block
//   BS       threads per block; PD prefetch depth in input-shard pairs (1 or 2)
//   ORD      tile order: 0 = a stripe's tiles consecutive, 1 = interleaved across all
//            stripes, 2/3/4/5 = interleaved within groups of 8/32/4/2 stripes, 6/7/8/9 =
//            interleaved across 8/32/16/64 column segments of one stripe, 10/11 = consecutive
//            with J = 8/32 consecutive tiles per XCD (tile_order.hpp block_tile; LDS kernel:
//            0, 2..11)
//   RING     LDS kernel input ring: 0 = three registers shifted each step (PD = 2);
//            1 = PD+1 slots with the loop unrolled PD+1 times (static slot indices)
//   NOMATH   measurement only (tools/kbench.hip): the LDS kernel with its lookups
//            replaced by one XOR per input dword -- same loads, stores, grid and tile
//            order -- i.e. the memory ceiling of a launch's traffic shape
//   REALIGN  LDS kernel, RING 0: input shards whose base is not 16-B aligned are read
//            with aligned 16-B loads and realigned in registers (neighbour lane's
//            vector by DPP wave_shl:1, v_alignbyte funnel shift) instead of unaligned
//            global_load_dwordx4
template <int WPE_, int U_, bool NT_LOAD_, bool NT_STORE_, bool PERSIST_, int BS_ = 256,
          int PD_ = 1, int ORD_ = 0, int RING_ = 0, bool NOMATH_ = false, int REALIGN_ = 0,
          bool SDWA_ = false, int PROBE_ = 0, int VPF_ = 0, int WIX_ = 0, int DMA_ = 0>
struct Policy {
  // > 0: input vectors staged through LDS by LDS-DMA (global_load_lds_dwordx4), DMA shards in
  // flight per wave in a per-wave ring of DMA 1 KiB slots behind the tables, read back by
  // ds_read_b128 (rs_apply.hpp "LDS-DMA ring"): loads in flight cost LDS, not VGPRs
  static constexpr int DMA = DMA_;
  static_assert(DMA_ == 0 || (REALIGN_ == 0 && WIX_ == 0 && RING_ == 0 && !NOMATH_ && !SDWA_ &&
                              VPF_ == 0 && PROBE_ == 0 && BS_ == 512 && U_ == 1),
                "DMA: aligned ring-of-three kernel shape only");
  // 1 (A/B build): R <= 4, input shards in triples, each byte position of a triple
  // resolved by four 6-bit lookups into 64-entry tables of 4-byte entries (built in LDS
  // from the nibble tables) instead of six nibble lookups;
  // 2: the same triple loads with the nibble lookups, any R <= 8 (production);
  // 2 with REALIGN: the realigning kernel's aligned loads issued in triples;
  // 3: triples double-buffered in two register sets (production for R <= 4, K >= 6);
  // 4 (kbench probe): as 1 with zeros past K; 5 (kbench probe): as 3 with pairs
  static constexpr int WIX = WIX_;
  // (WIX 2 with VPF: the aligned triple loop with early compare loads)
  static_assert(!WIX_ || ((REALIGN_ == 0 || WIX_ == 2 || (WIX_ == 3 && REALIGN_ == 2)) && (VPF_ == 0 || ((WIX_ == 2 || WIX_ == 3) && REALIGN_ == 0)) &&
                          RING_ == 0 && !NOMATH_ && !SDWA_),
                "WIX: ring-of-three kernel only; 6-bit lookups on aligned shards only");
  // > 0: Verify rows' stored vectors are loaded VPF shards before the end of the input
  // loop instead of after it (R <= 4, plain loads, ring of three only)
  static constexpr int VPF = VPF_;
  static_assert(VPF_ == 0 || (REALIGN_ == 0 && RING_ == 0), "VPF: plain ring-of-three kernel only");
  // tools/kbench layout probes (never dispatched): 1 = 63-vector waves (the REALIGN
  // tiling) with plain loads, lane 63 idle; 2 = 64-vector waves, lane 63 idle
  static constexpr int PROBE = PROBE_;
  static constexpr bool NOMATH = NOMATH_;
  // LDS table addresses by v_or_b32_sdwa (byte select + OR) instead of v_perm_b32
  static constexpr bool SDWA = SDWA_;
  // 0: plain; 1: aligned loads realigned in registers (63 vectors per wave); 2: loads and
  // parity stores both aligned (62 vectors per wave, edge bytes in the first tile)
  static constexpr int REALIGN = REALIGN_;
  // 16-B vectors per tile: REALIGN waves produce 63 vectors from 64 aligned loads
  // (5: misaligned inputs, aligned outputs, 64 vectors per wave: lane 63 loads its
  // neighbour vector itself)
  static constexpr int WAVE_VECS = REALIGN_ == 2 ? 62 : ((REALIGN_ && REALIGN_ != 5) || PROBE_ == 1) ? 63 : 64;
  static constexpr int TILE_VECS = WAVE_VECS < 64 ? BS_ / 64 * WAVE_VECS : BS_ * U_;
  static constexpr int WPE = WPE_;
  static constexpr int U = U_;
  static constexpr bool NT_LOAD = NT_LOAD_;
  static constexpr bool NT_STORE = NT_STORE_;
  static constexpr bool PERSIST = PERSIST_;
  static constexpr int BS = BS_;
  static constexpr int PD = PD_;
  static constexpr int ORD = ORD_;
  static constexpr int RING = RING_;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <class P>
__device__ __forceinline__ uint4 load16(const uint4* p) {
  if constexpr (P::NT_LOAD) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}

template <class P>
__device__ __forceinline__ void store16(uint4* p, const uint4& v) {
  if constexpr (P::NT_STORE) {
    const u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
  } else {
    *p = v;
  }
}

template <int RT, int U>
__device__ __forceinline__ void mac_pair(uint32_t (&acc)[U][RT][4], const uint4 (&xa)[U],
                                         const uint4 (&xb)[U], cptr<uint32_t> ta,
                                         cptr<uint32_t> tb) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const Sel sa = selectors(word(xa[u], w)), sb = selectors(word(xb[u], w));
#pragma unroll
      for (int r = 0; r < RT; ++r)
        acc[u][r][w] = fma2(acc[u][r][w], gf_mul4(sa, ta + r * 5), gf_mul4(sb, tb + r * 5));
    }
}

template <int RT, int U>
__device__ __forceinline__ void mac_one(uint32_t (&acc)[U][RT][4], const uint4 (&xa)[U],
                                        cptr<uint32_t> ta) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const Sel sa = selectors(word(xa[u], w));
#pragma unroll
      for (int r = 0; r < RT; ++r) acc[u][r][w] = fma1(acc[u][r][w], gf_mul4(sa, ta + r * 5));
    }
}

// The ragged tail S % 16 of every shard, run by the stripe's first tile of the v_perm
// kernel (one byte per thread): odd-S launches need no second kernel. The first tile, not
// the last: the tail is a chain of K byte loads, and in the stripe's last tile (the
// grid's last for the last stripe) it outlasted the other waves and delayed the kernel's
// end by ~2 %. Loads are issued tail_loads<RT>() at a time: 8 where the
// kernel has registers to spare (R <= 4), 4 otherwise (8 took R = 8 from 68 to 73 VGPRs).
template <int RT>
constexpr int tail_loads() { return RT <= 4 ? 8 : 4; }
// Which wave takes a stripe's ragged tail (S % 16 bytes): ApplyArgs::tail_in_vec, chosen on
// the host (rs_kernels.hip tail_code) = (tile << 2) | (last wave << 1) | 1. For stripes of
// few tiles the block's last wave in the stripe's last tile when that wave holds no
// vectors (the last tile is partial), so no wave that streams vectors waits for the
// tail's byte loads; otherwise wave 0 of the stripe's first tile, whose wait is hidden
// behind the rest of a long stripe (in the last tile of the grid's last stripe the tail's
// load chain delays the kernel's end). Returns the thread's byte index in the tail, or ~0u.
// (Decided on the host: the 64-bit tile arithmetic in the kernel cost the v_perm kernel's
// R = 2 instances 4 SGPRs and a wave.)
template <int BS>
__device__ __forceinline__ uint32_t tail_lane(uint32_t code, uint32_t tile) {
  const uint32_t tid0 = (code & 2u) ? BS - 64 : 0u;
  return tile == (code >> 2) && threadIdx.x >= tid0 ? threadIdx.x - tid0 : ~0u;
}

template <int RT>
__device__ __forceinline__ void tail_bytes(cptr<const uint8_t*> in, uint64_t b, int i0, int K,
                                           uint32_t (&x)[tail_loads<RT>()]) {
#pragma unroll
  for (int j = 0; j < tail_loads<RT>(); ++j) x[j] = i0 + j < K ? in[i0 + j][b] : 0u;
}
template <int RT>
__device__ __forceinline__ void vec_tail(const ApplyArgs& a, cptr<const uint8_t*> in,
                                         cptr<uint8_t*> out, uint32_t stripe,
                                         cptr<uint32_t> tabs, uint32_t j) {
  const uint32_t nt = static_cast<uint32_t>(a.S - a.nvec * 16);
  if (j >= nt) return;
  const uint64_t b = a.nvec * 16 + j;
  uint32_t acc[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) acc[r] = 0;
  for (int i0 = 0; i0 < a.K; i0 += tail_loads<RT>()) {
    uint32_t x[tail_loads<RT>()];
    tail_bytes<RT>(in, b, i0, a.K, x);
    for (int j = 0; j < tail_loads<RT>() && i0 + j < a.K; ++j) {
      const Sel sel = selectors(x[j]);
      const cptr<uint32_t> t = tabs + static_cast<size_t>(i0 + j) * RT * 5;
#pragma unroll
      for (int r = 0; r < RT; ++r) acc[r] = fma1(acc[r], gf_mul4(sel, t + r * 5));
    }
  }
  bool bad = false;
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const uint8_t v = static_cast<uint8_t>(acc[r]);
    if ((a.verify_mask >> r) & 1u) bad |= out[r][b] != v;
    else out[r][b] = v;
  }
  if (bad) atomicOr(a.status + static_cast<size_t>(stripe) * a.status_stride, 1);
}

// Tiles: a stripe's nvec vectors are cut into tiles of BS*U; tile t covers stripe
// t / tiles_per_stripe (ORD 0) or t % batch (ORD 1). Every tile is wave-uniform in its
// stripe, so shard pointers stay scalar.
template <int KT, int RT, class P>
__global__ __launch_bounds__(P::BS) __attribute__((amdgpu_waves_per_eu(P::WPE, 8)))
void rs_apply_vec(ApplyArgs a) {
  constexpr int U = P::U;
  constexpr int BS = P::BS;
  const int K = a.K;
  const int npairs = K >> 1;
  const uint32_t tile_vecs = BS * U;
  const uint32_t tps = static_cast<uint32_t>((a.nvec + tile_vecs - 1) / tile_vecs);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.batch);
  const cptr<uint32_t> tabs = as_const(a.tabs);

  for (uint32_t t = a.t_base + blockIdx.x; t < ntiles; t += (P::PERSIST ? gridDim.x : ntiles)) {
    uint32_t stripe, tile;
    if constexpr (P::ORD == 1) {
      tile = t / static_cast<uint32_t>(a.batch);
      stripe = t - tile * static_cast<uint32_t>(a.batch);
    } else {
      map_tile<P::ORD>(t, tps, static_cast<uint32_t>(a.batch), stripe, tile);
    }
    const uint64_t v0 = static_cast<uint64_t>(tile) * tile_vecs + threadIdx.x;
    cptr<const uint8_t*> in = as_const(a.in_tab) + static_cast<size_t>(stripe) * K;
    cptr<uint8_t*> out = as_const(a.out_tab) + static_cast<size_t>(stripe) * RT;
    if (a.tail_in_vec) {
      const uint32_t j = tail_lane<BS>(a.tail_in_vec, tile);
      if (j != ~0u) vec_tail<RT>(a, in, out, stripe, tabs, j);
    }
    bool live[U];
#pragma unroll
    for (int u = 0; u < U; ++u) live[u] = v0 + static_cast<uint64_t>(u) * BS < a.nvec;
    if (!live[0]) continue;

    auto ld = [&](int i, uint4 (&x)[U]) {
      const uint4* src = reinterpret_cast<const uint4*>(in[i]) + v0;
#pragma unroll
      for (int u = 0; u < U; ++u)
        x[u] = (u == 0 || live[u]) ? load16<P>(src + u * BS) : make_uint4(0, 0, 0, 0);
    };

    uint32_t acc[U][RT][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int w = 0; w < 4; ++w) acc[u][r][w] = 0;

    // register ring of PD+1 input pairs: pair p is consumed while pairs p+1..p+PD load
    uint4 xa[U], xb[U], ya[U], yb[U];
    if (npairs) {
      ld(0, xa);
      ld(1, xb);
    }
    if (P::PD > 1 && npairs > 1) {
      ld(2, ya);
      ld(3, yb);
    }
#pragma unroll 1
    for (int p = 0; p < npairs; ++p) {
      uint4 za[U], zb[U];
      const int nxt = p + P::PD;
      if (nxt < npairs) {
        ld(2 * nxt, za);
        ld(2 * nxt + 1, zb);
      }
      const cptr<uint32_t> ta = tabs + static_cast<size_t>(2 * p) * RT * 5;
      mac_pair<RT, U>(acc, xa, xb, ta, ta + RT * 5);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (P::PD > 1) {
          xa[u] = ya[u];
          xb[u] = yb[u];
          ya[u] = za[u];
          yb[u] = zb[u];
        } else {
          xa[u] = za[u];
          xb[u] = zb[u];
        }
      }
    }
    if (K & 1) {
      ld(K - 1, xa);
      mac_one<RT, U>(acc, xa, tabs + static_cast<size_t>(K - 1) * RT * 5);
    }

    bool bad = false;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      uint4* dst = reinterpret_cast<uint4*>(out[r]) + v0;
      const bool cmp = (a.verify_mask >> r) & 1u;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!live[u]) continue;
        const uint4 o = make_uint4(acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]);
        if (cmp) {
          const uint4 y = load16<P>(dst + u * BS);  // non-temporal, as in rs_apply_lds
          bad |= ((y.x ^ o.x) | (y.y ^ o.y) | (y.z ^ o.z) | (y.w ^ o.w)) != 0;
        } else {
          store16<P>(dst + u * BS, o);
        }
      }
    }
    if (bad) atomicOr(a.status + static_cast<size_t>(stripe) * a.status_stride, 1);
  }
}

// ---- realigned loads of misaligned shards (Policy::REALIGN) ----------------------------
// A shard at p with d = p & 15: vector v (bytes [16v, 16v+16) of p) lies in the aligned
// vectors A[v] = (p-d)[v] and A[v+1]. A REALIGN wave loads 64 consecutive aligned vectors
// A[w0 .. w0+63], one per lane, and produces the 63 vectors w0 .. w0+62: lane l takes
// A[l+1] from lane l+1 by DPP wave_shl:1 and funnel-shifts the pair by d bytes
// (v_alignbyte). Lane 63 only loads. Each lane issues one aligned global_load_dwordx4
// per shard, as the unaligned kernel does, and every realigned byte comes from the wave's
// own loads. The next wave reloads its first vector, 1/64 of the lines, from cache.
// Load addresses are clamped to A[nvec] (d > 0) or A[nvec-1] (d = 0). Every aligned
// vector up to A[nvec] contains a byte of the shard (A[nvec] starts at
// p + 16*nvec - d <= p + S - 1). An aligned 16-B block never straddles a page, so no
// load can fault outside the shard's pages. (Two vector loads per shard, A[v] and A[v+1],
// measured 9-13 points slower, and a per-lane tail load or a scalar tail load cost
// waits: these kernels are sensitive to the count of memory instructions, not only to
// HBM bytes.)
template <int Q>
__device__ __forceinline__ uint4 funnel16(const uint4& A, const uint4& B, uint32_t r) {
  const uint32_t s[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
  return make_uint4(__builtin_amdgcn_alignbyte(s[Q + 1], s[Q], r),
                    __builtin_amdgcn_alignbyte(s[Q + 2], s[Q + 1], r),
                    __builtin_amdgcn_alignbyte(s[Q + 3], s[Q + 2], r),
                    __builtin_amdgcn_alignbyte(s[Q + 4], s[Q + 3], r));
}

__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x130, 0xf, 0xf, false));
}

// Aligned load of A[v] of shard p (v clamped as above); nvec >= 1.
template <class P>
__device__ __forceinline__ uint4 ld_aligned(const uint8_t* p, uint64_t v, uint64_t nvec) {
  const uint32_t d = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)) & 15u;
  const uint64_t vmax = d ? nvec : nvec - 1;
  return load16<P>(reinterpret_cast<const uint4*>(p - d) + (v < vmax ? v : vmax));
}

// Bytes d..15 of this lane's A followed by bytes 0..d-1 of the next lane's A (d
// wave-uniform); every lane of the wave executes this (lane 63's result is not used).
__device__ __forceinline__ uint4 shift_from_next(const uint4& A, uint32_t d) {
  if (d == 0) return A;  // wave-uniform
  const uint4 B = make_uint4(from_next_lane(A.x), from_next_lane(A.y), from_next_lane(A.z),
                             from_next_lane(A.w));
  const uint32_t r = d & 3u;
  switch (d >> 2) {  // wave-uniform
    case 0: return funnel16<0>(A, B, r);
    case 1: return funnel16<1>(A, B, r);
    case 2: return funnel16<2>(A, B, r);
    default: return funnel16<3>(A, B, r);
  }
}

// Vector v of shard p from this lane's aligned A[v] and the next lane's A[v+1].
__device__ __forceinline__ uint4 realign(const uint8_t* p, const uint4& A) {
  return shift_from_next(A, static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)) & 15u);
}

// shift_from_next without branches: the dword shift d >> 2 by two rounds of selects on
// wave-uniform conditions, the byte shift by v_alignbyte (alignbyte(hi, lo, 0) = lo, so
// d = 0 needs no case). For loops that realign several shards per iteration (the triple
// loads): three branchy realigns per iteration took the kernel to 202 VGPRs.
__device__ __forceinline__ uint4 shift_from_next_sel(const uint4& A, uint32_t d) {
  const uint32_t s[8] = {A.x, A.y, A.z, A.w, from_next_lane(A.x), from_next_lane(A.y),
                         from_next_lane(A.z), from_next_lane(A.w)};
  // v_perm byte selects, not C selects: LLVM folds `c ? s[k + 1] : s[k]` into an indexed
  // load of s, which it places in scratch
  const uint32_t sel1 = d & 4u ? 0x07060504u : 0x03020100u, sel2 = d & 8u ? 0x07060504u : 0x03020100u;
  uint32_t u[7], t[5];
#pragma unroll
  for (int k = 0; k < 7; ++k) u[k] = __builtin_amdgcn_perm(s[k + 1], s[k], sel1);
#pragma unroll
  for (int j = 0; j < 5; ++j) t[j] = __builtin_amdgcn_perm(u[j + 2], u[j], sel2);
  const uint32_t r = d & 3u;
  return make_uint4(__builtin_amdgcn_alignbyte(t[1], t[0], r), __builtin_amdgcn_alignbyte(t[2], t[1], r),
                    __builtin_amdgcn_alignbyte(t[3], t[2], r), __builtin_amdgcn_alignbyte(t[4], t[3], r));
}
__device__ __forceinline__ uint4 realign_sel(const uint8_t* p, const uint4& A) {
  return shift_from_next_sel(A, static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)) & 15u);
}

// REALIGN 5 (outputs 16-B aligned): waves of 64 vectors, so every wave's stores fill
// whole 1 KiB windows of the output rows. Lane 63's A[v+1] is the first vector of the
// next wave's window: lane 63 alone loads it (one single-lane load per shard, E below) and
// the DPP that hands every other lane its neighbour's A leaves E in lane 63 (bound_ctrl
// off: a lane whose source is out of the wave keeps the `old` operand).
__device__ __forceinline__ uint4 shift_from_next_e(const uint4& A, const uint4& E, uint32_t d) {
  if (d == 0) return A;  // wave-uniform
  auto nx = [](uint32_t v, uint32_t old) {
    return static_cast<uint32_t>(
        __builtin_amdgcn_update_dpp(static_cast<int>(old), static_cast<int>(v), 0x130, 0xf, 0xf, false));
  };
  const uint4 B = make_uint4(nx(A.x, E.x), nx(A.y, E.y), nx(A.z, E.z), nx(A.w, E.w));
  const uint32_t r = d & 3u;
  switch (d >> 2) {  // wave-uniform
    case 0: return funnel16<0>(A, B, r);
    case 1: return funnel16<1>(A, B, r);
    case 2: return funnel16<2>(A, B, r);
    default: return funnel16<3>(A, B, r);
  }
}

// ---- aligned parity stores of misaligned rows (Policy::REALIGN == 2) -----------------
// Row q with mo = q & 15 != 0 and f = 16 - mo: the aligned 16-B block at q + f + 16v holds
// bytes f..15 of result vector v and bytes 0..f-1 of vector v+1, so lane l stores
// shift_from_next(R[v0], f) there for v0 <= nvec - 2. A wave computes 63 valid results
// (lanes 0..62, REALIGN loads) and stores 62 blocks (lanes 0..61); the next wave starts
// at the 62nd. Each stripe's first tile writes the bytes no aligned block covers, one
// byte per thread (lds_edges): the head [0, f) and the tail [16(nvec-1) + f, S) of every
// misaligned row, [16 nvec, S) of aligned rows and Verify rows.

// ---- LDS nibble-table variant ---------------------------------------------------------
// Per data byte two LDS lookups (low / high nibble) return the products for all RT rows
// at once (ds_read_b32 / b64 / b128 for RT <= 4 / 8 / 16), so the cost per data dword
// is about 20-28 VALU + 8 LDS reads for any RT, versus 5 + 4.5*RT VALU for the v_perm
// kernel. Tables (gf256.hpp nibble_tables): 32*W bytes per input shard at LDS offset
// 32*W*i, low table first, high table at +16*W; W = 8 (RT <= 8) or 16. Loaded once
// per block.
// Addresses: a v_perm drops the per-byte nibble*W (precomputed for the 4 bytes of a
// dword in one register) into byte 0 of the table base, which is 256-B aligned (W=16
// high tables sit at +256; for W=8 the +128 of the high table is bit 7 of that byte):
// one VALU per lookup.
// Accumulation is per data-byte position (T[w][j] = RT row products of byte j of dword
// w, XORed over the shards); a final byte transpose (3 VALU per row) forms row words.
struct u32x4_acc {
  uint32_t v[4];
};

__device__ __forceinline__ u32x4_acc operator^(const u32x4_acc& a, const u32x4_acc& b) {
  return u32x4_acc{{a.v[0] ^ b.v[0], a.v[1] ^ b.v[1], a.v[2] ^ b.v[2], a.v[3] ^ b.v[3]}};
}

template <int RT>
struct LdsAcc {
  static constexpr int W = RT > 8 ? 16 : 8;  // table entry bytes
  using T = typename std::conditional<
      (RT > 8), u32x4_acc, typename std::conditional<(RT > 4), uint64_t, uint32_t>::type>::type;
};

template <class T>
using lds_ptr = const __attribute__((address_space(3))) T*;

// Dynamic LDS bytes of rs_apply_lds for K input shards and RT rows.
inline size_t lds_bytes(int K, int RT) { return static_cast<size_t>(K) * 32 * (RT > 8 ? 16 : 8); }

// One table entry at an absolute 32-bit LDS address (no base add per lookup).
template <int RT>
__device__ __forceinline__ typename LdsAcc<RT>::T lds_lookup(uint32_t addr) {
  using T = typename LdsAcc<RT>::T;
  if constexpr (RT > 8) {
    const u32x4 q = *(lds_ptr<u32x4>)(static_cast<uintptr_t>(addr));
    return T{{q.x, q.y, q.z, q.w}};
  } else {
    return *(lds_ptr<T>)(static_cast<uintptr_t>(addr));
  }
}

// a ^ b ^ c with one v_bitop3 per dword.
__device__ __forceinline__ uint32_t lds_x3(uint32_t a, uint32_t b, uint32_t c) {
  return xor3(a, b, c);
}
__device__ __forceinline__ uint64_t lds_x3(uint64_t a, uint64_t b, uint64_t c) {
  return (static_cast<uint64_t>(xor3(a >> 32, b >> 32, c >> 32)) << 32) |
         xor3(static_cast<uint32_t>(a), static_cast<uint32_t>(b), static_cast<uint32_t>(c));
}
__device__ __forceinline__ u32x4_acc lds_x3(const u32x4_acc& a, const u32x4_acc& b,
                                            const u32x4_acc& c) {
  return u32x4_acc{{xor3(a.v[0], b.v[0], c.v[0]), xor3(a.v[1], b.v[1], c.v[1]),
                    xor3(a.v[2], b.v[2], c.v[2]), xor3(a.v[3], b.v[3], c.v[3])}};
}

// base | byte J of x in one v_or_b32_sdwa (SDWA source select; base in an SGPR).
template <int J>
__device__ __forceinline__ uint32_t or_byte(uint32_t x, uint32_t base) {
  uint32_t r;
  if constexpr (J == 0)
    asm("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
        : "=v"(r) : "v"(x), "s"(base));
  else if constexpr (J == 1)
    asm("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
        : "=v"(r) : "v"(x), "s"(base));
  else if constexpr (J == 2)
    asm("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
        : "=v"(r) : "v"(x), "s"(base));
  else
    asm("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
        : "=v"(r) : "v"(x), "s"(base));
  return r;
}

// base: absolute LDS address of input shard i's tables (256-B aligned).
// All 8 lookups of a data dword are issued before any is consumed; for 16-byte entries
// a sched_group_barrier keeps them together (the default schedule reused one register
// quad and waited after every pair: 2 reads in flight instead of 8).
template <int RT, bool SD = false>
__device__ __forceinline__ void lds_mac(typename LdsAcc<RT>::T (&acc)[4][4], const uint4& x,
                                        uint32_t base) {
  using T = typename LdsAcc<RT>::T;
  constexpr int W = LdsAcc<RT>::W;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t xw = word(x, w);
    uint32_t xl, xh, base_hi;
    if constexpr (W == 8) {
      xl = (xw << 3) & 0x78787878u;
      xh = ((xw >> 1) & 0x78787878u) | 0x80808080u;  // +128: the high table
      base_hi = base;
    } else {
      xl = (xw << 4) & 0xf0f0f0f0u;
      xh = xw & 0xf0f0f0f0u;
      base_hi = base + 256u;
    }
    T lo[4], hi[4];
    if constexpr (SD) {
      const uint32_t sb = __builtin_amdgcn_readfirstlane(base);
      const uint32_t sbh = __builtin_amdgcn_readfirstlane(base_hi);
      lo[0] = lds_lookup<RT>(or_byte<0>(xl, sb));
      hi[0] = lds_lookup<RT>(or_byte<0>(xh, sbh));
      lo[1] = lds_lookup<RT>(or_byte<1>(xl, sb));
      hi[1] = lds_lookup<RT>(or_byte<1>(xh, sbh));
      lo[2] = lds_lookup<RT>(or_byte<2>(xl, sb));
      hi[2] = lds_lookup<RT>(or_byte<2>(xh, sbh));
      lo[3] = lds_lookup<RT>(or_byte<3>(xl, sb));
      hi[3] = lds_lookup<RT>(or_byte<3>(xh, sbh));
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t sel = 0x07060500u | static_cast<uint32_t>(j);
        lo[j] = lds_lookup<RT>(__builtin_amdgcn_perm(base, xl, sel));
        hi[j] = lds_lookup<RT>(__builtin_amdgcn_perm(base_hi, xh, sel));
      }
    }
    if constexpr (W == 16) {
      __builtin_amdgcn_sched_group_barrier(0x0100, 8, 0);  // the 8 DS reads
      __builtin_amdgcn_sched_group_barrier(0x0002, 64, 0);  // then VALU
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[w][j] = lds_x3(acc[w][j], lo[j], hi[j]);
  }
}

// ---- 6-bit lookups over shard triples (Policy::WIX, R <= 4) ---------------------------
// Three shards A, B, C give 24 bits per byte position; four 6-bit pieces cover them:
// P0 = A[5:0], P1 = A[7:6] | B[3:0] << 2, P2 = B[7:4] | C[1:0] << 4, P3 = C[7:2]. Each piece
// indexes a 64-entry table of 4-byte entries (the R <= 4 row products of its bits), 256 B,
// so every entry still owns its bank and the lookups never conflict. Per byte position of
// a triple: 4 lookups instead of 6 nibble lookups, 2 XOR3 instead of 3.
// LDS layout: the nibble tables (K * 32 * 8 B) first, then per triple g four tables at
// wix_base(K) + 1024 g + 256 t; entries are built from the nibble tables after they land.
__host__ __device__ inline uint32_t wix_base(int K) { return static_cast<uint32_t>(K) * 256u; }
inline size_t lds_bytes_wix(int K) { return static_cast<size_t>(K) * 256 + static_cast<size_t>(K / 3) * 1024; }

// Entry e of table t of triple g from the nibble tables at lds0 (low table of shard i at
// 256 i + 8 n, high at 256 i + 128 + 8 n; the first 4 bytes hold rows 0..3).
__device__ __forceinline__ uint32_t wix_entry(uint32_t lds0, uint32_t g, uint32_t t, uint32_t e) {
  const uint32_t A = lds0 + 768u * g, B = A + 256u, C = B + 256u;
  uint32_t p, q;
  switch (t) {
    case 0: p = A + 8u * (e & 15u); q = A + 128u + 8u * (e >> 4); break;
    case 1: p = A + 128u + 8u * ((e & 3u) << 2); q = B + 8u * (e >> 2); break;
    case 2: p = B + 128u + 8u * (e & 15u); q = C + 8u * (e >> 4); break;
    default: p = C + 8u * ((e & 3u) << 2); q = C + 128u + 8u * (e >> 2); break;
  }
  return *(lds_ptr<uint32_t>)(static_cast<uintptr_t>(p)) ^ *(lds_ptr<uint32_t>)(static_cast<uintptr_t>(q));
}

// acc[w][j] ^= products of byte j of dword w of shards a, b, c (tables at `base`, 256-B
// aligned: v_perm drops the scaled piece into its low byte).
template <int RT>
__device__ __forceinline__ void wix_mac(uint32_t (&acc)[4][4], const uint4& a, const uint4& b,
                                        const uint4& c, uint32_t base) {
  static_assert(RT <= 4, "4-byte entries");
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t aw = word(a, w), bw = word(b, w), cw = word(c, w);
    // piece * 4 in every byte
    const uint32_t q0 = (aw << 2) & 0xfcfcfcfcu;
    const uint32_t q1 = ((aw >> 4) & 0x0c0c0c0cu) | ((bw << 4) & 0xf0f0f0f0u);
    const uint32_t q2 = ((bw >> 2) & 0x3c3c3c3cu) | ((cw << 6) & 0xc0c0c0c0u);
    const uint32_t q3 = cw & 0xfcfcfcfcu;
    uint32_t l[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t sel = 0x07060500u | static_cast<uint32_t>(j);
      l[j][0] = *(lds_ptr<uint32_t>)(static_cast<uintptr_t>(__builtin_amdgcn_perm(base, q0, sel)));
      l[j][1] = *(lds_ptr<uint32_t>)(static_cast<uintptr_t>(__builtin_amdgcn_perm(base + 256u, q1, sel)));
      l[j][2] = *(lds_ptr<uint32_t>)(static_cast<uintptr_t>(__builtin_amdgcn_perm(base + 512u, q2, sel)));
      l[j][3] = *(lds_ptr<uint32_t>)(static_cast<uintptr_t>(__builtin_amdgcn_perm(base + 768u, q3, sel)));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[w][j] = xor3(xor3(acc[w][j], l[j][0], l[j][1]), l[j][2], l[j][3]);
  }
}

// Row r's word = byte r of T[0..3].
template <int RT>
__device__ __forceinline__ uint32_t lds_row(const typename LdsAcc<RT>::T (&t)[4], int r) {
  uint32_t t0, t1, t2, t3;
  const int rr = r & 3;
  if constexpr (RT > 8) {
    const int d = r >> 2;
    t0 = t[0].v[d]; t1 = t[1].v[d]; t2 = t[2].v[d]; t3 = t[3].v[d];
  } else if constexpr (RT > 4) {
    const int sh = r >= 4 ? 32 : 0;
    t0 = static_cast<uint32_t>(t[0] >> sh);
    t1 = static_cast<uint32_t>(t[1] >> sh);
    t2 = static_cast<uint32_t>(t[2] >> sh);
    t3 = static_cast<uint32_t>(t[3] >> sh);
  } else {
    t0 = t[0]; t1 = t[1]; t2 = t[2]; t3 = t[3];
  }
  const uint32_t lo = __builtin_amdgcn_perm(t1, t0, 0x0c0c0400u | (0x0101u * rr));
  const uint32_t hi = __builtin_amdgcn_perm(t3, t2, 0x04000c0cu | (0x01010000u * rr));
  return lo | hi;
}

// x in every dword of an accumulator element (NOMATH ceiling variant only).
template <int RT>
__device__ __forceinline__ typename LdsAcc<RT>::T lds_splat(uint32_t x) {
  if constexpr (RT > 8) return typename LdsAcc<RT>::T{{x, x, x, x}};
  else if constexpr (RT > 4) return (static_cast<uint64_t>(x) << 32) | x;
  else return x;
}

template <int RT>
__device__ __forceinline__ typename LdsAcc<RT>::T lds_zero() {
  if constexpr (RT > 8) return typename LdsAcc<RT>::T{{0, 0, 0, 0}};
  else return 0;
}

// Byte r of a table entry / accumulator (row r's product for one data byte).
template <int RT>
__device__ __forceinline__ uint32_t lds_byte(const typename LdsAcc<RT>::T& t, int r) {
  if constexpr (RT > 8) {  // select, not an indexed load: a runtime index into t.v would
                          // put the accumulator in scratch for the whole kernel
    const uint32_t q = r < 4 ? t.v[0] : r < 8 ? t.v[1] : r < 12 ? t.v[2] : t.v[3];
    return (q >> (8 * (r & 3))) & 0xffu;
  }
  else return static_cast<uint32_t>(t >> (8 * r)) & 0xffu;
}

// The ragged tail S % 16 of every shard, run by the stripe's first tile (one byte per
// thread, the same LDS tables; first, not last: see vec_tail), so that launches with odd
// S need no second kernel
// (launch_apply sets ApplyArgs::tail_in_vec). Entry e of input i's low / high table is
// at lds0 + 32*W*i + W*e / + 16*W + W*e.
template <int RT>
__device__ __forceinline__ void lds_tail(const ApplyArgs& a, cptr<const uint8_t*> in,
                                         cptr<uint8_t*> out, uint32_t stripe, uint32_t lds0,
                                         uint32_t j) {
  constexpr int W = LdsAcc<RT>::W;
  const uint32_t nt = static_cast<uint32_t>(a.S - a.nvec * 16);
  if (j >= nt) return;
  const uint64_t b = a.nvec * 16 + j;
  typename LdsAcc<RT>::T t = lds_zero<RT>();
  for (int i0 = 0; i0 < a.K; i0 += tail_loads<RT>()) {
    uint32_t x[tail_loads<RT>()];
    tail_bytes<RT>(in, b, i0, a.K, x);
    for (int j = 0; j < tail_loads<RT>() && i0 + j < a.K; ++j) {
      const uint32_t base = lds0 + static_cast<uint32_t>(i0 + j) * 32u * W;
      t = t ^ lds_lookup<RT>(base + (x[j] & 15u) * W) ^
          lds_lookup<RT>(base + 16u * W + (x[j] >> 4) * W);
    }
  }
  bool bad = false;
  for (int r = 0; r < a.R && r < RT; ++r) {
    const uint8_t v = static_cast<uint8_t>(lds_byte<RT>(t, r));
    if ((a.verify_mask >> r) & 1u) bad |= out[r][b] != v;
    else out[r][b] = v;
  }
  if (bad) atomicOr(a.status + static_cast<size_t>(stripe) * a.status_stride, 1);
}

// Edge bytes of a REALIGN == 2 launch (see "aligned parity stores" above); threads
// 0..15 take the head bytes 0..15, threads 16.. the bytes from 16 (nvec - 1) on.
template <int RT>
__device__ __forceinline__ void lds_edges(const ApplyArgs& a, cptr<const uint8_t*> in,
                                          cptr<uint8_t*> out, uint32_t stripe, uint32_t lds0) {
  constexpr int W = LdsAcc<RT>::W;
  const uint64_t t0 = a.nvec * 16 - 16;  // nvec >= 1 on this path
  const uint32_t j = threadIdx.x;
  const bool head = j < 16u;
  const uint64_t b = head ? j : t0 + (j - 16u);
  if (!head && b >= a.S) return;
  if (head && b >= a.S) return;
  typename LdsAcc<RT>::T t = lds_zero<RT>();
  for (int i0 = 0; i0 < a.K; i0 += tail_loads<RT>()) {
    uint32_t x[tail_loads<RT>()];
    tail_bytes<RT>(in, b, i0, a.K, x);
    for (int jj = 0; jj < tail_loads<RT>() && i0 + jj < a.K; ++jj) {
      const uint32_t base = lds0 + static_cast<uint32_t>(i0 + jj) * 32u * W;
      t = t ^ lds_lookup<RT>(base + (x[jj] & 15u) * W) ^
          lds_lookup<RT>(base + 16u * W + (x[jj] >> 4) * W);
    }
  }
  bool bad = false;
  for (int r = 0; r < a.R && r < RT; ++r) {
    const uint8_t v = static_cast<uint8_t>(lds_byte<RT>(t, r));
    const bool verify = (a.verify_mask >> r) & 1u;
    const uint32_t f = (16u - (static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out[r])) & 15u)) & 15u;
    const bool mine = head ? (!verify && b < f)
                           : (verify || f == 0) ? b >= a.nvec * 16 : b >= t0 + f;
    if (!mine) continue;
    if (verify) bad |= out[r][b] != v;
    else out[r][b] = v;
  }
  if (bad) atomicOr(a.status + static_cast<size_t>(stripe) * a.status_stride, 1);
}

// ---- LDS-DMA ring (Policy::DMA) --------------------------------------------------------
// Each wave owns DMA slots of 1 KiB at dma_stage_off(K) + wave * DMA KiB of the block's LDS,
// behind the tables. Shard i's 64 lane vectors land in slot i % DMA through one
// global_load_lds_dwordx4 (lane l's 16 B at slot + 16 l; non-temporal), so the loads in flight
// hold LDS bytes instead of VGPRs; each lane reads its vector back with ds_read_b128 (slot + 16
// lane: the 64 lanes' reads cover the slot once, no bank conflict). The DMA is issued by inline
// asm, outside the compiler's vmcnt bookkeeping: issued through the builtin, hipcc waits
// vmcnt(0) before every ds_read of the kernel (the table lookups included), which would drain
// the ring at every lookup. The loop counts the DMAs itself (s_waitcnt vmcnt(n): all but the
// n youngest vector-memory operations done; inside the loop only DMAs are issued), and a slot
// is reloaded only after its ds_read_b128 has returned (lgkmcnt(0)). A wave reads only its own
// slots, so no barrier is needed: the DMA's vmcnt completes when its bytes are in LDS.
__host__ __device__ inline uint32_t dma_stage_off(int K, int RT) {
  return (static_cast<uint32_t>(K) * 32u * (RT > 8 ? 16u : 8u) + 1023u) & ~1023u;
}
// dynamic LDS of a DMA-ring launch (512-thread blocks: 8 waves)
inline size_t lds_bytes_dma(int K, int RT, int D) {
  return dma_stage_off(K, RT) + static_cast<size_t>(8 * 1024) * D;
}

__device__ __forceinline__ void dma16(const uint4* src, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_dst)
      : "memory");
}

// s_waitcnt vmcnt(n), n wave-uniform in [0, 7]
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
  }
}

// Waves per SIMD the LDS kernel may be limited to: 16-byte entries keep 8 b128 reads
// (32 VGPRs) in flight, which the register allocator only grants below 5 waves.
template <int RT>
constexpr int lds_max_waves() { return RT > 8 ? 4 : 8; }

template <int RT, class P>
__global__ __launch_bounds__(P::BS) __attribute__((amdgpu_waves_per_eu(P::WPE, lds_max_waves<RT>())))
void rs_apply_lds(ApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int BS = P::BS;
  constexpr int W = LdsAcc<RT>::W;
  using AccT = typename LdsAcc<RT>::T;
  const int K = a.K;
  // the launch passes R == RT; kept as a runtime stride so an RT instance can also
  // serve fewer rows (rows >= R are computed and dropped)
  const int R = a.R;
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.ltabs);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    for (int j = threadIdx.x; j < K * 2 * W; j += BS) dst[j] = src[j];
  }
  __syncthreads();
  if constexpr (P::WIX == 1) {  // the triples' 6-bit tables, from the nibble tables
    const uint32_t l0 = static_cast<uint32_t>(
        reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)smem));
    const uint32_t n = static_cast<uint32_t>(K / 3) * 256u;
    for (uint32_t j = threadIdx.x; j < n; j += BS)
      *(__attribute__((address_space(3))) uint32_t*)(static_cast<uintptr_t>(l0 + wix_base(K) + 4u * j)) =
          wix_entry(l0, j >> 8, (j >> 6) & 3u, j & 63u);
    __syncthreads();
  }
  // absolute LDS address of the tables (0 unless static LDS is ever added)
  const uint32_t lds0 = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)smem));
  constexpr int TV = P::TILE_VECS;
  const uint32_t tps = static_cast<uint32_t>((a.nvec + TV - 1) / TV);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.batch);
  // one tile per block (vec_grid), or (PERSIST) grid-stride over tiles so that the
  // table prologue is paid once per block; either way the blocks in flight cover a
  // window of consecutive t, which is what the tile order arranges
  const uint32_t t0 = a.t_base + (P::PERSIST ? blockIdx.x : block_tile<P::ORD>(blockIdx.x, gridDim.x));
  for (uint32_t t = t0; t < ntiles; t += (P::PERSIST ? gridDim.x : ntiles)) {
    uint32_t stripe, tile;
    map_tile<P::ORD>(t, tps, static_cast<uint32_t>(a.batch), stripe, tile);
    // REALIGN: wave w of the tile produces vectors tile*TV + 63w + lane (lanes 0..62)
    const uint32_t lane = threadIdx.x & 63u;
    constexpr uint32_t WV = P::WAVE_VECS;
    const uint64_t v0 = WV < 64 ? static_cast<uint64_t>(tile) * TV + (threadIdx.x >> 6) * WV + lane
                                : static_cast<uint64_t>(tile) * BS + threadIdx.x;
    cptr<const uint8_t*> in = as_const(a.in_tab) + static_cast<size_t>(stripe) * K;
    cptr<uint8_t*> out = as_const(a.out_tab) + static_cast<size_t>(stripe) * R;
    if constexpr (P::REALIGN == 2) {
      if (tile == 0) lds_edges<RT>(a, in, out, stripe, lds0);
    } else {
      if (a.tail_in_vec) {
        const uint32_t j = tail_lane<BS>(a.tail_in_vec, tile);
        if (j != ~0u) lds_tail<RT>(a, in, out, stripe, lds0, j);
      }
    }
    // lanes that store (REALIGN: lane 63 -- REALIGN 2: lanes 62, 63 -- and lanes past the
    // shard only load)
    const bool active = v0 < a.nvec && lane < WV && !(P::PROBE == 2 && lane == 63u);
    if (P::REALIGN ? (v0 - lane >= a.nvec) : !active) continue;  // REALIGN: whole wave idle
    auto ld = [&](int i) { return load16<P>(reinterpret_cast<const uint4*>(in[i]) + v0); };
    AccT acc[4][4];
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[w][j] = lds_zero<RT>();
    // Verify rows' stored vectors, loaded VPF shards before the end of the input loop:
    // a compare load issued after the loop leaves each wave a full memory latency with
    // nothing to do (profiles/r02/verify_prefetch/: one write + three compare rows 71.6
    // -> 74.1 %, four compare rows 78.0 -> 80.9 %)
    constexpr bool kVpf = P::VPF > 0 && RT <= 4;
    uint4 vpre[kVpf ? RT : 1];
#pragma unroll
    for (int r = 0; r < (kVpf ? RT : 1); ++r) vpre[r] = make_uint4(0, 0, 0, 0);

    if constexpr (P::REALIGN && P::WIX != 3) {
      static_assert(!P::NOMATH, "REALIGN: no NOMATH form");
      auto lda = [&](int i) { return ld_aligned<P>(in[i], v0, a.nvec); };
      if constexpr (P::REALIGN == 5) {
        // ring of three (aligned vector, lane 63's extra) pairs, realigned when consumed
        auto lde = [&](int i) {
          uint4 e = make_uint4(0, 0, 0, 0);
          if (lane == 63u) e = ld_aligned<P>(in[i], v0 + 1, a.nvec);
          return e;
        };
        uint4 x0 = lda(0), e0 = lde(0), x1 = x0, e1 = e0, x2 = x0, e2 = e0;
        if (K > 1) {
          x1 = lda(1);
          e1 = lde(1);
        }
#pragma unroll 1
        for (int i = 0; i < K; ++i) {
          if (i + 2 < K) {
            x2 = lda(i + 2);
            e2 = lde(i + 2);
          }
          lds_mac<RT>(acc, shift_from_next_e(x0, e0, static_cast<uint32_t>(reinterpret_cast<uintptr_t>(in[i])) & 15u),
                      lds0 + static_cast<uint32_t>(i) * 32u * W);
          x0 = x1;
          e0 = e1;
          x1 = x2;
          e1 = e2;
        }
      } else if constexpr (P::WIX == 2) {
        // triples of aligned loads (as the aligned triple loop below): the next triple's
        // three loads in flight while one is realigned and looked up
        const int KT = K / 3;
        uint4 x0 = lda(0), x1 = K > 1 ? lda(1) : x0, x2 = K > 2 ? lda(2) : x0;
#pragma unroll 1
        for (int g = 0; g < KT; ++g) {
          const int i = 3 * g + 3;
          const uint4 n0 = i < K ? lda(i) : x0, n1 = i + 1 < K ? lda(i + 1) : x0,
                      n2 = i + 2 < K ? lda(i + 2) : x0;
          const uint32_t b = lds0 + static_cast<uint32_t>(3 * g) * 32u * W;
          lds_mac<RT>(acc, realign_sel(in[3 * g], x0), b);
          lds_mac<RT>(acc, realign_sel(in[3 * g + 1], x1), b + 32u * W);
          lds_mac<RT>(acc, realign_sel(in[3 * g + 2], x2), b + 64u * W);
          x0 = n0;
          x1 = n1;
          x2 = n2;
        }
        if (3 * KT < K)
          lds_mac<RT>(acc, realign_sel(in[3 * KT], x0), lds0 + static_cast<uint32_t>(3 * KT) * 32u * W);
        if (3 * KT + 1 < K)
          lds_mac<RT>(acc, realign_sel(in[3 * KT + 1], x1), lds0 + static_cast<uint32_t>(3 * KT + 1) * 32u * W);
      } else {
        // ring of three aligned vectors, realigned when consumed
        uint4 x0 = lda(0), x1 = K > 1 ? lda(1) : x0, x2 = x0;
#pragma unroll 1
        for (int i = 0; i < K; ++i) {
          if (i + 2 < K) x2 = lda(i + 2);
          lds_mac<RT, P::SDWA>(acc, realign(in[i], x0), lds0 + static_cast<uint32_t>(i) * 32u * W);
          x0 = x1;
          x1 = x2;
        }
      }
    } else if constexpr (P::DMA > 0) {
      // LDS-DMA ring (see above): D shards in flight per wave, consumed in order
      constexpr int D = P::DMA;
      static_assert(D >= 2 && D <= 8, "vm_wait counts up to 7 younger DMAs");
      const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const uint32_t ring = __builtin_amdgcn_readfirstlane(lds0 + dma_stage_off(K, RT) + wave * (D * 1024u));
      const uint32_t mine = ring + lane * 16u;
      auto src = [&](int i) { return reinterpret_cast<const uint4*>(in[i]) + v0; };
      auto take = [&](uint32_t slot) {
        const u32x4 q = *(lds_ptr<u32x4>)(static_cast<uintptr_t>(mine + slot * 1024u));
        return make_uint4(q.x, q.y, q.z, q.w);
      };
      const int npre = K < D ? K : D;
      for (int i = 0; i < npre; ++i) dma16(src(i), ring + static_cast<uint32_t>(i) * 1024u);
      uint32_t slot = 0;
      int i = 0;
#pragma unroll 1
      for (; i < K - D; ++i) {  // steady state: D - 1 younger DMAs in flight
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
        const uint4 x = take(slot);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read: reload it
        dma16(src(i + D), ring + slot * 1024u);
        lds_mac<RT>(acc, x, lds0 + static_cast<uint32_t>(i) * 32u * W);
        slot = slot + 1 == D ? 0u : slot + 1;
      }
#pragma unroll 1
      for (; i < K; ++i) {  // the last D shards: nothing left to issue
        vm_wait(K - 1 - i);
        lds_mac<RT>(acc, take(slot), lds0 + static_cast<uint32_t>(i) * 32u * W);
        slot = slot + 1 == D ? 0u : slot + 1;
      }
    } else if constexpr (P::WIX == 3 || P::WIX == 5) {
      // groups of G = 3 (WIX 3) or 2 (WIX 5) shards double-buffered in two register sets,
      // with no conditional load anywhere: the loop runs while both its groups exist, and
      // the last one or two groups with the K % G remainder run as straight-line tails, one
      // per case (a load skipped on a runtime condition, or a join after one, makes the
      // compiler wait for every load in flight; so do the rotation copies of a ring). Set A
      // is consumed while set B loads and vice versa: 2G loads in flight. K >= G.
      // (REALIGN 2 with WIX 3: the realigning kernel's aligned loads double-buffered the
      // same way, each vector realigned when its group is consumed)
      constexpr int G = P::WIX == 3 ? 3 : 2;
      const int KG = K / G, rem = K - G * KG;
      const uint32_t tb = 32u * W;
      uint4 A[G], B[G];
      auto ldx = [&](int i) {
        if constexpr (P::REALIGN != 0) return ld_aligned<P>(in[i], v0, a.nvec);
        else return ld(i);
      };
      auto load_g = [&](uint4 (&x)[G], int i0) {
#pragma unroll
        for (int j = 0; j < G; ++j) x[j] = ldx(i0 + j);
        __builtin_amdgcn_sched_barrier(0);  // the loads stay ahead of the lookups
      };
      auto mac_g = [&](const uint4 (&x)[G], int i0, int n) {
        const uint32_t b = lds0 + static_cast<uint32_t>(i0) * tb;
#pragma unroll
        for (int j = 0; j < G; ++j)
          if (j < n) {
            if constexpr (P::REALIGN != 0)
              lds_mac<RT>(acc, realign_sel(in[i0 + j], x[j]), b + static_cast<uint32_t>(j) * tb);
            else
              lds_mac<RT>(acc, x[j], b + static_cast<uint32_t>(j) * tb);
          }
      };
      auto load_rem = [&](uint4 (&x)[G], int i0, int n) {  // n = 1 .. G - 1, uniform
        if (n == 1) {
          x[0] = ldx(i0);
        } else {
          x[0] = ldx(i0);
          x[1] = ldx(i0 + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      // VPF: the Verify rows' compare loads go out with the loads of the last groups
      auto load_vpf = [&]() {
        if constexpr (kVpf) {
#pragma unroll
          for (int r = 0; r < RT; ++r)
            if (r < R && ((a.verify_mask >> r) & 1u))
              vpre[r] = load16<P>(reinterpret_cast<const uint4*>(out[r]) + v0);
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      load_g(A, 0);
      int g = 0;
#pragma unroll 1
      for (; g + 2 < KG; g += 2) {
        load_g(B, G * g + G);
        mac_g(A, G * g, G);
        load_g(A, G * g + 2 * G);
        mac_g(B, G * g + G, G);
      }
      const int i = G * g + G;  // first shard after group g
      if (KG - g == 2) {        // groups g (in A) and g + 1, then the remainder
        load_g(B, i);
        load_vpf();
        if (rem == 0) {
          mac_g(A, G * g, G);
          mac_g(B, i, G);
        } else if (rem == 1) {
          mac_g(A, G * g, G);
          load_rem(A, i + G, 1);
          mac_g(B, i, G);
          mac_g(A, i + G, 1);
        } else {
          mac_g(A, G * g, G);
          load_rem(A, i + G, 2);
          mac_g(B, i, G);
          mac_g(A, i + G, 2);
        }
      } else {  // group g (in A), then the remainder
        if (rem == 0) {
          load_vpf();
          mac_g(A, G * g, G);
        } else if (rem == 1) {
          load_rem(B, i, 1);
          load_vpf();
          mac_g(A, G * g, G);
          mac_g(B, i, 1);
        } else {
          load_rem(B, i, 2);
          load_vpf();
          mac_g(A, G * g, G);
          mac_g(B, i, 2);
        }
      }
    } else if constexpr (P::WIX) {
      // triples: the next triple's three loads are in flight while one is consumed; the
      // K % 3 shards left over take the nibble tables (WIX 4, A/B probe: loads past K
      // leave zeros instead of a copy of x0)
      const int KT = K / 3;
      // VPF: the Verify rows' compare loads go out with the triple whose loads reach K - VPF
      // (or with the last triple when the remainder shards do)
      const int gv = kVpf ? std::min(KT - 1, (std::max(3, K - P::VPF) - 3) / 3) : -1;
      constexpr bool kz = P::WIX == 4;
      const uint4 zv = make_uint4(0, 0, 0, 0);
      uint4 x0 = ld(0), x1 = K > 1 ? ld(1) : (kz ? zv : x0), x2 = K > 2 ? ld(2) : (kz ? zv : x0);
#pragma unroll 1
      for (int g = 0; g < KT; ++g) {
        const int i = 3 * g + 3;
        const uint4 d = kz ? zv : x0;
        const uint4 n0 = i < K ? ld(i) : d, n1 = i + 1 < K ? ld(i + 1) : d,
                    n2 = i + 2 < K ? ld(i + 2) : d;
        if constexpr (kVpf) {
          if (g == gv) {
#pragma unroll
            for (int r = 0; r < RT; ++r)
              if (r < R && ((a.verify_mask >> r) & 1u))
                vpre[r] = load16<P>(reinterpret_cast<const uint4*>(out[r]) + v0);
          }
        }
        if constexpr (P::WIX == 1) {
          wix_mac<RT>(acc, x0, x1, x2, lds0 + wix_base(K) + 1024u * static_cast<uint32_t>(g));
        } else {
          const uint32_t b = lds0 + static_cast<uint32_t>(3 * g) * 32u * W;
          lds_mac<RT>(acc, x0, b);
          lds_mac<RT>(acc, x1, b + 32u * W);
          lds_mac<RT>(acc, x2, b + 64u * W);
        }
        x0 = n0;
        x1 = n1;
        x2 = n2;
      }
      if (3 * KT < K) lds_mac<RT>(acc, x0, lds0 + static_cast<uint32_t>(3 * KT) * 32u * W);
      if (3 * KT + 1 < K) lds_mac<RT>(acc, x1, lds0 + static_cast<uint32_t>(3 * KT + 1) * 32u * W);
    } else if constexpr (P::RING == 0) {
      // ring of three shard vectors: shard i is consumed while i+1, i+2 load
      uint4 x0 = ld(0), x1 = K > 1 ? ld(1) : x0, x2 = x0;
#pragma unroll 1
      for (int i = 0; i < K; ++i) {
        if (i + 2 < K) x2 = ld(i + 2);
        if constexpr (kVpf) {
          if (i == (K > P::VPF ? K - P::VPF : 0)) {
#pragma unroll
            for (int r = 0; r < RT; ++r)
              if (r < R && ((a.verify_mask >> r) & 1u))
                vpre[r] = load16<P>(reinterpret_cast<const uint4*>(out[r]) + v0);
          }
        }
        if constexpr (P::NOMATH) {
#pragma unroll
          for (int w = 0; w < 4; ++w) acc[w][0] = acc[w][0] ^ lds_splat<RT>(word(x0, w));
        } else {
          lds_mac<RT, P::SDWA>(acc, x0, lds0 + static_cast<uint32_t>(i) * 32u * W);
        }
        x0 = x1;
        x1 = x2;
      }
    } else {
      // PD+1 slots, shard i in slot i % NR; shard i+PD loads into the slot shard i-1 left
      constexpr int PD = P::PD, NR = P::PD + 1;
      uint4 xr[NR];
#pragma unroll
      for (int s = 0; s < PD; ++s) xr[s] = s < K ? ld(s) : make_uint4(0, 0, 0, 0);
#pragma unroll 1
      for (int i0 = 0; i0 < K; i0 += NR) {
#pragma unroll
        for (int s = 0; s < NR; ++s) {
          const int i = i0 + s;
          if (i < K) {
            if (i + PD < K) xr[(s + PD) % NR] = ld(i + PD);
            if constexpr (P::NOMATH) {
#pragma unroll
              for (int w = 0; w < 4; ++w) acc[w][0] = acc[w][0] ^ lds_splat<RT>(word(xr[s], w));
            } else {
              lds_mac<RT, P::SDWA>(acc, xr[s], lds0 + static_cast<uint32_t>(i) * 32u * W);
            }
          }
        }
      }
    }

    bool bad = false;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      if (r >= R) continue;  // wave-uniform
      const uint4 o = make_uint4(lds_row<RT>(acc[0], r), lds_row<RT>(acc[1], r),
                                 lds_row<RT>(acc[2], r), lds_row<RT>(acc[3], r));
      uint4* dst = reinterpret_cast<uint4*>(out[r]) + v0;
      if constexpr (P::REALIGN == 2) {
        if (!((a.verify_mask >> r) & 1u)) {
          const uint32_t mo = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out[r])) & 15u;
          if (mo) {  // wave-uniform: aligned block at out[r] + f + 16 v0 (see above)
            const uint32_t f = 16u - mo;
            const uint4 O = shift_from_next(o, f);  // every lane: DPP reads lane + 1
            if (active && v0 + 1 < a.nvec)
              store16<P>(reinterpret_cast<uint4*>(out[r] + f) + v0, O);
            continue;
          }
        }
      }
      if (P::REALIGN && !active) continue;
      if ((a.verify_mask >> r) & 1u) {
        // non-temporal like the input loads: the all-Verify decode (every download,
        // codec.go:59) ran 76.3-77.9 -> 79.7-80.2 % with them (round-2 probe, profiles/notebook_r01_r04.md)
        uint4 y;
        if constexpr (kVpf) y = vpre[r];
        else y = load16<P>(dst);
        if constexpr (P::NOMATH)  // compares junk: keep the load, not a status atomic per lane
          bad |= ((y.x ^ o.x) | (y.y ^ o.y) | (y.z ^ o.z) | (y.w ^ o.w)) == 0x9e3779b9u;
        else
          bad |= ((y.x ^ o.x) | (y.y ^ o.y) | (y.z ^ o.z) | (y.w ^ o.w)) != 0;
      } else {
        store16<P>(dst, o);
      }
    }
    if (bad) atomicOr(a.status + static_cast<size_t>(stripe) * a.status_stride, 1);
  }
}

// ---- traffic ceilings of a launch (measurement only; rs_plan_launch_ceiling) ----------
// The launch's read streams alone (its K inputs and its Verify rows) and its write
// streams alone (its other rows), on the production grid and tile order: 512 threads, one
// 16-B vector per lane per shard, non-temporal, no LDS. bench.py adds the two times: the
// HBM rate of the launch's bytes if its reads and writes each ran at their own best rate
// one after the other, an achievable-rate denominator that does not depend on how the
// kernel interleaves them. The read kernel stores nothing (its XOR reaches memory only if
// it equals a value random data never gives, which keeps the loads alive); the write
// kernel stores a lane pattern. On a misaligned batch (Split layout) both time aligned
// 16-B accesses -- the traffic the realigning kernel issues -- not unaligned ones: reads
// from each shard's base rounded down to 16 B (same page), stores from its first 16-B
// boundary on, inside the shard.
__device__ __forceinline__ const uint4* align16(const uint8_t* p) {
  return reinterpret_cast<const uint4*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
}

// AL > 16 (measurement probe): each shard is read from its first AL-byte boundary on, so
// every wave-instruction's 1 KiB load starts on an AL-byte boundary
template <int AL>
__device__ __forceinline__ const uint4* align_read(const uint8_t* p) {
  if constexpr (AL == 16) return align16(p);
  else return reinterpret_cast<const uint4*>((reinterpret_cast<uintptr_t>(p) + AL - 1) & ~uintptr_t(AL - 1));
}

template <int ORD, int AL = 16>
__global__ __launch_bounds__(512) void rs_stream_read(ApplyArgs a) {
  const uint32_t tps = static_cast<uint32_t>((a.nvec + 511) / 512);
  uint32_t stripe, tile;
  map_tile<ORD>(a.t_base + block_tile<ORD>(blockIdx.x, gridDim.x), tps,
                static_cast<uint32_t>(a.batch), stripe, tile);
  const uint64_t v0 = static_cast<uint64_t>(tile) * 512 + threadIdx.x;
  if (v0 + (AL > 16 ? AL / 16 : 0) >= a.nvec) return;
  cptr<const uint8_t*> in = as_const(a.in_tab) + static_cast<size_t>(stripe) * a.K;
  cptr<uint8_t*> out = as_const(a.out_tab) + static_cast<size_t>(stripe) * a.R;
  using P = Policy<2, 1, true, true, false, 512>;
  uint4 acc = make_uint4(0, 0, 0, 0);
  auto mix = [&acc](const uint4& x) {
    acc.x ^= x.x; acc.y ^= x.y; acc.z ^= x.z; acc.w ^= x.w;
  };
  // 8 loads in flight per lane before any is consumed (64 VGPRs, 8 waves per SIMD)
  for (int i0 = 0; i0 < a.K; i0 += 8) {
    uint4 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i0 + j < a.K) x[j] = load16<P>(align_read<AL>(in[i0 + j]) + v0);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i0 + j < a.K) mix(x[j]);
  }
  for (int r0 = 0; r0 < a.R; r0 += 8) {
    uint4 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (r0 + j < a.R && ((a.verify_mask >> (r0 + j)) & 1u))
        x[j] = load16<P>(align_read<AL>(out[r0 + j]) + v0);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (r0 + j < a.R && ((a.verify_mask >> (r0 + j)) & 1u)) mix(x[j]);
  }
  if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u && acc.z == 0xf39cc060u && acc.w == 0x5cedc834u)
    a.status[0] = static_cast<int>(v0);
}

// AL > 16 (measurement probe): each row is written from its first AL-byte boundary on, so
// every wave-instruction's 1 KiB store starts on an AL-byte boundary
template <int ORD, int AL = 16>
__global__ __launch_bounds__(512) void rs_stream_write(ApplyArgs a) {
  const uint32_t tps = static_cast<uint32_t>((a.nvec + 511) / 512);
  uint32_t stripe, tile;
  map_tile<ORD>(a.t_base + block_tile<ORD>(blockIdx.x, gridDim.x), tps,
                static_cast<uint32_t>(a.batch), stripe, tile);
  const uint64_t v0 = static_cast<uint64_t>(tile) * 512 + threadIdx.x;
  if (v0 >= a.nvec) return;
  cptr<uint8_t*> out = as_const(a.out_tab) + static_cast<size_t>(stripe) * a.R;
  using P = Policy<2, 1, true, true, false, 512>;
  const uint32_t x = static_cast<uint32_t>(v0) * 0x01000193u;
  for (int r = 0; r < a.R; ++r)
    if (!((a.verify_mask >> r) & 1u)) {
      // aligned blocks inside the row: from the first 16-B boundary at or after its base,
      // one block fewer when the base is misaligned (never a byte outside [base, base + S))
      const uintptr_t q = reinterpret_cast<uintptr_t>(out[r]);
      const uintptr_t up = (q + AL - 1) & ~uintptr_t(AL - 1);
      if (up + 16 * (v0 + 1) > q + a.S) continue;
      store16<P>(reinterpret_cast<uint4*>(up) + v0, make_uint4(x, x + 1, x + 2, x + r));
    }
}


// One byte position per lane over [b0, S): ragged tails (S % 16).
template <int RT>
__global__ __launch_bounds__(kBlock) void rs_apply_bytes(ApplyArgs a, uint64_t b0) {
  const uint64_t b = b0 + static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (b >= a.S) return;
  const cptr<uint32_t> tabs = as_const(a.tabs);
  for (int stripe = blockIdx.y; stripe < a.batch; stripe += gridDim.y) {
    cptr<const uint8_t*> in = as_const(a.in_tab) + static_cast<size_t>(stripe) * a.K;
    cptr<uint8_t*> out = as_const(a.out_tab) + static_cast<size_t>(stripe) * RT;
    uint32_t acc[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = 0;
    for (int i = 0; i < a.K; ++i) {
      const Sel s = selectors(in[i][b]);
      const cptr<uint32_t> t = tabs + static_cast<size_t>(i) * RT * 5;
#pragma unroll
      for (int r = 0; r < RT; ++r) acc[r] = fma1(acc[r], gf_mul4(s, t + r * 5));
    }
    bool bad = false;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const uint8_t v = static_cast<uint8_t>(acc[r]);
      if ((a.verify_mask >> r) & 1u) bad |= out[r][b] != v;
      else out[r][b] = v;
    }
    if (bad) atomicOr(a.status + static_cast<size_t>(stripe) * a.status_stride, 1);
  }
}

// ---- one-dispatch small calls (rs_kernels.hpp SmallArgs) -------------------------------
// A host-memory call of a few KiB spent ~29 us in an H2D blit, the kernel and a D2H blit,
// each a dispatch that waits for the previous one (6.6 + 7.6 + 4.2 us on the GPU plus ~20 us
// on the host, profiles/r03/small_path/r03_smalltrace2). This kernel reads the
// lane's host-coherent staging buffer over PCIe and writes the outputs back into it: one
// dispatch per call. Each lane owns one 16-B column vector of one stripe, so a call waits
// for few PCIe round trips; the GF multiply is the v_perm form (tables in SGPRs, no LDS prologue).
// 16 loads are issued before any is consumed (one PCIe round trip for k <= 16).
// Shard pitch in staging is S rounded up to 16, so the last vector of a shard covers bytes
// past S: they are computed and stored (never copied out) and masked out of compares.
template <int RT>
__device__ __forceinline__ void small_vector(const SmallArgs& a, uint32_t v) {
  const uint8_t* s = a.base + static_cast<size_t>(blockIdx.y) * a.spitch;
  const cptr<uint32_t> tabs = as_const(a.tabs);
  // shard indices as dwords (scalar loads; byte loads would be per-lane vector loads, each
  // waited for before the data load it addresses)
  const cptr<uint32_t> idx = as_const(reinterpret_cast<const uint32_t*>(a.idx));
  uint32_t acc[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[r][w] = 0;
  // 16 loads in flight before any is consumed: a call with k <= 16 waits for one PCIe round
  // trip of reads. Loads past K re-read shard K-1 (unconditional loads keep them in flight
  // together; their values are not used).
  for (int i0 = 0; i0 < a.K; i0 += 16) {
    uint32_t iw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) iw[q] = i0 == 0 ? a.idx_in[q] : idx[(i0 >> 2) + q];
    const uint32_t lw = a.K <= 16 ? a.idx_in[(a.K - 1) >> 2] : idx[(a.K - 1) >> 2];
    const uint32_t last = lw >> (8 * ((a.K - 1) & 3)) & 0xffu;
    uint4 x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t sh = i0 + j < a.K ? (iw[j >> 2] >> (8 * (j & 3))) & 0xffu : last;
      x[j] = *(reinterpret_cast<const uint4*>(s + a.cpitch * sh) + v);
    }
    // keep the 16 loads ahead of every use (left alone, the scheduler sank each load next
    // to its consumer: 16 PCIe round trips one after another)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      // past K: input 0 through shard K-1's tables adds nothing (no branch in the loop)
      const bool in = i0 + j < a.K;
      if (!in) x[j] = make_uint4(0, 0, 0, 0);
      const cptr<uint32_t> t = tabs + static_cast<size_t>(in ? i0 + j : a.K - 1) * RT * 5;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const Sel sel = selectors(word(x[j], w));
#pragma unroll
        for (int r = 0; r < RT; ++r) acc[r][w] = fma1(acc[r][w], gf_mul4(sel, t + r * 5));
      }
    }
  }
  // bytes of this vector that lie inside the shard (compares ignore the rest)
  const uint32_t live = a.S - v * 16u >= 16u ? 16u : a.S - v * 16u;
  uint32_t mask[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t b = live > 4u * w ? live - 4u * w : 0u;
    mask[w] = b >= 4u ? ~0u : (1u << (8u * b)) - 1u;
  }
  bool bad = false;
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const uint32_t row = (a.idx_out[r >> 2] >> (8 * (r & 3))) & 0xffu;
    uint4* dst = reinterpret_cast<uint4*>(const_cast<uint8_t*>(s) + a.cpitch * row) + v;
    const uint4 o = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
    if ((a.verify_mask >> r) & 1u) {
      const uint4 y = *dst;
      bad |= (((y.x ^ o.x) & mask[0]) | ((y.y ^ o.y) & mask[1]) | ((y.z ^ o.z) & mask[2]) |
              ((y.w ^ o.w) & mask[3])) != 0;
    } else {
      *dst = o;
    }
  }
  if (bad) a.status[blockIdx.y] = 1;  // every writer stores the same flag: no atomic
}

// The completion flag (SmallArgs::done): the host spins on it instead of waiting for the
// runtime's completion signal, which returned ~5 us after the kernel had ended
// (profiles/r03/small_path/r03_smalltrace2). Every thread makes its own stores visible
// system-wide (a system-scope release per wave: the workgroup-scope release in __syncthreads does not wait
// for another wave's PCIe stores), then the block counts itself done on a device-memory
// counter; the last block resets the counter and releases the call's sequence number into
// the host flag.
template <int RT>
__global__ __launch_bounds__(256) void rs_apply_small(SmallArgs a) {
  const uint32_t v = blockIdx.x * 256u + threadIdx.x;
  if (v < a.nvec) small_vector<RT>(a, v);
  if (a.done) {  // launch-uniform
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence_system();
      const unsigned total = gridDim.x * gridDim.y;
      if (atomicAdd(a.counter, 1u) == total - 1u) {
        atomicExch(a.counter, 0u);
        __threadfence_system();
        __hip_atomic_store(a.done, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// Grid for the vector kernel: one tile per block, or (PERSIST) a fixed grid of
// `blocks_per_cu` blocks on each of the 256 CUs.
template <class P>
inline unsigned vec_grid(uint64_t nvec, int batch, int blocks_per_cu = 8) {
  const uint64_t tile = static_cast<uint64_t>(P::TILE_VECS);
  const uint64_t ntiles = (nvec + tile - 1) / tile * static_cast<uint64_t>(batch);
  if (P::PERSIST) return static_cast<unsigned>(std::min<uint64_t>(ntiles, 256ull * blocks_per_cu));
  return static_cast<unsigned>(ntiles);
}

}  // namespace dev
}  // namespace callfs
