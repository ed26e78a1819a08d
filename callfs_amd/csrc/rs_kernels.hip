// GF(2^8) shard-matrix kernels for gfx950 (MI355X, CDNA4).
//
// Replaces the SIMD kernels of github.com/klauspost/reedsolomon v1.13.3 (go.mod:13)
// behind erasure/codec.go:36 (Encode), :55 (Reconstruct) and :59 (Verify).
//
// Design (see DESIGN.md "Kernels"):
//  * Byte-wise integer work, HBM-bound: no MFMA, no LDS. Each lane owns one 16-byte
//    column vector of a stripe and streams it through all K input shards with
//    global_load_dwordx4, keeping the R output vectors in registers, then writes (or,
//    for Verify rows, compares) them once: (K + R) * 16 bytes of compulsory traffic
//    per lane, nothing re-read.
//  * GF multiply by a wave-uniform coefficient c on 4 packed bytes = three v_perm_b32
//    byte-selects from 8-byte tables: c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6]
//    (gf256.hpp perm_tables). The three selectors depend only on the data word, so
//    they are shared by all R rows; per row and data word: 3 v_perm + 2 XOR. The
//    tables are wave-uniform and arrive by s_load into SGPRs (no LDS, no bank
//    conflicts on random data, no VGPR tables).
//  * Ragged tails (S % 16) and unaligned shard pointers take the byte kernel.
#include "rs_kernels.hpp"

#include <array>
#include <utility>

namespace callfs {

namespace {

constexpr int kBlock = 256;

// Read-only, wave-uniform tables (shard pointers, v_perm tables) are read through the
// constant address space so they arrive by s_load into SGPRs.
template <class T>
using cptr = const __attribute__((address_space(4))) T*;

template <class T>
__device__ __forceinline__ cptr<T> as_const(const T* p) {
  return (cptr<T>)(p);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

// c*x for 4 packed bytes, as the three partial products (XOR them to finish).
struct Prod {
  uint32_t p0, p1, p2;
};

struct Sel {
  uint32_t i0, i1, i2;
};

__device__ __forceinline__ Sel selectors(uint32_t x) {
  return Sel{x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

__device__ __forceinline__ Prod gf_mul4(const Sel& s, cptr<uint32_t> t) {
  return Prod{__builtin_amdgcn_perm(t[1], t[0], s.i0), __builtin_amdgcn_perm(t[3], t[2], s.i1),
              __builtin_amdgcn_perm(t[4], t[4], s.i2)};
}

// acc ^= a*x ^ b*y with three v_bitop3 XORs for the six partial products.
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

template <int RT>
__device__ __forceinline__ void mac_pair(uint32_t (&acc)[RT][4], const uint4& xa, const uint4& xb,
                                         cptr<uint32_t> ta, cptr<uint32_t> tb) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const Sel sa = selectors(word(xa, w)), sb = selectors(word(xb, w));
#pragma unroll
    for (int r = 0; r < RT; ++r)
      acc[r][w] = fma2(acc[r][w], gf_mul4(sa, ta + r * 5), gf_mul4(sb, tb + r * 5));
  }
}

template <int RT>
__device__ __forceinline__ void mac_one(uint32_t (&acc)[RT][4], const uint4& xa,
                                        cptr<uint32_t> ta) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const Sel sa = selectors(word(xa, w));
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r][w] = fma1(acc[r][w], gf_mul4(sa, ta + r * 5));
  }
}

// KT: compile-time K (0 = runtime a.K). RT: rows per launch. WPE: minimum waves per
// SIMD the register allocation must allow. One 16-B column vector per lane; the input
// shards are consumed in pairs with the next pair's loads in flight (software
// pipeline, depth 1), so VGPR use stays independent of K.
template <int KT, int RT, int WPE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
void rs_apply_vec(ApplyArgs a) {
  const int K = KT ? KT : a.K;
  const uint64_t v = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (v >= a.nvec) return;
  const int npairs = K >> 1;

  for (int stripe = blockIdx.y; stripe < a.batch; stripe += gridDim.y) {
    cptr<const uint8_t*> in = as_const(a.in_tab) + static_cast<size_t>(stripe) * K;
    cptr<uint8_t*> out = as_const(a.out_tab) + static_cast<size_t>(stripe) * RT;
    auto ld = [&](int i) { return reinterpret_cast<const uint4*>(in[i])[v]; };
    const cptr<uint32_t> tabs = as_const(a.tabs);

    uint32_t acc[RT][4];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int w = 0; w < 4; ++w) acc[r][w] = 0;

    uint4 xa = make_uint4(0, 0, 0, 0), xb = xa;
    if (npairs) {
      xa = ld(0);
      xb = ld(1);
    }
#pragma unroll 1
    for (int p = 0; p < npairs; ++p) {
      uint4 ya = xa, yb = xb;
      if (p + 1 < npairs) {
        ya = ld(2 * p + 2);
        yb = ld(2 * p + 3);
      }
      const cptr<uint32_t> ta = tabs + static_cast<size_t>(2 * p) * RT * 5;
      mac_pair<RT>(acc, xa, xb, ta, ta + RT * 5);
      xa = ya;
      xb = yb;
    }
    if (K & 1) mac_one<RT>(acc, ld(K - 1), tabs + static_cast<size_t>(K - 1) * RT * 5);

    bool bad = false;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      uint4* __restrict__ dst = reinterpret_cast<uint4*>(out[r]);
      const uint4 o = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
      if ((a.verify_mask >> r) & 1u) {
        const uint4 y = dst[v];
        bad |= ((y.x ^ o.x) | (y.y ^ o.y) | (y.z ^ o.z) | (y.w ^ o.w)) != 0;
      } else {
        dst[v] = o;
      }
    }
    if (bad) atomicOr(a.status, 1);
  }
}

// One byte position per lane over [b0, S): ragged tails and unaligned pointers.
template <int RT>
__global__ __launch_bounds__(kBlock) void rs_apply_bytes(ApplyArgs a, uint64_t b0) {
  const uint64_t b = b0 + static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (b >= a.S) return;
  for (int stripe = blockIdx.y; stripe < a.batch; stripe += gridDim.y) {
    cptr<const uint8_t*> in = as_const(a.in_tab) + static_cast<size_t>(stripe) * a.K;
    cptr<uint8_t*> out = as_const(a.out_tab) + static_cast<size_t>(stripe) * RT;
    const cptr<uint32_t> tabs = as_const(a.tabs);
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
    if (bad) atomicOr(a.status, 1);
  }
}

using VecFn = void (*)(ApplyArgs);
using ByteFn = void (*)(ApplyArgs, uint64_t);

#ifndef RS_VEC_WPE
#define RS_VEC_WPE 4
#endif

template <int KT, int RT>
constexpr VecFn vec_kernel() {
  return &rs_apply_vec<KT, RT, RS_VEC_WPE>;
}

// Compile-time K for 1..16 (full unroll: all K loads in flight per lane); runtime K
// beyond. Indexed [K][R-1].
template <int RT, int... Ks>
constexpr auto vec_row(std::integer_sequence<int, Ks...>) {
  return std::array<VecFn, sizeof...(Ks)>{vec_kernel<Ks, RT>()...};
}

template <int... Rs>
constexpr auto vec_table(std::integer_sequence<int, Rs...>) {
  // table[r][k] with k = 0 meaning runtime K
  return std::array<std::array<VecFn, 17>, sizeof...(Rs)>{
      vec_row<Rs + 1>(std::make_integer_sequence<int, 17>{})...};
}

template <int... Rs>
constexpr auto byte_table(std::integer_sequence<int, Rs...>) {
  return std::array<ByteFn, sizeof...(Rs)>{&rs_apply_bytes<Rs + 1>...};
}

const auto kVec = vec_table(std::make_integer_sequence<int, kMaxRowsPerLaunch>{});
const auto kByte = byte_table(std::make_integer_sequence<int, kMaxRowsPerLaunch>{});

}  // namespace

hipError_t launch_apply(ApplyArgs a, bool aligned, hipStream_t stream) {
  if (a.R < 1 || a.R > kMaxRowsPerLaunch || a.K < 1 || a.K > kMaxK || a.batch < 1)
    return hipErrorInvalidValue;
  if (a.S == 0) return hipSuccess;
  const unsigned gy = static_cast<unsigned>(a.batch < 65535 ? a.batch : 65535);
  uint64_t tail0 = 0;
  if (aligned) {
    a.nvec = a.S / 16;
    tail0 = a.nvec * 16;
    if (a.nvec) {
      const uint64_t gx = (a.nvec + kBlock - 1) / kBlock;
      VecFn fn = kVec[a.R - 1][a.K <= 16 ? a.K : 0];
      hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(gx), gy), dim3(kBlock), 0, stream, a);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  } else {
    a.nvec = 0;
  }
  if (tail0 < a.S) {
    const uint64_t gx = (a.S - tail0 + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(kByte[a.R - 1], dim3(static_cast<unsigned>(gx), gy), dim3(kBlock), 0,
                       stream, a, tail0);
    return hipGetLastError();
  }
  return hipSuccess;
}

}  // namespace callfs
