// Batched SHA-256 for gfx950: erasure.ShardChecksum (erasure/codec.go:81-84) over
// many device-resident shards at once.
//
// SHA-256 of one message is a serial chain of 64-byte compressions, so the only
// parallelism is across messages: one lane per message (MPB messages per 64-lane
// wave, the rest of the wave idle, to spread few messages over more SIMDs). Rotates
// lower to v_alignbit_b32, Ch/Maj/XOR3 to v_bitop3_b32, the sums to v_add3_u32. Each
// lane issues the next block's four 16-B loads before the current block's 64 rounds.
// Messages are read as dwordx4 at any alignment; padding and the big-endian length
// follow FIPS 180-4 exactly (bit-exact with Go's crypto/sha256).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sha256.hpp"

namespace callfs {

namespace {

__constant__ uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

__device__ __forceinline__ uint32_t be32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One compression; w holds the 16 big-endian message words.
__device__ __forceinline__ void compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    if (t >= 16) {
      const uint32_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
      const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      w[t & 15] = w[t & 15] + s0 + w[(t + 9) & 15] + s1;
    }
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // e ? f : g
    const uint32_t t1 = h + S1 + ch + kK[t] + w[t & 15];
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t maj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + maj;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void load_block16(const uint8_t* p, uint4 (&q)[4]) {
  const u32x4* v = reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4 x = __builtin_nontemporal_load(v + i);
    q[i] = make_uint4(x.x, x.y, x.z, x.w);
  }
}

template <int MPB>
__global__ __launch_bounds__(64) void sha256_kernel(Sha256Args a) {
  if (static_cast<int>(threadIdx.x) >= MPB) return;
  const int idx = blockIdx.x * MPB + threadIdx.x;
  if (idx >= a.count) return;
  const uint8_t* msg = a.msgs[idx];
  const uint64_t len = a.lens[idx];
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint64_t full = len / 64;
  uint32_t w[16];
  // 16-B loads at any byte address (legal on gfx950, rs_kernels.hpp): no byte path
  uint4 q[4];
  if (full) load_block16(msg, q);
  for (uint64_t blk = 0; blk < full; ++blk) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[4 * i + 0] = be32(q[i].x);
      w[4 * i + 1] = be32(q[i].y);
      w[4 * i + 2] = be32(q[i].z);
      w[4 * i + 3] = be32(q[i].w);
    }
    if (blk + 1 < full) load_block16(msg + 64 * (blk + 1), q);
    compress(st, w);
  }
  // tail: remaining bytes, 0x80, zeros, 64-bit big-endian bit length (1 or 2 blocks)
  const uint32_t rem = static_cast<uint32_t>(len - full * 64);
  const uint8_t* p = msg + full * 64;
  const int nblk = rem < 56 ? 1 : 2;
  for (int tb = 0; tb < nblk; ++tb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t pos = tb * 64 + 4 * i + j;
        uint32_t byte = 0;
        if (pos < rem) byte = p[pos];
        else if (pos == rem) byte = 0x80;
        word = (word << 8) | byte;
      }
      w[i] = word;
    }
    if (tb == nblk - 1) {
      const uint64_t bits = len * 8;
      w[14] = static_cast<uint32_t>(bits >> 32);
      w[15] = static_cast<uint32_t>(bits);
    }
    compress(st, w);
  }
  uint32_t* o = a.digests + static_cast<size_t>(idx) * 8;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = be32(st[i]);  // digest bytes in order
}

}  // namespace

hipError_t launch_sha256(const Sha256Args& a, int msgs_per_wave, hipStream_t stream) {
  if (a.count <= 0) return hipSuccess;
  switch (msgs_per_wave) {
#define CASE(M)                                                                          \
  case M:                                                                                \
    hipLaunchKernelGGL(sha256_kernel<M>, dim3((a.count + M - 1) / M), dim3(64), 0, stream, a); \
    break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16) CASE(32) CASE(64)
#undef CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace callfs
