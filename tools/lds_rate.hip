// LDS nibble-lookup rate on MI355X (development tool): the production kernel's lookup
// pattern with no HBM traffic, to price the LDS roofline of the wide / many-input launch
// groups. Each lane holds 16 data bytes in registers and repeatedly looks
// up both nibbles of every byte in 16-entry tables of W = 4, 8 or 16 bytes (ds_read_b32 /
// b64 / b128; addresses as in rs_apply_lds: byte j of (x << s) & mask dropped into the low
// byte of a 256-B-aligned table base), XORing the entries, 512-thread blocks, 8 blocks per
// CU worth of grid. Reports lookups per second, LDS bytes per second and bytes per CU per
// clock at the given clock.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lds_rate.hip -o tools/lds_rate
// run:   tools/lds_rate [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::printf("error %s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int W>
__global__ __launch_bounds__(512) void lds_rate(const uint32_t* seed, uint32_t* out, int iters) {
  __shared__ __attribute__((aligned(256))) uint8_t tab[32 * 16 * 16];  // 16 shards x 2 tables
  for (int j = threadIdx.x; j < 32 * 16 * 16 / 4; j += 512)
    reinterpret_cast<uint32_t*>(tab)[j] = j * 2654435761u;
  __syncthreads();
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)tab));
  uint32_t x[4];
  for (int w = 0; w < 4; ++w) x[w] = seed[(blockIdx.x * 512 + threadIdx.x) * 4 + w];
  u32x4 acc = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    const uint32_t base = lds0 + static_cast<uint32_t>(it & 15) * 32u * W;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      uint32_t xl, xh, bh;
      if constexpr (W == 16) {
        xl = (x[w] << 4) & 0xf0f0f0f0u;
        xh = x[w] & 0xf0f0f0f0u;
        bh = base + 256u;
      } else if constexpr (W == 8) {
        xl = (x[w] << 3) & 0x78787878u;
        xh = ((x[w] >> 1) & 0x78787878u) | 0x80808080u;
        bh = base;
      } else {
        xl = (x[w] << 2) & 0x3c3c3c3cu;
        xh = ((x[w] >> 2) & 0x3c3c3c3cu) | 0x40404040u;
        bh = base;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t sel = 0x07060500u | static_cast<uint32_t>(j);
        const uint32_t al = __builtin_amdgcn_perm(base, xl, sel), ah = __builtin_amdgcn_perm(bh, xh, sel);
        if constexpr (W == 16) {
          const u32x4 a = *(const __attribute__((address_space(3))) u32x4*)(static_cast<uintptr_t>(al));
          const u32x4 b = *(const __attribute__((address_space(3))) u32x4*)(static_cast<uintptr_t>(ah));
          acc ^= a ^ b;
        } else if constexpr (W == 8) {
          const u32x2 a = *(const __attribute__((address_space(3))) u32x2*)(static_cast<uintptr_t>(al));
          const u32x2 b = *(const __attribute__((address_space(3))) u32x2*)(static_cast<uintptr_t>(ah));
          acc.x ^= a.x ^ b.x;
          acc.y ^= a.y ^ b.y;
        } else {
          const uint32_t a = *(const __attribute__((address_space(3))) uint32_t*)(static_cast<uintptr_t>(al));
          const uint32_t b = *(const __attribute__((address_space(3))) uint32_t*)(static_cast<uintptr_t>(ah));
          acc.x ^= a ^ b;
        }
      }
      x[w] = x[w] * 1664525u + 1013904223u;  // next data word (random addresses, no chain)
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

// Wider-index variant (round 3 probe): 2^B-entry tables of W bytes (B = 5 with W = 8, B = 6
// with W = 4: 256 B per table, so every entry still owns its banks), each lookup resolving
// B input bits. The index of each lookup is assembled from two data words the way a
// piece spanning two shards would be (two shifts and one three-input op per 4 lookups).
template <int W, int B>
__global__ __launch_bounds__(512) void lds_rate_wide(const uint32_t* seed, uint32_t* out, int iters) {
  __shared__ __attribute__((aligned(256))) uint8_t tab[32 * 16 * 16];
  for (int j = threadIdx.x; j < 32 * 16 * 16 / 4; j += 512)
    reinterpret_cast<uint32_t*>(tab)[j] = j * 2654435761u;
  __syncthreads();
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)tab));
  uint32_t x[4];
  for (int w = 0; w < 4; ++w) x[w] = seed[(blockIdx.x * 512 + threadIdx.x) * 4 + w];
  u32x2 acc = {0, 0};
  constexpr uint32_t kMask = (((1u << B) - 1u) * W) * 0x01010101u;  // idx*W in each byte
  static_assert(((1 << B) - 1) * W < 256, "entry offset must fit a byte");
  for (int it = 0; it < iters; ++it) {
    const uint32_t base = lds0 + static_cast<uint32_t>(it & 15) * 512u;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // piece word: low bits from x[w], high bits from x[w+1] (a piece across two shards)
        const uint32_t lo = x[w] >> (h ? 3 : 1), hi = x[(w + 1) & 3] << (h ? 5 : 2);
        const uint32_t p = (lo & kMask) ^ (hi & kMask & 0xE0E0E0E0u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t sel = 0x07060500u | static_cast<uint32_t>(j);
          const uint32_t a = __builtin_amdgcn_perm(base + 256u * h, p, sel);
          if constexpr (W == 8) {
            acc ^= *(const __attribute__((address_space(3))) u32x2*)(static_cast<uintptr_t>(a));
          } else {
            acc.x ^= *(const __attribute__((address_space(3))) uint32_t*)(static_cast<uintptr_t>(a));
          }
        }
      }
      x[w] = x[w] * 1664525u + 1013904223u;
    }
  }
  if ((acc.x ^ acc.y) == 0x12345678u) out[0] = 1;
}

template <int W, int B>
void run_wide(const uint32_t* seed, uint32_t* out, int blocks, int iters, size_t dyn) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((lds_rate_wide<W, B>), dim3(blocks), dim3(512), dyn, 0, seed, out, iters);
  CK(hipGetLastError());
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int rep = 0; rep < reps; ++rep) hipLaunchKernelGGL((lds_rate_wide<W, B>), dim3(blocks), dim3(512), dyn, 0, seed, out, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double lookups = static_cast<double>(blocks) * 512 * iters * 32 * reps;
  const double s = ms * 1e-3;
  std::printf("{\"W\": %d, \"index_bits\": %d, \"waves_per_simd\": %d, \"lookups_per_s\": %.4g, \"lds_TBps\": %.2f, "
              "\"data_bytes_per_s_TB\": %.2f}\n",
              W, B, dyn ? static_cast<int>(8 * ((160u << 10) / (dyn + 8192)) / 4) : 8, lookups / s, lookups * W / s / 1e12,
              lookups * B / 8.0 / s / 1e12);
}

template <int W>
void run(const uint32_t* seed, uint32_t* out, int blocks, int iters, double ghz, size_t dyn) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(lds_rate<W>, dim3(blocks), dim3(512), dyn, 0, seed, out, iters);
  CK(hipGetLastError());
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int rep = 0; rep < reps; ++rep) hipLaunchKernelGGL(lds_rate<W>, dim3(blocks), dim3(512), dyn, 0, seed, out, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double lookups = static_cast<double>(blocks) * 512 * iters * 32 * reps;  // 16 bytes x 2
  const double s = ms * 1e-3;
  const double bytes = lookups * W;
  std::printf("{\"W\": %d, \"waves_per_simd\": %d, \"lookups_per_s\": %.4g, \"lds_TBps\": %.2f, \"bytes_per_cu_clk_at_%.1fGHz\": %.1f, "
              "\"data_bytes_per_s_TB\": %.2f}\n",
              W, dyn ? static_cast<int>(8 * ((160u << 10) / (dyn + 8192)) / 4) : 8, lookups / s, bytes / s / 1e12, ghz, bytes / s / 256 / (ghz * 1e9), lookups / 2 / s / 1e12);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  const double ghz = argc > 2 ? std::atof(argv[2]) : 2.4;
  const int blocks = 256 * 8;
  uint32_t *seed, *out;
  CK(hipMalloc(&seed, sizeof(uint32_t) * blocks * 512 * 4));
  CK(hipMalloc(&out, 64));
  uint32_t* h = static_cast<uint32_t*>(std::malloc(sizeof(uint32_t) * blocks * 512 * 4));
  for (size_t i = 0; i < static_cast<size_t>(blocks) * 512 * 4; ++i) h[i] = static_cast<uint32_t>(i * 2246822519u + 3266489917u);
  CK(hipMemcpy(seed, h, sizeof(uint32_t) * blocks * 512 * 4, hipMemcpyHostToDevice));
  // dynamic LDS padding limits blocks per CU: 0 -> 4 blocks (8 waves per SIMD), 64 KiB ->
  // 2 blocks (4 waves per SIMD), 40 KiB -> 3 blocks (6 waves per SIMD)
  for (size_t dyn : {static_cast<size_t>(0), static_cast<size_t>(40u << 10), static_cast<size_t>(64u << 10)}) {
    if (dyn > (64u << 10)) continue;
    if (dyn) {
      CK(hipFuncSetAttribute(reinterpret_cast<const void*>(lds_rate<4>), hipFuncAttributeMaxDynamicSharedMemorySize, (160 << 10) - 8192));
      CK(hipFuncSetAttribute(reinterpret_cast<const void*>(lds_rate<8>), hipFuncAttributeMaxDynamicSharedMemorySize, (160 << 10) - 8192));
      CK(hipFuncSetAttribute(reinterpret_cast<const void*>(lds_rate<16>), hipFuncAttributeMaxDynamicSharedMemorySize, (160 << 10) - 8192));
    }
    run<4>(seed, out, blocks, iters, ghz, dyn);
    run<8>(seed, out, blocks, iters, ghz, dyn);
    run<16>(seed, out, blocks, iters, ghz, dyn);
    if (dyn) {
      CK(hipFuncSetAttribute(reinterpret_cast<const void*>(lds_rate_wide<8, 5>), hipFuncAttributeMaxDynamicSharedMemorySize, (160 << 10) - 8192));
      CK(hipFuncSetAttribute(reinterpret_cast<const void*>(lds_rate_wide<4, 6>), hipFuncAttributeMaxDynamicSharedMemorySize, (160 << 10) - 8192));
    }
    run_wide<8, 5>(seed, out, blocks, iters, dyn);
    run_wide<4, 6>(seed, out, blocks, iters, dyn);
  }
  return 0;
}
