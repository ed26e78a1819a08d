// Write-stream pattern probe (development tool, not product): what HBM serves best for the
// parity writes of long shards. Every block (512 threads, one 16-B store per lane per row)
// writes an 8 KiB tile of each of R rows; rows sit `pitch` bytes apart, stripes of R rows
// back to back (the planar parity region). Tile order: block b -> (stripe, tile) as
// consecutive (a stripe's tiles in order), G-interleaved (the same tile of G stripes on
// neighbouring blocks) or Q-segmented. Also a pure linear write of the same byte count.
// Prints GB/s per variant, best of `reps` launches, after a warm-up.
//
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/write_pattern.hip -o tools/write_pattern
// run:   tools/write_pattern [reps] [pitch]   (pitch: rows of 1 MiB shards at 1, 2, 6.4
//         and 8 MiB pitch, then 6.4 MiB shards; does the written span's contiguity matter?)
//        tools/write_pattern [reps] burst   (each block writes U = 1, 2, 4 or 8 consecutive 8 KiB
//         pieces of every row: each row front advances 8-64 KiB per block; verdict r05 item 7)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Args {
  uint8_t* base;
  uint64_t pitch;   // bytes between rows
  uint32_t R;       // rows per stripe
  uint32_t tps;     // tiles per row
  uint32_t batch;   // stripes
  uint32_t order;   // 0 consecutive, 1 G-interleave, 2 Q-segments, 3 linear
  uint32_t g;       // G or Q
  uint32_t read;    // 1: read the same bytes instead of writing them
  uint32_t rowwave; // 1: a wave's R stores go to consecutive 1 KiB pieces of one row (the
                    // block's 8R pieces dealt wave-major) instead of one piece of each row;
                    // 2: one piece of each row, each store waited for before the next
  uint32_t split;   // 1: each block stores ONE of the R rows of its tile; the R blocks of a
                    // tile are neighbours in launch order (the same rows in flight chip-wide
                    // as R-row blocks, one row per block)
  uint32_t burst;   // U >= 1: a block's tile is U * blockDim * 16 bytes of every row, each lane
                    // storing U vectors per row (wave w's stores cover 1 KiB pieces w, w + nw, ...)
  uint32_t* sink;
};

__global__ __launch_bounds__(1024) void pattern(Args a) {
  const uint32_t t = a.split ? blockIdx.x / a.R : blockIdx.x;
  const uint32_t only = a.split ? blockIdx.x % a.R : 0;
  uint32_t stripe, tile;
  if (a.order == 1) {
    const uint32_t per = a.g * a.tps, grp = t / per, r = t - grp * per;
    const uint32_t gsz = min(a.g, a.batch - grp * a.g);
    tile = r / gsz;
    stripe = grp * a.g + (r - tile * gsz);
  } else if (a.order == 2) {
    stripe = t / a.tps;
    const uint32_t r = t - stripe * a.tps, seg = a.tps / a.g;
    tile = r < seg * a.g ? (r % a.g) * seg + r / a.g : r;
  } else {
    stripe = t / a.tps;
    tile = t - stripe * a.tps;
  }
  const uint32_t x = t * 0x9E3779B1u + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const uint32_t U = a.burst ? a.burst : 1;
  const uint64_t tb = blockDim.x * 16ull * U;  // tile bytes per row
  for (uint32_t i = 0; i < a.R * U; ++i) {
    if (a.split && i != only) continue;
    if (U > 1) {  // burst: row i / U, the u-th run of nw pieces of the row's tile
      const uint32_t r = i / U, u = i % U;
      uint8_t* row = a.base + (static_cast<uint64_t>(stripe) * a.R + r) * a.pitch +
                     static_cast<uint64_t>(tile) * tb;
      u32x4* p = reinterpret_cast<u32x4*>(row + (u * nw + w) * 1024ull) + lane;
      const u32x4 v = {x, x + r, x ^ r, u};
      __builtin_nontemporal_store(v, p);
      continue;
    }
    // piece f of the block's nw*R 1 KiB pieces: row f / nw, piece f % nw of the row's tile
    const uint32_t f = a.rowwave ? w * a.R + i : i * nw + w;
    const uint32_t r = f / nw, piece = f % nw;
    uint8_t* row = a.order == 3
                       ? a.base + (static_cast<uint64_t>(t) * a.R + r) * tb
                       : a.base + (static_cast<uint64_t>(stripe) * a.R + r) * a.pitch +
                             static_cast<uint64_t>(tile) * tb;
    u32x4* p = reinterpret_cast<u32x4*>(row + piece * 1024) + lane;
    if (a.read) {
      acc ^= __builtin_nontemporal_load(p);
    } else {
      const u32x4 v = {x, x + r, x ^ r, r};
      __builtin_nontemporal_store(v, p);
      if (a.rowwave == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // one store in flight
    }
  }
  if (a.read && acc.x == 0x12345678u && acc.y == 0x9abcdef0u) a.sink[0] = acc.z;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 10;
  const uint64_t total = 6ull << 30;  // bytes written per launch (approximately)
  uint8_t* buf;
  CK(hipMalloc(&buf, total + (64ull << 20)));
  uint32_t* sink;
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    const char* name;
    uint64_t S;
    uint32_t R, order, g, read, rowwave, bs;
    uint64_t pitch;  // 0: S
    uint32_t split;
    uint32_t burst;
  };
  std::vector<V> vs;
  const uint64_t shapes[] = {1ull << 20, 2ull << 20, 6710912, 8ull << 20, 64ull << 20};
  if (argc > 2 && argv[2][0] == 'b') {
    // each row front advancing U * 8 KiB per block (512 threads), R = 4 and 8 rows
    for (int rep = 0; rep < 2; ++rep)
      for (uint64_t S : {1ull << 20, 6710912ull})
        for (uint32_t R : {4u, 8u})
          for (uint32_t U : {1u, 2u, 4u, 8u}) {
            vs.push_back({"consecutive", S, R, 0, 0, 0, 0, 512, 0, 0, U});
            vs.push_back({"G8", S, R, 1, 8, 0, 0, 512, 0, 0, U});
            vs.push_back({"Q8", S, R, 2, 8, 0, 0, 512, 0, 0, U});
          }
  } else if (argc > 2 && argv[2][0] == 's') {
    // one row per block against R rows per block, same rows in flight (split probe)
    for (int rep = 0; rep < 2; ++rep)
      for (uint64_t S : {1ull << 20, 6710912ull})
        for (uint32_t R : {1u, 4u, 8u})
          for (uint32_t sp : {0u, 1u}) {
            if (R == 1 && sp) continue;
            vs.push_back({"consecutive", S, R, 0, 0, 0, 0, 512, 0, sp});
            vs.push_back({"G8", S, R, 1, 8, 0, 0, 512, 0, sp});
          }
  } else if (argc > 2) {
    const uint64_t pitches[] = {1ull << 20, (2ull << 20) + 256, 6710912, 8ull << 20};
    for (int rep = 0; rep < 2; ++rep)
      for (uint64_t P : pitches)
        for (uint32_t R : {1u, 4u}) {
          vs.push_back({"consecutive", 1ull << 20, R, 0, 0, 0, 0, 512, P});
          vs.push_back({"G8", 1ull << 20, R, 1, 8, 0, 0, 512, P});
          if (P == 6710912) {
            vs.push_back({"consecutive", P, R, 0, 0, 0, 0, 512, P});
            vs.push_back({"G8", P, R, 1, 8, 0, 0, 512, P});
          }
        }
  } else {
    for (uint32_t bs : {128u, 256u, 512u, 1024u})
      for (uint64_t S : shapes)
        for (uint32_t R : {1u, 4u, 8u}) {
          vs.push_back({"consecutive", S, R, 0, 0, 0, 0, bs, 0});
          vs.push_back({"G8", S, R, 1, 8, 0, 0, bs, 0});
          vs.push_back({"Q8", S, R, 2, 8, 0, 0, bs, 0});
        }
  }
  std::printf("variant,shard_bytes,pitch,rows,block,mode,split,burst,GBps\n");
  for (const V& v : vs) {
    Args a{};
    a.base = buf;
    a.pitch = v.pitch ? v.pitch : v.S;
    a.R = v.R;
    const uint64_t tb = v.bs * 16ull * (v.burst ? v.burst : 1);
    a.tps = static_cast<uint32_t>(v.S / tb);
    a.batch = static_cast<uint32_t>(total / (a.pitch * v.R));
    a.order = v.order;
    a.g = v.g;
    a.read = v.read;
    a.rowwave = v.rowwave;
    a.sink = sink;
    a.split = v.split;
    a.burst = v.burst;
    uint32_t grid = a.tps * a.batch * (v.split ? v.R : 1);
    if (v.order == 3) {
      a.tps = 1;
      grid = static_cast<uint32_t>(total / (tb * v.R));
      a.batch = grid;
    }
    const double bytes = static_cast<double>(grid) * (v.split ? 1 : v.R) * tb;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(pattern, dim3(grid), dim3(v.bs), 0, 0, a);
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(pattern, dim3(grid), dim3(v.bs), 0, 0, a);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("%s,%llu,%llu,%u,%u,%s,%u,%u,%.0f\n", v.name, static_cast<unsigned long long>(v.S),
                static_cast<unsigned long long>(a.pitch), v.R, v.bs, v.read ? "read" : "write",
                v.split, v.burst ? v.burst : 1, bytes / (best * 1e-3) / 1e9);
    std::fflush(stdout);
  }
  CK(hipFree(buf));
  return 0;
}
