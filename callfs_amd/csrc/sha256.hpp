// Batched SHA-256 (sha256.hip): erasure.ShardChecksum (codec.go:81-84) for many
// device-resident shards in one launch.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace callfs {

struct Sha256Args {
  const uint8_t* const* msgs;  // [count] device pointers
  const uint64_t* lens;        // [count] byte lengths
  uint32_t* digests;           // [count][8] words = 32 digest bytes each, in output order
  int count;
};

// msgs_per_wave in {1,2,4,8,16,32,64}: lanes of each 64-lane wave given a message.
hipError_t launch_sha256(const Sha256Args& a, int msgs_per_wave, hipStream_t stream);

// Full waves: the kernel is VALU-issue-bound (about 1,300 VALU per 64-B block), so a
// message per lane beats spreading few messages over more SIMDs. Measured on MI355X,
// 3,584 x 1 MiB messages: 64/wave 84 GB/s, 16/wave 61, 8/wave 34, 1/wave 17
// (tools/sha_bench.py, profiles/r01/sha_bench.json).
inline int default_msgs_per_wave(int /*count*/) { return 64; }

}  // namespace callfs
