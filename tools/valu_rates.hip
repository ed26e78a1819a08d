// VALU issue rate per instruction kind on gfx950 (development tool, not product).
// Every lane runs 8 independent dependency chains of one instruction kind; 8 waves per
// SIMD on every CU. Each kind is timed in 3 rotated rounds and the fastest round counts;
// prints wave-instructions per SIMD per clock at the device's peak clock (2 cycles per wave64
// instruction on a SIMD-32 = 0.5). The RS kernels and SHA-256 are VALU-issue-heavy
// (DESIGN.md §5, §5.7): which encodings issue at the full rate decides how they are written.
// build: hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

// Inline asm so the compiler can neither fold repeated operations nor pick another
// instruction. b, c: VGPRs; s: an SGPR.
template <int OP>
__device__ __forceinline__ void op(uint32_t& a, uint32_t b, uint32_t c, uint32_t s) {
  if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
  if constexpr (OP == 1) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == 3)
    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == 4) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == 5) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a));
  // byte select + OR (the LDS kernel's table address): SDWA with VGPR / SGPR base
  if constexpr (OP == 6)
    asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
                 : "+v"(a) : "v"(b));
  if constexpr (OP == 7)
    asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
                 : "+v"(a) : "s"(s));
  if constexpr (OP == 8) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == 9) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
  if constexpr (OP == 10) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a));
  if constexpr (OP == 11) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a));
  // the bit-sliced kernels' transposes and networks (bitslice_gen.hpp tr8, x2, x3)
  if constexpr (OP == 12) asm volatile("v_lshlrev_b32 %0, 4, %0" : "+v"(a));
  if constexpr (OP == 13) asm volatile("v_lshrrev_b32 %0, 4, %0" : "+v"(a));
  if constexpr (OP == 14) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a) : "v"(c));
  if constexpr (OP == 15)
    asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xca" : "+v"(a) : "s"(s), "v"(b));
  if constexpr (OP == 16)
    asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xca" : "+v"(a) : "v"(c), "v"(b));
  if constexpr (OP == 17) asm volatile("v_bitop3_b32 %0, %0, %1, 0 bitop3:0x3c" : "+v"(a) : "v"(b));
  if constexpr (OP == 18) asm volatile("v_add_u32 %0, %0, %0" : "+v"(a));
  if constexpr (OP == 19) asm volatile("v_pk_lshlrev_b16 %0, 4, %0" : "+v"(a));
  if constexpr (OP == 20) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a) : "s"(s));
  if constexpr (OP == 21) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a) : "s"(s));
  if constexpr (OP == 22) asm volatile("v_lshlrev_b32_e64 %0, 4, %0" : "+v"(a));
  if constexpr (OP == 24) asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a) : "v"(b));
  if constexpr (OP == 25) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(a));
  if constexpr (OP == 26) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a) : "v"(b));
  if constexpr (OP == 27) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a));
}

template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(uint32_t* out, int iters, uint32_t s) {
  if constexpr (OP == 23) {  // 64-bit shifts: one instruction shifts a register pair
    uint64_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (uint64_t(threadIdx.x) << 32) * 7 + i + s;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_lshlrev_b64 %0, 4, %0" : "+v"(x[i]));
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= x[i];
    if (acc == 0x12345678u) out[blockIdx.x] = uint32_t(acc);
  } else {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 7 + i + s;
    const uint32_t b = s ^ 0x01020304u, c = (s & 7) | 0x03020100u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) op<OP>(x[i], b, c, s);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= x[i];
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
  }
}

template <int... OPS>
struct Table {
  static constexpr int n = sizeof...(OPS);
  static hipError_t launch(int op, int blocks, uint32_t* out, int iters) {
    const void* fns[] = {reinterpret_cast<const void*>(&valu_kernel<OPS>)...};
    uint32_t s = 0x0f0f0f0fu;
    void* args[] = {&out, &iters, &s};
    return hipLaunchKernel(fns[op], dim3(blocks), dim3(256), args, 0, 0);
  }
};
using Ops = Table<0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22,
                  23, 24, 25, 26, 27>;

int main() {
  uint32_t* out;
  CK(hipMalloc(&out, 1 << 20));
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
  const int iters = 1000;
  const char* names[] = {"v_add_u32", "v_perm_b32", "v_alignbit_b32 (vgpr shift)",
                         "v_bitop3_b32 0x96 (3 vgpr)", "v_add3_u32", "v_alignbit_b32 (rotate imm)",
                         "v_or_b32_sdwa (vgpr)", "v_or_b32_sdwa (sgpr)", "v_and_or_b32", "v_xor_b32",
                         "v_lshrrev_b32 8", "v_bfe_u32", "v_lshlrev_b32 4", "v_lshrrev_b32 4",
                         "v_lshlrev_b32 (vgpr amount)", "v_bitop3_b32 0xca (sgpr mask)",
                         "v_bitop3_b32 0xca (vgpr mask)", "v_bitop3_b32 0x3c (inline 0)",
                         "v_add_u32 x, x", "v_pk_lshlrev_b16 4", "v_xor_b32 (sgpr)",
                         "v_and_b32 (sgpr)", "v_lshlrev_b32_e64 4", "v_lshlrev_b64 4",
                         "v_lshl_or_b32", "v_mov_b32", "v_and_b32 (vgpr)", "v_lshlrev_b32 1"};
  static_assert(sizeof(names) / sizeof(names[0]) == Ops::n, "one name per kind");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best[Ops::n];
  for (int i = 0; i < Ops::n; ++i) best[i] = 1e30f;
  for (int round = 0; round < 3; ++round) {
    for (int opi = 0; opi < Ops::n; ++opi) {
      CK(Ops::launch(opi, blocks, out, iters));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      CK(Ops::launch(opi, blocks, out, iters));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best[opi]) best[opi] = ms;
    }
  }
  for (int opi = 0; opi < Ops::n; ++opi) {
    const double wave_instr = double(blocks) * 4 * iters * 16 * 8;  // 4 waves per block
    const double per_simd_per_clk = wave_instr / 1024.0 / (best[opi] * 1e-3 * clk_khz * 1e3);
    printf("%-32s %8.3f ms  %.3f wave-instr per SIMD per clock (at %d MHz)\n", names[opi],
           best[opi], per_simd_per_clk, clk_khz / 1000);
  }
  return 0;
}
