// VALU issue rate per instruction kind on gfx950 (development tool, not product).
// Every lane runs 8 independent dependency chains of one instruction kind; 8 waves per
// SIMD on every CU. Prints wave-instructions per SIMD per clock at the clock read from
// the device (SHA-256 and the RS kernels are VALU-issue-heavy: DESIGN.md §5).
// build: hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

// Inline asm so the compiler can neither fold repeated operations nor pick another
// instruction.
template <int OP>
__device__ __forceinline__ void op(uint32_t& a, uint32_t b, uint32_t c) {
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
                 : "+v"(a) : "s"(b));
  if constexpr (OP == 8) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == 9) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
  if constexpr (OP == 10) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a));
  if constexpr (OP == 11) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a));
}

template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(uint32_t* out, int iters, uint32_t s) {
  uint32_t x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 7 + i + s;
  const uint32_t b = s ^ 0x01020304u, c = (s & 7) | 0x03020100u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) op<OP>(x[i], b, c);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc ^= x[i];
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  uint32_t* out;
  CK(hipMalloc(&out, 1 << 20));
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
  const int iters = 2000;
  const char* names[] = {"v_add_u32", "v_perm_b32", "v_alignbit_b32 (vgpr shift)", "v_bitop3_b32",
                         "v_add3_u32", "v_alignbit_b32 (rotate imm)", "v_or_b32_sdwa (vgpr)",
                         "v_or_b32_sdwa (sgpr)", "v_and_or_b32", "v_xor_b32", "v_lshrrev_b32",
                         "v_bfe_u32"};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int opi = 0; opi < 12; ++opi) {
    auto launch = [&]() {
      switch (opi) {
        case 0: hipLaunchKernelGGL(valu_kernel<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 1: hipLaunchKernelGGL(valu_kernel<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 2: hipLaunchKernelGGL(valu_kernel<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 3: hipLaunchKernelGGL(valu_kernel<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 4: hipLaunchKernelGGL(valu_kernel<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 5: hipLaunchKernelGGL(valu_kernel<5>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 6: hipLaunchKernelGGL(valu_kernel<6>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 7: hipLaunchKernelGGL(valu_kernel<7>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 8: hipLaunchKernelGGL(valu_kernel<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 9: hipLaunchKernelGGL(valu_kernel<9>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 10: hipLaunchKernelGGL(valu_kernel<10>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
        case 11: hipLaunchKernelGGL(valu_kernel<11>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u); break;
      }
    };
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double wave_instr = double(blocks) * 4 * iters * 16 * 8;  // 4 waves per block
    const double per_simd_per_clk = wave_instr / 1024.0 / (ms * 1e-3 * clk_khz * 1e3);
    printf("%-30s %8.3f ms  %.3f wave-instr per SIMD per clock (at %d MHz)\n", names[opi], ms,
           per_simd_per_clk, clk_khz / 1000);
  }
  return 0;
}
