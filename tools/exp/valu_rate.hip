// valu_rate.hip -- issue cost of single VALU instructions on gfx950 with the
// SIMDs full (8 waves each): every lane runs 8 independent chains of one
// instruction, K iterations; cycles per wave-instruction per SIMD =
// duration * clock * SIMDs / (waves * 8 * K).  Sets the integer VALU peak the
// injection roofline is priced against (tools/exp/run_valu_rate.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CHAINS8(OP)                                                                                 \
  asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t" OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t" \
               OP " %4, %4, %8\n\t" OP " %5, %5, %8\n\t" OP " %6, %6, %8\n\t" OP " %7, %7, %8"     \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)    \
               : "v"(b))
#define CHAINS8_B3(OP)                                                                                         \
  asm volatile(OP " %0, %0, %8, %8 bitop3:0x96\n\t" OP " %1, %1, %8, %8 bitop3:0x96\n\t" OP " %2, %2, %8, %8 bitop3:0x96\n\t" OP " %3, %3, %8, %8 bitop3:0x96\n\t" \
               OP " %4, %4, %8, %8 bitop3:0x96\n\t" OP " %5, %5, %8, %8 bitop3:0x96\n\t" OP " %6, %6, %8, %8 bitop3:0x96\n\t" OP " %7, %7, %8, %8 bitop3:0x96"     \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                \
               : "v"(b))
#define CHAINS8_3(OP)                                                                                         \
  asm volatile(OP " %0, %0, %8, %8\n\t" OP " %1, %1, %8, %8\n\t" OP " %2, %2, %8, %8\n\t" OP " %3, %3, %8, %8\n\t" \
               OP " %4, %4, %8, %8\n\t" OP " %5, %5, %8, %8\n\t" OP " %6, %6, %8, %8\n\t" OP " %7, %7, %8, %8"     \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                \
               : "v"(b))

template <int OPC>
__global__ __launch_bounds__(256) void valu_kernel(uint32_t *out, int iters, uint32_t seed) {
  uint32_t a0 = seed ^ threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7, b = seed * 3 + 1;
  for (int i = 0; i < iters; ++i) {
    if constexpr (OPC == 0) CHAINS8("v_add_u32");
    if constexpr (OPC == 1) CHAINS8("v_xor_b32");
    if constexpr (OPC == 2) CHAINS8("v_mul_lo_u32");
    if constexpr (OPC == 3) CHAINS8("v_mul_hi_u32");
    if constexpr (OPC == 4) CHAINS8("v_mul_u32_u24");
    if constexpr (OPC == 5) CHAINS8("v_add_f32");
    if constexpr (OPC == 6) CHAINS8_3("v_fma_f32");
    if constexpr (OPC == 7) CHAINS8_B3("v_bitop3_b32");
    if constexpr (OPC == 8) CHAINS8_3("v_add3_u32");
    if constexpr (OPC == 9) CHAINS8("v_lshlrev_b32");
    if constexpr (OPC == 10) CHAINS8("v_mul_hi_u32_u24");
    if constexpr (OPC == 11) CHAINS8_3("v_mad_u32_u24");
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

extern "C" __attribute__((visibility("default"))) int valu_rate(int op, uint32_t *out, int blocks, int iters,
                                                                 void *stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (op) {
#define C(N) case N: hipLaunchKernelGGL(valu_kernel<N>, dim3(blocks), dim3(256), 0, s, out, iters, 7u); break;
    C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11)
#undef C
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
