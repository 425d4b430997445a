// valu_rate2.hip -- issue cost of VALU instructions on gfx950 as a function of
// the independent work in flight: CH independent dependency chains per lane
// (CH = 1 .. 16) and W waves per SIMD (the launch: W 256-thread workgroups per
// CU, one wave per SIMD each).  With one chain and one wave the time per
// instruction is the instruction's latency; once the chains x waves in flight
// cover that latency it is the SIMD's issue cost, flat in CH and W.  That is
// the number the injection roofline prices its opcode mix at
// (tools/exp/run_valu_rate2.py -> profiles/r06/valu_rate2.json).
//
// MIX: chains alternate between OP_A (even) and OP_B (odd).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define V2(OP) asm volatile(OP " %0, %0, %1" : "+v"(a[k]) : "v"(b))
#define V3(OP) asm volatile(OP " %0, %0, %1, %1" : "+v"(a[k]) : "v"(b))
#define VB3(OP) asm volatile(OP " %0, %0, %1, %1 bitop3:0x96" : "+v"(a[k]) : "v"(b))

template <int OPC>
__device__ __forceinline__ void one(uint32_t (&a)[16], int k, uint32_t b) {
  if constexpr (OPC == 0) V2("v_add_u32");
  if constexpr (OPC == 1) V2("v_xor_b32");
  if constexpr (OPC == 2) V2("v_mul_lo_u32");
  if constexpr (OPC == 3) V2("v_mul_hi_u32");
  if constexpr (OPC == 4) V2("v_lshlrev_b32");
  if constexpr (OPC == 5) V3("v_add3_u32");
  if constexpr (OPC == 6) VB3("v_bitop3_b32");
  if constexpr (OPC == 7) V2("v_add_f32");
  if constexpr (OPC == 8) V2("v_and_b32");
  if constexpr (OPC == 9) V2("v_lshrrev_b32");
}

template <int OPA, int OPB, int CH>
__global__ __launch_bounds__(256) void valu2_kernel(uint32_t *out, int iters, uint32_t seed) {
  uint32_t a[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) a[k] = seed ^ (threadIdx.x + 977u * k);
  const uint32_t b = (seed * 3 + 1) | 1u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      if (k % 2 == 0)
        one<OPA>(a, k, b);
      else
        one<OPB>(a, k, b);
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) x ^= a[k];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

// ops: (opa, opb) pairs by index; chains 1, 2, 4, 8, 16
struct Pair {
  int a, b;
};
static const Pair kPairs[] = {{0, 0}, {1, 1}, {2, 2}, {3, 3}, {4, 4}, {5, 5}, {6, 6}, {7, 7}, {8, 8}, {9, 9},
                              {0, 4}, {0, 3}, {4, 3}, {6, 3}};

template <int A, int B>
static int launch_pair(int chains, uint32_t *out, int blocks, int iters, hipStream_t s) {
  switch (chains) {
#define C(N) case N: hipLaunchKernelGGL((valu2_kernel<A, B, N>), dim3(blocks), dim3(256), 0, s, out, iters, 7u); break;
    C(1) C(2) C(4) C(8) C(16)
#undef C
    default: return -1;
  }
  return 0;
}

extern "C" __attribute__((visibility("default"))) int valu2_pairs(void) {
  return (int)(sizeof(kPairs) / sizeof(kPairs[0]));
}

extern "C" __attribute__((visibility("default"))) int valu2_pair(int p, int *a, int *b) {
  *a = kPairs[p].a;
  *b = kPairs[p].b;
  return 0;
}

extern "C" __attribute__((visibility("default"))) int valu2_rate(int p, int chains, uint32_t *out, int blocks, int iters,
                                                                  void *stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = -1;
  switch (p) {
#define P(I, A, B) case I: rc = launch_pair<A, B>(chains, out, blocks, iters, s); break;
    P(0, 0, 0) P(1, 1, 1) P(2, 2, 2) P(3, 3, 3) P(4, 4, 4) P(5, 5, 5) P(6, 6, 6) P(7, 7, 7) P(8, 8, 8) P(9, 9, 9)
    P(10, 0, 4) P(11, 0, 3) P(12, 4, 3) P(13, 6, 3)
#undef P
    default: return -1;
  }
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
