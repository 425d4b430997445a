// philox_exp.hip -- Philox4x32-10 throughput: 32-bit mul_hi/mul_lo vs 64-bit mad forms.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int FORM>
__device__ __forceinline__ uint32_t w0(uint32_t ctr, uint32_t k0) {
  uint32_t k1 = (uint32_t)((int32_t)k0 >> 31);
  uint32_t c0 = ctr, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hb, lb, ha, la;
    if (FORM == 0) {
      hb = __umulhi(0xCD9E8D57u, c2); lb = 0xCD9E8D57u * c2;
      ha = __umulhi(0xD2511F53u, c0); la = 0xD2511F53u * c0;
    } else {
      uint64_t pb = (uint64_t)c2 * 0xCD9E8D57u, pa = (uint64_t)c0 * 0xD2511F53u;
      hb = (uint32_t)(pb >> 32); lb = (uint32_t)pb; ha = (uint32_t)(pa >> 32); la = (uint32_t)pa;
    }
    c0 = hb ^ c1 ^ k0; c2 = ha ^ c3 ^ k1; c1 = lb; c3 = la;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c0;
}

template <int FORM>
__global__ __launch_bounds__(256) void pk(uint32_t *out, uint32_t base, int iters) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x, m = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int b = 0; b < 24; ++b) m += w0<FORM>(i + it, base + i * 24 + b) < 21474836u;
  }
  out[i] = m;
}

extern "C" __attribute__((visibility("default"))) int philox_bench(int form, uint32_t *out, int blocks, int iters,
                                                                    void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (form == 0) hipLaunchKernelGGL(pk<0>, dim3(blocks), dim3(256), 0, s, out, 12345u, iters);
  else hipLaunchKernelGGL(pk<1>, dim3(blocks), dim3(256), 0, s, out, 12345u, iters);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
