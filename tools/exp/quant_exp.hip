// quant_exp.hip -- fp16 quantize + H(8,4) encode geometry A/B (D = 128 rows, 16 lanes per row,
// one 16-byte chunk per lane): rows in flight per lane (U), a prefetch of the next iteration's
// chunks (PF), packed-fp32 quotient math (PK).  Fast path only (every scale in recip range).
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/kvecc_internal.h"

using namespace kvecc;
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int U, bool PF, bool PK>
__global__ __launch_bounds__(256) void k(const __half *__restrict__ x, uint8_t *__restrict__ cw,
                                         float *__restrict__ scales, int64_t rows) {
  constexpr int LPR = 16, VEC = 8, D = 128, RPW = 4;
  const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane % LPR;
  const int64_t waves = (int64_t)gridDim.x * 4;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const int64_t step = waves * RPW;
  u32x4 cur[U], nxt[U];
  int64_t r0 = wave_id * RPW;
  auto load = [&](u32x4 *dst, int64_t base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = base + u * step + sub;
      if (r < rows) dst[u] = ld_stream(reinterpret_cast<const u32x4 *>(x + r * D + li * VEC));
    }
  };
  if (PF) load(cur, r0);
  for (; r0 < rows; r0 += U * step) {
    if (PF) {
      load(nxt, r0 + U * step);
    } else {
      load(cur, r0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = r0 + u * step + sub;
      const bool live = r < rows;
      __half hv[8];
      __builtin_memcpy(hv, &cur[u], 16);
      float f[8];
      float amax = 0.0f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        f[e] = live ? __half2float(hv[e]) : 0.0f;
        amax = fmaxf(amax, fabsf(f[e]));
      }
      amax = group_max_nonneg<LPR>(amax);
      const float scale = row_scale(amax, 1);
      if (!live) continue;
      if (li == 0) scales[r] = scale;
      const float inv = div_rn(1.0f, scale);
      uint32_t nq[8];
      if (PK) {
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 xv = {f[e], f[e + 1]};
          const f32x2 q0 = xv * f32x2{inv, inv};
          const f32x2 rr = __builtin_elementwise_fma(f32x2{-scale, -scale}, q0, xv);
          const f32x2 q = __builtin_elementwise_fma(rr, f32x2{inv, inv}, q0);
          nq[e] = nibble_of_quotient(q.x);
          nq[e + 1] = nibble_of_quotient(q.y);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) nq[e] = nibble_of_quotient(div_recip(f[e], scale, inv));
      }
      uint32_t w0 = nq[0] | nq[1] << 8 | nq[2] << 16 | nq[3] << 24;
      uint32_t w1 = nq[4] | nq[5] << 8 | nq[6] << 16 | nq[7] << 24;
      const uint64_t bits = (uint64_t)h84_encode4(w0) | (uint64_t)h84_encode4(w1) << 32;
      st_stream(reinterpret_cast<uint64_t *>(cw + r * D + li * VEC), bits);
    }
    if (PF) {
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
  }
}

template <int U, bool PF, bool PK>
static void L(const void *x, void *cw, void *sc, int64_t rows, int grid, hipStream_t s) {
  hipLaunchKernelGGL((k<U, PF, PK>), dim3(grid), dim3(256), 0, s, (const __half *)x, (uint8_t *)cw,
                     (float *)sc, rows);
}

extern "C" int quant_exp(int v, const void *x, void *cw, void *sc, int64_t rows, int grid, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (v) {
    case 0: L<2, false, false>(x, cw, sc, rows, grid, s); break;
    case 1: L<1, false, false>(x, cw, sc, rows, grid, s); break;
    case 2: L<4, false, false>(x, cw, sc, rows, grid, s); break;
    case 3: L<1, true, false>(x, cw, sc, rows, grid, s); break;
    case 4: L<2, true, false>(x, cw, sc, rows, grid, s); break;
    case 5: L<2, false, true>(x, cw, sc, rows, grid, s); break;
    case 6: L<2, true, true>(x, cw, sc, rows, grid, s); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
