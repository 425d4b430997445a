// interp_exp.hip -- interpolation geometry A/B: rows per lane, XCD-aware block
// order (neighbouring row blocks on one XCD so the halo rows hit its L2), and
// non-temporal vs default-policy halo loads.  Full row blocks only.
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/kvecc_internal.h"

using namespace kvecc;

__device__ __forceinline__ u32x4 iv(u32x4 q, u32x4 l, u32x4 r, u32x4 e) {
  u32x4 o;
  o.x = interp_word(q.x, l.x, r.x, e.x);
  o.y = interp_word(q.y, l.y, r.y, e.y);
  o.z = interp_word(q.z, l.z, r.z, e.z);
  o.w = interp_word(q.w, l.w, r.w, e.w);
  return o;
}

template <int R, bool SWZ, bool HALO_NT>
__global__ __launch_bounds__(256) void k(const u32x4 *__restrict__ q, const u32x4 *__restrict__ err,
                                         u32x4 *__restrict__ out, int64_t outer, int64_t len,
                                         int64_t chunks) {
  const int64_t rblocks = len / R;
  const int64_t items = outer * rblocks * chunks;
  int64_t b = blockIdx.x;
  const int64_t G = gridDim.x;
  if (SWZ && G % 8 == 0) b = (b % 8) * (G / 8) + b / 8;
  for (int64_t it = b * 256 + threadIdx.x; it < items; it += G * 256) {
    const int64_t c = it % chunks;
    const int64_t t = it / chunks;
    const int64_t rb = t % rblocks;
    const int64_t o = t / rblocks;
    const int64_t l0 = rb * R;
    const int64_t base = o * len * chunks + c;
    u32x4 qr[R + 2], er[R];
    const u32x4 *hl = q + base + (l0 > 0 ? l0 - 1 : 0) * chunks;
    const u32x4 *hr = q + base + (l0 + R < len ? l0 + R : len - 1) * chunks;
    qr[0] = HALO_NT ? ld_stream(hl) : *hl;
#pragma unroll
    for (int j = 0; j < R; ++j) qr[j + 1] = ld_stream(q + base + (l0 + j) * chunks);
    qr[R + 1] = HALO_NT ? ld_stream(hr) : *hr;
#pragma unroll
    for (int j = 0; j < R; ++j) er[j] = ld_stream(err + base + (l0 + j) * chunks);
#pragma unroll
    for (int j = 0; j < R; ++j) st_stream(out + base + (l0 + j) * chunks, iv(qr[j + 1], qr[j], qr[j + 2], er[j]));
  }
}

template <int R, bool SWZ, bool HNT>
static void L(const void *q, const void *e, void *o, int64_t outer, int64_t len, int64_t chunks,
              int grid, hipStream_t s) {
  hipLaunchKernelGGL((k<R, SWZ, HNT>), dim3(grid), dim3(256), 0, s, (const u32x4 *)q,
                     (const u32x4 *)e, (u32x4 *)o, outer, len, chunks);
}

extern "C" int interp_exp(int v, const void *q, const void *e, void *o, int64_t outer, int64_t len,
                          int64_t chunks, int grid, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (v) {
    case 0: L<8, false, true>(q, e, o, outer, len, chunks, grid, s); break;
    case 1: L<8, true, true>(q, e, o, outer, len, chunks, grid, s); break;
    case 2: L<8, true, false>(q, e, o, outer, len, chunks, grid, s); break;
    case 3: L<16, false, true>(q, e, o, outer, len, chunks, grid, s); break;
    case 4: L<16, true, true>(q, e, o, outer, len, chunks, grid, s); break;
    case 5: L<16, true, false>(q, e, o, outer, len, chunks, grid, s); break;
    case 6: L<4, true, false>(q, e, o, outer, len, chunks, grid, s); break;
    case 7: L<8, false, false>(q, e, o, outer, len, chunks, grid, s); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
