// golay_exp.hip -- A/B variants of the Golay decode kernel + copy ceilings.
// Experimental only (tools/, never shipped): compiled to tools/exp/libexp.so and
// timed by tools/exp/run_exp.py against the production kernel.
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/kvecc_internal.h"

using namespace kvecc;

template <bool NT>
__device__ __forceinline__ u32x4 ld4(const u32x4 *p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st(T *p, T v) {
  if (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// ---- copy ceilings ---------------------------------------------------------------
template <bool NT, int U>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4 *__restrict__ s, u32x4 *__restrict__ d,
                                                   int64_t n) {
  const int64_t tile = 256 * U;
  for (int64_t b = (int64_t)blockIdx.x * tile; b < n; b += (int64_t)gridDim.x * tile) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 + threadIdx.x < n) v[u] = ld4<NT>(s + b + u * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 + threadIdx.x < n) st<NT>(d + b + u * 256 + threadIdx.x, v[u]);
  }
}

// ---- decode variants ---------------------------------------------------------------
__device__ __forceinline__ uint32_t spread_nibbles(uint32_t d) {
  return (d & 0xFu) | (d & 0xF0u) << 4 | (d & 0xF00u) << 8;
}

__device__ __forceinline__ uint32_t dec1(uint32_t w, const uint16_t *lds, uint32_t &c) {
  uint32_t lo = w & 0xFFFu;
  uint32_t syn = ((w >> 12) & 0xFFFu) ^ lds[lo];
  uint32_t e = lds[4096 + syn];
  c = e >> 12;
  return lo ^ (e & 0xFFFu);
}

__device__ __forceinline__ void load_tables(uint16_t *lds, const uint16_t *par, const uint16_t *cor) {
  const u32x4 *p = reinterpret_cast<const u32x4 *>(par);
  const u32x4 *c = reinterpret_cast<const u32x4 *>(cor);
  u32x4 *l = reinterpret_cast<u32x4 *>(lds);
  for (int i = threadIdx.x; i < 512; i += 256) {
    l[i] = p[i];
    l[512 + i] = c[i];
  }
  __syncthreads();
}

// LAYOUT 0: lane owns 4 groups of 4 consecutive codewords, each wave
// instruction contiguous (production layout).  PIPE: prefetch next tile.
template <bool NTL, bool NTS, bool PIPE>
__global__ __launch_bounds__(256) void dec_l0(const u32x4 *__restrict__ cw, uint32_t *__restrict__ trip,
                                              uint32_t *__restrict__ counts, int64_t ntiles,
                                              const uint16_t *__restrict__ par,
                                              const uint16_t *__restrict__ cor,
                                              uint64_t *__restrict__ stats) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[8192];
  load_tables(lds, par, cor);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t bits = 0, unc = 0;
  int64_t t = blockIdx.x;
  u32x4 nxt[4];
  auto issue = [&](int64_t tt, u32x4 *v) {
    const int64_t base = tt * 4096 + wave * 1024 + lane * 4;
#pragma unroll
    for (int g = 0; g < 4; ++g) v[g] = ld4<NTL>(cw + (base + g * 256) / 4);
  };
  if (PIPE && t < ntiles) issue(t, nxt);
  for (; t < ntiles; t += gridDim.x) {
    const int64_t base = t * 4096 + wave * 1024 + lane * 4;
    u32x4 v[4];
    if (PIPE) {
#pragma unroll
      for (int g = 0; g < 4; ++g) v[g] = nxt[g];
      if (t + gridDim.x < ntiles) issue(t + gridDim.x, nxt);
    } else {
      issue(t, v);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint32_t c0, c1, c2, c3;
      uint32_t e0 = spread_nibbles(dec1(v[g].x, lds, c0));
      uint32_t e1 = spread_nibbles(dec1(v[g].y, lds, c1));
      uint32_t e2 = spread_nibbles(dec1(v[g].z, lds, c2));
      uint32_t e3 = spread_nibbles(dec1(v[g].w, lds, c3));
      uint32_t *p = trip + (base + g * 256) * 3 / 4;
      st<NTS>(p, e0 | e1 << 24);
      st<NTS>(p + 1, e1 >> 8 | e2 << 16);
      st<NTS>(p + 2, e2 >> 16 | e3 << 8);
      uint32_t cc = c0 | c1 << 8 | c2 << 16 | c3 << 24;
      st<NTS>(counts + (base + g * 256) / 4, cc);
      bits += ((cc & 0x03030303u) * 0x01010101u) >> 24;
      unc += __builtin_popcount(cc & 0x04040404u);
    }
  }
  flush_stats2(stats, bits, unc);
}

// LAYOUT 1: lane owns 16 consecutive codewords; loads/stores are 16 B per
// lane at a 64/48/16-B lane stride (instructions not contiguous, but every
// store is a full dwordx4).
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void dec_l1(const u32x4 *__restrict__ cw, u32x4 *__restrict__ trip,
                                              u32x4 *__restrict__ counts, int64_t ntiles,
                                              const uint16_t *__restrict__ par,
                                              const uint16_t *__restrict__ cor,
                                              uint64_t *__restrict__ stats) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[8192];
  load_tables(lds, par, cor);
  uint32_t bits = 0, unc = 0;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t c0 = t * 4096 + threadIdx.x * 16;  // first codeword of this lane
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = ld4<NTL>(cw + c0 / 4 + k);
    uint32_t e[16], c[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[4 * k + 0] = spread_nibbles(dec1(v[k].x, lds, c[4 * k + 0]));
      e[4 * k + 1] = spread_nibbles(dec1(v[k].y, lds, c[4 * k + 1]));
      e[4 * k + 2] = spread_nibbles(dec1(v[k].z, lds, c[4 * k + 2]));
      e[4 * k + 3] = spread_nibbles(dec1(v[k].w, lds, c[4 * k + 3]));
    }
    uint32_t w[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) w[j] = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int bit = 24 * i, j = bit / 32, s = bit % 32;
      w[j] |= e[i] << s;
      if (s > 8) w[j + 1] |= e[i] >> (32 - s);
    }
    u32x4 *tp = trip + c0 * 3 / 16;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      u32x4 o;
      o.x = w[4 * k];
      o.y = w[4 * k + 1];
      o.z = w[4 * k + 2];
      o.w = w[4 * k + 3];
      st<NTS>(tp + k, o);
    }
    u32x4 cc;
    cc.x = c[0] | c[1] << 8 | c[2] << 16 | c[3] << 24;
    cc.y = c[4] | c[5] << 8 | c[6] << 16 | c[7] << 24;
    cc.z = c[8] | c[9] << 8 | c[10] << 16 | c[11] << 24;
    cc.w = c[12] | c[13] << 8 | c[14] << 16 | c[15] << 24;
    st<NTS>(counts + c0 / 16, cc);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      bits += c[i] & 3u;
      unc += c[i] >> 2;
    }
  }
  flush_stats2(stats, bits, unc);
}

extern "C" {

__attribute__((visibility("default"))) int exp_copy(const void *s, void *d, int64_t bytes, int variant,
                                                    int grid, void *stream) {
  int64_t n = bytes / 16;
  auto S = reinterpret_cast<const u32x4 *>(s);
  auto D = reinterpret_cast<u32x4 *>(d);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (variant) {
    case 0: hipLaunchKernelGGL((copy_kernel<false, 4>), dim3(grid), dim3(256), 0, st, S, D, n); break;
    case 1: hipLaunchKernelGGL((copy_kernel<true, 4>), dim3(grid), dim3(256), 0, st, S, D, n); break;
    case 2: hipLaunchKernelGGL((copy_kernel<false, 8>), dim3(grid), dim3(256), 0, st, S, D, n); break;
    case 3: hipLaunchKernelGGL((copy_kernel<true, 8>), dim3(grid), dim3(256), 0, st, S, D, n); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

__attribute__((visibility("default"))) int exp_golay_decode(int variant, const int32_t *cw, uint8_t *trip,
                                                            uint8_t *counts, int64_t m, uint64_t *stats,
                                                            const uint16_t *tables, int grid,
                                                            void *stream) {
  int64_t ntiles = m / 4096;  // caller passes a multiple of 4096
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint16_t *par = tables, *cor = tables + 4096;
  auto C = reinterpret_cast<const u32x4 *>(cw);
  auto T = reinterpret_cast<uint32_t *>(trip);
  auto N = reinterpret_cast<uint32_t *>(counts);
  auto T4 = reinterpret_cast<u32x4 *>(trip);
  auto N4 = reinterpret_cast<u32x4 *>(counts);
  switch (variant) {
    case 0: hipLaunchKernelGGL((dec_l0<true, true, false>), dim3(grid), dim3(256), 0, st, C, T, N, ntiles, par, cor, stats); break;
    case 1: hipLaunchKernelGGL((dec_l0<false, false, false>), dim3(grid), dim3(256), 0, st, C, T, N, ntiles, par, cor, stats); break;
    case 2: hipLaunchKernelGGL((dec_l0<true, false, false>), dim3(grid), dim3(256), 0, st, C, T, N, ntiles, par, cor, stats); break;
    case 3: hipLaunchKernelGGL((dec_l0<false, true, false>), dim3(grid), dim3(256), 0, st, C, T, N, ntiles, par, cor, stats); break;
    case 4: hipLaunchKernelGGL((dec_l0<true, true, true>), dim3(grid), dim3(256), 0, st, C, T, N, ntiles, par, cor, stats); break;
    case 5: hipLaunchKernelGGL((dec_l0<false, false, true>), dim3(grid), dim3(256), 0, st, C, T, N, ntiles, par, cor, stats); break;
    case 6: hipLaunchKernelGGL((dec_l1<true, true>), dim3(grid), dim3(256), 0, st, C, T4, N4, ntiles, par, cor, stats); break;
    case 7: hipLaunchKernelGGL((dec_l1<false, false>), dim3(grid), dim3(256), 0, st, C, T4, N4, ntiles, par, cor, stats); break;
    case 8: hipLaunchKernelGGL((dec_l1<true, false>), dim3(grid), dim3(256), 0, st, C, T4, N4, ntiles, par, cor, stats); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
}

// ---- ceiling study: block size / unroll / read-only / write-only ---------------
template <bool NT, int U, int BS>
__global__ __launch_bounds__(BS) void copy_bs(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, int64_t n) {
  const int64_t tile = (int64_t)BS * U;
  for (int64_t b = (int64_t)blockIdx.x * tile; b < n; b += (int64_t)gridDim.x * tile) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * BS + threadIdx.x < n) v[u] = ld4<NT>(s + b + u * BS + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * BS + threadIdx.x < n) st<NT>(d + b + u * BS + threadIdx.x, v[u]);
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void read_only(const u32x4 *__restrict__ s, int64_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (int64_t b = (int64_t)blockIdx.x * 1024; b < n; b += (int64_t)gridDim.x * 1024) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b + u * 256 + threadIdx.x < n) v[u] = ld4<NT>(s + b + u * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <bool NT>
__global__ __launch_bounds__(256) void write_only(u32x4 *__restrict__ d, int64_t n) {
  u32x4 v;
  v.x = v.y = v.z = v.w = threadIdx.x;
  for (int64_t b = (int64_t)blockIdx.x * 1024; b < n; b += (int64_t)gridDim.x * 1024) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b + u * 256 + threadIdx.x < n) st<NT>(d + b + u * 256 + threadIdx.x, v);
  }
}

// write-only through buffer stores with a cache-policy immediate (gfx950: sc0 = 1, nt = 2, sc1 = 16)
template <int AUX>
__global__ __launch_bounds__(256) void write_only_pol(u32x4 *__restrict__ d, int64_t n) {
  u32x4 v;
  v.x = v.y = v.z = v.w = threadIdx.x;
  for (int64_t b = (int64_t)blockIdx.x * 1024; b < n; b += (int64_t)gridDim.x * 1024) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<char *>(d + b), 0, (int)(min<int64_t>(1024, n - b) * 16), 0x00020000);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                             rs, (uint32_t)(u * 256 + threadIdx.x) * 16u, 0, AUX);
  }
}

extern "C" __attribute__((visibility("default"))) int exp_ceiling(const void *s, void *d, int64_t bytes, int variant,
                                                                  int grid, void *stream) {
  int64_t n = bytes / 16;
  auto S = reinterpret_cast<const u32x4 *>(s);
  auto D = reinterpret_cast<u32x4 *>(d);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (variant) {
    case 0: hipLaunchKernelGGL((copy_bs<true, 4, 256>), dim3(grid), dim3(256), 0, st, S, D, n); break;
    case 1: hipLaunchKernelGGL((copy_bs<true, 2, 256>), dim3(grid), dim3(256), 0, st, S, D, n); break;
    case 2: hipLaunchKernelGGL((copy_bs<true, 1, 256>), dim3(grid), dim3(256), 0, st, S, D, n); break;
    case 3: hipLaunchKernelGGL((copy_bs<true, 4, 512>), dim3(grid), dim3(512), 0, st, S, D, n); break;
    case 4: hipLaunchKernelGGL((copy_bs<true, 2, 1024>), dim3(grid), dim3(1024), 0, st, S, D, n); break;
    case 5: hipLaunchKernelGGL((read_only<true>), dim3(grid), dim3(256), 0, st, S, n, reinterpret_cast<uint32_t *>(d)); break;
    case 6: hipLaunchKernelGGL((read_only<false>), dim3(grid), dim3(256), 0, st, S, n, reinterpret_cast<uint32_t *>(d)); break;
    case 7: hipLaunchKernelGGL((write_only<true>), dim3(grid), dim3(256), 0, st, D, n); break;
    case 8: hipLaunchKernelGGL((write_only<false>), dim3(grid), dim3(256), 0, st, D, n); break;
    case 9: hipLaunchKernelGGL((write_only_pol<0>), dim3(grid), dim3(256), 0, st, D, n); break;
    case 10: hipLaunchKernelGGL((write_only_pol<2>), dim3(grid), dim3(256), 0, st, D, n); break;
    case 11: hipLaunchKernelGGL((write_only_pol<16>), dim3(grid), dim3(256), 0, st, D, n); break;
    case 12: hipLaunchKernelGGL((write_only_pol<17>), dim3(grid), dim3(256), 0, st, D, n); break;
    case 13: hipLaunchKernelGGL((write_only_pol<18>), dim3(grid), dim3(256), 0, st, D, n); break;
    case 14: hipLaunchKernelGGL((write_only_pol<1>), dim3(grid), dim3(256), 0, st, D, n); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
