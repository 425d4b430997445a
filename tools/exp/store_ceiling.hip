// store_ceiling.hip -- write-only and read+write stream ceilings by store shape.
// Experimental only (tools/, never shipped): built to tools/exp/libstore.so and
// driven by tools/exp/run_store_ceiling.py.
//
// One kernel covers every shape.  A wave owns units u = w, w + nwaves, ...; per
// unit it loads `rch` bytes (16 B per lane, contiguous) from src + u * rch and
// stores `wch` bytes to dst + u * wch, W bytes per lane per store instruction
// (64 W contiguous bytes per wave-instruction).  wch == 64 W is the plain
// grid-stride stream; wch = 4096 is the fused read's tile (16 rows x 256 B).
// The stored value depends on the unit's loads, so stores wait for them, as in
// the fused read.  PF issues the next unit's loads before the current unit's
// stores (the fused read's prefetch).  Dynamic LDS caps workgroups per CU.
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/kvecc_internal.h"
#include <hip/hip_ext.h>

using namespace kvecc;

template <int W>
struct Vec;
template <>
struct Vec<4> {
  using T = uint32_t;
  __device__ static T make(uint32_t x) { return x; }
};
template <>
struct Vec<8> {
  using T = __attribute__((ext_vector_type(2))) uint32_t;
  __device__ static T make(uint32_t x) { return T{x, x ^ 1u}; }
};
template <>
struct Vec<16> {
  using T = u32x4;
  __device__ static T make(uint32_t x) { return T{x, x ^ 1u, x ^ 2u, x ^ 3u}; }
};

// per > 0: a wave owns the `per` consecutive units [gw * per, gw * per + per)
// instead of the grid stride; tab > 0: each workgroup first copies `tab` bytes
// of an L2-resident table into LDS (the fused read's 32 KiB Golay tables).
template <int W, bool NT, int BS, bool PF>
__global__ __launch_bounds__(BS) void probe(const char *__restrict__ src, char *__restrict__ dst, uint32_t rch,
                                            uint32_t wch, uint32_t units, uint32_t per, uint32_t tab,
                                            const u32x4 *__restrict__ table) {
  using T = typename Vec<W>::T;
  extern __shared__ u32x4 lds[];
  if (tab) {
    for (uint32_t i = threadIdx.x; i < tab / 16; i += BS) lds[i] = table[i];
    __syncthreads();
  }
  const uint32_t lane = threadIdx.x % 64;
  const uint32_t gw = blockIdx.x * (BS / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint32_t nwaves = per ? 1u : gridDim.x * (BS / 64);
  uint32_t u = per ? gw * per : gw;
  if (per) units = min(units, u + per);
  const uint32_t nl = (rch + 1023) / 1024;  // <= 4 load instructions per unit
  u32x4 r[4];
  auto load = [&](uint32_t uu) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t off = 1024 * i + 16 * lane;
      if (i < (int)nl && off < rch)
        r[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + (size_t)uu * rch + off));
      else
        r[i] = u32x4{0, 0, 0, 0};
    }
  };
  if (rch && u < units) load(u);
  for (; u < units; u += nwaves) {
    uint32_t acc = lane;
    if (rch) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc ^= r[i].x ^ r[i].y ^ r[i].z ^ r[i].w;
      if (PF && u + nwaves < units) load(u + nwaves);
    }
    if (tab) acc ^= reinterpret_cast<const uint32_t *>(lds)[(acc + lane) % (tab / 4)];
    const T v = Vec<W>::make(acc);
    char *base = dst + (size_t)u * wch + W * lane;
    const uint32_t ni = wch / (64 * W);
#pragma unroll 4
    for (uint32_t i = 0; i < ni; ++i) {
      T *p = reinterpret_cast<T *>(base + (size_t)i * 64 * W);
      if (NT)
        __builtin_nontemporal_store(v, p);
      else
        *p = v;
    }
    if (rch && !PF && u + nwaves < units) load(u + nwaves);
  }
}

static uint32_t g_per = 0, g_tab = 0;
static const u32x4 *g_table = nullptr;

template <int W, bool NT, int BS, bool PF>
static int launch(const char *s, char *d, uint32_t rch, uint32_t wch, uint32_t units, int grid, int lds,
                  hipStream_t st) {
  hipLaunchKernelGGL((probe<W, NT, BS, PF>), dim3(grid), dim3(BS), lds, st, s, d, rch, wch, units, g_per, g_tab,
                     g_table);
  return 0;
}

template <int W, bool NT, bool PF>
static int by_bs(int bs, const char *s, char *d, uint32_t rch, uint32_t wch, uint32_t units, int grid, int lds,
                 hipStream_t st) {
  switch (bs) {
    case 256: return launch<W, NT, 256, PF>(s, d, rch, wch, units, grid, lds, st);
    case 512: return launch<W, NT, 512, PF>(s, d, rch, wch, units, grid, lds, st);
    case 1024: return launch<W, NT, 1024, PF>(s, d, rch, wch, units, grid, lds, st);
  }
  return -1;
}

template <int W>
static int by_flags(bool nt, bool pf, int bs, const char *s, char *d, uint32_t rch, uint32_t wch, uint32_t units,
                    int grid, int lds, hipStream_t st) {
  if (nt) return pf ? by_bs<W, true, true>(bs, s, d, rch, wch, units, grid, lds, st)
                    : by_bs<W, true, false>(bs, s, d, rch, wch, units, grid, lds, st);
  return pf ? by_bs<W, false, true>(bs, s, d, rch, wch, units, grid, lds, st)
            : by_bs<W, false, false>(bs, s, d, rch, wch, units, grid, lds, st);
}

// FIX: the fused-read mix (rch 2816, wch 4096, W 16) with a fixed instruction
// count per unit -- 3 loads (the last one masked through the offset), 4 stores,
// the next unit's loads always issued (clamped to the last unit) and the
// preheader's loads drained explicitly -- so every path into the loop header
// has the same VMEM ops after the loads and the compiler can wait for the
// loads alone (vmcnt(4)) instead of for the previous unit's stores (vmcnt(0)).
template <bool PF>
__global__ __launch_bounds__(256) void probe_fix(const char *__restrict__ src, char *__restrict__ dst, uint32_t units,
                                                uint32_t per) {
  const uint32_t lane = threadIdx.x % 64;
  const uint32_t gw = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint32_t nwaves = per ? 1u : gridDim.x * 4;
  uint32_t u = per ? gw * per : gw;
  const uint32_t uend = per ? min(units, u + per) : units;
  if (u >= uend) return;
  u32x4 r[3];
  auto load = [&](uint32_t uu) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char *>(src) + (size_t)__builtin_amdgcn_readfirstlane(uu) * 2816, 0, 2816, 0x00020000);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      r[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 * i + 16 * lane, 0, 2));
  };
  load(u);
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) expcnt(7) lgkmcnt(0): drain the preheader
  for (;;) {
    uint32_t acc = lane;
#pragma unroll
    for (int i = 0; i < 3; ++i) acc ^= r[i].x ^ r[i].y ^ r[i].z ^ r[i].w;
    const uint32_t cur = u;
    u += nwaves;
    const bool more = u < uend;
    load(more ? u : cur);  // always issued: a fixed VMEM count per iteration
    const __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(
        dst + (size_t)__builtin_amdgcn_readfirstlane(cur) * 4096, 0, 4096, 0x00020000);
    const u32x4 v{acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), ws,
                                             1024 * i + 16 * lane, 0, 2);
    if (!more) break;
  }
}

extern "C" __attribute__((visibility("default"))) int store_probe_fix(const void *src, void *dst, uint32_t units,
                                                                      uint32_t per, int grid, int lds, void *stream) {
  hipLaunchKernelGGL((probe_fix<true>), dim3(grid), dim3(256), lds, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const char *>(src), reinterpret_cast<char *>(dst), units, per);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// DYN: the fused-read mix, persistent workgroups of 4 waves taking groups of 4
// consecutive units from 8 interleaved atomic counters (counter x hands out
// groups x, x + 8, ...), so units are taken in ascending order across the chip
// as a dispatcher would hand them out, while a workgroup lives for the whole
// launch (the fused Golay read stages 32 KiB of tables per workgroup).
__global__ __launch_bounds__(256) void probe_dyn(const char *__restrict__ src, char *__restrict__ dst, uint32_t units,
                                                 uint32_t *ctr) {
  __shared__ uint32_t grab;
  const uint32_t lane = threadIdx.x % 64;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint32_t x = blockIdx.x % 8;
  const uint32_t groups = (units + 3) / 4;
  for (;;) {
    if (threadIdx.x == 0) grab = atomicAdd(ctr + 32 * x, 1u) * 8 + x;
    __syncthreads();
    const uint32_t g = __builtin_amdgcn_readfirstlane(grab);
    __syncthreads();
    if (g >= groups) break;
    const uint32_t u = g * 4 + wave;
    if (u < units) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char *>(src) + (size_t)u * 2816, 0, 2816, 0x00020000);
      u32x4 r[3];
#pragma unroll
      for (int i = 0; i < 3; ++i)
        r[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 * i + 16 * lane, 0, 2));
      uint32_t acc = lane;
#pragma unroll
      for (int i = 0; i < 3; ++i) acc ^= r[i].x ^ r[i].y ^ r[i].z ^ r[i].w;
      const u32x4 v{acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
      u32x4 *o = reinterpret_cast<u32x4 *>(dst + (size_t)u * 4096) + lane;
#pragma unroll
      for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(v, o + 64 * i);
    }
  }
}

extern "C" __attribute__((visibility("default"))) int store_probe_dyn(const void *src, void *dst, uint32_t units,
                                                                      void *ctr, int grid, int lds, void *start,
                                                                      void *stop, void *stream) {
  hipExtLaunchKernelGGL(probe_dyn, dim3(grid), dim3(256), lds, reinterpret_cast<hipStream_t>(stream),
                        reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop), 0u,
                        reinterpret_cast<const char *>(src), reinterpret_cast<char *>(dst), units,
                        reinterpret_cast<uint32_t *>(ctr));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// PERM: the fused-read mix with the reads gathered like the shim cache's:
// unit u = (side, bh, lb) with lb fastest (256 logical blocks per (b, h), 32
// heads, 8 sequences, 2 sides); its 2816 source bytes sit at physical block
// perm[b * 256 + lb] of that head (random permutation of 2048 blocks), the
// 32 heads of a block adjacent.  One unit per wave, full grid.
__global__ __launch_bounds__(256) void probe_perm(const char *__restrict__ src, char *__restrict__ dst,
                                                  uint32_t units, const int32_t *__restrict__ perm) {
  const uint32_t lane = threadIdx.x % 64;
  const uint32_t u = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  if (u >= units) return;
  const uint32_t per_side = units / 2, side = u / per_side, r = u - side * per_side;
  const uint32_t lb = r % 256, bh = r / 256, b = bh / 32, h = bh % 32;
  const uint32_t blk = perm ? (uint32_t)perm[b * 256 + lb] : b * 256 + lb;
  const size_t su = ((size_t)side * 2048 + blk) * 32 + h;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(src) + su * 2816, 0, 2816, 0x00020000);
  u32x4 rr[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    rr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 * i + 16 * lane, 0, 2));
  uint32_t acc = lane;
#pragma unroll
  for (int i = 0; i < 3; ++i) acc ^= rr[i].x ^ rr[i].y ^ rr[i].z ^ rr[i].w;
  const u32x4 v{acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
  u32x4 *o = reinterpret_cast<u32x4 *>(dst + (size_t)u * 4096) + lane;
#pragma unroll
  for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(v, o + 64 * i);
}

extern "C" __attribute__((visibility("default"))) int store_probe_perm(const void *src, void *dst, uint32_t units,
                                                                       const void *perm, int lds, void *stream) {
  hipLaunchKernelGGL(probe_perm, dim3((units + 3) / 4), dim3(256), lds, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const char *>(src), reinterpret_cast<char *>(dst), units,
                     reinterpret_cast<const int32_t *>(perm));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" __attribute__((visibility("default"))) void store_probe_mode(uint32_t per, uint32_t tab,
                                                                       const void *table) {
  g_per = per;
  g_tab = tab;
  g_table = reinterpret_cast<const u32x4 *>(table);
}

extern "C" __attribute__((visibility("default"))) int store_probe(const void *src, void *dst, uint32_t rch,
                                                                  uint32_t wch, uint32_t units, int w, int nt, int pf,
                                                                  int bs, int grid, int lds, void *stream) {
  if (wch % (64 * w) || rch > 4096) return -3;
  auto s = reinterpret_cast<const char *>(src);
  auto d = reinterpret_cast<char *>(dst);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int rc;
  switch (w) {
    case 4: rc = by_flags<4>(nt, pf, bs, s, d, rch, wch, units, grid, lds, st); break;
    case 8: rc = by_flags<8>(nt, pf, bs, s, d, rch, wch, units, grid, lds, st); break;
    case 16: rc = by_flags<16>(nt, pf, bs, s, d, rch, wch, units, grid, lds, st); break;
    default: return -1;
  }
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
