// golay_read_exp.hip -- experimental variants of the fused Golay read
// (csrc/shim.hip shim_read_golay_tiles_kernel), NOT shipped.  Built with the
// product sources (this file #includes shim.hip for its tile helpers) into
// tools/exp/libgread.so; tools/exp/run_golay_read_exp.py times every variant
// against the product kernel in one process and compares the outputs.
//
// Variant axes (template parameters, so one library holds all of them and a
// rocprofv3 run tells them apart by kernel name):
//   SCHED  0: the product's persistent grid + dynamic tail; 1: a full grid,
//          wave w takes tiles [w CHUNK, w CHUNK + CHUNK) and workgroups retire
//   STAGE  0: tables staged first (VGPR copy), then the first tile's loads (the
//          product); 1: the first tile's loads first, then the VGPR copy;
//          2: the first tile's loads first, then the tables by LDS-DMA
//          (global_load_lds_dwordx4: no VGPRs, no wait before the barrier)
//   GATHER 0: the real table lookups; 1: lookups at lane-private, conflict-free
//          addresses (same instruction count, WRONG values: attributes the LDS
//          bank conflicts); 2: no lookups (WRONG values: the memory ceiling)
//          3: split parity in LDS, the correction entry from the global table;
//          4: uint16 tables (8.25 KiB); 5: the byte-class tables (5.1 KiB, below)
//   SPLITP the parity half as two 64-entry tables (16.5 KiB of tables)
//   PAD    extra bytes per staged row in the phase-2 tile
//   BLOCK  threads per workgroup
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/shim.hip"

#include <vector>

#include "golay_bc.h"

namespace kvecc {
namespace exp {

// ORDER 1: tile u -> (side, b, lb, ch, h), heads fastest: the waves of one
// window read whole physical blocks (all heads of a block are contiguous in
// the cache) instead of one head's 2.75 KB slice of randomly placed blocks;
// the outputs (one 4 KiB [pos, d] tile per wave) land 1 MiB apart instead of
// contiguous.  0: the product's order (shim_tile), lb fastest.
template <int ORDER>
__device__ __forceinline__ ShimTile tile_at(const ShimTileArgs &a, uint32_t u) {
  if (ORDER == 0) return shim_tile(a, u);
  ShimTile t;
  const uint32_t per_side = a.units / 2;
  t.side = u >= per_side ? 1u : 0u;
  u -= t.side * per_side;
  const uint32_t h = u % a.hkv;
  u /= a.hkv;
  const uint32_t ch = u % a.tpb;
  u /= a.tpb;
  const uint32_t lb = u % a.nlb;
  const uint32_t b = u / a.nlb;
  t.bh = b * a.hkv + h;
  t.pos0 = lb * a.bs + ch * a.tr;
  t.rows = t.pos0 < a.ctx ? min(min(a.tr, a.bs - ch * a.tr), a.ctx - t.pos0) : 0u;
  const int32_t blk = ld_scalar(a.table + (int64_t)b * a.tstride + lb);
  t.row0 = blk < 0 ? -1 : (((int64_t)blk * a.layers + a.layer) * a.hkv + h) * a.bs + ch * a.tr;
  return t;
}

template <int SCHED, int CHUNK, int STAGE, int GATHER, int SPLITP, int PAD, int BLOCK, bool PACKED, int PCT = 65,
          int ORDER = 0>
__global__ __launch_bounds__(BLOCK) void golay_read_exp_kernel(ShimTileArgs a, const uint16_t *par16,
                                                               const uint16_t *cor16) {
  using TO = __half;
  constexpr int kW = BLOCK / kWave;
  // GATHER 3: only the split parity tables in LDS; the correction entry comes
  // from the global table (16 KiB, cache-resident; ~79 % of lanes read entry 0)
  // GATHER 4: uint16 tables, 8.25 KiB: split parity (12 bits) and the correction
  // (data error | count << 12); the nibbles are spread by VALU
  // GATHER 5: the byte-class decoder (bc_tables below), 5.1 KiB
  constexpr int kTab = GATHER == 5 ? kBcAlloc : GATHER == 3 ? 128 : GATHER == 4 ? (128 + 4096) / 2 : SPLITP ? 128 + 4096 : 8192;
  __shared__ __attribute__((aligned(16))) uint32_t tab[kTab];
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kW][kTileStage];
  __shared__ float scale_all[kW][kWave];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  const uint32_t nwaves = gridDim.x * kW;
  const uint32_t lr = a.lr + PAD;
  const uint32_t groups = a.tr * a.gpr;
  constexpr int V = kVpl<TO>, NC = kTileChunks * 8 / V;
  const uint32_t dv = a.d / V;
  const uint32_t chunks = a.tr * dv;
  TileItems it;
#pragma unroll
  for (int i = 0; i < kTileGroups; ++i) {
    const uint32_t f = lane + kWave * i;
    it.r1[i] = f / a.gpr;
    it.q1[i] = f - it.r1[i] * a.gpr;
  }
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const uint32_t v = lane + kWave * i;
    it.r2[i] = v / dv;
    it.j2[i] = it.r2[i] * lr + V * (v - it.r2[i] * dv);
    it.o2[i] = (it.r2[i] * a.d + V * (v - it.r2[i] * dv)) * (uint32_t)sizeof(TO);
  }
  uint32_t bits = 0, unc = 0;
  const uint32_t gw = blockIdx.x * kW + wave;
  uint32_t u = SCHED ? gw * CHUNK : gw;
  const uint32_t uend = SCHED ? min(a.units, u + CHUNK) : a.units;
  TileSchedule sched;
  ShimTile cur;
  u32x4 w[kTileGroups];
  float scale;
  const bool active = u < uend;
  auto stage_tables = [&]() {
    if (STAGE == 2) {
      // LDS-DMA: each wave-instruction writes 1 KiB (lane l at base + 16 l)
      const char *src = reinterpret_cast<const char *>(GATHER == 5 ? reinterpret_cast<const void *>(par16) : a.atab);
      if (GATHER == 5) {
        for (int c = wave; c < kBcAlloc / 256; c += kW)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + 1024 * c + 16 * lane),
                                           reinterpret_cast<__attribute__((address_space(3))) void *>(
                                               reinterpret_cast<uintptr_t>(tab) + 1024 * c),
                                           16, 0, 0);
        return;
      } else if (SPLITP) {
        // parity pieces are gathers (entries i and i << 6): plain copy below
      } else {
        for (int c = wave; c < 32; c += kW)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + 1024 * c + 16 * lane),
                                           reinterpret_cast<__attribute__((address_space(3))) void *>(
                                               reinterpret_cast<uintptr_t>(tab) + 1024 * c),
                                           16, 0, 0);
        return;
      }
    }
    if (GATHER == 5) {
      const u32x4 *s4 = reinterpret_cast<const u32x4 *>(par16);
      u32x4 *d4 = reinterpret_cast<u32x4 *>(tab);
      for (int i = threadIdx.x; i < kBcWords / 4; i += BLOCK) d4[i] = s4[i];
    } else if (GATHER == 4) {
      uint16_t *t16 = reinterpret_cast<uint16_t *>(tab);
      for (int i = threadIdx.x; i < 128; i += BLOCK) t16[i] = par16[i < 64 ? i : (i - 64) << 6];
      const u32x4 *s4 = reinterpret_cast<const u32x4 *>(cor16);
      u32x4 *d4 = reinterpret_cast<u32x4 *>(t16 + 128);
      for (int i = threadIdx.x; i < 512; i += BLOCK) d4[i] = s4[i];
    } else if (GATHER == 3) {
      for (int i = threadIdx.x; i < 128; i += BLOCK) tab[i] = a.atab[i < 64 ? i : (i - 64) << 6];
    } else if (SPLITP) {
      for (int i = threadIdx.x; i < 128; i += BLOCK) tab[i] = a.atab[i < 64 ? i : (i - 64) << 6];
      const u32x4 *s4 = reinterpret_cast<const u32x4 *>(a.atab + 4096);
      u32x4 *d4 = reinterpret_cast<u32x4 *>(tab + 128);
      for (int i = threadIdx.x; i < 1024; i += BLOCK) d4[i] = s4[i];
    } else {
      const u32x4 *s4 = reinterpret_cast<const u32x4 *>(a.atab);
      u32x4 *d4 = reinterpret_cast<u32x4 *>(tab);
#pragma unroll
      for (int i = threadIdx.x; i < 2048; i += BLOCK) d4[i] = s4[i];
    }
  };
  if (STAGE == 0) {
    stage_tables();
    __syncthreads();
    if (!active) return;
    if (SCHED == 0) sched.init(a.units, a.dyn, gw, nwaves, lane, PCT);
    cur = tile_at<ORDER>(a, u);
    tile_issue<PACKED>(a, cur, lane, it, w, scale);
  } else {
    // the first tile's loads go out before the tables (a full grid has no
    // inactive waves; a persistent one may: they still help stage)
    if (active) {
      if (SCHED == 0) sched.init(a.units, a.dyn, gw, nwaves, lane, PCT);
      cur = tile_at<ORDER>(a, u);
      tile_issue<PACKED>(a, cur, lane, it, w, scale);
    }
    stage_tables();
    if (STAGE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!active) return;
  }
  uint8_t *stage = stage_all[wave];
  const __amdgpu_buffer_rsrc_t crs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(a.atab + 4096), 0, 16384, 0x00020000);
  for (;;) {
    scale_all[wave][lane] = scale;
    uint32_t cnt = 0, bc_tot = 0, bc_unc = 0;
#pragma unroll
    for (int i = 0; i < kTileGroups; ++i) {
      if (i * kWave >= (int)groups) break;
      const uint32_t q = it.q1[i];
      uint32_t sp[4];
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {
        const int c = c4;
        uint32_t cw = tile_cw<PACKED>(w[i], c);
        if (c > 0) cw = 4 * q + c < a.g ? cw : 0u;
        const char *tb = reinterpret_cast<const char *>(tab);
        uint32_t p, e;
        if (GATHER == 5) {
          // p: spread(lo) | parity(lo) << 20; s: syndrome; us: spread(B s);
          // b: the syndrome's class byte; de = flag ? B (s ^ m) : m, spread
          const uint8_t *c8 = reinterpret_cast<const uint8_t *>(tab + kBcBytes);
          const uint32_t p = tab[cw & 63u] ^ tab[64 + ((cw >> 6) & 63u)];
          const uint32_t s = ((cw >> 12) ^ (p >> 20)) & 0xFFFu;
          const uint32_t us = tab[128 + (s & 63u)] ^ tab[192 + (s >> 6)];
          const uint32_t b = c8[s];
          const uint32_t k = tab[256 + (b & 31u)];
          const uint32_t mask = (uint32_t)__builtin_amdgcn_sbfe((int)b, 4, 1);
          sp[c4] = __builtin_amdgcn_bitop3_b32(p, (mask & us) ^ k, 0x000F0F0Fu, 0x28);
          bc_tot += b >> 5;  // n: 0-3 bits corrected, 4 uncorrectable
          bc_unc += b >> 7;
          continue;
        } else if (GATHER == 4) {
          const uint16_t *t16 = reinterpret_cast<const uint16_t *>(tab);
          const uint32_t par = (uint32_t)t16[cw & 63u] ^ (uint32_t)t16[64 + ((cw >> 6) & 63u)];
          const uint32_t c = t16[128 + (((cw >> 12) ^ par) & 0xFFFu)];  // error | count << 12
          const uint32_t x = (cw ^ c) & 0xFFFu;
          sp[c4] = (x & 0xFu) | (x & 0xF0u) << 4 | (x & 0xF00u) << 8;
          const uint32_t n = c >> 12;  // 0-3 bits corrected, 4 = uncorrectable
          cnt += n + (n >> 2) * 60u;  // (n & 3) | uncorrectable << 6
          continue;
        } else if (GATHER == 2) {
          p = cw;
          e = 0;
        } else if (GATHER == 3) {
          p = *reinterpret_cast<const uint32_t *>(tb + ((cw << 2) & 0xFCu)) ^
              *reinterpret_cast<const uint32_t *>(tb + 256 + ((cw >> 4) & 0xFCu));
          e = __builtin_amdgcn_raw_buffer_load_b32(crs, ((cw >> 10) ^ (p >> 18)) & 0x3FFCu, 0, 0);
        } else if (GATHER == 1) {  // bank = lane % 32: conflict-free, data-dependent row
          p = *reinterpret_cast<const uint32_t *>(tb + 4 * ((lane & 31u) + 32u * (cw & 127u)));
          e = *reinterpret_cast<const uint32_t *>(tb + 4 * (kTab - 4096) +
                                                   4 * ((lane & 31u) + 32u * (((cw >> 12) ^ p) & 127u)));
        } else {
          if (SPLITP)
            p = *reinterpret_cast<const uint32_t *>(tb + ((cw << 2) & 0xFCu)) ^
                *reinterpret_cast<const uint32_t *>(tb + 256 + ((cw >> 4) & 0xFCu));
          else
            p = *reinterpret_cast<const uint32_t *>(tb + ((cw << 2) & 0x3FFCu));
          e = *reinterpret_cast<const uint32_t *>(tb + 4 * (kTab - 4096) + (((cw >> 10) ^ (p >> 18)) & 0x3FFCu));
        }
        sp[c] = __builtin_amdgcn_bitop3_b32(p, e, 0x000F0F0Fu, 0x28);
        cnt += e >> 24;
      }
      if (it.r1[i] < a.tr) {
        uint32_t *dst = reinterpret_cast<uint32_t *>(stage + it.r1[i] * lr + 12 * q);
        dst[0] = sp[0] | sp[1] << 24;
        dst[1] = sp[1] >> 8 | sp[2] << 16;
        dst[2] = sp[2] >> 16 | sp[3] << 8;
      }
    }
    bits += (cnt & 63u) + bc_tot - 4u * bc_unc;
    unc += (cnt >> 6) + bc_unc;
    wave_lds_sync();
    const ShimTile t = cur;
    u = SCHED == 0 ? sched.next(u, lane) : u + 1;
    const bool more = u < uend;
    if (more) {
      cur = tile_at<ORDER>(a, u);
      tile_issue<PACKED>(a, cur, lane, it, w, scale);
    }
    const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
    const bool dead = t.row0 < 0;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      if (i * kWave >= (int)chunks) break;
      const uint32_t *src = reinterpret_cast<const uint32_t *>(stage + it.j2[i]);
      const uint32_t nb[2] = {src[0], src[1]};
      tile_store(os, it.o2[i], dq16<TO>(nb, scale_all[wave][min(it.r2[i], a.tr - 1)], dead));
    }
    if (!more) break;
    wave_lds_sync();
  }
  bits = wave_sum(bits);
  unc = wave_sum(unc);
  if (lane == 0) {
    uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
    if (bits) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)bits);
    if (unc) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)unc);
  }
}

// Two tiles of codeword loads in flight per wave: while tile t is decoded and
// stored, the loads of t + 1 (issued one tile earlier) and t + 2 (issued after
// t's phase 1) are outstanding.  Persistent grid with the product's schedule.
template <int BLOCK, bool PACKED, int PCT>
__global__ __launch_bounds__(BLOCK) void golay_read_pf2_kernel(ShimTileArgs a, const uint16_t *, const uint16_t *) {
  using TO = __half;
  constexpr int kW = BLOCK / kWave;
  __shared__ __attribute__((aligned(16))) uint32_t tab[8192];
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kW][kTileStage];
  __shared__ float scale_all[kW][kWave];
  {
    const u32x4 *s4 = reinterpret_cast<const u32x4 *>(a.atab);
    u32x4 *d4 = reinterpret_cast<u32x4 *>(tab);
#pragma unroll
    for (int i = threadIdx.x; i < 2048; i += BLOCK) d4[i] = s4[i];
  }
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  const uint32_t nwaves = gridDim.x * kW;
  const uint32_t groups = a.tr * a.gpr;
  constexpr int V = kVpl<TO>, NC = kTileChunks * 8 / V;
  const uint32_t dv = a.d / V;
  const uint32_t chunks = a.tr * dv;
  TileItems it;
#pragma unroll
  for (int i = 0; i < kTileGroups; ++i) {
    const uint32_t f = lane + kWave * i;
    it.r1[i] = f / a.gpr;
    it.q1[i] = f - it.r1[i] * a.gpr;
  }
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const uint32_t v = lane + kWave * i;
    const uint32_t r = v / dv, j = v - r * dv;
    it.r2[i] = min(r, a.tr - 1);
    it.j2[i] = it.r2[i] * a.lr + V * j;
    it.o2[i] = (r * a.d + V * j) * (uint32_t)sizeof(TO);
  }
  uint32_t bits = 0, unc = 0;
  const uint32_t gw = blockIdx.x * kW + wave;
  if (gw >= a.units) return;
  TileSchedule sched;
  sched.init(a.units, a.dyn, gw, nwaves, lane, PCT);
  uint8_t *stage = stage_all[wave];
  struct Buf {
    ShimTile t;
    u32x4 w[kTileGroups];
    float s;
    bool v;
  };
  Buf A, B;
  uint32_t ulast = gw;  // the index of the most recently issued tile
  bool done = false;    // the schedule ran out
  auto refill = [&](Buf &x) {
    x.v = false;
    if (done) return;
    ulast = sched.next(ulast, lane);
    if (ulast >= a.units) {
      done = true;
      return;
    }
    x.v = true;
    x.t = shim_tile(a, ulast);
    tile_issue<PACKED>(a, x.t, lane, it, x.w, x.s);
  };
  A.v = true;
  A.t = shim_tile(a, gw);
  tile_issue<PACKED>(a, A.t, lane, it, A.w, A.s);
  refill(B);
  auto process = [&](Buf &x) {
    scale_all[wave][lane] = x.s;
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < kTileGroups; ++i) {
      if (i * kWave >= (int)groups) break;
      const uint32_t q = it.q1[i];
      uint32_t sp[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t cw = tile_cw<PACKED>(x.w[i], c);
        if (c > 0) cw = 4 * q + c < a.g ? cw : 0u;
        const char *tb = reinterpret_cast<const char *>(tab);
        const uint32_t p = *reinterpret_cast<const uint32_t *>(tb + ((cw << 2) & 0x3FFCu));
        const uint32_t e = *reinterpret_cast<const uint32_t *>(tb + 16384 + (((cw >> 10) ^ (p >> 18)) & 0x3FFCu));
        sp[c] = __builtin_amdgcn_bitop3_b32(p, e, 0x000F0F0Fu, 0x28);
        cnt += e >> 24;
      }
      if (it.r1[i] < a.tr) {
        uint32_t *dst = reinterpret_cast<uint32_t *>(stage + it.r1[i] * a.lr + 12 * q);
        dst[0] = sp[0] | sp[1] << 24;
        dst[1] = sp[1] >> 8 | sp[2] << 16;
        dst[2] = sp[2] >> 16 | sp[3] << 8;
      }
    }
    bits += cnt & 63u;
    unc += cnt >> 6;
    wave_lds_sync();
    const ShimTile t = x.t;
    refill(x);  // the tile after the other buffer's
    const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
    const bool dead = t.row0 < 0;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      if (i * kWave >= (int)chunks) break;
      const uint32_t *src = reinterpret_cast<const uint32_t *>(stage + it.j2[i]);
      const uint32_t nb[2] = {src[0], src[1]};
      tile_store(os, it.o2[i], dq16<TO>(nb, scale_all[wave][it.r2[i]], dead));
    }
    wave_lds_sync();
  };
  for (;;) {
    process(A);
    if (!B.v) break;
    process(B);
    if (!A.v) break;
  }
  bits = wave_sum(bits);
  unc = wave_sum(unc);
  if (lane == 0) {
    uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
    if (bits) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)bits);
    if (unc) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)unc);
  }
}

// DIRECT: no LDS tile.  Lane l of a wave takes output chunk j = l & 15 (values
// 8j..8j+7 of a row: one 16-byte store) of row 4i + (l >> 4), i = 0..3, of the
// wave's 16-row tile: it loads the 4 codewords c0 = 8j/3 .. c0 + 3 of its row
// (16 bytes at a 4-byte aligned offset; the last lane's 4th is past the row and
// unused), decodes them, and selects its 8 nibbles with two v_perm.  Each
// codeword is decoded by up to two lanes; the statistics count it at the lane
// holding its first nibble.  d = 128 (43 codewords per row), fp16 out, int32 caches.
// SCHED 0: the product's persistent schedule (PCT static); 1: a full grid.
// TABK 0: the 32 KiB spread tables; 1: the byte-class tables (golay_bc.h).
// STG 1 (full grid): the tables come by LDS-DMA, issued first; then the
// wave's tile loads; a counted vmcnt retires only the DMA before a raw
// s_barrier, so the tile's HBM loads are in flight while the tables land.
template <int SCHED, int TABK, int BLOCK, int PCT = 30, int STG = 0>
__global__ __launch_bounds__(BLOCK) void golay_read_direct_kernel(ShimTileArgs a, const uint16_t *bc16,
                                                                  const uint16_t *) {
  using TO = __half;
  constexpr int kW = BLOCK / kWave;
  constexpr int kTab = TABK ? (STG ? kBcAlloc : kBcWords) : 8192;
  __shared__ __attribute__((aligned(16))) uint32_t tab[kTab];
  const uint32_t *tsrc = TABK ? reinterpret_cast<const uint32_t *>(bc16) : a.atab;
  if (STG == 0) {
    const u32x4 *s4 = reinterpret_cast<const u32x4 *>(tsrc);
    u32x4 *d4 = reinterpret_cast<u32x4 *>(tab);
    for (int i = threadIdx.x; i < kTab / 4; i += BLOCK) d4[i] = s4[i];
    __syncthreads();
  }
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  const uint32_t rg = lane >> 4, j = lane & 15;
  const uint32_t c0 = (8 * j) / 3, f = (8 * j) % 3;
  const uint32_t selA = f == 0 ? 0x04020100u : f == 1 ? 0x05040201u : 0x06050402u;
  const uint32_t selB = f == 0 ? 0x05040201u : f == 1 ? 0x06050402u : 0x04020100u;
  const bool f2 = f == 2;
  uint32_t own = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (3 * (c0 + k) >= 8 * j && 3 * (c0 + k) <= 8 * j + 7) own |= 1u << k;
  const uint32_t gw = blockIdx.x * kW + wave, nwaves = gridDim.x * kW;
  uint32_t u = gw;
  if (STG == 0 && u >= a.units) return;
  TileSchedule sched;
  if (STG == 0 && SCHED == 0) sched.init(a.units, a.dyn, gw, nwaves, lane, PCT);
  auto issue = [&](const ShimTile &t, u32x4 (&w)[4], float (&sc)[4]) {
    const bool live = t.row0 >= 0;
    const int64_t row0 = live ? t.row0 : 0;
    const uint32_t side = uni(t.side);
    const char *base = uni(reinterpret_cast<const char *>(a.cache[side]) + row0 * (int64_t)a.rowb);
    const char *sbase = uni(reinterpret_cast<const char *>(a.scales[side] + row0));
    const uint32_t nrows = uni(live ? t.rows : 0u);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), 0, (int)(nrows * a.rowb), 0x00020000);
    const __amdgpu_buffer_rsrc_t ss =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(sbase), 0, (int)(4 * nrows), 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t r = 4 * i + rg;
      w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, r * a.rowb + 4 * c0, 0, kTileAux));
      sc[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ss, 4 * r, 0, 0));
    }
  };
  ShimTile cur;
  u32x4 w[4];
  float sc[4];
  if (STG == 1) {
    static_assert(STG == 0 || SCHED == 1, "LDS-DMA staging: full grid only");
    const char *src = reinterpret_cast<const char *>(tsrc);
    for (int c = wave; c < kTab / 256; c += kW)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + 1024 * c + 16 * lane),
                                       reinterpret_cast<__attribute__((address_space(3))) void *>(
                                           reinterpret_cast<uintptr_t>(tab) + 1024 * c),
                                       16, 0, 0);
    const bool active = u < a.units;
    if (active) {
      cur = shim_tile(a, u);
      issue(cur, w, sc);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // the DMA (issued first) has landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (!active) return;
  } else {
    cur = shim_tile(a, u);
    issue(cur, w, sc);
  }
  uint32_t bits = 0, unc = 0;
  const char *tb = reinterpret_cast<const char *>(tab);
  for (;;) {
    const ShimTile t = cur;
    u32x4 wc[4];
    float scc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wc[i] = w[i];
      scc[i] = sc[i];
    }
    bool more = false;
    if (SCHED == 0) {
      u = sched.next(u, lane);
      more = u < a.units;
      if (more) {
        cur = shim_tile(a, u);
        issue(cur, w, sc);
      }
    }
    const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
    const bool dead = t.row0 < 0;
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t sp[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t cw = wc[i][k];
        uint32_t n;
        if (TABK) {
          sp[k] = bc_decode(tab, cw, n);
          n = (n & 3u) | (n >> 2) << 6;
        } else {
          const uint32_t p = *reinterpret_cast<const uint32_t *>(tb + ((cw << 2) & 0x3FFCu));
          const uint32_t e = *reinterpret_cast<const uint32_t *>(tb + 16384 + (((cw >> 10) ^ (p >> 18)) & 0x3FFCu));
          sp[k] = __builtin_amdgcn_bitop3_b32(p, e, 0x000F0F0Fu, 0x28);
          n = e >> 24;
        }
        cnt += (own >> k) & 1u ? n : 0u;
      }
      const uint32_t nb[2] = {__builtin_amdgcn_perm(sp[1], sp[0], selA),
                              __builtin_amdgcn_perm(f2 ? sp[3] : sp[2], f2 ? sp[2] : sp[1], selB)};
      const uint32_t r = 4 * i + rg;
      tile_store(os, (r * 128u + 8u * j) * 2u, dq16<TO>(nb, scc[i], dead));
    }
    bits += cnt & 63u;
    unc += cnt >> 6;
    if (!more) break;
  }
  bits = wave_sum(bits);
  unc = wave_sum(unc);
  if (lane == 0) {
    uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
    if (bits) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)bits);
    if (unc) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)unc);
  }
}

// PROBE (no decode, WRONG values): the fused read's bytes moved with a given
// load pattern, to price the pattern itself.  Full grid, one tile per wave,
// the tile's 16 row scales loaded, 4 KiB stored per tile as the product does.
//   MODE 0: the tile's 2752 bytes as 16-byte loads at 16-byte aligned offsets
//           (1 KiB contiguous per wave-instruction; tile bases are 64-byte aligned)
//   MODE 1: the product's pattern (row r, 4-codeword group q at r * 172 + 16 q)
//   MODE 2: the direct kernel's (4 codewords from 8j/3 of row 4i + l/16)
template <int MODE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void golay_read_probe_kernel(ShimTileArgs a, const uint16_t *, const uint16_t *) {
  constexpr int kW = BLOCK / kWave;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  const uint32_t u = blockIdx.x * kW + wave;
  if (u >= a.units) return;
  const ShimTile t = shim_tile(a, u);
  const bool live = t.row0 >= 0;
  const int64_t row0 = live ? t.row0 : 0;
  const uint32_t side = uni(t.side);
  const char *base = uni(reinterpret_cast<const char *>(a.cache[side]) + row0 * (int64_t)a.rowb);
  const char *sbase = uni(reinterpret_cast<const char *>(a.scales[side] + row0));
  const uint32_t nrows = uni(live ? t.rows : 0u);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), 0, (int)(nrows * a.rowb), 0x00020000);
  const __amdgpu_buffer_rsrc_t ss =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(sbase), 0, (int)(4 * nrows), 0x00020000);
  u32x4 acc = {lane, 0u, 0u, 0u};
  auto mix = [&](const u32x4 &v) { acc = u32x4{acc.x ^ v.x, acc.y ^ v.y, acc.z ^ v.z, acc.w ^ v.w}; };
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      mix(__builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 * i + 16 * lane, 0, kTileAux)));
  } else if (MODE == 1) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const uint32_t f = lane + 64 * i, r = f / 11, q = f - 11 * r;
      if (f < 176)
        mix(__builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, r * a.rowb + 16 * q, 0, kTileAux)));
    }
  } else {
    const uint32_t j = lane & 15, c0 = (8 * j) / 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t r = 4 * i + (lane >> 4);
      mix(__builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, r * a.rowb + 4 * c0, 0, kTileAux)));
    }
  }
  const uint32_t sc = __builtin_amdgcn_raw_buffer_load_b32(ss, 4 * (lane & 15), 0, 0);
  const __amdgpu_buffer_rsrc_t os = tile_out<__half>(a, t);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    tile_store(os, 1024 * i + 16 * lane, u32x4{acc.x ^ sc, acc.y ^ (uint32_t)i, acc.z, acc.w});
}

struct Variant {
  const char *name;
  void (*kern)(ShimTileArgs, const uint16_t *, const uint16_t *);
  int sched, chunk, block;
  int bc;  // passes the byte-class tables (GATHER 5)
};

#define GV(NAME, S, C, ST, G, SP, PD, B, PK) \
  {NAME, golay_read_exp_kernel<S, C, ST, G, SP, PD, B, PK>, S, C, B}
#define GVP(NAME, B, PK, PCT) {NAME, golay_read_exp_kernel<0, 1, 0, 0, 0, 0, B, PK, PCT>, 0, 1, B}

static const Variant kVariants[] = {
    // persistent (product schedule)
    GV("pers", 0, 1, 0, 0, 0, 0, 512, false),
    GV("pers_cfree", 0, 1, 0, 1, 0, 0, 512, false),
    GV("pers_nogather", 0, 1, 0, 2, 0, 0, 512, false),
    GV("pers_pad8", 0, 1, 0, 0, 0, 8, 512, false),
    GV("pers_fetch1st", 0, 1, 1, 0, 0, 0, 512, false),
    GV("pers_glds", 0, 1, 2, 0, 0, 0, 512, false),
    // full grid
    GV("full1_s0", 1, 1, 0, 0, 0, 0, 512, false),
    GV("full1_s1", 1, 1, 1, 0, 0, 0, 512, false),
    GV("full1_glds", 1, 1, 2, 0, 0, 0, 512, false),
    GV("full2_glds", 1, 2, 2, 0, 0, 0, 512, false),
    GV("full4_glds", 1, 4, 2, 0, 0, 0, 512, false),
    GV("full1_glds_b1024", 1, 1, 2, 0, 0, 0, 1024, false),
    GV("full2_glds_b1024", 1, 2, 2, 0, 0, 0, 1024, false),
    GV("full1_splitp_s1", 1, 1, 1, 0, 1, 0, 512, false),
    GV("full2_splitp_s1", 1, 2, 1, 0, 1, 0, 512, false),
    GV("full1_glds_nogather", 1, 1, 2, 2, 0, 0, 512, false),
    GV("full1_glds_cfree", 1, 1, 2, 1, 0, 0, 512, false),
    // packed
    GV("pk_pers", 0, 1, 0, 0, 0, 0, 512, true),
    GV("pk_full1_glds", 1, 1, 2, 0, 0, 0, 512, true),
    GV("pk_full2_glds", 1, 2, 2, 0, 0, 0, 512, true),
    // persistent grids of other workgroup sizes / static shares (waves per CU =
    // block / 64 * per_cu)
    GVP("pers_b256", 256, false, 65),
    GVP("pers_b384", 384, false, 65),
    GVP("pers_b768", 768, false, 65),
    GVP("pers_b1024", 1024, false, 65),
    GVP("pers_b256_p50", 256, false, 50),
    GVP("pers_b256_p75", 256, false, 75),
    GVP("pers_b512_p50", 512, false, 50),
    GVP("pers_b512_p75", 512, false, 75),
    GVP("pk_pers_b256", 256, true, 65),
    GVP("pk_pers_b384", 384, true, 65),
    GVP("pk_pers_b768", 768, true, 65),
    GVP("pk_pers_b256_p50", 256, true, 50),
    GVP("pk_pers_b256_p40", 256, true, 40),
    GVP("pers_b256_p40", 256, false, 40),
    GVP("pers_b256_p30", 256, false, 30),
    GVP("pers_b256_p20", 256, false, 20),
    GVP("pers_b256_p10", 256, false, 10),
    GVP("pk_pers_b256_p30", 256, true, 30),
    GVP("pk_pers_b256_p20", 256, true, 20),
    GVP("pers_b128_p30", 128, false, 30),
    GVP("pers_b384_p30", 384, false, 30),
    {"pers_u16_b256_p30", golay_read_exp_kernel<0, 1, 0, 4, 0, 0, 256, false, 30>, 0, 1, 256},
    {"pers_u16_b512_p30", golay_read_exp_kernel<0, 1, 0, 4, 0, 0, 512, false, 30>, 0, 1, 512},
    {"pers_splitp_b256_p30", golay_read_exp_kernel<0, 1, 0, 0, 1, 0, 256, false, 30>, 0, 1, 256},
    {"pk_pers_u16_b256_p30", golay_read_exp_kernel<0, 1, 0, 4, 0, 0, 256, true, 30>, 0, 1, 256},
    // global correction table, split parity in LDS (0.5 KiB staged per workgroup)
    GV("full1_gc", 1, 1, 0, 3, 1, 0, 512, false),
    GV("full2_gc", 1, 2, 0, 3, 1, 0, 512, false),
    GV("full1_gc_b256", 1, 1, 0, 3, 1, 0, 256, false),
    GV("full2_gc_b256", 1, 2, 0, 3, 1, 0, 256, false),
    GV("pers_gc", 0, 1, 0, 3, 1, 0, 512, false),
    GV("full1_splitp_s0", 1, 1, 0, 0, 1, 0, 512, false),
    GV("full2_splitp_s0", 1, 2, 0, 0, 1, 0, 512, false),
    GV("pk_full1_gc", 1, 1, 0, 3, 1, 0, 512, true),
    GV("pk_full1_gc_b256", 1, 1, 0, 3, 1, 0, 256, true),
    // uint16 tables (8.25 KiB), nibbles spread by VALU
    GV("full1_u16", 1, 1, 0, 4, 0, 0, 512, false),
    GV("full1_u16_b256", 1, 1, 0, 4, 0, 0, 256, false),
    GV("full2_u16", 1, 2, 0, 4, 0, 0, 512, false),
    GV("pers_u16", 0, 1, 0, 4, 0, 0, 512, false),
    GV("full1_splitp_s0_b256", 1, 1, 0, 0, 1, 0, 256, false),
    GV("pk_full1_u16", 1, 1, 0, 4, 0, 0, 512, true),
    GV("pk_full1_splitp_s0", 1, 1, 0, 0, 1, 0, 512, true),
    // heads-fastest tile order
    {"pers_hm", golay_read_exp_kernel<0, 1, 0, 0, 0, 0, 512, false, 65, 1>, 0, 1, 512},
    {"pers_hm_p50", golay_read_exp_kernel<0, 1, 0, 0, 0, 0, 512, false, 50, 1>, 0, 1, 512},
    {"full1_u16_hm", golay_read_exp_kernel<1, 1, 0, 4, 0, 0, 512, false, 65, 1>, 1, 1, 512},
    {"full2_u16_hm", golay_read_exp_kernel<1, 2, 0, 4, 0, 0, 512, false, 65, 1>, 1, 2, 512},
    {"pk_pers_hm", golay_read_exp_kernel<0, 1, 0, 0, 0, 0, 512, true, 65, 1>, 0, 1, 512},
    // byte-class decoder (5.1 KiB of tables): full grids and the product's persistent shape
    {"full1_bc", golay_read_exp_kernel<1, 1, 0, 5, 0, 0, 512, false>, 1, 1, 512, 1},
    {"full2_bc", golay_read_exp_kernel<1, 2, 0, 5, 0, 0, 512, false>, 1, 2, 512, 1},
    {"full1_bc_b256", golay_read_exp_kernel<1, 1, 0, 5, 0, 0, 256, false>, 1, 1, 256, 1},
    {"full2_bc_b256", golay_read_exp_kernel<1, 2, 0, 5, 0, 0, 256, false>, 1, 2, 256, 1},
    {"full1_bc_s1", golay_read_exp_kernel<1, 1, 1, 5, 0, 0, 512, false>, 1, 1, 512, 1},
    {"full1_bc_glds", golay_read_exp_kernel<1, 1, 2, 5, 0, 0, 512, false>, 1, 1, 512, 1},
    {"full2_bc_glds", golay_read_exp_kernel<1, 2, 2, 5, 0, 0, 512, false>, 1, 2, 512, 1},
    {"full1_bc_b1024", golay_read_exp_kernel<1, 1, 0, 5, 0, 0, 1024, false>, 1, 1, 1024, 1},
    {"full1_bc_glds_b1024", golay_read_exp_kernel<1, 1, 2, 5, 0, 0, 1024, false>, 1, 1, 1024, 1},
    {"pers_bc_b256_p30", golay_read_exp_kernel<0, 1, 0, 5, 0, 0, 256, false, 30>, 0, 1, 256, 1},
    {"pk_full1_bc", golay_read_exp_kernel<1, 1, 0, 5, 0, 0, 512, true>, 1, 1, 512, 1},
    {"pk_full2_bc", golay_read_exp_kernel<1, 2, 0, 5, 0, 0, 512, true>, 1, 2, 512, 1},
    {"pk_pers_bc_b256_p30", golay_read_exp_kernel<0, 1, 0, 5, 0, 0, 256, true, 30>, 0, 1, 256, 1},
    // no LDS tile (golay_read_direct_kernel)
    {"direct_pers_b256_p30", golay_read_direct_kernel<0, 0, 256, 30>, 0, 1, 256, 0},
    {"direct_pers_b512_p30", golay_read_direct_kernel<0, 0, 512, 30>, 0, 1, 512, 0},
    {"direct_full_b512", golay_read_direct_kernel<1, 0, 512>, 1, 1, 512, 0},
    {"direct_full_bc_b512", golay_read_direct_kernel<1, 1, 512>, 1, 1, 512, 1},
    {"direct_full_bc_b256", golay_read_direct_kernel<1, 1, 256>, 1, 1, 256, 1},
    {"direct_pers_bc_b256_p30", golay_read_direct_kernel<0, 1, 256, 30>, 0, 1, 256, 1},
    {"direct_full_bc_dma_b512", golay_read_direct_kernel<1, 1, 512, 30, 1>, 1, 1, 512, 1},
    {"direct_full_bc_dma_b256", golay_read_direct_kernel<1, 1, 256, 30, 1>, 1, 1, 256, 1},
    {"direct_full_bc_dma_b1024", golay_read_direct_kernel<1, 1, 1024, 30, 1>, 1, 1, 1024, 1},
    {"direct_full_dma_b512", golay_read_direct_kernel<1, 0, 512, 30, 1>, 1, 1, 512, 0},
    // load-pattern probes (no decode)
    {"probe_aligned_b256", golay_read_probe_kernel<0, 256>, 1, 1, 256},
    {"probe_rows_b256", golay_read_probe_kernel<1, 256>, 1, 1, 256},
    {"probe_direct_b256", golay_read_probe_kernel<2, 256>, 1, 1, 256},
    {"probe_aligned_b512", golay_read_probe_kernel<0, 512>, 1, 1, 512},
    {"probe_rows_b512", golay_read_probe_kernel<1, 512>, 1, 1, 512},
    {"probe_direct_b512", golay_read_probe_kernel<2, 512>, 1, 1, 512},
    {"pk_probe_aligned_b256", golay_read_probe_kernel<0, 256>, 1, 1, 256},
    {"pk_probe_aligned_b512", golay_read_probe_kernel<0, 512>, 1, 1, 512},
    {"pf2", golay_read_pf2_kernel<512, false, 65>, 0, 1, 512},
    {"pf2_b256", golay_read_pf2_kernel<256, false, 65>, 0, 1, 256},
    {"pf2_p50", golay_read_pf2_kernel<512, false, 50>, 0, 1, 512},
    {"pk_pf2", golay_read_pf2_kernel<512, true, 65>, 0, 1, 512},
};

}  // namespace exp
}  // namespace kvecc

extern "C" {

__attribute__((visibility("default"))) int kvecc_exp_gread_count(void) {
  return (int)(sizeof(kvecc::exp::kVariants) / sizeof(kvecc::exp::kVariants[0]));
}

__attribute__((visibility("default"))) const char *kvecc_exp_gread_name(int v) {
  return kvecc::exp::kVariants[v].name;
}

// the fused Golay read of shim_read_batch (fp16 out, statistics on) through
// variant v; per_cu: persistent workgroups per CU; lds_pad: dynamic LDS bytes
__attribute__((visibility("default"))) int kvecc_exp_gread(int v, const void *k_cache, const void *v_cache,
                                                          const float *k_scales, const float *v_scales,
                                                          const int32_t *table, int64_t tstride, int64_t batch,
                                                          int64_t ctx, int64_t hkv, int64_t d, int64_t block_size,
                                                          int packed, void *k_out, void *v_out, uint64_t *stats,
                                                          int per_cu, int lds_pad, void *stream) {
  using namespace kvecc;
  const exp::Variant &var = exp::kVariants[v];
  ShimTileArgs a{};
  a.cache[0] = k_cache;
  a.cache[1] = v_cache;
  a.scales[0] = k_scales;
  a.scales[1] = v_scales;
  a.out[0] = k_out;
  a.out[1] = v_out;
  a.table = table;
  a.atab = golay_attn_table_dev();
  a.stats = stats;
  const int64_t g = (d + 2) / 3, gpr = cdiv(g, 4), lr = 12 * gpr;
  a.tstride = (uint32_t)tstride;
  a.hkv = (uint32_t)hkv;
  a.d = (uint32_t)d;
  a.g = (uint32_t)g;
  a.layers = 1;
  a.bs = (uint32_t)block_size;
  a.layer = 0;
  a.ctx = (uint32_t)ctx;
  a.gpr = (uint32_t)gpr;
  a.lr = (uint32_t)lr;
  a.tr = (uint32_t)std::min<int64_t>({block_size, (kTileStage - 16) / (lr + 8), (int64_t)kWave * kTileGroups / gpr,
                                      (int64_t)kWave, (int64_t)kWave * kTileChunks / (d / 8)});
  a.tpb = (uint32_t)cdiv(block_size, a.tr);
  a.nlb = (uint32_t)cdiv(ctx, block_size);
  a.units = (uint32_t)(2 * batch * hkv * a.nlb * a.tpb);
  a.rowb = (uint32_t)(packed ? KVECC_GOLAY_PACKED_ROW(g) : 4 * g);
  a.dyn = shim_dyn_slot(stream);
  const int kw = var.block / kWave;
  unsigned grid;
  if (var.sched == 0)
    grid = (unsigned)std::min<int64_t>(cdiv(a.units, kw), (int64_t)cu_count() * per_cu);
  else
    grid = (unsigned)cdiv(cdiv(a.units, var.chunk), kw);
  const uint16_t *t0 = golay_parity_table_dev();
  if (var.bc) {
    t0 = reinterpret_cast<const uint16_t *>(exp::bc_tables_dev());
    if (!t0) return set_error(KVECC_EHIP, "exp_gread: byte-class tables");
  }
  KVECC_LAUNCH(var.kern, dim3(grid), dim3(var.block), (unsigned)lds_pad, as_stream(stream), a, t0,
               golay_correct_table_dev());
  return check_launch("exp_gread");
}

}  // extern "C"

// the product's fused Golay read (persistent grid, its launch shape) with fixed
// phase-1 / phase-2 item counts (ng, nc rounds per lane): no per-item exit test
extern "C" __attribute__((visibility("default"))) int kvecc_exp_gread_fixed(
    int ng, int nc, const void *k_cache, const void *v_cache, const float *k_scales, const float *v_scales,
    const int32_t *table, int64_t tstride, int64_t batch, int64_t ctx, int64_t hkv, int64_t d, int64_t block_size,
    int packed, void *k_out, void *v_out, uint64_t *stats, void *stream) {
  using namespace kvecc;
  ShimTileArgs a{};
  a.cache[0] = k_cache;
  a.cache[1] = v_cache;
  a.scales[0] = k_scales;
  a.scales[1] = v_scales;
  a.out[0] = k_out;
  a.out[1] = v_out;
  a.table = table;
  a.atab = golay_attn_table_dev();
  a.stats = stats;
  const int64_t g = (d + 2) / 3, gpr = cdiv(g, 4), lr = 12 * gpr;
  a.tstride = (uint32_t)tstride;
  a.hkv = (uint32_t)hkv;
  a.d = (uint32_t)d;
  a.g = (uint32_t)g;
  a.layers = 1;
  a.bs = (uint32_t)block_size;
  a.layer = 0;
  a.ctx = (uint32_t)ctx;
  a.gpr = (uint32_t)gpr;
  a.lr = (uint32_t)lr;
  a.tr = (uint32_t)std::min<int64_t>({block_size, kTileStage / lr, (int64_t)kWave * kTileGroups / gpr,
                                      (int64_t)kWave, (int64_t)kWave * kTileChunks / (d / 8)});
  a.tpb = (uint32_t)cdiv(block_size, a.tr);
  a.nlb = (uint32_t)cdiv(ctx, block_size);
  a.units = (uint32_t)(2 * batch * hkv * a.nlb * a.tpb);
  a.rowb = (uint32_t)(packed ? KVECC_GOLAY_PACKED_ROW(g) : 4 * g);
  a.dyn = shim_dyn_slot(stream);
  if ((int64_t)cdiv(a.tr * a.gpr, kWave) != ng || (int64_t)a.tr * (d / 8) != (int64_t)nc * kWave)
    return set_error(KVECC_EINVAL, "fixed counts %d / %d do not match the tile", ng, nc);
  const unsigned grid = tile_grid(a.units);
  hipStream_t st = as_stream(stream);
  if (ng == 3 && nc == 4 && !packed)
    KVECC_LAUNCH((shim_read_golay_tiles_kernel<__half, true, false, 3, 4>), dim3(grid), dim3(kGolayTileBlock), 0, st, a);
  else if (ng == 3 && nc == 4 && packed)
    KVECC_LAUNCH((shim_read_golay_tiles_kernel<__half, true, true, 3, 4>), dim3(grid), dim3(kGolayTileBlock), 0, st, a);
  else
    return set_error(KVECC_EINVAL, "no instance for %d / %d", ng, nc);
  return check_launch("exp_gread_fixed");
}
