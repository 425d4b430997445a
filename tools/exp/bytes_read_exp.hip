// bytes_read_exp.hip -- experimental variants of the fused Hamming(8,4) read
// (csrc/shim.hip shim_read_bytes_tiles_kernel), NOT shipped: this file
// #includes shim.hip for its tile helpers; tools/exp/run_bytes_read_exp.py
// times them against the product (kvecc_shim_read_batch) in one process.
//
// (Round 4 also ran the product's tile kernel of the time at other work
// distributions -- full grids of 1-8 tiles per wave, persistent grids of 2-3
// workgroups per CU: profiles/r04/fused/bytes_read_grid_ab.log.)
//
// kvecc_exp_bytes_read_ipwg: the interpolating read on a full grid, neighbour
// rows exchanged between the waves of a workgroup (bytes_read_ipwg_kernel).
//
// kvecc_exp_bytes_read_ip: round 3's interpolating read (fp16 out, statistics
// on, persistent grid + dynamic tail, each tile prefetching its two neighbour
// rows from memory) -- "ip" is that product kernel -- rewritten with
//   TBL3   the tile's block-table entry and its two neighbour rows' entries
//          loaded together (one scalar round trip before the tile's loads
//          issue; the product waits for the tile's entry, issues the tile,
//          then waits again for the neighbours')
//   HBUF   the neighbour rows by two buffer loads (uniform descriptors) instead
//          of a 64-bit-addressed global load
//   WPE    amdgpu_waves_per_eu minimum (register budget; 1 = none)
//   DC     the head size as a compile-time constant (0: runtime, the product)
//   ORDER  1: tiles heads fastest (golay_read_exp.hip tile_at)
//   MG     phase-2 (row, chunk) by a reciprocal multiply (bytes_ladder_kernel INC)
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/shim.hip"

namespace kvecc {
namespace exp {

template <bool TBL3, bool HBUF, int WPE, int DC = 0, int ORDER = 0, bool MG = false>
__global__ __launch_bounds__(kTileBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void bytes_read_ip_kernel(
    ShimTileArgs a) {
  using TO = __half;
  const uint32_t kd = DC ? (uint32_t)DC : a.d;  // DC: the head size as a compile-time constant
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kTileWaves][kTileStage];
  __shared__ float scale_all[kTileWaves][kWave];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  uint8_t *stage = stage_all[wave];
  const uint32_t nwaves = gridDim.x * kTileWaves;
  const uint32_t cpr = kd / 16;
  const uint32_t items = a.tr * cpr;
  uint32_t ir[kByteTileItems], ic[kByteTileItems];
  constexpr int V = kVpl<TO>, NI2 = kByteTileItems * 16 / V;
  uint32_t i2r[NI2], i2c[NI2];
#pragma unroll
  for (int i = 0; i < kByteTileItems; ++i) {
    const uint32_t f = lane + kWave * i;
    ir[i] = f / cpr;
    ic[i] = f - ir[i] * cpr;
  }
#pragma unroll
  for (int i = 0; i < NI2; ++i) {
    const uint32_t f = lane + kWave * i;
    i2r[i] = f / (cpr * 16 / V);
    i2c[i] = f - i2r[i] * (cpr * 16 / V);
  }
  const uint32_t per2 = cpr * 16 / V;
  const uint32_t mg = uni((65536u + per2 - 1) / per2);
  uint32_t n1 = 0, n2 = 0;
  const uint32_t gw = blockIdx.x * kTileWaves + wave;
  uint32_t u = gw;
  if (u >= a.units) return;
  TileSchedule sched;
  sched.init(a.units, a.dyn, gw, nwaves, lane, kShimReadStaticPct);

  ShimTile cur;
  u32x4 w[kByteTileItems], hw = u32x4{0u, 0u, 0u, 0u};
  float scale;
  bool has_hw = false;
  auto fetch = [&](uint32_t uu) {
    // the tile (shim_tile) and its neighbour rows' positions
    const uint32_t per_side = a.units / 2;
    const uint32_t side = uu >= per_side ? 1u : 0u;
    uint32_t v = uu - side * per_side;
    uint32_t ch, lb, bh, b, h;
    if (ORDER == 0) {
      ch = v % a.tpb;
      v /= a.tpb;
      lb = v % a.nlb;
      bh = v / a.nlb;
      b = bh / a.hkv;
      h = bh - b * a.hkv;
    } else {  // heads fastest
      h = v % a.hkv;
      v /= a.hkv;
      ch = v % a.tpb;
      v /= a.tpb;
      lb = v % a.nlb;
      b = v / a.nlb;
      bh = b * a.hkv + h;
    }
    cur.side = side;
    cur.bh = bh;
    cur.pos0 = lb * a.bs + ch * a.tr;
    cur.rows = cur.pos0 < a.ctx ? min(min(a.tr, a.bs - ch * a.tr), a.ctx - cur.pos0) : 0u;
    const uint32_t pa = cur.pos0 > 0 ? cur.pos0 - 1 : 0u, pb = min(cur.pos0 + cur.rows, a.ctx - 1);
    const int32_t *trow = a.table + (int64_t)b * a.tstride;
    int32_t blk, ba = -1, bb = -1;
    if (TBL3) {
      blk = ld_scalar(trow + lb);
      ba = ld_scalar(trow + pa / a.bs);
      bb = ld_scalar(trow + pb / a.bs);
    } else {
      blk = ld_scalar(trow + lb);
    }
    cur.row0 = blk < 0 ? -1 : (((int64_t)blk * a.layers + a.layer) * a.hkv + h) * a.bs + ch * a.tr;
    const bool live = cur.row0 >= 0;
    const char *base = uni(reinterpret_cast<const char *>(a.cache[side]) + (live ? cur.row0 : 0) * (int64_t)kd);
    const char *sbase = uni(reinterpret_cast<const char *>(a.scales[side] + (live ? cur.row0 : 0)));
    const uint32_t nrows = uni(live ? cur.rows : 0u);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), 0, (int)(nrows * kd), 0x00020000);
    const __amdgpu_buffer_rsrc_t ss =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(sbase), 0, (int)(4 * nrows), 0x00020000);
    scale = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ss, 4 * lane, 0, 0));
#pragma unroll
    for (int i = 0; i < kByteTileItems; ++i) {
      if (i * kWave >= (int)items) break;
      w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ir[i] * kd + 16 * ic[i], 0, 2));
    }
    has_hw = cur.rows > 0;
    if (!has_hw) return;
    if (!TBL3) {
      ba = ld_scalar(trow + pa / a.bs);
      bb = ld_scalar(trow + pb / a.bs);
    }
    const int64_t rowa = (((int64_t)ba * a.layers + a.layer) * a.hkv + h) * a.bs + (pa - pa / a.bs * a.bs);
    const int64_t rowb = (((int64_t)bb * a.layers + a.layer) * a.hkv + h) * a.bs + (pb - pb / a.bs * a.bs);
    const bool below = lane >= cpr;
    if (HBUF) {
      const char *c = reinterpret_cast<const char *>(a.cache[side]);
      const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char *>(uni(c + (ba >= 0 ? rowa : 0) * (int64_t)kd)), 0, ba >= 0 ? (int)kd : 0, 0x00020000);
      const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char *>(uni(c + (bb >= 0 ? rowb : 0) * (int64_t)kd)), 0, bb >= 0 ? (int)kd : 0, 0x00020000);
      hw = u32x4{0u, 0u, 0u, 0u};
      if (!below)
        hw = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, 16 * lane, 0, 2));
      else if (lane < 2 * cpr)
        hw = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, 16 * (lane - cpr), 0, 2));
    } else {
      const int32_t bl = below ? bb : ba;
      hw = u32x4{0u, 0u, 0u, 0u};
      if (lane < 2 * cpr && bl >= 0)
        hw = ld_stream(reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(a.cache[side]) +
                                                       (below ? rowb : rowa) * kd) +
                       (below ? lane - cpr : lane));
    }
  };
  auto dec = [&](uint32_t cw, bool count, uint32_t &dbl) -> uint32_t {
    uint32_t q = cw, t = 0, s1 = 0, s2 = 0;
    h84_decode4(cw, q, t, s1, s2);
    if (count) {
      n1 += s1;
      n2 += s2;
      dbl |= s2;
    }
    return q | t << 4;
  };
  fetch(u);
  for (;;) {
    const uint32_t off0 = kd;
    scale_all[wave][lane] = scale;
    bool dbl_any = false;
#pragma unroll
    for (int i = 0; i < kByteTileItems; ++i) {
      if (i * kWave >= (int)items) break;
      const bool real = ir[i] < cur.rows;
      uint32_t dbl = 0;
      const u32x4 d4{dec(w[i].x, real, dbl), dec(w[i].y, real, dbl), dec(w[i].z, real, dbl),
                     dec(w[i].w, real, dbl)};
      dbl_any |= dbl != 0;
      if (ir[i] < cur.rows) *reinterpret_cast<u32x4 *>(stage + off0 + ir[i] * kd + 16 * ic[i]) = d4;
    }
    const bool tile_dbl = __builtin_amdgcn_ballot_w64(dbl_any) != 0;
    if (has_hw && lane < 2 * cpr) {
      uint32_t none = 0;
      const u32x4 d4{dec(hw.x, false, none), dec(hw.y, false, none), dec(hw.z, false, none),
                     dec(hw.w, false, none)};
      const uint32_t r = lane >= cpr ? cur.rows + 1 : 0u;
      *reinterpret_cast<u32x4 *>(stage + r * kd + 16 * (lane >= cpr ? lane - cpr : lane)) = d4;
    }
    wave_lds_sync();
    const ShimTile t = cur;
    u = sched.next(u, lane);
    const bool more = u < a.units;
    if (more) fetch(u);
    const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
    const bool dead = t.row0 < 0;
    auto phase2 = [&](auto interp_c) {
      constexpr bool IP = decltype(interp_c)::value;
#pragma unroll
      for (int i = 0; i < NI2; ++i) {
        if (i * kWave >= (int)(items * 16 / V)) break;
        // MG: (row, chunk) by a reciprocal multiply (see bytes_ladder_kernel INC)
        const uint32_t f = lane + kWave * i;
        const uint32_t fq = __umul24(f, mg) >> 16;
        const uint32_t rr = MG ? fq : i2r[i], c = MG ? f - fq * per2 : i2c[i];
        const uint32_t r = min(rr, a.tr - 1);
        const uint8_t *row = stage + off0 + r * kd + V * c;
        uint32_t q[2] = {0u, 0u};
#pragma unroll
        for (int k = 0; k < V / 4; ++k) {
          const uint32_t v = reinterpret_cast<const uint32_t *>(row)[k];
          if (IP) {
            const uint32_t up = reinterpret_cast<const uint32_t *>(row - kd)[k];
            const uint32_t dn = reinterpret_cast<const uint32_t *>(row + kd)[k];
            q[k] = interp_word(v & 0x0F0F0F0Fu, up & 0x0F0F0F0Fu, dn & 0x0F0F0F0Fu, (v >> 4) & 0x03030303u);
          } else {
            q[k] = v & 0x0F0F0F0Fu;
          }
        }
        tile_store(os, (rr * kd + V * c) * (uint32_t)sizeof(TO), dq16<TO>(q, scale_all[wave][r], dead));
      }
    };
    if (tile_dbl)
      phase2(std::integral_constant<bool, true>{});
    else
      phase2(std::integral_constant<bool, false>{});
    if (!more) break;
    wave_lds_sync();
  }
  n1 = wave_sum(n1);
  n2 = wave_sum(n2);
  if (lane == 0) {
    uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
    if (n1) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)n1);
    if (n2) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)n2);
  }
}

// Full grid, one tile per wave, neighbour rows exchanged inside the workgroup:
// its 8 waves hold 8 consecutive tiles of the static order (mostly 8 adjacent
// blocks of one sequence), so a tile's row above is the previous wave's last
// decoded row and its row below the next wave's first, read from their LDS
// stages after one workgroup barrier.  Only a tile that holds a double (~5 % at
// BER 1e-3) needs them at all; of those, only wave 0's row above and wave 7's
// row below come from memory (a synchronous load).  The clamps at the context's
// ends are the product's (the tile's own first / last row).
//   FLAGS false: one workgroup barrier after phase 1 (every wave waits for the
//   slowest); true: each wave clears its LDS word, one barrier at the start
//   (before any load: nothing in flight to wait for), then publishes "phase 1
//   done" in the word, and only a wave that needs a neighbour's row spins on
//   that neighbour's word
template <typename TO, bool STATS, bool FLAGS = false>
__global__ __launch_bounds__(kTileBlock) void bytes_read_ipwg_kernel(ShimTileArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kTileWaves][kTileStage];
  __shared__ float scale_all[kTileWaves][kWave];
  __shared__ uint32_t done[kTileWaves];
  constexpr uint32_t tag = 1;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  uint8_t *stage = stage_all[wave];
  const uint32_t cpr = a.d / 16;
  const uint32_t items = a.tr * cpr;
  uint32_t ir[kByteTileItems], ic[kByteTileItems];
  constexpr int V = kVpl<TO>, NI2 = kByteTileItems * 16 / V;
  uint32_t i2r[NI2], i2c[NI2];
#pragma unroll
  for (int i = 0; i < kByteTileItems; ++i) {
    const uint32_t f = lane + kWave * i;
    ir[i] = f / cpr;
    ic[i] = f - ir[i] * cpr;
  }
#pragma unroll
  for (int i = 0; i < NI2; ++i) {
    const uint32_t f = lane + kWave * i;
    i2r[i] = f / (cpr * 16 / V);
    i2c[i] = f - i2r[i] * (cpr * 16 / V);
  }
  uint32_t n1 = 0, n2 = 0;
  auto dec = [&](uint32_t cw, bool count, uint32_t &dbl) -> uint32_t {
    uint32_t q = cw, t = 0, s1 = 0, s2 = 0;
    h84_decode4(cw, q, t, s1, s2);
    if (count) {
      if (STATS) {
        n1 += s1;
        n2 += s2;
      }
      dbl |= s2;
    }
    return q | t << 4;
  };
  if (FLAGS) {  // LDS holds whatever the last workgroup left: clear before anyone looks
    if (lane == 0) *reinterpret_cast<volatile uint32_t *>(&done[wave]) = 0u;
    __syncthreads();
  }
  const uint32_t u = blockIdx.x * kTileWaves + wave;
  const bool active = u < a.units;  // every wave reaches the barrier
  ShimTile t;
  t.rows = 0;
  t.row0 = -1;
  t.pos0 = t.side = t.bh = 0;
  bool tile_dbl = false;
  const uint32_t off0 = a.d;  // tile row r at (r + 1) d; rows 0 and rows + 1: the neighbours
  if (active) {
    t = shim_tile(a, u);
    const bool live = t.row0 >= 0;
    const uint32_t side = uni(t.side);
    const char *base = uni(reinterpret_cast<const char *>(a.cache[side]) + (live ? t.row0 : 0) * (int64_t)a.d);
    const char *sbase = uni(reinterpret_cast<const char *>(a.scales[side] + (live ? t.row0 : 0)));
    const uint32_t nrows = uni(live ? t.rows : 0u);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), 0, (int)(nrows * a.d), 0x00020000);
    const __amdgpu_buffer_rsrc_t ss =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(sbase), 0, (int)(4 * nrows), 0x00020000);
    const float scale = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ss, 4 * lane, 0, 0));
    u32x4 w[kByteTileItems];
#pragma unroll
    for (int i = 0; i < kByteTileItems; ++i) {
      if (i * kWave >= (int)items) break;
      w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ir[i] * a.d + 16 * ic[i], 0, 2));
    }
    scale_all[wave][lane] = scale;
    bool dbl_any = false;
#pragma unroll
    for (int i = 0; i < kByteTileItems; ++i) {
      if (i * kWave >= (int)items) break;
      const bool real = ir[i] < t.rows;
      uint32_t dbl = 0;
      const u32x4 d4{dec(w[i].x, real, dbl), dec(w[i].y, real, dbl), dec(w[i].z, real, dbl),
                     dec(w[i].w, real, dbl)};
      dbl_any |= dbl != 0;
      if (real) *reinterpret_cast<u32x4 *>(stage + off0 + ir[i] * a.d + 16 * ic[i]) = d4;
    }
    tile_dbl = __builtin_amdgcn_ballot_w64(dbl_any) != 0;
  }
  if (FLAGS) {
    wave_lds_sync();  // this wave's decoded rows are in LDS
    if (lane == 0) *reinterpret_cast<volatile uint32_t *>(&done[wave]) = tag;
  } else {
    __syncthreads();  // every wave's decoded rows are in LDS
  }
  if (active && t.rows > 0) {
    if (tile_dbl) {  // wave-uniform: the neighbour rows into stage rows 0 and rows + 1
      const bool top_clamp = t.pos0 == 0, bot_clamp = t.pos0 + t.rows >= a.ctx;
      const bool ext_a = !top_clamp && wave == 0;                // row above in the previous workgroup
      const bool ext_b = !bot_clamp && wave == kTileWaves - 1;   // row below in the next one
      const bool below = lane >= cpr;
      const uint32_t l = below ? lane - cpr : lane;
      u32x4 hw{0u, 0u, 0u, 0u};
      if (ext_a || ext_b) {  // one side at most (kTileWaves > 1)
        const uint32_t bh = uni(t.bh), b = bh / a.hkv, h = bh - b * a.hkv;
        const uint32_t pos = uni(ext_a ? t.pos0 - 1 : t.pos0 + t.rows);
        const int32_t blk = ld_scalar(a.table + (int64_t)b * a.tstride + pos / a.bs);
        if (blk >= 0 && l < cpr && below == ext_b) {
          const int64_t row = (((int64_t)blk * a.layers + a.layer) * a.hkv + h) * a.bs + (pos - pos / a.bs * a.bs);
          hw = ld_stream(reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(a.cache[uni(t.side)]) +
                                                         row * a.d) + l);
        }
        uint32_t none = 0;
        hw = u32x4{dec(hw.x, false, none), dec(hw.y, false, none), dec(hw.z, false, none), dec(hw.w, false, none)};
      }
      if (FLAGS) {  // wait for the neighbours whose rows this tile reads (uniform)
        const bool need_a = !top_clamp && !ext_a, need_b = !bot_clamp && !ext_b;
        if (need_a)
          while (*reinterpret_cast<volatile uint32_t *>(&done[wave - 1]) != tag) __builtin_amdgcn_s_sleep(1);
        if (need_b)
          while (*reinterpret_cast<volatile uint32_t *>(&done[wave + 1]) != tag) __builtin_amdgcn_s_sleep(1);
      }
      if (lane < 2 * cpr) {
        u32x4 v = hw;
        if (below ? !ext_b : !ext_a) {
          const uint8_t *src = below ? (bot_clamp ? stage + t.rows * a.d : stage_all[wave + 1] + off0)
                                     : (top_clamp ? stage + off0 : stage_all[wave - 1] + a.tr * a.d);
          v = reinterpret_cast<const u32x4 *>(src)[l];
        }
        *reinterpret_cast<u32x4 *>(stage + (below ? t.rows + 1 : 0u) * a.d + 16 * l) = v;
      }
      wave_lds_sync();
    }
    const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
    const bool dead = t.row0 < 0;
    auto phase2 = [&](auto interp_c) {
      constexpr bool IP = decltype(interp_c)::value;
#pragma unroll
      for (int i = 0; i < NI2; ++i) {
        if (i * kWave >= (int)(items * 16 / V)) break;
        const uint32_t r = min(i2r[i], a.tr - 1), c = i2c[i];
        const uint8_t *row = stage + off0 + r * a.d + V * c;
        uint32_t q[2] = {0u, 0u};
#pragma unroll
        for (int k = 0; k < V / 4; ++k) {
          const uint32_t v = reinterpret_cast<const uint32_t *>(row)[k];
          if (IP) {
            const uint32_t up = reinterpret_cast<const uint32_t *>(row - a.d)[k];
            const uint32_t dn = reinterpret_cast<const uint32_t *>(row + a.d)[k];
            q[k] = interp_word(v & 0x0F0F0F0Fu, up & 0x0F0F0F0Fu, dn & 0x0F0F0F0Fu, (v >> 4) & 0x03030303u);
          } else {
            q[k] = v & 0x0F0F0F0Fu;
          }
        }
        tile_store(os, (i2r[i] * a.d + V * c) * (uint32_t)sizeof(TO), dq16<TO>(q, scale_all[wave][r], dead));
      }
    };
    if (tile_dbl)
      phase2(std::integral_constant<bool, true>{});
    else
      phase2(std::integral_constant<bool, false>{});
  }
  if (STATS) {
    n1 = wave_sum(n1);
    n2 = wave_sum(n2);
    if (lane == 0) {
      uint64_t *slot = a.stats + ((blockIdx.x * kTileWaves + wave) % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
      if (n1) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)n1);
      if (n2) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)n2);
    }
  }
}

// The ladder from the plain read to the workgroup-exchange interpolating read,
// one feature per level (BER 0: every level computes the right values; above
// it only level 6 interpolates correctly):
//   0 the plain H(8,4) read (full grid, one tile per wave)
//   1 + error types stored with the data and the double-error ballot
//   2 + the tile staged one row down (rows 0 / rows + 1 kept for neighbours)
//   3 + the interpolating phase-2 body, chosen per tile by the ballot
//   4 + rows past the tile masked in phase 1 (statistics and LDS stores)
//   5 + the start barrier and the per-wave "decoded" words (LDS, plain stores)
//   6 + the neighbour-row exchange (the full kernel)
//   7 levels 0-4, then a tile holding a double loads both neighbour rows from
//     memory (synchronously; no barrier, no words, no exchange)
//   8 levels 0-4, every tile's two neighbour rows issued with its own loads
//     (asynchronous; decoded only by a tile holding a double)
//   INC: phase 2 derives each item's (row, chunk) by a reciprocal multiply
//   (one 24-bit multiply and a shift) instead of holding a divided (row,
//   chunk) per item -- which the compiler, short of registers once the
//   interpolating body exists, re-derived by integer division after phase 1
//   (~135 instructions on every wave's critical path)
template <int LV, bool INC = false>
__global__ __launch_bounds__(kTileBlock) void bytes_ladder_kernel(ShimTileArgs a) {
  using TO = __half;
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kTileWaves][kTileStage];
  __shared__ float scale_all[kTileWaves][kWave];
  __shared__ uint32_t decoded[kTileWaves];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  if (LV == 5 || LV == 6) {
    if (lane == 0) decoded[wave] = 0u;
    __syncthreads();
  }
  uint8_t *stage = stage_all[wave];
  const uint32_t cpr = a.d / 16;
  const uint32_t items = a.tr * cpr;
  uint32_t ir[kByteTileItems], ic[kByteTileItems];
  constexpr int V = kVpl<TO>, NI2 = kByteTileItems * 16 / V;
  uint32_t i2r[NI2], i2c[NI2];
#pragma unroll
  for (int i = 0; i < kByteTileItems; ++i) {
    const uint32_t f = lane + kWave * i;
    ir[i] = f / cpr;
    ic[i] = f - ir[i] * cpr;
  }
#pragma unroll
  for (int i = 0; i < NI2; ++i) {
    const uint32_t f = lane + kWave * i;
    i2r[i] = f / (cpr * 16 / V);
    i2c[i] = f - i2r[i] * (cpr * 16 / V);
  }
  uint32_t n1 = 0, n2 = 0;
  const uint32_t gw = blockIdx.x * kTileWaves + wave;
  if ((LV < 5 || LV >= 7) && gw >= a.units) return;
  const bool active = gw < a.units;
  ShimTile t;
  t.rows = 0;
  t.row0 = -1;
  t.pos0 = t.side = t.bh = 0;
  bool tile_dbl = false;
  const uint32_t off0 = LV >= 2 ? a.d : 0u;
  if (active) {
    t = shim_tile(a, gw);
    const bool live = t.row0 >= 0;
    const uint32_t side = uni(t.side);
    const char *base = uni(reinterpret_cast<const char *>(a.cache[side]) + (live ? t.row0 : 0) * (int64_t)a.d);
    const char *sbase = uni(reinterpret_cast<const char *>(a.scales[side] + (live ? t.row0 : 0)));
    const uint32_t nrows = uni(live ? t.rows : 0u);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), 0, (int)(nrows * a.d), 0x00020000);
    const __amdgpu_buffer_rsrc_t ss =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(sbase), 0, (int)(4 * nrows), 0x00020000);
    const float scale = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ss, 4 * lane, 0, 0));
    u32x4 w[kByteTileItems];
#pragma unroll
    for (int i = 0; i < kByteTileItems; ++i) {
      if (i * kWave >= (int)items) break;
      w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ir[i] * a.d + 16 * ic[i], 0, 2));
    }
    // level 8: the two neighbour rows issued with the tile's loads (as round 3's
    // persistent kernel prefetched them), decoded only if the tile needs them
    u32x4 hw8{0u, 0u, 0u, 0u};
    if (LV == 8 && t.rows > 0) {
      const bool top_clamp = t.pos0 == 0, bot_clamp = t.pos0 + t.rows >= a.ctx;
      const bool below = lane >= cpr;
      const uint32_t l = below ? lane - cpr : lane;
      const uint32_t bh = uni(t.bh), b = bh / a.hkv, h = bh - b * a.hkv;
      const uint32_t pa = uni(top_clamp ? 0u : t.pos0 - 1), pb = uni(bot_clamp ? 0u : t.pos0 + t.rows);
      const int32_t ba = top_clamp ? -1 : ld_scalar(a.table + (int64_t)b * a.tstride + pa / a.bs);
      const int32_t bb = bot_clamp ? -1 : ld_scalar(a.table + (int64_t)b * a.tstride + pb / a.bs);
      const uint32_t pos = below ? pb : pa;
      const int32_t blk = below ? bb : ba;
      if (blk >= 0 && l < cpr && lane < 2 * cpr) {
        const int64_t row = (((int64_t)blk * a.layers + a.layer) * a.hkv + h) * a.bs + (pos - pos / a.bs * a.bs);
        hw8 = ld_stream(reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(a.cache[side]) +
                                                        row * a.d) + l);
      }
    }
    scale_all[wave][lane] = scale;
    bool dbl_any = false;
    auto dec = [&](uint32_t cw, bool count, uint32_t &dbl) -> uint32_t {
      uint32_t q = cw, tt = 0, s1 = 0, s2 = 0;
      h84_decode4(cw, q, tt, s1, s2);
      if (count) {
        n1 += s1;
        n2 += s2;
        dbl |= s2;
      }
      return LV >= 1 ? q | tt << 4 : q;
    };
#pragma unroll
    for (int i = 0; i < kByteTileItems; ++i) {
      if (i * kWave >= (int)items) break;
      const bool real = LV >= 4 ? ir[i] < t.rows : true;
      uint32_t dbl = 0;
      const u32x4 d4{dec(w[i].x, real, dbl), dec(w[i].y, real, dbl), dec(w[i].z, real, dbl),
                     dec(w[i].w, real, dbl)};
      dbl_any |= dbl != 0;
      if (LV >= 4 ? real : ir[i] < a.tr) *reinterpret_cast<u32x4 *>(stage + off0 + ir[i] * a.d + 16 * ic[i]) = d4;
    }
    if (LV >= 1) tile_dbl = __builtin_amdgcn_ballot_w64(dbl_any) != 0;
    if (LV == 8 && tile_dbl) {  // neighbours: decoded (clamped: the tile's own first / last row)
      wave_lds_sync();
      if (lane < 2 * cpr) {
        const bool top_clamp = t.pos0 == 0, bot_clamp = t.pos0 + t.rows >= a.ctx;
        const bool below = lane >= cpr;
        const uint32_t l = below ? lane - cpr : lane;
        u32x4 v;
        if (below ? bot_clamp : top_clamp) {
          v = reinterpret_cast<const u32x4 *>(stage + off0 + (below ? t.rows - 1 : 0u) * a.d)[l];
        } else {
          uint32_t none = 0;
          v = u32x4{dec(hw8.x, false, none), dec(hw8.y, false, none), dec(hw8.z, false, none),
                    dec(hw8.w, false, none)};
        }
        *reinterpret_cast<u32x4 *>(stage + (below ? t.rows + 1 : 0u) * a.d + 16 * l) = v;
      }
    }
  }
  wave_lds_sync();
  if ((LV == 5 || LV == 6) && lane == 0)
    __hip_atomic_store(&decoded[wave], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (!active || t.rows == 0) return;
  if (LV >= 6 && tile_dbl) {
    const bool top_clamp = t.pos0 == 0, bot_clamp = t.pos0 + t.rows >= a.ctx;
    // level 7: both neighbour rows from memory, no exchange
    const bool ext_a = !top_clamp && (LV == 7 || wave == 0), ext_b = !bot_clamp && (LV == 7 || wave == kTileWaves - 1);
    if (LV == 6 && !top_clamp && !ext_a)
      while (__hip_atomic_load(&decoded[wave - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
        __builtin_amdgcn_s_sleep(1);
    if (LV == 6 && !bot_clamp && !ext_b)
      while (__hip_atomic_load(&decoded[wave + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
        __builtin_amdgcn_s_sleep(1);
    const bool below = lane >= cpr;
    const uint32_t l = below ? lane - cpr : lane;
    u32x4 hw{0u, 0u, 0u, 0u};
    if (ext_a || ext_b) {
      const uint32_t bh = uni(t.bh), b = bh / a.hkv, h = bh - b * a.hkv;
      const uint32_t pa = uni(ext_a ? t.pos0 - 1 : 0u), pb = uni(ext_b ? t.pos0 + t.rows : 0u);
      const int32_t ba = ext_a ? ld_scalar(a.table + (int64_t)b * a.tstride + pa / a.bs) : -1;
      const int32_t bb = ext_b ? ld_scalar(a.table + (int64_t)b * a.tstride + pb / a.bs) : -1;
      const uint32_t pos = below ? pb : pa;
      const int32_t blk = below ? bb : ba;
      if (blk >= 0 && l < cpr && (below ? ext_b : ext_a)) {
        const int64_t row = (((int64_t)blk * a.layers + a.layer) * a.hkv + h) * a.bs + (pos - pos / a.bs * a.bs);
        hw = ld_stream(reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(a.cache[uni(t.side)]) +
                                                       row * a.d) + l);
      }
      uint32_t q, tt, s1, s2;
      uint32_t *hv = reinterpret_cast<uint32_t *>(&hw);
      for (int k = 0; k < 4; ++k) {
        q = hv[k];
        h84_decode4(hv[k], q, tt, s1, s2);
        hv[k] = q | tt << 4;
      }
    }
    if (lane < 2 * cpr) {
      u32x4 v = hw;
      if (below ? !ext_b : !ext_a) {
        const uint8_t *src = below ? (bot_clamp ? stage + t.rows * a.d : stage_all[wave + 1] + off0)
                                   : (top_clamp ? stage + off0 : stage_all[wave - 1] + a.tr * a.d);
        v = reinterpret_cast<const u32x4 *>(src)[l];
      }
      *reinterpret_cast<u32x4 *>(stage + (below ? t.rows + 1 : 0u) * a.d + 16 * l) = v;
    }
    wave_lds_sync();
  }
  const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
  const bool dead = t.row0 < 0;
  const uint32_t per2 = cpr * 16 / V;  // V-value chunks per row (<= 64)
  // f / per2 for f < 2^9 as (f * m) >> 16, m = ceil(2^16 / per2): exact, as
  // f (m - 2^16 / per2) < 2^9 / 2^16 < 1 / per2
  const uint32_t m = uni((65536u + per2 - 1) / per2);
  auto phase2 = [&](auto interp_c) {
    constexpr bool IP = decltype(interp_c)::value;
#pragma unroll
    for (int i = 0; i < NI2; ++i) {
      if (i * kWave >= (int)(items * 16 / V)) break;
      const uint32_t f = lane + kWave * i;
      const uint32_t fq = __umul24(f, m) >> 16;
      const uint32_t rr = INC ? fq : i2r[i], c = INC ? f - fq * per2 : i2c[i];
      const uint32_t r = min(rr, a.tr - 1);
      const uint8_t *row = stage + off0 + r * a.d + V * c;
      uint32_t q[2] = {0u, 0u};
#pragma unroll
      for (int k = 0; k < V / 4; ++k) {
        const uint32_t v = reinterpret_cast<const uint32_t *>(row)[k];
        if (IP) {
          const uint32_t up = reinterpret_cast<const uint32_t *>(row - a.d)[k];
          const uint32_t dn = reinterpret_cast<const uint32_t *>(row + a.d)[k];
          q[k] = interp_word(v & 0x0F0F0F0Fu, up & 0x0F0F0F0Fu, dn & 0x0F0F0F0Fu, (v >> 4) & 0x03030303u);
        } else {
          q[k] = v & 0x0F0F0F0Fu;
        }
      }
      tile_store(os, (rr * a.d + V * c) * (uint32_t)sizeof(TO), dq16<TO>(q, scale_all[wave][r], dead));
    }
  };
  if (LV >= 3 && tile_dbl)
    phase2(std::integral_constant<bool, true>{});
  else
    phase2(std::integral_constant<bool, false>{});
  n1 = wave_sum(n1);
  n2 = wave_sum(n2);
  if (lane == 0) {
    uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
    if (n1) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)n1);
    if (n2) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)n2);
  }
}

struct IpVariant {
  const char *name;
  void (*kern)(ShimTileArgs);
};
static const IpVariant kIpVariants[] = {
    {"ip", bytes_read_ip_kernel<false, false, 1>},      {"ip_tbl3", bytes_read_ip_kernel<true, false, 1>},
    {"ip_hbuf", bytes_read_ip_kernel<false, true, 1>},  {"ip_tbl3_hbuf", bytes_read_ip_kernel<true, true, 1>},
    {"ip_w6", bytes_read_ip_kernel<false, false, 6>},   {"ip_tbl3_hbuf_w6", bytes_read_ip_kernel<true, true, 6>},
    {"ip_d128", bytes_read_ip_kernel<false, false, 1, 128>},
    {"ip_tbl3_d128", bytes_read_ip_kernel<true, false, 1, 128>},
    {"ip_tbl3_hbuf_d128", bytes_read_ip_kernel<true, true, 1, 128>},
    {"ip_tbl3_d128_w6", bytes_read_ip_kernel<true, false, 6, 128>},
    {"ip_mg", bytes_read_ip_kernel<false, false, 1, 0, 0, true>},
    {"ip_tbl3_mg", bytes_read_ip_kernel<true, false, 1, 0, 0, true>},
    {"ip_hm", bytes_read_ip_kernel<false, false, 1, 0, 1>},
    {"ip_tbl3_hm", bytes_read_ip_kernel<true, false, 1, 0, 1>},
};

static ShimTileArgs bytes_args(int interp, const void *k_cache, const void *v_cache, const float *k_scales,
                               const float *v_scales, const int32_t *table, int64_t tstride, int64_t batch,
                               int64_t ctx, int64_t hkv, int64_t d, int64_t block_size, void *k_out, void *v_out,
                               uint64_t *stats, void *stream) {
  ShimTileArgs a{};
  a.cache[0] = k_cache;
  a.cache[1] = v_cache;
  a.scales[0] = k_scales;
  a.scales[1] = v_scales;
  a.out[0] = k_out;
  a.out[1] = v_out;
  a.table = table;
  a.stats = stats;
  a.tstride = (uint32_t)tstride;
  a.hkv = (uint32_t)hkv;
  a.d = a.g = a.lr = a.rowb = (uint32_t)d;
  a.layers = 1;
  a.bs = (uint32_t)block_size;
  a.layer = 0;
  a.ctx = (uint32_t)ctx;
  const int64_t cpr = d / 16;
  a.tr = (uint32_t)std::min<int64_t>({block_size, (int64_t)kTileStage / d - (interp ? 2 : 0), (int64_t)kWave,
                                      (int64_t)kWave * kByteTileItems / cpr});
  a.tpb = (uint32_t)cdiv(block_size, a.tr);
  a.nlb = (uint32_t)cdiv(ctx, block_size);
  a.units = (uint32_t)(2 * batch * hkv * a.nlb * a.tpb);
  a.dyn = shim_dyn_slot(stream);
  return a;
}

}  // namespace exp
}  // namespace kvecc

#define EXP_API extern "C" __attribute__((visibility("default")))
#define BYTES_PARAMS                                                                                              \
  const void *k_cache, const void *v_cache, const float *k_scales, const float *v_scales, const int32_t *table, \
      int64_t tstride, int64_t batch, int64_t ctx, int64_t hkv, int64_t d, int64_t block_size, void *k_out,       \
      void *v_out, uint64_t *stats, void *stream

EXP_API int kvecc_exp_bytes_ip_count(void) {
  return (int)(sizeof(kvecc::exp::kIpVariants) / sizeof(kvecc::exp::kIpVariants[0]));
}
EXP_API const char *kvecc_exp_bytes_ip_name(int v) { return kvecc::exp::kIpVariants[v].name; }

EXP_API int kvecc_exp_bytes_read_ip(int v, int per_cu, BYTES_PARAMS) {
  using namespace kvecc;
  const ShimTileArgs a = exp::bytes_args(1, k_cache, v_cache, k_scales, v_scales, table, tstride, batch, ctx, hkv,
                                         d, block_size, k_out, v_out, stats, stream);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(a.units, kTileWaves), (int64_t)cu_count() * per_cu);
  KVECC_LAUNCH(exp::kIpVariants[v].kern, dim3(grid), dim3(kTileBlock), 0, as_stream(stream), a);
  return check_launch("exp_bytes_read_ip");
}

// the workgroup-exchange interpolating read (fp16, statistics), full grid;
// lds_pad bytes of dynamic LDS cap the workgroups per CU
EXP_API int kvecc_exp_bytes_read_ipwg(int lds_pad, BYTES_PARAMS) {
  using namespace kvecc;
  const ShimTileArgs a = exp::bytes_args(1, k_cache, v_cache, k_scales, v_scales, table, tstride, batch, ctx, hkv,
                                         d, block_size, k_out, v_out, stats, stream);
  const unsigned grid = (unsigned)cdiv(a.units, kTileWaves);
  // lds_pad bit 0: the flag form (pads are whole KiB)
  if (lds_pad & 1)
    KVECC_LAUNCH((exp::bytes_read_ipwg_kernel<__half, true, true>), dim3(grid), dim3(kTileBlock),
                 (unsigned)(lds_pad & ~1), as_stream(stream), a);
  else
    KVECC_LAUNCH((exp::bytes_read_ipwg_kernel<__half, true>), dim3(grid), dim3(kTileBlock), (unsigned)lds_pad,
                 as_stream(stream), a);
  return check_launch("exp_bytes_read_ipwg");
}

// the ladder (bytes_ladder_kernel<level>; level + 10: INC), full grid, 16 KiB dynamic LDS
EXP_API int kvecc_exp_bytes_ladder(int level, BYTES_PARAMS) {
  using namespace kvecc;
  const ShimTileArgs a = exp::bytes_args(1, k_cache, v_cache, k_scales, v_scales, table, tstride, batch, ctx, hkv,
                                         d, block_size, k_out, v_out, stats, stream);
  const unsigned grid = (unsigned)cdiv(a.units, kTileWaves);
  hipStream_t st = as_stream(stream);
  switch (level) {
#define LC(L) \
  case L: KVECC_LAUNCH((exp::bytes_ladder_kernel<L>), dim3(grid), dim3(kTileBlock), 16384u, st, a); break;   \
  case 10 + L: KVECC_LAUNCH((exp::bytes_ladder_kernel<L, true>), dim3(grid), dim3(kTileBlock), 16384u, st, a); break;
    LC(0) LC(1) LC(2) LC(3) LC(4) LC(5) LC(6) LC(7) LC(8)
#undef LC
    default: return set_error(KVECC_EINVAL, "ladder level");
  }
  return check_launch("exp_bytes_ladder");
}
