// shim.hip -- the ECC shim's KV-cache write and read as one launch each.
//
// Reference: kv_cache/ecc_shim.py.  Write (:557-721): per (batch, pos, head)
// row, quantize (absmax/7, torch round-half-even), encode, inject with the
// row's own seed (K: seed0 + r, V: seed0 + r + 1, r = the row's running index)
// and store into the paged cache; every batch writes the same seq_id slots, so
// only the last batch's rows survive (:626-637).  Read (:990-1071): gather the
// context's codewords, decode (stats += corrected / detected), optionally
// interpolate H(8,4) double errors along the context axis, dequantize
// ((q - 8) * scale) and hand K/V to attention.
//
// The reference runs these as Python loops issuing per-row Triton launches;
// here the write is one launch (a wave per surviving row of K or V, the row's
// absmax is a wave reduction, Golay triplets go through LDS) and the read is
// one launch (a lane per 4 codewords of a row, neighbours re-decoded for
// interpolation, output written head-major [Hkv, ctx, D] in the attention
// dtype so it feeds SDPA without a permute copy).
//
// Cache layout (SimpleBlockManager): codewords [blocks, layers, Hkv, bs, P]
// with P = D (uint8) or ceil(D/3) (int32 Golay); scales fp32 [blocks, layers,
// Hkv, bs]; logical block b of the sequence is physical block table[b].
#include <algorithm>
#include <type_traits>

#include "kvecc_internal.h"

namespace kvecc {

constexpr int kMaxShimD = 512;  // a lane holds <= 8 elements of a row
constexpr int kWavesPerBlock = kBlock / kWave;

struct ShimGeom {
  const int32_t *table;
  // 32-bit index math (the host checks every count fits): 64-bit division is
  // ~100 instructions on gfx950
  uint32_t hkv, d, g;  // g = codewords per token row: d, or ceil(d/3) for Golay
                       // (packed Golay rows are KVECC_GOLAY_PACKED_ROW(g) bytes)
  uint32_t layers, bs, layer;
  __device__ __forceinline__ int64_t slot(uint32_t pos, uint32_t h) const {
    const uint32_t lb = pos / bs;
    const int64_t blk = table[lb];
    return ((blk * layers + layer) * hkv + h) * bs + (pos - lb * bs);
  }
};

struct ShimWriteArgs {
  ShimGeom geo;
  const void *x[2];  // K, V: [batch, seq, hkv, d], each head's d values contiguous
  int64_t xb[2], xs[2], xh[2];  // element strides of the batch, seq and head dims
  void *cache[2];
  float *scales[2];
  int64_t batch, seq;
  uint32_t seed0, rowmul, nbits, thr;
  int nb_eff, inject, scale_rule;
};

// one wave per (side, pos, head) row of the last batch
template <typename T, int CODEC, int NB>
__global__ __launch_bounds__(kBlock) void shim_write_kernel(ShimWriteArgs a) {
  __shared__ uint8_t nib[kWavesPerBlock][kMaxShimD + 4];
  const ShimGeom &geo = a.geo;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const uint32_t per_side = (uint32_t)a.seq * geo.hkv;
  const uint32_t item = blockIdx.x * kWavesPerBlock + w;
  const bool live = item < 2 * per_side;
  const int side = live && item >= per_side ? 1 : 0;
  const uint32_t rr = live ? item - side * per_side : 0;
  const uint32_t pos = rr / geo.hkv, h = rr - pos * geo.hkv;
  const int64_t r = (a.batch - 1) * (int64_t)per_side + rr;  // running row index of the write
  const uint32_t key0 = (a.seed0 + (uint32_t)r + (uint32_t)side) * a.rowmul;
  const int64_t slot = live ? geo.slot(pos, h) : 0;

  constexpr int kPer = kMaxShimD / kWave;
  float v[kPer];
  float amax = 0.0f;
  if (live) {
    const T *x = reinterpret_cast<const T *>(a.x[side]) + (a.batch - 1) * a.xb[side] +
                 (int64_t)pos * a.xs[side] + (int64_t)h * a.xh[side];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t e = lane + i * kWave;
      v[i] = e < geo.d ? to_f32<T>(x[e]) : 0.0f;
      amax = fmaxf(amax, fabsf(v[i]));
    }
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, kWave));
  const float scale = row_scale(amax, a.scale_rule);
  if (live && lane == 0) a.scales[side][slot] = scale;
  // x / scale: reciprocal + FMA correction for 16-bit rows (codec_math.h div_recip)
  const bool recip = sizeof(T) == 2 && recip_ok(scale);
  const float inv = div_rn(1.0f, scale);
  auto quant = [&](float x) {
    return recip ? nibble_of_quotient(div_recip(x, scale, inv)) : quantize_nibble(x, scale);
  };

  constexpr bool kGolay = CODEC == KVECC_CODEC_GOLAY || CODEC == KVECC_CODEC_GOLAY_PACKED;
  if (!kGolay) {
    if (!live) return;
    uint8_t *c = reinterpret_cast<uint8_t *>(a.cache[side]) + slot * geo.g;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t e = lane + i * kWave;
      if (e < geo.d) {
        uint32_t cw = encode_nibble(quant(v[i]), CODEC);
        if (a.inject) cw ^= philox_flip_mask<NB>(key0 + e * a.nbits, e, a.thr, a.nb_eff);
        c[e] = (uint8_t)cw;
      }
    }
    return;
  }
  // Golay: the row's nibbles go through LDS, then one lane per codeword of 3
  if (live) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t e = lane + i * kWave;
      if (e < geo.d) nib[w][e] = (uint8_t)quant(v[i]);
    }
    if ((uint32_t)lane < 3 * geo.g - geo.d) nib[w][geo.d + lane] = 0;  // per-head zero padding
  }
  __syncthreads();
  if (!live) return;
  for (uint32_t k = lane; k < geo.g; k += kWave) {
    const uint32_t dw = golay_pack(nib[w][3 * k], nib[w][3 * k + 1], nib[w][3 * k + 2]);
    uint32_t cw = dw | golay_parity12(dw) << 12;
    if (a.inject)
      cw ^= philox_flip_mask<NB>(key0 + k * a.nbits, k, a.thr, a.nb_eff);
    if (CODEC == KVECC_CODEC_GOLAY_PACKED) {
      uint8_t *c = reinterpret_cast<uint8_t *>(a.cache[side]) + slot * KVECC_GOLAY_PACKED_ROW(geo.g) + 3 * k;
      c[0] = (uint8_t)cw;
      c[1] = (uint8_t)(cw >> 8);
      c[2] = (uint8_t)(cw >> 16);
    } else {
      reinterpret_cast<int32_t *>(a.cache[side])[slot * geo.g + k] = (int32_t)cw;
    }
  }
}

struct ShimReadArgs {
  ShimGeom geo;
  const void *cache[2];
  const float *scales[2];
  void *out[2];  // [hkv, ctx, d]
  uint32_t ctx;
  const uint16_t *par, *cor;  // Golay tables
  uint64_t *stats;
};

template <typename TO>
__device__ __forceinline__ void dequant4(TO *o, uint32_t q, float s) {
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = from_f32<TO>(dequant1(q >> (8 * k) & 0xFFu, s));
}

__device__ __forceinline__ uint32_t ld_word(const uint8_t *base, int64_t slot, uint32_t d, uint32_t c) {
  return *reinterpret_cast<const uint32_t *>(base + slot * d + 4 * c);
}

// codewords 4c..4c+3 of row `pos`, or 0 when its block is missing (table entry
// -1): the tile kernels' and the host twin's reading of a missing block
__device__ __forceinline__ uint32_t ld_word_or0(const ShimGeom &geo, const uint8_t *base, uint32_t pos, uint32_t h,
                                                uint32_t c) {
  if (geo.table[pos / geo.bs] < 0) return 0u;
  return ld_word(base, geo.slot(pos, h), geo.d, c);
}

// byte codecs (raw INT4, H(7,4), H(8,4)): one lane per 4 codewords (d % 4 == 0)
template <typename TO, int CODEC, bool INTERP, bool STATS>
__global__ __launch_bounds__(kBlock) void shim_read_bytes_kernel(ShimReadArgs a) {
  const ShimGeom &geo = a.geo;
  const uint32_t c4 = geo.d / 4;
  const uint32_t per_side = geo.hkv * a.ctx * c4;
  uint32_t n1 = 0, n2 = 0;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < 2 * per_side; i += gridDim.x * kBlock) {
    const int side = i >= per_side ? 1 : 0;
    const uint32_t t = i - side * per_side;
    const uint32_t hl = t / c4, c = t - hl * c4;
    const uint32_t h = hl / a.ctx, l = hl - h * a.ctx;
    const uint8_t *base = reinterpret_cast<const uint8_t *>(a.cache[side]);
    TO *o = reinterpret_cast<TO *>(a.out[side]) + ((int64_t)h * a.ctx + l) * geo.d + 4 * c;
    if (geo.table[l / geo.bs] < 0) {  // no physical block: +0, as the tile kernels
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = from_f32<TO>(0.0f);
      continue;
    }
    const int64_t slot = geo.slot(l, h);
    const uint32_t w = ld_word(base, slot, geo.d, c);
    uint32_t q = w, type;
    if (CODEC == KVECC_CODEC_H84) {
      h84_decode4(w, q, type, n1, n2);
      if (INTERP) {  // neighbours are the decoded (not interpolated) values; a missing one reads as 0
        const uint32_t lp = l > 0 ? l - 1 : 0, ln = l + 1 < a.ctx ? l + 1 : a.ctx - 1;
        uint32_t ql, qr, tt, u1 = 0, u2 = 0;
        h84_decode4(ld_word_or0(geo, base, lp, h, c), ql, tt, u1, u2);
        h84_decode4(ld_word_or0(geo, base, ln, h, c), qr, tt, u1, u2);
        q = interp_word(q, ql, qr, type);
      }
    } else if (CODEC == KVECC_CODEC_H74) {
      h74_decode4(w, q, type, n1);
    }
    dequant4(o, q, a.scales[side][slot]);
  }
  if (STATS) flush_stats2(a.stats, n1, n2);
}

// Golay: one lane per codeword of a token row (PACKED: 3-byte codewords)
template <typename TO, bool STATS, bool PACKED>
__global__ __launch_bounds__(kBlock) void shim_read_golay_kernel(ShimReadArgs a) {
  const ShimGeom &geo = a.geo;
  const uint32_t per_side = geo.hkv * a.ctx * geo.g;
  uint32_t bits = 0, unc = 0;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < 2 * per_side; i += gridDim.x * kBlock) {
    const int side = i >= per_side ? 1 : 0;
    const uint32_t t = i - side * per_side;
    const uint32_t hl = t / geo.g, k = t - hl * geo.g;
    const uint32_t h = hl / a.ctx, l = hl - h * a.ctx;
    TO *o = reinterpret_cast<TO *>(a.out[side]) + ((int64_t)h * a.ctx + l) * geo.d + 3 * k;
    const uint32_t left = geo.d - 3 * k;
    if (geo.table[l / geo.bs] < 0) {  // no physical block: zeros
      o[0] = from_f32<TO>(0.0f);
      if (left > 1) o[1] = from_f32<TO>(0.0f);
      if (left > 2) o[2] = from_f32<TO>(0.0f);
      continue;
    }
    const int64_t slot = geo.slot(l, h);
    uint32_t w;
    if (PACKED) {
      const uint8_t *c = reinterpret_cast<const uint8_t *>(a.cache[side]) +
                         slot * KVECC_GOLAY_PACKED_ROW(geo.g) + 3 * k;
      w = (uint32_t)c[0] | (uint32_t)c[1] << 8 | (uint32_t)c[2] << 16;
    } else {
      w = (uint32_t)reinterpret_cast<const int32_t *>(a.cache[side])[slot * geo.g + k];
    }
    uint32_t cnt;
    const uint32_t dw = golay_decode1(w, a.par, a.cor, cnt);
    bits += cnt & 3u;
    unc += cnt >> 2;
    const float s = a.scales[side][slot];
    o[0] = from_f32<TO>(dequant1(dw & 0xFu, s));
    if (left > 1) o[1] = from_f32<TO>(dequant1(dw >> 4 & 0xFu, s));
    if (left > 2) o[2] = from_f32<TO>(dequant1(dw >> 8, s));
  }
  if (STATS) flush_stats2(a.stats, bits, unc);
}

// ---- Golay read through wave tiles (the fused decode the headline names) -------
// A wave owns a tile: up to `tr` (<= 64) consecutive token rows of one (side,
// sequence, head, block) -- contiguous codewords in the cache, a contiguous run
// of the [hkv, ctx, d] output.  Phase 1: each lane takes groups of 4 codewords
// of a row (one 16-byte buffer load; packed: 12 bytes), decodes them through the
// spread tables in LDS (2 lookups + a v_bitop3 per codeword, nibbles one per
// byte, the error count in byte 3 of the correction entry) and writes 12
// nibble bytes to the wave's LDS tile (rows `lr` bytes apart).  Phase 2: each
// lane takes 8 consecutive values of a row (two LDS dwords), dequantizes
// (q - 8) * scale in fp32 and writes them with one non-temporal 16-byte store
// (fp16/bf16).  The next tile's codewords AND row scales (lane r holds row r's
// scale, handed to phase 2 by ds_bpermute) are loaded before phase 2, so no
// dependent global load sits inside a tile.  Every lane's (row, group) and
// (row, 8-value chunk) items are the same for every tile: computed once.  HBM
// traffic is the algorithm's: 4 B (3 B packed) per codeword in, d * sizeof(TO)
// per row out, 4 B of scale per row.
// Tuned constants of the wave-tile reads (A/B history: DESIGN.md §3, the
// experiment forks under tools/exp).  None of them changes a result.
//   * 512-thread workgroups, 2 per CU for the Golay kernel (LDS: 32 KiB of
//     tables + a 2.25 KiB tile per wave): beat 3 per CU (24 waves) and 256-thread
//     variants by 6-12 % (tools/exp/run_shim_read.py); r04 re-checked 256 x 3,
//     384 x 2, 768 x 1, 1024 x 1 (161-168 us vs 160.8, profiles/r04/fused/).
//   * non-temporal codeword loads and output stores (-5 %).
//   * the byte-codec read without interpolation runs the full grid, one tile
//     per wave, capped at 4 workgroups per CU by 16 KiB of dynamic LDS: H(8,4)
//     -> fp16 at [8,4096,32,128] 137.6-138.6 us against 147.2 persistent (8 per
//     CU 138.6, 2: 174.2, 1: 261.4); the interpolating read and the Golay read
//     keep the persistent grid with the dynamic tail (172.1 vs 158.9 full grid
//     for interpolation; Golay full grids 162-335 us, profiles/r04/fused/).
//   * dynamic tail: a wave takes the first 65 % of its even share of tiles
//     statically (w, w + nwaves, ...) and the rest from per-launch work
//     counters (TileSchedule, kvecc_internal.h), one atomic per tile issued a
//     tile ahead.  With equal static shares the waves of one launch finished
//     119-166 us apart (mean 143 us; memory latency is not even across the
//     chip), and handing tiles to whichever CU asks costs locality (a static
//     order with the waves scrambled over the tiles of each round ran 8 %
//     slower), so the dynamic part is the tail: 65 % ran Golay 161.0 / packed
//     147.0 / H(8,4)+interp 156.2 us against 161.6 / 148.0 / 159.8 at 75 and
//     166-168 / 153-155 / 164-166 at 85-90 (profiles/r03/fused/static_pct_ab1.log).
//   * round 5: the Golay read's workgroups went from 8 waves, 2 per CU and a
//     65 % static share to 4 waves, 3 per CU (12 waves per CU, each workgroup
//     staging the 32 KiB of tables for 4 waves) and a 30 % static share: int32
//     161.7 -> 158.8 us, packed 147.6 -> 143.5 (interleaved A/B,
//     profiles/r05/golay_read_ab3.log; 50 / 40 / 20 / 10 % 160.7 / 159.4 /
//     159.2 / 158.9, 4 waves at 2 per CU 169.8).
constexpr int kTileBlock = 512;                    // rounds 3-5's 8-wave byte-codec reads (tools/exp forks)
constexpr int kTileWaves = kTileBlock / kWave;
// the byte-codec reads (plain and interpolating): 2-wave workgroups on a full
// grid, one tile per wave; no dynamic LDS cap.  Plain H(8,4) -> fp16 at
// [8,4096,32,128]: 137.9-138.8 us against 139.0-139.9 for 8-wave workgroups
// capped at 4 per CU (profiles/r06/interp_read_ab_*.txt, "pl2" vs "plain")
constexpr int kBytesReadWaves = 2;
constexpr int kGolayTileBlock = 256;               // Golay read: 4 waves per workgroup
constexpr int kGolayTileWaves = kGolayTileBlock / kWave;
constexpr int kShimTilePerCu = 3;                  // Golay read: persistent grid
constexpr int kShimBytesLdsPad = 16384;            // rounds 3-5: capped the 8-wave reads at 4 per CU (tools/exp)
constexpr uint32_t kShimReadStaticPct = 30;        // Golay read: static share of the dynamic-tail schedule
constexpr int kTileStage = 2304;                   // LDS bytes per wave tile
constexpr int kTileGroups = 4;                     // codeword groups per lane per tile (max)
constexpr int kTileChunks = 5;                     // 8-value output chunks per lane per tile (max)
constexpr int kTileAux = 2;                        // buffer cache policy: nt

struct ShimTileArgs {
  const void *cache[2];
  const float *scales[2];
  void *out[2];           // [batch, hkv, ctx, d]
  const int32_t *table;   // [batch, tstride]
  const uint32_t *atab;   // spread tables (golay_attn_table_dev)
  uint64_t *stats;
  uint32_t tstride, hkv, d, g, layers, bs, layer, ctx;
  uint32_t gpr;           // 4-codeword groups per row: ceil(g / 4)
  uint32_t lr;            // LDS bytes per staged row: 12 * gpr
  uint32_t tr;            // rows per tile (<= 64)
  uint32_t tpb;           // tiles per block: ceil(bs / tr)
  uint32_t nlb;           // logical blocks covering ctx
  uint32_t units;         // 2 * batch * hkv * nlb * tpb
  uint32_t rowb;          // bytes per cache row (4g int32, KVECC_GOLAY_PACKED_ROW(g) packed)
  uint32_t *dyn;          // work-counter slot (shim_dyn_slot) of the dynamic schedule
};



// a wave's tile: rows [row0, row0 + rows) of one cache side (wave-uniform)
struct ShimTile {
  uint32_t side, rows, pos0, bh;
  int64_t row0;  // first cache row; -1 = no physical block (zeros out)
};

__device__ __forceinline__ ShimTile shim_tile(const ShimTileArgs &a, uint32_t u) {
  ShimTile t;
  const uint32_t per_side = a.units / 2;
  t.side = u >= per_side ? 1u : 0u;
  u -= t.side * per_side;
  const uint32_t ch = u % a.tpb;
  u /= a.tpb;
  const uint32_t lb = u % a.nlb;
  t.bh = u / a.nlb;
  const uint32_t b = t.bh / a.hkv, h = t.bh - b * a.hkv;
  t.pos0 = lb * a.bs + ch * a.tr;
  t.rows = t.pos0 < a.ctx ? min(min(a.tr, a.bs - ch * a.tr), a.ctx - t.pos0) : 0u;
  const int32_t blk = ld_scalar(a.table + (int64_t)b * a.tstride + lb);
  t.row0 = blk < 0 ? -1 : (((int64_t)blk * a.layers + a.layer) * a.hkv + h) * a.bs + ch * a.tr;
  return t;
}

// per-lane items, identical for every tile
struct TileItems {
  uint32_t r1[kTileGroups], q1[kTileGroups];  // phase 1: row, 4-codeword group
  uint32_t r2[2 * kTileChunks], j2[2 * kTileChunks];  // phase 2: row, the chunk's LDS byte offset
  uint32_t o2[2 * kTileChunks];                       // phase 2: output byte offset in the tile
};

// the tile's codewords and its rows' scales, into registers.  Buffer
// descriptors cover exactly the tile's bytes: past them (rows >= t.rows, a
// missing block, a row's last group running into the next row) loads return 0,
// which decodes to 0 with no error count; the overrun codeword is masked
// out of the statistics and never reaches the output.
// the tile's codewords (raw: packed rows' 3 dwords are unpacked where used, so
// nothing waits on the loads here) and its rows' scales, into registers.
// Buffer descriptors cover exactly the tile's bytes: past them (rows >=
// t.rows, a missing block, a row's last group running into the next row)
// loads return 0, which decodes to 0 with no error count; the overrun
// codeword is masked out of the statistics and never reaches the output.
template <bool PACKED, int NG = 0>
__device__ __forceinline__ void tile_issue(const ShimTileArgs &a, const ShimTile &t, uint32_t lane,
                                           const TileItems &it, u32x4 (&w)[kTileGroups], float &scale) {
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
  scale = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ss, 4 * lane, 0, 0));
  const uint32_t groups = a.tr * a.gpr;
#pragma unroll
  for (int i = 0; i < (NG ? NG : kTileGroups); ++i) {
    if (!NG && i * kWave >= (int)groups) break;  // uniform (NG: the fixed count)
    const uint32_t off = it.r1[i] * a.rowb + (PACKED ? 12u : 16u) * it.q1[i];
    if (PACKED) {  // 4 three-byte codewords in 3 dwords
      const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, kTileAux);
      w[i] = u32x4{v[0], v[1], v[2], 0u};
    } else {
      w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kTileAux));
    }
  }
}

// codeword k of group w (packed: from its 3 raw dwords)
template <bool PACKED>
__device__ __forceinline__ uint32_t tile_cw(const u32x4 &w, int k) {
  if (!PACKED) return w[k];
  switch (k) {
    case 0: return w[0];
    case 1: return __builtin_amdgcn_alignbyte(w[1], w[0], 3);
    case 2: return __builtin_amdgcn_alignbyte(w[2], w[1], 2);
    default: return w[2] >> 8;
  }
}

// values per lane per output item: one 16-byte store (fp16/bf16: 8, fp32: 4),
// so each wave-instruction writes 1 KiB contiguous (32-byte lane strides, two
// stores per lane, halved the store rate)
template <typename TO>
constexpr int kVpl = 16 / (int)sizeof(TO);

// packed dequantization (dq4 / pack2 / dq16): kvecc_internal.h

// 16-byte store through a tile's output descriptor (offsets past it are dropped)
__device__ __forceinline__ void tile_store(const __amdgpu_buffer_rsrc_t &os, uint32_t off, const u32x4 &v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), os,
                                         off, 0, kTileAux);
}

// a tile's output rows [pos0, pos0 + rows) of [bh, ctx, d] as a buffer resource
template <typename TO>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_out(const ShimTileArgs &a, const ShimTile &t) {
  char *base = const_cast<char *>(uni(reinterpret_cast<const char *>(a.out[uni(t.side)]) +
                                      ((int64_t)uni(t.bh) * a.ctx + uni(t.pos0)) * a.d * (int64_t)sizeof(TO)));
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)uni(t.rows * a.d * (uint32_t)sizeof(TO)), 0x00020000);
}

template <typename TO, bool STATS, bool PACKED, int NG = 0, int NCF = 0>
__global__ __launch_bounds__(kGolayTileBlock) void shim_read_golay_tiles_kernel(ShimTileArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[8192];
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kGolayTileWaves][kTileStage];
  // row scales of the staged tile: written in phase 1, read in phase 2 (a
  // scale kept in a register across the next tile's prefetch made the compiler
  // wait for that prefetch before phase 2)
  __shared__ float scale_all[kGolayTileWaves][kWave];
  {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(a.atab);
    u32x4 *dst = reinterpret_cast<u32x4 *>(tab);
#pragma unroll
    for (int i = threadIdx.x; i < 2048; i += kGolayTileBlock) dst[i] = src[i];
  }
  __syncthreads();
  // wave-uniform from here on (readfirstlane: the compiler cannot prove it)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  const uint32_t nwaves = gridDim.x * kGolayTileWaves;
  const uint32_t groups = a.tr * a.gpr;  // <= 64 * kTileGroups (host check)
  constexpr int V = kVpl<TO>, NC = kTileChunks * 8 / V;  // output chunks per lane (max)
  const uint32_t dv = a.d / V;
  const uint32_t chunks = a.tr * dv;     // <= 64 * NC (host check: tr * d / 8 <= 64 * kTileChunks)
  TileItems it;
#pragma unroll
  for (int i = 0; i < kTileGroups; ++i) {
    const uint32_t f = lane + kWave * i;
    it.r1[i] = f / a.gpr;
    it.q1[i] = f - it.r1[i] * a.gpr;
  }
  // fp32 output (NC = 10): the compiler keeps the phase-2 loop rolled, and
  // per-lane item arrays indexed by its counter went to scratch (116 B, a
  // vmcnt(0) wait per item); there the row is computed per item instead, by a
  // reciprocal multiply exact for v < 2^32 / dv (v < 64 NC, dv = d / 4 >= 2)
  constexpr bool kItemsInRegs = NC <= 8;
  const uint32_t inv_dv = kItemsInRegs ? 0u : (uint32_t)(((1ull << 32) + dv - 1) / dv);
  if (kItemsInRegs) {  // r2: row, j2: the item's LDS byte offset in the tile
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      // rows past the tile (r >= tr: a lane's last items) store outside the
      // output descriptor (dropped); their LDS reads use row tr - 1, so every
      // LDS index stays inside the wave's tile
      const uint32_t v = lane + kWave * i;
      const uint32_t r = v / dv, j = v - r * dv;
      it.r2[i] = min(r, a.tr - 1);
      it.j2[i] = it.r2[i] * a.lr + V * j;
      it.o2[i] = (r * a.d + V * j) * (uint32_t)sizeof(TO);
    }
  }
  uint32_t bits = 0, unc = 0;
  // waves retire independently: no workgroup barrier below
  const uint32_t gw = blockIdx.x * kGolayTileWaves + wave;
  uint32_t u = gw;
  if (u >= a.units) return;
  TileSchedule sched;
  sched.init(a.units, a.dyn, gw, nwaves, lane, kShimReadStaticPct);
  ShimTile cur = shim_tile(a, u);
  u32x4 w[kTileGroups];
  float scale;
  tile_issue<PACKED, NG>(a, cur, lane, it, w, scale);
  uint8_t *stage = stage_all[wave];
  const char *tb = reinterpret_cast<const char *>(tab);
  for (;;) {
    // ---- phase 1: decode 4 codewords per group into the LDS tile ---------------
    scale_all[wave][lane] = scale;
    // (n & 3) | uncorrectable << 6 per codeword (the correction table's byte
    // 3), summed over the lane's <= 16 codewords of the tile: no carry
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < (NG ? NG : kTileGroups); ++i) {
      if (!NG && i * kWave >= (int)groups) break;  // uniform
      const uint32_t q = it.q1[i];
      uint32_t sp[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t cw = tile_cw<PACKED>(w[i], c);
        // a row's last group runs into the next row: that codeword decodes
        // as 0 (no count), and its bytes land in the LDS row's padding
        if (c > 0) cw = 4 * q + c < a.g ? cw : 0u;
        const uint32_t p = *reinterpret_cast<const uint32_t *>(tb + ((cw << 2) & 0x3FFCu));
        // syndrome = parity bits ^ parity(data), as a byte offset: ((cw >> 12 ^ p >> 20) & 0xFFF) * 4
        const uint32_t e = *reinterpret_cast<const uint32_t *>(tb + 16384 + (((cw >> 10) ^ (p >> 18)) & 0x3FFCu));
        sp[c] = __builtin_amdgcn_bitop3_b32(p, e, 0x000F0F0Fu, 0x28);  // (p ^ e) & mask
        if (STATS) cnt += e >> 24;
      }
      if (it.r1[i] < a.tr) {  // groups past the tile's last row are never staged
        uint32_t *dst = reinterpret_cast<uint32_t *>(stage + it.r1[i] * a.lr + 12 * q);
        dst[0] = sp[0] | sp[1] << 24;
        dst[1] = sp[1] >> 8 | sp[2] << 16;
        dst[2] = sp[2] >> 16 | sp[3] << 8;
      }
    }
    if (STATS) {
      bits += cnt & 63u;
      unc += cnt >> 6;
    }
    wave_lds_sync();
    // ---- prefetch the next tile's codewords and scales ----------------------------
    const ShimTile t = cur;
    u = sched.next(u, lane);
    const bool more = u < a.units;
    if (more) {
      cur = shim_tile(a, u);
      tile_issue<PACKED, NG>(a, cur, lane, it, w, scale);
    }
    // ---- phase 2: dequantize VPL values per lane, one 16-byte store each -------
    // (stores of rows past the tile fall outside its output descriptor: dropped)
    const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
    const bool dead = t.row0 < 0;
#pragma unroll
    for (int i = 0; i < (NCF ? NCF : NC); ++i) {
      if (!NCF && i * kWave >= (int)chunks) break;  // uniform (NCF: the fixed count)
      uint32_t r, l, o;
      if (kItemsInRegs) {
        r = it.r2[i];
        l = it.j2[i];
        o = it.o2[i];
      } else {
        const uint32_t v = lane + kWave * i;
        const uint32_t rv = __umulhi(v, inv_dv), j = v - rv * dv;
        r = min(rv, a.tr - 1);  // as it.r2: LDS reads stay inside the tile
        l = r * a.lr + V * j;
        o = (rv * a.d + V * j) * (uint32_t)sizeof(TO);
      }
      const uint32_t *src = reinterpret_cast<const uint32_t *>(stage + l);
      const uint32_t nb[2] = {src[0], V == 8 ? src[1] : 0u};
      tile_store(os, o, dq16<TO>(nb, scale_all[wave][r], dead));
    }
    if (!more) break;
    wave_lds_sync();  // phase 2 reads done before the next phase 1 overwrites
  }
  if (STATS) {  // wave reduction, one atomic pair per wave
    bits = wave_sum(bits);
    unc = wave_sum(unc);
    if (lane == 0) {
      uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
      if (bits) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)bits);
      if (unc) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)unc);
    }
  }
}

// ---- byte codecs (raw INT4, H(7,4), H(8,4) [+ interpolation]) through wave tiles
// The Golay tile scheme for one-byte codewords (d % 16 == 0): a wave owns the
// `tr` rows of one (side, sequence, head, block), on a full grid -- one tile
// per wave, workgroups retiring and being replaced, which evens out the waves'
// uneven memory latency with no schedule (137-143 us against 147 for a
// persistent grid).  Phase 1: each lane decodes 16-byte chunks
// of codewords (16 values, SWAR through the v_perm tables) into the wave's LDS
// tile, one byte per value.  Phase 2: each lane dequantizes a chunk of a row
// and writes a 16-byte non-temporal store, 1 KiB contiguous per
// wave-instruction.  A row in a missing block (table entry -1) reads as zero
// codewords and outputs +0, as in the Golay kernel and the host twin.
constexpr int kByteTileItems = 4;  // 16-value chunks per lane per phase (max)

// the tile's codewords (one 16-byte chunk per item: row ir, chunk ic) and its
// rows' scales; rows past the tile and missing blocks load as 0 through the
// buffer bounds (codeword 0 decodes clean)
__device__ __forceinline__ float byte_tile_issue(const ShimTileArgs &a, const ShimTile &t, uint32_t lane,
                                                 const uint32_t *ir, const uint32_t *ic, uint32_t items,
                                                 u32x4 *w) {
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
#pragma unroll
  for (int i = 0; i < kByteTileItems; ++i) {
    if (i * kWave >= (int)items) break;  // uniform
    w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ir[i] * a.d + 16 * ic[i], 0, 2));
  }
  return scale;
}

template <typename TO, int CODEC, bool STATS>
__global__ __launch_bounds__(kBytesReadWaves * kWave) void shim_read_bytes_tiles_kernel(ShimTileArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kBytesReadWaves][kTileStage];
  __shared__ float scale_all[kBytesReadWaves][kWave];  // row scales, staged like the rows
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  uint8_t *stage = stage_all[wave];
  const uint32_t cpr = a.d / 16;       // 16-byte chunks per row
  const uint32_t items = a.tr * cpr;   // <= 64 * kByteTileItems (host check)
  uint32_t ir[kByteTileItems], ic[kByteTileItems];          // phase 1: row, 16-value chunk
  constexpr int V = kVpl<TO>, NI2 = kByteTileItems * 16 / V;  // phase 2: V-value chunks
  uint32_t i2r[NI2], i2c[NI2];                              // phase 2: row, chunk
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
  const uint32_t gw = blockIdx.x * kBytesReadWaves + wave;
  if (gw >= a.units) return;
  const ShimTile t = shim_tile(a, gw);
  u32x4 w[kByteTileItems];
  scale_all[wave][lane] = byte_tile_issue(a, t, lane, ir, ic, items, w);
  uint32_t n1 = 0, n2 = 0;
  auto dec = [&](uint32_t cw) -> uint32_t {  // 4 codewords -> data per byte (and the statistics)
    uint32_t q = cw, tt = 0, s1 = 0, s2 = 0;
    if (CODEC == KVECC_CODEC_H84) {
      h84_decode4(cw, q, tt, s1, s2);
    } else if (CODEC == KVECC_CODEC_H74) {
      h74_decode4(cw, q, tt, s1);
    }
    if (STATS) {
      n1 += s1;
      n2 += s2;
    }
    return q;
  };
#pragma unroll
  for (int i = 0; i < kByteTileItems; ++i) {
    if (i * kWave >= (int)items) break;  // uniform
    const u32x4 d4{dec(w[i].x), dec(w[i].y), dec(w[i].z), dec(w[i].w)};
    if (ir[i] < a.tr) *reinterpret_cast<u32x4 *>(stage + ir[i] * a.d + 16 * ic[i]) = d4;
  }
  wave_lds_sync();
  // phase 2: rows past the tile fall outside its output descriptor (dropped);
  // their LDS reads use row tr - 1
  const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
  const bool dead = t.row0 < 0;
#pragma unroll
  for (int i = 0; i < NI2; ++i) {
    if (i * kWave >= (int)(items * 16 / V)) break;  // uniform
    const uint32_t r = min(i2r[i], a.tr - 1), c = i2c[i];
    const uint8_t *row = stage + r * a.d + V * c;
    uint32_t q[2] = {0u, 0u};
#pragma unroll
    for (int k = 0; k < V / 4; ++k) {
      const uint32_t v = reinterpret_cast<const uint32_t *>(row)[k];
      q[k] = CODEC == KVECC_CODEC_NONE ? v : v & 0x0F0F0F0Fu;  // raw bytes as stored, unmasked
    }
    tile_store(os, (i2r[i] * a.d + V * c) * (uint32_t)sizeof(TO), dq16<TO>(q, scale_all[wave][r], dead));
  }
  if (STATS) {
    n1 = wave_sum(n1);
    n2 = wave_sum(n2);
    if (lane == 0) {
      uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
      if (n1) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)n1);
      if (n2) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)n2);
    }
  }
}

// ---- H(8,4) with double-error interpolation (ecc_shim.py:1038-1059,
// interpolation_triton.py:120-159) on the same full grid.
// Interpolating row r needs the decoded rows r - 1 and r + 1.  Only a double
// error changes a value, so only a tile whose decode saw one interpolates (a
// wave ballot: ~5.6 % of 16-row tiles at BER 1e-3), from its own LDS tile --
// the tile is staged one row down, stage rows 0 and rows + 1 holding the
// neighbour rows.  Those rows belong to other tiles, and only a double in the
// tile's FIRST or LAST row reads them (a second ballot, ~0.7 % of tiles): that
// wave loads the one row from memory (through the block table) and decodes it;
// at the context's ends the row is the tile's own first / last row, as the
// composed read clamps.  Every wave is independent -- no start barrier, no
// flags between waves -- and workgroups are 2 waves, so a wave that does go
// to memory holds one other wave's slot, not seven.  Phase 2 derives each
// item's (row, chunk) by a reciprocal multiply (with the interpolating body
// present the compiler otherwise re-derived per-item divisions after phase 1,
// on every wave's critical path).
// [8,4096,32,128] K+V fp16, BER 1e-3: 140.2 us, the plain read's time (140.2),
// against 148.3 for round 5's kernel -- 8-wave workgroups exchanging edge rows
// through LDS words behind a start barrier; 1e-2: 184.8 against 190.1; BER 0:
// 139.9 against 142.4 (profiles/r06/interp_read_ab_*.txt,
// tools/exp/interp_read_exp.hip: 1 / 4 / 8 waves per workgroup 140.4 / 140.8
// / 143.0 at 1e-3).  N1 > 0: the tile has exactly N1 * 64 phase-1 items (the
// host checks), so both phases run a fixed item count with no per-item exit
// test: the compiler then issues every item's LDS reads before the first wait
// instead of one read-wait-store chain per item (140.0-140.7 against
// 141.6-142.6 us at 1e-3; the plain read gains nothing from it,
// profiles/r06/interp_read_fixed_*.txt).

template <typename TO, bool STATS, int N1 = 0>
__global__ __launch_bounds__(kBytesReadWaves * kWave) void shim_read_h84_interp_kernel(ShimTileArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kBytesReadWaves][kTileStage];
  __shared__ float scale_all[kBytesReadWaves][kWave];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  uint8_t *stage = stage_all[wave];
  const uint32_t cpr = a.d / 16;
  const uint32_t items = a.tr * cpr;
  uint32_t ir[kByteTileItems], ic[kByteTileItems];
#pragma unroll
  for (int i = 0; i < kByteTileItems; ++i) {
    const uint32_t f = lane + kWave * i;
    ir[i] = f / cpr;
    ic[i] = f - ir[i] * cpr;
  }
  constexpr int V = kVpl<TO>, NI2 = kByteTileItems * 16 / V;
  const uint32_t gw = blockIdx.x * kBytesReadWaves + wave;
  if (gw >= a.units) return;
  const ShimTile t = shim_tile(a, gw);
  u32x4 w[kByteTileItems];
  scale_all[wave][lane] = byte_tile_issue(a, t, lane, ir, ic, items, w);
  uint32_t n1 = 0, n2 = 0;
  bool dbl_any = false, dbl_top = false, dbl_bot = false;
  const uint32_t off0 = a.d;  // tile row r at stage row r + 1
  // data | error type << 4 per byte of 4 codewords
  auto dec = [&](uint32_t cw, uint32_t &dbl) -> uint32_t {
    uint32_t q = cw, tt = 0, s1 = 0, s2 = 0;
    h84_decode4(cw, q, tt, s1, s2);
    if (STATS) {
      n1 += s1;
      n2 += s2;
    }
    dbl |= s2;
    return q | tt << 4;
  };
#pragma unroll
  for (int i = 0; i < (N1 ? N1 : kByteTileItems); ++i) {
    if (!N1 && i * kWave >= (int)items) break;  // uniform (N1: the fixed count)
    // rows past the tile: no statistics, no doubles, no LDS store (it would
    // land on the row-below slot)
    if (ir[i] < t.rows) {
      uint32_t dbl = 0;
      const u32x4 d4{dec(w[i].x, dbl), dec(w[i].y, dbl), dec(w[i].z, dbl), dec(w[i].w, dbl)};
      dbl_any |= dbl != 0;
      dbl_top |= dbl != 0 && ir[i] == 0;
      dbl_bot |= dbl != 0 && ir[i] + 1 == t.rows;
      *reinterpret_cast<u32x4 *>(stage + off0 + ir[i] * a.d + 16 * ic[i]) = d4;
    }
  }
  const bool tile_dbl = __builtin_amdgcn_ballot_w64(dbl_any) != 0;
  wave_lds_sync();
  if (tile_dbl) {  // wave-uniform: the neighbour rows the edge rows' doubles need
    const bool need_top = __builtin_amdgcn_ballot_w64(dbl_top) != 0;
    const bool need_bot = __builtin_amdgcn_ballot_w64(dbl_bot) != 0;
    const bool below = lane >= cpr;  // lanes [0, cpr): the row above; [cpr, 2 cpr): below
    const uint32_t l = below ? lane - cpr : lane;
    if (lane < 2 * cpr && (below ? need_bot : need_top)) {
      u32x4 v;
      if (below ? t.pos0 + t.rows >= a.ctx : t.pos0 == 0) {  // clamped: the tile's own edge row
        v = reinterpret_cast<const u32x4 *>(stage + off0 + (below ? t.rows - 1 : 0u) * a.d)[l];
      } else {
        const uint32_t b = t.bh / a.hkv, h = t.bh - b * a.hkv;
        const uint32_t pos = below ? t.pos0 + t.rows : t.pos0 - 1;
        const int32_t blk = a.table[(int64_t)b * a.tstride + pos / a.bs];
        u32x4 hw{0u, 0u, 0u, 0u};  // a missing block reads as zero codewords
        if (blk >= 0) {
          const int64_t row = (((int64_t)blk * a.layers + a.layer) * a.hkv + h) * a.bs + (pos % a.bs);
          hw = ld_stream(reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(a.cache[t.side]) +
                                                         row * a.d) + l);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // decoded as the tile's rows; neighbours add no statistics
          uint32_t q = hw[k], tt = 0, s1 = 0, s2 = 0;
          h84_decode4(hw[k], q, tt, s1, s2);
          v[k] = q | tt << 4;
        }
      }
      *reinterpret_cast<u32x4 *>(stage + (below ? t.rows + 1 : 0u) * a.d + 16 * l) = v;
    }
    wave_lds_sync();
  }
  const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
  const bool dead = t.row0 < 0;
  // item i: f = lane + 64 i, row f / per, chunk f % per; f / per as
  // (f m) >> 16 with m = ceil(2^16 / per), exact since f (m - 2^16 / per) <
  // 2^9 / 2^16 < 1 / per for f < 2^9, per <= 64
  const uint32_t per = cpr * 16 / V;
  const uint32_t m = uni((65536u + per - 1) / per);
  // one straight-line body per case (a branch per item serialised its LDS reads)
  auto phase2 = [&](auto interp_c) {
    constexpr bool IP = decltype(interp_c)::value;
#pragma unroll
    for (int i = 0; i < (N1 ? N1 * 16 / V : NI2); ++i) {
      if (!N1 && i * kWave >= (int)(items * 16 / V)) break;  // uniform
      const uint32_t f = lane + kWave * i;
      const uint32_t rr = __umul24(f, m) >> 16, c = f - rr * per;
      const uint32_t r = min(rr, a.tr - 1);  // rows past the tile: stores dropped, reads in the tile
      const uint8_t *row = stage + off0 + r * a.d + V * c;
      uint32_t q[2] = {0u, 0u};
#pragma unroll
      for (int k = 0; k < V / 4; ++k) {
        const uint32_t v = reinterpret_cast<const uint32_t *>(row)[k];
        if (IP) {  // a neighbour row no double reads may be stale LDS: interp_word ignores it
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
  if (tile_dbl)
    phase2(std::integral_constant<bool, true>{});
  else
    phase2(std::integral_constant<bool, false>{});
  if (STATS) {
    n1 = wave_sum(n1);
    n2 = wave_sum(n2);
    if (lane == 0) {
      uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
      if (n1) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)n1);
      if (n2) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)n2);
    }
  }
}

template <typename T, int CODEC>
static void launch_write_nb(const ShimWriteArgs &a, unsigned grid, hipStream_t st) {
  constexpr int NB = CODEC == KVECC_CODEC_GOLAY || CODEC == KVECC_CODEC_GOLAY_PACKED ? 24
                     : CODEC == KVECC_CODEC_H84 ? 8
                     : CODEC == KVECC_CODEC_H74 ? 7
                                                : 4;
  if (a.nb_eff == NB)
    KVECC_LAUNCH((shim_write_kernel<T, CODEC, NB>), dim3(grid), dim3(kBlock), 0, st, a);
  else
    KVECC_LAUNCH((shim_write_kernel<T, CODEC, -1>), dim3(grid), dim3(kBlock), 0, st, a);
}

template <typename T>
static void launch_write(int codec, const ShimWriteArgs &a, unsigned grid, hipStream_t st) {
  switch (codec) {
    case KVECC_CODEC_NONE: launch_write_nb<T, KVECC_CODEC_NONE>(a, grid, st); break;
    case KVECC_CODEC_H74: launch_write_nb<T, KVECC_CODEC_H74>(a, grid, st); break;
    case KVECC_CODEC_H84: launch_write_nb<T, KVECC_CODEC_H84>(a, grid, st); break;
    case KVECC_CODEC_GOLAY_PACKED: launch_write_nb<T, KVECC_CODEC_GOLAY_PACKED>(a, grid, st); break;
    default: launch_write_nb<T, KVECC_CODEC_GOLAY>(a, grid, st); break;
  }
}

template <typename TO, int CODEC, bool INTERP>
static void launch_read_bytes(const ShimReadArgs &a, unsigned grid, hipStream_t st) {
  if (a.stats)
    KVECC_LAUNCH((shim_read_bytes_kernel<TO, CODEC, INTERP, true>), dim3(grid), dim3(kBlock), 0, st, a);
  else
    KVECC_LAUNCH((shim_read_bytes_kernel<TO, CODEC, INTERP, false>), dim3(grid), dim3(kBlock), 0, st, a);
}

template <typename TO>
static void launch_read(int codec, int interp, const ShimReadArgs &a, hipStream_t st) {
  if (codec == KVECC_CODEC_GOLAY || codec == KVECC_CODEC_GOLAY_PACKED) {
    const unsigned grid = grid_for(2 * a.geo.hkv * a.ctx * a.geo.g, kBlock);
    const bool pk = codec == KVECC_CODEC_GOLAY_PACKED;
    if (a.stats && pk)
      KVECC_LAUNCH((shim_read_golay_kernel<TO, true, true>), dim3(grid), dim3(kBlock), 0, st, a);
    else if (a.stats)
      KVECC_LAUNCH((shim_read_golay_kernel<TO, true, false>), dim3(grid), dim3(kBlock), 0, st, a);
    else if (pk)
      KVECC_LAUNCH((shim_read_golay_kernel<TO, false, true>), dim3(grid), dim3(kBlock), 0, st, a);
    else
      KVECC_LAUNCH((shim_read_golay_kernel<TO, false, false>), dim3(grid), dim3(kBlock), 0, st, a);
    return;
  }
  const unsigned grid = grid_for(2 * a.geo.hkv * a.ctx * (a.geo.d / 4), kBlock);
  if (codec == KVECC_CODEC_H84) {
    if (interp)
      launch_read_bytes<TO, KVECC_CODEC_H84, true>(a, grid, st);
    else
      launch_read_bytes<TO, KVECC_CODEC_H84, false>(a, grid, st);
  } else if (codec == KVECC_CODEC_H74) {
    launch_read_bytes<TO, KVECC_CODEC_H74, false>(a, grid, st);
  } else {
    launch_read_bytes<TO, KVECC_CODEC_NONE, false>(a, grid, st);
  }
}

// the Golay read's persistent grid: kShimTilePerCu workgroups per CU
static unsigned tile_grid(uint32_t units) {
  return (unsigned)std::min<int64_t>(cdiv(units, kGolayTileWaves), (int64_t)cu_count() * kShimTilePerCu);
}

template <typename TO>
static void launch_read_tiles(bool packed, const ShimTileArgs &a, hipStream_t st) {
  const unsigned grid = tile_grid(a.units);
  constexpr unsigned pad = 0;
  if (a.stats && packed)
    KVECC_LAUNCH((shim_read_golay_tiles_kernel<TO, true, true>), dim3(grid), dim3(kGolayTileBlock), pad, st, a);
  else if (a.stats)
    KVECC_LAUNCH((shim_read_golay_tiles_kernel<TO, true, false>), dim3(grid), dim3(kGolayTileBlock), pad, st, a);
  else if (packed)
    KVECC_LAUNCH((shim_read_golay_tiles_kernel<TO, false, true>), dim3(grid), dim3(kGolayTileBlock), pad, st, a);
  else
    KVECC_LAUNCH((shim_read_golay_tiles_kernel<TO, false, false>), dim3(grid), dim3(kGolayTileBlock), pad, st, a);
}

// byte codecs: a full grid, one tile per wave, 2-wave workgroups
template <typename TO, int CODEC>
static void launch_bytes_plain(const ShimTileArgs &a, hipStream_t st) {
  const unsigned grid = (unsigned)cdiv(a.units, kBytesReadWaves);
  if (a.stats)
    KVECC_LAUNCH((shim_read_bytes_tiles_kernel<TO, CODEC, true>), dim3(grid), dim3(kBytesReadWaves * kWave), 0, st, a);
  else
    KVECC_LAUNCH((shim_read_bytes_tiles_kernel<TO, CODEC, false>), dim3(grid), dim3(kBytesReadWaves * kWave), 0, st, a);
}

// the interpolating read with N1 fixed phase-1 items per lane (0: the generic count)
template <typename TO, int N1>
static void launch_interp_read(const ShimTileArgs &a, unsigned grid, hipStream_t st) {
  if (a.stats)
    KVECC_LAUNCH((shim_read_h84_interp_kernel<TO, true, N1>), dim3(grid), dim3(kBytesReadWaves * kWave), 0, st, a);
  else
    KVECC_LAUNCH((shim_read_h84_interp_kernel<TO, false, N1>), dim3(grid), dim3(kBytesReadWaves * kWave), 0, st, a);
}

template <typename TO>
static void launch_bytes_tiles(int codec, int interp, const ShimTileArgs &a, hipStream_t st) {
  if (codec == KVECC_CODEC_H84 && interp) {
    const unsigned grid = (unsigned)cdiv(a.units, kBytesReadWaves);
    const uint32_t items = a.tr * (a.d / 16);
    if (items == 2 * kWave)  // e.g. head_dim 128 in 16-row tiles
      launch_interp_read<TO, 2>(a, grid, st);
    else if (items == kWave)  // e.g. head_dim 64 in 16-row tiles (GPT-2)
      launch_interp_read<TO, 1>(a, grid, st);
    else
      launch_interp_read<TO, 0>(a, grid, st);
  } else if (codec == KVECC_CODEC_H84) {
    launch_bytes_plain<TO, KVECC_CODEC_H84>(a, st);
  } else if (codec == KVECC_CODEC_H74) {
    launch_bytes_plain<TO, KVECC_CODEC_H74>(a, st);
  } else {
    launch_bytes_plain<TO, KVECC_CODEC_NONE>(a, st);
  }
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

static int shim_write_impl(const void *k, const void *v, const int64_t xb[2], const int64_t xs[2],
                           const int64_t xh[2], int x_dtype, int64_t batch, int64_t seq, int64_t hkv, int64_t d,
                           int codec, int scale_rule, int n_bits, int inject, float ber,
                           int64_t seed0, void *k_cache, void *v_cache, float *k_scales,
                           float *v_scales, const int32_t *block_table, int64_t num_layers,
                           int64_t block_size, int64_t layer, void *stream) {
  if (batch < 0 || seq < 0 || hkv < 0 || d < 0) return set_error(KVECC_EINVAL, "shim_write: negative size");
  if (batch == 0 || seq == 0 || hkv == 0) return KVECC_OK;
  if (d < 1 || d > kMaxShimD) return set_error(KVECC_EINVAL, "shim_write: head_dim %lld not in [1, %d]", (long long)d, kMaxShimD);
  if (codec < KVECC_CODEC_NONE || codec > KVECC_CODEC_GOLAY_PACKED)
    return set_error(KVECC_EINVAL, "shim_write: bad codec %d", codec);
  const bool golay = codec == KVECC_CODEC_GOLAY || codec == KVECC_CODEC_GOLAY_PACKED;
  if (scale_rule != KVECC_SCALE_DIV7 && scale_rule != KVECC_SCALE_MUL_INV7)
    return set_error(KVECC_EINVAL, "shim_write: bad scale rule %d", scale_rule);
  if (num_layers < 1 || block_size < 1 || layer < 0 || layer >= num_layers)
    return set_error(KVECC_EINVAL, "shim_write: bad cache geometry");
  if (!k || !v || !k_cache || !v_cache || !k_scales || !v_scales || !block_table)
    return set_error(KVECC_EINVAL, "shim_write: null pointer");
  if (2 * seq * hkv > 0x7FFFFFFFLL || num_layers * hkv * block_size > 0x7FFFFFFFLL)
    return set_error(KVECC_EINVAL, "shim_write: sizes exceed 32-bit indexing");
  for (int s = 0; s < 2; ++s)
    if (xb[s] < 0 || xs[s] < 0 || xh[s] < d)
      return set_error(KVECC_EINVAL, "shim_write: negative stride or head stride < head_dim");
  ShimWriteArgs a;
  a.geo = {block_table, (uint32_t)hkv, (uint32_t)d,
           (uint32_t)(golay ? (d + 2) / 3 : d), (uint32_t)num_layers,
           (uint32_t)block_size, (uint32_t)layer};
  a.x[0] = k;
  a.x[1] = v;
  for (int s = 0; s < 2; ++s) {
    a.xb[s] = xb[s];
    a.xs[s] = xs[s];
    a.xh[s] = xh[s];
  }
  a.cache[0] = k_cache;
  a.cache[1] = v_cache;
  a.scales[0] = k_scales;
  a.scales[1] = v_scales;
  a.batch = batch;
  a.seq = seq;
  a.seed0 = (uint32_t)(uint64_t)seed0;
  a.rowmul = (uint32_t)((uint64_t)a.geo.g * (uint64_t)n_bits);
  a.nbits = (uint32_t)n_bits;
  a.thr = kvecc_ber_threshold(ber);
  a.inject = inject != 0 && ber > 0.0f;
  a.scale_rule = scale_rule;
  // same bit-count clamps as the flat kernels (uint8 caches draw >= 1, <= 8 bits)
  a.nb_eff = golay ? (n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits))
                                        : (n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits));
  const int64_t waves = 2 * seq * hkv;
  const int64_t blocks = cdiv(waves, kWavesPerBlock);
  if (blocks > 0x7FFFFFFF) return set_error(KVECC_EINVAL, "shim_write: too many rows");
  hipStream_t st = as_stream(stream);
  switch (x_dtype) {
    case KVECC_F32: launch_write<float>(codec, a, (unsigned)blocks, st); break;
    case KVECC_F16: launch_write<__half>(codec, a, (unsigned)blocks, st); break;
    case KVECC_BF16: launch_write<__hip_bfloat16>(codec, a, (unsigned)blocks, st); break;
    default: return set_error(KVECC_EINVAL, "shim_write: bad dtype %d", x_dtype);
  }
  return check_launch("shim_write");
}

KVECC_API int kvecc_shim_write(const void *k, const void *v, int x_dtype, int64_t batch,
                               int64_t seq, int64_t hkv, int64_t d, int codec, int scale_rule,
                               int n_bits, int inject, float ber, int64_t seed0, void *k_cache, void *v_cache,
                               float *k_scales, float *v_scales, const int32_t *block_table,
                               int64_t num_layers, int64_t block_size, int64_t layer,
                               void *stream) {
  const int64_t xh[2] = {d, d}, xs[2] = {hkv * d, hkv * d}, xb[2] = {seq * hkv * d, seq * hkv * d};
  return shim_write_impl(k, v, xb, xs, xh, x_dtype, batch, seq, hkv, d, codec, scale_rule, n_bits,
                         inject, ber, seed0, k_cache, v_cache, k_scales, v_scales, block_table,
                         num_layers, block_size, layer, stream);
}

KVECC_API int kvecc_shim_write_strided(const void *k, const void *v, int64_t k_batch_stride,
                                       int64_t k_seq_stride, int64_t k_head_stride,
                                       int64_t v_batch_stride, int64_t v_seq_stride,
                                       int64_t v_head_stride, int x_dtype, int64_t batch,
                                       int64_t seq, int64_t hkv, int64_t d, int codec,
                                       int scale_rule, int n_bits, int inject, float ber,
                                       int64_t seed0, void *k_cache, void *v_cache,
                                       float *k_scales, float *v_scales,
                                       const int32_t *block_table, int64_t num_layers,
                                       int64_t block_size, int64_t layer, void *stream) {
  const int64_t xb[2] = {k_batch_stride, v_batch_stride}, xs[2] = {k_seq_stride, v_seq_stride};
  const int64_t xh[2] = {k_head_stride, v_head_stride};
  return shim_write_impl(k, v, xb, xs, xh, x_dtype, batch, seq, hkv, d, codec, scale_rule, n_bits,
                         inject, ber, seed0, k_cache, v_cache, k_scales, v_scales, block_table,
                         num_layers, block_size, layer, stream);
}

static int shim_read_impl(const void *k_cache, const void *v_cache, const float *k_scales,
                          const float *v_scales, const int32_t *block_table, int64_t tstride,
                          int64_t batch, int64_t ctx, int64_t hkv, int64_t d, int64_t num_layers,
                          int64_t block_size, int64_t layer, int codec, int interp, void *k_out,
                          void *v_out, int out_dtype, uint64_t *stats, void *stream) {
  if (batch < 0 || ctx < 0 || hkv < 0 || d < 0) return set_error(KVECC_EINVAL, "shim_read: negative size");
  if (batch == 0 || ctx == 0 || hkv == 0 || d == 0) return KVECC_OK;
  if (codec < KVECC_CODEC_NONE || codec > KVECC_CODEC_GOLAY_PACKED)
    return set_error(KVECC_EINVAL, "shim_read: bad codec %d", codec);
  const bool golay = codec == KVECC_CODEC_GOLAY || codec == KVECC_CODEC_GOLAY_PACKED;
  if (!golay && d % 4 != 0)
    return set_error(KVECC_EINVAL, "shim_read: head_dim %lld must be a multiple of 4", (long long)d);
  if (interp && codec != KVECC_CODEC_H84)
    return set_error(KVECC_EINVAL, "shim_read: interpolation needs the hamming84 codec");
  if (num_layers < 1 || block_size < 1 || layer < 0 || layer >= num_layers)
    return set_error(KVECC_EINVAL, "shim_read: bad cache geometry");
  if (!k_cache || !v_cache || !k_scales || !v_scales || !block_table || !k_out || !v_out)
    return set_error(KVECC_EINVAL, "shim_read: null pointer");
  if (batch > 1 && tstride < cdiv(ctx, block_size))
    return set_error(KVECC_EINVAL, "shim_read: table stride %lld < %lld blocks", (long long)tstride,
                     (long long)cdiv(ctx, block_size));
  if (2 * hkv * ctx * d > 0x7FFFFFFFLL || num_layers * hkv * block_size > 0x7FFFFFFFLL)
    return set_error(KVECC_EINVAL, "shim_read: sizes exceed 32-bit indexing");
  if (out_dtype != KVECC_F32 && out_dtype != KVECC_F16 && out_dtype != KVECC_BF16)
    return set_error(KVECC_EINVAL, "shim_read: bad dtype %d", out_dtype);
  hipStream_t st = as_stream(stream);
  const int64_t g = golay ? (d + 2) / 3 : d;
  const int64_t gpr = cdiv(g, 4), lr = 12 * gpr;
  if (golay && d % 8 == 0 && lr <= kTileStage && aligned(k_out, 16) && aligned(v_out, 16) &&
      2 * batch * hkv * cdiv(ctx, block_size) * block_size <= 0x7FFFFFFFLL) {
    // Golay: the wave-tile kernel, all sequences in one launch
    ShimTileArgs a;
    a.cache[0] = k_cache;
    a.cache[1] = v_cache;
    a.scales[0] = k_scales;
    a.scales[1] = v_scales;
    a.out[0] = k_out;
    a.out[1] = v_out;
    a.table = block_table;
    a.atab = golay_attn_table_dev();
    if (!a.atab) return KVECC_EHIP;
    a.stats = stats;
    a.tstride = (uint32_t)tstride;
    a.hkv = (uint32_t)hkv;
    a.d = (uint32_t)d;
    a.g = (uint32_t)g;
    a.layers = (uint32_t)num_layers;
    a.bs = (uint32_t)block_size;
    a.layer = (uint32_t)layer;
    a.ctx = (uint32_t)ctx;
    a.gpr = (uint32_t)gpr;
    a.lr = (uint32_t)lr;
    a.tr = (uint32_t)std::min<int64_t>({block_size, kTileStage / lr, (int64_t)kWave * kTileGroups / gpr,
                                        (int64_t)kWave, (int64_t)kWave * kTileChunks / (d / 8)});
    a.tpb = (uint32_t)cdiv(block_size, a.tr);
    a.nlb = (uint32_t)cdiv(ctx, block_size);
    a.units = (uint32_t)(2 * batch * hkv * a.nlb * a.tpb);
    a.rowb = (uint32_t)(codec == KVECC_CODEC_GOLAY_PACKED ? KVECC_GOLAY_PACKED_ROW(g) : 4 * g);
    a.dyn = shim_dyn_slot(stream);
    if (!a.dyn) return KVECC_EHIP;
    const bool pk = codec == KVECC_CODEC_GOLAY_PACKED;
    switch (out_dtype) {
      case KVECC_F32: launch_read_tiles<float>(pk, a, st); break;
      case KVECC_F16: launch_read_tiles<__half>(pk, a, st); break;
      default: launch_read_tiles<__hip_bfloat16>(pk, a, st); break;
    }
    return check_launch("shim_read");
  }
  if (!golay && d % 16 == 0 && (!interp || d <= kWave * 16 / 2) && aligned(k_cache, 16) && aligned(v_cache, 16) && aligned(k_out, 16) && aligned(v_out, 16) &&
      2 * batch * hkv * cdiv(ctx, block_size) * block_size <= 0x7FFFFFFFLL) {
    // byte codecs: the wave-tile kernel, all sequences in one launch
    ShimTileArgs a{};
    a.cache[0] = k_cache;
    a.cache[1] = v_cache;
    a.scales[0] = k_scales;
    a.scales[1] = v_scales;
    a.out[0] = k_out;
    a.out[1] = v_out;
    a.table = block_table;
    a.stats = stats;
    a.tstride = (uint32_t)tstride;
    a.hkv = (uint32_t)hkv;
    a.d = a.g = a.lr = a.rowb = (uint32_t)d;
    a.layers = (uint32_t)num_layers;
    a.bs = (uint32_t)block_size;
    a.layer = (uint32_t)layer;
    a.ctx = (uint32_t)ctx;
    const int64_t cpr = d / 16;
    a.tr = (uint32_t)std::min<int64_t>({block_size, (int64_t)kTileStage / d - (interp ? 2 : 0), (int64_t)kWave,
                                        (int64_t)kWave * kByteTileItems / cpr});
    if (a.tr >= 1) {
      a.tpb = (uint32_t)cdiv(block_size, a.tr);
      a.nlb = (uint32_t)cdiv(ctx, block_size);
      a.units = (uint32_t)(2 * batch * hkv * a.nlb * a.tpb);
      a.dyn = nullptr;  // full grids: no work counters
      switch (out_dtype) {
        case KVECC_F32: launch_bytes_tiles<float>(codec, interp, a, st); break;
        case KVECC_F16: launch_bytes_tiles<__half>(codec, interp, a, st); break;
        default: launch_bytes_tiles<__hip_bfloat16>(codec, interp, a, st); break;
      }
      return check_launch("shim_read");
    }
  }
  const int64_t osz = out_dtype == KVECC_F32 ? 4 : 2;
  for (int64_t b = 0; b < batch; ++b) {  // one launch per sequence
    ShimReadArgs a;
    a.geo = {block_table + b * tstride, (uint32_t)hkv, (uint32_t)d, (uint32_t)g, (uint32_t)num_layers,
             (uint32_t)block_size, (uint32_t)layer};
    a.cache[0] = k_cache;
    a.cache[1] = v_cache;
    a.scales[0] = k_scales;
    a.scales[1] = v_scales;
    a.out[0] = reinterpret_cast<char *>(k_out) + b * hkv * ctx * d * osz;
    a.out[1] = reinterpret_cast<char *>(v_out) + b * hkv * ctx * d * osz;
    a.ctx = (uint32_t)ctx;
    a.stats = stats;
    a.par = a.cor = nullptr;
    if (golay) {
      a.par = golay_parity_table_dev();
      a.cor = golay_correct_table_dev();
      if (!a.par || !a.cor) return KVECC_EHIP;
    }
    switch (out_dtype) {
      case KVECC_F32: launch_read<float>(codec, interp, a, st); break;
      case KVECC_F16: launch_read<__half>(codec, interp, a, st); break;
      default: launch_read<__hip_bfloat16>(codec, interp, a, st); break;
    }
  }
  return check_launch("shim_read");
}

KVECC_API int kvecc_shim_read(const void *k_cache, const void *v_cache, const float *k_scales,
                              const float *v_scales, const int32_t *block_table, int64_t ctx,
                              int64_t hkv, int64_t d, int64_t num_layers, int64_t block_size,
                              int64_t layer, int codec, int interp, void *k_out, void *v_out,
                              int out_dtype, uint64_t *stats, void *stream) {
  return shim_read_impl(k_cache, v_cache, k_scales, v_scales, block_table, 0, 1, ctx, hkv, d,
                        num_layers, block_size, layer, codec, interp, k_out, v_out, out_dtype, stats,
                        stream);
}

KVECC_API int kvecc_shim_read_batch(const void *k_cache, const void *v_cache, const float *k_scales,
                                    const float *v_scales, const int32_t *block_table,
                                    int64_t table_stride, int64_t batch, int64_t ctx, int64_t hkv,
                                    int64_t d, int64_t num_layers, int64_t block_size, int64_t layer,
                                    int codec, int interp, void *k_out, void *v_out, int out_dtype,
                                    uint64_t *stats, void *stream) {
  return shim_read_impl(k_cache, v_cache, k_scales, v_scales, block_table, table_stride, batch, ctx,
                        hkv, d, num_layers, block_size, layer, codec, interp, k_out, v_out, out_dtype,
                        stats, stream);
}

}  // extern "C"
