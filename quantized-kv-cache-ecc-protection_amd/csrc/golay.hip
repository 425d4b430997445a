// golay.hip -- extended Golay(24,12) encode/decode of INT4 triplets.
//
// Reference: ecc_codecs/triton_kernels/golay_triton.py:99-157 (encode) and
// :213-295 (decode).  Codeword = data12 | parity12 << 12 with
// data12 = n0 | n1 << 4 | n2 << 8.
//
// gfx950 design (HBM-bound, 7 B/codeword encode, 8 B/codeword decode):
//  * Two 4096-entry uint16 tables live in LDS (16 KiB per workgroup):
//      parity[d]  = the 12 parity bits of data word d
//      correct[s] = data-error(12) | count(3) << 12 for syndrome s
//    so encode is one LDS gather per codeword, and decode is two: the
//    syndrome is (cw >> 12) ^ parity[cw & 0xFFF] (H = [B^T | I], B symmetric)
//    instead of the reference's 12 masked popcounts, and the correction comes
//    from `correct`, which folds the reference's error-pattern table and its
//    popcount.  Only the data half of an error pattern matters for the output.
//  * Each lane owns kGroups groups of 4 consecutive codewords, and each
//    wave-instruction covers one contiguous span (1 KiB of codewords, 768 B
//    of triplets, 256 B of counts), so every access is fully coalesced:
//    global_load_dwordx4 (codewords), dwordx3 + dword stores (decode), all
//    non-temporal (plain stores ran at ~65% of the nt rate).
//  * Geometry measured on MI355X with interleaved cold-cache A/B runs
//    (tools/exp/run_exp2.py, run_exp3.py): 2 groups per lane, 512-thread
//    decode / 1024-thread encode workgroups, up to 32 / 16 workgroups per CU
//    grid-strided.  More work per lane (4 groups) or lane-contiguous layouts
//    lost 8-45%; computing the parity with VALU instead of the LDS table lost
//    12-20% (the kernel turns VALU-bound).
#include <algorithm>

#include "kvecc_internal.h"

namespace kvecc {

// geometry (tuned by interleaved cold-cache A/B: tools/exp/run_golay_geom.py,
// profiles/r01/golay/geometry_ab.log; DESIGN.md §3 Golay decode)
constexpr int kGroups = 2;                          // 4-codeword groups per lane per tile
constexpr int kDecBlock = 512, kEncBlock = 1024;    // threads per workgroup
constexpr int kDecPerCu = 32, kEncPerCu = 16;       // workgroups per CU (grid-strided)
constexpr int kRowsPerCu = 3;                       // rows decode: persistent workgroups per CU (256 threads, ~41 KB LDS)
constexpr int kDecTile = kDecBlock * kGroups * 4;   // 4096 codewords
constexpr int kEncTile = kEncBlock * kGroups * 4;   // 8192 codewords
constexpr int kWaveCw = kWave * kGroups * 4;        // codewords per wave per tile

// copy the 4096-entry tables (8 KiB each) into LDS
template <int BS>
__device__ __forceinline__ void load_tables(uint16_t *lds, const uint16_t *__restrict__ par,
                                            const uint16_t *__restrict__ cor, bool need_cor) {
  const u32x4 *p = reinterpret_cast<const u32x4 *>(par);
  u32x4 *l = reinterpret_cast<u32x4 *>(lds);
  for (int i = threadIdx.x; i < 512; i += BS) l[i] = p[i];
  if (need_cor) {
    const u32x4 *c = reinterpret_cast<const u32x4 *>(cor);
    for (int i = threadIdx.x; i < 512; i += BS) l[512 + i] = c[i];
  }
  __syncthreads();
}

// triplet packing / unpacking and the table decode: codec_math.h
// ---- encode -------------------------------------------------------------------

// Codewords past the last whole tile (m - ntiles * tile < tile of them) are
// encoded / decoded one per thread by the first workgroups, before their
// tiles: no tail launch (flat M_f = 44,739,243 codewords leaves 2,731; the
// separate tail kernel cost ~2 us of launch per call)
__global__ __launch_bounds__(kEncBlock) void golay_encode_kernel(const uint32_t *__restrict__ trip,
                                                                 u32x4 *__restrict__ cw,
                                                                 int64_t ntiles, int64_t m,
                                                                 const uint16_t *__restrict__ par) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[4096];
  load_tables<kEncBlock>(lds, par, nullptr, false);
  {
    const uint8_t *t8 = reinterpret_cast<const uint8_t *>(trip);
    int32_t *c32 = reinterpret_cast<int32_t *>(cw);
    for (int64_t i = ntiles * kEncTile + (int64_t)blockIdx.x * kEncBlock + threadIdx.x; i < m;
         i += (int64_t)gridDim.x * kEncBlock) {
      const uint32_t d = golay_pack(t8[3 * i], t8[3 * i + 1], t8[3 * i + 2]);
      c32[i] = (int32_t)(d | (uint32_t)lds[d] << 12);
    }
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    // codeword index of this lane's group g: tile + wave*kWaveCw + g*256 + lane*4
    const int64_t base = t * kEncTile + wave * kWaveCw + lane * 4;
    uint32_t w[kGroups][3];
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
      const uint32_t *p = trip + (base + g * 256) * 3 / 4;  // 12 B per 4 codewords
      w[g][0] = ld_stream(p);
      w[g][1] = ld_stream(p + 1);
      w[g][2] = ld_stream(p + 2);
    }
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
      uint32_t d[4];
      golay_unpack4(w[g][0], w[g][1], w[g][2], d);
      u32x4 out;
      out.x = d[0] | (uint32_t)lds[d[0]] << 12;
      out.y = d[1] | (uint32_t)lds[d[1]] << 12;
      out.z = d[2] | (uint32_t)lds[d[2]] << 12;
      out.w = d[3] | (uint32_t)lds[d[3]] << 12;
      st_stream(cw + (base + g * 256) / 4, out);
    }
  }
}

// scalar path: codewords [begin, m), any alignment
__global__ __launch_bounds__(kBlock) void golay_encode_tail_kernel(const uint8_t *__restrict__ trip,
                                                                   int32_t *__restrict__ cw,
                                                                   int64_t begin, int64_t m,
                                                                   const uint16_t *__restrict__ par) {
  for (int64_t i = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * kBlock) {
    uint32_t d = golay_pack(trip[3 * i], trip[3 * i + 1], trip[3 * i + 2]);
    cw[i] = (int32_t)(d | (uint32_t)par[d] << 12);
  }
}

// ---- decode -------------------------------------------------------------------

// LDS holds parity[4096] then correct[4096]; returns the 12-bit data word,
// `c` = 0..3 corrected bits or 4 = uncorrectable (data kept)
__device__ __forceinline__ uint32_t decode_one(uint32_t w, const uint16_t *lds, uint32_t &c) {
  return golay_decode1(w, lds, lds + 4096, c);
}

template <bool WITH_COUNTS, bool WITH_STATS>
__global__ __launch_bounds__(kDecBlock) void golay_decode_kernel(const u32x4 *__restrict__ cw,
                                                                 uint32_t *__restrict__ trip,
                                                                 uint32_t *__restrict__ counts,
                                                                 int64_t ntiles, int64_t m,
                                                                 const uint16_t *__restrict__ par,
                                                                 const uint16_t *__restrict__ cor,
                                                                 uint64_t *__restrict__ stats) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[8192];
  load_tables<kDecBlock>(lds, par, cor, true);
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  uint32_t bits = 0, unc = 0;
  {  // the tail (see golay_encode_kernel)
    const int32_t *c32 = reinterpret_cast<const int32_t *>(cw);
    uint8_t *t8 = reinterpret_cast<uint8_t *>(trip);
    uint8_t *n8 = reinterpret_cast<uint8_t *>(counts);
    for (int64_t i = ntiles * kDecTile + (int64_t)blockIdx.x * kDecBlock + threadIdx.x; i < m;
         i += (int64_t)gridDim.x * kDecBlock) {
      uint32_t c;
      const uint32_t d = decode_one((uint32_t)c32[i], lds, c);
      t8[3 * i] = (uint8_t)(d & 0xFu);
      t8[3 * i + 1] = (uint8_t)(d >> 4 & 0xFu);
      t8[3 * i + 2] = (uint8_t)(d >> 8);
      if (WITH_COUNTS) n8[i] = (uint8_t)c;
      if (WITH_STATS) {
        bits += c & 3u;
        unc += c >> 2;
      }
    }
  }
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t base = t * kDecTile + wave * kWaveCw + lane * 4;
    u32x4 v[kGroups];
#pragma unroll
    for (int g = 0; g < kGroups; ++g) v[g] = ld_stream(cw + (base + g * 256) / 4);
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
      uint32_t c0, c1, c2, c3;
      uint32_t e0 = golay_spread(decode_one(v[g].x, lds, c0));
      uint32_t e1 = golay_spread(decode_one(v[g].y, lds, c1));
      uint32_t e2 = golay_spread(decode_one(v[g].z, lds, c2));
      uint32_t e3 = golay_spread(decode_one(v[g].w, lds, c3));
      uint32_t *p = trip + (base + g * 256) * 3 / 4;
      st_stream(p, e0 | e1 << 24);
      st_stream(p + 1, e1 >> 8 | e2 << 16);
      st_stream(p + 2, e2 >> 16 | e3 << 8);
      uint32_t cc = c0 | c1 << 8 | c2 << 16 | c3 << 24;
      if (WITH_COUNTS) st_stream(counts + (base + g * 256) / 4, cc);
      if (WITH_STATS) {
        // bytes are 0..4: low two bits = corrected bits (0 for 4), bit 2 = uncorrectable
        uint32_t lowbits = cc & 0x03030303u;
        bits += (lowbits * 0x01010101u) >> 24;  // byte sum (max 12, no carry)
        unc += __builtin_popcount(cc & 0x04040404u);
      }
    }
  }
  if (WITH_STATS) flush_stats2<kDecBlock>(stats, bits, unc);
}

__global__ __launch_bounds__(kBlock) void golay_decode_tail_kernel(
    const int32_t *__restrict__ cw, uint8_t *__restrict__ trip, uint8_t *__restrict__ counts,
    int64_t begin, int64_t m, const uint16_t *__restrict__ par, const uint16_t *__restrict__ cor,
    uint64_t *__restrict__ stats) {
  uint32_t bits = 0, unc = 0;
  for (int64_t i = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * kBlock) {
    uint32_t w = (uint32_t)cw[i];
    uint32_t lo = w & 0xFFFu;
    uint32_t e = cor[((w >> 12) & 0xFFFu) ^ par[lo]];
    uint32_t c = e >> 12;
    uint32_t d = lo ^ (e & 0xFFFu);
    trip[3 * i] = (uint8_t)(d & 0xF);
    trip[3 * i + 1] = (uint8_t)(d >> 4 & 0xF);
    trip[3 * i + 2] = (uint8_t)(d >> 8);
    if (counts) counts[i] = (uint8_t)c;
    bits += c & 3u;
    unc += c >> 2;
  }
  if (stats) flush_stats2(stats, bits, unc);
}

// ---- per-head row packing (ecc_shim.py:623-682, :990-1008) -----------------------

// one thread per codeword: row r, codeword j covers nibbles 3j..3j+2 (zero padded)
__global__ __launch_bounds__(kBlock) void golay_encode_rows_kernel(
    const uint8_t *__restrict__ nib, int32_t *__restrict__ cw, int64_t rows, int64_t d,
    int64_t g, const uint16_t *__restrict__ par) {
  const int64_t total = rows * g;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    int64_t r = i / g, j = i - r * g;
    const uint8_t *row = nib + r * d;
    int64_t c = 3 * j;
    uint32_t b0 = row[c];
    uint32_t b1 = c + 1 < d ? row[c + 1] : 0u;
    uint32_t b2 = c + 2 < d ? row[c + 2] : 0u;
    uint32_t dw = golay_pack(b0, b1, b2);
    cw[i] = (int32_t)(dw | (uint32_t)par[dw] << 12);
  }
}

__global__ __launch_bounds__(kBlock) void golay_decode_rows_kernel(
    const int32_t *__restrict__ cw, uint8_t *__restrict__ nib, int64_t rows, int64_t d, int64_t g,
    const uint16_t *__restrict__ par, const uint16_t *__restrict__ cor,
    uint64_t *__restrict__ stats) {
  const int64_t total = rows * g;
  uint32_t bits = 0, unc = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    int64_t r = i / g, j = i - r * g;
    uint32_t w = (uint32_t)cw[i];
    uint32_t lo = w & 0xFFFu;
    uint32_t e = cor[((w >> 12) & 0xFFFu) ^ par[lo]];
    uint32_t c = e >> 12;
    uint32_t dd = lo ^ (e & 0xFFFu);
    uint8_t *row = nib + r * d;
    int64_t k = 3 * j;
    row[k] = (uint8_t)(dd & 0xF);
    if (k + 1 < d) row[k + 1] = (uint8_t)(dd >> 4 & 0xF);
    if (k + 2 < d) row[k + 2] = (uint8_t)(dd >> 8);
    bits += c & 3u;
    unc += c >> 2;
  }
  if (stats) flush_stats2(stats, bits, unc);
}

// Tiled per-head packing.  A row of D nibbles and its ceil(D/3) codewords are
// not 16-byte multiples (128 B and 172 B at D = 128), and a codeword's three
// nibbles straddle lanes.  Each WAVE owns a tile of R whole rows (R * D and
// R * ceil(D/3) * 4 both multiples of 16 B, ~2 KiB of nibbles): the tile moves
// through HBM as 16-byte accesses, is staged in the wave's own LDS region, and
// the codewords are built there (rows in turn, lane = codeword: no division).
// The regions are wave-private, so no workgroup barrier sits between the
// phases, and the next tile's loads are issued into registers before the
// current tile is processed (one tile of loads in flight per wave throughout).
// The one-thread-per-codeword kernels above stay for short rows (a wave would
// idle on < 16 codewords per row) and for tiles over 64 KiB of LDS.
constexpr int kTiledMaxD = 512;
constexpr int kRowWaves = kBlock / kWave;
constexpr int kTilePre = 4;  // 16-B vectors per lane held for the next tile

struct RowTile {
  int rows;      // R rows per wave tile
  int in_bytes;  // R * d rounded up to 16
  int cw_bytes;  // R * g * 4
};

inline int gcd_i(int a, int b) { return b ? gcd_i(b, a % b) : a; }
inline RowTile row_tile(int64_t d, int64_t g) {
  const int r0 = 16 / gcd_i((int)(d % 16), 16), r1 = 4 / gcd_i((int)(g % 4), 4);
  int r = r0 / gcd_i(r0, r1) * r1;  // lcm: both byte counts are 16-B multiples
  while (2 * r * d <= 2048) r *= 2;  // ~2 KiB of nibbles per wave tile
  RowTile t;
  t.rows = r;
  t.in_bytes = (int)((r * d + 15) & ~15LL);
  t.cw_bytes = (int)(r * g * 4);
  return t;
}
inline size_t row_tile_lds(const RowTile &t, bool decode) {
  return (decode ? 16384 : 8192) + (size_t)kRowWaves * (t.in_bytes + t.cw_bytes);
}
inline bool row_tiled(int64_t d, int64_t g, bool decode) {
  return g >= 16 && d <= kTiledMaxD && row_tile_lds(row_tile(d, g), decode) <= 65536;
}

// The streamed-in side of a wave tile: `bytes` from global `src` into the
// wave's LDS region.  Full aligned tiles of <= kTilePre vectors per lane go
// through registers loaded one tile ahead (prefetch / land); anything else is
// copied in place (byte loop when unaligned or partial).
struct TileIn {
  u32x4 v[kTilePre];
  __device__ __forceinline__ void prefetch(const uint8_t *src, int nvec, int lane) {
#pragma unroll
    for (int k = 0; k < kTilePre; ++k)
      if (lane + k * kWave < nvec) v[k] = ld_stream(reinterpret_cast<const u32x4 *>(src) + lane + k * kWave);
  }
  __device__ __forceinline__ void land(uint8_t *lds, int nvec, int lane) const {
#pragma unroll
    for (int k = 0; k < kTilePre; ++k)
      if (lane + k * kWave < nvec) reinterpret_cast<u32x4 *>(lds)[lane + k * kWave] = v[k];
  }
};

// wave-cooperative copy of `bytes` (16-B vectors when `vec`)
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, int bytes, bool vec,
                                          bool to_global, int lane) {
  if (vec) {
    for (int v = lane; v < bytes / 16; v += kWave) {
      if (to_global)
        st_stream(reinterpret_cast<u32x4 *>(dst) + v, reinterpret_cast<const u32x4 *>(src)[v]);
      else
        reinterpret_cast<u32x4 *>(dst)[v] = ld_stream(reinterpret_cast<const u32x4 *>(src) + v);
    }
  } else {
    for (int b = lane; b < bytes; b += kWave) dst[b] = src[b];
  }
}

// Tile loop shared by encode and decode: `in` / `in_tile_bytes` / `in_row_bytes`
// describe the streamed-in array; body(r0, nr) processes rows [r0, r0 + nr)
// from `lds_in` and stores its results.
template <typename Body>
__device__ __forceinline__ void row_tiles(const uint8_t *in, int64_t rows, int rows_per_tile,
                                          int in_row_bytes, bool aligned16, uint8_t *lds_in,
                                          int lane, int wave, Body body) {
  const int64_t ntiles = (rows + rows_per_tile - 1) / rows_per_tile;
  const int64_t stride = (int64_t)gridDim.x * kRowWaves;
  const int tile_bytes = rows_per_tile * in_row_bytes;
  const int nvec = tile_bytes / 16;
  const bool pre_ok = aligned16 && nvec <= kTilePre * kWave;
  auto full = [&](int64_t t) { return pre_ok && (t + 1) * rows_per_tile <= rows; };
  TileIn nxt;
  int64_t t = (int64_t)blockIdx.x * kRowWaves + wave;
  if (t < ntiles && full(t)) nxt.prefetch(in + t * tile_bytes, nvec, lane);
  for (; t < ntiles; t += stride) {
    const int64_t r0 = t * rows_per_tile;
    const int nr = (int)min<int64_t>(rows_per_tile, rows - r0);
    if (full(t))
      nxt.land(lds_in, nvec, lane);
    else
      wave_copy(lds_in, in + t * tile_bytes, nr * in_row_bytes, aligned16 && nr == rows_per_tile,
                false, lane);
    // lanes read each other's LDS bytes through other types in the next phase:
    // keep the compiler from moving LDS accesses across the phase boundaries
    wave_lds_sync();
    if (t + stride < ntiles && full(t + stride)) nxt.prefetch(in + (t + stride) * tile_bytes, nvec, lane);
    body(r0, nr);
    wave_lds_sync();
  }
}

// Quad items: when d % 4 == 0 a lane takes 4 consecutive codewords of a row
// (12 nibble bytes = 3 aligned dwords of the LDS row), item k = lane + 64 * it
// of the tile -> (row k / Q, quad k % Q), Q = ceil(g / 4), mapped once per
// kernel; tiles of up to kQuadIters * 64 items.  Otherwise a lane takes one
// codeword of a row in turn (3 byte reads).
constexpr int kQuadIters = 4;
struct QuadItems {
  int rr[kQuadIters], jj[kQuadIters];
  __device__ __forceinline__ QuadItems(int lane, int q) {
#pragma unroll
    for (int it = 0; it < kQuadIters; ++it) {
      const int k = lane + it * kWave;
      rr[it] = k / q;
      jj[it] = k - rr[it] * q;
    }
  }
};
inline bool quad_ok(int64_t d, int64_t g, const RowTile &t) {
  return d % 4 == 0 && t.rows * ((g + 3) / 4) <= kQuadIters * kWave;
}

__global__ __launch_bounds__(kBlock) void golay_encode_rows_tiled_kernel(
    const uint8_t *__restrict__ nib, int32_t *__restrict__ cw, int64_t rows, int d, int g,
    RowTile tl, bool aligned16, bool quads, const uint16_t *__restrict__ par) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t *tab = reinterpret_cast<uint16_t *>(smem);
  for (int i = threadIdx.x; i < 512; i += kBlock)
    reinterpret_cast<u32x4 *>(tab)[i] = reinterpret_cast<const u32x4 *>(par)[i];
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  uint8_t *tin = smem + 8192 + wave * (tl.in_bytes + tl.cw_bytes);
  uint32_t *tcw = reinterpret_cast<uint32_t *>(tin + tl.in_bytes);
  const int q = (g + 3) / 4;
  const QuadItems qi(lane, q);
  row_tiles(nib, rows, tl.rows, d, aligned16, tin, lane, wave, [&](int64_t r0, int nr) {
    if (quads) {
#pragma unroll
      for (int it = 0; it < kQuadIters; ++it) {
        const int rr = qi.rr[it], jj = qi.jj[it];
        if (rr >= nr) continue;
        const uint32_t *rw = reinterpret_cast<const uint32_t *>(tin + rr * d) + 3 * jj;
        const int nw = min(3, (d - 12 * jj) / 4);  // dwords of this quad inside the row
        uint32_t dd[4];
        golay_unpack4(rw[0], nw > 1 ? rw[1] : 0u, nw > 2 ? rw[2] : 0u, dd);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (4 * jj + k < g) tcw[rr * g + 4 * jj + k] = dd[k] | (uint32_t)tab[dd[k]] << 12;
      }
    } else {
    for (int rr = 0; rr < nr; ++rr) {
      const uint8_t *row = tin + rr * d;
      for (int j = lane; j < g; j += kWave) {
        const int c = 3 * j;
        const uint32_t dw = golay_pack(row[c], c + 1 < d ? row[c + 1] : 0u, c + 2 < d ? row[c + 2] : 0u);
        tcw[rr * g + j] = dw | (uint32_t)tab[dw] << 12;
      }
    }
    }
    wave_lds_sync();
    wave_copy(reinterpret_cast<uint8_t *>(cw + r0 * g), reinterpret_cast<const uint8_t *>(tcw),
              nr * g * 4, aligned16 && nr == tl.rows, true, lane);
  });
}

__global__ __launch_bounds__(kBlock) void golay_decode_rows_tiled_kernel(
    const int32_t *__restrict__ cw, uint8_t *__restrict__ nib, int64_t rows, int d, int g,
    RowTile tl, bool aligned16, bool quads, const uint16_t *__restrict__ par,
    const uint16_t *__restrict__ cor, uint64_t *__restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t *tab = reinterpret_cast<uint16_t *>(smem);
  for (int i = threadIdx.x; i < 512; i += kBlock) {
    reinterpret_cast<u32x4 *>(tab)[i] = reinterpret_cast<const u32x4 *>(par)[i];
    reinterpret_cast<u32x4 *>(tab)[512 + i] = reinterpret_cast<const u32x4 *>(cor)[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  uint8_t *tout = smem + 16384 + wave * (tl.in_bytes + tl.cw_bytes);
  uint32_t *tcw = reinterpret_cast<uint32_t *>(tout + tl.in_bytes);
  uint32_t bits = 0, unc = 0;
  const int q = (g + 3) / 4;
  const QuadItems qi(lane, q);
  row_tiles(reinterpret_cast<const uint8_t *>(cw), rows, tl.rows, g * 4, aligned16,
            reinterpret_cast<uint8_t *>(tcw), lane, wave, [&](int64_t r0, int nr) {
    if (quads) {
#pragma unroll
      for (int it = 0; it < kQuadIters; ++it) {
        const int rr = qi.rr[it], jj = qi.jj[it];
        if (rr >= nr) continue;
        uint32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          e[k] = 0;
          if (4 * jj + k < g) {
            uint32_t c;
            e[k] = golay_spread(golay_decode1(tcw[rr * g + 4 * jj + k], tab, tab + 4096, c));
            bits += c & 3u;
            unc += c >> 2;
          }
        }
        uint32_t *ow = reinterpret_cast<uint32_t *>(tout + rr * d) + 3 * jj;
        const int nw = min(3, (d - 12 * jj) / 4);
        ow[0] = e[0] | e[1] << 24;
        if (nw > 1) ow[1] = e[1] >> 8 | e[2] << 16;
        if (nw > 2) ow[2] = e[2] >> 16 | e[3] << 8;
      }
    } else {
    for (int rr = 0; rr < nr; ++rr) {
      uint8_t *row = tout + rr * d;
      for (int j = lane; j < g; j += kWave) {
        uint32_t c;
        const uint32_t dd = golay_decode1(tcw[rr * g + j], tab, tab + 4096, c);
        bits += c & 3u;
        unc += c >> 2;
        const int k = 3 * j;
        row[k] = (uint8_t)(dd & 0xFu);
        if (k + 1 < d) row[k + 1] = (uint8_t)(dd >> 4 & 0xFu);
        if (k + 2 < d) row[k + 2] = (uint8_t)(dd >> 8);
      }
    }
    }
    wave_lds_sync();
    wave_copy(nib + r0 * d, tout, nr * d, aligned16 && nr == tl.rows, true, lane);
  });
  if (stats) flush_stats2(stats, bits, unc);
}

// ---- per-head rows through register tiles (d % 16 == 0) --------------------------
// The layout of the shim's fused read (shim.hip): a wave owns a tile of `tr`
// whole rows, contiguous in both arrays.  The codeword side moves as 16-byte
// buffer loads straight into registers, one 4-codeword group of a row per lane
// (rows are 4g bytes, so a group may start on any dword; a row's last group
// reads up to 3 codewords of the next row, which are decoded but masked out of
// the statistics and never staged); the nibble side moves as 16-byte
// non-temporal accesses of the tile's contiguous rows through a wave-private
// LDS tile whose rows are `lr` = 16-byte-rounded 12 * ceil(g / 4) bytes apart,
// so every LDS access of that side is one aligned ds_read/write_b128.
//  decode: codewords -> registers -> spread-table decode (nibbles one per byte,
//          exactly the output format) -> LDS rows -> 16-byte stores
//  encode: nibbles -> 16-byte loads -> LDS rows -> 4 data words per lane ->
//          parity table -> LDS codeword tile -> 16-byte stores
// Every lane's (row, group) and (row, 16-byte chunk) items are the same for
// every tile, computed once; the next tile's loads are issued before the
// current tile's stores.  Per-lane offsets are 32-bit inside a tile, tile
// bases 64-bit and wave-uniform (descriptors in SGPRs).
// dynamic tail schedule (kvecc_internal.h TileSchedule), as the fused reads
// the rows decode's persistent shape: 4-wave workgroups at 3 per CU with a 30 %
// static share (as the fused Golay read, shim.hip): 52.6 -> 51.7 us against 8 waves,
// 2 per CU and 75 % (profiles/r05/rows_dec_ab.log; 4 per CU 57.1)
constexpr int kRegBlock = 256;
constexpr int kRegWaves = kRegBlock / kWave;
constexpr uint32_t kRowsDecStaticPct = 30;
constexpr int kRegGroups = 4;        // 4-codeword groups per lane per tile (max)
constexpr int kRegChunks = 3;        // 16-byte nibble chunks per lane per tile (max)
constexpr int kRegDecStage = 2304;   // decode: LDS nibble rows per wave
constexpr int kRegEncIn = 2304;      // encode: LDS nibble rows per wave
constexpr int kRegEncOut = 2816;     // encode: LDS codeword tile per wave

struct RegRowsArgs {
  const void *src;  // decode: int32 codewords; encode: uint8 nibbles
  void *dst;        // decode: uint8 nibbles; encode: int32 codewords
  int64_t rows, ntiles;
  uint32_t d, g, gpr, lr, tr;
  const void *tab;  // decode: spread tables (uint32[8192]); encode: parity (uint16[4096])
  uint64_t *stats;
  uint32_t *dyn;    // work-counter slot of the dynamic tail (ntiles < 2^32)
};

struct RegItems {
  uint32_t r1[kRegGroups], q1[kRegGroups];  // row, 4-codeword group
  uint32_t r2[kRegChunks], j2[kRegChunks];  // row, 16-byte nibble chunk
  __device__ __forceinline__ RegItems(uint32_t lane, uint32_t gpr, uint32_t d16) {
#pragma unroll
    for (int i = 0; i < kRegGroups; ++i) {
      const uint32_t f = lane + kWave * i;
      r1[i] = f / gpr;
      q1[i] = f - r1[i] * gpr;
    }
#pragma unroll
    for (int i = 0; i < kRegChunks; ++i) {
      const uint32_t v = lane + kWave * i;
      r2[i] = v / d16;
      j2[i] = v - r2[i] * d16;
    }
  }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(uni(reinterpret_cast<const char *>(base))), 0,
                                           (int)uni(bytes), 0x00020000);
}

// BLOCK / PCT: workgroup size and static share (the product's: kRegBlock, kRowsDecStaticPct;
// tools/exp/r05_exp.hip instantiates others)
template <bool STATS, int BLOCK = kRegBlock, uint32_t PCT = kRowsDecStaticPct>
__global__ __launch_bounds__(BLOCK) void golay_decode_rows_reg_kernel(RegRowsArgs a) {
  constexpr int kW = BLOCK / kWave;
  __shared__ __attribute__((aligned(16))) uint32_t tab[8192];
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kW][kRegDecStage];
  for (int i = threadIdx.x; i < 2048; i += BLOCK)
    reinterpret_cast<u32x4 *>(tab)[i] = reinterpret_cast<const u32x4 *>(a.tab)[i];
  __syncthreads();
  const uint32_t wave = uni((uint32_t)threadIdx.x / kWave), lane = threadIdx.x % kWave;
  uint8_t *stage = stage_all[wave];
  const uint32_t d16 = a.d / 16, groups = a.tr * a.gpr, chunks = a.tr * d16;
  const RegItems it(lane, a.gpr, d16);
  const int32_t *cw = reinterpret_cast<const int32_t *>(a.src);
  uint8_t *nib = reinterpret_cast<uint8_t *>(a.dst);
  uint32_t bits = 0, unc = 0;

  int64_t t = (int64_t)blockIdx.x * kW + wave;
  if (t >= a.ntiles) return;  // no workgroup barrier below
  const int64_t tstride = (int64_t)gridDim.x * kW;
  TileSchedule sched;
  sched.init((uint32_t)a.ntiles, a.dyn, (uint32_t)t, (uint32_t)tstride, lane, PCT);
  u32x4 w[kRegGroups];
  auto issue = [&](int64_t tt) {
    const uint32_t rows = (uint32_t)min<int64_t>(a.tr, a.rows - tt * a.tr);
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(cw + tt * a.tr * a.g, rows * a.g * 4u);
#pragma unroll
    for (int i = 0; i < kRegGroups; ++i) {
      if (i * kWave >= (int)groups) break;  // uniform
      w[i] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, it.r1[i] * a.g * 4u + 16u * it.q1[i], 0, 2));
    }
  };
  issue(t);
  for (;;) {
#pragma unroll
    for (int i = 0; i < kRegGroups; ++i) {
      if (i * kWave >= (int)groups) break;  // uniform
      const uint32_t q = it.q1[i];
      uint32_t sp[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t c = w[i][k];
        const uint32_t p = tab[c & 0xFFFu];
        const uint32_t e = tab[4096 + (((c >> 12) ^ (p >> 20)) & 0xFFFu)];
        sp[k] = __builtin_amdgcn_bitop3_b32(p, e, 0x000F0F0Fu, 0x28);  // (p ^ e) & mask
        if (STATS && 4 * q + k < a.g) {  // past the tile: loads gave 0, count 0
          bits += e >> 24 & 3u;
          unc += e >> 30;
        }
      }
      if (it.r1[i] < a.tr) {
        uint32_t *o = reinterpret_cast<uint32_t *>(stage + it.r1[i] * a.lr + 12 * q);
        o[0] = sp[0] | sp[1] << 24;
        o[1] = sp[1] >> 8 | sp[2] << 16;
        o[2] = sp[2] >> 16 | sp[3] << 8;
      }
    }
    wave_lds_sync();
    const int64_t cur = t;
    t = (int64_t)sched.next((uint32_t)t, lane);
    const bool more = t < a.ntiles;
    if (more) issue(t);
    const uint32_t rows = (uint32_t)min<int64_t>(a.tr, a.rows - cur * a.tr);
    uint8_t *out = nib + cur * a.tr * a.d;
#pragma unroll
    for (int i = 0; i < kRegChunks; ++i) {
      if (i * kWave >= (int)chunks) break;  // uniform
      if (it.r2[i] < rows)
        st_stream(reinterpret_cast<u32x4 *>(out + it.r2[i] * a.d) + it.j2[i],
                  *reinterpret_cast<const u32x4 *>(stage + it.r2[i] * a.lr + 16 * it.j2[i]));
    }
    if (!more) break;
    wave_lds_sync();
  }
  if (STATS) {
    bits = wave_sum(bits);
    unc = wave_sum(unc);
    if (lane == 0) {
      uint64_t *slot = a.stats + ((blockIdx.x * kW + wave) % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
      if (bits) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)bits);
      if (unc) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)unc);
    }
  }
}

// Per-head rows encode on a full grid: one tile of `tr` rows per wave,
// workgroups of kEncRowWaves waves retiring (no schedule, no counter slot).
// The parity comes from two 64-entry tables, parity(d) = T[d & 63] ^ T[64 + (d >> 6)]
// (256 B of LDS per workgroup, conflict-free), not the 8 KiB table a
// persistent grid could afford to stage.  Each lane loads its 4-codeword
// groups' 12 nibble bytes straight from HBM (buffer_load_dwordx3 at
// r * d + 12 q, 4-byte aligned; a row's last group reads into the next row,
// whose bytes are masked to the per-head zero padding), encodes them into a
// wave-private LDS codeword tile, and the tile leaves contiguous as 16-byte
// non-temporal stores (stored straight from registers the 16-byte stores are
// misaligned: half rate).  [8,4096,32,128]: 56.9 us for round 4's
// persistent kernel, 55.3 with the full grid and the nibbles landed in LDS
// first, 52.2 loading them straight (profiles/r05/rows_enc_ab.log; 4-wave
// workgroups 52.7, 2-wave 55.4).
constexpr int kEncRowWaves = 8;
__global__ __launch_bounds__(kEncRowWaves * kWave) void golay_encode_rows_full_kernel(RegRowsArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t tlo[64], thi[64];
  __shared__ __attribute__((aligned(16))) uint8_t out_all[kEncRowWaves][kRegEncOut];
  if (threadIdx.x < 64) {
    const uint16_t *par = reinterpret_cast<const uint16_t *>(a.tab);
    tlo[threadIdx.x] = par[threadIdx.x];
    thi[threadIdx.x] = par[threadIdx.x << 6];
  }
  __syncthreads();
  const uint32_t wave = uni((uint32_t)threadIdx.x / kWave), lane = threadIdx.x % kWave;
  uint32_t *sout = reinterpret_cast<uint32_t *>(out_all[wave]);
  const uint32_t groups = a.tr * a.gpr;
  const RegItems it(lane, a.gpr, a.d / 16);
  const uint8_t *nib = reinterpret_cast<const uint8_t *>(a.src);
  uint32_t *cw = reinterpret_cast<uint32_t *>(a.dst);
  const int64_t t = (int64_t)blockIdx.x * kEncRowWaves + wave;
  if (t >= a.ntiles) return;
  const uint32_t rows = (uint32_t)min<int64_t>(a.tr, a.rows - t * a.tr);
  // ---- the tile's groups, straight into registers (past the tile: 0)
  const __amdgpu_buffer_rsrc_t rs = tile_rsrc(nib + t * a.tr * a.d, rows * a.d);
  uint32_t w[kRegGroups][3];
#pragma unroll
  for (int i = 0; i < kRegGroups; ++i) {
    if (i * kWave >= (int)groups) break;  // uniform
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, it.r1[i] * a.d + 12u * it.q1[i], 0, 2);
    w[i][0] = v[0];
    w[i][1] = v[1];
    w[i][2] = v[2];
  }
  // ---- 4 codewords per lane into the LDS codeword tile
#pragma unroll
  for (int i = 0; i < kRegGroups; ++i) {
    if (i * kWave >= (int)groups) break;  // uniform
    const uint32_t r = it.r1[i], q = it.q1[i];
    if (r < rows) {
      // bytes at or past the row's end are the per-head padding: zero
      const int valid = (int)a.d - 12 * (int)q;  // bytes of the group inside the row
      uint32_t b[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int lo = valid - 4 * k;
        b[k] = lo >= 4 ? w[i][k] : lo <= 0 ? 0u : w[i][k] & ((1u << (8 * lo)) - 1u);
      }
      uint32_t dd[4];
      golay_unpack4(b[0], b[1], b[2], dd);
      uint32_t *o = sout + r * a.g + 4 * q;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (4 * q + k < a.g) o[k] = dd[k] | (uint32_t)(tlo[dd[k] & 63u] ^ thi[dd[k] >> 6]) << 12;
    }
  }
  wave_lds_sync();
  // ---- the tile's codewords, contiguous, as 16-byte stores
  const uint32_t nw = rows * a.g;  // words
  uint32_t *out = cw + t * a.tr * a.g;
  for (uint32_t k = lane; k < nw / 4; k += kWave)
    st_stream(reinterpret_cast<u32x4 *>(out) + k, reinterpret_cast<const u32x4 *>(sout)[k]);
  for (uint32_t k = nw / 4 * 4 + lane; k < nw; k += kWave) st_stream(out + k, sout[k]);  // last tile's tail
}

// tile geometry of the register-tile row kernels (0 rows: not applicable)
struct RegGeom {
  uint32_t gpr, lr, tr;
};
inline RegGeom reg_geom(int64_t d, int64_t g, bool encode) {
  RegGeom r{0, 0, 0};
  if (d % 16 != 0 || g < 16 || d > kTiledMaxD) return r;
  r.gpr = (uint32_t)cdiv(g, 4);
  r.lr = (12 * r.gpr + 15) / 16 * 16;
  int64_t tr = std::min<int64_t>({(int64_t)(encode ? kRegEncIn : kRegDecStage) / r.lr,
                                  (int64_t)kWave * kRegGroups / r.gpr, (int64_t)kWave * kRegChunks / (d / 16)});
  if (encode) {
    tr = std::min<int64_t>(tr, kRegEncOut / (4 * g));
    const int64_t m = 4 / gcd_i((int)(g % 4), 4);  // tiles stay 16-byte aligned: tr * g % 4 == 0
    tr = tr / m * m;
  }
  r.tr = (uint32_t)std::max<int64_t>(tr, 0);
  return r;
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int kvecc_golay_encode(const uint8_t *triplets, int32_t *codewords, int64_t m,
                                 void *stream) {
  if (m < 0) return set_error(KVECC_EINVAL, "golay_encode: negative m");
  if (m == 0) return KVECC_OK;
  if (!triplets || !codewords) return set_error(KVECC_EINVAL, "golay_encode: null pointer");
  const uint16_t *par = golay_parity_table_dev();
  if (!par) return KVECC_EHIP;
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  if (aligned(triplets, 4) && aligned(codewords, 16)) {
    int64_t ntiles = m / kEncTile;
    if (ntiles > 0) {  // the tile kernel also takes the tail
      unsigned g = grid_for(ntiles, 1, kEncPerCu);  // grid-strided
      KVECC_LAUNCH(golay_encode_kernel, dim3(g), dim3(kEncBlock), 0, st,
                         reinterpret_cast<const uint32_t *>(triplets),
                         reinterpret_cast<u32x4 *>(codewords), ntiles, m, par);
      done = m;
    }
  }
  if (done < m) {
    unsigned g = grid_for(m - done, kBlock);
    KVECC_LAUNCH(golay_encode_tail_kernel, dim3(g), dim3(kBlock), 0, st, triplets, codewords,
                       done, m, par);
  }
  return check_launch("golay_encode");
}

KVECC_API int kvecc_golay_decode(const int32_t *codewords, uint8_t *triplets, uint8_t *counts,
                                 int64_t m, uint64_t *stats, void *stream) {
  if (m < 0) return set_error(KVECC_EINVAL, "golay_decode: negative m");
  if (m == 0) return KVECC_OK;
  if (!triplets || !codewords) return set_error(KVECC_EINVAL, "golay_decode: null pointer");
  const uint16_t *par = golay_parity_table_dev();
  const uint16_t *cor = golay_correct_table_dev();
  if (!par || !cor) return KVECC_EHIP;
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  if (aligned(codewords, 16) && aligned(triplets, 4) && (!counts || aligned(counts, 4))) {
    int64_t ntiles = m / kDecTile;
    if (ntiles > 0) {
      unsigned g = grid_for(ntiles, 1, kDecPerCu);  // grid-strided
      auto c = reinterpret_cast<const u32x4 *>(codewords);
      auto t = reinterpret_cast<uint32_t *>(triplets);
      auto n = reinterpret_cast<uint32_t *>(counts);
      const dim3 b(kDecBlock);
      if (counts && stats)
        KVECC_LAUNCH((golay_decode_kernel<true, true>), dim3(g), b, 0, st, c, t, n, ntiles, m, par, cor, stats);
      else if (counts)
        KVECC_LAUNCH((golay_decode_kernel<true, false>), dim3(g), b, 0, st, c, t, n, ntiles, m, par, cor, stats);
      else if (stats)
        KVECC_LAUNCH((golay_decode_kernel<false, true>), dim3(g), b, 0, st, c, t, n, ntiles, m, par, cor, stats);
      else
        KVECC_LAUNCH((golay_decode_kernel<false, false>), dim3(g), b, 0, st, c, t, n, ntiles, m, par, cor, stats);
      done = m;  // the tile kernel also takes the tail
    }
  }
  if (done < m) {
    unsigned g = grid_for(m - done, kBlock);
    KVECC_LAUNCH(golay_decode_tail_kernel, dim3(g), dim3(kBlock), 0, st, codewords, triplets,
                       counts, done, m, par, cor, stats);
  }
  return check_launch("golay_decode");
}

KVECC_API int kvecc_golay_encode_rows(const uint8_t *nibbles, int32_t *codewords, int64_t rows,
                                      int64_t d, void *stream) {
  if (rows < 0 || d < 0) return set_error(KVECC_EINVAL, "golay_encode_rows: negative size");
  if (rows == 0 || d == 0) return KVECC_OK;
  if (!nibbles || !codewords) return set_error(KVECC_EINVAL, "golay_encode_rows: null pointer");
  const uint16_t *par = golay_parity_table_dev();
  if (!par) return KVECC_EHIP;
  int64_t g = (d + 2) / 3;
  const RegGeom rg = reg_geom(d, g, true);
  if (rg.tr > 0 && aligned(nibbles, 16) && aligned(codewords, 16) &&
      cdiv(rows, rg.tr) < (1LL << 31)) {
    const RegRowsArgs a{nibbles, codewords, rows, cdiv(rows, rg.tr), (uint32_t)d, (uint32_t)g, rg.gpr, rg.lr,
                        rg.tr, par, nullptr};
    KVECC_LAUNCH(golay_encode_rows_full_kernel, dim3((unsigned)cdiv(a.ntiles, kEncRowWaves)),
                 dim3(kEncRowWaves * kWave), 0, as_stream(stream), a);
    return check_launch("golay_encode_rows");
  }
  if (row_tiled(d, g, false)) {
    const RowTile tl = row_tile(d, g);
    const bool a16 = aligned(nibbles, 16) && aligned(codewords, 16);
    const unsigned grid = grid_for(cdiv(rows, tl.rows), kRowWaves, 8);
    KVECC_LAUNCH(golay_encode_rows_tiled_kernel, dim3(grid), dim3(kBlock), row_tile_lds(tl, false),
                 as_stream(stream), nibbles, codewords, rows, (int)d, (int)g, tl, a16,
                 quad_ok(d, g, tl), par);
    return check_launch("golay_encode_rows");
  }
  unsigned grid = grid_for(rows * g, kBlock);
  KVECC_LAUNCH(golay_encode_rows_kernel, dim3(grid), dim3(kBlock), 0, as_stream(stream),
                     nibbles, codewords, rows, d, g, par);
  return check_launch("golay_encode_rows");
}

KVECC_API int kvecc_golay_decode_rows(const int32_t *codewords, uint8_t *nibbles, int64_t rows,
                                      int64_t d, uint64_t *stats, void *stream) {
  if (rows < 0 || d < 0) return set_error(KVECC_EINVAL, "golay_decode_rows: negative size");
  if (rows == 0 || d == 0) return KVECC_OK;
  if (!nibbles || !codewords) return set_error(KVECC_EINVAL, "golay_decode_rows: null pointer");
  const uint16_t *par = golay_parity_table_dev();
  const uint16_t *cor = golay_correct_table_dev();
  if (!par || !cor) return KVECC_EHIP;
  int64_t g = (d + 2) / 3;
  const RegGeom rg = reg_geom(d, g, false);
  if (rg.tr > 0 && aligned(nibbles, 16) && aligned(codewords, 4) &&
      cdiv(rows, rg.tr) < (1LL << 31)) {
    const uint32_t *atab = golay_attn_table_dev();
    if (!atab) return KVECC_EHIP;
    RegRowsArgs a{codewords, nibbles, rows, cdiv(rows, rg.tr), (uint32_t)d, (uint32_t)g, rg.gpr, rg.lr, rg.tr,
                  atab, stats};
    if (!(a.dyn = shim_dyn_slot(stream))) return KVECC_EHIP;
    const unsigned grid = (unsigned)std::min<int64_t>(cdiv(a.ntiles, kRegWaves), (int64_t)cu_count() * kRowsPerCu);
    if (stats)
      KVECC_LAUNCH(golay_decode_rows_reg_kernel<true>, dim3(grid), dim3(kRegBlock), 0, as_stream(stream), a);
    else
      KVECC_LAUNCH(golay_decode_rows_reg_kernel<false>, dim3(grid), dim3(kRegBlock), 0, as_stream(stream), a);
    return check_launch("golay_decode_rows");
  }
  if (row_tiled(d, g, true)) {
    const RowTile tl = row_tile(d, g);
    const bool a16 = aligned(nibbles, 16) && aligned(codewords, 16);
    const unsigned grid = grid_for(cdiv(rows, tl.rows), kRowWaves, 8);
    KVECC_LAUNCH(golay_decode_rows_tiled_kernel, dim3(grid), dim3(kBlock), row_tile_lds(tl, true),
                 as_stream(stream), codewords, nibbles, rows, (int)d, (int)g, tl, a16,
                 quad_ok(d, g, tl), par, cor, stats);
    return check_launch("golay_decode_rows");
  }
  unsigned grid = grid_for(rows * g, kBlock);
  KVECC_LAUNCH(golay_decode_rows_kernel, dim3(grid), dim3(kBlock), 0, as_stream(stream),
                     codewords, nibbles, rows, d, g, par, cor, stats);
  return check_launch("golay_decode_rows");
}

}  // extern "C"
